#!/bin/bash
# Round-6 session: ResNet-50 bs256 bench and kernel summary of the final tree
# (flat BN passes from 64 MB, slack-0.3 wgrad grids).  Each GPU step under its
# own time limit; fault / abort / timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r14e"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log" | cut -c1-700
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
step bench 300 python bench.py --steps 30 --warmup 10
cd /tmp && export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 3
cd "$ROOT"
f=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/kernel_stats.py "$f" --last-steps 3 --top 70 > "$OUT/kernel_summary.txt"
step bench2 300 python bench.py --steps 30 --warmup 10
echo done
