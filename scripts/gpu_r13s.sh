#!/bin/bash
# Round-6 session: MobileNet-v2 bs128 kernel summary after the depthwise and ReLU6
# changes, to rank what is left.  Each GPU step under its own
# time limit; fault / abort / timeout stops the script.
#
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r13s"; mkdir -p "$OUT"
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
cd /tmp && export TMPDIR=/tmp
for m in "mobilenet 128"; do
  set -- $m
  step prof_$1 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$1" -o run -- python3 "$ROOT/bench.py" --model $1 --batch_size $2 --steps 5 --warmup 4
  f=$(find "$OUT/prof_$1" -name "*kernel_trace.csv" | head -n 1)
  [ -n "$f" ] && python3 "$ROOT/scripts/kernel_stats.py" "$f" --last-steps 3 --top 40 > "$OUT/kernels_$1.txt"
done
echo done
