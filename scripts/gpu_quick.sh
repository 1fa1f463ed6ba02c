#!/bin/bash
# Focused GPU check: selected pytest files, then the 1-GPU bench and a
# rocprofv3 kernel-trace of the bench (summary over the last 4 steps).
#   usage: scripts/gpu_quick.sh <tag> "<pytest targets>" [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="$1"; TESTS="$2"; shift 2
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
if [ -n "$TESTS" ]; then
  step pytest 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
fi
step bench 600 python bench.py --verbose "$@"
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps 6 --warmup 6 "$@"
  cd "$ROOT"
  f=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -n 1)
  [ -n "$f" ] && python3 scripts/kernel_stats.py "$f" --last-steps 4 --top 60 > "$OUT/kernel_summary.txt"
  rm -f "$OUT"/prof/*kernel_stats.csv "$OUT"/prof/*domain_stats.csv
fi
echo done
