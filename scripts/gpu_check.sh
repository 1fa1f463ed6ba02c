#!/bin/bash
# GPU-box check script: smoke, GPU tests, 1-GPU bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault / abort / timeout stops the
# script (no further GPU work), a plain test failure does not.
#   usage: scripts/gpu_check.sh [tag] [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-run}"; shift || true
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0

fatal() {  # exit codes that mean the GPU step died rather than failed
  case "$1" in 124|134|137|139|-6|-11) return 0;; *) return 1;; esac
}

step() {  # step <name> <timeout> <cmd...>
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s): $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}

step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
fi
if [ "${CONV_BENCH:-0}" = "1" ]; then
  step conv_bench 600 python scripts/bench_conv.py --json "$OUT/conv_bench.json"
fi
step bench 900 python bench.py --verbose "$@"
if [ -n "${BENCH_B:-}" ]; then
  step bench_b 900 python bench.py --verbose $BENCH_B
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 3 ${PROF_ARGS:-}
  cd "$ROOT"
  f=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -n 1)
  [ -n "$f" ] && python3 scripts/kernel_stats.py "$f" --steps 8 --top 60 > "$OUT/kernel_summary.txt"
fi
echo "done"
