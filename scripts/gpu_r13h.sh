#!/bin/bash
# Round-6 session: collectives issued on the caller's stream (no comm stream
# of their own): the distributed GPU tests, the DeepSpeech2 fixes, and the
# 1-rank RCCL bench taped / eager next to the no-group bench.  Each GPU step
# under its own time limit; fault / abort / timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r13h"; mkdir -p "$OUT"
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
B="python bench.py --steps 30 --warmup 8"
step pytest 600 python -u -m pytest tests/test_dist_gpu.py tests/test_tape_gpu.py::test_deepspeech2_with_launch_tape tests/test_rnn.py tests/test_comm_selftest.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread
step nopg 200 $B
step rccl_taped 200 env KFB_FORCE_PG=1 $B
step rccl_eager 200 env KFB_FORCE_PG=1 $B --launch_tape 0
step nopg2 200 $B
step rccl_taped2 200 env KFB_FORCE_PG=1 $B
echo done
