#!/bin/bash
# Round-6 session: the two r13t tier failures - the depthwise filter gradient
# in deterministic mode (NASNet tape oracle) and the MobileNet ReLU6 gradient
# check - with the dgrad bit-mask epilogue at MobileNet widths.  Each GPU
# step under its own time limit; fault / abort / timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r13u"; mkdir -p "$OUT"
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
step pytest_bits 600 python -u -m pytest tests/test_conv_gpu.py -k "dgrad_fused_epilogue or mobilenet_widths" -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
step pytest_fix 600 env KFB_AUTOTUNE_LOG=1 python -u -m pytest tests/test_tape_gpu.py::test_nasnet_tape_bitwise_matches_eager tests/test_kernels_gpu.py::test_mobilenet_relu6_in_bn_matches_separate_pass -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread
echo done
