#!/bin/bash
# re-run of the round-end tier's failures, then the first half of the zoo refresh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10r}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_conv_s1_gpu.py::test_s1_finalizes_bn" \
  "tests/test_dist_gpu.py::test_pair_averaging_store_never_tears_over_hip_ipc" \
  "tests/test_dist_gpu.py::test_two_ranks_pair_averaging_training" \
  "tests/test_dist_gpu.py::test_two_ranks_pair_averaging_taped" \
  tests/test_model_gpu.py tests/test_tape_gpu.py > "$OUT/fix.log" 2>&1
rc=$?; echo "fix rc=$rc"; tail -5 "$OUT/fix.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_zoo_r9.sh zoo_r9a 1
