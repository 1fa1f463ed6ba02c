#!/bin/bash
# round-4 features on the GPU: GPU JPEG path, raw tape, BN fold, stem S7, taped KungFu options
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10n}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name="$1" t="$2"; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
step jpegtest 200 $PT --timeout 120 tests/test_jpeg_path.py -m gpu
step tapetest 600 $PT --timeout 300 tests/test_tape_gpu.py -k "natively or bitwise or raw_tape or real_data"
step foldtest 400 $PT --timeout 300 tests/test_bn_fin_gpu.py
step s7test 300 $PT --timeout 120 tests/test_stem_gpu.py
step disttest 600 $PT --timeout 280 tests/test_dist_gpu.py -k "one_rank_rccl_is_identity or averaging_taped"
step nasnet 400 $PT --timeout 380 tests/test_tape_gpu.py -k nasnet
