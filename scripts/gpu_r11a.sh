#!/bin/bash
# stream-K on the few-tile layers (small batches): A/B
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r11a}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name="$1" args="$2"; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout-method thread --timeout 200 tests/test_conv_gpu.py -k "sk" > "$OUT/sktest.log" 2>&1; echo "sktest rc=$?"; tail -2 "$OUT/sktest.log"
for r in 1 2; do
  run r152_nosk_$r "--model resnet152 --batch_size 32" KFB_IGEMM_SK_SMALL=0
  run r152_sk_$r "--model resnet152 --batch_size 32" KFB_IGEMM_SK_SMALL=1
  run r50_64_nosk_$r "--model resnet50 --batch_size 64" KFB_IGEMM_SK_SMALL=0
  run r50_64_sk_$r "--model resnet50 --batch_size 64" KFB_IGEMM_SK_SMALL=1
done
run r50_256_sk "" KFB_IGEMM_SK_SMALL=1
