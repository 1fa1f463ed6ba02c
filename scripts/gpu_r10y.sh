#!/bin/bash
# channel-block BN fold: its tests, then an interleaved A/B against the finalize launches
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10y}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout-method thread --timeout 300 tests/test_bn_fin_gpu.py > "$OUT/foldtest.log" 2>&1
rc=$?; echo "foldtest rc=$rc"; tail -3 "$OUT/foldtest.log"; [ $rc -eq 0 ] || exit $rc
run() {
  local name="$1" args="$2"; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 $args > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
for r in 1 2 3; do
  run off_$r "" KFB_BN_FOLD=0
  run fold_$r "" KFB_BN_FOLD=1
done
run r152_off "--model resnet152 --batch_size 32" KFB_BN_FOLD=0
run r152_fold "--model resnet152 --batch_size 32" KFB_BN_FOLD=1
