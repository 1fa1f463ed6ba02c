#!/bin/bash
# small-batch A/B: BN finalize folded into the apply passes vs launches (ResNet-152 bs32, ResNet-50 bs64)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10t}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name="$1" args="$2"; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
for r in 1 2 3; do
  run base_$r "" KFB_POOL_LINK=0
  run plink_$r "" KFB_POOL_LINK=1
done
for r in 1 2; do
  run r152_off_$r "--model resnet152 --batch_size 32" KFB_BN_FOLD=0
  run r152_fold_$r "--model resnet152 --batch_size 32" KFB_BN_FOLD=1
  run r50_64_off_$r "--model resnet50 --batch_size 64" KFB_BN_FOLD=0
  run r50_64_fold_$r "--model resnet50 --batch_size 64" KFB_BN_FOLD=1
done
