#!/bin/bash
# BN fold only on small tensors (KFB_BN_FOLD=2): A/B at bs32 / bs64 / bs256
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r11b}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name="$1" args="$2"; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
for r in 1 2; do
  run r152_off_$r "--model resnet152 --batch_size 32" KFB_BN_FOLD=0
  run r152_small_$r "--model resnet152 --batch_size 32" KFB_BN_FOLD=2
  run r50_off_$r "" KFB_BN_FOLD=0
  run r50_small_$r "" KFB_BN_FOLD=2
done
