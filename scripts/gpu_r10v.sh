#!/bin/bash
# BN fold workgroup cap A/B (ResNet-50 bs256)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10v}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name="$1"; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
for r in 1 2; do
  run off_$r KFB_BN_FOLD=0
  run f512_$r KFB_BN_FOLD=1 KFB_BN_FOLD_GRID=512
  run f256_$r KFB_BN_FOLD=1 KFB_BN_FOLD_GRID=256
done
