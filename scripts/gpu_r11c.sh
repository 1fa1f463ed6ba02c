#!/bin/bash
# default BN fold mode 2 (small tensors): A/B at bs32 / bs64 / bs256, then the full GPU tier
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r11c}"
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
  run r152_def_$r "--model resnet152 --batch_size 32" KFB_X=0
  run r50_64_off_$r "--model resnet50 --batch_size 64" KFB_BN_FOLD=0
  run r50_64_def_$r "--model resnet50 --batch_size 64" KFB_X=0
  run r50_off_$r "" KFB_BN_FOLD=0
  run r50_def_$r "" KFB_X=0
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tier.log" 2>&1
rc=$?; echo "tier rc=$rc"; tail -3 "$OUT/tier.log"; grep -E "^FAILED" "$OUT/tier.log" | head
