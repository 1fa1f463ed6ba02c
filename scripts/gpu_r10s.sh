#!/bin/bash
# in-network A/B: weight-gradient split caps, stem pool link
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10s}"
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
  run base_$r KFB_X=0
  run cap512_$r KFB_WGRAD_MAXBLOCKS=512
  run cap384_$r KFB_WGRAD_MAXBLOCKS=384
  run plink_$r KFB_POOL_LINK=1
done
