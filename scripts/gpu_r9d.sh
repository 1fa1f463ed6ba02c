#!/bin/bash
# bench A/B: in-kernel BN finalize on/off, S3 on/off (same box, interleaved)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r9d}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name="$1"; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 124|134|137|139) exit $rc;; esac
}
for r in 1 2; do
  run base_$r KFB_BN_FIN=0 KFB_IGEMM_NOS3=1
  run fin_$r KFB_BN_FIN=1 KFB_IGEMM_NOS3=1
  run s3_$r KFB_BN_FIN=0 KFB_IGEMM_NOS3=0
  run both_$r KFB_BN_FIN=1 KFB_IGEMM_NOS3=0
  run bothprio_$r KFB_BN_FIN=1 KFB_IGEMM_NOS3=0 KFB_COMPUTE_PRIORITY=1
done
