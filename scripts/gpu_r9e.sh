#!/bin/bash
# bench A/B: streaming 3x3 kernel forward-only vs forward+dgrad, priority
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r9e}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name="$1"; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 124|134|137|139) exit $rc;; esac
}
for r in 1 2 3; do
  run base_$r KFB_IGEMM_NOS3=1
  run s3all_$r KFB_S3_DGRAD=1
  run s3fwd_$r KFB_S3_DGRAD=0
  run s3fwdprio_$r KFB_S3_DGRAD=0 KFB_COMPUTE_PRIORITY=1
done
