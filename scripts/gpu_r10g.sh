#!/bin/bash
# bench A/B: weight-gradient side stream vs serial, by layer size
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10g}"
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
  run side_$r KFB_WGRAD_STREAM=1
  run serial_$r KFB_WGRAD_STREAM=0
  run max5e5_$r KFB_WGRAD_SIDE_MAX=5e5
  run max1e5_$r KFB_WGRAD_SIDE_MAX=1e5
done
