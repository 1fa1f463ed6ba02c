#!/bin/bash
# dgrad-tail BN backward finalize: tests + bench A/B
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10i}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name="$1" t="$2"; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step s1test 300 python -u -m pytest tests/test_conv_s1_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "finalize or fwd_stats"
step fintest 400 python -u -m pytest tests/test_bn_fin_gpu.py tests/test_conv_stream_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
run() {
  local name="$1"; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
for r in 1 2; do
  run fin_$r KFB_BN_FIN=persistent
  run grad_$r KFB_BN_FIN=grad
  run nofin_$r KFB_BN_FIN=0
done
