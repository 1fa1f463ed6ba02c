#!/bin/bash
# S1: two workgroups per CU vs one (micro-bench), tests, bench A/B
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10e}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name="$1" t="$2"; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step s1test 300 python -u -m pytest tests/test_conv_s1_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step wpc2 300 python -u scripts/bench_s1.py --algos s1
KFB_S1_WPC=1 step wpc1 300 python -u scripts/bench_s1.py --algos s1
paste "$OUT/wpc1.log" "$OUT/wpc2.log" | grep -v amdgpu | cut -c1-150
run() {
  local name="$1"; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
for r in 1 2; do
  run base_$r KFB_IGEMM_NOS1=1
  run s1_$r KFB_IGEMM_NOS1=0
  run s1w1_$r KFB_S1_WPC=1
done
