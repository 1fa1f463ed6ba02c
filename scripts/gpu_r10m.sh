#!/bin/bash
# stem conv, raw tape replay, BN fold, dist: tests, micro-bench, bench A/B
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10l}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name="$1" t="$2"; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step jpegtest 200 python -u -m pytest tests/test_jpeg_path.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu
step s7test 300 python -u -m pytest tests/test_stem_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step s7bench 200 python -u scripts/bench_s7.py
step tapetest 500 python -u -m pytest tests/test_tape_gpu.py -x -q -p no:cacheprovider --timeout 400 --timeout-method thread -k "natively or nasnet or bitwise or raw_tape"
step foldtest 400 python -u -m pytest tests/test_bn_fin_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step disttest 600 python -u -m pytest tests/test_dist_gpu.py -x -q -p no:cacheprovider --timeout 280 --timeout-method thread -k "one_rank_rccl_is_identity or averaging_taped"
run() {
  local name="$1"; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
KFB_TAPE_PROFILE=1 step tprof_raw 300 python bench.py --steps 20 --warmup 8
KFB_TAPE_PROFILE=1 KFB_TAPE_RAW=0 step tprof_entry 300 python bench.py --steps 20 --warmup 8
for r in 1 2; do
  run base_$r KFB_IGEMM_NOS7=1 KFB_BN_FOLD=0
  run s7_$r KFB_IGEMM_NOS7=0 KFB_BN_FOLD=0
  run s7fold_$r KFB_IGEMM_NOS7=0 KFB_BN_FOLD=1
done
step mkdata 400 python -u scripts/make_imagenet_like.py /tmp/imnet 2048 8
run_real() {
  local name="$1"; shift
  env "$@" timeout -k 10 400 python bench.py --steps 20 --warmup 8 --data_dir /tmp/imnet --input_threads 16 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/$name.log") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
run_real real_gpujpeg KFB_GPU_JPEG=1
run_real real_hostjpeg KFB_GPU_JPEG=0
run_real real_gpujpeg_2 KFB_GPU_JPEG=1
