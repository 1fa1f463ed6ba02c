#!/bin/bash
# BN fold (all slot loads in flight) test + A/B; real-data runs (host decode exit fix, GPU JPEG eager)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10p}"
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
run() {
  local name="$1" extra="$2"; shift 2
  env "$@" timeout -k 10 400 python bench.py --steps 20 --warmup 8 $extra > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/$name.log") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log") $(grep -o '"launch_tape": [a-z]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
step probe 120 python -u scripts/tape_launch_probe.py
step realtape 400 python -u -m pytest -x -q -p no:cacheprovider --timeout-method thread --timeout 300 tests/test_tape_gpu.py -k real_data
step foldtest 400 python -u -m pytest -x -q -p no:cacheprovider --timeout-method thread --timeout 300 tests/test_bn_fin_gpu.py
for r in 1 2; do
  run off_$r "" KFB_BN_FOLD=0
  run fold_$r "" KFB_BN_FOLD=1
done
timeout -k 10 300 python -u scripts/make_imagenet_like.py /tmp/imnet 2048 8 > "$OUT/mkdata.log" 2>&1 || exit 1
R="--data_dir /tmp/imnet --input_threads 16"
run real_hostjpeg "$R" KFB_GPU_JPEG=0
run real_gpujpeg_eager "$R --launch_tape 0" KFB_GPU_JPEG=1
run real_gpujpeg "$R" KFB_GPU_JPEG=1
