#!/bin/bash
# round-4 benches: tape host profile (raw vs entry), bench A/B (S7 + BN fold + raw tape), real data
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10o}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name="$1"; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
run tprof_raw KFB_TAPE_PROFILE=1 KFB_TAPE_RAW=1
grep "tape host time" "$OUT/tprof_raw.log"
run tprof_entry KFB_TAPE_PROFILE=1 KFB_TAPE_RAW=0
grep "tape host time" "$OUT/tprof_entry.log"
for r in 1 2; do
  run base_$r KFB_IGEMM_NOS7=1 KFB_BN_FOLD=0 KFB_TAPE_RAW=0
  run new_$r KFB_IGEMM_NOS7=0 KFB_BN_FOLD=1 KFB_TAPE_RAW=1
  run s7_$r KFB_IGEMM_NOS7=0 KFB_BN_FOLD=0 KFB_TAPE_RAW=1
done
timeout -k 10 300 python -u scripts/make_imagenet_like.py /tmp/imnet 2048 8 > "$OUT/mkdata.log" 2>&1 || exit 1
run_real() {
  local name="$1" extra="$2"; shift 2
  env "$@" timeout -k 10 400 python bench.py --steps 20 --warmup 8 --data_dir /tmp/imnet --input_threads 16 $extra > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/$name.log") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log") $(grep -o '"launch_tape": [a-z]*' "$OUT/$name.log")"
  case $rc in 0) ;; *) exit $rc;; esac
}
run_real real_gpujpeg "" KFB_GPU_JPEG=1 KFB_TAPE_RAW=1
run_real real_hostjpeg "" KFB_GPU_JPEG=0 KFB_TAPE_RAW=1
run_real real_gpujpeg_eager "--launch_tape 0" KFB_GPU_JPEG=1 KFB_TAPE_RAW=1
