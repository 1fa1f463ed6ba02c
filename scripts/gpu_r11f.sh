#!/bin/bash
# two-pass GPU JPEG reconstruction: bitwise test, real-data bench, kernel times
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r11f}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q -p no:cacheprovider --timeout-method thread --timeout 120 tests/test_jpeg_path.py -m gpu > "$OUT/jpegtest.log" 2>&1
rc=$?; echo "jpegtest rc=$rc"; tail -2 "$OUT/jpegtest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/make_imagenet_like.py /tmp/imnet 2048 8 > "$OUT/mkdata.log" 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 8 --data_dir /tmp/imnet --input_threads 16 > "$OUT/real_$r.log" 2>&1 || exit $?
  echo "real_$r $(grep -o '"value": [0-9.]*' "$OUT/real_$r.log") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/real_$r.log")"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof" -o run -- python bench.py --steps 10 --warmup 5 --data_dir /tmp/imnet --input_threads 16 > "$OUT/prof.log" 2>&1 || exit $?
echo prof done
