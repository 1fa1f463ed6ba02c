#!/bin/bash
# real-data run under the kernel tracer: the JPEG reconstruction kernels' share of the step
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r11e}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u scripts/make_imagenet_like.py /tmp/imnet 2048 8 > "$OUT/mkdata.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python bench.py --steps 20 --warmup 8 --data_dir /tmp/imnet --input_threads 16 > "$OUT/bench.log" 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$OUT/bench.log"
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -25 "$f" | cut -c1-200
