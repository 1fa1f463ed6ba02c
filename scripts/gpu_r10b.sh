#!/bin/bash
# S1 in-network: autotune choices + kernel-trace stats with and without S1
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10b}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
KFB_AUTOTUNE_LOG=1 timeout -k 10 300 python bench.py --steps 10 --warmup 5 > "$OUT/tune.log" 2>&1 || exit $?
grep -c autotune "$OUT/tune.log"
KFB_IGEMM_NOS1=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_s1" -o run -- python bench.py --steps 10 --warmup 5 > "$OUT/prof_s1.log" 2>&1 || exit $?
KFB_IGEMM_NOS1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_base" -o run -- python bench.py --steps 10 --warmup 5 > "$OUT/prof_base.log" 2>&1 || exit $?
ls -R "$OUT" | head -30
