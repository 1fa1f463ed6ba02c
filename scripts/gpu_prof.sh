#!/bin/bash
# kernel-trace profile of the headline bench: gpurun_out/<tag>/prof/run_results.db
# (+ the autotune log); summarize with scripts/prof_db.py
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-prof}"; shift || true
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
env "$@" KFB_AUTOTUNE_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof" -o run -- python bench.py --steps 10 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' "$OUT/bench.log"
