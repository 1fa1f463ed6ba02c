#!/bin/bash
# kernel-trace profiles: ResNet-50 bs256 BN fold on vs off; ResNet-152 bs32 (small-batch step)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10u}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
prof() {
  local name="$1" args="$2"; shift 2
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$name" -o run -- python bench.py --steps 10 --warmup 5 $args > "$OUT/$name.log" 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log"
}
prof off "" KFB_BN_FOLD=0
prof fold "" KFB_BN_FOLD=1
prof r152 "--model resnet152 --batch_size 32"
python scripts/prof_db.py "$OUT/off/run_results.db" "$OUT/fold/run_results.db" --top 45 > "$OUT/fold_vs_off.txt" 2>&1
python scripts/prof_db.py "$OUT/r152/run_results.db" --top 45 > "$OUT/r152.txt" 2>&1
head -50 "$OUT/fold_vs_off.txt"
head -50 "$OUT/r152.txt"
