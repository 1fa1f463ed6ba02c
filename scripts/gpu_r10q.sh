#!/bin/bash
# round-end checks: the full GPU tier, smoke(), the default bench, a kernel-trace profile
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r10q}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tier.log" 2>&1
rc=$?; echo "tier rc=$rc"; tail -3 "$OUT/tier.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-200
bash scripts/gpu_prof.sh "${1:-r10q}/p" && python scripts/prof_db.py "$OUT/p/prof/run_results.db" --top 60 > "$OUT/prof_summary.txt" 2>&1; head -40 "$OUT/prof_summary.txt"
