#!/bin/bash
# HBM bytes per kernel of one training step: two rocprofv3 counter passes
# (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2: one pass each) over a short
# bench run with kernel traces, then scripts/bytes_roofline.py joins them.
#   usage: scripts/pmc_bytes.sh <tag> [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pass $c"
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/$c" -o run -- \
      python3 "$ROOT/bench.py" --steps 2 --warmup 4 "$@" > "$OUT/$c.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$c.log"; exit $rc; fi
done
python3 "$ROOT/scripts/bytes_roofline.py" "$OUT" > "$OUT/bytes_roofline.txt"
rm -f "$OUT"/*/run_kernel_stats.csv "$OUT"/*/run_domain_stats.csv "$OUT"/*/run_agent_info.csv
echo done
