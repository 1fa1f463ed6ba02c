#!/bin/bash
# Generic GPU-box driver: runs the named steps in order, each under its own
# time limit; a fault / abort / timeout ends the script (no further GPU work).
#   usage: scripts/gpu_steps.sh <tag> <step>...
#   step:  pytest:<pytest args...> | bench:<bench.py args...> | prof:<bench.py args...>
#          | py:<python args...> | smoke:   (env VAR=value pairs may prefix bench/prof args)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
n=0
for spec in "$@"; do
  n=$((n + 1))
  kind="${spec%%:*}"; args="${spec#*:}"
  log="$OUT/$n.$kind.log"
  echo "== step $n $kind: $args"
  case "$kind" in
    pytest) timeout -k 10 900 python -u -m pytest $args -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$log" 2>&1 ;;
    bench) env $(echo "$args" | tr ' ' '\n' | grep '=' | grep -v '^--') timeout -k 10 600 python bench.py $(echo "$args" | tr ' ' '\n' | grep -v '^[A-Z_]*=' ) > "$log" 2>&1 ;;
    smoke) timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    py) env $(echo "$args" | tr ' ' '\n' | grep '^[A-Z_][A-Z0-9_]*=' ) timeout -k 10 600 python $(echo "$args" | tr ' ' '\n' | grep -v '^[A-Z_][A-Z0-9_]*=' ) > "$log" 2>&1 ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
         -d "$OUT/prof$n" -o run -- python3 "$ROOT/bench.py" $args) > "$log" 2>&1 ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
  rc=$?
  echo "== step $n rc=$rc"; tail -n 6 "$log"
  if [ "$kind" = prof ] && [ $rc -eq 0 ]; then
    f=$(find "$OUT/prof$n" -name "*kernel_trace.csv" | head -n 1)
    [ -n "$f" ] && python3 scripts/kernel_stats.py "$f" --last-steps 4 --top 40 > "$OUT/kernel_summary$n.txt" && head -n 25 "$OUT/kernel_summary$n.txt"
    [ -n "$f" ] && (cd scripts && python3 step_overlap.py "$f" > "$OUT/overlap$n.txt" 2>&1; head -n 8 "$OUT/overlap$n.txt")
    rm -f "$OUT"/prof$n/*kernel_stats.csv "$OUT"/prof$n/*domain_stats.csv
  fi
  case $rc in 124|134|137|139) echo "FATAL in step $n, stopping"; exit $rc;; esac
done
echo done
