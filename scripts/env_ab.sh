#!/bin/bash
# Interleaved A/B of one environment switch on bench.py:
#   usage: scripts/env_ab.sh <tag> <VAR> <valA> <valB> <rounds> <bench args...>
# Each round runs A then B; every run's JSON line goes to gpurun_out/<tag>/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="$1"; VAR="$2"; A="$3"; B="$4"; ROUNDS="$5"; shift 5
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 300 python bench.py "$@" > "$OUT/${VAR}_${v}_$r.log" 2>&1
    rc=$?
    echo "== $VAR=$v round $r rc=$rc: $(tail -n 1 "$OUT/${VAR}_${v}_$r.log" | cut -c1-160)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
