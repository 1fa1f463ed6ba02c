#!/bin/bash
# Interleaved A/B of bench.py in one GPU session (same box, same clocks):
#   usage: scripts/ab_bench.sh <tag> "<env A>" "<env B>" [rounds] [bench args...]
# e.g. scripts/ab_bench.sh ab1 "KFB_MASK_RECOMPUTE=0" "KFB_MASK_RECOMPUTE=1" 3
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="$1"; A="$2"; B="$3"; R="${4:-3}"; shift 4 || shift $#
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for v in A B; do
    if [ "$v" = A ]; then E="$A"; else E="$B"; fi
    # "--..." variants are bench.py arguments, anything else environment assignments
    if [ "${E#--}" != "$E" ]; then ARGS="$E"; ENVS=""; else ARGS=""; ENVS="$E"; fi
    env $ENVS timeout -k 10 300 python bench.py --steps 30 --warmup 8 $ARGS "$@" > "$OUT/$v$r.log" 2>&1 || exit $?
    echo "$v ($E) round $r: $(grep -o '"value": [0-9.]*' "$OUT/$v$r.log")"
  done
done
