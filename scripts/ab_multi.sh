#!/bin/bash
# Interleaved multi-arm A/B of bench.py in one GPU session (same box):
#   usage: scripts/ab_multi.sh <tag> <rounds> "<env arm 1>" "<env arm 2>" ...
# ("-" = no extra environment).  Every run under its own time limit; a
# fault / abort / timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="$1"; R="$2"; shift 2
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in $(seq 1 "$R"); do
  i=0
  for E in "$@"; do
    i=$((i + 1))
    ENVS=""; [ "$E" != "-" ] && ENVS="$E"
    env $ENVS timeout -k 10 300 python bench.py --steps 30 --warmup 8 > "$OUT/arm$i.r$r.log" 2>&1
    rc=$?
    case $rc in 124|134|137|139) echo "FATAL rc=$rc in arm $i round $r"; exit $rc;; esac
    echo "arm$i ($E) round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/arm$i.r$r.log")"
  done
done
