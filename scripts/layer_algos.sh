#!/bin/bash
# Every igemm kernel forced on a subset of the ResNet-50 conv shapes
# (bench_conv.py --shapes), one table per algo:
#   usage: scripts/layer_algos.sh <tag> <shape indices> <algo> [<algo> ...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="$1"; SHAPES="$2"; shift 2
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
for algo in "$@"; do
  if [ "$algo" = auto ]; then unset KFB_IGEMM_ALGO; else export KFB_IGEMM_ALGO=$algo; fi
  timeout -k 10 120 python scripts/bench_conv.py --hip_only --shapes "$SHAPES" > "$OUT/$algo.log" 2>&1 || exit $?
  echo "== $algo"; grep -E "fwd|dgrad" "$OUT/$algo.log" | grep -v shape | cut -c1-50
done
