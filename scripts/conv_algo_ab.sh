#!/bin/bash
# Per-layer conv times with the autotuned choice and with each named igemm
# kernel forced (KFB_IGEMM_ALGO), HIP kernels only.
#   usage: scripts/conv_algo_ab.sh <tag> <algo> [<algo> ...]   (algo "auto" = autotune)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
for algo in "$@"; do
  if [ "$algo" = auto ]; then unset KFB_IGEMM_ALGO; else export KFB_IGEMM_ALGO=$algo; fi
  timeout -k 10 300 python scripts/bench_conv.py --hip_only --json "$OUT/$algo.json" > "$OUT/$algo.log" 2>&1
  rc=$?
  echo "== $algo rc=$rc"; tail -n 2 "$OUT/$algo.log"
  case $rc in 0) ;; *) exit $rc;; esac
done
