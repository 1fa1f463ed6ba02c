#!/bin/bash
# Short 1-GPU training runs of the model zoo (bf16, synthetic data).  Each
# model runs under its own time limit; a fault/timeout stops the script.
#   usage: scripts/zoo_bench.sh <tag> [model:batch[:extra,bench,args] ...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-zoo}"; shift || true
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
MODELS="${*:-mobilenet:128 nasnet:64 official_resnet50:128 resnet152:128 vgg16:128 inception3:128 googlenet:128 alexnet:512}"
for mb in $MODELS; do
  IFS=: read -r m b extra <<< "$mb"
  extra="${extra//,/ }"
  echo "== $m bs $b $extra"
  timeout -k 10 300 python bench.py --model "$m" --batch_size "$b" --steps 10 --warmup 3 $extra \
      > "$OUT/${m}_${b}.log" 2>&1
  rc=$?
  tail -n 1 "$OUT/${m}_${b}.log"
  case $rc in 0) ;; 124|134|137|139) echo "FATAL rc=$rc in $m"; exit $rc;; *) echo "rc=$rc";; esac
done
echo done
