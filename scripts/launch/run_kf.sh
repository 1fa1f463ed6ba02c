#!/bin/bash
# One-node KungFu-style job (role of tcb/run_kf.sh): N peers, one per
# MI355X, synchronous SGD over RCCL/xGMI, launched by the native kfb-run
# launcher (kungfu-run compatible output prefixes and per-peer logs).
#SBATCH --job-name=kfb-kungfu
#SBATCH --nodes=1
#SBATCH --gres=gpu:8
#SBATCH --exclusive
#   usage: scripts/launch/run_kf.sh [np] [model] [batch per GPU] [kungfu option]
set -euo pipefail
NP="${1:-8}"; MODEL="${2:-resnet50}"; BS="${3:-256}"; OPT="${4:-sync_sgd}"
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m kf_benchmarks_amd.build
exec python -m kf_benchmarks_amd.parallel.launcher -np "$NP" -logdir "logs/kf_${MODEL}_np${NP}" \
    python3 tf_cnn_benchmarks.py --model="$MODEL" --batch_size="$BS" --num_gpus=1 \
    --use_bf16 --optimizer=momentum --variable_update=kungfu --kungfu_option="$OPT" \
    --num_warmup_batches=10 --num_batches=100 --display_every=10
