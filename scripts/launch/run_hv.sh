#!/bin/bash
# One-node Horovod-mode job (role of tcb/run_hv.sh, which runs `mpirun -np N
# python3 tf_cnn_benchmarks.py --variable_update=horovod`): N ranks, one per
# MI355X, summed gradient all-reduce over RCCL/xGMI.  torch.distributed.run
# plays mpirun's part (rank / local rank / world size in the environment).
#SBATCH --job-name=kfb-horovod
#SBATCH --nodes=1
#SBATCH --gres=gpu:8
#SBATCH --exclusive
#   usage: scripts/launch/run_hv.sh [np] [model] [batch per GPU]
set -euo pipefail
NP="${1:-8}"; MODEL="${2:-resnet50}"; BS="${3:-256}"
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m kf_benchmarks_amd.build
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NP" \
    --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29511}" \
    tf_cnn_benchmarks.py --model="$MODEL" --batch_size="$BS" --num_gpus=1 --use_bf16 \
    --optimizer=momentum --variable_update=horovod --num_warmup_batches=10 \
    --num_batches=100 --display_every=10
