#!/bin/bash
# Round-6 measurements on one box: DeepSpeech2 taped at bs 16, the 1-rank
# RCCL bench (exposed all-reduce under the tape), then the MIOpen bar
# (scripts/gpu_miopen_bar.sh).  Each GPU step under its own time limit; a
# fault, abort or timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-misc}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
step ds2_bs16 400 python bench.py --model deepspeech2 --batch_size 16 --steps 5 --warmup 4
step rccl_1rank 300 env KFB_FORCE_PG=1 python bench.py --steps 20 --warmup 6
bash scripts/gpu_miopen_bar.sh "$TAG" || exit $?
# probe: can two ranks share the box's one GPU over our native RCCL
# communicator (the N > 1 native + tape path)?  RCCL may refuse duplicate
# devices; the watchdog bounds any hang (KFB_COMM_TIMEOUT_S)
step rccl_2rank_1gpu 300 env HIP_VISIBLE_DEVICES=0 KFB_COMM_TIMEOUT_S=90 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 \
    --steps 10 --warmup 5 --batch_size 64
echo done
