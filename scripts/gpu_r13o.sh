#!/bin/bash
# Round-6 session: where the NASNet step's host time goes (tape host
# profile), and the zoo entries that need extra flags.  Each GPU step
# under its own time limit; fault / abort / timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r13o"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log" | cut -c1-700
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
step nasnet_tape_profile 300 env KFB_TAPE_PROFILE=1 python bench.py --model nasnet --batch_size 64 --steps 10 --warmup 3
bash scripts/zoo_bench.sh zoo_r13c resnet56:128:--data_name,cifar10 densenet40_k12:64:--data_name,cifar10 ncf:2048:--dtype,fp32,--optimizer,adam || exit $?
echo done
