#!/bin/bash
# Same-session MIOpen bar: every ResNet-50 conv geometry x
# fwd/dgrad/wgrad, our HIP kernels vs PyTorch/MIOpen, then whole-step
# bench.py with our kernels and with stock PyTorch ops (MIOpen convs), back
# to back on one box.  Each GPU step under its own time limit; a fault,
# abort or timeout stops the script.
#   usage: scripts/gpu_miopen_bar.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-miopen}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 6 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
step conv_vs_miopen 900 python -u scripts/bench_conv.py --iters 20 --json "$OUT/conv_vs_miopen.json"
step bench_hip 400 python bench.py --steps 30 --warmup 10
step bench_torch 600 python bench.py --steps 10 --warmup 5 --kernel_impl torch
step bench_hip2 400 python bench.py --steps 30 --warmup 10
echo done
