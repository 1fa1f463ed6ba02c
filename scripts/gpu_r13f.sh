#!/bin/bash
# Round-6 session: the 1-rank native RCCL slowdown (does an enqueue block the
# host? stream priority? hardware queues?) and the GPU tests changed since
# r13e.  Each GPU step under its own time limit; fault / abort / timeout
# stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r13f"; mkdir -p "$OUT"
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
step probe_native 150 python -u scripts/probe_rccl_host_block.py native
step probe_lowprio 150 python -u scripts/probe_rccl_host_block.py native_lowprio
step probe_torch 150 python -u scripts/probe_rccl_host_block.py torch
step rccl_eager_q4 200 env KFB_FORCE_PG=1 KFB_HW_QUEUES=4 python bench.py --steps 20 --warmup 6 --launch_tape 0
step rccl_eager_q16 200 env KFB_FORCE_PG=1 KFB_HW_QUEUES=16 python bench.py --steps 20 --warmup 6 --launch_tape 0
step pytest 900 python -u -m pytest tests/test_model_gpu.py::test_stream_and_autotune_knobs_keep_the_gradients tests/test_model_gpu.py::test_forced_conv_kernel_in_network_keeps_the_gradients tests/test_tape_gpu.py tests/test_stem_gpu.py tests/test_rnn.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread
echo done
