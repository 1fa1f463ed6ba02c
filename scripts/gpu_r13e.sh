#!/bin/bash
# Round-6 session: fixes re-run (tape oracles, forced-kernel sweep, DS2
# taped) and the 1-rank RCCL slowdown diagnosis.  Each GPU step under its
# own time limit; fault / abort / timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r13e"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-700
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
step pytest 600 python -u -m pytest tests/test_model_gpu.py -k "forced_conv_kernel or knobs" tests/test_tape_gpu.py tests/test_stem_gpu.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread
step ds2_bs16 300 python bench.py --model deepspeech2 --batch_size 16 --steps 5 --warmup 4
step rccl_taped 200 env KFB_FORCE_PG=1 python bench.py --steps 20 --warmup 6
step rccl_eager 200 env KFB_FORCE_PG=1 python bench.py --steps 20 --warmup 6 --launch_tape 0
step torchpg_eager 200 env KFB_FORCE_PG=1 KFB_NATIVE_COMM=0 python bench.py --steps 20 --warmup 6
step nopg_eager 200 python bench.py --steps 20 --warmup 6 --launch_tape 0
cd /tmp && export TMPDIR=/tmp
step prof_rccl 300 env KFB_FORCE_PG=1 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 4 --warmup 6
echo done
