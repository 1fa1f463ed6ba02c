#!/bin/bash
# Round-6 session: 1-rank native RCCL A/B (comm stream priority, collectives
# on the caller's stream, exposed-time probe off) against torch's group, and
# the DeepSpeech2 GPU tests fixed after r13f.  Each GPU step under its own
# time limit; fault / abort / timeout stops the script.
# (The KFB_AB_* switches were temporary and were removed after this A/B.)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r13g"; mkdir -p "$OUT"
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
B="python bench.py --steps 20 --warmup 6"
step torchpg_eager 200 env KFB_FORCE_PG=1 KFB_NATIVE_COMM=0 $B
step native_eager 200 env KFB_FORCE_PG=1 $B --launch_tape 0
step native_prio0 200 env KFB_FORCE_PG=1 KFB_AB_COMM_PRIO=0 $B --launch_tape 0
step native_same 200 env KFB_FORCE_PG=1 KFB_AB_COMM_SAME=1 $B --launch_tape 0
step native_noprobe 200 env KFB_FORCE_PG=1 KFB_AB_PROBE=0 $B --launch_tape 0
step native_taped_prio0 200 env KFB_FORCE_PG=1 KFB_AB_COMM_PRIO=0 $B
step native_taped_same 200 env KFB_FORCE_PG=1 KFB_AB_COMM_SAME=1 $B
step pytest 400 python -u -m pytest tests/test_tape_gpu.py::test_deepspeech2_with_launch_tape tests/test_rnn.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread
echo done
