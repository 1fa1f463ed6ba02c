#!/bin/bash
# round-9 check b: S3 tests, BN-finalize diagnosis, exact tape oracle, taped models
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r9b}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 8 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
step s3test 300 python -u -m pytest tests/test_conv_stream_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step s3bench 200 python scripts/bench_s3.py --passes wgrad
step diagfin2 300 python scripts/diag_bnfin2.py resnet50 8
step tape 500 python -u -m pytest tests/test_tape_gpu.py -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "bitwise or dropped"
step zoo_nasnet 300 python bench.py --model nasnet --batch_size 32 --steps 5 --warmup 4 --verbose
echo done
