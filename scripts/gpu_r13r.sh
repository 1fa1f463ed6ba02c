#!/bin/bash
# Round-6 session: depthwise filter gradient for any filter width (column
# groups): its tests and the MobileNet / NASNet benches.  Each GPU step under
# its own time limit; fault / abort / timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r13r"; mkdir -p "$OUT"
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
step pytest 300 python -u -m pytest tests/test_conv_gpu.py -k depthwise -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" "$OUT/pytest.log" && ! grep -q " failed" "$OUT/pytest.log" || { echo "tests failed, stopping"; exit 1; }
step mobilenet 300 python bench.py --model mobilenet --batch_size 128 --steps 10 --warmup 3
step nasnet 300 python bench.py --model nasnet --batch_size 64 --steps 10 --warmup 3
echo done
