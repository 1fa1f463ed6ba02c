#!/bin/bash
# Round-6 session: ReLU6 applied by the BN (MobileNet-v2) - the BN kernel
# tests, the MobileNet equivalence test, then the rest of the model zoo.
# Each GPU step under its own time limit; fault / abort / timeout stops
# the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r13n"; mkdir -p "$OUT"
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
step pytest 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_fin_gpu.py tests/test_conv_gpu.py::test_bn_apply_writes_relu_bits -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" "$OUT/pytest.log" && ! grep -q " failed" "$OUT/pytest.log" || { echo "tests failed, stopping"; exit 1; }
bash scripts/zoo_bench.sh zoo_r13b mobilenet:128 nasnet:64 googlenet:128 vgg11:128 vgg16:128 vgg19:128 alexnet:512 overfeat:256 nasnetlarge:16 trivial:256 lenet:256 ncf:2048 deepspeech2:16 || exit $?
echo done
