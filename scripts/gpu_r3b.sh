set -u
mkdir -p gpurun_out/r3b
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r3b/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r3b/pytest.log; echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
KFB_FORCE_PG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/r3b/bench_forcepg.log 2>&1
rc=$?; tail -2 gpurun_out/r3b/bench_forcepg.log; echo "bench rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/r3b/bench_gpus2.log 2>&1
echo "gpus2 rc=$? (expect 2)"; tail -2 gpurun_out/r3b/bench_gpus2.log
