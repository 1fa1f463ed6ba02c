mkdir -p gpurun_out/r13d
timeout -k 10 720 python -u -m pytest tests/test_model_gpu.py::test_stream_and_autotune_knobs_keep_the_gradients tests/test_rnn.py tests/test_stem_gpu.py tests/test_tape_gpu.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r13d/pytest_rest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r13d/pytest_rest.log | cut -c1-300
case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/gpu_misc_r13.sh r13d
