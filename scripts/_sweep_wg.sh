# wgrad launch-shape sweep (scratch): tests first, then conv bench per setting
set -e
mkdir -p gpurun_out/sweep4
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py -x -q -p no:cacheprovider > gpurun_out/sweep4/pytest.log 2>&1
tail -2 gpurun_out/sweep4/pytest.log
for b in 384 512 768 1024 1536; do
  KFB_WGRAD_BLOCKS=$b timeout -k 10 300 python scripts/bench_conv.py --hip_only --json gpurun_out/sweep4/wg_$b.json > gpurun_out/sweep4/wg_$b.log 2>&1
  echo "blocks $b done"
done
