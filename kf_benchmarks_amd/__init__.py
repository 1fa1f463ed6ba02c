"""kf_benchmarks_amd: an MI355X-native CNN training benchmark framework.

Capabilities of tf_cnn_benchmarks + KungFu (Panlichen/kf-benchmarks),
re-designed for AMD Instinct MI355X (gfx950): PyTorch-ROCm eager execution,
hand-written HIP/CDNA4 kernels for the hot ops, RCCL over xGMI for
data-parallel training, one process per GPU.
"""

__version__ = "0.1.0"
