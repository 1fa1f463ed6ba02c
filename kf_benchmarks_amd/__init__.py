"""kf_benchmarks_amd: an MI355X-native CNN training benchmark framework.

Capabilities of tf_cnn_benchmarks + KungFu (Panlichen/kf-benchmarks),
re-designed for AMD Instinct MI355X (gfx950): PyTorch-ROCm eager execution,
hand-written HIP/CDNA4 kernels for the hot ops, RCCL over xGMI for
data-parallel training, one process per GPU.
"""

import os as _os

__version__ = "0.1.0"

# Hardware queues per process.  A training step runs on several streams at
# once (compute, weight-gradient side stream, RCCL's streams, input copies);
# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default) in
# creation order, and two streams sharing a queue serialize.  With RCCL's
# streams present, 4 queues put the weight-gradient stream behind the dgrad
# chain (ResNet-50 bs256 with a 1-rank RCCL group: 22.3 ms/step at 4 queues,
# 21.4 at 8, 20.8 without RCCL).  Must be set before HIP initializes, i.e.
# before the first GPU call of the process.  KFB_HW_QUEUES overrides
# (clamped to 1..32).
_q = _os.environ.get("KFB_HW_QUEUES")
if _q is None:
    try:
        _cur = int(_os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        _cur = 4
    _q = max(_cur, 8)
_os.environ["GPU_MAX_HW_QUEUES"] = str(min(max(int(_q), 1), 32))  # HIP allows 1..32
del _q
