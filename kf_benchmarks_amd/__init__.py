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
# before the first GPU call of the process.  Precedence: KFB_HW_QUEUES, then
# a GPU_MAX_HW_QUEUES other than HIP's own default of 4 (respected as is;
# some environments export the default explicitly, and that is not a
# choice: ask for exactly 4 with KFB_HW_QUEUES=4), then 8.  Clamped to 1..32.


def _set_hw_queues():
    import sys
    import warnings
    v = _os.environ.get("KFB_HW_QUEUES")
    if v is None and _os.environ.get("GPU_MAX_HW_QUEUES", "4").strip() != "4":
        return  # the user's explicit choice
    try:
        q = int(v) if v is not None else 8
    except ValueError:
        warnings.warn("KFB_HW_QUEUES=%r is not an integer; using 8" % v)
        q = 8
    torch = sys.modules.get("torch")
    if torch is not None and getattr(torch, "cuda", None) is not None:
        try:
            if torch.cuda.is_initialized():
                warnings.warn("kf_benchmarks_amd imported after the GPU runtime started: "
                              "GPU_MAX_HW_QUEUES=%d has no effect in this process" % q)
        except Exception:  # noqa: BLE001
            pass
    _os.environ["GPU_MAX_HW_QUEUES"] = str(min(max(q, 1), 32))


_set_hw_queues()
