"""Probe: does a native RCCL collective block the host?  Queues ~40 ms of
GPU work, then times the host cost of 7 all-reduces (native communicator or
torch's ProcessGroupNCCL) with no synchronize in between.  A non-blocking
enqueue costs tens of microseconds; a blocking one costs the queued work.
1-rank group (KFB_FORCE_PG=1 semantics: WORLD_SIZE=1, MASTER_* set here)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29655")
os.environ["KFB_FORCE_PG"] = "1"
import torch  # noqa: E402
from kf_benchmarks_amd.parallel import comm  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "native"  # native | native_lowprio | torch
os.environ["KFB_NATIVE_COMM"] = "0" if mode == "torch" else "1"
w = comm.init_world("cuda", device_index=0)
dev = torch.device("cuda", 0)
if mode == "native_lowprio":  # same communicator, an ordinary-priority stream
    w.native.stream = torch.cuda.Stream(dev)
    w.native.stream_h = w.native.stream.cuda_stream
print(mode, "native comm" if w.native is not None else "torch group", flush=True)
bufs = [torch.ones(6 << 20, device=dev) for _ in range(7)]
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
for it in range(4):
    torch.cuda.synchronize()
    for _ in range(40):  # ~queued GPU work
        a = (a @ a).clamp_(-1, 1)
    t0 = time.perf_counter()
    works = [comm.all_reduce(b, async_op=True) for b in bufs]
    t1 = time.perf_counter()
    for wk in works:
        if wk is not None:
            wk.wait()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print("%s iter %d: enqueue 7 all-reduces %.3f ms, waits %.3f ms, drain %.3f ms"
          % (mode, it, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2)), flush=True)
w.shutdown()
