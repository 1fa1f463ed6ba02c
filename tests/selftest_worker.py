"""One gloo rank of tests/test_comm_selftest.py: the native-communicator
startup self-test (parallel/comm.py) against a candidate communicator that
is correct, or wrong on one rank.

usage: selftest_worker.py <out.json> <good|bad>"""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


class _Work:
    def wait(self):
        pass


class FakeComm:
    """A device communicator stand-in over the gloo group (host tensors);
    ``bad_rank`` corrupts its sum all-reduce results of large buffers."""

    def __init__(self, rank, bad_rank=-1):
        self.rank, self.bad_rank, self.closed = rank, bad_rank, False
        self.device = None

    def all_reduce(self, t, op="sum"):
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op])
        if op == "sum" and self.rank == self.bad_rank and t.numel() > 1000:
            t[7] += 1
        return _Work()

    def broadcast(self, t, src=0):
        dist.broadcast(t, src)
        return _Work()

    def barrier(self):
        dist.barrier()

    def close(self, abort=False):
        self.closed = True


def main():
    out, kind = sys.argv[1], sys.argv[2]
    from kf_benchmarks_amd.parallel import comm
    w = comm.init_world("cpu")
    cand = FakeComm(w.rank, bad_rank=1 if kind == "bad" else -1)
    sizes = [1, 4097, 1 << 16]
    st = comm.selftest_device_collectives(cand, sizes, (torch.float32, torch.bfloat16))
    # the bench/CLI path: validate_native on the world's communicator
    os.environ["KFB_NATIVE_COMM"] = "auto"
    w.native = cand
    v = comm.validate_native(sizes)
    res = {"selftest": st, "validate": v, "native_after": w.native is not None,
           "closed": cand.closed, "backend": w.device_backend}
    with open(out, "w") as f:
        json.dump(res, f)
    w.native = None
    w.shutdown()


if __name__ == "__main__":
    main()
