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

    def reduce(self, t, dst=0, op="sum"):
        dist.reduce(t, dst, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op])
        return _Work()

    def broadcast(self, t, src=0):
        dist.broadcast(t, src)
        return _Work()

    def barrier(self):
        dist.barrier()

    def close(self, abort=False):
        self.closed = True


# VGG-16 (BASELINE #5) variable sizes in the flat model's order: 13 3x3
# convs and 3 FC layers, each a kernel then a bias
_VGG16 = []
for cin, cout in ((3, 64), (64, 64), (64, 128), (128, 128), (128, 256), (256, 256), (256, 256),
                  (256, 512), (512, 512), (512, 512), (512, 512), (512, 512), (512, 512)):
    _VGG16 += [9 * cin * cout, cout]
for fin, fout in ((25088, 4096), (4096, 4096), (4096, 1001)):
    _VGG16 += [fin * fout, fout]


class _Seg:
    pass


class _FakeFlat:
    """Just enough of optim.FlatParams for BucketReducer's bucket cut."""

    def __init__(self, numels):
        self._segs, off = [], 0
        for i, n in enumerate(numels):
            self._segs.append(("v%d" % i, _Seg(), off, n))
            off += n
        self.numel = off

    def segments(self):
        return self._segs


def vgg16_bucket_sizes(bucket_mb=25.0):
    from kf_benchmarks_amd.parallel.bucket import BucketReducer
    r = BucketReducer(_FakeFlat(_VGG16), bucket_mb, overlap=False)
    return sorted({e - s for s, e in r.buckets} | {1, sum(_VGG16)})


def main():
    out, kind = sys.argv[1], sys.argv[2]
    from kf_benchmarks_amd.parallel import comm
    w = comm.init_world("cpu")
    if kind == "vgg16":
        # the startup cost on the largest BASELINE model must not grow with
        # it: every distinct bucket size, fp32 and the fp16 wire dtype
        import time
        sizes = vgg16_bucket_sizes()
        cand = FakeComm(w.rank)
        t0 = time.time()
        st = comm.selftest_device_collectives(cand, sizes, (torch.float32, torch.float16))
        took = time.time() - t0
        with open(out, "w") as f:
            json.dump({"selftest": st, "seconds": took, "sizes": sizes}, f)
        w.shutdown()
        return
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
