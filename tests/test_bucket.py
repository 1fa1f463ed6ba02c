"""BucketReducer readiness bookkeeping (CPU, single process)."""

import torch

from kf_benchmarks_amd.parallel.bucket import BucketReducer


class _Flat:
    def __init__(self, sizes):
        self.params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
        self.offsets, off = [], 0
        for n in sizes:
            self.offsets.append(off)
            off += n
        self.numel = off
        self.grad = torch.zeros(off)

    def segments(self):
        return [("p%d" % i, p, o, p.numel())
                for i, (p, o) in enumerate(zip(self.params, self.offsets))]


def test_each_parameter_counts_once_per_backward():
    """A direct-sink parameter reports through _kfb_ready_cb and then again
    through autograd's post-accumulate hook; the second report must not
    count, or a bucket launches before its other gradients exist."""
    flat = _Flat([16, 16, 16, 16])
    red = BucketReducer(flat, bucket_mb=32 * 4 / float(1 << 20))  # 2 params per bucket
    assert red.num_buckets == 2
    launched = []
    red._launch = lambda b, src=None: launched.append(b)
    red.begin()
    p0, p1, p2, p3 = flat.params
    p0._kfb_ready_cb(p0)
    red._hook(p0)  # duplicate report of the same parameter
    assert launched == []
    p1._kfb_ready_cb(p1)
    assert launched == [0]
    red._hook(p2)
    red._hook(p2)
    assert launched == [0]
    red._hook(p3)
    assert launched == [0, 1]
    red.finish()
    # next backward: counts re-armed
    red.begin()
    for p in flat.params:
        red._hook(p)
    assert launched == [0, 1, 0, 1]
