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


def test_geometric_tail_buckets():
    """Buckets are cut from the end of the ready order with caps growing
    from tail_mb: the last bucket (its all-reduce is exposed after backward)
    stays small, every element is covered once, in order."""
    mb = 1 << 18  # elements per MB (fp32)
    flat = _Flat([mb // 4] * 200)  # 50 MB in 0.25 MB parameters
    red = BucketReducer(flat, bucket_mb=16, tail_mb=1)
    sizes = [(e - s) / mb for s, e in red.buckets]
    assert sizes[-4:] == [8.0, 4.0, 2.0, 1.0]
    assert all(s <= 16 for s in sizes)
    assert red.buckets[0][0] == 0 and red.buckets[-1][1] == flat.numel
    assert all(a[1] == b[0] for a, b in zip(red.buckets, red.buckets[1:]))
    assert sum(red.sizes) == 200
    # tail_mb=0: the size-capped layout, cut from the end
    red0 = BucketReducer(flat, bucket_mb=16, tail_mb=0)
    assert [(e - s) / mb for s, e in red0.buckets] == [2.0, 16.0, 16.0, 16.0]
