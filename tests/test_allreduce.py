"""All-reduce spec / packing utilities and in-process batch all-reduce
algorithms (tcb/allreduce_test.py, VariableMgrLocalReplicatedTest of
tcb/benchmark_cnn_test.py:1368-1476)."""

import pytest
import torch

from kf_benchmarks_amd import constants, params as P
from kf_benchmarks_amd.parallel import allreduce, batch_allreduce


def test_group_key():
    d0 = ["/job:worker/replica:0/task:0/device:GPU:%d" % i for i in (1, 0, 3)]
    d1 = ["/job:worker/replica:0/task:1/device:GPU:%d" % i for i in (1, 0, 3)]
    d2 = ["/job:worker/replica:0/task:1/device:GPU:%d" % i for i in (1, 3, 0)]
    d3 = ["/job:worker/replica:0/task:1/device:GPU:%d" % i for i in (1, 3, 2)]
    d4 = ["/job:worker/task:0/device:GPU:%d" % i for i in (1, 2, 3)]
    d5 = ["/job:worker/task:0/device:CPU:1", "/job:worker/task:0/device:CPU:2"]
    d6 = ["/job:worker/task:0/device:CPU:2", "/job:worker/task:0/device:CPU:1"]
    g = [allreduce.collective_group_key(d) for d in (d0, d1, d2, d3, d4, d5, d6)]
    assert g[0] == g[1] == g[2] and g[0] != g[3] and g[3] == g[4] and g[5] == g[6]
    assert g[4] != g[5]


@pytest.mark.parametrize("x,ranges,singles", [
    ([], [], []), ([1, 3, 4, 6, 7, 8, 9], [[3, 4], [6, 9]], [1]),
    ([1, 2, 3, 4, 6, 7, 8, 9], [[1, 4], [6, 9]], []),
    ([1, 3, 4, 6, 7, 9], [[3, 4], [6, 7]], [1, 9]), ([1, 3, 6, 9], [], [1, 3, 6, 9])])
def test_extract_ranges(x, ranges, singles):
    assert allreduce.extract_ranges(x) == (ranges, singles)


def _t(*vals, shape=None):
    t = torch.tensor(vals, dtype=torch.float32)
    return t.reshape(shape) if shape else t


T0, T1 = _t(0, 1, 2, 3), _t(4, 5, 6, 7)
T2 = torch.arange(9, dtype=torch.float32).reshape(3, 3)


def test_pack_range_and_unpack():
    packing = {}
    new = allreduce.pack_range("0:0", packing, [(T0, "v0"), (T1, "v1")], [0, 1])
    assert new.shape == (8,)
    assert packing == {"0:0": allreduce.GradPackTuple(range(2), ["v0", "v1"], [(4,), (4,)])}
    packing = {}
    gv = [(T0, "v0"), (T1, "v1"), (T2, "v2"), (T2.clone(), "v3")]
    new = allreduce.pack_range("1:0", packing, gv, [0, 3])
    assert new.shape == (26,)
    out = allreduce.unpack_grad_tuple((new, "packing_var_placeholder"), packing["1:0"])
    assert [v for _, v in out] == ["v0", "v1", "v2", "v3"]
    assert [tuple(g.shape) for g, _ in out] == [(4,), (4,), (3, 3), (3, 3)]
    assert torch.equal(out[2][0], T2)


def test_pack_small_tensors():
    towers = [[(T0, "v_%d_0" % d), (T1, "v_%d_1" % d), (T2, "v_%d_2" % d), (T2, "v_%d_3" % d)]
              for d in range(3)]
    new, packing = allreduce.pack_small_tensors(towers, max_bytes=12, max_group=10)
    assert new is towers and packing is None
    new, packing = allreduce.pack_small_tensors(towers, max_bytes=16, max_group=10)
    assert len(new) == 3 and len(new[0]) == 3 and new[0][0][0].shape == (8,)
    assert packing["2:0"] == allreduce.GradPackTuple(range(2), ["v_2_0", "v_2_1"], [(4,), (4,)])
    new, packing = allreduce.pack_small_tensors(towers, max_bytes=256, max_group=10)
    assert len(new[0]) == 1 and new[0][0][0].shape == (26,)
    restored = allreduce.unpack_small_tensors(new, packing)
    for d in range(3):
        assert [v for _, v in restored[d]] == ["v_%d_%d" % (d, i) for i in range(4)]


def test_unpack_small_tensors_interleaved():
    packing = {}
    for d in range(2):
        packing["%d:0" % d] = allreduce.GradPackTuple(range(2), ["v_%d_0" % d, "v_%d_1" % d],
                                                      [(4,), (4,)])
        packing["%d:1" % d] = allreduce.GradPackTuple(range(3, 5), ["v_%d_3" % d, "v_%d_4" % d],
                                                      [(3, 3), (3, 3)])
    t0 = torch.arange(8, dtype=torch.float32)
    t2 = torch.cat([torch.arange(9.0), torch.arange(9.0)])
    towers = [[(t0, "p"), (t2, "p"), (_t(17, 17), "v_%d_2" % d), (_t(0), "v_%d_5" % d)]
              for d in range(2)]
    out = allreduce.unpack_small_tensors(towers, packing)
    for d, tg in enumerate(out):
        assert [v for _, v in tg] == ["v_%d_%d" % (d, i) for i in range(6)]
        assert [tuple(g.shape) for g, _ in tg] == [(4,), (4,), (2,), (3, 3), (3, 3), (1,)]


def test_parse_spec():
    assert allreduce.parse_general_int("32k") == 32768
    assert allreduce.parse_general_int("2M") == 2 << 20
    s = allreduce.parse_all_reduce_spec("psgpu#4:32k:xring")
    assert s == [allreduce.AllReduceSpecTuple("psgpu", 4, 32768),
                 allreduce.AllReduceSpecTuple("xring", 1, -1)]
    with pytest.raises(ValueError):
        allreduce.parse_all_reduce_spec("bogus")
    with pytest.raises(ValueError):
        allreduce.parse_all_reduce_spec("nccl:32k")
    assert allreduce.rccl_env_for_spec("xring#2") == {"NCCL_ALGO": "Ring",
                                                      "NCCL_MIN_NCHANNELS": "2"}


def test_group_device_names_and_split_by_size():
    g = allreduce.group_device_names(["a", "b", "c"], 2)
    assert g == [["a", "c"], ["b", "a"]]
    with pytest.raises(ValueError):
        allreduce.group_device_names(["a"], 2)
    small, large = allreduce.split_grads_by_size(4, [[(T0, "a"), (T2, "b")]])
    assert [v for _, v in small[0]] == ["a"] and [v for _, v in large[0]] == ["b"]


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8, 10])
def test_reduction_algorithms_exact(n):
    ts = [torch.arange(13, dtype=torch.float32) * (i + 1) for i in range(n)]
    ref = sum(ts)
    for fn in (allreduce.reduce_ring, allreduce.reduce_halving_doubling, allreduce.reduce_nccl,
               lambda t: allreduce.reduce_shuffle(t, [torch.device("cpu")] * 2, 4)):
        for out in fn(ts):
            assert torch.equal(out, ref)


def _tower_grads(num_towers=10):
    # tower d: tensor j = constant (d + 1) * (j + 1), shapes vary
    shapes = [(4,), (3, 3), (1,), (2, 5), (7,)]
    return [[torch.full(s, float((d + 1) * (j + 1))) for j, s in enumerate(shapes)]
            for d in range(num_towers)]


def _expected(grads):
    n = len(grads)
    tot = n * (n + 1) / 2
    return [[torch.full(t.shape, tot * (j + 1)) for j, t in enumerate(grads[0])]
            for _ in range(n)]


@pytest.mark.parametrize("kw", [
    dict(), dict(gradient_repacking=2), dict(gradient_repacking=2, compact_gradient_transfer=True),
    dict(all_reduce_spec="pscpu"), dict(all_reduce_spec="xring"),
    dict(all_reduce_spec="nccl/rechd"), dict(all_reduce_spec="psgpu#4"),
    dict(all_reduce_spec="nccl", agg_small_grads_max_bytes=64),
    dict(all_reduce_spec="pscpu/pscpu"), dict(all_reduce_spec="nccl/xring"),
    dict(hierarchical_copy=True, num_gpus=8, network_topology="dgx1"),
    dict(hierarchical_copy=True, num_gpus=8, network_topology="gcp_v100"),
    dict(hierarchical_copy=True, num_gpus=8, network_topology="xgmi_mesh")])
def test_batch_all_reduce_sums(kw):
    kw = dict(kw)
    towers = 8 if kw.get("hierarchical_copy") else 10
    kw.setdefault("num_gpus", towers)
    repack = kw.pop("gradient_repacking", 0)
    compact = kw.pop("compact_gradient_transfer", False)
    params = P.make_params(**kw)
    alg = batch_allreduce.algorithm_from_params(params)
    grads = _tower_grads(towers)
    out, _ = alg.batch_all_reduce(grads, repack, compact, False)
    for got, exp in zip(out, _expected(grads)):
        for g, e in zip(got, exp):
            assert g.shape == e.shape and g.dtype == torch.float32
            torch.testing.assert_close(g, e, rtol=1e-3 if compact else 0, atol=0)


def test_batch_all_reduce_deferred():
    alg = batch_allreduce.CopyToDeviceAlgorithm(["/cpu:0"])
    g1 = _tower_grads(3)
    out1, _ = alg.batch_all_reduce(g1, 0, False, True)
    assert all(float(t.abs().sum()) == 0 for dt in out1 for t in dt)
    g2 = [[t * 2 for t in dt] for dt in g1]
    out2, _ = alg.batch_all_reduce(g2, 0, False, True)
    for got, exp in zip(out2, _expected(g1)):
        for g, e in zip(got, exp):
            assert torch.equal(g, e)


def test_hierarchical_requires_eight_on_gcp():
    alg = batch_allreduce.HierarchicalCopyAlgorithm(constants.NetworkTopology.GCP_V100)
    with pytest.raises(ValueError):
        alg.batch_all_reduce(_tower_grads(4))
