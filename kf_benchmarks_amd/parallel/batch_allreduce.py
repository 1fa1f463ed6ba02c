"""Batch all-reduce of many gradients across in-process towers (role of
tcb/batch_allreduce.py).

``all_device_tensors[i][j]`` is tensor j on tower i; a batch all-reduce
returns the same structure with every tensor summed over towers.  Options:

* ``num_splits`` (``--gradient_repacking``): concatenate every gradient of a
  tower into one buffer and split it into ``num_splits`` equal packs before
  reducing (fewer, larger transfers), then undo;
* ``compact_tensors`` (``--compact_gradient_transfer``): reduce in fp16;
* ``defer_tensors`` (``--variable_consistency=relaxed``): return the result
  of the *previous* call (zeros the first time) - the StagingArea trick of
  tcb/batch_allreduce.py:353-389, here a per-algorithm stash.

Algorithms: :class:`CopyToDeviceAlgorithm` (reduce on owner devices,
round-robin), :class:`HierarchicalCopyAlgorithm` (two half-groups reduced on
topology-chosen main devices, cross-group sum, fan-out; DGX1 / GCP_V100 as in
the reference plus XGMI_MESH, where every pair is one xGMI hop so the main
devices simply rotate), :class:`AllReduceSpecAlgorithm` (parallel/allreduce.py).

On MI355X the production path is one process per GPU (parallel/bucket.py
implements the same repacking / compaction / deferral on RCCL buckets);
these classes serve single-process multi-tower runs and tests.
"""

from __future__ import annotations

import abc
from typing import List, Optional

import torch

from .. import constants
from . import allreduce


def _all_reduce_using_copy(tensors_across_devices, use_mean, device=None):
    device = device if device is not None else tensors_across_devices[0].device
    out = allreduce._sum_on(tensors_across_devices, device)
    if use_mean:
        out.mul_(1.0 / len(tensors_across_devices))
    return out


class _TensorPacker:
    def __init__(self, num_splits, compact):
        self._num_splits = num_splits
        self._compact = compact
        self._before_compact_dtypes: List[torch.dtype] = []

    def maybe_concat_tensors(self, device_tensors):
        if not self._num_splits:
            return device_tensors
        self._orig_shapes = [tuple(t.shape) for t in device_tensors]
        self._orig_sizes = [t.numel() for t in device_tensors]
        return [torch.cat([t.reshape(-1) for t in device_tensors])]

    def maybe_split_tensors(self, concatenated):
        if not self._num_splits:
            return concatenated
        if len(concatenated) != 1:
            raise RuntimeError("tensors must be concatenated via maybe_concat_tensors() "
                               "before splitting")
        t = concatenated[0]
        total = t.numel()
        size = total // self._num_splits
        sizes = [size] * (self._num_splits - 1) + [total - size * (self._num_splits - 1)]
        return list(torch.split(t, sizes))

    def undo_maybe_split_tensors(self, packs):
        if not self._num_splits:
            return packs
        return [torch.cat(list(packs))]

    def undo_maybe_concat_tensors(self, concatenated):
        if not self._num_splits:
            return concatenated
        if len(concatenated) != 1:
            raise RuntimeError("undo_maybe_split_tensors() must be called before "
                               "undo_maybe_concat_tensors when num_splits is greater than 1")
        parts = torch.split(concatenated[0], self._orig_sizes)
        return [p.reshape(s) for p, s in zip(parts, self._orig_shapes)]

    def maybe_compact_tensors(self, device_tensors):
        if not self._compact:
            return device_tensors
        if self._before_compact_dtypes:
            raise RuntimeError("maybe_compact_tensors can only be called once.")
        self._before_compact_dtypes = [t.dtype for t in device_tensors]
        return [t.to(torch.float16) for t in device_tensors]

    def undo_maybe_compact_tensors(self, compact):
        if not self._compact:
            return compact
        if not self._before_compact_dtypes:
            raise RuntimeError("maybe_compact_tensors() must be called before "
                               "undo_maybe_compact_tensors()")
        return [t.to(d) for t, d in zip(compact, self._before_compact_dtypes)]


class BatchAllReduceAlgorithm(abc.ABC):
    def __init__(self):
        self._deferred = None

    def batch_all_reduce(self, all_device_tensors, num_splits=0, compact_tensors=False,
                         defer_tensors=False):
        """Returns (reduced_all_device_tensors, warmup_ops).  ``warmup_ops`` is
        kept for API parity; deferral needs no warm-up op here."""
        packers = [_TensorPacker(num_splits, compact_tensors) for _ in all_device_tensors]
        packed = []
        for packer, dt in zip(packers, all_device_tensors):
            t = packer.maybe_concat_tensors(list(dt))
            t = packer.maybe_compact_tensors(t)
            packed.append(packer.maybe_split_tensors(t))
        reduced = self._do_batch_all_reduce(packed)
        out = []
        for packer, dt in zip(packers, reduced):
            t = packer.undo_maybe_split_tensors(list(dt))
            t = packer.undo_maybe_compact_tensors(t)
            out.append(packer.undo_maybe_concat_tensors(t))
        if defer_tensors:
            prev = self._deferred
            self._deferred = out
            if prev is None:
                prev = [[torch.zeros_like(t) for t in dt] for dt in out]
            out = prev
        return out, []

    @abc.abstractmethod
    def _do_batch_all_reduce(self, all_device_tensors):
        ...


class CopyToDeviceAlgorithm(BatchAllReduceAlgorithm):
    """Tensor j is summed on devices_to_reduce_on[j % n] and every tower
    reads that result."""

    def __init__(self, devices_to_reduce_on, use_mean=False):
        super().__init__()
        self._devices = list(devices_to_reduce_on)
        self._use_mean = use_mean

    def _do_batch_all_reduce(self, all_device_tensors):
        reduced = []
        for i, across in enumerate(zip(*all_device_tensors)):
            dev = allreduce._torch_device(self._devices[i % len(self._devices)],
                                          across[0].device)
            reduced.append(_all_reduce_using_copy(across, self._use_mean, dev))
        return [[r.to(dt[0].device) for r in reduced] for dt in all_device_tensors]


class HierarchicalCopyAlgorithm(BatchAllReduceAlgorithm):
    """Reduce each half of the towers on its main device, add the two
    partial sums on the first main device, broadcast back to both group
    roots and fan out inside each group."""

    def __init__(self, network_topology):
        super().__init__()
        self._network_topology = network_topology

    def _main_devices(self, tensor_index, num_devices):
        topo = self._network_topology
        if topo in (constants.NetworkTopology.DGX1, constants.NetworkTopology.XGMI_MESH):
            return tensor_index % num_devices, (tensor_index + num_devices // 2) % num_devices
        if topo == constants.NetworkTopology.GCP_V100:
            if num_devices != 8:
                raise ValueError("HierarchicalCopy only supports eight devices in %s." % topo)
            pairs = [(0, 5), (2, 7), (5, 0), (7, 2)]
            return pairs[tensor_index % len(pairs)]
        raise ValueError("HierarchicalCopy is not supported for %s network topology." % topo)

    def _do_batch_all_reduce(self, all_device_tensors):
        devices = [dt[0].device for dt in all_device_tensors]
        n = len(devices)
        half = n // 2
        per_tensor = []
        for i, across in enumerate(zip(*all_device_tensors)):
            m0, m1 = self._main_devices(i, n)
            g0, g1 = (0, half) if m0 < half else (half, 0)
            r0 = _all_reduce_using_copy(across[g0:g0 + half], False, devices[m0])
            r1 = _all_reduce_using_copy(across[g1:g1 + half], False, devices[m1])
            total = _all_reduce_using_copy([r0, r1], False, devices[m0])
            b0 = total
            b1 = total.to(devices[m1], copy=True)
            outs = []
            for j in range(len(across)):
                src = b0 if (m0 < half) == (j < half) else b1
                outs.append(src.to(devices[j], copy=True))
            per_tensor.append(outs)
        return [list(x) for x in zip(*per_tensor)]


class AllReduceSpecAlgorithm(BatchAllReduceAlgorithm):
    def __init__(self, all_reduce_spec, gpu_indices, agg_small_grads_max_bytes,
                 agg_small_grads_max_group):
        super().__init__()
        spec = allreduce.parse_all_reduce_spec(all_reduce_spec)
        if len(spec) != 1:
            raise ValueError("Replicated mode does not support hybrid all-reduce strategies")
        self._spec = spec[0]
        self._gpu_indices = gpu_indices
        self._max_bytes = agg_small_grads_max_bytes
        self._max_group = agg_small_grads_max_group

    def _do_batch_all_reduce(self, all_device_tensors):
        tower_grads = [[(t, None) for t in dt] for dt in all_device_tensors]
        out = allreduce.sum_gradients_all_reduce(
            ["/job:localhost"], tower_grads, 1, self._spec.alg, self._spec.shards,
            self._gpu_indices, agg_small_grads_max_bytes=self._max_bytes,
            agg_small_grads_max_group=self._max_group)
        return [[t for t, _ in gv] for gv in out]


def algorithm_from_params(params) -> BatchAllReduceAlgorithm:
    if params.all_reduce_spec:
        if params.gpu_indices:
            gpu_indices = [int(x) for x in params.gpu_indices.split(",")]
        else:
            gpu_indices = list(range(params.num_gpus))
        return AllReduceSpecAlgorithm(params.all_reduce_spec, gpu_indices,
                                      params.agg_small_grads_max_bytes,
                                      params.agg_small_grads_max_group)
    if params.hierarchical_copy:
        return HierarchicalCopyAlgorithm(constants.NetworkTopology(params.network_topology))
    if params.local_parameter_device == "gpu":
        devices = ["/gpu:%d" % i for i in range(params.num_gpus)]
    else:
        devices = ["/cpu:0"]
    return CopyToDeviceAlgorithm(devices)
