"""All-reduce specs and the collective algorithms they select
(role of tcb/allreduce.py, tcb/batch_allreduce.py).

The reference builds its all-reduce *inside one TF graph* over the tower
devices of a process: ``--all_reduce_spec`` picks per tensor-size range an
algorithm (``nccl`` / ``xring`` / ``nccl/rechd`` / ``pscpu`` / ``psgpu`` /
hierarchical forms / ``collective``) and a shard count, and small tensors
are concatenated into packs first (tcb/allreduce.py:58-104, 344-417,
514-588; tcb/batch_allreduce.py:173-317, 391-481).

On MI355X every GPU is its own process and gradients already live in one
contiguous flat buffer reduced in contiguous buckets
(:mod:`kf_benchmarks_amd.parallel.bucket`), so packing is structural and the
algorithm choice becomes a choice of *process-level collective* per bucket,
made here from the same spec grammar:

=====================================  =========================================
spec algorithm                         collective issued for a bucket
=====================================  =========================================
``nccl``, ``collective``               RCCL all-reduce (RCCL picks ring / tree)
``xring``, ``nccl/xring``              RCCL all-reduce, ring algorithm pinned
``nccl/rechd``                         RCCL all-reduce, tree algorithm pinned
``psgpu``, ``pscpu``, ``nccl/pscpu``,  parameter-server style: RCCL reduce to a
``pscpu/pscpu``                        root rank, then broadcast from it; the root
                                       rotates over buckets (the reference spreads
                                       PS shards over devices greedily); the sum
                                       stays on the root GPU - a host round trip
                                       would only slow the xGMI path down
=====================================  =========================================

``--hierarchical_copy`` (tcb/batch_allreduce.py:173-267, the DGX-1 two-level
copy) becomes a two-level collective over process subgroups
(:class:`Hierarchical`): reduce to each group's leader, all-reduce among the
leaders, broadcast back inside each group.  Groups follow
``--network_topology``: the NVLink halves {0-3}, {4-7} for ``dgx1`` /
``gcp_v100``; one group per 8 ranks for ``xgmi_mesh`` (every MI355X of a node
is one xGMI hop from every other, so the node is the natural group and the
leader level only matters across nodes).

``alg#k`` issues each bucket as k concurrent collectives (channels), and the
``:limit:`` ranges choose the algorithm by bucket size.  RCCL's ring / tree
choice is communicator-wide, so a spec naming ``xring`` anywhere pins ring,
else one naming ``rechd`` pins tree (:func:`rccl_env_for_spec`).

Spec grammar (tcb/allreduce.py:58-104): ``alg[#shards][:limit:alg[#shards]]*``
where ``limit`` is an element count with optional k/M/G/T suffix; tensors of
at most ``limit`` elements use the algorithm before it.
"""

from __future__ import annotations

import collections
import re
from typing import Dict, List, Optional

AllReduceSpecTuple = collections.namedtuple("AllReduceSpecTuple", "alg shards limit")

VALID_ALGS = ("nccl", "nccl/xring", "nccl/rechd", "nccl/pscpu", "xring", "pscpu", "psgpu",
              "pscpu/pscpu", "collective")
PS_ALGS = ("psgpu", "pscpu", "nccl/pscpu", "pscpu/pscpu")


def parse_general_int(s: str) -> int:
    """'32k' -> 32768 (power-of-2 suffixes K/k, M, G, T)."""
    mo = re.match(r"(\d+)([KkMGT]?)$", s)
    if not mo:
        return int(s)
    v = int(mo.group(1))
    return v * {"": 1, "K": 1 << 10, "k": 1 << 10, "M": 1 << 20, "G": 1 << 30,
                "T": 1 << 40}[mo.group(2)]


def parse_all_reduce_spec(all_reduce_spec: str) -> List[AllReduceSpecTuple]:
    parts = all_reduce_spec.split(":") + ["-1"]
    if len(parts) % 2:
        raise ValueError("all_reduce_spec not well formed: %s" % all_reduce_spec)
    spec = []
    alg, shards = None, 1
    for i, part in enumerate(parts):
        if i % 2:
            try:
                limit = parse_general_int(part)
            except ValueError:
                raise ValueError("all_reduce_spec (%s) contains non-integer range %s"
                                 % (all_reduce_spec, part))
            spec.append(AllReduceSpecTuple(alg=alg, shards=shards, limit=limit))
        else:
            pieces = part.split("#")
            alg = pieces[0]
            shards = 1
            if len(pieces) > 1:
                try:
                    shards = int(pieces[1])
                except ValueError:
                    raise ValueError("all_reduce_spec (%s) contains non-integer shards %s"
                                     % (all_reduce_spec, pieces[1]))
            if alg not in VALID_ALGS:
                raise ValueError("all_reduce_spec (%s) contains invalid alg %s"
                                 % (all_reduce_spec, alg))
    return spec




def algorithm_for(spec: Optional[List[AllReduceSpecTuple]], numel: int) -> AllReduceSpecTuple:
    """The spec entry whose range holds a bucket of ``numel`` elements
    (default: plain RCCL all-reduce, one shard)."""
    if not spec:
        return AllReduceSpecTuple("nccl", 1, -1)
    for t in spec:
        if t.limit < 0 or numel <= t.limit:
            return t
    return spec[-1]


def is_parameter_server(alg: str) -> bool:
    return alg in PS_ALGS


def _side_stream(buf):
    """Context of a chained collective's stages.  Device buffers: the
    caller's stream itself - the bucket reducer issues from the weight-
    gradient side stream, which already follows the producers, and one
    stream orders the stages (a further stream waiting on it cost 7-11
    ms/step, profiles/r13_comm_stream_ab.txt).  Host (gloo) buffers: no
    stream; the stages are ordered by host waits."""
    return _null()


def launch_collective(comm, buf, alg: str, bucket_index: int, world_size: int, op: str = "sum",
                      hierarchical: Optional["Hierarchical"] = None):
    """Issue one bucket piece's collective(s) asynchronously; returns the
    list of work handles (the last one completes the piece).

    Multi-stage chains (parameter-server reduce -> broadcast, and the
    hierarchical reduce -> leader all-reduce -> broadcast) order their stages
    with ``Work.wait()``: on the native communicator the stages share the
    issuing stream (the wait is a no-op), on gloo - the CPU test
    backend, whose async ops are not ordered - it is a host wait inside the
    backward hook.  The chains are verified over gloo at 2-8 ranks
    (tests/test_variable_update.py, tests/test_scale_rehearsal.py) and over
    a 1-rank RCCL group; their RCCL form at more than one GPU runs for the
    first time on the round-end multi-GPU node."""
    if hierarchical is not None and world_size > 1:
        return hierarchical.launch(buf, op)
    if is_parameter_server(alg) and world_size > 1:
        root = bucket_index % world_size
        with _side_stream(buf):
            w1 = comm.reduce(buf, dst=root, op=op, async_op=True)
            if w1 is not None:
                w1.wait()  # the broadcast must see the finished sum
            w2 = comm.broadcast(buf, src=root, async_op=True)
        return [w2] if w2 is not None else []
    w = comm.all_reduce(buf, op=op, async_op=True)
    return [w] if w is not None else []


class Hierarchical:
    """Two-level all-reduce over torch.distributed subgroups.  Built
    collectively (every rank constructs it, same order).  The three stages
    run in order on the issuing stream (the bucket reducer's weight-gradient
    side stream, :func:`_side_stream`), so the compute stream is only
    blocked by the final wait."""

    def __init__(self, world_size: int, rank: int, topology: str = "dgx1"):
        import torch.distributed as dist
        gsize = 4 if topology in ("dgx1", "gcp_v100") else 8
        if topology == "gcp_v100" and world_size != 8:
            raise ValueError("HierarchicalCopy on gcp_v100 only supports 8 GPUs per worker")
        gsize = max(1, min(gsize, world_size))
        self.rank, self.size, self.gsize = rank, world_size, gsize
        groups = [list(range(i, min(i + gsize, world_size))) for i in range(0, world_size, gsize)]
        self.my = rank // gsize
        self.members = groups[self.my]
        self.leader = self.members[0]
        leaders = [g[0] for g in groups]
        self.is_leader = rank == self.leader
        self.closed = False
        from . import comm as _comm
        world = _comm.get_world()
        self.native = None
        if world.native is not None:
            # one RCCL communicator family: the subgroups are native
            # communicators like the world one (no ProcessGroupNCCL beside it)
            from . import rccl as _rccl
            store = dist.distributed_c10d._get_default_store()
            self.native = (_rccl.subgroup(world.native, self.members, store, "hier%d" % self.my),
                           _rccl.subgroup(world.native, leaders, store, "hier_leaders")
                           if len(groups) > 1 else None)
            return
        # device tensors need RCCL subgroups when the world's device backend
        # is RCCL; gloo (CPU rehearsals) otherwise
        be = "nccl" if world.device_backend in ("rccl", "nccl") else None
        self.groups = [dist.new_group(g, backend=be) for g in groups]  # collective: all ranks
        self.leaders = dist.new_group(leaders, backend=be)

    def _launch_native(self, buf, op):
        g, lead = self.native
        with _side_stream(buf):
            g.reduce(buf, dst=0, op=op).wait()  # the leader is member 0
            if self.is_leader and lead is not None:
                lead.all_reduce(buf, op=op).wait()
            return [g.broadcast(buf, src=0)]

    def close(self):
        """Destroys the native subgroup communicators (the world's own is
        destroyed by comm.World.shutdown).  Idempotent."""
        if self.native and not self.closed:
            for c in self.native:
                if c is not None:
                    c.close()
        self.closed = True

    def launch(self, buf, op: str = "sum"):
        if self.closed:
            raise RuntimeError("Hierarchical all-reduce used after close()")
        if self.native is not None:
            return self._launch_native(buf, op)
        import torch.distributed as dist
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op]
        g = self.groups[self.my]
        works = []
        with _side_stream(buf):
            w = dist.reduce(buf, dst=self.leader, op=rop, group=g, async_op=True)
            w.wait()  # orders the next stage after this one (on the side stream)
            if self.is_leader and len(self.groups) > 1:
                w = dist.all_reduce(buf, op=rop, group=self.leaders, async_op=True)
                w.wait()
            works.append(dist.broadcast(buf, src=self.leader, group=g, async_op=True))
        return works


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


# ------------------------------------------------------- process level
def rccl_env_for_spec(all_reduce_spec: Optional[str]) -> Dict[str, str]:
    """RCCL environment implied by a spec for the one-process-per-GPU mode
    (set before the communicator is created): ``xring`` -> ring algorithm,
    ``rechd`` -> tree; ``#shards`` -> at least that many channels."""
    if not all_reduce_spec:
        return {}
    env = {}
    spec = parse_all_reduce_spec(all_reduce_spec)
    algs = {s.alg for s in spec}
    if any("xring" in a for a in algs):
        env["NCCL_ALGO"] = "Ring"
    elif any("rechd" in a for a in algs):
        env["NCCL_ALGO"] = "Tree"
    shards = max(s.shards for s in spec)
    if shards > 1:
        env["NCCL_MIN_NCHANNELS"] = str(shards)
    return env
