"""All-reduce specs, tensor packing and in-process reduction algorithms
(role of tcb/allreduce.py).

Two levels exist on MI355X:

* **across processes** (one per GPU, the normal mode): RCCL collectives over
  xGMI via ``torch.distributed``; an ``--all_reduce_spec`` selects the RCCL
  algorithm (``xring`` -> ring, ``nccl/rechd`` -> tree) and the number of
  concurrent shards per bucket (``alg#shards``); see :func:`rccl_env_for_spec`
  and :class:`kf_benchmarks_amd.parallel.bucket.BucketReducer`.
* **inside one process** over a list of device tensors (CPU tensors in the
  tests, or several GPUs driven from one process): the algorithms below
  implement the reference's menu directly - ``nccl`` (RCCL multi-device
  all-reduce when the tensors sit on distinct GPUs), ``xring`` (explicit ring
  reduce-scatter + all-gather), ``nccl/rechd`` (recursive halving-doubling),
  ``pscpu``/``psgpu`` (shuffle: shards reduced on auxiliary devices), the
  hierarchical ``a/b`` forms, and ``collective`` (local sum + cross-process
  all-reduce).  The reference left everything except ``nccl``/``collective``
  as NotImplementedError (tcb/allreduce.py:300-317).

Spec grammar (tcb/allreduce.py:58-104): ``alg[#shards][:limit:alg[#shards]]*``
where ``limit`` is an element count with optional k/M/G/T suffix; tensors of
at most ``limit`` elements use the algorithm before it.
"""

from __future__ import annotations

import collections
import re
from typing import Dict, List, Optional, Sequence, Tuple

import torch

AllReduceSpecTuple = collections.namedtuple("AllReduceSpecTuple", "alg shards limit")
GradPackTuple = collections.namedtuple("GradPackTuple", "indices vars shapes")

VALID_ALGS = ("nccl", "nccl/xring", "nccl/rechd", "nccl/pscpu", "xring", "pscpu", "psgpu",
              "pscpu/pscpu", "collective")


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


def build_all_reduce_device_prefixes(job_name: str, num_tasks: int) -> List[str]:
    if job_name != "localhost":
        return ["/job:%s/task:%d" % (job_name, d) for d in range(num_tasks)]
    assert num_tasks == 1
    return ["/job:%s" % job_name]


def group_device_names(devices: Sequence[str], group_size: int) -> List[List[str]]:
    """Round-robin ``devices`` into ceil(n / group_size) groups of exactly
    ``group_size`` (devices repeat when n is not a multiple)."""
    n = len(devices)
    if group_size > n:
        raise ValueError("only %d devices, but group_size=%d" % (n, group_size))
    num_groups = n // group_size + (1 if n % group_size else 0)
    groups: List[List[str]] = [[] for _ in range(num_groups)]
    for i in range(num_groups * group_size):
        groups[i % num_groups].append(devices[i % n])
    return groups


def split_grads_by_size(threshold_size: int, device_grads):
    """(small, large) lists of per-device [(g, v)] by element count."""
    small, large = [], []
    for dl in device_grads:
        s = [[g, v] for g, v in dl if g.numel() <= threshold_size]
        lg = [[g, v] for g, v in dl if g.numel() > threshold_size]
        if s:
            small.append(s)
        if lg:
            large.append(lg)
    return small, large


_instance_key = 1
_group_key = 1
_group_key_table: Dict[str, int] = {}


def new_collective_instance_key() -> int:
    global _instance_key
    v = _instance_key
    _instance_key += 1
    return v


def _device_type_index(d: str) -> str:
    m = re.search(r"(?:device:)?([A-Za-z]+):(\d+)\s*$", d)
    if not m:
        raise ValueError("cannot parse device %s" % d)
    return "%s:%d" % (m.group(1).upper(), int(m.group(2)))


def collective_group_key(devices: Sequence[str]) -> int:
    """Stable key per *set* of (type, index) devices, independent of order and
    of job/task prefixes."""
    global _group_key
    concat = ",".join(sorted(_device_type_index(d) for d in devices))
    if concat not in _group_key_table:
        _group_key_table[concat] = _group_key
        _group_key += 1
    return _group_key_table[concat]


def contains_any(haystack: str, needles: Sequence[str]) -> bool:
    return any(n in haystack for n in needles)


# ------------------------------------------------------------------ packing
def extract_ranges(index_list: Sequence[int], range_size_limit: int = 32):
    """Consecutive runs (as [first, last], each at most range_size_limit+1
    long) and the remaining singles of a monotone index list."""
    if not index_list:
        return [], []
    first = last = index_list[0]
    ranges, singles = [], []
    for i in index_list[1:]:
        if i == last + 1 and (last - first) <= range_size_limit:
            last = i
        else:
            (ranges.append([first, last]) if last > first else singles.append(first))
            first = last = i
    (ranges.append([first, last]) if last > first else singles.append(first))
    return ranges, singles


def pack_range(key, packing: dict, grad_vars, rng) -> torch.Tensor:
    """Concatenates grad_vars[rng[0]..rng[1]] (flattened) and records how to
    undo it under ``packing[key]``."""
    to_pack = grad_vars[rng[0]:rng[1] + 1]
    packing[key] = GradPackTuple(indices=range(rng[0], rng[1] + 1),
                                 vars=[v for _, v in to_pack],
                                 shapes=[tuple(g.shape) for g, _ in to_pack])
    return torch.cat([g.reshape(-1) for g, _ in to_pack])


def unpack_grad_tuple(gv, gpt: GradPackTuple):
    widths = [int(torch.Size(s).numel()) for s in gpt.shapes]
    parts = torch.split(gv[0], widths)
    return [(p.reshape(gpt.shapes[i]), gpt.vars[i]) for i, p in enumerate(parts)]


def pack_small_tensors(tower_grads, max_bytes: int = 0, max_group: int = 0):
    """Concatenate runs of small fp32 gradients; packed tensors come first
    in each tower's list, followed by the untouched ones."""
    small, large = [], []
    for idx, (g, _) in enumerate(tower_grads[0]):
        if g.dtype == torch.float32 and 4 * g.numel() <= max_bytes:
            small.append(idx)
        else:
            large.append(idx)
    ranges, singles = extract_ranges(small, range_size_limit=max_group)
    large = sorted(large + singles)
    if not ranges:
        return tower_grads, None
    packing = {}
    n = len(tower_grads[0])
    out = []
    for dev, gv_list in enumerate(tower_grads):
        assert len(gv_list) == n
        new = []
        for r in ranges:
            key = "%d:%d" % (dev, len(new))
            new.append((pack_range(key, packing, gv_list, r), "packing_var_placeholder"))
        new.extend(gv_list[i] for i in large)
        out.append(new)
    return out, packing


def unpack_small_tensors(tower_grads, packing):
    if not packing:
        return tower_grads
    out = []
    num_packed = len(packing) // len(tower_grads)
    for dev, gv_list in enumerate(tower_grads):
        new = list(gv_list[num_packed:])
        for i in range(num_packed):
            gpt = packing["%d:%d" % (dev, i)]
            for gi, (idx, gv) in enumerate(zip(gpt.indices, unpack_grad_tuple(gv_list[i], gpt))):
                new.insert(idx, gv)
        out.append(new)
    return out


# ------------------------------------------------- in-process reductions
def _sum_on(tensors: Sequence[torch.Tensor], device) -> torch.Tensor:
    acc = tensors[0].to(device, copy=True)
    for t in tensors[1:]:
        acc.add_(t.to(device))
    return acc


def reduce_nccl(tensors: List[torch.Tensor]) -> List[torch.Tensor]:
    """Multi-device all-reduce.  Distinct GPUs -> RCCL (torch.cuda.nccl);
    otherwise sum on the first device and copy back."""
    devs = [t.device for t in tensors]
    if all(d.type == "cuda" for d in devs) and len(set(devs)) == len(devs) and len(devs) > 1:
        from torch.cuda import nccl
        out = [t.clone() for t in tensors]
        nccl.all_reduce(out)
        return out
    total = _sum_on(tensors, devs[0])
    return [total.to(d, copy=True) for d in devs]


def reduce_ring(tensors: List[torch.Tensor]) -> List[torch.Tensor]:
    """Ring all-reduce: n-1 reduce-scatter steps then n-1 all-gather steps,
    each device only talking to its ring successor."""
    n = len(tensors)
    if n == 1:
        return [tensors[0].clone()]
    flat = [t.reshape(-1).clone() for t in tensors]
    chunks = [list(torch.tensor_split(f, n)) for f in flat]
    for step in range(n - 1):  # reduce-scatter
        sends = [(r, (r - step) % n) for r in range(n)]
        payload = [chunks[r][c].clone() for r, c in sends]
        for (r, c), p in zip(sends, payload):
            dst = (r + 1) % n
            chunks[dst][c].add_(p.to(chunks[dst][c].device))
    for step in range(n - 1):  # all-gather
        sends = [(r, (r + 1 - step) % n) for r in range(n)]
        payload = [chunks[r][c].clone() for r, c in sends]
        for (r, c), p in zip(sends, payload):
            dst = (r + 1) % n
            chunks[dst][c].copy_(p.to(chunks[dst][c].device))
    return [f.reshape(t.shape) for f, t in zip(flat, tensors)]


def reduce_halving_doubling(tensors: List[torch.Tensor]) -> List[torch.Tensor]:
    """Recursive halving (reduce-scatter) + doubling (all-gather); device
    counts that are not powers of two fold the extra devices first."""
    n = len(tensors)
    p = 1
    while p * 2 <= n:
        p *= 2
    work = [t.reshape(-1).clone() for t in tensors]
    for extra in range(p, n):  # fold extras into the power-of-two core
        work[extra - p].add_(work[extra].to(work[extra - p].device))
    lo = [0] * p
    hi = [work[0].numel()] * p
    dist_ = p // 2
    while dist_ >= 1:
        for r in range(p):
            partner = r ^ dist_
            if partner < r:
                continue
            mid = (lo[r] + hi[r]) // 2
            # r keeps [lo, mid), partner keeps [mid, hi)
            a, b = work[r], work[partner]
            a[lo[r]:mid].add_(b[lo[r]:mid].to(a.device))
            b[mid:hi[r]].add_(a[mid:hi[r]].to(b.device))
            lo[partner], hi[partner] = mid, hi[r]
            hi[r] = mid
        dist_ //= 2
    dist_ = 1
    while dist_ < p:
        for r in range(p):
            partner = r ^ dist_
            if partner < r:
                continue
            a, b = work[r], work[partner]
            a[lo[partner]:hi[partner]].copy_(b[lo[partner]:hi[partner]].to(a.device))
            b[lo[r]:hi[r]].copy_(a[lo[r]:hi[r]].to(b.device))
            lo[r] = lo[partner] = min(lo[r], lo[partner])
            hi[r] = hi[partner] = max(hi[r], hi[partner])
        dist_ *= 2
    for extra in range(p, n):
        work[extra].copy_(work[extra - p].to(work[extra].device))
    return [w.reshape(t.shape) for w, t in zip(work, tensors)]


def reduce_shuffle(tensors: List[torch.Tensor], aux_devices: Sequence,
                   num_shards: int = 1) -> List[torch.Tensor]:
    """Shuffle all-reduce: each shard of the tensor is summed on one
    auxiliary device, then every device gathers all shards."""
    aux = list(aux_devices) or [tensors[0].device]
    shards = max(num_shards, len(aux))
    flat = [t.reshape(-1) for t in tensors]
    reduced = []
    for s, pieces in enumerate(zip(*[torch.tensor_split(f, shards) for f in flat])):
        reduced.append(_sum_on(pieces, aux[s % len(aux)]))
    return [torch.cat([r.to(t.device) for r in reduced]).reshape(t.shape) for t in tensors]


def _torch_device(name, default):
    if isinstance(name, torch.device):
        return name
    m = re.search(r"(cpu|gpu|cuda):(\d+)", str(name).lower())
    if not m or m.group(1) == "cpu":
        return torch.device("cpu")
    if not torch.cuda.is_available():
        return default
    return torch.device("cuda", int(m.group(2)) % torch.cuda.device_count())


def sum_grad_and_var_all_reduce(grad_and_vars, alg: str, aux_devices=None, num_shards=1,
                                num_workers: int = 1):
    """One variable's per-device gradients -> summed copy on every device."""
    grads = [g for g, _ in grad_and_vars]
    if alg == "collective":
        from . import comm
        total = _sum_on(grads, grads[0].device)
        comm.all_reduce(total)
        summed = [total.to(g.device, copy=True) for g in grads]
    elif alg == "nccl":
        summed = reduce_nccl(grads)
    elif alg == "xring":
        summed = reduce_ring(grads)
    elif alg in ("pscpu", "psgpu"):
        aux = [_torch_device(d, grads[0].device) for d in (aux_devices or [])]
        summed = reduce_shuffle(grads, aux, num_shards)
    elif "/" in alg:
        # hierarchical: first alg inside each worker's devices, second alg
        # across workers (one process = one worker here, so the outer stage
        # is the cross-process all-reduce when the job has several workers)
        inner, outer = alg.split("/")
        summed = sum_grad_and_var_all_reduce(grad_and_vars, inner if inner != "nccl" else "nccl",
                                             aux_devices, num_shards)
        summed = [s for s, _ in summed]
        if num_workers > 1:
            from . import comm
            comm.all_reduce(summed[0])
            summed = [summed[0].to(g.device, copy=True) for g in grads]
        del outer
    elif alg == "rechd":
        summed = reduce_halving_doubling(grads)
    else:
        raise ValueError("unsupported all_reduce alg: %s" % alg)
    return [[g, v] for (_, v), g in zip(grad_and_vars, summed)]


def sum_gradients_all_reduce(dev_prefixes, tower_grads, num_workers, alg, num_shards,
                             gpu_indices, agg_small_grads_max_bytes=0,
                             agg_small_grads_max_group=10, allreduce_merge_scope=1):
    """All-reduce every gradient across the towers of ``tower_grads``
    (list over devices of [(grad, var)]) with one spec algorithm."""
    if "pscpu" in alg:
        aux_devices = [prefix + "/cpu:0" for prefix in dev_prefixes]
    elif "psgpu" in alg:
        aux_devices = [prefix + "/gpu:%d" % i for i in range(len(gpu_indices))
                       for prefix in dev_prefixes]
    else:
        aux_devices = ["/job:localhost/cpu:0"]
    shuffle = contains_any(alg, ["pscpu", "psgpu"])
    groups = group_device_names(aux_devices, num_shards if (alg != "collective" and shuffle)
                                else 1)
    packing = None
    if agg_small_grads_max_bytes > 0 and agg_small_grads_max_group > 0:
        tower_grads, packing = pack_small_tensors(tower_grads, agg_small_grads_max_bytes,
                                                  agg_small_grads_max_group)
    reduced = []
    gi = 0
    for grad_and_vars in zip(*tower_grads):
        aux = aux_devices if "/" in alg else groups[gi]
        reduced.append(sum_grad_and_var_all_reduce(grad_and_vars, alg.replace("nccl/rechd",
                                                                              "rechd"),
                                                   aux, num_shards, num_workers))
        gi = (gi + 1) % len(groups)
    new = [list(x) for x in zip(*reduced)]
    return unpack_small_tensors(new, packing) if packing else new


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
