"""Gradient-aggregation strategies (--variable_update / --kungfu_option).

The reference implements each mode as a TF VariableMgr (tcb/variable_mgr.py)
that places variables and rewires the gradient graph.  On MI355X every mode
runs as one process per GPU over RCCL, and what distinguishes the modes is
only *what is reduced, how it is scaled, and when*:

=========================  =============================================  ====================
mode                       reference semantics                            here
=========================  =============================================  ====================
parameter_server           grads averaged over towers, applied on PS      all-reduce SUM of per
                           vars by each worker (W updates / step)         worker mean grads
distributed_replicated     same aggregation via PS shadow vars            as parameter_server
replicated                 towers' grads SUMMED (LR /num_gpus in model)   all-reduce SUM
collective_all_reduce      CollectiveReduce SUM over all devices          all-reduce SUM
distributed_all_reduce     all-reduce SUM over workers x towers           all-reduce SUM
horovod                    hvd.allreduce(average=False)                   all-reduce SUM
independent                no communication                               none
kungfu sync_sgd            SynchronousSGDOptimizer: sum / cluster size    all-reduce, x 1/W
kungfu async_sgd           PairAveragingOptimizer                         P2P model store
kungfu sma                 SynchronousAveragingOptimizer                  all-reduce of weights
kungfu ada_sgd             (not wired in the reference)                   SMA -> S-SGD switch
=========================  =============================================  ====================

The 1/W of S-SGD, the loss-scale unscale and the weight decay are folded
into the fused optimizer launch (grad_scale), so the all-reduce itself is a
plain SUM on contiguous gradient buckets overlapped with backward.
"""

from __future__ import annotations

from typing import Optional

import torch

from . import comm
from .bucket import BucketReducer


class Strategy:
    name = "none"
    reduces_gradients = False
    each_tower_has_variables = True

    def __init__(self, params, world: comm.World, flat, bucket_mb=64.0, wire_dtype=None,
                 overlap=True, tower_scale=1.0, num_buckets=0, relaxed=False, shards=1,
                 spec=None, hierarchical=False):
        self.params = params
        self.world = world
        self.flat = flat
        self.tower_scale = float(tower_scale)
        self.reducer: Optional[BucketReducer] = None
        if self.reduces_gradients and world.communicates:
            hier = None
            # (a forced 1-rank group builds it too: the GPU tests' real
            # communicator path, tests/test_dist_gpu.py)
            if hierarchical and (world.size > 1 or comm.force_pg()):
                from .allreduce import Hierarchical
                hier = Hierarchical(world.size, world.rank,
                                    str(getattr(params, "network_topology", "dgx1")))
            self.reducer = BucketReducer(flat, bucket_mb, wire_dtype, overlap=overlap,
                                         num_buckets=num_buckets, relaxed=relaxed,
                                         shards=shards, spec=spec, hierarchical=hier)

    @property
    def grad_scale(self) -> float:
        return self.tower_scale

    @property
    def aggregates_gradients(self) -> bool:
        """Whether this step's applied gradient is a sum over workers (then
        it carries every worker's L2 term; see BenchmarkCNN._l2_multiplier)."""
        return self.reduces_gradients

    def broadcast_initial_model(self, slots=()):
        """Rank-0 broadcast of every variable (+ optimizer slots, BN stats):
        what horovod.broadcast_global_variables(0) / kungfu broadcast do at
        init (tcb/benchmark_cnn.py:2094-2100)."""
        if not self.world.communicates:
            return
        comm.broadcast(self.flat.flat, 0)
        for t in slots:
            comm.broadcast(t, 0)
        for layer in self.flat.net.ordered_layers():
            for b in layer.buffers(recurse=False):
                comm.broadcast(b, 0)
        self.flat.refresh_lp()

    def before_backward(self, step: int):
        if self.reducer is not None:
            self.reducer.begin()

    def after_backward(self, step: int):
        if self.reducer is not None:
            self.reducer.finish()

    def before_update(self, step: int):
        pass

    def after_update(self, step: int):
        pass

    def abort_update(self, step: int):
        """Called instead of after_update when the update raised."""

    def fused_update(self):
        """(mix, wout) for the optimizer's single pass (FusedOptimizer.step):
        model averaging folded into the update, and where to copy the
        updated weights.  Called between before_update and the step."""
        return None, None

    @property
    def update_is_empty(self) -> bool:
        """True when the gradient to apply is the all-zero first step of
        --variable_consistency=relaxed (no weight decay either)."""
        return self.reducer is not None and self.reducer.deferred_empty

    # ---------------------------------------------------- launch tape hooks
    def tape_blocker(self) -> Optional[str]:
        """Why a step of this strategy cannot be replayed from a launch tape
        (None: it can).  A taped step replays the recorded native calls; the
        strategy's per-step host logic runs in tape_pre / tape_post around
        the replay and feeds it per-step values."""
        if not self.world.communicates:
            return None
        r = self.reducer
        if not self.reduces_gradients or r is None:
            return "%s runs host-side logic every step" % self.name
        if r.relaxed or r.hierarchical is not None:
            return "relaxed / hierarchical reductions keep host-side state"
        return None

    def steps_use_collectives(self) -> bool:
        """Whether every step issues device collectives (then a launch tape
        needs them as native calls: the native communicator)."""
        return self.reducer is not None

    def tape_phase(self, step: int):
        """Steps in different phases record different launch sequences (a
        recorded tape is re-recorded when the phase changes)."""
        return 0

    def tape_pre(self, step: int) -> dict:
        """Host half of the strategy's step before a replay; returns the
        per-step values (native.dyn keys) of the replay."""
        return {}

    def tape_post(self, step: int):
        """Host half of the strategy's step after a replay was enqueued."""

    def describe(self) -> str:
        return self.name

    def close(self):
        if self.reducer is not None:
            self.reducer.close()


class IndependentStrategy(Strategy):
    name = "independent"

    def tape_blocker(self):
        return None  # no per-step communication at all


class SumAllReduceStrategy(Strategy):
    """parameter_server / replicated / distributed_* / collective / horovod."""
    reduces_gradients = True

    def __init__(self, name, *a, **kw):
        self.name = name
        super().__init__(*a, **kw)


class KungFuSyncSGD(Strategy):
    """SynchronousSGDOptimizer: all-reduce(sum) every gradient, divide by the
    cluster size, then apply the wrapped optimizer."""
    name = "kungfu/sync_sgd"
    reduces_gradients = True

    @property
    def grad_scale(self):
        return self.tower_scale / self.world.size


class KungFuSMA(Strategy):
    """SynchronousAveragingOptimizer: every step all-reduce-average the model,
    move the local model toward it (w <- w - alpha (w - avg)), then apply the
    local gradient.

    The average is of the weights the step's forward used (w_t), so its
    all-reduce is launched as soon as w_t exists - right after the previous
    update, whose fused kernel also writes the copy of w_t that is reduced
    (``wout``) - and runs beside the next forward/backward.  The update waits
    for it (a stream wait on RCCL) and folds the averaging into its single
    pass (``mix``): no separate copy or elementwise passes over the model."""
    name = "kungfu/sma"

    def __init__(self, *a, alpha=0.1, **kw):
        super().__init__(*a, **kw)
        self.alpha = float(alpha)
        self._avg = None
        self._work = None

    def _launch(self):
        self._work = comm.all_reduce(self._avg, async_op=True)

    def broadcast_initial_model(self, slots=()):
        super().broadcast_initial_model(slots)
        if self.world.communicates:
            self._avg = self.flat.flat.clone()
            self._launch()

    def before_update(self, step):
        if not self.world.communicates:
            return
        if self._avg is None:  # no initial broadcast: start from the local model
            self._avg = self.flat.update_target.clone()
            self._launch()
        if self._work is not None:
            self._work.wait()
            self._work = None

    def fused_update(self):
        if not self.world.communicates or self._avg is None:
            return None, None
        # w <- (1 - alpha) w + alpha * sum / size; then the updated w goes to
        # the buffer the next all-reduce sums
        return (self._avg, 1.0 - self.alpha, self.alpha / self.world.size, None), self._avg

    def after_update(self, step):
        if self.world.communicates and self._avg is not None:
            self._launch()

    def steps_use_collectives(self):
        return True

    def tape_blocker(self):
        # the model all-reduce and its stream waits are native calls on
        # fixed buffers: a recorded step replays them (the all-reduce a
        # replay enqueues at its end is the one the next replay waits for)
        return None

    def tape_pre(self, step):
        return {"wout": self._avg.data_ptr()} if self._avg is not None else {}

    def abort_update(self, step):
        self._work = None

    def close(self):
        if self._work is not None:
            self._work.wait()
            self._work = None
        super().close()


class KungFuAdaSGD(Strategy):
    """Adaptive variant (not wired in the reference, tcb/benchmark_cnn.py:1202-1204):
    SMA for the first ``switch_step`` steps, synchronous SGD afterwards."""
    name = "kungfu/ada_sgd"
    reduces_gradients = True

    def __init__(self, *a, alpha=0.1, switch_step=100, **kw):
        super().__init__(*a, **kw)
        self.sma = KungFuSMA(*a, alpha=alpha, **{k: v for k, v in kw.items()})
        self.switch_step = int(switch_step)
        self._step = 0

    @property
    def grad_scale(self):
        return 1.0 / self.world.size if self._step >= self.switch_step else 1.0

    @property
    def aggregates_gradients(self):
        # the averaging phase applies each worker's own gradient
        return self._step >= self.switch_step

    def before_backward(self, step):
        self._step = step
        if step >= self.switch_step:
            super().before_backward(step)

    def after_backward(self, step):
        if step >= self.switch_step:
            super().after_backward(step)

    def broadcast_initial_model(self, slots=()):
        super().broadcast_initial_model(slots)
        if self.switch_step > 0:
            self.sma._avg = None  # started lazily by the first SMA update

    def before_update(self, step):
        if step < self.switch_step:
            self.sma.before_update(step)

    def fused_update(self):
        if self._step < self.switch_step:
            return self.sma.fused_update()
        return None, None

    def after_update(self, step):
        # launch the next average only if the next step still averages
        if step + 1 < self.switch_step:
            self.sma.after_update(step)

    def tape_blocker(self):
        r = self.reducer
        if self.world.communicates and r is not None and (r.relaxed or
                                                          r.hierarchical is not None):
            return "relaxed / hierarchical reductions keep host-side state"
        return None

    def steps_use_collectives(self):
        return True

    def tape_phase(self, step):
        # averaging steps, the last averaging step (launches no next
        # average), synchronous-SGD steps: three launch sequences
        return (step < self.switch_step, step + 1 < self.switch_step)

    def tape_pre(self, step):
        return self.sma.tape_pre(step) if step < self.switch_step else {}

    def close(self):
        self.sma.close()
        super().close()


MEAN_OVER_TOWERS = ("parameter_server", "distributed_replicated")


def make_strategy(params, world, flat, tower_mode=False, num_gpus=1):
    """``tower_mode``: the ranks are the towers of ONE worker (--num_gpus=N
    relaunched as N processes).  The reference averages tower gradients in
    parameter_server mode and sums them in the replicated/all-reduce modes;
    with a SUM all-reduce that is a 1/N scale for the former.  Without a
    launcher the N towers run as one big batch (already a tower mean), so
    the sum modes scale by N instead."""
    vu = params.variable_update
    wire = {"auto": None, "fp32": None, "bf16": torch.bfloat16,
            "fp16": torch.float16}[params.gradient_wire_dtype]
    if params.gradient_wire_dtype == "auto" and params.compact_gradient_transfer \
            and params.gradient_repacking:
        wire = torch.float16
    if tower_mode:
        tower_scale = 1.0 / num_gpus if vu in MEAN_OVER_TOWERS else 1.0
    elif num_gpus > 1:
        tower_scale = 1.0 if vu in MEAN_OVER_TOWERS else float(num_gpus)
    else:
        tower_scale = 1.0
    spec = None
    if params.all_reduce_spec:
        from .allreduce import parse_all_reduce_spec
        spec = parse_all_reduce_spec(params.all_reduce_spec)
    kw = dict(bucket_mb=params.bucket_size_mb, wire_dtype=wire,
              overlap=params.overlap_gradient_allreduce, tower_scale=tower_scale,
              num_buckets=params.gradient_repacking,
              relaxed=params.variable_consistency == "relaxed", spec=spec,
              hierarchical=bool(params.hierarchical_copy))
    if vu == "independent":
        return IndependentStrategy(params, world, flat, **kw)
    if vu == "kungfu":
        opt = params.kungfu_option
        if opt == "sync_sgd":
            return KungFuSyncSGD(params, world, flat, **kw)
        if opt == "sma":
            return KungFuSMA(params, world, flat, alpha=params.kungfu_sma_alpha, **kw)
        if opt == "ada_sgd":
            return KungFuAdaSGD(params, world, flat, alpha=params.kungfu_sma_alpha,
                                switch_step=params.kungfu_ada_switch_step, **kw)
        if opt == "async_sgd":
            from .kungfu import PairAveraging
            return PairAveraging(params, world, flat, **kw)
        raise ValueError('KungFu distributed option "%s" was not recognized' % opt)
    if vu == "parameter_server" and not params.cross_replica_sync and world.size > 1 \
            and not tower_mode:
        from .async_ps import AsyncParameterServer
        return AsyncParameterServer(params, world, flat, **kw)
    if vu in ("parameter_server", "replicated", "distributed_replicated", "collective_all_reduce",
              "distributed_all_reduce", "horovod"):
        return SumAllReduceStrategy(vu, params, world, flat, **kw)
    raise ValueError("Invalid variable_update in local mode: %s" % vu)
