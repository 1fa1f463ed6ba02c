"""One rank of the 2-rank GPU rehearsal (tests/test_dist_gpu.py): a real
model stepping through the HIP kernels with bucketed all-reduce hooks
overlapped with backward.  Both ranks share the box's one GPU, so the
process group is gloo over CUDA tensors (KFB_DIST_BACKEND=gloo); the
collective call sequence is the one RCCL runs on an 8-GPU node.

usage: dist_gpu_worker.py <out.json> '<json flag kwargs>' <steps>"""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    out, kw, steps = sys.argv[1], json.loads(sys.argv[2]), int(sys.argv[3])
    import torch
    from kf_benchmarks_amd import params as P
    from kf_benchmarks_amd.benchmark import BenchmarkCNN
    from kf_benchmarks_amd.parallel import comm
    p = P.make_params(**kw)
    trace = []
    if os.environ.get("KFB_TEST_TRACE_BUCKETS"):
        from kf_benchmarks_amd.parallel import bucket
        oh, ol = bucket.BucketReducer._hook, bucket.BucketReducer._launch

        def hook(self, q):
            trace.append(("hook", getattr(q, "_kfb_name", "?"), self.param_bucket.get(id(q)),
                          self._active))
            oh(self, q)

        def launch(self, b, src=None):
            trace.append(("launch", b, list(self._pending)))
            ol(self, b, src)
        bucket.BucketReducer._hook, bucket.BucketReducer._launch = hook, launch
    bench = BenchmarkCNN(p)
    bench.build()
    for name, q, _, _ in bench.flat.segments():
        q._kfb_name = name
    bench.strategy.broadcast_initial_model(bench.optimizer.slot_tensors().values())
    w0 = bench.flat.flat.detach().double().sum().item()
    gsegs = []
    if os.environ.get("KFB_TEST_GRAD_SEGS"):
        orig = bench.strategy.after_backward

        def after_backward(step):
            orig(step)
            torch.cuda.synchronize()
            g = bench.flat.grad
            gsegs.append({name: g[off:off + n].double().sum().item()
                          for name, _, off, n in bench.flat.segments()})
        bench.strategy.after_backward = after_backward
    torn = _inject_torn_snapshot(bench, comm.get_world().rank)
    losses = []
    for _ in range(steps):
        loss, _ = bench.train_step(need_loss=True)
        losses.append(float(loss))
    torch.cuda.synchronize()
    # exposed all-reduce per step from the reducer's native timing events
    # (recorded into the launch tape too, so replayed steps report as well)
    exposed = (bench.strategy.reducer.pop_exposed_ms()
               if bench.strategy.reducer is not None else [])
    reduce_identity = None
    if os.environ.get("KFB_TEST_REDUCE_IDENTITY") and bench.strategy.reducer is not None:
        # one more synchronous all-reduce of the last gradient over the group:
        # at world size 1 RCCL must return it bit for bit
        g0 = bench.flat.grad.detach().clone()
        bench.strategy.reducer.reduce_now()
        torch.cuda.synchronize()
        reduce_identity = bool(torch.equal(g0, bench.flat.grad)) and bool(g0.abs().sum() > 0)
    hier_identity = None
    if os.environ.get("KFB_TEST_HIER"):
        # a hierarchical (HierarchicalCopy) reducer over the same world: in a
        # native-communicator run its subgroups are native communicators too
        from kf_benchmarks_amd.parallel import allreduce as _ar
        h = _ar.Hierarchical(comm.get_world().size, comm.get_world().rank)
        t = torch.arange(4096, dtype=torch.float32, device="cuda")
        for w in h.launch(t):
            w.wait()
        torch.cuda.synchronize()
        hier_identity = bool(torch.equal(t, torch.arange(4096, dtype=torch.float32,
                                                         device="cuda")))
    import torch.distributed as dist
    nccl_pgs = 0
    if dist.is_initialized():
        for pg in list(dist.distributed_c10d._world.pg_map.keys()):
            try:
                if dist.get_backend(pg) == "nccl":
                    nccl_pgs += 1
            except Exception:  # noqa: BLE001 - a group this rank is not in
                pass
    flat = bench.flat.flat.detach()
    res = {"reduce_identity": reduce_identity, "hier_identity": hier_identity,
           "nccl_pgs": nccl_pgs, "losses": losses, "w0": w0, "wsum": flat.double().sum().item(),
           "wabs": flat.double().abs().sum().item(), "head": flat[:64].cpu().tolist(),
           "tail": flat[-64:].cpu().tolist(), "rank": comm.get_world().rank,
           "gsegs": gsegs, "trace": trace, "exposed_ms": exposed,
           "segs": {name: flat[off:off + n].double().sum().item()
                    for name, _, off, n in bench.flat.segments()},
           "size": comm.get_world().size, "backend": comm.get_world().device_backend,
           "taped": getattr(getattr(bench, "_tape", None), "replays", 0),
           "tower_mode": bench.tower_mode,
           "bucket_launches": (bench.strategy.reducer.launch_count
                               if bench.strategy.reducer is not None else 0),
           "num_buckets": (bench.strategy.reducer.num_buckets
                           if bench.strategy.reducer is not None else 0)}
    state = getattr(bench.strategy, "state", None)
    if state is not None:  # asynchronous parameter server
        comm.get_world().barrier()
        res["ps_global_step"] = state.global_step
        # every rank reads the SAME shared model (rank 0's device memory,
        # mapped into the others): equal checksums mean the applies landed
        # in one model, not in per-rank copies
        torch.cuda.synchronize()
        res["ps_shared_sum"] = [float(t.double().sum()) for t in state.shared]
        res["ps_shared_views"] = [t.data_ptr() for t in state.shared]
        comm.get_world().barrier()
        bench.strategy.close()
    elif getattr(bench.strategy, "store", None) is not None:  # PairAveraging
        res["pa_publishes"] = bench.strategy.store.publishes
        res["pa_retries"] = bench.strategy.store.retries
        bench.strategy.close()  # collective: no peer is still reading our slots
        res["pa_torn"] = bench.strategy.torn_snapshots
        res["torn_check"] = torn
    with open(out, "w") as f:
        json.dump(res, f)
    comm.get_world().shutdown()


def _inject_torn_snapshot(bench, rank):
    """KFB_TEST_TORN_STEP=s (rank 0, PairAveraging): at step s the pull's
    expected sequence word is off by one publish, as if the peer rewrote the
    slot during the copy; the device seqlock check must reject the snapshot
    and the fused update skip the averaging.  Records the update's inputs
    and output at that step (filled in as the step runs)."""
    import torch
    s = int(os.environ.get("KFB_TEST_TORN_STEP", "-1"))
    st = bench.strategy
    out = {}
    if s < 0 or rank != 0 or getattr(st, "store", None) is None:
        return out
    store = st.store
    orig_pv = store.pull_values

    def pull_values(peer):
        v = orig_pv(peer)
        if bench.global_step == s:
            v = dict(v, pa_seq=v["pa_seq"] + 2)
        return v
    store.pull_values = pull_values
    opt = bench.optimizer
    orig_step = opt.step

    def step(lr, grad_scale=1.0, weight_decay=0.0, clip=None, grad=None, mix=None, wout=None,
             **k):
        if bench.global_step != s:
            return orig_step(lr, grad_scale, weight_decay, clip, grad, mix, wout, **k)
        torch.cuda.synchronize()
        w = bench.flat.flat.detach().clone()
        g = bench.flat.grad.detach().clone()
        peer = mix[0].detach().clone()
        r = orig_step(lr, grad_scale, weight_decay, clip, grad, mix, wout, **k)
        torch.cuda.synchronize()
        post = bench.flat.flat.detach()
        gk = g * grad_scale
        nomix = w - lr * (gk + weight_decay * w)
        avg = 0.5 * w + 0.5 * peer
        withmix = avg - lr * (gk + weight_decay * w)
        scale = float(post.abs().max())
        out.update(err_nomix=float((post - nomix).abs().max()) / scale,
                   err_mix=float((post - withmix).abs().max()) / scale,
                   peer_differs=bool(float((peer - w).abs().max()) > 0),
                   ok_flag=int(mix[3].item()) if mix[3] is not None else None)
        return r
    opt.step = step
    return out


if __name__ == "__main__":
    main()
