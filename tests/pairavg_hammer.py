"""One rank of the PairAveraging model-store hammer test: rank 0 publishes
constant-valued snapshots (value = publish index) as fast as it can, rank 1
pulls concurrently; every accepted snapshot must be uniform (no torn read).

usage: pairavg_hammer.py <out.json> <device cpu|cuda> <numel> <seconds> [pace_us]

pace_us: the publisher's pause between snapshots.  A publisher rewriting
both slots faster than one pull completes starves the reader (every copy
overlaps a rewrite), which the store reports as TornReadError after its
bounded retries - counted here as a give-up, never as an accepted copy."""

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    out, device, n, seconds = sys.argv[1], sys.argv[2], int(sys.argv[3]), float(sys.argv[4])
    pace = float(sys.argv[5]) * 1e-6 if len(sys.argv) > 5 else 0.0
    import torch
    from kf_benchmarks_amd.parallel import comm
    from kf_benchmarks_amd.parallel.kungfu import ModelStore, TornReadError
    world = comm.init_world("cpu")  # gloo: both ranks may share one GPU
    dev = torch.device("cuda", 0) if device == "cuda" else torch.device("cpu")
    flat = torch.zeros(n, dtype=torch.float32, device=dev)
    store = ModelStore(flat, world)
    res = {"rank": world.rank}
    t_end = time.time() + seconds
    if world.rank == 0:
        k = 0
        while time.time() < t_end:
            k += 1
            flat.fill_(float(k))
            store.publish(flat)
            if pace:
                time.sleep(pace)
        store.flush()
        res["publishes"] = k
    else:
        buf = torch.empty_like(flat)
        pulls, torn, seen, gave_up = 0, 0, set(), 0
        while time.time() < t_end:
            try:
                store.pull(0, buf)
            except TornReadError:
                gave_up += 1
                continue
            lo, hi = float(buf.min()), float(buf.max())
            pulls += 1
            if lo != hi:
                torn += 1
            seen.add(lo)
        res.update(pulls=pulls, torn=torn, distinct=len(seen), retries=store.retries,
                   gave_up=gave_up)
    world.barrier()
    store.close()
    with open(out, "w") as f:
        json.dump(res, f)
    world.shutdown()


if __name__ == "__main__":
    main()
