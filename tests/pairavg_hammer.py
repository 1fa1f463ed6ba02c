"""One rank of the PairAveraging model-store hammer test: rank 0 publishes
constant-valued snapshots (value = publish index) as fast as it can, rank 1
pulls concurrently; every accepted snapshot must be uniform (no torn read).

usage: pairavg_hammer.py <out.json> <device cpu|cuda> <numel> <seconds>"""

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    out, device, n, seconds = sys.argv[1], sys.argv[2], int(sys.argv[3]), float(sys.argv[4])
    import torch
    from kf_benchmarks_amd.parallel import comm
    from kf_benchmarks_amd.parallel.kungfu import ModelStore
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
        store.flush()
        res["publishes"] = k
    else:
        buf = torch.empty_like(flat)
        pulls, torn, seen = 0, 0, set()
        while time.time() < t_end:
            store.pull(0, buf)
            lo, hi = float(buf.min()), float(buf.max())
            pulls += 1
            if lo != hi:
                torn += 1
            seen.add(lo)
        res.update(pulls=pulls, torn=torn, distinct=len(seen), retries=store.retries)
    world.barrier()
    store.close()
    with open(out, "w") as f:
        json.dump(res, f)
    world.shutdown()


if __name__ == "__main__":
    main()
