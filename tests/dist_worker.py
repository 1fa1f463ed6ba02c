"""One rank of a multi-process CPU (gloo) test run with the analytic model.

usage: dist_worker.py <out.json> '<json flag kwargs>'
(role of tcb/benchmark_cnn_distributed_test_runner.py)."""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import kfb_test_util as tu  # noqa: E402


def main():
    out, kw = sys.argv[1], json.loads(sys.argv[2])
    params = tu.get_var_update_params(**kw)
    losses, _ = tu.run_test_model(params)
    from kf_benchmarks_amd.parallel import comm
    # the last bench is reachable through the world only; recompute vars via a fresh read
    import kf_benchmarks_amd.benchmark as bm  # noqa: F401
    with open(out, "w") as f:
        json.dump({"losses": losses, "vars": tu.LAST_VARS, "stats": tu.LAST_STATS}, f)
    comm.get_world().shutdown()


if __name__ == "__main__":
    main()
