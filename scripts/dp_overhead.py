"""Cost of the data-parallel update path on one GPU: the bench workload with and without a single-rank RCCL
communicator (bucketed all-reduce on the communicator stream; identity reductions).  Development tool."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "q-learning_amd"))
import qlx  # noqa: E402


def run(dp, steps=30):
    p = qlx.Parameter(n_envs=1024, batch_size=1024, update_after_actions=128, history_buffer_len=100_000)
    L = qlx.SelfDrivingQLearner(p)
    if dp:
        L.dist_init(1, 0, qlx.dist_unique_id())
    L.run(55)
    L.sync()
    t0 = time.perf_counter()
    L.run(steps)
    L.sync()
    dt = (time.perf_counter() - t0) / steps
    L.close()
    return dt * 1e3


for dp in (False, True, "seq", True):
    if dp == "seq":
        os.environ["QLX_DP_OVERLAP"] = "0"
    else:
        os.environ.pop("QLX_DP_OVERLAP", None)
    print(f"dp={dp}: {run(dp):.3f} ms per vector step", flush=True)
