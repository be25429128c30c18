"""Generates tests/golden/c1_learner_f32.npz: the fp32 oracle's run of config C1 - the reference loop
with Parameter::default(), 1 env, B = 32, 10,000 env-steps - for tests/test_gpu_learner.py::
test_f32_c1_reference_loop_golden.  Runs the CPU restatement only (oracle/liboracle.so, ~2-3 minutes on 8 cores).

    python tests/golden/make_c1_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle as O   # noqa: E402


def main():
    ref = O.Learner(O.default_params(n_envs=1, batch_size=32))
    acts, rews, dones, losses = [], [], [], []
    h_idx, h_tg = hashlib.sha256(), hashlib.sha256()
    for _ in range(10_000):
        ref.vector_step()
        r = ref.last()
        acts.append(r["actions"][0]); rews.append(r["rewards"][0]); dones.append(r["dones"][0])
        if len(r["losses"]):
            losses.extend(r["losses"].tolist())
            h_idx.update(r["indices"].astype(np.uint64).tobytes())
            h_tg.update(r["targets"].astype(np.float32).tobytes())
    q = ref.qnet(0)
    hw = hashlib.sha256()
    for v in range(10):
        for which in range(3):
            hw.update(q.get(v, which).astype(np.float32).tobytes())
    out = os.path.join(HERE, "c1_learner_f32.npz")
    np.savez(out, actions=np.array(acts, np.uint8), rewards=np.array(rews, np.float32), dones=np.array(dones, np.uint8),
             losses=np.array(losses, np.float32), indices_sha256=np.array(h_idx.hexdigest()),
             targets_sha256=np.array(h_tg.hexdigest()), model_sha256=np.array(hw.hexdigest()))
    c = ref.counters()
    print(f"wrote {out}: {len(losses)} updates, episodes {c['episode_count']}, last loss {losses[-1]:.6f}")


if __name__ == "__main__":
    main()
