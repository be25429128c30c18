"""The flow of tests/test_gpu_qnet32_paths.py test_frame_sparsity under pytest (the process where the 32-region A/B
build fails it), with the acting-frame check repeated: run as `pytest -s scripts/ls_pytest_probe.py`."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, ROOT + "/tests", ROOT + "/q-learning_amd"]
import oracle as O  # noqa: E402,F401  (imported as the test module does)
from test_gpu_qnet32_paths import _sparsity_ref  # noqa: E402


def test_probe():
    import qlx
    p = qlx.Parameter(n_envs=256, batch_size=64, update_after_actions=8, history_buffer_len=20_000, env_seed=11,
                      epsilon_pure_random_steps=0)
    L = qlx.SelfDrivingQLearner(p)
    try:
        L.prefill(40)
        L.run(3)
        f1 = L.frame_sparsity()
        f2 = L.frame_sparsity()
        want = _sparsity_ref(np.ascontiguousarray(L.environment.state().transpose(0, 3, 1, 2)))
        f3 = L.frame_sparsity()
        print("\nf1", f1["act"], "\nf2", f2["act"], "\nf3", f3["act"], "\nwant", want, flush=True)
        print("train", f1["train"], f2["train"], flush=True)
    finally:
        L.close()
