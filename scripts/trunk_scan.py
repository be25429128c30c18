"""Batch-size scan of the Q-net forward (q_values) to separate per-launch fixed cost from per-sample cost
of the fused trunk kernel; run under rocprofv3 --kernel-trace --stats."""
import sys

import numpy as np

sys.path.insert(0, "q-learning_amd")
import qlx  # noqa: E402

m = qlx.DeepQLearningModel(seed=3)
rng = np.random.default_rng(0)
for B in (256, 512, 1024, 2048, 4096):
    x = rng.integers(0, 256, size=(B, 84, 84, 4), dtype=np.uint8)
    for _ in range(5):
        m.q_values(x)
    print(B, "done", flush=True)
