"""A/B probe of the background-row list regions (kListSlots): the fp32 forward with row lists on against the dense one
(QLX_F32_BG=0) at several batch sizes, bit for bit, then the learner scenario of tests/test_gpu_qnet32_paths.py
test_frame_sparsity checked after every step.  Run with QLX_LIB_PATH pointing at the build under test."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, ROOT + "/tests", ROOT + "/q-learning_amd"]
import qlx  # noqa: E402
from test_gpu_qnet32 import env_states  # noqa: E402
from test_gpu_qnet32_paths import _sparsity_ref  # noqa: E402

MODE = sys.argv[1] if len(sys.argv) > 1 else "all"   # all | learner (no models first) | late (first check after run(3))
xs = env_states(9000 if MODE == "all" else 1, seed=5)
models = {}
for bg in (("1", "0") if MODE == "all" else ()):
    os.environ["QLX_F32_BG"] = bg
    m = qlx.DeepQLearningModel(seed=7)
    models[bg] = m
os.environ.pop("QLX_F32_BG", None)
for v in range(10 if MODE == "all" else 0):
    models["0"].set(v, models["1"].get(v, 0))
for n in () if MODE != "all" else (1, 3, 64, 256, 300, 1024, 3000, 9000):
    q = {bg: models[bg].q_values(xs[:n])[0] for bg in ("1", "0")}
    bad = int((q["1"].view(np.uint32) != q["0"].view(np.uint32)).sum())
    print(f"n={n}: q differ {bad} of {q['1'].size}", flush=True)

p = qlx.Parameter(n_envs=256, batch_size=64, update_after_actions=8, history_buffer_len=20_000, env_seed=11,
                  epsilon_pure_random_steps=0)
L = qlx.SelfDrivingQLearner(p)
try:
    L.prefill(40)
    if MODE == "late":
        L.run(3)
    for k in range(4):
        f = L.frame_sparsity()
        want = _sparsity_ref(np.ascontiguousarray(L.environment.state().transpose(0, 3, 1, 2)))
        print(f"step {k}: act {np.asarray(f['act'])} want {want}", flush=True)
        L.run(1)
finally:
    L.close()
