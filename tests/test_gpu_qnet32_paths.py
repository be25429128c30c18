"""The fp32 Q-net's A/B code paths are bit-exact too, not only the default one.

The switches kept in the product (they have reporting roles: the bench's dense-frame figure) are exact alternatives:
the dense conv2 / conv3 forward without background rows (QLX_F32_BG=0) and conv1 issuing its all-zero frame steps
(QLX_F32_C1_SKIP=0), alone and together; and the grid shapes of a part with few CUs (QLX_NUM_CUS=8: a CPX partition
of an MI300X / MI355X - conv1 then runs more than two blocks per CU so that no block holds more than 64 samples).
Each must give the oracle's bits (oracle/qnet32_ref.cpp, the same chains as tests/test_gpu_qnet32.py): Q values and the
conv2 / conv3 activations of a 1,024-sample forward, Q of a 3,000-sample (chunk-size kernels) forward, and one training
step at B = 1,024 (loss, all ten gradients, the clip norms, w / m / v after Adam).

Most switches are read once per process (static), so each variant runs in a child process (one at a time, so at most
two processes hold the GPU) on inputs and weights the parent wrote; the parent compares against the oracle.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from test_gpu_qnet32 import env_states, mixed_states, randomize, same

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path[:0] = [sys.argv[3], sys.argv[3] + "/tests", sys.argv[3] + "/q-learning_amd"]
import ctypes
import qlx
d = np.load(sys.argv[1])
m = qlx.DeepQLearningModel(seed=7)
for v in range(10):
    m.set(v, d[f"w{v}"])
out = {}
out["q1"], _ = m.q_values(d["x1"])
for layer in (2, 3):
    n = d["x1"].shape[0] * (5184 if layer == 2 else 3136)
    got = np.zeros(n, np.float32)
    assert qlx.lib().qlx_model_last_activation(m.h, layer, got.ctypes.data_as(ctypes.c_void_p)) == 0
    out[f"a{layer}"] = got
out["q2"], _ = m.q_values(d["x2"])
loss, grads, norms = m.train(d["xt"], d["at"], d["yt"], want_grads=True)
out["loss"] = np.float32(loss)
out["norms"] = np.asarray(norms, np.float32)
for v in range(10):
    out[f"g{v}"] = grads[v]
    for which in range(3):
        out[f"s{v}_{which}"] = m.get(v, which)
np.savez(sys.argv[2], **out)
"""


@pytest.fixture(scope="module")
def case(tmp_path_factory):
    d = tmp_path_factory.mktemp("paths")
    ref = O.QNet(seed=7, f32=True)

    class _W:   # randomize() sets both; the child receives the weights through the file
        def __init__(self):
            self.w = {}

        def set(self, v, w):
            self.w[v] = w
    w = _W()
    randomize(w, ref, 1124)
    B = 1024
    x1 = env_states(B, seed=321)
    x2 = env_states(3000, seed=99)
    xt = mixed_states(B, B)
    rng = np.random.default_rng(B)
    at = rng.integers(0, 3, B).astype(np.uint8)
    q0 = ref.forward(xt)
    yt = (q0[np.arange(B), at] + rng.normal(0, 1.5, B)).astype(np.float32)
    inp = str(d / "in.npz")
    np.savez(inp, x1=x1, x2=x2, xt=xt, at=at, yt=yt, **{f"w{v}": w.w[v] for v in range(10)})
    exp = {}
    exp["q1"], acts = ref.forward(x1, acts=True)
    exp["a2"], exp["a3"] = acts[1].ravel(), acts[2].ravel()
    exp["q2"] = ref.forward(x2)
    loss, grads, norms = ref.train(xt, at, yt)
    exp["loss"], exp["norms"] = np.float32(loss), np.asarray(norms, np.float32)
    for v in range(10):
        exp[f"g{v}"] = grads[v]
        for which in range(3):
            exp[f"s{v}_{which}"] = ref.get(v, which)
    return d, inp, exp


@pytest.mark.parametrize("env", [{}, {"QLX_F32_BG": "0"}, {"QLX_F32_C1_SKIP": "0"},
                                 {"QLX_F32_BG": "0", "QLX_F32_C1_SKIP": "0"}, {"QLX_NUM_CUS": "8"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()) or "default")
def test_path_bit_exact(case, env):
    d, inp, exp = case
    out = str(d / ("out_" + ("_".join(f"{k}{v}" for k, v in env.items()) or "default") + ".npz"))
    cenv = {k: v for k, v in os.environ.items() if not k.startswith("QLX_F32_") and k != "QLX_NUM_CUS"}
    cenv.update(env)
    r = subprocess.run([sys.executable, "-c", CHILD, inp, out, ROOT], env=cenv, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    for k, want in exp.items():
        g = got[k]
        if g.size == np.asarray(want).size:
            g = g.reshape(np.asarray(want).shape)
        bad = np.flatnonzero(np.asarray(g).ravel().view(np.uint32) != np.asarray(want, np.float32).ravel().view(np.uint32))
        assert same(g, want), f"{env}: {k}: {bad.size} elements differ (first {bad[:5]})"
