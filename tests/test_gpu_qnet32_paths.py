"""The fp32 Q-net's A/B code paths are bit-exact too, not only the default one.

The switches kept in the product (they have reporting roles: the bench's dense-frame figure) are exact alternatives:
the dense conv2 / conv3 forward without background rows (QLX_F32_BG=0) and conv1 issuing its all-zero frame steps
(QLX_F32_C1_SKIP=0), alone and together; the dense variables' update on the model's second stream beside the conv backward
(QLX_F32_DENSE_OVERLAP=1) or on the learner stream (=0); and the grid shapes of a part with few CUs (QLX_NUM_CUS=8: a CPX partition
of an MI300X / MI355X - conv1 then runs more than two blocks per CU so that no block holds more than 64 samples).
Each must give the oracle's bits (oracle/qnet32_ref.cpp, the same chains as tests/test_gpu_qnet32.py; QLX_F32_BG=0 those of its dense
mode, orc_qnet32_set_dense: the conv weight gradients over every row): Q values and the
conv2 / conv3 activations of a 1,024-sample forward, Q of a 3,000-sample (chunk-size kernels) forward, and one training
step at B = 1,024 (loss, all ten gradients, the clip norms, w / m / v after Adam).

QLX_F32_BG / QLX_F32_C1_SKIP are read when a model is created (bench.py builds its dense-frame learner in-process),
QLX_NUM_CUS once per process; each variant runs in a child process (one at a time, so at most two processes hold the
GPU) on inputs and weights the parent wrote; the parent compares against the oracle.

test_frame_sparsity: the diagnostic that reports how much of that work the skips leave out (qlx_learner_frame_sparsity,
bench.py's per-step fractions) against a numpy restatement of the kernels' predicates.
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
    # the training step twice: the default chains (background-row compaction of the conv weight gradients) and the
    # dense-frame path's (QLX_F32_BG=0: every row)
    snap = {(v, which): ref.get(v, which) for v in range(10) for which in range(3)}
    it0 = ref.iterations()
    exps = {}
    for dense in (False, True):
        for (v, which), a in snap.items():
            ref.set(v, a, which)
        ref.set_iterations(it0)
        O.lib().orc_qnet32_set_dense(int(dense))
        e = dict(exp)
        loss, grads, norms = ref.train(xt, at, yt)
        e["loss"], e["norms"] = np.float32(loss), np.asarray(norms, np.float32)
        for v in range(10):
            e[f"g{v}"] = grads[v]
            for which in range(3):
                e[f"s{v}_{which}"] = ref.get(v, which)
        exps[dense] = e
    O.lib().orc_qnet32_set_dense(0)
    return d, inp, exps


@pytest.mark.parametrize("env", [{}, {"QLX_F32_BG": "0"}, {"QLX_F32_C1_SKIP": "0"},
                                 {"QLX_F32_BG": "0", "QLX_F32_C1_SKIP": "0"}, {"QLX_NUM_CUS": "8"},
                                 {"QLX_F32_DENSE_OVERLAP": "1"}, {"QLX_F32_DENSE_OVERLAP": "0"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()) or "default")
def test_path_bit_exact(case, env):
    d, inp, exps = case
    exp = exps[env.get("QLX_F32_BG") == "0"]
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


def _s2d(img):
    """[n, 4, 84, 84] u8 frames -> the replay's s2d layout [n, 4, 7056]: byte (bx * 21 + by) * 16 + xl * 4 + yl holds
    pixel (4 bx + xl, 4 by + yl)"""
    n = img.shape[0]
    return np.ascontiguousarray(img.reshape(n, 4, 21, 4, 21, 4).transpose(0, 1, 2, 4, 3, 5).reshape(n, 4, 7056))


def _sparsity_ref(img):
    """numpy restatement: conv1 forward (tile t, kq) steps - tile t = the 4 x 4 output patch (4 (t / 5), 4 (t % 5)),
    kq = (kh, hw): pixels (4 oh + kh, 4 (ow + hw) .. + 3) of every frame; conv1 weight-gradient (wave w, rs) steps -
    positions r = 4 rs + g (g < 4), pixels (4 oh + kh, 4 (ow + h) .. + 3), kh in {2 w, 2 w + 1}, h in {0, 1}; conv2 / conv3
    background rows - the 20 x 20 / 36 x 36 pixel field from (8 i, 8 j) all zero"""
    n = img.shape[0]
    nz = (img != 0).any(axis=1)                                   # [n, 84, 84]
    quad = nz.reshape(n, 84, 21, 4).any(axis=3)                   # [n, 84 rows, 21 dword columns]
    f = 0
    for t in range(25):
        for kq in range(16):
            kh, hw = kq >> 1, kq & 1
            rows = [4 * (4 * (t // 5) + a) + kh for a in range(4)]
            cols = [4 * (t % 5) + c + hw for c in range(4)]
            f += int((~quad[:, rows][:, :, cols].reshape(n, -1).any(axis=1)).sum())
    w_ = 0
    for w in range(4):
        for rs in range(100):
            rows, cols = [], []
            for g in range(4):
                r = 4 * rs + g
                oh, ow = divmod(r, 20)
                for kh in (2 * w, 2 * w + 1):
                    for h in (0, 1):
                        rows.append(4 * oh + kh)
                        cols.append(ow + h)
            w_ += int((~quad[:, rows, cols].any(axis=1)).sum())
    b2 = sum(int((~nz[:, 8 * i:8 * i + 20, 8 * j:8 * j + 20].reshape(n, -1).any(axis=1)).sum()) for i in range(9) for j in range(9))
    b3 = sum(int((~nz[:, 8 * i:8 * i + 36, 8 * j:8 * j + 36].reshape(n, -1).any(axis=1)).sum()) for i in range(7) for j in range(7))
    return np.array([f / (400.0 * n), w_ / (400.0 * n), b2 / (81.0 * n), b3 / (49.0 * n)])


def test_frame_sparsity():
    """qlx_learner_frame_sparsity against the numpy restatement on the same frames: the last vector step's sampled
    states (replay get_many of its indices) and the acting frames (the learner's env)"""
    import qlx
    p = qlx.Parameter(n_envs=256, batch_size=64, update_after_actions=8, history_buffer_len=20_000, env_seed=11,
                      epsilon_pure_random_steps=0)
    L = qlx.SelfDrivingQLearner(p)
    try:
        L.prefill(40)
        L.run(3)
        f = L.frame_sparsity()
        # (called again at once on the same frames: the read-back of the second of two back-to-back calls once came
        # back as zeros - the diagnostic's stream-ordered allocation, DESIGN.md round-5 notes)
        assert L.frame_sparsity() == f
        last = L.last()
        idx = last["indices"].ravel()
        assert idx.size == last["losses"].shape[0] * 64 > 0
        s = L.replay_buffer.get_many(idx)["state"].transpose(0, 3, 1, 2)
        want_t = _sparsity_ref(np.ascontiguousarray(s))
        want_a = _sparsity_ref(np.ascontiguousarray(L.environment.state().transpose(0, 3, 1, 2)))
        assert np.array_equal(np.asarray(f["train"]), want_t), (f["train"], want_t)
        assert np.array_equal(np.asarray(f["act"]), want_a), (f["act"], want_a)
        assert 0.2 < want_t[0] < 1.0 and 0.2 < want_t[2] < 1.0   # a real mix, not all-zero / all-live
    finally:
        L.close()
