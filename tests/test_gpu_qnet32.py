"""GPU Q-network in fp32 (QLX_ARCH_NATURE_DQN, the reference's float32 arithmetic) vs the fp32 oracle: BIT-EXACT.

The reference graph is float32 Keras (create_ql_model_breakout_84x84x4_3_32.py:20-61).  The product runs it on
v_mfma_f32_16x16x4_f32, which is a k-ordered fmaf chain (scripts/mfma_f32_probe.hip, measured on MI355X), with ONE
accumulator per output over the whole reduction; oracle/qnet32_ref.cpp restates the same chains on the CPU
(DESIGN.md §6 fixes every order).  So forward activations, Q values, the loss, all ten raw gradients, the clip_by_norm
norms and the post-Adam weights / Adam slots must be equal bit for bit, at every batch size, for any number of
consecutive steps.  tests/test_oracle_qnet32_pin.py pins that oracle (qnet32_ref.cpp) against float64 torch autograd:
activations / Q / loss 1e-5, gradients 1e-4, norms, and w / m / v after two Adam steps.
"""
import ctypes

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _qlx():
    import qlx
    return qlx


def rand_states(B, seed, sparse=False):
    rng = np.random.default_rng(seed)
    if sparse:   # Breakout-like: mostly background, a few bright blocks
        x = np.zeros((B, 84, 84, 4), np.uint8)
        for b in range(B):
            for _ in range(6):
                i, j = rng.integers(0, 80, 2)
                x[b, i:i + 4, j:j + 4, rng.integers(0, 4)] = rng.choice([96, 236, 255])
        return x
    return rng.integers(0, 256, size=(B, 84, 84, 4), dtype=np.uint8)


def edge_states(B):
    """One bright pixel per sample (every x and y over the batch, all four frames): the background classification's
    block boundaries (4-pixel blocks, 20 / 36-pixel receptive fields at stride 8) are crossed at every offset."""
    x = np.zeros((B, 84, 84, 4), np.uint8)
    for b in range(B):
        x[b, b % 84, (b * 13 + b // 84) % 84, b % 4] = 1 + b % 255
    return x


def env_states(B, seed=123):
    """Real Breakout observations from the oracle env (random play)."""
    out = []
    env = O.Env(seed=seed)
    rng = np.random.default_rng(5)
    while len(out) < B:
        r, d = env.step(int(rng.integers(0, 3)))
        out.append(env.tensor())
        if d:
            env.reset()
    return np.stack(out)


def mixed_states(B, seed):
    return np.concatenate([env_states(B // 2, seed), rand_states(B - B // 2, seed, sparse=True)])


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def randomize(m, ref, seed):
    """Non-trivial weights and biases (GlorotUniform-sized, biases non-zero) set identically on both."""
    rng = np.random.default_rng(seed)
    for v in range(10):
        w = ref.get(v)
        if v % 2 == 1:
            w = rng.normal(0, 0.05, w.shape).astype(np.float32)
        else:
            w = (w * rng.uniform(0.5, 1.5)).astype(np.float32)
        m.set(v, w)
        ref.set(v, w)


def test_init_weights_bit_identical():
    m = _qlx().DeepQLearningModel(seed=2)
    ref = O.QNet(seed=2, f32=True)
    for v in range(10):
        assert same(m.get(v), ref.get(v)), f"var {v}"


@pytest.mark.parametrize("B,kind", [(1, "env"), (31, "rand"), (129, "sparse"), (256, "env"), (1024, "mixed"), (64, "zero"),
                                    (3000, "env"), (336, "edge"), (2600, "edge")])
def test_forward_bit_exact(B, kind):
    """Every layer bit for bit.  The conv2 / conv3 forward computes the non-background rows as a GEMM and writes the
    constant rows of the background ones (qnet32_kernels.h C1Lists): env frames are mostly background, random frames
    have none, zero frames are nothing else; B = 3,000 runs the chunk-size kernels."""
    qlx = _qlx()
    m = qlx.DeepQLearningModel(seed=2)
    ref = O.QNet(seed=2, f32=True)
    randomize(m, ref, B)
    x = {"env": lambda: env_states(B), "rand": lambda: rand_states(B, B), "sparse": lambda: rand_states(B, B, True),
         "mixed": lambda: mixed_states(B, B), "zero": lambda: np.zeros((B, 84, 84, 4), np.uint8), "edge": lambda: edge_states(B)}[kind]()
    q, a = m.q_values(x)
    qr, acts = ref.forward(x, acts=True)
    for layer in range(1, 5):
        got = np.zeros(acts[layer - 1].size, np.float32)
        assert qlx.lib().qlx_model_last_activation(m.h, layer, got.ctypes.data_as(ctypes.c_void_p)) == 0
        bad = np.flatnonzero(got.view(np.uint32) != acts[layer - 1].ravel().view(np.uint32))
        assert bad.size == 0, f"layer {layer}: {bad.size} elements differ, first {bad[:5]}"
    assert same(q, qr)
    assert np.array_equal(a, np.argmax(qr, axis=1))
    mx = m.batch_predict_max_future_reward(x)
    assert same(mx, qr.max(axis=1))


# (round 6) ragged batches and frames with no / only background rows exercise the compacted weight gradients' chunk
# tables (a partial last chunk, chunks with nothing kept, every row kept) and B > 2,048 the persistent conv1 forward's
# step masks and row flags
@pytest.mark.parametrize("B,kind", [(32, "mixed"), (320, "mixed"), (1024, "mixed"), (37, "mixed"), (1000, "env"), (64, "zero"),
                                    (96, "rand"), (3000, "sparse")])
def test_train_step_bit_exact(B, kind):
    m = _qlx().DeepQLearningModel(seed=7)
    ref = O.QNet(seed=7, f32=True)
    randomize(m, ref, 100 + B)
    x = {"env": lambda: env_states(B), "rand": lambda: rand_states(B, B), "sparse": lambda: rand_states(B, B, True),
         "mixed": lambda: mixed_states(B, B), "zero": lambda: np.zeros((B, 84, 84, 4), np.uint8)}[kind]()
    rng = np.random.default_rng(B)
    a = rng.integers(0, 3, B).astype(np.uint8)
    q0 = ref.forward(x)
    y = (q0[np.arange(B), a] + rng.normal(0, 1.5, B)).astype(np.float32)   # a mix of |e| < 1 and > 1
    loss, grads, norms = m.train(x, a, y, want_grads=True)
    loss_r, grads_r, norms_r = ref.train(x, a, y)
    assert same(np.float32(loss), np.float32(loss_r)), (loss, loss_r)
    for v in range(10):
        bad = np.flatnonzero(grads[v].ravel().view(np.uint32) != grads_r[v].ravel().view(np.uint32))
        assert bad.size == 0, f"gradient of var {v}: {bad.size} of {grads[v].size} differ (first {bad[:5]})"
    assert same(norms, norms_r)
    for v in range(10):
        for which in range(3):
            assert same(m.get(v, which), ref.get(v, which)), f"var {v} slot {which} after Adam"
    assert m.iterations() == ref.iterations() == 1


def test_consecutive_steps_stay_bit_exact():
    """16 updates, fresh batches and targets each step, Adam state carried: no drift at all."""
    m = _qlx().DeepQLearningModel(seed=11)
    ref = O.QNet(seed=11, f32=True)
    B = 128
    rng = np.random.default_rng(1)
    for step in range(16):
        x = mixed_states(B, 1000 + step)
        a = rng.integers(0, 3, B).astype(np.uint8)
        y = rng.normal(0, 1, B).astype(np.float32)
        l1 = m.train(x, a, y)
        l2, _, _ = ref.train(x, a, y)
        assert same(np.float32(l1), np.float32(l2)), f"step {step}: {l1} vs {l2}"
    for v in range(10):
        for which in range(3):
            assert same(m.get(v, which), ref.get(v, which)), f"var {v} slot {which}"


def test_chunked_forward_bit_exact():
    """B above the fp32 forward chunk (8,192 samples) runs the conv layers chunk by chunk: same bits."""
    m = _qlx().DeepQLearningModel(seed=3)
    ref = O.QNet(seed=3, f32=True)
    x = rand_states(8192 + 200, 17, sparse=True)
    q, a = m.q_values(x)
    sl = np.r_[0:64, 8150:8392]
    qr = ref.forward(x[sl])
    assert same(q[sl], qr)


def test_checkpoint_roundtrip_f32():
    import os
    import tempfile
    qlx = _qlx()
    m = qlx.DeepQLearningModel(seed=9)
    x = env_states(8)
    m.train(x, np.zeros(8, np.uint8), np.ones(8, np.float32))
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ckpt.qlx")
        m.write_checkpoint(path)
        m2 = qlx.DeepQLearningModel(seed=1)
        m2.read_checkpoint(path)
        for v in range(10):
            for which in range(3):
                assert same(m.get(v, which), m2.get(v, which))
        assert m2.iterations() == 1
        assert same(m.q_values(x)[0], m2.q_values(x)[0])
