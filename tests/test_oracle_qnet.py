"""Pins the fp32 Q-network oracle against an independent float64 torch-autograd restatement of the
reference Keras graph (create_ql_model_breakout_84x84x4_3_32.py:20-33, train semantics q_a = Q(s)[a],
Huber(1) mean, tf.clip_by_norm per variable, ResourceApplyAdam)."""
import numpy as np
import pytest
import torch

import oracle as O


def torch_forward(ws, x_u8):
    """x: [B][84][84][4] (x, y, slot) = NHWC with H = x. Keras HWIO kernels."""
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64))
    x = t(x_u8).permute(0, 3, 1, 2)                       # NCHW
    k0, b0, k1, b1, k2, b2, k3, b3, k4, b4 = [t(w).requires_grad_(True) for w in ws]
    h = torch.relu(torch.nn.functional.conv2d(x, k0.permute(3, 2, 0, 1), b0, stride=4))
    h = torch.relu(torch.nn.functional.conv2d(h, k1.permute(3, 2, 0, 1), b1, stride=2))
    h = torch.relu(torch.nn.functional.conv2d(h, k2.permute(3, 2, 0, 1), b2, stride=1))
    h = h.permute(0, 2, 3, 1).reshape(x.shape[0], -1)    # Flatten of NHWC: (h, w, c)
    h = torch.relu(h @ k3 + b3)
    q = h @ k4 + b4
    return q, [k0, b0, k1, b1, k2, b2, k3, b3, k4, b4]


def rand_states(B, seed):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 256, size=(B, 84, 84, 4), dtype=np.uint8)
    x[:, :, :, rng.integers(0, 4)] = 0      # a zeroed slot like after a reset
    return x


def test_oracle_forward_matches_torch():
    net = O.QNet(seed=2)
    ws = net.weights()
    x = rand_states(3, 0)
    q = net.forward(x)
    qt, _ = torch_forward(ws, x)
    assert np.allclose(q, qt.detach().numpy(), rtol=1e-5, atol=1e-5 * np.abs(q).max())


def test_oracle_train_matches_torch_and_legacy_adam():
    net = O.QNet(seed=3)
    ws = [w.copy() for w in net.weights()]
    B = 4
    x = rand_states(B, 1)
    a = np.array([0, 2, 1, 2], np.uint8)
    q0 = net.forward(x)
    y = (q0[np.arange(B), a] + np.array([0.3, -2.5, 0.9, 1.7], np.float32)).astype(np.float32)
    loss, grads, norms = net.train(x, a, y)
    # torch reference: Huber(delta=1) mean over batch, q_a = Q(s)[a]
    qt, params = torch_forward(ws, x)
    qa = qt[torch.arange(B), torch.as_tensor(a.astype(np.int64))]
    lt = torch.nn.functional.huber_loss(qa, torch.as_tensor(y.astype(np.float64)), delta=1.0, reduction="mean")
    lt.backward()
    assert abs(loss - lt.item()) <= 1e-5 * max(1.0, abs(lt.item()))
    for g, p in zip(grads, params):
        ref = p.grad.numpy()
        scale = np.abs(ref).max() + 1e-12
        assert np.abs(g - ref).max() <= 1e-4 * scale
    # clip_by_norm + ResourceApplyAdam, restated in numpy fp32 (t = 1)
    lr, b1, b2, eps = np.float32(2.5e-4), np.float32(0.9), np.float32(0.999), np.float32(1e-7)
    alpha = lr * np.sqrt(np.float32(1) - b2) / (np.float32(1) - b1)
    for v in range(10):
        g = grads[v].astype(np.float32)
        n = np.float32(np.sqrt(np.sum(g.astype(np.float64) ** 2)))
        assert abs(n - norms[v]) <= 1e-5 * max(n, 1e-20)
        gc = g / np.maximum(n, np.float32(1.0))
        m = (gc - 0) * (np.float32(1) - b1)
        vv = (gc * gc - 0) * (np.float32(1) - b2)
        w_ref = ws[v] - (m * alpha) / (np.sqrt(vv) + eps)
        assert np.allclose(net.get(v), w_ref, rtol=0, atol=1e-7 + 1e-6 * np.abs(ws[v]).max())
    assert net.iterations() == 1


def test_glorot_limits_and_determinism():
    a, b = O.QNet(seed=5), O.QNet(seed=5)
    fans = [(256, 2048), (512, 1024), (576, 576), (3136, 512), (512, 3)]
    for l, (fi, fo) in enumerate(fans):
        w = a.get(2 * l)
        lim = np.sqrt(6.0 / (fi + fo))
        assert np.abs(w).max() <= lim and np.abs(w).max() > 0.9 * lim
        assert np.array_equal(w, b.get(2 * l))
        assert not a.get(2 * l + 1).any()
