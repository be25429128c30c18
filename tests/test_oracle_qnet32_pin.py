"""Pins oracle/qnet32_ref.cpp - the fp32 arithmetic the product's QLX_ARCH_NATURE_DQN path is bit-exact to - against an
independent float64 torch-autograd restatement of the reference Keras graph and train step:
create_ql_model_breakout_84x84x4_3_32.py:20-33 (Conv2D 32/8/s4, 64/4/s2, 64/3/s1, Flatten, Dense 512, Dense 3; valid
padding, NHWC with H = x, ReLU), :63-82 (train: Huber(delta 1) mean over the batch of q_a = Q(s)[a] vs y, legacy Keras
Adam(lr 2.5e-4, clipnorm 1.0) = tf.clip_by_norm per variable + ResourceApplyAdam).

Checked per batch (B 4 / 32 / 256, env-rendered frames and random frames): all four activations and Q, the loss, all ten
raw gradients, the ten clip norms, and the weights and both Adam slots after two consecutive train steps (the second
step's gradients are taken by torch at the oracle's weights after the first, so each step is pinned on its own).
The gradient references use the oracle's ReLU decisions, after checking that every unit where they differ from torch's
sits at the kink (kink_masks).  Tolerances (measured margins >= 3x): forward and loss <= 1e-5 relative to the tensor's max |value|, gradients <= 1e-4,
norms <= 1e-5 against float64 norms of the same gradients, Adam state against a float64 restatement of clip_by_norm +
ResourceApplyAdam fed the oracle's own fp32 gradients (m, v <= 1e-5 relative; w within 1e-7 + 1e-6 max|w|).
The last test compares the fp32 chain oracle with the double-accumulating restatement (oracle/qnet_ref.cpp) at B = 1024.
"""
import numpy as np
import pytest
import torch

import oracle as O

# Keras holds the hyperparameters as float32 tensors: their float32 values, widened exactly
LR, B1, B2, EPS, CLIP = (float(np.float32(c)) for c in (2.5e-4, 0.9, 0.999, 1e-7, 1.0))


def torch_forward(ws, x_u8, masks=None):
    """float64 Keras graph: x [B][84][84][4] u8 (x, y, slot) = NHWC with H = x; HWIO kernels.  Returns q, the post-ReLU
    activations and the pre-activations in the oracle's NHWC layouts, and the leaf parameters.  masks (NHWC bool per
    layer) replaces each ReLU's own decision z > 0 (see kink_masks)."""
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64))
    x = t(x_u8).permute(0, 3, 1, 2)
    params = [t(w).requires_grad_(True) for w in ws]
    k0, b0, k1, b1, k2, b2, k3, b3, k4, b4 = params
    pre, acts = [], []

    def relu(z, l, nchw):
        pre.append((z.permute(0, 2, 3, 1) if nchw else z).detach().numpy())
        if masks is None:
            h = torch.relu(z)
        else:
            m = torch.as_tensor(masks[l])
            h = z * (m.permute(0, 3, 1, 2) if nchw else m)
        acts.append(h.permute(0, 2, 3, 1) if nchw else h)
        return h

    h = relu(torch.nn.functional.conv2d(x, k0.permute(3, 2, 0, 1), b0, stride=4), 0, True)
    h = relu(torch.nn.functional.conv2d(h, k1.permute(3, 2, 0, 1), b1, stride=2), 1, True)
    h = relu(torch.nn.functional.conv2d(h, k2.permute(3, 2, 0, 1), b2, stride=1), 2, True)
    f = h.permute(0, 2, 3, 1).reshape(x.shape[0], -1)    # Flatten of NHWC: (h, w, c)
    h = relu(f @ k3 + b3, 3, False)
    q = h @ k4 + b4
    return q, acts, pre, params


def kink_masks(net, x):
    """The oracle's ReLU decisions (a > 0) for the batch, after checking that every unit where they differ from float64
    torch's own sits at the kink: |z| <= 1e-5 max|z| of its layer.  With the masks aligned, a gradient comparison measures
    the arithmetic, not a unit whose pre-activation rounds to the other side of zero (observed: one such unit moves the
    conv1 / conv2 gradients of a 256-sample batch by up to 3e-3 relative)."""
    _, acts = net.forward(x, acts=True)
    _, _, pre, _ = torch_forward(net.weights(), x)
    masks = []
    for l in range(4):
        m = acts[l] > 0
        diff = m != (pre[l] > 0)
        assert np.all(np.abs(pre[l][diff]) <= 1e-5 * np.abs(pre[l]).max()), f"layer {l + 1}: mask differs off the kink"
        masks.append(m)
    return masks


def torch_loss_grads(ws, x, a, y, masks=None):
    q, _, _, params = torch_forward(ws, x, masks)
    B = x.shape[0]
    qa = q[torch.arange(B), torch.as_tensor(a.astype(np.int64))]
    loss = torch.nn.functional.huber_loss(qa, torch.as_tensor(y.astype(np.float64)), delta=1.0, reduction="mean")
    loss.backward()
    return loss.item(), [p.grad.numpy() for p in params]


def adam_f64(w, m, v, g, t):
    """tf.clip_by_norm(g, 1) + legacy ResourceApplyAdam at step t (1-based), in float64."""
    g = g.astype(np.float64)
    n = np.sqrt(np.sum(g * g))
    gc = g * CLIP / max(n, CLIP)
    alpha = LR * np.sqrt(1 - B2 ** t) / (1 - B1 ** t)
    m = m + (gc - m) * (1 - B1)
    v = v + (gc * gc - v) * (1 - B2)
    return w - m * alpha / (np.sqrt(v) + EPS), m, v, n


def relmax(a, ref):
    return float(np.abs(np.asarray(a, np.float64) - ref).max() / (np.abs(ref).max() + 1e-30))


def frames(kind, B):
    if kind == "env":   # frames rendered by the restated Breakout env after 40 random-action steps per env
        _, _, _, _, tens = O.envs_run(0x5EED, B, 40, 7, want_tensors=True)
        return tens
    rng = np.random.default_rng(B)
    x = rng.integers(0, 256, size=(B, 84, 84, 4), dtype=np.uint8)
    x[:, :, :, rng.integers(0, 4)] = 0      # a zeroed ring slot, as after a reset
    return x


@pytest.mark.parametrize("B,kind", [(4, "random"), (32, "env"), (32, "random"), (256, "env"), (256, "random")])
def test_qnet32_oracle_pinned_by_float64_torch(B, kind):
    net = O.QNet(seed=11 + B, f32=True)
    x = frames(kind, B)
    rng = np.random.default_rng(100 + B)
    a = rng.integers(0, 3, size=B).astype(np.uint8)
    w = [v.astype(np.float64) for v in net.weights()]
    m = [np.zeros_like(v) for v in w]
    vv = [np.zeros_like(v) for v in w]

    # forward: activations and Q
    q, acts = net.forward(x, acts=True)
    qt, at, _, _ = torch_forward(net.weights(), x)
    assert relmax(q, qt.detach().numpy()) <= 1e-5
    for l in range(4):
        assert relmax(acts[l], at[l].detach().numpy()) <= 1e-5, f"a{l + 1}"

    for step in (1, 2):
        q = net.forward(x)
        # targets on both sides of the Huber knee
        y = (q[np.arange(B), a] + rng.choice([-2.5, -0.4, 0.3, 1.7], size=B)).astype(np.float32)
        ws32 = net.weights()
        loss_t, grads_t = torch_loss_grads(ws32, x, a, y, kink_masks(net, x))
        loss, grads, norms = net.train(x, a, y)
        assert abs(loss - loss_t) <= 1e-5 * max(abs(loss_t), 1e-30), (step, loss, loss_t)
        for v in range(10):
            assert relmax(grads[v], grads_t[v]) <= 1e-4, (step, v, relmax(grads[v], grads_t[v]))
            g64 = grads[v].astype(np.float64)
            assert abs(norms[v] - np.sqrt(np.sum(g64 * g64))) <= 1e-5 * np.sqrt(np.sum(g64 * g64)) + 1e-30, (step, v)
            assert abs(norms[v] - np.linalg.norm(grads_t[v])) <= 1e-4 * np.linalg.norm(grads_t[v]), (step, v)
            # Adam state against the float64 restatement fed the oracle's own gradients, from the oracle's prior state
            w[v], m[v], vv[v], _ = adam_f64(w[v], m[v], vv[v], grads[v], step)
            assert relmax(net.get(v, 1), m[v]) <= 1e-5, (step, v, "m")
            assert relmax(net.get(v, 2), vv[v]) <= 1e-5, (step, v, "v")
            assert np.abs(net.get(v, 0) - w[v]).max() <= 1e-7 + 1e-6 * np.abs(w[v]).max(), (step, v, "w")
            # continue from the oracle's own fp32 state (each step pinned on its own)
            w[v], m[v], vv[v] = (net.get(v, k).astype(np.float64) for k in range(3))
        assert net.iterations() == step


def test_qnet32_oracle_agrees_with_double_accumulating_oracle_b1024():
    """The fp32 chain definition against the double-accumulating restatement (qnet_ref.cpp) at a training batch:
    Q and all ten gradients."""
    B = 1024
    x = frames("env", B)
    a = np.random.default_rng(5).integers(0, 3, size=B).astype(np.uint8)
    n32, n64 = O.QNet(seed=9, f32=True), O.QNet(seed=9, f32=False)
    q32, q64 = n32.forward(x), n64.forward(x)
    assert relmax(q32, q64.astype(np.float64)) <= 1e-5
    y = (q64[np.arange(B), a] + np.random.default_rng(6).choice([-2.0, 0.5], size=B)).astype(np.float32)
    l32, g32, nr32 = n32.train(x, a, y)
    l64, g64, nr64 = n64.train(x, a, y)
    assert abs(l32 - l64) <= 1e-5 * abs(l64)
    for v in range(10):
        assert relmax(g32[v], g64[v].astype(np.float64)) <= 1e-4, (v, relmax(g32[v], g64[v].astype(np.float64)))
        assert abs(nr32[v] - nr64[v]) <= 1e-4 * nr64[v], v
