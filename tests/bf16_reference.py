"""Float64 torch reference of the GPU Q-network's *mixed-precision contract* (test infrastructure).

The product computes the Nature-DQN with bf16 MFMA operands and fp32 accumulation.  Its storage points
are: bf16 copies of the conv1..conv3 / full_layer kernels (fp32 master kept), bf16 post-ReLU activations
a1..a4, bf16 activation gradients dz1..dz4; the action layer, biases, Huber and Adam stay fp32.  This
module reproduces exactly those rounding points (round-to-nearest-even, like v_cvt_pk_bf16_f32) and
computes everything else in float64, so the GPU kernels can be checked tightly (only accumulation
order differs), independently of the bf16-vs-fp32 precision gap that the fp32 oracle comparison states.
"""
import numpy as np
import torch


def bf16(t):
    return t.to(torch.bfloat16).to(torch.float64)


class _RoundBoth(torch.autograd.Function):
    """Rounds the value and the incoming gradient to bf16 (stored activation and activation grad)."""

    @staticmethod
    def forward(ctx, x):
        return bf16(x)

    @staticmethod
    def backward(ctx, g):
        return bf16(g)


def forward_backward(weights, x_u8, actions=None, y=None):
    """Returns q (float64 numpy) and, when actions/y are given, (loss, grads list in Keras layouts)."""
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64))
    ws = [t(w) for w in weights]
    for i in (0, 2, 4, 6):
        ws[i] = bf16(ws[i])
    params = [w.clone().requires_grad_(True) for w in ws]
    k0, b0, k1, b1, k2, b2, k3, b3, k4, b4 = params
    R = _RoundBoth.apply
    x = t(x_u8).permute(0, 3, 1, 2)
    h = R(torch.relu(torch.nn.functional.conv2d(x, k0.permute(3, 2, 0, 1), b0, stride=4)))
    h = R(torch.relu(torch.nn.functional.conv2d(h, k1.permute(3, 2, 0, 1), b1, stride=2)))
    h = R(torch.relu(torch.nn.functional.conv2d(h, k2.permute(3, 2, 0, 1), b2, stride=1)))
    h = h.permute(0, 2, 3, 1).reshape(x.shape[0], -1)
    h = R(torch.relu(h @ k3 + b3))
    q = h @ k4 + b4
    if actions is None:
        return q.detach().numpy()
    B = x.shape[0]
    qa = q[torch.arange(B), torch.as_tensor(np.asarray(actions, dtype=np.int64))]
    loss = torch.nn.functional.huber_loss(qa, t(y), delta=1.0, reduction="mean")
    loss.backward()
    return q.detach().numpy(), loss.item(), [p.grad.numpy() for p in params]
