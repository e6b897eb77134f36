"""ORACLE (test infrastructure only) -- CPU fp32 restatement of the reference score network.

Restates ``NCSN_LiDAR_small.forward`` (LiDARGen/models/ncsnv2.py:484-518) and the blocks
it is built from (LiDARGen/models/layers.py, LiDARGen/models/normalization.py) as plain
PyTorch-CPU functional code over a ``{state_dict key: tensor}`` mapping.  It is the
checker for the HIP score network, never the thing measured or shipped: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.

Pinned by ``tests/golden/scorenet_*.npz`` (outputs of the reference module itself,
produced by ``oracle/gen_golden.py``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def conv2d(x, w, b=None, dilation=1, circular=True, pad=None):
    """nn.Conv2d(k, stride 1, padding=pad, dilation, padding_mode='circular'|'zeros').

    conv3x3 (layers.py:37-44), dilated_conv3x3 (layers.py:55-60) use circular padding;
    begin/end conv (ncsnv2.py:433,436) and ConvMeanPool's conv (layers.py:291-301) zeros.
    """
    k = w.shape[-1]
    p = (k // 2) * dilation if pad is None else pad
    if p and circular:
        x = F.pad(x, (p, p, p, p), mode="circular")
        return F.conv2d(x, w, b, dilation=dilation)
    return F.conv2d(x, w, b, padding=p, dilation=dilation)


def elu(x):
    """get_act -> nn.ELU() (layers.py:11-13)."""
    return F.elu(x)


def instance_norm_pp(x, P, name):
    """InstanceNorm2dPlus.forward with bias=True (normalization.py:163-176)."""
    means = torch.mean(x, dim=(2, 3))
    m = torch.mean(means, dim=-1, keepdim=True)
    v = torch.var(means, dim=-1, keepdim=True)
    means = (means - m) / torch.sqrt(v + 1e-5)
    h = F.instance_norm(x, eps=1e-5)
    h = h + means[..., None, None] * P[name + ".alpha"][..., None, None]
    C = x.shape[1]
    return P[name + ".gamma"].view(-1, C, 1, 1) * h + P[name + ".beta"].view(-1, C, 1, 1)


def mean_pool2(o):
    """ConvMeanPool's 2x2 phase average (layers.py:309-313)."""
    return sum([o[:, :, ::2, ::2], o[:, :, 1::2, ::2], o[:, :, ::2, 1::2], o[:, :, 1::2, 1::2]]) / 4.0


def residual_block(x, P, name, cin, cout, down, dil):
    """ResidualBlock.forward (layers.py:443-456) incl. the ConvMeanPool/dilated variants (:405-441)."""
    d = 1 if dil is None else dil
    out = instance_norm_pp(x, P, name + ".normalize1")
    out = elu(out)
    out = conv2d(out, P[name + ".conv1.weight"], P[name + ".conv1.bias"], dilation=d)
    out = instance_norm_pp(out, P, name + ".normalize2")
    out = elu(out)
    if down and dil is None:
        out = mean_pool2(conv2d(out, P[name + ".conv2.conv.weight"], P[name + ".conv2.conv.bias"], circular=False))
        sc = mean_pool2(conv2d(x, P[name + ".shortcut.conv.weight"], P[name + ".shortcut.conv.bias"], circular=False))
    else:
        out = conv2d(out, P[name + ".conv2.weight"], P[name + ".conv2.bias"], dilation=d)
        if down or cin != cout:
            sc = conv2d(x, P[name + ".shortcut.weight"], P[name + ".shortcut.bias"], dilation=d)
        else:
            sc = x
    return sc + out


def rcu(x, P, name, n_blocks, n_stages=2):
    """RCUBlock.forward (layers.py:126-134): in-place residual x += residual."""
    for i in range(n_blocks):
        residual = x
        for j in range(n_stages):
            x = elu(x)
            x = conv2d(x, P[f"{name}.{i + 1}_{j + 1}_conv.weight"])
        x = x + residual
    return x


def crp(x, P, name, n_stages=2):
    """CRPBlock.forward (layers.py:76-83), maxpool 5x5 s1 p2."""
    x = elu(x)
    path = x
    for i in range(n_stages):
        path = F.max_pool2d(path, kernel_size=5, stride=1, padding=2)
        path = conv2d(path, P[f"{name}.convs.{i}.weight"])
        x = path + x
    return x


def msf(xs, P, name, shape):
    """MSFBlock.forward (layers.py:179-184): conv+bias, bilinear(align_corners=True), sum."""
    sums = None
    for i, h in enumerate(xs):
        h = conv2d(h, P[f"{name}.convs.{i}.weight"], P[f"{name}.convs.{i}.bias"])
        h = F.interpolate(h, size=shape, mode="bilinear", align_corners=True)
        sums = h if sums is None else sums + h
    # reference starts from zeros: 0 + h0 + h1 (bitwise identical to h0 + h1)
    return sums


def refine_block(xs, P, name, shape, n_in, end=False):
    """RefineBlock.forward (layers.py:234-249)."""
    hs = [rcu(x, P, f"{name}.adapt_convs.{i}", 2) for i, x in enumerate(xs)]
    h = msf(hs, P, f"{name}.msf", shape) if n_in > 1 else hs[0]
    h = crp(h, P, f"{name}.crp")
    return rcu(h, P, f"{name}.output_convs", 3 if end else 1)


def input_prep(x):
    """ncsnv2.py:485-496: h = 2x-1, append (xs, ys) = meshgrid(linspace(0,1,W), linspace(0,1,H))."""
    h = 2 * x - 1.0
    B, _, H, W = h.shape
    xs = torch.linspace(0, 1, steps=W)
    ys = torch.linspace(0, 1, steps=H)
    ys, xs = torch.meshgrid(ys, xs, indexing="ij")
    xy = torch.stack((xs, ys), dim=0).view(1, 2, H, W).repeat(B, 1, 1, 1)
    return torch.cat((h, xy), dim=1)


def scorenet_forward(P, x, y, ngf=128):
    """NCSN_LiDAR_small.forward(x, y) (ncsnv2.py:484-518).

    P: dict key -> float32 CPU tensor (incl. 'sigmas'); x: [B,2,H,W] f32; y: [B] long.
    """
    h = input_prep(x)
    out = conv2d(h, P["begin_conv.weight"], P["begin_conv.bias"], circular=False)
    l1 = residual_block(out, P, "res1.0", ngf, ngf, False, None)
    l1 = residual_block(l1, P, "res1.1", ngf, ngf, False, None)
    l2 = residual_block(l1, P, "res2.0", ngf, 2 * ngf, True, None)
    l2 = residual_block(l2, P, "res2.1", 2 * ngf, 2 * ngf, False, None)
    l3 = residual_block(l2, P, "res3.0", 2 * ngf, 2 * ngf, True, 2)
    l3 = residual_block(l3, P, "res3.1", 2 * ngf, 2 * ngf, False, 2)
    l4 = residual_block(l3, P, "res4.0", 2 * ngf, 2 * ngf, True, 4)
    l4 = residual_block(l4, P, "res4.1", 2 * ngf, 2 * ngf, False, 4)
    r1 = refine_block([l4], P, "refine1", l4.shape[2:], 1)
    r2 = refine_block([l3, r1], P, "refine2", l3.shape[2:], 2)
    r3 = refine_block([l2, r2], P, "refine3", l2.shape[2:], 2)
    o = refine_block([l1, r3], P, "refine4", l1.shape[2:], 2, end=True)
    o = instance_norm_pp(o, P, "normalizer")
    o = elu(o)
    o = conv2d(o, P["end_conv.weight"], P["end_conv.bias"], circular=False)
    used = P["sigmas"][y].view(x.shape[0], 1, 1, 1)
    return o / used


def to_torch_params(sd):
    return {k: torch.as_tensor(v) for k, v in sd.items()}


def dsm_loss(scores, used_sigmas, noise, masks, anneal_power=2.0):
    """Loss of anneal_dsm_score_estimation_with_mask with used_sigmas given (losses/dsm.py:80-93)."""
    B = scores.shape[0]
    target = -1 / (used_sigmas ** 2) * noise
    masks = masks.reshape(B, -1)
    target = target.reshape(B, -1)
    s = scores.reshape(B, -1)
    num_pixels = masks.sum()
    loss = 1 / 2. * (((masks * (s - target)) ** 2).sum(dim=-1) * masks.shape[-1] / num_pixels) \
        * used_sigmas.squeeze() ** anneal_power
    return loss.mean(dim=0)


def dsm_loss_and_grads(P, X, noise, masks, labels, anneal_power=2.0):
    """(loss, scores, {key: d loss/d param}) by autograd through scorenet_forward (the
    reference's loss.backward(), runners/ncsn_runner_kitti_simultaneous.py:230)."""
    Q = {k: (v.clone().requires_grad_(k != "sigmas")) for k, v in P.items()}
    used = Q["sigmas"].detach()[labels].view(X.shape[0], 1, 1, 1)
    scores = scorenet_forward(Q, X, labels)
    loss = dsm_loss(scores, used, noise, masks, anneal_power)
    loss.backward()
    grads = {k: v.grad for k, v in Q.items() if k != "sigmas"}
    return loss.detach(), scores.detach(), grads
