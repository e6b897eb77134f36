"""CPU emulation: does a Winograd F(2x2,3x3) conv with the fp32x3 (bf16 hi/lo, 3-pass) products
keep the score net within the parity tolerance (1e-4 of max|out|)?

Runs the oracle network (oracle/scorenet_ref.py) with its circular 3x3 convs replaced by
  direct: the fp32x3 direct conv the HIP kernel runs today (split the conv operands, 3 passes)
  wino:   F(2x2,3x3) Winograd on the d x d polyphase sub-grids: V = B^T d B and U = G g G^T in
          fp32, split to bf16 hi/lo, M = sum_c Uh*Vh + Uh*Vl + Ul*Vh (fp32 sums), Y = A^T M A
and compares each with a float64 run of the same network.  Test infrastructure only.
"""
import sys
import os

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd"))
from oracle import scorenet_ref as R  # noqa: E402
from oracle import golden_inputs as GI  # noqa: E402
from sdp.weights import synthetic_state_dict  # noqa: E402

_orig = R.conv2d


def split(t):
    hi = t.to(torch.bfloat16).to(torch.float32)
    lo = (t - hi).to(torch.bfloat16).to(torch.float32)
    return hi, lo


def direct3(x, w, b=None, dilation=1, circular=True, pad=None):
    if x.dtype == torch.float64:
        return _orig(x, w, b, dilation, circular, pad)
    xh, xl = split(x)
    wh, wl = split(w)
    o = _orig(xh, wh, None, dilation, circular, pad) + _orig(xh, wl, None, dilation, circular, pad) \
        + _orig(xl, wh, None, dilation, circular, pad)
    return o if b is None else o + b.view(1, -1, 1, 1)


BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float32)
G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float32)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float32)


def wino_subgrid(xp, w, mode):
    """xp: [B,C,h+2,w+2] padded sub-grid, w: [O,C,3,3] -> [B,O,h,w] (h, w even)."""
    B, C, Hp, Wp = xp.shape
    h, wd = Hp - 2, Wp - 2
    th, tw = h // 2, wd // 2
    # d[b,c,i,j,4,4]
    d = xp.unfold(2, 4, 2).unfold(3, 4, 2)           # [B,C,th,tw,4,4]
    V = torch.einsum("pa,bcijak,qk->bcijpq", BT, d, BT)   # B^T d B
    U = torch.einsum("pa,ocak,qk->ocpq", G, w, G)         # G g G^T
    V = V.reshape(B, C, th * tw, 16)
    U = U.reshape(w.shape[0], C, 16)
    if mode == "f64":
        M = torch.einsum("ocp,bctp->botp", U, V)
    else:
        Vh, Vl = split(V)
        Uh, Ul = split(U)
        M = (torch.einsum("ocp,bctp->botp", Uh, Vh) + torch.einsum("ocp,bctp->botp", Uh, Vl)
             + torch.einsum("ocp,bctp->botp", Ul, Vh))
    M = M.reshape(B, -1, th, tw, 4, 4)
    Y = torch.einsum("ra,boijak,sk->boijrs", AT.to(M.dtype), M, AT.to(M.dtype))   # [B,O,th,tw,2,2]
    return Y.permute(0, 1, 2, 4, 3, 5).reshape(B, -1, h, wd)


def wino3(x, w, b=None, dilation=1, circular=True, pad=None):
    k = w.shape[-1]
    if k != 3 or x.dtype == torch.float64 or not circular:
        return direct3(x, w, b, dilation, circular, pad)
    d = dilation
    B, C, H, W = x.shape
    out = torch.empty(B, w.shape[0], H, W)
    for a in range(d):
        for c in range(d):
            sub = x[:, :, a::d, c::d]
            xp = F.pad(sub, (1, 1, 1, 1), mode="circular")
            out[:, :, a::d, c::d] = wino_subgrid(xp, w, "x3")
    return out if b is None else out + b.view(1, -1, 1, 1)


def wino1d_subgrid(xp, w):
    """F(2,3) along W, direct along H: xp [B,C,h+2,w+2] -> [B,O,h,w]."""
    B, C, Hp, Wp = xp.shape
    h, wd = Hp - 2, Wp - 2
    d = xp.unfold(3, 4, 2)                               # [B,C,h+2,wd/2,4]
    V = torch.einsum("pa,bcrqa->bcrqp", BT, d)           # [B,C,h+2,pairs,4]
    U = torch.einsum("pa,oc ka->ockp".replace(" ", ""), G, w)   # [O,C,3(kh),4]
    Vh, Vl = split(V)
    Uh, Ul = split(U)
    M = 0
    for kh in range(3):
        for a_, b_ in ((Uh, Vh), (Uh, Vl), (Ul, Vh)):
            M = M + torch.einsum("ocp,bcrqp->borqp", a_[:, :, kh], b_[:, :, kh:kh + h])
    Y = torch.einsum("sa,borqa->borqs", AT, M)           # [B,O,h,pairs,2]
    return Y.reshape(B, -1, h, wd)


def wino1d(x, w, b=None, dilation=1, circular=True, pad=None):
    k = w.shape[-1]
    if k != 3 or x.dtype == torch.float64 or not circular:
        return direct3(x, w, b, dilation, circular, pad)
    d = dilation
    B, C, H, W = x.shape
    out = torch.empty(B, w.shape[0], H, W)
    for a in range(d):
        for c in range(d):
            xp = F.pad(x[:, :, a::d, c::d], (1, 1, 1, 1), mode="circular")
            out[:, :, a::d, c::d] = wino1d_subgrid(xp, w)
    return out if b is None else out + b.view(1, -1, 1, 1)


def run(conv, P, x, y):
    R.conv2d = conv
    try:
        with torch.no_grad():
            return R.scorenet_forward(P, x, y)
    finally:
        R.conv2d = _orig


def main():
    torch.set_num_threads(8)
    H, W, B = 64, int(sys.argv[1]) if len(sys.argv) > 1 else 256, 2
    sd = synthetic_state_dict(128)
    P = R.to_torch_params(sd)
    P64 = {k: v.double() for k, v in P.items()}
    x = torch.from_numpy(GI.scorenet_input(f"ngf128_b2_64x{W}", B, H, W))
    y = torch.tensor([0, 231]) if B == 2 else torch.tensor([0])
    ref64 = run(_orig, P64, x.double(), y).numpy()
    f32 = run(_orig, P, x, y).numpy()
    d3 = run(direct3, P, x, y).numpy()
    w3 = run(wino3, P, x, y).numpy()
    w1 = run(wino1d, P, x, y).numpy()
    for name, o in (("fp32 direct", f32), ("fp32x3 direct", d3), ("fp32x3 winograd", w3), ("fp32x3 wino 1d", w1)):
        err = max(np.abs(o[b] - ref64[b]).max() / np.abs(ref64[b]).max() for b in range(B))
        print(f"{name:18s} max err / max|ref| = {err:.3e}")


if __name__ == "__main__":
    main()
