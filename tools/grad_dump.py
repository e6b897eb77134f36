"""Dump every parameter gradient of one bf16-tape DSM forward + backward at 64x1024, B=8 (the bench's training
config, fixed inputs) to compare two libsdp builds bit for bit: SDP_LIB=... python tools/grad_dump.py OUT.npz"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd")]
from sdp.scorenet import ScoreNet  # noqa: E402
from sdp.training import Trainer, anneal_dsm_score_estimation_with_mask  # noqa: E402

dev = "cuda:0"
H, W, B = 64, 1024, 8
tr = Trainer(ScoreNet(H=H, W=W, precision="bf16").load_synthetic(), tape_bf16=True)
g = torch.Generator().manual_seed(7)
X = torch.rand(B, 2, H, W, generator=g)
sig = tr.net.sigmas if hasattr(tr.net, "sigmas") else None
lab = torch.randint(0, 200, (B,), generator=g)
from sdp.weights import get_sigmas_np  # noqa: E402
sigmas = torch.from_numpy(get_sigmas_np().astype(np.float32))
used = sigmas[lab].view(B, 1, 1, 1)
noise = torch.randn(B, 2, H, W, generator=g) * used
mask = (torch.rand(B, 2, H, W, generator=g) > 0.3).float()
loss, _ = anneal_dsm_score_estimation_with_mask(tr, (X + noise).to(dev), used.to(dev), noise.to(dev), mask.to(dev), None,
                                                sigmas.to(dev), lab.to(dev))
tr.backward()
torch.cuda.synchronize()
np.savez(sys.argv[1], loss=np.float64(loss.item()), **{k: v.cpu().numpy() for k, v in tr.named_grads()})
print("dumped", sys.argv[1])
