"""Dump consistency-merge outputs (corrected x and new images) of the bench's geometry for many random states, to
compare two libsdp builds bit for bit: SDP_LIB=... python tools/merge_dump.py OUT.npz
kitti 32-view megabatch (config 4, 4 output views) and AllForOne 9 views (config 3); x in [-1, 1] (negative depth
codes take the flip/roll branch); sigmas on both sides of 1 (the sigma-mod path)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd")]
from bench import CIRCLE9  # noqa: E402
from sdp.merge import Merger, allforone_origins  # noqa: E402
from sdp.synthetic import exist_mask, scene_views  # noqa: E402

dev = "cuda:0"
H, W = 64, 1024
out = {}
for tag, n_src, o_begin, n_out in (("k32", 32, 8, 4), ("a9", 9, 0, 9)):
    sc = scene_views(n_src, H, W)
    if tag == "k32":
        m = Merger(n_src, n_src, H, W, dev, torch.from_numpy(exist_mask(H, W)), torch.from_numpy(sc["sky"]),
                   torch.from_numpy(sc["mask"]), toWorld=torch.from_numpy(sc["toWorld"]),
                   fromWorld=torch.from_numpy(sc["fromWorld"]), o_begin=o_begin, n_out=n_out)
        setting = 5
    else:
        m = Merger(n_src, n_src, H, W, dev, torch.from_numpy(exist_mask(H, W)), torch.from_numpy(sc["sky"]),
                   torch.from_numpy(sc["mask"]), origins=allforone_origins(CIRCLE9[:n_src]), o_begin=o_begin, n_out=n_out)
        setting = 7
    for k, sigma in enumerate((0.01, 0.3, 1.0, 2.5, 40.0)):
        g = torch.Generator(device=dev).manual_seed(100 + k)
        x = torch.rand(n_src, 2, H, W, device=dev, generator=g) * 2 - 1
        if k == 4:
            x[:, 0] *= 0.2
        absmax = torch.zeros(1, dtype=torch.int32, device=dev)   # max 0: the correction runs
        new = torch.zeros(n_out, 2, H, W, device=dev)
        m(x, sigma, setting, 10.0, 0.01, absmax, new_images=new)
        torch.cuda.synchronize()
        out[f"{tag}_{k}_x"] = x[o_begin:o_begin + n_out].cpu().numpy()
        out[f"{tag}_{k}_new"] = new.cpu().numpy()
np.savez(sys.argv[1], **out)
print("dumped", len(out), "arrays to", sys.argv[1])
