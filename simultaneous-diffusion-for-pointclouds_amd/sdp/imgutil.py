"""PNG image grids of the runners: ``make_grid`` / ``save_image`` as the
reference imports them from torchvision.utils (runners/ncsn_runner_kitti_simultaneous.py:13,
658-691, 859-870).  torchvision is not installed in this image, so this restates its published
algorithm (torchvision.utils, 0.x series, defaults padding=2, pad_value=0, normalize=False):
the images are tiled ``nrow`` per row, each framed by ``padding`` pixels of ``pad_value``; a
batch of one returns the image itself; ``save_image`` writes grid * 255 + 0.5 clamped to
[0, 255] as 8-bit RGB through PIL.  Host-side output formatting, no GPU work.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def make_grid(tensor: torch.Tensor, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> torch.Tensor:
    if tensor.dim() == 2:
        tensor = tensor.unsqueeze(0)
    if tensor.dim() == 3:
        tensor = tensor.unsqueeze(0) if tensor.size(0) in (1, 3) else tensor.unsqueeze(1)
    if tensor.size(1) == 1:
        tensor = torch.cat((tensor, tensor, tensor), 1)
    if tensor.size(0) == 1:
        return tensor.squeeze(0)
    nmaps = tensor.size(0)
    xmaps = min(nrow, nmaps)
    ymaps = int(math.ceil(float(nmaps) / xmaps))
    height, width = int(tensor.size(2) + padding), int(tensor.size(3) + padding)
    grid = tensor.new_full((tensor.size(1), height * ymaps + padding, width * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= nmaps:
                break
            grid[:, y * height + padding:(y + 1) * height, x * width + padding:(x + 1) * width] = tensor[k]
            k += 1
    return grid


def save_image(tensor: torch.Tensor, fp, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> None:
    from PIL import Image
    grid = make_grid(tensor.detach().cpu(), nrow=nrow, padding=padding, pad_value=pad_value)
    nd = grid.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    Image.fromarray(np.ascontiguousarray(nd)).save(fp)
