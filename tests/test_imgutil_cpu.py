"""PNG grids (sdp/imgutil.py): the torchvision.utils make_grid / save_image layout the runners
write (kitti:658-691). torchvision is absent from this image, so the layout is checked against
its published rule directly (parity unpinned against torchvision itself)."""
import numpy as np
import torch
from PIL import Image

from sdp.imgutil import make_grid, save_image


def test_grid_layout_and_padding():
    x = torch.rand(5, 3, 4, 6)
    g = make_grid(x, 2)
    assert g.shape == (3, 3 * (4 + 2) + 2, 2 * (6 + 2) + 2)
    for k in range(5):
        y, c = divmod(k, 2)
        r0, c0 = y * 6 + 2, c * 8 + 2
        assert torch.equal(g[:, r0:r0 + 4, c0:c0 + 6], x[k])
    assert torch.equal(g[:, 12 + 2:, 8 + 2:], torch.zeros(3, 6, 8))   # the unused 6th cell
    assert torch.equal(g[:, :2], torch.zeros(3, 2, g.shape[2]))       # top padding


def test_single_image_and_gray_input():
    x = torch.rand(1, 1, 4, 6)
    g = make_grid(x, 3)
    assert g.shape == (3, 4, 6) and torch.equal(g[0], x[0, 0]) and torch.equal(g[2], x[0, 0])


def test_save_image_quantisation(tmp_path):
    x = torch.tensor([0.0, 0.2, 0.5, 1.0, 1.3, -0.1]).reshape(1, 1, 1, 6).repeat(2, 3, 1, 1)
    save_image(x, tmp_path / "g.png", nrow=1)
    a = np.asarray(Image.open(tmp_path / "g.png"))
    assert a.shape == (2 * 3 + 2, 6 + 4, 3) and a.dtype == np.uint8
    assert list(a[2, 2:8, 0]) == [0, 51, 128, 255, 255, 0]     # floor(x * 255 + 0.5), clamped
