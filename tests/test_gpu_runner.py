"""main.py --sample end to end on the GPU (real libsdp samplers), on a reduced Line config."""
import os

import numpy as np
import pytest
import yaml

import main as sdp_main

CFG_DIR = os.path.join(os.path.dirname(sdp_main.__file__), "configs")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["HDVMine_Line.yml", "HDVMine_Circle.yml"])
def test_main_sample_small(tmp_path, name):
    with open(os.path.join(CFG_DIR, name)) as f:
        c = yaml.safe_load(f)
    c["sampling"].update(batch_size=6, actualBatchSize=3, n_steps_each=1)
    c["data"].update(image_width=256, modifications=c["data"]["modifications"][:3])
    cfg = tmp_path / "small.yml"
    cfg.write_text(yaml.safe_dump(c))
    assert sdp_main.main(["--config", str(cfg), "--sample", "--ni", "--exp", str(tmp_path / "exp"),
                          "--verbose", "warning"]) == 0
    out = tmp_path / "exp" / "image_samples" / "images"
    kitti = "Line" in name
    views = [4, 6, 6] if kitti else [4, 6, 2]
    for d, n in enumerate(views):
        m = np.load(out / f"{d}_0_3__Masked_completion_897.pth.npy")
        assert m.shape == (2 * n, 3, 64, 256)
        assert np.isfinite(m).all() and 0 <= m.min() and m.max() <= 1
    pngs = sorted(p.name for p in out.glob("*_image_grid_*.png"))
    assert "0_0_Input_image_grid_897.png" in pngs or "0_0_3__Input_image_grid_897.png" in pngs, pngs
    assert len([p for p in pngs if "Masked_image_grid" in p]) == 3, pngs
    # the known pixels were written back by the final consistency step
    inp = np.load(out / "0_0_3__Input_completion_897.pth.npy")
    last = np.load(out / f"1_0_3__Masked_completion_897.pth.npy")
    known = inp > 0                      # doThis=1 samples all 6 views, in input order
    assert last.shape == inp.shape and np.abs(last[known] - inp[known]).max() < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["HDVMine_Line.yml", "HDVMine_Circle.yml"])
def test_main_sample_from_kitti_tree(tmp_path, name):
    """--kitti_root: the batch comes from the GPU-rendered KITTI-360 dataset (sdp.kitti360)."""
    from kitti_tree import write_tree
    root = tmp_path / "KITTI-360"
    write_tree(str(root), n_poses=40, n_points=20000)
    with open(os.path.join(CFG_DIR, name)) as f:
        c = yaml.safe_load(f)
    c["sampling"].update(batch_size=3, actualBatchSize=3, n_steps_each=1)
    c["data"].update(image_width=256, modifications=c["data"]["modifications"][:3])
    cfg = tmp_path / "small.yml"
    cfg.write_text(yaml.safe_dump(c))
    assert sdp_main.main(["--config", str(cfg), "--sample", "--ni", "--exp", str(tmp_path / "exp"),
                          "--verbose", "warning", "--kitti_root", str(root)]) == 0
    out = tmp_path / "exp" / "image_samples" / "images"
    files = sorted(p.name for p in out.iterdir())
    masked = [f for f in files if f.startswith("0_") and "Masked_completion" in f]
    assert masked, files
    m = np.load(out / masked[0])
    assert m.shape[1:] == (3, 64, 256) and np.isfinite(m).all() and 0 <= m.min() and m.max() <= 1
    inp = np.load(out / masked[0].replace("Masked", "Input"))
    assert inp.max() > 0           # real depth codes reached the sampler
