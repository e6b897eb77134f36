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


def _train_cfg(tmp_path, W=256, B=2):
    with open(os.path.join(CFG_DIR, "HDVMine_Densification.yml")) as f:
        c = yaml.safe_load(f)
    c["data"]["image_width"] = W
    c["training"].update(batch_size=B)
    cfg = tmp_path / "train.yml"
    cfg.write_text(yaml.safe_dump(c))
    return cfg


@pytest.mark.gpu
def test_main_train_writes_and_reloads_checkpoints(tmp_path):
    """main.py without --sample runs the kitti runner's train() (kitti:83-348): curriculum,
    snapshot_freq list-format checkpoints, then --resume_training reloads one (kitti:115-128)."""
    import torch
    from sdp.scorenet import ScoreNet
    cfg = _train_cfg(tmp_path)
    exp = tmp_path / "exp"
    assert sdp_main.main(["--config", str(cfg), "--ni", "--exp", str(exp), "--verbose", "warning", "--precision",
                          "fp32x3", "--n_iters", "5", "--snapshot_freq", "2", "--max_epochs", "10"]) == 0
    log = exp / "logs" / "HDVMine"
    names = sorted(p.name for p in log.iterdir())
    assert "checkpoint.pth" in names and "checkpoint_2.pth" in names and "config.yml" in names, names
    states = torch.load(log / "checkpoint.pth", map_location="cpu", weights_only=True)
    assert len(states) == 5 and isinstance(states[2], int) and isinstance(states[3], int)
    assert all(k.startswith("module.") for k in states[0])
    assert set(states[4]) == {k[7:] for k in states[0] if k != "module.sigmas"}
    assert states[1]["param_groups"][0]["lr"] == 1e-4 and len(states[1]["state"]) == len(states[4])
    # the sampler's loader reads it back (EMA shadow applied) and runs a finite forward
    net = ScoreNet(H=64, W=256).load_checkpoint(str(log / "checkpoint.pth"))
    x = torch.rand(1, 2, 64, 256, device="cuda")
    assert torch.isfinite(net(x, torch.tensor([3], device="cuda"))).all()
    # resume: shape-filtered load of that checkpoint, training continues
    assert sdp_main.main(["--config", str(cfg), "--ni", "--exp", str(exp), "--verbose", "warning", "--precision",
                          "fp32x3", "--n_iters", "2", "--resume_training", "--ckpt", str(log / "checkpoint.pth")]) == 0


@pytest.mark.gpu
def test_train_loop_lowers_the_loss_and_follows_the_curriculum(tmp_path):
    """The runner's loop on the procedural scene: the timestep curriculum grows every 20 true
    steps, and the DSM loss at timestep 0 drops over the run."""
    import argparse
    from sdp.runner import Runner
    with open(_train_cfg(tmp_path)) as f:
        c = sdp_main.dict2namespace(yaml.safe_load(f))
    import torch
    c.device = torch.device("cuda")
    c.training.n_iters = 30
    c.training.snapshot_freq = 10 ** 9
    args = argparse.Namespace(seed=1234, precision="fp32x3", num_batches=1, max_epochs=30, kitti_root=None,
                              log_path=str(tmp_path / "log"), resume_training=False, ckpt=None)
    r = Runner(args, c)
    r.train()
    L = r.losses
    assert len(L) > 30 and all(np.isfinite(L))            # the curriculum added timesteps past step 20
    assert np.mean(L[-3:]) < np.mean(L[:3])
