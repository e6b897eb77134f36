"""The drop-in runner's sweep and output files (runners/ncsn_runner_kitti_simultaneous.py:461-893,
runners/ncsn_runner_AllForOne.py:468-990), with the samplers stubbed (they are tested on the GPU)."""
import os

import numpy as np
import pytest
import torch
import yaml

import main as sdp_main
from sdp import runner as R

CFG_DIR = os.path.join(os.path.dirname(sdp_main.__file__), "configs")


class _FakeNet:
    def __init__(self, **kw):
        self.kw = kw

    def load_synthetic(self):
        return self

    def load_state_dict(self, sd, ema_shadow=None):
        return self


def _config(name, B=14, W=128):
    with open(os.path.join(CFG_DIR, name)) as f:
        c = yaml.safe_load(f)
    c["sampling"]["batch_size"] = B
    c["data"]["image_width"] = W
    ns = sdp_main.dict2namespace(c)
    ns.device = torch.device("cpu")
    return ns


def _args(folder):
    import argparse
    return argparse.Namespace(image_folder=str(folder), seed=1234, ckpt="/nonexistent.pth", precision="fp32x3",
                              num_batches=1)


@pytest.fixture
def calls(monkeypatch):
    log = []

    def base(init, ref, mask, score, sigmas, n, lr, denoise=True, grad_ref=1, sampling_step=4, **kw):
        log.append(("baseline", init.shape[0], None))
        return [init + 0.25, init + 0.5, init * 2], []

    def kitti(init, ref, mask, sky, idx, start, setting, allowance, score, sigmas, fromW, toW, aB, *a, **kw):
        assert fromW.shape == (init.shape[0], 4, 4) and sky.shape[0] == init.shape[0]
        log.append(("kitti", init.shape[0], aB, setting, start, kw["correlation_coefficient"]))
        return [init + 0.5, init * 2], [], []

    def a41(init, ref, mask, sky, idx, start, setting, score, sigmas, mods, aB, *a, **kw):
        assert tuple(mods.shape) == (7, 3)
        log.append(("allforone", init.shape[0], aB, setting))
        return [init + 0.5, init * 2], [], []

    monkeypatch.setattr(R, "ScoreNet", _FakeNet)
    monkeypatch.setattr(R, "anneal_Langevin_dynamics_inpainting", base)
    monkeypatch.setattr(R, "anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti", kitti)
    monkeypatch.setattr(R, "anneal_Langevin_dynamics_inpainting_simultaneous_basic", a41)
    return log


def test_line_sweep_and_files(tmp_path, calls):
    c = _config("HDVMine_Line.yml")
    R.Runner(_args(tmp_path), c).sample()
    # doThis 0..4: first doThis+2 views of each of the 2 megabatches; 5: all; 6: baseline on all 14
    assert [x[1] for x in calls] == [4, 6, 8, 10, 12, 14, 14]
    assert calls[-1][0] == "baseline" and all(x[0] == "kitti" for x in calls[:-1])
    assert calls[0][2:] == (2, 5, 2, 0.01)
    assert calls[5][2] == 7
    files = set(os.listdir(tmp_path))
    sn = "0_7_"
    for f in ["toWorld_" + sn + ".npy", "fromWorld_" + sn + ".npy", f"0_{sn}_Input_completion_897.pth.npy",
              f"0_{sn}_GT_completion_897.pth.npy", f"0_{sn}_SKY_897.pth.npy"]:
        assert f in files, f
    for d, n in enumerate([4, 6, 8, 10, 12, 14, 14]):
        m = np.load(tmp_path / f"{d}_{sn}_Masked_completion_897.pth.npy")
        assert m.shape == (2 * n, 3, 64, 128) and m.min() >= 0 and m.max() <= 1
        assert (m[:, 0] == m[:, 1]).all() and (m[:, 0] == m[:, 2]).all()
        assert np.load(tmp_path / f"{d}_{sn}_TimeTaken.npy").shape == ()
    assert np.load(tmp_path / ("toWorld_" + sn + ".npy")).shape == (14, 4, 4)
    gt = np.load(tmp_path / f"0_{sn}_GT_completion_897.pth.npy")
    inp = np.load(tmp_path / f"0_{sn}_Input_completion_897.pth.npy")
    assert gt.shape == inp.shape == (28, 3, 64, 128) and (gt >= inp).all() and (gt != inp).any()


def test_circle_sweep(tmp_path, calls):
    R.Runner(_args(tmp_path), _config("HDVMine_Circle.yml")).sample()
    # doThis 0..4 -> doThis+2 views per megabatch; 5 -> all; 6 -> baseline on the first view of each
    assert [x[1] for x in calls] == [4, 6, 8, 10, 12, 14, 2]
    assert calls[-1][0] == "baseline" and calls[0][2:] == (2, 7)
    sh = np.load(tmp_path / "6_0_7__Shared_completion_initial897.pth.npy")
    assert sh.shape == (4, 3, 64, 128)
    gt = np.load(tmp_path / "0_0_7__GT_completion_897.pth.npy")
    np.testing.assert_array_equal(gt, np.load(tmp_path / "0_0_7__Input_completion_897.pth.npy"))


def test_densification_sweep(tmp_path, calls):
    R.Runner(_args(tmp_path), _config("HDVMine_Densification.yml")).sample()
    # endPoint 2, toAdd aB-2: doThis 0 -> all views jointly, doThis 1 -> baseline
    assert [(x[0], x[1]) for x in calls] == [("allforone", 14), ("baseline", 2)]


def test_first_views_matches_reference_slice():
    t = torch.arange(14 * 2 * 3).reshape(14, 2, 3, 1)
    got = R._first_views(t, 2, 7, 3)
    assert got.shape == (6, 2, 3, 1)
    np.testing.assert_array_equal(got[3].numpy(), t[7].numpy())


def test_cli_refuses_without_gpu(tmp_path):
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="HIP device"):
        sdp_main.main(["--config", "HDVMine_Line.yml", "--sample", "--ni", "--exp", str(tmp_path)])
