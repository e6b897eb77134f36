"""§8(f)-3 scene completion, CPU side: the view-origin geometry (sdp/completion.py, exact rational
circle cuts) against the oracle's independent float formulation, and the Completion runner's files
(runners/ncsn_runner_Completion.py:468-940) with the sampler stubbed (it runs on the GPU)."""
import os

import numpy as np
import pytest
import torch
import yaml

import main as sdp_main
from oracle import completion_ref as CR
from sdp import completion as CP
from sdp import grid_subsampling as GS
from sdp import runner as R
from ssc_tree import write_ssc_tree

CFG_DIR = os.path.join(os.path.dirname(sdp_main.__file__), "configs")


@pytest.mark.parametrize("R_,x,y", [(35, 6000.0, 1500.5), (40, -120.0, 7999.1), (50, 3.0, -9999.9), (30, 5000, 0.0),
                                    (30, 0.0, 6000.0)])
def test_circle_cut_matches_the_float_formulation(R_, x, y):
    a = CP.circle_line_first(R_, x, y)
    b = CR.circle_cut(R_, x, y)
    np.testing.assert_allclose(a, b, atol=1e-9)
    assert R_ * np.cos(np.pi / 64) - 1e-9 <= np.hypot(*a) <= R_ + 1e-9     # on the 64-gon
    assert a[0] <= 0 or (a[0] == 0 and a[1] <= 0) or np.allclose(a, b)    # the smaller-x crossing


def test_view_origins_of_a_scan(tmp_path):
    write_ssc_tree(str(tmp_path), n_scans=1)
    scan = np.load(tmp_path / "data_3d_raw/data_3d_ssc_test/velodyne_points/data/000000.npy")
    scan = scan - np.median(scan, axis=0) + CP.ROUGH_MEDIAN
    sub = GS.grid_sub_sampling(scan.astype(np.float32))
    sub = np.concatenate((sub, np.zeros((len(sub), 1), np.float32)), 1)
    mods = np.array([[0, 0, 0], [5, -5, 0], [-5, -5, 0], [0, 5, 0], [-10, 10, 0]])
    for nib in range(5):
        o = CP.view_origin(sub, nib, mods)
        np.testing.assert_allclose(o, CR.view_origin(sub, nib, mods), atol=1e-9)
        if nib < 4:
            assert abs(np.hypot(o[0], o[1]) - [35, 40, 50, 30][nib]) < 0.2
    assert (CP.view_origin(sub, 4, mods) == 0).all()


def test_completion_runner_files(tmp_path, monkeypatch):
    import argparse
    log = []

    class _Net:
        def __init__(self, **kw):
            pass

        def load_synthetic(self):
            return self

        def load_state_dict(self, sd, ema_shadow=None):
            return self

    def a41(init, ref, mask, sky, idx, start, setting, score, sigmas, mods, aB, *a, **kw):
        log.append((init.shape[0], start, setting, tuple(mods.shape), kw["correlation_coefficient"], kw["grad_ref"]))
        return [init + 0.5, init * 2], [], []
    monkeypatch.setattr(R, "ScoreNet", _Net)
    monkeypatch.setattr(R, "anneal_Langevin_dynamics_inpainting_simultaneous_basic", a41)
    with open(os.path.join(CFG_DIR, "HDVMineCompletion.yml")) as f:
        c = yaml.safe_load(f)
    c["data"]["image_width"] = 128
    cfg = sdp_main.dict2namespace(c)
    cfg.device = torch.device("cpu")
    args = argparse.Namespace(image_folder=str(tmp_path), seed=1234, ckpt="/nonexistent.pth", precision="fp32x3",
                              num_batches=1)
    R.Runner(args, cfg).sample()
    assert log == [(5, 2, 7, (5, 3), 0.01, 1)]      # doThis 0 samples nothing; doThis 1 the AllForOne sampler
    files = set(os.listdir(tmp_path))
    for f in ["0_000000_Input_completion_897.pth.npy", "0_000000_SKY_897.pth.npy", "0_000000_ORIGINS_897.pth.npy",
              "1_000000_TimeTaken.npy", "1_000000_Masked_completion_897.pth.npy",
              "1_0_Shared_completion_initial897.pth.npy", "1_000000_Masked_image_grid_897.png"]:
        assert f in files, (f, sorted(files))
    assert np.load(tmp_path / "1_000000_TimeTaken.npy") > 999999            # the reference's initial value
    assert np.load(tmp_path / "1_000000_Masked_completion_897.pth.npy").shape == (10, 3, 64, 128)
    assert np.load(tmp_path / "0_000000_ORIGINS_897.pth.npy").shape == (5, 1, 3)
