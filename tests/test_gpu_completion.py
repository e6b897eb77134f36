"""§8(f)-3 scene completion on the GPU: the dataset item (host grid subsampling + origin, GPU
projection + SDP_VIEW_COMPLETION post-processing) against oracle/completion_ref.py (projection pinned
to the reference, subsampling = the reference's compiled C++), and main.py --sample with the
HDVMineCompletion config end to end (runners/ncsn_runner_Completion.py:468-940)."""
import os

import numpy as np
import pytest
import torch
import yaml

import main as sdp_main
from oracle import completion_ref as CR
from ssc_tree import write_ssc_tree

pytestmark = pytest.mark.gpu
CFG_DIR = os.path.join(os.path.dirname(sdp_main.__file__), "configs")


def _cfg(W=1024):
    with open(os.path.join(CFG_DIR, "HDVMineCompletion.yml")) as f:
        c = yaml.safe_load(f)
    c["data"]["image_width"] = W
    return c


@pytest.mark.parametrize("nib", [0, 1, 2, 3, 4])
def test_completion_item_matches_oracle(tmp_path, nib):
    from sdp.completion import kitti360_im_SceneCompletion
    names = write_ssc_tree(str(tmp_path), n_scans=1)
    cfg = sdp_main.dict2namespace(_cfg())
    ds = kitti360_im_SceneCompletion(None, cfg, split="test", root=str(tmp_path), device="cuda")
    real, notmask, notsky, index, name, origin = ds[nib]
    d = tmp_path / "data_3d_raw" / "data_3d_ssc_test"
    r2, m2, s2, i2, o2 = CR.item(str(d / "velodyne_points" / "data" / names[0]), str(d / "Final" / names[0]), nib,
                                 cfg.data.modifications)
    assert name == names[0][:-4]
    np.testing.assert_allclose(origin, o2, atol=1e-9)
    # float64 projection on device vs numpy: a point on a bin edge may move (<= 1e-4 of the pixels)
    assert np.mean(notmask != m2) <= 1e-4 and np.mean(notsky != s2) <= 1e-4
    assert np.mean(np.abs(real - r2) > 1e-12) <= 1e-4
    assert np.mean(index != i2) <= 1e-4
    np.testing.assert_array_equal(real[1], real[0])          # (real, real): the reference's second channel
    assert not notmask[1].any()                               # (mask, ones)


def test_main_sample_scene_completion(tmp_path):
    root = tmp_path / "KITTI-360"
    write_ssc_tree(str(root), n_scans=1)
    c = _cfg(W=256)
    c["sampling"]["n_steps_each"] = 1
    c["model"]["num_classes"] = 4                  # 4 sigma levels keep the run short; the merge runs from level 2
    cfg = tmp_path / "completion.yml"
    cfg.write_text(yaml.safe_dump(c))
    assert sdp_main.main(["--config", str(cfg), "--sample", "--ni", "--exp", str(tmp_path / "exp"), "--verbose",
                          "warning", "--kitti_root", str(root)]) == 0
    out = tmp_path / "exp" / "image_samples" / "images"
    m = np.load(out / "1_000000_Masked_completion_897.pth.npy")
    assert m.shape == (10, 3, 64, 256) and np.isfinite(m).all() and 0 <= m.min() and m.max() <= 1
    sh = np.load(out / "1_0_Shared_completion_initial897.pth.npy")
    assert sh.shape == m.shape and (sh > 0).mean() > 0.05        # the last merge produced shared points
    inp = np.load(out / "0_000000_Input_completion_897.pth.npy")
    known = inp > 0
    assert np.abs(m[known] - inp[known]).max() < 1e-5            # final consistency wrote the known pixels back
    assert np.load(out / "0_000000_ORIGINS_897.pth.npy").shape == (5, 1, 3)
