"""Host side of the KITTI-360 view renderer (sdp/kitti360.py) against the oracle restatement
(oracle/kitti_ref.py): pose chain, dataset length, the sampler's batch order and the
reference's error behaviour -- no device work."""
import numpy as np
import pytest

from kitti_tree import config, write_tree
from oracle import kitti_ref
from sdp import kitti360


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("kitti360"))
    write_tree(root, n_poses=12, n_points=2000)
    return root


def test_pose_chain_matches_oracle(tree):
    f0, t0 = kitti360.pose_chain(tree)
    f1, t1 = kitti_ref.poses(tree)
    assert np.array_equal(f0, f1)
    assert list(t0) == list(t1)
    for k in t0:
        assert np.array_equal(t0[k], t1[k])


def test_dataset_length_and_split(tree):
    ds = kitti360.KITTI360_im_8batch("unused", config(4), split="test", root=tree)
    assert len(ds) == 12 * 4
    assert len(ds.full_list) == 12
    tr = kitti360.KITTI360_im_8batch("unused", config(4), split="train", root=tree)
    assert tr.full_list == []          # the 0000 drive is the test split (8Batch:27-30)


def test_last_pose_goal_raises_like_the_reference(tree):
    ds = kitti360.KITTI360_im_8batch("unused", config(4), split="test", root=tree)
    with pytest.raises(IndexError):     # goal pose clamped to the last pose, then frames[pd + 1]
        ds.render(len(ds) - 1)


def test_single_channel_is_rejected_like_the_reference(tree):
    c = config(4)
    c.data.channels = 1
    ds = kitti360.KITTI360_im_AllForOne("unused", c, split="test", root=tree)
    with pytest.raises(NameError):
        ds.render(0)


def test_sampler_batches():
    np.random.seed(3)
    order = list(kitti360.MySampler(5, 4, random=False))
    np.random.seed(3)
    opts = np.arange(5)
    np.random.shuffle(opts)
    want = [int(n) * 4 + i for n in opts for i in range(4)]
    assert order == want
