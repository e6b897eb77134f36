"""Writes a small synthetic KITTI-360 tree (the directory layout the datasets read,
kitti360_im_8Batch.py:25,49-59,106-111) for the view-rendering tests: calibration files,
data_poses/<drive>/poses.txt with gaps between frame numbers, and one float32 [N][4]
velodyne .bin per pose (named by frame - 1, as the datasets look them up)."""
import os
from types import SimpleNamespace

import numpy as np

from oracle.golden_inputs import projection_cloud

DRIVE = "2013_05_28_drive_0000_sync"


def write_tree(root, n_poses=24, n_points=40000, seed=5):
    r = np.random.default_rng(seed)
    cal = os.path.join(root, "calibration")
    os.makedirs(cal, exist_ok=True)
    # camera -> velodyne: KITTI-like axis swap plus a small offset
    c2v = np.array([[0.0, -1.0, 0.0, 0.04], [0.0, 0.0, -1.0, -0.07], [1.0, 0.0, 0.0, -0.27]])
    c2v[:, :3] += r.normal(0, 1e-3, (3, 3))
    np.savetxt(os.path.join(cal, "calib_cam_to_velo.txt"), c2v.reshape(1, 12))
    c2p = np.stack([np.concatenate([np.eye(3) + r.normal(0, 1e-3, (3, 3)), r.normal(0, 0.5, (3, 1))], 1).ravel()
                    for _ in range(4)])      # image_00 .. image_03; the datasets take row 0
    np.savetxt(os.path.join(cal, "calib_cam_to_pose.txt"), c2p)
    frames = 1 + np.cumsum(r.integers(1, 4, n_poses))          # gaps of 1..3 frames
    rows = []
    for k, f in enumerate(frames):
        th = 0.04 * k + 0.3
        R = np.array([[np.cos(th), -np.sin(th), 0.0], [np.sin(th), np.cos(th), 0.0], [0.0, 0.0, 1.0]])
        t = np.array([1.7 * k + 100.0, -0.4 * k + 50.0, 0.02 * k + 110.0])
        rows.append(np.concatenate([[f], np.concatenate([R, t[:, None]], 1).ravel()]))
    pose_dir = os.path.join(root, "data_poses", DRIVE)
    os.makedirs(pose_dir, exist_ok=True)
    np.savetxt(os.path.join(pose_dir, "poses.txt"), np.array(rows), fmt="%.10g")
    data = os.path.join(root, "data_3d_raw", DRIVE, "velodyne_points", "data")
    os.makedirs(data, exist_ok=True)
    for f in frames:
        pts = projection_cloud(f"kitti_{int(f)}", n_points).astype(np.float32)
        pts.tofile(os.path.join(data, str(int(f) - 1).zfill(10) + ".bin"))
    return frames


def config(batch=4, random_roll=False, H=64, W=1024):
    mods = [[0, 0, 0], [5, -5, 0], [-5, -5, 0], [0, 5, 0], [-10, 10, 0], [10, 10, 0], [-10, 0, 0], [10, 0, 0]]
    return SimpleNamespace(data=SimpleNamespace(channels=2, random_roll=random_roll, modifications=mods[:max(batch, 1)],
                                                image_size=H, image_width=W),
                           sampling=SimpleNamespace(actualBatchSize=batch))
