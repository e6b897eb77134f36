"""ORACLE (test infrastructure only) -- numpy restatement of the KITTI-360 datasets'
``__getitem__``, the checker for sdp/kitti360.py (sdp_view_transform,
sdp_view_gather, sdp_view_finalize over sdp_range_project).  Only tests/ may import it.

Follows, statement by statement (paths under /root/reference/LiDARGen/datasets):
  pose chain        kitti360_im_8Batch.py:49-68
  8batch item       kitti360_im_8Batch.py:94-304
  AllForOne item    kitti360_im_AllForOne.py:94-354
  densification     kitti360_im_simultenous_densification.py:94-339
with point_cloud_to_range_image = oracle.projection_ref (pinned to the reference's own
outputs by tests/golden/projection_*.npz).  Pinning: the dataset modules themselves cannot be
imported here (they import h5py, which this image lacks), so these item functions are a
restatement checked through their pinned projection; the pose algebra and post-processing
they add are plain numpy statements copied in meaning from the lines cited.
"""
from __future__ import annotations

import os

import numpy as np

from .projection_ref import point_cloud_to_range_image

MAX_RANGE = 2057.701
DRIVE = "2013_05_28_drive_0000_sync"


def read_bin(path):
    return np.fromfile(path, dtype=np.float32).reshape(-1, 4)


def poses(root):
    """kitti360_im_8Batch.py:49-68 -> (frames, Tr_pose_world)."""
    v2c = np.loadtxt(os.path.join(root, "calibration/calib_cam_to_velo.txt"))
    v2c = np.reshape(v2c, [3, 4])
    v2c = np.concatenate((v2c, np.array([0., 0., 0., 1.]).reshape(1, 4)))
    v2c = np.linalg.inv(v2c)
    c2p = np.loadtxt(os.path.join(root, "calibration/calib_cam_to_pose.txt"))[0]
    c2p = np.reshape(c2p, [3, 4])
    c2p = np.concatenate((c2p, np.array([0., 0., 0., 1.]).reshape(1, 4)))
    v2p = np.matmul(c2p, v2c)
    p = np.loadtxt(os.path.join(root, "data_poses", DRIVE, "poses.txt"))
    frames = p[:, 0] - 1
    mats = np.reshape(p[:, 1:], [-1, 3, 4])
    tr = {}
    for f, m in zip(frames, mats):
        m = np.concatenate((m, np.array([0., 0., 0., 1.]).reshape(1, 4)))
        tr[f] = np.matmul(m, v2p)
    return frames, tr


def _post(real, intensity, mask, sky, goal_depth, goal_intensity, H, W, roll, variant, number_in_batch):
    """The shared tail of the three items (8Batch:221-291 with the variants' differences)."""
    mask = np.where(real >= MAX_RANGE, 1, mask)
    real = np.where(real >= MAX_RANGE, 0, real) + 0.0001
    goal_depth = np.where(goal_depth >= MAX_RANGE, 0, goal_depth) + 0.0001
    real = np.log2(real + 1) / 6
    goal_depth = np.log2(goal_depth + 1) / 6
    real = np.clip(real, 0, 1)
    goal_depth = np.clip(goal_depth, 0, 1)
    if roll is not None:
        real = np.roll(real, roll, axis=1)
        mask = np.roll(mask, roll, axis=1)
        sky = np.roll(sky, roll, axis=1)
    mask = np.where(intensity >= 1, 1, mask)          # unrolled intensity (8Batch:272, AllForOne:276)
    real = real[None]
    mask = mask[None]
    goal_depth = goal_depth[None]
    goal_intensity = goal_intensity[None]
    if variant == 2 and number_in_batch == 0:         # densification:271-282
        m3 = np.zeros_like(real).astype(int)
        m3[:, :, :(W // 4)] = 1
        mask = np.logical_or(np.zeros_like(mask), m3)
    sky = sky.copy()
    sky[1:] = sky[:-1]
    sky[1:] = sky[:-1]
    sky[1:] = sky[:-1]
    sky = sky[None]
    intensity = np.where(intensity >= 1, 0, intensity) + 0.0001
    intensity = np.clip(intensity, 0, 1.0)
    goal_intensity = np.where(goal_intensity >= 1, 0, goal_intensity) + 0.0001
    goal_intensity = np.clip(goal_intensity, 0, 1.0)
    if roll is not None:
        intensity = np.roll(intensity, roll, axis=1)
    real = np.concatenate((real, intensity[None]), axis=0)
    goal_depth = np.concatenate((goal_depth, goal_intensity), axis=0)
    mask = np.concatenate((mask, mask), axis=0)
    return real, np.logical_not(mask), np.logical_not(sky), goal_depth


def item(root, variant, idx, batch_size, modifications, H=64, W=1024, random_roll=False, rng=None):
    """One __getitem__ (channels == 2) of variant 0 = 8batch, 1 = AllForOne, 2 = densification.
    ``rng``: a numpy RandomState whose randint(W) plays np.random.randint (drawn every item)."""
    frames, tr = poses(root)
    data_dir = os.path.join(root, "data_3d_raw", DRIVE, "velodyne_points/data")
    name = lambda f: os.path.join(data_dir, str(int(f)).zfill(10) + ".bin")
    nb = idx % batch_size
    pose_num = idx // batch_size
    scan_no = int(frames[pose_num])
    pts = read_bin(name(scan_no))
    to_world = tr[scan_no]
    to_og = np.linalg.inv(to_world)
    mods = np.array(modifications)
    if variant == 2:
        og = point_cloud_to_range_image(pts, mods[0], True, rowMax=H, colMax=W)
        index = og[5]
        index[:, :(W // 4)] = -2
        goal_pts = pts.copy()
        pts = pts[index[index >= 0].astype(int)]
        origin = mods[nb]
        ret_to, ret_from = to_world, to_og
    else:
        inten = pts[:, -1]
        pv = np.concatenate((np.transpose(pts[:, :-1]), np.expand_dims(np.ones_like(inten), 0)), 0)
        pv = np.matmul(to_world, pv)
        moved = (nb + 1) * 5 if variant == 0 else 2 * 5
        pd = pose_num + moved
        if pd >= len(frames):
            pd = len(frames) - 1
        to_world2 = tr[frames[pd]]
        stack = []
        for k in range(int(frames[pd + 1] - frames[pd])):
            if k > 0:
                continue
            stack.append(read_bin(name(frames[pd] + k)))
        goal_pts = np.concatenate(stack, 0)
        from_world = np.linalg.inv(to_world2)
        pv = np.matmul(from_world, pv)
        pts = np.transpose(np.concatenate((pv[:-1], np.expand_dims(inten, 0)), 0))
        origin = np.zeros(3) if variant == 0 else mods[nb]
        ret_to, ret_from = to_world2, from_world
    real, notmask, notsky, index, goal = render_arrays(pts, goal_pts, origin, H, W, variant, nb,
                                                       roll_draw=lambda: (rng or np.random).randint(W),
                                                       random_roll=random_roll)
    return real, notmask, notsky, index[None], ret_to[None], ret_from[None], goal, to_og, scan_no


def render_arrays(pts, goal_pts, origin, H, W, variant=0, nb=0, roll_draw=None, random_roll=False):
    """The two projections and the post-processing of one item (the compute of 8Batch:199-291)."""
    real, intensity, mask, _, sky, index = point_cloud_to_range_image(pts, origin, True, rowMax=H, colMax=W)
    gd, gi, _, _, _, _ = point_cloud_to_range_image(goal_pts, origin, True, rowMax=H, colMax=W)
    roll = roll_draw() if roll_draw is not None else 0
    real, notmask, notsky, goal = _post(real, intensity, mask, sky, gd, gi, H, W, roll if random_roll else None,
                                        variant, nb)
    return real, notmask, notsky, index, goal


def transform(pts, to_world, from_world):
    """8Batch:146-190: fromWorld @ (toWorld @ [x y z 1]) with the intensity re-attached."""
    inten = pts[:, -1]
    pv = np.concatenate((np.transpose(pts[:, :-1]), np.expand_dims(np.ones_like(inten), 0)), 0)
    pv = np.matmul(from_world, np.matmul(to_world, pv))
    return np.transpose(np.concatenate((pv[:-1], np.expand_dims(inten, 0)), 0))
