"""KITTI-360 datasets with the per-view rendering on the GPU.

Drop-ins for the three datasets the simultaneous-sampling configs name
(LiDARGen/datasets/__init__.py picks them by ``config.data.dataset``):
  KITTI360_im_8batch                       datasets/kitti360_im_8Batch.py
  KITTI360_im_AllForOne                    datasets/kitti360_im_AllForOne.py
  KITTI360_im_simultaneous_densification   datasets/kitti360_im_simultenous_densification.py
Same constructor, ``__len__`` and ``__getitem__`` (the 9-tuple of numpy arrays the
DataLoader collates).  What the reference does on the CPU per view -- the pose chain applied
to every point, point_cloud_to_range_image (argsort + np.unique z-buffer) for the view and
its goal scan, and the post-processing -- runs here in libsdp (``sdp_view_transform``,
``sdp_range_project``, ``sdp_view_gather``, ``sdp_view_finalize``); only the .bin read and the
4x4 pose algebra stay on the host.  ``render(idx)`` returns the same views as device tensors
for callers that keep them in HBM.

``root`` replaces the hard-coded "/data/KITTI-360" (kitti360_im_8Batch.py:25,49,53,58); the
directory layout is the reference's.  Reference behaviour kept: ``frames`` are the pose file's
frame numbers minus 1 (L63), a goal pose past the end is clamped but its successor is still
read (L166-178, IndexError on the last pose as in the reference), ``np.random.randint`` for the
roll is drawn on every item (L234), 8batch / AllForOne need 2 channels (their goalIntensity
is undefined otherwise, L246), the densification variant needs 2 channels (6-value unpack,
L186).
"""
from __future__ import annotations

import os
from glob import glob

import numpy as np
import torch

from . import _lib

KITTI360_ROOT = "/data/KITTI-360"
DRIVE = "2013_05_28_drive_0000_sync"
MAX_RANGE = 2057.701
VARIANTS = {"KITTI360_im_8batch": 0, "KITTI360_im_AllForOne": 1, "KITTI360_im_simultaneous_densification": 2}


def load_velodyne(path):
    """kitti360_im_8Batch.py:309-315."""
    if not os.path.isfile(path):
        raise RuntimeError("%s does not exist!" % path)
    return np.fromfile(path, dtype=np.float32).reshape(-1, 4)


def pose_chain(root, drive=DRIVE):
    """kitti360_im_8Batch.py:49-68: (frames - 1, {frame: pose @ camToPose @ inv(camToVelo)})."""
    velo_to_cam = np.loadtxt(os.path.join(root, "calibration/calib_cam_to_velo.txt")).reshape(3, 4)
    velo_to_cam = np.linalg.inv(np.concatenate((velo_to_cam, np.array([0., 0., 0., 1.]).reshape(1, 4))))
    cam_to_pose = np.loadtxt(os.path.join(root, "calibration/calib_cam_to_pose.txt"))[0].reshape(3, 4)
    cam_to_pose = np.concatenate((cam_to_pose, np.array([0., 0., 0., 1.]).reshape(1, 4)))
    velo_to_pose = np.matmul(cam_to_pose, velo_to_cam)
    poses = np.loadtxt(os.path.join(root, "data_poses", drive, "poses.txt"))
    frames = poses[:, 0] - 1
    tr = {}
    for frame, pose in zip(frames, poses[:, 1:].reshape(-1, 3, 4)):
        tr[frame] = np.matmul(np.concatenate((pose, np.array([0., 0., 0., 1.]).reshape(1, 4))), velo_to_pose)
    return frames, tr


class _Workspace:
    def __init__(self, H, W, device):
        n = _lib.SZ()
        _lib.check(_lib.lib().sdp_range_project_workspace_size(H, W, _lib.C.byref(n)), "range_project_ws")
        self.ws = torch.empty(n.value, dtype=torch.uint8, device=device)


class _KITTI360View:
    """Shared body of the three datasets; ``variant`` selects the per-item semantics."""
    variant = -1

    def __init__(self, path, config, split="train", resolution=None, transform=None, root=KITTI360_ROOT, device=None):
        self.transform = transform
        self.return_remission = config.data.channels == 2
        self.random_roll = config.data.random_roll
        self.modifications = np.array(config.data.modifications)
        self.batchSize = config.sampling.actualBatchSize
        self.rowMax = config.data.image_size
        self.colMax = config.data.image_width
        full_list = glob(os.path.join(root, "data_3d_raw", DRIVE, "velodyne_points/data/*.bin"))
        if split == "test":
            self.full_list = [f for f in full_list if "0000_sync" in f or "0001_sync" in f]
        else:
            self.full_list = [f for f in full_list if "0000_sync" not in f]
        self.frames, self.Tr_pose_world = pose_chain(root)
        self.length = len(self.frames) * self.batchSize
        self.saveNum = 0
        self.device = torch.device(device) if device is not None else None    # resolved on first render
        self._ws = None

    def __len__(self):
        return self.length

    # ------------------------------------------------------------------ device steps
    def _project(self, pts64, origin, masks=True):
        """sdp_range_project; masks=False (a goal scan: only depth and intensity are used) skips
        the sky / obfuscation scan."""
        H, W, dev = self.rowMax, self.colMax, self.device
        if self._ws is None:
            self._ws = _Workspace(H, W, dev)
        depth = torch.empty(H, W, dtype=torch.float64, device=dev)
        inten = torch.empty(H, W, dtype=torch.float64, device=dev)
        obf = torch.empty(H, W, dtype=torch.uint8, device=dev) if masks else None
        sky = torch.empty(H, W, dtype=torch.uint8, device=dev) if masks else None
        index = torch.empty(H, W, dtype=torch.int64, device=dev)
        o = np.ascontiguousarray(np.asarray(origin, dtype=np.float64).reshape(3))
        N = pts64.shape[0]
        _lib.check(_lib.lib().sdp_range_project(pts64.data_ptr() if N else None, N, 4, 1, o.ctypes.data, H, W,
                                                depth.data_ptr(), inten.data_ptr(), _lib.ptr(obf), _lib.ptr(sky),
                                                index.data_ptr(), self._ws.ws.data_ptr(), self._ws.ws.numel(),
                                                _lib.stream()), "range_project")
        return depth, inten, obf, sky, index

    def _to_view(self, scan, m1=None, m2=None):
        pts = torch.from_numpy(np.ascontiguousarray(scan, dtype=np.float32)).to(self.device)
        out = torch.empty(pts.shape[0], 4, dtype=torch.float64, device=self.device)
        a1 = np.ascontiguousarray(m1, dtype=np.float64) if m1 is not None else None
        a2 = np.ascontiguousarray(m2, dtype=np.float64) if m2 is not None else None
        _lib.check(_lib.lib().sdp_view_transform(pts.data_ptr(), pts.shape[0], a1.ctypes.data if a1 is not None else None,
                                                 a2.ctypes.data if a2 is not None else None, out.data_ptr(),
                                                 _lib.stream()), "view_transform")
        return pts, out

    def _scan_name(self, frame):
        d = self.full_list[0]
        return d[:-len(d.split("/")[-1])] + str(int(frame)).zfill(10) + ".bin"

    def _goal_scan(self, pose_desired):
        frames = self.frames
        stack = []
        for frame_count in range(int(frames[pose_desired + 1] - frames[pose_desired])):   # L178-184
            if frame_count > 0:
                continue
            stack.append(load_velodyne(self._scan_name(frames[pose_desired] + frame_count)))
        return np.concatenate(stack, 0)

    # ------------------------------------------------------------------ one item
    def render(self, idx):
        """Device form of __getitem__: dict of cuda tensors + the host matrices."""
        if not self.return_remission:
            raise NameError("name 'goalIntensity' is not defined")   # 8Batch:246 / 6-value unpack (densification)
        H, W = self.rowMax, self.colMax
        number_in_batch = idx % self.batchSize
        pose_num = idx // self.batchSize
        if self.variant != 2:                                         # the host-side failure comes first
            pose_desired = min(pose_num + ((number_in_batch + 1) * 5 if self.variant == 0 else 10),
                               len(self.frames) - 1)
            goal_scan = self._goal_scan(pose_desired)
        if self.device is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        initial_scan = int(self.frames[pose_num])
        scan = load_velodyne(self._scan_name(initial_scan))
        to_world = self.Tr_pose_world[initial_scan]
        to_og_view = np.linalg.inv(to_world)
        if self.variant == 2:      # densification: subsample from modifications[0], view from modifications[k]
            raw, pts64 = self._to_view(scan)
            _, _, _, _, idx0 = self._project(pts64, self.modifications[0])
            sub = torch.empty(H * W, 4, dtype=torch.float64, device=self.device)
            cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
            _lib.check(_lib.lib().sdp_view_gather(idx0.data_ptr(), H, W, W // 4, raw.data_ptr(), sub.data_ptr(),
                                                  cnt.data_ptr(), _lib.stream()), "view_gather")
            view_pts = sub[: int(cnt.item())]
            goal_pts = pts64
            origin = self.modifications[number_in_batch]
            ret_to_world, ret_from_world = to_world, to_og_view
        else:
            # goal pose 5(k+1) (8Batch:162-168) or 10 (AllForOne:166-172) poses ahead, clamped
            goal_to_world = self.Tr_pose_world[self.frames[pose_desired]]
            from_world = np.linalg.inv(goal_to_world)
            _, view_pts = self._to_view(scan, to_world, from_world)
            _, goal_pts = self._to_view(goal_scan)
            origin = np.zeros(3) if self.variant == 0 else self.modifications[number_in_batch]
            ret_to_world, ret_from_world = goal_to_world, from_world
        depth, inten, obf, sky, index = self._project(view_pts, origin)
        gdepth, ginten, _, _, _ = self._project(goal_pts, origin, masks=False)
        roll = int(np.random.randint(self.colMax))          # drawn on every item (8Batch:234)
        C = 2
        real = torch.empty(C, H, W, dtype=torch.float64, device=self.device)
        goal = torch.empty(C, H, W, dtype=torch.float64, device=self.device)
        notmask = torch.empty(C, H, W, dtype=torch.uint8, device=self.device)
        notsky = torch.empty(1, H, W, dtype=torch.uint8, device=self.device)
        _lib.check(_lib.lib().sdp_view_finalize(depth.data_ptr(), inten.data_ptr(), obf.data_ptr(), sky.data_ptr(),
                                                gdepth.data_ptr(), ginten.data_ptr(), H, W, C,
                                                roll if self.random_roll else -1, self.variant,
                                                1 if number_in_batch == 0 else 0, real.data_ptr(), notmask.data_ptr(),
                                                notsky.data_ptr(), goal.data_ptr(), _lib.stream()), "view_finalize")
        return dict(real=real, notmask=notmask.bool(), notsky=notsky.bool(), index=index.unsqueeze(0),
                    toWorld=np.expand_dims(ret_to_world, 0), fromWorld=np.expand_dims(ret_from_world, 0), goal=goal,
                    toOGView=to_og_view, initialScan=initial_scan)

    def __getitem__(self, idx):
        r = self.render(idx)
        return (r["real"].cpu().numpy(), r["notmask"].cpu().numpy(), r["notsky"].cpu().numpy(),
                r["index"].cpu().numpy().astype(np.float64), r["toWorld"], r["fromWorld"], r["goal"].cpu().numpy(),
                r["toOGView"], r["initialScan"])


class KITTI360_im_8batch(_KITTI360View):
    """datasets/kitti360_im_8Batch.py:13-315 (view k of a megabatch = the scan re-rendered from
    the pose 5(k+1) frames ahead; goal = that pose's own scan)."""
    variant = 0


class KITTI360_im_AllForOne(_KITTI360View):
    """datasets/kitti360_im_AllForOne.py (points moved to the pose 10 frames ahead, view k
    rendered from config.data.modifications[k])."""
    variant = 1


class KITTI360_im_simultaneous_densification(_KITTI360View):
    """datasets/kitti360_im_simultenous_densification.py (the scan subsampled to the pixels
    seen from modifications[0] outside the first W/4 columns, view k rendered from
    modifications[k]; view 0's mask is the first W/4 columns)."""
    variant = 2


class MySampler:
    """runners/ncsn_runner_kitti_simultaneous.py:54-74: megabatches of ``batch_size``
    consecutive items, in an order drawn by np.random.shuffle even when random=False."""

    def __init__(self, num_batches, batch_size, random=True):
        self.n_batches, self.batch_size, self.random = num_batches, batch_size, random

    def __iter__(self):
        numbers = np.arange(self.n_batches)
        if self.random:
            np.random.shuffle(numbers)
        options = np.arange(self.n_batches)
        np.random.shuffle(options)
        return iter([int(numbers[c]) * self.batch_size + i for c in options for i in range(self.batch_size)])


def val_size(root, actual_batch_size, drive=DRIVE):
    """kitti:503-510: number of sampler megabatches = poses - 5 * actualBatchSize."""
    return np.loadtxt(os.path.join(root, "data_poses", drive, "poses.txt")).shape[0] - actual_batch_size * 5


def collate(items):
    """torch default_collate of the 9-tuples: stacked tensors, the scan numbers as int64."""
    out = []
    for k, parts in enumerate(zip(*items)):
        out.append(torch.as_tensor(np.asarray(parts)) if k != 8 else torch.tensor(parts, dtype=torch.int64))
    return tuple(out)


def get_dataset(name, path, config, split="test", **kw):
    """Name -> class as datasets/__init__.py:get_dataset does for these three."""
    cls = {"KITTI360_im_8batch": KITTI360_im_8batch, "KITTI360_im_AllForOne": KITTI360_im_AllForOne,
           "KITTI360_im_simultaneous_densification": KITTI360_im_simultaneous_densification}[name]
    return cls(path, config, split=split, **kw)
