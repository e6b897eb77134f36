"""Scene-completion data front end: the SemanticKITTI-SSC dataset of the
Completion runner, with its voxel-grid subsampling on libsdp's host C++ and its range-image
projection + post-processing on the GPU.

  kitti360_im_SceneCompletion  LiDARGen/datasets/kitti360_im_SceneCompletion.py:38-513
      __getitem__(idx) -> (real f64 [2,H,W], notmask bool [2,H,W], notsky bool [1,H,W],
                           index [1,H,W], scan name (str), origin f64 [1,3])
  view_origin                  the per-view origin of lines 188-316 (linregress ground plane + the
                               principal direction through the scan, cut with circles of 35/40/50/30 m)

Per item: load the scan (.npy, [N,3]) and its "Final" companion, recentre both on the scan's median
+ a fixed offset (L157-167), grid-subsample the scan at 0.05 (grid_subsampling.compute, L172),
derive the view origin from the subsampled scan (L188-316), project the FULL recentred scan from
that origin (sdp_range_project, L342-345; the subsampled points only steer the origin, as in the
reference) and post-process (sdp_view_finalize, variant SDP_VIEW_COMPLETION: the second channel is
the depth code again with an all-ones mask -- the reference returns (real, real) / (mask, ones)).

Circle intersection.  The reference intersects a LineString with
``shapely.geometry.Point(0, 0).buffer(R).boundary`` -- GEOS's 64-segment polygon approximation of
the circle (quadrant segments 16, vertices at angles -k*2*pi/64 from (R, 0)) -- and takes
``geoms[0]``, the intersection point with the smallest (x, y) (GEOS OverlayNG emits result points in
coordinate order).  shapely is not in this image, so this is a restatement of that GEOS behaviour:
the segment intersections are computed exactly (rationals) and rounded, as GEOS's double-double
intersection does; parity of this step against shapely itself is unpinned.
"""
from __future__ import annotations

import math
import os
from fractions import Fraction
from glob import glob

import numpy as np
import torch

from . import _lib
from .grid_subsampling import grid_sub_sampling

ROUGH_MEDIAN = np.array([0.73530043, 0.12196524, -1.23688836])     # L157
SSC_SCANS = "data_3d_raw/data_3d_ssc_test/velodyne_points/data/*.npy"
SSC_FINAL = "data_3d_raw/data_3d_ssc_test/Final/"
RADII = {0: 35, 1: 40, 2: 50, 3: 30}          # first, second, third, fourth point (L210-296)


def _ring(R, quad_segs=16):
    n = 4 * quad_segs
    inc = 2.0 * math.pi / n
    pts = [(float(R), 0.0)]
    for i in range(1, n):
        a = 0.0 + (-1) * i * inc
        pts.append((0.0 + R * math.cos(a), 0.0 + R * math.sin(a)))
    pts.append(pts[0])
    return pts


def _seg_intersection(p0, p1, q0, q1):
    """Exact intersection point of segments p0p1 and q0q1 (None if they do not cross)."""
    P0, P1, Q0, Q1 = ([Fraction(c) for c in v] for v in (p0, p1, q0, q1))
    r = (P1[0] - P0[0], P1[1] - P0[1])
    s = (Q1[0] - Q0[0], Q1[1] - Q0[1])
    den = r[0] * s[1] - r[1] * s[0]
    if den == 0:
        return None
    qp = (Q0[0] - P0[0], Q0[1] - P0[1])
    t = (qp[0] * s[1] - qp[1] * s[0]) / den
    u = (qp[0] * r[1] - qp[1] * r[0]) / den
    if not (0 <= t <= 1 and 0 <= u <= 1):
        return None
    return (float(P0[0] + t * r[0]), float(P0[1] + t * r[1]))


def circle_line_first(R, x, y):
    """Point(0,0).buffer(R).boundary.intersection(LineString([(-x,-y),(x,y)])).geoms[0]."""
    ring = _ring(R)
    hits = set()
    for a, b in zip(ring[:-1], ring[1:]):
        h = _seg_intersection((-x, -y), (x, y), a, b)
        if h is not None:
            hits.add(h)
    if not hits:
        raise IndexError("tuple index out of range")      # shapely: an empty intersection has no geoms[0]
    return np.array(sorted(hits)[0])


def _direction(slope, intercept, R, start_y):
    """L198-205 (start_y: y = 1 first) / L224-231 (x = 1 first): the far end (x, y) of the line."""
    if start_y:
        y = 1
        x = y * slope + intercept
        mod = (R * 200) / np.sqrt(np.square(x) + np.square(y))
        x = x * mod
        y = x * slope + intercept
    else:
        x = 1
        y = x * slope + intercept
        mod = (R * 200) / np.sqrt(np.square(x) + np.square(y))
        x = x * mod
        y = x * slope + intercept
    return x, y


def view_origin(scan_sub, number_in_batch, modifications):
    """kitti360_im_SceneCompletion.py:186-318 on the subsampled scan (float32 [M,3] + a zero column)."""
    from scipy import stats
    origin = modifications[number_in_batch] if number_in_batch < len(modifications) else None
    if number_in_batch >= 8:
        return origin
    zslope, zintercept = stats.linregress(scan_sub[:, 0], scan_sub[:, 2])[:2]
    above = scan_sub[:, 0] * zslope + zintercept + 0.1 <= scan_sub[:, 2]
    pts = scan_sub[above]
    slope, intercept = stats.linregress(pts[:, 0], pts[:, 1])[:2]
    ends = {}
    for k, R in RADII.items():
        x, y = _direction(slope, intercept, R, start_y=(k in (0, 3)))   # first (35) and fourth (30) start from y = 1
        ends[k] = circle_line_first(R, x, y)
    zintercept = zintercept + (1.23688836 / 2)
    if number_in_batch <= 3:
        p = ends[number_in_batch]
        return np.concatenate((p, np.expand_dims(p[0] * zslope + zintercept, 0)), 0)
    if number_in_batch == 4:
        return np.zeros(3)
    return origin


class kitti360_im_SceneCompletion:
    """datasets/kitti360_im_SceneCompletion.py:38-513 (items rendered on the GPU)."""

    def __init__(self, path, config, split="train", resolution=None, transform=None, root="/data/KITTI-360",
                 device=None):
        self.transform = transform
        self.return_remission = config.data.channels == 2
        self.random_roll = config.data.random_roll
        self.modifications = np.array(config.data.modifications)
        self.batchSize = config.sampling.batch_size
        self.rowMax = config.data.image_size
        self.colMax = config.data.image_width
        self.root = root
        self.full_list = glob(os.path.join(root, SSC_SCANS))      # unsorted, as the reference's glob
        self.length = len(self.full_list) * self.batchSize
        self.device = torch.device(device) if device is not None else None
        self._ws = None

    def __len__(self):
        return self.length

    def _project(self, pts64, origin):
        from .kitti360 import _Workspace
        H, W, dev = self.rowMax, self.colMax, self.device
        if self._ws is None:
            self._ws = _Workspace(H, W, dev)
        f64 = lambda: torch.empty(H, W, dtype=torch.float64, device=dev)
        depth, inten = f64(), f64()
        obf = torch.empty(H, W, dtype=torch.uint8, device=dev)
        sky = torch.empty(H, W, dtype=torch.uint8, device=dev)
        index = torch.empty(H, W, dtype=torch.int64, device=dev)
        o = np.ascontiguousarray(np.asarray(origin, dtype=np.float64).reshape(3))
        N = pts64.shape[0]
        _lib.check(_lib.lib().sdp_range_project(pts64.data_ptr() if N else None, N, 4, 1, o.ctypes.data, H, W,
                                                depth.data_ptr(), inten.data_ptr(), obf.data_ptr(), sky.data_ptr(),
                                                index.data_ptr(), self._ws.ws.data_ptr(), self._ws.ws.numel(),
                                                _lib.stream()), "range_project")
        return depth, inten, obf, sky, index

    def prepare(self, idx):
        """Host part of __getitem__: (points f64 [N,4] to project, origin, scan name, number in batch)."""
        number_in_batch = idx % self.batchSize
        initial_scan = idx // self.batchSize
        desired = self.full_list[initial_scan]
        name = desired.split("/")[-1]
        original = np.load(desired)
        extra = np.load(os.path.join(self.root, SSC_FINAL + name))
        extra[:, 3] = 0
        med = np.median(original, axis=0)
        original = original - med + ROUGH_MEDIAN
        extra[:, :3] = extra[:, :3] - med + ROUGH_MEDIAN
        scan = grid_sub_sampling(original.astype(np.float32))
        scan = np.concatenate((scan, np.expand_dims(np.zeros_like(scan[:, 0]), axis=1)), 1)
        original = np.concatenate((original, np.expand_dims(np.zeros_like(original[:, 0]), axis=1)), 1)
        origin = view_origin(scan, number_in_batch, self.modifications)
        return original, origin, name, number_in_batch

    def __getitem__(self, idx):
        if not self.return_remission:
            raise NotImplementedError("1-channel scene completion is outside the built path (channels: 2)")
        original, origin, name, _ = self.prepare(idx)
        if self.device is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        H, W = self.rowMax, self.colMax
        pts = torch.from_numpy(np.ascontiguousarray(original, dtype=np.float64)).to(self.device)
        depth, inten, obf, sky, index = self._project(pts, origin)
        roll = int(np.random.randint(self.colMax))            # drawn on every item (L367)
        real = torch.empty(2, H, W, dtype=torch.float64, device=self.device)
        notmask = torch.empty(2, H, W, dtype=torch.uint8, device=self.device)
        notsky = torch.empty(1, H, W, dtype=torch.uint8, device=self.device)
        _lib.check(_lib.lib().sdp_view_finalize(depth.data_ptr(), inten.data_ptr(), obf.data_ptr(), sky.data_ptr(),
                                                None, None, H, W, 2, roll if self.random_roll else -1, 3, 0,
                                                real.data_ptr(), notmask.data_ptr(), notsky.data_ptr(), None,
                                                _lib.stream()), "view_finalize")
        return (real.cpu().numpy(), notmask.bool().cpu().numpy(), notsky.bool().cpu().numpy(),
                index.unsqueeze(0).cpu().numpy().astype(np.float64), name[:-4], np.expand_dims(origin, axis=0))


def val_size(root):
    """ncsn_runner_Completion.py:500: the number of SSC test scans."""
    return len(glob(os.path.join(root, SSC_SCANS)))


def collate(items):
    """default_collate of the 6-tuples (the names stay a list of str)."""
    out = []
    for k, parts in enumerate(zip(*items)):
        out.append(list(parts) if k == 4 else torch.as_tensor(np.asarray(parts)))
    return tuple(out)
