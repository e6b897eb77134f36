"""ORACLE (test infrastructure only) -- numpy restatement of the scene-completion dataset item
(SURVEY §8(f)-3), the checker for sdp/completion.py.  Only tests/ may import it.

Follows datasets/kitti360_im_SceneCompletion.py (under /root/reference/LiDARGen):
  scan / Final loading, median recentring      L134-167
  grid_sub_sampling(points, grid 0.05)         L18-36, L172  -> the reference's own C++ (oracle/_ref)
  view origin (linregress + circle cuts)       L186-318
  projection                                   L342-345      -> oracle.projection_ref (pinned)
  post-processing                              L349-513
Pinning: the module cannot be imported here (h5py and shapely are absent), so the statements are
restated; the projection is pinned by tests/golden/projection_*.npz and the subsampling by the
reference's compiled C++.  The circle cut restates shapely (GEOS 64-gon buffer, result points in
coordinate order) with plain float parametric intersections -- a second, independent formulation of
what sdp/completion.py computes with rationals (agreement to 1e-9 m); parity vs shapely unpinned.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

from .projection_ref import point_cloud_to_range_image

MAX_RANGE = 2057.701
ROUGH_MEDIAN = np.array([0.73530043, 0.12196524, -1.23688836])
_HERE = os.path.dirname(os.path.abspath(__file__))


def grid_sub_sampling_ref(points, dl=0.05):
    """The reference's barycenter subsampling, run from its compiled sources (oracle/_ref)."""
    path = os.path.join(_HERE, "_ref", "libgrid_ref.so")
    if not os.path.exists(path):
        raise FileNotFoundError("oracle/_ref/libgrid_ref.so: run oracle/build_ref.sh")
    L = C.CDLL(path)
    L.ref_grid_subsample.restype = C.c_int64
    L.ref_grid_subsample.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_float,
                                     C.c_void_p, C.c_void_p, C.c_void_p]
    p = np.ascontiguousarray(points, np.float32)
    out = np.empty((len(p), 3), np.float32)
    m = L.ref_grid_subsample(p.ctypes.data, len(p), None, 0, None, 0, dl, out.ctypes.data, None, None)
    return out[:m]


def circle_cut(R, x, y):
    """First (smallest x, then y) crossing of segment (-x,-y)-(x,y) with the 64-gon of radius R."""
    n = 64
    verts = [(R * math.cos(-2 * math.pi * k / n), R * math.sin(-2 * math.pi * k / n)) for k in range(n)]
    verts[0] = (float(R), 0.0)
    hits = []
    for k in range(n):
        (ax, ay), (bx, by) = verts[k], verts[(k + 1) % n]
        dx, dy, ex, ey = 2 * x, 2 * y, bx - ax, by - ay
        den = dx * ey - dy * ex
        if den == 0:
            continue
        t = ((ax + x) * ey - (ay + y) * ex) / den
        u = ((ax + x) * dy - (ay + y) * dx) / den
        if -1e-12 <= t <= 1 + 1e-12 and -1e-12 <= u <= 1 + 1e-12:
            hits.append((-x + t * dx, -y + t * dy))
    hits.sort()
    return np.array(hits[0])


def view_origin(scan, nib, modifications):
    from scipy import stats
    origin = modifications[nib] if nib < len(modifications) else None
    if nib >= 8:
        return origin
    zs, zi = stats.linregress(scan[:, 0], scan[:, 2])[:2]
    scan = scan[scan[:, 0] * zs + zi + 0.1 <= scan[:, 2]]
    slope, icpt = stats.linregress(scan[:, 0], scan[:, 1])[:2]

    def far(R, from_y):
        if from_y:
            xx = 1 * slope + icpt
            xx = xx * (R * 200) / np.sqrt(np.square(xx) + 1)
        else:
            yy = 1 * slope + icpt
            xx = 1 * (R * 200) / np.sqrt(1 + np.square(yy))
        return xx, xx * slope + icpt
    pts = [circle_cut(35, *far(35, True)), circle_cut(40, *far(40, False)), circle_cut(50, *far(50, False)),
           circle_cut(30, *far(30, True))]
    zi = zi + (1.23688836 / 2)
    if nib <= 3:
        p = pts[nib]
        return np.array([p[0], p[1], p[0] * zs + zi])
    if nib == 4:
        return np.zeros(3)
    return origin


def item(scan_path, final_path, nib, modifications, H=64, W=1024, roll=None):
    """(real, notmask, notsky, index, origin[1,3]) of one __getitem__ (channels 2)."""
    original = np.load(scan_path)
    extra = np.load(final_path)
    extra[:, 3] = 0
    med = np.median(original, axis=0)
    original = original - med + ROUGH_MEDIAN
    scan = grid_sub_sampling_ref(original.astype(np.float32))
    scan = np.concatenate((scan, np.zeros((len(scan), 1), scan.dtype)), 1)
    original = np.concatenate((original, np.zeros((len(original), 1))), 1)
    origin = view_origin(scan, nib, np.asarray(modifications))
    real, intensity, mask, _, sky, index = point_cloud_to_range_image(original, origin, True, H, W)
    mask = np.where(real >= MAX_RANGE, 1, mask)
    real = np.where(real >= MAX_RANGE, 0, real) + 0.0001
    real = np.clip(np.log2(real + 1) / 6, 0, 1)
    if roll is not None:
        real, mask, sky = (np.roll(a, roll, axis=1) for a in (real, mask, sky))
    real, mask = real[None], mask[None]
    sky = sky.copy()
    for _ in range(3):
        sky[1:] = sky[:-1]
    sky, index = sky[None], index[None]
    mask = np.where(intensity >= 1, 1, mask)
    real = np.concatenate((real, real), axis=0)
    mask = np.concatenate((mask, np.ones_like(mask)), axis=0)
    return real, np.logical_not(mask), np.logical_not(sky), index, np.expand_dims(origin, 0)
