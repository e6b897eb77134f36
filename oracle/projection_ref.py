"""ORACLE (test infrastructure only) -- numpy restatement of the reference's point-cloud ->
range-image projection, ``point_cloud_to_range_image`` (LiDARGen/datasets/lidar_utils.py:54-347),
the data front end of SURVEY §8(f)-1.  Checker for ``sdp_range_project`` (csrc/projection.hip);
only tests/ may import it.  Pinned by tests/golden/projection_*.npz (outputs of the reference
function itself, made by oracle/gen_golden.py).

Semantics kept (file:line of lidar_utils.py):
  * float64 geometry: relative points, xy, depth, atan2 angles (L159-166); bins by np.round
    (half to even) of (angle - min)/step (L167-168), clamped to the image (L172-180);
  * ``inGrid`` excludes row 0 and column 0 (L196);
  * nearest point per pixel (argsort by depth + unique first occurrence, L241-252); the
    reference's quicksort leaves ties between equal depths unspecified -- here the lowest
    point index wins;
  * a pixel whose nearest depth is exactly 0 stays empty (``tempDepth != 0``, L254-261);
  * empty pixels: depth and xy = maxRange 2057.701, intensity 0, index -1 (L138-141, L75);
  * np.flip of both axes (L270-279);
  * the sky / obfuscation scan over rows 2..H-2 and the last row (L283-306); the sky mask is
    cleared afterwards (L304).
"""
from __future__ import annotations

import math

import numpy as np

MAX_RANGE = 2057.701


def geometry(rowMax=64, colMax=1024):
    hA = math.radians(360) / colMax
    vA = math.radians(28) / rowMax
    hMin = colMax // (-2) * hA + hA / 2
    vMin = math.radians(3 - 28)
    return hA, vA, hMin, vMin


def point_cloud_to_range_image(point_cloud, origin, return_remission=False, rowMax=64, colMax=1024):
    pc = np.asarray(point_cloud, dtype=np.float64)
    intensity = pc[:, 3] if return_remission else None
    pts = pc[:, :3]
    N = len(pts)
    hA, vA, hMin, vMin = geometry(rowMax, colMax)
    rel = pts - np.asarray(origin, dtype=np.float64)
    xy2 = np.square(rel[:, 0]) + np.square(rel[:, 1])
    depth = np.sqrt(xy2 + np.square(rel[:, 2]))
    horizontal = np.arctan2(rel[:, 1], rel[:, 0])
    xy = np.sqrt(xy2)
    vertical = np.arctan2(rel[:, 2], xy)
    col = np.round(np.divide(horizontal - hMin, hA)).astype(int)
    row = np.round(np.divide(vertical - vMin, vA)).astype(int)
    col = np.maximum(0, np.minimum(colMax - 1, col))
    row = np.maximum(0, np.minimum(rowMax - 1, row))
    ing = (col > 0) & (col < colMax) & (row > 0) & (row < rowMax)
    idx = np.nonzero(ing)[0]
    # nearest per pixel, lowest index on equal depth
    order = np.lexsort((idx, depth[idx]))
    idx = idx[order]
    pix = row[idx] * colMax + col[idx]
    _, first = np.unique(pix, return_index=True)
    win = idx[first]
    img_depth = np.full((rowMax, colMax), MAX_RANGE)
    img_xy = np.full((rowMax, colMax), MAX_RANGE)
    img_int = np.zeros((rowMax, colMax))
    img_idx = np.full((rowMax, colMax), -1.0)
    keep = depth[win] != 0
    win = win[keep]
    r, c = row[win], col[win]
    img_depth[r, c] = depth[win]
    img_xy[r, c] = xy[win]
    img_idx[r, c] = win
    if return_remission:
        img_int[r, c] = intensity[win]
    img_depth, img_int, img_xy, img_idx = (np.flip(a).copy() for a in (img_depth, img_int, img_xy, img_idx))
    obf, sky = sky_scan(img_xy)
    if return_remission:
        return img_depth, img_int, obf, 0, sky, img_idx
    return img_depth, obf, 0, sky, img_idx


def sky_scan(img_xy):
    """lidar_utils.py:283-306 on the flipped xy image; returns (obfuscationMask, skyMask)."""
    H, W = img_xy.shape
    obf = np.zeros((H, W), bool)
    min_depth = np.zeros(W) + MAX_RANGE
    sky = np.zeros((H, W), bool)
    sky[0] = True
    sky[1] = True
    for row in range(2, H - 1):
        obf[row] = img_xy[row] > min_depth + 5
        e = ((img_xy[row] != min_depth).astype(int) + (img_xy[row - 1] != min_depth).astype(int)
             + (img_xy[row + 1] != min_depth).astype(int))
        e = np.concatenate(([0], e, [0]))
        e = e[1:-1] + e[:-2] + e[2:]
        cur = (e <= 1) & sky[row - 1]
        sky[row] = cur
        nm = np.minimum(img_xy[row], min_depth)
        min_depth[~cur] = nm[~cur]
    sky[:] = False
    obf[-1] = img_xy[-1] > min_depth + 5
    return obf, sky
