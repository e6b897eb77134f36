"""TEST INFRASTRUCTURE ONLY (the checker, never the product): numpy restatement of the reference's
voxel-grid subsampling, order-free (cells sorted by voxel index; the reference returns them in
std::unordered_map order, which oracle/_ref -- the reference's own C++ compiled by
oracle/build_ref.sh -- pins instead).

  barycenters  LiDARGen/datasets/cpp_wrappers/cpp_subsampling/grid_subsampling/grid_subsampling.cpp:19-102
  lidar        .../grid_subsampling/grid_subsampling_lidar.cpp:19-120
Float arithmetic follows the C++: float32 corner/divisions (cloud.h floor / operator*), float32
running sums in point order, barycenter = sum * float(1.0 / count), features / float(count).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def voxel_keys(points: np.ndarray, dl: float) -> np.ndarray:
    """grid_subsampling.cpp:24-61: mapIdx = iX + nX*iY + nX*nY*iZ (size_t)."""
    p = np.asarray(points, np.float32)
    dl = F32(dl)
    lo, hi = p.min(0), p.max(0)
    org = np.floor(lo * (F32(1) / dl)).astype(np.float32) * dl
    nx = np.uint64(np.floor((hi[0] - org[0]) / dl)) + np.uint64(1)
    ny = np.uint64(np.floor((hi[1] - org[1]) / dl)) + np.uint64(1)
    idx = np.floor((p - org) / dl).astype(np.float32).astype(np.uint64)
    return idx[:, 0] + nx * idx[:, 1] + nx * ny * idx[:, 2]


def _alignment(gx, gy):
    """grid_subsampling_lidar.cpp:68-76 (C truncation and remainder)."""
    ix, iy = int(np.trunc(gx)), int(np.trunc(gy))
    best = 0
    for m in range(1, 17):
        p = 2 ** m
        if int(np.fmod(ix, p)) != 0 and int(np.fmod(iy, p)) != 0:
            best = m
        else:
            break
    return best


def subsample(points, features=None, classes=None, dl=0.1, lidar=False):
    """-> dict(key -> (point f32[3], features f32[d] | None, labels i32[l] | None)), one per voxel."""
    p = np.asarray(points, np.float32)
    f = None if features is None else np.asarray(features, np.float32)
    c = None if classes is None else np.asarray(classes, np.int32).reshape(len(p), -1)
    keys = voxel_keys(p, dl)
    cells = {}
    for i, k in enumerate(keys.tolist()):
        cell = cells.setdefault(k, {"n": 0, "best": -1, "pt": np.zeros(3, np.float32),
                                    "f": None if f is None else np.zeros(f.shape[1], np.float32),
                                    "h": None if c is None else [dict() for _ in range(c.shape[1])]})
        if not lidar:
            cell["n"] += 1
            cell["pt"] = (cell["pt"] + p[i]).astype(np.float32)
            if f is not None:
                cell["f"] = (cell["f"] + f[i]).astype(np.float32)
            if c is not None:
                for j, v in enumerate(c[i]):
                    cell["h"][j][int(v)] = cell["h"][j].get(int(v), 0) + 1
            continue
        if f is not None:
            # alignment coordinates: the two floats before point i's feature row (i = 0: (0, 0))
            flat = f.reshape(-1)
            b = _alignment(0.0, 0.0) if i == 0 else _alignment(flat[i * f.shape[1] - 2], flat[i * f.shape[1] - 1])
            if cell["best"] < b:
                cell.update(best=b, n=cell["n"] + 1, pt=p[i].copy(), f=f[i].copy())
                if c is not None:
                    cell["h"] = [{int(v): 1} for v in c[i]]
        else:
            cell["n"] += 1
            cell["pt"] = p[i].copy()
            if c is not None:
                for j, v in enumerate(c[i]):
                    cell["h"][j][int(v)] = cell["h"][j].get(int(v), 0) + 1
    out = {}
    for k, cell in cells.items():
        if lidar:
            pt, ff = cell["pt"], cell["f"]
        else:
            pt = (cell["pt"] * F32(1.0 / cell["n"])).astype(np.float32)
            ff = None if cell["f"] is None else (cell["f"] / F32(cell["n"])).astype(np.float32)
        # majority label; equal votes -> any of the maxima (the C++ keeps its hash order's first)
        lab = None if cell["h"] is None else [max(h.values()) for h in cell["h"]]
        out[k] = (pt, ff, cell["h"], lab)
    return out
