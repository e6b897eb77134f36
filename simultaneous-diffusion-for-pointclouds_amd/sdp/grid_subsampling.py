"""Voxel-grid subsampling: the reference's CPython modules on libsdp's host C++.

  compute(points, *, features, classes, sampleDl, method, verbose)        grid_subsampling.compute
  compute_lidar(points, *, features, classes, sampleDl, method, verbose)  grid_subsampling_lidar.compute
      (LiDARGen/datasets/cpp_wrappers/cpp_subsampling/wrapper.cpp:58-285, wrapper_lidar.cpp)
  grid_sub_sampling(points, features, labels, grid_size, verbose)         kitti360_im_SceneCompletion.py:18-36

Same argument handling and return convention as the CPython wrapper: points float32 [N,3];
optional features float32 [N,d] and classes int32 [N] / [N,d]; returns the points array alone, or
a tuple (points, features), (points, classes) or (points, features, classes); classes come back
[M, ldim]; `method` must be "barycenters" or "voxelcenters" and is otherwise unused (as in the
reference); errors raise RuntimeError.  Host memory in and out: this is CPU data preparation.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


def _run(points, features, classes, sampleDl, method, lidar):
    if method not in ("barycenters", "voxelcenters"):
        raise RuntimeError('Error parsing method. Valid method names are "barycenters" and "voxelcenters" ')
    pts = np.ascontiguousarray(np.asarray(points, dtype=np.float32))
    if pts.ndim != 2 or pts.shape[1] != 3:
        raise RuntimeError("Wrong dimensions : points.shape is not (N, 3)")
    n = pts.shape[0]
    f = c = None
    fdim, ldim = 0, 1
    if features is not None:
        f = np.ascontiguousarray(np.asarray(features, dtype=np.float32))
        if f.ndim != 2 or f.shape[0] != n:
            raise RuntimeError("Wrong dimensions : features.shape is not (N, d)")
        fdim = f.shape[1]
    if classes is not None:
        c = np.ascontiguousarray(np.asarray(classes, dtype=np.int32))
        if c.ndim > 2 or c.shape[0] != n:
            raise RuntimeError("Wrong dimensions : classes.shape is not (N,) or (N, d)")
        ldim = c.shape[1] if c.ndim == 2 else 1
    if n < 1 or (f is not None and fdim < 1):
        raise RuntimeError("Error")
    op = np.empty((n, 3), np.float32)
    of = np.empty((n, fdim), np.float32) if f is not None else None
    oc = np.empty((n, ldim), np.int32) if c is not None else None
    m = C.c_int64()
    ptr = lambda a: None if a is None else a.ctypes.data
    _lib.check(_lib.lib().sdp_grid_subsample(ptr(pts), n, ptr(f), fdim, ptr(c), ldim, float(np.float32(sampleDl)),
                                             1 if lidar else 0, ptr(op), ptr(of), ptr(oc), C.byref(m)),
               "grid_subsample")
    k = m.value
    if k < 1:
        raise RuntimeError("Error")
    out = [op[:k].copy()]
    if of is not None:
        out.append(of[:k].copy())
    if oc is not None:
        out.append(oc[:k].copy())
    return out[0] if len(out) == 1 else tuple(out)


def compute(points, *, features=None, classes=None, sampleDl=0.1, method="barycenters", verbose=0):
    """grid_subsampling.compute: per voxel the barycenter, mean features and majority labels."""
    return _run(points, features, classes, sampleDl, method, lidar=False)


def compute_lidar(points, *, features=None, classes=None, sampleDl=0.1, method="barycenters", verbose=0):
    """grid_subsampling_lidar.compute: per voxel the best power-of-2 aligned point (see csrc)."""
    return _run(points, features, classes, sampleDl, method, lidar=True)


def grid_sub_sampling(points, features=None, labels=None, grid_size=0.05, verbose=0):
    """kitti360_im_SceneCompletion.py:18-36."""
    if features is None and labels is None:
        return compute(points, sampleDl=grid_size, verbose=verbose)
    if labels is None:
        return compute(points, features=features, sampleDl=grid_size, verbose=verbose)
    if features is None:
        return compute(points, classes=labels, sampleDl=grid_size, verbose=verbose)
    return compute(points, features=features, classes=labels, sampleDl=grid_size, verbose=verbose)
