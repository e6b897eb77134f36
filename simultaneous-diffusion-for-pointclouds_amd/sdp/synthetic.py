"""Synthetic Line.yml-shaped inputs (no KITTI-360 offline): procedural scene range images.

SURVEY §8(d): view k sits at translation (5k m, 0, 0) (the "+5 frames per view" of
kitti360_im_8Batch.py:162-168); the scene is a ground plane z=-1.73 m, two walls y=+-8 m and
a few boxes; depth code = log2(d+1)/6 clipped to [0,1]; intensity U[0,0.5]; mask hides a
contiguous 25 % azimuth sector (kitti360_im_simultenous_densification.py:193-197); sky all
true (lidar_utils.py:295 clears it); existMask = the reference's hit-count fixture
thresholded and eroded as runners/ncsn_runner_kitti_simultaneous.py:527-530.
"""
from __future__ import annotations

import math
import os

import numpy as np

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def exist_mask(H: int = 64, W: int = 1024) -> np.ndarray:
    packed = np.load(os.path.join(_DATA, "exist_mask_64x1024_packed.npy"))
    ex = np.unpackbits(packed)[: 64 * 1024].reshape(64, 1024).astype(bool)
    if (H, W) != (64, 1024):
        ex = ex[:: max(1, 64 // H), :: max(1, 1024 // W)][:H, :W]
    return np.ascontiguousarray(ex)


def _angles(H, W):
    hA = math.radians(360) / W
    vA = math.radians(28) / H
    hMin = ((W * -180) // 360) * hA + hA / 2
    vMin = ((H * -25) // 28) * vA + vA / 2
    az = np.arange(W - 1, -1, -1) * hA + hMin
    el = np.arange(H - 1, -1, -1) * vA + vMin
    return az, el


def scene_views(n_views: int, H: int = 64, W: int = 1024, seed: int = 1234, spacing: float = 5.0):
    """Returns dict(ref [V,2,H,W] f32, mask [V,2,H,W] i32, sky [V,1,H,W] bool,
    toWorld/fromWorld [V,4,4] f64)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    az, el = _angles(H, W)
    d = np.stack([np.cos(el)[:, None] * np.cos(az)[None, :], np.cos(el)[:, None] * np.sin(az)[None, :],
                  np.broadcast_to(np.sin(el)[:, None], (H, W))], 0)          # [3,H,W]
    boxes = [(rng.uniform(-10, 10 + spacing * n_views), rng.uniform(-6, 6), rng.uniform(0.8, 2.5),
              rng.uniform(0.8, 2.5)) for _ in range(12)]
    ref = np.zeros((n_views, 2, H, W), np.float32)
    mask = np.zeros((n_views, 2, H, W), np.int32)
    toW = np.zeros((n_views, 4, 4))
    fromW = np.zeros((n_views, 4, 4))
    for k in range(n_views):
        o = np.array([spacing * k, 0.0, 0.0])
        t = np.full((H, W), np.inf)
        with np.errstate(divide="ignore", invalid="ignore"):
            tg = (-1.73 - o[2]) / d[2]
            t = np.where((tg > 0), np.minimum(t, tg), t)
            for wy in (-8.0, 8.0):
                tw = (wy - o[1]) / d[1]
                t = np.where(tw > 0, np.minimum(t, tw), t)
            for (bx, by, hx, hy) in boxes:   # axis-aligned boxes, slab test, height 0..2 m above ground
                lo = np.array([bx - hx, by - hy, -1.73])[:, None, None]
                hi = np.array([bx + hx, by + hy, 0.27])[:, None, None]
                t1 = (lo - o[:, None, None]) / d
                t2 = (hi - o[:, None, None]) / d
                tn = np.nanmax(np.minimum(t1, t2), 0)
                tf = np.nanmin(np.maximum(t1, t2), 0)
                hit = (tf >= tn) & (tn > 0)
                t = np.where(hit, np.minimum(t, tn), t)
        hitm = np.isfinite(t) & (t < 80)
        depth = np.where(hitm, t, 0.0)
        ref[k, 0] = np.clip(np.log2(depth + 1) / 6, 0, 1)
        ref[k, 1] = np.where(hitm, rng.uniform(0, 0.5, (H, W)), 0)
        m = hitm.copy()
        c0 = int(rng.integers(0, W))
        m[:, (np.arange(W) - c0) % W < W // 4] = False
        mask[k] = m[None]
        T = np.eye(4)
        T[:3, 3] = o
        toW[k] = T
        fromW[k] = np.linalg.inv(T)
    sky = np.ones((n_views, 1, H, W), bool)
    return dict(ref=ref, mask=mask, sky=sky, toWorld=toW, fromWorld=fromW)
