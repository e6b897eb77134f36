"""ORACLE (test infrastructure only) -- frozen, seeded input generators for the golden fixtures.

``oracle/gen_golden.py`` feeds these inputs to the reference code to produce the expected
outputs in ``tests/golden/``; the tests regenerate the same inputs from the same seeds
(numpy PCG64 streams are stable across platforms and numpy versions), so the fixtures
only have to store outputs.  Do not change a generator without regenerating fixtures.
"""
from __future__ import annotations

import os
import zlib

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def rng(tag: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(zlib.crc32(tag.encode("utf-8"))))


def exist_mask_full() -> np.ndarray:
    """The reference's MeasureResults/existTotalLiDARGenSettings.npy, thresholded and eroded
    exactly as runners/ncsn_runner_kitti_simultaneous.py:527-530 does (bool [64,1024]).

    The committed fixture ``tests/golden/exist_mask_64x1024.npy`` holds that result
    (packed bits, produced by gen_golden.py from the reference data file).
    """
    packed = np.load(os.path.join(GOLDEN_DIR, "exist_mask_64x1024_packed.npy"))
    return np.unpackbits(packed)[: 64 * 1024].reshape(64, 1024).astype(bool)


def exist_mask(W: int) -> np.ndarray:
    ex = exist_mask_full()
    step = 1024 // W
    return np.ascontiguousarray(ex[:, ::step])


def scorenet_input(tag: str, B: int, H: int, W: int):
    r = rng("scorenet-x-" + tag)
    x = r.random((B, 2, H, W), dtype=np.float64).astype(np.float32)
    return x


def yaw_pose(yaw_deg: float, t):
    c, s = np.cos(np.radians(yaw_deg)), np.sin(np.radians(yaw_deg))
    T = np.eye(4)
    T[:3, :3] = [[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]]
    T[:3, 3] = t
    return T


def merge_case(tag: str, B: int, H: int, W: int, sigma_mod: float = 1.0, neg_frac: float = 0.05,
               identity: bool = False):
    """Inputs for one consistency-merge step (KITTISampling.py:6-7 argument set).

    Returns dict: x [B,2,H,W] f32, ref [B,2,H,W] f32, mask int32 [B,2,H,W] (1 = known),
    sky bool [B,1,H,W], exist bool [B,H,W], toWorld/fromWorld f64 [B,4,4].
    Depth codes are log2(d+1)/6 * sigma_mod of a smooth synthetic scene plus noise.
    """
    r = rng("merge-" + tag)
    rows = np.arange(H)[:, None] / max(H - 1, 1)
    cols = np.arange(W)[None, :] / W
    x = np.empty((B, 2, H, W), np.float32)
    for b in range(B):
        d = 4.0 + 20.0 * rows + 6.0 * (1 + np.sin(2 * np.pi * (cols * (b + 1)) + b)) + r.uniform(0, 2.0, (H, W))
        code = np.log2(d + 1.0) / 6.0 * sigma_mod
        neg = r.random((H, W)) < neg_frac
        code = np.where(neg, -code, code)
        x[b, 0] = code
        x[b, 1] = r.random((H, W))
    ref = np.empty_like(x)
    ref[:, 0] = np.clip(x[:, 0] + r.normal(0, 0.02, (B, H, W)), 0, None)
    ref[:, 1] = r.random((B, H, W))
    mask = np.ones((B, 2, H, W), np.int32)
    for b in range(B):
        c0 = int(r.integers(0, W))
        sector = (np.arange(W) - c0) % W < W // 4
        mask[b, :, :, sector] = 0
    mask &= (r.random((B, 1, H, W)) > 0.1).astype(np.int32)
    sky = r.random((B, 1, H, W)) > 0.1
    exist = np.broadcast_to(exist_mask(W), (B, H, W)).copy()
    toWorld = np.empty((B, 4, 4))
    fromWorld = np.empty((B, 4, 4))
    for b in range(B):
        if identity:
            T = np.eye(4)
        else:
            T = yaw_pose(10.0 * b - 5.0, [5.0 * b, 0.7 * b, 0.1 * b])
        toWorld[b] = T
        fromWorld[b] = np.linalg.inv(T)
    return dict(x=x, ref=ref, mask=mask, sky=sky, exist=exist, toWorld=toWorld, fromWorld=fromWorld)


def noise(tag: str, k: int, shape) -> np.ndarray:
    return rng(f"noise-{tag}-{k}").standard_normal(shape).astype(np.float32)


def projection_cloud(tag: str, n: int = 60000) -> np.ndarray:
    """Synthetic LiDAR-like point cloud [n, 4] float64 (x, y, z, intensity): a ground plane,
    two walls, boxes and free clutter around the origin -- the input shape
    datasets/kitti360_im_8Batch.py:199 hands to point_cloud_to_range_image."""
    r = rng("projection_" + tag)
    k = n // 4
    ang = r.uniform(-np.pi, np.pi, k)
    rad = np.sqrt(r.uniform(1.0, 45.0 ** 2, k))
    ground = np.stack([rad * np.cos(ang), rad * np.sin(ang), -1.73 + r.normal(0, 0.02, k)], 1)
    wy = np.where(r.random(k) < 0.5, -8.0, 8.0)
    walls = np.stack([r.uniform(-40, 40, k), wy + r.normal(0, 0.05, k), r.uniform(-1.73, 3.0, k)], 1)
    bc = r.uniform(-20, 20, (12, 2))
    bi = r.integers(0, 12, k)
    boxes = np.stack([bc[bi, 0] + r.uniform(-1.5, 1.5, k), bc[bi, 1] + r.uniform(-1.5, 1.5, k),
                      r.uniform(-1.73, 0.5, k)], 1)
    m = n - 3 * k
    clutter = np.stack([r.uniform(-60, 60, m), r.uniform(-60, 60, m), r.uniform(-3, 8, m)], 1)
    xyz = np.concatenate([ground, walls, boxes, clutter], 0)
    inten = r.uniform(0, 1, n).astype(np.float32).astype(np.float64)
    return np.ascontiguousarray(np.concatenate([xyz, inten[:, None]], 1))


PROJECTION_CASES = {"scene_o0": (60000, (0.0, 0.0, 0.0)), "scene_off": (60000, (2.5, -1.25, 0.4))}
