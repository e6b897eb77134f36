"""A synthetic SemanticKITTI-SSC test tree for the scene-completion dataset: scans
data_3d_raw/data_3d_ssc_test/velodyne_points/data/<name>.npy (float32 [N,3]) and their
companions data_3d_raw/data_3d_ssc_test/Final/<name>.npy ([M,4]): a street (ground sloping a
little, two facades along a tilted axis, boxes), the geometry the dataset's origin rule expects."""
import os

import numpy as np


def write_ssc_tree(root, n_scans=2, n_points=30000, seed=5):
    r = np.random.default_rng(seed)
    d = os.path.join(root, "data_3d_raw", "data_3d_ssc_test")
    os.makedirs(os.path.join(d, "velodyne_points", "data"), exist_ok=True)
    os.makedirs(os.path.join(d, "Final"), exist_ok=True)
    names = []
    for s in range(n_scans):
        th = 0.3 + 0.2 * s
        k = n_points // 3
        u = r.uniform(-45, 45, k)
        v = r.uniform(-7, 7, k)
        ground = np.stack([u, v, -1.7 + 0.01 * u + r.normal(0, 0.02, k)], 1)
        w = r.uniform(-45, 45, k)
        facade = np.stack([w, np.where(r.random(k) < 0.5, -8.0, 8.0), r.uniform(-1.7, 6.0, k)], 1)
        m = n_points - 2 * k
        boxes = np.stack([r.uniform(-30, 30, m), r.uniform(-5, 5, m), r.uniform(-1.7, 0.5, m)], 1)
        pts = np.concatenate([ground, facade, boxes])
        rot = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
        pts = (pts @ rot.T + np.array([2.0 * s, -1.0, 0.3])).astype(np.float32)
        name = f"{s:06d}.npy"
        np.save(os.path.join(d, "velodyne_points", "data", name), pts)
        extra = np.concatenate([pts[::7] + r.normal(0, 0.05, pts[::7].shape).astype(np.float32),
                                r.random((len(pts[::7]), 1)).astype(np.float32)], 1)
        np.save(os.path.join(d, "Final", name), extra)
        names.append(name)
    return names
