"""GPU parity of the point cloud -> range image front end (csrc/projection.hip) against the
reference's own outputs (tests/golden/projection_*.npz, datasets/lidar_utils.py:54-347) and
the oracle.  Float64 geometry: bins, depths, xy, intensities and indices are expected bit-exact;
the device atan2/sqrt may differ from the host libm by an ulp, so at most 1e-4 of the pixels
may differ (a point exactly on a bin edge), every other pixel must match exactly."""
import numpy as np
import pytest
import torch

from oracle import golden_inputs as GI
from oracle import projection_ref as PR
from sdp.projection import point_cloud_to_range_image, project_device

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", sorted(GI.PROJECTION_CASES))
def test_projection_matches_reference_golden(tag):
    n, origin = GI.PROJECTION_CASES[tag]
    f = np.load(f"{GI.GOLDEN_DIR}/projection_{tag}.npz")
    d, inten, obf, save_num, sky, idx = point_cloud_to_range_image(GI.projection_cloud(tag, n), np.array(origin), True)
    assert save_num == 0 and d.dtype == np.float64 and d.shape == (64, 1024)
    assert np.mean(d != f["depth"]) <= 1e-4
    assert np.mean(inten.astype(np.float32) != f["intensity"]) <= 1e-4
    assert np.mean(idx.astype(np.int32) != f["index"]) <= 1e-4
    assert np.mean(obf != f["obf"]) <= 1e-3
    assert not sky.any()


def test_projection_edge_cases():
    """Empty cloud, points on row/col 0 (excluded), a point at the origin (depth 0 -> empty),
    exact duplicates (lowest index wins), no remission."""
    pts = np.array([[0.0, 0.0, 0.0, 0.9],          # at the origin: nearest depth 0 -> stays empty
                    [0.0, 10.0, 0.0, 0.5],
                    [0.0, 10.0, 0.0, 0.7],         # duplicate of point 1: index 1 wins
                    [5.0, 0.0, -30.0, 0.1]], np.float64)   # far below the vertical scope -> row 0 -> excluded
    d, obf, _, sky, idx = point_cloud_to_range_image(pts, np.zeros(3), False)
    rd, robf, _, rsky, ridx = PR.point_cloud_to_range_image(pts, np.zeros(3), False)
    assert np.array_equal(d, rd) and np.array_equal(idx, ridx) and np.array_equal(obf, robf)
    assert (idx == 1).sum() == 1 and (idx == 2).sum() == 0 and (idx == 3).sum() == 0
    e = project_device(torch.zeros(0, 4, dtype=torch.float64, device="cuda"), np.zeros(3))
    assert (e["depth"] == 2057.701).all() and (e["index"] == -1).all()
