"""The merge parity flags (oracle/sampling_ref.py flag_cells, SURVEY 8(c) "exact mask and row/col bins;
ties excluded") checked on CPU against the reference's own merge outputs: asking for flags changes no
result, every pixel where the reference-generated golden differs from the oracle is flagged, and the
flags stay rare (<= 2e-3 of the pixels), so the GPU gate built on them (tests/test_gpu_parity.py
_assert_merge_exact) grades almost every pixel exactly."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import golden_inputs as GI
from oracle import sampling_ref as S
from oracle.gen_golden import CIRCLE9, CIRCLE_MODS, MERGE_CASES


def _after_update(case):
    x = case["x"]
    return (x + (-case["mask"]).astype(np.float32) * (x - case["ref"])).astype(np.float32)


def _final_dc(x, case):
    return (x + (-case["mask"]).astype(np.float32) * (x - case["ref"])).astype(np.float32)


def _check(new, xc, fl, f, case, v=None):
    fx = _final_dc(xc, case)
    if v is not None:
        new, fx, fl = new[v], fx[v], fl[v]
    F = np.broadcast_to(fl[:, None], new.shape)
    bad = (np.abs(new - f["new"]) > 1e-6 + 1e-5 * np.abs(f["new"])) | ((new != 0) != (f["new"] != 0))
    badx = np.abs(fx - f["x"]) > 1e-6 + 1e-5 * np.abs(f["x"])
    assert not (bad & ~F).any() and not (badx & ~F).any()
    assert fl.mean() <= 2e-3
    return int(bad.sum())


@pytest.mark.parametrize("case_def", MERGE_CASES, ids=[c[0] for c in MERGE_CASES])
def test_kitti_flags_cover_reference_differences(case_def):
    tag, B, aB, H, W, sigma, kw = case_def
    case = GI.merge_case(tag, B, H, W, **kw)
    args = (_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"], case["fromWorld"], aB, sigma)
    new, xc, fl = S.kitti_merge(*args, flags=True)
    n0, x0 = S.kitti_merge(*args)
    np.testing.assert_array_equal(new, n0)
    np.testing.assert_array_equal(xc, x0)
    _check(new, xc, fl, np.load(os.path.join(GOLDEN, f"merge_{tag}.npz")), case)


@pytest.mark.parametrize("tag,setting,mods,aB", [("a_b7_s05_set7", 7, CIRCLE_MODS, 7), ("a_b7_s05_set5", 5, CIRCLE_MODS, 7),
                                                 ("a_b7_s05_set8", 8, CIRCLE_MODS, 7), ("a_b9_s05_set7", 7, CIRCLE9, 9)])
def test_allforone_flags_cover_reference_differences(tag, setting, mods, aB):
    case = GI.merge_case(tag, aB, 64, 256)
    cc = 1.0 if setting == 5 else 0.01
    new, xc, fl = S.allforone_merge(_after_update(case), case["mask"], case["sky"], case["exist"], mods, aB, 0.5,
                                    setting, cc, flags=True)
    _check(new, xc, fl, np.load(os.path.join(GOLDEN, f"merge_{tag}.npz")), case)


def test_megabatch32_flags_cover_the_bin_edge_point():
    """The one value of 393,216 where numpy's and torch's float64 atan2 put a point on different sides of
    a bin edge (test_oracle_golden.py) is a flagged pixel."""
    case = GI.merge_case("k_b32a32_full", 32, 64, 1024)
    f = np.load(os.path.join(GOLDEN, "merge_k_b32a32_full.npz"))
    v = [int(i) for i in f["views"]]
    new, xc, fl = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                                case["fromWorld"], 32, 0.5, views=v, flags=True)
    assert _check(new, xc, fl, f, case, v) >= 1


def test_flags_mark_a_forced_tie():
    """Two source views holding the same scene at the same pose put equal depths in every cell: the
    nearest-depth choice is a tie wherever their intensities differ, and those pixels are flagged."""
    case = GI.merge_case("k_b2a2_full", 2, 64, 256)
    x = _after_update(case)
    x[1] = x[0]
    x[1, 1] += 0.25                                      # same depths, other intensities
    tw = case["toWorld"].copy()
    fw = case["fromWorld"].copy()
    tw[1], fw[1] = tw[0], fw[0]
    sky = case["sky"].copy()
    sky[1] = sky[0]
    ex = case["exist"].copy()
    _, _, fl = S.kitti_merge(x, case["mask"], sky, ex, tw, fw, 2, 0.5, setting=1, flags=True)
    assert fl.mean() > 0.2                               # most covered pixels hold a two-way tie
