"""BASELINE config 4 on one GPU: what each of the 8 view-split ranks executes.

Under config 4 (Line.yml, one 32-view megabatch, 4 views per GPU) every rank all-gathers the
megabatch and merges all 32 source views into its OWN 4 output views
(``Merger(..., o_begin=4*rank, n_out=4)``, sdp/sampling.py ``_simultaneous``; reference
KITTISampling.py:160-490, where one process merges all 32 outputs).  These tests run that
rank-local path of the HIP merge (o_begin > 0, n_out < n_src) on the device:

  * every 4-view output slice equals the same views of the full n_out=32 merge, bit for bit
    (new images and corrected x), and views 0 / 17 / 31 match the reference-generated
    golden ``merge_k_b32a32_full`` at the merge tolerance of test_gpu_parity.py;
  * an emulation of the 8 ranks on one device -- per-rank fused forward + Langevin update with
    the rank's Philox counters, the all-gather replaced by a shared buffer, 8 rank-local
    Mergers each on its own copy of that buffer, tooHigh as the max over the ranks -- equals
    the single-process 32-view step bit for bit over several merged steps.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import golden_inputs as GI

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N_SRC, PER_RANK, H, W = 32, 4, 64, 1024


@pytest.fixture(scope="module")
def case():
    return GI.merge_case("k_b32a32_full", N_SRC, H, W)


def _merger(case, o_begin, n_out):
    from sdp.merge import Merger
    return Merger(N_SRC, N_SRC, H, W, DEV, torch.from_numpy(case["exist"]), torch.from_numpy(case["sky"]),
                  torch.from_numpy(case["mask"]), toWorld=torch.from_numpy(case["toWorld"]),
                  fromWorld=torch.from_numpy(case["fromWorld"]), o_begin=o_begin, n_out=n_out)


def _after_update(case):
    x = case["x"]
    return (x + (-case["mask"]).astype(np.float32) * (x - case["ref"])).astype(np.float32)


def _absmax(x):
    return torch.tensor([np.abs(x[:, 0]).max()], dtype=torch.float32).view(torch.int32).to(DEV)


def test_rank_local_merge_equals_full_merge_and_golden(case):
    x0 = _after_update(case)
    full_x = torch.from_numpy(x0).to(DEV)
    full_new = torch.empty(N_SRC, 2, H, W, device=DEV)
    _merger(case, 0, N_SRC)(full_x, 0.5, 5, 10, 0.01, _absmax(x0), full_new)
    full_x, full_new = full_x.cpu().numpy(), full_new.cpu().numpy()
    f = np.load(os.path.join(GOLDEN, "merge_k_b32a32_full.npz"))
    golden_views = [int(v) for v in f["views"]]
    seen = {}
    for o_begin in range(0, N_SRC, PER_RANK):
        xr = torch.from_numpy(x0).to(DEV)
        new = torch.empty(PER_RANK, 2, H, W, device=DEV)
        _merger(case, o_begin, PER_RANK)(xr, 0.5, 5, 10, 0.01, _absmax(x0), new)
        xr, new = xr.cpu().numpy(), new.cpu().numpy()
        own = slice(o_begin, o_begin + PER_RANK)
        np.testing.assert_array_equal(new, full_new[own])
        np.testing.assert_array_equal(xr[own], full_x[own])
        # the other views of the rank's buffer are the gathered input, untouched
        np.testing.assert_array_equal(np.delete(xr, np.r_[own], axis=0), np.delete(x0, np.r_[own], axis=0))
        for v in golden_views:
            if o_begin <= v < o_begin + PER_RANK:
                seen[v] = new[v - o_begin]
    assert sorted(seen) == sorted(golden_views)
    got = np.stack([seen[v] for v in golden_views])
    from oracle import sampling_ref as S
    from test_gpu_parity import _assert_merge_exact
    _, _, fl = S.kitti_merge(x0, case["mask"], case["sky"], case["exist"], case["toWorld"], case["fromWorld"], N_SRC,
                             0.5, views=golden_views, flags=True)
    gx = (full_x + (-case["mask"]).astype(np.float32) * (full_x - case["ref"])).astype(np.float32)[golden_views]
    _assert_merge_exact(got, f["new"], gx, f["x"], fl[golden_views], "config-4 rank-local")


def test_eight_rank_viewsplit_emulation_is_bit_identical(case):
    """Three merged Langevin steps (score net + fused update + merge) of the 32-view megabatch:
    one process holding all 32 views vs 8 emulated ranks of 4 views each."""
    from sdp.scorenet import ScoreNet
    from sdp.weights import get_sigmas_np
    net = ScoreNet(H=H, W=W, precision="fp32x3").load_synthetic()
    sig = get_sigmas_np()
    c, seed = 150, 2024
    s = np.float32(6.2e-6) * (np.float32(sig[c]) / np.float32(sig[-1])) ** 2
    ns = np.float32(np.sqrt(np.float32(s * np.float32(2))))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    ref, mask = t(case["ref"]), t(case["mask"])
    per_view4 = 2 * H * W // 4
    y_all = torch.full((N_SRC,), c, dtype=torch.int64, device=DEV)
    y_r = y_all[:PER_RANK]

    # single process: 32 views, one merger over all outputs
    x1 = t(case["x"])
    lik1 = torch.empty_like(x1)
    am1 = torch.zeros(1, dtype=torch.int32, device=DEV)
    m1 = _merger(case, 0, N_SRC)
    # 8 ranks: own views + their own megabatch buffer + their own merger
    R = N_SRC // PER_RANK
    xs = [t(case["x"][r * PER_RANK:(r + 1) * PER_RANK]) for r in range(R)]
    bufs = [torch.empty(N_SRC, 2, H, W, device=DEV) for _ in range(R)]
    ms = [_merger(case, r * PER_RANK, PER_RANK) for r in range(R)]
    liks = [torch.empty_like(xs[0]) for _ in range(R)]
    ams = [torch.zeros(1, dtype=torch.int32, device=DEV) for _ in range(R)]
    for step in range(3):
        offset = step * N_SRC * per_view4                     # _Stepper.offset_stride over the megabatch
        am1.zero_()
        net.forward_langevin(x1, y_all, ref, mask, None, seed, offset, float(s), float(ns), 1.0, True, lik1, am1)
        m1(x1, sig[c], 5, 10, 0.01, am1)
        for r in range(R):
            own = slice(r * PER_RANK, (r + 1) * PER_RANK)
            ams[r].zero_()
            net.forward_langevin(xs[r], y_r, ref[own].contiguous(), mask[own].contiguous(), None, seed,
                                 offset + r * PER_RANK * per_view4, float(s), float(ns), 1.0, True, liks[r], ams[r])
        gathered = torch.cat(xs)                               # all_gather_into_tensor
        am_max = torch.stack(ams).max(dim=0).values            # all_reduce(MAX) of the int32 bit pattern
        for r in range(R):
            own = slice(r * PER_RANK, (r + 1) * PER_RANK)
            bufs[r].copy_(gathered)
            ms[r](bufs[r], sig[c], 5, 10, 0.01, am_max)
            xs[r].copy_(bufs[r][own])
        assert am_max.item() == am1.item()
        got = torch.cat(xs)
        torch.testing.assert_close(got, x1, rtol=0, atol=0, msg=f"step {step}")
        for r in range(R):
            own = slice(r * PER_RANK, (r + 1) * PER_RANK)
            torch.testing.assert_close(liks[r], lik1[own], rtol=0, atol=0)
