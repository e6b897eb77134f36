"""HIP path vs the reference's golden outputs and the CPU oracle (MI355X only).

Tolerances (stated once, used below):
  * score net, fp32x3 (3-pass bf16 split MFMA): max|err| <= 1e-4 * max|ref| per image
  * score net, fp32 (exact fp32 MFMA):           max|err| <= 2e-5 * max|ref| per image
  * Langevin update: bit-exact (same float32 ops and order, injected noise); the update fused
    into the score net's last kernel: bit-identical to the two-call form
  * merge (exact mask and bins, ties excluded): the oracle flags the pixels whose
    result a float-rounding perturbation of the projection can change (a point within rounding of a
    bin edge or of the depth filter, a nearest-depth tie, a controlled-average branch on its edge;
    oracle/sampling_ref.py flag_cells); everywhere else the zero pattern must agree exactly and the
    new images / corrected x within rtol 1e-5, atol 2e-6 -- no fraction of mismatches allowed.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import golden_inputs as GI
from oracle import sampling_ref as S
from oracle.gen_golden import CIRCLE_MODS, MERGE_CASES

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _g(name):
    return np.load(os.path.join(GOLDEN, name))


def _net(W, precision="fp32x3", H=64):
    from sdp.scorenet import ScoreNet
    return ScoreNet(H=H, W=W, precision=precision).load_synthetic()


@pytest.fixture(scope="module")
def net256():
    return _net(256)


def _rel_err(out, ref):
    return max(np.abs(out[b] - ref[b]).max() / np.abs(ref[b]).max() for b in range(ref.shape[0]))


@pytest.mark.parametrize("precision,tol", [("fp32x3", 1e-4), ("fp32", 2e-5)])
@pytest.mark.parametrize("tag,B,H,W", [("ngf128_b2_64x256", 2, 64, 256), ("ngf128_b1_64x1024", 1, 64, 1024)])
def test_scorenet_matches_reference_golden(precision, tol, tag, B, H, W):
    f = _g(f"scorenet_{tag}.npz")
    net = _net(W, precision)
    x = torch.from_numpy(GI.scorenet_input(tag, B, H, W)).to(DEV)
    out = net(x, torch.from_numpy(f["y"]).to(DEV)).cpu().numpy()
    assert np.isfinite(out).all()
    err = _rel_err(out, f["out"])
    print(f"{precision} {tag}: max err / max|ref| = {err:.3e}")
    assert err <= tol


def test_scorenet_batch_invariance_and_oracle(net256):
    """B=4 with mixed labels == per-image results; also vs the torch-CPU oracle."""
    from oracle import scorenet_ref as R
    from sdp.weights import synthetic_state_dict
    x = torch.from_numpy(GI.scorenet_input("b4", 4, 64, 256))
    y = torch.tensor([0, 57, 200, 231])
    out4 = net256(x.to(DEV), y.to(DEV)).cpu().numpy()
    for b in range(4):
        o1 = net256(x[b:b + 1].to(DEV), y[b:b + 1].to(DEV)).cpu().numpy()
        np.testing.assert_array_equal(o1[0], out4[b])  # no cross-image coupling, deterministic
    with torch.no_grad():
        ref = R.scorenet_forward(R.to_torch_params(synthetic_state_dict(128)), x, y).numpy()
    assert _rel_err(out4, ref) <= 1e-4


def test_langevin_step_bit_exact():
    from sdp import _lib
    f = _g("langevin_step.npz")
    case = GI.merge_case("langevin", 2, 64, 256)
    g = GI.rng("langevin-grad").standard_normal((2, 2, 64, 256)).astype(np.float32) * 3.0
    g[0, 0, 0, :4] = [np.nan, np.inf, -np.inf, 0.0]
    sig = __import__("sdp").get_sigmas_np()[100:101]
    s = S.step_size_of(6.2e-6, sig[0], sig[-1])
    ns = np.float32(np.sqrt(np.float32(s * np.float32(2))))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    x, gg, ref, mask = t(case["x"]), t(g), t(case["ref"]), t(case["mask"])
    noise = t(GI.noise("langevin", 0, g.shape))
    lik = torch.empty_like(x)
    absmax = torch.zeros(1, dtype=torch.int32, device=DEV)
    _lib.check(_lib.lib().sdp_langevin_step(x.data_ptr(), gg.data_ptr(), ref.data_ptr(), mask.data_ptr(),
                                            noise.data_ptr(), 0, 0, float(s), float(ns), 1.0, 0, 2, 2, 64 * 256,
                                            lik.data_ptr(), absmax.data_ptr(), _lib.stream()))
    np.testing.assert_array_equal(x.cpu().numpy(), f["x1"])
    x1 = f["x1"][:, 0]
    want = np.abs(x1[np.isfinite(x1)]).max() if not np.isnan(x1).any() else None
    if want is not None:
        assert absmax.cpu().view(torch.float32).item() == want


def test_philox_noise_statistics():
    from sdp import _lib
    n = 2 * 2 * 64 * 1024
    x = torch.zeros(2, 2, 64 * 1024, device=DEV)
    g = torch.zeros_like(x)
    ref = torch.zeros_like(x)
    mask = torch.zeros(2, 2, 64 * 1024, dtype=torch.int32, device=DEV)
    _lib.check(_lib.lib().sdp_langevin_step(x.data_ptr(), g.data_ptr(), ref.data_ptr(), mask.data_ptr(), None, 1234,
                                            0, 0.0, 1.0, 1.0, 1, 2, 2, 64 * 1024, None, None, _lib.stream()))
    v = x.cpu().numpy().reshape(-1)
    assert abs(v.mean()) < 0.01 and abs(v.std() - 1) < 0.01
    assert len(np.unique(v)) > 0.99 * n
    # the stream itself: Philox4x32-10 + Box-Muller restated in numpy (oracle/philox_ref.py);
    # device __logf/__sincosf vs numpy float32 log/sin/cos
    from oracle import philox_ref
    want = philox_ref.normal(1234, 0, n)
    assert np.abs(v - want).max() <= 2e-5 * np.abs(want).max()


def test_philox_view_shard_draws_the_single_process_stream():
    """A rank holding views [2, 4) of a 4-view megabatch (counter offset 2 views) draws exactly
    the noise the single-process call applies to those views (sdp/sampling.py _Stepper)."""
    from sdp import _lib
    HW = 64 * 1024

    def run(B, offset):
        x = torch.zeros(B, 2, HW, device=DEV)
        z = torch.zeros_like(x)
        m = torch.zeros(B, 2, HW, dtype=torch.int32, device=DEV)
        _lib.check(_lib.lib().sdp_langevin_step(x.data_ptr(), z.data_ptr(), z.data_ptr(), m.data_ptr(), None, 77,
                                                offset, 0.0, 1.0, 1.0, 1, B, 2, HW, None, None, _lib.stream()))
        return x.cpu().numpy()

    per_view4 = 2 * HW // 4
    full = run(4, 3 * 4 * per_view4)            # step 3 of the single-process run
    part = run(2, 3 * 4 * per_view4 + 2 * per_view4)
    np.testing.assert_array_equal(part, full[2:])


@pytest.mark.parametrize("noise_kind", ["philox", "injected"])
def test_fused_forward_langevin_bit_identical(net256, noise_kind):
    """sdp_net_forward_langevin (update in the end_conv epilogue) == sdp_net_forward followed by
    sdp_langevin_step, bit for bit: x, lik, max|x[:,0]| and the scores; Philox at a nonzero
    counter, or an injected noise buffer."""
    from sdp import _lib
    B, H, W = 2, 64, 256
    case = GI.merge_case("langevin", B, H, W)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    x0, ref, mask = t(case["x"]), t(case["ref"]), t(case["mask"])
    y = torch.tensor([3, 150], device=DEV)
    noise = t(GI.noise("fused", 0, (B, 2, H, W))) if noise_kind == "injected" else None
    sig = __import__("sdp").get_sigmas_np()
    s = S.step_size_of(6.2e-6, sig[150], sig[-1])
    ns = np.float32(np.sqrt(np.float32(s * np.float32(2))))
    seed, offset = 4321, 7 * B * 2 * H * W // 4

    x_a = x0.clone()
    g_a = net256(x_a, y)
    lik_a = torch.empty_like(x_a)
    am_a = torch.zeros(1, dtype=torch.int32, device=DEV)
    _lib.check(_lib.lib().sdp_langevin_step(x_a.data_ptr(), g_a.data_ptr(), ref.data_ptr(), mask.data_ptr(),
                                            _lib.ptr(noise), seed, offset, float(s), float(ns), 0.7, 1, B, 2, H * W,
                                            lik_a.data_ptr(), am_a.data_ptr(), _lib.stream()))
    x_b = x0.clone()
    lik_b = torch.empty_like(x_b)
    am_b = torch.zeros(1, dtype=torch.int32, device=DEV)
    g_b = torch.empty_like(x_b)
    net256.forward_langevin(x_b, y, ref, mask, noise, seed, offset, float(s), float(ns), 0.7, True, lik_b, am_b, g_b)
    torch.testing.assert_close(g_b, g_a, rtol=0, atol=0)
    torch.testing.assert_close(x_b, x_a, rtol=0, atol=0)
    torch.testing.assert_close(lik_b, lik_a, rtol=0, atol=0)
    assert am_b.item() == am_a.item() != 0
    # without the optional outputs the update is the same
    x_c = x0.clone()
    net256.forward_langevin(x_c, y, ref, mask, noise, seed, offset, float(s), float(ns), 0.7, True, None, None)
    torch.testing.assert_close(x_c, x_a, rtol=0, atol=0)


def test_split_forward_is_bit_identical(net256):
    """sdp_net_set_split: 1, 2, 3 and 4 part-batch streams give the same scores and the same fused
    Langevin update, bit for bit (B=5: uneven parts)."""
    from sdp import _lib
    B, H, W = 5, 64, 256
    case = GI.merge_case("split", B, H, W)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    x0, ref, mask = t(case["x"]), t(case["ref"]), t(case["mask"])
    y = torch.tensor([0, 17, 99, 150, 231], device=DEV)
    outs = []
    try:
        for ways in (1, 2, 3, 4):
            net256.set_split(ways)
            g = net256(x0, y)
            x = x0.clone()
            lik = torch.empty_like(x)
            am = torch.zeros(1, dtype=torch.int32, device=DEV)
            net256.forward_langevin(x, y, ref, mask, None, 5, 1234, 1e-5, 4e-3, 0.5, True, lik, am)
            outs.append((g.cpu(), x.cpu(), lik.cpu(), am.item()))
    finally:
        net256.set_split(0)
    for g, x, lik, am in outs[1:]:
        torch.testing.assert_close(g, outs[0][0], rtol=0, atol=0)
        torch.testing.assert_close(x, outs[0][1], rtol=0, atol=0)
        torch.testing.assert_close(lik, outs[0][2], rtol=0, atol=0)
        assert am == outs[0][3]
    with pytest.raises(RuntimeError):
        _lib.check(_lib.lib().sdp_net_set_split(net256._h, 5), "set_split")


def test_sampler_fused_path_equals_two_call_path(net256):
    """The samplers take the fused path with libsdp's ScoreNet; hiding forward_langevin (a plain
    callable) gives the two-call path: same images, bit for bit (Philox noise, verbose reports)."""
    from sdp.sampling import anneal_Langevin_dynamics_inpainting
    case = GI.merge_case("langevin", 2, 64, 256)
    sig = __import__("sdp").get_sigmas_np()[[0, 40, 231]]

    def run(scorenet):
        x = torch.from_numpy(case["x"]).to(DEV)
        imgs, _ = anneal_Langevin_dynamics_inpainting(x, torch.from_numpy(case["ref"]), torch.from_numpy(case["mask"]),
                                                      scorenet, sig, n_steps_each=2, verbose=True, seed=99)
        return [i.numpy() for i in imgs]

    fused = run(net256)
    plain = run(lambda x, y: net256(x, y))
    assert len(fused) == len(plain)
    for a, b in zip(fused, plain):
        np.testing.assert_array_equal(a, b)


def _after_update(case):
    x = case["x"]
    return (x + (-case["mask"]).astype(np.float32) * (x - case["ref"])).astype(np.float32)


def _final_dc(x, case):
    return (x + (-case["mask"]).astype(np.float32) * (x - case["ref"])).astype(np.float32)


def _gpu_merge(case, aB, sigma, setting, allowance, cc, origins=None, too_high=None):
    from sdp.merge import Merger
    B, _, H, W = case["x"].shape
    x = torch.from_numpy(_after_update(case)).to(DEV)
    kw = dict(origins=origins) if origins is not None else dict(toWorld=torch.from_numpy(case["toWorld"]),
                                                                 fromWorld=torch.from_numpy(case["fromWorld"]))
    m = Merger(B, aB, H, W, DEV, torch.from_numpy(case["exist"]), torch.from_numpy(case["sky"]),
               torch.from_numpy(case["mask"]), **kw)
    absmax = torch.tensor([np.abs(_after_update(case)[:, 0]).max()], dtype=torch.float32).view(torch.int32).to(DEV)
    if too_high is not None:
        absmax = torch.tensor([too_high], dtype=torch.float32).view(torch.int32).to(DEV)
    new = torch.empty(B, 2, H, W, device=DEV)
    m(x, sigma, setting, allowance, cc, absmax, new)
    return new.cpu().numpy(), x.cpu().numpy()


def _close_frac(a, b, rtol=1e-5, atol=2e-6):
    return np.mean(np.abs(a - b) > atol + rtol * np.abs(b))


def _assert_merge_exact(got_new, want_new, got_x, want_x, flagged, what=""):
    """SURVEY 8(c) merge gate: outside the pixels the oracle flags (oracle/sampling_ref.py flag_cells:
    a point within float rounding of a bin edge or of the depth filter, a nearest-depth tie, a
    controlled-average branch on its edge) the zero pattern (mask / bins) must agree exactly and every
    value within float rounding (rtol 1e-5, atol 2e-6: float64 sums in another order, the device's float32
    exp2); no fraction of mismatches is allowed.  Prints the flagged count."""
    fl = np.broadcast_to(np.asarray(flagged)[:, None], got_new.shape)
    ok = ~fl
    bad_new = (np.abs(got_new - want_new) > 2e-6 + 1e-5 * np.abs(want_new)) & ok
    bad_zero = ((got_new != 0) != (want_new != 0)) & ok
    bad_x = (np.abs(got_x - want_x) > 2e-6 + 1e-5 * np.abs(want_x)) & ok
    print(f"merge {what}: {int(np.asarray(flagged).sum())} of {np.asarray(flagged).size} pixels flagged, "
          f"mismatches outside them: values {int(bad_new.sum())}, zero pattern {int(bad_zero.sum())}, x {int(bad_x.sum())}")
    assert np.asarray(flagged).mean() <= 2e-3, "the oracle flags too much to grade"
    assert not bad_zero.any(), np.argwhere(bad_zero)[:8]
    assert not bad_new.any(), np.argwhere(bad_new)[:8]
    assert not bad_x.any(), np.argwhere(bad_x)[:8]


@pytest.mark.parametrize("case_def", MERGE_CASES, ids=[c[0] for c in MERGE_CASES])
def test_kitti_merge_matches_reference_golden(case_def):
    tag, B, aB, H, W, sigma, kw = case_def
    case = GI.merge_case(tag, B, H, W, **kw)
    f = _g(f"merge_{tag}.npz")
    new, xc = _gpu_merge(case, aB, sigma, 5, 10, 0.01)
    _, _, fl = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                             case["fromWorld"], aB, sigma, flags=True)
    _assert_merge_exact(new, f["new"], _final_dc(xc, case), f["x"], fl, tag)


def test_kitti_merge_nan_points_match_oracle():
    """NaN codes and intensities in the merged views (a NaN x[:, 0] reaches the merge as a NaN world point; the
    Langevin golden carries NaN/inf lanes): the reference's numpy projection gives NaN bins, which fail its
    range test, so such a point lands nowhere (KITTISampling.py:244-251), while a NaN intensity poisons the
    sums of the cell it lands in.  The device must not turn a NaN bin into a cell index (a float64 -> int
    conversion of NaN is 0 on gfx950), and the NaN pattern of the outputs must be the oracle's."""
    import warnings
    from sdp.merge import Merger
    tag, B, aB, H, W, sigma, kw = MERGE_CASES[0]
    case = GI.merge_case(tag, B, H, W, **kw)
    x = _after_update(case)
    r = np.random.default_rng(5)
    idx = r.choice(H * W, 40, replace=False)
    x.reshape(B, 2, -1)[:, 0, idx[:20]] = np.nan
    x.reshape(B, 2, -1)[:, 1, idx[20:]] = np.nan
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want_new, want_x, fl = S.kitti_merge(x, case["mask"], case["sky"], case["exist"], case["toWorld"],
                                             case["fromWorld"], aB, sigma, flags=True)
    xg = torch.from_numpy(x).to(DEV)
    m = Merger(B, aB, H, W, DEV, torch.from_numpy(case["exist"]), torch.from_numpy(case["sky"]),
               torch.from_numpy(case["mask"]), toWorld=torch.from_numpy(case["toWorld"]),
               fromWorld=torch.from_numpy(case["fromWorld"]))
    absmax = torch.tensor([np.nan], dtype=torch.float32).view(torch.int32).to(DEV)   # max|x| of the oracle: NaN
    new = torch.empty(B, 2, H, W, device=DEV)
    m(xg, sigma, 5, 10, 0.01, absmax, new)
    got_new, got_x = new.cpu().numpy(), xg.cpu().numpy()
    ok = ~np.broadcast_to(fl[:, None], got_new.shape)
    assert np.isnan(want_new).any() and np.isnan(want_x).any()
    assert np.array_equal(np.isnan(got_new) & ok, np.isnan(want_new) & ok)
    assert np.array_equal(np.isnan(got_x) & ok, np.isnan(want_x) & ok)
    fin = ok & ~np.isnan(want_new)
    assert np.all(np.abs(got_new - want_new)[fin] <= 2e-6 + 1e-5 * np.abs(want_new)[fin])
    finx = ok & ~np.isnan(want_x)
    assert np.all(np.abs(got_x - want_x)[finx] <= 2e-6 + 1e-5 * np.abs(want_x)[finx])


@pytest.mark.parametrize("tag,setting", [("a_b7_s05_set7", 7), ("a_b7_s05_set5", 5), ("a_b7_s05_set8", 8)])
def test_allforone_merge_matches_reference_golden(tag, setting):
    """Settings 5 (cc ramp), 7 (controlled average) and 8 (controlled, allowance 5:
    models/__init__.py:469-470)."""
    from sdp.merge import allforone_origins
    case = GI.merge_case(tag, 7, 64, 256)
    f = _g(f"merge_{tag}.npz")
    cc = 1.0 if setting == 5 else 0.01
    allowance = 5 if setting >= 8 else 10
    new, xc = _gpu_merge(case, 7, 0.5, setting, allowance, cc, origins=allforone_origins(CIRCLE_MODS))
    _, _, fl = S.allforone_merge(_after_update(case), case["mask"], case["sky"], case["exist"], CIRCLE_MODS, 7, 0.5,
                                 setting, cc, flags=True)
    _assert_merge_exact(new, f["new"], _final_dc(xc, case), f["x"], fl, tag)


def test_allforone9_merge_matches_reference_golden():
    """BASELINE config 3 geometry: target + 8 aux origins in one megabatch, setting 7."""
    from oracle.gen_golden import CIRCLE9
    from sdp.merge import allforone_origins
    case = GI.merge_case("a_b9_s05_set7", 9, 64, 256)
    f = _g("merge_a_b9_s05_set7.npz")
    new, xc = _gpu_merge(case, 9, 0.5, 7, 10, 0.01, origins=allforone_origins(CIRCLE9))
    _, _, fl = S.allforone_merge(_after_update(case), case["mask"], case["sky"], case["exist"], CIRCLE9, 9, 0.5, 7,
                                 0.01, flags=True)
    _assert_merge_exact(new, f["new"], _final_dc(xc, case), f["x"], fl, "a_b9_s05_set7")


def test_megabatch32_full_width_matches_reference_golden():
    """BASELINE config 4 geometry: one 32-view megabatch at the full 64x1024 (views 0/17/31 stored)."""
    case = GI.merge_case("k_b32a32_full", 32, 64, 1024)
    f = _g("merge_k_b32a32_full.npz")
    v = list(f["views"])
    new, xc = _gpu_merge(case, 32, 0.5, 5, 10, 0.01)
    _, _, fl = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                             case["fromWorld"], 32, 0.5, views=v, flags=True)
    _assert_merge_exact(new[v], f["new"], _final_dc(xc, case)[v], f["x"], fl[v], "k_b32a32_full")


def test_merge_too_high_disables_correction():
    case = GI.merge_case("k_b4a4_s05", 4, 64, 256)
    _, xc = _gpu_merge(case, 4, 0.5, 5, 10, 0.01, too_high=9.0)   # 9*6/1 > 50
    np.testing.assert_array_equal(xc, _after_update(case))


def test_merge_megabatch8_w512_vs_oracle():
    """aB=8 (more views than any golden) against the oracle restatement."""
    case = GI.merge_case("big8", 8, 64, 512)
    new, xc = _gpu_merge(case, 8, 0.7, 5, 10, 0.01)
    on, ox, fl = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                               case["fromWorld"], 8, 0.7, flags=True)
    _assert_merge_exact(new, on, xc, ox, fl, "big8")


@pytest.mark.parametrize("aB,W", [(16, 256), (32, 128)])
def test_merge_large_megabatch_vs_oracle(aB, W):
    """Megabatches of 16 / 32 views (the BASELINE config-4 megabatch is 32): the binned
    accumulation sums many 4096-record segments per destination row, against the oracle."""
    case = GI.merge_case(f"big{aB}", aB, 64, W)
    new, xc = _gpu_merge(case, aB, 0.7, 5, 10, 0.01)
    on, ox, fl = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                               case["fromWorld"], aB, 0.7, flags=True)
    _assert_merge_exact(new, on, xc, ox, fl, f"big{aB}")


def test_merge_near_the_output_view_limit_vs_oracle():
    """140 output views (35 megabatches of 4) at 64 x 32: the scatter's LDS holds the tile cursors
    (140 x 114 x 4 B) AND the scanned block totals (>= 4 K of them) -- past the old 64 KB check
    (ADVICE r05), under the 96 KB attribute set per device; every view against the oracle."""
    case = GI.merge_case("many140", 140, 64, 32)
    new, xc = _gpu_merge(case, 4, 0.7, 5, 10, 0.01)
    on, ox, fl = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                               case["fromWorld"], 4, 0.7, flags=True)
    _assert_merge_exact(new, on, xc, ox, fl, "140 views")


def _noise_feed(tag):
    k = [0]

    def fn(shape):
        n = torch.from_numpy(GI.noise(tag, k[0], shape))
        k[0] += 1
        return n
    return fn


def test_config1_baseline_sampler_matches_golden(net256):
    from sdp.sampling import anneal_Langevin_dynamics_inpainting
    from sdp.weights import get_sigmas_np
    f = _g("config1_b1_64x256.npz")
    case = GI.merge_case("config1", 1, 64, 256)
    x0 = torch.from_numpy(GI.scorenet_input("config1", 1, 64, 256)).to(DEV)
    imgs, _ = anneal_Langevin_dynamics_inpainting(
        x0, torch.from_numpy(case["ref"]).to(DEV), torch.from_numpy(case["mask"]).to(DEV), net256,
        get_sigmas_np()[:1], n_steps_each=5, step_lr=6.2e-6, denoise=True, verbose=False, grad_ref=1,
        noise_fn=_noise_feed("config1"), keep_all=True)
    for k, i in (("step1", 0), ("step5", 4), ("denoised", 5), ("final", 6)):
        got = imgs[i].numpy()
        assert np.abs(got - f[k]).max() <= 1e-4 * np.abs(f[k]).max(), k


@pytest.mark.parametrize("tag,setting,fname", [("e2e", 5, "kitti_e2e_b2_64x256.npz"),
                                                ("e2e_set7", 7, "kitti_e2e_set7_b2_64x256.npz")])
def test_kitti_sampler_end_to_end_matches_golden(net256, tag, setting, fname):
    """The kitti loop vs the reference-generated golden; setting 7 pins the cc ramp
    (KITTISampling.py:106-109, sdp/sampling.py ramp)."""
    from sdp.sampling import anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti as samp
    from sdp.weights import get_sigmas_np
    f = _g(fname)
    case = GI.merge_case(tag, 2, 64, 256)
    x0 = torch.from_numpy(GI.scorenet_input(tag, 2, 64, 256)).to(DEV)
    t = lambda a: torch.from_numpy(a).to(DEV)
    images, _, _ = samp(x0, t(case["ref"]), t(case["mask"]), t(case["sky"]), None, 2, setting, 10, net256,
                        get_sigmas_np()[229:232], t(case["fromWorld"].reshape(2, 1, 4, 4)),
                        t(case["toWorld"].reshape(2, 1, 4, 4)), 2, n_steps_each=2, step_lr=6.2e-6,
                        existMask=t(case["exist"]), denoise=True, verbose=False, grad_ref=1,
                        correlation_coefficient=0.01, noise_fn=_noise_feed(tag))
    assert len(images) == 3
    for got, want in ((images[0].numpy(), f["new"]), (images[1].numpy(), f["new2"]), (images[2].numpy(), f["final"])):
        assert _close_frac(got, want, rtol=1e-4, atol=1e-4 * np.abs(want).max()) <= 1e-3


@pytest.mark.parametrize("setting,min_step", [(5, 0), (7, 1)])
def test_allforone_sampler_end_to_end_matches_golden(net256, setting, min_step):
    """AllForOne loop (models/__init__.py:112-602) vs the reference-generated golden: the setting-5
    cc ramp over L=3 levels, the level-0 shared images, denoise + final consistency."""
    from oracle.gen_golden import CIRCLE_MODS
    from sdp.sampling import anneal_Langevin_dynamics_inpainting_simultaneous_basic as samp
    from sdp.weights import get_sigmas_np
    tag = f"a_e2e_set{setting}"
    f = _g(f"allforone_e2e_set{setting}_b3_64x256.npz")
    case = GI.merge_case(tag, 3, 64, 256)
    x0 = torch.from_numpy(GI.scorenet_input(tag, 3, 64, 256)).to(DEV)
    t = lambda a: torch.from_numpy(a).to(DEV)
    images, _, shared = samp(x0, t(case["ref"]), t(case["mask"]), t(case["sky"]), None, min_step, setting, net256,
                             get_sigmas_np()[229:232], torch.tensor(CIRCLE_MODS[:3]), 3, n_steps_each=2,
                             step_lr=6.2e-6, existMask=t(case["exist"]), denoise=True, verbose=False, grad_ref=1,
                             correlation_coefficient=0.01, noise_fn=_noise_feed(tag))
    assert len(images) == 3 and len(shared) == (2 if min_step == 0 else 0)
    for got, k in zip(images + shared, ("new", "new2", "final", "shared0", "shared1")):
        want = f[k]
        assert _close_frac(got.numpy(), want, rtol=1e-4, atol=1e-4 * np.abs(want).max()) <= 1e-3, k



def _nccl_world1():
    import socket
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    return dist


def test_merge_absmax_event_orders_only_the_correction_pass():
    """sdp_consistency_merge_ev (multi-rank tooHigh): the merge's correction pass waits
    for the event of the all_reduce(MAX) running on another stream.  The side stream sleeps, then
    raises absmax past tooHigh and all-reduces it (RCCL, world 1): the correction must see the raised
    word (x unchanged); with AbsmaxAllReduce and no delay the result is bit-identical to the blocking
    merge."""
    from sdp.merge import AbsmaxAllReduce, Merger
    dist = _nccl_world1()
    try:
        case = GI.merge_case("k_b4a4_s05", 4, 64, 256)
        B, _, H, W = case["x"].shape
        mk = lambda: Merger(B, 4, H, W, DEV, torch.from_numpy(case["exist"]), torch.from_numpy(case["sky"]),
                            torch.from_numpy(case["mask"]), toWorld=torch.from_numpy(case["toWorld"]),
                            fromWorld=torch.from_numpy(case["fromWorld"]))
        low = np.abs(_after_update(case)[:, 0]).max()
        bits = lambda v: torch.tensor([v], dtype=torch.float32).view(torch.int32).to(DEV)
        # 1. ordering: the raised word arrives late on the side stream
        m = mk()
        x = torch.from_numpy(_after_update(case)).to(DEV)
        absmax = bits(low)
        comm, ev = torch.cuda.Stream(), torch.cuda.Event()
        comm.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(comm):
            torch.cuda._sleep(100_000_000)
            absmax.copy_(bits(9.0))                       # 9*6/1 > 50: tooHigh
            dist.all_reduce(absmax, op=dist.ReduceOp.MAX)
            ev.record()
        m(x, 0.5, 5, 10, 0.01, absmax, None, absmax_event=ev)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(x.cpu().numpy(), _after_update(case))
        # 2. AbsmaxAllReduce + the event form == the blocking merge, bit for bit
        new_ref, x_ref = _gpu_merge(case, 4, 0.5, 5, 10, 0.01)
        m = mk()
        x = torch.from_numpy(_after_update(case)).to(DEV)
        absmax = bits(low)
        new = torch.empty(B, 2, H, W, device=DEV)
        ev = AbsmaxAllReduce()(absmax)
        m(x, 0.5, 5, 10, 0.01, absmax, new, absmax_event=ev)
        np.testing.assert_array_equal(x.cpu().numpy(), x_ref)
        np.testing.assert_array_equal(new.cpu().numpy(), new_ref)
        assert not np.array_equal(x_ref, _after_update(case))   # (the correction did run)
    finally:
        dist.destroy_process_group()
