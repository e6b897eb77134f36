"""Pin the CPU oracle to the reference's own outputs (tests/golden, made by oracle/gen_golden.py)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import golden_inputs as GI
from oracle import sampling_ref as S
from oracle import scorenet_ref as R
from oracle.gen_golden import CIRCLE_MODS, MERGE_CASES
from sdp.weights import get_sigmas_np, synthetic_state_dict

ORACLE_THREADS = min(8, os.cpu_count() or 1)


@pytest.fixture(autouse=True)
def _oracle_threads():
    """The torch-CPU oracle's float32 convs round by their thread split: these checks (1e-6 of max) hold at the
    thread count they were pinned with, whatever an earlier test of the session left set (an in-process
    world-1 sampler run sets 1 thread)."""
    prev = torch.get_num_threads()
    torch.set_num_threads(ORACLE_THREADS)
    yield
    torch.set_num_threads(prev)


def _g(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="module")
def params128():
    return R.to_torch_params(synthetic_state_dict(128))


def test_exist_mask_fixture():
    ex = GI.exist_mask_full()
    assert ex.shape == (64, 1024) and 0.5 < ex.mean() < 0.8


@pytest.mark.parametrize("tag,B,H,W", [("ngf128_b2_64x256", 2, 64, 256), ("ngf128_b1_64x1024", 1, 64, 1024)])
def test_scorenet_oracle_matches_reference(params128, tag, B, H, W):
    f = _g(f"scorenet_{tag}.npz")
    x = torch.from_numpy(GI.scorenet_input(tag, B, H, W))
    with torch.no_grad():
        out = R.scorenet_forward(params128, x, torch.from_numpy(f["y"])).numpy()
    # same float32 ops in the same order -> bitwise equal on this CPU; allow 1e-6 of max
    for b in range(B):
        assert np.abs(out[b] - f["out"][b]).max() <= 1e-6 * np.abs(f["out"][b]).max()


def test_ops_oracle_matches_reference():
    import torch.nn.functional as F
    from sdp.weights import synthetic_param
    f = _g("ops_small.npz")
    r = GI.rng("ops")
    x = torch.from_numpy(r.standard_normal((2, 8, 16, 64)).astype(np.float32))
    xs = torch.from_numpy(r.standard_normal((2, 8, 8, 32)).astype(np.float32))

    def P(prefix, names_shapes):
        return {f"{prefix}.{k}": torch.from_numpy(synthetic_param(f"{prefix}.{k}", s)) for k, s in names_shapes}

    got = {}
    p = P("op.inpp", [("alpha", (8,)), ("gamma", (8,)), ("beta", (8,))])
    got["in_pp"] = R.instance_norm_pp(x, p, "op.inpp")
    p = P("op.conv", [("weight", (8, 8, 3, 3)), ("bias", (8,))])
    got["conv3x3_circ"] = R.conv2d(x, p["op.conv.weight"], p["op.conv.bias"])
    for d in (2, 4):
        p = P(f"op.dil{d}", [("weight", (8, 8, 3, 3)), ("bias", (8,))])
        got[f"conv3x3_dil{d}"] = R.conv2d(x, p[f"op.dil{d}.weight"], p[f"op.dil{d}.bias"], dilation=d)
    for k in (3, 1):
        p = P(f"op.cmp{k}", [("conv.weight", (16, 8, k, k)), ("conv.bias", (16,))])
        got[f"convmeanpool{k}"] = R.mean_pool2(R.conv2d(x, p[f"op.cmp{k}.conv.weight"], p[f"op.cmp{k}.conv.bias"],
                                                        circular=False))
    p = P("op.crp", [("convs.0.weight", (8, 8, 3, 3)), ("convs.1.weight", (8, 8, 3, 3))])
    got["crp"] = R.crp(x, p, "op.crp")
    p = P("op.rcu", [(f"{i}_{j}_conv.weight", (8, 8, 3, 3)) for i in (1, 2) for j in (1, 2)])
    got["rcu"] = R.rcu(x, p, "op.rcu", 2)
    p = P("op.msf", [("convs.0.weight", (8, 8, 3, 3)), ("convs.0.bias", (8,)),
                     ("convs.1.weight", (8, 8, 3, 3)), ("convs.1.bias", (8,))])
    got["msf"] = R.msf([x, xs], p, "op.msf", (16, 64))
    names = [("normalize1.alpha", (8,)), ("normalize1.gamma", (8,)), ("normalize1.beta", (8,)),
             ("conv1.weight", (8, 8, 3, 3)), ("conv1.bias", (8,)),
             ("normalize2.alpha", (8,)), ("normalize2.gamma", (8,)), ("normalize2.beta", (8,)),
             ("conv2.conv.weight", (16, 8, 3, 3)), ("conv2.conv.bias", (16,)),
             ("shortcut.conv.weight", (16, 8, 1, 1)), ("shortcut.conv.bias", (16,))]
    got["resblock_down"] = R.residual_block(x, P("op.rbd", names), "op.rbd", 8, 16, True, None)
    for k, v in got.items():
        np.testing.assert_allclose(v.detach().numpy(), f[k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_langevin_oracle_matches_reference():
    f = _g("langevin_step.npz")
    case = GI.merge_case("langevin", 2, 64, 256)
    g = GI.rng("langevin-grad").standard_normal((2, 2, 64, 256)).astype(np.float32) * 3.0
    g[0, 0, 0, :4] = [np.nan, np.inf, -np.inf, 0.0]
    sig = get_sigmas_np()[100:101]
    s = S.step_size_of(6.2e-6, sig[0], sig[-1])
    x1, _ = S.langevin_update(case["x"], g, case["ref"], case["mask"], GI.noise("langevin", 0, g.shape), s, 1.0)
    np.testing.assert_array_equal(x1, f["x1"])  # bit exact (incl. the NaN/inf lanes)


def _after_update(case):
    x = case["x"]
    return (x + (-case["mask"]).astype(np.float32) * (x - case["ref"])).astype(np.float32)


def _final_dc(x, case):
    return (x + (-case["mask"]).astype(np.float32) * (x - case["ref"])).astype(np.float32)


@pytest.mark.parametrize("case_def", MERGE_CASES, ids=[c[0] for c in MERGE_CASES])
def test_kitti_merge_oracle_matches_reference(case_def):
    tag, B, aB, H, W, sigma, kw = case_def
    case = GI.merge_case(tag, B, H, W, **kw)
    f = _g(f"merge_{tag}.npz")
    new, xc = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                            case["fromWorld"], aB, sigma)
    np.testing.assert_allclose(new, f["new"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(_final_dc(xc, case), f["x"], rtol=1e-5, atol=1e-6)
    assert ((new != 0) == (f["new"] != 0)).all()


def test_identity_pose_row_shift():
    """Appendix B.1: with identity poses output row r+1 is fed by source row r, row 0 is empty."""
    case = GI.merge_case("k_b2a2_ident", 2, 64, 256, identity=True, neg_frac=0.0)
    new, _ = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                           case["fromWorld"], 2, 0.5)
    assert (new[:, :, 0] == 0).all()
    assert (new[:, 0, 1:] != 0).mean() > 0.5


@pytest.mark.parametrize("tag,setting", [("a_b7_s05_set7", 7), ("a_b7_s05_set5", 5), ("a_b7_s05_set8", 8)])
def test_allforone_merge_oracle_matches_reference(tag, setting):
    case = GI.merge_case(tag, 7, 64, 256)
    f = _g(f"merge_{tag}.npz")
    cc = 1 / (1 / 1) if setting == 5 else 0.01   # models/__init__.py:209-212 ramp at L=1, c=0
    new, xc = S.allforone_merge(_after_update(case), case["mask"], case["sky"], case["exist"], CIRCLE_MODS, 7, 0.5,
                                setting, cc)
    np.testing.assert_allclose(new, f["new"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(_final_dc(xc, case), f["x"], rtol=1e-5, atol=1e-6)


def test_allforone9_merge_oracle_matches_reference():
    """Config 3 geometry: target + 8 aux origins (CIRCLE9), setting 7."""
    from oracle.gen_golden import CIRCLE9
    case = GI.merge_case("a_b9_s05_set7", 9, 64, 256)
    f = _g("merge_a_b9_s05_set7.npz")
    new, xc = S.allforone_merge(_after_update(case), case["mask"], case["sky"], case["exist"], CIRCLE9, 9, 0.5, 7,
                                0.01)
    np.testing.assert_allclose(new, f["new"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(_final_dc(xc, case), f["x"], rtol=1e-5, atol=1e-6)


def test_megabatch32_full_width_oracle_matches_reference():
    """Config 4 geometry: one 32-view megabatch at 64x1024 (stored output views only)."""
    case = GI.merge_case("k_b32a32_full", 32, 64, 1024)
    f = _g("merge_k_b32a32_full.npz")
    v = list(f["views"])
    new, xc = S.kitti_merge(_after_update(case), case["mask"], case["sky"], case["exist"], case["toWorld"],
                            case["fromWorld"], 32, 0.5, views=v)
    # 2M points land in each output view: numpy's vs torch's float64 atan2 can differ by an ulp and
    # move a point sitting exactly on a bin edge (measured: 1 of 393,216 values), so this case is
    # graded by the fraction of values outside rtol 1e-5 / atol 1e-6 (<= 1e-5), not by allclose
    bad = lambda a, b: np.mean(np.abs(a - b) > 1e-6 + 1e-5 * np.abs(b))
    assert bad(new[v], f["new"]) <= 1e-5
    assert bad(_final_dc(xc, case)[v], f["x"]) <= 1e-5
    assert np.mean((new[v] != 0) != (f["new"] != 0)) <= 1e-5


def _score_fn(params):
    def score(x, y):
        with torch.no_grad():
            return R.scorenet_forward(params, torch.from_numpy(x), torch.from_numpy(y)).numpy()
    return score


def _noise_feed(tag):
    k = [0]

    def fn(shape):
        n = GI.noise(tag, k[0], shape)
        k[0] += 1
        return n
    return fn


def test_config1_baseline_sampler(params128):
    f = _g("config1_b1_64x256.npz")
    case = GI.merge_case("config1", 1, 64, 256)
    x0 = GI.scorenet_input("config1", 1, 64, 256)
    imgs = S.sampler_baseline(x0, case["ref"], case["mask"], _score_fn(params128), get_sigmas_np()[:1], 5, 6.2e-6,
                              _noise_feed("config1"))
    for k, i in (("step1", 0), ("step5", 4), ("denoised", 5), ("final", 6)):
        np.testing.assert_allclose(imgs[i], f[k], rtol=1e-5, atol=1e-5, err_msg=k)


@pytest.mark.parametrize("tag,setting,fname", [("e2e", 5, "kitti_e2e_b2_64x256.npz"),
                                                ("e2e_set7", 7, "kitti_e2e_set7_b2_64x256.npz")])
def test_kitti_sampler_end_to_end(params128, tag, setting, fname):
    """oracle sampler_kitti == the reference kitti loop; setting 7 pins the cc ramp
    (KITTISampling.py:106-109)."""
    f = _g(fname)
    case = GI.merge_case(tag, 2, 64, 256)
    x0 = GI.scorenet_input(tag, 2, 64, 256)
    images, _, _ = S.sampler_kitti(x0, case["ref"], case["mask"], case["sky"], 2, setting, 10, _score_fn(params128),
                                   get_sigmas_np()[229:232], case["fromWorld"], case["toWorld"], 2, 2, 6.2e-6,
                                   case["exist"], _noise_feed(tag))
    assert len(images) == 3
    np.testing.assert_allclose(images[0], f["new"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(images[1], f["new2"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(images[2], f["final"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("setting,min_step", [(5, 0), (7, 1)])
def test_allforone_sampler_end_to_end(params128, setting, min_step):
    """oracle sampler_allforone == the reference AllForOne loop (models/__init__.py:112-602):
    the setting-5 cc ramp at L=3, the level-0 shared images, denoise and final consistency."""
    from oracle.gen_golden import CIRCLE_MODS
    tag = f"a_e2e_set{setting}"
    f = _g(f"allforone_e2e_set{setting}_b3_64x256.npz")
    case = GI.merge_case(tag, 3, 64, 256)
    x0 = GI.scorenet_input(tag, 3, 64, 256)
    images, _, shared = S.sampler_allforone(x0, case["ref"], case["mask"], case["sky"], min_step, setting,
                                            _score_fn(params128), get_sigmas_np()[229:232], np.array(CIRCLE_MODS[:3]),
                                            3, 2, 6.2e-6, case["exist"], _noise_feed(tag))
    assert len(images) == 3 and len(shared) == (2 if min_step == 0 else 0)
    assert (f["new"] != 0).mean() > 0.3          # the merge populated the views
    for got, k in zip(images + shared, ("new", "new2", "final", "shared0", "shared1")):
        np.testing.assert_allclose(got, f[k], rtol=1e-5, atol=1e-5, err_msg=k)


def dsm_case(H, W, B, tag="dsm"):
    """Inputs of oracle/gen_golden.py gen_dsm (same generator stream)."""
    r = GI.rng(tag)
    X = torch.from_numpy(r.random((B, 2, H, W)).astype(np.float32))
    noise = torch.from_numpy(r.standard_normal((B, 2, H, W)).astype(np.float32))
    mask = torch.from_numpy((r.random((B, 2, H, W)) > 0.3).astype(np.float32))
    labels = torch.tensor([3, 200][:B])
    return X, noise, mask, labels


def test_dsm_loss_and_gradients_oracle_matches_reference(params128):
    """The oracle's autograd DSM loss/gradients reproduce the reference module's loss.backward()."""
    f = _g("dsm_ngf128_b2_64x128.npz")
    X, noise, mask, labels = dsm_case(64, 128, 2)
    noise = noise * params128["sigmas"][labels].view(2, 1, 1, 1)
    loss, scores, grads = R.dsm_loss_and_grads(params128, X + noise, noise, mask, labels)
    assert abs(loss.item() - float(f["loss"])) <= 1e-5 * abs(float(f["loss"]))
    assert np.abs(scores.numpy() - f["scores"]).max() <= 1e-6 * np.abs(f["scores"]).max()
    keys = [str(k) for k in f["grad_keys"]]
    assert set(keys) == set(grads)
    for k, gn in zip(keys, f["grad_norms"]):
        assert abs(grads[k].norm().item() - gn) <= 1e-4 * gn + 1e-6, k


@pytest.mark.parametrize("tag", sorted(GI.PROJECTION_CASES))
def test_projection_oracle_matches_reference(tag):
    """oracle/projection_ref.py == datasets/lidar_utils.py:point_cloud_to_range_image, bit for bit."""
    from oracle import projection_ref as PR
    n, origin = GI.PROJECTION_CASES[tag]
    f = _g(f"projection_{tag}.npz")
    d, inten, obf, _, sky, idx = PR.point_cloud_to_range_image(GI.projection_cloud(tag, n), np.array(origin), True)
    assert np.array_equal(d, f["depth"])
    assert np.array_equal(inten.astype(np.float32), f["intensity"])
    assert np.array_equal(obf, f["obf"]) and np.array_equal(sky, f["sky"])
    assert np.array_equal(idx.astype(np.int32), f["index"])
