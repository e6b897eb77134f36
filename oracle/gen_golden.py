"""ORACLE fixture generator -- runs the REFERENCE code (this container only) and writes the
expected outputs under ``tests/golden/``.

Usage (from the repo root; the reference tree is read-only, so no bytecode):
    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py

It imports ``/root/reference/LiDARGen/{models,losses}`` with one harness shim
(``Tensor.cuda = identity``, because ncsnv2.py:495 hard-codes ``.cuda()`` and this
container's torch is CPU-only).  Inputs come from ``oracle/golden_inputs.py`` (seeded),
weights from ``sdp.weights.synthetic_state_dict`` (seeded), so the fixtures hold only the
reference's outputs.  The reference itself never travels to the GPU box; these files do.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import scipy.ndimage
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/LiDARGen"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd"))

from oracle import golden_inputs as GI  # noqa: E402
from sdp.weights import synthetic_state_dict, synthetic_param, get_sigmas_np  # noqa: E402

OUT = GI.GOLDEN_DIR


def _ref_imports():
    sys.path.insert(0, REF)
    torch.Tensor.cuda = lambda self, *a, **k: self  # harness shim (ncsnv2.py:495)
    import models  # noqa: F401
    from models import layers, normalization  # noqa: F401
    return models


def ns(d):
    n = argparse.Namespace()
    for k, v in d.items():
        setattr(n, k, ns(v) if isinstance(v, dict) else v)
    return n


def model_cfg(ngf, H, W):
    return ns({"data": {"channels": 2, "image_size": H, "image_width": W, "logit_transform": False,
                        "rescaled": False},
               "model": {"sigma_begin": 50, "sigma_end": 0.01, "num_classes": 232, "sigma_dist": "geometric",
                         "normalization": "InstanceNorm++", "nonlinearity": "elu", "ngf": ngf},
               "device": torch.device("cpu")})


def build_net(ngf, H, W):
    from models.ncsnv2 import NCSN_LiDAR_small
    m = NCSN_LiDAR_small(model_cfg(ngf, H, W)).eval()
    sd = synthetic_state_dict(ngf)
    m.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()}, strict=True)
    return m


def save(name, **arrs):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrs)
    print("wrote", path, os.path.getsize(path), "bytes")


def gen_exist():
    """runners/ncsn_runner_kitti_simultaneous.py:527-530 on the reference's data file."""
    ex = np.load(os.path.join(os.path.dirname(REF), "MeasureResults", "existTotalLiDARGenSettings.npy"))
    ex = ex > np.max(ex) / 3
    ex[2:] = scipy.ndimage.binary_erosion(ex[2:], border_value=1, iterations=4)
    np.save(os.path.join(OUT, "exist_mask_64x1024_packed.npy"), np.packbits(ex.reshape(-1)))
    print("exist mask true fraction", ex.mean())


def gen_scorenet():
    with torch.no_grad():
        for tag, B, H, W, labels in [("ngf128_b2_64x256", 2, 64, 256, [0, 231]),
                                     ("ngf128_b1_64x1024", 1, 64, 1024, [100])]:
            m = build_net(128, H, W)
            x = GI.scorenet_input(tag, B, H, W)
            y = torch.tensor(labels, dtype=torch.long)
            out = m(torch.from_numpy(x), y).numpy()
            save(f"scorenet_{tag}.npz", y=np.array(labels, np.int64), out=out)


def _load_synth(mod, prefix):
    sd = {k: torch.as_tensor(synthetic_param(prefix + "." + k, tuple(v.shape))) for k, v in mod.state_dict().items()}
    mod.load_state_dict(sd)
    return mod


def gen_ops():
    """Per-op fixtures on small tensors [2,8,16,64] (layers.py / normalization.py modules)."""
    from models import layers
    from models.normalization import InstanceNorm2dPlus
    torch.manual_seed(0)
    r = GI.rng("ops")
    x = torch.from_numpy(r.standard_normal((2, 8, 16, 64)).astype(np.float32))
    xs = torch.from_numpy(r.standard_normal((2, 8, 8, 32)).astype(np.float32))
    out = {}
    with torch.no_grad():
        out["in_pp"] = _load_synth(InstanceNorm2dPlus(8), "op.inpp")(x)
        out["conv3x3_circ"] = _load_synth(layers.conv3x3(8, 8), "op.conv")(x)
        out["conv3x3_dil2"] = _load_synth(layers.dilated_conv3x3(8, 8, 2), "op.dil2")(x)
        out["conv3x3_dil4"] = _load_synth(layers.dilated_conv3x3(8, 8, 4), "op.dil4")(x)
        out["convmeanpool3"] = _load_synth(layers.ConvMeanPool(8, 16, 3), "op.cmp3")(x)
        out["convmeanpool1"] = _load_synth(layers.ConvMeanPool(8, 16, 1), "op.cmp1")(x)
        out["crp"] = _load_synth(layers.CRPBlock(8, 2, torch.nn.ELU()), "op.crp")(x)
        out["rcu"] = _load_synth(layers.RCUBlock(8, 2, 2, torch.nn.ELU()), "op.rcu")(x.clone())
        out["msf"] = _load_synth(layers.MSFBlock([8, 8], 8), "op.msf")([x, xs], (16, 64))
        out["resblock_down"] = _load_synth(layers.ResidualBlock(8, 16, resample="down", act=torch.nn.ELU(),
                                                                normalization=InstanceNorm2dPlus), "op.rbd")(x)
    save("ops_small.npz", **{k: v.numpy() for k, v in out.items()})


class _NoiseFeed:
    """Replaces torch.randn_like with seeded fixture noise, call by call."""

    def __init__(self, tag):
        self.tag, self.k, self.orig = tag, 0, torch.randn_like

    def __enter__(self):
        def fake(t, *a, **kw):
            n = torch.from_numpy(GI.noise(self.tag, self.k, tuple(t.shape)))
            self.k += 1
            return n
        torch.randn_like = fake
        return self

    def __exit__(self, *exc):
        torch.randn_like = self.orig


def gen_langevin():
    """One plain Langevin update (models/__init__.py:1397-1416) with a stub score."""
    models = _ref_imports()
    B, H, W = 2, 64, 256
    case = GI.merge_case("langevin", B, H, W)
    g = GI.rng("langevin-grad").standard_normal((B, 2, H, W)).astype(np.float32) * 3.0
    g[0, 0, 0, :4] = [np.nan, np.inf, -np.inf, 0.0]

    def stub(x, y):
        return torch.from_numpy(g.copy())

    sig = get_sigmas_np()
    with torch.no_grad(), _NoiseFeed("langevin"):
        imgs, _ = models.anneal_Langevin_dynamics_inpainting(
            torch.from_numpy(case["x"]), torch.from_numpy(case["ref"]), torch.from_numpy(case["mask"]),
            stub, sig[100:101], n_steps_each=1, step_lr=6.2e-6, denoise=False, verbose=False, grad_ref=1)
    save("langevin_step.npz", x1=imgs[0].numpy())


def _kitti_merge(models, case, aB, sigma, setting=5, allowance=10, cc=0.01):
    from models.KITTISampling import anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti as S

    def zero(x, y):
        return torch.zeros_like(x)

    B = case["x"].shape[0]
    with torch.no_grad(), _NoiseFeed("merge"):
        imgs, _, shared = S(torch.from_numpy(case["x"]), torch.from_numpy(case["ref"]), torch.from_numpy(case["mask"]),
                            torch.from_numpy(case["sky"]), None, 0, setting, allowance, zero,
                            np.array([sigma], np.float32),
                            torch.from_numpy(case["fromWorld"].reshape(B, 1, 4, 4)),
                            torch.from_numpy(case["toWorld"].reshape(B, 1, 4, 4)), aB,
                            n_steps_each=1, step_lr=0.0, existMask=torch.from_numpy(case["exist"]),
                            denoise=False, verbose=False, grad_ref=1, correlation_coefficient=cc)
    return imgs[0].numpy(), imgs[1].numpy()


MERGE_CASES = [
    # tag, B, aB, H, W, sigma, kwargs for merge_case
    ("k_b4a2_s05", 4, 2, 64, 256, 0.5, {}),
    ("k_b4a4_s05", 4, 4, 64, 256, 0.5, {}),
    ("k_b4a4_s3", 4, 4, 64, 256, 3.0, {"sigma_mod": 3.0}),
    ("k_b2a2_ident", 2, 2, 64, 256, 0.5, {"identity": True, "neg_frac": 0.0}),
    ("k_b2a2_full", 2, 2, 64, 1024, 0.5, {}),
]


def gen_merge():
    models = _ref_imports()
    for tag, B, aB, H, W, sigma, kw in MERGE_CASES:
        case = GI.merge_case(tag, B, H, W, **kw)
        new, xf = _kitti_merge(models, case, aB, sigma)
        save(f"merge_{tag}.npz", new=new, x=xf)


CIRCLE_MODS = [[0, 0, 0], [5, -5, 0], [-5, -5, 0], [0, 5, 0], [-10, 10, 0], [10, 10, 0], [-10, 0, 0]]


def gen_allforone():
    models = _ref_imports()

    def zero(x, y):
        return torch.zeros_like(x)

    B = aB = 7
    # setting 8: the controlled average with allowance 5 (models/__init__.py:469-470)
    for tag, sigma, setting in [("a_b7_s05_set7", 0.5, 7), ("a_b7_s05_set5", 0.5, 5), ("a_b7_s05_set8", 0.5, 8)]:
        case = GI.merge_case(tag, B, 64, 256)
        with torch.no_grad(), _NoiseFeed("merge"):
            imgs, _, _ = models.anneal_Langevin_dynamics_inpainting_simultaneous_basic(
                torch.from_numpy(case["x"]), torch.from_numpy(case["ref"]), torch.from_numpy(case["mask"]),
                torch.from_numpy(case["sky"]), None, 0, setting, zero, np.array([sigma], np.float32),
                torch.from_numpy(np.array(CIRCLE_MODS)), aB, n_steps_each=1, step_lr=0.0,
                existMask=torch.from_numpy(case["exist"]), denoise=False, verbose=False, grad_ref=1,
                correlation_coefficient=0.01)
        save(f"merge_{tag}.npz", new=imgs[0].numpy(), x=imgs[1].numpy())


# Inpainting.yml (HDVMine_Circle.yml:73) origins + 2 more: the target + 8 aux views of BASELINE config 3
CIRCLE9 = CIRCLE_MODS + [[10, 0, 0], [0, -10, 0]]
BIG_VIEWS = [0, 17, 31]          # output views kept from the 32-view megabatch (each depends on all 32)


def gen_allforone9():
    """Config 3 geometry: B=aB=9 origin-offset merge, setting 7 (64x256)."""
    models = _ref_imports()

    def zero(x, y):
        return torch.zeros_like(x)

    case = GI.merge_case("a_b9_s05_set7", 9, 64, 256)
    with torch.no_grad(), _NoiseFeed("merge"):
        imgs, _, _ = models.anneal_Langevin_dynamics_inpainting_simultaneous_basic(
            torch.from_numpy(case["x"]), torch.from_numpy(case["ref"]), torch.from_numpy(case["mask"]),
            torch.from_numpy(case["sky"]), None, 0, 7, zero, np.array([0.5], np.float32),
            torch.from_numpy(np.array(CIRCLE9)), 9, n_steps_each=1, step_lr=0.0,
            existMask=torch.from_numpy(case["exist"]), denoise=False, verbose=False, grad_ref=1,
            correlation_coefficient=0.01)
    save("merge_a_b9_s05_set7.npz", new=imgs[0].numpy(), x=imgs[1].numpy())


def gen_big():
    """Config 4 geometry: ONE 32-view megabatch at the full 64x1024 (kitti poses, setting 5);
    only BIG_VIEWS of the outputs are stored (3 MB instead of 33 MB)."""
    models = _ref_imports()
    case = GI.merge_case("k_b32a32_full", 32, 64, 1024)
    new, xf = _kitti_merge(models, case, 32, 0.5)
    save("merge_k_b32a32_full.npz", views=np.array(BIG_VIEWS), new=new[BIG_VIEWS], x=xf[BIG_VIEWS])


def gen_config1():
    """Config 1: baseline sampler, B=1, sigmas[:1], 5 steps + denoise, injected noise (64x256)."""
    models = _ref_imports()
    H, W = 64, 256
    m = build_net(128, H, W)
    case = GI.merge_case("config1", 1, H, W)
    x0 = GI.scorenet_input("config1", 1, H, W)
    sig = get_sigmas_np()
    with torch.no_grad(), _NoiseFeed("config1"):
        imgs, _ = models.anneal_Langevin_dynamics_inpainting(
            torch.from_numpy(x0), torch.from_numpy(case["ref"]), torch.from_numpy(case["mask"]), m,
            sig[:1], n_steps_each=5, step_lr=6.2e-6, denoise=True, verbose=False, grad_ref=1)
    save("config1_b1_64x256.npz", step1=imgs[0].numpy(), step5=imgs[4].numpy(), denoised=imgs[5].numpy(),
         final=imgs[6].numpy())


# kitti sampler end to end: (tag, setting, file).  Setting 5 keeps cc; setting 7 ramps
# cc = 0.5 / (L / (c + 1)) over the levels (KITTISampling.py:106-109)
KITTI_E2E = [("e2e", 5, "kitti_e2e_b2_64x256.npz"), ("e2e_set7", 7, "kitti_e2e_set7_b2_64x256.npz")]


def gen_kitti_e2e():
    """Simultaneous kitti sampler end to end: B=aB=2, 3 levels x 2 steps + denoise (64x256)."""
    from models.KITTISampling import anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti as S
    H, W, B = 64, 256, 2
    m = build_net(128, H, W)
    sig = get_sigmas_np()[229:232]
    for tag, setting, fname in KITTI_E2E:
        case = GI.merge_case(tag, B, H, W)
        x0 = GI.scorenet_input(tag, B, H, W)
        with torch.no_grad(), _NoiseFeed(tag):
            imgs, _, shared = S(torch.from_numpy(x0), torch.from_numpy(case["ref"]), torch.from_numpy(case["mask"]),
                                torch.from_numpy(case["sky"]), None, 2, setting, 10, m, sig,
                                torch.from_numpy(case["fromWorld"].reshape(B, 1, 4, 4)),
                                torch.from_numpy(case["toWorld"].reshape(B, 1, 4, 4)), B,
                                n_steps_each=2, step_lr=6.2e-6, existMask=torch.from_numpy(case["exist"]),
                                denoise=True, verbose=False, grad_ref=1, correlation_coefficient=0.01)
        # images = [newImages (last level, step 1), newImages (step 2), final x]  (KITTISampling.py:418-419, 511)
        assert len(imgs) == 3
        save(fname, new=imgs[0].numpy(), new2=imgs[1].numpy(), final=imgs[2].numpy())


# AllForOne sampler loop end to end: (setting, minStepToShare).  Setting 5 ramps cc = (c+1)/L over
# the 3 levels (models/__init__.py:209-212) and, with minStepToShare 0, keeps the level-0 shared
# images (L505-506); setting 7 is the controlled average the AllForOne runner uses (AllForOne:589).
ALLFORONE_E2E = [(5, 0), (7, 1)]


def gen_allforone_e2e():
    """anneal_Langevin_dynamics_inpainting_simultaneous_basic (models/__init__.py:112-602) end to end:
    B=aB=3 origins (Circle.yml's first three), ngf=128 net, 3 late levels x 2 steps + denoise (64x256)."""
    models = _ref_imports()
    H, W, B = 64, 256, 3
    m = build_net(128, H, W)
    sig = get_sigmas_np()[229:232]
    for setting, min_step in ALLFORONE_E2E:
        tag = f"a_e2e_set{setting}"
        case = GI.merge_case(tag, B, H, W)
        x0 = GI.scorenet_input(tag, B, H, W)
        with torch.no_grad(), _NoiseFeed(tag):
            imgs, _, shared = models.anneal_Langevin_dynamics_inpainting_simultaneous_basic(
                torch.from_numpy(x0), torch.from_numpy(case["ref"]), torch.from_numpy(case["mask"]),
                torch.from_numpy(case["sky"]), None, min_step, setting, m, sig,
                torch.from_numpy(np.array(CIRCLE_MODS[:B])), B, n_steps_each=2, step_lr=6.2e-6,
                existMask=torch.from_numpy(case["exist"]), denoise=True, verbose=False, grad_ref=1,
                correlation_coefficient=0.01)
        # images = [newImages (last level, step 1), (step 2), final x]; shared = level-0 newImages (L505-508)
        assert len(imgs) == 3 and len(shared) == (2 if min_step == 0 else 0)
        extra = {"shared0": shared[0].numpy(), "shared1": shared[1].numpy()} if shared else {}
        save(f"allforone_e2e_set{setting}_b3_64x256.npz", new=imgs[0].numpy(), new2=imgs[1].numpy(),
             final=imgs[2].numpy(), **extra)


def gen_dsm():
    """Masked DSM loss (losses/dsm.py:67-119) + parameter-gradient norms, ngf=128 at 64x128, B=2."""
    sys.path.insert(0, REF)
    from losses.dsm import anneal_dsm_score_estimation_with_mask
    H, W, B = 64, 128, 2
    m = build_net(128, H, W).train()
    r = GI.rng("dsm")
    X = torch.from_numpy(r.random((B, 2, H, W)).astype(np.float32))
    noise = torch.from_numpy(r.standard_normal((B, 2, H, W)).astype(np.float32))
    mask = torch.from_numpy((r.random((B, 2, H, W)) > 0.3).astype(np.float32))
    labels = torch.tensor([3, 200])
    sig = m.sigmas
    used = sig[labels].view(B, 1, 1, 1)
    noise = noise * used
    loss, scores = anneal_dsm_score_estimation_with_mask(m, X + noise, used, noise, mask, None, sig, labels)
    loss.backward()
    gn = {k: p.grad.norm().item() for k, p in m.named_parameters()}
    save("dsm_ngf128_b2_64x128.npz", loss=np.array(loss.item()), scores=scores.detach().numpy(),
         grad_keys=np.array(list(gn.keys())), grad_norms=np.array(list(gn.values())))


def gen_projection():
    """point_cloud_to_range_image (datasets/lidar_utils.py:54-347) on synthetic clouds, with
    remission -- imported by file path (datasets/__init__.py needs torchvision)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("lidar_utils", os.path.join(REF, "datasets", "lidar_utils.py"))
    lu = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lu)
    for tag, (n, origin) in GI.PROJECTION_CASES.items():
        pc = GI.projection_cloud(tag, n)
        depth, inten, obf, _, sky, index = lu.point_cloud_to_range_image(pc, np.array(origin), True)
        save(f"projection_{tag}.npz", depth=depth, intensity=inten.astype(np.float32), obf=obf, sky=sky,
             index=index.astype(np.int32))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    what = sys.argv[1:] or ["exist", "scorenet", "ops", "langevin", "merge", "allforone", "config1", "e2e", "dsm",
                            "projection", "allforone9", "big", "allforone_e2e"]
    _ref_imports()
    for w in what:
        {"exist": gen_exist, "scorenet": gen_scorenet, "ops": gen_ops, "langevin": gen_langevin,
         "merge": gen_merge, "allforone": gen_allforone, "config1": gen_config1, "e2e": gen_kitti_e2e,
         "dsm": gen_dsm, "projection": gen_projection, "allforone9": gen_allforone9, "big": gen_big,
         "allforone_e2e": gen_allforone_e2e}[w]()
