"""§8(f)-2 runner orchestration pinned numerically: ``main.py --sample`` (the sampling runner on
libsdp) against the CPU oracle samplers on the same megabatch slices.

The reference runner (runners/ncsn_runner_kitti_simultaneous.py:549-893, AllForOne:560-1000) loops
doThis over the first doThis+2 views of every megabatch (the last doThis is the single-view baseline
on the whole batch), runs the sampler, and saves the final images through
``inverse_data_transform`` (clamp to [0, 1], datasets/__init__.py:206-215) in the grid layout
[2B', 3, H, W] (depth rows then intensity rows, channel tripled, kitti:650-663, 859-893).

Each sampler call the runner makes is recorded (its inputs and noise counters); the oracle sampler
(oracle/sampling_ref.py: sampler_kitti / sampler_allforone / sampler_baseline, with the torch-CPU
oracle score net at the same synthetic weights and the Philox stream restated in
oracle/philox_ref.py) is run on the views the REFERENCE's slicing selects from the batch, and the
file the runner wrote must equal the clamped grid layout of the oracle's final images.
The sigma schedule is 3 late levels (0.05 .. 0.01), so the step sizes keep the images in the data
range.  Tolerance: as the kitti end-to-end golden (test_gpu_parity.py): |err| <= 1e-4 (rel) + 1e-4 * max
on all but 1e-3 of the values (device vs numpy transcendental ulps can move a merge bin edge)."""
import glob
import os

import numpy as np
import pytest
import torch
import yaml

import main as sdp_main

CFG_DIR = os.path.join(os.path.dirname(sdp_main.__file__), "configs")
H, W = 64, 128


def _close_frac(a, b, rtol=1e-4, atol=1e-4):
    return np.mean(np.abs(a - b) > atol * np.abs(b).max() + rtol * np.abs(b))


def _layout(x):
    """[B,2,H,W] -> clamp [0,1] -> [2B,3,H,W] (kitti:650-663)."""
    x = np.clip(x, 0.0, 1.0)
    x = np.transpose(x, (1, 0, 2, 3)).reshape(-1, 1, x.shape[2], x.shape[3])
    return np.concatenate([x, x, x], axis=1)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["HDVMine_Line.yml", "HDVMine_Circle.yml"])
def test_runner_files_equal_oracle_samplers(tmp_path, name, monkeypatch):
    from oracle import philox_ref
    from oracle import sampling_ref as S
    from oracle import scorenet_ref as R
    from sdp import runner as RN
    from sdp.weights import get_sigmas_np, synthetic_state_dict

    with open(os.path.join(CFG_DIR, name)) as f:
        c = yaml.safe_load(f)
    B, aB = 6, 3
    c["sampling"].update(batch_size=B, actualBatchSize=aB, n_steps_each=1)
    c["data"].update(image_width=W, modifications=c["data"]["modifications"][:aB])
    # 3 late-schedule levels: the step sizes keep x in the data range.  (From sigma 50 the first
    # step is 155 x the score and x leaves [0, 1] by tens; the denoise step then cancels two such
    # numbers to O(1), so the score net's relative error, not the orchestration, sets the result.)
    c["model"].update(num_classes=3, sigma_begin=0.05, sigma_end=0.01)
    cfg = tmp_path / "small.yml"
    cfg.write_text(yaml.safe_dump(c))
    kitti = "Line" in name

    calls = []

    def snap(v):    # the call's inputs, copied before the sampler runs
        return v.detach().cpu().numpy().copy() if torch.is_tensor(v) else v

    def rec(kind, fn):
        def wrapped(*a, **k):
            calls.append((kind, [snap(v) for v in a], {n_: snap(v) for n_, v in k.items()}))
            return fn(*a, **k)
        return wrapped
    for kind in ("anneal_Langevin_dynamics_inpainting", "anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti",
                 "anneal_Langevin_dynamics_inpainting_simultaneous_basic"):
        monkeypatch.setattr(RN, kind, rec(kind, getattr(RN, kind)))
    exp = tmp_path / "exp"
    assert sdp_main.main(["--config", str(cfg), "--sample", "--ni", "--exp", str(exp), "--verbose", "warning"]) == 0
    out = exp / "image_samples" / "images"

    # the batch the runner sampled (the procedural source, batch 0) and the reference's slicing
    batch = RN.synthetic_batch(0, B, aB, H, W, seed=1234)
    ref_full, mask_full = batch[0].float().numpy(), batch[1].int().numpy()
    sd = synthetic_state_dict(128)
    sd["sigmas"] = get_sigmas_np(0.05, 0.01, 3)          # the model's sigma buffer of this config (ncsnv2.py:430)
    P = R.to_torch_params(sd)

    def score(x, y):
        with torch.no_grad():
            return R.scorenet_forward(P, torch.from_numpy(np.ascontiguousarray(x)), torch.from_numpy(y)).numpy()

    n_mega = B // aB
    assert len(calls) == aB                              # doThis 0 .. aB-1, the last the baseline
    for do, (kind, a, k) in enumerate(calls):
        t = np.asarray
        x0 = t(a[0])
        sig = t(a[4] if kind == "anneal_Langevin_dynamics_inpainting" else a[9] if kind.endswith("_kitti") else a[8])
        n = x0.shape[0]
        kk = n // n_mega if kind != "anneal_Langevin_dynamics_inpainting" or n != B else aB
        idx = [m * aB + i for m in range(n_mega) for i in range(kk)] if n != B else list(range(B))
        # the views the reference selects: the first kk of every megabatch
        np.testing.assert_array_equal(t(a[1]), ref_full[idx])
        np.testing.assert_array_equal(t(a[2]).astype(np.int32), mask_full[idx])
        nv0, nv_all = k.get("noise_views") or (0, n)
        per_view4 = 2 * H * W // 4
        ctr = [nv0 * per_view4]

        def noise_fn(shape, seed=k.get("seed", 1234)):
            v = philox_ref.normal(seed, ctr[0], int(np.prod(shape))).reshape(shape)
            ctr[0] += nv_all * per_view4
            return v
        if kind == "anneal_Langevin_dynamics_inpainting":
            imgs = S.sampler_baseline(x0, t(a[1]), t(a[2]), score, sig, a[5], a[6], noise_fn,
                                      denoise=k["denoise"], grad_ref=k["grad_ref"])
        elif kind.endswith("_kitti"):
            imgs, _, _ = S.sampler_kitti(x0, t(a[1]), t(a[2]), t(a[3]).astype(bool), a[5], a[6], a[7], score, sig,
                                         t(a[10]).reshape(n, 4, 4), t(a[11]).reshape(n, 4, 4), a[12], a[13], a[14],
                                         t(k["existMask"]).astype(bool), noise_fn, denoise=k["denoise"],
                                         grad_ref=k["grad_ref"], cc=k["correlation_coefficient"])
        else:
            imgs, _, _ = S.sampler_allforone(x0, t(a[1]), t(a[2]), t(a[3]).astype(bool), a[5], a[6], score, sig,
                                             t(a[9]), a[10], a[11], a[12], t(k["existMask"]).astype(bool), noise_fn,
                                             denoise=k["denoise"], grad_ref=k["grad_ref"],
                                             cc=k["correlation_coefficient"])
        want = _layout(imgs[-1])
        files = glob.glob(str(out / f"{do}_*_Masked_completion_*.pth.npy"))
        assert len(files) == 1, (do, files)
        got = np.load(files[0])
        assert got.shape == want.shape, (got.shape, want.shape)
        frac = _close_frac(got, want)
        err = np.abs(got - want)
        print(f"{name} doThis {do} ({kind}, {n} views): mismatch fraction {frac:.2e}; |err| max {err.max():.3e} "
              f"q99.9 {np.quantile(err, 0.999):.3e} q99 {np.quantile(err, 0.99):.3e}; depth rows bad "
              f"{np.mean(err[:n] > 1e-4):.2e}, intensity rows bad {np.mean(err[n:] > 1e-4):.2e}; "
              f"saturated {np.mean((want == 0) | (want == 1)):.2f}")
        if os.environ.get("SDP_PIN_DUMP"):
            np.savez(os.path.join(os.environ["SDP_PIN_DUMP"], f"pin_{name[:-4]}_{do}.npz"), got=got, want=want)
        assert frac <= 1e-3
