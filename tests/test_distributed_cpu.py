"""gloo tests (world 2, 3 and 4) of the view-sharded simultaneous sampler (the multi-GPU path).

Device ops are replaced by the CPU oracle (langevin / merge), and the score network by a
cheap deterministic stand-in, so this checks exactly the sharding logic: per-rank views,
the per-step all-gather of the megabatch, the all_reduce(MAX) that keeps tooHigh global,
and each rank merging into its own views.  The sharded result must equal the single-process
run bit for bit.  World 4 has interior ranks (1, 2: neither first nor last block of the megabatch);
world 3 over 8 views is an uneven split (3 + 3 + 2 views, the padded all-gather of
sdp/sampling.py:_gather_views).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import golden_inputs as GI
from oracle import philox_ref
from oracle import sampling_ref as S

B_ALL, H, W = 8, 64, 128
SIGMAS = np.array([0.9, 0.6, 0.3], np.float32)


class OracleMerger:
    def __init__(self, n_all, aB, H, W, dev, exist, sky, refmask, toWorld=None, fromWorld=None, origins=None,
                 o_begin=0, n_out=None):
        self.aB, self.o_begin, self.n_out = aB, o_begin, n_out
        self.exist = np.asarray(exist)
        self.sky = np.asarray(sky).reshape(n_all, 1, H, W)
        self.refmask = np.asarray(refmask)
        # origin-offset variant: the origins are already 10*sign(m), which the oracle maps to themselves
        self.mods = None if origins is None else np.asarray(origins)
        if origins is None:
            self.toWorld = np.asarray(toWorld).reshape(n_all, 4, 4)
            self.fromWorld = np.asarray(fromWorld).reshape(n_all, 4, 4)

    def __call__(self, x_all, sigma, setting, allowance, cc, absmax, new):
        amax = absmax.view(torch.float32).item()
        if self.mods is not None:
            n, xc = S.allforone_merge(x_all.numpy(), self.refmask, self.sky, self.exist, self.mods, self.aB, sigma,
                                      setting, cc, absmax=amax)
        else:
            n, xc = S.kitti_merge(x_all.numpy(), self.refmask, self.sky, self.exist, self.toWorld, self.fromWorld,
                                  self.aB, sigma, setting, allowance, cc, absmax=amax)
        sl = slice(self.o_begin, self.o_begin + self.n_out)
        x_all[sl] = torch.from_numpy(xc[sl])
        if new is not None:
            new.copy_(torch.from_numpy(n[sl]))


class OracleOps:
    def langevin(self, x, grad, ref, mask, noise, seed, offset, step, nscale, grad_ref, nan_to_num, lik, absmax):
        g = S.nan_to_num(grad.numpy()) if nan_to_num else grad.numpy()
        if noise is None:   # the kernel's Philox stream (seed, counter = offset + element/4)
            noise = torch.from_numpy(philox_ref.normal(seed, offset, x.numel()).reshape(x.shape))
        lk = (-mask.numpy()).astype(np.float32) * (x.numpy() - ref.numpy())
        v = (((x.numpy() + np.float32(step) * g) + np.float32(grad_ref) * lk) + noise.numpy() * np.float32(nscale))
        x.copy_(torch.from_numpy(v.astype(np.float32)))
        lik.copy_(torch.from_numpy(lk))
        absmax.copy_(torch.tensor([np.abs(v[:, 0]).max()], dtype=torch.float32).view(torch.int32))

    def axpy(self, x, g, a, lik, mask, ref, b):
        if g is not None:
            x.copy_(((x + np.float32(a) * g) + np.float32(b) * lik))
        else:
            x.copy_(x + np.float32(b) * ((-mask).float() * (x - ref)))

    def make_merger(self, *a, **kw):
        return OracleMerger(*a, **kw)


def fake_score(x, y):
    """Deterministic stand-in for the score net (depends on x and on the label)."""
    return -(x - 0.5) * (1.0 + 0.01 * y.view(-1, 1, 1, 1).float()) + 0.05 * torch.sin(7 * x)


def _inputs():
    case = GI.merge_case("dist", B_ALL, H, W)
    x0 = GI.scorenet_input("dist", B_ALL, H, W)
    return case, x0


def _run(rank, world, port, out_dir, philox=False):
    from sdp.sampling import anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti as samp
    from sdp.sampling import view_blocks
    torch.set_num_threads(1)
    if world > 1:
        torch.distributed.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                             world_size=world)
    case, x0 = _inputs()
    v0, nv = view_blocks(B_ALL, world)[rank]
    sl = slice(v0, v0 + nv)
    k = [0]

    def noise_fn(shape):  # slice of the single-process noise stream
        n = GI.noise("dist", k[0], (B_ALL, 2, H, W))[sl]
        k[0] += 1
        return torch.from_numpy(np.ascontiguousarray(n))

    t = torch.from_numpy
    images, _, shared = samp(
        t(x0[sl].copy()), t(case["ref"][sl].copy()), t(case["mask"][sl].copy()), t(case["sky"][sl].copy()), None, 1, 5,
        10, fake_score, SIGMAS, t(case["fromWorld"]), t(case["toWorld"]), B_ALL, n_steps_each=2, step_lr=6.2e-6,
        existMask=t(case["exist"]), denoise=True, verbose=False, grad_ref=1, correlation_coefficient=0.01,
        noise_fn=None if philox else noise_fn, view_shard=(rank, world) if world > 1 else None, all_refer_mask=t(case["mask"]),
        all_sky=t(case["sky"]), ops=OracleOps())
    np.save(os.path.join(out_dir, f"w{world}_r{rank}{'_p' if philox else ''}.npy"), np.stack([im.numpy() for im in images]))
    if world > 1:
        torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_view_blocks_tile_the_megabatch():
    from sdp.sampling import view_blocks
    for n in range(1, 33):
        for w in range(1, n + 1):
            bl = view_blocks(n, w)
            assert [v for v0, c in bl for v in range(v0, v0 + c)] == list(range(n))
            assert max(c for _, c in bl) - min(c for _, c in bl) <= 1


@pytest.mark.parametrize("world,philox", [(2, False), (2, True), (4, True), (3, True)],
                         ids=["w2_injected_noise", "w2_philox_noise", "w4_interior_ranks", "w3_uneven_split"])
def test_view_sharded_sampler_matches_single_process(tmp_path, world, philox):
    """philox_noise: no noise_fn, so each rank draws the kernel's own counter-based stream; the
    sharded run must draw the single-process noise for its views (counter offset = first view)."""
    _run(0, 1, 0, str(tmp_path), philox)
    mp.spawn(_run, args=(world, _free_port(), str(tmp_path), philox), nprocs=world, join=True)
    sfx = "_p" if philox else ""
    single = np.load(tmp_path / f"w1_r0{sfx}.npy")                 # [n_images, B_ALL, 2, H, W]
    shard = np.concatenate([np.load(tmp_path / f"w{world}_r{r}{sfx}.npy") for r in range(world)], axis=1)
    assert single.shape == shard.shape
    np.testing.assert_array_equal(shard, single)
    assert np.abs(single[-1] - GI.scorenet_input("dist", B_ALL, H, W)).max() > 1e-3   # the sampler did move x
