"""Annealed-Langevin samplers with the reference's signatures, running on libsdp.

  anneal_Langevin_dynamics_inpainting ....................... models/__init__.py:1385-1442
  anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti  models/KITTISampling.py:6-513
  anneal_Langevin_dynamics_inpainting_simultaneous_basic ....... models/__init__.py:112-602

Each step is: ``scorenet(x, labels)`` (libsdp forward, or any callable returning a device
tensor), the fused Langevin kernel (update + max|x[:,0]| for tooHigh), and -- from level
``minStepToShare`` on -- the device consistency merge.  With libsdp's ScoreNet the first two are
one call (``forward_langevin``: the update runs in the net's last kernel, bit-identical).  Host-side scalars (step size, noise
scale, correlation ramps) are computed with the reference's numpy float32 arithmetic.

Keyword-only extras (not in the reference): ``noise_fn(shape) -> tensor`` injects the
noise (parity tests); otherwise noise is Philox N(0,1) from ``seed``, one counter per 4
elements of the whole job, so ``noise_views=(first_view, total_views)`` lets a call that
holds a contiguous slice of a larger job (megabatch sharding) draw that slice's noise.  ``dist_group`` makes
tooHigh global across ranks (one 4-byte all_reduce(MAX) per merged step); with
``view_shard=(rank, world)`` the call's views are one megabatch split across ranks in
contiguous blocks (``view_blocks``: the first megabatch % world ranks hold one view more): each
rank passes only its own views, the megabatch images are all-gathered every merged step
(the cross-view consistency gather) and each rank merges into its own views.
Documented deviations: B=1 works for the kitti sampler (the reference's ``torch.squeeze``
of the poses breaks it); the baseline keeps only the images it returns
(it does not hold every step on the CPU, Appendix B.8) unless ``keep_all=True``.
"""
from __future__ import annotations

import numpy as np
import torch

from .merge import AbsmaxAllReduce, Merger, allforone_origins

F32 = np.float32


class DeviceOps:
    """The device operations of a step, on libsdp (one HIP stream: torch's current)."""

    def langevin(self, x, grad, ref, mask, noise, seed, offset, step, nscale, grad_ref, nan_to_num, lik, absmax):
        from . import _lib
        B, C, H, W = x.shape
        _lib.check(_lib.lib().sdp_langevin_step(
            x.data_ptr(), grad.data_ptr(), ref.data_ptr(), mask.data_ptr(), _lib.ptr(noise), seed, offset,
            float(step), float(nscale), float(grad_ref), 1 if nan_to_num else 0, B, C, H * W, lik.data_ptr(),
            absmax.data_ptr(), _lib.stream()), "langevin_step")

    def axpy(self, x, g, a, lik, mask, ref, b):
        from . import _lib
        _lib.check(_lib.lib().sdp_axpy_step(x.data_ptr(), _lib.ptr(g), float(a), _lib.ptr(lik), _lib.ptr(mask),
                                            _lib.ptr(ref), float(b), x.numel(), _lib.stream()), "axpy")

    def make_merger(self, *args, **kw):
        return Merger(*args, **kw)


class _Stepper:
    """Per-call state shared by the samplers.  ``x`` is this rank's views; with a view shard
    it is a contiguous slice of ``x_all`` (the whole megabatch)."""

    def __init__(self, x_mod, refer_image, refer_mask, noise_fn, seed, ops, n_all=None, own0=0, noise_views=None):
        self.ops = ops
        x = x_mod.detach().to(torch.float32).contiguous()
        self.B, self.C, self.H, self.W = x.shape
        self.dev = x.device
        n_all = self.B if n_all is None else n_all
        self.x_all = torch.zeros((n_all, self.C, self.H, self.W), dtype=torch.float32, device=self.dev)
        self.own0 = own0
        self.x = self.x_all[own0:own0 + self.B]
        self.x.copy_(x)
        self.ref = refer_image.to(self.dev, torch.float32).contiguous()
        self.mask = refer_mask.to(self.dev).to(torch.int32).contiguous()
        self.HW = self.H * self.W
        self.lik = torch.empty_like(self.x)
        self.absmax = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.noise_fn = noise_fn
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        # Philox counters are per 4 elements of the WHOLE megabatch: a rank holding views
        # [own0, own0+B) draws exactly the noise the single-process run draws for those views
        # (noise_views = (first view, views of the whole job) when the job is split by megabatch)
        nv0, nv_all = noise_views if noise_views is not None else (own0, n_all)
        self.per_view4 = self.C * self.H * self.W // 4
        self.offset = nv0 * self.per_view4
        self.offset_stride = nv_all * self.per_view4
        self._labels = {}

    def labels(self, c):
        t = self._labels.get(c)
        if t is None:
            t = torch.full((self.B,), int(c), dtype=torch.int64, device=self.dev)
            self._labels[c] = t
        return t

    def _noise(self):
        if self.noise_fn is None:
            return None
        return self.noise_fn(tuple(self.x.shape)).to(self.dev, torch.float32).contiguous()

    def step(self, grad, step_size, grad_ref, nan_to_num):
        grad = grad.to(self.dev, torch.float32).contiguous()
        noise = self._noise()
        nscale = F32(np.sqrt(F32(step_size * F32(2))))
        self.absmax.zero_()
        self.ops.langevin(self.x, grad, self.ref, self.mask, noise, self.seed, self.offset, step_size, nscale,
                          grad_ref, nan_to_num, self.lik, self.absmax)
        self.offset += self.offset_stride

    def langevin_step(self, scorenet, c, step_size, grad_ref, nan_to_num, want_grad):
        """scorenet + Langevin update.  On libsdp (DeviceOps and a ScoreNet) the update runs in the
        net's last kernel (sdp_net_forward_langevin, bit-identical to the two-call form); the
        scores are materialised only when asked (want_grad: the report of a level).  Returns them
        (or None)."""
        if isinstance(self.ops, DeviceOps) and hasattr(scorenet, "forward_langevin"):
            noise = self._noise()
            nscale = F32(np.sqrt(F32(step_size * F32(2))))
            grad = torch.empty_like(self.x) if want_grad else None
            self.absmax.zero_()
            scorenet.forward_langevin(self.x, self.labels(c), self.ref, self.mask, noise, self.seed, self.offset,
                                      step_size, nscale, grad_ref, nan_to_num, self.lik, self.absmax, grad)
            self.offset += self.offset_stride
            return grad
        grad = scorenet(self.x, self.labels(c))
        self.step(grad, step_size, grad_ref, nan_to_num)
        return grad

    def denoise(self, grad, sigma_last, grad_ref):
        grad = grad.to(self.dev, torch.float32).contiguous()
        self.ops.axpy(self.x, grad, F32(sigma_last) ** 2, self.lik, None, None, grad_ref)

    def final_consistency(self, grad_ref):
        self.ops.axpy(self.x, None, 0.0, None, self.mask, self.ref, grad_ref)

    def report(self, grad_ref, c, step_size, grad):
        d = (self.x - self.ref).abs()
        print("grad_ref: {}, mean: {}, median: {}".format(grad_ref, d.mean(), d.median()))
        gn = torch.norm(grad.reshape(self.B, -1), dim=-1).mean()
        ln = torch.norm(self.lik.reshape(self.B, -1), dim=-1).mean()
        xn = torch.norm(self.x.reshape(self.B, -1), dim=-1).mean()
        print("level: {}, step_size: {}, grad_norm: {}, grad_likelihood_norm: {}, image_norm: {}".format(
            c, step_size, gn.item(), ln.item(), xn.item()))


def _step_size(step_lr, sigma, sigma_last):
    """KITTISampling.py:135 in numpy float32 (python float * np.float32 stays float32)."""
    return F32(step_lr) * (F32(sigma) / F32(sigma_last)) ** 2


@torch.no_grad()
def anneal_Langevin_dynamics_inpainting(x_mod, refer_image, refer_mask, scorenet, sigmas, n_steps_each=100,
                                        step_lr=0.000008, denoise=True, verbose=True, grad_ref=0.1, sampling_step=16,
                                        *, noise_fn=None, seed=1234, keep_all=False, ops=None, noise_views=None):
    """Single-view baseline (models/__init__.py:1385-1442). No nan_to_num, as in the reference."""
    S = _Stepper(x_mod, refer_image, refer_mask, noise_fn, seed, ops or DeviceOps(), noise_views=noise_views)
    sigmas = np.asarray(sigmas, dtype=np.float32)
    images, targets = [], []
    last = None
    for c, sigma in enumerate(sigmas):
        step = _step_size(step_lr, sigma, sigmas[-1])
        for i in range(n_steps_each):
            grad = S.langevin_step(scorenet, c, step, grad_ref, False, verbose and c % 20 == 0 and i == n_steps_each - 1)
            if keep_all:
                images.append(S.x.to("cpu"))
            last = grad
        if verbose and c % 20 == 0 and last is not None:
            S.report(grad_ref, c, step, last)
    if not keep_all and len(sigmas) * n_steps_each > 0:
        images.append(S.x.to("cpu"))
    if denoise:
        grad = scorenet(S.x, S.labels(len(sigmas) - 1))
        S.denoise(grad, sigmas[-1], grad_ref)
        images.append(S.x.to("cpu"))
    S.final_consistency(grad_ref)
    images.append(S.x.to("cpu"))
    targets.append(refer_image.to("cpu"))
    return images, targets


def _gather_views(S, group):
    """All-gather every rank's views into the megabatch buffer (RCCL over xGMI on GPUs).  Equal
    blocks land in place; uneven ones (megabatch % world != 0) travel padded to the largest block
    and are copied into place."""
    dist = torch.distributed
    blocks = S.blocks
    cmax = max(c for _, c in blocks)
    if all(c == cmax for _, c in blocks):
        if S.x_all.is_cuda:
            dist.all_gather_into_tensor(S.x_all, S.x, group=group)
        else:  # gloo: list form
            parts = list(S.x_all.chunk(len(blocks)))
            dist.all_gather(parts, S.x.clone(), group=group)
        return
    pad = torch.zeros((cmax,) + tuple(S.x.shape[1:]), dtype=S.x.dtype, device=S.dev)
    pad[:S.B].copy_(S.x)
    buf = torch.empty((len(blocks) * cmax,) + tuple(S.x.shape[1:]), dtype=S.x.dtype, device=S.dev)
    if S.x_all.is_cuda:
        dist.all_gather_into_tensor(buf, pad, group=group)
    else:
        dist.all_gather(list(buf.chunk(len(blocks))), pad, group=group)
    for r, (v0, c) in enumerate(blocks):
        S.x_all[v0:v0 + c].copy_(buf[r * cmax:r * cmax + c])


def _simultaneous(S, scorenet, sigmas, min_step, setting, n_steps_each, step_lr, denoise, verbose, grad_ref, cc0,
                  merger, allowance, cc_ramp, dist_group, view_split, print_rule):
    sigmas = np.asarray(sigmas, dtype=np.float32)
    images, shared = [], []
    L = len(sigmas)
    cc = cc0
    absmax_reduce = AbsmaxAllReduce(dist_group)
    for c, sigma in enumerate(sigmas):
        cc = cc_ramp(cc, c, L)
        step = _step_size(step_lr, sigma, sigmas[-1])
        grad = None
        report = print_rule(c, verbose)
        for i in range(n_steps_each):
            grad = S.langevin_step(scorenet, c, step, grad_ref, True, report and i == n_steps_each - 1)
            if c >= min_step:
                if view_split:
                    _gather_views(S, dist_group)
                ev = None
                if dist_group is not None or (view_split and torch.distributed.is_initialized()):
                    ev = absmax_reduce(S.absmax)      # overlaps the merge up to its correction pass
                want = c in (0, 20, 110) or c == L - 1
                new = torch.empty(merger.n_out, S.C, S.H, S.W, device=S.dev) if want else None
                if ev is None:
                    merger(S.x_all, sigma, setting, allowance, cc, S.absmax, new)
                else:
                    merger(S.x_all, sigma, setting, allowance, cc, S.absmax, new, absmax_event=ev)
                if c in (0, 20, 110):
                    shared.append(new.to("cpu"))
                if c == L - 1:
                    images.append(new.to("cpu"))
        if print_rule(c, verbose) and grad is not None:
            S.report(grad_ref, c, step, grad)
    if denoise:
        grad = scorenet(S.x, S.labels(L - 1))
        S.denoise(grad, sigmas[-1], grad_ref)
    S.final_consistency(grad_ref)
    images.append(S.x.to("cpu"))
    return images, [], shared


def view_blocks(n_all, world):
    """[(v0, count)] per rank: the contiguous view block each rank of a view-split megabatch owns --
    the first n_all % world ranks take one view more (the reference's DataParallel scatters its batch
    in ceil-sized chunks, runners/ncsn_runner_kitti_simultaneous.py:481; any contiguous split merges
    the same views)."""
    base, extra = divmod(int(n_all), int(world))
    return [(r * base + min(r, extra), base + (1 if r < extra else 0)) for r in range(world)]


def _shard_setup(x_mod, actualBatchSize, view_shard):
    """(n_all, own0, blocks): the views this call's buffers hold, where this rank's start, and every
    rank's (first view, count) -- None without a view shard."""
    B = x_mod.shape[0]
    if view_shard is None:
        return B, 0, None
    rank, world = view_shard
    blocks = view_blocks(actualBatchSize, world)
    if blocks[-1][1] == 0:
        raise ValueError("view_shard: a megabatch of actualBatchSize views cannot give every one of the world ranks a view")
    if B != blocks[rank][1]:
        raise ValueError(f"view_shard: rank {rank} of {world} must hold views [{blocks[rank][0]}, "
                         f"{blocks[rank][0] + blocks[rank][1]}) of ONE megabatch of {actualBatchSize}, got {B}")
    return actualBatchSize, blocks[rank][0], blocks


@torch.no_grad()
def anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti(
        x_mod, refer_image, refer_mask, sky, x_indices, minStepToShare, setting, allowance, scorenet, sigmas, fromWorld,
        toWorld, actualBatchSize, n_steps_each=100, step_lr=0.000008, existMask=None, denoise=True, verbose=True,
        grad_ref=0.1, correlation_coefficient=0.1, sampling_step=16, *, noise_fn=None, seed=1234, dist_group=None,
        view_shard=None, all_refer_mask=None, all_sky=None, ops=None, noise_views=None):
    """Pose-matrix simultaneous sampler (KITTISampling.py:6-513); x_indices/sampling_step unused as there.

    With ``view_shard=(rank, world)``: x_mod/refer_* hold this rank's views, while fromWorld,
    toWorld, ``all_sky`` and ``all_refer_mask`` describe every view of the megabatch.
    """
    ops = ops or DeviceOps()
    n_all, own0, blocks = _shard_setup(x_mod, actualBatchSize, view_shard)
    S = _Stepper(x_mod, refer_image, refer_mask, noise_fn, seed, ops, n_all, own0, noise_views)
    S.blocks = blocks
    sky_all = sky if view_shard is None else all_sky
    mask_all = S.mask if view_shard is None else all_refer_mask
    merger = ops.make_merger(n_all, actualBatchSize, S.H, S.W, S.dev, existMask, sky_all, mask_all, toWorld=toWorld,
                             fromWorld=fromWorld, o_begin=own0, n_out=S.B)

    def ramp(cc, c, L):  # KITTISampling.py:108-111
        if setting == 6:
            return 1 / (L / (c + 1))
        if setting == 7:
            return 0.5 / (L / (c + 1))
        return cc

    return _simultaneous(S, scorenet, sigmas, minStepToShare, setting, n_steps_each, step_lr, denoise, verbose,
                         grad_ref, correlation_coefficient, merger, allowance, ramp, dist_group, view_shard is not None,
                         lambda c, v: v and c % 20 == 0 or c == 1 or c == 2)  # KITTISampling.py:497 precedence


@torch.no_grad()
def anneal_Langevin_dynamics_inpainting_simultaneous_basic(
        x_mod, refer_image, refer_mask, sky, x_indices, minStepToShare, setting, scorenet, sigmas, modificationList,
        actualBatchSize, n_steps_each=100, step_lr=0.000008, existMask=None, denoise=True, verbose=True, grad_ref=0.1,
        correlation_coefficient=0.1, sampling_step=16, *, noise_fn=None, seed=1234, dist_group=None, view_shard=None,
        all_refer_mask=None, all_sky=None, ops=None, noise_views=None):
    """Origin-offset (AllForOne) simultaneous sampler (models/__init__.py:112-602)."""
    ops = ops or DeviceOps()
    n_all, own0, blocks = _shard_setup(x_mod, actualBatchSize, view_shard)
    S = _Stepper(x_mod, refer_image, refer_mask, noise_fn, seed, ops, n_all, own0, noise_views)
    S.blocks = blocks
    sky_all = sky if view_shard is None else all_sky
    mask_all = S.mask if view_shard is None else all_refer_mask
    origins = allforone_origins(modificationList)
    merger = ops.make_merger(n_all, actualBatchSize, S.H, S.W, S.dev, existMask, sky_all, mask_all, origins=origins,
                             o_begin=own0, n_out=S.B)
    allowance = 5 if setting >= 8 else 10

    def ramp(cc, c, L):  # models/__init__.py:209-212
        if setting == 5:
            return 1 / (L / (c + 1))
        if setting == 6:
            return 0.5 / (L / (c + 1))
        return cc

    return _simultaneous(S, scorenet, sigmas, minStepToShare, setting, n_steps_each, step_lr, denoise, verbose,
                         grad_ref, correlation_coefficient, merger, allowance, ramp, dist_group, view_shard is not None,
                         lambda c, v: v and c % 20 == 0)
