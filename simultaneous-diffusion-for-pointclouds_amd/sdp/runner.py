"""Sampling runner: the reference's ``runner.sample()`` contract over the libsdp samplers.

Mirrors the view-count sweep and output files of
  runners/ncsn_runner_kitti_simultaneous.py:461-893   (KITTI360_im_8batch, pose-matrix merge)
  runners/ncsn_runner_AllForOne.py:468-900            (KITTI360_im_AllForOne / _simultaneous_densification)
Per batch of ``sampling.batch_size`` views (megabatches of ``actualBatchSize``) and per
``doThis``: the first doThis+2 views of every megabatch are sampled jointly (all of them
at the end of the sweep) and the single-view baseline runs last; files are written exactly
as the reference names them (np.save appends .npy):
  toWorld_{saveNum}.npy, fromWorld_{saveNum}.npy,
  {doThis}_{saveNum}_{Input,GT}_completion_{ckpt}.pth.npy, {doThis}_{saveNum}_SKY_{ckpt}.pth.npy,
  {doThis}_{saveNum}_Masked_completion_{ckpt}.pth.npy, {doThis}_{saveNum}_TimeTaken.npy,
  {doThis}_{saveNum}_Shared_completion_initial{ckpt}.pth.npy (AllForOne runner only)
Images are saved as inverse_data_transform (clamp [0,1], datasets/__init__.py:206-215) and
transposed to [2B',3,H,W] (rows [0,B') depth, [B',2B') intensity, 3 identical channels).

Data: with ``args.kitti_root`` the views come from the KITTI-360 datasets of sdp.kitti360
(rendered on the GPU) in the order of the reference's MySampler over the pose file
(kitti:494-515); otherwise from the procedural scene of ``sdp.synthetic`` (same 9-tuple
contract, kitti360_im_8Batch.py:304).

Multi-GPU (the reference's DataParallel, kitti:481): under torchrun (one process per GPU,
torch.distributed initialised by main.py) every batch's megabatches are split into contiguous
blocks, one per rank; each rank samples its block (tooHigh stays global through the samplers'
4-byte all_reduce(MAX) over the active ranks, and each view draws the noise it would draw in a
single-process run), the sampled images are gathered to rank 0, and rank 0 writes the files --
the same files, bit for bit, as one process would.

``train()`` is the kitti runner's DSM training loop (kitti:83-348; identical in
ncsn_runner_AllForOne.py:88-353) on libsdp, data parallel over ranks (see ``train``).
"""
from __future__ import annotations

import logging
import os
import time

import numpy as np
import torch

from . import kitti360, synthetic
from .weights import synthetic_state_dict
from .imgutil import make_grid, save_image
from .sampling import (anneal_Langevin_dynamics_inpainting,
                       anneal_Langevin_dynamics_inpainting_simultaneous_basic,
                       anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti)
from .scorenet import ScoreNet
from .weights import get_sigmas_np

REF_CKPT = "/data/kitti_pretrained/logs/kitti/checkpoint_100000.pth"   # kitti:472


def inverse_data_transform(x):
    """datasets/__init__.py:206-215 for these configs (not rescaled, no logit): clamp to [0,1]."""
    return torch.clamp(x, 0.0, 1.0)


def to_grid_layout(x):
    """[B,2,H,W] -> [2B,3,H,W]: depth rows then intensity rows, channel tripled (kitti:650-663)."""
    x = x.transpose(1, 0)
    x = x.reshape(x.size(0) * x.size(1), 1, x.size(2), x.size(3))
    return torch.cat((x, x, x), 1)


def synthetic_batch(batch_index, B, aB, H, W, seed=1234):
    """The dataset's 9-tuple for one DataLoader batch of B views (B/aB megabatches):
    (masked refer, mask, sky, indices, toWorld, fromWorld, goal, toOGView, saveNum)."""
    parts = [synthetic.scene_views(aB, H, W, seed=seed + 7919 * batch_index + m) for m in range(B // aB)]
    cat = {k: torch.from_numpy(np.concatenate([p[k] for p in parts])) for k in ("ref", "mask", "sky", "toWorld",
                                                                              "fromWorld")}
    ref, mask = cat["ref"], cat["mask"]
    indices = torch.zeros(B, 1, H, W, dtype=torch.int64)
    save_num = torch.arange(B) + batch_index * B
    return (ref * mask, mask, cat["sky"], indices, cat["toWorld"], cat["fromWorld"], ref.clone(),
            cat["fromWorld"].clone(), save_num)


def shard_megabatches(n_mega, rank, world):
    """[m0, m1): the contiguous block of megabatches rank `rank` samples (the first
    n_mega % world ranks take one more; ranks past n_mega get none)."""
    base, extra = divmod(n_mega, world)
    m0 = rank * base + min(rank, extra)
    return m0, m0 + base + (1 if rank < extra else 0)


def _dist():
    d = torch.distributed
    if d.is_available() and d.is_initialized():
        return d.get_rank(), d.get_world_size()
    return 0, 1


def _first_views(t, n_mega, aB, k):
    """Keep the first k views of every megabatch (the reference's reshape-and-slice, kitti:720-739)."""
    shp = t.shape
    return t.reshape(n_mega, aB, -1)[:, :k].reshape((n_mega * k,) + tuple(shp[1:]))


class Runner:
    def __init__(self, args, config, score=None, ops=None):
        """score / ops: injected score network and device ops (tests); default libsdp."""
        self.args, self.config = args, config
        self._score, self.ops = score, ops
        self.device = getattr(config, "device", None) or torch.device("cuda", torch.cuda.current_device())
        sim = getattr(config, "simultaneous", None)
        g = (lambda k, d: getattr(sim, k, d)) if sim is not None else (lambda k, d: d)
        self.start_step = g("startStep", 2)
        self.cc = g("correlation_coefficient", 0.01)
        self.grad_ref = g("grad_ref", 1)
        self.allowance = g("allowance", 10)
        self.setting = g("setting", 5 if config.data.dataset == "KITTI360_im_8batch" else 7)

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize()

    def load_score(self):
        if self._score is not None:
            return self._score
        c = self.config
        net = ScoreNet(H=c.data.image_size, W=c.data.image_width, ngf=c.model.ngf, channels=c.data.channels,
                       num_classes=c.model.num_classes, precision=getattr(self.args, "precision", "fp32x3"))
        ckpt = getattr(self.args, "ckpt", None) or REF_CKPT
        if os.path.exists(ckpt):
            logging.info("loading checkpoint %s (EMA shadow applied: %s)", ckpt, c.model.ema)
            states = torch.load(ckpt, map_location="cpu", weights_only=True)
            net.load_state_dict(states[0], states[-1] if c.model.ema else None)
        else:
            logging.warning("checkpoint %s not found: using synthetic random-init weights", ckpt)
            net.load_state_dict(self._synthetic_sd())
        return net

    def _synthetic_sd(self):
        """Synthetic weights with the model's sigma buffer of THIS config: NCSN registers
        get_sigmas(config) (ncsnv2.py:430), and the score is divided by it (ncsnv2.py:516)."""
        c = self.config
        sd = synthetic_state_dict(c.model.ngf, c.data.channels, c.model.num_classes)
        sd["sigmas"] = get_sigmas_np(c.model.sigma_begin, c.model.sigma_end, c.model.num_classes,
                                     getattr(c.model, "sigma_dist", "geometric"))
        return sd

    def _png(self, grid_views, name, nrow):
        """make_grid + save_image of a [2B',3,H,W] layout (kitti:658-661)."""
        save_image(make_grid(grid_views.detach().float().cpu(), max(nrow, 1)), os.path.join(self.args.image_folder, name))

    def _batch_source(self, ds, B, aB, H, W):
        """bi -> the DataLoader's 9-tuple for batch bi (kitti:514-538)."""
        root = getattr(self.args, "kitti_root", None)
        if not root:
            return lambda bi: synthetic_batch(bi, B, aB, H, W, seed=getattr(self.args, "seed", 1234))
        dset = kitti360.get_dataset(ds, None, self.config, split="test", root=root, device=self.device)
        order = iter(kitti360.MySampler(kitti360.val_size(root, aB), aB, random=False))

        def fetch(bi):
            b = list(kitti360.collate([dset[next(order)] for _ in range(B)]))
            b[4], b[5] = b[4].reshape(B, 4, 4), b[5].reshape(B, 4, 4)   # [B,1,4,4] -> [B,4,4]
            return tuple(b)
        return fetch

    def _active_group(self, n_mega, world):
        """The process group of the ranks that hold megabatches (they share tooHigh), created once
        per active set and reused by later sample() calls (every rank joins new_group); None on one
        process.  Ranks without megabatches idle through the sampling calls."""
        if world <= 1:
            return None
        active = tuple(r for r in range(world) if shard_megabatches(n_mega, r, world)[1] > shard_megabatches(n_mega, r, world)[0])
        cache = self.__dict__.setdefault("_groups", {})
        if active not in cache:
            cache[active] = torch.distributed.group.WORLD if len(active) == world else torch.distributed.new_group(list(active))
        return cache[active]

    def _gather(self, t, world):
        """Rank-ordered concatenation of every rank's [n, ...] CPU tensor (None = no views)."""
        if world == 1:
            return t
        objs = [None] * world
        torch.distributed.all_gather_object(objs, None if t is None else t.numpy())
        return torch.from_numpy(np.concatenate([o for o in objs if o is not None]))

    def sample(self):
        if self.config.data.dataset == "kitti360_im_SceneCompletion":
            return self.sample_completion()
        c = self.config
        rank, world = _dist()
        B, aB = c.sampling.batch_size, c.sampling.actualBatchSize
        H, W = c.data.image_size, c.data.image_width
        n_mega = B // aB
        ds = c.data.dataset
        kitti = ds == "KITTI360_im_8batch"
        if not kitti and ds not in ("KITTI360_im_AllForOne", "KITTI360_im_simultaneous_densification"):
            raise NotImplementedError(f"dataset {ds} is outside the simultaneous-sampling path")
        score = self.load_score()
        sigmas = get_sigmas_np(c.model.sigma_begin, c.model.sigma_end, c.model.num_classes, c.model.sigma_dist)
        ex = torch.from_numpy(np.broadcast_to(synthetic.exist_mask(H, W), (B, H, W)).copy())
        folder = self.args.image_folder
        ck = c.sampling.ckpt_id
        n_batches = getattr(self.args, "num_batches", None) or 1
        time_taken = np.zeros(aB)
        end_point, to_add = aB, 0
        if ds == "KITTI360_im_simultaneous_densification":   # AllForOne:553-558
            end_point, to_add = 2, aB - 2
        m0, m1 = shard_megabatches(n_mega, rank, world)
        group = self._active_group(n_mega, world)
        writer = rank == 0
        fetch = self._batch_source(ds, B, aB, H, W)
        for bi in range(n_batches):
            (ref_full, mask_full, sky_full, idx_full, toWorld_full, fromWorld_full, goal, toOG,
             save_arr) = fetch(bi)
            save_num = "".join(str(int(save_arr[m * aB])) + "_" for m in range(n_mega))
            png_id = str(bi) if kitti else save_num      # kitti names the PNGs by batchesToDo (kitti:534,661)
            if writer:
                np.save(os.path.join(folder, "toWorld_" + save_num), toWorld_full.numpy())
                np.save(os.path.join(folder, "fromWorld_" + save_num), toOG.numpy())
            for do in range(end_point):
                init = torch.rand(B, c.data.channels, H, W, device=self.device)   # same seed on every rank
                ref = ref_full.float().to(self.device)
                mask = mask_full.int().to(self.device)
                sky, toWorld, fromWorld = sky_full.clone(), toWorld_full.clone(), fromWorld_full.clone()
                if do == 0 and writer:
                    inp = to_grid_layout(inverse_data_transform(ref_full * mask_full))
                    self._png(inp, f"{do}_{png_id}_Input_image_grid_{ck}.png", int(np.sqrt(B)))
                    np.save(os.path.join(folder, f"{do}_{save_num}_Input_completion_{ck}.pth"), inp.numpy())
                    # kitti saves the goal scans (kitti:678-694); AllForOne re-saves the masked
                    # input as "GT" (AllForOne:667-711, the second transpose is skipped) -- kept.
                    gt = to_grid_layout(inverse_data_transform(goal if kitti else ref_full * mask_full))
                    self._png(gt, f"{do}_{png_id}_GT_image_grid_{ck}.png", int(np.sqrt(B)))
                    np.save(os.path.join(folder, f"{do}_{save_num}_GT_completion_{ck}.pth"), gt.numpy())
                    np.save(os.path.join(folder, f"{do}_{save_num}_SKY_{ck}.pth"), sky_full.numpy())
                baseline = (do == aB - 1) if kitti else (do + to_add == aB - 1)
                k = do + 2 if (do + to_add) < aB - 2 else aB
                if baseline and not kitti:
                    k = 1                                   # AllForOne baseline: first view of each megabatch
                if baseline and kitti:
                    k = aB                                  # kitti baseline runs on the whole batch (kitti:711-716)
                if k < aB:
                    init, ref, mask = (_first_views(t, n_mega, aB, k) for t in (init, ref, mask))
                    sky, toWorld, fromWorld = (_first_views(t, n_mega, aB, k) for t in (sky, toWorld, fromWorld))
                n_views = init.shape[0]
                v0, v1 = m0 * k, m1 * k                     # this rank's views (whole megabatches)
                sl = slice(v0, v1)
                self._sync()
                t0 = time.time()
                outs = None
                if v1 > v0:
                    common = dict(noise_views=(v0, n_views), ops=self.ops)
                    if baseline:
                        outs, _ = anneal_Langevin_dynamics_inpainting(
                            init[sl], ref[sl], mask[sl], score, sigmas, c.sampling.n_steps_each, c.sampling.step_lr,
                            denoise=c.sampling.denoise, grad_ref=1, sampling_step=4, **common)
                    elif kitti:
                        outs, _, _ = anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti(
                            init[sl], ref[sl], mask[sl], sky[sl], None, self.start_step, self.setting, self.allowance,
                            score, sigmas, fromWorld[sl], toWorld[sl], k, c.sampling.n_steps_each, c.sampling.step_lr,
                            existMask=ex[sl], denoise=c.sampling.denoise, grad_ref=self.grad_ref,
                            correlation_coefficient=self.cc, sampling_step=4, dist_group=group, **common)
                    else:
                        mods = torch.from_numpy(np.array(c.data.modifications))
                        outs, _, _ = anneal_Langevin_dynamics_inpainting_simultaneous_basic(
                            init[sl], ref[sl], mask[sl], sky[sl], None, self.start_step, self.setting, score, sigmas,
                            mods, k, c.sampling.n_steps_each, c.sampling.step_lr, existMask=ex[sl],
                            denoise=c.sampling.denoise, grad_ref=self.grad_ref, correlation_coefficient=self.cc,
                            sampling_step=4, dist_group=group, **common)
                final = self._gather(None if outs is None else outs[-1], world)
                shared = None if kitti else self._gather(None if outs is None else outs[-2], world)
                self._sync()
                time_taken[do] += time.time() - t0
                if not writer:
                    continue
                logging.info("--- %s seconds --- (doThis %d, %d views)", time_taken[do] / (bi + 1), do, n_views)
                np.save(os.path.join(folder, f"{do}_{save_num}_TimeTaken.npy"), time_taken[do])
                # grid width: sqrt of the views sampled (kitti:859-870, AllForOne:946-991)
                if baseline and not kitti:
                    nrow = int(np.sqrt(1 * n_mega))
                elif do + to_add < aB - 2:
                    nrow = int(np.sqrt((do + 2) * n_mega))
                else:
                    nrow = int(np.sqrt(B))
                sample = inverse_data_transform(final.view(n_views, c.data.channels, H, W))
                self._png(to_grid_layout(sample), f"{do}_{png_id}_Masked_image_grid_{ck}.png", nrow)
                np.save(os.path.join(folder, f"{do}_{save_num}_Masked_completion_{ck}.pth"),
                        to_grid_layout(sample).numpy())
                if not kitti:   # AllForOne:971-988: all_outputs[-2] (last merge image / denoised)
                    shared = inverse_data_transform(shared.view(n_views, c.data.channels, H, W))
                    self._png(to_grid_layout(shared), f"{do}_{png_id}_Shared_image_grid_initial{ck}.png", nrow)
                    np.save(os.path.join(folder, f"{do}_{save_num}_Shared_completion_initial{ck}.pth"),
                            to_grid_layout(shared).numpy())

    # ------------------------------------------------------------------------------ scene completion
    def _completion_source(self, B, aB, H, W):
        """bi -> the DataLoader's 6-tuple (real, notmask, notsky, index, names, origins) for batch
        bi: the SSC dataset of sdp.completion with --kitti_root (MySampler(valSize, actualBatchSize,
        random=False), Completion:500-504), else procedural views (origins = the view positions)."""
        from . import completion
        root = getattr(self.args, "kitti_root", None)
        if not root:
            seed = getattr(self.args, "seed", 1234)

            def synth(bi):
                sc = synthetic.scene_views(B, H, W, seed=seed + 7919 * bi)
                ref, mask = torch.from_numpy(sc["ref"]), torch.from_numpy(sc["mask"])
                origins = torch.from_numpy(sc["toWorld"][:, :3, 3]).unsqueeze(1)
                idx = torch.zeros(B, 1, H, W, dtype=torch.float64)
                # (the dataset's masks come back logical_not-ed: True = known pixel / not sky)
                return ref.double(), mask.bool(), torch.from_numpy(sc["sky"]), idx, [f"{bi:06d}"] * B, origins
            return synth, 1
        dset = completion.kitti360_im_SceneCompletion(None, self.config, split="test", root=root, device=self.device)
        n_val = completion.val_size(root)
        order = iter(kitti360.MySampler(n_val, aB, random=False))

        def fetch(bi):
            return completion.collate([dset[next(order)] for _ in range(B)])
        return fetch, n_val

    def sample_completion(self):
        """runners/ncsn_runner_Completion.py:468-940 (inpainting, final_only): per batch of
        sampling.batch_size views, doThis 0 saves the inputs (Input grid/npy, SKY, ORIGINS) and
        samples nothing; doThis 1 runs the origin-offset simultaneous sampler with the dataset's
        per-view origins (startStep 2, setting 7, correlation 0.01, grad_ref 1, Completion:548-566)
        and saves TimeTaken, the Masked and the Shared (last merge) images.  Quirks kept: the
        dataset's mask (True = known after logical_not) multiplies the input as in the reference,
        TimeTaken starts at 999999 (L512), the Shared files are named by the batch counter."""
        c = self.config
        rank, world = _dist()
        B, aB = c.sampling.batch_size, c.sampling.actualBatchSize
        H, W = c.data.image_size, c.data.image_width
        score = self.load_score()
        sigmas = get_sigmas_np(c.model.sigma_begin, c.model.sigma_end, c.model.num_classes, c.model.sigma_dist)
        ex = torch.from_numpy(np.broadcast_to(synthetic.exist_mask(H, W), (B, H, W)).copy())
        folder = self.args.image_folder
        ck = c.sampling.ckpt_id
        fetch, n_val = self._completion_source(B, aB, H, W)
        nb = getattr(self.args, "num_batches", None)
        # --num_batches 0 (or -1) = the whole validation split, as the reference iterates its dataloader
        n_batches = n_val if nb is not None and nb <= 0 else min(nb or 1, n_val)
        time_taken = np.zeros(max(n_val, 2)) + 999999
        writer = rank == 0
        n_mega = B // aB
        m0, m1 = shard_megabatches(n_mega, rank, world)
        group = self._active_group(n_mega, world)     # ranks without megabatches idle, as in sample()
        for bi in range(n_batches):
            ref_full, mask_full, sky_full, idx_full, names, origins = fetch(bi)
            save_num = names[0]
            for do in range(2):
                init = torch.rand(B, c.data.channels, H, W, device=self.device)
                ref = ref_full.float().to(self.device)
                mask = mask_full.int().to(self.device)
                refer = to_grid_layout(inverse_data_transform(ref_full * mask_full))
                if do == 0:
                    if writer:
                        self._png(refer, f"{do}_{save_num}_Input_image_grid_{ck}.png", int(np.sqrt(B)))
                        np.save(os.path.join(folder, f"{do}_{save_num}_Input_completion_{ck}.pth"), refer.numpy())
                        np.save(os.path.join(folder, f"{do}_{save_num}_SKY_{ck}.pth"), sky_full.numpy())
                        np.save(os.path.join(folder, f"{do}_{save_num}_ORIGINS_{ck}.pth"), origins.numpy())
                    continue
                mods = torch.squeeze(origins).reshape(B, 3)
                sl = slice(m0 * aB, m1 * aB)
                self._sync()
                t0 = time.time()
                outs = None
                if m1 > m0:
                    outs, _, _ = anneal_Langevin_dynamics_inpainting_simultaneous_basic(
                        init[sl], ref[sl], mask[sl], sky_full[sl], None, 2, 7, score, sigmas, mods, aB,
                        c.sampling.n_steps_each, c.sampling.step_lr, existMask=ex[sl], denoise=c.sampling.denoise,
                        grad_ref=1, correlation_coefficient=0.01, sampling_step=4, dist_group=group,
                        noise_views=(sl.start, B), ops=self.ops)
                final = self._gather(None if outs is None else outs[-1], world)
                shared = self._gather(None if outs is None else outs[-2], world)
                self._sync()
                time_taken[do] += time.time() - t0
                if not writer:
                    continue
                np.save(os.path.join(folder, f"{do}_{save_num}_TimeTaken.npy"), time_taken[do])
                sample = to_grid_layout(inverse_data_transform(final.view(B, c.data.channels, H, W)))
                initial = to_grid_layout(inverse_data_transform(shared.view(B, c.data.channels, H, W)))
                nrow = int(np.sqrt(B))
                self._png(sample, f"{do}_{save_num}_Masked_image_grid_{ck}.png", nrow)
                np.save(os.path.join(folder, f"{do}_{save_num}_Masked_completion_{ck}.pth"), sample.numpy())
                self._png(initial, f"{do}_{bi}_Shared_image_grid_initial{ck}.png", nrow)
                np.save(os.path.join(folder, f"{do}_{bi}_Shared_completion_initial{ck}.pth"), initial.numpy())

    # ------------------------------------------------------------------------------ training
    def _train_source(self, Bt, rank, world):
        """Training batches of the (X, mask, sky) triple the loop unpacks (kitti:179).  The
        datasets now return the 9-tuple of kitti360_im_8Batch.py:304 (the reference's 3-tuple
        return is commented out, kitti360_im_simultenous_densification.py:338-339), so its first
        three items are taken -- the reference's loop would fail to unpack it.  Ranks draw
        disjoint batches (rank r takes batches r, r + world, ...)."""
        c = self.config
        H, W = c.data.image_size, c.data.image_width
        root = getattr(self.args, "kitti_root", None)
        if not root:
            seed = getattr(self.args, "seed", 1234)

            def synth(i):
                sc = synthetic.scene_views(Bt, H, W, seed=seed + 104729 * (i * world + rank))
                ref, mask = torch.from_numpy(sc["ref"]), torch.from_numpy(sc["mask"])
                return ref * mask, mask, torch.from_numpy(sc["sky"])
            return synth
        dset = kitti360.get_dataset(c.data.dataset, None, c, split="train", root=root, device=self.device)
        n_batches = len(dset) // Bt
        state = {"it": None}

        def fetch(i):
            if state["it"] is None:
                state["it"] = iter(kitti360.MySampler(n_batches, Bt, random=True))
            items = []
            for _ in range(Bt * world):           # one global batch; this rank keeps its slice
                try:
                    items.append(next(state["it"]))
                except StopIteration:
                    state["it"] = iter(kitti360.MySampler(n_batches, Bt, random=True))
                    items.append(next(state["it"]))
            b = kitti360.collate([dset[j] for j in items[rank * Bt:(rank + 1) * Bt]])
            return b[0], b[1], b[2]
        return fetch

    def _test_source(self, Bt):
        """Test batches of the every-100-steps EMA evaluation (kitti:84-95, 247-251): the test split
        of the dataset (``get_dataset``'s second return) through its own MySampler iterator, never
        the training iterator.  Only rank 0 evaluates, so the draws (the sampler shuffles and every
        item's roll come from the global np.random stream) run on an np.random state of their own
        (seeded once, carried from evaluation to evaluation) swapped in around each draw: the ranks'
        training streams stay in lockstep, their global-batch slices disjoint, and the evaluation
        never re-draws the numbers the next training batch will draw."""
        c = self.config
        H, W = c.data.image_size, c.data.image_width
        root = getattr(self.args, "kitti_root", None)
        if not root:
            seed = getattr(self.args, "seed", 1234)

            def synth(i):
                sc = synthetic.scene_views(Bt, H, W, seed=seed + 7919 * i + 1)
                ref, mask = torch.from_numpy(sc["ref"]), torch.from_numpy(sc["mask"])
                return ref * mask, mask, torch.from_numpy(sc["sky"])
            return synth
        dset = kitti360.get_dataset(c.data.dataset, None, c, split="test", root=root, device=self.device)
        n_batches = max(1, len(dset) // Bt)
        eval_seed = (getattr(self.args, "seed", 1234) * 1000003 + 0x5EED) % (2 ** 32)
        state = {"it": None, "rng": np.random.RandomState(eval_seed).get_state()}

        def fetch(i):
            saved = np.random.get_state()
            np.random.set_state(state["rng"])
            try:
                items = []
                for _ in range(Bt):
                    try:
                        if state["it"] is None:
                            raise StopIteration
                        items.append(next(state["it"]))
                    except StopIteration:    # the reference re-creates test_iter on exhaustion
                        state["it"] = iter(kitti360.MySampler(n_batches, Bt, random=True))
                        items.append(next(state["it"]))
                b = kitti360.collate([dset[j] for j in items])
            finally:
                state["rng"] = np.random.get_state()
                np.random.set_state(saved)
            return b[0], b[1], b[2]
        return fetch

    def _batches_per_epoch(self, Bt, world):
        """One epoch = one pass of the DataLoader over the training split (kitti:172): the dataset's
        len // (Bt * world) global batches with --kitti_root; --num_batches overrides it (and is the
        epoch length of the procedural source, which has no length)."""
        nb = getattr(self.args, "num_batches", None)
        if nb:
            return nb
        root = getattr(self.args, "kitti_root", None)
        if root:
            c = self.config
            dset = kitti360.get_dataset(c.data.dataset, None, c, split="train", root=root, device=self.device)
            return max(1, len(dset) // (Bt * world))
        return 1

    def _initial_state_dict(self):
        """Random-init weights; with --resume_training the reference's shape-filtered partial
        load of a list-format checkpoint (kitti:115-128: keys whose shape matches replace the
        fresh weights, the rest stay random)."""
        sd = self._synthetic_sd()
        if getattr(self.args, "resume_training", False):
            path = getattr(self.args, "ckpt", None) or "diffusionNet/checkpoint_148.pth"
            states = torch.load(path, map_location="cpu", weights_only=True)
            loaded = 0
            for key, v in states[0].items():
                k = key[7:] if key.startswith("module.") else key
                if k in sd and tuple(v.shape) == tuple(np.shape(sd[k])):
                    sd[k] = v.detach().cpu().numpy() if torch.is_tensor(v) else v
                    loaded += 1
            logging.info("resume: %d of %d tensors loaded from %s (shape-filtered, strict=False)", loaded,
                         len(states[0]), path)
        return sd

    def _save_checkpoint(self, trainer, epoch, step):
        """torch.save([score.state_dict() ('module.'-prefixed, DataParallel), optimizer.state_dict(),
        epoch, step, ema_helper.state_dict()]) -- kitti:295-306, the list format of ncsn_runner.py:169-179
        that ``ScoreNet.load_checkpoint`` / the sampler's loader read back."""
        sd = {"module." + k: v.cpu() for k, v in trainer.state_dict().items()}
        sd["module.sigmas"] = trainer.net.sigmas.clone()
        optim = trainer.optimizer_state_dict()
        states = [sd, optim, epoch, step]
        if trainer.shadow is not None:
            states.append({k: v.cpu() for k, v in trainer.ema_state_dict().items()})
        os.makedirs(self.args.log_path, exist_ok=True)
        torch.save(states, os.path.join(self.args.log_path, "checkpoint_{}.pth".format(step)))
        torch.save(states, os.path.join(self.args.log_path, "checkpoint.pth"))

    def _test_loss(self, trainer, test_batch, sigmas, max_t, gen):
        """The every-100-steps EMA evaluation (kitti:240-290): the curriculum's timesteps on a
        test batch with the EMA weights, mean DSM loss (no gradient)."""
        from .training import dsm_loss_value
        c = self.config
        ema_net = ScoreNet(H=c.data.image_size, W=c.data.image_width, ngf=c.model.ngf, channels=c.data.channels,
                           num_classes=c.model.num_classes, precision=trainer.net.precision)
        sd = trainer.ema_state_dict() if trainer.shadow is not None else trainer.state_dict()
        sd["sigmas"] = trainer.net.sigmas
        ema_net.load_state_dict(sd)
        X, y, _ = (t.to(self.device) for t in test_batch)
        X, y = X.float(), y.float()
        sig = torch.as_tensor(sigmas, dtype=torch.float32, device=self.device)
        orig = X.clone()
        B = X.shape[0]
        X = X + torch.randn(X.shape, device=X.device, generator=gen) * sig[0] * torch.logical_not(y).int()
        total = 0.0
        for t in range(max_t):
            used = sig[t].view(1, 1, 1, 1).expand(B, 1, 1, 1)
            noise = torch.randn(X.shape, device=X.device, generator=gen) * used
            X = X + noise * y
            labels = torch.full((B,), t, device=X.device, dtype=torch.int64)
            grad = ema_net(X.contiguous(), labels)
            total += float(dsm_loss_value(grad, used, noise, y))
            step_size = float(c.sampling.step_lr * (float(sig[t]) / float(sig[-1])) ** 2)
            for _ in range(c.sampling.n_steps_each):
                pred = X + step_size * grad + torch.randn(X.shape, device=X.device, generator=gen) * np.sqrt(step_size * 2)
                X = orig * y + pred * torch.logical_not(y).int()
        return total / max_t

    def train(self):
        """kitti:83-348 on libsdp: per batch, the curriculum over maxTimeStepReachable (one more
        timestep every 20 true steps, kitti:292-294), each timestep = noise the known pixels at
        sigma[t], masked DSM loss, 5 Langevin predictions of the unknown pixels, backward, Adam,
        EMA; the EMA test loss every 100 steps; list-format checkpoints every snapshot_freq true
        steps (kitti:295-306); stops at n_iters.  Data parallel: one process per GPU, each rank its
        own batch of training.batch_size images, gradients averaged over ranks by one RCCL
        all-reduce (the reference's DataParallel splits one batch instead -- DESIGN §6)."""
        from .training import get_optimizer, train_step
        c = self.config
        rank, world = _dist()
        group = torch.distributed.group.WORLD if world > 1 else None
        if getattr(c.training, "snapshot_sampling", False):
            raise NotImplementedError("training.snapshot_sampling runs the unconditional anneal_Langevin_dynamics "
                                      "(models/__init__.py:20-57), which is outside this path")
        precision = getattr(self.args, "precision", "fp32x3")
        if precision == "fp32":
            raise ValueError("training runs in --precision fp32x3 or bf16")
        net = ScoreNet(H=c.data.image_size, W=c.data.image_width, ngf=c.model.ngf, channels=c.data.channels,
                       num_classes=c.model.num_classes, precision=precision)
        net.load_state_dict(self._initial_state_dict())
        trainer = get_optimizer(c, net, dist_group=group)
        sigmas = get_sigmas_np(c.model.sigma_begin, c.model.sigma_end, c.model.num_classes, c.model.sigma_dist)
        sig = torch.as_tensor(sigmas, dtype=torch.float32, device=self.device)
        Bt = c.training.batch_size
        source = self._train_source(Bt, rank, world)
        test_source = self._test_source(Bt) if rank == 0 else None
        gen = torch.Generator(device=self.device).manual_seed(getattr(self.args, "seed", 1234) + rank)
        max_epochs = getattr(self.args, "max_epochs", None) or getattr(c.training, "n_epochs", 500000)
        batches_per_epoch = self._batches_per_epoch(Bt, world)
        step = true_step = 0
        max_t = 1
        self.losses = []
        for epoch in range(max_epochs):
            for i in range(batches_per_epoch):
                step += 1
                X, mask, sky = source(epoch * batches_per_epoch + i)
                X = X.float().to(self.device)
                mask = mask.float().to(self.device)
                original = X.clone()
                # max noise into the untrusted pixels (kitti:183-186)
                X = X + torch.randn(X.shape, device=X.device, generator=gen) * sig[0] * torch.logical_not(mask).int()
                for t in range(max_t):
                    true_step += 1
                    loss, X = train_step(trainer, X, original, mask, sigmas, t, c.sampling.step_lr,
                                         c.sampling.n_steps_each, c.training.anneal_power, generator=gen)
                    lv = float(loss)
                    self.losses.append(lv)
                    if rank == 0:
                        logging.info("step: {}, timestep: {}, loss: {}".format(step, t, lv))
                    if step >= c.training.n_iters:
                        return 0
                    if step % 100 == 0 and t == 0 and rank == 0:
                        tl = self._test_loss(trainer, test_source(step // 100), sigmas, max_t, gen)
                        logging.info("step: {}, test_loss: {}".format(step, tl))
                    if true_step % 20 == 0 and max_t < len(sigmas):
                        max_t += 1
                    if true_step % c.training.snapshot_freq == 0 and rank == 0:
                        self._save_checkpoint(trainer, epoch, step)
        return 0
