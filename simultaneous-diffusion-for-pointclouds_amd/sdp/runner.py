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
"""
from __future__ import annotations

import logging
import os
import time

import numpy as np
import torch

from . import kitti360, synthetic
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


def _first_views(t, n_mega, aB, k):
    """Keep the first k views of every megabatch (the reference's reshape-and-slice, kitti:720-739)."""
    shp = t.shape
    return t.reshape(n_mega, aB, -1)[:, :k].reshape((n_mega * k,) + tuple(shp[1:]))


class Runner:
    def __init__(self, args, config):
        self.args, self.config = args, config
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
            net.load_synthetic()
        return net

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

    def sample(self):
        c = self.config
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
        n_batches = getattr(self.args, "num_batches", 1)
        time_taken = np.zeros(aB)
        end_point, to_add = aB, 0
        if ds == "KITTI360_im_simultaneous_densification":   # AllForOne:553-558
            end_point, to_add = 2, aB - 2
        fetch = self._batch_source(ds, B, aB, H, W)
        for bi in range(n_batches):
            (ref_full, mask_full, sky_full, idx_full, toWorld_full, fromWorld_full, goal, toOG,
             save_arr) = fetch(bi)
            save_num = "".join(str(int(save_arr[m * aB])) + "_" for m in range(n_mega))
            png_id = str(bi) if kitti else save_num      # kitti names the PNGs by batchesToDo (kitti:534,661)
            np.save(os.path.join(folder, "toWorld_" + save_num), toWorld_full.numpy())
            np.save(os.path.join(folder, "fromWorld_" + save_num), toOG.numpy())
            for do in range(end_point):
                init = torch.rand(B, c.data.channels, H, W, device=self.device)
                ref = ref_full.float().to(self.device)
                mask = mask_full.int().to(self.device)
                sky, toWorld, fromWorld = sky_full.clone(), toWorld_full.clone(), fromWorld_full.clone()
                if do == 0:
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
                self._sync()
                t0 = time.time()
                if baseline:
                    outs, _ = anneal_Langevin_dynamics_inpainting(init, ref, mask, score, sigmas, c.sampling.n_steps_each,
                                                                  c.sampling.step_lr, denoise=c.sampling.denoise,
                                                                  grad_ref=1, sampling_step=4)
                elif kitti:
                    outs, _, _ = anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti(
                        init, ref, mask, sky, None, self.start_step, self.setting, self.allowance, score, sigmas,
                        fromWorld, toWorld, k, c.sampling.n_steps_each, c.sampling.step_lr, existMask=ex,
                        denoise=c.sampling.denoise, grad_ref=self.grad_ref, correlation_coefficient=self.cc,
                        sampling_step=4)
                else:
                    mods = torch.from_numpy(np.array(c.data.modifications))
                    outs, _, _ = anneal_Langevin_dynamics_inpainting_simultaneous_basic(
                        init, ref, mask, sky, None, self.start_step, self.setting, score, sigmas, mods, k,
                        c.sampling.n_steps_each, c.sampling.step_lr, existMask=ex, denoise=c.sampling.denoise,
                        grad_ref=self.grad_ref, correlation_coefficient=self.cc, sampling_step=4)
                self._sync()
                time_taken[do] += time.time() - t0
                logging.info("--- %s seconds --- (doThis %d, %d views)", time_taken[do] / (bi + 1), do, init.shape[0])
                np.save(os.path.join(folder, f"{do}_{save_num}_TimeTaken.npy"), time_taken[do])
                # grid width: sqrt of the views sampled (kitti:859-870, AllForOne:946-991)
                if baseline and not kitti:
                    nrow = int(np.sqrt(1 * n_mega))
                elif do + to_add < aB - 2:
                    nrow = int(np.sqrt((do + 2) * n_mega))
                else:
                    nrow = int(np.sqrt(B))
                sample = inverse_data_transform(outs[-1].view(init.shape[0], c.data.channels, H, W))
                self._png(to_grid_layout(sample), f"{do}_{png_id}_Masked_image_grid_{ck}.png", nrow)
                np.save(os.path.join(folder, f"{do}_{save_num}_Masked_completion_{ck}.pth"),
                        to_grid_layout(sample).numpy())
                if not kitti:   # AllForOne:971-988: all_outputs[-2] (last merge image / denoised)
                    shared = inverse_data_transform(outs[-2].view(init.shape[0], c.data.channels, H, W))
                    self._png(to_grid_layout(shared), f"{do}_{png_id}_Shared_image_grid_initial{ck}.png", nrow)
                    np.save(os.path.join(folder, f"{do}_{save_num}_Shared_completion_initial{ck}.pth"),
                            to_grid_layout(shared).numpy())
