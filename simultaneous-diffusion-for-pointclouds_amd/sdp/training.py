"""DSM training of the score network on libsdp (BASELINE config 5).

Mirrors the reference's training interface:
  * ``anneal_dsm_score_estimation_with_mask`` -- LiDARGen/losses/dsm.py:67-119 (same
    arguments; returns ``(loss, scores)``), computed by ``sdp_net_forward_train`` +
    ``sdp_dsm_loss``;
  * ``Trainer.backward()`` -- ``loss.backward()`` (runners/ncsn_runner_kitti_simultaneous.py:230)
    through ``sdp_net_backward``;
  * ``Trainer.step()`` -- ``optimizer.step()`` of ``get_optimizer`` (losses/__init__.py:3-13:
    Adam with weight_decay / amsgrad, RMSprop, SGD with momentum 0.9) and ``EMAHelper.update``
    (models/ema.py:16-21) in one fused kernel, then the packed conv weights are rebuilt on the
    device;
  * ``train_step`` -- one inner-loop iteration of the kitti runner's ``train()``
    (runners/ncsn_runner_kitti_simultaneous.py:186-235).

Data-parallel training: one process per GPU; the flat gradient arena is averaged over the ranks
of ``dist_group`` in buckets whose RCCL all-reduces overlap the backward (sdp/gradreduce.py;
bf16 on the wire for bf16 training, the fp32 arena stays the master copy) -- the DDP equivalent of
the reference's DataParallel.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .scorenet import ScoreNet


class Trainer:
    """Device-resident training state of one ScoreNet: parameter arena (bound to the net),
    gradient arena, optimizer state and the EMA shadow, all in the net's parameter layout.

    ``optimizer``: "Adam" (betas (beta1, beta2), eps, weight_decay, amsgrad), "RMSProp"
    (torch.optim.RMSprop: alpha 0.99, eps 1e-8, weight_decay) or "SGD" (momentum 0.9) --
    the three optimizers of get_optimizer (losses/__init__.py:3-13)."""

    OPTIMIZERS = {"Adam": 0, "RMSProp": 1, "SGD": 2}

    def __init__(self, net: ScoreNet, lr: float = 1e-4, beta1: float = 0.9, beta2: float = 0.999,
                 eps: float = 1e-8, ema: bool = True, ema_mu: float = 0.999, device="cuda", dist_group=None,
                 optimizer: str = "Adam", weight_decay: float = 0.0, amsgrad: bool = False,
                 alpha: float = 0.99, momentum: float = 0.9, grad_wire_dtype=None, bucket_floats=None,
                 tape_bf16: bool = True):
        if net.precision not in ("fp32x3", "bf16"):
            raise ValueError("training runs in precision fp32x3 or bf16")
        # bf16 precision: the tape (activations, output gradients) in bf16 (sdp_net_set_tape); fp32x3 keeps
        # float32 tensors whatever this says
        net.set_tape(tape_bf16)
        if optimizer not in self.OPTIMIZERS:
            raise NotImplementedError("Optimizer {} not understood.".format(optimizer))   # losses/__init__.py:12-13
        L = _lib.lib()
        self.net, self.L = net, L
        self.optimizer = optimizer
        self.lr, self.beta1, self.beta2, self.eps = lr, beta1, beta2, eps
        self.weight_decay, self.amsgrad, self.alpha, self.momentum = float(weight_decay), bool(amsgrad), alpha, momentum
        self.ema, self.ema_mu = ema, ema_mu
        self.dist_group = dist_group
        # gradient all-reduce on the wire: fp32 by default, as the reference's DataParallel reduce
        # (an RCCL ring SUM in bf16 rounds the running sum at every hop, up to world-1 times);
        # grad_wire_dtype=torch.bfloat16 halves the bytes (59.4 MB) at that cost
        self.grad_wire_dtype = grad_wire_dtype or torch.float32
        self.bucket_floats = bucket_floats
        self._reducer = None
        n = _lib.SZ()
        _lib.check(L.sdp_net_param_arena_floats(net._h, _lib.C.byref(n)), "param_arena_floats")
        cnt = _lib.I()
        _lib.check(L.sdp_net_param_count(net._h, _lib.C.byref(cnt)), "param_count")
        self.layout = []
        key = _lib.C.create_string_buffer(256)
        off, numel = _lib.SZ(), _lib.SZ()
        for i in range(cnt.value):
            _lib.check(L.sdp_net_param_info(net._h, i, key, 256, _lib.C.byref(off), _lib.C.byref(numel)), "param_info")
            self.layout.append((key.value.decode(), off.value, numel.value))
        self.shapes = dict(net.param_shapes())
        self.params = torch.empty(n.value, dtype=torch.float32, device=device)
        _lib.check(L.sdp_net_bind_params(net._h, self.params.data_ptr(), _lib.stream()), "bind_params")
        self.grads = torch.zeros_like(self.params)
        # optimizer state buffers (torch's state names)
        names = {"Adam": ["exp_avg", "exp_avg_sq"] + (["max_exp_avg_sq"] if self.amsgrad else []),
                 "RMSProp": ["square_avg"], "SGD": ["momentum_buffer"]}[optimizer]
        self.opt_state = {k: torch.zeros_like(self.params) for k in names}
        self.exp_avg = self.opt_state.get("exp_avg")
        self.exp_avg_sq = self.opt_state.get("exp_avg_sq")
        self.shadow = self.params.clone() if ema else None       # EMAHelper.register (ema.py:10-14)
        self.steps = 0
        self._ws = {}
        self._dscore = None
        self._part = None
        self._B = None

    # ------------------------------------------------------------------ parameter views
    def named_parameters(self, arena: torch.Tensor | None = None):
        """(key, view) in the reference module's registration order (param_shapes), wherever the
        arena keeps the parameter: checkpoints keep the reference's key order."""
        a = self.params if arena is None else arena
        where = {k: (off, numel) for k, off, numel in self.layout}
        for k in self.shapes:
            off, numel = where[k]
            yield k, a[off:off + numel].view(self.shapes[k])

    def named_grads(self):
        return self.named_parameters(self.grads)

    def state_dict(self):
        return {k: v.detach().clone() for k, v in self.named_parameters()}

    def ema_state_dict(self):
        return {k: v.detach().clone() for k, v in self.named_parameters(self.shadow)}

    # ------------------------------------------------------------------ forward / loss / backward
    def set_tape(self, bf16: bool):
        """Switch the bf16 tape on or off (bf16 precision); the next forward re-sizes the workspace."""
        self.net.set_tape(bf16)
        self._ws.clear()

    def _workspace(self, B):
        ws = self._ws.get(B)
        if ws is None:
            n = _lib.SZ()
            _lib.check(self.L.sdp_net_train_workspace_size(self.net._h, B, _lib.C.byref(n)), "train_workspace_size")
            ws = torch.empty(n.value, dtype=torch.uint8, device=self.params.device)
            self._ws[B] = ws
        return ws

    def forward(self, x: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """scores = scorenet(x, labels) in training mode (keeps the tape for backward)."""
        net = self.net
        if not x.is_cuda or x.dtype != torch.float32 or x.shape[1:] != (net.channels, net.H, net.W):
            raise ValueError(f"Trainer.forward expects cuda float32 [B,{net.channels},{net.H},{net.W}]")
        x = x.contiguous()
        B = x.shape[0]
        labels = labels.to(device=x.device, dtype=torch.int64).contiguous()
        out = torch.empty_like(x)
        ws = self._workspace(B)
        _lib.check(self.L.sdp_net_forward_train(net._h, x.data_ptr(), labels.data_ptr(), out.data_ptr(), B,
                                                ws.data_ptr(), ws.numel(), _lib.stream()), "forward_train")
        self._B = B
        return out

    def dsm_loss(self, scores, used_sigmas, noise, masks, anneal_power=2.0):
        """Masked DSM loss of losses/dsm.py:78-93; keeps d loss / d scores for backward()."""
        B = scores.shape[0]
        n_img = scores[0].numel()
        sig = used_sigmas.reshape(B).to(device=scores.device, dtype=torch.float32).contiguous()
        noise = noise.to(dtype=torch.float32).contiguous()
        masks = masks.reshape(scores.shape).to(dtype=torch.float32).contiguous()
        self._dscore = torch.empty_like(scores)
        loss = torch.empty(1, dtype=torch.float32, device=scores.device)
        per = torch.empty(B, dtype=torch.float32, device=scores.device)
        if self._part is None or self._part.numel() < 2 * B * 64:
            self._part = torch.empty(2 * B * 64, dtype=torch.float32, device=scores.device)
        _lib.check(self.L.sdp_dsm_loss(scores.contiguous().data_ptr(), noise.data_ptr(), masks.data_ptr(),
                                       sig.data_ptr(), B, n_img, float(anneal_power), self._dscore.data_ptr(),
                                       loss.data_ptr(), per.data_ptr(), self._part.data_ptr(), _lib.stream()),
                   "dsm_loss")
        self.loss_per_sample = per
        return loss.view(())

    def zero_grad(self):
        self.grads.zero_()

    def reducer(self):
        """The bucketed gradient all-reduce over dist_group (sdp/gradreduce.py), built on first use."""
        if self._reducer is None:
            from .gradreduce import DEFAULT_BUCKET_FLOATS, BucketedGradReducer
            self._reducer = BucketedGradReducer(self.grads, self.layout, self.dist_group,
                                                self.bucket_floats or DEFAULT_BUCKET_FLOATS, self.grad_wire_dtype)
        return self._reducer

    def backward(self, dscore: torch.Tensor | None = None):
        """loss.backward(): gradient arena <- d loss / d parameters (averaged over ranks, the
        reduce of each bucket overlapping the rest of the backward)."""
        d = self._dscore if dscore is None else dscore.contiguous()
        if d is None or self._B is None:
            raise RuntimeError("Trainer.backward: run forward + dsm_loss first")
        ws = self._workspace(self._B)
        if self.dist_group is None:
            _lib.check(self.L.sdp_net_backward(self.net._h, d.data_ptr(), self._B, ws.data_ptr(), ws.numel(),
                                               self.grads.data_ptr(), _lib.stream()), "backward")
            return
        red = self.reducer()
        n = len(red.ends)
        ends = (_lib.SZ * n)(*red.ends)
        evs = (_lib.P * n)(*red.event_handles())
        _lib.check(self.L.sdp_net_backward_buckets(self.net._h, d.data_ptr(), self._B, ws.data_ptr(), ws.numel(),
                                                   self.grads.data_ptr(), n, ends, evs, _lib.stream()),
                   "backward_buckets")
        red.reduce(self.grads)

    def step(self):
        """optimizer.step() + ema_helper.update(score), then re-pack the conv weights."""
        self.steps += 1
        st = list(self.opt_state.values()) + [None, None]
        kind = self.OPTIMIZERS[self.optimizer]
        if kind == 0:
            b1, b2, eps = self.beta1, self.beta2, self.eps
        elif kind == 1:
            b1, b2, eps = 0.0, self.alpha, 1e-8          # torch.optim.RMSprop defaults (alpha, eps)
        else:
            b1, b2, eps = self.momentum, 0.0, 0.0
        ptr = lambda t: t.data_ptr() if t is not None else None
        _lib.check(self.L.sdp_optim_ema_step(kind, self.params.data_ptr(), self.grads.data_ptr(), ptr(st[0]),
                                             ptr(st[1]), ptr(st[2]), ptr(self.shadow), self.params.numel(),
                                             self.lr, b1, b2, eps, self.weight_decay, self.steps, self.ema_mu,
                                             _lib.stream()), "optim_ema_step")
        _lib.check(self.L.sdp_net_repack(self.net._h, _lib.stream()), "repack")

    def optimizer_state_dict(self):
        """optimizer.state_dict() in torch's format: per-parameter state keyed by the index of the
        parameter in the module's parameters() order (NCSN_LiDAR_small registration order, the
        order of sdp.weights.param_spec), independent of the device arena's layout."""
        where = {k: (off, numel) for k, off, numel in self.layout}
        state = {}
        for i, k in enumerate(self.shapes):
            off, numel = where[k]
            e = {n: t[off:off + numel].view(self.shapes[k]).cpu() for n, t in self.opt_state.items()}
            if self.optimizer != "SGD":
                e["step"] = torch.tensor(float(self.steps))
            state[i] = e
        group = {"lr": self.lr, "weight_decay": self.weight_decay, "params": list(range(len(self.shapes)))}
        if self.optimizer == "Adam":
            group.update(betas=(self.beta1, self.beta2), eps=self.eps, amsgrad=self.amsgrad)
        elif self.optimizer == "RMSProp":
            group.update(alpha=self.alpha, eps=1e-8, momentum=0, centered=False)
        else:
            group.update(momentum=self.momentum, dampening=0, nesterov=False)
        return {"state": state, "param_groups": [group]}


def anneal_dsm_score_estimation_with_mask(scorenet: Trainer, perturbed_samples, used_sigmas, noise, masks, sky,
                                          sigmas, labels=None, anneal_power=2., hook=None):
    """losses/dsm.py:67-119 on libsdp.  ``scorenet`` is a Trainer; returns (loss, scores) and
    leaves d loss / d scores in the trainer for ``scorenet.backward()`` (loss.backward())."""
    B = perturbed_samples.shape[0]
    if labels is None:
        labels = torch.randint(0, len(sigmas), (B,), device=perturbed_samples.device)
    if used_sigmas is None:
        used_sigmas = sigmas[labels].view(B, *([1] * len(perturbed_samples.shape[1:])))
        noise = torch.randn_like(perturbed_samples) * used_sigmas
        perturbed_samples = perturbed_samples + noise
    scores = scorenet.forward(perturbed_samples.float(), labels)
    loss = scorenet.dsm_loss(scores, used_sigmas, noise, masks, anneal_power)
    if hook is not None:
        hook(scorenet.loss_per_sample, labels)
    return loss, scores


def dsm_loss_value(scores, used_sigmas, noise, masks, anneal_power=2.0):
    """losses/dsm.py:80-93 as device torch ops, for evaluation (no gradient): the runner's test loss."""
    B = scores.shape[0]
    target = -1 / (used_sigmas ** 2) * noise
    m = masks.reshape(B, -1).float()
    diff = m * (scores.reshape(B, -1) - target.reshape(B, -1))
    loss = 0.5 * (diff ** 2).sum(dim=-1) * (scores[0].numel() / m.sum()) * used_sigmas.reshape(B) ** anneal_power
    return loss.mean()


def get_optimizer(config, net: ScoreNet, **kw) -> Trainer:
    """losses/__init__.py:3-13: Adam(lr, weight_decay, betas=(beta1, 0.999), amsgrad, eps),
    RMSprop(lr, weight_decay), SGD(lr, momentum=0.9); anything else raises NotImplementedError."""
    o = config.optim
    ema = bool(getattr(config.model, "ema", True))
    common = dict(ema=ema, ema_mu=getattr(config.model, "ema_rate", 0.999), **kw)
    if o.optimizer == "Adam":
        return Trainer(net, lr=o.lr, beta1=o.beta1, beta2=0.999, eps=o.eps, optimizer="Adam",
                       weight_decay=getattr(o, "weight_decay", 0.0), amsgrad=getattr(o, "amsgrad", False), **common)
    if o.optimizer == "RMSProp":
        return Trainer(net, lr=o.lr, optimizer="RMSProp", weight_decay=getattr(o, "weight_decay", 0.0), **common)
    if o.optimizer == "SGD":
        return Trainer(net, lr=o.lr, optimizer="SGD", momentum=0.9, **common)
    raise NotImplementedError("Optimizer {} not understood.".format(o.optimizer))


def train_step(trainer: Trainer, X, originalX, mask, sigmas, timestep: int, step_lr: float, n_steps_each: int,
               anneal_power: float = 2.0, generator=None):
    """One timestep of the kitti runner's training loop (ncsn_runner_kitti_simultaneous.py:186-235):
    noise the known pixels at sigma[timestep], DSM loss + backward + Adam + EMA, and advance X
    by n_steps_each Langevin predictions of the unknown pixels.  Returns (loss, X_next)."""
    B = X.shape[0]
    labels = torch.full((B,), timestep, device=X.device, dtype=torch.int64)
    sig = torch.as_tensor(sigmas, dtype=torch.float32, device=X.device)
    used = sig[labels].view(B, 1, 1, 1)
    noise = torch.randn(X.shape, device=X.device, generator=generator) * used
    X = X + noise * mask
    loss, grad = anneal_dsm_score_estimation_with_mask(trainer, X, used, noise, mask, None, sig, labels, anneal_power)
    step_size = float(step_lr * (float(sig[timestep]) / float(sig[-1])) ** 2)
    notm = torch.logical_not(mask).int()
    for _ in range(n_steps_each):
        noise2 = torch.randn(X.shape, device=X.device, generator=generator)
        prediction = X + step_size * grad + noise2 * np.sqrt(step_size * 2)
        X = originalX * mask + prediction * notm
    trainer.zero_grad()
    trainer.backward()
    trainer.step()
    return loss, X
