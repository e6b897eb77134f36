"""Drop-in score network: ``scorenet(x, y)`` of NCSN_LiDAR_small backed by libsdp.

Mirrors the reference module's interface (LiDARGen/models/ncsnv2.py:420-518): called as
``net(x: float32 [B,2,H,W] cuda, y: int64 [B] cuda) -> float32 [B,2,H,W]``, with a
``state_dict``-compatible loader (same keys; a DataParallel ``module.`` prefix is stripped)
and the runner's EMA application (runners/ncsn_runner_kitti_simultaneous.py:472-489).
Every forward runs on the caller's current HIP stream through the C ABI.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .weights import param_spec, synthetic_state_dict


class ScoreNet:
    def __init__(self, H: int = 64, W: int = 1024, ngf: int = 128, channels: int = 2, num_classes: int = 232,
                 precision: str = "fp32x3"):
        L = _lib.lib()
        self.H, self.W, self.ngf, self.channels, self.num_classes = H, W, ngf, channels, num_classes
        self.precision = precision
        d = _lib.NetDesc(ngf, channels, H, W, num_classes, _lib.PREC[precision])
        h = _lib.P()
        _lib.check(L.sdp_net_create(_lib.C.byref(d), _lib.C.byref(h)), "net_create")
        self._h = h
        self._ws = {}
        self._ready = False
        self.sigmas = None

    # ------------------------------------------------------------------ parameters
    def load_state_dict(self, sd, ema_shadow=None):
        """Reference state_dict (optionally DataParallel-prefixed) [+ EMAHelper shadow]."""
        L = _lib.lib()
        sd = {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}
        if ema_shadow is not None:  # EMAHelper.ema: copy the shadow over the parameters (ema.py:23-28)
            sd.update({k[7:] if k.startswith("module.") else k: v for k, v in ema_shadow.items()})
        need = set(param_spec(self.ngf, self.channels)) | {"sigmas"}
        missing = need - set(sd)
        if missing:
            raise KeyError(f"missing parameters: {sorted(missing)[:5]} ...")
        for k in need:
            a = np.ascontiguousarray(np.asarray(sd[k].detach().cpu() if torch.is_tensor(sd[k]) else sd[k],
                                                dtype=np.float32))
            shape = (_lib.C.c_int64 * a.ndim)(*a.shape)
            _lib.check(L.sdp_net_set_param(self._h, k.encode(), a.ctypes.data, shape, a.ndim), "set_param " + k)
        _lib.check(L.sdp_net_finalize(self._h), "finalize")
        s = sd["sigmas"]
        self.sigmas = torch.as_tensor(np.asarray(s.cpu() if torch.is_tensor(s) else s, np.float32))
        self._ready = True
        return self

    def param_shapes(self):
        """(state_dict key, shape) of every learnable parameter (no 'sigmas' buffer)."""
        return param_spec(self.ngf, self.channels).items()

    def load_synthetic(self):
        return self.load_state_dict(synthetic_state_dict(self.ngf, self.channels, self.num_classes))

    def load_checkpoint(self, path):
        """LiDARGen checkpoint list [state_dict, optim, epoch, step, ema_shadow] (ncsn_runner.py:169-179)."""
        states = torch.load(path, map_location="cpu", weights_only=True)
        return self.load_state_dict(states[0], states[-1] if len(states) >= 5 else None)

    # ------------------------------------------------------------------ forward
    def workspace(self, B: int, device) -> torch.Tensor:
        key = (B, str(device))
        ws = self._ws.get(key)
        if ws is None:
            n = _lib.SZ()
            _lib.check(_lib.lib().sdp_net_workspace_size(self._h, B, _lib.C.byref(n)), "workspace_size")
            ws = torch.empty(n.value, dtype=torch.uint8, device=device)
            self._ws[key] = ws
        return ws

    def forward(self, x: torch.Tensor, y: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if not self._ready:
            raise RuntimeError("ScoreNet: load weights first")
        if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 or x.shape[1:] != (self.channels, self.H, self.W):
            raise ValueError(f"ScoreNet expects cuda float32 [B,{self.channels},{self.H},{self.W}], got "
                             f"{tuple(x.shape)} {x.dtype} {x.device}")
        x = x.contiguous()
        B = x.shape[0]
        y = y.to(device=x.device, dtype=torch.int64).contiguous()
        if out is None:
            out = torch.empty_like(x)
        ws = self.workspace(B, x.device)
        _lib.check(_lib.lib().sdp_net_forward(self._h, x.data_ptr(), y.data_ptr(), out.data_ptr(), B, ws.data_ptr(),
                                              ws.numel(), _lib.stream()), "net_forward")
        return out

    __call__ = forward

    def forward_langevin(self, x: torch.Tensor, y: torch.Tensor, ref: torch.Tensor, mask: torch.Tensor,
                         noise: torch.Tensor | None, seed: int, offset: int, step: float, nscale: float,
                         grad_ref: float, nan_to_num: bool, lik: torch.Tensor | None, absmax: torch.Tensor | None,
                         grad_out: torch.Tensor | None = None) -> None:
        """One Langevin step with the update fused into the net's last kernel
        (sdp_net_forward_langevin): x is updated in place exactly as ``forward`` followed by
        sdp_langevin_step would; grad_out (optional) receives the scores."""
        if not self._ready:
            raise RuntimeError("ScoreNet: load weights first")
        if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 or x.shape[1:] != (self.channels, self.H, self.W) \
                or not x.is_contiguous():
            raise ValueError(f"forward_langevin expects contiguous cuda float32 [B,{self.channels},{self.H},{self.W}] "
                             f"(updated in place), got {tuple(x.shape)} {x.dtype} {x.device}")
        for name, t, dt in (("ref", ref, torch.float32), ("mask", mask, torch.int32), ("noise", noise, torch.float32),
                            ("lik", lik, torch.float32), ("grad_out", grad_out, torch.float32)):
            if t is not None and (t.shape != x.shape or t.dtype != dt or not t.is_contiguous() or t.device != x.device):
                raise ValueError(f"forward_langevin: {name} must be contiguous {dt} {tuple(x.shape)} on {x.device}")
        if absmax is not None and (absmax.dtype != torch.int32 or absmax.device != x.device):
            raise ValueError("forward_langevin: absmax must be an int32 device tensor")
        B = x.shape[0]
        y = y.to(device=x.device, dtype=torch.int64).contiguous()
        ws = self.workspace(B, x.device)
        p = _lib.LangevinParams(ref.data_ptr(), mask.data_ptr(), _lib.ptr(noise), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                int(offset), float(step), float(nscale), float(grad_ref), 1 if nan_to_num else 0,
                                _lib.ptr(lik), _lib.ptr(absmax), _lib.ptr(grad_out))
        _lib.check(_lib.lib().sdp_net_forward_langevin(self._h, x.data_ptr(), y.data_ptr(), B, _lib.C.byref(p),
                                                       ws.data_ptr(), ws.numel(), _lib.stream()), "net_forward_langevin")

    def set_split(self, ways: int):
        """Run each forward as `ways` part-batch forwards on as many streams (0 = the default, 2;
        1 = off).  Results are identical; only the launch schedule changes."""
        _lib.check(_lib.lib().sdp_net_set_split(self._h, int(ways)), "set_split")
        self._ws.clear()                    # the workspace size depends on it

    def set_tape(self, bf16: bool):
        """bf16 precision, training: keep the tape (activations, output gradients) in bf16 (True, the
        default) or float32 (False).  Parameters, gradients and scores stay float32 either way."""
        _lib.check(_lib.lib().sdp_net_set_tape(self._h, 1 if bf16 else 0), "set_tape")

    # ------------------------------------------------------------------ measurement
    def profile(self, enable: bool = True):
        _lib.check(_lib.lib().sdp_net_profile_enable(self._h, 1 if enable else 0), "profile_enable")

    def profile_read(self):
        """{launch class: (launches, total_ms, flops_per_launch, algorithmic_bytes_per_launch)} of the
        forwards since the last read (conv classes and the memory-bound kernels)."""
        buf = _lib.C.create_string_buffer(1 << 16)
        n = _lib.I()
        _lib.check(_lib.lib().sdp_net_profile_read(self._h, buf, len(buf), _lib.C.byref(n)), "profile_read")
        out = {}
        for line in buf.value.decode().splitlines():
            cls, cnt, ms, fl, by = line.split("\t")
            out[cls] = (int(cnt), float(ms), float(fl), float(by))
        return out

    def eval(self):
        return self

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                _lib.lib().sdp_net_destroy(self._h)
                self._h = None
        except Exception:
            pass
