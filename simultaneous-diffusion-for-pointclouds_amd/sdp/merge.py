"""Host side of the cross-view consistency merge (device work in csrc/merge.hip).

``Merger`` prepares the per-call static inputs once (poses or view origins, existMask,
sky, reference mask, workspace) and then runs one merge per Langevin step on device,
with no host synchronisation (tooHigh is read on device from the Langevin kernel's
max|x[:,0]| word).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def allforone_origins(modification_list) -> torch.Tensor:
    """models/__init__.py:221-231 evaluated with the same float32 torch ops: 10*sign(m) up to rounding."""
    og = torch.as_tensor(np.asarray(modification_list)).cpu()
    og = og.unsqueeze(-1).unsqueeze(-1)
    o = (torch.log2(torch.abs(og) + 1) / 6) * 1
    o = torch.pow(2, (o * 6)) - 1
    o = o / (og + 0.00000001) * 10
    return o[:, :, 0, 0].float().contiguous()


class Merger:
    def __init__(self, B: int, aB: int, H: int, W: int, device, exist, sky, refmask, *, toWorld=None, fromWorld=None,
                 origins=None, o_begin: int = 0, n_out: int | None = None):
        if B % aB:
            raise ValueError(f"batch {B} is not a multiple of actualBatchSize {aB}")
        self.B, self.aB, self.H, self.W = B, aB, H, W
        self.o_begin = o_begin
        self.n_out = B - o_begin if n_out is None else n_out
        dev = torch.device(device)
        self.variant = _lib.MERGE_POSES if origins is None else _lib.MERGE_ORIGINS
        if self.variant == _lib.MERGE_POSES:
            # the reference's torch.squeeze breaks B=1 (Appendix B.5); reshape instead
            self.toWorld = torch.as_tensor(toWorld).reshape(B, 4, 4).to(dev, torch.float64).contiguous()
            self.fromWorld = torch.as_tensor(fromWorld).reshape(B, 4, 4).to(dev, torch.float64).contiguous()
            self.origins = None
        else:
            self.toWorld = self.fromWorld = None
            self.origins = torch.as_tensor(origins)[:aB].to(dev, torch.float32).contiguous()
        ex = torch.as_tensor(exist)
        if ex.dim() == 2:
            ex = ex.unsqueeze(0).expand(aB, H, W)
        self.exist = ex[:aB].to(dev).to(torch.uint8).contiguous()
        self.sky = torch.as_tensor(sky).reshape(B, H, W).to(dev).to(torch.uint8).contiguous()
        self.refmask = torch.as_tensor(refmask).to(dev, torch.int32).contiguous()
        n = _lib.SZ()
        _lib.check(_lib.lib().sdp_merge_workspace_bytes(B, aB, self.n_out, H, W, _lib.C.byref(n)), "merge_ws")
        self.ws = torch.empty(n.value, dtype=torch.uint8, device=dev)

    def __call__(self, x: torch.Tensor, sigma, setting: int, allowance: float, cc: float, absmax: torch.Tensor,
                 new_images: torch.Tensor | None = None, absmax_event: torch.cuda.Event | None = None) -> None:
        """Correct x [B,2,H,W] in place (output views [o_begin, o_begin+n_out)).  ``absmax_event``: the
        final correction pass (the only reader of ``absmax``) waits for it (``AbsmaxAllReduce``)."""
        prm = _lib.MergeParams(self.variant, int(setting), float(np.float32(sigma)), float(allowance), float(cc))
        _lib.check(_lib.lib().sdp_consistency_merge_ev(
            x.data_ptr(), self.B, self.aB, self.o_begin, self.n_out, self.H, self.W,
            _lib.ptr(self.toWorld), _lib.ptr(self.fromWorld), _lib.ptr(self.origins),
            self.exist.data_ptr(), self.sky.data_ptr(), self.refmask.data_ptr(), _lib.C.byref(prm),
            absmax.data_ptr(), _lib.ptr(new_images), self.ws.data_ptr(), self.ws.numel(), _lib.stream(),
            absmax_event.cuda_event if absmax_event is not None else None), "merge")


class AbsmaxAllReduce:
    """tooHigh's global max|x[:,0]| over the ranks (KITTISampling.py:162; one 4-byte all_reduce(MAX)
    per merged step).  On GPUs the all_reduce runs on a side stream after the Langevin
    update that wrote the word, and the returned event is handed to ``Merger`` so that only the merge's
    final correction pass waits for it; the merge's projection and binning passes run meanwhile.  On
    CPU tensors (gloo) it is the plain blocking all_reduce and returns None."""

    def __init__(self, group=None):
        self.group = group
        self.comm = None
        self.event = None

    def __call__(self, absmax: torch.Tensor):
        dist = torch.distributed
        if not absmax.is_cuda:
            dist.all_reduce(absmax, op=dist.ReduceOp.MAX, group=self.group)
            return None
        if self.comm is None:
            self.comm = torch.cuda.Stream(device=absmax.device)
            self.event = torch.cuda.Event()
        self.comm.wait_stream(torch.cuda.current_stream(absmax.device))
        with torch.cuda.stream(self.comm):
            dist.all_reduce(absmax, op=dist.ReduceOp.MAX, group=self.group)
            self.event.record()
        # the next writer of absmax (the next step's zero_ on the current stream) is ordered after
        # the merge's correction pass, which waits for this event
        return self.event
