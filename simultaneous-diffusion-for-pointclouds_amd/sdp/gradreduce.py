"""Data-parallel gradient averaging in buckets, overlapped with the backward.

The reference trains under ``torch.nn.DataParallel`` (runners/ncsn_runner_kitti_simultaneous.py:104,
481), whose backward reduces the replicas' gradients onto GPU 0 before ``optimizer.step()``.  Here
each GPU is its own process and the gradient arena (one flat fp32 tensor in the parameter layout,
sdp_net_param_info) is averaged over the ranks with RCCL all-reduces:

* the arena is cut into buckets at parameter boundaries.  libsdp lays the arena out in the order
  the backward finishes the gradients (sdp_net_finalize), so bucket i is final as soon as the
  backward has passed its last layer; ``sdp_net_backward_buckets`` records a HIP event there;
* per bucket, a communication stream waits for that event, casts the bucket to the wire dtype
  (fp32 by default, the reference's reduce; bf16 on request: 59.4 MB on the wire for 29.7 M
  parameters instead of 118.8 MB, but a ring SUM in bf16 rounds the running sum at every hop),
  all-reduces it (SUM) and writes the average back into the fp32 arena.  The all-reduces of the
  early buckets run while the backward computes the later layers;
* invariant (train.hip TrainPlan::finished): no backward launch writes a parameter's gradient range
  after the bucket event that covers it, so the communication stream may read and rewrite a
  bucket while the backward runs on.  tests/test_gpu_training.py checks it by poisoning every
  finished bucket on the side stream and comparing the final gradients;
* the optimizer step waits for the communication stream (the fp32 arena stays the master copy:
  only the wire carries bf16).

On gloo / CPU tensors (the multi-process tests) the same buckets are reduced one after the other.
"""
from __future__ import annotations

import torch

DEFAULT_BUCKET_FLOATS = 8 << 20     # 8 M parameters = 32 MB of fp32 per all-reduce


def bucket_ends(layout, arena_floats: int, bucket_floats: int = DEFAULT_BUCKET_FLOATS):
    """Cut [0, arena_floats) into buckets of about ``bucket_floats`` at parameter boundaries.
    ``layout``: (key, offset, numel) in arena order.  Returns the increasing bucket ends."""
    starts = sorted(off for _, off, _ in layout)
    ends, cur = [], 0
    for s in starts[1:]:
        if s - cur >= bucket_floats:
            ends.append(s)
            cur = s
    ends.append(int(arena_floats))
    return ends


class BucketedGradReducer:
    """Averages ``grads`` (flat fp32, the parameter arena layout) over the ranks of ``group``."""

    def __init__(self, grads: torch.Tensor, layout, group=None, bucket_floats: int = DEFAULT_BUCKET_FLOATS,
                 wire_dtype: torch.dtype = torch.float32):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.ends = bucket_ends(layout, grads.numel(), bucket_floats)
        self.wire_dtype = wire_dtype
        self.cast = wire_dtype != grads.dtype
        self.wire = torch.empty(grads.numel(), dtype=wire_dtype, device=grads.device) if self.cast else None
        self.cuda = grads.is_cuda
        self.comm = torch.cuda.Stream(device=grads.device) if self.cuda else None
        self.events = [torch.cuda.Event() for _ in self.ends] if self.cuda else None

    def ranges(self):
        a = 0
        for b in self.ends:
            yield a, b
            a = b

    def event_handles(self):
        """hipEvent_t handles for sdp_net_backward_buckets (created on first use)."""
        hs = []
        for e in self.events:
            if e.cuda_event == 0:
                e.record()            # creates the event; the backward re-records it
            hs.append(e.cuda_event)
        return hs

    def reduce(self, grads: torch.Tensor, wait_events: bool = True) -> None:
        """Enqueue the bucket all-reduces (after each bucket's event when ``wait_events``) and make
        the current stream wait for the averaged arena."""
        dist = self.dist
        inv = 1.0 / self.world
        if not self.cuda:
            for a, b in self.ranges():
                t = self.wire[a:b].copy_(grads[a:b]) if self.cast else grads[a:b]
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
                grads[a:b].copy_(t).mul_(inv)
            return
        main = torch.cuda.current_stream(grads.device)
        if not wait_events:
            self.comm.wait_stream(main)
        works = []
        with torch.cuda.stream(self.comm):
            for i, (a, b) in enumerate(self.ranges()):
                if wait_events:
                    self.comm.wait_event(self.events[i])
                t = self.wire[a:b].copy_(grads[a:b]) if self.cast else grads[a:b]
                works.append((dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True), a, b))
            for w, a, b in works:
                w.wait()                  # the communication stream waits for this bucket's all-reduce
                if self.cast:
                    grads[a:b].copy_(self.wire[a:b])
                grads[a:b].mul_(inv)
        main.wait_stream(self.comm)
