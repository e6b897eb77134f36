"""World-size-2 gloo test of the bucketed data-parallel gradient average (sdp/gradreduce.py, the
config-5 replacement of DataParallel's gradient reduce, runners/ncsn_runner_kitti_simultaneous.py:
104,481): buckets at parameter boundaries covering the arena, and the bucketed average equal to the
single-process average of the ranks' gradients -- exactly with an fp32 wire, within bf16 rounding
(each rank's value and the sum rounded to bf16: |err| <= 2^-7 * mean(|g_r|)) with a bf16 wire.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from sdp.gradreduce import BucketedGradReducer, bucket_ends

# a parameter layout like the arena's: (key, offset, numel), 64-float aligned offsets
SIZES = [589824, 256, 256, 256, 294912, 128, 128, 128, 147456, 2304, 2, 4608, 128, 128, 589824, 256]


def layout():
    out, off = [], 0
    for i, n in enumerate(SIZES):
        out.append((f"p{i}", off, n))
        off += (n + 63) // 64 * 64
    return out, off


def rank_grads(rank, n):
    g = torch.from_numpy(np.random.default_rng(1000 + rank).standard_normal(n).astype(np.float32))
    return g * torch.linspace(1e-3, 10.0, n)       # a range of magnitudes, as gradients have


def test_bucket_ends_cut_at_parameter_boundaries():
    lay, n = layout()
    starts = {off for _, off, _ in lay}
    for bf in (1, 100000, 300000, 1 << 30):
        ends = bucket_ends(lay, n, bf)
        assert ends[-1] == n and all(a < b for a, b in zip(ends, ends[1:]))
        assert all(e in starts for e in ends[:-1])
    assert len(bucket_ends(lay, n, 1 << 30)) == 1
    assert len(bucket_ends(lay, n, 1)) == len(lay)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, wire, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lay, n = layout()
        g = rank_grads(rank, n)
        red = BucketedGradReducer(g, lay, None, bucket_floats=300000, wire_dtype=wire)
        red.reduce(g)
        q.put((rank, len(red.ends), g.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
def test_bucketed_average_world2_gloo(wire):
    lay, n = layout()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, wire, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (nb, g)) for r, nb, g in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0, g1 = rank_grads(0, n).numpy(), rank_grads(1, n).numpy()
    want = (g0.astype(np.float64) + g1) / 2
    assert res[0][0] == res[1][0] == 4                      # bucket count at 300k floats
    np.testing.assert_array_equal(res[0][1], res[1][1])     # every rank holds the same average
    got = res[0][1].astype(np.float64)
    if wire == torch.float32:
        np.testing.assert_allclose(got, want, rtol=1e-7, atol=0)
    else:
        bound = 2.0 ** -7 * (np.abs(g0) + np.abs(g1)) / 2 + 1e-30
        assert np.all(np.abs(got - want) <= bound)
        assert np.abs(got - want).max() > 0                 # (it really went over the wire in bf16)
