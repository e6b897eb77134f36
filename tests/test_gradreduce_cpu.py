"""World-size-2 and -4 gloo tests of the bucketed data-parallel gradient average (sdp/gradreduce.py, the
config-5 replacement of DataParallel's gradient reduce, runners/ncsn_runner_kitti_simultaneous.py:
104,481): buckets at parameter boundaries covering the arena, and the bucketed average equal to the
single-process average of the ranks' gradients -- to fp32 rounding of the ring's partial sums with an fp32
wire (exact at world 2), within bf16 rounding with a bf16 wire (every hop's running sum rounded to bf16:
|err| <= (world - 1) * 2^-7 * mean(|g_r|)) -- and every rank, interior ones included, holding the same bits.
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


@pytest.mark.parametrize("world,wire", [(2, torch.float32), (2, torch.bfloat16), (4, torch.float32),
                                        (4, torch.bfloat16)])
def test_bucketed_average_gloo(world, wire):
    lay, n = layout()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, wire, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r, (nb, g)) for r, nb, g in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    gs = [rank_grads(r, n).numpy() for r in range(world)]
    want = np.sum([g.astype(np.float64) for g in gs], axis=0) / world
    assert all(res[r][0] == 4 for r in range(world))        # bucket count at 300k floats
    for r in range(1, world):                                # every rank holds the same average
        np.testing.assert_array_equal(res[r][1], res[0][1])
    got = res[0][1].astype(np.float64)
    mean_abs = np.mean([np.abs(g) for g in gs], axis=0)
    if wire == torch.float32:
        if world == 2:
            np.testing.assert_allclose(got, want, rtol=1e-7, atol=0)
        else:   # fp32 partial sums in the reduction order gloo picks: a few ulps of the magnitudes summed
            assert np.all(np.abs(got - want) <= 4 * 2.0 ** -24 * world * mean_abs + 1e-30)
    else:
        bound = (world - 1) * 2.0 ** -7 * mean_abs + 1e-30
        assert np.all(np.abs(got - want) <= bound)
        assert np.abs(got - want).max() > 0                 # (it really went over the wire in bf16)
