"""main.py under torchrun: the sampling runner splits every batch's megabatches across ranks
(replacing the reference's DataParallel, runners/ncsn_runner_kitti_simultaneous.py:481), and the
files rank 0 writes must equal a single-process run bit for bit.  gloo world 2 and 4 on CPU (3
megabatches per batch: 2 + 1 at world 2; at world 4 ranks 1 and 2 are interior and rank 3 holds no
megabatch, so it idles outside the active group that keeps tooHigh global); the device
ops are the CPU oracle (Langevin update with the kernel's Philox noise stream, merge), the score
network a cheap deterministic stand-in -- so this checks exactly the split: contiguous megabatch
blocks, global tooHigh over the active ranks, per-view noise counters, the gather to rank 0."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
import yaml

import main as sdp_main
from sdp import runner as R
from test_distributed_cpu import OracleOps, fake_score

CFG_DIR = os.path.join(os.path.dirname(sdp_main.__file__), "configs")


def _config(name):
    with open(os.path.join(CFG_DIR, name)) as f:
        c = yaml.safe_load(f)
    c["sampling"].update(batch_size=6, actualBatchSize=2, n_steps_each=1)
    c["data"]["image_width"] = 128
    c["model"].update(num_classes=3, sigma_begin=0.9, sigma_end=0.3)
    c["simultaneous"] = dict(startStep=1, correlation_coefficient=0.01, grad_ref=1, allowance=10,
                             setting=5 if c["data"]["dataset"] == "KITTI360_im_8batch" else 7)
    ns = sdp_main.dict2namespace(c)
    ns.device = torch.device("cpu")
    return ns


def _run(rank, world, port, cfg_name, out):
    import argparse
    if world > 1:
        torch.distributed.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                             world_size=world)
    torch.manual_seed(1234)
    args = argparse.Namespace(image_folder=out, seed=1234, ckpt=None, precision="fp32x3", num_batches=1)
    R.Runner(args, _config(cfg_name), score=fake_score, ops=OracleOps()).sample()
    if world > 1:
        torch.distributed.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_megabatches_covers_every_megabatch_once():
    for n in range(1, 9):
        for w in range(1, 6):
            blocks = [R.shard_megabatches(n, r, w) for r in range(w)]
            got = [m for a, b in blocks for m in range(a, b)]
            assert got == list(range(n))


@pytest.mark.parametrize("cfg,world", [("HDVMine_Line.yml", 2), ("HDVMine_Circle.yml", 2), ("HDVMine_Line.yml", 4),
                                       ("HDVMine_Circle.yml", 4)])
def test_sharded_runner_writes_the_single_process_files(tmp_path, cfg, world):
    one, two = tmp_path / "w1", tmp_path / f"w{world}"
    one.mkdir()
    two.mkdir()
    _run(0, 1, 0, cfg, str(one))
    mp.spawn(_run, args=(world, _port(), cfg, str(two)), nprocs=world, join=True)
    names = sorted(f for f in os.listdir(one) if f.endswith(".npy") and "TimeTaken" not in f)
    assert names and names == sorted(f for f in os.listdir(two) if f.endswith(".npy") and "TimeTaken" not in f)
    assert any("Masked_completion" in f for f in names)
    for f in names:
        np.testing.assert_array_equal(np.load(two / f), np.load(one / f), err_msg=f)
