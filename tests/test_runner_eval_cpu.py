"""The training loop's every-100-steps EMA evaluation draws its batch from the TEST split through its
own sampler (runners/ncsn_runner_kitti_simultaneous.py:84-95, 247-251), on rank 0 only.  Every item
of the datasets draws a roll from the global np.random stream (kitti360_im_8Batch.py:234) and the
MySampler shuffles use it too, so an evaluation must not advance rank 0's stream: the ranks'
global batches would stop lining up and their slices could overlap.  gloo world 2 on CPU, with a
stand-in dataset that records the indices it serves and draws its roll like the real one."""
import argparse
import json
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from sdp import kitti360
from sdp import runner as R
from test_runner_dist_cpu import _config

N_TRAIN, N_TEST, BT, H, W = 40, 12, 2, 4, 8


class _FakeSet:
    def __init__(self, n, tag):
        self.n, self.tag, self.served = n, tag, []

    def __len__(self):
        return self.n

    def __getitem__(self, j):
        roll = int(np.random.randint(W))                  # as the real __getitem__: one draw per item
        self.served.append(j)
        img = np.full((2, H, W), float(j), np.float32)
        mask = np.ones((2, H, W), np.float32)
        return img, mask, np.zeros((1, H, W), bool), roll, 0, 0, 0, 0, j


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, out):
    torch.distributed.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    np.random.seed(1234)
    sets = {}

    def get_dataset(name, path, config, split="test", **kw):
        sets[split] = _FakeSet(N_TRAIN if split == "train" else N_TEST, split)
        return sets[split]
    kitti360.get_dataset = get_dataset
    args = argparse.Namespace(seed=1234, kitti_root="/nonexistent", num_batches=None)
    run = R.Runner(args, _config("HDVMine_Line.yml"), score=None, ops=None)
    train = run._train_source(BT, rank, world)
    test = run._test_source(BT) if rank == 0 else None
    batches = []
    for i in range(30):                                   # past an epoch boundary (sampler re-shuffle)
        X = train(i)[0]
        batches.append(sorted(int(v) for v in X[:, 0, 0, 0]))
        if test is not None and i % 7 == 3:              # the evaluation, rank 0 only
            test(i)
    st = np.random.get_state()
    state = [int(np.bitwise_xor.reduce(st[1])), int(st[2])]   # the MT key digest and its position
    objs = [None] * world
    torch.distributed.all_gather_object(objs, (batches, state, sets["train"].served, run._batches_per_epoch(BT, world)))
    if rank == 0:
        with open(os.path.join(out, "res.json"), "w") as f:
            json.dump(objs, f)
        assert sets["test"].served, "the evaluation drew from the test split"
    torch.distributed.destroy_process_group()


def test_eval_draws_keep_rank_batches_disjoint(tmp_path):
    mp.spawn(_run, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    with open(tmp_path / "res.json") as f:
        res = json.load(f)
    (b0, s0, served0, bpe), (b1, s1, served1, _) = res
    assert s0 == s1                                       # np.random streams still in lockstep
    for i, (x, y) in enumerate(zip(b0, b1)):
        assert not set(x) & set(y), f"batch {i}: ranks overlap {x} {y}"
    assert all(j < N_TRAIN for j in served0 + served1)    # training never served a test item
    assert bpe == N_TRAIN // (BT * 2)                     # one epoch = one pass over the training split
