"""bench.py -- Langevin image-steps/s of the simultaneous sampler on MI355X (BASELINE.json metric).

One step = one Langevin step of every view: score-net forward (libsdp) + fused update +
cross-view consistency merge (a level >= minStepToShare, so the merge runs every step).

Modes (one process per GPU; torchrun sets RANK/LOCAL_RANK/WORLD_SIZE):
  viewsplit (default): ONE megabatch of 4*N views (Line.yml 4 views on 1 GPU = config 2;
      32 views on 8 GPUs = config 4); each rank owns 4 views, all-gathers the megabatch's
      images over RCCL every step (the cross-view consistency gather) and merges into its own.
  megabatch: every rank runs an independent 4-view megabatch (zero data exchange).
Both: one 4-byte all_reduce(MAX) per step keeps the reference's global tooHigh exact.
Per-GPU work is fixed as N grows ("scaling": "weak").  `value` = all views x steps / max-over-
ranks wall time.  The dominant conv class is timed live with HIP events on the forward's
stream (roofline); the CPU baseline is the oracle restatement timed on this host (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "Langevin denoising steps/sec on 64×1024 range images, 1/2/4/8 MI355X"
PEAK = {"fp32": 157.3, "fp32x3": 2500.0 / 3, "bf16": 2500.0}  # dense MFMA TFLOP/s in algorithmic fp32 FLOPs


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--views", type=int, default=4, help="views per GPU")
    ap.add_argument("--mode", choices=["viewsplit", "megabatch"], default="viewsplit")
    ap.add_argument("--precision", choices=["fp32x3", "fp32", "bf16"], default="fp32x3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    return ap.parse_args()


def cpu_baseline(V, H, W, threads):
    """Oracle restatement (torch-CPU score net + numpy update + numpy merge), one step of V views."""
    from oracle import sampling_ref as S
    from oracle import scorenet_ref as R
    from sdp.synthetic import exist_mask, scene_views
    from sdp.weights import get_sigmas_np, synthetic_state_dict
    torch.set_num_threads(max(1, min(threads, os.cpu_count() or 1)))
    P = R.to_torch_params(synthetic_state_dict(128))
    sc = scene_views(V, H, W)
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(V, 2, H, W, generator=g)
    sig = get_sigmas_np()
    c = 100
    ex = np.broadcast_to(exist_mask(H, W), (V, H, W))
    t0 = time.perf_counter()
    with torch.no_grad():
        grad = R.scorenet_forward(P, x, torch.full((V,), c, dtype=torch.long)).numpy()
    s = S.step_size_of(6.2e-6, sig[c], sig[-1])
    x1, _ = S.langevin_update(x.numpy(), S.nan_to_num(grad), sc["ref"], sc["mask"],
                              np.random.default_rng(0).standard_normal(x.shape).astype(np.float32), s, 1.0)
    S.kitti_merge(x1, sc["mask"], sc["sky"], ex, sc["toWorld"], sc["fromWorld"], V, sig[c])
    dt = time.perf_counter() - t0
    return {"value": V / dt, "unit": "image-steps/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"1 Langevin step of {V} views at {H}x{W} (fwd + update + merge), oracle restatement "
                      f"(torch CPU fp32 + numpy), {dt:.2f} s"}


def pmc_traffic(precision, V):
    """HBM bytes per launch of the dominant conv class from the committed PMC passes
    (tools/pmc_traffic.sh -> profiles/r01_traffic.json: TCC_EA0_RDREQ x 64 B x 2 (gfx950 wide-read
    correction) + TCC_EA0_WRREQ bytes, averaged over that kernel's launches at this grid)."""
    mode = {"fp32": 0, "fp32x3": 1, "bf16": 2}[precision]
    name = f"void sdp::conv_mfma_kernel<{mode}, 1, 64, 3, false, true>(sdp::ConvArgs)"
    grid = V * (32 * 512 // 128) * 256
    try:
        with open(os.path.join(REPO, "profiles", "r01_traffic.json")) as f:
            rows = json.load(f)
    except OSError:
        return None
    for r in rows:
        if r["kernel"] == name and r["grid"] == grid and "hbm_bytes" in r:
            return round(r["hbm_bytes"])
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        torch.distributed.init_process_group("nccl", device_id=dev)
    from sdp import _lib
    from sdp.merge import Merger
    from sdp.scorenet import ScoreNet
    from sdp.synthetic import exist_mask, scene_views
    from sdp.weights import get_sigmas_np

    H, W, V = 64, 1024, args.views
    N = world
    if args.mode == "viewsplit":
        n_src, aB, o_begin = V * N, V * N, rank * V
        sc = scene_views(n_src, H, W)
    else:
        n_src, aB, o_begin = V, V, 0
        sc = scene_views(V, H, W, seed=1234 + rank)
    net = ScoreNet(H=H, W=W, precision=args.precision).load_synthetic()
    g = torch.Generator(device=dev).manual_seed(1234)
    x_all = torch.rand(n_src, 2, H, W, device=dev, generator=g)
    x = x_all[o_begin:o_begin + V]                      # own views: a contiguous slice of the megabatch
    ref = torch.from_numpy(sc["ref"][o_begin:o_begin + V]).to(dev)
    mask = torch.from_numpy(sc["mask"][o_begin:o_begin + V]).to(dev)
    merger = Merger(n_src, aB, H, W, dev, torch.from_numpy(exist_mask(H, W)), torch.from_numpy(sc["sky"]),
                    torch.from_numpy(sc["mask"]), toWorld=torch.from_numpy(sc["toWorld"]),
                    fromWorld=torch.from_numpy(sc["fromWorld"]), o_begin=o_begin, n_out=V)
    sig = get_sigmas_np()
    lik = torch.empty_like(x)
    absmax = torch.zeros(1, dtype=torch.int32, device=dev)
    labels = {c: torch.full((V,), c, dtype=torch.int64, device=dev) for c in range(len(sig))}
    grad = torch.empty_like(x)
    L = _lib.lib()
    st = _lib.stream()
    offset = [0]

    def step(i):
        c = 2 + (i % (len(sig) - 2))          # levels >= minStepToShare: the merge always runs
        s = np.float32(6.2e-6) * (sig[c] / sig[-1]) ** 2
        ns = np.float32(np.sqrt(np.float32(s * np.float32(2))))
        net(x, labels[c], out=grad)
        absmax.zero_()
        _lib.check(L.sdp_langevin_step(x.data_ptr(), grad.data_ptr(), ref.data_ptr(), mask.data_ptr(), None,
                                       1234 + rank, offset[0], float(s), float(ns), 1.0, 1, V, 2, H * W,
                                       lik.data_ptr(), absmax.data_ptr(), st), "langevin")
        offset[0] += x.numel() // 4
        if dist:
            if args.mode == "viewsplit":
                torch.distributed.all_gather_into_tensor(x_all, x)     # cross-view consistency gather
            torch.distributed.all_reduce(absmax, op=torch.distributed.ReduceOp.MAX)
        merger(x_all, sig[c], 5, 10, 0.01, absmax)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    net.profile(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    prof = net.profile_read()
    net.profile(False)
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()
    assert torch.isfinite(x_all).all(), "non-finite images"
    if rank == 0:
        for k, (n_, ms_, fl_) in sorted(prof.items(), key=lambda kv: -kv[1][1]):
            print(f"[conv] {k:34s} launches {n_:5d} avg {ms_ / n_ * 1e3:8.1f} us  {fl_ / (ms_ / n_ / 1e3) / 1e12:7.1f} TF/s",
                  file=sys.stderr)
        value = N * V * args.steps / dt
        cls, (n, ms, fl) = max(prof.items(), key=lambda kv: kv[1][1])
        avg_s = ms / n / 1e3
        achieved = fl / avg_s / 1e12
        conv_ms = sum(v[1] for v in prof.values()) / args.steps
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(PEAK[args.precision], 1),
                "unit": "TFLOP/s", "frac": round(achieved / PEAK[args.precision], 4),
                "traffic": pmc_traffic(args.precision, V), "traffic_unit": "bytes/launch (PMC, profiles/r01_traffic.json)",
                "algorithmic_bytes": 2 * V * 32 * 512 * 256 * 4 + 256 * 256 * 9 * (2 if args.precision == "bf16" else 4),
                "kernel": f"conv_mfma_kernel [{cls}]", "avg_launch_us": round(avg_s * 1e6, 2),
                "flops_per_launch": fl, "conv_ms_per_step": round(conv_ms, 3)}
        cpu = None
        if N == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(V, H, W, args.cpu_threads)
        line = {"metric": METRIC, "value": round(value, 3), "unit": "image-steps/s", "n_gpus": N,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic (procedural Line.yml-style scene, random-init NCSN_LiDAR_small weights)",
                "config": {"workload": "Line.yml simultaneous sampling step (score-net fwd + Langevin update + "
                                       "consistency merge), 64x1024x2 range images",
                           "views_per_gpu": V, "megabatch_views": aB, "mode": args.mode,
                           "conv_arithmetic": args.precision, "parallelism": f"views{N}"},
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line))
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
