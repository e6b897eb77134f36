"""bench.py -- Langevin image-steps/s of the simultaneous sampler on MI355X (BASELINE.json metric).

Workloads (--workload):
  line (default; BASELINE configs 2 and 4): one step = one Langevin step of every view:
      score-net forward (libsdp) + fused update + cross-view consistency merge (a level >=
      minStepToShare, so the merge runs every step), pose-matrix (kitti) merge, setting 5.
  allforone (config 3): the same step with the origin-offset (AllForOne / Inpainting.yml)
      merge, setting 7, target + 8 aux views = 9 views per GPU.
  train (config 5): one DSM training step of the kitti runner (score-net forward, masked DSM
      loss, backward, gradient all-reduce over RCCL, Adam + EMA, weight re-pack, 5 Langevin
      predictions of the unknown pixels), batch 8 per GPU, bf16.  Prints its own metric.
  project: one step = the KITTI360_im_8batch __getitem__ compute of a
      megabatch of 8 views from a 120k-point scan resident in HBM (pose-chain transform, view
      and goal projections, post-processing).  Prints its own metric.

Modes for line (one process per GPU; torchrun sets RANK/LOCAL_RANK/WORLD_SIZE):
  viewsplit (default): ONE megabatch of 4*N views (Line.yml 4 views on 1 GPU = config 2;
      32 views on 8 GPUs = config 4); each rank owns 4 views, all-gathers the megabatch's
      images over RCCL every step (the cross-view consistency gather) and merges into its own.
  megabatch: every rank runs an independent megabatch (zero data exchange).
Both: one 4-byte all_reduce(MAX) per step keeps the reference's global tooHigh exact; it runs on a
side stream beside the merge, whose final correction pass alone waits for it (sdp.merge.AbsmaxAllReduce).
Per-GPU work is fixed as N grows ("scaling": "weak").  `value` = all views x steps / max-over-
ranks wall time.  The dominant conv class is timed live with HIP events on the forward's
stream (roofline); the CPU baseline is the oracle restatement timed on this host (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
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
TRAIN_METRIC = "DSM training image-steps/sec on 64×1024 range images (fwd+bwd+Adam+EMA), 1/2/4/8 MI355X"
PROJECT_METRIC = ("KITTI-360 views rendered/sec (pose chain + view and goal point_cloud_to_range_image + "
                  "post-processing) at 64×1024, 1/2/4/8 MI355X")
HBM_PEAK = 8000.0             # GB/s, MI355X_MICROARCH.md
PEAK = {"fp32": 157.3, "fp32x3": 2500.0 / 3, "bf16": 2500.0}  # dense MFMA TFLOP/s in algorithmic fp32 FLOPs
DTYPE_NOTE = {
    "fp32x3": "fp32 I/O, accumulation and non-conv ops; conv products as 3 bf16 MFMA passes of the hi/lo split "
              "(hi*hi + hi*lo + lo*hi, ~2^-17 relative product error; parity tol 1e-4 of max|out|)",
    "fp32": "exact fp32 products (v_mfma_f32_32x32x2_f32), fp32 everywhere",
    "bf16": "bf16 conv operands, fp32 accumulation and non-conv ops"}
FWD_FLOP = 1.2663e12          # score-net forward FLOPs per 64x1024 image
# Inpainting.yml (HDVMine_Circle.yml) data.modifications + 2 more origins: 8 aux views (config 3)
CIRCLE9 = [[0, 0, 0], [5, -5, 0], [-5, -5, 0], [0, 5, 0], [-10, 10, 0], [10, 10, 0], [-10, 0, 0], [10, 0, 0],
           [0, -10, 0]]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node; without torchrun's env, N > 1 spawns N ranks itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["line", "allforone", "train", "project"], default="line")
    ap.add_argument("--views", type=int, default=None, help="views (or training images) per GPU")
    ap.add_argument("--mode", choices=["viewsplit", "megabatch"], default="viewsplit")
    ap.add_argument("--megabatch-views", type=int, default=None,
                    help="viewsplit on ONE GPU: merge against a megabatch this large (the other views' images stay "
                         "fixed) -- one rank's per-step work of BASELINE config 4 (32) without the all-gather")
    ap.add_argument("--precision", choices=["fp32x3", "fp32", "bf16"], default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks join a gloo group and rank 0 prints the world it saw")
    ap.add_argument("--no-fp32-line", action="store_true",
                    help="skip the exact-fp32 (v_mfma_f32_32x32x2_f32) companion measurement of the line workload")
    ap.add_argument("--split", type=int, default=0,
                    help="part-batch streams per score-net forward (sdp_net_set_split; 0 = library default)")
    ap.add_argument("--unfused", action="store_true",
                    help="line/allforone: score net and Langevin update as two calls (sdp_net_forward + "
                         "sdp_langevin_step) instead of sdp_net_forward_langevin")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--fp32-tape", action="store_true",
                    help="train workload, bf16: keep the training tape in float32 (A/B against the bf16 tape)")
    ap.add_argument("--sustained-s", type=float, default=3.0,
                    help="line/allforone: also time >= this many seconds of back-to-back steps after >= "
                         "--sustained-warm-s of warm load (the clock under MFMA load settles only after ~2 s; "
                         "0 = skip); reported as the `sustained` companion, the headline stays the K timed steps")
    ap.add_argument("--sustained-warm-s", type=float, default=2.0)
    a = ap.parse_args()
    if a.views is None:
        a.views = {"line": 4, "allforone": 9, "train": 8, "project": 8}[a.workload]
    if a.precision is None:
        a.precision = "bf16" if a.workload == "train" else "fp32x3"
    if a.workload == "allforone":
        a.mode = "megabatch"
    return a


# ----------------------------------------------------------------------------- CPU baselines
def cpu_baseline(V, H, W, threads, workload):
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
    if workload == "allforone":
        S.allforone_merge(x1, sc["mask"], sc["sky"], ex, np.asarray(CIRCLE9[:V]), V, sig[c])
    else:
        S.kitti_merge(x1, sc["mask"], sc["sky"], ex, sc["toWorld"], sc["fromWorld"], V, sig[c])
    dt = time.perf_counter() - t0
    return {"value": V / dt, "unit": "image-steps/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"1 Langevin step of {V} views at {H}x{W} (fwd + update + {workload} merge), oracle "
                      f"restatement (torch CPU fp32 + numpy), {dt:.2f} s"}


def cpu_baseline_train(H, W, threads):
    """Oracle autograd DSM step (fwd + loss + backward) of ONE image, torch CPU fp32."""
    from oracle import scorenet_ref as R
    from sdp.weights import synthetic_state_dict
    torch.set_num_threads(max(1, min(threads, os.cpu_count() or 1)))
    P = R.to_torch_params(synthetic_state_dict(128))
    g = torch.Generator().manual_seed(1234)
    X = torch.rand(1, 2, H, W, generator=g)
    noise = torch.randn(1, 2, H, W, generator=g) * 50
    mask = (torch.rand(1, 2, H, W, generator=g) > 0.25).float()
    t0 = time.perf_counter()
    R.dsm_loss_and_grads(P, X + noise, noise, mask, torch.tensor([0]))
    dt = time.perf_counter() - t0
    return {"value": 1 / dt, "unit": "image-steps/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"1 DSM step (fwd + loss + backward, no optimizer) of 1 image at {H}x{W}, oracle autograd "
                      f"(torch CPU fp32), {dt:.2f} s"}


def pmc_traffic(precision, V, cls):
    """HBM bytes per launch of the dominant conv class, read from the committed PMC passes
    (tools/class_traffic.sh -> profiles/rNN_traffic.json, newest round first: TCC_EA0_RDREQ x 64 B x 2
    (gfx950 wide-read correction) + TCC_EA0_WRREQ bytes per launch of that kernel at this grid).  PMC
    counters cannot be read inside this process, so the value is tagged with the hash of the conv
    kernel's sources (sdp/_build.py conv_source_hash: common.h, conv_kernel.h, conv.hip -- what
    tools/conv_bench is built from): when no file matches the current tree the traffic is reported as
    null (stale), never as current."""
    import glob
    from sdp import _build
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]_traffic.json")), reverse=True)
    doc = None
    for fn in files:
        try:
            with open(fn) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if isinstance(d, dict) and d.get("conv_source_hash") == _build.conv_source_hash():
            doc, src = d, fn
            break
    if doc is None:
        return None, ("stale: no profiles/rNN_traffic.json was measured on this conv kernel source" if files else None)
    for r in doc.get("rows", []):
        if r.get("precision") == precision and r.get("views") == V and r.get("class") == cls:
            return round(r["hbm_bytes"]), (f"{os.path.basename(src)} (PMC, conv source "
                                           f"{doc['conv_source_hash'][:12]})")
    return None, None


def conv_clock(cls):
    """Clock the chip held and MFMA-busy fraction of conv class `cls` in this network, from the committed
    PMC + in-kernel-clock passes (tools/conv_clock.sh -> profiles/rNN_conv_clock.json, newest first),
    keyed like pmc_traffic by the conv source hash: None when no file matches the current tree."""
    import glob
    from sdp import _build
    for fn in sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]_conv_clock.json")), reverse=True):
        try:
            with open(fn) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if not isinstance(d, dict) or d.get("conv_source_hash") != _build.conv_source_hash():
            continue
        for r in d.get("classes", []):
            if r.get("class") == cls and "clock_GHz" in r:
                return {"clock_GHz": r["clock_GHz"], "mfma_busy_frac": r["mfma_busy_frac"],
                        "source": f"{os.path.basename(fn)} (conv source {d['conv_source_hash'][:12]})"}
    return None


def split_overlap():
    """Per memory-bound kernel class, the fraction of its time that ran under a conv of the OTHER forward
    stream in the default two-stream step (tools/overlap.py over a rocprofv3 --kernel-trace of
    `bench.py`, --split 2 -> profiles/rNN_overlap.json, newest first), keyed by the libsdp source hash
    (sdp/_build.py source_hash): None when no file matches the current tree.  The per-kernel durations
    above come from a profiled pass with one launch per layer; this says how much of that time the
    default schedule hides."""
    import glob
    from sdp import _build
    for fn in sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]_overlap.json")), reverse=True):
        try:
            with open(fn) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if isinstance(d, dict) and d.get("libsdp_source_hash") == _build.source_hash():
            return d.get("classes", {}), os.path.basename(fn)
    return None, None


def overlap_of(kernel, classes):
    keys = {"inpp_finalize": ("inpp_moments", "inpp_ss"), "maxpool5": ("maxpool5",), "begin_conv": ("begin_conv",),
            "end_conv": ("end_conv+langevin",), "avgpool2": ("avgpool2",)}
    for prefix, cl in keys.items():
        if kernel.startswith(prefix):
            tot = sum(classes[c]["total_us"] for c in cl if c in classes)
            hid = sum(classes[c]["hidden_us"] for c in cl if c in classes)
            return round(hid / tot, 4) if tot else None
    return None


# ----------------------------------------------------------------------------- timing harness
def timed(step, args, dist, dev):
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()
    return dt


def viewsplit_layout(args, rank, N):
    """(n_src, aB, o_begin): the megabatch views a rank's merge reads, its megabatch size and the first
    of the V views the rank owns.  viewsplit: one megabatch of V*N views, rank r owns [r*V, (r+1)*V)
    (its Philox counters start at o_begin * per_view4, sdp/sampling.py); megabatch: an independent
    megabatch of V views per rank."""
    V = args.views
    if args.mode == "viewsplit":
        n_src = V * N if args.megabatch_views is None else args.megabatch_views
        if args.megabatch_views is not None and (N != 1 or n_src < V):
            raise SystemExit("--megabatch-views emulates a larger megabatch on one GPU only")
        return n_src, n_src, rank * V
    return V, V, 0


def dry_run_viewsplit(args, rank, N, dist):
    """CPU/gloo rehearsal of the viewsplit step's bookkeeping (no GPU, no libsdp): the rank layout of
    viewsplit_layout, the Philox counter offsets, the per-step all-gather of the megabatch and the
    all_reduce(MAX) of tooHigh, with a deterministic stand-in for the update (a function of each view's
    global index and its counter offset) and for the merge (every owned view pulled towards the
    megabatch mean, corrected by the global max).  Returns the sha256 of the final megabatch images:
    equal for every N when the exchange and the offsets are right (tests/test_bench_launcher_cpu.py)."""
    import hashlib
    V, H, W = args.views, 4, 32
    n_all = V * N
    n_src, aB, o_begin = viewsplit_layout(args, rank, N)
    assert n_src == n_all
    per_view4 = 2 * H * W // 4
    g = torch.Generator().manual_seed(1234)
    x_all = torch.rand(n_all, 2, H, W, generator=g, dtype=torch.float32)
    x = x_all[o_begin:o_begin + V]
    offset = o_begin * per_view4
    for i in range(args.steps):
        views = torch.arange(o_begin, o_begin + V, dtype=torch.float32).view(V, 1, 1, 1)
        ctr = (offset + (views - o_begin) * per_view4) % 9973.0   # each view's own Philox counter
        x.add_(torch.sin(x * 3.0 + ctr * 1e-3 + views) * np.float32(1e-2))
        offset += n_src * per_view4
        amax = x[:, 0].abs().max().reshape(1)
        if dist:
            parts = list(x_all.chunk(N))
            torch.distributed.all_gather(parts, x.clone())
            torch.distributed.all_reduce(amax, op=torch.distributed.ReduceOp.MAX)
        mean = x_all.mean(0, keepdim=True)
        x.add_((mean - x) * np.float32(0.05) / amax)
    if dist:
        torch.distributed.all_gather(list(x_all.chunk(N)), x.clone())
    return hashlib.sha256(x_all.numpy().tobytes()).hexdigest()


def run_sampling(args, rank, N, dist, dev):
    from sdp import _lib
    from sdp.merge import AbsmaxAllReduce, Merger, allforone_origins
    from sdp.scorenet import ScoreNet
    from sdp.synthetic import exist_mask, scene_views
    from sdp.weights import get_sigmas_np

    H, W, V = 64, 1024, args.views
    n_src, aB, o_begin = viewsplit_layout(args, rank, N)
    sc = scene_views(n_src, H, W) if args.mode == "viewsplit" else scene_views(V, H, W, seed=1234 + rank)
    net = ScoreNet(H=H, W=W, precision=args.precision).load_synthetic()
    g = torch.Generator(device=dev).manual_seed(1234)
    x_all = torch.rand(n_src, 2, H, W, device=dev, generator=g)
    x = x_all[o_begin:o_begin + V]                      # own views: a contiguous slice of the megabatch
    ref = torch.from_numpy(sc["ref"][o_begin:o_begin + V]).to(dev)
    mask = torch.from_numpy(sc["mask"][o_begin:o_begin + V]).to(dev)
    if args.workload == "allforone":
        if V > len(CIRCLE9):
            raise SystemExit(f"allforone: at most {len(CIRCLE9)} views")
        merger = Merger(n_src, aB, H, W, dev, torch.from_numpy(exist_mask(H, W)), torch.from_numpy(sc["sky"]),
                        torch.from_numpy(sc["mask"]), origins=allforone_origins(CIRCLE9[:V]), o_begin=o_begin,
                        n_out=V)
        setting = 7
    else:
        merger = Merger(n_src, aB, H, W, dev, torch.from_numpy(exist_mask(H, W)), torch.from_numpy(sc["sky"]),
                        torch.from_numpy(sc["mask"]), toWorld=torch.from_numpy(sc["toWorld"]),
                        fromWorld=torch.from_numpy(sc["fromWorld"]), o_begin=o_begin, n_out=V)
        setting = 5
    sig = get_sigmas_np()
    lik = torch.empty_like(x)
    absmax = torch.zeros(1, dtype=torch.int32, device=dev)
    absmax_reduce = AbsmaxAllReduce()
    labels = {c: torch.full((V,), c, dtype=torch.int64, device=dev) for c in range(len(sig))}
    grad = torch.empty_like(x)
    L = _lib.lib()
    st = _lib.stream()
    per_view4 = 2 * H * W // 4
    offset = [o_begin * per_view4]            # Philox counters of the whole megabatch (sdp/sampling.py)

    def step(i):
        c = 2 + (i % (len(sig) - 2))          # levels >= minStepToShare: the merge always runs
        s = np.float32(6.2e-6) * (sig[c] / sig[-1]) ** 2
        ns = np.float32(np.sqrt(np.float32(s * np.float32(2))))
        seed = 1234 + (rank if args.mode == "megabatch" else 0)
        absmax.zero_()
        if args.unfused:
            net_box[0](x, labels[c], out=grad)
            _lib.check(L.sdp_langevin_step(x.data_ptr(), grad.data_ptr(), ref.data_ptr(), mask.data_ptr(), None, seed,
                                           offset[0], float(s), float(ns), 1.0, 1, V, 2, H * W, lik.data_ptr(),
                                           absmax.data_ptr(), st), "langevin")
        else:   # the update in the net's last kernel (sdp_net_forward_langevin), as sdp.sampling runs it
            net_box[0].forward_langevin(x, labels[c], ref, mask, None, seed, offset[0], float(s), float(ns), 1.0, True,
                                        lik, absmax)
        offset[0] += n_src * per_view4
        ev = None
        if dist:
            if args.mode == "viewsplit":
                torch.distributed.all_gather_into_tensor(x_all, x)     # cross-view consistency gather
            ev = absmax_reduce(absmax)     # side stream; only the merge's correction pass waits for it
        if merge_ev is not None:
            ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ea.record()
            merger(x_all, sig[c], setting, 10, 0.01, absmax, absmax_event=ev)
            eb.record()
            merge_ev.append((ea, eb))
        else:
            merger(x_all, sig[c], setting, 10, 0.01, absmax, absmax_event=ev)

    # consistency merge (7 kernels on the forward's stream), SURVEY §8(d) compulsory bytes per
    # megabatch-step: per source view read x + mask + exist/sky, per output view write x and its
    # 114 x W accumulator grid written and read (24 B per cell) -- 7.3 MB per view at N = 1
    HWp = H * W
    merge_bytes = n_src * (8 * HWp + 8 * HWp + 2 * HWp) + V * (8 * HWp + 2 * 24 * ((50 * H) // 28) * W)
    merge_ev = None

    def measure(prec, steps, warmup):
        """Time `steps` steps with the score net at conv arithmetic `prec` (profiling OFF), then a
        separate profiled pass of a few steps for the per-kernel rooflines; return (dt, roofline)."""
        net_box[0] = net if prec == args.precision else ScoreNet(H=H, W=W, precision=prec).load_synthetic()
        cur = net_box[0]
        if args.split:
            cur.set_split(args.split)
        cur.profile(False)
        for i in range(warmup):
            step(i)
        dt = timed(step, argparse.Namespace(warmup=0, steps=steps), dist, dev)
        psteps = min(steps, 5)
        cur.profile(True)
        cur.profile_read()
        nonlocal merge_ev
        merge_ev = []
        for i in range(psteps):
            step(warmup + steps + i)
        torch.cuda.synchronize()
        prof = cur.profile_read()
        cur.profile(False)
        merge_us = sum(ea.elapsed_time(eb) for ea, eb in merge_ev) / len(merge_ev) * 1e3
        merge_ev = None
        steps = psteps                                  # per-step figures below are over the profiled pass
        if rank == 0:
            for k, (n_, ms_, fl_, by_) in sorted(prof.items(), key=lambda kv: -kv[1][1]):
                t_ = ms_ / n_ / 1e3
                print(f"[{prec}] {k:34s} launches {n_:5d} avg {t_ * 1e6:8.1f} us  {fl_ / t_ / 1e12:7.1f} TF/s  "
                      f"{by_ / t_ / 1e9:7.1f} GB/s", file=sys.stderr)
        convs = {k: v for k, v in prof.items() if v[2] > 0}
        cls, (n, ms, fl, _) = max(convs.items(), key=lambda kv: kv[1][1])
        avg_s = ms / n / 1e3
        achieved = fl / avg_s / 1e12
        conv_ms = sum(v[1] for v in convs.values()) / steps
        # memory-bound kernels of the forward against the HBM roofline (north_star): algorithmic
        # bytes per launch / average launch time, HIP events on the forward's stream
        mem = []
        ov_classes, ov_src = split_overlap() if args.workload == "line" else (None, None)
        for k, (n_, ms_, fl_, by_) in sorted(prof.items(), key=lambda kv: -kv[1][1]):
            if fl_ == 0 and by_ > 0:
                t_ = ms_ / n_ / 1e3
                mem.append({"kernel": k, "launches_per_step": round(n_ / steps, 2), "avg_launch_us": round(t_ * 1e6, 2),
                            "algorithmic_bytes": int(by_), "achieved_GBps": round(by_ / t_ / 1e9, 1),
                            "frac": round(by_ / t_ / 1e9 / HBM_PEAK, 4)})
                if ov_classes is not None:
                    hf = overlap_of(k, ov_classes)
                    if hf is not None:
                        mem[-1].update(hidden_frac_split2=hf, hidden_source=ov_src)
        mem.append({"kernel": "consistency_merge (7 kernels, HIP events around sdp_consistency_merge)",
                    "launches_per_step": 1, "avg_launch_us": round(merge_us, 2), "algorithmic_bytes": int(merge_bytes),
                    "achieved_GBps": round(merge_bytes / (merge_us * 1e-6) / 1e9, 1),
                    "frac": round(merge_bytes / (merge_us * 1e-6) / 1e9 / HBM_PEAK, 4),
                    "bytes_basis": "SURVEY 8(d): 7.3 MB per view; latency/atomic-bound, not HBM-bound"})
        traffic, tsrc = pmc_traffic(prec, V, cls) if args.workload == "line" else (None, None)
        clk = conv_clock(cls) if (args.workload == "line" and prec == "fp32x3") else None
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(PEAK[prec], 1),
                "unit": "TFLOP/s", "frac": round(achieved / PEAK[prec], 4),
                "traffic": traffic, "traffic_source": tsrc,
                "algorithmic_bytes": 2 * V * 32 * 512 * 256 * 4 + 256 * 256 * 9 * (2 if prec == "bf16" else 4),
                "kernel": f"conv_mfma_kernel [{cls}]", "avg_launch_us": round(avg_s * 1e6, 2),
                "flops_per_launch": fl, "conv_ms_per_step": round(conv_ms, 3), "memory_bound": mem}
        if clk is not None:
            # the peak at the clock the chip held under this load (power-limited DVFS), this run's time
            roof.update(clock_GHz=clk["clock_GHz"], mfma_busy_frac=clk["mfma_busy_frac"],
                        frac_at_clock=round(achieved / (PEAK[prec] * clk["clock_GHz"] / 2.4), 4),
                        clock_source=clk["source"])
        return dt, roof

    net_box = [net]
    dt, roof = measure(args.precision, args.steps, args.warmup)
    sustained = None
    if args.sustained_s > 0:
        # dt is the max over ranks, so every rank derives the same step counts (no collective mismatch)
        per = dt / args.steps
        n_warm = max(1, int(np.ceil(args.sustained_warm_s / per)))
        n_meas = max(1, int(np.ceil(args.sustained_s / per)))
        net_box[0] = net
        for i in range(n_warm):
            step(i)
        dts = timed(step, argparse.Namespace(warmup=0, steps=n_meas), dist, dev)
        # the dominant conv class right after the window, while the clock is still at its loaded level
        net.profile(True)
        net.profile_read()
        for i in range(5):
            step(n_warm + n_meas + i)
        torch.cuda.synchronize()
        sprof = net.profile_read()
        net.profile(False)
        cls_name = roof["kernel"][len("conv_mfma_kernel ["):-1]
        sn, sms, sfl, _ = sprof[cls_name]
        s_avg = sms / sn / 1e3
        sustained = {"value": round(N * V * n_meas / dts, 3), "ms_per_step": round(dts / n_meas * 1e3, 3),
                     "steps": n_meas, "seconds": round(dts, 3), "warm_steps": n_warm,
                     "warm_s": round(n_warm * per, 3),
                     "dominant_conv": {"class": cls_name, "avg_launch_us": round(s_avg * 1e6, 2),
                                       "achieved": round(sfl / s_avg / 1e12, 2),
                                       "frac": round(sfl / s_avg / 1e12 / PEAK[args.precision], 4)},
                     "note": "back-to-back steps after >= 2 s of warm load (steady DVFS clock), same step as value"}
    exact = None
    if args.workload == "line" and args.precision != "fp32" and not args.no_fp32_line:
        k = min(args.steps, 5)
        dt32, roof32 = measure("fp32", k, 1)
        exact = {"value": round(N * V * k / dt32, 3), "ms_per_step": round(dt32 / k * 1e3, 3), "steps": k,
                 "dtype": "fp32", "roofline": roof32,
                 "note": "same step with exact-fp32 conv products (v_mfma_f32_32x32x2_f32)"}
    assert torch.isfinite(x_all).all(), "non-finite images"
    if rank != 0:
        return None
    value = N * V * args.steps / dt
    cpu = None
    if N == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(V, H, W, args.cpu_threads, args.workload)
    if args.workload == "allforone":
        wl = ("Inpainting.yml AllForOne simultaneous sampling step (score-net fwd + Langevin update + origin-offset "
              "consistency merge, setting 7), target + 8 aux views, 64x1024x2 range images")
    else:
        wl = ("Line.yml simultaneous sampling step (score-net fwd + Langevin update + consistency merge), "
              "64x1024x2 range images")
    return {"metric": METRIC, "value": round(value, 3), "unit": "image-steps/s", "n_gpus": N,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "dtype_note": DTYPE_NOTE[args.precision],
            "data": "synthetic (procedural Line.yml-style scene, random-init NCSN_LiDAR_small weights)",
            "config": {"workload": wl + (" (megabatch emulated on one GPU)" if args.megabatch_views else ""),
                       "views_per_gpu": V, "megabatch_views": aB, "mode": args.mode,
                       "conv_arithmetic": args.precision, "parallelism": f"views{N}"},
            "roofline": roof, "cpu_baseline": cpu, "fp32_exact": exact, "sustained": sustained}


def run_train(args, rank, N, dist, dev):
    from sdp.scorenet import ScoreNet
    from sdp.synthetic import scene_views
    from sdp.training import Trainer, train_step
    from sdp.weights import get_sigmas_np

    H, W, Bg = 64, 1024, args.views
    net = ScoreNet(H=H, W=W, precision=args.precision).load_synthetic()
    tr = Trainer(net, lr=1e-4, dist_group=torch.distributed.group.WORLD if dist else None, tape_bf16=not args.fp32_tape)
    sc = scene_views(Bg, H, W, seed=1234 + rank)
    X0 = torch.from_numpy(sc["ref"]).to(dev)
    mask = torch.from_numpy(sc["mask"]).to(dev).float()
    sig = get_sigmas_np()
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    state = {"X": X0.clone(), "t": 0}
    losses = []

    def step(i):
        t = i % 4                    # the runner's curriculum: timesteps 0 .. maxTimeStepReachable-1
        loss, state["X"] = train_step(tr, state["X"], X0, mask, sig, t, 6.2e-6, 5, generator=gen)
        losses.append(loss)

    dt = timed(step, args, dist, dev)
    if not all(np.isfinite(float(v)) for v in losses):
        raise SystemExit("non-finite training loss")
    if rank != 0:
        return None
    value = N * Bg * args.steps / dt
    ms = dt / args.steps * 1e3
    flops = 3 * FWD_FLOP * Bg                          # fwd + dgrad + wgrad conv FLOPs per GPU-step
    achieved = flops / (ms / 1e3) / 1e12
    roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(PEAK[args.precision], 1),
            "unit": "TFLOP/s", "frac": round(achieved / PEAK[args.precision], 4), "traffic": None,
            "kernel": "whole training step (conv fwd + dgrad + wgrad FLOPs / step time)"}
    cpu = None
    if N == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_train(H, W, args.cpu_threads)
    return {"metric": TRAIN_METRIC, "value": round(value, 3), "unit": "image-steps/s", "n_gpus": N,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (procedural scene range images, random-init NCSN_LiDAR_small weights)",
            "config": {"workload": "Densification.yml DSM training step (kitti runner loop body: fwd + masked DSM "
                                   "loss + backward + grad all-reduce + Adam + EMA + 5 Langevin predictions)",
                       "batch_per_gpu": Bg, "global_batch": Bg * N, "parallelism": f"dp{N}",
                       "conv_arithmetic": args.precision,
                       "tape": "float32" if (args.fp32_tape or args.precision != "bf16") else "bf16"},
            "roofline": roof, "cpu_baseline": cpu, "final_loss": float(losses[-1])}


def synthetic_scan(n, seed):
    """A LiDAR-like float32 [n, 4] scan (x, y, z, intensity): ground ring, two walls, boxes, clutter."""
    r = np.random.default_rng(seed)
    k = n // 4
    a = r.uniform(-np.pi, np.pi, k)
    rad = np.sqrt(r.uniform(1.0, 45.0 ** 2, k))
    ground = np.stack([rad * np.cos(a), rad * np.sin(a), -1.73 + r.normal(0, 0.02, k)], 1)
    walls = np.stack([r.uniform(-40, 40, k), np.where(r.random(k) < 0.5, -8.0, 8.0), r.uniform(-1.73, 3.0, k)], 1)
    bc = r.uniform(-20, 20, (12, 2))
    bi = r.integers(0, 12, k)
    boxes = np.stack([bc[bi, 0] + r.uniform(-1.5, 1.5, k), bc[bi, 1] + r.uniform(-1.5, 1.5, k),
                      r.uniform(-1.73, 0.5, k)], 1)
    m = n - 3 * k
    clutter = np.stack([r.uniform(-60, 60, m), r.uniform(-60, 60, m), r.uniform(-3, 8, m)], 1)
    xyz = np.concatenate([ground, walls, boxes, clutter], 0)
    return np.concatenate([xyz, r.uniform(0, 1, (n, 1))], 1).astype(np.float32)


def view_poses(V, seed):
    """toWorld of the scan's pose and fromWorld = inv(toWorld of the goal pose 5(k+1) ahead)."""
    r = np.random.default_rng(seed)

    def pose(k):
        th = 0.04 * k + r.uniform(-0.01, 0.01)
        m = np.eye(4)
        m[:3, :3] = [[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]]
        m[:3, 3] = [1.7 * k + 100.0, -0.4 * k + 50.0, 110.0]
        return m
    return pose(0), [np.linalg.inv(pose(5 * (k + 1))) for k in range(V)]


def cpu_baseline_project(H, W, n_pts):
    """The oracle restatement of one 8batch item's compute (numpy, single-threaded)."""
    from oracle import kitti_ref
    scan, goal = synthetic_scan(n_pts, 1), synthetic_scan(n_pts, 2)
    to_world, from_worlds = view_poses(1, 3)
    t0 = time.perf_counter()
    n = 0
    while True:
        pts = kitti_ref.transform(scan, to_world, from_worlds[0])
        kitti_ref.render_arrays(pts, goal, np.zeros(3), H, W)
        n += 1
        if time.perf_counter() - t0 > 10.0 or n >= 120:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "views/s", "cores": 1, "kind": "port",
            "sample": f"{n} KITTI360_im_8batch items ({n_pts} points, {H}x{W}) through the numpy restatement "
                      f"(oracle/kitti_ref.py: np.matmul pose chain, argsort z-buffer projection x2, post), {dt:.2f} s"}


def run_project(args, rank, N, dist, dev):
    from sdp import _lib
    H, W, V, NP = 64, 1024, args.views, 120000
    L, st = _lib.lib(), _lib.stream()
    scan = torch.from_numpy(synthetic_scan(NP, 1 + rank)).to(dev)
    goal32 = torch.from_numpy(synthetic_scan(NP, 1000 + rank)).to(dev)
    goal = torch.empty(NP, 4, dtype=torch.float64, device=dev)
    _lib.check(L.sdp_view_transform(goal32.data_ptr(), NP, None, None, goal.data_ptr(), st), "widen")
    to_world, from_worlds = view_poses(V, 7 + rank)
    mats = [(np.ascontiguousarray(to_world), np.ascontiguousarray(f)) for f in from_worlds]
    n = _lib.SZ()
    _lib.check(L.sdp_range_project_workspace_size(H, W, _lib.C.byref(n)), "ws")
    ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
    o = np.zeros(3)
    pts = torch.empty(NP, 4, dtype=torch.float64, device=dev)
    f64 = lambda *s: torch.empty(*s, dtype=torch.float64, device=dev)
    u8 = lambda *s: torch.empty(*s, dtype=torch.uint8, device=dev)
    img = dict(d=f64(H, W), i=f64(H, W), o=u8(H, W), s=u8(H, W), x=torch.empty(H, W, dtype=torch.int64, device=dev),
               gd=f64(H, W), gi=f64(H, W))
    out = [dict(real=f64(2, H, W), goal=f64(2, H, W), nm=u8(2, H, W), ns=u8(1, H, W)) for _ in range(V)]

    def project(p, d, i, ob, sk, ix):
        _lib.check(L.sdp_range_project(p.data_ptr(), NP, 4, 1, o.ctypes.data, H, W, d.data_ptr(), i.data_ptr(),
                                       _lib.ptr(ob), _lib.ptr(sk), _lib.ptr(ix),
                                       ws.data_ptr(), ws.numel(), st), "project")

    def step(i):
        for v in range(V):
            m1, m2 = mats[v]
            _lib.check(L.sdp_view_transform(scan.data_ptr(), NP, m1.ctypes.data, m2.ctypes.data, pts.data_ptr(), st),
                       "transform")
            project(pts, img["d"], img["i"], img["o"], img["s"], img["x"])
            project(goal, img["gd"], img["gi"], None, None, None)      # goal: depth + intensity only
            r = out[v]
            _lib.check(L.sdp_view_finalize(img["d"].data_ptr(), img["i"].data_ptr(), img["o"].data_ptr(),
                                           img["s"].data_ptr(), img["gd"].data_ptr(), img["gi"].data_ptr(), H, W, 2,
                                           -1, 0, 1 if v == 0 else 0, r["real"].data_ptr(), r["nm"].data_ptr(),
                                           r["ns"].data_ptr(), r["goal"].data_ptr(), st), "finalize")

    for i in range(args.warmup):
        step(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    dt = timed(step, argparse.Namespace(warmup=0, steps=args.steps), dist, dev)
    e1.record()
    e1.synchronize()
    dev_ms_per_view = e0.elapsed_time(e1) / (args.steps * V)
    assert all(bool(torch.isfinite(r["real"]).all()) for r in out)
    if rank != 0:
        return None
    # algorithmic bytes per view: transform 16 B in + 32 B out per point; per projection two
    # passes over the points (32 B + an 8-B atomic each) and per pixel the winner's 32 B and the
    # outputs (33 B; the view's also the 10-B sky scan); finalize 34 B in + 35 B out per pixel
    HW = H * W
    view_bytes = 48 * NP + 2 * (80 * NP + 65 * HW) + 10 * HW + 69 * HW
    achieved = view_bytes / (dev_ms_per_view * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK, 4), "traffic": None,
            "kernel": "one view's launch sequence (sdp_view_transform + 2 x sdp_range_project + sdp_view_finalize), "
                      "HIP events on the launch stream",
            "algorithmic_bytes_per_view": view_bytes, "avg_view_us": round(dev_ms_per_view * 1e3, 2)}
    cpu = None
    if N == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_project(H, W, NP)
    return {"metric": PROJECT_METRIC, "value": round(N * V * args.steps / dt, 2), "unit": "views/s", "n_gpus": N,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": f"synthetic ({NP}-point LiDAR-like scans, resident in HBM)",
            "config": {"workload": "KITTI360_im_8batch __getitem__ compute for a megabatch of views "
                                   "(datasets/kitti360_im_8Batch.py:146-291)", "views_per_gpu": V,
                       "points_per_scan": NP, "parallelism": f"views{N}"},
            "roofline": roof, "cpu_baseline": cpu}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher_cmd(gpus, argv, port):
    """The torchrun command that runs this bench as one process per GPU (RCCL over xGMI)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        # `bench.py --gpus N` without a launcher: spawn N ranks (this parent never touches the GPU)
        if not args.dry_run:
            from sdp import _build
            _build.ensure_built()
        sys.exit(subprocess.call(launcher_cmd(args.gpus, sys.argv[1:], _free_port())))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if args.dry_run:
        if dist:
            torch.distributed.init_process_group("gloo")
            t = torch.tensor([rank], dtype=torch.int64)
            torch.distributed.all_reduce(t)
            digest = dry_run_viewsplit(args, rank, world, dist)
            if rank == 0:
                print(json.dumps({"dry_run": True, "n_gpus": world, "world_size": torch.distributed.get_world_size(),
                                  "rank_sum": int(t.item()), "viewsplit_sha256": digest}))
            torch.distributed.destroy_process_group()
        else:
            print(json.dumps({"dry_run": True, "n_gpus": 1, "world_size": 1, "rank_sum": 0,
                              "viewsplit_sha256": dry_run_viewsplit(args, 0, 1, False)}))
        return
    from sdp import _build
    _build.ensure_built()          # a fresh checkout has no libsdp.so (git-ignored): build before any GPU call
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        torch.distributed.init_process_group("nccl", device_id=dev)
    if args.workload == "train":
        line = run_train(args, rank, world, dist, dev)
    elif args.workload == "project":
        line = run_project(args, rank, world, dist, dev)
    else:
        line = run_sampling(args, rank, world, dist, dev)
    if line is not None:
        if dist:
            line["world_size"] = torch.distributed.get_world_size()
            line["backend"] = torch.distributed.get_backend()
        print(json.dumps(line))
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
