"""Drop-in CLI: ``python main.py --config HDVMine_Line.yml --sample [--ni] [--exp DIR] [-i FOLDER]``
(sampling) and ``python main.py --config HDVMine_Densification.yml [--ni] [--resume_training]``
(DSM training, runner.train()).  Under torchrun (one process per GPU) both shard across the GPUs
over RCCL, replacing the reference's DataParallel.

Same flags, YAML schema and output locations as LiDARGen/main.py:17-163 (YAML from
``configs/<name>`` relative to the working directory, else this package's configs/;
samples under ``{exp}/image_samples/{image_folder}``; seeds 1234).  Documented fixes: the
AllForOne / densification datasets are routed to the AllForOne sampler (the reference
sends them to the Completion runner, which crashes silently), and
errors propagate with a non-zero exit status instead of being logged and swallowed.
Extra flags: --ckpt (LiDARGen checkpoint; default the reference's path, else synthetic
weights), --precision {fp32x3,fp32,bf16}, --num_batches (sampling batches; training batches per
epoch), --n_iters / --snapshot_freq / --max_epochs (override the config's training schedule).
"""
import argparse
import logging
import os
import shutil
import sys

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import torch  # noqa: E402


def dict2namespace(config):
    ns = argparse.Namespace()
    for k, v in config.items():
        setattr(ns, k, dict2namespace(v) if isinstance(v, dict) else v)
    return ns


def parse_args_and_config(argv=None):
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--config", type=str, default="HDVMine_Line.yml", help="Path to the config file")
    p.add_argument("--seed", type=int, default=1234, help="Random seed")
    p.add_argument("--exp", type=str, default="exp", help="Path for saving running related data.")
    p.add_argument("--doc", type=str, default="HDVMine", help="Name of the log folder.")
    p.add_argument("--comment", type=str, default="", help="A string for experiment comment")
    p.add_argument("--verbose", type=str, default="info", help="Verbose level: info | debug | warning | critical")
    p.add_argument("--test", action="store_true")
    p.add_argument("--sample", action="store_true", help="Whether to produce samples from the model")
    p.add_argument("--densification", action="store_true", default=False)
    p.add_argument("--nvs", action="store_true")
    p.add_argument("--fast_fid", action="store_true")
    p.add_argument("--resume_training", action="store_true")
    p.add_argument("-i", "--image_folder", type=str, default="images", help="The folder name of samples")
    p.add_argument("--ni", action="store_true", help="No interaction")
    p.add_argument("--ckpt", type=str, default=None, help="LiDARGen checkpoint (list format with EMA shadow)")
    p.add_argument("--precision", type=str, default="fp32x3", choices=["fp32x3", "fp32", "bf16"])
    p.add_argument("--num_batches", type=int, default=None,
                   help="sampling: batches to sample (default 1; scene completion: 0 or -1 = the whole "
                        "validation split); training: batches per epoch "
                        "(default: the training split's length // global batch, 1 for the procedural source)")
    p.add_argument("--n_iters", type=int, default=None)
    p.add_argument("--snapshot_freq", type=int, default=None)
    p.add_argument("--max_epochs", type=int, default=None)
    p.add_argument("--kitti_root", type=str, default=None,
                   help="KITTI-360 root (the reference's /data/KITTI-360); views rendered on the GPU "
                        "(sdp.kitti360). Without it the procedural scene of sdp.synthetic is used.")
    args = p.parse_args(argv)
    args.log_path = os.path.join(args.exp, "logs", args.doc)
    path = args.config if os.path.exists(args.config) else os.path.join("configs", args.config)
    if not os.path.exists(path):
        path = os.path.join(HERE, "configs", os.path.basename(args.config))
    with open(path) as f:
        config = yaml.safe_load(f)
    config["data"].setdefault("image_width", config["data"]["image_size"])
    config["sampling"]["densification"] = args.densification   # main.py:46-48
    config["sampling"]["interpolation"] = False
    config["sampling"]["inpainting"] = True
    if args.n_iters is not None:
        config["training"]["n_iters"] = args.n_iters
    if args.snapshot_freq is not None:
        config["training"]["snapshot_freq"] = args.snapshot_freq
    new_config = dict2namespace(config)
    level = getattr(logging, args.verbose.upper(), None)
    if not isinstance(level, int):
        raise ValueError(f"level {args.verbose} not supported")
    rank = int(os.environ.get("RANK", "0"))
    training = not (args.test or args.sample or args.nvs or args.fast_fid)
    if training and rank == 0 and not args.resume_training:     # main.py:54-77
        if os.path.exists(args.log_path):
            if not args.ni and input("Folder already exists. Overwrite? (Y/N)").upper() != "Y":
                print("Folder exists. Program halted.")
                sys.exit(0)
            shutil.rmtree(args.log_path)
        os.makedirs(args.log_path)
        with open(os.path.join(args.log_path, "config.yml"), "w") as f:
            yaml.safe_dump(config, f, default_flow_style=False)
    handlers = [logging.StreamHandler()]
    if training and rank == 0:
        os.makedirs(args.log_path, exist_ok=True)
        handlers.append(logging.FileHandler(os.path.join(args.log_path, "stdout.txt")))
    logging.basicConfig(level=level, format="%(levelname)s - %(filename)s - %(asctime)s - %(message)s",
                        handlers=handlers, force=True)
    if args.sample:
        args.image_folder = os.path.join(args.exp, "image_samples", args.image_folder)
    if args.sample and rank == 0:
        if os.path.exists(args.image_folder):
            if not args.ni and input("Image folder already exists. Overwrite? (Y/N)").upper() != "Y":
                print("Output image folder exists. Program halted.")
                sys.exit(0)
            shutil.rmtree(args.image_folder)
        os.makedirs(args.image_folder)
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    if not torch.cuda.is_available():
        raise RuntimeError("an MI355X (HIP device) is required: libsdp has no CPU path")
    torch.cuda.manual_seed_all(args.seed)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    new_config.device = torch.device("cuda", local)
    return args, new_config


def init_distributed(device):
    """torchrun env -> one process group over RCCL (xGMI); the ranks of a sampling run share
    tooHigh and gather their megabatches' images, the ranks of a training run average gradients."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not torch.distributed.is_initialized():
        torch.distributed.init_process_group("nccl", device_id=device)
        return True
    return False


def main(argv=None):
    args, config = parse_args_and_config(argv)
    logging.info("Config = %s", config.data.dataset)
    dist = init_distributed(config.device)
    if dist and args.sample:
        torch.distributed.barrier()          # rank 0 has (re)created the image folder
    from sdp.runner import Runner
    runner = Runner(args, config)
    try:
        if args.sample:
            runner.sample()
        elif args.test or args.nvs or args.fast_fid:
            raise NotImplementedError("--test / --nvs / --fast_fid are outside the simultaneous-sampling path")
        else:
            runner.train()
    finally:
        if dist:
            torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
