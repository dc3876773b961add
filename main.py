#!/usr/bin/env python3
"""Entry point mirroring the reference's `main.py --mode train|eval` (main.py:41-339, 501-549)
on the MI355X engine.  Other modes (inference over NIfTI, preprocess, analysis)
are outside the engine's scope and exit with a message.

    python main.py --mode train --config configs/c2_unet_96_bf16.yaml
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 main.py --mode train \
        --config configs/c3_dual_encoder_96_dp.yaml
"""
import argparse
import os
import sys
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import mmseg_amd  # noqa: E402,F401
from mmseg_amd.data import get_dataloader  # noqa: E402
from mmseg_amd.distributed import ddp  # noqa: E402
from mmseg_amd.models import build_model  # noqa: E402
from mmseg_amd.trainer import Trainer  # noqa: E402
from mmseg_amd.utils import load_config, set_seed, setup_logger  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Multi-Modal Medical Image Segmentation (MI355X engine)")
    p.add_argument("--mode", required=True, choices=["train", "eval", "inference", "preprocess", "analysis"])
    p.add_argument("--config", default="configs/c2_unet_96_bf16.yaml")
    p.add_argument("--exp-name", default=None)
    p.add_argument("--output-dir", default=None)
    p.add_argument("--input", default=None)
    p.add_argument("--output", default=None)
    p.add_argument("--checkpoint", default=None)
    p.add_argument("--resume", default=None)
    p.add_argument("--device", default=None, choices=["cuda", "cpu", "mps"])
    p.add_argument("--num-workers", type=int, default=None)
    p.add_argument("--epochs", type=int, default=None)
    p.add_argument("--batch-size", type=int, default=None)
    p.add_argument("--lr", type=float, default=None)
    p.add_argument("--model", default=None, choices=["swin_unetr", "unet", "attention_unet", "dual_encoder"])
    p.add_argument("--fusion", default=None, choices=["early", "late", "attention", "cross_attention"])
    p.add_argument("--modalities", nargs="+", default=None)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--verbose", "-v", action="store_true")
    p.add_argument("--debug", action="store_true")
    return p.parse_args(argv)


def merge_config_with_args(config, args):
    """reference main.py:245-307 (training-relevant keys)."""
    ex, hw, tr, md = config["experiment"], config["hardware"], config["training"], config["model"]
    if args.exp_name is not None:
        ex["name"] = args.exp_name
    if args.output_dir is not None:
        ex["output_dir"] = args.output_dir
    if args.seed is not None:
        ex["seed"] = args.seed
    if args.device is not None:
        hw["device"] = args.device
    if args.num_workers is not None:
        hw["num_workers"] = args.num_workers
    if args.epochs is not None:
        tr["epochs"] = args.epochs
    if args.batch_size is not None:
        tr["batch_size"] = args.batch_size
    if args.lr is not None:
        tr["optimizer"]["lr"] = args.lr
    if args.model is not None:
        md["name"] = args.model
    if args.fusion is not None:
        md.setdefault("fusion", {})["type"] = args.fusion
    if args.modalities is not None:
        config["data"]["modalities"] = args.modalities
    config["_args"] = {"mode": args.mode, "input": args.input, "output": args.output, "checkpoint": args.checkpoint,
                       "resume": args.resume, "verbose": args.verbose, "debug": args.debug}
    return config


def run_train(config, logger):
    train_loader = get_dataloader(config, split="train")
    val_loader = get_dataloader(config, split="val")
    model = build_model(config)
    trainer = Trainer(config=config, model=model, train_loader=train_loader, val_loader=val_loader, logger=logger,
                      resume_from=config["_args"].get("resume"))
    return trainer.train()


def run_eval(config, logger):
    from mmseg_amd.models.build import load_checkpoint
    model = build_model(config)
    if config["_args"].get("checkpoint"):
        load_checkpoint(model, config["_args"]["checkpoint"])
    trainer = Trainer(config=config, model=model, val_loader=get_dataloader(config, split="val"), logger=logger)
    metrics = trainer.evaluate()
    logger.info(f"Dice: {metrics['dice']:.4f} per class: {metrics['dice_per_class']}")
    return metrics


def main(argv=None):
    args = parse_args(argv)
    config = merge_config_with_args(load_config(args.config), args)
    local = ddp.init_from_env()
    if config["hardware"].get("device") == "cuda":
        import torch
        torch.cuda.set_device(local)
    log_dir = Path(config["experiment"].get("log_dir", "logs")) / config["experiment"]["name"]
    logger = setup_logger("main", log_dir / f"{args.mode}.log" if ddp.rank() == 0 else None,
                          "DEBUG" if args.debug else "INFO")
    set_seed(config["experiment"]["seed"])
    logger.info(f"Mode: {args.mode}  Config: {args.config}  world={ddp.world()}")
    if args.mode == "train":
        run_train(config, logger)
        logger.info("Training completed")
    elif args.mode == "eval":
        run_eval(config, logger)
    else:
        logger.error(f"--mode {args.mode} is outside the MI355X engine's scope (DESIGN.md 'Out of scope')")
        sys.exit(2)


if __name__ == "__main__":
    main()
