"""Throughput benchmark: 96^3 CT+PET training patches/s/node for the
DualEncoder + "cross_attention" (= mean fusion in the reference) training
step on the HIP engine, 1..8 MI355X (BASELINE.json metric / configs[2]).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = Trainer.train_step on one pre-staged synthetic phantom batch
(forward, DiceCE, backward, RCCL gradient all-reduce for N>1, AdamW),
accumulation_steps=1, dropout 0, bf16 activations / fp32 params+grads.
Per-GPU batch is fixed (weak scaling); value = N*B*K / max-over-ranks time.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0    # dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0

# Whole-step algorithmic work per 96^3 sample (SURVEY §8d / BASELINE.md): FLOPs of forward + backward
# (2 per MAC, torch FlopCounterMode on the reference) and compulsory HBM bytes with bf16 activations.
STEP_WORK = {("unet", 2): (1206.2e9, 4.15e9), ("dual_encoder", 2): (1559.4e9, 6.31e9),
             ("dual_encoder", 3): (1915.6e9, 8.20e9)}


def make_config(model, batch, dtype, out_channels=6, modalities=("CT", "PET"), size=96, loss="dice_ce",
                kernels="hip", amp="bf16", fp8=False):
    backbone = {"features": [32, 64, 128, 256, 512], "norm": "instance"}
    if model == "swin_unetr":     # config c4: SwinUNETR feature_size 48 (swin_unetr.py:180-200 defaults otherwise)
        backbone = {"img_size": [size] * 3, "feature_size": 48}
    return {
        "experiment": {"name": "bench", "output_dir": "/tmp/mmseg_bench", "seed": 42},
        "data": {"modalities": list(modalities)},
        "model": {"name": model, "in_channels": len(modalities), "out_channels": out_channels,
                  "backbone": backbone,
                  "fusion": {"type": "cross_attention"}, "head": {"dropout": 0.0}},
        "training": {"epochs": 1, "batch_size": batch, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": 1e-4, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": loss, "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None,
                              "tversky_alpha": 0.5, "tversky_beta": 0.5},
                     "checkpoint": {"save_last": False, "save_best": False}},
        "hardware": {"device": "cuda", "mixed_precision": dtype == "bf16", "kernels": kernels, "fp8": fp8,
                     # torch-op backend: bf16 autocast, or the reference's own fp16 autocast + GradScaler
                     "engine_dtype": "bfloat16" if dtype == "bf16" and not (kernels == "torch" and amp == "fp16")
                     else "float32"},
        "distributed": {"bucket_mb": 32},
    }


# ---------------------------------------------------------------------------------------------------------------
# Committed rocprofv3 summaries (profiles/*_steady.json, *_pmc_traffic.json, *_pmc_sq.json; tools/rocprof_families.py)
# carry the workload they were measured on ("_workload": workload_key() of the profiled bench run) and when
# ("_created").  A bench line reads only summaries of ITS OWN workload -- the newest by "_created" -- and leaves
# the rocprof / PMC fields null when none matches (then the dominant family comes from the live timer alone).
# ---------------------------------------------------------------------------------------------------------------
CONFIG_TAGS = {  # BASELINE.json configs (1 GPU per-rank shapes) -> tag used in profile file names
    ("dual_encoder", 2, 96, 2, "bf16", "dice_ce", False): "c3",
    ("unet", 2, 96, 2, "bf16", "dice_ce", False): "c2",
    ("swin_unetr", 2, 128, 1, "bf16", "dice_ce", False): "c4",
    ("dual_encoder", 3, 96, 2, "bf16", "tversky", False): "c5",
    ("dual_encoder", 3, 96, 2, "bf16", "tversky", True): "c5fp8",
}

WORKLOAD = None      # set by main(): workload_key(args)


def workload_key(model: str, modalities: int, size: int, batch: int, dtype: str, loss: str, fp8: bool,
                 kernels: str = "hip") -> dict:
    """What a profile summary must match to be used on a bench line: the per-GPU step's shape and arithmetic."""
    return {"model": model, "modalities": int(modalities), "size": int(size), "batch": int(batch), "dtype": dtype,
            "loss": loss, "fp8": bool(fp8), "kernels": kernels}


def workload_tag(w: dict) -> str:
    t = CONFIG_TAGS.get((w["model"], w["modalities"], w["size"], w["batch"], w["dtype"], w["loss"], w["fp8"]))
    if t is not None and w.get("kernels", "hip") == "hip":
        return t
    return f"{w['model']}-m{w['modalities']}-s{w['size']}-b{w['batch']}-{w['dtype']}-{w['loss']}" + \
        ("-fp8" if w["fp8"] else "") + ("" if w.get("kernels", "hip") == "hip" else "-" + w["kernels"])


_PROFILE_CACHE = {}


def _profile(kind: str):
    """(summary dict, repo-relative path) of the newest committed `kind` summary measured on WORKLOAD, else
    (None, None).  kind: steady | pmc_traffic | pmc_sq."""
    import glob
    if kind in _PROFILE_CACHE:
        return _PROFILE_CACHE[kind]
    best = (None, None, "")
    if WORKLOAD is not None:
        for f in glob.glob(os.path.join(ROOT, "profiles", f"*_{kind}.json")):
            try:
                with open(f) as fh:
                    d = json.load(fh)
            except (OSError, ValueError):
                continue
            if not isinstance(d, dict) or d.get("_workload") != WORKLOAD:
                continue
            created = str(d.get("_created", ""))
            if best[0] is None or created > best[2]:
                best = (d, os.path.relpath(f, ROOT), created)
    _PROFILE_CACHE[kind] = best[:2]
    return best[:2]


def _family_key(d: dict, kernel: str):
    """The timer's family name (mmseg_last_kernel(), e.g. conv3_brickr_kernel<BN64>) as a key of a rocprofv3
    summary (tools/rocprof_families.py: the same name, possibly with a [bf16] / [f32] suffix, or the bare kernel
    name for families the trace does not split by template)."""
    if kernel in d:
        return kernel
    for suf in ("[bf16]", "[f32]"):
        if kernel + suf in d:
            return kernel + suf
        if kernel.endswith(suf) and kernel[:-len(suf)] in d:
            return kernel[:-len(suf)]
    base = kernel.split("<")[0]
    return base if base in d else None


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from this workload's PMC summary (FETCH_SIZE x 2 + WRITE_SIZE)."""
    d, src = _profile("pmc_traffic")
    if d is None:
        return None, src
    key = _family_key(d, kernel)
    if key is None:
        return None, src
    return d[key]["hbm_bytes_per_launch"], src


def pmc_mfma_busy(kernel: str):
    """MFMA-pipe busy fraction of `kernel` from this workload's SQ counter summary (profiles/*_pmc_sq.json,
    tools/rocprof_families.py sq, from a separate rocprofv3 --pmc pass over this bench): SQ_VALU_MFMA_BUSY_CYCLES
    (summed over the 1,024 SIMDs) / (1,024 x GRBM_GUI_ACTIVE / 8 XCDs), with the VALU / LDS instructions issued
    per MFMA."""
    d, src = _profile("pmc_sq")
    if d is None:
        return None, None
    key = _family_key(d, kernel)
    if key is None:
        return None, src
    v = d[key]
    out = {"mfma_busy": round(v["mfma_busy"], 4)}
    for k in ("valu_per_mfma", "lds_per_mfma", "clock_ghz", "counter_gflop"):
        if v.get(k) is not None:
            out[k] = round(v[k], 3)
    return out, src


def rocprof_steady(kernel: str):
    """The kernel's steady-state average launch duration from this workload's rocprofv3 kernel-trace summary
    (profiles/*_steady.json: tools/rocprof_families.py steady over the last steps of a traced run of this bench),
    to set beside the live timer's."""
    d, src = _profile("steady")
    if d is None:
        return None, None
    key = _family_key(d, kernel)
    return (d[key]["avg_launch_ms"] if key is not None else None), src


def pmc_step_bytes():
    """HBM bytes of one whole training step from this workload's PMC summary: every kernel's bytes per launch x
    launches, over the steps the profiled run executed (its '_steps', else the AdamW launch count: one per step);
    the runtime's buffer copies / fills (input staging, arena set-up) are not part of a step."""
    d, src = _profile("pmc_traffic")
    if d is None:
        return None, None
    steps = d.get("_steps") or (d.get("adamw_pack_kernel") or d.get("adamw4_kernel") or {}).get("launches")
    if not steps:
        return None, src
    tot = sum(v["hbm_bytes_per_launch"] * v["launches"] for k, v in d.items()
              if not k.startswith(("_", "__amd_rocclr")) and isinstance(v, dict))
    return tot / steps, src


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_threads() -> int:
    """Threads for the CPU baseline: this process's CPU share (the GPU box's cgroup / OMP_NUM_THREADS: 16 per
    GPU there), not os.cpu_count(), which reports the whole host."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline_swin(model, batch, size, out_channels, modalities, threads, steps=1):
    """Config c4 on the host: oracle/swin_oracle.py (torch-CPU fp32 restatement of MONAI 1.3's SwinUNETR forward;
    parity vs MONAI itself unpinned) + the reference's DiceCE + backward + AdamW, from the GPU model's initial
    weights, on the same seeded phantoms: 1 warm-up step on a 64^3 patch, then `steps` timed full-size steps."""
    from oracle import mmseg_oracle as O
    from oracle import swin_oracle as SO
    from mmseg_amd.data.synthetic import SyntheticSegDataset
    torch.set_num_threads(threads)
    M = len(modalities)
    bb = model.backbone
    p = {k: v.detach().float().cpu() for k, v in bb.model.named_parameters()}
    fwd = lambda pp, x: SO.swin_unetr_forward(pp, x, bb.depths, bb.num_heads)  # noqa: E731
    st = O.OracleStep(p, fwd, O.dice_ce_loss)
    g = torch.Generator().manual_seed(5)
    st.step(torch.randn(1, M, 64, 64, 64, generator=g), torch.randint(0, out_channels, (1, 64, 64, 64), generator=g))
    ds = SyntheticSegDataset(steps * batch, size, out_channels, modalities, seed=1234)
    batches = []
    for i in range(steps):
        items = [ds[i * batch + j] for j in range(batch)]
        batches.append((torch.stack([it["image"] for it in items]), torch.stack([it["label"] for it in items])))
    t0 = time.perf_counter()
    for x, y in batches:
        st.step(x, y)
    dt = (time.perf_counter() - t0) / steps
    return {"value": batch / dt, "unit": "patches/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"{steps} oracle train step(s) (oracle/swin_oracle.py fwd + DiceCE + bwd + AdamW), swin_unetr "
                      f"fs=48 M={M} B={batch} {size}^3 fp32 on seeded phantoms, {dt:.2f} s/step on {threads} threads"}


def cpu_baseline(model_name, batch, size, out_channels, modalities, threads, loss="dice_ce", steps=3):
    """The oracle (torch-CPU fp32 restatement of the reference step: forward, loss, backward, AdamW) on the
    host cores, on the same seeded phantom batches as the GPU run: 1 warm-up step on a 32^3 patch, then `steps`
    timed full-size steps (a bounded sample, ~10-30 s); value = patches / mean step time."""
    from oracle import mmseg_oracle as O
    from mmseg_amd.data.synthetic import SyntheticSegDataset
    torch.set_num_threads(threads)
    M = len(modalities)
    feats = [32, 64, 128, 256, 512]
    torch.manual_seed(0)
    if model_name == "dual_encoder":
        p = O.init_dual_encoder(M, out_channels, feats, "cross_attention")
        fwd = lambda pp, x: O.dual_encoder_forward(pp, x, "cross_attention")  # noqa: E731
    else:
        p = O.init_unet3d(M, out_channels, feats)
        fwd = O.unet3d_forward
    st = O.OracleStep(p, fwd, O.tversky_loss if loss == "tversky" else O.dice_ce_loss)
    g = torch.Generator().manual_seed(5)
    st.step(torch.randn(1, M, 32, 32, 32, generator=g), torch.randint(0, out_channels, (1, 32, 32, 32), generator=g))
    ds = SyntheticSegDataset(steps * batch, size, out_channels, modalities, seed=1234)
    batches = []
    for i in range(steps):
        items = [ds[i * batch + j] for j in range(batch)]
        batches.append((torch.stack([it["image"] for it in items]), torch.stack([it["label"] for it in items])))
    t0 = time.perf_counter()
    for x, y in batches:
        st.step(x, y)
    dt = (time.perf_counter() - t0) / steps
    return {"value": batch / dt, "unit": "patches/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"{steps} oracle train steps (fwd+{'Tversky' if loss == 'tversky' else 'DiceCE'}+bwd+AdamW), "
                      f"{model_name} M={M} B={batch} {size}^3 fp32 on seeded phantoms, {dt:.2f} s/step on "
                      f"{threads} threads"}


def bench_infer(args, trainer, model, mods, dev):
    """Sliding-window inference at the config's window (roi 96^3, sw_batch 4, overlap 0.5): --infer-volumes
    seeded phantom volumes of --infer-size^3 resident in HBM, one warm-up call, then --steps timed calls."""
    from mmseg_amd.data import device_batches
    model.eval()
    S, V = args.infer_size, args.infer_volumes
    img = device_batches(1, V, S, 6, mods, dev, seed=4321)[0]["image"]
    with torch.no_grad():
        for _ in range(max(args.warmup, 1)):
            out = trainer._sliding_window_inference(img)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = trainer._sliding_window_inference(img)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    import math
    nwin = 1
    for _ in range(3):
        iv = int(96 * 0.5)
        num = int(math.ceil(S / iv))
        nwin *= next((i for i in range(num) if i * iv + 96 >= S), num - 1) + 1
    ms_vol = el / (args.steps * V) * 1e3
    print(json.dumps({
        "metric": f"sliding-window inference {S}^3 {len(mods)}-modality volumes/sec (roi 96^3, sw_batch 4, "
                  f"overlap 0.5)", "value": round(1e3 / ms_vol, 3), "unit": "volumes/s", "n_gpus": 1,
        "steps": args.steps, "warmup": max(args.warmup, 1), "ms_per_volume": round(ms_vol, 3),
        "higher_is_better": True, "dtype": args.dtype, "data": "synthetic (seeded phantoms, resident in HBM)",
        "windows_per_volume": nwin, "ms_per_window": round(ms_vol / nwin, 3),
        "config": {"workload": f"{args.model} sliding_window_inference, {V} x {S}^3, 6 classes",
                   "model": args.model, "volumes": V, "size": S, "roi": [96, 96, 96], "sw_batch": 4,
                   "overlap": 0.5},
        "out_finite": bool(torch.isfinite(out).all().item())}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="dual_encoder", choices=["dual_encoder", "unet", "swin_unetr"],
                    help="swin_unetr = config c4 (use --size 128 --batch 1)")
    ap.add_argument("--batch", type=int, default=2, help="per-GPU batch")
    ap.add_argument("--size", type=int, default=96)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--modalities", default="CT,PET", help="c5: CT,PET,MRI")
    ap.add_argument("--loss", default="dice_ce", choices=["dice_ce", "tversky"], help="c5: tversky")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: this process's CPU share (cpu_threads())")
    ap.add_argument("--cpu-steps", type=int, default=3, help="timed oracle steps in the CPU baseline")
    ap.add_argument("--timer-steps", type=int, default=3, help="extra steps timed per kernel family (roofline)")
    ap.add_argument("--kernels", default="hip", choices=["hip", "torch"],
                    help="torch: the same model / step through PyTorch-ROCm ops (MIOpen convs; hardware.kernels A/B)")
    ap.add_argument("--fp8", action="store_true",
                    help="config c5's mixed bf16/fp8: e4m3 forward convolutions where the kernel takes them")
    ap.add_argument("--fresh-inputs", action="store_true",
                    help="every step's batch at a new device address (a DataLoader's pattern): the captured step "
                         "runs its copy-graph path (trainer/step_graph.py) instead of a pointer-keyed graph")
    ap.add_argument("--timer-dump", default="", help="write every timed launch (family, site, ms, flops) as JSON")
    ap.add_argument("--amp", default="bf16", choices=["bf16", "fp16"],
                    help="--kernels torch autocast dtype (fp16 + GradScaler = the reference's GPU mode)")
    ap.add_argument("--dp-rehearsal", action="store_true",
                    help="one GPU, the data-parallel step: an RCCL process group of world size 1 with "
                         "distributed.reduce_single_rank, so the bucket all-reduces really run through RCCL inside the "
                         "captured step at the points each rank of the N-GPU job issues them.  At world size 1 the "
                         "collective is SUM (AVG is the identity there; RCCL's single-rank AVG adds a scaling pass, "
                         "~0.24 ms/step, that an N-rank AVG folds into the reduction), so that pass is not in the "
                         "rehearsed time")
    ap.add_argument("--bucket-mb", type=float, default=32.0, help="DP gradient bucket size (distributed.bucket_mb)")
    ap.add_argument("--infer", action="store_true",
                    help="secondary line: sliding-window inference (Trainer._sliding_window_inference, reference "
                         "trainer.py:370-395 with default.yaml's roi 96^3 / sw_batch 4 / overlap 0.5) over "
                         "--infer-volumes volumes of --infer-size^3, timed per volume; not the headline metric")
    ap.add_argument("--infer-size", type=int, default=160)
    ap.add_argument("--infer-volumes", type=int, default=2)
    ap.add_argument("--workload-out", default="", help="write this run's workload key (JSON) for the profile "
                                                       "summaries of tools/rocprof_families.py")
    args = ap.parse_args()
    global WORKLOAD
    WORKLOAD = workload_key(args.model, len(args.modalities.split(",")), args.size, args.batch, args.dtype, args.loss,
                            args.fp8, args.kernels)
    if args.workload_out:
        with open(args.workload_out, "w") as f:
            json.dump(WORKLOAD, f)

    import mmseg_amd  # noqa: F401
    from mmseg_amd.data import device_batches
    from mmseg_amd.distributed import ddp
    from mmseg_amd.engine.profiler import TIMER
    from mmseg_amd.models.build import build_model
    from mmseg_amd.trainer.trainer import Trainer

    # MMSEG_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin)
    local = ddp.init_from_env(os.environ.get("MMSEG_DIST_BACKEND", "nccl"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    rank, world = ddp.rank(), ddp.world()
    n_gpus = world
    if args.dp_rehearsal:
        if world != 1:
            raise SystemExit("--dp-rehearsal is the one-GPU rehearsal of the DP step (world size 1)")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)

    mods = args.modalities.split(",")
    cfg = make_config(args.model, args.batch, args.dtype, size=args.size, modalities=mods, loss=args.loss,
                      kernels=args.kernels, amp=args.amp, fp8=args.fp8)
    cfg["distributed"]["bucket_mb"] = args.bucket_mb
    if args.dp_rehearsal:
        cfg["distributed"]["reduce_single_rank"] = True
    if args.kernels == "torch":
        args.no_cpu_baseline = True
        args.timer_steps = 0
    if args.infer:
        cfg["inference"] = {"sliding_window": {"roi_size": [96, 96, 96], "overlap": 0.5}, "batch_size": 4}
        torch.manual_seed(42)
        model = build_model(cfg)
        trainer = Trainer(cfg, model)
        bench_infer(args, trainer, model, mods, dev)
        return
    torch.manual_seed(42)
    model = build_model(cfg)
    trainer = Trainer(cfg, model)
    batches = device_batches(4, args.batch, args.size, 6, mods, dev, seed=1234 + 1000 * rank)

    def barrier():
        if world > 1:
            dist.barrier()

    if args.fresh_inputs:
        # no pointer-keyed graphs: every replay first copies its batch into the static input buffers of the copy
        # graph, as it does for a loader that hands over a new address every step
        trainer._graphs.MAX_GRAPHS = 0
    step = 0
    for _ in range(args.warmup):
        trainer.train_step(batches[step % len(batches)], step, sync=False)
        step += 1
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = trainer.train_step(batches[step % len(batches)], step, sync=False)
        step += 1
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    loss_val = float(last.item()) if last is not None else float("nan")

    # per-kernel-family timing over a separate live window: eager steps (a captured graph has no per-launch
    # timing) whose every library kernel is launched with hipExtLaunchKernelGGL start / stop events, stamped by
    # the runtime from the dispatch itself -- the interval rocprofv3's kernel trace reports (engine/profiler.py)
    TIMER.start()
    for _ in range(args.timer_steps):
        trainer.train_step(batches[step % len(batches)], step, sync=False)
        step += 1
    TIMER.stop()
    if args.timer_dump and rank == 0:
        with open(args.timer_dump, "w") as f:
            json.dump({"timer_steps": args.timer_steps, "launches": TIMER.records()}, f)
    fam = TIMER.summary()
    # the dominant MFMA kernel: the family with algorithmic FLOPs and the largest time per step (helper launches
    # without FLOPs -- split reduces, packing, norms -- are HBM-bound and listed in kernel_families)
    mfma = {k: v for k, v in fam.items() if v["flops"] > 0}
    dom = max(mfma.items(), key=lambda kv: kv[1]["ms"]) if mfma else None
    # ... chosen by rocprofv3 time per step of the captured step where a committed steady-state trace summary
    # names the family (tools/rocprof_families.py uses the timer's family names), else by the timer's own time
    steady, _ = _profile("steady")
    if mfma and steady:
        def _rp_ms(kv):
            key = _family_key(steady, kv[0])
            return steady[key]["ms_per_step"] if key is not None else -1.0
        best = max(mfma.items(), key=_rp_ms)
        if _rp_ms(best) > 0:
            dom = best

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    value = n_gpus * args.batch * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    roofline = None
    if dom is not None:
        name, a = dom
        avg_ms = a["ms"] / a["launches"]
        flops_per_launch = a["flops"] / a["launches"]
        bytes_per_launch = a["bytes"] / a["launches"]
        achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12
        peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
        traffic, tsrc = pmc_traffic(name)
        roofline = {"bound": "mfma", "kernel": name, "achieved": round(achieved, 2), "peak": peak,
                    "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                    "traffic": round(traffic) if traffic is not None else None, "traffic_unit": "B/launch",
                    "traffic_source": tsrc,
                    "avg_launch_ms": round(avg_ms, 4), "launches_per_step": a["launches"] // max(args.timer_steps, 1),
                    "algorithmic_gflop_per_launch": round(flops_per_launch / 1e9, 3),
                    "algorithmic_bytes_per_launch": round(bytes_per_launch),
                    "timer": "hipExtLaunchKernelGGL start/stop events on the launching stream (dispatch "
                             "timestamps, the rocprofv3 kernel-trace interval)"}
        rp, rsrc = rocprof_steady(name)
        if rp is not None:
            # the same family in the committed rocprofv3 trace (steady-state steps): frac from its duration
            roofline["rocprof_avg_launch_ms"] = round(rp, 4)
            roofline["rocprof_frac"] = round(flops_per_launch / (rp * 1e-3) / 1e12 / peak, 4)
            roofline["rocprof_vs_timer"] = round(rp / avg_ms, 4)
            roofline["rocprof_source"] = rsrc
        busy, bsrc = pmc_mfma_busy(name)
        if busy is not None:
            # SQ_VALU_MFMA_BUSY_CYCLES x 1,024 FLOPs / SIMD-cycle re-counts the MFMA work from the counters alone:
            # counter_gflop / algorithmic_gflop ~ 1 (above 1 only by K padding) pins the FLOPs `achieved` divides
            if busy.get("counter_gflop") is not None:
                busy["counter_gflop_per_launch"] = round(busy.pop("counter_gflop"), 3)
                busy["counter_vs_algorithmic"] = round(busy["counter_gflop_per_launch"] * 1e9 / flops_per_launch, 4)
            roofline.update(busy)
            roofline["mfma_busy_source"] = bsrc
    families = {k: {"ms_per_step": round(v["ms"] / args.timer_steps, 3),
                    "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1) if v["ms"] > 0 else None}
                for k, v in sorted(fam.items(), key=lambda kv: -kv[1]["ms"])}
    # every MFMA family of the step with its algorithmic work, frac of the dense peak (live timer), and -- from this
    # workload's committed rocprofv3 summaries -- its trace duration and SQ counters
    peak_f = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
    mfma_families = {}
    for k, v in sorted(mfma.items(), key=lambda kv: -kv[1]["ms"]):
        fl = v["flops"] / v["launches"]
        e = {"ms_per_step": round(v["ms"] / max(args.timer_steps, 1), 4), "launches_per_step":
             round(v["launches"] / max(args.timer_steps, 1), 2), "gflop_per_launch": round(fl / 1e9, 4),
             "avg_launch_ms": round(v["ms"] / v["launches"], 4),
             "frac": round(fl / (v["ms"] / v["launches"] * 1e-3) / 1e12 / peak_f, 4)}
        rp, _ = rocprof_steady(k)
        if rp:
            e["rocprof_avg_launch_ms"] = round(rp, 4)
            e["rocprof_frac"] = round(fl / (rp * 1e-3) / 1e12 / peak_f, 4)
        busy, _ = pmc_mfma_busy(k)
        if busy is not None:
            e.update({kk: busy[kk] for kk in ("mfma_busy", "valu_per_mfma", "lds_per_mfma") if kk in busy})
        tr, _ = pmc_traffic(k)
        if tr is not None:
            e["traffic_vs_algorithmic"] = round(tr / max(v["bytes"] / v["launches"], 1.0), 3)
        # the family's own roofline: below the ridge (peak FLOP/s / peak B/s = 312.5 FLOP/B for bf16) a launch is
        # bound by its compulsory HBM bytes, not by the matrix cores (the SwinUNETR token GEMMs, K = 48..192)
        nb = v["bytes"] / v["launches"]
        if nb > 0:
            e["gbyte_per_launch"] = round(nb / 1e9, 5)
            e["gbps"] = round(nb / (v["ms"] / v["launches"] * 1e-3) / 1e9, 1)
            e["hbm_frac"] = round(e["gbps"] / PEAK_HBM_GBS, 4)
            e["bound"] = "hbm" if fl / nb < peak_f / (PEAK_HBM_GBS / 1e3) else "mfma"
        mfma_families[k] = e
    step = None
    work = STEP_WORK.get((args.model, len(mods)))
    if work is not None and args.size == 96 and args.dtype == "bf16":
        F, Bt = work[0] * args.batch, work[1] * args.batch
        t_mfma, t_hbm = F / (PEAK_BF16_TFLOPS * 1e12), Bt / (PEAK_HBM_GBS * 1e9)
        t_roof = max(t_mfma, t_hbm)
        counter, csrc = pmc_step_bytes() if args.kernels == "hip" and not args.fp8 else (None, None)
        step = {"bound": "hbm" if t_hbm >= t_mfma else "mfma", "algorithmic_tflop": round(F / 1e12, 3),
                "compulsory_gb": round(Bt / 1e9, 3), "t_mfma_ms": round(t_mfma * 1e3, 3),
                "t_hbm_ms": round(t_hbm * 1e3, 3), "t_roof_ms": round(t_roof * 1e3, 3),
                "frac": round(t_roof * 1e3 / ms_per_step, 4),
                "counter_gb": round(counter / 1e9, 3) if counter is not None else None,
                "counter_source": csrc,
                "counter_tbps": round(counter / (ms_per_step * 1e-3) / 1e12, 3) if counter is not None else None}
    elif args.dtype == "bf16" and args.timer_steps > 0 and fam:
        # no SURVEY 8(d) whole-step model for this workload (c4 SwinUNETR 128^3): the step's algorithmic work is
        # the sum over every timed launch of its region's algorithmic FLOPs and compulsory bytes (each kernel's
        # inputs + outputs once, engine/layers.py / swin.py regions) -- per-kernel compulsory traffic, so an
        # upper bound on the whole-step compulsory bytes (tensors passed between kernels are counted twice)
        F = sum(v["flops"] for v in fam.values()) / args.timer_steps
        Bt = sum(v["bytes"] for v in fam.values()) / args.timer_steps
        t_mfma, t_hbm = F / (PEAK_BF16_TFLOPS * 1e12), Bt / (PEAK_HBM_GBS * 1e9)
        t_roof = max(t_mfma, t_hbm)
        counter, csrc = pmc_step_bytes() if args.kernels == "hip" and not args.fp8 else (None, None)
        step = {"bound": "hbm" if t_hbm >= t_mfma else "mfma", "algorithmic_tflop": round(F / 1e12, 3),
                "compulsory_gb": round(Bt / 1e9, 3), "t_mfma_ms": round(t_mfma * 1e3, 3),
                "t_hbm_ms": round(t_hbm * 1e3, 3), "t_roof_ms": round(t_roof * 1e3, 3),
                "frac": round(t_roof * 1e3 / ms_per_step, 4),
                "work_source": "sum of the timed launches' algorithmic FLOPs / per-kernel compulsory bytes",
                "counter_gb": round(counter / 1e9, 3) if counter is not None else None,
                "counter_source": csrc,
                "counter_tbps": round(counter / (ms_per_step * 1e-3) / 1e12, 3) if counter is not None else None}
    if step is not None:
        if args.timer_steps > 0 and fam:
            step["timer_sum_tflop"] = round(sum(v["flops"] for v in fam.values()) / args.timer_steps / 1e12, 3)
            step["timer_sum_gb"] = round(sum(v["bytes"] for v in fam.values()) / args.timer_steps / 1e9, 3)
        if roofline is not None:
            roofline["step"] = step
        else:
            roofline = {"step": step}
    cpu = None
    if n_gpus == 1 and not args.no_cpu_baseline and args.model == "swin_unetr":
        cpu = cpu_baseline_swin(model, args.batch, args.size, 6, mods, args.cpu_threads or cpu_threads(),
                                steps=max(1, min(args.cpu_steps, 1)))
    elif n_gpus == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.model, args.batch, args.size, 6, mods, args.cpu_threads or cpu_threads(),
                           loss=args.loss, steps=args.cpu_steps)
    workload = {"dual_encoder": "DualEncoder fusion=cross_attention (mean, dual_encoder.py:193-195)",
                "unet": "UNet3D early_fusion",
                "swin_unetr": "SwinUNETR feature_size 48 (MONAI architecture; parity vs MONAI unpinned)"}[
        args.model]
    out = {
        "metric": f"{args.size}^3 {len(mods)}-modality patches/sec/node (train step)",
        "value": round(value, 3), "unit": "patches/s", "n_gpus": n_gpus, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": (args.dtype + ("+fp8" if args.fp8 else "")) if args.kernels == "hip"
        else f"{args.amp if args.dtype == 'bf16' else 'fp32'}-autocast",
        "data": f"synthetic (seeded {'/'.join(mods)} phantoms, pre-staged in HBM"
                f"{', a new address every step (copy-graph path)' if args.fresh_inputs else ''})",
        "config": {"workload": f"{workload} {args.size}^3, modalities {'+'.join(mods)}, 6 classes, "
                               f"{'DiceCE' if args.loss == 'dice_ce' else 'Tversky'}, AdamW, per-GPU batch {args.batch}",
                   "model": args.model, "global_batch": args.batch * n_gpus, "patch": [args.size] * 3,
                   "parallelism": f"dp{n_gpus}" + ("-rccl-rehearsal" if args.dp_rehearsal else ""),
                   "kernels": args.kernels, "tag": workload_tag(WORKLOAD)},
        "loss": round(loss_val, 5),
        # the timed steps replay captured graphs (trainer/step_graph.py): how many were captured (0: eager steps)
        "captured_graphs": (len(trainer._graphs.graphs) + (trainer._graphs.copy_graph is not None))
        if getattr(trainer, "_graphs", None) is not None else 0,
        "roofline": roofline,
        "cpu_baseline": cpu,
        "kernel_families": families,
        "mfma_families": mfma_families,
        "profiles": {kind: _profile(kind)[1] for kind in ("steady", "pmc_traffic", "pmc_sq")},
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    elif args.dp_rehearsal:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
