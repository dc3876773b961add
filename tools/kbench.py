"""In-process A/B of kernel variants (env knobs read at launch time), interleaved
rounds in ONE process (cdna_hip_programming.md §5.4 rule 24).

    python tools/kbench.py --variants "MMSEG_WGRAD_ROW=0,1" "MMSEG_BRICK8=0,1"
Prints per-variant median step time and per-kernel-family ms/step.
"""
import argparse
import itertools
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="*", default=[])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--model", default="dual_encoder")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--layers", action="store_true", help="also print every timed launch of the last step")
    args = ap.parse_args()
    # eager steps: a captured step graph would replay the first variant's kernels for every variant
    os.environ.setdefault("MMSEG_STEP_GRAPH", "0")
    import mmseg_amd  # noqa: F401
    from bench import make_config
    from mmseg_amd.data import device_batches
    from mmseg_amd.engine.profiler import TIMER
    from mmseg_amd.models.build import build_model
    from mmseg_amd.trainer.trainer import Trainer

    dev = torch.device("cuda", 0)
    cfg = make_config(args.model, 2, args.dtype)
    torch.manual_seed(0)
    tr = Trainer(cfg, build_model(cfg))
    batches = device_batches(2, 2, 96, 6, ["CT", "PET"], dev)
    knobs = []
    for v in args.variants:
        k, vals = v.split("=")
        knobs.append([(k, x) for x in vals.split(",")])
    combos = list(itertools.product(*knobs)) or [()]
    res = {c: [] for c in combos}
    fams = {c: None for c in combos}
    step = 0
    for c in combos:  # warm every variant once
        for k, x in c:
            os.environ[k] = x
        for _ in range(2):
            tr.train_step(batches[step % 2], step, sync=False)
            step += 1
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for c in combos:
            for k, x in c:
                os.environ[k] = x
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.train_step(batches[step % 2], step, sync=False)
                step += 1
            torch.cuda.synchronize()
            res[c].append((time.perf_counter() - t0) / args.steps * 1e3)
            if r == args.rounds - 1:
                TIMER.start()
                tr.train_step(batches[step % 2], step, sync=False)
                step += 1
                TIMER.stop()
                fams[c] = {k: round(v["ms"], 3) for k, v in sorted(TIMER.summary().items(), key=lambda kv: -kv[1]["ms"])}
                if args.layers:
                    for i, (name, fl, nb, s0, s1) in enumerate(TIMER.records):
                        us = s0.elapsed_time(s1) * 1e3
                        print(f"layer {i:3d} {name:45s} {fl / 1e9:8.2f} GF {nb / 1e6:8.1f} MB {us:8.1f} us "
                              f"{fl / us / 1e6 if us else 0:7.1f} TF/s")
    for c in combos:
        print(json.dumps({"variant": dict(c), "median_ms": round(statistics.median(res[c]), 3),
                          "min_ms": round(min(res[c]), 3), "families": fams[c]}))


if __name__ == "__main__":
    main()
