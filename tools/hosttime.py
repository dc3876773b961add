"""Host-side submission time of one training step (no synchronisation inside the timed window) against the
GPU wall time per step: if the two are close, the step is bound by host launch overhead, not by the GPU.

    python tools/hosttime.py [--steps 3]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--model", default="dual_encoder")
    args = ap.parse_args()
    import mmseg_amd  # noqa: F401
    from bench import make_config
    from mmseg_amd.data import device_batches
    from mmseg_amd.models.build import build_model
    from mmseg_amd.trainer.trainer import Trainer

    dev = torch.device("cuda", 0)
    cfg = make_config(args.model, 2, "bf16")
    torch.manual_seed(0)
    tr = Trainer(cfg, build_model(cfg))
    batches = device_batches(2, 2, 96, 6, ["CT", "PET"], dev)
    for i in range(5):
        tr.train_step(batches[i % 2], i, sync=False)
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        host = []
        for i in range(args.steps):
            h0 = time.perf_counter()
            tr.train_step(batches[i % 2], i, sync=False)
            host.append(time.perf_counter() - h0)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host per step {[round(h * 1e3, 2) for h in host]} ms; submit {1e3 * (t1 - t0) / args.steps:.2f} "
              f"ms/step; wall {1e3 * (t2 - t0) / args.steps:.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
