"""Data parallelism through the real engine on one GPU: two gloo ranks share
cuda:0, each runs Trainer.train_step on its half of the global batch, and the
result must equal one rank running the whole batch ("N ranks x B ==
1 rank x N*B").

This drives the device-tensor path of GradBuckets end to end: the engine's
flat.mark callbacks from several modality streams, the dedicated comm stream
waiting on the writers' events, async all-reduce + wk.wait(), and finish()'s
late buckets.  RCCL itself needs one GPU per rank, so its two-rank run is
left to the 8-GPU node (DESIGN (e)); gloo over device tensors takes the same
stream / event path with SUM after a pre-scale on the comm stream.

Also: validation with fewer validation batches than ranks (a rank with none
still packs its device accumulators and its batch count of 0)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FEATS = [8, 16, 32, 64, 128]
S, B_GLOBAL, M, C, STEPS = 32, 4, 2, 3, 2


def _cfg(tmp):
    return {
        "experiment": {"name": "dp", "output_dir": tmp, "seed": 0},
        "data": {"modalities": ["CT", "PET"]},
        "model": {"name": "dual_encoder", "in_channels": M, "out_channels": C,
                  "backbone": {"features": FEATS, "norm": "instance"},
                  "fusion": {"type": "cross_attention"}, "head": {"dropout": 0.0}},
        "training": {"epochs": 1, "batch_size": B_GLOBAL, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": 1e-3, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": "dice_ce", "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None},
                     "checkpoint": {"save_last": False, "save_best": False}},
        "distributed": {"bucket_mb": 0.25},      # many buckets: most reduce while the backward still runs
        # eager steps: the test reads the gradient arena inside optimizer.step, which a replayed captured step
        # (world size 1, trainer/step_graph.py) does not call
        "hardware": {"device": "cuda", "mixed_precision": False, "engine_dtype": "float32", "step_graph": False},
    }


def _data():
    g = torch.Generator().manual_seed(77)
    xs = torch.randn(STEPS, B_GLOBAL, M, S, S, S, generator=g)
    ys = torch.randint(0, C, (STEPS, B_GLOBAL, S, S, S), generator=g)
    return xs, ys


def _run(rank, world, val_batches):
    """Train STEPS steps on this rank's shard; return the gradient arena before every optimizer step,
    the final weights, and the validation result."""
    import mmseg_amd  # noqa: F401
    from mmseg_amd.distributed import ddp
    from mmseg_amd.models.build import build_model
    from mmseg_amd.trainer.trainer import Trainer
    cfg = _cfg(f"/tmp/mmseg_dp_{rank}_{world}")
    torch.manual_seed(0)
    model = build_model(cfg)
    tr = Trainer(cfg, model, val_loader=val_batches)
    grads = []
    step = tr.optimizer.step

    def step_and_capture(*a, **k):
        torch.cuda.synchronize()
        grads.append(tr._engine_flat().grad_flat.detach().cpu().clone())
        return step(*a, **k)

    tr.optimizer.step = step_and_capture
    xs, ys = _data()
    idx = ddp.shard_indices(B_GLOBAL, rank, world)
    losses = [tr.train_step({"image": xs[s][idx], "label": ys[s][idx]}, s) for s in range(STEPS)]
    torch.cuda.synchronize()
    weights = torch.cat([p.detach().reshape(-1).cpu() for n, p in model.named_parameters()
                         if n.endswith("weight")])
    vloss, met = tr._validate()
    return {"grads": [g.numpy() for g in grads], "weights": weights.numpy(), "losses": losses,
            "vloss": vloss, "dice": met["dice_per_class"], "idx": idx}


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK="0")
        if ROOT not in sys.path:
            sys.path.insert(0, ROOT)
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        xs, ys = _data()
        # one validation batch in all: rank 0 gets it, rank 1 none (n_val < world)
        val = [{"image": xs[0][:2], "label": ys[0][:2]}] if rank == 0 else []
        res = _run(rank, world, val)
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # surface worker failures instead of a queue timeout
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _l2rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_two_gloo_ranks_on_one_gpu_equal_one_rank_full_batch(dev):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in res:
        assert r[1] == "ok", r[2]
    res = {r[0]: r[2] for r in res}
    assert res[0]["idx"] == [0, 2] and res[1]["idx"] == [1, 3]

    xs, ys = _data()
    single = _run(0, 1, [{"image": xs[0][:2], "label": ys[0][:2]}])
    for s in range(STEPS):
        # both ranks hold the same averaged gradient, and it is the full-batch gradient
        assert np.array_equal(res[0]["grads"][s], res[1]["grads"][s]), f"ranks disagree at step {s}"
        err = _l2rel(res[0]["grads"][s], single["grads"][s])
        # step 0: same weights, so only the reduction order differs.  Step 1 starts from weights that
        # differ by AdamW's rounding of near-equal gradients (first-step updates are lr * g / (|g| + eps),
        # steep where |g| ~ eps), which flips a few ReLU / MaxPool decisions and routes those voxels'
        # gradients discretely (DESIGN (c)): L2 ~1e-3 measured.
        assert err < (1e-5 if s == 0 else 1e-2), (s, err)
        # per-rank losses average to the full-batch loss (Dice mean over (b,c), CE mean over voxels)
        assert abs((res[0]["losses"][s] + res[1]["losses"][s]) / 2 - single["losses"][s]) < (1e-5 if s == 0
                                                                                               else 1e-4)
    assert np.array_equal(res[0]["weights"], res[1]["weights"])
    # the weights inherit step 1's gradient differences through AdamW, whose early updates are ~lr * sign(g)
    # wherever |g| is near eps: a rounding-level gradient difference there moves a weight by up to ~lr, so the
    # bound is lr-scaled per element and loose in L2 (< 1e-4 measured, then 3.6e-4 after the weight-gradient
    # reduce changed its fixed summation order)
    lr = 1e-3
    assert np.abs(res[0]["weights"] - single["weights"]).max() <= 2 * lr * STEPS
    assert _l2rel(res[0]["weights"], single["weights"]) < 1e-3
    # validation: the one batch lives on rank 0; both ranks report the same result, which is the
    # single-rank one up to the trained weights' rounding differences
    assert res[0]["vloss"] == res[1]["vloss"] and res[0]["dice"] == res[1]["dice"]
    assert abs(res[0]["vloss"] - single["vloss"]) < 1e-4
    assert np.abs(np.array(res[0]["dice"]) - np.array(single["dice"])).max() < 1e-3


def _bad_label_worker(rank, world, port, q):
    """Step 0 good on both ranks; step 1: rank 1's batch holds one label == C.  Every rank must raise at step
    1 and keep the weights of step 0 (the summed guard makes every rank's AdamW kernel skip)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK="0")
        if ROOT not in sys.path:
            sys.path.insert(0, ROOT)
        import torch.distributed as dist
        import mmseg_amd  # noqa: F401
        from mmseg_amd.distributed import ddp
        from mmseg_amd.models.build import build_model
        from mmseg_amd.trainer.trainer import Trainer
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cfg = _cfg(f"/tmp/mmseg_dpbad_{rank}")
        torch.manual_seed(0)
        model = build_model(cfg)
        tr = Trainer(cfg, model)
        xs, ys = _data()
        idx = ddp.shard_indices(B_GLOBAL, rank, world)
        tr.train_step({"image": xs[0][idx], "label": ys[0][idx]}, 0)
        w0 = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
        lab = ys[1][idx].clone()
        if rank == 1:
            lab[0, 0, 0, 0] = C
        raised = False
        try:
            tr.train_step({"image": xs[1][idx], "label": lab}, 1)
        except RuntimeError as e:
            raised = "outside" in str(e)
        w1 = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
        dist.destroy_process_group()
        q.put((rank, "ok", {"raised": raised, "unchanged": bool(torch.equal(w0, w1)), "w": w1.numpy()}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_bad_labels_on_one_rank_raise_on_every_rank(dev):
    """under DP only the rank with bad labels used to raise, and the others went on to the next
    all-reduce and hung.  The guard count now rides with the first gradient bucket (SUM)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bad_label_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in res:
        assert r[1] == "ok", r[2]
    res = {r[0]: r[2] for r in res}
    for r in (0, 1):
        assert res[r]["raised"], f"rank {r} did not raise"
        assert res[r]["unchanged"], f"rank {r} updated its weights on the bad step"
    assert np.array_equal(res[0]["w"], res[1]["w"])


def _rccl_graph_worker(port, q):
    """One process, RCCL (backend "nccl") at world size 1 with distributed.reduce_single_rank: the bucket
    all-reduces (ReduceOp.AVG on the comm stream) really run, eagerly and recorded inside the captured step.
    Three runs of the same steps: eager DP, captured DP, captured without DP."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        if ROOT not in sys.path:
            sys.path.insert(0, ROOT)
        import torch.distributed as dist
        import mmseg_amd  # noqa: F401
        from mmseg_amd.models.build import build_model
        from mmseg_amd.trainer.trainer import Trainer
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        xs, ys = _data()
        dev = torch.device("cuda", 0)
        batches = [{"image": xs[s].to(dev), "label": ys[s].to(dev)} for s in range(STEPS)]
        from mmseg_amd.trainer import step_graph as SG
        out = {}
        for tag, graph, dp, fail in (("eager_dp", False, True, False), ("graph_dp", True, True, False),
                                     ("graph", True, False, False), ("graph_dp_fail", True, True, True)):
            os.environ["MMSEG_STEP_GRAPH"] = "1" if graph else "0"
            cfg = _cfg(f"/tmp/mmseg_rccl_{tag}")
            cfg["hardware"]["step_graph"] = True
            cfg["distributed"]["reduce_single_rank"] = dp
            torch.manual_seed(0)
            from mmseg_amd.distributed import ddp
            orig = ddp.GradBuckets._reduce
            calls = []
            if fail:
                # a DP capture that fails MID-BACKWARD (advisor r05): the first bucket's collective raises inside
                # the capture, after the engine has already reported gradients; the trainer must fall back to the
                # eager DP step with a clean bucket state, every bucket reduced exactly once per eager step
                def _boom(self, b):
                    if torch.cuda.is_current_stream_capturing():
                        raise RuntimeError("injected capture failure")
                    calls.append(b)
                    return orig(self, b)
                ddp.GradBuckets._reduce = _boom
            try:
                model = build_model(cfg)
                tr = Trainer(cfg, model)
                losses = [tr.train_step(batches[s % STEPS], s) for s in range(5)]
            finally:
                ddp.GradBuckets._reduce = orig
            torch.cuda.synchronize()
            w = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
            out[tag] = {"losses": losses, "w": w.numpy(),
                        "graphs": len(tr._graphs.graphs) if tr._graphs is not None else -1, "dp": tr.dp,
                        "buckets": 0 if tr._buckets is None else len(tr._buckets.buckets),
                        "backend": dist.get_backend(), "calls": list(calls)}
        dist.destroy_process_group()
        q.put((0, "ok", out))
    except Exception:
        import traceback
        q.put((0, "error", traceback.format_exc()))


def test_rccl_dp_step_captured_bitwise_equal_to_eager(dev):
    """The DP step as one captured graph over RCCL (trainer/step_graph.py): bitwise equal to the eager DP step,
    which at one rank (AVG = identity) is bitwise equal to the step without DP.  RCCL with more than one rank
    needs one GPU per rank (the driver's 8-GPU node); this runs the same code path -- collectives recorded on
    the comm stream inside the capture, guard with the first bucket, finish() joined before AdamW."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_graph_worker, args=(_free_port(), q))
    p.start()
    try:
        r = q.get(timeout=300)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert r[1] == "ok", r[2]
    res = r[2]
    print("\n", {k: (v["losses"][-1], v["graphs"], v["dp"], v["buckets"], v["backend"]) for k, v in res.items()})
    assert res["graph_dp"]["backend"] == "nccl"
    assert res["eager_dp"]["dp"] and res["graph_dp"]["dp"] and not res["graph"]["dp"]
    assert res["graph_dp"]["buckets"] > 4, "bucketing did not engage"
    assert res["graph_dp"]["graphs"] == STEPS and res["eager_dp"]["graphs"] == 0
    assert res["eager_dp"]["losses"] == res["graph_dp"]["losses"] == res["graph"]["losses"]
    assert np.array_equal(res["eager_dp"]["w"], res["graph_dp"]["w"])
    assert np.array_equal(res["graph"]["w"], res["graph_dp"]["w"])
    # a failed first capture of the DP step: eager from then on, bitwise the eager DP run
    assert res["graph_dp_fail"]["graphs"] == -1
    nb = res["graph_dp_fail"]["buckets"]
    calls = res["graph_dp_fail"]["calls"]
    assert sorted(calls) == sorted(list(range(nb)) * 5), "eager DP steps after the failed capture mis-fired buckets"
    assert res["graph_dp_fail"]["losses"] == res["eager_dp"]["losses"]
    assert np.array_equal(res["graph_dp_fail"]["w"], res["eager_dp"]["w"])
