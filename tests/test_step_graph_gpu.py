"""The captured training step (trainer/step_graph.py) against the eager step: same kernels, same order, same
buffers, so losses, parameters and AdamW moments must be BITWISE equal after several steps -- for the tiny
configs in fp32 / bf16, for the benchmark's own 96^3 DualEncoder bf16 step, through the copy-graph fallback
(more distinct input addresses than pointer-keyed graphs), and with a bad-label batch (the guard inside the
graph skips the update, the trainer raises, the weights stay put)."""
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.trainer import Trainer

pytestmark = pytest.mark.gpu


def _cfg(model, C, feats, dtype, lr=1e-3, mods=("CT", "PET")):
    return {
        "experiment": {"name": "graph", "output_dir": "/tmp/mmseg_graph", "seed": 0},
        "data": {"modalities": list(mods)},
        "model": {"name": model, "in_channels": len(mods), "out_channels": C,
                  "backbone": {"features": list(feats), "norm": "instance"},
                  "fusion": {"type": "cross_attention"}, "head": {"dropout": 0.0}},
        "training": {"epochs": 1, "batch_size": 2, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": lr, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": "dice_ce", "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None},
                     "checkpoint": {"save_last": False, "save_best": False}},
        "hardware": {"device": "cuda", "mixed_precision": dtype == "bfloat16", "engine_dtype": dtype},
    }


def _batches(dev, n, S, M, C, seed=3):
    g = torch.Generator().manual_seed(seed)
    return [{"image": torch.randn(2, M, S, S, S, generator=g).to(dev),
             "label": torch.randint(0, C, (2, S, S, S), generator=g).to(dev)} for _ in range(n)]


def _run(cfg, batches, steps, graph, monkeypatch, sync=True, sched_every=0):
    monkeypatch.setenv("MMSEG_STEP_GRAPH", "1" if graph else "0")
    torch.manual_seed(0)
    m = build_model(cfg)
    tr = Trainer(cfg, m)
    losses = []
    for i in range(steps):
        lv = tr.train_step(batches[i % len(batches)], i, sync=sync)
        losses.append(lv if sync else lv.item())
        if sched_every and (i + 1) % sched_every == 0:
            tr.scheduler.step()
    torch.cuda.synchronize()
    params = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
    mv = [t.clone() for t in tr.optimizer._flat[0]]
    return tr, losses, params, mv


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("model", ["unet", "dual_encoder"])
def test_step_graph_bitwise_equal_to_eager(dev, model, dtype, monkeypatch):
    cfg = _cfg(model, 3, [8, 16, 32, 64, 128], dtype)
    batches = _batches(dev, 3, 32, 2, 3)
    _, l0, p0, mv0 = _run(cfg, batches, 6, False, monkeypatch)
    tr, l1, p1, mv1 = _run(cfg, batches, 6, True, monkeypatch)
    assert len(tr._graphs.graphs) == 3, "graph replay did not engage"
    assert l0 == l1
    assert torch.equal(p0, p1)
    assert all(torch.equal(a, b) for a, b in zip(mv0, mv1))
    assert int(tr.optimizer.state[next(tr.model.parameters())]["step"]) == 6


def test_step_graph_with_cosine_scheduler(dev, monkeypatch):
    """The shipped configs use a cosine LR scheduler, which wraps optimizer.step (torch lr_scheduler.py
    patch_track_step_called): the captured step must still engage, follow the scheduler's lr (a device
    hyper-parameter refreshed before each replay) and stay bitwise equal to the eager step."""
    cfg = _cfg("unet", 3, [8, 16, 32, 64, 128], "float32")
    cfg["training"]["epochs"] = 4
    cfg["training"]["scheduler"] = {"name": "cosine", "warmup_epochs": 0, "min_lr": 1e-6}
    batches = _batches(dev, 2, 32, 2, 3, seed=5)
    import warnings
    with warnings.catch_warnings():
        warnings.filterwarnings("error", message=".*lr_scheduler.step.*before.*optimizer.step")
        _, l0, p0, mv0 = _run(cfg, batches, 6, False, monkeypatch, sched_every=2)
        tr, l1, p1, mv1 = _run(cfg, batches, 6, True, monkeypatch, sched_every=2)
    assert getattr(tr.optimizer.step, "_wrapped_by_lr_sched", False)
    assert len(tr._graphs.graphs) == 2, "graph replay did not engage under the cosine scheduler"
    assert tr.optimizer.param_groups[0]["lr"] < 1e-3
    assert l0 == l1
    assert torch.equal(p0, p1)
    assert all(torch.equal(a, b) for a, b in zip(mv0, mv1))


def test_step_graph_bench_workload_bitwise(dev, monkeypatch):
    """bench.py's workload: DualEncoder mean fusion, CT+PET 96^3, B=2, 6 classes, bf16, lr 1e-4, sync=False."""
    cfg = _cfg("dual_encoder", 6, [32, 64, 128, 256, 512], "bfloat16", lr=1e-4)
    from mmseg_amd.data import device_batches
    batches = device_batches(2, 2, 96, 6, ["CT", "PET"], dev, seed=1234)
    _, l0, p0, mv0 = _run(cfg, batches, 4, False, monkeypatch, sync=False)
    tr, l1, p1, mv1 = _run(cfg, batches, 4, True, monkeypatch, sync=False)
    assert len(tr._graphs.graphs) == 2
    assert l0 == l1
    assert torch.equal(p0, p1)
    assert all(torch.equal(a, b) for a, b in zip(mv0, mv1))


def test_step_graph_copy_fallback(dev, monkeypatch):
    from mmseg_amd.trainer.step_graph import StepGraphs
    monkeypatch.setattr(StepGraphs, "MAX_GRAPHS", 1)
    cfg = _cfg("unet", 3, [8, 16, 32, 64, 128], "float32")
    batches = _batches(dev, 3, 32, 2, 3, seed=9)
    _, l0, p0, _ = _run(cfg, batches, 7, False, monkeypatch)
    tr, l1, p1, _ = _run(cfg, batches, 7, True, monkeypatch)
    assert len(tr._graphs.graphs) == 1 and tr._graphs.copy_graph is not None
    assert l0 == l1 and torch.equal(p0, p1)


def test_step_graph_bad_labels(dev, monkeypatch):
    cfg = _cfg("unet", 3, [8, 16, 32, 64, 128], "float32")
    batches = _batches(dev, 2, 32, 2, 3, seed=4)
    monkeypatch.setenv("MMSEG_STEP_GRAPH", "1")
    torch.manual_seed(0)
    m = build_model(cfg)
    tr = Trainer(cfg, m)
    tr.train_step(batches[0], 0)
    tr.train_step(batches[1], 1)
    assert len(tr._graphs.graphs) == 1
    before = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
    bad = {"image": batches[0]["image"], "label": batches[0]["label"].clone()}
    bad["label"][1, 3, 3, 3] = 7
    with pytest.raises(RuntimeError, match="outside"):
        tr.train_step(bad, 2)
    assert len(tr._graphs.graphs) == 2
    assert torch.equal(before, torch.cat([p.detach().reshape(-1) for p in m.parameters()]))
    assert int(tr.optimizer.state[next(m.parameters())]["step"]) == 2


@pytest.mark.parametrize("graph", [True, False])
def test_deferred_bad_labels_raise_at_next_sync(dev, monkeypatch, graph):
    """sync=False (no host read per step): a bad-label step skips its update on the device, returns a NaN loss,
    and the trainer raises at its next synchronisation point with the step count rolled back."""
    cfg = _cfg("unet", 3, [8, 16, 32, 64, 128], "float32")
    batches = _batches(dev, 2, 32, 2, 3, seed=4)
    monkeypatch.setenv("MMSEG_STEP_GRAPH", "1" if graph else "0")
    torch.manual_seed(0)
    m = build_model(cfg)
    tr = Trainer(cfg, m)
    tr.train_step(batches[0], 0)
    tr.train_step(batches[1], 1, sync=False)
    torch.cuda.synchronize()
    before = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
    bad = {"image": batches[0]["image"], "label": batches[0]["label"].clone()}
    bad["label"][0, 1, 2, 3] = 9
    lv = tr.train_step(bad, 2, sync=False)
    assert torch.isnan(lv).item()
    assert torch.equal(before, torch.cat([p.detach().reshape(-1) for p in m.parameters()]))
    with pytest.raises(RuntimeError, match="outside"):
        tr.check_deferred()
    assert int(tr.optimizer.state[next(m.parameters())]["step"]) == 2
    tr.check_deferred()                 # cleared: no second raise


@pytest.mark.parametrize("graph", [True, False])
def test_deferred_bad_then_sync_bad(dev, monkeypatch, graph):
    """A bad sync=False step followed by a bad sync=True step: one raise reports both, and BOTH step counts are
    rolled back (the current step's guard is handled before the deferred raise)."""
    cfg = _cfg("unet", 3, [8, 16, 32, 64, 128], "float32")
    batches = _batches(dev, 2, 32, 2, 3, seed=4)
    monkeypatch.setenv("MMSEG_STEP_GRAPH", "1" if graph else "0")
    torch.manual_seed(0)
    m = build_model(cfg)
    tr = Trainer(cfg, m)
    tr.train_step(batches[0], 0)
    tr.train_step(batches[1], 1)
    before = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
    bad = {"image": batches[0]["image"], "label": batches[0]["label"].clone()}
    bad["label"][0, 1, 2, 3] = 9
    assert torch.isnan(tr.train_step(bad, 2, sync=False)).item()
    with pytest.raises(RuntimeError, match="outside.*earlier training step"):
        tr.train_step(bad, 3)
    assert torch.equal(before, torch.cat([p.detach().reshape(-1) for p in m.parameters()]))
    assert int(tr.optimizer.state[next(m.parameters())]["step"]) == 2
    tr.check_deferred()                 # nothing left to raise
    tr.train_step(batches[1], 4)        # and training continues
    assert int(tr.optimizer.state[next(m.parameters())]["step"]) == 3
