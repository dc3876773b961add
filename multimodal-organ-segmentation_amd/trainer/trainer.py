"""Trainer — mirror of the reference's src/trainer/trainer.py (Trainer 21-433)
with the per-batch body factored into `train_step(batch, batch_idx)`
(the reference inlines it at trainer.py:231-261).

Same constructor, config keys, history / checkpoint format and epoch loop.
MI355X-specific behaviour:
  * mixed precision = the engine's bf16 activation storage with fp32
    parameters / gradients / optimizer state, so no GradScaler is needed
    (bf16 has fp32's exponent range); the reference's fp16 autocast +
    GradScaler (trainer.py:237-248) therefore maps to a no-op scaler;
  * AdamW runs as one HIP kernel over the flat parameter arena (FlatAdamW);
  * data parallelism (one process per GPU, torchrun env) averages gradients
    with bucketed RCCL all-reduces overlapped with the backward; only the
    accumulation boundary micro-step communicates; rank 0 logs/checkpoints;
  * validation accumulates Dice counts on the device (fused argmax + counts),
    one host sync per validation pass instead of one per batch.

`hardware.kernels: torch` (models/build.py) is the A/B backend: the model's
and the losses' own PyTorch-ROCm forwards, torch.optim.AdamW, and the
reference's step body verbatim in behaviour (trainer.py:236-258: autocast fp16
+ GradScaler when mixed_precision, or bf16 autocast without a scaler when
hardware.engine_dtype is bfloat16).  Never a fallback: selected explicitly.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Dict, Optional, Tuple, Union

import torch
import torch.nn as nn

from ..distributed import ddp
from ..models.build import kernels_from_config, load_checkpoint, save_checkpoint
from .losses import get_loss
from .metrics import DiceMetric, get_metrics
from .optim import FlatAdamW, pack_source

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    def tqdm(it, **kw):
        return it


class Trainer:
    def __init__(self, config: Dict[str, Any], model: nn.Module, train_loader=None, val_loader=None,
                 logger: Optional[Any] = None, resume_from: Optional[str] = None):
        self.config = config
        self.model = model
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.logger = logger
        self.epochs = config["training"]["epochs"]
        self.device = self._get_device()
        self.model = self.model.to(self.device)
        self.kernels = kernels_from_config(config)
        self.optimizer = self._setup_optimizer()
        if isinstance(self.optimizer, FlatAdamW):
            # its launch also refreshes the engine's weight images (mmseg_adamw_pack): no pack in the next forward
            self.optimizer._pack_source = pack_source(self.model)
        self.scheduler = self._setup_scheduler()
        self.criterion = get_loss(config)
        self.metrics = get_metrics(config)
        self.use_amp = config["hardware"].get("mixed_precision", False)
        self.scaler = None  # bf16 engine: no loss scaling needed (see module docstring)
        self._amp_dtype = None
        if self.kernels == "torch" and self.use_amp:
            bf16 = str(config["hardware"].get("engine_dtype", "")).lower() in ("bfloat16", "bf16")
            self._amp_dtype = torch.bfloat16 if bf16 else torch.float16
            if not bf16:
                self.scaler = torch.amp.GradScaler("cuda")
        self.accumulation_steps = config["training"].get("accumulation_steps", 1)
        self.rank, self.world = ddp.rank(), ddp.world()
        # gradient all-reduce active: more than one rank, or distributed.reduce_single_rank with a process group
        # (the one-GPU rehearsal of the RCCL path, ddp.GradBuckets force)
        self.dp = self.world > 1 or (bool(config.get("distributed", {}).get("reduce_single_rank", False))
                                     and ddp.initialized())
        self.output_dir = Path(config["experiment"]["output_dir"]) / config["experiment"]["name"]
        if self.rank == 0:
            self.output_dir.mkdir(parents=True, exist_ok=True)
        self.current_epoch = 0
        self.best_metric = 0.0
        self.history = {"train_loss": [], "val_loss": [], "val_dice": []}
        self._buckets = None
        self._deferred_bad = None       # device count of sync=False steps whose labels were out of range
        self._one = torch.ones((), dtype=torch.float32, device=self.device)
        from .step_graph import StepGraphs
        self._graphs = StepGraphs(self)
        self._graph_ok = False
        # fused head + loss training step (engine.run_engine_loss): hardware.fused_head_loss (the
        # MMSEG_FUSED_HEAD_LOSS env var overrides it per step, for A/B runs)
        self.fused_head_loss = bool(config["hardware"].get("fused_head_loss", True))
        if resume_from:
            self._resume(resume_from)

    # ------------------------------------------------------------- setup
    def _get_device(self) -> torch.device:
        dev = self.config["hardware"]["device"]
        if dev == "cuda" and torch.cuda.is_available():
            return torch.device("cuda", torch.cuda.current_device())
        raise RuntimeError("the MI355X trainer needs hardware.device == 'cuda' on a ROCm GPU (no CPU path)")

    def _setup_optimizer(self) -> torch.optim.Optimizer:
        oc = self.config["training"]["optimizer"]
        name = oc["name"].lower()
        lr, wd = oc["lr"], oc.get("weight_decay", 0)
        params = list(self.model.parameters())
        if self.kernels == "torch":      # reference trainer.py:104-122
            if name == "adam":
                return torch.optim.Adam(params, lr=lr, weight_decay=wd)
            if name == "sgd":
                return torch.optim.SGD(params, lr=lr, momentum=oc.get("momentum", 0.9), weight_decay=wd)
            betas = tuple(oc.get("betas", [0.9, 0.999])) if name == "adamw" else (0.9, 0.999)
            return torch.optim.AdamW(params, lr=lr, weight_decay=wd, betas=betas)
        if name == "adamw":
            return FlatAdamW(params, lr=lr, weight_decay=wd, betas=tuple(oc.get("betas", [0.9, 0.999])))
        if name == "adam":
            return torch.optim.Adam(params, lr=lr, weight_decay=wd)
        if name == "sgd":
            return torch.optim.SGD(params, lr=lr, momentum=oc.get("momentum", 0.9), weight_decay=wd)
        return FlatAdamW(params, lr=lr, weight_decay=wd)

    def _setup_scheduler(self):
        sc = self.config["training"].get("scheduler", {})
        name = sc.get("name", "cosine").lower()
        if name == "cosine":
            warm = sc.get("warmup_epochs", 0)
            return torch.optim.lr_scheduler.CosineAnnealingLR(self.optimizer, T_max=self.epochs - warm,
                                                              eta_min=sc.get("min_lr", 1e-6))
        if name == "step":
            return torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=sc.get("step_size", 30),
                                                   gamma=sc.get("gamma", 0.1))
        if name == "plateau":
            return torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer, mode="max",
                                                              patience=sc.get("patience", 10),
                                                              factor=sc.get("factor", 0.1))
        return None

    def _resume(self, path: str) -> None:
        """reference trainer.py:150-164 (scheduler / history not restored, as in the reference)."""
        ckpt = load_checkpoint(self.model, path)
        if "optimizer_state_dict" in ckpt:
            self.optimizer.load_state_dict(ckpt["optimizer_state_dict"])
        if "epoch" in ckpt:
            self.current_epoch = ckpt["epoch"]
        if "best_metric" in ckpt:
            self.best_metric = ckpt["best_metric"]
        if self.logger:
            self.logger.info(f"Resumed from epoch {self.current_epoch}")

    # ----------------------------------------------------------- DP hooks
    def _engine_flat(self):
        bb = getattr(self.model, "backbone", self.model)
        eng = bb.__dict__.get("_engine")
        return eng.flat if eng is not None else None

    def _arm_buckets(self, communicate: bool, guard: Optional[torch.Tensor] = None):
        if not self.dp:
            return
        flat = self._engine_flat()
        if flat is None:
            return
        if self._buckets is None or self._buckets.grad is not flat.grad_flat:
            mb = float(self.config.get("distributed", {}).get("bucket_mb", 32))
            self._buckets = ddp.GradBuckets(flat.grad_flat, flat.offsets, flat.sizes, bucket_mb=mb, force=True)
        flat.on_ready = self._buckets.param_ready if communicate else None
        self._buckets.guard = guard if communicate else None
        # the batched weight-gradient reduces stay on under DP: the queue is flushed right before each bucket's
        # collective (one batched launch per bucket instead of one reduce launch per layer)
        bb = getattr(self.model, "backbone", self.model)
        rt = getattr(bb.__dict__.get("_engine"), "rt", None)
        batched = communicate and rt is not None and rt.batch_wred   # (per-layer reduces under DP: +0.05 ms, r05h)
        flat.flush_before_ready = rt.flush_wred if batched else None

        def pre_reduce():
            if rt._wred_active:       # inside the backward session: the queue may hold this bucket's reduces
                rt.flush_wred()
        self._buckets.pre_reduce = pre_reduce if batched else None

    def _fused_loss(self, images: torch.Tensor, labels: torch.Tensor) -> Optional[torch.Tensor]:
        """The step's loss through the fused head + loss node when the model / loss / shape allow it, else None.
        Same values as criterion(model(images), labels): the logits are recomputed in the backward with the
        forward's operation order, so no logits / dlogits tensors are written (five passes become two)."""
        env = os.environ.get("MMSEG_FUSED_HEAD_LOSS")
        if not ((env != "0") if env is not None else self.fused_head_loss):
            return None
        from ..engine.engine import fused_loss_supported, run_engine_loss
        from ..models.backbones.dual_encoder import DualEncoder
        from ..models.backbones.unet import UNet3D
        from .losses import _HipLoss
        crit = self.criterion
        if not isinstance(crit, _HipLoss) or getattr(crit, "reduction", "mean") != "mean":
            return None
        bb = getattr(self.model, "backbone", self.model)
        kind = "unet" if isinstance(bb, UNet3D) else "dual_encoder" if isinstance(bb, DualEncoder) else None
        if kind is None or not fused_loss_supported(bb, kind, images):
            return None
        N = images.shape[0]
        if labels.dtype not in (torch.int64, torch.uint8):
            labels = labels.long()
        labels = labels.contiguous()
        if labels.numel() != N * images[0, 0].numel():
            raise ValueError(f"target shape {tuple(labels.shape)} does not match images {tuple(images.shape)}")
        cw = getattr(crit, "class_weights", None)
        cw = None if cw is None else cw.to(images.device, torch.float32).contiguous()
        loss = run_engine_loss(bb, kind, images, labels, crit._spec(), cw)
        crit.__dict__["_last_ws"] = bb.__dict__["_engine"].loss_ws     # for check_labels()
        return loss

    # ----------------------------------------------------------- training
    def train_step(self, batch: Dict[str, torch.Tensor], batch_idx: int, sync: bool = True) -> Union[float, torch.Tensor]:
        """One per-batch body of the reference's _train_epoch (trainer.py:231-261):
        H2D, forward, loss / accumulation_steps, backward, optimizer step + zero_grad
        every accumulation_steps batches.  Returns the un-scaled loss (python float,
        or a device scalar with sync=False)."""
        images = batch["image"].to(self.device, non_blocking=True)
        labels = batch["label"].to(self.device, non_blocking=True)
        boundary = (batch_idx + 1) % self.accumulation_steps == 0
        if self.kernels == "torch":
            return self._torch_step(images, labels, boundary, sync)
        if self._graph_ok and self._graphs is not None and self._graphs.usable(images, labels):
            # the whole step (forward, fused loss, backward, AdamW) as one captured graph (trainer/step_graph.py)
            if labels.dtype not in (torch.int64, torch.uint8):
                labels = labels.long()
            try:
                out, guard = self._graphs.run(images.contiguous(), labels.contiguous())
            except RuntimeError as e:
                # the captured data-parallel step over several ranks has not run on hardware (step_graph.py): if its
                # first capture fails -- on every rank alike, they run the same code -- the step stays eager
                if not (self.dp and self._graphs.graphs == {} and self._graphs.copy_graph is None):
                    raise
                import warnings
                warnings.warn(f"captured data-parallel step failed to capture ({e}); the DP step runs eagerly",
                              RuntimeWarning, stacklevel=2)
                self._graphs, self._graph_ok = None, False
                if self._buckets is not None:
                    # a capture that failed mid-backward left decremented pending counts, stored works and
                    # events: the eager step must start from a clean bucket state (StepGraphs._capture resets
                    # too; this covers a failure raised outside it)
                    self._buckets.reset()
            else:
                if not sync:
                    self._defer_guard(guard)
                    return out.clone()
                return self._after_step(out.item(), guard, boundary=True, guarded=True)
        loss = self._fused_loss(images, labels)
        fused = loss is not None
        if loss is None:
            loss = self.criterion(self.model(images), labels)
        # the loss kernels count labels outside [0, C) on the device (the reference raises in F.one_hot before
        # any update): that count guards the optimizer kernel, which skips the update when it is non-zero, and
        # under DP it is summed over the ranks with the first gradient bucket so every rank skips together
        ws = self.criterion.__dict__.get("_last_ws")
        guard = ws[-1:] if ws is not None else None
        if self.accumulation_steps != 1:
            loss = loss / self.accumulation_steps
        self._arm_buckets(boundary, guard)
        loss.backward(self._one)         # a constant output gradient: no fill kernel per step
        guarded = boundary and isinstance(self.optimizer, FlatAdamW)
        if boundary:
            if self._buckets is not None and self.dp:
                self._buckets.finish()
            if guarded:
                self.optimizer.guard = guard
            self.optimizer.step()
            if guarded:
                self.optimizer.guard = None
            self.optimizer.zero_grad()
        # the first eager step planned every buffer and allocated the optimizer moments: later steps may replay
        self._graph_ok = fused and boundary and self._graphs is not None
        out = loss.detach()
        if self.accumulation_steps != 1:
            out = out * self.accumulation_steps
        if not sync:
            if guarded:
                self._defer_guard(guard)
            return out
        return self._after_step(out.item(), guard, boundary, guarded)

    def _defer_guard(self, guard: Optional[torch.Tensor]) -> None:
        """sync=False (bench.py's timed loop, anything that batches its host syncs): no host read per step.  The
        AdamW kernel has already skipped the update of a step whose labels were out of range (the guard); such
        steps are counted on the device and check_deferred() -- called by the next synchronous train_step and by
        _validate -- rolls their step counts back and raises, as the synchronous step would have at once.  Steps
        that ran between the bad one and the check used the advanced step count in their bias corrections."""
        if guard is None:
            return
        bad = guard.reshape(()).sign()
        self._deferred_bad = bad if self._deferred_bad is None else self._deferred_bad.add_(bad)

    def _take_deferred(self) -> int:
        """Count of earlier sync=False steps whose labels were out of range (their step counts rolled back,
        gradients cleared); resets the device counter."""
        if self._deferred_bad is None:
            return 0
        # under DP each step's guard was summed over the ranks by the first gradient bucket, so every rank
        # counts the same steps and raises together
        nbad, self._deferred_bad = int(self._deferred_bad.item()), None
        if nbad:
            for _ in range(nbad):
                self.optimizer.undo_step_count()
            self.optimizer.zero_grad()
        return nbad

    @staticmethod
    def _deferred_error(nbad: int) -> RuntimeError:
        return RuntimeError(f"{nbad} earlier training step(s) had target voxels with a class index outside "
                            "[0, num_classes) (the reference raises in F.one_hot / cross_entropy on such "
                            "labels); their updates were skipped")

    def check_deferred(self) -> None:
        nbad = self._take_deferred()
        if nbad:
            raise self._deferred_error(nbad)

    def _torch_step(self, images, labels, boundary: bool, sync: bool):
        """The reference's per-batch body (trainer.py:236-258) on the torch-op backend."""
        if self._amp_dtype is not None:
            with torch.autocast("cuda", dtype=self._amp_dtype):
                loss = self.criterion(self.model(images), labels) / self.accumulation_steps
        else:
            loss = self.criterion(self.model(images), labels) / self.accumulation_steps
        if self.scaler is not None:
            self.scaler.scale(loss).backward()
        else:
            loss.backward()
        if boundary:
            if self.world > 1:           # plain per-tensor averaging (the reference is single-process)
                for p in self.model.parameters():
                    if p.grad is not None:
                        ddp.allreduce_sum_(p.grad)
                        p.grad.div_(self.world)
            if self.scaler is not None:
                self.scaler.step(self.optimizer)
                self.scaler.update()
            else:
                self.optimizer.step()
            self.optimizer.zero_grad()
        out = loss.detach() * self.accumulation_steps
        return out.item() if sync else out

    def _after_step(self, lv: float, guard, boundary: bool, guarded: bool) -> float:
        """Host side of a synchronous step: raise (on every rank) when the step's labels were out of range.
        The current step's guard is handled first (its step count rolled back when the kernel skipped it), then
        the earlier deferred steps', so one raise reports both and neither's bookkeeping is skipped."""
        cur_bad = False
        if guard is not None and (lv != lv or self.world > 1):
            if self.world > 1 and (not boundary or self._buckets is None):
                ddp.allreduce_sum_(guard)      # no bucket carried it on this micro-step
            if guard.item():                 # every rank sees the summed count and raises together
                cur_bad = True
                if guarded:
                    self.optimizer.undo_step_count()    # the kernel skipped the update
                self.optimizer.zero_grad()
        nbad = self._take_deferred()
        if cur_bad:
            try:
                self.criterion.check_labels()
            except RuntimeError as e:
                if nbad:
                    raise RuntimeError(f"{e}; and {self._deferred_error(nbad)}") from None
                raise
        if nbad:
            raise self._deferred_error(nbad)
        return lv

    def _train_epoch(self) -> float:
        self.model.train()
        total = 0.0
        n = len(self.train_loader)
        self.optimizer.zero_grad()
        it = tqdm(self.train_loader, desc=f"Epoch {self.current_epoch + 1}") if self.rank == 0 else self.train_loader
        for batch_idx, batch in enumerate(it):
            lv = self.train_step(batch, batch_idx)
            total += lv
            if self.rank == 0 and hasattr(it, "set_postfix"):
                it.set_postfix({"loss": f"{lv:.4f}"})
        return total / n

    def _validate(self) -> Tuple[float, Dict[str, float]]:
        self.check_deferred()
        self.model.eval()
        dm = DiceMetric(num_classes=self.config["model"]["out_channels"], device=self.device)
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        n = 0
        with torch.no_grad():
            for batch in self.val_loader:
                images = batch["image"].to(self.device, non_blocking=True)
                labels = batch["label"].to(self.device, non_blocking=True)
                outputs = self.model(images)
                total += self.criterion(outputs, labels).double()
                dm.update_from_logits(outputs, labels)
                n += 1
        if self.world > 1:
            # one all-reduce of [loss sum, batch count, I, U]: the real per-rank batch counts are summed,
            # and a rank with no validation batches contributes zeros (its accumulators are on the device)
            nb = torch.tensor([float(n)], device=self.device)
            packed = torch.cat([total.view(1).float(), nb, dm.intersection, dm.union])
            ddp.allreduce_sum_(packed)
            C = dm.num_classes
            total = packed[0].double()
            n = int(round(packed[1].item()))
            dm.intersection, dm.union = packed[2:2 + C], packed[2 + C:]
        return (total / n).item() if n else float("nan"), dm.compute()

    def evaluate(self) -> Dict[str, float]:
        _, metrics = self._validate()
        return metrics

    def train(self) -> Dict[str, Any]:
        es = self.config["training"].get("early_stopping", {})
        patience = es.get("patience", 30)
        no_improve = 0
        for epoch in range(self.current_epoch, self.epochs):
            self.current_epoch = epoch
            train_loss = self._train_epoch()
            self.history["train_loss"].append(train_loss)
            val_loss, val_metrics = self._validate()
            self.history["val_loss"].append(val_loss)
            self.history["val_dice"].append(val_metrics.get("dice", 0))
            if self.logger and self.rank == 0:
                self.logger.info(f"Epoch [{epoch + 1}/{self.epochs}] Train Loss: {train_loss:.4f} "
                                 f"Val Loss: {val_loss:.4f} Val Dice: {val_metrics.get('dice', 0):.4f}")
            if self.scheduler is not None:
                if isinstance(self.scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
                    self.scheduler.step(val_metrics.get("dice", 0))
                else:
                    self.scheduler.step()
            self._save_checkpoints(val_metrics)
            if val_metrics.get("dice", 0) > self.best_metric:
                self.best_metric = val_metrics.get("dice", 0)
                no_improve = 0
            else:
                no_improve += 1
            if es.get("enabled", False) and no_improve >= patience:
                if self.logger and self.rank == 0:
                    self.logger.info(f"Early stopping at epoch {epoch + 1}")
                break
        return self.history

    def predict(self, input_path, output_path) -> None:  # pragma: no cover - NIfTI I/O is out of scope
        raise NotImplementedError("inference over NIfTI folders is outside the engine's scope (SURVEY §8f rank 2); "
                                  "volumes already in memory go through _sliding_window_inference")

    def _sliding_window_inference(self, image: torch.Tensor) -> torch.Tensor:
        """reference trainer.py:370-395: MONAI sliding_window_inference(image, roi_size, sw_batch_size=
        inference.batch_size, predictor=model, overlap) on device (inference/sliding_window.py).  The
        reference's ImportError fallback (one full-volume forward) is not taken: the device restatement
        always exists."""
        from ..inference import sliding_window_inference
        inf = self.config.get("inference", {})
        sw = inf.get("sliding_window", {})
        return sliding_window_inference(image.to(self.device), tuple(sw.get("roi_size", (96, 96, 96))),
                                        int(inf.get("batch_size", 4)), self.model, float(sw.get("overlap", 0.5)))

    def _save_checkpoints(self, metrics: Dict[str, float]) -> None:
        """reference trainer.py:397-433 (rank 0 only)."""
        if self.rank != 0:
            return
        cc = self.config["training"].get("checkpoint", {})
        if cc.get("save_last", True):
            save_checkpoint(self.model, self.optimizer, self.current_epoch, str(self.output_dir / "last.pth"),
                            best_metric=self.best_metric, history=self.history)
        if cc.get("save_best", True) and metrics.get("dice", 0) >= self.best_metric:
            save_checkpoint(self.model, self.optimizer, self.current_epoch, str(self.output_dir / "best.pth"),
                            best_metric=metrics.get("dice", 0), history=self.history)
        every = cc.get("save_every", 0)
        if every > 0 and (self.current_epoch + 1) % every == 0:
            save_checkpoint(self.model, self.optimizer, self.current_epoch,
                            str(self.output_dir / f"epoch_{self.current_epoch + 1}.pth"), best_metric=self.best_metric)
