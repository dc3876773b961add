"""Data parallelism over RCCL (torch.distributed backend "nccl" == RCCL on
ROCm), one process per GPU.  The reference is single-process;
this is new work whose oracle is "N ranks x B == 1 rank x N*B".

  * sharding: rank r takes samples r, r+W, ... of the index list padded by
    wrap-around to a multiple of W (DistributedSampler semantics), so every
    rank runs the same number of batches — see `shard_indices`;
  * gradients live in the engine's flat arena; `GradBuckets` splits it into
    ~bucket_mb buckets (reverse registration order = backward order) and
    all-reduces each bucket with ReduceOp.AVG as soon as the engine has
    written every gradient in it, so RCCL traffic over xGMI overlaps the rest
    of the backward; `finish()` joins them before the optimizer step;
  * validation counts (Dice I/U) are summed with one all_reduce;
  * over RCCL the whole step, collectives included, is captured as one HIP graph (trainer/step_graph.py):
    the bucket all-reduces are recorded at the points of the backward where their gradients become final,
    on the comm stream forked from the capture stream, and joined before the AdamW kernel.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def backend() -> Optional[str]:
    return dist.get_backend() if initialized() else None


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def init_from_env(backend: Optional[str] = None) -> int:
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*); returns local rank."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not dist.is_initialized():
        if backend is None:   # MMSEG_DIST_BACKEND=gloo rehearses N ranks on one GPU (RCCL needs one GPU per rank)
            backend = os.environ.get("MMSEG_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return local


def shard_indices(n_samples: int, r: int, w: int, pad: bool = True) -> List[int]:
    """torch DistributedSampler(shuffle=False) order: pad the index list by wrapping around to
    ceil(n/W)*W, then rank r takes r, r+W, ...  Every rank gets the same count, so no rank runs
    an extra train_step (which would wait forever in a gradient all-reduce).  pad=False (validation):
    plain r::W slicing, so every sample is scored exactly once (the validation all-reduce sums each
    rank's real batch count, so unequal shards are fine there)."""
    if n_samples <= 0:
        return []
    if not pad:
        return list(range(r, n_samples, w))
    total = -(-n_samples // w) * w
    idx = list(range(n_samples))
    while len(idx) < total:
        idx += idx[:total - len(idx)]
    return idx[r:total:w]


class GradBuckets:
    """Bucketed, backward-overlapped gradient averaging over a flat arena."""

    def __init__(self, grad_flat: torch.Tensor, param_offsets: List[int], param_sizes: List[int],
                 bucket_mb: float = 32.0, group=None, force: bool = False):
        self.grad = grad_flat
        self.group = group
        self.w = world()
        # force: issue the collectives at world size 1 too (distributed.reduce_single_rank) -- the one-GPU box
        # runs the real RCCL + AVG (+ graph capture) path that way; at one rank AVG is the identity
        self.active = self.w > 1 or force
        nbytes = int(bucket_mb * 1024 * 1024)
        # buckets over parameter index ranges, from the END of the arena (backward order)
        self.buckets = []          # (lo_param, hi_param, lo_elem, hi_elem)
        hi = len(param_offsets)
        while hi > 0:
            lo = hi - 1
            size = param_sizes[lo]
            while lo > 0 and (size + param_sizes[lo - 1]) * 4 <= nbytes:
                lo -= 1
                size += param_sizes[lo]
            self.buckets.append((lo, hi, param_offsets[lo], param_offsets[hi - 1] + param_sizes[hi - 1]))
            hi = lo
        self.comm = None
        # called on the compute stream right before a bucket's collective is issued: the engine's batched
        # weight-gradient reduces (Runtime.flush_wred) still queued then write that bucket's gradients first
        self.pre_reduce = None
        self.owner = [0] * len(param_offsets)
        for b, (lo, hi, _, _) in enumerate(self.buckets):
            for i in range(lo, hi):
                self.owner[i] = b
        self.reset()

    def reset(self):
        self.pending = [hi - lo for (lo, hi, _, _) in self.buckets]
        self.works = []
        self.events = [dict() for _ in self.buckets]   # bucket -> {stream handle: event after its last write}
        # guard: one device float written by the step's loss forward (its count of out-of-range labels).  It is
        # summed over the ranks together with the first bucket, so the optimizer kernel of EVERY rank sees a
        # non-zero count and skips the update when any rank had a bad batch (the ranks stay identical)
        self.guard: Optional[torch.Tensor] = None
        self.guard_sent = False

    def _record(self, b: int):
        """Replace the bucket's writer streams by events recorded on them now (after their last write)."""
        for key, st in list(self.events[b].items()):
            if isinstance(st, torch.cuda.Stream):
                ev = torch.cuda.Event()
                ev.record(st)
                self.events[b][key] = ev

    def _reduce(self, b: int):
        _, _, lo, hi = self.buckets[b]
        t = self.grad[lo:hi]
        if self.grad.is_cuda:
            # The engine may write a bucket's gradients from several HIP streams (one per modality encoder):
            # the collective is issued from a dedicated stream that first waits for every contributing
            # stream's last write, so no compute stream is blocked and no write is missed.  The same path
            # runs for RCCL and for gloo over device tensors (ranks sharing one GPU in the tests).
            if self.comm is None:
                self.comm = torch.cuda.Stream(self.grad.device)
            for ev in self.events[b].values():
                self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm):
                if dist.get_backend(self.group) == "nccl":
                    # AVG over ranks; at world size 1 (reduce_single_rank: the one-GPU rehearsal) AVG is the
                    # identity and SUM is the same collective without RCCL's single-rank scaling pass
                    op = dist.ReduceOp.AVG if self.w > 1 else dist.ReduceOp.SUM
                else:                       # gloo has no AVG: pre-scale on the comm stream, then SUM
                    t.div_(self.w)
                    op = dist.ReduceOp.SUM
                self.works.append(dist.all_reduce(t, op=op, group=self.group, async_op=True))
                self._send_guard()
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t.div_(self.w)
            self._send_guard()

    def _send_guard(self):
        """All-reduce (SUM) the guard count on the comm stream, once per step; the loss forward that wrote it
        precedes every gradient write, so the bucket events already order it."""
        if self.guard is None or self.guard_sent:
            return
        self.guard_sent = True
        if self.guard.is_cuda:
            self.works.append(dist.all_reduce(self.guard, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        else:
            dist.all_reduce(self.guard, op=dist.ReduceOp.SUM, group=self.group)

    def param_ready(self, idx: int):
        if not self.active:
            return
        b = self.owner[idx]
        self.pending[b] -= 1
        if self.grad.is_cuda:
            # the streams that wrote this bucket; their events are recorded once the bucket is complete (one event
            # per stream and bucket, not one per parameter: inside a captured step each is a graph dependency)
            cur = torch.cuda.current_stream(self.grad.device)
            self.events[b].setdefault(cur.cuda_stream, cur)
        if self.pending[b] == 0:
            if self.pre_reduce is not None:
                self.pre_reduce()
            self._record(b)
            self._reduce(b)

    def finish(self):
        if not self.active:
            return
        late = [b for b, n in enumerate(self.pending) if n > 0]
        if late and self.pre_reduce is not None:
            self.pre_reduce()
        if late and self.grad.is_cuda:
            # writes to unreported parameters may still be queued on the current stream: the late
            # collectives wait for everything issued on it so far
            cur = torch.cuda.current_stream(self.grad.device)
            for b in late:
                self.events[b][cur.cuda_stream] = cur
                self._record(b)
        for b in late:         # a parameter the engine did not report: reduce anyway (correctness first)
            self.pending[b] = 0
            self._reduce(b)
        if self.guard is not None and not self.guard_sent:
            if self.grad.is_cuda:
                with torch.cuda.stream(self.comm):
                    self._send_guard()
            else:
                self._send_guard()
        for wk in self.works:
            wk.wait()      # makes the current (optimizer) stream wait for the collective
        self.reset()


def allreduce_sum_(t: torch.Tensor) -> torch.Tensor:
    if world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t
