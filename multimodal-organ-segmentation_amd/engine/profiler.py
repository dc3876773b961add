"""Optional per-kernel-family timer (HIP events on the launching stream).

Disabled by default (zero cost).  bench.py enables it for a separate timed
window to report the dominant kernel's average launch duration next to its
algorithmic FLOPs / bytes (the `roofline` object)."""
from __future__ import annotations

from collections import defaultdict
from contextlib import contextmanager

import torch


class KernelTimer:
    def __init__(self):
        self.enabled = False
        self.records = []   # (name, flops, bytes, start_event, end_event)

    def start(self):
        self.records = []
        self.enabled = True

    def stop(self):
        self.enabled = False

    @contextmanager
    def region(self, name, flops: float = 0.0, nbytes: float = 0.0):
        """`name` may be a callable evaluated after the launch (e.g. the kernel the library chose)."""
        if not self.enabled:
            yield
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        self.records.append((name() if callable(name) else name, flops, nbytes, s, e))

    def summary(self):
        torch.cuda.synchronize()
        agg = defaultdict(lambda: {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
        for name, fl, nb, s, e in self.records:
            a = agg[name]
            a["launches"] += 1
            a["ms"] += s.elapsed_time(e)
            a["flops"] += fl
            a["bytes"] += nb
        return dict(agg)


TIMER = KernelTimer()
