"""Optional per-kernel-family timer.

Disabled by default (zero cost).  bench.py enables it for a separate timed window to report the dominant
kernel's average launch duration next to its algorithmic FLOPs / bytes (the `roofline` object).

Durations come from the library's launch timing (mmseg_timing_*, csrc/api.cpp): while the timer runs, every
kernel of libmmseg_hip.so is launched with hipExtLaunchKernelGGL start / stop events, which the HIP runtime
stamps from the dispatch itself -- the kernel's own begin / end, the same interval rocprofv3's kernel trace
reports.  Event-record packets around a launch (the round-3 timer) also counted the barrier / dispatch latency
between them and any helper kernel of the same entry point (a split-K reduce), which inflated short kernels
(12^3 conv: 28.7 us against rocprofv3's 20.5).

A region names the entry point's main kernel (mmseg_last_kernel(), the rocprofv3 family name) and carries its
algorithmic FLOPs / bytes; the launches inside it are attributed launch by launch: the one whose launch-site
kernel matches the region's name gets the region's family and work, every other one (split-K reduces, packing)
its own launch-site name and no work."""
from __future__ import annotations

import ctypes
import re
from collections import defaultdict
from contextlib import contextmanager

import torch


def _base(name: str) -> str:
    """Kernel identifier of a family / launch-site name: '(wgrad_dma_kernel<4, true>)' -> 'wgrad_dma_kernel'."""
    m = re.search(r"[A-Za-z_][A-Za-z0-9_]*", name)
    return m.group(0) if m else name


class KernelTimer:
    def __init__(self):
        self.enabled = False
        self.regions = []   # (name, flops, bytes, first launch, end launch)

    def _lib(self):
        from .._lib import lib
        return lib()

    def start(self):
        self.regions = []
        self._lib().mmseg_timing_begin()
        self.enabled = True

    def stop(self):
        self.enabled = False
        self._lib().mmseg_timing_end()

    @contextmanager
    def region(self, name, flops: float = 0.0, nbytes: float = 0.0, more=()):
        """`name` may be a callable evaluated after the launch (e.g. the kernel the library chose).  `more`:
        further (name, flops, bytes) of other main kernels of the same entry point (an entry that launches two
        MFMA kernels, e.g. the window-attention backward), each matched to its own launch."""
        if not self.enabled:
            yield
            return
        L = self._lib()
        i0 = L.mmseg_timing_count()
        yield
        i1 = L.mmseg_timing_count()
        self.regions.append((name() if callable(name) else name, flops, nbytes, i0, i1))
        for nm, fl, nb in more:
            self.regions.append((nm, fl, nb, i0, i1))

    def launches(self):
        """[(launch-site kernel expression, ms)] of every library launch in the window."""
        torch.cuda.synchronize()
        L = self._lib()
        out = []
        ms = ctypes.c_float()
        nm = ctypes.c_char_p()
        for i in range(L.mmseg_timing_count()):
            L.mmseg_timing_get(i, ctypes.addressof(ms), ctypes.addressof(nm))
            out.append((nm.value.decode(), float(ms.value)))
        return out

    def records(self):
        """Per launch, in issue order: (family, launch-site kernel, ms, flops, bytes)."""
        launches = self.launches()
        owner = {}
        mains = set()
        for name, fl, nb, i0, i1 in self.regions:
            if i1 <= i0:
                continue
            want = _base(name)
            free = [i for i in range(i0, i1) if i not in mains] or list(range(i0, i1))
            main = next((i for i in free if _base(launches[i][0]) == want),
                        max(free, key=lambda i: launches[i][1]))
            mains.add(main)
            for i in range(i0, i1):
                if i == main:
                    owner[i] = (name, fl, nb)
                elif i not in mains:
                    owner[i] = (_base(launches[i][0]), 0.0, 0.0)
        out = []
        for i, (site, ms) in enumerate(launches):
            name, fl, nb = owner.get(i, (_base(site), 0.0, 0.0))
            out.append((name, site, ms, fl, nb))
        return out

    def summary(self):
        agg = defaultdict(lambda: {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
        for name, _, ms, fl, nb in self.records():
            a = agg[name]
            a["launches"] += 1
            a["ms"] += ms
            a["flops"] += fl
            a["bytes"] += nb
        return dict(agg)


TIMER = KernelTimer()
