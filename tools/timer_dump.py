"""Summarise a bench.py --timer-dump file: per family (ms/step, launches/step, TF/s) and the N longest launch
sites in step order.

    python tools/timer_dump.py gpurun_out/<TAG>/timer.json [N]
"""
import json
import sys
from collections import defaultdict


def main():
    d = json.load(open(sys.argv[1]))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    steps = max(1, d["timer_steps"])
    rec = d["launches"]
    fam = defaultdict(lambda: [0, 0.0, 0.0])
    for name, site, ms, fl, nb in rec:
        a = fam[name]
        a[0] += 1
        a[1] += ms
        a[2] += fl
    tot = sum(a[1] for a in fam.values())
    print(f"{len(rec) // steps} launches / step, {tot / steps:.3f} ms of kernels / step")
    print(f"{'family':44s} {'n/step':>7s} {'ms/step':>8s} {'avg_us':>8s} {'TF/s':>7s} {'%':>6s}")
    for k, (n, ms, fl) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 and fl > 0 else 0.0
        print(f"{k[:44]:44s} {n / steps:7.1f} {ms / steps:8.3f} {1e3 * ms / n:8.1f} {tf:7.0f} {100 * ms / tot:6.2f}")
    per = len(rec) // steps
    step0 = rec[:per]
    print(f"\nlongest {top} launches of the first timed step (index: family, site, us, TF/s)")
    for i, (name, site, ms, fl, nb) in sorted(enumerate(step0), key=lambda t: -t[1][2])[:top]:
        tf = fl / (ms * 1e-3) / 1e12 if fl > 0 else 0.0
        print(f"{i:4d} {name[:40]:40s} {site[:50]:50s} {1e3 * ms:8.1f} {tf:6.0f}")


if __name__ == "__main__":
    main()
