"""Per-family totals of a bench.py --timer-dump file (launches [family, site, ms, flops, bytes]).
usage: python tools/timer_families.py TIMER.json [TOP]"""
import collections
import json
import sys

d = json.load(open(sys.argv[1]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
steps = max(1, int(d.get("timer_steps", 1)))
agg = collections.defaultdict(lambda: [0, 0.0])
for fam, _site, ms, *_ in d["launches"]:
    agg[fam][0] += 1
    agg[fam][1] += ms
tot = sum(v[1] for v in agg.values())
print(f"{len(d['launches']) / steps:.0f} launches / step, {tot / steps:.3f} ms of kernels / step")
for k, (n, ms) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{k:48s} {n / steps:6.1f} {ms / steps:8.3f} {1e3 * ms / n:8.1f} us")
