"""Print rocprofv3 kernel stats (calls, average us) filtered by name substrings.

    python tools/kstats.py <rocprofv3 output dir> [substring ...]
"""
import csv
import glob
import sys

for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if len(sys.argv) > 2 and not any(k in r["Name"] for k in sys.argv[2:]):
            continue
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg={float(r['AverageNs']) / 1e3:8.2f} us")
