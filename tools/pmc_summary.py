"""Average rocprofv3 --pmc counters per kernel: python tools/pmc_summary.py DIR [name-filter ...]"""
import collections
import csv
import glob
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if len(sys.argv) > 2 and not any(k in r["Kernel_Name"] for k in sys.argv[2:]):
            continue
        d[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in d.items():
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
