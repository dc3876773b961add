"""Average duration of each run of identical consecutive kernels in a rocprofv3 kernel trace (launch order).

    python tools/trace_runs.py k_kernel_trace.csv [bytes-per-launch hints ignored]
Prints one line per run: kernel (shortened), grid, launches, average us.
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::|void |_ZN12_GLOBAL__N_1\d+", "", n)
    return n[:58]


for f in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    runs = []
    for r in rows:
        key = (r["Kernel_Name"], r.get("Grid_Size_X", r.get("Grid_Size")))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if runs and runs[-1][0] == key:
            runs[-1][1].append(d)
        else:
            runs.append((key, [d]))
    print(f"== {f}")
    for (name, grid), ds in runs:
        ds2 = ds[1:] if len(ds) > 2 else ds
        print(f"  {short(name):58s} grid {grid:>9} x{len(ds):3d} avg {sum(ds2) / len(ds2):8.2f} us")
