"""Summarise rocprofv3 CSV output by the engine's kernel families.

    python tools/rocprof_families.py stats  <prof_kernel_stats.csv>  [steps]
    python tools/rocprof_families.py traffic <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json [steps]]
    python tools/rocprof_families.py sq <sq_counter_collection.csv> [out.json]
    python tools/rocprof_families.py steady <prof_kernel_trace.csv> <out.json> [last_steps]
    (any of them: --workload <file> written by `bench.py --workload-out`, stamped into the summary as
    "_workload" with "_created"; bench.py uses only the summaries of its own workload)

`stats` prints per-family calls / average duration (the same family names the
in-process timer reports through mmseg_last_kernel(), so bench.py's
`roofline.avg_launch_ms` can be checked against the trace).

`traffic` turns two separate PMC passes (FETCH_SIZE, WRITE_SIZE; one counter
group per pass) into HBM bytes per launch per family, with the gfx950
correction of MI355X_MICROARCH.md: FETCH_SIZE counts 128-B streaming requests
at 64 B, so it is doubled; WRITE_SIZE is taken as is.  Both counters are in KB.
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict

_MODES = {"0": "conv3", "1": "point", "2": "convT_fwd", "3": "convT_dgrad"}
_GEMM_TILES = {("4", "1", "2", "2"): "128x32", ("2", "2", "4", "2"): "128x64", ("1", "4", "4", "4"): "64x256",
               ("2", "2", "2", "2"): "64x64", ("1", "4", "4", "2"): "64x128", ("2", "2", "4", "3"): "128x96",
               ("1", "4", "4", "3"): "64x192", ("4", "1", "2", "3"): "128x48"}


def _mangled_base(name: str):
    """Function name of an Itanium-mangled kernel symbol (the traces are taken with rocprofv3 -M: its demangler
    garbles the __bf16 template arguments, DF16b): the last <length><identifier> of the nested name,
    _ZN12_GLOBAL__N_115conv_gemm_kernelI... -> conv_gemm_kernel."""
    if not name.startswith("_Z"):
        return None
    i = 3 if name.startswith("_ZN") else 2
    last = None
    while i < len(name) and name[i].isdigit():
        j = i
        while j < len(name) and name[j].isdigit():
            j += 1
        n = int(name[i:j])
        last, i = name[j:j + n], j + n
    return last


def family(name: str) -> str:
    """Map a (mangled or demangled) kernel name to the engine's family name."""
    dt = "bf16" if ("DF16b" in name or "__bf16" in name) else "f32"
    m = re.search(r"conv3_brick2_kernelI(?:DF16b|f)Li(\d+)ELi(\d+)E", name)
    if m:
        return f"conv3_brick2_kernel<BN{m.group(1)},ZW{m.group(2)}>[{dt}]"
    m = re.search(r"conv3_brickr_kernelI(?:DF16b|f)Li(\d+)E(?:Li\d+E){4}Lb[01]ELb[01]ELi(\d+)E", name)
    if m and m.group(2) != "1":   # the in-block K split (template KW), as mmseg_last_kernel() names it
        return f"conv3_brickr_kernel<BN{m.group(1)},KW{m.group(2)}>[{dt}]"
    m = re.search(r"conv3_brickr_kernelI(?:DF16b|f)Li(\d+)E", name)
    if m:
        return f"conv3_brickr_kernel<BN{m.group(1)}>[{dt}]"
    m = re.search(r"conv3_brick_kernelI(?:DF16b|f)Li(\d+)E", name)
    if m:
        return f"conv3_brick_kernel<BN{m.group(1)}>[{dt}]"
    m = re.search(r"conv_gemm_kernelI(?:DF16b|f)Li(\d)ELi(\d)ELi(\d)ELi(\d)ELi(\d)E", name)
    if m:
        # (WM, WN, TM, TN) template arguments -> the tile name mmseg_last_kernel() reports (conv_gemm.hip)
        tile = _GEMM_TILES.get(m.group(2, 3, 4, 5), "128x64")
        return f"conv_gemm_kernel<{_MODES[m.group(1)]},{tile}>[{dt}]"
    # brick6 / brick8 under the timer's family names (engine/profiler.py: mmseg_last_kernel()), so a family
    # means the same launches in the live timer and in the trace: brick6 split by its INP / F8 forms, brick8 by BN
    m = (re.search(r"conv3_brick6_kernelILb[01]ELi\d+ELi\d+ELb([01])ELb([01])E", name) or
         re.search(r"conv3_brick6_kernel<(?:true|false), \d+, \d+, (true|false), (true|false)>", name))
    if m:
        inp, f8 = (m.group(1) in ("1", "true")), (m.group(2) in ("1", "true"))
        return "conv3_brick6_kernel<BN32" + (",INP" if inp else "") + (",F8" if f8 else "") + ">[bf16]"   # bf16 only
    m = re.search(r"conv3_brick8_kernelILi(\d+)E", name) or re.search(r"conv3_brick8_kernel<(\d+),", name)
    if m:
        return f"conv3_brick8_kernel<BN{m.group(1)}>[bf16]"   # bf16 only
    if "conv3_brick4_kernel" in name:
        return "conv3_brick4_kernel<BN32>[bf16]"
    m = re.search(r"conv3_brick3_kernelI(?:DF16b|f)Li(\d+)E", name)
    if m:
        return f"conv3_brick3_kernel<BN{m.group(1)}>[{dt}]"
    m = re.search(r"wgrad_brick([2r])_kernelI(?:DF16b|f)Li(\d+)E(?:Li(\d)E)?", name)
    if m:
        # compile-time bricks of the runtime-brick kernel: 3x6x6 (12^3 / 6^3, "V3"), 4x4x8 (grouped 48^3 / 24^3)
        v3 = {"3": ",V3", "4": ",B448"}.get(m.group(3), "")
        return f"wgrad_brick{m.group(1)}_kernel<CO{int(m.group(2)) * 16}{v3}>[{dt}]"
    m = re.search(r"wgrad_row_kernelILb([01])E|wgrad_row_kernel<(true|false)", name)
    if m:   # (the deferred-norm and plain forms under the timer's names; bf16, 32 co only)
        return "wgrad_row_kernel<CO32" + (",NORM" if (m.group(1) or m.group(2)) in ("1", "true") else "") + ">[bf16]"
    m = re.search(r"wgrad_dma_kernelILi(\d+)E|wgrad_dma_kernel<(\d+)", name)
    if m:
        return f"wgrad_dma_kernel<CO{int(m.group(1) or m.group(2)) * 16}>"
    m = re.search(r"wgrad_reduce_kernelILi(\d+)E|wgrad_reduce_kernel<(\d+)>", name)
    if m:
        return f"wgrad_reduce_kernel<{m.group(1) or m.group(2)}>"
    if "wgrad_brick_kernel" in name:
        return f"wgrad_brick_kernel[{dt}]"
    m = re.search(r"(?<![a-z_])wgrad_kernelI(?:DF16b|f)Li(\d)E", name)
    if m:
        return f"wgrad_kernel<{_MODES[m.group(1)]}>[{dt}]"
    m = re.search(r"\(anonymous namespace\)::([A-Za-z_][A-Za-z0-9_]*)[<(]", name)
    if m:
        return m.group(1)
    base = _mangled_base(name)
    if base:
        return base
    m = re.search(r"(?:_GLOBAL__N_1\d+|::)([A-Za-z_][A-Za-z0-9_]*?)(?:I|\(|E|$)", name)
    return m.group(1) if m else name


def stats(path: str, steps: int = 1):
    agg = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            a = agg[family(r["Name"])]
            a[0] += int(r["Calls"])
            a[1] += float(r["TotalDurationNs"])
    tot = sum(v[1] for v in agg.values())
    print(f"{'family':48s} {'calls':>7s} {'avg_us':>9s} {'ms/step':>8s} {'%':>6s}")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:48s} {c:7d} {t / c / 1e3:9.1f} {t / steps / 1e6:8.3f} {100 * t / tot:6.2f}")


def steady(trace_csv: str, last: int = 8):
    """Per family over the LAST `last` training steps of a rocprofv3 kernel trace (a step ends with its AdamW
    launch): average duration per launch and launches per step.  The first steps of a bench run (warm-up, graph
    capture) run at ramping clocks -- wgrad_dma 47 us there against 42 us in steady state (r04d) -- and would
    bias prof_kernel_stats.csv's all-dispatch averages; bench.py's timer window runs after the timed steps."""
    with open(trace_csv) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    opt = ("adamw_pack_kernel", "adamw4_kernel", "adamw_kernel")
    ends = [i for i, r in enumerate(rows) if family(r["Kernel_Name"]) in opt]
    # one AdamW family per step (the fused AdamW + pack, else adamw4, else the scalar kernel): with several
    # present (large + small parameter groups, or an eager first step) keep the first of those that occurs
    for k in opt:
        if any(family(rows[i]["Kernel_Name"]) == k for i in ends):
            ends = [i for i in ends if family(rows[i]["Kernel_Name"]) == k]
            break
    if len(ends) < 2:
        raise SystemExit("steady: fewer than two AdamW launches in the trace")
    last = min(last, len(ends) - 1)
    lo, hi = ends[-last - 1], ends[-1]
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows[lo + 1:hi + 1]:
        a = agg[family(r["Kernel_Name"])]
        a[0] += 1
        a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6   # ms
    span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])) * 1e-6
    res = {"_steps": last, "_span_ms_per_step": span / last}
    for k, (n, ms) in agg.items():
        res[k] = {"launches_per_step": n / last, "avg_launch_ms": ms / n, "ms_per_step": ms / last}
    return res


def _counter_rows(path: str, counter: str):
    """{dispatch_id: (family, value_bytes)} summed over the counter's instances."""
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            fam = family(r["Kernel_Name"])
            v = float(r["Counter_Value"]) * 1024.0  # KB -> bytes
            if did in out:
                out[did] = (fam, out[did][1] + v)
            else:
                out[did] = (fam, v)
    return out


def traffic(fetch_csv: str, write_csv: str):
    fetch = _counter_rows(fetch_csv, "FETCH_SIZE")
    write = _counter_rows(write_csv, "WRITE_SIZE")
    fam_f, fam_w = defaultdict(list), defaultdict(list)
    for fam, v in fetch.values():
        fam_f[fam].append(2.0 * v)  # gfx950: FETCH_SIZE reports half of a wide streaming read
    for fam, v in write.values():
        fam_w[fam].append(v)
    res = {}
    for fam in sorted(set(fam_f) | set(fam_w)):
        f = fam_f.get(fam, [])
        w = fam_w.get(fam, [])
        fb = sum(f) / len(f) if f else 0.0
        wb = sum(w) / len(w) if w else 0.0
        res[fam] = {"launches": max(len(f), len(w)), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                    "hbm_bytes_per_launch": fb + wb}
    return res


SQ_COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS",
               "GRBM_GUI_ACTIVE")
N_SIMD, N_XCD = 1024, 8


def sq(csv_path: str, trace_stats: str = None):
    """Per family, averaged over its dispatches: MFMA-pipe busy = SQ_VALU_MFMA_BUSY_CYCLES (summed over the SIMDs)
    / (1,024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), the VALU and LDS instructions issued per MFMA, the MFMA FLOPs the
    busy cycles account for (counter_gflop, bf16 rate: divided by the kernel-trace duration this is the kernel's
    TFLOP/s from rocprofv3 alone), and -- when the rows carry timestamps -- the effective clock GRBM_GUI_ACTIVE /
    8 / duration (MI355X_MICROARCH.md DVFS; it reads high on dispatches under ~0.3 ms, so the busy fraction reads
    low there)."""
    per = defaultdict(lambda: defaultdict(float))
    fam_of, dur = {}, {}
    with open(csv_path) as f:
        for r in csv.DictReader(f):
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            fam_of[did] = family(r["Kernel_Name"])
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    acc = defaultdict(lambda: defaultdict(list))
    for did, c in per.items():
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        if gui <= 0:
            continue
        a = acc[fam_of[did]]
        a["mfma_busy"].append(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (N_SIMD * gui / N_XCD))
        nm = c.get("SQ_INSTS_MFMA", 0.0)
        if nm > 0:
            a["valu_per_mfma"].append(c.get("SQ_INSTS_VALU", 0.0) / nm)
            a["lds_per_mfma"].append(c.get("SQ_INSTS_LDS", 0.0) / nm)
        a["mfma_insts"].append(nm)
        # dense bf16 MFMA: 1,024 FLOPs per SIMD per busy cycle (16x16x32 = 16,384 FLOPs in 16 cycles,
        # MI355X_MICROARCH.md: 32 cycles per 32x32x16), so the busy cycles re-count the kernel's MFMA FLOPs
        a["mfma_busy_cycles"].append(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0))
        a["counter_gflop"].append(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) * 1024 / 1e9)
        if did in dur and dur[did] > 0:
            a["clock_ghz"].append(gui / N_XCD / dur[did] / 1e9)
    res = {}
    for fam, a in sorted(acc.items()):
        res[fam] = {k: (sum(v) / len(v) if v else None) for k, v in a.items()}
        res[fam]["launches"] = len(a["mfma_busy"])
    return res


def _stamp(res: dict) -> dict:
    """Tag a summary with the workload of the profiled bench run (--workload FILE, written by bench.py
    --workload-out) and its creation time: bench.py reads only summaries of its own workload, newest first."""
    if WORKLOAD_FILE:
        with open(WORKLOAD_FILE) as f:
            res["_workload"] = json.load(f)
    import datetime
    res["_created"] = datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
    return res


WORKLOAD_FILE = None

if __name__ == "__main__":
    if "--workload" in sys.argv:
        i = sys.argv.index("--workload")
        WORKLOAD_FILE = sys.argv[i + 1]
        del sys.argv[i:i + 2]
    if sys.argv[1] == "stats":
        stats(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1)
    elif sys.argv[1] == "steady":
        r = _stamp(steady(sys.argv[2], int(sys.argv[4]) if len(sys.argv) > 4 else 8))
        with open(sys.argv[3], "w") as f:
            f.write(json.dumps(r, indent=1) + "\n")
        fam = {k: v for k, v in r.items() if not k.startswith("_")}
        if r.get("_workload"):
            print("workload", json.dumps(r["_workload"]))
        tot = sum(v["ms_per_step"] for v in fam.values())
        print(f"last {r['_steps']} steps, {r['_span_ms_per_step']:.3f} ms/step wall, {tot:.3f} ms/step of kernels")
        print(f"{'family':48s} {'n/step':>7s} {'avg_us':>9s} {'ms/step':>8s} {'%':>6s}")
        for k, v in sorted(fam.items(), key=lambda kv: -kv[1]["ms_per_step"]):
            print(f"{k:48s} {v['launches_per_step']:7.1f} {v['avg_launch_ms'] * 1e3:9.1f} {v['ms_per_step']:8.3f} "
                  f"{100 * v['ms_per_step'] / tot:6.2f}")
    elif sys.argv[1] == "sq":
        r = _stamp(sq(sys.argv[2]))
        js = json.dumps(r, indent=1)
        if len(sys.argv) > 3:
            with open(sys.argv[3], "w") as f:
                f.write(js + "\n")
        print(js)
    elif sys.argv[1] == "traffic":
        r = traffic(sys.argv[2], sys.argv[3])
        if len(sys.argv) > 5:      # training steps the profiled run executed (bench: warmup + steps + timer)
            r["_steps"] = int(sys.argv[5])
        r = _stamp(r)
        js = json.dumps(r, indent=1)
        if len(sys.argv) > 4:
            with open(sys.argv[4], "w") as f:
                f.write(js + "\n")
        print(js)
