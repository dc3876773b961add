"""Instruction mix of a kernel's loops from hipcc device assembly (offline, no GPU).

usage: hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o /tmp/k.s FILE.hip
       python tools/asm_loops.py /tmp/k.s SYMBOL_SUBSTRING

Prints, for the whole function and for every backward-branch loop in it, the count of MFMA, VALU (v_*, with
v_accvgpr moves and conversions split out), SALU (s_*), LDS (ds_*), vector-memory (buffer_/global_) and waitcnt
instructions, and the VALU / SALU / LDS per MFMA ratios the SQ_INSTS_* counters report at run time.
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("v_cvt") or op.startswith("v_perm") or op.startswith("v_pack"):
        return "cvt"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    return "other"


def function_body(lines, sym):
    start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(sym) + r"\S*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or
               re.match(r"^\.Lfunc_end", lines[i]))
    return lines[start:end]


def mix(body):
    c = Counter()
    for l in body:
        s = l.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        c[classify(s.split()[0])] += 1
    return c


def report(name, c):
    m = max(c["mfma"], 1)
    v = c["valu"] + c["accmov"] + c["cvt"]
    print(f"{name}: mfma {c['mfma']} valu {c['valu']} accmov {c['accmov']} cvt {c['cvt']} salu {c['salu']} "
          f"lds {c['lds']} vmem {c['vmem']} wait {c['wait']} barrier {c['barrier']} | per MFMA: "
          f"VALU {v / m:.2f} SALU {c['salu'] / m:.2f} LDS {c['lds'] / m:.2f}")


def main():
    lines = open(sys.argv[1]).read().splitlines()
    body = function_body(lines, sys.argv[2])
    report("function", mix(body))
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
    for i, l in enumerate(body):
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            report(f"loop {m.group(2)} (lines {labels[m.group(2)]}-{i})", mix(body[labels[m.group(2)]:i + 1]))


if __name__ == "__main__":
    main()
