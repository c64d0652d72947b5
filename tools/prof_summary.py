"""Summarise a rocprofv3 kernel trace (sqlite .db or kernel_trace.csv) into per-kernel stats.

usage: python tools/prof_summary.py <results.db|kernel_trace.csv> [out.csv]
"""
import csv
import os
import re
import sqlite3
import sys
from collections import defaultdict


_TY = {"DF16b": "bf16", "DF16_": "f16", "f": "f32"}


def _half(name):
    """The 16-bit type of a kernel that is not templated on it: the fp16 build's kernels live in the inline
    namespace `f16` (csrc/scd_common.h SCD_KERNEL_NS_BEGIN)."""
    return "f16" if ("f16::" in name or "_GLOBAL__N_13f16" in name) else "bf16"


def short(name):
    half = _half(name)
    n = re.sub(r"_ZN12_GLOBAL__N_1(3f16)?\d+", "", name)
    m = re.match(r"(\w+?)I(DF16b|DF16_|f)Li(\d+)ELi(\d+)E(Lb([01])E)?", n)
    if m:
        tail = ""
        if m.group(6) == "1":
            tail = ",fastx" if m.group(1).startswith("conv_wgrad") else ",heads"
        return "%s<%s,%s,%s%s>" % (m.group(1), _TY[m.group(2)], m.group(3), m.group(4), tail)
    m = re.match(r"(\w+?)I(DF16b|DF16_|f)E", n)
    if m:
        return "%s<%s>" % (m.group(1), _TY[m.group(2)])
    n = n.replace("(anonymous namespace)::", "").replace("f16::", "")
    m = re.search(r"conv_gemm_pp_kernel<(\d+)(, (true|false))?(, (true|false))?>", n)
    if m:
        return "conv_gemm_pp_kernel<%s,256,%s%s%s>" % (half, m.group(1), ",heads" if m.group(3) == "true" else "",
                                                      ",bnbwd" if m.group(5) == "true" else "")
    m = re.search(r"(conv_gemm_halo_kernel|conv_wgrad_pp_kernel)<([\d, ]+)>", n)
    if m:
        return "%s<%s>" % (m.group(1), m.group(2).replace(" ", ""))
    m = re.search(r"conv_gemm_ring_kernel<(true|false)(, (true|false))?>", n)
    if m:
        return "conv_gemm_ring_kernel<%s,256,128%s%s>" % (half, ",heads" if m.group(1) == "true" else "",
                                                          ",bnbwd" if m.group(3) == "true" else "")
    m = re.search(r"conv_gemm_pp_kernel<(\d+), (true|false)>", n)
    if m:
        return "conv_gemm_pp_kernel<%s,256,%s%s>" % (half, m.group(1), ",heads" if m.group(2) == "true" else "")
    m = re.search(r"conv_gemm_l1p_kernel<(\d+), (true|false), (true|false)>", n)
    if m:
        return "conv_gemm_l1p_kernel<%s,%s%s%s>" % (half, m.group(1), ",dgrad" if m.group(2) == "true" else "",
                                                   ",bnbwd" if m.group(3) == "true" else "")
    m = re.match(r"(\w+?)ENS_\d+\w*Params", n)         # mangled, non-template kernels of the anonymous namespace
    if m:
        n = m.group(1)
    m = re.match(r"(\w+?_kernel)E(P|i|S)", n)          # mangled kernels with plain pointer / int arguments
    if m:
        n = m.group(1)
    n = n.split("(")[0][:80]
    return n + " [f16]" if half == "f16" and "<" not in n else n


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur in c.execute("select name, duration from kernels"):
            yield name, float(dur)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Kernel_Name"], float(r["End_Timestamp"]) - float(r["Start_Timestamp"])


def main():
    src = sys.argv[1]
    agg = defaultdict(lambda: [0, 0.0])
    for name, dur in rows_from(src):
        a = agg[short(name)]
        a[0] += 1
        a[1] += dur
    total = sum(v[1] for v in agg.values())
    out = sys.argv[2] if len(sys.argv) > 2 else None
    lines = [("kernel", "calls", "total_us", "avg_us", "pct")]
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append((k, n, "%.1f" % (t / 1e3), "%.2f" % (t / 1e3 / n), "%.2f" % (100 * t / total)))
    if out:
        with open(out, "w", newline="") as f:
            csv.writer(f).writerows(lines)
    for l in lines[:40]:
        print("%-60s %6s %12s %10s %6s" % l)


if __name__ == "__main__":
    main()
