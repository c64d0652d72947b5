"""Per-kernel SQ counter summary of rocprofv3 --pmc counter_collection.csv outputs (tools/gpu_pmc_sq.sh).

python tools/sq_summary.py [--by-grid] <pass dir> [<pass dir> ...]
--by-grid: one row per (kernel, grid size), i.e. per launch shape (the step launches one kernel on several shapes).
Prints, per kernel name: launches, and each counter's mean per launch; plus derived ratios (wait / active shares of
wave cycles, LDS bank-conflict cycles per LDS instruction, effective clock from GRBM_GUI_ACTIVE / 8 / duration is not
available here: the clock line uses GRBM_GUI_ACTIVE / 8 per launch in cycles).
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


BY_GRID = False


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit("no counter_collection.csv under %s" % d)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for row in csv.DictReader(open(f[0])):
        k = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
        k = short(k)
        if BY_GRID:
            k = "%s grid=%s" % (k, row.get("Grid_Size") or row.get("Grid-Size") or "?")
        c = row.get("Counter_Name") or row.get("Counter-Name")
        v = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
        did = row.get("Dispatch_Id") or row.get("Dispatch-Id")
        acc[k][c] += v
        disp[k].add(did)
    return acc, disp


def main():
    global BY_GRID
    args = sys.argv[1:]
    if args and args[0] == "--by-grid":
        BY_GRID = True
        args = args[1:]
    tot = collections.defaultdict(dict)
    n = {}
    for d in args:
        acc, disp = load(d)
        for k, cs in acc.items():
            n[k] = max(n.get(k, 0), len(disp[k]))
            for c, v in cs.items():
                tot[k][c] = v
    for k in sorted(tot):
        cs = tot[k]
        m = {c: v / max(1, n[k]) for c, v in cs.items()}
        print("%s  (%d launches)" % (k[:100], n[k]))
        for c in sorted(m):
            print("    %-26s %16.1f" % (c, m[c]))
        wc = m.get("SQ_WAVE_CYCLES", 0)
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_WAIT_INST_LDS"):
                if c in m:
                    print("    %-26s %15.1f%%" % (c + " / WAVE_CYCLES", 100.0 * m[c] / wc))
        if m.get("GRBM_GUI_ACTIVE") and m.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            # MFMA busy cycles are summed over SIMDs (1024 on the chip); GUI_ACTIVE over the 8 XCDs
            print("    %-26s %15.1f%%" % ("MFMA busy / (GUI_ACTIVE/8 x 1024 SIMDs)",
                                          100.0 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)))
        if m.get("SQ_INSTS_LDS"):
            print("    %-26s %16.2f" % ("LDS_BANK_CONFLICT / INSTS_LDS", m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"]))


if __name__ == "__main__":
    main()
