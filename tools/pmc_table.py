"""Per-kernel mean of every PMC counter in rocprofv3 counter_collection CSVs under a directory.

usage: python tools/pmc_table.py <dir> [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for sub in sorted(glob.glob(os.path.join(root, "*"))):
        files = glob.glob(os.path.join(sub, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
        for f in files:
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if filt and filt not in k:
                    continue
                acc[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        print("==", os.path.basename(sub))
        for k, cs in acc.items():
            vals = ", ".join("%s=%.4g" % (c, sum(d.values()) / len(d)) for c, d in sorted(cs.items()))
            print("  %-45s %s" % (k, vals))


if __name__ == "__main__":
    main()
