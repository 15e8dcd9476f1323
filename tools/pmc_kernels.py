#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 PMC counters (one --pmc pass directory per
argument), grouped by kernel symbol: where the wave-cycles (the CU time a
kernel holds, the quantity concurrent Band workers compete for) go.
usage: tools/pmc_kernels.py <pass_dir> [<pass_dir> ...]"""
import collections
import csv
import glob
import os
import re
import sys


def base(name):
    m = re.search(r"bh::(\w+)", name)
    return m.group(1) if m else name.split("(")[0]


def main(dirs):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = base(r["Kernel_Name"])
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    counters = sorted({c for v in tot.values() for c in v})
    key = "SQ_WAVE_CYCLES" if "SQ_WAVE_CYCLES" in counters else counters[0]
    allk = sum(v.get(key, 0.0) for v in tot.values())
    print("%-26s %6s %7s " % ("kernel", "disp", "%" + key[:10]) + " ".join("%14s" % c[:14] for c in counters))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1].get(key, 0.0)):
        n = len(disp[k])
        print("%-26s %6d %6.1f%% " % (k[:26], n, 100 * v.get(key, 0.0) / max(allk, 1)) +
              " ".join("%14.0f" % (v.get(c, 0.0) / n) for c in counters))


if __name__ == "__main__":
    main(sys.argv[1:])
