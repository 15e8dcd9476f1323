#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 PMC counters (one --pmc pass directory per
argument), grouped by kernel symbol: where the wave-cycles (the CU time a
kernel holds, the quantity concurrent Band workers compete for) go.

--full groups by the whole instantiation (template arguments kept) and adds
the per-dispatch register / LDS allocation the trace reports plus the
derived stall shares (SQ_WAIT_INST_ANY / SQ_WAIT_ANY / SQ_ACTIVE_INST_ANY
over SQ_WAVE_CYCLES, VALU instructions per wave).
usage: tools/pmc_kernels.py [--full] <pass_dir> [<pass_dir> ...]"""
import collections
import csv
import glob
import os
import re
import sys


def base(name, full):
    if full:
        n = name.split("(")[0] if "(" in name and "<" not in name.split("(")[0] else name
        m = re.search(r"bh::(\w+<[^()]*>)", n) or re.search(r"bh::(\w+)", n)
        return m.group(1) if m else n[:60]
    m = re.search(r"bh::(\w+)", name)
    return m.group(1) if m else name.split("(")[0]


RES_COLS = ("VGPR_Count", "Arch_VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Lds_Size",
            "Workgroup_Size", "Grid_Size")


def main(argv):
    full = "--full" in argv
    dirs = [a for a in argv if a != "--full"]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    res = collections.defaultdict(dict)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = base(r["Kernel_Name"], full)
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((d, r["Dispatch_Id"]))
                for c in RES_COLS:
                    if c in r and r[c] not in ("", None):
                        res[k][c] = r[c]
    counters = sorted({c for v in tot.values() for c in v})
    key = "SQ_WAVE_CYCLES" if "SQ_WAVE_CYCLES" in counters else counters[0]
    allk = sum(v.get(key, 0.0) for v in tot.values())
    npass = max(1, len(dirs))
    print("%-26s %6s %7s " % ("kernel", "disp", "%" + key[:10]) + " ".join("%14s" % c[:14] for c in counters))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1].get(key, 0.0)):
        n = max(1, len(disp[k]) // npass)
        print("%-26s %6d %6.1f%% " % (k[:26], n, 100 * v.get(key, 0.0) / max(allk, 1)) +
              " ".join("%14.0f" % (v.get(c, 0.0) / n) for c in counters))
    if not full:
        return
    print("\nper instantiation: stall shares of SQ_WAVE_CYCLES, instructions per wave, allocation")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1].get(key, 0.0)):
        wc = v.get("SQ_WAVE_CYCLES", 0.0)
        waves = v.get("SQ_WAVES", 0.0)
        if wc <= 0:
            continue
        parts = []
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES"):
            if c in v:
                parts.append("%s %.1f%%" % (c[3:], 100 * v[c] / wc))
        if waves > 0:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_I8", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                      "SQ_INSTS_VMEM"):
                if c in v:
                    parts.append("%s/wave %.0f" % (c[9:] or c, v[c] / waves))
        if "SQ_LDS_BANK_CONFLICT" in v:
            parts.append("LDS_BANK_CONFLICT/disp %.0f" % (v["SQ_LDS_BANK_CONFLICT"] / max(1, len(disp[k]) // npass)))
        print("%s\n    %s\n    %s" % (k, "; ".join(parts), " ".join("%s=%s" % kv for kv in sorted(res[k].items()))))


if __name__ == "__main__":
    main(sys.argv[1:])
