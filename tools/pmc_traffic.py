#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, then
WRITE_SIZE, each with --kernel-trace --output-format csv), as
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes:
  * separate passes (the TCC block cannot host both counters at once);
  * FETCH_SIZE / WRITE_SIZE are kilobytes;
  * on gfx950 FETCH_SIZE reports half the bytes of 16-byte-per-lane
    streaming reads -> doubled here (our kernels' hot loads are 16-byte
    global loads; other widths are uncalibrated, so this is an estimate);
  * Infinity-Cache hits are counted, not excluded.

usage: tools/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> <out.json> [--batch B] [--config TEXT]
The output carries a _meta record: the kernel-source tag of this tree
(bench.kernel_source_tag) and the pass batch, so bench.py only reports the
traffic for the kernels and batch it was measured on.
Groups dispatches by kernel symbol (bh::<name><...>(...) -> <name>) and
writes per-kernel means per dispatch.
"""
import csv
import glob
import json
import os
import re
import sys


def base(name):
    m = re.search(r"bh::(\w+)", name)
    return m.group(1) if m else name.split("(")[0]


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = base(r["Kernel_Name"])
            key = (r.get("Dispatch_Id"), k)
            per.setdefault(k, {})
            per[k][key] = per[k].get(key, 0.0) + float(r["Counter_Value"])
    return {k: (len(v), sum(v.values()) / max(len(v), 1)) for k, v in per.items()}


def main(fd, wd, out, batch=24, config=""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_source_tag
    fetch = load(fd, "FETCH_SIZE")
    write = load(wd, "WRITE_SIZE") if wd != "-" else {}  # "-": a FETCH_SIZE pass only
    res = {}
    for k in sorted(set(fetch) | set(write)):
        nf, f = fetch.get(k, (0, 0.0))
        nw, w = write.get(k, (0, 0.0))
        res[k] = dict(dispatches_fetch_pass=nf, dispatches_write_pass=nw, fetch_kb_mean=f, write_kb_mean=w,
                      traffic_bytes_per_launch=2.0 * f * 1024.0 + w * 1024.0)
        print("%-28s fetch %9.1f KB  write %9.1f KB  -> %10.0f B/launch (x2 fetch)  [%d/%d dispatches]"
              % (k, f, w, res[k]["traffic_bytes_per_launch"], nf, nw))
    res["_meta"] = dict(kernel_source_tag=kernel_source_tag(), pass_batch=batch, config=config,
                        fetch_correction="FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section)")
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1, sort_keys=True)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--config", default="")
    a = ap.parse_args()
    main(a.fetch_dir, a.write_dir, a.out, a.batch, a.config)
