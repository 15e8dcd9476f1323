#!/usr/bin/env python3
"""Per-launch device-time breakdown of the C3 mix at a given job batch.

Usage: python tools/mix_breakdown.py [--batch 24] [--iters 20] [--top 40]

Prepares each C3 model (MobileNetV2, SSD-MobileNetV2, DeepLabV3,
PoseNet; 224x224 int8, the bench's synthetic weights) with a leading batch
of B, times every launch with HIP events in program order
(HipModelExecutor::ProfileSubgraph: per-dispatch begin / end timestamps) and prints
the launches sorted by time with their layer shape, kernel and the
algorithmic rates they imply; then a per-kernel summary.  This is where the
next kernel work is chosen.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--models", default="")
    a = ap.parse_args()
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
    from band_amd import tflite_synth as S
    from band_amd.tflite_reader_py import read

    names = a.models.split(",") if a.models else list(S.MIX_C3)
    rows, keep, floors = [], [], []
    for mid, name in enumerate(names):
        buf = getattr(S, name)(np.int8, size=224, batch=a.batch)
        desc = read(buf)
        m = HipModel(mid)
        assert m.FromBuffer(buf).ok()
        ex = HipModelExecutor(mid, 1, DeviceFlag.kGPU)
        assert ex.PrepareSubgraph(m).ok()
        key = SubgraphKey(mid, 1)
        for _ in range(3):
            assert ex.ExecuteSubgraph(key).ok()
        ex.TimeSubgraph(key, iters=20)  # untimed: the first replays after an idle GPU run at a lower clock
        dev_us = ex.TimeSubgraph(key, iters=50)
        prof, floor = ex.ProfileSubgraph(key, iters=a.iters, with_floor=True)
        floors.append(floor)
        ex.SetUseGraph(False)
        eager_us = ex.TimeSubgraph(key, iters=20)
        ex.SetUseGraph(True)
        ko_sum = sum(r["ms"] for r in prof) * 1e3
        for r in prof:
            op = desc["ops"][r["op_index"]]
            ins = desc["tensors"][op["inputs"][0]]["shape"] if op["inputs"] else []
            outs = desc["tensors"][op["outputs"][0]]["shape"]
            extra = ""
            if op["builtin"] in (3, 4) and len(op["inputs"]) > 1:
                w = desc["tensors"][op["inputs"][1]]["shape"]
                extra = "k%dx%d" % (w[1], w[2])
            us = max(r["ms"] * 1e3, 1e-3)
            rows.append(dict(model=name, op=r["op_index"], kernel=r["kernel"], ins=ins, outs=outs, extra=extra,
                             us=us, bytes=r["alg_bytes"], ops=r["alg_ops"]))
        print("%-28s graph replay %.1f us per pass (%.2f per inference), eager %.1f; %d launches; "
              "empty kernel %.2f us, kernel-only sum %.1f" % (name, dev_us, dev_us / a.batch, eager_us, len(prof),
                                                             floor, ko_sum), flush=True)
        keep.append((m, ex))
    tot = sum(r["us"] for r in rows)
    print("\nsum of kernel-only launch times: %.1f us for one pass of every model (batch %d)" % (tot, a.batch))
    print("%-24s %4s %-24s %-20s %-20s %-6s %8s %7s %7s %6s" % ("model", "op", "kernel", "in", "out", "filt", "us",
                                                               "%", "GB/s", "TOPS"))
    for r in sorted(rows, key=lambda r: -r["us"])[:a.top]:
        t = r["us"] * 1e-6
        print("%-24s %4d %-24s %-20s %-20s %-6s %8.2f %6.2f%% %7.0f %6.1f" % (
            r["model"][:24], r["op"], r["kernel"][:24], r["ins"], r["outs"], r["extra"], r["us"],
            100 * r["us"] / tot, r["bytes"] / t / 1e9, r["ops"] / t / 1e12))
    summ = {}
    for r in rows:
        s = summ.setdefault(r["kernel"].split("+")[0], [0, 0.0])
        s[0] += 1
        s[1] += r["us"]
    print("\nper kernel (share of summed kernel-only time):")
    for k, (n, us) in sorted(summ.items(), key=lambda kv: -kv[1][1]):
        print("  %-26s launches %4d  %8.1f us  %6.1f%%" % (k, n, us, 100 * us / tot))


if __name__ == "__main__":
    main()
