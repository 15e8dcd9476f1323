#!/usr/bin/env python3
"""Device time per inference vs job batch size, per model of the C3 mix.

Usage: python tools/batch_probe.py [--batches 1,8,32,128] [--models mobilenet_v2,...] [--ops B]
Prints, per (model, batch): device us per pass (graph replays back to back)
and us per inference; --ops B adds the per-launch breakdown of MobileNetV2 at
batch B (algorithmic GB/s and TOPS per launch).
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,32,128")
    ap.add_argument("--models", default="mobilenet_v2,ssd_mobilenet_v2,deeplab_v3_mobilenet_v2,posenet_mobilenet_v1")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ops", type=int, default=0)
    a = ap.parse_args()
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
    from band_amd import tflite_synth as S

    mid = 0
    for name in a.models.split(","):
        for b in [int(x) for x in a.batches.split(",")]:
            t0 = time.time()
            buf = getattr(S, name)(np.int8, batch=b)
            m = HipModel(mid)
            assert m.FromBuffer(buf).ok()
            ex = HipModelExecutor(mid, 1, DeviceFlag.kGPU)
            assert ex.PrepareSubgraph(m).ok()
            key = SubgraphKey(mid, 1)
            for _ in range(3):
                assert ex.ExecuteSubgraph(key).ok()
            us = ex.TimeSubgraph(key, iters=a.iters)
            print("%-26s B=%4d  %9.1f us/pass  %8.2f us/inf  %9.0f inf/s  (prep %.1f s)" %
                  (name, b, us, us / b, 1e6 * b / us, time.time() - t0), flush=True)
            if a.ops and b == a.ops and name == "mobilenet_v2":
                rows = ex.ProfileSubgraph(key, iters=5)
                agg = {}
                for r in rows:
                    us_l = r["ms"] * 1e3
                    print("   op %3d %-22s %8.1f us %8.1f GB/s %7.1f TOPS" %
                          (r["op_index"], r["kernel"], us_l, r["alg_bytes"] / us_l / 1e3 if us_l else 0,
                           r["alg_ops"] / us_l / 1e6 if us_l else 0))
                    g = agg.setdefault(r["kernel"], [0, 0.0, 0.0, 0.0])
                    g[0] += 1
                    g[1] += us_l
                    g[2] += r["alg_bytes"]
                    g[3] += r["alg_ops"]
                for k, g in sorted(agg.items(), key=lambda kv: -kv[1][1]):
                    print("   %-22s n=%3d %9.1f us  %8.1f GB/s  %7.1f TOPS" %
                          (k, g[0], g[1], g[2] / g[1] / 1e3, g[3] / g[1] / 1e6))
            del ex, m
            mid += 1


if __name__ == "__main__":
    main()
