#!/usr/bin/env python3
"""Per-op HIP-event timing of one model through the HIP executor.

Usage: python tools/profile_ops.py [--model mobilenet_v2_int8] [--iters 50]
Prints one line per launch (op, kernel, shape, us, algorithmic GB/s, TOPS)
and a per-kernel summary; --json writes the rows to a file.
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mobilenet_v2_int8")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
    from band_amd import tflite_synth as S
    from band_amd.tflite_reader_py import read

    if a.model == "mobilenet_v2_int8":
        buf = S.mobilenet_v2(np.int8, seed=0, batch=a.batch)
    elif a.model == "mobilenet_v1_int8":
        buf = S.mobilenet_v1(np.int8, seed=0, batch=a.batch)
    elif hasattr(S, a.model):  # e.g. ssd_mobilenet_v2, deeplab_v3_mobilenet_v2, posenet_mobilenet_v1
        buf = getattr(S, a.model)(np.int8, batch=a.batch)
    else:
        buf = open(a.model, "rb").read()
    desc = read(buf)
    m = HipModel(0)
    assert m.FromBuffer(buf).ok()
    ex = HipModelExecutor(0, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, 1)
    for _ in range(3):
        assert ex.ExecuteSubgraph(key).ok()
    rows = ex.ProfileSubgraph(key, iters=a.iters)
    names = {0: "ADD", 1: "AVGPOOL", 3: "CONV", 4: "DWCONV", 9: "FC", 17: "MAXPOOL", 18: "MUL", 22: "RESHAPE"}
    tot = 0.0
    summary = {}
    for r in rows:
        op = desc["ops"][r["op_index"]]
        ins = desc["tensors"][op["inputs"][0]]["shape"]
        outs = desc["tensors"][op["outputs"][0]]["shape"]
        extra = ""
        if op["builtin"] in (3, 4):
            w = desc["tensors"][op["inputs"][1]]["shape"]
            extra = "k%dx%d" % (w[1], w[2])
        us = r["ms"] * 1e3
        tot += us
        gbs = r["alg_bytes"] / (r["ms"] * 1e-3) / 1e9 if r["ms"] > 0 else 0
        tops = r["alg_ops"] / (r["ms"] * 1e-3) / 1e12 if r["ms"] > 0 else 0
        r.update(op=names.get(op["builtin"], str(op["builtin"])), in_shape=ins, out_shape=outs, us=us, gbs=gbs, tops=tops)
        s = summary.setdefault(r["kernel"], [0, 0.0, 0.0])
        s[0] += 1
        s[1] += us
        s[2] += r["alg_bytes"]
        print("%3d %-8s %-18s %-20s -> %-20s %-6s %8.2f us %8.1f GB/s %6.2f TOPS" % (
            r["op_index"], r["op"], r["kernel"], ins, outs, extra, us, gbs, tops))
    print("total %.1f us per inference (sum of per-launch event times)" % tot)
    for k, (n, us, b) in sorted(summary.items(), key=lambda kv: -kv[1][1]):
        print("  %-18s launches %3d  %8.1f us  avg %6.2f us  %7.1f GB/s" % (k, n, us, us / n, b / (us * 1e-6) / 1e9))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
