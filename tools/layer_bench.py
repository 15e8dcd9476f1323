#!/usr/bin/env python3
"""Kernel-level throughput of the MobileNetV2 layer shapes at job batch B.

Usage: python tools/layer_bench.py [--batch 64] [--iters 20] [--only conv|dw|stem]
Each layer: the C-ABI launch (bh_conv2d_i8 / bh_dwconv2d_i8) issued `iters`
times back to back on one stream between two HIP events; prints us per
launch, algorithmic GB/s (input + output + filter bytes) and the fraction of
the 8 TB/s HBM peak.  Random data (parity is the tests' job).
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (kind, spatial_in, cin, cout, k, stride) - MobileNetV2-1.0-224 layers, deduplicated
MNV2 = [
    ("stem", 224, 3, 32, 3, 2),
    ("dw", 112, 32, 32, 3, 1), ("conv", 112, 32, 16, 1, 1), ("conv", 112, 16, 96, 1, 1),
    ("dw", 112, 96, 96, 3, 2), ("conv", 56, 96, 24, 1, 1), ("conv", 56, 24, 144, 1, 1),
    ("dw", 56, 144, 144, 3, 1), ("conv", 56, 144, 24, 1, 1), ("dw", 56, 144, 144, 3, 2),
    ("conv", 28, 144, 32, 1, 1), ("conv", 28, 32, 192, 1, 1), ("dw", 28, 192, 192, 3, 1),
    ("conv", 28, 192, 32, 1, 1), ("dw", 28, 192, 192, 3, 2), ("conv", 14, 192, 64, 1, 1),
    ("conv", 14, 64, 384, 1, 1), ("dw", 14, 384, 384, 3, 1), ("conv", 14, 384, 64, 1, 1),
    ("conv", 14, 384, 96, 1, 1), ("conv", 14, 96, 576, 1, 1), ("dw", 14, 576, 576, 3, 1),
    ("conv", 14, 576, 96, 1, 1), ("dw", 14, 576, 576, 3, 2), ("conv", 7, 576, 160, 1, 1),
    ("conv", 7, 160, 960, 1, 1), ("dw", 7, 960, 960, 3, 1), ("conv", 7, 960, 160, 1, 1),
    ("conv", 7, 960, 320, 1, 1), ("conv", 7, 320, 1280, 1, 1),
]

# MobileNetV1-1.0-224 (PoseNet's backbone), deduplicated
MNV1 = [
    ("stem", 224, 3, 32, 3, 2),
    ("dw", 112, 32, 32, 3, 1), ("conv", 112, 32, 64, 1, 1), ("dw", 112, 64, 64, 3, 2),
    ("conv", 56, 64, 128, 1, 1), ("dw", 56, 128, 128, 3, 1), ("conv", 56, 128, 128, 1, 1),
    ("dw", 56, 128, 128, 3, 2), ("conv", 28, 128, 256, 1, 1), ("dw", 28, 256, 256, 3, 1),
    ("conv", 28, 256, 256, 1, 1), ("dw", 28, 256, 256, 3, 2), ("conv", 14, 256, 512, 1, 1),
    ("dw", 14, 512, 512, 3, 1), ("conv", 14, 512, 512, 1, 1), ("dw", 14, 512, 512, 3, 2),
    ("conv", 7, 512, 1024, 1, 1), ("dw", 7, 1024, 1024, 3, 1), ("conv", 7, 1024, 1024, 1, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--dtype", default="int8")
    ap.add_argument("--net", default="mnv2", choices=["mnv2", "mnv1"])
    ap.add_argument("--layer", type=int, default=-1, help="only this row of the MNV2 table (0-based)")
    ap.add_argument("--no-taps", action="store_true", help="depthwise: the per-tap kernel (no tap table)")
    ap.add_argument("--dw-hint", type=int, default=0, help="depthwise kernel: 0 auto, 1 run, 2 dot, 3 mfma")
    a = ap.parse_args()
    from band_amd import _abi
    from tests.kernel_harness import ConvCase
    lib = _abi.load()
    s = ctypes.c_void_p()
    lib.bh_stream_create(ctypes.byref(s))
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.bh_event_create(ctypes.byref(e0))
    lib.bh_event_create(ctypes.byref(e1))
    rng = np.random.default_rng(0)
    dt = np.int8 if a.dtype == "int8" else np.uint8
    tot = {}
    for li, (kind, sp, ci, co, k, st) in enumerate(MNV2 if a.net == "mnv2" else MNV1):
        if a.only and kind != a.only:
            continue
        if a.layer >= 0 and li != a.layer:
            continue
        dw = kind == "dw"
        c = ConvCase(rng, a.batch, sp, sp, ci, co, k, k, stride=(st, st), depthwise=dw, dtype=dt,
                     taps=not a.no_taps, kernel_hint=a.dw_hint)
        keep = []
        p = c.params(lib, keep)
        fn = lib.bh_dwconv2d_i8 if dw else lib.bh_conv2d_i8
        _abi.check(fn(ctypes.byref(p), s), "launch")
        lib.bh_stream_sync(s)
        lib.bh_event_record(e0, s)
        for _ in range(a.iters):
            fn(ctypes.byref(p), s)
        lib.bh_event_record(e1, s)
        lib.bh_stream_sync(s)
        ms = ctypes.c_float()
        lib.bh_event_elapsed_ms(e0, e1, ctypes.byref(ms))
        us = ms.value * 1e3 / a.iters
        oh = c.oh
        nin = a.batch * sp * sp * ci
        nout = a.batch * oh * oh * (ci if dw else co)
        nw = k * k * (ci if dw else ci * co)
        gbs = (nin + nout + nw) / (us * 1e-6) / 1e9
        macs = nout * k * k * (1 if dw else ci)
        print("%-5s %3d %4d->%4d k%d s%d  %8.1f us  %7.0f GB/s  %5.1f%% HBM  %6.1f TOPS" %
              (kind, sp, ci, co, k, st, us, gbs, 100 * gbs / 8000, 2 * macs / (us * 1e-6) / 1e12), flush=True)
        t = tot.setdefault(kind, [0.0, 0.0])
        t[0] += us
        t[1] += nin + nout + nw
        del keep
    for kind, (us, b) in tot.items():
        print("total %-5s %9.1f us  %7.0f GB/s (batch %d, each distinct layer once)" %
              (kind, us, b / (us * 1e-6) / 1e9, a.batch))


if __name__ == "__main__":
    main()
