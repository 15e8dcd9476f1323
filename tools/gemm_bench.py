#!/usr/bin/env python3
"""A-B of the two kernels for the batched deep / wide 1x1 conv layers of the
C3 mix: conv_mfma_kernel (BH_CONV_MFMA) vs the LDS-staged conv_gemm_kernel
(BH_CONV_GEMM), each shape at job batch B, both forms checked equal.

Usage: python tools/gemm_bench.py [--batch 24] [--iters 20]
Per launch: back-to-back launches between two HIP events (the dispatch gap
is included, equally for both), algorithmic TOPS and GB/s.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (spatial, in_c, out_c): the 1x1 stride-1 layers of MobileNetV2 / SSD /
# DeepLabV3 / PoseNet (224x224) that conv_xs_kernel does not take
SHAPES = [
    (14, 384, 64), (14, 384, 96), (14, 576, 96), (7, 576, 160), (7, 160, 960), (7, 960, 160), (7, 960, 320),
    (7, 320, 1280), (7, 1280, 256), (14, 576, 273), (7, 1280, 546), (14, 576, 160), (14, 960, 160),
    (14, 960, 320), (14, 512, 256), (14, 512, 512), (14, 512, 1024), (14, 1024, 1024), (14, 1024, 32),
    (14, 576, 12), (14, 256, 21),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", type=int, default=-1, help="only this row of SHAPES")
    ap.add_argument("--hints", default="1,2", help="kernel hints to run (1 mfma, 2 gemm)")
    a = ap.parse_args()
    hints = [int(h) for h in a.hints.split(",")]
    from band_amd import _abi
    from tests.kernel_harness import ConvCase
    lib = _abi.load()
    s = ctypes.c_void_p()
    lib.bh_stream_create(ctypes.byref(s))
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.bh_event_create(ctypes.byref(e0))
    lib.bh_event_create(ctypes.byref(e1))
    rng = np.random.default_rng(0)
    tot = {1: 0.0, 2: 0.0}
    for row, (sp, ci, co) in enumerate(SHAPES):
        if a.only >= 0 and row != a.only:
            continue
        c = ConvCase(rng, a.batch, sp, sp, ci, co, 1, 1)
        res, outs = {}, {}
        for hint in hints:
            c.kernel_hint = hint
            keep = []
            p = c.params(lib, keep)
            name = lib.bh_conv2d_i8_kernel(ctypes.byref(p)).decode()
            _abi.check(lib.bh_conv2d_i8(ctypes.byref(p), s), "launch")
            lib.bh_stream_sync(s)
            outs[hint] = c._dy.download(np.int8, (a.batch, sp, sp, co))
            lib.bh_event_record(e0, s)
            for _ in range(a.iters):
                lib.bh_conv2d_i8(ctypes.byref(p), s)
            lib.bh_event_record(e1, s)
            lib.bh_stream_sync(s)
            ms = ctypes.c_float()
            lib.bh_event_elapsed_ms(e0, e1, ctypes.byref(ms))
            res[hint] = (ms.value * 1e3 / a.iters, name)
            del keep
        if len(hints) < 2:
            print("%3d %5d->%5d hint %d: %.2f us %s" % (sp, ci, co, hints[0], *res[hints[0]]), flush=True)
            continue
        same = np.array_equal(outs[1], outs[2])
        M = a.batch * sp * sp
        ops = 2.0 * M * co * ci
        by = M * ci + M * co + ci * co
        line = "%3d %5d->%5d M %6d  %.2f GOP" % (sp, ci, co, M, ops / 1e9)
        for hint in (1, 2):
            us, name = res[hint]
            tot[hint] += us
            line += "  | %-17s %7.2f us %6.1f TOPS %5.0f GB/s" % (name, us, ops / us / 1e6, by / us / 1e3)
        line += "  | x%.2f %s" % (res[1][0] / res[2][0], "equal" if same else "DIFFER")
        print(line, flush=True)
    print("total mfma %.1f us, gemm %.1f us" % (tot[1], tot[2]))


if __name__ == "__main__":
    main()
