#!/usr/bin/env python3
"""MFMA-i8 roofline of every MobileNetV2-1.0-224 Conv2D shape at job batch
B in {1, 32, 256} (north_star's ">= 40 % MFMA-i8
roofline on MobileNetV2 Conv2D"), plus the PoseNet / SSD heads with the
highest arithmetic intensity.

Each layer runs through bh_conv2d_i8 with the route the executor would take
(or --hint), on random int8 operands (MFMA cycles do not depend on data,
but the chip's clock does: MI355X_MICROARCH.md 'DVFS give-back').  Kernel
time is the dispatch's own begin / end timestamps (bh_profile_events ->
hipExtLaunchKernel), averaged over --iters launches issued back to back.
Per layer:
  ops      = 2 M N K (M = B * OH * OW, K = kh * kw * Cin)
  bytes    = M Cin + M N + N K + 12 N (input once, output, filters, tables)
  TOPS     = ops / time;  frac = TOPS / 5000 (dense i8 peak, 5.0 POPS)
  attain   = min(5000, ops/bytes * 8 TB/s) TOPS (roofline at this intensity)
  of_att   = TOPS / attain

Usage: python tools/mfma_layer_bench.py [--batches 1,32,256] [--iters 20]
       [--json out.json]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TOPS = 5000.0  # dense int8 MFMA, MI355X (2x bf16's 2.5 PF)
HBM_TBS = 8.0

# (name, spatial_in, in_c, out_c, k, stride): MobileNetV2-1.0-224's Conv2D
# layers (stem, the 1x1 expand / project layers, the 1280 head), then the
# highest-intensity 1x1 layers of the other C3 models
LAYERS = [
    ("mnv2 stem 3x3 s2", 224, 3, 32, 3, 2),
    ("mnv2 112 32->16", 112, 32, 16, 1, 1), ("mnv2 112 16->96", 112, 16, 96, 1, 1),
    ("mnv2 56 96->24", 56, 96, 24, 1, 1), ("mnv2 56 24->144", 56, 24, 144, 1, 1),
    ("mnv2 56 144->24", 56, 144, 24, 1, 1), ("mnv2 28 144->32", 28, 144, 32, 1, 1),
    ("mnv2 28 32->192", 28, 32, 192, 1, 1), ("mnv2 28 192->32", 28, 192, 32, 1, 1),
    ("mnv2 14 192->64", 14, 192, 64, 1, 1), ("mnv2 14 64->384", 14, 64, 384, 1, 1),
    ("mnv2 14 384->64", 14, 384, 64, 1, 1), ("mnv2 14 384->96", 14, 384, 96, 1, 1),
    ("mnv2 14 96->576", 14, 96, 576, 1, 1), ("mnv2 14 576->96", 14, 576, 96, 1, 1),
    ("mnv2 7 576->160", 7, 576, 160, 1, 1), ("mnv2 7 160->960", 7, 160, 960, 1, 1),
    ("mnv2 7 960->160", 7, 960, 160, 1, 1), ("mnv2 7 960->320", 7, 960, 320, 1, 1),
    ("mnv2 7 320->1280", 7, 320, 1280, 1, 1),
    ("posenet 14 512->512", 14, 512, 512, 1, 1), ("posenet 14 512->1024", 14, 512, 1024, 1, 1),
    ("posenet 14 1024->1024", 14, 1024, 1024, 1, 1), ("ssd 7 1280->256", 7, 1280, 256, 1, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,32,256")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--hint", type=int, default=0, help="force a conv form (BH_CONV_*), 0 = routed")
    ap.add_argument("--only", default="", help="substring filter on layer names ('a|b': either)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    from band_amd import _abi
    from tests.kernel_harness import ConvCase
    lib = _abi.load()
    s = ctypes.c_void_p()
    lib.bh_stream_create(ctypes.byref(s))
    st, sp = ctypes.c_void_p(), ctypes.c_void_p()
    lib.bh_event_create(ctypes.byref(st))
    lib.bh_event_create(ctypes.byref(sp))
    rng = np.random.default_rng(0)
    rows = []
    for B in [int(b) for b in a.batches.split(",")]:
        for name, sp_in, ci, co, k, stride in LAYERS:
            if a.only and not any(o in name for o in a.only.split("|")):
                continue
            c = ConvCase(rng, B, sp_in, sp_in, ci, co, k, k, stride=(stride, stride), act=3, kernel_hint=a.hint)
            keep = []
            p = c.params(lib, keep)
            kern = lib.bh_conv2d_i8_kernel(ctypes.byref(p)).decode()
            _abi.check(lib.bh_conv2d_i8(ctypes.byref(p), s), "warm-up launch")
            lib.bh_stream_sync(s)
            tot = 0.0
            for _ in range(a.iters):
                lib.bh_event_record(st, s)
                lib.bh_profile_events(st, sp)
                _abi.check(lib.bh_conv2d_i8(ctypes.byref(p), s), "launch")
                if lib.bh_profile_events(None, None) == 0:
                    lib.bh_event_record(sp, s)
                lib.bh_stream_sync(s)
                ms = ctypes.c_float()
                lib.bh_event_elapsed_ms(st, sp, ctypes.byref(ms))
                tot += ms.value
            us = tot * 1e3 / a.iters
            M = B * c.oh * c.ow
            K = k * k * ci
            ops = 2.0 * M * co * K
            byts = B * sp_in * sp_in * ci + M * co + co * K + 12 * co  # the input once, not its im2col
            tops = ops / us / 1e6
            attain = min(PEAK_TOPS, ops / byts * HBM_TBS)  # op/B x TB/s = TOPS
            r = dict(layer=name, batch=B, M=M, N=co, K=K, kernel=kern, us=round(us, 2), gop=round(ops / 1e9, 3),
                     tops=round(tops, 1), frac_peak=round(tops / PEAK_TOPS, 4), op_per_byte=round(ops / byts, 1),
                     attainable_tops=round(attain, 1), frac_attainable=round(tops / attain, 4),
                     gbs=round(byts / us / 1e3, 1))
            rows.append(r)
            print("B%-4d %-24s %-22s M %7d N %5d K %5d  %9.2f us %8.1f TOPS  %5.1f %% peak  AI %6.1f  "
                  "%5.1f %% of attainable" % (B, name, kern, M, co, K, us, tops, 100 * tops / PEAK_TOPS,
                                               ops / byts, 100 * tops / attain), flush=True)
            del keep
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"peak_tops": PEAK_TOPS, "hbm_tbs": HBM_TBS, "iters": a.iters, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
