#!/usr/bin/env python3
"""Device time of one bh_chain_i8 launch per MobileNetV2 chain shape.

Usage: python tools/chain_bench.py [--batch 24] [--iters 50] [--px 1,2,4]

Each launch is timed back to back behind a spin kernel (HIP events on one
stream), so the figure is execution time plus the in-stream dispatch gap,
comparable to tools/mix_breakdown.py's event figures.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--px", default="1,2,4,1w16,1w8,4p,t,1d,1w8d,2d,g1w8,G1w8s2",
                    help="forms: px_blocks [wN waves] [p persistent] [d deep-issue]; t = the 2-D tile form, "
                         "t3 / t4 = runs of 2 / 4 tiles per workgroup; "
                         "sN suffix = the phase-C split over N workgroups; "
                         "g prefix = the stage form (g1w8s2: 1 pixel block, 8 waves, 2 slices)")
    ap.add_argument("--only", default="", help="comma-separated chain indices")
    a = ap.parse_args()
    from band_amd import _abi
    from tests.chain_harness import MNV2_CHAINS, ChainCase
    lib = _abi.load()
    st = ctypes.c_void_p()
    _abi.check(lib.bh_stream_create(ctypes.byref(st)), "stream")
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.bh_event_create(ctypes.byref(e0))
    lib.bh_event_create(ctypes.byref(e1))
    total = {}
    only = [int(v) for v in a.only.split(",")] if a.only else list(range(len(MNV2_CHAINS)))
    for (h, ce, s, cout, res, ce2) in [MNV2_CHAINS[i] for i in only]:
        c = ChainCase(np.random.default_rng(1), a.batch, h, h, ce, s, cout, res, ce2)
        row = []
        for form in a.px.split(","):
            label = form
            split = 0
            # "g1w8s2": the stage form, 1 block, 8 waves, 2 slices; "G": with loader waves (stage 2)
            stage = 1 if form.startswith("g") else (2 if form.startswith("G") else 0)
            form = form[1:] if stage else form
            if "s" in form and not form.startswith("t"):  # "1s2": the phase-C split over 2 workgroups
                form, split = form.split("s")[0], int(form.split("s")[1])
            tile = {"t": 1, "t3": 3, "t4": 4}.get(form, 0)
            persist = int(form.endswith("p") and not tile)
            deep = int(form.endswith("d"))
            f = "4" if tile else form.rstrip("pd")
            px, waves = (int(f.split("w")[0]), int(f.split("w")[1])) if "w" in f else (int(f), 4)
            keep = []
            q = c.params(lib, px, keep, waves, persist, tile, deep, split, stage)
            if lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0:
                row.append("   -   ")
                continue
            for _ in range(3):
                _abi.check(lib.bh_chain_i8(ctypes.byref(q), st), "chain")
            lib.bh_spin_us(st, 300 + 60 * a.iters)
            lib.bh_event_record(e0, st)
            for _ in range(a.iters):
                lib.bh_chain_i8(ctypes.byref(q), st)
            lib.bh_event_record(e1, st)
            lib.bh_stream_sync(st)
            ms = ctypes.c_float()
            lib.bh_event_elapsed_ms(e0, e1, ctypes.byref(ms))
            us = 1e3 * ms.value / a.iters
            total[label] = total.get(label, 0.0) + us
            row.append("%7.2f" % us)
        print("%3dx%-3d ce %4d s%d -> %3d%s -> %4d   %s" % (h, h, ce, s, cout, "+res" if res else "    ", ce2,
                                                           "  ".join(row)), flush=True)
    print("sum", {k: round(v, 1) for k, v in total.items()})


if __name__ == "__main__":
    main()
