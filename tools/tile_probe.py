#!/usr/bin/env python3
"""Where a chain_tile_kernel workgroup spends its time.

Usage: python tools/tile_probe.py [--batch 24] [--only 0,2]

Runs the tile form of bh_chain_i8 on MobileNetV2 chain shapes with
bh_chain_params.debug_stamps set: each workgroup records s_memtime (shader
clock) at its phase boundaries - start, DMA issued, DMA landed (after the
barrier), phase A (depthwise), phase B (first 1x1), phase C (second 1x1),
copy-out issued.  Prints per phase the mean / p90 over workgroups in clocks,
and the workgroup count.
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
    ap.add_argument("--only", default="")
    ap.add_argument("--raster", default="", help="probe chain_kernel in this form instead (e.g. 4, 2, 1, 1w8)")
    a = ap.parse_args()
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    from tests.chain_harness import MNV2_CHAINS, ChainCase
    lib = _abi.load()
    only = [int(v) for v in a.only.split(",")] if a.only else list(range(len(MNV2_CHAINS)))
    names = ["prologue"] + (["issue", "land", "A", "B", "C", "out"] if not a.raster else ["A", "B", "o1 out", "C", "out"])
    print("chain                              wgs   " + "  ".join("%14s" % n for n in names))
    for (h, ce, s, cout, res, ce2) in [MNV2_CHAINS[i] for i in only]:
        c = ChainCase(np.random.default_rng(1), a.batch, h, h, ce, s, cout, res, ce2)
        keep = []
        if a.raster:
            f = a.raster
            px, waves = (int(f.split("w")[0]), int(f.split("w")[1])) if "w" in f else (int(f), 4)
            q = c.params(lib, px, keep, waves, 0, 0)
            wgs = (a.batch * c.oh * c.ow + 16 * px - 1) // (16 * px)
        else:
            q = c.params(lib, 4, keep, 4, 0, 1)
            wgs = a.batch * ((c.oh + 7) // 8) * ((c.ow + 7) // 8)
        if lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0:
            continue
        st = DeviceBuffer(wgs * 8 * 8)
        keep.append(st)
        for _ in range(3):
            _abi.check(lib.bh_chain_i8(ctypes.byref(q), None), "chain")
        q.debug_stamps = st.value
        _abi.check(lib.bh_chain_i8(ctypes.byref(q), None), "chain")
        t = st.download(np.uint64, (wgs, 8)).astype(np.int64)
        last = (6 if ce2 else 4) if not a.raster else (5 if ce2 else 3)
        d = np.diff(t[:, :last + 1], axis=1)
        cells = ["%6.0f/%6.0f" % (d[:, k].mean(), np.percentile(d[:, k], 90)) for k in range(last)]
        pro = t[:, 0] - t[:, 7]  # kernel entry -> first stamp: the kernarg prologue
        cells = ["%6.0f/%6.0f" % (pro.mean(), np.percentile(pro, 90))] + cells
        span = t[:, last].max() - t[:, 0].min()
        print("%3dx%-3d ce %4d s%d -> %3d%s -> %4d %5d   %s   span %d clk, start spread %d" % (
            h, h, ce, s, cout, "+res" if res else "    ", ce2, wgs, "  ".join(cells), span,
            t[:, 0].max() - t[:, 0].min()), flush=True)


if __name__ == "__main__":
    main()
