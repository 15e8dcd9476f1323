#!/usr/bin/env python3
"""Per-phase timing of the fused inverted-residual kernel (bh_irb_i8).

For each MobileNetV2 block shape and tile size, runs the kernel with
debug_stamps set and prints the mean / max (over workgroups) time spent in
each phase (s_memrealtime, 100 MHz), plus the event-timed kernel duration.
Diagnostic only.
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    from tests.irb_harness import MNV2_BLOCKS, IrbCase
    lib = _abi.load()
    ev0, ev1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.bh_event_create(ctypes.byref(ev0))
    lib.bh_event_create(ctypes.byref(ev1))
    s = ctypes.c_void_p()
    lib.bh_stream_create(ctypes.byref(s))
    names = ["pre+p0", "p1 expand", "p2 dw", "zero", "p3 proj", "p4 epi"]
    tiles = [int(t) for t in (sys.argv[1].split(",") if len(sys.argv) > 1 else "1,2,4,7,8".split(","))]
    for (h, cin, t, cout, st) in MNV2_BLOCKS:
        c = IrbCase(np.random.default_rng(0), 1, h, h, cin, cin * t, cout, st, has_expand=t != 1)
        for tile in tiles:
            keep = []
            q = c.params(lib, tile, keep)
            lds = lib.bh_irb_lds_bytes(ctypes.byref(q))
            if lds == 0:
                continue
            oh, ow = c.out_shape[1], c.out_shape[2]
            nwg = ((oh + tile - 1) // tile) * ((ow + tile - 1) // tile)
            stamps = DeviceBuffer(nwg * 16 * 8)
            # timing without stamps
            for _ in range(3):
                lib.bh_irb_i8(ctypes.byref(q), s)
            lib.bh_event_record(ev0, s)
            n = 20
            for _ in range(n):
                lib.bh_irb_i8(ctypes.byref(q), s)
            lib.bh_event_record(ev1, s)
            lib.bh_stream_sync(s)
            ms = ctypes.c_float()
            lib.bh_event_elapsed_ms(ev0, ev1, ctypes.byref(ms))
            q.debug_stamps = stamps.value
            lib.bh_irb_i8(ctypes.byref(q), s)
            lib.bh_stream_sync(s)
            st16 = stamps.download(np.uint64, (nwg, 16)).astype(np.float64)
            st_ = st16[:, :8]
            d = np.diff(st_[:, :7], axis=1) * 0.01  # 100 MHz ticks -> us
            span = (st_[:, 6].max() - st_[:, 0].min()) * 0.01
            clk = np.median(st_[:, 7] / np.maximum((st_[:, 6] - st_[:, 0]) * 0.01, 1e-3)) / 1e3  # GHz
            print("blk %3d %3d->%4d->%3d s%d tile %d wg %4d lds %6d  kernel %6.2f us  wg-span %6.2f clk %.2fGHz " % (
                h, cin, cin * t, cout, st, tile, nwg, lds, ms.value * 1e3 / n, span, clk) +
                " ".join("%s %.2f/%.2f" % (nm, d[:, i].mean(), d[:, i].max()) for i, nm in enumerate(names)))
            # wave-0 cycle stamps (s_memtime): phase-1 start 11, item0 weights ready 8,
            # MFMA done 9, requant+stores done 10; phase-2 start 12, taps done 13,
            # requant+store done 14; end 15
            c = st16[0]
            if c[11] > 0:
                print("    cycles: p1 start->w %d, w->mfma %d, mfma->req+st %d | p2 start->taps %d, taps->req+st %d | p1 start->end %d" % (
                    c[8] - c[11], c[9] - c[8], c[10] - c[9], c[13] - c[12], c[14] - c[13], c[15] - c[11]))
            sys.stdout.flush()


if __name__ == "__main__":
    main()
