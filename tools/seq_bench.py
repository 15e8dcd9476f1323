#!/usr/bin/env python3
"""Timing of the image-resident chain sequence (bh_chain_seq_i8) against the
same chains launched one by one (bh_chain_i8, a given raster form), on random
MobileNetV2-shaped runs.  usage: tools/seq_bench.py [--batch 1] [--iters 200]
[--runs 6,6,6,7,8,8,9,10,10,11:8,8:...]  (indices into MNV2_CHAINS)"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--runs", default="6,6,6,7,8,8,9,10,10,11:6,6,6,7:8,8,9:10,10,11")
    ap.add_argument("--forms", default="1w16,1w8s2,1w16s2", help="per-chain raster forms to compare (chain_bench syntax)")
    a = ap.parse_args()
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    from tests.test_chain_seq_gpu import build_run, mnv2
    lib = _abi.load()
    st = ctypes.c_void_p()
    _abi.check(lib.bh_stream_create(ctypes.byref(st)), "stream")
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.bh_event_create(ctypes.byref(e0))
    lib.bh_event_create(ctypes.byref(e1))

    def timed(fn):
        for _ in range(3):
            fn()
        lib.bh_spin_us(st, 300 + 40 * a.iters)
        lib.bh_event_record(e0, st)
        for _ in range(a.iters):
            fn()
        lib.bh_event_record(e1, st)
        lib.bh_stream_sync(st)
        ms = ctypes.c_float()
        lib.bh_event_elapsed_ms(e0, e1, ctypes.byref(ms))
        return 1e3 * ms.value / a.iters

    for run in a.runs.split(":"):
        idx = [int(v) for v in run.split(",")]
        cases = build_run(np.random.default_rng(1), a.batch, mnv2(idx))
        keep = []
        ps = [c.params(lib, 1, keep) for c in cases]
        for k in range(1, len(ps)):
            ps[k].dw.input = ps[k - 1].pw2.output
            if cases[k].residual:
                ps[k].pw1.residual = ps[k - 1].pw1.output
        n = len(ps)
        arr = (_abi.ChainParams * n)(*ps)
        row = "run %-32s b%-3d" % (run, a.batch)
        if lib.bh_chain_seq_lds_bytes(arr, n):
            host = ctypes.create_string_buffer(lib.bh_chain_seq_table_bytes())
            _abi.check(lib.bh_chain_seq_plan(arr, n, host), "plan")
            table = DeviceBuffer.from_array(np.frombuffer(host.raw, np.uint8))
            keep.append(table)
            us = timed(lambda: lib.bh_chain_seq_i8(arr, table.value, n, st))
            row += " seq %8.2f us" % us
        else:
            row += " seq   (unsupported)"
        for form in a.forms.split(","):
            split = int(form.split("s")[1]) if "s" in form else 0
            f = form.split("s")[0]
            px, waves = (int(f.split("w")[0]), int(f.split("w")[1])) if "w" in f else (int(f), 4)
            qs = []
            for k, p in enumerate(ps):
                q = _abi.ChainParams.from_buffer_copy(p)
                q.px_blocks, q.waves, q.c_split = px, waves, split
                if lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0:
                    q.c_split = 0
                if lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0:
                    q.px_blocks, q.waves = 1, 4
                qs.append(q)

            def chain_all():
                for q in qs:
                    lib.bh_chain_i8(ctypes.byref(q), st)
            row += "  %s %8.2f" % (form, timed(chain_all))
        print(row, flush=True)
    lib.bh_event_destroy(e0)
    lib.bh_event_destroy(e1)


if __name__ == "__main__":
    main()
