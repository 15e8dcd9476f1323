#!/usr/bin/env python3
"""Dynamic LDS, registers and resident workgroups per CU of every chain
launch the tuner chose for the batch-24 mix (the MobileNetV2-family and
PoseNet chains of a tune file), with the launch's time.

For each `ch<v>:<ordinal>:<batch>:...` key of the tune file whose choice is
a fused chain, rebuilds the chain (tests/chain_harness.py: random int8
operands of that geometry), asks the library for its dynamic LDS
(bh_chain_lds_bytes), maps the form to the kernel instantiation
bh_chain_i8 launches (fused_chain.hip: bh_chain_i8; chain_tile.hip for the
tile form), reads that instantiation's registers from a
tools/kernel_resources.py table, and derives the workgroups one CU holds at
once: min(waves per SIMD allowed by VGPR+AGPR and by SGPRs / waves per SIMD
of one workgroup, 160 KiB / LDS, 32 waves per CU / waves per workgroup)
(MI355X_MICROARCH.md "Register files", "Residency and cooperative launch").
`rounds` = grid / (256 CUs x resident workgroups): below 1 the launch does
not fill the chip; the launch time is measured here with HIP events.

usage: python tools/chain_occupancy.py --tune profiles/r06s_tune.txt \
         --resources <tools/kernel_resources.py output> [--batch 24]
"""
import argparse
import ctypes
import math
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CUS = 256


def decode(choice):
    """fusion.cc FuseChains: choice code -> form fields"""
    if choice >= 100000:  # kStageChoice + 1000 (stage - 1) + 100 slices + 10 px_blocks + (8 waves)
        c = choice - 100000
        return dict(stage=1 + c // 1000, c_split=(c % 1000) // 100, px_blocks=(c // 10) % 10,
                    waves=8 if c % 10 else 4, deep=0, three=True, persist=0, tile=0, fused=True)
    f = dict(stage=0)
    f["c_split"] = choice // 2000 + 1 if choice >= 2000 else 0
    choice %= 2000
    f["deep"] = int(choice >= 1000)
    choice %= 1000
    f["three"] = choice > 0 and choice % 100 < 10
    f["px_blocks"] = choice % 10
    f["waves"] = 8 if 300 <= choice < 400 else (16 if 100 <= choice < 200 else 4)
    f["persist"] = int(200 <= choice < 300)
    f["tile"] = choice // 100 - 3 if 400 <= choice < 800 else 0
    f["fused"] = choice > 0
    return f


def load_resources(path):
    res = {}
    for line in open(path):
        parts = line.split(None, 9)
        if len(parts) < 10 or not parts[0].isdigit():
            continue
        name = parts[9].strip().replace("void bh::", "")
        res[name] = dict(sgpr=int(parts[0]), vgpr=int(parts[1]), agpr=int(parts[2]), wps=int(parts[8]))
    return res


def instantiation(q, f, fast):
    F = "true" if fast else "false"
    if f["stage"]:
        return "chain_stage_kernel<%d, %s" % (f["px_blocks"], F), f["waves"]
    if f["tile"]:
        return "chain_tile_kernel<8, 8, %s" % F, 4
    k2 = (not q.has_pw2) or q.pw2.k_pad <= 128
    kx = 2 if k2 else 5
    var = 2 if f["c_split"] > 1 else 0
    if f["deep"]:
        rb, nw = (2, 4) if f["px_blocks"] == 2 else (1, f["waves"] if f["waves"] == 8 else 4)
        return "chain_kernel<%d, %s, %d, %d, false, 6, 0>" % (rb, F, kx, nw), nw
    if f["waves"] in (8, 16):
        return "chain_kernel<1, %s, %d, %d, false, 2, %d>" % (F, kx, f["waves"], var), f["waves"]
    t_main = (q.pw2.out_c + 15) // 16 if q.has_pw2 else (q.pw1.out_c + 15) // 16
    if f["px_blocks"] == 4 and k2 and t_main >= 8:
        return "chain_kernel<4, %s, 2, 4, true, 2, %d>" % (F, var), 4
    return "chain_kernel<%d, %s, %d, 4, false, 2, %d>" % (f["px_blocks"], F, kx, var), 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", required=True)
    ap.add_argument("--resources", required=True)
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from band_amd import _abi
    from tests.chain_harness import ChainCase
    lib = _abi.load()
    res = load_resources(a.resources)
    st = ctypes.c_void_p()
    _abi.check(lib.bh_stream_create(ctypes.byref(st)), "stream")
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.bh_event_create(ctypes.byref(e0))
    lib.bh_event_create(ctypes.byref(e1))
    pat = re.compile(r"^ch\d+:0:(\d+):(\d+)x(\d+)x(\d+):s(\d+)d(\d+):(\d+):(\d):(\d+):(\d):f\d+ (\d+)$")
    print("%-40s %-6s %-44s %7s %6s %5s %4s %4s %-14s %6s %8s" % (
        "chain (H, C, stride, cout, res, next)", "form", "instantiation", "LDS KB", "grid", "regs", "w/S", "WG/CU",
        "(limit)", "rounds", "us"))
    seen = set()
    for line in open(a.tune):
        m = pat.match(line.strip())
        if not m or int(m.group(1)) != a.batch:
            continue
        _, h, w, c, s, dil, cout, r, ce2, store, choice = (int(v) for v in m.groups())
        f = decode(choice)
        if not f["fused"] or f["persist"]:
            continue
        nxt = ce2 if f["three"] else 0
        tag = (h, w, c, s, dil, cout, r, nxt, store)
        if tag in seen:
            continue
        seen.add(tag)
        case = ChainCase(np.random.default_rng(1), a.batch, h, w, c, s, cout, bool(r), nxt, dil=dil,
                         store_pw1=bool(store) if f["three"] else True)
        keep = []
        q = case.params(lib, max(f["px_blocks"], 1), keep, f["waves"], 0, f["tile"], f["deep"], f["c_split"],
                        f["stage"])
        lds = lib.bh_chain_lds_bytes(ctypes.byref(q))
        if lds == 0:
            print("%-40s choice %d: not launchable here" % (str(tag), choice))
            continue
        fast = bool(q.dw.requant_fast and q.pw1.requant_fast and (not q.has_pw2 or q.pw2.requant_fast))
        name, nw = instantiation(q, f, fast)
        rr = [v for k, v in res.items() if k.startswith(name)]
        P = a.batch * q.dw.out_h * q.dw.out_w
        if f["tile"]:
            grid = a.batch * math.ceil(q.dw.out_h / 8) * math.ceil(q.dw.out_w / 8)
        else:
            grid = math.ceil(P / (16 * f["px_blocks"])) * max(f["c_split"], 1)
        if rr:
            r0 = rr[0]
            per_simd = math.ceil(nw / 4)
            lim = {"regs": r0["wps"] // per_simd, "LDS": 163840 // lds, "32 waves": 32 // nw}
            wg = min(lim.values())
            limit = min(lim, key=lim.get)
            regs = "%d" % (r0["vgpr"] + r0["agpr"])
            wps = r0["wps"]
        else:
            wg, limit, regs, wps = 0, "?", "?", 0
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
        form = ("t%d" % f["tile"]) if f["tile"] else "%s%d%s%s%s" % (
            "gG"[f["stage"] - 1] if f["stage"] else "", f["px_blocks"], "w%d" % f["waves"] if f["waves"] != 4 else "", "d" if f["deep"] else "",
            "s%d" % f["c_split"] if f["c_split"] > 1 else "")
        label = "%dx%d x%d s%d d%d -> %d%s -> %d" % (h, w, c, s, dil, cout, "+res" if r else "", nxt)
        print("%-40s %-6s %-44s %7.1f %6d %5s %4d %4d %-14s %6.2f %8.2f" % (
            label, form, name.replace("chain_", ""), lds / 1024, grid, regs, wps, wg, "(%s)" % limit,
            grid / (CUS * wg) if wg else 0, us), flush=True)
    lib.bh_event_destroy(e0)
    lib.bh_event_destroy(e1)


if __name__ == "__main__":
    main()
