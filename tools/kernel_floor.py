#!/usr/bin/env python3
"""Per-launch device time of single MobileNetV2 layers inside dependent
hipGraph chains (each launch reads what the previous one wrote), next to the
same chain issued eagerly.  Compare with tools/launch_probe (an empty /
trivial kernel's floor) to see how much of a layer's time is the kernel
itself.  Diagnostic only; random data.
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    from tests.irb_harness import IrbCase
    from tests.kernel_harness import ConvCase
    lib = _abi.load()
    s = ctypes.c_void_p()
    lib.bh_stream_create(ctypes.byref(s))
    ev0, ev1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.bh_event_create(ctypes.byref(ev0))
    lib.bh_event_create(ctypes.byref(ev1))
    N = 40
    rng = np.random.default_rng(0)

    def chain(name, make, nbytes):
        a, b = DeviceBuffer(nbytes), DeviceBuffer(nbytes)
        keep = [a, b]
        calls = [make(a if i % 2 == 0 else b, b if i % 2 == 0 else a, keep) for i in range(2)]
        res = {}
        for mode in ("stream", "graph"):
            g = ctypes.c_void_p()
            if mode == "graph":
                _abi.check(lib.bh_capture_begin(s), "capture")
                for i in range(N):
                    calls[i % 2]()
                _abi.check(lib.bh_capture_end(s, ctypes.byref(g)), "capture end")
            best = 1e30
            for _ in range(5):
                lib.bh_event_record(ev0, s)
                if mode == "graph":
                    lib.bh_graph_launch(g, s)
                else:
                    for i in range(N):
                        calls[i % 2]()
                lib.bh_event_record(ev1, s)
                lib.bh_stream_sync(s)
                ms = ctypes.c_float()
                lib.bh_event_elapsed_ms(ev0, ev1, ctypes.byref(ms))
                best = min(best, ms.value)
            res[mode] = best * 1e3 / N
            if mode == "graph":
                lib.bh_graph_destroy(g)
        print("%-40s stream %6.2f us  graph %6.2f us" % (name, res["stream"], res["graph"]))
        sys.stdout.flush()

    def conv(h, ic, oc, k=1, stride=1, dw=False):
        c = ConvCase(rng, 1, h, h, ic, oc, k, k, stride=(stride, stride), depthwise=dw)
        fn = lib.bh_dwconv2d_i8 if dw else lib.bh_conv2d_i8

        def make(x, y, keep):
            p = c.params(lib, keep, dx=x, dy=y)
            keep.append(p)
            return lambda: _abi.check(fn(ctypes.byref(p), s), "launch")
        nb = max(h * h * ic, c.oh * c.ow * c.oc)
        chain("%s %dx%dx%d -> %d k%d s%d" % ("dw" if dw else "conv", h, h, ic, c.oc, k, stride), make, nb)

    def irb(h, cin, t, cout, st, tile):
        c = IrbCase(rng, 1, h, h, cin, cin * t, cout, st, has_expand=t != 1)

        def make(x, y, keep):
            q = c.params(lib, tile, keep)
            q.input, q.output = x.value, y.value
            keep.append(q)
            return lambda: _abi.check(lib.bh_irb_i8(ctypes.byref(q), s), "irb")
        chain("irb %dx%dx%d->%d->%d s%d tile %d" % (h, h, cin, cin * t, cout, st, tile), make,
              max(h * h * cin, (h // st) ** 2 * cout))

    # code switching: alternate two different kernels; cold weights: rotate
    # 16 copies of one layer's weights
    c1 = ConvCase(rng, 1, 7, 7, 160, 960, 1, 1)
    c2 = ConvCase(rng, 1, 7, 7, 960, 960, 3, 3, depthwise=True)
    c3 = ConvCase(rng, 1, 7, 7, 960, 160, 1, 1)

    def make_alt(x, y, keep):
        p1 = c1.params(lib, keep, dx=x, dy=y)
        p2 = c2.params(lib, keep, dx=y, dy=x)
        p3 = c3.params(lib, keep, dx=x, dy=y)
        keep += [p1, p2, p3]
        return lambda: (_abi.check(lib.bh_conv2d_i8(ctypes.byref(p1), s), "c1"),
                        _abi.check(lib.bh_dwconv2d_i8(ctypes.byref(p2), s), "c2"),
                        _abi.check(lib.bh_conv2d_i8(ctypes.byref(p3), s), "c3"))
    chain("3 launches: conv160->960, dw960, conv960->160", make_alt, 7 * 7 * 960)

    copies = [ConvCase(rng, 1, 7, 7, 960, 160, 1, 1) for _ in range(16)]
    rot = [0]

    def make_rot(x, y, keep):
        ps = [c.params(lib, keep, dx=x, dy=y) for c in copies]
        keep += ps

        def call():
            rot[0] = (rot[0] + 1) % len(ps)
            _abi.check(lib.bh_conv2d_i8(ctypes.byref(ps[rot[0]]), s), "rot")
        return call
    chain("conv 7x7x960->160, 16 weight copies", make_rot, 7 * 7 * 960)

    conv(224, 3, 32, k=3, stride=2)
    conv(112, 32, 32, k=3, dw=True)
    conv(112, 32, 16)
    conv(56, 144, 144, k=3, dw=True)
    conv(56, 24, 144)
    conv(28, 192, 192, k=3, dw=True)
    conv(14, 576, 576, k=3, dw=True)
    conv(14, 64, 384)
    conv(14, 384, 64)
    conv(7, 960, 960, k=3, dw=True)
    conv(7, 160, 960)
    conv(7, 960, 160)
    conv(7, 320, 1280)
    irb(14, 64, 6, 64, 1, 1)
    irb(28, 32, 6, 32, 1, 1)
    irb(28, 32, 6, 32, 1, 2)
    irb(56, 24, 6, 24, 1, 2)

    # global average pool 7x7x1280 and the classifier GEMV
    def make_pool(x, y, keep):
        p = _abi.PoolParams(kind=0, in_signed=1, batch=1, in_h=7, in_w=7, channels=1280, out_h=1, out_w=1,
                            f_h=7, f_w=7, stride_h=1, stride_w=1, pad_h=0, pad_w=0, act_min=-128, act_max=127,
                            input=x.value, output=y.value)
        keep.append(p)
        return lambda: _abi.check(lib.bh_pool_i8(ctypes.byref(p), s), "pool")
    chain("avgpool 7x7x1280", make_pool, 7 * 7 * 1280)

    w = DeviceBuffer.from_array(rng.integers(-127, 128, (1001, 1280)).astype(np.int8))
    tb = DeviceBuffer.from_array(np.ones(1001, np.int32))

    def make_fc(x, y, keep):
        p = _abi.FcParams(rows=1, depth=1280, depth_pad=1280, units=1001, in_xor=0, in_zp=0, w_zp=0, out_zp=0,
                          act_min=-128, act_max=127, input=x.value, output=y.value, weights=w.value,
                          bias_eff=tb.value, mult=tb.value, shift=tb.value)
        keep.append(p)
        return lambda: _abi.check(lib.bh_fc_i8(ctypes.byref(p), s), "fc")
    chain("fc 1280 -> 1001", make_fc, 1280)


if __name__ == "__main__":
    main()
