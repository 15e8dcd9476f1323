"""Random int8 inverted-residual blocks for the fused bh_irb_i8 kernel:
oracle = the 3-4 TFLite ops run one by one (oracle/ C restatement); GPU =
one bh_irb_i8 launch through the C ABI.  Also used by tools/irb_probe.py.
"""
import ctypes

import numpy as np

from oracle import runner as orc

RELU6_SCALE = 6.0 / 255.0

# MobileNetV2-1.0-224 blocks: (H=W of block input, cin, expansion, cout, stride)
MNV2_BLOCKS = [
    (112, 32, 1, 16, 1), (112, 16, 6, 24, 2), (56, 24, 6, 24, 1), (56, 24, 6, 32, 2),
    (28, 32, 6, 32, 1), (28, 32, 6, 64, 2), (14, 64, 6, 64, 1), (14, 64, 6, 96, 1),
    (14, 96, 6, 96, 1), (14, 96, 6, 160, 2), (7, 160, 6, 160, 1), (7, 160, 6, 320, 1),
]


class IrbCase:
    def __init__(self, rng, b, h, w, cin, ce, cout, stride, has_expand=True, residual=None, fast=True):
        self.fast = fast
        self.b, self.h, self.w, self.cin, self.ce, self.cout, self.stride = b, h, w, cin, ce, cout, stride
        self.has_expand = has_expand
        if residual is None:
            residual = stride == 1 and cin == cout
        self.residual = residual
        self.x = rng.integers(-128, 128, (b, h, w, cin)).astype(np.int8)
        self.x_s, self.x_zp = float(rng.uniform(0.02, 0.05)), int(rng.integers(-20, 21))

        def conv_w(oc, ic, k, s_in, s_out, K):
            base = 40.0 * s_out / (s_in * np.sqrt(K) * 45.0 * 73.0)
            ws = (base * np.exp(rng.uniform(-0.4, 0.4, oc))).astype(np.float32)
            w = rng.integers(-127, 128, (oc, k, k, ic)).astype(np.int8)
            bias = rng.integers(-int(np.sqrt(K) * 1000), int(np.sqrt(K) * 1000), oc).astype(np.int32)
            return w, ws, bias

        e_in_s = self.x_s
        if has_expand:
            self.e_s, self.e_zp = RELU6_SCALE, -128
            self.we, self.we_s, self.be = conv_w(ce, cin, 1, self.x_s, self.e_s, cin)
        else:
            assert ce == cin
            self.e_s, self.e_zp = self.x_s, self.x_zp
        e_in_s = self.e_s
        self.d_s, self.d_zp = RELU6_SCALE, -128
        wd, self.wd_s, self.bd = conv_w(ce, 1, 3, e_in_s, self.d_s, 9)
        self.wd = np.ascontiguousarray(wd.reshape(ce, 3, 3).transpose(1, 2, 0).reshape(1, 3, 3, ce))
        self.p_s, self.p_zp = float(self.e_s * rng.uniform(2, 4)), int(rng.integers(-10, 11))
        self.wp, self.wp_s, self.bp = conv_w(cout, ce, 1, self.d_s, self.p_s, ce)
        self.o_s, self.o_zp = float(max(self.p_s, self.x_s) * 1.3), int(rng.integers(-10, 11))

    # --- oracle: ops one by one ------------------------------------------
    def oracle(self):
        x = self.x
        h, w = self.h, self.w
        if self.has_expand:
            m, s = orc.conv_multipliers(self.x_s, self.we_s, self.ce, self.e_s, False)
            lo, hi = orc.act_range(3, self.e_s, self.e_zp, True)
            e = orc.conv2d(x, self.we, self.be, in_zp=self.x_zp, w_zp=0, out_zp=self.e_zp, mult=m, shift=s,
                           amin=lo, amax=hi, out_hw=(h, w))
        else:
            e = x
        oh = orc.out_size(True, h, 3, self.stride, 1)
        ow = orc.out_size(True, w, 3, self.stride, 1)
        ph, pw = orc.padding(self.stride, 1, h, 3, oh), orc.padding(self.stride, 1, w, 3, ow)
        m, s = orc.conv_multipliers(self.e_s, self.wd_s, self.ce, self.d_s, False)
        lo, hi = orc.act_range(3, self.d_s, self.d_zp, True)
        d = orc.dwconv2d(e, self.wd, self.bd, dm=1, in_zp=self.e_zp, w_zp=0, out_zp=self.d_zp, mult=m, shift=s,
                         amin=lo, amax=hi, stride=(self.stride, self.stride), pad=(ph, pw), out_hw=(oh, ow))
        m, s = orc.conv_multipliers(self.d_s, self.wp_s, self.cout, self.p_s, False)
        lo, hi = orc.act_range(0, self.p_s, self.p_zp, True)
        p = orc.conv2d(d, self.wp, self.bp, in_zp=self.d_zp, w_zp=0, out_zp=self.p_zp, mult=m, shift=s,
                       amin=lo, amax=hi, out_hw=(oh, ow))
        if not self.residual:
            return p
        prm = orc.add_params(self.p_s, self.x_s, self.o_s)
        lo, hi = orc.act_range(0, self.o_s, self.o_zp, True)
        return orc.add(p, x, a_zp=self.p_zp, b_zp=self.x_zp, out_zp=self.o_zp, params=prm, amin=lo, amax=hi)

    # --- GPU: one fused launch -------------------------------------------
    def params(self, lib, tile, keep):
        from band_amd import _abi
        from band_amd.device import DeviceBuffer

        def dev(a):
            d = DeviceBuffer.from_array(np.ascontiguousarray(a))
            keep.append(d)
            return d.value

        def pack(w, oc, k, in_zp, ws, s_in, s_out, bias):
            kp, npd = ctypes.c_int(), ctypes.c_int()
            lib.bh_conv_packed_geometry(oc, k, ctypes.byref(kp), ctypes.byref(npd))
            packed = np.zeros((npd.value, kp.value), np.int8)
            beff = np.zeros(oc, np.int32)
            wf = np.ascontiguousarray(w.reshape(oc, k))
            _abi.check(lib.bh_pack_conv_weights(wf.ctypes.data_as(ctypes.c_void_p), 1, oc, k, kp.value, npd.value,
                                                bias.ctypes.data_as(ctypes.c_void_p), in_zp, 0,
                                                packed.ctypes.data_as(ctypes.c_void_p),
                                                beff.ctypes.data_as(ctypes.c_void_p)), "pack")
            m, s = orc.conv_multipliers(s_in, ws, oc, s_out, False)
            return dev(packed), kp.value, dev(beff), dev(m.astype(np.int32)), dev(s.astype(np.int32))

        oh = orc.out_size(True, self.h, 3, self.stride, 1)
        ow = orc.out_size(True, self.w, 3, self.stride, 1)
        q = _abi.IrbParams()
        q.batch, q.in_h, q.in_w, q.in_c, q.exp_c = self.b, self.h, self.w, self.cin, self.ce
        q.out_h, q.out_w, q.out_c, q.stride = oh, ow, self.cout, self.stride
        q.pad_h, q.pad_w = orc.padding(self.stride, 1, self.h, 3, oh), orc.padding(self.stride, 1, self.w, 3, ow)
        q.has_expand = int(self.has_expand)
        q.tile_h = q.tile_w = tile
        if self.has_expand:
            q.exp_w, q.exp_k_pad, q.exp_bias_eff, q.exp_mult, q.exp_shift = pack(
                self.we, self.ce, self.cin, self.x_zp, self.we_s, self.x_s, self.e_s, self.be)
            q.x_zp = self.x_zp
            q.e_act_min, q.e_act_max = orc.act_range(3, self.e_s, self.e_zp, True)
        q.e_zp = self.e_zp
        q.dw_w = dev(self.wd.reshape(-1))
        m, s = orc.conv_multipliers(self.e_s, self.wd_s, self.ce, self.d_s, False)
        q.dw_bias, q.dw_mult, q.dw_shift = dev(self.bd), dev(m.astype(np.int32)), dev(s.astype(np.int32))
        q.d_zp = self.d_zp
        q.d_act_min, q.d_act_max = orc.act_range(3, self.d_s, self.d_zp, True)
        q.proj_w, q.proj_k_pad, q.proj_bias_eff, q.proj_mult, q.proj_shift = pack(
            self.wp, self.cout, self.ce, self.d_zp, self.wp_s, self.d_s, self.p_s, self.bp)
        q.p_zp = self.p_zp
        q.p_act_min, q.p_act_max = orc.act_range(0, self.p_s, self.p_zp, True)
        if self.residual:
            prm = [int(v) for v in orc.add_params(self.p_s, self.x_s, self.o_s)]
            q.has_residual = 1
            q.add_p_off, q.add_x_off, q.add_o_off = -self.p_zp, -self.x_zp, self.o_zp
            q.add_p_mult, q.add_p_shift, q.add_x_mult, q.add_x_shift, q.add_o_mult, q.add_o_shift = prm[:6]
            q.add_left_shift = prm[6]
            q.add_act_min, q.add_act_max = orc.act_range(0, self.o_s, self.o_zp, True)
        # single-step requant per stage, as the executor decides it
        # (fast=False forces the two-step form everywhere)
        def fast_ok(s_in, ws, n, k, s_out, bias):
            m, sh = orc.conv_multipliers(s_in, ws, n, s_out, False)
            m = np.ascontiguousarray(m, np.int32)
            sh = np.ascontiguousarray(sh, np.int32)
            return int(lib.bh_conv_requant_fast_ok(m.ctypes.data_as(ctypes.c_void_p), sh.ctypes.data_as(ctypes.c_void_p),
                                                   n, k, int(np.abs(np.asarray(bias, np.int64)).max())))
        if self.fast:
            q.requant_fast = ((fast_ok(self.x_s, self.we_s, self.ce, self.cin, self.e_s, self.be) if self.has_expand
                               else 0) | (fast_ok(self.e_s, self.wd_s, self.ce, 9, self.d_s, self.bd) << 1) |
                              (fast_ok(self.d_s, self.wp_s, self.cout, self.ce, self.p_s, self.bp) << 2))
        q.input = dev(self.x)
        self.out_shape = (self.b, oh, ow, self.cout)
        from band_amd.device import DeviceBuffer as DB
        out = DB(int(np.prod(self.out_shape)))
        keep.append(out)
        q.output = out.value
        self._out = out
        return q

    def supported(self, lib, tile):
        keep = []
        return lib.bh_irb_lds_bytes(ctypes.byref(self.params(lib, tile, keep))) > 0

    def gpu(self, lib, tile):
        from band_amd import _abi
        keep = []
        q = self.params(lib, tile, keep)
        assert lib.bh_irb_lds_bytes(ctypes.byref(q)) > 0, "tile %d unsupported" % tile
        _abi.check(lib.bh_irb_i8(ctypes.byref(q), None), "bh_irb_i8")
        return self._out.download(np.int8, self.out_shape)
