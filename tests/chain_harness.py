"""Random int8 depthwise -> 1x1 [-> ADD] [-> 1x1] chains for the fused
bh_chain_i8 kernel: oracle = the 2-4 TFLite ops run one by one (oracle/ C
restatement of TFLite 2.9.2); GPU = one bh_chain_i8 launch through the C ABI.
"""
import ctypes

import numpy as np

from oracle import runner as orc

RELU6_SCALE = 6.0 / 255.0

# MobileNetV2-1.0-224 chains: (H=W of the depthwise input, expanded channels,
# stride, project channels, residual, next expand channels or 0)
MNV2_CHAINS = [
    (112, 32, 1, 16, False, 96), (112, 96, 2, 24, False, 144), (56, 144, 1, 24, True, 144),
    (56, 144, 2, 32, False, 192), (28, 192, 1, 32, True, 192), (28, 192, 2, 64, False, 384),
    (14, 384, 1, 64, True, 384), (14, 384, 1, 96, False, 576), (14, 576, 1, 96, True, 576),
    (14, 576, 2, 160, False, 960), (7, 960, 1, 160, True, 960), (7, 960, 1, 320, False, 1280),
]


class ChainCase:
    def __init__(self, rng, b, h, w, ce, stride, cout, residual, ce2, dil=1, store_pw1=None, fast=True):
        self.b, self.h, self.w, self.ce, self.stride, self.dil = b, h, w, ce, stride, dil
        self.cout, self.residual, self.ce2, self.fast = cout, residual, ce2, fast
        # the first conv's result goes to HBM when something else reads it
        self.store_pw1 = (residual or not ce2) if store_pw1 is None else store_pw1
        self.oh = orc.out_size(True, h, 3, stride, dil)
        self.ow = orc.out_size(True, w, 3, stride, dil)
        self.pad = (orc.padding(stride, dil, h, 3, self.oh), orc.padding(stride, dil, w, 3, self.ow))
        self.e = rng.integers(-128, 128, (b, h, w, ce)).astype(np.int8)
        self.e_s, self.e_zp = RELU6_SCALE, -128 if rng.random() < 0.7 else int(rng.integers(-30, 30))

        def conv_w(oc, ic, k, s_in, s_out, K):
            base = 40.0 * s_out / (s_in * np.sqrt(K) * 45.0 * 73.0)
            ws = (base * np.exp(rng.uniform(-0.4, 0.4, oc))).astype(np.float32)
            w = rng.integers(-127, 128, (oc, k, k, ic)).astype(np.int8)
            bias = rng.integers(-int(np.sqrt(K) * 1000), int(np.sqrt(K) * 1000), oc).astype(np.int32)
            return w, ws, bias

        self.d_s, self.d_zp = RELU6_SCALE, -128
        wd, self.wd_s, self.bd = conv_w(ce, 1, 3, self.e_s, self.d_s, 9)
        self.wd = np.ascontiguousarray(wd.reshape(ce, 3, 3).transpose(1, 2, 0).reshape(1, 3, 3, ce))
        self.p_s, self.p_zp = float(self.e_s * rng.uniform(2, 4)), int(rng.integers(-10, 11))
        self.wp, self.wp_s, self.bp = conv_w(cout, ce, 1, self.d_s, self.p_s, ce)
        if residual:
            self.x = rng.integers(-128, 128, (b, self.oh, self.ow, cout)).astype(np.int8)
            self.x_s, self.x_zp = float(self.p_s * rng.uniform(0.7, 1.3)), int(rng.integers(-10, 11))
            self.o_s, self.o_zp = float(max(self.p_s, self.x_s) * 1.3), int(rng.integers(-10, 11))
            y_s = self.o_s
        else:
            y_s = self.p_s
        self.y_s = y_s
        if ce2:
            self.f_s, self.f_zp = RELU6_SCALE, -128
            self.wf, self.wf_s, self.bf = conv_w(ce2, cout, 1, y_s, self.f_s, cout)

    # --- oracle: ops one by one ------------------------------------------
    def oracle(self):
        m, s = orc.conv_multipliers(self.e_s, self.wd_s, self.ce, self.d_s, False)
        lo, hi = orc.act_range(3, self.d_s, self.d_zp, True)
        d = orc.dwconv2d(self.e, self.wd, self.bd, dm=1, in_zp=self.e_zp, w_zp=0, out_zp=self.d_zp, mult=m, shift=s,
                         amin=lo, amax=hi, stride=(self.stride, self.stride), dilation=(self.dil, self.dil),
                         pad=self.pad, out_hw=(self.oh, self.ow))
        m, s = orc.conv_multipliers(self.d_s, self.wp_s, self.cout, self.p_s, False)
        lo, hi = orc.act_range(0, self.p_s, self.p_zp, True)
        y = orc.conv2d(d, self.wp, self.bp, in_zp=self.d_zp, w_zp=0, out_zp=self.p_zp, mult=m, shift=s,
                       amin=lo, amax=hi, out_hw=(self.oh, self.ow))
        y_zp = self.p_zp
        if self.residual:
            prm = orc.add_params(self.p_s, self.x_s, self.o_s)
            lo, hi = orc.act_range(0, self.o_s, self.o_zp, True)
            y = orc.add(y, self.x, a_zp=self.p_zp, b_zp=self.x_zp, out_zp=self.o_zp, params=prm, amin=lo, amax=hi)
            y_zp = self.o_zp
        if not self.ce2:
            return y, None
        m, s = orc.conv_multipliers(self.y_s, self.wf_s, self.ce2, self.f_s, False)
        lo, hi = orc.act_range(3, self.f_s, self.f_zp, True)
        f = orc.conv2d(y, self.wf, self.bf, in_zp=y_zp, w_zp=0, out_zp=self.f_zp, mult=m, shift=s,
                       amin=lo, amax=hi, out_hw=(self.oh, self.ow))
        return y, f

    # --- GPU: one fused launch -------------------------------------------
    def params(self, lib, px_blocks, keep, waves=4, persist=0, tile=0, deep=0, c_split=0, stage=0):
        from band_amd import _abi
        from band_amd.device import DeviceBuffer

        def dev(a):
            d = DeviceBuffer.from_array(np.ascontiguousarray(a))
            keep.append(d)
            return d.value

        def fast_ok(m, sh, n, k, bias):
            m = np.ascontiguousarray(m, np.int32)
            sh = np.ascontiguousarray(sh, np.int32)
            if not self.fast:
                return 0
            return int(lib.bh_conv_requant_fast_ok(m.ctypes.data_as(ctypes.c_void_p), sh.ctypes.data_as(ctypes.c_void_p),
                                                   n, k, int(np.abs(np.asarray(bias, np.int64)).max())))

        def conv(w, oc, k, in_zp, ws, s_in, s_out, bias, out_zp, act):
            q = _abi.ConvParams()
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
            q.batch, q.in_h, q.in_w, q.in_c = self.b, self.oh, self.ow, k
            q.out_h, q.out_w, q.out_c = self.oh, self.ow, oc
            q.k_h = q.k_w = q.stride_h = q.stride_w = q.dil_h = q.dil_w = 1
            q.k_pad, q.n_pad = kp.value, npd.value
            q.in_zp, q.w_zp, q.out_zp = in_zp, 0, out_zp
            q.act_min, q.act_max = orc.act_range(act, s_out, out_zp, True)
            q.weights, q.bias_eff = dev(packed), dev(beff)
            q.mult, q.shift = dev(m.astype(np.int32)), dev(s.astype(np.int32))
            q.requant_fast = fast_ok(m, s, oc, k, bias)
            return q

        c = _abi.ChainParams()
        d = c.dw
        d.batch, d.in_h, d.in_w, d.in_c = self.b, self.h, self.w, self.ce
        d.out_h, d.out_w, d.out_c, d.depth_multiplier = self.oh, self.ow, self.ce, 1
        d.k_h = d.k_w = 3
        d.stride_h = d.stride_w = self.stride
        d.dil_h = d.dil_w = self.dil
        d.pad_h, d.pad_w = self.pad
        d.in_zp, d.w_zp, d.out_zp = self.e_zp, 0, self.d_zp
        d.act_min, d.act_max = orc.act_range(3, self.d_s, self.d_zp, True)
        wdr = np.ascontiguousarray(self.wd.reshape(-1))
        m, s = orc.conv_multipliers(self.e_s, self.wd_s, self.ce, self.d_s, False)
        taps = np.zeros((self.ce, 4), np.int32)
        _abi.check(lib.bh_pack_dw_taps(wdr.ctypes.data_as(ctypes.c_void_p), self.ce,
                                       self.bd.ctypes.data_as(ctypes.c_void_p), self.e_zp, 0,
                                       taps.ctypes.data_as(ctypes.c_void_p)), "taps")
        d.input, d.weights, d.bias = dev(self.e), dev(wdr), dev(self.bd)
        d.mult, d.shift, d.taps = dev(m.astype(np.int32)), dev(s.astype(np.int32)), dev(taps)
        d.requant_fast = fast_ok(m, s, self.ce, 9, self.bd)
        c.pw1 = conv(self.wp, self.cout, self.ce, self.d_zp, self.wp_s, self.d_s, self.p_s, self.bp, self.p_zp, 0)
        y_zp = self.p_zp
        if self.residual:
            a = c.pw1
            prm = [int(v) for v in orc.add_params(self.p_s, self.x_s, self.o_s)]
            a.residual = dev(self.x)
            a.add_y_off, a.add_r_off, a.add_o_off = -self.p_zp, -self.x_zp, self.o_zp
            a.add_y_mult, a.add_y_shift, a.add_r_mult, a.add_r_shift, a.add_o_mult, a.add_o_shift = prm[:6]
            a.add_left_shift = prm[6]
            a.add_act_min, a.add_act_max = orc.act_range(0, self.o_s, self.o_zp, True)
            y_zp = self.o_zp
        from band_amd.device import DeviceBuffer as DB
        px = self.b * self.oh * self.ow
        self._y = self._f = None
        if self.store_pw1:
            self._y = DB(px * self.cout)
            keep.append(self._y)
            c.pw1.output = self._y.value
        if self.ce2:
            c.has_pw2 = 1
            c.pw2 = conv(self.wf, self.ce2, self.cout, y_zp, self.wf_s, self.y_s, self.f_s, self.bf, self.f_zp, 3)
            self._f = DB(px * self.ce2)
            keep.append(self._f)
            c.pw2.output = self._f.value
        c.px_blocks = px_blocks
        c.waves = waves
        c.persist = persist
        c.tile = tile
        c.deep = deep
        c.c_split = c_split
        c.stage = stage
        if tile or stage:
            nb = lib.bh_chain_tile_blob_bytes(ctypes.byref(c))
            if nb:
                blob = DB(nb)
                keep.append(blob)
                _abi.check(lib.bh_chain_tile_pack(ctypes.byref(c), blob.value, None), "bh_chain_tile_pack")
                c.tile_blob = blob.value
        return c

    def gpu(self, lib, px_blocks, waves=4, persist=0, tile=0, deep=0, c_split=0, stage=0):
        from band_amd import _abi
        keep = []
        c = self.params(lib, px_blocks, keep, waves, persist, tile, deep, c_split, stage)
        assert lib.bh_chain_lds_bytes(ctypes.byref(c)) > 0, "chain unsupported"
        _abi.check(lib.bh_chain_i8(ctypes.byref(c), None), "bh_chain_i8")
        y = self._y.download(np.int8, (self.b, self.oh, self.ow, self.cout)) if self._y else None
        f = self._f.download(np.int8, (self.b, self.oh, self.ow, self.ce2)) if self._f else None
        return y, f
