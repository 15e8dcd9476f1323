"""Shared helpers for op-level parity tests: random quantised layers, the
oracle result (oracle/ C restatement of TFLite 2.9.2) and the HIP result
through the C ABI (include/band_hip_kernels.h).
"""
import ctypes

import numpy as np

from oracle import runner as orc


def rand_q(rng, shape, dtype):
    if dtype == np.int8:
        return rng.integers(-128, 128, size=shape, dtype=np.int16).astype(np.int8)
    return rng.integers(0, 256, size=shape, dtype=np.int16).astype(np.uint8)


def dom(zp, dtype):
    """zero point expressed in the kernels' int8 domain"""
    return int(zp) - (0 if np.dtype(dtype) == np.int8 else 128)


def xor_of(dtype):
    return 0 if np.dtype(dtype) == np.int8 else 0x80


class ConvCase:
    def __init__(self, rng, b, ih, iw, ic, oc, kh, kw, stride=(1, 1), dil=(1, 1), same=True,
                 dtype=np.int8, per_channel=True, act=3, depthwise=False, dm=1, requant_fast=None,
                 taps=True, kernel_hint=0):
        self.dtype = dtype
        self.taps = taps
        self.kernel_hint = kernel_hint  # BH_DW_* / BH_CONV_* (0 = the shape's own route)
        self.requant_fast = requant_fast
        self.depthwise = depthwise
        self.dm = dm
        if depthwise:
            oc = ic * dm
        self.x = rand_q(rng, (b, ih, iw, ic), dtype)
        wshape = (1, kh, kw, oc) if depthwise else (oc, kh, kw, ic)
        if dtype == np.int8:
            self.w = rng.integers(-127, 128, size=wshape, dtype=np.int16).astype(np.int8)
            self.w_zp = 0
        else:
            self.w = rand_q(rng, wshape, np.uint8)
            self.w_zp = int(rng.integers(90, 170))
        self.bias = rng.integers(-(1 << 15), 1 << 15, size=oc).astype(np.int32)
        self.in_scale = float(rng.uniform(0.01, 0.05))
        self.in_zp = int(rng.integers(-128, 128)) if dtype == np.int8 else int(rng.integers(0, 256))
        nsc = oc if (per_channel and dtype == np.int8) else 1
        self.w_scales = np.exp(rng.uniform(np.log(1e-3), np.log(2e-2), size=nsc)).astype(np.float32)
        K = kh * kw * (1 if depthwise else ic)
        acc_std = np.sqrt(K) * 74.0 * 74.0
        self.out_scale = float(self.in_scale * float(np.mean(self.w_scales)) * acc_std / 40.0)
        self.out_zp = int(rng.integers(-20, 20)) if dtype == np.int8 else int(rng.integers(100, 156))
        self.stride, self.dil = stride, dil
        self.oh = orc.out_size(same, ih, kh, stride[0], dil[0])
        self.ow = orc.out_size(same, iw, kw, stride[1], dil[1])
        self.pad = (orc.padding(stride[0], dil[0], ih, kh, self.oh),
                    orc.padding(stride[1], dil[1], iw, kw, self.ow))
        legacy = dtype == np.uint8
        self.mult, self.shift = orc.conv_multipliers(self.in_scale, self.w_scales, oc, self.out_scale, legacy)
        self.amin, self.amax = orc.act_range(act, self.out_scale, self.out_zp, dtype == np.int8)
        self.b, self.ih, self.iw, self.ic, self.oc, self.kh, self.kw = b, ih, iw, ic, oc, kh, kw

    def oracle(self):
        kw = dict(in_zp=self.in_zp, w_zp=self.w_zp, out_zp=self.out_zp, mult=self.mult,
                  shift=self.shift, amin=self.amin, amax=self.amax, stride=self.stride,
                  dilation=self.dil, pad=self.pad, out_hw=(self.oh, self.ow))
        if self.depthwise:
            return orc.dwconv2d(self.x, self.w, self.bias, dm=self.dm, **kw)
        return orc.conv2d(self.x, self.w, self.bias, **kw)

    def gpu(self, lib, stream=None):
        keep = []
        p = self.params(lib, keep)
        fn = lib.bh_dwconv2d_i8 if self.depthwise else lib.bh_conv2d_i8
        from band_amd import _abi
        _abi.check(fn(ctypes.byref(p), stream), "bh_dwconv2d_i8" if self.depthwise else "bh_conv2d_i8")
        out = self._dy.download(self.dtype, (self.b, self.oh, self.ow, self.oc))
        del keep
        return out

    def params(self, lib, keep, dx=None, dy=None):
        """C-ABI params on device copies of the case (buffers appended to
        `keep`); dx / dy override the activation buffers (timing chains)."""
        from band_amd import _abi
        from band_amd.device import DeviceBuffer
        out_shape = (self.b, self.oh, self.ow, self.oc)
        if dx is None:
            dx = DeviceBuffer.from_array(self.x)
        if dy is None:
            dy = DeviceBuffer(int(np.prod(out_shape)))
        self._dy = dy
        dmult = DeviceBuffer.from_array(self.mult.astype(np.int32))
        dshift = DeviceBuffer.from_array(self.shift.astype(np.int32))
        keep += [dx, dy, dmult, dshift]
        in_zp_d = dom(self.in_zp, self.dtype)
        w_zp_d = dom(self.w_zp, self.dtype) if self.dtype == np.uint8 else 0
        if self.depthwise:
            wd = self.w.astype(np.int8) if self.dtype == np.int8 else (self.w.view(np.uint8) ^ 0x80).view(np.int8)
            dw = DeviceBuffer.from_array(np.ascontiguousarray(wd))
            db = DeviceBuffer.from_array(self.bias)
            keep += [dw, db]
            p = _abi.DwConvParams(
                batch=self.b, in_h=self.ih, in_w=self.iw, in_c=self.ic, out_h=self.oh, out_w=self.ow,
                out_c=self.oc, depth_multiplier=self.dm, k_h=self.kh, k_w=self.kw,
                stride_h=self.stride[0], stride_w=self.stride[1], dil_h=self.dil[0], dil_w=self.dil[1],
                pad_h=self.pad[0], pad_w=self.pad[1], in_xor=xor_of(self.dtype), in_zp=in_zp_d,
                w_zp=w_zp_d, out_zp=self.out_zp, act_min=self.amin, act_max=self.amax,
                input=dx.value, output=dy.value, weights=dw.value, bias=db.value,
                mult=dmult.value, shift=dshift.value)
            m32 = np.ascontiguousarray(self.mult, np.int32)
            s32 = np.ascontiguousarray(self.shift, np.int32)
            fast = lib.bh_conv_requant_fast_ok(m32.ctypes.data_as(ctypes.c_void_p),
                                               s32.ctypes.data_as(ctypes.c_void_p), self.oc, 9,
                                               int(np.abs(self.bias.astype(np.int64)).max()))
            p.requant_fast = fast if self.requant_fast is None else int(self.requant_fast and fast)
            p.kernel_hint = self.kernel_hint
            # tap table (dot4 kernel) for 3x3 / dm 1 / C % 4 == 0, as the
            # executor lowers it; taps=False keeps the per-tap kernel
            if self.taps and self.kh == 3 and self.kw == 3 and self.dm == 1 and self.oc % 4 == 0:
                taps = np.zeros((self.oc, 4), np.int32)
                wt = np.ascontiguousarray(wd.reshape(9, self.oc))
                bias = np.ascontiguousarray(self.bias, np.int32)
                _abi.check(lib.bh_pack_dw_taps(wt.ctypes.data_as(ctypes.c_void_p), self.oc,
                                               bias.ctypes.data_as(ctypes.c_void_p), in_zp_d, w_zp_d,
                                               taps.ctypes.data_as(ctypes.c_void_p)), "bh_pack_dw_taps")
                dt = DeviceBuffer.from_array(taps)
                keep.append(dt)
                p.taps = dt.value
        else:
            K = self.kh * self.kw * self.ic
            kp, npd = ctypes.c_int(), ctypes.c_int()
            _abi.check(lib.bh_conv_packed_geometry(self.oc, K, ctypes.byref(kp), ctypes.byref(npd)), "geom")
            packed = np.zeros((npd.value, kp.value), np.int8)
            beff = np.zeros(self.oc, np.int32)
            wflat = np.ascontiguousarray(self.w.reshape(self.oc, K))
            _abi.check(lib.bh_pack_conv_weights(
                wflat.ctypes.data_as(ctypes.c_void_p), int(self.dtype == np.int8), self.oc, K,
                kp.value, npd.value, self.bias.ctypes.data_as(ctypes.c_void_p), in_zp_d, w_zp_d,
                packed.ctypes.data_as(ctypes.c_void_p), beff.ctypes.data_as(ctypes.c_void_p)), "pack")
            dw = DeviceBuffer.from_array(packed)
            db = DeviceBuffer.from_array(beff)
            keep += [dw, db]
            p = _abi.ConvParams(
                batch=self.b, in_h=self.ih, in_w=self.iw, in_c=self.ic, out_h=self.oh, out_w=self.ow,
                out_c=self.oc, k_h=self.kh, k_w=self.kw, stride_h=self.stride[0], stride_w=self.stride[1],
                dil_h=self.dil[0], dil_w=self.dil[1], pad_h=self.pad[0], pad_w=self.pad[1],
                k_pad=kp.value, n_pad=npd.value, in_xor=xor_of(self.dtype), in_zp=in_zp_d, w_zp=w_zp_d,
                out_zp=self.out_zp, act_min=self.amin, act_max=self.amax, input=dx.value,
                output=dy.value, weights=dw.value, bias_eff=db.value, mult=dmult.value, shift=dshift.value)
            m32 = np.ascontiguousarray(self.mult, np.int32)
            s32 = np.ascontiguousarray(self.shift, np.int32)
            fast = lib.bh_conv_requant_fast_ok(m32.ctypes.data_as(ctypes.c_void_p),
                                               s32.ctypes.data_as(ctypes.c_void_p), self.oc, K,
                                               int(np.abs(self.bias.astype(np.int64)).max()))
            # requant_fast: None = what the executor would choose, else forced
            p.requant_fast = fast if self.requant_fast is None else int(self.requant_fast and fast)
            p.kernel_hint = self.kernel_hint
        return p


# The 21 distinct MobileNetV2-1.0-224 conv GEMM shapes:
# (spatial, in_c, out_c) for 1x1 layers, batch 1.
MNV2_POINTWISE = [
    (112, 32, 16), (112, 16, 96), (56, 96, 24), (56, 24, 144), (56, 144, 24), (28, 144, 32),
    (28, 32, 192), (28, 192, 32), (14, 192, 64), (14, 64, 384), (14, 384, 64), (14, 384, 96),
    (14, 96, 576), (14, 576, 96), (7, 576, 160), (7, 160, 960), (7, 960, 160), (7, 960, 320),
    (7, 320, 1280), (1, 1280, 1001),
]
# depthwise 3x3 layers: (spatial_in, channels, stride)
MNV2_DEPTHWISE = [
    (112, 32, 1), (112, 96, 2), (56, 144, 1), (56, 144, 2), (28, 192, 1), (28, 192, 2),
    (14, 384, 1), (14, 576, 1), (14, 576, 2), (7, 960, 1),
]
