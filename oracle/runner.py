"""ORACLE — test infrastructure only.

Whole-model CPU runner restating what `tflite::Interpreter::Invoke` computes
for the op set on Band's hot path (`band/backend/tfl/model_executor.cc:249-255`
-> TFLite 2.9.2 builtin kernels).  The op-level Prepare logic (quantisation
parameter derivation) mirrors TFLite 2.9.2's `kernels/{conv,depthwise_conv,
fully_connected,add,sub,mul,pooling,reshape}.cc`; the arithmetic runs in the C
restatement `oracle/tflite_ref.c` (loaded via ctypes from `liboracle.so`).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module.  It is never on the product path.
"""
import ctypes
import os

import numpy as np

from .tflite_fb import Model, OP

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

P_U8 = ctypes.POINTER(ctypes.c_uint8)
P_I32 = ctypes.POINTER(ctypes.c_int32)
P_F32 = ctypes.POINTER(ctypes.c_float)


def build():
    """Compile liboracle.so with the committed Makefile (gcc)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.tfl_set_num_threads.argtypes = [ctypes.c_int]
        L.tfl_srdhm.restype = ctypes.c_int32
        L.tfl_srdhm.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.tfl_rdbypot.restype = ctypes.c_int32
        L.tfl_rdbypot.argtypes = [ctypes.c_int32, ctypes.c_int]
        L.tfl_mbqm.restype = ctypes.c_int32
        L.tfl_mbqm.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int]
        L.tfl_quantize_multiplier.argtypes = [ctypes.c_double, P_I32, ctypes.POINTER(ctypes.c_int)]
        L.tfl_act_range_quantized.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_int32,
                                              ctypes.c_int, P_I32, P_I32]
        L.tfl_conv_multipliers.argtypes = [ctypes.c_float, P_F32, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_float, ctypes.c_int, P_I32, P_I32]
        L.tfl_add_params.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float, P_I32]
        L.tfl_mul_params.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float, P_I32, P_I32]
        L.tfl_out_size.restype = ctypes.c_int
        L.tfl_padding.restype = ctypes.c_int
        c_i, c_l, c_f, c_i32, vp = ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_int32, ctypes.c_void_p
        L.tfl_requantize.argtypes = [vp, c_i, c_l, c_i32, c_i32, c_i, c_i, c_i32, vp]
        L.tfl_quantize_f32.argtypes = [vp, c_l, c_f, c_i32, c_i, vp]
        L.tfl_dequantize.argtypes = [vp, c_i, c_l, c_f, c_i32, vp]
        L.tfl_relu_params.argtypes = [c_f, c_f, c_i32, c_i, c_f, c_f, c_i, P_I32, P_I32, P_I32, P_I32]
        L.tfl_relu_x.argtypes = [vp, c_i, c_l, c_i32, c_i32, c_i32, c_i, c_i32, c_i32, vp]
        L.tfl_logistic_table.argtypes = [c_f, c_i32, c_f, c_i32, c_i, vp]
        L.tfl_lookup.argtypes = [vp, c_l, vp, vp]
        L.tfl_hard_swish.restype = c_i
        L.tfl_hard_swish.argtypes = [vp, c_i, c_l, c_f, c_i32, c_f, c_i32, vp]
        L.tfl_softmax.argtypes = [vp, c_i, c_l, c_i, c_f, c_f, c_f, c_i32, vp]
        L.tfl_softmax_table.argtypes = [c_f, c_f, vp]
        L.tfl_transpose_conv_i8.argtypes = [vp, c_i, c_i, c_i, c_i, vp, c_i, c_i, c_i, vp, vp, c_i, c_i, c_i, c_i,
                                            c_i, c_i, c_i32, c_i32, vp, vp]
        L.tfl_concat.argtypes = [c_i, ctypes.POINTER(vp), P_I32, c_l, c_l, P_F32, P_I32, c_f, c_i32, c_i, vp]
        L.tfl_pad.argtypes = [vp, P_I32, P_I32, ctypes.c_uint8, vp]
        L.tfl_nearest_index.restype = c_i
        L.tfl_nearest_index.argtypes = [c_i, c_i, c_i, c_i, c_i]
        L.tfl_resize_nearest.argtypes = [vp, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, vp]
        L.tfl_resize_bilinear_i8.argtypes = [vp, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, vp]
        L.tfl_resize_bilinear_u8.argtypes = [vp, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, vp]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def quantize_multiplier(m):
    q = ctypes.c_int32()
    s = ctypes.c_int()
    lib().tfl_quantize_multiplier(float(m), ctypes.byref(q), ctypes.byref(s))
    return q.value, s.value


def act_range(act, scale, zp, signed):
    lo = ctypes.c_int32()
    hi = ctypes.c_int32()
    lib().tfl_act_range_quantized(int(act), float(scale), int(zp), int(signed),
                                  ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


def conv_multipliers(in_scale, w_scales, n_channels, out_scale, legacy):
    w = np.ascontiguousarray(np.asarray(w_scales, np.float32))
    mult = np.zeros(n_channels, np.int32)
    shift = np.zeros(n_channels, np.int32)
    lib().tfl_conv_multipliers(float(in_scale), _p(w, P_F32), len(w), n_channels,
                               float(out_scale), int(legacy), _p(mult, P_I32), _p(shift, P_I32))
    return mult, shift


def out_size(same, n, f, s, d):
    return lib().tfl_out_size(int(same), n, f, s, d)


def padding(s, d, n, f, o):
    return lib().tfl_padding(s, d, n, f, o)


def _u8(a):
    return np.ascontiguousarray(a).view(np.uint8)


def _signed(dt):
    return 1 if np.dtype(dt) == np.int8 else 0


def conv2d(x, w, bias, *, in_zp, w_zp, out_zp, mult, shift, amin, amax,
           stride=(1, 1), dilation=(1, 1), pad=(0, 0), out_hw=None, out_dtype=None):
    """x NHWC, w OHWI; returns NHWC output (dtype of x unless out_dtype)."""
    b, ih, iw, ic = x.shape
    oc, kh, kw, _ = w.shape
    oh, ow = out_hw
    out = np.zeros((b, oh, ow, oc), out_dtype or x.dtype)
    bias = None if bias is None else np.ascontiguousarray(bias, np.int32)
    mult = np.ascontiguousarray(mult, np.int32)
    shift = np.ascontiguousarray(shift, np.int32)
    lib().tfl_conv2d(_p(_u8(x), P_U8), _signed(x.dtype), b, ih, iw, ic,
                     _p(_u8(w), P_U8), _signed(w.dtype), oc, kh, kw,
                     None if bias is None else _p(bias, P_I32), _p(out.view(np.uint8), P_U8),
                     oh, ow, stride[0], stride[1], dilation[0], dilation[1], pad[0], pad[1],
                     ctypes.c_int32(-in_zp), ctypes.c_int32(-w_zp), ctypes.c_int32(out_zp),
                     _p(mult, P_I32), _p(shift, P_I32), ctypes.c_int32(amin), ctypes.c_int32(amax))
    return out


def dwconv2d(x, w, bias, *, dm, in_zp, w_zp, out_zp, mult, shift, amin, amax,
             stride=(1, 1), dilation=(1, 1), pad=(0, 0), out_hw=None):
    b, ih, iw, ic = x.shape
    _, kh, kw, oc = w.shape
    oh, ow = out_hw
    out = np.zeros((b, oh, ow, oc), x.dtype)
    bias = None if bias is None else np.ascontiguousarray(bias, np.int32)
    mult = np.ascontiguousarray(mult, np.int32)
    shift = np.ascontiguousarray(shift, np.int32)
    lib().tfl_dwconv2d(_p(_u8(x), P_U8), _signed(x.dtype), b, ih, iw, ic,
                       _p(_u8(w), P_U8), _signed(w.dtype), dm, kh, kw,
                       None if bias is None else _p(bias, P_I32), _p(out.view(np.uint8), P_U8),
                       oh, ow, stride[0], stride[1], dilation[0], dilation[1], pad[0], pad[1],
                       ctypes.c_int32(-in_zp), ctypes.c_int32(-w_zp), ctypes.c_int32(out_zp),
                       _p(mult, P_I32), _p(shift, P_I32), ctypes.c_int32(amin), ctypes.c_int32(amax))
    return out


def fully_connected(x2d, w, bias, *, in_zp, w_zp, out_zp, mult, shift, amin, amax):
    rows, depth = x2d.shape
    units = w.shape[0]
    out = np.zeros((rows, units), x2d.dtype)
    bias = None if bias is None else np.ascontiguousarray(bias, np.int32)
    mult = np.ascontiguousarray(np.broadcast_to(mult, (units,)), np.int32)
    shift = np.ascontiguousarray(np.broadcast_to(shift, (units,)), np.int32)
    lib().tfl_fully_connected(_p(_u8(x2d), P_U8), _signed(x2d.dtype), rows, depth,
                              _p(_u8(w), P_U8), _signed(w.dtype), units,
                              None if bias is None else _p(bias, P_I32), _p(out.view(np.uint8), P_U8),
                              ctypes.c_int32(-in_zp), ctypes.c_int32(-w_zp), ctypes.c_int32(out_zp),
                              _p(mult, P_I32), _p(shift, P_I32), ctypes.c_int32(amin), ctypes.c_int32(amax))
    return out


def _shape4(s):
    s = list(s)
    return [1] * (4 - len(s)) + s


def _bshape(a, b):
    sa, sb = _shape4(a.shape), _shape4(b.shape)
    so = [max(x, y) for x, y in zip(sa, sb)]
    return (np.array(sa, np.int32), np.array(sb, np.int32), np.array(so, np.int32),
            np.broadcast_shapes(a.shape, b.shape))


def add_params(s1, s2, so):
    p = np.zeros(7, np.int32)
    lib().tfl_add_params(float(s1), float(s2), float(so), _p(p, P_I32))
    return p


def add(a, b, *, a_zp, b_zp, out_zp, params, amin, amax, sub=False):
    sa, sb, so, oshape = _bshape(a, b)
    out = np.zeros(oshape, a.dtype)
    lib().tfl_add(_p(_u8(a), P_U8), _p(sa, P_I32), _p(_u8(b), P_U8), _p(sb, P_I32),
                  _p(out.view(np.uint8), P_U8), _p(so, P_I32), _signed(a.dtype),
                  ctypes.c_int32(-a_zp), ctypes.c_int32(-b_zp), ctypes.c_int32(out_zp),
                  _p(np.ascontiguousarray(params, np.int32), P_I32), int(sub),
                  ctypes.c_int32(amin), ctypes.c_int32(amax))
    return out


def mul_params(s1, s2, so):
    m = np.zeros(1, np.int32)
    s = np.zeros(1, np.int32)
    lib().tfl_mul_params(float(s1), float(s2), float(so), _p(m, P_I32), _p(s, P_I32))
    return int(m[0]), int(s[0])


def mul(a, b, *, a_zp, b_zp, out_zp, mult, shift, amin, amax):
    sa, sb, so, oshape = _bshape(a, b)
    out = np.zeros(oshape, a.dtype)
    lib().tfl_mul(_p(_u8(a), P_U8), _p(sa, P_I32), _p(_u8(b), P_U8), _p(sb, P_I32),
                  _p(out.view(np.uint8), P_U8), _p(so, P_I32), _signed(a.dtype),
                  ctypes.c_int32(-a_zp), ctypes.c_int32(-b_zp), ctypes.c_int32(out_zp),
                  ctypes.c_int32(mult), ctypes.c_int32(shift), ctypes.c_int32(amin), ctypes.c_int32(amax))
    return out


def pool2d(x, *, kind, filt, stride, pad, out_hw, amin, amax):
    b, ih, iw, c = x.shape
    oh, ow = out_hw
    out = np.zeros((b, oh, ow, c), x.dtype)
    fn = lib().tfl_avg_pool if kind == "avg" else lib().tfl_max_pool
    fn(_p(_u8(x), P_U8), _signed(x.dtype), b, ih, iw, c, _p(out.view(np.uint8), P_U8),
       oh, ow, filt[0], filt[1], stride[0], stride[1], pad[0], pad[1],
       ctypes.c_int32(amin), ctypes.c_int32(amax))
    return out


def add_f32(a, b, amin=-np.inf, amax=np.inf, sub=False):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    sa, sb, so, oshape = _bshape(a, b)
    out = np.zeros(oshape, np.float32)
    lib().tfl_add_f32(_p(a, P_F32), _p(sa, P_I32), _p(b, P_F32), _p(sb, P_I32),
                      _p(out, P_F32), _p(so, P_I32), ctypes.c_float(amin), ctypes.c_float(amax), int(sub))
    return out


def _vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def requantize(x, *, in_scale, in_zp, out_scale, out_zp, out_dtype):
    """QUANTIZE between 8-bit types (quantize.cc -> reference_ops::Requantize)."""
    m, sh = quantize_multiplier(float(np.float64(np.float32(in_scale)) / np.float64(np.float32(out_scale))))
    x = np.ascontiguousarray(x)
    out = np.zeros(x.shape, out_dtype)
    lib().tfl_requantize(_vp(x), _signed(x.dtype), x.size, in_zp, m, sh, _signed(out_dtype), out_zp, _vp(out))
    return out


def quantize_f32(x, *, scale, zp, out_dtype):
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros(x.shape, out_dtype)
    lib().tfl_quantize_f32(_vp(x), x.size, scale, zp, _signed(out_dtype), _vp(out))
    return out


def dequantize(x, *, scale, zp):
    x = np.ascontiguousarray(x)
    out = np.zeros(x.shape, np.float32)
    lib().tfl_dequantize(_vp(x), _signed(x.dtype), x.size, scale, zp, _vp(out))
    return out


def relu_params(in_scale, out_scale, out_zp, signed, act_min, act_max):
    """act_max=None: open upper bound (RELU)"""
    v = [ctypes.c_int32() for _ in range(4)]
    lib().tfl_relu_params(in_scale, out_scale, out_zp, int(signed), act_min,
                          0.0 if act_max is None else act_max, int(act_max is None), *[ctypes.byref(t) for t in v])
    return tuple(t.value for t in v)  # mult, shift, qmin, qmax


def relu_x(x, *, in_zp, out_zp, params):
    m, sh, lo, hi = params
    x = np.ascontiguousarray(x)
    out = np.zeros_like(x)
    lib().tfl_relu_x(_vp(x), _signed(x.dtype), x.size, in_zp, out_zp, m, sh, lo, hi, _vp(out))
    return out


def logistic_table(in_scale, in_zp, out_scale, out_zp, signed):
    t = np.zeros(256, np.uint8)
    lib().tfl_logistic_table(in_scale, in_zp, out_scale, out_zp, int(signed), _vp(t))
    return t


def lookup(x, table):
    x = np.ascontiguousarray(x)
    out = np.zeros_like(x)
    lib().tfl_lookup(_vp(x), x.size, _vp(np.ascontiguousarray(table, np.uint8)), _vp(out))
    return out


def softmax(x, *, in_scale, beta, out_scale, out_zp):
    x = np.ascontiguousarray(x)
    out = np.zeros_like(x)
    depth = x.shape[-1]
    lib().tfl_softmax(_vp(x), _signed(x.dtype), x.size // depth, depth, in_scale, beta, out_scale, out_zp, _vp(out))
    return out


def transpose_conv_i8(x, w, bias, *, in_zp, out_zp, mult, shift, stride, pad, out_hw):
    x = np.ascontiguousarray(x, np.int8)
    w = np.ascontiguousarray(w, np.int8)
    b, ih, iw, ic = x.shape
    oc, kh, kw, _ = w.shape
    out = np.zeros((b, out_hw[0], out_hw[1], oc), np.int8)
    bias = None if bias is None else np.ascontiguousarray(bias, np.int32)
    m = np.ascontiguousarray(mult, np.int32)
    s = np.ascontiguousarray(shift, np.int32)
    lib().tfl_transpose_conv_i8(_vp(x), b, ih, iw, ic, _vp(w), oc, kh, kw, None if bias is None else _vp(bias),
                                _vp(out), out_hw[0], out_hw[1], stride[0], stride[1], pad[0], pad[1], -in_zp,
                                out_zp, _vp(m), _vp(s))
    return out


def softmax_table(in_scale, beta):
    t = np.zeros(256, np.float32)
    lib().tfl_softmax_table(in_scale, beta, _vp(t))
    return t


def concat(xs, axis, *, scales, zps, out_scale, out_zp):
    xs = [np.ascontiguousarray(x) for x in xs]
    rank = xs[0].ndim
    axis = axis % rank
    shape = list(xs[0].shape)
    shape[axis] = sum(x.shape[axis] for x in xs)
    out = np.zeros(shape, xs[0].dtype)
    outer = int(np.prod(shape[:axis], dtype=np.int64))
    inner = int(np.prod(shape[axis + 1:], dtype=np.int64))
    ptrs = (ctypes.c_void_p * len(xs))(*[x.ctypes.data for x in xs])
    sizes = np.array([x.shape[axis] for x in xs], np.int32)
    sc = np.array(scales, np.float32)
    zp = np.array(zps, np.int32)
    lib().tfl_concat(len(xs), ptrs, _p(sizes, P_I32), outer, inner, _p(sc, P_F32), _p(zp, P_I32),
                     out_scale, out_zp, _signed(out.dtype), _vp(out))
    return out


def pad(x, pads, value):
    """x 4-D; pads [[before, after]] * 4"""
    x = np.ascontiguousarray(x)
    p = np.ascontiguousarray(np.asarray(pads, np.int32).reshape(4, 2))
    shape = [x.shape[d] + p[d, 0] + p[d, 1] for d in range(4)]
    out = np.zeros(shape, x.dtype)
    lib().tfl_pad(_vp(x), _p(np.array(x.shape, np.int32), P_I32), _p(p.reshape(-1), P_I32),
                  ctypes.c_uint8(int(value) & 0xff), _vp(out))
    return out


def mirror_pad(x, pads, mode):
    """MIRROR_PAD (TFLite 2.9.2 kernels/mirror_pad.cc: GetInputDimension maps a
    padded index back into the input, REFLECT skipping the edge element,
    SYMMETRIC repeating it) - for pads within the input, the same map as
    numpy's 'reflect' / 'symmetric' pad modes.  mode: "REFLECT" / "SYMMETRIC"."""
    return np.pad(x, [tuple(int(v) for v in p) for p in pads], mode=mode.lower())


def mean_q8_hw(x, *, in_scale, in_zp, out_scale, out_zp):
    """quantized MEAN over axes {1, 2} with keep_dims (TFLite 2.9.2 reduce.cc
    EvalMean -> optimized_integer_ops::Mean for int8, optimized_ops::Mean for
    uint8): int32 sum, then MultiplyByQuantizedMultiplier(sum, M, shift) +
    bias, clamped to the type; M / shift = QuantizeMultiplier of the float
    in_scale / (H*W * out_scale), bias = out_zp - int(float(in_zp * in_scale
    / out_scale)) with every product in float32 as written there.
    Parity unpinned: no reference fixture holds MEAN outputs."""
    n = np.float32(x.shape[1] * x.shape[2])
    fin, fout = np.float32(in_scale), np.float32(out_scale)
    bias = int(out_zp) - int(np.float32(np.float32(np.float32(in_zp) * fin) / fout))
    real = np.float32(fin / np.float32(n * fout))
    m, sh = quantize_multiplier(float(real))
    acc = x.astype(np.int32).sum(axis=(1, 2), keepdims=True)
    out = np.array([lib().tfl_mbqm(int(a), m, sh) for a in acc.reshape(-1)], np.int64).reshape(acc.shape) + bias
    lo, hi = (-128, 127) if x.dtype == np.int8 else (0, 255)
    return np.clip(out, lo, hi).astype(x.dtype)


def hard_swish_q8(x, *, in_scale, in_zp, out_scale, out_zp):
    """HARD_SWISH 8-bit (TFLite 2.9.2 activations.cc HardSwishPrepare +
    reference_ops::HardSwish): oracle/tflite_ref.c tfl_hard_swish.
    Parity unpinned: no reference fixture holds HARD_SWISH outputs."""
    x = np.ascontiguousarray(x)
    out = np.zeros_like(x)
    rc = lib().tfl_hard_swish(_vp(x), int(x.dtype == np.int8), x.size, float(in_scale), int(in_zp),
                              float(out_scale), int(out_zp), _vp(out))
    if rc != 0:
        raise ValueError("HARD_SWISH: output multiplier exponent > 0")
    return out


def squared_difference_f32(a, b):
    """SQUARED_DIFFERENCE (float32, broadcast): (a - b)^2 in float32"""
    d = (a.astype(np.float32) - b.astype(np.float32)).astype(np.float32)
    return (d * d).astype(np.float32)


def rsqrt_f32(x):
    """RSQRT (float32): 1 / sqrt(x)"""
    return (np.float32(1.0) / np.sqrt(x.astype(np.float32))).astype(np.float32)


def nearest_index(v, in_size, out_size, align_corners, half_pixel_centers):
    return lib().tfl_nearest_index(v, in_size, out_size, int(align_corners), int(half_pixel_centers))


def resize_nearest(x, out_hw, align_corners=False, half_pixel_centers=False):
    x = np.ascontiguousarray(x)
    b, ih, iw, c = x.shape
    out = np.zeros((b, out_hw[0], out_hw[1], c), x.dtype)
    lib().tfl_resize_nearest(_vp(x), b, ih, iw, c, out_hw[0], out_hw[1], int(align_corners),
                             int(half_pixel_centers), _vp(out))
    return out


def resize_bilinear_i8(x, out_hw, align_corners=False, half_pixel_centers=False):
    x = np.ascontiguousarray(x, np.int8)
    b, ih, iw, c = x.shape
    out = np.zeros((b, out_hw[0], out_hw[1], c), np.int8)
    lib().tfl_resize_bilinear_i8(_vp(x), b, ih, iw, c, out_hw[0], out_hw[1], int(align_corners),
                                 int(half_pixel_centers), _vp(out))
    return out


def resize_bilinear_u8(x, out_hw, align_corners=False, half_pixel_centers=False):
    """optimized_ops::ResizeBilinear<uint8> float path (parity unpinned)."""
    x = np.ascontiguousarray(x, np.uint8)
    b, ih, iw, c = x.shape
    out = np.zeros((b, out_hw[0], out_hw[1], c), np.uint8)
    lib().tfl_resize_bilinear_u8(_vp(x), b, ih, iw, c, out_hw[0], out_hw[1], int(align_corners),
                                 int(half_pixel_centers), _vp(out))
    return out


# ---------------------------------------------------------------------------
# whole-model runner
# ---------------------------------------------------------------------------

def _q(t):
    return float(t.scale[0]), int(t.zero_point[0])


def _act_range_for(act, t):
    s, z = _q(t)
    return act_range(act, s, z, t.np_dtype == np.int8)


def _f32_act(act):
    return {1: (0.0, np.inf), 2: (-1.0, 1.0), 3: (0.0, 6.0)}.get(act, (-np.inf, np.inf))


class OracleInterpreter:
    """Runs the primary subgraph of a .tflite model op by op on the CPU."""

    SUPPORTED = {OP["CONV_2D"], OP["DEPTHWISE_CONV_2D"], OP["FULLY_CONNECTED"],
                 OP["ADD"], OP["SUB"], OP["MUL"], OP["AVERAGE_POOL_2D"],
                 OP["MAX_POOL_2D"], OP["RESHAPE"], OP["SQUEEZE"], OP["CONCATENATION"], OP["PAD"],
                 OP["PADV2"], OP["QUANTIZE"], OP["DEQUANTIZE"], OP["RELU"], OP["RELU6"],
                 OP["RELU_N1_TO_1"], OP["LOGISTIC"], OP["SOFTMAX"], OP["RESIZE_NEAREST_NEIGHBOR"],
                 OP["RESIZE_BILINEAR"], OP["TRANSPOSE_CONV"], OP["CUSTOM"]}

    def __init__(self, model):
        self.model = model if isinstance(model, Model) else Model.from_path(model)

    def unsupported_ops(self):
        return [i for i, o in enumerate(self.model.operators) if o.builtin not in self.SUPPORTED]

    def run(self, inputs, ops=None):
        """inputs: {tensor_index: ndarray}. Returns {tensor_index: ndarray}."""
        m = self.model
        vals = {}
        for t in m.tensors:
            if t.is_const:
                vals[t.index] = t.data
        for k, v in inputs.items():
            t = m.tensors[k]
            vals[k] = np.asarray(v, t.np_dtype).reshape(t.shape)
        order = range(len(m.operators)) if ops is None else sorted(ops)
        for i in order:
            o = m.operators[i]
            outs = self._op(o, vals)
            for idx, val in zip(o.outputs, outs):
                vals[idx] = np.asarray(val).reshape(m.tensors[idx].shape).astype(m.tensors[idx].np_dtype, copy=False)
        return vals

    _FLOAT_OPS = ("CONV_2D", "DEPTHWISE_CONV_2D", "FULLY_CONNECTED", "ADD", "SUB", "MUL", "AVERAGE_POOL_2D",
                  "MAX_POOL_2D", "RELU", "RELU6", "RELU_N1_TO_1", "LOGISTIC", "SOFTMAX", "CONCATENATION")

    def _op_float(self, o, vals):
        """float32 graphs (oracle/float_ref.py)"""
        from . import float_ref as F
        T = self.model.tensors
        opt = o.options
        code = o.builtin
        x = vals[o.inputs[0]]
        to = T[o.outputs[0]]
        if code in (OP["CONV_2D"], OP["DEPTHWISE_CONV_2D"]):
            dw = code == OP["DEPTHWISE_CONV_2D"]
            w = vals[o.inputs[1]]
            bias = vals.get(o.inputs[2]) if len(o.inputs) > 2 and o.inputs[2] >= 0 else None
            same = opt.scalar(0, "b", 0) == 0
            sw, sh = opt.scalar(1, "i", 1), opt.scalar(2, "i", 1)
            if dw:
                dm, act = opt.scalar(3, "i", 1), opt.scalar(4, "b", 0)
                dw_, dh_ = opt.scalar(5, "i", 1), opt.scalar(6, "i", 1)
                kh, kw = w.shape[1], w.shape[2]
            else:
                act = opt.scalar(3, "b", 0)
                dw_, dh_ = opt.scalar(4, "i", 1), opt.scalar(5, "i", 1)
                kh, kw = w.shape[1], w.shape[2]
            ih, iw = x.shape[1], x.shape[2]
            oh, ow = out_size(same, ih, kh, sh, dh_), out_size(same, iw, kw, sw, dw_)
            pad = (padding(sh, dh_, ih, kh, oh), padding(sw, dw_, iw, kw, ow))
            lo, hi = _f32_act(act)
            if dw:
                return [F.dwconv2d_f32(x, w, bias, dm, (sh, sw), (dh_, dw_), pad, (oh, ow), lo, hi)]
            return [F.conv2d_f32(x, w, bias, (sh, sw), (dh_, dw_), pad, (oh, ow), lo, hi)]
        if code == OP["FULLY_CONNECTED"]:
            w = vals[o.inputs[1]]
            bias = vals.get(o.inputs[2]) if len(o.inputs) > 2 and o.inputs[2] >= 0 else None
            lo, hi = _f32_act(opt.scalar(0, "b", 0) if opt is not None else 0)
            return [F.fully_connected_f32(x, w, bias, lo, hi)]
        if code in (OP["ADD"], OP["SUB"], OP["MUL"]):
            lo, hi = _f32_act(opt.scalar(0, "b", 0) if opt is not None else 0)
            kind = {OP["ADD"]: "add", OP["SUB"]: "sub", OP["MUL"]: "mul"}[code]
            return [F.eltwise_f32(x, vals[o.inputs[1]], kind, lo, hi)]
        if code in (OP["AVERAGE_POOL_2D"], OP["MAX_POOL_2D"]):
            same = opt.scalar(0, "b", 0) == 0
            sw, sh = opt.scalar(1, "i", 1), opt.scalar(2, "i", 1)
            fw, fh = opt.scalar(3, "i", 1), opt.scalar(4, "i", 1)
            lo, hi = _f32_act(opt.scalar(5, "b", 0))
            ih, iw = x.shape[1], x.shape[2]
            oh, ow = out_size(same, ih, fh, sh, 1), out_size(same, iw, fw, sw, 1)
            pad = (padding(sh, 1, ih, fh, oh), padding(sw, 1, iw, fw, ow))
            kind = "avg" if code == OP["AVERAGE_POOL_2D"] else "max"
            return [F.pool2d_f32(x, kind, (fh, fw), (sh, sw), pad, (oh, ow), lo, hi)]
        if code in (OP["RELU"], OP["RELU6"], OP["RELU_N1_TO_1"]):
            lo, hi = {OP["RELU"]: (0.0, np.inf), OP["RELU6"]: (0.0, 6.0), OP["RELU_N1_TO_1"]: (-1.0, 1.0)}[code]
            return [np.clip(x, lo, hi).astype(np.float32)]
        if code == OP["LOGISTIC"]:
            return [F.logistic_f32(x)]
        if code == OP["SOFTMAX"]:
            return [F.softmax_f32(x, opt.scalar(0, "f", 1.0) if opt is not None else 1.0)]
        if code == OP["CONCATENATION"]:
            return [np.concatenate([vals[i] for i in o.inputs], axis=opt.scalar(0, "i", 0))]
        raise NotImplementedError("oracle: float op %s" % o.name)

    def _op(self, o, vals):
        m = self.model
        T = m.tensors
        opt = o.options
        code = o.builtin
        if (o.inputs and o.inputs[0] >= 0 and T[o.inputs[0]].np_dtype == np.float32 and
                o.name in self._FLOAT_OPS):
            return self._op_float(o, vals)
        if code == OP["DEQUANTIZE"] and T[o.inputs[0]].np_dtype == np.float16:
            return [vals[o.inputs[0]].astype(np.float32)]
        if code in (OP["CONV_2D"], OP["DEPTHWISE_CONV_2D"]):
            dw = code == OP["DEPTHWISE_CONV_2D"]
            x, w = vals[o.inputs[0]], vals[o.inputs[1]]
            bias = vals.get(o.inputs[2]) if len(o.inputs) > 2 and o.inputs[2] >= 0 else None
            ti, tw, to = T[o.inputs[0]], T[o.inputs[1]], T[o.outputs[0]]
            pad_same = opt.scalar(0, "b", 0) == 0
            sw, sh = opt.scalar(1, "i", 1), opt.scalar(2, "i", 1)
            if dw:
                dm = opt.scalar(3, "i", 1)
                act = opt.scalar(4, "b", 0)
                dw_, dh_ = opt.scalar(5, "i", 1), opt.scalar(6, "i", 1)
                kh, kw, oc = w.shape[1], w.shape[2], w.shape[3]
            else:
                act = opt.scalar(3, "b", 0)
                dw_, dh_ = opt.scalar(4, "i", 1), opt.scalar(5, "i", 1)
                oc, kh, kw = w.shape[0], w.shape[1], w.shape[2]
            ih, iw = x.shape[1], x.shape[2]
            oh = out_size(pad_same, ih, kh, sh, dh_)
            ow = out_size(pad_same, iw, kw, sw, dw_)
            ph = padding(sh, dh_, ih, kh, oh)
            pw = padding(sw, dw_, iw, kw, ow)
            in_s, in_z = _q(ti)
            out_s, out_z = _q(to)
            legacy = ti.np_dtype == np.uint8
            mult, shift = conv_multipliers(in_s, tw.scale, oc, out_s, legacy)
            amin, amax = _act_range_for(act, to)
            w_zp = int(tw.zero_point[0]) if legacy else 0
            kw_args = dict(in_zp=in_z, w_zp=w_zp, out_zp=out_z, mult=mult, shift=shift,
                           amin=amin, amax=amax, stride=(sh, sw), dilation=(dh_, dw_),
                           pad=(ph, pw), out_hw=(oh, ow))
            if dw:
                return [dwconv2d(x, w, bias, dm=dm, **kw_args)]
            return [conv2d(x, w, bias, **kw_args)]
        if code == OP["FULLY_CONNECTED"]:
            x, w = vals[o.inputs[0]], vals[o.inputs[1]]
            bias = vals.get(o.inputs[2]) if len(o.inputs) > 2 and o.inputs[2] >= 0 else None
            ti, tw, to = T[o.inputs[0]], T[o.inputs[1]], T[o.outputs[0]]
            act = opt.scalar(0, "b", 0) if opt is not None else 0
            depth = w.shape[1]
            x2 = x.reshape(-1, depth)
            in_s, in_z = _q(ti)
            out_s, out_z = _q(to)
            mult, shift = conv_multipliers(in_s, tw.scale[:1], 1, out_s, True)
            amin, amax = _act_range_for(act, to)
            return [fully_connected(x2, w, bias, in_zp=in_z, w_zp=int(tw.zero_point[0]),
                                    out_zp=out_z, mult=mult[0], shift=shift[0], amin=amin, amax=amax)]
        if code in (OP["ADD"], OP["SUB"]):
            a, b = vals[o.inputs[0]], vals[o.inputs[1]]
            ta, tb, to = T[o.inputs[0]], T[o.inputs[1]], T[o.outputs[0]]
            act = opt.scalar(0, "b", 0) if opt is not None else 0
            if to.np_dtype == np.float32:
                lo, hi = _f32_act(act)
                return [add_f32(a, b, lo, hi, sub=code == OP["SUB"])]
            sa, za = _q(ta)
            sb, zb = _q(tb)
            so, zo = _q(to)
            amin, amax = _act_range_for(act, to)
            return [add(a, b, a_zp=za, b_zp=zb, out_zp=zo, params=add_params(sa, sb, so),
                        amin=amin, amax=amax, sub=code == OP["SUB"])]
        if code == OP["MUL"]:
            a, b = vals[o.inputs[0]], vals[o.inputs[1]]
            ta, tb, to = T[o.inputs[0]], T[o.inputs[1]], T[o.outputs[0]]
            act = opt.scalar(0, "b", 0) if opt is not None else 0
            sa, za = _q(ta)
            sb, zb = _q(tb)
            so, zo = _q(to)
            mult, shift = mul_params(sa, sb, so)
            amin, amax = _act_range_for(act, to)
            return [mul(a, b, a_zp=za, b_zp=zb, out_zp=zo, mult=mult, shift=shift, amin=amin, amax=amax)]
        if code in (OP["AVERAGE_POOL_2D"], OP["MAX_POOL_2D"]):
            x = vals[o.inputs[0]]
            to = T[o.outputs[0]]
            pad_same = opt.scalar(0, "b", 0) == 0
            sw, sh = opt.scalar(1, "i", 1), opt.scalar(2, "i", 1)
            fw, fh = opt.scalar(3, "i", 1), opt.scalar(4, "i", 1)
            act = opt.scalar(5, "b", 0)
            ih, iw = x.shape[1], x.shape[2]
            oh, ow = out_size(pad_same, ih, fh, sh, 1), out_size(pad_same, iw, fw, sw, 1)
            ph, pw = padding(sh, 1, ih, fh, oh), padding(sw, 1, iw, fw, ow)
            amin, amax = _act_range_for(act, to)
            kind = "avg" if code == OP["AVERAGE_POOL_2D"] else "max"
            return [pool2d(x, kind=kind, filt=(fh, fw), stride=(sh, sw), pad=(ph, pw),
                           out_hw=(oh, ow), amin=amin, amax=amax)]
        if code in (OP["RESHAPE"], OP["SQUEEZE"]):
            return [vals[o.inputs[0]].copy()]
        if code == OP["TRANSPOSE_CONV"]:
            # inputs: output_shape, weights (OHWI), input, [bias]
            w, x = vals[o.inputs[1]], vals[o.inputs[2]]
            tw, tx, to = T[o.inputs[1]], T[o.inputs[2]], T[o.outputs[0]]
            bias = vals.get(o.inputs[3]) if len(o.inputs) > 3 and o.inputs[3] >= 0 else None
            if tx.np_dtype != np.int8:
                raise NotImplementedError("oracle: TRANSPOSE_CONV restated for int8 only")
            same = opt.scalar(0, "b", 0) == 0
            sw, sh = opt.scalar(1, "i", 1), opt.scalar(2, "i", 1)
            oh, ow = to.shape[1], to.shape[2]
            kh, kw = w.shape[1], w.shape[2]
            # transpose_conv.cc: padding as for a conv whose input is the output
            ph = padding(sh, 1, oh, kh, out_size(same, oh, kh, sh, 1))
            pw = padding(sw, 1, ow, kw, out_size(same, ow, kw, sw, 1))
            mult, shift = conv_multipliers(_q(tx)[0], tw.scale, w.shape[0], _q(to)[0], False)
            return [transpose_conv_i8(x, w, bias, in_zp=_q(tx)[1], out_zp=_q(to)[1], mult=mult, shift=shift,
                                      stride=(sh, sw), pad=(ph, pw), out_hw=(oh, ow))]
        x = vals[o.inputs[0]]
        ti, to = T[o.inputs[0]], T[o.outputs[0]]
        if code == OP["CONCATENATION"]:
            axis = opt.scalar(0, "i", 0)
            xs = [vals[i] for i in o.inputs]
            return [concat(xs, axis, scales=[_q(T[i])[0] for i in o.inputs], zps=[_q(T[i])[1] for i in o.inputs],
                           out_scale=_q(to)[0], out_zp=_q(to)[1])]
        if code in (OP["PAD"], OP["PADV2"]):
            pads = np.asarray(vals[o.inputs[1]], np.int64).reshape(-1, 2)
            pads = np.concatenate([np.zeros((4 - len(pads), 2), np.int64), pads]) if len(pads) < 4 else pads
            x4 = x.reshape([1] * (4 - x.ndim) + list(x.shape))
            if code == OP["PADV2"] and len(o.inputs) > 2 and o.inputs[2] >= 0:
                value = int(np.asarray(vals[o.inputs[2]]).reshape(-1)[0])
            else:
                value = _q(to)[1]
            return [pad(x4, pads, value)]
        if code == OP["QUANTIZE"]:
            s_o, z_o = _q(to)
            if ti.np_dtype == np.float32:
                return [quantize_f32(x, scale=s_o, zp=z_o, out_dtype=to.np_dtype)]
            s_i, z_i = _q(ti)
            return [requantize(x, in_scale=s_i, in_zp=z_i, out_scale=s_o, out_zp=z_o, out_dtype=to.np_dtype)]
        if code == OP["DEQUANTIZE"]:
            s_i, z_i = _q(ti)
            return [dequantize(x, scale=s_i, zp=z_i)]
        if code in (OP["RELU"], OP["RELU6"], OP["RELU_N1_TO_1"]):
            lo, hi = {OP["RELU"]: (0.0, None), OP["RELU6"]: (0.0, 6.0), OP["RELU_N1_TO_1"]: (-1.0, 1.0)}[code]
            s_i, z_i = _q(ti)
            s_o, z_o = _q(to)
            prm = relu_params(s_i, s_o, z_o, to.np_dtype == np.int8, lo, hi)
            return [relu_x(x, in_zp=z_i, out_zp=z_o, params=prm)]
        if code == OP["LOGISTIC"]:
            s_i, z_i = _q(ti)
            s_o, z_o = _q(to)
            return [lookup(x, logistic_table(s_i, z_i, s_o, z_o, ti.np_dtype == np.int8))]
        if code == OP["SOFTMAX"]:
            beta = opt.scalar(0, "f", 1.0) if opt is not None else 1.0
            s_o, z_o = _q(to)
            return [softmax(x, in_scale=_q(ti)[0], beta=beta, out_scale=s_o, out_zp=z_o)]
        if code in (OP["RESIZE_NEAREST_NEIGHBOR"], OP["RESIZE_BILINEAR"]):
            oh, ow = to.shape[1], to.shape[2]
            if code == OP["RESIZE_NEAREST_NEIGHBOR"]:
                ac, hp = opt.scalar(0, "b", 0) if opt else 0, opt.scalar(1, "b", 0) if opt else 0
                return [resize_nearest(x, (oh, ow), ac, hp)]
            ac, hp = opt.scalar(2, "b", 0) if opt else 0, opt.scalar(3, "b", 0) if opt else 0
            if ti.np_dtype == np.uint8:
                return [resize_bilinear_u8(x, (oh, ow), ac, hp)]
            if ti.np_dtype != np.int8:
                raise NotImplementedError("oracle: RESIZE_BILINEAR restated for int8 / uint8 only")
            return [resize_bilinear_i8(x, (oh, ow), ac, hp)]
        if code == OP["CUSTOM"] and o.custom == "TFLite_Detection_PostProcess":
            from .detection_postprocess import detection_postprocess, read_flexbuffer_map
            return list(detection_postprocess(vals[o.inputs[0]], vals[o.inputs[1]], vals[o.inputs[2]],
                                              read_flexbuffer_map(o.custom_options)))
        raise NotImplementedError("oracle: op %s not restated" % o.name)
