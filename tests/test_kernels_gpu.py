"""Op-level parity: HIP kernels (through the C ABI) vs the CPU oracle, bit-exact.

Oracle = TFLite 2.9.2 integer reference kernels restated in oracle/tflite_ref.c
(pinned by tests/test_oracle.py against the reference's own known answers).
"""
import ctypes
import zlib

import numpy as np
import pytest

from oracle import runner as orc
from tests.kernel_harness import (MNV2_DEPTHWISE, MNV2_POINTWISE, ConvCase, dom, rand_q)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("spatial,ic,oc", MNV2_POINTWISE)
def test_conv1x1_mnv2_shapes_int8(gpu_lib, spatial, ic, oc):
    rng = np.random.default_rng(1000 + spatial * 7 + ic + oc)
    c = ConvCase(rng, 1, spatial, spatial, ic, oc, 1, 1, act=3)
    np.testing.assert_array_equal(c.gpu(gpu_lib), c.oracle())


# batched 1x1 layers (job batching): M = b*h*w >= 32768 output pixels take
# conv_rows_kernel (channel-major tiles, packed stores); N / K tails, uint8
# per-tensor filters (row-sum correction), whole-N and chunked-N grids
@pytest.mark.parametrize("b,spatial,ic,oc,dtype", [
    (4, 112, 16, 96, np.int8), (4, 112, 32, 16, np.uint8), (12, 56, 24, 144, np.int8),
    (12, 56, 144, 24, np.uint8), (44, 28, 32, 192, np.int8), (44, 28, 192, 32, np.int8),
    (170, 14, 64, 384, np.int8), (170, 14, 96, 20, np.uint8), (700, 7, 64, 520, np.int8),
    (700, 7, 40, 1001 + 3, np.int8), (45, 28, 12, 72, np.uint8)])
def test_conv1x1_rows_batched(gpu_lib, b, spatial, ic, oc, dtype):
    rng = np.random.default_rng(4000 + b + spatial + ic + oc)
    c = ConvCase(rng, b, spatial, spatial, ic, oc, 1, 1, dtype=dtype, act=3)
    ref = c.oracle()
    np.testing.assert_array_equal(c.gpu(gpu_lib), ref)
    c.requant_fast = False  # the two-step requantisation path
    np.testing.assert_array_equal(c.gpu(gpu_lib), ref)


# the LDS-staged GEMM (conv_gemm_kernel, forced with BH_CONV_GEMM = 2) beside
# conv_mfma_kernel (BH_CONV_MFMA = 1) on the batched deep / wide 1x1 layers:
# both configurations (128x128 over 8 waves, 64x64 over 8 waves), M / N / K tails (K < 64, K % 64 != 0,
# N not a tile multiple, N % 4 != 0), both requantisation paths
@pytest.mark.parametrize("b,spatial,ic,oc", [
    (6, 14, 512, 1024), (24, 14, 960, 160), (8, 7, 1280, 546), (6, 14, 576, 273), (1, 14, 16, 24),
    (3, 9, 48, 20), (6, 14, 1024, 17), (2, 7, 160, 960), (24, 7, 320, 1280), (5, 13, 96, 64),
    (24, 14, 512, 1024), (24, 14, 192, 1000)])
def test_conv1x1_gemm_vs_mfma(gpu_lib, b, spatial, ic, oc):
    rng = np.random.default_rng(6000 + b + spatial + ic + oc)
    c = ConvCase(rng, b, spatial, spatial, ic, oc, 1, 1, act=3)
    ref = c.oracle()
    for hint in (3, 2, 1):  # BH_CONV_GEMM_BIG, BH_CONV_GEMM, BH_CONV_MFMA
        c.kernel_hint = hint
        for fast in (None, False):
            c.requant_fast = fast
            np.testing.assert_array_equal(c.gpu(gpu_lib), ref, err_msg="hint %d fast %s" % (hint, fast))


# conv_gemm_big_kernel at the sizes it is routed to (M in the tens of
# thousands: job batches of 32 / 256): MobileNetV2's 320 -> 1280 head at
# B = 256, K < 64, N not a multiple of 16 / of the tile, M tails
@pytest.mark.parametrize("b,spatial,ic,oc", [
    (256, 7, 320, 1280), (256, 14, 64, 256), (64, 28, 32, 512), (300, 7, 48, 1000), (257, 13, 16, 120)])
def test_conv1x1_gemm_big_routed(gpu_lib, b, spatial, ic, oc):
    rng = np.random.default_rng(6100 + b + spatial + ic + oc)
    c = ConvCase(rng, b, spatial, spatial, ic, oc, 1, 1, act=3)
    ref = c.oracle()
    keep = []
    p = c.params(gpu_lib, keep)
    routed = gpu_lib.bh_conv2d_i8_kernel(ctypes.byref(p)).decode()
    if ic >= 128 and oc >= 128:  # wide K and N: the big tiles (else the activation-stream kernels may win)
        assert routed == "conv_gemm_big_kernel", routed
    del keep
    for hint in (0, 3):  # the routed kernel, then the big GEMM forced
        c.kernel_hint = hint
        for fast in (None, False):
            c.requant_fast = fast
            np.testing.assert_array_equal(c.gpu(gpu_lib), ref, err_msg="hint %d fast %s" % (hint, fast))


# the big GEMM's folded residual ADD and 8-bit output table, applied per byte
# on its copy-out path (conv_store4's arithmetic): against the oracle's conv
# -> ADD -> table, and against conv_mfma_kernel on the same parameters
@pytest.mark.parametrize("b,spatial,ch", [(8, 14, 256), (3, 9, 96), (16, 7, 160)])
def test_conv1x1_gemm_big_residual_table(gpu_lib, b, spatial, ch):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(6200 + b + spatial + ch)
    c = ConvCase(rng, b, spatial, spatial, ch, ch, 1, 1, act=0)
    y = c.oracle()
    r = rng.integers(-128, 128, y.shape).astype(np.int8)
    r_scale, r_zp = 0.037, int(rng.integers(-10, 10))
    o_scale, o_zp = 0.051, int(rng.integers(-10, 10))
    prm = orc.add_params(c.out_scale, r_scale, o_scale)
    amin, amax = orc.act_range(1, o_scale, o_zp, True)  # RELU on the ADD
    z = orc.add(y, r, a_zp=c.out_zp, b_zp=r_zp, out_zp=o_zp, params=prm, amin=amin, amax=amax)
    table = rng.permutation(256).astype(np.uint8)
    ref = table[z.view(np.uint8)].view(np.int8)
    outs = {}
    for hint in (3, 1):
        keep = []
        p = c.params(gpu_lib, keep)
        dr = DeviceBuffer.from_array(r)
        dt = DeviceBuffer.from_array(table)
        keep += [dr, dt]
        p.residual, p.out_table = dr.value, dt.value
        p.add_left_shift = int(prm[6])
        p.add_y_off, p.add_r_off, p.add_o_off = -c.out_zp, -r_zp, o_zp
        p.add_y_mult, p.add_y_shift = int(prm[0]), int(prm[1])
        p.add_r_mult, p.add_r_shift = int(prm[2]), int(prm[3])
        p.add_o_mult, p.add_o_shift = int(prm[4]), int(prm[5])
        p.add_act_min, p.add_act_max = amin, amax
        p.kernel_hint = hint
        _abi.check(gpu_lib.bh_conv2d_i8(ctypes.byref(p), None), "bh_conv2d_i8")
        outs[hint] = c._dy.download(np.int8, y.shape)
        del keep
        np.testing.assert_array_equal(outs[hint], ref, err_msg="hint %d" % hint)


# the RGB stem kernel (conv_stem_kernel: aligned row gathers + byte path at
# the image's left / right edge and the tensor's end): SAME / VALID padding,
# stride 1 / 2, odd widths, batch, uint8 (filter zero point), both
# requantisation paths; the persistent LDS form's multi-tile workgroups
# (> 768 tiles: batch 64 at 57x61 mixes staged tiles and tiles that span two
# images, batch 32 at 224x224 is the bench's shape)
@pytest.mark.parametrize("b,h,w,oc,stride,same,dtype", [
    (2, 224, 224, 32, 2, True, np.int8), (3, 37, 41, 16, 2, True, np.uint8), (1, 15, 13, 24, 1, True, np.int8),
    (5, 31, 29, 32, 1, True, np.uint8), (24, 224, 224, 32, 2, True, np.int8), (2, 11, 10, 64, 2, False, np.uint8),
    (2, 20, 23, 8, 1, False, np.uint8), (4, 9, 9, 48, 2, False, np.int8), (1, 224, 224, 64, 2, True, np.uint8),
    (64, 57, 61, 16, 1, True, np.uint8), (32, 224, 224, 32, 2, True, np.int8)])
def test_conv_stem(gpu_lib, b, h, w, oc, stride, same, dtype):
    rng = np.random.default_rng(5000 + b * h * w + oc + stride)
    c = ConvCase(rng, b, h, w, 3, oc, 3, 3, stride=(stride, stride), same=same, dtype=dtype, act=3)
    ref = c.oracle()
    # the routed form (LDS-staged VALU stem), then the VALU form
    # (BH_CONV_STEM_VALU = 4), the MFMA form (BH_CONV_STEM_MFMA = 5, out_c %
    # 16 == 0, <= 64) and the scalar-cache VALU form (BH_CONV_STEM_SCALAR =
    # 6) forced; both requantisation paths
    for hint in (0, 4, 5, 6):
        c.kernel_hint = hint
        for fast in (None, False):
            c.requant_fast = fast
            np.testing.assert_array_equal(c.gpu(gpu_lib), ref, err_msg="hint %d fast %s" % (hint, fast))


def test_conv_first_layer_3x3_s2_int8(gpu_lib):
    rng = np.random.default_rng(7)
    c = ConvCase(rng, 1, 224, 224, 3, 32, 3, 3, stride=(2, 2), act=3)
    np.testing.assert_array_equal(c.gpu(gpu_lib), c.oracle())


@pytest.mark.parametrize("spatial,ic,oc", MNV2_POINTWISE[::4])
def test_conv1x1_uint8_per_tensor(gpu_lib, spatial, ic, oc):
    rng = np.random.default_rng(2000 + spatial + ic + oc)
    c = ConvCase(rng, 1, spatial, spatial, ic, oc, 1, 1, dtype=np.uint8, act=3)
    np.testing.assert_array_equal(c.gpu(gpu_lib), c.oracle())


@pytest.mark.parametrize("args", [
    dict(b=1, ih=224, iw=224, ic=3, oc=32, kh=3, kw=3, stride=(2, 2), dtype=np.uint8),
    dict(b=2, ih=17, iw=13, ic=16, oc=40, kh=3, kw=3, stride=(1, 1)),
    dict(b=1, ih=20, iw=20, ic=24, oc=72, kh=3, kw=3, stride=(2, 2)),
    dict(b=1, ih=11, iw=9, ic=13, oc=21, kh=5, kw=3, stride=(1, 2), same=False),
    dict(b=1, ih=16, iw=16, ic=32, oc=64, kh=3, kw=3, dil=(2, 2)),
    dict(b=3, ih=8, iw=8, ic=40, oc=24, kh=1, kw=1, stride=(2, 2)),
    dict(b=1, ih=9, iw=9, ic=20, oc=17, kh=1, kw=1, act=0),
    dict(b=1, ih=6, iw=7, ic=8, oc=130, kh=3, kw=3, dtype=np.uint8, act=1),
    # small-K direct kernel (conv_direct.hip): K 63 / 25 / 18, channel tails
    dict(b=2, ih=15, iw=12, ic=7, oc=12, kh=3, kw=3, stride=(2, 2)),
    dict(b=1, ih=10, iw=10, ic=1, oc=8, kh=5, kw=5, dtype=np.uint8),
    dict(b=1, ih=9, iw=9, ic=2, oc=19, kh=3, kw=3, dil=(2, 2), same=False),
])
def test_conv_general(gpu_lib, args):
    rng = np.random.default_rng(zlib.crc32(repr(sorted(args.items())).encode()))
    c = ConvCase(rng, **args)
    np.testing.assert_array_equal(c.gpu(gpu_lib), c.oracle())


@pytest.mark.parametrize("spatial,ch,stride", MNV2_DEPTHWISE)
def test_dwconv_mnv2_shapes(gpu_lib, spatial, ch, stride):
    rng = np.random.default_rng(3000 + spatial + ch + stride)
    c = ConvCase(rng, 1, spatial, spatial, ch, ch, 3, 3, stride=(stride, stride), depthwise=True)
    np.testing.assert_array_equal(c.gpu(gpu_lib), c.oracle())


# the dot4 kernel (tap table) and the per-tap kernel against the oracle:
# int8 / uint8 (filter zero point), the single-step and two-step
# requantisation, odd sizes (image-border taps on every side), batch, the
# three vector widths (C % 16, % 8, % 4) and dilation
@pytest.mark.parametrize("b,h,w,ch,stride,dil,dtype", [
    (1, 112, 112, 32, 1, 1, np.int8), (3, 57, 55, 144, 2, 1, np.int8), (2, 28, 28, 192, 1, 1, np.uint8),
    (5, 15, 13, 24, 2, 1, np.uint8), (2, 9, 9, 12, 1, 1, np.int8), (1, 17, 17, 20, 1, 2, np.int8),
    (16, 14, 14, 576, 1, 1, np.int8), (4, 7, 7, 960, 1, 1, np.uint8),
    # grids >= 40k threads: the run kernel (4 pixels x 4 channels per thread),
    # both strides, widths not a multiple of 4, uint8
    (4, 112, 112, 32, 1, 1, np.int8), (8, 57, 55, 144, 2, 1, np.int8), (6, 28, 27, 192, 1, 1, np.uint8),
    (32, 29, 30, 96, 2, 1, np.uint8), (64, 7, 7, 960, 1, 1, np.int8),
    # dilation 2 (DeepLab's atrous depthwise layers) in the run form
    (24, 14, 14, 576, 1, 2, np.int8), (32, 17, 15, 96, 1, 2, np.uint8)])
def test_dwconv_taps_vs_per_tap(gpu_lib, b, h, w, ch, stride, dil, dtype):
    rng = np.random.default_rng(3100 + b * h * w + ch + stride + dil)
    c = ConvCase(rng, b, h, w, ch, ch, 3, 3, stride=(stride, stride), dil=(dil, dil), depthwise=True, dtype=dtype)
    ref = c.oracle()
    # every form the shape allows: its own route, then each forced one
    # (BH_DW_RUN / _DOT / _MFMA; a form the shape cannot take falls back)
    for hint in (0, 1, 2, 3):
        c.kernel_hint = hint
        for fast in (None, False):
            c.requant_fast = fast
            np.testing.assert_array_equal(c.gpu(gpu_lib), ref, err_msg="hint %d requant_fast %s" % (hint, fast))
    c.kernel_hint, c.taps = 0, False
    np.testing.assert_array_equal(c.gpu(gpu_lib), ref)


# the MFMA form (block-diagonal filter fragments) on every MobileNetV2
# depthwise layer at the headline's job batch, int8 and uint8 (w_zp != 0:
# the ones-matrix row sums), plus pixel counts that are not a multiple of 16
@pytest.mark.parametrize("h,ch,stride", [(112, 32, 1), (112, 96, 2), (56, 144, 1), (56, 144, 2), (28, 192, 1),
                                         (28, 192, 2), (14, 384, 1), (14, 576, 1), (14, 576, 2), (7, 960, 1),
                                         (13, 48, 1), (9, 16, 2)])
@pytest.mark.parametrize("dtype", [np.int8, np.uint8])
def test_dwconv_mfma_mnv2_layers(gpu_lib, h, ch, stride, dtype):
    b = 24 if h >= 14 else 5
    rng = np.random.default_rng(7700 + h * ch + stride + (dtype == np.uint8))
    c = ConvCase(rng, b, h, h, ch, ch, 3, 3, stride=(stride, stride), depthwise=True, dtype=dtype, kernel_hint=3)
    ref = c.oracle()
    np.testing.assert_array_equal(c.gpu(gpu_lib), ref)
    c.requant_fast = False
    np.testing.assert_array_equal(c.gpu(gpu_lib), ref)


@pytest.mark.parametrize("args", [
    dict(b=1, ih=56, iw=56, ic=144, oc=0, kh=3, kw=3, stride=(2, 2), dtype=np.uint8),
    dict(b=2, ih=13, iw=11, ic=6, oc=0, kh=3, kw=3, depthwise=True, dm=2),
    dict(b=1, ih=15, iw=15, ic=7, oc=0, kh=5, kw=5, stride=(2, 2), same=False),
    dict(b=1, ih=12, iw=12, ic=16, oc=0, kh=3, kw=3, dil=(2, 2)),
])
def test_dwconv_general(gpu_lib, args):
    args = dict(args)
    args["depthwise"] = True
    rng = np.random.default_rng(zlib.crc32(repr(sorted(args.items())).encode()))
    c = ConvCase(rng, **args)
    np.testing.assert_array_equal(c.gpu(gpu_lib), c.oracle())


def _elt(gpu_lib, a, b, kind, dtype, rng, sub=False):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    sa, sb = float(rng.uniform(0.01, 0.1)), float(rng.uniform(0.01, 0.1))
    so = float(rng.uniform(0.02, 0.15))
    if dtype == np.int8:
        za, zb, zo = (int(v) for v in rng.integers(-128, 128, 3))
    else:
        za, zb, zo = (int(v) for v in rng.integers(0, 256, 3))
    amin, amax = orc.act_range(1, so, zo, dtype == np.int8)
    if kind == "add":
        prm = orc.add_params(sa, sb, so)
        ref = orc.add(a, b, a_zp=za, b_zp=zb, out_zp=zo, params=prm, amin=amin, amax=amax, sub=sub)
    else:
        m, s = orc.mul_params(sa, sb, so)
        ref = orc.mul(a, b, a_zp=za, b_zp=zb, out_zp=zo, mult=m, shift=s, amin=amin, amax=amax)
    s4 = lambda s: [1] * (4 - len(s)) + list(s)
    p = _abi.EltwiseParams()
    p.kind = 0 if kind == "add" else 1
    p.in_signed = int(dtype == np.int8)
    for i, (x, y, z) in enumerate(zip(s4(a.shape), s4(b.shape), s4(ref.shape))):
        p.shape_a[i], p.shape_b[i], p.shape_o[i] = x, y, z
    p.a_off, p.b_off, p.o_off = -za, -zb, zo
    if kind == "add":
        p.a_mult, p.a_shift, p.b_mult, p.b_shift, p.o_mult, p.o_shift, p.left_shift = [int(v) for v in prm]
        if sub:
            p.b_mult = -p.b_mult
    else:
        p.o_mult, p.o_shift = m, s
    p.act_min, p.act_max = amin, amax
    da, db = DeviceBuffer.from_array(a), DeviceBuffer.from_array(b)
    do = DeviceBuffer(ref.nbytes)
    p.a, p.b, p.out = da.value, db.value, do.value
    _abi.check(gpu_lib.bh_eltwise_i8(ctypes.byref(p), None), "eltwise")
    np.testing.assert_array_equal(do.download(dtype, ref.shape), ref)


@pytest.mark.parametrize("dtype", [np.int8, np.uint8])
@pytest.mark.parametrize("shape", [(1, 56, 56, 24), (1, 7, 7, 160), (1, 5, 3, 3), (2, 3, 3, 1)])
def test_add_same_shape(gpu_lib, dtype, shape):
    rng = np.random.default_rng(sum(shape) + (dtype == np.int8))
    _elt(gpu_lib, rand_q(rng, shape, dtype), rand_q(rng, shape, dtype), "add", dtype, rng)


def test_sub_and_broadcast(gpu_lib):
    rng = np.random.default_rng(5)
    a = rand_q(rng, (1, 16, 16, 3), np.int8)
    _elt(gpu_lib, a, rand_q(rng, (1, 1, 1, 3), np.int8), "add", np.int8, rng, sub=True)
    _elt(gpu_lib, a, rand_q(rng, (3,), np.int8), "add", np.int8, rng)


@pytest.mark.parametrize("dtype", [np.int8, np.uint8])
def test_mul(gpu_lib, dtype):
    rng = np.random.default_rng(11)
    _elt(gpu_lib, rand_q(rng, (1, 10, 10, 8), dtype), rand_q(rng, (1, 10, 10, 8), dtype), "mul", dtype, rng)
    _elt(gpu_lib, rand_q(rng, (1, 10, 10, 8), dtype), rand_q(rng, (1, 1, 1, 1), dtype), "mul", dtype, rng)


@pytest.mark.parametrize("kind", ["avg", "max"])
@pytest.mark.parametrize("cfg", [
    dict(shape=(1, 7, 7, 1280), f=(7, 7), s=(1, 1), same=False, dtype=np.uint8),
    dict(shape=(1, 7, 7, 1280), f=(7, 7), s=(1, 1), same=False, dtype=np.int8),
    dict(shape=(2, 13, 11, 6), f=(3, 3), s=(2, 2), same=True, dtype=np.int8),
    dict(shape=(1, 9, 9, 5), f=(2, 2), s=(2, 2), same=True, dtype=np.uint8),
    # wide-window path (pool_wide_kernel): clipped edge windows, several pixels
    dict(shape=(2, 9, 9, 40), f=(5, 5), s=(3, 3), same=True, dtype=np.int8),
    dict(shape=(1, 20, 20, 8), f=(8, 8), s=(4, 4), same=True, dtype=np.uint8),
    dict(shape=(1, 12, 12, 260), f=(12, 12), s=(1, 1), same=False, dtype=np.int8),
    # > 64 taps: 16 waves per workgroup (DeepLab's image pooling; clipped windows)
    dict(shape=(16, 14, 14, 320), f=(14, 14), s=(1, 1), same=False, dtype=np.int8),
    dict(shape=(3, 30, 30, 12), f=(10, 10), s=(7, 7), same=True, dtype=np.uint8),
])
def test_pool(gpu_lib, kind, cfg):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(17)
    x = rand_q(rng, cfg["shape"], cfg["dtype"])
    b, ih, iw, c = x.shape
    (fh, fw), (sh, sw) = cfg["f"], cfg["s"]
    oh, ow = orc.out_size(cfg["same"], ih, fh, sh, 1), orc.out_size(cfg["same"], iw, fw, sw, 1)
    ph, pw = orc.padding(sh, 1, ih, fh, oh), orc.padding(sw, 1, iw, fw, ow)
    signed = cfg["dtype"] == np.int8
    amin, amax = (-128, 127) if signed else (0, 255)
    ref = orc.pool2d(x, kind=kind, filt=(fh, fw), stride=(sh, sw), pad=(ph, pw), out_hw=(oh, ow),
                     amin=amin, amax=amax)
    dx = DeviceBuffer.from_array(x)
    dy = DeviceBuffer(ref.nbytes)
    p = _abi.PoolParams(kind=0 if kind == "avg" else 1, in_signed=int(signed), batch=b, in_h=ih, in_w=iw,
                        channels=c, out_h=oh, out_w=ow, f_h=fh, f_w=fw, stride_h=sh, stride_w=sw,
                        pad_h=ph, pad_w=pw, act_min=amin, act_max=amax, input=dx.value, output=dy.value)
    _abi.check(gpu_lib.bh_pool_i8(ctypes.byref(p), None), "pool")
    np.testing.assert_array_equal(dy.download(x.dtype, ref.shape), ref)


@pytest.mark.parametrize("rows,depth,units,dtype", [
    (1, 1280, 1001, np.int8), (1, 1280, 1001, np.uint8), (3, 37, 10, np.int8), (2, 64, 5, np.uint8),
])
def test_fully_connected(gpu_lib, rows, depth, units, dtype):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(rows * 1000 + depth + units)
    x = rand_q(rng, (rows, depth), dtype)
    w = rand_q(rng, (units, depth), dtype) if dtype == np.uint8 else \
        rng.integers(-127, 128, (units, depth)).astype(np.int8)
    bias = rng.integers(-(1 << 15), 1 << 15, units).astype(np.int32)
    in_zp = int(rng.integers(-128, 128)) if dtype == np.int8 else int(rng.integers(0, 256))
    w_zp = 0 if dtype == np.int8 else int(rng.integers(90, 170))
    in_s, w_s = 0.02, 0.005
    out_s = in_s * w_s * np.sqrt(depth) * 74 * 74 / 40
    out_zp = 3 if dtype == np.int8 else 130
    mult, shift = orc.conv_multipliers(in_s, [w_s], 1, out_s, True)
    amin, amax = orc.act_range(0, out_s, out_zp, dtype == np.int8)
    ref = orc.fully_connected(x, w, bias, in_zp=in_zp, w_zp=w_zp, out_zp=out_zp, mult=mult[0],
                              shift=shift[0], amin=amin, amax=amax)
    # host packing identical to the executor's (int8 domain, bias folding)
    depth_pad = (depth + 15) // 16 * 16
    wd = w.astype(np.int32) - (0 if dtype == np.int8 else 128)
    in_zd, w_zd = dom(in_zp, dtype), dom(w_zp, dtype) if dtype == np.uint8 else 0
    packed = np.zeros((units, depth_pad), np.int8)
    packed[:, :depth] = wd.astype(np.int8)
    beff = (bias.astype(np.int64) - in_zd * wd.sum(1) + depth * in_zd * w_zd).astype(np.int32)
    dx, dy = DeviceBuffer.from_array(x), DeviceBuffer(ref.nbytes)
    dw, db = DeviceBuffer.from_array(packed), DeviceBuffer.from_array(beff)
    dm = DeviceBuffer.from_array(np.full(units, mult[0], np.int32))
    ds = DeviceBuffer.from_array(np.full(units, shift[0], np.int32))
    p = _abi.FcParams(rows=rows, depth=depth, depth_pad=depth_pad, units=units,
                      in_xor=0 if dtype == np.int8 else 0x80, in_zp=in_zd, w_zp=w_zd, out_zp=out_zp,
                      act_min=amin, act_max=amax, input=dx.value, output=dy.value, weights=dw.value,
                      bias_eff=db.value, mult=dm.value, shift=ds.value)
    _abi.check(gpu_lib.bh_fc_i8(ctypes.byref(p), None), "fc")
    np.testing.assert_array_equal(dy.download(dtype, ref.shape), ref)


# conv_group_kernel (bh_conv_group_i8): independent small convs in ONE
# dispatch - detector / pose heads - each member bit-exact with the oracle
# (the same tile arithmetic as its own bh_conv2d_i8 launch): deep and shallow
# K (the split-K and 2x2-wave member forms), N tails, uint8 with a filter zero
# point, batch > 1, and a 3x3 group (the general-window instantiation)
@pytest.mark.parametrize("cases,is1x1", [
    ([(24, 7, 1280, 24), (24, 4, 512, 546), (24, 2, 256, 24), (24, 1, 128, 546), (24, 14, 576, 12)], 1),
    ([(1, 14, 1024, 17), (1, 14, 1024, 34), (1, 14, 1024, 32), (1, 14, 1024, 32)], 1),
    ([(3, 5, 48, 20, np.uint8), (2, 9, 64, 100)], 1),
    ([(24, 14, 576, 200), (5, 20, 128, 512), (2, 3, 32, 8)], 1),  # member forms 2 / 3 / 1
    ([(4, 7, 256, 64, np.int8, 3), (4, 4, 128, 40, np.int8, 3)], 0),
])
def test_conv_group(gpu_lib, cases, is1x1):
    import ctypes
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(7100 + len(cases) + is1x1)
    convs, keep, params = [], [], []
    for c in cases:
        b, sp, ic, oc = c[:4]
        dtype = c[4] if len(c) > 4 else np.int8
        k = c[5] if len(c) > 5 else 1
        cc = ConvCase(rng, b, sp, sp, ic, oc, k, k, dtype=dtype, act=3)
        convs.append(cc)
        params.append(cc.params(gpu_lib, keep))
        cc._dy_keep = cc._dy
    for cc, p in zip(convs, params):
        assert gpu_lib.bh_conv_group_ok(ctypes.byref(p)) == 1
    arr = (_abi.ConvParams * len(params))(*params)
    nbytes = gpu_lib.bh_conv_group_table_bytes(len(params))
    host = np.zeros(nbytes, np.uint8)
    g = _abi.ConvGroup()
    _abi.check(gpu_lib.bh_conv_group_plan(arr, len(params), host.ctypes.data_as(ctypes.c_void_p), ctypes.byref(g)),
               "plan")
    assert g.n == len(params) and g.is1x1 == is1x1
    dt = DeviceBuffer.from_array(host)
    g.table = dt.value
    _abi.check(gpu_lib.bh_conv_group_i8(ctypes.byref(g), None), "bh_conv_group_i8")
    for i, cc in enumerate(convs):
        got = cc._dy_keep.download(cc.dtype, (cc.b, cc.oh, cc.ow, cc.oc))
        np.testing.assert_array_equal(got, cc.oracle(), err_msg="member %d" % i)
    del keep, dt


# a conv storing each image at a row stride into a wider tensor
# (bh_conv_params.out_img_stride: a CONCATENATION slice written in place),
# bytes outside the slice untouched; odd channel counts take the byte path
@pytest.mark.parametrize("b,sp,ic,oc,off,extra", [(4, 7, 64, 12, 0, 100), (3, 4, 96, 273, 37, 555),
                                                   (2, 2, 128, 546, 1001, 3)])
def test_conv_strided_image_output(gpu_lib, b, sp, ic, oc, off, extra):
    import ctypes
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(7300 + oc)
    c = ConvCase(rng, b, sp, sp, ic, oc, 1, 1, act=3)
    keep = []
    p = c.params(gpu_lib, keep)
    per = sp * sp * oc
    stride = off + per + extra
    fill = np.full(b * stride, 0x5a, np.uint8)
    dbig = DeviceBuffer.from_array(fill)
    p.output = dbig.value + off
    p.out_img_stride = stride
    _abi.check(gpu_lib.bh_conv2d_i8(ctypes.byref(p), None), "bh_conv2d_i8")
    got = dbig.download(np.uint8, (b * stride,))
    ref = c.oracle().reshape(b, per).view(np.uint8)
    for n in range(b):
        np.testing.assert_array_equal(got[n * stride + off:n * stride + off + per], ref[n], err_msg="image %d" % n)
        assert (got[n * stride:n * stride + off] == 0x5a).all()
        assert (got[n * stride + off + per:(n + 1) * stride] == 0x5a).all()
    del keep
