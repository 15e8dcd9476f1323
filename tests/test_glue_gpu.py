"""Glue ops on the MI355X: kernel-level parity of each
C-ABI launcher against the oracle's restatement of the TFLite 2.9.2 kernel,
then whole models through the HIP executor (synthetic glue-op models and the
reference's own int8 retinaface, every tensor bit-exact)."""
import ctypes
import os

import numpy as np
import pytest

from oracle import runner as orc
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model
from tests.kernel_harness import rand_q

pytestmark = pytest.mark.gpu


def _dev(a):
    from band_amd.device import DeviceBuffer
    return DeviceBuffer.from_array(np.ascontiguousarray(a))


def _check(rc, what):
    from band_amd import _abi
    _abi.check(rc, what)


@pytest.mark.parametrize("n,offset", [(4096, 0), (1000, 0), (37, 0), (777, 3)])
def test_lut_u8_requantize_table(gpu_lib, n, offset):
    """QUANTIZE int8 -> uint8 through the table gather: aligned 16-byte path,
    tails and a misaligned (byte path) view"""
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(n)
    x = rand_q(rng, (n + offset,), np.int8)
    ref = orc.requantize(x[offset:], in_scale=0.03, in_zp=-5, out_scale=0.07, out_zp=120, out_dtype=np.uint8)
    table = orc.requantize(np.arange(256, dtype=np.uint8).view(np.int8), in_scale=0.03, in_zp=-5,
                           out_scale=0.07, out_zp=120, out_dtype=np.uint8)
    dx, dt, dy = _dev(x), _dev(table), DeviceBuffer(n + offset)
    _check(gpu_lib.bh_lut_u8(dx.value + offset, dy.value + offset, n, dt.value, None), "lut")
    np.testing.assert_array_equal(dy.download(np.uint8, (n + offset,))[offset:], ref)


def test_lut_f32_and_quantize_f32(gpu_lib):
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(1)
    x = rand_q(rng, (3001,), np.uint8)
    ref = orc.dequantize(x, scale=0.0123, zp=131)
    table = orc.dequantize(np.arange(256, dtype=np.uint8), scale=0.0123, zp=131)
    dx, dt, dy = _dev(x), _dev(table), DeviceBuffer(4 * x.size)
    _check(gpu_lib.bh_lut_f32(dx.value, dy.value, x.size, dt.value, None), "lut_f32")
    np.testing.assert_array_equal(dy.download(np.float32, x.shape), ref)
    f = (rng.standard_normal(5000) * 3).astype(np.float32)
    f[:8] = [0.5, -0.5, 1.5, -2.5, 0.0249999, 1e9, -1e9, 0.075]  # ties and saturation
    for dtype, zp in ((np.int8, -3), (np.uint8, 128)):
        ref = orc.quantize_f32(f, scale=0.025, zp=zp, out_dtype=dtype)
        df, dq = _dev(f), DeviceBuffer(f.size)
        _check(gpu_lib.bh_quantize_f32(df.value, dq.value, f.size, ctypes.c_float(0.025), zp,
                                       int(dtype == np.int8), None), "quantize")
        np.testing.assert_array_equal(dq.download(dtype, f.shape), ref)


@pytest.mark.parametrize("shapes,axis,dtype", [
    ([(1, 5, 6, 8), (1, 5, 6, 4), (1, 5, 6, 12)], 3, np.int8),     # dword path
    ([(2, 3, 4, 3), (2, 3, 4, 5)], 3, np.int8),                    # byte path
    ([(1, 4, 6, 8), (1, 2, 6, 8), (1, 7, 6, 8)], 1, np.uint8),     # rescaled uint8
    ([(3, 10), (3, 6), (3, 1)], 1, np.uint8),
])
def test_concat(gpu_lib, shapes, axis, dtype):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(len(shapes) * 10 + axis)
    xs = [rand_q(rng, s, dtype) for s in shapes]
    signed = dtype == np.int8
    scales = [0.05] * len(xs) if signed else [float(rng.uniform(0.02, 0.08)) for _ in xs]
    zps = [4] * len(xs) if signed else [int(rng.integers(100, 156)) for _ in xs]
    out_s, out_z = (0.05, 4) if signed else (0.08, 127)
    ref = orc.concat(xs, axis, scales=scales, zps=zps, out_scale=out_s, out_zp=out_z)
    p = _abi.ConcatParams()
    p.n_inputs = len(xs)
    keep = []
    outer = int(np.prod(ref.shape[:axis]))
    inner = int(np.prod(ref.shape[axis + 1:]))
    p.outer = outer
    for k, x in enumerate(xs):
        d = _dev(x)
        keep.append(d)
        p.input[k] = d.value
        p.row[k] = x.shape[axis] * inner
        if not signed and (scales[k] != out_s or zps[k] != out_z):
            t = orc.concat([np.arange(256, dtype=np.uint8).reshape(256, 1)], 1, scales=[scales[k]], zps=[zps[k]],
                           out_scale=out_s, out_zp=out_z).reshape(-1)
            # single-input concat with scaling = the rescale map itself
            dt = _dev(t)
            keep.append(dt)
            p.table[k] = dt.value
    dy = DeviceBuffer(ref.nbytes)
    p.output = dy.value
    _check(gpu_lib.bh_concat(ctypes.byref(p), None), "concat")
    np.testing.assert_array_equal(dy.download(dtype, ref.shape), ref)


@pytest.mark.parametrize("shape,pads,elem", [
    ((1, 7, 9, 5), [[0, 0], [1, 2], [3, 0], [0, 0]], 1),
    ((2, 4, 4, 3), [[1, 0], [0, 1], [2, 2], [1, 1]], 1),
    ((1, 5, 5, 4), [[0, 0], [2, 2], [2, 2], [0, 0]], 4),
])
def test_pad(gpu_lib, shape, pads, elem):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(elem)
    if elem == 1:
        x = rand_q(rng, shape, np.int8)
        ref = orc.pad(x, pads, -7)
        value = (-7) & 0xff
    else:
        x = rng.standard_normal(shape).astype(np.float32)
        ref = np.pad(x, pads, constant_values=0.0)
        value = 0
    p = _abi.PadParams(elem_bytes=elem, value=value)
    for d in range(4):
        p.in_shape[d] = shape[d]
        p.pad_before[d], p.pad_after[d] = pads[d]
    dx, dy = _dev(x), DeviceBuffer(ref.nbytes)
    p.input, p.output = dx.value, dy.value
    _check(gpu_lib.bh_pad(ctypes.byref(p), None), "pad")
    np.testing.assert_array_equal(dy.download(x.dtype, ref.shape), ref)


# b >= 16 with tall outputs: the column-blend form's multi-row workgroups
# (DeepLab's batch-32 upsample; 261 rows = 65 groups of 4 + one of 1, with a
# 493-byte row that takes the byte-store tail)
@pytest.mark.parametrize("ih,iw,oh,ow,c,ac,hp,b", [
    (5, 5, 10, 10, 8, 0, 0, 2), (10, 10, 20, 20, 3, 0, 1, 2), (7, 9, 13, 4, 4, 1, 0, 2), (6, 6, 3, 3, 5, 0, 1, 2),
    (14, 14, 224, 224, 21, 0, 0, 2), (14, 14, 224, 224, 16, 1, 0, 2), (3, 5, 37, 41, 7, 0, 1, 2),
    (2, 515, 3, 1030, 1, 0, 0, 2), (14, 14, 224, 224, 21, 0, 0, 32), (5, 7, 261, 29, 17, 0, 1, 16),
])
def test_resize(gpu_lib, ih, iw, oh, ow, c, ac, hp, b):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(ih * 100 + oh)
    x = rand_q(rng, (b, ih, iw, c), np.int8)
    # nearest: host-built index tables, as the executor builds them
    yi = np.array([orc.nearest_index(y, ih, oh, ac, hp) for y in range(oh)], np.int32)
    xi = np.array([orc.nearest_index(v, iw, ow, ac, hp) for v in range(ow)], np.int32)
    ref = orc.resize_nearest(x, (oh, ow), ac, hp)
    dx, dyi, dxi, dy = _dev(x), _dev(yi), _dev(xi), DeviceBuffer(ref.nbytes)
    p = _abi.ResizeNearestParams(batch=b, in_h=ih, in_w=iw, out_h=oh, out_w=ow, row_bytes=c,
                                 y_index=dyi.value, x_index=dxi.value, input=dx.value, output=dy.value)
    _check(gpu_lib.bh_resize_nearest(ctypes.byref(p), None), "nearest")
    np.testing.assert_array_equal(dy.download(np.int8, ref.shape), ref)
    # bilinear int8 (ResizeBilinearInteger)
    ref = orc.resize_bilinear_i8(x, (oh, ow), ac, hp)

    def tab(n_in, n_out):
        s = ((1 << 10) * n_in + n_out // 2) // n_out
        if ac and n_out > 1:
            s = ((1 << 10) * (n_in - 1) + (n_out - 1) // 2) // (n_out - 1)
        t = []
        for v in range(n_out):
            sc = v * s + s // 2 - (1 << 9) if hp else v * s
            lo = max(int(np.trunc(sc / 1024)), 0)
            hi = min(int(np.trunc((sc + 1023) / 1024)), n_in - 1)
            t += [lo, hi, sc]
        return np.array(t, np.int32)
    dty, dtx, dy2 = _dev(tab(ih, oh)), _dev(tab(iw, ow)), DeviceBuffer(ref.nbytes)
    q = _abi.ResizeBilinearParams(batch=b, in_h=ih, in_w=iw, channels=c, out_h=oh, out_w=ow, y_tab=dty.value,
                                  x_tab=dtx.value, input=dx.value, output=dy2.value)
    _check(gpu_lib.bh_resize_bilinear_i8(ctypes.byref(q), None), "bilinear")
    np.testing.assert_array_equal(dy2.download(np.int8, ref.shape), ref)


@pytest.mark.parametrize("ih,iw,oh,ow,c,ac,hp", [
    (5, 5, 10, 10, 8, 0, 0), (10, 10, 20, 20, 3, 0, 1), (7, 9, 13, 4, 4, 1, 0), (14, 14, 224, 224, 21, 0, 0),
    (2, 515, 3, 1030, 1, 0, 1),
])
def test_resize_bilinear_u8(gpu_lib, ih, iw, oh, ow, c, ac, hp):
    """uint8 bilinear launcher with host float tables (the executor's
    BilinearFloatTable restated in numpy float32) vs the oracle"""
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(ih * 7 + ow)
    x = rng.integers(0, 256, (2, ih, iw, c)).astype(np.uint8)
    ref = orc.resize_bilinear_u8(x, (oh, ow), ac, hp)
    f32 = np.float32

    def tab(n_in, n_out):
        s = f32(n_in - 1) / f32(n_out - 1) if ac and n_out > 1 else f32(n_in) / f32(n_out)
        v = np.arange(n_out, dtype=f32)
        sc = (v + f32(0.5)) * s - f32(0.5) if hp else v * s
        lo = np.maximum(np.floor(sc).astype(np.int32), 0)
        hi = np.minimum(np.ceil(sc).astype(np.int32), n_in - 1)
        return np.stack([lo, hi], 1).astype(np.int32).reshape(-1), (sc - lo.astype(f32)).astype(f32)
    yi, yf = tab(ih, oh)
    xi, xf = tab(iw, ow)
    keep = [_dev(a) for a in (x, yi, xi, yf, xf)]
    dy = DeviceBuffer(ref.nbytes)
    q = _abi.ResizeBilinearU8Params(batch=2, in_h=ih, in_w=iw, channels=c, out_h=oh, out_w=ow, y_idx=keep[1].value,
                                    x_idx=keep[2].value, y_frac=keep[3].value, x_frac=keep[4].value,
                                    input=keep[0].value, output=dy.value)
    _check(gpu_lib.bh_resize_bilinear_u8(ctypes.byref(q), None), "bilinear_u8")
    np.testing.assert_array_equal(dy.download(np.uint8, ref.shape), ref)


@pytest.mark.parametrize("dtype,depth", [(np.int8, 2), (np.int8, 91), (np.uint8, 10)])
def test_softmax(gpu_lib, dtype, depth):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(depth)
    x = rand_q(rng, (3, 7, depth), dtype)
    in_s, beta = 0.09, 1.3
    zp = -128 if dtype == np.int8 else 0
    ref = orc.softmax(x, in_scale=in_s, beta=beta, out_scale=1 / 256, out_zp=zp)
    t2 = orc.softmax_table(in_s, beta)
    dx, dt, dy = _dev(x), _dev(t2), DeviceBuffer(x.nbytes)
    p = _abi.SoftmaxParams(rows=x.size // depth, depth=depth, is_signed=int(dtype == np.int8), table=dt.value,
                           out_scale=1 / 256, out_zp=zp, input=dx.value, output=dy.value)
    _check(gpu_lib.bh_softmax_i8(ctypes.byref(p), None), "softmax")
    np.testing.assert_array_equal(dy.download(dtype, x.shape), ref)


def _run_model(buf, mid, feed_seed=0, all_tensors=True):
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
    om = Model(buf)
    model = HipModel(mid)
    assert model.FromBuffer(buf).ok()
    ex = HipModelExecutor(mid, 1, DeviceFlag.kGPU)
    spec = ex.InvestigateModelSpec(model)
    assert spec.unsupported_ops[DeviceFlag.kGPU] == set(), spec.unsupported_ops[DeviceFlag.kGPU]
    assert ex.PrepareSubgraph(model).ok()
    key = SubgraphKey(mid, 1)
    inter = sorted({t for o in om.operators for t in o.outputs}) if all_tensors else list(om.outputs)
    views = {t: ex.GetTensorView(key, t) for t in inter}
    rng = np.random.default_rng(feed_seed)
    feed = {}
    for t in om.inputs:
        tt = om.tensors[t]
        feed[t] = rand_q(rng, tt.shape, tt.np_dtype)
        ex.GetTensorView(key, t).GetData()[...] = feed[t]
    ref = OracleInterpreter(om).run(feed)
    for _ in range(2):  # eager, then captured graph
        assert ex.ExecuteSubgraph(key).ok()
        for t in inter:
            np.testing.assert_array_equal(views[t].GetData(), ref[t].reshape(views[t].GetDims()),
                                          err_msg="tensor %d (%s)" % (t, om.tensors[t].name))
    return om


@pytest.mark.parametrize("dtype", [np.int8, np.uint8])
@pytest.mark.parametrize("all_tensors", [True, False])
def test_glue_zoo_model(gpu_lib, dtype, all_tensors):
    """all_tensors=False views only the outputs, so every fusion is active"""
    from tests.glue_models import glue_zoo
    _run_model(glue_zoo(dtype), 40 + int(dtype == np.uint8), all_tensors=all_tensors)


@pytest.mark.parametrize("dtype", [np.int8, np.uint8])
@pytest.mark.parametrize("all_tensors", [True, False])
def test_fpn_merge_not_fused_across_later_producer(gpu_lib, dtype, all_tensors):
    from tests.glue_models import fpn
    _run_model(fpn(dtype), 42 + int(dtype == np.uint8), all_tensors=all_tensors)


@pytest.mark.parametrize("all_tensors", [True, False])
def test_retinaface_whole_model(gpu_lib, golden_dir, all_tensors):
    """The reference's int8 retinaface (PAD, QUANTIZE, CONCATENATION, RELU,
    RESIZE_NEAREST_NEIGHBOR, RESHAPE, SOFTMAX around the conv stack) runs
    whole on the GPU; every tensor (or, with fusion active, every output)
    matches the oracle."""
    with open(os.path.join(golden_dir, "retinaface_mbv2_quant_160.tflite"), "rb") as f:
        buf = f.read()
    _run_model(buf, 45 + int(all_tensors), all_tensors=all_tensors)


def test_zero_insert(gpu_lib):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(9)
    for shape, (sh, sw), fill in (((2, 5, 7, 8), (2, 2), -3), ((1, 4, 3, 5), (3, 2), 17)):
        x = rand_q(rng, shape, np.int8)
        b, ih, iw, c = shape
        uh, uw = (ih - 1) * sh + 1, (iw - 1) * sw + 1
        ref = np.full((b, uh, uw, c), fill, np.int8)
        ref[:, ::sh, ::sw, :] = x
        dx, dy = _dev(x), DeviceBuffer(ref.nbytes)
        p = _abi.ZeroInsertParams(batch=b, in_h=ih, in_w=iw, channels=c, stride_h=sh, stride_w=sw, out_h=uh,
                                  out_w=uw, fill=fill & 0xff, input=dx.value, output=dy.value)
        _check(gpu_lib.bh_zero_insert(ctypes.byref(p), None), "zero_insert")
        np.testing.assert_array_equal(dy.download(np.int8, ref.shape), ref)


@pytest.mark.parametrize("all_tensors", [True, False])
def test_transpose_conv_models(gpu_lib, all_tensors):
    """TRANSPOSE_CONV as zero insertion + stride-1 MFMA conv with flipped
    filters, against the oracle's restatement of TFLite's scatter kernel"""
    from tests.glue_models import tconv_zoo
    _run_model(tconv_zoo(), 50 + int(all_tensors), all_tensors=all_tensors)


@pytest.mark.parametrize("all_tensors", [True, False])
def test_icn_whole_model(gpu_lib, golden_dir, all_tensors):
    """The reference's int8 ICN (47 CONV_2D, 22 ADD, 4 TRANSPOSE_CONV,
    DEPTHWISE, QUANTIZE, CONCATENATION) runs whole on the GPU"""
    with open(os.path.join(golden_dir, "ICN_quant.tflite"), "rb") as f:
        buf = f.read()
    _run_model(buf, 52 + int(all_tensors), all_tensors=all_tensors)
