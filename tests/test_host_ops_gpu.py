"""MIRROR_PAD / SQUARED_DIFFERENCE / RSQRT / MEAN / HARD_SWISH on the GPU
(pad_kernel's mirror mode, eltwise_f32_kernel, unary_f32_kernel,
mean_kernel, the HARD_SWISH byte table) vs the oracle restatements, and the
reference's magenta style-transfer fixture through a Band engine over
[CPU, GPU] workers against the CPU-only engine.  Float tolerance as the other
float tests: |got - ref| <= 1e-3 |ref| + 1e-4 max(1, max |ref|)."""
import ctypes
import os

import numpy as np
import pytest

from band_amd import DeviceFlag
from tests.glue_models import norm_zoo
from tests.test_host_ops_cpu import norm_zoo_oracle, run_executor

pytestmark = pytest.mark.gpu


def _close(got, ref):
    ref = np.asarray(ref, np.float64)
    tol = 1e-3 * np.abs(ref) + 1e-4 * max(1.0, float(np.abs(ref).max()))
    assert np.all(np.abs(np.asarray(got, np.float64) - ref) <= tol)


def test_norm_zoo_gpu_executor(gpu_lib):
    x = np.random.default_rng(2).uniform(-1, 1, (1, 9, 11, 4)).astype(np.float32)
    got = run_executor(norm_zoo(with_mean=False), x, DeviceFlag.kGPU, worker=1)
    ref = norm_zoo_oracle(x, with_mean=False)
    np.testing.assert_array_equal(got[0].reshape(ref[0].shape), ref[0])  # mirror pads: copies
    np.testing.assert_array_equal(got[1].reshape(ref[1].shape), ref[1])
    for g, r in zip(got[2:], ref[2:]):
        _close(g.reshape(r.shape), r)


@pytest.mark.parametrize("dtype,shape,pads,mode", [
    (np.int8, (2, 5, 7, 3), [[0, 0], [4, 3], [2, 6], [0, 0]], "REFLECT"),
    (np.uint8, (1, 6, 4, 5), [[1, 0], [6, 6], [0, 4], [2, 5]], "SYMMETRIC"),
    (np.float32, (1, 384, 384, 3), [[0, 0], [4, 4], [4, 4], [0, 0]], "REFLECT"),
])
def test_mirror_pad_launcher(gpu_lib, dtype, shape, pads, mode):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    from oracle import runner as orc
    rng = np.random.default_rng(sum(shape))
    x = (rng.standard_normal(shape) * 40).astype(dtype)
    ref = orc.mirror_pad(x, pads, mode)
    dx, dy = DeviceBuffer.from_array(x), DeviceBuffer(ref.nbytes)
    p = _abi.PadParams(elem_bytes=np.dtype(dtype).itemsize, mode=1 if mode == "REFLECT" else 2,
                       input=dx.value, output=dy.value)
    for d in range(4):
        p.in_shape[d] = shape[d]
        p.pad_before[d], p.pad_after[d] = pads[d]
    _abi.check(gpu_lib.bh_pad(ctypes.byref(p), None), "mirror pad")
    np.testing.assert_array_equal(dy.download(dtype, ref.shape), ref)
    # a mirror pad wider than the input is refused
    p.pad_before[1] = shape[1] + (0 if mode == "REFLECT" else 1)
    assert gpu_lib.bh_pad(ctypes.byref(p), None) != 0


def test_magenta_cpu_gpu_engine(golden_dir, tmp_path):
    from band_amd.engine import (CPUMaskFlag, Engine, Model, SchedulerType, SubgraphPreparationType, kBandOk,
                                 make_config)
    path = os.path.join(golden_dir, "magenta_arbitrary-image-stylization-v1-256_int8_transfer_1.tflite")
    rng = np.random.default_rng(5)
    outs = {}
    for label, workers in (("cpu", [DeviceFlag.kCPU]), ("cpu+gpu", [DeviceFlag.kCPU, DeviceFlag.kGPU])):
        cfg = make_config([SchedulerType.kHeterogeneousEarliestFinishTime], workers, num_threads=[4] * len(workers),
                          num_warmups=1, num_runs=1, profile_path=str(tmp_path / ("p_%s.json" % label)),
                          subgraph_type=SubgraphPreparationType.kMergeUnitSubgraph, minimum_subgraph_size=7)
        e = Engine(cfg)
        m = Model()
        assert m.FromPath(path)
        assert e.RegisterModel(m)
        ins = []
        for i in range(e.GetNumInputTensors(m)):
            t = e.CreateInputTensor(m, i)
            t.data()[...] = np.random.default_rng(10 + i).uniform(0, 1, t.data().shape)
            ins.append(t)
        o = e.CreateOutputTensor(m, 0)
        assert e.RequestSync(m, ins, [o]) == kBandOk
        outs[label] = o.data().copy()
        e.close()
    _close(outs["cpu+gpu"], outs["cpu"])


from oracle import runner as orc  # noqa: E402
from tests.glue_models import HARD_SWISH_CASES, all_bytes, hard_swish_model  # noqa: E402


@pytest.mark.parametrize("dtype,s_in,zp_in,s_out,zp_out", HARD_SWISH_CASES)
def test_hard_swish_gpu_executor(gpu_lib, dtype, s_in, zp_in, s_out, zp_out):
    x = all_bytes(dtype)
    got = run_executor(hard_swish_model(dtype, s_in, zp_in, s_out, zp_out), x, DeviceFlag.kGPU, worker=1)[0]
    ref = orc.hard_swish_q8(x, in_scale=s_in, in_zp=zp_in, out_scale=s_out, out_zp=zp_out)
    np.testing.assert_array_equal(got.reshape(ref.shape), ref)


def test_norm_zoo_gpu_executor_with_mean(gpu_lib):
    """the whole norm zoo, int8 MEAN included, on one GPU executor"""
    x = np.random.default_rng(3).uniform(-1, 1, (1, 9, 11, 4)).astype(np.float32)
    got = run_executor(norm_zoo(), x, DeviceFlag.kGPU, worker=1)
    ref = norm_zoo_oracle(x)
    for g, r in zip(got[:3], ref[:3]):  # mirror pads, int8 MEAN: exact
        np.testing.assert_array_equal(g.reshape(r.shape), r)
    for g, r in zip(got[3:], ref[3:]):
        _close(g.reshape(r.shape), r)


@pytest.mark.parametrize("dtype,shape", [(np.int8, (2, 7, 7, 1280)), (np.uint8, (3, 14, 9, 40)),
                                         (np.int8, (1, 56, 56, 24)), (np.float32, (2, 7, 7, 96))])
def test_mean_launcher(gpu_lib, dtype, shape):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    rng = np.random.default_rng(sum(shape))
    if dtype == np.float32:
        x = rng.standard_normal(shape).astype(np.float32)
        ref = x.mean(axis=(1, 2), keepdims=True, dtype=np.float64)
        m, sh, bias = 0, 0, 0
    else:
        lo, hi = (-128, 128) if dtype == np.int8 else (0, 256)
        x = rng.integers(lo, hi, shape).astype(dtype)
        s_in, zp_in, s_out, zp_out = 0.02, int(rng.integers(lo, hi)), 0.013, int(rng.integers(lo // 4, hi // 4))
        ref = orc.mean_q8_hw(x, in_scale=s_in, in_zp=zp_in, out_scale=s_out, out_zp=zp_out)
        n = np.float32(shape[1] * shape[2])
        bias = zp_out - int(np.float32(np.float32(np.float32(zp_in) * np.float32(s_in)) / np.float32(s_out)))
        m, sh = orc.quantize_multiplier(float(np.float32(np.float32(s_in) / np.float32(n * np.float32(s_out)))))
    dx = DeviceBuffer.from_array(x)
    dy = DeviceBuffer(ref.size * np.dtype(dtype).itemsize)
    p = _abi.MeanParams(outer=shape[0], reduce=shape[1] * shape[2], inner=shape[3],
                        type={np.float32: 0, np.int8: 1, np.uint8: 2}[dtype], multiplier=m, shift=sh, bias=bias,
                        input=dx.value, output=dy.value)
    _abi.check(gpu_lib.bh_mean(ctypes.byref(p), None), "bh_mean")
    got = dy.download(dtype, ref.shape)
    if dtype == np.float32:
        _close(got, ref)
    else:
        np.testing.assert_array_equal(got, ref)
    p.reduce = 0
    assert gpu_lib.bh_mean(ctypes.byref(p), None) != 0


from tests.glue_models import BILINEAR_CASES, bilinear_model  # noqa: E402


@pytest.mark.parametrize("in_hw,out_hw,c,ac,hp", BILINEAR_CASES + [((14, 14), (224, 224), 21, 0, 0)])
def test_resize_bilinear_u8_gpu_executor(gpu_lib, in_hw, out_hw, c, ac, hp):
    """uint8 RESIZE_BILINEAR through resize_bilinear_u8_kernel vs the oracle"""
    rng = np.random.default_rng(in_hw[0] * 31 + out_hw[1])
    x = rng.integers(0, 256, (2, in_hw[0], in_hw[1], c)).astype(np.uint8)
    got = run_executor(bilinear_model(np.uint8, in_hw, out_hw, c, ac, hp), x, DeviceFlag.kGPU, worker=1)[0]
    ref = orc.resize_bilinear_u8(x, out_hw, ac, hp)
    np.testing.assert_array_equal(got.reshape(ref.shape), ref)
