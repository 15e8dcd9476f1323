"""MIRROR_PAD, int8 MEAN, SQUARED_DIFFERENCE and RSQRT (the ops of the
reference's magenta style-transfer fixture outside the round-1 kernel set)
on the kCPU executor vs the oracle restatements (oracle/runner.py:
mirror_pad, mean_q8_hw, squared_difference_f32, rsqrt_f32).  MEAN's parity
is unpinned (no reference fixture holds MEAN outputs); the float ops are
exact here (same float32 operation order)."""
import numpy as np

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
from oracle import runner as orc
from tests.glue_models import norm_zoo


def norm_zoo_oracle(x, with_mean=True):
    xr = orc.mirror_pad(x, [[0, 0], [2, 1], [1, 2], [0, 0]], "REFLECT")
    xs = orc.mirror_pad(x, [[0, 0], [3, 0], [0, 11], [1, 0]], "SYMMETRIC")
    outs = [xr, xs]
    if with_mean:
        q = orc.quantize_f32(xr, scale=0.02, zp=-3, out_dtype=np.int8)
        m = orc.mean_q8_hw(q, in_scale=0.02, in_zp=-3, out_scale=0.011, out_zp=2)
        c = orc.dequantize(m, scale=0.011, zp=2)
        outs.append(m)
    else:
        c = np.linspace(-0.3, 0.4, 4).astype(np.float32).reshape(1, 1, 1, 4)
    sd = orc.squared_difference_f32(xr, c)
    r = orc.rsqrt_f32((sd + np.float32(1e-3)).astype(np.float32))
    return outs + [sd, r]


def run_executor(buf, x, flag, worker=0):
    m = HipModel(0)
    assert m.FromBuffer(buf).ok()
    ex = HipModelExecutor(0, worker, flag)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, worker)
    ex.GetTensorView(key, ex.GetInputs(key)[0]).GetData()[...] = x
    assert ex.ExecuteSubgraph(key).ok()
    return [ex.GetTensorView(key, t).GetData().copy() for t in ex.GetOutputs(key)]


def test_norm_zoo_cpu_executor():
    x = np.random.default_rng(1).uniform(-1, 1, (1, 9, 11, 4)).astype(np.float32)
    got = run_executor(norm_zoo(), x, DeviceFlag.kCPU)
    ref = norm_zoo_oracle(x)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g.reshape(r.shape), r)


def test_mean_requant_edges():
    """the MEAN restatement at saturation and rounding ties: all -128 / +127
    inputs, and zero-point-only inputs"""
    for v in (-128, 127, -3):
        q = np.full((2, 5, 7, 3), v, np.int8)
        m = orc.mean_q8_hw(q, in_scale=0.02, in_zp=-3, out_scale=0.011, out_zp=2)
        assert m.shape == (2, 1, 1, 3) and len(np.unique(m)) == 1
    # zero-point-only input: TFLite's separately rounded bias and double-rounded
    # MultiplyByQuantizedMultiplier land within 1 of the output zero point
    # (here -48 * 0.1136 -> SaturatingRoundingDoublingHighMul -44 ->
    # RoundingDivideByPOT(-44, 3) = -6, bias 7: 1, not 2)
    assert orc.mean_q8_hw(np.full((1, 4, 4, 1), -3, np.int8), in_scale=0.02, in_zp=-3, out_scale=0.011,
                          out_zp=2).item() == 1


import pytest  # noqa: E402

from tests.glue_models import HARD_SWISH_CASES, all_bytes, hard_swish_model  # noqa: E402


@pytest.mark.parametrize("dtype,s_in,zp_in,s_out,zp_out", HARD_SWISH_CASES)
def test_hard_swish_cpu_executor(dtype, s_in, zp_in, s_out, zp_out):
    """HARD_SWISH as the executor's 256-entry table (kCPU worker) vs the
    oracle's element-wise restatement, every input byte.  Parity unpinned (no
    reference fixture holds HARD_SWISH outputs); the fixed-point result stays
    within 1 of the float formula x * relu6(x + 3) / 6."""
    x = all_bytes(dtype)
    got = run_executor(hard_swish_model(dtype, s_in, zp_in, s_out, zp_out), x, DeviceFlag.kCPU)[0]
    ref = orc.hard_swish_q8(x, in_scale=s_in, in_zp=zp_in, out_scale=s_out, out_zp=zp_out)
    np.testing.assert_array_equal(got.reshape(ref.shape), ref)
    xf = np.float32(s_in) * (x.astype(np.float32) - zp_in)
    lo, hi = (-128, 127) if np.dtype(dtype) == np.int8 else (0, 255)
    fl = np.clip(np.round(xf * np.clip(xf + 3, 0, 6) / 6 / s_out) + zp_out, lo, hi)
    assert np.abs(ref.astype(np.int32) - fl).max() <= 1


from tests.glue_models import BILINEAR_CASES, bilinear_model, bilinear_u8_numpy  # noqa: E402


@pytest.mark.parametrize("in_hw,out_hw,c,ac,hp", BILINEAR_CASES)
def test_resize_bilinear_u8_cpu_executor(in_hw, out_hw, c, ac, hp):
    """uint8 RESIZE_BILINEAR (optimized_ops::ResizeBilinear float path) on the
    kCPU worker vs the C oracle, and the C oracle vs a numpy float32
    restatement.  Parity unpinned: no reference fixture holds uint8 bilinear
    outputs."""
    rng = np.random.default_rng(in_hw[0] * 31 + out_hw[1])
    x = rng.integers(0, 256, (2, in_hw[0], in_hw[1], c)).astype(np.uint8)
    x.flat[:4] = [0, 255, 255, 0]
    ref = orc.resize_bilinear_u8(x, out_hw, ac, hp)
    np.testing.assert_array_equal(ref, bilinear_u8_numpy(x, out_hw, ac, hp))
    got = run_executor(bilinear_model(np.uint8, in_hw, out_hw, c, ac, hp), x, DeviceFlag.kCPU)[0]
    np.testing.assert_array_equal(got.reshape(ref.shape), ref)
