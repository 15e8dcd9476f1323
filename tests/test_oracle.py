"""Pin the CPU oracle against the reference's own known-answer tests.

* band/test/backend/tfl_minimal_test.cc:379-457 (ClassificationQuantTest) and
  band/test/c/c_api_test.cc:266-320: mobilenet_v2_1.0_224_quant.tflite (uint8,
  per-tensor) on cat.jpg resized to 224x224 -> argmax 282 (tiger cat).
* band/test/backend/tfl_minimal_test.cc:62-90 (InterfaceInvoke): add.tflite,
  input {1, 3, ...} -> output {3, 9, ...}.
* band/test/backend/tfl_minimal_test.cc:36-51 (ModelSpec): add.tflite has
  2 ops, 1 input, 1 output.
"""
import os

import numpy as np
import pytest

from oracle import runner as orc
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model


def load_cat(golden_dir):
    from PIL import Image
    img = Image.open(os.path.join(golden_dir, "cat.jpg")).convert("RGB")
    return np.asarray(img.resize((224, 224), Image.BILINEAR), np.uint8)[None]


def test_mobilenet_v2_quant_cat_is_282(golden_dir):
    m = Model.from_path(os.path.join(golden_dir, "mobilenet_v2_1.0_224_quant.tflite"))
    vals = OracleInterpreter(m).run({m.inputs[0]: load_cat(golden_dir)})
    out = vals[m.outputs[0]].reshape(-1)
    assert out.dtype == np.uint8 and out.shape == (1001,)
    assert int(np.argmax(out)) == 282


def test_add_known_answer(golden_dir):
    m = Model.from_path(os.path.join(golden_dir, "add.tflite"))
    assert len(m.operators) == 2 and len(m.inputs) == 1 and len(m.outputs) == 1
    x = np.zeros((1, 8, 8, 3), np.float32)
    x.flat[0], x.flat[1] = 1, 3
    out = OracleInterpreter(m).run({m.inputs[0]: x})[m.outputs[0]]
    assert out.flat[0] == 3 and out.flat[1] == 9


# Hand-checked fixed-point facts of TFLite's common.h / quantization_util.cc.
def test_quantize_multiplier_facts():
    assert orc.quantize_multiplier(0.5) == (1 << 30, 0)
    assert orc.quantize_multiplier(1.0) == (1 << 30, 1)
    assert orc.quantize_multiplier(0.0) == (0, 0)
    # 2^-40 flushes to zero (shift < -31)
    assert orc.quantize_multiplier(2.0 ** -40) == (0, 0)
    # q rounds to 2^31 -> halved, exponent incremented
    q, s = orc.quantize_multiplier(1.0 - 2.0 ** -40)
    assert (q, s) == (1 << 30, 1)


def test_fixed_point_rounding_facts():
    L = orc.lib()
    # SaturatingRoundingDoublingHighMul saturates only for INT_MIN*INT_MIN
    assert L.tfl_srdhm(-2 ** 31, -2 ** 31) == 2 ** 31 - 1
    # round half away from zero in RoundingDivideByPOT
    assert L.tfl_rdbypot(5, 1) == 3 and L.tfl_rdbypot(-5, 1) == -3
    assert L.tfl_rdbypot(4, 1) == 2 and L.tfl_rdbypot(-4, 1) == -2
    assert L.tfl_rdbypot(6, 2) == 2 and L.tfl_rdbypot(-6, 2) == -2
    # MultiplyByQuantizedMultiplier(x, 0.5 in Q31, 0): gemmlowp's nudge rounds
    # +3.5 up to 4 but -3.5 to -3 (the negative nudge is 1 - 2^30).
    assert L.tfl_mbqm(7, 1 << 30, 0) == 4 and L.tfl_mbqm(-7, 1 << 30, 0) == -3
    # with a right shift the final RoundingDivideByPOT rounds half away from 0
    assert L.tfl_mbqm(-12, 1 << 30, -2) == -2 and L.tfl_mbqm(12, 1 << 30, -2) == 2


def test_activation_ranges():
    assert orc.act_range(3, 0.0235, 0, False) == (0, 255)  # RELU6 on uint8 MNv2 scale
    assert orc.act_range(3, 0.05, -128, True) == (-128, -8)
    assert orc.act_range(1, 0.1, 5, True) == (5, 127)
    assert orc.act_range(0, 0.1, 5, True) == (-128, 127)


def test_padding_rules():
    # SAME, stride 2, 224 -> 112, pad 0 (TFLite puts the odd pixel at the end)
    assert orc.out_size(True, 224, 3, 2, 1) == 112
    assert orc.padding(2, 1, 224, 3, 112) == 0
    assert orc.out_size(True, 7, 3, 1, 1) == 7 and orc.padding(1, 1, 7, 3, 7) == 1
    assert orc.out_size(False, 7, 7, 1, 1) == 1


def test_single_step_requant_identity():
    """The kernels' single-step requantisation (common.hpp requant_out<true>,
    enabled per layer by bh_conv_requant_fast_ok) equals TFLite's two-step
    MultiplyByQuantizedMultiplier (the oracle's tfl_mbqm) plus the zero point
    for M in (2^30, 2^31), shift -e <= 0 and |x| inside the fast_ok bound;
    random multipliers, multipliers with zeroed low bits (rounding ties are
    then frequent) and exact half-way accumulators."""
    L = orc.lib()
    rng = np.random.default_rng(2024)
    n = 0
    for trial in range(400):
        e = int(rng.integers(0, 21))
        if trial % 3 == 0:
            M = int(rng.integers((1 << 30) + 1, 1 << 31))
        else:  # low bits zero: x*M lands on .5 boundaries often
            M = (1 << 30) + (int(rng.integers(1, 1 << 10)) << 20)
        zp = int(rng.integers(-128, 128))
        bound = (1 << 30) - 255 * (1 << e) - 1
        xs = rng.integers(-bound, bound + 1, size=200).tolist()
        # accumulators whose product with M is an exact multiple of 2^30 (ties)
        xs += [int(k) << 10 for k in rng.integers(-(bound >> 10), (bound >> 10) + 1, size=50)]
        xs += [0, 1, -1, bound, -bound]
        for x in xs:
            z = x * M + (1 << 30) + ((1 << (30 + e)) if e > 0 else 0)
            u = z >> 31
            s = -1 if (e > 0 and x < 0) else 0
            v = (u + s + (zp << e)) >> e
            ref = L.tfl_mbqm(x, M, -e) + zp
            assert v == ref, (x, M, e, zp, v, ref)
            n += 1
    assert n > 100000
