"""fp16-weight float models (TFLite post-training float16 quantization) on
the CPU worker vs the float oracle (oracle/float_ref.py), with the stated
tolerance: |got - ref| <= 1e-3 * |ref| + 1e-4 * max(1, max |ref|)
(float32 summation order differs from the float64 oracle; not bit-exact)."""
import numpy as np
import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey, tflite_synth as S
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model as OModel

RTOL = 1e-3
ATOL_REL = 1e-4


def assert_float_close(got, ref, msg=""):
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    atol = ATOL_REL * max(1.0, float(np.abs(ref).max()))
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=atol, err_msg=msg)


MODELS = {
    "mobilenet_v2_fp16": lambda size: S.mobilenet_v2(np.float16, size=size),
    "mobilenet_v1_fp16": lambda size: S.mobilenet_v1(np.float16, size=size),
    "ssd_mobilenet_v2_fp16": lambda size: S.ssd_mobilenet_v2(np.float16, size=size),
}


@pytest.mark.parametrize("name", sorted(MODELS))
def test_fp16_models_cpu_worker(tmp_path, name):
    buf = MODELS[name](96)
    p = str(tmp_path / "m.tflite")
    open(p, "wb").write(buf)
    om = OModel(buf)
    assert any(t.np_dtype == np.float16 for t in om.tensors)  # weights stored as float16
    m = HipModel(0)
    assert m.FromPath(p).ok()
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU, num_threads=8)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, 0)
    x = np.random.default_rng(0).uniform(-1, 1, om.tensors[om.inputs[0]].shape).astype(np.float32)
    ex.GetTensorView(key, ex.GetInputs(key)[0]).GetData()[...] = x
    assert ex.ExecuteSubgraph(key).ok()
    ref = OracleInterpreter(om).run({om.inputs[0]: x})
    for t in om.outputs:
        assert_float_close(ex.GetTensorView(key, t).GetData(), ref[t], "%s tensor %d" % (name, t))
