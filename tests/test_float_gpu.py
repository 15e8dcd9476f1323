"""fp16-weight float models on the MI355X (bh_*_f32 kernels) vs the float
oracle, with the stated tolerance of tests/test_float_cpu.py; the CPU worker
and the GPU worker run the same lowered program."""
import os

import numpy as np
import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey, tflite_synth as S
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model as OModel
from tests.glue_models import float_zoo
from tests.test_float_cpu import assert_float_close

pytestmark = pytest.mark.gpu

MODELS = {
    "mobilenet_v2_fp16": lambda: S.mobilenet_v2(np.float16),
    "mobilenet_v1_fp16": lambda: S.mobilenet_v1(np.float16),
    "ssd_mobilenet_v2_fp16": lambda: S.ssd_mobilenet_v2(np.float16),
    "float_zoo": float_zoo,
}


@pytest.mark.parametrize("name", sorted(MODELS))
def test_float_models_gpu(gpu_lib, tmp_path, name):
    buf = MODELS[name]()
    p = str(tmp_path / "m.tflite")
    open(p, "wb").write(buf)
    om = OModel(buf)
    m = HipModel(0)
    assert m.FromPath(p).ok()
    ex = HipModelExecutor(0, 1, DeviceFlag.kGPU)
    spec = ex.InvestigateModelSpec(m)
    assert spec.unsupported_ops[DeviceFlag.kGPU] == set()
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, 1)
    rng = np.random.default_rng(1)
    ref_interp = OracleInterpreter(om)
    for it in range(3):  # eager, capture, graph replay
        x = rng.uniform(-1, 1, om.tensors[om.inputs[0]].shape).astype(np.float32)
        ex.GetTensorView(key, ex.GetInputs(key)[0]).GetData()[...] = x
        assert ex.ExecuteSubgraph(key).ok()
        ref = ref_interp.run({om.inputs[0]: x})
        for t in om.outputs:
            assert_float_close(ex.GetTensorView(key, t).GetData(), ref[t], "%s run %d tensor %d" % (name, it, t))
