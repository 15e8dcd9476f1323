"""Diagnostic: retinaface outputs-only run (fusion active) vs oracle."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model

path = "tests/golden/retinaface_mbv2_quant_160.tflite"
buf = open(path, "rb").read()
om = Model(buf)
model = HipModel(1)
assert model.FromBuffer(buf).ok()
ex = HipModelExecutor(1, 1, DeviceFlag.kGPU)
ex.InvestigateModelSpec(model)
assert ex.PrepareSubgraph(model).ok()
key = SubgraphKey(1, 1)
rng = np.random.default_rng(42)
x = rng.integers(-128, 128, om.tensors[om.inputs[0]].shape).astype(np.int8)
ex.GetTensorView(key, om.inputs[0]).GetData()[...] = x
assert ex.ExecuteSubgraph(key).ok()
ref = OracleInterpreter(om).run({om.inputs[0]: x})
bad = 0
for t in om.outputs:
    got = ex.GetTensorView(key, t).GetData()
    n = int((got != ref[t].reshape(got.shape)).sum())
    bad += n
    print("output", t, "mismatches", n)
prof = ex.ProfileSubgraph(key, iters=1)
print("launches:", " ".join("%d:%s" % (r["op_index"], r["kernel"]) for r in prof))
print("RESULT", "ok" if bad == 0 else "BAD")
