"""Run the split_zoo parts on GPU executors (CPU for the float op) and
compare every produced tensor with the oracle; prints the first mismatch."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey  # noqa: E402
from oracle.runner import OracleInterpreter  # noqa: E402
from oracle.tflite_fb import Model as OM  # noqa: E402
from tests.glue_models import split_zoo  # noqa: E402

p = "/tmp/split_zoo.tflite"
open(p, "wb").write(split_zoo())
om = OM.from_path(p)
m = HipModel(0)
assert m.FromPath(p).ok()
parts = [(list(range(0, 11)) + [26], DeviceFlag.kGPU), ([11], DeviceFlag.kCPU), (list(range(12, 26)), DeviceFlag.kGPU)]
x = np.random.default_rng(0).integers(-128, 128, (1, 16, 16, 8)).astype(np.int8)
ref = OracleInterpreter(om).run({om.inputs[0]: x})
vals = {om.inputs[0]: x}
for i, (ops, dev) in enumerate(parts):
    ex = HipModelExecutor(0, 10 + i, dev)
    assert ex.PrepareSubgraph(m, ops, [i]).ok()
    k = SubgraphKey(0, 10 + i, [i])
    produced = sorted({t for o in ops for t in om.operators[o].outputs})
    views = {t: ex.GetTensorView(k, t) for t in produced}
    for t in ex.GetInputs(k):
        ex.GetTensorView(k, t).GetData()[...] = vals[t]
    assert ex.ExecuteSubgraph(k).ok()
    for t in produced:
        v = views[t].GetData().copy()
        vals[t] = v
        ok = np.array_equal(v.reshape(-1), ref[t].reshape(-1))
        print("part %d op-out tensor %d %s %s" % (i, t, "ok" if ok else "MISMATCH",
                                                 "" if ok else str(np.abs(v.reshape(-1).astype(np.int64) -
                                                                          ref[t].reshape(-1).astype(np.int64)).max())))
