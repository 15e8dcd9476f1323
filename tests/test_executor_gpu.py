"""Model-level parity on the MI355X: the HIP IModelExecutor vs the CPU oracle.

Drives the executor exactly the way Band's engine does (InvestigateModelSpec
-> PrepareSubgraph -> GetTensorView/CopyDataFrom -> ExecuteSubgraph ->
GetTensorView of the outputs; band/engine.cc:51-289, 843-850, 1247-1365), on
the reference's own fixtures, and requires bit-exact int8/uint8 outputs.
"""
import os

import numpy as np
import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model
from tests.test_oracle import load_cat

pytestmark = pytest.mark.gpu


def _load(golden_dir, name, mid):
    m = HipModel(mid)
    assert m.FromPath(os.path.join(golden_dir, name)).ok()
    return m


def test_mnv2_quant_cat_282_and_bit_exact(gpu_lib, golden_dir):
    path = os.path.join(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    model = _load(golden_dir, "mobilenet_v2_1.0_224_quant.tflite", 0)
    ex = HipModelExecutor(0, 1, DeviceFlag.kGPU)
    spec = ex.InvestigateModelSpec(model)
    assert spec.num_ops == 65 and spec.unsupported_ops[DeviceFlag.kGPU] == set()
    assert ex.PrepareSubgraph(model).ok()
    key = SubgraphKey(0, 1)
    x = load_cat(golden_dir)
    ex.GetTensorView(key, ex.GetInputs(key)[0]).GetData()[...] = x
    assert ex.ExecuteSubgraph(key).ok()
    out = ex.GetTensorView(key, ex.GetOutputs(key)[0]).GetData().reshape(-1).copy()
    assert int(np.argmax(out)) == 282
    om = Model.from_path(path)
    ref = OracleInterpreter(om).run({om.inputs[0]: x})[om.outputs[0]].reshape(-1)
    np.testing.assert_array_equal(out, ref)


def test_mnv2_quant_every_intermediate_bit_exact(gpu_lib, golden_dir):
    path = os.path.join(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    model = _load(golden_dir, "mobilenet_v2_1.0_224_quant.tflite", 0)
    ex = HipModelExecutor(0, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(model).ok()
    key = SubgraphKey(0, 1)
    om = Model.from_path(path)
    inter = sorted({t for o in om.operators for t in o.outputs})
    views = {t: ex.GetTensorView(key, t) for t in inter}
    rng = np.random.default_rng(0)
    x = rng.integers(0, 256, (1, 224, 224, 3)).astype(np.uint8)
    ex.GetTensorView(key, om.inputs[0]).GetData()[...] = x
    assert ex.ExecuteSubgraph(key).ok()
    ref = OracleInterpreter(om).run({om.inputs[0]: x})
    for t in inter:
        np.testing.assert_array_equal(views[t].GetData(), ref[t].reshape(views[t].GetDims()),
                                      err_msg="tensor %d (%s)" % (t, om.tensors[t].name))


def _segments(spec, n_ops):
    """maximal runs of consecutive GPU-supported ops"""
    bad = spec.unsupported_ops[DeviceFlag.kGPU]
    segs, cur = [], []
    for i in range(n_ops):
        if i in bad:
            if cur:
                segs.append(cur)
            cur = []
        else:
            cur.append(i)
    if cur:
        segs.append(cur)
    return segs


@pytest.mark.parametrize("name", ["retinaface_mbv2_quant_160.tflite", "ICN_quant.tflite"])
def test_int8_per_channel_model_segments(gpu_lib, golden_dir, name):
    """Real int8 per-channel models: every maximal GPU-supported op run,
    prepared as a subgraph and fed random inputs, matches the oracle."""
    path = os.path.join(golden_dir, name)
    model = _load(golden_dir, name, 3)
    ex = HipModelExecutor(3, 1, DeviceFlag.kGPU)
    spec = ex.InvestigateModelSpec(model)
    om = Model.from_path(path)
    orc = OracleInterpreter(om)
    segs = [s for s in _segments(spec, spec.num_ops) if not any(
        om.operators[i].builtin not in orc.SUPPORTED for i in s)]
    assert segs, "no runnable segment"
    rng = np.random.default_rng(42)
    checked = 0
    for u, seg in enumerate(segs[:12]):
        assert ex.PrepareSubgraph(model, ops=seg, unit_indices=[u]).ok()
        key = SubgraphKey(3, 1, [u])
        ins = ex.GetInputs(key)
        assert ins == sorted(spec.GetPureInputTensors(seg))
        assert set(ex.GetOutputs(key)) <= spec.GetOutputTensors(seg)
        feed = {}
        for t in ins:
            tt = om.tensors[t]
            feed[t] = rng.integers(-128, 128, tt.shape).astype(np.int8) if tt.np_dtype == np.int8 else \
                rng.integers(0, 256, tt.shape).astype(np.uint8)
            ex.GetTensorView(key, t).GetData()[...] = feed[t]
        assert ex.ExecuteSubgraph(key).ok()
        ref = orc.run(feed, ops=seg)
        for t in ex.GetOutputs(key):
            np.testing.assert_array_equal(ex.GetTensorView(key, t).GetData(), ref[t].reshape(om.tensors[t].shape),
                                          err_msg="%s seg %s tensor %d" % (name, seg, t))
        checked += 1
    assert checked >= 1


def test_graph_replay_matches_eager(gpu_lib, golden_dir):
    model = _load(golden_dir, "mobilenet_v2_1.0_224_quant.tflite", 0)
    eg = HipModelExecutor(0, 1, DeviceFlag.kGPU)
    ee = HipModelExecutor(0, 2, DeviceFlag.kGPU)
    ee.SetUseGraph(False)
    assert eg.PrepareSubgraph(model).ok() and ee.PrepareSubgraph(model).ok()
    kg, ke = SubgraphKey(0, 1), SubgraphKey(0, 2)
    rng = np.random.default_rng(3)
    for _ in range(4):  # run 0 eager, run 1 captures, runs 2+ replay
        x = rng.integers(0, 256, (1, 224, 224, 3)).astype(np.uint8)
        eg.GetTensorView(kg, 171).GetData()[...] = x
        ee.GetTensorView(ke, 171).GetData()[...] = x
        assert eg.ExecuteSubgraph(kg).ok() and ee.ExecuteSubgraph(ke).ok()
        np.testing.assert_array_equal(eg.GetTensorView(kg, 172).GetData(), ee.GetTensorView(ke, 172).GetData())


def test_error_behaviour(gpu_lib, golden_dir):
    model = _load(golden_dir, "add.tflite", 5)
    ex = HipModelExecutor(5, 1, DeviceFlag.kGPU)
    st = ex.ExecuteSubgraph(SubgraphKey(5, 1))
    assert not st.ok() and st.message() == "Cannot find subgraph"
    wrong = HipModelExecutor(6, 1, DeviceFlag.kGPU)
    assert not wrong.PrepareSubgraph(model).ok()
    # float ADD is in the float32 kernel set: the whole model prepares on kGPU
    spec = ex.InvestigateModelSpec(model)
    assert spec.unsupported_ops[DeviceFlag.kGPU] == set()
    assert ex.PrepareSubgraph(model).ok()
    # TFLite_Detection_PostProcess is CPU-only: reported, and a whole-model
    # subgraph containing it is refused on kGPU
    from tests.glue_models import split_zoo
    split = HipModel(7)
    assert split.FromBuffer(split_zoo()).ok()
    ex7 = HipModelExecutor(7, 1, DeviceFlag.kGPU)
    bad = ex7.InvestigateModelSpec(split).unsupported_ops[DeviceFlag.kGPU]
    # the postprocess, plus the two DEQUANTIZEs feeding only it (placed with
    # it on the CPU side: the hand-off then carries int8, not float32)
    assert len(bad) == 3
    assert not ex7.PrepareSubgraph(split).ok()


@pytest.mark.parametrize("arch,dtype,batch", [
    ("mobilenet_v2", np.int8, 1), ("mobilenet_v2", np.int8, 3), ("mobilenet_v2", np.uint8, 1),
    ("mobilenet_v1", np.int8, 1), ("mobilenet_v2", np.int8, 8),
    ("ssd_mobilenet_v2", np.int8, 1), ("deeplab_v3_mobilenet_v2", np.int8, 1),
    ("posenet_mobilenet_v1", np.int8, 1), ("ssd_mobilenet_v2", np.uint8, 1), ("posenet_mobilenet_v1", np.int8, 2)])
def test_synthetic_models_bit_exact(gpu_lib, arch, dtype, batch):
    """The bench models (BASELINE C1/C2, synthetic weights), fused epilogues on."""
    from band_amd import tflite_synth as S
    buf = getattr(S, arch)(dtype, seed=7, batch=batch)
    model = HipModel(11)
    assert model.FromBuffer(buf).ok()
    ex = HipModelExecutor(11, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(model).ok()
    key = SubgraphKey(11, 1)
    om = Model(buf)
    t = om.tensors[om.inputs[0]]
    rng = np.random.default_rng(batch)
    lo, hi = (-128, 128) if dtype == np.int8 else (0, 256)
    for _ in range(2):
        x = rng.integers(lo, hi, t.shape).astype(dtype)
        ex.GetTensorView(key, om.inputs[0]).GetData()[...] = x
        assert ex.ExecuteSubgraph(key).ok()
        ref = OracleInterpreter(om).run({om.inputs[0]: x})
        for o in om.outputs:
            got = ex.GetTensorView(key, o).GetData()
            np.testing.assert_array_equal(got, ref[o].reshape(got.shape), err_msg="%s output %d" % (arch, o))


def test_view_of_fused_tensor_materialises_it(gpu_lib):
    """Asking for a view of a conv output that an ADD epilogue fused away
    re-lowers without that fusion; both the tensor and the final output match."""
    from band_amd import tflite_synth as S
    buf = S.mobilenet_v2(np.int8, seed=3)
    om = Model(buf)
    add_op = next(o for o in om.operators if o.name == "ADD")
    conv_out = add_op.inputs[0]
    model = HipModel(12)
    assert model.FromBuffer(buf).ok()
    ex = HipModelExecutor(12, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(model).ok()
    key = SubgraphKey(12, 1)
    v = ex.GetTensorView(key, conv_out)
    x = np.random.default_rng(0).integers(-128, 128, (1, 224, 224, 3)).astype(np.int8)
    ex.GetTensorView(key, om.inputs[0]).GetData()[...] = x
    assert ex.ExecuteSubgraph(key).ok()
    ref = OracleInterpreter(om).run({om.inputs[0]: x})
    np.testing.assert_array_equal(v.GetData(), ref[conv_out])
    np.testing.assert_array_equal(ex.GetTensorView(key, om.outputs[0]).GetData(), ref[om.outputs[0]])
