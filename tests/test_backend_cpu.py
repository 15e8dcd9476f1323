"""CPU-side checks of the HIP backend (no GPU needed).

* The C-ABI library loads and exports every symbol include/*.h declares.
* InvestigateModelSpec / PrepareSubgraph / GetTensorView metadata follow the
  reference contract (band/backend/tfl/model_executor.cc:48-229) and the
  I/O rules Band's engine checks (band/engine.cc:153-233), on CPU-worker
  executors (which Band always creates: band/engine.cc:248-252).
"""
import os
import re

import numpy as np
import pytest

from band_amd import DataType, DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
from band_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    syms = set()
    for h in ("band_hip_kernels.h", "band_hip_backend.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        syms |= set(re.findall(r"\b(bhx?_[a-z0-9_]+)\s*\(", src))
    return syms


def _declared_c_api():
    """Band engine C API (include/band_c_api.h): the exported functions"""
    src = open(os.path.join(ROOT, "include", "band_c_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"BAND_CAPI_EXPORT\s+[\w\s\*]*?\b(Bandx?[A-Z]\w*)\s*\(", src))


def test_library_exports_every_declared_symbol():
    lib = _abi.load()
    syms = _declared_symbols()
    assert len(syms) > 50
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_mirror_binds_every_symbol():
    import band_amd.backend  # noqa: F401  (registers bhx_* prototypes)
    bound = set(_abi.KERNEL_SYMBOLS) | set(_abi.BACKEND_SYMBOLS)
    assert _declared_symbols() <= bound | {"bh_set_last_error"}


def test_library_exports_band_c_api():
    """the drop-in C API: every function of include/band_c_api.h (the
    reference's band/c/c_api.h names plus Bandx extensions) is exported and
    bound by band_amd.engine (logging / variadic config calls are called
    without prototypes)"""
    import band_amd.engine  # noqa: F401
    lib = _abi.load()
    syms = _declared_c_api()
    assert len(syms) >= 45
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    unbound = syms - set(_abi.BACKEND_SYMBOLS) - {"BandAddConfig", "BandSetLogReporter", "BandUnsetLogReporter"}
    assert not unbound, unbound


def _model(golden_dir, name, mid=0):
    m = HipModel(mid)
    st = m.FromPath(os.path.join(golden_dir, name))
    assert st.ok(), st
    return m


def test_model_load_errors():
    m = HipModel(0)
    st = m.FromPath("/nonexistent.tflite")
    assert not st.ok() and st.message() == "Cannot load from file."
    assert not m.IsInitialized()
    st = m.FromBuffer(b"\x00" * 64)
    assert not st.ok() and st.message() == "Cannot load from buffer."


def test_model_from_buffer(golden_dir):
    data = open(os.path.join(golden_dir, "add.tflite"), "rb").read()
    m = HipModel(0)
    assert m.FromBuffer(data).ok() and m.IsInitialized()


def test_model_spec_add(golden_dir):
    # band/test/backend/tfl_minimal_test.cc:36-51
    m = _model(golden_dir, "add.tflite")
    spec = HipModelExecutor(0, 0, DeviceFlag.kCPU).InvestigateModelSpec(m)
    assert spec.num_ops == 2
    assert len(spec.input_tensors) == 1 and len(spec.output_tensors) == 1
    assert spec.tensor_types and all(t == DataType.kFloat32 for t in spec.tensor_types)
    assert DeviceFlag.kDSP in spec.unavailable_devices and DeviceFlag.kNPU in spec.unavailable_devices


def test_model_spec_mobilenet(golden_dir):
    m = _model(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    spec = HipModelExecutor(0, 0, DeviceFlag.kCPU).InvestigateModelSpec(m)
    assert (spec.num_ops, spec.num_tensors) == (65, 173)
    assert spec.input_tensors == {171} and spec.output_tensors == {172}
    # constants (weights/biases/shape) never appear as op inputs
    assert all(len(s) in (1, 2) for s in spec.op_input_tensors)
    assert spec.path.endswith("mobilenet_v2_1.0_224_quant.tflite")


def test_unsupported_ops_reported_for_glue(golden_dir):
    m = _model(golden_dir, "retinaface_mbv2_quant_160.tflite")
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU)
    spec = ex.InvestigateModelSpec(m)
    assert spec.unsupported_ops[DeviceFlag.kCPU] == set()


def test_prepare_io_contract_random_subsets(golden_dir):
    """GetInputs == sorted pure inputs; GetOutputs ⊆ op outputs (band/engine.cc:153-173)."""
    m = _model(golden_dir, "retinaface_mbv2_quant_160.tflite")
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU)
    spec = ex.InvestigateModelSpec(m)
    rng = np.random.default_rng(0)
    for u in range(20):
        lo = int(rng.integers(0, spec.num_ops - 1))
        hi = int(rng.integers(lo + 1, min(spec.num_ops, lo + 30) + 1))
        ops = list(range(lo, hi))
        assert ex.PrepareSubgraph(m, ops=ops, unit_indices=[u]).ok()
        key = SubgraphKey(0, 0, [u])
        assert ex.GetInputs(key) == sorted(spec.GetPureInputTensors(ops))
        outs = ex.GetOutputs(key)
        assert outs == sorted(outs) and set(outs) <= spec.GetOutputTensors(ops)
        assert ex.GetNumNodes(key) == len(ops)
        for i, t in enumerate(ex.GetInputs(key)):
            assert ex.GetInputName(key, i) == ex.GetTensorView(key, t).GetName()
    assert ex.GetLargestSubgraphKey().IsValid()
    seen = []
    ex.ForEachSubgraph(seen.append)
    assert len(seen) == 20


def test_whole_model_io_is_model_order(golden_dir):
    m = _model(golden_dir, "retinaface_mbv2_quant_160.tflite")
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, 0)
    assert ex.GetInputs(key) == [0] and ex.GetOutputs(key) == [259, 255, 262]
    assert ex.GetOutputName(key, 0) == "Identity"


def test_tensor_view_semantics(golden_dir):
    m = _model(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, 0)
    v = ex.GetTensorView(key, 171)
    assert v.GetType() == DataType.kUInt8 and v.GetDims() == [1, 224, 224, 3]
    assert v.GetBytes() == 150528 and v.GetName() == "input"
    q = v.GetQuantization()
    assert q["scale"] == [0.0078125] and q["zero_point"] == [128]
    data = np.arange(150528, dtype=np.uint32).astype(np.uint8).reshape(1, 224, 224, 3)
    v.GetData()[...] = data
    np.testing.assert_array_equal(ex.GetTensorView(key, 171).GetData(), data)  # views alias
    other = ex.GetTensorView(key, 172)
    assert not v.CopyDataFrom(other).ok()  # type/dims mismatch -> error, like ITensor::CopyDataFrom
    w = ex.GetTensorView(key, 2)  # constant filter: host view of the model buffer
    assert w.GetDims() == [32, 3, 3, 3]


def test_cpu_executor_unknown_key(golden_dir):
    m = _model(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU)
    assert ex.PrepareSubgraph(m).ok()
    assert ex.ExecuteSubgraph(SubgraphKey(0, 7)).message() == "Cannot find subgraph"


def test_cpu_worker_add_kat(golden_dir):
    """tfl_minimal_test.cc:76-86 on a kCPU worker: add.tflite {1,3} -> {3,9}"""
    m = _model(golden_dir, "add.tflite")
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, 0)
    x = ex.GetTensorView(key, ex.GetInputs(key)[0])
    x.GetData().reshape(-1)[:2] = [1, 3]
    assert ex.ExecuteSubgraph(key).ok()
    y = ex.GetTensorView(key, ex.GetOutputs(key)[0]).GetData().reshape(-1)
    assert list(y[:2]) == [3, 9]


def test_cpu_worker_mnv2_cat_282_bit_exact(golden_dir):
    """the kCPU worker runs the same lowered program as the GPU (host
    kernels); bit-exact with the oracle and argmax 282 on cat.jpg"""
    from oracle.runner import OracleInterpreter
    from oracle.tflite_fb import Model
    from tests.test_oracle import load_cat
    path = os.path.join(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    m = _model(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU, num_threads=4)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, 0)
    x = load_cat(golden_dir)
    ex.GetTensorView(key, ex.GetInputs(key)[0]).GetData()[...] = x
    assert ex.ExecuteSubgraph(key).ok()
    out = ex.GetTensorView(key, ex.GetOutputs(key)[0]).GetData().reshape(-1).copy()
    assert int(np.argmax(out)) == 282
    om = Model.from_path(path)
    ref = OracleInterpreter(om).run({om.inputs[0]: x})[om.outputs[0]].reshape(-1)
    np.testing.assert_array_equal(out, ref)


def test_prepare_wrong_model_id(golden_dir):
    m = _model(golden_dir, "add.tflite", mid=4)
    ex = HipModelExecutor(5, 0, DeviceFlag.kCPU)
    st = ex.PrepareSubgraph(m)
    assert not st.ok() and "model id" in st.message()


def test_gpu_executor_without_device_fails_loudly(golden_dir):
    from band_amd import device
    if device.device_count() > 0:
        pytest.skip("a GPU is visible")
    m = _model(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    st = HipModelExecutor(0, 1, DeviceFlag.kGPU).PrepareSubgraph(m)
    assert not st.ok() and "gfx950" in st.message()


@pytest.mark.parametrize("dtype", [np.int8, np.uint8])
def test_dw_tap_table_identity(dtype):
    """bh_pack_dw_taps (host code, no GPU): the dot4 kernel's sum over the
    table equals the oracle's accumulator bias + sum (x - zx)(w - zw) over
    in-image taps, with out-of-image taps read as zx (dwconv.hip)."""
    import ctypes
    lib = _abi.load()
    rng = np.random.default_rng(11)
    C = 24
    w = rng.integers(-128, 128, size=(9, C)).astype(np.int8)  # int8-domain
    bias = rng.integers(-(1 << 15), 1 << 15, size=C).astype(np.int32)
    zx = int(rng.integers(-128, 128))
    zw = 0 if dtype == np.int8 else int(rng.integers(-40, 40))
    taps = np.zeros((C, 4), np.int32)
    assert lib.bh_pack_dw_taps(w.ctypes.data_as(ctypes.c_void_p), C, bias.ctypes.data_as(ctypes.c_void_p),
                               zx, zw, taps.ctypes.data_as(ctypes.c_void_p)) == 0
    tb = taps.view(np.uint8).reshape(C, 4, 4).astype(np.int8).astype(np.int64)
    for trial in range(20):
        x = rng.integers(-128, 128, size=(9, C)).astype(np.int64)
        inside = rng.random(9) < 0.7
        ref = bias.astype(np.int64) + ((x - zx) * (w.astype(np.int64) - zw) * inside[:, None]).sum(0)
        xp = np.where(inside[:, None], x, zx)  # padded taps read as zx
        for c in range(C):
            j = c % 4
            tcol = np.concatenate([xp[0:8, c], [xp[8, c - j + 0], xp[8, c - j + 1], xp[8, c - j + 2], xp[8, c - j + 3]]])
            wcol = np.concatenate([tb[c, 0], tb[c, 1], tb[c, 2]])
            acc = int(taps[c, 3]) + int((tcol * wcol).sum())
            if zw:
                acc -= zw * int(xp[:, c].sum())
            assert acc == ref[c], (trial, c)


# the conv launcher's routing is host logic (no device call): the RGB stem
# takes the MFMA form at every batch (r06ag), the LDS-staged VALU form only
# when forced (BH_CONV_STEM_VALU = 4) or outside the MFMA form's channel
# range, the scalar-cache form above 64 channels per workgroup; pointers are
# placeholders, never dereferenced
@pytest.mark.parametrize("batch,oc,hint,want", [
    (1, 32, 0, "conv_stem_mfma_kernel"), (32, 32, 0, "conv_stem_mfma_kernel"), (256, 32, 0, "conv_stem_mfma_kernel"),
    (32, 64, 0, "conv_stem_mfma_kernel"), (32, 32, 4, "conv_stem_lds_kernel"), (32, 24, 0, "conv_stem_lds_kernel"),
    (32, 80, 0, "conv_stem_kernel")])
def test_stem_routing(batch, oc, hint, want):
    import ctypes
    lib = _abi.load()
    p = _abi.ConvParams(batch=batch, in_h=224, in_w=224, in_c=3, out_h=112, out_w=112, out_c=oc, k_h=3, k_w=3,
                        stride_h=2, stride_w=2, dil_h=1, dil_w=1, pad_h=0, pad_w=0, k_pad=64, n_pad=(oc + 63) // 64 * 64,
                        kernel_hint=hint)
    p.input, p.output, p.weights = 1 << 20, 2 << 20, 3 << 20
    assert lib.bh_conv2d_i8_kernel(ctypes.byref(p)).decode() == want
