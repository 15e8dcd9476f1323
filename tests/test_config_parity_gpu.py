"""Whole-model parity at the configurations the bench numbers come from.

* C3: every mix model (MobileNetV2, SSD-MobileNetV2, DeepLabV3, PoseNet) at
  224x224 int8, run through job batching's ExecuteJobBatch at n in {1, 7, 17, 24, 2, 13}
  - the passes bench.py's headline is made of - every slot's every output
  bit-exact vs the oracle (the TFLite 2.9.2 restatement), eager pass and
  graph replay both.
* C4: EfficientDet-Lite2 at its configured 448x448 through the engine, HEFT
  over [CPU, GPU, GPU] (band/scheduler/heterogeneous_earliest_finish_time_
  scheduler.cc:11-142): the network on the GPU workers, the detection
  postprocess on the CPU worker, outputs bit-exact.
* C5: the 8-DNN int8 + fp16 mix as an open-loop Poisson request stream under
  shortest_expected_latency with the online latency estimator
  (band/scheduler/shortest_expected_latency_scheduler.cc:13-94) over
  [CPU, GPU, GPU]: every job's outputs vs the oracle, int8 bit-exact, fp16
  at the float tolerance of tests/test_float_cpu.py.

The oracle runs multi-threaded (oracle/tflite_ref.c OpenMP loops; each
output element is still computed by one thread, so its values do not depend
on the thread count).
"""
import os

import numpy as np
import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey, tflite_synth as S
from band_amd.engine import Engine, JobStatus, Model, SchedulerType, SubgraphPreparationType, make_config, kBandOk
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model as OModel
from tests.test_float_cpu import assert_float_close

pytestmark = pytest.mark.gpu

N_SLOTS = 24


def _inputs(om, n, seed):
    t = om.tensors[om.inputs[0]]
    rng = np.random.default_rng(seed)
    if t.np_dtype == np.float32:
        return [rng.uniform(-1, 1, t.shape).astype(np.float32) for _ in range(n)]
    lo, hi = (-128, 128) if t.np_dtype == np.int8 else (0, 256)
    return [rng.integers(lo, hi, t.shape).astype(t.np_dtype) for _ in range(n)]


@pytest.mark.parametrize("arch", list(S.MIX_C3))
def test_c3_job_batches_224_bit_exact(gpu_lib, arch):
    buf = getattr(S, arch)(np.int8, size=224)
    om = OModel(buf)
    xs = _inputs(om, N_SLOTS, 4200 + len(arch))
    refs = [OracleInterpreter(om).run({om.inputs[0]: x}) for x in xs]
    m = HipModel(31)
    assert m.FromBuffer(buf).ok()
    ex = HipModelExecutor(31, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(31, 1)
    assert ex.PrepareJobBatches(m, key, N_SLOTS).ok()
    assert ex.MaxJobBatch(key) == N_SLOTS
    for n in (1, 7, 17, N_SLOTS, 2, 13):  # every size has its own variant, all on one arena
        # slot s of the n-job pass carries input (s * 5 + n) % 24: every
        # slot a different input, and a different one in each pass
        pick = [(s * 5 + n) % N_SLOTS for s in range(n)]
        for s, i in enumerate(pick):
            ex.GetJobSlotView(key, om.inputs[0], n, s).GetData()[...] = xs[i]
        for rep in range(2):  # eager pass, then the captured graph
            assert ex.ExecuteJobBatch(key, n).ok()
            for s, i in enumerate(pick):
                for o in om.outputs:
                    got = ex.GetJobSlotView(key, o, n, s).GetData()
                    np.testing.assert_array_equal(got, refs[i][o].reshape(got.shape),
                                                  err_msg="%s n=%d slot %d run %d output %d" % (arch, n, s, rep, o))
    ex._model_ref = m


def _register(e, tmp_path, name, buf):
    p = str(tmp_path / (name + ".tflite"))
    with open(p, "wb") as f:
        f.write(buf)
    m = Model()
    assert m.FromPath(p)
    assert e.RegisterModel(m), name
    return m


def _check_job(e, m, om, h, outs, ref, name, atol_float=False):
    assert e.Wait(h, outs) == kBandOk, name
    r = e.GetJobRecord(h)
    assert r.status == JobStatus.kSuccess, name
    # the engine orders a model's outputs by tensor index (ModelSpec keeps
    # them in a std::set, band/model_spec.h)
    for k, t in enumerate(sorted(om.outputs)):
        got = outs[k].data().reshape(-1)
        if atol_float:
            assert_float_close(got, ref[t].reshape(-1), "%s output %d" % (name, t))
        else:
            np.testing.assert_array_equal(got, ref[t].reshape(-1), err_msg="%s output %d" % (name, t))
    return r


def test_c4_efficientdet_lite2_448_heft(gpu_lib, tmp_path):
    buf = S.efficientdet_lite2(np.int8, size=448)
    om = OModel(buf)
    e = Engine(make_config([SchedulerType.kHeterogeneousEarliestFinishTime],
                           [DeviceFlag.kCPU, DeviceFlag.kGPU, DeviceFlag.kGPU], num_threads=[8, 1, 1],
                           subgraph_type=SubgraphPreparationType.kMergeUnitSubgraph))
    m = _register(e, tmp_path, "edet448", buf)
    subs = e.GetSubgraphs(m)
    gpu = [k for k in subs if k[0] in (1, 2)]
    cpu = [k for k in subs if k[0] == 0]
    assert gpu and cpu
    last_unit = max(k[1].bit_length() for k in subs) - 1
    assert all(not (k[1] >> last_unit) & 1 for k in gpu)  # the postprocess unit never on a GPU
    xs = _inputs(om, 3, 448)
    ins = [e.CreateInputTensor(m, 0) for _ in xs]
    hs = []
    for t, x in zip(ins, xs):
        t.data()[...] = x
        hs.append(e.RequestAsync(m, [t]))
    workers = set()
    for h, x in zip(hs, xs):
        outs = [e.CreateOutputTensor(m, k) for k in range(e.GetNumOutputTensors(m))]
        ref = OracleInterpreter(om).run({om.inputs[0]: x})
        workers.add(_check_job(e, m, om, h, outs, ref, "edet448").worker_id)
    e.close()


def test_c4_boundary_dequantize_on_cpu(gpu_lib):
    """the DEQUANTIZEs feeding TFLite_Detection_PostProcess are declared
    unsupported on the GPU (the analyzer then keeps them on the CPU side and
    the GPU -> CPU hand-off carries int8), every other DEQUANTIZE is not"""
    from band_amd import HipModel, HipModelExecutor
    buf = S.efficientdet_lite2(np.int8, size=448)
    om = OModel(buf)
    m = HipModel(3)
    assert m.FromBuffer(buf).ok()
    spec = HipModelExecutor(3, 1, DeviceFlag.kGPU).InvestigateModelSpec(m)
    custom = [i for i, op in enumerate(om.operators) if op.builtin == 32]
    assert custom and set(custom) <= spec.unsupported_ops[DeviceFlag.kGPU]
    feeding = {i for i, op in enumerate(om.operators) if op.builtin == 6
               and any(set(op.outputs) & set(om.operators[c].inputs) for c in custom)}
    assert feeding and feeding <= spec.unsupported_ops[DeviceFlag.kGPU]
    others = {i for i, op in enumerate(om.operators) if op.builtin == 6} - feeding
    assert not (others & spec.unsupported_ops[DeviceFlag.kGPU])


C5_MODELS = [("mobilenet_v1_int8", lambda: S.mobilenet_v1(np.int8)),
             ("mobilenet_v2_int8", lambda: S.mobilenet_v2(np.int8)),
             ("ssd_mobilenet_v2_int8", lambda: S.ssd_mobilenet_v2(np.int8)),
             ("deeplab_v3_mobilenet_v2_int8", lambda: S.deeplab_v3_mobilenet_v2(np.int8)),
             ("posenet_mobilenet_v1_int8", lambda: S.posenet_mobilenet_v1(np.int8)),
             ("efficientdet_lite2_int8", lambda: S.efficientdet_lite2(np.int8, size=448)),
             ("mobilenet_v2_fp16", lambda: S.mobilenet_v2(np.float16)),
             ("ssd_mobilenet_v2_fp16", lambda: S.ssd_mobilenet_v2(np.float16))]


def test_c5_poisson_sel_latency_estimator(gpu_lib, tmp_path):
    e = Engine(make_config([SchedulerType.kShortestExpectedLatency],
                           [DeviceFlag.kCPU, DeviceFlag.kGPU, DeviceFlag.kGPU], num_threads=[8, 1, 1],
                           num_warmups=1, num_runs=2))
    models = []
    for i, (name, make) in enumerate(C5_MODELS):
        buf = make()
        om = OModel(buf)
        m = _register(e, tmp_path, name, buf)
        xs = _inputs(om, 2, 500 + i)
        refs = [OracleInterpreter(om).run({om.inputs[0]: x}) for x in xs]
        models.append((name, m, om, xs, refs))
    # the latency estimator profiled every subgraph of every model online
    prof = e.GetProfileJson()
    assert all(len(v) > 0 for k, v in prof.items() if k != "hash")
    # open-loop Poisson arrivals (seeded), uniform over the 8 models, each
    # request with its own input tensor
    rng = np.random.default_rng(5489)
    gaps = rng.exponential(1.0 / 400.0, 48)
    picks = rng.integers(0, len(models), 48)
    import time
    jobs = []
    t0 = time.perf_counter()
    due = 0.0
    for g, k in zip(gaps, picks):
        due += g
        wait = t0 + due - time.perf_counter()
        if wait > 0:
            time.sleep(wait)
        name, m, om, xs, refs = models[k]
        j = len(jobs) % 2
        t = e.CreateInputTensor(m, 0)
        t.data()[...] = xs[j]
        jobs.append((e.RequestAsync(m, [t]), k, j, t))
    assert all(h >= 0 for h, _, _, _ in jobs)
    workers = set()
    for h, k, j, _ in jobs:
        name, m, om, xs, refs = models[k]
        outs = [e.CreateOutputTensor(m, q) for q in range(e.GetNumOutputTensors(m))]
        r = _check_job(e, m, om, h, outs, refs[j], name, atol_float=name.endswith("fp16"))
        workers.add(r.worker_id)
    assert workers & {1, 2}, workers  # SEL used the GPU workers
    e.close()
