"""The native Band harness with MI355X workers (C2, C3-like and C4-like
configurations), results bit-exact with the oracle.

Engine -> planner -> worker -> HipModelExecutor::ExecuteSubgraph, driven
through the Band C API exactly as a client of the reference would
(band/test/c/c_api_test.cc), with every scheduler family:
  fixed_worker on one GPU worker            (C2)
  round_robin over two GPU workers, 4 models (C3, scaled down)
  HEFT / SEL / LSF over a CPU + GPU pair on a model the model analyzer
  splits around a CPU-only op               (C4's mechanism)
"""
import os

import numpy as np
import pytest

from band_amd import DeviceFlag, tflite_synth
from band_amd.engine import (Engine, JobStatus, Model, SchedulerType, SubgraphPreparationType, make_config,
                             BenchmarkRun, kBandOk)
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model as OModel
from tests.glue_models import split_zoo
from tests.test_oracle import load_cat

pytestmark = pytest.mark.gpu


def _model(path):
    m = Model()
    assert m.FromPath(path)
    return m


def _write(tmp_path, name, data):
    p = str(tmp_path / name)
    with open(p, "wb") as f:
        f.write(data)
    return p


def _run_and_check(e, m, path, xs, expect_workers=None):
    om = OModel.from_path(path)
    n_out = e.GetNumOutputTensors(m)
    ins = [[e.CreateInputTensor(m, 0)] for _ in xs]
    outs = [[e.CreateOutputTensor(m, k) for k in range(n_out)] for _ in xs]
    hs = []
    for t, x in zip(ins, xs):
        t[0].data()[...] = x
        hs.append(e.RequestAsync(m, t))
    assert all(h >= 0 for h in hs)
    workers = set()
    for h, o, x in zip(hs, outs, xs):
        assert e.Wait(h, o) == kBandOk
        r = e.GetJobRecord(h)
        assert r.status == JobStatus.kSuccess
        workers.add(r.worker_id)
        ref = OracleInterpreter(om).run({om.inputs[0]: x})
        # the engine orders a model's outputs by tensor index (ModelSpec
        # holds them in a std::set, band/model_spec.h)
        for k, t in enumerate(sorted(om.outputs)):
            np.testing.assert_array_equal(o[k].data().reshape(-1), ref[t].reshape(-1), err_msg="output %d" % k)
    if expect_workers is not None:
        assert workers == set(expect_workers)
    return outs


def test_c2_fixed_worker_single_gpu(gpu_lib, golden_dir):
    path = os.path.join(golden_dir, "mobilenet_v2_1.0_224_quant.tflite")
    e = Engine(make_config([SchedulerType.kFixedWorker], [DeviceFlag.kGPU]))
    m = _model(path)
    assert e.RegisterModel(m)
    assert e.GetWorkerDevice(0) == DeviceFlag.kGPU
    x = load_cat(golden_dir)
    rng = np.random.default_rng(0)
    outs = _run_and_check(e, m, path, [x] + [rng.integers(0, 256, x.shape).astype(np.uint8) for _ in range(3)],
                          expect_workers={0})
    assert int(np.argmax(outs[0][0].data())) == 282
    # the online profile measured the GPU subgraph
    js = e.GetProfileJson()
    assert js[path]["0"][0] > 0


def test_c3_round_robin_two_gpu_workers_mix(gpu_lib, tmp_path):
    e = Engine(make_config([SchedulerType.kRoundRobin], [DeviceFlag.kGPU, DeviceFlag.kGPU]))
    rng = np.random.default_rng(1)
    for i, name in enumerate(tflite_synth.MIX_C3):
        path = _write(tmp_path, name + ".tflite", getattr(tflite_synth, name)(size=96))
        m = _model(path)
        assert e.RegisterModel(m)
        shape = OModel.from_path(path).tensors[OModel.from_path(path).inputs[0]].shape
        xs = [rng.integers(-128, 128, shape).astype(np.int8) for _ in range(4)]
        _run_and_check(e, m, path, xs, expect_workers={0, 1})


@pytest.mark.parametrize("sched,prep", [
    (SchedulerType.kHeterogeneousEarliestFinishTime, SubgraphPreparationType.kMergeUnitSubgraph),
    (SchedulerType.kHeterogeneousEarliestFinishTimeReserved, SubgraphPreparationType.kMergeUnitSubgraph),
    (SchedulerType.kShortestExpectedLatency, SubgraphPreparationType.kUnitSubgraph),
    (SchedulerType.kLeastSlackTimeFirst, SubgraphPreparationType.kMergeUnitSubgraph),
    (SchedulerType.kShortestExpectedLatency, SubgraphPreparationType.kFallbackPerWorker),
])
def test_split_model_cpu_gpu(gpu_lib, tmp_path, sched, prep):
    path = _write(tmp_path, "split_zoo.tflite", split_zoo())
    e = Engine(make_config([sched], [DeviceFlag.kCPU, DeviceFlag.kGPU], num_threads=[2, 1], subgraph_type=prep,
                           minimum_subgraph_size=7))
    m = _model(path)
    assert e.RegisterModel(m)
    subs = e.GetSubgraphs(m)
    gpu_keys = [k for k in subs if k[0] == 1]
    assert gpu_keys, subs  # the GPU worker prepared subgraphs around the CPU-only op
    if prep != SubgraphPreparationType.kFallbackPerWorker:
        assert all(k[1] != 0b111 for k in gpu_keys)  # never the whole model on the GPU
    rng = np.random.default_rng(2)
    xs = [rng.integers(-128, 128, (1, 16, 16, 8)).astype(np.int8) for _ in range(6)]
    _run_and_check(e, m, path, xs)


def test_benchmark_tool_gpu_stream(gpu_lib, golden_dir):
    cfg = {
        "models": [{"graph": os.path.join(golden_dir, "mobilenet_v2_1.0_224_quant.tflite"), "batch_size": 4}],
        "execution_mode": "stream", "running_time_ms": 500, "schedulers": ["round_robin"],
        "workers": [{"device": "GPU"}, {"device": "GPU"}],
    }
    r = BenchmarkRun(cfg)
    assert r["failed"] == 0 and r["completed"] > 100
    assert min(r["jobs_per_worker"]) > 0


def test_c4_efficientdet_split_heft(gpu_lib, tmp_path):
    """C4's mechanism: EfficientDet-Lite2 with TFLite_Detection_PostProcess;
    HEFT over [CPU, GPU, GPU] runs the network on a GPU worker and the
    postprocess on the CPU worker; outputs bit-exact vs the oracle."""
    path = _write(tmp_path, "edet.tflite", tflite_synth.efficientdet_lite2(size=256))
    e = Engine(make_config([SchedulerType.kHeterogeneousEarliestFinishTime],
                           [DeviceFlag.kCPU, DeviceFlag.kGPU, DeviceFlag.kGPU], num_threads=[8, 1, 1],
                           subgraph_type=SubgraphPreparationType.kMergeUnitSubgraph))
    m = _model(path)
    assert e.RegisterModel(m)
    subs = e.GetSubgraphs(m)
    gpu = [k for k in subs if k[0] in (1, 2)]
    cpu = [k for k in subs if k[0] == 0]
    assert gpu and cpu
    last_unit = max(k[1].bit_length() for k in subs) - 1
    assert all(not (k[1] >> last_unit) & 1 for k in gpu)  # the postprocess unit never on a GPU
    rng = np.random.default_rng(4)
    xs = [rng.integers(-128, 128, (1, 256, 256, 3)).astype(np.int8) for _ in range(3)]
    _run_and_check(e, m, path, xs)
