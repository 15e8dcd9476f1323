"""The reference's remaining known-answer tests, ported (no GPU):

* band/test/backend/tfl_subgraph_test.cc:72-85 - ICN, magenta and retinaface
  (the reference's own .tflite fixtures) register under kMergeUnitSubgraph
  with the test's runtime config (LSF, minimum subgraph size 7, two CPU
  workers with 3 / 4 threads, online profiling 1 warm-up + 1 run).  The
  lite0 EfficientDet fixture it also lists is not in band/test/data.  Here
  each model then serves one request through the engine.
* band/test/tool/benchmark_test.cc:22-42 - the benchmark tool loads and runs
  band/test/data/benchmark_config.json (retinaface x2, HEFT, periodic,
  500 ms), and refuses an empty config.
* band/test/c/c_api_test.cc:31-57 - the ConfigLoad sequence of BandAddConfig
  calls builds a config; plus the builder's rejections
  (band/test/config_builder_test.cc: negative num_runs / window size,
  worker list lengths that disagree).
"""
import json
import os

import numpy as np
import pytest

from band_amd.engine import (BenchmarkRun, ConfigBuilder, ConfigField, CPUMaskFlag, Engine, Model, SchedulerType,
                             SubgraphPreparationType, kBandOk, make_config)
from band_amd import DeviceFlag
from band_amd._abi import BandHipError

MODELS = ["ICN_quant.tflite", "magenta_arbitrary-image-stylization-v1-256_int8_transfer_1.tflite",
          "retinaface_mbv2_quant_160.tflite"]


@pytest.mark.parametrize("name", MODELS)
def test_model_partition_merge_unit_subgraph(golden_dir, tmp_path, name):
    cfg = make_config([SchedulerType.kLeastSlackTimeFirst], [DeviceFlag.kCPU, DeviceFlag.kCPU], num_threads=[3, 4],
                      cpu_masks=[CPUMaskFlag.kBig, CPUMaskFlag.kLittle], window_size=10, online=True, num_warmups=1,
                      num_runs=1, smoothing=0.1, profile_path=str(tmp_path / "profile.json"),
                      log_path=str(tmp_path / "log.json"), subgraph_type=SubgraphPreparationType.kMergeUnitSubgraph,
                      minimum_subgraph_size=7)
    e = Engine(cfg)
    m = Model()
    assert m.FromPath(os.path.join(golden_dir, name))
    assert e.RegisterModel(m)
    # one request end to end (random inputs of each input's type)
    rng = np.random.default_rng(0)
    ins = []
    for i in range(e.GetNumInputTensors(m)):
        t = e.CreateInputTensor(m, i)
        a = t.data()
        if a.dtype == np.float32:
            a[...] = rng.uniform(0, 1, a.shape)
        else:
            a[...] = rng.integers(np.iinfo(a.dtype).min, np.iinfo(a.dtype).max, a.shape, endpoint=True)
        ins.append(t)
    outs = [e.CreateOutputTensor(m, i) for i in range(e.GetNumOutputTensors(m))]
    assert e.RequestSync(m, ins, outs) == kBandOk
    if "magenta" in name:  # the stylised image: a LOGISTIC output in [0, 1]
        o = outs[0].data()
        assert o.shape == (1, 384, 384, 3) and np.all((o >= 0) & (o <= 1))
    e.close()


def _benchmark_config(golden_dir, tmp_path):
    with open(os.path.join(golden_dir, "benchmark_config.json")) as f:
        cfg = json.load(f)
    for m in cfg["models"]:
        m["graph"] = os.path.join(golden_dir, os.path.basename(m["graph"]))
    cfg["log_path"] = str(tmp_path / "log.json")
    cfg["profile_data_path"] = str(tmp_path / "profile.json")
    return cfg


def test_benchmark_config_load_and_run(golden_dir, tmp_path):
    cfg = _benchmark_config(golden_dir, tmp_path)
    assert cfg["execution_mode"] == "periodic" and cfg["running_time_ms"] == 500
    r = BenchmarkRun(cfg)
    assert r.get("ok", True) and r.get("num_requests", 1) >= 1, r


def test_benchmark_config_load_fail(golden_dir, tmp_path):
    with pytest.raises(BandHipError):
        BenchmarkRun("")
    with pytest.raises(BandHipError):
        BenchmarkRun({"execution_mode": "periodic"})  # no models / schedulers


def test_c_api_config_load(golden_dir):
    b = ConfigBuilder()
    b.add(ConfigField.BAND_PLANNER_LOG_PATH, "band/test/data/log.json")
    b.add(ConfigField.BAND_PLANNER_SCHEDULERS, int(SchedulerType.kRoundRobin))
    b.add(ConfigField.BAND_MINIMUM_SUBGRAPH_SIZE, 7)
    b.add(ConfigField.BAND_SUBGRAPH_PREPARATION_TYPE, int(SubgraphPreparationType.kMergeUnitSubgraph))
    b.add(ConfigField.BAND_CPU_MASK, int(CPUMaskFlag.kAll))
    b.add(ConfigField.BAND_PLANNER_CPU_MASK, int(CPUMaskFlag.kPrimary))
    b.add(ConfigField.BAND_WORKER_WORKERS, int(DeviceFlag.kCPU), int(DeviceFlag.kCPU))
    b.add(ConfigField.BAND_WORKER_NUM_THREADS, 3, 4)
    b.add(ConfigField.BAND_WORKER_CPU_MASKS, int(CPUMaskFlag.kBig), int(CPUMaskFlag.kLittle))
    b.add(ConfigField.BAND_PROFILE_SMOOTHING_FACTOR, 0.1)
    b.add(ConfigField.BAND_PROFILE_DATA_PATH, "band/test/data/profile.json")
    b.add(ConfigField.BAND_PROFILE_ONLINE, True)
    b.add(ConfigField.BAND_PROFILE_NUM_WARMUPS, 1)
    b.add(ConfigField.BAND_PROFILE_NUM_RUNS, 1)
    b.add(ConfigField.BAND_WORKER_ALLOW_WORKSTEAL, True)
    b.add(ConfigField.BAND_WORKER_AVAILABILITY_CHECK_INTERVAL_MS, 30000)
    b.add(ConfigField.BAND_PLANNER_SCHEDULE_WINDOW_SIZE, 10)
    assert b.build() is not None
    # the same runtime values as tests/golden/config.json (the reference's
    # runtime-config fixture) - its scheduler is given as an integer there
    with open(os.path.join(golden_dir, "config.json")) as f:
        j = json.load(f)
    assert j["schedulers"] == [int(SchedulerType.kRoundRobin)] and j["minimum_subgraph_size"] == 7
    assert [w["num_threads"] for w in j["workers"]] == [3, 4]


@pytest.mark.parametrize("field,values", [
    (ConfigField.BAND_PROFILE_NUM_RUNS, (-1,)),
    (ConfigField.BAND_PLANNER_SCHEDULE_WINDOW_SIZE, (-1,)),
    (ConfigField.BAND_WORKER_NUM_THREADS, (1, 1, 1)),  # 3 thread counts for 2 workers
])
def test_c_api_config_rejects(field, values):
    b = ConfigBuilder()
    b.add(ConfigField.BAND_PLANNER_SCHEDULERS, int(SchedulerType.kFixedWorker))
    b.add(ConfigField.BAND_WORKER_WORKERS, int(DeviceFlag.kCPU), int(DeviceFlag.kCPU))
    b.add(field, *values)
    with pytest.raises(BandHipError):
        b.build()
