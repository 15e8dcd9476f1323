"""Host thread placement and the planner's dispatch ceiling (no GPU needed).

* A kCPU executor pins its host thread pool to the CpuSet Band hands it
  (band/interface/model_executor.h:41-50; the reference passes the mask to
  the interpreter's pool, band/backend/tfl/model_executor.cc:356-359).
* Worker threads pin themselves to a non-empty worker CpuSet
  (band/worker.cc:195-205) and are named band-w<id>; the planner thread is
  band-planner (band/planner.cc:268-293).
* tools/planner_ceiling.py drives the engine with ~zero-cost jobs and
  reports jobs/s and the busiest threads.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
from band_amd.engine import Engine, Model, SchedulerType, make_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _threads():
    out = []
    for tid in os.listdir("/proc/self/task"):
        try:
            with open("/proc/self/task/%s/status" % tid) as f:
                st = dict(line.rstrip("\n").split(":\t", 1) for line in f if ":\t" in line)
            out.append((int(tid), st.get("Name", ""), st.get("Cpus_allowed_list", "")))
        except OSError:
            pass
    return out


def test_cpu_executor_pool_honours_cpuset(golden_dir):
    before = {t for t, _, _ in _threads()}
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU, num_threads=3, cpus=[0])
    new = [t for t in _threads() if t[0] not in before]
    # the pool's own threads (num_threads - 1; the caller is the third)
    assert len(new) == 2, new
    assert all(c == "0" for _, _, c in new), new
    m = HipModel(0)
    assert m.FromPath(os.path.join(golden_dir, "add.tflite")).ok()
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(0, 0)
    ex.GetTensorView(key, ex.GetInputs(key)[0]).GetData()[...] = 1.0
    assert ex.ExecuteSubgraph(key).ok()
    assert float(ex.GetTensorView(key, ex.GetOutputs(key)[0]).GetData().reshape(-1)[0]) == 3.0
    del ex


def test_cpu_executor_without_mask_is_unpinned():
    allowed = [c for _, _, c in _threads() if c][0]
    before = {t for t, _, _ in _threads()}
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU, num_threads=2)
    new = [t for t in _threads() if t[0] not in before]
    assert len(new) == 1 and new[0][2] == allowed, (new, allowed)
    del ex


def test_engine_threads_are_named(golden_dir):
    e = Engine(make_config([SchedulerType.kRoundRobin], [DeviceFlag.kCPU, DeviceFlag.kCPU], num_threads=[1, 1]))
    m = Model()
    assert m.FromPath(os.path.join(golden_dir, "add.tflite"))
    assert e.RegisterModel(m)
    time.sleep(0.1)
    names = {n for _, n, _ in _threads()}
    assert "band-planner" in names
    assert {"band-w0", "band-w1"} <= names
    e.close()


def test_planner_ceiling_tool_runs():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "planner_ceiling.py"), "--workers", "2,8",
                        "--jobs", "4000", "--models", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert [x["workers"] for x in lines] == [2, 8]
    for x in lines:
        assert x["jobs"] == 4000 and x["jobs_per_s"] > 1000
        assert x["workers_used"] == x["workers"]  # round_robin reaches every worker
        assert x["busiest_threads"] and all(isinstance(n, str) for n, _ in x["busiest_threads"])
