"""Job coalescing on the MI355X (backend/hip/coalescer.h).

Band runs one job per ExecuteSubgraph (band/worker.cc:222-323 ->
band/engine.cc:843-850 -> band/backend/tfl/model_executor.cc:249-255), one
executor per (model, worker).  Inside the backend, concurrent calls on the
executors of one model on one GPU run as one job-batch pass; every caller
must still get exactly its own job's outputs, bit-exact with the oracle.
"""
import threading

import numpy as np
import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SetWorkerDevice, SubgraphKey, tflite_synth
from band_amd.backend import CoalescerStats
from band_amd.engine import Engine, JobStatus, Model, SchedulerType, make_config, kBandOk
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model as OModel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("io", ["dma", "copy"])
@pytest.mark.parametrize("arch", ["mobilenet_v2", "ssd_mobilenet_v2"])
def test_concurrent_execute_subgraph_bit_exact(gpu_lib, monkeypatch, arch, io):
    """6 threads, each on its own executor of one model (6 Band workers on
    GPU 0), call ExecuteSubgraph at the same moment, round after round, each
    with its own input; every output of every call equals the oracle's for
    that call's input, and some calls ran as coalesced passes."""
    monkeypatch.setenv("BAND_HIP_COALESCE", "4")
    monkeypatch.setenv("BAND_HIP_COALESCE_LANES", "2")
    monkeypatch.setenv("BAND_HIP_COALESCE_IO", io)
    buf = getattr(tflite_synth, arch)(np.int8, size=96)
    om = OModel(buf)
    t_in = om.tensors[om.inputs[0]]
    rng = np.random.default_rng(11)
    xs = [rng.integers(-128, 128, t_in.shape).astype(np.int8) for _ in range(5)]
    refs = [OracleInterpreter(om).run({om.inputs[0]: x}) for x in xs]
    mid = 31
    m = HipModel(mid)
    assert m.FromBuffer(buf).ok()
    W = 6
    execs = []
    for w in range(W):
        SetWorkerDevice(100 + w, 0)
        ex = HipModelExecutor(mid, 100 + w, DeviceFlag.kGPU)
        assert ex.PrepareSubgraph(m).ok()
        execs.append((ex, SubgraphKey(mid, 100 + w)))
    for ex, _ in execs:
        assert ex.Coalescer() == (W, True)
    CoalescerStats(reset=True)
    rounds = 8
    barrier = threading.Barrier(W)
    errors = []

    def run(tid):
        ex, key = execs[tid]
        try:
            for r in range(rounds):
                k = (tid + r) % len(xs)
                ex.GetTensorView(key, om.inputs[0]).GetData()[...] = xs[k]
                barrier.wait(timeout=60)
                st = ex.ExecuteSubgraph(key)
                assert st.ok(), st
                for o in om.outputs:
                    got = ex.GetTensorView(key, o).GetData()
                    np.testing.assert_array_equal(got, refs[k][o].reshape(got.shape),
                                                  err_msg="%s thread %d round %d output %d" % (arch, tid, r, o))
        except BaseException as e:  # noqa: BLE001 - reported below
            errors.append(e)
            barrier.abort()

    ths = [threading.Thread(target=run, args=(t,)) for t in range(W)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ths), "a coalesced call never returned"
    if errors:
        raise errors[0]
    s = CoalescerStats()
    assert s["calls"] == W * rounds, s
    assert s["group_passes"] > 0 and s["group_jobs"] >= 2 * s["group_passes"], s
    assert s["max_group"] <= 4, s
    # a lone executor afterwards: its own batch-1 pass, still exact
    ex, key = execs[0]
    ex.GetTensorView(key, om.inputs[0]).GetData()[...] = xs[1]
    assert ex.ExecuteSubgraph(key).ok()
    got = ex.GetTensorView(key, om.outputs[0]).GetData()
    np.testing.assert_array_equal(got, refs[1][om.outputs[0]].reshape(got.shape))


def test_single_executor_does_not_build_lanes(gpu_lib):
    buf = tflite_synth.mobilenet_v2(np.int8, size=96)
    m = HipModel(32)
    assert m.FromBuffer(buf).ok()
    SetWorkerDevice(120, 0)
    ex = HipModelExecutor(32, 120, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(m).ok()
    assert ex.Coalescer() == (1, False)


@pytest.mark.parametrize("sync", ["adaptive", "spin", "poller"])
def test_engine_one_job_per_pass_coalesced_bit_exact(gpu_lib, monkeypatch, sync):
    """Band's own contract (max_job_batch 1: the engine calls only
    band/interface) with 6 GPU workers under round_robin: a burst of
    requests from several submitter threads; every request's outputs equal
    the oracle's, and the backend coalesced some of the jobs.  sync=poller:
    the waiting threads sleep and the GPU's CompletionPoller wakes them;
    adaptive (the default): sleep through most of the expected wait, then
    spin."""
    monkeypatch.setenv("BAND_HIP_COALESCE", "6")
    monkeypatch.setenv("BAND_HIP_SYNC", sync)
    buf = tflite_synth.mobilenet_v2(np.int8, size=96)
    om = OModel(buf)
    t_in = om.tensors[om.inputs[0]]
    rng = np.random.default_rng(5)
    xs = [rng.integers(-128, 128, t_in.shape).astype(np.int8) for _ in range(4)]
    refs = [OracleInterpreter(om).run({om.inputs[0]: x})[om.outputs[0]].reshape(-1) for x in xs]
    e = Engine(make_config([SchedulerType.kRoundRobin], [DeviceFlag.kGPU] * 6, max_job_batch=1))
    m = Model()
    assert m.FromBuffer(buf)
    assert e.RegisterModel(m)
    CoalescerStats(reset=True)
    n_sub, per = 4, 24
    errors = []

    def submit(tid):
        try:
            t = e.CreateInputTensor(m, 0)
            o = e.CreateOutputTensor(m, 0)
            hs = []
            for j in range(per):
                t.data()[...] = xs[(tid + j) % 4]
                hs.append(e.RequestAsync(m, [t]))
            for j, h in enumerate(hs):
                assert h >= 0
                assert e.Wait(h, [o]) == kBandOk
                assert e.GetJobRecord(h).status == JobStatus.kSuccess
                np.testing.assert_array_equal(o.data().reshape(-1), refs[(tid + j) % 4],
                                              err_msg="submitter %d request %d" % (tid, j))
        except BaseException as ex:  # noqa: BLE001
            errors.append(ex)

    ths = [threading.Thread(target=submit, args=(i,)) for i in range(n_sub)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ths)
    if errors:
        raise errors[0]
    s = CoalescerStats()
    assert s["calls"] >= n_sub * per, s
    assert s["group_jobs"] > 0, s
    e.close()


def test_failed_lane_build_turns_coalescing_off(gpu_lib, monkeypatch):
    """A lane build that fails (as out of device memory would) leaves
    coalescing OFF: every call runs its own executor's pass at once, several
    at a time (no lane token caps them), bit-exact with the oracle."""
    monkeypatch.setenv("BAND_HIP_COALESCE", "4")
    monkeypatch.setenv("BAND_HIP_COALESCE_FAIL_BUILD", "1")
    buf = tflite_synth.mobilenet_v2(np.int8, size=96)
    om = OModel(buf)
    t_in = om.tensors[om.inputs[0]]
    rng = np.random.default_rng(17)
    xs = [rng.integers(-128, 128, t_in.shape).astype(np.int8) for _ in range(3)]
    refs = [OracleInterpreter(om).run({om.inputs[0]: x}) for x in xs]
    mid = 33
    m = HipModel(mid)
    assert m.FromBuffer(buf).ok()
    W = 6
    execs = []
    for w in range(W):
        SetWorkerDevice(140 + w, 0)
        ex = HipModelExecutor(mid, 140 + w, DeviceFlag.kGPU)
        assert ex.PrepareSubgraph(m).ok()
        execs.append((ex, SubgraphKey(mid, 140 + w)))
    for ex, _ in execs:
        assert ex.Coalescer() == (W, False)
    CoalescerStats(reset=True)
    rounds = 6
    barrier = threading.Barrier(W)
    errors = []

    def run(tid):
        ex, key = execs[tid]
        try:
            for r in range(rounds):
                k = (tid + r) % len(xs)
                ex.GetTensorView(key, om.inputs[0]).GetData()[...] = xs[k]
                barrier.wait(timeout=60)
                assert ex.ExecuteSubgraph(key).ok()
                for o in om.outputs:
                    got = ex.GetTensorView(key, o).GetData()
                    np.testing.assert_array_equal(got, refs[k][o].reshape(got.shape))
        except BaseException as e:  # noqa: BLE001 - reported below
            errors.append(e)
            barrier.abort()

    ths = [threading.Thread(target=run, args=(t,)) for t in range(W)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ths)
    if errors:
        raise errors[0]
    s = CoalescerStats()
    assert s["calls"] == W * rounds and s["bypass_calls"] == W * rounds, s
    assert s["group_passes"] == 0, s
    assert s["max_bypass_inflight"] >= 2, s
