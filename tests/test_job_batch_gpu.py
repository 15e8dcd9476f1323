"""Job batching on the MI355X (backend/hip/job_batching.h extension):
n queued whole-model jobs of one model run as one pass over a batch-B
variant of the subgraph; every job's outputs stay bit-exact with the oracle.

Band itself runs one job per ExecuteSubgraph (band/worker.cc:222-323); these
tests pin that batching changes nothing a job can observe except timing.
"""
import numpy as np
import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey, tflite_synth
from band_amd.engine import Engine, JobStatus, Model, SchedulerType, make_config, kBandOk
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model as OModel
from tests.glue_models import split_zoo

pytestmark = pytest.mark.gpu


def _exec(buf, mid):
    m = HipModel(mid)
    assert m.FromBuffer(buf).ok()
    ex = HipModelExecutor(mid, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(m).ok()
    ex._model_ref = m
    return m, ex, SubgraphKey(mid, 1)


@pytest.mark.parametrize("arch", ["mobilenet_v2", "ssd_mobilenet_v2"])
def test_executor_job_batches_bit_exact(gpu_lib, arch):
    buf = getattr(tflite_synth, arch)(np.int8, size=96)
    m, ex, key = _exec(buf, 21)
    assert ex.MaxJobBatch(key) == 1
    assert ex.PrepareJobBatches(m, key, 8).ok()
    assert ex.MaxJobBatch(key) == 8
    om = OModel(buf)
    t_in = om.tensors[om.inputs[0]]
    rng = np.random.default_rng(3)
    for n in (2, 3, 5, 8):
        xs = [rng.integers(-128, 128, t_in.shape).astype(np.int8) for _ in range(n)]
        for s, x in enumerate(xs):
            v = ex.GetJobSlotView(key, om.inputs[0], n, s)
            assert v.GetDims() == list(t_in.shape) and v.GetBytes() == x.nbytes
            v.GetData()[...] = x
        refs = [OracleInterpreter(om).run({om.inputs[0]: x}) for x in xs]
        for _ in range(2):  # eager pass, then the captured graph
            assert ex.ExecuteJobBatch(key, n).ok()
            for s, ref in enumerate(refs):
                for o in om.outputs:
                    got = ex.GetJobSlotView(key, o, n, s).GetData()
                    np.testing.assert_array_equal(got, ref[o].reshape(got.shape),
                                                  err_msg="%s n=%d slot %d output %d" % (arch, n, s, o))
    # batch-1 path untouched
    x = rng.integers(-128, 128, t_in.shape).astype(np.int8)
    ex.GetTensorView(key, om.inputs[0]).GetData()[...] = x
    assert ex.ExecuteSubgraph(key).ok()
    ref = OracleInterpreter(om).run({om.inputs[0]: x})
    for o in om.outputs:
        got = ex.GetTensorView(key, o).GetData()
        np.testing.assert_array_equal(got, ref[o].reshape(got.shape))


def test_job_batches_refused_for_custom_ops(gpu_lib):
    buf = split_zoo()
    m = HipModel(22)
    assert m.FromBuffer(buf).ok()
    ex = HipModelExecutor(22, 1, DeviceFlag.kGPU)
    spec = ex.InvestigateModelSpec(m)
    gpu_ops = [i for i in range(spec.num_ops) if i not in spec.unsupported_ops[DeviceFlag.kGPU]][:5]
    assert ex.PrepareSubgraph(m, gpu_ops, [0]).ok()
    key = SubgraphKey(22, 1, [0])
    st = ex.PrepareJobBatches(m, key, 4)
    assert not st.ok() and "CUSTOM" in st.message()
    assert ex.MaxJobBatch(key) == 1


@pytest.mark.parametrize("direct", ["1", "0"])
@pytest.mark.parametrize("sched,workers", [(SchedulerType.kFixedWorker, 1), (SchedulerType.kRoundRobin, 2)])
def test_engine_batches_queued_jobs_bit_exact(gpu_lib, tmp_path, monkeypatch, sched, workers, direct):
    """max_job_batch 8: fixed_worker's queued jobs / round_robin's same-model
    requests handed to an idle worker run together (same invoke / end time
    in their job records), each output equal to the oracle's; with the
    passes' I/O DMA'd straight between the page-locked request rings and the
    device (direct, the default) and staged through the slot views"""
    monkeypatch.setenv("BAND_HIP_DIRECT_IO", direct)
    e = Engine(make_config([sched], [DeviceFlag.kGPU] * workers, max_job_batch=8))
    rng = np.random.default_rng(4)
    models = []
    for name in ("mobilenet_v2", "posenet_mobilenet_v1"):
        buf = getattr(tflite_synth, name)(np.int8, size=96)
        path = str(tmp_path / (name + ".tflite"))
        with open(path, "wb") as f:
            f.write(buf)
        m = Model()
        assert m.FromPath(path)
        assert e.RegisterModel(m)
        models.append((m, OModel(buf)))
    prepared = []
    for i in range(48):
        m, om = models[i % 2]
        t = e.CreateInputTensor(m, 0)
        x = rng.integers(-128, 128, om.tensors[om.inputs[0]].shape).astype(np.int8)
        t.data()[...] = x
        outs = [e.CreateOutputTensor(m, k) for k in range(e.GetNumOutputTensors(m))]
        prepared.append((m, om, t, x, outs))
    # submitted back to back, so requests queue while the workers are busy
    jobs = [(e.RequestAsync(m, [t]), m, om, x, outs) for m, om, t, x, outs in prepared]
    invoke = {}
    for h, m, om, x, outs in jobs:
        assert h >= 0 and e.Wait(h, outs) == kBandOk
        r = e.GetJobRecord(h)
        assert r.status == JobStatus.kSuccess
        invoke.setdefault((r.model_id, r.invoke_time_us, r.end_time_us), []).append(h)
        ref = OracleInterpreter(om).run({om.inputs[0]: x})
        for k, t in enumerate(sorted(om.outputs)):
            np.testing.assert_array_equal(outs[k].data().reshape(-1), ref[t].reshape(-1))
    assert max(len(v) for v in invoke.values()) > 1, "no two jobs shared a batched pass"
    e.close()


def test_engine_direct_io_across_ring_wrap(gpu_lib, tmp_path, monkeypatch):
    """more requests of one model than its request ring has slots (20), in
    rounds of 16 submitted at once: batched passes whose slots straddle the
    ring's end are split into contiguous DMA runs; every output equals the
    oracle's"""
    monkeypatch.setenv("BANDX_REQUEST_RING_SLOTS", "20")
    e = Engine(make_config([SchedulerType.kFixedWorker], [DeviceFlag.kGPU], max_job_batch=8))
    buf = tflite_synth.mobilenet_v2(np.int8, size=96)
    path = str(tmp_path / "mnv2.tflite")
    with open(path, "wb") as f:
        f.write(buf)
    m = Model()
    assert m.FromPath(path)
    assert e.RegisterModel(m)
    om = OModel(buf)
    rng = np.random.default_rng(12)
    shared = 0
    for rnd in range(3):
        jobs = []
        for i in range(16):
            t = e.CreateInputTensor(m, 0)
            x = rng.integers(-128, 128, om.tensors[om.inputs[0]].shape).astype(np.int8)
            t.data()[...] = x
            outs = [e.CreateOutputTensor(m, k) for k in range(e.GetNumOutputTensors(m))]
            jobs.append((e.RequestAsync(m, [t]), x, outs))
        invoke = {}
        for h, x, outs in jobs:
            assert h >= 0 and e.Wait(h, outs) == kBandOk
            r = e.GetJobRecord(h)
            assert r.status == JobStatus.kSuccess
            invoke.setdefault((r.invoke_time_us, r.end_time_us), []).append(h)
            ref = OracleInterpreter(om).run({om.inputs[0]: x})
            for k, t in enumerate(sorted(om.outputs)):
                np.testing.assert_array_equal(outs[k].data().reshape(-1), ref[t].reshape(-1))
        shared += max(len(v) for v in invoke.values()) > 1
    assert shared > 0, "no batched pass"
    e.close()
