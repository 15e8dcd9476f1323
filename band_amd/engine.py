"""Python mirror of the Band engine C API served by libband_hip.so.

Same functions as the reference's C API (band/c/c_api.h:47-190) and its
Python-facing names: BandConfigBuilder / BandAddConfig, Model, Engine with
RegisterModel / CreateInputTensor / RequestSync / RequestAsync / Wait.  The
engine behind it is the native C++ harness (band_amd/csrc/engine): planner
thread, per-device workers, schedulers, latency estimator, model analyzer.
Every call goes through the C ABI; nothing here computes.
"""
import ctypes
import enum
import json
from ctypes import POINTER, c_bool, c_char_p, c_double, c_float, c_int, c_int64, c_size_t, c_uint64, c_void_p

import numpy as np

from . import _abi


class SchedulerType(enum.IntEnum):  # band/c/c_api_type.h:49-58
    kFixedWorker = 0
    kRoundRobin = 1
    kShortestExpectedLatency = 2
    kFixedWorkerGlobalQueue = 3
    kHeterogeneousEarliestFinishTime = 4
    kLeastSlackTimeFirst = 5
    kHeterogeneousEarliestFinishTimeReserved = 6


class SubgraphPreparationType(enum.IntEnum):
    kNoFallbackSubgraph = 0
    kFallbackPerWorker = 1
    kUnitSubgraph = 2
    kMergeUnitSubgraph = 3


class CPUMaskFlag(enum.IntEnum):
    kAll = 0
    kLittle = 1
    kBig = 2
    kPrimary = 3


class ConfigField(enum.IntEnum):  # band/c/c_api_type.h:145-166
    BAND_PROFILE_ONLINE = 0
    BAND_PROFILE_NUM_WARMUPS = 1
    BAND_PROFILE_NUM_RUNS = 2
    BAND_PROFILE_SMOOTHING_FACTOR = 3
    BAND_PROFILE_DATA_PATH = 4
    BAND_PLANNER_SCHEDULE_WINDOW_SIZE = 5
    BAND_PLANNER_SCHEDULERS = 6
    BAND_PLANNER_CPU_MASK = 7
    BAND_PLANNER_LOG_PATH = 8
    BAND_WORKER_WORKERS = 9
    BAND_WORKER_CPU_MASKS = 10
    BAND_WORKER_NUM_THREADS = 11
    BAND_WORKER_ALLOW_WORKSTEAL = 12
    BAND_WORKER_AVAILABILITY_CHECK_INTERVAL_MS = 13
    BAND_MINIMUM_SUBGRAPH_SIZE = 14
    BAND_SUBGRAPH_PREPARATION_TYPE = 15
    BAND_CPU_MASK = 16
    BANDX_WORKER_MAX_JOB_BATCH = 1000  # extension (include/band_c_api.h)
    BANDX_PROFILE_SHARE_IDENTICAL = 1001  # extension
    BANDX_WORKER_PASS_TARGET_US = 1002  # extension: pass-size policy of job batching


class JobStatus(enum.IntEnum):  # band/common.h:185-200
    kEnqueueFailed = 0
    kQueued = 1
    kSuccess = 2
    kSLOViolation = 3
    kInputCopyFailure = 4
    kOutputCopyFailure = 5
    kInvokeFailure = 6


kBandOk, kBandErr = 0, 1
kBandTfLite = 0


class RequestOption(ctypes.Structure):  # band/c/c_api_type.h:190-195
    _fields_ = [("target_worker", c_int), ("require_callback", c_bool), ("slo_us", c_int), ("slo_scale", c_float)]


class JobRecord(ctypes.Structure):  # BandxJobRecord
    _fields_ = [("job_id", c_int), ("model_id", c_int), ("worker_id", c_int), ("status", c_int),
                ("enqueue_time_us", c_int64), ("invoke_time_us", c_int64), ("end_time_us", c_int64),
                ("expected_latency_us", c_int64), ("slo_us", c_int64), ("unit_indices", c_uint64)]


CALLBACK = ctypes.CFUNCTYPE(None, c_void_p, c_int, c_int)

_abi.BACKEND_SYMBOLS.update({
    "BandSetLogSeverity": (None, [c_int]),
    "BandConfigBuilderCreate": (c_void_p, []),
    "BandConfigBuilderDelete": (None, [c_void_p]),
    "BandConfigCreate": (c_void_p, [c_void_p]),
    "BandConfigDelete": (None, [c_void_p]),
    "BandModelCreate": (c_void_p, []),
    "BandModelDelete": (None, [c_void_p]),
    "BandModelAddFromBuffer": (c_int, [c_void_p, c_int, c_void_p, c_size_t]),
    "BandModelAddFromFile": (c_int, [c_void_p, c_int, c_char_p]),
    "BandTensorDelete": (None, [c_void_p]),
    "BandTensorGetType": (c_int, [c_void_p]),
    "BandTensorGetData": (c_void_p, [c_void_p]),
    "BandTensorGetNumDims": (c_size_t, [c_void_p]),
    "BandTensorGetDims": (POINTER(c_int), [c_void_p]),
    "BandTensorGetBytes": (c_size_t, [c_void_p]),
    "BandTensorGetName": (c_char_p, [c_void_p]),
    "BandTensorGetQuantizationType": (c_int, [c_void_p]),
    "BandTensorGetQuantizationParams": (c_void_p, [c_void_p]),
    "BandRequestOptionGetDefault": (RequestOption, []),
    "BandEngineCreateWithDefaultConfig": (c_void_p, []),
    "BandEngineCreate": (c_void_p, [c_void_p]),
    "BandEngineDelete": (None, [c_void_p]),
    "BandEngineRegisterModel": (c_int, [c_void_p, c_void_p]),
    "BandEngineGetNumInputTensors": (c_int, [c_void_p, c_void_p]),
    "BandEngineGetNumOutputTensors": (c_int, [c_void_p, c_void_p]),
    "BandEngineGetNumWorkers": (c_int, [c_void_p]),
    "BandEngineGetWorkerDevice": (c_int, [c_void_p, c_int]),
    "BandEngineCreateInputTensor": (c_void_p, [c_void_p, c_void_p, c_size_t]),
    "BandEngineCreateOutputTensor": (c_void_p, [c_void_p, c_void_p, c_size_t]),
    "BandEngineRequestSync": (c_int, [c_void_p, c_void_p, POINTER(c_void_p), POINTER(c_void_p)]),
    "BandEngineRequestAsync": (c_int, [c_void_p, c_void_p, POINTER(c_void_p)]),
    "BandEngineRequestSyncOptions": (c_int, [c_void_p, c_void_p, RequestOption, POINTER(c_void_p),
                                             POINTER(c_void_p)]),
    "BandEngineRequestAsyncOptions": (c_int, [c_void_p, c_void_p, RequestOption, POINTER(c_void_p)]),
    "BandEngineWait": (c_int, [c_void_p, c_int, POINTER(c_void_p), c_size_t]),
    "BandEngineSetOnEndRequest": (c_int, [c_void_p, CALLBACK, c_void_p]),
    "BandEngineUnsetOnEndRequest": (c_int, [c_void_p, c_int]),
    "BandxEngineGetJobRecord": (c_int, [c_void_p, c_int, POINTER(JobRecord)]),
    "BandxModelGetId": (c_int, [c_void_p]),
    "BandxEngineGetProfileJson": (c_size_t, [c_void_p, c_char_p, c_size_t]),
    "BandxEngineDumpProfile": (c_int, [c_void_p]),
    "BandxEngineGetSubgraphs": (c_int, [c_void_p, c_void_p, POINTER(c_int), POINTER(c_uint64), c_int]),
    "BandxEngineGetExpectedLatency": (c_int64, [c_void_p, c_void_p, c_int, c_uint64]),
    "BandxEngineWaitAll": (None, [c_void_p]),
    "BandxEngineGetWorkerJobCount": (c_int64, [c_void_p, c_int]),
    "BandxEngineGetWorkerPhaseTimes": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int64)]),
    "BandxEngineGetDriverStats": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "BandxEngineGetRequestPhaseTimes": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    "BandxEngineRequestsAsync": (c_int, [c_void_p, POINTER(c_void_p), c_int, POINTER(c_void_p), POINTER(c_int)]),
    "BandxBenchmarkRun": (c_size_t, [c_char_p, c_char_p, c_size_t]),
    "BandxEngineRunClosedLoop": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p), c_int, c_int, c_int,
                                         POINTER(c_double), POINTER(c_int), POINTER(c_double)]),
    "BandxEngineRunClosedLoopEx": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p), c_int, c_int, c_int,
                                           POINTER(c_double), POINTER(c_int), POINTER(c_int), POINTER(c_double)]),
    "BandxEngineRunPoisson": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p), c_int, c_int, c_double, c_uint64,
                                      c_int, POINTER(c_double), POINTER(c_int), POINTER(c_int), POINTER(c_double)]),
})


def _lib():
    return _abi.load()


class ConfigBuilder:
    """BandConfigBuilder + BandAddConfig (band/c/c_api.cc:86-196)."""

    def __init__(self):
        self.lib = _lib()
        self.handle = c_void_p(self.lib.BandConfigBuilderCreate())

    def add(self, field, *values):
        args = []
        for v in values:
            if isinstance(v, str):
                args.append(c_char_p(v.encode()))
            elif isinstance(v, float):
                args.append(c_double(v))
            else:
                args.append(c_int(int(v)))
        fn = self.lib.BandAddConfig
        fn.restype = None
        fn.argtypes = None  # variadic
        fn(self.handle, c_int(int(field)), c_int(len(values)), *args)
        return self

    def build(self):
        cfg = self.lib.BandConfigCreate(self.handle)
        if not cfg:
            raise _abi.BandHipError("BandConfigCreate: invalid configuration")
        return Config(c_void_p(cfg))

    def __del__(self):
        if getattr(self, "handle", None):
            self.lib.BandConfigBuilderDelete(self.handle)
            self.handle = None


class Config:
    def __init__(self, handle):
        self.lib = _lib()
        self.handle = handle

    def __del__(self):
        if getattr(self, "handle", None):
            self.lib.BandConfigDelete(self.handle)
            self.handle = None


def make_config(schedulers, workers, num_threads=None, cpu_masks=None, window_size=None, online=True,
                num_warmups=1, num_runs=1, smoothing=0.1, profile_path=None, log_path=None,
                subgraph_type=None, minimum_subgraph_size=None, max_job_batch=None, share_identical=None,
                pass_target_us=None):
    b = ConfigBuilder()
    b.add(ConfigField.BAND_PLANNER_SCHEDULERS, *[int(s) for s in schedulers])
    b.add(ConfigField.BAND_WORKER_WORKERS, *[int(w) for w in workers])
    b.add(ConfigField.BAND_WORKER_NUM_THREADS, *(num_threads or [1] * len(workers)))
    b.add(ConfigField.BAND_WORKER_CPU_MASKS, *(cpu_masks or [CPUMaskFlag.kAll] * len(workers)))
    b.add(ConfigField.BAND_PROFILE_ONLINE, bool(online))
    b.add(ConfigField.BAND_PROFILE_NUM_WARMUPS, num_warmups)
    b.add(ConfigField.BAND_PROFILE_NUM_RUNS, num_runs)
    b.add(ConfigField.BAND_PROFILE_SMOOTHING_FACTOR, float(smoothing))
    if profile_path:
        b.add(ConfigField.BAND_PROFILE_DATA_PATH, profile_path)
    if log_path:
        b.add(ConfigField.BAND_PLANNER_LOG_PATH, log_path)
    if window_size:
        b.add(ConfigField.BAND_PLANNER_SCHEDULE_WINDOW_SIZE, window_size)
    if subgraph_type is not None:
        b.add(ConfigField.BAND_SUBGRAPH_PREPARATION_TYPE, int(subgraph_type))
    if minimum_subgraph_size is not None:
        b.add(ConfigField.BAND_MINIMUM_SUBGRAPH_SIZE, minimum_subgraph_size)
    if max_job_batch is not None:
        b.add(ConfigField.BANDX_WORKER_MAX_JOB_BATCH, max_job_batch)
    if share_identical is not None:
        b.add(ConfigField.BANDX_PROFILE_SHARE_IDENTICAL, int(bool(share_identical)))
    if pass_target_us:
        b.add(ConfigField.BANDX_WORKER_PASS_TARGET_US, int(pass_target_us))
    return b.build()


class Model:
    """BandModel (band/model.h): one model, backend models per backend type."""

    def __init__(self):
        self.lib = _lib()
        self.handle = c_void_p(self.lib.BandModelCreate())

    def FromPath(self, path, backend=kBandTfLite):
        return self.lib.BandModelAddFromFile(self.handle, backend, path.encode()) == kBandOk

    def FromBuffer(self, data, backend=kBandTfLite):
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        self._buf = buf
        return self.lib.BandModelAddFromBuffer(self.handle, backend, buf, len(data)) == kBandOk

    def GetId(self):
        return int(self.lib.BandxModelGetId(self.handle))

    def __del__(self):
        if getattr(self, "handle", None):
            self.lib.BandModelDelete(self.handle)
            self.handle = None


_NP = {1: np.float32, 2: np.int32, 3: np.uint8, 4: np.int64, 6: np.bool_, 7: np.int16, 9: np.int8,
       10: np.float16, 11: np.float64}


class Tensor:
    """BandTensor: a host tensor the engine created for a model's I/O."""

    def __init__(self, handle):
        self.lib = _lib()
        if not handle:
            raise _abi.BandHipError("tensor creation failed")
        self.handle = c_void_p(handle)

    def type(self):
        return int(self.lib.BandTensorGetType(self.handle))

    def dims(self):
        n = self.lib.BandTensorGetNumDims(self.handle)
        d = self.lib.BandTensorGetDims(self.handle)
        return [d[i] for i in range(n)]

    def nbytes(self):
        return int(self.lib.BandTensorGetBytes(self.handle))

    def name(self):
        r = self.lib.BandTensorGetName(self.handle)
        return r.decode() if r else ""

    def data(self):
        """numpy view of the tensor bytes (aliases the BandTensor)"""
        ptr = self.lib.BandTensorGetData(self.handle)
        dt = np.dtype(_NP.get(self.type(), np.uint8))
        n = self.nbytes() // dt.itemsize
        arr = np.ctypeslib.as_array(ctypes.cast(ptr, POINTER(ctypes.c_uint8)), shape=(self.nbytes(),))
        return arr.view(dt)[:n].reshape(self.dims())

    def __del__(self):
        if getattr(self, "handle", None):
            self.lib.BandTensorDelete(self.handle)
            self.handle = None


def _ptrs(tensors):
    return (c_void_p * max(len(tensors), 1))(*[t.handle.value for t in tensors])


class Engine:
    """BandEngine (band/engine.h): RegisterModel, tensors, requests."""

    def __init__(self, config=None):
        self.lib = _lib()
        h = self.lib.BandEngineCreate(config.handle) if config is not None else \
            self.lib.BandEngineCreateWithDefaultConfig()
        if not h:
            raise _abi.BandHipError("BandEngineCreate failed")
        self.handle = c_void_p(h)
        self._models = []
        self._callbacks = {}

    def RegisterModel(self, model):
        ok = self.lib.BandEngineRegisterModel(self.handle, model.handle) == kBandOk
        if ok:
            self._models.append(model)
        return ok

    def GetNumWorkers(self):
        return int(self.lib.BandEngineGetNumWorkers(self.handle))

    def GetWorkerDevice(self, worker_id):
        return int(self.lib.BandEngineGetWorkerDevice(self.handle, worker_id))

    def GetNumInputTensors(self, model):
        return int(self.lib.BandEngineGetNumInputTensors(self.handle, model.handle))

    def GetNumOutputTensors(self, model):
        return int(self.lib.BandEngineGetNumOutputTensors(self.handle, model.handle))

    def CreateInputTensor(self, model, index):
        return Tensor(self.lib.BandEngineCreateInputTensor(self.handle, model.handle, index))

    def CreateOutputTensor(self, model, index):
        return Tensor(self.lib.BandEngineCreateOutputTensor(self.handle, model.handle, index))

    def RequestSync(self, model, inputs, outputs, option=None):
        if option is None:
            return self.lib.BandEngineRequestSync(self.handle, model.handle, _ptrs(inputs), _ptrs(outputs))
        return self.lib.BandEngineRequestSyncOptions(self.handle, model.handle, option, _ptrs(inputs),
                                                     _ptrs(outputs))

    def RequestAsync(self, model, inputs, option=None):
        if option is None:
            return int(self.lib.BandEngineRequestAsync(self.handle, model.handle, _ptrs(inputs)))
        return int(self.lib.BandEngineRequestAsyncOptions(self.handle, model.handle, option, _ptrs(inputs)))

    def RequestsAsync(self, models, inputs):
        """One batched RequestAsync (Band's vector overload) of len(models)
        requests; returns the job handles, or None when the call is refused"""
        n = len(models)
        ms = (c_void_p * n)(*[m.handle.value for m in models])
        keep = [_ptrs(x) for x in inputs]
        ins = (c_void_p * n)(*[ctypes.cast(k, c_void_p) for k in keep])
        hs = (c_int * n)()
        if self.lib.BandxEngineRequestsAsync(self.handle, ms, n, ins, hs) != kBandOk:
            return None
        return list(hs)

    def Wait(self, handle, outputs):
        return self.lib.BandEngineWait(self.handle, handle, _ptrs(outputs), len(outputs))

    def WaitAll(self):
        self.lib.BandxEngineWaitAll(self.handle)

    def SetOnEndRequest(self, fn):
        cb = CALLBACK(lambda user, job, status: fn(job, status))
        h = int(self.lib.BandEngineSetOnEndRequest(self.handle, cb, None))
        self._callbacks[h] = cb
        return h

    def UnsetOnEndRequest(self, h):
        rc = self.lib.BandEngineUnsetOnEndRequest(self.handle, h)
        self._callbacks.pop(h, None)
        return rc

    def GetJobRecord(self, handle):
        r = JobRecord()
        if self.lib.BandxEngineGetJobRecord(self.handle, handle, ctypes.byref(r)) != kBandOk:
            return None
        return r

    def GetProfileJson(self):
        n = self.lib.BandxEngineGetProfileJson(self.handle, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        self.lib.BandxEngineGetProfileJson(self.handle, buf, n + 1)
        return json.loads(buf.value.decode())

    def DumpProfile(self):
        return self.lib.BandxEngineDumpProfile(self.handle) == kBandOk

    def GetSubgraphs(self, model):
        n = self.lib.BandxEngineGetSubgraphs(self.handle, model.handle, None, None, 0)
        ws = (c_int * max(n, 1))()
        ms = (c_uint64 * max(n, 1))()
        self.lib.BandxEngineGetSubgraphs(self.handle, model.handle, ws, ms, n)
        return [(ws[i], ms[i]) for i in range(n)]

    def GetWorkerJobCount(self, worker_id):
        """subgraph executions worker `worker_id` has finished (each job of a
        batched pass counted once; a split model once per subgraph)"""
        return int(self.lib.BandxEngineGetWorkerJobCount(self.handle, int(worker_id)))

    def GetWorkerPhaseTimes(self, worker_id):
        """host microseconds worker `worker_id` spent copying inputs, invoking
        (launch + sync) and copying outputs, and the passes it ran"""
        out = (c_int64 * 4)()
        if self.lib.BandxEngineGetWorkerPhaseTimes(self.handle, int(worker_id), out) != 0:
            raise _abi.BandHipError("GetWorkerPhaseTimes: bad worker id %d" % worker_id)
        return dict(copy_in_us=out[0], invoke_us=out[1], copy_out_us=out[2], passes=out[3])

    def GetDriverStats(self):
        """the last RunClosedLoop / RunPoisson call: wall time, mean requests
        inside the engine and waiting for a reader, submitter and reader time
        (include/band_c_api.h BandxEngineGetDriverStats)"""
        out = (ctypes.c_double * 8)()
        self.lib.BandxEngineGetDriverStats(self.handle, out)
        readers, lanes = int(out[7]) % 1000, int(out[7]) // 1000
        return dict(wall_us=out[0], mean_in_engine=out[1], mean_awaiting_read=out[2], submit_wait_us=out[3],
                    submit_call_us=out[4], read_busy_us=out[5], read_idle_us=out[6], readers=readers,
                    submitters=lanes)

    def GetRequestPhaseTimes(self):
        """{jobs, alloc_us, copy_us, enqueue_us}: cumulative RequestAsync cost
        split (include/band_c_api.h BandxEngineGetRequestPhaseTimes)"""
        out = (ctypes.c_int64 * 4)()
        self.lib.BandxEngineGetRequestPhaseTimes(self.handle, out)
        return dict(jobs=out[0], alloc_us=out[1], copy_us=out[2], enqueue_us=out[3])

    def GetExpectedLatency(self, model, worker_id, unit_mask):
        return int(self.lib.BandxEngineGetExpectedLatency(self.handle, model.handle, worker_id, unit_mask))

    def RunClosedLoop(self, models, n_jobs, max_inflight, inputs=None, with_models=False):
        """Native closed-loop driver (BandxEngineRunClosedLoopEx): n_jobs
        requests round-robin over `models`, <= max_inflight outstanding.
        Returns (latency_us array, worker id array, wall seconds), with the
        model index of every job before the wall time when with_models."""
        ms = (c_void_p * len(models))(*[m.handle.value for m in models])
        ins = None
        if inputs is not None:
            ins = (c_void_p * len(models))(*[t.handle.value if t is not None else None for t in inputs])
        lat = np.zeros(max(n_jobs, 1), np.float64)
        wid = np.zeros(max(n_jobs, 1), np.int32)
        mid = np.zeros(max(n_jobs, 1), np.int32)
        wall = c_double(0)
        rc = self.lib.BandxEngineRunClosedLoopEx(self.handle, ms, ins, len(models), int(n_jobs), int(max_inflight),
                                                 lat.ctypes.data_as(POINTER(c_double)),
                                                 wid.ctypes.data_as(POINTER(c_int)),
                                                 mid.ctypes.data_as(POINTER(c_int)), ctypes.byref(wall))
        if rc != kBandOk:
            raise _abi.BandHipError("BandxEngineRunClosedLoop: a job failed")
        if with_models:
            return lat[:n_jobs], wid[:n_jobs], mid[:n_jobs], wall.value
        return lat[:n_jobs], wid[:n_jobs], wall.value

    def RunPoisson(self, models, n_jobs, rate_per_s, seed=5489, max_inflight=64, inputs=None):
        """Native open-loop Poisson driver (BandxEngineRunPoisson).  Returns
        (latency_us, worker ids, model index per job, wall seconds)."""
        ms = (c_void_p * len(models))(*[m.handle.value for m in models])
        ins = None
        if inputs is not None:
            ins = (c_void_p * len(models))(*[t.handle.value if t is not None else None for t in inputs])
        lat = np.zeros(max(n_jobs, 1), np.float64)
        wid = np.zeros(max(n_jobs, 1), np.int32)
        mid = np.zeros(max(n_jobs, 1), np.int32)
        wall = c_double(0)
        rc = self.lib.BandxEngineRunPoisson(self.handle, ms, ins, len(models), int(n_jobs), float(rate_per_s),
                                            int(seed), int(max_inflight), lat.ctypes.data_as(POINTER(c_double)),
                                            wid.ctypes.data_as(POINTER(c_int)), mid.ctypes.data_as(POINTER(c_int)),
                                            ctypes.byref(wall))
        if rc != kBandOk:
            raise _abi.BandHipError("BandxEngineRunPoisson: a job failed")
        return lat[:n_jobs], wid[:n_jobs], mid[:n_jobs], wall.value

    def close(self):
        if getattr(self, "handle", None):
            self.lib.BandEngineDelete(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


def RequestOptionGetDefault():
    return _lib().BandRequestOptionGetDefault()


def BenchmarkRun(config):
    """band/tool/benchmark.cc over the native engine: `config` is the
    reference's benchmark JSON (dict or text); returns the result dict."""
    text = config if isinstance(config, str) else json.dumps(config)
    lib = _lib()
    cap = 1 << 20
    buf = ctypes.create_string_buffer(cap)
    n = lib.BandxBenchmarkRun(text.encode(), buf, cap)
    out = json.loads(buf.value.decode())
    if n == 0:
        raise _abi.BandHipError("benchmark failed: %s" % out.get("error"))
    return out
