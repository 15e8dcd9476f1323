"""Python mirror of Band's backend plugin interface over the HIP backend.

Same class / method names, argument meaning and error behaviour as the
reference's C++ interface (band/interface/*.h) and TFLite backend
(band/backend/tfl/*), so parity tests read like the reference's own
(band/test/backend/tfl_minimal_test.cc).  Every call goes through the C ABI
of libband_hip.so (include/band_hip_backend.h); there is no Python compute
and no fallback: a missing library raises.
"""
import ctypes
import enum
import json

import numpy as np

from . import _abi

c_int, c_void_p, c_size_t, c_uint64 = ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64


class TensorInfo(ctypes.Structure):
    _fields_ = [("type", c_int), ("ndims", c_int), ("dims", c_int * 8), ("data", c_void_p),
                ("bytes", c_size_t), ("name", ctypes.c_char_p), ("quant_type", c_int),
                ("n_quant", c_int), ("scale", ctypes.POINTER(ctypes.c_float)),
                ("zero_point", ctypes.POINTER(ctypes.c_int32)), ("quantized_dimension", c_int)]


class OpTiming(ctypes.Structure):
    _fields_ = [("op_index", c_int), ("kernel", ctypes.c_char_p), ("ms", ctypes.c_double),
                ("alg_bytes", ctypes.c_double), ("alg_ops", ctypes.c_double)]


_KEY = [c_void_p, c_int, c_int, c_uint64]
_abi.BACKEND_SYMBOLS.update({
    "bhx_last_error": (ctypes.c_char_p, []),
    "bhx_available_devices": (c_int, [ctypes.POINTER(ctypes.c_uint32)]),
    "bhx_set_worker_device": (c_int, [c_int, c_int]),
    "bhx_worker_device": (c_int, [c_int]),
    "bhx_model_create": (c_int, [c_int, ctypes.POINTER(c_void_p)]),
    "bhx_model_from_path": (c_int, [c_void_p, ctypes.c_char_p]),
    "bhx_model_from_buffer": (c_int, [c_void_p, ctypes.c_char_p, c_size_t]),
    "bhx_model_is_initialized": (c_int, [c_void_p]),
    "bhx_model_get_id": (c_int, [c_void_p]),
    "bhx_model_destroy": (None, [c_void_p]),
    "bhx_executor_create": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_void_p)]),
    "bhx_executor_create_masked": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_int), c_int,
                                           ctypes.POINTER(c_void_p)]),
    "bhx_executor_destroy": (None, [c_void_p]),
    "bhx_gpu_numa_node": (c_int, [c_int]),
    "bhx_gpu_numa_cpus": (c_int, [c_int, ctypes.POINTER(c_int), c_int]),
    "bhx_pin_process_to_gpu": (c_int, [c_int]),
    "bhx_pin_process_to_cpus": (c_int, [ctypes.POINTER(c_int), c_int]),
    "bhx_ring_page_nodes": (c_int, [ctypes.POINTER(ctypes.c_longlong), c_int]),
    "bhx_ring_host_alloc": (c_void_p, [c_size_t]),
    "bhx_ring_host_free": (None, [c_void_p]),
    "bhx_pin_worker_thread": (c_int, [c_int]),
    "bhx_investigate_model_spec": (c_int, [c_void_p, c_void_p, ctypes.c_char_p, c_size_t,
                                           ctypes.POINTER(c_size_t)]),
    "bhx_prepare_subgraph": (c_int, [c_void_p, c_void_p, ctypes.POINTER(c_int), c_int,
                                     ctypes.POINTER(c_int), c_int]),
    "bhx_has_subgraph": (c_int, _KEY),
    "bhx_get_inputs": (c_int, _KEY + [ctypes.POINTER(c_int), c_int, ctypes.POINTER(c_int)]),
    "bhx_get_outputs": (c_int, _KEY + [ctypes.POINTER(c_int), c_int, ctypes.POINTER(c_int)]),
    "bhx_get_input_name": (ctypes.c_char_p, _KEY + [c_int]),
    "bhx_get_output_name": (ctypes.c_char_p, _KEY + [c_int]),
    "bhx_get_num_tensors": (c_size_t, _KEY),
    "bhx_get_num_nodes": (c_size_t, _KEY),
    "bhx_get_tensor_view": (c_int, _KEY + [c_int, ctypes.POINTER(TensorInfo)]),
    "bhx_get_largest_subgraph_key": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                             ctypes.POINTER(c_uint64)]),
    "bhx_list_subgraphs": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                   ctypes.POINTER(c_uint64), c_int, ctypes.POINTER(c_int)]),
    "bhx_execute_subgraph": (c_int, _KEY),
    "bhx_run_jobs": (c_int, _KEY + [ctypes.POINTER(c_void_p), c_int, c_size_t, c_void_p, c_size_t, c_int,
                                    ctypes.POINTER(ctypes.c_double)]),
    "bhx_executor_set_graph": (c_int, [c_void_p, c_int]),
    "bhx_executor_device": (c_int, [c_void_p, ctypes.POINTER(c_int)]),
    "bhx_executor_coalescer": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "bhx_coalescer_stats": (c_int, [ctypes.POINTER(ctypes.c_longlong), c_int]),
    "bhx_profile_subgraph": (c_int, _KEY + [c_int, ctypes.POINTER(OpTiming), c_int, ctypes.POINTER(c_int),
                                            ctypes.POINTER(ctypes.c_double)]),
    "bhx_time_subgraph": (c_int, _KEY + [c_int, ctypes.POINTER(ctypes.c_double)]),
    "bhx_prepare_job_batches": (c_int, [c_void_p, c_void_p, c_int, c_int, ctypes.c_uint64, c_int]),
    "bhx_max_job_batch": (c_int, _KEY + [ctypes.POINTER(c_int)]),
    "bhx_job_slot_view": (c_int, _KEY + [c_int, c_int, c_int, ctypes.POINTER(TensorInfo)]),
    "bhx_execute_job_batch": (c_int, _KEY + [c_int]),
    "bhx_run_mixed_jobs": (c_int, [c_int, ctypes.POINTER(c_void_p), ctypes.POINTER(c_int), c_int, ctypes.c_uint64,
                                   ctypes.POINTER(c_void_p), c_int, c_int, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(c_int)]),
})


class DeviceFlag(enum.IntEnum):  # band/common.h:163-168
    kCPU = 0
    kGPU = 1
    kDSP = 2
    kNPU = 3


class DataType(enum.IntEnum):  # band/common.h:115-128 (== TfLiteType)
    kNoType = 0
    kFloat32 = 1
    kInt32 = 2
    kUInt8 = 3
    kInt64 = 4
    kString = 5
    kBool = 6
    kInt16 = 7
    kComplex64 = 8
    kInt8 = 9
    kFloat16 = 10
    kFloat64 = 11


NP_OF = {DataType.kFloat32: np.float32, DataType.kInt32: np.int32, DataType.kUInt8: np.uint8,
         DataType.kInt64: np.int64, DataType.kBool: np.bool_, DataType.kInt16: np.int16,
         DataType.kInt8: np.int8, DataType.kFloat16: np.float16, DataType.kFloat64: np.float64}


class StatusCode(enum.IntEnum):
    kOk = 0
    kInternal = 13


class Status:
    """absl::Status stand-in returned by the mirrored methods."""

    def __init__(self, code=0, message=""):
        self._code = int(code)
        self._message = message

    def ok(self):
        return self._code == 0

    def code(self):
        return self._code

    def message(self):
        return self._message

    def __bool__(self):
        return self.ok()

    def __repr__(self):
        return "Status(OK)" if self.ok() else "Status(%d, %r)" % (self._code, self._message)

    @staticmethod
    def from_rc(rc):
        if rc == 0:
            return Status()
        msg = _abi.load().bhx_last_error()
        return Status(rc, msg.decode() if msg else "")


class SubgraphKey:
    """band/common.h:293-319 — (model id, worker id, unit-subgraph bitmask)."""

    def __init__(self, model_id=-1, worker_id=-1, unit_indices=()):
        self.model_id = int(model_id)
        self.worker_id = int(worker_id)
        self.mask = 0
        for u in unit_indices:
            self.mask |= 1 << int(u)

    @classmethod
    def from_mask(cls, model_id, worker_id, mask):
        k = cls(model_id, worker_id)
        k.mask = int(mask)
        return k

    def GetModelId(self):
        return self.model_id

    def GetWorkerId(self):
        return self.worker_id

    def GetUnitIndicesSet(self):
        return {i for i in range(64) if self.mask >> i & 1}

    def IsValid(self):
        return self.model_id != -1 and self.worker_id != -1

    def _args(self):
        return (self.model_id, self.worker_id, self.mask)

    def __eq__(self, o):
        return isinstance(o, SubgraphKey) and self._args() == o._args()

    def __hash__(self):
        return hash(self._args())

    def __repr__(self):
        return "SubgraphKey(%d, %d, %s)" % (self.model_id, self.worker_id, sorted(self.GetUnitIndicesSet()))


class ModelSpec:
    """band/model_spec.h — what InvestigateModelSpec returns."""

    def __init__(self, d):
        self.num_ops = d["num_ops"]
        self.num_tensors = d["num_tensors"]
        self.tensor_types = [DataType(t) for t in d["tensor_types"]]
        self.input_tensors = set(d["input_tensors"])
        self.output_tensors = set(d["output_tensors"])
        self.op_input_tensors = [set(s) for s in d["op_input_tensors"]]
        self.op_output_tensors = [set(s) for s in d["op_output_tensors"]]
        self.unsupported_ops = {DeviceFlag(int(k)): set(v) for k, v in d["unsupported_ops"].items()}
        self.unavailable_devices = {DeviceFlag(f) for f in d["unavailable_devices"]}
        self.path = d["path"]

    def GetPureInputTensors(self, ops):  # band/model_spec.cc:9-31
        ins = set()
        for o in ops:
            ins |= self.op_input_tensors[o]
        for o in ops:
            ins -= self.op_output_tensors[o]
        return ins

    def GetOutputTensors(self, ops):  # band/model_spec.cc:33-43
        out = set()
        for o in ops:
            out |= self.op_output_tensors[o]
        return out


def GetAvailableDevices():
    """IBackendUtil::GetAvailableDevices (band/interface/backend.h:21-26)."""
    m = ctypes.c_uint32()
    _abi.check(_abi.load().bhx_available_devices(ctypes.byref(m)), "GetAvailableDevices")
    return {DeviceFlag(i) for i in range(4) if m.value >> i & 1}


def SetWorkerDevice(worker_id, ordinal):
    _abi.load().bhx_set_worker_device(int(worker_id), int(ordinal))


def WorkerDevice(worker_id):
    """the GPU ordinal worker `worker_id`'s executors use (DeviceRegistry)"""
    return int(_abi.load().bhx_worker_device(int(worker_id)))


class HipModel:
    """IModel (band/interface/model.h:17-38) of the HIP backend."""

    def __init__(self, model_id):
        self.lib = _abi.load()
        h = c_void_p()
        _abi.check(self.lib.bhx_model_create(int(model_id), ctypes.byref(h)), "CreateModel")
        self.handle = h
        self._path = ""

    def FromPath(self, filename):
        self._path = str(filename)
        return Status.from_rc(self.lib.bhx_model_from_path(self.handle, str(filename).encode()))

    def FromBuffer(self, buffer):
        b = bytes(buffer)
        return Status.from_rc(self.lib.bhx_model_from_buffer(self.handle, b, len(b)))

    def IsInitialized(self):
        return bool(self.lib.bhx_model_is_initialized(self.handle))

    def GetId(self):
        return self.lib.bhx_model_get_id(self.handle)

    def GetPath(self):
        return self._path

    def __del__(self):
        try:
            if self.handle:
                self.lib.bhx_model_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class HipTensorView:
    """ITensorView (band/interface/tensor.h:27-50): aliases executor memory."""

    def __init__(self, info, owner):
        self._info = info
        self._owner = owner  # keeps the executor (and its memory) alive

    def GetType(self):
        return DataType(self._info.type)

    def GetDims(self):
        return [self._info.dims[i] for i in range(self._info.ndims)]

    def GetNumDims(self):
        return self._info.ndims

    def GetBytes(self):
        return int(self._info.bytes)

    def GetNumElements(self):
        return int(np.prod(self.GetDims())) if self._info.ndims else 1

    def GetName(self):
        return self._info.name.decode() if self._info.name else ""

    def GetQuantization(self):
        if self._info.quant_type != 1:
            return None
        n = self._info.n_quant
        return dict(scale=[self._info.scale[i] for i in range(n)],
                    zero_point=[self._info.zero_point[i] for i in range(n)],
                    quantized_dimension=self._info.quantized_dimension)

    def GetData(self):
        """numpy array aliasing the view's host memory (typed, shaped)."""
        if not self._info.data:
            return None
        dt = NP_OF[self.GetType()]
        buf = (ctypes.c_char * self.GetBytes()).from_address(self._info.data)
        return np.frombuffer(buf, dtype=dt).reshape(self.GetDims())

    def __eq__(self, rhs):  # band/interface/tensor.cc:24-34
        return self.GetType() == rhs.GetType() and self.GetDims() == rhs.GetDims()

    def CopyDataFrom(self, rhs):  # band/interface/tensor.cc:55-69
        if rhs is None:
            return Status(13, "Tried to copy null tensor")
        if not (self == rhs):
            return Status(13, "")
        src = rhs.GetData() if isinstance(rhs, HipTensorView) else np.asarray(rhs)
        dst = self.GetData()
        dst.reshape(-1).view(np.uint8)[:] = np.ascontiguousarray(src).reshape(-1).view(np.uint8)
        return Status()


class HipModelExecutor:
    """IModelExecutor (band/interface/model_executor.h:30-180) of the HIP backend."""

    def __init__(self, model_id, worker_id, device_flag, num_threads=-1, cpus=None):
        """cpus: the executor's CpuSet (CPU ids); a kCPU executor pins its host
        thread pool to it (band/backend/tfl/model_executor.cc:356-359)"""
        self.lib = _abi.load()
        h = c_void_p()
        if cpus:
            arr = (c_int * len(cpus))(*[int(c) for c in cpus])
            _abi.check(self.lib.bhx_executor_create_masked(int(model_id), int(worker_id), int(device_flag),
                                                           int(num_threads), arr, len(cpus), ctypes.byref(h)),
                       "CreateModelExecutor")
        else:
            _abi.check(self.lib.bhx_executor_create(int(model_id), int(worker_id), int(device_flag),
                                                    int(num_threads), ctypes.byref(h)), "CreateModelExecutor")
        self.handle = h
        self.model_id, self.worker_id, self.device_flag = int(model_id), int(worker_id), DeviceFlag(device_flag)

    def InvestigateModelSpec(self, model):
        need = c_size_t(0)
        self.lib.bhx_investigate_model_spec(self.handle, model.handle, None, 0, ctypes.byref(need))
        if need.value == 0:
            raise _abi.BandHipError(self.lib.bhx_last_error().decode())
        buf = ctypes.create_string_buffer(need.value)
        _abi.check(self.lib.bhx_investigate_model_spec(self.handle, model.handle, buf, need.value,
                                                       ctypes.byref(need)), "InvestigateModelSpec")
        return ModelSpec(json.loads(buf.value.decode()))

    def PrepareSubgraph(self, model, ops=(), unit_indices=()):
        ops = sorted(set(ops))
        units = sorted(set(unit_indices))
        oa = (c_int * max(len(ops), 1))(*ops)
        ua = (c_int * max(len(units), 1))(*units)
        return Status.from_rc(self.lib.bhx_prepare_subgraph(self.handle, model.handle, oa, len(ops), ua, len(units)))

    def _idx(self, fn, key):
        n = c_int(0)
        fn(self.handle, *key._args(), None, 0, ctypes.byref(n))
        arr = (c_int * max(n.value, 1))()
        fn(self.handle, *key._args(), arr, n.value, ctypes.byref(n))
        return [arr[i] for i in range(n.value)]

    def GetInputs(self, key):
        return self._idx(self.lib.bhx_get_inputs, key)

    def GetOutputs(self, key):
        return self._idx(self.lib.bhx_get_outputs, key)

    def GetInputName(self, key, index):
        r = self.lib.bhx_get_input_name(self.handle, *key._args(), int(index))
        return r.decode() if r is not None else None

    def GetOutputName(self, key, index):
        r = self.lib.bhx_get_output_name(self.handle, *key._args(), int(index))
        return r.decode() if r is not None else None

    def GetNumTensors(self, key):
        return int(self.lib.bhx_get_num_tensors(self.handle, *key._args()))

    def GetNumNodes(self, key):
        return int(self.lib.bhx_get_num_nodes(self.handle, *key._args()))

    def GetTensorView(self, key, index):
        info = TensorInfo()
        rc = self.lib.bhx_get_tensor_view(self.handle, *key._args(), int(index), ctypes.byref(info))
        return None if rc != 0 else HipTensorView(info, self)

    def HasSubgraph(self, key):
        return bool(self.lib.bhx_has_subgraph(self.handle, *key._args()))

    def GetLargestSubgraphKey(self):
        m, w, k = c_int(), c_int(), c_uint64()
        self.lib.bhx_get_largest_subgraph_key(self.handle, ctypes.byref(m), ctypes.byref(w), ctypes.byref(k))
        return SubgraphKey.from_mask(m.value, w.value, k.value)

    def ForEachSubgraph(self, visitor):
        n = c_int(0)
        self.lib.bhx_list_subgraphs(self.handle, None, None, None, 0, ctypes.byref(n))
        cnt = max(n.value, 1)
        ms, ws, ks = (c_int * cnt)(), (c_int * cnt)(), (c_uint64 * cnt)()
        self.lib.bhx_list_subgraphs(self.handle, ms, ws, ks, n.value, ctypes.byref(n))
        for i in range(n.value):
            visitor(SubgraphKey.from_mask(ms[i], ws[i], ks[i]))

    def ExecuteSubgraph(self, key):
        return Status.from_rc(self.lib.bhx_execute_subgraph(self.handle, *key._args()))

    # ---- job batching (backend/hip/job_batching.h) -------------------
    def PrepareJobBatches(self, model, key, max_batch):
        return Status.from_rc(self.lib.bhx_prepare_job_batches(self.handle, model.handle, *key._args(),
                                                               int(max_batch)))

    def MaxJobBatch(self, key):
        n = c_int(1)
        _abi.check(self.lib.bhx_max_job_batch(self.handle, *key._args(), ctypes.byref(n)), "MaxJobBatch")
        return n.value

    def GetJobSlotView(self, key, index, n, slot):
        info = TensorInfo()
        rc = self.lib.bhx_job_slot_view(self.handle, *key._args(), int(index), int(n), int(slot), ctypes.byref(info))
        return None if rc != 0 else HipTensorView(info, self)

    def ExecuteJobBatch(self, key, n):
        return Status.from_rc(self.lib.bhx_execute_job_batch(self.handle, *key._args(), int(n)))

    # ---- extensions -----------------------------------------------------
    def RunJobs(self, key, inputs, n_jobs, out=None):
        """Native Band-worker loop (bhx_run_jobs): returns per-job latency in us."""
        arrs = [np.ascontiguousarray(a) for a in inputs]
        slots = (c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        lat = np.zeros(max(n_jobs, 1), np.float64)
        out_p = out.ctypes.data if out is not None else None
        out_n = out.nbytes if out is not None else 0
        rc = self.lib.bhx_run_jobs(self.handle, *key._args(), slots, len(arrs), arrs[0].nbytes, out_p, out_n,
                                   int(n_jobs), lat.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        st = Status.from_rc(rc)
        if not st.ok():
            raise _abi.BandHipError("bhx_run_jobs: " + st.message())
        return lat[:n_jobs]

    def SetUseGraph(self, enabled):
        _abi.check(self.lib.bhx_executor_set_graph(self.handle, int(bool(enabled))), "set_graph")

    def DeviceOrdinal(self):
        o = c_int(-1)
        _abi.check(self.lib.bhx_executor_device(self.handle, ctypes.byref(o)), "device")
        return o.value

    def Coalescer(self):
        """(members, lanes_ready) of the job coalescer this executor's
        whole-model subgraph joined ((0, False): none)"""
        m, r = c_int(0), c_int(0)
        _abi.check(self.lib.bhx_executor_coalescer(self.handle, ctypes.byref(m), ctypes.byref(r)), "coalescer")
        return m.value, bool(r.value)

    def ProfileSubgraph(self, key, iters=10, with_floor=False):
        """per-launch kernel durations in program order (ms each; dispatch
        begin / end timestamps, as rocprofv3 reports them); with_floor: also
        the duration (us) of an empty single-wave kernel"""
        n = c_int(0)
        cap = 4096
        arr = (OpTiming * cap)()
        floor = ctypes.c_double(0)
        _abi.check(self.lib.bhx_profile_subgraph(self.handle, *key._args(), int(iters), arr, cap, ctypes.byref(n),
                                                 ctypes.byref(floor)), "ProfileSubgraph")
        rows = [dict(op_index=arr[i].op_index, kernel=arr[i].kernel.decode(), ms=arr[i].ms,
                     alg_bytes=arr[i].alg_bytes, alg_ops=arr[i].alg_ops) for i in range(min(n.value, cap))]
        return (rows, floor.value) if with_floor else rows

    def TimeSubgraph(self, key, iters=100):
        """device microseconds per subgraph pass, passes issued back to back"""
        us = ctypes.c_double(0)
        _abi.check(self.lib.bhx_time_subgraph(self.handle, *key._args(), int(iters), ctypes.byref(us)),
                   "TimeSubgraph")
        return us.value

    def __del__(self):
        try:
            if self.handle:
                self.lib.bhx_executor_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def RunMixedJobs(executors, keys, requests, n_jobs, first_model=0):
    """Native Band-worker loop over a mixed request stream (bhx_run_mixed_jobs).
    executors / keys / requests: one per model, all keys on the same worker.
    Returns (latency_us[n_jobs], model_of_job[n_jobs])."""
    lib = _abi.load()
    n = len(executors)
    wids = {k.worker_id for k in keys}
    if len(wids) != 1 or len(keys) != n or len(requests) != n:
        raise ValueError("one executor / key / request per model, one worker")
    arrs = [np.ascontiguousarray(r) for r in requests]
    ex_arr = (c_void_p * n)(*[e.handle for e in executors])
    mids = (c_int * n)(*[k.model_id for k in keys])
    req = (c_void_p * n)(*[a.ctypes.data for a in arrs])
    lat = np.zeros(max(n_jobs, 1), np.float64)
    mo = np.zeros(max(n_jobs, 1), np.int32)
    rc = lib.bhx_run_mixed_jobs(n, ex_arr, mids, keys[0].worker_id, keys[0]._args()[2], req, int(first_model),
                                int(n_jobs), lat.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                mo.ctypes.data_as(ctypes.POINTER(c_int)))
    st = Status.from_rc(rc)
    if not st.ok():
        raise _abi.BandHipError("bhx_run_mixed_jobs: " + st.message())
    return lat[:n_jobs], mo[:n_jobs]


def GpuNumaCpus(ordinal):
    """(NUMA node, CPUs of that node the process may use) of GPU `ordinal`:
    where a kGPU executor pins its worker thread (backend/hip/affinity.h)"""
    lib = _abi.load()
    node = int(lib.bhx_gpu_numa_node(int(ordinal)))
    cap = 4096
    arr = (c_int * cap)()
    n = int(lib.bhx_gpu_numa_cpus(int(ordinal), arr, cap))
    return node, [arr[i] for i in range(min(n, cap))]


def PinProcessToGpu(ordinal):
    """pins every thread of this process to GPU `ordinal`'s NUMA node
    (backend/hip/affinity.h PinProcessToGpu); returns the threads pinned
    (0: nothing to do)"""
    return int(_abi.load().bhx_pin_process_to_gpu(int(ordinal)))


def PinProcessToCpus(cpus):
    """pins every thread of this process to `cpus` (the core of
    PinProcessToGpu); returns the threads pinned, -1 on failure"""
    cpus = list(cpus)
    arr = (c_int * max(1, len(cpus)))(*cpus)
    return int(_abi.load().bhx_pin_process_to_cpus(arr, len(cpus)))


def CoalescerStats(reset=False):
    """process-wide job coalescing totals: calls, solo passes, group passes,
    jobs in group passes, largest group, calls run with coalescing off (no
    lanes) and the most of those at once (coalescer.h)"""
    arr = (ctypes.c_longlong * 7)()
    _abi.check(_abi.load().bhx_coalescer_stats(arr, int(bool(reset))), "coalescer_stats")
    keys = ("calls", "solo_passes", "group_passes", "group_jobs", "max_group", "bypass_calls",
            "max_bypass_inflight")
    return {k: int(v) for k, v in zip(keys, arr)}


def RingPageNodes():
    """{node: bytes} of the page-locked request-ring memory allocated so far
    (-1: node unknown), sampled every 16th page"""
    cap = 65
    arr = (ctypes.c_longlong * cap)()
    n = int(_abi.load().bhx_ring_page_nodes(arr, cap))
    return {(i if i < 64 else -1): int(arr[i]) for i in range(min(n, cap)) if arr[i]}
