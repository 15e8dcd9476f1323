// C ABI over the HIP backend (include/band_hip_backend.h).  Objects are
// created through Band's own BackendFactory so the registration path
// (TfLiteRegisterCreators -> RegisterBackendCreators) is exercised exactly
// as a Band engine would exercise it.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include "backend/hip/affinity.h"
#include "backend/hip/backend.h"
#include "band_hip_backend.h"

using band::BackendFactory;
using band::BackendType;
using band::DeviceFlag;
using band::SubgraphKey;

struct bhx_model {
  std::unique_ptr<band::interface::IModel> model;
};
struct bhx_executor {
  std::unique_ptr<band::interface::IModelExecutor> exec;
};

namespace {
thread_local std::string g_err;

int Fail(const absl::Status& s) {
  g_err = s.message();
  return static_cast<int>(s.code());
}
int Fail(const char* m) {
  g_err = m;
  return static_cast<int>(absl::StatusCode::kInternal);
}

SubgraphKey Key(int model_id, int worker_id, uint64_t mask) {
  std::set<int> units;
  for (int i = 0; i < 64; ++i)
    if (mask >> i & 1ull) units.insert(i);
  return SubgraphKey(model_id, worker_id, units);
}

void JsonSet(std::string& s, const std::set<int>& v) {
  s += "[";
  bool first = true;
  for (int x : v) {
    if (!first) s += ",";
    s += std::to_string(x);
    first = false;
  }
  s += "]";
}
}  // namespace

extern "C" {

const char* bhx_last_error(void) { return g_err.c_str(); }

int bhx_available_devices(uint32_t* mask) {
  if (!mask) return Fail("null mask");
  std::unique_ptr<band::interface::IBackendUtil> u(BackendFactory::GetBackendUtil(BackendType::kTfLite));
  if (!u) return Fail("HIP backend not registered");
  *mask = 0;
  for (DeviceFlag f : u->GetAvailableDevices()) *mask |= 1u << static_cast<int>(f);
  return 0;
}

int bhx_set_worker_device(int worker_id, int ordinal) {
  band::hip::DeviceRegistry::Get().SetWorkerOrdinal(worker_id, ordinal);
  return 0;
}

int bhx_worker_device(int worker_id) { return band::hip::DeviceRegistry::Get().OrdinalForWorker(worker_id); }

int bhx_model_create(int model_id, bhx_model** out) {
  if (!out) return Fail("null out");
  auto* m = BackendFactory::CreateModel(BackendType::kTfLite, model_id);
  if (!m) return Fail("HIP backend not registered");
  *out = new bhx_model{std::unique_ptr<band::interface::IModel>(m)};
  return 0;
}
int bhx_model_from_path(bhx_model* m, const char* path) {
  if (!m) return Fail("null model");
  auto s = m->model->FromPath(path);
  return s.ok() ? 0 : Fail(s);
}
int bhx_model_from_buffer(bhx_model* m, const char* buf, size_t n) {
  if (!m) return Fail("null model");
  auto s = m->model->FromBuffer(buf, n);
  return s.ok() ? 0 : Fail(s);
}
int bhx_model_is_initialized(const bhx_model* m) { return m && m->model->IsInitialized() ? 1 : 0; }
int bhx_model_get_id(const bhx_model* m) { return m ? m->model->GetId() : -1; }
void bhx_model_destroy(bhx_model* m) { delete m; }

int bhx_executor_create(int model_id, int worker_id, int device_flag, int num_threads, bhx_executor** out) {
  if (!out || device_flag < 0 || device_flag > 3) return Fail("bad arguments");
  auto* e = BackendFactory::CreateModelExecutor(BackendType::kTfLite, model_id, worker_id,
                                                static_cast<DeviceFlag>(device_flag),
                                                band::BandCPUMaskGetSet(band::CPUMaskFlag::kAll), num_threads);
  if (!e) return Fail("HIP backend not registered");
  *out = new bhx_executor{std::unique_ptr<band::interface::IModelExecutor>(e)};
  return 0;
}
int bhx_executor_create_masked(int model_id, int worker_id, int device_flag, int num_threads, const int* cpus,
                               int n_cpus, bhx_executor** out) {
  if (!out || device_flag < 0 || device_flag > 3 || n_cpus < 0 || (n_cpus > 0 && !cpus)) return Fail("bad arguments");
  band::CpuSet mask;  // empty: "no constraint", like an all-CPU set
  for (int i = 0; i < n_cpus; ++i) mask.Enable(cpus[i]);
  auto* e = BackendFactory::CreateModelExecutor(BackendType::kTfLite, model_id, worker_id,
                                                static_cast<DeviceFlag>(device_flag), mask, num_threads);
  if (!e) return Fail("HIP backend not registered");
  *out = new bhx_executor{std::unique_ptr<band::interface::IModelExecutor>(e)};
  return 0;
}
void bhx_executor_destroy(bhx_executor* e) { delete e; }

int bhx_gpu_numa_node(int ordinal) { return band::hip::GpuNumaNode(ordinal); }

int bhx_gpu_numa_cpus(int ordinal, int* cpus, int cap) {
  const std::vector<int> v = band::hip::GpuNumaCpus(ordinal);
  for (int i = 0; i < cap && i < static_cast<int>(v.size()); ++i) cpus[i] = v[i];
  return static_cast<int>(v.size());
}

int bhx_ring_page_nodes(long long* bytes_per_node, int cap) {
  if (cap < 0 || (cap > 0 && !bytes_per_node)) return Fail("bad arguments");
  return band::hip::RingPageNodes(bytes_per_node, cap);
}

int bhx_pin_process_to_gpu(int ordinal) { return band::hip::PinProcessToGpu(ordinal); }

int bhx_pin_worker_thread(int worker_id) {
  const int ordinal = band::hip::DeviceRegistry::Get().FindWorkerOrdinal(worker_id);
  if (ordinal < 0) return -1;
  return band::hip::PinCallingThreadToGpu(ordinal) ? 1 : 0;
}

int bhx_pin_process_to_cpus(const int* cpus, int n_cpus) {
  if (n_cpus <= 0 || !cpus) return -1;
  return band::hip::PinProcessToCpus(std::vector<int>(cpus, cpus + n_cpus));
}

int bhx_investigate_model_spec(bhx_executor* e, bhx_model* m, char* buf, size_t cap, size_t* needed) {
  if (!e || !m) return Fail("null argument");
  auto r = e->exec->InvestigateModelSpec(m->model.get());
  if (!r.ok()) return Fail(r.status());
  const band::ModelSpec& s = r.value();
  std::string j = "{\"num_ops\":" + std::to_string(s.num_ops) + ",\"num_tensors\":" + std::to_string(s.num_tensors);
  j += ",\"tensor_types\":[";
  for (size_t i = 0; i < s.tensor_types.size(); ++i)
    j += (i ? "," : "") + std::to_string(static_cast<int>(s.tensor_types[i]));
  j += "],\"input_tensors\":";
  JsonSet(j, s.input_tensors);
  j += ",\"output_tensors\":";
  JsonSet(j, s.output_tensors);
  j += ",\"op_input_tensors\":[";
  for (size_t i = 0; i < s.op_input_tensors.size(); ++i) {
    if (i) j += ",";
    JsonSet(j, s.op_input_tensors[i]);
  }
  j += "],\"op_output_tensors\":[";
  for (size_t i = 0; i < s.op_output_tensors.size(); ++i) {
    if (i) j += ",";
    JsonSet(j, s.op_output_tensors[i]);
  }
  j += "],\"unsupported_ops\":{";
  bool first = true;
  for (const auto& kv : s.unsupported_ops) {
    if (!first) j += ",";
    first = false;
    j += "\"" + std::to_string(static_cast<int>(kv.first)) + "\":";
    JsonSet(j, kv.second);
  }
  j += "},\"unavailable_devices\":[";
  first = true;
  for (DeviceFlag f : s.unavailable_devices) {
    if (!first) j += ",";
    first = false;
    j += std::to_string(static_cast<int>(f));
  }
  j += "],\"path\":\"";
  for (char c : s.path) {
    if (c == '"' || c == '\\') j += '\\';
    j += c;
  }
  j += "\"}";
  if (needed) *needed = j.size() + 1;
  if (!buf || cap < j.size() + 1) return Fail("buffer too small");
  std::memcpy(buf, j.c_str(), j.size() + 1);
  return 0;
}

int bhx_prepare_subgraph(bhx_executor* e, bhx_model* m, const int* ops, int n_ops, const int* units, int n_units) {
  if (!e || !m) return Fail("null argument");
  std::set<int> o, u;
  for (int i = 0; i < n_ops; ++i) o.insert(ops[i]);
  for (int i = 0; i < n_units; ++i) u.insert(units[i]);
  auto s = e->exec->PrepareSubgraph(m->model.get(), o, u);
  return s.ok() ? 0 : Fail(s);
}

int bhx_has_subgraph(bhx_executor* e, int mid, int wid, uint64_t mask) {
  return e && e->exec->HasSubgraph(Key(mid, wid, mask)) ? 1 : 0;
}

static int CopyIdx(const std::vector<int>& v, int* out, int cap, int* n) {
  if (n) *n = static_cast<int>(v.size());
  for (int i = 0; i < cap && i < static_cast<int>(v.size()); ++i) out[i] = v[i];
  return 0;
}
int bhx_get_inputs(bhx_executor* e, int mid, int wid, uint64_t mask, int* out, int cap, int* n) {
  if (!e) return Fail("null executor");
  return CopyIdx(e->exec->GetInputs(Key(mid, wid, mask)), out, cap, n);
}
int bhx_get_outputs(bhx_executor* e, int mid, int wid, uint64_t mask, int* out, int cap, int* n) {
  if (!e) return Fail("null executor");
  return CopyIdx(e->exec->GetOutputs(Key(mid, wid, mask)), out, cap, n);
}
const char* bhx_get_input_name(bhx_executor* e, int mid, int wid, uint64_t mask, int index) {
  return e ? e->exec->GetInputName(Key(mid, wid, mask), index) : nullptr;
}
const char* bhx_get_output_name(bhx_executor* e, int mid, int wid, uint64_t mask, int index) {
  return e ? e->exec->GetOutputName(Key(mid, wid, mask), index) : nullptr;
}
size_t bhx_get_num_tensors(bhx_executor* e, int mid, int wid, uint64_t mask) {
  return e ? e->exec->GetNumTensors(Key(mid, wid, mask)) : 0;
}
size_t bhx_get_num_nodes(bhx_executor* e, int mid, int wid, uint64_t mask) {
  return e ? e->exec->GetNumNodes(Key(mid, wid, mask)) : 0;
}

namespace {
int FillInfo(const std::shared_ptr<band::interface::ITensorView>& v, bhx_tensor_info* info) {
  if (!v) return Fail("Cannot find tensor view");
  std::memset(info, 0, sizeof(*info));
  info->type = static_cast<int>(v->GetType());
  info->ndims = static_cast<int>(v->GetNumDims());
  for (int i = 0; i < info->ndims && i < 8; ++i) info->dims[i] = v->GetDims()[i];
  info->data = v->GetData();
  info->bytes = v->GetBytes();
  info->name = v->GetName();
  band::Quantization q = v->GetQuantization();
  info->quant_type = static_cast<int>(q.GetType());
  if (q.GetType() == band::QuantizationType::kAffineQuantization && q.GetParams()) {
    auto* a = static_cast<band::hip::QAffine*>(q.GetParams());
    info->n_quant = a->scale->size;
    info->scale = a->scale->data;
    info->zero_point = a->zero_point->data;
    info->quantized_dimension = a->quantized_dimension;
  }
  return 0;
}
}  // namespace

int bhx_get_tensor_view(bhx_executor* e, int mid, int wid, uint64_t mask, int t, bhx_tensor_info* info) {
  if (!e || !info) return Fail("null argument");
  return FillInfo(e->exec->GetTensorView(Key(mid, wid, mask), t), info);
}

int bhx_get_largest_subgraph_key(bhx_executor* e, int* mid, int* wid, uint64_t* mask) {
  if (!e) return Fail("null executor");
  SubgraphKey k = e->exec->GetLargestSubgraphKey();
  if (mid) *mid = k.GetModelId();
  if (wid) *wid = k.GetWorkerId();
  if (mask) *mask = k.GetUnitIndices().to_ullong();
  return 0;
}

int bhx_list_subgraphs(bhx_executor* e, int* mids, int* wids, uint64_t* masks, int cap, int* n) {
  if (!e) return Fail("null executor");
  int i = 0;
  e->exec->ForEachSubgraph([&](const SubgraphKey& k) {
    if (i < cap) {
      if (mids) mids[i] = k.GetModelId();
      if (wids) wids[i] = k.GetWorkerId();
      if (masks) masks[i] = k.GetUnitIndices().to_ullong();
    }
    ++i;
  });
  if (n) *n = i;
  return 0;
}

int bhx_execute_subgraph(bhx_executor* e, int mid, int wid, uint64_t mask) {
  if (!e) return Fail("null executor");
  auto s = e->exec->ExecuteSubgraph(Key(mid, wid, mask));
  return s.ok() ? 0 : Fail(s);
}

int bhx_run_jobs(bhx_executor* e, int mid, int wid, uint64_t mask, const void* const* in_slots, int n_slots,
                 size_t in_bytes, void* out, size_t out_bytes, int n_jobs, double* latency_us) {
  if (!e || !in_slots || n_slots <= 0 || n_jobs < 0) return Fail("bad arguments");
  const SubgraphKey key = Key(mid, wid, mask);
  const auto& ins = e->exec->GetInputs(key);
  const auto& outs = e->exec->GetOutputs(key);
  if (ins.size() != 1 || outs.size() != 1) return Fail("bhx_run_jobs needs a single-input, single-output subgraph");
  auto iv = e->exec->GetTensorView(key, ins[0]);
  auto ov = e->exec->GetTensorView(key, outs[0]);
  if (!iv || !ov || iv->GetBytes() != in_bytes || (out && ov->GetBytes() != out_bytes))
    return Fail("request / view size mismatch");
  for (int j = 0; j < n_jobs; ++j) {
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(iv->GetData(), in_slots[j % n_slots], in_bytes);
    absl::Status s = e->exec->ExecuteSubgraph(key);
    if (!s.ok()) return Fail(s);
    if (out) std::memcpy(out, ov->GetData(), out_bytes);
    if (latency_us)
      latency_us[j] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  return 0;
}

int bhx_run_mixed_jobs(int n_models, bhx_executor* const* execs, const int* mids, int wid, uint64_t mask,
                       const void* const* requests, int first_model, int n_jobs, double* latency_us,
                       int* model_of_job) {
  if (n_models <= 0 || !execs || !mids || !requests || n_jobs < 0) return Fail("bad arguments");
  struct Slot {
    band::interface::IModelExecutor* ex;
    SubgraphKey key;
    std::shared_ptr<band::interface::ITensorView> in;
    std::vector<std::shared_ptr<band::interface::ITensorView>> outs;
    std::vector<char> sink;  // the job's output ring slot (TryCopyOutputTensors)
  };
  std::vector<Slot> slots;
  for (int m = 0; m < n_models; ++m) {
    if (!execs[m] || !requests[m]) return Fail("bad arguments");
    Slot sl{execs[m]->exec.get(), Key(mids[m], wid, mask), nullptr, {}, {}};
    const auto& ins = sl.ex->GetInputs(sl.key);
    if (ins.size() != 1) return Fail("bhx_run_mixed_jobs needs single-input subgraphs");
    sl.in = sl.ex->GetTensorView(sl.key, ins[0]);
    size_t ob = 0;
    for (int t : sl.ex->GetOutputs(sl.key)) {
      sl.outs.push_back(sl.ex->GetTensorView(sl.key, t));
      if (!sl.outs.back()) return Fail("no output view");
      ob += sl.outs.back()->GetBytes();
    }
    if (!sl.in) return Fail("no input view");
    sl.sink.resize(ob);
    slots.push_back(std::move(sl));
  }
  for (int j = 0; j < n_jobs; ++j) {
    const int m = (first_model + j) % n_models;
    Slot& sl = slots[m];
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(sl.in->GetData(), requests[m], sl.in->GetBytes());  // TryCopyInputTensors
    absl::Status s = sl.ex->ExecuteSubgraph(sl.key);                 // Engine::Invoke
    if (!s.ok()) return Fail(s);
    size_t off = 0;
    for (auto& v : sl.outs) {                                         // TryCopyOutputTensors
      std::memcpy(sl.sink.data() + off, v->GetData(), v->GetBytes());
      off += v->GetBytes();
    }
    if (latency_us)
      latency_us[j] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (model_of_job) model_of_job[j] = m;
  }
  return 0;
}

int bhx_executor_set_graph(bhx_executor* e, int enabled) {
  auto* h = e ? dynamic_cast<band::hip::HipModelExecutor*>(e->exec.get()) : nullptr;
  if (!h) return Fail("not a HIP executor");
  h->SetUseGraph(enabled != 0);
  return 0;
}

int bhx_executor_device(bhx_executor* e, int* ordinal) {
  auto* h = e ? dynamic_cast<band::hip::HipModelExecutor*>(e->exec.get()) : nullptr;
  if (!h || !ordinal) return Fail("not a HIP executor");
  *ordinal = h->ordinal();
  return 0;
}

int bhx_executor_coalescer(bhx_executor* e, int* members, int* lanes_ready) {
  auto* h = e ? dynamic_cast<band::hip::HipModelExecutor*>(e->exec.get()) : nullptr;
  if (!h || !members || !lanes_ready) return Fail("not a HIP executor");
  const band::hip::JobCoalescer* c = h->coalescer();
  *members = c ? c->members() : 0;
  *lanes_ready = c && c->lanes_ready() ? 1 : 0;
  return 0;
}

int bhx_coalescer_stats(long long* out, int reset) {
  if (!out) return Fail("bad arguments");
  const band::hip::JobCoalescer::Stats s = band::hip::JobCoalescer::Totals();
  out[0] = s.calls;
  out[1] = s.solo_passes;
  out[2] = s.group_passes;
  out[3] = s.group_jobs;
  out[4] = s.max_group;
  out[5] = s.bypass_calls;
  out[6] = s.max_bypass_inflight;
  if (reset) band::hip::JobCoalescer::ResetTotals();
  return 0;
}

int bhx_profile_subgraph(bhx_executor* e, int mid, int wid, uint64_t mask, int iters, bhx_op_timing* out, int cap,
                         int* n, double* floor_us) {
  auto* h = e ? dynamic_cast<band::hip::HipModelExecutor*>(e->exec.get()) : nullptr;
  if (!h) return Fail("not a HIP executor");
  std::vector<band::hip::OpTiming> t;
  auto s = h->ProfileSubgraph(Key(mid, wid, mask), iters, &t, floor_us);
  if (!s.ok()) return Fail(s);
  if (n) *n = static_cast<int>(t.size());
  for (int i = 0; i < cap && i < static_cast<int>(t.size()); ++i)
    out[i] = bhx_op_timing{t[i].op_index, t[i].kernel, t[i].ms, t[i].alg_bytes, t[i].alg_ops};
  return 0;
}

int bhx_prepare_job_batches(bhx_executor* e, bhx_model* m, int mid, int wid, uint64_t mask, int max_batch) {
  auto* b = e ? dynamic_cast<band::hip::IJobBatching*>(e->exec.get()) : nullptr;
  if (!b || !m) return Fail("executor without job batching");
  auto s = b->PrepareJobBatches(m->model.get(), Key(mid, wid, mask), max_batch);
  return s.ok() ? 0 : Fail(s);
}

int bhx_max_job_batch(bhx_executor* e, int mid, int wid, uint64_t mask, int* max_batch) {
  auto* b = e ? dynamic_cast<band::hip::IJobBatching*>(e->exec.get()) : nullptr;
  if (!max_batch) return Fail("null argument");
  *max_batch = b ? b->MaxJobBatch(Key(mid, wid, mask)) : 1;
  return 0;
}

int bhx_job_slot_view(bhx_executor* e, int mid, int wid, uint64_t mask, int t, int n, int slot,
                      bhx_tensor_info* info) {
  auto* b = e ? dynamic_cast<band::hip::IJobBatching*>(e->exec.get()) : nullptr;
  if (!b || !info) return Fail("executor without job batching");
  return FillInfo(b->GetJobSlotView(Key(mid, wid, mask), t, n, slot), info);
}

int bhx_execute_job_batch(bhx_executor* e, int mid, int wid, uint64_t mask, int n) {
  auto* b = e ? dynamic_cast<band::hip::IJobBatching*>(e->exec.get()) : nullptr;
  if (!b) return Fail("executor without job batching");
  auto s = b->ExecuteJobBatch(Key(mid, wid, mask), n);
  return s.ok() ? 0 : Fail(s);
}

int bhx_time_subgraph(bhx_executor* e, int mid, int wid, uint64_t mask, int iters, double* us) {
  auto* h = e ? dynamic_cast<band::hip::HipModelExecutor*>(e->exec.get()) : nullptr;
  if (!h) return Fail("not a HIP executor");
  auto s = h->TimeSubgraph(Key(mid, wid, mask), iters, us);
  if (!s.ok()) return Fail(s);
  return 0;
}

}  // extern "C"
