// Band C API over the native harness (band/c/c_api.cc restated; see
// include/band_c_api.h for the contract).
#include <pthread.h>
#include <set>
#include <unordered_map>
#include "band_c_api.h"

#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstring>
#include <deque>
#include <functional>
#include <random>
#include <mutex>
#include <thread>
#include <list>
#include <memory>
#include <string>
#include <vector>

#include "engine/engine.h"
#include "engine/logger.h"
#include "engine/planner.h"
#include "engine/time.h"

struct BandConfigBuilder {
  band::RuntimeConfig config;
  bool cfg_online = true;
  // the builder starts with no scheduler; Build() requires one
  // (band/config_builder.cc:34-40)
};

struct BandConfig {
  band::RuntimeConfig impl;
};

struct BandModel {
  BandModel() : impl(std::make_shared<band::Model>()) {}
  std::shared_ptr<band::Model> impl;
};

struct BandTensor {
  explicit BandTensor(band::Tensor* t) : impl(t) {}
  std::unique_ptr<band::Tensor> impl;
};

struct BandEngine {
  explicit BandEngine(std::unique_ptr<band::Engine> e) : impl(std::move(e)) {}
  std::list<std::shared_ptr<band::Model>> models;
  std::unique_ptr<band::Engine> impl;
  // the last DriveRequests call (BandxEngineGetDriverStats)
  double driver_stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

namespace {
using band::LogSeverity;

// only an internal error is an error for C callers (band/c/c_api.cc:33-47)
BandStatus ToBandStatus(const absl::Status& s) {
  return s.code() == absl::StatusCode::kInternal ? kBandErr : kBandOk;
}

band::Tensors ToVec(BandTensor** tensors, int n) {
  band::Tensors v;
  for (int i = 0; tensors && i < n; ++i) v.push_back(tensors[i] ? tensors[i]->impl.get() : nullptr);
  return v;
}

band::RequestOption ToOption(const BandRequestOption& o) {
  band::RequestOption r;
  r.target_worker = o.target_worker;
  r.require_callback = o.require_callback;
  r.slo_us = o.slo_us;
  r.slo_scale = o.slo_scale;
  return r;
}

// validity rules of band/config_builder.cc:12-80
absl::Status Validate(const band::RuntimeConfig& c) {
  const auto& p = c.profile_config;
  if (p.num_warmups <= 0) return absl::InvalidArgumentError("[ProfileConfigBuilder] num_warmups_ > 0");
  if (p.num_runs <= 0) return absl::InvalidArgumentError("[ProfileConfigBuilder] num_runs_ > 0");
  if (p.smoothing_factor < 0.f || p.smoothing_factor > 1.f)
    return absl::InvalidArgumentError("[ProfileConfigBuilder] smoothing_factor_ in [0, 1]");
  if (!p.online && p.profile_data_path.empty())
    return absl::InvalidArgumentError("[ProfileConfigBuilder] profile_data_path_ != \"\"");
  if (c.planner_config.schedule_window_size <= 0)
    return absl::InvalidArgumentError("[PlannerConfigBuilder] schedule_window_size_ > 0");
  if (c.planner_config.schedulers.empty())
    return absl::InvalidArgumentError("[PlannerConfigBuilder] schedulers_.size() > 0");
  const auto& w = c.worker_config;
  for (auto f : w.workers)
    if (static_cast<size_t>(f) >= band::EnumLength<band::DeviceFlag>())
      return absl::InvalidArgumentError("[WorkerConfigBuilder] invalid device");
  if (w.cpu_masks.size() != w.workers.size())
    return absl::InvalidArgumentError("[WorkerConfigBuilder] cpu_masks_.size() == workers_.size()");
  if (w.num_threads.size() != w.workers.size())
    return absl::InvalidArgumentError("[WorkerConfigBuilder] num_threads_.size() == workers_.size()");
  for (int t : w.num_threads)
    if (t < 0) return absl::InvalidArgumentError("[WorkerConfigBuilder] num_threads_[i] >= 0");
  if (w.max_job_batch < 1) return absl::InvalidArgumentError("max_job_batch >= 1");
  if (w.pass_target_us < 0) return absl::InvalidArgumentError("pass_target_us >= 0");
  if (w.availability_check_interval_ms <= 0)
    return absl::InvalidArgumentError("[WorkerConfigBuilder] availability_check_interval_ms_ > 0");
  if (c.subgraph_config.minimum_subgraph_size <= 0)
    return absl::InvalidArgumentError("[RuntimeConfigBuilder] minimum_subgraph_size_ > 0");
  return absl::OkStatus();
}
}  // namespace

extern "C" {

void BandSetLogSeverity(BandLogSeverity severity) {
  band::Logger::Get().SetVerbosity(static_cast<LogSeverity>(severity));
}

BandCallbackHandle BandSetLogReporter(void (*reporter)(BandLogSeverity, const char*)) {
  return band::Logger::Get().SetReporter(
      [reporter](LogSeverity s, const char* m) { reporter(static_cast<BandLogSeverity>(s), m); });
}

void BandUnsetLogReporter(BandCallbackHandle handle) {
  if (!band::Logger::Get().RemoveReporter(handle))
    BAND_LOG(LogSeverity::kWarning, "Failed to remove reporter with handle %d", handle);
}

BandConfigBuilder* BandConfigBuilderCreate(void) { return new BandConfigBuilder; }

void BandAddConfig(BandConfigBuilder* b, int field, int count, ...) {
  if (!b) {
    BAND_LOG(LogSeverity::kError, "BandConfigBuilder is null");
    return;
  }
  band::RuntimeConfig& c = b->config;
  va_list vl;
  va_start(vl, count);
  switch (field) {
    case BAND_PROFILE_ONLINE: c.profile_config.online = va_arg(vl, int) != 0; break;
    case BAND_PROFILE_NUM_WARMUPS: c.profile_config.num_warmups = va_arg(vl, int); break;
    case BAND_PROFILE_NUM_RUNS: c.profile_config.num_runs = va_arg(vl, int); break;
    case BAND_PROFILE_SMOOTHING_FACTOR: c.profile_config.smoothing_factor = static_cast<float>(va_arg(vl, double)); break;
    case BAND_PROFILE_DATA_PATH: c.profile_config.profile_data_path = va_arg(vl, const char*); break;
    case BAND_PLANNER_SCHEDULE_WINDOW_SIZE: c.planner_config.schedule_window_size = va_arg(vl, int); break;
    case BAND_PLANNER_SCHEDULERS: {
      std::vector<band::SchedulerType> s;
      for (int i = 0; i < count; ++i) s.push_back(static_cast<band::SchedulerType>(va_arg(vl, int)));
      if (!s.empty()) c.planner_config.schedulers = s;
    } break;
    case BAND_PLANNER_CPU_MASK: c.planner_config.cpu_mask = static_cast<band::CPUMaskFlag>(va_arg(vl, int)); break;
    case BAND_PLANNER_LOG_PATH: c.planner_config.log_path = va_arg(vl, const char*); break;
    case BAND_WORKER_WORKERS: {
      std::vector<band::DeviceFlag> w;
      for (int i = 0; i < count; ++i) w.push_back(static_cast<band::DeviceFlag>(va_arg(vl, int)));
      if (!w.empty()) c.worker_config.workers = w;
    } break;
    case BAND_WORKER_CPU_MASKS: {
      std::vector<band::CPUMaskFlag> m;
      for (int i = 0; i < count; ++i) m.push_back(static_cast<band::CPUMaskFlag>(va_arg(vl, int)));
      if (!m.empty()) c.worker_config.cpu_masks = m;
    } break;
    case BAND_WORKER_NUM_THREADS: {
      std::vector<int> t;
      for (int i = 0; i < count; ++i) t.push_back(va_arg(vl, int));
      if (!t.empty()) c.worker_config.num_threads = t;
    } break;
    case BAND_WORKER_ALLOW_WORKSTEAL: c.worker_config.allow_worksteal = va_arg(vl, int) != 0; break;
    case BAND_WORKER_AVAILABILITY_CHECK_INTERVAL_MS:
      c.worker_config.availability_check_interval_ms = va_arg(vl, int);
      break;
    case BAND_MINIMUM_SUBGRAPH_SIZE: c.subgraph_config.minimum_subgraph_size = va_arg(vl, int); break;
    case BAND_SUBGRAPH_PREPARATION_TYPE:
      c.subgraph_config.subgraph_preparation_type = static_cast<band::SubgraphPreparationType>(va_arg(vl, int));
      break;
    case BAND_CPU_MASK: c.cpu_mask = static_cast<band::CPUMaskFlag>(va_arg(vl, int)); break;
    case BAND_RESOURCE_MONITOR_DEVICE_PATH:
      (void)va_arg(vl, int);
      (void)va_arg(vl, const char*);
      break;  // no resource monitor on this platform
    case BAND_RESOURCE_MONITOR_INTERVAL_MS: (void)va_arg(vl, int); break;
    case BAND_RESOURCE_MONITOR_LOG_PATH: (void)va_arg(vl, const char*); break;
    case BANDX_WORKER_MAX_JOB_BATCH: c.worker_config.max_job_batch = va_arg(vl, int); break;
    case BANDX_WORKER_PASS_TARGET_US: c.worker_config.pass_target_us = va_arg(vl, int); break;
    case BANDX_PROFILE_SHARE_IDENTICAL: c.profile_config.share_identical_workers = va_arg(vl, int) != 0; break;
    default: BAND_LOG(LogSeverity::kWarning, "unknown config field %d", field);
  }
  va_end(vl);
}

void BandConfigBuilderDelete(BandConfigBuilder* b) { delete b; }

BandConfig* BandConfigCreate(BandConfigBuilder* b) {
  if (!b) return nullptr;
  absl::Status s = Validate(b->config);
  if (!s.ok()) {
    BAND_LOG(LogSeverity::kError, "invalid config: %s", s.message().c_str());
    return nullptr;
  }
  return new BandConfig{b->config};
}

void BandConfigDelete(BandConfig* config) { delete config; }

BandModel* BandModelCreate(void) { return new BandModel; }
void BandModelDelete(BandModel* model) { delete model; }

BandStatus BandModelAddFromBuffer(BandModel* model, BandBackendType backend_type, const void* data, size_t size) {
  if (!model) return kBandErr;
  return ToBandStatus(
      model->impl->FromBuffer(static_cast<band::BackendType>(backend_type), static_cast<const char*>(data), size));
}

BandStatus BandModelAddFromFile(BandModel* model, BandBackendType backend_type, const char* path) {
  if (!model || !path) return kBandErr;
  return ToBandStatus(model->impl->FromPath(static_cast<band::BackendType>(backend_type), path));
}

void BandTensorDelete(BandTensor* t) { delete t; }
BandDataType BandTensorGetType(BandTensor* t) {
  return t ? static_cast<BandDataType>(t->impl->GetType()) : kBandNumDataType;
}
void* BandTensorGetData(BandTensor* t) { return t ? t->impl->GetData() : nullptr; }
size_t BandTensorGetNumDims(BandTensor* t) { return t ? t->impl->GetNumDims() : 0; }
const int* BandTensorGetDims(BandTensor* t) { return t ? t->impl->GetDims() : nullptr; }
size_t BandTensorGetBytes(BandTensor* t) { return t ? t->impl->GetBytes() : 0; }
const char* BandTensorGetName(BandTensor* t) { return t ? t->impl->GetName() : nullptr; }
BandQuantizationType BandTensorGetQuantizationType(BandTensor* t) {
  return t ? static_cast<BandQuantizationType>(t->impl->GetQuantization().GetType()) : kBandNumQuantizationType;
}
void* BandTensorGetQuantizationParams(BandTensor* t) { return t ? t->impl->GetQuantization().GetParams() : nullptr; }

BandRequestOption BandRequestOptionGetDefault(void) { return {-1, true, -1, -1.f}; }

// band::RuntimeConfigBuilder::GetDefaultConfig (band/config_builder.cc:181-204),
// minus its Android paths
BandEngine* BandEngineCreateWithDefaultConfig(void) {
  BandConfig config;
  auto& c = config.impl;
  c.planner_config.schedulers = {band::SchedulerType::kHeterogeneousEarliestFinishTime};
  c.planner_config.schedule_window_size = 10;
  c.subgraph_config.minimum_subgraph_size = 7;
  c.subgraph_config.subgraph_preparation_type = band::SubgraphPreparationType::kMergeUnitSubgraph;
  c.worker_config.workers = {band::DeviceFlag::kCPU, band::DeviceFlag::kGPU, band::DeviceFlag::kDSP,
                             band::DeviceFlag::kNPU};
  c.worker_config.num_threads = {1, 1, 1, 1};
  c.worker_config.cpu_masks.assign(4, band::CPUMaskFlag::kBig);
  c.worker_config.allow_worksteal = true;
  return BandEngineCreate(&config);
}

BandEngine* BandEngineCreate(BandConfig* config) {
  if (!config) return nullptr;
  auto engine = band::Engine::Create(config->impl);
  return engine ? new BandEngine(std::move(engine)) : nullptr;
}

void BandEngineDelete(BandEngine* engine) { delete engine; }

BandStatus BandEngineRegisterModel(BandEngine* engine, BandModel* model) {
  if (!engine || !model) return kBandErr;
  absl::Status s = engine->impl->RegisterModel(model->impl.get());
  if (s.ok()) engine->models.push_back(model->impl);
  else BAND_LOG(LogSeverity::kError, "RegisterModel: %s", s.message().c_str());
  return ToBandStatus(s);
}

int BandEngineGetNumInputTensors(BandEngine* engine, BandModel* model) {
  if (!engine || !model) return -1;
  return static_cast<int>(engine->impl->GetInputTensorIndices(model->impl->GetId()).size());
}

int BandEngineGetNumOutputTensors(BandEngine* engine, BandModel* model) {
  if (!engine || !model) return -1;
  return static_cast<int>(engine->impl->GetOutputTensorIndices(model->impl->GetId()).size());
}

int BandEngineGetNumWorkers(BandEngine* engine) { return engine ? static_cast<int>(engine->impl->GetNumWorkers()) : -1; }

BandDeviceFlag BandEngineGetWorkerDevice(BandEngine* engine, int worker_id) {
  if (!engine || worker_id < 0 || worker_id >= static_cast<int>(engine->impl->GetNumWorkers())) return kBandNumDeviceFlag;
  return static_cast<BandDeviceFlag>(engine->impl->GetWorkerDevice(worker_id));
}

BandTensor* BandEngineCreateInputTensor(BandEngine* engine, BandModel* model, size_t index) {
  if (!engine || !model) return nullptr;
  auto idx = engine->impl->GetInputTensorIndices(model->impl->GetId());
  if (index >= idx.size()) return nullptr;
  band::Tensor* t = engine->impl->CreateTensor(model->impl->GetId(), idx[index]);
  return t ? new BandTensor(t) : nullptr;
}

BandTensor* BandEngineCreateOutputTensor(BandEngine* engine, BandModel* model, size_t index) {
  if (!engine || !model) return nullptr;
  auto idx = engine->impl->GetOutputTensorIndices(model->impl->GetId());
  if (index >= idx.size()) return nullptr;
  band::Tensor* t = engine->impl->CreateTensor(model->impl->GetId(), idx[index]);
  return t ? new BandTensor(t) : nullptr;
}

BandStatus BandEngineRequestSync(BandEngine* engine, BandModel* model, BandTensor** inputs, BandTensor** outputs) {
  return BandEngineRequestSyncOptions(engine, model, BandRequestOptionGetDefault(), inputs, outputs);
}

BandRequestHandle BandEngineRequestAsync(BandEngine* engine, BandModel* model, BandTensor** inputs) {
  return BandEngineRequestAsyncOptions(engine, model, BandRequestOptionGetDefault(), inputs);
}

BandStatus BandEngineRequestSyncOptions(BandEngine* engine, BandModel* model, BandRequestOption options,
                                        BandTensor** inputs, BandTensor** outputs) {
  if (!engine || !model) return kBandErr;
  return ToBandStatus(engine->impl->RequestSync(model->impl->GetId(), ToOption(options),
                                                ToVec(inputs, BandEngineGetNumInputTensors(engine, model)),
                                                ToVec(outputs, BandEngineGetNumOutputTensors(engine, model))));
}

BandRequestHandle BandEngineRequestAsyncOptions(BandEngine* engine, BandModel* model, BandRequestOption options,
                                                BandTensor** inputs) {
  if (!engine || !model) return -1;
  auto id = engine->impl->RequestAsync(model->impl->GetId(), ToOption(options),
                                       ToVec(inputs, BandEngineGetNumInputTensors(engine, model)));
  if (!id.ok()) {
    BAND_LOG(LogSeverity::kError, "RequestAsync: %s", id.status().message().c_str());
    return -1;
  }
  return id.value();
}

BandStatus BandEngineWait(BandEngine* engine, BandRequestHandle handle, BandTensor** outputs, size_t num_outputs) {
  if (!engine) return kBandErr;
  return ToBandStatus(engine->impl->Wait(handle, ToVec(outputs, static_cast<int>(num_outputs))));
}

BandCallbackHandle BandEngineSetOnEndRequest(BandEngine* engine, void (*cb)(void*, BandRequestHandle, BandStatus),
                                             void* user_data) {
  if (!engine || !cb) return -1;
  return engine->impl->SetOnEndRequest(
      [cb, user_data](int job_id, absl::Status s) { cb(user_data, job_id, ToBandStatus(s)); });
}

BandStatus BandEngineUnsetOnEndRequest(BandEngine* engine, BandCallbackHandle handle) {
  if (!engine) return kBandErr;
  return ToBandStatus(engine->impl->UnsetOnEndRequest(handle));
}

BandStatus BandxEngineGetJobRecord(BandEngine* engine, BandRequestHandle handle, BandxJobRecord* r) {
  if (!engine || !r) return kBandErr;
  band::Job j = engine->impl->GetFinishedJob(handle);
  if (j.job_id == -1) return kBandErr;
  r->job_id = j.job_id;
  r->model_id = j.model_id;
  r->worker_id = j.subgraph_key.GetWorkerId();
  r->status = static_cast<int>(j.status);
  r->enqueue_time_us = j.enqueue_time;
  r->invoke_time_us = j.invoke_time;
  r->end_time_us = j.end_time;
  r->expected_latency_us = j.expected_latency;
  r->slo_us = j.slo_us;
  r->unit_indices = j.subgraph_key.GetUnitIndices().to_ullong();
  return kBandOk;
}

int BandxModelGetId(BandModel* model) { return model ? model->impl->GetId() : -1; }

size_t BandxEngineGetProfileJson(BandEngine* engine, char* buf, size_t cap) {
  if (!engine) return 0;
  const std::string s = engine->impl->ProfileToJson();
  if (buf && cap) {
    const size_t n = std::min(cap - 1, s.size());
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return s.size();
}

BandStatus BandxEngineDumpProfile(BandEngine* engine) {
  return engine ? ToBandStatus(engine->impl->DumpProfile()) : kBandErr;
}

int BandxEngineGetSubgraphs(BandEngine* engine, BandModel* model, int* worker_ids, uint64_t* masks, int cap) {
  if (!engine || !model) return -1;
  auto keys = engine->impl->GetSubgraphKeys(model->impl->GetId());
  for (int i = 0; i < static_cast<int>(keys.size()) && i < cap; ++i) {
    if (worker_ids) worker_ids[i] = keys[i].GetWorkerId();
    if (masks) masks[i] = keys[i].GetUnitIndices().to_ullong();
  }
  return static_cast<int>(keys.size());
}

int64_t BandxEngineGetExpectedLatency(BandEngine* engine, BandModel* model, int worker_id, uint64_t unit_mask) {
  if (!engine || !model) return -1;
  std::set<int> units;
  for (int i = 0; i < 64; ++i)
    if (unit_mask >> i & 1) units.insert(i);
  return engine->impl->GetExpected(band::SubgraphKey(model->impl->GetId(), worker_id, units));
}

namespace {
// request driver shared by the closed-loop and Poisson entry points:
// `next_arrival(j)` returns the time (us since start) job j may be submitted
// (0 = as soon as the in-flight bound allows) and its model index
//
// Latency: closed loop, end - enqueue of the job record; open loop (Poisson),
// end - the job's SCHEDULED arrival, so time a request waited to be submitted
// (in-flight bound, ring back-pressure) counts as the queueing it is rather
// than vanishing from the percentiles (no coordinated omission).
// Outputs are read in COMPLETION order: an end-of-request callback queues
// each finished request and reader threads copy its outputs out, so one slow
// request does not hold the finished ones behind it (read in submission
// order, a request of a slow batched pass kept every later one counted as in
// flight and starved the closed loop).  Per model, a request is submitted
// only while it is fewer than ring - submitters submissions ahead of that
// model's oldest unread request, so no result is overwritten in the output
// ring before it is read (the engine may hand concurrent submitters their
// ring handles in a different order, by at most the submitter count).
BandStatus DriveRequests(BandEngine* engine, BandModel** models, BandTensor** inputs, int n_models, int n_jobs,
                         int max_inflight, bool open_loop,
                         const std::function<std::pair<int64_t, int>(int, int)>& next_arrival, double* latency_us,
                         int* worker_ids, int* model_index, double* wall_s, int burst_hint = 1) {
  if (!engine || !models || n_models <= 0 || n_jobs < 0 || max_inflight <= 0) return kBandErr;
  band::Engine& e = *engine->impl;
  // per model: one input tensor (copied into the request ring at submit)
  std::vector<std::vector<std::unique_ptr<band::Tensor>>> own_in(n_models);
  std::vector<band::Tensors> in_ptrs(n_models);
  for (int m = 0; m < n_models; ++m) {
    const band::ModelId id = models[m]->impl->GetId();
    const auto in_idx = e.GetInputTensorIndices(id);
    if (inputs && inputs[m] && in_idx.size() == 1) {
      in_ptrs[m].push_back(inputs[m]->impl.get());
    } else {
      for (int t : in_idx) {
        own_in[m].emplace_back(e.CreateTensor(id, t));
        if (!own_in[m].back()) return kBandErr;
        std::memset(own_in[m].back()->GetData(), 0, own_in[m].back()->GetBytes());
        in_ptrs[m].push_back(own_in[m].back().get());
      }
    }
  }
  // Submitters (BANDX_DRIVER_LANES, default 1) copy requests into the rings
  // (150 KB per 224x224 job); readers (BANDX_DRIVER_READERS, default 6) copy
  // results out (DeepLab's are 1 MB), each into output tensors of its own.
  int lanes = 1;
  if (const char* lv = std::getenv("BANDX_DRIVER_LANES")) lanes = std::max(1, std::atoi(lv));
  // a shard of the models per lane up to one model per shard (below); more
  // lanes than models share a shard: its runs are dealt to them in turn
  // (one engine over several GPUs needs several submitters per model)
  lanes = std::max(1, std::min({lanes, n_jobs > 0 ? n_jobs : 1, max_inflight}));
  const int n_shards = std::min(lanes, std::max(1, n_models));
  // submitter lanes of a model's shard: each can hold a run's slots reserved
  // but not yet allocated in the ring
  const int lanes_per_shard = (lanes + n_shards - 1) / n_shards;
  // requests of one model submitted per RequestAsync call (closed loop:
  // the job -> model order is run-major, `burst` jobs per model in turn)
  int burst = burst_hint > 0 ? burst_hint : 1;
  if (const char* bv = std::getenv("BANDX_DRIVER_BURST")) burst = std::max(1, std::atoi(bv));
  burst = std::max(1, std::min(burst, max_inflight / std::max(1, lanes)));
  for (int m = 0; m < n_models; ++m)
    burst = std::max(1, std::min(burst, e.RequestRingSize(models[m]->impl->GetId()) /
                                            (2 * std::max(n_shards, lanes_per_shard + 1))));
  int readers = 6;
  if (const char* rv = std::getenv("BANDX_DRIVER_READERS")) readers = std::max(1, std::atoi(rv));
  readers = std::max(1, std::min(readers, n_jobs > 0 ? n_jobs : 1));
  readers = std::max(readers, n_shards);  // every shard has a reader
  std::vector<std::vector<std::vector<std::unique_ptr<band::Tensor>>>> reader_outs(readers);
  std::vector<std::vector<band::Tensors>> reader_out_ptrs(readers);
  for (int r = 0; r < readers; ++r) {
    reader_outs[r].resize(n_models);
    reader_out_ptrs[r].resize(n_models);
    for (int m = 0; m < n_models; ++m) {
      const band::ModelId id = models[m]->impl->GetId();
      for (int t : e.GetOutputTensorIndices(id)) {
        reader_outs[r][m].emplace_back(e.CreateTensor(id, t));
        if (!reader_outs[r][m].back()) return kBandErr;
        reader_out_ptrs[r][m].push_back(reader_outs[r][m].back().get());
      }
    }
  }
  struct Pending {
    int index, model;
    int64_t arrival;  // open loop: scheduled arrival (NowMicros clock)
    long seq;         // submission number within its model
  };
  // The driver's state is sharded by model: submitter lane l owns the models
  // of shard l (and readers r = l, l + lanes, ...), with its own lock and
  // condition variables, so lanes never contend with each other; with one
  // lane (the default) it is a single shard.  A request's finished-job record
  // arrives with the group end-of-request callback (Engine::SetOnEndRequests),
  // so no request depends on the planner's 1000-record window.
  struct Shard {
    std::mutex mu;
    // readers wait on cv_read (a finished request, or the end), submitters on
    // cv_sub (a retired request): each event wakes only the side it concerns
    std::condition_variable cv_read, cv_sub;
    std::unordered_map<band::JobId, Pending> pending;  // submitted, not yet read
    std::deque<std::pair<band::JobId, band::Job>> done;  // finished, with their records
    std::unordered_map<band::JobId, band::Job> early;  // finished before the submitter recorded it
    int inflight = 0, taken = 0, n_jobs = 0, max_inflight = 1, readers = 0;
    // stats (under mu): time integrals of the requests inside the engine
    // (submitted, end-of-request not yet seen) and of the finished ones
    // waiting for a reader; submitter wait / call and reader busy / idle time
    int in_engine = 0;
    double int_engine = 0, int_done = 0, submit_wait = 0, submit_call = 0, read_busy = 0, read_idle = 0;
    int64_t last_tick = band::time::NowMicros();
    void tick() {  // under mu, before in_engine or done changes
      const int64_t now = band::time::NowMicros();
      int_engine += double(in_engine) * double(now - last_tick);
      int_done += double(done.size()) * double(now - last_tick);
      last_tick = now;
    }
  };
  std::vector<std::unique_ptr<Shard>> shards;
  for (int i = 0; i < n_shards; ++i) shards.emplace_back(new Shard());
  // a model's shard follows its engine id (a model listed twice shares one)
  std::unordered_map<band::ModelId, int> shard_of_id;
  std::vector<int> shard_of(n_models);
  for (int m = 0; m < n_models; ++m) {
    const band::ModelId id = models[m]->impl->GetId();
    auto it = shard_of_id.emplace(id, m % n_shards).first;
    shard_of[m] = it->second;
  }
  std::vector<int> models_in(n_shards, 0);
  for (int m = 0; m < n_models; ++m) ++models_in[shard_of[m]];
  for (int i = 0; i < n_shards; ++i)
    shards[i]->max_inflight = std::max(1, (int)((long)max_inflight * std::max(1, models_in[i]) / n_models));
  for (int r = 0; r < readers; ++r) ++shards[r % n_shards]->readers;
  std::vector<int> unread(n_models, 0), ring(n_models, 0);  // under the model's shard lock
  for (int m = 0; m < n_models; ++m) ring[m] = std::max(1, e.RequestRingSize(models[m]->impl->GetId()));
  std::vector<long> next_seq(n_models, 0);
  std::vector<std::set<long>> unread_seq(n_models);
  std::atomic<bool> failed{false};
  // arrivals are drawn in job order (the open-loop schedule is one sequence)
  std::vector<std::pair<int64_t, int>> arrivals(n_jobs);
  for (int j = 0; j < n_jobs; ++j) {
    arrivals[j] = next_arrival(j, burst);
    ++shards[shard_of[arrivals[j].second]]->n_jobs;
  }
  // one call per group of finished requests (a batched pass ends up to its
  // batch at once): one lock and one wake-up per side for the group
  const band::CallbackId cb = e.SetOnEndRequests([&](const std::vector<const band::Job*>& jobs) {
    size_t i = 0;
    while (i < jobs.size()) {
      auto sit = shard_of_id.find(jobs[i]->model_id);
      if (sit == shard_of_id.end()) {  // not a driver request
        ++i;
        continue;
      }
      Shard& sh = *shards[sit->second];
      std::lock_guard<std::mutex> lk(sh.mu);
      sh.tick();
      int to_read = 0;
      for (; i < jobs.size(); ++i) {
        auto nit = shard_of_id.find(jobs[i]->model_id);
        if (nit == shard_of_id.end() || nit->second != sit->second) break;
        const band::Job* rec = jobs[i];
        --sh.in_engine;
        if (sh.pending.count(rec->job_id)) {
          sh.done.emplace_back(rec->job_id, *rec);
          ++to_read;
        } else {
          sh.early.emplace(rec->job_id, *rec);
        }
      }
      if (to_read == 0) continue;
      if (to_read == 1) sh.cv_read.notify_one();
      else sh.cv_read.notify_all();
    }
  });
  auto retire = [&](Shard& sh, const Pending& item, bool ok) {  // under sh.mu
    if (!ok) failed = true;
    --sh.inflight;
    --unread[item.model];
    unread_seq[item.model].erase(item.seq);
  };
  const int64_t t0 = band::time::NowMicros();
  std::vector<std::thread> threads;
  for (int r = 0; r < readers; ++r) {
    threads.emplace_back([&, r] {
      pthread_setname_np(pthread_self(), "bandx-reader");
      Shard& sh = *shards[r % n_shards];
      while (true) {
        const int64_t w0 = band::time::NowMicros();
        std::unique_lock<std::mutex> lk(sh.mu);
        sh.cv_read.wait(lk, [&] { return !sh.done.empty() || sh.taken >= sh.n_jobs; });
        const int64_t w1 = band::time::NowMicros();
        sh.read_idle += double(w1 - w0);
        if (sh.done.empty()) break;
        sh.tick();
        // a fair share of what is ready (at most 8): fewer lock round trips
        // when a batched pass finishes many requests at once
        const size_t k = std::min<size_t>(8, (sh.done.size() + sh.readers - 1) / sh.readers);
        std::vector<std::pair<band::Job, Pending>> mine;
        mine.reserve(k);
        for (size_t q = 0; q < k; ++q) {
          const band::JobId id = sh.done.front().first;
          auto pit = sh.pending.find(id);
          mine.emplace_back(std::move(sh.done.front().second), pit->second);
          mine.back().first.job_id = mine.back().first.job_id == id ? id : -1;
          sh.pending.erase(pit);
          sh.done.pop_front();
          if (++sh.taken >= sh.n_jobs) sh.cv_read.notify_all();  // the other readers may leave
        }
        if (!sh.done.empty()) sh.cv_read.notify_one();
        lk.unlock();
        std::vector<bool> oks(mine.size());
        for (size_t q = 0; q < mine.size(); ++q) {
          const band::Job& j = mine[q].first;
          const Pending& item = mine[q].second;
          absl::Status st = j.job_id >= 0 ? e.GetOutputTensorsOf(j, reader_out_ptrs[r][item.model])
                                          : absl::InternalError("no finished record");
          oks[q] = st.ok() && j.status == band::JobStatus::kSuccess;
          if (!oks[q])
            BAND_LOG(band::LogSeverity::kError, "request driver: job (model %d) failed: %s; record %d, status %s",
                     item.model, std::string(st.message()).c_str(), j.job_id,
                     band::ToString<band::JobStatus>(j.status));
          if (latency_us)
            latency_us[item.index] = static_cast<double>(j.end_time - (open_loop ? item.arrival : j.enqueue_time));
          if (worker_ids) worker_ids[item.index] = j.subgraph_key.GetWorkerId();
          if (model_index) model_index[item.index] = item.model;
        }
        lk.lock();
        sh.read_busy += double(band::time::NowMicros() - w1);
        for (size_t q = 0; q < mine.size(); ++q) retire(sh, mine[q].second, oks[q]);
        sh.cv_sub.notify_all();
      }
    });
  }
  // Runs: consecutive jobs of one model that are due are submitted as ONE
  // vector RequestAsync (band/engine.cc:455-529, the overload Band's own
  // benchmark tool uses with batch_size >= 2), up to `burst` requests: one
  // ring allocation, one planner enqueue and one wake-up per run instead of
  // per request.  Lane l takes the runs of its shard's models, in order.
  // lane l serves shard l % n_shards; a shard's runs go to its lanes in turn
  std::vector<std::vector<std::pair<int, int>>> runs(lanes);  // (first job, length) per lane
  {
    std::vector<int> dealt(n_shards, 0);
    for (int j = 0; j < n_jobs;) {
      int k = j + 1;
      while (k < n_jobs && k - j < burst && arrivals[k].second == arrivals[j].second &&
             arrivals[k].first == arrivals[j].first)
        ++k;
      const int sh = shard_of[arrivals[j].second];
      const int in_shard = (lanes - sh + n_shards - 1) / n_shards;  // lanes sh, sh + n_shards, ...
      runs[sh + n_shards * (dealt[sh]++ % in_shard)].emplace_back(j, k - j);
      j = k;
    }
  }
  for (int l = 0; l < lanes; ++l) {
    threads.emplace_back([&, l] {
      pthread_setname_np(pthread_self(), "bandx-submit");
      Shard& sh = *shards[l % n_shards];
      std::vector<band::ModelId> ids;
      std::vector<band::RequestOption> opts;
      std::vector<band::Tensors> ins;
      std::vector<long> seqs;
      for (const auto& run : runs[l]) {
        const int j0 = run.first, r = run.second;
        const auto& arrival = arrivals[j0];
        const int64_t now = band::time::NowMicros() - t0;
        if (arrival.first > now) band::time::SleepForMicros(arrival.first - now);
        const int m = arrival.second;
        // a run is < ring - (lanes of the shard) x burst submissions ahead of
        // the model's oldest unread request: the runs other lanes of the
        // shard have reserved but not yet allocated (their ring handles may
        // come before this run's) still leave this run's ring slots free
        const long span = std::max(1, ring[m] - lanes_per_shard * burst);
        const int64_t w0 = band::time::NowMicros();
        seqs.clear();
        {
          std::unique_lock<std::mutex> lk(sh.mu);
          sh.cv_sub.wait(lk, [&] {
            return sh.inflight + r <= std::max(sh.max_inflight, r) && unread[m] + r <= ring[m] &&
                   (unread_seq[m].empty() || next_seq[m] + r - 1 - *unread_seq[m].begin() < span);
          });
          sh.inflight += r;
          unread[m] += r;
          sh.tick();
          sh.in_engine += r;
          for (int k = 0; k < r; ++k) {
            seqs.push_back(next_seq[m]++);
            unread_seq[m].insert(seqs.back());
          }
        }
        const int64_t w1 = band::time::NowMicros();
        ids.assign(r, models[m]->impl->GetId());
        opts.assign(r, band::RequestOption::GetDefaultOption());
        ins.assign(r, in_ptrs[m]);
        auto handles = e.RequestAsync(ids, opts, ins);
        const int64_t w2 = band::time::NowMicros();
        std::lock_guard<std::mutex> lk(sh.mu);
        sh.submit_wait += double(w1 - w0);
        sh.submit_call += double(w2 - w1);
        int to_read = 0;
        for (int k = 0; k < r; ++k) {
          const Pending item{j0 + k, m, t0 + arrivals[j0 + k].first, seqs[k]};
          if (!handles.ok()) {
            if (k == 0)
              BAND_LOG(band::LogSeverity::kError, "request driver: submit of jobs %d..%d failed: %s", j0, j0 + r - 1,
                       std::string(handles.status().message()).c_str());
            if (++sh.taken >= sh.n_jobs) sh.cv_read.notify_all();
            sh.tick();
            --sh.in_engine;
            retire(sh, item, false);
            sh.cv_sub.notify_all();
            continue;
          }
          const band::JobId id = handles.value()[k];
          sh.pending[id] = item;
          auto ea = sh.early.find(id);
          if (ea != sh.early.end()) {
            sh.tick();
            sh.done.emplace_back(id, std::move(ea->second));
            sh.early.erase(ea);
            ++to_read;
          }
        }
        if (to_read) sh.cv_read.notify_all();
      }
    });
  }
  for (auto& t : threads) t.join();
  (void)e.UnsetOnEndRequest(cb);
  const double wall_us = double(band::time::NowMicros() - t0);
  double int_engine = 0, int_done = 0, submit_wait = 0, submit_call = 0, read_busy = 0, read_idle = 0;
  for (auto& shp : shards) {
    Shard& sh = *shp;
    sh.tick();
    int_engine += sh.int_engine;
    int_done += sh.int_done;
    submit_wait += sh.submit_wait;
    submit_call += sh.submit_call;
    read_busy += sh.read_busy;
    read_idle += sh.read_idle;
  }
  double* st = engine->driver_stats;
  st[0] = wall_us;
  st[1] = wall_us > 0 ? int_engine / wall_us : 0;
  st[2] = wall_us > 0 ? int_done / wall_us : 0;
  st[3] = submit_wait;
  st[4] = submit_call;
  st[5] = read_busy;
  st[6] = read_idle;
  st[7] = double(readers) + 1000.0 * lanes;
  if (wall_s) *wall_s = wall_us * 1e-6;
  return failed.load() ? kBandErr : kBandOk;
}
}  // namespace

BandStatus BandxEngineRunClosedLoopEx(BandEngine* engine, BandModel** models, BandTensor** inputs, int n_models,
                                      int n_jobs, int max_inflight, double* latency_us, int* worker_ids,
                                      int* model_index, double* wall_s) {
  // closed loop: runs of `burst` requests per model, models in turn (the
  // burst DriveRequests settles on, so model_index is the one to key on)
  return DriveRequests(
      engine, models, inputs, n_models, n_jobs, max_inflight, false,
      [&](int j, int burst) { return std::make_pair(int64_t(0), (j / burst) % std::max(n_models, 1)); },
      latency_us, worker_ids, model_index, wall_s, 4);
}

BandStatus BandxEngineRunClosedLoop(BandEngine* engine, BandModel** models, BandTensor** inputs, int n_models,
                                    int n_jobs, int max_inflight, double* latency_us, int* worker_ids,
                                    double* wall_s) {
  return BandxEngineRunClosedLoopEx(engine, models, inputs, n_models, n_jobs, max_inflight, latency_us, worker_ids,
                                    nullptr, wall_s);
}

BandStatus BandxEngineRunPoisson(BandEngine* engine, BandModel** models, BandTensor** inputs, int n_models,
                                 int n_jobs, double rate_per_s, uint64_t seed, int max_inflight, double* latency_us,
                                 int* worker_ids, int* model_index, double* wall_s) {
  if (!(rate_per_s > 0)) return kBandErr;
  std::mt19937_64 rng(seed);
  std::exponential_distribution<double> gap(rate_per_s);
  std::uniform_int_distribution<int> pick(0, std::max(n_models, 1) - 1);
  double t = 0;
  return DriveRequests(
      engine, models, inputs, n_models, n_jobs, max_inflight, true,
      [&](int, int) {
        t += gap(rng) * 1e6;
        return std::make_pair(static_cast<int64_t>(t), pick(rng));
      },
      latency_us, worker_ids, model_index, wall_s, 1);
}

int64_t BandxEngineGetWorkerJobCount(BandEngine* engine, int worker_id) {
  if (!engine || worker_id < 0 || worker_id >= static_cast<int>(engine->impl->GetNumWorkers())) return -1;
  const band::Worker* w = engine->impl->GetWorker(worker_id);
  return w ? w->GetJobsRun() : -1;
}

int BandxEngineGetDriverStats(BandEngine* engine, double out[8]) {
  if (!engine || !out) return -1;
  for (int i = 0; i < 8; ++i) out[i] = engine->driver_stats[i];
  return 0;
}

int BandxEngineGetRequestPhaseTimes(BandEngine* engine, int64_t out[4]) {
  if (!engine || !out) return -1;
  engine->impl->GetRequestPhaseTimes(out);
  return 0;
}

int BandxEngineGetWorkerPhaseTimes(BandEngine* engine, int worker_id, int64_t out[4]) {
  if (!engine || !out || worker_id < 0 || worker_id >= static_cast<int>(engine->impl->GetNumWorkers())) return -1;
  const band::Worker* w = engine->impl->GetWorker(worker_id);
  if (!w) return -1;
  w->GetPhaseTimes(out);
  return 0;
}

void BandxEngineWaitAll(BandEngine* engine) {
  if (engine) engine->impl->WaitAll();
}

BandStatus BandxEngineRequestsAsync(BandEngine* engine, BandModel** models, int n, BandTensor*** inputs,
                                    BandRequestHandle* handles) {
  if (!engine || !models || n <= 0 || !inputs || !handles) return kBandErr;
  std::vector<band::ModelId> ids;
  std::vector<band::RequestOption> opts;
  std::vector<band::Tensors> ins;
  for (int i = 0; i < n; ++i) {
    if (!models[i]) return kBandErr;
    ids.push_back(models[i]->impl->GetId());
    opts.push_back(band::RequestOption::GetDefaultOption());
    ins.push_back(ToVec(inputs[i], BandEngineGetNumInputTensors(engine, models[i])));
  }
  auto r = engine->impl->RequestAsync(ids, opts, ins);
  if (!r.ok()) {
    BAND_LOG(LogSeverity::kError, "RequestsAsync: %s", r.status().message().c_str());
    return kBandErr;
  }
  for (int i = 0; i < n; ++i) handles[i] = r.value()[i];
  return kBandOk;
}

}  // extern "C"
