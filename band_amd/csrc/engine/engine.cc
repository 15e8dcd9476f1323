#include "engine/engine.h"

#include <cstdlib>

#include "backend/hip/job_batching.h"

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstring>

#include "engine/logger.h"
#include <limits>

#include "band/backend_factory.h"
#include "band/interface/tensor_view.h"
#include "engine/time.h"

// Optional page-locked ring memory from the HIP backend
// (include/band_hip_backend.h); weak, so an engine linked without that
// backend keeps heap rings.
extern "C" void* bhx_ring_host_alloc(size_t bytes) __attribute__((weak));
extern "C" void bhx_ring_host_free(void* p) __attribute__((weak));

namespace band {

std::unique_ptr<Engine> Engine::Create(const RuntimeConfig& config, absl::Status* status) {
  std::unique_ptr<Engine> engine(new Engine());
  absl::Status s = engine->Init(config);
  if (status) *status = s;
  if (!s.ok()) {
    BAND_LOG(LogSeverity::kError, "engine creation failed: %s", s.message().c_str());
    return nullptr;
  }
  return engine;
}

Engine::~Engine() {
  for (auto& w : workers_) w->End();
  planner_.reset();
  model_executors_.clear();
  workers_.clear();
}

// band/engine.cc:635-716
absl::Status Engine::Init(const RuntimeConfig& config) {
  planner_.reset(new Planner(*this));
  absl::Status s = planner_->Init(config.planner_config);
  if (!s.ok()) return s;
  subgraph_config_ = config.subgraph_config;
  latency_estimator_.reset(new LatencyEstimator(this));
  s = latency_estimator_->Init(config.profile_config);
  if (!s.ok()) return s;

  std::set<DeviceFlag> valid;
  for (BackendType b : BackendFactory::GetAvailableBackends()) {
    std::unique_ptr<interface::IBackendUtil> util(BackendFactory::GetBackendUtil(b));
    if (!util) continue;
    for (DeviceFlag f : util->GetAvailableDevices()) valid.insert(f);
  }
  const bool global = planner_->GetWorkerType() == static_cast<int>(WorkerType::kGlobalQueue);
  max_job_batch_ = std::max(1, config.worker_config.max_job_batch);
  pass_target_us_ = std::max(0, config.worker_config.pass_target_us);
  rotate_ties_ = config.profile_config.share_identical_workers;
  for (DeviceFlag flag : config.worker_config.workers) {
    if (!valid.count(flag)) {
      BAND_LOG(LogSeverity::kWarning, "%s worker is not created (device unavailable)", ToString(flag));
      continue;
    }
    const WorkerId id = static_cast<WorkerId>(workers_.size());
    std::unique_ptr<Worker> w;
    if (global) w.reset(new GlobalQueueWorker(this, id, flag));
    else w.reset(new DeviceQueueWorker(this, id, flag));
    if (!w->Init(config.worker_config).ok())
      return absl::InternalError(std::string("Worker::Init() failed for worker : ") + ToString(flag));
    w->Start();
    workers_.push_back(std::move(w));
    workers_waiting_[id] = 0;
  }
  return absl::OkStatus();
}

// band/engine.cc:51-289
absl::Status Engine::RegisterModel(Model* model) {
  if (!model) return absl::InternalError("Model is empty.");
  if (model->GetSupportedBackends().empty()) return absl::InternalError("No supported backends.");
  const ModelId model_id = model->GetId();

  for (BackendType backend : model->GetSupportedBackends()) {
    interface::IModel* backend_model = model->GetBackendModel(backend);
    ModelAnalyzer analyzer(*this, planner_->NeedFallbackSubgraphs(), subgraph_config_, backend_model, backend);
    auto result = analyzer.CreateSubgraphs();
    if (!result.ok()) {
      UnregisterModel(model);
      return result.status();
    }
    const ModelSpec& spec = result.value().first;
    const std::vector<SubgraphDef>& defs = result.value().second;

    bool added = false;
    for (WorkerId w = 0; w < static_cast<WorkerId>(workers_.size()); ++w) {
      if (spec.unavailable_devices.count(GetWorkerDevice(w))) continue;
      const Worker* worker = workers_[w].get();
      std::unique_ptr<interface::IModelExecutor> exec(BackendFactory::CreateModelExecutor(
          backend, model_id, w, GetWorkerDevice(w), worker->GetWorkerThreadAffinity(), worker->GetNumThreads()));
      if (!exec) continue;
      model_executors_[{model_id, w}] = std::move(exec);
      added = true;
    }
    if (!added) {
      UnregisterModel(model);
      return absl::InternalError("Failed to create model executor on all worker types");
    }
    model_specs_.erase(model_id);
    model_specs_.emplace(model_id, spec);

    for (const SubgraphDef& def : defs) {
      const SubgraphKey key(model_id, def.worker_id, def.unit_subgraph_indices);
      auto it = model_executors_.find({model_id, def.worker_id});
      if (it == model_executors_.end())
        return absl::InternalError("Subgraph logic created a subgraph for worker " + std::to_string(def.worker_id) +
                                   " that does not supports model " + std::to_string(model_id));
      interface::IModelExecutor* exec = it->second.get();
      absl::Status ps = exec->PrepareSubgraph(backend_model, def.op_indices, def.unit_subgraph_indices);
      if (!ps.ok()) {
        BAND_LOG(LogSeverity::kError, "PrepareSubgraph failed on worker %d (%s): %s", def.worker_id,
                     def.ToString().c_str(), ps.message().c_str());
        continue;
      }
      if (!exec->HasSubgraph(key))
        return absl::InternalError("A subgraph for worker " + std::to_string(def.worker_id) + " that does not exists");
      // the executor's I/O must match the spec (band/engine.cc:153-173)
      const std::set<int> inputs = spec.GetPureInputTensors(def.op_indices);
      const std::set<int> outputs = spec.GetOutputTensors(def.op_indices);
      const auto& ein = exec->GetInputs(key);
      const auto& eout = exec->GetOutputs(key);
      if (ein.size() != inputs.size() || !std::equal(ein.begin(), ein.end(), inputs.begin()))
        return absl::InternalError("Input format is not correct for worker " + std::to_string(def.worker_id));
      const std::set<int> eout_set(eout.begin(), eout.end());
      if (!std::includes(outputs.begin(), outputs.end(), eout_set.begin(), eout_set.end()))
        return absl::InternalError("Output format is not correct for worker " + std::to_string(def.worker_id));
      // job batching for whole-model subgraphs on GPU workers (config extension)
      if (max_job_batch_ > 1 &&
          (GetWorkerDevice(def.worker_id) == DeviceFlag::kGPU || GetWorkerDevice(def.worker_id) == DeviceFlag::kCPU) &&
          static_cast<int>(def.op_indices.size()) == spec.num_ops) {
        if (auto* jb = dynamic_cast<hip::IJobBatching*>(exec)) {
          absl::Status bs = jb->PrepareJobBatches(backend_model, key, max_job_batch_);
          if (!bs.ok())
            BAND_LOG(LogSeverity::kWarning, "model %d runs unbatched on worker %d: %s", model_id, def.worker_id,
                     bs.message().c_str());
          else if (pass_target_us_ > 0) {
            bool have;
            {
              std::lock_guard<std::mutex> lock(pass_mu_);
              have = pass_cap_.count(model_id) != 0;
            }
            if (!have) {
              const int cap = PassCap(jb, key);
              std::lock_guard<std::mutex> lock(pass_mu_);
              pass_cap_[model_id] = cap;
            }
          }
        }
      }
      unit_subgraphs_to_subgraph_keys_[model_id][*def.unit_subgraph_indices.begin()]
                                      [*def.unit_subgraph_indices.rbegin()]
                                          .push_back(key);
    }

    // tensors crossing workers must agree in type and shape (band/engine.cc:187-233)
    for (const SubgraphDef& l : defs)
      for (const SubgraphDef& r : defs) {
        if (&l == &r || l.worker_id == r.worker_id) continue;
        const SubgraphKey lk(model_id, l.worker_id, l.unit_subgraph_indices);
        const SubgraphKey rk(model_id, r.worker_id, r.unit_subgraph_indices);
        auto* le = GetModelExecutor(lk);
        auto* re = GetModelExecutor(rk);
        if (!le || !re || !le->HasSubgraph(lk) || !re->HasSubgraph(rk)) continue;
        const std::set<int> louts(le->GetOutputs(lk).begin(), le->GetOutputs(lk).end());
        for (int t : re->GetInputs(rk)) {
          if (!louts.count(t)) continue;
          auto lv = le->GetTensorView(lk, t);
          auto rv = re->GetTensorView(rk, t);
          if (!lv || !rv || !(*lv == *rv))
            return absl::InternalError(lk.ToString() + " and " + rk.ToString() + " disagree on tensor " +
                                       std::to_string(t));
        }
      }

    // request ring buffers, shaped from the views of the first worker
    // (preferring a CPU worker) that hosts the whole-model I/O
    WorkerId host = -1;
    for (WorkerId w = 0; w < static_cast<WorkerId>(workers_.size()) && host < 0; ++w)
      if (GetWorkerDevice(w) == DeviceFlag::kCPU && GetLargestSubgraphKey(model_id, w).IsValid()) host = w;
    std::vector<std::shared_ptr<interface::ITensor>> in_views, out_views;
    for (WorkerId w = (host >= 0 ? host : 0); w < static_cast<WorkerId>(workers_.size()); ++w) {
      const SubgraphKey key = GetLargestSubgraphKey(model_id, w);
      interface::IModelExecutor* exec = GetModelExecutor(key);
      if (!key.IsValid() || !exec) continue;
      in_views.clear();
      out_views.clear();
      bool ok = true;
      for (int t : spec.input_tensors) {
        auto v = exec->GetTensorView(key, t);
        ok &= v != nullptr;
        in_views.push_back(v);
      }
      for (int t : spec.output_tensors) {
        auto v = exec->GetTensorView(key, t);
        ok &= v != nullptr;
        out_views.push_back(v);
      }
      if (ok) break;
      in_views.clear();
      out_views.clear();
      if (host >= 0) break;
    }
    if (in_views.size() != spec.input_tensors.size() || out_views.size() != spec.output_tensors.size())
      return absl::InternalError("no worker exposes the model's input/output tensors");
    // request slots per model: the reference's 128, or BANDX_REQUEST_RING_SLOTS
    // (a slot is held from RequestAsync until the job finishes, and slots
    // are taken in order, so one slow job stalls new requests of its model
    // once 128 younger ones are outstanding - deep closed loops over
    // several workers want more)
    int slots = 128;
    if (const char* rs = std::getenv("BANDX_REQUEST_RING_SLOTS")) slots = std::max(1, std::atoi(rs));
    const RingHostAllocator ring_alloc = RingAllocatorFor(model_id, spec.num_ops);
    model_input_buffer_[model_id].reset(new TensorRingBuffer(
        in_views, std::vector<int>(spec.input_tensors.begin(), spec.input_tensors.end()), slots, ring_alloc));
    model_output_buffer_[model_id].reset(new TensorRingBuffer(
        out_views, std::vector<int>(spec.output_tensors.begin(), spec.output_tensors.end()), slots, ring_alloc));

    absl::Status ls = latency_estimator_->ProfileModel(model_id);
    if (!ls.ok()) return ls;
  }
  return absl::OkStatus();
}

// Page-locked rings pay only where a GPU worker runs the whole model (its
// one-job and batched passes DMA the ring slots directly); every other model
// keeps heap rings, so CPU-only engines pin nothing and initialise no GPU.
RingHostAllocator Engine::RingAllocatorFor(ModelId model_id, int num_ops) const {
  RingHostAllocator a;
  if (!bhx_ring_host_alloc || !bhx_ring_host_free) return a;
  for (WorkerId w = 0; w < static_cast<WorkerId>(workers_.size()); ++w) {
    if (GetWorkerDevice(w) != DeviceFlag::kGPU) continue;
    const SubgraphKey key = GetLargestSubgraphKey(model_id, w);
    const interface::IModelExecutor* exec = key.IsValid() ? GetModelExecutor(key) : nullptr;
    if (exec && static_cast<int>(exec->GetNumNodes(key)) == num_ops) {
      a.alloc = bhx_ring_host_alloc;
      a.free = bhx_ring_host_free;
      break;
    }
  }
  return a;
}

absl::Status Engine::UnregisterModel(Model* model) {
  if (!model) return absl::InternalError("Failed to unregister null model.");
  const ModelId id = model->GetId();
  for (auto it = model_executors_.begin(); it != model_executors_.end();)
    it = it->first.first == id ? model_executors_.erase(it) : std::next(it);
  model_specs_.erase(id);
  unit_subgraphs_to_subgraph_keys_.erase(id);
  model_input_buffer_.erase(id);
  model_output_buffer_.erase(id);
  cache_.clear();
  return absl::OkStatus();
}

Tensor* Engine::CreateTensor(ModelId model_id, int tensor_index) {
  for (WorkerId w = 0; w < static_cast<WorkerId>(workers_.size()); ++w) {
    const SubgraphKey key = GetLargestSubgraphKey(model_id, w);
    auto* exec = GetModelExecutor(key);
    if (!exec) continue;
    auto view = exec->GetTensorView(key, tensor_index);
    if (view) return new Tensor(view.get());
  }
  return nullptr;
}

std::vector<int> Engine::GetInputTensorIndices(ModelId model_id) const {
  const ModelSpec* s = GetModelSpec(model_id);
  return s ? std::vector<int>(s->input_tensors.begin(), s->input_tensors.end()) : std::vector<int>();
}

std::vector<int> Engine::GetOutputTensorIndices(ModelId model_id) const {
  const ModelSpec* s = GetModelSpec(model_id);
  return s ? std::vector<int>(s->output_tensors.begin(), s->output_tensors.end()) : std::vector<int>();
}

absl::Status Engine::RequestSync(ModelId model_id, RequestOption options, Tensors inputs, Tensors outputs) {
  auto id = RequestAsync(model_id, options, inputs);
  if (!id.ok()) return id.status();
  return Wait(id.value(), outputs);
}

absl::Status Engine::RequestSync(std::vector<ModelId> model_ids, std::vector<RequestOption> options,
                                 std::vector<Tensors> inputs, std::vector<Tensors> outputs) {
  auto ids = RequestAsync(model_ids, options, inputs);
  if (!ids.ok()) return ids.status();
  return Wait(ids.value(), outputs);
}

absl::StatusOr<JobId> Engine::RequestAsync(ModelId model_id, RequestOption options, Tensors inputs) {
  std::vector<Tensors> in;
  if (!inputs.empty()) in.push_back(inputs);
  auto ids = RequestAsync(std::vector<ModelId>{model_id}, std::vector<RequestOption>{options}, in);
  if (!ids.ok()) return ids.status();
  return ids.value()[0];
}

// band/engine.cc:455-529.  Every request is validated before any ring slot
// is taken, so a refused call leaves no slot held.
absl::StatusOr<std::vector<JobId>> Engine::RequestAsync(std::vector<ModelId> model_ids,
                                                        std::vector<RequestOption> options,
                                                        std::vector<Tensors> inputs) {
  if (model_ids.size() != options.size())
    return absl::InternalError("# Model requests (" + std::to_string(model_ids.size()) + ") != # Worker ids (" +
                               std::to_string(options.size()) + ")");
  std::vector<Job> jobs;
  jobs.reserve(model_ids.size());
  for (size_t i = 0; i < model_ids.size(); ++i) {
    Job job(model_ids[i]);
    job.require_callback = options[i].require_callback;
    int64_t slo = options[i].slo_us;
    if (options[i].slo_scale != -1) {
      if (options[i].slo_scale <= 0)
        return absl::InternalError("Specified slo_scale is invalid (" + std::to_string(options[i].slo_scale) +
                                   " <= 0)");
      slo = static_cast<int64_t>(GetWorst(model_ids[i]) * options[i].slo_scale);
    }
    if (options[i].slo_us != -1) slo = options[i].slo_us;
    job.slo_us = slo;
    if (options[i].target_worker != -1) {
      if (!GetWorker(options[i].target_worker))
        return absl::InternalError("Request assigned to invalid worker id (" +
                                   std::to_string(options[i].target_worker) + ")");
      job.target_worker_id = options[i].target_worker;
    }
    if (i < inputs.size() && (!model_input_buffer_.count(model_ids[i]) || !model_output_buffer_.count(model_ids[i])))
      return absl::InternalError("Input copy failure for model " + std::to_string(model_ids[i]));
    // every input is checked before any run is enqueued, so a refused call
    // has started no job
    if (i < inputs.size() && !model_input_buffer_.at(model_ids[i])->CheckTensors(inputs[i]).ok())
      return absl::InternalError("Input copy failure for model " + std::to_string(model_ids[i]));
    jobs.push_back(std::move(job));
  }
  // Ring slots are taken per run of consecutive same-model requests, all of
  // a run's slots in one step (AllocBlockingN), and the run is enqueued at
  // once: a call never holds slots of jobs it has not enqueued, so neither a
  // call larger than the ring nor two concurrent calls sharing a model can
  // wait on each other forever.  A run larger than the ring is refused
  // before anything is taken.
  const size_t n_in = std::min(jobs.size(), inputs.size());
  for (size_t i = 0; i < n_in;) {
    size_t j = i;
    while (j < n_in && model_ids[j] == model_ids[i]) ++j;
    const int ring = model_input_buffer_.at(model_ids[i])->size();
    if (static_cast<int>(j - i) > ring)
      return absl::InternalError("RequestAsync: " + std::to_string(j - i) + " consecutive requests of model " +
                                 std::to_string(model_ids[i]) + " exceed its request ring (" + std::to_string(ring) +
                                 " slots)");
    i = j;
  }
  std::vector<JobId> ids;
  ids.reserve(jobs.size());
  for (size_t i = 0; i < jobs.size();) {
    size_t j = i;
    int64_t t_copy_start = time::NowMicros();
    if (i < n_in) {
      while (j < n_in && model_ids[j] == model_ids[i]) ++j;
      TensorRingBuffer* in_ring = model_input_buffer_.at(model_ids[i]).get();
      // blocks while the model's ring has fewer than j - i free slots
      const int64_t t_alloc = time::NowMicros();
      const int first = in_ring->AllocBlockingN(static_cast<int>(j - i));
      const int64_t t_copy = time::NowMicros();
      req_alloc_us_ += t_copy - t_alloc;
      t_copy_start = t_copy;
      for (size_t k = i; k < j; ++k) {
        const int handle = first + static_cast<int>(k - i);
        if (!in_ring->PutTensorsToHandle(inputs[k], handle).ok()) {
          for (size_t r = i; r < j; ++r) in_ring->Release(first + static_cast<int>(r - i));
          return absl::InternalError("Input copy failure for model " + std::to_string(model_ids[k]));
        }
        jobs[k].input_handle = handle;
        jobs[k].output_handle = model_output_buffer_.at(model_ids[k])->Claim(handle);
      }
    } else {
      j = jobs.size();  // requests without inputs (no ring slot)
    }
    const int64_t t_enq = time::NowMicros();
    std::vector<Job> run(std::make_move_iterator(jobs.begin() + i), std::make_move_iterator(jobs.begin() + j));
    for (JobId id : EnqueueBatch(std::move(run))) ids.push_back(id);
    const int64_t t_end = time::NowMicros();
    req_copy_us_ += t_enq - t_copy_start;
    req_enqueue_us_ += t_end - t_enq;
    req_jobs_ += static_cast<int64_t>(j - i);
    i = j;
  }
  return ids;
}

void Engine::GetRequestPhaseTimes(int64_t out[4]) const {
  out[0] = req_jobs_.load();
  out[1] = req_alloc_us_.load();
  out[2] = req_copy_us_.load();
  out[3] = req_enqueue_us_.load();
}

void Engine::ReleaseRequest(const Job& job) {
  if (job.input_handle < 0) return;
  auto it = model_input_buffer_.find(job.model_id);
  if (it != model_input_buffer_.end()) it->second->Release(job.input_handle);
}

void Engine::HoldOutput(const Job& job) {
  if (job.output_handle < 0) return;
  auto it = model_output_buffer_.find(job.model_id);
  if (it != model_output_buffer_.end()) it->second->Hold(job.output_handle);
}

void Engine::UnholdOutput(const Job& job) {
  if (job.output_handle < 0) return;
  auto it = model_output_buffer_.find(job.model_id);
  if (it != model_output_buffer_.end()) it->second->Unhold(job.output_handle);
}

int Engine::RequestRingSize(ModelId model_id) const {
  auto it = model_input_buffer_.find(model_id);
  return it == model_input_buffer_.end() ? 0 : it->second->size();
}

absl::Status Engine::Wait(JobId job_id, Tensors outputs) {
  std::vector<Tensors> out;
  if (!outputs.empty()) out.push_back(outputs);
  return Wait(std::vector<JobId>{job_id}, out);
}

absl::Status Engine::Wait(std::vector<JobId> job_ids, std::vector<Tensors> outputs) {
  planner_->Wait(job_ids);
  for (size_t i = 0; i < outputs.size() && i < job_ids.size(); ++i) {
    absl::Status s = GetOutputTensors(job_ids[i], outputs[i]);
    if (!s.ok()) return s;
  }
  return absl::OkStatus();
}

void Engine::WaitAll() { planner_->WaitAll(); }

// band/engine.cc:574-617
absl::Status Engine::GetOutputTensors(JobId job_id, Tensors outputs) {
  if (outputs.empty() || job_id == -1)
    return absl::InternalError("Invalid job id / num outputs to copy: (" + std::to_string(job_id) + ", " +
                               std::to_string(outputs.size()) + ")");
  return GetOutputTensorsOf(planner_->GetFinishedJob(job_id), outputs);
}

absl::Status Engine::GetOutputTensorsOf(const Job& job, Tensors outputs) {
  if (outputs.empty()) return absl::InternalError("Invalid num outputs to copy: 0");
  if (job.job_id == -1) return absl::InternalError("Invalid job id / not finished or invalidated.");
  if (job.output_handle == -1)
    return absl::InternalError("Invalid output handle : " + std::to_string(job.output_handle));
  if (job.status == JobStatus::kSLOViolation) return absl::DeadlineExceededError("SLO violation");
  if (job.status != JobStatus::kSuccess)
    return absl::InternalError(std::string("Job failed with status : ") + ToString(job.status));
  auto it = model_output_buffer_.find(job.model_id);
  if (it == model_output_buffer_.end()) return absl::InternalError("Invalid model id : " + std::to_string(job.model_id));
  return it->second->GetTensorsFromHandle(outputs, job.output_handle);
}

CallbackId Engine::SetOnEndRequest(std::function<void(int, absl::Status)> cb) {
  return planner_->SetOnEndRequest(std::move(cb));
}

absl::Status Engine::UnsetOnEndRequest(CallbackId id) { return planner_->UnsetOnEndRequest(id); }

void Engine::UpdateWorkersWaiting() const {
  for (WorkerId w = 0; w < static_cast<WorkerId>(workers_.size()); ++w)
    workers_waiting_[w] = workers_[w]->GetWaitingTime();
}

std::set<WorkerId> Engine::GetIdleWorkers() const {
  std::set<WorkerId> idle;
  for (const auto& kv : workers_waiting_)
    if (kv.second == 0) idle.insert(kv.first);
  return idle;
}

std::set<WorkerId> Engine::GetIdleWorkersNow() {
  std::set<WorkerId> idle;
  for (WorkerId w = 0; w < static_cast<WorkerId>(workers_.size()); ++w)
    if (workers_[w]->IsIdleNow()) idle.insert(idle.end(), w);
  return idle;
}

DeviceFlag Engine::GetWorkerDevice(WorkerId id) const {
  return id >= 0 && id < static_cast<WorkerId>(workers_.size()) ? workers_[id]->GetDeviceFlag()
                                                                 : DeviceFlag::kNPU;  // never matches a worker
}

Worker* Engine::GetWorker(WorkerId id) {
  return id >= 0 && id < static_cast<WorkerId>(workers_.size()) ? workers_[id].get() : nullptr;
}

const Worker* Engine::GetWorker(WorkerId id) const {
  return id >= 0 && id < static_cast<WorkerId>(workers_.size()) ? workers_[id].get() : nullptr;
}

WorkerId Engine::GetDeviceWorkerId(DeviceFlag flag) const {
  for (WorkerId w = 0; w < static_cast<WorkerId>(workers_.size()); ++w)
    if (workers_[w]->GetDeviceFlag() == flag) return w;
  return -1;
}

SubgraphKey Engine::GetLargestSubgraphKey(ModelId model_id, WorkerId worker_id) const {
  auto it = model_executors_.find({model_id, worker_id});
  return it == model_executors_.end() ? SubgraphKey() : it->second->GetLargestSubgraphKey();
}

const ModelSpec* Engine::GetModelSpec(ModelId model_id) const {
  auto it = model_specs_.find(model_id);
  return it == model_specs_.end() ? nullptr : &it->second;
}

// the planner's model -> worker map; unmapped models go to worker 0 as in
// the reference, whose map is never filled (band/planner.h:118)
WorkerId Engine::GetModelWorker(ModelId model_id) const {
  auto& m = planner_->GetModelWorkerMap();
  auto it = m.find(model_id);
  return it == m.end() ? 0 : it->second;
}

bool Engine::IsBegin(const SubgraphKey& key) const {
  const ModelSpec* spec = GetModelSpec(key.GetModelId());
  if (!spec) return false;
  for (int u : key.GetUnitIndicesSet())
    if (static_cast<size_t>(u) >= spec->GetNumUnitSubgraphs() || spec->GetUnitSubgraphDependency(u).any())
      return false;
  return true;
}

bool Engine::IsEnd(const SubgraphKey& key) const {
  const ModelSpec* spec = GetModelSpec(key.GetModelId());
  return spec && (key.GetUnitIndices().none() ||
                  (spec->GetNumUnitSubgraphs() > 0 && key.GetUnitIndices().test(spec->GetNumUnitSubgraphs() - 1)));
}

bool Engine::HasSubgraph(const SubgraphKey& key) const {
  auto it = model_executors_.find({key.GetModelId(), key.GetWorkerId()});
  return it != model_executors_.end() && it->second->HasSubgraph(key);
}

void Engine::ForEachSubgraph(std::function<void(const SubgraphKey&)> visitor) const {
  for (auto& kv : model_executors_) kv.second->ForEachSubgraph(visitor);
}

std::vector<SubgraphKey> Engine::GetSubgraphKeys(ModelId model_id) const {
  std::vector<SubgraphKey> keys;
  for (auto& kv : model_executors_)
    if (kv.first.first == model_id) kv.second->ForEachSubgraph([&](const SubgraphKey& k) { keys.push_back(k); });
  return keys;
}

absl::Status Engine::Invoke(const SubgraphKey& key) {
  auto it = model_executors_.find({key.GetModelId(), key.GetWorkerId()});
  if (it == model_executors_.end()) return absl::InternalError("Failed to find a subgraph key");
  return it->second->ExecuteSubgraph(key);
}

interface::IModelExecutor* Engine::GetModelExecutor(const SubgraphKey& key) {
  auto it = model_executors_.find({key.GetModelId(), key.GetWorkerId()});
  return it == model_executors_.end() ? nullptr : it->second.get();
}

const interface::IModelExecutor* Engine::GetModelExecutor(const SubgraphKey& key) const {
  auto it = model_executors_.find({key.GetModelId(), key.GetWorkerId()});
  return it == model_executors_.end() ? nullptr : it->second.get();
}

std::pair<std::vector<SubgraphKey>, int64_t> Engine::GetSubgraphWithShortestLatency(
    const Job& job, const WorkerWaitingTime& waiting) const {
  if (subgraph_config_.subgraph_preparation_type == SubgraphPreparationType::kFallbackPerWorker) {
    auto best = GetShortestLatency(job.model_id, job.resolved_unit_subgraphs, 0, waiting);
    return {{best.first}, best.second};
  }
  const ModelSpec* spec = GetModelSpec(job.model_id);
  if (!spec || spec->GetNumUnitSubgraphs() == 0) return {{}, std::numeric_limits<int32_t>::max()};
  int start = 0;
  for (size_t i = 0; i < spec->GetNumUnitSubgraphs(); ++i)
    if (job.resolved_unit_subgraphs.test(i)) start = static_cast<int>(i) + 1;
  return GetShortestLatencyWithUnitSubgraph(job.model_id, start, waiting);
}

// memo[j] = best plan covering units [start, j]: the cheapest last subgraph
// (i..j) started after memo[i-1] finished (band/engine.cc:966-1058)
std::pair<std::vector<SubgraphKey>, int64_t> Engine::GetShortestLatencyWithUnitSubgraph(
    ModelId model_id, int start, const WorkerWaitingTime& waiting) const {
  const ModelSpec* spec = GetModelSpec(model_id);
  const int n = static_cast<int>(spec->GetNumUnitSubgraphs());
  std::vector<std::pair<std::vector<SubgraphKey>, int64_t>> memo(
      n, {std::vector<SubgraphKey>(), std::numeric_limits<int>::max()});
  if (start >= n) return {{}, std::numeric_limits<int32_t>::max()};
  auto model_it = unit_subgraphs_to_subgraph_keys_.find(model_id);
  for (int j = start; j < n; ++j) {
    std::pair<std::vector<SubgraphKey>, int64_t> local{{}, -1};
    for (int i = j; i >= start; --i) {
      if (model_it == unit_subgraphs_to_subgraph_keys_.end()) continue;
      auto first_it = model_it->second.find(i);
      if (first_it == model_it->second.end()) continue;
      auto last_it = first_it->second.find(j);
      if (last_it == first_it->second.end()) continue;
      const int64_t begin = i > start ? memo[i - 1].second : 0;
      auto cand = GetShortestSubgraphKey(last_it->second, begin, waiting);
      if (local.second == -1 || cand.second < local.second) {
        local.first = i > start ? memo[i - 1].first : std::vector<SubgraphKey>();
        local.first.push_back(cand.first);
        local.second = cand.second;
      }
    }
    memo[j] = local;
  }
  return memo[n - 1];
}

// fallback-per-worker recursion with a start-time-independent cache
// (band/engine.cc:856-964)
std::pair<SubgraphKey, int64_t> Engine::GetShortestLatency(ModelId model_id, BitMask resolved, int64_t start_time,
                                                           const WorkerWaitingTime& waiting) const {
  const std::pair<ModelId, unsigned long long> cache_key{model_id, resolved.to_ullong()};
  bool stale = true;  // every worker frees up before start_time
  for (const auto& kv : waiting)
    if (kv.second > start_time) stale = false;
  if (stale) {
    auto it = cache_.find(cache_key);
    if (it != cache_.end()) return {it->second.first, it->second.second + start_time};
  }
  std::map<unsigned long long, std::vector<SubgraphKey>> by_units;
  for (const SubgraphKey& k : GetSubgraphCandidates(model_id, resolved))
    by_units[k.GetUnitIndices().to_ullong()].push_back(k);
  std::pair<SubgraphKey, int64_t> best{SubgraphKey(), std::numeric_limits<int64_t>::max()};
  for (const auto& group : by_units) {
    auto first = GetShortestSubgraphKey(group.second, start_time, waiting);
    std::pair<SubgraphKey, int64_t> finish =
        IsEnd(first.first) ? first
                           : GetShortestLatency(model_id, resolved | first.first.GetUnitIndices(), first.second, waiting);
    if (finish.second < best.second) best = {first.first, finish.second};
  }
  if (stale && best.first.IsValid()) cache_[cache_key] = {best.first, best.second - start_time};
  return best;
}

// subgraphs not yet run whose unit dependencies are resolved
// (band/engine.cc:1107-1156)
std::vector<SubgraphKey> Engine::GetSubgraphCandidates(ModelId model_id, BitMask resolved) const {
  std::vector<SubgraphKey> out;
  const ModelSpec* spec = GetModelSpec(model_id);
  for (const auto& kv : model_executors_) {
    if (kv.first.first != model_id) continue;
    kv.second->ForEachSubgraph([&](const SubgraphKey& key) {
      if (resolved.none()) {
        if (IsBegin(key)) out.push_back(key);
        return;
      }
      if ((key.GetUnitIndices() & resolved).any() || !spec) return;
      const BitMask deps = spec->GetUnitSubgraphDependency(key.GetUnitIndices());
      if (deps == (deps & resolved)) out.push_back(key);
    });
  }
  return out;
}

// the key finishing first: expected latency after max(worker wait, start)
// (band/engine.cc:1158-1178); ties go to the later key
std::pair<SubgraphKey, int64_t> Engine::GetShortestSubgraphKey(const std::vector<SubgraphKey>& keys,
                                                               int64_t start_time,
                                                               const WorkerWaitingTime& waiting) const {
  int64_t best = std::numeric_limits<int64_t>::max();
  SubgraphKey best_key;
  // The reference keeps the LAST of equal totals (band/engine.cc:1158-1178).
  // With shared estimates (share_identical_workers) identical idle workers
  // tie exactly, so that rule sends every job to the highest worker id that
  // is idle; ties then go round-robin instead (the scan starts one key later
  // on every call and keeps the first minimum).
  const size_t n = keys.size();
  const size_t r0 = rotate_ties_ && n ? tie_rotation_.fetch_add(1, std::memory_order_relaxed) % n : 0;
  for (size_t i = 0; i < n; ++i) {
    const SubgraphKey& k = keys[(r0 + i) % n];
    auto it = waiting.find(k.GetWorkerId());
    const int64_t wait = it == waiting.end() ? 0 : it->second;
    const int64_t total = GetExpected(k) + std::max(wait, start_time);
    if (rotate_ties_ ? best > total : best >= total) {
      best = total;
      best_key = k;
    }
  }
  return {best_key, best};
}

// previous subgraphs' outputs first, then the request's ring slot
// (band/engine.cc:1247-1319)
absl::Status Engine::TryCopyInputTensors(const Job& job) {
  if (job.input_handle < 0) return absl::OkStatus();
  const SubgraphKey& key = job.subgraph_key;
  interface::IModelExecutor* exec = GetModelExecutor(key);
  if (!exec) return absl::InternalError("no executor for " + key.ToString());
  return CopyInputs(job, [&](int t) { return exec->GetTensorView(key, t); });
}

absl::Status Engine::CopyInputs(const Job& job, const ViewFn& view) {
  const SubgraphKey& key = job.subgraph_key;
  interface::IModelExecutor* exec = GetModelExecutor(key);
  std::set<int> unresolved(exec->GetInputs(key).begin(), exec->GetInputs(key).end());
  if (job.intermediates) {
    for (auto it = unresolved.begin(); it != unresolved.end();) {
      auto hit = job.intermediates->find(*it);
      if (hit == job.intermediates->end()) {
        ++it;
        continue;
      }
      auto dst = view(*it);
      if (!dst || dst->GetBytes() != hit->second.size())
        return absl::InternalError("intermediate tensor " + std::to_string(*it) + " does not fit its view");
      std::memcpy(dst->GetData(), hit->second.data(), hit->second.size());
      it = unresolved.erase(it);
    }
  }
  for (const SubgraphKey& prev : job.previous_subgraph_keys) {
    interface::IModelExecutor* pexec = GetModelExecutor(prev);
    if (!pexec) continue;
    for (int t : pexec->GetOutputs(prev)) {
      if (!unresolved.count(t)) continue;
      auto src = pexec->GetTensorView(prev, t);
      auto dst = view(t);
      if (!src || !dst || !dst->CopyDataFrom(src.get()).ok())
        return absl::InternalError("Tensor data copy failure for tensor " + std::to_string(t));
      unresolved.erase(t);
    }
  }
  auto ring = model_input_buffer_.find(job.model_id);
  if (ring == model_input_buffer_.end())
    return absl::InternalError("Failed to find input tensor ring buffer for model " + std::to_string(job.model_id));
  for (auto it = unresolved.begin(); it != unresolved.end();) {
    if (!ring->second->IsTensorIndexValid(*it)) {
      ++it;
      continue;
    }
    auto dst = view(*it);
    if (!dst || !ring->second->GetTensorFromHandle(dst.get(), *it, job.input_handle).ok())
      return absl::InternalError("Failed to copy input tensor " + std::to_string(*it) + " for model " +
                                 std::to_string(job.model_id));
    it = unresolved.erase(it);
  }
  if (!unresolved.empty()) return absl::InternalError("Some tensors fail to be resolved.");
  return absl::OkStatus();
}

// captures what this subgraph produced for the rest of the job, on the
// worker thread right after ExecuteSubgraph, before that worker can run
// another request (see Job::intermediates)
absl::Status Engine::SaveIntermediates(Job& job) {
  if (job.following_jobs.empty()) return absl::OkStatus();
  const SubgraphKey& key = job.subgraph_key;
  interface::IModelExecutor* exec = GetModelExecutor(key);
  if (!exec) return absl::InternalError("no executor for " + key.ToString());
  auto snap = std::make_shared<std::map<int, std::vector<char>>>();
  if (job.intermediates) *snap = *job.intermediates;
  for (int t : exec->GetOutputs(key)) {
    auto v = exec->GetTensorView(key, t);
    if (!v) return absl::InternalError("no view of output tensor " + std::to_string(t));
    const char* d = v->GetData();
    (*snap)[t].assign(d, d + v->GetBytes());
  }
  for (Job& f : job.following_jobs) f.intermediates = snap;
  return absl::OkStatus();
}

absl::Status Engine::TryCopyOutputTensors(const Job& job) {
  if (job.output_handle < 0) return absl::OkStatus();
  const SubgraphKey& key = job.subgraph_key;
  interface::IModelExecutor* exec = GetModelExecutor(key);
  if (!exec) return absl::InternalError("no executor for " + key.ToString());
  return CopyOutputs(job, [&](int t) { return exec->GetTensorView(key, t); });
}

absl::Status Engine::CopyOutputs(const Job& job, const ViewFn& view) {
  const SubgraphKey& key = job.subgraph_key;
  interface::IModelExecutor* exec = GetModelExecutor(key);
  auto ring = model_output_buffer_.find(job.model_id);
  if (ring == model_output_buffer_.end())
    return absl::InternalError("Failed to find output tensor ring buffer for model " + std::to_string(job.model_id));
  // the slot becomes this request's (after any callback still reading the
  // previous request's outputs there has returned)
  if (!ring->second->AcquireForWrite(job.output_handle))
    return absl::DeadlineExceededError("output slot of request " + std::to_string(job.output_handle) + " of model " +
                                       std::to_string(job.model_id) + " is held by an end-request callback");
  for (int t : exec->GetOutputs(key)) {
    if (!ring->second->IsTensorIndexValid(t)) continue;
    auto src = view(t);
    if (!src || !ring->second->PutTensorToHandle(src.get(), t, job.output_handle).ok())
      return absl::InternalError("Failed to copy output tensor " + std::to_string(t) + " for model " +
                                 std::to_string(job.model_id));
  }
  return absl::OkStatus();
}

int Engine::MaxJobBatch(const SubgraphKey& key) const {
  if (max_job_batch_ <= 1) return 1;
  auto* jb = dynamic_cast<const hip::IJobBatching*>(GetModelExecutor(key));
  const int n = jb ? jb->MaxJobBatch(key) : 1;
  if (pass_target_us_ <= 0) return n;
  std::lock_guard<std::mutex> lock(pass_mu_);
  auto cap = pass_cap_.find(key.GetModelId());
  return cap == pass_cap_.end() ? n : std::min(n, cap->second);
}

// The pass-size policy (WorkerConfig::pass_target_us): the model's largest
// batch variant is timed once (best of 3 passes after one warm-up, inputs
// whatever the slots hold), the pass time taken as linear in the jobs, and
// the batch capped where it reaches the target.  A model whose full pass
// is 2x the target then runs half-size passes: its jobs no longer wait
// behind the longest pass of the mix, which sets the job-latency tail.
int Engine::PassCap(hip::IJobBatching* jb, const SubgraphKey& key) {
  const int b = jb->MaxJobBatch(key);
  if (b <= 1 || !jb->ExecuteJobBatch(key, b).ok()) return b;
  int64_t best = INT64_MAX;
  for (int i = 0; i < 3; ++i) {
    const int64_t t0 = time::NowMicros();
    if (!jb->ExecuteJobBatch(key, b).ok()) return b;
    best = std::min(best, time::NowMicros() - t0);
  }
  const int cap = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(b, pass_target_us_ * b / std::max<int64_t>(1, best))));
  BAND_LOG(LogSeverity::kInfo, "model %d: %d-job pass %lld us, pass target %d us -> at most %d jobs per pass",
           key.GetModelId(), b, static_cast<long long>(best), pass_target_us_, cap);
  return cap;
}

absl::Status Engine::TryCopyInputTensorsToSlot(const Job& job, int n, int slot) {
  if (job.input_handle < 0) return absl::OkStatus();
  const SubgraphKey& key = job.subgraph_key;
  auto* jb = dynamic_cast<hip::IJobBatching*>(GetModelExecutor(key));
  if (!jb) return absl::InternalError("no batching executor for " + key.ToString());
  return CopyInputs(job, [&](int t) { return jb->GetJobSlotView(key, t, n, slot); });
}

absl::Status Engine::InvokeJobBatch(const SubgraphKey& key, int n) {
  auto* jb = dynamic_cast<hip::IJobBatching*>(GetModelExecutor(key));
  if (!jb) return absl::InternalError("no batching executor for " + key.ToString());
  return jb->ExecuteJobBatch(key, n);
}

absl::Status Engine::InvokeJobBatchDirect(const SubgraphKey& key, const std::vector<Job*>& jobs) {
  // max_job_batch 1 is Band's own contract: the worker copies through the
  // executor's views around ExecuteSubgraph (band/worker.cc:222-323) and
  // the engine calls nothing beyond band/interface
  if (max_job_batch_ <= 1) return absl::UnimplementedError("job batching off");
  auto* jb = dynamic_cast<hip::IJobBatching*>(GetModelExecutor(key));
  interface::IModelExecutor* exec = GetModelExecutor(key);
  const int n = static_cast<int>(jobs.size());
  if (!jb || !exec || n < 1) return absl::UnimplementedError("direct job batch I/O");
  const ModelId model = jobs[0]->model_id;
  auto in_it = model_input_buffer_.find(model);
  auto out_it = model_output_buffer_.find(model);
  if (in_it == model_input_buffer_.end() || out_it == model_output_buffer_.end())
    return absl::UnimplementedError("no request rings");
  const std::vector<int>& ins = exec->GetInputs(key);
  const std::vector<int>& outs = exec->GetOutputs(key);
  std::vector<const interface::ITensor*> in(ins.size() * n, nullptr);
  std::vector<interface::ITensor*> out(outs.size() * n, nullptr);
  for (int s = 0; s < n; ++s) {
    const Job& j = *jobs[s];
    if (j.model_id != model || j.input_handle < 0 || j.output_handle < 0 || !j.following_jobs.empty())
      return absl::UnimplementedError("job without request slots");
    for (size_t k = 0; k < ins.size(); ++k) {
      Tensor* t = in_it->second->SlotTensor(ins[k], j.input_handle);
      if (!t || !t->IsRingMemory()) return absl::UnimplementedError("input slot not page-locked");
      in[k * n + s] = t;
    }
    for (size_t k = 0; k < outs.size(); ++k)
      // a subgraph output outside the output ring feeds a later subgraph:
      // it must reach the executor's own views
      if (!out_it->second->IsTensorIndexValid(outs[k])) return absl::UnimplementedError("intermediate output");
    // as in CopyOutputs, but without waiting: a slot held right now sends
    // the pass to the staged path at once, whose CopyOutputs waits (bounded,
    // once) and fails that job's output copy alone if the hold outlasts it
    if (!out_it->second->TryAcquireForWrite(j.output_handle)) return absl::UnimplementedError("output slot held");
    for (size_t k = 0; k < outs.size(); ++k) {
      Tensor* t = out_it->second->SlotTensor(outs[k], j.output_handle);
      if (!t || !t->IsRingMemory()) return absl::UnimplementedError("output slot not page-locked");
      out[k * n + s] = t;
    }
  }
  return jb->ExecuteJobBatchDirect(key, n, in, out);
}

absl::Status Engine::TryCopyOutputTensorsFromSlot(const Job& job, int n, int slot) {
  if (job.output_handle < 0) return absl::OkStatus();
  const SubgraphKey& key = job.subgraph_key;
  auto* jb = dynamic_cast<hip::IJobBatching*>(GetModelExecutor(key));
  if (!jb) return absl::InternalError("no batching executor for " + key.ToString());
  return CopyOutputs(job, [&](int t) { return jb->GetJobSlotView(key, t, n, slot); });
}

}  // namespace band
