#include "engine/planner.h"

#include <pthread.h>

#include <cstdio>

#include "engine/logger.h"
#include <fstream>

#include "engine/time.h"
#include "engine/worker.h"

namespace band {

void SafeBool::notify() {
  {
    std::lock_guard<std::mutex> l(mu_);
    flag_ = true;
  }
  cv_.notify_all();
}

void SafeBool::terminate() {
  {
    std::lock_guard<std::mutex> l(mu_);
    terminated_ = true;
  }
  cv_.notify_all();
}

bool SafeBool::wait() {
  std::unique_lock<std::mutex> l(mu_);
  cv_.wait(l, [this] { return flag_ || terminated_; });
  flag_ = false;
  return terminated_;
}

Planner::Planner(IEngine& engine) : engine_(engine), jobs_finished_record_(kNumFinishedRecords) {
  planner_thread_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "band-planner");
    absl::Status s = Plan();
    if (!s.ok()) BAND_LOG(LogSeverity::kError, "planner thread failed: %s", s.message().c_str());
  });
}

Planner::~Planner() {
  if (!log_path_.empty()) DumpLog();
  planner_safe_bool_.terminate();
  planner_thread_.join();
}

absl::Status Planner::Init(const PlannerConfig& config) {
  schedule_window_size_ = config.schedule_window_size;
  log_path_ = config.log_path;
  if (config.schedulers.empty() || config.schedulers.size() > 2)
    return absl::InternalError("[Planner] Not supported for " + std::to_string(config.schedulers.size()) +
                               " schedulers");
  for (SchedulerType t : config.schedulers) {
    std::unique_ptr<IScheduler> s;
    switch (t) {
      case SchedulerType::kFixedWorker: s.reset(new FixedWorkerScheduler(engine_)); break;
      case SchedulerType::kFixedWorkerGlobalQueue: s.reset(new FixedWorkerGlobalQueueScheduler(engine_)); break;
      case SchedulerType::kRoundRobin: s.reset(new RoundRobinScheduler(engine_)); break;
      case SchedulerType::kShortestExpectedLatency:
        s.reset(new ShortestExpectedLatencyScheduler(engine_, schedule_window_size_));
        break;
      case SchedulerType::kHeterogeneousEarliestFinishTime:
        s.reset(new HEFTScheduler(engine_, schedule_window_size_, false));
        break;
      case SchedulerType::kLeastSlackTimeFirst:
        s.reset(new LeastSlackFirstScheduler(engine_, schedule_window_size_));
        break;
      case SchedulerType::kHeterogeneousEarliestFinishTimeReserved:
        s.reset(new HEFTScheduler(engine_, schedule_window_size_, true));
        break;
      default: return absl::InternalError("[Planner] Unsupported scheduler type.");
    }
    if (!schedulers_.empty() && schedulers_[0]->NeedFallbackSubgraphs() != s->NeedFallbackSubgraphs())
      return absl::InternalError("[Planner] Different type of scheduler requirements.");
    schedulers_.push_back(std::move(s));
  }
  local_queues_.resize(schedulers_.size());
  if (GetWorkerType() == (static_cast<int>(WorkerType::kDeviceQueue) | static_cast<int>(WorkerType::kGlobalQueue)))
    return absl::InternalError("All schedulers must have the same worker type.");
  return absl::OkStatus();
}

absl::Status Planner::AddScheduler(std::unique_ptr<IScheduler> scheduler) {
  schedulers_.push_back(std::move(scheduler));
  local_queues_.resize(schedulers_.size());
  if (GetWorkerType() == (static_cast<int>(WorkerType::kDeviceQueue) | static_cast<int>(WorkerType::kGlobalQueue)))
    return absl::InternalError("All schedulers must have the same worker type.");
  return absl::OkStatus();
}

JobId Planner::EnqueueRequest(Job job, bool push_front) { return EnqueueBatch({std::move(job)}, push_front)[0]; }

std::vector<JobId> Planner::EnqueueBatch(std::vector<Job> jobs, bool push_front) {
  std::vector<JobId> ids(jobs.size());
  {
    std::lock_guard<std::mutex> lock(requests_mtx_);
    const int64_t now = time::NowMicros();
    for (size_t i = 0; i < jobs.size(); ++i) {
      Job& j = jobs[i];
      if (j.enqueue_time == 0) j.enqueue_time = now;  // kept for the rest of a split job
      if (j.job_id == -1) j.job_id = num_submitted_jobs_++;
      ids[i] = j.job_id;
    }
    requests_.insert(push_front ? requests_.begin() : requests_.end(), std::make_move_iterator(jobs.begin()),
                     std::make_move_iterator(jobs.end()));
  }
  planner_safe_bool_.notify();
  return ids;
}

void Planner::Wait(const std::vector<int>& job_ids) {
  if (job_ids.empty()) return;
  std::unique_lock<std::mutex> lock(job_finished_mtx_);
  end_invoke_.wait(lock, [&] {
    for (int id : job_ids)
      if (IsJobIdValid(id) && jobs_finished_record_[RecordIndex(id)].job_id != id) return false;
    return true;
  });
}

void Planner::WaitAll() {
  std::unique_lock<std::mutex> lock(job_finished_mtx_);
  end_invoke_.wait(lock, [this] { return num_finished_jobs_ >= num_submitted_jobs_; });
}

void Planner::EnqueueFinishedJob(Job& job) { EnqueueFinishedJobs({&job}); }

// The finished records of a group of jobs (one batched pass, or a single
// job) under one lock and one wake-up of the waiters; then every request
// slot is freed and the callbacks run once for the group.  Per job the order
// is the reference's (band/planner.cc:133-165): record, then callbacks.
void Planner::EnqueueFinishedJobs(const std::vector<Job*>& jobs) {
  std::vector<const Job*> ended;  // requests that end here (not a split job's inner subgraph)
  ended.reserve(jobs.size());
  {
    std::lock_guard<std::mutex> lock(job_finished_mtx_);
    for (Job* job : jobs) {
      if (!engine_.IsEnd(job->subgraph_key) && job->status == JobStatus::kSuccess) continue;
      Job& rec = jobs_finished_record_[RecordIndex(job->job_id)];
      rec = *job;
      rec.following_jobs.clear();  // the record only needs the times / status
      num_finished_jobs_++;
      ended.push_back(job);
    }
    if (!ended.empty()) end_invoke_.notify_all();
  }
  // callbacks may re-enter the engine, so they run outside the lock.  The
  // request's input slot was consumed when the job started: free it before
  // the callbacks, which may submit into this model's full ring; the output
  // slot stays held until they return, so a request that reuses the slot
  // cannot overwrite (or invalidate) the outputs a callback reads
  std::vector<const Job*> notify;
  for (const Job* job : ended) {
    if (job->require_callback) {
      engine_.HoldOutput(*job);
      notify.push_back(job);
    }
    engine_.ReleaseRequest(*job);
  }
  if (notify.empty()) return;
  {
    std::lock_guard<std::mutex> cb_lock(on_end_request_mtx_);
    for (auto& cb : on_end_requests_callbacks_) cb.second(notify);
    for (const Job* job : notify) {
      const absl::Status s =
          job->status == JobStatus::kSuccess ? absl::OkStatus() : absl::InternalError("Job failed.");
      for (auto& cb : on_end_request_callbacks_) cb.second(job->job_id, s);
    }
  }
  for (const Job* job : notify) engine_.UnholdOutput(*job);
}

void Planner::PrepareReenqueue(Job& job) {
  job.invoke_time = 0;
  job.end_time = 0;
  job.resolved_unit_subgraphs = 0;
  job.following_jobs.clear();
}

bool Planner::NeedFallbackSubgraphs() const {
  for (const auto& s : schedulers_)
    if (s->NeedFallbackSubgraphs()) return true;
  return false;
}

int Planner::GetWorkerType() const {
  int t = 0;
  for (const auto& s : schedulers_) t |= static_cast<int>(s->GetWorkerType());
  return t;
}

Job Planner::GetFinishedJob(int job_id) {
  std::lock_guard<std::mutex> lock(job_finished_mtx_);
  if (IsJobIdValid(job_id) && jobs_finished_record_[RecordIndex(job_id)].job_id == job_id)
    return jobs_finished_record_[RecordIndex(job_id)];
  return Job();
}

std::vector<Job> Planner::GetFinishedJobs() {
  std::lock_guard<std::mutex> lock(job_finished_mtx_);
  std::vector<Job> out;
  const int first = std::max(0, num_submitted_jobs_ - kNumFinishedRecords);
  for (int id = first; id < num_submitted_jobs_; ++id) {
    const Job& r = jobs_finished_record_[RecordIndex(id)];
    if (r.job_id == id) out.push_back(r);
  }
  return out;
}

CallbackId Planner::SetOnEndRequest(std::function<void(int, absl::Status)> on_end_request) {
  std::lock_guard<std::mutex> lock(on_end_request_mtx_);
  on_end_request_callbacks_[next_callback_id_] = std::move(on_end_request);
  return next_callback_id_++;
}

CallbackId Planner::SetOnEndRequests(EndRequestsCallback on_end_requests) {
  std::lock_guard<std::mutex> lock(on_end_request_mtx_);
  on_end_requests_callbacks_[next_callback_id_] = std::move(on_end_requests);
  return next_callback_id_++;
}

absl::Status Planner::UnsetOnEndRequest(CallbackId id) {
  std::lock_guard<std::mutex> lock(on_end_request_mtx_);
  if (!on_end_request_callbacks_.erase(id) && !on_end_requests_callbacks_.erase(id))
    return absl::InternalError("Callback id not found.");
  return absl::OkStatus();
}

// planner thread (band/planner.cc:268-293)
absl::Status Planner::Plan() {
  while (!planner_safe_bool_.wait()) {
    CopyToLocalQueues();
    bool reschedule = false;
    for (size_t i = 0; i < schedulers_.size() && i < local_queues_.size(); ++i)
      reschedule |= !schedulers_[i]->Schedule(local_queues_[i]);
    if (reschedule) planner_safe_bool_.notify();
  }
  return absl::OkStatus();
}

// one scheduler takes everything; with two, SLO jobs go to the first
// (band/planner.cc:295-320)
void Planner::CopyToLocalQueues() {
  std::lock_guard<std::mutex> lock(requests_mtx_);
  if (requests_.empty() || local_queues_.empty()) return;
  if (local_queues_.size() == 1) {
    local_queues_[0].insert(local_queues_[0].end(), std::make_move_iterator(requests_.begin()),
                            std::make_move_iterator(requests_.end()));
  } else {
    for (Job& j : requests_) local_queues_[j.slo_us > 0 ? 0 : 1].push_back(std::move(j));
  }
  requests_.clear();
}

// band/planner.cc:322-365.  A job whose worker cannot take it right now goes
// back to the head of the request queue WITHOUT waking the planner: the
// worker triggers the planner when it frees up, so the job is retried then
// (the reference notifies immediately and spins the planner thread).
bool Planner::EnqueueToWorker(const std::vector<ScheduleAction>& actions) {
  bool ok = true;
  std::vector<Job> rejected;  // back to the queue head in their original order
  // consecutive actions for one subgraph key (a batched assignment) take the
  // worker's lock once and read the key's latency estimates once
  for (size_t i = 0; i < actions.size();) {
    const SubgraphKey& key = actions[i].second;
    size_t end = i + 1;
    while (end < actions.size() && actions[end].second == key) ++end;
    Worker* worker = engine_.GetWorker(key.GetWorkerId());
    std::vector<Job> ready;
    ready.reserve(end - i);
    for (; i < end; ++i) {
      Job job = actions[i].first;
      if (worker == nullptr) {
        BAND_LOG(LogSeverity::kWarning, "EnqueueToWorker: null worker id %d", key.GetWorkerId());
        job.status = JobStatus::kEnqueueFailed;
        EnqueueFinishedJob(job);
      } else if (IsSLOViolated(job)) {
        job.status = JobStatus::kSLOViolation;
        job.invoke_time = -1;  // dropped before running
        job.end_time = time::NowMicros();
        ok = false;
        EnqueueFinishedJob(job);
      } else {
        ready.push_back(std::move(job));
      }
    }
    if (ready.empty()) continue;
    const int64_t profiled = engine_.GetProfiled(key), expected = engine_.GetExpected(key);
    std::unique_lock<std::mutex> lock(worker->GetDeviceMtx());
    for (Job& job : ready) {
      if (worker->IsEnqueueReady()) {
        UpdateJobScheduleStatus(job, key, profiled, expected);
        worker->EnqueueJob(job);
      } else {
        rejected.push_back(std::move(job));
      }
    }
  }
  if (!rejected.empty()) {
    std::lock_guard<std::mutex> rl(requests_mtx_);
    requests_.insert(requests_.begin(), std::make_move_iterator(rejected.begin()),
                     std::make_move_iterator(rejected.end()));
  }
  return ok;
}

bool Planner::IsSLOViolated(const Job& job) {
  if (job.status == JobStatus::kSLOViolation) return true;
  if (job.slo_us <= 0) return false;
  const WorkerWaitingTime waiting = engine_.GetWorkerWaitingTime();
  auto it = waiting.find(job.subgraph_key.GetWorkerId());
  const int64_t wait = it == waiting.end() ? 0 : it->second;
  const int64_t expected = wait + job.expected_execution_time;
  const int64_t remaining = job.slo_us - (time::NowMicros() - job.enqueue_time);
  return expected > remaining;
}

// stamp the job with its subgraph and, if the subgraph does not finish the
// model, attach the remainder as a following job (band/planner.cc:380-404)
void Planner::UpdateJobScheduleStatus(Job& job, const SubgraphKey& key, int64_t profiled, int64_t expected) {
  job.subgraph_key = key;
  job.profiled_execution_time = profiled;
  job.expected_execution_time = expected;
  job.resolved_unit_subgraphs |= key.GetUnitIndices();
  if (!engine_.IsEnd(key)) {
    Job rest(job.model_id);
    rest.model_fname = job.model_fname;
    rest.slo_us = job.slo_us;
    rest.enqueue_time = job.enqueue_time;
    rest.following_jobs = job.following_jobs;
    rest.expected_latency = job.expected_latency;
    rest.job_id = job.job_id;
    rest.input_handle = job.input_handle;
    rest.output_handle = job.output_handle;
    rest.require_callback = job.require_callback;
    rest.resolved_unit_subgraphs = job.resolved_unit_subgraphs;
    rest.previous_subgraph_keys = job.previous_subgraph_keys;
    rest.previous_subgraph_keys.push_back(job.subgraph_key);
    job.following_jobs.clear();
    job.following_jobs.push_back(std::move(rest));
  }
}

// finished-job log (the reference dumps a chrome trace, band/job_tracer.cc);
// one JSON object per line with the fields of Job::ToJson
void Planner::DumpLog() {
  std::ofstream f(log_path_);
  if (!f) return;
  for (const Job& j : GetFinishedJobs())
    f << "{\"enqueue_time\":" << j.enqueue_time << ",\"invoke_time\":" << j.invoke_time
      << ",\"end_time\":" << j.end_time << ",\"profiled_execution_time\":" << j.profiled_execution_time
      << ",\"expected_execution_time\":" << j.expected_execution_time
      << ",\"expected_latency\":" << j.expected_latency << ",\"slo_us\":" << j.slo_us
      << ",\"model_id\":" << j.model_id << ",\"unit_indices\":\"" << j.subgraph_key.GetUnitIndicesString()
      << "\",\"worker_id\":" << j.subgraph_key.GetWorkerId() << ",\"job_id\":" << j.job_id
      << ",\"status\":\"" << ToString(j.status) << "\"}\n";
}

}  // namespace band
