#include "engine/worker.h"

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cstdio>

#include "engine/logger.h"

#include "engine/time.h"

// Optional hook of the HIP backend (include/band_hip_backend.h): pins the
// calling worker thread to its GPU's NUMA node.  Weak, so a harness linked
// without that backend simply does not pin.
extern "C" int bhx_pin_worker_thread(int worker_id) __attribute__((weak));

namespace band {

namespace {
// the CPUs a worker's CpuSet names, read as Band reads a mask
// (band/device/cpu.h:21-40); empty when it names none or all of them
std::vector<int> NamedCpus(const CpuSet& set) {
  std::vector<int> cpus;
  const int n = static_cast<int>(std::min<size_t>(GetCPUCount(), CPU_SETSIZE));
  for (int i = 0; i < n; ++i)
    if (set.IsEnabled(i)) cpus.push_back(i);
  cpu_set_t proc;
  CPU_ZERO(&proc);
  if (cpus.empty() || sched_getaffinity(0, sizeof(proc), &proc) != 0) return {};
  bool all = true;
  for (int c = 0; c < CPU_SETSIZE && all; ++c)
    if (CPU_ISSET(c, &proc) && !set.IsEnabled(c)) all = false;
  return all ? std::vector<int>() : cpus;
}
}  // namespace

Worker::Worker(IEngine* engine, WorkerId worker_id, DeviceFlag device_flag)
    : engine_(engine), worker_id_(worker_id), device_flag_(device_flag) {}

Worker::~Worker() {
  if (started_ && !kill_worker_) End();
}

absl::Status Worker::Init(const WorkerConfig& config) {
  availability_check_interval_ms_ = config.availability_check_interval_ms;
  // per-worker settings are indexed by worker id (band/worker.cc:35-45)
  const size_t i = static_cast<size_t>(worker_id_);
  const CPUMaskFlag mask = i < config.cpu_masks.size() ? config.cpu_masks[i] : CPUMaskFlag::kAll;
  cpu_set_ = BandCPUMaskGetSet(mask);
  num_threads_ = i < config.num_threads.size() ? config.num_threads[i] : 1;
  return absl::OkStatus();
}

void Worker::Start() {
  std::call_once(start_once_, [this] {
    started_ = true;
    thread_ = std::thread([this] {
      // named for per-thread profiles (tools/planner_ceiling.py); a CpuSet
      // that names a proper subset of the CPUs pins the worker thread
      // (band/worker.cc:195-205 does this on mobile builds, where
      // BandCPUMaskGetSet fills the sets)
      char name[16];
      std::snprintf(name, sizeof(name), "band-w%d", worker_id_);
      pthread_setname_np(pthread_self(), name);
      if (!NamedCpus(cpu_set_).empty()) {
        cpu_pinned_ = true;
        if (!SetCPUThreadAffinity(cpu_set_).ok())
          BAND_LOG(LogSeverity::kWarning, "worker %d: could not set its CPU affinity", worker_id_);
      }
      Work();
    });
  });
}

void Worker::End() {
  {
    std::lock_guard<std::mutex> lock(device_mtx_);
    kill_worker_ = true;
  }
  request_cv_.notify_all();
  if (thread_.joinable()) thread_.join();
}

void Worker::Pause() {
  std::lock_guard<std::mutex> lock(device_mtx_);
  is_paused_ = true;
  RefreshIdle();
}

void Worker::Resume() {
  {
    std::lock_guard<std::mutex> lock(device_mtx_);
    is_paused_ = false;
    RefreshIdle();
  }
  request_cv_.notify_one();
}

void Worker::Wait() {
  std::unique_lock<std::mutex> lock(device_mtx_);
  wait_cv_.wait(lock, [this] { return !HasJob(); });
}

bool Worker::IsValid(const Job& job) {
  return job.model_id >= 0 && job.subgraph_key.IsValid() && job.enqueue_time > 0 && job.invoke_time == 0 &&
         job.end_time == 0;
}

// The per-job hot loop (band/worker.cc:222-323).  Differences from the
// reference: an invoke error finishes the job as kInvokeFailure instead of
// entering HandleDeviceError (which double-locks its mutex there,
// band/worker_device_queue.cc), and the job stays at the queue head until
// it is done so GetWaitingTime() keeps counting it.
void Worker::Work() {
  while (true) {
    std::unique_lock<std::mutex> lock(device_mtx_);
    if (!HasJob()) wait_cv_.notify_all();
    request_cv_.wait(lock, [this] { return kill_worker_ || (HasJob() && !is_paused_); });
    if (kill_worker_) break;
    Job* job = GetCurrentJob();
    lock.unlock();

    if (!job || !IsValid(*job)) {
      BAND_LOG(LogSeverity::kError, "worker %d spotted an invalid job (model %d)", worker_id_,
                   job ? job->model_id : -1);
      lock.lock();
      if (job) {
        job->status = JobStatus::kInvokeFailure;
        Job failed = *job;
        EndEnqueue();
        RefreshIdle();
        lock.unlock();
        engine_->EnqueueFinishedJob(failed);
        engine_->Trigger();
      }
      continue;
    }

    // a GPU worker whose CpuSet names no CPUs goes to its GPU's NUMA node
    // once that GPU is known (its first executor exists), before its first
    // job's GPU call; only this engine-owned thread moves
    if (!cpu_pinned_ && device_flag_ == DeviceFlag::kGPU && bhx_pin_worker_thread)
      cpu_pinned_ = bhx_pin_worker_thread(worker_id_) >= 0;

    const SubgraphKey key = job->subgraph_key;
    const int max_batch = engine_->MaxJobBatch(key);
    if (max_batch > 1 && Batchable(*job)) {
      std::vector<Job> partners;
      lock.lock();
      TakeBatchPartners(*job, max_batch - 1, &partners);
      partners_expected_us_ = 0;
      for (const Job& p : partners) partners_expected_us_ += engine_->GetExpected(p.subgraph_key);
      lock.unlock();
      if (!partners.empty()) {
        WorkBatch(job, partners);
        continue;
      }
    }
    const int64_t t_in = time::NowMicros();
    // a whole-model job whose executor reads / writes the request ring slots
    // directly (no staging copies); Unimplemented: the copy path below
    absl::Status direct = absl::UnimplementedError("");
    if (job->following_jobs.empty()) {
      lock.lock();
      job->invoke_time = time::NowMicros();
      lock.unlock();
      direct = engine_->InvokeJobBatchDirect(key, {job});
    }
    if (!absl::IsUnimplemented(direct)) {
      job->end_time = time::NowMicros();
      phase_us_[1].fetch_add(job->end_time - job->invoke_time, std::memory_order_relaxed);
      if (direct.ok()) {
        engine_->UpdateLatency(key, job->end_time - job->invoke_time);
        job->status = JobStatus::kSuccess;
      } else {
        BAND_LOG(LogSeverity::kError, "worker %d failed to invoke job %d: %s", worker_id_, job->job_id,
                 direct.message().c_str());
        job->status = JobStatus::kInvokeFailure;
      }
    } else if (engine_->TryCopyInputTensors(*job).ok()) {
      lock.lock();
      job->invoke_time = time::NowMicros();
      lock.unlock();
      phase_us_[0].fetch_add(job->invoke_time - t_in, std::memory_order_relaxed);
      const absl::Status status = engine_->Invoke(key);
      job->end_time = time::NowMicros();
      phase_us_[1].fetch_add(job->end_time - job->invoke_time, std::memory_order_relaxed);
      if (status.ok()) {
        engine_->UpdateLatency(key, job->end_time - job->invoke_time);
        if (!job->following_jobs.empty()) {
          const absl::Status snap = engine_->SaveIntermediates(*job);
          if (!snap.ok()) BAND_LOG(LogSeverity::kError, "%s", snap.message().c_str());
          engine_->EnqueueBatch(job->following_jobs, true);
        }
        const absl::Status out = engine_->TryCopyOutputTensors(*job);
        phase_us_[2].fetch_add(time::NowMicros() - job->end_time, std::memory_order_relaxed);
        job->status = out.ok() ? JobStatus::kSuccess : JobStatus::kOutputCopyFailure;
        if (!out.ok()) BAND_LOG(LogSeverity::kWarning, "%s", out.message().c_str());
      } else {
        BAND_LOG(LogSeverity::kError, "worker %d failed to invoke job %d: %s", worker_id_, job->job_id,
                     status.message().c_str());
        job->status = JobStatus::kInvokeFailure;
      }
    } else {
      BAND_LOG(LogSeverity::kError, "worker %d failed to copy input of job %d", worker_id_, job->job_id);
      job->status = JobStatus::kInputCopyFailure;
    }
    jobs_run_.fetch_add(1, std::memory_order_relaxed);
    phase_us_[3].fetch_add(1, std::memory_order_relaxed);
    engine_->EnqueueFinishedJob(*job);
    lock.lock();
    EndEnqueue();
    RefreshIdle();
    lock.unlock();
    engine_->Trigger();
  }
}

// A batch is the head job plus queued jobs of the same whole-model subgraph
// (no split job state to carry).  All of them get the batch's invoke / end
// times; the latency estimator is not fed batched passes (they are not the
// per-job latency it models).
void Worker::WorkBatch(Job* head, std::vector<Job>& partners) {
  std::vector<Job*> jobs{head};
  for (Job& p : partners) jobs.push_back(&p);
  const int n = static_cast<int>(jobs.size());
  const SubgraphKey key = head->subgraph_key;
  std::vector<bool> copied(n, true);
  const int64_t t_in = time::NowMicros();
  // the pass's I/O straight between the request rings and the device when
  // the executor and the rings allow it; else staged through the slot views
  int64_t invoke_time = time::NowMicros();
  {
    std::lock_guard<std::mutex> lock(device_mtx_);
    head->invoke_time = invoke_time;
  }
  absl::Status status = engine_->InvokeJobBatchDirect(key, jobs);
  const bool direct = !absl::IsUnimplemented(status);
  if (!direct) {
    for (int i = 0; i < n; ++i) {
      copied[i] = engine_->TryCopyInputTensorsToSlot(*jobs[i], n, i).ok();
      if (!copied[i]) {
        BAND_LOG(LogSeverity::kError, "worker %d failed to copy input of job %d", worker_id_, jobs[i]->job_id);
        jobs[i]->status = JobStatus::kInputCopyFailure;
      }
    }
    invoke_time = time::NowMicros();
    {
      std::lock_guard<std::mutex> lock(device_mtx_);
      head->invoke_time = invoke_time;
    }
    status = engine_->InvokeJobBatch(key, n);
  }
  const int64_t end_time = time::NowMicros();
  phase_us_[0].fetch_add(invoke_time - t_in, std::memory_order_relaxed);
  phase_us_[1].fetch_add(end_time - invoke_time, std::memory_order_relaxed);
  for (int i = 0; i < n; ++i) {
    Job& j = *jobs[i];
    j.invoke_time = invoke_time;
    j.end_time = end_time;
    if (!copied[i]) continue;
    if (!status.ok()) {
      j.status = JobStatus::kInvokeFailure;
      continue;
    }
    if (direct) {  // the outputs are already in the request's output slot
      j.status = JobStatus::kSuccess;
      continue;
    }
    const absl::Status out = engine_->TryCopyOutputTensorsFromSlot(j, n, i);
    j.status = out.ok() ? JobStatus::kSuccess : JobStatus::kOutputCopyFailure;
    if (!out.ok()) BAND_LOG(LogSeverity::kWarning, "%s", out.message().c_str());
  }
  if (!status.ok())
    BAND_LOG(LogSeverity::kError, "worker %d failed to invoke a batch of %d jobs: %s", worker_id_, n,
             status.message().c_str());
  jobs_run_.fetch_add(n, std::memory_order_relaxed);
  phase_us_[2].fetch_add(time::NowMicros() - end_time, std::memory_order_relaxed);
  phase_us_[3].fetch_add(1, std::memory_order_relaxed);
  // partners first, the head (still at the queue front) last, as one group
  std::rotate(jobs.begin(), jobs.begin() + 1, jobs.end());
  engine_->EnqueueFinishedJobs(jobs);
  {
    std::lock_guard<std::mutex> lock(device_mtx_);
    partners_expected_us_ = 0;
    EndEnqueue();
    RefreshIdle();
  }
  engine_->Trigger();
}

bool Worker::Batchable(const Job& job) {
  return job.following_jobs.empty() && job.previous_subgraph_keys.empty() && !job.intermediates;
}

void DeviceQueueWorker::TakeBatchPartners(const Job& head, int max, std::vector<Job>* out) {
  if (requests_.size() < 2 || max <= 0) return;
  // the head stays at the front (GetWaitingTime counts it); partners are
  // moved out of the queue in FIFO order
  JobQueue rest;
  auto it = std::next(requests_.begin());
  for (; it != requests_.end(); ++it) {
    if (static_cast<int>(out->size()) < max && it->subgraph_key == head.subgraph_key && IsValid(*it) &&
        Batchable(*it))
      out->push_back(std::move(*it));
    else
      rest.push_back(std::move(*it));
  }
  requests_.erase(std::next(requests_.begin()), requests_.end());
  for (Job& j : rest) requests_.push_back(std::move(j));
}

bool DeviceQueueWorker::EnqueueJob(Job& job) {
  if (!IsEnqueueReady()) return false;
  requests_.push_back(job);
  idle_.store(false, std::memory_order_release);
  request_cv_.notify_one();
  return true;
}

// sum of the expected latencies of the queued jobs, minus the elapsed part
// of the running one (band/worker_device_queue.cc:41-66)
int64_t DeviceQueueWorker::GetWaitingTime() {
  std::lock_guard<std::mutex> lock(device_mtx_);
  if (!IsAvailable()) return kLargeWaitingTime;
  int64_t total = partners_expected_us_;
  for (auto it = requests_.begin(); it != requests_.end(); ++it) {
    const int64_t expected = engine_->GetExpected(it->subgraph_key);
    total += expected;
    if (it == requests_.begin() && it->invoke_time > 0) {
      const int64_t elapsed = time::NowMicros() - it->invoke_time;
      if (elapsed > 0) total -= std::min(elapsed, expected);
    }
  }
  return total;
}

bool GlobalQueueWorker::EnqueueJob(Job& job) {
  if (!IsEnqueueReady()) return false;
  current_job_ = job;
  is_busy_ = true;
  idle_.store(false, std::memory_order_release);
  request_cv_.notify_one();
  return true;
}

// expected remaining time of the running job (band/worker_global_queue.cc:130-160)
int64_t GlobalQueueWorker::GetWaitingTime() {
  std::unique_lock<std::mutex> lock(device_mtx_);
  if (!IsAvailable()) return kLargeWaitingTime;
  if (!is_busy_) return 0;
  const int64_t invoke_time = current_job_.invoke_time;
  const SubgraphKey key = current_job_.subgraph_key;
  lock.unlock();
  const int64_t expected = engine_->GetExpected(key);
  if (invoke_time == 0) return expected;
  return std::max<int64_t>(expected - (time::NowMicros() - invoke_time), 0);
}

}  // namespace band
