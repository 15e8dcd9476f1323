// Planner (band/planner.h/.cc): owns the request queue and the planner
// thread that moves requests into the schedulers' local queues, runs the
// schedulers and hands jobs to workers; records finished jobs in a
// 1000-slot ring that Wait() / GetFinishedJob() read.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "engine/config.h"
#include "engine/engine_interface.h"
#include "engine/scheduler.h"

namespace band {

using CallbackId = int;

// a level-triggered wake-up flag with termination (band/safe_bool.h)
class SafeBool {
 public:
  void notify();
  void terminate();
  // blocks until notified; returns true once terminated
  bool wait();

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  bool flag_ = false;
  bool terminated_ = false;
};

class Planner {
 public:
  static constexpr int kNumFinishedRecords = 1000;

  explicit Planner(IEngine& engine);
  ~Planner();
  absl::Status Init(const PlannerConfig& config);
  absl::Status AddScheduler(std::unique_ptr<IScheduler> scheduler);

  JobId EnqueueRequest(Job job, bool push_front = false);
  std::vector<JobId> EnqueueBatch(std::vector<Job> jobs, bool push_front = false);
  void Wait(const std::vector<int>& job_ids);
  void WaitAll();
  void EnqueueFinishedJob(Job& job);
  void EnqueueFinishedJobs(const std::vector<Job*>& jobs);
  void PrepareReenqueue(Job& job);
  bool EnqueueToWorker(const std::vector<ScheduleAction>& actions);
  void Trigger() { planner_safe_bool_.notify(); }

  bool NeedFallbackSubgraphs() const;
  int GetWorkerType() const;
  Job GetFinishedJob(int job_id);
  CallbackId SetOnEndRequest(std::function<void(int, absl::Status)> on_end_request);
  // extension: one call per group of finished requests (a batched pass ends
  // many at once) with their finished records; same id space and mutex as the
  // per-request callbacks, removed by UnsetOnEndRequest
  using EndRequestsCallback = std::function<void(const std::vector<const Job*>&)>;
  CallbackId SetOnEndRequests(EndRequestsCallback on_end_requests);
  absl::Status UnsetOnEndRequest(CallbackId id);
  std::map<ModelId, WorkerId>& GetModelWorkerMap() { return model_worker_map_; }
  // all finished records still in the ring, oldest first (job tracer)
  std::vector<Job> GetFinishedJobs();

 private:
  absl::Status Plan();
  void CopyToLocalQueues();
  bool IsSLOViolated(const Job& job);
  void UpdateJobScheduleStatus(Job& job, const SubgraphKey& target_key, int64_t profiled, int64_t expected);
  bool IsJobIdValid(int job_id) const { return job_id >= 0 && num_submitted_jobs_ - job_id <= kNumFinishedRecords; }
  static int RecordIndex(int job_id) { return job_id % kNumFinishedRecords; }
  void DumpLog();

  IEngine& engine_;
  SafeBool planner_safe_bool_;
  std::thread planner_thread_;

  std::mutex requests_mtx_;
  JobQueue requests_;
  std::vector<JobQueue> local_queues_;
  std::vector<std::unique_ptr<IScheduler>> schedulers_;
  int schedule_window_size_ = INT32_MAX;
  std::string log_path_;

  std::mutex job_finished_mtx_;
  std::condition_variable end_invoke_;
  std::vector<Job> jobs_finished_record_;
  std::atomic<int> num_submitted_jobs_{0};
  int num_finished_jobs_ = 0;

  std::mutex on_end_request_mtx_;
  std::map<CallbackId, std::function<void(int, absl::Status)>> on_end_request_callbacks_;
  std::map<CallbackId, EndRequestsCallback> on_end_requests_callbacks_;
  CallbackId next_callback_id_ = 0;
  std::map<ModelId, WorkerId> model_worker_map_;
};

}  // namespace band
