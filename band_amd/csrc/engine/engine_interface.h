// The engine surface that schedulers, the planner, workers and the latency
// estimator see (band/engine_interface.h).  Kept abstract so schedulers can
// be unit-tested against a mock engine, as the reference's
// band/test/scheduler_test.cc does.
#pragma once
#include <deque>
#include <functional>
#include <map>
#include <set>
#include <utility>
#include <vector>

#include "absl/status/status.h"
#include "band/common.h"
#include "band/model_spec.h"

namespace band {

class Worker;
using JobQueue = std::deque<Job>;
using ScheduleAction = std::pair<Job, SubgraphKey>;
using WorkerWaitingTime = std::map<WorkerId, int64_t>;

class IEngine {
 public:
  virtual ~IEngine() = default;

  // workers
  virtual void UpdateWorkersWaiting() const = 0;
  virtual WorkerWaitingTime GetWorkerWaitingTime() const = 0;
  virtual std::set<WorkerId> GetIdleWorkers() const = 0;
  // idle workers read directly (round_robin needs no waiting times): one
  // lock per worker instead of pricing every queue; the default is the
  // reference's UpdateWorkersWaiting + GetIdleWorkers
  virtual std::set<WorkerId> GetIdleWorkersNow() {
    UpdateWorkersWaiting();
    return GetIdleWorkers();
  }
  virtual size_t GetNumWorkers() const = 0;
  virtual DeviceFlag GetWorkerDevice(WorkerId id) const = 0;
  virtual Worker* GetWorker(WorkerId id) = 0;
  virtual const Worker* GetWorker(WorkerId id) const = 0;

  // subgraphs
  virtual SubgraphKey GetLargestSubgraphKey(ModelId model_id, WorkerId worker_id) const = 0;
  virtual const ModelSpec* GetModelSpec(ModelId model_id) const = 0;
  virtual WorkerId GetModelWorker(ModelId model_id) const = 0;
  virtual bool IsBegin(const SubgraphKey& key) const = 0;
  virtual bool IsEnd(const SubgraphKey& key) const = 0;
  virtual bool HasSubgraph(const SubgraphKey& key) const = 0;
  virtual void ForEachSubgraph(std::function<void(const SubgraphKey&)> visitor) const = 0;
  virtual absl::Status Invoke(const SubgraphKey& key) = 0;

  // scheduling helpers
  virtual std::pair<std::vector<SubgraphKey>, int64_t> GetSubgraphWithShortestLatency(
      const Job& job, const WorkerWaitingTime& worker_waiting) const = 0;
  virtual std::pair<SubgraphKey, int64_t> GetShortestSubgraphKey(const std::vector<SubgraphKey>& keys,
                                                                 int64_t start_time,
                                                                 const WorkerWaitingTime& worker_waiting) const = 0;

  // job data movement (worker thread)
  virtual absl::Status TryCopyInputTensors(const Job& job) = 0;
  virtual absl::Status TryCopyOutputTensors(const Job& job) = 0;
  // snapshot a non-final subgraph's outputs into the job's following jobs
  virtual absl::Status SaveIntermediates(Job& job) { return absl::OkStatus(); }

  // job batching (backend/hip/job_batching.h): n jobs of one subgraph, job i
  // in slot i; MaxJobBatch == 1 means the worker never batches `key`
  virtual int MaxJobBatch(const SubgraphKey& key) const { return 1; }
  virtual absl::Status TryCopyInputTensorsToSlot(const Job& job, int n, int slot) {
    return absl::InternalError("job batching unsupported");
  }
  virtual absl::Status InvokeJobBatch(const SubgraphKey& key, int n) { return absl::InternalError("job batching unsupported"); }
  // one batched pass whose I/O goes straight between the request rings'
  // slots and the device (IJobBatching::ExecuteJobBatchDirect);
  // Unimplemented: use the slot copies + InvokeJobBatch
  virtual absl::Status InvokeJobBatchDirect(const SubgraphKey& key, const std::vector<Job*>& jobs) {
    return absl::UnimplementedError("direct job batch I/O");
  }
  virtual absl::Status TryCopyOutputTensorsFromSlot(const Job& job, int n, int slot) {
    return absl::InternalError("job batching unsupported");
  }

  // latency estimator
  virtual void UpdateLatency(const SubgraphKey& key, int64_t latency) = 0;
  virtual int64_t GetProfiled(const SubgraphKey& key) const = 0;
  virtual int64_t GetExpected(const SubgraphKey& key) const = 0;
  virtual int64_t GetWorst(ModelId model_id) const = 0;

  // planner
  virtual void Trigger() = 0;
  virtual JobId EnqueueRequest(Job job, bool push_front = false) = 0;
  virtual std::vector<JobId> EnqueueBatch(std::vector<Job> jobs, bool push_front = false) = 0;
  virtual void PrepareReenqueue(Job& job) = 0;
  virtual void EnqueueFinishedJob(Job& job) = 0;
  // the jobs of one batched pass, in order: one record update and one
  // callback round instead of one per job
  virtual void EnqueueFinishedJobs(const std::vector<Job*>& jobs) {
    for (Job* j : jobs) EnqueueFinishedJob(*j);
  }
  // a finished request frees its request-ring slot (ring back-pressure)
  virtual void ReleaseRequest(const Job& job) {}
  // keeps a finished request's output slot from being rewritten by a newer
  // request while the end-request callbacks read it (Hold before the input
  // slot is released, Unhold after the callbacks)
  virtual void HoldOutput(const Job& job) {}
  virtual void UnholdOutput(const Job& job) {}
  virtual bool EnqueueToWorker(const ScheduleAction& action) = 0;
  virtual bool EnqueueToWorkerBatch(const std::vector<ScheduleAction>& actions) = 0;
};

}  // namespace band
