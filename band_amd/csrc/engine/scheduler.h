// Schedulers (band/scheduler/*.h).  A scheduler drains (part of) the
// planner's local queue into worker queues through IEngine::EnqueueToWorker
// and returns false when a job must be rescheduled.  Each declares whether
// it needs fallback subgraphs (model_analyzer partitions the model) and
// which worker type it drives.
#pragma once
#include <map>

#include "engine/engine_interface.h"

namespace band {

class IScheduler {
 public:
  explicit IScheduler(IEngine& engine) : engine_(engine) {}
  virtual ~IScheduler() = default;
  virtual bool Schedule(JobQueue& requests) = 0;
  virtual bool NeedFallbackSubgraphs() = 0;
  virtual WorkerType GetWorkerType() = 0;

 protected:
  IEngine& engine_;
};

// request.target_worker_id, else the engine's model->worker map; always the
// largest subgraph of the model on that worker (fixed_worker_scheduler.cc:4-26)
class FixedWorkerScheduler : public IScheduler {
 public:
  using IScheduler::IScheduler;
  bool Schedule(JobQueue& requests) override;
  bool NeedFallbackSubgraphs() override { return false; }
  WorkerType GetWorkerType() override { return WorkerType::kDeviceQueue; }
};

// Global-queue variant of fixed_worker: a job waits in the planner until its
// worker is idle.  (The reference declares it and leaves the body
// unimplemented, fixed_worker_global_queue_scheduler.cc:4-56.)
class FixedWorkerGlobalQueueScheduler : public IScheduler {
 public:
  using IScheduler::IScheduler;
  bool Schedule(JobQueue& requests) override;
  bool NeedFallbackSubgraphs() override { return false; }
  WorkerType GetWorkerType() override { return WorkerType::kGlobalQueue; }
};

// one job per idle worker, first job in queue order that the worker can run
// (round_robin_scheduler.cc:7-30).  Deviation: the reference never refreshes
// the waiting times, so every worker looks idle forever and requests that
// arrive one at a time all land on the lowest worker id (SURVEY.md s7 hard
// part 3).  Here the waiting times are refreshed and the scan starts after
// the worker served last, so arrivals rotate over the idle workers; a job
// with no idle worker waits in the planner until a worker frees up.
// Job batching (extension, WorkerConfig::max_job_batch > 1): an idle worker
// also takes the following queued requests of the same model, up to its
// executor's batch, which its DeviceQueueWorker runs as one pass.
class RoundRobinScheduler : public IScheduler {
 public:
  using IScheduler::IScheduler;
  bool Schedule(JobQueue& requests) override;
  bool NeedFallbackSubgraphs() override { return false; }
  WorkerType GetWorkerType() override { return WorkerType::kDeviceQueue; }

 private:
  WorkerId next_ = 0;  // scan starts here
  // job batching, BANDX_BATCH_GROUP=largest: an idle worker's pass takes the
  // model with the most queued requests (its oldest first) instead of the
  // queue head's model, so passes are fuller (deviation; off by default)
  int group_largest_ = -1;  // -1: read the environment on first use
};

// repeatedly place the job whose best plan finishes last ("largest shortest
// latency") on the first subgraph of that plan
// (shortest_expected_latency_scheduler.cc:9-93)
class ShortestExpectedLatencyScheduler : public IScheduler {
 public:
  ShortestExpectedLatencyScheduler(IEngine& engine, int window_size)
      : IScheduler(engine), window_size_(window_size) {}
  bool Schedule(JobQueue& requests) override;
  bool NeedFallbackSubgraphs() override { return true; }
  WorkerType GetWorkerType() override { return WorkerType::kGlobalQueue; }

 private:
  const int window_size_;
};

// HEFT over idle workers, optionally reserving the next subgraph of each
// split job (heterogeneous_earliest_finish_time_scheduler.cc:6-140)
class HEFTScheduler : public IScheduler {
 public:
  HEFTScheduler(IEngine& engine, int window_size, bool reserve)
      : IScheduler(engine), window_size_(window_size), reserve_(reserve) {}
  bool Schedule(JobQueue& requests) override;
  bool NeedFallbackSubgraphs() override { return true; }
  WorkerType GetWorkerType() override { return WorkerType::kGlobalQueue; }

 private:
  const int window_size_;
  const bool reserve_;
  std::map<JobId, SubgraphKey> reserved_;
};

// least slack first within the window; jobs that cannot meet their SLO are
// dropped as SLO violations (least_slack_first_scheduler.cc:7-97)
class LeastSlackFirstScheduler : public IScheduler {
 public:
  LeastSlackFirstScheduler(IEngine& engine, int window_size) : IScheduler(engine), window_size_(window_size) {}
  bool Schedule(JobQueue& requests) override;
  bool NeedFallbackSubgraphs() override { return true; }
  WorkerType GetWorkerType() override { return WorkerType::kGlobalQueue; }

 private:
  int64_t GetSlackTime(int64_t current_time, const Job& job) const;
  const int window_size_;
};

}  // namespace band
