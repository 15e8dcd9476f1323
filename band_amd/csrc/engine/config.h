// Runtime configuration of the harness (band/config.h:10-89): profiling,
// planner, workers and subgraph preparation.  Defaults are the reference's.
#pragma once
#include <limits>
#include <string>
#include <vector>

#include "band/common.h"

namespace band {

struct ProfileConfig {
  bool online = true;
  int num_warmups = 1;
  int num_runs = 1;
  std::string profile_data_path;
  float smoothing_factor = 0.1f;
  // extension (BANDX_PROFILE_SHARE_IDENTICAL): workers of one device kind
  // (same DeviceFlag, thread count and CPU mask) share their latency
  // estimates - see LatencyEstimator::UpdateLatency
  bool share_identical_workers = false;
};

struct PlannerConfig {
  int schedule_window_size = std::numeric_limits<int>::max();
  std::vector<SchedulerType> schedulers;
  CPUMaskFlag cpu_mask = CPUMaskFlag::kAll;
  std::string log_path;
};

struct WorkerConfig {
  // one worker per device flag unless configured (band/config.h:46-56)
  WorkerConfig() {
    for (size_t i = 0; i < EnumLength<DeviceFlag>(); i++) workers.push_back(static_cast<DeviceFlag>(i));
    cpu_masks.assign(workers.size(), CPUMaskFlag::kAll);
    num_threads.assign(workers.size(), 1);
  }
  std::vector<DeviceFlag> workers;
  std::vector<CPUMaskFlag> cpu_masks;
  std::vector<int> num_threads;
  bool allow_worksteal = false;
  int availability_check_interval_ms = 30000;
  // Extension (not in band/config.h): a device-queue worker runs up to this
  // many queued whole-model jobs of one subgraph as one batched pass when
  // the executor implements interface::IJobBatching.  1 = Band's behaviour.
  int max_job_batch = 1;
  // Extension: the pass-size policy of job batching (Engine::MaxJobBatch):
  // a batched pass of a model takes at most the jobs whose expected pass
  // time fits this target in microseconds (0 = off: up to max_job_batch).
  int pass_target_us = 0;
};

struct SubgraphConfig {
  int minimum_subgraph_size = 7;
  SubgraphPreparationType subgraph_preparation_type = SubgraphPreparationType::kMergeUnitSubgraph;
};

struct RuntimeConfig {
  CPUMaskFlag cpu_mask = CPUMaskFlag::kAll;
  SubgraphConfig subgraph_config;
  ProfileConfig profile_config;
  PlannerConfig planner_config;
  WorkerConfig worker_config;
};

}  // namespace band
