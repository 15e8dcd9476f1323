// Workers (band/worker.h, worker_device_queue.cc, worker_global_queue.cc):
// one thread per configured device worker that pops jobs, copies their
// inputs into the executor's views, runs ExecuteSubgraph, feeds the latency
// estimator, forwards the remaining subgraphs of a split job to the planner
// and copies the outputs out.
//   DeviceQueueWorker - own FIFO (fixed_worker / round_robin)
//   GlobalQueueWorker - one job at a time, the planner holds the queue
//                       (SEL / HEFT / LSF)
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

#include "band/device/cpu.h"
#include "engine/config.h"
#include "engine/engine_interface.h"

namespace band {

class Worker {
 public:
  // waiting time reported while paused / throttled (band/worker.h)
  static constexpr int64_t kLargeWaitingTime = INT32_MAX / 2;

  Worker(IEngine* engine, WorkerId worker_id, DeviceFlag device_flag);
  virtual ~Worker();

  absl::Status Init(const WorkerConfig& config);
  void Start();
  void End();
  void Pause();
  void Resume();
  // blocks until the worker has no job (profiling pauses then waits)
  void Wait();

  WorkerId GetId() const { return worker_id_; }
  DeviceFlag GetDeviceFlag() const { return device_flag_; }
  const CpuSet& GetWorkerThreadAffinity() const { return cpu_set_; }
  int GetNumThreads() const { return num_threads_; }
  std::mutex& GetDeviceMtx() { return device_mtx_; }
  bool IsAvailable() const { return !is_throttling_ && !is_paused_; }

  // all of these expect device_mtx_ held by the caller except GetWaitingTime
  virtual bool IsEnqueueReady() const { return IsAvailable(); }
  virtual bool EnqueueJob(Job& job) = 0;
  virtual bool HasJob() = 0;
  virtual int GetCurrentJobId() = 0;
  virtual int64_t GetWaitingTime() = 0;
  // no queued or running job and available: what GetWaitingTime() == 0
  // means, read without the lock or pricing a queue (the planner's
  // round_robin scan touches every worker on every wake-up)
  bool IsIdleNow() const { return idle_.load(std::memory_order_acquire); }
  // subgraph executions finished by this worker (each job of a batched pass)
  int64_t GetJobsRun() const { return jobs_run_.load(std::memory_order_relaxed); }
  // host time of the worker's job phases, microseconds since start:
  // [0] input copies (request ring -> executor), [1] invoke (launch + sync),
  // [2] output copies (executor -> output ring), [3] passes run
  void GetPhaseTimes(int64_t out[4]) const {
    for (int i = 0; i < 4; ++i) out[i] = phase_us_[i].load(std::memory_order_relaxed);
  }

 protected:
  virtual Job* GetCurrentJob() = 0;
  virtual void EndEnqueue() = 0;
  // Job batching (extension; device_mtx_ held): moves up to `max` queued
  // jobs that can share one batched pass with `head` into `out`.
  virtual void TakeBatchPartners(const Job& head, int max, std::vector<Job>* out) {}
  void Work();
  // runs `head` + `partners` as one batched pass (device_mtx_ not held)
  void WorkBatch(Job* head, std::vector<Job>& partners);
  static bool IsValid(const Job& job);
  static bool Batchable(const Job& job);

  IEngine* const engine_;
  const WorkerId worker_id_;
  const DeviceFlag device_flag_;
  std::mutex device_mtx_;
  std::condition_variable request_cv_;
  std::condition_variable wait_cv_;
  bool kill_worker_ = false;
  bool is_paused_ = false;
  bool is_throttling_ = false;
  CpuSet cpu_set_;
  // the thread's placement is settled: its CpuSet pinned it, or the GPU
  // backend's NUMA hook ran (worker thread only)
  bool cpu_pinned_ = false;
  int num_threads_ = -1;
  int availability_check_interval_ms_ = 30000;
  // expected latency of the batch partners of the running pass (device_mtx_):
  // they left the queue but the worker has not finished them, so
  // GetWaitingTime keeps counting them (at their one-job latency, an upper
  // bound of their share of the batched pass)
  int64_t partners_expected_us_ = 0;
  // IsIdleNow's flag, recomputed under device_mtx_ wherever the queue or
  // the availability changes
  std::atomic<bool> idle_{true};
  std::atomic<int64_t> jobs_run_{0};
  std::atomic<int64_t> phase_us_[4] = {{0}, {0}, {0}, {0}};
  void RefreshIdle() {
    idle_.store(IsAvailable() && !HasJob() && partners_expected_us_ == 0, std::memory_order_release);
  }

 private:
  std::thread thread_;
  std::once_flag start_once_;
  bool started_ = false;
};

class DeviceQueueWorker : public Worker {
 public:
  using Worker::Worker;
  bool EnqueueJob(Job& job) override;
  bool HasJob() override { return !requests_.empty(); }
  int GetCurrentJobId() override { return requests_.empty() ? -1 : requests_.front().job_id; }
  int64_t GetWaitingTime() override;

 protected:
  Job* GetCurrentJob() override { return requests_.empty() ? nullptr : &requests_.front(); }
  void EndEnqueue() override { requests_.pop_front(); }
  void TakeBatchPartners(const Job& head, int max, std::vector<Job>* out) override;

 private:
  JobQueue requests_;  // deque: pointers to elements survive push_back
};

class GlobalQueueWorker : public Worker {
 public:
  using Worker::Worker;
  bool IsEnqueueReady() const override { return !is_busy_ && IsAvailable(); }
  bool EnqueueJob(Job& job) override;
  bool HasJob() override { return is_busy_; }
  int GetCurrentJobId() override { return current_job_.job_id; }
  int64_t GetWaitingTime() override;

 protected:
  Job* GetCurrentJob() override { return is_busy_ ? &current_job_ : nullptr; }
  void EndEnqueue() override { is_busy_ = false; }

 private:
  Job current_job_;
  bool is_busy_ = false;
};

}  // namespace band
