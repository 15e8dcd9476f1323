// JobCoalescer: batches concurrent ExecuteSubgraph calls of one model on one
// GPU into job-batch passes, inside the backend, under Band's unchanged
// worker loop.
//
// Band runs one job per ExecuteSubgraph (band/worker.cc:222-323 ->
// Engine::Invoke band/engine.cc:843-850 -> IModelExecutor::ExecuteSubgraph,
// band/backend/tfl/model_executor.cc:249-255), one executor per (model,
// worker), and each call is synchronous.  At batch 1 a MobileNet layer is a
// latency-bound launch, so a GPU served that way
// stays mostly idle.  Several Band workers on one GPU call ExecuteSubgraph
// on their own executors of the same model at the same time; the coalescer
// joins those calls:
//
//  - every whole-model kGPU executor of one (model object, GPU) joins one
//    coalescer at PrepareSubgraph.  When the second one joins, the
//    coalescer prepares `lanes` private executors of the model, each with
//    its own stream, activation arena and job-batch variants for 2..max
//    jobs (HipModelExecutor::PrepareJobBatches);
//  - a call queues itself; while a lane is free the queued calls are taken
//    in arrival order, up to max per pass.  A lone call runs its own
//    executor's batch-1 pass (the path without coalescing).  A group of n
//    calls runs as ONE pass of the lane's n-job variant: each member copies
//    its job's inputs (Band already copied them into the member's views)
//    into its slot of the lane's page-locked staging, the first member
//    (the leader) issues H2D -> kernels -> D2H on the lane's stream and
//    waits for the GPU, and every member copies its slot's outputs back
//    into its own views, where Band's TryCopyOutputTensors reads them;
//  - followers block on a condition variable (no spinning): only a pass's
//    leader waits on the GPU.  With every lane busy, new calls accumulate
//    and the next free lane takes them all (natural batching: no timer, no
//    added latency at low load).
//
// Each caller still returns only when its own outputs are in its views, so
// Band's per-job contract (synchronous ExecuteSubgraph, timestamps around
// it, band/worker.cc:274-291) holds unchanged.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "absl/status/status.h"
#include "band/common.h"
#include "band/interface/model.h"

namespace band {
namespace hip {

class HipModelExecutor;
struct PreparedSubgraph;

class JobCoalescer {
 public:
  struct Stats {
    int64_t calls = 0;        // ExecuteSubgraph calls routed here
    int64_t solo_passes = 0;  // calls that ran alone on their own executor
    int64_t group_passes = 0; // lane passes (>= 2 jobs)
    int64_t group_jobs = 0;   // jobs in those passes
    int64_t max_group = 0;
    int64_t bypass_calls = 0;         // calls that ran without lanes (none built: coalescing off)
    int64_t max_bypass_inflight = 0;  // the most such calls running at once
  };

  // Registers `e`'s whole-model subgraph `key` of `model` on GPU `ordinal`;
  // returns the shared coalescer.  Prepares the lanes when a second
  // executor joins (max_batch jobs per pass, `lanes` passes in flight).
  static std::shared_ptr<JobCoalescer> Join(HipModelExecutor* e, interface::IModel* model, const SubgraphKey& key,
                                            int ordinal, int max_batch, int lanes);
  void Leave(HipModelExecutor* e);
  // one job of `e` (its inputs in sg's host views); returns when its
  // outputs are in sg's host views
  absl::Status Run(HipModelExecutor* e, PreparedSubgraph* sg);

  ~JobCoalescer();
  int members() const;
  bool lanes_ready() const;
  Stats stats() const;
  // process-wide totals over every coalescer (bench.py)
  static Stats Totals();
  static void ResetTotals();

 private:
  struct Group;
  struct Member {
    HipModelExecutor* exec;
    PreparedSubgraph* sg;
    Group* group = nullptr;
    int slot = -1;
    std::condition_variable cv;  // woken when the member is put in a group
  };
  struct Group {
    int lane = -1;
    int n = 0;
    std::vector<Member*> members;  // slot order
    int inputs_left = 0;   // members still copying their inputs in
    int outputs_left = 0;  // members still copying their outputs out
    bool finished = false;
    absl::Status status;
    std::condition_variable cv;
  };
  struct Lane {
    std::unique_ptr<HipModelExecutor> exec;
    SubgraphKey key;
    void* stream = nullptr;
  };

  JobCoalescer() = default;
  absl::Status BuildLanes(HipModelExecutor* e, interface::IModel* model, const SubgraphKey& key);
  // forms groups from the queue while a lane is free (mu_ held).  Unless
  // `force`, a group waits for want() queued calls: the head of the queue
  // then waits up to wait_us_ for more (JobCoalescer::Run) before it forces
  // a smaller one
  void Dispatch(bool force = false);
  // calls a free lane waits for: the size of the group that finished last
  // (its members are the calls coming back next), at most max_batch_
  int want() const;
  // releases a finished group's lane (mu_ held)
  void Release(Group* g);
  void Account(int n);
  void AccountBypass(int inflight);

  mutable std::mutex mu_;
  std::vector<HipModelExecutor*> members_;
  std::deque<Member*> pending_;
  std::vector<int> free_lanes_;  // lane tokens (solo passes hold one too)
  std::vector<Lane> lanes_;      // built when the second member joins
  bool lanes_ready_ = false;
  bool build_failed_ = false;  // also set while the one build runs
  int max_batch_ = 16;
  int num_lanes_ = 1;
  // BAND_HIP_COALESCE_IO: "copy" (default) - each member memcpys its job
  // into / out of the lane's staging and the lane moves the batch in one
  // DMA; "dma" - the leader DMAs each member's page-locked views straight
  // into / out of the lane's arena (no host copies; n small DMAs per tensor:
  // less CPU, 5-10 % less throughput on the C3 mix, profiles/r05b_*)
  bool dma_io_ = false;
  // BAND_HIP_COALESCE_WAIT_US (default 100): how long a free lane waits for
  // want() calls; 0 = dispatch whatever is queued at once
  int wait_us_ = 100;
  int last_group_ = 1;  // size of the group that released its lane last
  int bypass_inflight_ = 0;  // calls running without lanes right now
  bool fail_build_ = false;  // BAND_HIP_COALESCE_FAIL_BUILD (tests)
  int ordinal_ = -1;
  std::vector<size_t> in_bytes_, out_bytes_;  // per boundary tensor, one job
  Stats stats_;
};

}  // namespace hip
}  // namespace band
