// CompletionPoller: one host thread per GPU that waits on the device for
// every pass in flight on it, so the threads that issued those passes can
// sleep instead of spinning.
//
// ExecuteSubgraph is synchronous (band/worker.cc:274-291 timestamps right
// after it), so every Band GPU worker blocks once per job until its pass is
// done.  hipStreamSynchronize does that by busy-polling: a core per worker
// for the whole pass - 8 cores per GPU at the C3 headline, 64 on an 8-GPU
// node with one engine.  A blocking-sync event sleeps, but its wake-up goes
// through the runtime's interrupt path and cost 15-20 % of throughput
// (profiles/r04e_*).  Here a waiting thread records an event after its pass
// and parks on a condition variable; the GPU's poller thread queries every
// registered event back to back (hipEventQuery reads the completion signal
// in host memory, no interrupt) and wakes each waiter as its pass ends: one
// polling core per GPU, whatever the number of workers.  The poller sleeps
// when nothing is in flight.  BAND_HIP_SYNC=poller selects it.
#pragma once

#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "band_hip_kernels.h"

namespace band {
namespace hip {

class CompletionPoller {
 public:
  // the poller of GPU `ordinal` (created on first use, lives to process exit)
  static CompletionPoller& ForDevice(int ordinal);
  // blocks until the work recorded in `ev` (on a stream of this GPU) is done;
  // returns bh_event_query's final code (0 = done)
  int Wait(bh_event_t ev);
  ~CompletionPoller();

 private:
  explicit CompletionPoller(int ordinal);
  struct Waiter {
    bh_event_t ev;
    bool done = false;
    int rc = 0;
    std::condition_variable cv;
  };
  void Run();

  const int ordinal_;
  std::mutex mu_;
  std::condition_variable work_cv_;  // the poller sleeps here while idle
  std::vector<Waiter*> waiters_;
  bool stop_ = false;
  std::thread thread_;
};

}  // namespace hip
}  // namespace band
