#include "backend/hip/completion.h"

#include <immintrin.h>
#include <pthread.h>

#include <map>

#include "backend/hip/affinity.h"

namespace band {
namespace hip {

CompletionPoller& CompletionPoller::ForDevice(int ordinal) {
  static std::mutex mu;
  static auto* pollers = new std::map<int, std::unique_ptr<CompletionPoller>>();  // never destroyed
  std::lock_guard<std::mutex> lock(mu);
  auto& p = (*pollers)[ordinal];
  if (!p) p.reset(new CompletionPoller(ordinal));
  return *p;
}

CompletionPoller::CompletionPoller(int ordinal) : ordinal_(ordinal) {
  thread_ = std::thread([this] { Run(); });
}

CompletionPoller::~CompletionPoller() {
  {
    std::lock_guard<std::mutex> lock(mu_);
    stop_ = true;
  }
  work_cv_.notify_all();
  if (thread_.joinable()) thread_.join();
}

int CompletionPoller::Wait(bh_event_t ev) {
  Waiter w;
  w.ev = ev;
  std::unique_lock<std::mutex> lock(mu_);
  waiters_.push_back(&w);
  if (waiters_.size() == 1) work_cv_.notify_one();
  w.cv.wait(lock, [&] { return w.done; });
  return w.rc;
}

void CompletionPoller::Run() {
  char name[16];
  std::snprintf(name, sizeof(name), "band-poll%d", ordinal_);
  pthread_setname_np(pthread_self(), name);
  // next to the GPU (and its workers) when the NUMA node is known
  PinCallingThreadToGpu(ordinal_);
  bh_set_device(ordinal_);
  std::vector<Waiter*> snap;
  std::unique_lock<std::mutex> lock(mu_);
  while (true) {
    work_cv_.wait(lock, [&] { return stop_ || !waiters_.empty(); });
    if (stop_) return;
    snap = waiters_;
    lock.unlock();
    // query outside the lock; a waiter stays registered (and alive) until
    // it is marked done below, under the lock
    std::vector<std::pair<Waiter*, int>> finished;
    for (Waiter* w : snap) {
      const int rc = bh_event_query(w->ev);
      if (rc != BH_ENOTREADY) finished.emplace_back(w, rc);
    }
    if (finished.empty())
      for (int i = 0; i < 64; ++i) _mm_pause();  // ~1-2 us between sweeps
    lock.lock();
    for (auto& f : finished) {
      for (size_t i = 0; i < waiters_.size(); ++i)
        if (waiters_[i] == f.first) {
          waiters_[i] = waiters_.back();
          waiters_.pop_back();
          break;
        }
      f.first->rc = f.second;
      f.first->done = true;
      f.first->cv.notify_one();
    }
  }
}

}  // namespace hip
}  // namespace band
