// Scheduler policies; each cites the reference policy it restates.
#include "engine/scheduler.h"

#include <cstdlib>
#include <map>
#include <string>

#include <algorithm>
#include <limits>
#include <unordered_set>

#include "engine/time.h"

namespace band {

namespace {
// the model -> worker choice of fixed_worker (request target first)
WorkerId FixedTarget(const IEngine& engine, const Job& job) {
  return job.target_worker_id != -1 ? job.target_worker_id : engine.GetModelWorker(job.model_id);
}
}  // namespace

bool FixedWorkerScheduler::Schedule(JobQueue& requests) {
  bool ok = true;
  while (!requests.empty()) {
    Job job = std::move(requests.front());
    requests.pop_front();
    const SubgraphKey key = engine_.GetLargestSubgraphKey(job.model_id, FixedTarget(engine_, job));
    ok &= engine_.EnqueueToWorker({job, key});
  }
  return ok;
}

bool FixedWorkerGlobalQueueScheduler::Schedule(JobQueue& requests) {
  bool ok = true;
  engine_.UpdateWorkersWaiting();
  std::set<WorkerId> idle = engine_.GetIdleWorkers();
  const WorkerWaitingTime waiting = engine_.GetWorkerWaitingTime();
  for (auto it = requests.begin(); it != requests.end() && !idle.empty();) {
    const WorkerId w = FixedTarget(engine_, *it);
    auto slot = idle.find(w);
    if (slot == idle.end()) {
      ++it;  // its worker is busy: the job stays queued
      continue;
    }
    Job job = std::move(*it);
    it = requests.erase(it);
    const SubgraphKey key = engine_.GetLargestSubgraphKey(job.model_id, w);
    job.expected_latency = waiting.at(w) + engine_.GetExpected(key);
    ok &= engine_.EnqueueToWorker({job, key});
    idle.erase(slot);
  }
  return ok;
}

bool RoundRobinScheduler::Schedule(JobQueue& requests) {
  bool ok = true;
  if (requests.empty()) return ok;
  const std::set<WorkerId> idle = engine_.GetIdleWorkersNow();
  if (idle.empty() || requests.empty()) return ok;
  // idle workers in rotation order, starting at next_
  std::vector<WorkerId> order(idle.lower_bound(next_), idle.end());
  order.insert(order.end(), idle.begin(), idle.lower_bound(next_));
  if (group_largest_ < 0) {
    const char* g = std::getenv("BANDX_BATCH_GROUP");
    group_largest_ = g && std::string(g) == "largest" ? 1 : 0;
  }
  for (WorkerId w : order) {
    if (requests.empty()) break;
    auto it = std::find_if(requests.begin(), requests.end(), [&](const Job& j) {
      return engine_.GetLargestSubgraphKey(j.model_id, w).IsValid();
    });
    if (it == requests.end()) continue;
    if (group_largest_ && requests.size() > 1) {
      // the model with the most queued requests this worker can run; its
      // oldest request leads the pass (ties: the older group)
      std::map<ModelId, int> count;
      for (const Job& j : requests) ++count[j.model_id];
      int most = 0;
      for (auto j = requests.begin(); j != requests.end(); ++j) {
        const int c = count[j->model_id];
        if (c > most && engine_.GetLargestSubgraphKey(j->model_id, w).IsValid()) {
          most = c;
          it = j;
        }
        count[j->model_id] = 0;  // later requests of a model are not its oldest
      }
    }
    const SubgraphKey key = engine_.GetLargestSubgraphKey(it->model_id, w);
    // job batching (extension): the idle worker also takes the next queued
    // requests of the same model, up to its batch, and runs them in one pass;
    // one EnqueueToWorkerBatch call keeps their FIFO order if it is refused.
    // They are taken out by one stable compaction of the span from the first
    // to the last taken request only (erasing each from the middle of the
    // deque moved the whole tail per job, and rebuilding the whole queue per
    // assignment moved every queued request: with hundreds queued and 24-job
    // batches either made the planner thread the bottleneck)
    std::vector<ScheduleAction> actions;
    const int batch = std::max(1, engine_.MaxJobBatch(key));
    actions.reserve(batch);
    if (batch == 1) {
      actions.emplace_back(std::move(*it), key);
      requests.erase(it);
    } else {
      const ModelId model = key.GetModelId();
      auto last = it;  // `it` is this model's first request
      int take = 0;
      for (auto j = it; j != requests.end() && take < batch; ++j)
        if (j->model_id == model) {
          last = j;
          ++take;
        }
      const auto end = std::next(last);
      auto out = it;
      for (auto r = it; r != end; ++r) {
        if (r->model_id == model && static_cast<int>(actions.size()) < take) {
          actions.emplace_back(std::move(*r), key);
        } else {
          if (out != r) *out = std::move(*r);
          ++out;
        }
      }
      requests.erase(out, end);
    }
    ok &= engine_.EnqueueToWorkerBatch(actions);
    next_ = w + 1;
  }
  return ok;
}

bool ShortestExpectedLatencyScheduler::Schedule(JobQueue& requests) {
  bool ok = true;
  const int window = std::min<int>(window_size_, static_cast<int>(requests.size()));
  JobQueue local(std::make_move_iterator(requests.begin()), std::make_move_iterator(requests.begin() + window));
  requests.erase(requests.begin(), requests.begin() + window);
  while (!local.empty()) {
    engine_.UpdateWorkersWaiting();
    const WorkerWaitingTime waiting = engine_.GetWorkerWaitingTime();
    int64_t most_urgent = -1;
    int target = -1;
    SubgraphKey target_key;
    std::unordered_set<std::pair<int, BitMask>, JobIdBitMaskHash> seen;
    for (size_t i = 0; i < local.size(); ++i) {
      const Job& j = local[i];
      if (!seen.insert({j.model_id, j.resolved_unit_subgraphs}).second) continue;
      auto best = engine_.GetSubgraphWithShortestLatency(j, waiting);
      if (best.first.empty()) continue;
      if (most_urgent < best.second) {
        most_urgent = best.second;
        target = static_cast<int>(i);
        target_key = best.first.front();
      }
    }
    if (target < 0 || !target_key.IsValid()) {
      // no job of the window has a runnable subgraph: hand them back
      // (the reference spins here forever)
      requests.insert(requests.begin(), std::make_move_iterator(local.begin()), std::make_move_iterator(local.end()));
      return false;
    }
    Job job = std::move(local[target]);
    local.erase(local.begin() + target);
    if (engine_.IsBegin(target_key)) job.expected_latency = most_urgent;
    ok &= engine_.EnqueueToWorker({job, target_key});
  }
  return ok;
}

bool HEFTScheduler::Schedule(JobQueue& requests) {
  bool ok = true;
  int window = std::min<int>(window_size_, static_cast<int>(requests.size()));
  while (window > 0) {
    engine_.UpdateWorkersWaiting();
    const std::set<WorkerId> idle = engine_.GetIdleWorkers();
    if (idle.empty()) break;
    WorkerWaitingTime waiting = engine_.GetWorkerWaitingTime();
    std::set<JobId> yielded;  // jobs whose best worker is busy this pass
    int64_t most_urgent;
    int target;
    SubgraphKey target_key, next_key;
    while (true) {
      most_urgent = -1;
      target = -1;
      std::unordered_set<std::pair<int, BitMask>, JobIdBitMaskHash> seen;
      for (int i = 0; i < window; ++i) {
        const Job& j = requests[i];
        if (yielded.count(j.job_id)) continue;
        if (!seen.insert({j.model_id, j.resolved_unit_subgraphs}).second) continue;
        // waiting time including the subgraphs reserved for other jobs
        WorkerWaitingTime with_reserved(waiting);
        for (const auto& r : reserved_)
          if (r.first != j.job_id) with_reserved[r.second.GetWorkerId()] += engine_.GetExpected(r.second);
        auto best = engine_.GetSubgraphWithShortestLatency(j, with_reserved);
        if (best.first.empty()) continue;
        if (most_urgent < best.second) {
          most_urgent = best.second;
          target = i;
          target_key = best.first.front();
          next_key = best.first.size() > 1 ? best.first[1] : SubgraphKey();
        }
      }
      if (target < 0) return ok;
      const WorkerId w = target_key.GetWorkerId();
      if (idle.count(w)) break;
      // the most urgent job cannot start now: account for it and look again
      waiting[w] += engine_.GetExpected(target_key);
      yielded.insert(requests[target].job_id);
    }
    Job job = std::move(requests[target]);
    requests.erase(requests.begin() + target);
    --window;
    if (engine_.IsBegin(target_key)) job.expected_latency = most_urgent;
    const JobId id = job.job_id;
    ok &= engine_.EnqueueToWorker({job, target_key});
    if (reserve_) {
      if (next_key != SubgraphKey()) reserved_[id] = next_key;
      else reserved_.erase(id);
    }
  }
  return ok;
}

int64_t LeastSlackFirstScheduler::GetSlackTime(int64_t now, const Job& job) const {
  if (job.slo_us <= 0) return std::numeric_limits<int>::max();
  return job.enqueue_time + job.slo_us - now - job.expected_latency;
}

bool LeastSlackFirstScheduler::Schedule(JobQueue& requests) {
  bool ok = true;
  engine_.UpdateWorkersWaiting();
  const int window = std::min<int>(window_size_, static_cast<int>(requests.size()));
  if (window <= 0) return ok;
  std::set<WorkerId> idle = engine_.GetIdleWorkers();
  if (idle.empty()) return ok;
  WorkerWaitingTime waiting = engine_.GetWorkerWaitingTime();
  const int64_t now = time::NowMicros();
  // refresh each job's best-plan latency, then order the window by slack
  for (int i = 0; i < window; ++i)
    requests[i].expected_latency = engine_.GetSubgraphWithShortestLatency(requests[i], waiting).second;
  std::sort(requests.begin(), requests.begin() + window,
            [&](const Job& a, const Job& b) { return GetSlackTime(now, a) < GetSlackTime(now, b); });
  std::vector<int> done;
  for (int i = 0; i < window; ++i) {
    Job& job = requests[i];
    auto plan = engine_.GetSubgraphWithShortestLatency(job, waiting);
    if (plan.first.empty()) continue;
    const SubgraphKey key = plan.first.front();
    if (job.slo_us > 0 && now + plan.second > job.enqueue_time + job.slo_us) {
      job.status = JobStatus::kSLOViolation;  // dropped by the planner
      ok &= engine_.EnqueueToWorker({job, key});
      done.push_back(i);
      continue;
    }
    const WorkerId w = key.GetWorkerId();
    if (idle.count(w)) {
      waiting[w] += engine_.GetExpected(key);
      ok &= engine_.EnqueueToWorker({job, key});
      done.push_back(i);
    }
  }
  for (auto it = done.rbegin(); it != done.rend(); ++it) requests.erase(requests.begin() + *it);
  return ok;
}

}  // namespace band
