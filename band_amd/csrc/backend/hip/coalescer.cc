#include "backend/hip/coalescer.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <tuple>

#include "backend/hip/model_executor.h"

namespace band {
namespace hip {

namespace {

// (model object, GPU ordinal, unit subgraph set) -> coalescer
using RegistryKey = std::tuple<const void*, int, std::vector<int>>;
std::mutex g_registry_mu;
std::map<RegistryKey, std::weak_ptr<JobCoalescer>>& Registry() {
  static auto* r = new std::map<RegistryKey, std::weak_ptr<JobCoalescer>>();
  return *r;
}

std::mutex g_totals_mu;
JobCoalescer::Stats g_totals;

}  // namespace

std::shared_ptr<JobCoalescer> JobCoalescer::Join(HipModelExecutor* e, interface::IModel* model,
                                                 const SubgraphKey& key, int ordinal, int max_batch, int lanes) {
  const std::set<int> units = key.GetUnitIndicesSet();
  RegistryKey rk{model, ordinal, std::vector<int>(units.begin(), units.end())};
  std::shared_ptr<JobCoalescer> c;
  {
    std::lock_guard<std::mutex> lock(g_registry_mu);
    auto& slot = Registry()[rk];
    c = slot.lock();
    if (!c) {
      c.reset(new JobCoalescer());
      c->max_batch_ = std::max(2, max_batch);
      c->num_lanes_ = std::max(1, lanes);
      c->ordinal_ = ordinal;
      for (int l = 0; l < c->num_lanes_; ++l) c->free_lanes_.push_back(l);
      if (const char* io = std::getenv("BAND_HIP_COALESCE_IO")) c->dma_io_ = std::string(io) == "dma";
      if (const char* w = std::getenv("BAND_HIP_COALESCE_WAIT_US")) c->wait_us_ = std::max(0, std::atoi(w));
      // test hook: the lane build fails as it would out of device memory
      if (const char* f = std::getenv("BAND_HIP_COALESCE_FAIL_BUILD")) c->fail_build_ = std::atoi(f) != 0;
      slot = c;
    }
  }
  bool build = false;
  {
    std::lock_guard<std::mutex> lock(c->mu_);
    if (std::find(c->members_.begin(), c->members_.end(), e) == c->members_.end()) c->members_.push_back(e);
    build = c->members_.size() >= 2 && !c->lanes_ready_ && !c->build_failed_;
    if (build) c->build_failed_ = true;  // one attempt (reset below on success)
  }
  if (build) {
    // Band prepares executors one at a time (Engine::RegisterModel), so the
    // lanes are built on the registering thread before any job can arrive;
    // until they are ready every call runs solo
    absl::Status s = c->BuildLanes(e, model, key);
    if (!s.ok()) {
      std::fprintf(stderr, "[band-hip] job coalescing off for model %d on GPU %d: %s\n", key.GetModelId(), ordinal,
                   std::string(s.message()).c_str());
      std::lock_guard<std::mutex> lock(c->mu_);
      c->lanes_.clear();
    } else {
      std::lock_guard<std::mutex> lock(c->mu_);
      c->build_failed_ = false;
    }
  }
  return c;
}

absl::Status JobCoalescer::BuildLanes(HipModelExecutor* e, interface::IModel* model, const SubgraphKey& key) {
  if (fail_build_) return absl::InternalError("coalescer: lane build failed (BAND_HIP_COALESCE_FAIL_BUILD)");
  PreparedSubgraph* base = e->Find(key);
  if (!base) return absl::InternalError("coalescer: no prepared subgraph");
  std::vector<size_t> in_bytes, out_bytes;
  for (int t : base->inputs) in_bytes.push_back(e->meta_[t]->bytes);
  for (int t : base->outputs) out_bytes.push_back(e->meta_[t]->bytes);
  std::vector<Lane> lanes;
  for (int l = 0; l < num_lanes_; ++l) {
    Lane lane;
    lane.exec = e->MakeLane();
    if (!lane.exec) return absl::InternalError("coalescer: lane stream");
    lane.stream = lane.exec->stream_;
    // the same op set as the member's (model-order I/O when that was {})
    std::set<int> ops;
    if (!base->model_order_io) ops.insert(base->ops.begin(), base->ops.end());
    absl::Status s = lane.exec->PrepareSubgraph(model, ops, key.GetUnitIndicesSet());
    if (!s.ok()) return s;
    lane.key = SubgraphKey(key.GetModelId(), lane.exec->worker_id_, key.GetUnitIndicesSet());
    PreparedSubgraph* ls = lane.exec->Find(lane.key);
    if (!ls || ls->inputs != base->inputs || ls->outputs != base->outputs)
      return absl::InternalError("coalescer: lane I/O differs from the subgraph's");
    s = lane.exec->PrepareJobBatches(model, lane.key, max_batch_);
    if (!s.ok()) return s;
    if (lane.exec->MaxJobBatch(lane.key) < max_batch_) return absl::InternalError("coalescer: lane has no batch variants");
    lanes.push_back(std::move(lane));
  }
  std::lock_guard<std::mutex> lock(mu_);
  lanes_ = std::move(lanes);
  in_bytes_ = in_bytes;
  out_bytes_ = out_bytes;
  lanes_ready_ = true;
  return absl::OkStatus();
}

void JobCoalescer::Leave(HipModelExecutor* e) {
  std::lock_guard<std::mutex> lock(mu_);
  members_.erase(std::remove(members_.begin(), members_.end(), e), members_.end());
}

JobCoalescer::~JobCoalescer() {
  std::lock_guard<std::mutex> lock(g_registry_mu);
  for (auto it = Registry().begin(); it != Registry().end();)
    it = it->second.expired() ? Registry().erase(it) : std::next(it);
}

int JobCoalescer::members() const {
  std::lock_guard<std::mutex> lock(mu_);
  return static_cast<int>(members_.size());
}

bool JobCoalescer::lanes_ready() const {
  std::lock_guard<std::mutex> lock(mu_);
  return lanes_ready_;
}

JobCoalescer::Stats JobCoalescer::stats() const {
  std::lock_guard<std::mutex> lock(mu_);
  return stats_;
}

JobCoalescer::Stats JobCoalescer::Totals() {
  std::lock_guard<std::mutex> lock(g_totals_mu);
  return g_totals;
}

void JobCoalescer::ResetTotals() {
  std::lock_guard<std::mutex> lock(g_totals_mu);
  g_totals = Stats();
}

void JobCoalescer::Account(int n) {
  stats_.calls += n;
  std::lock_guard<std::mutex> lock(g_totals_mu);
  if (n == 1) {
    ++stats_.solo_passes;
    ++g_totals.solo_passes;
  } else {
    ++stats_.group_passes;
    stats_.group_jobs += n;
    stats_.max_group = std::max<int64_t>(stats_.max_group, n);
    ++g_totals.group_passes;
    g_totals.group_jobs += n;
    g_totals.max_group = std::max<int64_t>(g_totals.max_group, n);
  }
  g_totals.calls += n;
}

void JobCoalescer::AccountBypass(int inflight) {
  ++stats_.calls;
  ++stats_.bypass_calls;
  stats_.max_bypass_inflight = std::max<int64_t>(stats_.max_bypass_inflight, inflight);
  std::lock_guard<std::mutex> lock(g_totals_mu);
  ++g_totals.calls;
  ++g_totals.bypass_calls;
  g_totals.max_bypass_inflight = std::max<int64_t>(g_totals.max_bypass_inflight, inflight);
}

int JobCoalescer::want() const {
  return lanes_ready_ && wait_us_ > 0 ? std::max(1, std::min(max_batch_, last_group_)) : 1;
}

void JobCoalescer::Dispatch(bool force) {
  while (!pending_.empty() && !free_lanes_.empty()) {
    if (!force && static_cast<int>(pending_.size()) < want()) {
      pending_.front()->cv.notify_one();  // the head times the wait
      return;
    }
    force = false;
    const int lane = free_lanes_.back();
    free_lanes_.pop_back();
    const int n = lanes_ready_ ? std::min<int>(max_batch_, static_cast<int>(pending_.size())) : 1;
    Group* g = new Group();
    g->lane = lane;
    g->n = n;
    g->inputs_left = n;
    g->outputs_left = n;
    for (int i = 0; i < n; ++i) {
      Member* m = pending_.front();
      pending_.pop_front();
      m->group = g;
      m->slot = i;
      g->members.push_back(m);
      if (dma_io_ && n > 1) --g->inputs_left;  // nothing for the member to copy in
      m->cv.notify_one();
    }
    Account(n);
  }
}

void JobCoalescer::Release(Group* g) {
  free_lanes_.push_back(g->lane);
  last_group_ = g->n;
  delete g;
  Dispatch();
}

absl::Status JobCoalescer::Run(HipModelExecutor* e, PreparedSubgraph* sg) {
  Member me{e, sg};
  std::unique_lock<std::mutex> lock(mu_);
  if (!lanes_ready_) {
    // no lanes (not built yet, or the build failed): coalescing is off, so
    // the call runs its own executor's pass at once, beside any others - it
    // takes no lane token, which would cap the model's concurrent calls on
    // this GPU at num_lanes_
    AccountBypass(++bypass_inflight_);
    lock.unlock();
    absl::Status s = e->RunPass(sg);
    lock.lock();
    --bypass_inflight_;
    return s;
  }
  pending_.push_back(&me);
  Dispatch();
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(wait_us_);
  while (!me.group) {
    if (pending_.front() == &me && !free_lanes_.empty()) {
      // a lane is free but fewer calls are queued than the last group had:
      // wait (bounded) for the rest of them, then take what is there
      if (!me.cv.wait_until(lock, deadline, [&] {
            return me.group != nullptr || static_cast<int>(pending_.size()) >= want() || free_lanes_.empty();
          })) {
        if (!me.group) Dispatch(true);
      } else if (!me.group) {
        Dispatch();
      }
    } else {
      me.cv.wait(lock);
    }
  }
  Group* g = me.group;

  if (g->n == 1) {
    // alone: this executor's own batch-1 pass (its graph, its stream)
    lock.unlock();
    absl::Status s = e->RunPass(sg);
    lock.lock();
    Release(g);
    return s;
  }

  Lane& lane = lanes_[g->lane];
  const int n = g->n;
  if (dma_io_) {
    if (me.slot == 0) {
      // the leader: every member's views straight to / from the lane's
      // arena around the n-job variant's kernels-only graph
      const size_t ni = sg->inputs.size(), no = sg->outputs.size();
      std::vector<HipTensorView> views;
      views.reserve((ni + no) * n);
      std::vector<const interface::ITensor*> in(ni * n);
      std::vector<interface::ITensor*> out(no * n);
      for (size_t k = 0; k < ni; ++k)
        for (int s = 0; s < n; ++s) {
          Member* m = g->members[s];
          const int t = sg->inputs[k];
          views.emplace_back(m->exec->meta_[t].get(), m->sg->host.at(t)->data());
          in[k * n + s] = &views.back();
        }
      for (size_t k = 0; k < no; ++k)
        for (int s = 0; s < n; ++s) {
          Member* m = g->members[s];
          const int t = sg->outputs[k];
          views.emplace_back(m->exec->meta_[t].get(), m->sg->host.at(t)->data());
          out[k * n + s] = &views.back();
        }
      lock.unlock();
      absl::Status s = lane.exec->ExecuteJobBatchDirect(lane.key, n, in, out);
      lock.lock();
      g->status = s;
      g->finished = true;
      g->cv.notify_all();
    } else {
      g->cv.wait(lock, [&] { return g->finished; });
    }
    absl::Status status = g->status;
    if (--g->outputs_left == 0) Release(g);
    return status;
  }
  lock.unlock();
  // this job's inputs into its slot of the lane's n-job staging (the
  // variant's page-locked boundary mirrors; slot s = the s-th batch-1 image)
  absl::Status copy = absl::OkStatus();
  for (size_t k = 0; k < sg->inputs.size(); ++k) {
    auto v = lane.exec->GetJobSlotView(lane.key, sg->inputs[k], n, me.slot);
    if (!v) {
      copy = absl::InternalError("coalescer: no slot view");
      break;
    }
    std::memcpy(v->GetData(), sg->host.at(sg->inputs[k])->data(), in_bytes_[k]);
  }
  lock.lock();
  if (!copy.ok()) g->status = copy;
  if (--g->inputs_left == 0) g->cv.notify_all();
  if (me.slot == 0) {
    // the leader: one pass for the group once every input is in
    g->cv.wait(lock, [&] { return g->inputs_left == 0; });
    absl::Status s = g->status;
    lock.unlock();
    if (s.ok()) s = lane.exec->ExecuteJobBatch(lane.key, n);
    lock.lock();
    g->status = s;
    g->finished = true;
    g->cv.notify_all();
  } else {
    g->cv.wait(lock, [&] { return g->finished; });
  }
  absl::Status status = g->status;
  lock.unlock();
  if (status.ok())
    for (size_t k = 0; k < sg->outputs.size(); ++k) {
      auto v = lane.exec->GetJobSlotView(lane.key, sg->outputs[k], n, me.slot);
      if (!v) {
        status = absl::InternalError("coalescer: no slot view");
        break;
      }
      std::memcpy(sg->host.at(sg->outputs[k])->data(), v->GetData(), out_bytes_[k]);
    }
  lock.lock();
  if (--g->outputs_left == 0) Release(g);  // the lane's staging is free again
  return status;
}

}  // namespace hip
}  // namespace band
