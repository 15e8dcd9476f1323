// HipModelExecutor: job batching (job_batching.h) - the batch variants of a
// subgraph on one shared arena, slot views, staged and direct (ring-slot DMA)
// batched passes.  Split from model_executor.cc.
#include "backend/hip/executor_internal.h"

#include "backend/hip/affinity.h"

namespace band {
namespace hip {

using namespace ex;

absl::Status HipModelExecutor::PrepareJobBatches(interface::IModel* model, const SubgraphKey& key, int max_batch) {
  // kGPU: batched graphs on the device; kCPU: the same lowering at batch n
  // run by the host kernels (one pass over n images instead of n passes)
  if (device_flag_ != DeviceFlag::kGPU && device_flag_ != DeviceFlag::kCPU)
    return absl::InternalError("job batching needs a kGPU or kCPU executor");
  PreparedSubgraph* base = Find(key);
  if (!base) return absl::InternalError("Cannot find subgraph");
  auto* hm = dynamic_cast<HipModel*>(model);
  if (!hm || hm != model_) return absl::InternalError("job batching: not the model this executor prepared");
  job_batches_.erase(key);
  // the harness batches this executor's jobs itself: no coalescing
  if (coalescer_) {
    coalescer_->Leave(this);
    coalescer_.reset();
  }
  if (max_batch <= 1) return absl::OkStatus();
  // anchors (2, 4, 8, .., max_batch) measure their fusion choices; every
  // other size reuses the next anchor's.  Anchors are prepared first, the
  // largest first of all: its arena and mirrors serve every variant.
  int step = 1;
  if (const char* e = std::getenv("BAND_HIP_BATCH_STEP")) step = std::max(1, std::atoi(e));
  std::vector<int> anchors;
  for (int b = 2; b < max_batch; b *= 2) anchors.push_back(b);
  anchors.push_back(max_batch);
  std::vector<int> order(anchors.rbegin(), anchors.rend());
  for (int b = max_batch - 1; b >= 2; --b)
    if ((b % step == 0) && std::find(anchors.begin(), anchors.end(), b) == anchors.end()) order.push_back(b);
  // the base's op set, or {} when the base was prepared as the whole model
  // (model-order I/O): the variants' I/O order is the base's
  std::set<int> ops;
  if (!base->model_order_io) ops.insert(base->ops.begin(), base->ops.end());
  const std::set<int> units = key.GetUnitIndicesSet();
  std::vector<JobBatchVariant> variants;
  HipModelExecutor* largest = nullptr;
  for (int b : order) {
    JobBatchVariant v;
    v.batch = b;
    RETURN_STATUS_IF(hm->CloneWithJobBatch(b, &v.model));
    t_variant_ctor = true;
    v.exec = std::make_unique<HipModelExecutor>(model_id_, worker_id_, device_flag_, thread_affinity_mask_,
                                                num_threads_);
    t_variant_ctor = false;
    v.exec->use_graph_ = use_graph_;
    v.exec->stream_ = stream_;  // a lane's variants run on the lane's stream
    v.exec->coalesce_ok_ = false;
    // direct job I/O captures the variants' graphs without host copies
    v.exec->io_mode_ = direct_io_ ? 1 : io_mode_;
    v.exec->direct_io_ = direct_io_;
    v.exec->block_sync_ = block_sync_;
    v.exec->sync_mode_ = sync_mode_;
    if (device_flag_ == DeviceFlag::kCPU) {  // one host pool per worker
      if (!cpu_pool_)
        cpu_pool_ = std::make_shared<CpuPool>(num_threads_ > 0 ? num_threads_ : 1,
                                              PinnableCpus(thread_affinity_mask_));
      v.exec->cpu_pool_ = cpu_pool_;
    }
    v.exec->io_stream_bytes_ = io_stream_bytes_;
    if (largest) {
      PreparedSubgraph* ls = largest->Find(key);
      v.exec->shared_arena_ = ls ? ls->arena : nullptr;
      v.exec->shared_host_from_ = ls;
    }
    if (std::find(anchors.begin(), anchors.end(), b) == anchors.end())
      v.exec->tune_batch_ = *std::lower_bound(anchors.begin(), anchors.end(), b);
    // the base subgraph's op set (a whole-model key prepares all ops)
    RETURN_STATUS_IF(v.exec->PrepareSubgraph(v.model.get(), ops, units));
    PreparedSubgraph* vs = v.exec->Find(key);
    if (!vs || vs->inputs != base->inputs || vs->outputs != base->outputs)
      return absl::InternalError("job batching: variant I/O differs from the subgraph's");
    if (!largest) largest = v.exec.get();
    variants.push_back(std::move(v));
  }
  // every variant's graph is captured here (one eager pass first, as
  // RunPass's second-run rule does): captured lazily, the first passes of a
  // rarely used size (a few jobs) captured inside the serving path, a
  // stall of that worker's lane of ~ms while its jobs wait.
  // BAND_HIP_PRECAPTURE=0 keeps the lazy capture (A-B runs).
  static const bool precapture = [] {
    const char* e = std::getenv("BAND_HIP_PRECAPTURE");
    return !(e && e[0] == '0');
  }();
  if (device_flag_ == DeviceFlag::kGPU && use_graph_ && precapture) {
    for (JobBatchVariant& v : variants) {
      PreparedSubgraph* vs = v.exec->Find(key);
      if (vs) RETURN_STATUS_IF(v.exec->PrecaptureGraph(vs));
    }
    RETURN_STATUS_IF(PrecaptureGraph(base));  // one-job passes
  }
  // ascending batch (VariantFor takes the smallest >= n); the largest
  // variant, whose arena / mirrors the others view, is destroyed last
  std::sort(variants.begin(), variants.end(),
            [](const JobBatchVariant& a, const JobBatchVariant& b) { return a.batch < b.batch; });
  job_batches_[key] = std::move(variants);
  return absl::OkStatus();
}

int HipModelExecutor::MaxJobBatch(const SubgraphKey& key) const {
  auto it = job_batches_.find(key);
  return it == job_batches_.end() || it->second.empty() ? 1 : it->second.back().batch;
}

const HipModelExecutor::JobBatchVariant* HipModelExecutor::VariantFor(const SubgraphKey& key, int n) const {
  auto it = job_batches_.find(key);
  if (it == job_batches_.end()) return nullptr;
  for (const JobBatchVariant& v : it->second)
    if (v.batch >= n) return &v;
  return nullptr;
}

std::shared_ptr<interface::ITensorView> HipModelExecutor::GetJobSlotView(const SubgraphKey& key, int index, int n,
                                                                          int slot) {
  if (n == 1 && slot == 0) return GetTensorView(key, index);
  const JobBatchVariant* v = VariantFor(key, n);
  if (!v || n < 1 || slot < 0 || slot >= n || index < 0 || index >= static_cast<int>(meta_.size())) return nullptr;
  PreparedSubgraph* vs = v->exec->Find(key);
  auto h = vs ? vs->host.find(index) : decltype(vs->host.end()){};
  if (!vs || h == vs->host.end()) return nullptr;  // slot views exist for boundary tensors only
  TensorMeta* m = meta_[index].get();
  return std::make_shared<HipTensorView>(m, h->second->data() + static_cast<size_t>(slot) * m->bytes);
}

absl::Status HipModelExecutor::ExecuteJobBatch(const SubgraphKey& key, int n) {
  if (n == 1) return ExecuteSubgraph(key);
  const JobBatchVariant* v = VariantFor(key, n);
  if (!v || n < 1) return absl::InternalError("no job batch variant for " + std::to_string(n) + " jobs");
  return v->exec->ExecuteSubgraph(key);
}

absl::Status HipModelExecutor::ExecuteJobBatchDirect(const SubgraphKey& key, int n,
                                                     const std::vector<const interface::ITensor*>& in,
                                                     const std::vector<interface::ITensor*>& out) {
  if (device_flag_ != DeviceFlag::kGPU || n < 1 || !direct_io_) return absl::UnimplementedError("direct job batch I/O");
  PreparedSubgraph* base = Find(key);
  if (n == 1) {
    // one job: the captured graph's own copy nodes, pointed at the job's
    // ring slots for this pass (back at the mirrors before any staged pass)
    if (!base || !use_graph_ || !base->graph || !base->io_in_graph || base->io_nodes.empty() ||
        !base->extra_d2h.empty() || in.size() != base->inputs.size() || out.size() != base->outputs.size())
      return absl::UnimplementedError("direct job batch I/O");
    for (size_t k = 0; k < in.size(); ++k)
      if (!in[k] || in[k]->GetBytes() != meta_[base->inputs[k]]->bytes)
        return absl::InternalError("direct job I/O: input size");
    for (size_t k = 0; k < out.size(); ++k)
      if (out[k] && out[k]->GetBytes() != meta_[base->outputs[k]]->bytes)
        return absl::InternalError("direct job I/O: output size");
    int rc = bh_set_device(ordinal_);
    if (rc) return HipErr(rc, "hipSetDevice");
    char* arena = static_cast<char*>(base->arena->ptr());
    // set first: a retarget that fails part-way leaves the nodes already
    // changed pointing at ring slots, and RestoreIoNodes must reset them all
    base->io_retargeted = true;
    for (const auto& nd : base->io_nodes) {
      char* dev = arena + base->offset.at(nd.tensor);
      const size_t bytes = meta_[nd.tensor]->bytes;
      if (nd.h2d) {
        const size_t k = std::find(base->inputs.begin(), base->inputs.end(), nd.tensor) - base->inputs.begin();
        rc = bh_graph_exec_set_memcpy(base->graph, nd.node, dev, in[k]->GetData(), bytes, 1);
      } else {
        const size_t k = std::find(base->outputs.begin(), base->outputs.end(), nd.tensor) - base->outputs.begin();
        char* host = out[k] ? out[k]->GetData() : base->host.at(nd.tensor)->data();
        rc = bh_graph_exec_set_memcpy(base->graph, nd.node, host, dev, bytes, 0);
      }
      if (rc) return HipErr(rc, "graph copy node");
    }
    rc = bh_graph_launch(base->graph, stream_);
    if (rc) return HipErr(rc, "graph launch");
    RETURN_STATUS_IF(WaitPass(base));
    ++base->runs;
    return absl::OkStatus();
  }

  const JobBatchVariant* v = VariantFor(key, n);
  if (!base || !v) return absl::InternalError("no job batch variant for " + std::to_string(n) + " jobs");
  if (in.size() != base->inputs.size() * n || out.size() != base->outputs.size() * n)
    return absl::InternalError("direct job batch I/O: tensor count mismatch");
  std::vector<size_t> per_job;
  for (int t : base->inputs) per_job.push_back(meta_[t]->bytes);
  for (int t : base->outputs) per_job.push_back(meta_[t]->bytes);
  PreparedSubgraph* vs = v->exec->Find(key);
  if (!vs) return absl::InternalError("job batch variant lost its subgraph");
  return v->exec->RunDirect(vs, n, per_job, in, out);
}

absl::Status HipModelExecutor::RunDirect(PreparedSubgraph* sg, int n, const std::vector<size_t>& per_job,
                                         const std::vector<const interface::ITensor*>& in,
                                         const std::vector<interface::ITensor*>& out) {
  // a graph that already holds its host copies, or intermediates a later
  // subgraph reads back, take the staged path
  if (!sg->extra_d2h.empty() || (use_graph_ && sg->graph && sg->io_in_graph))
    return absl::UnimplementedError("direct job batch I/O");
  const size_t ni = sg->inputs.size();
  for (size_t i = 0; i < in.size(); ++i)
    if (!in[i] || in[i]->GetBytes() != per_job[i / n]) return absl::InternalError("direct job batch I/O: input size");
  for (size_t i = 0; i < out.size(); ++i)
    if (out[i] && out[i]->GetBytes() != per_job[ni + i / n]) return absl::InternalError("direct job batch I/O: output size");
  int rc = bh_set_device(ordinal_);
  if (rc) return HipErr(rc, "hipSetDevice");
  if (use_graph_ && !sg->graph && sg->runs > 0) {  // kernels-only graph (variants stream their I/O)
    RETURN_STATUS_IF(CaptureGraph(sg));
    if (sg->io_in_graph) return absl::UnimplementedError("direct job batch I/O");
  }
  char* arena = static_cast<char*>(sg->arena->ptr());
  // jobs whose host tensors are adjacent (consecutive ring slots of one
  // page-locked block) go in one DMA: a run of slots s0..s1 of tensor k
  for (size_t k = 0; k < ni; ++k)
    for (int s0 = 0; s0 < n;) {
      const char* h0 = in[k * n + s0]->GetData();
      int s1 = s0 + 1;
      while (s1 < n && in[k * n + s1]->GetData() == h0 + (s1 - s0) * per_job[k]) ++s1;
      rc = bh_memcpy_h2d_async(arena + sg->offset.at(sg->inputs[k]) + s0 * per_job[k], h0, (s1 - s0) * per_job[k],
                               stream_);
      if (rc) return HipErr(rc, "H2D input");
      s0 = s1;
    }
  if (use_graph_ && sg->graph) {
    rc = bh_graph_launch(sg->graph, stream_);
    if (rc) return HipErr(rc, "graph launch");
  } else {
    RETURN_STATUS_IF(EnqueueLaunches(sg));
  }
  for (size_t k = 0; k < sg->outputs.size(); ++k) {
    const size_t pb = per_job[ni + k];
    for (int s0 = 0; s0 < n;) {
      interface::ITensor* o = out[k * n + s0];
      if (!o) {
        ++s0;
        continue;
      }
      char* h0 = o->GetData();
      int s1 = s0 + 1;
      while (s1 < n && out[k * n + s1] && out[k * n + s1]->GetData() == h0 + (s1 - s0) * pb) ++s1;
      rc = bh_memcpy_d2h_async(h0, arena + sg->offset.at(sg->outputs[k]) + s0 * pb, (s1 - s0) * pb, stream_);
      if (rc) return HipErr(rc, "D2H output");
      s0 = s1;
    }
  }
  RETURN_STATUS_IF(WaitPass(sg));
  ++sg->runs;
  return absl::OkStatus();
}


}  // namespace hip
}  // namespace band
