// Job batching: an optional capability of the HIP executor, used by this
// repo's Band-compatible harness (engine/worker.cc DeviceQueueWorker).  Not
// part of the reference's interface (band/interface/ has no batching;
// band/worker.cc:222-323 runs one job per ExecuteSubgraph), so it lives with
// the backend: HipModelExecutor also derives from this class, and an engine
// that wants batched passes finds it with dynamic_cast.  Band's own engine
// never calls it, and the executor behaves exactly as before for
// ExecuteSubgraph.
//
// A job batch is n whole-model jobs of one subgraph run as one pass over a
// subgraph prepared with a leading batch of B >= n (slots n..B-1 carry stale
// bytes and their outputs are ignored).  Slot s of a boundary tensor is the
// s-th contiguous batch-1 image of that tensor, so a slot view has the
// batch-1 tensor's type, dims and bytes and Band's tensor copies
// (band/interface/tensor.cc:55-69) apply to it unchanged.
#pragma once

#include <memory>
#include <vector>

#include "absl/status/status.h"
#include "band/common.h"
#include "band/interface/model.h"
#include "band/interface/tensor.h"
#include "band/interface/tensor_view.h"

namespace band {
namespace hip {

class IJobBatching {
 public:
  virtual ~IJobBatching() = default;
  // Prepares batch variants of `key` (already prepared by PrepareSubgraph)
  // for up to `max_batch` jobs.  An error leaves the subgraph unbatched.
  virtual absl::Status PrepareJobBatches(interface::IModel* model, const SubgraphKey& key, int max_batch) = 0;
  // 1 when `key` has no batch variants.
  virtual int MaxJobBatch(const SubgraphKey& key) const = 0;
  // View of slot `slot` (< n) of boundary tensor `index` in the variant
  // that runs n jobs; valid until the executor is destroyed.
  virtual std::shared_ptr<interface::ITensorView> GetJobSlotView(const SubgraphKey& key, int index, int n, int slot) = 0;
  // Runs n (1 <= n <= MaxJobBatch) jobs whose inputs were written through
  // the slot views; synchronous like ExecuteSubgraph.
  virtual absl::Status ExecuteJobBatch(const SubgraphKey& key, int n) = 0;
  // Optional: runs n (>= 2) jobs reading job s's input tensor k (the order
  // of GetInputs(key)) from in[k * n + s] and writing its output tensor k
  // (GetOutputs(key) order) into out[k * n + s] (nullptr: not wanted) - host
  // tensors, typically the request rings' slots in page-locked memory - with
  // no staging through the slot views; synchronous.  Unimplemented: the
  // caller uses the slot views and ExecuteJobBatch instead.
  virtual absl::Status ExecuteJobBatchDirect(const SubgraphKey& key, int n, const std::vector<const interface::ITensor*>& in,
                                             const std::vector<interface::ITensor*>& out) {
    return absl::UnimplementedError("direct job batch I/O");
  }
};

}  // namespace hip
}  // namespace band
