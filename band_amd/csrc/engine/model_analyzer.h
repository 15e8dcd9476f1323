// Model analyzer (band/model_analyzer.h/.cc): partitions a model into unit
// subgraphs - maximal runs of ops supported by the same set of workers - and
// derives the subgraphs each worker prepares, according to
// SubgraphPreparationType:
//   kNoFallbackSubgraph / kUnitSubgraph  the unit subgraphs
//   kMergeUnitSubgraph                   + every chain of units on one worker
//   kFallbackPerWorker                   per worker: alternating device /
//                                        CPU-fallback op runs
// Schedulers that do not need fallback subgraphs get the whole model as a
// single unit on every valid worker.
#pragma once
#include <memory>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "absl/status/statusor.h"
#include "band/interface/model.h"
#include "band/model_spec.h"
#include "engine/config.h"
#include "engine/engine_interface.h"

namespace band {

struct SubgraphDef {
  WorkerId worker_id;
  std::set<int> op_indices;
  std::set<int> unit_subgraph_indices;
  std::string ToString() const;
};

std::string SetToString(const std::set<int>& set);
std::string SummarizeSubgraphs(const std::vector<SubgraphDef>& subgraph_defs);

class ModelAnalyzer {
 public:
  // investigates `model` with a worker-0 / kCPU executor, as the reference
  // does (band/model_analyzer.cc:227-233)
  ModelAnalyzer(const IEngine& engine, bool need_fallback_subgraph, SubgraphConfig subgraph_config,
                interface::IModel* model, BackendType backend_type);
  // from an already investigated spec (tests, and the engine when the spec
  // is known)
  ModelAnalyzer(const IEngine& engine, bool need_fallback_subgraph, SubgraphConfig subgraph_config,
                const ModelSpec& spec);

  absl::StatusOr<std::pair<ModelSpec, std::vector<SubgraphDef>>> CreateSubgraphs();
  const absl::Status& init_status() const { return init_status_; }

 private:
  absl::Status GetUnitSubgraphs(std::vector<SubgraphDef>& unit_subgraphs);
  std::vector<SubgraphDef> GetSubgraphsForFallbackOps(WorkerId worker_id);
  std::vector<SubgraphDef> MergeUnitSubgraphs(const std::vector<SubgraphDef>& unit_subgraphs);
  bool NeedFallbackSubgraph() const;
  bool IsWorkerValid(WorkerId worker_id) const;
  bool IsResolved(const std::set<int>& resolved_tensors, int op_index) const;
  const std::set<int>& UnsupportedOps(DeviceFlag flag) const;

  const IEngine& engine_;
  const bool need_fallback_subgraph_;
  const SubgraphConfig subgraph_config_;
  std::shared_ptr<ModelSpec> model_spec_;
  absl::Status init_status_;
};

}  // namespace band
