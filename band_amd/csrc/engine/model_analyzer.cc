#include "engine/model_analyzer.h"

#include <algorithm>
#include <cstdio>
#include <iterator>
#include <map>

#include "band/backend_factory.h"
#include "engine/worker.h"

namespace band {

// "{0-3,5,7-9}" (band/model_analyzer.cc:17-40)
std::string SetToString(const std::set<int>& set) {
  std::string out = "{";
  bool first = true;
  for (auto it = set.begin(); it != set.end();) {
    int lo = *it, hi = lo;
    auto next = std::next(it);
    while (next != set.end() && *next == hi + 1) {
      hi = *next;
      ++next;
    }
    out += (first ? "" : ",") + (lo == hi ? std::to_string(lo) : std::to_string(lo) + "-" + std::to_string(hi));
    first = false;
    it = next;
  }
  return out + "}";
}

std::string SubgraphDef::ToString() const {
  return "Index " + SetToString(unit_subgraph_indices) + " Ops " + SetToString(op_indices);
}

// availability table of unit subgraphs per worker, then merged subgraphs
// (band/model_analyzer.cc:49-120)
std::string SummarizeSubgraphs(const std::vector<SubgraphDef>& defs) {
  std::string out = "\n";
  std::set<int> units;
  int num_workers = 0;
  for (const auto& d : defs) {
    if (d.unit_subgraph_indices.size() == 1) units.insert(*d.unit_subgraph_indices.begin());
    num_workers = std::max(num_workers, d.worker_id + 1);
  }
  if (!units.empty()) {
    out += "UnitSubgraph Definitions\n";
    for (const auto& d : defs)
      if (d.unit_subgraph_indices.size() == 1 && d.worker_id == 0) out += "\t" + d.ToString() + "\n";
    out += "UnitSubgraph Availabilities\n";
    for (int w = 0; w < num_workers; ++w) {
      out += "\t Worker " + std::to_string(w) + "\t";
      for (int u : units) {
        bool has = false;
        for (const auto& d : defs)
          has |= d.worker_id == w && d.unit_subgraph_indices.size() == 1 && *d.unit_subgraph_indices.begin() == u;
        out += has ? "O\t" : "X\t";
      }
      out += "\n";
    }
  }
  bool merged = false;
  for (const auto& d : defs) merged |= d.unit_subgraph_indices.size() > 1;
  if (merged) {
    out += "MergedSubgraphs\n";
    for (int w = 0; w < num_workers; ++w)
      for (const auto& d : defs) {
        if (d.worker_id != w || d.unit_subgraph_indices.size() <= 1) continue;
        out += "\t Worker " + std::to_string(w) + "\t";
        for (int u : units) out += d.unit_subgraph_indices.count(u) ? "-\t" : " \t";
        out += "\n";
      }
  }
  return out;
}

ModelAnalyzer::ModelAnalyzer(const IEngine& engine, bool need_fallback_subgraph, SubgraphConfig subgraph_config,
                             interface::IModel* model, BackendType backend_type)
    : engine_(engine), need_fallback_subgraph_(need_fallback_subgraph), subgraph_config_(subgraph_config) {
  std::unique_ptr<interface::IModelExecutor> probe(
      BackendFactory::CreateModelExecutor(backend_type, model->GetId(), 0, DeviceFlag::kCPU));
  if (!probe) {
    init_status_ = absl::InternalError("no model executor for the backend");
    model_spec_ = std::make_shared<ModelSpec>();
    return;
  }
  auto spec = probe->InvestigateModelSpec(model);
  if (!spec.ok()) {
    init_status_ = spec.status();
    model_spec_ = std::make_shared<ModelSpec>();
    return;
  }
  model_spec_ = std::make_shared<ModelSpec>(spec.value());
}

ModelAnalyzer::ModelAnalyzer(const IEngine& engine, bool need_fallback_subgraph, SubgraphConfig subgraph_config,
                             const ModelSpec& spec)
    : engine_(engine),
      need_fallback_subgraph_(need_fallback_subgraph),
      subgraph_config_(subgraph_config),
      model_spec_(std::make_shared<ModelSpec>(spec)) {}

absl::StatusOr<std::pair<ModelSpec, std::vector<SubgraphDef>>> ModelAnalyzer::CreateSubgraphs() {
  if (!init_status_.ok()) return init_status_;
  std::vector<SubgraphDef> units;
  absl::Status s = GetUnitSubgraphs(units);
  if (!s.ok()) return s;

  std::vector<SubgraphDef> defs;
  switch (subgraph_config_.subgraph_preparation_type) {
    case SubgraphPreparationType::kFallbackPerWorker:
      for (WorkerId w = 0; w < static_cast<WorkerId>(engine_.GetNumWorkers()); ++w) {
        for (SubgraphDef& d : GetSubgraphsForFallbackOps(w)) {
          for (const SubgraphDef& u : units)
            if (std::includes(d.op_indices.begin(), d.op_indices.end(), u.op_indices.begin(), u.op_indices.end()))
              d.unit_subgraph_indices.insert(u.unit_subgraph_indices.begin(), u.unit_subgraph_indices.end());
          defs.push_back(std::move(d));
        }
      }
      break;
    case SubgraphPreparationType::kNoFallbackSubgraph:
    case SubgraphPreparationType::kUnitSubgraph: defs = units; break;
    case SubgraphPreparationType::kMergeUnitSubgraph: defs = MergeUnitSubgraphs(units); break;
    default: return absl::InternalError("Failed to create subgraph. Unsupported subgraph preparation type");
  }
  for (const SubgraphDef& d : defs) {
    if (d.unit_subgraph_indices.empty()) return absl::InternalError("subgraph " + d.ToString() + " has no unit");
    const int lo = *d.unit_subgraph_indices.begin(), hi = *d.unit_subgraph_indices.rbegin();
    if (hi - lo != static_cast<int>(d.unit_subgraph_indices.size()) - 1)
      return absl::InternalError("Failed to create subgraph. Unit subgraph indices in subgraph " + d.ToString() +
                                 " are not continous for model " + model_spec_->path);
  }
  return std::make_pair(*model_spec_, defs);
}

const std::set<int>& ModelAnalyzer::UnsupportedOps(DeviceFlag flag) const {
  static const std::set<int> kNone;
  auto it = model_spec_->unsupported_ops.find(flag);
  return it == model_spec_->unsupported_ops.end() ? kNone : it->second;
}

// band/model_analyzer.cc:305-475.  Deviation: an op's support on a worker
// is looked up by that worker's device flag (the reference indexes its
// per-worker map with the device flag value as if it were a worker id).
absl::Status ModelAnalyzer::GetUnitSubgraphs(std::vector<SubgraphDef>& unit_subgraphs) {
  const int num_workers = static_cast<int>(engine_.GetNumWorkers());
  const int num_ops = model_spec_->num_ops;
  unit_subgraphs.clear();
  if (!NeedFallbackSubgraph()) {
    std::set<int> all;
    for (int i = 0; i < num_ops; ++i) all.insert(i);
    for (WorkerId w = 0; w < num_workers; ++w)
      if (IsWorkerValid(w)) unit_subgraphs.push_back({w, all, {0}});
  } else {
    if (num_workers > static_cast<int>(BitMask().size()))
      return absl::InternalError("Number of workers is larger than BitMask");
    // device runs shorter than minimum_subgraph_size stay on the CPU
    std::map<WorkerId, std::set<int>> too_small;
    for (WorkerId w = 0; w < num_workers; ++w) {
      if (engine_.GetWorkerDevice(w) == DeviceFlag::kCPU) continue;
      for (const SubgraphDef& d : GetSubgraphsForFallbackOps(w))
        if (static_cast<int>(d.op_indices.size()) < subgraph_config_.minimum_subgraph_size)
          too_small[w].insert(d.op_indices.begin(), d.op_indices.end());
    }
    std::vector<BitMask> support(num_ops);
    for (int op = 0; op < num_ops; ++op)
      for (WorkerId w = 0; w < num_workers; ++w) {
        if (!IsWorkerValid(w)) continue;
        const DeviceFlag flag = engine_.GetWorkerDevice(w);
        if (flag == DeviceFlag::kCPU || (!UnsupportedOps(flag).count(op) && !too_small[w].count(op)))
          support[op].set(w);
      }
    std::set<int> resolved(model_spec_->input_tensors.begin(), model_spec_->input_tensors.end());
    std::set<int> remaining;
    for (int i = 0; i < num_ops; ++i) remaining.insert(i);
    int unit_index = 0;
    while (true) {
      // grow one unit: every resolvable op with the same worker support set
      std::set<int> unit_ops;
      BitMask workers;
      while (true) {
        std::vector<int> add;
        for (int op : remaining) {
          if (!IsResolved(resolved, op)) continue;
          if (workers.any() && workers != support[op]) continue;
          if (workers.none()) workers = support[op];
          add.push_back(op);
        }
        if (add.empty()) break;
        for (int op : add) {
          unit_ops.insert(op);
          remaining.erase(op);
          resolved.insert(model_spec_->op_output_tensors[op].begin(), model_spec_->op_output_tensors[op].end());
        }
      }
      if (unit_ops.empty()) break;
      for (WorkerId w = 0; w < num_workers; ++w)
        if (IsWorkerValid(w) && workers.test(w)) unit_subgraphs.push_back({w, unit_ops, {unit_index}});
      ++unit_index;
    }
    if (!remaining.empty()) return absl::InternalError("Not empty remaining ops");
  }

  std::set<int> unique;
  for (const auto& d : unit_subgraphs) unique.insert(*d.unit_subgraph_indices.begin());
  std::vector<std::set<int>> unit_ops(unique.size());
  for (const auto& d : unit_subgraphs) unit_ops[*d.unit_subgraph_indices.begin()] = d.op_indices;
  absl::Status s = model_spec_->SetUnitSubgraphs(unit_ops);
  if (!s.ok()) return s;

  for (size_t a = 0; a < unit_subgraphs.size(); ++a)
    for (size_t b = 0; b < unit_subgraphs.size(); ++b) {
      if (a == b) continue;
      const auto& l = unit_subgraphs[a];
      const auto& r = unit_subgraphs[b];
      if (*l.unit_subgraph_indices.begin() == *r.unit_subgraph_indices.begin()) {
        if (l.op_indices != r.op_indices)
          return absl::InternalError("Failed to create unit subgraph. Unit subgraph with same idx has different ops");
      } else {
        std::set<int> common;
        std::set_intersection(l.op_indices.begin(), l.op_indices.end(), r.op_indices.begin(), r.op_indices.end(),
                              std::inserter(common, common.begin()));
        if (!common.empty())
          return absl::InternalError("Failed to create unit subgraph. Units share operators " + SetToString(common));
      }
    }
  return absl::OkStatus();
}

// alternate maximal runs of device-supported ops and CPU-fallback ops in
// dependency order (band/model_analyzer.cc:484-606)
std::vector<SubgraphDef> ModelAnalyzer::GetSubgraphsForFallbackOps(WorkerId worker_id) {
  if (!engine_.GetWorker(worker_id) || !IsWorkerValid(worker_id)) return {};
  const int num_ops = model_spec_->num_ops;
  if (!NeedFallbackSubgraph()) {
    std::set<int> all;
    for (int i = 0; i < num_ops; ++i) all.insert(i);
    return {{worker_id, all, {0}}};
  }
  const DeviceFlag flag = engine_.GetWorkerDevice(worker_id);
  const std::set<int>& unsupported = UnsupportedOps(flag);
  std::vector<WorkerId> cpu_workers;
  for (WorkerId w = 0; w < static_cast<WorkerId>(engine_.GetNumWorkers()); ++w)
    if (engine_.GetWorkerDevice(w) == DeviceFlag::kCPU) cpu_workers.push_back(w);

  std::vector<SubgraphDef> out;
  std::set<int> resolved(model_spec_->input_tensors.begin(), model_spec_->input_tensors.end());
  std::set<int> remaining;
  for (int i = 0; i < num_ops; ++i) remaining.insert(i);
  bool fallback = false;
  while (!remaining.empty()) {
    std::set<int> run;
    for (bool found = true; found;) {
      found = false;
      for (auto it = remaining.begin(); it != remaining.end();) {
        const int op = *it;
        if (fallback != static_cast<bool>(unsupported.count(op)) || !IsResolved(resolved, op)) {
          ++it;
          continue;
        }
        found = true;
        run.insert(op);
        resolved.insert(model_spec_->op_output_tensors[op].begin(), model_spec_->op_output_tensors[op].end());
        it = remaining.erase(it);
      }
    }
    if (!run.empty()) {
      if (fallback && flag != DeviceFlag::kCPU) {
        for (WorkerId c : cpu_workers) out.push_back({c, run, {}});
      } else {
        out.push_back({worker_id, run, {}});
      }
    }
    fallback = !fallback;
  }
  return out;
}

// add every union of two subgraphs on one worker where the first's outputs
// cover the second's inputs, until nothing new appears
// (band/model_analyzer.cc:616-680)
std::vector<SubgraphDef> ModelAnalyzer::MergeUnitSubgraphs(const std::vector<SubgraphDef>& units) {
  std::vector<SubgraphDef> result = units;
  auto exists = [&](WorkerId w, const std::set<int>& ops) {
    for (const auto& d : result)
      if (d.worker_id == w && d.op_indices == ops) return true;
    return false;
  };
  for (bool added = true; added;) {
    added = false;
    std::vector<SubgraphDef> fresh;
    for (size_t a = 0; a < result.size(); ++a) {
      const std::set<int> outs = model_spec_->GetOutputTensors(result[a].op_indices);
      for (size_t b = 0; b < result.size(); ++b) {
        if (a == b || result[a].worker_id != result[b].worker_id) continue;
        const std::set<int> ins = model_spec_->GetPureInputTensors(result[b].op_indices);
        if (!std::includes(outs.begin(), outs.end(), ins.begin(), ins.end())) continue;
        std::set<int> ops = result[a].op_indices;
        ops.insert(result[b].op_indices.begin(), result[b].op_indices.end());
        std::set<int> idx = result[a].unit_subgraph_indices;
        idx.insert(result[b].unit_subgraph_indices.begin(), result[b].unit_subgraph_indices.end());
        if (!exists(result[a].worker_id, ops)) fresh.push_back({result[a].worker_id, ops, idx});
      }
    }
    for (auto& d : fresh) {
      if (exists(d.worker_id, d.op_indices)) continue;
      result.push_back(std::move(d));
      added = true;
    }
  }
  return result;
}

bool ModelAnalyzer::NeedFallbackSubgraph() const {
  return need_fallback_subgraph_ &&
         subgraph_config_.subgraph_preparation_type != SubgraphPreparationType::kNoFallbackSubgraph;
}

bool ModelAnalyzer::IsWorkerValid(WorkerId w) const {
  return !model_spec_->unavailable_devices.count(engine_.GetWorkerDevice(w));
}

bool ModelAnalyzer::IsResolved(const std::set<int>& resolved, int op) const {
  for (int t : model_spec_->op_input_tensors[op])
    if (!resolved.count(t)) return false;
  return true;
}

}  // namespace band
