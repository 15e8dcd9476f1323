#include "band/model_spec.h"

namespace band {
std::set<int> ModelSpec::GetPureInputTensors(const std::set<int>& ops) const {
  std::set<int> in;
  for (int op : ops) in.insert(op_input_tensors[op].begin(), op_input_tensors[op].end());
  for (int op : ops)
    for (int t : op_output_tensors[op]) in.erase(t);
  return in;
}

std::set<int> ModelSpec::GetOutputTensors(const std::set<int>& ops) const {
  std::set<int> out;
  for (int op : ops) out.insert(op_output_tensors[op].begin(), op_output_tensors[op].end());
  return out;
}

absl::Status ModelSpec::SetUnitSubgraphs(std::vector<std::set<int>> ops) {
  std::set<int> covered;
  for (const auto& u : ops) covered.insert(u.begin(), u.end());
  if ((int)covered.size() != num_ops || (num_ops > 0 && *covered.rbegin() != num_ops - 1))
    return absl::InternalError("Failed to set unit subgraphs. Unit subgraph does not covers all operators");
  unit_subgraph_ops = std::move(ops);
  const size_t n = unit_subgraph_ops.size();
  unit_subgraph_dependencies.assign(n, BitMask());
  std::vector<std::set<int>> produced(n), consumed(n);
  for (size_t u = 0; u < n; ++u) {
    produced[u] = GetOutputTensors(unit_subgraph_ops[u]);
    consumed[u] = GetPureInputTensors(unit_subgraph_ops[u]);
  }
  for (size_t child = 0; child < n; ++child)
    for (size_t parent = 0; parent < child; ++parent)
      for (int t : consumed[child])
        if (produced[parent].count(t)) {
          unit_subgraph_dependencies[child].set(parent);
          break;
        }
  return absl::OkStatus();
}

BitMask ModelSpec::GetUnitSubgraphDependency(const BitMask& units) const {
  BitMask deps;
  for (size_t i = 0; i < GetNumUnitSubgraphs(); ++i)
    if (units.test(i)) deps |= unit_subgraph_dependencies[i];
  return deps & ~units;
}
}  // namespace band
