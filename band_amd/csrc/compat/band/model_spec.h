// Stand-in for band/model_spec.h: the ModelSpec that
// IModelExecutor::InvestigateModelSpec returns (band/model_spec.h:20-79).
#pragma once
#include <map>
#include <set>
#include <string>
#include <vector>

#include "absl/status/status.h"
#include "band/common.h"

namespace band {
class ModelSpec {
 public:
  ModelSpec() : ModelSpec(0, 0, {}, {}, {}, {}, {}, {}, {}) {}
  ModelSpec(int num_ops, int num_tensors, std::vector<DataType> tensor_types,
            std::set<int> input_tensors, std::set<int> output_tensors,
            std::vector<std::set<int>> op_input_tensors,
            std::vector<std::set<int>> op_output_tensors,
            std::map<DeviceFlag, std::set<int>> unsupported_ops,
            std::set<DeviceFlag> unavailable_devices)
      : num_ops(num_ops), num_tensors(num_tensors), tensor_types(tensor_types),
        input_tensors(input_tensors), output_tensors(output_tensors),
        op_input_tensors(op_input_tensors), op_output_tensors(op_output_tensors),
        unsupported_ops(unsupported_ops), unavailable_devices(unavailable_devices) {}

  // non-constant inputs of `op_indices` minus tensors produced inside them
  std::set<int> GetPureInputTensors(const std::set<int>& op_indices) const;
  // every non-constant output of `op_indices`
  std::set<int> GetOutputTensors(const std::set<int>& op_indices) const;

  // Unit subgraphs (band/model_spec.cc:53-118): the model_analyzer's
  // partition of the ops; unit i depends on unit j < i when i consumes a
  // tensor j produces.
  absl::Status SetUnitSubgraphs(std::vector<std::set<int>> ops);
  size_t GetNumUnitSubgraphs() const { return unit_subgraph_ops.size(); }
  const std::set<int>& GetUnitSubgraphOps(size_t index) const { return unit_subgraph_ops[index]; }
  const BitMask& GetUnitSubgraphDependency(size_t index) const { return unit_subgraph_dependencies[index]; }
  // dependencies of a set of units on units outside the set
  BitMask GetUnitSubgraphDependency(const BitMask& unit_subgraphs) const;

  const int num_ops;
  const int num_tensors;
  const std::vector<DataType> tensor_types;
  const std::set<int> input_tensors;
  const std::set<int> output_tensors;
  const std::vector<std::set<int>> op_input_tensors;
  const std::vector<std::set<int>> op_output_tensors;
  const std::map<DeviceFlag, std::set<int>> unsupported_ops;
  const std::set<DeviceFlag> unavailable_devices;
  std::string path;

 private:
  std::vector<std::set<int>> unit_subgraph_ops;
  std::vector<BitMask> unit_subgraph_dependencies;
};
}  // namespace band
