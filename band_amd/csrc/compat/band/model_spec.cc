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
}  // namespace band
