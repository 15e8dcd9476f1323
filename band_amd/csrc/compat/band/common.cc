// Implementations for the stand-in band/common.h (see that header).
#include "band/common.h"

#include <functional>

namespace band {

size_t GetDataTypeBytes(DataType type) {
  switch (type) {
    case DataType::kFloat32: case DataType::kInt32: return 4;
    case DataType::kUInt8: case DataType::kInt8: case DataType::kBool: return 1;
    case DataType::kInt64: case DataType::kFloat64: case DataType::kComplex64: return 8;
    case DataType::kInt16: case DataType::kFloat16: return 2;
    default: return 0;
  }
}

template <> size_t EnumLength<BackendType>() { return 1; }
template <> size_t EnumLength<DataType>() { return static_cast<size_t>(DataType::kFloat64) + 1; }
template <> size_t EnumLength<DeviceFlag>() { return static_cast<size_t>(DeviceFlag::kNPU) + 1; }
template <> size_t EnumLength<QuantizationType>() { return 2; }
template <> size_t EnumLength<SchedulerType>() {
  return static_cast<size_t>(SchedulerType::kHeterogeneousEarliestFinishTimeReserved) + 1;
}
template <> size_t EnumLength<SubgraphPreparationType>() { return 4; }
template <> size_t EnumLength<JobStatus>() { return static_cast<size_t>(JobStatus::kInvokeFailure) + 1; }
template <> size_t EnumLength<CPUMaskFlag>() { return 4; }

template <> const char* ToString(BackendType) { return "tfl"; }
template <> const char* ToString(DataType t) {
  static const char* names[] = {"NoType", "Float32", "Int32", "UInt8", "Int64", "String",
                                "Bool", "Int16", "Complex64", "Int8", "Float16", "Float64"};
  size_t i = static_cast<size_t>(t);
  return i < 12 ? names[i] : "Unknown";
}
template <> const char* ToString(DeviceFlag t) {
  static const char* names[] = {"CPU", "GPU", "DSP", "NPU"};
  size_t i = static_cast<size_t>(t);
  return i < 4 ? names[i] : "Unknown";
}
template <> const char* ToString(QuantizationType t) {
  return t == QuantizationType::kAffineQuantization ? "AffineQuantization" : "NoQuantization";
}

template <> const char* ToString(SchedulerType t) {
  static const char* names[] = {"fixed_worker",
                                "round_robin",
                                "shortest_expected_latency",
                                "fixed_worker_global_queue",
                                "heterogeneous_earliest_finish_time",
                                "least_slack_time_first",
                                "heterogeneous_earliest_finish_time_reserved"};
  size_t i = static_cast<size_t>(t);
  return i < 7 ? names[i] : "Unknown scheduler type";
}
template <> const char* ToString(SubgraphPreparationType t) {
  static const char* names[] = {"no_fallback_subgraph", "fallback_per_worker", "unit_subgraph",
                                "merge_unit_subgraph"};
  size_t i = static_cast<size_t>(t);
  return i < 4 ? names[i] : "Unknown subgraph preparation type";
}
template <> const char* ToString(JobStatus t) {
  static const char* names[] = {"EnqueueFailed",     "Queued",           "Success",      "SLOViolation",
                                "InputCopyFailure", "OutputCopyFailure", "InvokeFailure"};
  size_t i = static_cast<size_t>(t);
  return i < 7 ? names[i] : "Unknown job status";
}
template <> const char* ToString(CPUMaskFlag t) {
  static const char* names[] = {"ALL", "LITTLE", "BIG", "PRIMARY"};
  size_t i = static_cast<size_t>(t);
  return i < 4 ? names[i] : "Unknown CPU mask";
}

std::string IndexSetToString(const std::set<int>& indices) {
  std::string s;
  for (int i : indices) s += (s.empty() ? "" : ",") + std::to_string(i);
  return s;
}

std::size_t JobIdBitMaskHash::operator()(const std::pair<int, BitMask>& p) const {
  return std::hash<int>()(p.first) ^ std::hash<unsigned long long>()(p.second.to_ullong());
}

SubgraphKey::SubgraphKey() {}
SubgraphKey::SubgraphKey(ModelId m, WorkerId w, std::set<int> units) : model_id(m), worker_id(w) {
  for (int u : units) unit_indices.set(u);
}
bool SubgraphKey::operator<(const SubgraphKey& k) const {
  if (model_id != k.model_id) return model_id < k.model_id;
  if (worker_id != k.worker_id) return worker_id < k.worker_id;
  return unit_indices.to_ullong() < k.unit_indices.to_ullong();
}
bool SubgraphKey::operator==(const SubgraphKey& k) const {
  return model_id == k.model_id && worker_id == k.worker_id && unit_indices == k.unit_indices;
}
bool SubgraphKey::operator!=(const SubgraphKey& k) const { return !(*this == k); }
const BitMask& SubgraphKey::GetUnitIndices() const { return unit_indices; }
std::set<int> SubgraphKey::GetUnitIndicesSet() const {
  std::set<int> s;
  for (size_t i = 0; i < unit_indices.size(); ++i)
    if (unit_indices.test(i)) s.insert(static_cast<int>(i));
  return s;
}
std::string SubgraphKey::GetUnitIndicesString() const { return IndexSetToString(GetUnitIndicesSet()); }
std::string SubgraphKey::ToString() const {
  return "Model id " + std::to_string(model_id) + " Worker id " + std::to_string(worker_id) +
         " Unit indices (" + GetUnitIndicesString() + ")";
}
bool SubgraphKey::IsValid() const { return model_id != -1 && worker_id != -1; }

std::size_t SubgraphHash::operator()(const SubgraphKey& p) const {
  std::size_t h = std::hash<int>()(p.GetModelId());
  h ^= std::hash<int>()(p.GetWorkerId()) + 0x9e3779b9 + (h << 6) + (h >> 2);
  h ^= std::hash<unsigned long long>()(p.GetUnitIndices().to_ullong()) + 0x9e3779b9 + (h << 6) + (h >> 2);
  return h;
}

}  // namespace band
