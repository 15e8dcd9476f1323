// Stand-in for the subset of Band's core types (band/common.h) that the
// backend plugin API touches.  Values and semantics follow the reference:
//   DataType == TfLiteType numbering        (band/common.h:115-128)
//   DeviceFlag {kCPU,kGPU,kDSP,kNPU}         (band/common.h:163-168)
//   SubgraphKey = (model, worker, 64-bit unit mask)  (band/common.h:293-319)
// Inside a Band build the real header replaces this file; this backend only
// relies on the declarations below.
#pragma once

#include <bitset>
#include <cstddef>
#include <cstdint>
#include <list>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

namespace band {

typedef int WorkerId;
typedef int ModelId;
typedef int JobId;
using BitMask = std::bitset<64>;

template <typename EnumType>
size_t EnumLength();
template <typename EnumType>
const char* ToString(EnumType t);

// String -> enum by scanning ToString over the enum's range; an unknown
// string falls back to the first value, as the reference does
// (band/common.h:61-71: e.g. "fixed_device" -> kFixedWorker).
template <typename EnumType>
EnumType FromString(const std::string& str) {
  for (size_t i = 0; i < EnumLength<EnumType>(); i++) {
    EnumType t = static_cast<EnumType>(i);
    if (str == ToString(t)) return t;
  }
  return static_cast<EnumType>(0);
}

enum class BackendType : size_t { kTfLite = 0 };

enum class CPUMaskFlag : size_t { kAll = 0, kLittle, kBig, kPrimary };

enum class DataType : size_t {
  kNoType = 0, kFloat32, kInt32, kUInt8, kInt64, kString, kBool, kInt16,
  kComplex64, kInt8, kFloat16, kFloat64,
};

size_t GetDataTypeBytes(DataType type);

enum class DeviceFlag : size_t { kCPU = 0, kGPU, kDSP, kNPU };

enum class QuantizationType : size_t { kNoQuantization = 0, kAffineQuantization };

// Harness enums (band/common.h:75-200); numbering matches the C API's
// BandSchedulerType / BandWorkerType / BandSubgraphPreparationType.
enum class SchedulerType : size_t {
  kFixedWorker = 0, kRoundRobin, kShortestExpectedLatency, kFixedWorkerGlobalQueue,
  kHeterogeneousEarliestFinishTime, kLeastSlackTimeFirst, kHeterogeneousEarliestFinishTimeReserved,
};
enum class WorkerType : size_t { kDeviceQueue = 1 << 0, kGlobalQueue = 1 << 1 };
enum class SubgraphPreparationType : size_t {
  kNoFallbackSubgraph = 0, kFallbackPerWorker, kUnitSubgraph, kMergeUnitSubgraph,
};
enum class JobStatus : size_t {
  kEnqueueFailed = 0, kQueued, kSuccess, kSLOViolation, kInputCopyFailure, kOutputCopyFailure, kInvokeFailure,
};

template <> size_t EnumLength<BackendType>();
template <> size_t EnumLength<DataType>();
template <> size_t EnumLength<DeviceFlag>();
template <> size_t EnumLength<QuantizationType>();
template <> size_t EnumLength<SchedulerType>();
template <> size_t EnumLength<SubgraphPreparationType>();
template <> size_t EnumLength<JobStatus>();
template <> size_t EnumLength<CPUMaskFlag>();
template <> const char* ToString(BackendType t);
template <> const char* ToString(DataType t);
template <> const char* ToString(DeviceFlag t);
template <> const char* ToString(QuantizationType t);
template <> const char* ToString(SchedulerType t);
template <> const char* ToString(SubgraphPreparationType t);
template <> const char* ToString(JobStatus t);
template <> const char* ToString(CPUMaskFlag t);

struct AffineQuantizationParams {
  std::vector<float> scale;
  std::vector<int32_t> zero_point;
  int32_t quantized_dimension;
};

class Quantization {
 public:
  Quantization(QuantizationType type, void* params) : type_(type), params_(params) {}
  QuantizationType GetType() { return type_; }
  void* GetParams() { return params_; }
  void SetParams(void* params) { params_ = params; }

 private:
  QuantizationType type_;
  void* params_;
};

class SubgraphKey {
 public:
  SubgraphKey();
  SubgraphKey(ModelId model_id, WorkerId worker_id, std::set<int> unit_indices = {});
  bool operator<(const SubgraphKey& key) const;
  bool operator==(const SubgraphKey& key) const;
  bool operator!=(const SubgraphKey& key) const;
  ModelId GetModelId() const { return model_id; }
  WorkerId GetWorkerId() const { return worker_id; }
  const BitMask& GetUnitIndices() const;
  std::set<int> GetUnitIndicesSet() const;
  std::string GetUnitIndicesString() const;
  std::string ToString() const;
  bool IsValid() const;

 private:
  ModelId model_id = -1;
  WorkerId worker_id = -1;
  BitMask unit_indices;
};

struct SubgraphHash {
  std::size_t operator()(const SubgraphKey& p) const;
};

// "1,2,3" (band/common.cc:428-437)
std::string IndexSetToString(const std::set<int>& indices);

// One request (or the remaining part of a split request) moving through
// planner -> worker (band/common.h:333-378).  Times are NowMicros().
struct Job {
  Job() : model_id(-1) {}
  explicit Job(ModelId model_id) : model_id(model_id) {}
  Job(ModelId model_id, int64_t slo) : model_id(model_id), slo_us(slo) {}

  ModelId model_id;
  int input_handle = -1;
  int output_handle = -1;
  JobId job_id = -1;
  std::string model_fname;
  bool require_callback = true;
  int64_t enqueue_time = 0;
  int64_t invoke_time = 0;
  int64_t end_time = 0;
  int64_t profiled_execution_time = 0;
  int64_t expected_execution_time = 0;
  int64_t expected_latency = 0;
  int64_t slo_us = 0;
  WorkerId target_worker_id = -1;
  JobStatus status = JobStatus::kQueued;
  SubgraphKey subgraph_key;
  std::vector<Job> following_jobs;
  BitMask resolved_unit_subgraphs;
  std::list<SubgraphKey> previous_subgraph_keys;
  // Harness addition: bytes of the tensors earlier subgraphs of this job
  // produced, captured right after they ran.  The reference re-reads the
  // previous executor's live views when the next subgraph starts
  // (band/engine.cc:1262-1285), by which time that worker may already have
  // run the same subgraph for another request and overwritten them.
  std::shared_ptr<std::map<int, std::vector<char>>> intermediates;
};

struct JobIdBitMaskHash {
  std::size_t operator()(const std::pair<int, BitMask>& p) const;
};

}  // namespace band
