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

enum class BackendType : size_t { kTfLite = 0 };

enum class CPUMaskFlag : size_t { kAll = 0, kLittle, kBig, kPrimary };

enum class DataType : size_t {
  kNoType = 0, kFloat32, kInt32, kUInt8, kInt64, kString, kBool, kInt16,
  kComplex64, kInt8, kFloat16, kFloat64,
};

size_t GetDataTypeBytes(DataType type);

enum class DeviceFlag : size_t { kCPU = 0, kGPU, kDSP, kNPU };

enum class QuantizationType : size_t { kNoQuantization = 0, kAffineQuantization };

template <> size_t EnumLength<BackendType>();
template <> size_t EnumLength<DataType>();
template <> size_t EnumLength<DeviceFlag>();
template <> size_t EnumLength<QuantizationType>();
template <> const char* ToString(BackendType t);
template <> const char* ToString(DataType t);
template <> const char* ToString(DeviceFlag t);
template <> const char* ToString(QuantizationType t);

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

}  // namespace band
