// HipTensorView: the ITensorView of the HIP backend (replaces
// band/backend/tfl/tensor.{h,cc}, TfLiteTensorView :24-87).
//
// Band memcpy's job inputs/outputs through GetData() (band/interface/tensor.cc:55-61,
// band/engine.cc:1262-1365), so a view's data pointer is the executor's
// host-pinned mirror of the tensor; the executor moves it to/from HBM inside
// ExecuteSubgraph.  The view aliases executor-owned metadata and stays valid
// for the executor's lifetime.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "band/interface/tensor_view.h"

namespace band {
namespace hip {

// Binary layout of TfLiteFloatArray / TfLiteIntArray / TfLiteAffineQuantization:
// Band reads GetQuantization().params as a TfLiteAffineQuantization*
// (band/tensor.cc:53-81), so the HIP backend hands out the same layout.
struct QFloatArray {
  int size;
  float data[1];
};
struct QIntArray {
  int size;
  int data[1];
};
struct QAffine {
  QFloatArray* scale;
  QIntArray* zero_point;
  int32_t quantized_dimension;
};

struct TensorMeta {
  DataType type = DataType::kNoType;
  std::vector<int> dims;
  std::string name;
  size_t bytes = 0;
  QAffine* quant = nullptr;  // owned, null if not quantised
  TensorMeta() = default;
  TensorMeta(const TensorMeta&) = delete;
  TensorMeta& operator=(const TensorMeta&) = delete;
  ~TensorMeta();
  void SetQuant(const std::vector<float>& scale, const std::vector<int64_t>& zp, int qdim);
};

class HipTensorView : public interface::ITensorView {
 public:
  HipTensorView(TensorMeta* meta, char* data) : meta_(meta), data_(data) {}
  BackendType GetBackendType() const override { return BackendType::kTfLite; }
  DataType GetType() const override { return meta_->type; }
  void SetType(DataType type) override { meta_->type = type; }
  const char* GetData() const override { return data_; }
  char* GetData() override { return data_; }
  const int* GetDims() const override { return meta_->dims.data(); }
  size_t GetNumDims() const override { return meta_->dims.size(); }
  void SetDims(const std::vector<int>& dims) override;
  size_t GetBytes() const override { return meta_->bytes; }
  const char* GetName() const override { return meta_->name.c_str(); }
  Quantization GetQuantization() const override;
  absl::Status SetQuantization(Quantization quantization) override;

 private:
  TensorMeta* meta_;
  char* data_;
};

}  // namespace hip
}  // namespace band
