// HipModel: the IModel of the HIP backend (replaces band/backend/tfl/model.{h,cc}:
// TfLiteModel::FromPath/FromBuffer, band/backend/tfl/model.cc:25-39).
// Owns the .tflite bytes and the parsed primary subgraph.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <vector>

#include "absl/status/status.h"
#include <string>
#include "backend/hip/tflite_reader.h"
#include "band/interface/model.h"

namespace band {
namespace hip {

class HipModel : public interface::IModel {
 public:
  explicit HipModel(ModelId id);
  BackendType GetBackendType() const override;
  absl::Status FromPath(const char* filename) override;
  absl::Status FromBuffer(const char* buffer, size_t buffer_size) override;
  bool IsInitialized() const override { return initialized_; }

  const TflModel& desc() const { return desc_; }
  // process-unique id of the loaded contents (keys the device weight cache)
  uint64_t serial() const { return serial_; }

  // Job batching (HipModelExecutor::PrepareJobBatches): a copy of this model
  // whose activation tensors carry a leading batch of `batch` jobs.  Every
  // non-constant tensor must have dim 0 == 1 and no op may mix the batch
  // axis (CONCATENATION on axis 0, CUSTOM ops); otherwise an error says why.
  // The copy keeps this model's serial, so device weights stay shared.
  absl::Status CloneWithJobBatch(int batch, std::unique_ptr<HipModel>* out) const;

 private:
  absl::Status Load(std::vector<uint8_t>&& bytes);
  std::vector<uint8_t> bytes_;
  TflModel desc_;
  bool initialized_ = false;
  uint64_t serial_ = 0;
};

}  // namespace hip
}  // namespace band
