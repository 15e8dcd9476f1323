// Band backend plugin API (stand-in; signatures of band/interface/tensor.h:27-50).
#pragma once
#include <vector>

#include "absl/status/status.h"
#include "band/common.h"

namespace band {
namespace interface {
struct ITensor {
 public:
  virtual ~ITensor() = default;
  virtual DataType GetType() const = 0;
  virtual void SetType(DataType type) = 0;
  virtual const char* GetData() const = 0;
  virtual char* GetData() = 0;
  virtual const int* GetDims() const = 0;
  virtual size_t GetNumDims() const = 0;
  virtual void SetDims(const std::vector<int>& dims) = 0;
  virtual const char* GetName() const = 0;
  virtual Quantization GetQuantization() const = 0;
  virtual absl::Status SetQuantization(Quantization quantization) = 0;
  bool operator==(const ITensor& rhs) const;
  bool operator!=(const ITensor& rhs) const;
  virtual size_t GetBytes() const;
  size_t GetNumElements() const;
  std::vector<int> GetDimsVector() const;
  absl::Status CopyDataFrom(const ITensor& rhs);
  absl::Status CopyDataFrom(const ITensor* rhs);
};
}  // namespace interface
}  // namespace band
