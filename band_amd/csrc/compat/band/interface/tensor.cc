// Default ITensor helpers with the reference's semantics
// (band/interface/tensor.cc:24-69): equality = same type and dims; copy =
// check then memcpy of GetBytes().
#include "band/interface/tensor.h"

#include <cstring>

namespace band {
namespace interface {
bool ITensor::operator==(const ITensor& rhs) const {
  return GetType() == rhs.GetType() && GetDimsVector() == rhs.GetDimsVector();
}
bool ITensor::operator!=(const ITensor& rhs) const { return !(*this == rhs); }
size_t ITensor::GetBytes() const { return GetDataTypeBytes(GetType()) * GetNumElements(); }
size_t ITensor::GetNumElements() const {
  size_t n = 1;
  for (size_t i = 0; i < GetNumDims(); ++i) n *= static_cast<size_t>(GetDims()[i]);
  return n;
}
std::vector<int> ITensor::GetDimsVector() const { return std::vector<int>(GetDims(), GetDims() + GetNumDims()); }
absl::Status ITensor::CopyDataFrom(const ITensor& rhs) {
  if (*this != rhs) return absl::InternalError("");
  std::memcpy(GetData(), rhs.GetData(), GetBytes());
  return absl::OkStatus();
}
absl::Status ITensor::CopyDataFrom(const ITensor* rhs) {
  if (!rhs) return absl::InternalError("Tried to copy null tensor");
  return CopyDataFrom(*rhs);
}
}  // namespace interface
}  // namespace band
