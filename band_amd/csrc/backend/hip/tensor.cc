#include "backend/hip/tensor.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace band {
namespace hip {

TensorMeta::~TensorMeta() {
  if (quant) {
    std::free(quant->scale);
    std::free(quant->zero_point);
    delete quant;
  }
}

void TensorMeta::SetQuant(const std::vector<float>& scale, const std::vector<int64_t>& zp, int qdim) {
  if (scale.empty()) return;
  quant = new QAffine();
  const int n = static_cast<int>(scale.size());
  quant->scale = static_cast<QFloatArray*>(std::calloc(1, sizeof(int) + sizeof(float) * n + sizeof(float)));
  quant->zero_point = static_cast<QIntArray*>(std::calloc(1, sizeof(int) + sizeof(int) * n + sizeof(int)));
  quant->scale->size = n;
  quant->zero_point->size = n;
  for (int i = 0; i < n; ++i) {
    quant->scale->data[i] = scale[i];
    quant->zero_point->data[i] = i < static_cast<int>(zp.size()) ? static_cast<int>(zp[i]) : 0;
  }
  quant->quantized_dimension = qdim;
}

void HipTensorView::SetDims(const std::vector<int>& dims) {
  // like TfLiteTensorView::SetDims: only same-rank updates are applied
  if (dims.size() == meta_->dims.size()) meta_->dims = dims;
}

Quantization HipTensorView::GetQuantization() const {
  return Quantization(meta_->quant ? QuantizationType::kAffineQuantization : QuantizationType::kNoQuantization,
                      meta_->quant);
}

absl::Status HipTensorView::SetQuantization(Quantization q) {
  if (q.GetType() != QuantizationType::kAffineQuantization) return absl::OkStatus();
  auto* in = static_cast<AffineQuantizationParams*>(q.GetParams());
  if (!in || !meta_->quant) return absl::OkStatus();
  const size_t ns = std::min<size_t>(in->scale.size(), meta_->quant->scale->size);
  const size_t nz = std::min<size_t>(in->zero_point.size(), meta_->quant->zero_point->size);
  std::memcpy(meta_->quant->scale->data, in->scale.data(), ns * sizeof(float));
  std::memcpy(meta_->quant->zero_point->data, in->zero_point.data(), nz * sizeof(int32_t));
  meta_->quant->quantized_dimension = in->quantized_dimension;
  return absl::OkStatus();
}

}  // namespace hip
}  // namespace band
