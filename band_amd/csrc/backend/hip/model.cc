#include "backend/hip/model.h"

#include <cstdio>

namespace band {
namespace hip {

namespace {
std::atomic<uint64_t> g_next_serial{1};
}

HipModel::HipModel(ModelId id) : interface::IModel(id) {}

BackendType HipModel::GetBackendType() const { return BackendType::kTfLite; }

absl::Status HipModel::Load(std::vector<uint8_t>&& bytes) {
  initialized_ = false;
  bytes_ = std::move(bytes);
  std::string err;
  desc_ = TflModel();
  if (!desc_.Parse(bytes_.data(), bytes_.size(), &err)) return absl::InternalError("Invalid TFLite model: " + err);
  serial_ = g_next_serial.fetch_add(1);
  initialized_ = true;
  return absl::OkStatus();
}

absl::Status HipModel::FromPath(const char* filename) {
  path_ = filename ? filename : "";
  FILE* f = filename ? std::fopen(filename, "rb") : nullptr;
  if (!f) return absl::InternalError("Cannot load from file.");
  std::vector<uint8_t> bytes;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (n > 0) {
    bytes.resize(static_cast<size_t>(n));
    if (std::fread(bytes.data(), 1, bytes.size(), f) != bytes.size()) bytes.clear();
  }
  std::fclose(f);
  if (bytes.empty()) return absl::InternalError("Cannot load from file.");
  absl::Status s = Load(std::move(bytes));
  return s.ok() ? s : absl::InternalError("Cannot load from file.");
}

absl::Status HipModel::FromBuffer(const char* buffer, size_t buffer_size) {
  if (!buffer || buffer_size == 0) return absl::InternalError("Cannot load from buffer.");
  std::vector<uint8_t> bytes(reinterpret_cast<const uint8_t*>(buffer),
                             reinterpret_cast<const uint8_t*>(buffer) + buffer_size);
  absl::Status s = Load(std::move(bytes));
  return s.ok() ? s : absl::InternalError("Cannot load from buffer.");
}

absl::Status HipModel::CloneWithJobBatch(int batch, std::unique_ptr<HipModel>* out) const {
  if (!initialized_) return absl::InternalError("job batching: model not loaded");
  if (batch < 1) return absl::InternalError("job batching: batch must be >= 1");
  for (const TflOperator& op : desc_.ops) {
    if (op.builtin == kTflCustom) return absl::InternalError("job batching: CUSTOM op " + op.custom_code);
    if (op.builtin == kTflConcatenation && op.options.valid() && !op.outputs.empty()) {
      const int rank = static_cast<int>(desc_.tensors[op.outputs[0]].shape.size());
      int axis = op.options.Int(0, 0);
      if (axis < 0) axis += rank;
      if (axis == 0) return absl::InternalError("job batching: CONCATENATION on the batch axis");
    }
  }
  for (const TflTensor& t : desc_.tensors)
    if (!t.is_const() && (t.shape.empty() || t.shape[0] != 1))
      return absl::InternalError("job batching: tensor '" + t.name + "' has no unit batch dimension");
  auto m = std::make_unique<HipModel>(id_);
  m->path_ = path_;
  std::vector<uint8_t> bytes = bytes_;
  absl::Status loaded = m->Load(std::move(bytes));
  if (!loaded.ok()) return loaded;
  for (TflTensor& t : m->desc_.tensors)
    if (!t.is_const()) t.shape[0] = batch;
  m->serial_ = serial_;
  *out = std::move(m);
  return absl::OkStatus();
}

}  // namespace hip
}  // namespace band
