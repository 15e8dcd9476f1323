#include "engine/tensor.h"

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "engine/logger.h"

namespace band {

namespace {
// TfLiteFloatArray / TfLiteIntArray / TfLiteAffineQuantization layout
struct FArr {
  int size;
  float data[1];
};
struct IArr {
  int size;
  int data[1];
};
struct Affine {
  FArr* scale;
  IArr* zero_point;
  int32_t quantized_dimension;
};

Affine* CloneAffine(const Affine* src) {
  if (!src) return nullptr;
  auto* a = static_cast<Affine*>(std::calloc(1, sizeof(Affine)));
  a->quantized_dimension = src->quantized_dimension;
  if (src->scale) {
    const int n = src->scale->size;
    a->scale = static_cast<FArr*>(std::calloc(1, sizeof(int) + sizeof(float) * (n > 0 ? n : 1)));
    a->scale->size = n;
    std::memcpy(a->scale->data, src->scale->data, sizeof(float) * n);
  }
  if (src->zero_point) {
    const int n = src->zero_point->size;
    a->zero_point = static_cast<IArr*>(std::calloc(1, sizeof(int) + sizeof(int) * (n > 0 ? n : 1)));
    a->zero_point->size = n;
    std::memcpy(a->zero_point->data, src->zero_point->data, sizeof(int) * n);
  }
  return a;
}
}  // namespace

namespace {
// Request inputs are copied into page-locked ring slots that the GPU's DMA
// engines read next; no CPU reads them back.  Streaming (non-temporal)
// stores skip the read-for-ownership of every destination line that plain
// stores pay (the slot was last touched by the DMA, so each line would come
// from DRAM) and leave the caches to the caller.  Large copies into ring
// memory only; BANDX_RING_NT=0 keeps memcpy.
bool UseStreamingStores() {
  static const bool on = [] {
    const char* e = std::getenv("BANDX_RING_NT");
    return !(e && e[0] == '0') && __builtin_cpu_supports("avx2");
  }();
  return on;
}

__attribute__((target("avx2"))) void StreamCopy(char* dst, const char* src, size_t n) {
  // head: up to the next 32-byte boundary of dst
  const size_t head = std::min(n, static_cast<size_t>((32 - (reinterpret_cast<uintptr_t>(dst) & 31)) & 31));
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
    const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
  }
  for (; i + 32 <= n; i += 32)
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i),
                        _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)));
  std::memcpy(dst + i, src + i, n - i);
  _mm_sfence();  // the streamed lines are globally visible before the request is queued
}

// src -> a ring slot tensor
absl::Status PutIntoSlot(Tensor* slot, const interface::ITensor* src) {
  constexpr size_t kStreamMin = 64 << 10;
  if (!src || !slot->IsRingMemory() || slot->GetBytes() < kStreamMin || !UseStreamingStores() ||
      *static_cast<const interface::ITensor*>(slot) != *src)
    return slot->CopyDataFrom(src);  // the checks and errors of ITensor::CopyDataFrom
  StreamCopy(slot->GetData(), src->GetData(), slot->GetBytes());
  return absl::OkStatus();
}
}  // namespace

Tensor::Tensor(const interface::ITensor* view, bool copy_data)
    : type_(view->GetType()),
      dims_(view->GetDims(), view->GetDims() + view->GetNumDims()),
      name_(view->GetName() ? view->GetName() : "") {
  const size_t bytes = view->GetBytes();
  data_.resize(bytes);
  Quantization q = view->GetQuantization();
  if (q.GetType() == QuantizationType::kAffineQuantization && q.GetParams()) {
    qtype_ = QuantizationType::kAffineQuantization;
    qparams_ = CloneAffine(static_cast<const Affine*>(q.GetParams()));
  }
  if (copy_data && bytes) std::memcpy(GetData(), view->GetData(), bytes);
}

Tensor::Tensor(const interface::ITensor* view, char* external)
    : type_(view->GetType()),
      dims_(view->GetDims(), view->GetDims() + view->GetNumDims()),
      ext_(external),
      ext_bytes_(view->GetBytes()),
      name_(view->GetName() ? view->GetName() : "") {
  Quantization q = view->GetQuantization();
  if (q.GetType() == QuantizationType::kAffineQuantization && q.GetParams()) {
    qtype_ = QuantizationType::kAffineQuantization;
    qparams_ = CloneAffine(static_cast<const Affine*>(q.GetParams()));
  }
}

Tensor::~Tensor() {
  FreeQuant();
}

void Tensor::FreeQuant() {
  if (!qparams_) return;
  auto* a = static_cast<Affine*>(qparams_);
  std::free(a->scale);
  std::free(a->zero_point);
  std::free(a);
  qparams_ = nullptr;
}

void Tensor::SetDims(const std::vector<int>& dims) {
  dims_ = dims;
  size_t n = GetDataTypeBytes(type_);
  for (int d : dims_) n *= static_cast<size_t>(d);
  if (ext_ && n != ext_bytes_) {  // a resized ring slot falls back to heap memory
    ext_ = nullptr;
    ext_bytes_ = 0;
  }
  if (!ext_) data_.resize(n);
}

Quantization Tensor::GetQuantization() const { return Quantization(qtype_, qparams_); }

absl::Status Tensor::SetQuantization(Quantization q) {
  FreeQuant();
  qtype_ = q.GetType();
  if (qtype_ == QuantizationType::kAffineQuantization && q.GetParams())
    qparams_ = CloneAffine(static_cast<const Affine*>(q.GetParams()));
  return absl::OkStatus();
}

TensorRingBuffer::TensorRingBuffer(const std::vector<std::shared_ptr<interface::ITensor>>& tensors,
                                   std::vector<int> tensor_indices, int size, RingHostAllocator a)
    : size_(size > 0 ? size : 1),
      num_tensors_(tensors.size()),
      slots_(size_),
      busy_(size_, 0),
      owner_(size_, -1),
      held_(size_, 0) {
  // read per ring (not once per process), so an engine created after a
  // change of the variable sees it
  const char* hold = std::getenv("BANDX_OUTPUT_HOLD_MS");
  hold_ms_ = hold ? std::max(0L, std::atol(hold)) : 2000L;
  std::vector<size_t> stride(tensors.size(), 0);
  if (a.alloc && a.free) {
    block_free_ = a.free;
    for (size_t i = 0; i < tensors.size(); ++i) {
      // slots back to back: consecutive handles form one contiguous run
      stride[i] = tensors[i]->GetBytes();
      char* b = stride[i] ? static_cast<char*>(a.alloc(stride[i] * size_)) : nullptr;
      blocks_.push_back(b);
    }
  }
  for (int s = 0; s < size_; ++s)
    for (size_t i = 0; i < tensors.size(); ++i) {
      char* b = i < blocks_.size() ? blocks_[i] : nullptr;
      slots_[s].emplace_back(b ? new Tensor(tensors[i].get(), b + s * stride[i]) : new Tensor(tensors[i].get()));
    }
  for (size_t i = 0; i < tensor_indices.size(); ++i) tensor_to_buffer_[tensor_indices[i]] = static_cast<int>(i);
}

TensorRingBuffer::~TensorRingBuffer() {
  slots_.clear();  // the slot tensors view the blocks
  for (char* b : blocks_)
    if (b) block_free_(b);
}

int TensorRingBuffer::Alloc() {
  std::lock_guard<std::mutex> lock(head_mtx_);
  return head_++;
}

int TensorRingBuffer::Claim(int handle) {
  std::lock_guard<std::mutex> lock(head_mtx_);
  if (handle + 1 > head_) head_ = handle + 1;
  return handle;
}

int TensorRingBuffer::AllocBlocking() { return AllocBlockingN(1); }

// Slots are handed out in handle order, so the n slots a call takes are the
// next n of the ring; the call waits until each of them is free.  Jobs of one
// model can finish out of order (several workers), so counting unfinished
// requests is not enough: a slot whose request is still pending must not be
// handed to a newer one (it would overwrite that request's input, and its
// handle would leave the ring's valid window before its output copy).
int TensorRingBuffer::AllocBlockingN(int n) {
  std::unique_lock<std::mutex> lock(head_mtx_);
  auto free_run = [this, n] {
    if (n > size_) return false;
    for (int k = 0; k < n; ++k)
      if (busy_[Slot(head_ + k)]) return false;
    return true;
  };
  slot_cv_.wait(lock, free_run);
  for (int k = 0; k < n; ++k) busy_[Slot(head_ + k)] = 1;
  outstanding_ += n;
  const int first = head_;
  head_ += n;
  return first;
}

void TensorRingBuffer::Release(int handle) {
  {
    std::lock_guard<std::mutex> lock(head_mtx_);
    if (handle < 0 || !busy_[Slot(handle)]) return;
    busy_[Slot(handle)] = 0;
    --outstanding_;
  }
  slot_cv_.notify_all();  // waiters may need different slot counts
}

bool TensorRingBuffer::TryAcquireForWrite(int handle) {
  if (handle < 0) return true;
  std::lock_guard<std::mutex> lock(head_mtx_);
  const int s = Slot(handle);
  if (held_[s] && owner_[s] != handle) return false;
  owner_[s] = handle;
  return true;
}

bool TensorRingBuffer::AcquireForWrite(int handle) {
  if (handle < 0) return true;
  const long hold_ms = hold_ms_;
  std::unique_lock<std::mutex> lock(head_mtx_);
  const int s = Slot(handle);
  if (!slot_cv_.wait_for(lock, std::chrono::milliseconds(hold_ms),
                         [&] { return !held_[s] || owner_[s] == handle; })) {
    BAND_LOG(LogSeverity::kWarning,
             "output slot %d of request %d is still held by request %d's end-request callback after %ld ms "
             "(does the callback wait for a newer request of its model?): output write refused",
             s, handle, owner_[s], hold_ms);
    return false;
  }
  owner_[s] = handle;
  return true;
}

void TensorRingBuffer::Hold(int handle) {
  if (handle < 0) return;
  std::lock_guard<std::mutex> lock(head_mtx_);
  if (owner_[Slot(handle)] == handle) held_[Slot(handle)] = 1;
}

void TensorRingBuffer::Unhold(int handle) {
  if (handle < 0) return;
  {
    std::lock_guard<std::mutex> lock(head_mtx_);
    if (owner_[Slot(handle)] != handle || !held_[Slot(handle)]) return;
    held_[Slot(handle)] = 0;
  }
  slot_cv_.notify_all();
}

int TensorRingBuffer::Outstanding() const {
  std::lock_guard<std::mutex> lock(head_mtx_);
  return outstanding_;
}

bool TensorRingBuffer::IsHandleValid(int handle) const {
  std::lock_guard<std::mutex> lock(head_mtx_);
  return handle >= 0 && ((head_ - size_ <= handle && handle < head_) || owner_[Slot(handle)] == handle);
}

Tensor* TensorRingBuffer::SlotTensor(int tensor_index, int handle) {
  auto it = tensor_to_buffer_.find(tensor_index);
  if (it == tensor_to_buffer_.end() || !IsHandleValid(handle)) return nullptr;
  return slots_[Slot(handle)][it->second].get();
}

absl::Status TensorRingBuffer::GetTensorFromHandle(interface::ITensor* dst, int tensor_index, int handle) const {
  auto it = tensor_to_buffer_.find(tensor_index);
  if (it == tensor_to_buffer_.end())
    return absl::InternalError("GetTensorFromHandle: Invalid tensor index: " + std::to_string(tensor_index));
  if (!IsHandleValid(handle))
    return absl::InternalError("GetTensorFromHandle: Invalid memory handle: " + std::to_string(handle));
  return dst->CopyDataFrom(slots_[Slot(handle)][it->second].get());
}

absl::Status TensorRingBuffer::PutTensorToHandle(const interface::ITensor* src, int tensor_index, int handle) {
  auto it = tensor_to_buffer_.find(tensor_index);
  if (it == tensor_to_buffer_.end())
    return absl::InternalError("PutTensorToHandle: Invalid tensor index: " + std::to_string(tensor_index));
  if (!IsHandleValid(handle))
    return absl::InternalError("PutTensorToHandle: Invalid memory handle: " + std::to_string(handle));
  return PutIntoSlot(slots_[Slot(handle)][it->second].get(), src);
}

absl::Status TensorRingBuffer::GetTensorsFromHandle(std::vector<interface::ITensor*>& dst, int handle) const {
  if (!IsHandleValid(handle))
    return absl::InternalError("GetTensorsFromHandle: Invalid memory handle: " + std::to_string(handle));
  if (dst.size() != num_tensors_) return absl::InternalError("Invalid tensor length");
  for (size_t i = 0; i < num_tensors_; ++i)
    if (!dst[i] || !dst[i]->CopyDataFrom(slots_[Slot(handle)][i].get()).ok())
      return absl::InternalError("Failed to copy tensors.");
  return absl::OkStatus();
}

absl::Status TensorRingBuffer::PutTensorsToHandle(const std::vector<interface::ITensor*>& src, int handle) {
  if (!IsHandleValid(handle))
    return absl::InternalError("PutTensorsToHandle: Invalid memory handle: " + std::to_string(handle));
  if (src.size() != num_tensors_) return absl::InternalError("Invalid tensor length");
  for (size_t i = 0; i < num_tensors_; ++i)
    if (!PutIntoSlot(slots_[Slot(handle)][i].get(), src[i]).ok())
      return absl::InternalError("Failed to copy tensors.");
  return absl::OkStatus();
}

absl::Status TensorRingBuffer::CheckTensors(const std::vector<interface::ITensor*>& src) const {
  if (src.size() != num_tensors_) return absl::InternalError("Invalid tensor length");
  for (size_t i = 0; i < num_tensors_; ++i)
    if (!src[i] || *static_cast<const interface::ITensor*>(slots_[0][i].get()) != *src[i])
      return absl::InternalError("Failed to copy tensors.");
  return absl::OkStatus();
}

}  // namespace band
