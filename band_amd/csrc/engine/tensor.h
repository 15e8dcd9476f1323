// band::Tensor - a host tensor owning its bytes, created from a backend
// tensor view (band/tensor.h/.cc); the element type of the request ring
// buffers and of the C API's BandTensor.  Affine quantization parameters are
// deep-copied in the TfLiteAffineQuantization layout the views hand out.
#pragma once
#include <condition_variable>
#include <memory>
#include <mutex>
#include <map>
#include <string>
#include <vector>

#include "band/interface/tensor.h"

namespace band {

// Host memory for the request rings' slots.  The engine hands a ring the
// backend's optional page-locked allocator (Engine::RingAllocatorFor: the
// HIP backend's bhx_ring_host_alloc, when a GPU worker runs the whole model)
// so a batched pass can DMA a request's input from its ring slot and its
// outputs into its output slot with no staging copy; `alloc` may return
// nullptr, and then plain heap memory is used.
struct RingHostAllocator {
  void* (*alloc)(size_t bytes) = nullptr;
  void (*free)(void* p) = nullptr;
};

class Tensor : public interface::ITensor {
 public:
  explicit Tensor(const interface::ITensor* view, bool copy_data = false);
  // a slot of a request ring's page-locked block: `external` holds
  // view->GetBytes() bytes, owned by the ring
  Tensor(const interface::ITensor* view, char* external);
  ~Tensor() override;
  Tensor(const Tensor&) = delete;
  Tensor& operator=(const Tensor&) = delete;

  DataType GetType() const override { return type_; }
  void SetType(DataType type) override { type_ = type; }
  const char* GetData() const override { return ext_ ? ext_ : data_.data(); }
  char* GetData() override { return ext_ ? ext_ : data_.data(); }
  const int* GetDims() const override { return dims_.data(); }
  size_t GetNumDims() const override { return dims_.size(); }
  void SetDims(const std::vector<int>& dims) override;
  size_t GetBytes() const override { return ext_ ? ext_bytes_ : data_.size(); }
  // the bytes came from a ring host allocator (page-locked)
  bool IsRingMemory() const { return ext_ != nullptr; }
  const char* GetName() const override { return name_.c_str(); }
  Quantization GetQuantization() const override;
  absl::Status SetQuantization(Quantization quantization) override;

 private:
  void FreeQuant();
  DataType type_;
  std::vector<int> dims_;
  std::vector<char> data_;
  char* ext_ = nullptr;  // a slot of a ring's page-locked block (data_ unused then)
  size_t ext_bytes_ = 0;
  std::string name_;
  QuantizationType qtype_ = QuantizationType::kNoQuantization;
  void* qparams_ = nullptr;  // TfLiteAffineQuantization layout, owned
};

// Per-model ring of request I/O slots (band/tensor_ring_buffer.h/.cc): a
// handle is a monotonically increasing slot number; slot = handle % size.
// Only the handle bookkeeping is under the lock - the memcpy of a slot runs
// outside it, so copies of different requests of one model proceed in
// parallel (the reference copies under the ring's mutex).
//
// Back-pressure (deviation): the reference's Alloc never waits, so a model
// with more than `size` unfinished requests reuses the slot of a request
// that has not run yet and that job later fails its input or output copy.
// AllocBlocking() waits until the next slot of the ring is free - the slot
// itself, not a count, since jobs of one model finish out of order; Release()
// frees a request's slot when its job is finished
// (Planner::EnqueueFinishedJob, before the end-request callbacks, so a
// callback may submit into a full ring).
class TensorRingBuffer {
 public:
  TensorRingBuffer(const std::vector<std::shared_ptr<interface::ITensor>>& tensors, std::vector<int> tensor_indices,
                   int size = 128, RingHostAllocator alloc = RingHostAllocator());
  ~TensorRingBuffer();
  int Alloc();
  // takes `handle` itself (the head moves past it): a model's output slot
  // uses its request's input handle, so the input ring's per-slot
  // back-pressure also keeps the output handle inside this ring's window
  // until the job has written it, whatever order concurrent callers finish in
  int Claim(int handle);
  // Alloc() once the next slot's request (if any) is finished
  int AllocBlocking();
  // n consecutive handles at once (the first is returned), once those n
  // slots are free; n must not exceed size()
  int AllocBlockingN(int n);
  // frees the slot of a handle taken with AllocBlocking[N]
  void Release(int handle);
  // Output-ring ownership.  A slot's outputs belong to the request whose job
  // wrote them last (AcquireForWrite, before the write); that handle stays
  // readable (IsHandleValid) until a newer request writes the slot, even
  // once newer submissions have moved the handle window past it.  Hold keeps
  // the owner's outputs in place - a newer writer waits in AcquireForWrite -
  // until Unhold (Planner::EnqueueFinishedJob brackets the end-request
  // callbacks with them).  The wait is bounded (BANDX_OUTPUT_HOLD_MS, default
  // 2000): a callback that waits synchronously for a newer request of its
  // own model (RequestSync / Wait) while that request's job needs the held
  // slot would otherwise wait for itself.  On timeout the write is refused
  // (false, a warning is logged) and the newer job fails its output copy;
  // the held outputs stay intact.
  bool AcquireForWrite(int handle);
  // the same without waiting: false when the slot is held right now
  bool TryAcquireForWrite(int handle);
  void Hold(int handle);
  void Unhold(int handle);
  int size() const { return size_; }
  int Outstanding() const;
  bool IsTensorIndexValid(int tensor_index) const { return tensor_to_buffer_.count(tensor_index) != 0; }
  bool IsHandleValid(int handle) const;
  int GetTensorsLength() const { return static_cast<int>(num_tensors_); }
  absl::Status GetTensorFromHandle(interface::ITensor* dst, int tensor_index, int handle) const;
  absl::Status PutTensorToHandle(const interface::ITensor* src, int tensor_index, int handle);
  absl::Status GetTensorsFromHandle(std::vector<interface::ITensor*>& dst, int handle) const;
  absl::Status PutTensorsToHandle(const std::vector<interface::ITensor*>& src, int handle);
  // whether PutTensorsToHandle would accept `src` (count, and each tensor's
  // type and dims, as ITensor::CopyDataFrom checks)
  absl::Status CheckTensors(const std::vector<interface::ITensor*>& src) const;
  // the slot tensor of `tensor_index` for a valid handle, else nullptr: a
  // batched pass reads a request's input from / writes its output into it
  // directly (a handle stays valid while its request is unfinished)
  Tensor* SlotTensor(int tensor_index, int handle);

 private:
  int Slot(int handle) const { return handle % size_; }
  const int size_;
  size_t num_tensors_;
  std::vector<std::vector<std::unique_ptr<Tensor>>> slots_;
  std::map<int, int> tensor_to_buffer_;
  mutable std::mutex head_mtx_;
  std::condition_variable slot_cv_;
  std::vector<char> busy_;  // per slot: taken by AllocBlocking[N], not yet released
  std::vector<int> owner_;  // per slot: handle whose outputs it holds (-1: none)
  std::vector<char> held_;  // per slot: the owner's outputs are being read
  long hold_ms_ = 2000;     // AcquireForWrite's bound (BANDX_OUTPUT_HOLD_MS at construction)
  // per tensor: one page-locked block holding every slot's bytes at a fixed
  // stride (consecutive handles are adjacent, so a batched pass copies a
  // run of them in one DMA); empty when the ring has no host allocator
  std::vector<char*> blocks_;
  void (*block_free_)(void*) = nullptr;
  int head_ = 0;
  int outstanding_ = 0;
};

}  // namespace band
