// Per-process GPU bookkeeping for the HIP backend.
//
// Band hands an executor only (model, worker, DeviceFlag, CpuSet, threads)
// (band/backend_factory.h:34-38) - no device index.  Worker -> GPU ordinal is
// therefore resolved here: an explicit mapping (bhx_set_worker_device, used
// by one-process-per-GPU launchers) wins; otherwise GPU workers are numbered
// in order of first appearance and wrapped over the visible devices, which
// is deterministic because Engine::RegisterModel walks worker ids in
// ascending order (band/engine.cc:91).  Each GPU worker owns one
// non-blocking stream that all of its executors share; calls on one worker
// are serialised by Band (band/worker.cc:222-323).
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "band_hip_kernels.h"

namespace band {
namespace hip {

// RAII device allocation; ordinal < 0 is host memory (the operands and
// arena of a kCPU executor, see cpu_kernels.h).
class DeviceBlob {
 public:
  DeviceBlob(int ordinal, size_t bytes);
  ~DeviceBlob();
  DeviceBlob(const DeviceBlob&) = delete;
  DeviceBlob& operator=(const DeviceBlob&) = delete;
  void* ptr() const { return ptr_; }
  size_t bytes() const { return bytes_; }
  int ordinal() const { return ordinal_; }
  bool ok() const { return ptr_ != nullptr; }
  bool host() const { return ordinal_ < 0; }
  // copies host bytes into the blob at `offset` (H2D for device blobs)
  bool Upload(size_t offset, const void* src, size_t bytes);

 private:
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
  int ordinal_ = 0;
};

// RAII host allocation: page-locked (hipHostMalloc) for GPU executors so
// the H2D/D2H of job I/O run at PCIe rate; plain aligned memory for
// CPU-worker executors.
class PinnedBuffer {
 public:
  explicit PinnedBuffer(size_t bytes, bool pinned = true);
  // a non-owning view of host memory someone else owns (a kCPU executor's
  // boundary tensors alias its host arena: no copy in or out)
  PinnedBuffer(char* external, size_t bytes) : ptr_(external), bytes_(bytes), pinned_(false), owned_(false) {}
  ~PinnedBuffer();
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  char* data() const { return static_cast<char*>(ptr_); }
  size_t bytes() const { return bytes_; }
  bool ok() const { return ptr_ != nullptr; }

 private:
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
  bool pinned_ = true;
  bool owned_ = true;
};

class DeviceRegistry {
 public:
  static DeviceRegistry& Get();
  int DeviceCount();
  bool GpuAvailable();  // at least one gfx950 device
  void SetWorkerOrdinal(int worker_id, int ordinal);
  int OrdinalForWorker(int worker_id);
  // the ordinal already mapped to worker_id (-1: none yet); assigns nothing
  int FindWorkerOrdinal(int worker_id);
  bh_stream_t StreamForWorker(int worker_id);

  // Device-resident constant operands shared by every executor of a model on
  // one GPU (weights are replicated per GPU, not per executor).
  std::shared_ptr<DeviceBlob> FindConst(int ordinal, const std::string& key);
  void PutConst(int ordinal, const std::string& key, const std::shared_ptr<DeviceBlob>& blob);

 private:
  DeviceRegistry() = default;
  void Probe();
  std::mutex mu_;
  bool probed_ = false;
  int count_ = 0;
  bool gfx950_ = false;
  std::map<int, int> worker_ordinal_;
  int next_auto_ = 0;
  std::map<std::pair<int, int>, bh_stream_t> streams_;  // (worker id, ordinal)
  std::map<std::pair<int, std::string>, std::weak_ptr<DeviceBlob>> consts_;
};

}  // namespace hip
}  // namespace band
