#include "backend/hip/device.h"

#include <cstdlib>
#include <cstring>

namespace band {
namespace hip {

DeviceBlob::DeviceBlob(int ordinal, size_t bytes) : bytes_(bytes), ordinal_(ordinal) {
  if (ordinal < 0) {
    const size_t n = ((bytes ? bytes : 16) + 63) / 64 * 64;
    ptr_ = std::aligned_alloc(64, n);
    if (ptr_) std::memset(ptr_, 0, n);
    return;
  }
  if (bh_set_device(ordinal) == 0 && bh_malloc(&ptr_, bytes ? bytes : 16) != 0) ptr_ = nullptr;
}
DeviceBlob::~DeviceBlob() {
  if (!ptr_) return;
  if (ordinal_ < 0) {
    std::free(ptr_);
    return;
  }
  bh_set_device(ordinal_);
  bh_free(ptr_);
}
bool DeviceBlob::Upload(size_t offset, const void* src, size_t bytes) {
  if (!ptr_ || offset + bytes > (bytes_ ? bytes_ : 16)) return false;
  if (ordinal_ < 0) {
    std::memcpy(static_cast<char*>(ptr_) + offset, src, bytes);
    return true;
  }
  return bh_set_device(ordinal_) == 0 && bh_memcpy_h2d(static_cast<char*>(ptr_) + offset, src, bytes) == 0;
}

PinnedBuffer::PinnedBuffer(size_t bytes, bool pinned) : bytes_(bytes), pinned_(pinned) {
  const size_t n = (bytes ? bytes : 16) + 63;
  if (pinned_) {
    if (bh_host_alloc(&ptr_, n) != 0) ptr_ = nullptr;
  } else {
    ptr_ = std::aligned_alloc(64, n / 64 * 64);
  }
  if (ptr_) std::memset(ptr_, 0, n / 64 * 64);
}
PinnedBuffer::~PinnedBuffer() {
  if (!ptr_ || !owned_) return;
  if (pinned_) bh_host_free(ptr_);
  else std::free(ptr_);
}

DeviceRegistry& DeviceRegistry::Get() {
  static DeviceRegistry* r = new DeviceRegistry();  // never destroyed: outlives executors
  return *r;
}

void DeviceRegistry::Probe() {
  if (probed_) return;
  probed_ = true;
  int n = 0;
  if (bh_device_count(&n) != 0) n = 0;
  count_ = n;
  for (int i = 0; i < n; ++i) {
    char arch[128] = {0};
    if (bh_device_arch(i, arch, sizeof(arch)) == 0 && std::strncmp(arch, "gfx950", 6) == 0) gfx950_ = true;
  }
}

int DeviceRegistry::DeviceCount() {
  std::lock_guard<std::mutex> l(mu_);
  Probe();
  return count_;
}

bool DeviceRegistry::GpuAvailable() {
  std::lock_guard<std::mutex> l(mu_);
  Probe();
  return count_ > 0 && gfx950_;
}

void DeviceRegistry::SetWorkerOrdinal(int worker_id, int ordinal) {
  std::lock_guard<std::mutex> l(mu_);
  worker_ordinal_[worker_id] = ordinal;
}

int DeviceRegistry::OrdinalForWorker(int worker_id) {
  std::lock_guard<std::mutex> l(mu_);
  Probe();
  auto it = worker_ordinal_.find(worker_id);
  if (it != worker_ordinal_.end()) return it->second;
  const int ord = count_ > 0 ? next_auto_++ % count_ : 0;
  worker_ordinal_[worker_id] = ord;
  return ord;
}

int DeviceRegistry::FindWorkerOrdinal(int worker_id) {
  std::lock_guard<std::mutex> l(mu_);
  auto it = worker_ordinal_.find(worker_id);
  return it != worker_ordinal_.end() ? it->second : -1;
}

bh_stream_t DeviceRegistry::StreamForWorker(int worker_id) {
  const int ord = OrdinalForWorker(worker_id);
  std::lock_guard<std::mutex> l(mu_);
  // keyed by (worker, ordinal): a later engine may map the same worker id
  // to another device (bench.py's single-engine line after the per-GPU ones)
  auto it = streams_.find({worker_id, ord});
  if (it != streams_.end()) return it->second;
  bh_stream_t s = nullptr;
  if (bh_set_device(ord) != 0 || bh_stream_create(&s) != 0) return nullptr;
  streams_[{worker_id, ord}] = s;
  return s;
}

std::shared_ptr<DeviceBlob> DeviceRegistry::FindConst(int ordinal, const std::string& key) {
  std::lock_guard<std::mutex> l(mu_);
  auto it = consts_.find({ordinal, key});
  if (it == consts_.end()) return nullptr;
  auto sp = it->second.lock();
  if (!sp) consts_.erase(it);
  return sp;
}

void DeviceRegistry::PutConst(int ordinal, const std::string& key, const std::shared_ptr<DeviceBlob>& blob) {
  std::lock_guard<std::mutex> l(mu_);
  consts_[{ordinal, key}] = blob;
}

}  // namespace hip
}  // namespace band
