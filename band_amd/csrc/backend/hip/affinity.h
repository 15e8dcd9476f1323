// Host thread placement for the HIP backend's workers.
//
// kCPU executors honour the CpuSet Band hands every executor
// (band/interface/model_executor.h:41-50): the reference passes it to the
// TFLite interpreter's thread pool (band/backend/tfl/model_executor.cc:356-359,
// InterpreterBuilder::SetCpuMasks), so a kCPU HipModelExecutor pins its host
// pool to it.  An empty set (what BandCPUMaskGetSet returns on Linux,
// band/device/cpu.cc:377-381) leaves the threads where they are.
//
// kGPU executors never move the thread that calls them (it may be the
// application's own).  An engine that owns its GPU worker threads may pin
// each one to the CPUs of its GPU's NUMA node (PCI sysfs numa_node of
// hipDeviceGetPCIBusId), intersected with the CPUs the process may use,
// through the optional bhx_pin_worker_thread hook (include/band_hip_backend.h;
// this repo's harness calls it from Worker::Work when the worker's CpuSet
// names no CPUs): the job's host copies then stay on the socket the GPU hangs
// off.  BANDX_NUMA_PIN=0 turns this off.
#pragma once

#include <pthread.h>

#include <string>
#include <vector>

namespace band {
class CpuSet;
namespace hip {

// The CPUs a CpuSet asks for, read with the reference's own API
// (band/device/cpu.h:21-40: IsEnabled(i) for i < GetCPUCount()).  Empty -
// "do not pin" - when the set enables nothing or every CPU the process may
// use: the reference's Linux build reports every CPU enabled
// (band/device/cpu.cc:72-92), and an all-CPU mask is no constraint.
std::vector<int> PinnableCpus(const CpuSet& set);

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}; malformed pieces are skipped
std::vector<int> ParseCpuList(const std::string& s);
// CPUs the process was started with (sched_getaffinity of the process,
// captured on first use, before any thread of ours narrowed its own)
const std::vector<int>& ProcessCpus();
// pins thread `t` to `cpus`; false when cpus is empty or the call fails
bool PinThread(pthread_t t, const std::vector<int>& cpus);
// CPUs of the calling thread's current affinity mask
std::vector<int> CallingThreadCpus();
// NUMA node of GPU `ordinal` (-1 when unknown: no sysfs entry, no NUMA)
int GpuNumaNode(int ordinal);
// CPUs of that node intersected with ProcessCpus(); empty when unknown
std::vector<int> GpuNumaCpus(int ordinal);
// pins the calling thread to GpuNumaCpus(ordinal), once per (thread,
// ordinal); returns whether the thread is now pinned to that node
bool PinCallingThreadToGpu(int ordinal);
// pins EVERY thread the process has now (/proc/self/task) to
// GpuNumaCpus(ordinal); threads they create later inherit the mask.  For a
// one-GPU process (bench.py's ranks): the request driver's submit/read
// threads, the planner and the HIP runtime's own threads then share the GPU's
// socket with the workers and the page-locked request rings.  Returns the
// number of threads pinned (0: nothing to do, BANDX_NUMA_PIN=0 or no NUMA
// information), -1 when a thread could not be pinned.
int PinProcessToGpu(int ordinal);
// the same for an explicit CPU list: every current thread to `cpus`
// (threads pinned, -1 on failure or an empty list)
int PinProcessToCpus(const std::vector<int>& cpus);

}  // namespace hip
}  // namespace band
