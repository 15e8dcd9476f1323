/*
 * band_hip_backend.h - C ABI over the HIP backend's Band plugin objects.
 *
 * Band binds its backend through C++ virtuals (band/interface/model.h:17-38,
 * band/interface/model_executor.h:30-180, band/interface/tensor.h:27-50,
 * band/interface/backend.h:21-26), created by BackendFactory
 * (band/backend_factory.h:31-70).  Inside a Band build those are used
 * directly.  This header exposes the same objects with
 * plain pointers and sizes so any FFI (ctypes, JNI, cgo) can drive them;
 * each function names the interface method it forwards to.
 *
 * Subgraph keys are passed as (model_id, worker_id, unit_mask) where bit i of
 * unit_mask is unit subgraph i (SubgraphKey's 64-bit BitMask,
 * band/common.h:293-319).  Device flags use Band's DeviceFlag numbering
 * (0 CPU, 1 GPU, 2 DSP, 3 NPU); data types use Band's DataType (== TfLiteType).
 *
 * Return codes: 0 = OK; otherwise the absl::StatusCode of the failing call
 * (13 = kInternal) with the message available from bhx_last_error().
 */
#ifndef BAND_HIP_BACKEND_H_
#define BAND_HIP_BACKEND_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bhx_model bhx_model;
typedef struct bhx_executor bhx_executor;

typedef struct bhx_tensor_info {
  int type;           /* Band DataType */
  int ndims;
  int dims[8];
  void* data;         /* host-addressable view data (ITensorView::GetData) */
  size_t bytes;       /* ITensorView::GetBytes */
  const char* name;   /* ITensorView::GetName */
  int quant_type;     /* QuantizationType: 0 none, 1 affine */
  int n_quant;        /* number of scales / zero points */
  const float* scale;
  const int32_t* zero_point;
  int quantized_dimension;
} bhx_tensor_info;

typedef struct bhx_op_timing {
  int op_index;
  const char* kernel;
  double ms;          /* mean HIP-event time of the launch */
  double alg_bytes;   /* algorithmic bytes per launch */
  double alg_ops;     /* algorithmic integer ops per launch (2 per MAC) */
} bhx_op_timing;

const char* bhx_last_error(void);

/* IBackendUtil::GetAvailableDevices -> bit i set = DeviceFlag i available */
int bhx_available_devices(uint32_t* mask);
/* pin a Band worker id to a GPU ordinal (one process per GPU launchers) */
int bhx_set_worker_device(int worker_id, int ordinal);
/* the ordinal a worker's executors use: its bhx_set_worker_device mapping,
 * else assigned on first use in ascending order modulo the device count */
int bhx_worker_device(int worker_id);

/* IModel (BackendFactory::CreateModel + FromPath/FromBuffer/IsInitialized) */
int bhx_model_create(int model_id, bhx_model** out);
int bhx_model_from_path(bhx_model* m, const char* path);
int bhx_model_from_buffer(bhx_model* m, const char* buffer, size_t size);
int bhx_model_is_initialized(const bhx_model* m);
int bhx_model_get_id(const bhx_model* m);
void bhx_model_destroy(bhx_model* m);

/* IModelExecutor (BackendFactory::CreateModelExecutor) */
int bhx_executor_create(int model_id, int worker_id, int device_flag, int num_threads, bhx_executor** out);
/* the same with an explicit CpuSet (band/interface/model_executor.h:41-50's
 * thread_affinity_mask): cpus[0..n_cpus) enabled; a kCPU executor pins its
 * host thread pool to it (band/backend/tfl/model_executor.cc:356-359) */
int bhx_executor_create_masked(int model_id, int worker_id, int device_flag, int num_threads, const int* cpus,
                               int n_cpus, bhx_executor** out);
void bhx_executor_destroy(bhx_executor* e);
/* NUMA node of GPU `ordinal` from its PCI sysfs entry (-1: unknown), and the
 * CPUs of that node the process may use (count returned, up to cap written):
 * where a kGPU executor pins its worker thread (affinity.h) */
int bhx_gpu_numa_node(int ordinal);
int bhx_gpu_numa_cpus(int ordinal, int* cpus, int cap);
/* pins every thread of the process (and, by inheritance, the threads it
 * creates later) to those CPUs: for a process that drives one GPU.  Returns
 * threads pinned, 0 when there is nothing to do (BANDX_NUMA_PIN=0, no NUMA
 * information, or the node is every CPU the process has), -1 on failure. */
int bhx_pin_process_to_gpu(int ordinal);
/* the same for an explicit list cpus[0..n_cpus): every current thread of the
 * process to it; threads pinned, -1 on failure */
int bhx_pin_process_to_cpus(const int* cpus, int n_cpus);
/* bytes of page-locked request-ring memory allocated so far on each NUMA
 * node (sampled every 16th page): bytes_per_node[i] for node i, the entry
 * after the last node counts pages whose node was unknown.  Returns the
 * number of entries that exist (up to cap written). */
int bhx_ring_page_nodes(long long* bytes_per_node, int cap);
/* Job coalescing totals over every coalescer of the process (coalescer.h:
 * concurrent ExecuteSubgraph calls of one model on one GPU run as job-batch
 * passes): out[0] calls, out[1] passes that ran one job alone, out[2]
 * passes of >= 2 jobs, out[3] jobs in those passes, out[4] the largest such
 * pass, out[5] calls that ran with coalescing off (no lanes: a lone
 * executor's model, or a failed lane build) and out[6] the most such calls
 * running at once (out must hold 7).  reset != 0 zeroes the totals after
 * reading them. */
int bhx_coalescer_stats(long long* out, int reset);
/* members and lanes-ready flag of the coalescer executor `e`'s whole-model
 * subgraph joined (0 / 0 when it joined none) */
int bhx_executor_coalescer(bhx_executor* e, int* members, int* lanes_ready);
/* Optional hooks for a Band-compatible engine, looked up as weak symbols
 * (engine/engine.cc, engine/worker.cc); Band itself never needs them.
 * bhx_ring_host_alloc: page-locked memory for a request ring's slots, so a
 * GPU worker DMAs a job's I/O straight from / into its ring slot; NULL (use
 * the heap) when no GPU is visible, BAND_HIP_PINNED_RINGS=0, or the total
 * would pass BAND_HIP_PINNED_RING_MB (default 8192).
 * bhx_pin_worker_thread: pins the calling engine-owned worker thread to the
 * CPUs of the NUMA node of the GPU `worker_id` runs on (affinity.h); 1 pinned,
 * 0 nothing to do (BANDX_NUMA_PIN=0, no NUMA information), -1 the worker has
 * no GPU ordinal yet (no kGPU executor created for it). */
void* bhx_ring_host_alloc(size_t bytes);
void bhx_ring_host_free(void* p);
int bhx_pin_worker_thread(int worker_id);
/* InvestigateModelSpec -> ModelSpec serialised as JSON into buf.
 * *needed receives the full length (+1); the call fails if cap < needed. */
int bhx_investigate_model_spec(bhx_executor* e, bhx_model* m, char* buf, size_t cap, size_t* needed);
/* PrepareSubgraph(model, ops, unit_indices); n_ops == 0 -> whole model */
int bhx_prepare_subgraph(bhx_executor* e, bhx_model* m, const int* ops, int n_ops,
                         const int* unit_indices, int n_units);
int bhx_has_subgraph(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask);
/* GetInputs / GetOutputs: writes up to cap indices, *n = total count */
int bhx_get_inputs(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int* out, int cap, int* n);
int bhx_get_outputs(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int* out, int cap, int* n);
const char* bhx_get_input_name(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int index);
const char* bhx_get_output_name(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int index);
size_t bhx_get_num_tensors(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask);
size_t bhx_get_num_nodes(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask);
/* GetTensorView: fills info; data stays valid for the executor's lifetime */
int bhx_get_tensor_view(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int tensor_index,
                        bhx_tensor_info* info);
int bhx_get_largest_subgraph_key(bhx_executor* e, int* model_id, int* worker_id, uint64_t* unit_mask);
/* ForEachSubgraph: writes up to cap keys */
int bhx_list_subgraphs(bhx_executor* e, int* model_ids, int* worker_ids, uint64_t* unit_masks, int cap, int* n);
/* ExecuteSubgraph (synchronous: returns when outputs are in the views) */
int bhx_execute_subgraph(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask);

/* --- native worker loop ------------------------------------------------
 * Runs n_jobs Band jobs back to back on one executor, exactly the per-job
 * work of Worker::Work (band/worker.cc:222-323) for a single-input /
 * single-output subgraph: CopyDataFrom(request slot j % n_slots) into the
 * input view (Engine::TryCopyInputTensors, band/engine.cc:1247-1319),
 * ExecuteSubgraph (band/engine.cc:843-850), copy the output view out
 * (TryCopyOutputTensors :1333-1365).  latency_us[j] (optional) receives
 * end - enqueue of job j.  Stops at the first failing job. */
int bhx_run_jobs(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, const void* const* in_slots,
                 int n_slots, size_t in_bytes, void* out, size_t out_bytes, int n_jobs, double* latency_us);

/* --- extensions (measurement / tuning; not part of Band's interface) --- */
int bhx_executor_set_graph(bhx_executor* e, int enabled);
int bhx_executor_device(bhx_executor* e, int* ordinal);
/* per-launch timing of a prepared subgraph: the launch sequence is queued
 * behind a spin kernel and runs once in program order (each kernel sees a
 * real pass's cache state); every kernel carries its dispatch begin / end
 * timestamps (hipExtLaunchKernel events), i.e. the kernel-only duration
 * rocprofv3's kernel trace reports; averaged over iters.  *floor_us (may be
 * NULL) = the same figure for an empty single-wave kernel: the fixed
 * dispatch cost inside every duration. */
int bhx_profile_subgraph(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int iters,
                         bhx_op_timing* out, int cap, int* n, double* floor_us);
/* A Band GPU worker serving a mixed request stream (BASELINE C3): worker
 * `wid` holds one prepared executor per model (as Band creates one executor
 * per (model, worker), band/engine.cc:91-106); job j runs model
 * (first_model + j) % n_models: copy its request into the input view,
 * ExecuteSubgraph, copy every output view out.  Per-job latency in us and
 * the model of each job are written when the arrays are given. */
int bhx_run_mixed_jobs(int n_models, bhx_executor* const* execs, const int* model_ids, int worker_id,
                       uint64_t unit_mask, const void* const* requests, int first_model, int n_jobs,
                       double* latency_us, int* model_of_job);
/* device microseconds per pass of a prepared subgraph, `iters` passes issued
 * back to back on the executor's stream (graph replay when captured) */
int bhx_time_subgraph(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int iters, double* us);

/* --- job batching (extension, backend/hip/job_batching.h) -------------
 * Not in the reference interface: Band runs one job per ExecuteSubgraph
 * (band/worker.cc:222-323).  A prepared kGPU subgraph gets batch variants
 * for up to max_batch jobs; slot views are batch-1 views into a variant's
 * pinned boundary mirrors; execute runs n jobs in one pass. */
int bhx_prepare_job_batches(bhx_executor* e, bhx_model* m, int model_id, int worker_id, uint64_t unit_mask,
                            int max_batch);
int bhx_max_job_batch(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int* max_batch);
int bhx_job_slot_view(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int tensor_index, int n,
                      int slot, bhx_tensor_info* info);
int bhx_execute_job_batch(bhx_executor* e, int model_id, int worker_id, uint64_t unit_mask, int n);

#ifdef __cplusplus
}
#endif
#endif /* BAND_HIP_BACKEND_H_ */
