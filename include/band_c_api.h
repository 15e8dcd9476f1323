/*
 * Band engine C API, served by libband_hip.so.
 *
 * Same entry points, types and enum values as the reference's public C API
 * (band/c/c_api.h:47-190, band/c/c_api_type.h:27-196), so a client built
 * against Band's C header links against this library unchanged.  The
 * engine behind it is the native harness in band_amd/csrc/engine (planner,
 * workers, schedulers, latency estimator, model analyzer) with the HIP
 * backend registered under kBandTfLite.
 *
 * Differences a client can observe:
 *   - BandEngineRequestAsync* return -1 on failure (the reference aborts
 *     in StatusOr::value(), band/c/c_api.cc:512-521);
 *   - Bandx* functions at the end are extensions (job records, profile
 *     persistence, the benchmark driver); the reference has no equivalent
 *     C entry points.
 * Status mapping follows the reference: only an internal error is kBandErr;
 * an SLO violation (DeadlineExceeded) is reported as kBandOk
 * (band/c/c_api.cc:33-47).
 */
#ifndef BAND_HIP_C_API_H_
#define BAND_HIP_C_API_H_

#include <stdarg.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#define BAND_CAPI_EXPORT __attribute__((visibility("default")))

#ifdef __cplusplus
extern "C" {
#endif

typedef enum BandLogSeverity { kBandInternal = 0, kBandInfo, kBandWarning, kBandError, kBandLogNumSeverities } BandLogSeverity;
typedef enum BandBackendType { kBandTfLite = 0, kBandNumBackendType } BandBackendType;
typedef enum BandStatus { kBandOk = 0, kBandErr, kBandDelegateErr } BandStatus;
typedef enum BandWorkerType { kBandDeviceQueue = 1 << 0, kBandGlobalQueue = 1 << 1 } BandWorkerType;
typedef enum BandSchedulerType {
  kBandFixedWorker = 0,
  kBandRoundRobin,
  kBandShortestExpectedLatency,
  kBandFixedWorkerGlobalQueue,
  kBandHeterogeneousEarliestFinishTime,
  kBandLeastSlackTimeFirst,
  kBandHeterogeneousEarliestFinishTimeReserved,
  kBandNumSchedulerType
} BandSchedulerType;
typedef enum BandCPUMaskFlag { kBandAll = 0, kBandLittle, kBandBig, kBandPrimary, kBandNumCpuMask } BandCPUMaskFlag;
typedef enum BandSubgraphPreparationType {
  kBandNoFallbackSubgraph = 0,
  kBandFallbackPerWorker,
  kBandUnitSubgraph,
  kBandMergeUnitSubgraph,
  kBandNumSubgraphPreparationType
} BandSubgraphPreparationType;
typedef enum {
  kBandNoType = 0,
  kBandFloat32,
  kBandInt32,
  kBandUInt8,
  kBandInt64,
  kBandString,
  kBandBool,
  kBandInt16,
  kBandComplex64,
  kBandInt8,
  kBandFloat16,
  kBandFloat64,
  kBandNumDataType,
} BandDataType;
typedef enum BandQuantizationType { kBandNoQuantization = 0, kBandAffineQuantization, kBandNumQuantizationType } BandQuantizationType;
typedef enum BandDeviceFlag { kBandCPU = 0, kBandGPU, kBandDSP, kBandNPU, kBandNumDeviceFlag } BandDeviceFlag;
typedef enum BandConfigField {
  BAND_PROFILE_ONLINE = 0,
  BAND_PROFILE_NUM_WARMUPS,
  BAND_PROFILE_NUM_RUNS,
  BAND_PROFILE_SMOOTHING_FACTOR,
  BAND_PROFILE_DATA_PATH,
  BAND_PLANNER_SCHEDULE_WINDOW_SIZE,
  BAND_PLANNER_SCHEDULERS,
  BAND_PLANNER_CPU_MASK,
  BAND_PLANNER_LOG_PATH,
  BAND_WORKER_WORKERS,
  BAND_WORKER_CPU_MASKS,
  BAND_WORKER_NUM_THREADS,
  BAND_WORKER_ALLOW_WORKSTEAL,
  BAND_WORKER_AVAILABILITY_CHECK_INTERVAL_MS,
  BAND_MINIMUM_SUBGRAPH_SIZE,
  BAND_SUBGRAPH_PREPARATION_TYPE,
  BAND_CPU_MASK,
  BAND_RESOURCE_MONITOR_DEVICE_PATH,
  BAND_RESOURCE_MONITOR_INTERVAL_MS,
  BAND_RESOURCE_MONITOR_LOG_PATH,
  /* extension: a GPU device-queue worker runs up to this many queued
   * whole-model jobs of one model as one batched pass (default 1 = Band) */
  BANDX_WORKER_MAX_JOB_BATCH = 1000,
  /* int: 1 = workers of one device kind (same device flag, thread count and
   * CPU mask: e.g. several GPU workers of one node) share latency estimates */
  BANDX_PROFILE_SHARE_IDENTICAL = 1001,
  /* int, microseconds (default 0 = off): pass-size policy of job batching -
   * a model's batched pass takes at most the jobs whose expected pass time
   * stays within this target (its largest batch variant timed once at
   * registration, pass time taken as linear in the jobs), at least 1 */
  BANDX_WORKER_PASS_TARGET_US = 1002,
} BandConfigField;

typedef struct BandRequestOption {
  int target_worker;
  bool require_callback;
  int slo_us;
  float slo_scale;
} BandRequestOption;

typedef struct BandConfigBuilder BandConfigBuilder;
typedef struct BandConfig BandConfig;
typedef struct BandModel BandModel;
typedef struct BandTensor BandTensor;
typedef struct BandEngine BandEngine;
typedef int BandRequestHandle;
typedef int BandCallbackHandle;

/* logging */
BAND_CAPI_EXPORT void BandSetLogSeverity(BandLogSeverity severity);
BAND_CAPI_EXPORT BandCallbackHandle BandSetLogReporter(void (*reporter)(BandLogSeverity severity, const char* msg));
BAND_CAPI_EXPORT void BandUnsetLogReporter(BandCallbackHandle handle);

/* config builder: BandAddConfig(b, field, count, values...) as in
 * band/c/c_api.cc:86-196 */
BAND_CAPI_EXPORT BandConfigBuilder* BandConfigBuilderCreate(void);
BAND_CAPI_EXPORT void BandAddConfig(BandConfigBuilder* b, int field, int count, ...);
BAND_CAPI_EXPORT void BandConfigBuilderDelete(BandConfigBuilder* b);
BAND_CAPI_EXPORT BandConfig* BandConfigCreate(BandConfigBuilder* b);
BAND_CAPI_EXPORT void BandConfigDelete(BandConfig* config);

/* model */
BAND_CAPI_EXPORT BandModel* BandModelCreate(void);
BAND_CAPI_EXPORT void BandModelDelete(BandModel* model);
BAND_CAPI_EXPORT BandStatus BandModelAddFromBuffer(BandModel* model, BandBackendType backend_type,
                                                   const void* model_data, size_t model_size);
BAND_CAPI_EXPORT BandStatus BandModelAddFromFile(BandModel* model, BandBackendType backend_type,
                                                 const char* model_path);

/* tensor */
BAND_CAPI_EXPORT void BandTensorDelete(BandTensor* tensor);
BAND_CAPI_EXPORT BandDataType BandTensorGetType(BandTensor* tensor);
BAND_CAPI_EXPORT void* BandTensorGetData(BandTensor* tensor);
BAND_CAPI_EXPORT size_t BandTensorGetNumDims(BandTensor* tensor);
BAND_CAPI_EXPORT const int* BandTensorGetDims(BandTensor* tensor);
BAND_CAPI_EXPORT size_t BandTensorGetBytes(BandTensor* tensor);
BAND_CAPI_EXPORT const char* BandTensorGetName(BandTensor* tensor);
BAND_CAPI_EXPORT BandQuantizationType BandTensorGetQuantizationType(BandTensor* tensor);
BAND_CAPI_EXPORT void* BandTensorGetQuantizationParams(BandTensor* tensor);

/* request option */
BAND_CAPI_EXPORT BandRequestOption BandRequestOptionGetDefault(void);

/* engine */
BAND_CAPI_EXPORT BandEngine* BandEngineCreateWithDefaultConfig(void);
BAND_CAPI_EXPORT BandEngine* BandEngineCreate(BandConfig* config);
BAND_CAPI_EXPORT void BandEngineDelete(BandEngine* engine);
BAND_CAPI_EXPORT BandStatus BandEngineRegisterModel(BandEngine* engine, BandModel* model);
BAND_CAPI_EXPORT int BandEngineGetNumInputTensors(BandEngine* engine, BandModel* model);
BAND_CAPI_EXPORT int BandEngineGetNumOutputTensors(BandEngine* engine, BandModel* model);
BAND_CAPI_EXPORT int BandEngineGetNumWorkers(BandEngine* engine);
BAND_CAPI_EXPORT BandDeviceFlag BandEngineGetWorkerDevice(BandEngine* engine, int worker_id);
BAND_CAPI_EXPORT BandTensor* BandEngineCreateInputTensor(BandEngine* engine, BandModel* model, size_t index);
BAND_CAPI_EXPORT BandTensor* BandEngineCreateOutputTensor(BandEngine* engine, BandModel* model, size_t index);
BAND_CAPI_EXPORT BandStatus BandEngineRequestSync(BandEngine* engine, BandModel* model, BandTensor** input_tensors,
                                                  BandTensor** output_tensors);
BAND_CAPI_EXPORT BandRequestHandle BandEngineRequestAsync(BandEngine* engine, BandModel* model,
                                                          BandTensor** input_tensors);
BAND_CAPI_EXPORT BandStatus BandEngineRequestSyncOptions(BandEngine* engine, BandModel* model,
                                                         BandRequestOption options, BandTensor** input_tensors,
                                                         BandTensor** output_tensors);
BAND_CAPI_EXPORT BandRequestHandle BandEngineRequestAsyncOptions(BandEngine* engine, BandModel* model,
                                                                 BandRequestOption options,
                                                                 BandTensor** input_tensors);
BAND_CAPI_EXPORT BandStatus BandEngineWait(BandEngine* engine, BandRequestHandle handle, BandTensor** output_tensors,
                                           size_t num_outputs);
// The finished request's output slot stays held until its callbacks
// return.  A callback that blocks on a newer request of the same model
// (BandEngineRequestSync / BandEngineWait) may need that slot: the worker
// writing it waits at most BANDX_OUTPUT_HOLD_MS (default 2000) and then
// fails that request (kBandErr) instead of deadlocking.  Callbacks should
// return promptly and not wait on the same model's requests.
BAND_CAPI_EXPORT BandCallbackHandle BandEngineSetOnEndRequest(BandEngine* engine,
                                                              void (*on_end_invoke)(void* user_data,
                                                                                    BandRequestHandle job_id,
                                                                                    BandStatus status),
                                                              void* user_data);
BAND_CAPI_EXPORT BandStatus BandEngineUnsetOnEndRequest(BandEngine* engine, BandCallbackHandle callback_handle);

/* ---- extensions (no reference counterpart) ---- */

/* the planner's record of a finished job (band/common.h:333-378 fields);
 * returns kBandErr when the job is unknown or not finished */
typedef struct BandxJobRecord {
  int job_id;
  int model_id;
  int worker_id;
  int status; /* band::JobStatus: 0 EnqueueFailed .. 6 InvokeFailure */
  int64_t enqueue_time_us;
  int64_t invoke_time_us;
  int64_t end_time_us;
  int64_t expected_latency_us;
  int64_t slo_us;
  uint64_t unit_indices; /* bit mask of the last subgraph's unit indices */
} BandxJobRecord;
BAND_CAPI_EXPORT BandStatus BandxEngineGetJobRecord(BandEngine* engine, BandRequestHandle handle,
                                                    BandxJobRecord* record);
/* the model id behind a BandModel (job records carry it) */
BAND_CAPI_EXPORT int BandxModelGetId(BandModel* model);
/* latency profile database as JSON text (reference layout, see
 * latency_estimator.h); returns the full length, writes at most cap bytes */
BAND_CAPI_EXPORT size_t BandxEngineGetProfileJson(BandEngine* engine, char* buf, size_t cap);
BAND_CAPI_EXPORT BandStatus BandxEngineDumpProfile(BandEngine* engine);
/* subgraph keys prepared for a model: up to cap (worker_id, unit mask)
 * pairs; returns the total count */
BAND_CAPI_EXPORT int BandxEngineGetSubgraphs(BandEngine* engine, BandModel* model, int* worker_ids,
                                             uint64_t* unit_masks, int cap);
/* expected latency (us) the estimator holds for one subgraph */
BAND_CAPI_EXPORT int64_t BandxEngineGetExpectedLatency(BandEngine* engine, BandModel* model, int worker_id,
                                                       uint64_t unit_mask);
/* blocks until every submitted job finished */
BAND_CAPI_EXPORT void BandxEngineWaitAll(BandEngine* engine);
/* jobs (subgraph executions) worker `worker_id` has finished since the
 * engine started, each job of a batched pass counted once; -1 for a bad id.
 * A model split over workers counts once per subgraph on each worker. */
BAND_CAPI_EXPORT int64_t BandxEngineGetWorkerJobCount(BandEngine* engine, int worker_id);
/* host time of worker `worker_id`'s job phases since the engine started:
 * out[0] input copies (request ring -> executor), out[1] invoke (launch +
 * device sync), out[2] output copies (executor -> output ring), all in
 * microseconds, and out[3] the passes run (a batched pass counts once).
 * Returns 0, or -1 for a bad id. */
BAND_CAPI_EXPORT int BandxEngineGetWorkerPhaseTimes(BandEngine* engine, int worker_id, int64_t out[4]);
/* the last BandxEngineRunClosedLoop / BandxEngineRunPoisson call: out[0] its
 * wall time (us), out[1] the mean requests inside the engine (submitted, not
 * yet finished), out[2] the mean finished requests waiting for a reader,
 * out[3] / out[4] submitter time waiting for a free slot / inside
 * RequestAsync, out[5] / out[6] reader time reading / waiting (us, summed
 * over threads), out[7] readers + 1000 x submitters.  Returns 0. */
BAND_CAPI_EXPORT int BandxEngineGetDriverStats(BandEngine* engine, double out[8]);
/* Cumulative RequestAsync cost split since the engine was created:
 * out = {jobs submitted, us waiting for request-ring slots, us copying
 * inputs into them, us enqueueing to the planner}. */
BAND_CAPI_EXPORT int BandxEngineGetRequestPhaseTimes(BandEngine* engine, int64_t out[4]);
/* One RequestAsync call for n requests (band/engine.cc:455-529, the batched
 * overload Band's own benchmark tool uses): request i runs models[i] on the
 * input tensors inputs[i] (that model's inputs, in order).  handles[i]
 * receives each job id.  A run of consecutive same-model requests larger
 * than that model's request ring is refused (kBandErr, nothing submitted). */
BAND_CAPI_EXPORT BandStatus BandxEngineRequestsAsync(BandEngine* engine, BandModel** models, int n,
                                                     BandTensor*** inputs, BandRequestHandle* handles);

/* Closed-loop request driver: submits exactly n_jobs requests, round-robin
 * over the n_models models (model j % n_models), with at most max_inflight
 * outstanding, and waits for all of them.  Inputs are the engine-created
 * tensors of each model (caller fills them first, or NULL for zeros).
 * A model never has more outstanding requests than its request ring holds
 * (128), so no result is overwritten before it is read.
 * latency_us[j] = end - enqueue of job j (band/common.h:351-353);
 * worker_ids[j] = worker that ran its last subgraph (may be NULL);
 * *wall_s = submission of the first job to completion of the last.
 * Jobs are submitted and read by BANDX_DRIVER_LANES (default 4) pairs of
 * submitter / waiter threads, job j on lane j % lanes. */
BAND_CAPI_EXPORT BandStatus BandxEngineRunClosedLoop(BandEngine* engine, BandModel** models, BandTensor** inputs,
                                                     int n_models, int n_jobs, int max_inflight, double* latency_us,
                                                     int* worker_ids, double* wall_s);
/* the same, and model_index[j] = the index into `models` of job j (may be
 * NULL): the per-model statistics key on it, not on an assumed burst */
BAND_CAPI_EXPORT BandStatus BandxEngineRunClosedLoopEx(BandEngine* engine, BandModel** models, BandTensor** inputs,
                                                       int n_models, int n_jobs, int max_inflight, double* latency_us,
                                                       int* worker_ids, int* model_index, double* wall_s);

/* Open-loop Poisson driver (BASELINE config C5): n_jobs arrivals with
 * exponential inter-arrival times at rate_per_s (all models together, seeded
 * std::mt19937_64), each arrival a model drawn uniformly; arrivals beyond
 * max_inflight outstanding wait for a completion, and so do arrivals of a
 * model with a full request ring (128 requests).  latency_us[j] = end - the
 * SCHEDULED arrival of job j, so submission delays count as queueing (no
 * coordinated omission).  Other outputs as BandxEngineRunClosedLoop. */
BAND_CAPI_EXPORT BandStatus BandxEngineRunPoisson(BandEngine* engine, BandModel** models, BandTensor** inputs,
                                                  int n_models, int n_jobs, double rate_per_s, uint64_t seed,
                                                  int max_inflight, double* latency_us, int* worker_ids,
                                                  int* model_index, double* wall_s);

/* The benchmark tool (band/tool/benchmark.cc) driven by a JSON config in the
 * reference's format (band/test/data/benchmark_config.json: "models",
 * "schedulers", "workers", "execution_mode" periodic|stream|workload, ...).
 * Writes a JSON result (per-model request counts, latency mean/p50/p99,
 * SLO satisfaction, throughput) into out (at most cap bytes); returns the
 * full length of the result, or 0 on error (message in the result). */
BAND_CAPI_EXPORT size_t BandxBenchmarkRun(const char* config_json, char* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* BAND_HIP_C_API_H_ */
