// HipModelExecutor: the IModelExecutor of the HIP backend - the drop-in for
// band/backend/tfl/model_executor.{h,cc} (TfLiteModelExecutor).
//
// Reference contract (file:line in /root/reference):
//   InvestigateModelSpec   band/backend/tfl/model_executor.cc:48-171
//   PrepareSubgraph        :173-192 (+ CreateTfLiteInterpreter :327-373)
//   GetInputs/Outputs/...  :198-224
//   GetTensorView          :226-229
//   GetLargestSubgraphKey / HasSubgraph / ForEachSubgraph :231-262
//   ExecuteSubgraph        :249-255  <- Engine::Invoke band/engine.cc:843-850
//
// MI355X design: one executor per (model, worker); weights, requantisation
// tables and an activation arena are resident in HBM; subgraph boundary
// tensors have host-pinned mirrors that Band memcpy's through GetData();
// ExecuteSubgraph = H2D inputs -> kernel sequence -> D2H outputs on the
// worker's stream, replayed from a hipGraph after the first run, and returns
// only when the results are on the host (Band timestamps right after,
// band/worker.cc:274-291).
#pragma once

#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "backend/hip/coalescer.h"
#include "backend/hip/cpu_kernels.h"
#include "backend/hip/device.h"
#include "backend/hip/model.h"
#include "backend/hip/tensor.h"
#include "backend/hip/job_batching.h"
#include "band/interface/model_executor.h"
#include "band_hip_kernels.h"

namespace band {
namespace hip {

struct Launch {
  enum Kind {
    kConv, kDwConv, kFc, kEltwise, kPool, kCopy, kIrb, kChain,
    kLutU8, kLutF32, kQuantF32, kConcat, kPad, kResizeNearest, kResizeBilinear, kSoftmax, kZeroInsert,
    kConvF32, kFcF32, kEltwiseF32, kPoolF32, kUnaryF32, kSoftmaxF32,  // float32 graphs
    kResizeBilinearU8,
    kDetectionPost,  // CPU-only TFLite_Detection_PostProcess
    kMean,           // CPU-only MEAN
    kConvGroup       // independent small convs in one dispatch (GroupConvs)
  } kind;
  int op_index = -1;
  int out_tensor = -1;  // tensor this launch materialises (after epilogue fusions)
  bh_conv_params conv{};
  bh_dwconv_params dw{};
  bh_fc_params fc{};
  bh_eltwise_params elt{};
  bh_pool_params pool{};
  bh_irb_params irb{};
  bh_chain_params chain{};
  // kConvGroup: the member convs (program order) and the planned group
  std::vector<bh_conv_params> members;
  bh_conv_group cgroup{};
  bh_concat_params concat{};
  bh_pad_params pad{};
  bh_resize_nearest_params rnear{};
  bh_resize_bilinear_params rbil{};
  bh_resize_bilinear_u8_params rbil8{};
  bh_softmax_params softmax{};
  bh_zero_insert_params zi{};
  bh_conv_f32_params convf{};
  bh_fc_f32_params fcf{};
  bh_eltwise_f32_params eltf{};
  bh_pool_f32_params poolf{};
  int unary_kind = 0;
  float lo = 0.f, hi = 0.f, beta = 1.f;
  int depth = 0;
  CpuDetectionParams det{};
  CpuMeanParams mean{};
  const void* table = nullptr;  // kLutU8 / kLutF32: 256-entry device table
  long count = 0;               // kLut* / kQuantF32: elements
  float q_scale = 0.f;          // kQuantF32
  int32_t q_zp = 0;
  int q_signed = 0;
  void* dst = nullptr;
  const void* src = nullptr;
  size_t bytes = 0;
  double alg_bytes = 0;  // algorithmic HBM bytes per launch (roofline numerator)
  double alg_ops = 0;    // algorithmic int ops (2 per MAC)
  const char* kernel = "";
};

struct OpTiming {
  int op_index;
  const char* kernel;
  double ms;
  double alg_bytes;
  double alg_ops;
};

struct PreparedSubgraph {
  std::vector<int> ops;
  std::vector<int> inputs, outputs;
  bool model_order_io = false;   // prepared with ops = {}: the model's own I/O order
  std::map<int, size_t> offset;  // arena offset of each non-constant tensor
  std::shared_ptr<DeviceBlob> arena;
  std::map<int, std::unique_ptr<PinnedBuffer>> host;  // boundary mirrors
  std::set<int> extra_d2h;                            // intermediates a view asked for
  std::set<int> fused_ops;      // ADD/SUB ops folded into the producing conv's epilogue
  std::set<int> fused_tensors;  // conv outputs that are therefore never materialised
  std::set<int> no_fuse;        // tensors a view needs materialised
  std::vector<Launch> launches;
  std::vector<std::shared_ptr<DeviceBlob>> consts;
  bh_graph_exec_t graph = nullptr;
  bool io_in_graph = true;  // the graph holds the host copies (set at capture)
  // with io_in_graph: the captured graph and its host-copy nodes, so a
  // one-job pass can point them at the request rings' slots
  // (ExecuteJobBatchDirect, n == 1) and back at the host mirrors
  void* graph_tmpl = nullptr;
  struct IoNode {
    void* node;
    int tensor;
    bool h2d;
  };
  std::vector<IoNode> io_nodes;
  bool io_retargeted = false;  // the nodes point at ring slots
  int runs = 0;
  // poll-wait (BAND_HIP_SYNC=poll): running mean of a pass's device time as
  // the waiting thread saw it (us), so it sleeps through most of the next one
  double wait_us = 0.0;
};

class HipModelExecutor : public interface::IModelExecutor, public IJobBatching {
 public:
  HipModelExecutor(ModelId model_id, WorkerId worker_id, DeviceFlag device_flag,
                   CpuSet thread_affinity_mask, int num_threads);
  ~HipModelExecutor() override;

  absl::StatusOr<ModelSpec> InvestigateModelSpec(interface::IModel* model) override;
  absl::Status PrepareSubgraph(interface::IModel* model, std::set<int> ops = {},
                               std::set<int> unit_indices = {}) override;
  BackendType GetBackendType() const override { return BackendType::kTfLite; }
  const std::vector<int>& GetInputs(const SubgraphKey& key) const override;
  const std::vector<int>& GetOutputs(const SubgraphKey& key) const override;
  const char* GetInputName(const SubgraphKey& key, int index) const override;
  const char* GetOutputName(const SubgraphKey& key, int index) const override;
  size_t GetNumTensors(const SubgraphKey& key) const override;
  size_t GetNumNodes(const SubgraphKey& key) const override;
  std::shared_ptr<interface::ITensorView> GetTensorView(const SubgraphKey& key, int index) override;
  bool HasSubgraph(const SubgraphKey& key) const override;
  SubgraphKey GetLargestSubgraphKey() const override;
  absl::Status ExecuteSubgraph(const SubgraphKey& key) override;
  void ForEachSubgraph(std::function<void(const SubgraphKey&)> visitor) override;

  // --- job batching (backend/hip/job_batching.h; kGPU executors) ---
  // A variant for every batch 2 .. max_batch (BAND_HIP_BATCH_STEP, default
  // 1), so a pass of n jobs computes exactly n images: each is an executor
  // of a batch-B copy of the model (HipModel::CloneWithJobBatch) over the
  // same op set, on this executor's stream, sharing its device weights.  All
  // variants of one subgraph share ONE activation arena and one set of
  // page-locked boundary mirrors, sized for max_batch (a worker runs one
  // pass at a time).  Measured fusion choices are taken at the anchor
  // batches 2, 4, 8, 16, .., max_batch and reused by the sizes between.
  absl::Status PrepareJobBatches(interface::IModel* model, const SubgraphKey& key, int max_batch) override;
  int MaxJobBatch(const SubgraphKey& key) const override;
  std::shared_ptr<interface::ITensorView> GetJobSlotView(const SubgraphKey& key, int index, int n,
                                                         int slot) override;
  absl::Status ExecuteJobBatch(const SubgraphKey& key, int n) override;
  absl::Status ExecuteJobBatchDirect(const SubgraphKey& key, int n, const std::vector<const interface::ITensor*>& in,
                                     const std::vector<interface::ITensor*>& out) override;

  // --- extensions used by the C ABI / bench (not part of Band's interface) ---
  void SetUseGraph(bool on) { use_graph_ = on; }
  // Times every launch of `key` with HIP events on the executor's stream
  // (eager enqueue in program order, averaged over `iters`); *floor_us = the
  // per-launch time of an equal chain of empty launches (event + dispatch
  // + gap), what an event figure holds beyond the kernel itself.
  absl::Status ProfileSubgraph(const SubgraphKey& key, int iters, std::vector<OpTiming>* out,
                               double* floor_us = nullptr);
  // Device time of one subgraph pass (us) with `iters` passes issued back to
  // back (replayed hipGraph when captured, else the launch sequence): no host
  // gaps, H2D/D2H included.  The latency floor of ExecuteSubgraph's device side.
  absl::Status TimeSubgraph(const SubgraphKey& key, int iters, double* us);
  int ordinal() const { return ordinal_; }
  // the coalescer this executor's whole-model subgraph joined (null: none)
  const JobCoalescer* coalescer() const { return coalescer_.get(); }

  // Whether the GPU kernel set covers `op` of `model` (drives unsupported_ops[kGPU]).
  static bool GpuSupports(const TflModel& model, const TflOperator& op, std::string* why);
  // The kCPU worker's set: the GPU set plus host-only ops (float graphs).
  static bool CpuSupports(const TflModel& model, const TflOperator& op, std::string* why);

 private:
  friend class JobCoalescer;
  PreparedSubgraph* Find(const SubgraphKey& key) const;
  // one batch-1 pass of sg on this executor's stream (graph captured on the
  // second run), returning when its outputs are in the host mirrors
  absl::Status RunPass(PreparedSubgraph* sg);
  // a private executor of this one's model on this GPU with a stream of its
  // own, for a coalescer lane (never joins a coalescer itself)
  std::unique_ptr<HipModelExecutor> MakeLane();
  absl::Status EnsureMeta(const HipModel& model);
  absl::Status Lower(const HipModel& model, int op_index, PreparedSubgraph* sg);
  absl::Status BuildLaunches(const HipModel& model, PreparedSubgraph* sg);
  bool TryFuseResidualAdd(const HipModel& model, int conv_op, PreparedSubgraph* sg, Launch* l);
  void FuseBlocks(const HipModel& model, PreparedSubgraph* sg);
  // dw3x3 -> conv1x1 [+ADD] [-> conv1x1] runs into one bh_chain_i8 launch
  bool PackChainTile(bh_chain_params* q, PreparedSubgraph* sg);
  void FuseChains(const HipModel& model, PreparedSubgraph* sg);
  // 8-bit unary table ops into the producing conv / FC / depthwise epilogue;
  // CONCATENATION with outer size 1 elided (producers write their slices)
  void FuseGlue(const HipModel& model, PreparedSubgraph* sg);
  // independent small convs (detector / pose heads) deferred past later
  // launches that do not touch them and issued as one conv_group launch
  absl::Status GroupConvs(PreparedSubgraph* sg);
  // Mean device time (us) of one pass over `ls`, or < 0 when it cannot be
  // measured (no GPU stream, or a launch failed).
  double TimeLaunches(const std::vector<const Launch*>& ls, int iters);
  absl::Status DevicePtr(const HipModel& model, int tensor, PreparedSubgraph* sg, void** ptr);
  // host-built constant (table) resident on this executor's device, shared
  // across executors by `key`
  absl::Status UploadConst(const std::string& key, const void* data, size_t bytes, PreparedSubgraph* sg,
                           const void** dev);
  absl::Status LowerFloat(const HipModel& model, int op_index, void* in_ptr, void* out_ptr, const std::string& ckey,
                          PreparedSubgraph* sg, Launch* l, bool* emit);
  absl::Status LowerTransposeConv(const HipModel& model, int op_index, void* out_ptr, const std::string& ckey,
                                  PreparedSubgraph* sg, Launch* l);
  absl::Status LowerGlue(const HipModel& model, int op_index, void* in_ptr, void* out_ptr, const std::string& ckey,
                         PreparedSubgraph* sg, Launch* l);
  absl::Status Enqueue(PreparedSubgraph* sg);
  // Enqueue's three parts: host->device inputs, the launches, device->host
  // outputs (and intermediates a later subgraph reads)
  absl::Status EnqueueInputs(PreparedSubgraph* sg);
  absl::Status EnqueueLaunches(PreparedSubgraph* sg);
  absl::Status EnqueueOutputs(PreparedSubgraph* sg);
  // one pass: the graph (captured on first use) or the eager launches
  absl::Status EnqueuePass(PreparedSubgraph* sg);
  // captures sg's pass into its graph (host copies inside when io_in_graph)
  absl::Status CaptureGraph(PreparedSubgraph* sg);
  // one eager pass of the kernels, then the graph capture a second pass
  // would do (PrepareJobBatches: no variant captures in the serving path)
  absl::Status PrecaptureGraph(PreparedSubgraph* sg);
  // drops sg's graph (and its captured template / copy nodes)
  void DropGraph(PreparedSubgraph* sg);
  // points sg's graph copy nodes at the host mirrors again
  absl::Status RestoreIoNodes(PreparedSubgraph* sg);
  // a job-batch variant's pass with each job's I/O copied straight between
  // host tensors and its slot of the boundary tensors (per_job: the
  // batch-1 bytes of each input, then of each output)
  absl::Status RunDirect(PreparedSubgraph* sg, int n, const std::vector<size_t>& per_job,
                         const std::vector<const interface::ITensor*>& in, const std::vector<interface::ITensor*>& out);
  absl::Status ExecuteOnHost(PreparedSubgraph* sg);
  absl::Status EnqueueLaunch(const Launch& l);

  struct JobBatchVariant {
    int batch = 1;
    std::unique_ptr<HipModel> model;
    std::unique_ptr<HipModelExecutor> exec;
  };
  // variant running n jobs (smallest batch >= n), or null
  const JobBatchVariant* VariantFor(const SubgraphKey& key, int n) const;
  std::map<SubgraphKey, std::vector<JobBatchVariant>> job_batches_;  // ascending batch

  const HipModel* model_ = nullptr;
  std::vector<std::unique_ptr<TensorMeta>> meta_;
  std::vector<std::vector<int>> consumers_;  // tensor -> ops reading it (whole model)
  std::vector<int> producer_;                // tensor -> op writing it (-1: input / constant)
  bool allow_fusion_ = true;
  bool allow_irb_ = true;  // BAND_HIP_FUSION=noirb / noadd: diagnostics
  bool allow_add_ = true;
  bool allow_chain_ = true;   // BAND_HIP_FUSION=nochain
  bool allow_group_ = true;   // BAND_HIP_FUSION=nogroup: one launch per conv
  bool force_chain_ = false;  // BAND_HIP_FUSION=forcechain
  bool force_tile_chain_ = false;  // BAND_HIP_FUSION=forcetile: every feasible chain in the tile form
  bool no_tile_chain_ = false;     // BAND_HIP_FUSION=notile: the tuner skips the tile form
  bool no_deep_chain_ = false;     // BAND_HIP_FUSION=nodeep: the tuner skips the deep-issue forms
  bool no_split_chain_ = false;    // BAND_HIP_FUSION=nosplit: the tuner skips the phase-C split forms
  bool force_deep_chain_ = false;  // BAND_HIP_FUSION=forcedeep: every feasible chain in the deep form
  bool force_stage_chain_ = false; // BAND_HIP_FUSION=forcestage: every chain the stage form takes, in it (parity)
  bool no_stage_chain_ = false;    // BAND_HIP_FUSION=nostage: the tuner skips the stage forms
  bool autotune_ = true;  // BAND_HIP_AUTOTUNE=0: pick fused tiles by the static model
  std::map<SubgraphKey, std::unique_ptr<PreparedSubgraph>> subgraphs_;
  int ordinal_ = -1;
  bh_stream_t stream_ = nullptr;
  std::shared_ptr<CpuPool> cpu_pool_;  // kCPU executors (shared with their job-batch variants)
  bool use_graph_ = true;
  // Where a graph pass's host copies go: captured into the graph (blit
  // kernels on the compute queue; lowest latency for small transfers) or
  // issued on the stream around a kernels-only graph (DMA engines, leaving
  // the CUs to the kernels of concurrent passes).  BAND_HIP_IO = graph |
  // stream | auto (default: stream from io_stream_bytes_ of host I/O per
  // pass, BAND_HIP_IO_STREAM_BYTES)
  int io_mode_ = 2;  // 0 graph, 1 stream, 2 auto
  // How a pass is waited for.  spin (BAND_HIP_SYNC=spin): hipStreamSynchronize, which
  // busy-polls - a core per GPU worker for the whole pass, and the lowest
  // completion latency.  block (BAND_HIP_SYNC=block): a blocking-sync event.
  // poll (BAND_HIP_SYNC=poll): the thread sleeps through most of the pass's
  // expected device time, then polls the pass's event every few us
  // (WaitPass).  On the C3 mix poll frees ~7 cores but the late wake-ups
  // cost 15-20 % of throughput, and block still spins inside HIP
  // (profiles/r04e_*: spin 83 / 94 k, poll 76 / 78 k, block 79 / 80 k).
  // poller (BAND_HIP_SYNC=poller): the thread parks on a condition variable
  // and the GPU's CompletionPoller thread (completion.h) wakes it when the
  // pass's event completes - one polling core per GPU instead of one per
  // waiting thread.
  // adaptive (default since round 5; BAND_HIP_SYNC=spin restores spinning):
  // sleep through BAND_HIP_SYNC_SLEEP (default 0.85) of the pass's expected
  // wait, then spin (WaitPass).  C3 headline, interleaved on one box
  // (profiles/r05p_*): spin 109.8k / 103.4k inf/s at 8.9 / 8.7 process
  // cores; adaptive 0.7 109.1k / 110.0k at 4.5 / 4.2; 0.85 108.4k / 109.6k
  // at 4.1 / 4.0 (one of them the request driver's submitter thread).
  enum SyncMode { kSyncSpin = 0, kSyncBlock = 1, kSyncPoll = 2, kSyncPoller = 3, kSyncAdaptive = 4 };
  int sync_mode_ = kSyncAdaptive;
  double sleep_frac_ = 0.85;
  double sleep_min_us_ = 500.0;  // BAND_HIP_SYNC_MIN_US: expected waits below this spin
  bool block_sync_ = false;  // sync_mode_ == kSyncBlock
  // waits for everything enqueued on stream_ (the pass of `sg`)
  absl::Status WaitPass(PreparedSubgraph* sg);
  // batched passes copy each job's I/O straight between the request rings'
  // page-locked slots and the device (ExecuteJobBatchDirect);
  // BAND_HIP_DIRECT_IO=0 stages them through the slot views instead
  bool direct_io_ = true;
  bh_event_t done_event_ = nullptr;
  size_t io_stream_bytes_ = 512 << 10;
  // job-batch variants: the arena / boundary mirrors of the largest variant
  // (PrepareSubgraph uses them when big enough), and the anchor batch whose
  // measured fusion choices this variant reuses (0: its own batch)
  std::shared_ptr<DeviceBlob> shared_arena_;
  const PreparedSubgraph* shared_host_from_ = nullptr;
  int tune_batch_ = 0;
  // Job coalescing (coalescer.h): whole-model kGPU subgraphs join the
  // coalescer of their (model, GPU); concurrent ExecuteSubgraph calls of
  // several executors then run as job-batch passes.  BAND_HIP_COALESCE = max
  // jobs per pass (default 16; 0 or 1: off), BAND_HIP_COALESCE_LANES =
  // passes in flight per (model, GPU) (default 2).  Off for lanes, job-batch
  // variants, and executors the harness batches itself (PrepareJobBatches).
  std::shared_ptr<JobCoalescer> coalescer_;
  SubgraphKey coalesced_key_;
  bool coalesce_ok_ = true;
  int coalesce_max_ = 16;
  int coalesce_lanes_ = 2;
  bh_stream_t owned_stream_ = nullptr;  // a lane's own stream
  static const std::vector<int> kEmpty;
};

}  // namespace hip
}  // namespace band
