// HipModelExecutor: the IModelExecutor of the HIP backend (model_executor.h):
// construction, the op-set support checks, InvestigateModelSpec,
// PrepareSubgraph, the metadata getters and views, and execution (graph
// capture / replay, host copies, waits, profiling).  The lowering lives in
// lower.cc, the fusion passes in fusion.cc, job batching in job_batch.cc.
#include "backend/hip/model_executor.h"

#include <sys/prctl.h>
#include <time.h>

#include <chrono>
#include <limits>
#include <mutex>
#include <unordered_map>

#include "backend/hip/affinity.h"
#include "backend/hip/completion.h"
#include "backend/hip/executor_internal.h"

namespace band {
namespace hip {

using namespace ex;

namespace ex {
thread_local bool t_variant_ctor = false;
}  // namespace ex


const std::vector<int> HipModelExecutor::kEmpty;

HipModelExecutor::HipModelExecutor(ModelId model_id, WorkerId worker_id, DeviceFlag device_flag,
                                   CpuSet mask, int num_threads)
    : IModelExecutor(model_id, worker_id, device_flag, mask, num_threads) {
  if (device_flag_ == DeviceFlag::kGPU && DeviceRegistry::Get().GpuAvailable()) {
    ordinal_ = DeviceRegistry::Get().OrdinalForWorker(worker_id_);
    stream_ = DeviceRegistry::Get().StreamForWorker(worker_id_);
  } else if (device_flag_ == DeviceFlag::kCPU && !t_variant_ctor) {
    // host execution of the lowered program (cpu_kernels.h), pinned to the
    // executor's CpuSet when it names a proper subset of the process's CPUs
    // (affinity.h PinnableCpus); job-batch variants share their base
    // executor's pool instead (PrepareJobBatches)
    cpu_pool_ = std::make_shared<CpuPool>(num_threads_ > 0 ? num_threads_ : 1, PinnableCpus(thread_affinity_mask_));
  }
  const char* g = std::getenv("BAND_HIP_GRAPH");
  if (g && g[0] == '0') use_graph_ = false;
  if (const char* io = std::getenv("BAND_HIP_IO")) {
    const std::string m(io);
    io_mode_ = m == "graph" ? 0 : m == "stream" ? 1 : 2;
  }
  if (const char* b = std::getenv("BAND_HIP_IO_STREAM_BYTES")) io_stream_bytes_ = std::strtoull(b, nullptr, 10);
  if (const char* sy = std::getenv("BAND_HIP_SYNC")) {
    const std::string m(sy);
    sync_mode_ = m == "block"    ? kSyncBlock
                 : m == "poll"     ? kSyncPoll
                 : m == "poller"   ? kSyncPoller
                 : m == "spin"     ? kSyncSpin
                                   : kSyncAdaptive;
  }
  if (const char* f = std::getenv("BAND_HIP_SYNC_SLEEP")) sleep_frac_ = std::min(0.95, std::max(0.0, std::atof(f)));
  if (const char* f = std::getenv("BAND_HIP_SYNC_MIN_US")) sleep_min_us_ = std::max(0.0, std::atof(f));
  block_sync_ = sync_mode_ == kSyncBlock;
  if (const char* d = std::getenv("BAND_HIP_DIRECT_IO")) direct_io_ = d[0] != '0';
  if (const char* c = std::getenv("BAND_HIP_COALESCE")) coalesce_max_ = std::atoi(c);
  if (const char* c = std::getenv("BAND_HIP_COALESCE_LANES")) coalesce_lanes_ = std::max(1, std::atoi(c));
}

HipModelExecutor::~HipModelExecutor() {
  if (coalescer_) coalescer_->Leave(this);
  coalescer_.reset();  // the last member takes the lanes with it
  job_batches_.clear();
  if (ordinal_ >= 0) {
    bh_set_device(ordinal_);
    if (stream_) bh_stream_sync(stream_);
    for (auto& kv : subgraphs_) DropGraph(kv.second.get());
    if (done_event_) bh_event_destroy(done_event_);
  }
  subgraphs_.clear();
  if (owned_stream_) bh_stream_destroy(owned_stream_);
}

std::unique_ptr<HipModelExecutor> HipModelExecutor::MakeLane() {
  if (device_flag_ != DeviceFlag::kGPU || ordinal_ < 0) return nullptr;
  auto lane = std::make_unique<HipModelExecutor>(model_id_, worker_id_, device_flag_, thread_affinity_mask_,
                                                 num_threads_);
  if (bh_set_device(ordinal_) != 0 || bh_stream_create(&lane->owned_stream_) != 0) return nullptr;
  lane->ordinal_ = ordinal_;
  lane->stream_ = lane->owned_stream_;
  lane->coalesce_ok_ = false;
  lane->use_graph_ = use_graph_;
  lane->io_mode_ = io_mode_;
  lane->io_stream_bytes_ = io_stream_bytes_;
  lane->sync_mode_ = sync_mode_;
  lane->block_sync_ = block_sync_;
  // kernels-only variant graphs: the coalescer moves each pass's I/O on the
  // lane's stream (from the members' views, or from the variants' mirrors)
  lane->direct_io_ = true;
  lane->autotune_ = autotune_;
  return lane;
}


bool HipModelExecutor::GpuSupports(const TflModel& m, const TflOperator& op, std::string* why) {
  auto no = [&](const char* w) {
    if (why) *why = w;
    return false;
  };
  auto T = [&](int i) -> const TflTensor& { return m.tensors[i]; };
  if (op.inputs.empty() || op.outputs.empty() || op.inputs[0] < 0) return no("no operands");
  const TflTensor& in = T(op.inputs[0]);
  const TflTensor& out = T(op.outputs[0]);
  if (IsFloatOp(m, op)) return FloatSupports(m, op, why);
  switch (op.builtin) {
    case kTflConv2D:
    case kTflDepthwiseConv2D:
    case kTflFullyConnected: {
      if (op.inputs.size() < 2 || op.inputs[1] < 0) return no("missing filter");
      const TflTensor& w = T(op.inputs[1]);
      if (!IsQ8(in.type) || w.type != in.type || out.type != in.type) return no("only int8/uint8 quantized");
      if (!w.is_const() || !HasQ(in) || !HasQ(w) || !HasQ(out)) return no("needs constant quantized filter");
      if (op.inputs.size() > 2 && op.inputs[2] >= 0) {
        const TflTensor& b = T(op.inputs[2]);
        if (!b.is_const() || b.type != DataType::kInt32) return no("bias must be constant int32");
      }
      if (op.builtin == kTflFullyConnected) {
        if (w.shape.size() != 2 || w.shape[1] <= 0) return no("FC weights must be 2-D");
        if (in.num_elements() % static_cast<size_t>(w.shape[1]) != 0) return no("FC input/depth mismatch");
        return true;
      }
      if (in.shape.size() != 4 || w.shape.size() != 4 || out.shape.size() != 4) return no("conv needs 4-D");
      if (op.builtin == kTflConv2D && w.shape[3] != in.shape[3]) return no("grouped conv unsupported");
      if (op.builtin == kTflDepthwiseConv2D && (in.shape[3] == 0 || w.shape[3] % in.shape[3] != 0))
        return no("bad depth multiplier");
      return true;
    }
    case kTflAdd:
    case kTflSub:
    case kTflMul: {
      if (op.inputs.size() != 2 || op.inputs[1] < 0) return no("binary op needs 2 inputs");
      const TflTensor& b = T(op.inputs[1]);
      if (!IsQ8(in.type) || b.type != in.type || out.type != in.type) return no("only int8/uint8 quantized");
      if (!HasQ(in) || !HasQ(b) || !HasQ(out)) return no("missing quantization");
      if (in.shape.size() > 4 || b.shape.size() > 4 || out.shape.size() > 4) return no("rank > 4");
      int sa[4], sb[4], so[4];
      Shape4(in.shape, sa);
      Shape4(b.shape, sb);
      Shape4(out.shape, so);
      for (int d = 0; d < 4; ++d)
        if ((sa[d] != so[d] && sa[d] != 1) || (sb[d] != so[d] && sb[d] != 1)) return no("bad broadcast");
      return true;
    }
    case kTflAveragePool2D:
    case kTflMaxPool2D:
      if (!IsQ8(in.type) || out.type != in.type || in.shape.size() != 4) return no("only int8/uint8 4-D");
      if (!HasQ(out)) return no("missing quantization");
      return true;
    case kTflReshape:
    case kTflSqueeze:
      if (out.type != in.type || out.num_elements() != in.num_elements()) return no("size mismatch");
      return true;
    case kTflQuantize:
      if (!IsQ8(out.type) || !HasQ(out)) return no("QUANTIZE output must be 8-bit quantized");
      if (in.type == DataType::kFloat32) return true;
      if (!IsQ8(in.type) || !HasQ(in)) return no("QUANTIZE input must be float32 or 8-bit");
      return true;
    case kTflDequantize:
      if (!IsQ8(in.type) || !HasQ(in) || out.type != DataType::kFloat32) return no("only 8-bit -> float32");
      return true;
    case kTflRelu:
    case kTflRelu6:
    case kTflReluN1To1:
    case kTflLogistic:
    case kTflHardSwish:
      if (!IsQ8(in.type) || out.type != in.type || !HasQ(in) || !HasQ(out)) return no("only 8-bit quantized");
      if (op.builtin == kTflHardSwish) {
        uint8_t t[256];
        if (!HardSwishTable(in.type == DataType::kInt8, Scale(in), Zp(in), Scale(out), Zp(out), t))
          return no("output multiplier exponent > 0 (TFLite HardSwishPrepare refuses it)");
      }
      return true;
    case kTflMean: {
      long o, r, i;
      if (!MeanArgs(m, op, &o, &r, &i)) return no("MEAN over one contiguous run of axes, 4-D keep_dims");
      return true;
    }
    case kTflSoftmax:
      if (!IsQ8(in.type) || out.type != in.type || !HasQ(in) || !HasQ(out) || in.shape.empty())
        return no("only 8-bit quantized in and out");
      return true;
    case kTflConcatenation: {
      if (op.inputs.size() > BH_CONCAT_MAX_INPUTS) return no("too many inputs");
      if (op.options.valid() && op.options.Int8(1, 0) != 0) return no("fused activation on CONCATENATION");
      for (int t : op.inputs) {
        if (t < 0) return no("missing input");
        const TflTensor& x = T(t);
        if (x.type != out.type || x.shape.size() != out.shape.size()) return no("type / rank mismatch");
        if (out.type == DataType::kInt8 && (Scale(x) != Scale(out) || Zp(x) != Zp(out)))
          return no("int8 inputs must share the output's quantization");
        if (out.type == DataType::kUInt8 && !HasQ(x)) return no("missing quantization");
      }
      const size_t eb = GetDataTypeBytes(out.type);
      if (eb == 0) return no("unsized type");
      return true;
    }
    case kTflPad:
    case kTflPadV2: {
      const size_t eb = GetDataTypeBytes(in.type);
      if ((eb != 1 && eb != 4) || out.type != in.type || in.shape.size() > 4) return no("1/4-byte types, rank <= 4");
      if (op.inputs.size() < 2 || op.inputs[1] < 0 || !T(op.inputs[1]).is_const()) return no("paddings must be constant");
      const TflTensor& pt = T(op.inputs[1]);
      if (pt.type != DataType::kInt32 && pt.type != DataType::kInt64) return no("paddings must be int32/int64");
      if (op.builtin == kTflPadV2 && op.inputs.size() > 2 && op.inputs[2] >= 0 && !T(op.inputs[2]).is_const())
        return no("constant value must be constant");
      return true;
    }
    case kTflResizeNearestNeighbor: {
      const size_t eb = GetDataTypeBytes(in.type);
      if (in.shape.size() != 4 || out.shape.size() != 4 || out.type != in.type || eb == 0) return no("4-D only");
      return true;
    }
    case kTflMirrorPad: {
      const size_t eb = GetDataTypeBytes(in.type);
      std::vector<int64_t> pads;
      int mode = 0;
      if ((eb != 1 && eb != 4) || out.type != in.type) return no("1/4-byte types");
      if (!MirrorPadArgs(m, op, &pads, &mode)) return no("constant paddings within the input, rank <= 4");
      return true;
    }
    case kTflTransposeConv: {
      // inputs: output_shape (const int32 [4]), weights OHWI, input, [bias]
      if (op.inputs.size() < 3 || op.inputs[1] < 0 || op.inputs[2] < 0) return no("missing operands");
      const TflTensor& os = T(op.inputs[0]);
      const TflTensor& w = T(op.inputs[1]);
      const TflTensor& x = T(op.inputs[2]);
      if (!os.is_const() || !w.is_const()) return no("output shape and filter must be constant");
      if (x.type != DataType::kInt8 || w.type != DataType::kInt8 || out.type != DataType::kInt8)
        return no("int8 only (reference_integer_ops::TransposeConv)");
      if (!HasQ(x) || !HasQ(w) || !HasQ(out)) return no("missing quantization");
      if (x.shape.size() != 4 || w.shape.size() != 4 || out.shape.size() != 4 || w.shape[3] != x.shape[3])
        return no("4-D, filter [oc][kh][kw][ic]");
      if (op.inputs.size() > 3 && op.inputs[3] >= 0) {
        const TflTensor& b = T(op.inputs[3]);
        if (!b.is_const() || b.type != DataType::kInt32) return no("bias must be constant int32");
      }
      return true;
    }
    case kTflResizeBilinear:
      if ((in.type != DataType::kInt8 && in.type != DataType::kUInt8) || out.type != in.type || in.shape.size() != 4 ||
          out.shape.size() != 4)
        return no("int8 / uint8 4-D only (ResizeBilinearInteger / the uint8 float path)");
      return true;
    default:
      return no("op not in the HIP kernel set");
  }
}


bool HipModelExecutor::CpuSupports(const TflModel& m, const TflOperator& op, std::string* why) {
  if (GpuSupports(m, op, nullptr)) return true;
  if (DetectionSupported(m, op, nullptr)) return true;
  long o, r, i;
  if (MeanArgs(m, op, &o, &r, &i)) return true;
  return GpuSupports(m, op, why);
}

absl::Status HipModelExecutor::EnsureMeta(const HipModel& model) {
  if (!meta_.empty()) return absl::OkStatus();
  const TflModel& d = model.desc();
  meta_.reserve(d.tensors.size());
  for (const TflTensor& t : d.tensors) {
    auto m = std::make_unique<TensorMeta>();
    m->type = t.type;
    m->dims = t.shape;
    m->name = t.name;
    m->bytes = GetDataTypeBytes(t.type) * t.num_elements();
    m->SetQuant(t.scale, t.zero_point, t.quantized_dimension);
    meta_.push_back(std::move(m));
  }
  consumers_.assign(d.tensors.size(), {});
  producer_.assign(d.tensors.size(), -1);
  for (int i = 0; i < static_cast<int>(d.ops.size()); ++i) {
    for (int t : d.ops[i].inputs)
      if (t >= 0) consumers_[t].push_back(i);
    for (int t : d.ops[i].outputs)
      if (t >= 0) producer_[t] = i;
  }
  const char* f = std::getenv("BAND_HIP_FUSION");
  if (f && f[0] == '0') allow_fusion_ = false;
  if (f && std::strcmp(f, "noirb") == 0) allow_irb_ = false;   // diagnostics: one fusion kind at a time
  if (f && std::strcmp(f, "noadd") == 0) allow_add_ = false;
  if (f && std::strcmp(f, "nochain") == 0) allow_chain_ = false;
  if (f && std::strcmp(f, "nogroup") == 0) allow_group_ = false;
  if (f && std::strcmp(f, "forcechain") == 0) force_chain_ = true;  // parity tests: every feasible chain
  if (f && std::strcmp(f, "forcetile") == 0) force_chain_ = force_tile_chain_ = true;  // ... in the tile form
  if (f && std::strcmp(f, "notile") == 0) no_tile_chain_ = true;  // A-B: the raster chain forms only
  if (f && std::strcmp(f, "nodeep") == 0) no_deep_chain_ = true;  // A-B: without the deep-issue forms
  if (f && std::strcmp(f, "nosplit") == 0) no_split_chain_ = true;  // A-B: without the phase-C split forms
  if (f && std::strcmp(f, "forcedeep") == 0) force_deep_chain_ = true;  // parity tests: deep form wherever it fits
  if (f && std::strcmp(f, "forcestage") == 0) force_chain_ = force_stage_chain_ = true;  // parity: ... stage form
  if (f && std::strcmp(f, "nostage") == 0) no_stage_chain_ = true;  // A-B: without the stage forms
  const char* at = std::getenv("BAND_HIP_AUTOTUNE");
  if (at && at[0] == '0') autotune_ = false;
  return absl::OkStatus();
}

absl::StatusOr<ModelSpec> HipModelExecutor::InvestigateModelSpec(interface::IModel* model) {
  auto* hm = dynamic_cast<HipModel*>(model);
  if (!hm || !hm->IsInitialized()) return absl::InternalError("Failed to investigate model: not a loaded HIP model");
  const TflModel& d = hm->desc();
  const int num_ops = static_cast<int>(d.ops.size());
  std::vector<DataType> tensor_types;
  std::vector<std::set<int>> op_in, op_out;
  for (const TflOperator& op : d.ops) {
    std::set<int> all, ins, outs;
    for (int t : op.inputs) {
      if (t < 0) continue;  // kTfLiteOptionalTensor
      all.insert(t);
      if (!d.tensors[t].is_const()) ins.insert(t);  // constants are kTfLiteMmapRo
    }
    for (int t : op.outputs) {
      if (t < 0) continue;
      all.insert(t);
      if (!d.tensors[t].is_const()) outs.insert(t);
    }
    for (int t : all) tensor_types.push_back(d.tensors[t].type);
    op_in.push_back(ins);
    op_out.push_back(outs);
  }
  std::map<DeviceFlag, std::set<int>> unsupported;
  std::set<DeviceFlag> unavailable;
  const bool gpu = DeviceRegistry::Get().GpuAvailable();
  for (size_t f = 0; f < EnumLength<DeviceFlag>(); ++f) {
    const DeviceFlag flag = static_cast<DeviceFlag>(f);
    unsupported[flag] = {};
    if (flag == DeviceFlag::kCPU) continue;
    if (flag != DeviceFlag::kGPU || !gpu) {
      unavailable.insert(flag);
      continue;
    }
    for (int i = 0; i < num_ops; ++i)
      if (!GpuSupports(d, d.ops[i], nullptr)) unsupported[flag].insert(i);
    // Placement at a CPU-only boundary: a DEQUANTIZE whose every consumer
    // only the CPU runs (TFLite_Detection_PostProcess's inputs) is declared
    // unsupported here too, so the model analyzer puts it on the CPU side and
    // the GPU -> CPU hand-off carries the 8-bit tensor instead of its float
    // expansion (EfficientDet-Lite2's 37,629 x 90 class scores: 3.4 MB
    // instead of 13.5 MB per job, copied four times on the way).  The
    // outputs are the same (DEQUANTIZE is one exact table either side).
    // BAND_HIP_CPU_BOUNDARY_DEQUANT=0 keeps every DEQUANTIZE on the GPU.
    const char* bd = std::getenv("BAND_HIP_CPU_BOUNDARY_DEQUANT");
    if (!(bd && bd[0] == '0')) {
      std::vector<std::vector<int>> users(d.tensors.size());
      for (int i = 0; i < num_ops; ++i)
        for (int t : d.ops[i].inputs)
          if (t >= 0) users[t].push_back(i);
      for (int i = 0; i < num_ops; ++i) {
        const TflOperator& op = d.ops[i];
        if (op.builtin != kTflDequantize || op.outputs.empty() || op.outputs[0] < 0) continue;
        const std::vector<int>& u = users[op.outputs[0]];
        if (u.empty()) continue;
        bool cpu_only = true;
        for (int c : u) cpu_only &= unsupported[flag].count(c) > 0;
        if (cpu_only && CpuSupports(d, op, nullptr)) unsupported[flag].insert(i);
      }
    }
  }
  for (int i = 0; i < num_ops; ++i)
    if (!CpuSupports(d, d.ops[i], nullptr)) unsupported[DeviceFlag::kCPU].insert(i);
  ModelSpec spec(num_ops, static_cast<int>(d.tensors.size()), tensor_types,
                 std::set<int>(d.inputs.begin(), d.inputs.end()),
                 std::set<int>(d.outputs.begin(), d.outputs.end()), op_in, op_out, unsupported, unavailable);
  spec.path = hm->GetPath();
  return spec;
}

absl::Status HipModelExecutor::PrepareSubgraph(interface::IModel* model, std::set<int> ops, std::set<int> unit_indices) {
  auto* hm = dynamic_cast<HipModel*>(model);
  if (!hm || model->GetId() != model_id_)
    return absl::InternalError("Failed to prepare subgraph: model id " + std::to_string(model ? model->GetId() : -1) +
                               " != executor's model id " + std::to_string(model_id_));
  if (!hm->IsInitialized()) return absl::InternalError("Failed to prepare subgraph: model not loaded");
  if (model_ && model_ != hm) return absl::InternalError("executor already bound to another model object");
  model_ = hm;
  RETURN_STATUS_IF(EnsureMeta(*hm));
  const TflModel& d = hm->desc();
  const int num_ops = static_cast<int>(d.ops.size());
  const bool whole = ops.empty();
  if (whole)
    for (int i = 0; i < num_ops; ++i) ops.insert(i);
  for (int i : ops)
    if (i < 0 || i >= num_ops) return absl::InternalError("op index out of range");

  if (device_flag_ == DeviceFlag::kGPU && (ordinal_ < 0 || !stream_))
    return absl::InternalError("Failed to create HIP executor: no gfx950 device");
  auto sg = std::make_unique<PreparedSubgraph>();
  sg->ops.assign(ops.begin(), ops.end());
  std::set<int> consumed, produced, touched;
  for (int i : sg->ops) {
    for (int t : d.ops[i].inputs)
      if (t >= 0 && !d.tensors[t].is_const()) { consumed.insert(t); touched.insert(t); }
    for (int t : d.ops[i].outputs)
      if (t >= 0 && !d.tensors[t].is_const()) { produced.insert(t); touched.insert(t); }
  }
  if (whole) {
    sg->model_order_io = true;
    sg->inputs = d.inputs;
    sg->outputs = d.outputs;
  } else {
    for (int t : consumed)
      if (!produced.count(t)) sg->inputs.push_back(t);
    std::set<int> needed_outside(d.outputs.begin(), d.outputs.end());
    for (int i = 0; i < num_ops; ++i)
      if (!ops.count(i))
        for (int t : d.ops[i].inputs)
          if (t >= 0) needed_outside.insert(t);
    for (int t : produced)
      if (needed_outside.count(t)) sg->outputs.push_back(t);
  }

  // host-pinned boundary mirrors (Band memcpy's job I/O through these)
  const bool pinned = device_flag_ == DeviceFlag::kGPU;
  const bool cpu = device_flag_ == DeviceFlag::kCPU;
  // a job-batch variant views the largest variant's mirrors (slot s of a
  // tensor sits at s * batch-1 bytes in every variant)
  auto mirror = [&](int t) -> std::unique_ptr<PinnedBuffer> {
    if (shared_host_from_) {
      auto it = shared_host_from_->host.find(t);
      if (it != shared_host_from_->host.end() && it->second->bytes() >= meta_[t]->bytes)
        return std::make_unique<PinnedBuffer>(it->second->data(), meta_[t]->bytes);
    }
    return std::make_unique<PinnedBuffer>(meta_[t]->bytes, pinned);
  };
  for (int t : sg->inputs) sg->host[t] = mirror(t);
  for (int t : sg->outputs)
    if (!sg->host.count(t)) sg->host[t] = mirror(t);
  for (auto& kv : sg->host)
    if (!kv.second->ok()) return absl::InternalError("pinned host allocation failed");

  if (device_flag_ == DeviceFlag::kGPU || cpu) {
    if (!cpu) {
      if (ordinal_ < 0 || !stream_) return absl::InternalError("Failed to create HIP executor: no gfx950 device");
      if (bh_set_device(ordinal_) != 0) return HipErr(1, "hipSetDevice");
    }
    // RESHAPE / SQUEEZE outputs alias their input's slot (same bytes, and
    // every tensor is immutable once produced), so they cost no launch.
    std::map<int, int> alias;
    for (int i : sg->ops) {
      const TflOperator& op = d.ops[i];
      if ((op.builtin == kTflReshape || op.builtin == kTflSqueeze) && !op.inputs.empty() && op.inputs[0] >= 0 &&
          !d.tensors[op.inputs[0]].is_const() && meta_[op.outputs[0]]->bytes == meta_[op.inputs[0]]->bytes) {
        int src = op.inputs[0];
        while (alias.count(src)) src = alias[src];
        alias[op.outputs[0]] = src;
      }
    }
    size_t total = 0;
    for (int t : touched) {
      if (alias.count(t)) continue;
      sg->offset[t] = total;
      total += (meta_[t]->bytes + kAlign - 1) / kAlign * kAlign;
    }
    for (const auto& kv : alias) sg->offset[kv.first] = sg->offset.at(kv.second);
    if (shared_arena_ && shared_arena_->bytes() >= total && shared_arena_->ordinal() == ordinal_)
      sg->arena = shared_arena_;  // job-batch variant: the largest variant's arena
    else
      sg->arena = std::make_shared<DeviceBlob>(ordinal_, total);
    if (!sg->arena->ok()) return absl::InternalError("arena allocation failed");
    if (cpu) {
      // a host executor's boundary tensors ARE its arena slots (every tensor
      // has its own slot): Band's copies land where the kernels read
      char* arena = static_cast<char*>(sg->arena->ptr());
      for (int t : sg->inputs) sg->host[t] = std::make_unique<PinnedBuffer>(arena + sg->offset.at(t), meta_[t]->bytes);
      for (int t : sg->outputs)
        sg->host[t] = std::make_unique<PinnedBuffer>(arena + sg->offset.at(t), meta_[t]->bytes);
    }
    RETURN_STATUS_IF(BuildLaunches(*hm, sg.get()));
  } else {
    return absl::InternalError(std::string("Unsupported device type ") + ToString(device_flag_));
  }
  SubgraphKey key(model->GetId(), worker_id_, unit_indices);
  auto old = subgraphs_.find(key);
  if (old != subgraphs_.end()) DropGraph(old->second.get());
  subgraphs_[key] = std::move(sg);
  // whole-model GPU subgraphs coalesce concurrent jobs with the other
  // executors of this model on this GPU (coalescer.h)
  // (Band's engine names every op of a whole model explicitly)
  if (static_cast<int>(ops.size()) == num_ops && device_flag_ == DeviceFlag::kGPU && coalesce_ok_ &&
      coalesce_max_ > 1 && !t_variant_ctor) {
    if (coalescer_) coalescer_->Leave(this);
    coalescer_ = JobCoalescer::Join(this, model, key, ordinal_, coalesce_max_, coalesce_lanes_);
    coalesced_key_ = key;
  }
  return absl::OkStatus();
}

PreparedSubgraph* HipModelExecutor::Find(const SubgraphKey& key) const {
  auto it = subgraphs_.find(key);
  return it == subgraphs_.end() ? nullptr : it->second.get();
}

const std::vector<int>& HipModelExecutor::GetInputs(const SubgraphKey& key) const {
  auto* sg = Find(key);
  return sg ? sg->inputs : kEmpty;
}
const std::vector<int>& HipModelExecutor::GetOutputs(const SubgraphKey& key) const {
  auto* sg = Find(key);
  return sg ? sg->outputs : kEmpty;
}
const char* HipModelExecutor::GetInputName(const SubgraphKey& key, int index) const {
  auto* sg = Find(key);
  if (!sg || index < 0 || index >= static_cast<int>(sg->inputs.size())) return nullptr;
  return meta_[sg->inputs[index]]->name.c_str();
}
const char* HipModelExecutor::GetOutputName(const SubgraphKey& key, int index) const {
  auto* sg = Find(key);
  if (!sg || index < 0 || index >= static_cast<int>(sg->outputs.size())) return nullptr;
  return meta_[sg->outputs[index]]->name.c_str();
}
size_t HipModelExecutor::GetNumTensors(const SubgraphKey& key) const { return Find(key) ? meta_.size() : 0; }
size_t HipModelExecutor::GetNumNodes(const SubgraphKey& key) const {
  auto* sg = Find(key);
  return sg ? sg->ops.size() : 0;
}
bool HipModelExecutor::HasSubgraph(const SubgraphKey& key) const { return Find(key) != nullptr; }

SubgraphKey HipModelExecutor::GetLargestSubgraphKey() const {
  SubgraphKey best;
  size_t most = 0;
  for (const auto& kv : subgraphs_)
    if (kv.second->ops.size() > most) {
      most = kv.second->ops.size();
      best = kv.first;
    }
  return best;
}

void HipModelExecutor::ForEachSubgraph(std::function<void(const SubgraphKey&)> visitor) {
  for (const auto& kv : subgraphs_) visitor(kv.first);
}

std::shared_ptr<interface::ITensorView> HipModelExecutor::GetTensorView(const SubgraphKey& key, int index) {
  auto* sg = Find(key);
  if (!sg || index < 0 || index >= static_cast<int>(meta_.size())) return nullptr;
  TensorMeta* m = meta_[index].get();
  auto h = sg->host.find(index);
  if (h != sg->host.end()) return std::make_shared<HipTensorView>(m, h->second->data());
  const TflTensor& t = model_->desc().tensors[index];
  if (t.is_const())
    return std::make_shared<HipTensorView>(m, const_cast<char*>(reinterpret_cast<const char*>(t.data)));
  if ((device_flag_ == DeviceFlag::kGPU || device_flag_ == DeviceFlag::kCPU) && sg->offset.count(index)) {
    // an intermediate of this subgraph: mirror it and copy it back on every run
    auto buf = std::make_unique<PinnedBuffer>(m->bytes);
    if (!buf->ok()) return nullptr;
    char* data = buf->data();
    sg->host[index] = std::move(buf);
    sg->extra_d2h.insert(index);
    if (ordinal_ >= 0) bh_set_device(ordinal_);
    DropGraph(sg);
    if (sg->fused_tensors.count(index)) {
      // the tensor was folded away by an epilogue fusion: re-lower with it materialised
      sg->no_fuse.insert(index);
      if (!BuildLaunches(*model_, sg).ok()) return nullptr;
    }
    return std::make_shared<HipTensorView>(m, data);
  }
  return std::make_shared<HipTensorView>(m, nullptr);
}

absl::Status HipModelExecutor::EnqueueLaunch(const Launch& l) {
  int rc = 0;
  switch (l.kind) {
    case Launch::kConv: rc = bh_conv2d_i8(&l.conv, stream_); break;
    case Launch::kDwConv: rc = bh_dwconv2d_i8(&l.dw, stream_); break;
    case Launch::kFc: rc = bh_fc_i8(&l.fc, stream_); break;
    case Launch::kEltwise: rc = bh_eltwise_i8(&l.elt, stream_); break;
    case Launch::kPool: rc = bh_pool_i8(&l.pool, stream_); break;
    case Launch::kIrb: rc = bh_irb_i8(&l.irb, stream_); break;
    case Launch::kChain: rc = bh_chain_i8(&l.chain, stream_); break;
    case Launch::kConvGroup: rc = bh_conv_group_i8(&l.cgroup, stream_); break;
    case Launch::kCopy: {
      // a kernel copy, not a blit: graphs replayed under rocprofv3's kernel
      // trace crash on blit (memcpy) nodes; BAND_HIP_BLIT_COPY=1 restores them
      static const bool blit = [] {
        const char* v = std::getenv("BAND_HIP_BLIT_COPY");
        return v && v[0] == '1';
      }();
      if (l.src != l.dst)
        rc = blit ? bh_memcpy_d2d_async(l.dst, l.src, l.bytes, stream_) : bh_copy_d2d(l.dst, l.src, l.bytes, stream_);
      break;
    }
    case Launch::kLutU8: rc = bh_lut_u8(l.src, l.dst, l.count, l.table, stream_); break;
    case Launch::kLutF32:
      rc = bh_lut_f32(l.src, l.dst, l.count, static_cast<const float*>(l.table), stream_);
      break;
    case Launch::kQuantF32:
      rc = bh_quantize_f32(static_cast<const float*>(l.src), l.dst, l.count, l.q_scale, l.q_zp, l.q_signed, stream_);
      break;
    case Launch::kConcat: rc = bh_concat(&l.concat, stream_); break;
    case Launch::kPad: rc = bh_pad(&l.pad, stream_); break;
    case Launch::kResizeNearest: rc = bh_resize_nearest(&l.rnear, stream_); break;
    case Launch::kResizeBilinear: rc = bh_resize_bilinear_i8(&l.rbil, stream_); break;
    case Launch::kResizeBilinearU8: rc = bh_resize_bilinear_u8(&l.rbil8, stream_); break;
    case Launch::kSoftmax: rc = bh_softmax_i8(&l.softmax, stream_); break;
    case Launch::kZeroInsert: rc = bh_zero_insert(&l.zi, stream_); break;
    case Launch::kConvF32: rc = bh_conv2d_f32(&l.convf, stream_); break;
    case Launch::kFcF32: rc = bh_fc_f32(&l.fcf, stream_); break;
    case Launch::kEltwiseF32: rc = bh_eltwise_f32(&l.eltf, stream_); break;
    case Launch::kPoolF32: rc = bh_pool_f32(&l.poolf, stream_); break;
    case Launch::kUnaryF32:
      rc = bh_unary_f32(l.unary_kind, static_cast<const float*>(l.src), static_cast<float*>(l.dst), l.count, l.lo,
                        l.hi, stream_);
      break;
    case Launch::kSoftmaxF32:
      rc = bh_softmax_f32(static_cast<const float*>(l.src), static_cast<float*>(l.dst), l.count, l.depth, l.beta,
                          stream_);
      break;
    case Launch::kDetectionPost: return absl::InternalError(std::string(l.kernel) + " is a CPU-worker op");
    case Launch::kMean: {
      bh_mean_params q{};
      q.outer = l.mean.outer;
      q.reduce = l.mean.reduce;
      q.inner = l.mean.inner;
      q.type = l.mean.type;
      q.multiplier = l.mean.multiplier;
      q.shift = l.mean.shift;
      q.bias = l.mean.bias;
      q.input = l.mean.input;
      q.output = l.mean.output;
      rc = bh_mean(&q, stream_);
      break;
    }
  }
  return rc ? HipErr(rc, l.kernel) : absl::OkStatus();
}

// diagnostics only (tools/concurrency_probe.py --no-io): kernels without
// the host copies, to separate device compute scaling from the transfers
static bool ProbeNoIo() {
  static const bool v = [] {
    const char* e = std::getenv("BAND_HIP_PROBE_NO_IO");
    return e && e[0] == '1';
  }();
  return v;
}

absl::Status HipModelExecutor::Enqueue(PreparedSubgraph* sg) {
  RETURN_STATUS_IF(EnqueueInputs(sg));
  RETURN_STATUS_IF(EnqueueLaunches(sg));
  return EnqueueOutputs(sg);
}

absl::Status HipModelExecutor::EnqueueLaunches(PreparedSubgraph* sg) {
  for (const Launch& l : sg->launches) RETURN_STATUS_IF(EnqueueLaunch(l));
  return absl::OkStatus();
}

void HipModelExecutor::DropGraph(PreparedSubgraph* sg) {
  if (sg->graph) bh_graph_destroy(sg->graph);
  if (sg->graph_tmpl) bh_graph_free(sg->graph_tmpl);
  sg->graph = nullptr;
  sg->graph_tmpl = nullptr;
  sg->io_nodes.clear();
  sg->io_retargeted = false;
}

absl::Status HipModelExecutor::RestoreIoNodes(PreparedSubgraph* sg) {
  if (!sg->io_retargeted) return absl::OkStatus();
  char* arena = static_cast<char*>(sg->arena->ptr());
  for (const auto& n : sg->io_nodes) {
    char* dev = arena + sg->offset.at(n.tensor);
    char* host = sg->host.at(n.tensor)->data();
    const int rc = bh_graph_exec_set_memcpy(sg->graph, n.node, n.h2d ? (void*)dev : (void*)host,
                                            n.h2d ? (const void*)host : (const void*)dev, meta_[n.tensor]->bytes,
                                            n.h2d ? 1 : 0);
    if (rc) return HipErr(rc, "graph copy node");
  }
  sg->io_retargeted = false;
  return absl::OkStatus();
}

absl::Status HipModelExecutor::CaptureGraph(PreparedSubgraph* sg) {
  size_t io_bytes = 0;
  for (int t : sg->inputs) io_bytes += meta_[t]->bytes;
  for (int t : sg->outputs) io_bytes += meta_[t]->bytes;
  for (int t : sg->extra_d2h) io_bytes += meta_[t]->bytes;
  sg->io_in_graph = io_mode_ == 0 || (io_mode_ == 2 && io_bytes < io_stream_bytes_);
  int rc = bh_capture_begin(stream_);
  if (rc) return HipErr(rc, "capture begin");
  absl::Status s = sg->io_in_graph ? Enqueue(sg) : EnqueueLaunches(sg);
  bh_graph_exec_t g = nullptr;
  void* tmpl = nullptr;
  rc = bh_capture_end_keep(stream_, &g, &tmpl);
  if (!s.ok()) {
    if (!rc) {
      bh_graph_destroy(g);
      bh_graph_free(tmpl);
    }
    return s;
  }
  if (rc) return HipErr(rc, "capture end");
  sg->graph = g;
  sg->graph_tmpl = tmpl;
  sg->io_nodes.clear();
  sg->io_retargeted = false;
  if (sg->io_in_graph) {
    // the copy nodes, told apart by their device-side address: input t's
    // H2D writes arena + offset(t), output t's D2H reads it
    constexpr int kMax = 64;
    void* nodes[kMax];
    void* dsts[kMax];
    const void* srcs[kMax];
    size_t bytes[kMax];
    int n = 0;
    char* arena = static_cast<char*>(sg->arena->ptr());
    if (bh_graph_memcpy_nodes(tmpl, nodes, dsts, srcs, bytes, kMax, &n) == 0 && n <= kMax) {
      for (int i = 0; i < n; ++i) {
        for (int t : sg->inputs)
          if (dsts[i] == arena + sg->offset.at(t) && bytes[i] == meta_[t]->bytes) sg->io_nodes.push_back({nodes[i], t, true});
        for (int t : sg->outputs)
          if (srcs[i] == arena + sg->offset.at(t) && bytes[i] == meta_[t]->bytes) sg->io_nodes.push_back({nodes[i], t, false});
      }
      if (sg->io_nodes.size() != sg->inputs.size() + sg->outputs.size()) sg->io_nodes.clear();
    }
  }
  return absl::OkStatus();
}

absl::Status HipModelExecutor::PrecaptureGraph(PreparedSubgraph* sg) {
  if (!use_graph_ || sg->graph) return absl::OkStatus();
  const int rc = bh_set_device(ordinal_);
  if (rc) return HipErr(rc, "hipSetDevice");
  RETURN_STATUS_IF(EnqueueLaunches(sg));
  if (bh_stream_sync(stream_) != 0) return HipErr(1, "stream sync");
  ++sg->runs;
  return CaptureGraph(sg);
}

absl::Status HipModelExecutor::EnqueuePass(PreparedSubgraph* sg) {
  if (!use_graph_ || !sg->graph) return Enqueue(sg);
  RETURN_STATUS_IF(RestoreIoNodes(sg));
  if (!sg->io_in_graph) RETURN_STATUS_IF(EnqueueInputs(sg));

  const int rc = bh_graph_launch(sg->graph, stream_);
  if (rc) return HipErr(rc, "graph launch");
  return sg->io_in_graph ? absl::OkStatus() : EnqueueOutputs(sg);
}

absl::Status HipModelExecutor::EnqueueInputs(PreparedSubgraph* sg) {
  if (ProbeNoIo()) return absl::OkStatus();
  char* arena = static_cast<char*>(sg->arena->ptr());
  for (int t : sg->inputs) {
    int rc = bh_memcpy_h2d_async(arena + sg->offset.at(t), sg->host.at(t)->data(), meta_[t]->bytes, stream_);
    if (rc) return HipErr(rc, "H2D input");
  }
  return absl::OkStatus();
}

absl::Status HipModelExecutor::EnqueueOutputs(PreparedSubgraph* sg) {
  if (ProbeNoIo()) return absl::OkStatus();
  char* arena = static_cast<char*>(sg->arena->ptr());
  for (int t : sg->outputs) {
    int rc = bh_memcpy_d2h_async(sg->host.at(t)->data(), arena + sg->offset.at(t), meta_[t]->bytes, stream_);
    if (rc) return HipErr(rc, "D2H output");
  }
  for (int t : sg->extra_d2h) {
    int rc = bh_memcpy_d2h_async(sg->host.at(t)->data(), arena + sg->offset.at(t), meta_[t]->bytes, stream_);
    if (rc) return HipErr(rc, "D2H intermediate");
  }
  return absl::OkStatus();
}

// kCPU worker: the same launch program over host memory (cpu_kernels.h)
absl::Status HipModelExecutor::ExecuteOnHost(PreparedSubgraph* sg) {
  char* arena = static_cast<char*>(sg->arena->ptr());
  auto sync = [&](int t, bool in) {  // no copy when the mirror is the arena slot
    char* slot = arena + sg->offset.at(t);
    char* mirror = sg->host.at(t)->data();
    if (slot != mirror) std::memcpy(in ? slot : mirror, in ? mirror : slot, meta_[t]->bytes);
  };
  for (int t : sg->inputs) sync(t, true);
  if (!cpu_pool_)
    cpu_pool_ = std::make_shared<CpuPool>(num_threads_ > 0 ? num_threads_ : 1, PinnableCpus(thread_affinity_mask_));
  CpuPool& pool = *cpu_pool_;
  for (const Launch& l : sg->launches) {
    switch (l.kind) {
      case Launch::kConv: CpuConv(l.conv, pool); break;
      case Launch::kDwConv: CpuDwConv(l.dw, pool); break;
      case Launch::kFc: CpuFc(l.fc, pool); break;
      case Launch::kEltwise: CpuEltwise(l.elt, pool); break;
      case Launch::kPool: CpuPool2D(l.pool, pool); break;
      case Launch::kCopy:
        if (l.src != l.dst) std::memmove(l.dst, l.src, l.bytes);
        break;
      case Launch::kLutU8: CpuLutU8(l.src, l.dst, l.count, static_cast<const uint8_t*>(l.table), pool); break;
      case Launch::kLutF32:
        CpuLutF32(l.src, static_cast<float*>(l.dst), l.count, static_cast<const float*>(l.table), pool);
        break;
      case Launch::kQuantF32:
        CpuQuantizeF32(static_cast<const float*>(l.src), l.dst, l.count, l.q_scale, l.q_zp, l.q_signed, pool);
        break;
      case Launch::kConcat: CpuConcat(l.concat); break;
      case Launch::kPad: CpuPad(l.pad); break;
      case Launch::kResizeNearest: CpuResizeNearest(l.rnear); break;
      case Launch::kResizeBilinear: CpuResizeBilinear(l.rbil); break;
      case Launch::kResizeBilinearU8: CpuResizeBilinearU8(l.rbil8); break;
      case Launch::kSoftmax: CpuSoftmax(l.softmax); break;
      case Launch::kZeroInsert: CpuZeroInsert(l.zi); break;
      case Launch::kConvF32: CpuConvF32(l.convf, pool); break;
      case Launch::kFcF32: CpuFcF32(l.fcf, pool); break;
      case Launch::kEltwiseF32: CpuEltwiseF32(l.eltf); break;
      case Launch::kPoolF32: CpuPoolF32(l.poolf); break;
      case Launch::kUnaryF32:
        CpuUnaryF32(l.unary_kind, static_cast<const float*>(l.src), static_cast<float*>(l.dst), l.count, l.lo, l.hi);
        break;
      case Launch::kSoftmaxF32:
        CpuSoftmaxF32(static_cast<const float*>(l.src), static_cast<float*>(l.dst), l.count, l.depth, l.beta);
        break;
      case Launch::kDetectionPost: CpuDetectionPostprocess(l.det, pool); break;
      case Launch::kMean: CpuMean(l.mean, pool); break;
      default: return absl::InternalError(std::string("no host implementation of ") + l.kernel);
    }
  }
  for (int t : sg->outputs) sync(t, false);
  for (int t : sg->extra_d2h) sync(t, false);
  ++sg->runs;
  return absl::OkStatus();
}

absl::Status HipModelExecutor::ExecuteSubgraph(const SubgraphKey& key) {
  PreparedSubgraph* sg = Find(key);
  if (!sg) return absl::InternalError("Cannot find subgraph");
  if (device_flag_ == DeviceFlag::kCPU) return ExecuteOnHost(sg);
  if (device_flag_ != DeviceFlag::kGPU) return absl::InternalError("Unsupported device type");
  // a view of an intermediate (extra_d2h) needs this executor's own pass
  if (coalescer_ && key == coalesced_key_ && sg->extra_d2h.empty()) return coalescer_->Run(this, sg);
  return RunPass(sg);
}

absl::Status HipModelExecutor::RunPass(PreparedSubgraph* sg) {
  int rc = bh_set_device(ordinal_);
  if (rc) return HipErr(rc, "hipSetDevice");
  if (use_graph_ && !sg->graph && sg->runs > 0) RETURN_STATUS_IF(CaptureGraph(sg));
  RETURN_STATUS_IF(EnqueuePass(sg));
  RETURN_STATUS_IF(WaitPass(sg));
  ++sg->runs;
  return absl::OkStatus();
}

absl::Status HipModelExecutor::WaitPass(PreparedSubgraph* sg) {
  int rc = 0;
  if (sync_mode_ == kSyncSpin || (sync_mode_ == kSyncAdaptive && !sg)) {
    rc = bh_stream_sync(stream_);
    return rc ? HipErr(rc, "stream sync") : absl::OkStatus();
  }
  if (sync_mode_ == kSyncAdaptive) {
    // sleep through sleep_frac_ of the pass's expected wait, then spin in
    // hipStreamSynchronize: the thread holds a core only for the tail of the
    // pass, and it is already running (no wake-up from an idle core, the
    // cost of the blocking forms) when the pass ends.  A wake-up that finds
    // the pass already done shortens the next sleep.
    thread_local bool slack = [] { return prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0) == 0; }();
    (void)slack;
    const auto t0 = std::chrono::steady_clock::now();
    // short passes (a batch-1 job: ~0.2 ms) spin: a sleep's wake-up jitter
    // is a large share of them (C2: 4.88k inf/s, p99 0.76 ms sleeping
    // against 5.09k, p99 0.37 ms spinning, profiles/r05r_c2*.json)
    const double sleep = sg->wait_us >= sleep_min_us_ ? sleep_frac_ * sg->wait_us : 0.0;
    bool overslept = false;
    if (sleep >= 20.0) {
      timespec ts{0, static_cast<long>(sleep * 1000.0)};
      nanosleep(&ts, nullptr);
      overslept = bh_stream_query(stream_) == 0;
    }
    rc = bh_stream_sync(stream_);
    if (rc) return HipErr(rc, "stream sync");
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (overslept) sg->wait_us *= 0.85;
    else sg->wait_us = sg->wait_us > 0 ? 0.9 * sg->wait_us + 0.1 * us : us;
    return absl::OkStatus();
  }
  if (!done_event_ && (sync_mode_ == kSyncBlock ? bh_event_create_blocking(&done_event_)
                                                : bh_event_create_untimed(&done_event_)) != 0)
    return HipErr(1, "event create");
  rc = bh_event_record(done_event_, stream_);
  if (rc) return HipErr(rc, "event record");
  if (sync_mode_ == kSyncPoller) {  // this GPU's poller thread waits for it (completion.h)
    rc = CompletionPoller::ForDevice(ordinal_).Wait(done_event_);
    return rc ? HipErr(rc, "event query") : absl::OkStatus();
  }
  if (sync_mode_ == kSyncBlock) {
    rc = bh_event_sync(done_event_);
    return rc ? HipErr(rc, "event sync") : absl::OkStatus();
  }
  // poll: sleep through ~3/4 of the expected time, then poll every kPollUs
  // (timer slack cut to 1 us for this thread, so the sleeps are that short)
  thread_local bool slack = [] { return prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0) == 0; }();
  (void)slack;
  constexpr int kPollUs = 8;
  const auto t0 = std::chrono::steady_clock::now();
  auto sleep_us = [](double us) {
    if (us < 1.0) return;
    timespec ts{0, static_cast<long>(us * 1000.0)};
    nanosleep(&ts, nullptr);
  };
  if (sg && sg->wait_us > 2 * kPollUs) sleep_us(0.75 * sg->wait_us - kPollUs);
  while ((rc = bh_event_query(done_event_)) == BH_ENOTREADY) sleep_us(kPollUs);
  if (rc) return HipErr(rc, "event query");
  if (sg) {
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    sg->wait_us = sg->wait_us > 0 ? 0.9 * sg->wait_us + 0.1 * us : us;
  }
  return absl::OkStatus();
}

absl::Status HipModelExecutor::TimeSubgraph(const SubgraphKey& key, int iters, double* us) {
  PreparedSubgraph* sg = Find(key);
  if (!sg) return absl::InternalError("Cannot find subgraph");
  if (device_flag_ != DeviceFlag::kGPU) return absl::InternalError("timing needs a GPU executor");
  if (iters <= 0 || !us) return absl::InternalError("bad arguments");
  // two ordinary runs first, so the graph (if enabled) is captured
  for (int i = 0; i < 2; ++i) RETURN_STATUS_IF(ExecuteSubgraph(key));
  bh_event_t e0 = nullptr, e1 = nullptr;
  if (bh_event_create(&e0) != 0 || bh_event_create(&e1) != 0) return HipErr(1, "event create");
  // At most kDepth passes queued ahead of the GPU: the host waits for pass
  // i - kDepth before issuing pass i, so the queue never drains (timing is
  // unchanged) but the number of outstanding dispatches stays bounded.
  // Unbounded, 100 queued batch-24 SSD passes (~7,700 kernel dispatches)
  // crash rocprofv3's kernel-trace interception.
  constexpr int kDepth = 4;
  bh_event_t ring[kDepth] = {nullptr};
  for (auto& e : ring)
    if (bh_event_create(&e) != 0) return HipErr(1, "event create");
  absl::Status status = absl::OkStatus();
  bh_event_record(e0, stream_);
  for (int i = 0; i < iters && status.ok(); ++i) {
    if (i >= kDepth && bh_event_sync(ring[i % kDepth]) != 0) status = HipErr(1, "event sync");
    if (!status.ok()) break;
    status = EnqueuePass(sg);
    bh_event_record(ring[i % kDepth], stream_);
  }
  bh_event_record(e1, stream_);
  float ms = 0.f;
  if (bh_stream_sync(stream_) != 0 && status.ok()) status = HipErr(1, "sync");
  if (status.ok() && bh_event_elapsed_ms(e0, e1, &ms) != 0) status = HipErr(1, "elapsed");
  bh_event_destroy(e0);
  bh_event_destroy(e1);
  for (auto e : ring) bh_event_destroy(e);
  if (status.ok()) *us = 1e3 * ms / iters;
  return status;
}

absl::Status HipModelExecutor::ProfileSubgraph(const SubgraphKey& key, int iters, std::vector<OpTiming>* out,
                                              double* floor_us) {
  PreparedSubgraph* sg = Find(key);
  if (!sg) return absl::InternalError("Cannot find subgraph");
  if (device_flag_ != DeviceFlag::kGPU) return absl::InternalError("profiling needs a GPU executor");
  if (bh_set_device(ordinal_) != 0) return HipErr(1, "hipSetDevice");
  const size_t n = sg->launches.size();
  std::vector<bh_event_t> st(n, nullptr), sp(n, nullptr);
  for (size_t i = 0; i < n; ++i)
    if (bh_event_create(&st[i]) != 0 || bh_event_create(&sp[i]) != 0) return HipErr(1, "event create");
  std::vector<double> acc(n, 0.0);
  double floor_acc = 0.0;
  absl::Status status = absl::OkStatus();
  // The launches run once each, in program order, queued back to back behind
  // a spin kernel (so the GPU runs them without host gaps, as in a replayed
  // graph), each kernel carrying its own dispatch begin / end timestamps
  // (bh_profile_events -> hipExtLaunchKernel): the kernel-only duration
  // rocprofv3's kernel trace reports, every kernel seeing the cache state of
  // a real pass (its input just written by its producer).  A launch that
  // issues no kernel (a copy) is timed by plain events around it.  The
  // second pass times empty single-wave kernels the same way: the fixed cost
  // of a dispatch inside every duration (floor_us).
  for (int it = 0; it < iters && status.ok(); ++it) {
    for (int pass = 0; pass < 2 && status.ok(); ++pass) {
      if (bh_spin_us(stream_, 300 + 40 * static_cast<int>(n)) != 0) status = HipErr(1, "spin");
      for (size_t i = 0; i < n && status.ok(); ++i) {
        bh_event_record(st[i], stream_);
        bh_profile_events(st[i], sp[i]);
        if (pass == 0) status = EnqueueLaunch(sg->launches[i]);
        else if (bh_empty_launch(stream_) != 0) status = HipErr(1, "empty launch");
        if (bh_profile_events(nullptr, nullptr) == 0) bh_event_record(sp[i], stream_);
      }
      if (bh_stream_sync(stream_) != 0) status = HipErr(1, "sync");
      for (size_t i = 0; i < n && status.ok(); ++i) {
        float ms = 0;
        bh_event_elapsed_ms(st[i], sp[i], &ms);
        if (pass == 0) acc[i] += ms;
        else floor_acc += ms * 1e3 / n;
      }
    }
  }
  bh_profile_events(nullptr, nullptr);
  for (auto e : st) bh_event_destroy(e);
  for (auto e : sp) bh_event_destroy(e);
  if (!status.ok()) return status;
  out->clear();
  for (size_t i = 0; i < n; ++i) {
    const Launch& l = sg->launches[i];
    out->push_back({l.op_index, l.kernel, acc[i] / std::max(iters, 1), l.alg_bytes, l.alg_ops});
  }
  if (floor_us) *floor_us = floor_acc / std::max(iters, 1);
  return absl::OkStatus();
}

}  // namespace hip
}  // namespace band
