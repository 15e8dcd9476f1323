// HipModelExecutor: lowering of TFLite ops to kernel launches (Launch records)
// - the per-op parameter derivation, constants packed and uploaded once per
// (model, GPU), the residual-ADD epilogue fold.  Split from model_executor.cc.
#include "backend/hip/executor_internal.h"

namespace band {
namespace hip {

using namespace ex;

absl::Status HipModelExecutor::DevicePtr(const HipModel& model, int t, PreparedSubgraph* sg, void** ptr) {
  const TflTensor& tt = model.desc().tensors[t];
  if (!tt.is_const()) {
    auto it = sg->offset.find(t);
    if (it == sg->offset.end()) return absl::InternalError("tensor without arena slot");
    *ptr = static_cast<char*>(sg->arena->ptr()) + it->second;
    return absl::OkStatus();
  }
  const std::string key = "m" + Hex(model.serial()) + "/t" + std::to_string(t);
  auto blob = DeviceRegistry::Get().FindConst(ordinal_, key);
  if (!blob) {
    blob = std::make_shared<DeviceBlob>(ordinal_, tt.data_size);
    if (!blob->ok() || !blob->Upload(0, tt.data, tt.data_size))
      return HipErr(1, "upload constant");
    DeviceRegistry::Get().PutConst(ordinal_, key, blob);
  }
  sg->consts.push_back(blob);
  *ptr = blob->ptr();
  return absl::OkStatus();
}

absl::Status HipModelExecutor::UploadConst(const std::string& key, const void* data, size_t bytes,
                                           PreparedSubgraph* sg, const void** dev) {
  auto blob = DeviceRegistry::Get().FindConst(ordinal_, key);
  if (!blob) {
    blob = std::make_shared<DeviceBlob>(ordinal_, bytes);
    if (!blob->ok() || !blob->Upload(0, data, bytes)) return HipErr(1, "upload table");
    DeviceRegistry::Get().PutConst(ordinal_, key, blob);
  }
  sg->consts.push_back(blob);
  *dev = blob->ptr();
  return absl::OkStatus();
}

// TRANSPOSE_CONV (int8; reference_integer_ops::TransposeConv scatters
// (x - zp) * w into an int32 scratch).  MI355X form: a transpose conv is a
// stride-1 CONV_2D over the zero-inserted input U (U[y*s][x*s] = x, the input
// zero point elsewhere, so inserted positions contribute exactly 0) with
// spatially flipped filters and top/left padding k-1-pad; integer sums are
// order-free, so the result is bit-identical.  Two launches: zero insertion
// into a per-subgraph scratch buffer, then the MFMA conv.
absl::Status HipModelExecutor::LowerTransposeConv(const HipModel& model, int oi, void* out_ptr,
                                                  const std::string& ckey, PreparedSubgraph* sg, Launch* L) {
  const TflModel& d = model.desc();
  const TflOperator& op = d.ops[oi];
  const TflTensor& w = d.tensors[op.inputs[1]];
  const TflTensor& x = d.tensors[op.inputs[2]];
  const TflTensor& out = d.tensors[op.outputs[0]];
  void* x_ptr = nullptr;
  RETURN_STATUS_IF(DevicePtr(model, op.inputs[2], sg, &x_ptr));
  const int32_t* bias = nullptr;
  if (op.inputs.size() > 3 && op.inputs[3] >= 0) bias = reinterpret_cast<const int32_t*>(d.tensors[op.inputs[3]].data);
  const FbTable& o = op.options;
  const bool same = !o.valid() || o.Int8(0, 0) == 0;
  const int sw = o.valid() ? o.Int(1, 1) : 1, sh = o.valid() ? o.Int(2, 1) : 1;
  const int b = x.shape[0], ih = x.shape[1], iw = x.shape[2], ic = x.shape[3];
  const int oc = w.shape[0], kh = w.shape[1], kw = w.shape[2];
  const int oh = out.shape[1], ow = out.shape[2];
  if (out.shape[0] != b || out.shape[3] != oc) return absl::InternalError("TRANSPOSE_CONV shape mismatch");
  // transpose_conv.cc: padding computed as for a conv whose input is the output
  const int ph = ComputePadding(sh, 1, oh, kh, ComputeOutSize(same, oh, kh, sh, 1));
  const int pw = ComputePadding(sw, 1, ow, kw, ComputeOutSize(same, ow, kw, sw, 1));
  const int uh = (ih - 1) * sh + 1, uw = (iw - 1) * sw + 1;
  // zero-inserted input in a scratch buffer owned by this subgraph
  auto scratch = std::make_shared<DeviceBlob>(ordinal_, static_cast<size_t>(b) * uh * uw * ic);
  if (!scratch->ok()) return absl::InternalError("HBM scratch allocation failed");
  sg->consts.push_back(scratch);
  Launch Z;
  Z.kind = Launch::kZeroInsert;
  Z.op_index = oi;
  Z.kernel = "zero_insert_kernel";
  Z.zi = bh_zero_insert_params{};
  Z.zi.batch = b; Z.zi.in_h = ih; Z.zi.in_w = iw; Z.zi.channels = ic;
  Z.zi.stride_h = sh; Z.zi.stride_w = sw; Z.zi.out_h = uh; Z.zi.out_w = uw;
  Z.zi.fill = static_cast<uint32_t>(Zp(x)) & 0xffu;
  Z.zi.input = x_ptr;
  Z.zi.output = scratch->ptr();
  Z.alg_bytes = static_cast<double>(x.num_elements()) + static_cast<double>(b) * uh * uw * ic;
  sg->launches.push_back(Z);
  // flipped, packed filters + folded bias (int8 filters: zero point 0)
  const int K = kh * kw * ic;
  int kp = 0, np = 0;
  bh_conv_packed_geometry(oc, K, &kp, &np);
  const size_t wbytes = static_cast<size_t>(kp) * np;
  const size_t tbytes = 12ull * oc;
  std::vector<int32_t> mult, shift;
  ConvMultipliers(Scale(x), w.scale, oc, Scale(out), false, &mult, &shift);
  auto blob = DeviceRegistry::Get().FindConst(ordinal_, ckey);
  if (!blob) {
    std::vector<int8_t> flipped(static_cast<size_t>(oc) * K);
    for (int co = 0; co < oc; ++co)
      for (int fy = 0; fy < kh; ++fy)
        for (int fx = 0; fx < kw; ++fx)
          for (int ci = 0; ci < ic; ++ci)
            flipped[((static_cast<size_t>(co) * kh + fy) * kw + fx) * ic + ci] = static_cast<int8_t>(
                w.data[((static_cast<size_t>(co) * kh + (kh - 1 - fy)) * kw + (kw - 1 - fx)) * ic + ci]);
    std::vector<int8_t> packed(wbytes);
    std::vector<int32_t> tables(3ull * oc);
    if (bh_pack_conv_weights(flipped.data(), 1, oc, K, kp, np, bias, Zp(x), 0, packed.data(), tables.data()) != 0)
      return absl::InternalError("weight packing failed");
    std::copy(mult.begin(), mult.end(), tables.begin() + oc);
    std::copy(shift.begin(), shift.end(), tables.begin() + 2 * oc);
    blob = std::make_shared<DeviceBlob>(ordinal_, wbytes + tbytes);
    if (!blob->ok() || !blob->Upload(0, packed.data(), wbytes) ||
        !blob->Upload(wbytes, tables.data(), tbytes))
      return HipErr(1, "upload transpose-conv operands");
    DeviceRegistry::Get().PutConst(ordinal_, ckey, blob);
  }
  sg->consts.push_back(blob);
  const int32_t* tab = reinterpret_cast<const int32_t*>(static_cast<char*>(blob->ptr()) + wbytes);
  bh_conv_params& p = L->conv;
  p = bh_conv_params{};
  p.batch = b; p.in_h = uh; p.in_w = uw; p.in_c = ic;
  p.out_h = oh; p.out_w = ow; p.out_c = oc; p.k_h = kh; p.k_w = kw;
  p.stride_h = 1; p.stride_w = 1; p.dil_h = 1; p.dil_w = 1;
  p.pad_h = kh - 1 - ph; p.pad_w = kw - 1 - pw;
  p.k_pad = kp; p.n_pad = np; p.in_xor = 0;
  p.in_zp = Zp(x); p.w_zp = 0; p.out_zp = Zp(out); p.act_min = -128; p.act_max = 127;
  p.input = scratch->ptr(); p.output = out_ptr;
  p.weights = static_cast<const int8_t*>(blob->ptr());
  p.bias_eff = tab; p.mult = tab + oc; p.shift = tab + 2 * oc;
  p.requant_fast = bh_conv_requant_fast_ok(mult.data(), shift.data(), oc, K, MaxAbs(bias, oc));
  L->kind = Launch::kConv;
  L->kernel = bh_conv2d_i8_kernel(&p);
  const double M = static_cast<double>(b) * oh * ow;
  L->alg_ops = 2.0 * M * oc * K;
  L->alg_bytes = static_cast<double>(b) * uh * uw * ic + M * oc + static_cast<double>(oc) * K + 12.0 * oc;
  return absl::OkStatus();
}

// Glue ops.  Every 8-bit unary op becomes a 256-entry
// table built here with TFLite's formula (quant.cc), so the device does a
// byte gather; index maps TFLite computes in float are tabulated here too.
absl::Status HipModelExecutor::LowerGlue(const HipModel& model, int oi, void* in_ptr, void* out_ptr,
                                         const std::string& ckey, PreparedSubgraph* sg, Launch* L) {
  const TflModel& d = model.desc();
  const TflOperator& op = d.ops[oi];
  auto T = [&](int i) -> const TflTensor& { return d.tensors[i]; };
  const TflTensor& in = T(op.inputs[0]);
  const TflTensor& out = T(op.outputs[0]);
  const bool i8 = in.type == DataType::kInt8;
  const double in_bytes = static_cast<double>(meta_[op.inputs[0]]->bytes);
  const double out_bytes = static_cast<double>(meta_[op.outputs[0]]->bytes);
  L->alg_bytes = in_bytes + out_bytes;
  switch (op.builtin) {
    case kTflQuantize:
    case kTflRelu:
    case kTflRelu6:
    case kTflReluN1To1:
    case kTflLogistic:
    case kTflHardSwish: {
      L->src = in_ptr;
      L->dst = out_ptr;
      L->count = static_cast<long>(out.num_elements());
      if (op.builtin == kTflQuantize && in.type == DataType::kFloat32) {
        L->kind = Launch::kQuantF32;
        L->kernel = "quantize_f32_kernel";
        L->q_scale = Scale(out);
        L->q_zp = Zp(out);
        L->q_signed = out.type == DataType::kInt8 ? 1 : 0;
        return absl::OkStatus();
      }
      uint8_t table[256];
      if (op.builtin == kTflQuantize) {
        RequantizeTable(i8, Scale(in), Zp(in), out.type == DataType::kInt8, Scale(out), Zp(out), table);
      } else if (op.builtin == kTflLogistic) {
        LogisticTable(i8, Scale(in), Zp(in), Scale(out), Zp(out), table);
      } else if (op.builtin == kTflHardSwish) {
        if (!HardSwishTable(i8, Scale(in), Zp(in), Scale(out), Zp(out), table))
          return absl::InternalError("HARD_SWISH: output multiplier exponent > 0");
      } else {
        const float lo = op.builtin == kTflReluN1To1 ? -1.0f : 0.0f;
        const float hi = op.builtin == kTflRelu6 ? 6.0f : 1.0f;
        ReluTable(i8, Scale(in), Zp(in), Scale(out), Zp(out), lo, hi, op.builtin == kTflRelu, table);
      }
      RETURN_STATUS_IF(UploadConst(ckey + "/lut", table, sizeof(table), sg, &L->table));
      L->kind = Launch::kLutU8;
      L->kernel = "lut_u8_kernel";
      return absl::OkStatus();
    }
    case kTflDequantize: {
      float table[256];
      DequantizeTable(i8, Scale(in), Zp(in), table);
      RETURN_STATUS_IF(UploadConst(ckey + "/lut", table, sizeof(table), sg, &L->table));
      L->kind = Launch::kLutF32;
      L->kernel = "lut_f32_kernel";
      L->src = in_ptr;
      L->dst = out_ptr;
      L->count = static_cast<long>(out.num_elements());
      return absl::OkStatus();
    }
    case kTflSoftmax: {
      const float beta = op.options.valid() ? op.options.Float(0, 1.0f) : 1.0f;
      float table[256];
      SoftmaxExpTable(Scale(in), beta, table);
      const void* dt = nullptr;
      RETURN_STATUS_IF(UploadConst(ckey + "/exp", table, sizeof(table), sg, &dt));
      bh_softmax_params& p = L->softmax;
      p = bh_softmax_params{};
      p.depth = in.shape.back();
      p.rows = static_cast<long>(in.num_elements() / std::max(p.depth, 1));
      p.is_signed = i8 ? 1 : 0;
      p.table = static_cast<const float*>(dt);
      p.out_scale = Scale(out);
      p.out_zp = Zp(out);
      p.input = in_ptr;
      p.output = out_ptr;
      L->kind = Launch::kSoftmax;
      L->kernel = "softmax_kernel";
      return absl::OkStatus();
    }
    case kTflConcatenation: {
      const int rank = static_cast<int>(out.shape.size());
      int axis = op.options.valid() ? op.options.Int(0, 0) : 0;
      if (axis < 0) axis += rank;
      if (axis < 0 || axis >= rank) return absl::InternalError("CONCATENATION axis out of range");
      long outer = 1, inner = static_cast<long>(GetDataTypeBytes(out.type));
      for (int i = 0; i < axis; ++i) outer *= out.shape[i];
      for (int i = axis + 1; i < rank; ++i) inner *= out.shape[i];
      bh_concat_params& p = L->concat;
      p = bh_concat_params{};
      p.n_inputs = static_cast<int>(op.inputs.size());
      p.outer = outer;
      p.output = out_ptr;
      L->alg_bytes = out_bytes;
      for (int k = 0; k < p.n_inputs; ++k) {
        const TflTensor& x = T(op.inputs[k]);
        void* xp = nullptr;
        RETURN_STATUS_IF(DevicePtr(model, op.inputs[k], sg, &xp));
        p.input[k] = xp;
        p.row[k] = static_cast<long>(x.shape[axis]) * inner;
        L->alg_bytes += static_cast<double>(meta_.size() > static_cast<size_t>(op.inputs[k]) && meta_[op.inputs[k]]
                                                ? meta_[op.inputs[k]]->bytes
                                                : 0);
        if (out.type == DataType::kUInt8 && (Zp(x) != Zp(out) || Scale(x) != Scale(out))) {
          uint8_t table[256];
          ConcatRescaleTable(Scale(x), Zp(x), Scale(out), Zp(out), table);
          RETURN_STATUS_IF(UploadConst(ckey + "/lut" + std::to_string(k), table, sizeof(table), sg, &p.table[k]));
        }
      }
      L->kind = Launch::kConcat;
      L->kernel = "concat_kernel";
      return absl::OkStatus();
    }
    case kTflPad:
    case kTflPadV2:
    case kTflMirrorPad: {
      const TflTensor& pt = T(op.inputs[1]);
      const int rank = static_cast<int>(in.shape.size());
      std::vector<int64_t> pads(2 * static_cast<size_t>(rank), 0);
      int mirror = 0;
      if (op.builtin == kTflMirrorPad && !MirrorPadArgs(d, op, &pads, &mirror))
        return absl::InternalError("MIRROR_PAD arguments");
      for (size_t i = 0; !mirror && i < pads.size() && i * (pt.type == DataType::kInt64 ? 8 : 4) < pt.data_size;
           ++i) {
        if (pt.type == DataType::kInt64) {
          int64_t v;
          std::memcpy(&v, pt.data + 8 * i, 8);
          pads[i] = v;
        } else {
          int32_t v;
          std::memcpy(&v, pt.data + 4 * i, 4);
          pads[i] = v;
        }
      }
      bh_pad_params& p = L->pad;
      p = bh_pad_params{};
      p.elem_bytes = static_cast<int>(GetDataTypeBytes(in.type));
      Shape4(in.shape, p.in_shape);
      const int lead = 4 - rank;
      for (int dd = 0; dd < rank; ++dd) {
        p.pad_before[lead + dd] = static_cast<int>(pads[2 * dd]);
        p.pad_after[lead + dd] = static_cast<int>(pads[2 * dd + 1]);
      }
      uint32_t value = 0;
      if (op.builtin == kTflPadV2 && op.inputs.size() > 2 && op.inputs[2] >= 0) {
        const TflTensor& cv = T(op.inputs[2]);
        std::memcpy(&value, cv.data, std::min<size_t>(cv.data_size, p.elem_bytes));
      } else if (IsQ8(in.type)) {
        value = static_cast<uint32_t>(Zp(out)) & 0xffu;  // quantized PAD pads with the output zero point
      }
      p.value = value;
      p.mode = mirror;
      p.input = in_ptr;
      p.output = out_ptr;
      L->kind = Launch::kPad;
      L->kernel = "pad_kernel";
      return absl::OkStatus();
    }
    case kTflResizeNearestNeighbor:
    case kTflResizeBilinear: {
      const int b = in.shape[0], ih = in.shape[1], iw = in.shape[2], c = in.shape[3];
      const int oh = out.shape[1], ow = out.shape[2];
      const bool nearest = op.builtin == kTflResizeNearestNeighbor;
      const bool ac = op.options.valid() && op.options.Bool(nearest ? 0 : 2, false);
      const bool hp = op.options.valid() && op.options.Bool(nearest ? 1 : 3, false);
      if (nearest) {
        std::vector<int32_t> tab(static_cast<size_t>(oh) + ow);
        for (int y = 0; y < oh; ++y) tab[y] = NearestNeighborIndex(y, ih, oh, ac, hp);
        for (int x = 0; x < ow; ++x) tab[oh + x] = NearestNeighborIndex(x, iw, ow, ac, hp);
        const void* dt = nullptr;
        RETURN_STATUS_IF(UploadConst(ckey + "/idx", tab.data(), tab.size() * 4, sg, &dt));
        bh_resize_nearest_params& p = L->rnear;
        p = bh_resize_nearest_params{};
        p.batch = b; p.in_h = ih; p.in_w = iw; p.out_h = oh; p.out_w = ow;
        p.row_bytes = c * static_cast<int>(GetDataTypeBytes(in.type));
        p.y_index = static_cast<const int32_t*>(dt);
        p.x_index = static_cast<const int32_t*>(dt) + oh;
        p.input = in_ptr;
        p.output = out_ptr;
        L->kind = Launch::kResizeNearest;
        L->kernel = "resize_nearest_kernel";
      } else if (in.type == DataType::kUInt8) {
        // uint8: optimized_ops::ResizeBilinear's float path
        std::vector<int32_t> iy, ix;
        std::vector<float> fy, fx;
        BilinearFloatTable(ih, oh, ac, hp, &iy, &fy);
        BilinearFloatTable(iw, ow, ac, hp, &ix, &fx);
        // one upload: {y_idx, x_idx} int32 then {y_frac, x_frac} float
        std::vector<int32_t> blob(iy);
        blob.insert(blob.end(), ix.begin(), ix.end());
        blob.resize(blob.size() + fy.size() + fx.size());
        std::memcpy(blob.data() + iy.size() + ix.size(), fy.data(), fy.size() * 4);
        std::memcpy(blob.data() + iy.size() + ix.size() + fy.size(), fx.data(), fx.size() * 4);
        const void* dt = nullptr;
        RETURN_STATUS_IF(UploadConst(ckey + "/tab8", blob.data(), blob.size() * 4, sg, &dt));
        const int32_t* t32 = static_cast<const int32_t*>(dt);
        bh_resize_bilinear_u8_params& p = L->rbil8;
        p = bh_resize_bilinear_u8_params{};
        p.batch = b; p.in_h = ih; p.in_w = iw; p.channels = c; p.out_h = oh; p.out_w = ow;
        p.y_idx = t32;
        p.x_idx = t32 + 2 * oh;
        p.y_frac = reinterpret_cast<const float*>(t32 + 2 * oh + 2 * ow);
        p.x_frac = reinterpret_cast<const float*>(t32 + 3 * oh + 2 * ow);
        p.input = in_ptr;
        p.output = out_ptr;
        L->kind = Launch::kResizeBilinearU8;
        L->kernel = "resize_bilinear_u8_kernel";
      } else {
        std::vector<int32_t> ty, tx;
        BilinearIntegerTable(ih, oh, ac, hp, &ty);
        BilinearIntegerTable(iw, ow, ac, hp, &tx);
        ty.insert(ty.end(), tx.begin(), tx.end());
        const void* dt = nullptr;
        RETURN_STATUS_IF(UploadConst(ckey + "/tab", ty.data(), ty.size() * 4, sg, &dt));
        bh_resize_bilinear_params& p = L->rbil;
        p = bh_resize_bilinear_params{};
        p.batch = b; p.in_h = ih; p.in_w = iw; p.channels = c; p.out_h = oh; p.out_w = ow;
        p.y_tab = static_cast<const int32_t*>(dt);
        p.x_tab = static_cast<const int32_t*>(dt) + 3 * oh;
        p.input = in_ptr;
        p.output = out_ptr;
        L->kind = Launch::kResizeBilinear;
        L->kernel = "resize_bilinear_kernel";  // (row forms resize_bilinear_rows_kernel / resize_bilinear_cols_kernel when the rows fit LDS)
      }
      return absl::OkStatus();
    }
    default:
      return absl::InternalError(std::string("no lowering for ") + TflBuiltinName(op.builtin));
  }
}

absl::Status HipModelExecutor::BuildLaunches(const HipModel& model, PreparedSubgraph* sg) {
  sg->launches.clear();
  sg->fused_ops.clear();
  sg->fused_tensors.clear();
  for (int i : sg->ops) {
    if (sg->fused_ops.count(i)) continue;
    RETURN_STATUS_IF(Lower(model, i, sg));
  }
  // fused chains / blocks are GPU kernels picked by on-device timing; chains
  // first (they cut more launches), blocks over what the chains left
  if (allow_fusion_ && allow_chain_ && device_flag_ == DeviceFlag::kGPU) FuseChains(model, sg);
  if (allow_fusion_ && allow_irb_ && device_flag_ == DeviceFlag::kGPU) FuseBlocks(model, sg);
  if (allow_fusion_) FuseGlue(model, sg);
  if (allow_fusion_ && allow_group_ && device_flag_ == DeviceFlag::kGPU) RETURN_STATUS_IF(GroupConvs(sg));
  return absl::OkStatus();
}


bool HipModelExecutor::TryFuseResidualAdd(const HipModel& model, int oi, PreparedSubgraph* sg, Launch* L) {
  if (!allow_fusion_ || !allow_add_) return false;
  const TflModel& d = model.desc();
  const int t = d.ops[oi].outputs[0];
  if (consumers_[t].size() != 1) return false;
  const int j = consumers_[t][0];
  if (j <= oi || !std::binary_search(sg->ops.begin(), sg->ops.end(), j)) return false;
  const TflOperator& add = d.ops[j];
  if ((add.builtin != kTflAdd && add.builtin != kTflSub) || add.inputs.size() != 2) return false;
  if (!GpuSupports(d, add, nullptr)) return false;
  if (sg->no_fuse.count(t) || sg->extra_d2h.count(t)) return false;
  if (std::find(sg->outputs.begin(), sg->outputs.end(), t) != sg->outputs.end()) return false;
  if (std::find(d.outputs.begin(), d.outputs.end(), t) != d.outputs.end()) return false;
  const bool conv_is_first = add.inputs[0] == t;
  const int other = conv_is_first ? add.inputs[1] : add.inputs[0];
  if (other == t) return false;
  // the epilogue reads the other operand while the conv runs, so it must
  // already exist then: produced by an earlier op (an FPN's ADD of a lateral
  // conv and an upsampled map produced later must stay unfused)
  if (other < 0 || producer_[other] > oi) return false;
  const TflTensor& tc = d.tensors[t];
  const TflTensor& tr = d.tensors[other];
  const TflTensor& to = d.tensors[add.outputs[0]];
  if (tr.shape != tc.shape || to.shape != tc.shape || tr.type != tc.type || to.type != tc.type) return false;
  void* rptr = nullptr;
  void* optr = nullptr;
  if (!DevicePtr(model, other, sg, &rptr).ok() || !DevicePtr(model, add.outputs[0], sg, &optr).ok()) return false;
  const TflTensor& t1 = d.tensors[add.inputs[0]];
  const TflTensor& t2 = d.tensors[add.inputs[1]];
  const AddParams ap = AddSubParams(Scale(t1), Scale(t2), Scale(to), add.builtin == kTflSub);
  bh_conv_params& p = L->conv;
  p.residual = rptr;
  p.output = optr;
  p.add_left_shift = ap.left_shift;
  p.add_y_off = -Zp(tc);
  p.add_r_off = -Zp(tr);
  p.add_o_off = Zp(to);
  p.add_y_mult = conv_is_first ? ap.m1 : ap.m2;
  p.add_y_shift = conv_is_first ? ap.s1 : ap.s2;
  p.add_r_mult = conv_is_first ? ap.m2 : ap.m1;
  p.add_r_shift = conv_is_first ? ap.s2 : ap.s1;
  p.add_o_mult = ap.mo;
  p.add_o_shift = ap.so;
  const int act = add.options.valid() ? add.options.Int8(0, 0) : 0;
  ActivationRangeQuantized(act, Scale(to), Zp(to), to.type == DataType::kInt8, &p.add_act_min, &p.add_act_max);
  L->alg_bytes += static_cast<double>(tr.num_elements());  // residual read; y never stored
  L->kernel = WithAdd(L->kernel);
  sg->fused_ops.insert(j);
  L->out_tensor = add.outputs[0];
  sg->fused_tensors.insert(t);
  return true;
}

// float32 graphs (fp16-weight models): constants (fp16 behind DEQUANTIZE,
// or float32) are folded on the host into the layouts the bh_*_f32 kernels
// read; a DEQUANTIZE whose consumers all fold it emits nothing.
absl::Status HipModelExecutor::LowerFloat(const HipModel& model, int oi, void* in_ptr, void* out_ptr,
                                          const std::string& ckey, PreparedSubgraph* sg, Launch* L, bool* emit) {
  const TflModel& d = model.desc();
  const TflOperator& op = d.ops[oi];
  auto T = [&](int i) -> const TflTensor& { return d.tensors[i]; };
  const TflTensor& in = T(op.inputs[0]);
  const TflTensor& out = T(op.outputs[0]);
  const double io_bytes = 4.0 * (static_cast<double>(in.num_elements()) + out.num_elements());
  L->alg_bytes = io_bytes;
  auto upload = [&](const std::string& key, const std::vector<float>& v, const void** dev) {
    return UploadConst(key, v.data(), v.size() * sizeof(float), sg, dev);
  };
  switch (op.builtin) {
    case kTflDequantize: {
      const int t = op.outputs[0];
      bool all_fold = true;
      for (int c : consumers_[t]) {
        const TflOperator& co = d.ops[c];
        const bool folds = (co.builtin == kTflConv2D || co.builtin == kTflDepthwiseConv2D ||
                            co.builtin == kTflFullyConnected) &&
                           co.inputs[0] != t;
        all_fold = all_fold && folds;
      }
      std::set<int> subgraph_outputs(sg->outputs.begin(), sg->outputs.end());
      if (all_fold && !subgraph_outputs.count(t) && !sg->no_fuse.count(t)) {
        *emit = false;
        return absl::OkStatus();
      }
      const void* dev = nullptr;
      RETURN_STATUS_IF(upload(ckey + "/f32", FloatData(d, t), &dev));
      L->kind = Launch::kCopy;
      L->kernel = "copy";
      L->src = dev;
      L->dst = out_ptr;
      L->bytes = 4 * out.num_elements();
      L->alg_bytes = 2.0 * L->bytes;
      return absl::OkStatus();
    }
    case kTflConv2D:
    case kTflDepthwiseConv2D: {
      const bool dw = op.builtin == kTflDepthwiseConv2D;
      const TflTensor& w = T(op.inputs[1]);
      const FbTable& o = op.options;
      const bool same = o.Int8(0, 0) == 0;
      const int sw = o.Int(1, 1), sh = o.Int(2, 1);
      const int act = dw ? o.Int8(4, 0) : o.Int8(3, 0);
      const int dlw = dw ? o.Int(5, 1) : o.Int(4, 1);
      const int dlh = dw ? o.Int(6, 1) : o.Int(5, 1);
      const int b = in.shape[0], ih = in.shape[1], iw = in.shape[2], ic = in.shape[3];
      const int oc = dw ? w.shape[3] : w.shape[0];
      const int kh = w.shape[1], kw = w.shape[2];
      const int oh = ComputeOutSize(same, ih, kh, sh, dlh), ow = ComputeOutSize(same, iw, kw, sw, dlw);
      if (out.shape != std::vector<int>{b, oh, ow, oc}) return absl::InternalError("conv output shape mismatch");
      std::vector<float> wf = FloatData(d, op.inputs[1]);
      std::vector<float> laid(wf.size());
      if (dw) {
        laid = wf;  // [1][kh][kw][oc] is already [kh*kw][oc]
      } else {
        const int K = kh * kw * ic;  // OHWI -> [K][oc]
        for (int c = 0; c < oc; ++c)
          for (int k = 0; k < K; ++k) laid[static_cast<size_t>(k) * oc + c] = wf[static_cast<size_t>(c) * K + k];
      }
      bh_conv_f32_params& p = L->convf;
      p = bh_conv_f32_params{};
      const void* wdev = nullptr;
      RETURN_STATUS_IF(upload(ckey + "/w", laid, &wdev));
      p.weights = static_cast<const float*>(wdev);
      if (op.inputs.size() > 2 && op.inputs[2] >= 0) {
        const void* bdev = nullptr;
        RETURN_STATUS_IF(upload(ckey + "/b", FloatData(d, op.inputs[2]), &bdev));
        p.bias = static_cast<const float*>(bdev);
      }
      p.batch = b; p.in_h = ih; p.in_w = iw; p.in_c = ic; p.out_h = oh; p.out_w = ow; p.out_c = oc;
      p.k_h = kh; p.k_w = kw; p.stride_h = sh; p.stride_w = sw; p.dil_h = dlh; p.dil_w = dlw;
      p.pad_h = ComputePadding(sh, dlh, ih, kh, oh);
      p.pad_w = ComputePadding(sw, dlw, iw, kw, ow);
      p.depthwise = dw ? 1 : 0;
      p.depth_multiplier = dw ? oc / ic : 1;
      FloatActRange(act, &p.act_min, &p.act_max);
      p.input = static_cast<const float*>(in_ptr);
      p.output = static_cast<float*>(out_ptr);
      L->kind = Launch::kConvF32;
      L->kernel = dw ? "dwconv_f32_kernel" : "conv_f32_kernel";
      L->alg_ops = 2.0 * b * oh * ow * oc * kh * kw * (dw ? 1 : ic);
      L->alg_bytes = io_bytes + 4.0 * laid.size() + 4.0 * oc;
      return absl::OkStatus();
    }
    case kTflFullyConnected: {
      const TflTensor& w = T(op.inputs[1]);
      const int units = w.shape[0], depth = w.shape[1];
      bh_fc_f32_params& p = L->fcf;
      p = bh_fc_f32_params{};
      const void* wdev = nullptr;
      RETURN_STATUS_IF(upload(ckey + "/w", FloatData(d, op.inputs[1]), &wdev));
      p.weights = static_cast<const float*>(wdev);
      if (op.inputs.size() > 2 && op.inputs[2] >= 0) {
        const void* bdev = nullptr;
        RETURN_STATUS_IF(upload(ckey + "/b", FloatData(d, op.inputs[2]), &bdev));
        p.bias = static_cast<const float*>(bdev);
      }
      p.rows = static_cast<int>(in.num_elements() / depth);
      p.depth = depth;
      p.units = units;
      FloatActRange(op.options.valid() ? op.options.Int8(0, 0) : 0, &p.act_min, &p.act_max);
      p.input = static_cast<const float*>(in_ptr);
      p.output = static_cast<float*>(out_ptr);
      L->kind = Launch::kFcF32;
      L->kernel = "fc_f32_kernel";
      L->alg_ops = 2.0 * p.rows * units * depth;
      L->alg_bytes = io_bytes + 4.0 * units * depth;
      return absl::OkStatus();
    }
    case kTflAdd:
    case kTflSub:
    case kTflMul:
    case kTflSquaredDifference: {
      const TflTensor& bt = T(op.inputs[1]);
      void* b_ptr = nullptr;
      RETURN_STATUS_IF(DevicePtr(model, op.inputs[1], sg, &b_ptr));
      bh_eltwise_f32_params& p = L->eltf;
      p = bh_eltwise_f32_params{};
      p.kind = op.builtin == kTflAdd   ? BH_ELTF_ADD
               : op.builtin == kTflSub ? BH_ELTF_SUB
               : op.builtin == kTflMul ? BH_ELTF_MUL
                                       : BH_ELTF_SQDIFF;
      Shape4(in.shape, p.shape_a);
      Shape4(bt.shape, p.shape_b);
      Shape4(out.shape, p.shape_o);
      FloatActRange(op.options.valid() ? op.options.Int8(0, 0) : 0, &p.act_min, &p.act_max);
      p.a = static_cast<const float*>(in_ptr);
      p.b = static_cast<const float*>(b_ptr);
      p.out = static_cast<float*>(out_ptr);
      L->kind = Launch::kEltwiseF32;
      L->kernel = "eltwise_f32_kernel";
      L->alg_bytes += 4.0 * bt.num_elements();
      return absl::OkStatus();
    }
    case kTflAveragePool2D:
    case kTflMaxPool2D: {
      const FbTable& o = op.options;
      const bool same = o.Int8(0, 0) == 0;
      const int sw = o.Int(1, 1), sh = o.Int(2, 1), fw = o.Int(3, 1), fh = o.Int(4, 1);
      bh_pool_f32_params& p = L->poolf;
      p = bh_pool_f32_params{};
      p.kind = op.builtin == kTflAveragePool2D ? BH_POOL_AVG : BH_POOL_MAX;
      p.batch = in.shape[0]; p.in_h = in.shape[1]; p.in_w = in.shape[2]; p.channels = in.shape[3];
      p.out_h = ComputeOutSize(same, p.in_h, fh, sh, 1);
      p.out_w = ComputeOutSize(same, p.in_w, fw, sw, 1);
      p.f_h = fh; p.f_w = fw; p.stride_h = sh; p.stride_w = sw;
      p.pad_h = ComputePadding(sh, 1, p.in_h, fh, p.out_h);
      p.pad_w = ComputePadding(sw, 1, p.in_w, fw, p.out_w);
      FloatActRange(o.Int8(5, 0), &p.act_min, &p.act_max);
      p.input = static_cast<const float*>(in_ptr);
      p.output = static_cast<float*>(out_ptr);
      L->kind = Launch::kPoolF32;
      L->kernel = "pool_f32_kernel";
      return absl::OkStatus();
    }
    case kTflSoftmax:
      L->kind = Launch::kSoftmaxF32;
      L->kernel = "softmax_f32_kernel";
      L->beta = op.options.valid() ? op.options.Float(0, 1.0f) : 1.0f;
      L->depth = in.shape.back();
      L->count = static_cast<long>(in.num_elements() / std::max(L->depth, 1));
      L->src = in_ptr;
      L->dst = out_ptr;
      return absl::OkStatus();
    default: {  // RELU / RELU6 / RELU_N1_TO_1 / LOGISTIC / RSQRT
      L->kind = Launch::kUnaryF32;
      L->kernel = "unary_f32_kernel";
      L->unary_kind = op.builtin == kTflLogistic ? BH_UNARY_LOGISTIC
                      : op.builtin == kTflRsqrt  ? BH_UNARY_RSQRT
                                                 : BH_UNARY_CLAMP;
      L->lo = op.builtin == kTflReluN1To1 ? -1.f : 0.f;
      L->hi = op.builtin == kTflRelu6 ? 6.f : (op.builtin == kTflReluN1To1 ? 1.f : std::numeric_limits<float>::infinity());
      L->count = static_cast<long>(in.num_elements());
      L->src = in_ptr;
      L->dst = out_ptr;
      return absl::OkStatus();
    }
  }
}

absl::Status HipModelExecutor::Lower(const HipModel& model, int oi, PreparedSubgraph* sg) {
  const TflModel& d = model.desc();
  const TflOperator& op = d.ops[oi];
  std::string why;
  const bool cpu = device_flag_ == DeviceFlag::kCPU;
  if (!(cpu ? CpuSupports(d, op, &why) : GpuSupports(d, op, &why)))
    return absl::InternalError("HIP backend cannot run op " + std::to_string(oi) + " (" +
                               TflBuiltinName(op.builtin) + ") on " + ToString(device_flag_) + ": " + why);
  auto T = [&](int i) -> const TflTensor& { return d.tensors[i]; };
  const TflTensor& in = T(op.inputs[0]);
  const TflTensor& out = T(op.outputs[0]);
  void* in_ptr = nullptr;
  void* out_ptr = nullptr;
  RETURN_STATUS_IF(DevicePtr(model, op.inputs[0], sg, &in_ptr));
  RETURN_STATUS_IF(DevicePtr(model, op.outputs[0], sg, &out_ptr));
  const bool i8 = in.type == DataType::kInt8;
  const std::string ckey = "m" + Hex(model.serial()) + "/op" + std::to_string(oi);
  Launch L;
  L.op_index = oi;
  L.out_tensor = op.outputs[0];

  if (IsFloatOp(d, op)) {
    bool emit = true;
    RETURN_STATUS_IF(LowerFloat(model, oi, in_ptr, out_ptr, ckey, sg, &L, &emit));
    if (emit) sg->launches.push_back(L);
    return absl::OkStatus();
  }
  if (op.builtin == kTflConv2D || op.builtin == kTflDepthwiseConv2D) {
    const bool dw = op.builtin == kTflDepthwiseConv2D;
    const TflTensor& w = T(op.inputs[1]);
    const int32_t* bias = nullptr;
    if (op.inputs.size() > 2 && op.inputs[2] >= 0) bias = reinterpret_cast<const int32_t*>(T(op.inputs[2]).data);
    const FbTable& o = op.options;
    const bool same = o.Int8(0, 0) == 0;
    const int sw = o.Int(1, 1), sh = o.Int(2, 1);
    const int act = dw ? o.Int8(4, 0) : o.Int8(3, 0);
    const int dlw = dw ? o.Int(5, 1) : o.Int(4, 1);
    const int dlh = dw ? o.Int(6, 1) : o.Int(5, 1);
    const int b = in.shape[0], ih = in.shape[1], iw = in.shape[2], ic = in.shape[3];
    const int oc = dw ? w.shape[3] : w.shape[0];
    const int kh = w.shape[1], kw = w.shape[2];
    const int oh = ComputeOutSize(same, ih, kh, sh, dlh);
    const int ow = ComputeOutSize(same, iw, kw, sw, dlw);
    if (out.shape != std::vector<int>{b, oh, ow, oc}) return absl::InternalError("conv output shape mismatch");
    const int ph = ComputePadding(sh, dlh, ih, kh, oh);
    const int pw = ComputePadding(sw, dlw, iw, kw, ow);
    std::vector<int32_t> mult, shift;
    ConvMultipliers(Scale(in), w.scale, oc, Scale(out), !i8, &mult, &shift);
    int32_t amin, amax;
    ActivationRangeQuantized(act, Scale(out), Zp(out), i8, &amin, &amax);
    const int32_t in_zp = Dom(in);
    const int32_t w_zp = i8 ? 0 : Dom(w);  // int8 kernels ignore the filter zero point
    const double M = static_cast<double>(b) * oh * ow;
    if (!dw) {
      const int K = kh * kw * ic;
      int kp = 0, np = 0;
      bh_conv_packed_geometry(oc, K, &kp, &np);
      const size_t wbytes = static_cast<size_t>(kp) * np;
      const size_t tbytes = 12ull * oc;
      auto blob = DeviceRegistry::Get().FindConst(ordinal_, ckey);
      if (!blob) {
        std::vector<int8_t> packed(wbytes);
        std::vector<int32_t> tables(3ull * oc);
        if (bh_pack_conv_weights(w.data, i8 ? 1 : 0, oc, K, kp, np, bias, in_zp, w_zp, packed.data(), tables.data()) != 0)
          return absl::InternalError("weight packing failed");
        std::copy(mult.begin(), mult.end(), tables.begin() + oc);
        std::copy(shift.begin(), shift.end(), tables.begin() + 2 * oc);
        blob = std::make_shared<DeviceBlob>(ordinal_, wbytes + tbytes);
        if (!blob->ok() || !blob->Upload(0, packed.data(), wbytes) ||
            !blob->Upload(wbytes, tables.data(), tbytes))
          return HipErr(1, "upload conv operands");
        DeviceRegistry::Get().PutConst(ordinal_, ckey, blob);
      }
      sg->consts.push_back(blob);
      const int32_t* tab = reinterpret_cast<const int32_t*>(static_cast<char*>(blob->ptr()) + wbytes);
      bh_conv_params& p = L.conv;
      p = bh_conv_params{};
      p.batch = b; p.in_h = ih; p.in_w = iw; p.in_c = ic;
      p.out_h = oh; p.out_w = ow; p.out_c = oc; p.k_h = kh; p.k_w = kw;
      p.stride_h = sh; p.stride_w = sw; p.dil_h = dlh; p.dil_w = dlw; p.pad_h = ph; p.pad_w = pw;
      p.k_pad = kp; p.n_pad = np; p.in_xor = i8 ? 0 : 0x80;
      p.in_zp = in_zp; p.w_zp = w_zp; p.out_zp = Zp(out); p.act_min = amin; p.act_max = amax;
      p.input = in_ptr; p.output = out_ptr;
      p.weights = static_cast<const int8_t*>(blob->ptr());
      p.bias_eff = tab; p.mult = tab + oc; p.shift = tab + 2 * oc;
      p.requant_fast = bh_conv_requant_fast_ok(mult.data(), shift.data(), oc, K, MaxAbs(bias, oc));
      L.kind = Launch::kConv;
      L.kernel = bh_conv2d_i8_kernel(&p);  // the kernel bh_conv2d_i8 dispatches to
      L.alg_ops = 2.0 * M * oc * K;
      L.alg_bytes = static_cast<double>(in.num_elements()) + M * oc + static_cast<double>(oc) * K + 12.0 * oc;
    } else {
      const int dm = oc / ic;
      const size_t wbytes = static_cast<size_t>(kh) * kw * oc;
      const size_t wpad = (wbytes + 15) / 16 * 16;
      const size_t tbytes = 12ull * oc;
      // 3x3 / dm 1 layers also get the dot4 kernel's tap table (bh_pack_dw_taps)
      const bool dot = kh == 3 && kw == 3 && dm == 1 && oc % 4 == 0;
      const size_t pbytes = dot ? 16ull * oc : 0;
      auto blob = DeviceRegistry::Get().FindConst(ordinal_, ckey);
      if (!blob) {
        std::vector<uint8_t> wd(wpad, 0);
        for (size_t i = 0; i < wbytes; ++i) wd[i] = i8 ? w.data[i] : static_cast<uint8_t>(w.data[i] ^ 0x80);
        std::vector<int32_t> tables(3ull * oc, 0);
        for (int c = 0; c < oc; ++c) tables[c] = bias ? bias[c] : 0;
        std::copy(mult.begin(), mult.end(), tables.begin() + oc);
        std::copy(shift.begin(), shift.end(), tables.begin() + 2 * oc);
        std::vector<int32_t> taps(pbytes / 4);
        if (dot && bh_pack_dw_taps(reinterpret_cast<const int8_t*>(wd.data()), oc, tables.data(), in_zp, w_zp,
                                   taps.data()) != 0)
          return absl::InternalError("depthwise tap packing failed");
        blob = std::make_shared<DeviceBlob>(ordinal_, wpad + tbytes + pbytes);
        if (!blob->ok() || !blob->Upload(0, wd.data(), wpad) ||
            !blob->Upload(wpad, tables.data(), tbytes) || (dot && !blob->Upload(wpad + tbytes, taps.data(), pbytes)))
          return HipErr(1, "upload depthwise operands");
        DeviceRegistry::Get().PutConst(ordinal_, ckey, blob);
      }
      sg->consts.push_back(blob);
      const int32_t* tab = reinterpret_cast<const int32_t*>(static_cast<char*>(blob->ptr()) + wpad);
      bh_dwconv_params& p = L.dw;
      p = bh_dwconv_params{};
      p.batch = b; p.in_h = ih; p.in_w = iw; p.in_c = ic;
      p.out_h = oh; p.out_w = ow; p.out_c = oc; p.depth_multiplier = dm; p.k_h = kh; p.k_w = kw;
      p.stride_h = sh; p.stride_w = sw; p.dil_h = dlh; p.dil_w = dlw; p.pad_h = ph; p.pad_w = pw;
      p.in_xor = i8 ? 0 : 0x80; p.in_zp = in_zp; p.w_zp = w_zp; p.out_zp = Zp(out);
      p.act_min = amin; p.act_max = amax; p.input = in_ptr; p.output = out_ptr;
      p.weights = static_cast<const int8_t*>(blob->ptr());
      p.bias = tab; p.mult = tab + oc; p.shift = tab + 2 * oc;
      if (dot && !blob->host()) p.taps = tab + 3 * oc;
      p.requant_fast = bh_conv_requant_fast_ok(mult.data(), shift.data(), oc, kh * kw, MaxAbs(bias, oc));
      L.kind = Launch::kDwConv;
      L.kernel = bh_dwconv2d_i8_kernel(&p);  // the kernel bh_dwconv2d_i8 dispatches to
      L.alg_ops = 2.0 * M * oc * kh * kw;
      L.alg_bytes = static_cast<double>(in.num_elements()) + M * oc + static_cast<double>(wbytes) + 12.0 * oc;
    }
  } else if (op.builtin == kTflFullyConnected) {
    const TflTensor& w = T(op.inputs[1]);
    const int32_t* bias = nullptr;
    if (op.inputs.size() > 2 && op.inputs[2] >= 0) bias = reinterpret_cast<const int32_t*>(T(op.inputs[2]).data);
    const int act = op.options.valid() ? op.options.Int8(0, 0) : 0;
    const int units = w.shape[0], depth = w.shape[1];
    const int rows = static_cast<int>(in.num_elements() / depth);
    const int depth_pad = (depth + 15) / 16 * 16;
    int32_t mult, shift, amin, amax;
    FullyConnectedMultiplier(Scale(in), Scale(w), Scale(out), &mult, &shift);
    ActivationRangeQuantized(act, Scale(out), Zp(out), i8, &amin, &amax);
    const int32_t in_zp = Dom(in), w_zp = Dom(w);
    const size_t wbytes = static_cast<size_t>(units) * depth_pad;
    const size_t tbytes = 12ull * units;
    auto blob = DeviceRegistry::Get().FindConst(ordinal_, ckey);
    if (!blob) {
      std::vector<int8_t> packed(wbytes, 0);
      std::vector<int32_t> tables(3ull * units);
      for (int u = 0; u < units; ++u) {
        int64_t s = 0;
        for (int k = 0; k < depth; ++k) {
          const uint8_t raw = w.data[static_cast<size_t>(u) * depth + k];
          const int v = i8 ? static_cast<int>(static_cast<int8_t>(raw)) : static_cast<int>(raw) - 128;
          packed[static_cast<size_t>(u) * depth_pad + k] = static_cast<int8_t>(v);
          s += v;
        }
        tables[u] = static_cast<int32_t>((bias ? bias[u] : 0) - static_cast<int64_t>(in_zp) * s +
                                         static_cast<int64_t>(depth) * in_zp * w_zp);
        tables[units + u] = mult;
        tables[2 * units + u] = shift;
      }
      blob = std::make_shared<DeviceBlob>(ordinal_, wbytes + tbytes);
      if (!blob->ok() || !blob->Upload(0, packed.data(), wbytes) ||
          !blob->Upload(wbytes, tables.data(), tbytes))
        return HipErr(1, "upload fc operands");
      DeviceRegistry::Get().PutConst(ordinal_, ckey, blob);
    }
    sg->consts.push_back(blob);
    const int32_t* tab = reinterpret_cast<const int32_t*>(static_cast<char*>(blob->ptr()) + wbytes);
    bh_fc_params& p = L.fc;
    p = bh_fc_params{};
    p.rows = rows; p.depth = depth; p.depth_pad = depth_pad; p.units = units;
    p.in_xor = i8 ? 0 : 0x80; p.in_zp = in_zp; p.w_zp = w_zp; p.out_zp = Zp(out);
    p.act_min = amin; p.act_max = amax; p.input = in_ptr; p.output = out_ptr;
    p.weights = static_cast<const int8_t*>(blob->ptr());
    p.bias_eff = tab; p.mult = tab + units; p.shift = tab + 2 * units;
    L.kind = Launch::kFc;
    L.kernel = "fc_kernel";
    L.alg_ops = 2.0 * rows * units * depth;
    L.alg_bytes = static_cast<double>(rows) * depth + static_cast<double>(rows) * units +
                  static_cast<double>(units) * depth + 12.0 * units;
  } else if (op.builtin == kTflAdd || op.builtin == kTflSub || op.builtin == kTflMul) {
    const TflTensor& b = T(op.inputs[1]);
    void* b_ptr = nullptr;
    RETURN_STATUS_IF(DevicePtr(model, op.inputs[1], sg, &b_ptr));
    const int act = op.options.valid() ? op.options.Int8(0, 0) : 0;
    bh_eltwise_params& p = L.elt;
    p = bh_eltwise_params{};
    p.in_signed = i8 ? 1 : 0;
    Shape4(in.shape, p.shape_a);
    Shape4(b.shape, p.shape_b);
    Shape4(out.shape, p.shape_o);
    p.a_off = -Zp(in);
    p.b_off = -Zp(b);
    p.o_off = Zp(out);
    ActivationRangeQuantized(act, Scale(out), Zp(out), i8, &p.act_min, &p.act_max);
    if (op.builtin == kTflMul) {
      p.kind = BH_ELT_MUL;
      MulMultiplier(Scale(in), Scale(b), Scale(out), &p.o_mult, &p.o_shift);
    } else {
      p.kind = BH_ELT_ADD;
      const AddParams ap = AddSubParams(Scale(in), Scale(b), Scale(out), op.builtin == kTflSub);
      p.left_shift = ap.left_shift;
      p.a_mult = ap.m1; p.a_shift = ap.s1;
      p.b_mult = ap.m2; p.b_shift = ap.s2;
      p.o_mult = ap.mo; p.o_shift = ap.so;
    }
    p.a = in_ptr; p.b = b_ptr; p.out = out_ptr;
    L.kind = Launch::kEltwise;
    L.kernel = "eltwise_kernel";
    L.alg_bytes = static_cast<double>(in.num_elements() + b.num_elements() + out.num_elements());
  } else if (op.builtin == kTflAveragePool2D || op.builtin == kTflMaxPool2D) {
    const FbTable& o = op.options;
    const bool same = o.Int8(0, 0) == 0;
    const int sw = o.Int(1, 1), sh = o.Int(2, 1), fw = o.Int(3, 1), fh = o.Int(4, 1);
    const int act = o.Int8(5, 0);
    bh_pool_params& p = L.pool;
    p = bh_pool_params{};
    p.kind = op.builtin == kTflAveragePool2D ? BH_POOL_AVG : BH_POOL_MAX;
    p.in_signed = i8 ? 1 : 0;
    p.batch = in.shape[0]; p.in_h = in.shape[1]; p.in_w = in.shape[2]; p.channels = in.shape[3];
    p.out_h = ComputeOutSize(same, p.in_h, fh, sh, 1);
    p.out_w = ComputeOutSize(same, p.in_w, fw, sw, 1);
    p.f_h = fh; p.f_w = fw; p.stride_h = sh; p.stride_w = sw;
    p.pad_h = ComputePadding(sh, 1, p.in_h, fh, p.out_h);
    p.pad_w = ComputePadding(sw, 1, p.in_w, fw, p.out_w);
    ActivationRangeQuantized(act, Scale(out), Zp(out), i8, &p.act_min, &p.act_max);
    p.input = in_ptr; p.output = out_ptr;
    L.kind = Launch::kPool;
    L.kernel = "pool_kernel";
    L.alg_bytes = static_cast<double>(in.num_elements() + out.num_elements());
  } else if (op.builtin == kTflCustom) {
    // TFLite_Detection_PostProcess (CPU worker only: CpuSupports)
    CpuDetectionParams& p = L.det;
    if (!DetectionSupported(d, op, &p)) return absl::InternalError("unsupported custom op " + op.custom_code);
    void* scores = nullptr;
    void* anchors = nullptr;
    void* outs[4];
    RETURN_STATUS_IF(DevicePtr(model, op.inputs[1], sg, &scores));
    RETURN_STATUS_IF(DevicePtr(model, op.inputs[2], sg, &anchors));
    for (int k = 0; k < 4; ++k) RETURN_STATUS_IF(DevicePtr(model, op.outputs[k], sg, &outs[k]));
    p.box_encodings = static_cast<const float*>(in_ptr);
    p.class_scores = static_cast<const float*>(scores);
    p.anchors = static_cast<const float*>(anchors);
    p.out_boxes = static_cast<float*>(outs[0]);
    p.out_classes = static_cast<float*>(outs[1]);
    p.out_scores = static_cast<float*>(outs[2]);
    p.out_num = static_cast<float*>(outs[3]);
    L.kind = Launch::kDetectionPost;
    L.kernel = "detection_postprocess_host";
  } else if (op.builtin == kTflMean) {
    // MEAN: host kernel on a CPU worker, mean_kernel on the GPU
    CpuMeanParams& p = L.mean;
    p = CpuMeanParams{};
    if (!MeanArgs(d, op, &p.outer, &p.reduce, &p.inner)) return absl::InternalError("unsupported MEAN");
    p.type = in.type == DataType::kFloat32 ? 0 : (in.type == DataType::kInt8 ? 1 : 2);
    if (p.type) {
      // optimized_integer_ops::Mean (TFLite 2.9.2): the float products as
      // written there, then QuantizeMultiplier of the float scale
      const float in_scale = Scale(in), out_scale = Scale(out);
      const float n = static_cast<float>(p.reduce);
      p.bias = Zp(out) - static_cast<int32_t>(Zp(in) * in_scale / out_scale);
      const float real_scale = in_scale / (n * out_scale);
      int shift = 0;
      QuantizeMultiplier(static_cast<double>(real_scale), &p.multiplier, &shift);
      p.shift = shift;
    }
    p.input = in_ptr;
    p.output = out_ptr;
    L.kind = Launch::kMean;
    L.kernel = device_flag_ == DeviceFlag::kGPU ? "mean_kernel" : "mean_host";
    L.alg_bytes = static_cast<double>(meta_[op.inputs[0]]->bytes + meta_[op.outputs[0]]->bytes);
  } else if (op.builtin == kTflTransposeConv) {
    RETURN_STATUS_IF(LowerTransposeConv(model, oi, out_ptr, ckey, sg, &L));
  } else if (op.builtin != kTflReshape && op.builtin != kTflSqueeze) {
    RETURN_STATUS_IF(LowerGlue(model, oi, in_ptr, out_ptr, ckey, sg, &L));
  } else {  // RESHAPE / SQUEEZE: same bytes, new dims
    L.kind = Launch::kCopy;
    L.kernel = "copy";
    L.src = in_ptr;
    L.dst = out_ptr;
    L.bytes = meta_[op.outputs[0]]->bytes;
    L.alg_bytes = 2.0 * L.bytes;
    if (L.src == L.dst) return absl::OkStatus();  // aliased slot: nothing to move
  }
  if (L.kind == Launch::kConv) {
    const bh_conv_params c = L.conv;
    const long M = static_cast<long>(c.batch) * c.out_h * c.out_w;
    if (c.k_h == 1 && c.k_w == 1 && c.stride_h == 1 && c.stride_w == 1 && M <= 4) {
      // a 1x1 conv over a handful of pixels (the classifier at batch 1) is
      // a GEMV: run it on the weight-streaming FC kernel with the same
      // packed operands (Bt rows are K-contiguous, bias_eff identical)
      Launch F;
      F.kind = Launch::kFc;
      F.op_index = oi;
      F.out_tensor = L.out_tensor;
      bh_fc_params& f = F.fc;
      f = bh_fc_params{};
      f.rows = static_cast<int>(M); f.depth = c.in_c; f.depth_pad = c.k_pad; f.units = c.out_c;
      f.in_xor = c.in_xor; f.in_zp = c.in_zp; f.w_zp = c.w_zp; f.out_zp = c.out_zp;
      f.act_min = c.act_min; f.act_max = c.act_max; f.input = c.input; f.output = c.output;
      f.weights = c.weights; f.bias_eff = c.bias_eff; f.mult = c.mult; f.shift = c.shift;
      F.kernel = "fc_kernel";
      F.alg_bytes = L.alg_bytes;
      F.alg_ops = L.alg_ops;
      L = F;
    } else {
      TryFuseResidualAdd(model, oi, sg, &L);
    }
  }
  sg->launches.push_back(L);
  return absl::OkStatus();
}


}  // namespace hip
}  // namespace band
