// Helpers shared by the HipModelExecutor translation units (model_executor.cc,
// lower.cc, fusion.cc, job_batch.cc): TFLite tensor / quantisation accessors
// and the op-set predicates the support checks and the lowering both use.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "backend/hip/model_executor.h"
#include "backend/hip/quant.h"

#define RETURN_STATUS_IF(expr)      \
  do {                              \
    absl::Status _st = (expr);      \
    if (!_st.ok()) return _st;      \
  } while (0)

namespace band {
namespace hip {
namespace ex {

// set while PrepareJobBatches constructs a variant executor: a kCPU variant
// then makes no host pool of its own (job_batch.cc)
extern thread_local bool t_variant_ctor;


constexpr size_t kAlign = 256;

inline bool IsQ8(DataType t) { return t == DataType::kInt8 || t == DataType::kUInt8; }

// zero point in the kernels' int8 domain (uint8 values are XOR 0x80 = x-128)
inline int32_t Dom(const TflTensor& t) {
  const int32_t zp = t.zero_point.empty() ? 0 : static_cast<int32_t>(t.zero_point[0]);
  return t.type == DataType::kUInt8 ? zp - 128 : zp;
}
inline int32_t Zp(const TflTensor& t) { return t.zero_point.empty() ? 0 : static_cast<int32_t>(t.zero_point[0]); }
inline float Scale(const TflTensor& t) { return t.scale.empty() ? 0.0f : t.scale[0]; }
inline bool HasQ(const TflTensor& t) { return !t.scale.empty(); }

inline std::string Hex(uint64_t v) {
  char b[32];
  std::snprintf(b, sizeof(b), "%llx", static_cast<unsigned long long>(v));
  return b;
}

inline void Shape4(const std::vector<int>& s, int* out) {
  const int pad = 4 - static_cast<int>(s.size());
  for (int i = 0; i < 4; ++i) out[i] = i < pad ? 1 : s[i - pad];
}

inline absl::Status HipErr(int rc, const char* what) {
  return absl::InternalError(std::string("HIP Error: ") + what + " (" + std::to_string(rc) + "): " + bh_last_error());
}


// "<conv kernel>+add": a conv launch with the following ADD in its epilogue
inline const char* WithAdd(const char* k) {
  static const char* const names[][2] = {{"conv_mfma_kernel", "conv_mfma_kernel+add"},
                                         {"conv_xs_kernel", "conv_xs_kernel+add"},
                                         {"conv_rows_kernel", "conv_rows_kernel+add"},
                                         {"conv_direct_kernel", "conv_direct_kernel+add"},
                                         {"conv_stem_kernel", "conv_stem_kernel+add"}};
  for (const auto& n : names)
    if (std::strcmp(k, n[0]) == 0) return n[1];
  return k;
}

inline int64_t MaxAbs(const int32_t* v, int n) {
  int64_t m = 0;
  for (int i = 0; v && i < n; ++i) m = std::max<int64_t>(m, v[i] < 0 ? -(int64_t)v[i] : (int64_t)v[i]);
  return m;
}

// TFLite fp16 post-training quantization keeps constants in float16 behind
// DEQUANTIZE ops; such a tensor is a constant of the float graph
inline const TflOperator* ProducerOf(const TflModel& m, int t) {
  for (const TflOperator& op : m.ops)
    for (int o : op.outputs)
      if (o == t) return &op;
  return nullptr;
}
inline bool FoldableF16(const TflModel& m, int t) {
  if (t < 0 || m.tensors[t].type != DataType::kFloat32) return false;
  const TflOperator* p = ProducerOf(m, t);
  return p && p->builtin == kTflDequantize && !p->inputs.empty() && p->inputs[0] >= 0 &&
         m.tensors[p->inputs[0]].is_const() && m.tensors[p->inputs[0]].type == DataType::kFloat16;
}
inline bool ConstFloat(const TflModel& m, int t) {
  return t >= 0 && ((m.tensors[t].is_const() && m.tensors[t].type == DataType::kFloat32) || FoldableF16(m, t));
}
inline float HalfToFloat(uint16_t h) {
  const uint32_t sign = (h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1fu, man = h & 0x3ffu, bits;
  if (exp == 0) {
    if (man == 0) {
      bits = sign;
    } else {  // subnormal: renormalise
      exp = 127 - 15 + 1;
      while (!(man & 0x400u)) {
        man <<= 1;
        --exp;
      }
      bits = sign | (exp << 23) | ((man & 0x3ffu) << 13);
    }
  } else if (exp == 31) {
    bits = sign | 0x7f800000u | (man << 13);
  } else {
    bits = sign | ((exp + 127 - 15) << 23) | (man << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}
// float values of a ConstFloat tensor
inline std::vector<float> FloatData(const TflModel& m, int t) {
  const TflTensor* src = &m.tensors[t];
  if (!src->is_const()) src = &m.tensors[ProducerOf(m, t)->inputs[0]];
  const size_t n = src->num_elements();
  std::vector<float> v(n);
  if (src->type == DataType::kFloat32) {
    std::memcpy(v.data(), src->data, 4 * n);
  } else {
    for (size_t i = 0; i < n; ++i) {
      uint16_t h;
      std::memcpy(&h, src->data + 2 * i, 2);
      v[i] = HalfToFloat(h);
    }
  }
  return v;
}
// fused activation bounds of a float op (kernels/kernel_util.h
// CalculateActivationRange)
inline void FloatActRange(int act, float* lo, float* hi) {
  const float inf = std::numeric_limits<float>::infinity();
  *lo = act == 1 || act == 3 ? 0.f : (act == 2 ? -1.f : -inf);
  *hi = act == 3 ? 6.f : (act == 2 ? 1.f : inf);
}
inline bool IsFloatOp(const TflModel& m, const TflOperator& op) {
  if (op.inputs.empty() || op.inputs[0] < 0) return false;
  const DataType t = m.tensors[op.inputs[0]].type;
  switch (op.builtin) {
    case kTflConv2D: case kTflDepthwiseConv2D: case kTflFullyConnected: case kTflAdd: case kTflSub: case kTflMul:
    case kTflAveragePool2D: case kTflMaxPool2D: case kTflRelu: case kTflRelu6: case kTflReluN1To1:
    case kTflLogistic: case kTflSoftmax: case kTflSquaredDifference: case kTflRsqrt:
      return t == DataType::kFloat32;
    case kTflDequantize:
      return t == DataType::kFloat16;
    default:
      return false;
  }
}
// the float32 op set (fp16-weight models)
inline bool FloatSupports(const TflModel& m, const TflOperator& op, std::string* why) {
  auto no = [&](const char* w) {
    if (why) *why = w;
    return false;
  };
  const TflTensor& in = m.tensors[op.inputs[0]];
  const TflTensor& out = m.tensors[op.outputs[0]];
  if (op.builtin == kTflDequantize)
    return in.is_const() && out.type == DataType::kFloat32 ? true : no("float16 DEQUANTIZE of a constant only");
  if (out.type != DataType::kFloat32) return no("float32 output expected");
  switch (op.builtin) {
    case kTflConv2D:
    case kTflDepthwiseConv2D:
    case kTflFullyConnected: {
      if (op.inputs.size() < 2 || !ConstFloat(m, op.inputs[1])) return no("filter must be a float constant");
      if (op.inputs.size() > 2 && op.inputs[2] >= 0 && !ConstFloat(m, op.inputs[2]))
        return no("bias must be a float constant");
      const TflTensor& w = m.tensors[op.inputs[1]];
      if (op.builtin == kTflFullyConnected)
        return w.shape.size() == 2 && w.shape[1] > 0 && in.num_elements() % w.shape[1] == 0 ? true
                                                                                          : no("FC weights");
      if (in.shape.size() != 4 || w.shape.size() != 4 || out.shape.size() != 4) return no("conv needs 4-D");
      if (op.builtin == kTflConv2D && w.shape[3] != in.shape[3]) return no("grouped conv unsupported");
      if (op.builtin == kTflDepthwiseConv2D && (in.shape[3] == 0 || w.shape[3] % in.shape[3] != 0))
        return no("bad depth multiplier");
      return true;
    }
    case kTflAdd:
    case kTflSub:
    case kTflMul:
    case kTflSquaredDifference: {
      if (op.inputs.size() != 2 || op.inputs[1] < 0) return no("binary op needs 2 inputs");
      const TflTensor& b = m.tensors[op.inputs[1]];
      if (b.type != DataType::kFloat32 || in.shape.size() > 4 || b.shape.size() > 4 || out.shape.size() > 4)
        return no("float32, rank <= 4");
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
      return in.shape.size() == 4 ? true : no("4-D only");
    case kTflSoftmax:
      return !in.shape.empty() ? true : no("rank >= 1");
    default:
      return true;  // RELU / RELU6 / RELU_N1_TO_1 / LOGISTIC / RSQRT
  }
}

// MIRROR_PAD paddings (constant [rank][2] int32 / int64) and mode
// (MirrorPadOptions.mode: 0 REFLECT, 1 SYMMETRIC -> bh_pad_params.mode 1 / 2)
inline bool MirrorPadArgs(const TflModel& m, const TflOperator& op, std::vector<int64_t>* pads, int* mode) {
  if (op.inputs.size() < 2 || op.inputs[1] < 0) return false;
  const TflTensor& in = m.tensors[op.inputs[0]];
  const TflTensor& pt = m.tensors[op.inputs[1]];
  if (!pt.is_const() || (pt.type != DataType::kInt32 && pt.type != DataType::kInt64)) return false;
  const int rank = static_cast<int>(in.shape.size());
  const size_t eb = pt.type == DataType::kInt64 ? 8 : 4;
  if (rank < 1 || rank > 4 || pt.data_size < 2 * rank * eb) return false;
  pads->assign(2 * static_cast<size_t>(rank), 0);
  for (int i = 0; i < 2 * rank; ++i) {
    if (eb == 8) {
      int64_t v;
      std::memcpy(&v, pt.data + 8 * i, 8);
      (*pads)[i] = v;
    } else {
      int32_t v;
      std::memcpy(&v, pt.data + 4 * i, 4);
      (*pads)[i] = v;
    }
  }
  *mode = op.options.valid() && op.options.Int8(0, 0) == 1 ? 2 : 1;
  for (int dd = 0; dd < rank; ++dd) {
    const int64_t lim = in.shape[dd] - (*mode == 1 ? 1 : 0);
    if ((*pads)[2 * dd] < 0 || (*pads)[2 * dd + 1] < 0 || (*pads)[2 * dd] > lim || (*pads)[2 * dd + 1] > lim)
      return false;
  }
  return true;
}

// MEAN: the reduced axes (constant int32, negatives resolved) must be one
// contiguous run; 8-bit tensors only in the form TFLite 2.9.2 runs through
// optimized_integer_ops::Mean / optimized_ops::Mean (4-D, keep_dims, axes
// {1, 2}), the one restated by CpuMean.
inline bool MeanArgs(const TflModel& m, const TflOperator& op, long* outer, long* reduce, long* inner) {
  if (op.builtin != kTflMean || op.inputs.size() < 2 || op.inputs[1] < 0 || op.outputs.empty()) return false;
  const TflTensor& in = m.tensors[op.inputs[0]];
  const TflTensor& out = m.tensors[op.outputs[0]];
  const TflTensor& ax = m.tensors[op.inputs[1]];
  if (!ax.is_const() || ax.type != DataType::kInt32 || out.type != in.type) return false;
  const int rank = static_cast<int>(in.shape.size());
  std::set<int> axes;
  for (size_t i = 0; i * 4 < ax.data_size; ++i) {
    int32_t v;
    std::memcpy(&v, ax.data + 4 * i, 4);
    if (v < 0) v += rank;
    if (v < 0 || v >= rank) return false;
    axes.insert(v);
  }
  if (axes.empty() || *axes.rbegin() - *axes.begin() + 1 != static_cast<int>(axes.size())) return false;
  if (in.type != DataType::kFloat32) {
    const bool keep = op.options.valid() && op.options.Int8(0, 0) != 0;
    if (!IsQ8(in.type) || !HasQ(in) || !HasQ(out) || rank != 4 || !keep || axes != std::set<int>{1, 2}) return false;
  }
  *outer = *reduce = *inner = 1;
  for (int dd = 0; dd < rank; ++dd) {
    if (dd < *axes.begin()) *outer *= in.shape[dd];
    else if (dd > *axes.rbegin()) *inner *= in.shape[dd];
    else *reduce *= in.shape[dd];
  }
  return *reduce > 0 && out.num_elements() == static_cast<size_t>(*outer * *inner);
}

// TFLite_Detection_PostProcess in the form the host kernel implements
inline bool DetectionSupported(const TflModel& m, const TflOperator& op, CpuDetectionParams* p) {
  if (op.builtin != kTflCustom || op.custom_code != "TFLite_Detection_PostProcess") return false;
  if (op.inputs.size() != 3 || op.outputs.size() != 4) return false;
  for (int t : op.inputs)
    if (t < 0) return false;
  const TflTensor& be = m.tensors[op.inputs[0]];
  const TflTensor& cs = m.tensors[op.inputs[1]];
  const TflTensor& an = m.tensors[op.inputs[2]];
  if (be.type != DataType::kFloat32 || cs.type != DataType::kFloat32 || an.type != DataType::kFloat32 ||
      !an.is_const())
    return false;
  FlexMap f;
  if (!f.Parse(op.custom_options, op.custom_options_size)) return false;
  if (f.Number("use_regular_nms", 0) != 0 || f.Number("max_classes_per_detection", 1) != 1) return false;
  const int n = an.shape.empty() ? 0 : an.shape[0];
  if (n <= 0 || be.num_elements() != static_cast<size_t>(n) * 4 || cs.num_elements() % n) return false;
  CpuDetectionParams d{};
  d.num_boxes = n;
  d.num_classes = static_cast<int>(f.Number("num_classes", 0));
  d.num_classes_with_background = static_cast<int>(cs.num_elements() / n);
  d.max_detections = static_cast<int>(f.Number("max_detections", 0));
  // options are read with AsFloat (float), detection_postprocess.cc Init()
  d.score_threshold = static_cast<float>(f.Number("nms_score_threshold", 0));
  d.iou_threshold = static_cast<float>(f.Number("nms_iou_threshold", 0));
  d.scale_y = static_cast<float>(f.Number("y_scale", 0));
  d.scale_x = static_cast<float>(f.Number("x_scale", 0));
  d.scale_h = static_cast<float>(f.Number("h_scale", 0));
  d.scale_w = static_cast<float>(f.Number("w_scale", 0));
  if (d.num_classes <= 0 || d.num_classes > d.num_classes_with_background || d.max_detections <= 0) return false;
  for (int k = 0; k < 4; ++k)
    if (m.tensors[op.outputs[k]].type != DataType::kFloat32) return false;
  if (m.tensors[op.outputs[0]].num_elements() != static_cast<size_t>(d.max_detections) * 4) return false;
  if (p) *p = d;
  return true;
}

}  // namespace ex
}  // namespace hip
}  // namespace band
