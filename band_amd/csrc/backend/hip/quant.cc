#include "backend/hip/quant.h"

#include <algorithm>
#include <cmath>

namespace band {
namespace hip {

void QuantizeMultiplier(double m, int32_t* q, int* shift) {
  if (m == 0.0) {
    *q = 0;
    *shift = 0;
    return;
  }
  int e = 0;
  const double frac = std::frexp(m, &e);
  int64_t fixed = static_cast<int64_t>(std::round(frac * static_cast<double>(1ll << 31)));
  if (fixed == (1ll << 31)) {
    fixed /= 2;
    ++e;
  }
  if (e < -31) {
    e = 0;
    fixed = 0;
  }
  *q = static_cast<int32_t>(fixed);
  *shift = e;
}

void ActivationRangeQuantized(int act, float scale, int32_t zp, bool is_int8, int32_t* lo, int32_t* hi) {
  const int32_t qmin = is_int8 ? -128 : 0;
  const int32_t qmax = is_int8 ? 127 : 255;
  auto quantize = [&](float f) { return zp + static_cast<int32_t>(std::round(f / scale)); };
  switch (act) {
    case 1:  // RELU
      *lo = std::max(qmin, quantize(0.0f));
      *hi = qmax;
      break;
    case 2:  // RELU_N1_TO_1
      *lo = std::max(qmin, quantize(-1.0f));
      *hi = std::min(qmax, quantize(1.0f));
      break;
    case 3:  // RELU6
      *lo = std::max(qmin, quantize(0.0f));
      *hi = std::min(qmax, quantize(6.0f));
      break;
    default:
      *lo = qmin;
      *hi = qmax;
  }
}

void ConvMultipliers(float in_scale, const std::vector<float>& w_scales, int channels, float out_scale,
                     bool legacy_uint8, std::vector<int32_t>* mult, std::vector<int32_t>* shift) {
  mult->assign(channels, 0);
  shift->assign(channels, 0);
  if (legacy_uint8) {
    const float product = in_scale * w_scales[0];  // float * float, as TFLite
    const double real = static_cast<double>(product) / static_cast<double>(out_scale);
    int32_t q;
    int e;
    QuantizeMultiplier(real, &q, &e);
    std::fill(mult->begin(), mult->end(), q);
    std::fill(shift->begin(), shift->end(), e);
    return;
  }
  for (int c = 0; c < channels; ++c) {
    const float ws = w_scales.size() > 1 ? w_scales[c] : w_scales[0];
    const double eff = static_cast<double>(in_scale) * static_cast<double>(ws) / static_cast<double>(out_scale);
    int32_t q;
    int e;
    QuantizeMultiplier(eff, &q, &e);
    (*mult)[c] = q;
    (*shift)[c] = e;
  }
}

void FullyConnectedMultiplier(float in_scale, float w_scale, float out_scale, int32_t* mult, int32_t* shift) {
  const float product = in_scale * w_scale;
  const double real = static_cast<double>(product) / static_cast<double>(out_scale);
  int e;
  QuantizeMultiplier(real, mult, &e);
  *shift = e;
}

AddParams AddSubParams(float s1, float s2, float so, bool is_sub) {
  AddParams p;
  p.left_shift = 20;
  const double twice_max = static_cast<double>(2 * std::max(s1, s2));
  const double r1 = s1 / twice_max;
  const double r2 = s2 / twice_max;
  const double ro = twice_max / static_cast<double>(static_cast<float>(1 << p.left_shift) * so);
  int e;
  QuantizeMultiplier(r1, &p.m1, &e);
  p.s1 = e;
  QuantizeMultiplier(r2, &p.m2, &e);
  p.s2 = e;
  QuantizeMultiplier(ro, &p.mo, &e);
  p.so = e;
  if (is_sub) p.m2 = -p.m2;
  return p;
}

void MulMultiplier(float s1, float s2, float so, int32_t* mult, int32_t* shift) {
  const float real = s1 * s2 / so;  // float arithmetic, as mul.cc
  int e;
  QuantizeMultiplier(static_cast<double>(real), mult, &e);
  *shift = e;
}

int ComputeOutSize(bool same, int in, int filter, int stride, int dilation) {
  const int eff = (filter - 1) * dilation + 1;
  return same ? (in + stride - 1) / stride : (in + stride - eff) / stride;
}

int ComputePadding(int stride, int dilation, int in, int filter, int out) {
  const int eff = (filter - 1) * dilation + 1;
  const int p = ((out - 1) * stride + eff - in) / 2;
  return p > 0 ? p : 0;
}

}  // namespace hip
}  // namespace band
