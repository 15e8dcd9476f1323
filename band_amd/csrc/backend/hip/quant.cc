#include "backend/hip/quant.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <limits>

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

namespace {
int32_t Srdhm(int32_t a, int32_t b) {
  const bool overflow = a == b && a == INT32_MIN;
  const int64_t ab = static_cast<int64_t>(a) * static_cast<int64_t>(b);
  const int32_t nudge = ab >= 0 ? (1 << 30) : (1 - (1 << 30));
  const int32_t hi = static_cast<int32_t>((ab + nudge) / (1ll << 31));
  return overflow ? INT32_MAX : hi;
}
int32_t Rdbypot(int32_t x, int e) {
  const int32_t mask = static_cast<int32_t>((1ll << e) - 1);
  const int32_t rem = x & mask;
  const int32_t thr = (mask >> 1) + (x < 0 ? 1 : 0);
  return (x >> e) + (rem > thr ? 1 : 0);
}
int32_t Clamp(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }
int32_t ByteValue(int b, bool is_signed) { return is_signed ? static_cast<int8_t>(b) : b; }
}  // namespace

int32_t MultiplyByQuantizedMultiplier(int32_t x, int32_t q, int shift) {
  const int left = shift > 0 ? shift : 0;
  const int right = shift > 0 ? 0 : -shift;
  return Rdbypot(Srdhm(static_cast<int32_t>(static_cast<uint32_t>(x) << left), q), right);
}

void RequantizeTable(bool in_signed, float in_scale, int32_t in_zp, bool out_signed, float out_scale,
                     int32_t out_zp, uint8_t table[256]) {
  int32_t q;
  int sh;
  QuantizeMultiplier(static_cast<double>(in_scale) / static_cast<double>(out_scale), &q, &sh);
  const int32_t lo = out_signed ? -128 : 0, hi = out_signed ? 127 : 255;
  for (int b = 0; b < 256; ++b)
    table[b] = static_cast<uint8_t>(
        Clamp(MultiplyByQuantizedMultiplier(ByteValue(b, in_signed) - in_zp, q, sh) + out_zp, lo, hi));
}

void ReluTable(bool is_signed, float in_scale, int32_t in_zp, float out_scale, int32_t out_zp, float act_min,
               float act_max, bool act_max_inf, uint8_t table[256]) {
  int32_t q;
  int sh;
  const double real = in_scale / out_scale;  // float quotient, as ReluPrepare
  QuantizeMultiplier(real, &q, &sh);
  const int32_t tmin = is_signed ? -128 : 0, tmax = is_signed ? 127 : 255;
  const int32_t qmin = std::max(tmin, out_zp + static_cast<int32_t>(std::roundf(act_min / out_scale)));
  const int32_t qmax =
      act_max_inf ? tmax : std::min(tmax, out_zp + static_cast<int32_t>(std::roundf(act_max / out_scale)));
  for (int b = 0; b < 256; ++b)
    table[b] = static_cast<uint8_t>(
        Clamp(out_zp + MultiplyByQuantizedMultiplier(ByteValue(b, is_signed) - in_zp, q, sh), qmin, qmax));
}

void LogisticTable(bool is_signed, float in_scale, int32_t in_zp, float out_scale, int32_t out_zp,
                   uint8_t table[256]) {
  const float inverse_scale = 1.0f / out_scale;
  const int32_t minval = is_signed ? -128 : 0, maxval = is_signed ? 127 : 255;
  for (int32_t val = minval; val <= maxval; ++val) {
    const float dequantized = in_scale * static_cast<float>(val - in_zp);
    const float transformed = 1.0f / (1.0f + std::exp(-dequantized));
    const float rescaled = std::round(transformed * inverse_scale);
    const int32_t quantized = static_cast<int32_t>(rescaled + static_cast<float>(out_zp));
    table[static_cast<uint8_t>(val)] = static_cast<uint8_t>(Clamp(quantized, minval, maxval));
  }
}

namespace {
// int16 fixed-point primitives of reference_ops::HardSwish (TFLite 2.9.2
// kernels/internal/reference/hard_swish.h and gemmlowp fixedpoint.h)
int16_t SatRoundDoublingHighMul16(int16_t a, int16_t b) {
  if (a == b && a == std::numeric_limits<int16_t>::min()) return std::numeric_limits<int16_t>::max();
  const int32_t ab = static_cast<int32_t>(a) * static_cast<int32_t>(b);
  const int32_t nudge = ab >= 0 ? (1 << 14) : (1 - (1 << 14));
  return static_cast<int16_t>((ab + nudge) / (1 << 15));
}
int16_t SatDoublingHighMul16(int16_t a, int16_t b) {  // no rounding nudge
  if (a == b && a == std::numeric_limits<int16_t>::min()) return std::numeric_limits<int16_t>::max();
  return static_cast<int16_t>((static_cast<int32_t>(a) * static_cast<int32_t>(b)) / (1 << 15));
}
int16_t SatLeftShift16(int16_t v, int amount) {
  const int64_t r = static_cast<int64_t>(v) * (int64_t{1} << amount);
  return static_cast<int16_t>(std::min<int64_t>(std::max<int64_t>(r, -32768), 32767));
}
int16_t RoundDivPot16(int16_t x, int e) {
  const int32_t mask = (1 << e) - 1;
  const int32_t rem = x & mask;
  const int32_t thr = (mask >> 1) + (x < 0 ? 1 : 0);
  return static_cast<int16_t>((x >> e) + (rem > thr ? 1 : 0));
}
// quantization_util.h DownScaleInt32ToInt16Multiplier
int16_t DownScaleMultiplier16(int32_t m) {
  if (m >= std::numeric_limits<int32_t>::max() - (1 << 15)) return std::numeric_limits<int16_t>::max();
  return static_cast<int16_t>((m + (1 << 15)) >> 16);
}
}  // namespace

bool HardSwishTable(bool is_signed, float in_scale, int32_t in_zp, float out_scale, int32_t out_zp,
                    uint8_t table[256]) {
  const float hires_input_scale = (1.0f / 128.0f) * in_scale;
  const float reluish_scale = 3.0f / 32768.0f;
  const float output_multiplier = hires_input_scale / out_scale;
  const float reluish_multiplier = hires_input_scale / reluish_scale;
  int32_t om = 0, rm = 0;
  int oexp = 0, rexp = 0;
  QuantizeMultiplier(output_multiplier, &om, &oexp);
  QuantizeMultiplier(reluish_multiplier, &rm, &rexp);
  if (oexp > 0) return false;  // TF_LITE_ENSURE(output_multiplier_exponent <= 0)
  const int16_t om16 = DownScaleMultiplier16(om), rm16 = DownScaleMultiplier16(rm);
  const int32_t minval = is_signed ? -128 : 0, maxval = is_signed ? 127 : 255;
  for (int32_t val = minval; val <= maxval; ++val) {
    const int16_t x = static_cast<int16_t>(val - in_zp);
    const int16_t hires = static_cast<int16_t>(x * (1 << 7));
    const int16_t pre_out = SatRoundDoublingHighMul16(hires, om16);
    int16_t reluish = hires;
    if (rexp > 0) reluish = SatLeftShift16(reluish, rexp - 1);
    reluish = SatRoundDoublingHighMul16(reluish, rm16);
    if (rexp > 0) reluish = SatLeftShift16(reluish, 1);
    if (rexp < 0) reluish = RoundDivPot16(reluish, -rexp);
    reluish = static_cast<int16_t>((static_cast<int32_t>(reluish) + (1 << 15)) >> 1);
    const int16_t pre = SatDoublingHighMul16(reluish, pre_out);
    int16_t y = RoundDivPot16(pre, -oexp);
    y = static_cast<int16_t>(y + out_zp);
    table[static_cast<uint8_t>(val)] = static_cast<uint8_t>(Clamp(static_cast<int32_t>(y), minval, maxval));
  }
  return true;
}

void DequantizeTable(bool is_signed, float scale, int32_t zp, float table[256]) {
  for (int b = 0; b < 256; ++b)
    table[b] = static_cast<float>(static_cast<double>(scale) * static_cast<double>(ByteValue(b, is_signed) - zp));
}

void ConcatRescaleTable(float in_scale, int32_t in_zp, float out_scale, int32_t out_zp, uint8_t table[256]) {
  const float inverse_output_scale = 1.f / out_scale;
  const float s = in_scale * inverse_output_scale;
  const float bias = -static_cast<float>(in_zp) * s;
  for (int b = 0; b < 256; ++b) {
    const int32_t v = static_cast<int32_t>(std::round(static_cast<float>(b) * s + bias)) + out_zp;
    table[b] = static_cast<uint8_t>(Clamp(v, 0, 255));
  }
}

void SoftmaxExpTable(float in_scale, float beta, float table[256]) {
  const float scale = -in_scale * beta;
  for (int32_t val = 0; val <= 255; ++val) table[255 - val] = std::exp(scale * static_cast<float>(val));
}

int NearestNeighborIndex(int v, int in_size, int out_size, bool align_corners, bool half_pixel_centers) {
  const float scale = (align_corners && out_size > 1)
                          ? static_cast<float>(in_size - 1) / static_cast<float>(out_size - 1)
                          : static_cast<float>(in_size) / static_cast<float>(out_size);
  const float offset = half_pixel_centers ? 0.5f : 0.0f;
  int32_t o = align_corners ? static_cast<int32_t>(std::round((static_cast<float>(v) + offset) * scale))
                            : static_cast<int32_t>(std::floor((static_cast<float>(v) + offset) * scale));
  o = std::min(o, in_size - 1);
  if (half_pixel_centers) o = std::max(0, o);
  return o;
}

void BilinearFloatTable(int in_size, int out_size, bool align_corners, bool half_pixel_centers,
                        std::vector<int32_t>* idx, std::vector<float>* frac) {
  float scale = static_cast<float>(in_size) / static_cast<float>(out_size);
  if (align_corners && out_size > 1) scale = static_cast<float>(in_size - 1) / static_cast<float>(out_size - 1);
  idx->assign(2 * static_cast<size_t>(out_size), 0);
  frac->assign(static_cast<size_t>(out_size), 0.f);
  for (int v = 0; v < out_size; ++v) {
    const float fv = static_cast<float>(v);
    const float scaled = half_pixel_centers ? (fv + 0.5f) * scale - 0.5f : fv * scale;
    const int32_t lo = std::max(static_cast<int32_t>(std::floor(scaled)), 0);
    const int32_t hi = std::min(static_cast<int32_t>(std::ceil(scaled)), in_size - 1);
    (*idx)[2 * v] = lo;
    (*idx)[2 * v + 1] = hi;
    (*frac)[v] = scaled - static_cast<float>(lo);
  }
}

void BilinearIntegerTable(int in_size, int out_size, bool align_corners, bool half_pixel_centers,
                          std::vector<int32_t>* tab) {
  int32_t scale_10 = ((1 << 10) * in_size + out_size / 2) / out_size;
  if (align_corners && out_size > 1) scale_10 = ((1 << 10) * (in_size - 1) + (out_size - 1) / 2) / (out_size - 1);
  tab->assign(3 * static_cast<size_t>(out_size), 0);
  for (int v = 0; v < out_size; ++v) {
    const int32_t scaled = half_pixel_centers ? v * scale_10 + scale_10 / 2 - (1 << 9) : v * scale_10;
    (*tab)[3 * v] = std::max(scaled / (1 << 10), 0);
    (*tab)[3 * v + 1] = std::min((scaled + (1 << 10) - 1) / (1 << 10), in_size - 1);
    (*tab)[3 * v + 2] = scaled;
  }
}

}  // namespace hip
}  // namespace band
