/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the TensorFlow Lite 2.9.2 integer reference kernels
 * that `tflite::Interpreter::Invoke` dispatches for Band's per-subgraph hot
 * path (`band/backend/tfl/model_executor.cc:249-255`).  TFLite itself is a
 * third-party dependency fetched by Bazel (`org_tensorflow` =
 * mrsnu/tensorflow tag v2.9.2_thread_affinity, `WORKSPACE:12-16`) and is NOT
 * present under /root/reference, so the algorithms below are restated from
 * the published TFLite 2.9.2 sources named in each comment:
 *   kernels/internal/common.h              (MultiplyByQuantizedMultiplier …)
 *   kernels/internal/quantization_util.cc  (QuantizeMultiplier)
 *   kernels/kernel_util.cc                 (CalculateActivationRangeQuantized,
 *                                           PopulateConvolutionQuantizationParams)
 *   kernels/padding.h                      (ComputePadding / ComputeOutSize)
 *   kernels/internal/reference/integer_ops/{conv,depthwise_conv,
 *       fully_connected,add,mul,pooling}.h and reference/{conv,
 *       depthwiseconv_uint8,fully_connected,add,mul,pooling}.h (uint8)
 *
 * Pinning: the whole-model runner (oracle/runner.py) built on these kernels
 * reproduces the reference's own known-answer tests
 * (`band/test/backend/tfl_minimal_test.cc:379-457`: MobileNetV2-quant + cat.jpg
 * -> argmax 282; `:62-90`: add.tflite {1,3} -> {3,9}); see tests/test_oracle.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product never links it.
 *
 * Conventions: every activation / weight tensor is passed as raw bytes plus a
 * signedness flag (1 = int8, 0 = uint8); the arithmetic is identical for both
 * because TFLite's uint8 and int8 reference kernels share the formula
 * acc = sum (x + in_off) * (w + w_off) + bias, requantised per output channel.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define I32MIN (-2147483647 - 1)
#define I32MAX 2147483647

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

/* gemmlowp::SaturatingRoundingDoublingHighMul (fixedpoint.h) */
int32_t tfl_srdhm(int32_t a, int32_t b) {
  int overflow = (a == b) && (a == I32MIN);
  int64_t ab = (int64_t)a * (int64_t)b;
  int32_t nudge = ab >= 0 ? (1 << 30) : (1 - (1 << 30));
  int32_t hi = (int32_t)((ab + nudge) / (1ll << 31)); /* C division truncates */
  return overflow ? I32MAX : hi;
}

/* gemmlowp::RoundingDivideByPOT (fixedpoint.h) */
int32_t tfl_rdbypot(int32_t x, int exponent) {
  int32_t mask = (int32_t)((1ll << exponent) - 1);
  int32_t remainder = x & mask;
  int32_t threshold = (mask >> 1) + (x < 0 ? 1 : 0);
  return (x >> exponent) + (remainder > threshold ? 1 : 0);
}

/* common.h MultiplyByQuantizedMultiplier (no TFLITE_SINGLE_ROUNDING) */
int32_t tfl_mbqm(int32_t x, int32_t qm, int shift) {
  int left = shift > 0 ? shift : 0;
  int right = shift > 0 ? 0 : -shift;
  return tfl_rdbypot(tfl_srdhm((int32_t)((uint32_t)x << left), qm), right);
}

/* common.h MultiplyByQuantizedMultiplierSmallerThanOneExp */
int32_t tfl_mbqm_lt1(int32_t x, int32_t qm, int left_shift) {
  return tfl_rdbypot(tfl_srdhm(x, qm), -left_shift);
}

/* quantization_util.cc QuantizeMultiplier (TfLiteRound = std::round) */
void tfl_quantize_multiplier(double m, int32_t* qm, int* shift) {
  if (m == 0.0) { *qm = 0; *shift = 0; return; }
  int e = 0;
  double q = frexp(m, &e);
  int64_t q_fixed = (int64_t)round(q * (double)(1ll << 31));
  if (q_fixed == (1ll << 31)) { q_fixed /= 2; ++e; }
  if (e < -31) { e = 0; q_fixed = 0; }
  *qm = (int32_t)q_fixed;
  *shift = e;
}

/* kernel_util.cc CalculateActivationRangeQuantized.
 * act: 0 NONE, 1 RELU, 2 RELU_N1_TO_1, 3 RELU6 (schema ActivationFunctionType) */
void tfl_act_range_quantized(int act, float scale, int32_t zp, int is_signed,
                             int32_t* amin, int32_t* amax) {
  int32_t qmin = is_signed ? -128 : 0, qmax = is_signed ? 127 : 255;
#define QUANT(f) (zp + (int32_t)roundf((float)(f) / scale))
  if (act == 1) { *amin = imax(qmin, QUANT(0.0f)); *amax = qmax; }
  else if (act == 3) { *amin = imax(qmin, QUANT(0.0f)); *amax = imin(qmax, QUANT(6.0f)); }
  else if (act == 2) { *amin = imax(qmin, QUANT(-1.0f)); *amax = imin(qmax, QUANT(1.0f)); }
  else { *amin = qmin; *amax = qmax; }
#undef QUANT
}

/* kernel_util.cc PopulateConvolutionQuantizationParams.
 * per_channel path: double(in)*double(w[c])/double(out), QuantizeMultiplier.
 * uint8 legacy path (GetQuantizedConvolutionMultipler): float(in*w) then
 * double / double(out); output_shift passed to the kernel = exponent. */
void tfl_conv_multipliers(float in_scale, const float* w_scales, int n_scales,
                          int n_channels, float out_scale, int legacy_u8,
                          int32_t* mult, int32_t* shift) {
  if (legacy_u8) {
    float prod = in_scale * w_scales[0];
    double real = (double)prod / (double)out_scale;
    int32_t q; int e;
    tfl_quantize_multiplier(real, &q, &e);
    for (int c = 0; c < n_channels; ++c) { mult[c] = q; shift[c] = e; }
    return;
  }
  for (int c = 0; c < n_channels; ++c) {
    float s = n_scales > 1 ? w_scales[c] : w_scales[0];
    double eff = (double)in_scale * (double)s / (double)out_scale;
    int32_t q; int e;
    tfl_quantize_multiplier(eff, &q, &e);
    mult[c] = q; shift[c] = e;
  }
}

/* padding.h */
int tfl_out_size(int same, int in, int filter, int stride, int dilation) {
  int eff = (filter - 1) * dilation + 1;
  return same ? (in + stride - 1) / stride : (in + stride - eff) / stride;
}
int tfl_padding(int stride, int dilation, int in, int filter, int out) {
  int eff = (filter - 1) * dilation + 1;
  int p = ((out - 1) * stride + eff - in) / 2;
  return p > 0 ? p : 0;
}

static inline int32_t ld(const uint8_t* p, long i, int is_signed) {
  return is_signed ? (int32_t)(int8_t)p[i] : (int32_t)p[i];
}
static inline int32_t clampi(int32_t v, int32_t lo, int32_t hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

/* reference_integer_ops::ConvPerChannel / reference_ops::Conv (uint8).
 * NHWC input [b,ih,iw,ic], OHWI filter [oc,kh,kw,ic], out [b,oh,ow,oc]. */
void tfl_conv2d(const uint8_t* in, int in_signed, int b, int ih, int iw, int ic,
                const uint8_t* w, int w_signed, int oc, int kh, int kw,
                const int32_t* bias, uint8_t* out, int oh, int ow,
                int stride_h, int stride_w, int dil_h, int dil_w,
                int pad_h, int pad_w, int32_t in_off, int32_t w_off,
                int32_t out_off, const int32_t* mult, const int32_t* shift,
                int32_t amin, int32_t amax) {
  for (int n = 0; n < b; ++n)
    for (int oy = 0; oy < oh; ++oy)
      for (int ox = 0; ox < ow; ++ox) {
        int y0 = oy * stride_h - pad_h, x0 = ox * stride_w - pad_w;
        for (int c = 0; c < oc; ++c) {
          int32_t acc = 0;
          for (int fy = 0; fy < kh; ++fy) {
            int y = y0 + dil_h * fy;
            if (y < 0 || y >= ih) continue;
            for (int fx = 0; fx < kw; ++fx) {
              int x = x0 + dil_w * fx;
              if (x < 0 || x >= iw) continue;
              const long ib = (((long)n * ih + y) * iw + x) * ic;
              const long wb = (((long)c * kh + fy) * kw + fx) * ic;
              for (int k = 0; k < ic; ++k)
                acc += (ld(w, wb + k, w_signed) + w_off) * (ld(in, ib + k, in_signed) + in_off);
            }
          }
          if (bias) acc += bias[c];
          acc = tfl_mbqm(acc, mult[c], shift[c]);
          acc += out_off;
          out[(((long)n * oh + oy) * ow + ox) * oc + c] = (uint8_t)clampi(acc, amin, amax);
        }
      }
}

/* reference_integer_ops::DepthwiseConvPerChannel / reference_ops::DepthwiseConv
 * (uint8, DepthwiseConvOutputRounding::kAwayFromZero == MultiplyByQuantizedMultiplier).
 * filter [1,kh,kw,ic*dm]. */
void tfl_dwconv2d(const uint8_t* in, int in_signed, int b, int ih, int iw, int ic,
                  const uint8_t* w, int w_signed, int dm, int kh, int kw,
                  const int32_t* bias, uint8_t* out, int oh, int ow,
                  int stride_h, int stride_w, int dil_h, int dil_w,
                  int pad_h, int pad_w, int32_t in_off, int32_t w_off,
                  int32_t out_off, const int32_t* mult, const int32_t* shift,
                  int32_t amin, int32_t amax) {
  const int oc = ic * dm;
  for (int n = 0; n < b; ++n)
    for (int oy = 0; oy < oh; ++oy)
      for (int ox = 0; ox < ow; ++ox)
        for (int c = 0; c < ic; ++c)
          for (int m = 0; m < dm; ++m) {
            const int o = c * dm + m;
            int32_t acc = 0;
            for (int fy = 0; fy < kh; ++fy) {
              int y = oy * stride_h - pad_h + dil_h * fy;
              if (y < 0 || y >= ih) continue;
              for (int fx = 0; fx < kw; ++fx) {
                int x = ox * stride_w - pad_w + dil_w * fx;
                if (x < 0 || x >= iw) continue;
                int32_t iv = ld(in, (((long)n * ih + y) * iw + x) * ic + c, in_signed);
                int32_t wv = ld(w, ((long)fy * kw + fx) * oc + o, w_signed);
                acc += (wv + w_off) * (iv + in_off);
              }
            }
            if (bias) acc += bias[o];
            acc = tfl_mbqm(acc, mult[o], shift[o]);
            acc += out_off;
            out[(((long)n * oh + oy) * ow + ox) * oc + o] = (uint8_t)clampi(acc, amin, amax);
          }
}

/* reference_integer_ops::FullyConnected / reference_ops::FullyConnected (uint8).
 * in [rows, depth], w [units, depth]; per-channel arrays of length units. */
void tfl_fully_connected(const uint8_t* in, int in_signed, int rows, int depth,
                         const uint8_t* w, int w_signed, int units,
                         const int32_t* bias, uint8_t* out, int32_t in_off,
                         int32_t w_off, int32_t out_off, const int32_t* mult,
                         const int32_t* shift, int32_t amin, int32_t amax) {
  for (int r = 0; r < rows; ++r)
    for (int u = 0; u < units; ++u) {
      int32_t acc = 0;
      for (int d = 0; d < depth; ++d)
        acc += (ld(w, (long)u * depth + d, w_signed) + w_off) *
               (ld(in, (long)r * depth + d, in_signed) + in_off);
      if (bias) acc += bias[u];
      acc = tfl_mbqm(acc, mult[u], shift[u]);
      acc += out_off;
      out[(long)r * units + u] = (uint8_t)clampi(acc, amin, amax);
    }
}

/* 4-D broadcast index (NdArrayDesc / SubscriptToIndex semantics):
 * shapes are already extended to 4-D; a dim of 1 broadcasts. */
static inline long bidx(const int* s, int a, int b_, int c, int d) {
  return (((long)(s[0] == 1 ? 0 : a) * s[1] + (s[1] == 1 ? 0 : b_)) * s[2] +
          (s[2] == 1 ? 0 : c)) * s[3] + (s[3] == 1 ? 0 : d);
}

/* add.cc Prepare for uint8/int8 (left_shift = 20). Outputs the 7 params. */
void tfl_add_params(float s1, float s2, float so, int32_t* p /* m1,sh1,m2,sh2,mo,sho,left */) {
  const int left_shift = 20;
  const double twice_max = (double)(2 * (s1 > s2 ? s1 : s2));
  const double r1 = s1 / twice_max;
  const double r2 = s2 / twice_max;
  const double ro = twice_max / (double)((float)(1 << left_shift) * so);
  int e;
  tfl_quantize_multiplier(r1, &p[0], &e); p[1] = e;
  tfl_quantize_multiplier(r2, &p[2], &e); p[3] = e;
  tfl_quantize_multiplier(ro, &p[4], &e); p[5] = e;
  p[6] = left_shift;
}

/* reference_integer_ops::Add / reference_ops::Add (uint8) with 4-D broadcast.
 * sub != 0 gives quantized SUB the way sub.cc PrepareGeneralSubOp sets it up:
 * same params as ADD with input2_multiplier negated, then the ADD kernel. */
void tfl_add(const uint8_t* a, const int* sa, const uint8_t* b_, const int* sb,
             uint8_t* out, const int* so, int is_signed, int32_t a_off,
             int32_t b_off, int32_t o_off, const int32_t* p, int sub,
             int32_t amin, int32_t amax) {
  for (int i0 = 0; i0 < so[0]; ++i0)
    for (int i1 = 0; i1 < so[1]; ++i1)
      for (int i2 = 0; i2 < so[2]; ++i2)
        for (int i3 = 0; i3 < so[3]; ++i3) {
          int32_t x1 = a_off + ld(a, bidx(sa, i0, i1, i2, i3), is_signed);
          int32_t x2 = b_off + ld(b_, bidx(sb, i0, i1, i2, i3), is_signed);
          int32_t s1 = tfl_mbqm_lt1(x1 * (1 << p[6]), p[0], p[1]);
          int32_t s2 = tfl_mbqm_lt1(x2 * (1 << p[6]), sub ? -p[2] : p[2], p[3]);
          int32_t raw = s1 + s2;
          int32_t o = tfl_mbqm_lt1(raw, p[4], p[5]) + o_off;
          out[(((long)i0 * so[1] + i1) * so[2] + i2) * so[3] + i3] = (uint8_t)clampi(o, amin, amax);
        }
}

/* mul.cc Prepare: float product/quotient, then QuantizeMultiplier. */
void tfl_mul_params(float s1, float s2, float so, int32_t* mult, int32_t* shift) {
  float real_f = s1 * s2 / so;
  int e;
  tfl_quantize_multiplier((double)real_f, mult, &e);
  *shift = e;
}

/* reference_integer_ops::Mul / reference_ops::Mul (uint8) with broadcast. */
void tfl_mul(const uint8_t* a, const int* sa, const uint8_t* b_, const int* sb,
             uint8_t* out, const int* so, int is_signed, int32_t a_off,
             int32_t b_off, int32_t o_off, int32_t mult, int32_t shift,
             int32_t amin, int32_t amax) {
  for (int i0 = 0; i0 < so[0]; ++i0)
    for (int i1 = 0; i1 < so[1]; ++i1)
      for (int i2 = 0; i2 < so[2]; ++i2)
        for (int i3 = 0; i3 < so[3]; ++i3) {
          int32_t x1 = a_off + ld(a, bidx(sa, i0, i1, i2, i3), is_signed);
          int32_t x2 = b_off + ld(b_, bidx(sb, i0, i1, i2, i3), is_signed);
          int32_t o = o_off + tfl_mbqm(x1 * x2, mult, shift);
          out[(((long)i0 * so[1] + i1) * so[2] + i2) * so[3] + i3] = (uint8_t)clampi(o, amin, amax);
        }
}

/* reference_integer_ops::AveragePool / reference_ops::AveragePool (uint8). */
void tfl_avg_pool(const uint8_t* in, int is_signed, int b, int ih, int iw, int c,
                  uint8_t* out, int oh, int ow, int fh, int fw, int sh, int sw,
                  int ph, int pw, int32_t amin, int32_t amax) {
  for (int n = 0; n < b; ++n)
    for (int oy = 0; oy < oh; ++oy)
      for (int ox = 0; ox < ow; ++ox)
        for (int ch = 0; ch < c; ++ch) {
          const int y0 = oy * sh - ph, x0 = ox * sw - pw;
          const int fy0 = imax(0, -y0), fy1 = imin(fh, ih - y0);
          const int fx0 = imax(0, -x0), fx1 = imin(fw, iw - x0);
          int32_t acc = 0; int cnt = 0;
          for (int fy = fy0; fy < fy1; ++fy)
            for (int fx = fx0; fx < fx1; ++fx) {
              acc += ld(in, (((long)n * ih + y0 + fy) * iw + x0 + fx) * c + ch, is_signed);
              ++cnt;
            }
          if (cnt == 0) cnt = 1;
          acc = acc > 0 ? (acc + cnt / 2) / cnt : (acc - cnt / 2) / cnt;
          out[(((long)n * oh + oy) * ow + ox) * c + ch] = (uint8_t)clampi(acc, amin, amax);
        }
}

/* reference_integer_ops::MaxPool / reference_ops::MaxPool (uint8). */
void tfl_max_pool(const uint8_t* in, int is_signed, int b, int ih, int iw, int c,
                  uint8_t* out, int oh, int ow, int fh, int fw, int sh, int sw,
                  int ph, int pw, int32_t amin, int32_t amax) {
  for (int n = 0; n < b; ++n)
    for (int oy = 0; oy < oh; ++oy)
      for (int ox = 0; ox < ow; ++ox)
        for (int ch = 0; ch < c; ++ch) {
          const int y0 = oy * sh - ph, x0 = ox * sw - pw;
          const int fy0 = imax(0, -y0), fy1 = imin(fh, ih - y0);
          const int fx0 = imax(0, -x0), fx1 = imin(fw, iw - x0);
          int32_t mx = is_signed ? -128 : 0;
          for (int fy = fy0; fy < fy1; ++fy)
            for (int fx = fx0; fx < fx1; ++fx) {
              int32_t v = ld(in, (((long)n * ih + y0 + fy) * iw + x0 + fx) * c + ch, is_signed);
              if (v > mx) mx = v;
            }
          out[(((long)n * oh + oy) * ow + ox) * c + ch] = (uint8_t)clampi(mx, amin, amax);
        }
}

/* Float ADD (reference_ops::Add float path with activation clamp), used by
 * the add.tflite known-answer test. */
void tfl_add_f32(const float* a, const int* sa, const float* b_, const int* sb,
                 float* out, const int* so, float amin, float amax, int sub) {
  for (int i0 = 0; i0 < so[0]; ++i0)
    for (int i1 = 0; i1 < so[1]; ++i1)
      for (int i2 = 0; i2 < so[2]; ++i2)
        for (int i3 = 0; i3 < so[3]; ++i3) {
          float v = sub ? a[bidx(sa, i0, i1, i2, i3)] - b_[bidx(sb, i0, i1, i2, i3)]
                        : a[bidx(sa, i0, i1, i2, i3)] + b_[bidx(sb, i0, i1, i2, i3)];
          v = v < amin ? amin : (v > amax ? amax : v);
          out[(((long)i0 * so[1] + i1) * so[2] + i2) * so[3] + i3] = v;
        }
}
