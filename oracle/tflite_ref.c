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
#ifdef _OPENMP
#include <omp.h>
#endif

/* threads of the conv / depthwise / fully-connected loops (test speed only;
 * every output element is computed by one thread, so results never depend
 * on it).  n <= 0 restores the OpenMP default. */
void tfl_set_num_threads(int n) {
#ifdef _OPENMP
  omp_set_num_threads(n > 0 ? n : omp_get_num_procs());
#else
  (void)n;
#endif
}

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
  /* output rows are independent: threads change the schedule, not a value */
#pragma omp parallel for collapse(2) schedule(static)
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
#pragma omp parallel for collapse(2) schedule(static)
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
#pragma omp parallel for collapse(2) schedule(static)
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

/* ======================================================================
 * Glue ops needed for whole-model residency.
 * ====================================================================== */

/* quantize.cc (int8/uint8 -> int8/uint8): effective scale
 * QuantizeMultiplier(double(in_scale) / double(out_scale)), then
 * reference_ops::Requantize: MBQM(x - in_zp) + out_zp, clamped to the output
 * type (its same-scale int8<->uint8 XOR fast path gives identical bytes). */
void tfl_requantize(const uint8_t* in, int in_signed, long n, int32_t in_zp, int32_t mult, int shift,
                    int out_signed, int32_t out_zp, uint8_t* out) {
  int32_t lo = out_signed ? -128 : 0, hi = out_signed ? 127 : 255;
  for (long i = 0; i < n; ++i) out[i] = (uint8_t)clampi(tfl_mbqm(ld(in, i, in_signed) - in_zp, mult, shift) + out_zp, lo, hi);
}

/* reference_ops::AffineQuantize (float -> int8/uint8):
 * (int32)TfLiteRound(val / scale) + zp, clamped; float division, roundf. */
void tfl_quantize_f32(const float* in, long n, float scale, int32_t zp, int out_signed, uint8_t* out) {
  int32_t lo = out_signed ? -128 : 0, hi = out_signed ? 127 : 255;
  for (long i = 0; i < n; ++i) out[i] = (uint8_t)clampi((int32_t)roundf(in[i] / scale) + zp, lo, hi);
}

/* reference_ops::Dequantize: float(double(scale) * (val - zp)) */
void tfl_dequantize(const uint8_t* in, int in_signed, long n, float scale, int32_t zp, float* out) {
  for (long i = 0; i < n; ++i) out[i] = (float)((double)scale * (double)(ld(in, i, in_signed) - zp));
}

/* activations.cc ReluPrepare + QuantizedReluX + reference_ops::ReluX:
 * multiplier = QuantizeMultiplier(in_scale / out_scale) (a float quotient),
 * bounds out_zp + roundf(act / out_scale) clipped to the type; act_max_inf
 * selects the open upper bound (RELU). */
void tfl_relu_params(float in_scale, float out_scale, int32_t out_zp, int out_signed, float act_min,
                     float act_max, int act_max_inf, int32_t* mult, int32_t* shift, int32_t* qmin,
                     int32_t* qmax) {
  double real = (double)(in_scale / out_scale);
  int e;
  tfl_quantize_multiplier(real, mult, &e);
  *shift = e;
  int32_t tmin = out_signed ? -128 : 0, tmax = out_signed ? 127 : 255;
  *qmin = imax(tmin, out_zp + (int32_t)roundf(act_min / out_scale));
  *qmax = act_max_inf ? tmax : imin(tmax, out_zp + (int32_t)roundf(act_max / out_scale));
}
void tfl_relu_x(const uint8_t* in, int is_signed, long n, int32_t in_zp, int32_t out_zp, int32_t mult, int shift,
                int32_t qmin, int32_t qmax, uint8_t* out) {
  for (long i = 0; i < n; ++i)
    out[i] = (uint8_t)clampi(out_zp + tfl_mbqm(ld(in, i, is_signed) - in_zp, mult, shift), qmin, qmax);
}

/* activations.cc PopulateLookupTable<T> (LOGISTIC, 8-bit, generic-optimized
 * kernel): dequantize in float, 1/(1+expf(-x)), roundf(y / out_scale as a
 * product with the float inverse) + zp, clamp; table indexed by the byte. */
void tfl_logistic_table(float in_scale, int32_t in_zp, float out_scale, int32_t out_zp, int is_signed,
                        uint8_t* table) {
  const float inverse_scale = 1.0f / out_scale;
  int32_t minval = is_signed ? -128 : 0, maxval = is_signed ? 127 : 255;
  for (int32_t val = minval; val <= maxval; ++val) {
    const float dequantized = in_scale * (float)(val - in_zp);
    const float transformed = 1.0f / (1.0f + expf(-dequantized));
    const float rescaled = roundf(transformed * inverse_scale);
    const int32_t quantized = (int32_t)(rescaled + (float)out_zp);
    table[(uint8_t)val] = (uint8_t)clampi(quantized, minval, maxval);
  }
}
/* HARD_SWISH, 8-bit (TFLite 2.9.2 activations.cc HardSwishPrepare +
 * reference/hard_swish.h HardSwish<T>): int16 fixed point throughout.
 * Prepare: hires_input_scale = in_scale / 128, reluish_scale = 3 / 32768,
 * QuantizeMultiplier of hires/out and hires/reluish, each multiplier then
 * DownScaleInt32ToInt16Multiplier'd ((m + 2^15) >> 16, saturating). */
static int16_t hs_sat16(int64_t v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }
static int16_t hs_srdhm16(int16_t a, int16_t b) { /* gemmlowp SaturatingRoundingDoublingHighMul<int16> */
  if (a == -32768 && b == -32768) return 32767;
  int32_t ab = (int32_t)a * b;
  return (int16_t)((ab + (ab >= 0 ? 16384 : -16383)) / 32768);
}
static int16_t hs_sdhm16(int16_t a, int16_t b) { /* SaturatingDoublingHighMul: truncating */
  if (a == -32768 && b == -32768) return 32767;
  return (int16_t)(((int32_t)a * b) / 32768);
}
static int16_t hs_rdbypot16(int16_t x, int e) {
  int32_t mask = (1 << e) - 1, rem = x & mask, thr = (mask >> 1) + (x < 0);
  return (int16_t)((x >> e) + (rem > thr));
}
static int16_t hs_down16(int32_t m) { return m >= 2147483647 - 32768 ? 32767 : (int16_t)((m + 32768) >> 16); }

int tfl_hard_swish(const uint8_t* in, int is_signed, long n, float in_scale, int32_t in_zp, float out_scale,
                   int32_t out_zp, uint8_t* out) {
  const float hires = (1.0f / 128.0f) * in_scale;
  int32_t om32, rm32;
  int oe, re;
  tfl_quantize_multiplier((double)(hires / out_scale), &om32, &oe);
  tfl_quantize_multiplier((double)(hires / (3.0f / 32768.0f)), &rm32, &re);
  if (oe > 0) return -1; /* TF_LITE_ENSURE(output_multiplier_exponent <= 0) */
  const int16_t om = hs_down16(om32), rm = hs_down16(rm32);
  const int lo = is_signed ? -128 : 0, hi = is_signed ? 127 : 255;
  for (long i = 0; i < n; ++i) {
    const int16_t v = (int16_t)((int16_t)(ld(in, i, is_signed) - in_zp) * 128);
    const int16_t on_out = hs_srdhm16(v, om);
    int16_t r = v;
    if (re > 0) r = hs_sat16((int64_t)r << (re - 1));
    r = hs_srdhm16(r, rm);
    if (re > 0) r = hs_sat16((int64_t)r * 2);
    else if (re < 0) r = hs_rdbypot16(r, -re);
    r = (int16_t)(((int32_t)r + 32768) >> 1);
    int16_t y = hs_rdbypot16(hs_sdhm16(r, on_out), -oe);
    y = (int16_t)(y + out_zp);
    out[i] = (uint8_t)clampi(y, lo, hi);
  }
  return 0;
}

void tfl_lookup(const uint8_t* in, long n, const uint8_t* table, uint8_t* out) {
  for (long i = 0; i < n; ++i) out[i] = table[in[i]];
}

/* optimized_ops::PopulateSoftmaxLookupTable + optimized_ops::Softmax
 * (int8/uint8 in and out, generic-optimized kernel):
 *   table[255 - v] = expf(-in_scale * beta * v), v = 0..255
 *   per row: max, sum_exp = sum table[255 - max + x] (in order),
 *   inv = 1 / (sum_exp * out_scale), q = round(table[..] * inv) + out_zp
 *   (uint8 output on x86: (int32)(p + 0.5f)), clamped. */
void tfl_softmax(const uint8_t* in, int is_signed, long rows, int depth, float in_scale, float beta,
                 float out_scale, int32_t out_zp, uint8_t* out) {
  float table[256];
  const float scale = -in_scale * beta;
  for (int32_t val = 0; val <= 255; ++val) table[255 - val] = expf(scale * (float)val);
  int32_t lo = is_signed ? -128 : 0, hi = is_signed ? 127 : 255;
  for (long r = 0; r < rows; ++r) {
    const uint8_t* x = in + r * depth;
    uint8_t* y = out + r * depth;
    int32_t max_val = is_signed ? -128 : 0;
    for (int j = 0; j < depth; ++j) max_val = imax(max_val, ld(x, j, is_signed));
    float sum_exp = 0.0f;
    const float* t = &table[255 - max_val];
    for (int j = 0; j < depth; ++j) sum_exp += t[ld(x, j, is_signed)];
    const float inv_sum_exp = 1.0f / (sum_exp * out_scale);
    for (int j = 0; j < depth; ++j) {
      const float p = t[ld(x, j, is_signed)] * inv_sum_exp;
      const int32_t q = is_signed ? (int32_t)roundf(p) + out_zp : (int32_t)(p + 0.5f) + out_zp;
      y[j] = (uint8_t)clampi(q, lo, hi);
    }
  }
}

/* concatenation.cc: int8 = reference_ops::Concatenation (all inputs share
 * the output's scale / zero point, checked in Prepare: a byte copy); uint8 =
 * reference_ops::ConcatenationWithScaling:
 *   same params -> copy, else (int32)round(x * s + b) + out_zp clamped to
 *   [0,255], s = in_scale * (1/out_scale), b = -in_zp * s (float). */
void tfl_concat(int n_in, const uint8_t* const* ins, const int* axis_sizes, long outer, long inner,
                const float* in_scales, const int32_t* in_zps, float out_scale, int32_t out_zp, int is_signed,
                uint8_t* out) {
  long out_axis = 0;
  for (int k = 0; k < n_in; ++k) out_axis += axis_sizes[k];
  const float inverse_output_scale = 1.0f / out_scale;
  long off = 0;
  for (int k = 0; k < n_in; ++k) {
    const long cp = (long)axis_sizes[k] * inner;
    const int same = is_signed || (in_zps[k] == out_zp && in_scales[k] == out_scale);
    const float s = in_scales[k] * inverse_output_scale;
    const float b = -(float)in_zps[k] * s;
    for (long o = 0; o < outer; ++o) {
      const uint8_t* src = ins[k] + o * cp;
      uint8_t* dst = out + o * out_axis * inner + off;
      if (same) {
        memcpy(dst, src, (size_t)cp);
      } else {
        for (long j = 0; j < cp; ++j) dst[j] = (uint8_t)clampi((int32_t)roundf((float)src[j] * s + b) + out_zp, 0, 255);
      }
    }
    off += cp;
  }
}

/* reference_ops::Pad (4-D, NHWC): pads[2*d], pads[2*d+1] = before / after;
 * quantized pad value = output zero point (PAD) or the constant (PADV2). */
void tfl_pad(const uint8_t* in, const int* in_shape, const int* pads, uint8_t value, uint8_t* out) {
  int os[4];
  for (int d = 0; d < 4; ++d) os[d] = in_shape[d] + pads[2 * d] + pads[2 * d + 1];
  long idx = 0;
  for (int b = 0; b < os[0]; ++b)
    for (int y = 0; y < os[1]; ++y)
      for (int x = 0; x < os[2]; ++x)
        for (int c = 0; c < os[3]; ++c, ++idx) {
          int ib = b - pads[0], iy = y - pads[2], ix = x - pads[4], ic = c - pads[6];
          int inside = ib >= 0 && ib < in_shape[0] && iy >= 0 && iy < in_shape[1] && ix >= 0 &&
                       ix < in_shape[2] && ic >= 0 && ic < in_shape[3];
          out[idx] = inside ? in[(((long)ib * in_shape[1] + iy) * in_shape[2] + ix) * in_shape[3] + ic] : value;
        }
}

/* reference_ops::ResizeNearestNeighbor index map (GetNearestNeighbor) */
int tfl_nearest_index(int v, int in_size, int out_size, int align_corners, int half_pixel_centers) {
  const float scale = (align_corners && out_size > 1) ? (float)(in_size - 1) / (float)(out_size - 1)
                                                      : (float)in_size / (float)out_size;
  const float offset = half_pixel_centers ? 0.5f : 0.0f;
  int32_t o = align_corners ? (int32_t)roundf(((float)v + offset) * scale) : (int32_t)floorf(((float)v + offset) * scale);
  o = imin(o, in_size - 1);
  if (half_pixel_centers) o = imax(0, o);
  return o;
}
void tfl_resize_nearest(const uint8_t* in, int b, int ih, int iw, int c, int oh, int ow, int align_corners,
                        int half_pixel_centers, uint8_t* out) {
  for (int n = 0; n < b; ++n)
    for (int y = 0; y < oh; ++y) {
      const int sy = tfl_nearest_index(y, ih, oh, align_corners, half_pixel_centers);
      for (int x = 0; x < ow; ++x) {
        const int sx = tfl_nearest_index(x, iw, ow, align_corners, half_pixel_centers);
        memcpy(out + (((long)n * oh + y) * ow + x) * c, in + (((long)n * ih + sy) * iw + sx) * c, (size_t)c);
      }
    }
}

/* reference_ops::ResizeBilinearInteger (int8): 10-bit fixed-point scales
 * and ComputeInterpolationValuesInteger; the four-tap sum in int64, rounded
 * half away from zero at 2^20. */
static void interp_int(int32_t value, int32_t scale_10, int half_pixel_centers, int32_t input_size,
                       int32_t* scaled, int32_t* lo, int32_t* hi) {
  *scaled = half_pixel_centers ? value * scale_10 + scale_10 / 2 - (1 << 9) : value * scale_10;
  *lo = imax(*scaled / (1 << 10), 0);
  *hi = imin((*scaled + (1 << 10) - 1) / (1 << 10), input_size - 1);
}
void tfl_resize_bilinear_i8(const int8_t* in, int b, int ih, int iw, int c, int oh, int ow, int align_corners,
                            int half_pixel_centers, int8_t* out) {
  int32_t hs = ((1 << 10) * ih + oh / 2) / oh;
  int32_t ws = ((1 << 10) * iw + ow / 2) / ow;
  if (align_corners && oh > 1) hs = ((1 << 10) * (ih - 1) + (oh - 1) / 2) / (oh - 1);
  if (align_corners && ow > 1) ws = ((1 << 10) * (iw - 1) + (ow - 1) / 2) / (ow - 1);
  const int32_t one = 1 << 10;
  for (int n = 0; n < b; ++n)
    for (int y = 0; y < oh; ++y) {
      int32_t iy, y0, y1;
      interp_int(y, hs, half_pixel_centers, ih, &iy, &y0, &y1);
      for (int x = 0; x < ow; ++x) {
        int32_t ix, x0, x1;
        interp_int(x, ws, half_pixel_centers, iw, &ix, &x0, &x1);
        for (int ch = 0; ch < c; ++ch) {
#define AT(yy, xx) ((int64_t)in[(((long)n * ih + (yy)) * iw + (xx)) * c + ch])
          const int64_t ll = AT(y0, x0) * ((one - (iy - one * y0)) * (one - (ix - one * x0)));
          const int64_t lu = AT(y1, x0) * ((iy - one * y0) * (one - (ix - one * x0)));
          const int64_t rl = AT(y0, x1) * ((one - (iy - one * y0)) * (ix - one * x0));
          const int64_t ru = AT(y1, x1) * ((iy - one * y0) * (ix - one * x0));
#undef AT
          const int64_t s = ll + lu + rl + ru;
          const int64_t rnd = s > 0 ? (1 << 19) : -(1 << 19);
          out[(((long)n * oh + y) * ow + x) * c + ch] = (int8_t)((s + rnd) / (1 << 20));
        }
      }
    }
}

/* optimized_ops::ResizeBilinear for uint8 (TFLite 2.9.2; TFLite is a
 * third-party dependency of Band, not vendored under /root/reference):
 * ResizeBilinearGenericSmallChannel<uint8> with float scales and
 * reference_ops::ComputeInterpolationValues; four float weights, the
 * weighted sum left to right, + 0.5f, truncated.  Parity unpinned: no
 * reference fixture covers this op. */
static void interp_float(int value, float scale, int half_pixel_centers, int input_size, float* scaled, int* lo,
                         int* hi) {
  *scaled = half_pixel_centers ? ((float)value + 0.5f) * scale - 0.5f : (float)value * scale;
  *lo = imax((int)floorf(*scaled), 0);
  *hi = imin((int)ceilf(*scaled), input_size - 1);
}
void tfl_resize_bilinear_u8(const uint8_t* in, int b, int ih, int iw, int c, int oh, int ow, int align_corners,
                            int half_pixel_centers, uint8_t* out) {
  const float hs = (align_corners && oh > 1) ? (float)(ih - 1) / (float)(oh - 1) : (float)ih / (float)oh;
  const float ws = (align_corners && ow > 1) ? (float)(iw - 1) / (float)(ow - 1) : (float)iw / (float)ow;
  for (int n = 0; n < b; ++n)
    for (int y = 0; y < oh; ++y) {
      float iy;
      int y0, y1;
      interp_float(y, hs, half_pixel_centers, ih, &iy, &y0, &y1);
      for (int x = 0; x < ow; ++x) {
        float ix;
        int x0, x1;
        interp_float(x, ws, half_pixel_centers, iw, &ix, &x0, &x1);
        const float w00 = (1 - (iy - y0)) * (1 - (ix - x0)), w01 = (1 - (iy - y0)) * (ix - x0);
        const float w10 = (iy - y0) * (1 - (ix - x0)), w11 = (iy - y0) * (ix - x0);
        for (int ch = 0; ch < c; ++ch) {
#define AT(yy, xx) in[(((long)n * ih + (yy)) * iw + (xx)) * c + ch]
          const float v = AT(y0, x0) * w00 + AT(y0, x1) * w01 + AT(y1, x0) * w10 + AT(y1, x1) * w11 + 0.5f;
#undef AT
          out[(((long)n * oh + y) * ow + x) * c + ch] = (uint8_t)(int)v;
        }
      }
    }
}

/* optimized_ops::PopulateSoftmaxLookupTable alone (the table tfl_softmax uses) */
void tfl_softmax_table(float in_scale, float beta, float* table) {
  const float scale = -in_scale * beta;
  for (int32_t val = 0; val <= 255; ++val) table[255 - val] = expf(scale * (float)val);
}

/* reference_integer_ops::TransposeConv (int8 per-channel), TFLite 2.9.2:
 * zeroed int32 scratch, scatter of (x + input_offset) * w over every
 * (input pixel, filter tap, out channel) that lands inside the output, then
 * bias + MultiplyByQuantizedMultiplier per channel + zp, clamped to int8.
 * Filter OHWI [oc][kh][kw][ic]; padding from padding.h computed with the
 * output as the conv input (transpose_conv.cc). */
void tfl_transpose_conv_i8(const int8_t* in, int b, int ih, int iw, int ic, const int8_t* w, int oc, int kh,
                           int kw, const int32_t* bias, int8_t* out, int oh, int ow, int sh, int sw, int ph,
                           int pw, int32_t input_offset, int32_t out_zp, const int32_t* mult, const int32_t* shift) {
  long n = (long)b * oh * ow * oc;
  int32_t* acc = (int32_t*)calloc((size_t)n, sizeof(int32_t));
  for (int bb = 0; bb < b; ++bb)
    for (int y = 0; y < ih; ++y)
      for (int x = 0; x < iw; ++x)
        for (int ci = 0; ci < ic; ++ci) {
          const int oy0 = y * sh - ph, ox0 = x * sw - pw;
          const int32_t v = (int32_t)in[(((long)bb * ih + y) * iw + x) * ic + ci] + input_offset;
          for (int fy = 0; fy < kh; ++fy)
            for (int fx = 0; fx < kw; ++fx)
              for (int co = 0; co < oc; ++co) {
                const int oy = oy0 + fy, ox = ox0 + fx;
                if (oy >= 0 && oy < oh && ox >= 0 && ox < ow)
                  acc[(((long)bb * oh + oy) * ow + ox) * oc + co] +=
                      v * (int32_t)w[(((long)co * kh + fy) * kw + fx) * ic + ci];
              }
        }
  for (long i = 0; i < n; ++i) {
    const int co = (int)(i % oc);
    int32_t a = acc[i] + (bias ? bias[co] : 0);
    a = tfl_mbqm(a, mult[co], shift[co]) + out_zp;
    out[i] = (int8_t)clampi(a, -128, 127);
  }
  free(acc);
}
