// float32 kernels for fp16-weight TFLite models (post-training float16
// quantization: fp16 constants behind DEQUANTIZE, float32 compute; the host
// folds the DEQUANTIZEs).  Semantics of TFLite 2.9.2 reference_ops float
// Conv / DepthwiseConv / FullyConnected / Add / Sub / Mul / AveragePool /
// MaxPool / Logistic / Softmax; results agree with the reference within a
// tolerance (the reduction order differs), not bit-exactly.
//
// Batch-1 float layers are small: these kernels aim at one memory round
// trip per operand and coalesced weight loads, not MFMA.
#include "common.hpp"

namespace bh {

__device__ __forceinline__ float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }

// CONV_2D as an implicit GEMM on VALU: an item = one output pixel x 4
// output channels (items of one pixel are consecutive, so their float4
// weight loads from [K][out_c] coalesce and their input loads broadcast).
// A workgroup holds 256 / ks items and splits the reduction over ks slices
// of the filter taps (ks chosen on the host so deep, narrow layers still
// fill the chip); slices meet in LDS.
__global__ __launch_bounds__(256) void conv_f32_kernel(bh_conv_f32_params p, FastDiv groups, FastDiv ow,
                                                       FastDiv oh, long total, int ks) {
  __shared__ float4 part[256];
  const int iw = 256 / ks;  // items per workgroup
  const int item_in_wg = threadIdx.x % iw;
  const int slice = threadIdx.x / iw;
  const long i = (long)blockIdx.x * iw + item_in_wg;
  const bool live = i < total;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t pix = 0;
  int c0 = 0;
  if (live) {
    pix = groups.div((uint32_t)i);
    c0 = 4 * (int)((uint32_t)i - pix * groups.d);
    const uint32_t t = ow.div(pix);
    const int ox = (int)(pix - t * p.out_w);
    const uint32_t n = oh.div(t);
    const int oy = (int)(t - n * p.out_h);
    const int K = p.k_h * p.k_w * p.in_c;
    const int per = (K + ks - 1) / ks;
    const int k0 = slice * per, k1 = min(K, k0 + per);
    const bool vec = (p.out_c % 4) == 0;
    const int nc = min(4, p.out_c - c0);
    // walk k = (fy * k_w + fx) * in_c + ci over this slice
    int ci = k0 % p.in_c;
    int tap = k0 / p.in_c;
    int fy = tap / p.k_w, fx = tap - (tap / p.k_w) * p.k_w;
    for (int k = k0; k < k1;) {
      const int y = oy * p.stride_h - p.pad_h + fy * p.dil_h;
      const int x = ox * p.stride_w - p.pad_w + fx * p.dil_w;
      const int run = min(k1 - k, p.in_c - ci);  // channels left in this tap
      if (y >= 0 && y < p.in_h && x >= 0 && x < p.in_w) {
        const float* src = p.input + (((long)n * p.in_h + y) * p.in_w + x) * p.in_c + ci;
        const float* w = p.weights + (long)k * p.out_c + c0;
        if (vec) {
#pragma unroll 4
          for (int j = 0; j < run; ++j) {
            const float xv = src[j];
            const float4 wv = *(const float4*)(w + (long)j * p.out_c);
            acc.x = fmaf(xv, wv.x, acc.x);
            acc.y = fmaf(xv, wv.y, acc.y);
            acc.z = fmaf(xv, wv.z, acc.z);
            acc.w = fmaf(xv, wv.w, acc.w);
          }
        } else {
          for (int j = 0; j < run; ++j) {
            const float xv = src[j];
            const float* wr = w + (long)j * p.out_c;
            acc.x = fmaf(xv, wr[0], acc.x);
            if (nc > 1) acc.y = fmaf(xv, wr[1], acc.y);
            if (nc > 2) acc.z = fmaf(xv, wr[2], acc.z);
            if (nc > 3) acc.w = fmaf(xv, wr[3], acc.w);
          }
        }
      }
      k += run;
      ci = 0;
      if (++fx == p.k_w) {
        fx = 0;
        ++fy;
      }
    }
  }
  if (ks > 1) {
    part[threadIdx.x] = acc;
    __syncthreads();
    if (slice != 0) return;
    for (int s2 = 1; s2 < ks; ++s2) {
      const float4 o = part[s2 * iw + item_in_wg];
      acc.x += o.x;
      acc.y += o.y;
      acc.z += o.z;
      acc.w += o.w;
    }
  }
  if (!live) return;
  const int nc = min(4, p.out_c - c0);
  const float r[4] = {acc.x, acc.y, acc.z, acc.w};
  float* out = p.output + (long)pix * p.out_c + c0;
  for (int c = 0; c < nc; ++c) out[c] = clampf(r[c] + (p.bias ? p.bias[c0 + c] : 0.f), p.act_min, p.act_max);
}

// DEPTHWISE_CONV_2D: one thread = one output pixel x 4 channels
__global__ __launch_bounds__(256) void dwconv_f32_kernel(bh_conv_f32_params p, FastDiv groups, FastDiv ow,
                                                         FastDiv oh, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const uint32_t pix = groups.div((uint32_t)i);
  const int c0 = 4 * (int)((uint32_t)i - pix * groups.d);
  const uint32_t t = ow.div(pix);
  const int ox = (int)(pix - t * p.out_w);
  const uint32_t n = oh.div(t);
  const int oy = (int)(t - n * p.out_h);
  const int nc = min(4, p.out_c - c0);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int fy = 0; fy < p.k_h; ++fy) {
    const int y = oy * p.stride_h - p.pad_h + fy * p.dil_h;
    if (y < 0 || y >= p.in_h) continue;
    for (int fx = 0; fx < p.k_w; ++fx) {
      const int x = ox * p.stride_w - p.pad_w + fx * p.dil_w;
      if (x < 0 || x >= p.in_w) continue;
      const float* src = p.input + (((long)n * p.in_h + y) * p.in_w + x) * p.in_c;
      const float* w = p.weights + (long)(fy * p.k_w + fx) * p.out_c + c0;
      for (int c = 0; c < nc; ++c) acc[c] = fmaf(src[(c0 + c) / p.depth_multiplier], w[c], acc[c]);
    }
  }
  float* out = p.output + (long)pix * p.out_c + c0;
  for (int c = 0; c < nc; ++c) out[c] = clampf(acc[c] + (p.bias ? p.bias[c0 + c] : 0.f), p.act_min, p.act_max);
}

// FULLY_CONNECTED: one wave per (row, unit), lanes stride the depth
__global__ __launch_bounds__(256) void fc_f32_kernel(bh_fc_f32_params p, long total) {
  const long wv = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wv >= total) return;
  const long r = wv / p.units;
  const int u = (int)(wv - r * p.units);
  const float* x = p.input + r * p.depth;
  const float* w = p.weights + (long)u * p.depth;
  float acc = 0.f;
  for (int k = lane; k < p.depth; k += 64) acc = fmaf(x[k], w[k], acc);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) p.output[wv] = clampf(acc + (p.bias ? p.bias[u] : 0.f), p.act_min, p.act_max);
}

__global__ __launch_bounds__(256) void eltwise_f32_kernel(bh_eltwise_f32_params p, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int* so = p.shape_o;
  const long i3 = i % so[3], t = i / so[3];
  const long i2 = t % so[2], t2 = t / so[2];
  const long i1 = t2 % so[1], i0 = t2 / so[1];
  const int* sa = p.shape_a;
  const int* sb = p.shape_b;
  const long ia = (((sa[0] == 1 ? 0 : i0) * sa[1] + (sa[1] == 1 ? 0 : i1)) * sa[2] + (sa[2] == 1 ? 0 : i2)) * sa[3] +
                  (sa[3] == 1 ? 0 : i3);
  const long ib = (((sb[0] == 1 ? 0 : i0) * sb[1] + (sb[1] == 1 ? 0 : i1)) * sb[2] + (sb[2] == 1 ? 0 : i2)) * sb[3] +
                  (sb[3] == 1 ? 0 : i3);
  const float a = p.a[ia], b = p.b[ib];
  const float v = p.kind == BH_ELTF_ADD ? a + b
                  : p.kind == BH_ELTF_SUB ? a - b
                  : p.kind == BH_ELTF_MUL ? a * b
                                          : (a - b) * (a - b);
  p.out[i] = clampf(v, p.act_min, p.act_max);
}

__global__ __launch_bounds__(256) void pool_f32_kernel(bh_pool_f32_params p, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % p.channels);
  const long pix = i / p.channels;
  const int ox = (int)(pix % p.out_w);
  const long t = pix / p.out_w;
  const int oy = (int)(t % p.out_h);
  const int n = (int)(t / p.out_h);
  const int y0 = oy * p.stride_h - p.pad_h, x0 = ox * p.stride_w - p.pad_w;
  const int fy0 = max(0, -y0), fy1 = min(p.f_h, p.in_h - y0);
  const int fx0 = max(0, -x0), fx1 = min(p.f_w, p.in_w - x0);
  float acc = p.kind == BH_POOL_AVG ? 0.f : -INFINITY;
  int cnt = 0;
  for (int fy = fy0; fy < fy1; ++fy)
    for (int fx = fx0; fx < fx1; ++fx) {
      const float v = p.input[(((long)n * p.in_h + y0 + fy) * p.in_w + x0 + fx) * p.channels + c];
      acc = p.kind == BH_POOL_AVG ? acc + v : fmaxf(acc, v);
      ++cnt;
    }
  if (p.kind == BH_POOL_AVG) acc = acc / (float)cnt;
  p.output[i] = clampf(acc, p.act_min, p.act_max);
}

__global__ __launch_bounds__(256) void unary_f32_kernel(int kind, const float* in, float* out, long n, float lo,
                                                        float hi) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = in[i];
  out[i] = kind == BH_UNARY_LOGISTIC ? 1.0f / (1.0f + expf(-x)) : kind == BH_UNARY_RSQRT ? 1.0f / sqrtf(x)
                                                                                      : clampf(x, lo, hi);
}

// one wave per row: max, sum of exp, normalise
__global__ __launch_bounds__(256) void softmax_f32_kernel(const float* in, float* out, long rows, int depth,
                                                          float beta) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* x = in + r * depth;
  float* y = out + r * depth;
  float mx = -INFINITY;
  for (int k = lane; k < depth; k += 64) mx = fmaxf(mx, x[k]);
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float sum = 0.f;
  for (int k = lane; k < depth; k += 64) sum += expf((x[k] - mx) * beta);
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  const float inv = 1.0f / sum;
  for (int k = lane; k < depth; k += 64) y[k] = expf((x[k] - mx) * beta) * inv;
}

inline unsigned blocks(long n, int per = 256) { return (unsigned)((n + per - 1) / per); }

}  // namespace bh

extern "C" int bh_conv2d_f32(const bh_conv_f32_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || !pp->weights || pp->out_c <= 0 || pp->in_c <= 0 || pp->stride_h <= 0 ||
      pp->stride_w <= 0 || (pp->depthwise && pp->out_c != pp->in_c * pp->depth_multiplier)) {
    bh_set_last_error("bh_conv2d_f32: invalid parameters");
    return BH_EINVAL;
  }
  const bh_conv_f32_params& p = *pp;
  const long pixels = (long)p.batch * p.out_h * p.out_w;
  const int groups = (p.out_c + 3) / 4;
  const long total = pixels * groups;
  if (total <= 0 || total > INT32_MAX) {
    bh_set_last_error("bh_conv2d_f32: size out of range");
    return BH_EINVAL;
  }
  bh::FastDiv dg((uint32_t)groups), dw((uint32_t)p.out_w), dh((uint32_t)p.out_h);
  if (p.depthwise) {
    BH_LAUNCH(bh::dwconv_f32_kernel, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, p, dg, dw, dh,
                       total);
  } else {
    // split the reduction until ~1024 workgroups or 16 taps-channels per slice
    const int K = p.k_h * p.k_w * p.in_c;
    int ks = 1;
    while (ks < 16 && (total * ks) / 256 < 1024 && K / (2 * ks) >= 16) ks *= 2;
    const long items_per_wg = 256 / ks;
    BH_LAUNCH(bh::conv_f32_kernel, dim3((unsigned)((total + items_per_wg - 1) / items_per_wg)), dim3(256),
                       0, (hipStream_t)s, p, dg, dw, dh, total, ks);
  }
  return bh_check_launch(p.depthwise ? "dwconv_f32_kernel" : "conv_f32_kernel");
}

extern "C" int bh_fc_f32(const bh_fc_f32_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || !pp->weights || pp->rows <= 0 || pp->depth <= 0 || pp->units <= 0) {
    bh_set_last_error("bh_fc_f32: invalid parameters");
    return BH_EINVAL;
  }
  const long total = (long)pp->rows * pp->units;
  BH_LAUNCH(bh::fc_f32_kernel, dim3(bh::blocks(total, 4)), dim3(256), 0, (hipStream_t)s, *pp, total);
  return bh_check_launch("fc_f32_kernel");
}

extern "C" int bh_eltwise_f32(const bh_eltwise_f32_params* pp, bh_stream_t s) {
  if (!pp || !pp->a || !pp->b || !pp->out || pp->kind < BH_ELTF_ADD || pp->kind > BH_ELTF_SQDIFF) {
    bh_set_last_error("bh_eltwise_f32: invalid parameters");
    return BH_EINVAL;
  }
  const int* so = pp->shape_o;
  const long n = (long)so[0] * so[1] * so[2] * so[3];
  if (n <= 0) return 0;
  BH_LAUNCH(bh::eltwise_f32_kernel, dim3(bh::blocks(n)), dim3(256), 0, (hipStream_t)s, *pp, n);
  return bh_check_launch("eltwise_f32_kernel");
}

extern "C" int bh_pool_f32(const bh_pool_f32_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || pp->channels <= 0 || pp->stride_h <= 0 || pp->stride_w <= 0) {
    bh_set_last_error("bh_pool_f32: invalid parameters");
    return BH_EINVAL;
  }
  const long total = (long)pp->batch * pp->out_h * pp->out_w * pp->channels;
  if (total <= 0) return 0;
  BH_LAUNCH(bh::pool_f32_kernel, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, *pp, total);
  return bh_check_launch("pool_f32_kernel");
}

extern "C" int bh_unary_f32(int kind, const float* in, float* out, long n, float lo, float hi, bh_stream_t s) {
  if (!in || !out || n < 0 || (kind != BH_UNARY_CLAMP && kind != BH_UNARY_LOGISTIC && kind != BH_UNARY_RSQRT)) {
    bh_set_last_error("bh_unary_f32: invalid parameters");
    return BH_EINVAL;
  }
  if (n == 0) return 0;
  BH_LAUNCH(bh::unary_f32_kernel, dim3(bh::blocks(n)), dim3(256), 0, (hipStream_t)s, kind, in, out, n, lo,
                     hi);
  return bh_check_launch("unary_f32_kernel");
}

extern "C" int bh_softmax_f32(const float* in, float* out, long rows, int depth, float beta, bh_stream_t s) {
  if (!in || !out || rows < 0 || depth <= 0) {
    bh_set_last_error("bh_softmax_f32: invalid parameters");
    return BH_EINVAL;
  }
  if (rows == 0) return 0;
  BH_LAUNCH(bh::softmax_f32_kernel, dim3(bh::blocks(rows, 4)), dim3(256), 0, (hipStream_t)s, in, out, rows,
                     depth, beta);
  return bh_check_launch("softmax_f32_kernel");
}
