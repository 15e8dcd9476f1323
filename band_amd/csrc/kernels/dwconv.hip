// DEPTHWISE_CONV_2D for gfx950.
//
// Stands in for TFLite 2.9.2 reference_integer_ops::DepthwiseConvPerChannel
// (int8) and reference_ops::DepthwiseConv (uint8, kAwayFromZero rounding ==
// MultiplyByQuantizedMultiplier) on Band's hot path
// (band/backend/tfl/model_executor.cc:249-255).  No cross-channel reduction,
// so it is VALU + memory work, never MFMA: one thread owns 4 consecutive
// channels of one output pixel (a dword of NHWC), loads each in-bounds tap as
// one dword and the matching dword of the [kh][kw][C] filter, and accumulates
// (x' - zp_in) * (w' - zp_w) exactly in int32.  Taps outside the image are
// skipped, as TFLite does.
#include "common.hpp"

namespace bh {

// VEC = 4: dm == 1 and C % 4 == 0 (every MobileNet-family layer).
template <int VEC>
__global__ __launch_bounds__(256) void dwconv_kernel(bh_dwconv_params p, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int groups = p.out_c / VEC;
  const int cg = (int)(idx % groups);
  long t = idx / groups;
  const int ox = (int)(t % p.out_w);
  t /= p.out_w;
  const int oy = (int)(t % p.out_h);
  const int n = (int)(t / p.out_h);
  const int c0 = cg * VEC;
  const uint8_t* in = (const uint8_t*)p.input;
  const uint8_t* wt = (const uint8_t*)p.weights;
  const uint32_t xorw = splat_byte(p.in_xor);

  int32_t acc[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) acc[v] = 0;

  const int y0 = oy * p.stride_h - p.pad_h;
  const int x0 = ox * p.stride_w - p.pad_w;
  const long img = (long)n * p.in_h * p.in_w * p.in_c;
  for (int fy = 0; fy < p.k_h; ++fy) {
    const int y = y0 + fy * p.dil_h;
    if (y < 0 || y >= p.in_h) continue;
    for (int fx = 0; fx < p.k_w; ++fx) {
      const int x = x0 + fx * p.dil_w;
      if (x < 0 || x >= p.in_w) continue;
      const long wo = ((long)fy * p.k_w + fx) * p.out_c + c0;
      if constexpr (VEC == 4) {
        const uint32_t xv = *(const uint32_t*)(in + img + ((long)y * p.in_w + x) * p.in_c + c0) ^ xorw;
        const uint32_t wv = *(const uint32_t*)(wt + wo);
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[v] += (sbyte(xv, v) - p.in_zp) * (sbyte(wv, v) - p.w_zp);
      } else {
        const int ic = c0 / p.depth_multiplier;
        const int32_t xv = (int32_t)(int8_t)(in[img + ((long)y * p.in_w + x) * p.in_c + ic] ^ (uint8_t)p.in_xor);
        const int32_t wv = (int32_t)(int8_t)wt[wo];
        acc[0] += (xv - p.in_zp) * (wv - p.w_zp);
      }
    }
  }

  uint8_t* out = (uint8_t*)p.output + (((long)n * p.out_h + oy) * p.out_w + ox) * p.out_c + c0;
  uint32_t packed = 0;
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    const int c = c0 + v;
    int32_t r = acc[v] + p.bias[c];
    r = requant(r, p.mult[c], p.shift[c]) + p.out_zp;
    r = clamp_i32(r, p.act_min, p.act_max);
    if constexpr (VEC == 4) packed |= ((uint32_t)r & 0xffu) << (8 * v);
    else out[v] = (uint8_t)r;
  }
  if constexpr (VEC == 4) *(uint32_t*)out = packed;
}

}  // namespace bh

extern "C" int bh_dwconv2d_i8(const bh_dwconv_params* pp, bh_stream_t stream) {
  if (!pp) return BH_EINVAL;
  const bh_dwconv_params& p = *pp;
  if (p.batch <= 0 || p.out_h <= 0 || p.out_w <= 0 || p.out_c <= 0 || p.depth_multiplier <= 0 ||
      p.out_c != p.in_c * p.depth_multiplier || !p.input || !p.output || !p.weights || !p.bias ||
      !p.mult || !p.shift || p.stride_h <= 0 || p.stride_w <= 0) {
    bh_set_last_error("bh_dwconv2d_i8: invalid parameters");
    return BH_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const long pixels = (long)p.batch * p.out_h * p.out_w;
  if (p.depth_multiplier == 1 && p.out_c % 4 == 0) {
    const long total = pixels * (p.out_c / 4);
    hipLaunchKernelGGL(bh::dwconv_kernel<4>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total);
  } else {
    const long total = pixels * p.out_c;
    hipLaunchKernelGGL(bh::dwconv_kernel<1>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total);
  }
  return bh_check_launch("dwconv_kernel");
}
