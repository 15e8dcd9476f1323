// DEPTHWISE_CONV_2D for gfx950.
//
// Stands in for TFLite 2.9.2 reference_integer_ops::DepthwiseConvPerChannel
// (int8) and reference_ops::DepthwiseConv (uint8, kAwayFromZero rounding ==
// MultiplyByQuantizedMultiplier) on Band's hot path
// (band/backend/tfl/model_executor.cc:249-255).  No cross-channel reduction,
// so it is VALU + memory work, never MFMA.  A thread owns CV consecutive
// channels of one output pixel (4/8/16 -> dword/dwordx2/dwordx4 accesses in
// NHWC), the 3x3 taps are fully unrolled with every in-bounds tap load
// issued before the arithmetic, and (x' - zp_in) * (w' - zp_w) accumulates
// exactly in int32.  Taps outside the image are skipped, as TFLite does.
#include "common.hpp"

namespace bh {

template <int CV>
struct Vec;
template <>
struct Vec<4> {
  static __device__ __forceinline__ void ld(const uint8_t* p, uint32_t* w) { w[0] = *(const uint32_t*)p; }
  static __device__ __forceinline__ void st(uint8_t* p, const uint32_t* w) { *(uint32_t*)p = w[0]; }
};
template <>
struct Vec<8> {
  static __device__ __forceinline__ void ld(const uint8_t* p, uint32_t* w) {
    v2i v = *(const v2i*)p;
    w[0] = v.x; w[1] = v.y;
  }
  static __device__ __forceinline__ void st(uint8_t* p, const uint32_t* w) { *(v2i*)p = (v2i){(int)w[0], (int)w[1]}; }
};
template <>
struct Vec<16> {
  static __device__ __forceinline__ void ld(const uint8_t* p, uint32_t* w) {
    v4i v = *(const v4i*)p;
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  }
  static __device__ __forceinline__ void st(uint8_t* p, const uint32_t* w) {
    *(v4i*)p = (v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
  }
};

// dm == 1, C % CV == 0, 3x3 filter (every MobileNet-family layer)
// thread index -> (pixel, channel group) divisors (FastDiv, host-built)
struct DwDivs {
  FastDiv groups, out_w, out_h, dm;
};

template <int CV>
__global__ __launch_bounds__(256) void dwconv3x3_kernel(bh_dwconv_params p, int total, DwDivs dv) {
  constexpr int NW = CV / 4;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int pix = dv.groups.div(idx);
  const int c0 = (idx - pix * (int)dv.groups.d) * CV;
  const int t = dv.out_w.div(pix);
  const int ox = pix - t * p.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
  const uint8_t* in = (const uint8_t*)p.input + (long)n * p.in_h * p.in_w * p.in_c + c0;
  const uint8_t* wt = (const uint8_t*)p.weights + c0;
  const uint32_t xorw = splat_byte(p.in_xor);
  const int y0 = oy * p.stride_h - p.pad_h;
  const int x0 = ox * p.stride_w - p.pad_w;

  uint32_t xv[9][NW], wv[9][NW];
  bool ok[9];
#pragma unroll
  for (int fy = 0; fy < 3; ++fy) {
#pragma unroll
    for (int fx = 0; fx < 3; ++fx) {
      const int tap = fy * 3 + fx;
      const int y = y0 + fy * p.dil_h;
      const int x = x0 + fx * p.dil_w;
      ok[tap] = y >= 0 && y < p.in_h && x >= 0 && x < p.in_w;
      Vec<CV>::ld(wt + (long)tap * p.out_c, wv[tap]);
      if (ok[tap]) Vec<CV>::ld(in + ((long)y * p.in_w + x) * p.in_c, xv[tap]);
    }
  }
  int32_t acc[CV];
#pragma unroll
  for (int v = 0; v < CV; ++v) acc[v] = 0;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    if (!ok[tap]) continue;
#pragma unroll
    for (int d = 0; d < NW; ++d) {
      const uint32_t xx = xv[tap][d] ^ xorw;
      const uint32_t ww = wv[tap][d];
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[d * 4 + b] += (sbyte(xx, b) - p.in_zp) * (sbyte(ww, b) - p.w_zp);
    }
  }
  uint32_t packed[NW];
#pragma unroll
  for (int d = 0; d < NW; ++d) {
    const v4i bb = *(const v4i*)(p.bias + c0 + 4 * d);
    const v4i mm = *(const v4i*)(p.mult + c0 + 4 * d);
    const v4i ss = *(const v4i*)(p.shift + c0 + 4 * d);
    uint32_t o = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      int32_t r = requant(acc[d * 4 + b] + bb[b], mm[b], ss[b]) + p.out_zp;
      r = clamp_i32(r, p.act_min, p.act_max);
      const uint32_t byte = p.out_table ? ((const uint8_t*)p.out_table)[(uint8_t)r] : ((uint32_t)r & 0xffu);
      o |= byte << (8 * b);
    }
    packed[d] = o;
  }
  Vec<CV>::st((uint8_t*)p.output + (((long)n * p.out_h + oy) * p.out_w + ox) * p.out_c + c0, packed);
}

// general filter size / depth multiplier: one output channel per thread
__global__ __launch_bounds__(256) void dwconv_generic_kernel(bh_dwconv_params p, int total, DwDivs dv) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int pix = dv.groups.div(idx);
  const int c = idx - pix * p.out_c;
  const int t = dv.out_w.div(pix);
  const int ox = pix - t * p.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
  const int ic = dv.dm.div(c);
  const uint8_t* in = (const uint8_t*)p.input + (long)n * p.in_h * p.in_w * p.in_c;
  const uint8_t* wt = (const uint8_t*)p.weights;
  int32_t acc = 0;
  const int y0 = oy * p.stride_h - p.pad_h;
  const int x0 = ox * p.stride_w - p.pad_w;
  for (int fy = 0; fy < p.k_h; ++fy) {
    const int y = y0 + fy * p.dil_h;
    if (y < 0 || y >= p.in_h) continue;
    for (int fx = 0; fx < p.k_w; ++fx) {
      const int x = x0 + fx * p.dil_w;
      if (x < 0 || x >= p.in_w) continue;
      const int32_t xv = (int32_t)(int8_t)(in[((long)y * p.in_w + x) * p.in_c + ic] ^ (uint8_t)p.in_xor);
      const int32_t wv = (int32_t)(int8_t)wt[((long)fy * p.k_w + fx) * p.out_c + c];
      acc += (xv - p.in_zp) * (wv - p.w_zp);
    }
  }
  int32_t r = requant(acc + p.bias[c], p.mult[c], p.shift[c]) + p.out_zp;
  const uint8_t byte = (uint8_t)clamp_i32(r, p.act_min, p.act_max);
  ((uint8_t*)p.output)[(((long)n * p.out_h + oy) * p.out_w + ox) * p.out_c + c] =
      p.out_table ? ((const uint8_t*)p.out_table)[byte] : byte;
}

static DwDivs dw_divs(const bh_dwconv_params& p, int groups) {
  DwDivs dv;
  dv.groups = FastDiv(groups);
  dv.out_w = FastDiv(p.out_w);
  dv.out_h = FastDiv(p.out_h);
  dv.dm = FastDiv(p.depth_multiplier);
  return dv;
}

template <int CV>
static void launch3x3(const bh_dwconv_params& p, long pixels, hipStream_t s) {
  const int total = (int)(pixels * (p.out_c / CV));
  hipLaunchKernelGGL(dwconv3x3_kernel<CV>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total,
                     dw_divs(p, p.out_c / CV));
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
  if (pixels * p.out_c >= INT32_MAX) {
    bh_set_last_error("bh_dwconv2d_i8: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  const bool fast = p.depth_multiplier == 1 && p.k_h == 3 && p.k_w == 3 && p.out_c % 4 == 0;
  if (fast) {
    // widest vector that still leaves enough threads to fill the chip
    if (p.out_c % 16 == 0 && pixels * (p.out_c / 16) >= 65536) bh::launch3x3<16>(p, pixels, s);
    else if (p.out_c % 8 == 0 && pixels * (p.out_c / 8) >= 32768) bh::launch3x3<8>(p, pixels, s);
    else bh::launch3x3<4>(p, pixels, s);
  } else {
    const int total = (int)(pixels * p.out_c);
    hipLaunchKernelGGL(bh::dwconv_generic_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total,
                       bh::dw_divs(p, p.out_c));
  }
  return bh_check_launch("dwconv_kernel");
}
