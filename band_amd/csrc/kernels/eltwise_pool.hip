// ADD / SUB / MUL and AVERAGE_POOL_2D / MAX_POOL_2D for gfx950.
//
// Stand-ins for TFLite 2.9.2 reference_integer_ops::{Add,Mul,AveragePool,
// MaxPool} and their uint8 reference_ops twins on Band's hot path
// (band/backend/tfl/model_executor.cc:249-255).  All are HBM/L2-bound byte
// streams: the same-shape path moves 4 elements per lane with dword loads
// and stores; broadcasting shapes fall back to per-element 4-D indexing.
//
// ADD (add.cc, left_shift = 20):
//   s_i = MBQMSmallerThanOneExp((q_i + off_i) << 20, M_i, sh_i)
//   y   = MBQMSmallerThanOneExp(s_1 + s_2, M_o, sh_o) + zp_o
// SUB is ADD with input2's multiplier negated (sub.cc).  MUL (mul.cc):
//   y = MBQM((q_1 + off_1) * (q_2 + off_2), M, sh) + zp_o
#include "common.hpp"

namespace bh {

__device__ __forceinline__ int32_t ld8(const uint8_t* p, long i, bool sgn) {
  return sgn ? (int32_t)(int8_t)p[i] : (int32_t)p[i];
}

__device__ __forceinline__ int32_t elt_op(const bh_eltwise_params& p, int32_t qa, int32_t qb) {
  const int32_t xa = qa + p.a_off;
  const int32_t xb = qb + p.b_off;
  int32_t o;
  if (p.kind == BH_ELT_ADD) {
    const int32_t sa = requant_lt1(xa * (1 << p.left_shift), p.a_mult, p.a_shift);
    const int32_t sb = requant_lt1(xb * (1 << p.left_shift), p.b_mult, p.b_shift);
    o = requant_lt1(sa + sb, p.o_mult, p.o_shift) + p.o_off;
  } else {
    o = requant(xa * xb, p.o_mult, p.o_shift) + p.o_off;
  }
  return clamp_i32(o, p.act_min, p.act_max);
}

// same shape, 4 elements per lane (n % 4 == 0, pointers dword aligned)
__global__ __launch_bounds__(256) void eltwise_flat4_kernel(bh_eltwise_params p, long n4) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const uint32_t a = ((const uint32_t*)p.a)[i];
  const uint32_t b = ((const uint32_t*)p.b)[i];
  uint32_t o = 0;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int32_t qa = p.in_signed ? sbyte(a, v) : (int32_t)((a >> (8 * v)) & 0xff);
    const int32_t qb = p.in_signed ? sbyte(b, v) : (int32_t)((b >> (8 * v)) & 0xff);
    o |= ((uint32_t)elt_op(p, qa, qb) & 0xffu) << (8 * v);
  }
  ((uint32_t*)p.out)[i] = o;
}

__global__ __launch_bounds__(256) void eltwise_bcast_kernel(bh_eltwise_params p, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int* so = p.shape_o;
  long t = i;
  const int i3 = (int)(t % so[3]); t /= so[3];
  const int i2 = (int)(t % so[2]); t /= so[2];
  const int i1 = (int)(t % so[1]);
  const int i0 = (int)(t / so[1]);
  const int* sa = p.shape_a;
  const int* sb = p.shape_b;
  const long ia = (((long)(sa[0] == 1 ? 0 : i0) * sa[1] + (sa[1] == 1 ? 0 : i1)) * sa[2] +
                   (sa[2] == 1 ? 0 : i2)) * sa[3] + (sa[3] == 1 ? 0 : i3);
  const long ib = (((long)(sb[0] == 1 ? 0 : i0) * sb[1] + (sb[1] == 1 ? 0 : i1)) * sb[2] +
                   (sb[2] == 1 ? 0 : i2)) * sb[3] + (sb[3] == 1 ? 0 : i3);
  const bool sg = p.in_signed != 0;
  ((uint8_t*)p.out)[i] = (uint8_t)elt_op(p, ld8((const uint8_t*)p.a, ia, sg), ld8((const uint8_t*)p.b, ib, sg));
}

// one thread per (output pixel, 4 channels) when C % 4 == 0, else per channel
template <int VEC>
__global__ __launch_bounds__(256) void pool_kernel(bh_pool_params p, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int groups = p.channels / VEC;
  const int cg = (int)(idx % groups);
  long t = idx / groups;
  const int ox = (int)(t % p.out_w);
  t /= p.out_w;
  const int oy = (int)(t % p.out_h);
  const int n = (int)(t / p.out_h);
  const int c0 = cg * VEC;
  const int y0 = oy * p.stride_h - p.pad_h;
  const int x0 = ox * p.stride_w - p.pad_w;
  const int fy0 = max(0, -y0), fy1 = min(p.f_h, p.in_h - y0);
  const int fx0 = max(0, -x0), fx1 = min(p.f_w, p.in_w - x0);
  const uint8_t* in = (const uint8_t*)p.input + (long)n * p.in_h * p.in_w * p.channels;
  const bool sg = p.in_signed != 0;
  int32_t acc[VEC];
  const int32_t init = p.kind == BH_POOL_AVG ? 0 : (sg ? -128 : 0);
#pragma unroll
  for (int v = 0; v < VEC; ++v) acc[v] = init;
  int cnt = 0;
  for (int fy = fy0; fy < fy1; ++fy) {
    for (int fx = fx0; fx < fx1; ++fx) {
      const long off = ((long)(y0 + fy) * p.in_w + (x0 + fx)) * p.channels + c0;
      uint32_t w;
      if constexpr (VEC == 4) w = *(const uint32_t*)(in + off);
      else w = in[off];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const int32_t q = sg ? sbyte(w, v) : (int32_t)((w >> (8 * v)) & 0xff);
        if (p.kind == BH_POOL_AVG) acc[v] += q;
        else acc[v] = q > acc[v] ? q : acc[v];
      }
      ++cnt;
    }
  }
  if (cnt == 0) cnt = 1;
  uint8_t* out = (uint8_t*)p.output + (((long)n * p.out_h + oy) * p.out_w + ox) * p.channels + c0;
  uint32_t packed = 0;
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    int32_t a = acc[v];
    if (p.kind == BH_POOL_AVG) a = a > 0 ? (a + cnt / 2) / cnt : (a - cnt / 2) / cnt;
    a = clamp_i32(a, p.act_min, p.act_max);
    if constexpr (VEC == 4) packed |= ((uint32_t)a & 0xffu) << (8 * v);
    else out[v] = (uint8_t)a;
  }
  if constexpr (VEC == 4) *(uint32_t*)out = packed;
}

}  // namespace bh

extern "C" int bh_eltwise_i8(const bh_eltwise_params* pp, bh_stream_t stream) {
  if (!pp || !pp->a || !pp->b || !pp->out || (pp->kind != BH_ELT_ADD && pp->kind != BH_ELT_MUL)) {
    bh_set_last_error("bh_eltwise_i8: invalid parameters");
    return BH_EINVAL;
  }
  const bh_eltwise_params& p = *pp;
  long n = 1;
  bool same = true;
  for (int d = 0; d < 4; ++d) {
    if (p.shape_o[d] <= 0) { bh_set_last_error("bh_eltwise_i8: bad shape"); return BH_EINVAL; }
    n *= p.shape_o[d];
    same = same && p.shape_a[d] == p.shape_o[d] && p.shape_b[d] == p.shape_o[d];
  }
  hipStream_t s = (hipStream_t)stream;
  const bool aligned = ((uintptr_t)p.a % 4 == 0) && ((uintptr_t)p.b % 4 == 0) && ((uintptr_t)p.out % 4 == 0);
  if (same && n % 4 == 0 && aligned) {
    const long n4 = n / 4;
    hipLaunchKernelGGL(bh::eltwise_flat4_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, p, n4);
  } else {
    hipLaunchKernelGGL(bh::eltwise_bcast_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n);
  }
  return bh_check_launch("eltwise_kernel");
}

extern "C" int bh_pool_i8(const bh_pool_params* pp, bh_stream_t stream) {
  if (!pp || !pp->input || !pp->output || pp->batch <= 0 || pp->channels <= 0 || pp->out_h <= 0 ||
      pp->out_w <= 0 || pp->f_h <= 0 || pp->f_w <= 0 || pp->stride_h <= 0 || pp->stride_w <= 0) {
    bh_set_last_error("bh_pool_i8: invalid parameters");
    return BH_EINVAL;
  }
  const bh_pool_params& p = *pp;
  hipStream_t s = (hipStream_t)stream;
  const long pixels = (long)p.batch * p.out_h * p.out_w;
  if (p.channels % 4 == 0) {
    const long total = pixels * (p.channels / 4);
    hipLaunchKernelGGL(bh::pool_kernel<4>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total);
  } else {
    const long total = pixels * p.channels;
    hipLaunchKernelGGL(bh::pool_kernel<1>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total);
  }
  return bh_check_launch("pool_kernel");
}
