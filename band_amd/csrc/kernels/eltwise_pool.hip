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

// output-shape divisors for the broadcast index math (FastDiv, host-built)
struct BcastDivs {
  FastDiv d3, d2, d1;
};

__global__ __launch_bounds__(256) void eltwise_bcast_kernel(bh_eltwise_params p, int n, BcastDivs dv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int t = dv.d3.div(i);
  const int i3 = i - t * (int)dv.d3.d;
  int t2 = dv.d2.div(t);
  const int i2 = t - t2 * (int)dv.d2.d;
  const int i0 = dv.d1.div(t2);
  const int i1 = t2 - i0 * (int)dv.d1.d;
  const int* sa = p.shape_a;
  const int* sb = p.shape_b;
  const long ia = (((long)(sa[0] == 1 ? 0 : i0) * sa[1] + (sa[1] == 1 ? 0 : i1)) * sa[2] +
                   (sa[2] == 1 ? 0 : i2)) * sa[3] + (sa[3] == 1 ? 0 : i3);
  const long ib = (((long)(sb[0] == 1 ? 0 : i0) * sb[1] + (sb[1] == 1 ? 0 : i1)) * sb[2] +
                   (sb[2] == 1 ? 0 : i2)) * sb[3] + (sb[3] == 1 ? 0 : i3);
  const bool sg = p.in_signed != 0;
  ((uint8_t*)p.out)[i] = (uint8_t)elt_op(p, ld8((const uint8_t*)p.a, ia, sg), ld8((const uint8_t*)p.b, ib, sg));
}

// Exact n / d for 0 <= n < 2^24, 0 < d < 2^24 with small quotients (pool
// window averages): float reciprocal estimate, then integer correction.
__device__ __forceinline__ int small_div(int n, int d) {
  int q = (int)((float)n * __frcp_rn((float)d));
  int r = n - q * d;
  q += (r >= d) - (r < 0);
  r = n - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

struct PoolDivs {
  FastDiv groups, out_w, out_h;
};

// one thread per (output pixel, 4 channels) when C % 4 == 0, else per channel
template <int VEC>
__global__ __launch_bounds__(256) void pool_kernel(bh_pool_params p, int total, PoolDivs dv) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int pix = dv.groups.div(idx);
  const int c0 = (idx - pix * (int)dv.groups.d) * VEC;
  const int t = dv.out_w.div(pix);
  const int ox = pix - t * p.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
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
  // flattened window, 8 taps' loads in flight before they are consumed
  const int wx = fx1 - fx0;
  const int cnt_total = (fy1 - fy0) * wx;
  int cnt = cnt_total > 0 ? cnt_total : 0;
  int fy = fy0, fx = fx0;  // window walk, row-major
  for (int t0 = 0; t0 < cnt_total; t0 += 8) {
    uint32_t w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      w[u] = 0;
      if (t0 + u < cnt_total) {
        const int off = ((y0 + fy) * p.in_w + (x0 + fx)) * p.channels + c0;
        if constexpr (VEC == 4) w[u] = *(const uint32_t*)(in + off);
        else w[u] = in[off];
        if (++fx == fx1) {
          fx = fx0;
          ++fy;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (t0 + u >= cnt_total) break;
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const int32_t q = sg ? sbyte(w[u], v) : (int32_t)((w[u] >> (8 * v)) & 0xff);
        if (p.kind == BH_POOL_AVG) acc[v] += q;
        else acc[v] = q > acc[v] ? q : acc[v];
      }
    }
  }
  if (cnt == 0) cnt = 1;
  uint8_t* out = (uint8_t*)p.output + (((long)n * p.out_h + oy) * p.out_w + ox) * p.channels + c0;
  uint32_t packed = 0;
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    int32_t a = acc[v];
    if (p.kind == BH_POOL_AVG) a = a > 0 ? small_div(a + cnt / 2, cnt) : -small_div(cnt / 2 - a, cnt);
    a = clamp_i32(a, p.act_min, p.act_max);
    if constexpr (VEC == 4) packed |= ((uint32_t)a & 0xffu) << (8 * v);
    else out[v] = (uint8_t)a;
  }
  if constexpr (VEC == 4) *(uint32_t*)out = packed;
}

// Few output pixels, large window (MobileNet's 7x7 global average pool):
// one workgroup per (output pixel, 64 channel quads); each wave takes every
// 4th tap of the clipped window with up to 16 loads in flight, then the 4
// partial sums / maxima meet in LDS - one memory round trip instead of one
// per 8 taps.
// NW waves per workgroup: 16 when the window holds more taps than 4 waves
// take in one round of 16 loads each (DeepLab's 14x14 image pooling: 196
// taps, 4 rounds on 4 waves)
template <int NW>
__global__ __launch_bounds__(NW * 64) void pool_wide_kernel(bh_pool_params p, PoolDivs dv) {
  __shared__ int32_t part[NW - 1][64][4];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int pix = blockIdx.x;
  const int c0 = (blockIdx.y * 64 + lane) * 4;
  const bool active = c0 < p.channels;
  const int t = dv.out_w.div(pix);
  const int ox = pix - t * p.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
  const int y0 = oy * p.stride_h - p.pad_h;
  const int x0 = ox * p.stride_w - p.pad_w;
  const int fy0 = max(0, -y0), fy1 = min(p.f_h, p.in_h - y0);
  const int fx0 = max(0, -x0), fx1 = min(p.f_w, p.in_w - x0);
  const int wx = max(fx1 - fx0, 0);
  const int cnt_total = max(fy1 - fy0, 0) * wx;
  const uint8_t* in = (const uint8_t*)p.input + (long)n * p.in_h * p.in_w * p.channels;
  const bool sg = p.in_signed != 0;
  const bool avg = p.kind == BH_POOL_AVG;
  const int32_t init = avg ? 0 : (sg ? -128 : 0);
  int32_t acc[4] = {init, init, init, init};
  for (int t0 = wave; t0 < cnt_total; t0 += NW * 16) {
    uint32_t w[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int tt = t0 + NW * u;
      w[u] = 0;
      if (active && tt < cnt_total) {
        const int ry = small_div(tt, wx);
        const int fy = fy0 + ry, fx = fx0 + (tt - ry * wx);
        w[u] = *(const uint32_t*)(in + ((y0 + fy) * p.in_w + (x0 + fx)) * p.channels + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (t0 + NW * u >= cnt_total) break;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int32_t q = sg ? sbyte(w[u], v) : (int32_t)((w[u] >> (8 * v)) & 0xff);
        acc[v] = avg ? acc[v] + q : max(acc[v], q);
      }
    }
  }
  if (wave > 0) {
#pragma unroll
    for (int v = 0; v < 4; ++v) part[wave - 1][lane][v] = acc[v];
  }
  __syncthreads();
  if (wave > 0 || !active) return;
#pragma unroll
  for (int z = 0; z < NW - 1; ++z)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[v] = avg ? acc[v] + part[z][lane][v] : max(acc[v], part[z][lane][v]);
  const int cnt = cnt_total > 0 ? cnt_total : 1;
  uint32_t packed = 0;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    int32_t a = acc[v];
    if (avg) a = a > 0 ? small_div(a + cnt / 2, cnt) : -small_div(cnt / 2 - a, cnt);
    a = clamp_i32(a, p.act_min, p.act_max);
    packed |= ((uint32_t)a & 0xffu) << (8 * v);
  }
  *(uint32_t*)((uint8_t*)p.output + (((long)n * p.out_h + oy) * p.out_w + ox) * p.channels + c0) = packed;
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
  if (n >= INT32_MAX) {
    bh_set_last_error("bh_eltwise_i8: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const bool aligned = ((uintptr_t)p.a % 4 == 0) && ((uintptr_t)p.b % 4 == 0) && ((uintptr_t)p.out % 4 == 0);
  if (same && n % 4 == 0 && aligned) {
    const long n4 = n / 4;
    BH_LAUNCH(bh::eltwise_flat4_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, p, n4);
  } else {
    bh::BcastDivs dv;
    dv.d3 = bh::FastDiv(p.shape_o[3]);
    dv.d2 = bh::FastDiv(p.shape_o[2]);
    dv.d1 = bh::FastDiv(p.shape_o[1]);
    BH_LAUNCH(bh::eltwise_bcast_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, (int)n, dv);
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
  if (pixels * p.channels >= INT32_MAX || (long)p.batch * p.in_h * p.in_w * p.channels >= INT32_MAX) {
    bh_set_last_error("bh_pool_i8: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  bh::PoolDivs dv;
  dv.out_w = bh::FastDiv(p.out_w);
  dv.out_h = bh::FastDiv(p.out_h);
  if (p.channels % 4 == 0 && pixels * (p.channels / 4) <= 65536 && p.f_h * p.f_w >= 16 && pixels <= 65535) {
    dv.groups = bh::FastDiv(p.channels / 4);
    const dim3 grid((unsigned)pixels, (unsigned)((p.channels / 4 + 63) / 64));
    if (p.f_h * p.f_w > 4 * 16)
      BH_LAUNCH(bh::pool_wide_kernel<16>, grid, dim3(1024), 0, s, p, dv);
    else
      BH_LAUNCH(bh::pool_wide_kernel<4>, grid, dim3(256), 0, s, p, dv);
  } else if (p.channels % 4 == 0) {
    const int total = (int)(pixels * (p.channels / 4));
    dv.groups = bh::FastDiv(p.channels / 4);
    BH_LAUNCH(bh::pool_kernel<4>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total, dv);
  } else {
    const int total = (int)(pixels * p.channels);
    dv.groups = bh::FastDiv(p.channels);
    BH_LAUNCH(bh::pool_kernel<1>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total, dv);
  }
  return bh_check_launch("pool_kernel");
}
