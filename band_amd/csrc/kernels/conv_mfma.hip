// CONV_2D for gfx950: implicit-im2col GEMM on the int8 matrix cores.
//
// Stands in for TFLite 2.9.2 reference_integer_ops::ConvPerChannel (int8,
// per-channel) and reference_ops::Conv (uint8, per-tensor), the kernels
// `Interpreter::Invoke` runs for CONV_2D on Band's hot path
// (band/backend/tfl/model_executor.cc:249-255).  Bit-exact with them:
//   acc[m][n] = sum_k x'[m][k] * w'[n][k] + bias_eff[n] - w_zp * sum_k x'[m][k]
//   y = clamp(MultiplyByQuantizedMultiplier(acc, M[n], shift[n]) + zp_out)
// where x'/w' are int8-domain operands (uint8 XOR 0x80), spatial padding is
// filled with the input zero point (so centred padding contributes exactly
// 0, like TFLite's skipped taps) and the K tail is zero-filled.
//
// GEMM view (NHWC / OHWI): M = batch*out_h*out_w pixels, N = out_c,
// K = k_h*k_w*in_c.  Both operands are K-contiguous, so each lane's MFMA
// fragment (16 consecutive k of one row) is a single 16-byte load for 1x1
// layers.  v_mfma_i32_16x16x64_i8: lane l supplies A[l&15][16*(l>>4)+j] and
// B[16*(l>>4)+j][l&15]; D lands as D[4*(l>>4)+r][l&15] (r = 0..3).
#include "common.hpp"

namespace bh {

struct RowInfo {
  long base;   // 1x1: byte offset of the input pixel; general: image base
  int y0, x0;  // general: top-left input coordinate of the window
  bool valid;
};

template <int VEC>
__device__ __forceinline__ void load_unit(const uint8_t* src, uint32_t* w, int u) {
  if constexpr (VEC == 16) {
    v4i v = *(const v4i*)src;
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else if constexpr (VEC == 8) {
    v2i v = *(const v2i*)src;
    w[2 * u] = v.x; w[2 * u + 1] = v.y;
  } else if constexpr (VEC == 4) {
    w[u] = *(const uint32_t*)src;
  } else {
    const int d = u >> 2, b = u & 3;
    w[d] = (w[d] & ~(0xffu << (8 * b))) | ((uint32_t)src[0] << (8 * b));
  }
}

template <int VEC>
__device__ __forceinline__ void fill_unit(uint32_t* w, int u, uint32_t pat) {
  if constexpr (VEC == 16) {
    w[0] = w[1] = w[2] = w[3] = pat;
  } else if constexpr (VEC == 8) {
    w[2 * u] = pat; w[2 * u + 1] = pat;
  } else if constexpr (VEC == 4) {
    w[u] = pat;
  } else {
    const int d = u >> 2, b = u & 3;
    w[d] = (w[d] & ~(0xffu << (8 * b))) | ((pat & 0xffu) << (8 * b));
  }
}

// 16 int8-domain A bytes of im2col row `ri`, k in [kb, kb+16).
template <bool IS1X1, int VEC>
__device__ __forceinline__ v4i load_a(const bh_conv_params& p, const RowInfo& ri, int K, int kb,
                                      uint32_t xorw, uint32_t padw) {
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  if (ri.valid) {
    const uint8_t* in = (const uint8_t*)p.input;
#pragma unroll
    for (int u = 0; u < 16 / VEC; ++u) {
      const int k = kb + u * VEC;
      if (k >= K) {
        fill_unit<VEC>(w, u, 0u);
      } else if constexpr (IS1X1) {
        load_unit<VEC>(in + ri.base + k, w, u);
        if constexpr (VEC == 1) {
          const int d = u >> 2, b = u & 3;
          w[d] ^= (xorw & (0xffu << (8 * b)));
        }
      } else {
        const int tap = k / p.in_c;
        const int ci = k - tap * p.in_c;
        const int fy = tap / p.k_w;
        const int fx = tap - fy * p.k_w;
        const int y = ri.y0 + fy * p.dil_h;
        const int x = ri.x0 + fx * p.dil_w;
        if (y >= 0 && y < p.in_h && x >= 0 && x < p.in_w) {
          load_unit<VEC>(in + ri.base + ((long)y * p.in_w + x) * p.in_c + ci, w, u);
          if constexpr (VEC == 1) {
            const int d = u >> 2, b = u & 3;
            w[d] ^= (xorw & (0xffu << (8 * b)));
          } else if constexpr (VEC == 8) {
            w[2 * u] ^= xorw; w[2 * u + 1] ^= xorw;
          } else if constexpr (VEC == 4) {
            w[u] ^= xorw;
          } else {
            w[0] ^= xorw; w[1] ^= xorw; w[2] ^= xorw; w[3] ^= xorw;
          }
        } else {
          fill_unit<VEC>(w, u, padw);
        }
      }
    }
    if constexpr (IS1X1 && VEC > 1) {
      // XOR only the loaded (k < K) part; K % VEC == 0 so whole units.
#pragma unroll
      for (int u = 0; u < 16 / VEC; ++u) {
        if (kb + u * VEC < K) {
          if constexpr (VEC == 16) { w[0] ^= xorw; w[1] ^= xorw; w[2] ^= xorw; w[3] ^= xorw; }
          else if constexpr (VEC == 8) { w[2 * u] ^= xorw; w[2 * u + 1] ^= xorw; }
          else { w[u] ^= xorw; }
        }
      }
    }
  }
  v4i r;
  r.x = (int)w[0]; r.y = (int)w[1]; r.z = (int)w[2]; r.w = (int)w[3];
  return r;
}

template <int WM, int WN, int WAVES_M, int WAVES_N, bool IS1X1, int VEC, bool WZP>
__global__ __launch_bounds__(256) void conv_mfma_kernel(bh_conv_params p, int M, int K, int N) {
  constexpr int TM = WAVES_M * WM * 16;
  constexpr int TN = WAVES_N * WN * 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  const int m0 = blockIdx.x * TM + wave_m * WM * 16;
  const int n0 = blockIdx.y * TN + wave_n * WN * 16;
  const int r16 = lane & 15;
  const int g = lane >> 4;

  const uint32_t xorw = splat_byte(p.in_xor);
  const uint32_t padw = splat_byte(p.in_zp);

  RowInfo ri[WM];
#pragma unroll
  for (int wm = 0; wm < WM; ++wm) {
    const int m = m0 + wm * 16 + r16;
    ri[wm].valid = m < M;
    const int mm = ri[wm].valid ? m : 0;
    const int ox = mm % p.out_w;
    const int t = mm / p.out_w;
    const int oy = t % p.out_h;
    const int n = t / p.out_h;
    if constexpr (IS1X1) {
      ri[wm].base = (((long)n * p.in_h + (long)oy * p.stride_h) * p.in_w + (long)ox * p.stride_w) * p.in_c;
      ri[wm].y0 = 0; ri[wm].x0 = 0;
    } else {
      ri[wm].base = (long)n * p.in_h * p.in_w * p.in_c;
      ri[wm].y0 = oy * p.stride_h - p.pad_h;
      ri[wm].x0 = ox * p.stride_w - p.pad_w;
    }
  }

  v4i acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = (v4i){0, 0, 0, 0};
  int rs[WM];
#pragma unroll
  for (int i = 0; i < WM; ++i) rs[i] = 0;

  const int8_t* wrow = p.weights + (long)(n0 + r16) * p.k_pad + g * 16;

  for (int kb0 = 0; kb0 < K; kb0 += 64) {
    const int kb = kb0 + g * 16;
    v4i a[WM], b[WN];
#pragma unroll
    for (int wm = 0; wm < WM; ++wm) a[wm] = load_a<IS1X1, VEC>(p, ri[wm], K, kb, xorw, padw);
#pragma unroll
    for (int wn = 0; wn < WN; ++wn) b[wn] = *(const v4i*)(wrow + (long)wn * 16 * p.k_pad + kb0);
#pragma unroll
    for (int wm = 0; wm < WM; ++wm)
#pragma unroll
      for (int wn = 0; wn < WN; ++wn)
        acc[wm][wn] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[wm], b[wn], acc[wm][wn], 0, 0, 0);
    if constexpr (WZP) {
#pragma unroll
      for (int wm = 0; wm < WM; ++wm) {
        rs[wm] = __builtin_amdgcn_sdot4(a[wm].x, 0x01010101, rs[wm], false);
        rs[wm] = __builtin_amdgcn_sdot4(a[wm].y, 0x01010101, rs[wm], false);
        rs[wm] = __builtin_amdgcn_sdot4(a[wm].z, 0x01010101, rs[wm], false);
        rs[wm] = __builtin_amdgcn_sdot4(a[wm].w, 0x01010101, rs[wm], false);
      }
    }
  }

  int rowsum[WM][4];
  if constexpr (WZP) {
#pragma unroll
    for (int wm = 0; wm < WM; ++wm) {
      int s = rs[wm];
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
#pragma unroll
      for (int r = 0; r < 4; ++r) rowsum[wm][r] = __shfl(s, 4 * g + r);
    }
  }

  uint8_t* out = (uint8_t*)p.output;
#pragma unroll
  for (int wn = 0; wn < WN; ++wn) {
    const int n = n0 + wn * 16 + r16;
    if (n >= N) continue;
    const int32_t be = p.bias_eff[n];
    const int32_t mu = p.mult[n];
    const int32_t sh = p.shift[n];
#pragma unroll
    for (int wm = 0; wm < WM; ++wm) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 16 + 4 * g + r;
        if (m >= M) continue;
        int32_t v = acc[wm][wn][r] + be;
        if constexpr (WZP) v -= p.w_zp * rowsum[wm][r];
        v = requant(v, mu, sh) + p.out_zp;
        out[(long)m * N + n] = (uint8_t)clamp_i32(v, p.act_min, p.act_max);
      }
    }
  }
}

template <int WM, int WN, int WAVES_M, int WAVES_N, bool IS1X1, int VEC, bool WZP>
static int launch_tile(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  constexpr int TM = WAVES_M * WM * 16;
  constexpr int TN = WAVES_N * WN * 16;
  dim3 grid((M + TM - 1) / TM, (N + TN - 1) / TN);
  hipLaunchKernelGGL((conv_mfma_kernel<WM, WN, WAVES_M, WAVES_N, IS1X1, VEC, WZP>), grid, dim3(256), 0, s,
                     p, M, K, N);
  return bh_check_launch("conv_mfma_kernel");
}

template <bool IS1X1, int VEC, bool WZP>
static int launch_shape(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  if (N <= 16) return launch_tile<2, 1, 4, 1, IS1X1, VEC, WZP>(p, M, K, N, s);
  if (N <= 32) return launch_tile<2, 2, 4, 1, IS1X1, VEC, WZP>(p, M, K, N, s);
  return launch_tile<2, 2, 2, 2, IS1X1, VEC, WZP>(p, M, K, N, s);
}

template <bool IS1X1, bool WZP>
static int launch_vec(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  const int c = p.in_c;
  if (c % 16 == 0) return launch_shape<IS1X1, 16, WZP>(p, M, K, N, s);
  if (c % 8 == 0) return launch_shape<IS1X1, 8, WZP>(p, M, K, N, s);
  if (c % 4 == 0) return launch_shape<IS1X1, 4, WZP>(p, M, K, N, s);
  return launch_shape<IS1X1, 1, WZP>(p, M, K, N, s);
}

}  // namespace bh

extern "C" int bh_conv_packed_geometry(int out_c, int k, int* k_pad, int* n_pad) {
  if (out_c <= 0 || k <= 0 || !k_pad || !n_pad) return BH_EINVAL;
  *k_pad = (k + 63) / 64 * 64;
  *n_pad = (out_c + 63) / 64 * 64;
  return 0;
}

extern "C" int bh_pack_conv_weights(const void* w, int w_signed, int out_c, int k, int k_pad,
                                    int n_pad, const int32_t* bias, int32_t in_zp, int32_t w_zp,
                                    int8_t* packed, int32_t* bias_eff) {
  if (!w || !packed || !bias_eff || k_pad < k || n_pad < out_c || (k_pad % 64) || (n_pad % 64))
    return BH_EINVAL;
  const uint8_t* src = (const uint8_t*)w;
  for (long i = 0; i < (long)n_pad * k_pad; ++i) packed[i] = 0;
  for (int c = 0; c < out_c; ++c) {
    int64_t s = 0;
    for (int i = 0; i < k; ++i) {
      const int v = w_signed ? (int)(int8_t)src[(long)c * k + i] : (int)src[(long)c * k + i] - 128;
      packed[(long)c * k_pad + i] = (int8_t)v;
      s += v;
    }
    const int64_t be = (bias ? (int64_t)bias[c] : 0) - (int64_t)in_zp * s + (int64_t)k * in_zp * w_zp;
    bias_eff[c] = (int32_t)be;
  }
  return 0;
}

extern "C" int bh_conv2d_i8(const bh_conv_params* pp, bh_stream_t stream) {
  if (!pp) return BH_EINVAL;
  const bh_conv_params& p = *pp;
  const long Ml = (long)p.batch * p.out_h * p.out_w;
  const int K = p.k_h * p.k_w * p.in_c;
  const int N = p.out_c;
  if (Ml <= 0 || Ml > INT32_MAX || K <= 0 || N <= 0 || p.k_pad < K || p.n_pad < N ||
      (p.k_pad % 64) || (p.n_pad % 64) || !p.input || !p.output || !p.weights || !p.bias_eff ||
      !p.mult || !p.shift || p.stride_h <= 0 || p.stride_w <= 0) {
    bh_set_last_error("bh_conv2d_i8: invalid parameters");
    return BH_EINVAL;
  }
  const int M = (int)Ml;
  hipStream_t s = (hipStream_t)stream;
  const bool is1x1 = p.k_h == 1 && p.k_w == 1 && p.pad_h == 0 && p.pad_w == 0;
  const bool wzp = p.w_zp != 0;
  if (is1x1) return wzp ? bh::launch_vec<true, true>(p, M, K, N, s) : bh::launch_vec<true, false>(p, M, K, N, s);
  return wzp ? bh::launch_vec<false, true>(p, M, K, N, s) : bh::launch_vec<false, false>(p, M, K, N, s);
}
