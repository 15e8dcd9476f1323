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
// 0, like TFLite's skipped taps) and the K tail is zero-filled.  An optional
// fused epilogue applies the following residual ADD (add.cc arithmetic) to
// y before it is stored, so y never round-trips HBM.
//
// GEMM view (NHWC / OHWI): M = batch*out_h*out_w pixels, N = out_c,
// K = k_h*k_w*in_c.  Both operands are K-contiguous, so each lane's MFMA
// fragment (16 consecutive k of one row) is one 16-byte load for 1x1
// layers.  v_mfma_i32_16x16x64_i8: lane l supplies A[l&15][16*(l>>4)+j] and
// B[16*(l>>4)+j][l&15]; D lands as D[4*(l>>4)+r][l&15] (r = 0..3).
//
// Batch-1 MobileNet layers are tiny (M*N*K ~ 1-25 MMAC), so the kernel is
// shaped for latency: the host picks the workgroup tile per layer so that
// enough workgroups exist, deep-K layers split K across the 4 waves of a
// workgroup (partials reduced through LDS), and each wave issues the loads
// of up to 4 K-steps before their MFMAs.
#include <cstdlib>

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
__device__ __forceinline__ void xor_unit(uint32_t* w, int u, uint32_t xorw) {
  if constexpr (VEC == 16) {
    w[0] ^= xorw; w[1] ^= xorw; w[2] ^= xorw; w[3] ^= xorw;
  } else if constexpr (VEC == 8) {
    w[2 * u] ^= xorw; w[2 * u + 1] ^= xorw;
  } else if constexpr (VEC == 4) {
    w[u] ^= xorw;
  } else {
    const int d = u >> 2, b = u & 3;
    w[d] ^= (xorw & (0xffu << (8 * b)));
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
// Runtime divisors of the index math, as multiply-high reciprocals (FastDiv)
struct ConvDivs {
  FastDiv out_w, out_h, in_c, k_w;
};

template <bool IS1X1, int VEC>
__device__ __forceinline__ v4i load_a(const bh_conv_params& p, const ConvDivs& dv, const RowInfo& ri, int K,
                                      int kb, uint32_t xorw, uint32_t padw) {
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
        xor_unit<VEC>(w, u, xorw);
      } else {
        const int tap = dv.in_c.div(k);
        const int ci = k - tap * p.in_c;
        const int fy = dv.k_w.div(tap);
        const int fx = tap - fy * p.k_w;
        const int y = ri.y0 + fy * p.dil_h;
        const int x = ri.x0 + fx * p.dil_w;
        if (y >= 0 && y < p.in_h && x >= 0 && x < p.in_w) {
          load_unit<VEC>(in + ri.base + ((long)y * p.in_w + x) * p.in_c + ci, w, u);
          xor_unit<VEC>(w, u, xorw);
        } else {
          fill_unit<VEC>(w, u, padw);
        }
      }
    }
  }
  v4i r;
  r.x = (int)w[0]; r.y = (int)w[1]; r.z = (int)w[2]; r.w = (int)w[3];
  return r;
}

__device__ __forceinline__ int rowsum16(v4i a, int s) {
  s = __builtin_amdgcn_sdot4(a.x, 0x01010101, s, false);
  s = __builtin_amdgcn_sdot4(a.y, 0x01010101, s, false);
  s = __builtin_amdgcn_sdot4(a.z, 0x01010101, s, false);
  return __builtin_amdgcn_sdot4(a.w, 0x01010101, s, false);
}

// Epilogue of one transposed 16x16 tile: the lane holds output channels
// nb..nb+3 of pixel m (D^T = W x X^T on the MFMA), so its four requantised
// bytes leave as one dword store when N % 4 == 0.  acc excludes the folded
// bias; rsum is pixel m's input row sum (uint8 filters).
__device__ __forceinline__ void conv_epilogue4(const bh_conv_params& p, v4i acc, int rsum, int m, int nb, int M,
                                               int N) {
  if (m >= M || nb >= N) return;
  // dword path: N % 4 == 0 (then nb + 3 < N too) and 4-byte aligned output /
  // residual bases (a concat-elided output may start at any byte)
  const bool vec = (N & 3) == 0 && (((uintptr_t)p.output | (uintptr_t)p.residual) & 3) == 0;
  int32_t be[4], mu[4], sh[4];
  if (vec) {
    const v4i b4 = *(const v4i*)(p.bias_eff + nb);
    const v4i m4 = *(const v4i*)(p.mult + nb);
    const v4i s4 = *(const v4i*)(p.shift + nb);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      be[r] = b4[r];
      mu[r] = m4[r];
      sh[r] = s4[r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nb + r < N ? nb + r : nb;
      be[r] = p.bias_eff[n];
      mu[r] = p.mult[n];
      sh[r] = p.shift[n];
    }
  }
  const long o = (long)m * N + nb;
  const uint8_t* res = (const uint8_t*)p.residual;
  const bool res_signed = p.in_xor == 0;  // residual shares the activation type
  const uint8_t* tab = (const uint8_t*)p.out_table;
  uint32_t rq = 0;
  if (res) {
    if (vec) {
      rq = *(const uint32_t*)(res + o);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (nb + r < N) rq |= (uint32_t)res[o + r] << (8 * r);
    }
  }
  uint32_t packed = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int32_t a = acc[r] + be[r];
    if (p.w_zp != 0) a -= p.w_zp * rsum;
    int32_t v = p.requant_fast ? requant_out<true>(a, chan_q(mu[r], sh[r], p.out_zp), p.out_zp, p.act_min, p.act_max)
                               : requant_out<false>(a, chan_q(mu[r], sh[r], p.out_zp), p.out_zp, p.act_min, p.act_max);
    if (res) {
      const uint32_t qb = (rq >> (8 * r)) & 0xffu;
      const int32_t q = res_signed ? (int32_t)(int8_t)qb : (int32_t)qb;
      const int32_t sy = requant_lt1((v + p.add_y_off) * (1 << p.add_left_shift), p.add_y_mult, p.add_y_shift);
      const int32_t sr = requant_lt1((q + p.add_r_off) * (1 << p.add_left_shift), p.add_r_mult, p.add_r_shift);
      v = clamp_i32(requant_lt1(sy + sr, p.add_o_mult, p.add_o_shift) + p.add_o_off, p.add_act_min, p.add_act_max);
    }
    const uint32_t byte = tab ? tab[(uint8_t)v] : ((uint32_t)v & 0xffu);
    packed |= byte << (8 * r);
  }
  uint8_t* out = (uint8_t*)p.output + o;
  if (vec) {
    *(uint32_t*)out = packed;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (nb + r < N) out[r] = (uint8_t)(packed >> (8 * r));
  }
}

constexpr int KU = 4;  // K-steps whose loads are issued together

// WM x WN 16x16 tiles per wave; waves arranged WAVES_M x WAVES_N x SPLITK.
template <int WM, int WN, int WAVES_M, int WAVES_N, int SPLITK, bool IS1X1, int VEC>
__global__ __launch_bounds__(256) void conv_mfma_kernel(bh_conv_params p, int M, int K, int N, int kchunk, ConvDivs dv,
                                                        int nblocks, int xcd) {
  static_assert(WAVES_M * WAVES_N * SPLITK == 4, "4 waves per workgroup");
  constexpr int TM = WAVES_M * WM * 16;
  constexpr int TN = WAVES_N * WN * 16;
  constexpr int NACC = WM * WN * 4;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int kz = wave / (WAVES_M * WAVES_N);
  const int wt = wave % (WAVES_M * WAVES_N);
  const int wave_m = wt % WAVES_M;
  const int wave_n = wt / WAVES_M;
  // 1-D grid, N-blocks fastest; with xcd each XCD (hardware ids i % 8) runs
  // a contiguous run of logical blocks, so all N-blocks of a pixel block -
  // which read the same input rows - share one L2
  const int logical = xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int bm = logical / nblocks;
  const int bn = logical - bm * nblocks;
  const int m0 = bm * TM + wave_m * WM * 16;
  const int n0 = bn * TN + wave_n * WN * 16;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const bool wzp = p.w_zp != 0;

  const uint32_t xorw = splat_byte(p.in_xor);
  const uint32_t padw = splat_byte(p.in_zp);

  RowInfo ri[WM];
#pragma unroll
  for (int wm = 0; wm < WM; ++wm) {
    const int m = m0 + wm * 16 + r16;
    ri[wm].valid = m < M;
    const int mm = ri[wm].valid ? m : 0;
    const int t = dv.out_w.div(mm);
    const int ox = mm - t * p.out_w;
    const int n = dv.out_h.div(t);
    const int oy = t - n * p.out_h;
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
  const int kbeg = kz * kchunk;
  const int kend = min(K, kbeg + kchunk);

  for (int kb0 = kbeg; kb0 < kend; kb0 += 64 * KU) {
    v4i a[KU][WM], b[KU][WN];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int kb = kb0 + u * 64;
      if (kb < kend) {
#pragma unroll
        for (int wm = 0; wm < WM; ++wm) a[u][wm] = load_a<IS1X1, VEC>(p, dv, ri[wm], K, kb + g * 16, xorw, padw);
#pragma unroll
        for (int wn = 0; wn < WN; ++wn) b[u][wn] = *(const v4i*)(wrow + (long)wn * 16 * p.k_pad + kb);
      }
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (kb0 + u * 64 < kend) {
#pragma unroll
        for (int wm = 0; wm < WM; ++wm)
#pragma unroll
          for (int wn = 0; wn < WN; ++wn)
            acc[wm][wn] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[u][wn], a[u][wm], acc[wm][wn], 0, 0, 0);
        if (wzp) {
#pragma unroll
          for (int wm = 0; wm < WM; ++wm) rs[wm] = rowsum16(a[u][wm], rs[wm]);
        }
      }
    }
  }

  // pixel row sums (uint8 filters): lane (g, r16) holds a 16-byte K slice of
  // pixel r16; the 4 slices of a K-step sit in lanes r16 + 16g
  if (wzp) {
#pragma unroll
    for (int wm = 0; wm < WM; ++wm) {
      rs[wm] += __shfl_xor(rs[wm], 16);
      rs[wm] += __shfl_xor(rs[wm], 32);
    }
  }
  if constexpr (SPLITK > 1) {
    // every wave parks its K-split partials in LDS; after one barrier wave w
    // sums and finishes tiles w, w+4, ... so the epilogue runs on all waves
    static_assert(WAVES_M * WAVES_N == 1, "split-K workgroups hold one wave tile");
    __shared__ int red[SPLITK][NACC + WM][64];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[kz][(i * WN + j) * 4 + r][lane] = acc[i][j][r];
#pragma unroll
    for (int i = 0; i < WM; ++i) red[kz][NACC + i][lane] = rs[i];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < WM * WN; ++t) {
      if (t % SPLITK != kz) continue;
      const int i = t / WN, j = t % WN;
      v4i sum = {0, 0, 0, 0};
      int rsum = 0;
#pragma unroll
      for (int z = 0; z < SPLITK; ++z) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sum[r] += red[z][t * 4 + r][lane];
        rsum += red[z][NACC + i][lane];
      }
      conv_epilogue4(p, sum, rsum, m0 + i * 16 + r16, n0 + j * 16 + 4 * g, M, N);
    }
  } else {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) conv_epilogue4(p, acc[i][j], rs[i], m0 + i * 16 + r16, n0 + j * 16 + 4 * g, M, N);
  }
}

template <int WM, int WN, int WAVES_M, int WAVES_N, int SPLITK, bool IS1X1, int VEC>
static int launch_cfg(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  constexpr int TM = WAVES_M * WM * 16;
  constexpr int TN = WAVES_N * WN * 16;
  const int ksteps = (K + 63) / 64;
  const int kchunk = (ksteps + SPLITK - 1) / SPLITK * 64;
  ConvDivs dv;
  dv.out_w = FastDiv(p.out_w);
  dv.out_h = FastDiv(p.out_h);
  dv.in_c = FastDiv(p.in_c);
  dv.k_w = FastDiv(p.k_w);
  const int gm = (M + TM - 1) / TM, gn = (N + TN - 1) / TN;
  static const int xcd = [] {
    const char* e = std::getenv("BH_CONV_XCD");  // A-B runs: 0 = plain order
    return e ? std::atoi(e) : 1;
  }();
  hipLaunchKernelGGL((conv_mfma_kernel<WM, WN, WAVES_M, WAVES_N, SPLITK, IS1X1, VEC>), dim3(gm * gn), dim3(256), 0,
                     s, p, M, K, N, kchunk, dv, gn, xcd);
  return bh_check_launch("conv_mfma_kernel");
}

static inline long wgs(int M, int N, int tm, int tn) { return (long)((M + tm - 1) / tm) * ((N + tn - 1) / tn); }

// Tile selection: the largest tile that still yields >= kTargetWG
// workgroups, else the smallest; deep-K layers (>= 3 K-steps) split K over
// the 4 waves of a workgroup.
constexpr long kTargetWG = 160;

template <bool IS1X1, int VEC>
static int launch_shape(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  const int ksteps = (K + 63) / 64;
  if (ksteps >= 3) {
    if (wgs(M, N, 32, 32) >= kTargetWG) return launch_cfg<2, 2, 1, 1, 4, IS1X1, VEC>(p, M, K, N, s);
    if (wgs(M, N, 16, 32) >= kTargetWG) return launch_cfg<1, 2, 1, 1, 4, IS1X1, VEC>(p, M, K, N, s);
    return launch_cfg<1, 1, 1, 1, 4, IS1X1, VEC>(p, M, K, N, s);
  }
  if (N <= 16) {
    if (wgs(M, N, 128, 16) >= kTargetWG) return launch_cfg<2, 1, 4, 1, 1, IS1X1, VEC>(p, M, K, N, s);
    return launch_cfg<1, 1, 4, 1, 1, IS1X1, VEC>(p, M, K, N, s);
  }
  if (N <= 32 && wgs(M, N, 128, 32) >= kTargetWG) return launch_cfg<2, 2, 4, 1, 1, IS1X1, VEC>(p, M, K, N, s);
  if (wgs(M, N, 64, 64) >= kTargetWG) return launch_cfg<2, 2, 2, 2, 1, IS1X1, VEC>(p, M, K, N, s);
  return launch_cfg<1, 1, 2, 2, 1, IS1X1, VEC>(p, M, K, N, s);
}

}  // namespace bh

int bh_conv_direct_launch(const bh_conv_params& p, int M, int K, hipStream_t s);  // conv_direct.hip
int bh_conv_stem_launch(const bh_conv_params& p, int M, int K, hipStream_t s);    // conv_direct.hip
int bh_conv_rows_launch(const bh_conv_params& p, int M, int K, int N, hipStream_t s);  // conv_rows.hip
int bh_conv_xs_launch(const bh_conv_params& p, int M, int K, int N, hipStream_t s);    // conv_rows.hip

namespace {
// batched 1x1 layers (K <= 320) at or above this many output pixels take the
// x-stationary kernel conv_xs_kernel: measured faster than conv_mfma_kernel
// on every MobileNetV2 1x1 shape from M = 3136 up (gpurun_out/lb_conv_*,
// DESIGN.md); BH_CONV_XS_MIN_M overrides (diagnostics / tuning)
long XsMinM() {
  static const long v = [] {
    const char* e = std::getenv("BH_CONV_XS_MIN_M");
    return e ? std::atol(e) : 2048L;
  }();
  return v;
}
// conv_rows_kernel (any K) is opt-in: BH_CONV_ROWS_MIN_M = the M from which
// deep-K batched 1x1 layers take it (default: never; slower than
// conv_mfma_kernel on every K > 320 MobileNet shape measured)
long RowsMinM() {
  static const long v = [] {
    const char* e = std::getenv("BH_CONV_ROWS_MIN_M");
    return e ? std::atol(e) : -1L;
  }();
  return v;
}

enum Route { kDirect, kStem, kXs, kRows, kMfma };

Route route(const bh_conv_params& p, long M, int K, int N) {
  const bool is1x1 = p.k_h == 1 && p.k_w == 1 && p.pad_h == 0 && p.pad_w == 0;
  // RGB-stem-like layers (tiny K, byte-granular gather): direct VALU kernel
  if (!is1x1 && K <= 64 && p.in_c < 8) {
    const bool stem = p.k_h == 3 && p.k_w == 3 && p.in_c == 3 && p.dil_w == 1 && N % 8 == 0 && !p.residual;
    return stem && !std::getenv("BH_CONV_NO_STEM") ? kStem : kDirect;
  }
  const bool aligned = (((uintptr_t)p.output | (uintptr_t)p.residual | (uintptr_t)p.input) & 3) == 0;
  if (is1x1 && p.stride_h == 1 && p.stride_w == 1 && N % 4 == 0 && K % 4 == 0 && aligned) {
    if (K <= 320 && M >= XsMinM()) return kXs;
    if (RowsMinM() >= 0 && M >= RowsMinM()) return kRows;
  }
  return kMfma;
}
}  // namespace

extern "C" const char* bh_conv2d_i8_kernel(const bh_conv_params* p) {
  if (!p) return "";
  static const char* const names[] = {"conv_direct_kernel", "conv_stem_kernel", "conv_xs_kernel",
                                      "conv_rows_kernel", "conv_mfma_kernel"};
  return names[route(*p, (long)p->batch * p->out_h * p->out_w, p->k_h * p->k_w * p->in_c, p->out_c)];
}

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
  const int c = p.in_c;
  switch (route(p, M, K, N)) {
    case kDirect: return bh_conv_direct_launch(p, M, K, s);
    case kStem: return bh_conv_stem_launch(p, M, K, s);
    case kXs: return bh_conv_xs_launch(p, M, K, N, s);
    case kRows: return bh_conv_rows_launch(p, M, K, N, s);
    case kMfma: break;
  }
  if (is1x1 && c % 16 == 0) return bh::launch_shape<true, 16>(p, M, K, N, s);
  if (is1x1 && c % 8 == 0) return bh::launch_shape<true, 8>(p, M, K, N, s);
  if (is1x1 && c % 4 == 0) return bh::launch_shape<true, 4>(p, M, K, N, s);
  if (c % 16 == 0) return bh::launch_shape<false, 16>(p, M, K, N, s);
  if (c % 8 == 0) return bh::launch_shape<false, 8>(p, M, K, N, s);
  if (c % 4 == 0) return bh::launch_shape<false, 4>(p, M, K, N, s);
  return bh::launch_shape<false, 1>(p, M, K, N, s);
}
