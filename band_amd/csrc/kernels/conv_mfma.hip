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

// Per-lane channel constants of a transposed 16x16 tile's epilogue: the lane
// owns output channels nb..nb+3 (every pixel row of the tile uses the same
// four), so kernels that store several pixel tiles per channel group build
// them once.
struct Chan4 {
  int32_t be[4];
  ChanQ q[4];
  bool vec;  // dword path: N % 4 == 0 and 4-byte aligned output / residual bases
};

__device__ __forceinline__ Chan4 chan4(const bh_conv_params& p, int nb, int N) {
  Chan4 c;
  // (a concat-elided output may start at any byte, and its images at any
  // stride)
  c.vec = (N & 3) == 0 && (((uintptr_t)p.output | (uintptr_t)p.residual | (uintptr_t)p.out_img_stride) & 3) == 0;
  int32_t mu[4], sh[4];
  if (c.vec) {
    const v4i b4 = *(const v4i*)(p.bias_eff + nb);
    const v4i m4 = *(const v4i*)(p.mult + nb);
    const v4i s4 = *(const v4i*)(p.shift + nb);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      c.be[r] = b4[r];
      mu[r] = m4[r];
      sh[r] = s4[r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nb + r < N ? nb + r : nb;
      c.be[r] = p.bias_eff[n];
      mu[r] = p.mult[n];
      sh[r] = p.shift[n];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) c.q[r] = chan_q(mu[r], sh[r], p.out_zp);
  return c;
}

// Epilogue of one transposed 16x16 tile: the lane holds output channels
// nb..nb+3 of pixel m (D^T = W x X^T on the MFMA), so its four requantised
// bytes leave as one dword store when N % 4 == 0.  acc excludes the folded
// bias; rsum is pixel m's input row sum (uint8 filters).
__device__ __forceinline__ void conv_store4(const bh_conv_params& p, v4i acc, int rsum, int m, int nb, int M, int N,
                                            const Chan4& c) {
  if (m >= M || nb >= N) return;
  const long o = (long)m * N + nb;
  const uint8_t* res = (const uint8_t*)p.residual;
  const bool res_signed = p.in_xor == 0;  // residual shares the activation type
  const uint8_t* tab = (const uint8_t*)p.out_table;
  uint32_t rq = 0;
  if (res) {
    if (c.vec) {
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
    int32_t a = acc[r] + c.be[r];
    if (p.w_zp != 0) a -= p.w_zp * rsum;
    int32_t v = p.requant_fast ? requant_out<true>(a, c.q[r], p.out_zp, p.act_min, p.act_max)
                               : requant_out<false>(a, c.q[r], p.out_zp, p.act_min, p.act_max);
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
  long oo = o;
  if (p.out_img_stride) {  // a slice of a concatenation: image n at n * stride (uniform branch)
    const int hw = p.out_h * p.out_w;
    const int img = m / hw;
    oo = (long)img * p.out_img_stride + (long)(m - img * hw) * N + nb;
  }
  uint8_t* out = (uint8_t*)p.output + oo;
  if (c.vec) {
    *(uint32_t*)out = packed;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (nb + r < N) out[r] = (uint8_t)(packed >> (8 * r));
  }
}

__device__ __forceinline__ void conv_epilogue4(const bh_conv_params& p, v4i acc, int rsum, int m, int nb, int M,
                                               int N) {
  if (m >= M || nb >= N) return;
  conv_store4(p, acc, rsum, m, nb, M, N, chan4(p, nb, N));
}

constexpr int KU = 4;  // K-steps whose loads are issued together

// WM x WN 16x16 tiles per wave; waves arranged WAVES_M x WAVES_N x SPLITK.
// One workgroup's tile: (bm, bn) in the layer's output-block grid
// (conv_mfma_kernel, or a member of a grouped launch).
template <int WM, int WN, int WAVES_M, int WAVES_N, int SPLITK, bool IS1X1, int VEC>
__device__ __forceinline__ void conv_mfma_tile(const bh_conv_params& p, int M, int K, int N, int kchunk,
                                               const ConvDivs& dv, int bm, int bn) {
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
__global__ __launch_bounds__(256) void conv_mfma_kernel(bh_conv_params p, int M, int K, int N, int kchunk, ConvDivs dv,
                                                        int gm, int gn, XcdSplit xs) {
  // 1-D grid in the 2-D XCD split (xcd_tile): each XCD's L2 holds one pixel
  // range of the input and one channel range of the filters
  int bm, bn;
  xcd_tile((int)blockIdx.x, (int)gridDim.x, xs, gm, gn, bm, bn);
  if (bm >= gm) return;
  conv_mfma_tile<WM, WN, WAVES_M, WAVES_N, SPLITK, IS1X1, VEC>(p, M, K, N, kchunk, dv, bm, bn);
}

// ---------------------------------------------------------------------------
// Grouped launch of independent small CONV_2D layers (conv_group_kernel):
// the heads of a detector / pose model (SSD's 12 box / class predictors,
// PoseNet's four 1x1 heads) are each a few hundred workgroups of work that
// would otherwise pay a whole dispatch (~4 us of fixed cost at the empty-
// kernel floor) one after another.  One launch carries
// all of them: workgroup b belongs to the member whose [blk0, blk0 + blocks)
// range holds b, and runs that member's conv_mfma_kernel tile - the same
// arithmetic, so the results are the members' own, bit for bit.  The member
// table (host-built, bh_conv_group_plan) lives in device memory.
// ---------------------------------------------------------------------------
struct ConvGroupMember {
  bh_conv_params p;
  ConvDivs dv;
  int M, K, N, kchunk, gn, form, blk0, blocks;
};
constexpr int kConvGroupMax = 32;

// Profiler workaround only, off by default: -DBH_CONV_GROUP_ARGS_PAD=1 pads
// the launch arguments to 256 bytes.  rocprofv3 7.2's hipGraphLaunch
// interception faults on graphs that mix copy and kernel nodes
// (tools/graph_copytrace_probe.hip reproduces it with no code of ours); one
// traced run with the 12-byte block faulted and one padded run traced
// (profiles/r04q_tr2_copytrace_crash.txt, r04u), so the padding moves the
// fault rather than removing it.  Traced runs use eager launches
// (bench.py --no-graph), which is the supported workaround.
#ifndef BH_CONV_GROUP_ARGS_PAD
#define BH_CONV_GROUP_ARGS_PAD 0
#endif
struct ConvGroupArgs {
  const ConvGroupMember* tab;
  int n;
#if BH_CONV_GROUP_ARGS_PAD
  int pad[61];
#endif
};

template <bool IS1X1>
__global__ __launch_bounds__(256) void conv_group_kernel(ConvGroupArgs a) {
  const ConvGroupMember* __restrict__ tab = a.tab;
  const int n = a.n;
  const int b = (int)blockIdx.x;
  int i = 0;
  while (i + 1 < n && tab[i + 1].blk0 <= b) ++i;  // uniform: scalar loads of the table
  const ConvGroupMember& e = tab[i];
  const int local = b - e.blk0;
  switch (e.form) {
    case 0: conv_mfma_tile<1, 1, 1, 1, 4, IS1X1, 16>(e.p, e.M, e.K, e.N, e.kchunk, e.dv, local / e.gn, local % e.gn); break;
    case 1: conv_mfma_tile<1, 1, 2, 2, 1, IS1X1, 16>(e.p, e.M, e.K, e.N, e.kchunk, e.dv, local / e.gn, local % e.gn); break;
    case 2: conv_mfma_tile<2, 2, 1, 1, 4, IS1X1, 16>(e.p, e.M, e.K, e.N, e.kchunk, e.dv, local / e.gn, local % e.gn); break;
    default: conv_mfma_tile<2, 2, 2, 2, 1, IS1X1, 16>(e.p, e.M, e.K, e.N, e.kchunk, e.dv, local / e.gn, local % e.gn); break;
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
  const XcdSplit xs = xcd_split((long)p.batch * p.in_h * p.in_w * p.in_c, (long)N * K, gm, gn);
  BH_LAUNCH((conv_mfma_kernel<WM, WN, WAVES_M, WAVES_N, SPLITK, IS1X1, VEC>), dim3(xcd_grid(xs)), dim3(256), 0,
                     s, p, M, K, N, kchunk, dv, gm, gn, xs);
  return bh_check_launch("conv_mfma_kernel");
}

// ---------------------------------------------------------------------------
// conv_gemm_kernel: the deep / wide batched 1x1 layers (stride 1, int8
// activations, symmetric int8 filters) as an LDS-staged GEMM.
//
// conv_mfma_kernel gives every wave its own fragments straight from L2, so a
// workgroup tile of 32x32 outputs re-reads its A rows and B rows once per
// tile: on PoseNet's 14x14 512->1024 layer at batch 24 that is ~300 MB of L2
// reads for 10 GOP.  Here a workgroup owns a BM x BN output tile (up to
// 128 x 128) and walks K in 64-byte steps: the step's A rows (pixels) and B
// rows (filters) go global -> LDS with 16-byte global_load_lds (no VGPR
// staging), two LDS buffers so the next step's DMA runs under this step's
// MFMAs, and each of the 4 waves reads its 16-byte fragments back with
// ds_read_b128 and issues (BM/2/16) x (BN/2/16) v_mfma_i32_16x16x64_i8 per
// step.  LDS image: staged row r (A rows first, then B rows) is 64 bytes
// whose four 16-byte chunks are stored XOR-swizzled, chunk c at (c ^ (r>>2))
// & 3, so the 16 lanes of a ds_read_b128 group (16 consecutive rows, one
// chunk) hit 16 distinct 4-bank slots; glds writes lane-linear, so the swizzle
// is applied to each lane's global source address and undone on the read.
// The K tail reads a harmless in-row address (the packed filters are zero
// there, so it adds 0).  Epilogue: the conv_mfma_kernel one (transposed D:
// a lane holds 4 consecutive channels of one pixel, one dword store).
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;

// vmcnt(n) with n a compile-time count (glds instructions left in flight)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int WM, int WN, int WAVES_M, int WAVES_N, int NB>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_gemm_kernel(bh_conv_params p, int M, int K, int gm,
                                                                          int gn, int ksteps, XcdSplit xs) {
  constexpr int W = WAVES_M * WAVES_N;
  static_assert(W == 4 || W == 8, "4 or 8 waves per workgroup");
  static_assert(NB >= 2 && NB <= 4, "LDS ring depth");
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  constexpr int ROWS = BM + BN;  // 64-byte rows staged per K-step
  // glds instructions per wave per K-step (16 rows each); when ROWS is not a
  // multiple of 16 * W the last instruction of some waves stages padding rows
  // (a valid filter row into LDS nobody reads), so every wave issues NI and
  // the counted vmcnt waits stay uniform
  constexpr int NI = (ROWS + 16 * W - 1) / (16 * W);
  constexpr int STAGE = NI * 16 * W * 64;
  constexpr int D = NB - 1;  // K-steps staged ahead of the one computed
  __shared__ __attribute__((aligned(16))) uint8_t lds[NB * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // the 2-D XCD split, as in conv_mfma_kernel
  int bm, bn;
  xcd_tile((int)blockIdx.x, (int)gridDim.x, xs, gm, gn, bm, bn);
  if (bm >= gm) return;
  const int tm0 = bm * BM;
  const int tn0 = bn * BN;
  const int N = p.out_c;

  // this lane's source for each of its wave's staging instructions
  const uint8_t* src[NI];
  int kval[NI], goff[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = 16 * (wave + W * j) + (lane >> 2);
    const int g = (lane & 3) ^ ((row >> 2) & 3);
    goff[j] = 16 * g;
    if (row < BM) {
      const int m = min(tm0 + row, M - 1);
      src[j] = (const uint8_t*)p.input + (long)m * K + 16 * g;
      kval[j] = K - 16 * g;
    } else {
      const int n = min(min(tn0 + row - BM, tn0 + BN - 1), p.n_pad - 1);  // padding rows: the tile's last
      src[j] = (const uint8_t*)p.weights + (long)n * p.k_pad + 16 * g;
      kval[j] = 0x7fffffff;
    }
  }
  auto stage = [&](int ks) {
    const int kb = ks * 64;
    uint8_t* dst = lds + (ks % NB) * STAGE + wave * 1024;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const uint8_t* s = kb < kval[j] ? src[j] + kb : src[j] - goff[j];
      __builtin_amdgcn_global_load_lds((const void*)s, (lds_void_t*)(dst + j * W * 1024), 16, 0, 0);
    }
  };

  const int r16 = lane & 15;
  const int g = lane >> 4;
  const int chunk = ((g ^ (r16 >> 2)) & 3) << 4;
  const int wm0 = (wave % WAVES_M) * WM * 16;
  const int wn0 = (wave / WAVES_M) * WN * 16;
  v4i acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = (v4i){0, 0, 0, 0};

  // prologue: D steps in flight
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < ksteps) stage(d);
  for (int ks = 0; ks < ksteps; ++ks) {
    // step ks landed: this wave leaves the glds of steps ks+1 .. ks+D-1 in
    // flight (counted wait, never 0 in the steady state), the raw barrier
    // then orders every wave's DMA before the reads; it also retires every
    // wave's reads of step ks-1, whose buffer step ks+D now refills
    const int ahead = min(D - 1, ksteps - 1 - ks);
    if (ahead >= 2) wait_vmcnt<2 * NI>();
    else if (ahead == 1) wait_vmcnt<NI>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (ks + D < ksteps) stage(ks + D);
    const uint8_t* buf = lds + (ks % NB) * STAGE;
    v4i a[WM], b[WN];
#pragma unroll
    for (int i = 0; i < WM; ++i) a[i] = *(const v4i*)(buf + (wm0 + i * 16 + r16) * 64 + chunk);
#pragma unroll
    for (int j = 0; j < WN; ++j) b[j] = *(const v4i*)(buf + (BM + wn0 + j * 16 + r16) * 64 + chunk);
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a[i], acc[i][j], 0, 0, 0);
    // this step's reads are done before any wave passes the next barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // channel constants once per channel group, shared by the WM pixel tiles
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int nb = tn0 + wn0 + j * 16 + 4 * g;
    if (nb >= N) continue;
    const Chan4 c = chan4(p, nb, N);
#pragma unroll
    for (int i = 0; i < WM; ++i) conv_store4(p, acc[i][j], 0, tm0 + wm0 + i * 16 + r16, nb, M, N, c);
  }
}

template <int WM, int WN, int WAVES_M, int WAVES_N, int NB>
static int launch_gemm(const bh_conv_params& p, int M, int K, hipStream_t s) {
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  const int gm = (M + BM - 1) / BM, gn = (p.out_c + BN - 1) / BN;
  const XcdSplit xs = xcd_split((long)M * K, (long)p.out_c * K, gm, gn);
  BH_LAUNCH((conv_gemm_kernel<WM, WN, WAVES_M, WAVES_N, NB>), dim3(xcd_grid(xs)), dim3(WAVES_M * WAVES_N * 64), 0,
            s, p, M, K, gm, gn, (K + 63) / 64, xs);
  return bh_check_launch("conv_gemm_kernel");
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

// conv_gemm_kernel configuration (tools/gemm_cfg_sweep.sh, batch-24 C3
// shapes): 128x128 tiles over 8 waves (64x32 each, 2 LDS buffers) once they
// still give one workgroup per CU - PoseNet's 512/1024-channel layers, 1.6-2.7x
// conv_mfma_kernel; otherwise 64x64 tiles over 8 waves (16x32 each, 3 LDS
// buffers), which keep ~4 waves per SIMD on the mid-size layers.
// BH_GEMM_CFG=1 selects the first 4-wave form (128x128 ... 64x64, 4 buffers);
// 5: the two-tile rule without the 160-row tile.  Deeper LDS rings (3-4
// K-steps ahead) and 4-wave 128x64 tiles measured no faster
// (profiles/r03y_gemm.txt).
static int launch_gemm_shape(const bh_conv_params& p, int M, int K, hipStream_t s) {
  const int N = p.out_c;
  static const int cfg = [] {
    const char* e = std::getenv("BH_GEMM_CFG");  // A-B experiments
    return e ? std::atoi(e) : 0;
  }();
  if (cfg == 1) {
    if (wgs(M, N, 128, 128) >= 256) return launch_gemm<4, 4, 2, 2, 4>(p, M, K, s);
    if (wgs(M, N, 128, 64) >= 256) return launch_gemm<4, 2, 2, 2, 4>(p, M, K, s);
    if (wgs(M, N, 64, 128) >= 256) return launch_gemm<2, 4, 2, 2, 4>(p, M, K, s);
    return launch_gemm<2, 2, 2, 2, 4>(p, M, K, s);
  }
  // 128 x 128 tiles over 8 waves once they give a workgroup per CU; when
  // they give more than one round of workgroups but 160 x 128 tiles fit in
  // one, those (8 waves, 64 B of padding rows per wave staged per K-step).
  // BH_GEMM_CFG=5: without the 160-row tile.  (4-wave 160 x 128 / 80 x 128
  // tiles measured slower than two rounds of 8-wave ones:
  // profiles/r03z_gemm.txt.)
  const long w128 = wgs(M, N, 128, 128);
  if (cfg != 5 && w128 > 256 && wgs(M, N, 160, 128) <= 256) return launch_gemm<5, 2, 2, 4, 2>(p, M, K, s);
  if (w128 >= 256) return launch_gemm<4, 2, 2, 4, 2>(p, M, K, s);
  return launch_gemm<1, 2, 4, 2, 3>(p, M, K, s);
}

}  // namespace bh

int bh_conv_direct_launch(const bh_conv_params& p, int M, int K, hipStream_t s);  // conv_direct.hip
int bh_conv_stem_launch(const bh_conv_params& p, int M, int K, hipStream_t s);    // conv_direct.hip
int bh_conv_rows_launch(const bh_conv_params& p, int M, int K, int N, hipStream_t s);  // conv_rows.hip
int bh_conv_xs_launch(const bh_conv_params& p, int M, int K, int N, hipStream_t s);    // conv_rows.hip
int bh_conv_gemm_big_launch(const bh_conv_params& p, int M, int K, hipStream_t s);  // conv_gemm_big.hip
int bh_conv_stem_mfma_ok(const bh_conv_params& p);                                  // conv_stem_mfma.hip
int bh_conv_stem_mfma_launch(const bh_conv_params& p, int M, hipStream_t s);       // conv_stem_mfma.hip
const char* bh_conv_stem_kernel_name(const bh_conv_params& p, int M);           // conv_direct.hip

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

// conv_gemm_kernel (LDS-staged GEMM): BH_CONV_GEMM=0 off, 1 (default) the
// eligible layers of at least GemmMinOps() ops, 2 every eligible layer
int GemmMode() {
  static const int v = [] {
    const char* e = std::getenv("BH_CONV_GEMM");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}
double GemmMinOps() {
  static const double v = [] {
    const char* e = std::getenv("BH_CONV_GEMM_MIN_GOP");
    return e ? std::atof(e) * 1e9 : 1.2e9;
  }();
  return v;
}

enum Route { kDirect, kStem, kXs, kRows, kMfma, kGemm, kGemmBig, kStemMfma };

Route route(const bh_conv_params& p, long M, int K, int N) {
  const bool is1x1 = p.k_h == 1 && p.k_w == 1 && p.pad_h == 0 && p.pad_w == 0;
  if (p.out_img_stride) return kMfma;  // only conv_mfma_kernel's epilogue stores strided images
  // RGB-stem-like layers (tiny K, byte-granular gather): direct VALU kernel
  if (!is1x1 && K <= 64 && p.in_c < 8) {
    const bool stem = p.k_h == 3 && p.k_w == 3 && p.in_c == 3 && p.dil_w == 1 && N % 8 == 0 && !p.residual;
    if (!stem || std::getenv("BH_CONV_NO_STEM")) return kDirect;
    // the window x filter contraction on MFMA (conv_stem_mfma.hip); the VALU
    // form when forced (BH_CONV_STEM_VALU) or outside the MFMA form's range
    return bh_conv_stem_mfma_ok(p) ? kStemMfma : kStem;
  }
  const bool aligned = (((uintptr_t)p.output | (uintptr_t)p.residual | (uintptr_t)p.input) & 3) == 0;
  // LDS-staged GEMM: int8 activations (glds cannot apply the uint8 XOR),
  // symmetric filters (no row sums), 16-byte K chunks
  const bool gemm_ok = is1x1 && p.stride_h == 1 && p.stride_w == 1 && p.in_xor == 0 && p.w_zp == 0 &&
                       K % 16 == 0 && aligned && ((uintptr_t)p.input & 15) == 0;
  // (the 256-row GEMM tiles go first where K and N are both wide: there the
  // layer is MFMA work, not an activation stream)
  const bool big_first = gemm_ok && GemmMode() > 0 && K >= 128 && N >= 128 && bh_conv_gemm_big_config(M, N) != 0;
  if (is1x1 && p.stride_h == 1 && p.stride_w == 1 && N % 4 == 0 && K % 4 == 0 && aligned && p.kernel_hint == 0 &&
      !big_first) {
    if (K <= 320 && M >= XsMinM()) return kXs;
    if (RowsMinM() >= 0 && M >= RowsMinM()) return kRows;
  }
  if (p.kernel_hint == BH_CONV_MFMA) return kMfma;
  if (p.kernel_hint == BH_CONV_GEMM) return gemm_ok ? kGemm : kMfma;
  if (p.kernel_hint == BH_CONV_GEMM_BIG) return gemm_ok ? kGemmBig : kMfma;
  // the 256-row tiles once the layer fills the chip with them (B = 32 / 256 passes)
  if (gemm_ok && GemmMode() > 0 && bh_conv_gemm_big_config(M, N) != 0) return kGemmBig;
  if (gemm_ok && GemmMode() > 0 && (GemmMode() == 2 || 2.0 * M * N * K >= GemmMinOps())) return kGemm;
  return kMfma;
}
}  // namespace

extern "C" const char* bh_conv2d_i8_kernel(const bh_conv_params* p) {
  if (!p) return "";
  static const char* const names[] = {"conv_direct_kernel", "conv_stem_kernel", "conv_xs_kernel",
                                      "conv_rows_kernel", "conv_mfma_kernel", "conv_gemm_kernel",
                                      "conv_gemm_big_kernel", "conv_stem_mfma_kernel"};
  const long M = (long)p->batch * p->out_h * p->out_w;
  const Route r = route(*p, M, p->k_h * p->k_w * p->in_c, p->out_c);
  if (r == kStem) return bh_conv_stem_kernel_name(*p, (int)M);
  return names[r];
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

extern "C" int bh_conv_group_ok(const bh_conv_params* pp) {
  if (!pp) return 0;
  const bh_conv_params& p = *pp;
  const long M = (long)p.batch * p.out_h * p.out_w;
  const int K = p.k_h * p.k_w * p.in_c;
  const int N = p.out_c;
  if (M <= 0 || M > INT32_MAX || K <= 0 || N <= 0 || p.k_pad < K || p.n_pad < N || (p.k_pad % 64) ||
      (p.n_pad % 64) || !p.input || !p.output || !p.weights || !p.bias_eff || !p.mult || !p.shift ||
      p.stride_h <= 0 || p.stride_w <= 0 || p.in_c % 16)
    return 0;
  return route(p, M, K, N) == kMfma ? 1 : 0;
}

extern "C" size_t bh_conv_group_table_bytes(int n) {
  return n > 0 && n <= bh::kConvGroupMax ? (size_t)n * sizeof(bh::ConvGroupMember) : 0;
}

extern "C" int bh_conv_group_plan(const bh_conv_params* members, int n, void* host_table, bh_conv_group* g) {
  if (!members || !host_table || !g || n < 1 || n > bh::kConvGroupMax) return BH_EINVAL;
  auto* tab = static_cast<bh::ConvGroupMember*>(host_table);
  int is1x1 = -1;
  long blocks = 0;
  for (int i = 0; i < n; ++i) {
    const bh_conv_params& p = members[i];
    if (!bh_conv_group_ok(&p)) return BH_EINVAL;
    const int one = p.k_h == 1 && p.k_w == 1 && p.pad_h == 0 && p.pad_w == 0;
    if (is1x1 >= 0 && one != is1x1) return BH_EINVAL;  // one instantiation per group
    is1x1 = one;
    bh::ConvGroupMember e{};
    e.p = p;
    e.M = p.batch * p.out_h * p.out_w;
    e.K = p.k_h * p.k_w * p.in_c;
    e.N = p.out_c;
    e.dv.out_w = bh::FastDiv(p.out_w);
    e.dv.out_h = bh::FastDiv(p.out_h);
    e.dv.in_c = bh::FastDiv(p.in_c);
    e.dv.k_w = bh::FastDiv(p.k_w);
    const int ksteps = (e.K + 63) / 64;
    // conv_mfma_kernel's forms by size: deep K splits K over the 4 waves of
    // a 16 x 16 (form 0) or, with >= 256 such workgroups, 32 x 32 tile
    // (form 2); shallow K takes 32 x 32 tiles over 2 x 2 waves (form 1) or
    // 64 x 64 ones (form 3) once those give >= 256 workgroups
    if (ksteps >= 3)
      e.form = bh::wgs(e.M, e.N, 32, 32) >= 256 ? 2 : 0;
    else
      e.form = bh::wgs(e.M, e.N, 64, 64) >= 256 ? 3 : 1;
    const int tm = e.form == 0 ? 16 : (e.form == 3 ? 64 : 32), tn = tm;
    e.kchunk = (e.form == 0 || e.form == 2) ? (ksteps + 3) / 4 * 64 : ksteps * 64;
    e.gn = (e.N + tn - 1) / tn;
    e.blocks = ((e.M + tm - 1) / tm) * e.gn;
    e.blk0 = (int)blocks;
    blocks += e.blocks;
    tab[i] = e;
  }
  if (blocks <= 0 || blocks > INT32_MAX / 2) return BH_EINVAL;
  g->n = n;
  g->blocks = (int)blocks;
  g->is1x1 = is1x1;
  return 0;
}

extern "C" int bh_conv_group_i8(const bh_conv_group* g, bh_stream_t stream) {
  if (!g || !g->table || g->n < 1 || g->n > bh::kConvGroupMax || g->blocks < 1) {
    bh_set_last_error("bh_conv_group_i8: invalid group");
    return BH_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  bh::ConvGroupArgs a{};
  a.tab = static_cast<const bh::ConvGroupMember*>(g->table);
  a.n = g->n;
  if (g->is1x1)
    BH_LAUNCH((bh::conv_group_kernel<true>), dim3(g->blocks), dim3(256), 0, s, a);
  else
    BH_LAUNCH((bh::conv_group_kernel<false>), dim3(g->blocks), dim3(256), 0, s, a);
  return bh_check_launch("conv_group_kernel");
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
    case kGemm: return bh::launch_gemm_shape(p, M, K, s);
    case kGemmBig: return bh_conv_gemm_big_launch(p, M, K, s);
    case kStemMfma: return bh_conv_stem_mfma_launch(p, M, s);
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
