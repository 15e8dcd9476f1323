// Fused pointwise chain for gfx950 (int8 per-channel):
//   DEPTHWISE_CONV_2D 3x3 -> CONV_2D 1x1 [-> ADD residual] [-> CONV_2D 1x1]
//
// Stands in for 2-3 consecutive TFLite 2.9.2 builtin kernels on Band's hot
// path (band/backend/tfl/model_executor.cc:249-255 -> Interpreter::Invoke):
// reference_integer_ops::DepthwiseConvPerChannel, ConvPerChannel (a
// MobileNetV2 block's project, with the block's residual ADD folded into its
// epilogue, or a MobileNetV1 pointwise layer) and ConvPerChannel again (the
// NEXT block's expand).  Every intermediate is requantised to its own 8-bit
// tensor exactly as TFLite stores it, so the result is bit-identical to the
// unfused launches.
//
// Why this cut and not the inverted-residual block (irb_kernel): the two 1x1
// layers map output pixel m to pixel m, so fusing across the block boundary
// (project -> next expand) needs no halo and no recompute.  Only the
// depthwise layer reads a 3x3 neighbourhood, and it reads it straight from
// HBM / L2 (neighbouring pixel blocks of a workgroup share an XCD).  Per
// MobileNet block that is one launch instead of three, and the depthwise
// output - 6x the block's channels - never leaves the CU.
//
// A workgroup (4 waves) owns RB x 16 consecutive output pixels:
//   phase A  depthwise on the matrix cores (block-diagonal 16x16x64 tiles,
//            as dwconv3x3_mfma_kernel): one 16-channel group per item,
//            requantised, 4 channels of one pixel per lane -> LDS [pix][C]
//   phase B  first 1x1 GEMM, D^T = W1 x X^T with X from LDS, K = C; requant
//            [+ residual ADD]; the 8-bit result -> HBM (when it has other
//            readers) and -> LDS [pix][N1]
//   phase C  second 1x1 GEMM from that LDS tile, K = N1; requant -> HBM
// Waves: wave w works on pixel block w % RB and on every (4/RB)-th channel
// tile from w / RB, so every phase keeps all four waves busy.
#include <algorithm>

#include "chain_dw.hpp"
#include "common.hpp"

namespace bh {

__device__ __forceinline__ uint32_t pack4(const int32_t v[4]) {
  // bytes 0 of v0..v3 -> one dword (v_perm_b32 selectors as in conv_xs_kernel)
  const uint32_t lo = __builtin_amdgcn_perm((uint32_t)v[1], (uint32_t)v[0], 0x0c0c0400u);
  const uint32_t hi = __builtin_amdgcn_perm((uint32_t)v[3], (uint32_t)v[2], 0x04000c0cu);
  return lo | hi;
}

// One 16-channel tile t of the 1x1 layer `c` for this lane's pixel row:
// `xrow` = the row's K bytes in LDS at this lane's 16-byte K offset.  The
// accumulator starts at the folded bias of the lane's 4 channels.  Four
// K-steps' weight fragments (global, L1/L2-resident) and pixel fragments
// (LDS) are issued before their MFMAs.
__device__ __forceinline__ v4i gemm_tile(const bh_conv_params& c, const unsigned char* xrow, int t, int KS, int r16,
                                         int g) {
  const int8_t* wrow = c.weights + (long)(t * 16 + r16) * c.k_pad + g * 16;
  const int nb = t * 16 + 4 * g;
  const int nl = nb < c.out_c ? nb : 0;
  v4i acc = *(const v4i*)(c.bias_eff + nl);
  int k = 0;
  for (; k + 8 <= KS; k += 8) {
    v4i w[8], x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      w[u] = *(const v4i*)(wrow + (k + u) * 64);
      x[u] = *(const v4i*)(xrow + (k + u) * 64);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(w[u], x[u], acc, 0, 0, 0);
  }
  for (; k + 4 <= KS; k += 4) {
    v4i w[4], x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      w[u] = *(const v4i*)(wrow + (k + u) * 64);
      x[u] = *(const v4i*)(xrow + (k + u) * 64);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(w[u], x[u], acc, 0, 0, 0);
  }
  for (; k < KS; ++k) {
    const v4i w = *(const v4i*)(wrow + k * 64);
    const v4i x = *(const v4i*)(xrow + k * 64);
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(w, x, acc, 0, 0, 0);
  }
  return acc;
}

template <bool FAST>
__device__ __forceinline__ void requant4(const bh_conv_params& c, int nb, v4i acc, int32_t v[4]) {
  const v4i vm = *(const v4i*)(c.mult + nb);
  const v4i vs = *(const v4i*)(c.shift + nb);
#pragma unroll
  for (int r = 0; r < 4; ++r)
    v[r] = requant_out<FAST>(acc[r], chan_q(vm[r], vs[r], c.out_zp), c.out_zp, c.act_min, c.act_max);
}

// x-stationary 1x1 GEMM for K <= 64 * KMAX: this lane's KS pixel fragments
// are read from LDS once; the wave then walks its channel tiles t0, t0 +
// tstep, ... two at a time, with both tiles' weight fragments and epilogue
// operands (folded bias, multipliers, shifts) issued before their MFMAs, so
// each pair costs one memory round trip.  epi(t, nb, acc, mult4, shift4)
// finishes a tile (nb = the lane's first channel; may be >= out_c).
template <int KMAX, typename Epi>
__device__ __forceinline__ void gemm_xs(const bh_conv_params& c, const unsigned char* xrow, int KS, int t0, int tstep,
                                        int r16, int g, Epi&& epi) {
  v4i x[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) x[k] = k < KS ? *(const v4i*)(xrow + k * 64) : (v4i){0, 0, 0, 0};
  const int T = (c.out_c + 15) >> 4;
  for (int t = t0; t < T; t += 2 * tstep) {
    const int tb = t + tstep < T ? t + tstep : t;
    const int8_t* ra = c.weights + (long)(t * 16 + r16) * c.k_pad + g * 16;
    const int8_t* rb = c.weights + (long)(tb * 16 + r16) * c.k_pad + g * 16;
    v4i wa[KMAX], wb[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < KS) {
        wa[k] = *(const v4i*)(ra + k * 64);
        wb[k] = *(const v4i*)(rb + k * 64);
      }
    const int na = t * 16 + 4 * g, nb = tb * 16 + 4 * g;
    const int la = na < c.out_c ? na : 0, lb = nb < c.out_c ? nb : 0;
    v4i acca = *(const v4i*)(c.bias_eff + la);
    v4i accb = *(const v4i*)(c.bias_eff + lb);
    const v4i ma = *(const v4i*)(c.mult + la), sa = *(const v4i*)(c.shift + la);
    const v4i mb = *(const v4i*)(c.mult + lb), sb = *(const v4i*)(c.shift + lb);
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < KS) {
        acca = __builtin_amdgcn_mfma_i32_16x16x64_i8(wa[k], x[k], acca, 0, 0, 0);
        accb = __builtin_amdgcn_mfma_i32_16x16x64_i8(wb[k], x[k], accb, 0, 0, 0);
      }
    epi(t, na, acca, ma, sa);
    if (tb != t) epi(tb, nb, accb, mb, sb);
  }
}

template <bool FAST>
__device__ __forceinline__ void requant4m(const bh_conv_params& c, v4i acc, v4i vm, v4i vs, int32_t v[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
    v[r] = requant_out<FAST>(acc[r], chan_q(vm[r], vs[r], c.out_zp), c.out_zp, c.act_min, c.act_max);
}

constexpr int kXsMax = 5;  // x-stationary GEMMs up to K = 320

// Workgroup-contiguous output: the tile's rows are consecutive pixels, so
// its bytes are one contiguous run of HBM; staged in LDS and written with
// 16-byte stores of consecutive addresses (a wave writes 1 KB per
// instruction instead of 16 separate 16-byte row pieces).
__device__ __forceinline__ void copy_out(const unsigned char* src, uint8_t* dst, int bytes) {
  const int n16 = bytes >> 4;
  for (int i = threadIdx.x; i < n16; i += blockDim.x) *(v4i*)(dst + i * 16) = *(const v4i*)(src + i * 16);
  const int rem = (bytes - (n16 << 4)) >> 2;  // bytes % 4 == 0
  if ((int)threadIdx.x < rem)
    *(uint32_t*)(dst + n16 * 16 + threadIdx.x * 4) = *(const uint32_t*)(src + n16 * 16 + threadIdx.x * 4);
}

// A channel slice [c0, c0 + cw) of `rows` staged pixels (row stride Nc)
// to HBM (the split phase C: each workgroup stores its channel tiles)
__device__ __forceinline__ void copy_out_slice(const unsigned char* src, uint8_t* dst, int Nc, int c0, int cw,
                                               int rows) {
  const bool v16 = ((c0 | cw | Nc) & 15) == 0;
  const int u = v16 ? cw >> 4 : cw >> 2;  // units per pixel (cw % 4 == 0)
  const float rcp = 1.0f / (float)u;
  for (int i = threadIdx.x; i < rows * u; i += blockDim.x) {
    const int r = (int)(((float)i + 0.5f) * rcp);
    const int k = i - r * u;
    const long o = (long)r * Nc + c0;
    if (v16) *(v4i*)(dst + o + k * 16) = *(const v4i*)(src + o + k * 16);
    else *(uint32_t*)(dst + o + k * 4) = *(const uint32_t*)(src + o + k * 4);
  }
}

// The non-persistent chain computes every GEMM UNtransposed, D = X W^T:
// lane (r16, g) of v_mfma_i32_16x16x64_i8 ends with D[4g + r][r16], i.e.
// FOUR PIXELS of ONE channel.  The channel's requantisation constants
// (ChanQ: a 64-bit rounding constant, shifts, masks) are then derived once
// for 4 values instead of once per value, and the results go to the LDS
// staging tiles as bytes (no packing); the HBM stores stay the contiguous
// 16-byte copy_out.  The operand fragments are the same bytes as the
// transposed form's: only the MFMA operand order changes.
template <int KB = 4>
__device__ __forceinline__ v4i gemm_tile_nt(const bh_conv_params& c, const unsigned char* xrow, int t, int KS,
                                            int r16, int g) {
  const int8_t* wrow = c.weights + (long)(t * 16 + r16) * c.k_pad + g * 16;
  const int n = t * 16 + r16;
  const int be = c.bias_eff[n < c.out_c ? n : 0];
  v4i acc = (v4i){be, be, be, be};
  // KB K-steps' filter fragments are issued before any of their MFMAs (a
  // ragged last batch included): K <= 64 * KB costs one L2 round trip
  // instead of one per K-step
  for (int k = 0; k < KS; k += KB) {
    v4i w[KB], x[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (k + u < KS) {
        w[u] = *(const v4i*)(wrow + (k + u) * 64);
        x[u] = *(const v4i*)(xrow + (k + u) * 64);
      }
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (k + u < KS) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(x[u], w[u], acc, 0, 0, 0);
  }
  return acc;
}

// x-stationary form of gemm_tile_nt for K <= 64 * KMAX: TT channel tiles
// per memory round trip (every tile's filter fragments and epilogue
// operands issued before their MFMAs); epi(t, n, acc, mult, shift)
// finishes a tile for this lane's channel n (may be >= out_c).
template <int KMAX, int TT = 2, typename Epi>
__device__ __forceinline__ void gemm_xs_nt(const bh_conv_params& c, const unsigned char* xrow, int KS, int t0,
                                           int tstep, int r16, int g, Epi&& epi, int t_end = -1) {
  v4i x[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) x[k] = k < KS ? *(const v4i*)(xrow + k * 64) : (v4i){0, 0, 0, 0};
  const int T = t_end >= 0 ? t_end : (c.out_c + 15) >> 4;
  for (int t = t0; t < T; t += TT * tstep) {
    int tt[TT], nn[TT], mu[TT], sh[TT];
    v4i w[TT][KMAX], acc[TT];
#pragma unroll
    for (int u = 0; u < TT; ++u) {
      tt[u] = t + u * tstep < T ? t + u * tstep : t;  // past the end: a duplicate, not finished
      const int8_t* r = c.weights + (long)(tt[u] * 16 + r16) * c.k_pad + g * 16;
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < KS) w[u][k] = *(const v4i*)(r + k * 64);
      nn[u] = tt[u] * 16 + r16;
      const int l = nn[u] < c.out_c ? nn[u] : 0;
      const int b = c.bias_eff[l];
      mu[u] = c.mult[l];
      sh[u] = c.shift[l];
      acc[u] = (v4i){b, b, b, b};
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < KS) {
#pragma unroll
        for (int u = 0; u < TT; ++u) acc[u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x[k], w[u][k], acc[u], 0, 0, 0);
      }
#pragma unroll
    for (int u = 0; u < TT; ++u)
      if (u == 0 || tt[u] != t) epi(tt[u], nn[u], acc[u], mu[u], sh[u]);
  }
}

// RB == 4 form of gemm_xs_nt: wave w takes channel tiles w, w+4, ... for
// ALL 64 pixels of the workgroup (4 pixel blocks), so a tile's filter
// fragments, folded bias and requantisation constants serve 16 values per
// lane instead of 4 (the conv_xs_kernel amortisation).  epi(n, acc[4], mult,
// shift) finishes channel n for the 4 pixel blocks.
template <int KMAX, typename Epi>
__device__ __forceinline__ void gemm_xs4_nt(const bh_conv_params& c, const unsigned char* base, int stride, int KS,
                                            int wave, int r16, int g, Epi&& epi, int t_begin = 0, int t_end = -1) {
  v4i x[4][KMAX];
#pragma unroll
  for (int pb = 0; pb < 4; ++pb)
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      x[pb][k] = k < KS ? *(const v4i*)(base + (pb * 16 + r16) * stride + g * 16 + k * 64) : (v4i){0, 0, 0, 0};
  const int T = t_end >= 0 ? t_end : (c.out_c + 15) >> 4;
  for (int t = t_begin + wave; t < T; t += 4) {
    const int n = t * 16 + r16;
    const int nl = n < c.out_c ? n : 0;
    const int8_t* wrow = c.weights + (long)(t * 16 + r16) * c.k_pad + g * 16;
    v4i w[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < KS) w[k] = *(const v4i*)(wrow + k * 64);
    const int be = c.bias_eff[nl], mu = c.mult[nl], sh = c.shift[nl];
    v4i acc[4];
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) acc[pb] = (v4i){be, be, be, be};
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < KS) {
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) acc[pb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x[pb][k], w[k], acc[pb], 0, 0, 0);
      }
    epi(n, acc, mu, sh);
  }
}

// BH_CHAIN_WPE (build-time A-B switch): ask the register allocator for at
// least that many waves per SIMD on the raster chain forms
#ifdef BH_CHAIN_WPE
#define BH_CHAIN_OCC __attribute__((amdgpu_waves_per_eu(BH_CHAIN_WPE)))
#else
#define BH_CHAIN_OCC
#endif
// VAR: compile-time form variants, so the default instantiation carries no
// code of the others (built as runtime branches they cost 1-3.6 us per
// launch on every chain at batch 24, profiles/r05m_*): bit 1 = the phase-C
// channel split over grid.y
template <int RB, bool FAST, int KX, int NW, bool AM, int DA = 2, int VAR = 0>
__global__ __launch_bounds__(NW * 64) BH_CHAIN_OCC void chain_kernel(bh_chain_params cp, int P, int S1, int S2, int off_pl, int off_o1,
                                                    int off_add, ChainDivs dv) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned long long t_entry = __builtin_amdgcn_s_memtime();  // before any kernarg load
  constexpr int WPB = NW / RB;  // waves per pixel block
  // channel tiles per round of the x-stationary 1x1 GEMMs (more when the
  // K fragments are few); the deep form (DA > 2) takes more as well
  constexpr int TTC = DA > 2 ? (KX <= 2 ? 6 : 3) : 2;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const int pb = wave % RB;
  const int wsub = wave / RB;
  const int blk = xcd_block(blockIdx.x, gridDim.x);
  const int m0 = blk * RB * 16;
  const int rows = min(RB * 16, P - m0);
  const int m = m0 + pb * 16 + r16;  // this lane's pixel as an A-operand row
  const bool mval = m < P;
  unsigned char* dl = smem;           // [RB*16][S1] depthwise output; then [RB*16][N2] second 1x1 output
  unsigned char* pl = smem + off_pl;  // [RB*16][S2] first 1x1 output (second 1x1's operand)
  unsigned char* o1 = smem + off_o1;  // [RB*16][N1] first 1x1 output staged for HBM
  // residual ADD: add.cc rescales each 8-bit operand on its own
  // (MultiplyByQuantizedMultiplierSmallerThanOneExp of (q + offset) << 20),
  // so both rescalings are 256-entry tables, built once per workgroup
  int* add_tab = (int*)(smem + off_add);  // [0, 256): first conv's output, [256, 512): residual
  if (cp.pw1.residual) {
    const bh_conv_params& a = cp.pw1;
    for (int i = threadIdx.x; i < 512; i += NW * 64) {
      const int q = (i & 255) - 128;
      add_tab[i] = i < 256 ? requant_lt1((q + a.add_y_off) * (1 << a.add_left_shift), a.add_y_mult, a.add_y_shift)
                           : requant_lt1((q + a.add_r_off) * (1 << a.add_left_shift), a.add_r_mult, a.add_r_shift);
    }
  }
  const int prow = pb * 16 + r16;     // this lane's operand row
  const int orow = pb * 16 + 4 * g;   // first of this lane's 4 result rows
  // diagnostics (tools/tile_probe.py --raster): shader-clock stamps at the
  // phase boundaries, debug_stamps[8 * workgroup]
  unsigned long long* stamps =
      cp.debug_stamps ? (unsigned long long*)cp.debug_stamps + 8 * (long)blockIdx.x : nullptr;
#define CHAIN_STAMP(k) \
  if (stamps && threadIdx.x == 0) stamps[k] = __builtin_amdgcn_s_memtime();
  CHAIN_STAMP(0)
  if (stamps && threadIdx.x == 0) stamps[7] = t_entry;

  // ---- phase A: depthwise 3x3 -> LDS -------------------------------------
  constexpr bool SPLIT = (VAR & 2) != 0;
  chain_dw_mfma<FAST, DA, WPB>(cp.dw, dv, m, mval, lane, r16, g, wsub, dl, S1, orow);
  __syncthreads();
  CHAIN_STAMP(1)

  // ---- phase B: first 1x1 (+ residual ADD) -> LDS (operand) / LDS (staged) -
  {
    const bh_conv_params& a = cp.pw1;
    const int N1 = a.out_c;
    const int T1 = (N1 + 15) >> 4;
    const int KS1 = a.k_pad >> 6;
    const unsigned char* xrow = dl + prow * S1 + g * 16;
    const uint8_t* res = (const uint8_t*)a.residual;
    const bool out1 = a.output != nullptr && (!SPLIT || blockIdx.y == 0);  // split: slice 0 stores it
    auto epi = [&](int t, int n, v4i acc, int mu, int sh) {
      if (n >= N1) return;
      const ChanQ q = chan_q(mu, sh, a.out_zp);
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[r], q, a.out_zp, a.act_min, a.act_max);
      if (res) {
        int32_t rq[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mr = m0 + orow + r;
          rq[r] = mr < P ? (int32_t)(int8_t)res[(long)mr * N1 + n] : 0;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int32_t sy = add_tab[v[r] + 128];
          const int32_t sr = add_tab[256 + rq[r] + 128];
          v[r] = clamp_i32(requant_lt1(sy + sr, a.add_o_mult, a.add_o_shift) + a.add_o_off, a.add_act_min,
                           a.add_act_max);
        }
      }
      if (out1) stage4(o1, N1, orow, n, v);
      if (cp.has_pw2) stage4(pl, S2, orow, n, v);
    };
    if (AM && KS1 <= KX) {
      gemm_xs4_nt<KX>(a, dl, S1, KS1, wave, r16, g, [&](int n, const v4i* acc, int mu, int sh) {
        if (n >= N1) return;
        const ChanQ q = chan_q(mu, sh, a.out_zp);
#pragma unroll
        for (int pb4 = 0; pb4 < 4; ++pb4) {
          const int rb = pb4 * 16 + 4 * g;
          int32_t v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[pb4][r], q, a.out_zp, a.act_min, a.act_max);
          if (res) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int mr = m0 + rb + r;
              const int32_t rq = mr < P ? (int32_t)(int8_t)res[(long)mr * N1 + n] : 0;
              v[r] = clamp_i32(requant_lt1(add_tab[v[r] + 128] + add_tab[256 + rq + 128], a.add_o_mult, a.add_o_shift) +
                                   a.add_o_off,
                               a.add_act_min, a.add_act_max);
            }
          }
          if (out1) stage4(o1, N1, rb, n, v);
          if (cp.has_pw2) stage4(pl, S2, rb, n, v);
        }
      });
    } else if (KS1 <= KX) {
      gemm_xs_nt<KX, TTC>(a, xrow, KS1, wsub, WPB, r16, g, epi);
    } else {
      for (int t = wsub; t < T1; t += WPB) {
        const v4i acc = gemm_tile_nt<(DA > 2 ? 8 : 4)>(a, xrow, t, KS1, r16, g);
        const int n = t * 16 + r16;
        const int nl = n < N1 ? n : 0;
        epi(t, n, acc, a.mult[nl], a.shift[nl]);
      }
    }
  }
  __syncthreads();
  CHAIN_STAMP(2)
  if (cp.pw1.output && (!SPLIT || blockIdx.y == 0))
    copy_out(o1, (uint8_t*)cp.pw1.output + (long)m0 * cp.pw1.out_c, rows * cp.pw1.out_c);
  CHAIN_STAMP(3)
  if (!cp.has_pw2) return;

  // ---- phase C: second 1x1 -> LDS staging (dl, row stride N2) -> HBM ------
  {
    const bh_conv_params& b = cp.pw2;
    const int N2 = b.out_c;
    const int KS2 = b.k_pad >> 6;
    const unsigned char* xrow = pl + prow * S2 + g * 16;
    auto epi4 = [&](int n, const v4i* acc, int mu, int sh) {
      if (n >= N2) return;
      const ChanQ q = chan_q(mu, sh, b.out_zp);
#pragma unroll
      for (int pb4 = 0; pb4 < 4; ++pb4) {
        int32_t v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[pb4][r], q, b.out_zp, b.act_min, b.act_max);
        stage4(dl, N2, pb4 * 16 + 4 * g, n, v);
      }
    };
    auto epi1 = [&](int t, int n, v4i acc, int mu, int sh) {
      if (n >= N2) return;
      const ChanQ q = chan_q(mu, sh, b.out_zp);
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[r], q, b.out_zp, b.act_min, b.act_max);
      stage4(dl, N2, orow, n, v);
    };
    if constexpr (SPLIT) {
      // this workgroup's channel tiles [t_lo, t_hi) (grid.y slices)
      const int T2 = (N2 + 15) >> 4;
      const int t_lo = (int)blockIdx.y * T2 / (int)gridDim.y, t_hi = ((int)blockIdx.y + 1) * T2 / (int)gridDim.y;
      if constexpr (AM) gemm_xs4_nt<KX>(b, pl, S2, KS2, wave, r16, g, epi4, t_lo, t_hi);
      else gemm_xs_nt<KX, TTC>(b, xrow, KS2, t_lo + wsub, WPB, r16, g, epi1, t_hi);
    } else {
      if constexpr (AM) gemm_xs4_nt<KX>(b, pl, S2, KS2, wave, r16, g, epi4);
      else gemm_xs_nt<KX, TTC>(b, xrow, KS2, wsub, WPB, r16, g, epi1);
    }
  }
  __syncthreads();
  CHAIN_STAMP(4)
  if constexpr (!SPLIT) {
    copy_out(dl, (uint8_t*)cp.pw2.output + (long)m0 * cp.pw2.out_c, rows * cp.pw2.out_c);
  } else {
    const int N2 = cp.pw2.out_c;
    const int T2 = (N2 + 15) >> 4;
    const int c_lo = (int)blockIdx.y * T2 / (int)gridDim.y * 16;
    const int c_hi = min(N2, ((int)blockIdx.y + 1) * T2 / (int)gridDim.y * 16);
    if (c_hi > c_lo)
      copy_out_slice(dl, (uint8_t*)cp.pw2.output + (long)m0 * N2, N2, c_lo, c_hi - c_lo, rows);
  }
  CHAIN_STAMP(5)
#undef CHAIN_STAMP
}

// LDS regions of one workgroup: dl (depthwise output, later the second
// 1x1's output), pl (the second 1x1's operand), o1 (the first 1x1's output
// for HBM); all 16-byte aligned
struct ChainLds {
  int S1, S2, off_pl, off_o1, off_add;
  size_t bytes;
};
static ChainLds chain_lds(const bh_chain_params& p) {
  ChainLds L;
  const int rows = p.px_blocks * 16;
  // rows of k_pad + 32 bytes: a ds_read_b128 lane group's 16 rows land on
  // 16 distinct bank slots (S / 16 = 2 mod 4; tools/lds_bank_model.py)
  L.S1 = p.pw1.k_pad + 32;
  L.S2 = p.has_pw2 ? p.pw2.k_pad + 32 : 0;
  const int dl_row = std::max(L.S1, p.has_pw2 ? (p.pw2.out_c + 15) / 16 * 16 : 0);
  L.off_pl = rows * dl_row;
  L.off_o1 = L.off_pl + rows * L.S2;
  L.off_add = L.off_o1 + (p.pw1.output ? rows * ((p.pw1.out_c + 15) / 16 * 16) : 0);
  L.bytes = (size_t)L.off_add + (p.pw1.residual ? 512 * sizeof(int) : 0);
  return L;
}


// ---- persistent form -------------------------------------------------------
// For chains whose filters fit in LDS (the 112x112 .. 28x28 MobileNet blocks
// and the 14x14 ones with narrow projections): a workgroup loads both 1x1
// filters, the depthwise filter and every epilogue table into LDS ONCE, then
// walks a contiguous range of 64-pixel blocks (ranges of one XCD adjacent,
// so depthwise halo rows stay in one L2).  Per block the only global round
// trips are the depthwise input loads - 12 per wave in flight (4 pixel
// blocks x 3 taps of one 16-channel group, as dwconv3x3_mfma_kernel) - and
// the residual reads; both 1x1 GEMMs run from LDS.  Outputs leave through
// the contiguous LDS-staged copy.
struct PersistLds {
  int ws1, ws2, S1, S2;
  int off_w2, off_t1, off_t2, off_dwt, off_dww, off_dl, off_pl, off_o1;
  size_t bytes;
};

__host__ __device__ inline PersistLds persist_lds(const bh_chain_params& p) {
  PersistLds L;
  const int T1 = (p.pw1.out_c + 15) / 16;
  const int T2 = p.has_pw2 ? (p.pw2.out_c + 15) / 16 : 0;
  const int C = p.dw.out_c;
  L.ws1 = p.pw1.k_pad + 16;
  L.ws2 = p.has_pw2 ? p.pw2.k_pad + 16 : 0;
  L.S1 = L.ws1;
  L.S2 = L.ws2;
  size_t o = (size_t)T1 * 16 * L.ws1;  // W1 at 0
  L.off_w2 = (int)o;
  o += (size_t)T2 * 16 * L.ws2;
  L.off_t1 = (int)o;
  o += 12 * (size_t)T1 * 16;
  L.off_t2 = (int)o;
  o += 12 * (size_t)T2 * 16;
  L.off_dwt = (int)o;
  o += 12 * (size_t)C;
  L.off_dww = (int)o;
  o += (9 * (size_t)C + 15) / 16 * 16;
  const int dl_row = L.S1 > (T2 * 16) ? L.S1 : T2 * 16;
  L.off_dl = (int)o;
  o += 64 * (size_t)dl_row;
  L.off_pl = (int)o;
  o += 64 * (size_t)L.S2;
  L.off_o1 = (int)o;
  o += p.pw1.output ? 64 * (size_t)T1 * 16 : 0;
  L.bytes = o;
  return L;
}

template <bool FAST, int KX>
__global__ __launch_bounds__(256) void chain_persist_kernel(bh_chain_params cp, int P, PersistLds L, ChainDivs dv) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const bh_dwconv_params& d = cp.dw;
  const bh_conv_params& a = cp.pw1;
  const bh_conv_params& b = cp.pw2;
  const int C = d.out_c, G = C >> 4;
  const int N1 = a.out_c, T1 = (N1 + 15) >> 4, KS1 = a.k_pad >> 6;
  const int N2 = cp.has_pw2 ? b.out_c : 0, T2 = (N2 + 15) >> 4, KS2 = cp.has_pw2 ? b.k_pad >> 6 : 0;
  unsigned char* W1 = smem;
  unsigned char* W2 = smem + L.off_w2;
  int* t1 = (int*)(smem + L.off_t1);   // bias_eff | mult | shift, T1*16 each (zero past N1)
  int* t2 = (int*)(smem + L.off_t2);
  int* dwt = (int*)(smem + L.off_dwt); // folded bias | mult | shift, C each
  unsigned char* dww = smem + L.off_dww;
  unsigned char* dl = smem + L.off_dl;
  unsigned char* pl = smem + L.off_pl;
  unsigned char* o1 = smem + L.off_o1;

  // ---- prologue: filters and tables -> LDS (once per workgroup) ----------
  {
    const int cpr1 = a.k_pad >> 4;
    for (int i = tid; i < T1 * 16 * cpr1; i += 256) {
      const int r = i / cpr1, c = i - r * cpr1;
      *(v4i*)(W1 + r * L.ws1 + c * 16) = *(const v4i*)(a.weights + (long)r * a.k_pad + c * 16);
    }
    if (cp.has_pw2) {
      const int cpr2 = b.k_pad >> 4;
      for (int i = tid; i < T2 * 16 * cpr2; i += 256) {
        const int r = i / cpr2, c = i - r * cpr2;
        *(v4i*)(W2 + r * L.ws2 + c * 16) = *(const v4i*)(b.weights + (long)r * b.k_pad + c * 16);
      }
    }
    for (int i = tid; i < T1 * 16; i += 256) {
      const bool v = i < N1;
      t1[i] = v ? a.bias_eff[i] : 0;
      t1[T1 * 16 + i] = v ? a.mult[i] : 0;
      t1[2 * T1 * 16 + i] = v ? a.shift[i] : 0;
    }
    for (int i = tid; i < T2 * 16; i += 256) {
      const bool v = i < N2;
      t2[i] = v ? b.bias_eff[i] : 0;
      t2[T2 * 16 + i] = v ? b.mult[i] : 0;
      t2[2 * T2 * 16 + i] = v ? b.shift[i] : 0;
    }
    for (int i = tid; i < C; i += 256) {
      dwt[i] = d.taps[4 * i + 3];
      dwt[C + i] = d.mult[i];
      dwt[2 * C + i] = d.shift[i];
    }
    for (int i = tid; i < 9 * C / 4; i += 256) ((uint32_t*)dww)[i] = ((const uint32_t*)d.weights)[i];
  }
  __syncthreads();

  const int nblocks = (P + 63) >> 6;
  const int logical = xcd_block(blockIdx.x, gridDim.x);
  const int per = (nblocks + gridDim.x - 1) / gridDim.x;
  const int kb0 = logical * per;
  const int kb1 = min(nblocks, kb0 + per);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)d.input, (short)0, d.batch * d.in_h * d.in_w * C, 0x00020000);
  const int zfill = (int)splat_byte(d.in_zp);
  const int dsel = r16 >> 2;
  const int bsh = 8 * (r16 & 3);
  const uint8_t* res = (const uint8_t*)a.residual;
  uint8_t* out1 = (uint8_t*)a.output;

  for (int kb = kb0; kb < kb1; ++kb) {
    const int m0 = kb * 64;
    const int rows = min(64, P - m0);
    // ---- phase A: wave w takes channel groups w, w+4, ... of all 64 pixels
    {
      int off[4][3];
      bool ok[4][3];
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        const int m = m0 + pb * 16 + r16;
        const bool mv = m < P;
        const int mm = mv ? m : 0;
        const int t = dv.out_w.div(mm);
        const int ox = mm - t * d.out_w;
        const int n = dv.out_h.div(t);
        const int oy = t - n * d.out_h;
        const int iy = oy * d.stride_h, ix = ox * d.stride_w, row0 = n * d.in_h;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int tap = 4 * s + g;
          const int fy = (tap * 11) >> 5;
          const int fx = tap - 3 * fy;
          const int y = iy + fy * d.dil_h - d.pad_h, x = ix + fx * d.dil_w - d.pad_w;
          ok[pb][s] = mv && tap < 9 && y >= 0 && y < d.in_h && x >= 0 && x < d.in_w;
          off[pb][s] = ok[pb][s] ? ((row0 + y) * d.in_w + x) * C : 0;
        }
      }
      for (int cg = wave; cg < G; cg += 4) {
        const int c0 = cg * 16;
        v4i xf[4][3];
#pragma unroll
        for (int pb = 0; pb < 4; ++pb)
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off[pb][s] + c0, 0, 0);
            xf[pb][s] = (v4i){ok[pb][s] ? (int)v.x : zfill, ok[pb][s] ? (int)v.y : zfill,
                              ok[pb][s] ? (int)v.z : zfill, ok[pb][s] ? (int)v.w : zfill};
          }
        v4i wf[3];
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int tap = 4 * s + g;
          const uint32_t wb = tap < 9 ? (uint32_t)dww[tap * C + c0 + r16] : 0u;
          const int w = (int)(wb << bsh);
          wf[s] = (v4i){dsel == 0 ? w : 0, dsel == 1 ? w : 0, dsel == 2 ? w : 0, dsel == 3 ? w : 0};
        }
        const int co = c0 + 4 * g;
        const v4i be = *(const v4i*)(dwt + co);
        const v4i mm4 = *(const v4i*)(dwt + C + co);
        const v4i ss4 = *(const v4i*)(dwt + 2 * C + co);
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          v4i acc = be;
#pragma unroll
          for (int s = 0; s < 3; ++s) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(wf[s], xf[pb][s], acc, 0, 0, 0);
          int32_t v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[r] = requant_out<FAST>(acc[r], chan_q(mm4[r], ss4[r], d.out_zp), d.out_zp, d.act_min, d.act_max);
          *(uint32_t*)(dl + (pb * 16 + r16) * L.S1 + co) = pack4(v);
        }
      }
    }
    __syncthreads();

    // ---- phase B: first 1x1 from LDS; wave w takes channel tiles w, w+4,
    // ... for all 64 pixels, so each tile's channel constants (ChanQ) are
    // derived once for 16 values per lane and its filter fragments read once
    {
      int mp[4];
      bool mv[4];
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        mp[pb] = m0 + pb * 16 + r16;
        mv[pb] = mp[pb] < P;
      }
      for (int t = wave; t < T1; t += 4) {
        const unsigned char* wrow = W1 + (t * 16 + r16) * L.ws1 + g * 16;
        const int nb = t * 16 + 4 * g;
        const v4i be = *(const v4i*)(t1 + nb);
        v4i acc[4] = {be, be, be, be};
        for (int k = 0; k < KS1; ++k) {
          const v4i w = *(const v4i*)(wrow + k * 64);
#pragma unroll
          for (int pb = 0; pb < 4; ++pb)
            acc[pb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                w, *(const v4i*)(dl + (pb * 16 + r16) * L.S1 + g * 16 + k * 64), acc[pb], 0, 0, 0);
        }
        if (nb >= N1) continue;
        const v4i vm = *(const v4i*)(t1 + T1 * 16 + nb);
        const v4i vs = *(const v4i*)(t1 + 2 * T1 * 16 + nb);
        ChanQ q[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = chan_q(vm[r], vs[r], a.out_zp);
        uint32_t rq[4];
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) rq[pb] = res && mv[pb] ? *(const uint32_t*)(res + (long)mp[pb] * N1 + nb) : 0u;
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          int32_t v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[pb][r], q[r], a.out_zp, a.act_min, a.act_max);
          if (res) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int32_t qv = sbyte(rq[pb], r);
              const int32_t sy =
                  requant_lt1((v[r] + a.add_y_off) * (1 << a.add_left_shift), a.add_y_mult, a.add_y_shift);
              const int32_t sr =
                  requant_lt1((qv + a.add_r_off) * (1 << a.add_left_shift), a.add_r_mult, a.add_r_shift);
              v[r] = clamp_i32(requant_lt1(sy + sr, a.add_o_mult, a.add_o_shift) + a.add_o_off, a.add_act_min,
                               a.add_act_max);
            }
          }
          const uint32_t pk = pack4(v);
          const int row = pb * 16 + r16;
          if (out1) *(uint32_t*)(o1 + row * N1 + nb) = pk;
          if (cp.has_pw2) *(uint32_t*)(pl + row * L.S2 + nb) = pk;
        }
      }
    }
    __syncthreads();
    if (out1) copy_out(o1, out1 + (long)m0 * N1, rows * N1);
    if (cp.has_pw2) {
      // ---- phase C: second 1x1 from LDS -> dl (row stride N2); the 64
      // pixels' K fragments stay in registers (K <= 64 * KX)
      v4i x[4][KX];
#pragma unroll
      for (int pb = 0; pb < 4; ++pb)
#pragma unroll
        for (int k = 0; k < KX; ++k)
          x[pb][k] = k < KS2 ? *(const v4i*)(pl + (pb * 16 + r16) * L.S2 + g * 16 + k * 64) : (v4i){0, 0, 0, 0};
      for (int t = wave; t < T2; t += 4) {
        const unsigned char* wrow = W2 + (t * 16 + r16) * L.ws2 + g * 16;
        const int nb = t * 16 + 4 * g;
        const v4i be = *(const v4i*)(t2 + nb);
        v4i acc[4] = {be, be, be, be};
#pragma unroll
        for (int k = 0; k < KX; ++k)
          if (k < KS2) {
            const v4i w = *(const v4i*)(wrow + k * 64);
#pragma unroll
            for (int pb = 0; pb < 4; ++pb) acc[pb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(w, x[pb][k], acc[pb], 0, 0, 0);
          }
        if (nb >= N2) continue;
        const v4i vm = *(const v4i*)(t2 + T2 * 16 + nb);
        const v4i vs = *(const v4i*)(t2 + 2 * T2 * 16 + nb);
        ChanQ q[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = chan_q(vm[r], vs[r], b.out_zp);
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          int32_t v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[pb][r], q[r], b.out_zp, b.act_min, b.act_max);
          *(uint32_t*)(dl + (pb * 16 + r16) * N2 + nb) = pack4(v);
        }
      }
      __syncthreads();
      copy_out(dl, (uint8_t*)b.output + (long)m0 * N2, rows * N2);
    }
    __syncthreads();  // dl / o1 are rewritten by the next block
  }
}

template <int RB, bool FAST, int KX, int NW, bool AM, int DA, int VAR>
static void launch_chain_v(const bh_chain_params& p, int P, const ChainLds& L, size_t lds, hipStream_t s) {
  if (lds > 64 * 1024) {
    // opt in to the CU's full 160 KiB of LDS for this instantiation (once per device)
    static thread_local int opted_device = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (opted_device != dev) {
      (void)hipFuncSetAttribute((const void*)chain_kernel<RB, FAST, KX, NW, AM, DA, VAR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      opted_device = dev;
    }
  }
  ChainDivs dv;
  dv.out_w = FastDiv(p.dw.out_w);
  dv.out_h = FastDiv(p.dw.out_h);
  const int blocks = (P + RB * 16 - 1) / (RB * 16);
  const int split = (VAR & 2) ? p.c_split : 1;
  BH_LAUNCH((chain_kernel<RB, FAST, KX, NW, AM, DA, VAR>), dim3(blocks, split), dim3(NW * 64), lds, s, p, P, L.S1,
            L.S2, L.off_pl, L.off_o1, L.off_add, dv);
}

// the split variant on the one- / two-block forms without the amortised
// GEMMs (bh_chain_lds_bytes admits nothing else)
template <int RB, bool FAST, int KX, int NW = 4, bool AM = false, int DA = 2>
static void launch_chain(const bh_chain_params& p, int P, const ChainLds& L, size_t lds, hipStream_t s) {
  if constexpr (DA == 2 && !AM && RB <= 2) {
    if (p.has_pw2 && p.c_split > 1) return launch_chain_v<RB, FAST, KX, NW, AM, DA, 2>(p, P, L, lds, s);
  }
  launch_chain_v<RB, FAST, KX, NW, AM, DA, 0>(p, P, L, lds, s);
}

template <bool FAST, int KX>
static void launch_persist(const bh_chain_params& p, int P, size_t lds, hipStream_t s) {
  static thread_local int opted_device = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (opted_device != dev) {
    (void)hipFuncSetAttribute((const void*)chain_persist_kernel<FAST, KX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    opted_device = dev;
  }
  ChainDivs dv;
  dv.out_w = FastDiv(p.dw.out_w);
  dv.out_h = FastDiv(p.dw.out_h);
  const int nblocks = (P + 63) / 64;
  // workgroups resident per CU (registers and LDS, <= 4), 256 CUs: one
  // wave of workgroups, each taking a contiguous range of pixel blocks
  static thread_local size_t cached_lds = 0;
  static thread_local int cached_per_cu = 1;
  if (cached_lds != lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, chain_persist_kernel<FAST, KX>, 256, lds) != hipSuccess)
      n = 1;
    cached_per_cu = std::max(1, std::min(4, n));
    cached_lds = lds;
  }
  const int per_cu = cached_per_cu;
  const int grid = std::min(nblocks, 256 * per_cu);
  BH_LAUNCH((chain_persist_kernel<FAST, KX>), dim3(grid), dim3(256), lds, s, p, P, persist_lds(p), dv);
}

static bool conv1x1_ok(const bh_conv_params& c, int in_c) {
  return c.k_h == 1 && c.k_w == 1 && c.stride_h == 1 && c.stride_w == 1 && c.pad_h == 0 && c.pad_w == 0 &&
         c.in_c == in_c && c.k_pad == (in_c + 63) / 64 * 64 && c.n_pad >= (c.out_c + 15) / 16 * 16 &&
         c.in_xor == 0 && c.w_zp == 0 && !c.out_table && c.out_c > 0 && c.out_c % 4 == 0 && c.weights &&
         c.bias_eff && c.mult && c.shift;
}

}  // namespace bh

extern "C" size_t bh_chain_lds_bytes(const bh_chain_params* pp) {
  if (!pp) return 0;
  const bh_chain_params& p = *pp;
  const bh_dwconv_params& d = p.dw;
  if (!p.tile && !p.stage) {
    if (p.px_blocks != 1 && p.px_blocks != 2 && p.px_blocks != 4) return 0;
    if (p.waves != 0 && p.waves != 4 && !((p.waves == 8 || p.waves == 16) && p.px_blocks == 1)) return 0;
  }
  if (d.k_h != 3 || d.k_w != 3 || d.depth_multiplier != 1 || d.in_c != d.out_c || d.out_c % 16 || !d.taps ||
      d.in_xor != 0 || d.w_zp != 0 || d.out_table || !d.input || !d.weights || !d.mult || !d.shift ||
      d.batch <= 0 || d.out_h <= 0 || d.out_w <= 0 || d.stride_h <= 0 || d.stride_w <= 0)
    return 0;
  if (!bh::conv1x1_ok(p.pw1, d.out_c)) return 0;
  const long P = (long)d.batch * d.out_h * d.out_w;
  if (p.pw1.batch * p.pw1.out_h * p.pw1.out_w != P) return 0;
  if (p.has_pw2) {
    if (!bh::conv1x1_ok(p.pw2, p.pw1.out_c) || p.pw2.residual || !p.pw2.output ||
        p.pw2.k_pad > 64 * bh::kXsMax)
      return 0;
    if ((long)p.pw2.batch * p.pw2.out_h * p.pw2.out_w != P) return 0;
  } else if (!p.pw1.output) {
    return 0;
  }
  const long widest = std::max<long>(std::max(d.out_c, p.pw1.out_c), p.has_pw2 ? p.pw2.out_c : 0);
  if (P * widest >= INT32_MAX || (long)d.batch * d.in_h * d.in_w * d.in_c >= INT32_MAX) return 0;
  if (p.stage) return bh_chain_stage_lds_bytes(pp);
  if (p.c_split < 0 || p.c_split > 4) return 0;
  if (p.c_split > 1 && (p.tile || p.persist || p.deep || p.px_blocks > 2 || !p.has_pw2 ||
                        (p.pw2.out_c + 15) / 16 < p.c_split))
    return 0;
  if (p.tile) return bh_chain_tile_lds_bytes(pp);
  if (p.deep && (p.persist || !((p.px_blocks == 1 && (p.waves == 0 || p.waves == 4 || p.waves == 8)) ||
                                (p.px_blocks == 2 && (p.waves == 0 || p.waves == 4)))))
    return 0;
  if (p.persist) {
    if (p.px_blocks != 4 || (p.waves != 0 && p.waves != 4)) return 0;
    const size_t bytes = bh::persist_lds(p).bytes;
    return bytes <= 160 * 1024 ? bytes : 0;
  }
  bh::ChainLds L = bh::chain_lds(p);
  return L.bytes <= 160 * 1024 ? L.bytes : 0;
}

extern "C" int bh_chain_i8(const bh_chain_params* pp, bh_stream_t stream) {
  const size_t lds = bh_chain_lds_bytes(pp);
  if (lds == 0) {
    bh_set_last_error("bh_chain_i8: invalid or unsupported parameters");
    return BH_EINVAL;
  }
  const bh_chain_params& p = *pp;
  if (p.stage) return bh_chain_stage_launch(pp, stream);
  if (p.tile) return bh_chain_tile_launch(pp, stream);
  const int P = p.dw.batch * p.dw.out_h * p.dw.out_w;
  const bh::ChainLds L = bh::chain_lds(p);
  const bool fast = p.dw.requant_fast && p.pw1.requant_fast && (!p.has_pw2 || p.pw2.requant_fast);
  hipStream_t s = (hipStream_t)stream;
  // K-steps of the register-resident (x-stationary) GEMMs: 2 when the
  // second 1x1 has K <= 128 (fewer VGPRs, higher occupancy), else 5
  const bool k2 = !p.has_pw2 || p.pw2.k_pad <= 128;
#define BH_CHAIN_CASE(RB)                                                          \
  if (k2) {                                                                        \
    if (fast) bh::launch_chain<RB, true, 2>(p, P, L, lds, s);                     \
    else bh::launch_chain<RB, false, 2>(p, P, L, lds, s);                         \
  } else {                                                                         \
    if (fast) bh::launch_chain<RB, true, bh::kXsMax>(p, P, L, lds, s);            \
    else bh::launch_chain<RB, false, bh::kXsMax>(p, P, L, lds, s);                \
  }
  if (p.persist) {
    if (k2) {
      if (fast) bh::launch_persist<true, 2>(p, P, lds, s);
      else bh::launch_persist<false, 2>(p, P, lds, s);
    } else {
      if (fast) bh::launch_persist<true, bh::kXsMax>(p, P, lds, s);
      else bh::launch_persist<false, bh::kXsMax>(p, P, lds, s);
    }
    return bh_check_launch("chain_persist_kernel");
  }
  if (p.deep) {  // deep-issue forms (DA = 6): px_blocks 1 with 4 or 8 waves, px_blocks 2 with 4
#define BH_DEEP(RB, NW)                                                                      \
  if (k2) {                                                                                  \
    if (fast) bh::launch_chain<RB, true, 2, NW, false, 6>(p, P, L, lds, s);                  \
    else bh::launch_chain<RB, false, 2, NW, false, 6>(p, P, L, lds, s);                      \
  } else {                                                                                   \
    if (fast) bh::launch_chain<RB, true, bh::kXsMax, NW, false, 6>(p, P, L, lds, s);         \
    else bh::launch_chain<RB, false, bh::kXsMax, NW, false, 6>(p, P, L, lds, s);             \
  }
    if (p.px_blocks == 2) {
      BH_DEEP(2, 4)
    } else if (p.waves == 8) {
      BH_DEEP(1, 8)
    } else {
      BH_DEEP(1, 4)
    }
#undef BH_DEEP
    return bh_check_launch("chain_kernel");
  }
  if (p.waves == 16) {  // one 16-pixel block, 16 waves (few-pixel layers)
    if (k2) {
      if (fast) bh::launch_chain<1, true, 2, 16>(p, P, L, lds, s);
      else bh::launch_chain<1, false, 2, 16>(p, P, L, lds, s);
    } else {
      if (fast) bh::launch_chain<1, true, bh::kXsMax, 16>(p, P, L, lds, s);
      else bh::launch_chain<1, false, bh::kXsMax, 16>(p, P, L, lds, s);
    }
    return bh_check_launch("chain_kernel");
  }
  if (p.waves == 8) {  // one 16-pixel block, 8 waves (mid-size layers)
    if (k2) {
      if (fast) bh::launch_chain<1, true, 2, 8>(p, P, L, lds, s);
      else bh::launch_chain<1, false, 2, 8>(p, P, L, lds, s);
    } else {
      if (fast) bh::launch_chain<1, true, bh::kXsMax, 8>(p, P, L, lds, s);
      else bh::launch_chain<1, false, bh::kXsMax, 8>(p, P, L, lds, s);
    }
    return bh_check_launch("chain_kernel");
  }
  // 64-pixel workgroups whose 1x1 layers have enough channel tiles to keep
  // all four waves busy take the amortised form (a wave's channel tile over
  // all 64 pixels; more registers, so only where it pays)
  const int t_main = p.has_pw2 ? (p.pw2.out_c + 15) / 16 : (p.pw1.out_c + 15) / 16;
  if (p.px_blocks == 4 && k2 && t_main >= 8) {
    if (fast) bh::launch_chain<4, true, 2, 4, true>(p, P, L, lds, s);
    else bh::launch_chain<4, false, 2, 4, true>(p, P, L, lds, s);
    return bh_check_launch("chain_kernel");
  }
  switch (p.px_blocks) {
    case 1: BH_CHAIN_CASE(1) break;
    case 2: BH_CHAIN_CASE(2) break;
    default: BH_CHAIN_CASE(4) break;
  }
#undef BH_CHAIN_CASE
  return bh_check_launch("chain_kernel");
}
