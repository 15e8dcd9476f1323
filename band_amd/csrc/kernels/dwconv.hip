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
#include <climits>
#include <cstdlib>

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
  FastDiv runs_w;  // run kernel: ceil(out_w / 4) runs of 4 output pixels per row
  int xcd;  // 1: XCD-contiguous workgroup order (xcd_block)
};

template <int CV>
__global__ __launch_bounds__(256) void dwconv3x3_kernel(bh_dwconv_params p, int total, DwDivs dv) {
  constexpr int NW = CV / 4;
  const int blk = dv.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int idx = blk * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int pix = dv.groups.div(idx);
  const int c0 = (idx - pix * (int)dv.groups.d) * CV;
  const int t = dv.out_w.div(pix);
  const int ox = pix - t * p.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
  // 32-bit offsets (tensor sizes < 2^31, checked by the launcher): no
  // 64-bit multiplies in the address math
  const uint8_t* in = (const uint8_t*)p.input + (n * p.in_h * p.in_w * p.in_c + c0);
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
      Vec<CV>::ld(wt + tap * p.out_c, wv[tap]);
      if (ok[tap]) Vec<CV>::ld(in + (y * p.in_w + x) * p.in_c, xv[tap]);
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
  Vec<CV>::st((uint8_t*)p.output + (((n * p.out_h + oy) * p.out_w + ox) * p.out_c + c0), packed);
}

// 3x3 / dm 1 with the host-packed tap table (bh_pack_dw_taps): the nine
// per-channel products are summed with v_dot4_i32_i8 instead of 36 byte
// extracts and multiply-adds per 4 channels.  The tap dwords a thread loads
// hold 4 CHANNELS of one tap; two 4x4 byte transposes (8 v_perm_b32 each)
// turn taps 0-3 and 4-7 into dwords holding 4 TAPS of one channel, which
// dot with that channel's packed filter dwords; tap 8 dots untransposed
// against a filter dword carrying w[8][c] in byte c % 4 only.  Out-of-image
// taps read as the input zero point, so (x - zp_in) vanishes for them
// exactly as TFLite's skipped taps do, and the zero-point terms fold into
// the table's bias:
//   sum (x - zx)(w - zw) = sum x*w - zw * sum x - zx * sum w + 9 * zx * zw.
template <int CV, bool FAST, bool WZP>
__global__ __launch_bounds__(256) void dwconv3x3_dot_kernel(bh_dwconv_params p, int total, DwDivs dv) {
  constexpr int NW = CV / 4;
  const int blk = dv.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int idx = blk * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int pix = dv.groups.div(idx);
  const int c0 = (idx - pix * (int)dv.groups.d) * CV;
  const int t = dv.out_w.div(pix);
  const int ox = pix - t * p.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
  const uint8_t* base = (const uint8_t*)p.input;
  const uint8_t* in = base + (n * p.in_h * p.in_w * p.in_c + c0);
  const uint32_t xorw = splat_byte(p.in_xor);
  const uint32_t zfill = splat_byte(p.in_zp);
  const int y0 = oy * p.stride_h - p.pad_h;
  const int x0 = ox * p.stride_w - p.pad_w;

  // all nine tap loads issue before any arithmetic; out-of-image taps load
  // from the tensor base (always readable) and are replaced afterwards
  uint32_t xv[9][NW];
#pragma unroll
  for (int fy = 0; fy < 3; ++fy) {
#pragma unroll
    for (int fx = 0; fx < 3; ++fx) {
      const int tap = fy * 3 + fx;
      const int y = y0 + fy * p.dil_h;
      const int x = x0 + fx * p.dil_w;
      const bool ok = y >= 0 && y < p.in_h && x >= 0 && x < p.in_w;
      Vec<CV>::ld(ok ? in + (y * p.in_w + x) * p.in_c : base, xv[tap]);
#pragma unroll
      for (int d = 0; d < NW; ++d) xv[tap][d] = ok ? xv[tap][d] ^ xorw : zfill;
    }
  }
  const v4i* tp = (const v4i*)p.taps + c0;
  uint32_t packed[NW];
#pragma unroll
  for (int d = 0; d < NW; ++d) {
    uint32_t T[4], U[4];
    {
      const uint32_t l01 = __builtin_amdgcn_perm(xv[1][d], xv[0][d], 0x05010400u);
      const uint32_t h01 = __builtin_amdgcn_perm(xv[1][d], xv[0][d], 0x07030602u);
      const uint32_t l23 = __builtin_amdgcn_perm(xv[3][d], xv[2][d], 0x05010400u);
      const uint32_t h23 = __builtin_amdgcn_perm(xv[3][d], xv[2][d], 0x07030602u);
      T[0] = __builtin_amdgcn_perm(l23, l01, 0x05040100u);
      T[1] = __builtin_amdgcn_perm(l23, l01, 0x07060302u);
      T[2] = __builtin_amdgcn_perm(h23, h01, 0x05040100u);
      T[3] = __builtin_amdgcn_perm(h23, h01, 0x07060302u);
    }
    {
      const uint32_t l01 = __builtin_amdgcn_perm(xv[5][d], xv[4][d], 0x05010400u);
      const uint32_t h01 = __builtin_amdgcn_perm(xv[5][d], xv[4][d], 0x07030602u);
      const uint32_t l23 = __builtin_amdgcn_perm(xv[7][d], xv[6][d], 0x05010400u);
      const uint32_t h23 = __builtin_amdgcn_perm(xv[7][d], xv[6][d], 0x07030602u);
      U[0] = __builtin_amdgcn_perm(l23, l01, 0x05040100u);
      U[1] = __builtin_amdgcn_perm(l23, l01, 0x07060302u);
      U[2] = __builtin_amdgcn_perm(h23, h01, 0x05040100u);
      U[3] = __builtin_amdgcn_perm(h23, h01, 0x07060302u);
    }
    const v4i mm = *(const v4i*)(p.mult + c0 + 4 * d);
    const v4i ss = *(const v4i*)(p.shift + c0 + 4 * d);
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const v4i w = tp[4 * d + j];  // filter taps 0-3, 4-7, 8 (byte j), folded bias
      int32_t acc = __builtin_amdgcn_sdot4((int)T[j], w.x, w.w, false);
      acc = __builtin_amdgcn_sdot4((int)U[j], w.y, acc, false);
      acc = __builtin_amdgcn_sdot4((int)xv[8][d], w.z, acc, false);
      if constexpr (WZP) {
        int32_t sx = __builtin_amdgcn_sdot4((int)T[j], 0x01010101, 0, false);
        sx = __builtin_amdgcn_sdot4((int)U[j], 0x01010101, sx, false);
        sx = __builtin_amdgcn_sdot4((int)xv[8][d], (int)(1u << (8 * j)), sx, false);
        acc -= p.w_zp * sx;
      }
      int32_t r = requant_out<FAST>(acc, chan_q(mm[j], ss[j], p.out_zp), p.out_zp, p.act_min, p.act_max);
      const uint32_t byte = p.out_table ? ((const uint8_t*)p.out_table)[(uint8_t)r] : ((uint32_t)r & 0xffu);
      o |= byte << (8 * j);
    }
    packed[d] = o;
  }
  Vec<CV>::st((uint8_t*)p.output + (((n * p.out_h + oy) * p.out_w + ox) * p.out_c + c0), packed);
}

// dot4 kernel, run form (dil 1 with stride S in {1, 2}, or dil D = 2 with
// stride 1): a thread owns a RUN of
// 4 horizontally adjacent output pixels x CV channels.  The run's input
// columns (3 + 3*S) are loaded once and shared by its pixels' windows
// (18 / 27 loads for 4 pixels instead of 36), and the channel operands -
// tap table entries, multipliers, shifts - once per run instead of per
// pixel.  rocprofv3 on the per-pixel form (56x56x144, batch 64) showed it
// texture-unit bound (TA busy ~60%, waves parked on vmcnt 86% of their
// cycles) with 33 bytes of L1 traffic per output byte; the run form needs
// about 10.
template <int CV, int S, int D, bool FAST, bool WZP>
__global__ __launch_bounds__(256) void dwconv3x3_run_kernel(bh_dwconv_params p, int total, DwDivs dv) {
  constexpr int NW = CV / 4;
  constexpr int PX = 4;
  constexpr int NCOL = 1 + 2 * D + (PX - 1) * S;  // input columns of the run (dilation D)
  const int blk = dv.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int idx = blk * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int run = dv.groups.div(idx);
  const int c0 = (idx - run * (int)dv.groups.d) * CV;
  const int t = dv.runs_w.div(run);
  const int ox0 = (run - t * (int)dv.runs_w.d) * PX;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
  const uint8_t* base = (const uint8_t*)p.input;
  const uint32_t xorw = splat_byte(p.in_xor);
  const uint32_t zfill = splat_byte(p.in_zp);
  const int y0 = oy * S - p.pad_h;
  const int x0 = ox0 * S - p.pad_w;
  // 32-bit offsets (tensor sizes < 2^31, checked by the launcher), one
  // multiply per row: the columns step by in_c
  const int rstride = p.in_w * p.in_c;
  const int off0 = n * p.in_h * rstride + y0 * rstride + x0 * p.in_c + c0;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, p.batch * p.in_h * rstride, 0x00020000);

  uint32_t X[3][NCOL][NW];
#pragma unroll
  for (int fy = 0; fy < 3; ++fy) {
    const int y = y0 + fy * D;
    const bool yok = y >= 0 && y < p.in_h;
#pragma unroll
    for (int col = 0; col < NCOL; ++col) {
      const int x = x0 + col;
      const bool ok = yok && x >= 0 && x < p.in_w;
      const int off = off0 + fy * D * rstride + col * p.in_c;
      if constexpr (CV == 4) {
        // raw buffer load: 32-bit offset, no 64-bit address math and no
        // address select - an out-of-image tap's offset may be anything
        // (negative ones are out of range and read 0); it is replaced below
        X[fy][col][0] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0);
      } else {
        Vec<CV>::ld(ok ? base + off : base, X[fy][col]);
      }
#pragma unroll
      for (int d = 0; d < NW; ++d) X[fy][col][d] = ok ? X[fy][col][d] ^ xorw : zfill;
    }
  }
  v4i tab[CV];
#pragma unroll
  for (int j = 0; j < CV; ++j) tab[j] = ((const v4i*)p.taps)[c0 + j];
  int32_t mu[CV], sh[CV];
#pragma unroll
  for (int d = 0; d < NW; ++d) {
    const v4i mm = *(const v4i*)(p.mult + c0 + 4 * d);
    const v4i ss = *(const v4i*)(p.shift + c0 + 4 * d);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mu[4 * d + j] = mm[j];
      sh[4 * d + j] = ss[j];
    }
  }
  const uint8_t* otab = (const uint8_t*)p.out_table;
  uint8_t* out = (uint8_t*)p.output + (((n * p.out_h + oy) * p.out_w + ox0) * p.out_c + c0);
#pragma unroll
  for (int px = 0; px < PX; ++px) {
    if (ox0 + px >= p.out_w) break;
    uint32_t packed[NW];
#pragma unroll
    for (int d = 0; d < NW; ++d) {
      // window taps (fy, fx) in row-major order: 0-3, 4-7 transposed, 8 as is
#define TAP(k) X[(k) / 3][px * S + ((k) % 3) * D][d]
      uint32_t T[4], U[4];
      {
        const uint32_t l01 = __builtin_amdgcn_perm(TAP(1), TAP(0), 0x05010400u);
        const uint32_t h01 = __builtin_amdgcn_perm(TAP(1), TAP(0), 0x07030602u);
        const uint32_t l23 = __builtin_amdgcn_perm(TAP(3), TAP(2), 0x05010400u);
        const uint32_t h23 = __builtin_amdgcn_perm(TAP(3), TAP(2), 0x07030602u);
        T[0] = __builtin_amdgcn_perm(l23, l01, 0x05040100u);
        T[1] = __builtin_amdgcn_perm(l23, l01, 0x07060302u);
        T[2] = __builtin_amdgcn_perm(h23, h01, 0x05040100u);
        T[3] = __builtin_amdgcn_perm(h23, h01, 0x07060302u);
      }
      {
        const uint32_t l01 = __builtin_amdgcn_perm(TAP(5), TAP(4), 0x05010400u);
        const uint32_t h01 = __builtin_amdgcn_perm(TAP(5), TAP(4), 0x07030602u);
        const uint32_t l23 = __builtin_amdgcn_perm(TAP(7), TAP(6), 0x05010400u);
        const uint32_t h23 = __builtin_amdgcn_perm(TAP(7), TAP(6), 0x07030602u);
        U[0] = __builtin_amdgcn_perm(l23, l01, 0x05040100u);
        U[1] = __builtin_amdgcn_perm(l23, l01, 0x07060302u);
        U[2] = __builtin_amdgcn_perm(h23, h01, 0x05040100u);
        U[3] = __builtin_amdgcn_perm(h23, h01, 0x07060302u);
      }
      const uint32_t x8 = TAP(8);
#undef TAP
      uint32_t o = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const v4i w = tab[4 * d + j];
        int32_t acc = __builtin_amdgcn_sdot4((int)T[j], w.x, w.w, false);
        acc = __builtin_amdgcn_sdot4((int)U[j], w.y, acc, false);
        acc = __builtin_amdgcn_sdot4((int)x8, w.z, acc, false);
        if constexpr (WZP) {
          int32_t sx = __builtin_amdgcn_sdot4((int)T[j], 0x01010101, 0, false);
          sx = __builtin_amdgcn_sdot4((int)U[j], 0x01010101, sx, false);
          sx = __builtin_amdgcn_sdot4((int)x8, (int)(1u << (8 * j)), sx, false);
          acc -= p.w_zp * sx;
        }
        const int32_t r =
            requant_out<FAST>(acc, chan_q(mu[4 * d + j], sh[4 * d + j], p.out_zp), p.out_zp, p.act_min, p.act_max);
        const uint32_t byte = otab ? otab[(uint8_t)r] : ((uint32_t)r & 0xffu);
        o |= byte << (8 * j);
      }
      packed[d] = o;
    }
    Vec<CV>::st(out + px * p.out_c, packed);
  }
}

// Depthwise 3x3 on the int8 matrix cores (depth multiplier 1, C % 16 == 0).
// For one 16-channel group the depthwise layer is a GEMM whose K = taps x
// channels and whose filter matrix is block diagonal: one
// v_mfma_i32_16x16x64_i8 contracts 4 taps x 16 channels of 16 pixels, so
// three of them (taps 0-3, 4-7, 8) produce a 16-pixel x 16-channel tile.  A
// lane's pixel fragment is the 16 channel bytes of one tap: ONE 16-byte
// load from NHWC, and no byte transposes (the dot4 forms spend 16
// v_perm_b32 per pixel and channel quad on them).  Computed transposed
// (D^T = W x X^T, as conv_xs_kernel) so a lane ends with 4 consecutive
// channels of one pixel and stores them as one dword.  The filter fragments
// are 15/16 zeros - the matrix cores do 16x the useful MACs - but at three
// MFMAs per 256 outputs that is far below the epilogue's VALU work.
//
// Out-of-image taps read the input zero point; the zero-point terms fold
// into the tap table's bias word (bh_pack_dw_taps, word 3) exactly as for
// the dot4 kernels, and uint8 filters (w_zp != 0) take the per-pixel sum of
// the nine taps from a second MFMA against a block-diagonal ones matrix:
//   sum (x - zx)(w - zw) = sum x*w - zw * sum x + (bias word - bias).
// A wave owns RB x 16 pixels of one channel group; channel groups are the
// fastest-varying wave index, so a workgroup's waves share input lines.
template <int RB, bool FAST, bool WZP>
__global__ __launch_bounds__(256) void dwconv3x3_mfma_kernel(bh_dwconv_params p, int P, int nblocks, DwDivs dv) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const int blk = dv.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int wv = blk * 4 + (threadIdx.x >> 6);
  const int pb = dv.groups.div(wv);  // pixel block
  if (pb >= nblocks) return;
  const int cg = wv - pb * (int)dv.groups.d;  // 16-channel group
  const int C = p.out_c;
  const int c0 = cg * 16;

  // filter fragments of K-steps s = 0..2 (taps 4s..4s+3 x channels c0..+15):
  // W^T row r16 holds w[tap][c0 + r16] in byte r16 and zeros elsewhere
  v4i wf[3], of[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int tap = 4 * s + g;
    const uint32_t wb = tap < 9 ? (uint32_t)(uint8_t)p.weights[tap * C + c0 + r16] : 0u;
    const uint32_t w = wb << (8 * (r16 & 3));
    const uint32_t o = (tap < 9 ? 1u : 0u) << (8 * (r16 & 3));
    const int d = r16 >> 2;
    wf[s] = (v4i){d == 0 ? (int)w : 0, d == 1 ? (int)w : 0, d == 2 ? (int)w : 0, d == 3 ? (int)w : 0};
    of[s] = (v4i){d == 0 ? (int)o : 0, d == 1 ? (int)o : 0, d == 2 ? (int)o : 0, d == 3 ? (int)o : 0};
  }
  // this lane's tap of each K-step, as an offset from the window origin
  int tdy[3], tdx[3];
  bool tok[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int tap = 4 * s + g;
    const int fy = (tap * 11) >> 5;  // tap / 3 for tap < 12
    const int fx = tap - 3 * fy;
    tdy[s] = fy * p.dil_h - p.pad_h;
    tdx[s] = fx * p.dil_w - p.pad_w;
    tok[s] = tap < 9;
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.input, (short)0, p.batch * p.in_h * p.in_w * C, 0x00020000);
  const uint32_t xorw = splat_byte(p.in_xor);
  const int zfill = (int)splat_byte(p.in_zp);

  // every pixel fragment load of the wave issues before the first MFMA
  v4i xf[RB][3];
  int mpix[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    const int m = (pb * RB + b) * 16 + r16;
    mpix[b] = m;
    const bool valid = m < P;
    const int mm = valid ? m : 0;
    const int t = dv.out_w.div(mm);
    const int ox = mm - t * p.out_w;
    const int n = dv.out_h.div(t);
    const int oy = t - n * p.out_h;
    const int iy = oy * p.stride_h, ix = ox * p.stride_w, row0 = n * p.in_h;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int y = iy + tdy[s], x = ix + tdx[s];
      const bool ok = valid && tok[s] && y >= 0 && y < p.in_h && x >= 0 && x < p.in_w;
      const int off = ok ? ((row0 + y) * p.in_w + x) * C + c0 : 0;
      const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
      xf[b][s] = (v4i){ok ? (int)(v.x ^ xorw) : zfill, ok ? (int)(v.y ^ xorw) : zfill,
                       ok ? (int)(v.z ^ xorw) : zfill, ok ? (int)(v.w ^ xorw) : zfill};
    }
  }
  // epilogue operands of this lane's 4 output channels
  const int co = c0 + 4 * g;
  const v4i* tp = (const v4i*)p.taps;
  const v4i mm4 = *(const v4i*)(p.mult + co);
  const v4i ss4 = *(const v4i*)(p.shift + co);
  int32_t be[4];
  ChanQ q[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    be[r] = tp[co + r].w;
    q[r] = chan_q(mm4[r], ss4[r], p.out_zp);
  }
  const uint8_t* otab = (const uint8_t*)p.out_table;
  uint8_t* out = (uint8_t*)p.output;
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    v4i acc = (v4i){0, 0, 0, 0};
    v4i sx = (v4i){0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(wf[s], xf[b][s], acc, 0, 0, 0);
      if constexpr (WZP) sx = __builtin_amdgcn_mfma_i32_16x16x64_i8(of[s], xf[b][s], sx, 0, 0, 0);
    }
    if (mpix[b] >= P) continue;
    int32_t v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int32_t a = acc[r] + be[r];
      if constexpr (WZP) a -= p.w_zp * sx[r];
      v[r] = requant_out<FAST>(a, q[r], p.out_zp, p.act_min, p.act_max);
      if (otab) v[r] = otab[(uint8_t)v[r]];
    }
    const uint32_t lo = __builtin_amdgcn_perm((uint32_t)v[1], (uint32_t)v[0], 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm((uint32_t)v[3], (uint32_t)v[2], 0x04000c0cu);
    *(uint32_t*)(out + mpix[b] * C + co) = lo | hi;
  }
}

// general filter size / depth multiplier: one output channel per thread
__global__ __launch_bounds__(256) void dwconv_generic_kernel(bh_dwconv_params p, int total, DwDivs dv) {
  const int blk = dv.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int idx = blk * blockDim.x + threadIdx.x;
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
  dv.xcd = 1;
  return dv;
}

template <int CV, int S, int D>
static void launch_run(const bh_dwconv_params& p, hipStream_t s) {
  const int runs_w = (p.out_w + 3) / 4;
  const int total = (int)((long)p.batch * p.out_h * runs_w * (p.out_c / CV));
  DwDivs dv = dw_divs(p, p.out_c / CV);
  dv.runs_w = FastDiv(runs_w);
  const dim3 grid((unsigned)((total + 255) / 256));
  if (p.w_zp != 0) {
    if (p.requant_fast) BH_LAUNCH((dwconv3x3_run_kernel<CV, S, D, true, true>), grid, dim3(256), 0, s, p, total, dv);
    else BH_LAUNCH((dwconv3x3_run_kernel<CV, S, D, false, true>), grid, dim3(256), 0, s, p, total, dv);
  } else {
    if (p.requant_fast) BH_LAUNCH((dwconv3x3_run_kernel<CV, S, D, true, false>), grid, dim3(256), 0, s, p, total, dv);
    else BH_LAUNCH((dwconv3x3_run_kernel<CV, S, D, false, false>), grid, dim3(256), 0, s, p, total, dv);
  }
}

// pixel tile rows per wave: 4 (64 pixels) when that still gives >= 2048
// waves, else 1
static int mfma_rb(const bh_dwconv_params& p) {
  const long P = (long)p.batch * p.out_h * p.out_w;
  return ((P + 63) / 64) * (p.out_c / 16) >= 2048 ? 4 : 1;
}

template <int RB>
static void launch_mfma(const bh_dwconv_params& p, hipStream_t s) {
  const int P = p.batch * p.out_h * p.out_w;
  const int nblocks = (P + RB * 16 - 1) / (RB * 16);
  const int groups = p.out_c / 16;
  const long waves = (long)nblocks * groups;
  DwDivs dv = dw_divs(p, groups);
  const dim3 grid((unsigned)((waves + 3) / 4));
  if (p.w_zp != 0) {
    if (p.requant_fast) BH_LAUNCH((dwconv3x3_mfma_kernel<RB, true, true>), grid, dim3(256), 0, s, p, P, nblocks, dv);
    else BH_LAUNCH((dwconv3x3_mfma_kernel<RB, false, true>), grid, dim3(256), 0, s, p, P, nblocks, dv);
  } else {
    if (p.requant_fast) BH_LAUNCH((dwconv3x3_mfma_kernel<RB, true, false>), grid, dim3(256), 0, s, p, P, nblocks, dv);
    else BH_LAUNCH((dwconv3x3_mfma_kernel<RB, false, false>), grid, dim3(256), 0, s, p, P, nblocks, dv);
  }
}

// the MFMA kernel's shapes: tap table, 3x3 dm 1, C % 16 == 0, any stride /
// dilation
static bool mfma_ok(const bh_dwconv_params& p) { return p.taps && p.out_c % 16 == 0; }

// the run kernel's shapes: tap table, dil 1, equal strides 1 / 2
static bool run_ok(const bh_dwconv_params& p) {
  // dil 1 with stride 1 / 2, or dil 2 with stride 1 (DeepLab's atrous layers)
  return p.taps && p.dil_h == p.dil_w && p.stride_h == p.stride_w &&
         ((p.dil_h == 1 && (p.stride_h == 1 || p.stride_h == 2)) || (p.dil_h == 2 && p.stride_h == 1));
}

template <int CV>
static void launch3x3(const bh_dwconv_params& p, long pixels, hipStream_t s) {
  const int total = (int)(pixels * (p.out_c / CV));
  const dim3 grid((unsigned)((total + 255) / 256));
  const DwDivs dv = dw_divs(p, p.out_c / CV);
  if (!p.taps) {
    BH_LAUNCH(dwconv3x3_kernel<CV>, grid, dim3(256), 0, s, p, total, dv);
  } else if (p.w_zp != 0) {
    if (p.requant_fast) BH_LAUNCH((dwconv3x3_dot_kernel<CV, true, true>), grid, dim3(256), 0, s, p, total, dv);
    else BH_LAUNCH((dwconv3x3_dot_kernel<CV, false, true>), grid, dim3(256), 0, s, p, total, dv);
  } else {
    if (p.requant_fast) BH_LAUNCH((dwconv3x3_dot_kernel<CV, true, false>), grid, dim3(256), 0, s, p, total, dv);
    else BH_LAUNCH((dwconv3x3_dot_kernel<CV, false, false>), grid, dim3(256), 0, s, p, total, dv);
  }
}

}  // namespace bh

namespace {
enum DwRoute { kRun1, kRun2, kRunD2, kDot16, kDot8, kDot4, kTap16, kTap8, kTap4, kGeneric, kMfma };

// MFMA form from this many 16x16 output tiles (BH_DW_MFMA_MIN_TILES; the
// round-2 default was 4096).  Off by default since round 3: the VALU run
// form is faster on the standalone depthwise layers of the batch-24 C3 mix
// (64 layers unfused: 397 vs 510 us; default fused tree: kernel sum 1432 vs
// 1447 us, PoseNet -13.5 us; profiles/r03aw_dwab_*), and it keeps MFMA on
// the dense contractions.  kernel_hint BH_DW_MFMA still forces it.
long MfmaMinTiles() {
  static const long v = [] {
    const char* e = std::getenv("BH_DW_MFMA_MIN_TILES");
    return e ? std::atol(e) : LONG_MAX;
  }();
  return v;
}

DwRoute dw_route(const bh_dwconv_params& p) {
  const long pixels = (long)p.batch * p.out_h * p.out_w;
  const bool fast = p.depth_multiplier == 1 && p.k_h == 3 && p.k_w == 3 && p.out_c % 4 == 0;
  if (!fast) return kGeneric;
  // forced forms (when the shape allows them)
  if (p.kernel_hint == BH_DW_MFMA && bh::mfma_ok(p)) return kMfma;
  if (p.kernel_hint == BH_DW_RUN && bh::run_ok(p))
    return p.dil_h == 2 ? kRunD2 : (p.stride_h == 1 ? kRun1 : kRun2);
  if (p.kernel_hint == BH_DW_DOT && p.taps) {
    if (p.out_c % 16 == 0) return kDot16;
    return p.out_c % 8 == 0 ? kDot8 : kDot4;
  }
  if (bh::mfma_ok(p) && (pixels + 15) / 16 * (p.out_c / 16) >= MfmaMinTiles()) return kMfma;
  // run kernel (4 channels x 4 pixels per thread) once the grid has >= ~40k
  // threads: measured 1.5-1.9x faster than the per-pixel kernels from there
  // (MobileNetV2 depthwise layers, batch 16 / 64); below it, at batch 1, the
  // per-pixel kernels' shorter per-thread chains win
  if (bh::run_ok(p) && (long)p.batch * p.out_h * ((p.out_w + 3) / 4) * (p.out_c / 4) >= 40000)
    return p.dil_h == 2 ? kRunD2 : (p.stride_h == 1 ? kRun1 : kRun2);
  // per-pixel kernels: widest vector that still leaves enough threads to fill the chip
  const int base = p.taps ? kDot16 : kTap16;
  if (p.out_c % 16 == 0 && pixels * (p.out_c / 16) >= 65536) return (DwRoute)base;
  if (p.out_c % 8 == 0 && pixels * (p.out_c / 8) >= 32768) return (DwRoute)(base + 1);
  return (DwRoute)(base + 2);
}
}  // namespace

extern "C" const char* bh_dwconv2d_i8_kernel(const bh_dwconv_params* p) {
  if (!p) return "";
  switch (dw_route(*p)) {
    case kRun1: case kRun2: case kRunD2: return "dwconv3x3_run_kernel";
    case kMfma: return "dwconv3x3_mfma_kernel";
    case kDot16: case kDot8: case kDot4: return "dwconv3x3_dot_kernel";
    case kTap16: case kTap8: case kTap4: return "dwconv3x3_kernel";
    default: return "dwconv_generic_kernel";
  }
}

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
  if (pixels * p.out_c >= INT32_MAX || (long)p.batch * p.in_h * p.in_w * p.in_c >= INT32_MAX) {
    bh_set_last_error("bh_dwconv2d_i8: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  const bool fast = p.depth_multiplier == 1 && p.k_h == 3 && p.k_w == 3 && p.out_c % 4 == 0;
  if (p.taps && !fast) {
    bh_set_last_error("bh_dwconv2d_i8: a tap table needs a 3x3, depth multiplier 1, out_c % 4 == 0 layer");
    return BH_EINVAL;
  }
  switch (dw_route(p)) {
    case kMfma:
      if (bh::mfma_rb(p) == 4) bh::launch_mfma<4>(p, s);
      else bh::launch_mfma<1>(p, s);
      break;
    case kRun1: bh::launch_run<4, 1, 1>(p, s); break;
    case kRun2: bh::launch_run<4, 2, 1>(p, s); break;
    case kRunD2: bh::launch_run<4, 1, 2>(p, s); break;
    case kDot16: case kTap16: bh::launch3x3<16>(p, pixels, s); break;
    case kDot8: case kTap8: bh::launch3x3<8>(p, pixels, s); break;
    case kDot4: case kTap4: bh::launch3x3<4>(p, pixels, s); break;
    case kGeneric: {
      const int total = (int)(pixels * p.out_c);
      BH_LAUNCH(bh::dwconv_generic_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, total,
                         bh::dw_divs(p, p.out_c));
      break;
    }
  }
  return bh_check_launch("dwconv_kernel");
}

extern "C" int bh_pack_dw_taps(const int8_t* w, int c, const int32_t* bias, int32_t in_zp, int32_t w_zp,
                               int32_t* taps) {
  if (!w || !taps || c <= 0 || c % 4) {
    bh_set_last_error("bh_pack_dw_taps: invalid parameters");
    return BH_EINVAL;
  }
  for (int ch = 0; ch < c; ++ch) {
    uint32_t d[3] = {0, 0, 0};
    int32_t wsum = 0;
    for (int tap = 0; tap < 9; ++tap) {
      const int8_t v = w[(long)tap * c + ch];
      wsum += v;
      if (tap < 8) d[tap / 4] |= (uint32_t)(uint8_t)v << (8 * (tap % 4));
      else d[2] = (uint32_t)(uint8_t)v << (8 * (ch % 4));
    }
    int32_t* o = taps + 4L * ch;
    o[0] = (int32_t)d[0];
    o[1] = (int32_t)d[1];
    o[2] = (int32_t)d[2];
    o[3] = (bias ? bias[ch] : 0) - in_zp * wsum + 9 * in_zp * w_zp;
  }
  return 0;
}
