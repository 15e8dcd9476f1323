// The RGB stem's 3x3 x 3-channel window of one output pixel as the
// k-ordered byte stream k = (fy*3 + fx)*3 + ci (27 bytes in seven dwords,
// one zero byte of tail), int8 domain, padding taps = the input zero point:
// three aligned dword loads + v_alignbyte per window row, the byte path
// where the window leaves the image horizontally or the aligned loads
// would run past the tensor.  The gather conv_stem_kernel (conv_direct.hip)
// does inline; chain_tile_kernel's fused-stem prologue uses this copy.
#pragma once
#include "common.hpp"

namespace bh {

// img: this image's first byte; end: one past the tensor; (y0, x0): the
// window's top-left input pixel (may be negative); in_h / in_w: image size
__device__ __forceinline__ void stem_window(const uint8_t* img, const uint8_t* end, int y0, int x0, int dil_h,
                                            int in_h, int in_w, uint32_t in_xor, uint32_t in_zp, uint32_t xw[7]) {
  const uint32_t xorw = splat_byte(in_xor);
  const uint32_t padw = splat_byte(in_zp);
  uint32_t r[3][3];  // row fy: window bytes 0-3, 4-7, 8
  const bool colok = x0 >= 0 && x0 + 3 <= in_w;
#pragma unroll
  for (int fy = 0; fy < 3; ++fy) {
    const int y = y0 + fy * dil_h;
    const bool rowok = y >= 0 && y < in_h;
    const uint8_t* a = img + ((long)y * in_w + x0) * 3;
    const uintptr_t ai = (uintptr_t)a;
    const uint32_t* base = (const uint32_t*)(ai & ~(uintptr_t)3);
    if (rowok && colok && (const uint8_t*)(base + 3) <= end) {
      const uint32_t o = (uint32_t)(ai & 3);
      const uint32_t d0 = base[0], d1 = base[1], d2 = base[2];
      r[fy][0] = __builtin_amdgcn_alignbyte(d1, d0, o) ^ xorw;
      r[fy][1] = __builtin_amdgcn_alignbyte(d2, d1, o) ^ xorw;
      r[fy][2] = ((d2 >> (8 * o)) ^ xorw) & 0xffu;
    } else if (!rowok) {
      r[fy][0] = padw;
      r[fy][1] = padw;
      r[fy][2] = padw & 0xffu;
    } else {
      uint32_t b[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int x = x0 + k / 3;
        b[k] = (x >= 0 && x < in_w) ? (uint32_t)(a[k] ^ (uint8_t)in_xor) : (padw & 0xffu);
      }
      r[fy][0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
      r[fy][1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
      r[fy][2] = b[8];
    }
  }
  xw[0] = r[0][0];
  xw[1] = r[0][1];
  xw[2] = __builtin_amdgcn_perm(r[1][0], r[0][2], 0x06050400u);  // R0[8] R1[0..2]
  xw[3] = __builtin_amdgcn_alignbyte(r[1][1], r[1][0], 3);        // R1[3..6]
  const uint32_t u = __builtin_amdgcn_perm(r[1][2], r[1][1], 0x0c0c0403u);  // R1[7] R1[8] 0 0
  xw[4] = u | (r[2][0] << 16);                                             // .. R2[0] R2[1]
  xw[5] = __builtin_amdgcn_alignbyte(r[2][1], r[2][0], 2);                 // R2[2..5]
  xw[6] = __builtin_amdgcn_alignbyte(r[2][2], r[2][1], 2);                 // R2[6..8] 0
}

// The same window read from input rows staged in LDS (conv_stem_lds_kernel
// with BH_STEM_ROWS): staged row r holds image row iy_lo + r from the
// 16-byte-aligned global address below its first byte, rw words apart, so
// pixel x of row y starts at byte (y - iy_lo) * 4 * rw + (rel_y & 15) + 3x,
// rel_y = the row's byte offset in the tensor (img_rel + y * in_w * 3).
__device__ __forceinline__ void stem_window_lds(const uint32_t* rows, int rw, int iy_lo, int img_rel, int y0, int x0,
                                                int dil_h, int in_h, int in_w, uint32_t in_xor, uint32_t in_zp,
                                                uint32_t xw[7]) {
  const uint32_t xorw = splat_byte(in_xor);
  const uint32_t padw = splat_byte(in_zp);
  const uint8_t* bytes = (const uint8_t*)rows;
  uint32_t r[3][3];
  const bool colok = x0 >= 0 && x0 + 3 <= in_w;
#pragma unroll
  for (int fy = 0; fy < 3; ++fy) {
    const int y = y0 + fy * dil_h;
    if (y < 0 || y >= in_h) {
      r[fy][0] = padw;
      r[fy][1] = padw;
      r[fy][2] = padw & 0xffu;
      continue;
    }
    const int rel = img_rel + y * in_w * 3;
    const int b = (y - iy_lo) * 4 * rw + (rel & 15) + x0 * 3;
    if (colok) {
      const uint32_t* w = rows + (b >> 2);
      const uint32_t o = (uint32_t)(b & 3);
      const uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
      r[fy][0] = __builtin_amdgcn_alignbyte(d1, d0, o) ^ xorw;
      r[fy][1] = __builtin_amdgcn_alignbyte(d2, d1, o) ^ xorw;
      r[fy][2] = ((d2 >> (8 * o)) ^ xorw) & 0xffu;
    } else {
      uint32_t bb[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int x = x0 + k / 3;
        bb[k] = (x >= 0 && x < in_w) ? (uint32_t)(bytes[b + k] ^ (uint8_t)in_xor) : (padw & 0xffu);
      }
      r[fy][0] = bb[0] | bb[1] << 8 | bb[2] << 16 | bb[3] << 24;
      r[fy][1] = bb[4] | bb[5] << 8 | bb[6] << 16 | bb[7] << 24;
      r[fy][2] = bb[8];
    }
  }
  xw[0] = r[0][0];
  xw[1] = r[0][1];
  xw[2] = __builtin_amdgcn_perm(r[1][0], r[0][2], 0x06050400u);
  xw[3] = __builtin_amdgcn_alignbyte(r[1][1], r[1][0], 3);
  const uint32_t u = __builtin_amdgcn_perm(r[1][2], r[1][1], 0x0c0c0403u);
  xw[4] = u | (r[2][0] << 16);
  xw[5] = __builtin_amdgcn_alignbyte(r[2][1], r[2][0], 2);
  xw[6] = __builtin_amdgcn_alignbyte(r[2][2], r[2][1], 2);
}

// One output channel of the stem as a 64-byte LDS record: the filter dwords
// 0..6 of the k-ordered window (and a zero), the folded bias and the
// requantisation constants (ChanQ precomputed).  Every lane of a wave reads
// the same record: four broadcast ds_read_b128.
struct StemChan {
  int32_t w[8];
  int32_t bias, mu, sh, e, emask, zpe, c0lo, c0hi;
};
static_assert(sizeof(StemChan) == 64, "one 64-byte record per channel");

// word j of channel oc's record (weights: the layer's [n_pad][k_pad] filter
// rows; kpw = k_pad / 4)
__device__ __forceinline__ int32_t stem_chan_word(const int32_t* weights, int kpw, const int32_t* bias,
                                                  const int32_t* mult, const int32_t* shift, int32_t out_zp, int oc,
                                                  int j) {
  if (j < 7) return weights[(long)oc * kpw + j];
  if (j == 7) return 0;
  if (j == 8) return bias[oc];
  const ChanQ q = chan_q(mult[oc], shift[oc], out_zp);
  return j == 9 ? q.mu : j == 10 ? q.sh : j == 11 ? q.e : j == 12 ? q.emask : j == 13 ? q.zpe
       : j == 14 ? (int32_t)(uint32_t)(uint64_t)q.c0 : (int32_t)(q.c0 >> 32);
}

// acc = bias + window . filter of one channel record (minus w_zp x the
// window's byte sum for uint8 filters: wzp is wave-uniform), then the
// requantised output value (int8 domain)
template <bool FAST>
__device__ __forceinline__ int32_t stem_chan_eval(const StemChan& k, const uint32_t xw[7], bool wzp,
                                                  int32_t wzp_rowsum, int32_t out_zp, int32_t lo, int32_t hi) {
  const v4i w0 = *(const v4i*)k.w, w1 = *(const v4i*)(k.w + 4);
  const v4i q0 = *(const v4i*)&k.bias, q1 = *(const v4i*)&k.emask;
  int acc = q0.x;
  acc = __builtin_amdgcn_sdot4((int)xw[0], w0.x, acc, false);
  acc = __builtin_amdgcn_sdot4((int)xw[1], w0.y, acc, false);
  acc = __builtin_amdgcn_sdot4((int)xw[2], w0.z, acc, false);
  acc = __builtin_amdgcn_sdot4((int)xw[3], w0.w, acc, false);
  acc = __builtin_amdgcn_sdot4((int)xw[4], w1.x, acc, false);
  acc = __builtin_amdgcn_sdot4((int)xw[5], w1.y, acc, false);
  acc = __builtin_amdgcn_sdot4((int)xw[6], w1.z, acc, false);
  if (wzp) acc -= wzp_rowsum;
  ChanQ q;
  q.mu = q0.y;
  q.sh = q0.z;
  q.e = q0.w;
  q.emask = q1.x;
  q.zpe = q1.y;
  q.c0 = (int64_t)(((uint64_t)(uint32_t)q1.w << 32) | (uint32_t)q1.z);
  return requant_out<FAST>(acc, q, out_zp, lo, hi);
}

}  // namespace bh
