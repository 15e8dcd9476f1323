// The fused chain's packed constant block and the LDS-DMA helpers its
// staged forms share (chain_tile.hip: the 2-D tile form; chain_stage.hip: the
// raster form with staged filters).  Device / host inline only.
#pragma once

#include "common.hpp"

namespace bh {

typedef __attribute__((address_space(3))) void lds_ptr_t;

__device__ __forceinline__ void dma16(const void* src, unsigned char* lds_lane0) {
  __builtin_amdgcn_global_load_lds(src, (lds_ptr_t*)lds_lane0, 16, 0, 0);
}
__device__ __forceinline__ void dma4(const void* src, unsigned char* lds_lane0) {
  __builtin_amdgcn_global_load_lds(src, (lds_ptr_t*)lds_lane0, 4, 0, 0);
}

// chunk c (16 bytes) of filter row `row` (R = k_pad / 16 chunks per row)
// sits at chunk swz(row, c, R).  A ds_read_b128 serves 64 lanes in four
// 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32), one 256-byte
// bank row per group; lane (r16, g) reads row 16t + r16 at chunk 4k + g.  The
// XOR spreads each group's 16 reads over the 16 distinct 16-byte bank slots
// for every row stride: R = 4 mod 8 puts rows r16 & 3 in 4 slot classes, R = 8
// mod 16 in 2 and R = 0 mod 16 in 1, and the XOR with (r16 >> 2) & 2, r16 & 7
// or r16 & 15 (within an aligned block of 4, 8 or 16 chunks, so inside the
// row) separates the lanes a class holds (tools/lds_bank_model.py).
__device__ __host__ __forceinline__ int swz_mask(int row, int R) {
  return (R & 15) == 0 ? (row & 15) : ((R & 15) == 8 ? (row & 7) : ((row >> 2) & 2));
}
__device__ __host__ __forceinline__ int swz(int row, int c, int R) { return c ^ swz_mask(row, R); }

// The packed constant block (byte offsets, all multiples of 16):
//   W1 [T1*16][k1] swizzled | b1 m1 s1 [N1] int32 | W2 [T2*16][k2] swizzled |
//   b2 m2 s2 [N2] | dw filter [9][C] | dw mult, shift, folded bias [C]
struct TileBlob {
  int w1, b1, m1, s1, w2, b2, m2, s2, dww, dwm, dws, dwb, bytes;
};

__host__ __device__ inline TileBlob tile_blob(const bh_chain_params& p) {
  TileBlob b{};
  const int C = p.dw.out_c;
  const int N1 = p.pw1.out_c, N2 = p.has_pw2 ? p.pw2.out_c : 0;
  const int T1 = (N1 + 15) / 16, T2 = (N2 + 15) / 16;
  int o = 0;
  b.w1 = o;
  o += T1 * 16 * p.pw1.k_pad;
  b.b1 = o;
  o += 4 * N1;
  b.m1 = o;
  o += 4 * N1;
  b.s1 = o;
  o += 4 * N1;
  b.w2 = o;
  o += p.has_pw2 ? T2 * 16 * p.pw2.k_pad : 0;
  b.b2 = o;
  o += 4 * N2;
  b.m2 = o;
  o += 4 * N2;
  b.s2 = o;
  o += 4 * N2;
  b.dww = o;
  o += 9 * C;
  b.dwm = o;
  o += 4 * C;
  b.dws = o;
  o += 4 * C;
  b.dwb = o;
  o += 4 * C;
  b.bytes = o;  // N % 4 == 0, C % 16 == 0: every piece is a multiple of 16
  return b;
}

}  // namespace bh
