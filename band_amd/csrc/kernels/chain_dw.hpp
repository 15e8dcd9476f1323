// Phase A of the raster chain forms (chain_kernel in fused_chain.hip, the
// staged form in chain_stage.hip): DEPTHWISE_CONV_2D 3x3 of one 16-pixel
// block on the matrix cores, requantised into the LDS tile [pixel][C].
// Stands in for TFLite 2.9.2 reference_integer_ops::DepthwiseConvPerChannel
// (Band's hot path band/backend/tfl/model_executor.cc:249-255 ->
// Interpreter::Invoke); bit-identical to dwconv3x3_mfma_kernel.
#pragma once

#include "common.hpp"

namespace bh {

struct ChainDivs {
  FastDiv out_w, out_h;
};

// The block-diagonal MFMA tile: one v_mfma_i32_16x16x64_i8 contracts 3 taps x
// 16 channels of 16 pixels per K-step (filter row s); this lane's pixel is
// `m` (valid when mval), its 4 result rows start at `orow` of the LDS tile
// `dl` (row stride S1); the wave takes channel groups wsub, wsub + WPB, ...,
// DA of them per memory round trip.
template <bool FAST, int DA, int WPB>
__device__ __forceinline__ void chain_dw_mfma(const bh_dwconv_params& d, const ChainDivs& dv, int m, bool mval,
                                              int lane, int r16, int g, int wsub, unsigned char* dl, int S1,
                                              int orow) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const int C = d.out_c;
  const int mm = mval ? m : 0;
  const int t = dv.out_w.div(mm);
  const int ox = mm - t * d.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * d.out_h;
  const int iy = oy * d.stride_h, ix = ox * d.stride_w, row0 = n * d.in_h;
  // K-step s takes filter row s and lane group g filter column g (group
  // 3 idles: zero filter bytes, so its operand bytes do not matter).
  // Column reuse: lane (p, g) reads input column ix + g*dil_w, which is
  // lane (p + dd, 0)'s column when dd = g*dil_w / stride_w is whole and
  // pixel p + dd lies in the same 16-pixel block and output row; such a
  // lane takes that lane's filled tap dwords by ds_bpermute instead of
  // loading them, so only group 0 and the block's edge lanes issue tap
  // loads (a quarter of the texture-path lane accesses at stride 1)
  const int gx = g * d.dil_w;
  const int dd = (g == 1 || g == 2) && gx % d.stride_w == 0 ? gx / d.stride_w : 0;
  const bool borrow = dd > 0 && r16 + dd < 16 && ox + dd < d.out_w;
  const bool need = g < 3 && !borrow;
  const int src4 = (borrow ? r16 + dd : lane) << 2;
  int off[3];
  bool ok[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int y = iy + s * d.dil_h - d.pad_h, x = ix + gx - d.pad_w;
    ok[s] = mval && g < 3 && y >= 0 && y < d.in_h && x >= 0 && x < d.in_w;
    off[s] = ok[s] ? ((row0 + y) * d.in_w + x) * C : 0;
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)d.input, (short)0, d.batch * d.in_h * d.in_w * C, 0x00020000);
  const int zfill = (int)splat_byte(d.in_zp);
  const int dsel = r16 >> 2;
  const int bsh = 8 * (r16 & 3);
  // this lane's filter byte of K-step s, tap 3s + g, in the tap table
  // row (bh_pack_dw_taps): dword tsel[s], bit offset tbit[s]; tap 8
  // sits in byte c % 4 of dword 2
  const int tsel1 = g == 0 ? 0 : 1, tbit1 = g == 0 ? 24 : 8 * (g - 1);
  const int tbit2 = g < 2 ? 8 * (2 + g) : bsh;
  // two channel groups per iteration: both items' loads (input taps,
  // the channel's tap-table row, requantisation operands) are issued
  // before either's MFMAs
  struct DwItem {
    v4i xf[3];
    v4i tw;
    int32_t mu, sh;
  };
  auto dw_load = [&](int cg, DwItem& it) {
    const int c0 = cg * 16;
    v4u v[3] = {};
    if (need) {
#pragma unroll
      for (int s = 0; s < 3; ++s) v[s] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off[s] + c0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < 3; ++s)
      it.xf[s] = (v4i){ok[s] ? (int)v[s].x : zfill, ok[s] ? (int)v[s].y : zfill, ok[s] ? (int)v[s].z : zfill,
                       ok[s] ? (int)v[s].w : zfill};
    const int c = c0 + r16;  // this lane's result channel
    it.tw = *(const v4i*)(d.taps + 4 * c);
    it.mu = d.mult[c];
    it.sh = d.shift[c];
  };
  auto dw_finish = [&](int cg, DwItem& it) {
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) it.xf[s][j] = __builtin_amdgcn_ds_bpermute(src4, it.xf[s][j]);
    const uint32_t t0 = (uint32_t)it.tw.x, t1 = (uint32_t)it.tw.y, t2 = (uint32_t)it.tw.z;
    uint32_t wb[3];
    wb[0] = (t0 >> (8 * g)) & 0xffu;
    wb[1] = ((tsel1 ? t1 : t0) >> tbit1) & 0xffu;
    wb[2] = ((g < 2 ? t1 : t2) >> tbit2) & 0xffu;
    v4i acc = (v4i){it.tw.w, it.tw.w, it.tw.w, it.tw.w};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int w = g < 3 ? (int)(wb[s] << bsh) : 0;
      const v4i wf = (v4i){dsel == 0 ? w : 0, dsel == 1 ? w : 0, dsel == 2 ? w : 0, dsel == 3 ? w : 0};
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(it.xf[s], wf, acc, 0, 0, 0);
    }
    const ChanQ q = chan_q(it.mu, it.sh, d.out_zp);
    int32_t v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[r], q, d.out_zp, d.act_min, d.act_max);
    stage4(dl, S1, orow, cg * 16 + r16, v);  // one ds_write_b32 per lane (common.hpp)
  };
  // DA channel groups per round: every item's loads (input taps, filter
  // bytes, epilogue operands) are issued before any item's MFMAs, so a
  // wave pays one global round trip per DA groups
  const int G = C >> 4;
  for (int cg = wsub; cg < G; cg += DA * WPB) {
    DwItem it[DA];
#pragma unroll
    for (int u = 0; u < DA; ++u) dw_load(cg + u * WPB < G ? cg + u * WPB : cg, it[u]);
#pragma unroll
    for (int u = 0; u < DA; ++u)
      if (u == 0 || cg + u * WPB < G) dw_finish(cg + u * WPB, it[u]);
  }
}

}  // namespace bh
