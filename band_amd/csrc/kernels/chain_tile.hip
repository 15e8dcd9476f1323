// Fused pointwise chain, 2-D tile form, for gfx950 (int8 per-channel):
//   DEPTHWISE_CONV_2D 3x3 -> CONV_2D 1x1 [-> ADD residual] [-> CONV_2D 1x1]
//
// The same three TFLite 2.9.2 builtin kernels as chain_kernel
// (fused_chain.hip: reference_integer_ops::DepthwiseConvPerChannel,
// ConvPerChannel [+ the residual ADD folded into its epilogue], ConvPerChannel
// - Band's hot path band/backend/tfl/model_executor.cc:249-255 ->
// Interpreter::Invoke), with every intermediate requantised exactly as
// TFLite stores it, so the results are bit-identical to the unfused launches.
//
// Why a second form.  chain_kernel's workgroup walks raster-contiguous
// pixels and takes its operands straight from memory: the depthwise taps
// two 16-channel groups at a time, the 1x1 filters two channel tiles at a
// time, the residual per value.  Each of those is a dependent global round
// trip, so a workgroup is a chain of 5-10 of them and the kernel is bound
// by that latency, not by bytes or instructions (r03a stall profile: waves
// waiting on memory 36-59 % of their cycles, 4 waves per SIMD).
//
// Here a workgroup owns a TH x TW tile of output pixels of one image and
// starts with ONE burst of LDS-DMA (global_load_lds, no VGPR staging) that
// brings in everything it will read:
//   * the depthwise input patch: the tile + its 3x3 halo, PH rows of PW*C
//     contiguous bytes each;
//   * the residual tile (4-byte units: the tensor is a multiple of 4 bytes);
//   * the chain's constant block, packed once at prepare time
//     (bh_chain_tile_pack): both 1x1 filters, their folded biases and
//     requantisation tables, the depthwise filter and tables - one flat run
//     from one pointer, so the DMA loop keeps no per-segment kernel
//     arguments live (the first version spent ~8k clocks per workgroup
//     re-loading them from the kernarg segment between segments).
// After one wait the three phases run from LDS only:
//   A  depthwise on the matrix cores (block-diagonal 16x16x64 tiles, as
//      dwconv3x3_mfma_kernel), requantised -> LDS [pixel][C]
//   B  first 1x1 GEMM (D = X W^T: a lane holds 4 pixels of one channel, so
//      the channel's requantisation constants serve 4 values), requant
//      [+ residual ADD via two 256-entry tables] -> LDS operand / staging
//   C  second 1x1 GEMM -> LDS staging
// and the tile's rows leave with 16-byte stores (a tile row of TW pixels is
// one contiguous run of HBM).  The halo costs (PH*PW)/(TH*TW) L2 reads per
// input byte (1.56x for 8x8 at stride 1); HBM sees each input byte about
// once because neighbouring tiles run on one XCD (xcd_block).
//
// Filters sit in the packed block with their 16-byte chunks XOR-swizzled
// within each 64-byte K-step, so the 16 rows a ds_read_b128 group touches
// fall on distinct LDS banks (the DMA writes LDS linearly; no padding).
#include <algorithm>
#include <cstring>

#include "chain_blob.hpp"
#include "common.hpp"

namespace bh {

// LDS layout of one workgroup (bytes): the DMA region (patch | residual |
// constant block) first, then the computed regions
struct TileGeom {
  int TH, TW, PH, PW, tiles_x, tiles_y;
  int S1, S2;          // LDS row strides of the dw output / the pw2 operand
  int T1, T2;          // 16-channel tiles of pw1 / pw2
  int patch_ru;        // 16-byte units per patch row (PW*C/16)
  int pmask, plog;     // C/16 - 1 and log2(C/16) when C/16 is a power of 2, else 0 (patch swizzle)
  int res_ru4;         // 4-byte units per residual tile row (TW*N1/4)
  int u_patch;         // 16-byte units of the patch
  int off_res, off_blob, blob_units;
  int off_dl, off_pl, off_o1, off_add, off_out;
  int out_pitch;       // bytes per pixel of the second 1x1's staging (N2, or N2 + 16)
  int o1_pitch;        // the same for the first 1x1's staging (N1, or N1 + 16)
  int buf_bytes;  // patch + residual region
  TileBlob blob;
  size_t bytes;
};

__host__ __device__ inline TileGeom tile_geom(const bh_chain_params& p, int TH, int TW) {
  TileGeom g{};
  const bh_dwconv_params& d = p.dw;
  const int C = d.out_c;
  const int N1 = p.pw1.out_c, N2 = p.has_pw2 ? p.pw2.out_c : 0;
  g.TH = TH;
  g.TW = TW;
  g.PH = (TH - 1) * d.stride_h + 2 * d.dil_h + 1;
  g.PW = (TW - 1) * d.stride_w + 2 * d.dil_w + 1;
  g.tiles_y = (d.out_h + TH - 1) / TH;
  g.tiles_x = (d.out_w + TW - 1) / TW;
  // rows of k_pad + 32 bytes: the 16 rows a ds_read_b128 lane group reads
  // (r16 * S / 16 + g slots) fall on 16 distinct bank slots (S / 16 = 2 mod 4)
  g.S1 = p.pw1.k_pad + 32;
  g.S2 = p.has_pw2 ? p.pw2.k_pad + 32 : 0;
  g.T1 = (N1 + 15) / 16;
  g.T2 = (N2 + 15) / 16;
  g.patch_ru = g.PW * C / 16;
  // patch pixel (py, px) keeps its 16-byte chunk c at chunk c ^ f, f = (3 py +
  // px) & (C/16 - 1): the 16 pixels x taps a ds_read_b128 lane group reads
  // then spread over the bank slots (C = 128: 656 -> 48 modelled extra LDS
  // cycles per wave, tools/lds_bank_model.py); the DMA applies it on the
  // source side, as it writes LDS lane-linearly
  const int m = C / 16;
  g.pmask = (m & (m - 1)) == 0 ? m - 1 : 0;
  g.plog = 0;
  while (g.pmask && (1 << g.plog) < m) ++g.plog;
  g.res_ru4 = p.pw1.residual ? TW * N1 / 4 : 0;
  g.u_patch = g.PH * g.patch_ru;
  const int rows = TH * TW;
  size_t o = (size_t)g.u_patch * 16;
  g.off_res = (int)o;
  o += p.pw1.residual ? (size_t)rows * N1 : 0;
  o = (o + 15) / 16 * 16;
  g.buf_bytes = (int)o;  // the patch + residual buffer
  g.off_blob = (int)o;
  g.blob = tile_blob(p);
  g.blob_units = g.blob.bytes / 16;
  o += g.blob.bytes;
  g.off_dl = (int)o;
  o += (size_t)rows * g.S1;
  g.off_pl = (int)o;
  o += (size_t)rows * g.S2;
  g.off_o1 = (int)o;
  g.o1_pitch = (N1 % 32 == 0) ? N1 + 16 : N1;  // see out_pitch below
  o += p.pw1.output ? (size_t)rows * g.o1_pitch : 0;
  g.off_add = (int)o;
  o += p.pw1.residual ? 512 * 4 : 0;
  // the second 1x1's staging reuses the patch (dead after phase A) when it fits
  // the staged pixels 4 apart (one quad-transposed ds_write_b32 lane pair)
  // sit 4 * pitch bytes apart: pitch = 0 mod 128 puts them on one bank, so
  // such rows get 16 bytes of pad (16-byte multiples keep the copy-out's
  // 16-byte reads aligned)
  g.out_pitch = (N2 % 32 == 0 && N2 > 0) ? N2 + 16 : N2;
  if ((size_t)rows * g.out_pitch <= (size_t)g.u_patch * 16) {
    g.off_out = 0;
  } else {
    g.off_out = (int)o;
    o += (size_t)rows * g.out_pitch;
  }
  g.bytes = (o + 15) / 16 * 16;
  return g;
}

struct TileDivs {
  FastDiv tiles_x, txy, patch_ru, res_ru4;
  int per;     // RUN: consecutive tiles per workgroup
  int ntiles;  // batch x tiles
};

// the staged tile (pixel p at byte p * pitch, pitch = Nc or Nc + pad with
// Nc % 16 == 0) to HBM: tile row i (TW pixels) is the contiguous run at
// pixel (oy0 + i, ox0)
__device__ __forceinline__ void tile_copy_out(const unsigned char* src, uint8_t* out, int Nc, int TH, int TW, int n,
                                              int oy0, int ox0, int OH, int OW, int tid, int nthreads,
                                              int pitch = 0) {
  const int vc = min(TW, OW - ox0);
  const int vr = min(TH, OH - oy0);
  const int rb = vc * Nc;               // valid bytes per tile row (multiple of 4)
  const int cpr = (TW * Nc + 15) >> 4;  // 16-byte chunks per staged row
  // i / cpr without the ~35-instruction integer division: (i + 0.5) / cpr
  // in float is within 2^-20 relative of the quotient, far from the next
  // integer for i < 2^16
  const float rcp = 1.0f / (float)cpr;
  const bool padded = pitch > Nc;
  const int cpp = Nc >> 4;  // padded: 16-byte chunks per pixel
  const float rcpp = padded ? 1.0f / (float)cpp : 0.0f;
  for (int i = tid; i < vr * cpr; i += nthreads) {
    const int r = (int)(((float)i + 0.5f) * rcp);
    const int c = i - r * cpr;
    const int b = c * 16;
    if (b >= rb) continue;
    const unsigned char* s;
    if (padded) {
      const int x = (int)(((float)c + 0.5f) * rcpp);  // pixel of the row; its chunk c - x * cpp
      s = src + (r * TW + x) * pitch + (c - x * cpp) * 16;
    } else {
      s = src + r * TW * Nc + b;
    }
    uint8_t* dst = out + ((long)(n * OH + oy0 + r) * OW + ox0) * Nc + b;
    if (b + 16 <= rb) {
      *(v4i*)dst = *(const v4i*)s;
    } else {
      for (int k = 0; k < rb - b; k += 4) *(uint32_t*)(dst + k) = *(const uint32_t*)(s + k);
    }
  }
}

// Builds the packed constant block (once per chain, at prepare time).
__global__ void chain_tile_pack_kernel(bh_chain_params p, TileBlob B, unsigned char* blob) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;  // 4-byte word of the block
  if (u * 4 >= B.bytes) return;
  const int o = u * 4;
  auto swz_word = [](const bh_conv_params& c, int rel) {  // LDS-image byte offset -> source word
    const int row = rel / c.k_pad, col = rel - row * c.k_pad;
    // the word at LDS chunk col >> 4 holds source chunk swz(row, col >> 4, R)
    // (an XOR: its own inverse)
    return (const uint32_t*)(c.weights + (long)row * c.k_pad + 16 * swz(row, col >> 4, c.k_pad >> 4) + (col & 15));
  };
  uint32_t v;
  if (o < B.b1) v = *swz_word(p.pw1, o - B.w1);
  else if (o < B.m1) v = (uint32_t)p.pw1.bias_eff[(o - B.b1) / 4];
  else if (o < B.s1) v = (uint32_t)p.pw1.mult[(o - B.m1) / 4];
  else if (o < B.w2) v = (uint32_t)p.pw1.shift[(o - B.s1) / 4];
  else if (o < B.b2) v = *swz_word(p.pw2, o - B.w2);
  else if (o < B.m2) v = (uint32_t)p.pw2.bias_eff[(o - B.b2) / 4];
  else if (o < B.s2) v = (uint32_t)p.pw2.mult[(o - B.m2) / 4];
  else if (o < B.dww) v = (uint32_t)p.pw2.shift[(o - B.s2) / 4];
  else if (o < B.dwm) v = *(const uint32_t*)(p.dw.weights + (o - B.dww));
  else if (o < B.dws) v = (uint32_t)p.dw.mult[(o - B.dwm) / 4];
  else if (o < B.dwb) v = (uint32_t)p.dw.shift[(o - B.dws) / 4];
  else v = (uint32_t)p.dw.taps[4 * ((o - B.dwb) / 4) + 3];  // folded bias: word 3 of the tap entry
  *(uint32_t*)(blob + o) = v;
}

// RUN: a workgroup walks dv.per consecutive tiles through ONE patch buffer
// (bh_chain_params.tile 3 / 4): the constant block is staged once per
// workgroup instead of once per tile (for the 112x112 x 32 chain it is 9.2 KB
// against a 3.2 KB patch), and each further tile's patch is DMA'd after the
// previous tile is done
template <int TH, int TW, bool FAST, int KX, bool RUN>
__global__ __launch_bounds__(256) void chain_tile_kernel(bh_chain_params cp, TileGeom G, TileDivs dv) {
  static_assert(TH * TW == 64, "4 pixel blocks of 16");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned long long t_entry = __builtin_amdgcn_s_memtime();  // before any kernarg load
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const bh_dwconv_params& d = cp.dw;
  const bh_conv_params& a = cp.pw1;
  const bh_conv_params& b = cp.pw2;
  const int OH = d.out_h, OW = d.out_w;

  const int logical = xcd_block(blockIdx.x, gridDim.x);
  // this workgroup's tiles: one (grid = batch x tiles), or RUN's run of
  // dv.per consecutive ones (neighbours share their halo rows in one L2)
  const int t_first = RUN ? logical * dv.per : logical;
  const int t_count = RUN ? min(dv.per, dv.ntiles - t_first) : 1;
  if (t_count <= 0) return;
  auto tile_xy = [&](int t, int& n, int& oy0, int& ox0) {
    n = dv.txy.div(t);
    const int rem = t - n * (int)dv.txy.d;
    const int ty = dv.tiles_x.div(rem);
    oy0 = ty * TH;
    ox0 = (rem - ty * G.tiles_x) * TW;
  };
  unsigned long long* stamps =
      cp.debug_stamps ? (unsigned long long*)cp.debug_stamps + 8 * (long)blockIdx.x : nullptr;
#define TILE_STAMP(k) \
  if (stamps && tid == 0) stamps[k] = __builtin_amdgcn_s_memtime();
  TILE_STAMP(0)
  if (stamps && tid == 0) stamps[7] = t_entry;

  // ---- LDS-DMA: patch + residual of a tile into buffer `buf`; the constant
  // block once -----------------------------------------------------------
  auto issue_tile = [&](int t, unsigned char* buf) {
    int n, oy0, ox0;
    tile_xy(t, n, oy0, ox0);
    const int C = d.out_c;
    const int y0 = oy0 * d.stride_h - d.pad_h;  // image coords of patch (0, 0)
    const uint8_t* in = (const uint8_t*)d.input;
    const long in_last = (long)d.batch * d.in_h * d.in_w * C - 16;
    const long row0 = (long)n * d.in_h;
    const long xoff = (long)(ox0 * d.stride_w - d.pad_w) * C;
    for (int base = wave * 64; base < G.u_patch; base += 256) {
      const int u = base + lane;
      if (u < G.u_patch) {
        const int r = dv.patch_ru.div(u);
        const int y = min(max(y0 + r, 0), d.in_h - 1);
        const int q = u - r * G.patch_ru;  // unit within the patch row: pixel q >> plog, chunk q & pmask
        const int f = (3 * r + (q >> G.plog)) & G.pmask;
        long off = (row0 + y) * d.in_w * C + xoff + (q ^ f) * 16;
        off = off < 0 ? 0 : (off > in_last ? in_last : off);
        dma16(in + off, buf + base * 16);
      }
    }
    if (a.residual) {
      const int N1 = a.out_c;
      const uint8_t* res = (const uint8_t*)a.residual;
      const long res_last = (long)a.batch * OH * OW * N1 - 4;
      const int ue = TH * G.res_ru4;
      for (int base = wave * 64; base < ue; base += 256) {
        const int u = base + lane;
        if (u < ue) {
          const int r = dv.res_ru4.div(u);
          const int y = min(oy0 + r, OH - 1);
          long off = ((long)(n * OH + y) * OW + ox0) * N1 + (u - r * G.res_ru4) * 4;
          off = off > res_last ? res_last : off;
          dma4(res + off, buf + G.off_res + base * 4);
        }
      }
    }
  };
  issue_tile(t_first, smem);
  {
    const unsigned char* blob = (const unsigned char*)cp.tile_blob;
    for (int base = wave * 64; base < G.blob_units; base += 256)
      if (base + lane < G.blob_units) dma16(blob + (base + lane) * 16, smem + G.off_blob + base * 16);
  }
  // residual ADD: add.cc rescales each 8-bit operand on its own, so both
  // rescalings are 256-entry tables (built while the DMA is in flight)
  int* add_tab = (int*)(smem + G.off_add);
  if (a.residual) {
    for (int i = tid; i < 512; i += 256) {
      const int q = (i & 255) - 128;
      add_tab[i] = i < 256 ? requant_lt1((q + a.add_y_off) * (1 << a.add_left_shift), a.add_y_mult, a.add_y_shift)
                           : requant_lt1((q + a.add_r_off) * (1 << a.add_left_shift), a.add_r_mult, a.add_r_shift);
    }
  }
  TILE_STAMP(1)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  TILE_STAMP(2)

  const unsigned char* cb = smem + G.off_blob;
  unsigned char* dl = smem + G.off_dl;
  unsigned char* pl = smem + G.off_pl;
  unsigned char* o1 = smem + G.off_o1;
  const int pb = wave;               // this wave's 16-pixel block of the tile
  const int orow = pb * 16 + 4 * g;  // first of this lane's 4 result rows

  for (int it = 0; it < t_count; ++it) {
  if (RUN && it > 0) {
    __syncthreads();  // every read of the previous tile's patch / staging is done
    issue_tile(t_first + it, smem);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  unsigned char* cur = smem;
  const unsigned char* patch = cur;
  const unsigned char* resl = cur + G.off_res;
  // the second 1x1's staging: the current patch (dead after phase A) when it fits
  unsigned char* ol = G.off_out == 0 ? cur : smem + G.off_out;
  int n, oy0, ox0;
  tile_xy(t_first + it, n, oy0, ox0);

  // ---- phase A: depthwise 3x3 from the patch -> dl ------------------------
  {
    const int C = d.out_c, G16 = C >> 4;
    const unsigned char* dww = cb + G.blob.dww;
    const int* dwm = (const int*)(cb + G.blob.dwm);
    const int* dws = (const int*)(cb + G.blob.dws);
    const int* dwb = (const int*)(cb + G.blob.dwb);
    const int p = pb * 16 + r16;     // this lane's pixel as an A-operand row
    const int ti = p / TW, tj = p % TW;
    const int oy = oy0 + ti, ox = ox0 + tj;
    int off[3], tapc[3], pf[3];
    bool ok[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int tap = 4 * s + g;
      const int fy = (tap * 11) >> 5;  // tap / 3 for tap < 12
      const int fx = tap - 3 * fy;
      const int py = ti * d.stride_h + fy * d.dil_h, px = tj * d.stride_w + fx * d.dil_w;
      const int y = oy * d.stride_h - d.pad_h + fy * d.dil_h, x = ox * d.stride_w - d.pad_w + fx * d.dil_w;
      ok[s] = tap < 9 && y >= 0 && y < d.in_h && x >= 0 && x < d.in_w;
      off[s] = tap < 9 ? (py * G.PW + px) * C : 0;  // always a valid patch address
      pf[s] = tap < 9 ? (3 * py + px) & G.pmask : 0;
      tapc[s] = (tap < 9 ? tap : 0) * C + r16;
    }
    const int zfill = (int)splat_byte(d.in_zp);
    const int dsel = r16 >> 2;
    const int bsh = 8 * (r16 & 3);
    const uint32_t tap8 = g == 0 ? 0xffffffffu : 0u;  // k-step 2 holds tap 8 in lane group 0 only
    auto item = [&](int cg, v4i* xf, v4i* wf, int& be, int& mu, int& sh) {
      const int c0 = cg * 16;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const v4i v = *(const v4i*)(patch + off[s] + ((cg ^ pf[s]) << 4));
        xf[s] = ok[s] ? v : (v4i){zfill, zfill, zfill, zfill};
        uint32_t wb = (uint32_t)dww[tapc[s] + c0];
        if (s == 2) wb &= tap8;
        const int w = (int)(wb << bsh);
        wf[s] = (v4i){dsel == 0 ? w : 0, dsel == 1 ? w : 0, dsel == 2 ? w : 0, dsel == 3 ? w : 0};
      }
      be = dwb[c0 + r16];
      mu = dwm[c0 + r16];
      sh = dws[c0 + r16];
    };
    auto finish = [&](int cg, const v4i* xf, const v4i* wf, int be, int mu, int sh) {
      v4i acc = (v4i){be, be, be, be};
#pragma unroll
      for (int s = 0; s < 3; ++s) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(xf[s], wf[s], acc, 0, 0, 0);
      const ChanQ q = chan_q(mu, sh, d.out_zp);
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[r], q, d.out_zp, d.act_min, d.act_max);
      stage4(dl, G.S1, orow, cg * 16 + r16, v);  // one ds_write_b32 per lane (common.hpp)
    };
    // two channel groups per iteration: both items' LDS reads issue first
    int cg = 0;
    for (; cg + 2 <= G16; cg += 2) {
      v4i xa[3], wa[3], xb[3], wb[3];
      int bea, mua, sha, beb, mub, shb;
      item(cg, xa, wa, bea, mua, sha);
      item(cg + 1, xb, wb, beb, mub, shb);
      finish(cg, xa, wa, bea, mua, sha);
      finish(cg + 1, xb, wb, beb, mub, shb);
    }
    if (cg < G16) {
      v4i xa[3], wa[3];
      int bea, mua, sha;
      item(cg, xa, wa, bea, mua, sha);
      finish(cg, xa, wa, bea, mua, sha);
    }
  }
  __syncthreads();
  TILE_STAMP(3)

  // ---- phase B: first 1x1 (+ residual ADD) -> pl (operand) / o1 (staged) ---
  {
    const int N1 = a.out_c;
    const int KS1 = a.k_pad >> 6;
    // the XOR depends on the row only through r16 (rows 16t + r16): one mask
    // per lane for the whole phase
    const int sx1 = swz_mask(r16, a.k_pad >> 4);
    const unsigned char* W1 = cb + G.blob.w1;
    const int* b1 = (const int*)(cb + G.blob.b1);
    const int* m1 = (const int*)(cb + G.blob.m1);
    const int* s1 = (const int*)(cb + G.blob.s1);
    const unsigned char* xrow = dl + (pb * 16 + r16) * G.S1 + g * 16;
    const bool out1 = a.output != nullptr;
    auto epi = [&](int nch, v4i acc) {
      if (nch >= N1) return;
      const ChanQ q = chan_q(m1[nch], s1[nch], a.out_zp);
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[r], q, a.out_zp, a.act_min, a.act_max);
      if (a.residual) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int32_t rq = (int32_t)(int8_t)resl[(orow + r) * N1 + nch];
          v[r] = clamp_i32(requant_lt1(add_tab[v[r] + 128] + add_tab[256 + rq + 128], a.add_o_mult, a.add_o_shift) +
                               a.add_o_off,
                           a.add_act_min, a.add_act_max);
        }
      }
      if (out1) stage4(o1, G.o1_pitch, orow, nch, v);
      if (cp.has_pw2) stage4(pl, G.S2, orow, nch, v);
    };
    // two channel tiles per iteration (their LDS reads issue together)
    for (int t = 0; t < G.T1; t += 2) {
      const bool two = t + 1 < G.T1;
      const int ra = t * 16 + r16, rb = (two ? t + 1 : t) * 16 + r16;
      const unsigned char* wa = W1 + ra * a.k_pad;
      const unsigned char* wb = W1 + rb * a.k_pad;
      const int ba = b1[ra < N1 ? ra : 0], bb = b1[rb < N1 ? rb : 0];
      v4i acca = (v4i){ba, ba, ba, ba}, accb = (v4i){bb, bb, bb, bb};
      for (int k = 0; k < KS1; ++k) {
        const v4i xv = *(const v4i*)(xrow + k * 64);
        const v4i w0 = *(const v4i*)(wa + 16 * ((4 * k + g) ^ sx1));
        const v4i w1 = *(const v4i*)(wb + 16 * ((4 * k + g) ^ sx1));
        acca = __builtin_amdgcn_mfma_i32_16x16x64_i8(xv, w0, acca, 0, 0, 0);
        accb = __builtin_amdgcn_mfma_i32_16x16x64_i8(xv, w1, accb, 0, 0, 0);
      }
      epi(ra, acca);
      if (two) epi(rb, accb);
    }
  }
  __syncthreads();
  TILE_STAMP(4)
  if (a.output) tile_copy_out(o1, (uint8_t*)a.output, a.out_c, TH, TW, n, oy0, ox0, OH, OW, tid, 256, G.o1_pitch);
  if (cp.has_pw2) {

  // ---- phase C: second 1x1 from pl -> ol (staged) -> HBM -------------------
  {
    const int N2 = b.out_c;
    const int KS2 = b.k_pad >> 6;
    const int sx2 = swz_mask(r16, b.k_pad >> 4);
    const unsigned char* W2 = cb + G.blob.w2;
    const int* b2 = (const int*)(cb + G.blob.b2);
    const int* m2 = (const int*)(cb + G.blob.m2);
    const int* s2 = (const int*)(cb + G.blob.s2);
    const unsigned char* xrow = pl + (pb * 16 + r16) * G.S2 + g * 16;
    v4i x[KX];
#pragma unroll
    for (int k = 0; k < KX; ++k) x[k] = k < KS2 ? *(const v4i*)(xrow + k * 64) : (v4i){0, 0, 0, 0};
    auto epi = [&](int nch, v4i acc) {
      if (nch >= N2) return;
      const ChanQ q = chan_q(m2[nch], s2[nch], b.out_zp);
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[r], q, b.out_zp, b.act_min, b.act_max);
      stage4(ol, G.out_pitch, orow, nch, v);
    };
    for (int t = 0; t < G.T2; t += 2) {
      const bool two = t + 1 < G.T2;
      const int ra = t * 16 + r16, rb = (two ? t + 1 : t) * 16 + r16;
      const unsigned char* wa = W2 + ra * b.k_pad;
      const unsigned char* wb = W2 + rb * b.k_pad;
      const int ba = b2[ra < N2 ? ra : 0], bb = b2[rb < N2 ? rb : 0];
      v4i acca = (v4i){ba, ba, ba, ba}, accb = (v4i){bb, bb, bb, bb};
#pragma unroll
      for (int k = 0; k < KX; ++k)
        if (k < KS2) {
          const v4i w0 = *(const v4i*)(wa + 16 * ((4 * k + g) ^ sx2));
          const v4i w1 = *(const v4i*)(wb + 16 * ((4 * k + g) ^ sx2));
          acca = __builtin_amdgcn_mfma_i32_16x16x64_i8(x[k], w0, acca, 0, 0, 0);
          accb = __builtin_amdgcn_mfma_i32_16x16x64_i8(x[k], w1, accb, 0, 0, 0);
        }
      epi(ra, acca);
      if (two) epi(rb, accb);
    }
  }
  __syncthreads();
  TILE_STAMP(5)
  tile_copy_out(ol, (uint8_t*)b.output, b.out_c, TH, TW, n, oy0, ox0, OH, OW, tid, 256, G.out_pitch);
  TILE_STAMP(6)
  }  // has_pw2
  }  // tiles
#undef TILE_STAMP
}

template <int TH, int TW, bool FAST, int KX, bool RUN>
static void launch_tile(const bh_chain_params& p, const TileGeom& G, hipStream_t s) {
  static thread_local int opted_device = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (opted_device != dev) {
    (void)hipFuncSetAttribute((const void*)chain_tile_kernel<TH, TW, FAST, KX, RUN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    opted_device = dev;
  }
  TileDivs dv;
  dv.tiles_x = FastDiv(G.tiles_x);
  dv.txy = FastDiv(G.tiles_x * G.tiles_y);
  dv.patch_ru = FastDiv(G.patch_ru);
  dv.res_ru4 = FastDiv(G.res_ru4 > 0 ? G.res_ru4 : 1);
  dv.ntiles = p.dw.batch * G.tiles_y * G.tiles_x;
  dv.per = 1;
  int blocks = dv.ntiles;
  if (RUN) {
    // bh_chain_params.tile 3 / 4: runs of 2 / 4 consecutive tiles
    dv.per = p.tile == 4 ? 4 : 2;
    blocks = (dv.ntiles + dv.per - 1) / dv.per;
  }
  BH_LAUNCH((chain_tile_kernel<TH, TW, FAST, KX, RUN>), dim3(blocks), dim3(256), G.bytes, s, p, G, dv);
}

}  // namespace bh

// Tile form of bh_chain_i8 (bh_chain_params.tile != 0): LDS bytes, or 0 if
// the parameters do not admit it.  Called by bh_chain_lds_bytes after the
// checks every chain form shares.
extern "C" size_t bh_chain_tile_lds_bytes(const bh_chain_params* pp) {
  const bh_chain_params& p = *pp;
  const bh_dwconv_params& d = p.dw;
  // 1: one tile per workgroup; 3 / 4: runs of 2 / 4 tiles per workgroup
  if (p.tile != 1 && p.tile != 3 && p.tile != 4) return 0;
  if (d.stride_h < 1 || d.stride_h > 2 || d.stride_w < 1 || d.stride_w > 2 || d.dil_h < 1 || d.dil_h > 2 ||
      d.dil_w < 1 || d.dil_w > 2)
    return 0;
  if (p.has_pw2 && p.pw2.k_pad > 64 * 5) return 0;
  if ((long)d.batch * d.in_h * d.in_w * d.in_c < 16) return 0;
  const bh::TileGeom G = bh::tile_geom(p, 8, 8);
  // a workgroup's grid index and the DMA unit counts stay in int range
  if ((long)d.batch * G.tiles_y * G.tiles_x >= INT32_MAX / 2) return 0;
  return G.bytes <= 160 * 1024 ? G.bytes : 0;
}

extern "C" size_t bh_chain_tile_blob_bytes(const bh_chain_params* pp) {
  if (!pp) return 0;
  if (pp->stage) return bh_chain_lds_bytes(pp) > 0 ? (size_t)bh::tile_blob(*pp).bytes : 0;
  bh_chain_params q = *pp;
  q.tile = 1;
  if (bh_chain_tile_lds_bytes(&q) == 0) return 0;
  return (size_t)bh::tile_blob(q).bytes;
}

extern "C" int bh_chain_tile_pack(const bh_chain_params* pp, void* blob, bh_stream_t stream) {
  const size_t bytes = bh_chain_tile_blob_bytes(pp);
  if (bytes == 0 || !blob) {
    bh_set_last_error("bh_chain_tile_pack: invalid or unsupported parameters");
    return BH_EINVAL;
  }
  const bh::TileBlob B = bh::tile_blob(*pp);
  const int words = (int)(bytes / 4);
  hipLaunchKernelGGL(bh::chain_tile_pack_kernel, dim3((words + 255) / 256), dim3(256), 0, (hipStream_t)stream, *pp, B,
                     (unsigned char*)blob);
  return bh_check_launch("chain_tile_pack_kernel");
}

extern "C" int bh_chain_tile_launch(const bh_chain_params* pp, bh_stream_t stream) {
  const bh_chain_params& p = *pp;
  if (!p.tile_blob) {
    bh_set_last_error("bh_chain_i8: the tile form needs tile_blob (bh_chain_tile_pack)");
    return BH_EINVAL;
  }
  const bh::TileGeom G = bh::tile_geom(p, 8, 8);
  const bool fast = p.dw.requant_fast && p.pw1.requant_fast && (!p.has_pw2 || p.pw2.requant_fast);
  const bool k2 = !p.has_pw2 || p.pw2.k_pad <= 128;
  const bool run = p.tile >= 3;
  hipStream_t s = (hipStream_t)stream;
  if (k2) {
    if (fast) run ? bh::launch_tile<8, 8, true, 2, true>(p, G, s) : bh::launch_tile<8, 8, true, 2, false>(p, G, s);
    else run ? bh::launch_tile<8, 8, false, 2, true>(p, G, s) : bh::launch_tile<8, 8, false, 2, false>(p, G, s);
  } else {
    if (fast) run ? bh::launch_tile<8, 8, true, 5, true>(p, G, s) : bh::launch_tile<8, 8, true, 5, false>(p, G, s);
    else run ? bh::launch_tile<8, 8, false, 5, true>(p, G, s) : bh::launch_tile<8, 8, false, 5, false>(p, G, s);
  }
  return bh_check_launch("chain_tile_kernel");
}
