// CONV_2D with a tiny reduction (K = k_h*k_w*in_c <= 64: the RGB stem of
// every 224x224 classifier, e.g. MobileNet's 3x3 s2 over 3 channels) for
// gfx950.  Same TFLite 2.9.2 arithmetic as conv_mfma.hip (ConvPerChannel /
// uint8 reference Conv via the int8 domain; bit-exact), different mapping:
// at K = 27 an MFMA tile would be mostly K padding and the im2col gather is
// byte-granular, so this kernel stays on VALU.  A thread owns one output
// pixel x 8 output channels; the channel group is uniform per workgroup, so
// filters, bias and multipliers arrive through scalar loads; every input
// byte of the window is loaded at once (one memory round trip) and the dot
// products are v_dot4_i32_i8.
#include "common.hpp"
#include "stem_window.hpp"

namespace bh {

struct DirectDivs {
  FastDiv out_w, out_h;
};

template <int K4MAX>
__global__ __launch_bounds__(256) void conv_direct_kernel(bh_conv_params p, int M, int K, DirectDivs dv) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  const int c0 = blockIdx.y * 8;  // first output channel of this workgroup
  if (m >= M) return;
  const int t = dv.out_w.div(m);
  const int ox = m - t * p.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
  const int y0 = oy * p.stride_h - p.pad_h;
  const int x0 = ox * p.stride_w - p.pad_w;
  const uint8_t* in = (const uint8_t*)p.input + (long)n * p.in_h * p.in_w * p.in_c;
  const uint32_t xorb = (uint32_t)p.in_xor & 0xffu;
  const uint32_t padb = (uint32_t)p.in_zp & 0xffu;

  // gather the K window bytes (k = (fy*k_w + fx)*in_c + ci) in the int8
  // domain: out-of-image taps hold the input zero point (contribute 0)
  uint32_t xw[K4MAX];
#pragma unroll
  for (int j = 0; j < K4MAX; ++j) xw[j] = 0;
  {
    int ci = 0, fx = 0, fy = 0;
#pragma unroll
    for (int k = 0; k < 4 * K4MAX; ++k) {
      if (k < K) {
        const int y = y0 + fy * p.dil_h, x = x0 + fx * p.dil_w;
        uint32_t b = padb;
        if (y >= 0 && y < p.in_h && x >= 0 && x < p.in_w) b = (in[((long)y * p.in_w + x) * p.in_c + ci] ^ xorb);
        xw[k >> 2] |= b << (8 * (k & 3));
        if (++ci == p.in_c) {
          ci = 0;
          if (++fx == p.k_w) {
            fx = 0;
            ++fy;
          }
        }
      }
    }
  }
  int rowsum = 0;
  if (p.w_zp != 0) {
#pragma unroll
    for (int j = 0; j < K4MAX; ++j) rowsum = __builtin_amdgcn_sdot4((int)xw[j], 0x01010101, rowsum, false);
  }
  uint32_t packed[2] = {0u, 0u};
  const uint8_t* res = (const uint8_t*)p.residual;
  const long obase = (long)m * p.out_c;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int oc = c0 + c;
    if (oc >= p.out_c) break;
    const int* wrow = (const int*)(p.weights + (long)oc * p.k_pad);  // K tail zero-packed
    int acc = p.bias_eff[oc];
#pragma unroll
    for (int j = 0; j < K4MAX; ++j) acc = __builtin_amdgcn_sdot4((int)xw[j], wrow[j], acc, false);
    if (p.w_zp != 0) acc -= p.w_zp * rowsum;
    int32_t v = clamp_i32(requant(acc, p.mult[oc], p.shift[oc]) + p.out_zp, p.act_min, p.act_max);
    if (res) {
      const int32_t q = p.in_xor == 0 ? (int32_t)(int8_t)res[obase + oc] : (int32_t)res[obase + oc];
      const int32_t sy = requant_lt1((v + p.add_y_off) * (1 << p.add_left_shift), p.add_y_mult, p.add_y_shift);
      const int32_t sr = requant_lt1((q + p.add_r_off) * (1 << p.add_left_shift), p.add_r_mult, p.add_r_shift);
      v = clamp_i32(requant_lt1(sy + sr, p.add_o_mult, p.add_o_shift) + p.add_o_off, p.add_act_min, p.add_act_max);
    }
    const uint32_t byte = p.out_table ? ((const uint8_t*)p.out_table)[(uint8_t)v] : ((uint32_t)v & 0xffu);
    packed[c >> 2] |= byte << (8 * (c & 3));
  }
  uint8_t* out = (uint8_t*)p.output + obase + c0;
  if (c0 + 8 <= p.out_c && (p.out_c % 8) == 0) {
    *(v2i*)out = (v2i){(int)packed[0], (int)packed[1]};
  } else {
    for (int c = 0; c < 8 && c0 + c < p.out_c; ++c) out[c] = (uint8_t)(packed[c >> 2] >> (8 * (c & 3)));
  }
}

// The 3x3 RGB stem (k_w * in_c == 9 contiguous bytes per window row,
// dil_w 1) with one thread per output pixel over ALL output channels: the
// window is gathered once - three aligned dword loads per row and
// v_alignbyte / v_perm_b32 into the k-ordered byte stream
// (k = (fy*3 + fx)*3 + ci, seven dwords) - instead of 27 byte loads per
// 8-channel group.  Filter dwords, bias and multipliers are uniform per
// channel group (scalar loads).  Threads whose window leaves the image
// horizontally, or whose aligned loads would run past the tensor, take the
// byte path of conv_direct_kernel.
template <bool FAST>
__global__ __launch_bounds__(256) void conv_stem_kernel(bh_conv_params p, int M, DirectDivs dv, int ch_per_y) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const int t = dv.out_w.div(m);
  const int ox = m - t * p.out_w;
  const int n = dv.out_h.div(t);
  const int oy = t - n * p.out_h;
  const int y0 = oy * p.stride_h - p.pad_h;
  const int x0 = ox * p.stride_w - p.pad_w;
  const long img = (long)p.in_h * p.in_w * 3;
  const uint8_t* in = (const uint8_t*)p.input + n * img;
  const uint8_t* end = (const uint8_t*)p.input + p.batch * img;
  const uint32_t xorw = splat_byte(p.in_xor);
  const uint32_t padw = splat_byte(p.in_zp);

  uint32_t r[3][3];  // row fy: window bytes 0-3, 4-7, 8 (int8 domain)
  const bool colok = x0 >= 0 && x0 + 3 <= p.in_w;
#pragma unroll
  for (int fy = 0; fy < 3; ++fy) {
    const int y = y0 + fy * p.dil_h;
    const bool rowok = y >= 0 && y < p.in_h;
    const uint8_t* a = in + ((long)y * p.in_w + x0) * 3;
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
        b[k] = (x >= 0 && x < p.in_w) ? (uint32_t)(a[k] ^ (uint8_t)p.in_xor) : (padw & 0xffu);
      }
      r[fy][0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
      r[fy][1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
      r[fy][2] = b[8];
    }
  }
  // k-ordered stream: rows of 9 bytes back to back, one zero byte of tail
  uint32_t xw[7];
  xw[0] = r[0][0];
  xw[1] = r[0][1];
  xw[2] = __builtin_amdgcn_perm(r[1][0], r[0][2], 0x06050400u);  // R0[8] R1[0..2]
  xw[3] = __builtin_amdgcn_alignbyte(r[1][1], r[1][0], 3);        // R1[3..6]
  {
    const uint32_t u = __builtin_amdgcn_perm(r[1][2], r[1][1], 0x0c0c0403u);  // R1[7] R1[8] 0 0
    xw[4] = u | (r[2][0] << 16);                                             // .. R2[0] R2[1]
  }
  xw[5] = __builtin_amdgcn_alignbyte(r[2][1], r[2][0], 2);  // R2[2..5]
  xw[6] = __builtin_amdgcn_alignbyte(r[2][2], r[2][1], 2);  // R2[6..8] 0
  int rowsum = 0;
  if (p.w_zp != 0) {
#pragma unroll
    for (int j = 0; j < 7; ++j) rowsum = __builtin_amdgcn_sdot4((int)xw[j], 0x01010101, rowsum, false);
  }
  uint8_t* out = (uint8_t*)p.output + (long)m * p.out_c;
  const uint8_t* tab = (const uint8_t*)p.out_table;
  const cst_ptr<int32_t> wts = as_const((const int32_t*)p.weights);
  const cst_ptr<int32_t> bias = as_const(p.bias_eff), mult = as_const(p.mult), shift = as_const(p.shift);
  const int kpw = p.k_pad >> 2;
  // grid.y splits the channels when the pixels alone give too few
  // workgroups (batch 1): this workgroup's range [cb, ce)
  const int cb = blockIdx.y * ch_per_y;
  const int ce = min(p.out_c, cb + ch_per_y);
  for (int c0 = cb; c0 < ce; c0 += 8) {
    uint32_t packed[2] = {0u, 0u};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int oc = c0 + c;
      const cst_ptr<int32_t> wrow = wts + oc * kpw;  // uniform: scalar loads
      int acc = bias[oc];
#pragma unroll
      for (int j = 0; j < 7; ++j) acc = __builtin_amdgcn_sdot4((int)xw[j], wrow[j], acc, false);
      if (p.w_zp != 0) acc -= p.w_zp * rowsum;
      int32_t v = requant_out<FAST>(acc, chan_q(mult[oc], shift[oc], p.out_zp), p.out_zp, p.act_min, p.act_max);
      const uint32_t byte = tab ? tab[(uint8_t)v] : ((uint32_t)v & 0xffu);
      packed[c >> 2] |= byte << (8 * (c & 3));
    }
    *(v2i*)(out + c0) = (v2i){(int)packed[0], (int)packed[1]};
  }
}

// conv_stem_lds_kernel: the same stem with every channel's constants staged
// in LDS once per workgroup - filter dwords, folded bias and the
// requantisation constants (ChanQ precomputed) in one 64-byte record per
// channel - instead of read through the scalar cache per wave.  The scalar
// form issues ~200 s_load per wave in SGPR-bounded batches, each a full
// round trip (PMC at B = 24: waves resident from start to end, 50 % of their
// cycles parked on those waits, profiles/r05t_stem_pmc.txt); here a channel
// is four broadcast ds_read_b128 (every lane reads the same record).
// Channel ranges of up to 64 (grid.y splits wider layers).

// PX pixels per thread (m, m + 256, ...: stores stay lane-consecutive): the
// channel records' LDS reads serve PX pixels and their dot / requant chains
// interleave
// BH_STEM_ROWS (build-time A-B switch, default on): input rows staged in LDS
#ifndef BH_STEM_ROWS
#define BH_STEM_ROWS 1
#endif
constexpr int kStemRowWords = 3072;  // 12 KB: nine 224-pixel RGB rows
// BH_STEM_STORE16 (build-time A-B switch, default on): 16-byte output stores
#ifndef BH_STEM_STORE16
#define BH_STEM_STORE16 1
#endif
template <bool FAST, int PX>
__global__ __launch_bounds__(256) void conv_stem_lds_kernel(bh_conv_params p, int M, DirectDivs dv, int ch_per_y) {
  __shared__ __attribute__((aligned(16))) StemChan sc[64];
  const int cb = blockIdx.y * ch_per_y;
  const int ce = min(p.out_c, cb + ch_per_y);
  const int nc = ce - cb;
  const int m0 = blockIdx.x * 256 * PX + threadIdx.x;
  const long img = (long)p.in_h * p.in_w * 3;
  uint32_t xw[PX][7];
  // staged rows (BH_STEM_ROWS, one pixel per thread): when the workgroup's
  // 256 pixels lie in one image and their input rows fit kStemRowWords,
  // the rows come in as 16-byte loads into LDS (one load per 16 bytes of
  // the image instead of nine dword loads per pixel) and each window is read
  // from there after the barrier
  bool staged = false;
  int iy_lo = 0, rw = 0, n_img = 0;
#if BH_STEM_ROWS
  __shared__ __attribute__((aligned(16))) uint32_t rows[kStemRowWords];
  if constexpr (PX == 1) {
    const int mf = blockIdx.x * 256, ml = min(mf + 255, M - 1);
    const int tf = dv.out_w.div(mf), tl = dv.out_w.div(ml);
    const int nf = dv.out_h.div(tf), nl = dv.out_h.div(tl);
    rw = (((15 + p.in_w * 3) >> 2) + 4) & ~3;
    const int nrows = (tl - nf * p.out_h - (tf - nf * p.out_h)) * p.stride_h + 2 * p.dil_h + 1;
    if (nf == nl && (((uintptr_t)p.input) & 15) == 0 && nrows * rw <= kStemRowWords && p.batch * img < INT32_MAX) {
      staged = true;
      n_img = nf;
      iy_lo = (tf - nf * p.out_h) * p.stride_h - p.pad_h;
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      const int total = (int)(p.batch * img);
      const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.input, (short)0, total, 0x00020000);
      const int cpr = rw >> 2;  // 16-byte chunks per staged row
      for (int i = threadIdx.x; i < nrows * cpr; i += 256) {
        const int r = i / cpr;
        const int k = i - r * cpr;
        const int y = iy_lo + r;
        if (y >= 0 && y < p.in_h) {
          const int rel = n_img * (int)img + y * p.in_w * 3;
          const int g = (rel & ~15) + 16 * k;
          v4u v;
          if (g + 16 <= total) {
            v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, g, 0, 0);
          } else {
            // the chunk that runs past the tensor's end (a range-checked
            // 16-byte load would drop its valid bytes too): bytewise
            uint32_t wv[4] = {0, 0, 0, 0};
            for (int j = 0; j < 16 && g + j < total; ++j)
              wv[j >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, g + j, 0, 0) << (8 * (j & 3));
            v = (v4u){wv[0], wv[1], wv[2], wv[3]};
          }
          *(v4u*)(rows + r * rw + 4 * k) = v;
        }
      }
    }
  }
#endif
  if (!staged) {
    // the windows first: their loads are in flight while the constants stage
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int mm = min(m0 + 256 * u, M - 1);
      const int t = dv.out_w.div(mm);
      const int ox = mm - t * p.out_w;
      const int n = dv.out_h.div(t);
      const int oy = t - n * p.out_h;
      stem_window((const uint8_t*)p.input + n * img, (const uint8_t*)p.input + p.batch * img,
                  oy * p.stride_h - p.pad_h, ox * p.stride_w - p.pad_w, p.dil_h, p.in_h, p.in_w, (uint32_t)p.in_xor,
                  (uint32_t)p.in_zp, xw[u]);
    }
  }
  {
    const int kpw = p.k_pad >> 2;
    const int32_t* wts = (const int32_t*)p.weights;
    for (int i = threadIdx.x; i < nc * 16; i += 256) {
      ((int32_t*)sc)[i] = stem_chan_word(wts, kpw, p.bias_eff, p.mult, p.shift, p.out_zp, cb + (i >> 4), i & 15);
    }
  }
  __syncthreads();
#if BH_STEM_ROWS
  if (staged) {
    const int mm = min(m0, M - 1);
    const int t = dv.out_w.div(mm);
    const int ox = mm - t * p.out_w;
    const int oy = t - n_img * p.out_h;
    stem_window_lds(rows, rw, iy_lo, n_img * (int)img, oy * p.stride_h - p.pad_h, ox * p.stride_w - p.pad_w, p.dil_h,
                    p.in_h, p.in_w, (uint32_t)p.in_xor, (uint32_t)p.in_zp, xw[0]);
  }
#endif
  if (m0 >= M) return;
  int rowsum[PX];
#pragma unroll
  for (int u = 0; u < PX; ++u) {
    rowsum[u] = 0;
    if (p.w_zp != 0) {
#pragma unroll
      for (int j = 0; j < 7; ++j) rowsum[u] = __builtin_amdgcn_sdot4((int)xw[u][j], 0x01010101, rowsum[u], false);
    }
  }
  const uint8_t* tab = (const uint8_t*)p.out_table;
#if BH_STEM_STORE16
  // 16 channels per store (one 16-byte store per pixel instead of four
  // dword stores) when the channel range and the row pitch allow it
  if ((nc & 15) == 0 && (p.out_c & 15) == 0 && (cb & 15) == 0) {
    for (int c0 = 0; c0 < nc; c0 += 16) {
      uint32_t packed[PX][4];
#pragma unroll
      for (int u = 0; u < PX; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) packed[u][j] = 0;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const StemChan& k = sc[c0 + c];
#pragma unroll
        for (int u = 0; u < PX; ++u) {
          const int32_t v =
              stem_chan_eval<FAST>(k, xw[u], p.w_zp != 0, p.w_zp * rowsum[u], p.out_zp, p.act_min, p.act_max);
          const uint32_t byte = tab ? tab[(uint8_t)v] : ((uint32_t)v & 0xffu);
          packed[u][c >> 2] |= byte << (8 * (c & 3));
        }
      }
#pragma unroll
      for (int u = 0; u < PX; ++u) {
        const int m = m0 + 256 * u;
        if (m < M)
          *(uint4*)((uint8_t*)p.output + (long)m * p.out_c + cb + c0) =
              make_uint4(packed[u][0], packed[u][1], packed[u][2], packed[u][3]);
      }
    }
    return;
  }
#endif
  for (int c0 = 0; c0 < nc; c0 += 4) {
    uint32_t packed[PX];
#pragma unroll
    for (int u = 0; u < PX; ++u) packed[u] = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const StemChan& k = sc[c0 + c];
#pragma unroll
      for (int u = 0; u < PX; ++u) {
        const int32_t v = stem_chan_eval<FAST>(k, xw[u], p.w_zp != 0, p.w_zp * rowsum[u], p.out_zp, p.act_min, p.act_max);
        const uint32_t byte = tab ? tab[(uint8_t)v] : ((uint32_t)v & 0xffu);
        packed[u] |= byte << (8 * c);
      }
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int m = m0 + 256 * u;
      if (m < M) *(uint32_t*)((uint8_t*)p.output + (long)m * p.out_c + cb + c0) = packed[u];
    }
  }
}

}  // namespace bh

// Launched by bh_conv2d_i8 for small-K layers (conv_mfma.hip); returns
// BH_EINVAL when the layer is outside this kernel's range.
int bh_conv_direct_launch(const bh_conv_params& p, int M, int K, hipStream_t s) {
  if (K > 64 || p.out_c <= 0 || (p.k_pad % 4)) return BH_EINVAL;
  bh::DirectDivs dv;
  dv.out_w = bh::FastDiv(p.out_w);
  dv.out_h = bh::FastDiv(p.out_h);
  const dim3 grid((unsigned)((M + 255) / 256), (unsigned)((p.out_c + 7) / 8));
  if (K <= 32) BH_LAUNCH(bh::conv_direct_kernel<8>, grid, dim3(256), 0, s, p, M, K, dv);
  else BH_LAUNCH(bh::conv_direct_kernel<16>, grid, dim3(256), 0, s, p, M, K, dv);
  return bh_check_launch("conv_direct_kernel");
}

// 3x3 / in_c 3 / dil_w 1 stems, out_c % 8 == 0, no residual (conv_mfma.hip
// routes them here); anything else takes conv_direct_kernel
namespace {
// the stem's grid (channels split over grid.y to reach ~min_wg workgroups,
// 8 at a time) and form: the LDS-staged constants (default; channel ranges
// of <= 64, out_c % 4 == 0 for its dword stores, aligned output, from 256
// workgroups - at batch 1 the staging is not repaid: 5.05 vs 4.87 us; B = 24:
// 13.6 vs 14.6 us, r05u_stem_*) or the scalar-cache form
// (BH_CONV_STEM_SCALAR, or BH_STEM_SCALAR=1 for A-B runs)
struct StemPlan {
  int gx, gy, ch_per_y;
  bool lds;
};
StemPlan stem_plan(const bh_conv_params& p, int M) {
  // channel groups over grid.y until 512 workgroups (splitting further only
  // adds waves that repeat the window gather, profiles/r05ax_breakdown_mw*)
  constexpr int min_wg = 512;
  StemPlan sp;
  sp.gx = (M + 255) / 256;
  const int groups = p.out_c / 8;
  int gy = (min_wg + sp.gx - 1) / sp.gx;
  gy = gy < 1 ? 1 : (gy > groups ? groups : gy);
  sp.ch_per_y = (groups + gy - 1) / gy * 8;
  sp.gy = (p.out_c + sp.ch_per_y - 1) / sp.ch_per_y;
  sp.lds = p.kernel_hint != BH_CONV_STEM_SCALAR && sp.ch_per_y <= 64 && p.out_c % 4 == 0 &&
           (((uintptr_t)p.output) & 3) == 0 && (sp.gx >= 256 || p.kernel_hint == BH_CONV_STEM_VALU);
  return sp;
}
bool stem_shape_ok(const bh_conv_params& p) {
  return p.k_h == 3 && p.k_w == 3 && p.in_c == 3 && p.dil_w == 1 && p.out_c % 8 == 0 && !p.residual && p.k_pad >= 28;
}
}  // namespace

// the kernel symbol conv_stem routing lands on (profiling attribution)
const char* bh_conv_stem_kernel_name(const bh_conv_params& p, int M) {
  if (!stem_shape_ok(p)) return "conv_direct_kernel";
  return stem_plan(p, M).lds ? "conv_stem_lds_kernel" : "conv_stem_kernel";
}

int bh_conv_stem_launch(const bh_conv_params& p, int M, int K, hipStream_t s) {
  if (!stem_shape_ok(p)) return bh_conv_direct_launch(p, M, K, s);
  bh::DirectDivs dv;
  dv.out_w = bh::FastDiv(p.out_w);
  dv.out_h = bh::FastDiv(p.out_h);
  const StemPlan sp = stem_plan(p, M);
  const int gx = sp.gx, gy = sp.gy, ch_per_y = sp.ch_per_y;
  const dim3 grid((unsigned)gx, (unsigned)gy);
  const bool lds = sp.lds;
  if (lds) {
    // one pixel per thread (two, sharing the channel records' LDS reads,
    // was slower: 17.5 vs 14.7 us at B = 24, profiles/r05x_stem_px{1,2}.txt -
    // half the waves, each with twice the dependent VALU chains)
    if (p.requant_fast) BH_LAUNCH((bh::conv_stem_lds_kernel<true, 1>), grid, dim3(256), 0, s, p, M, dv, ch_per_y);
    else BH_LAUNCH((bh::conv_stem_lds_kernel<false, 1>), grid, dim3(256), 0, s, p, M, dv, ch_per_y);
    return bh_check_launch("conv_stem_lds_kernel");
  }
  if (p.requant_fast) BH_LAUNCH(bh::conv_stem_kernel<true>, grid, dim3(256), 0, s, p, M, dv, ch_per_y);
  else BH_LAUNCH(bh::conv_stem_kernel<false>, grid, dim3(256), 0, s, p, M, dv, ch_per_y);
  return bh_check_launch("conv_stem_kernel");
}
