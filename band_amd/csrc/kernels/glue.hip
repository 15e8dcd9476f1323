// Glue ops for whole-model residency on gfx950:
// the TFLite 2.9.2 builtins around the conv stack of detection /
// segmentation / pose models.  All are byte movers bound by HBM (or, at
// batch 1, by launch latency), so the design goal is one memory round trip
// and no per-element division:
//   * 8-bit unary ops -> one table gather (bh_lut_u8 / bh_lut_f32).  The host
//     evaluates TFLite's exact formula for all 256 input bytes, so the device
//     never re-derives float or fixed-point rounding.
//   * index maps that TFLite computes in float (RESIZE_NEAREST_NEIGHBOR) or in
//     10-bit fixed point (RESIZE_BILINEAR int8) -> host-built per-row and
//     per-column tables; the device only gathers and (bilinear) does the
//     integer 4-tap blend.
//   * float sequences (softmax, mean, uint8 bilinear) keep TFLite's operation
//     order; the Makefile builds this file with -ffp-contract=off, since HIP's
//     _rn intrinsics are plain operators that would otherwise fuse to FMA.
//   * SOFTMAX (8-bit, lookup-table path) -> host-built float exp table; the
//     per-row sum runs sequentially in TFLite's order, so the float result is
//     the same.
#include "common.hpp"

namespace bh {

// ---- table lookups ----------------------------------------------------------
// Table staged in LDS; 16 input bytes per thread when both pointers are
// 16-byte aligned, a byte loop for the tail.
__global__ __launch_bounds__(256) void lut_u8_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                     long n, long n16, const uint8_t* __restrict__ table) {
  __shared__ uint8_t t[256];
  if (threadIdx.x < 64) *(uint32_t*)(t + 4 * threadIdx.x) = *(const uint32_t*)(table + 4 * threadIdx.x);
  __syncthreads();
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) {
    v4i v = *(const v4i*)(in + 16 * i);
    v4i o;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t x = (uint32_t)v[w];
      o[w] = (int)((uint32_t)t[x & 0xff] | ((uint32_t)t[(x >> 8) & 0xff] << 8) |
                   ((uint32_t)t[(x >> 16) & 0xff] << 16) | ((uint32_t)t[x >> 24] << 24));
    }
    *(v4i*)(out + 16 * i) = o;
  } else {
    const long j = 16 * n16 + (i - n16);
    if (j < n) out[j] = t[in[j]];
  }
}

__global__ __launch_bounds__(256) void lut_f32_kernel(const uint8_t* __restrict__ in, float* __restrict__ out,
                                                      long n, const float* __restrict__ table) {
  __shared__ float t[256];
  t[threadIdx.x] = table[threadIdx.x];
  __syncthreads();
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = t[in[i]];
}

// reference_ops::AffineQuantize: (int32)TfLiteRound(x / scale) + zp, with
// IEEE division and round-half-away-from-zero
__global__ __launch_bounds__(256) void quantize_f32_kernel(const float* __restrict__ in, uint8_t* __restrict__ out,
                                                           long n, float scale, int32_t zp, int32_t lo, int32_t hi) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = (uint8_t)clamp_i32((int32_t)roundf(__fdiv_rn(in[i], scale)) + zp, lo, hi);
}

// ---- concatenation -----------------------------------------------------------
struct ConcatDivs {
  FastDiv row[BH_CONCAT_MAX_INPUTS];
  long off[BH_CONCAT_MAX_INPUTS];  // byte offset of input k inside an output row
  int blk0[BH_CONCAT_MAX_INPUTS + 1];  // first workgroup of input k (1-D grid)
  long out_row;
  int vec4;                        // every row / offset / pointer dword aligned
};

// One 1-D grid over the inputs' own ranges (input k owns workgroups
// [blk0[k], blk0[k+1]), found by a wave-uniform scan), so no workgroup exits
// idle for the smaller inputs (a grid.y per input launched max-input-sized
// ranges for every input: SSD's 6-input class concat ran 6x the workgroups
// it needed).  A thread copies 4 bytes: one dword when everything is
// aligned, else 4 bytes that may cross an output row, through the input's
// rescale table when one is given.
__global__ __launch_bounds__(256) void concat_kernel(bh_concat_params p, ConcatDivs dv) {
  int k = 0;
  for (int q = 1; q < p.n_inputs; ++q) k += (int)blockIdx.x >= dv.blk0[q];
  const uint8_t* src = (const uint8_t*)p.input[k];
  const uint8_t* tab = (const uint8_t*)p.table[k];
  uint8_t* dst = (uint8_t*)p.output + dv.off[k];
  const long row = p.row[k];
  const long i = (long)((int)blockIdx.x - dv.blk0[k]) * 256 + threadIdx.x;  // 4-byte unit
  if (dv.vec4 && !tab) {
    const long units = p.outer * (row / 4);
    if (i >= units) return;
    const uint32_t o = dv.row[k].div((uint32_t)(4 * i));  // FastDiv over bytes
    const long j = 4 * i - (long)o * row;
    *(uint32_t*)(dst + o * dv.out_row + j) = *(const uint32_t*)(src + 4 * i);
  } else {
    const long total = p.outer * row;
    const long b0 = 4 * i;
    if (b0 >= total) return;
    long o = dv.row[k].div((uint32_t)b0);
    long j = b0 - o * row;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (b0 + b < total) {
        const uint8_t v = src[b0 + b];
        dst[o * dv.out_row + j] = tab ? tab[v] : v;
      }
      if (++j == row) {
        j = 0;
        ++o;
      }
    }
  }
}

// ---- pad --------------------------------------------------------------------
struct PadDivs {
  FastDiv c, w, h;
  int os[4];
};

// MIRROR_PAD source index of padded position i along a dimension of n
// elements with `before` leading pads (TFLite 2.9.2 mirror_pad.cc
// GetInputDimension; offset 1 = REFLECT skips the edge, 0 = SYMMETRIC)
__host__ __device__ inline int mirror_index(int i, int before, int n, int mode) {
  const int offset = mode == 1 ? 1 : 0;
  if (i < before) {
    const int orig = before + offset - 1;
    return orig - min(i, orig - offset);
  }
  i -= before;
  if (i >= n) {
    i -= n;
    const int orig = n - (1 + offset);
    return orig - min(i, orig);
  }
  return i;
}

template <typename T>
__global__ __launch_bounds__(256) void pad_kernel(bh_pad_params p, PadDivs dv, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  uint32_t t = dv.c.div((uint32_t)i);
  const int c = (int)(i - (long)t * dv.os[3]);
  uint32_t t2 = dv.w.div(t);
  const int x = (int)(t - t2 * dv.os[2]);
  const uint32_t b = dv.h.div(t2);
  const int y = (int)(t2 - b * dv.os[1]);
  const int ib = (int)b - p.pad_before[0], iy = y - p.pad_before[1], ix = x - p.pad_before[2],
            ic = c - p.pad_before[3];
  T v = (T)p.value;
  if (p.mode) {
    const int jb = mirror_index((int)b, p.pad_before[0], p.in_shape[0], p.mode);
    const int jy = mirror_index(y, p.pad_before[1], p.in_shape[1], p.mode);
    const int jx = mirror_index(x, p.pad_before[2], p.in_shape[2], p.mode);
    const int jc = mirror_index(c, p.pad_before[3], p.in_shape[3], p.mode);
    v = ((const T*)p.input)[(((long)jb * p.in_shape[1] + jy) * p.in_shape[2] + jx) * p.in_shape[3] + jc];
  } else if (ib >= 0 && ib < p.in_shape[0] && iy >= 0 && iy < p.in_shape[1] && ix >= 0 && ix < p.in_shape[2] &&
             ic >= 0 && ic < p.in_shape[3]) {
    v = ((const T*)p.input)[(((long)ib * p.in_shape[1] + iy) * p.in_shape[2] + ix) * p.in_shape[3] + ic];
  }
  ((T*)p.output)[i] = v;
}

// ---- resize -----------------------------------------------------------------
struct ResizeDivs {
  FastDiv units, ow, oh;
};

// one thread per (output pixel, 4-byte unit of its row) when rows are dword
// multiples, else per byte (UNIT = 4 / 1)
template <int UNIT>
__global__ __launch_bounds__(256) void resize_nearest_kernel(bh_resize_nearest_params p, ResizeDivs dv, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const uint32_t pix = dv.units.div((uint32_t)i);
  const int u = (int)(i - (long)pix * (p.row_bytes / UNIT));
  const uint32_t t = dv.ow.div(pix);
  const int x = (int)(pix - t * p.out_w);
  const uint32_t n = dv.oh.div(t);
  const int y = (int)(t - n * p.out_h);
  const long src = (((long)n * p.in_h + p.y_index[y]) * p.in_w + p.x_index[x]) * p.row_bytes + (long)u * UNIT;
  if constexpr (UNIT == 4) ((uint32_t*)p.output)[i] = *(const uint32_t*)((const uint8_t*)p.input + src);
  else ((uint8_t*)p.output)[i] = ((const uint8_t*)p.input)[src];
}

// ResizeBilinearInteger: the four 2^10-fixed-point weights and the int64 sum
// rounded half away from zero at 2^20
__global__ __launch_bounds__(256) void resize_bilinear_kernel(bh_resize_bilinear_params p, ResizeDivs dv, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const uint32_t pix = dv.units.div((uint32_t)i);  // units = channels
  const int ch = (int)(i - (long)pix * p.channels);
  const uint32_t t = dv.ow.div(pix);
  const int x = (int)(pix - t * p.out_w);
  const uint32_t n = dv.oh.div(t);
  const int y = (int)(t - n * p.out_h);
  const int y0 = p.y_tab[3 * y], y1 = p.y_tab[3 * y + 1], iy = p.y_tab[3 * y + 2];
  const int x0 = p.x_tab[3 * x], x1 = p.x_tab[3 * x + 1], ix = p.x_tab[3 * x + 2];
  // 32-bit throughout: |s| <= 128 * 2^20 (the four weights sum to 2^20), so
  // TFLite's int64 accumulation never leaves int32 range; offsets < 2^31
  // (checked by the launcher)
  const int8_t* in = (const int8_t*)p.input + ((int)n * p.in_h * p.in_w * p.channels + ch);
  const int r0 = y0 * p.in_w, r1 = y1 * p.in_w;
  const int32_t v00 = in[(r0 + x0) * p.channels], v10 = in[(r1 + x0) * p.channels];
  const int32_t v01 = in[(r0 + x1) * p.channels], v11 = in[(r1 + x1) * p.channels];
  constexpr int32_t one = 1 << 10;
  const int32_t fy = iy - one * y0, fx = ix - one * x0;
  const int32_t s = v00 * ((one - fy) * (one - fx)) + v10 * (fy * (one - fx)) + v01 * ((one - fy) * fx) +
                    v11 * (fy * fx);
  const int32_t rnd = s > 0 ? (1 << 19) : -(1 << 19);
  ((int8_t*)p.output)[i] = (int8_t)((s + rnd) / (1 << 20));
}

// Row form (DeepLab's 14x14 -> 224x224 logits upsample: 25 MB out per
// batch-24 pass, which the byte-per-thread kernel spread over ~400k waves).
// One workgroup per output row (image n, row y): the two input rows it
// blends (y0, y1) and the column table are staged in LDS once; each thread
// then produces 16 consecutive bytes of the row (x, channel advanced
// incrementally, no division in the loop) and stores them as one 16-byte
// store.  The blend is TFLite's four-term sum, factored exactly (integer
// arithmetic) as (1-fy)(v00(1-fx) + v01 fx) + fy(v10(1-fx) + v11 fx).
constexpr int kRzRow = 8192;   // staged input row bytes (in_w * channels)
constexpr int kRzCols = 1024;  // staged output columns

__global__ __launch_bounds__(256) void resize_bilinear_rows_kernel(bh_resize_bilinear_params p, FastDiv chans,
                                                                   int vec_ok) {
  __shared__ __attribute__((aligned(16))) int8_t rows[2][kRzRow];
  __shared__ int xt[3 * kRzCols];
  const int y = blockIdx.x % p.out_h;
  const int n = blockIdx.x / p.out_h;
  const int C = p.channels;
  const int in_row = p.in_w * C;
  const int y0 = p.y_tab[3 * y], y1 = p.y_tab[3 * y + 1], iy = p.y_tab[3 * y + 2];
  const int8_t* src0 = (const int8_t*)p.input + ((long)n * p.in_h + y0) * in_row;
  const int8_t* src1 = (const int8_t*)p.input + ((long)n * p.in_h + y1) * in_row;
  for (int i = threadIdx.x; i < in_row; i += 256) {
    rows[0][i] = src0[i];
    rows[1][i] = src1[i];
  }
  for (int i = threadIdx.x; i < 3 * p.out_w; i += 256) xt[i] = p.x_tab[i];
  __syncthreads();
  constexpr int32_t one = 1 << 10;
  const int32_t fy = iy - one * y0;
  const int row_bytes = p.out_w * C;
  int8_t* dst = (int8_t*)p.output + ((long)n * p.out_h + y) * row_bytes;
  for (int f0 = threadIdx.x * 16; f0 < row_bytes; f0 += 256 * 16) {
    int x = (int)chans.div((uint32_t)f0);
    int ch = f0 - x * C;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      if (f0 + b < row_bytes) {
        const int x0 = xt[3 * x], x1 = xt[3 * x + 1];
        const int32_t fx = xt[3 * x + 2] - one * x0;
        const int32_t h0 = (int32_t)rows[0][x0 * C + ch] * (one - fx) + (int32_t)rows[0][x1 * C + ch] * fx;
        const int32_t h1 = (int32_t)rows[1][x0 * C + ch] * (one - fx) + (int32_t)rows[1][x1 * C + ch] * fx;
        const int32_t s = h0 * (one - fy) + h1 * fy;
        const int32_t rnd = s > 0 ? (1 << 19) : -(1 << 19);
        const uint32_t v = (uint32_t)(uint8_t)(int8_t)((s + rnd) / (1 << 20));
        w[b >> 2] |= v << (8 * (b & 3));
      }
      if (++ch == C) {
        ch = 0;
        ++x;
      }
    }
    if (vec_ok && f0 + 16 <= row_bytes) {
      *(v4i*)(dst + f0) = (v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    } else {
      for (int b = 0; b < 16 && f0 + b < row_bytes; ++b) dst[f0 + b] = (int8_t)(w[b >> 2] >> (8 * (b & 3)));
    }
  }
}

// TFLite's (s + (s > 0 ? 2^19 : -2^19)) / 2^20 (C division, toward zero)
// for |s| < 2^30 as one arithmetic shift: s > 0 gives floor((s + 2^19) /
// 2^20); s <= 0 gives trunc((s - 2^19) / 2^20) = floor((s + 2^19 - 1) / 2^20)
__device__ __forceinline__ int32_t rz_round20(int32_t s) {
  return (s + ((1 << 19) - 1) + (int32_t)((uint32_t)(-s) >> 31)) >> 20;
}

// Column-blend form for channels >= 16 (DeepLab's 21-class logits): the two
// input rows of an output row are blended VERTICALLY once into int32
// V[xi][c] = r0[xi][c] (1 - fy) + r1[xi][c] fy (dynamic LDS, in_w * C words
// per row), so each output byte is (V[x0][c] (1 - fx) + V[x1][c] fx), the
// same exact integer sum as TFLite's four terms (|s| <= 2^29, no overflow).
// With C >= 16 a thread's 16 consecutive bytes span at most two output
// pixels: their column entries are read once (not per byte) and each byte
// picks one of the two with a select, so a byte costs 2 LDS reads and ~12
// VALU instead of 7 LDS reads and ~30 VALU (the row kernel above was
// VALU-bound).  A workgroup takes `nr` consecutive output rows of one image
// (one row each: 7,168 workgroups of 4.7 KB output at DeepLab's batch 32,
// each paying its own load round trip and a 15 %-occupied second pass).
__global__ __launch_bounds__(256) void resize_bilinear_cols_kernel(bh_resize_bilinear_params p, FastDiv chans,
                                                                   int vec_ok, int nr, FastDiv groups,
                                                                   FastDiv cpr_div) {
  extern __shared__ __attribute__((aligned(16))) int32_t rz_lds[];
  const int n = groups.div(blockIdx.x);
  const int y_first = (blockIdx.x - n * (int)groups.d) * nr;
  const int rows = min(nr, p.out_h - y_first);
  const int C = p.channels;
  const int in_row = p.in_w * C;
  int32_t* X0 = rz_lds;          // [out_w]: x0 * C
  int32_t* X1 = X0 + p.out_w;    // [out_w]: x1 * C
  int32_t* FX = X1 + p.out_w;    // [out_w]: fx
  int32_t* V = FX + p.out_w;     // [rows][in_row]
  constexpr int32_t one = 1 << 10;
  for (int i = threadIdx.x; i < rows * in_row; i += 256) {
    const int r = i / in_row;  // rows <= 8: a short division
    const int k = i - r * in_row;
    const int y = y_first + r;
    const int y0 = p.y_tab[3 * y], y1 = p.y_tab[3 * y + 1];
    const int32_t fy = p.y_tab[3 * y + 2] - one * y0;
    const int8_t* in = (const int8_t*)p.input + (long)n * p.in_h * in_row;
    V[i] = __mul24((int32_t)in[y0 * in_row + k], one - fy) + __mul24((int32_t)in[y1 * in_row + k], fy);
  }
  for (int x = threadIdx.x; x < p.out_w; x += 256) {
    const int x0 = p.x_tab[3 * x];
    X0[x] = x0 * C;
    X1[x] = p.x_tab[3 * x + 1] * C;
    FX[x] = p.x_tab[3 * x + 2] - one * x0;
  }
  __syncthreads();
  const int row_bytes = p.out_w * C;
  const int cpr = (int)cpr_div.d;  // 16-byte chunks per output row
  for (int i = threadIdx.x; i < rows * cpr; i += 256) {
    const int r = (int)cpr_div.div((uint32_t)i);
    const int f0 = (i - r * cpr) * 16;
    const int32_t* Vr = V + r * in_row;
    int8_t* dst = (int8_t*)p.output + ((long)n * p.out_h + y_first + r) * row_bytes;
    const int x = (int)chans.div((uint32_t)f0);
    const int ch0 = f0 - x * C;
    const int k = C - ch0;  // bytes b < k belong to pixel x, the rest to x + 1
    const int xn = x + 1 < p.out_w ? x + 1 : x;
    // per-pixel bases with the byte index folded out: byte b reads Vr[base + b]
    const int a0 = X0[x] + ch0, a1 = X1[x] + ch0, fa = FX[x];
    const int b0 = X0[xn] - k, b1 = X1[xn] - k, fb = FX[xn];
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const bool first = b < k;
      const int o0 = (first ? a0 : b0) + b, o1 = (first ? a1 : b1) + b;
      const int32_t fx = first ? fa : fb;
      const int32_t v0 = Vr[o0], v1 = Vr[o1];
      // |V| <= 2^17, fx <= 2^10: 24-bit multiplies (v_mul_i32_i24, full
      // rate; v_mul_lo_u32 is quarter rate) are exact
      const int32_t s = __mul24(v0, one - fx) + __mul24(v1, fx);
      w[b >> 2] |= ((uint32_t)rz_round20(s) & 0xffu) << (8 * (b & 3));
    }
    if (vec_ok && f0 + 16 <= row_bytes) {
      *(v4i*)(dst + f0) = (v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    } else {
      for (int b = 0; b < 16 && f0 + b < row_bytes; ++b) dst[f0 + b] = (int8_t)(w[b >> 2] >> (8 * (b & 3)));
    }
  }
}

// ---- softmax ----------------------------------------------------------------
// One thread per row; the float operations are issued exactly as the
// reference's loop runs them (no contraction: explicit _rn intrinsics).
__global__ __launch_bounds__(256) void softmax_kernel(bh_softmax_params p) {
  __shared__ float t[256];
  t[threadIdx.x] = p.table[threadIdx.x];
  __syncthreads();
  const long r = (long)blockIdx.x * 256 + threadIdx.x;
  if (r >= p.rows) return;
  const uint8_t* x = (const uint8_t*)p.input + r * p.depth;
  uint8_t* y = (uint8_t*)p.output + r * p.depth;
  const bool sg = p.is_signed != 0;
  int32_t mx = sg ? -128 : 0;
  for (int j = 0; j < p.depth; ++j) mx = max(mx, sg ? (int32_t)(int8_t)x[j] : (int32_t)x[j]);
  const float* to = t + 255 - mx;
  float sum = 0.0f;
  for (int j = 0; j < p.depth; ++j) sum = __fadd_rn(sum, to[sg ? (int32_t)(int8_t)x[j] : (int32_t)x[j]]);
  const float inv = __fdiv_rn(1.0f, __fmul_rn(sum, p.out_scale));
  const int32_t lo = sg ? -128 : 0, hi = sg ? 127 : 255;
  for (int j = 0; j < p.depth; ++j) {
    const float pr = __fmul_rn(to[sg ? (int32_t)(int8_t)x[j] : (int32_t)x[j]], inv);
    const int32_t q = sg ? (int32_t)roundf(pr) + p.out_zp : (int32_t)__fadd_rn(pr, 0.5f) + p.out_zp;
    y[j] = (uint8_t)clamp_i32(q, lo, hi);
  }
}

// ---- zero insertion (TRANSPOSE_CONV as a stride-1 conv) -------------------
struct ZiDivs {
  FastDiv units, ow, oh, sh, sw;
};

// one thread per (U pixel, UNIT bytes of its channels)
template <int UNIT>
__global__ __launch_bounds__(256) void zero_insert_kernel(bh_zero_insert_params p, ZiDivs dv, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const uint32_t pix = dv.units.div((uint32_t)i);
  const int u = (int)(i - (long)pix * dv.units.d);
  const uint32_t t = dv.ow.div(pix);
  const int x = (int)(pix - t * p.out_w);
  const uint32_t n = dv.oh.div(t);
  const int y = (int)(t - n * p.out_h);
  const uint32_t iy = dv.sh.div((uint32_t)y), ix = dv.sw.div((uint32_t)x);
  const bool hit = (int)iy * p.stride_h == y && (int)ix * p.stride_w == x;
  if constexpr (UNIT == 4) {
    uint32_t v = p.fill * 0x01010101u;
    if (hit) v = ((const uint32_t*)p.input)[(((long)n * p.in_h + iy) * p.in_w + ix) * dv.units.d + u];
    ((uint32_t*)p.output)[i] = v;
  } else {
    uint8_t v = (uint8_t)p.fill;
    if (hit) v = ((const uint8_t*)p.input)[(((long)n * p.in_h + iy) * p.in_w + ix) * p.channels + u];
    ((uint8_t*)p.output)[i] = v;
  }
}

inline unsigned blocks(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace bh

extern "C" int bh_lut_u8(const void* in, void* out, long n, const void* table, bh_stream_t s) {
  if (!in || !out || !table || n < 0 || n >= (1l << 36)) {
    bh_set_last_error("bh_lut_u8: invalid parameters");
    return BH_EINVAL;
  }
  if (n == 0) return 0;
  const bool al = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
  const long n16 = al ? n / 16 : 0;
  const long threads = n16 + (n - 16 * n16);
  BH_LAUNCH(bh::lut_u8_kernel, dim3(bh::blocks(threads)), dim3(256), 0, (hipStream_t)s,
                     (const uint8_t*)in, (uint8_t*)out, n, n16, (const uint8_t*)table);
  return bh_check_launch("lut_u8_kernel");
}

extern "C" int bh_lut_f32(const void* in, void* out, long n, const float* table, bh_stream_t s) {
  if (!in || !out || !table || n < 0) {
    bh_set_last_error("bh_lut_f32: invalid parameters");
    return BH_EINVAL;
  }
  if (n == 0) return 0;
  BH_LAUNCH(bh::lut_f32_kernel, dim3(bh::blocks(n)), dim3(256), 0, (hipStream_t)s, (const uint8_t*)in,
                     (float*)out, n, table);
  return bh_check_launch("lut_f32_kernel");
}

extern "C" int bh_quantize_f32(const float* in, void* out, long n, float scale, int32_t zp, int out_signed,
                               bh_stream_t s) {
  if (!in || !out || n < 0 || !(scale > 0.f)) {
    bh_set_last_error("bh_quantize_f32: invalid parameters");
    return BH_EINVAL;
  }
  if (n == 0) return 0;
  BH_LAUNCH(bh::quantize_f32_kernel, dim3(bh::blocks(n)), dim3(256), 0, (hipStream_t)s, in, (uint8_t*)out,
                     n, scale, zp, out_signed ? -128 : 0, out_signed ? 127 : 255);
  return bh_check_launch("quantize_f32_kernel");
}

extern "C" int bh_concat(const bh_concat_params* pp, bh_stream_t s) {
  if (!pp || pp->n_inputs <= 0 || pp->n_inputs > BH_CONCAT_MAX_INPUTS || pp->outer <= 0 || !pp->output) {
    bh_set_last_error("bh_concat: invalid parameters");
    return BH_EINVAL;
  }
  const bh_concat_params& p = *pp;
  bh::ConcatDivs dv{};
  long off = 0, maxbytes = 0;
  bool vec4 = (uintptr_t)p.output % 4 == 0;
  for (int k = 0; k < p.n_inputs; ++k) {
    if (!p.input[k] || p.row[k] < 0) {
      bh_set_last_error("bh_concat: invalid input");
      return BH_EINVAL;
    }
    dv.row[k] = bh::FastDiv((uint32_t)(p.row[k] > 0 ? p.row[k] : 1));
    dv.off[k] = off;
    vec4 = vec4 && p.row[k] % 4 == 0 && off % 4 == 0 && (uintptr_t)p.input[k] % 4 == 0;
    off += p.row[k];
    maxbytes = p.outer * p.row[k] > maxbytes ? p.outer * p.row[k] : maxbytes;
  }
  dv.out_row = off;
  dv.vec4 = vec4 ? 1 : 0;
  if (p.outer * off >= INT32_MAX) {
    bh_set_last_error("bh_concat: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  if (maxbytes == 0) return 0;
  // 4 bytes per thread; input k's workgroups follow input k-1's
  int blk = 0;
  for (int k = 0; k < p.n_inputs; ++k) {
    dv.blk0[k] = blk;
    blk += (int)bh::blocks((p.outer * p.row[k] + 3) / 4);
  }
  dv.blk0[p.n_inputs] = blk;
  if (blk == 0) return 0;
  BH_LAUNCH(bh::concat_kernel, dim3((unsigned)blk), dim3(256), 0, (hipStream_t)s, p, dv);
  return bh_check_launch("concat_kernel");
}

extern "C" int bh_pad(const bh_pad_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || (pp->elem_bytes != 1 && pp->elem_bytes != 4)) {
    bh_set_last_error("bh_pad: invalid parameters");
    return BH_EINVAL;
  }
  const bh_pad_params& p = *pp;
  bh::PadDivs dv{};
  long total = 1;
  for (int d = 0; d < 4; ++d) {
    if (p.in_shape[d] <= 0 || p.pad_before[d] < 0 || p.pad_after[d] < 0) {
      bh_set_last_error("bh_pad: bad shape");
      return BH_EINVAL;
    }
    // mirror pads index inside the input: REFLECT < dim, SYMMETRIC <= dim
    const int lim = p.in_shape[d] - (p.mode == 1 ? 1 : 0);
    if ((p.mode < 0 || p.mode > 2) || (p.mode && (p.pad_before[d] > lim || p.pad_after[d] > lim))) {
      bh_set_last_error("bh_pad: mirror pad wider than the input");
      return BH_EINVAL;
    }
    dv.os[d] = p.in_shape[d] + p.pad_before[d] + p.pad_after[d];
    total *= dv.os[d];
  }
  if (total >= INT32_MAX) {
    bh_set_last_error("bh_pad: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  dv.c = bh::FastDiv(dv.os[3]);
  dv.w = bh::FastDiv(dv.os[2]);
  dv.h = bh::FastDiv(dv.os[1]);
  if (p.elem_bytes == 1)
    BH_LAUNCH(bh::pad_kernel<uint8_t>, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, p, dv, total);
  else
    BH_LAUNCH(bh::pad_kernel<uint32_t>, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, p, dv, total);
  return bh_check_launch("pad_kernel");
}

extern "C" int bh_resize_nearest(const bh_resize_nearest_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || !pp->y_index || !pp->x_index || pp->batch <= 0 || pp->out_h <= 0 ||
      pp->out_w <= 0 || pp->row_bytes <= 0) {
    bh_set_last_error("bh_resize_nearest: invalid parameters");
    return BH_EINVAL;
  }
  const bh_resize_nearest_params& p = *pp;
  const long pixels = (long)p.batch * p.out_h * p.out_w;
  const bool v4 = p.row_bytes % 4 == 0 && (uintptr_t)p.input % 4 == 0 && (uintptr_t)p.output % 4 == 0;
  const int units = v4 ? p.row_bytes / 4 : p.row_bytes;
  const long total = pixels * units;
  if (pixels * p.row_bytes >= INT32_MAX) {
    bh_set_last_error("bh_resize_nearest: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  bh::ResizeDivs dv;
  dv.units = bh::FastDiv(units);
  dv.ow = bh::FastDiv(p.out_w);
  dv.oh = bh::FastDiv(p.out_h);
  if (v4)
    BH_LAUNCH(bh::resize_nearest_kernel<4>, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, p, dv, total);
  else
    BH_LAUNCH(bh::resize_nearest_kernel<1>, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, p, dv, total);
  return bh_check_launch("resize_nearest_kernel");
}

extern "C" int bh_resize_bilinear_i8(const bh_resize_bilinear_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || !pp->y_tab || !pp->x_tab || pp->batch <= 0 || pp->channels <= 0 ||
      pp->out_h <= 0 || pp->out_w <= 0) {
    bh_set_last_error("bh_resize_bilinear_i8: invalid parameters");
    return BH_EINVAL;
  }
  const bh_resize_bilinear_params& p = *pp;
  const long total = (long)p.batch * p.out_h * p.out_w * p.channels;
  if (total >= INT32_MAX || (long)p.batch * p.in_h * p.in_w * p.channels >= INT32_MAX) {
    bh_set_last_error("bh_resize_bilinear_i8: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  if ((long)p.in_w * p.channels <= bh::kRzRow && p.out_w <= bh::kRzCols &&
      (long)p.batch * p.out_h < INT32_MAX) {
    // 16-byte stores when every output row starts 16-byte aligned
    const int vec_ok = ((p.out_w * p.channels) % 16 == 0 && ((uintptr_t)p.output & 15) == 0) ? 1 : 0;
    const size_t lds = ((size_t)p.in_w * p.channels + 3 * (size_t)p.out_w) * sizeof(int32_t);
    if (p.channels >= 16 && lds <= 64 * 1024) {
      // output rows per workgroup: up to 8 while >= 1024 workgroups remain
      // and the blended rows fit 48 KB (4 at DeepLab's batch 24 / 32: 26.8
      // us at batch 32 against 30.0 for one row, 28.3 for 2, 30.1 for 8,
      // profiles/r06ah_resize_rows.txt)
      const size_t row_lds = (size_t)p.in_w * p.channels * sizeof(int32_t);
      int nr = 1;
      while (nr < 8 && (long)p.batch * ((p.out_h + 2 * nr - 1) / (2 * nr)) >= 1024 &&
             lds + (2 * nr - 1) * row_lds <= 48 * 1024)
        nr *= 2;
      const int groups = (p.out_h + nr - 1) / nr;
      const size_t lds_nr = lds + (size_t)(nr - 1) * row_lds;
      BH_LAUNCH(bh::resize_bilinear_cols_kernel, dim3(p.batch * groups), dim3(256), lds_nr, (hipStream_t)s, p,
                bh::FastDiv(p.channels), vec_ok, nr, bh::FastDiv(groups),
                bh::FastDiv((p.out_w * p.channels + 15) / 16));
      return bh_check_launch("resize_bilinear_cols_kernel");
    }
    BH_LAUNCH(bh::resize_bilinear_rows_kernel, dim3(p.batch * p.out_h), dim3(256), 0, (hipStream_t)s, p,
              bh::FastDiv(p.channels), vec_ok);
    return bh_check_launch("resize_bilinear_rows_kernel");
  }
  bh::ResizeDivs dv;
  dv.units = bh::FastDiv(p.channels);
  dv.ow = bh::FastDiv(p.out_w);
  dv.oh = bh::FastDiv(p.out_h);
  BH_LAUNCH(bh::resize_bilinear_kernel, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, p, dv, total);
  return bh_check_launch("resize_bilinear_kernel");
}

extern "C" int bh_softmax_i8(const bh_softmax_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || !pp->table || pp->rows < 0 || pp->depth <= 0) {
    bh_set_last_error("bh_softmax_i8: invalid parameters");
    return BH_EINVAL;
  }
  if (pp->rows == 0) return 0;
  BH_LAUNCH(bh::softmax_kernel, dim3(bh::blocks(pp->rows)), dim3(256), 0, (hipStream_t)s, *pp);
  return bh_check_launch("softmax_kernel");
}

extern "C" int bh_zero_insert(const bh_zero_insert_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || pp->batch <= 0 || pp->channels <= 0 || pp->stride_h <= 0 ||
      pp->stride_w <= 0 || pp->out_h != (pp->in_h - 1) * pp->stride_h + 1 ||
      pp->out_w != (pp->in_w - 1) * pp->stride_w + 1) {
    bh_set_last_error("bh_zero_insert: invalid parameters");
    return BH_EINVAL;
  }
  const bh_zero_insert_params& p = *pp;
  const long pixels = (long)p.batch * p.out_h * p.out_w;
  if (pixels * p.channels >= INT32_MAX) {
    bh_set_last_error("bh_zero_insert: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  const bool v4 = p.channels % 4 == 0 && (uintptr_t)p.input % 4 == 0 && (uintptr_t)p.output % 4 == 0;
  bh::ZiDivs dv;
  dv.units = bh::FastDiv(v4 ? p.channels / 4 : p.channels);
  dv.ow = bh::FastDiv(p.out_w);
  dv.oh = bh::FastDiv(p.out_h);
  dv.sh = bh::FastDiv(p.stride_h);
  dv.sw = bh::FastDiv(p.stride_w);
  const long total = pixels * dv.units.d;
  if (v4)
    BH_LAUNCH(bh::zero_insert_kernel<4>, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, p, dv, total);
  else
    BH_LAUNCH(bh::zero_insert_kernel<1>, dim3(bh::blocks(total)), dim3(256), 0, (hipStream_t)s, p, dv, total);
  return bh_check_launch("zero_insert_kernel");
}

// ---- MEAN ---------------------------------------------------------------
// reduce.cc EvalMean (TFLite 2.9.2): optimized_integer_ops::Mean (int8) /
// optimized_ops::Mean (uint8) sum the reduced window in int32, then
// MultiplyByQuantizedMultiplier + the float-derived bias, clamped to the
// type; float32 sums in order and divides by the count.  A thread owns one
// output; neighbouring threads are neighbouring `inner` (channel) indices,
// so every step of the reduction loop is one coalesced row read.
namespace bh {
__global__ __launch_bounds__(256) void mean_kernel(bh_mean_params p, long total) {
  const long o = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= total) return;
  const long a = o / p.inner;
  const long c = o - a * p.inner;
  const long base = a * p.reduce * p.inner + c;
  if (p.type == 0) {
    const float* x = (const float*)p.input;
    float s = 0.f;
    for (long r = 0; r < p.reduce; ++r) s = __fadd_rn(s, x[base + r * p.inner]);
    ((float*)p.output)[o] = __fdiv_rn(s, (float)p.reduce);
    return;
  }
  int32_t acc = 0;
  if (p.type == 1) {
    const int8_t* x = (const int8_t*)p.input;
    for (long r = 0; r < p.reduce; ++r) acc += x[base + r * p.inner];
  } else {
    const uint8_t* x = (const uint8_t*)p.input;
    for (long r = 0; r < p.reduce; ++r) acc += x[base + r * p.inner];
  }
  acc = requant(acc, p.multiplier, p.shift) + p.bias;
  if (p.type == 1) ((int8_t*)p.output)[o] = (int8_t)clamp_i32(acc, -128, 127);
  else ((uint8_t*)p.output)[o] = (uint8_t)clamp_i32(acc, 0, 255);
}
}  // namespace bh

extern "C" int bh_mean(const bh_mean_params* pp, bh_stream_t stream) {
  if (!pp || pp->outer <= 0 || pp->reduce <= 0 || pp->inner <= 0 || pp->type < 0 || pp->type > 2 || !pp->input ||
      !pp->output || pp->reduce * 255 >= (1l << 31)) {
    bh_set_last_error("bh_mean: invalid parameters");
    return BH_EINVAL;
  }
  const long total = pp->outer * pp->inner;
  BH_LAUNCH(bh::mean_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *pp, total);
  return bh_check_launch("mean_kernel");
}

// ---- RESIZE_BILINEAR uint8 ----------------------------------------------------
// optimized_ops::ResizeBilinear<uint8> (TFLite 2.9.2) -> ResizeBilinear-
// GenericSmallChannel: the four weights and the weighted sum in float, in
// the reference's operation order (explicit _rn intrinsics: no contraction),
// + 0.5f, truncated to uint8.  One thread per output byte; the float
// interpolation coordinates come from host tables (ComputeInterpolationValues).
namespace bh {
__global__ __launch_bounds__(256) void resize_bilinear_u8_kernel(bh_resize_bilinear_u8_params p, ResizeDivs dv,
                                                                 long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int pix = (int)dv.units.div((uint32_t)i);
  const int c = (int)(i - (long)pix * p.channels);
  const int t = (int)dv.ow.div((uint32_t)pix);
  const int x = pix - t * p.out_w;
  const int n = (int)dv.oh.div((uint32_t)t);
  const int y = t - n * p.out_h;
  const int y0 = p.y_idx[2 * y], y1 = p.y_idx[2 * y + 1];
  const int x0 = p.x_idx[2 * x], x1 = p.x_idx[2 * x + 1];
  const float dy = p.y_frac[y], dx = p.x_frac[x];
  const float s0 = __fmul_rn(__fsub_rn(1.0f, dy), __fsub_rn(1.0f, dx));
  const float s1 = __fmul_rn(__fsub_rn(1.0f, dy), dx);
  const float s2 = __fmul_rn(dy, __fsub_rn(1.0f, dx));
  const float s3 = __fmul_rn(dy, dx);
  const uint8_t* b = (const uint8_t*)p.input + (long)n * p.in_h * p.in_w * p.channels;
  const float a0 = (float)b[((long)y0 * p.in_w + x0) * p.channels + c];
  const float a1 = (float)b[((long)y0 * p.in_w + x1) * p.channels + c];
  const float a2 = (float)b[((long)y1 * p.in_w + x0) * p.channels + c];
  const float a3 = (float)b[((long)y1 * p.in_w + x1) * p.channels + c];
  float v = __fadd_rn(__fmul_rn(a0, s0), __fmul_rn(a1, s1));
  v = __fadd_rn(v, __fmul_rn(a2, s2));
  v = __fadd_rn(v, __fmul_rn(a3, s3));
  v = __fadd_rn(v, 0.5f);
  ((uint8_t*)p.output)[i] = (uint8_t)(int)v;
}
}  // namespace bh

extern "C" int bh_resize_bilinear_u8(const bh_resize_bilinear_u8_params* pp, bh_stream_t s) {
  if (!pp || !pp->input || !pp->output || !pp->y_idx || !pp->x_idx || !pp->y_frac || !pp->x_frac || pp->batch <= 0 ||
      pp->in_h <= 0 || pp->in_w <= 0 || pp->channels <= 0 || pp->out_h <= 0 || pp->out_w <= 0) {
    bh_set_last_error("bh_resize_bilinear_u8: invalid parameters");
    return BH_EINVAL;
  }
  const bh_resize_bilinear_u8_params& p = *pp;
  const long total = (long)p.batch * p.out_h * p.out_w * p.channels;
  if (total >= INT32_MAX) {
    bh_set_last_error("bh_resize_bilinear_u8: tensor too large for 32-bit indexing");
    return BH_EINVAL;
  }
  bh::ResizeDivs dv;
  dv.units = bh::FastDiv(p.channels);
  dv.ow = bh::FastDiv(p.out_w);
  dv.oh = bh::FastDiv(p.out_h);
  BH_LAUNCH(bh::resize_bilinear_u8_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)s, p, dv,
            total);
  return bh_check_launch("resize_bilinear_u8_kernel");
}
