// Fused MobileNet inverted-residual block for gfx950 (int8 per-channel):
//   [CONV_2D 1x1 expand ->] DEPTHWISE_CONV_2D 3x3 -> CONV_2D 1x1 project [-> ADD]
//
// Stands in for 3-4 consecutive TFLite 2.9.2 builtin kernels on Band's hot
// path (band/backend/tfl/model_executor.cc:249-255 -> Interpreter::Invoke):
// reference_integer_ops::ConvPerChannel (expand), DepthwiseConvPerChannel,
// ConvPerChannel (project) and reference_integer_ops::Add.  Every
// intermediate is requantised to its own 8-bit tensor exactly as TFLite
// stores it, so the result is bit-identical to running the ops one by one.
//
// MI355X design: one launch per block instead of 3-4 (each launch costs a
// few microseconds at batch 1), and the expanded activation - the largest
// tensor of the block - never leaves the CU:
//   phase 0  input region (output tile + dw halo) HBM -> LDS
//   phase 1  expand GEMM on v_mfma_i32_16x16x64_i8, A from LDS, requant -> LDS
//   phase 2  depthwise 3x3 on VALU from LDS, requant -> LDS
//   phase 3  project GEMM on MFMA, split-K over waves, int32 partials summed
//            with LDS atomics into the (dead) phase-1 buffer
//   phase 4  requant + residual ADD by all threads, coalesced stores -> HBM
// A workgroup of NW waves owns tile_h x tile_w output pixels of one image.
// Work inside a phase is a flat list of 16x16 MFMA tiles dealt round-robin
// to the waves, so no wave runs a long serial chain (at batch 1 a block has
// few workgroups; latency, not FLOPs, is the cost).
#include "common.hpp"

namespace bh {

struct IrbGeom {
  int RH, RW, R;        // input region (tile + halo) in dw-input pixels
  int cin_p, xs;        // K-padded input channels, LDS row stride of x
  int es;               // LDS row stride of the expanded tensor
  int ce_p, ds;         // K-padded expanded channels, LDS row stride of dw output
  int T, MT1, MT3;      // tile pixels, 16-row tiles of region / tile
  int np3;              // padded output channels (phase-3 accumulator row)
  size_t x_off, e_off, d_off, a_off, w_off, bytes;
  // w region: dw filter [9][ce16] bytes, then int32 dw bias/mult/shift [ce],
  // then int32 project bias_eff/mult/shift [out_c]
  int ce16;
};

__host__ __device__ inline IrbGeom irb_geom(const bh_irb_params& p) {
  IrbGeom g;
  g.RH = (p.tile_h - 1) * p.stride + 3;
  g.RW = (p.tile_w - 1) * p.stride + 3;
  g.R = g.RH * g.RW;
  g.cin_p = (p.in_c + 63) / 64 * 64;
  g.xs = g.cin_p + 16;
  g.es = (p.exp_c + 15) / 16 * 16 + 16;
  g.ce_p = (p.exp_c + 63) / 64 * 64;
  g.ds = g.ce_p + 16;
  g.T = p.tile_h * p.tile_w;
  g.MT1 = (g.R + 15) / 16;
  g.MT3 = (g.T + 15) / 16;
  g.np3 = (p.out_c + 15) / 16 * 16;
  g.x_off = 0;
  const size_t xb = p.has_expand ? (size_t)g.MT1 * 16 * g.xs : 0;
  g.e_off = xb;
  // int32 phase-3 accumulators get their own region, zeroed during phase 0
  // (no extra barrier)
  const size_t eb = (size_t)g.R * g.es;
  g.d_off = (g.e_off + eb + 15) / 16 * 16;
  g.a_off = (g.d_off + (size_t)g.MT3 * 16 * g.ds + 15) / 16 * 16;
  g.w_off = (g.a_off + (size_t)g.MT3 * 16 * g.np3 * 4 + 15) / 16 * 16;
  g.ce16 = (p.exp_c + 15) / 16 * 16;
  g.bytes = g.w_off + 9 * (size_t)g.ce16 + 12 * (size_t)g.ce16 + 12 * (size_t)p.out_c;
  return g;
}

// Runtime divisors of the kernel's index math, as multiply-high reciprocals
// (see FastDiv): built once on the host per launch.
struct IrbDivs {
  FastDiv upr;     // 8-byte (expand) / 4-byte (no expand) units per region row
  FastDiv rw;      // region width
  FastDiv groups;  // exp_c / 4
  FastDiv expc;    // exp_c (one-channel depthwise items)
  FastDiv tile_w;
  FastDiv out_c;
  FastDiv mt1;     // 16-row tiles of the region
  FastDiv mt3;     // 16-row tiles of the output tile
  FastDiv ksplit;
};

template <int NW>
__global__ __launch_bounds__(NW * 64) void irb_kernel(bh_irb_params p, int ksplit, int kper, IrbDivs dv) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NT = NW * 64;
  const IrbGeom G = irb_geom(p);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const int n = blockIdx.z;
  const int oy0 = blockIdx.y * p.tile_h;
  const int ox0 = blockIdx.x * p.tile_w;
  const int ry0 = oy0 * p.stride - p.pad_h;  // image coords of region (0,0)
  const int rx0 = ox0 * p.stride - p.pad_w;
  const int8_t* x = (const int8_t*)p.input + (long)n * p.in_h * p.in_w * p.in_c;
  unsigned long long* stamps =
      p.debug_stamps ? (unsigned long long*)p.debug_stamps +
                           16 * (((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x)
                     : nullptr;
#define IRB_STAMP(k) \
  if (stamps && tid == 0) stamps[k] = __builtin_amdgcn_s_memrealtime();
  IRB_STAMP(0)
  const unsigned long long clk0 = stamps ? __builtin_amdgcn_s_memtime() : 0ull;
  unsigned char* xl = smem + G.x_off;
  unsigned char* el = smem + G.e_off;
  unsigned char* dl = smem + G.d_off;
  unsigned char* wl = smem + G.w_off;                                // dw filter
  int* dwt = (int*)(wl + 9 * G.ce16);                                // dw bias | mult | shift
  int* pjt = dwt + 3 * G.ce16;                                       // proj bias_eff | mult | shift

  const int NT1 = p.exp_c / 16;
  const int KS1 = G.cin_p / 64;  // <= 4 (host-checked)
  const int NT3 = G.np3 / 16;
  const int KS3 = G.ce_p / 64;
  // Expand filter fragments + tables of this wave's first phase-1 item: issued
  // first, so their latency hides behind the prologue.
  const int n_items1 = p.has_expand ? G.MT1 * NT1 : 0;
  v4i b1[4];
  int32_t be1 = 0, mu1 = 0, sh1 = 0;
  auto load_b1 = [&](int item, v4i* b, int32_t& be, int32_t& mu, int32_t& sh) {
    const int col = dv.mt1.div(item) * 16 + r16;
    const int8_t* wrow = p.exp_w + (long)col * p.exp_k_pad + g * 16;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      if (ks < KS1) b[ks] = *(const v4i*)(wrow + ks * 64);
    be = p.exp_bias_eff[col];
    mu = p.exp_mult[col];
    sh = p.exp_shift[col];
  };
  if (wave < n_items1) load_b1(wave, b1, be1, mu1, sh1);

  // ---- phase 0: depthwise filter + int32 tables + input region -> LDS -------
  // One loop, each iteration issuing ALL its loads (tables, filter, a batch of
  // region units) before any store, so the prologue costs one memory round
  // trip per iteration (usually one).
  {
    const int n16 = 9 * p.exp_c / 16;  // dw filter [9][exp_c], exp_c % 16 == 0
    const int c16 = p.exp_c / 4;
    const int p16 = p.out_c / 4;       // out_c % 4 == 0 (host-checked)
    const int span = max(n16, max(c16, p16));
    // region: 8-byte units (expand input; pad pixels = x_zp, K tail = 0) or
    // 4-byte units (no expand: the region is the depthwise input)
    const int upr = p.has_expand ? G.cin_p / 8 : p.in_c / 4;
    const int units = p.has_expand ? G.MT1 * 16 * upr : G.R * upr;
    const uint32_t zpw = splat_byte(p.x_zp);
    for (int it = 0; it * NT < span || it * 4 * NT < units; ++it) {
      const int u = it * NT + tid;
      v4i w = {0, 0, 0, 0}, t0 = w, t1 = w, t2 = w, q0 = w, q1 = w, q2 = w;
      if (u < n16) w = *(const v4i*)(p.dw_w + u * 16);
      if (u < c16) {
        t0 = *(const v4i*)(p.dw_bias + u * 4);
        t1 = *(const v4i*)(p.dw_mult + u * 4);
        t2 = *(const v4i*)(p.dw_shift + u * 4);
      }
      if (u < p16) {
        q0 = *(const v4i*)(p.proj_bias_eff + u * 4);
        q1 = *(const v4i*)(p.proj_mult + u * 4);
        q2 = *(const v4i*)(p.proj_shift + u * 4);
      }
      v2i v[4];
      int dst[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ru = it * 4 * NT + j * NT + tid;
        dst[j] = -1;
        v[j] = (v2i){0, 0};
        if (ru >= units) continue;
        const int r = dv.upr.div(ru);
        if (p.has_expand) {
          const int k = (ru - r * upr) * 8;
          dst[j] = r * G.xs + k;
          if (r < G.R && k < p.in_c) {
            const int ry = dv.rw.div(r);
            const int iy = ry0 + ry, ix = rx0 + (r - ry * G.RW);
            if (iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w)
              v[j] = *(const v2i*)(x + ((long)iy * p.in_w + ix) * p.in_c + k);
            else
              v[j] = (v2i){(int)zpw, (int)zpw};
          }
        } else {
          const int k = (ru - r * upr) * 4;
          dst[j] = r * G.es + k;
          const int ry = dv.rw.div(r);
          const int iy = ry0 + ry, ix = rx0 + (r - ry * G.RW);
          if (iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w)
            v[j].x = *(const int*)(x + ((long)iy * p.in_w + ix) * p.in_c + k);
        }
      }
      if (u < n16) *(v4i*)(wl + u * 16) = w;
      if (u < c16) {
        *(v4i*)(dwt + u * 4) = t0;
        *(v4i*)(dwt + G.ce16 + u * 4) = t1;
        *(v4i*)(dwt + 2 * G.ce16 + u * 4) = t2;
      }
      if (u < p16) {
        *(v4i*)(pjt + u * 4) = q0;
        *(v4i*)(pjt + p.out_c + u * 4) = q1;
        *(v4i*)(pjt + 2 * p.out_c + u * 4) = q2;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (dst[j] < 0) continue;
        if (p.has_expand) *(v2i*)(xl + dst[j]) = v[j];
        else *(int*)(el + dst[j]) = v[j].x;
      }
    }
  }
  int* accl = (int*)(smem + G.a_off);
  for (int i = tid; i < G.MT3 * 16 * G.np3; i += NT) accl[i] = 0;
  __syncthreads();
  IRB_STAMP(1)

  // ---- phase 1: expand 1x1 (MFMA) -> LDS --------------------------------
  if (p.has_expand) {
    // software pipeline: the next item's filter fragments and tables are in
    // flight while this item multiplies and requantises
    for (int item = wave; item < n_items1; item += NW) {
      const int nt = dv.mt1.div(item);
      const int mt = item - nt * G.MT1;
      const int col = nt * 16 + r16;
      v4i bn[4];
      int32_t ben = 0, mun = 0, shn = 0;
      const bool next = item + NW < n_items1;
      if (next) load_b1(item + NW, bn, ben, mun, shn);
      v4i acc = (v4i){0, 0, 0, 0};
      const unsigned char* arow = xl + (mt * 16 + r16) * G.xs + g * 16;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        if (ks < KS1) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(*(const v4i*)(arow + ks * 64), b1[ks], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + 4 * g + r;
        if (row < G.R) {
          const int32_t v = requant_clamp(acc[r] + be1, mu1, sh1, p.e_zp, p.e_act_min, p.e_act_max, p.requant_fast & 1);
          el[row * G.es + col] = (unsigned char)v;
        }
      }
      if (next) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) b1[ks] = bn[ks];
        be1 = ben;
        mu1 = mun;
        sh1 = shn;
      }
    }
    __syncthreads();
  }
  IRB_STAMP(2)

  const int n_items3 = G.MT3 * NT3 * ksplit;

  // ---- phase 2: depthwise 3x3 (VALU) -> LDS -----------------------------
  // Only the T tile rows are produced: the MFMA padding rows of dl feed
  // accumulator rows phase 4 never reads, and the K tail of the project
  // operand meets zero-packed weights, so neither needs initialising.  Four
  // channels per item when that still covers every thread, else one (small
  // tiles: a 4x shorter per-thread chain).
  if (G.T * (p.exp_c / 4) >= NT) {
    const int groups = p.exp_c / 4;
    for (int it = tid; it < G.T * groups; it += NT) {
      const int pi = dv.groups.div(it);
      const int c0 = (it - pi * groups) * 4;
      uint32_t packed = 0;
      const int ty = dv.tile_w.div(pi);
      const int tx = pi - ty * p.tile_w;
      const int oy = oy0 + ty;
      const int ox = ox0 + tx;
      if (oy < p.out_h && ox < p.out_w) {
        int32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
        for (int fy = 0; fy < 3; ++fy) {
          const int iy = oy * p.stride - p.pad_h + fy;
          if (iy < 0 || iy >= p.in_h) continue;
#pragma unroll
          for (int fx = 0; fx < 3; ++fx) {
            const int ix = ox * p.stride - p.pad_w + fx;
            if (ix < 0 || ix >= p.in_w) continue;
            const int er = (ty * p.stride + fy) * G.RW + tx * p.stride + fx;
            const uint32_t ev = *(const uint32_t*)(el + er * G.es + c0);
            const uint32_t wv = *(const uint32_t*)(wl + (fy * 3 + fx) * G.ce16 + c0);
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[b] += (sbyte(ev, b) - p.e_zp) * sbyte(wv, b);
          }
        }
        const v4i bb = *(const v4i*)(dwt + c0);
        const v4i mm = *(const v4i*)(dwt + G.ce16 + c0);
        const v4i ss = *(const v4i*)(dwt + 2 * G.ce16 + c0);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int32_t v = requant_clamp(acc[b] + bb[b], mm[b], ss[b], p.d_zp, p.d_act_min, p.d_act_max, p.requant_fast & 2);
          packed |= ((uint32_t)v & 0xffu) << (8 * b);
        }
      }
      *(uint32_t*)(dl + pi * G.ds + c0) = packed;
    }
  } else {
    for (int it = tid; it < G.T * p.exp_c; it += NT) {
      const int pi = dv.expc.div(it);
      const int c = it - pi * p.exp_c;
      const int ty = dv.tile_w.div(pi);
      const int tx = pi - ty * p.tile_w;
      const int oy = oy0 + ty, ox = ox0 + tx;
      int32_t v = 0;
      if (oy < p.out_h && ox < p.out_w) {
        int32_t acc = 0;
#pragma unroll
        for (int fy = 0; fy < 3; ++fy) {
          const int iy = oy * p.stride - p.pad_h + fy;
          if (iy < 0 || iy >= p.in_h) continue;
#pragma unroll
          for (int fx = 0; fx < 3; ++fx) {
            const int ix = ox * p.stride - p.pad_w + fx;
            if (ix < 0 || ix >= p.in_w) continue;
            const int er = (ty * p.stride + fy) * G.RW + tx * p.stride + fx;
            acc += ((int32_t)(int8_t)el[er * G.es + c] - p.e_zp) * (int32_t)(int8_t)wl[(fy * 3 + fx) * G.ce16 + c];
          }
        }
        v = requant_clamp(acc + dwt[c], dwt[G.ce16 + c], dwt[2 * G.ce16 + c], p.d_zp, p.d_act_min, p.d_act_max,
                          p.requant_fast & 2);
      }
      dl[pi * G.ds + c] = (unsigned char)v;
    }
  }
  __syncthreads();
  IRB_STAMP(3)
  IRB_STAMP(4)

  // ---- phase 3: project 1x1 (MFMA), split-K, LDS-atomic accumulation -----
  {
    for (int item = wave; item < n_items3; item += NW) {
      const int tile = dv.ksplit.div(item);
      const int kz = item - tile * ksplit;
      const int nt = dv.mt3.div(tile);
      const int mt = tile - nt * G.MT3;
      const int col = nt * 16 + r16;
      const int8_t* wrow = p.proj_w + (long)col * p.proj_k_pad + g * 16;
      const unsigned char* arow = dl + (mt * 16 + r16) * G.ds + g * 16;
      const int k_begin = kz * kper;
      const int k_end = min(KS3, k_begin + kper);
      v4i acc = (v4i){0, 0, 0, 0};
      for (int k0 = k_begin; k0 < k_end; k0 += 4) {
        v4i a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (k0 + u < k_end) {
            b[u] = *(const v4i*)(wrow + (k0 + u) * 64);
            a[u] = *(const v4i*)(arow + (k0 + u) * 64);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (k0 + u < k_end) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b[u], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(&accl[(mt * 16 + 4 * g + r) * G.np3 + col], acc[r]);
    }
  }
  __syncthreads();
  IRB_STAMP(5)

  // ---- phase 4: requant + residual ADD, coalesced stores ------------------
  {
    int8_t* out = (int8_t*)p.output + (long)n * p.out_h * p.out_w * p.out_c;
    const int total = G.T * p.out_c;
    for (int i0 = tid; i0 < total; i0 += 4 * NT) {
      int32_t q[4];
      long o[4];
      bool ok[4];
      int pis[4], cols[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int idx = i0 + j * NT;
        const int pi = dv.out_c.div(idx);
        const int col = idx - pi * p.out_c;
        pis[j] = pi;
        cols[j] = col;
        const int ty = dv.tile_w.div(pi);
        const int tx = pi - ty * p.tile_w;
        const int oy = oy0 + ty;
        const int ox = ox0 + tx;
        ok[j] = idx < total && oy < p.out_h && ox < p.out_w;
        o[j] = ((long)oy * p.out_w + ox) * p.out_c + col;
        q[j] = 0;
        if (ok[j] && p.has_residual) {
          // stride 1, in_c == out_c: the block input pixel sits in the staged
          // region at (ty + pad, tx + pad); without expand read it from HBM
          q[j] = p.has_expand ? (int32_t)(int8_t)xl[((ty + p.pad_h) * G.RW + tx + p.pad_w) * G.xs + col]
                              : (int32_t)x[o[j]];
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!ok[j]) continue;
        const int pi = pis[j];
        const int col = cols[j];
        int32_t v = accl[pi * G.np3 + col] + pjt[col];
        v = requant_clamp(v, pjt[p.out_c + col], pjt[2 * p.out_c + col], p.p_zp, p.p_act_min, p.p_act_max,
                          p.requant_fast & 4);
        if (p.has_residual) {
          const int32_t sp = requant_lt1((v + p.add_p_off) * (1 << p.add_left_shift), p.add_p_mult, p.add_p_shift);
          const int32_t sx = requant_lt1((q[j] + p.add_x_off) * (1 << p.add_left_shift), p.add_x_mult, p.add_x_shift);
          v = clamp_i32(requant_lt1(sp + sx, p.add_o_mult, p.add_o_shift) + p.add_o_off, p.add_act_min, p.add_act_max);
        }
        out[o[j]] = (int8_t)v;
      }
    }
  }
  IRB_STAMP(6)
  if (stamps && tid == 0) stamps[7] = __builtin_amdgcn_s_memtime() - clk0;  // shader clocks
#undef IRB_STAMP
}

template <int NW>
static int launch_irb(const bh_irb_params& p, size_t lds, hipStream_t s) {
  if (lds > 64 * 1024) {
    // opt in to the CU's full 160 KiB of LDS for this kernel (once per device)
    static thread_local int opted_device = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (opted_device != dev) {
      (void)hipFuncSetAttribute((const void*)irb_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      opted_device = dev;
    }
  }
  const IrbGeom G = irb_geom(p);
  const int tiles3 = G.MT3 * (G.np3 / 16);
  const int KS3 = G.ce_p / 64;
  int ksplit = 1;
  while (ksplit < 4 && tiles3 * ksplit < NW && ksplit * 2 <= KS3) ksplit *= 2;
  IrbDivs dv;
  dv.upr = FastDiv(p.has_expand ? G.cin_p / 8 : p.in_c / 4);
  dv.rw = FastDiv(G.RW);
  dv.groups = FastDiv(p.exp_c / 4);
  dv.expc = FastDiv(p.exp_c);
  dv.tile_w = FastDiv(p.tile_w);
  dv.out_c = FastDiv(p.out_c);
  dv.mt1 = FastDiv(G.MT1);
  dv.mt3 = FastDiv(G.MT3);
  dv.ksplit = FastDiv(ksplit);
  dim3 grid((p.out_w + p.tile_w - 1) / p.tile_w, (p.out_h + p.tile_h - 1) / p.tile_h, p.batch);
  BH_LAUNCH(irb_kernel<NW>, grid, dim3(NW * 64), lds, s, p, ksplit, (KS3 + ksplit - 1) / ksplit, dv);
  return bh_check_launch("irb_kernel");
}

}  // namespace bh

extern "C" size_t bh_irb_lds_bytes(const bh_irb_params* pp) {
  if (!pp) return 0;
  const bh_irb_params& p = *pp;
  if (p.tile_h <= 0 || p.tile_w <= 0 || (p.stride != 1 && p.stride != 2)) return 0;
  if (p.exp_c % 16 || p.exp_c <= 0 || p.out_c % 4) return 0;
  if (p.has_expand && (p.in_c % 8 || (p.in_c + 63) / 64 > 4 || p.exp_k_pad != (p.in_c + 63) / 64 * 64)) return 0;
  if (!p.has_expand && (p.in_c != p.exp_c || p.in_c % 4)) return 0;
  if (p.proj_k_pad != (p.exp_c + 63) / 64 * 64) return 0;
  if (p.has_residual && (p.stride != 1 || p.in_c != p.out_c || p.in_h != p.out_h || p.in_w != p.out_w)) return 0;
  const bh::IrbGeom g = bh::irb_geom(p);
  return g.bytes <= 160 * 1024 ? g.bytes : 0;
}

extern "C" int bh_irb_i8(const bh_irb_params* pp, bh_stream_t stream) {
  const size_t lds = bh_irb_lds_bytes(pp);
  if (!pp || lds == 0 || !pp->input || !pp->output || !pp->dw_w || !pp->proj_w ||
      (pp->has_expand && !pp->exp_w) || pp->batch <= 0) {
    bh_set_last_error("bh_irb_i8: invalid or unsupported parameters");
    return BH_EINVAL;
  }
  // 16 waves: at batch 1 a block has fewer workgroups than CUs, so each
  // workgroup owns a CU anyway and more waves shorten every phase's item chain
  return bh::launch_irb<16>(*pp, lds, (hipStream_t)stream);
}
