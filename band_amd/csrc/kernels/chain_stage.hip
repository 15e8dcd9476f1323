// Fused pointwise chain, raster form with staged filters ("stage" form), for
// gfx950 (int8 per-channel):
//   DEPTHWISE_CONV_2D 3x3 -> CONV_2D 1x1 [-> ADD residual] -> CONV_2D 1x1
//
// The same three TFLite 2.9.2 builtin kernels as chain_kernel
// (fused_chain.hip: reference_integer_ops::DepthwiseConvPerChannel,
// ConvPerChannel [+ the residual ADD folded into its epilogue], ConvPerChannel
// - Band's hot path band/backend/tfl/model_executor.cc:249-255 ->
// Interpreter::Invoke), every intermediate requantised exactly as TFLite
// stores it, so the result is bit-identical to the unfused launches.
//
// Why a third raster form.  On the few-pixel layers (28x28 stride 2, 14x14,
// 7x7) chain_kernel's workgroup owns 16 pixels and streams both 1x1 filters
// from L2 two channel tiles per round trip: a workgroup is a chain of 6-10
// dependent L2 round trips (phase B and C alone are ~58 % of its time,
// profiles/r05ba_chain_*), each filter byte serving 16 pixels.  Here the
// workgroup issues ONE burst of LDS-DMA (global_load_lds, no VGPR staging) at
// its start - the first 1x1's filter and tables, ITS slice of the second 1x1's
// filter and tables (the packed constant block of bh_chain_tile_pack), and
// the residual rows - then runs the depthwise phase from global memory while
// the burst lands, and both 1x1 GEMMs from LDS only:
//   A  depthwise on the matrix cores (chain_dw_mfma, as chain_kernel)
//   B  first 1x1 from LDS W1 [+ residual ADD from the DMA'd rows] -> LDS
//   C  second 1x1, this workgroup's channel slice (grid.y), from LDS W2
// and the slice leaves with 16-byte stores.  The slices of one pixel block
// recompute A and B (grid.y = c_split up to 8), so a 14x14 layer at batch 1
// still spreads over ~100 workgroups.
#include <algorithm>

#include "chain_blob.hpp"
#include "chain_dw.hpp"
#include "common.hpp"

namespace bh {

// LDS layout (bytes, every region 16-byte aligned): W1 | b1 m1 s1 (the blob's
// first run, verbatim) | W2 slice [TS*16][k2] | b2 m2 s2 slices [TS*16] each |
// dl [rows][S1] | pl [rows][S2] | o1 [rows][N1] | residual [rows][N1] | add
// tables | phase-C staging (in dl when it fits)
struct StageGeom {
  int S1, S2;        // row strides: depthwise output / the second 1x1's operand
  int TS;            // channel tiles of a phase-C slice (at most)
  int w1_bytes;      // blob [0, w2): W1 and its tables
  int blob_w2, blob_b2, blob_m2, blob_s2;
  int off_w2, off_t2, off_dl, off_pl, off_o1, off_res, off_add, off_out;
  int out_pitch;     // bytes per pixel of the phase-C staging
  size_t bytes;
};

static size_t up16(size_t v) { return (v + 15) / 16 * 16; }

static StageGeom stage_geom(const bh_chain_params& p) {
  StageGeom G{};
  const TileBlob B = tile_blob(p);
  const int rows = p.px_blocks * 16;
  const int N1 = p.pw1.out_c, N2 = p.pw2.out_c;
  const int T2 = (N2 + 15) / 16;
  const int S = std::max(1, p.c_split);
  G.TS = (T2 + S - 1) / S;
  // rows of k_pad + 32 bytes: a ds_read_b128 lane group's 16 rows land on 16
  // distinct bank slots (as chain_kernel / chain_tile_kernel)
  G.S1 = p.pw1.k_pad + 32;
  G.S2 = p.pw2.k_pad + 32;
  G.w1_bytes = B.w2;
  G.blob_w2 = B.w2;
  G.blob_b2 = B.b2;
  G.blob_m2 = B.m2;
  G.blob_s2 = B.s2;
  size_t o = B.w2;
  G.off_w2 = (int)o;
  o += (size_t)G.TS * 16 * p.pw2.k_pad;
  G.off_t2 = (int)o;
  o += 3 * (size_t)G.TS * 64;
  G.off_dl = (int)o;
  o += (size_t)rows * G.S1;
  G.off_pl = (int)o;
  o += (size_t)rows * G.S2;
  G.off_o1 = (int)o;
  o += p.pw1.output ? up16((size_t)rows * N1) : 0;
  G.off_res = (int)o;
  o += p.pw1.residual ? up16((size_t)rows * N1) : 0;
  G.off_add = (int)o;
  o += p.pw1.residual ? 512 * 4 : 0;
  // staged pixels 4 apart (one quad-transposed ds_write_b32 lane pair) sit 4
  // pitches apart: a pitch of 0 mod 32 would put them on one bank
  const int cw = G.TS * 16;
  G.out_pitch = cw % 32 == 0 ? cw + 16 : cw;
  if ((size_t)rows * G.out_pitch <= (size_t)rows * G.S1) {
    G.off_out = G.off_dl;  // the depthwise output is dead after phase B
  } else {
    G.off_out = (int)o;
    o += (size_t)rows * G.out_pitch;
  }
  G.bytes = up16(o);
  return G;
}

// `bytes` (a multiple of 4) contiguous bytes LDS -> HBM, 16-byte stores
__device__ __forceinline__ void stage_copy_rows(const unsigned char* src, uint8_t* dst, int bytes, int tid,
                                                int nthreads) {
  const int n16 = bytes >> 4;
  for (int i = tid; i < n16; i += nthreads) *(v4i*)(dst + i * 16) = *(const v4i*)(src + i * 16);
  const int rem = (bytes - (n16 << 4)) >> 2;
  if (tid < rem) *(uint32_t*)(dst + n16 * 16 + tid * 4) = *(const uint32_t*)(src + n16 * 16 + tid * 4);
}

// `rows` pixels' channel slice [c0, c0 + cw) from the staging (pitch bytes
// per pixel) to the NHWC tensor of Nc channels
__device__ __forceinline__ void stage_copy_out(const unsigned char* src, int pitch, uint8_t* dst, int Nc, int c0,
                                               int cw, int rows, int tid, int nthreads) {
  const bool v16 = ((c0 | cw | Nc) & 15) == 0;
  const int u = v16 ? cw >> 4 : cw >> 2;  // units per pixel (cw % 4 == 0)
  const float rcp = 1.0f / (float)u;      // i / u in float: exact for i < 2^16
  for (int i = tid; i < rows * u; i += nthreads) {
    const int r = (int)(((float)i + 0.5f) * rcp);
    const int k = i - r * u;
    if (v16) *(v4i*)(dst + (long)r * Nc + c0 + k * 16) = *(const v4i*)(src + r * pitch + k * 16);
    else *(uint32_t*)(dst + (long)r * Nc + c0 + k * 4) = *(const uint32_t*)(src + r * pitch + k * 4);
  }
}

// LW: loader waves.  0 - every wave issues its share of the burst, then
// runs phase A (whose first tap loads then queue behind the burst in the
// wave's own in-order memory counter); > 0 - the last LW waves issue the
// whole burst and the first NW - LW run phase A meanwhile, so the depthwise
// loads and the burst are in flight together
template <int RB, bool FAST, int KX, int NW, int LW>
__global__ __launch_bounds__(NW * 64) void chain_stage_kernel(bh_chain_params cp, int P, StageGeom G, ChainDivs dv) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int WPB = NW / RB;  // waves per pixel block
  constexpr int NA = NW - LW;   // phase-A waves
  constexpr int NL = LW ? LW : NW;  // waves issuing the burst
  static_assert(NA % RB == 0, "phase-A waves cover every pixel block");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const int pb = wave % RB;
  const int wsub = wave / RB;
  const int blk = xcd_block(blockIdx.x, gridDim.x);
  const int m0 = blk * RB * 16;
  const int rows = min(RB * 16, P - m0);
  const int m = m0 + pb * 16 + r16;
  const int orow = pb * 16 + 4 * g;  // first of this lane's 4 result rows
  const bh_conv_params& a = cp.pw1;
  const bh_conv_params& b = cp.pw2;
  const int N1 = a.out_c, N2 = b.out_c;
  const int T1 = (N1 + 15) >> 4, T2 = (N2 + 15) >> 4;
  // this workgroup's channel tiles of the second 1x1 (as chain_kernel's split)
  const int t_lo = (int)blockIdx.y * T2 / (int)gridDim.y;
  const int t_hi = ((int)blockIdx.y + 1) * T2 / (int)gridDim.y;
  const int nt = t_hi - t_lo;
  unsigned char* dl = smem + G.off_dl;
  unsigned char* pl = smem + G.off_pl;
  unsigned char* o1 = smem + G.off_o1;
  unsigned char* ol = smem + G.off_out;
  const unsigned char* resl = smem + G.off_res;

  // ---- LDS-DMA burst: W1 + tables, this slice of W2 + tables, residual ----
  if (LW == 0 || wave >= NA) {
    const int lw = LW ? wave - NA : wave;
    const unsigned char* blob = (const unsigned char*)cp.tile_blob;
    auto run16 = [&](const unsigned char* src, unsigned char* dst, int units) {
      for (int base = lw * 64; base < units; base += NL * 64)
        if (base + lane < units) dma16(src + (base + lane) * 16, dst + base * 16);
    };
    run16(blob, smem, G.w1_bytes >> 4);
    run16(blob + G.blob_w2 + (long)t_lo * 16 * b.k_pad, smem + G.off_w2, nt * b.k_pad);  // nt*16 rows / 16
    // 64 bytes (4 units) of each table per channel tile; a last tile past N2
    // reads the next table's bytes, never used
    run16(blob + G.blob_b2 + 64 * t_lo, smem + G.off_t2, 4 * nt);
    run16(blob + G.blob_m2 + 64 * t_lo, smem + G.off_t2 + G.TS * 64, 4 * nt);
    run16(blob + G.blob_s2 + 64 * t_lo, smem + G.off_t2 + 2 * G.TS * 64, 4 * nt);
    if (a.residual) {
      const uint8_t* res = (const uint8_t*)a.residual + (long)m0 * N1;
      const int units = (rows * N1) >> 2;  // N1 % 4 == 0
      for (int base = lw * 64; base < units; base += NL * 64)
        if (base + lane < units) dma4(res + (base + lane) * 4, smem + G.off_res + base * 4);
    }
  }
  // residual ADD: add.cc rescales each 8-bit operand on its own, so both
  // rescalings are 256-entry tables (built while the burst is in flight)
  int* add_tab = (int*)(smem + G.off_add);
  if (a.residual) {
    for (int i = tid; i < 512; i += NW * 64) {
      const int q = (i & 255) - 128;
      add_tab[i] = i < 256 ? requant_lt1((q + a.add_y_off) * (1 << a.add_left_shift), a.add_y_mult, a.add_y_shift)
                           : requant_lt1((q + a.add_r_off) * (1 << a.add_left_shift), a.add_r_mult, a.add_r_shift);
    }
  }

  // ---- phase A: depthwise 3x3 (global taps) -> dl -------------------------
  if (LW == 0 || wave < NA) chain_dw_mfma<FAST, 2, NA / RB>(cp.dw, dv, m, m < P, lane, r16, g, wsub, dl, G.S1, orow);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of the burst
  __syncthreads();

  // ---- phase B: first 1x1 from LDS (+ residual ADD) -> pl / o1 ------------
  {
    const int k1 = a.k_pad;
    const int KS1 = k1 >> 6;
    const int sx1 = swz_mask(r16, k1 >> 4);  // rows 16t + r16: one XOR mask per lane
    const int* b1 = (const int*)(smem + T1 * 16 * k1);
    const int* m1 = b1 + N1;
    const int* s1 = m1 + N1;
    const unsigned char* xrow = dl + (pb * 16 + r16) * G.S1 + g * 16;
    const bool out1 = a.output != nullptr && blockIdx.y == 0;  // slice 0 stores the block output
    auto epi = [&](int nch, v4i acc) {
      if (nch >= N1) return;
      const ChanQ q = chan_q(m1[nch], s1[nch], a.out_zp);
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[r], q, a.out_zp, a.act_min, a.act_max);
      if (a.residual) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int32_t rq = (int32_t)(int8_t)resl[(orow + r) * N1 + nch];  // rows past `rows`: never stored
          v[r] = clamp_i32(requant_lt1(add_tab[v[r] + 128] + add_tab[256 + rq + 128], a.add_o_mult, a.add_o_shift) +
                               a.add_o_off,
                           a.add_act_min, a.add_act_max);
        }
      }
      if (out1) stage4(o1, N1, orow, nch, v);
      stage4(pl, G.S2, orow, nch, v);
    };
    // two channel tiles per iteration (their LDS reads issue together)
    for (int t = wsub; t < T1; t += 2 * WPB) {
      const bool two = t + WPB < T1;
      const int ra = t * 16 + r16, rb = (two ? t + WPB : t) * 16 + r16;
      const unsigned char* wa = smem + ra * k1;
      const unsigned char* wb = smem + rb * k1;
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
  if (a.output && blockIdx.y == 0) stage_copy_rows(o1, (uint8_t*)a.output + (long)m0 * N1, rows * N1, tid, NW * 64);

  // ---- phase C: this slice of the second 1x1 from LDS -> ol -> HBM --------
  {
    const int k2 = b.k_pad;
    const int KS2 = k2 >> 6;
    const int sx2 = swz_mask(r16, k2 >> 4);  // slice rows start at a multiple of 16
    const unsigned char* W2 = smem + G.off_w2;
    const int* b2 = (const int*)(smem + G.off_t2);
    const int* m2 = b2 + G.TS * 16;
    const int* s2 = m2 + G.TS * 16;
    const unsigned char* xrow = pl + (pb * 16 + r16) * G.S2 + g * 16;
    v4i x[KX];
#pragma unroll
    for (int k = 0; k < KX; ++k) x[k] = k < KS2 ? *(const v4i*)(xrow + k * 64) : (v4i){0, 0, 0, 0};
    auto epi = [&](int lc, v4i acc) {  // lc: the channel within the slice
      if (t_lo * 16 + lc >= N2) return;
      const ChanQ q = chan_q(m2[lc], s2[lc], b.out_zp);
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = requant_out<FAST>(acc[r], q, b.out_zp, b.act_min, b.act_max);
      stage4(ol, G.out_pitch, orow, lc, v);
    };
    for (int t = wsub; t < nt; t += 2 * WPB) {
      const bool two = t + WPB < nt;
      const int ra = t * 16 + r16, rb = (two ? t + WPB : t) * 16 + r16;
      const unsigned char* wa = W2 + ra * k2;
      const unsigned char* wb = W2 + rb * k2;
      const int ba = t_lo * 16 + ra < N2 ? b2[ra] : 0, bb = t_lo * 16 + rb < N2 ? b2[rb] : 0;
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
  const int c_lo = t_lo * 16, c_hi = min(N2, t_hi * 16);
  if (c_hi > c_lo)
    stage_copy_out(ol, G.out_pitch, (uint8_t*)b.output + (long)m0 * N2, N2, c_lo, c_hi - c_lo, rows, tid, NW * 64);
}

template <int RB, bool FAST, int KX, int NW, int LW>
static void launch_stage(const bh_chain_params& p, int P, const StageGeom& G, hipStream_t s) {
  if (G.bytes > 64 * 1024) {
    // opt in to the CU's full 160 KiB of LDS for this instantiation (once per device)
    static thread_local int opted_device = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (opted_device != dev) {
      (void)hipFuncSetAttribute((const void*)chain_stage_kernel<RB, FAST, KX, NW, LW>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      opted_device = dev;
    }
  }
  ChainDivs dv;
  dv.out_w = FastDiv(p.dw.out_w);
  dv.out_h = FastDiv(p.dw.out_h);
  const int blocks = (P + RB * 16 - 1) / (RB * 16);
  BH_LAUNCH((chain_stage_kernel<RB, FAST, KX, NW, LW>), dim3(blocks, std::max(1, p.c_split)), dim3(NW * 64), G.bytes, s,
            p, P, G, dv);
}

template <bool FAST, int KX>
static void launch_stage_form(const bh_chain_params& p, int P, const StageGeom& G, hipStream_t s) {
  const int nw = p.waves == 8 ? 8 : 4;
  if (p.stage == 2) {  // loader waves: the upper half of the workgroup
    if (p.px_blocks == 2) {
      if (nw == 8) launch_stage<2, FAST, KX, 8, 4>(p, P, G, s);
      else launch_stage<2, FAST, KX, 4, 2>(p, P, G, s);
    } else {
      if (nw == 8) launch_stage<1, FAST, KX, 8, 4>(p, P, G, s);
      else launch_stage<1, FAST, KX, 4, 2>(p, P, G, s);
    }
    return;
  }
  if (p.px_blocks == 2) {
    if (nw == 8) launch_stage<2, FAST, KX, 8, 0>(p, P, G, s);
    else launch_stage<2, FAST, KX, 4, 0>(p, P, G, s);
  } else {
    if (nw == 8) launch_stage<1, FAST, KX, 8, 0>(p, P, G, s);
    else launch_stage<1, FAST, KX, 4, 0>(p, P, G, s);
  }
}

}  // namespace bh

// Stage form of bh_chain_i8 (bh_chain_params.stage != 0): LDS bytes, or 0 if
// the parameters do not admit it.  Called by bh_chain_lds_bytes after the
// checks every chain form shares.
extern "C" size_t bh_chain_stage_lds_bytes(const bh_chain_params* pp) {
  const bh_chain_params& p = *pp;
  if (!p.has_pw2 || p.pw2.k_pad > 64 * 5) return 0;
  if (p.px_blocks != 1 && p.px_blocks != 2) return 0;
  if (p.waves != 0 && p.waves != 4 && p.waves != 8) return 0;
  if (p.tile || p.persist || p.deep || p.stage < 0 || p.stage > 2) return 0;
  if (p.c_split < 0 || p.c_split > 8 || (p.pw2.out_c + 15) / 16 < std::max(1, p.c_split)) return 0;
  const bh::StageGeom G = bh::stage_geom(p);
  return G.bytes <= 160 * 1024 ? G.bytes : 0;
}

extern "C" int bh_chain_stage_launch(const bh_chain_params* pp, bh_stream_t stream) {
  const bh_chain_params& p = *pp;
  if (!p.tile_blob) {
    bh_set_last_error("bh_chain_i8: the stage form needs tile_blob (bh_chain_tile_pack)");
    return BH_EINVAL;
  }
  const int P = p.dw.batch * p.dw.out_h * p.dw.out_w;
  const bh::StageGeom G = bh::stage_geom(p);
  const bool fast = p.dw.requant_fast && p.pw1.requant_fast && p.pw2.requant_fast;
  const bool k2 = p.pw2.k_pad <= 128;
  hipStream_t s = (hipStream_t)stream;
  if (k2) {
    if (fast) bh::launch_stage_form<true, 2>(p, P, G, s);
    else bh::launch_stage_form<false, 2>(p, P, G, s);
  } else {
    if (fast) bh::launch_stage_form<true, 5>(p, P, G, s);
    else bh::launch_stage_form<false, 5>(p, P, G, s);
  }
  return bh_check_launch("chain_stage_kernel");
}
