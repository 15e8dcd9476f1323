// conv_gemm_big_kernel: large batched 1x1 convolutions (stride 1, int8
// activations, symmetric int8 filters) as a 256x256-tile int8 GEMM on
// v_mfma_i32_32x32x32_i8.
//
// Stands in for reference_integer_ops::ConvPerChannel (TFLite 2.9.2) on the
// 1x1 layers Band's hot path runs (band/backend/tfl/model_executor.cc:249-255
// -> Interpreter::Invoke), at the sizes where the layer is a real GEMM:
// M = batch x H x W output pixels in the thousands to tens of thousands
// (job-batch passes, SURVEY.md section 8(d)'s B = 32 / 256), N and K in the
// hundreds.  conv_gemm_kernel's 128x128 tiles give each of its 8 waves 8
// MFMAs (128 cycles) per K-step between barriers; here a wave owns a
// WTM x WTN = 128 x 64 sub-tile, 16 MFMAs of 32 cycles per K-step, so the
// once-per-K-step barrier and the LDS fragment reads are amortised over 8x
// the matrix work; a 256x256 tile also halves the L2 -> LDS bytes per MAC
// of a 128x128 one (each staged byte serves 256 output rows or columns).
//
//   - operands: A = the packed filters Bt[n_pad][k_pad] (rows = output
//     channels), B = the activations X[M][K] (rows = pixels); both are
//     "row x K-bytes" images, so one staging path serves both: a K-step is
//     64 bytes of BM pixel rows and BN filter rows, global -> LDS with
//     16-byte global_load_lds, NB LDS buffers, D = NB-1 K-steps in flight
//     across the barrier (counted vmcnt + raw s_barrier, never vmcnt(0) in
//     the loop);
//   - LDS image: row r of a stage holds its 64 bytes as four 16-byte chunks,
//     chunk c at physical slot c ^ ((r >> 2) & 3); the 16 lanes of a
//     ds_read_b128 phase (16 consecutive rows, one chunk) then cover all 64
//     banks once.  glds writes lane-linear, so the swizzle is applied to each
//     lane's GLOBAL source address;
//   - MFMA D[ch][px] = sum_k W[ch][k] X[px][k]: lane l ends with pixel
//     (l & 31) of its 32-pixel block and channels 8q + 4(l >> 5) + 0..3,
//     q = 0..3 - four consecutive channels of one pixel, so the
//     per-channel requantisation constants are loaded once per (channel
//     group, lane) and serve the wave's RM pixel blocks;
//   - epilogue: requantised bytes -> an LDS tile [BM][BN + 16] (the staging
//     buffers are free by then), then whole output rows leave with 16-byte
//     stores of consecutive addresses; a folded residual ADD and / or 8-bit
//     table (conv_store4's arithmetic) are applied per byte on the way out;
//   - the workgroup -> tile map is XCD-contiguous with the N-blocks of one
//     pixel block consecutive, so a pixel block is fetched from HBM once per
//     XCD and re-read by its N-blocks from that XCD's L2.
#include "common.hpp"

namespace bh {

typedef int v16i __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_big_t;

template <int N>
__device__ __forceinline__ void big_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// conv_store4's residual ADD + table for one requantised byte `y` (output
// domain) and its residual byte `r`
__device__ __forceinline__ uint8_t big_post(const bh_conv_params& p, uint8_t y, uint8_t r, bool y_signed,
                                            bool r_signed, const uint8_t* tab, bool res) {
  int32_t v = y_signed ? (int32_t)(int8_t)y : (int32_t)y;
  if (res) {
    const int32_t q = r_signed ? (int32_t)(int8_t)r : (int32_t)r;
    const int32_t sy = requant_lt1((v + p.add_y_off) * (1 << p.add_left_shift), p.add_y_mult, p.add_y_shift);
    const int32_t sr = requant_lt1((q + p.add_r_off) * (1 << p.add_left_shift), p.add_r_mult, p.add_r_shift);
    v = clamp_i32(requant_lt1(sy + sr, p.add_o_mult, p.add_o_shift) + p.add_o_off, p.add_act_min, p.add_act_max);
  }
  return tab ? tab[(uint8_t)v] : (uint8_t)v;
}

template <int BM, int BN, int WAVES_M, int WAVES_N, int NB, bool FAST>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_gemm_big_kernel(bh_conv_params p, int M, int K,
                                                                              int gn, int ksteps) {
  constexpr int W = WAVES_M * WAVES_N;
  constexpr int T = W * 64;
  constexpr int WTM = BM / WAVES_M;  // pixels per wave
  constexpr int WTN = BN / WAVES_N;  // channels per wave
  constexpr int RM = WTM / 32, RN = WTN / 32;
  static_assert(RM * 32 == WTM && RN * 32 == WTN, "32x32 MFMA blocks");
  constexpr int ROWS = BM + BN;
  static_assert(ROWS % (16 * W) == 0, "whole glds instructions per wave");
  constexpr int NI = ROWS / (16 * W);  // glds instructions per wave per K-step
  constexpr int STAGE = ROWS * 64;
  constexpr int D = NB - 1;
  static_assert(D >= 1 && D <= 3, "1..3 K-steps in flight");
  constexpr int OPITCH = BN + 16;  // output staging row pitch (bank spread)
  constexpr int MAIN = NB * STAGE > BM * OPITCH ? NB * STAGE : BM * OPITCH;
  // the tile's per-channel epilogue constants (bias_eff, mult, shift), staged
  // once before the K loop so the epilogue reads them from LDS instead of
  // paying a dependent global round trip per channel group
  constexpr int CONST = MAIN;
  constexpr int LDS = MAIN + 3 * BN * 4;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int logical = xcd_block(blockIdx.x, gridDim.x);
  const int bm = logical / gn;
  const int bn = logical - bm * gn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int N = p.out_c;

  // this lane's global source for each of its NI staging instructions:
  // instruction j of wave w stages rows 16 (w + W j) .. +15, lane -> row
  // + (lane >> 2), physical chunk lane & 3 (logical chunk c = that ^ swizzle)
  const uint8_t* src[NI];
  int kval[NI], goff[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = 16 * (wave + W * j) + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3);
    goff[j] = 16 * c;
    if (row < BM) {
      const int m = min(m0 + row, M - 1);
      src[j] = (const uint8_t*)p.input + (long)m * K + 16 * c;
      kval[j] = K - 16 * c;  // chunks at or past K read the row's start (their filters are 0)
    } else {
      const int n = min(n0 + row - BM, p.n_pad - 1);
      src[j] = (const uint8_t*)p.weights + (long)n * p.k_pad + 16 * c;
      kval[j] = 0x7fffffff;
    }
  }
  auto stage = [&](int ks) {
    const int kb = ks * 64;
    uint8_t* dst = lds + (ks % NB) * STAGE + wave * 1024;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const uint8_t* s = kb < kval[j] ? src[j] + kb : src[j] - goff[j];
      __builtin_amdgcn_global_load_lds((const void*)s, (lds_void_big_t*)(dst + j * W * 1024), 16, 0, 0);
    }
  };

  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int wm0 = (wave % WAVES_M) * WTM;
  const int wn0 = (wave / WAVES_M) * WTN;
  v16i acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  {
    int32_t* cst = (int32_t*)(lds + CONST);
    for (int i = threadIdx.x; i < 3 * BN; i += T) {
      const int a = i / BN, c = i - a * BN;
      const int n = min(n0 + c, N - 1);
      cst[i] = a == 0 ? p.bias_eff[n] : (a == 1 ? p.mult[n] : p.shift[n]);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < ksteps) stage(d);
  for (int ks = 0; ks < ksteps; ++ks) {
    // step ks landed (this wave's glds of the later steps stay in flight);
    // the barrier orders every wave's DMA before the reads, and retires the
    // reads of step ks-1, whose buffer step ks+D refills
    const int ahead = min(D - 1, ksteps - 1 - ks);
    if (ahead >= 2) big_wait_vmcnt<2 * NI>();
    else if (ahead == 1) big_wait_vmcnt<NI>();
    else big_wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (ks + D < ksteps) stage(ks + D);
    const uint8_t* buf = lds + (ks % NB) * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 2 * s + h;  // this lane's 16 K-bytes of the 32-deep sub-step
      v4i a[RN], b[RM];
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = BM + wn0 + j * 32 + r32;
        a[j] = *(const v4i*)(buf + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = wm0 + i * 32 + r32;
        b[i] = *(const v4i*)(buf + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[j], b[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  big_wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();  // every wave is done with the staging buffers

  // requantise into the LDS output tile [BM][OPITCH]
#pragma unroll
  for (int j = 0; j < RN; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ch = wn0 + j * 32 + 8 * q + 4 * h;  // tile-local, 4 consecutive channels
      const int32_t* cst = (const int32_t*)(lds + CONST);
      const v4i b4 = *(const v4i*)(cst + ch);
      const v4i m4 = *(const v4i*)(cst + BN + ch);
      const v4i s4 = *(const v4i*)(cst + 2 * BN + ch);
      int32_t be[4], mu[4], sh[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        be[r] = b4[r];
        mu[r] = m4[r];
        sh[r] = s4[r];
      }
      ChanQ cq[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) cq[r] = chan_q(mu[r], sh[r], p.out_zp);
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int px = wm0 + i * 32 + r32;
        uint32_t packed = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int32_t v = requant_out<FAST>(acc[i][j][4 * q + r] + be[r], cq[r], p.out_zp, p.act_min, p.act_max);
          packed |= ((uint32_t)v & 0xffu) << (8 * r);
        }
        *(uint32_t*)(lds + px * OPITCH + ch) = packed;
      }
    }
  __syncthreads();

  // whole rows out: 16-byte chunks of consecutive addresses
  constexpr int CPR = BN / 16;  // chunks per tile row
  const bool post = p.residual || p.out_table;
  const bool fast_rows = !post && (N & 15) == 0 && (((uintptr_t)p.output) & 15) == 0;
  const uint8_t* res = (const uint8_t*)p.residual;
  const uint8_t* tab = (const uint8_t*)p.out_table;
  const bool y_signed = p.act_min < 0;  // int8 output (a uint8 domain is never negative)
  const bool r_signed = p.in_xor == 0;
  uint8_t* out = (uint8_t*)p.output;
  for (int idx = threadIdx.x; idx < BM * CPR; idx += T) {
    const int px = idx / CPR;
    const int cc = idx - px * CPR;
    const int m = m0 + px;
    const int n = n0 + cc * 16;
    if (m >= M || n >= N) continue;
    const v4i val = *(const v4i*)(lds + px * OPITCH + cc * 16);
    const long o = (long)m * N + n;
    if (fast_rows) {
      *(v4i*)(out + o) = val;
      continue;
    }
    const uint8_t* vb = (const uint8_t*)&val;
    const int cnt = min(16, N - n);
    for (int b = 0; b < cnt; ++b) out[o + b] = big_post(p, vb[b], res ? res[o + b] : 0, y_signed, r_signed, tab, res);
  }
}

template <int BM, int BN, int WAVES_M, int WAVES_N, int NB>
static int launch_big(const bh_conv_params& p, int M, int K, hipStream_t s) {
  const int gm = (M + BM - 1) / BM, gn = (p.out_c + BN - 1) / BN;
  const int ksteps = (K + 63) / 64;
  if (p.requant_fast)
    BH_LAUNCH((conv_gemm_big_kernel<BM, BN, WAVES_M, WAVES_N, NB, true>), dim3(gm * gn),
              dim3(WAVES_M * WAVES_N * 64), 0, s, p, M, K, gn, ksteps);
  else
    BH_LAUNCH((conv_gemm_big_kernel<BM, BN, WAVES_M, WAVES_N, NB, false>), dim3(gm * gn),
              dim3(WAVES_M * WAVES_N * 64), 0, s, p, M, K, gn, ksteps);
  return bh_check_launch("conv_gemm_big_kernel");
}

}  // namespace bh

static long big_wgs(long M, long N, int tm, int tn) { return ((M + tm - 1) / tm) * ((N + tn - 1) / tn); }

// Configurations (BH_GEMM_BIG_CFG forces one for A-B runs): 1 = 256x256
// tiles (8 waves of 128 x 64) with 3 K-steps in flight (4 LDS buffers),
// 2 = 256x128 / 3 = 128x256 (8 waves of 64 x 64) with 2 in flight (two
// workgroups per CU), 4 = 256x256 with 2 in flight, 5 = 256x128 with 3.
// Returns 0 when the layer is too small for this kernel.
extern "C" int bh_conv_gemm_big_config(long M, int N) {
  static const int cfg = [] {
    const char* e = std::getenv("BH_GEMM_BIG_CFG");
    return e ? std::atoi(e) : 0;
  }();
  if (cfg > 0) return cfg;
  // two workgroups per CU (72 KB of LDS each) beat one 256 x 256 tile with a
  // deeper pipeline on every layer measured: the second workgroup's K loop
  // runs under the first one's barriers and epilogue (PoseNet 1024 -> 1024
  // at B = 256: 92-95 vs 110 us; MobileNetV2 320 -> 1280: 18.3 vs 30.9 us,
  // profiles/r05j_gemm_big_cfg.txt).  128 x 256 when N fills the 256
  // columns, else 256 x 128; from one round of 256 workgroups.
  if (N >= 256 && big_wgs(M, N, 128, 256) >= 256) return 3;
  if (big_wgs(M, N, 256, 128) >= 256) return 2;
  return 0;
}

int bh_conv_gemm_big_launch(const bh_conv_params& p, int M, int K, hipStream_t s) {
  switch (bh_conv_gemm_big_config(M, p.out_c)) {
    case 2: return bh::launch_big<256, 128, 4, 2, 3>(p, M, K, s);
    case 4: return bh::launch_big<256, 256, 2, 4, 3>(p, M, K, s);
    case 5: return bh::launch_big<256, 128, 4, 2, 4>(p, M, K, s);
    case 1: return bh::launch_big<256, 256, 2, 4, 4>(p, M, K, s);
    default: return bh::launch_big<128, 256, 2, 4, 3>(p, M, K, s);
  }
}
