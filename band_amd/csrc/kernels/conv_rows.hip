// CONV_2D 1x1 / stride 1 for batched passes: channel-major MFMA tiles with
// packed 4-byte output stores.
//
// Same arithmetic as conv_mfma_kernel (TFLite 2.9.2 ConvPerChannel / uint8
// Conv, bit-exact), shaped for throughput rather than latency: at job batch
// >= 8 a MobileNet 1x1 layer has 10^5-10^6 output pixels and the kernel is
// bound by writing them (expand layers: N = 96-960 output bytes per K = 16-
// 160 input bytes) and by the requant epilogue's VALU work.
//
// The GEMM is computed transposed, D^T = W x X^T: the MFMA's "rows" are 16
// output channels and its "columns" 16 pixels.  With
// v_mfma_i32_16x16x64_i8 lane l then holds D^T[4*(l>>4)+r][l&15], i.e.
// FOUR CONSECUTIVE CHANNELS of ONE pixel - the four requantised bytes pack
// into one dword and go out with one 4-byte store (16 pixels x 16 B per
// wave instruction), with no cross-lane shuffles and no LDS staging.  The
// operand fragments are the same bytes as in conv_mfma_kernel: a pixel
// fragment is 16 contiguous K-bytes of one NHWC input row, a weight
// fragment 16 contiguous K-bytes of one packed filter row.
//
// Workgroup: 4 waves; each wave owns RB x 16 consecutive pixels and the
// workgroup's NT x 16 channels (grid.y covers N in NT*16-channel chunks).
// Workgroup ids are remapped so that the chunks of one pixel block run on
// one XCD (its L2 then serves the block's input rows to every chunk).
#include "common.hpp"

namespace bh {

// 16 int8-domain bytes of one row at k in [0, 16) (zero where k >= K or
// the row is invalid).  Branch-free: out-of-range units load from `safe`
// (any readable address) and are zeroed afterwards, so a wave's loads issue
// back to back instead of each behind its own exec-mask branch and wait.
template <int VEC>
__device__ __forceinline__ v4i load_row16(const uint8_t* row, int K, int kb, bool valid, uint32_t xorw,
                                          const uint8_t* safe) {
  uint32_t w[4];
#pragma unroll
  for (int u = 0; u < 16 / VEC; ++u) {
    const int k = kb + u * VEC;
    const bool ok = valid && k < K;
    const uint8_t* src = ok ? row + k : safe;
    if constexpr (VEC == 16) {
      v4i v = *(const v4i*)src;
      w[0] = ok ? v.x ^ xorw : 0u; w[1] = ok ? v.y ^ xorw : 0u;
      w[2] = ok ? v.z ^ xorw : 0u; w[3] = ok ? v.w ^ xorw : 0u;
    } else if constexpr (VEC == 8) {
      v2i v = *(const v2i*)src;
      w[2 * u] = ok ? v.x ^ xorw : 0u; w[2 * u + 1] = ok ? v.y ^ xorw : 0u;
    } else {
      const uint32_t v = *(const uint32_t*)src;
      w[u] = ok ? v ^ xorw : 0u;
    }
  }
  v4i r;
  r.x = (int)w[0]; r.y = (int)w[1]; r.z = (int)w[2]; r.w = (int)w[3];
  return r;
}

__device__ __forceinline__ int rowsum16b(v4i a, int s) {
  s = __builtin_amdgcn_sdot4(a.x, 0x01010101, s, false);
  s = __builtin_amdgcn_sdot4(a.y, 0x01010101, s, false);
  s = __builtin_amdgcn_sdot4(a.z, 0x01010101, s, false);
  return __builtin_amdgcn_sdot4(a.w, 0x01010101, s, false);
}

// ChanQ / chan_q / requant_out: common.hpp

template <int RB, int NT, int VEC, bool FAST>
__global__ __launch_bounds__(256) void conv_rows_kernel(bh_conv_params p, int M, int K, int N, int mblocks,
                                                        int nchunks) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  // XCD-aware order: hardware id i runs on XCD i % 8; give each XCD a
  // contiguous run of logical ids (logical = pixel block major, chunk
  // minor); the ids of an incomplete last round keep their own number
  const int total = mblocks * nchunks;
  const int hw = blockIdx.x;
  const int per = total >> 3;
  const int logical = hw < (per << 3) ? (hw & 7) * per + (hw >> 3) : hw;
  const int mb = logical / nchunks;
  const int nc = logical - mb * nchunks;
  const int m0 = (mb * 4 + wave) * (RB * 16);
  const int n0 = nc * (NT * 16);
  const bool wzp = p.w_zp != 0;
  const uint32_t xorw = splat_byte(p.in_xor);
  const uint8_t* in = (const uint8_t*)p.input;

  const uint8_t* prow[RB];
  bool pval[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    const int m = m0 + b * 16 + r16;
    pval[b] = m < M;
    prow[b] = in + (long)(pval[b] ? m : 0) * K + g * 16;
  }
  const int8_t* wrow = p.weights + (long)(n0 + r16) * p.k_pad + g * 16;

  // accumulators start at the folded bias of this lane's 4 channels
  v4i acc[RB][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int nb = n0 + t * 16 + 4 * g;
    const v4i be = nb < N ? *(const v4i*)(p.bias_eff + nb) : (v4i){0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < RB; ++b) acc[b][t] = be;
  }
  int rs[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) rs[b] = 0;

  for (int kb = 0; kb < K; kb += 64) {
    v4i x[RB], w[NT];
#pragma unroll
    for (int b = 0; b < RB; ++b) x[b] = load_row16<VEC>(prow[b] + kb, K - kb - g * 16, 0, pval[b], xorw, in);
#pragma unroll
    for (int t = 0; t < NT; ++t)
      w[t] = n0 + t * 16 < N ? *(const v4i*)(wrow + (long)t * 16 * p.k_pad + kb) : (v4i){0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[b][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(w[t], x[b], acc[b][t], 0, 0, 0);
    if (wzp) {
#pragma unroll
      for (int b = 0; b < RB; ++b) rs[b] = rowsum16b(x[b], rs[b]);
    }
  }
  if (wzp) {
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      rs[b] += __shfl_xor(rs[b], 16);
      rs[b] += __shfl_xor(rs[b], 32);
    }
  }

  uint8_t* out = (uint8_t*)p.output;
  const uint8_t* res = (const uint8_t*)p.residual;
  const bool res_signed = p.in_xor == 0;
  const uint8_t* tab = (const uint8_t*)p.out_table;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int nb = n0 + t * 16 + 4 * g;  // this lane's 4 channels
    if (nb >= N) continue;               // N % 4 == 0: all 4 valid
    ChanQ q[4];
    {
      const v4i vm = *(const v4i*)(p.mult + nb);
      const v4i vs = *(const v4i*)(p.shift + nb);
      q[0] = chan_q(vm.x, vs.x, p.out_zp);
      q[1] = chan_q(vm.y, vs.y, p.out_zp);
      q[2] = chan_q(vm.z, vs.z, p.out_zp);
      q[3] = chan_q(vm.w, vs.w, p.out_zp);
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const int m = m0 + b * 16 + r16;
      if (m >= M) continue;
      const long o = (long)m * N + nb;
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int32_t a = acc[b][t][r];
        if (wzp) a -= p.w_zp * rs[b];
        v[r] = requant_out<FAST>(a, q[r], p.out_zp, p.act_min, p.act_max);
      }
      if (res) {
        const uint32_t rq = *(const uint32_t*)(res + o);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t qb = (rq >> (8 * r)) & 0xffu;
          const int32_t qv = res_signed ? (int32_t)(int8_t)qb : (int32_t)qb;
          const int32_t sy =
              requant_lt1((v[r] + p.add_y_off) * (1 << p.add_left_shift), p.add_y_mult, p.add_y_shift);
          const int32_t sr = requant_lt1((qv + p.add_r_off) * (1 << p.add_left_shift), p.add_r_mult, p.add_r_shift);
          v[r] = clamp_i32(requant_lt1(sy + sr, p.add_o_mult, p.add_o_shift) + p.add_o_off, p.add_act_min,
                           p.add_act_max);
        }
      }
      if (tab) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = tab[(uint8_t)v[r]];
      }
      // bytes 0 of v0..v3 -> one dword (v_perm_b32: selector bytes 0-3 pick
      // from the second operand, 4-7 from the first)
      const uint32_t lo = __builtin_amdgcn_perm((uint32_t)v[1], (uint32_t)v[0], 0x0c0c0400u);
      const uint32_t hi = __builtin_amdgcn_perm((uint32_t)v[3], (uint32_t)v[2], 0x04000c0cu);
      *(uint32_t*)(out + o) = lo | hi;
    }
  }
}

// x-stationary variant for K <= 64*KS (expand layers and the 14x14 / 7x7
// layers of a batch): a wave loads its 16*RB pixels' whole K once, then
// walks its range of channel tiles - per tile: KS weight fragments, RB*KS
// MFMAs, the requant epilogue and one packed store per pixel and lane.
// Only RB accumulators are live, so occupancy stays high; the weights
// stream through L1 / L2 (shared by every wave of the CU).
template <int RB, int KS, int VEC, bool FAST>
__global__ __launch_bounds__(256) void conv_xs_kernel(bh_conv_params p, int M, int K, int N, int pwgs, int chunks,
                                                      int tiles_per_chunk) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const int total = pwgs * chunks;
  const int hw = blockIdx.x;
  const int per = total >> 3;
  const int logical = hw < (per << 3) ? (hw & 7) * per + (hw >> 3) : hw;
  const int pw = logical / chunks;
  const int ch = logical - pw * chunks;
  const int m0 = (pw * 4 + wave) * (RB * 16);
  if (m0 >= M) return;
  const int tiles = (N + 15) >> 4;
  const int t0 = ch * tiles_per_chunk;
  const int t1 = min(tiles, t0 + tiles_per_chunk);
  const bool wzp = p.w_zp != 0;
  const uint32_t xorw = splat_byte(p.in_xor);
  const uint8_t* in = (const uint8_t*)p.input;

  v4i x[RB][KS];
  int rs[RB];
  bool pval[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    const int m = m0 + b * 16 + r16;
    pval[b] = m < M;
    const uint8_t* row = in + (long)(pval[b] ? m : 0) * K + g * 16;
#pragma unroll
    for (int k = 0; k < KS; ++k) x[b][k] = load_row16<VEC>(row + k * 64, K - k * 64 - g * 16, 0, pval[b], xorw, in);
  }
  // uint8 filters: per-pixel input sums for the w_zp correction
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    rs[b] = 0;
    if (wzp) {
#pragma unroll
      for (int k = 0; k < KS; ++k) rs[b] = rowsum16b(x[b][k], rs[b]);
      rs[b] += __shfl_xor(rs[b], 16);
      rs[b] += __shfl_xor(rs[b], 32);
    }
  }

  uint8_t* out = (uint8_t*)p.output;
  const uint8_t* res = (const uint8_t*)p.residual;
  const bool res_signed = p.in_xor == 0;
  const uint8_t* tab = (const uint8_t*)p.out_table;
  // operands of one channel tile: filter fragments + folded bias,
  // multipliers, shifts of this lane's 4 channels (zero past N)
  struct TileOps {
    v4i w[KS];
    v4i be, vm, vs;
  };
  auto load_tile = [&](int t, TileOps& o) {
    const int8_t* wrow = p.weights + (long)(t * 16 + r16) * p.k_pad + g * 16;
#pragma unroll
    for (int k = 0; k < KS; ++k) o.w[k] = *(const v4i*)(wrow + k * 64);
    // unconditional loads (channel 0 stands in past N; the epilogue skips
    // those lanes): no exec-mask branches, so the waits stay exact
    const int nb = t * 16 + 4 * g;
    const int nl = nb < N ? nb : 0;
    o.be = *(const v4i*)(p.bias_eff + nl);
    o.vm = *(const v4i*)(p.mult + nl);
    o.vs = *(const v4i*)(p.shift + nl);
  };
  // software pipeline, two tiles deep: tile t+2's operands are issued
  // while tile t's MFMAs, epilogue and stores run.  vmcnt counts loads and
  // stores in one queue, so with one tile of lookahead every tile would
  // also wait for the previous tile's stores; two keep a store batch in
  // flight behind each wait.
  TileOps cur, nx1, nx2;
  load_tile(t0, cur);
  load_tile(min(t0 + 1, t1 - 1), nx1);
  for (int t = t0; t < t1; ++t) {
    load_tile(min(t + 2, t1 - 1), nx2);  // past the end: reloads (no branch)
    const v4i* w = cur.w;
    const v4i be = cur.be, vm = cur.vm, vs = cur.vs;
    const int nb = t * 16 + 4 * g;  // this lane's 4 channels
    const bool nval = nb < N;       // N % 4 == 0: all 4 valid
    v4i acc[RB];
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      acc[b] = be;
#pragma unroll
      for (int k = 0; k < KS; ++k) acc[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(w[k], x[b][k], acc[b], 0, 0, 0);
    }
    cur = nx1;
    nx1 = nx2;
    if (!nval) continue;
    ChanQ q[4];
    q[0] = chan_q(vm.x, vs.x, p.out_zp);
    q[1] = chan_q(vm.y, vs.y, p.out_zp);
    q[2] = chan_q(vm.z, vs.z, p.out_zp);
    q[3] = chan_q(vm.w, vs.w, p.out_zp);
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const int m = m0 + b * 16 + r16;
      if (m >= M) continue;
      const long o = (long)m * N + nb;
      int32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int32_t a = acc[b][r];
        if (wzp) a -= p.w_zp * rs[b];
        v[r] = requant_out<FAST>(a, q[r], p.out_zp, p.act_min, p.act_max);
      }
      if (res) {
        const uint32_t rq = *(const uint32_t*)(res + o);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t qb = (rq >> (8 * r)) & 0xffu;
          const int32_t qv = res_signed ? (int32_t)(int8_t)qb : (int32_t)qb;
          const int32_t sy =
              requant_lt1((v[r] + p.add_y_off) * (1 << p.add_left_shift), p.add_y_mult, p.add_y_shift);
          const int32_t sr = requant_lt1((qv + p.add_r_off) * (1 << p.add_left_shift), p.add_r_mult, p.add_r_shift);
          v[r] = clamp_i32(requant_lt1(sy + sr, p.add_o_mult, p.add_o_shift) + p.add_o_off, p.add_act_min,
                           p.add_act_max);
        }
      }
      if (tab) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = tab[(uint8_t)v[r]];
      }
      const uint32_t lo = __builtin_amdgcn_perm((uint32_t)v[1], (uint32_t)v[0], 0x0c0c0400u);
      const uint32_t hi = __builtin_amdgcn_perm((uint32_t)v[3], (uint32_t)v[2], 0x04000c0cu);
      *(uint32_t*)(out + o) = lo | hi;
    }
  }
}

template <int RB, int KS, int VEC>
static int launch_xs(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  const int tiles = (N + 15) / 16;
  const int pwaves = (M + RB * 16 - 1) / (RB * 16);
  const int pwgs = (pwaves + 3) / 4;
  // enough waves to fill the chip (~8 per CU): split the channel tiles
  // into chunks when the pixels alone give too few
  constexpr int kTargetWaves = 2048;
  int chunks = (kTargetWaves + pwaves - 1) / pwaves;
  chunks = chunks < 1 ? 1 : (chunks > tiles ? tiles : chunks);
  const int tpc = (tiles + chunks - 1) / chunks;
  chunks = (tiles + tpc - 1) / tpc;
  if (p.requant_fast)
    BH_LAUNCH((conv_xs_kernel<RB, KS, VEC, true>), dim3(pwgs * chunks), dim3(256), 0, s, p, M, K, N, pwgs,
                       chunks, tpc);
  else
    BH_LAUNCH((conv_xs_kernel<RB, KS, VEC, false>), dim3(pwgs * chunks), dim3(256), 0, s, p, M, K, N,
                       pwgs, chunks, tpc);
  return bh_check_launch("conv_xs_kernel");
}

template <int VEC>
static int launch_xs_vec(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  const int ks = (K + 63) / 64;
  switch (ks) {
    case 1: return launch_xs<4, 1, VEC>(p, M, K, N, s);
    case 2: return launch_xs<2, 2, VEC>(p, M, K, N, s);
    case 3: return launch_xs<2, 3, VEC>(p, M, K, N, s);
    case 4: return launch_xs<2, 4, VEC>(p, M, K, N, s);
    default: return launch_xs<1, 5, VEC>(p, M, K, N, s);
  }
}

template <int RB, int NT, int VEC>
static int launch_rows(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  const int mblocks = (M + 4 * RB * 16 - 1) / (4 * RB * 16);
  const int nchunks = (N + NT * 16 - 1) / (NT * 16);
  if (p.requant_fast)
    BH_LAUNCH((conv_rows_kernel<RB, NT, VEC, true>), dim3(mblocks * nchunks), dim3(256), 0, s, p, M, K, N,
                       mblocks, nchunks);
  else
    BH_LAUNCH((conv_rows_kernel<RB, NT, VEC, false>), dim3(mblocks * nchunks), dim3(256), 0, s, p, M, K,
                       N, mblocks, nchunks);
  return bh_check_launch("conv_rows_kernel");
}

// NT = channel tiles per workgroup: the whole N when it is <= 12 tiles
// (a pixel block's input is then read once), else chunks of 8 tiles
template <int VEC>
static int launch_rows_vec(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  const int tiles = (N + 15) / 16;
  switch (tiles) {
    case 1: return launch_rows<4, 1, VEC>(p, M, K, N, s);
    case 2: return launch_rows<4, 2, VEC>(p, M, K, N, s);
    case 3: return launch_rows<4, 3, VEC>(p, M, K, N, s);
    case 4: return launch_rows<2, 4, VEC>(p, M, K, N, s);
    case 5: case 6: return launch_rows<2, 6, VEC>(p, M, K, N, s);
    case 7: case 8: return launch_rows<2, 8, VEC>(p, M, K, N, s);
    case 9: return launch_rows<2, 9, VEC>(p, M, K, N, s);
    case 10: case 11: case 12: return launch_rows<2, 12, VEC>(p, M, K, N, s);
    default: return launch_rows<2, 8, VEC>(p, M, K, N, s);
  }
}

}  // namespace bh

// 1x1 / stride 1 / unpadded, N % 4 == 0, K % 4 == 0, K <= 320 (conv_mfma.hip dispatches)
int bh_conv_xs_launch(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  if (K % 16 == 0) return bh::launch_xs_vec<16>(p, M, K, N, s);
  if (K % 8 == 0) return bh::launch_xs_vec<8>(p, M, K, N, s);
  return bh::launch_xs_vec<4>(p, M, K, N, s);
}

// 1x1 / stride 1 / unpadded, N % 4 == 0, K % 4 == 0 (conv_mfma.hip dispatches)
int bh_conv_rows_launch(const bh_conv_params& p, int M, int K, int N, hipStream_t s) {
  if (K % 16 == 0) return bh::launch_rows_vec<16>(p, M, K, N, s);
  if (K % 8 == 0) return bh::launch_rows_vec<8>(p, M, K, N, s);
  return bh::launch_rows_vec<4>(p, M, K, N, s);
}

extern "C" int bh_conv_requant_fast_ok(const int32_t* mult, const int32_t* shift, int n, int k,
                                       int64_t max_abs_bias) {
  if (!mult || !shift || n <= 0 || k <= 0 || max_abs_bias < 0) return 0;
  for (int c = 0; c < n; ++c) {
    if (mult[c] <= (1 << 30) || shift[c] > 0 || shift[c] < -30) return 0;
    const int64_t bound = ((int64_t)k << 16) + max_abs_bias + ((int64_t)255 << (-shift[c]));
    if (bound >= (1ll << 30)) return 0;
  }
  return 1;
}
