// Device-side helpers shared by the gfx950 kernels.
//
// The fixed-point requantisation below is the device restatement of TFLite
// 2.9.2's kernels/internal/common.h MultiplyByQuantizedMultiplier (double
// rounding: SaturatingRoundingDoublingHighMul then RoundingDivideByPOT), the
// arithmetic every int8 op on Band's hot path ends with
// (band/backend/tfl/model_executor.cc:249-255 -> Interpreter::Invoke).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "band_hip_kernels.h"

namespace bh {

// Per-dispatch timestamps for the profiler (bh_profile_events): while `stop`
// is set, launches go through hipExtLaunchKernel, whose start / stop events
// carry the dispatch's own begin / end timestamps - the duration rocprofv3's
// kernel trace reports, without the event-to-event dispatch gap.  The first
// kernel of a launcher takes `start`, every kernel re-records `stop`, so a
// launcher that issues several kernels is timed from the first one's begin
// to the last one's end.
struct ProfEvents {
  hipEvent_t start = nullptr;
  hipEvent_t stop = nullptr;
  int launched = 0;  // kernels issued under these events
};
extern thread_local ProfEvents g_prof;

#define BH_LAUNCH(kern, grid, block, shmem, stream, ...)                                            \
  do {                                                                                              \
    if (::bh::g_prof.stop) {                                                                        \
      hipExtLaunchKernelGGL(kern, grid, block, shmem, stream, ::bh::g_prof.start, ::bh::g_prof.stop, 0, \
                            __VA_ARGS__);                                                           \
      ::bh::g_prof.start = nullptr;                                                                 \
      ++::bh::g_prof.launched;                                                                      \
    } else {                                                                                        \
      hipLaunchKernelGGL(kern, grid, block, shmem, stream, __VA_ARGS__);                            \
    }                                                                                               \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;

// gemmlowp SaturatingRoundingDoublingHighMul(a, b) = trunc((a*b + nudge) / 2^31)
// with nudge = a*b >= 0 ? 2^30 : 1 - 2^30.  For every a*b that equals
// floor((a*b + 2^30) / 2^31) = (a*b + 2^30) >> 31 (the two sign cases are
// the same floor / ceil identity), i.e. one v_mad_i64_i32 and one funnel
// shift.  Its saturation case a == b == INT32_MIN cannot occur: TFLite
// multipliers are QuantizeMultiplier outputs (|b| < 2^31) or their negation.
// Checked against the reference formula on 2e8 random and all edge pairs.
__device__ __forceinline__ int32_t srdhm(int32_t a, int32_t b) {
  return (int32_t)(((int64_t)a * (int64_t)b + (1ll << 30)) >> 31);
}

// gemmlowp RoundingDivideByPOT (0 <= e <= 31), 32-bit arithmetic
__device__ __forceinline__ int32_t rdbypot(int32_t x, int e) {
  const int32_t mask = (int32_t)((1u << e) - 1u);
  const int32_t rem = x & mask;
  const int32_t thr = (mask >> 1) + (x < 0 ? 1 : 0);
  return (x >> e) + (rem > thr ? 1 : 0);
}

// MultiplyByQuantizedMultiplier(x, m, shift): shift > 0 is a left shift.
__device__ __forceinline__ int32_t requant(int32_t x, int32_t m, int32_t shift) {
  const int left = shift > 0 ? shift : 0;
  const int right = shift > 0 ? 0 : -shift;
  return rdbypot(srdhm((int32_t)((uint32_t)x << left), m), right);
}

// MultiplyByQuantizedMultiplierSmallerThanOneExp(x, m, left_shift<=0)
__device__ __forceinline__ int32_t requant_lt1(int32_t x, int32_t m, int32_t left_shift) {
  return rdbypot(srdhm(x, m), -left_shift);
}

__device__ __forceinline__ int32_t clamp_i32(int32_t v, int32_t lo, int32_t hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

// sign-extend byte b of a dword
__device__ __forceinline__ int32_t sbyte(uint32_t w, int b) {
  return (int32_t)(int8_t)((w >> (8 * b)) & 0xff);
}

__device__ __forceinline__ uint32_t splat_byte(int32_t v) {
  return ((uint32_t)v & 0xffu) * 0x01010101u;
}

// bytes 0 of v0..v3 -> one dword
__device__ __forceinline__ uint32_t pack4_bytes(const int32_t v[4]) {
  const uint32_t lo = __builtin_amdgcn_perm((uint32_t)v[1], (uint32_t)v[0], 0x0c0c0400u);
  const uint32_t hi = __builtin_amdgcn_perm((uint32_t)v[3], (uint32_t)v[2], 0x04000c0cu);
  return lo | hi;
}

// 4x4 byte transpose across the 4 lanes of a quad (lanes 4q .. 4q+3): lane
// i holds [a_i0 a_i1 a_i2 a_i3] (byte k = a_ik) and gets [a_0i a_1i a_2i
// a_3i].  Two DPP quad permutes and two v_perm_b32.  An MFMA lane (r16, g)
// of the D = X W^T form holds 4 PIXELS of one channel; after the transpose
// lane 4j+i holds 4 CHANNELS (4j..4j+3 of its 16) of pixel i, so the LDS
// staging takes one ds_write_b32 per lane instead of four ds_write_b8 - and
// byte stores of 4 lanes into one dword are 4 distinct addresses on a bank
// (a 4-way conflict per store).  Every lane of the quad must be active.
__device__ __forceinline__ uint32_t quad_transpose8(uint32_t p) {
  const int i = (int)(threadIdx.x & 3);
  const uint32_t x = (uint32_t)__builtin_amdgcn_mov_dpp((int)p, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  const uint32_t n = __builtin_amdgcn_perm(x, p, (i & 2) ? 0x03020706u : 0x05040100u);
  const uint32_t y = (uint32_t)__builtin_amdgcn_mov_dpp((int)n, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  return __builtin_amdgcn_perm(y, n, (i & 1) ? 0x03070105u : 0x06020400u);
}

// Stages a D = X W^T epilogue's 4 values (pixels row0 .. row0 + 3 of channel
// `col`, this lane's r16 = col % 16) into an LDS tile of row stride `stride`:
// quad-transposed, one dword per lane (BH_QUAD_STORE=1, default), or four
// byte stores (0; build-time A-B switch).
#ifndef BH_QUAD_STORE
#define BH_QUAD_STORE 1
#endif
__device__ __forceinline__ void stage4(unsigned char* tile, int stride, int row0, int col, const int32_t v[4]) {
#if BH_QUAD_STORE
  const int r16 = col & 15;
  *(uint32_t*)(tile + (row0 + (r16 & 3)) * stride + col - r16 + (r16 & ~3)) = quad_transpose8(pack4_bytes(v));
#else
#pragma unroll
  for (int r = 0; r < 4; ++r) tile[(row0 + r) * stride + col] = (unsigned char)v[r];
#endif
}

// Division by a runtime-invariant divisor for dividends < 2^31, by the
// multiply-high method (Granlund & Montgomery): q = umulhi(n, m) >> s.
// CDNA has no integer divide instruction - a plain `/` or `%` by a runtime
// value is a ~40-instruction VALU sequence, which dominates these
// latency-bound kernels' index math.  Built on the host, passed by value.
struct FastDiv {
  uint32_t d = 1, m = 0, s = 0;
  FastDiv() = default;
  __host__ __device__ explicit FastDiv(uint32_t div) : d(div ? div : 1) {
    if (d > 1) {
      uint32_t l = 0;
      while ((1u << l) < d) ++l;  // ceil(log2 d)
      const uint64_t p = 31 + l;
      m = (uint32_t)(((1ull << p) + d - 1) / d);
      s = (uint32_t)(p - 32);
    }
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return d == 1 ? n : (__umulhi(n, m) >> s); }
  __device__ __forceinline__ uint32_t mod(uint32_t n) const { return n - div(n) * d; }
};

// TFLite requantisation of one accumulator to the clamped output value.
// FAST: the single-step identity of bh_conv_requant_fast_ok (one
// v_mad_i64_i32, a funnel shift and four 32-bit ops; checked against the
// two-step reference on 1.9e8 values incl. every rounding tie class).
struct ChanQ {
  int32_t mu, sh;        // multiplier / TFLite shift
  int32_t e, emask, zpe; // FAST: right shift, sign-correction mask, zp << e
  int64_t c0;
};

__device__ __forceinline__ ChanQ chan_q(int32_t mu, int32_t sh, int32_t zp) {
  ChanQ q;
  q.mu = mu;
  q.sh = sh;
  q.e = -sh;
  q.emask = q.e > 0 ? -1 : 0;
  q.zpe = (int32_t)((uint32_t)zp << (q.e & 31));
  q.c0 = (1ll << 30) + (q.e > 0 ? (1ll << (30 + q.e)) : 0ll);
  return q;
}

// clamp to [lo, hi] in one v_med3_i32 (min(max()) compiles to two VALU
// when both bounds are wave-uniform: gfx9's VOP3 reads one SGPR, so the
// compiler will not form the med3 itself); BH_MED3=0 at build time keeps
// min / max
#ifndef BH_MED3
#define BH_MED3 1
#endif
__device__ __forceinline__ int32_t med3_clamp(int32_t v, int32_t lo, int32_t hi) {
#if BH_MED3
  int32_t r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "s"(lo), "v"(hi));
  return r;
#else
  return min(max(v, lo), hi);
#endif
}

template <bool FAST>
__device__ __forceinline__ int32_t requant_out(int32_t acc, const ChanQ& q, int32_t zp, int32_t lo, int32_t hi) {
  int32_t v;
  if constexpr (FAST) {
    const int64_t z = (int64_t)acc * q.mu + q.c0;
    const int32_t u = (int32_t)(z >> 31);
    v = (u + ((acc >> 31) & q.emask) + q.zpe) >> q.e;
  } else {
    v = requant(acc, q.mu, q.sh) + zp;
  }
  return med3_clamp(v, lo, hi);
}

// requant + zero point + clamp, the single-step identity when `fast`
// (uniform per layer) and TFLite's two-step form otherwise
__device__ __forceinline__ int32_t requant_clamp(int32_t acc, int32_t mu, int32_t sh, int32_t zp, int32_t lo,
                                                 int32_t hi, bool fast) {
  return fast ? requant_out<true>(acc, chan_q(mu, sh, zp), zp, lo, hi) : clamp_i32(requant(acc, mu, sh) + zp, lo, hi);
}

// Read-only operand tables (filters, folded biases, multipliers) seen
// through the constant address space: a wave-uniform index then compiles to
// s_load (scalar cache, no texture-unit work) even though the kernel also
// stores through other pointers, which keeps the compiler from proving the
// generic pointer unclobbered.
template <typename T>
using cst_ptr = const T __attribute__((address_space(4)))*;
template <typename T>
__device__ __forceinline__ cst_ptr<T> as_const(const T* p) {
  return (cst_ptr<T>)(uintptr_t)p;
}

// Workgroup id -> logical id such that each XCD (hardware ids i % 8 run on
// XCD i % 8) gets one contiguous run of logical ids; the ids of an
// incomplete last round keep their own number.  Neighbouring tiles (e.g. the
// halo rows of a convolution) then share one L2.
__device__ __forceinline__ int xcd_block(int hw, int total) {
  const int per = total >> 3;
  return hw < (per << 3) ? (hw & 7) * per + (hw >> 3) : hw;
}

// 2-D XCD split of a GEMM's gm x gn output-block grid: (8 / xb) pixel
// ranges x xb channel ranges, one per XCD, so each L2 pulls 1 / (8 / xb) of
// the input and 1 / xb of the filters (xb = 1: the input read once and the
// filters 8 times; xb = 8: the other way round; 2 / 4 between).  Hardware
// block i runs on XCD i % 8 and walks that XCD's ranges N-blocks fastest;
// the ranges are balanced (sizes differ by at most one block), the grid is
// 8 x the largest range pair, and the blocks past an XCD's share get
// bm = gm and must exit.  xb 0: the 1-D order of xcd_block over the
// row-major grid (N-blocks fastest), for grids the split would pad by more
// than 1/8.
struct XcdSplit {
  int xb, sub_m, sub_n;
};
__device__ __forceinline__ void xcd_tile(int hw, int total, const XcdSplit& x, int gm, int gn, int& bm, int& bn) {
  if (x.xb == 0) {
    const int l = xcd_block(hw, total);
    bm = l / gn;
    bn = l - bm * gn;
    return;
  }
  const int a = 8 / x.xb;
  const int xcd = hw & 7, j = hw >> 3;
  const int pa = xcd / x.xb, pb = xcd - pa * x.xb;
  const int m_lo = pa * gm / a, sm = (pa + 1) * gm / a - m_lo;
  const int n_lo = pb * gn / x.xb, sn = (pb + 1) * gn / x.xb - n_lo;
  if (j >= sm * sn) {
    bm = gm;
    bn = 0;
    return;
  }
  const int jm = j / sn;
  bm = m_lo + jm;
  bn = n_lo + (j - jm * sn);
}
// host: the split with the fewest L2-fill bytes xb * in + (8 / xb) * w over
// the splits that give every XCD at least one pixel and one channel block
// and pad the grid by at most 1/8 (ties: fewer channel ranges); else xb 0
inline XcdSplit xcd_split(long in_bytes, long w_bytes, int gm, int gn) {
  XcdSplit best{0, gm, gn};
  long cost = -1;
  const long blocks = (long)gm * gn;
  for (int xb = 1; xb <= 8; xb *= 2) {
    const int a = 8 / xb;
    if (xb > gn || a > gm) continue;
    const int sub_m = (gm + a - 1) / a, sub_n = (gn + xb - 1) / xb;
    if (8L * sub_m * sub_n * 8 > blocks * 9) continue;
    const long c = xb * in_bytes + a * w_bytes;
    if (cost < 0 || c < cost) {
      cost = c;
      best = {xb, sub_m, sub_n};
    }
  }
  return best;
}
inline int xcd_grid(const XcdSplit& x) { return x.xb ? 8 * x.sub_m * x.sub_n : x.sub_m * x.sub_n; }

}  // namespace bh

// thread-local last-error plumbing for the C ABI (defined in capi_runtime.hip)
extern "C" void bh_set_last_error(const char* msg);
int bh_check_launch(const char* what);
