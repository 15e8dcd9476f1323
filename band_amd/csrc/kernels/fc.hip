// FULLY_CONNECTED for gfx950 (and the batch-1 1x1-conv classifier, which is
// the same GEMV).  Stands in for TFLite 2.9.2
// reference_integer_ops::FullyConnected / reference_ops::FullyConnected
// (uint8) on Band's hot path (band/backend/tfl/model_executor.cc:249-255).
//
// At batch 1 this is a weight stream (HBM/L2-bound GEMV), so it uses the
// VALU dot product v_dot4_i32_i8 instead of MFMA: one wave per
// (row, output unit); lanes stride over the K-contiguous weight row in
// 16-byte chunks, reduce with cross-lane shuffles, then the TFLite
// requantisation in lane 0.
//   acc = sum x'w' + bias_eff - w_zp * sum x'   (int8 domain, exact)
#include "common.hpp"

namespace bh {

template <int VEC>
__device__ __forceinline__ void load_x(const uint8_t* x, int d, int depth, uint32_t xorw, uint32_t* w) {
  // 16 bytes starting at d; bytes >= depth read as 0 (no XOR)
  if constexpr (VEC == 16) {
    if (d + 16 <= depth) {
      v4i v = *(const v4i*)(x + d);
      w[0] = v.x ^ xorw; w[1] = v.y ^ xorw; w[2] = v.z ^ xorw; w[3] = v.w ^ xorw;
      return;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int k = d + 4 * q + b;
      if (k < depth) r |= ((uint32_t)(x[k] ^ (uint8_t)xorw)) << (8 * b);
    }
    w[q] = r;
  }
}

template <int VEC, bool WZP>
__global__ __launch_bounds__(256) void fc_kernel(bh_fc_params p, FastDiv units) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int job = blockIdx.x * 4 + wave;
  if (job >= p.rows * p.units) return;
  const int r = units.div(job);
  const int u = job - r * p.units;
  const uint8_t* x = (const uint8_t*)p.input + (long)r * p.depth;
  const int8_t* w = p.weights + (long)u * p.depth_pad;
  const uint32_t xorw = splat_byte(p.in_xor);
  int acc = 0, xs = 0;
  for (int d = lane * 16; d < p.depth; d += 64 * 16) {
    uint32_t xv[4];
    load_x<VEC>(x, d, p.depth, xorw, xv);
    const v4i wv = *(const v4i*)(w + d);
    acc = __builtin_amdgcn_sdot4((int)xv[0], wv.x, acc, false);
    acc = __builtin_amdgcn_sdot4((int)xv[1], wv.y, acc, false);
    acc = __builtin_amdgcn_sdot4((int)xv[2], wv.z, acc, false);
    acc = __builtin_amdgcn_sdot4((int)xv[3], wv.w, acc, false);
    if constexpr (WZP) {
#pragma unroll
      for (int q = 0; q < 4; ++q) xs = __builtin_amdgcn_sdot4((int)xv[q], 0x01010101, xs, false);
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    acc += __shfl_xor(acc, o);
    if constexpr (WZP) xs += __shfl_xor(xs, o);
  }
  if (lane == 0) {
    int32_t v = acc + p.bias_eff[u];
    if constexpr (WZP) v -= p.w_zp * xs;
    v = requant(v, p.mult[u], p.shift[u]) + p.out_zp;
    const uint8_t byte = (uint8_t)clamp_i32(v, p.act_min, p.act_max);
    ((uint8_t*)p.output)[(long)r * p.units + u] = p.out_table ? ((const uint8_t*)p.out_table)[byte] : byte;
  }
}

}  // namespace bh

extern "C" int bh_fc_i8(const bh_fc_params* pp, bh_stream_t stream) {
  if (!pp || !pp->input || !pp->output || !pp->weights || !pp->bias_eff || !pp->mult || !pp->shift ||
      pp->rows <= 0 || pp->depth <= 0 || pp->units <= 0 || pp->depth_pad < pp->depth || (pp->depth_pad % 16)) {
    bh_set_last_error("bh_fc_i8: invalid parameters");
    return BH_EINVAL;
  }
  const bh_fc_params& p = *pp;
  hipStream_t s = (hipStream_t)stream;
  const long jobs = (long)p.rows * p.units;
  if (jobs >= INT32_MAX) {
    bh_set_last_error("bh_fc_i8: too many output elements for 32-bit indexing");
    return BH_EINVAL;
  }
  const bh::FastDiv units(p.units);
  dim3 grid((unsigned)((jobs + 3) / 4));
  const bool vec16 = (p.depth % 16 == 0) && ((uintptr_t)p.input % 16 == 0);
  if (p.w_zp != 0) {
    if (vec16) BH_LAUNCH((bh::fc_kernel<16, true>), grid, dim3(256), 0, s, p, units);
    else BH_LAUNCH((bh::fc_kernel<1, true>), grid, dim3(256), 0, s, p, units);
  } else {
    if (vec16) BH_LAUNCH((bh::fc_kernel<16, false>), grid, dim3(256), 0, s, p, units);
    else BH_LAUNCH((bh::fc_kernel<1, false>), grid, dim3(256), 0, s, p, units);
  }
  return bh_check_launch("fc_kernel");
}
