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

}  // namespace bh

// Launched by bh_conv2d_i8 for small-K layers (conv_mfma.hip); returns
// BH_EINVAL when the layer is outside this kernel's range.
int bh_conv_direct_launch(const bh_conv_params& p, int M, int K, hipStream_t s) {
  if (K > 64 || p.out_c <= 0 || (p.k_pad % 4)) return BH_EINVAL;
  bh::DirectDivs dv;
  dv.out_w = bh::FastDiv(p.out_w);
  dv.out_h = bh::FastDiv(p.out_h);
  const dim3 grid((unsigned)((M + 255) / 256), (unsigned)((p.out_c + 7) / 8));
  if (K <= 32) hipLaunchKernelGGL(bh::conv_direct_kernel<8>, grid, dim3(256), 0, s, p, M, K, dv);
  else hipLaunchKernelGGL(bh::conv_direct_kernel<16>, grid, dim3(256), 0, s, p, M, K, dv);
  return bh_check_launch("conv_direct_kernel");
}
