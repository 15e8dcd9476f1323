// conv_stem_mfma_kernel: the RGB stem (CONV_2D 3x3, 3 input channels, the
// first layer of every C3 model) as an im2col x filter contraction on
// v_mfma_i32_16x16x64_i8, for gfx950.
//
// Stands in for reference_integer_ops::ConvPerChannel / the uint8 reference
// Conv (TFLite 2.9.2) on the first layer Band's hot path runs
// (band/backend/tfl/model_executor.cc:249-255 -> Interpreter::Invoke); same
// int8-domain arithmetic as conv_mfma.hip, bit-exact.
//
// conv_stem_kernel (conv_direct.hip) gives a thread one pixel and walks the
// output channels with v_dot4 against filters read through the scalar cache:
// at batch 24 its waves wait on memory half their cycles and issue ~680
// scalar instructions each (profiles/r04z_stall.txt) - the per-channel
// operand loads, one dependent round trip after another.  Here the window
// x filter product is the dense contraction MFMA exists for: K = 27 window
// bytes (padded to one 64-deep K-step), a 16-pixel x 16-channel tile per
// instruction, D^T = W X^T so a lane ends with 4 consecutive channels of one
// pixel.  A lane's 16 K-bytes are bytes 16g .. 16g+15 of its pixel's
// k-ordered window (k = (ky*3 + kx)*3 + c): lane group 0 holds window rows
// 0-1, group 1 rows 1-2 (+ zero tail), groups 2-3 only zeros, so half the
// wave gathers - three aligned dwords + v_alignbyte per window row, as
// conv_stem_kernel does.  The filter fragments and every lane's
// requantisation constants (4 channels per 16-channel block) are loaded
// once per wave; a wave then runs PB 16-pixel blocks with all their loads
// issued before any MFMA.
#include "common.hpp"

namespace bh {

struct StemDivs {
  FastDiv out_w, out_h;
};

// the 9 window bytes of row y starting at column x0 (int8 domain) as
// dwords r[0] = bytes 0-3, r[1] = 4-7, r[2] = byte 8
__device__ __forceinline__ void stem_row(const bh_conv_params& p, const uint8_t* img, const uint8_t* end, int y, int x0,
                                         uint32_t xorw, uint32_t padw, uint32_t r[3]) {
  const bool rowok = y >= 0 && y < p.in_h;
  const bool colok = x0 >= 0 && x0 + 3 <= p.in_w;
  const uint8_t* a = img + ((long)y * p.in_w + x0) * 3;
  const uintptr_t ai = (uintptr_t)a;
  const uint32_t* base = (const uint32_t*)(ai & ~(uintptr_t)3);
  if (rowok && colok && (const uint8_t*)(base + 3) <= end) {
    const uint32_t o = (uint32_t)(ai & 3);
    const uint32_t d0 = base[0], d1 = base[1], d2 = base[2];
    r[0] = __builtin_amdgcn_alignbyte(d1, d0, o) ^ xorw;
    r[1] = __builtin_amdgcn_alignbyte(d2, d1, o) ^ xorw;
    r[2] = ((d2 >> (8 * o)) ^ xorw) & 0xffu;
  } else if (!rowok) {
    r[0] = padw;
    r[1] = padw;
    r[2] = padw & 0xffu;
  } else {
    uint32_t b[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int x = x0 + k / 3;
      b[k] = (x >= 0 && x < p.in_w) ? (uint32_t)(a[k] ^ (uint8_t)p.in_xor) : (padw & 0xffu);
    }
    r[0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
    r[1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
    r[2] = b[8];
  }
}

// Launch bound: the 4-block forms of up to 48 channels are held to 64-76
// VGPRs (>= 6 waves per SIMD: a batch-32 stem's 24.5 waves per CU resident
// at once; unbounded they took 90-104, 4-5 waves per SIMD, and ran in two
// rounds: 17.0 vs 15.1 us at batch 32, profiles/r06ag_stem_forms.txt).
// 64 channels at that bound would spill.
template <int NB, int PB, bool FAST>
__global__ __launch_bounds__(256, (PB == 4 && NB <= 3 ? 6 : 1)) void conv_stem_mfma_kernel(bh_conv_params p, int M, StemDivs dv) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const int wave_id = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int m_base = wave_id * PB * 16;
  if (m_base >= M) return;
  const long img = (long)p.in_h * p.in_w * 3;
  const uint8_t* end = (const uint8_t*)p.input + p.batch * img;
  const uint32_t xorw = splat_byte(p.in_xor);
  const uint32_t padw = splat_byte(p.in_zp);

  // filter fragments W[ch = 16b + r16][16g .. 16g+15] (k_pad = 64, zero tail)
  v4i wf[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) wf[b] = *(const v4i*)(p.weights + (long)(16 * b + r16) * p.k_pad + 16 * g);
  // D = X W^T: lane (r16, g) gets pixels 4g .. 4g+3 of channel 16b + r16, so
  // one set of requantisation constants per channel block serves every
  // value the lane produces (the transposed form derived them per value)
  int32_t be[NB];
  ChanQ cq[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int c = 16 * b + r16;
    be[b] = p.bias_eff[c];
    cq[b] = chan_q(p.mult[c], p.shift[c], p.out_zp);
  }

  // gather: the PB blocks' window fragments, every load issued first
  v4i xf[PB];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    const int m = min(m_base + pb * 16 + r16, M - 1);
    xf[pb] = (v4i){0, 0, 0, 0};
    if (g < 2) {
      const int t = dv.out_w.div(m);
      const int ox = m - t * p.out_w;
      const int n = dv.out_h.div(t);
      const int oy = t - n * p.out_h;
      const int y0 = oy * p.stride_h - p.pad_h;
      const int x0 = ox * p.stride_w - p.pad_w;
      const uint8_t* im = (const uint8_t*)p.input + n * img;
      uint32_t ra[3], rb[3];
      stem_row(p, im, end, y0 + g * p.dil_h, x0, xorw, padw, ra);        // row g
      stem_row(p, im, end, y0 + (g + 1) * p.dil_h, x0, xorw, padw, rb);  // row g + 1
      if (g == 0) {
        // k 0..15: R0[0..8] R1[0..6]
        xf[pb].x = (int)ra[0];
        xf[pb].y = (int)ra[1];
        xf[pb].z = (int)__builtin_amdgcn_perm(rb[0], ra[2], 0x06050400u);  // R0[8] R1[0..2]
        xf[pb].w = (int)__builtin_amdgcn_alignbyte(rb[1], rb[0], 3);         // R1[3..6]
      } else {
        // k 16..31: R1[7..8] R2[0..8] + 5 zero bytes (ra = R1, rb = R2)
        const uint32_t u = __builtin_amdgcn_perm(ra[2], ra[1], 0x0c0c0403u);  // R1[7] R1[8] 0 0
        xf[pb].x = (int)(u | (rb[0] << 16));                                    // .. R2[0] R2[1]
        xf[pb].y = (int)__builtin_amdgcn_alignbyte(rb[1], rb[0], 2);           // R2[2..5]
        xf[pb].z = (int)__builtin_amdgcn_alignbyte(rb[2], rb[1], 2);           // R2[6..8] 0
        xf[pb].w = 0;
      }
    }
  }
  // uint8 filters: the window byte sum of each of this lane's 4 pixels (the
  // pixel's two halves sit in lane groups 0 and 1 at lane r16 = pixel)
  int rsum[PB][4];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb)
#pragma unroll
    for (int i = 0; i < 4; ++i) rsum[pb][i] = 0;
  if (p.w_zp != 0) {
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      int s = 0;
      s = __builtin_amdgcn_sdot4(xf[pb].x, 0x01010101, s, false);
      s = __builtin_amdgcn_sdot4(xf[pb].y, 0x01010101, s, false);
      s = __builtin_amdgcn_sdot4(xf[pb].z, 0x01010101, s, false);
      s = __builtin_amdgcn_sdot4(xf[pb].w, 0x01010101, s, false);
#pragma unroll
      for (int i = 0; i < 4; ++i) rsum[pb][i] = __shfl(s, 4 * g + i) + __shfl(s, 4 * g + i + 16);
    }
  }
  const uint8_t* tab = (const uint8_t*)p.out_table;
  const int qi = lane & 3, qj = (lane >> 2) & 3;  // after the quad transpose: pixel 4g + qi, channels 4qj..4qj+3
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    const int m = m_base + pb * 16 + 4 * g + qi;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(xf[pb], wf[b], (v4i){0, 0, 0, 0}, 0, 0, 0);
      int32_t v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int32_t a = acc[i] + be[b];
        if (p.w_zp != 0) a -= p.w_zp * rsum[pb][i];
        v[i] = requant_out<FAST>(a, cq[b], p.out_zp, p.act_min, p.act_max);
        if (tab) v[i] = tab[(uint8_t)v[i]];
      }
      // lane 4qj + qi of the r16 group: channels 16b + 4qj .. +3 of its pixel
      const uint32_t packed = quad_transpose8(pack4_bytes(v));
      if (m < M) *(uint32_t*)((uint8_t*)p.output + (long)m * p.out_c + 16 * b + 4 * qj) = packed;
    }
  }
}

template <int NB, int PB>
static void launch_stem_pb(const bh_conv_params& p, int M, const StemDivs& dv, hipStream_t s) {
  const int waves = (M + PB * 16 - 1) / (PB * 16);
  const dim3 grid((unsigned)((waves + 3) / 4));
  if (p.requant_fast) BH_LAUNCH((conv_stem_mfma_kernel<NB, PB, true>), grid, dim3(256), 0, s, p, M, dv);
  else BH_LAUNCH((conv_stem_mfma_kernel<NB, PB, false>), grid, dim3(256), 0, s, p, M, dv);
}

// 16-pixel blocks per wave: 4 (all four blocks' gathers in flight) while
// that still leaves >= 4096 waves, else fewer blocks and more waves
template <int NB>
static int launch_stem_mfma(const bh_conv_params& p, int M, hipStream_t s) {
  StemDivs dv;
  dv.out_w = FastDiv(p.out_w);
  dv.out_h = FastDiv(p.out_h);
  if (M >= 4096 * 64) launch_stem_pb<NB, 4>(p, M, dv, s);
  else if (M >= 4096 * 32) launch_stem_pb<NB, 2>(p, M, dv, s);
  else launch_stem_pb<NB, 1>(p, M, dv, s);
  return bh_check_launch("conv_stem_mfma_kernel");
}

}  // namespace bh

// 3x3 stems over 3 channels, dilation-1 columns, out_c in {16, 32, 48, 64}
// (4-byte aligned output), no residual: 1 when this kernel takes the layer
int bh_conv_stem_mfma_ok(const bh_conv_params& p) {
  // every batch unless a VALU form is forced: batch 1 4.2-4.3 us against
  // 4.9 for the scalar-cache VALU form and 5.2-5.6 for the LDS-staged one
  // (r05z2_stem_h*); with the launch bound above 9.4 / 11.7 / 15.1 us at
  // batch 16 / 24 / 32 against 11.9 / 14.0 / 18.9 for the LDS-staged form
  // (profiles/r06ag_stem_forms.txt; that form's broadcast record reads leave
  // its waves 48 % of their cycles in memory waits, r06af_stem_*_stall_b32).
  // The round-4 transposed epilogue derived the requantisation constants
  // per value and lost everywhere (r05l_stem_ab.txt).
  const bool want = p.kernel_hint == BH_CONV_STEM_MFMA ||
                    (p.kernel_hint != BH_CONV_STEM_VALU && p.kernel_hint != BH_CONV_STEM_SCALAR);
  return want && p.k_h == 3 && p.k_w == 3 && p.in_c == 3 && p.dil_w == 1 && p.k_pad == 64 && p.out_c % 16 == 0 &&
         p.out_c >= 16 && p.out_c <= 64 && !p.residual && !p.out_img_stride && (((uintptr_t)p.output) & 3) == 0;
}

int bh_conv_stem_mfma_launch(const bh_conv_params& p, int M, hipStream_t s) {
  switch (p.out_c / 16) {
    case 1: return bh::launch_stem_mfma<1>(p, M, s);
    case 2: return bh::launch_stem_mfma<2>(p, M, s);
    case 3: return bh::launch_stem_mfma<3>(p, M, s);
    default: return bh::launch_stem_mfma<4>(p, M, s);
  }
}
