// Image-resident chain sequence for gfx950 (int8 per-channel): a run of n
// consecutive fused chains (fused_chain.hip: DEPTHWISE_CONV_2D 3x3 ->
// CONV_2D 1x1 [-> ADD residual] -> CONV_2D 1x1, the second conv being the
// next MobileNetV2 block's expand) executed by ONE workgroup per image.
//
// Stands in for 3n-4n consecutive TFLite 2.9.2 builtin kernels on Band's hot
// path (band/backend/tfl/model_executor.cc:249-255 -> Interpreter::Invoke):
// reference_integer_ops::DepthwiseConvPerChannel, ConvPerChannel, Add and
// ConvPerChannel per chain, every intermediate requantised to its own 8-bit
// tensor exactly as TFLite stores it (bit-identical to the launches it
// replaces).
//
// Why: at batch 1 the 14x14 / 7x7 part of a MobileNetV2 is a dozen short
// launches, each paying a kernel boundary and a cold operand round trip, on
// a few dozen workgroups of a 256-CU chip.  A 14x14 image's block output
// (<= 196 x 160 bytes) fits one CU's LDS, and a 3x3 depthwise over a whole
// image needs no halo from anyone else, so one 8-wave workgroup can walk
// every block of the run without a grid barrier or a launch in between:
//
//   per chain i, per chunk of <= 256 expanded channels:
//     E  expand (chain i-1's second 1x1) of the previous block output Y
//        (LDS) -> the chunk of the depthwise input, in an LDS image with a
//        one-pixel border of the input zero point (chain 0: the chunk is
//        read from HBM instead)
//     D  depthwise 3x3 on the matrix cores (block-diagonal 16x16x64 tiles
//        as chain_dw_mfma, taps from the LDS image) -> LDS [pixel][chunk]
//     P  first 1x1: accumulate the chunk's K slice into int32 registers
//   epilogue: requantise, residual ADD (previous Y from LDS; chain 0: HBM),
//   -> the next Y (LDS, ping-pong)
//   after the last chain: its first 1x1 output and its second 1x1 (the next
//   block's expand) go to HBM.
// The expanded tensors (the largest of each block) never exist whole: each
// is produced, consumed and dropped one chunk at a time.
// Every GEMM phase is weight-stationary: a wave loads its channel tile's
// filter fragments once (one memory round trip) and walks the pixel tiles
// from LDS.
#include <algorithm>

#include "common.hpp"

namespace bh {

constexpr int kSeqNT = 512;  // 8 waves: 256 VGPRs each (16 waves spill at 128)
constexpr int kSeqW = kSeqNT / 64;
constexpr int kSeqTpw = 10;   // first-1x1 accumulator tiles per wave (<= 80 tiles)
constexpr int kSeqChMax = 256;

struct SeqChain {
  int hin, win, hout, wout;  // depthwise input / output image
  int pin, pout, ptin, ptout;  // pixels, 16-pixel tiles
  int c, ch;                 // expanded channels; channels per chunk (multiple of 64)
  int n1, sy;                // first 1x1 out channels; LDS row stride of its output Y
  int se, sd;                // LDS row strides of the chunk's depthwise input / output
  int str, oy, ox;           // depthwise stride; border offsets 1 - pad
  int res;                   // residual ADD in the first 1x1's epilogue
  int kp2;                   // second 1x1's K (= roundup(n1, 64))
  FastDiv dwin, dwout;       // image widths
};

// the run's constant table (bh_chain_seq_plan -> device memory): geometry
// and the chains' filter / table pointers, read with scalar loads
struct SeqTable {
  int n, c2;  // chains; last chain's second 1x1 out_c (0: none)
  int off_y0, off_y1, off_e, off_d, off_tab, lds;
  SeqChain g[BH_SEQ_MAX];
  bh_chain_params c[BH_SEQ_MAX];
};

// per launch: the run's HBM inputs and outputs
struct SeqIo {
  const int8_t* in0;   // chain 0's depthwise input
  const int8_t* res0;  // chain 0's residual (NULL: none)
  int8_t* y_out;       // last chain's first 1x1 output (NULL: not stored)
  int8_t* e_out;       // last chain's second 1x1 output (NULL: none)
};

// one 16x16 tile of a 1x1 layer, D = X W^T: KS K-steps of this lane's pixel
// row (LDS) against filter fragments already in registers
// (unrolled to the 5-step bound: a register array indexed by a runtime
// trip count would live in scratch)
__device__ __forceinline__ v4i seq_tile(const unsigned char* xrow, const v4i* w, int KS, v4i acc) {
#pragma unroll
  for (int k = 0; k < 5; ++k)
    if (k < KS) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(*(const v4i*)(xrow + k * 64), w[k], acc, 0, 0, 0);
  return acc;
}

// a chain's geometry from the constant table into registers (SGPRs)
__device__ __forceinline__ SeqChain seq_chain(const cst_ptr<SeqTable>& A, int i) {
  SeqChain G;
  G.hin = A->g[i].hin;
  G.win = A->g[i].win;
  G.hout = A->g[i].hout;
  G.wout = A->g[i].wout;
  G.pin = A->g[i].pin;
  G.pout = A->g[i].pout;
  G.ptin = A->g[i].ptin;
  G.ptout = A->g[i].ptout;
  G.c = A->g[i].c;
  G.ch = A->g[i].ch;
  G.n1 = A->g[i].n1;
  G.sy = A->g[i].sy;
  G.se = A->g[i].se;
  G.sd = A->g[i].sd;
  G.str = A->g[i].str;
  G.oy = A->g[i].oy;
  G.ox = A->g[i].ox;
  G.res = A->g[i].res;
  G.kp2 = A->g[i].kp2;
  G.dwin.d = A->g[i].dwin.d;
  G.dwin.m = A->g[i].dwin.m;
  G.dwin.s = A->g[i].dwin.s;
  G.dwout.d = A->g[i].dwout.d;
  G.dwout.m = A->g[i].dwout.m;
  G.dwout.s = A->g[i].dwout.s;
  return G;
}

__global__ __launch_bounds__(kSeqNT) void chain_seq_kernel(const SeqTable* tab, SeqIo io) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: tile math on SALU
  const int r16 = lane & 15, g = lane >> 4;
  const long img = blockIdx.x;
  const cst_ptr<SeqTable> A = as_const(tab);
  const cst_ptr<bh_chain_params> T = as_const(tab->c);
  unsigned char* E = smem + A->off_e;
  unsigned char* Dl = smem + A->off_d;
  int* add_tab = (int*)(smem + A->off_tab);
  unsigned char* Yw = smem + A->off_y0;  // written by the current chain
  unsigned char* Yr = smem + A->off_y1;  // the previous chain's block output

  for (int i = 0; i < A->n; ++i) {
    const SeqChain G = seq_chain(A, i);
    const int gw = G.win + 2;  // row length of the bordered depthwise image
    // ---- chain prologue: ADD tables, the image border, accumulators ------
    if (G.res) {
      const int yoff = T[i].pw1.add_y_off, roff = T[i].pw1.add_r_off, ls = T[i].pw1.add_left_shift;
      const int ym = T[i].pw1.add_y_mult, ys = T[i].pw1.add_y_shift;
      const int rm = T[i].pw1.add_r_mult, rs = T[i].pw1.add_r_shift;
      for (int k = tid; k < 512; k += kSeqNT) {
        const int q = (k & 255) - 128;
        add_tab[k] = k < 256 ? requant_lt1((q + yoff) * (1 << ls), ym, ys) : requant_lt1((q + roff) * (1 << ls), rm, rs);
      }
    }
    {
      const int nu = G.ch >> 4;
      const int nb = 2 * gw + 2 * G.hin;
      const int zb = (int)splat_byte(T[i].dw.in_zp);
      const v4i zf = (v4i){zb, zb, zb, zb};
      for (int u = tid; u < nb * nu; u += kSeqNT) {
        const int b = u / nu, k = u - b * nu;
        int pos;
        if (b < gw) pos = b;
        else if (b < 2 * gw) pos = (G.hin + 1) * gw + (b - gw);
        else pos = ((b - 2 * gw) >> 1) * gw + gw + (((b - 2 * gw) & 1) ? G.win + 1 : 0);
        *(v4i*)(E + pos * G.se + k * 16) = zf;
      }
    }
    const int8_t* w1 = T[i].pw1.weights;
    const int kp1 = G.c;  // the first 1x1's K (= C, a multiple of 64)
    const int nt1 = G.n1 >> 4;
    const int ntile = G.ptout * nt1;
    const int tpw = (ntile + kSeqW - 1) / kSeqW;
    v4i acc[kSeqTpw];
#pragma unroll
    for (int j = 0; j < kSeqTpw; ++j) {
      const int q = wave * tpw + j;
      const int nt = q / G.ptout;
      const int32_t be = j < tpw && q < ntile ? T[i].pw1.bias_eff[nt * 16 + r16] : 0;
      acc[j] = (v4i){be, be, be, be};
    }

    for (int c0 = 0; c0 < G.c; c0 += G.ch) {
      const int chc = min(G.ch, G.c - c0);
      const int nct = chc >> 4;
      // waves per channel tile in the weight-stationary phases
      const int wpc = max(1, kSeqW / nct);
      const int my_ct = wave / wpc, my_sub = wave - my_ct * wpc;
      // ---- phase E: the chunk of the depthwise input -> bordered LDS image
      if (i == 0) {
        const int units = G.pin * nct;
        for (int u = tid; u < units; u += kSeqNT) {
          const int p = u / nct, k = u - p * nct;
          const int y = G.dwin.div(p), x = p - y * G.win;
          const v4i v = *(const v4i*)(io.in0 + (img * G.pin + p) * G.c + c0 + k * 16);
          *(v4i*)(E + ((y + 1) * gw + x + 1) * G.se + k * 16) = v;
        }
      } else {
        for (int ct = my_ct; ct < nct; ct += kSeqW / wpc) {
          const SeqChain Gp = seq_chain(A, i - 1);
          const int KS = Gp.kp2 >> 6;
          const int ch = c0 + ct * 16 + r16;  // this lane's expanded channel
          const int8_t* wrow = T[i - 1].pw2.weights + (long)ch * Gp.kp2 + g * 16;
          v4i w[5];
  #pragma unroll
          for (int k = 0; k < 5; ++k)
            if (k < KS) w[k] = *(const v4i*)(wrow + k * 64);
          const int32_t be = T[i - 1].pw2.bias_eff[ch];
          const int zp = T[i - 1].pw2.out_zp, lo = T[i - 1].pw2.act_min, hi = T[i - 1].pw2.act_max;
          const ChanQ q = chan_q(T[i - 1].pw2.mult[ch], T[i - 1].pw2.shift[ch], zp);
          for (int pt = my_sub; pt < G.ptin; pt += wpc) {
            const v4i a = seq_tile(Yr + (pt * 16 + r16) * Gp.sy + g * 16, w, KS, (v4i){be, be, be, be});
            int32_t v[4];
  #pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = requant_out<true>(a[r], q, zp, lo, hi);
            // quad transpose: this lane then holds 4 channels of one pixel
            const uint32_t word = quad_transpose8(pack4_bytes(v));
            const int pp = pt * 16 + 4 * g + (r16 & 3);
            if (pp < G.pin) {
              const int y = G.dwin.div(pp), x = pp - y * G.win;
              *(uint32_t*)(E + ((y + 1) * gw + x + 1) * G.se + ct * 16 + (r16 & ~3)) = word;
            }
          }
        }
      }
      __syncthreads();
      // ---- phase D: depthwise 3x3 on the matrix cores, LDS -> LDS --------
      for (int ct = my_ct; ct < nct; ct += kSeqW / wpc) {
        const int c = c0 + ct * 16 + r16;  // this lane's result channel
        const v4i tw = *(const v4i*)(T[i].dw.taps + 4 * c);
        const int zp = T[i].dw.out_zp, lo = T[i].dw.act_min, hi = T[i].dw.act_max;
        const ChanQ q = chan_q(T[i].dw.mult[c], T[i].dw.shift[c], zp);
        // filter bytes of K-step s (filter row s), tap 3s + g, as in chain_dw_mfma
        const int bsh = 8 * (r16 & 3), dsel = r16 >> 2;
        const uint32_t t0 = (uint32_t)tw.x, t1 = (uint32_t)tw.y, t2 = (uint32_t)tw.z;
        const int tbit1 = g == 0 ? 24 : 8 * (g - 1);
        const int tbit2 = g < 2 ? 8 * (2 + g) : bsh;
        uint32_t wb[3];
        wb[0] = (t0 >> (8 * g)) & 0xffu;
        wb[1] = ((g == 0 ? t0 : t1) >> tbit1) & 0xffu;
        wb[2] = ((g < 2 ? t1 : t2) >> tbit2) & 0xffu;
        v4i wf[3];
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int wv = g < 3 ? (int)(wb[s] << bsh) : 0;
          wf[s] = (v4i){dsel == 0 ? wv : 0, dsel == 1 ? wv : 0, dsel == 2 ? wv : 0, dsel == 3 ? wv : 0};
        }
        for (int pt = my_sub; pt < G.ptout; pt += wpc) {
          const int p = pt * 16 + r16;
          const int pc = p < G.pout ? p : 0;
          const int oy = G.dwout.div(pc), ox = pc - oy * G.wout;
          const unsigned char* base = E + ((oy * G.str + G.oy) * gw + ox * G.str + G.ox + (g < 3 ? g : 0)) * G.se + ct * 16;
          v4i a = (v4i){tw.w, tw.w, tw.w, tw.w};
#pragma unroll
          for (int s = 0; s < 3; ++s) a = __builtin_amdgcn_mfma_i32_16x16x64_i8(*(const v4i*)(base + s * gw * G.se), wf[s], a, 0, 0, 0);
          int32_t v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = requant_out<true>(a[r], q, zp, lo, hi);
          stage4(Dl, G.sd, pt * 16 + 4 * g, ct * 16 + r16, v);
        }
      }
      __syncthreads();
      // ---- phase P: the first 1x1's K slice [c0, c0 + chc) ---------------
      {
        const int KS = chc >> 6;
        for (int k = 0; k < KS; ++k) {
          v4i b[kSeqTpw];
#pragma unroll
          for (int j = 0; j < kSeqTpw; ++j) {
            const int q = wave * tpw + j;
            if (j < tpw && q < ntile) {
              const int nt = q / G.ptout;
              b[j] = *(const v4i*)(w1 + (long)(nt * 16 + r16) * kp1 + c0 + k * 64 + g * 16);
            }
          }
#pragma unroll
          for (int j = 0; j < kSeqTpw; ++j) {
            const int q = wave * tpw + j;
            if (j < tpw && q < ntile) {
              const int nt = q / G.ptout, pt = q - nt * G.ptout;
              const v4i a = *(const v4i*)(Dl + (pt * 16 + r16) * G.sd + k * 64 + g * 16);
              acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b[j], acc[j], 0, 0, 0);
            }
          }
        }
      }
      // the next chunk's phase E writes only E; its barrier orders this
      // phase's D reads before the next phase D
    }
    // ---- chain epilogue: requantise [+ residual ADD] -> Y (LDS) ----------
    {
      const int zp = T[i].pw1.out_zp, lo = T[i].pw1.act_min, hi = T[i].pw1.act_max;
      const int ooff = T[i].pw1.add_o_off, om = T[i].pw1.add_o_mult, os = T[i].pw1.add_o_shift;
      const int alo = T[i].pw1.add_act_min, ahi = T[i].pw1.add_act_max;
      const int syp = i > 0 ? A->g[i - 1].sy : 0;
#pragma unroll
      for (int j = 0; j < kSeqTpw; ++j) {
        const int q = wave * tpw + j;
        if (!(j < tpw && q < ntile)) continue;
        const int nt = q / G.ptout, pt = q - nt * G.ptout;
        const int n = nt * 16 + r16;
        const ChanQ cq = chan_q(T[i].pw1.mult[n], T[i].pw1.shift[n], zp);
        int32_t v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = requant_out<true>(acc[j][r], cq, zp, lo, hi);
        if (G.res) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int pp = pt * 16 + 4 * g + r;
            int32_t rq = 0;
            if (pp < G.pout)
              rq = i == 0 ? (int32_t)io.res0[(img * G.pout + pp) * G.n1 + n] : (int32_t)(int8_t)Yr[pp * syp + n];
            v[r] = clamp_i32(requant_lt1(add_tab[v[r] + 128] + add_tab[256 + rq + 128], om, os) + ooff, alo, ahi);
          }
        }
        stage4(Yw, G.sy, pt * 16 + 4 * g, n, v);
      }
    }
    __syncthreads();
    unsigned char* t = Yw;
    Yw = Yr;
    Yr = t;
  }

  // ---- the run's outputs: last chain's first 1x1 (Yr) and second 1x1 ----
  const SeqChain L = seq_chain(A, A->n - 1);
  if (io.y_out) {
    const int nu = L.n1 >> 4;
    for (int u = tid; u < L.pout * nu; u += kSeqNT) {
      const int p = u / nu, k = u - p * nu;
      *(v4i*)(io.y_out + (img * L.pout + p) * L.n1 + k * 16) = *(const v4i*)(Yr + p * L.sy + k * 16);
    }
  }
  if (A->c2 > 0) {
    const int i = A->n - 1;
    const int KS = L.kp2 >> 6;
    const int nct2 = A->c2 >> 4;
    const int zp = T[i].pw2.out_zp, lo = T[i].pw2.act_min, hi = T[i].pw2.act_max;
    for (int ct = wave; ct < nct2; ct += kSeqW) {
      const int ch = ct * 16 + r16;
      const int8_t* wrow = T[i].pw2.weights + (long)ch * L.kp2 + g * 16;
      v4i w[5];
#pragma unroll
      for (int k = 0; k < 5; ++k)
        if (k < KS) w[k] = *(const v4i*)(wrow + k * 64);
      const int32_t be = T[i].pw2.bias_eff[ch];
      const ChanQ q = chan_q(T[i].pw2.mult[ch], T[i].pw2.shift[ch], zp);
      for (int pt = 0; pt < L.ptout; ++pt) {
        const v4i a = seq_tile(Yr + (pt * 16 + r16) * L.sy + g * 16, w, KS, (v4i){be, be, be, be});
        int32_t v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = requant_out<true>(a[r], q, zp, lo, hi);
        const uint32_t word = quad_transpose8(pack4_bytes(v));
        const int pp = pt * 16 + 4 * g + (r16 & 3);
        if (pp < L.pout) *(uint32_t*)(io.e_out + (img * L.pout + pp) * A->c2 + ct * 16 + (r16 & ~3)) = word;
      }
    }
  }
}

// ---- host: validation, geometry, launch ------------------------------------

static bool seq_conv1x1(const bh_conv_params& c) {
  return c.k_h == 1 && c.k_w == 1 && c.stride_h == 1 && c.stride_w == 1 && c.pad_h == 0 && c.pad_w == 0 &&
         c.in_xor == 0 && c.w_zp == 0 && c.requant_fast && !c.out_table && c.out_img_stride == 0 && c.weights &&
         c.bias_eff && c.mult && c.shift && c.out_c % 16 == 0;
}

// geometry of a run; false when the kernel does not cover it
static bool seq_plan(const bh_chain_params* c, int n, SeqTable* A) {
  if (!c || n < 2 || n > BH_SEQ_MAX) return false;
  const int batch = c[0].dw.batch;
  size_t ymax = 0;
  for (int i = 0; i < n; ++i) {
    const bh_dwconv_params& d = c[i].dw;
    const bh_conv_params& a = c[i].pw1;
    const bh_conv_params& b = c[i].pw2;
    if (d.batch != batch || batch <= 0 || d.k_h != 3 || d.k_w != 3 || d.depth_multiplier != 1 || d.dil_h != 1 ||
        d.dil_w != 1 || d.stride_h != d.stride_w || (d.stride_h != 1 && d.stride_h != 2) || d.in_xor || d.w_zp ||
        !d.taps || !d.requant_fast || d.out_table || d.in_c != d.out_c || d.out_c % 64 || d.out_c > 1280 ||
        d.in_h > 16 || d.in_w > 16 || d.pad_h < 0 || d.pad_h > 1 || d.pad_w < 0 || d.pad_w > 1 || !d.mult || !d.shift)
      return false;
    if (!seq_conv1x1(a) || a.in_c != d.out_c || a.k_pad != d.out_c || a.out_h != d.out_h || a.out_w != d.out_w ||
        a.batch != batch)
      return false;
    const int ptout = (d.out_h * d.out_w + 15) / 16;
    if ((ptout * (a.out_c / 16) + kSeqW - 1) / kSeqW > kSeqTpw) return false;
    const bool last = i == n - 1;
    if (!last && !c[i].has_pw2) return false;
    if (c[i].has_pw2) {
      if (!seq_conv1x1(b) || b.residual || b.in_c != a.out_c || b.k_pad != (a.out_c + 63) / 64 * 64 ||
          b.k_pad > 320 || b.batch != batch)
        return false;
    }
    if (!last) {
      const bh_dwconv_params& dn = c[i + 1].dw;
      if (b.out_c != dn.out_c || dn.input != b.output || dn.in_h != d.out_h || dn.in_w != d.out_w) return false;
      // the next residual, if any, is this chain's block output
      if (c[i + 1].pw1.residual &&
          (c[i + 1].pw1.residual != a.output || !a.output || c[i + 1].pw1.out_c != a.out_c || dn.stride_h != 1))
        return false;
    }
    if (i == 0 && !d.input) return false;
    if (a.residual && !(i == 0 || c[i].pw1.residual == c[i - 1].pw1.output)) return false;
    const size_t sy = (size_t)(a.out_c + 63) / 64 * 64 + 16;
    ymax = std::max(ymax, (size_t)ptout * 16 * sy);
  }
  if ((c[n - 1].has_pw2 && !c[n - 1].pw2.output) || (!c[n - 1].has_pw2 && !c[n - 1].pw1.output)) return false;
  ymax = (ymax + 15) / 16 * 16;
  const size_t tab = 2048;
  if (2 * ymax + tab >= 163840) return false;
  const size_t budget = 163840 - 2 * ymax - tab;
  size_t emax = 0, dmax = 0;
  for (int i = 0; i < n; ++i) {
    const bh_dwconv_params& d = c[i].dw;
    SeqChain& G = A->g[i];
    G.hin = d.in_h;
    G.win = d.in_w;
    G.hout = d.out_h;
    G.wout = d.out_w;
    G.pin = d.in_h * d.in_w;
    G.pout = d.out_h * d.out_w;
    G.ptin = (G.pin + 15) / 16;
    G.ptout = (G.pout + 15) / 16;
    G.c = d.out_c;
    G.n1 = c[i].pw1.out_c;
    G.sy = (G.n1 + 63) / 64 * 64 + 16;
    G.str = d.stride_h;
    G.oy = 1 - d.pad_h;
    G.ox = 1 - d.pad_w;
    G.res = c[i].pw1.residual ? 1 : 0;
    G.kp2 = c[i].has_pw2 ? c[i].pw2.k_pad : 0;
    G.dwin = FastDiv((uint32_t)G.win);
    G.dwout = FastDiv((uint32_t)G.wout);
    // the last depthwise tap row / column stays inside the bordered image
    if ((G.hout - 1) * G.str + 2 + G.oy > G.hin + 1 || (G.wout - 1) * G.str + 2 + G.ox > G.win + 1) return false;
    // chunk: equal slices of at most 256 channels whose E + D buffers fit
    const size_t rows_e = (size_t)(G.hin + 2) * (G.win + 2), rows_d = (size_t)G.ptout * 16;
    int chunks = (G.c + kSeqChMax - 1) / kSeqChMax;
    for (;; ++chunks) {
      const int ch = (G.c / 64 + chunks - 1) / chunks * 64;
      if (ch < 64) return false;
      const size_t s = (size_t)ch + 16;
      if ((rows_e * s + 15) / 16 * 16 + rows_d * s <= budget) {
        G.ch = ch;
        G.se = G.sd = (int)s;
        emax = std::max(emax, (rows_e * s + 15) / 16 * 16);
        dmax = std::max(dmax, rows_d * s);
        break;
      }
      if (ch == 64) return false;
    }
  }
  A->n = n;
  A->c2 = c[n - 1].has_pw2 ? c[n - 1].pw2.out_c : 0;
  A->off_y0 = 0;
  A->off_y1 = (int)ymax;
  A->off_e = (int)(2 * ymax);
  A->off_d = (int)(2 * ymax + emax);
  A->off_tab = (int)(2 * ymax + emax + dmax);
  A->lds = (int)(2 * ymax + emax + dmax + tab);
  for (int i = 0; i < n; ++i) A->c[i] = c[i];
  return A->lds <= 163840;
}

}  // namespace bh

extern "C" size_t bh_chain_seq_lds_bytes(const bh_chain_params* chains, int n) {
  bh::SeqTable A{};
  return bh::seq_plan(chains, n, &A) ? (size_t)A.lds : 0;
}

extern "C" size_t bh_chain_seq_table_bytes(void) { return sizeof(bh::SeqTable); }

extern "C" int bh_chain_seq_plan(const bh_chain_params* chains, int n, void* host_table) {
  if (!host_table || !bh::seq_plan(chains, n, (bh::SeqTable*)host_table)) {
    bh_set_last_error("bh_chain_seq_plan: unsupported chain run");
    return BH_EINVAL;
  }
  return 0;
}

extern "C" int bh_chain_seq_i8(const bh_chain_params* chains, const void* table, int n, bh_stream_t stream) {
  bh::SeqTable A{};
  if (!table || !bh::seq_plan(chains, n, &A)) {
    bh_set_last_error("bh_chain_seq_i8: unsupported chain run");
    return BH_EINVAL;
  }
  bh::SeqIo io;
  io.in0 = (const int8_t*)chains[0].dw.input;
  io.res0 = (const int8_t*)chains[0].pw1.residual;
  io.y_out = (int8_t*)chains[n - 1].pw1.output;
  io.e_out = chains[n - 1].has_pw2 ? (int8_t*)chains[n - 1].pw2.output : nullptr;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)bh::chain_seq_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr = true;
  }
  BH_LAUNCH(bh::chain_seq_kernel, dim3(chains[0].dw.batch), dim3(bh::kSeqNT), (size_t)A.lds, (hipStream_t)stream,
            (const bh::SeqTable*)table, io);
  return bh_check_launch("chain_seq_kernel");
}
