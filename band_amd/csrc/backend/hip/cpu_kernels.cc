#include "backend/hip/cpu_kernels.h"

#include "backend/hip/affinity.h"

#include "backend/hip/quant.h"

#include <pthread.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>

namespace band {
namespace hip {

// ---- pool ---------------------------------------------------------------------

CpuPool::CpuPool(int num_threads, const std::vector<int>& cpus) {
  for (int i = 1; i < std::max(1, num_threads); ++i) {
    threads_.emplace_back([this, i] { Loop(i); });
    pthread_setname_np(threads_.back().native_handle(), "band-cpupool");
    // the executor's CpuSet (affinity.h); pinned before the thread's first job
    if (!cpus.empty()) PinThread(threads_.back().native_handle(), cpus);
  }
}

CpuPool::~CpuPool() {
  {
    std::lock_guard<std::mutex> l(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

namespace {
void Chunk(long n, int parts, int id, long* b, long* e) {
  const long per = (n + parts - 1) / parts;
  *b = std::min(n, per * id);
  *e = std::min(n, *b + per);
}
}  // namespace

void CpuPool::Loop(int id) {
  int seen = 0;
  while (true) {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [&] { return stop_ || generation_ != seen; });
    if (stop_) return;
    seen = generation_;
    const auto* fn = job_;
    const long n = n_;
    l.unlock();
    long b, e;
    Chunk(n, size(), id, &b, &e);
    if (b < e) (*fn)(b, e);
    l.lock();
    if (--pending_ == 0) done_cv_.notify_one();
  }
}

void CpuPool::ParallelFor(long n, const std::function<void(long, long)>& fn) {
  if (n <= 0) return;
  if (threads_.empty() || n == 1) {
    fn(0, n);
    return;
  }
  {
    std::lock_guard<std::mutex> l(mu_);
    job_ = &fn;
    n_ = n;
    pending_ = static_cast<int>(threads_.size());
    ++generation_;
  }
  cv_.notify_all();
  long b, e;
  Chunk(n, size(), 0, &b, &e);
  if (b < e) fn(b, e);
  std::unique_lock<std::mutex> l(mu_);
  done_cv_.wait(l, [&] { return pending_ == 0; });
}

// ---- fixed point (TFLite 2.9.2 kernels/internal/common.h) ------------------

namespace {
inline int32_t Srdhm(int32_t a, int32_t b) {
  // exact for every multiplier except INT32_MIN, which QuantizeMultiplier
  // never produces
  return static_cast<int32_t>((static_cast<int64_t>(a) * b + (1ll << 30)) >> 31);
}
inline int32_t Rdbypot(int32_t x, int e) {
  const int32_t mask = static_cast<int32_t>((1u << e) - 1u);
  const int32_t rem = x & mask;
  const int32_t thr = (mask >> 1) + (x < 0 ? 1 : 0);
  return (x >> e) + (rem > thr ? 1 : 0);
}
inline int32_t Requant(int32_t x, int32_t m, int32_t shift) {
  const int left = shift > 0 ? shift : 0;
  const int right = shift > 0 ? 0 : -shift;
  return Rdbypot(Srdhm(static_cast<int32_t>(static_cast<uint32_t>(x) << left), m), right);
}
inline int32_t RequantLt1(int32_t x, int32_t m, int32_t left_shift) { return Rdbypot(Srdhm(x, m), -left_shift); }
inline int32_t Clamp(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

// int8 x int8 dot product (vectorised per target by the compiler)
__attribute__((target_clones("arch=skylake-avx512", "avx2", "default"))) int32_t Dot(const int8_t* a, const int8_t* b, int n) {
  int32_t s = 0;
  for (int i = 0; i < n; ++i) s += static_cast<int32_t>(a[i]) * static_cast<int32_t>(b[i]);
  return s;
}

__attribute__((target_clones("arch=skylake-avx512", "avx2", "default"))) void Dot4(const int8_t* a, const int8_t* w0,
                                                                        const int8_t* w1, const int8_t* w2,
                                                                        const int8_t* w3, int n, int32_t* out) {
  int32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int i = 0; i < n; ++i) {
    const int32_t x = a[i];
    s0 += x * w0[i];
    s1 += x * w1[i];
    s2 += x * w2[i];
    s3 += x * w3[i];
  }
  out[0] = s0;
  out[1] = s1;
  out[2] = s2;
  out[3] = s3;
}

inline int32_t Load8(const uint8_t* p, long i, bool is_signed) {
  return is_signed ? static_cast<int32_t>(static_cast<int8_t>(p[i])) : static_cast<int32_t>(p[i]);
}
}  // namespace

// ---- CONV_2D: packed [n_pad][k_pad] int8-domain filters, folded bias ---------

void CpuConv(const bh_conv_params& p, CpuPool& pool) {
  const long M = static_cast<long>(p.batch) * p.out_h * p.out_w;
  const int K = p.k_h * p.k_w * p.in_c;
  const uint8_t* in = static_cast<const uint8_t*>(p.input);
  const int8_t* W = p.weights;
  uint8_t* out = static_cast<uint8_t*>(p.output);
  const uint8_t* res = static_cast<const uint8_t*>(p.residual);
  const uint8_t* tab = static_cast<const uint8_t*>(p.out_table);
  const uint8_t xorb = static_cast<uint8_t>(p.in_xor);
  const int8_t padv = static_cast<int8_t>(p.in_zp);
  pool.ParallelFor(M, [&](long m0, long m1) {
    std::vector<int8_t> row(static_cast<size_t>(K));
    std::vector<int32_t> acc(static_cast<size_t>(p.out_c) + 4);
    for (long m = m0; m < m1; ++m) {
      const int ox = static_cast<int>(m % p.out_w);
      const long t = m / p.out_w;
      const int oy = static_cast<int>(t % p.out_h);
      const int n = static_cast<int>(t / p.out_h);
      const int y0 = oy * p.stride_h - p.pad_h, x0 = ox * p.stride_w - p.pad_w;
      // im2col row in the int8 domain; out-of-image taps hold the input zp
      int k = 0;
      for (int fy = 0; fy < p.k_h; ++fy) {
        const int y = y0 + fy * p.dil_h;
        for (int fx = 0; fx < p.k_w; ++fx) {
          const int x = x0 + fx * p.dil_w;
          if (y < 0 || y >= p.in_h || x < 0 || x >= p.in_w) {
            std::memset(&row[k], static_cast<uint8_t>(padv), p.in_c);
          } else {
            const uint8_t* src = in + ((static_cast<long>(n) * p.in_h + y) * p.in_w + x) * p.in_c;
            for (int c = 0; c < p.in_c; ++c) row[k + c] = static_cast<int8_t>(src[c] ^ xorb);
          }
          k += p.in_c;
        }
      }
      int32_t rowsum = 0;
      if (p.w_zp != 0)
        for (int i = 0; i < K; ++i) rowsum += row[i];
      int c = 0;
      for (; c + 4 <= p.out_c; c += 4) {
        const int8_t* w = W + static_cast<long>(c) * p.k_pad;
        Dot4(row.data(), w, w + p.k_pad, w + 2 * p.k_pad, w + 3 * p.k_pad, K, &acc[c]);
      }
      for (; c < p.out_c; ++c) acc[c] = Dot(row.data(), W + static_cast<long>(c) * p.k_pad, K);
      uint8_t* o = out + m * p.out_c;
      for (c = 0; c < p.out_c; ++c) {
        int32_t a = acc[c] + p.bias_eff[c];
        if (p.w_zp != 0) a -= p.w_zp * rowsum;
        int32_t v = Clamp(Requant(a, p.mult[c], p.shift[c]) + p.out_zp, p.act_min, p.act_max);
        if (res) {
          const int32_t q = Load8(res, m * p.out_c + c, p.in_xor == 0);
          const int32_t sy = RequantLt1((v + p.add_y_off) * (1 << p.add_left_shift), p.add_y_mult, p.add_y_shift);
          const int32_t sr = RequantLt1((q + p.add_r_off) * (1 << p.add_left_shift), p.add_r_mult, p.add_r_shift);
          v = Clamp(RequantLt1(sy + sr, p.add_o_mult, p.add_o_shift) + p.add_o_off, p.add_act_min, p.add_act_max);
        }
        const uint8_t byte = static_cast<uint8_t>(v);
        o[c] = tab ? tab[byte] : byte;
      }
    }
  });
}

// ---- DEPTHWISE_CONV_2D: [kh][kw][out_c] int8-domain filters, raw bias -------

void CpuDwConv(const bh_dwconv_params& p, CpuPool& pool) {
  const long pixels = static_cast<long>(p.batch) * p.out_h * p.out_w;
  const uint8_t* in = static_cast<const uint8_t*>(p.input);
  uint8_t* out = static_cast<uint8_t*>(p.output);
  const uint8_t* tab = static_cast<const uint8_t*>(p.out_table);
  const int32_t xorb = p.in_xor;
  pool.ParallelFor(pixels, [&](long m0, long m1) {
    std::vector<int32_t> acc(static_cast<size_t>(p.out_c));
    for (long m = m0; m < m1; ++m) {
      const int ox = static_cast<int>(m % p.out_w);
      const long t = m / p.out_w;
      const int oy = static_cast<int>(t % p.out_h);
      const int n = static_cast<int>(t / p.out_h);
      std::fill(acc.begin(), acc.end(), 0);
      for (int fy = 0; fy < p.k_h; ++fy) {
        const int y = oy * p.stride_h - p.pad_h + fy * p.dil_h;
        if (y < 0 || y >= p.in_h) continue;
        for (int fx = 0; fx < p.k_w; ++fx) {
          const int x = ox * p.stride_w - p.pad_w + fx * p.dil_w;
          if (x < 0 || x >= p.in_w) continue;
          const uint8_t* src = in + ((static_cast<long>(n) * p.in_h + y) * p.in_w + x) * p.in_c;
          const int8_t* w = p.weights + (static_cast<long>(fy) * p.k_w + fx) * p.out_c;
          for (int oc = 0; oc < p.out_c; ++oc) {
            const int32_t xv = static_cast<int8_t>(src[oc / p.depth_multiplier] ^ xorb);
            acc[oc] += (xv - p.in_zp) * (static_cast<int32_t>(w[oc]) - p.w_zp);
          }
        }
      }
      uint8_t* o = out + m * p.out_c;
      for (int oc = 0; oc < p.out_c; ++oc) {
        const int32_t r = Clamp(Requant(acc[oc] + p.bias[oc], p.mult[oc], p.shift[oc]) + p.out_zp, p.act_min, p.act_max);
        const uint8_t byte = static_cast<uint8_t>(r);
        o[oc] = tab ? tab[byte] : byte;
      }
    }
  });
}

// ---- FULLY_CONNECTED: acc = sum x'w' + bias_eff - w_zp * sum x' ---------------

void CpuFc(const bh_fc_params& p, CpuPool& pool) {
  const uint8_t* in = static_cast<const uint8_t*>(p.input);
  uint8_t* out = static_cast<uint8_t*>(p.output);
  const uint8_t* tab = static_cast<const uint8_t*>(p.out_table);
  const long work = static_cast<long>(p.rows) * p.units;
  pool.ParallelFor(work, [&](long i0, long i1) {
    std::vector<int8_t> row(static_cast<size_t>(p.depth));
    long cur = -1;
    int32_t xs = 0;
    for (long i = i0; i < i1; ++i) {
      const long r = i / p.units;
      const int u = static_cast<int>(i % p.units);
      if (r != cur) {
        cur = r;
        xs = 0;
        for (int k = 0; k < p.depth; ++k) {
          row[k] = static_cast<int8_t>(in[r * p.depth + k] ^ static_cast<uint8_t>(p.in_xor));
          xs += row[k];
        }
      }
      int32_t v = Dot(row.data(), p.weights + static_cast<long>(u) * p.depth_pad, p.depth) + p.bias_eff[u];
      if (p.w_zp != 0) v -= p.w_zp * xs;
      const int32_t q = Clamp(Requant(v, p.mult[u], p.shift[u]) + p.out_zp, p.act_min, p.act_max);
      const uint8_t byte = static_cast<uint8_t>(q);
      out[i] = tab ? tab[byte] : byte;
    }
  });
}

// ---- ADD / SUB / MUL (8-bit) with 4-D broadcast ------------------------------

void CpuEltwise(const bh_eltwise_params& p, CpuPool& pool) {
  const int* so = p.shape_o;
  const long n = static_cast<long>(so[0]) * so[1] * so[2] * so[3];
  const bool sg = p.in_signed != 0;
  const uint8_t* A = static_cast<const uint8_t*>(p.a);
  const uint8_t* B = static_cast<const uint8_t*>(p.b);
  uint8_t* O = static_cast<uint8_t*>(p.out);
  auto index = [](const int* s, long i0, long i1, long i2, long i3) {
    return (((s[0] == 1 ? 0 : i0) * s[1] + (s[1] == 1 ? 0 : i1)) * s[2] + (s[2] == 1 ? 0 : i2)) * s[3] +
           (s[3] == 1 ? 0 : i3);
  };
  pool.ParallelFor(n, [&](long b, long e) {
    for (long i = b; i < e; ++i) {
      const long i3 = i % so[3], t = i / so[3];
      const long i2 = t % so[2], t2 = t / so[2];
      const long i1 = t2 % so[1], i0 = t2 / so[1];
      const int32_t xa = Load8(A, index(p.shape_a, i0, i1, i2, i3), sg) + p.a_off;
      const int32_t xb = Load8(B, index(p.shape_b, i0, i1, i2, i3), sg) + p.b_off;
      int32_t o;
      if (p.kind == BH_ELT_ADD) {
        const int32_t sa = RequantLt1(xa * (1 << p.left_shift), p.a_mult, p.a_shift);
        const int32_t sb = RequantLt1(xb * (1 << p.left_shift), p.b_mult, p.b_shift);
        o = RequantLt1(sa + sb, p.o_mult, p.o_shift) + p.o_off;
      } else {
        o = Requant(xa * xb, p.o_mult, p.o_shift) + p.o_off;
      }
      O[i] = static_cast<uint8_t>(Clamp(o, p.act_min, p.act_max));
    }
  });
}

// ---- AVERAGE / MAX POOL_2D ---------------------------------------------------

void CpuPool2D(const bh_pool_params& p, CpuPool& pool) {
  const long pixels = static_cast<long>(p.batch) * p.out_h * p.out_w;
  const bool sg = p.in_signed != 0;
  const uint8_t* in = static_cast<const uint8_t*>(p.input);
  uint8_t* out = static_cast<uint8_t*>(p.output);
  pool.ParallelFor(pixels, [&](long m0, long m1) {
    for (long m = m0; m < m1; ++m) {
      const int ox = static_cast<int>(m % p.out_w);
      const long t = m / p.out_w;
      const int oy = static_cast<int>(t % p.out_h);
      const int n = static_cast<int>(t / p.out_h);
      const int y0 = oy * p.stride_h - p.pad_h, x0 = ox * p.stride_w - p.pad_w;
      const int fy0 = std::max(0, -y0), fy1 = std::min(p.f_h, p.in_h - y0);
      const int fx0 = std::max(0, -x0), fx1 = std::min(p.f_w, p.in_w - x0);
      for (int c = 0; c < p.channels; ++c) {
        int32_t a = p.kind == BH_POOL_AVG ? 0 : (sg ? -128 : 0);
        int cnt = 0;
        for (int fy = fy0; fy < fy1; ++fy)
          for (int fx = fx0; fx < fx1; ++fx) {
            const int32_t q = Load8(in, ((static_cast<long>(n) * p.in_h + y0 + fy) * p.in_w + x0 + fx) * p.channels + c, sg);
            a = p.kind == BH_POOL_AVG ? a + q : std::max(a, q);
            ++cnt;
          }
        if (p.kind == BH_POOL_AVG && cnt > 0) a = a > 0 ? (a + cnt / 2) / cnt : (a - cnt / 2) / cnt;
        out[m * p.channels + c] = static_cast<uint8_t>(Clamp(a, p.act_min, p.act_max));
      }
    }
  });
}

// ---- glue ops ---------------------------------------------------------------

// element-wise kernels split over the pool above this many elements
constexpr long kParallelElems = 1 << 16;

void CpuLutU8(const void* in, void* out, long n, const uint8_t* table, CpuPool& pool) {
  const uint8_t* s = static_cast<const uint8_t*>(in);
  uint8_t* d = static_cast<uint8_t*>(out);
  auto run = [&](long b, long e) {
    for (long i = b; i < e; ++i) d[i] = table[s[i]];
  };
  if (n >= kParallelElems) pool.ParallelFor(n, run);
  else run(0, n);
}

void CpuLutF32(const void* in, float* out, long n, const float* table, CpuPool& pool) {
  const uint8_t* s = static_cast<const uint8_t*>(in);
  auto run = [&](long b, long e) {
    for (long i = b; i < e; ++i) out[i] = table[s[i]];
  };
  if (n >= kParallelElems) pool.ParallelFor(n, run);
  else run(0, n);
}

// quantize.cc AffineQuantize: round(x / scale) + zp, clamped
void CpuQuantizeF32(const float* in, void* out, long n, float scale, int32_t zp, int out_signed, CpuPool& pool) {
  uint8_t* d = static_cast<uint8_t*>(out);
  const int32_t lo = out_signed ? -128 : 0, hi = out_signed ? 127 : 255;
  auto run = [&](long b, long e) {
    for (long i = b; i < e; ++i) {
      const volatile float q = in[i] / scale;  // one IEEE division, no contraction
      d[i] = static_cast<uint8_t>(Clamp(static_cast<int32_t>(std::round(static_cast<float>(q))) + zp, lo, hi));
    }
  };
  if (n >= kParallelElems) pool.ParallelFor(n, run);
  else run(0, n);
}

void CpuConcat(const bh_concat_params& p) {
  long out_row = 0;
  for (int k = 0; k < p.n_inputs; ++k) out_row += p.row[k];
  long off = 0;
  uint8_t* out = static_cast<uint8_t*>(p.output);
  for (int k = 0; k < p.n_inputs; ++k) {
    const uint8_t* src = static_cast<const uint8_t*>(p.input[k]);
    const uint8_t* tab = static_cast<const uint8_t*>(p.table[k]);
    for (long o = 0; o < p.outer; ++o) {
      uint8_t* dst = out + o * out_row + off;
      const uint8_t* s = src + o * p.row[k];
      if (tab) {
        for (long j = 0; j < p.row[k]; ++j) dst[j] = tab[s[j]];
      } else if (dst != s) {
        std::memmove(dst, s, static_cast<size_t>(p.row[k]));
      }
    }
    off += p.row[k];
  }
}

namespace {
// MIRROR_PAD source index (TFLite 2.9.2 mirror_pad.cc GetInputDimension;
// mode 1 REFLECT skips the edge element, 2 SYMMETRIC repeats it)
int MirrorIndex(int i, int before, int n, int mode) {
  const int offset = mode == 1 ? 1 : 0;
  if (i < before) {
    const int orig = before + offset - 1;
    return orig - std::min(i, orig - offset);
  }
  i -= before;
  if (i >= n) {
    i -= n;
    const int orig = n - (1 + offset);
    return orig - std::min(i, orig);
  }
  return i;
}
}  // namespace

void CpuPad(const bh_pad_params& p) {
  int os[4];
  for (int d = 0; d < 4; ++d) os[d] = p.in_shape[d] + p.pad_before[d] + p.pad_after[d];
  const int eb = p.elem_bytes;
  const uint8_t* in = static_cast<const uint8_t*>(p.input);
  uint8_t* out = static_cast<uint8_t*>(p.output);
  uint8_t value[8] = {0};
  std::memcpy(value, &p.value, std::min<size_t>(sizeof(p.value), sizeof(value)));
  long i = 0;
  for (int b = 0; b < os[0]; ++b)
    for (int y = 0; y < os[1]; ++y)
      for (int x = 0; x < os[2]; ++x)
        for (int c = 0; c < os[3]; ++c, ++i) {
          const int ib = b - p.pad_before[0], iy = y - p.pad_before[1], ix = x - p.pad_before[2],
                    ic = c - p.pad_before[3];
          const bool inside = ib >= 0 && ib < p.in_shape[0] && iy >= 0 && iy < p.in_shape[1] && ix >= 0 &&
                              ix < p.in_shape[2] && ic >= 0 && ic < p.in_shape[3];
          if (p.mode) {
            const long src = ((static_cast<long>(MirrorIndex(b, p.pad_before[0], p.in_shape[0], p.mode)) *
                                   p.in_shape[1] +
                               MirrorIndex(y, p.pad_before[1], p.in_shape[1], p.mode)) *
                                  p.in_shape[2] +
                              MirrorIndex(x, p.pad_before[2], p.in_shape[2], p.mode)) *
                                 p.in_shape[3] +
                             MirrorIndex(c, p.pad_before[3], p.in_shape[3], p.mode);
            std::memcpy(out + i * eb, in + src * eb, eb);
          } else if (inside) {
            const long src = ((static_cast<long>(ib) * p.in_shape[1] + iy) * p.in_shape[2] + ix) * p.in_shape[3] + ic;
            std::memcpy(out + i * eb, in + src * eb, eb);
          } else {
            std::memcpy(out + i * eb, value, eb);
          }
        }
}

void CpuResizeNearest(const bh_resize_nearest_params& p) {
  const uint8_t* in = static_cast<const uint8_t*>(p.input);
  uint8_t* out = static_cast<uint8_t*>(p.output);
  for (int n = 0; n < p.batch; ++n)
    for (int y = 0; y < p.out_h; ++y)
      for (int x = 0; x < p.out_w; ++x)
        std::memcpy(out + ((static_cast<long>(n) * p.out_h + y) * p.out_w + x) * p.row_bytes,
                    in + ((static_cast<long>(n) * p.in_h + p.y_index[y]) * p.in_w + p.x_index[x]) * p.row_bytes,
                    static_cast<size_t>(p.row_bytes));
}

// reference_ops::ResizeBilinearInteger (int8, 10-bit fixed point)
void CpuResizeBilinear(const bh_resize_bilinear_params& p) {
  const int8_t* in = static_cast<const int8_t*>(p.input);
  int8_t* out = static_cast<int8_t*>(p.output);
  constexpr int32_t one = 1 << 10;
  long i = 0;
  for (int n = 0; n < p.batch; ++n)
    for (int y = 0; y < p.out_h; ++y) {
      const int y0 = p.y_tab[3 * y], y1 = p.y_tab[3 * y + 1], fy = p.y_tab[3 * y + 2] - one * y0;
      for (int x = 0; x < p.out_w; ++x) {
        const int x0 = p.x_tab[3 * x], x1 = p.x_tab[3 * x + 1], fx = p.x_tab[3 * x + 2] - one * x0;
        const int8_t* b = in + static_cast<long>(n) * p.in_h * p.in_w * p.channels;
        for (int c = 0; c < p.channels; ++c, ++i) {
          const int64_t v00 = b[(static_cast<long>(y0) * p.in_w + x0) * p.channels + c];
          const int64_t v10 = b[(static_cast<long>(y1) * p.in_w + x0) * p.channels + c];
          const int64_t v01 = b[(static_cast<long>(y0) * p.in_w + x1) * p.channels + c];
          const int64_t v11 = b[(static_cast<long>(y1) * p.in_w + x1) * p.channels + c];
          const int64_t s = v00 * ((one - fy) * (one - fx)) + v10 * (fy * (one - fx)) + v01 * ((one - fy) * fx) +
                            v11 * (fy * fx);
          const int64_t rnd = s > 0 ? (1 << 19) : -(1 << 19);
          out[i] = static_cast<int8_t>((s + rnd) / (1 << 20));
        }
      }
    }
}

// optimized_ops::ResizeBilinear<uint8> (float weights, + 0.5f, truncation);
// this file is built with -ffp-contract=off, so every product and sum is
// rounded separately as in the reference's x86 build
void CpuResizeBilinearU8(const bh_resize_bilinear_u8_params& p) {
  const uint8_t* in = static_cast<const uint8_t*>(p.input);
  uint8_t* out = static_cast<uint8_t*>(p.output);
  long i = 0;
  for (int n = 0; n < p.batch; ++n)
    for (int y = 0; y < p.out_h; ++y) {
      const int y0 = p.y_idx[2 * y], y1 = p.y_idx[2 * y + 1];
      const float dy = p.y_frac[y];
      for (int x = 0; x < p.out_w; ++x) {
        const int x0 = p.x_idx[2 * x], x1 = p.x_idx[2 * x + 1];
        const float dx = p.x_frac[x];
        const float s0 = (1.0f - dy) * (1.0f - dx), s1 = (1.0f - dy) * dx, s2 = dy * (1.0f - dx), s3 = dy * dx;
        const uint8_t* b = in + static_cast<long>(n) * p.in_h * p.in_w * p.channels;
        for (int c = 0; c < p.channels; ++c, ++i) {
          const float v = static_cast<float>(b[(static_cast<long>(y0) * p.in_w + x0) * p.channels + c]) * s0 +
                          static_cast<float>(b[(static_cast<long>(y0) * p.in_w + x1) * p.channels + c]) * s1 +
                          static_cast<float>(b[(static_cast<long>(y1) * p.in_w + x0) * p.channels + c]) * s2 +
                          static_cast<float>(b[(static_cast<long>(y1) * p.in_w + x1) * p.channels + c]) * s3 + 0.5f;
          out[i] = static_cast<uint8_t>(static_cast<int>(v));
        }
      }
    }
}

// optimized_ops::Softmax (8-bit) with the exp table built on the host
void CpuSoftmax(const bh_softmax_params& p) {
  const bool sg = p.is_signed != 0;
  const int32_t lo = sg ? -128 : 0, hi = sg ? 127 : 255;
  for (long r = 0; r < p.rows; ++r) {
    const uint8_t* x = static_cast<const uint8_t*>(p.input) + r * p.depth;
    uint8_t* y = static_cast<uint8_t*>(p.output) + r * p.depth;
    int32_t mx = lo;
    for (int j = 0; j < p.depth; ++j) mx = std::max(mx, Load8(x, j, sg));
    const float* to = p.table + 255 - mx;
    volatile float sum = 0.0f;
    for (int j = 0; j < p.depth; ++j) sum = sum + to[Load8(x, j, sg)];
    const volatile float denom = sum * p.out_scale;
    const volatile float inv = 1.0f / denom;
    for (int j = 0; j < p.depth; ++j) {
      const volatile float pr = to[Load8(x, j, sg)] * inv;
      int32_t q;
      if (sg) {
        q = static_cast<int32_t>(std::round(static_cast<float>(pr))) + p.out_zp;
      } else {
        const volatile float h = pr + 0.5f;
        q = static_cast<int32_t>(static_cast<float>(h)) + p.out_zp;
      }
      y[j] = static_cast<uint8_t>(Clamp(q, lo, hi));
    }
  }
}

void CpuZeroInsert(const bh_zero_insert_params& p) {
  const uint8_t* in = static_cast<const uint8_t*>(p.input);
  uint8_t* out = static_cast<uint8_t*>(p.output);
  const size_t total = static_cast<size_t>(p.batch) * p.out_h * p.out_w * p.channels;
  std::memset(out, static_cast<int>(p.fill & 0xffu), total);
  for (int n = 0; n < p.batch; ++n)
    for (int y = 0; y < p.in_h; ++y)
      for (int x = 0; x < p.in_w; ++x)
        std::memcpy(out + ((static_cast<long>(n) * p.out_h + y * p.stride_h) * p.out_w + x * p.stride_w) * p.channels,
                    in + ((static_cast<long>(n) * p.in_h + y) * p.in_w + x) * p.channels,
                    static_cast<size_t>(p.channels));
}

namespace {
inline float ClampF(float v, float lo, float hi) { return std::min(std::max(v, lo), hi); }
}  // namespace

void CpuConvF32(const bh_conv_f32_params& p, CpuPool& pool) {
  const long pixels = static_cast<long>(p.batch) * p.out_h * p.out_w;
  pool.ParallelFor(pixels, [&](long m0, long m1) {
    std::vector<float> acc(static_cast<size_t>(p.out_c));
    for (long m = m0; m < m1; ++m) {
      const int ox = static_cast<int>(m % p.out_w);
      const long t = m / p.out_w;
      const int oy = static_cast<int>(t % p.out_h);
      const int n = static_cast<int>(t / p.out_h);
      std::fill(acc.begin(), acc.end(), 0.f);
      for (int fy = 0; fy < p.k_h; ++fy) {
        const int y = oy * p.stride_h - p.pad_h + fy * p.dil_h;
        if (y < 0 || y >= p.in_h) continue;
        for (int fx = 0; fx < p.k_w; ++fx) {
          const int x = ox * p.stride_w - p.pad_w + fx * p.dil_w;
          if (x < 0 || x >= p.in_w) continue;
          const float* src = p.input + ((static_cast<long>(n) * p.in_h + y) * p.in_w + x) * p.in_c;
          if (p.depthwise) {
            const float* w = p.weights + static_cast<long>(fy * p.k_w + fx) * p.out_c;
            for (int c = 0; c < p.out_c; ++c) acc[c] += src[c / p.depth_multiplier] * w[c];
          } else {
            const float* w = p.weights + static_cast<long>((fy * p.k_w + fx) * p.in_c) * p.out_c;
            for (int ci = 0; ci < p.in_c; ++ci) {
              const float xv = src[ci];
              const float* wr = w + static_cast<long>(ci) * p.out_c;
              for (int c = 0; c < p.out_c; ++c) acc[c] += xv * wr[c];
            }
          }
        }
      }
      float* o = p.output + m * p.out_c;
      for (int c = 0; c < p.out_c; ++c) o[c] = ClampF(acc[c] + (p.bias ? p.bias[c] : 0.f), p.act_min, p.act_max);
    }
  });
}

void CpuFcF32(const bh_fc_f32_params& p, CpuPool& pool) {
  pool.ParallelFor(static_cast<long>(p.rows) * p.units, [&](long b, long e) {
    for (long i = b; i < e; ++i) {
      const long r = i / p.units;
      const int u = static_cast<int>(i % p.units);
      const float* x = p.input + r * p.depth;
      const float* w = p.weights + static_cast<long>(u) * p.depth;
      float acc = 0.f;
      for (int k = 0; k < p.depth; ++k) acc += x[k] * w[k];
      p.output[i] = ClampF(acc + (p.bias ? p.bias[u] : 0.f), p.act_min, p.act_max);
    }
  });
}

void CpuEltwiseF32(const bh_eltwise_f32_params& p) {
  const int* so = p.shape_o;
  const long n = static_cast<long>(so[0]) * so[1] * so[2] * so[3];
  auto index = [](const int* s, long i0, long i1, long i2, long i3) {
    return (((s[0] == 1 ? 0 : i0) * s[1] + (s[1] == 1 ? 0 : i1)) * s[2] + (s[2] == 1 ? 0 : i2)) * s[3] +
           (s[3] == 1 ? 0 : i3);
  };
  for (long i = 0; i < n; ++i) {
    const long i3 = i % so[3], t = i / so[3];
    const long i2 = t % so[2], t2 = t / so[2];
    const long i1 = t2 % so[1], i0 = t2 / so[1];
    const float a = p.a[index(p.shape_a, i0, i1, i2, i3)];
    const float b = p.b[index(p.shape_b, i0, i1, i2, i3)];
    const float v = p.kind == BH_ELTF_ADD   ? a + b
                    : p.kind == BH_ELTF_SUB ? a - b
                    : p.kind == BH_ELTF_MUL ? a * b
                                            : (a - b) * (a - b);  // SQUARED_DIFFERENCE
    p.out[i] = ClampF(v, p.act_min, p.act_max);
  }
}

void CpuPoolF32(const bh_pool_f32_params& p) {
  long i = 0;
  for (int n = 0; n < p.batch; ++n)
    for (int oy = 0; oy < p.out_h; ++oy)
      for (int ox = 0; ox < p.out_w; ++ox) {
        const int y0 = oy * p.stride_h - p.pad_h, x0 = ox * p.stride_w - p.pad_w;
        const int fy0 = std::max(0, -y0), fy1 = std::min(p.f_h, p.in_h - y0);
        const int fx0 = std::max(0, -x0), fx1 = std::min(p.f_w, p.in_w - x0);
        for (int c = 0; c < p.channels; ++c, ++i) {
          float acc = p.kind == BH_POOL_AVG ? 0.f : -std::numeric_limits<float>::infinity();
          int cnt = 0;
          for (int fy = fy0; fy < fy1; ++fy)
            for (int fx = fx0; fx < fx1; ++fx) {
              const float v = p.input[((static_cast<long>(n) * p.in_h + y0 + fy) * p.in_w + x0 + fx) * p.channels + c];
              acc = p.kind == BH_POOL_AVG ? acc + v : std::max(acc, v);
              ++cnt;
            }
          if (p.kind == BH_POOL_AVG) acc = acc / static_cast<float>(cnt);
          p.output[i] = ClampF(acc, p.act_min, p.act_max);
        }
      }
}

void CpuUnaryF32(int kind, const float* in, float* out, long n, float lo, float hi) {
  for (long i = 0; i < n; ++i)
    out[i] = kind == BH_UNARY_LOGISTIC ? 1.0f / (1.0f + std::exp(-in[i]))
             : kind == BH_UNARY_RSQRT  ? 1.0f / std::sqrt(in[i])
                                       : ClampF(in[i], lo, hi);
}

void CpuSoftmaxF32(const float* in, float* out, long rows, int depth, float beta) {
  for (long r = 0; r < rows; ++r) {
    const float* x = in + r * depth;
    float* y = out + r * depth;
    float mx = -std::numeric_limits<float>::infinity();
    for (int k = 0; k < depth; ++k) mx = std::max(mx, x[k]);
    float sum = 0.f;
    for (int k = 0; k < depth; ++k) sum += std::exp((x[k] - mx) * beta);
    for (int k = 0; k < depth; ++k) y[k] = std::exp((x[k] - mx) * beta) / sum;
  }
}

// DecodeCenterSizeBoxes + MultiClassFastNMS (max_classes_per_detection 1)
// + NonMaxSuppressionSingleClassHelper, in the reference's arithmetic order
void CpuDetectionPostprocess(const CpuDetectionParams& p, CpuPool& pool) {
  const int n = p.num_boxes;
  struct Box {
    float ymin, xmin, ymax, xmax;
  };
  std::vector<Box> boxes(static_cast<size_t>(n));
  std::vector<float> max_score(static_cast<size_t>(n));
  std::vector<int> best(static_cast<size_t>(n));
  const int label_offset = p.num_classes_with_background - p.num_classes;
  pool.ParallelFor(n, [&](long b, long e) {
    for (long i = b; i < e; ++i) {
      const float* be = p.box_encodings + 4 * i;
      const float* an = p.anchors + 4 * i;
      const float yc = static_cast<float>(static_cast<double>(be[0]) / static_cast<double>(p.scale_y) *
                                              static_cast<double>(an[2]) +
                                          static_cast<double>(an[0]));
      const float xc = static_cast<float>(static_cast<double>(be[1]) / static_cast<double>(p.scale_x) *
                                              static_cast<double>(an[3]) +
                                          static_cast<double>(an[1]));
      const float hh = static_cast<float>(0.5 * std::exp(static_cast<double>(be[2]) / static_cast<double>(p.scale_h)) *
                                          static_cast<double>(an[2]));
      const float hw = static_cast<float>(0.5 * std::exp(static_cast<double>(be[3]) / static_cast<double>(p.scale_w)) *
                                          static_cast<double>(an[3]));
      boxes[i] = {yc - hh, xc - hw, yc + hh, xc + hw};
      const float* sc = p.class_scores + i * p.num_classes_with_background + label_offset;
      int arg = 0;
      float mx = sc[0];
      for (int c = 1; c < p.num_classes; ++c)
        if (sc[c] > mx) {
          mx = sc[c];
          arg = c;
        }
      max_score[i] = mx;
      best[i] = arg;
    }
  });
  // Greedy NMS in stable descending score order, as the reference's
  // stable_sort + suppression sweep: only SELECTED boxes suppress, so a
  // candidate is selected iff its IoU with every box selected before it is
  // <= iou_threshold.  The candidates are therefore drawn lazily from a heap
  // (score descending, index ascending = the stable order) and each is
  // checked against the <= max_detections boxes selected so far; the draw
  // stops once max_detections are selected.  Same selections, same float
  // expressions (IoU of the selected box against the candidate), without
  // sorting every box above the threshold or sweeping them per selection.
  std::vector<int> heap;
  for (int i = 0; i < n; ++i)
    if (max_score[i] >= p.score_threshold) heap.push_back(i);
  const int out_size = std::min(static_cast<int>(heap.size()), p.max_detections);
  auto later = [&](int a, int b) {  // heap order: a is drawn after b
    return max_score[a] < max_score[b] || (max_score[a] == max_score[b] && a > b);
  };
  std::make_heap(heap.begin(), heap.end(), later);
  auto area = [&](const Box& b) { return (b.ymax - b.ymin) * (b.xmax - b.xmin); };
  std::vector<int> selected;
  while (!heap.empty() && static_cast<int>(selected.size()) < out_size) {
    std::pop_heap(heap.begin(), heap.end(), later);
    const int cand = heap.back();
    heap.pop_back();
    const Box& bj = boxes[cand];
    const float aj = area(bj);
    bool keep_it = true;
    for (int s : selected) {
      const Box& bi = boxes[s];
      const float ai = area(bi);
      float iou = 0.0f;
      if (ai > 0.0f && aj > 0.0f) {
        const float iy0 = std::max(bi.ymin, bj.ymin), ix0 = std::max(bi.xmin, bj.xmin);
        const float iy1 = std::min(bi.ymax, bj.ymax), ix1 = std::min(bi.xmax, bj.xmax);
        const float inter = std::max(iy1 - iy0, 0.0f) * std::max(ix1 - ix0, 0.0f);
        iou = inter / (ai + aj - inter);
      }
      if (iou > p.iou_threshold) {
        keep_it = false;
        break;
      }
    }
    if (keep_it) selected.push_back(cand);
  }
  std::memset(p.out_boxes, 0, sizeof(float) * 4 * p.max_detections);
  std::memset(p.out_classes, 0, sizeof(float) * p.max_detections);
  std::memset(p.out_scores, 0, sizeof(float) * p.max_detections);
  for (size_t k = 0; k < selected.size(); ++k) {
    const Box& b = boxes[selected[k]];
    p.out_boxes[4 * k] = b.ymin;
    p.out_boxes[4 * k + 1] = b.xmin;
    p.out_boxes[4 * k + 2] = b.ymax;
    p.out_boxes[4 * k + 3] = b.xmax;
    p.out_classes[k] = static_cast<float>(best[selected[k]]);
    p.out_scores[k] = max_score[selected[k]];
  }
  p.out_num[0] = static_cast<float>(selected.size());
}

void CpuMean(const CpuMeanParams& p, CpuPool& pool) {
  pool.ParallelFor(p.outer * p.inner, [&](long lo, long hi) {
    for (long o = lo; o < hi; ++o) {
      const long a = o / p.inner, c = o % p.inner;
      const long base = a * p.reduce * p.inner + c;
      if (p.type == 0) {
        const float* x = static_cast<const float*>(p.input);
        float s = 0.f;
        for (long r = 0; r < p.reduce; ++r) s += x[base + r * p.inner];
        static_cast<float*>(p.output)[o] = s / static_cast<float>(p.reduce);
        continue;
      }
      int32_t acc = 0;
      if (p.type == 1) {
        const int8_t* x = static_cast<const int8_t*>(p.input);
        for (long r = 0; r < p.reduce; ++r) acc += x[base + r * p.inner];
      } else {
        const uint8_t* x = static_cast<const uint8_t*>(p.input);
        for (long r = 0; r < p.reduce; ++r) acc += x[base + r * p.inner];
      }
      acc = MultiplyByQuantizedMultiplier(acc, p.multiplier, p.shift) + p.bias;
      if (p.type == 1) static_cast<int8_t*>(p.output)[o] = static_cast<int8_t>(std::min(std::max(acc, -128), 127));
      else static_cast<uint8_t*>(p.output)[o] = static_cast<uint8_t>(std::min(std::max(acc, 0), 255));
    }
  });
}

}  // namespace hip
}  // namespace band
