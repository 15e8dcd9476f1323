// HipModelExecutor: fusion passes over the lowered launch program - grouped
// independent convs, the inverted-residual block, the fused chains (every
// form timed on the real buffers, decisions cached per geometry / device and
// in BAND_HIP_TUNE_FILE), glue-op epilogue folds.  Split from model_executor.cc.
#include "backend/hip/executor_internal.h"
#include <mutex>
#include <unordered_map>

namespace band {
namespace hip {

using namespace ex;

namespace {
// Device pointers a launch reads and writes (tensor bases or slices inside
// the arena; constants are filtered out by the caller).  false: a launch kind
// not analysed here - grouping treats it as a barrier.
bool LaunchIo(const Launch& l, std::vector<const void*>* rd, std::vector<const void*>* wr) {
  switch (l.kind) {
    case Launch::kConv:
      *rd = {l.conv.input, l.conv.residual};
      *wr = {l.conv.output};
      return true;
    case Launch::kDwConv:
      *rd = {l.dw.input};
      *wr = {l.dw.output};
      return true;
    case Launch::kChain:
      *rd = {l.chain.dw.input, l.chain.pw1.residual};
      *wr = {l.chain.pw1.output, l.chain.has_pw2 ? l.chain.pw2.output : nullptr};
      return true;
    case Launch::kIrb:
      *rd = {l.irb.input};
      *wr = {l.irb.output};
      return true;
    case Launch::kFc:
      *rd = {l.fc.input};
      *wr = {l.fc.output};
      return true;
    case Launch::kEltwise:
      *rd = {l.elt.a, l.elt.b};
      *wr = {l.elt.out};
      return true;
    case Launch::kPool:
      *rd = {l.pool.input};
      *wr = {l.pool.output};
      return true;
    case Launch::kLutU8:
    case Launch::kCopy:
      *rd = {l.src};
      *wr = {l.dst};
      return true;
    case Launch::kConcat:
      rd->assign(l.concat.input, l.concat.input + l.concat.n_inputs);
      *wr = {l.concat.output};
      return true;
    case Launch::kConvGroup:
      rd->clear();
      wr->clear();
      for (const bh_conv_params& m : l.members) {
        rd->push_back(m.input);
        rd->push_back(m.residual);
        wr->push_back(m.output);
      }
      return true;
    default:
      return false;
  }
}
}  // namespace

// Detector and pose heads are many small convs that read feature maps
// produced long before and write tensors read only at the end (SSD's 12
// box / class predictors feed two CONCATENATIONs; PoseNet's four heads are
// the outputs).  Each alone is a dispatch at the ~4 us empty-kernel floor.
// Walking the launches in order, a conv that routes to the general MFMA
// kernel joins a pending set instead of being emitted; a later launch that
// reads or overwrites a pending conv's output, or writes a pending conv's
// input, first flushes that conv (alone); a launch kind not analysed here
// flushes everything.  What stays pending to the end of a run is emitted as
// one conv_group launch at the position of the first launch that needs any
// of it - every member then still runs after its producers and before its
// consumers.  Members of a group never read each other's outputs.
absl::Status HipModelExecutor::GroupConvs(PreparedSubgraph* sg) {
  // accesses by arena slot (the tensor slot, aliases excluded, holding the
  // pointer) and byte interval within it: [lo, hi) in every image at
  // `stride` (0: one interval).  Only conv outputs are known exactly (heads
  // writing per-image slices of one concatenated tensor must not conflict
  // with each other); anything else covers its whole slot.
  std::vector<std::pair<uintptr_t, uintptr_t>> slots;
  {
    const uintptr_t base = reinterpret_cast<uintptr_t>(sg->arena->ptr());
    std::map<size_t, size_t> by_off;
    for (const auto& kv : sg->offset) {
      size_t& b = by_off[kv.second];
      b = std::max(b, meta_[kv.first]->bytes);
    }
    for (const auto& kv : by_off) slots.emplace_back(base + kv.first, base + kv.first + kv.second);
  }
  struct Acc {
    int slot;
    long lo, hi, stride;
  };
  constexpr long kAll = std::numeric_limits<long>::max();
  auto acc_of = [&](const void* p, long bytes, long stride) -> Acc {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto it = std::upper_bound(slots.begin(), slots.end(), std::make_pair(a, ~uintptr_t(0)));
    if (!p || it == slots.begin()) return Acc{-1, 0, 0, 0};
    --it;
    if (a >= it->second) return Acc{-1, 0, 0, 0};
    const long lo = static_cast<long>(a - it->first);
    return Acc{static_cast<int>(it - slots.begin()), bytes > 0 ? lo : 0, bytes > 0 ? lo + bytes : kAll, stride};
  };
  auto accesses = [&](const std::vector<const void*>& ps) {
    std::vector<Acc> out;
    for (const void* p : ps) {
      const Acc a = acc_of(p, 0, 0);
      if (a.slot >= 0) out.push_back(a);
    }
    return out;
  };
  auto conv_write = [&](const bh_conv_params& c) {
    const long hwn = static_cast<long>(c.out_h) * c.out_w * c.out_c;
    return c.out_img_stride ? acc_of(c.output, hwn, c.out_img_stride) : acc_of(c.output, hwn * c.batch, 0);
  };
  auto overlap = [&](const Acc& a, const Acc& b) {
    if (a.slot != b.slot) return false;
    if (a.stride != b.stride) return true;  // (per-image vs whole-tensor: conservative)
    return a.lo < b.hi && b.lo < a.hi;
  };
  auto intersects = [&](const std::vector<Acc>& x, const std::vector<Acc>& y) {
    for (const Acc& a : x)
      for (const Acc& b : y)
        if (overlap(a, b)) return true;
    return false;
  };
  struct Pending {
    Launch l;
    std::vector<Acc> rd, wr;
  };
  std::vector<Launch> out;
  std::vector<Pending> pending;
  // emits `set` (mutually independent convs) as one group per window type
  auto emit = [&](std::vector<Pending>& set) -> absl::Status {
    for (int one = 1; one >= 0; --one) {
      std::vector<const Launch*> ms;
      for (const Pending& p : set) {
        const bh_conv_params& c = p.l.conv;
        const int is1 = c.k_h == 1 && c.k_w == 1 && c.pad_h == 0 && c.pad_w == 0;
        if (is1 == one) ms.push_back(&p.l);
      }
      if (ms.empty()) continue;
      if (ms.size() == 1) {
        out.push_back(*ms[0]);
        continue;
      }
      Launch G;
      G.kind = Launch::kConvGroup;
      G.op_index = ms[0]->op_index;
      G.out_tensor = ms[0]->out_tensor;
      G.kernel = "conv_group_kernel";
      for (const Launch* m : ms) {
        G.members.push_back(m->conv);
        G.alg_bytes += m->alg_bytes;
        G.alg_ops += m->alg_ops;
      }
      std::vector<char> host(bh_conv_group_table_bytes(static_cast<int>(ms.size())));
      if (host.empty() || bh_conv_group_plan(G.members.data(), static_cast<int>(ms.size()), host.data(),
                                             &G.cgroup) != 0) {
        for (const Launch* m : ms) out.push_back(*m);  // not groupable after all: keep them
        continue;
      }
      auto blob = std::make_shared<DeviceBlob>(ordinal_, host.size());
      if (!blob->ok() || !blob->Upload(0, host.data(), host.size())) return HipErr(1, "upload conv group table");
      sg->consts.push_back(blob);
      G.cgroup.table = blob->ptr();
      out.push_back(std::move(G));
    }
    set.clear();
    return absl::OkStatus();
  };
  const size_t max_members = 32;
  for (Launch& l : sg->launches) {
    std::vector<const void*> rdp, wrp;
    if (!LaunchIo(l, &rdp, &wrp)) {
      RETURN_STATUS_IF(emit(pending));
      out.push_back(std::move(l));
      continue;
    }
    const std::vector<Acc> rd = accesses(rdp);
    std::vector<Acc> wr = accesses(wrp);
    if (l.kind == Launch::kConv) {
      const Acc w = conv_write(l.conv);
      wr.clear();
      if (w.slot >= 0) wr.push_back(w);
    }
    const bool groupable = l.kind == Launch::kConv && bh_conv_group_ok(&l.conv) && !rd.empty() && !wr.empty();
    // pending convs this launch depends on (reads or overwrites their
    // output) or that depend on it (it overwrites their input)
    std::vector<Pending> hit, keep;
    for (Pending& p : pending)
      (intersects(rd, p.wr) || intersects(wr, p.wr) || intersects(wr, p.rd) ? hit : keep).push_back(std::move(p));
    pending = std::move(keep);
    if (!hit.empty()) {
      if (groupable) {
        // a conv consuming pending ones (a detector's next extra layer):
        // only those go now, the rest keep waiting for more members
        RETURN_STATUS_IF(emit(hit));
      } else {
        // a consumer of the group (CONCATENATION, ...): everything pending
        // runs here, as one launch
        for (Pending& p : hit) pending.push_back(std::move(p));
        RETURN_STATUS_IF(emit(pending));
      }
    }
    if (groupable && pending.size() < max_members) {
      pending.push_back(Pending{std::move(l), rd, wr});
      continue;
    }
    // a launch that stays put: pending convs it does not touch are deferred
    // past it
    out.push_back(std::move(l));
  }
  RETURN_STATUS_IF(emit(pending));
  sg->launches = std::move(out);
  return absl::OkStatus();
}

namespace {
bool Is1x1S1(const bh_conv_params& c) {
  return c.k_h == 1 && c.k_w == 1 && c.stride_h == 1 && c.stride_w == 1 && c.pad_h == 0 && c.pad_w == 0;
}

// Static latency model for a fused block's tile (used when it cannot be
// measured): (workgroup rounds over 256 CUs) x (MFMA tiles + depthwise /
// epilogue work per workgroup) / waves - halo recompute of small tiles
// against too few workgroups of large ones.
double IrbModelCost(const bh_irb_params& q, int t, size_t lds) {
  const int R = ((t - 1) * q.stride + 3) * ((t - 1) * q.stride + 3);
  const double mt1 = (R + 15) / 16, mt3 = (t * t + 15) / 16;
  const double ks1 = (q.in_c + 63) / 64, ks3 = (q.exp_c + 63) / 64;
  const double work = (q.has_expand ? mt1 * (q.exp_c / 16) * (1.0 + ks1) : 0.0) +  // +1: epilogue
                      mt3 * 16 * q.exp_c / 256.0 * 3.0 +                          // depthwise
                      mt3 * ((q.out_c + 15) / 16) * ks3 + t * t * q.out_c / 64.0;
  const int nw = lds > 80 * 1024 ? 16 : 8;
  const double per_cu = lds > 80 * 1024 ? 1 : 2;
  const long wg = static_cast<long>(q.batch) * ((q.out_h + t - 1) / t) * ((q.out_w + t - 1) / t);
  const double rounds = std::ceil(static_cast<double>(wg) / (256.0 * per_cu));
  return rounds * (work / nw + 8.0);  // + fixed per-workgroup latency
}

// Measured choices, shared by every executor of the process: one block
// geometry is timed once per device.  Value: tile edge, or 0 = keep unfused.
std::mutex g_tune_mu;
std::unordered_map<std::string, int> g_tune;

// BAND_HIP_TUNE_FILE: decisions persist across processes ("<key> <tile>"
// lines), so a profiled run replays exactly the launch sequence a timed run
// chose (the profiler's per-dispatch overhead would otherwise bias a fresh
// measurement).  Loaded once; new decisions are appended.
const char* TuneFile() {
  const char* f = std::getenv("BAND_HIP_TUNE_FILE");
  return f && f[0] ? f : nullptr;
}
void LoadTuneFileLocked() {
  static bool loaded = false;
  if (loaded) return;
  loaded = true;
  const char* path = TuneFile();
  if (!path) return;
  if (FILE* fp = std::fopen(path, "r")) {
    char key[256];
    int tile = 0;
    while (std::fscanf(fp, "%255s %d", key, &tile) == 2) g_tune[key] = tile;
    std::fclose(fp);
  }
}
void AppendTuneFileLocked(const std::string& key, int tile) {
  const char* path = TuneFile();
  if (!path) return;
  if (FILE* fp = std::fopen(path, "a")) {
    std::fprintf(fp, "%s %d\n", key.c_str(), tile);
    std::fclose(fp);
  }
}

// bumped whenever a chain form's LDS layout or parameter rules change, so a
// tune file written by an older kernel tree is not replayed against this one
// (11: column-reuse depthwise phase, every raster form re-measured)
constexpr int kChainTuneVersion = 12;
// chain choices from here up name a stage form (FuseChains)
constexpr int kStageChoice = 100000;

std::string IrbKey(int ordinal, const bh_irb_params& q) {
  char buf[256];
  std::snprintf(buf, sizeof(buf), "%d:%d:%dx%dx%d:%d:%d:%dx%d:%d:%d:%d", ordinal, q.batch, q.in_h, q.in_w, q.in_c,
                q.exp_c, q.out_c, q.out_h, q.out_w, q.stride, q.has_expand, q.has_residual);
  return buf;
}
}  // namespace

double HipModelExecutor::TimeLaunches(const std::vector<const Launch*>& ls, int iters) {
  if (device_flag_ != DeviceFlag::kGPU || !stream_ || ls.empty()) return -1.0;
  bh_event_t e0 = nullptr, e1 = nullptr;
  if (bh_event_create(&e0) != 0) return -1.0;
  if (bh_event_create(&e1) != 0) {
    bh_event_destroy(e0);
    return -1.0;
  }
  double us = -1.0;
  bool ok = true;
  for (int w = 0; w < 2 && ok; ++w)
    for (const Launch* l : ls) ok = ok && EnqueueLaunch(*l).ok();
  // head start: the whole timed sequence is queued before the GPU reaches
  // it, so the events see back-to-back execution (as in a replayed graph),
  // not host submission gaps
  ok = ok && bh_spin_us(stream_, 300 + 40 * iters * static_cast<int>(ls.size())) == 0;
  if (ok && bh_event_record(e0, stream_) == 0) {
    for (int it = 0; it < iters && ok; ++it)
      for (const Launch* l : ls) ok = ok && EnqueueLaunch(*l).ok();
    float ms = 0.f;
    if (ok && bh_event_record(e1, stream_) == 0 && bh_stream_sync(stream_) == 0 &&
        bh_event_elapsed_ms(e0, e1, &ms) == 0)
      us = 1e3 * ms / iters;
  }
  bh_stream_sync(stream_);
  bh_event_destroy(e0);
  bh_event_destroy(e1);
  return us;
}

// Rewrites [conv1x1 ->] dw3x3 -> conv1x1 [+fused ADD] launch runs into one
// bh_irb_i8 launch when the intermediates are private to the run.
void HipModelExecutor::FuseBlocks(const HipModel& model, PreparedSubgraph* sg) {
  const TflModel& d = model.desc();
  auto private_tensor = [&](int t, int only_consumer) {
    if (consumers_[t].size() != 1 || consumers_[t][0] != only_consumer) return false;
    if (sg->no_fuse.count(t) || sg->extra_d2h.count(t)) return false;
    if (std::find(sg->outputs.begin(), sg->outputs.end(), t) != sg->outputs.end()) return false;
    return std::find(d.outputs.begin(), d.outputs.end(), t) == d.outputs.end();
  };
  std::vector<Launch> out;
  const auto& L = sg->launches;
  for (size_t i = 0; i < L.size(); ++i) {
    // candidate run: [E] D P
    const Launch* E = nullptr;
    size_t j = i;
    if (L[i].kind == Launch::kConv && i + 2 < L.size() && L[i + 1].kind == Launch::kDwConv &&
        L[i + 2].kind == Launch::kConv) {
      E = &L[i];
      j = i + 1;
    } else if (!(L[i].kind == Launch::kDwConv && i + 1 < L.size() && L[i + 1].kind == Launch::kConv)) {
      out.push_back(L[i]);
      continue;
    }
    const Launch& D = L[j];
    const Launch& P = L[j + 1];
    const bh_dwconv_params& dw = D.dw;
    const bh_conv_params& pc = P.conv;
    bool ok = dw.in_xor == 0 && dw.w_zp == 0 && dw.depth_multiplier == 1 && dw.k_h == 3 && dw.k_w == 3 &&
              dw.dil_h == 1 && dw.dil_w == 1 && dw.stride_h == dw.stride_w && pc.in_xor == 0 && pc.w_zp == 0 &&
              Is1x1S1(pc) && pc.input == dw.output &&
              private_tensor(d.ops[D.op_index].outputs[0], P.op_index);
    if (ok && E) {
      const bh_conv_params& ec = E->conv;
      ok = ec.in_xor == 0 && ec.w_zp == 0 && Is1x1S1(ec) && !ec.residual && ec.output == dw.input &&
           private_tensor(d.ops[E->op_index].outputs[0], D.op_index);
    }
    if (ok && pc.residual) {
      const void* x = E ? E->conv.input : dw.input;
      ok = pc.residual == x;
    }
    bh_irb_params q{};
    if (ok) {
      const bh_conv_params* ec = E ? &E->conv : nullptr;
      q.batch = dw.batch;
      q.in_h = dw.in_h; q.in_w = dw.in_w;
      q.in_c = ec ? ec->in_c : dw.in_c;
      q.exp_c = dw.in_c;
      q.out_h = dw.out_h; q.out_w = dw.out_w; q.out_c = pc.out_c;
      q.stride = dw.stride_h; q.pad_h = dw.pad_h; q.pad_w = dw.pad_w;
      q.has_expand = ec ? 1 : 0;
      if (ec) {
        q.exp_w = ec->weights; q.exp_k_pad = ec->k_pad;
        q.exp_bias_eff = ec->bias_eff; q.exp_mult = ec->mult; q.exp_shift = ec->shift;
        q.x_zp = ec->in_zp;
        q.e_zp = ec->out_zp; q.e_act_min = ec->act_min; q.e_act_max = ec->act_max;
      }
      q.dw_w = dw.weights; q.dw_bias = dw.bias; q.dw_mult = dw.mult; q.dw_shift = dw.shift;
      if (!ec) q.e_zp = dw.in_zp;
      q.d_zp = dw.out_zp; q.d_act_min = dw.act_min; q.d_act_max = dw.act_max;
      q.proj_w = pc.weights; q.proj_k_pad = pc.k_pad;
      q.proj_bias_eff = pc.bias_eff; q.proj_mult = pc.mult; q.proj_shift = pc.shift;
      q.p_zp = pc.out_zp; q.p_act_min = pc.act_min; q.p_act_max = pc.act_max;
      q.has_residual = pc.residual ? 1 : 0;
      q.add_p_off = pc.add_y_off; q.add_x_off = pc.add_r_off; q.add_o_off = pc.add_o_off;
      q.add_left_shift = pc.add_left_shift;
      q.add_p_mult = pc.add_y_mult; q.add_p_shift = pc.add_y_shift;
      q.add_x_mult = pc.add_r_mult; q.add_x_shift = pc.add_r_shift;
      q.add_o_mult = pc.add_o_mult; q.add_o_shift = pc.add_o_shift;
      q.add_act_min = pc.add_act_min; q.add_act_max = pc.add_act_max;
      q.requant_fast = (ec && ec->requant_fast ? 1 : 0) | (dw.requant_fast ? 2 : 0) | (pc.requant_fast ? 4 : 0);
      q.input = ec ? ec->input : dw.input;
      q.output = pc.output;
      // Tile edge: measured on this device when possible (each feasible
      // tile, and the unfused launches, timed on the real buffers; the
      // winner is cached per block geometry), else the static model.
      int tile = 0;
      bh_irb_params kq = q;
      if (tune_batch_ > 0) kq.batch = tune_batch_;  // a job-batch variant reuses its anchor's choice
      const std::string key = IrbKey(ordinal_, kq);
      bool cached = false;
      if (autotune_) {
        std::lock_guard<std::mutex> lk(g_tune_mu);
        LoadTuneFileLocked();
        auto it = g_tune.find(key);
        if (it != g_tune.end()) {
          tile = it->second;
          cached = true;
        }
      }
      if (!cached) {
        double best_model = 1e300, best_us = 1e300;
        int model_tile = 0;
        bool measured = autotune_;
        if (measured) {
          std::vector<const Launch*> unfused;
          if (E) unfused.push_back(E);
          unfused.push_back(&D);
          unfused.push_back(&P);
          const double u = TimeLaunches(unfused, 10);
          measured = u > 0;
          best_us = u * 0.98;  // fusion must win by > 2% to be taken
        }
        for (int t = 8; t >= 1; --t) {
          q.tile_h = q.tile_w = t;
          const size_t lds = bh_irb_lds_bytes(&q);
          if (lds == 0) continue;
          const double est = IrbModelCost(q, t, lds);
          if (est < best_model * 0.97) {
            best_model = est;
            model_tile = t;
          }
          if (measured) {
            Launch F;
            F.kind = Launch::kIrb;
            F.irb = q;
            const double us = TimeLaunches({&F}, 10);
            if (us > 0 && us < best_us) {
              best_us = us;
              tile = t;
            }
          }
        }
        if (!measured) tile = model_tile;
        if (autotune_ && measured) {
          std::lock_guard<std::mutex> lk(g_tune_mu);
          if (!g_tune.count(key)) AppendTuneFileLocked(key, tile);
          g_tune[key] = tile;
        }
      }
      q.tile_h = q.tile_w = tile;
      ok = tile > 0 && bh_irb_lds_bytes(&q) > 0;
    }
    if (!ok) {
      out.push_back(L[i]);
      continue;
    }
    Launch F;
    F.kind = Launch::kIrb;
    F.op_index = E ? E->op_index : D.op_index;
    F.out_tensor = P.out_tensor;
    F.irb = q;
    F.kernel = "irb_kernel";
    // algorithmic bytes: block input + block output + all filters/tables
    const double x_bytes = static_cast<double>(q.batch) * q.in_h * q.in_w * q.in_c;
    const double y_bytes = static_cast<double>(q.batch) * q.out_h * q.out_w * q.out_c;
    F.alg_bytes = x_bytes + y_bytes + 12.0 * (q.exp_c + q.out_c) + 9.0 * q.exp_c +
                  static_cast<double>(q.exp_c) * q.out_c + (E ? static_cast<double>(q.exp_c) * q.in_c + 12.0 * q.exp_c : 0);
    F.alg_ops = (E ? E->alg_ops : 0) + D.alg_ops + P.alg_ops;
    out.push_back(F);
    // intermediates now live only in LDS; a later view of one re-lowers
    sg->fused_tensors.insert(d.ops[D.op_index].outputs[0]);
    if (E) sg->fused_tensors.insert(d.ops[E->op_index].outputs[0]);
    i = j + 1;  // consumed [E] D P
  }
  sg->launches.swap(out);
}

// Rewrites dw3x3 -> conv1x1 [+fused ADD] [-> conv1x1] launch runs into one
// bh_chain_i8 launch (a block's depthwise + project and the next block's
// expand) when the depthwise output is private to the first conv.  The
// first conv's output is stored only when something besides the second conv
// reads it (the next block's residual, a subgraph output).  Taken per run
// geometry by on-device timing against the unfused launches, as FuseBlocks.
// The tile form's constant block (bh_chain_tile_pack): built on the device
// from the chain's filter / table pointers, owned by the subgraph.
bool HipModelExecutor::PackChainTile(bh_chain_params* q, PreparedSubgraph* sg) {
  const size_t nb = bh_chain_tile_blob_bytes(q);
  if (nb == 0 || ordinal_ < 0) return false;
  auto blob = std::make_shared<DeviceBlob>(ordinal_, nb);
  if (!blob->ok() || bh_chain_tile_pack(q, blob->ptr(), stream_) != 0 || bh_stream_sync(stream_) != 0) return false;
  q->tile_blob = blob->ptr();
  sg->consts.push_back(blob);
  return true;
}

void HipModelExecutor::FuseChains(const HipModel& model, PreparedSubgraph* sg) {
  const TflModel& d = model.desc();
  auto private_tensor = [&](int t, int only_consumer) {
    if (t < 0 || consumers_[t].size() != 1 || consumers_[t][0] != only_consumer) return false;
    if (sg->no_fuse.count(t) || sg->extra_d2h.count(t)) return false;
    if (std::find(sg->outputs.begin(), sg->outputs.end(), t) != sg->outputs.end()) return false;
    return std::find(d.outputs.begin(), d.outputs.end(), t) == d.outputs.end();
  };
  std::vector<Launch> out;
  const auto& L = sg->launches;
  for (size_t i = 0; i < L.size(); ++i) {
    const bool head = L[i].kind == Launch::kDwConv && i + 1 < L.size() && L[i + 1].kind == Launch::kConv &&
                      L[i + 1].conv.input == L[i].dw.output && !L[i].dw.out_table &&
                      private_tensor(L[i].out_tensor, L[i + 1].op_index);
    if (!head) {
      out.push_back(L[i]);
      continue;
    }
    const Launch& D = L[i];
    const Launch& P1 = L[i + 1];
    const Launch* P2 = nullptr;
    if (i + 2 < L.size() && L[i + 2].kind == Launch::kConv && L[i + 2].conv.input == P1.conv.output &&
        Is1x1S1(L[i + 2].conv) && !L[i + 2].conv.residual)
      P2 = &L[i + 2];
    bh_chain_params c{};
    c.dw = D.dw;
    c.pw1 = P1.conv;
    c.px_blocks = 4;
    // the two candidate forms: with the second conv, and without it
    bh_chain_params c3 = c, c2 = c;
    bool ok3 = false;
    if (P2) {
      c3.has_pw2 = 1;
      c3.pw2 = P2->conv;
      if (private_tensor(P1.out_tensor, P2->op_index)) c3.pw1.output = nullptr;
      ok3 = bh_chain_lds_bytes(&c3) > 0;
    }
    const bool ok2 = bh_chain_lds_bytes(&c2) > 0;
    if (!ok2 && !ok3) {
      out.push_back(L[i]);
      continue;
    }
    // choice: 0 = unfused, 1/2/4 = px_blocks of the 3-launch form, 11/12/14
    // = px_blocks of the 2-launch form (the second conv stays a launch),
    // +100 = 16 waves per workgroup, +200 = persistent form, +300 = 8 waves
    char key[256];
    std::snprintf(key, sizeof(key), "ch%d:%d:%d:%dx%dx%d:s%dd%d:%d:%d:%d:%d:f%d%d%d%d", kChainTuneVersion, ordinal_,
                  tune_batch_ > 0 ? tune_batch_ : D.dw.batch, D.dw.in_h,
                  D.dw.in_w, D.dw.in_c, D.dw.stride_h, D.dw.dil_h, P1.conv.out_c, P1.conv.residual ? 1 : 0,
                  ok3 ? c3.pw2.out_c : 0, ok3 && c3.pw1.output ? 1 : 0, no_tile_chain_, no_deep_chain_,
                  no_split_chain_, no_stage_chain_);
    int choice = force_chain_ ? (ok3 ? 4 : 14) : -1;
    if (force_stage_chain_ && ok3) {
      bh_chain_params q = c3;
      q.px_blocks = 1;
      q.waves = 8;
      q.c_split = 2;
      q.stage = 1;
      if (bh_chain_lds_bytes(&q) > 0) choice = kStageChoice + 2 * 100 + 1 * 10 + 1;  // 1 block, 8 waves, 2 slices
      q.stage = 2;
      if (bh_chain_lds_bytes(&q) > 0) choice += 1000;  // ... with loader waves
    }
    if (force_tile_chain_) {
      bh_chain_params q = ok3 ? c3 : c2;
      q.tile = 1;
      if (bh_chain_lds_bytes(&q) > 0) choice += 400;
    }
    if (force_deep_chain_) {
      bh_chain_params q = ok3 ? c3 : c2;
      q.px_blocks = 1;
      q.deep = 1;
      choice = bh_chain_lds_bytes(&q) > 0 ? (ok3 ? 1001 : 1011) : (ok3 ? 4 : 14);
    }
    if (autotune_ && choice < 0) {
      std::lock_guard<std::mutex> lk(g_tune_mu);
      LoadTuneFileLocked();
      auto it = g_tune.find(key);
      if (it != g_tune.end()) choice = it->second;
    }
    if (choice < 0) {
      choice = 0;
      bool measured = autotune_;
      if (measured) {
        std::vector<const Launch*> base = {&D, &P1};
        if (ok3) base.push_back(P2);
        const double u = TimeLaunches(base, 10);
        const double u_p2 = ok3 ? TimeLaunches({P2}, 10) : 0.0;
        measured = u > 0 && u_p2 >= 0;
        // BAND_HIP_TUNE_LOG=1: every measured form of every chain on stderr
        static const bool tune_log = std::getenv("BAND_HIP_TUNE_LOG") != nullptr;
        if (tune_log) std::fprintf(stderr, "[chain-tune] %s unfused %.2f (pw2 %.2f)\n", key, u, u_p2);
        double best = u * 0.98;  // fusion must win by > 2% to be taken
        // (px_blocks, waves): 64 / 32 / 16 pixels per 4-wave workgroup, or
        // 16 pixels over 16 waves (few-pixel, many-channel layers)
        // {px_blocks, waves, persist}: the last is the persistent form
        // (filters in LDS, 64-pixel blocks walked by one wave of workgroups)
        // {.., tile}: the 2-D tile form (8 x 8 pixels, one LDS-DMA burst)
        // {.., deep}: the deep-issue raster forms
        // {.., tile 3 / 4}: runs of 2 / 4 tiles per workgroup, the constant
        // block staged once per run
        // {.., split}: the second 1x1's channel tiles over 2..4 workgroups
        // per pixel block (3-launch form only; BAND_HIP_FUSION=nosplit: none)
        const int forms[19][6] = {
            {4, 4, 0, 0, 0, 0}, {2, 4, 0, 0, 0, 0}, {1, 4, 0, 0, 0, 0}, {1, 8, 0, 0, 0, 0},
            {1, 16, 0, 0, 0, 0}, {4, 4, 1, 0, 0, 0}, {4, 4, 0, 1, 0, 0}, {4, 4, 0, 3, 0, 0},
            {4, 4, 0, 4, 0, 0}, {2, 4, 0, 0, 1, 0}, {1, 4, 0, 0, 1, 0}, {1, 8, 0, 0, 1, 0},
            {1, 4, 0, 0, 0, 2}, {1, 8, 0, 0, 0, 2}, {2, 4, 0, 0, 0, 2}, {1, 16, 0, 0, 0, 2},
            {1, 4, 0, 0, 0, 3}, {1, 8, 0, 0, 0, 3}, {1, 4, 0, 0, 0, 4}};
        // the stage forms (3-launch only): {px_blocks, waves, phase-C slices,
        // stage (2: loader waves)}
        const int stage_forms[16][4] = {{1, 4, 0, 1}, {1, 8, 0, 1}, {2, 4, 0, 1}, {2, 8, 0, 1}, {1, 8, 2, 1},
                                        {2, 8, 2, 1}, {1, 8, 4, 1}, {1, 8, 8, 1}, {1, 8, 0, 2}, {2, 8, 0, 2},
                                        {1, 4, 0, 2}, {1, 8, 2, 2}, {2, 8, 2, 2}, {1, 8, 3, 2}, {1, 8, 4, 2},
                                        {1, 8, 8, 2}};
        for (const auto& sf : stage_forms) {
          if (no_stage_chain_ || !ok3 || !measured) break;
          bh_chain_params q = c3;
          q.px_blocks = sf[0];
          q.waves = sf[1];
          q.c_split = sf[2];
          q.stage = sf[3];
          if (bh_chain_lds_bytes(&q) == 0 || !PackChainTile(&q, sg)) continue;
          Launch F;
          F.kind = Launch::kChain;
          F.chain = q;
          const double us = TimeLaunches({&F}, 10);
          if (tune_log)
            std::fprintf(stderr, "[chain-tune]   form3 stage%d px%d w%d split%d: %.2f\n", sf[3], sf[0], sf[1], sf[2],
                         us);
          if (us > 0 && us < best) {
            best = us;
            choice = kStageChoice + (sf[3] - 1) * 1000 + sf[2] * 100 + sf[0] * 10 + (sf[1] == 8 ? 1 : 0);
          }
        }
        for (const auto& pw : forms) {
          if (pw[3] && no_tile_chain_) continue;
          if (pw[4] && no_deep_chain_) continue;
          if (pw[5] && no_split_chain_) continue;
          for (int form = 0; form < 2 && measured; ++form) {
            bh_chain_params q = form == 0 ? c3 : c2;
            if (form == 0 ? !ok3 : !ok2) continue;
            q.px_blocks = pw[0];
            q.waves = pw[1];
            q.persist = pw[2];
            q.tile = pw[3];
            q.deep = pw[4];
            q.c_split = pw[5];
            if (pw[5] > 1 && form != 0) continue;
            if (bh_chain_lds_bytes(&q) == 0) continue;
            if (q.tile && !PackChainTile(&q, sg)) continue;
            Launch F;
            F.kind = Launch::kChain;
            F.chain = q;
            const double us = TimeLaunches({&F}, 10);
            const double total = us + (form == 1 && ok3 ? u_p2 : 0.0);
            if (tune_log)
              std::fprintf(stderr, "[chain-tune]   form%d px%d w%d persist%d tile%d deep%d split%d: %.2f\n", 3 - form,
                           pw[0], pw[1], pw[2], pw[3], pw[4], pw[5], total);
            if (us > 0 && total < best) {
              best = total;
              choice = (form == 0 ? 0 : 10) + pw[0] + (pw[1] == 16 ? 100 : 0) + (pw[1] == 8 ? 300 : 0) +
                       (pw[2] ? 200 : 0) + (pw[3] == 1 ? 400 : 0) + (pw[3] == 3 ? 600 : 0) +
                       (pw[3] == 4 ? 700 : 0) + (pw[4] ? 1000 : 0) + (pw[5] > 1 ? 2000 * (pw[5] - 1) : 0);
            }
          }
        }
      }
      if (!measured) choice = ok3 ? 4 : 14;  // no device timing: the 3-launch form when it applies
      if (measured && std::getenv("BAND_HIP_TUNE_LOG")) std::fprintf(stderr, "[chain-tune] %s -> %d\n", key, choice);
      if (autotune_ && measured) {
        std::lock_guard<std::mutex> lk(g_tune_mu);
        if (!g_tune.count(key)) AppendTuneFileLocked(key, choice);
        g_tune[key] = choice;
      }
    }
    // choice: px_blocks, +10 for the 2-launch form, +100 for 16 waves,
    // +200 for the persistent form, +300 for 8 waves, +400 for the tile
    // form, +600 / +700 for runs of 2 / 4 tiles, +1000 for the deep-issue
    // form, +2000 x (s - 1) for the s-way phase-C split; the stage form is
    // kStageChoice + 1000 x (stage - 1) + 100 x slices + 10 x px_blocks + (8 waves)
    int stage = choice >= kStageChoice ? 1 : 0;
    int stage_split = 0, stage_px = 1, stage_waves = 4;
    if (stage) {
      int c = choice - kStageChoice;
      stage = 1 + c / 1000;
      c %= 1000;
      stage_split = c / 100;
      stage_px = (c / 10) % 10;
      stage_waves = c % 10 ? 8 : 4;
      choice = 1;  // a 3-launch form
    }
    const int c_split = choice >= 2000 ? choice / 2000 + 1 : 0;
    choice %= 2000;
    const int deep = choice >= 1000 ? 1 : 0;
    choice %= 1000;
    const bool three = choice > 0 && choice % 100 < 10;
    if (choice == 0 || (three && !ok3) || (!three && !ok2)) {
      out.push_back(L[i]);
      continue;
    }
    Launch F;
    F.kind = Launch::kChain;
    F.op_index = D.op_index;
    F.chain = three ? c3 : c2;
    F.chain.px_blocks = choice % 10;
    F.chain.waves = choice >= 300 && choice < 400 ? 8 : (choice >= 100 && choice < 200 ? 16 : 4);
    F.chain.persist = choice >= 200 && choice < 300 ? 1 : 0;
    F.chain.tile = choice >= 400 && choice < 800 ? choice / 100 - 3 : 0;
    F.chain.deep = deep;
    F.chain.c_split = c_split;
    if (stage) {
      F.chain.px_blocks = stage_px;
      F.chain.waves = stage_waves;
      F.chain.c_split = stage_split;
      F.chain.stage = stage;
    }
    // a choice read from a tune file written by another kernel tree may name
    // a form these parameters do not admit: keep the unfused launches then
    if (bh_chain_lds_bytes(&F.chain) == 0 || ((F.chain.tile || F.chain.stage) && !PackChainTile(&F.chain, sg))) {
      out.push_back(L[i]);
      continue;
    }
    F.out_tensor = three ? P2->out_tensor : P1.out_tensor;
    F.kernel = F.chain.stage ? "chain_stage_kernel" : (F.chain.tile ? "chain_tile_kernel" : "chain_kernel");
    const bh_dwconv_params& dw = F.chain.dw;
    const bh_conv_params& a = F.chain.pw1;
    const double px = static_cast<double>(dw.batch) * dw.out_h * dw.out_w;
    F.alg_bytes = static_cast<double>(dw.batch) * dw.in_h * dw.in_w * dw.in_c + 9.0 * dw.out_c + 28.0 * dw.out_c +
                  (a.residual ? px * a.out_c : 0.0) + (a.output ? px * a.out_c : 0.0) +
                  static_cast<double>(a.out_c) * a.in_c + 12.0 * a.out_c;
    F.alg_ops = D.alg_ops + P1.alg_ops;
    if (three) {
      const bh_conv_params& b = F.chain.pw2;
      F.alg_bytes += px * b.out_c + static_cast<double>(b.out_c) * b.in_c + 12.0 * b.out_c;
      F.alg_ops += P2->alg_ops;
      if (!a.output) sg->fused_tensors.insert(P1.out_tensor);
    }
    out.push_back(F);
    sg->fused_tensors.insert(D.out_tensor);
    i += three ? 2 : 1;
  }
  sg->launches.swap(out);
}

namespace {
void** OutSlot(Launch& l) {
  switch (l.kind) {
    case Launch::kChain: return l.chain.has_pw2 ? &l.chain.pw2.output : &l.chain.pw1.output;
    case Launch::kConv: return &l.conv.output;
    case Launch::kDwConv: return &l.dw.output;
    case Launch::kFc: return &l.fc.output;
    case Launch::kEltwise: return &l.elt.out;
    case Launch::kPool: return &l.pool.output;
    case Launch::kIrb: return &l.irb.output;
    case Launch::kLutU8: return &l.dst;
    default: return nullptr;
  }
}
const void** TableSlot(Launch& l) {
  switch (l.kind) {
    case Launch::kConv: return l.conv.residual ? nullptr : &l.conv.out_table;  // + ADD epilogue: keep apart
    case Launch::kDwConv: return &l.dw.out_table;
    case Launch::kFc: return &l.fc.out_table;
    default: return nullptr;
  }
}
}  // namespace

void HipModelExecutor::FuseGlue(const HipModel& model, PreparedSubgraph* sg) {
  const TflModel& d = model.desc();
  auto in_outputs = [&](int t) {
    return std::find(sg->outputs.begin(), sg->outputs.end(), t) != sg->outputs.end() ||
           std::find(d.outputs.begin(), d.outputs.end(), t) != d.outputs.end();
  };
  // t reaches op `to` through RESHAPE / SQUEEZE aliases only, every tensor on
  // the way read by nothing else and needed by nobody outside; collects them
  auto private_chain = [&](int t, int to, std::vector<int>* chain) {
    while (t >= 0) {
      if (consumers_[t].size() != 1 || in_outputs(t) || sg->no_fuse.count(t) || sg->extra_d2h.count(t)) return false;
      chain->push_back(t);
      const int c = consumers_[t][0];
      if (c == to) return true;
      const TflOperator& op = d.ops[c];
      if ((op.builtin != kTflReshape && op.builtin != kTflSqueeze) ||
          !std::binary_search(sg->ops.begin(), sg->ops.end(), c))
        return false;
      t = op.outputs[0];
    }
    return false;
  };
  auto producer_of = [&](size_t i, const void* ptr) -> int {
    for (size_t j = i; j-- > 0;) {
      void** o = OutSlot(sg->launches[j]);
      if (o && *o == ptr) return static_cast<int>(j);
    }
    return -1;
  };
  std::vector<bool> dead(sg->launches.size(), false);
  // (1) byte tables into the producer's epilogue; a CONCATENATION without
  // rescale tables takes the table as every input's copy table (and may
  // hand it on to its producers in (2))
  for (size_t i = 0; i < sg->launches.size(); ++i) {
    Launch& L = sg->launches[i];
    if (L.kind != Launch::kLutU8) continue;
    const int j = producer_of(i, L.src);
    if (j < 0 || dead[j]) continue;
    Launch& P = sg->launches[j];
    std::vector<int> chain;
    if (P.kind == Launch::kConcat) {
      bool plain = P.concat.output == L.src;
      for (int k = 0; k < P.concat.n_inputs && plain; ++k) plain = P.concat.table[k] == nullptr;
      if (!plain || !private_chain(P.out_tensor, L.op_index, &chain)) continue;
      for (int k = 0; k < P.concat.n_inputs; ++k) P.concat.table[k] = L.table;
      P.concat.output = L.dst;
    } else {
      const void** ts = TableSlot(P);
      if (!ts || *ts || !private_chain(P.out_tensor, L.op_index, &chain)) continue;
      *ts = L.table;
      *OutSlot(P) = L.dst;
    }
    P.out_tensor = L.out_tensor;
    P.alg_bytes += 0;  // same bytes: the table gather happens on the stored value
    for (int t : chain) sg->fused_tensors.insert(t);
    sg->fused_ops.insert(L.op_index);
    dead[i] = true;
  }
  // (2) CONCATENATION whose inputs are slices of the output: contiguous
  // ones (outer size 1) from any producer; per-image slices (outer = batch
  // > 1, a detector's per-anchor concat) from convs, which store each image
  // at the concat's row stride (bh_conv_params.out_img_stride); an input
  // copy table moves into the producer's epilogue table
  for (size_t i = 0; i < sg->launches.size(); ++i) {
    Launch& C = sg->launches[i];
    if (C.kind != Launch::kConcat) continue;
    const bool strided = C.concat.outer != 1;
    if (strided && device_flag_ != DeviceFlag::kGPU) continue;  // (the host conv stores dense images)
    long total_row = 0;
    for (int k = 0; k < C.concat.n_inputs; ++k) total_row += C.concat.row[k];
    bool ok = true;
    std::vector<int> prod(C.concat.n_inputs, -1);
    std::vector<int> chain;
    for (int k = 0; k < C.concat.n_inputs && ok; ++k) {
      const int j = producer_of(i, C.concat.input[k]);
      ok = j >= 0 && !dead[j] && OutSlot(sg->launches[j]) &&
           private_chain(sg->launches[j].out_tensor, C.op_index, &chain);
      if (ok && C.concat.table[k]) {
        const void** ts = TableSlot(sg->launches[j]);
        ok = ts && *ts == nullptr;
      }
      if (ok && strided) {
        const Launch& P = sg->launches[j];
        ok = P.kind == Launch::kConv && P.conv.out_img_stride == 0 && P.conv.batch == C.concat.outer &&
             static_cast<long>(P.conv.out_h) * P.conv.out_w * P.conv.out_c == C.concat.row[k];
      }
      if (ok) prod[k] = j;
      for (int kk = 0; kk < k && ok; ++kk) ok = prod[kk] != j;  // one producer per slice
    }
    if (!ok) continue;
    long off = 0;
    for (int k = 0; k < C.concat.n_inputs; ++k) {
      Launch& P = sg->launches[prod[k]];
      *OutSlot(P) = static_cast<char*>(C.concat.output) + off;
      if (C.concat.table[k]) *TableSlot(P) = C.concat.table[k];
      if (strided) P.conv.out_img_stride = total_row;
      off += C.concat.row[k];
    }
    for (int t : chain) sg->fused_tensors.insert(t);
    sg->fused_ops.insert(C.op_index);
    dead[i] = true;
  }
  std::vector<Launch> out;
  for (size_t i = 0; i < sg->launches.size(); ++i)
    if (!dead[i]) out.push_back(sg->launches[i]);
  sg->launches.swap(out);
}

// Folds `conv -> ADD/SUB(conv_out, residual)` into the conv epilogue when the
// conv output has no other reader and nobody needs it materialised.  The
// epilogue reproduces both TFLite ops exactly (conv requant + clamp to the
// conv's 8-bit output, then add.cc's arithmetic), so the result is
// bit-identical to running the two ops.

}  // namespace hip
}  // namespace band
