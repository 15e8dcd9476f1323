// The benchmark tool (band/tool/benchmark.cc, benchmark_config.h) over the
// native engine, reachable through BandxBenchmarkRun(config_json).
//
// Config: the reference's JSON (band/test/data/benchmark_config.json).
// Execution modes:
//   periodic  one client thread per model, RequestSync(batch) every period_ms
//   stream    back-to-back RequestSync of every model's batch
//             ("stream_clients": N concurrent stream loops, default 1 as in
//             the reference)
//   workload  open-loop Poisson arrivals, "request_rate" (req/s) per model,
//             "seed" (the reference leaves this mode unimplemented,
//             band/tool/benchmark.cc:495)
// Inputs are filled once per model as the reference does (default-seeded
// mt19937; int8 U{-127..127}, uint8 U{0..254}, f32 U(-0.5,0.5)).
// Latency of a job = end_time - enqueue_time from the planner's record.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "band_c_api.h"
#include "engine/engine.h"
#include "engine/json.h"
#include "engine/logger.h"
#include "engine/time.h"

namespace band {
namespace tool {
namespace {

struct ModelConfig {
  std::string path;
  int batch_size = 1;
  int period_ms = 0;
  int worker_id = -1;
  int slo_us = -1;
  float slo_scale = -1.f;
  double request_rate = 0;  // workload mode
};

struct ModelContext {
  Model model;
  ModelConfig config;
  std::vector<std::unique_ptr<Tensor>> inputs;  // filled once
  std::vector<int> input_indices, output_indices;
};

struct Sample {
  int model;
  int worker;
  JobStatus status;
  int64_t enqueue, invoke, end;
  int64_t slo;
};

template <typename T, typename D>
void Fill(void* p, size_t n, D dist) {
  std::mt19937 rng;  // default seed, as band/tool/benchmark.cc:279-287
  T* t = static_cast<T*>(p);
  for (size_t i = 0; i < n; ++i) t[i] = static_cast<T>(dist(rng));
}

void FillRandom(Tensor* t) {
  const size_t n = t->GetNumElements();
  switch (t->GetType()) {
    case DataType::kUInt8: Fill<uint8_t>(t->GetData(), n, std::uniform_int_distribution<int32_t>(0, 254)); break;
    case DataType::kInt8: Fill<int8_t>(t->GetData(), n, std::uniform_int_distribution<int32_t>(-127, 127)); break;
    case DataType::kInt16: Fill<int16_t>(t->GetData(), n, std::uniform_int_distribution<int16_t>(0, 99)); break;
    case DataType::kInt32: Fill<int32_t>(t->GetData(), n, std::uniform_int_distribution<int32_t>(0, 99)); break;
    case DataType::kInt64: Fill<int64_t>(t->GetData(), n, std::uniform_int_distribution<int64_t>(0, 99)); break;
    case DataType::kFloat32: Fill<float>(t->GetData(), n, std::uniform_real_distribution<float>(-0.5f, 0.5f)); break;
    case DataType::kFloat64: Fill<double>(t->GetData(), n, std::uniform_real_distribution<double>(-0.5, 0.5)); break;
    default: break;
  }
}

json::Value Percentiles(std::vector<int64_t> v) {
  json::Value o = json::Value::Object();
  if (v.empty()) return o;
  std::sort(v.begin(), v.end());
  double sum = 0;
  for (int64_t x : v) sum += static_cast<double>(x);
  auto pct = [&](double p) {
    size_t i = static_cast<size_t>(p / 100.0 * (v.size() - 1) + 0.5);
    return static_cast<double>(v[std::min(i, v.size() - 1)]);
  };
  o["mean"] = json::Value::Number(sum / v.size());
  o["p50"] = json::Value::Number(pct(50));
  o["p90"] = json::Value::Number(pct(90));
  o["p99"] = json::Value::Number(pct(99));
  o["max"] = json::Value::Number(static_cast<double>(v.back()));
  return o;
}

class Benchmark {
 public:
  absl::Status Parse(const std::string& text);
  absl::Status Initialize();
  absl::Status Run();
  std::string Report() const;

 private:
  RequestOption Option(const ModelConfig& c) const;
  void Record(const std::vector<JobId>& ids, std::vector<Sample>* out);
  void RunPeriodic();
  void RunStream();
  void RunWorkload();

  RuntimeConfig runtime_;
  std::vector<ModelConfig> models_;
  std::string mode_;
  int running_time_ms_ = 60000;
  int warmup_ms_ = 0;
  int stream_clients_ = 1;
  uint64_t seed_ = 5489;
  std::unique_ptr<Engine> engine_;
  std::vector<std::unique_ptr<ModelContext>> contexts_;
  std::mutex samples_mu_;
  std::vector<Sample> samples_;
  int64_t window_begin_ = 0, window_end_ = 0;
  std::atomic<int64_t> dropped_{0};
};

absl::Status Benchmark::Parse(const std::string& text) {
  json::Value root;
  std::string err;
  if (!json::Parse(text, &root, &err)) return absl::InvalidArgumentError("config: " + err);
  const json::Value* mode = root.find("execution_mode");
  const json::Value* models = root.find("models");
  if (!mode || !mode->is_string() || !models || !models->is_array() || models->size() == 0)
    return absl::InvalidArgumentError("config needs execution_mode and models");
  mode_ = mode->as_string();
  if (mode_ != "periodic" && mode_ != "stream" && mode_ != "workload")
    return absl::InvalidArgumentError("execution mode " + mode_ + " is not valid");
  auto num = [&](const json::Value& o, const char* k, double d) {
    const json::Value* v = o.find(k);
    return v && v->is_number() ? v->as_number() : d;
  };
  auto str = [&](const json::Value& o, const char* k, const std::string& d) {
    const json::Value* v = o.find(k);
    return v && v->is_string() ? v->as_string() : d;
  };
  running_time_ms_ = static_cast<int>(num(root, "running_time_ms", 60000));
  if (running_time_ms_ <= 0) return absl::InvalidArgumentError("running_time_ms must be > 0");
  warmup_ms_ = static_cast<int>(num(root, "warmup_ms", 0));
  stream_clients_ = std::max(1, static_cast<int>(num(root, "stream_clients", 1)));
  seed_ = static_cast<uint64_t>(num(root, "seed", 5489));
  for (size_t i = 0; i < models->size(); ++i) {
    const json::Value& m = models->at(i);
    ModelConfig c;
    c.path = str(m, "graph", "");
    if (c.path.empty()) return absl::InvalidArgumentError("model config without `graph`");
    c.batch_size = std::max(1, static_cast<int>(num(m, "batch_size", 1)));
    c.period_ms = static_cast<int>(num(m, "period_ms", 0));
    if (mode_ == "periodic" && c.period_ms <= 0) return absl::InvalidArgumentError("periodic mode needs period_ms > 0");
    c.worker_id = static_cast<int>(num(m, "worker_id", -1));
    c.slo_us = static_cast<int>(num(m, "slo_us", -1));
    c.slo_scale = static_cast<float>(num(m, "slo_scale", -1));
    c.request_rate = num(m, "request_rate", 0);
    if (mode_ == "workload" && c.request_rate <= 0)
      return absl::InvalidArgumentError("workload mode needs request_rate > 0");
    models_.push_back(c);
  }

  // runtime config (band/tool/benchmark.cc:166-266)
  RuntimeConfig& r = runtime_;
  r.profile_config.num_warmups = static_cast<int>(num(root, "profile_warmup_runs", 1));
  r.profile_config.num_runs = static_cast<int>(num(root, "profile_num_runs", 1));
  r.profile_config.smoothing_factor = static_cast<float>(num(root, "profile_smoothing_factor", 0.1));
  r.profile_config.profile_data_path = str(root, "profile_data_path", "");
  if (const json::Value* on = root.find("profile_online")) r.profile_config.online = on->as_bool(true);
  r.planner_config.schedule_window_size = static_cast<int>(num(root, "schedule_window_size", INT32_MAX));
  const json::Value* scheds = root.find("schedulers");
  if (!scheds || !scheds->is_array() || scheds->size() == 0) return absl::InvalidArgumentError("config needs schedulers");
  for (size_t i = 0; i < scheds->size(); ++i)
    r.planner_config.schedulers.push_back(FromString<SchedulerType>(scheds->at(i).as_string()));
  r.planner_config.log_path = str(root, "log_path", "");
  if (const json::Value* ws = root.find("workers")) {
    r.worker_config.workers.clear();
    r.worker_config.cpu_masks.clear();
    r.worker_config.num_threads.clear();
    for (size_t i = 0; i < ws->size(); ++i) {
      const json::Value& w = ws->at(i);
      r.worker_config.workers.push_back(FromString<DeviceFlag>(str(w, "device", "CPU")));
      r.worker_config.num_threads.push_back(static_cast<int>(num(w, "num_threads", 1)));
      r.worker_config.cpu_masks.push_back(FromString<CPUMaskFlag>(str(w, "cpu_masks", "ALL")));
    }
  }
  r.worker_config.availability_check_interval_ms =
      static_cast<int>(num(root, "availability_check_interval_ms", 30000));
  r.worker_config.max_job_batch = static_cast<int>(num(root, "max_job_batch", 1));  // extension
  r.subgraph_config.minimum_subgraph_size = static_cast<int>(num(root, "minimum_subgraph_size", 7));
  r.subgraph_config.subgraph_preparation_type =
      FromString<SubgraphPreparationType>(str(root, "subgraph_preparation_type", "merge_unit_subgraph"));
  r.cpu_mask = FromString<CPUMaskFlag>(str(root, "cpu_masks", "ALL"));
  return absl::OkStatus();
}

RequestOption Benchmark::Option(const ModelConfig& c) const {
  RequestOption o = RequestOption::GetDefaultOption();
  if (c.worker_id >= 0) o.target_worker = c.worker_id;
  if (c.slo_us >= 0) o.slo_us = c.slo_us;
  if (c.slo_scale >= 0) o.slo_scale = c.slo_scale;
  return o;
}

absl::Status Benchmark::Initialize() {
  absl::Status s;
  engine_ = Engine::Create(runtime_, &s);
  if (!engine_) return s.ok() ? absl::InternalError("Failed to create engine") : s;
  for (ModelConfig& c : models_) {
    auto ctx = std::make_unique<ModelContext>();
    ctx->config = c;
    s = ctx->model.FromPath(BackendType::kTfLite, c.path.c_str());
    if (!s.ok()) return s;
    s = engine_->RegisterModel(&ctx->model);
    if (!s.ok()) return s;
    const ModelId id = ctx->model.GetId();
    ctx->input_indices = engine_->GetInputTensorIndices(id);
    ctx->output_indices = engine_->GetOutputTensorIndices(id);
    for (int t : ctx->input_indices) {
      Tensor* tensor = engine_->CreateTensor(id, t);
      if (!tensor) return absl::InternalError("cannot create input tensor");
      FillRandom(tensor);
      ctx->inputs.emplace_back(tensor);
    }
    // an SLO given as a scale of the worst profiled latency
    // (band/tool/benchmark.cc:333-355)
    if (ctx->config.slo_us <= 0 && ctx->config.slo_scale > 0.f) {
      int64_t worst = 0;
      for (WorkerId w = 0; w < static_cast<WorkerId>(engine_->GetNumWorkers()); ++w) {
        const SubgraphKey k = engine_->GetLargestSubgraphKey(id, w);
        if (k.IsValid()) worst = std::max(worst, engine_->GetProfiled(k));
      }
      if (worst > 0) ctx->config.slo_us = static_cast<int>(worst * ctx->config.slo_scale);
    }
    contexts_.push_back(std::move(ctx));
  }
  return absl::OkStatus();
}

void Benchmark::Record(const std::vector<JobId>& ids, std::vector<Sample>* out) {
  for (JobId id : ids) {
    Job j = engine_->GetFinishedJob(id);
    if (j.job_id != id) {
      dropped_++;
      continue;
    }
    int model = -1;
    for (size_t m = 0; m < contexts_.size(); ++m)
      if (contexts_[m]->model.GetId() == j.model_id) model = static_cast<int>(m);
    out->push_back({model, j.subgraph_key.GetWorkerId(), j.status, j.enqueue_time, j.invoke_time, j.end_time, j.slo_us});
  }
}

// per-request I/O tensors of one model's batch
struct BatchIO {
  std::vector<std::vector<std::unique_ptr<Tensor>>> in, out;
  std::vector<Tensors> in_ptrs, out_ptrs;
};

static void MakeBatch(Engine& e, ModelContext& ctx, BatchIO* b) {
  const ModelId id = ctx.model.GetId();
  for (int i = 0; i < ctx.config.batch_size; ++i) {
    b->in.emplace_back();
    b->out.emplace_back();
    Tensors ip, op;
    for (size_t k = 0; k < ctx.input_indices.size(); ++k) {
      b->in.back().emplace_back(e.CreateTensor(id, ctx.input_indices[k]));
      b->in.back().back()->CopyDataFrom(ctx.inputs[k].get());
      ip.push_back(b->in.back().back().get());
    }
    for (int t : ctx.output_indices) {
      b->out.back().emplace_back(e.CreateTensor(id, t));
      op.push_back(b->out.back().back().get());
    }
    b->in_ptrs.push_back(ip);
    b->out_ptrs.push_back(op);
  }
}

void Benchmark::RunPeriodic() {
  std::atomic<bool> stop{false};
  std::vector<std::thread> threads;
  for (auto& ctx_ptr : contexts_) {
    ModelContext* ctx = ctx_ptr.get();
    threads.emplace_back([this, ctx, &stop] {
      BatchIO b;
      MakeBatch(*engine_, *ctx, &b);
      std::vector<ModelId> ids(ctx->config.batch_size, ctx->model.GetId());
      std::vector<RequestOption> opts(ctx->config.batch_size, Option(ctx->config));
      std::vector<Sample> local;
      while (!stop) {
        const int64_t t0 = time::NowMicros();
        auto jobs = engine_->RequestAsync(ids, opts, b.in_ptrs);
        if (!jobs.ok()) break;
        engine_->Wait(jobs.value(), b.out_ptrs);
        Record(jobs.value(), &local);
        const int64_t spent = time::NowMicros() - t0;
        const int64_t period = static_cast<int64_t>(ctx->config.period_ms) * 1000;
        if (spent < period) time::SleepForMicros(period - spent);
      }
      std::lock_guard<std::mutex> l(samples_mu_);
      samples_.insert(samples_.end(), local.begin(), local.end());
    });
  }
  time::SleepForMicros(static_cast<int64_t>(warmup_ms_ + running_time_ms_) * 1000);
  stop = true;
  for (auto& t : threads) t.join();
}

void Benchmark::RunStream() {
  std::atomic<bool> stop{false};
  std::vector<std::thread> threads;
  for (int c = 0; c < stream_clients_; ++c) {
    threads.emplace_back([this, &stop] {
      std::vector<std::unique_ptr<BatchIO>> batches;
      std::vector<ModelId> ids;
      std::vector<RequestOption> opts;
      std::vector<Tensors> ins, outs;
      for (auto& ctx : contexts_) {
        batches.emplace_back(new BatchIO);
        MakeBatch(*engine_, *ctx, batches.back().get());
        for (int i = 0; i < ctx->config.batch_size; ++i) {
          ids.push_back(ctx->model.GetId());
          opts.push_back(Option(ctx->config));
          ins.push_back(batches.back()->in_ptrs[i]);
          outs.push_back(batches.back()->out_ptrs[i]);
        }
      }
      std::vector<Sample> local;
      while (!stop) {
        auto jobs = engine_->RequestAsync(ids, opts, ins);
        if (!jobs.ok()) break;
        engine_->Wait(jobs.value(), outs);
        Record(jobs.value(), &local);
      }
      std::lock_guard<std::mutex> l(samples_mu_);
      samples_.insert(samples_.end(), local.begin(), local.end());
    });
  }
  time::SleepForMicros(static_cast<int64_t>(warmup_ms_ + running_time_ms_) * 1000);
  stop = true;
  for (auto& t : threads) t.join();
}

// open-loop Poisson arrivals per model; a waiter thread collects jobs in
// submission order.  Outstanding requests per model are capped below the
// request ring size (128); arrivals beyond the cap are counted as dropped.
void Benchmark::RunWorkload() {
  struct Pending {
    JobId id;
    int model;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Pending> pending;
  std::vector<int> outstanding(contexts_.size(), 0);
  bool done = false;
  std::vector<std::unique_ptr<BatchIO>> io;
  for (auto& ctx : contexts_) {
    io.emplace_back(new BatchIO);
    MakeBatch(*engine_, *ctx, io.back().get());
  }
  std::thread waiter([&] {
    std::vector<Sample> local;
    while (true) {
      std::unique_lock<std::mutex> l(mu);
      cv.wait(l, [&] { return done || !pending.empty(); });
      if (pending.empty() && done) break;
      Pending p = pending.front();
      pending.pop_front();
      l.unlock();
      engine_->Wait(p.id, io[p.model]->out_ptrs[0]);
      Record({p.id}, &local);
      l.lock();
      outstanding[p.model]--;
    }
    std::lock_guard<std::mutex> l(samples_mu_);
    samples_.insert(samples_.end(), local.begin(), local.end());
  });
  std::mt19937_64 rng(seed_);
  const int64_t start = time::NowMicros();
  const int64_t stop_at = start + static_cast<int64_t>(warmup_ms_ + running_time_ms_) * 1000;
  std::vector<int64_t> next(contexts_.size());
  for (size_t m = 0; m < contexts_.size(); ++m)
    next[m] = start + static_cast<int64_t>(std::exponential_distribution<double>(contexts_[m]->config.request_rate)(rng) * 1e6);
  while (true) {
    size_t m = static_cast<size_t>(std::min_element(next.begin(), next.end()) - next.begin());
    if (next[m] >= stop_at) break;
    const int64_t now = time::NowMicros();
    if (next[m] > now) time::SleepForMicros(next[m] - now);
    bool admit;
    {
      std::lock_guard<std::mutex> l(mu);
      admit = outstanding[m] < 120;
      if (admit) outstanding[m]++;
    }
    if (admit) {
      auto id = engine_->RequestAsync(contexts_[m]->model.GetId(), Option(contexts_[m]->config), io[m]->in_ptrs[0]);
      std::lock_guard<std::mutex> l(mu);
      if (id.ok()) pending.push_back({id.value(), static_cast<int>(m)});
      else outstanding[m]--;
      cv.notify_one();
    } else {
      dropped_++;
    }
    next[m] += static_cast<int64_t>(std::exponential_distribution<double>(contexts_[m]->config.request_rate)(rng) * 1e6);
  }
  {
    std::lock_guard<std::mutex> l(mu);
    done = true;
  }
  cv.notify_one();
  waiter.join();
}

absl::Status Benchmark::Run() {
  window_begin_ = time::NowMicros() + static_cast<int64_t>(warmup_ms_) * 1000;
  if (mode_ == "periodic") RunPeriodic();
  else if (mode_ == "stream") RunStream();
  else RunWorkload();
  window_end_ = window_begin_ + static_cast<int64_t>(running_time_ms_) * 1000;
  return absl::OkStatus();
}

std::string Benchmark::Report() const {
  json::Value r = json::Value::Object();
  r["execution_mode"] = json::Value::String(mode_);
  r["running_time_ms"] = json::Value::Number(running_time_ms_);
  r["warmup_ms"] = json::Value::Number(warmup_ms_);
  json::Value sched = json::Value::Array();
  for (auto s : runtime_.planner_config.schedulers) sched.push_back(json::Value::String(ToString(s)));
  r["schedulers"] = sched;
  json::Value workers = json::Value::Array();
  for (WorkerId w = 0; w < static_cast<WorkerId>(engine_->GetNumWorkers()); ++w)
    workers.push_back(json::Value::String(ToString(engine_->GetWorkerDevice(w))));
  r["workers"] = workers;
  // jobs that ended inside the measurement window
  std::vector<int64_t> all_lat;
  std::vector<int> per_worker(engine_->GetNumWorkers(), 0);
  int64_t first_end = INT64_MAX, last_end = 0;
  size_t ok = 0, failed = 0, slo_viol = 0;
  json::Value per_model = json::Value::Array();
  std::vector<std::vector<int64_t>> lat(contexts_.size());
  std::vector<size_t> m_ok(contexts_.size()), m_slo_ok(contexts_.size()), m_fail(contexts_.size());
  for (const Sample& s : samples_) {
    if (s.end < window_begin_ || s.end > window_end_ || s.model < 0) continue;
    if (s.status == JobStatus::kSuccess) {
      ok++;
      m_ok[s.model]++;
      const int64_t l = s.end - s.enqueue;
      all_lat.push_back(l);
      lat[s.model].push_back(l);
      if (s.slo > 0 && l <= s.slo) m_slo_ok[s.model]++;
      if (s.worker >= 0 && s.worker < static_cast<int>(per_worker.size())) per_worker[s.worker]++;
      first_end = std::min(first_end, s.end);
      last_end = std::max(last_end, s.end);
    } else if (s.status == JobStatus::kSLOViolation) {
      slo_viol++;
      m_fail[s.model]++;
    } else {
      failed++;
      m_fail[s.model]++;
    }
  }
  const double window_s = (window_end_ - window_begin_) / 1e6;
  r["completed"] = json::Value::Number(static_cast<double>(ok));
  r["failed"] = json::Value::Number(static_cast<double>(failed));
  r["slo_violations"] = json::Value::Number(static_cast<double>(slo_viol));
  r["dropped"] = json::Value::Number(static_cast<double>(dropped_.load()));
  r["window_s"] = json::Value::Number(window_s);
  r["throughput_rps"] = json::Value::Number(window_s > 0 ? ok / window_s : 0);
  r["latency_us"] = Percentiles(all_lat);
  json::Value pw = json::Value::Array();
  for (int n : per_worker) pw.push_back(json::Value::Number(n));
  r["jobs_per_worker"] = pw;
  for (size_t m = 0; m < contexts_.size(); ++m) {
    json::Value o = json::Value::Object();
    o["graph"] = json::Value::String(contexts_[m]->config.path);
    o["batch_size"] = json::Value::Number(contexts_[m]->config.batch_size);
    o["slo_us"] = json::Value::Number(contexts_[m]->config.slo_us);
    o["completed"] = json::Value::Number(static_cast<double>(m_ok[m]));
    o["failed_or_dropped_by_slo"] = json::Value::Number(static_cast<double>(m_fail[m]));
    o["throughput_rps"] = json::Value::Number(window_s > 0 ? m_ok[m] / window_s : 0);
    o["latency_us"] = Percentiles(lat[m]);
    if (contexts_[m]->config.slo_us > 0) {
      const double n = static_cast<double>(m_ok[m] + m_fail[m]);
      o["slo_satisfactory_rate"] = json::Value::Number(n > 0 ? 100.0 * m_slo_ok[m] / n : 0);
    }
    per_model.push_back(o);
  }
  r["models"] = per_model;
  return r.Dump();
}

}  // namespace
}  // namespace tool
}  // namespace band

extern "C" size_t BandxBenchmarkRun(const char* config_json, char* out, size_t cap) {
  using band::tool::Benchmark;
  std::string result;
  size_t rc = 0;
  {
    Benchmark b;
    absl::Status s = config_json ? b.Parse(config_json) : absl::InvalidArgumentError("null config");
    if (s.ok()) s = b.Initialize();
    if (s.ok()) s = b.Run();
    if (s.ok()) {
      result = b.Report();
      rc = result.size();
    } else {
      band::json::Value e = band::json::Value::Object();
      e["error"] = band::json::Value::String(s.message());
      result = e.Dump();
    }
  }
  if (out && cap) {
    const size_t n = std::min(cap - 1, result.size());
    std::memcpy(out, result.data(), n);
    out[n] = 0;
  }
  return rc;
}
