// Host-only unit tests of the native harness (no GPU, no backend): the
// schedulers against a mock engine with the reference's parameterised
// cases (band/test/scheduler_test.cc), the model analyzer's unit-subgraph
// partitioning, the latency estimator's profile JSON and the JSON reader.
// Built and run by tests/test_engine_native.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "engine/json.h"
#include "engine/model_analyzer.h"
#include "engine/scheduler.h"
#include "engine/tensor.h"
#include "engine/worker.h"

using namespace band;

static int g_failures = 0;
static int g_checks = 0;
#define CHECK_EQ(a, b)                                                                                   \
  do {                                                                                                   \
    ++g_checks;                                                                                          \
    auto _va = (a);                                                                                      \
    auto _vb = (b);                                                                                      \
    if (!(_va == _vb)) {                                                                                 \
      ++g_failures;                                                                                      \
      std::fprintf(stderr, "%s:%d CHECK_EQ(%s, %s) failed\n", __FILE__, __LINE__, #a, #b);               \
    }                                                                                                    \
  } while (0)
#define CHECK(c) CHECK_EQ(static_cast<bool>(c), true)

// ---- a mock engine in the spirit of the reference's scheduler test -------
struct MockEngine : public IEngine {
  explicit MockEngine(std::set<WorkerId> idle) : idle_(idle.begin(), idle.end()) {
    for (WorkerId w : idle_) waiting_[w] = 0;
  }
  std::vector<WorkerId> idle_;
  mutable WorkerWaitingTime waiting_;
  std::vector<ScheduleAction> actions;
  mutable size_t next_fixed = 0;
  std::vector<std::unique_ptr<Worker>> workers;
  std::vector<DeviceFlag> devices;

  void UpdateWorkersWaiting() const override {
    for (WorkerId w : idle_) waiting_[w] = 0;
    for (const auto& a : actions) waiting_[a.second.GetWorkerId()] += a.first.expected_latency;
  }
  WorkerWaitingTime GetWorkerWaitingTime() const override { return waiting_; }
  std::set<WorkerId> GetIdleWorkers() const override {
    std::set<WorkerId> s;
    for (auto& kv : waiting_)
      if (kv.second == 0) s.insert(kv.first);
    return s;
  }
  size_t GetNumWorkers() const override { return devices.size(); }
  DeviceFlag GetWorkerDevice(WorkerId id) const override { return devices.at(id); }
  Worker* GetWorker(WorkerId id) override { return id < (int)workers.size() ? workers[id].get() : nullptr; }
  const Worker* GetWorker(WorkerId id) const override {
    return id < (int)workers.size() ? workers[id].get() : nullptr;
  }
  SubgraphKey GetLargestSubgraphKey(ModelId m, WorkerId w) const override { return SubgraphKey(m, w, {0}); }
  const ModelSpec* GetModelSpec(ModelId) const override { return nullptr; }
  WorkerId GetModelWorker(ModelId) const override {
    return next_fixed < idle_.size() ? idle_[next_fixed++] : -1;
  }
  bool IsBegin(const SubgraphKey&) const override { return true; }
  bool IsEnd(const SubgraphKey&) const override { return true; }
  bool HasSubgraph(const SubgraphKey&) const override { return true; }
  void ForEachSubgraph(std::function<void(const SubgraphKey&)>) const override {}
  absl::Status Invoke(const SubgraphKey&) override { return absl::OkStatus(); }
  // the job's own expected_latency stands for its shortest plan
  std::pair<std::vector<SubgraphKey>, int64_t> GetSubgraphWithShortestLatency(
      const Job& job, const WorkerWaitingTime&) const override {
    const WorkerId w = job.target_worker_id != -1 ? job.target_worker_id : *idle_.begin();
    return {{SubgraphKey(job.model_id, w, {0}), SubgraphKey(job.model_id, 0, {0})}, job.expected_latency};
  }
  std::pair<SubgraphKey, int64_t> GetShortestSubgraphKey(const std::vector<SubgraphKey>&, int64_t,
                                                         const WorkerWaitingTime&) const override {
    return {SubgraphKey(), 0};
  }
  absl::Status TryCopyInputTensors(const Job&) override { return absl::OkStatus(); }
  absl::Status TryCopyOutputTensors(const Job&) override { return absl::OkStatus(); }
  void UpdateLatency(const SubgraphKey&, int64_t) override {}
  int64_t GetProfiled(const SubgraphKey&) const override { return 10; }
  int64_t GetExpected(const SubgraphKey&) const override { return 10; }
  int64_t GetWorst(ModelId) const override { return 10; }
  void Trigger() override {}
  JobId EnqueueRequest(Job, bool) override { return 0; }
  std::vector<JobId> EnqueueBatch(std::vector<Job>, bool) override { return {}; }
  void PrepareReenqueue(Job&) override {}
  void EnqueueFinishedJob(Job&) override {}
  bool EnqueueToWorker(const ScheduleAction& a) override {
    actions.push_back(a);
    return true;
  }
  bool EnqueueToWorkerBatch(const std::vector<ScheduleAction>& as) override {
    actions.insert(actions.end(), as.begin(), as.end());
    return true;
  }
};

static JobQueue Jobs(const std::vector<int>& models) {
  JobQueue q;
  for (int m : models) q.emplace_back(m);
  return q;
}

static void TestRoundRobin() {
  struct Case {
    std::vector<int> models;
    std::set<int> workers;
  } cases[] = {{{0, 1, 2}, {0, 1, 2}}, {{0, 1}, {0, 1, 2}}, {{0, 1, 2}, {0, 1}}};
  for (auto& c : cases) {
    MockEngine e(c.workers);
    JobQueue q = Jobs(c.models);
    RoundRobinScheduler s(e);
    s.Schedule(q);
    CHECK_EQ(e.actions.size(), std::min(c.models.size(), c.workers.size()));
    CHECK_EQ(c.models.size(), q.size() + e.actions.size());
  }
}

static void TestFixedWorker() {
  MockEngine e({0, 1, 2});
  JobQueue q = Jobs({0, 1, 2});
  FixedWorkerScheduler s(e);
  s.Schedule(q);
  CHECK_EQ(e.actions.size(), 3u);
  CHECK_EQ(q.size(), 0u);
  std::map<int, int> seen;
  for (auto& a : e.actions) seen[a.second.GetModelId()]++;
  for (int m : {0, 1, 2}) CHECK_EQ(seen[m], 1);
  // explicit target worker wins
  MockEngine e2({0, 1, 2});
  JobQueue q2 = Jobs({0, 1, 2});
  for (auto& j : q2) j.target_worker_id = 0;
  FixedWorkerScheduler s2(e2);
  s2.Schedule(q2);
  CHECK_EQ(e2.actions.size(), 3u);
  for (auto& a : e2.actions) CHECK_EQ(a.second.GetWorkerId(), 0);
}

static void TestSEL() {
  MockEngine e({0, 1, 2});
  std::vector<int64_t> lat = {2, 1, 3};
  JobQueue q;
  for (int i = 0; i < 3; ++i) {
    Job j(i);
    j.expected_latency = lat[i];
    q.push_back(j);
  }
  ShortestExpectedLatencyScheduler s(e, 3);
  s.Schedule(q);
  CHECK_EQ(e.actions.size(), 3u);
  CHECK_EQ(q.size(), 0u);
  const int expect[] = {2, 0, 1};  // largest shortest latency first
  for (int i = 0; i < 3; ++i) CHECK_EQ(e.actions[i].first.model_id, expect[i]);
}

static void TestHEFT() {
  struct Case {
    bool reserve;
    std::vector<int64_t> lat;
    std::vector<int> target;
    std::set<int> workers;
    std::vector<int> expect;
  } cases[] = {
      {false, {2, 1, 3}, {0, 1, 2}, {}, {}},
      {false, {2, 1, 3}, {0, 0, 0}, {0, 1, 2}, {2}},
      {false, {2, 1, 3}, {0, 1, 2}, {0, 1, 2}, {2, 0, 1}},
      {false, {2, 1, 3}, {0, 1, 2}, {0, 2}, {2, 0}},
      {false, {2, 3, 3}, {0, 0, 2}, {0, 1, 2}, {1, 2}},
  };
  for (auto& c : cases) {
    MockEngine e(c.workers);
    JobQueue q;
    for (size_t i = 0; i < c.lat.size(); ++i) {
      Job j(static_cast<int>(i));
      j.job_id = static_cast<int>(i);
      j.expected_latency = c.lat[i];
      j.target_worker_id = c.target[i];
      q.push_back(j);
    }
    HEFTScheduler s(e, static_cast<int>(c.lat.size()), c.reserve);
    s.Schedule(q);
    CHECK_EQ(e.actions.size(), c.expect.size());
    CHECK_EQ(c.lat.size() - e.actions.size(), q.size());
    for (size_t i = 0; i < c.expect.size() && i < e.actions.size(); ++i)
      CHECK_EQ(e.actions[i].first.model_id, c.expect[i]);
  }
}

static void TestLSF() {
  for (bool slo : {true, false}) {
    MockEngine e({0, 1, 2});
    JobQueue q;
    q.emplace_back(0, slo ? 100 : 0);
    q.emplace_back(1, slo ? 80 : 0);
    LeastSlackFirstScheduler s(e, 5);
    s.Schedule(q);
    CHECK_EQ(e.actions.size(), 2u);
    CHECK_EQ(q.size(), 0u);
    // with SLOs the least slack (model 1) goes first, else queue order
    CHECK_EQ(e.actions[0].second.GetModelId(), slo ? 1 : 0);
    CHECK_EQ(e.actions[1].second.GetModelId(), slo ? 0 : 1);
    if (slo) CHECK(e.actions[0].first.status == JobStatus::kSLOViolation);
  }
}

static void TestFixedWorkerGlobalQueue() {
  MockEngine e({0, 1});
  JobQueue q = Jobs({0, 1, 2});
  for (auto& j : q) j.target_worker_id = 1;
  FixedWorkerGlobalQueueScheduler s(e);
  s.Schedule(q);
  // one idle target worker: one job goes, the rest wait in the planner
  CHECK_EQ(e.actions.size(), 1u);
  CHECK_EQ(q.size(), 2u);
}

// ---- model analyzer ------------------------------------------------------
// a chain of n ops: op i reads tensor i, writes tensor i + 1
static ModelSpec Chain(int n, std::set<int> gpu_unsupported) {
  std::vector<std::set<int>> in(n), out(n);
  for (int i = 0; i < n; ++i) {
    in[i] = {i};
    out[i] = {i + 1};
  }
  std::map<DeviceFlag, std::set<int>> unsup{{DeviceFlag::kCPU, {}}, {DeviceFlag::kGPU, gpu_unsupported}};
  return ModelSpec(n, n + 1, std::vector<DataType>(n + 1, DataType::kInt8), {0}, {n}, in, out, unsup,
                   {DeviceFlag::kDSP, DeviceFlag::kNPU});
}

static MockEngine Workers(std::vector<DeviceFlag> devs) {
  std::set<int> ids;
  for (size_t i = 0; i < devs.size(); ++i) ids.insert(static_cast<int>(i));
  MockEngine e(ids);
  e.devices = devs;
  for (size_t i = 0; i < devs.size(); ++i)
    e.workers.emplace_back(new DeviceQueueWorker(&e, static_cast<int>(i), devs[i]));
  return e;
}

static void TestModelAnalyzer() {
  auto e = Workers({DeviceFlag::kCPU, DeviceFlag::kGPU, DeviceFlag::kGPU});
  SubgraphConfig cfg;
  cfg.minimum_subgraph_size = 1;
  cfg.subgraph_preparation_type = SubgraphPreparationType::kUnitSubgraph;
  {
    ModelAnalyzer a(e, true, cfg, Chain(10, {4}));
    auto r = a.CreateSubgraphs();
    CHECK(r.ok());
    const auto& spec = r.value().first;
    const auto& defs = r.value().second;
    // units: {0-3} on every worker, {4} on the CPU, {5-9} on every worker
    CHECK_EQ(spec.GetNumUnitSubgraphs(), 3u);
    CHECK_EQ(defs.size(), 7u);
    CHECK(spec.GetUnitSubgraphOps(1) == std::set<int>({4}));
    CHECK(spec.GetUnitSubgraphDependency(2).test(1));
    int cpu_only = 0;
    for (auto& d : defs)
      if (*d.unit_subgraph_indices.begin() == 1) {
        CHECK_EQ(d.worker_id, 0);
        cpu_only++;
      }
    CHECK_EQ(cpu_only, 1);
  }
  {
    // merged: every chain of units a worker can run end to end
    cfg.subgraph_preparation_type = SubgraphPreparationType::kMergeUnitSubgraph;
    ModelAnalyzer a(e, true, cfg, Chain(10, {4}));
    auto r = a.CreateSubgraphs();
    CHECK(r.ok());
    int whole_cpu = 0;
    for (auto& d : r.value().second)
      if (d.worker_id == 0 && d.op_indices.size() == 10) whole_cpu++;
    CHECK_EQ(whole_cpu, 1);
    for (auto& d : r.value().second)
      if (d.worker_id != 0) CHECK(!d.op_indices.count(4));
  }
  {
    // GPU runs shorter than minimum_subgraph_size stay on the CPU
    cfg.minimum_subgraph_size = 7;
    cfg.subgraph_preparation_type = SubgraphPreparationType::kUnitSubgraph;
    ModelAnalyzer a(e, true, cfg, Chain(10, {4}));
    auto r = a.CreateSubgraphs();
    CHECK(r.ok());
    CHECK_EQ(r.value().first.GetNumUnitSubgraphs(), 1u);
    CHECK_EQ(r.value().second.size(), 1u);
    CHECK_EQ(r.value().second[0].worker_id, 0);
  }
  {
    // no fallback (fixed_worker / round_robin): whole model on every worker
    ModelAnalyzer a(e, false, cfg, Chain(10, {4}));
    auto r = a.CreateSubgraphs();
    CHECK(r.ok());
    CHECK_EQ(r.value().second.size(), 3u);
    for (auto& d : r.value().second) CHECK_EQ(d.op_indices.size(), 10u);
  }
  {
    // fallback per worker: GPU worker gets {0-3},{5-9}; the CPU op goes to the CPU worker
    cfg.minimum_subgraph_size = 1;
    cfg.subgraph_preparation_type = SubgraphPreparationType::kFallbackPerWorker;
    ModelAnalyzer a(e, true, cfg, Chain(10, {4}));
    auto r = a.CreateSubgraphs();
    CHECK(r.ok());
    int gpu1 = 0;
    for (auto& d : r.value().second)
      if (d.worker_id == 1) gpu1++;
    CHECK_EQ(gpu1, 2);
  }
  CHECK_EQ(SetToString({0, 1, 2, 3, 5, 7, 8, 9}), std::string("{0-3,5,7-9}"));
}

static void TestJson() {
  json::Value v;
  CHECK(json::Parse("{\"a\": [1, 2.5, null, true], \"b\": {\"c\": \"x\\ny\"}}", &v));
  CHECK_EQ(v.find("a")->size(), 4u);
  CHECK_EQ(v.find("a")->at(1).as_number(), 2.5);
  CHECK(v.find("a")->at(2).is_null());
  CHECK_EQ(v.find("b")->find("c")->as_string(), std::string("x\ny"));
  json::Value w;
  CHECK(json::Parse(v.Dump(), &w));
  CHECK_EQ(w.Dump(), v.Dump());
  CHECK(!json::Parse("{\"a\": [1,}", &w));
}

// ---- request-ring slots in ring-allocator memory: the streaming-store copy
// into a slot (engine/tensor.cc PutIntoSlot) returns the bytes unchanged, for
// aligned and misaligned sources and sizes that are not a multiple of 32
struct ViewTensor : public interface::ITensor {
  ViewTensor(std::vector<int> d, char* p) : dims(std::move(d)), data(p) {}
  DataType GetType() const override { return DataType::kUInt8; }
  void SetType(DataType) override {}
  const char* GetData() const override { return data; }
  char* GetData() override { return data; }
  const int* GetDims() const override { return dims.data(); }
  size_t GetNumDims() const override { return dims.size(); }
  void SetDims(const std::vector<int>& d) override { dims = d; }
  const char* GetName() const override { return "view"; }
  Quantization GetQuantization() const override { return Quantization(QuantizationType::kNoQuantization, nullptr); }
  absl::Status SetQuantization(Quantization) override { return absl::OkStatus(); }
  std::vector<int> dims;
  char* data;
};

static void TestRingSlotCopies() {
  RingHostAllocator a;
  a.alloc = [](size_t n) -> void* { return std::aligned_alloc(4096, (n + 4095) / 4096 * 4096); };
  a.free = [](void* p) { std::free(p); };
  const std::vector<std::vector<int>> shapes = {{1, 224, 224, 3}, {1, 70001}, {1, 100}};
  std::vector<std::vector<char>> backing;
  std::vector<std::shared_ptr<interface::ITensor>> views;
  for (const auto& d : shapes) {
    size_t n = 1;
    for (int x : d) n *= static_cast<size_t>(x);
    backing.emplace_back(n + 64, 0);
    views.push_back(std::make_shared<ViewTensor>(d, backing.back().data()));
  }
  {
    TensorRingBuffer ring(views, {0, 1, 2}, 3, a);
    for (int round = 0; round < 5; ++round) {
      const int h = ring.AllocBlocking();
      std::vector<std::unique_ptr<ViewTensor>> src, dst;
      std::vector<interface::ITensor*> src_p, dst_p;
      for (size_t i = 0; i < shapes.size(); ++i) {
        const size_t n = views[i]->GetBytes();
        char* base = backing[i].data() + (round % 4) * 3;  // misaligned sources too
        for (size_t k = 0; k < n; ++k) base[k] = static_cast<char>((k * 131 + i * 7 + round) & 0xff);
        src.emplace_back(new ViewTensor(shapes[i], base));
        src_p.push_back(src.back().get());
      }
      CHECK(ring.PutTensorsToHandle(src_p, h).ok());
      CHECK(ring.SlotTensor(0, h) && ring.SlotTensor(0, h)->IsRingMemory());
      std::vector<std::vector<char>> out;
      for (size_t i = 0; i < shapes.size(); ++i) out.emplace_back(views[i]->GetBytes(), 0);
      for (size_t i = 0; i < shapes.size(); ++i) {
        dst.emplace_back(new ViewTensor(shapes[i], out[i].data()));
        dst_p.push_back(dst.back().get());
      }
      CHECK(ring.GetTensorsFromHandle(dst_p, h).ok());
      for (size_t i = 0; i < shapes.size(); ++i)
        CHECK(std::memcmp(out[i].data(), src[i]->GetData(), out[i].size()) == 0);
      // a source of another shape is refused, as ITensor::CopyDataFrom does
      ViewTensor wrong({1, 224, 224, 4}, backing[0].data());
      CHECK(!ring.PutTensorToHandle(&wrong, 0, h).ok());
      ring.Release(h);
    }
  }
}

int main() {
  TestRoundRobin();
  TestFixedWorker();
  TestSEL();
  TestHEFT();
  TestLSF();
  TestFixedWorkerGlobalQueue();
  TestModelAnalyzer();
  TestJson();
  TestRingSlotCopies();
  std::printf("%d checks, %d failures\n", g_checks, g_failures);
  return g_failures ? 1 : 0;
}
