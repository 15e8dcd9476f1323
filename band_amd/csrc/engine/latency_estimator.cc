#include "engine/latency_estimator.h"

#include <algorithm>
#include <cstdio>

#include "engine/logger.h"
#include <fstream>
#include <limits>
#include <sstream>
#include <thread>

#include "engine/json.h"
#include "engine/time.h"
#include "engine/worker.h"

namespace band {

absl::Status LatencyEstimator::Init(const ProfileConfig& config) {
  profile_data_path_ = config.profile_data_path;
  profile_online_ = config.online;
  profile_num_warmups_ = config.num_warmups;
  profile_num_runs_ = config.num_runs;
  profile_smoothing_factor_ = config.smoothing_factor;
  share_identical_ = config.share_identical_workers;
  if (!profile_online_) {
    std::ifstream f(profile_data_path_);
    if (f) {
      std::stringstream ss;
      ss << f.rdbuf();
      profile_json_text_ = ss.str();
    } else {
      BAND_LOG(LogSeverity::kWarning, "offline profile %s not readable", profile_data_path_.c_str());
    }
  }
  return absl::OkStatus();
}

std::vector<WorkerId> LatencyEstimator::IdenticalWorkers(WorkerId w) const {
  std::vector<WorkerId> out;
  const Worker* a = engine_->GetWorker(w);
  if (!a) return out;
  for (WorkerId v = 0; v < static_cast<WorkerId>(engine_->GetNumWorkers()); ++v) {
    const Worker* b = engine_->GetWorker(v);
    if (b && b->GetDeviceFlag() == a->GetDeviceFlag() && b->GetNumThreads() == a->GetNumThreads() &&
        b->GetWorkerThreadAffinity().GetCPUMaskFlag() == a->GetWorkerThreadAffinity().GetCPUMaskFlag())
      out.push_back(v);
  }
  return out;
}

// EWMA with the configured smoothing factor (band/latency_estimator.cc:32-45).
//
// Extension (share_identical_workers): the reference keeps one estimate per
// (subgraph, worker) and moves it only when that worker runs the subgraph.
// Under shortest_expected_latency an idle worker is chosen by its estimate
// alone, so among IDENTICAL workers the ones whose first profile happened to
// read high are never chosen, never run, and their estimates never move:
// they starve (r02 C5: three of eight GPU workers of one MI355X got 2, 8 and
// 66 jobs against ~450-1150).  With sharing, a latency observed on one worker
// updates the same subgraph on every worker of the same device kind.
void LatencyEstimator::UpdateLatency(const SubgraphKey& key, int64_t latency) {
  std::vector<WorkerId> peers;
  if (share_identical_) peers = IdenticalWorkers(key.GetWorkerId());
  std::lock_guard<std::mutex> lock(mu_);
  auto ewma = [&](const SubgraphKey& k) {
    auto it = profile_database_.find(k);
    if (it == profile_database_.end()) return;
    it->second.moving_averaged = static_cast<int64_t>(profile_smoothing_factor_ * latency +
                                                      (1 - profile_smoothing_factor_) * it->second.moving_averaged);
  };
  if (peers.empty()) {
    ewma(key);
    return;
  }
  const std::set<int> units = key.GetUnitIndicesSet();
  for (WorkerId w : peers) ewma(SubgraphKey(key.GetModelId(), w, units));
}

// Online: pause each worker, let it drain, and time every subgraph of the
// model on that worker from a separate thread (band/latency_estimator.cc:62-126).
absl::Status LatencyEstimator::ProfileModel(ModelId model_id) {
  if (profile_online_) {
    for (WorkerId w = 0; w < static_cast<WorkerId>(engine_->GetNumWorkers()); ++w) {
      Worker* worker = engine_->GetWorker(w);
      worker->Pause();
      worker->Wait();
      std::thread profiler([&] {
        engine_->ForEachSubgraph([&](const SubgraphKey& key) {
          if (key.GetWorkerId() != w || key.GetModelId() != model_id) return;
          for (int i = 0; i < profile_num_warmups_; ++i)
            if (!engine_->Invoke(key).ok())
              BAND_LOG(LogSeverity::kError, "profiler failed to invoke model %d on worker %d", model_id, w);
          int64_t total = 0;
          for (int i = 0; i < profile_num_runs_; ++i) {
            const int64_t t0 = time::NowMicros();
            if (!engine_->Invoke(key).ok())
              BAND_LOG(LogSeverity::kError, "profiler failed to invoke model %d on worker %d", model_id, w);
            total += time::NowMicros() - t0;
          }
          const int64_t avg = profile_num_runs_ > 0 ? total / profile_num_runs_ : 0;
          std::lock_guard<std::mutex> lock(mu_);
          profile_database_[key] = {avg, avg};
        });
      });
      profiler.join();
      worker->Resume();
    }
    if (share_identical_) {
      // identical workers start from one estimate: the median of their
      // profiles of each subgraph
      std::lock_guard<std::mutex> lock(mu_);
      std::map<std::pair<unsigned long long, WorkerId>, std::vector<int64_t>> groups;  // (units, first peer)
      std::map<SubgraphKey, WorkerId> head;
      for (const auto& kv : profile_database_) {
        if (kv.first.GetModelId() != model_id) continue;
        const std::vector<WorkerId> peers = IdenticalWorkers(kv.first.GetWorkerId());
        const WorkerId h = peers.empty() ? kv.first.GetWorkerId() : peers.front();
        head[kv.first] = h;
        groups[{kv.first.GetUnitIndices().to_ullong(), h}].push_back(kv.second.moving_averaged);
      }
      for (auto& kv : groups) std::sort(kv.second.begin(), kv.second.end());
      for (auto& kv : profile_database_) {
        auto h = head.find(kv.first);
        if (h == head.end()) continue;
        const auto& v = groups[{kv.first.GetUnitIndices().to_ullong(), h->second}];
        kv.second.moving_averaged = v[v.size() / 2];
      }
    }
    engine_->Trigger();  // jobs bounced while the workers were paused
  } else if (const ModelSpec* spec = engine_->GetModelSpec(model_id)) {
    auto entries = JsonToModelProfile(spec->path, model_id);
    if (entries.empty())
      BAND_LOG(LogSeverity::kWarning, "no profile entries for model %s", spec->path.c_str());
    std::lock_guard<std::mutex> lock(mu_);
    profile_database_.insert(entries.begin(), entries.end());
  }
  return absl::OkStatus();
}

int64_t LatencyEstimator::GetProfiled(const SubgraphKey& key) const {
  std::lock_guard<std::mutex> lock(mu_);
  auto it = profile_database_.find(key);
  return it == profile_database_.end() ? -1 : it->second.profiled;
}

int64_t LatencyEstimator::GetExpected(const SubgraphKey& key) const {
  std::lock_guard<std::mutex> lock(mu_);
  auto it = profile_database_.find(key);
  return it == profile_database_.end() ? std::numeric_limits<int32_t>::max() : it->second.moving_averaged;
}

int64_t LatencyEstimator::GetWorst(ModelId model_id) const {
  std::lock_guard<std::mutex> lock(mu_);
  int64_t worst = 0;
  for (const auto& kv : profile_database_)
    if (kv.first.GetModelId() == model_id) worst = std::max(worst, kv.second.moving_averaged);
  return worst;
}

// identifies the worker layout a profile was taken on
// (band/latency_estimator.cc:177-189)
size_t LatencyEstimator::GetProfileHash() const {
  size_t h = engine_->GetNumWorkers();
  for (WorkerId w = 0; w < static_cast<WorkerId>(engine_->GetNumWorkers()); ++w) {
    const Worker* worker = engine_->GetWorker(w);
    h ^= static_cast<size_t>(worker->GetDeviceFlag());
    h ^= static_cast<size_t>(worker->GetNumThreads());
    h ^= static_cast<size_t>(worker->GetWorkerThreadAffinity().GetCPUMaskFlag());
  }
  return h;
}

std::string LatencyEstimator::ProfileToJson() const {
  json::Value root = json::Value::Object();
  root["hash"] = json::Value::Number(static_cast<double>(GetProfileHash()));
  std::lock_guard<std::mutex> lock(mu_);
  for (const auto& kv : profile_database_) {
    const ModelSpec* spec = engine_->GetModelSpec(kv.first.GetModelId());
    if (!spec || spec->path.empty()) continue;
    // worker ids index an array, as jsoncpp writes Value[int]
    json::Value& per_worker = root[spec->path][kv.first.GetUnitIndicesString()];
    if (!per_worker.is_array()) per_worker = json::Value::Array();
    std::vector<json::Value> slots;
    for (size_t i = 0; i < per_worker.size(); ++i) slots.push_back(per_worker.at(i));
    const size_t w = static_cast<size_t>(kv.first.GetWorkerId());
    if (slots.size() <= w) slots.resize(w + 1);
    slots[w] = json::Value::Number(static_cast<double>(kv.second.profiled));
    per_worker = json::Value::Array();
    for (auto& s : slots) per_worker.push_back(s);
  }
  return root.Dump();
}

absl::Status LatencyEstimator::DumpProfile() {
  std::ofstream f(profile_data_path_);
  if (!f) return absl::InternalError("cannot write profile " + profile_data_path_);
  f << ProfileToJson();
  return absl::OkStatus();
}

std::map<SubgraphKey, LatencyEstimator::Latency> LatencyEstimator::JsonToModelProfile(const std::string& path,
                                                                                      ModelId model_id) const {
  std::map<SubgraphKey, Latency> out;
  json::Value root;
  if (profile_json_text_.empty() || !json::Parse(profile_json_text_, &root)) return out;
  const json::Value* hash = root.find("hash");
  if (!hash || static_cast<size_t>(hash->as_number()) != GetProfileHash()) {
    BAND_LOG(LogSeverity::kWarning, "profile hash does not match %s; ignored", profile_data_path_.c_str());
    return out;
  }
  const json::Value* model = root.find(path);
  if (!model || !model->is_object()) return out;
  for (const auto& units : model->items()) {
    std::set<int> unit_set;
    std::stringstream ss(units.first);
    for (int u; ss >> u;) {
      unit_set.insert(u);
      if (ss.peek() == ',') ss.ignore();
    }
    auto add = [&](int worker, const json::Value& v) {
      const int64_t us = v.as_int(0);
      if (us > 0) out[SubgraphKey(model_id, worker, unit_set)] = {us, us};
    };
    if (units.second.is_array()) {
      for (size_t w = 0; w < units.second.size(); ++w) add(static_cast<int>(w), units.second.at(w));
    } else {
      for (const auto& wv : units.second.items()) add(std::atoi(wv.first.c_str()), wv.second);
    }
  }
  return out;
}

}  // namespace band
