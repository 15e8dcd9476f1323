// Latency estimator (band/latency_estimator.h/.cc): per-subgraph profiled
// latency (online: measured at RegisterModel on every worker; offline: read
// from a profile JSON) and an exponentially smoothed expected latency that
// workers update after every job.
#pragma once
#include <map>
#include <mutex>
#include <string>

#include "engine/config.h"
#include "engine/engine_interface.h"

namespace band {

class LatencyEstimator {
 public:
  explicit LatencyEstimator(IEngine* engine) : engine_(engine) {}
  absl::Status Init(const ProfileConfig& config);
  void UpdateLatency(const SubgraphKey& key, int64_t latency);
  absl::Status ProfileModel(ModelId model_id);
  int64_t GetProfiled(const SubgraphKey& key) const;
  int64_t GetExpected(const SubgraphKey& key) const;
  int64_t GetWorst(ModelId model_id) const;
  absl::Status DumpProfile();
  size_t GetProfileHash() const;
  // JSON text of the profile database in the reference's layout
  // {"hash": H, "<model path>": {"<unit indices>": {"<worker id>": us}}}
  std::string ProfileToJson() const;

 private:
  struct Latency {
    int64_t profiled;
    int64_t moving_averaged;
  };
  std::map<SubgraphKey, Latency> JsonToModelProfile(const std::string& model_path, ModelId model_id) const;

  IEngine* const engine_;
  mutable std::mutex mu_;
  std::map<SubgraphKey, Latency> profile_database_;
  bool profile_online_ = true;
  int profile_num_warmups_ = 1;
  int profile_num_runs_ = 1;
  float profile_smoothing_factor_ = 0.1f;
  std::string profile_data_path_;
  std::string profile_json_text_;
  bool share_identical_ = false;
  // workers of the same device kind as w (w included), for share_identical_
  std::vector<WorkerId> IdenticalWorkers(WorkerId w) const;
};

}  // namespace band
