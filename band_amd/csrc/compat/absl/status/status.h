// Minimal stand-in for the subset of absl::Status that Band's backend API
// uses (band/interface/*.h return absl::Status / absl::StatusOr).  When this
// backend is built inside Band, the real Abseil headers take its place.
#pragma once
#include <string>
#include <utility>

namespace absl {
enum class StatusCode : int {
  kOk = 0, kCancelled = 1, kUnknown = 2, kInvalidArgument = 3, kDeadlineExceeded = 4,
  kNotFound = 5, kAlreadyExists = 6, kPermissionDenied = 7, kResourceExhausted = 8,
  kFailedPrecondition = 9, kAborted = 10, kOutOfRange = 11, kUnimplemented = 12,
  kInternal = 13, kUnavailable = 14, kDataLoss = 15, kUnauthenticated = 16,
};

class Status {
 public:
  Status() = default;
  Status(StatusCode code, std::string msg) : code_(code), msg_(std::move(msg)) {}
  bool ok() const { return code_ == StatusCode::kOk; }
  StatusCode code() const { return code_; }
  const std::string& message() const { return msg_; }
  std::string ToString() const { return ok() ? "OK" : msg_; }
  bool operator==(const Status& o) const { return code_ == o.code_ && msg_ == o.msg_; }
  bool operator!=(const Status& o) const { return !(*this == o); }

 private:
  StatusCode code_ = StatusCode::kOk;
  std::string msg_;
};

inline Status OkStatus() { return Status(); }
inline Status InternalError(std::string m) { return Status(StatusCode::kInternal, std::move(m)); }
inline Status InvalidArgumentError(std::string m) { return Status(StatusCode::kInvalidArgument, std::move(m)); }
inline Status DeadlineExceededError(std::string m) { return Status(StatusCode::kDeadlineExceeded, std::move(m)); }
inline Status NotFoundError(std::string m) { return Status(StatusCode::kNotFound, std::move(m)); }
inline Status UnavailableError(std::string m) { return Status(StatusCode::kUnavailable, std::move(m)); }
inline Status UnimplementedError(std::string m) { return Status(StatusCode::kUnimplemented, std::move(m)); }
inline bool IsUnimplemented(const Status& s) { return s.code() == StatusCode::kUnimplemented; }
}  // namespace absl
