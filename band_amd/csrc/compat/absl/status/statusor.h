// Minimal absl::StatusOr stand-in (see status.h).
#pragma once
#include <cstdlib>
#include <optional>
#include <utility>

#include "absl/status/status.h"

namespace absl {
template <typename T>
class StatusOr {
 public:
  StatusOr(const Status& s) : status_(s) {
    if (status_.ok()) status_ = InternalError("StatusOr constructed from OK status without value");
  }
  StatusOr(const T& v) : value_(v) {}
  StatusOr(T&& v) : value_(std::move(v)) {}
  bool ok() const { return status_.ok(); }
  const Status& status() const { return status_; }
  T& value() & {
    if (!ok()) std::abort();
    return *value_;
  }
  const T& value() const& {
    if (!ok()) std::abort();
    return *value_;
  }
  T&& value() && {
    if (!ok()) std::abort();
    return std::move(*value_);
  }
  T& operator*() { return value(); }
  T* operator->() { return &value(); }

 private:
  Status status_;
  std::optional<T> value_;
};
}  // namespace absl
