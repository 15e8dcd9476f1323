// A small JSON value / parser / writer for the harness's own files (the
// latency profile database and benchmark configs).  The reference uses
// jsoncpp (band/json_util.cc), which is not available here.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace band {
namespace json {

class Value {
 public:
  enum class Kind { kNull, kBool, kNumber, kString, kArray, kObject };
  Value() = default;
  static Value Number(double v);
  static Value String(std::string s);
  static Value Bool(bool b);
  static Value Array();
  static Value Object();

  Kind kind() const { return kind_; }
  bool is_null() const { return kind_ == Kind::kNull; }
  bool is_object() const { return kind_ == Kind::kObject; }
  bool is_array() const { return kind_ == Kind::kArray; }
  bool is_number() const { return kind_ == Kind::kNumber; }
  bool is_string() const { return kind_ == Kind::kString; }
  double as_number(double dflt = 0) const { return kind_ == Kind::kNumber ? num_ : dflt; }
  int64_t as_int(int64_t dflt = 0) const { return kind_ == Kind::kNumber ? static_cast<int64_t>(num_) : dflt; }
  bool as_bool(bool dflt = false) const { return kind_ == Kind::kBool ? b_ : dflt; }
  const std::string& as_string() const { return str_; }

  // object access (creates on write)
  Value& operator[](const std::string& key);
  const Value* find(const std::string& key) const;
  const std::vector<std::pair<std::string, Value>>& items() const { return obj_; }
  // array access
  void push_back(Value v);
  size_t size() const { return kind_ == Kind::kArray ? arr_.size() : obj_.size(); }
  const Value& at(size_t i) const { return arr_[i]; }

  std::string Dump() const;

 private:
  Kind kind_ = Kind::kNull;
  double num_ = 0;
  bool b_ = false;
  std::string str_;
  std::vector<Value> arr_;
  std::vector<std::pair<std::string, Value>> obj_;  // insertion order
};

// returns false (and leaves `out` null) on malformed input
bool Parse(const std::string& text, Value* out, std::string* error = nullptr);
bool LoadFile(const std::string& path, Value* out, std::string* error = nullptr);

}  // namespace json
}  // namespace band
