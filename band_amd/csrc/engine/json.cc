#include "engine/json.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace band {
namespace json {

Value Value::Number(double v) {
  Value x;
  x.kind_ = Kind::kNumber;
  x.num_ = v;
  return x;
}
Value Value::String(std::string s) {
  Value x;
  x.kind_ = Kind::kString;
  x.str_ = std::move(s);
  return x;
}
Value Value::Bool(bool b) {
  Value x;
  x.kind_ = Kind::kBool;
  x.b_ = b;
  return x;
}
Value Value::Array() {
  Value x;
  x.kind_ = Kind::kArray;
  return x;
}
Value Value::Object() {
  Value x;
  x.kind_ = Kind::kObject;
  return x;
}

Value& Value::operator[](const std::string& key) {
  if (kind_ != Kind::kObject) *this = Object();
  for (auto& kv : obj_)
    if (kv.first == key) return kv.second;
  obj_.emplace_back(key, Value());
  return obj_.back().second;
}

const Value* Value::find(const std::string& key) const {
  if (kind_ != Kind::kObject) return nullptr;
  for (const auto& kv : obj_)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

void Value::push_back(Value v) {
  if (kind_ != Kind::kArray) *this = Array();
  arr_.push_back(std::move(v));
}

namespace {
void DumpString(const std::string& s, std::ostringstream& o) {
  o << '"';
  for (char c : s) {
    switch (c) {
      case '"': o << "\\\""; break;
      case '\\': o << "\\\\"; break;
      case '\n': o << "\\n"; break;
      case '\t': o << "\\t"; break;
      case '\r': o << "\\r"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          o << buf;
        } else {
          o << c;
        }
    }
  }
  o << '"';
}

void DumpValue(const Value& v, std::ostringstream& o) {
  switch (v.kind()) {
    case Value::Kind::kNull: o << "null"; break;
    case Value::Kind::kBool: o << (v.as_bool() ? "true" : "false"); break;
    case Value::Kind::kNumber: {
      const double d = v.as_number();
      if (std::floor(d) == d && std::fabs(d) < 9e15) o << static_cast<long long>(d);
      else o << d;
    } break;
    case Value::Kind::kString: DumpString(v.as_string(), o); break;
    case Value::Kind::kArray: {
      o << '[';
      for (size_t i = 0; i < v.size(); ++i) {
        if (i) o << ',';
        DumpValue(v.at(i), o);
      }
      o << ']';
    } break;
    case Value::Kind::kObject: {
      o << '{';
      bool first = true;
      for (const auto& kv : v.items()) {
        if (!first) o << ',';
        first = false;
        DumpString(kv.first, o);
        o << ':';
        DumpValue(kv.second, o);
      }
      o << '}';
    } break;
  }
}

struct Parser {
  const std::string& t;
  size_t i = 0;
  std::string err;
  explicit Parser(const std::string& text) : t(text) {}
  void ws() {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\t' || t[i] == '\r')) ++i;
  }
  bool fail(const char* m) {
    if (err.empty()) err = std::string(m) + " at offset " + std::to_string(i);
    return false;
  }
  bool lit(const char* s) {
    size_t n = std::char_traits<char>::length(s);
    if (t.compare(i, n, s) != 0) return fail("bad literal");
    i += n;
    return true;
  }
  bool str(std::string* out) {
    if (i >= t.size() || t[i] != '"') return fail("expected string");
    ++i;
    out->clear();
    while (i < t.size() && t[i] != '"') {
      char c = t[i++];
      if (c == '\\') {
        if (i >= t.size()) return fail("bad escape");
        char e = t[i++];
        switch (e) {
          case 'n': out->push_back('\n'); break;
          case 't': out->push_back('\t'); break;
          case 'r': out->push_back('\r'); break;
          case 'b': out->push_back('\b'); break;
          case 'f': out->push_back('\f'); break;
          case 'u': {
            if (i + 4 > t.size()) return fail("bad \\u escape");
            unsigned cp = std::strtoul(t.substr(i, 4).c_str(), nullptr, 16);
            i += 4;
            if (cp < 0x80) {
              out->push_back(static_cast<char>(cp));
            } else if (cp < 0x800) {
              out->push_back(static_cast<char>(0xC0 | (cp >> 6)));
              out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
            } else {
              out->push_back(static_cast<char>(0xE0 | (cp >> 12)));
              out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
              out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
            }
          } break;
          default: out->push_back(e);
        }
      } else {
        out->push_back(c);
      }
    }
    if (i >= t.size()) return fail("unterminated string");
    ++i;
    return true;
  }
  bool value(Value* v) {
    ws();
    if (i >= t.size()) return fail("unexpected end");
    char c = t[i];
    if (c == '{') {
      ++i;
      *v = Value::Object();
      ws();
      if (i < t.size() && t[i] == '}') {
        ++i;
        return true;
      }
      while (true) {
        ws();
        std::string k;
        if (!str(&k)) return false;
        ws();
        if (i >= t.size() || t[i] != ':') return fail("expected ':'");
        ++i;
        Value child;
        if (!value(&child)) return false;
        (*v)[k] = std::move(child);
        ws();
        if (i < t.size() && t[i] == ',') {
          ++i;
          continue;
        }
        if (i < t.size() && t[i] == '}') {
          ++i;
          return true;
        }
        return fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++i;
      *v = Value::Array();
      ws();
      if (i < t.size() && t[i] == ']') {
        ++i;
        return true;
      }
      while (true) {
        Value child;
        if (!value(&child)) return false;
        v->push_back(std::move(child));
        ws();
        if (i < t.size() && t[i] == ',') {
          ++i;
          continue;
        }
        if (i < t.size() && t[i] == ']') {
          ++i;
          return true;
        }
        return fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      std::string s;
      if (!str(&s)) return false;
      *v = Value::String(std::move(s));
      return true;
    }
    if (c == 't') {
      if (!lit("true")) return false;
      *v = Value::Bool(true);
      return true;
    }
    if (c == 'f') {
      if (!lit("false")) return false;
      *v = Value::Bool(false);
      return true;
    }
    if (c == 'n') {
      if (!lit("null")) return false;
      *v = Value();
      return true;
    }
    const char* start = t.c_str() + i;
    char* end = nullptr;
    double d = std::strtod(start, &end);
    if (end == start) return fail("bad value");
    i += static_cast<size_t>(end - start);
    *v = Value::Number(d);
    return true;
  }
};
}  // namespace

std::string Value::Dump() const {
  std::ostringstream o;
  o.precision(17);
  DumpValue(*this, o);
  return o.str();
}

bool Parse(const std::string& text, Value* out, std::string* error) {
  Parser p(text);
  Value v;
  bool ok = p.value(&v);
  if (ok) {
    p.ws();
    if (p.i != text.size()) ok = p.fail("trailing characters");
  }
  if (!ok) {
    if (error) *error = p.err;
    *out = Value();
    return false;
  }
  *out = std::move(v);
  return true;
}

bool LoadFile(const std::string& path, Value* out, std::string* error) {
  std::ifstream f(path);
  if (!f) {
    if (error) *error = "cannot open " + path;
    *out = Value();
    return false;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  return Parse(ss.str(), out, error);
}

}  // namespace json
}  // namespace band
