#include "backend/hip/tflite_reader.h"

#include <cstring>

namespace band {
namespace hip {

namespace {
template <typename T>
bool ReadAt(const uint8_t* buf, size_t size, size_t pos, T* out) {
  if (pos > size || size - pos < sizeof(T)) return false;
  std::memcpy(out, buf + pos, sizeof(T));
  return true;
}
}  // namespace

const char* TflBuiltinName(int c) {
  switch (c) {
    case kTflAdd: return "ADD";
    case kTflAveragePool2D: return "AVERAGE_POOL_2D";
    case kTflConcatenation: return "CONCATENATION";
    case kTflConv2D: return "CONV_2D";
    case kTflDepthwiseConv2D: return "DEPTHWISE_CONV_2D";
    case kTflDequantize: return "DEQUANTIZE";
    case kTflFullyConnected: return "FULLY_CONNECTED";
    case kTflLogistic: return "LOGISTIC";
    case kTflMaxPool2D: return "MAX_POOL_2D";
    case kTflMul: return "MUL";
    case kTflRelu: return "RELU";
    case kTflReluN1To1: return "RELU_N1_TO_1";
    case kTflRelu6: return "RELU6";
    case kTflPadV2: return "PADV2";
    case kTflReshape: return "RESHAPE";
    case kTflResizeBilinear: return "RESIZE_BILINEAR";
    case kTflSoftmax: return "SOFTMAX";
    case kTflCustom: return "CUSTOM";
    case kTflPad: return "PAD";
    case kTflMean: return "MEAN";
    case kTflSub: return "SUB";
    case kTflRsqrt: return "RSQRT";
    case kTflSquaredDifference: return "SQUARED_DIFFERENCE";
    case kTflMirrorPad: return "MIRROR_PAD";
    case kTflSqueeze: return "SQUEEZE";
    case kTflTransposeConv: return "TRANSPOSE_CONV";
    case kTflResizeNearestNeighbor: return "RESIZE_NEAREST_NEIGHBOR";
    case kTflQuantize: return "QUANTIZE";
    case kTflHardSwish: return "HARD_SWISH";
    default: return "UNKNOWN";
  }
}

DataType SchemaTypeToDataType(int t) {
  switch (t) {
    case 0: return DataType::kFloat32;
    case 1: return DataType::kFloat16;
    case 2: return DataType::kInt32;
    case 3: return DataType::kUInt8;
    case 4: return DataType::kInt64;
    case 5: return DataType::kString;
    case 6: return DataType::kBool;
    case 7: return DataType::kInt16;
    case 8: return DataType::kComplex64;
    case 9: return DataType::kInt8;
    case 10: return DataType::kFloat64;
    default: return DataType::kNoType;
  }
}

FbTable::FbTable(const uint8_t* buf, size_t size, uint32_t pos) {
  int32_t soff;
  if (!ReadAt(buf, size, pos, &soff)) return;
  const int64_t vt = static_cast<int64_t>(pos) - soff;
  uint16_t vt_len;
  if (vt < 0 || !ReadAt(buf, size, static_cast<size_t>(vt), &vt_len) || vt_len < 4 ||
      static_cast<size_t>(vt) + vt_len > size)
    return;
  buf_ = buf;
  size_ = size;
  pos_ = pos;
  vt_ = static_cast<uint32_t>(vt);
  vt_len_ = vt_len;
}

uint16_t FbTable::FieldOffset(int slot) const {
  if (!buf_) return 0;
  const uint32_t o = 4 + 2 * static_cast<uint32_t>(slot);
  if (o + 2 > vt_len_) return 0;
  uint16_t v = 0;
  ReadAt(buf_, size_, vt_ + o, &v);
  return v;
}

#define FB_SCALAR(NAME, T)                                 \
  T FbTable::NAME(int slot, T def) const {                 \
    const uint16_t o = FieldOffset(slot);                  \
    T v;                                                   \
    if (!o || !ReadAt(buf_, size_, pos_ + o, &v)) return def; \
    return v;                                              \
  }
FB_SCALAR(Int, int32_t)
FB_SCALAR(Int8, int8_t)
FB_SCALAR(UInt8, uint8_t)
FB_SCALAR(UInt, uint32_t)
FB_SCALAR(Float, float)
#undef FB_SCALAR

bool FbTable::Deref(int slot, uint32_t* target) const {
  const uint16_t o = FieldOffset(slot);
  uint32_t rel;
  if (!o || !ReadAt(buf_, size_, pos_ + o, &rel)) return false;
  const uint64_t t = static_cast<uint64_t>(pos_) + o + rel;
  if (t >= size_) return false;
  *target = static_cast<uint32_t>(t);
  return true;
}

FbTable FbTable::Table(int slot) const {
  uint32_t t;
  if (!Deref(slot, &t)) return FbTable();
  return FbTable(buf_, size_, t);
}

bool FbTable::VecHeader(int slot, size_t elem, uint32_t* start, uint32_t* n) const {
  uint32_t t;
  if (!Deref(slot, &t)) return false;
  uint32_t len;
  if (!ReadAt(buf_, size_, t, &len)) return false;
  if (static_cast<uint64_t>(t) + 4 + static_cast<uint64_t>(len) * elem > size_) return false;
  *start = t + 4;
  *n = len;
  return true;
}

std::string FbTable::String(int slot) const {
  uint32_t s, n;
  if (!VecHeader(slot, 1, &s, &n)) return std::string();
  return std::string(reinterpret_cast<const char*>(buf_ + s), n);
}

bool FbTable::VecInt32(int slot, std::vector<int32_t>* out) const {
  uint32_t s, n;
  if (!VecHeader(slot, 4, &s, &n)) return false;
  out->resize(n);
  if (n) std::memcpy(out->data(), buf_ + s, 4ull * n);
  return true;
}
bool FbTable::VecInt64(int slot, std::vector<int64_t>* out) const {
  uint32_t s, n;
  if (!VecHeader(slot, 8, &s, &n)) return false;
  out->resize(n);
  if (n) std::memcpy(out->data(), buf_ + s, 8ull * n);
  return true;
}
bool FbTable::VecFloat(int slot, std::vector<float>* out) const {
  uint32_t s, n;
  if (!VecHeader(slot, 4, &s, &n)) return false;
  out->resize(n);
  if (n) std::memcpy(out->data(), buf_ + s, 4ull * n);
  return true;
}
bool FbTable::VecBytes(int slot, const uint8_t** data, size_t* n) const {
  uint32_t s, len;
  if (!VecHeader(slot, 1, &s, &len)) return false;
  *data = buf_ + s;
  *n = len;
  return true;
}
bool FbTable::VecTables(int slot, std::vector<FbTable>* out) const {
  uint32_t s, n;
  if (!VecHeader(slot, 4, &s, &n)) return false;
  out->clear();
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t e = s + 4 * i;
    uint32_t rel;
    if (!ReadAt(buf_, size_, e, &rel)) return false;
    const uint64_t t = static_cast<uint64_t>(e) + rel;
    if (t >= size_) return false;
    FbTable tab(buf_, size_, static_cast<uint32_t>(t));
    if (!tab.valid()) return false;
    out->push_back(tab);
  }
  return true;
}

bool TflModel::Parse(const uint8_t* buf, size_t size, std::string* error) {
  auto fail = [&](const char* m) {
    if (error) *error = m;
    return false;
  };
  uint32_t root_off;
  if (!buf || !ReadAt(buf, size, 0, &root_off)) return fail("buffer too small");
  FbTable root(buf, size, root_off);
  if (!root.valid()) return fail("invalid root table");
  version = root.UInt(0, 0);
  if (version != 3) return fail("unsupported TFLite schema version (need 3)");

  std::vector<FbTable> opcodes, subgraphs, buffers;
  if (!root.VecTables(1, &opcodes)) return fail("missing operator_codes");
  if (!root.VecTables(2, &subgraphs) || subgraphs.empty()) return fail("missing subgraphs");
  root.VecTables(4, &buffers);

  std::vector<std::pair<int, std::string>> codes;
  for (auto& oc : opcodes) {
    const int dep = oc.Int8(0, 0);
    const int code = oc.Int(3, 0);
    codes.emplace_back(dep > code ? dep : code, oc.String(1));
  }

  const FbTable& sg = subgraphs[0];
  std::vector<FbTable> tt, ot;
  if (!sg.VecTables(0, &tt)) return fail("subgraph has no tensors");
  sg.VecTables(3, &ot);
  std::vector<int32_t> v;
  if (!sg.VecInt32(1, &v)) return fail("subgraph has no inputs");
  inputs.assign(v.begin(), v.end());
  if (!sg.VecInt32(2, &v)) return fail("subgraph has no outputs");
  outputs.assign(v.begin(), v.end());

  tensors.clear();
  for (auto& t : tt) {
    TflTensor x;
    std::vector<int32_t> shp;
    t.VecInt32(0, &shp);
    x.shape.assign(shp.begin(), shp.end());
    for (int d : x.shape)
      if (d < 0) return fail("dynamic tensor shapes are not supported");
    x.schema_type = t.Int8(1, 0);
    x.type = SchemaTypeToDataType(x.schema_type);
    const uint32_t bidx = t.UInt(2, 0);
    x.name = t.String(3);
    FbTable q = t.Table(4);
    if (q.valid()) {
      q.VecFloat(2, &x.scale);
      q.VecInt64(3, &x.zero_point);
      if (!x.scale.empty() && x.zero_point.size() != x.scale.size()) x.zero_point.assign(x.scale.size(), 0);
      x.quantized_dimension = q.Int(6, 0);
    }
    if (bidx != 0 && bidx < buffers.size()) {
      const uint8_t* d = nullptr;
      size_t n = 0;
      if (buffers[bidx].VecBytes(0, &d, &n) && n > 0) {
        x.data = d;
        x.data_size = n;
      }
    }
    tensors.push_back(std::move(x));
  }
  const int nt = static_cast<int>(tensors.size());
  for (int i : inputs)
    if (i < 0 || i >= nt) return fail("input tensor index out of range");
  for (int i : outputs)
    if (i < 0 || i >= nt) return fail("output tensor index out of range");

  ops.clear();
  for (auto& o : ot) {
    TflOperator op;
    const uint32_t ci = o.UInt(0, 0);
    if (ci >= codes.size()) return fail("opcode index out of range");
    op.builtin = codes[ci].first;
    op.custom_code = codes[ci].second;
    std::vector<int32_t> a;
    o.VecInt32(1, &a);
    op.inputs.assign(a.begin(), a.end());
    a.clear();
    o.VecInt32(2, &a);
    op.outputs.assign(a.begin(), a.end());
    for (int i : op.inputs)
      if (i < -1 || i >= nt) return fail("operator input index out of range");
    for (int i : op.outputs)
      if (i < 0 || i >= nt) return fail("operator output index out of range");
    op.options_type = o.UInt8(3, 0);
    op.options = o.Table(4);
    o.VecBytes(5, &op.custom_options, &op.custom_options_size);
    ops.push_back(std::move(op));
  }
  return true;
}

namespace {
uint64_t ReadU(const uint8_t* p, int w) {
  uint64_t v = 0;
  for (int i = 0; i < w; ++i) v |= static_cast<uint64_t>(p[i]) << (8 * i);
  return v;
}
int64_t ReadI(const uint8_t* p, int w) {
  const uint64_t u = ReadU(p, w);
  if (w >= 8) return static_cast<int64_t>(u);
  const uint64_t sign = 1ull << (8 * w - 1);
  return static_cast<int64_t>((u ^ sign) - sign);
}
}  // namespace

// FlexBuffers: the root (offset, packed type, byte width) sits at the end;
// a map's elements are preceded by [keys vector offset, keys width, size]
// and followed by one packed type byte per element (type << 2 | width).
bool FlexMap::Parse(const uint8_t* buf, size_t size) {
  items_.clear();
  if (!buf || size < 3) return false;
  const int rw = buf[size - 1];
  const uint8_t rtype = buf[size - 2];
  if ((rtype >> 2) != 9 || (rw != 1 && rw != 2 && rw != 4 && rw != 8) || size < static_cast<size_t>(2 + rw))
    return false;
  const size_t root = size - 2 - rw;
  const uint64_t off = ReadU(buf + root, rw);
  if (off > root) return false;
  const size_t m = root - off;
  const int w = 1 << (rtype & 3);
  if (m < static_cast<size_t>(3 * w)) return false;
  const uint64_t n = ReadU(buf + m - w, w);
  const int kw = static_cast<int>(ReadU(buf + m - 2 * w, w));
  const uint64_t koff = ReadU(buf + m - 3 * w, w);
  if (koff > m - 3 * w || (kw != 1 && kw != 2 && kw != 4 && kw != 8) || m + n * (w + 1) > size) return false;
  const size_t keys = m - 3 * w - koff;
  for (uint64_t i = 0; i < n; ++i) {
    const size_t kp = keys + i * kw;
    if (kp + kw > size) return false;
    const uint64_t so = ReadU(buf + kp, kw);
    if (so > kp) return false;
    const size_t ks = kp - so;
    size_t ke = ks;
    while (ke < size && buf[ke]) ++ke;
    if (ke >= size) return false;
    const std::string key(reinterpret_cast<const char*>(buf + ks), ke - ks);
    const uint8_t t = buf[m + n * w + i] >> 2;
    const uint8_t* v = buf + m + i * w;
    double value;
    switch (t) {
      case 1: value = static_cast<double>(ReadI(v, w)); break;       // INT
      case 2: case 26: value = static_cast<double>(ReadU(v, w)); break;  // UINT / BOOL
      case 3: {                                                        // FLOAT
        if (w == 8) {
          double d;
          std::memcpy(&d, v, 8);
          value = d;
        } else if (w == 4) {
          float f;
          std::memcpy(&f, v, 4);
          value = f;
        } else {
          return false;
        }
      } break;
      default: continue;  // not a scalar this backend reads
    }
    items_.emplace_back(key, value);
  }
  return true;
}

bool FlexMap::Has(const std::string& key) const {
  for (const auto& kv : items_)
    if (kv.first == key) return true;
  return false;
}

double FlexMap::Number(const std::string& key, double dflt) const {
  for (const auto& kv : items_)
    if (kv.first == key) return kv.second;
  return dflt;
}

}  // namespace hip
}  // namespace band
