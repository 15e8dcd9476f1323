// Bounds-checked reader for TFLite schema-v3 flatbuffers (.tflite).
//
// Replaces what the reference gets from tflite::FlatBufferModel
// (band/backend/tfl/model.cc:25-39): the HIP backend needs the primary
// subgraph's tensors (shape, type, constant data, quantisation) and its
// operators (builtin code, tensor indices, builtin options).  No flatbuffers
// library is used; every offset is validated against the buffer size so a
// truncated or hostile file fails with an error instead of a wild read.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "band/common.h"

namespace band {
namespace hip {

// schema.fbs BuiltinOperator codes used by this backend
enum TflBuiltin : int {
  kTflAdd = 0, kTflAveragePool2D = 1, kTflConcatenation = 2, kTflConv2D = 3,
  kTflDepthwiseConv2D = 4, kTflDequantize = 6, kTflFullyConnected = 9, kTflLogistic = 14,
  kTflMaxPool2D = 17, kTflMul = 18, kTflRelu = 19, kTflReluN1To1 = 20, kTflRelu6 = 21, kTflReshape = 22,
  kTflResizeBilinear = 23, kTflSoftmax = 25, kTflCustom = 32, kTflPad = 34, kTflMean = 40,
  kTflSub = 41, kTflRsqrt = 76, kTflSquaredDifference = 99, kTflMirrorPad = 100, kTflSqueeze = 43, kTflPadV2 = 60, kTflTransposeConv = 67, kTflResizeNearestNeighbor = 97,
  kTflQuantize = 114, kTflHardSwish = 117,
};

const char* TflBuiltinName(int code);

// A validated view of one flatbuffer table.
class FbTable {
 public:
  FbTable() = default;
  FbTable(const uint8_t* buf, size_t size, uint32_t pos);
  bool valid() const { return buf_ != nullptr; }
  bool Has(int slot) const { return FieldOffset(slot) != 0; }
  int32_t Int(int slot, int32_t def) const;
  int8_t Int8(int slot, int8_t def) const;
  uint8_t UInt8(int slot, uint8_t def) const;
  uint32_t UInt(int slot, uint32_t def) const;
  float Float(int slot, float def) const;
  bool Bool(int slot, bool def) const { return UInt8(slot, def ? 1 : 0) != 0; }
  FbTable Table(int slot) const;
  std::string String(int slot) const;
  // vector accessors; return false when absent or out of bounds
  bool VecInt32(int slot, std::vector<int32_t>* out) const;
  bool VecInt64(int slot, std::vector<int64_t>* out) const;
  bool VecFloat(int slot, std::vector<float>* out) const;
  bool VecBytes(int slot, const uint8_t** data, size_t* n) const;
  bool VecTables(int slot, std::vector<FbTable>* out) const;

 private:
  uint16_t FieldOffset(int slot) const;
  bool Deref(int slot, uint32_t* target) const;
  bool VecHeader(int slot, size_t elem, uint32_t* start, uint32_t* n) const;
  const uint8_t* buf_ = nullptr;
  size_t size_ = 0;
  uint32_t pos_ = 0;
  uint32_t vt_ = 0;
  uint16_t vt_len_ = 0;
};

struct TflTensor {
  std::vector<int> shape;
  int schema_type = 0;          // schema TensorType
  DataType type = DataType::kNoType;  // Band DataType (== TfLiteType)
  const uint8_t* data = nullptr;  // constant (buffer-backed) data, else null
  size_t data_size = 0;
  std::string name;
  std::vector<float> scale;
  std::vector<int64_t> zero_point;
  int quantized_dimension = 0;
  bool is_const() const { return data != nullptr; }
  size_t num_elements() const {
    size_t n = 1;
    for (int d : shape) n *= static_cast<size_t>(d);
    return n;
  }
};

struct TflOperator {
  int builtin = -1;
  std::string custom_code;
  std::vector<int> inputs, outputs;
  int options_type = 0;
  FbTable options;  // builtin_options table (slot meanings per op, schema.fbs)
  const uint8_t* custom_options = nullptr;  // FlexBuffers bytes (CUSTOM ops)
  size_t custom_options_size = 0;
};

// Scalars of a FlexBuffers map (TFLite custom options, e.g.
// TFLite_Detection_PostProcess's, detection_postprocess.cc Init()).
class FlexMap {
 public:
  bool Parse(const uint8_t* buf, size_t size);
  bool Has(const std::string& key) const;
  double Number(const std::string& key, double dflt) const;

 private:
  std::vector<std::pair<std::string, double>> items_;
};

struct TflModel {
  uint32_t version = 0;
  std::vector<TflTensor> tensors;
  std::vector<TflOperator> ops;
  std::vector<int> inputs, outputs;
  // Parses `buf` (which must outlive the model).  Returns false + message.
  bool Parse(const uint8_t* buf, size_t size, std::string* error);
};

// schema TensorType -> Band DataType
DataType SchemaTypeToDataType(int schema_type);

}  // namespace hip
}  // namespace band
