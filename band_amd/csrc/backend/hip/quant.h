// Host-side quantisation parameter derivation, restating what TFLite 2.9.2's
// Prepare() functions compute for the ops on Band's hot path (the reference
// builds these inside tflite::Interpreter during PrepareSubgraph,
// band/backend/tfl/model_executor.cc:173-192 -> CreateTfLiteInterpreter
// :327-373 -> AllocateTensors).  Bit-exactness of every kernel depends on
// reproducing the float/double arithmetic order here exactly:
//   QuantizeMultiplier            quantization_util.cc  (frexp + round, Q31 fix-up)
//   CalculateActivationRangeQuantized  kernel_util.cc (float divide, roundf)
//   PopulateConvolutionQuantizationParams kernel_util.cc (double per-channel;
//       uint8 legacy path = float(in*w)/out via GetQuantizedConvolutionMultipler)
//   add.cc / sub.cc Prepare (left_shift 20, twice_max_input_scale)
//   mul.cc Prepare (float in1*in2/out)
//   padding.h ComputePadding / ComputeOutSize
#pragma once

#include <cstdint>
#include <vector>

namespace band {
namespace hip {

void QuantizeMultiplier(double m, int32_t* q, int* shift);

// act: schema ActivationFunctionType (0 NONE, 1 RELU, 2 RELU_N1_TO_1, 3 RELU6)
void ActivationRangeQuantized(int act, float scale, int32_t zero_point, bool is_int8,
                              int32_t* act_min, int32_t* act_max);

// Per-output-channel multipliers for CONV_2D / DEPTHWISE_CONV_2D.
void ConvMultipliers(float in_scale, const std::vector<float>& w_scales, int channels,
                     float out_scale, bool legacy_uint8, std::vector<int32_t>* mult,
                     std::vector<int32_t>* shift);

// FULLY_CONNECTED (per-tensor, GetQuantizedConvolutionMultipler).
void FullyConnectedMultiplier(float in_scale, float w_scale, float out_scale, int32_t* mult,
                              int32_t* shift);

struct AddParams {
  int32_t m1, s1, m2, s2, mo, so, left_shift;
};
AddParams AddSubParams(float s1, float s2, float so, bool is_sub);

void MulMultiplier(float s1, float s2, float so, int32_t* mult, int32_t* shift);

int ComputeOutSize(bool same, int in, int filter, int stride, int dilation);
int ComputePadding(int stride, int dilation, int in, int filter, int out);

// ---- glue-op tables: TFLite's formula evaluated for every 8-bit input byte.
// The device gathers from these (bh_lut_u8 / bh_lut_f32 / bh_softmax_i8), so
// all float and fixed-point rounding happens here, in the reference's order.

// common.h MultiplyByQuantizedMultiplier (double rounding; no
// TFLITE_SINGLE_ROUNDING)
int32_t MultiplyByQuantizedMultiplier(int32_t x, int32_t q, int shift);

// quantize.cc (8-bit -> 8-bit): QuantizeMultiplier(double(s_in)/double(s_out)),
// reference_ops::Requantize
void RequantizeTable(bool in_signed, float in_scale, int32_t in_zp, bool out_signed, float out_scale,
                     int32_t out_zp, uint8_t table[256]);
// activations.cc ReluPrepare + QuantizedReluX + ReluX; act_max_inf = RELU
void ReluTable(bool is_signed, float in_scale, int32_t in_zp, float out_scale, int32_t out_zp, float act_min,
               float act_max, bool act_max_inf, uint8_t table[256]);
// activations.cc PopulateLookupTable<T> with 1 / (1 + exp(-x))
void LogisticTable(bool is_signed, float in_scale, int32_t in_zp, float out_scale, int32_t out_zp,
                   uint8_t table[256]);
// activations.cc HardSwishPrepare (16-bit fixed-point multipliers) +
// reference_ops::HardSwish<T> evaluated for every input byte; false when
// TFLite's Prepare would refuse the scales (output exponent > 0)
bool HardSwishTable(bool is_signed, float in_scale, int32_t in_zp, float out_scale, int32_t out_zp,
                    uint8_t table[256]);
// reference_ops::Dequantize: float(double(scale) * (q - zp))
void DequantizeTable(bool is_signed, float scale, int32_t zp, float table[256]);
// concatenation.cc ConcatenationWithScaling (uint8): round(q*s + b) + zp_out
void ConcatRescaleTable(float in_scale, int32_t in_zp, float out_scale, int32_t out_zp, uint8_t table[256]);
// optimized_ops::PopulateSoftmaxLookupTable: table[255 - v] = expf(-s_in*beta*v)
void SoftmaxExpTable(float in_scale, float beta, float table[256]);
// reference_ops::ResizeNearestNeighbor GetNearestNeighbor
int NearestNeighborIndex(int v, int in_size, int out_size, bool align_corners, bool half_pixel_centers);
// reference_ops::ResizeBilinearInteger: per output row / column
// {lower, upper, 10-bit scaled coordinate}
// resize_bilinear.h ComputeInterpolationValues in float (the uint8 / float
// path): idx = {lower, upper} per output coordinate, frac = scaled - lower
void BilinearFloatTable(int in_size, int out_size, bool align_corners, bool half_pixel_centers,
                        std::vector<int32_t>* idx, std::vector<float>* frac);
void BilinearIntegerTable(int in_size, int out_size, bool align_corners, bool half_pixel_centers,
                          std::vector<int32_t>* tab);

}  // namespace hip
}  // namespace band
