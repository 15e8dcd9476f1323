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

}  // namespace hip
}  // namespace band
