// Host execution of the lowered launch program for kCPU workers.
//
// Band runs a model on a CPU worker when the configuration has one (C1:
// MobileNetV1 on 1 CPU worker) and places the ops the GPU cannot run on it
// when the model analyzer splits a model (band/model_analyzer.cc:484-606).
// A kCPU HipModelExecutor lowers its subgraph exactly as a kGPU one does
// (same packed operands, folded biases, requantisation tables and epilogue
// fusions, all in host memory) and runs every launch here, with the
// TFLite 2.9.2 integer arithmetic the HIP kernels implement.  This is the CPU
// *device* of the backend, not a fallback of the GPU path: a kGPU executor
// never calls into this file.
#pragma once

#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "band_hip_kernels.h"

namespace band {
namespace hip {

// A fixed pool of worker threads (the executor's num_threads; the calling
// thread is one of them) running ParallelFor over index ranges.  A non-empty
// `cpus` pins the pool's own threads to those CPUs (the executor's CpuSet).
class CpuPool {
 public:
  explicit CpuPool(int num_threads, const std::vector<int>& cpus = {});
  ~CpuPool();
  CpuPool(const CpuPool&) = delete;
  CpuPool& operator=(const CpuPool&) = delete;
  int size() const { return static_cast<int>(threads_.size()) + 1; }
  // fn(begin, end) over [0, n) split into contiguous chunks
  void ParallelFor(long n, const std::function<void(long, long)>& fn);

 private:
  void Loop(int id);
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(long, long)>* job_ = nullptr;
  long n_ = 0;
  int generation_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

// the launch kinds of model_executor.h with their host implementations
void CpuConv(const bh_conv_params& p, CpuPool& pool);
void CpuDwConv(const bh_dwconv_params& p, CpuPool& pool);
void CpuFc(const bh_fc_params& p, CpuPool& pool);
void CpuEltwise(const bh_eltwise_params& p, CpuPool& pool);
void CpuPool2D(const bh_pool_params& p, CpuPool& pool);
void CpuLutU8(const void* in, void* out, long n, const uint8_t* table, CpuPool& pool);
void CpuLutF32(const void* in, float* out, long n, const float* table, CpuPool& pool);
void CpuQuantizeF32(const float* in, void* out, long n, float scale, int32_t zp, int out_signed, CpuPool& pool);
void CpuConcat(const bh_concat_params& p);
void CpuPad(const bh_pad_params& p);
void CpuResizeNearest(const bh_resize_nearest_params& p);
void CpuResizeBilinear(const bh_resize_bilinear_params& p);
void CpuResizeBilinearU8(const bh_resize_bilinear_u8_params& p);
void CpuSoftmax(const bh_softmax_params& p);
void CpuZeroInsert(const bh_zero_insert_params& p);

// float32 graphs (the bh_*_f32 kernels' host forms)
void CpuConvF32(const bh_conv_f32_params& p, CpuPool& pool);
void CpuFcF32(const bh_fc_f32_params& p, CpuPool& pool);
void CpuEltwiseF32(const bh_eltwise_f32_params& p);
void CpuPoolF32(const bh_pool_f32_params& p);
void CpuUnaryF32(int kind, const float* in, float* out, long n, float lo, float hi);
void CpuSoftmaxF32(const float* in, float* out, long rows, int depth, float beta);

// TFLite_Detection_PostProcess (CUSTOM, detection_postprocess.cc): float
// inputs, fast class-agnostic NMS, one class per detection; CPU-only
struct CpuDetectionParams {
  int num_boxes, num_classes, num_classes_with_background, max_detections;
  float score_threshold, iou_threshold;
  float scale_y, scale_x, scale_h, scale_w;
  const float* box_encodings;  // [num_boxes, 4] (y, x, h, w)
  const float* class_scores;   // [num_boxes, num_classes_with_background]
  const float* anchors;        // [num_boxes, 4] (y, x, h, w)
  float* out_boxes;            // [max_detections, 4] (ymin, xmin, ymax, xmax)
  float* out_classes;          // [max_detections]
  float* out_scores;           // [max_detections]
  float* out_num;              // [1]
};
void CpuDetectionPostprocess(const CpuDetectionParams& p, CpuPool& pool);

// MEAN over a contiguous run of axes: the input viewed as [outer][reduce]
// [inner] and reduced over the middle.  Quantized (8-bit): TFLite 2.9.2
// optimized_integer_ops::Mean / optimized_ops::Mean (4-D, keep_dims, axes
// {1, 2}): acc = sum; MultiplyByQuantizedMultiplier(acc, multiplier, shift)
// + bias, clamped to the type's range.  Float: sum / count.
struct CpuMeanParams {
  long outer, reduce, inner;
  int type;  // 0 float32, 1 int8, 2 uint8
  int32_t multiplier, shift, bias;
  const void* input;
  void* output;
};
void CpuMean(const CpuMeanParams& p, CpuPool& pool);

}  // namespace hip
}  // namespace band
