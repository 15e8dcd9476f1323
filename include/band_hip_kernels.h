/*
 * band_hip_kernels.h — thin C ABI between the host-side HIP backend
 * (band_amd/csrc/backend/hip/) and the hand-written gfx950 kernels.
 *
 * This is the "Thin C ABI (build-internal)" of SURVEY.md §8(b): plain
 * pointers, sizes and POD parameter blocks, no C++ or torch types.  Every
 * entry point returns 0 on success or a hipError_t value (>0), or BH_EINVAL
 * (-1) for a parameter block that fails host-side validation.  Launch entry
 * points are asynchronous on the given stream (nullptr = the calling
 * thread's current-device null stream is NOT used: pass a real stream).
 *
 * Each op launcher stands in for one TFLite 2.9.2 builtin kernel that
 * `tflite::Interpreter::Invoke` dispatches from the reference hot path
 * `TfLiteModelExecutor::ExecuteSubgraph` (band/backend/tfl/model_executor.cc:249-255):
 *   bh_conv2d_i8      <- CONV_2D            (reference_integer_ops::ConvPerChannel,
 *                                            reference_ops::Conv uint8)
 *   bh_dwconv2d_i8    <- DEPTHWISE_CONV_2D  (reference_integer_ops::DepthwiseConvPerChannel)
 *   bh_fc_i8          <- FULLY_CONNECTED    (reference_integer_ops::FullyConnected)
 *   bh_eltwise_i8     <- ADD / SUB / MUL    (reference_integer_ops::Add / Mul, sub.cc)
 *   bh_pool_i8        <- AVERAGE_POOL_2D / MAX_POOL_2D (reference_integer_ops::{Average,Max}Pool)
 *   bh_irb_i8         <- [CONV_2D 1x1 ->] DEPTHWISE_CONV_2D 3x3 -> CONV_2D 1x1 [-> ADD], fused
 *   bh_chain_i8       <- DEPTHWISE_CONV_2D 3x3 -> CONV_2D 1x1 [-> ADD] [-> CONV_2D 1x1], fused
 *   bh_lut_u8         <- QUANTIZE (8-bit -> 8-bit), RELU / RELU6 / RELU_N1_TO_1, LOGISTIC
 *   bh_lut_f32        <- DEQUANTIZE (8-bit -> float32)
 *   bh_quantize_f32   <- QUANTIZE (float32 -> 8-bit, reference_ops::AffineQuantize)
 *   bh_concat         <- CONCATENATION      (reference_ops::Concatenation[WithScaling])
 *   bh_pad            <- PAD / PADV2        (reference_ops::Pad)
 *   bh_resize_nearest <- RESIZE_NEAREST_NEIGHBOR (reference_ops::ResizeNearestNeighbor)
 *   bh_resize_bilinear_i8 <- RESIZE_BILINEAR int8 (reference_ops::ResizeBilinearInteger)
 *   bh_resize_bilinear_u8 <- RESIZE_BILINEAR uint8 (optimized_ops::ResizeBilinear, float path)
 *   bh_softmax_i8     <- SOFTMAX 8-bit      (optimized_ops::Softmax, lookup-table path)
 *   bh_mean           <- MEAN               (optimized_integer_ops::Mean / optimized_ops::Mean)
 *   (HARD_SWISH 8-bit runs as a bh_lut_u8 table of reference_ops::HardSwish)
 *   bh_zero_insert + bh_conv2d_i8 <- TRANSPOSE_CONV int8 (reference_integer_ops::TransposeConv)
 *   bh_conv2d_f32 / bh_fc_f32 / bh_eltwise_f32 / bh_pool_f32 / bh_unary_f32 / bh_softmax_f32
 *                     <- the float32 forms of CONV_2D, DEPTHWISE_CONV_2D, FULLY_CONNECTED,
 *                        ADD/SUB/MUL, AVERAGE/MAX_POOL_2D, LOGISTIC/RELU*, SOFTMAX
 *                        (reference_ops float kernels) for fp16-weight models
 *
 * Quantised tensors live on the device as raw bytes in their TFLite type
 * (int8 or uint8).  Kernels work in the "int8 domain": a uint8 input is
 * mapped to int8 by XOR 0x80 on load (x - 128), and every zero point handed
 * to a kernel is already expressed in that domain.  Outputs are clamped to
 * [act_min, act_max] of the OUTPUT tensor's own type and stored as bytes, so
 * uint8 and int8 outputs are both bit-exact with TFLite.
 */
#ifndef BAND_HIP_KERNELS_H_
#define BAND_HIP_KERNELS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BH_EINVAL (-1)

typedef void* bh_stream_t;
typedef void* bh_graph_exec_t;
typedef void* bh_event_t;

/* ---- device / memory / stream (runtime plumbing) ------------------------ */
int bh_device_count(int* count);
int bh_set_device(int ordinal);
int bh_get_device(int* ordinal);
/* arch name of `ordinal` (e.g. "gfx950:sramecc+:xnack-"), NUL-terminated */
int bh_device_arch(int ordinal, char* buf, size_t cap);
/* PCI bus id of `ordinal` ("0000:75:00.0", hipDeviceGetPCIBusId), NUL-terminated; cap >= 13 */
int bh_device_pci_bus_id(int ordinal, char* buf, int cap);
int bh_stream_create(bh_stream_t* stream);
int bh_stream_destroy(bh_stream_t stream);
int bh_stream_sync(bh_stream_t stream);
/* 0 when all work on the stream is done, BH_ENOTREADY while some is not */
int bh_stream_query(bh_stream_t stream);
int bh_malloc(void** ptr, size_t bytes);
int bh_free(void* ptr);
int bh_host_alloc(void** ptr, size_t bytes); /* pinned, portable */
int bh_host_free(void* ptr);
int bh_memcpy_h2d_async(void* dst, const void* src, size_t bytes, bh_stream_t s);
int bh_memcpy_d2h_async(void* dst, const void* src, size_t bytes, bh_stream_t s);
int bh_memcpy_d2d_async(void* dst, const void* src, size_t bytes, bh_stream_t s);
/* the same copy as a kernel launch (bh_copy_kernel), not a runtime blit */
int bh_copy_d2d(void* dst, const void* src, size_t bytes, bh_stream_t s);
int bh_memset_async(void* dst, int value, size_t bytes, bh_stream_t s);
int bh_memcpy_h2d(void* dst, const void* src, size_t bytes);
int bh_memcpy_d2h(void* dst, const void* src, size_t bytes);

/* ---- stream capture -> hipGraph (one graph per prepared subgraph) ------- */
int bh_capture_begin(bh_stream_t s);
int bh_capture_end(bh_stream_t s, bh_graph_exec_t* exec);
int bh_graph_launch(bh_graph_exec_t exec, bh_stream_t s);
/* capture end that also returns the captured graph (free: bh_graph_free),
 * whose memcpy nodes bh_graph_memcpy_nodes lists (handle, dst, src, bytes;
 * up to max, *n = the count) and bh_graph_exec_set_memcpy retargets in the
 * instance (a 1-D host<->device copy of the same size) */
int bh_capture_end_keep(bh_stream_t s, bh_graph_exec_t* exec, void** graph);
int bh_graph_free(void* graph);
int bh_graph_memcpy_nodes(void* graph, void** nodes, void** dsts, const void** srcs, size_t* bytes, int max, int* n);
int bh_graph_exec_set_memcpy(bh_graph_exec_t exec, void* node, void* dst, const void* src, size_t bytes, int h2d);
int bh_graph_destroy(bh_graph_exec_t exec);

/* ---- events (timing) ---------------------------------------------------- */
int bh_event_create(bh_event_t* ev);
/* an event whose bh_event_sync sleeps until the GPU signals it (no
 * timing); replaces bh_stream_sync's spin-wait */
int bh_event_create_blocking(bh_event_t* ev);
/* an event with no timing whose waits spin (for bh_event_query polling) */
int bh_event_create_untimed(bh_event_t* ev);
int bh_event_destroy(bh_event_t ev);
int bh_event_record(bh_event_t ev, bh_stream_t s);
int bh_event_sync(bh_event_t ev);
/* 0 when the work before the event's record has finished, BH_ENOTREADY while
 * it is still running, else an error (non-blocking: hipEventQuery) */
#define BH_ENOTREADY (-2)
int bh_event_query(bh_event_t ev);
int bh_event_elapsed_ms(bh_event_t start, bh_event_t end, float* ms);
/* hold the stream for `us` microseconds (<= 100 ms): lets a profiler enqueue
 * a launch sequence before the GPU starts it, so events time execution */
int bh_spin_us(bh_stream_t s, int us);
/* one empty single-wave launch (profilers time chains of them to measure
 * the dispatch + gap an event pair adds around a real launch) */
int bh_empty_launch(bh_stream_t s);
/* this thread's next kernel launches carry dispatch timestamps: the first
 * kernel records `start` at its begin, every kernel records `stop` at its end
 * (hipExtLaunchKernel); bh_profile_events(NULL, NULL) turns it off.
 * Returns the number of kernels the previous setting timed. */
int bh_profile_events(bh_event_t start, bh_event_t stop);

/* ---- op parameter blocks ------------------------------------------------ */

/* CONV_2D.  Input NHWC [batch,in_h,in_w,in_c] bytes; output NHWC
 * [batch,out_h,out_w,out_c] bytes.  `weights` is the packed operand made by
 * bh_pack_conv_weights: int8-domain B^T [n_pad][k_pad] with
 * k = (ky*k_w + kx)*in_c + ci, zero padded.  bias_eff[c] already folds the
 * int32 bias and every zero-point cross term that does not depend on the
 * activations (see bh_pack_conv_weights); when w_zp != 0 (uint8 weights) the
 * kernel subtracts w_zp * sum_k x'[m][k] per output pixel. */
typedef struct bh_conv_params {
  int batch, in_h, in_w, in_c;
  int out_h, out_w, out_c;
  int k_h, k_w;
  int stride_h, stride_w, dil_h, dil_w;
  int pad_h, pad_w;               /* top / left padding (TFLite padding.h) */
  int k_pad, n_pad;               /* packed weight geometry */
  int in_xor;                     /* 0x80 when the input tensor is uint8 */
  int32_t in_zp;                  /* int8-domain input zero point (pad value) */
  int32_t w_zp;                   /* int8-domain weight zero point (0 if symmetric) */
  int32_t out_zp;                 /* output tensor zero point (own domain) */
  int32_t act_min, act_max;       /* output tensor domain */
  const void* input;
  void* output;
  const int8_t* weights;
  const int32_t* bias_eff;        /* [out_c] */
  const int32_t* mult;            /* [out_c] Q31 multipliers */
  const int32_t* shift;           /* [out_c] TFLite exponent (>0 = left) */
  /* Optional fused residual ADD (TFLite ADD applied to this conv's
   * requantised 8-bit output y and `residual`, same shape as the output):
   *   out = ADD(y, residual) with add.cc's left_shift-20 arithmetic.
   * Enabled when residual != NULL; y itself is then never stored. */
  const void* residual;
  int32_t add_y_off, add_r_off, add_o_off;    /* negated zps of y / residual, output zp */
  int32_t add_left_shift;
  int32_t add_y_mult, add_y_shift, add_r_mult, add_r_shift, add_o_mult, add_o_shift;
  int32_t add_act_min, add_act_max;
  /* optional 256-entry byte table applied to every stored output byte: a
   * following 8-bit unary op (QUANTIZE / RELU family / LOGISTIC) folded into
   * this epilogue (NULL = none) */
  const void* out_table;
  /* 1 when bh_conv_requant_fast_ok() holds for this layer's multipliers:
   * the kernels may then evaluate TFLite's two-step requantisation with one
   * 64-bit multiply-add and shifts (same results, fewer instructions) */
  int32_t requant_fast;
  /* kernel choice: BH_CONV_AUTO (by shape), or force one form where the
   * layer allows it (parity tests cover every form; A-B timing) */
  int32_t kernel_hint;
  /* 0: dense NHWC output.  Else output image n starts at output +
   * n * out_img_stride bytes (its out_h*out_w*out_c bytes contiguous): the
   * conv writes its slice of a CONCATENATION along a non-batch axis directly
   * (the concat launch is elided).  Such a layer runs conv_mfma_kernel. */
  int64_t out_img_stride;
} bh_conv_params;

/* Grouped launch of independent CONV_2D layers that each route to the
 * general MFMA kernel (bh_conv_group_ok): one dispatch runs every member's
 * workgroups (conv_group_kernel), each member computing exactly what its own
 * bh_conv2d_i8 launch would.  The members must not read each other's
 * outputs, and share one window type (all 1x1 unpadded, or none).
 * bh_conv_group_plan fills `host_table` (bh_conv_group_table_bytes(n)
 * bytes, n <= 32) and *g; the caller copies the table to device memory and
 * sets g->table before bh_conv_group_i8. */
typedef struct bh_conv_group {
  int n, blocks, is1x1;
  const void* table; /* device copy of the member table */
} bh_conv_group;
int bh_conv_group_ok(const bh_conv_params* p);
size_t bh_conv_group_table_bytes(int n);
int bh_conv_group_plan(const bh_conv_params* members, int n, void* host_table, bh_conv_group* g);
int bh_conv_group_i8(const bh_conv_group* g, bh_stream_t stream);
#define BH_CONV_AUTO 0
#define BH_CONV_MFMA 1 /* conv_mfma_kernel: per-wave fragments from L2, split-K deep layers */
#define BH_CONV_GEMM 2 /* conv_gemm_kernel: LDS-staged GEMM (1x1 s1, int8 in, symmetric filters) */
#define BH_CONV_GEMM_BIG 3 /* conv_gemm_big_kernel: 256-row tiles on 32x32x32 MFMA (same layers, large M) */
#define BH_CONV_STEM_VALU 4 /* RGB stems: conv_stem_kernel (VALU dot4) instead of conv_stem_mfma_kernel */
#define BH_CONV_STEM_MFMA 5 /* RGB stems: conv_stem_mfma_kernel (the routed form wherever its shape rules allow) */
#define BH_CONV_STEM_SCALAR 6 /* RGB stems: conv_stem_kernel with filters read through the scalar cache (round-4 form) */
/* the tile configuration conv_gemm_big_kernel takes for an M x N layer when
 * routed automatically (1: 256x256, 2: 256x128; BH_GEMM_BIG_CFG overrides),
 * 0 when the layer is too small for it (conv_gemm_kernel then) */
int bh_conv_gemm_big_config(long M, int N);

/* DEPTHWISE_CONV_2D.  weights: int8-domain [k_h][k_w][out_c] (TFLite layout
 * [1,kh,kw,oc] with XOR applied for uint8 filters).  Exact int32 math
 * (x'-in_zp)*(w'-w_zp) per tap, taps outside the image skipped. */
typedef struct bh_dwconv_params {
  int batch, in_h, in_w, in_c;
  int out_h, out_w, out_c, depth_multiplier;
  int k_h, k_w;
  int stride_h, stride_w, dil_h, dil_w;
  int pad_h, pad_w;
  int in_xor;
  int32_t in_zp, w_zp, out_zp;
  int32_t act_min, act_max;
  const void* input;
  void* output;
  const int8_t* weights;
  const int32_t* bias;            /* [out_c] raw int32 bias (zeros if absent) */
  const int32_t* mult;
  const int32_t* shift;
  /* optional 256-entry byte table applied to every stored output byte: a
   * following 8-bit unary op (QUANTIZE / RELU family / LOGISTIC) folded into
   * this epilogue (NULL = none) */
  const void* out_table;
  /* optional [out_c][4] int32 tap table from bh_pack_dw_taps (3x3, depth
   * multiplier 1, out_c % 4 == 0): the dot4 kernel then replaces the
   * per-tap one (weights / bias are not read).  NULL = per-tap kernel */
  const int32_t* taps;
  /* 1 when bh_conv_requant_fast_ok(mult, shift, out_c, 9, max|bias|) holds */
  int32_t requant_fast;
  /* kernel choice: BH_DW_AUTO (by shape), or force one form where the
   * shape allows it (parity tests cover every form; A-B timing) */
  int32_t kernel_hint;
} bh_dwconv_params;
#define BH_DW_AUTO 0
#define BH_DW_RUN 1   /* dwconv3x3_run_kernel: 4 pixels x 4 channels per thread */
#define BH_DW_DOT 2   /* dwconv3x3_dot_kernel: one pixel per thread */
#define BH_DW_MFMA 3  /* dwconv3x3_mfma_kernel: block-diagonal MFMA, C % 16 == 0 */

/* FULLY_CONNECTED.  input [rows][depth] bytes, weights int8-domain
 * [units][depth_pad] (depth_pad multiple of 16, zero padded); bias_eff as
 * for conv (folds bias - in_zp*sum(w') + depth*in_zp*w_zp). */
typedef struct bh_fc_params {
  int rows, depth, depth_pad, units;
  int in_xor;
  int32_t in_zp, w_zp, out_zp;
  int32_t act_min, act_max;
  const void* input;
  void* output;
  const int8_t* weights;
  const int32_t* bias_eff;
  const int32_t* mult;            /* [units] */
  const int32_t* shift;
  /* optional 256-entry byte table applied to every stored output byte: a
   * following 8-bit unary op (QUANTIZE / RELU family / LOGISTIC) folded into
   * this epilogue (NULL = none) */
  const void* out_table;
} bh_fc_params;

/* ADD / SUB / MUL with TFLite 4-D broadcasting.  Shapes are extended to 4-D
 * (leading 1s); a dimension of 1 in an input broadcasts.  Offsets are the
 * NEGATED zero points in each tensor's own domain (TFLite input*_offset). */
#define BH_ELT_ADD 0
#define BH_ELT_MUL 1
typedef struct bh_eltwise_params {
  int kind;                       /* BH_ELT_ADD (also SUB) or BH_ELT_MUL */
  int in_signed;                  /* 1 int8, 0 uint8 (both inputs, output) */
  int shape_a[4], shape_b[4], shape_o[4];
  int32_t a_off, b_off, o_off;
  int32_t left_shift;             /* ADD: 20 */
  int32_t a_mult, a_shift;        /* ADD: input1 (shift <= 0) */
  int32_t b_mult, b_shift;        /* ADD: input2 (negated mult for SUB) */
  int32_t o_mult, o_shift;        /* ADD: output; MUL: the only multiplier */
  int32_t act_min, act_max;
  const void* a;
  const void* b;
  void* out;
} bh_eltwise_params;

/* AVERAGE_POOL_2D / MAX_POOL_2D (no rescale: in/out share scale). */
#define BH_POOL_AVG 0
#define BH_POOL_MAX 1
typedef struct bh_pool_params {
  int kind;
  int in_signed;
  int batch, in_h, in_w, channels;
  int out_h, out_w;
  int f_h, f_w, stride_h, stride_w, pad_h, pad_w;
  int32_t act_min, act_max;
  const void* input;
  void* output;
} bh_pool_params;

/* Fused MobileNet inverted-residual block (int8 per-channel models):
 *   [CONV_2D 1x1 expand ->] DEPTHWISE_CONV_2D 3x3 -> CONV_2D 1x1 project [-> ADD x]
 * exactly as the 3-4 TFLite ops compute it (each intermediate is requantised
 * to its own 8-bit tensor), but one launch: a workgroup owns a tile of
 * output pixels, stages the input region (tile + halo) in LDS, computes the
 * expanded activation for the region into LDS (MFMA), the depthwise output
 * into LDS (VALU), then the projection (MFMA) + residual epilogue to HBM.
 * Intermediates never touch HBM. */
typedef struct bh_irb_params {
  int batch, in_h, in_w, in_c;        /* x: NHWC int8 */
  int exp_c;                          /* expanded channels (== in_c when no expand) */
  int out_h, out_w, out_c;            /* y: NHWC int8 */
  int stride, pad_h, pad_w;           /* depthwise 3x3 */
  int has_expand;
  int tile_h, tile_w;                 /* output pixels per workgroup */
  /* expand 1x1 (packed like bh_pack_conv_weights: [n_pad][k_pad]) */
  const int8_t* exp_w; int exp_k_pad;
  const int32_t* exp_bias_eff; const int32_t* exp_mult; const int32_t* exp_shift;
  int32_t x_zp;                       /* x zero point */
  int32_t e_zp, e_act_min, e_act_max; /* expanded tensor quantisation */
  /* depthwise [3][3][exp_c] */
  const int8_t* dw_w;
  const int32_t* dw_bias; const int32_t* dw_mult; const int32_t* dw_shift;
  int32_t d_zp, d_act_min, d_act_max;
  /* project 1x1 ([n_pad][k_pad], bias_eff folds d_zp) */
  const int8_t* proj_w; int proj_k_pad;
  const int32_t* proj_bias_eff; const int32_t* proj_mult; const int32_t* proj_shift;
  int32_t p_zp, p_act_min, p_act_max;
  /* optional residual ADD(p, x) (has_residual: stride 1, in_c == out_c) */
  int has_residual;
  int32_t add_p_off, add_x_off, add_o_off, add_left_shift;
  int32_t add_p_mult, add_p_shift, add_x_mult, add_x_shift, add_o_mult, add_o_shift;
  int32_t add_act_min, add_act_max;
  const void* input;
  void* output;
  /* diagnostics: when non-NULL, wave 0 of each workgroup writes 8 uint64
   * s_memrealtime stamps (100 MHz) at phase boundaries to
   * debug_stamps[16 * workgroup] (slots 0-7 used); NULL in production */
  void* debug_stamps;
  /* single-step requantisation allowed (bh_conv_requant_fast_ok) per stage:
   * bit 0 expand, bit 1 depthwise, bit 2 project */
  int32_t requant_fast;
} bh_irb_params;

/* LDS bytes one workgroup of bh_irb_i8 needs for a tile (0 if unsupported) */
size_t bh_irb_lds_bytes(const bh_irb_params* p);
int bh_irb_i8(const bh_irb_params* p, bh_stream_t s);

/* Fused pointwise chain across a block boundary (int8 per-channel models):
 *   DEPTHWISE_CONV_2D 3x3 -> CONV_2D 1x1 [-> ADD residual] [-> CONV_2D 1x1]
 * i.e. a MobileNetV2 block's depthwise + project (+ its residual ADD) and the
 * NEXT block's expand, or a MobileNetV1 depthwise + pointwise pair, exactly
 * as the 2-3 TFLite ops compute them (every intermediate requantised to its
 * own 8-bit tensor), in one launch.  No halo recompute: the 1x1 layers map
 * pixel m to pixel m, so a workgroup owns px_blocks x 16 consecutive output
 * pixels, computes their depthwise output for every channel into LDS
 * (block-diagonal MFMA), the first 1x1 GEMM from LDS (MFMA) with its
 * residual epilogue, and the second 1x1 GEMM from that result in LDS.
 * Parameter blocks are the unfused launches' own (same packed operands):
 *   dw.output and pw1.input are ignored (the depthwise result stays in LDS);
 *   pw1.output may be NULL (the block output is private to pw2) or the
 *   tensor to store; pw2 is read only when has_pw2.
 * Supported: dw 3x3, depth multiplier 1, tap table, out_c % 16 == 0, any
 * stride / dilation; all stages int8 in / symmetric filters (in_xor == 0,
 * w_zp == 0), no out_table; pw1 / pw2 1x1 stride 1 with out_c % 4 == 0;
 * pw2 without residual and with K = pw1.out_c <= 320.  px_blocks in {1, 2, 4};
 * 16 waves (px_blocks 1) spread few-pixel layers' channel work wider. */
typedef struct bh_chain_params {
  bh_dwconv_params dw;
  bh_conv_params pw1;
  bh_conv_params pw2;
  int has_pw2;
  int px_blocks;
  int waves;  /* waves per workgroup: 4 (0 = 4), or 8 / 16 with px_blocks == 1 */
  /* 1: persistent form - both 1x1 filters, the depthwise filter and all
   * tables staged in LDS once per workgroup, which then walks a contiguous
   * range of 64-pixel blocks (px_blocks 4, 4 waves; filters must fit LDS) */
  int persist;
  /* 1: 2-D tile form (chain_tile_kernel) - a workgroup owns an 8 x 8 tile of
   * output pixels and stages its depthwise input patch (tile + halo), the
   * residual tile, both 1x1 filters and every table in LDS with one burst of
   * LDS-DMA; stride / dilation 1 or 2, pw2 K <= 320.  px_blocks, waves and
   * persist are ignored.  3 / 4: runs of 2 / 4 consecutive tiles per
   * workgroup through ONE buffer (the constant block staged once per run) */
  int tile;
  /* tile form: the chain's constant block (both 1x1 filters swizzled for
   * LDS, every table, the depthwise filter) built once by
   * bh_chain_tile_pack into bh_chain_tile_blob_bytes() of device memory */
  const void* tile_blob;
  /* tile form, diagnostics: when non-NULL each workgroup writes 8 shader-
   * clock stamps (s_memtime) at its phase boundaries to
   * debug_stamps[8 * workgroup]; NULL in production */
  void* debug_stamps;
  /* 1: deep-issue form - each wave issues the loads of 6 depthwise channel
   * groups per round (instead of 2) and the x-stationary 1x1 GEMMs take 3-6
   * channel tiles per round; px_blocks 1 (4 or 8 waves) or 2 (4 waves) */
  int deep;
  /* raster forms with a second 1x1 (0 / 1: off): the second 1x1's channel
   * tiles are split over c_split workgroups per pixel block (grid.y); each
   * recomputes the depthwise and first 1x1 for its pixels and stores its
   * channel slice - more, shorter workgroups for the few-pixel 14x14 / 7x7
   * layers.  2..4 */
  int c_split;
  /* 1: raster form with staged filters (chain_stage_kernel) - a workgroup of
   * px_blocks (1 / 2) x 16 pixels and `waves` (4 / 8) waves starts with one
   * burst of LDS-DMA of the first 1x1's filter and tables, its c_split slice
   * (0 / 1 .. 8, grid.y) of the second 1x1's and the residual rows from
   * tile_blob (bh_chain_tile_pack), runs the depthwise from global memory
   * and both 1x1 GEMMs from LDS; has_pw2 only, pw2 K <= 320.  2: the same
   * with the burst issued by the upper half of the waves while the lower
   * half runs the depthwise phase */
  int stage;
} bh_chain_params;

/* LDS bytes one workgroup of bh_chain_i8 needs (0 if unsupported) */
size_t bh_chain_lds_bytes(const bh_chain_params* p);
/* the stage form's share of bh_chain_lds_bytes / bh_chain_i8 (stage != 0) */
size_t bh_chain_stage_lds_bytes(const bh_chain_params* p);
int bh_chain_stage_launch(const bh_chain_params* p, bh_stream_t s);
/* the tile form's share of bh_chain_lds_bytes / bh_chain_i8 (tile != 0) */
size_t bh_chain_tile_lds_bytes(const bh_chain_params* p);
int bh_chain_tile_launch(const bh_chain_params* p, bh_stream_t s);
/* the tile / stage forms' constant block: its size for these parameters (as
 * if tile == 1, or for the stage form when stage != 0; 0 if the form does not
 * apply) and a device pass that builds it from the params' filter / table
 * pointers into `blob` */
size_t bh_chain_tile_blob_bytes(const bh_chain_params* p);
int bh_chain_tile_pack(const bh_chain_params* p, void* blob, bh_stream_t s);
int bh_chain_i8(const bh_chain_params* p, bh_stream_t s);

/* MEAN over one contiguous run of axes (TFLite 2.9.2 reduce.cc EvalMean ->
 * optimized_integer_ops::Mean int8 / optimized_ops::Mean uint8 / float):
 * the input viewed as [outer][reduce][inner]; out[o][i] = for 8-bit types
 * clamp(MultiplyByQuantizedMultiplier(sum_r x, multiplier, shift) + bias),
 * for float32 (sum_r x in order) / reduce.  One thread per output. */
typedef struct bh_mean_params {
  long outer, reduce, inner;
  int type;                       /* 0 float32, 1 int8, 2 uint8 */
  int32_t multiplier, shift, bias;
  const void* input;
  void* output;
} bh_mean_params;
int bh_mean(const bh_mean_params* p, bh_stream_t s);

/* ---- host-side operand packing (pure CPU, no device calls) -------------- */

/* Pack OHWI conv weights ([out_c][k_h*k_w*in_c] bytes, signed or unsigned)
 * into the int8-domain padded B^T operand and compute bias_eff:
 *   bias_eff[c] = bias[c] - in_zp*S_c + K*in_zp*w_zp,  S_c = sum_k w'[c][k]
 * where w' = w (int8) or w-128 (uint8) and in_zp/w_zp are int8-domain.
 * packed must hold n_pad*k_pad bytes; bias may be NULL. */
int bh_pack_conv_weights(const void* w, int w_signed, int out_c, int k,
                         int k_pad, int n_pad, const int32_t* bias,
                         int32_t in_zp, int32_t w_zp, int8_t* packed,
                         int32_t* bias_eff);

/* Tile geometry the conv launcher expects for a layer (k_pad, n_pad). */
int bh_conv_packed_geometry(int out_c, int k, int* k_pad, int* n_pad);
/* DEPTHWISE_CONV_2D 3x3 / depth multiplier 1 tap table: for channel c,
 * taps[4c..4c+3] = {w[0..3][c] as bytes, w[4..7][c] as bytes,
 * w[8][c] << 8*(c%4), bias[c] - in_zp*sum_t w[t][c] + 9*in_zp*w_zp}.
 * w: int8-domain [9][c]; in_zp / w_zp int8-domain; c % 4 == 0. */
int bh_pack_dw_taps(const int8_t* w, int c, const int32_t* bias, int32_t in_zp, int32_t w_zp, int32_t* taps);
/* Whether a conv layer may use the single-step requantisation identity
 *   rdbypot(srdhm(x, M), e) + zp == (((x*M + c0) >> 31) + s + (zp << e)) >> e
 *   c0 = 2^30 + (e > 0 ? 2^(30+e) : 0),  s = (e > 0 && x < 0) ? -1 : 0
 * (TFLite MultiplyByQuantizedMultiplier with shift = -e <= 0).  Holds when
 * every multiplier is in (2^30, 2^31), every shift <= 0 and the int32
 * accumulators are small enough that nothing overflows:
 *   K * 2^16 + max|bias| + 255 * 2^e < 2^30.  Returns 1 / 0. */
int bh_conv_requant_fast_ok(const int32_t* mult, const int32_t* shift, int n, int k, int64_t max_abs_bias);

/* ---- launchers ---------------------------------------------------------- */
int bh_conv2d_i8(const bh_conv_params* p, bh_stream_t s);
/* Symbol of the kernel bh_conv2d_i8 dispatches these parameters to
 * ("conv_mfma_kernel", "conv_xs_kernel", "conv_rows_kernel",
 * "conv_direct_kernel"); static storage.  Profiling attribution only. */
const char* bh_conv2d_i8_kernel(const bh_conv_params* p);
int bh_dwconv2d_i8(const bh_dwconv_params* p, bh_stream_t s);
/* Symbol of the kernel bh_dwconv2d_i8 dispatches these parameters to
 * ("dwconv3x3_run_kernel", "dwconv3x3_dot_kernel", "dwconv3x3_kernel",
 * "dwconv_generic_kernel"); static storage.  Profiling attribution only. */
const char* bh_dwconv2d_i8_kernel(const bh_dwconv_params* p);
int bh_fc_i8(const bh_fc_params* p, bh_stream_t s);
int bh_eltwise_i8(const bh_eltwise_params* p, bh_stream_t s);
int bh_pool_i8(const bh_pool_params* p, bh_stream_t s);

/* ---- glue ops (whole-model residency) ------------- */

/* out[i] = table[in[i]]: every 8-bit unary op whose result depends only on
 * the input byte.  The host fills the 256-entry device table (indexed by the
 * raw byte) with TFLite's own formula: QUANTIZE between 8-bit types
 * (Requantize), RELU / RELU6 / RELU_N1_TO_1 (ReluX), LOGISTIC (the 8-bit
 * lookup table of activations.cc).  bh_lut_f32: 256 float entries
 * (DEQUANTIZE: float(double(scale) * (q - zp))). */
int bh_lut_u8(const void* in, void* out, long n, const void* table, bh_stream_t s);
int bh_lut_f32(const void* in, void* out, long n, const float* table, bh_stream_t s);
/* float32 -> 8-bit: clamp((int)roundf(x / scale) + zp) */
int bh_quantize_f32(const float* in, void* out, long n, float scale, int32_t zp, int out_signed,
                    bh_stream_t s);

/* ---- float32 graphs ------------------------------------------------------
 * TFLite fp16 models (post-training float16 quantization) compute in float32
 * with fp16 constant weights behind DEQUANTIZE ops; the host folds those
 * DEQUANTIZEs and hands these kernels float32 operands.  Float results match
 * the reference within a stated tolerance (summation order differs), not
 * bit-exactly.  act_min / act_max are the fused activation's float bounds
 * (+-inf for NONE). */
typedef struct {
  int batch, in_h, in_w, in_c, out_h, out_w, out_c, k_h, k_w;
  int stride_h, stride_w, dil_h, dil_w, pad_h, pad_w;
  int depthwise, depth_multiplier;   /* depthwise: out_c = in_c * depth_multiplier */
  float act_min, act_max;
  const float* input;
  float* output;
  const float* weights; /* conv: [k_h*k_w*in_c][out_c]; depthwise: [k_h*k_w][out_c] */
  const float* bias;    /* [out_c] or NULL */
} bh_conv_f32_params;
int bh_conv2d_f32(const bh_conv_f32_params* p, bh_stream_t s);

typedef struct {
  int rows, depth, units;
  float act_min, act_max;
  const float* input;   /* [rows][depth] */
  float* output;        /* [rows][units] */
  const float* weights; /* [units][depth] */
  const float* bias;    /* [units] or NULL */
} bh_fc_f32_params;
int bh_fc_f32(const bh_fc_f32_params* p, bh_stream_t s);

#define BH_ELTF_ADD 0
#define BH_ELTF_SUB 1
#define BH_ELTF_MUL 2
#define BH_ELTF_SQDIFF 3 /* SQUARED_DIFFERENCE: (a - b)^2 */
typedef struct {
  int kind;
  int shape_a[4], shape_b[4], shape_o[4]; /* 4-D, broadcast dims are 1 */
  float act_min, act_max;
  const float* a;
  const float* b;
  float* out;
} bh_eltwise_f32_params;
int bh_eltwise_f32(const bh_eltwise_f32_params* p, bh_stream_t s);

typedef struct {
  int kind; /* BH_POOL_AVG / BH_POOL_MAX */
  int batch, in_h, in_w, channels, out_h, out_w, f_h, f_w, stride_h, stride_w, pad_h, pad_w;
  float act_min, act_max;
  const float* input;
  float* output;
} bh_pool_f32_params;
int bh_pool_f32(const bh_pool_f32_params* p, bh_stream_t s);

#define BH_UNARY_CLAMP 0    /* RELU / RELU6 / RELU_N1_TO_1: min(max(x, lo), hi) */
#define BH_UNARY_LOGISTIC 1 /* 1 / (1 + exp(-x)) */
#define BH_UNARY_RSQRT 2    /* RSQRT: 1 / sqrt(x) */
int bh_unary_f32(int kind, const float* in, float* out, long n, float lo, float hi, bh_stream_t s);

/* reference_ops::Softmax (float): per row exp((x - max) * beta) / sum */
int bh_softmax_f32(const float* in, float* out, long rows, int depth, float beta, bh_stream_t s);

#define BH_CONCAT_MAX_INPUTS 16
typedef struct {
  int n_inputs;
  long outer;                              /* product of the dims before the axis */
  long row[BH_CONCAT_MAX_INPUTS];          /* bytes per outer index of input k */
  const void* input[BH_CONCAT_MAX_INPUTS];
  const void* table[BH_CONCAT_MAX_INPUTS]; /* optional 256-B rescale table (uint8
                                              ConcatenationWithScaling), NULL = copy */
  void* output;                            /* row of outer index o: sum_k row[k] bytes */
} bh_concat_params;
int bh_concat(const bh_concat_params* p, bh_stream_t s);

typedef struct {
  int elem_bytes;                 /* 1 or 4 */
  int in_shape[4];                /* NHWC (lower ranks padded with leading 1s) */
  int pad_before[4], pad_after[4];
  uint32_t value;                 /* bit pattern of the pad element */
  const void* input;
  void* output;
  /* 0: constant fill (PAD / PADV2); MIRROR_PAD: 1 REFLECT, 2 SYMMETRIC
   * (mirror_pad.cc GetInputDimension; pads < dim for REFLECT, <= dim) */
  int32_t mode;
} bh_pad_params;
int bh_pad(const bh_pad_params* p, bh_stream_t s);

typedef struct {
  int batch, in_h, in_w, out_h, out_w;
  int row_bytes;                  /* channels * element bytes */
  const int32_t* y_index;         /* [out_h] source row (host-computed, TFLite float formula) */
  const int32_t* x_index;         /* [out_w] source column */
  const void* input;
  void* output;
} bh_resize_nearest_params;
int bh_resize_nearest(const bh_resize_nearest_params* p, bh_stream_t s);

typedef struct {
  int batch, in_h, in_w, channels, out_h, out_w;
  const int32_t* y_tab;           /* [out_h][3]: lower row, upper row, 10-bit scaled y */
  const int32_t* x_tab;           /* [out_w][3] */
  const void* input;              /* int8 */
  void* output;
} bh_resize_bilinear_params;
int bh_resize_bilinear_i8(const bh_resize_bilinear_params* p, bh_stream_t s);

/* RESIZE_BILINEAR uint8 (TFLite 2.9.2 optimized_ops::ResizeBilinear for
 * uint8 -> ResizeBilinearGenericSmallChannel<uint8>): float interpolation.
 * Host tables from ComputeInterpolationValues (float scale, floor / ceil):
 * y_idx [2*out_h] = {y0, y1}, y_frac [out_h] = input_y - y0 (float), same
 * for x.  Per output byte, in float with no contraction:
 *   (uint8)(v00*(1-dy)(1-dx) + v01*(1-dy)dx + v10*dy(1-dx) + v11*dy*dx + 0.5f)
 * summed left to right as the reference's expression. */
typedef struct {
  int batch, in_h, in_w, channels, out_h, out_w;
  const int32_t* y_idx;
  const int32_t* x_idx;
  const float* y_frac;
  const float* x_frac;
  const void* input;
  void* output;
} bh_resize_bilinear_u8_params;
int bh_resize_bilinear_u8(const bh_resize_bilinear_u8_params* p, bh_stream_t s);

typedef struct {
  long rows;
  int depth;                      /* softmax over the last dim */
  int is_signed;                  /* int8 (1) or uint8 (0), input and output */
  const float* table;             /* [256] device: table[255 - v] = expf(-in_scale * beta * v) */
  float out_scale;
  int32_t out_zp;
  const void* input;
  void* output;
} bh_softmax_params;
int bh_softmax_i8(const bh_softmax_params* p, bh_stream_t s);

/* TRANSPOSE_CONV support: U[y*sh][x*sw][:] = in[y][x][:], every other
 * position of U (out_h x out_w = (in-1)*stride+1) holds `fill` (the input
 * zero point, so it contributes 0).  A transpose conv is then a stride-1
 * CONV_2D over U with spatially flipped filters and padding k-1-pad. */
typedef struct {
  int batch, in_h, in_w, channels, stride_h, stride_w, out_h, out_w;
  uint32_t fill;                  /* byte */
  const void* input;
  void* output;
} bh_zero_insert_params;
int bh_zero_insert(const bh_zero_insert_params* p, bh_stream_t s);

/* human-readable name of the last error set on this thread */
const char* bh_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* BAND_HIP_KERNELS_H_ */
