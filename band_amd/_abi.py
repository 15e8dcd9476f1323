"""ctypes binding of the C ABI exported by band_amd/libband_hip.so.

Mirrors include/band_hip_kernels.h (kernel layer, `bh_*`) and
include/band_hip_backend.h (executor layer, `bhx_*`).  Loading fails loudly
when the library has not been built: there is no CPU fallback on the product
path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# BAND_HIP_LIB_VARIANT=x loads libband_hip_x.so instead: an in-tree build of
# the same sources with one compile-time switch flipped, for A-B timing
LIB_PATH = os.path.join(_HERE, "libband_hip%s.so" % (
    "_" + os.environ["BAND_HIP_LIB_VARIANT"] if os.environ.get("BAND_HIP_LIB_VARIANT") else ""))

c_int, c_int32, c_void_p, c_size_t = ctypes.c_int, ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t


class ConvParams(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "batch", "in_h", "in_w", "in_c", "out_h", "out_w", "out_c", "k_h", "k_w",
        "stride_h", "stride_w", "dil_h", "dil_w", "pad_h", "pad_w", "k_pad", "n_pad", "in_xor")] + [
        (n, c_int32) for n in ("in_zp", "w_zp", "out_zp", "act_min", "act_max")] + [
        (n, c_void_p) for n in ("input", "output", "weights", "bias_eff", "mult", "shift", "residual")] + [
        (n, c_int32) for n in ("add_y_off", "add_r_off", "add_o_off", "add_left_shift", "add_y_mult",
                               "add_y_shift", "add_r_mult", "add_r_shift", "add_o_mult", "add_o_shift",
                               "add_act_min", "add_act_max")] + [("out_table", c_void_p), ("requant_fast", c_int32),
                                                                  ("kernel_hint", c_int32),
                                                                  ("out_img_stride", ctypes.c_int64)]


class ConvGroup(ctypes.Structure):
    _fields_ = [("n", c_int), ("blocks", c_int), ("is1x1", c_int), ("table", c_void_p)]


class DwConvParams(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "batch", "in_h", "in_w", "in_c", "out_h", "out_w", "out_c", "depth_multiplier",
        "k_h", "k_w", "stride_h", "stride_w", "dil_h", "dil_w", "pad_h", "pad_w", "in_xor")] + [
        (n, c_int32) for n in ("in_zp", "w_zp", "out_zp", "act_min", "act_max")] + [
        (n, c_void_p) for n in ("input", "output", "weights", "bias", "mult", "shift", "out_table", "taps")] + [
        ("requant_fast", c_int32), ("kernel_hint", c_int32)]


class FcParams(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("rows", "depth", "depth_pad", "units", "in_xor")] + [
        (n, c_int32) for n in ("in_zp", "w_zp", "out_zp", "act_min", "act_max")] + [
        (n, c_void_p) for n in ("input", "output", "weights", "bias_eff", "mult", "shift", "out_table")]


class EltwiseParams(ctypes.Structure):
    _fields_ = [("kind", c_int), ("in_signed", c_int), ("shape_a", c_int * 4),
                ("shape_b", c_int * 4), ("shape_o", c_int * 4)] + [
        (n, c_int32) for n in ("a_off", "b_off", "o_off", "left_shift", "a_mult", "a_shift",
                               "b_mult", "b_shift", "o_mult", "o_shift", "act_min", "act_max")] + [
        (n, c_void_p) for n in ("a", "b", "out")]


class PoolParams(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "kind", "in_signed", "batch", "in_h", "in_w", "channels", "out_h", "out_w",
        "f_h", "f_w", "stride_h", "stride_w", "pad_h", "pad_w")] + [
        (n, c_int32) for n in ("act_min", "act_max")] + [
        (n, c_void_p) for n in ("input", "output")]


class IrbParams(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "batch", "in_h", "in_w", "in_c", "exp_c", "out_h", "out_w", "out_c", "stride", "pad_h", "pad_w",
        "has_expand", "tile_h", "tile_w")] + [
        ("exp_w", c_void_p), ("exp_k_pad", c_int), ("exp_bias_eff", c_void_p), ("exp_mult", c_void_p),
        ("exp_shift", c_void_p)] + [(n, c_int32) for n in ("x_zp", "e_zp", "e_act_min", "e_act_max")] + [
        ("dw_w", c_void_p), ("dw_bias", c_void_p), ("dw_mult", c_void_p), ("dw_shift", c_void_p)] + [
        (n, c_int32) for n in ("d_zp", "d_act_min", "d_act_max")] + [
        ("proj_w", c_void_p), ("proj_k_pad", c_int), ("proj_bias_eff", c_void_p), ("proj_mult", c_void_p),
        ("proj_shift", c_void_p)] + [(n, c_int32) for n in ("p_zp", "p_act_min", "p_act_max")] + [
        ("has_residual", c_int)] + [(n, c_int32) for n in (
            "add_p_off", "add_x_off", "add_o_off", "add_left_shift", "add_p_mult", "add_p_shift", "add_x_mult",
            "add_x_shift", "add_o_mult", "add_o_shift", "add_act_min", "add_act_max")] + [
        ("input", c_void_p), ("output", c_void_p), ("debug_stamps", c_void_p), ("requant_fast", c_int32)]


class MeanParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_long) for n in ("outer", "reduce", "inner")] + [("type", c_int)] + [
        (n, c_int32) for n in ("multiplier", "shift", "bias")] + [("input", c_void_p), ("output", c_void_p)]


class ChainParams(ctypes.Structure):
    _fields_ = [("dw", DwConvParams), ("pw1", ConvParams), ("pw2", ConvParams), ("has_pw2", c_int),
                ("px_blocks", c_int), ("waves", c_int), ("persist", c_int), ("tile", c_int),
                ("tile_blob", c_void_p), ("debug_stamps", c_void_p), ("deep", c_int), ("c_split", c_int),
                ("stage", c_int)]


# symbol -> (restype, argtypes)
CONCAT_MAX_INPUTS = 16


class ConcatParams(ctypes.Structure):
    _fields_ = [("n_inputs", c_int), ("outer", ctypes.c_long),
                ("row", ctypes.c_long * CONCAT_MAX_INPUTS), ("input", c_void_p * CONCAT_MAX_INPUTS),
                ("table", c_void_p * CONCAT_MAX_INPUTS), ("output", c_void_p)]


class PadParams(ctypes.Structure):
    _fields_ = [("elem_bytes", c_int), ("in_shape", c_int * 4), ("pad_before", c_int * 4),
                ("pad_after", c_int * 4), ("value", ctypes.c_uint32), ("input", c_void_p), ("output", c_void_p),
                ("mode", c_int32)]


class ResizeNearestParams(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("batch", "in_h", "in_w", "out_h", "out_w", "row_bytes")] + [
        (n, c_void_p) for n in ("y_index", "x_index", "input", "output")]


class ResizeBilinearParams(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("batch", "in_h", "in_w", "channels", "out_h", "out_w")] + [
        (n, c_void_p) for n in ("y_tab", "x_tab", "input", "output")]


class ResizeBilinearU8Params(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("batch", "in_h", "in_w", "channels", "out_h", "out_w")] + [
        (n, c_void_p) for n in ("y_idx", "x_idx", "y_frac", "x_frac", "input", "output")]


class SoftmaxParams(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_long), ("depth", c_int), ("is_signed", c_int), ("table", c_void_p),
                ("out_scale", ctypes.c_float), ("out_zp", c_int32), ("input", c_void_p), ("output", c_void_p)]


class ZeroInsertParams(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("batch", "in_h", "in_w", "channels", "stride_h", "stride_w", "out_h",
                                     "out_w")] + [("fill", ctypes.c_uint32), ("input", c_void_p), ("output", c_void_p)]


class ConvF32Params(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "batch", "in_h", "in_w", "in_c", "out_h", "out_w", "out_c", "k_h", "k_w", "stride_h", "stride_w",
        "dil_h", "dil_w", "pad_h", "pad_w", "depthwise", "depth_multiplier")] + [
        ("act_min", ctypes.c_float), ("act_max", ctypes.c_float)] + [
        (n, c_void_p) for n in ("input", "output", "weights", "bias")]


class FcF32Params(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("rows", "depth", "units")] + [
        ("act_min", ctypes.c_float), ("act_max", ctypes.c_float)] + [
        (n, c_void_p) for n in ("input", "output", "weights", "bias")]


class EltwiseF32Params(ctypes.Structure):
    _fields_ = [("kind", c_int), ("shape_a", c_int * 4), ("shape_b", c_int * 4), ("shape_o", c_int * 4),
                ("act_min", ctypes.c_float), ("act_max", ctypes.c_float)] + [(n, c_void_p) for n in ("a", "b", "out")]


class PoolF32Params(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "kind", "batch", "in_h", "in_w", "channels", "out_h", "out_w", "f_h", "f_w", "stride_h", "stride_w",
        "pad_h", "pad_w")] + [("act_min", ctypes.c_float), ("act_max", ctypes.c_float)] + [
        (n, c_void_p) for n in ("input", "output")]


KERNEL_SYMBOLS = {
    "bh_device_count": (c_int, [ctypes.POINTER(c_int)]),
    "bh_set_device": (c_int, [c_int]),
    "bh_get_device": (c_int, [ctypes.POINTER(c_int)]),
    "bh_device_arch": (c_int, [c_int, ctypes.c_char_p, c_size_t]),
    "bh_device_pci_bus_id": (c_int, [c_int, ctypes.c_char_p, c_int]),
    "bh_stream_create": (c_int, [ctypes.POINTER(c_void_p)]),
    "bh_stream_destroy": (c_int, [c_void_p]),
    "bh_stream_sync": (c_int, [c_void_p]),
    "bh_stream_query": (c_int, [c_void_p]),
    "bh_malloc": (c_int, [ctypes.POINTER(c_void_p), c_size_t]),
    "bh_free": (c_int, [c_void_p]),
    "bh_host_alloc": (c_int, [ctypes.POINTER(c_void_p), c_size_t]),
    "bh_host_free": (c_int, [c_void_p]),
    "bh_memcpy_h2d_async": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bh_memcpy_d2h_async": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bh_memcpy_d2d_async": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bh_copy_d2d": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bh_memset_async": (c_int, [c_void_p, c_int, c_size_t, c_void_p]),
    "bh_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_size_t]),
    "bh_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_size_t]),
    "bh_capture_begin": (c_int, [c_void_p]),
    "bh_capture_end": (c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    "bh_graph_launch": (c_int, [c_void_p, c_void_p]),
    "bh_graph_destroy": (c_int, [c_void_p]),
    "bh_event_create": (c_int, [ctypes.POINTER(c_void_p)]),
    "bh_event_create_blocking": (c_int, [ctypes.POINTER(c_void_p)]),
    "bh_capture_end_keep": (c_int, [c_void_p, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p)]),
    "bh_graph_free": (c_int, [c_void_p]),
    "bh_graph_memcpy_nodes": (c_int, [c_void_p, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p),
                                      ctypes.POINTER(c_void_p), ctypes.POINTER(c_size_t), c_int,
                                      ctypes.POINTER(c_int)]),
    "bh_graph_exec_set_memcpy": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int]),
    "bh_event_destroy": (c_int, [c_void_p]),
    "bh_event_record": (c_int, [c_void_p, c_void_p]),
    "bh_event_sync": (c_int, [c_void_p]),
    "bh_event_query": (c_int, [c_void_p]),
    "bh_event_create_untimed": (c_int, [ctypes.POINTER(c_void_p)]),
    "bh_event_elapsed_ms": (c_int, [c_void_p, c_void_p, ctypes.POINTER(ctypes.c_float)]),
    "bh_spin_us": (c_int, [c_void_p, c_int]),
    "bh_empty_launch": (c_int, [c_void_p]),
    "bh_profile_events": (c_int, [c_void_p, c_void_p]),
    "bh_pack_conv_weights": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                     c_int32, c_int32, c_void_p, c_void_p]),
    "bh_conv_packed_geometry": (c_int, [c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "bh_pack_dw_taps": (c_int, [c_void_p, c_int, c_void_p, c_int32, c_int32, c_void_p]),
    "bh_conv_requant_fast_ok": (c_int, [c_void_p, c_void_p, c_int, c_int, ctypes.c_int64]),
    "bh_conv2d_i8": (c_int, [ctypes.POINTER(ConvParams), c_void_p]),
    "bh_conv_group_ok": (c_int, [ctypes.POINTER(ConvParams)]),
    "bh_conv_group_table_bytes": (ctypes.c_size_t, [c_int]),
    "bh_conv_group_plan": (c_int, [ctypes.POINTER(ConvParams), c_int, c_void_p, ctypes.POINTER(ConvGroup)]),
    "bh_conv_group_i8": (c_int, [ctypes.POINTER(ConvGroup), c_void_p]),
    "bh_conv2d_i8_kernel": (ctypes.c_char_p, [ctypes.POINTER(ConvParams)]),
    "bh_conv_gemm_big_config": (ctypes.c_int, [ctypes.c_long, ctypes.c_int]),
    "bh_dwconv2d_i8_kernel": (ctypes.c_char_p, [ctypes.POINTER(DwConvParams)]),
    "bh_lut_u8": (c_int, [c_void_p, c_void_p, ctypes.c_long, c_void_p, c_void_p]),
    "bh_lut_f32": (c_int, [c_void_p, c_void_p, ctypes.c_long, c_void_p, c_void_p]),
    "bh_quantize_f32": (c_int, [c_void_p, c_void_p, ctypes.c_long, ctypes.c_float, c_int32, c_int, c_void_p]),
    "bh_concat": (c_int, [ctypes.POINTER(ConcatParams), c_void_p]),
    "bh_pad": (c_int, [ctypes.POINTER(PadParams), c_void_p]),
    "bh_resize_nearest": (c_int, [ctypes.POINTER(ResizeNearestParams), c_void_p]),
    "bh_resize_bilinear_i8": (c_int, [ctypes.POINTER(ResizeBilinearParams), c_void_p]),
    "bh_resize_bilinear_u8": (c_int, [ctypes.POINTER(ResizeBilinearU8Params), c_void_p]),
    "bh_softmax_i8": (c_int, [ctypes.POINTER(SoftmaxParams), c_void_p]),
    "bh_zero_insert": (c_int, [ctypes.POINTER(ZeroInsertParams), c_void_p]),
    "bh_conv2d_f32": (c_int, [ctypes.POINTER(ConvF32Params), c_void_p]),
    "bh_fc_f32": (c_int, [ctypes.POINTER(FcF32Params), c_void_p]),
    "bh_eltwise_f32": (c_int, [ctypes.POINTER(EltwiseF32Params), c_void_p]),
    "bh_pool_f32": (c_int, [ctypes.POINTER(PoolF32Params), c_void_p]),
    "bh_unary_f32": (c_int, [c_int, c_void_p, c_void_p, ctypes.c_long, ctypes.c_float, ctypes.c_float, c_void_p]),
    "bh_softmax_f32": (c_int, [c_void_p, c_void_p, ctypes.c_long, c_int, ctypes.c_float, c_void_p]),
    "bh_dwconv2d_i8": (c_int, [ctypes.POINTER(DwConvParams), c_void_p]),
    "bh_fc_i8": (c_int, [ctypes.POINTER(FcParams), c_void_p]),
    "bh_eltwise_i8": (c_int, [ctypes.POINTER(EltwiseParams), c_void_p]),
    "bh_pool_i8": (c_int, [ctypes.POINTER(PoolParams), c_void_p]),
    "bh_irb_i8": (c_int, [ctypes.POINTER(IrbParams), c_void_p]),
    "bh_irb_lds_bytes": (c_size_t, [ctypes.POINTER(IrbParams)]),
    "bh_chain_i8": (c_int, [ctypes.POINTER(ChainParams), c_void_p]),
    "bh_mean": (c_int, [ctypes.POINTER(MeanParams), c_void_p]),
    "bh_chain_lds_bytes": (c_size_t, [ctypes.POINTER(ChainParams)]),
    "bh_chain_tile_lds_bytes": (c_size_t, [ctypes.POINTER(ChainParams)]),
    "bh_chain_tile_launch": (c_int, [ctypes.POINTER(ChainParams), c_void_p]),
    "bh_chain_tile_blob_bytes": (c_size_t, [ctypes.POINTER(ChainParams)]),
    "bh_chain_tile_pack": (c_int, [ctypes.POINTER(ChainParams), c_void_p, c_void_p]),
    "bh_chain_stage_lds_bytes": (c_size_t, [ctypes.POINTER(ChainParams)]),
    "bh_chain_stage_launch": (c_int, [ctypes.POINTER(ChainParams), c_void_p]),
    "bh_last_error": (ctypes.c_char_p, []),
}

BACKEND_SYMBOLS = {}  # filled by backend.py

_lib = None
_configured = set()


class BandHipError(RuntimeError):
    pass


def load():
    """Load libband_hip.so; raises if it is missing (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BandHipError(
                "libband_hip.so not built (%s); run __graft_entry__.build() / make -C band_amd/csrc" % LIB_PATH)
        _lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in list(KERNEL_SYMBOLS.items()) + list(BACKEND_SYMBOLS.items()):
        if name in _configured:
            continue
        fn = getattr(_lib, name)
        fn.restype = res
        fn.argtypes = args
        _configured.add(name)
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = load().bh_last_error()
        raise BandHipError("%s failed (rc=%d): %s" % (what, rc, msg.decode() if msg else ""))
    return rc
