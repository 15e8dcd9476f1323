"""Small synthetic models that put every glue op of the HIP kernel set
between real conv layers (test fixtures, built with band_amd.tflite_synth)."""
import numpy as np

from band_amd.tflite_synth import OPT, ModelBuilder, QGraph, Table


def glue_zoo(dtype, seed=3):
    g = QGraph(dtype, seed=seed, name="glue_zoo")
    x = g.input([1, 12, 10, 8], scale=0.05)
    a = g.conv(x, 16, k=3, act="NONE")
    b = g.dwconv(x, act="RELU6")
    c = g.concat([a, b, g.relu(a, "RELU")])
    d = g.pad(c, [[0, 0], [1, 2], [2, 1], [0, 0]])
    e = g.resize(d, (20, 26))
    f = g.resize(g.conv(e, 8, k=1, act="NONE"), (9, 7), bilinear=True, half_pixel_centers=True)
    h = g.logistic(f)
    k = g.softmax(g.relu(g.quantize(f, 0.1, 3 if np.dtype(dtype) == np.int8 else 130), "RELU_N1_TO_1"), beta=0.7)
    g.output(h)
    g.output(k)
    g.output(g.dequantize(g.relu(e, "RELU6")))
    return g.build()


def fpn(dtype, seed=5):
    """Feature-pyramid merge: ADD(lateral 1x1 conv, upsampled deeper map) where
    the lateral conv is produced BEFORE the other ADD operand (the residual
    epilogue fusion must not fire), plus a residual ADD that may fuse."""
    g = QGraph(dtype, seed=seed, name="fpn")
    x = g.input([1, 16, 16, 8], scale=0.05)
    c1 = g.conv(x, 16, k=3, stride=2, act="RELU6")          # 8x8
    lat = g.conv(c1, 16, k=1, act="NONE")                    # lateral, consumed only by the ADD
    c2 = g.conv(c1, 24, k=3, stride=2, act="RELU6")          # 4x4, produced after lat
    up = g.resize(g.conv(c2, 16, k=1, act="NONE"), (8, 8))
    p = g.add(lat, up)
    r = g.add(g.conv(p, 16, k=1, act="NONE"), p)             # residual that can fuse
    g.output(r)
    return g.build()


def tconv_zoo(seed=7):
    """TRANSPOSE_CONV variants (int8): stride 2 / 1 / 3, SAME / VALID, with and
    without bias, odd spatial sizes and channel counts"""
    g = QGraph(np.int8, seed=seed, name="tconv_zoo")
    x = g.input([1, 5, 7, 12], scale=0.05)
    a = g.transpose_conv(x, 16, k=3, stride=2, padding="SAME")
    b = g.transpose_conv(a, 8, k=2, stride=2, padding="VALID", bias=False)
    c = g.transpose_conv(x, 5, k=3, stride=1, padding="SAME")
    d = g.transpose_conv(x, 6, k=4, stride=3, padding="VALID")
    g.output(b)
    g.output(c)
    g.output(d)
    return g.build()


def split_zoo(dtype=np.int8, seed=11):
    """A model the model analyzer must split GPU -> CPU -> GPU: a GPU run of
    >= 7 ops, then TFLite_Detection_PostProcess (CPU worker only) on
    DEQUANTIZEd box / class maps, then a GPU run over the QUANTIZEd
    detection scores, plus side outputs from both GPU runs."""
    g = QGraph(dtype, seed=seed, name="split_zoo")
    x = g.input([1, 16, 16, 8], scale=0.05)
    a = g.conv(x, 16, k=3, act="RELU6")
    for _ in range(3):
        a = g.add(g.conv(g.dwconv(a), 16, k=1, act="NONE"), a)
    n = 16 * 16
    boxes = g.dequantize(g.reshape(g.conv(a, 4, k=1, act="NONE"), [1, n, 4]))
    scores = g.dequantize(g.logistic(g.reshape(g.conv(a, 3, k=1, act="NONE", bias_offset_lsb=-20), [1, n, 3])))
    rng = np.random.default_rng(seed)
    anchors = np.concatenate([rng.uniform(0.1, 0.9, (n, 2)), rng.uniform(0.05, 0.3, (n, 2))], 1)
    det_boxes, det_classes, det_scores, num = g.detection_postprocess(boxes, scores, anchors, 3, max_detections=8,
                                                                      score_threshold=0.3)
    q = g.quantize_float(det_scores, 1.0 / 256)
    q4 = g.reshape(q, [1, 1, 1, 8])
    b = g.conv(q4, 24, k=1, act="RELU6")
    for _ in range(3):
        b = g.add(g.conv(g.dwconv(b), 24, k=1, act="NONE"), b)
    g.output(g.fully_connected(g.reshape(b, [1, 24]), 10))
    g.output(g.logistic(a))
    g.output(det_boxes)
    g.output(num)
    return g.build()


def float_zoo(seed=13):
    """float32 op variety for the fp16 path: odd channel counts, depth
    multiplier 2, dilation, strides, VALID padding, broadcast MUL, pools,
    FC, SOFTMAX, LOGISTIC, RELU_N1_TO_1"""
    from band_amd.tflite_synth import FGraph
    g = FGraph(seed=seed, name="float_zoo")
    x = g.input([1, 13, 11, 5])
    a = g.conv(x, 6, k=3, stride=2, act="RELU")                  # 7x6x6, out_c % 4 != 0
    b = g.dwconv(a, k=3, dm=2, act="RELU6")                     # 12 channels
    c = g.dwconv(b, k=3, dilation=2, act="NONE")
    d = g.conv(c, 7, k=2, padding="VALID", act="NONE")
    gate = g.logistic(g.avgpool(d, (6, 5)))                      # [1,1,1,7]
    e = g.mul(d, gate)                                           # broadcast
    f = g.maxpool(e, (2, 2), 2)
    h = g.relu(f, "RELU_N1_TO_1")
    v = g.reshape(h, [1, int(np.prod(g.meta[h][0]))])
    g.output(g.softmax(g.fully_connected(v, 9), beta=0.8))
    g.output(e)
    return g.build()


def norm_zoo(with_mean=True):
    """The instance-norm / padding ops of the reference's magenta
    style-transfer model (band/test/data/magenta_...tflite): MIRROR_PAD
    (REFLECT and SYMMETRIC), QUANTIZE, int8 MEAN over H, W with keep_dims,
    DEQUANTIZE, SQUARED_DIFFERENCE, ADD, RSQRT (float32 unless noted).
    with_mean=False drops the MEAN (the GPU set has no MEAN)."""
    mb = ModelBuilder("norm_zoo")
    f32 = np.float32
    x = mb.tensor("x", [1, 9, 11, 4], f32)
    mb.inputs = [x]
    p1 = mb.tensor("pads_reflect", [4, 2], np.int32, data=[[0, 0], [2, 1], [1, 2], [0, 0]])
    xr = mb.tensor("x_reflect", [1, 12, 14, 4], f32)
    mb.op(100, [x, p1], [xr], OPT_MIRROR_PAD, Table().set(0, "b", 0))  # REFLECT
    p2 = mb.tensor("pads_symmetric", [4, 2], np.int32, data=[[0, 0], [3, 0], [0, 11], [1, 0]])
    xs = mb.tensor("x_symmetric", [1, 12, 22, 5], f32)
    mb.op(100, [x, p2], [xs], OPT_MIRROR_PAD, Table().set(0, "b", 1))  # SYMMETRIC
    outs = [xr, xs]
    if with_mean:
        q = mb.tensor("q", [1, 12, 14, 4], np.int8, scale=0.02, zero_point=-3)
        mb.op("QUANTIZE", [xr], [q], OPT["QuantizeOptions"], Table())
        ax = mb.tensor("axes", [2], np.int32, data=[1, 2])
        m = mb.tensor("mean", [1, 1, 1, 4], np.int8, scale=0.011, zero_point=2)
        mb.op(40, [q, ax], [m], OPT_REDUCER, Table().set(0, "b", 1))  # keep_dims
        c = mb.tensor("mean_f32", [1, 1, 1, 4], f32)
        mb.op("DEQUANTIZE", [m], [c], OPT["DequantizeOptions"], Table())
        outs.append(m)
    else:
        c = mb.tensor("centre", [1, 1, 1, 4], f32, data=np.linspace(-0.3, 0.4, 4))
    sd = mb.tensor("sqdiff", [1, 12, 14, 4], f32)
    mb.op(99, [xr, c], [sd], OPT_SQDIFF, Table())
    one = mb.tensor("eps", [1], f32, data=[1e-3])
    v = mb.tensor("var_eps", [1, 12, 14, 4], f32)
    mb.op("ADD", [sd, one], [v], OPT["AddOptions"], Table().set(0, "b", 0))
    r = mb.tensor("rsqrt", [1, 12, 14, 4], f32)
    mb.op(76, [v], [r])
    mb.outputs = outs + [sd, r]
    return mb.build()


# BuiltinOptions union indices of the ops above (schema.fbs)
OPT_REDUCER, OPT_SQDIFF, OPT_MIRROR_PAD = 27, 76, 77


def hard_swish_model(dtype, in_scale=0.05, in_zp=3, out_scale=0.03, out_zp=-10):
    """x [1, 4, 8, 8] 8-bit -> HARD_SWISH -> y (every input byte appears once)"""
    mb = ModelBuilder("hard_swish")
    x = mb.tensor("x", [1, 4, 8, 8], dtype, scale=in_scale, zero_point=in_zp)
    y = mb.tensor("y", [1, 4, 8, 8], dtype, scale=out_scale, zero_point=out_zp)
    mb.inputs = [x]
    mb.op(117, [x], [y])
    mb.outputs = [y]
    return mb.build()


def all_bytes(dtype):
    lo = -128 if np.dtype(dtype) == np.int8 else 0
    return np.arange(lo, lo + 256).astype(dtype).reshape(1, 4, 8, 8)


HARD_SWISH_CASES = [  # (dtype, in_scale, in_zp, out_scale, out_zp)
    (np.int8, 0.05, 3, 0.03, -10), (np.int8, 0.02, -128, 0.02, -100), (np.int8, 0.2, 0, 0.1, 0),
    (np.uint8, 0.1, 128, 0.05, 20), (np.uint8, 0.03, 60, 0.04, 10),
]


def bilinear_model(dtype, in_hw, out_hw, c, align_corners=False, half_pixel_centers=False):
    """x [2, ih, iw, c] -> RESIZE_BILINEAR -> y [2, oh, ow, c]"""
    g = QGraph(dtype, seed=17, name="bilinear")
    x = g.input([2, in_hw[0], in_hw[1], c], scale=0.05)
    g.output(g.resize(x, out_hw, bilinear=True, align_corners=align_corners, half_pixel_centers=half_pixel_centers))
    return g.build()


BILINEAR_CASES = [  # (in_hw, out_hw, c, align_corners, half_pixel_centers)
    ((5, 5), (10, 10), 8, 0, 0), ((10, 10), (20, 20), 3, 0, 1), ((7, 9), (13, 4), 4, 1, 0), ((6, 6), (3, 3), 5, 0, 1),
    ((3, 5), (37, 41), 7, 0, 1), ((4, 4), (4, 4), 2, 1, 1), ((1, 1), (3, 5), 3, 0, 0),
]


def bilinear_u8_numpy(x, out_hw, ac, hp):
    """A second, numpy float32 restatement of the uint8 float path (checks
    the C oracle): ComputeInterpolationValues + four weights + 0.5f"""
    f32 = np.float32
    _, ih, iw, _ = x.shape

    def coords(n_in, n_out):
        s = f32(n_in - 1) / f32(n_out - 1) if ac and n_out > 1 else f32(n_in) / f32(n_out)
        v = np.arange(n_out, dtype=f32)
        sc = (v + f32(0.5)) * s - f32(0.5) if hp else v * s
        lo = np.maximum(np.floor(sc).astype(np.int64), 0)
        hi = np.minimum(np.ceil(sc).astype(np.int64), n_in - 1)
        return lo, hi, (sc - lo.astype(f32)).astype(f32)
    y0, y1, dy = coords(ih, out_hw[0])
    x0, x1, dx = coords(iw, out_hw[1])
    dy, dx = dy[None, :, None, None], dx[None, None, :, None]
    one = f32(1)
    a = x.astype(f32)
    v = (a[:, y0][:, :, x0] * ((one - dy) * (one - dx)) + a[:, y0][:, :, x1] * ((one - dy) * dx)
         + a[:, y1][:, :, x0] * (dy * (one - dx)) + a[:, y1][:, :, x1] * (dy * dx) + f32(0.5))
    return v.astype(np.int32).astype(np.uint8)
