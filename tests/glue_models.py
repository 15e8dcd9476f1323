"""Small synthetic models that put every glue op of the HIP kernel set
between real conv layers (test fixtures, built with band_amd.tflite_synth)."""
import numpy as np

from band_amd.tflite_synth import QGraph


def glue_zoo(dtype, seed=3):
    g = QGraph(dtype, seed=seed, name="glue_zoo")
    x = g.input([1, 12, 10, 8], scale=0.05)
    a = g.conv(x, 16, k=3, act="NONE")
    b = g.dwconv(x, act="RELU6")
    c = g.concat([a, b, g.relu(a, "RELU")])
    d = g.pad(c, [[0, 0], [1, 2], [2, 1], [0, 0]])
    e = g.resize(d, (20, 26))
    f = g.resize(g.conv(e, 8, k=1, act="NONE"), (9, 7), bilinear=(np.dtype(dtype) == np.int8),
                 half_pixel_centers=True)
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
    """A model the model analyzer must split: two GPU runs of >= 7 ops around
    a float32 ADD only the CPU worker runs (DEQUANTIZE -> ADD(x, x) ->
    QUANTIZE), plus a side output from the first run."""
    g = QGraph(dtype, seed=seed, name="split_zoo")
    x = g.input([1, 16, 16, 8], scale=0.05)
    a = g.conv(x, 16, k=3, act="RELU6")
    for _ in range(3):
        a = g.add(g.conv(g.dwconv(a), 16, k=1, act="NONE"), a)
    f = g.dequantize(a)
    f = g.float_add(f, f)
    q = g.quantize_float(f, 0.1)
    b = g.conv(q, 24, k=3, stride=2, act="RELU6")
    for _ in range(3):
        b = g.add(g.conv(g.dwconv(b), 24, k=1, act="NONE"), b)
    g.output(g.fully_connected(g.reshape(g.avgpool(b, (8, 8)), [1, 24]), 10))
    g.output(g.logistic(a))
    return g.build()
