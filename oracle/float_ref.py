"""ORACLE — test infrastructure only.

Float32 graphs (TFLite fp16 post-training quantization: float16 constants
behind DEQUANTIZE, float32 compute) restated from TFLite 2.9.2's float
reference kernels (reference_ops::Conv / DepthwiseConv / FullyConnected /
Add / Mul / AveragePool / MaxPool / Logistic / Softmax).  Each op is
evaluated in float64 and rounded to float32 at its output, so the oracle is
at least as accurate as any float32 summation order; GPU and CPU-worker
results are compared against it with a stated tolerance, not bit-exactly.
"""
import numpy as np


def _act(y, lo, hi):
    return np.clip(y, lo, hi)


def conv2d_f32(x, w, bias, stride, dilation, pad, out_hw, lo, hi):
    """x [N,H,W,C], w [O,KH,KW,C] (OHWI)"""
    x = x.astype(np.float64)
    w = w.astype(np.float64)
    n, ih, iw, c = x.shape
    o, kh, kw, _ = w.shape
    oh, ow = out_hw
    (sh, sw), (dh, dw), (ph, pw) = stride, dilation, pad
    acc = np.zeros((n, oh, ow, o))
    ys = np.arange(oh) * sh - ph
    xs = np.arange(ow) * sw - pw
    for fy in range(kh):
        for fx in range(kw):
            yy, xx = ys + fy * dh, xs + fx * dw
            vy = (yy >= 0) & (yy < ih)
            vx = (xx >= 0) & (xx < iw)
            patch = np.zeros((n, oh, ow, c))
            patch[:, vy[:, None] & vx[None, :]] = x[:, yy[vy]][:, :, xx[vx]].reshape(n, -1, c)
            acc += np.tensordot(patch, w[:, fy, fx, :], axes=([3], [1]))
    if bias is not None:
        acc += bias.astype(np.float64)
    return _act(acc, lo, hi).astype(np.float32)


def dwconv2d_f32(x, w, bias, dm, stride, dilation, pad, out_hw, lo, hi):
    """x [N,H,W,C], w [1,KH,KW,C*dm]"""
    x = x.astype(np.float64)
    w = w.astype(np.float64)
    n, ih, iw, c = x.shape
    _, kh, kw, oc = w.shape
    oh, ow = out_hw
    (sh, sw), (dh, dw), (ph, pw) = stride, dilation, pad
    xr = np.repeat(x, dm, axis=3) if dm > 1 else x
    acc = np.zeros((n, oh, ow, oc))
    ys = np.arange(oh) * sh - ph
    xs = np.arange(ow) * sw - pw
    for fy in range(kh):
        for fx in range(kw):
            yy, xx = ys + fy * dh, xs + fx * dw
            vy = (yy >= 0) & (yy < ih)
            vx = (xx >= 0) & (xx < iw)
            patch = np.zeros((n, oh, ow, oc))
            patch[:, vy[:, None] & vx[None, :]] = xr[:, yy[vy]][:, :, xx[vx]].reshape(n, -1, oc)
            acc += patch * w[0, fy, fx]
    if bias is not None:
        acc += bias.astype(np.float64)
    return _act(acc, lo, hi).astype(np.float32)


def fully_connected_f32(x, w, bias, lo, hi):
    depth = w.shape[1]
    y = x.astype(np.float64).reshape(-1, depth) @ w.astype(np.float64).T
    if bias is not None:
        y += bias.astype(np.float64)
    return _act(y, lo, hi).astype(np.float32)


def eltwise_f32(a, b, kind, lo, hi):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    y = a + b if kind == "add" else (a - b if kind == "sub" else a * b)
    return _act(y, lo, hi).astype(np.float32)


def pool2d_f32(x, kind, filt, stride, pad, out_hw, lo, hi):
    n, ih, iw, c = x.shape
    (fh, fw), (sh, sw), (ph, pw), (oh, ow) = filt, stride, pad, out_hw
    out = np.zeros((n, oh, ow, c))
    xd = x.astype(np.float64)
    for oy in range(oh):
        y0 = oy * sh - ph
        for ox in range(ow):
            x0 = ox * sw - pw
            win = xd[:, max(0, y0):min(ih, y0 + fh), max(0, x0):min(iw, x0 + fw)]
            out[:, oy, ox] = win.mean(axis=(1, 2)) if kind == "avg" else win.max(axis=(1, 2))
    return _act(out, lo, hi).astype(np.float32)


def logistic_f32(x):
    return (1.0 / (1.0 + np.exp(-x.astype(np.float64)))).astype(np.float32)


def softmax_f32(x, beta):
    xd = x.astype(np.float64)
    e = np.exp((xd - xd.max(axis=-1, keepdims=True)) * beta)
    return (e / e.sum(axis=-1, keepdims=True)).astype(np.float32)
