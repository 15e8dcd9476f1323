"""ORACLE — test infrastructure only.

CPU restatement of TFLite 2.9.2's `TFLite_Detection_PostProcess` custom op
(third-party `tensorflow/lite/kernels/detection_postprocess.cc`, absent from
/root/reference; called by Band through `Interpreter::Invoke` on the CPU
worker when the model analyzer places it there, band/model_analyzer.cc:484-606)
for the configuration the BASELINE detection models use: float inputs, fast
(class-agnostic) NMS, one class per detection.

  DecodeCenterSizeBoxes: ycenter = float(double(y) / double(y_scale) *
    double(anchor.h) + double(anchor.y)); half_h = float(0.5 *
    exp(double(h) / double(h_scale)) * double(anchor.h)); corners in float.
  MultiClassFastNMS: per anchor the first maximum over the non-background
    classes; scores >= threshold; stable descending sort; greedy IoU
    suppression (iou > threshold) up to max_detections; IoU in float.

PARITY UNPINNED: no fixture in the reference exercises this op; the formula
is the published one restated above.  Custom options are a FlexBuffers map
(parsed by `read_flexbuffer_map`).
"""
import math
import struct

import numpy as np

_FBT = {1: "int", 2: "uint", 3: "float", 26: "bool"}


def read_flexbuffer_map(buf):
    """{key: scalar} of a FlexBuffers map of inline scalars"""
    buf = bytes(buf)
    rw = buf[-1]
    rtype = buf[-2]
    root = len(buf) - 2 - rw
    off = int.from_bytes(buf[root:root + rw], "little")
    if rtype >> 2 != 9:
        raise ValueError("flexbuffer root is not a map")
    w = 1 << (rtype & 3)
    m = root - off

    def u(pos, width):
        return int.from_bytes(buf[pos:pos + width], "little")

    n = u(m - w, w)
    keys_w = u(m - 2 * w, w)
    keys = (m - 3 * w) - u(m - 3 * w, w)
    out = {}
    for i in range(n):
        kp = keys + i * keys_w
        ks = kp - u(kp, keys_w)
        key = buf[ks:buf.index(b"\0", ks)].decode()
        t = buf[m + n * w + i]
        kind = _FBT.get(t >> 2)
        raw = buf[m + i * w:m + (i + 1) * w]
        if kind == "float":
            v = struct.unpack("<d" if w == 8 else "<f", raw)[0] if w >= 4 else None
        elif kind == "int":
            v = int.from_bytes(raw, "little", signed=True)
        elif kind in ("uint", "bool"):
            v = int.from_bytes(raw, "little")
            v = bool(v) if kind == "bool" else v
        else:
            raise ValueError("unsupported flexbuffer value type %d" % (t >> 2))
        out[key] = v
    return out


def _f32(v):
    return float(np.float32(v))


def detection_postprocess(box_enc, cls, anchors, opts):
    """returns (boxes [1,D,4], classes [1,D], scores [1,D], num [1]) float32"""
    num_classes = int(opts["num_classes"])
    max_det = int(opts["max_detections"])
    max_cls = int(opts.get("max_classes_per_detection", 1))
    if opts.get("use_regular_nms", False) or max_cls != 1:
        raise NotImplementedError("oracle: detection postprocess restated for fast NMS, one class per detection")
    # options are read as float (AsFloat) then widened where the op does
    ys, xs, hs, ws = (float(np.float32(opts[k])) for k in ("y_scale", "x_scale", "h_scale", "w_scale"))
    score_th = np.float32(opts["nms_score_threshold"])
    iou_th = np.float32(opts["nms_iou_threshold"])
    b = np.asarray(box_enc, np.float32).reshape(-1, 4).astype(np.float64)
    a = np.asarray(anchors, np.float32).reshape(-1, 4).astype(np.float64)
    n = a.shape[0]
    yc = (b[:, 0] / ys * a[:, 2] + a[:, 0]).astype(np.float32)
    xc = (b[:, 1] / xs * a[:, 3] + a[:, 1]).astype(np.float32)
    eh = np.array([math.exp(v) for v in (b[:, 2] / hs).tolist()])
    ew = np.array([math.exp(v) for v in (b[:, 3] / ws).tolist()])
    hh = (0.5 * eh * a[:, 2]).astype(np.float32)
    hw = (0.5 * ew * a[:, 3]).astype(np.float32)
    boxes = np.stack([yc - hh, xc - hw, yc + hh, xc + hw], axis=1).astype(np.float32)  # ymin xmin ymax xmax
    s = np.asarray(cls, np.float32).reshape(n, -1)
    label_offset = s.shape[1] - num_classes
    s = s[:, label_offset:label_offset + num_classes]
    best = np.argmax(s, axis=1)  # first maximum
    max_scores = s[np.arange(n), best]
    keep = np.nonzero(max_scores >= score_th)[0]
    order = sorted(range(len(keep)), key=lambda i: -float(max_scores[keep[i]]))  # stable
    cand = [int(keep[i]) for i in order]
    area = ((boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])).astype(np.float32)
    active = [True] * len(cand)
    selected = []
    zero = np.float32(0)
    for i in range(len(cand)):
        if len(selected) >= min(len(cand), max_det):
            break
        if not active[i]:
            continue
        selected.append(cand[i])
        active[i] = False
        bi = cand[i]
        for j in range(i + 1, len(cand)):
            if not active[j]:
                continue
            bj = cand[j]
            if area[bi] <= zero or area[bj] <= zero:
                iou = zero
            else:
                iy0 = max(boxes[bi, 0], boxes[bj, 0])
                ix0 = max(boxes[bi, 1], boxes[bj, 1])
                iy1 = min(boxes[bi, 2], boxes[bj, 2])
                ix1 = min(boxes[bi, 3], boxes[bj, 3])
                inter = np.float32(max(np.float32(iy1 - iy0), zero) * max(np.float32(ix1 - ix0), zero))
                iou = np.float32(inter / np.float32(np.float32(area[bi] + area[bj]) - inter))
            if iou > iou_th:
                active[j] = False
    ob = np.zeros((1, max_det, 4), np.float32)
    oc = np.zeros((1, max_det), np.float32)
    osc = np.zeros((1, max_det), np.float32)
    for k, bi in enumerate(selected):
        ob[0, k] = boxes[bi]
        oc[0, k] = best[bi]
        osc[0, k] = max_scores[bi]
    return ob, oc, osc, np.array([len(selected)], np.float32)
