"""TFLite_Detection_PostProcess on the CPU worker, and EfficientDet-Lite2
(BASELINE C4) whole on a kCPU executor, bit-exact with the oracle.

The custom op is not in the GPU set: Band's model analyzer places it on the
CPU worker (band/model_analyzer.cc:484-606); tests/test_engine_gpu.py runs
the split.  Parity for this op is unpinned (no reference fixture holds it);
both sides restate detection_postprocess.cc (oracle/detection_postprocess.py).
"""
import os

import numpy as np
import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey, tflite_synth as S
from oracle.detection_postprocess import read_flexbuffer_map
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model as OModel


def _run_cpu(buf, feeds, tmp_path, threads=4):
    p = str(tmp_path / "m.tflite")
    with open(p, "wb") as f:
        f.write(buf)
    m = HipModel(0)
    assert m.FromPath(p).ok()
    ex = HipModelExecutor(0, 0, DeviceFlag.kCPU, num_threads=threads)
    st = ex.PrepareSubgraph(m)
    assert st.ok(), st
    key = SubgraphKey(0, 0)
    for t, v in feeds.items():
        ex.GetTensorView(key, t).GetData()[...] = v
    assert ex.ExecuteSubgraph(key).ok()
    return {t: ex.GetTensorView(key, t).GetData().copy() for t in ex.GetOutputs(key)}


def test_flexbuffer_roundtrip():
    d = dict(max_detections=7, use_regular_nms=False, nms_score_threshold=0.25, num_classes=3, h_scale=5.0)
    assert read_flexbuffer_map(S.flexbuffer_map(d)) == d


def _postprocess_only(n, classes, background, seed, max_det=10, score_th=0.3, iou_th=0.5):
    rng = np.random.default_rng(seed)
    mb = S.ModelBuilder("dpp")
    be = mb.tensor("box_encodings", [1, n, 4], np.float32)
    cs = mb.tensor("class_predictions", [1, n, classes + background], np.float32)
    # clustered anchors so boxes overlap and NMS suppresses
    centers = rng.uniform(0.2, 0.8, (max(1, n // 6), 2))
    anc = np.concatenate([centers[rng.integers(0, len(centers), n)] + rng.normal(0, 0.01, (n, 2)),
                          rng.uniform(0.05, 0.3, (n, 2))], axis=1).astype(np.float32)
    at = mb.tensor("anchors", [n, 4], np.float32, data=anc)
    outs = [mb.tensor("boxes", [1, max_det, 4], np.float32), mb.tensor("classes", [1, max_det], np.float32),
            mb.tensor("scores", [1, max_det], np.float32), mb.tensor("num", [1], np.float32)]
    opts = S.flexbuffer_map(dict(max_detections=max_det, max_classes_per_detection=1, detections_per_class=100,
                                 use_regular_nms=False, nms_score_threshold=score_th, nms_iou_threshold=iou_th,
                                 num_classes=classes, y_scale=10.0, x_scale=10.0, h_scale=5.0, w_scale=5.0))
    mb.op("CUSTOM", [be, cs, at], outs, custom="TFLite_Detection_PostProcess", custom_options=opts)
    mb.inputs, mb.outputs = [be, cs], outs
    feeds = {be: rng.normal(0, 1, (1, n, 4)).astype(np.float32),
             # coarse scores: many exact ties (stable-order and first-max rules)
             cs: (rng.integers(0, 17, (1, n, classes + background)) / 16.0).astype(np.float32)}
    return mb.build(), feeds


@pytest.mark.parametrize("n,classes,background,seed,max_det,score_th", [
    (50, 3, 1, 0, 10, 0.3), (300, 7, 0, 1, 25, 0.5), (1000, 2, 1, 2, 100, 0.0), (64, 5, 1, 3, 5, 1.1),
    # heavy suppression over many tied candidates (the lazy-heap NMS draws
    # far past max_detections before it fills the output)
    (6000, 4, 1, 4, 100, 0.0), (4000, 90, 1, 5, 25, 0.2)])
def test_detection_postprocess_vs_oracle(tmp_path, n, classes, background, seed, max_det, score_th):
    buf, feeds = _postprocess_only(n, classes, background, seed, max_det, score_th)
    got = _run_cpu(buf, feeds, tmp_path)
    om = OModel(buf)
    ref = OracleInterpreter(om).run(feeds)
    for t in om.outputs:
        np.testing.assert_array_equal(got[t].reshape(-1), ref[t].reshape(-1))
    num = int(ref[om.outputs[3]][0])
    assert 0 <= num <= max_det
    if score_th > 1.0:
        assert num == 0


def test_efficientdet_lite2_cpu_worker_vs_oracle(tmp_path):
    buf = S.efficientdet_lite2(size=256)
    om = OModel(buf)
    x = np.random.default_rng(0).integers(-128, 128, (1, 256, 256, 3)).astype(np.int8)
    got = _run_cpu(buf, {om.inputs[0]: x}, tmp_path, threads=8)
    ref = OracleInterpreter(om).run({om.inputs[0]: x})
    for t in om.outputs:
        np.testing.assert_array_equal(got[t].reshape(-1), ref[t].reshape(-1))
    assert int(ref[om.outputs[3]][0]) > 0  # the synthetic class prior lets some anchors through
