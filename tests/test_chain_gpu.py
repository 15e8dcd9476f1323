"""Parity of the fused depthwise -> 1x1 [-> ADD] [-> 1x1] chain (bh_chain_i8)
against the oracle running the TFLite ops one by one.  Bit-exact:

* kernel level: every MobileNetV2 chain shape (a block's depthwise + project
  [+ residual ADD] and the next block's expand), MobileNetV1 depthwise +
  pointwise pairs, DeepLab's dilated chains, ragged pixel tails, every
  px_blocks form, single-step and two-step requantisation;
* executor level: the C3 mix models at 224x224 with every feasible chain
  forced (BAND_HIP_FUSION=forcechain), one-job and job-batched passes.
"""
import os

import numpy as np
import pytest

from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey, tflite_synth as S
from oracle.runner import OracleInterpreter
from oracle.tflite_fb import Model as OModel
from tests.chain_harness import MNV2_CHAINS, ChainCase

pytestmark = pytest.mark.gpu


def _check(c, lib, px, waves=4, persist=0, tile=0, deep=0, c_split=0, stage=0):
    y_ref, f_ref = c.oracle()
    y, f = c.gpu(lib, px, waves, persist, tile, deep, c_split, stage)
    if c.store_pw1:
        np.testing.assert_array_equal(y, y_ref, err_msg="first conv, px_blocks %d" % px)
    if c.ce2:
        np.testing.assert_array_equal(f, f_ref, err_msg="second conv, px_blocks %d" % px)


@pytest.mark.parametrize("h,ce,s,cout,res,ce2", MNV2_CHAINS)
def test_chain_mnv2(gpu_lib, h, ce, s, cout, res, ce2):
    rng = np.random.default_rng(h * 1000 + ce + cout + s)
    c = ChainCase(rng, 1, h, h, ce, s, cout, res, ce2)
    for px in (4, 2, 1):
        _check(c, gpu_lib, px)
    _check(c, gpu_lib, 1, waves=16)
    _check(c, gpu_lib, 1, waves=8)
    for px, w in ((1, 4), (1, 8), (2, 4)):  # the deep-issue forms
        _check(c, gpu_lib, px, waves=w, deep=1)
    if _persist_fits(c, gpu_lib):
        _check(c, gpu_lib, 4, persist=1)
    c.fast = False  # TFLite's two-step requantisation in every stage
    _check(c, gpu_lib, 4)
    _check(c, gpu_lib, 1, deep=1)
    if _persist_fits(c, gpu_lib):
        _check(c, gpu_lib, 4, persist=1)


@pytest.mark.parametrize("args", [
    dict(b=2, h=112, w=112, ce=32, stride=1, cout=64, residual=False, ce2=0),      # MobileNetV1 pairs
    dict(b=1, h=56, w=56, ce=128, stride=2, cout=256, residual=False, ce2=0),
    dict(b=1, h=14, w=14, ce=512, stride=1, cout=512, residual=False, ce2=0),
    dict(b=3, h=7, w=7, ce=1024, stride=1, cout=1024, residual=False, ce2=0),
    dict(b=2, h=14, w=14, ce=576, stride=1, cout=96, residual=True, ce2=576, dil=2),  # DeepLab atrous
    dict(b=1, h=14, w=14, ce=960, stride=1, cout=160, residual=True, ce2=960, dil=2),
    dict(b=3, h=9, w=13, ce=48, stride=1, cout=24, residual=True, ce2=96),          # ragged pixel tail
    dict(b=1, h=11, w=10, ce=64, stride=2, cout=40, residual=False, ce2=128),
    dict(b=2, h=5, w=7, ce=16, stride=1, cout=8, residual=True, ce2=48),
    dict(b=1, h=28, w=28, ce=144, stride=1, cout=24, residual=False, ce2=144, store_pw1=True),
    dict(b=24, h=56, w=56, ce=144, stride=1, cout=24, residual=True, ce2=144),       # a batch-24 pass
])
def test_chain_general(gpu_lib, args):
    rng = np.random.default_rng(sum(v for v in args.values() if isinstance(v, int)))
    c = ChainCase(rng, **args)
    for px in (4, 1):
        _check(c, gpu_lib, px)
    _check(c, gpu_lib, 1, waves=16)
    _check(c, gpu_lib, 1, waves=8)
    for px, w in ((1, 4), (1, 8), (2, 4)):
        _check(c, gpu_lib, px, waves=w, deep=1)
    if _persist_fits(c, gpu_lib):
        _check(c, gpu_lib, 4, persist=1)


def _tile_fits(c, lib, tile=1):
    import ctypes
    keep = []
    return lib.bh_chain_lds_bytes(ctypes.byref(c.params(lib, 4, keep, 4, 0, tile))) > 0


@pytest.mark.parametrize("h,ce,s,cout,res,ce2", MNV2_CHAINS)
def test_chain_tile_mnv2(gpu_lib, h, ce, s, cout, res, ce2):
    """the 2-D tile form (chain_tile_kernel): every MobileNetV2 chain whose
    tile fits LDS, at batch 1 and 3 (ragged tiles at 7x7 / 14x14 / 28x28 /
    56x56 edges are all 8-tile multiples only at 56 / 112)"""
    for b in (1, 3):
        rng = np.random.default_rng(h * 1000 + ce + cout + s + b)
        c = ChainCase(rng, b, h, h, ce, s, cout, res, ce2)
        if not _tile_fits(c, gpu_lib):
            # LDS holds patch + both filters: the wide 14x14 / 7x7 chains
            # stay with the raster forms
            assert ce >= 384, "tile form should cover the %dx%dx%d chain" % (h, h, ce)
            continue
        _check(c, gpu_lib, 4, tile=1)
        _check(c, gpu_lib, 4, tile=3)  # runs of 2 / 4 tiles through one buffer
        _check(c, gpu_lib, 4, tile=4)
        c.fast = False
        _check(c, gpu_lib, 4, tile=1)
        _check(c, gpu_lib, 4, tile=4)


@pytest.mark.parametrize("args", [
    dict(b=2, h=112, w=112, ce=32, stride=1, cout=64, residual=False, ce2=0),      # MobileNetV1 pairs
    dict(b=1, h=56, w=56, ce=128, stride=2, cout=256, residual=False, ce2=0),
    dict(b=2, h=28, w=28, ce=256, stride=1, cout=256, residual=False, ce2=0),
    dict(b=2, h=14, w=14, ce=192, stride=1, cout=64, residual=True, ce2=192, dil=2),  # dilated
    dict(b=3, h=9, w=13, ce=48, stride=1, cout=24, residual=True, ce2=96),          # ragged tiles
    dict(b=1, h=11, w=10, ce=64, stride=2, cout=40, residual=False, ce2=128),
    dict(b=2, h=5, w=7, ce=16, stride=1, cout=8, residual=True, ce2=48),
    dict(b=1, h=3, w=2, ce=16, stride=2, cout=4, residual=False, ce2=16),           # one partial tile
    dict(b=1, h=28, w=28, ce=144, stride=1, cout=24, residual=False, ce2=144, store_pw1=True),
    dict(b=1, h=20, w=20, ce=96, stride=1, cout=40, residual=True, ce2=320),         # pw2 K 320 (KX 5)
    dict(b=24, h=56, w=56, ce=144, stride=1, cout=24, residual=True, ce2=144),       # a batch-24 pass
    dict(b=24, h=112, w=112, ce=32, stride=1, cout=16, residual=False, ce2=96),
])
def test_chain_tile_general(gpu_lib, args):
    rng = np.random.default_rng(7 + sum(v for v in args.values() if isinstance(v, int)))
    c = ChainCase(rng, **args)
    assert _tile_fits(c, gpu_lib)
    _check(c, gpu_lib, 4, tile=1)
    _check(c, gpu_lib, 4, tile=3)
    _check(c, gpu_lib, 4, tile=4)


def test_chain_tile_rejects(gpu_lib):
    import ctypes
    rng = np.random.default_rng(9)
    keep = []
    c = ChainCase(rng, 1, 8, 8, 32, 1, 16, False, 48).params(gpu_lib, 4, keep, tile=1)
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(c)) > 0
    c.tile = 5  # no such form (2: persistent, 3 / 4: runs of tiles)
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(c)) == 0
    assert gpu_lib.bh_chain_i8(ctypes.byref(c), None) != 0
    c.tile = 1
    c.dw.stride_h = c.dw.stride_w = 3  # the tile's patch is sized for stride <= 2
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(c)) == 0


def _persist_fits(c, lib):
    import ctypes
    keep = []
    return lib.bh_chain_lds_bytes(ctypes.byref(c.params(lib, 4, keep, 4, 1))) > 0


def test_chain_rejects_unsupported(gpu_lib):
    import ctypes
    rng = np.random.default_rng(5)
    keep = []
    c = ChainCase(rng, 1, 8, 8, 32, 1, 16, False, 48).params(gpu_lib, 4, keep)
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(c)) > 0
    c.deep = 1
    c.px_blocks = 4  # the deep forms take 16 or 32 pixels per workgroup
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(c)) == 0
    c.deep, c.px_blocks = 0, 4
    for field, bad in (("px_blocks", 3), ("waves", 12)):
        old = getattr(c, field)
        setattr(c, field, bad)
        assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(c)) == 0
        assert gpu_lib.bh_chain_i8(ctypes.byref(c), None) != 0
        setattr(c, field, old)
    c.dw.w_zp = 3  # asymmetric depthwise filter: not this kernel's
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(c)) == 0
    c.dw.w_zp = 0
    c.pw2.residual = c.pw1.weights  # the second conv never takes a residual
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(c)) == 0


@pytest.fixture(params=["forcechain", "forcetile", "forcedeep", "forcestage"])
def forcechain(request):
    old = os.environ.get("BAND_HIP_FUSION")
    os.environ["BAND_HIP_FUSION"] = request.param
    yield request.param
    if old is None:
        del os.environ["BAND_HIP_FUSION"]
    else:
        os.environ["BAND_HIP_FUSION"] = old


@pytest.mark.parametrize("arch", list(S.MIX_C3))
def test_chain_forced_mix_models(gpu_lib, forcechain, arch):
    buf = getattr(S, arch)(np.int8, size=224)
    om = OModel(buf)
    t = om.tensors[om.inputs[0]]
    rng = np.random.default_rng(77 + len(arch))
    xs = [rng.integers(-128, 128, t.shape).astype(np.int8) for _ in range(5)]
    refs = [OracleInterpreter(om).run({om.inputs[0]: x}) for x in xs]
    m = HipModel(41)
    assert m.FromBuffer(buf).ok()
    ex = HipModelExecutor(41, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(41, 1)
    kernels = [r["kernel"] for r in ex.ProfileSubgraph(key, iters=1)]
    assert any(k in kernels for k in ("chain_kernel", "chain_tile_kernel", "chain_stage_kernel")), kernels
    if forcechain == "forcetile":
        assert "chain_tile_kernel" in kernels, kernels
    if forcechain == "forcestage" and arch != "posenet_mobilenet_v1":  # MobileNetV1: pairs, no second 1x1
        assert "chain_stage_kernel" in kernels, kernels
    for rep in range(2):  # eager, then graph replay
        ex.GetTensorView(key, om.inputs[0]).GetData()[...] = xs[0]
        assert ex.ExecuteSubgraph(key).ok()
        for o in om.outputs:
            got = ex.GetTensorView(key, o).GetData()
            np.testing.assert_array_equal(got, refs[0][o].reshape(got.shape), err_msg="%s run %d" % (arch, rep))
    assert ex.PrepareJobBatches(m, key, 5).ok()
    for s, x in enumerate(xs):
        ex.GetJobSlotView(key, om.inputs[0], 5, s).GetData()[...] = x
    assert ex.ExecuteJobBatch(key, 5).ok()
    for s in range(5):
        for o in om.outputs:
            got = ex.GetJobSlotView(key, o, 5, s).GetData()
            np.testing.assert_array_equal(got, refs[s][o].reshape(got.shape), err_msg="%s slot %d" % (arch, s))
    ex._model_ref = m


@pytest.mark.parametrize("h,ce,s,cout,res,ce2", [c for c in MNV2_CHAINS if c[5]])
def test_chain_split_phase_c(gpu_lib, h, ce, s, cout, res, ce2):
    """the second 1x1's channel tiles split over 2 / 3 / 4 workgroups per pixel
    block (c_split, grid.y): every slice recomputes the depthwise and first
    1x1 and stores its channel range; the first 1x1's output (when stored)
    comes from slice 0.  Batch 2, 4-, 8- and 16-wave and 2-block forms, both
    requant forms, bit-exact"""
    import ctypes
    rng = np.random.default_rng(h * 7 + ce + cout)
    c = ChainCase(rng, 2, h, h, ce, s, cout, res, ce2, store_pw1=True)
    for px, waves, split in ((1, 4, 2), (1, 8, 2), (2, 4, 2), (1, 16, 2), (1, 4, 3), (1, 8, 3), (1, 4, 4)):
        keep = []
        if gpu_lib.bh_chain_lds_bytes(ctypes.byref(c.params(gpu_lib, px, keep, waves, 0, 0, 0, split))) == 0:
            continue
        _check(c, gpu_lib, px, waves, c_split=split)
    c.fast = False
    _check(c, gpu_lib, 1, 4, c_split=2)


def _stage_fits(c, lib, px, waves, split):
    import ctypes
    keep = []
    return lib.bh_chain_lds_bytes(ctypes.byref(c.params(lib, px, keep, waves, 0, 0, 0, split, 1))) > 0


@pytest.mark.parametrize("h,ce,s,cout,res,ce2", [c for c in MNV2_CHAINS if c[5]])
def test_chain_stage_mnv2(gpu_lib, h, ce, s, cout, res, ce2):
    """the stage form (chain_stage_kernel): the first 1x1's filter, the
    workgroup's slice of the second's and the residual rows staged by one
    LDS-DMA burst, both GEMMs from LDS; 1 / 2 pixel blocks, 4 / 8 waves, 1-8
    phase-C slices, batch 1 and a ragged batch 3, both requant forms"""
    for b in (1, 3):
        rng = np.random.default_rng(h * 31 + ce + cout + b)
        c = ChainCase(rng, b, h, h, ce, s, cout, res, ce2, store_pw1=True if b == 3 else None)
        ran = 0
        for px, waves, split in ((1, 4, 0), (1, 8, 0), (2, 4, 0), (2, 8, 0), (1, 8, 2), (1, 4, 3), (2, 8, 4),
                                 (1, 8, 8)):
            if not _stage_fits(c, gpu_lib, px, waves, split):
                continue
            _check(c, gpu_lib, px, waves, c_split=split, stage=1)
            _check(c, gpu_lib, px, waves, c_split=split, stage=2)  # loader waves
            ran += 1
        # LDS holds the whole first filter: only the 7x7 x 960 chains do not fit
        assert ran or ce >= 960, "stage form should cover the %dx%dx%d chain" % (h, h, ce)
        if ran:
            c.fast = False
            for px, waves, split in ((1, 8, 2), (2, 4, 0)):
                if _stage_fits(c, gpu_lib, px, waves, split):
                    _check(c, gpu_lib, px, waves, c_split=split, stage=1)
                    _check(c, gpu_lib, px, waves, c_split=split, stage=2)


@pytest.mark.parametrize("args", [
    dict(b=2, h=14, w=14, ce=192, stride=1, cout=64, residual=True, ce2=192, dil=2),  # dilated
    dict(b=3, h=9, w=13, ce=48, stride=1, cout=24, residual=True, ce2=96),          # ragged pixel tail
    dict(b=1, h=11, w=10, ce=64, stride=2, cout=40, residual=False, ce2=128),       # N2 % 16 != 0 slices
    dict(b=2, h=5, w=7, ce=16, stride=1, cout=8, residual=True, ce2=48),
    dict(b=1, h=3, w=2, ce=16, stride=2, cout=4, residual=False, ce2=20),           # one partial block
    dict(b=1, h=20, w=20, ce=96, stride=1, cout=40, residual=True, ce2=320),        # pw2 K 320 (KX 5)
    dict(b=24, h=14, w=14, ce=384, stride=1, cout=64, residual=True, ce2=384),      # a batch-24 pass
])
def test_chain_stage_general(gpu_lib, args):
    rng = np.random.default_rng(11 + sum(v for v in args.values() if isinstance(v, int)))
    c = ChainCase(rng, store_pw1=True, **args)
    for px, waves, split in ((1, 4, 0), (2, 8, 0), (1, 8, 2), (2, 4, 3), (1, 8, 8)):
        if _stage_fits(c, gpu_lib, px, waves, split):
            _check(c, gpu_lib, px, waves, c_split=split, stage=1)
            _check(c, gpu_lib, px, waves, c_split=split, stage=2)


def test_chain_stage_rejects(gpu_lib):
    import ctypes
    keep = []
    c = ChainCase(np.random.default_rng(3), 1, 14, 14, 64, 1, 32, False, 64)
    q = c.params(gpu_lib, 1, keep, 8, 0, 0, 0, 2, 1)
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(q)) > 0
    for field, bad in (("px_blocks", 4), ("waves", 16), ("c_split", 9), ("deep", 1), ("stage", 3)):
        old = getattr(q, field)
        setattr(q, field, bad)
        assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0, field
        setattr(q, field, old)
    q.c_split = 5  # 64 channels = 4 tiles < 5 slices
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0
    q.c_split = 2
    q.has_pw2 = 0  # the stage form always has the second 1x1
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0
    q.has_pw2 = 1
    q.tile_blob = None
    assert gpu_lib.bh_chain_i8(ctypes.byref(q), None) != 0  # no constant block: refused, nothing launched


def test_chain_split_rejects(gpu_lib):
    import ctypes
    rng = np.random.default_rng(3)
    keep = []
    q = ChainCase(rng, 1, 8, 8, 32, 1, 16, False, 48).params(gpu_lib, 1, keep, c_split=2)
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(q)) > 0
    q.c_split = 5  # at most 4
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0
    q.c_split = 4  # 48 channels = 3 tiles < 4 slices
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0
    q.c_split = 2
    q.persist = 1  # raster forms only
    assert gpu_lib.bh_chain_lds_bytes(ctypes.byref(q)) == 0


@pytest.mark.parametrize("arch,size", [("deeplab_v3_mobilenet_v2", 100), ("deeplab_v3_mobilenet_v2", 57),
                                       ("posenet_mobilenet_v1", 90), ("posenet_mobilenet_v1", 57),
                                       ("ssd_mobilenet_v2", 100)])
def test_chain_tile_ragged_models(gpu_lib, monkeypatch, arch, size):
    """whole models in the tile form (BAND_HIP_FUSION=forcetile) on image
    sizes whose layers are not multiples of the 8 x 8 tile (ragged right /
    bottom tiles, odd sizes: SAME padding with a one-sided pad); one-job
    and job-batched passes bit-exact vs the oracle"""
    monkeypatch.setenv("BAND_HIP_FUSION", "forcetile")
    buf = getattr(S, arch)(np.int8, size=size)
    om = OModel(buf)
    t = om.tensors[om.inputs[0]]
    rng = np.random.default_rng(size + len(arch))
    xs = [rng.integers(-128, 128, t.shape).astype(np.int8) for _ in range(3)]
    refs = [OracleInterpreter(om).run({om.inputs[0]: x}) for x in xs]
    m = HipModel(43)
    assert m.FromBuffer(buf).ok()
    ex = HipModelExecutor(43, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(43, 1)
    kernels = [r["kernel"] for r in ex.ProfileSubgraph(key, iters=1)]
    assert "chain_tile_kernel" in kernels, kernels
    for rep in range(2):
        ex.GetTensorView(key, om.inputs[0]).GetData()[...] = xs[0]
        assert ex.ExecuteSubgraph(key).ok()
        for o in om.outputs:
            got = ex.GetTensorView(key, o).GetData()
            np.testing.assert_array_equal(got, refs[0][o].reshape(got.shape), err_msg="%s run %d" % (arch, rep))
    assert ex.PrepareJobBatches(m, key, 3).ok()
    for s_, x in enumerate(xs):
        ex.GetJobSlotView(key, om.inputs[0], 3, s_).GetData()[...] = x
    assert ex.ExecuteJobBatch(key, 3).ok()
    for s_ in range(3):
        for o in om.outputs:
            got = ex.GetJobSlotView(key, o, 3, s_).GetData()
            np.testing.assert_array_equal(got, refs[s_][o].reshape(got.shape), err_msg="%s slot %d" % (arch, s_))
    ex._model_ref = m
