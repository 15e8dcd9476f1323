"""Image-resident chain sequence (bh_chain_seq_i8, chain_seq_kernel): a run of
MobileNet chains executed by one workgroup per image, bit-exact against the
oracle running every TFLite op of every chain one by one (the chain i+1
depthwise input is chain i's second 1x1 output, its residual chain i's first
1x1 output)."""
import ctypes

import numpy as np
import pytest

from tests.chain_harness import MNV2_CHAINS, ChainCase

pytestmark = pytest.mark.gpu


def build_run(rng, b, specs, fast=True):
    """specs: (h, w, ce, stride, cout, residual, ce2) per chain, consecutive"""
    cases = []
    for k, (h, w, ce, s, cout, res, ce2) in enumerate(specs):
        nxt_res = k + 1 < len(specs) and specs[k + 1][5]
        cases.append(ChainCase(rng, b, h, w, ce, s, cout, res, ce2, store_pw1=bool(nxt_res or not ce2), fast=fast))
    for k in range(1, len(cases)):
        prev, c = cases[k - 1], cases[k]
        c.e_s, c.e_zp = prev.f_s, prev.f_zp
        if c.residual:
            c.x_s, c.x_zp = prev.y_s, (prev.o_zp if prev.residual else prev.p_zp)
    return cases


def run_oracle(cases):
    ys, fs = [], []
    for k, c in enumerate(cases):
        if k:
            c.e = fs[-1]
            if c.residual:
                c.x = ys[-1]
        y, f = c.oracle()
        ys.append(y)
        fs.append(f)
    return ys[-1], fs[-1]


def run_gpu(lib, cases, keep):
    from band_amd import _abi
    from band_amd.device import DeviceBuffer
    ps = [c.params(lib, 1, keep) for c in cases]
    for k in range(1, len(ps)):
        ps[k].dw.input = ps[k - 1].pw2.output
        if cases[k].residual:
            ps[k].pw1.residual = ps[k - 1].pw1.output
    arr = (_abi.ChainParams * len(ps))(*ps)
    n = len(ps)
    if lib.bh_chain_seq_lds_bytes(arr, n) == 0:
        return None
    host = ctypes.create_string_buffer(lib.bh_chain_seq_table_bytes())
    _abi.check(lib.bh_chain_seq_plan(arr, n, host), "bh_chain_seq_plan")
    table = DeviceBuffer.from_array(np.frombuffer(host.raw, np.uint8))
    keep.append(table)
    _abi.check(lib.bh_chain_seq_i8(arr, table.value, n, None), "bh_chain_seq_i8")
    last = cases[-1]
    y = last._y.download(np.int8, (last.b, last.oh, last.ow, last.cout)) if last._y else None
    f = last._f.download(np.int8, (last.b, last.oh, last.ow, last.ce2)) if last._f else None
    return y, f


def check_run(lib, rng, b, specs):
    cases = build_run(rng, b, specs)
    y_ref, f_ref = run_oracle(cases)
    keep = []
    out = run_gpu(lib, cases, keep)
    assert out is not None, "run not supported"
    y, f = out
    if cases[-1].store_pw1:
        np.testing.assert_array_equal(y, y_ref, err_msg="last first-1x1 output")
    if cases[-1].ce2:
        np.testing.assert_array_equal(f, f_ref, err_msg="last second-1x1 output")


def mnv2(idx):
    return [(h, h, ce, s, cout, res, ce2) for (h, ce, s, cout, res, ce2) in (MNV2_CHAINS[i] for i in idx)]


# MobileNetV2's 14x14 and 7x7 stages: blocks 8-17's chains (the tail at batch 1)
MNV2_TAIL = [6, 6, 6, 7, 8, 8, 9, 10, 10, 11]


@pytest.mark.parametrize("b", [1, 3])
def test_seq_mnv2_tail(gpu_lib, b):
    check_run(gpu_lib, np.random.default_rng(100 + b), b, mnv2(MNV2_TAIL))


@pytest.mark.parametrize("idx", [[6, 6], [7, 8], [8, 9], [9, 10], [10, 11], [6, 7, 8, 8, 9]])
def test_seq_mnv2_runs(gpu_lib, idx):
    check_run(gpu_lib, np.random.default_rng(sum(idx)), 2, mnv2(idx))


@pytest.mark.parametrize("specs", [
    # ragged image, stride 2 inside the run, N1 % 64 != 0 (K padding of the expand)
    [(9, 13, 128, 1, 32, True, 128), (9, 13, 128, 1, 32, True, 128), (9, 13, 128, 2, 48, False, 192)],
    # last chain without a second 1x1: its first 1x1 output is the run's output
    [(7, 7, 960, 1, 160, True, 960), (7, 7, 960, 1, 320, False, 0)],
    # odd image, residual on the first chain only, 64-channel chunks
    [(5, 11, 64, 1, 16, True, 64), (5, 11, 64, 2, 32, False, 256), (3, 6, 256, 1, 32, True, 64)],
])
def test_seq_general(gpu_lib, specs):
    check_run(gpu_lib, np.random.default_rng(len(specs) * 7 + specs[0][2]), 2, specs)


def test_seq_rejects(gpu_lib):
    from band_amd import _abi
    rng = np.random.default_rng(5)
    keep = []
    cases = build_run(rng, 1, mnv2([8, 8]))
    ps = [c.params(gpu_lib, 1, keep) for c in cases]
    arr = (_abi.ChainParams * 2)(*ps)
    # not linked: chain 1's depthwise input is not chain 0's second 1x1 output
    assert gpu_lib.bh_chain_seq_lds_bytes(arr, 2) == 0
    arr[1].dw.input = arr[0].pw2.output
    arr[1].pw1.residual = arr[0].pw1.output
    assert gpu_lib.bh_chain_seq_lds_bytes(arr, 2) > 0
    assert gpu_lib.bh_chain_seq_lds_bytes(arr, 1) == 0  # a run is >= 2 chains
    arr[1].pw1.requant_fast = 0  # single-step requantisation only
    assert gpu_lib.bh_chain_seq_lds_bytes(arr, 2) == 0
    arr[1].pw1.requant_fast = 1
    arr[0].dw.in_h = 17  # images up to 16 x 16
    assert gpu_lib.bh_chain_seq_lds_bytes(arr, 2) == 0
    arr[0].dw.in_h = 14
    assert gpu_lib.bh_chain_seq_i8(arr, None, 2, None) != 0  # no table: refused, nothing launched
