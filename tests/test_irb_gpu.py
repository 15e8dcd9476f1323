"""Op-level parity of the fused inverted-residual kernel (bh_irb_i8) against
the oracle running the 3-4 TFLite ops one by one.  Bit-exact, every
MobileNetV2 block shape, several tile sizes (halo / edge handling)."""
import numpy as np
import pytest

from tests.irb_harness import MNV2_BLOCKS, IrbCase

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("h,cin,t,cout,s", MNV2_BLOCKS)
def test_irb_mnv2_blocks(gpu_lib, h, cin, t, cout, s):
    rng = np.random.default_rng(h * 1000 + cin * 10 + cout + s)
    c = IrbCase(rng, 1, h, h, cin, cin * t, cout, s, has_expand=t != 1)
    ref = c.oracle()
    for tile in (1, 3, 4, 8):
        # tile 1 must always fit; larger tiles may exceed the 160 KB LDS budget
        if tile > 1 and not c.supported(gpu_lib, tile):
            continue
        np.testing.assert_array_equal(c.gpu(gpu_lib, tile), ref, err_msg="tile %d" % tile)
    c.fast = False  # TFLite's two-step requantisation in every stage
    np.testing.assert_array_equal(c.gpu(gpu_lib, 1), ref, err_msg="two-step requant")


@pytest.mark.parametrize("args", [
    dict(b=2, h=9, w=13, cin=24, ce=96, cout=24, stride=1),
    dict(b=1, h=11, w=10, cin=16, ce=64, cout=40, stride=2),
    dict(b=3, h=5, w=5, cin=8, ce=48, cout=8, stride=1, residual=False),
    dict(b=1, h=6, w=7, cin=32, ce=32, cout=16, stride=1, has_expand=False),
    dict(b=1, h=8, w=8, cin=16, ce=16, cout=16, stride=1, has_expand=False),  # no expand + residual
    dict(b=2, h=7, w=9, cin=32, ce=32, cout=32, stride=1, has_expand=False),
])
def test_irb_general(gpu_lib, args):
    rng = np.random.default_rng(len(args) * 7 + args["cin"] + args["cout"])
    c = IrbCase(rng, **args)
    ref = c.oracle()
    for tile in (1, 2, 5):
        np.testing.assert_array_equal(c.gpu(gpu_lib, tile), ref, err_msg="tile %d" % tile)
