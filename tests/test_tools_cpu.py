"""CPU checks of the occupancy tools (tools/chain_occupancy.py,
tools/kernel_resources.py): the tuner's choice codes decode to the forms
fusion.cc (FuseChains) encodes, and the waves-per-SIMD rules match
MI355X_MICROARCH.md's register and SGPR tables."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import chain_occupancy as co  # noqa: E402
import kernel_resources as kr  # noqa: E402


def test_choice_codes_decode_like_fusion_cc():
    # px_blocks, +10 two-launch form, +100 16 waves, +200 persistent,
    # +300 8 waves, +400.. tile, +1000 deep, +2000*(s-1) split; stage forms
    # from 100000
    f = co.decode(2101)
    assert (f["c_split"], f["waves"], f["px_blocks"], f["three"], f["tile"]) == (2, 16, 1, True, 0)
    f = co.decode(404)
    assert (f["tile"], f["three"], f["c_split"]) == (1, True, 0)
    f = co.decode(414)
    assert (f["tile"], f["three"]) == (1, False)
    f = co.decode(301)
    assert (f["waves"], f["px_blocks"], f["three"], f["persist"]) == (8, 1, True, 0)
    f = co.decode(12)
    assert (f["px_blocks"], f["three"], f["waves"]) == (2, False, 4)
    f = co.decode(1001)
    assert (f["deep"], f["px_blocks"]) == (1, 1)
    f = co.decode(100000 + 1000 + 200 + 10 + 1)  # stage 2, 2 slices, 1 block, 8 waves
    assert (f["stage"], f["c_split"], f["px_blocks"], f["waves"], f["three"]) == (2, 2, 1, 8, True)
    f = co.decode(2000 * 3 + 101)  # 16 waves, 4 slices
    assert (f["deep"], f["waves"], f["c_split"], f["px_blocks"], f["three"]) == (0, 16, 4, 1, True)
    assert not co.decode(0)["fused"]


def test_instantiation_names():
    # the kernel names chain_occupancy looks up in the resource table
    class Conv:
        k_pad = 960

    class Q:
        has_pw2 = True
        pw2 = Conv()

    assert co.instantiation(Q, co.decode(2000 * 3 + 101), True)[0] == "chain_kernel<1, true, 5, 16, false, 2, 2>"
    assert co.instantiation(Q, co.decode(1301), False)[0] == "chain_kernel<1, false, 5, 8, false, 6, 0>"
    assert co.instantiation(Q, co.decode(100000 + 1000 + 200 + 10 + 1), True) == ("chain_stage_kernel<1, true", 8)


def test_waves_per_simd_tables():
    # VGPR+AGPR allocation granule 8: <=64 -> 8, 72 -> 7, 80 -> 6, 88-96 -> 5,
    # 104-128 -> 4, 136-168 -> 3, 176-256 -> 2
    assert kr.waves_per_simd(64, 0, 80)[0] == 8
    assert kr.waves_per_simd(85, 0, 80)[0] == 5
    assert kr.waves_per_simd(84, 8, 80)[0] == 5
    assert kr.waves_per_simd(127, 16, 80)[0] == 3
    assert kr.waves_per_simd(121, 0, 80)[0] == 4
    assert kr.waves_per_simd(165, 24, 80)[0] == 2
    # SGPRs: 800 per SIMD, ceil(sgpr / 16) * 16 + 16 per wave
    assert kr.waves_per_simd(32, 0, 80)[1] == 8
    assert kr.waves_per_simd(32, 0, 96)[1] == 7
    assert kr.waves_per_simd(32, 0, 106)[1] == 6
