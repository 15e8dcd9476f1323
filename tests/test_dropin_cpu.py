"""The HIP backend is a drop-in for band/backend/tfl: every
band_amd/csrc/backend/hip/*.cc compiles against the reference's own band/
headers (not this repo's compat/ stand-ins), and the stand-ins the harness
builds with declare the reference's signatures.  Skipped where the reference
tree is absent (the GPU box)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "band", "interface", "model_executor.h")),
                                reason="reference tree not present")


def test_backend_compiles_against_reference_headers():
    r = subprocess.run([os.path.join(ROOT, "tools", "check_dropin.sh"), REF], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok   ") >= 10


def _decls(text, names):
    """normalised declarations (one per line) of the given function names"""
    text = re.sub(r"//[^\n]*", "", text)
    out = set()
    for line in text.splitlines():
        line = " ".join(line.split())
        m = re.match(r"^(?:const )?[\w:<>&* ]+?\b(\w+)\(.*\)( const)?;$", line)
        if m and m.group(1) in names:
            out.add(line)
    return out


def test_cpuset_stand_in_is_signature_identical():
    names = {"CpuSet", "Enable", "Disable", "DisableAll", "IsEnabled", "NumEnabled", "GetCPUMaskFlag",
             "GetMaskBits", "GetMaskBitsVector", "ToString", "GetCPUCount", "GetLittleCPUCount",
             "GetBigCPUCount", "SetCPUThreadAffinity", "GetCPUThreadAffinity", "BandCPUMaskGetSet"}
    ref = _decls(open(os.path.join(REF, "band", "device", "cpu.h")).read(), names)
    ours = _decls(open(os.path.join(ROOT, "band_amd", "csrc", "compat", "band", "device", "cpu.h")).read(), names)
    assert len(ref) >= 15, ref
    assert ref == ours, (ref ^ ours)


def test_backend_includes_no_harness_header():
    d = os.path.join(ROOT, "band_amd", "csrc", "backend", "hip")
    for f in os.listdir(d):
        src = open(os.path.join(d, f)).read()
        assert not re.search(r'#include "(engine|compat)/', src), f
        assert "band/interface/job_batching.h" not in src, f
