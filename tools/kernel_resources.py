#!/usr/bin/env python3
"""Register / LDS resources of every kernel instantiation in a HIP source,
as the compiler allocates them for gfx950, and the waves per SIMD they allow.

Compiles the file with -Rpass-analysis=kernel-resource-usage (the same flags
as band_amd/csrc/Makefile) and prints one line per kernel: demangled name,
SGPRs, arch VGPRs, AGPRs, static LDS, scratch, and the compiler's occupancy.
Waves per SIMD allowed by registers follow MI355X_MICROARCH.md "Register
files": alloc = ceil((VGPR + AGPR) / 8) * 8, min(8, 512 // alloc); by SGPRs:
800 // (ceil(SGPR / 16) * 16 + 16) ("Residency and cooperative launch").

usage: tools/kernel_resources.py [-DNAME=V ...] band_amd/csrc/kernels/fused_chain.hip [more.hip] > out.txt
(the Makefile's -amdgpu-mfma-vgpr-form build; -D options are build-time A-B switches)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "band_amd", "csrc")


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.split("\n")
        return out[:len(names)]
    except (OSError, subprocess.CalledProcessError):
        return names


def resources(src, defines=()):
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
               "-mllvm", "-amdgpu-mfma-vgpr-form"] + list(defines) + [
               "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(CSRC, "kernels"),
               "-I" + os.path.join(CSRC, "compat"), "-I" + CSRC, "-Rpass-analysis=kernel-resource-usage",
               "-c", src, "-o", os.path.join(td, "k.o")]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.exit("hipcc failed:\n" + r.stderr[-2000:])
    rows = []
    for blk in r.stderr.split("remark: Function Name: ")[1:]:
        name = blk.split("\n")[0].split(" [-Rpass")[0].strip()

        def num(key):
            m = re.search(key + r": (\d+)", blk)
            return int(m.group(1)) if m else 0
        rows.append(dict(name=name, sgpr=num("SGPRs"), vgpr=num("VGPRs"), agpr=num("AGPRs"),
                         lds=num(r"LDS Size \[bytes/block\]"), scratch=num(r"ScratchSize \[bytes/lane\]"),
                         occ=num(r"Occupancy \[waves/SIMD\]")))
    for r_, d in zip(rows, demangle([r_["name"] for r_ in rows])):
        r_["demangled"] = d
    return rows


def waves_per_simd(vgpr, agpr, sgpr):
    alloc = -(-(vgpr + agpr) // 8) * 8
    by_v = min(8, 512 // max(alloc, 8))
    by_s = 800 // (-(-sgpr // 16) * 16 + 16)
    return by_v, by_s


def main():
    print("%-6s %-5s %-5s %-5s %-7s %-7s %-4s %-5s %-5s  %s" % (
        "sgpr", "vgpr", "agpr", "lds", "scratch", "occ", "v/S", "s/S", "w/S", "kernel (demangled)"))
    defines = [a for a in sys.argv[1:] if a.startswith("-D")]
    for src in (a for a in sys.argv[1:] if not a.startswith("-D")):
        for r in resources(src, defines):
            bv, bs = waves_per_simd(r["vgpr"], r["agpr"], r["sgpr"])
            print("%-6d %-5d %-5d %-5d %-7d %-7d %-4d %-5d %-5d  %s" % (
                r["sgpr"], r["vgpr"], r["agpr"], r["lds"], r["scratch"], r["occ"], bv, bs, min(bv, bs),
                r["demangled"].split("(")[0]))


if __name__ == "__main__":
    main()
