#!/usr/bin/env python3
"""Lower bound on the L2-fill (FETCH + WRITE) bytes of a conv launch on
MI355X's 8 XCDs, each with its own L2, against its algorithmic bytes.

Every XCD that computes part of the output must pull the operand bytes that
part needs into its own L2.  With the output split over the XCDs as an a x b
grid of (pixel ranges) x (channel ranges), a * b = X, the input is read b
times and the filters a times:
    T(a, b) = b * A + a * W + O        (A input, W filters, O output)
and the best any workgroup order can do is min over a * b = X of T.  X is
min(8, workgroups).  A 3x3 conv's input is counted once (its halo between
pixel ranges is ignored, so this stays a lower bound).  Reading the
FETCH_SIZE counter, Infinity-Cache hits count as traffic too, so a kernel at
this bound shows T / algorithmic in its PMC ratio however the L2s are used.

usage: tools/xcd_traffic_bound.py <mix_breakdown.txt> [--kernels conv_mfma_kernel,conv_gemm_kernel]
prints per launch: algorithmic MB, bound MB, bound / algorithmic; and the
launch-weighted ratio per kernel (the figure tools/pmc_traffic.py reports
per kernel is a mean over launches of traffic, divided by the mean of
algorithmic bytes)
"""
import argparse
import re


def parse(path, kernels):
    rows = []
    pat = re.compile(r"^(\S+)\s+(\d+)\s+(\S+)\s+\[([\d, ]+)\]\s+\[([\d, ]+)\]\s+(k\dx\d)?\s*([\d.]+)")
    for line in open(path):
        m = pat.match(line)
        if not m or m.group(3).split("+")[0] not in kernels:
            continue
        i = [int(v) for v in m.group(4).split(",")]
        o = [int(v) for v in m.group(5).split(",")]
        k = int(m.group(6)[1]) if m.group(6) else 1
        rows.append(dict(model=m.group(1), op=int(m.group(2)), kernel=m.group(3), inp=i, out=o, k=k,
                         us=float(m.group(7))))
    return rows


def bound(r, tile_m=64, tile_n=64):
    B, H, W, C = r["inp"]
    _, OH, OW, N = r["out"]
    A = B * H * W * C
    Wt = N * r["k"] * r["k"] * C
    O = B * OH * OW * N
    M = B * OH * OW
    wgs = -(-M // tile_m) * -(-N // tile_n)
    X = max(1, min(8, wgs))
    best = min(b * A + (X // b) * Wt for b in (1, 2, 4, 8) if X % b == 0)
    alg = A + Wt + O
    return alg, best + O, X


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("breakdown")
    ap.add_argument("--kernels", default="conv_mfma_kernel,conv_gemm_kernel")
    a = ap.parse_args()
    ks = a.kernels.split(",")
    rows = parse(a.breakdown, ks)
    tot = {}
    for r in rows:
        alg, tb, X = bound(r)
        t = tot.setdefault(r["kernel"].split("+")[0], [0, 0.0, 0.0])
        t[0] += 1
        t[1] += alg
        t[2] += tb
        print("%-24s %3d %-18s in %-20s out %-20s k%d  alg %6.2f MB  bound %6.2f MB  %.2fx (%d XCDs)" % (
            r["model"], r["op"], r["kernel"], r["inp"], r["out"], r["k"], alg / 1e6, tb / 1e6, tb / alg, X))
    for k, (n, alg, tb) in tot.items():
        print("%-20s %2d launches: mean algorithmic %.3f MB, mean bound %.3f MB per launch; bound / algorithmic = %.2fx"
              % (k, n, alg / n / 1e6, tb / n / 1e6, tb / alg))


if __name__ == "__main__":
    main()
