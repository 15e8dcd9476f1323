#!/usr/bin/env python3
"""GPU occupancy of a rocprofv3 kernel trace (run_kernel_trace.csv): over
the last FRACTION of the run (the timed loop, after tuning and warm-up),
the share of time with no kernel running, the mean number of kernels in
flight, the time at each concurrency level, and per hardware queue its
busy share and the gaps between its kernels.

usage: python3 tools/timeline_summary.py <run_kernel_trace.csv> [fraction=0.6]"""
import collections
import csv
import sys

import numpy as np


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.6
    st = np.array([int(r["Start_Timestamp"]) for r in rows])
    en = np.array([int(r["End_Timestamp"]) for r in rows])
    q = np.array([int(r["Queue_Id"]) for r in rows])
    o = np.argsort(st)
    st, en, q = st[o], en[o], q[o]
    t0 = st[int(len(st) * (1 - frac))]
    t1 = en.max()
    m = st >= t0
    S, E, Q = st[m], en[m], q[m]
    span = t1 - t0
    busy, cur_s, cur_e = 0, S[0], E[0]
    for s, e in zip(S[1:], E[1:]):
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print("window %.2f ms, kernels %d, busy (union) %.1f%%, mean kernels in flight %.2f (over busy time %.2f)" % (
        span / 1e6, m.sum(), 100 * busy / span, (E - S).sum() / span, (E - S).sum() / busy))
    ev = np.concatenate([np.stack([S, np.ones_like(S)], 1), np.stack([E, -np.ones_like(E)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    hist, c, last = collections.Counter(), 0, ev[0, 0]
    for t, d in ev:
        hist[c] += t - last
        c += d
        last = t
    tot = sum(hist.values())
    print("time at concurrency:", " ".join("%d:%.1f%%" % (k, 100 * v / tot) for k, v in sorted(hist.items())))
    for qq in sorted(set(Q.tolist())):
        mm = Q == qq
        s, e = S[mm], E[mm]
        gaps = s[1:] - e[:-1]
        print("queue %d: %d kernels, busy %.1f%%, median gap %.1f us, mean gap %.1f us, p90 gap %.1f us" % (
            qq, mm.sum(), 100 * (e - s).sum() / span, np.median(gaps) / 1e3, gaps.mean() / 1e3,
            np.percentile(gaps, 90) / 1e3))


if __name__ == "__main__":
    main()
