#!/usr/bin/env python3
"""Rewrite a round-4 tune file (chain keys version 6) into this tree's key
format (version 10, form-set flags f0000), other keys unchanged: replays the
round-4 tuner's chain choices on this tree's kernels for a same-box A/B.
usage: tools/tune_translate.py in.txt out.txt"""
import sys

out = []
for line in open(sys.argv[1]):
    p = line.split()
    if len(p) != 2:
        continue
    k, v = p
    if k.startswith("ch6:"):
        k = "ch10:" + k[4:] + ":f0000"
    out.append("%s %s\n" % (k, v))
open(sys.argv[2], "w").writelines(out)
print("%d entries" % len(out))
