#!/usr/bin/env python3
"""Device-side concurrency scaling of the batched passes, without the Band
engine: S executors (one per worker id, so one HIP stream each) replay the
same model's graph back to back from S host threads at once; prints the
aggregate passes/s and inferences/s for each S.  If S = 4 gives little more
than S = 1, the passes compete for one device resource; if it scales, the
engine-level line is bound elsewhere (host side, copies, queue mapping).

usage: python3 tools/concurrency_probe.py [--model mobilenet_v2] [--batch 24] [--streams 1,2,4,8] [--iters 100]
       [--no-io]
       (--model mix: each stream replays the four C3 models in turn)"""
import argparse
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mobilenet_v2")
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--streams", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--no-io", action="store_true", help="kernels only: no H2D / D2H in the passes (diagnostic)")
    a = ap.parse_args()
    if a.no_io:
        os.environ["BAND_HIP_PROBE_NO_IO"] = "1"
    import numpy as np
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SetWorkerDevice, SubgraphKey
    from band_amd import tflite_synth as S
    names = list(S.MIX_C3) if a.model == "mix" else [a.model]
    paths = []
    for name in names:
        f = tempfile.NamedTemporaryFile(suffix=".tflite", delete=False)
        f.write(getattr(S, name)(np.int8, size=224, batch=a.batch))
        f.close()
        paths.append(f.name)
    smax = max(int(s) for s in a.streams.split(","))
    execs = []  # per stream: [(ex, key), ...] one per model
    keep = []
    for w in range(smax):
        wid = 500 + w
        SetWorkerDevice(wid, 0)
        per = []
        for i, path in enumerate(paths):
            mid = 1000 * (w + 1) + i
            hm = HipModel(mid)
            assert hm.FromPath(path).ok()
            ex = HipModelExecutor(mid, wid, DeviceFlag.kGPU)
            assert ex.PrepareSubgraph(hm).ok()
            keep.append(hm)
            key = SubgraphKey(mid, wid)
            assert ex.ExecuteSubgraph(key).ok()
            per.append((ex, key))
        execs.append(per)
    for p in paths:
        os.unlink(p)
    base = None
    for s in [int(v) for v in a.streams.split(",")]:
        barrier = threading.Barrier(s + 1)

        def run(per):
            barrier.wait()
            for _ in range(2):
                for ex, key in per:
                    ex.TimeSubgraph(key, iters=a.iters // 2)

        threads = [threading.Thread(target=run, args=(execs[w],)) for w in range(s)]
        for t in threads:
            t.start()
        barrier.wait()
        t0 = time.perf_counter()
        for t in threads:
            t.join()
        el = time.perf_counter() - t0
        passes = s * a.iters * len(names)
        rate = passes / el
        base = base or rate / s
        print("streams %2d: %8.0f passes/s  %9.0f inferences/s  (x%.2f of one stream)" % (
            s, rate, rate * a.batch, rate / base), flush=True)


if __name__ == "__main__":
    main()
