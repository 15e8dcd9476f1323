#!/usr/bin/env python3
"""Single-threaded replay of the bench's batched passes for rocprofv3 --pmc.

bench.py under `rocprofv3 --pmc` (engine worker + planner threads, profiling
executors) crashed inside the tool's dispatch interception (SIGSEGV in
hipLaunchKernel, r01c); this replays the same launch sequences from one
thread: the C3 mix models at the bench's job batch, one HipModelExecutor
each (eager launches, the tuning decisions of BAND_HIP_TUNE_FILE), `iters`
ExecuteSubgraph calls per model.  tools/pmc_traffic.py then reads the
per-dispatch FETCH_SIZE / WRITE_SIZE.

usage: python3 tools/pmc_pass.py [--model mix_c3] [--batch 24] [--iters 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mix_c3")
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import tempfile

    import bench
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SetWorkerDevice, SubgraphKey
    SetWorkerDevice(7, 0)
    for mid, (name, buf) in enumerate(bench.model_list(a.model, 0, batch=a.batch)):
        tmp = tempfile.NamedTemporaryFile(prefix="pmc_%s_" % name, suffix=".tflite", delete=False)
        tmp.write(buf)
        tmp.close()
        hm = HipModel(mid)
        assert hm.FromPath(tmp.name).ok()
        ex = HipModelExecutor(mid, 7, DeviceFlag.kGPU)
        ex.SetUseGraph(False)
        spec = ex.InvestigateModelSpec(hm)
        gpu_ops = [i for i in range(spec.num_ops) if i not in spec.unsupported_ops[DeviceFlag.kGPU]]
        assert ex.PrepareSubgraph(hm, gpu_ops if len(gpu_ops) < spec.num_ops else ()).ok()
        key = SubgraphKey(mid, 7)
        for _ in range(a.iters):
            assert ex.ExecuteSubgraph(key).ok()
        print("%s: %d passes of batch %d" % (name, a.iters, a.batch), flush=True)
        del ex
        os.unlink(tmp.name)


if __name__ == "__main__":
    main()
