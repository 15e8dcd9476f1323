"""Executor-level reproducer for the rocprofv3 graph-launch crash (see
tools/graph_probe.hip for the plain-HIP side): prepares one HipModelExecutor
on a model and replays its subgraph a few times, graph on or off.
usage: python3 tools/rocprof_probe.py <add|mnv2|mix0..3|mix> [--batch B] [--no-graph]
(mix: the four C3 models, one executor each on ONE worker, sharing its stream)"""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10, help="graph launches queued back to back by TimeSubgraph")
    ap.add_argument("--wid", type=int, default=1, help="worker id of the executors (bench.py profiles as 1000)")
    ap.add_argument("--mid-base", type=int, default=0)
    ap.add_argument("--investigate", action="store_true", help="call InvestigateModelSpec first, as bench.py does")
    ap.add_argument("--unlink", action="store_true", help="delete the model files after preparing, as bench.py does")
    ap.add_argument("--profile", action="store_true",
                    help="ProfileSubgraph (events between launches, spin head start, empty-launch floor) "
                         "before the timed replays, as bench.py's roofline does")
    ap.add_argument("--sets", type=int, default=1,
                    help="prepare and run the executors this many times over, earlier sets kept alive "
                         "(bench.py --profile-only prepares the profiled models twice)")
    ap.add_argument("--new-ids", action="store_true", help="later sets use fresh model ids")
    ap.add_argument("--hwq", default=None, help="set GPU_MAX_HW_QUEUES before loading the library")
    a = ap.parse_args()
    if a.hwq:
        os.environ["GPU_MAX_HW_QUEUES"] = a.hwq
    import numpy as np
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SetWorkerDevice, SubgraphKey
    from band_amd import tflite_synth as S
    paths = []
    if a.model == "add":
        paths = [os.path.join(ROOT, "tests", "golden", "add.tflite")]
    elif a.model == "mix":
        for name in S.MIX_C3:
            f = tempfile.NamedTemporaryFile(suffix=".tflite", delete=False)
            f.write(getattr(S, name)(np.int8, size=224, batch=a.batch))
            f.close()
            paths.append(f.name)
    else:
        if a.model == "mnv2":
            buf = S.mobilenet_v2(np.int8, size=224, batch=a.batch)
        else:
            buf = getattr(S, S.MIX_C3[int(a.model[3:])])(np.int8, size=224, batch=a.batch)
        f = tempfile.NamedTemporaryFile(suffix=".tflite", delete=False)
        f.write(buf)
        f.close()
        paths = [f.name]
    SetWorkerDevice(a.wid, 0)
    alive = []
    for rep in range(a.sets):
        execs = []
        for i, path in enumerate(paths):
            mid = a.mid_base + i + (100 * rep if a.new_ids else 0)
            hm = HipModel(mid)
            assert hm.FromPath(path).ok()
            ex = HipModelExecutor(mid, a.wid, DeviceFlag.kGPU)
            if a.no_graph:
                ex.SetUseGraph(False)
            if a.investigate:
                ex.InvestigateModelSpec(hm)
            assert ex.PrepareSubgraph(hm).ok()
            ex._model_ref = hm
            execs.append((ex, SubgraphKey(mid, a.wid)))
        if a.profile:
            for ex, key in execs:
                rows, floor = ex.ProfileSubgraph(key, iters=20, with_floor=True)
                print("profiled", key, len(rows), "launches, floor us", floor, flush=True)
        for ex, key in execs:
            for i in range(a.runs):
                st = ex.ExecuteSubgraph(key)
                assert st.ok(), st
            print("model", key, "ok", flush=True)
            print("timed us", ex.TimeSubgraph(key, iters=a.iters), flush=True)
        alive.append(execs)
        print("set", rep, "done", flush=True)
    if a.unlink and a.model != "add":
        for path in paths:
            os.unlink(path)
    print("probe done:", a.model, "batch", a.batch, "graph", not a.no_graph)


if __name__ == "__main__":
    main()
