#!/usr/bin/env python3
"""Headline benchmark: multi-DNN inferences/s + p99 job latency (BASELINE.json).

Workload (default, N=1): BASELINE config C3 - the 4-DNN int8 mix
(MobileNetV2, SSD-MobileNetV2, DeepLabV3-MobileNetV2, PoseNet-MobileNetV1;
224x224, synthetic seeded weights with TFLite-converter-shaped quantisation)
served round-robin by the Band GPU workers of one MI355X.  `--model
mobilenet_v2_int8` etc. run the single-model configs (C2).  A "step" is one
Band job: the per-job work of `Worker::Work` (band/worker.cc:222-323) - copy
the request into the executor's input view (Engine::TryCopyInputTensors,
band/engine.cc:1247-1319), `IModelExecutor::ExecuteSubgraph`
(band/engine.cc:843-850), copy the output views out (TryCopyOutputTensors
:1333-1365).  Job latency = end - enqueue (band/common.h:351-353).  Each Band
GPU worker holds one executor per model (band/engine.cc:91-106) on its own
HIP stream, like AddWorkers({kGPU, kGPU, ...}).

N>1: one process per GPU (torchrun), jobs shard across GPUs with no
data-path collective (weak scaling); a gloo process group only provides the
barrier and the max-over-ranks timing.  The GPU is driven exclusively
through libband_hip.so; torch never touches the device here.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import tempfile
import threading
import time

import numpy as np


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4000, help="jobs per rank in the timed region")
    p.add_argument("--warmup", type=int, default=400)
    p.add_argument("--workers-per-gpu", type=int, default=8)
    p.add_argument("--hw-queues", type=int, default=4,
                   help="GPU_MAX_HW_QUEUES for this process (HIP default 4; <= 32)")
    p.add_argument("--model", default="mix_c3",
                   choices=["mix_c3", "mobilenet_v2_int8", "mobilenet_v2_uint8", "mobilenet_v1_int8",
                            "ssd_mobilenet_v2_int8", "deeplab_v3_mobilenet_v2_int8", "posenet_mobilenet_v1_int8"])
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--profile-iters", type=int, default=20)
    return p.parse_args()


def model_list(name):
    """[(model name, .tflite bytes)] of the workload"""
    from band_amd import tflite_synth as S
    if name == "mix_c3":
        return [(m, getattr(S, m)(np.int8)) for m in S.MIX_C3]
    if name == "mobilenet_v2_int8":
        return [(name, S.mobilenet_v2(np.int8, seed=0))]
    if name == "mobilenet_v2_uint8":
        return [(name, S.mobilenet_v2(np.uint8, seed=0))]
    if name == "mobilenet_v1_int8":
        return [(name, S.mobilenet_v1(np.int8, seed=0))]
    base = name[:-len("_int8")]
    return [(name, getattr(S, base)(np.int8))]


class Dist:
    """barrier + max/gather over ranks (gloo, CPU only) when WORLD_SIZE > 1"""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, v):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def run_worker(execs, keys, requests, n_jobs, first, lat, results, idx):
    """One Band GPU worker thread: closed-loop jobs over the mixed stream
    (C++ loop bhx_run_mixed_jobs; the GIL is released for the whole batch)."""
    from band_amd import RunMixedJobs
    try:
        us, _ = RunMixedJobs(execs, keys, requests, n_jobs, first_model=first)
        lat.extend((us * 1e-6).tolist())
        results[idx] = True
    except Exception as e:  # noqa: BLE001
        results[idx] = str(e)


def cpu_baseline(models, seconds):
    """Oracle (scalar C port of TFLite's reference kernels) on the host, the
    same round-robin request stream over the models."""
    from oracle.runner import OracleInterpreter
    from oracle.tflite_fb import Model
    rng = np.random.default_rng(5489)
    runs = []
    for _, buf in models:
        m = Model(buf)
        t_in = m.tensors[m.inputs[0]]
        lo, hi = (-127, 128) if t_in.np_dtype == np.int8 else (0, 255)
        x = rng.integers(lo, hi, t_in.shape).astype(t_in.np_dtype)
        interp = OracleInterpreter(m)
        interp.run({m.inputs[0]: x})  # warm
        runs.append((interp, {m.inputs[0]: x}))
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        interp, feed = runs[n % len(runs)]
        interp.run(feed)
        n += 1
    dt = time.perf_counter() - t0
    names = "+".join(name for name, _ in models)
    return dict(value=n / dt, unit="inferences/s", cores=1, kind="port",
                sample="%d round-robin jobs of %s (224x224 int8) on 1 host core, %.1f s" % (n, names, dt))


def main():
    args = parse()
    # hardware queues are fixed at HIP runtime init: one per concurrently
    # running Band GPU worker stream (must be set before libband_hip loads)
    # (explicit assignment: the GPU box exports HIP's default of 4)
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(32, args.hw_queues)))
    D = Dist()
    import band_amd
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey

    models = model_list(args.model)
    M = len(models)
    W = max(1, args.workers_per_gpu)
    hip_models = []
    for mid, (name, buf) in enumerate(models):
        tmp = tempfile.NamedTemporaryFile(prefix="band_bench_", suffix=".tflite", delete=False)
        tmp.write(buf)
        tmp.close()
        hm = HipModel(mid)  # one IModel per model, shared by every worker's executor, as in Band
        st = hm.FromPath(tmp.name)
        os.unlink(tmp.name)
        assert st.ok(), st
        hip_models.append(hm)
    workers = []  # per worker: ([executor per model], [key per model])
    for w in range(W):
        wid = 1 + w  # worker 0 is Band's CPU worker
        band_amd.SetWorkerDevice(wid, D.local_rank)
        execs, keys = [], []
        for mid, hm in enumerate(hip_models):
            ex = HipModelExecutor(mid, wid, DeviceFlag.kGPU)
            if args.no_graph:
                ex.SetUseGraph(False)
            spec = ex.InvestigateModelSpec(hm)
            assert not spec.unsupported_ops[DeviceFlag.kGPU], spec.unsupported_ops
            st = ex.PrepareSubgraph(hm)
            assert st.ok(), st
            execs.append(ex)
            keys.append(SubgraphKey(mid, wid))
        workers.append((execs, keys))

    # synthetic requests: int8 U{-127..127} / uint8 U{0..254} (band/tool/benchmark.cc:279-287)
    rng = np.random.default_rng(5489 + D.rank)
    requests = []
    for ex, key in zip(*workers[0]):
        arr = ex.GetTensorView(key, ex.GetInputs(key)[0]).GetData()
        lo, hi = (-127, 128) if arr.dtype == np.int8 else (0, 255)
        requests.append(rng.integers(lo, hi, arr.shape).astype(arr.dtype))

    def run(n_total):
        lats = [[] for _ in range(W)]
        res = [None] * W
        share = [n_total // W + (1 if i < n_total % W else 0) for i in range(W)]
        ths = [threading.Thread(target=run_worker, args=(execs, keys, requests, share[i], i % M, lats[i], res, i))
               for i, (execs, keys) in enumerate(workers)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        bad = [r for r in res if r is not True]
        if bad:
            raise RuntimeError("job failed: %s" % bad)
        return [x for l in lats for x in l]

    run(max(args.warmup, 2 * W * M))
    D.barrier()
    t0 = time.perf_counter()
    lat = run(args.steps)
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.max(t1 - t0)
    all_lat = [x for part in D.gather(lat) for x in part]

    # roofline of the dominant kernel: per-launch HIP events on the worker's
    # stream, over one inference of each model (the mix is uniform)
    by_k = {}
    execs0, keys0 = workers[0]
    for ex, key in zip(execs0, keys0):
        for r in ex.ProfileSubgraph(key, iters=args.profile_iters):
            # group by kernel symbol ("conv_mfma_kernel+add" is conv_mfma_kernel
            # with its residual epilogue), as rocprofv3 reports them
            k = by_k.setdefault(r["kernel"].split("+")[0], dict(ms=0.0, bytes=0.0, ops=0.0, launches=0))
            k["ms"] += r["ms"] / M
            k["bytes"] += r["alg_bytes"] / M
            k["ops"] += r["alg_ops"] / M
            k["launches"] += 1.0 / M
    dom_name = max(by_k, key=lambda k: by_k[k]["ms"])
    dom = by_k[dom_name]
    avg_ms = dom["ms"] / dom["launches"]
    bytes_per_launch = dom["bytes"] / dom["launches"]
    ops_per_launch = dom["ops"] / dom["launches"]
    achieved_gbs = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    gpu_ms_total = sum(v["ms"] for v in by_k.values())
    # HBM traffic of the dominant kernel from the committed rocprofv3 PMC
    # passes (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE, gfx950
    # corrections of MI355X_MICROARCH.md), per launch; null when absent
    traffic, traffic_src = None, None
    import glob
    pmc = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*pmc_traffic.json")))
    if pmc:
        with open(pmc[-1]) as f:
            tj = json.load(f)
        if dom_name in tj:
            traffic, traffic_src = tj[dom_name]["traffic_bytes_per_launch"], os.path.basename(pmc[-1])
    # device-side floor of one job: each model's passes replayed back to back
    # (graph incl. H2D/D2H), no host gaps; the rest of the job latency is
    # host launch + sync wakeup
    device_us = {name: ex.TimeSubgraph(key, iters=100) for (name, _), ex, key in zip(models, execs0, keys0)}

    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(models, args.cpu_baseline_seconds)

    if D.rank == 0:
        n = D.world
        total_jobs = args.steps * n
        lat_ms = np.array(all_lat) * 1e3
        line = {
            "metric": "multi-DNN inferences/sec + p99 job latency, 4-model int8 mix @1/2/4/8 GPU",
            "value": total_jobs / elapsed,
            "unit": "inferences/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8" if "int8" in args.model else "uint8",
            "data": "synthetic (seeded int8 inputs and weights; no checkpoint)",
            "config": {"workload": ("C3: 4-DNN int8 mix (%s), 224x224 batch-1 jobs round-robin over %d Band GPU "
                                    "worker(s) per MI355X" % (", ".join(nm for nm, _ in models), W))
                       if M > 1 else ("C2: %s 224x224 batch-1 jobs, %d Band GPU worker(s) per MI355X, fixed_worker"
                                      % (args.model, W)),
                       "model": args.model, "global_batch": n * W, "seq_len": None,
                       "parallelism": "job-sharded x%d (no collective)" % n, "hipgraph": not args.no_graph,
                       "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))},
            "p50_job_latency_ms": float(np.percentile(lat_ms, 50)),
            "p99_job_latency_ms": float(np.percentile(lat_ms, 99)),
            "gpu_kernel_ms_per_inference": gpu_ms_total,
            "device_us_per_inference": float(np.mean(list(device_us.values()))),
            "device_us_per_model": device_us,
            "roofline": {
                "kernel": dom_name, "bound": "hbm", "achieved": achieved_gbs, "peak": 8000.0, "unit": "GB/s",
                "frac": achieved_gbs / 8000.0, "traffic": traffic, "traffic_source": traffic_src,
                "alg_bytes_per_launch": bytes_per_launch, "avg_launch_us": avg_ms * 1e3,
                "launches_per_inference": dom["launches"],
                "mfma_i8_tops": ops_per_launch / (avg_ms * 1e-3) / 1e12,
                "mfma_i8_frac": ops_per_launch / (avg_ms * 1e-3) / 5.0e15,
            },
            "cpu_baseline": cpu,
            "host": platform.node(),
        }
        print(json.dumps(line), flush=True)
    D.close()


if __name__ == "__main__":
    main()
