#!/usr/bin/env python3
"""Headline benchmark: multi-DNN inferences/s + p99 job latency (BASELINE.json).

Workload (default, N=1): BASELINE config C3 - the 4-DNN int8 mix
(MobileNetV2, SSD-MobileNetV2, DeepLabV3-MobileNetV2, PoseNet-MobileNetV1;
224x224, synthetic seeded weights with TFLite-converter-shaped quantisation)
served by the native Band engine (band_amd/csrc/engine) with round_robin over
`--workers-per-gpu` Band GPU workers of one MI355X (AddWorkers({kGPU, ...})).
`--model mobilenet_v2_int8` etc. run single-model configs (C2).

A "step" is one Band job, end to end through the harness: RequestAsync
(user tensor -> request ring, band/engine.cc:455-529) -> planner thread ->
scheduler -> worker queue (band/planner.cc:268-365) -> Worker::Work: input
copy into the executor's view, IModelExecutor::ExecuteSubgraph on the GPU,
output copy (band/worker.cc:222-323) -> Wait.  A native closed-loop driver
(BandxEngineRunClosedLoop) keeps 2 x workers x job-batch requests in
flight.  Job latency = end - enqueue of the planner's job record
(band/common.h:351-353).

Job batching (--job-batch B, default 24; BANDX_WORKER_MAX_JOB_BATCH): an
idle GPU worker takes up to B queued requests of one model from round_robin
and runs them as ONE pass over a batch-B variant of the model's subgraph
(every job still gets its own input copy, its own outputs, its own job
record).  Band itself runs one job per ExecuteSubgraph; that configuration
(8 GPU workers, no batching) is measured in the same run and reported as
"band_one_job_per_pass".  --job-batch 1 makes it the headline instead.

N>1: one process per GPU (torchrun), each with its own engine over its GPU;
jobs shard across GPUs with no data-path collective (weak scaling); a gloo
process group only provides the barrier and the max-over-ranks timing.  The
GPU is driven exclusively through libband_hip.so; torch never touches it.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import tempfile
import time

import numpy as np


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20000, help="jobs per rank in the timed region")
    p.add_argument("--warmup", type=int, default=2000)
    p.add_argument("--workers-per-gpu", type=int, default=8)
    p.add_argument("--hw-queues", type=int, default=4,
                   help="GPU_MAX_HW_QUEUES for this process (HIP default 4; <= 32)")
    p.add_argument("--model", default="mix_c3",
                   choices=["mix_c3", "mobilenet_v2_int8", "mobilenet_v2_uint8", "mobilenet_v1_int8",
                            "ssd_mobilenet_v2_int8", "deeplab_v3_mobilenet_v2_int8", "posenet_mobilenet_v1_int8",
                            "efficientdet_lite2_int8", "mix_c5"])
    p.add_argument("--rate", type=float, default=0.0,
                   help="mix_c5: Poisson arrival rate (requests/s per GPU); default 0.8 x the closed-loop capacity")
    p.add_argument("--cpu-workers", type=int, default=-1,
                   help="Band CPU workers (worker ids first); default: 1 when the model has CPU-only ops")
    p.add_argument("--cpu-threads", type=int, default=8, help="num_threads of each CPU worker")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--profile-iters", type=int, default=20)
    p.add_argument("--scheduler", default="round_robin",
                   choices=["round_robin", "fixed_worker", "shortest_expected_latency",
                            "heterogeneous_earliest_finish_time"])
    p.add_argument("--inflight", type=int, default=0, help="outstanding requests (default 2 x workers)")
    p.add_argument("--device", default="gpu", choices=["gpu", "cpu"],
                   help="cpu: --workers-per-gpu Band CPU workers instead of GPU workers (C1 / CPU tests; no roofline)")
    p.add_argument("--size", type=int, default=0, help="input edge (default 224; EfficientDet 448)")
    p.add_argument("--no-batch1", action="store_true",
                   help="skip the one-job-per-pass (Band semantics) line reported beside a job-batched run")
    p.add_argument("--job-batch", type=int, default=24,
                   help="max queued jobs of one model a GPU worker runs as one batched pass "
                        "(BANDX_WORKER_MAX_JOB_BATCH; 1 = Band's one job per ExecuteSubgraph)")
    return p.parse_args()


def model_list(name, size=0, batch=1):
    """[(model name, .tflite bytes)] of the workload (size 0: the configs'
    224x224, EfficientDet-Lite2 448x448); batch > 1: the same models with a
    leading batch (profiling the passes job batching runs)"""
    from band_amd import tflite_synth as S
    sz = size or 224
    ed = size or 448
    b = batch
    if name == "mix_c3":
        return [(m, getattr(S, m)(np.int8, size=sz, batch=b)) for m in S.MIX_C3]
    if name == "mobilenet_v2_int8":
        return [(name, S.mobilenet_v2(np.int8, seed=0, size=sz, batch=b))]
    if name == "mobilenet_v2_uint8":
        return [(name, S.mobilenet_v2(np.uint8, seed=0, size=sz, batch=b))]
    if name == "mobilenet_v1_int8":
        return [(name, S.mobilenet_v1(np.int8, seed=0, size=sz, batch=b))]
    if name == "efficientdet_lite2_int8":
        return [(name, S.efficientdet_lite2(np.int8, size=ed))]
    if name == "mix_c5":
        # 8 DNNs, int8 + fp16 (float16 weights, float32 compute)
        return [("mobilenet_v1_int8", S.mobilenet_v1(np.int8, size=sz)),
                ("mobilenet_v2_int8", S.mobilenet_v2(np.int8, size=sz)),
                ("ssd_mobilenet_v2_int8", S.ssd_mobilenet_v2(np.int8, size=sz)),
                ("deeplab_v3_mobilenet_v2_int8", S.deeplab_v3_mobilenet_v2(np.int8, size=sz)),
                ("posenet_mobilenet_v1_int8", S.posenet_mobilenet_v1(np.int8, size=sz)),
                ("efficientdet_lite2_int8", S.efficientdet_lite2(np.int8, size=ed)),
                ("mobilenet_v2_fp16", S.mobilenet_v2(np.float16, size=sz)),
                ("ssd_mobilenet_v2_fp16", S.ssd_mobilenet_v2(np.float16, size=sz))]
    base = name[:-len("_int8")]
    return [(name, getattr(S, base)(np.int8, size=sz, batch=b))]


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


def cpu_baseline(models, seconds, edge=224):
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
                sample="%d round-robin jobs of %s (%dx%d) on 1 host core, %.1f s" % (n, names, edge, edge, dt))


def workload_label(args, models, n_cpu, W, poisson):
    """config.workload: which BASELINE config (C1-C5) this run measures"""
    names = ", ".join(nm for nm, _ in models)
    edge = args.size or 224
    if args.device == "cpu":
        return ("%s%s %dx%d batch-1 jobs through the Band engine, %s over %d Band CPU worker(s) (%d threads each)"
                % ("C1: " if args.model == "mobilenet_v1_int8" and W == 1 else "", names, edge, edge,
                   args.scheduler, W, args.cpu_threads))
    if args.model == "mix_c5":
        return ("C5: 8-DNN int8 + fp16 mix (%s), open-loop Poisson arrivals at %.0f req/s per GPU, %s + "
                "latency estimator over [%d CPU, %d GPU] Band workers per MI355X"
                % (names, poisson["rate_per_s_per_gpu"], args.scheduler, n_cpu, W))
    if len(models) > 1:
        return ("C3: 4-DNN int8 mix (%s), %dx%d batch-1 jobs through the Band engine, %s over %d Band GPU "
                "worker(s) per MI355X" % (names, edge, edge, args.scheduler, W))
    if args.model == "efficientdet_lite2_int8":
        e = args.size or 448
        return ("C4: EfficientDet-Lite2 int8 %dx%d batch-1 jobs through the Band engine, model_analyzer split "
                "(network on GPU workers, TFLite_Detection_PostProcess on %d CPU worker(s)), %s over %d Band GPU "
                "worker(s) per MI355X" % (e, e, n_cpu, args.scheduler, W))
    return ("C2: %s %dx%d batch-1 jobs through the Band engine, %s over %d Band GPU worker(s) per MI355X"
            % (args.model, edge, edge, args.scheduler, W))


def profile_roofline(args, D, models, paths):
    """per-launch roofline of the dominant kernel + device time per model
    (GPU runs only)"""
    import band_amd
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
    M = len(models)
    # with job batching the workers run batch-B passes: profile those (the
    # same models with a leading batch of B), per-inference figures / B
    B = args.job_batch if args.job_batch > 1 and args.model not in ("efficientdet_lite2_int8", "mix_c5") else 1
    if B > 1:
        paths = []
        for name, buf in model_list(args.model, args.size, batch=B):
            tmp = tempfile.NamedTemporaryFile(prefix="band_prof_%s_" % name, suffix=".tflite", delete=False)
            tmp.write(buf)
            tmp.close()
            paths.append(tmp.name)
    # profiling executors (outside the engine, same backend code) for the
    # per-kernel roofline and the device-side floor of a job
    prof_wid = 1000
    band_amd.SetWorkerDevice(prof_wid, D.local_rank)
    execs0, keys0 = [], []
    for mid, path in enumerate(paths):
        hm = HipModel(100 + mid)
        assert hm.FromPath(path).ok()
        ex = HipModelExecutor(100 + mid, prof_wid, DeviceFlag.kGPU)
        if args.no_graph:
            ex.SetUseGraph(False)
        spec = ex.InvestigateModelSpec(hm)
        gpu_ops = [i for i in range(spec.num_ops) if i not in spec.unsupported_ops[DeviceFlag.kGPU]]
        # a split model: profile its GPU part (ops before the first CPU-only op)
        assert ex.PrepareSubgraph(hm, gpu_ops if len(gpu_ops) < spec.num_ops else ()).ok()
        execs0.append(ex)
        keys0.append(SubgraphKey(100 + mid, prof_wid))
        ex._model_ref = hm

    # roofline of the dominant kernel: per-launch HIP events on the worker's
    # stream, over one inference of each model (the mix is uniform)
    by_k = {}
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
    device_us = {name: ex.TimeSubgraph(key, iters=100) / B for (name, _), ex, key in zip(models, execs0, keys0)}
    if B > 1:
        for path in paths:
            os.unlink(path)
    # per inference: kernel time of a batch-B pass / B
    for k in by_k.values():
        for f in ("ms", "bytes", "ops", "launches"):
            k[f] /= B
    return dom_name, dom, by_k, traffic, traffic_src, device_us, B


def make_engine(args, D, paths, sched, workers, n_cpu, W, job_batch):
    """this rank's Band engine with the models registered and one synthetic
    request tensor per model"""
    from band_amd.engine import Engine, Model, make_config
    on_gpu = args.device == "gpu"
    engine = Engine(make_config([sched], workers,
                                num_threads=[args.cpu_threads] * n_cpu + [1 if on_gpu else args.cpu_threads] * W,
                                num_warmups=3, num_runs=5,
                                max_job_batch=job_batch if job_batch > 1 else None))
    band_models, inputs = [], []
    rng = np.random.default_rng(5489 + D.rank)
    for path in paths:
        m = Model()
        assert m.FromPath(path), path
        assert engine.RegisterModel(m), path
        band_models.append(m)
        # synthetic requests: int8 U{-127..127} / uint8 U{0..254} (band/tool/benchmark.cc:279-287)
        t = engine.CreateInputTensor(m, 0)
        arr = t.data()
        if arr.dtype == np.float32:  # f32 U(-0.5, 0.5) (band/tool/benchmark.cc:279-287)
            arr[...] = rng.uniform(-0.5, 0.5, arr.shape).astype(np.float32)
        else:
            lo, hi = (-127, 128) if arr.dtype == np.int8 else (0, 255)
            arr[...] = rng.integers(lo, hi, arr.shape).astype(arr.dtype)
        inputs.append(t)
    return engine, band_models, inputs


def main():
    args = parse()
    # hardware queues are fixed at HIP runtime init: one per concurrently
    # running Band GPU worker stream (must be set before libband_hip loads)
    # (explicit assignment: the GPU box exports HIP's default of 4)
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(32, args.hw_queues)))
    D = Dist()
    import band_amd
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
    from band_amd.engine import Engine, Model, SchedulerType, make_config

    models = model_list(args.model, args.size)
    M = len(models)
    W = max(1, args.workers_per_gpu)
    paths = []
    for name, buf in models:
        tmp = tempfile.NamedTemporaryFile(prefix="band_bench_%s_" % name, suffix=".tflite", delete=False)
        tmp.write(buf)
        tmp.close()
        paths.append(tmp.name)
    if args.no_graph:
        os.environ["BAND_HIP_GRAPH"] = "0"

    # this rank's Band engine: [CPU workers] + W GPU workers, all GPU
    # workers on the local MI355X (worker id -> device ordinal; each worker
    # owns one HIP stream)
    needs_cpu = args.model in ("efficientdet_lite2_int8", "mix_c5")
    n_cpu = args.cpu_workers if args.cpu_workers >= 0 else (1 if needs_cpu else 0)
    if args.model == "mix_c5" and args.scheduler == "round_robin":
        args.scheduler = "shortest_expected_latency"  # C5: SEL + latency estimator
    on_gpu = args.device == "gpu"
    if not on_gpu:
        n_cpu = 0
    workers = [DeviceFlag.kCPU] * n_cpu + [DeviceFlag.kGPU if on_gpu else DeviceFlag.kCPU] * W
    for w in range(n_cpu, n_cpu + W):
        if on_gpu:
            band_amd.SetWorkerDevice(w, D.local_rank)
    sched = {"round_robin": SchedulerType.kRoundRobin, "fixed_worker": SchedulerType.kFixedWorker,
             "shortest_expected_latency": SchedulerType.kShortestExpectedLatency,
             "heterogeneous_earliest_finish_time": SchedulerType.kHeterogeneousEarliestFinishTime}[args.scheduler]
    if n_cpu and args.scheduler in ("round_robin", "fixed_worker"):
        sched = SchedulerType.kHeterogeneousEarliestFinishTime  # a split model needs fallback subgraphs
        args.scheduler = "heterogeneous_earliest_finish_time"
    if not (on_gpu and n_cpu == 0 and args.scheduler == "round_robin"):
        args.job_batch = 1  # job batching applies to round_robin over GPU workers only
    batching = args.job_batch > 1
    engine, band_models, inputs = make_engine(args, D, paths, sched, workers, n_cpu, W, args.job_batch)
    # 2 x workers x job batch requests in flight, at most 120 per model: Band's
    # per-model output ring buffers hold 128 slots (TensorRingBuffer), and a
    # request whose slot was reused before its output was copied fails
    inflight = args.inflight or min(2 * W * (args.job_batch if batching else 1), 120 * M)

    engine.RunClosedLoop(band_models, max(args.warmup, 2 * W * M), inflight, inputs)
    poisson = None
    if args.model == "mix_c5":
        # C5: open-loop Poisson arrivals at 0.8 x this engine's closed-loop capacity
        # (or --rate), uniform over the 8 models
        rate = args.rate
        if rate <= 0:
            _, _, cap_wall = engine.RunClosedLoop(band_models, max(args.steps // 4, 8 * M), inflight, inputs)
            rate = 0.8 * max(args.steps // 4, 8 * M) / cap_wall
        poisson = dict(rate_per_s_per_gpu=rate, seed=5489 + D.rank)
    D.barrier()
    t0 = time.perf_counter()
    if poisson:
        lat_us, worker_ids, model_idx, _ = engine.RunPoisson(band_models, args.steps, poisson["rate_per_s_per_gpu"],
                                                            seed=poisson["seed"], max_inflight=max(64, inflight),
                                                            inputs=inputs)
    else:
        lat_us, worker_ids, _ = engine.RunClosedLoop(band_models, args.steps, inflight, inputs)
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.max(t1 - t0)
    all_lat = [x for part in D.gather((lat_us * 1e-6).tolist()) for x in part]
    jobs_per_worker = np.bincount(worker_ids, minlength=n_cpu + W).tolist()
    engine.close()

    # Band's own semantics beside it: one job per ExecuteSubgraph (no job
    # batching), the same mix and scheduler over 8 GPU workers per GPU
    batch1 = None
    # (only where job batching applies: round_robin over GPU workers alone)
    if batching and not poisson and not args.no_batch1:
        W1 = 8
        e1, bm1, in1 = make_engine(args, D, paths, sched, [DeviceFlag.kGPU] * W1, 0, W1, 1)
        n1 = max(args.steps // 2, 16 * M)
        e1.RunClosedLoop(bm1, max(args.warmup // 2, 2 * W1 * M), 2 * W1, in1)
        D.barrier()
        t0 = time.perf_counter()
        lat1, _, _ = e1.RunClosedLoop(bm1, n1, 2 * W1, in1)
        t1 = time.perf_counter()
        D.barrier()
        el1 = D.max(t1 - t0)
        l1 = np.array([x for part in D.gather((lat1 * 1e-3).tolist()) for x in part])
        batch1 = {"value": n1 * D.world / el1, "unit": "inferences/s", "workers_per_gpu": W1, "steps": n1,
                  "p50_job_latency_ms": float(np.percentile(l1, 50)),
                  "p99_job_latency_ms": float(np.percentile(l1, 99))}
        e1.close()

    roof, dev = None, None
    if on_gpu:
        dom_name, dom, by_k, traffic, traffic_src, device_us, prof_batch = profile_roofline(args, D, models, paths)
        avg_ms = dom["ms"] / dom["launches"]
        bytes_per_launch = dom["bytes"] / dom["launches"]
        ops_per_launch = dom["ops"] / dom["launches"]
        achieved_gbs = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        roof = {
            "kernel": dom_name, "bound": "hbm", "achieved": achieved_gbs, "peak": 8000.0, "unit": "GB/s",
            "frac": achieved_gbs / 8000.0, "traffic": traffic, "traffic_source": traffic_src,
            "alg_bytes_per_launch": bytes_per_launch, "avg_launch_us": avg_ms * 1e3,
            "launches_per_inference": dom["launches"],
            "profiled_pass_batch": prof_batch,
            "mfma_i8_tops": ops_per_launch / (avg_ms * 1e-3) / 1e12,
            "mfma_i8_frac": ops_per_launch / (avg_ms * 1e-3) / 5.0e15,
        }
        dev = dict(gpu_ms_total=sum(v["ms"] for v in by_k.values()), device_us=device_us)

    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(models, args.cpu_baseline_seconds, args.size or 224)

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
            "dtype": "uint8" if args.model.endswith("uint8") else ("int8+fp16" if args.model == "mix_c5" else "int8"),
            "data": "synthetic (seeded inputs and weights; no checkpoint)",
            "device": args.device,
            "config": {"workload": workload_label(args, models, n_cpu, W, poisson) + (
                           "; each GPU worker runs up to %d queued jobs of one model as one batched pass "
                           "(job batching)" % args.job_batch if args.job_batch > 1 else ""),
                       "harness": "native Band engine (planner + workers + %s), %d requests in flight"
                                  % (args.scheduler, inflight),
                       "jobs_per_worker_rank0": jobs_per_worker,
                       "max_job_batch": args.job_batch,
                       "model": args.model, "global_batch": n * W * max(1, args.job_batch), "seq_len": None,
                       "parallelism": "job-sharded x%d (no collective)" % n, "hipgraph": not args.no_graph,
                       "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))},
            "p50_job_latency_ms": float(np.percentile(lat_ms, 50)),
            "p99_job_latency_ms": float(np.percentile(lat_ms, 99)),
            "gpu_kernel_ms_per_inference": dev["gpu_ms_total"] if dev else None,
            "device_us_per_inference": float(np.mean(list(dev["device_us"].values()))) if dev else None,
            "device_us_per_model": dev["device_us"] if dev else None,
            "band_one_job_per_pass": batch1,
            "roofline": roof,
            "cpu_baseline": cpu,
            "host": platform.node(),
        }
        print(json.dumps(line), flush=True)
    for path in paths:
        os.unlink(path)
    D.close()


if __name__ == "__main__":
    main()
