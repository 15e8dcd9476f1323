#!/usr/bin/env python3
"""Headline benchmark: multi-DNN inferences/s + p99 job latency (BASELINE.json).

Workload (default, N=1): BASELINE config C3 - the 4-DNN int8 mix
(MobileNetV2, SSD-MobileNetV2, DeepLabV3-MobileNetV2, PoseNet-MobileNetV1;
224x224, synthetic seeded weights with TFLite-converter-shaped quantisation)
served by the native Band engine (band_amd/csrc/engine) with round_robin over
`--workers-per-gpu` Band GPU workers of one MI355X (AddWorkers({kGPU, ...})).
`--model mobilenet_v2_int8` etc. run single-model configs (C2); C4 / C5 have
their own models (`efficientdet_lite2_int8`, `mix_c5`).

A job is one Band request end to end through the harness: RequestAsync (user
tensor -> request ring, band/engine.cc:455-529) -> planner thread ->
scheduler -> worker queue (band/planner.cc:268-365) -> Worker::Work: input
copy into the executor's view, IModelExecutor::ExecuteSubgraph on the GPU,
output copy (band/worker.cc:222-323) -> Wait.  A native closed-loop driver
(BandxEngineRunClosedLoop) keeps 1.25 x workers x job-batch requests in
flight (2 x workers with one job per pass); the engine's request rings apply
back-pressure beyond 128 per model.

A STEP is one round of `--jobs-per-step` jobs (default 1024, 256 of each mix
model): `--steps K --warmup W` times exactly K x 1024 jobs after W x 1024
warm-up jobs, so the driver's `--steps 20 --warmup 5` times 20,480 jobs in
steady state.  Job latency = end - enqueue of the planner's job record
(band/common.h:351-353).

Job batching (--job-batch B, default 32; BANDX_WORKER_MAX_JOB_BATCH): an
idle GPU worker takes up to B queued requests of one model from round_robin
and runs them as ONE pass over a batch-B variant of the model's subgraph
(every job still gets its own input copy, its own outputs, its own job
record).  The pass-size policy (--pass-target-us, default 700;
BANDX_WORKER_PASS_TARGET_US) caps a model's pass at the jobs whose expected
pass time fits the target, so the slowest model of the mix (DeepLab, whose
32-job pass is ~1.3 ms) does not set every job's latency tail.  Band itself runs one job per ExecuteSubgraph; that configuration
(8 GPU workers, no batching) is measured in the same run and reported as
"band_one_job_per_pass"; "latency_point" is the same engine with smaller
passes and fewer requests in flight (--latency-point, default job batch 24,
450 us pass target, 200 in flight), the tail-latency side of the trade.

N>1 (torchrun, one process per GPU): each rank serves its own job stream
with its own engine over its GPU; jobs shard across GPUs with no data-path
collective (weak scaling); a gloo group only provides the barrier and the
max-over-ranks timing.  After that line is measured, rank 0 alone runs ONE
Band engine whose GPU workers span all N GPUs (worker w -> GPU w % N,
round_robin, Band's single planner thread) and reports it as
"single_engine" beside the per-process value (the other ranks have closed
their engines and wait at the barrier).  `--single-engine` makes that the
headline.  The GPU is driven exclusively through libband_hip.so.

Roofline: every launch of the profiled passes (the same models at the job
batch) is timed in program order on the executor's stream
(HipModelExecutor::ProfileSubgraph): each kernel carries HIP events that
hold its own dispatch begin / end timestamps (hipExtLaunchKernel), the
kernel-only duration rocprofv3's kernel trace reports.  The dominant kernel
(largest total time) and the next two are reported with their algorithmic
bytes and ops per launch.

Prints ONE JSON line on rank 0.  `--profile-only` runs just the profiled
passes (for rocprofv3 kernel traces / PMC passes of exactly those launches).
"""
import argparse
import glob
import hashlib
import json
import os
import platform
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20, help="timed steps (one step = --jobs-per-step jobs)")
    p.add_argument("--warmup", type=int, default=5, help="untimed warm-up steps")
    p.add_argument("--jobs-per-step", type=int, default=1024)
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
    p.add_argument("--fresh-tuning", action="store_true",
                   help="let the fusion tuner measure every choice in this process instead of replaying the "
                        "committed profile set's decisions (profiles/<tag>_tune.tsv of the PMC traffic file that "
                        "matches this kernel tree)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--sample-threads", action="store_true",
                   help="diagnostics: sample every thread's /proc state through the timed loop")
    p.add_argument("--no-roofline", action="store_true",
                   help="skip the per-launch roofline / device-time profile (e.g. under a rocprofv3 trace)")
    p.add_argument("--cpu-baseline-seconds", type=float, default=8.0, help="per CPU-baseline mode")
    p.add_argument("--profile-iters", type=int, default=20)
    p.add_argument("--scheduler", default="round_robin",
                   choices=["round_robin", "fixed_worker", "shortest_expected_latency",
                            "heterogeneous_earliest_finish_time"])
    p.add_argument("--inflight", type=int, default=0,
                   help="outstanding requests (default 1.25 x workers x job batch; 2 x workers without batching)")
    p.add_argument("--device", default="gpu", choices=["gpu", "cpu"],
                   help="cpu: --workers-per-gpu Band CPU workers instead of GPU workers (C1 / CPU tests; no roofline)")
    p.add_argument("--size", type=int, default=0, help="input edge (default 224; EfficientDet 448)")
    p.add_argument("--no-batch1", action="store_true",
                   help="skip the one-job-per-pass (Band semantics) line reported beside a job-batched run")
    p.add_argument("--band1-workers", type=int, default=48,
                   help="GPU workers per GPU of the band_one_job_per_pass line (Band's own contract)")
    p.add_argument("--job-batch", type=int, default=32,
                   help="max queued jobs of one model a GPU worker runs as one batched pass "
                        "(BANDX_WORKER_MAX_JOB_BATCH; 1 = Band's one job per ExecuteSubgraph)")
    p.add_argument("--pass-target-us", type=int, default=700,
                   help="pass-size policy of job batching (BANDX_WORKER_PASS_TARGET_US): a model's pass takes at "
                        "most the jobs whose expected pass time fits this many microseconds (0 = off)")
    p.add_argument("--latency-point", default="24,450,200",
                   help="JOB_BATCH,PASS_TARGET_US,INFLIGHT of the latency_point line beside a job-batched N = 1 "
                        "headline (the same engine with smaller passes and fewer requests in flight); '' = skip")
    p.add_argument("--share-profiles", type=int, default=-1, choices=[-1, 0, 1],
                   help="BANDX_PROFILE_SHARE_IDENTICAL: identical workers share latency estimates; -1 (default) = "
                        "on for the latency-driven schedulers (SEL / HEFT: C4, C5), 0 = the reference's "
                        "per-worker estimates")
    p.add_argument("--single-engine", action="store_true",
                   help="headline = one process, one Band engine, GPU workers over all --gpus GPUs")
    p.add_argument("--no-single-engine", action="store_true", help="N>1: skip the single-engine line")
    p.add_argument("--per-process-headline", action="store_true",
                   help="N>1: keep the per-process line (one engine per GPU) as the headline")
    p.add_argument("--single-engine-wpg", type=int, default=0,
                   help="--single-engine: GPU workers per GPU (default --workers-per-gpu; 1 = one Worker per GPU)")
    p.add_argument("--profile-only", action="store_true",
                   help="run only the profiled batch passes (rocprofv3 traces); prints their per-kernel table")
    return p.parse_args()


def default_inflight(workers, job_batch):
    """requests the closed loop keeps in flight: 1.25 x workers x job batch
    (a pass's worth per worker plus a quarter queued: in-flight 384 -> 320 at
    8 x 32 cut p99 4.5 -> 4.2 ms at equal throughput, profiles/r06g_*), or
    2 x workers with one job per pass; the engine's request rings hold back
    a model's 129th unfinished request"""
    if job_batch > 1:
        return max(2 * workers, int(1.25 * workers * job_batch))
    return 2 * workers


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


def write_models(models, prefix):
    paths = []
    for name, buf in models:
        tmp = tempfile.NamedTemporaryFile(prefix="%s_%s_" % (prefix, name), suffix=".tflite", delete=False)
        tmp.write(buf)
        tmp.close()
        paths.append(tmp.name)
    return paths


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


def host_cores():
    """host cores this process may use: its affinity set, capped by the
    per-job CPU share the box grants (OMP_NUM_THREADS, 16 on the GPU box) and
    by the container's cgroup CPU quota"""
    n = len(os.sched_getaffinity(0))
    try:
        cap = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        cap = 0
    n = min(n, cap) if cap > 0 else n
    quota, _ = cgroup_cpu_quota()
    return max(1, min(n, int(quota))) if quota else n


def cgroup_cpu_quota():
    """the container's CPU quota in CPUs (cgroup v2 cpu.max, or v1
    cpu.cfs_quota_us / cpu.cfs_period_us), None when unlimited or unknown"""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            return (None if q == "max" else round(int(q) / int(per), 2)), path
        except (OSError, ValueError):
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return (None if q < 0 else round(q / per, 2)), "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"
    except (OSError, ValueError):
        return None, None


_START_AFFINITY = None


def host_info():
    """nproc / lscpu facts of the host, read from /proc (no subprocess)"""
    global _START_AFFINITY
    if _START_AFFINITY is None:
        _START_AFFINITY = os.sched_getaffinity(0)
    quota, qsrc = cgroup_cpu_quota()
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cgroup_cpu_quota": quota, "cgroup_cpu_source": qsrc}
    try:
        with open("/proc/cpuinfo") as f:
            txt = f.read()
        models = [l.split(":", 1)[1].strip() for l in txt.splitlines() if l.startswith("model name")]
        phys = {(l1, l2) for l1, l2 in zip([l for l in txt.splitlines() if l.startswith("physical id")],
                                           [l for l in txt.splitlines() if l.startswith("core id")])}
        info["cpu_model"] = models[0] if models else platform.processor()
        info["physical_cores_total"] = len(phys) or None
    except OSError:
        pass
    return info


def cpu_baseline(args, models, paths, seconds):
    """The product's own kCPU path (the same lowered program and integer
    arithmetic on the host, backend/hip/cpu_kernels.cc) through the same Band
    harness, as BASELINE.md section 2 prescribes: (i) one CPU worker with
    every core as its thread pool, (ii) one single-threaded CPU worker per
    core; round_robin over the same models and request stream, each mode run
    for about `seconds`.  Plus the scalar oracle port on one core (test
    infrastructure, kept as a reference point)."""
    from band_amd import DeviceFlag
    from band_amd.engine import Engine, Model, SchedulerType, make_config
    # the GPU path pins the threads that call it to the GPU's NUMA node
    # (backend/hip/affinity.h); the CPU workers of this baseline are created
    # from this thread, so it goes back to the process's starting CPU set
    if _START_AFFINITY:
        os.sched_setaffinity(0, _START_AFFINITY)
    T = host_cores()
    M = len(models)
    modes = []
    for label, n_workers, threads in (("1 CPU worker x %d threads" % T, 1, T),
                                      ("%d CPU workers x 1 thread" % T, T, 1)):
        prof = os.path.join(tempfile.gettempdir(), "band_bench_cpu_profile_%d.json" % os.getpid())
        e = Engine(make_config([SchedulerType.kRoundRobin], [DeviceFlag.kCPU] * n_workers,
                               num_threads=[threads] * n_workers, online=False, profile_path=prof))
        ms, ins = [], []
        rng = np.random.default_rng(5489)
        for path in paths:
            m = Model()
            assert m.FromPath(path), path
            assert e.RegisterModel(m), path
            t = e.CreateInputTensor(m, 0)
            arr = t.data()
            lo, hi = (-127, 128) if arr.dtype == np.int8 else (0, 255)
            arr[...] = rng.integers(lo, hi, arr.shape).astype(arr.dtype)
            ms.append(m)
            ins.append(t)
        inflight = 2 * n_workers
        n0 = max(M, 2 * n_workers) // M * M
        _, _, w0 = e.RunClosedLoop(ms, n0, inflight, ins)  # warm + calibrate
        n = max(n0, int(seconds * n0 / max(w0, 1e-6)) // M * M)
        lat, _, wall = e.RunClosedLoop(ms, n, inflight, ins)
        modes.append(dict(mode=label, workers=n_workers, threads_per_worker=threads, value=n / wall, jobs=n,
                          seconds=wall, p99_job_latency_ms=float(np.percentile(lat * 1e-3, 99))))
        e.close()
    best = max(modes, key=lambda m: m["value"])
    # scalar oracle port (test infrastructure) on one core, a short sample
    from oracle.runner import OracleInterpreter, lib as oracle_lib
    from oracle.tflite_fb import Model as OModel
    oracle_lib().tfl_set_num_threads(1)  # the scalar port on ONE core
    rng = np.random.default_rng(5489)
    runs = []
    for _, buf in models:
        om = OModel(buf)
        t_in = om.tensors[om.inputs[0]]
        lo, hi = (-127, 128) if t_in.np_dtype == np.int8 else (0, 255)
        runs.append((OracleInterpreter(om), {om.inputs[0]: rng.integers(lo, hi, t_in.shape).astype(t_in.np_dtype)}))
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < min(3.0, seconds) or n < len(runs):
        interp, feed = runs[n % len(runs)]
        interp.run(feed)
        n += 1
    oracle = dict(value=n / (time.perf_counter() - t0), cores=1, jobs=n)
    oracle_lib().tfl_set_num_threads(0)
    names = "+".join(name for name, _ in models)
    return dict(value=best["value"], unit="inferences/s", cores=T, kind="port",
                sample="Band engine kCPU workers (the product's host kernels), round_robin over %s 224x224 int8; "
                       "best of BASELINE.md modes (i) 1 worker x %d threads and (ii) %d workers x 1 thread, ~%.0f s "
                       "each; best: %s" % (names, T, T, seconds, best["mode"]),
                modes=modes, oracle_scalar_port_1core=oracle, host=host_info(),
                cores_reason="min(affinity, OMP_NUM_THREADS, cgroup quota): the GPU box grants each GPU job a "
                             "16-CPU share (OMP_NUM_THREADS=16 there, and pools are to be sized to it), so BASELINE.md's "
                             "'all physical cores' becomes the job's share; the host's own core count is reported "
                             "beside it")


def kernel_source_tag():
    """hash of the kernel sources and their build recipe (compiler flags
    change the code): PMC traffic figures are only reported for the tree
    they were measured on"""
    h = hashlib.sha1()
    for f in sorted(glob.glob(os.path.join(ROOT, "band_amd", "csrc", "kernels", "*"))) + \
            [os.path.join(ROOT, "include", "band_hip_kernels.h"), os.path.join(ROOT, "band_amd", "csrc", "Makefile")]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def replay_tuning():
    """The fusion tuner's decisions of the committed profile set whose PMC
    traffic file matches this kernel tree (BAND_HIP_TUNE_FILE, copied to a
    scratch file the tuner may append to): the headline then runs the chain
    forms the traffic was measured on, so `roofline.traffic` describes the
    same launches; otherwise close calls between forms flip from process to
    process.  Returns the source file or None."""
    if os.environ.get("BAND_HIP_TUNE_FILE"):
        return None
    tag = kernel_source_tag()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json"))):
        try:
            with open(f) as fh:
                meta = json.load(fh).get("_meta", {})
        except (OSError, ValueError):
            continue
        # (.tsv: the committed copy travels to the GPU box, profiles/*.txt do not)
        tunes = [f[:-len("_pmc_traffic.json")] + "_tune" + ext for ext in (".tsv", ".txt")]
        tune = next((t for t in tunes if os.path.exists(t)), None)
        if meta.get("kernel_source_tag") == tag and tune:
            import shutil
            import tempfile
            fd, scratch = tempfile.mkstemp(prefix="band_tune_", suffix=".txt")
            os.close(fd)
            shutil.copyfile(tune, scratch)
            os.environ["BAND_HIP_TUNE_FILE"] = scratch

            def _drop(path=scratch):
                try:
                    os.unlink(path)
                except OSError:
                    pass
            import atexit
            atexit.register(_drop)
            return os.path.relpath(tune, ROOT)
    return None


def profiled_batch(args):
    return args.job_batch if args.job_batch > 1 and args.model not in ("efficientdet_lite2_int8", "mix_c5") else 1


def profile_executors(args, D, models, paths, batch=None):
    """profiling executors (outside the engine, same backend code) over the
    passes the workers run: with job batching, the same models with a
    leading batch of B (`batch` overrides it)"""
    import band_amd
    from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey
    B = batch or profiled_batch(args)
    tmp = []
    if B > 1:
        paths = tmp = write_models(model_list(args.model, args.size, batch=B), "band_prof")
    prof_wid = 1000
    band_amd.SetWorkerDevice(prof_wid, D.local_rank)
    execs = []
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
        ex._model_ref = hm
        execs.append((ex, SubgraphKey(100 + mid, prof_wid)))
    for path in tmp:
        os.unlink(path)
    return execs, B


def profile_roofline(args, D, models, paths):
    """per-launch roofline of the dominant kernels + device time per model
    (GPU runs only)"""
    execs, B = profile_executors(args, D, models, paths)
    M = len(models)
    by_k, floors = {}, []
    for ex, key in execs:
        rows, empty_us = ex.ProfileSubgraph(key, iters=args.profile_iters, with_floor=True)
        floors.append(empty_us)
        for r in rows:
            # group by kernel symbol ("conv_mfma_kernel+add" is conv_mfma_kernel
            # with its residual epilogue), as rocprofv3 reports them
            k = by_k.setdefault(r["kernel"].split("+")[0], dict(us=0.0, bytes=0.0, ops=0.0, launches=0))
            k["us"] += r["ms"] * 1e3
            k["bytes"] += r["alg_bytes"]
            k["ops"] += r["alg_ops"]
            k["launches"] += 1
    # device-side floor of one job: each model's passes replayed back to back
    # (graph incl. H2D/D2H), no host gaps; the rest of the job latency is
    # host launch + sync wakeup
    # (one untimed round first: the first replay after an idle GPU runs at a
    # lower clock - the first model timed read ~2x its eager time,
    # profiles/r04o_breakdown_b24.txt)
    for ex, key in execs:
        ex.TimeSubgraph(key, iters=20)
    device_us = {name: ex.TimeSubgraph(key, iters=100) / B for (name, _), (ex, key) in zip(models, execs)}
    total_us = sum(k["us"] for k in by_k.values())
    ranked = sorted(by_k.items(), key=lambda kv: -kv[1]["us"])
    # HBM traffic per launch from the committed rocprofv3 PMC passes
    # (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE, the gfx950
    # corrections of MI355X_MICROARCH.md), only when measured on this
    # kernel source tree and at this pass batch
    tag = kernel_source_tag()
    pmc = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json"))):
        with open(f) as fh:
            tj = json.load(fh)
        meta = tj.get("_meta", {})
        if meta.get("kernel_source_tag") == tag and meta.get("pass_batch") == B:
            pmc = dict(tj, _file=os.path.basename(f))

    def roof(name, k):
        us = k["us"] / k["launches"]
        b = k["bytes"] / k["launches"]
        o = k["ops"] / k["launches"]
        gbs = b / (us * 1e-6) / 1e9
        t = pmc.get(name, {}).get("traffic_bytes_per_launch")
        return {"kernel": name, "bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
                "traffic": t, "traffic_over_algorithmic": (t / b) if t else None,
                "traffic_source": pmc.get("_file") if t else
                "null: no PMC file measured on this kernel tree (tag %s) at pass batch %d" % (tag, B),
                "alg_bytes_per_launch": b, "alg_ops_per_launch": o, "avg_launch_us": us,
                "launches_per_pass": k["launches"] / M, "share_of_kernel_time": k["us"] / total_us,
                "mfma_i8_tops": o / (us * 1e-6) / 1e12, "mfma_i8_frac": o / (us * 1e-6) / 5.0e15,
                # achieved / min(P_mfma, AI x BW_hbm), the attainable
                # rate at this kernel's arithmetic intensity (algorithmic ops / bytes)
                "arith_intensity_op_per_byte": o / b if b else None,
                "attainable_tops": min(5.0e15, (o / b) * 8.0e12) / 1e12 if b else None,
                "attainable_frac": (o / (us * 1e-6)) / min(5.0e15, (o / b) * 8.0e12) if b and o else None}

    top = [roof(n, k) for n, k in ranked[:6]]
    dom = dict(top[0])
    dom.update(profiled_pass_batch=B, timing="per-dispatch begin/end timestamps (hipExtLaunchKernel events)",
               empty_kernel_us=float(np.mean(floors)), kernel_source_tag=tag, next_kernels=top[1:])
    return dom, dict(gpu_us_per_inference=total_us / M / B, device_us=device_us), execs


def profile_only(args, D, models, paths):
    """only the profiled passes (graph replays of the batch-B variants),
    for rocprofv3: its per-kernel averages then describe exactly the launches
    the roofline line reports"""
    dom, dev, _ = profile_roofline(args, D, models, paths)
    print(json.dumps({"profile_only": True, "pass_batch": profiled_batch(args), "roofline": dom, "device": dev}),
          flush=True)


def make_engine(args, D, paths, sched, workers, n_cpu, W, job_batch, seed_offset=0):
    """a Band engine with the models registered and one synthetic request
    tensor per model"""
    from band_amd.engine import Engine, Model, make_config
    on_gpu = args.device == "gpu"
    engine = Engine(make_config([sched], workers,
                                num_threads=[args.cpu_threads] * n_cpu + [1 if on_gpu else args.cpu_threads] * W,
                                num_warmups=3, num_runs=5,
                                max_job_batch=job_batch if job_batch > 1 else None,
                                share_identical=(args.share_profiles > 0) if args.share_profiles >= 0 else None,
                                pass_target_us=args.pass_target_us if job_batch > 1 else None))
    band_models, inputs = [], []
    rng = np.random.default_rng(5489 + seed_offset)
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


def thread_cpu():
    """CPU seconds (user + system) of every thread of this process, keyed by
    (tid, name): the engine names its threads band-planner, band-w<id> and
    bandx-waiter; the closed-loop submitter is the calling (python) thread"""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open("/proc/self/task/%s/stat" % tid) as f:
                raw = f.read()
            st = raw.rsplit(")", 1)[1].split()
            name = raw[raw.index("(") + 1:raw.rindex(")")]
            if int(tid) == os.getpid():
                name += "(main)"  # unnamed runtime threads inherit the process name
            out[(tid, name)] = (int(st[11]) + int(st[12])) / tick
        except (OSError, ValueError):
            pass
    return out


HOST_THREADS = {}
HOST_THREAD_STATES = {}
COALESCE = {}  # backend job coalescing over the last timed loop (coalescer.h)
LAST_MODEL_IDX = []  # the model index of every job of the last timed closed loop (driver-reported)


def cgroup_cpu_stat():
    """cgroup v2 cpu.stat counters (usage / throttling), {} when absent"""
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def cgroup_delta(g0, g1, dt):
    """the container's CPU use (cores) and CFS throttling over a timed region"""
    return dict(usage_cores=round((g1.get("usage_usec", 0) - g0.get("usage_usec", 0)) * 1e-6 / dt, 2),
                throttled_share=round((g1.get("throttled_usec", 0) - g0.get("throttled_usec", 0)) * 1e-6 / dt, 3),
                nr_throttled=g1.get("nr_throttled", 0) - g0.get("nr_throttled", 0))


SAMPLE_THREADS = False


class ThreadSampler:
    """Diagnostics (--sample-threads): a Python thread reads every thread's
    /proc/self/task/<tid>/syscall each ~0.5 ms while the native loop runs
    (the GIL is released there): 'running' (user space), or the syscall it is
    blocked in and the library its PC falls in.  Answers what an unnamed
    runtime thread near 1.0 CPU is doing."""

    def __init__(self):
        import threading
        self.counts = {}
        self.stop_flag = False
        self.maps = []
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6 and "x" in parts[1]:
                    lo, hi = (int(x, 16) for x in parts[0].split("-"))
                    self.maps.append((lo, hi, os.path.basename(parts[5])))
        self.th = threading.Thread(target=self.run, daemon=True)
        self.th.start()

    def lib_of(self, pc):
        for lo, hi, name in self.maps:
            if lo <= pc < hi:
                return name
        return "?"

    def run(self):
        while not self.stop_flag:
            for tid in os.listdir("/proc/self/task"):
                try:
                    with open("/proc/self/task/%s/comm" % tid) as f:
                        name = f.read().strip()
                    with open("/proc/self/task/%s/syscall" % tid) as f:
                        sc = f.read().split()
                except OSError:
                    continue
                if not sc:
                    continue
                if sc[0] == "running":
                    state = "running"
                else:
                    state = "sys%s@%s" % (sc[0], self.lib_of(int(sc[-1], 16)) if len(sc) > 2 else "?")
                key = "%s/%s" % (name, tid)
                d = self.counts.setdefault(key, {})
                d[state] = d.get(state, 0) + 1
            time.sleep(0.0005)

    def stop(self):
        self.stop_flag = True
        self.th.join()
        out = {}
        for k, d in self.counts.items():
            n = sum(d.values())
            if d.get("running", 0) / n > 0.05 or k.startswith("python"):
                out[k] = {s: round(c / n, 3) for s, c in sorted(d.items(), key=lambda x: -x[1])[:4]}
        return out


def run_closed(engine, band_models, inputs, n_warm, n_timed, inflight, D):
    """warm-up, barrier, exactly n_timed jobs, barrier; max over ranks.  The
    CPU share of each host thread over the timed loop goes to HOST_THREADS
    (a thread near 1.0 is a host-side ceiling)"""
    engine.RunClosedLoop(band_models, n_warm, inflight, inputs)
    D.barrier()
    n_workers = engine.GetNumWorkers()
    p0 = [engine.GetWorkerPhaseTimes(w) for w in range(n_workers)]
    r0 = engine.GetRequestPhaseTimes()
    c0 = thread_cpu()
    g0 = cgroup_cpu_stat()
    sampler = ThreadSampler() if SAMPLE_THREADS else None
    coalesce = None
    try:
        from band_amd import backend as _backend
        coalesce = _backend.CoalescerStats
        coalesce(reset=True)
    except Exception:  # the CPU-only stand-in runs have no HIP library loaded
        coalesce = None
    t0 = time.perf_counter()
    lat_us, worker_ids, model_idx, _ = engine.RunClosedLoop(band_models, n_timed, inflight, inputs,
                                                            with_models=True)
    t1 = time.perf_counter()
    LAST_MODEL_IDX[:] = [int(v) for v in model_idx]
    COALESCE.clear()
    if coalesce:
        cs = coalesce()
        if cs["calls"]:
            cs["mean_jobs_per_group_pass"] = round(cs["group_jobs"] / max(1, cs["group_passes"]), 2)
            cs["share_of_jobs_coalesced"] = round(cs["group_jobs"] / cs["calls"], 3)
        COALESCE.update(cs)
    c1 = thread_cpu()
    g1 = cgroup_cpu_stat()
    if sampler:
        HOST_THREAD_STATES.clear()
        HOST_THREAD_STATES.update(sampler.stop())
    p1 = [engine.GetWorkerPhaseTimes(w) for w in range(n_workers)]
    drv = engine.GetDriverStats()
    r1 = engine.GetRequestPhaseTimes()
    D.barrier()
    busy = sorted((((c1[k] - c0.get(k, 0.0)) / (t1 - t0), k[1]) for k in c1), reverse=True)
    HOST_THREADS.clear()
    HOST_THREADS.update(busiest=[[n, round(b, 3)] for b, n in busy[:12]],
                        process_cpu_cores=round(sum(b for b, _ in busy), 2))
    # the container's CPU quota: time its threads were throttled (CFS) and its
    # whole CPU use over the loop (cores), when cgroup v2 reports them
    if g0 and g1:
        HOST_THREADS.update(cgroup=cgroup_delta(g0, g1, t1 - t0))
    # where the workers' wall time went over the timed loop (fractions of
    # workers x wall): input copies, invoke (launch + device sync), output
    # copies; the rest is waiting for work
    ph = {k: sum(b[k] - a[k] for a, b in zip(p0, p1)) for k in p0[0]} if n_workers else {}
    if ph.get("passes"):
        wall_us = (t1 - t0) * 1e6 * n_workers
        HOST_THREADS.update(worker_phases=dict(
            copy_in=round(ph["copy_in_us"] / wall_us, 3), invoke=round(ph["invoke_us"] / wall_us, 3),
            copy_out=round(ph["copy_out_us"] / wall_us, 3), passes=ph["passes"],
            us_per_pass=dict(copy_in=round(ph["copy_in_us"] / ph["passes"], 1),
                             invoke=round(ph["invoke_us"] / ph["passes"], 1),
                             copy_out=round(ph["copy_out_us"] / ph["passes"], 1))))
    # NUMA nodes of the page-locked request rings (MB per node)
    try:
        from band_amd import backend as _backend
        HOST_THREADS.update(ring_page_nodes_mb={str(k): round(v / 2 ** 20, 1)
                                                for k, v in _backend.RingPageNodes().items()})
    except Exception as ex:  # diagnostics only
        HOST_THREADS.update(ring_page_nodes_mb=repr(ex))
    # the request driver: requests inside the engine vs finished and waiting
    # for a reader (means over the loop), and its threads' busy shares
    if drv["wall_us"] > 0:
        w = drv["wall_us"]
        HOST_THREADS.update(request_driver=dict(
            mean_in_engine=round(drv["mean_in_engine"], 1), mean_awaiting_read=round(drv["mean_awaiting_read"], 1),
            submit_wait=round(drv["submit_wait_us"] / (w * drv["submitters"]), 3),
            submit_call=round(drv["submit_call_us"] / (w * drv["submitters"]), 3),
            submit_call_us_per_job=round(drv["submit_call_us"] / max(1, n_timed), 2),
            read_busy=round(drv["read_busy_us"] / (w * drv["readers"]), 3),
            read_us_per_job=round(drv["read_busy_us"] / max(1, n_timed), 2),
            readers=drv["readers"], submitters=drv["submitters"]))
        # inside RequestAsync: waiting for ring slots / copying the input into
        # the slot / handing the job to the planner, us per job
        nj = max(1, r1["jobs"] - r0["jobs"])
        HOST_THREADS["request_driver"].update(request_async_us_per_job=dict(
            ring_wait=round((r1["alloc_us"] - r0["alloc_us"]) / nj, 2),
            input_copy=round((r1["copy_us"] - r0["copy_us"]) / nj, 2),
            enqueue=round((r1["enqueue_us"] - r0["enqueue_us"]) / nj, 2)))
    return D.max(t1 - t0), lat_us, worker_ids


def single_engine_line(args, D, paths, sched, W, n_gpus, n_warm, n_timed, names=()):
    """ONE Band engine over n_gpus GPUs in this process: W GPU workers per GPU,
    worker w on GPU w % n_gpus (so round_robin's rotation alternates GPUs),
    one planner thread (band/engine.cc:681-713, band/planner.cc:268-293)"""
    import band_amd
    from band_amd import DeviceFlag
    n_workers = W * n_gpus
    for w in range(n_workers):
        band_amd.SetWorkerDevice(w, w % n_gpus)

    class Local:  # no barrier partners: this process alone drives the GPUs
        def barrier(self):
            pass

        def max(self, v):
            return v

    # --device cpu: Band CPU workers stand in for the GPUs (CPU tests of this
    # path); the worker -> device mapping is the same
    flag = DeviceFlag.kGPU if args.device == "gpu" else DeviceFlag.kCPU
    # the request driver of N GPUs' job stream: 2 submitter lanes per GPU
    # (lanes beyond the model count share a model's shard) and 6 readers per
    # GPU, free to run on every CPU of the process (the GPU workers pin
    # themselves to their own GPU's NUMA node); the N = 1 settings otherwise
    saved = {k: os.environ.get(k) for k in ("BANDX_DRIVER_LANES", "BANDX_DRIVER_READERS")}
    if n_gpus > 1:
        os.environ.setdefault("BANDX_DRIVER_LANES", str(2 * n_gpus))
        os.environ.setdefault("BANDX_DRIVER_READERS", str(6 * n_gpus))
        if flag == DeviceFlag.kGPU and _START_AFFINITY:
            from band_amd import backend as _backend
            _backend.PinProcessToCpus(sorted(_START_AFFINITY))
    try:
        e, bm, ins = make_engine(args, D, paths, sched, [flag] * n_workers, 0, n_workers, args.job_batch)
        inflight = args.inflight * n_gpus if args.inflight else default_inflight(n_workers, args.job_batch)
        el, lat, wid = run_closed(e, bm, ins, n_warm, n_timed, inflight, Local())
        per_model = per_model_latency(lat, list(names), len(bm), LAST_MODEL_IDX)
        e.close()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        if n_gpus > 1 and flag == DeviceFlag.kGPU and _START_AFFINITY and os.environ.get("BANDX_NUMA_PIN") != "0":
            from band_amd import backend as _backend
            _backend.PinProcessToGpu(D.local_rank)
    per_gpu = np.bincount(np.asarray(wid) % n_gpus, minlength=n_gpus).tolist()
    for w in range(n_workers):  # back to the per-process mapping
        band_amd.SetWorkerDevice(w, D.local_rank)
    return {"value": n_timed / el, "unit": "inferences/s", "n_gpus": n_gpus, "jobs": n_timed,
            "driver": {"lanes": int(os.environ.get("BANDX_DRIVER_LANES", 2 * n_gpus if n_gpus > 1 else 1)),
                       "readers": int(os.environ.get("BANDX_DRIVER_READERS", 6 * n_gpus if n_gpus > 1 else 6))},
            "ms_per_step": el * 1e3 / max(1, n_timed // args.jobs_per_step),
            "workers": n_workers, "worker_to_gpu": "w %% %d" % n_gpus, "jobs_per_gpu": per_gpu,
            "p50_job_latency_ms": float(np.percentile(lat * 1e-3, 50)),
            "p99_job_latency_ms": float(np.percentile(lat * 1e-3, 99)),
            "job_latency_ms_per_model": per_model}


def latency_tail(lat_us, worker_ids, model_idx, names, ms=10.0):
    """where an open-loop stream's slow jobs (> `ms`) fall: how many, per
    model and worker, and how they cluster in arrival order (runs of slow
    jobs at most 64 arrivals apart) - one tight cluster is a stall of the
    whole engine, a spread is a scheduling effect"""
    lat = np.asarray(lat_us) * 1e-3
    slow = np.flatnonzero(lat > ms)
    if slow.size == 0:
        return {"threshold_ms": ms, "jobs": 0}
    runs = np.split(slow, np.flatnonzero(np.diff(slow) > 64) + 1)
    mid, wid = np.asarray(model_idx), np.asarray(worker_ids)
    return {"threshold_ms": ms, "jobs": int(slow.size), "max_ms": round(float(lat.max()), 2),
            "per_model": {names[int(m)] if int(m) < len(names) else str(int(m)): int(c)
                          for m, c in zip(*np.unique(mid[slow], return_counts=True))},
            "per_worker": {str(int(w)): int(c) for w, c in zip(*np.unique(wid[slow], return_counts=True))},
            "clusters": [{"first_job": int(r[0]), "last_job": int(r[-1]), "jobs": int(r.size),
                          "max_ms": round(float(lat[r].max()), 2)} for r in runs[:8]]}


def per_model_latency(lat_us, names, n_models, model_idx):
    """rank 0's p50 / p99 job latency per model of the closed loop, keyed on
    the model index the driver reports for every job
    (BandxEngineRunClosedLoopEx, band_amd/csrc/engine/c_api.cc)"""
    lat = np.asarray(lat_us) * 1e-3
    mid = np.asarray(model_idx)
    if n_models < 1 or lat.size == 0 or mid.size != lat.size:
        return None
    out = {}
    for m in range(n_models):
        v = lat[mid == m]
        if v.size:
            key = names[m] if m < len(names) else str(m)
            out[key] = {"p50": round(float(np.percentile(v, 50)), 3), "p99": round(float(np.percentile(v, 99)), 3)}
    return out


def main():
    args = parse()
    global SAMPLE_THREADS
    SAMPLE_THREADS = args.sample_threads
    # hardware queues are fixed at HIP runtime init: one per concurrently
    # running Band GPU worker stream (must be set before libband_hip loads)
    # (explicit assignment: the GPU box exports HIP's default of 4)
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(32, args.hw_queues)))
    # before libband_hip loads: the tuner reads the file at its first decision
    tuning = None if args.fresh_tuning else replay_tuning()
    hinfo = host_info()  # before any GPU runtime is touched
    D = Dist()
    import band_amd
    from band_amd import DeviceFlag
    from band_amd.engine import SchedulerType

    models = model_list(args.model, args.size)
    M = len(models)
    W = max(1, args.workers_per_gpu)
    paths = write_models(models, "band_bench")
    if args.no_graph:
        os.environ["BAND_HIP_GRAPH"] = "0"
    if args.profile_only:
        profile_only(args, D, models, paths)
        for path in paths:
            os.unlink(path)
        D.close()
        return

    # a one-GPU process: every thread (request driver, planner, HIP runtime)
    # to the GPU's NUMA node, where the workers pin themselves and the
    # page-locked request rings live; threads created later inherit the mask
    # (BANDX_NUMA_PIN=0: off).  Restored for the CPU baseline.
    if args.device == "gpu" and not args.single_engine:
        from band_amd import backend as _backend
        node, _ = _backend.GpuNumaCpus(D.local_rank)
        hinfo["numa_pin"] = {"gpu_numa_node": node, "threads_pinned": _backend.PinProcessToGpu(D.local_rank),
                             "affinity_after": len(os.sched_getaffinity(0))}

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
    if args.share_profiles < 0:
        args.share_profiles = int(args.scheduler in ("shortest_expected_latency", "heterogeneous_earliest_finish_time"))
    batching = args.job_batch > 1
    jps = max(M, args.jobs_per_step // M * M)
    args.jobs_per_step = jps
    n_warm, n_timed = max(1, args.warmup) * jps, max(1, args.steps) * jps
    inflight = args.inflight or default_inflight(W, args.job_batch)

    poisson = None
    single = None
    host_threads = None
    head_model_idx = []
    if args.single_engine:
        # headline: one process, one engine over all --gpus GPUs
        assert D.world == 1, "--single-engine runs in one process (no torchrun)"
        single = single_engine_line(args, D, paths, sched, args.single_engine_wpg or W, max(1, args.gpus), n_warm,
                                    n_timed, names=[m[0] for m in models])
        elapsed, lat_us, worker_ids = n_timed / single["value"], None, []
        jobs_per_worker = single["jobs_per_gpu"]
        subgraph_jobs = None
        n_ranks = 1
    else:
        engine, band_models, inputs = make_engine(args, D, paths, sched, workers, n_cpu, W, args.job_batch,
                                                  seed_offset=D.rank)
        if args.model == "mix_c5":
            # C5: open-loop Poisson arrivals at 0.8 x this engine's closed-loop
            # capacity (or --rate), uniform over the 8 models; latency from
            # each request's scheduled arrival
            engine.RunClosedLoop(band_models, n_warm, inflight, inputs)
            rate = args.rate
            if rate <= 0:
                _, _, cap_wall = engine.RunClosedLoop(band_models, n_timed // 4, inflight, inputs)
                rate = 0.8 * (n_timed // 4) / cap_wall
            poisson = dict(rate_per_s_per_gpu=rate, seed=5489 + D.rank)
            D.barrier()
            cg0 = cgroup_cpu_stat()
            t0 = time.perf_counter()
            lat_us, worker_ids, poisson_mid, _ = engine.RunPoisson(band_models, n_timed, rate, seed=poisson["seed"],
                                                                   max_inflight=1 << 20, inputs=inputs)
            head_model_idx = [int(v) for v in poisson_mid]
            poisson["tail"] = latency_tail(lat_us, worker_ids, poisson_mid, [m[0] for m in models])
            t1 = time.perf_counter()
            cg1 = cgroup_cpu_stat()
            if cg0 and cg1:  # CFS throttling inside the stream (a p99 tail's suspect)
                host_threads = dict(cgroup=cgroup_delta(cg0, cg1, t1 - t0))
            D.barrier()
            elapsed = D.max(t1 - t0)
        else:
            elapsed, lat_us, worker_ids = run_closed(engine, band_models, inputs, n_warm, n_timed, inflight, D)
            head_model_idx = list(LAST_MODEL_IDX)  # the side lines below run their own loops
            host_threads = dict(HOST_THREADS)
            if HOST_THREAD_STATES:
                host_threads["thread_states"] = dict(HOST_THREAD_STATES)
        jobs_per_worker = np.bincount(worker_ids, minlength=n_cpu + W).tolist()
        # every subgraph execution per worker (warm-up included): a split
        # model's GPU share is invisible in the last-subgraph counts above
        subgraph_jobs = [engine.GetWorkerJobCount(w) for w in range(n_cpu + W)]
        engine.close()
        n_ranks = D.world
    all_lat = [x for part in D.gather((lat_us * 1e-6).tolist() if lat_us is not None else []) for x in part]

    # Band's own semantics beside it: one job per ExecuteSubgraph (no job
    # batching), the same mix and scheduler over 8 GPU workers per GPU
    batch1 = None
    if batching and not poisson and not args.no_batch1 and not args.single_engine:
        def band1_line(W1, n1):
            e1, bm1, in1 = make_engine(args, D, paths, sched, [DeviceFlag.kGPU] * W1, 0, W1, 1, seed_offset=D.rank)
            el1, lat1, _ = run_closed(e1, bm1, in1, max(n_warm // 4, 2 * W1 * M), n1, 2 * W1, D)
            e1.close()
            l1 = np.array([x for part in D.gather((lat1 * 1e-3).tolist()) for x in part])
            return {"value": n1 * D.world / el1, "unit": "inferences/s", "workers_per_gpu": W1, "jobs": n1,
                    "p50_job_latency_ms": float(np.percentile(l1, 50)),
                    "p99_job_latency_ms": float(np.percentile(l1, 99)),
                    "engine_calls": "band/interface only (max_job_batch 1): TryCopyInputTensors -> "
                                    "ExecuteSubgraph -> TryCopyOutputTensors per job",
                    "backend_coalescing": dict(COALESCE),
                    "process_cpu_cores": HOST_THREADS.get("process_cpu_cores"),
                    "busiest_threads": HOST_THREADS.get("busiest", [])[:6]}
        n1 = max(n_timed // 4, 16 * M)
        batch1 = band1_line(args.band1_workers, n1)
        # the same contract at a worker count an 8-GPU engine can carry
        # (12 per GPU = 96 worker threads on a node)
        if args.band1_workers > 12:
            batch1["at_12_workers_per_gpu"] = band1_line(12, max(n1 // 2, 16 * M))

    # the latency / throughput trade beside the headline: the same workload
    # and engine shape with smaller passes and fewer requests in flight
    # (p99 near 3 ms at about 105k inf/s per GPU)
    latency_point = None
    if (batching and not poisson and not args.single_engine and D.world == 1 and on_gpu and args.latency_point
            and not args.no_batch1):
        jb2, pt2, inf2 = (int(v) for v in args.latency_point.split(","))
        pt_head = args.pass_target_us
        args.pass_target_us = pt2
        try:
            e2, bm2, in2 = make_engine(args, D, paths, sched, workers, n_cpu, W, jb2, seed_offset=D.rank)
        finally:
            args.pass_target_us = pt_head
        el2, lat2, _ = run_closed(e2, bm2, in2, n_warm, n_timed, inf2, D)
        e2.close()
        l2 = np.asarray(lat2) * 1e-3
        latency_point = {"value": n_timed / el2, "unit": "inferences/s", "job_batch": jb2, "pass_target_us": pt2,
                         "inflight": inf2, "jobs": n_timed,
                         "p50_job_latency_ms": float(np.percentile(l2, 50)),
                         "p99_job_latency_ms": float(np.percentile(l2, 99)),
                         "job_latency_ms_per_model": per_model_latency(lat2, [m[0] for m in models], M,
                                                                       LAST_MODEL_IDX)}

    # N > 1: the same C3 workload through ONE engine spanning every GPU, with
    # W workers per GPU and with one worker per GPU (north_star's "One Worker
    # per GPU via worker_device_queue")
    single_1wpg = None
    if D.world == 1 and W != 1 and not args.no_single_engine and not poisson and on_gpu and batching:
        # N = 1: the headline engine IS the single engine; north_star's one
        # GPU worker per GPU (worker_device_queue) is measured beside it
        single_1wpg = single_engine_line(args, D, paths, sched, 1, 1, n_warm, n_timed, names=[m[0] for m in models])
    if D.world > 1 and not args.no_single_engine and not poisson:
        D.barrier()  # every rank has closed its engines
        if D.rank == 0:
            try:
                single = single_engine_line(args, D, paths, sched, W, D.world, n_warm, n_timed * D.world,
                                            names=[m[0] for m in models])
            except Exception as ex:  # the per-process line stays the headline
                single = {"error": repr(ex)}
                print("bench: single-engine line failed: %r" % (ex,), file=sys.stderr, flush=True)
            if W != 1 and "error" not in single:
                single_1wpg = single_engine_line(args, D, paths, sched, 1, D.world, n_warm, n_timed * D.world,
                                                  names=[m[0] for m in models])
        D.barrier()

    roof, dev = None, None
    if on_gpu and D.rank == 0 and not args.no_roofline:
        roof, dev, _ = profile_roofline(args, D, models, paths)
        # the same kernel-time figure at the pass size the timed loop really
        # ran (mean jobs per worker pass), not only at full B-job passes
        wp = (host_threads or {}).get("worker_phases", {})
        if wp.get("passes") and profiled_batch(args) > 1:
            b_mean = max(1, int(round(n_timed / wp["passes"])))
            if b_mean != profiled_batch(args):
                execs_m, _ = profile_executors(args, D, models, paths, batch=b_mean)
                us = 0.0
                for ex, key in execs_m:
                    us += sum(r["ms"] * 1e3 for r in ex.ProfileSubgraph(key, iters=args.profile_iters))
                dev["gpu_us_per_inference_at_mean_pass"] = dict(pass_batch=b_mean, us=us / len(models) / b_mean)
            else:
                dev["gpu_us_per_inference_at_mean_pass"] = dict(pass_batch=b_mean, us=dev["gpu_us_per_inference"])

    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, models, paths, args.cpu_baseline_seconds)

    if D.rank == 0:
        total_jobs = n_timed * n_ranks
        value = total_jobs / elapsed if not args.single_engine else single["value"]
        lat_ms = np.array(all_lat) * 1e3 if all_lat else None
        # N > 1: the headline is C3's own shape - ONE Band engine (one planner
        # thread, round_robin) whose GPU workers span the N GPUs; the
        # per-process line (N engines, one per GPU) is reported beside it
        per_process = None
        if D.world > 1 and single and "error" not in single and not args.per_process_headline:
            per_process = {"value": value, "unit": "inferences/s", "engines": D.world, "jobs": total_jobs,
                           "ms_per_step": elapsed * 1e3 / args.steps,
                           "p50_job_latency_ms": float(np.percentile(lat_ms, 50)) if lat_ms is not None else None,
                           "p99_job_latency_ms": float(np.percentile(lat_ms, 99)) if lat_ms is not None else None}
            value = single["value"]
            elapsed = single["jobs"] / single["value"]
            total_jobs = single["jobs"]
            lat_ms = None
        one_engine = args.single_engine or per_process is not None
        line = {
            "metric": "multi-DNN inferences/sec + p99 job latency, 4-model int8 mix @1/2/4/8 GPU",
            "value": value,
            "unit": "inferences/s",
            "n_gpus": n_ranks if not args.single_engine else max(1, args.gpus),
            "steps": args.steps,
            "warmup": args.warmup,
            "jobs_per_step": jps,
            "jobs_timed": total_jobs,
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
                       "harness": ("ONE native Band engine over %d GPUs (single planner)" % max(1, args.gpus, n_ranks)
                                   if one_engine else
                                   "native Band engine per GPU (planner + workers + %s)" % args.scheduler) +
                                  ", %d requests in flight per engine" % inflight,
                       "step": "%d jobs (%d of each model), round-robin over the models" % (jps, jps // M),
                       "jobs_per_worker_rank0": jobs_per_worker,
                       "subgraph_jobs_per_worker_rank0": subgraph_jobs,
                       "max_job_batch": args.job_batch, "pass_target_us": args.pass_target_us,
                       "share_profiles": bool(args.share_profiles),
                       "model": args.model, "global_batch": n_ranks * W * max(1, args.job_batch), "seq_len": None,
                       "parallelism": ("one engine, workers over %d GPUs" % max(1, args.gpus, n_ranks)) if one_engine
                       else "job-sharded x%d (no collective)" % n_ranks,
                       "hipgraph": not args.no_graph,
                       "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "fusion_tuning": ("decisions replayed from %s" % tuning) if tuning else
                                        "measured in this process"},
            "latency_tail": poisson.get("tail") if poisson else None,
            "p50_job_latency_ms": float(np.percentile(lat_ms, 50)) if lat_ms is not None else
            single["p50_job_latency_ms"],
            "p99_job_latency_ms": float(np.percentile(lat_ms, 99)) if lat_ms is not None else
            single["p99_job_latency_ms"],
            "job_latency_ms_per_model": single.get("job_latency_ms_per_model") if single and "value" in single else
            (per_model_latency(lat_us, [m[0] for m in models], M, head_model_idx)
             if lat_us is not None else None),
            "gpu_kernel_us_per_inference": dev["gpu_us_per_inference"] if dev else None,
            "gpu_kernel_us_per_inference_at_mean_pass": dev.get("gpu_us_per_inference_at_mean_pass") if dev else None,
            "device_us_per_inference": float(np.mean(list(dev["device_us"].values()))) if dev else None,
            "device_us_per_model": dev["device_us"] if dev else None,
            "band_one_job_per_pass": batch1,
            "latency_point": latency_point,
            "single_engine": single,
            "per_process": per_process,
            "single_engine_one_worker_per_gpu": single_1wpg,
            "roofline": roof,
            "cpu_baseline": cpu,
            "host": dict(hinfo, node=platform.node()),
            "host_threads_timed": host_threads,
            "backend_coalescing": dict(COALESCE) if not batching else None,
        }
        print(json.dumps(line), flush=True)
    for path in paths:
        os.unlink(path)
    D.close()


def heartbeat(period_s=60.0):
    """one stderr line a minute while the (GIL-free) native engine runs, so
    long configurations (C4 / C5 at many steps) never look hung"""
    t0 = time.time()

    def run():
        while True:
            time.sleep(period_s)
            print("bench: running, %.0f s" % (time.time() - t0), file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


if __name__ == "__main__":
    heartbeat()
    main()
