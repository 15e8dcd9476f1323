#!/usr/bin/env python3
"""Dispatch ceiling of the Band harness's single planner thread.

The reference routes every job of an engine through ONE planner thread
(band/planner.cc:268-293 Plan -> scheduler -> EnqueueToWorker,
band/engine.cc:681-713 for the worker set), so C3's "round_robin across 8
MI355X Workers" can only scale as far as that thread dispatches.  This tool
measures how many jobs/s the repo's engine/planner.cc carries when the work
itself costs ~nothing: N kCPU workers (1 thread each) run the reference's
add.tflite fixture (two float ADDs on 8x8x3: a few hundred ns), round_robin,
a native closed loop (BandxEngineRunClosedLoop) keeping `--inflight` requests
outstanding over `--models` registered copies of the model (the request ring
holds 128 per model).  What it reports is therefore the whole per-job
harness path: RequestAsync (user tensor -> ring) -> planner -> scheduler ->
worker queue -> Worker::Work (input copy, ExecuteSubgraph, output copy) ->
EnqueueFinishedJob -> Wait.

Usage: python tools/planner_ceiling.py [--workers 8,64] [--jobs 200000]
Prints one JSON line per worker count.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def thread_cpu():
    """CPU seconds (user + system) of every thread of this process, keyed by
    (tid, name): the engine names its threads band-planner, band-w<id>,
    bandx-waiter; the closed-loop driver runs on the calling (python) thread."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open("/proc/self/task/%s/stat" % tid) as f:
                raw = f.read()
            name = raw[raw.index("(") + 1:raw.rindex(")")]
            st = raw.rsplit(")", 1)[1].split()
            out[(tid, name)] = (int(st[11]) + int(st[12])) / tick
        except (OSError, ValueError):
            pass
    return out


def measure(n_workers, n_jobs, inflight, n_models, job_batch=None, gpu=False):
    from band_amd import engine as E

    # gpu: GPU workers (DeviceFlag kGPU = 1) whose passes can carry up to
    # job_batch jobs (job batching): the per-job dispatch cost with batched
    # assignments; the add.tflite pass is a few us of device work
    flag = 1 if gpu else 0
    cfg = E.make_config([E.SchedulerType.kRoundRobin], [flag] * n_workers, num_threads=[1] * n_workers,
                        max_job_batch=job_batch)
    eng = E.Engine(cfg)
    models = []
    for _ in range(n_models):
        m = E.Model()
        m.FromPath(os.path.join(ROOT, "tests", "golden", "add.tflite"))
        eng.RegisterModel(m)
        models.append(m)
    # warm-up, then the timed closed loop
    eng.RunClosedLoop(models, min(n_jobs, 4 * inflight), inflight)
    t0 = thread_cpu()
    sampler = None
    if os.environ.get("PLANNER_CEILING_SAMPLE"):
        from bench import ThreadSampler  # /proc state of every thread through the loop
        sampler = ThreadSampler()
    rq0 = eng.GetRequestPhaseTimes()
    lat, wid, wall = eng.RunClosedLoop(models, n_jobs, inflight)
    rq1 = eng.GetRequestPhaseTimes()
    t1 = thread_cpu()
    states = sampler.stop() if sampler else None
    drv = eng.GetDriverStats()
    phases = [eng.GetWorkerPhaseTimes(w) for w in range(n_workers)]
    # per-thread CPU share over the timed loop: the busiest threads name the
    # bottleneck (the planner thread is one of them; workers are named by the
    # engine only through their count, so the top shares are reported)
    busy = sorted((((t1[k] - t0.get(k, 0.0)) / wall, k[1]) for k in t1), reverse=True)
    used = np.bincount(wid, minlength=n_workers)
    out = {
        "worker_device": "gpu" if gpu else "cpu",
        "job_batch": job_batch or 1,
        "workers": n_workers,
        "models": n_models,
        "inflight": inflight,
        "jobs": n_jobs,
        "jobs_per_s": round(n_jobs / wall, 1),
        "us_per_job": round(wall * 1e6 / n_jobs, 3),
        "p50_us": round(float(np.percentile(lat, 50)), 1),
        "p99_us": round(float(np.percentile(lat, 99)), 1),
        "workers_used": int((used > 0).sum()),
        "max_worker_share": round(float(used.max()) / n_jobs, 4),
        "busiest_threads": [[n, round(b, 3)] for b, n in busy[:4]],
        "process_cpu_cores": round(sum(b for b, _ in busy), 2),
        "host_cpus": os.cpu_count(),
    }
    out["driver"] = dict(mean_in_engine=round(drv["mean_in_engine"], 1),
                         mean_awaiting_read=round(drv["mean_awaiting_read"], 1),
                         submit_wait=round(drv["submit_wait_us"] / drv["wall_us"], 3),
                         submit_call=round(drv["submit_call_us"] / drv["wall_us"], 3))
    # worker passes over the whole run (warm-up included): jobs per pass and
    # the mean pass time
    passes = sum(p["passes"] for p in phases)
    out["jobs_per_pass"] = round(sum(eng.GetWorkerJobCount(w) for w in range(n_workers)) / max(1, passes), 2)
    out["pass_us"] = round(sum(p["invoke_us"] for p in phases) / max(1, passes), 1)
    # RequestAsync's own cost per request (ring slot, input copy, planner enqueue)
    nrq = max(1, rq1["jobs"] - rq0["jobs"])
    out["request_async_us_per_job"] = {k: round((rq1[k] - rq0[k]) / nrq, 3)
                                       for k in ("alloc_us", "copy_us", "enqueue_us")}
    out["driver_env"] = {k: os.environ[k] for k in ("BANDX_DRIVER_BURST", "BANDX_DRIVER_LANES", "BANDX_DRIVER_READERS")
                         if k in os.environ}
    if states:
        out["thread_states"] = states
    eng.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", default="8,64")
    ap.add_argument("--jobs", type=int, default=200000)
    ap.add_argument("--inflight", type=int, default=0, help="default: min(4 x workers, 128 x models)")
    ap.add_argument("--models", type=int, default=8, help="registered copies of add.tflite (128 ring slots each)")
    ap.add_argument("--gpu", action="store_true", help="GPU workers (job batching possible)")
    ap.add_argument("--job-batch", type=int, default=0, help="max jobs per worker pass (GPU workers)")
    a = ap.parse_args()
    if a.job_batch and "BANDX_DRIVER_BURST" not in os.environ:
        # the closed loop submits each model's requests in runs of one batch
        # (one vector RequestAsync per run): otherwise the single submitter
        # thread, not the engine, sets the rate
        os.environ["BANDX_DRIVER_BURST"] = str(a.job_batch)
    for w in [int(x) for x in a.workers.split(",")]:
        jb = a.job_batch or 1
        inflight = a.inflight or min(4 * w * jb, 128 * a.models)
        print(json.dumps(measure(w, a.jobs, inflight, a.models, a.job_batch or None, a.gpu)), flush=True)


if __name__ == "__main__":
    main()
