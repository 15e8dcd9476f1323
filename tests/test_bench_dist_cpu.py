"""bench.py's multi-rank path on the CPU (gloo, world_size 2), and the C1 line.

The N>1 bench is one process per GPU with no data-path collective: each
rank serves its own job stream, a gloo group provides only the barrier,
the max-over-ranks time and the latency gather (bench.py `Dist`); then
rank 0 runs the headline, ONE engine whose workers span every GPU (C3's
one-planner shape).  With
`--device cpu` the same code runs its engine on Band CPU workers, so the
whole launch / barrier / reduction / JSON contract is exercised here
without a GPU.
"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _env():
    env = dict(os.environ)
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_bench_two_ranks_gloo():
    steps = 12
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--device", "cpu", "--model", "mix_c3", "--size", "64", "--workers-per-gpu", "1",
           "--cpu-threads", "2", "--steps", str(steps), "--warmup", "4", "--jobs-per-step", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2 and line["steps"] == steps and line["scaling"] == "weak"
    # headline: ONE engine (one planner) whose workers span both devices -
    # C3's shape; value = its jobs / its time, ms_per_step that time / steps
    elapsed_s = line["ms_per_step"] * steps / 1e3
    # (a step = --jobs-per-step jobs: 4, one of each mix model, per device)
    assert line["jobs_per_step"] == 4 and line["jobs_timed"] == 2 * 4 * steps
    assert abs(line["value"] - 2 * 4 * steps / elapsed_s) < 1e-6 * line["value"]
    assert line["single_engine"]["value"] == line["value"] and line["single_engine"]["n_gpus"] == 2
    assert sum(line["single_engine"]["jobs_per_gpu"]) == 2 * 4 * steps
    assert line["p99_job_latency_ms"] >= line["p50_job_latency_ms"] > 0
    assert "one engine" in line["config"]["parallelism"]
    # beside it, the per-process line: each rank's own engine, all ranks'
    # jobs / max-over-ranks time (gloo barrier + reduction)
    pp = line["per_process"]
    assert pp["engines"] == 2 and pp["jobs"] == 2 * 4 * steps and pp["value"] > 0
    assert abs(pp["value"] - pp["jobs"] / (pp["ms_per_step"] * steps / 1e3)) < 1e-6 * pp["value"]
    assert pp["p99_job_latency_ms"] >= pp["p50_job_latency_ms"] > 0
    assert sum(line["config"]["jobs_per_worker_rank0"]) == 4 * steps
    assert line["cpu_baseline"] is None  # rank 0 at N=1 only
    assert line["roofline"] is None  # no GPU kernels on CPU workers


def test_bench_c1_cpu_worker_line():
    """C1: MobileNetV1 int8 on one Band CPU worker, fixed_worker"""
    cmd = [sys.executable, "bench.py", "--device", "cpu", "--model", "mobilenet_v1_int8", "--size", "64",
           "--workers-per-gpu", "1", "--scheduler", "fixed_worker", "--cpu-threads", "2", "--steps", "8",
           "--warmup", "2", "--cpu-baseline-seconds", "0.5", "--jobs-per-step", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 1 and line["config"]["workload"].startswith("C1: ")
    assert line["config"]["jobs_per_worker_rank0"] == [8]
    cb = line["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 0
    # both CPU modes through the Band harness, host facts recorded
    assert [m["workers"] for m in cb["modes"]] == [1, 1] and cb["host"]["nproc"] >= 1
    assert cb["oracle_scalar_port_1core"]["value"] > 0


def test_bench_single_engine_cpu_stand_ins():
    """--single-engine: ONE Band engine (one planner thread) whose workers are
    spread over N devices, worker w on device w % N (band/engine.cc:681-713);
    CPU workers stand in for the GPUs"""
    cmd = [sys.executable, "bench.py", "--single-engine", "--gpus", "2", "--device", "cpu", "--model", "mix_c3",
           "--size", "64", "--workers-per-gpu", "2", "--cpu-threads", "1", "--steps", "6", "--warmup", "2",
           "--jobs-per-step", "8", "--job-batch", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    se = line["single_engine"]
    assert line["n_gpus"] == 2 and se["n_gpus"] == 2 and se["workers"] == 4 and se["worker_to_gpu"] == "w % 2"
    assert se["jobs"] == 6 * 8 and sum(se["jobs_per_gpu"]) == 6 * 8 and min(se["jobs_per_gpu"]) > 0
    assert line["value"] == se["value"] and "single planner" in line["config"]["harness"]


def test_bench_single_engine_two_submitters_per_model():
    """the single engine's request driver with more submitter lanes than
    models (8 lanes over the 4-model mix: two per model shard, sharing its
    ring-slot accounting): every job completes, on both devices"""
    env = _env()
    env["BANDX_DRIVER_LANES"] = "8"
    env["BANDX_DRIVER_READERS"] = "5"
    cmd = [sys.executable, "bench.py", "--single-engine", "--gpus", "2", "--device", "cpu", "--model", "mix_c3",
           "--size", "64", "--workers-per-gpu", "2", "--cpu-threads", "1", "--steps", "6", "--warmup", "2",
           "--jobs-per-step", "16", "--job-batch", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    se = _json_line(r.stdout)["single_engine"]
    assert se["driver"] == {"lanes": 8, "readers": 5}
    assert se["jobs"] == 6 * 16 and sum(se["jobs_per_gpu"]) == 6 * 16 and min(se["jobs_per_gpu"]) > 0


def test_worker_device_mapping():
    """DeviceRegistry (backend/hip/device.cc): an explicit worker -> ordinal
    mapping is returned as set and can be changed (bench.py remaps workers for
    its single-engine line); without a device an unmapped worker reads 0"""
    import band_amd
    band_amd.SetWorkerDevice(7001, 3)
    band_amd.SetWorkerDevice(7002, 5)
    assert band_amd.WorkerDevice(7001) == 3 and band_amd.WorkerDevice(7002) == 5
    band_amd.SetWorkerDevice(7001, 1)
    assert band_amd.WorkerDevice(7001) == 1
    assert band_amd.WorkerDevice(7999) == 0
