"""Host thread placement (backend/hip/affinity.h), on CPU.

PinProcessToCpus pins every current thread of the process and the threads
created afterwards inherit the mask; PinProcessToGpu is a no-op when the
GPU's NUMA node is unknown (no GPU here) or BANDX_NUMA_PIN=0.  Each case runs
in a child process so the test runner's own affinity is left alone."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import json, os, sys, threading
    sys.path.insert(0, %r)
    from band_amd import backend
    stop = threading.Event()
    ts = [threading.Thread(target=stop.wait) for _ in range(3)]
    for t in ts:
        t.start()
    target = sorted(os.sched_getaffinity(0))[:1]
    n = backend.PinProcessToCpus(target)
    def allowed(tid):
        for line in open("/proc/self/task/%%s/status" %% tid):
            if line.startswith("Cpus_allowed_list:"):
                return line.split(":", 1)[1].strip()
    masks = {tid: allowed(tid) for tid in os.listdir("/proc/self/task")}
    seen = []
    late = threading.Thread(target=lambda: seen.append(sorted(os.sched_getaffinity(0))))
    late.start(); late.join()
    stop.set()
    for t in ts:
        t.join()
    print(json.dumps(dict(n=n, tasks=len(masks), masks=sorted(set(masks.values())), target=target, late=seen[0])))
""") % ROOT


def _run(code, env=None):
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=e)
    assert r.returncode == 0, r.stderr
    return r.stdout.split("\n")[-2]


def test_pin_process_to_cpus_pins_every_thread_and_is_inherited():
    if len(os.sched_getaffinity(0)) < 2:
        pytest.skip("needs 2+ CPUs to see a narrowed mask")
    r = json.loads(_run(CHILD))
    cpu = r["target"][0]
    assert r["n"] >= 4 and r["n"] == r["tasks"]  # main + 3 waiting threads (+ runtime threads)
    assert r["masks"] == [str(cpu)]
    assert r["late"] == [cpu]


def test_pin_process_to_cpus_rejects_empty_and_bad_lists():
    out = _run("import sys; sys.path.insert(0, %r); from band_amd import backend; "
               "print(backend.PinProcessToCpus([]), backend.PinProcessToCpus([-5]))" % ROOT)
    assert out == "-1 -1"


@pytest.mark.parametrize("env", [{}, {"BANDX_NUMA_PIN": "0"}])
def test_pin_process_to_gpu_without_numa_information_is_a_noop(env):
    code = ("import os, sys; sys.path.insert(0, %r); from band_amd import backend; "
            "before = os.sched_getaffinity(0); n = backend.PinProcessToGpu(0); "
            "print(n, os.sched_getaffinity(0) == before)" % ROOT)
    if env == {}:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present: the node is known")
    assert _run(code, env) == "0 True"
