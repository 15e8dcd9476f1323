#!/usr/bin/env python3
"""One line per bench.py JSON: value, p99, jobs per pass and the request
driver's state (requests inside the engine / awaiting a reader, submitter and
reader cost per job).  usage: python3 tools/bench_show.py <name> <bench.json>"""
import json
import sys


def main():
    name, path = sys.argv[1], sys.argv[2]
    d = json.load(open(path))
    h = d.get("host_threads_timed") or {}
    ph = h.get("worker_phases") or {}
    r = h.get("request_driver") or {}
    jpp = round(d["jobs_timed"] / ph["passes"], 1) if ph.get("passes") else None
    print(name, round(d["value"]), round(d["p99_job_latency_ms"], 2), "j/p", jpp, "eng", r.get("mean_in_engine"),
          "await", r.get("mean_awaiting_read"), "sub_us", r.get("submit_call_us_per_job"), "sub_wait",
          r.get("submit_wait"), "read_us", r.get("read_us_per_job"))


if __name__ == "__main__":
    main()
