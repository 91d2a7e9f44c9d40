"""Isolated vs back-to-back collect launches of one request shape on one synthetic shard (the 125M-doc per-GPU shape).

    python3 tools/back2back.py --docs 125000000 --launches 8 --reps 5 [--only north_star]

isolated: reset, collect, wait (kbench's kernel_ms: the GPU idle before each launch);
back_to_back: reset, then `launches` collects of the same segment queued on the plan's stream with no wait in
between (counts accumulate -- the result is not read), the last launch's HIP-event time and the wall time per launch.
"""
import argparse
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
os.environ.setdefault("ESGPU_MALLOC_TUNE", "1")

import elasticsearch_amd as ea  # noqa: E402
from kbench import variants  # noqa: E402

FIELDS = {"north_star": ("host", "@timestamp", "response_time_ms"), "ns_avg": ("host", "@timestamp", "response_time_ms"),
          "config5": ("status", "bytes", "host", "@timestamp", "response_time_ms"),
          "config2_dh_ext": ("@timestamp", "response_time_ms"), "config3_url": ("url",),
          "config4_card": ("client_ip.hash",)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=125_000_000)
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="north_star")
    a = ap.parse_args()
    e = ea.Engine(0)
    V = variants()
    for name in a.only.split(","):
        aggs, filters = V[name]
        seg = e.synthetic_segment(a.docs, fields=FIELDS[name])
        plan = e.plan(aggs, filters=filters)
        iso = []
        for r in range(a.reps + 1):
            plan.reset()
            plan.collect(seg)
            k, _, _ = plan.last_collect_stats()
            plan.build()
            if r:
                iso.append(k)
        b2b, wall = [], []
        for r in range(a.reps + 1):
            plan.reset()
            plan.collect(seg)
            plan.last_collect_stats()
            t0 = time.perf_counter()
            for _ in range(a.launches):
                plan.collect(seg)
            k, _, _ = plan.last_collect_stats()  # (waits for the stream)
            t1 = time.perf_counter()
            plan.build()
            if r:
                b2b.append(k)
                wall.append((t1 - t0) * 1e3 / a.launches)
        print(json.dumps({"name": name, "docs": a.docs, "isolated_kernel_ms": round(statistics.median(iso), 4),
                          "back_to_back_last_kernel_ms": round(statistics.median(b2b), 4),
                          "back_to_back_wall_ms_per_launch": round(statistics.median(wall), 4)}), flush=True)
        plan.close()
        seg.close()
    e.close()


if __name__ == "__main__":
    main()
