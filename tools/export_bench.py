#!/usr/bin/env python3
"""K11 export path: esgpu_segment_upload of a north-star shard's columns (host u32, @timestamp i64,
response_time_ms i64) from page-locked host buffers (esgpu_host_alloc) and from pageable numpy memory.

    python tools/export_bench.py --docs 250000000 --reps 3

Prints one JSON line per source kind: host->HBM GB/s of the whole upload call (copies + zone-map pass + sync), the
SURVEY §8(d) "export ... reported separately" number.  The host columns are generated once with the job's threads.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))

import numpy as np  # noqa: E402

import elasticsearch_amd as ea  # noqa: E402
from elasticsearch_amd import _native as N  # noqa: E402
from helpers import host_threads, synthetic_columns  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=250_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    fields = ("host", "@timestamp", "response_time_ms")
    t = time.time()
    cols = synthetic_columns(fields, args.docs)
    gen_s = time.time() - t
    nbytes = sum(c["values"].nbytes for c in cols.values())
    e = ea.Engine(0)
    pinned = {}
    t = time.time()
    for f, c in cols.items():
        a = ea.pinned_empty(len(c["values"]), c["values"].dtype)
        a[:] = c["values"]
        pinned[f] = dict(c, values=a)
    pin_s = time.time() - t
    for kind, src in (("pinned", pinned), ("pageable", cols)):
        times = []
        for _ in range(args.reps):
            t = time.perf_counter()
            seg = e.upload_segment(src, args.docs)
            times.append(time.perf_counter() - t)
            seg.close()
        best = min(times)
        print(json.dumps({"kind": kind, "docs": args.docs, "bytes": nbytes, "upload_s": round(best, 4),
                          "gbs": round(nbytes / best / 1e9, 2), "all_s": [round(x, 4) for x in times],
                          "host_gen_s": round(gen_s, 2), "pin_fill_s": round(pin_s, 2), "threads": host_threads()}),
              flush=True)
    e.close()


if __name__ == "__main__":
    main()
