#!/usr/bin/env python3
"""Kernel-level sweep: collect-kernel time and algorithmic GB/s for each §8 request shape on one synthetic shard.

    python tools/kbench.py --docs 1000000000 --reps 5 [--only name,name]

Prints one JSON line per variant: {"name", "kernel_ms", "bytes", "gbs", "frac", "path", "step_ms"}.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
os.environ.setdefault("ESGPU_MALLOC_TUNE", "1")  # as bench.py: the host process opts into the library's malloc settings

import elasticsearch_amd as ea  # noqa: E402
from elasticsearch_amd import AggregationBuilders as AB  # noqa: E402
from elasticsearch_amd import QueryBuilders as QB  # noqa: E402


def variants():
    ns = lambda m: AB.terms("hosts").field("host").size(10).subAggregation(  # noqa: E731
        AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(m))
    return {
        "terms_host": ([AB.terms("hosts").field("host")], None),
        "date_hist": ([AB.dateHistogram("h").field("@timestamp").interval("1h")], None),
        "config2_dh_ext": ([AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(
            AB.extendedStats("rt").field("response_time_ms"))], None),
        "dh_stats": ([AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(
            AB.stats("rt").field("response_time_ms"))], None),
        "terms_dh": ([AB.terms("hosts").field("host").subAggregation(AB.dateHistogram("h").field("@timestamp").interval("1h"))], None),
        "config1_terms_stats": ([AB.terms("hosts").field("host").subAggregation(AB.stats("rt").field("response_time_ms"))], None),
        "north_star": ([ns(AB.stats("rt").field("response_time_ms"))], None),
        "ns_avg": ([ns(AB.avg("rt").field("response_time_ms"))], None),
        "config5": ([ns(AB.avg("rt").field("response_time_ms"))],
                    [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)]),
        "config4_card": ([AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)], None),
        "config3_url": ([AB.terms("urls").field("url").size(10)], None),
        # config 3 under a query filter keeping 80 % of the docs (bytes uniform in [0, 1e6)): the scatter form
        "config3_url_f": ([AB.terms("urls").field("url").size(10)], [QB.rangeQuery("bytes").lt(800000)]),
        # terms under terms over 1,000 x 10M ordinals: outer counts in the collect, the inner terms replayed at build
        # (breadth-first) -- the replay's time is in parts_ms.build
        "hosts_urls": ([AB.terms("hosts").field("host").size(10).subAggregation(AB.terms("urls").field("url").size(3))], None),
        "dh_terms": ([AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(
            AB.terms("hosts").field("host").size(10))], None),
        "heatmap": ([AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(
            AB.histogram("lat").field("response_time_ms").interval(100))], None),
    }


def _dict_blob(field):
    """term bytes + offsets of the synthetic keyword fields (host-%04d / /p/%08x), built as an uploaded dictionary"""
    n = 1000 if field == "host" else 10_000_000
    width, prefix = (4, b"host-") if field == "host" else (8, b"/p/")
    ids = np.arange(n, dtype=np.uint64)
    if field == "host":
        digits = (ids[:, None] // (10 ** np.arange(width - 1, -1, -1, dtype=np.uint64))) % 10
        chars = np.frombuffer(b"0123456789", dtype=np.uint8)[digits.astype(np.int64)]
    else:
        digits = (ids[:, None] >> (np.arange(width - 1, -1, -1, dtype=np.uint64) * 4)) & 15
        chars = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)[digits.astype(np.int64)]
    L = len(prefix) + width
    out = np.empty((n, L), dtype=np.uint8)
    out[:, :len(prefix)] = np.frombuffer(prefix, dtype=np.uint8)
    out[:, len(prefix):] = chars
    return out.reshape(-1), np.arange(0, L * (n + 1), L, dtype=np.uint64)


def _with_real_dicts(e, seg, n, fields):
    """the same columns, uploaded through esgpu_segment_upload (keyword fields with their dictionaries)"""
    cols = {}
    for f in fields:
        t = ea._native.SYNTH_TYPES[f]
        dt = {ea._native.COL_ORD_U32: np.uint32, ea._native.COL_I64: np.int64, ea._native.COL_F64: np.float64,
              ea._native.COL_U64: np.uint64}[t]
        c = {"type": t, "values": seg.read_column(f, 0, n, dt)}
        if f in ("host", "url"):
            c["terms_blob"] = _dict_blob(f)
        cols[f] = c
    seg.close()
    return e.upload_segment(cols, n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--ts-jitter", type=int, default=0,
                    help="@timestamp displacement bound in ms (0 = time-sorted docs; 60000 / 3600000 = roughly sorted)")
    ap.add_argument("--shards", type=int, default=1, help="number_of_shards of the request (terms shard_size heuristic)")
    ap.add_argument("--deletes", type=float, default=0.0,
                    help="fraction of deleted docs: every request passes a live-docs accept bitset with that many random "
                         "docs cleared (Lucene liveDocs; the high-cardinality terms path then takes its scatter form)")
    ap.add_argument("--real-dict", action="store_true",
                    help="re-upload host/url as ordinary keyword columns with their term bytes (esgpu_segment_upload with a "
                         "dictionary), so the build resolves winners through a real 10M-term dictionary")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    e = ea.Engine(0)
    vs = {k: v for k, v in variants().items() if not only or k in only}
    fields = {"host", "@timestamp", "response_time_ms", "status", "bytes", "client_ip.hash"}
    if "config3_url" in vs or "config3_url_f" in vs or "hosts_urls" in vs:
        fields.add("url")
    t = time.time()
    seg = e.synthetic_segment(args.docs, fields=tuple(sorted(fields)), ts_jitter_ms=args.ts_jitter)
    if args.real_dict:
        seg = _with_real_dicts(e, seg, args.docs, sorted(fields))
    accept = None
    if args.deletes > 0:  # live docs: a random `deletes` fraction cleared, as u64 words (include/esgpu.h layout)
        rng = np.random.default_rng(7)
        words = np.full((args.docs + 63) // 64, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
        dead = rng.choice(args.docs, size=int(args.docs * args.deletes), replace=False)
        np.bitwise_and.at(words, dead // 64, ~(np.uint64(1) << (dead % 64).astype(np.uint64)))
        if args.docs % 64:
            words[-1] &= np.uint64((1 << (args.docs % 64)) - 1)
        accept = words
    print(json.dumps({"generated_s": time.time() - t, "hbm_gb": e.hbm_used() / 1e9, "ts_jitter_ms": args.ts_jitter,
                      "shards": args.shards, "deletes": args.deletes}), flush=True)
    for name, (aggs, flt) in vs.items():
        plan = e.plan(aggs, filters=flt, number_of_shards=args.shards)
        ms = []
        steps = []
        parts = {"reset": [], "collect_call": [], "kernel_wait": [], "build": [], "build_wait": [], "reduce": []}
        for r in range(args.reps + 1):
            t0 = time.perf_counter()
            plan.reset()
            t1 = time.perf_counter()
            plan.collect(seg, accept_bits=accept)
            t2 = time.perf_counter()
            k, nbytes, path = plan.last_collect_stats()
            t3 = time.perf_counter()
            res = plan.build()
            t4 = time.perf_counter()
            bwait = plan.last_build_stats()[1]
            ea.reduce([res])
            t5 = time.perf_counter()
            dt = (t5 - t0) * 1e3
            if r:  # first is warmup
                ms.append(k)
                steps.append(dt)
                for key, a, b in (("reset", t0, t1), ("collect_call", t1, t2), ("kernel_wait", t2, t3),
                                  ("build", t3, t4), ("reduce", t4, t5)):
                    parts[key].append((b - a) * 1e3)
                parts["build_wait"].append(bwait)
        kms = sorted(ms)[len(ms) // 2]
        gbs = nbytes / (kms / 1e3) / 1e9
        print(json.dumps({"name": name, "ts_jitter_ms": args.ts_jitter, "deletes": args.deletes, "kernel_ms": round(kms, 4), "bytes": nbytes, "gbs": round(gbs, 1),
                          "frac": round(gbs / 8000, 4), "path": path, "step_ms": round(sorted(steps)[len(steps) // 2], 3),
                          "docs_per_s": args.docs / (kms / 1e3),
                          "parts_ms": {k: round(sorted(v)[len(v) // 2], 3) for k, v in parts.items()}}), flush=True)
        plan.close()


if __name__ == "__main__":
    main()
