"""N ranks on one GPU (one thread and one esgpu context per rank, an in-process transport): the per-rank host time of
the device-resident reduce across ranks (esgpu_comm_build_reduce) per request of S shards.

    python3 tools/rank_sim.py --workload north_star --ranks 8 --docs 125000000 --reqs 20

Every rank collects its shard, then calls build_reduce (root 0); the library reports each call's host time after
the rank's collects have finished (selection launch, header / records / rows exchanges, skeleton reduce, pack, and
on the root the merge and the rebuild).  The ranks' collects share the one GPU, so the figure is the host side of the
reduce, not a scaling measurement (the driver's 8-GPU run is that).
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE)]

import elasticsearch_amd as ea  # noqa: E402
from elasticsearch_amd import AggregationBuilders as AB  # noqa: E402
from elasticsearch_amd import QueryBuilders as QB  # noqa: E402


def request(workload):
    hour = AB.dateHistogram("per_hour").field("@timestamp").interval("1h")
    if workload == "config3":
        return [AB.terms("urls").field("url").size(10)], ("url",), None
    if workload == "config4":
        return [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)], ("client_ip.hash",), None
    if workload == "config5":
        return ([AB.terms("hosts").field("host").size(10).subAggregation(hour.subAggregation(AB.avg("rt").field("response_time_ms")))],
                ("status", "bytes", "host", "@timestamp", "response_time_ms"),
                [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)])
    return ([AB.terms("hosts").field("host").size(10).subAggregation(hour.subAggregation(AB.stats("rt").field("response_time_ms")))],
            ("host", "@timestamp", "response_time_ms"), None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="north_star", choices=["north_star", "config3", "config4", "config5"])
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--docs", type=int, default=125_000_000)
    ap.add_argument("--reqs", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-align", dest="align", action="store_false",
                    help="do not wait for every rank's collect before the reduce")
    ap.add_argument("--rccl", action="store_true",
                    help="one rank over an RCCL communicator (the collectives on the device, no in-process barriers or "
                         "stream waits): the library's own host time per request on the path a GPU per rank takes")
    a = ap.parse_args()
    if a.rccl:
        a.ranks = 1
    aggs, fields, filters = request(a.workload)
    W = a.ranks
    host_ms = [[] for _ in range(W)]
    paths = set()
    wall = {}
    errs = []
    ready = threading.Barrier(W)

    def rank(r):
        try:
            eng = ea.Engine(0)
            comm = (ea.Communicator(eng, 1, 0, ea.Communicator.unique_id()) if a.rccl
                    else ea.Communicator.local("rank_sim", W, r))
            seg = eng.synthetic_segment(a.docs, fields=fields, shard=r)
            plan = eng.plan(aggs, filters=filters, number_of_shards=W)
            ready.wait()
            for i in range(a.warmup + a.reqs):
                if i == a.warmup and r == 0:
                    wall["t0"] = time.perf_counter()
                plan.reset()
                plan.collect(seg)
                if a.align:
                    # every rank's collect finished first: on one shared GPU a rank's collect otherwise ends up to
                    # (ranks - 1) collects later than another's, and the exchange's first barrier would count that wait
                    plan.last_collect_stats()
                    ready.wait()
                res = comm.build_reduce([plan], root=0)
                path, ms = comm.last_build_reduce()
                paths.add(path)
                if i >= a.warmup:
                    host_ms[r].append(ms)
                if r == 0 and i == a.warmup + a.reqs - 1:
                    wall["t1"] = time.perf_counter()
                    d = res.to_dict()
                    top = next(iter(d.values()))
                    wall["buckets"] = len(top["buckets"]) if "buckets" in top else top.get("value")
            comm.close()
            plan.close()
            seg.close()
            eng.close()
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=rank, args=(r,), daemon=True) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    if errs:
        print(json.dumps({"errors": errs}))
        sys.exit(1)
    per_rank = [statistics.median(h) for h in host_ms]
    print(json.dumps({
        "workload": a.workload, "ranks": W, "transport": "rccl" if a.rccl else "in-process", "aligned": a.align, "docs_per_shard": a.docs, "requests": a.reqs, "paths": sorted(paths),
        "host_ms_per_request_median_by_rank": [round(x, 4) for x in per_rank],
        "host_ms_per_request_root": round(per_rank[0], 4),
        "host_ms_per_request_max_rank": round(max(per_rank), 4),
        "wall_ms_per_request": round((wall["t1"] - wall["t0"]) * 1e3 / a.reqs, 3),
        "terms_buckets_or_value": wall.get("buckets"),
    }))


if __name__ == "__main__":
    main()
