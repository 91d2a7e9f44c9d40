#!/usr/bin/env python3
"""bench.py — per-shard aggregation throughput on MI355X (BASELINE.json metric).

Workload (default, `north_star`): terms(host){date_histogram(@timestamp,1h){stats(response_time_ms)}} over a
1,000,000,000-doc synthetic log shard per GPU (BASELINE.md "north star": 1B docs / 1 shard / 1 GPU), columns
HBM-resident before timing.  One step = one request: for each of the GPU's shards reset accumulators, collect the
segment (fused gfx950 kernel), postCollection + buildAggregation (top-k on the host or GPU, winners' rows compacted on
the GPU), then the coordinator reduce (RCCL across ranks when N > 1).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line.  value = docs aggregated per second for the whole job, with `--inflight` requests in
flight (default 2: one request's builds and reduce overlap the next one's collects).  ms_per_request_latency: one request
at a time, its shards collected back to back (one plan and HIP stream per shard) and built on worker threads, as
Elasticsearch runs one SEARCH thread per shard.  ms_per_step_sequential: nothing overlapping at all (one plan, collect
-> build per shard, then the reduce); the collect kernels' HIP-event times come from that phase.
roofline = algorithmic HBM bytes of the collect kernel per launch / its HIP-event time.  cpu_baseline = the oracle
(line-by-line restatement of the reference Java collect loop, oracle/cpu_ref.cpp) on the host cores over a bounded
synthetic sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# bytes per doc of the request's columns at their upload width
UPLOAD_BYTES = {"north_star": 20, "config2": 16, "config3": 4, "config4": 8, "config5": 36}

WORKLOADS = {
    # name: (fields, builder fn, filters fn, description, number_of_docs default)
    "north_star": (("host", "@timestamp", "response_time_ms"), "terms(host){date_histogram(1h){stats(response_time_ms)}}"),
    "config2": (("@timestamp", "response_time_ms"), "date_histogram(@timestamp,1h){extended_stats(response_time_ms)}"),
    "config3": (("url",), "terms(url, size 10 => shard_size 80)"),
    "config4": (("client_ip.hash",), "cardinality(client_ip.hash, precision_threshold 40000)"),
    "config5": (("status", "bytes", "host", "@timestamp", "response_time_ms"),
                "bool.filter[term(status:200), range(bytes:[1024,65536])] -> terms(host){date_histogram(1h){avg(response_time_ms)}}"),
}


def build_request(workload, world):
    from elasticsearch_amd import AggregationBuilders as AB
    from elasticsearch_amd import QueryBuilders as QB
    if workload == "north_star":
        return [AB.terms("hosts").field("host").size(10).subAggregation(
            AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(
                AB.stats("rt").field("response_time_ms")))], None
    if workload == "config2":
        return [AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(
            AB.extendedStats("rt").field("response_time_ms"))], None
    if workload == "config3":
        return [AB.terms("urls").field("url").size(10)], None
    if workload == "config4":
        return [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)], None
    if workload == "config5":
        return ([AB.terms("hosts").field("host").size(10).subAggregation(
            AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.avg("rt").field("response_time_ms")))],
            [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)])
    raise SystemExit(f"unknown workload {workload}")


def host_cpu():
    """(model name, logical CPUs visible to this process) -- what `lscpu` reports for the box."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return model, n


def cpu_baseline(workload, world, sample_docs, threads, single_docs):
    """The oracle (cpu_ref: the reference's Java collect/build loops restated in C++) on the host cores, one shard per
    thread as Elasticsearch runs one SEARCH thread per shard.  `threads` shards of
    sample_docs / threads docs each, generated and collected concurrently; the wall time of the collect+build
    phase over all of them gives the node-level CPU rate.  A separate single-thread run over one shard of
    `single_docs` docs gives the one-core rate (the reference's per-shard latency path)."""
    import threading
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import oracle as O
    from helpers import synthetic_columns
    fields = WORKLOADS[workload][0]
    aggs, filters = build_request(workload, world)
    per = max(sample_docs // threads, 1)
    cols = [None] * threads
    secs = [0.0] * threads

    def gen(i):
        cols[i] = synthetic_columns(fields, per, shard=i, threads=1)

    def work(i):
        _, secs[i] = O.run([(cols[i], per)], aggs, filters=filters, number_of_shards=world, return_seconds=True)

    for fn in (gen, work):
        ts = [threading.Thread(target=fn, args=(i,)) for i in range(threads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        wall = time.perf_counter() - t0
    cols = None
    one = synthetic_columns(fields, single_docs, shard=0)
    _, one_secs = O.run([(one, single_docs)], aggs, filters=filters, number_of_shards=world, return_seconds=True)
    one = None
    model, visible = host_cpu()
    value = per * threads / wall
    return {"value": value, "unit": "docs/s", "cores": threads, "kind": "port",
            "single_core_value": single_docs / one_secs,
            "cpu_model": model, "host_cpus_visible": visible,
            "sample": f"oracle/cpu_ref.cpp (the reference's Java collect+build loops restated), {threads} synthetic "
                      f"shards x {per:,} docs of the same request, one host thread per shard, run concurrently on the "
                      f"{threads} cores this job is allotted ({wall:.2f} s wall), plus one shard of {single_docs:,} docs "
                      f"on one thread ({single_docs / one_secs / 1e6:.1f}M docs/s); {model}, {visible} logical CPUs "
                      f"visible"}


def self_check(workload, res, docs_total, matching=None):
    """Size-independent properties of the timed request's final result (outside the timed region): every counted doc
    is in a bucket or in sum_other_doc_count, a term's hour buckets add up to its doc count, each bucket's metric count
    equals its doc count (dense metric column), and the cardinality estimate is within 5 % of the distinct values the
    generator can produce.  Returns (ok, details)."""
    errs = []
    expect = docs_total if matching is None else matching
    if workload in ("north_star", "config5", "config3"):
        t = res["hosts"] if workload != "config3" else res["urls"]
        total = sum(b["doc_count"] for b in t["buckets"]) + t["sum_other_doc_count"]
        if total != expect:
            errs.append(f"sum(doc_count) + sum_other_doc_count = {total} != {expect}")
        for b in t["buckets"] if workload != "config3" else []:
            hours = b["per_hour"]["buckets"]
            if sum(h["doc_count"] for h in hours) != b["doc_count"]:
                errs.append(f"term {b['key']}: hour buckets do not add up")
            for h in hours:
                cnt = h["rt"]["count"] if workload == "north_star" else h["rt"]["_internal"]["count"]
                if cnt != h["doc_count"]:
                    errs.append(f"term {b['key']} hour {h['key']}: metric count {cnt} != doc_count {h['doc_count']}")
                    break
    elif workload == "config2":
        hours = res["per_hour"]["buckets"]
        if sum(h["doc_count"] for h in hours) != expect:
            errs.append("hour buckets do not add up to the docs")
        if any(h["rt"]["count"] != h["doc_count"] for h in hours):
            errs.append("metric count != doc_count")
    elif workload == "config4":
        import math
        pool = 1 << 27  # client_ip.hash draws from 2^27 distinct IPs
        distinct = pool * (1.0 - math.exp(-docs_total / pool))
        v = res["ips"]["value"]
        if abs(v - distinct) > 0.05 * distinct or res["ips"]["_internal"]["mode"] != "hll":
            errs.append(f"cardinality {v} vs ~{distinct:.0f} expected distinct")
    return not errs, errs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=1_000_000_000, help="docs per shard")
    ap.add_argument("--shards", type=int, default=0,
                    help="shards of the job, shards / GPUs per GPU, collected in turn (0 = one shard per GPU: weak "
                         "scaling; S > 0 fixes the job's size: strong scaling, e.g. --shards 8 --docs 125000000 is "
                         "BASELINE configs 3-5's 1B docs in 8 shards)")
    ap.add_argument("--workload", default="north_star", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-docs", type=int, default=640_000_000, help="CPU baseline sample size (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the CPU baseline, one shard each (0 = every CPU this job is allotted: its "
                         "affinity, capped by OMP_NUM_THREADS)")
    ap.add_argument("--cpu-single-docs", type=int, default=20_000_000, help="docs of the single-thread CPU shard")
    ap.add_argument("--inflight", type=int, default=0, choices=(0, 1, 2, 3, 4),
                    help="requests in flight (0 = 2): plan sets that alternate, one plan per shard of a request")
    ap.add_argument("--scheme", default="auto", choices=("auto", "inline", "rotate", "sets"),
                    help="pipelined phase: inline = one unit per request, the next request's collect launched before this "
                         "one is built and reduced on the main thread (no worker threads); rotate = `inflight` plans taken "
                         "in turn by the shards of consecutive requests, builds on worker threads; sets = one plan per "
                         "shard, `inflight` sets of them alternating between requests; auto = inline for one-unit "
                         "requests, else rotate")
    ap.add_argument("--no-colo", action="store_true",
                    help="build every shard result and reduce them on the host, instead of the co-located reduce "
                         "(esgpu_plans_build_reduce) for a GPU's terms shards on one GPU")
    ap.add_argument("--traffic", default=os.path.join(HERE, "profiles", "hbm_traffic.json"),
                    help="PMC-derived HBM bytes per collect launch (profiles/), if measured for this workload")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = max(world, 1)
    shards = args.shards if args.shards > 0 else world
    if shards % world:
        raise SystemExit(f"--shards {shards} must be a multiple of the {world} GPUs")
    per_gpu = shards // world

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", rank=rank, world_size=world)

    # the bench is the host process: it opts into the library's malloc settings (large result arrays stay on the heap
    # instead of an mmap / munmap per request); an embedding JVM leaves them off
    os.environ.setdefault("ESGPU_MALLOC_TUNE", "1")
    import elasticsearch_amd as ea
    engine = ea.Engine(local_rank if world > 1 else 0)
    fields, desc = WORKLOADS[args.workload]
    aggs, filters = build_request(args.workload, shards)
    # this rank's shards: global shards rank * per_gpu ... (rank-major = the reduce's shard order)
    segs = [engine.synthetic_segment(args.docs, fields=fields, shard=rank * per_gpu + i) for i in range(per_gpu)]
    probe = engine.plan(aggs, filters=filters, number_of_shards=shards)
    # fixed-shape requests (no terms): this GPU's shards are collected into one plan, one build per request; terms
    # requests build one shard result per shard (per-shard top-k) and reduce them with the other ranks'
    merged = probe.shard_mergeable() and per_gpu > 1
    probe.close()
    units_per_request = 1 if merged or per_gpu == 1 else per_gpu
    # a terms request's shards on one GPU (one process): built and reduced in one call (esgpu_plans_build_reduce, the
    # same result as reducing every shard build); with several ranks each rank's shards go to the cross-rank reduce
    # with several ranks, a shape the device merge takes goes to the device-resident reduce across ranks
    # (esgpu_comm_build_reduce: device selections and rows exchanged device to device, the merge on rank 0)
    colo = units_per_request > 1 and not merged and not args.no_colo
    if colo:
        probe_plans = [engine.plan(aggs, filters=filters, number_of_shards=shards) for _ in range(max(units_per_request, 2))]
        colo = ea.colocated(probe_plans)  # a shape the device merge takes (else the builds run on worker threads)
        for pp in probe_plans:
            pp.close()
    # several ranks: every request goes to esgpu_comm_build_reduce, which exchanges device buffers for the co-located
    # shapes (north star, config 5), plain terms (config 3) and top-level cardinality (config 4), and builds + reduces
    # every other shape across the ranks
    xr = world > 1 and not args.no_colo
    if xr:
        colo = units_per_request > 1
    if colo:
        args.scheme = "sets"  # one plan per shard: a request's plans are all alive at its reduce
    # plan sets: one plan per unit (a shard, or all of a fixed-shape request's shards); `inflight` sets alternate, so
    # one request's builds and reduce run while the next request's collects are on the GPU
    inflight = args.inflight or 2
    sets = [[engine.plan(aggs, filters=filters, number_of_shards=shards) for _ in range(units_per_request)]
            for _ in range(inflight)]
    comm = None
    if world > 1:
        uid = [ea.Communicator.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = ea.Communicator(engine, world, rank, uid[0])

    kernel_ms, kernel_bytes = [0.0], [0]
    final = None

    def launch(p, unit, record):
        p.reset()
        for seg in (segs if merged or per_gpu == 1 else [segs[unit]]):
            p.collect(seg)
            if record:  # HIP-event time of this collect (synchronises: serial phase only)
                ms, nbytes, _ = p.last_collect_stats()
                kernel_ms[0] += ms
                kernel_bytes[0] += nbytes

    host_ms = {"build": 0.0, "reduce": 0.0}
    if colo or xr:
        host_ms = {"build_reduce": 0.0}
    # A request's shard builds run on worker threads -- Elasticsearch runs one SEARCH thread per shard of a request --
    # and the coordinating reduce of a request on its own worker (a coordinating node merges one request while the
    # data nodes collect the next).  Requests are reduced in order; every one finishes inside the timed region.
    from collections import deque
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from helpers import host_threads
    builders = ThreadPoolExecutor(max(1, min(units_per_request, host_threads() - 2)))
    reducer = ThreadPoolExecutor(1)

    def build_unit(p):
        t = time.perf_counter()
        r = p.build()
        host_ms["build"] += (time.perf_counter() - t) * 1e3
        return r

    def reduce_request(futs):
        parts = [f.result() for f in futs]
        t = time.perf_counter()
        out = comm.reduce(parts) if comm else ea.reduce(parts)
        host_ms["reduce"] += (time.perf_counter() - t) * 1e3
        return out

    def colo_request(plans):
        t = time.perf_counter()
        out = comm.build_reduce(plans, root=0) if xr else ea.build_reduce(plans)
        host_ms["build_reduce"] += (time.perf_counter() - t) * 1e3
        return out

    def run(n_requests, depth):
        """n requests on `depth` plan sets: a request's collects are issued back to back (each plan has its own HIP
        stream), its builds go to the builder threads, its reduce to the reducer; a set is reused once its previous
        request is reduced.  depth 1: one request at a time (its shards still in parallel), the request latency."""
        nonlocal final
        pend = deque()
        for r in range(n_requests):
            while len(pend) >= depth:
                final = pend.popleft().result()
            futs = []
            for unit, p in enumerate(sets[r % depth]):
                launch(p, unit, False)
                if not (colo or xr):
                    futs.append(builders.submit(build_unit, p))
            pend.append(reducer.submit(colo_request, sets[r % depth]) if colo or xr else reducer.submit(reduce_request, futs))
        while pend:
            final = pend.popleft().result()

    def run_rotate(n_requests, depth):
        """`depth` plans taken in turn by the units of consecutive requests (one plan's unit is built on a worker
        thread while the next plans' collects run); a plan is reset only once its previous unit is built"""
        nonlocal final
        plans = [st[0] for st in sets[:depth]]
        owner = [None] * depth
        pend = deque()
        k = 0
        for _ in range(n_requests):
            futs = []
            for unit in range(units_per_request):
                i = k % depth
                k += 1
                if owner[i] is not None:
                    owner[i].result()
                launch(plans[i], unit, False)
                owner[i] = builders.submit(build_unit, plans[i])
                futs.append(owner[i])
            while len(pend) >= 2:
                final = pend.popleft().result()
            pend.append(reducer.submit(reduce_request, futs))
        while pend:
            final = pend.popleft().result()

    def run_inline(n_requests, depth):
        """one unit per request on `depth` plans taken in turn, no worker threads: request r + 1's collect is launched
        (on its plan's stream) before request r is built and reduced here, so the GPU runs the next collect while the
        host builds -- for small requests the thread handoffs of `run_rotate` cost more than the build"""
        nonlocal final
        plans = [st[0] for st in sets[:depth]]
        if n_requests == 0:
            return
        launch(plans[0], 0, False)
        for r in range(n_requests):
            if r + 1 < n_requests:
                launch(plans[(r + 1) % depth], 0, False)
            if xr:
                final = comm.build_reduce([plans[r % depth]], root=0)
                continue
            part = plans[r % depth].build()
            final = comm.reduce([part]) if comm else ea.reduce([part])

    def run_serial(n_requests):
        """one unit at a time on one plan: collect, build, and finally reduce, nothing overlapping -- the collect
        kernels' HIP-event times are taken here, where no two kernels run at once"""
        nonlocal final
        p = sets[0][0]
        for _ in range(n_requests):
            if colo or xr:  # the request's shards collected one after the other, then built and reduced in one call
                for unit, pu in enumerate(sets[0]):
                    launch(pu, unit, True)
                final = colo_request(sets[0])
                continue
            parts = []
            for unit in range(units_per_request):
                launch(p, unit, True)
                parts.append(build_unit(p))
            t = time.perf_counter()
            final = comm.reduce(parts) if comm else ea.reduce(parts)
            host_ms["reduce"] += (time.perf_counter() - t) * 1e3

    def timed(fn, *a):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(*a)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    precomputed = None
    if args.workload == "config3" and per_gpu > 1:
        # the per-segment statistics of the 10M-ordinal column (hot set, recoded column, cold postings: built on a
        # segment's first request and cached with it, as Elasticsearch caches global ordinals) -- their build time and
        # HBM footprint, measured on this GPU's segments 1.. (segment 0's first collect also allocates the plan's grid)
        p = sets[0][0]
        p.reset()
        p.collect(segs[0])
        p.last_collect_stats()
        first, hbm = [], []
        for seg in segs[1:]:
            p.reset()
            h0 = engine.hbm_used()
            t0 = time.perf_counter()
            p.collect(seg)
            k_ms, _, _ = p.last_collect_stats()
            first.append((time.perf_counter() - t0) * 1e3 - k_ms)
            hbm.append(engine.hbm_used() - h0)
        precomputed = {"what": "per-segment hot/cold statistics of the url ordinals (cached with the segment)",
                       "build_ms_per_shard": round(sum(first) / len(first), 3),
                       "hbm_bytes_per_shard": int(sum(hbm) / len(hbm)),
                       "column_bytes_per_shard": 4 * args.docs}
        p.build()
    else:
        # the compact columns (16-bit ordinals, 32-bit timestamp deltas: DESIGN §3) of each segment of this GPU, built on
        # its first collect and cached with it -- their build time and HBM footprint, outside the timed region
        p = sets[0][0]
        first, hbm, cold = [], [], []
        for seg in segs:
            p.reset()
            h0 = engine.hbm_used()
            t0 = time.perf_counter()
            p.collect(seg)
            k_ms, _, _ = p.last_collect_stats()
            first.append((time.perf_counter() - t0) * 1e3 - k_ms)
            hbm.append(engine.hbm_used() - h0)
            p.build()
            cold.append((time.perf_counter() - t0) * 1e3)  # a request on the cold segment: products, collect, build
        if sum(hbm) >= 2 * args.docs * len(segs):  # at least 2 B per doc: compact columns were built
            what = ("compact columns of the segment (u16 ordinals, timestamp block deltas or u32 deltas, u16 / u32 metric "
                    "deltas; cached with it; the first segment's figure includes the plan's grid)")
            if args.workload == "config4":
                what = ("HLL++ encodeHash words of the murmur3 field, 4 B per doc (the hash's index bits and its run-length "
                        "count past them, HyperLogLogPlusPlus.java:335-346: what the register updates read instead of the "
                        "8-B hashes), built on the segment's first request and cached with it; the first segment's figure "
                        "includes the plan's registers and sets")
            precomputed = {"what": what,
                           "build_ms_per_segment": round(sum(first) / len(first), 3),
                           "hbm_bytes_per_segment": int(sum(hbm) / len(hbm)),
                           # one request on a segment whose products are not built yet (they are built inside it)
                           "cold_first_request_ms": round(sum(cold) / len(cold), 3)}
    if args.scheme == "auto":
        args.scheme = "inline" if units_per_request == 1 and not colo and inflight > 1 else "rotate"
    if xr and args.scheme == "rotate":  # (rotating plans build units one by one: the cross-rank call takes a request's plans)
        args.scheme = "sets"
    pipelined = {"inline": run_inline, "rotate": run_rotate}.get(args.scheme, run)
    pipelined(args.warmup, inflight)
    elapsed = timed(pipelined, args.steps, inflight)
    elapsed_latency = timed(run, args.steps, 1) if inflight > 1 else elapsed
    for k in host_ms:  # host times per request, from the serial phase
        host_ms[k] = 0.0
    elapsed_seq = timed(run_serial, args.steps)
    host_ms = {k: round(v / args.steps, 4) for k, v in host_ms.items()}
    exchange = None
    if comm:
        ar, ag, ncoll = comm.last_exchange()
        exchange = {"allreduce_bytes": ar, "allgather_bytes": ag, "collectives": ncoll, "ms": comm.last_exchange_ms()}
        if xr:
            path, xms = comm.last_build_reduce()
            exchange.update({"device_resident": path == 1, "build_reduce_host_ms": round(xms, 4)})

    # self-check of the last timed request's final result (outside the timed region)
    matching = None
    if args.workload == "config5":  # docs the query matches: a filter aggregation over the same clauses, per shard
        fp = engine.plan([ea.AggregationBuilders.filter("m", filters)], number_of_shards=shards)
        matching = 0
        for seg in segs:
            fp.reset()
            fp.collect(seg)
            matching += fp.build().to_dict()["m"]["doc_count"]
        fp.close()
        if dist:
            t = torch.tensor([matching], dtype=torch.int64, device=f"cuda:{local_rank}")
            dist.all_reduce(t)
            matching = int(t.item())
    docs_total = args.docs * shards
    # (the device-resident reduce across ranks leaves the result on rank 0 only: the other ranks check nothing)
    checked, check_errors = (self_check(args.workload, final.to_dict(), docs_total, matching) if not xr or rank == 0
                             else (True, []))

    ms_per_step = elapsed * 1000.0 / args.steps
    value = docs_total / (elapsed / args.steps)
    avg_kernel_ms = kernel_ms[0] / args.steps
    bytes_per_step = kernel_bytes[0] // args.steps
    achieved = bytes_per_step / (avg_kernel_ms / 1000.0) / 1e9
    launches = args.steps * (per_gpu if per_gpu > 1 else 1)
    traffic = None
    if os.path.exists(args.traffic):
        try:
            with open(args.traffic) as f:
                tr = json.load(f)
            # entries keyed by (workload, docs per shard, shards): tools/pmc_traffic.py --merge; the entry must have been
            # measured on the layout this run reads (the same algorithmic bytes per launch within 0.1 %: config 3's
            # postings bytes differ a little from shard to shard), scaled to this run's bytes
            alg = kernel_bytes[0] // launches
            for e in tr.get("entries", [tr]):
                ea_bytes = e.get("algorithmic_bytes_per_launch") or 0
                if (e.get("workload") == args.workload and e.get("docs") == args.docs and e.get("shards", 1) == shards and
                        ea_bytes and abs(ea_bytes - alg) <= ea_bytes // 1000):
                    traffic = int(e.get("hbm_bytes_per_launch") * alg / ea_bytes)
        except Exception:
            traffic = None

    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_docs > 0:
            threads = args.cpu_threads if args.cpu_threads > 0 else host_threads()
            cpu = cpu_baseline(args.workload, shards, args.cpu_docs, threads, args.cpu_single_docs)
        out = {
            "metric": "docs aggregated/sec (node) + achieved HBM GB/s, terms+date_histogram, 1B docs",
            "value": value,
            "unit": "docs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "inflight_requests": inflight,
            "scheme": args.scheme,
            "ms_per_request_latency": elapsed_latency * 1000.0 / args.steps,
            "ms_per_step_sequential": elapsed_seq * 1000.0 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if args.shards > 0 else "weak",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic (deterministic splitmix64 log docs generated in HBM, seed 0x5EEDE1A5, shard = global shard id)",
            "config": {"workload": args.workload, "request": desc, "docs_per_shard": args.docs, "shards": shards,
                       "shards_per_gpu": per_gpu, "docs_total": docs_total,
                       "collect": ("merged (one plan per GPU)" if merged else "per shard") +
                                  (", reduce across ranks through esgpu_comm_build_reduce" if xr else
                                   ", co-located reduce (esgpu_plans_build_reduce)" if colo else ""),
                       "parallelism": f"{per_gpu} shard(s) per GPU x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                         # two figures: frac_physical = the bytes the GPU layout must move (compact columns,
                         # packed metric: DESIGN §3 / §5; PMC traffic within a few % of it) over the kernel time -- the
                         # kernel-quality figure, = frac; frac_s8d = SURVEY §8(d)'s upload-width bytes over the same
                         # time (an effective rate, above 1 when the layout moves fewer bytes than §8(d) counts)
                         "frac_physical": achieved / PEAK_HBM_GBS,
                         "frac_s8d": (UPLOAD_BYTES[args.workload] * args.docs * per_gpu / (avg_kernel_ms / 1000.0) / 1e9) / PEAK_HBM_GBS
                                     if args.workload in UPLOAD_BYTES else None,
                         "bytes_per_doc": round(bytes_per_step / max(args.docs * per_gpu, 1), 3),
                         "upload_width_bytes_per_doc": UPLOAD_BYTES.get(args.workload),
                         "effective_gbs": UPLOAD_BYTES[args.workload] * args.docs * per_gpu / (avg_kernel_ms / 1000.0) / 1e9
                                          if args.workload in UPLOAD_BYTES else None,
                         "kernel": "collect_kernel", "kernel_ms": avg_kernel_ms * args.steps / launches,
                         "algorithmic_bytes_per_launch": kernel_bytes[0] // launches},
            "exchange": exchange,
            "precomputed": precomputed,
            "host_ms_per_request": host_ms,
            "cpu_baseline": cpu,
            "checked": checked,
            "check_errors": check_errors[:5],
        }
        print(json.dumps(out), flush=True)
    builders.shutdown()
    reducer.shutdown()
    for st in sets:
        for p in st:
            p.close()
    for seg in segs:
        seg.close()
    if comm:
        comm.close()
    engine.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
