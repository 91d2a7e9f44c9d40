"""The device-resident reduce across ranks (esgpu_comm_build_reduce; VERDICT round 4 "what's missing" #1).

Each rank passes its collected shard plans; for the co-located shape (terms{histogram{metric leaves}}: the north star,
config 5) the shards' terms selections run on each device, their {count, ordinal} records are all-gathered from device
memory, InternalTerms.doReduce runs once per rank on the skeletons, and only the surviving terms' histogram rows are
all-gathered device to device and merged in global shard order.  The result must be identical to esgpu_reduce over
the shards' own builds (and to the oracle), for every transport:
  * in-process ranks (Communicator.local: one thread and one context per rank on this GPU), world 2 / 4 / 8;
  * RCCL with one rank (two local shards);
  * gloo between two processes sharing this GPU (Communicator.over_process_group: the host transport).
Shapes the co-located reduce does not take fall back to builds + esgpu_comm_reduce (path 0), with the same result.
Two shapes have device exchanges of their own (round 6): a plain terms aggregation (config 3: each shard's GPU top-k or
device selection made into a record, [header | records] all-gathered in one collective) and a top-level cardinality
(config 4: one all-reduce (max) of the u8 registers from device memory); a cardinality that may end in
LINEAR_COUNTING falls back (path 0).
"""
import json
import os
import tempfile
import threading

import pytest

import elasticsearch_amd as ea
import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import QueryBuilders as QB
from helpers import assert_same, synthetic_columns

pytestmark = pytest.mark.gpu

NS_FIELDS = ("host", "@timestamp", "response_time_ms")
C5_FIELDS = ("status", "bytes", "host", "@timestamp", "response_time_ms")


def _hour(metric):
    return AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(metric)


SHAPES = {
    "north_star": (lambda: [AB.terms("hosts").field("host").size(10).subAggregation(_hour(AB.stats("rt").field("response_time_ms")))],
                   NS_FIELDS, None, True),
    "config5": (lambda: [AB.terms("hosts").field("host").size(10).subAggregation(_hour(AB.avg("rt").field("response_time_ms")))],
                C5_FIELDS, [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)], True),
    "ext_stats_term_order": (lambda: [AB.terms("hosts").field("host").size(7).order(ea.Order.term(True)).subAggregation(
        AB.dateHistogram("d").field("@timestamp").interval("1d").minDocCount(0).subAggregation(
            AB.extendedStats("x").field("response_time_ms")).subAggregation(AB.avg("a").field("response_time_ms")))],
        NS_FIELDS, None, True),
    "count_asc_small_shard_size": (lambda: [AB.terms("hosts").field("host").size(5).shardSize(6).order(ea.Order.count(True))
                                            .minDocCount(2).subAggregation(_hour(AB.avg("rt").field("response_time_ms")))],
                                   NS_FIELDS, None, True),
    "count_desc_errors_shown": (lambda: [AB.terms("hosts").field("host").size(3).shardSize(4).showTermDocCountError(True)
                                         .subAggregation(_hour(AB.stats("rt").field("response_time_ms")))],
                                NS_FIELDS, None, True),
    "terms_stats_fallback": (lambda: [AB.terms("hosts").field("host").size(5).subAggregation(AB.stats("s").field("response_time_ms"))],
                             NS_FIELDS, None, False),
    # config 3: 10M url ordinals, the GPU top-k's keys made into records on the device
    "config3_urls": (lambda: [AB.terms("urls").field("url").size(10)], ("url",), None, True),
    # ... under a range filter: each shard's hot slots from the folded bitset, the scatter form deferred to the top-k
    "config3_urls_filtered": (lambda: [AB.terms("urls").field("url").size(10)], ("url", "bytes"),
                              [QB.rangeQuery("bytes").lt(800000)], True),
    "urls_count_asc_errors": (lambda: [AB.terms("urls").field("url").size(4).shardSize(9).order(ea.Order.count(True))
                                       .showTermDocCountError(True)], ("url",), None, True),
    # plain terms over 1,000 hosts: the co-located device selection (count and term orders)
    "hosts_plain": (lambda: [AB.terms("hosts").field("host").size(5)], ("host",), None, True),
    "hosts_plain_term_desc": (lambda: [AB.terms("hosts").field("host").size(6).order(ea.Order.term(False))], ("host",), None, True),
    # config 4: a sketch in HYPERLOGLOG on every shard
    "config4_card": (lambda: [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)], ("client_ip.hash",),
                     None, True),
    "card_p14_hll": (lambda: [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(1000)], ("client_ip.hash",),
                     None, True),
    # every shard in LINEAR_COUNTING and a small union: builds + reduce (path 0)
    "card_lc_fallback": (lambda: [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)], ("client_ip.hash",),
                         None, False, 3_000),
}
DOCS = 1_500_000


def _docs(shape):
    t = SHAPES[shape]
    return t[4] if len(t) > 4 else DOCS


def _expected(shape, nshards):
    aggs_f, fields, filters = SHAPES[shape][:3]
    eng = ea.Engine(0)
    res = []
    for s in range(nshards):
        seg = eng.synthetic_segment(_docs(shape) + 1000 * s, fields=fields, shard=s)
        plan = eng.plan(aggs_f(), filters=filters, number_of_shards=nshards)
        plan.collect(seg)
        res.append(plan.build())
        plan.close()
        seg.close()
    want = ea.reduce(res).to_dict()
    eng.close()
    return want


def _rank(shape, world, rank, n_local, group, out, root):
    aggs_f, fields, filters = SHAPES[shape][:3]
    eng = ea.Engine(0)
    comm = ea.Communicator.local(group, world, rank)
    segs, plans = [], []
    for i in range(n_local):
        s = rank * n_local + i
        segs.append(eng.synthetic_segment(_docs(shape) + 1000 * s, fields=fields, shard=s))
        plans.append(eng.plan(aggs_f(), filters=filters, number_of_shards=world * n_local))
    for rep in range(2):  # a second request on the same plans (reset, collect again)
        for p, seg in zip(plans, segs):
            p.reset()
            p.collect(seg)
        r = comm.build_reduce(plans, root=root)
        out[(rank, rep)] = (r.to_dict(), comm.last_build_reduce())
    comm.close()
    for p in plans:
        p.close()
    for s in segs:
        s.close()
    eng.close()


def _run_local(shape, world, n_local, root):
    out, errs = {}, []

    def body(r):
        try:
            _rank(shape, world, r, n_local, f"t-{shape}-{world}-{n_local}", out, root)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    assert len(out) == 2 * world
    return out


@pytest.mark.parametrize("world,n_local", [(2, 1), (4, 2), (8, 1)])
@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_local_ranks_match_reduce_of_builds(shape, world, n_local):
    want = _expected(shape, world * n_local)
    out = _run_local(shape, world, n_local, root=0)
    device = SHAPES[shape][3]
    for rep in range(2):
        got, (path, ms) = out[(0, rep)]
        assert path == (1 if device else 0), (shape, path)
        assert_same(got, want, f"{shape} w{world} rep{rep}")
        for r in range(1, world):
            other, (p2, _) = out[(r, rep)]
            assert p2 == path
            if device:
                assert other == {}  # the root only
            else:
                assert_same(other, want, f"rank {r}")


@pytest.mark.parametrize("shape", ["north_star", "config3_urls", "config4_card"])
def test_local_ranks_every_rank_gets_the_result(shape):
    want = _expected(shape, 4)
    out = _run_local(shape, 4, 1, root=-1)
    for r in range(4):
        assert_same(out[(r, 1)][0], want, f"rank {r}")


def test_local_ranks_against_the_oracle():
    aggs_f, fields, filters = SHAPES["config5"][:3]
    world = 4
    shards = [(synthetic_columns(fields, DOCS + 1000 * s, shard=s), DOCS + 1000 * s) for s in range(world)]
    want = O.run(shards, aggs_f(), filters=filters, number_of_shards=world)["reduced"]
    out = _run_local("config5", world, 1, root=0)
    assert_same(out[(0, 0)][0], want, "config5 vs oracle")


@pytest.mark.parametrize("shape", ["north_star", "config3_urls", "config4_card"])
def test_rccl_one_rank_device_exchange(engine, shape):
    """RCCL with one rank and two local shards: the selection records and rows go through ncclAllGather, the
    cardinality registers through ncclAllReduce (max)."""
    aggs_f, fields = SHAPES[shape][:2]
    want = _expected(shape, 2)
    comm = ea.Communicator(engine, 1, 0, ea.Communicator.unique_id())
    segs = [engine.synthetic_segment(_docs(shape) + 1000 * s, fields=fields, shard=s) for s in range(2)]
    plans = [engine.plan(aggs_f(), number_of_shards=2) for _ in range(2)]
    for rep in range(2):
        for p, s in zip(plans, segs):
            p.reset()
            p.collect(s)
        got = comm.build_reduce(plans, root=0).to_dict()
        assert comm.last_build_reduce()[0] == 1
        assert_same(got, want, f"rccl one rank {shape} rep{rep}")
    comm.close()
    for p in plans:
        p.close()
    for s in segs:
        s.close()


def _gloo_worker(rank, world, port, path, shape="north_star"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    aggs_f, fields = SHAPES[shape][:2]
    eng = ea.Engine(0)
    comm = ea.Communicator.over_process_group()
    seg = eng.synthetic_segment(_docs(shape) + 1000 * rank, fields=fields, shard=rank)
    plan = eng.plan(aggs_f(), number_of_shards=world)
    plan.collect(seg)
    r = comm.build_reduce([plan], root=0)
    if rank == 0:
        with open(path, "w") as f:
            json.dump({"result": r.to_dict(), "path": comm.last_build_reduce()[0]}, f)
    comm.close()
    plan.close()
    seg.close()
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("shape", ["north_star", "config3_urls", "config4_card"])
def test_gloo_two_processes_host_transport(shape):
    import socket

    import torch.multiprocessing as mp
    want = _expected(shape, 2)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "r0.json")
        mp.start_processes(_gloo_worker, args=(2, port, path, shape), nprocs=2, join=True, start_method="spawn")
        with open(path) as f:
            got = json.load(f)
    assert got["path"] == 1
    assert_same(got["result"], want, f"gloo world 2 {shape}")
