"""The shard reduce across ranks (esgpu_comm_reduce) on CPU: world_size 2 and 4 over gloo (the host transport of
esgpu_comm_init_host), several shards per rank, against esgpu_reduce over every shard in shard order and against the
oracle's coordinator reduce.

Fixed-shape partials (top-level histograms with metric subs, top-level metrics, top-level cardinality) take the
all-reduce path (their f64 sums all-gathered per shard and added in shard order); terms take the all-gather path, in
two phases when their order is a count or term order (terms-level skeletons first, then only the surviving buckets'
sub-aggregations).  Both reduces must produce identical JSON, for integer-valued and non-integer doubles alike."""
import json
import socket

import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, ShardResult, reduce
from helpers import assert_same, synthetic_columns
from result_stream import cardinality, encode, from_shard_json

SHARDS = 4


def _request(metric_field):
    return [AB.terms("hosts").field("host").size(5).subAggregation(AB.stats("rt").field(metric_field)),
            AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(
                AB.extendedStats("x").field(metric_field)).subAggregation(AB.avg("a").field("response_time_ms")),
            AB.histogram("rt_hist").field("response_time_ms").interval(100).minDocCount(0).extendedBounds(-300, 1500)
              .subAggregation(AB.stats("s").field(metric_field)),
            AB.dateHistogram("busy").field("@timestamp").interval("6h").minDocCount(2000),
            AB.extendedStats("all").field(metric_field),
            AB.terms("ns").field("host").size(3).subAggregation(AB.dateHistogram("h").field("@timestamp").interval("1h")
                                                                 .subAggregation(AB.stats("s").field(metric_field))),
            AB.terms("by_term").field("host").size(4).order(Order.term(False)).subAggregation(
                AB.terms("inner").field("host").size(2).order(Order.count(True)))]


def _cards(shard, rng):
    """Three cardinality aggregations (p = 13, threshold 1536): every shard LC with a small union (stays LC), every shard
    LC with a union past the threshold (upgraded in the union), and shard 2 already in HYPERLOGLOG."""
    p = 13
    L = O.lib()

    def parts(hashes):
        regs = np.zeros(1 << p, dtype=np.uint8)
        enc = set()
        for h in hashes:
            idx = L.oracle_index(int(h), p)
            regs[idx] = max(regs[idx], L.oracle_run_len(int(h), p))
            enc.add(L.oracle_encode_hash(int(h), p) & 0xFFFFFFFF)
        return regs, enc

    out = []
    for name, n in (("small", 300), ("union", 1000), ("hll", 1000)):
        vals = rng.integers(0, 2**40, n + (5000 if name == "hll" and shard == 2 else 0))
        hashes = [L.oracle_mix64(int(v)) for v in vals]
        regs, enc = parts(hashes)
        thr = int((1 << p) / 4 * 0.75)
        out.append(cardinality(name, p, lc=enc) if len(enc) <= thr else cardinality(name, p, registers=regs))
    return out


def _shard_blobs(metric_field):
    aggs = _request(metric_field)
    fields = ("host", "@timestamp", "response_time_ms", metric_field)
    shards = [(synthetic_columns(fields, 150_000, shard=s), 150_000) for s in range(SHARDS)]
    want = O.run(shards, aggs, number_of_shards=SHARDS)
    rng = np.random.default_rng(7)
    blobs = [encode(from_shard_json(aggs, want["shards"][s], SHARDS) + _cards(s, rng)) for s in range(SHARDS)]
    return blobs, want


def _worker(rank, world, port, blobs, q):
    import torch.distributed as dist
    from elasticsearch_amd import Communicator
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = Communicator.over_process_group()
    per = len(blobs) // world
    local = [ShardResult.deserialize(b) for b in blobs[rank * per:(rank + 1) * per]]
    red = comm.reduce(local)
    ex = comm.last_exchange() + (comm.last_exchange_ms(),)
    again = comm.reduce(local)  # communicator state is reused across requests
    q.put((rank, red.to_json(), again.to_json(), ex))
    comm.close()
    dist.destroy_process_group()


def _run(world, blobs):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, blobs, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, js, js2, ex = q.get(timeout=180)
        out[r] = (json.loads(js), json.loads(js2), ex)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_comm_reduce_matches_shard_order_reduce(world):
    blobs, want = _shard_blobs("response_time_ms")
    ref = reduce([ShardResult.deserialize(b) for b in blobs]).to_dict()
    out = _run(world, blobs)
    for r in range(world):
        got, again, (ar_bytes, ag_bytes, ncoll, ex_ms) = out[r]
        assert json.dumps(got, sort_keys=True) == json.dumps(ref, sort_keys=True), f"rank {r}"
        assert again == got
        assert ar_bytes > (1 << 13)  # the HYPERLOGLOG registers and the dense histogram partials were all-reduced
        assert ag_bytes > 0 and ncoll >= 6 and ex_ms > 0
    for name in ("hosts", "per_hour", "rt_hist", "busy", "all", "ns", "by_term"):  # the oracle's coordinator reduce
        assert_same(out[0][0][name], want["reduced"][name], name)
    modes = {k: out[0][0][k]["_internal"]["mode"] for k in ("small", "union", "hll")}
    assert modes == {"small": "lc", "union": "hll", "hll": "hll"}


def test_comm_reduce_float_sums_bit_identical():
    """Non-integer doubles: the cross-rank sums are added in global shard order, so they are bit-identical to the
    shard-order reduce (the oracle's reduce is compared at the parity bar: its shard sums are its own collect's)."""
    blobs, want = _shard_blobs("price")
    ref = reduce([ShardResult.deserialize(b) for b in blobs]).to_dict()
    out = _run(2, blobs)
    assert json.dumps(out[1][0], sort_keys=True) == json.dumps(ref, sort_keys=True)
    for name in ("hosts", "per_hour", "rt_hist", "all", "ns"):
        assert_same(out[1][0][name], want["reduced"][name], name, exact_floats=False)


def test_two_phase_terms_exchange_moves_fewer_bytes():
    """The terms-level skeletons + surviving sub-trees move fewer all-gather bytes than whole shard records would
    (esgpu_comm_gather_reduce on the same shards sends whole records for every aggregation) -- same JSON."""
    aggs = [AB.terms("ns").field("host").size(2).subAggregation(AB.dateHistogram("h").field("@timestamp").interval("1h")
                                                                .subAggregation(AB.stats("s").field("response_time_ms")))]
    fields = ("host", "@timestamp", "response_time_ms")
    shards = [(synthetic_columns(fields, 200_000, shard=s), 200_000) for s in range(2)]
    want = O.run(shards, aggs, number_of_shards=2)
    blobs = [encode(from_shard_json(aggs, want["shards"][s], 2)) for s in range(2)]
    out = _run(2, blobs)
    full = sum(len(b) for b in blobs)
    got, _, (_, ag_bytes, _, _) = out[0]
    assert_same(got, want["reduced"], "reduced")
    assert ag_bytes < full / 2, (ag_bytes, full)
