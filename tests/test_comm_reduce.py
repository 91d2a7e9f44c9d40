"""The shard reduce across ranks (esgpu_comm_reduce) on CPU: world_size 2 and 4 over gloo (the host transport of
esgpu_comm_init_host), several shards per rank, against esgpu_reduce over every shard in shard order and against the
oracle's coordinator reduce.

Fixed-shape partials (top-level histograms with metric subs, top-level metrics, top-level cardinality) take the
all-reduce path; terms take the all-gather path.  With integer-valued metrics the two reduces must produce identical
JSON; with non-integer doubles the sums agree within the parity bar (1e-12 relative)."""
import json
import socket

import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import ShardResult, reduce
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
            AB.extendedStats("all").field(metric_field)]


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
    ex = comm.last_exchange()
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
        got, again, (ar_bytes, ag_bytes, ncoll) = out[r]
        assert json.dumps(got, sort_keys=True) == json.dumps(ref, sort_keys=True), f"rank {r}"
        assert again == got
        assert ar_bytes > (1 << 13)  # the HYPERLOGLOG registers and the dense histogram partials were all-reduced
        assert ag_bytes > 0 and ncoll >= 6
    for name in ("hosts", "per_hour", "rt_hist", "busy", "all"):  # the oracle's coordinator reduce
        assert_same(out[0][0][name], want["reduced"][name], name)
    modes = {k: out[0][0][k]["_internal"]["mode"] for k in ("small", "union", "hll")}
    assert modes == {"small": "lc", "union": "hll", "hll": "hll"}


def test_comm_reduce_float_sums_within_parity_bar():
    blobs, want = _shard_blobs("price")
    ref = reduce([ShardResult.deserialize(b) for b in blobs]).to_dict()
    out = _run(2, blobs)
    assert_same(out[1][0], ref, "vs shard-order reduce", exact_floats=False)
    for name in ("hosts", "per_hour", "rt_hist", "all"):
        assert_same(out[1][0][name], want["reduced"][name], name, exact_floats=False)
