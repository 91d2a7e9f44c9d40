"""GPU parity of the floored-stream HLL pass (config 4 on one fresh 125M-doc plan).

When a request's distinct values per register are many, the register pass keeps only hashes whose run length reaches a
floor F, logs them by register range and gathers them once; registers still below F are finished by the tail pass from
the hashes below F.  F comes from the segment's distinct count, estimated from the registers of an earlier request that
collected the segment alone (the first request on a segment runs the register phases), so every case runs its request
twice.  Each case runs under the context option `hll_floor`: 0 = the register phases (snapshot + logs), 1 = the floored
stream, 4 = the floor raised by 3 (thousands of registers end below it: the tail pass does real work).  Registers
(FNV-1a over the register bytes), mode and estimate must equal the oracle's (HyperLogLogPlusPlus.java:232-268 collect,
:363-376 merge) in every mode and on both requests.
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same, synthetic_columns

pytestmark = pytest.mark.gpu

MODES = [0, 1, 4]


class floor_mode:
    def __init__(self, engine, v):
        self.e, self.v = engine, v

    def __enter__(self):
        self.e.set_option("hll_floor", self.v)

    def __exit__(self, *a):
        self.e.set_option("hll_floor", 1)


def _twice(engine, aggs, segs, mode, number_of_shards=1):
    """the request twice over the same segments (the first one leaves the segments' distinct estimates)"""
    out = []
    with floor_mode(engine, mode):
        plan = engine.plan(aggs, number_of_shards=number_of_shards)
        for _ in range(2):
            plan.reset()
            for s in segs:
                plan.collect(s)
            out.append(plan.build())
        plan.close()
    return out


@pytest.fixture(scope="module")
def c4_125m():
    n = 125_000_000
    aggs = [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)]
    want = O.run([(synthetic_columns(("client_ip.hash",), n, shard=5), n)], aggs)
    return n, aggs, want


@pytest.mark.parametrize("mode", MODES)
def test_config4_fresh_125m_plan(engine, c4_125m, mode):
    """The 8-GPU per-GPU shape: one fresh plan over one 125M-doc shard (p = 18, ~81M distinct values: F = 5)."""
    n, aggs, want = c4_125m
    seg = engine.synthetic_segment(n, fields=("client_ip.hash",), shard=5)
    for k, res in enumerate(_twice(engine, aggs, [seg], mode)):
        got = res.to_dict()
        assert got["ips"]["_internal"]["mode"] == "hll"
        assert_same(got, want["shards"][0], f"mode {mode} request {k} shard")
        assert_same(reduce([res]).to_dict(), want["reduced"], f"mode {mode} request {k} reduced")
    seg.close()


@pytest.mark.parametrize("mode", MODES)
def test_merged_shards_continue_the_floor(engine, mode):
    """4 x 15M-doc segments into one plan after each was collected alone once (their distinct estimates; each later
    segment's floor comes from the largest estimate so far).  At p = 18 (~14M distinct per segment) no segment reaches a
    floor (the phases run); at p = 14 every segment takes F = 6."""
    n, shards = 15_000_000, 4
    fields = ("client_ip.hash",)
    for thr in (40000, 2000):
        aggs = [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(thr)]
        want = O.run([(synthetic_columns(fields, n, shard=10 + s), n) for s in range(shards)], aggs, number_of_shards=shards)
        segs = [engine.synthetic_segment(n, fields=fields, shard=10 + s) for s in range(shards)]
        with floor_mode(engine, mode):
            for seg in segs:  # each segment alone first: its distinct estimate
                p1 = engine.plan(aggs)
                p1.collect(seg)
                p1.build()
                p1.close()
        for k, res in enumerate(_twice(engine, aggs, segs, mode, number_of_shards=shards)):
            assert_same(reduce([res]).to_dict(), want["reduced"], f"threshold {thr} mode {mode} request {k} merged")
        for seg in segs:
            seg.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("field,thr", [("client_ip.hash", 1000), ("price", 1000), ("price", 40000)])
def test_smaller_precision_and_double_values(engine, mode, field, thr):
    """p = 13 (128 register ranges of 64 instead of 256) and a double column (doubleToLongBits, NaN canonicalised) over
    8M docs (F = 7: the stream takes segments of up to 1,024 values per register); at p = 18 the double column has too
    few values per register for a floor (the phases run in every mode)."""
    n = 8_000_000
    aggs = [AB.cardinality("c").field(field).precisionThreshold(thr)]
    want = O.run([(synthetic_columns((field,), n, shard=7), n)], aggs)
    seg = engine.synthetic_segment(n, fields=(field,), shard=7)
    for k, res in enumerate(_twice(engine, aggs, [seg], mode)):
        assert_same(res.to_dict(), want["shards"][0], f"mode {mode} {field} request {k}")
    seg.close()


def test_repeated_values(engine):
    """120M docs over a pool of 2^26 longs (~56M distinct, ~2 docs per value): the floor follows the distinct count
    (F = 4), not the doc count (F = 5 would leave registers below it for the tail pass); then the same with the floor
    raised (tail pass)."""
    rng = np.random.default_rng(77)
    n = 120_000_000
    cols = {"v": {"type": N.COL_I64, "values": rng.integers(0, 1 << 26, size=n, dtype=np.int64)}}
    aggs = [AB.cardinality("c").field("v").precisionThreshold(40000)]
    want = O.run([(cols, n)], aggs)
    seg = engine.upload_segment(cols, n)
    del cols
    for mode in (1, 4):
        for k, res in enumerate(_twice(engine, aggs, [seg], mode)):
            got = res.to_dict()
            assert got["c"]["_internal"]["mode"] == "hll"
            assert_same(got, want["shards"][0], f"mode {mode} request {k}")
    seg.close()
