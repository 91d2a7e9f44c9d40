"""GPU parity of the floored-stream HLL pass (config 4 on one fresh 125M-doc plan).

When a request's values per register are many, the register pass keeps only hashes whose run length reaches a floor F
(chosen from the doc count so that a register ending below F is a ~1e-3 event), logs them by register range and
gathers them once; registers still below F are finished by the tail pass from the hashes below F.  Each case runs the
same request under the context option `hll_floor`: 0 = the register phases (snapshot + logs), 1 = the floored stream,
4 = the floor raised by 3 (thousands of registers end below it: the tail pass does real work).  Registers (FNV-1a over
the register bytes), mode and estimate must equal the oracle's (HyperLogLogPlusPlus.java:232-268 collect, :363-376
merge) in every mode.
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


@pytest.fixture(scope="module")
def c4_125m():
    n = 125_000_000
    aggs = [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)]
    want = O.run([(synthetic_columns(("client_ip.hash",), n, shard=5), n)], aggs)
    return n, aggs, want


@pytest.mark.parametrize("mode", MODES)
def test_config4_fresh_125m_plan(engine, c4_125m, mode):
    """The 8-GPU per-GPU shape: one fresh plan over one 125M-doc shard (p = 18, ~477 values per register: F = 5)."""
    n, aggs, want = c4_125m
    seg = engine.synthetic_segment(n, fields=("client_ip.hash",), shard=5)
    with floor_mode(engine, mode):
        plan = engine.plan(aggs)
        plan.collect(seg)
        res = plan.build()
        plan.close()
    seg.close()
    got = res.to_dict()
    assert got["ips"]["_internal"]["mode"] == "hll"
    assert_same(got, want["shards"][0], f"mode {mode} shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], f"mode {mode} reduced")


@pytest.mark.parametrize("mode", MODES)
def test_merged_shards_continue_the_floor(engine, mode):
    """4 x 30M-doc segments into one plan: the floor is chosen from the values the registers will have seen after each
    segment (30M values over 2^18 registers: too few for a floor, the phases; then F = 4, 5, 5), so later segments keep
    fewer hashes."""
    n, shards = 30_000_000, 4
    fields = ("client_ip.hash",)
    aggs = [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)]
    want = O.run([(synthetic_columns(fields, n, shard=10 + s), n) for s in range(shards)], aggs, number_of_shards=shards)
    segs = [engine.synthetic_segment(n, fields=fields, shard=10 + s) for s in range(shards)]
    with floor_mode(engine, mode):
        plan = engine.plan(aggs, number_of_shards=shards)
        for seg in segs:
            plan.collect(seg)
        got = reduce([plan.build()]).to_dict()
        plan.close()
    for seg in segs:
        seg.close()
    assert_same(got, want["reduced"], f"mode {mode} merged")


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("field,thr", [("client_ip.hash", 1000), ("price", 1000), ("price", 40000)])
def test_smaller_precision_and_double_values(engine, mode, field, thr):
    """p = 13 (128 register ranges of 64 instead of 256) and a double column (doubleToLongBits, NaN canonicalised) over 24M
    docs; at p = 18 the double column has too few values per register for a floor (the phases run in every mode)."""
    n = 24_000_000
    aggs = [AB.cardinality("c").field(field).precisionThreshold(thr)]
    want = O.run([(synthetic_columns((field,), n, shard=7), n)], aggs)
    seg = engine.synthetic_segment(n, fields=(field,), shard=7)
    with floor_mode(engine, mode):
        plan = engine.plan(aggs)
        plan.collect(seg)
        got = plan.build().to_dict()
        plan.close()
    seg.close()
    assert_same(got, want["shards"][0], f"mode {mode} {field}")


def test_upload_segment_with_few_distinct_values(engine):
    """A column with 5,000 distinct longs repeated over 100M docs: most registers stay 0 (below any floor), so the
    floored stream's gather leaves ~2^18 unresolved registers and the tail pass decides them; the request ends in
    LINEAR_COUNTING (5,000 distinct <= 40,000) exactly as the reference's hash set would."""
    rng = np.random.default_rng(77)
    n = 100_000_000
    vals = rng.integers(-(1 << 62), 1 << 62, size=5000)[rng.integers(0, 5000, size=n)].astype(np.int64)
    cols = {"v": {"type": N.COL_I64, "values": vals}}
    aggs = [AB.cardinality("c").field("v").precisionThreshold(40000)]
    want = O.run([(cols, n)], aggs)
    for mode in (1, 4):
        with floor_mode(engine, mode):
            seg = engine.upload_segment(cols, n)
            plan = engine.plan(aggs)
            plan.collect(seg)
            got = plan.build().to_dict()
            plan.close()
            seg.close()
        assert got["c"]["_internal"]["mode"] == "lc"
        assert_same(got, want["shards"][0], f"mode {mode}")
