"""Floating-point parity at the BASELINE sizes ("float parity").

north_star's bar for floating sums and averages is 1e-12 relative.  The reference adds doubles in doc order, so for
non-integer values (the synthetic `price`) and for integer sums past 2^53 (sum_of_squares of `bytes`) its own result
carries a rounding error that grows like sqrt(n) * 2^-53 -- about 1e-12 at 1e8 values in one bucket.  The oracle is
therefore run with exact=True: every stats / extended_stats / avg result carries "_exact", the exact sums it
approximates (double-double shadow accumulators, pinned against math.fsum in test_float_exact_oracle.py), and
helpers.assert_same_exact requires the GPU's compensated sums (plain f64 cells per workgroup, double-double flushes
into the grid, DESIGN §5 "Float parity") to lie within 1e-12 of them.  The largest errors of the oracle and of the GPU
against the exact values are written to $ESGPU_FLOAT_REPORT (JSON) when set.

Non-finite and subnormal values go through each accumulation path: LDS cells (terms{stats}), per-thread run
accumulators (histogram-only grids and top-level metrics), global atomics (a grid too large for LDS) and the
multi-valued kernel.
"""
import json
import math
import os

import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import FloatReport, assert_same_exact, bits_from_mask, synthetic_columns

pytestmark = pytest.mark.gpu

REPORT = {}


@pytest.fixture(scope="module", autouse=True)
def _write_report():
    yield
    path = os.environ.get("ESGPU_FLOAT_REPORT")
    if path and REPORT:
        with open(path, "w") as f:
            json.dump(REPORT, f, indent=1, sort_keys=True)


def _check(name, got, want, exact_floats=False):
    rep = FloatReport()
    assert_same_exact(got, want, name, exact_floats=exact_floats, report=rep, strict=True)
    REPORT[name] = rep.as_dict()
    return rep


def _synthetic(engine, aggs, fields, n, shard=0):
    cols = synthetic_columns(fields, n, shard=shard)
    want = O.run([(cols, n)], aggs, exact=True)
    del cols
    seg = engine.synthetic_segment(n, fields=fields, shard=shard)
    plan = engine.plan(aggs)
    plan.collect(seg)
    res = plan.build()
    got_shard, got = res.to_dict(), reduce([res]).to_dict()
    plan.close()
    seg.close()
    return got_shard, got, want


HOUR = AB.dateHistogram("per_hour").field("@timestamp").interval("1h")


def test_north_star_shape_over_price_100m(engine):
    """terms(host){date_histogram(1h){stats(price)}}, 100M docs: f64 LDS cells under a sliding key window."""
    aggs = [AB.terms("hosts").field("host").size(10).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.stats("p").field("price")))]
    got_shard, got, want = _synthetic(engine, aggs, ("host", "@timestamp", "price"), 100_000_000)
    _check("north_star_price_100m.shard", got_shard, want["shards"][0])
    _check("north_star_price_100m.reduced", got, want["reduced"])


def test_config2_over_price_100m(engine):
    """date_histogram(1h){extended_stats(price)} and a top-level extended_stats(price), 100M docs: the run accumulators
    of the histogram-only grid, and one cell summing 1e8 values (the oracle's own error is largest there)."""
    aggs = [AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.extendedStats("x").field("price")),
            AB.extendedStats("all").field("price"), AB.avg("avg").field("price")]
    got_shard, got, want = _synthetic(engine, aggs, ("@timestamp", "price"), 100_000_000)
    _check("config2_price_100m.shard", got_shard, want["shards"][0])
    _check("config2_price_100m.reduced", got, want["reduced"])


def test_extended_stats_bytes_past_2_53_100m(engine):
    """extended_stats(bytes): sums of squares reach 3e19 (past 2^53, every addition rounds), top level, under a 1-hour
    histogram and under terms; the sums of bytes themselves stay exact integers (bit-identical to the oracle)."""
    aggs = [AB.extendedStats("all").field("bytes"),
            AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.extendedStats("x").field("bytes")),
            AB.terms("hosts").field("host").size(5).subAggregation(AB.extendedStats("t").field("bytes"))]
    got_shard, got, want = _synthetic(engine, aggs, ("@timestamp", "host", "bytes"), 100_000_000)
    _check("ext_stats_bytes_100m.shard", got_shard, want["shards"][0], exact_floats=True)
    rep = _check("ext_stats_bytes_100m.reduced", got, want["reduced"], exact_floats=True)
    assert rep.oracle["sum_of_squares"] > 0.0  # the oracle's doc-order sums of squares did round
    assert got["all"]["sum_of_squares"] > 2.0 ** 53


def _special_column(rng, n, kind):
    v = rng.random(n) * 1000.0
    if kind == "inf":
        v[rng.integers(0, n, 20)] = math.inf
    elif kind == "inf_ninf":
        v[rng.integers(0, n, 20)] = math.inf
        v[rng.integers(0, n, 20)] = -math.inf
    elif kind == "nan":
        v[rng.integers(0, n, 5)] = math.nan
    elif kind == "subnormal":
        v = (rng.random(n) - 0.3) * 2.0 ** -1040
    elif kind == "mixed":  # -0.0, negative values and subnormals among ordinary values
        v[rng.integers(0, n, 50)] = -0.0
        v[rng.integers(0, n, 5000)] *= -1.0
        v[rng.integers(0, n, 100)] = 2.0 ** -1070
    return v


SPECIAL = ["inf", "inf_ninf", "nan", "subnormal", "mixed"]


@pytest.mark.parametrize("kind", SPECIAL)
def test_special_values_through_every_sum_path(engine, kind):
    """+-Inf (Inf + -Inf = NaN in Java), NaN, subnormals, -0.0 and negative values through: f64 LDS cells
    (terms{stats}), run accumulators (date_histogram{stats}, top-level stats / avg), global atomics (terms over 300,000
    ordinals: the grid exceeds LDS) and the multi-valued kernel (a second value on some docs)."""
    rng = np.random.default_rng(SPECIAL.index(kind) + 100)
    n = 2_000_000
    nt = 300_000
    t0 = 1_441_065_600_000
    price = _special_column(rng, n, kind)
    cols = {
        "host": {"type": N.COL_ORD_U32, "values": (rng.integers(0, 50, n)).astype(np.uint32),
                 "terms": ["h%03d" % i for i in range(50)]},
        "big": {"type": N.COL_ORD_U32, "values": rng.integers(0, nt, n).astype(np.uint32),
                "terms": ["t%06d" % i for i in range(nt)]},
        "@timestamp": {"type": N.COL_I64, "values": np.sort(rng.integers(t0, t0 + 86_400_000, n)).astype(np.int64)},
        "price": {"type": N.COL_F64, "values": price},
    }
    # multi-valued copy: every 7th doc has a second value (CSR)
    counts = np.ones(n, dtype=np.int64)
    counts[::7] = 2
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(counts)
    mv = np.empty(int(offs[-1]), dtype=np.float64)
    mv[offs[:-1].astype(np.int64)] = price
    second = offs[:-1][::7].astype(np.int64) + 1
    mv[second] = _special_column(rng, len(second), kind)
    cols["mprice"] = {"type": N.COL_F64, "values": mv, "offsets": offs}
    aggs = [AB.terms("hosts").field("host").size(50).subAggregation(AB.stats("s").field("price")),
            AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.extendedStats("x").field("price")),
            AB.stats("all").field("price"), AB.avg("avg").field("price"),
            AB.terms("big").field("big").size(20).subAggregation(AB.extendedStats("g").field("price")),
            AB.terms("mh").field("host").size(50).subAggregation(AB.extendedStats("m").field("mprice")),
            AB.stats("mall").field("mprice")]
    want = O.run([(cols, n)], aggs, exact=True)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs)
    plan.collect(seg)
    got = plan.build().to_dict()
    plan.close()
    seg.close()
    _check(f"special_{kind}", got, want["shards"][0])


def test_packed_cells_sums_past_2_53(engine):
    """Packed integer cells decode count * base + sum of deltas exactly; with a 10^12 base the cell sums pass 2^53 and
    are added into the grid as double-doubles: the GPU's sums are the exact sums rounded once."""
    rng = np.random.default_rng(42)
    n = 3_000_000
    t0 = 1_441_065_600_000
    cols = {
        "host": {"type": N.COL_ORD_U32, "values": rng.integers(0, 40, n).astype(np.uint32),
                 "terms": ["h%02d" % i for i in range(40)]},
        "@timestamp": {"type": N.COL_I64, "values": np.sort(rng.integers(t0, t0 + 86_400_000, n)).astype(np.int64)},
        "rt": {"type": N.COL_I64, "values": rng.integers(10 ** 12, 10 ** 12 + 999, n).astype(np.int64)},
    }
    aggs = [AB.terms("h").field("host").size(40).subAggregation(
                AB.dateHistogram("d").field("@timestamp").interval("1h").subAggregation(AB.stats("s").field("rt"))),
            AB.terms("a").field("host").size(9).subAggregation(AB.avg("m").field("rt"))]
    want = O.run([(cols, n)], aggs, exact=True)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs)
    plan.collect(seg)
    got = plan.build().to_dict()
    plan.close()
    seg.close()
    rep = _check("packed_base_1e12", got, want["shards"][0], exact_floats=True)
    assert rep.got["sum"] <= 1.2e-16  # the exact sum, rounded once


def test_live_docs_over_price_multi_segment(engine):
    """Two segments (the compensated low parts folded after each) with 30 % deleted docs, date_histogram{avg(price)}."""
    n = 5_000_000
    fields = ("@timestamp", "price")
    rng = np.random.default_rng(7)
    aggs = [AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.avg("a").field("price")),
            AB.extendedStats("all").field("price")]
    cols = [synthetic_columns(fields, n, shard=s) for s in range(2)]
    live = [bits_from_mask(rng.random(n) >= 0.3) for _ in range(2)]
    allc = {f: dict(cols[0][f], values=np.concatenate([c[f]["values"] for c in cols])) for f in fields}
    bits = np.concatenate([np.unpackbits(live[s].view(np.uint8), bitorder="little")[:n] for s in range(2)]).astype(bool)
    want = O.run([(allc, 2 * n)], aggs, accept=[bits_from_mask(bits)], exact=True)
    segs = [engine.synthetic_segment(n, fields=fields, shard=s) for s in range(2)]
    plan = engine.plan(aggs)
    for s in range(2):
        plan.collect(segs[s], accept_bits=live[s])
    got = plan.build().to_dict()
    plan.close()
    for s in segs:
        s.close()
    _check("live_docs_price_2seg", got, want["shards"][0])
