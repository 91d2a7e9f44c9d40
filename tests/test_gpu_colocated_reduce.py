"""GPU parity of the co-located reduce (esgpu_plans_build_reduce): the shards of one request whose plans
live on one device, reduced without building every shard result.  Each case compares build_reduce(plans) with the
reduce of the shard builds (InternalAggregations.reduce, shard order) bit for bit, and with the oracle's reduce.

Covered: the north star and config 5 shapes over 4-8 shards, several metric leaves (stats, avg, extended_stats on one
histogram), shards whose key ranges differ (a timestamp span per shard), a sparse metric (value counts apart from doc
counts), double metrics with NaN and -0.0 (Java Math.min / max over the shards), term and ascending count orders,
histogram options (min_doc_count 3 with key-descending order, extended bounds, min_doc_count 1), and shapes outside the
merge (terms{stats}, histograms ordered by count, a second child) that build and reduce instead.
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, QueryBuilders as QB
from elasticsearch_amd import _native as N
from elasticsearch_amd import build_reduce, colocated, reduce
from helpers import assert_same, bits_from_mask, synthetic_columns

pytestmark = pytest.mark.gpu

NS_FIELDS = ("host", "@timestamp", "response_time_ms")
C5_FIELDS = ("status", "bytes", "host", "@timestamp", "response_time_ms")


def _both(engine, aggs, segs, filters=None):
    """(build_reduce result, reduce-of-builds result) over one plan per segment"""
    shards = len(segs)
    plans = [engine.plan(aggs, filters=filters, number_of_shards=shards) for _ in segs]
    for p, s in zip(plans, segs):
        p.collect(s)
    fused = build_reduce(plans).to_dict()
    for p, s in zip(plans, segs):
        p.reset()
        p.collect(s)
    plain = reduce([p.build() for p in plans]).to_dict()
    for p in plans:
        p.close()
    return fused, plain


@pytest.mark.parametrize("shards", [2, 8])
def test_north_star_shards(engine, shards):
    n = 1_500_000
    aggs = [AB.terms("hosts").field("host").size(10).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("response_time_ms")))]
    segs = [engine.synthetic_segment(n, fields=NS_FIELDS, shard=s) for s in range(shards)]
    probe = [engine.plan(aggs, number_of_shards=shards) for _ in segs]
    assert colocated(probe)
    for p in probe:
        p.close()
    fused, plain = _both(engine, aggs, segs)
    assert_same(fused, plain, "fused vs builds")
    want = O.run([(synthetic_columns(NS_FIELDS, n, shard=s), n) for s in range(shards)], aggs, number_of_shards=shards)
    assert_same(fused, want["reduced"], "fused vs oracle")
    for s in segs:
        s.close()


def test_config5_shape_several_leaves(engine):
    n, shards = 1_200_000, 6
    aggs = [AB.terms("hosts").field("host").size(7).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("3h")
        .subAggregation(AB.avg("a").field("response_time_ms"))
        .subAggregation(AB.stats("s").field("bytes"))
        .subAggregation(AB.extendedStats("e").field("response_time_ms")))]
    filters = [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)]
    segs = [engine.synthetic_segment(n, fields=C5_FIELDS, shard=s) for s in range(shards)]
    fused, plain = _both(engine, aggs, segs, filters=filters)
    assert_same(fused, plain, "fused vs builds")
    want = O.run([(synthetic_columns(C5_FIELDS, n, shard=s), n) for s in range(shards)], aggs, filters=filters,
                 number_of_shards=shards)
    assert_same(fused, want["reduced"], "fused vs oracle", exact_floats=False)
    for s in segs:
        s.close()


def _log_shard(rng, n, t0, span_ms, metric, present=None, nterms=200):
    ranks = np.minimum(rng.zipf(1.3, size=n) - 1, nterms - 1)
    cols = {
        "host": {"type": N.COL_ORD_U32, "values": ((ranks * 17 + 3) % nterms).astype(np.uint32),
                 "terms": ["h%03d" % i for i in range(nterms)]},
        "@timestamp": {"type": N.COL_I64, "values": np.sort(rng.integers(t0, t0 + span_ms, size=n)).astype(np.int64)},
        "m": metric,
    }
    if present is not None:
        cols["m"] = dict(metric, present=bits_from_mask(present))
    return cols


def test_shards_with_different_key_ranges_sparse_and_double_metrics(engine):
    """Shard s covers days s .. s+2 (its grid's first key differs), the metric is a double column with NaN and -0.0 in
    some shards and missing on 20 % of the docs (value counts apart from doc counts)."""
    rng = np.random.default_rng(91)
    t0 = 1_441_065_600_000
    shard_cols = []
    for s in range(5):
        n = 400_000 + 50_000 * s
        vals = rng.normal(100.0, 30.0, size=n)
        if s == 1:
            vals[::997] = np.nan
        if s == 3:
            vals[::501] = -0.0
        pres = rng.random(n) >= 0.2
        vals[~pres] = 0.0
        shard_cols.append((_log_shard(rng, n, t0 + s * 86_400_000, 3 * 86_400_000, {"type": N.COL_F64, "values": vals},
                                      present=pres), n))
    aggs = [AB.terms("t").field("host").size(12).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("2h")
        .subAggregation(AB.stats("s").field("m")).subAggregation(AB.extendedStats("e").field("m")))]
    segs = [engine.upload_segment(c, n) for c, n in shard_cols]
    fused, plain = _both(engine, aggs, segs)
    # double sums are accumulated by device atomics: the two collects' per-shard sums may differ in the last bits
    assert_same(fused, plain, "fused vs builds", exact_floats=False)
    want = O.run(shard_cols, aggs, number_of_shards=len(shard_cols))
    assert_same(fused, want["reduced"], "fused vs oracle", exact_floats=False)
    for s in segs:
        s.close()


@pytest.mark.parametrize("order", [Order.term(True), Order.term(False), Order.count(True)])
def test_other_orders(engine, order):
    n, shards = 800_000, 4
    aggs = [AB.terms("hosts").field("host").size(6).order(order).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("1d").subAggregation(AB.avg("a").field("response_time_ms")))]
    segs = [engine.synthetic_segment(n, fields=NS_FIELDS, shard=10 + s) for s in range(shards)]
    fused, plain = _both(engine, aggs, segs)
    assert_same(fused, plain, "fused vs builds")
    for s in segs:
        s.close()


def test_shards_with_their_own_dictionaries(engine):
    """Each shard's segment has its own term dictionary (the same term has different ordinals in different shards): the
    final terms are matched to each shard's rows by their bytes."""
    rng = np.random.default_rng(17)
    t0 = 1_441_065_600_000
    shard_cols = []
    for s in range(4):
        n = 250_000
        cols = _log_shard(rng, n, t0, 86_400_000, {"type": N.COL_I64, "values": rng.integers(0, 500, size=n).astype(np.int64)})
        cols["host"]["terms"] = sorted("h%03d" % (i + 37 * s) for i in range(200))  # shifted: shared terms, other ordinals
        shard_cols.append((cols, n))
    aggs = [AB.terms("t").field("host").size(15).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.stats("s").field("m")))]
    segs = [engine.upload_segment(c, n) for c, n in shard_cols]
    fused, plain = _both(engine, aggs, segs)
    assert_same(fused, plain, "fused vs builds")
    want = O.run(shard_cols, aggs, number_of_shards=len(shard_cols))
    assert_same(fused, want["reduced"], "fused vs oracle")
    for s in segs:
        s.close()


@pytest.mark.parametrize("T", [1000, 150_000])
def test_plain_terms_builds_side_by_side(engine, T):
    """terms without sub-aggregations (config 3's shape): the shards' builds run side by side on the host pool and the
    reference reduce follows -- 1,000 terms (host selection) and 150,000 (the high-cardinality path and its GPU top-k)."""
    rng = np.random.default_rng(T)
    shard_cols = []
    for s in range(4):
        n = 600_000
        ranks = np.minimum(rng.zipf(1.1, size=n) - 1, T - 1)
        cols = {"kw": {"type": N.COL_ORD_U32, "values": ((ranks * 7919 + 17 * s) % T).astype(np.uint32),
                       "terms": ["u%07d" % i for i in range(T)]}}
        shard_cols.append((cols, n))
    aggs = [AB.terms("c").field("kw").size(15), AB.terms("a").field("kw").size(6).order(Order.count(True))]
    segs = [engine.upload_segment(c, n) for c, n in shard_cols]
    probe = [engine.plan(aggs, number_of_shards=len(segs)) for _ in segs]
    assert not colocated(probe)  # two top-level aggregations: built and reduced
    for p in probe:
        p.close()
    aggs = aggs[:1]
    probe = [engine.plan(aggs, number_of_shards=len(segs)) for _ in segs]
    assert colocated(probe)
    for p in probe:
        p.close()
    fused, plain = _both(engine, aggs, segs)
    assert_same(fused, plain, "fused vs builds")
    want = O.run(shard_cols, aggs, number_of_shards=len(shard_cols))
    assert_same(fused, want["reduced"], "fused vs oracle")
    for s in segs:
        s.close()


@pytest.mark.parametrize("nterms", [3000, 6000])
def test_many_terms_and_shard_min_doc_count(engine, nterms):
    """Over 4,096 terms the shards' selection runs on the host (select_terms), up to 4,096 on the device; a
    shard_min_doc_count bounds the candidates either way."""
    rng = np.random.default_rng(nterms)
    t0 = 1_441_065_600_000
    shard_cols = []
    for s in range(3):
        n = 300_000
        vals = rng.integers(0, 1000, size=n).astype(np.int64)
        shard_cols.append((_log_shard(rng, n, t0, 2 * 86_400_000, {"type": N.COL_I64, "values": vals}, nterms=nterms), n))
    aggs = [AB.terms("t").field("host").size(40).shardSize(60).shardMinDocCount(3).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("3h").subAggregation(AB.stats("s").field("m")))]
    segs = [engine.upload_segment(c, n) for c, n in shard_cols]
    fused, plain = _both(engine, aggs, segs)
    assert_same(fused, plain, "fused vs builds")
    want = O.run(shard_cols, aggs, number_of_shards=len(shard_cols))
    assert_same(fused, want["reduced"], "fused vs oracle")
    for s in segs:
        s.close()


@pytest.mark.parametrize("hist", ["mdc3_desc", "bounds", "mdc1"])
def test_histogram_options(engine, hist):
    """min_doc_count above 1 with key-descending order, extended bounds wider than the data (min_doc_count 0's empty
    buckets outside the keys), min_doc_count 1 (no empty buckets)"""
    n, shards = 700_000, 4
    h = AB.dateHistogram("h").field("@timestamp").interval("1h")
    if hist == "mdc3_desc":
        h = h.minDocCount(3).order(Order.KEY_DESC)
    elif hist == "bounds":
        ts = [synthetic_columns(("@timestamp",), n, shard=30 + s)["@timestamp"]["values"] for s in range(shards)]
        lo, hi = min(int(t.min()) for t in ts), max(int(t.max()) for t in ts)
        h = h.extendedBounds(lo - 5 * 86_400_000, hi + 3 * 86_400_000)
    else:
        h = h.minDocCount(1)
    aggs = [AB.terms("hosts").field("host").size(8).subAggregation(h.subAggregation(AB.stats("s").field("response_time_ms")))]
    segs = [engine.synthetic_segment(n, fields=NS_FIELDS, shard=30 + s) for s in range(shards)]
    probe = [engine.plan(aggs, number_of_shards=shards) for _ in segs]
    assert colocated(probe)
    for p in probe:
        p.close()
    fused, plain = _both(engine, aggs, segs)
    assert_same(fused, plain, f"{hist}: fused vs builds")
    for s in segs:
        s.close()


@pytest.mark.parametrize("shape", ["terms_stats", "count_order", "two_children"])
def test_shapes_outside_the_merge(engine, shape):
    n, shards = 600_000, 3
    if shape == "terms_stats":
        aggs = [AB.terms("hosts").field("host").size(5).subAggregation(AB.stats("s").field("response_time_ms"))]
    elif shape == "count_order":
        aggs = [AB.terms("hosts").field("host").size(5).subAggregation(
            AB.dateHistogram("h").field("@timestamp").interval("1d").order(Order.COUNT_DESC).subAggregation(AB.avg("a").field("response_time_ms")))]
    else:
        aggs = [AB.terms("hosts").field("host").size(5)
                .subAggregation(AB.dateHistogram("h").field("@timestamp").interval("1d"))
                .subAggregation(AB.avg("a").field("response_time_ms"))]
    segs = [engine.synthetic_segment(n, fields=NS_FIELDS, shard=20 + s) for s in range(shards)]
    probe = [engine.plan(aggs, number_of_shards=shards) for _ in segs]
    assert not colocated(probe)
    for p in probe:
        p.close()
    fused, plain = _both(engine, aggs, segs)
    assert_same(fused, plain, f"{shape}: fused vs builds")
    for s in segs:
        s.close()
