"""Three bucket levels on the GPU path (two terms and one histogram, the histogram at any level): the deepest level is
collected over the composite ordinal of the two terms fields (a * |B| + b) as the grid's ordinal dimension, and built
from the cells of the winners' composite rows (A/AggregatorFactories.java:68-79: every level's aggregators built per
owning bucket; GlobalOrdinalsStringTermsAggregator / HistogramAggregator .buildAggregation at each level).  Shard
results, the multi-shard reduce and the transport bytes are compared with the oracle."""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, reduce
from elasticsearch_amd import _native as N
from helpers import assert_same, bits_from_mask

pytestmark = pytest.mark.gpu

T0 = 1441065600000
DAY = 86_400_000


def _segment(seed, n, t_a=300, t_b=12):
    rng = np.random.default_rng(seed)
    a = ((np.minimum(rng.zipf(1.2, size=n) - 1, t_a - 1) * 7919 + 13) % t_a).astype(np.uint32)
    a[rng.random(n) < 0.03] = 0xFFFFFFFF
    b = rng.integers(0, t_b, size=n).astype(np.uint32)
    b[rng.random(n) < 0.05] = 0xFFFFFFFF
    ts = T0 + np.sort(rng.integers(0, 6 * DAY, size=n)).astype(np.int64)
    num = rng.integers(0, 1000, size=n).astype(np.int64)
    present = rng.random(n) >= 0.1
    return {
        "a": {"type": N.COL_ORD_U32, "values": a, "terms": ["a%04d" % i for i in range(t_a)]},
        "b": {"type": N.COL_ORD_U32, "values": b, "terms": ["b%02d" % i for i in range(t_b)]},
        "@timestamp": {"type": N.COL_I64, "values": ts},
        "num": {"type": N.COL_I64, "values": np.where(present, num, 0), "present": bits_from_mask(present)},
        "h": {"type": N.COL_U64, "values": rng.integers(0, 5000, size=n).astype(np.uint64)},
    }


def _run(engine, aggs, shards=2, n=150_000):
    cols = [_segment(40 + s, n) for s in range(shards)]
    lookups = {f: {t: i for i, t in enumerate(cols[0][f]["terms"])} for f in ("a", "b")}
    ord_lookup = lambda f, t: lookups.get(f, {}).get(t, -1)  # noqa: E731
    want = O.run([(c, n) for c in cols], aggs, ord_lookup=ord_lookup, number_of_shards=shards, streams=True)
    plan = engine.plan(aggs, ord_lookup=ord_lookup, number_of_shards=shards)
    results = []
    for s in range(shards):
        seg = engine.upload_segment(cols[s], n)
        plan.reset()
        plan.collect(seg)
        r = plan.build()
        assert_same(r.to_dict(), want["shards"][s], f"shard{s}")
        assert r.to_stream() == want["streams"][s], f"shard{s} transport bytes"
        results.append(r)
        seg.close()
    red = reduce(results).to_dict()
    assert_same(red, want["reduced"], "reduced")
    plan.close()
    return red


def test_terms_terms_histogram(engine):
    """terms{terms{date_histogram{stats, cardinality}}} beside a metric of the middle level"""
    aggs = [AB.terms("A").field("a").size(6).subAggregation(
        AB.terms("B").field("b").size(4).subAggregation(AB.avg("n").field("num")).subAggregation(
            AB.dateHistogram("d").field("@timestamp").interval("1d")
            .subAggregation(AB.stats("s").field("num"))
            .subAggregation(AB.cardinality("c").field("h").precisionThreshold(100))))]
    red = _run(engine, aggs)
    assert red["A"]["buckets"][0]["B"]["buckets"][0]["d"]["buckets"]


def test_terms_histogram_terms(engine):
    """terms{date_histogram{terms{avg}}} with the deepest terms in count-asc order and min_doc_count 0"""
    aggs = [AB.terms("A").field("a").size(5).subAggregation(
        AB.dateHistogram("d").field("@timestamp").interval("2d").minDocCount(0)
        .extendedBounds(T0 - DAY, T0 + 8 * DAY).subAggregation(
            AB.terms("B").field("b").size(3).order(Order.count(True)).minDocCount(0)
            .subAggregation(AB.avg("n").field("num"))))]
    _run(engine, aggs)


@pytest.mark.parametrize("order", ["count", "term", "agg"])
def test_histogram_terms_terms(engine, order):
    """date_histogram{terms{terms{stats}}}: the middle terms per key, the deepest per (key, term)"""
    inner = AB.terms("B").field("b").size(3).subAggregation(AB.stats("s").field("num"))
    if order == "term":
        inner.order(Order.term(False))
    elif order == "agg":
        inner.order(Order.aggregation("s.max", True))
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("1d").subAggregation(
        AB.terms("A").field("a").size(4).subAggregation(inner))]
    _run(engine, aggs)


def test_three_levels_refusals(engine):
    """four levels, three terms, or a deep bucket that is not the middle level's last sub-aggregation stay refused"""
    four = [AB.terms("A").field("a").subAggregation(AB.terms("B").field("b").subAggregation(
        AB.dateHistogram("d").field("@timestamp").interval("1d").subAggregation(
            AB.histogram("x").field("num").interval(100))))]
    three_terms = [AB.terms("A").field("a").subAggregation(AB.terms("B").field("b").subAggregation(
        AB.terms("C").field("a")))]
    not_last = [AB.terms("A").field("a").subAggregation(AB.terms("B").field("b").subAggregation(
        AB.dateHistogram("d").field("@timestamp").interval("1d")).subAggregation(AB.avg("n").field("num")))]
    for aggs in (four, three_terms, not_last):
        with pytest.raises(N.UnsupportedOnGpu):
            engine.plan(aggs, ord_lookup=lambda f, t: -1)
