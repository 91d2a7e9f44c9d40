"""GPU parity for general aggregator trees: a bucket aggregation with several children of mixed
kinds -- metrics beside a bucket sub-aggregation, metrics on different fields, sibling bucket sub-aggregations --
compiled to one pipeline per (inner bucket, metric field) and assembled into one result tree, the way
AggregatorFactories.createSubAggregators (A/AggregatorFactories.java:68-79) gives every child its own aggregator;
and terms ordered by a metric sub-aggregation (InternalOrder.Aggregation, A/bucket/terms/InternalOrder.java:149-225;
the doc_count_error -1 rule of InternalTerms.doReduce, :195-196)."""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, QueryBuilders as QB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same, bits_from_mask, synthetic_columns

pytestmark = pytest.mark.gpu

FIELDS = ("host", "@timestamp", "response_time_ms", "bytes", "status", "price", "client_ip.hash")


def _both(engine, aggs, n=600_000, filters=None, shards=1, exact=True, fields=FIELDS):
    want = O.run([(synthetic_columns(fields, n, shard=s), n) for s in range(shards)], aggs, filters=filters,
                 number_of_shards=shards)
    results = []
    plan = engine.plan(aggs, filters=filters, number_of_shards=shards)
    for s in range(shards):
        seg = engine.synthetic_segment(n, fields=fields, shard=s)
        plan.reset()
        plan.collect(seg)
        r = plan.build()
        assert_same(r.to_dict(), want["shards"][s], f"shard{s}", exact)
        results.append(r)
        seg.close()
    red = reduce(results).to_dict()
    assert_same(red, want["reduced"], "reduced", exact)
    plan.close()
    return red


def test_metrics_beside_a_bucket_sub_aggregation(engine):
    aggs = [AB.terms("hosts").field("host").size(8).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("6h").subAggregation(AB.stats("rt").field("response_time_ms")))
        .subAggregation(AB.stats("rt_all").field("response_time_ms")).subAggregation(AB.avg("b").field("bytes"))]
    _both(engine, aggs)


def test_metrics_on_different_fields_at_one_level(engine):
    aggs = [AB.terms("hosts").field("host").size(12).subAggregation(AB.stats("rt").field("response_time_ms"))
            .subAggregation(AB.avg("b").field("bytes")).subAggregation(AB.extendedStats("rt_x").field("response_time_ms"))
            .subAggregation(AB.cardinality("ips").field("client_ip.hash").precisionThreshold(100)),
            AB.dateHistogram("d").field("@timestamp").interval("1d").subAggregation(AB.avg("s").field("status"))
            .subAggregation(AB.extendedStats("b").field("bytes"))]
    _both(engine, aggs, shards=2)


def test_sibling_bucket_sub_aggregations(engine):
    aggs = [AB.terms("hosts").field("host").size(5).subAggregation(
                AB.dateHistogram("h").field("@timestamp").interval("1d").subAggregation(AB.avg("rt").field("response_time_ms"))
                .subAggregation(AB.stats("b").field("bytes")))
            .subAggregation(AB.histogram("rt_h").field("response_time_ms").interval(100).subAggregation(AB.avg("s").field("status")))
            .subAggregation(AB.avg("all").field("bytes")),
            AB.dateHistogram("days").field("@timestamp").interval("1d").subAggregation(
                AB.terms("top").field("host").size(3).subAggregation(AB.avg("rt").field("response_time_ms")))
            .subAggregation(AB.terms("bottom").field("host").size(2).order(Order.count(True)))
            .subAggregation(AB.stats("rt").field("response_time_ms"))]
    _both(engine, aggs, shards=3)


@pytest.mark.parametrize("order", [Order.aggregation("rt.avg", False), Order.aggregation("a", True),
                                   Order.aggregation("x.max", False), Order.aggregation("x.std_upper", True),
                                   Order.aggregation("x.count", True), Order.aggregation("a.value", False)])
def test_terms_ordered_by_a_metric(engine, order):
    aggs = [AB.terms("hosts").field("host").size(6).order(order).subAggregation(AB.stats("rt").field("response_time_ms"))
            .subAggregation(AB.avg("a").field("bytes")).subAggregation(AB.extendedStats("x").field("response_time_ms"))
            .subAggregation(AB.dateHistogram("h").field("@timestamp").interval("1d"))]
    red = _both(engine, aggs, shards=3)
    assert red["hosts"]["doc_count_error_upper_bound"] == -1  # InternalTerms.doReduce: not a count-desc order


def test_terms_ordered_by_a_metric_min_doc_count_zero_and_nan(engine):
    """Zero-count terms (min_doc_count 0) have a NaN average: Comparators.compareDiscardNaN puts them last in both
    directions; the rt field is missing on 40 % of the docs."""
    n = 400_000
    rng = np.random.default_rng(3)
    cols = synthetic_columns(("host", "response_time_ms"), n)
    host = cols["host"]["values"].copy()
    host[host >= 900] = 5  # hosts 900..999 never occur
    cols["host"]["values"] = host
    cols["response_time_ms"]["present"] = bits_from_mask(rng.random(n) >= 0.4)
    for asc in (True, False):
        aggs = [AB.terms("hosts").field("host").size(1000).minDocCount(0).order(Order.aggregation("a", asc))
                .subAggregation(AB.avg("a").field("response_time_ms"))]
        want = O.run([(cols, n)], aggs)
        seg = engine.upload_segment(cols, n)
        plan = engine.plan(aggs)
        plan.collect(seg)
        res = plan.build()
        assert_same(res.to_dict(), want["shards"][0], "shard")
        assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")
        plan.close()
        seg.close()


def test_nested_terms_ordered_by_a_metric_under_a_histogram(engine):
    aggs = [AB.dateHistogram("days").field("@timestamp").interval("1d").subAggregation(
        AB.terms("hosts").field("host").size(4).order(Order.aggregation("rt.max", True))
        .subAggregation(AB.stats("rt").field("response_time_ms")))]
    _both(engine, aggs, shards=2)


def test_high_cardinality_terms_ordered_by_a_metric(engine):
    aggs = [AB.terms("urls").field("url").size(10).order(Order.aggregation("rt", False))
            .subAggregation(AB.avg("rt").field("response_time_ms"))]
    _both(engine, aggs, n=1_000_000, fields=("url", "response_time_ms"))


def test_inner_bucket_field_unmapped(engine):
    """terms{date_histogram(missing)} still counts the terms; histogram{terms(missing)} still counts the keys."""
    aggs = [AB.terms("hosts").field("host").size(5).subAggregation(
                AB.dateHistogram("h").field("no_such_date").interval("1h").subAggregation(AB.avg("rt").field("response_time_ms"))),
            AB.histogram("rt_h").field("response_time_ms").interval(250).subAggregation(
                AB.terms("t").field("no_such_keyword").subAggregation(AB.stats("b").field("bytes")))]
    _both(engine, aggs, fields=("host", "response_time_ms", "bytes"))


def test_inner_field_missing_in_one_segment(engine):
    """A later segment lacks the inner histogram's field: its docs count for the terms only."""
    n = 200_000
    a = synthetic_columns(("host", "@timestamp", "response_time_ms"), n)
    b = {"host": synthetic_columns(("host",), n, shard=1)["host"],
         "response_time_ms": synthetic_columns(("response_time_ms",), n, shard=1)["response_time_ms"]}
    aggs = [AB.terms("hosts").field("host").size(7).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("12h").subAggregation(AB.avg("rt").field("response_time_ms")))
        .subAggregation(AB.stats("rt").field("response_time_ms"))]
    one = {"host": dict(a["host"], values=np.concatenate([a["host"]["values"], b["host"]["values"]])),
           "response_time_ms": dict(a["response_time_ms"], values=np.concatenate([a["response_time_ms"]["values"],
                                                                                    b["response_time_ms"]["values"]])),
           "@timestamp": {"type": N.COL_I64, "values": np.concatenate([a["@timestamp"]["values"], np.zeros(n, np.int64)]),
                          "present": bits_from_mask(np.arange(2 * n) < n)}}
    want = O.run([(one, 2 * n)], aggs)
    segs = [engine.upload_segment(a, n), engine.upload_segment(b, n)]
    plan = engine.plan(aggs)
    for s in segs:
        plan.collect(s)
    assert_same(plan.build().to_dict(), want["shards"][0], "shard")
    plan.close()


def test_filter_aggregation_with_mixed_children(engine):
    aggs = [AB.filter("ok", QB.termQuery("status", 200)).subAggregation(
        AB.terms("hosts").field("host").size(4).subAggregation(AB.avg("rt").field("response_time_ms"))
        .subAggregation(AB.dateHistogram("d").field("@timestamp").interval("1d"))
        .order(Order.aggregation("rt", False))).subAggregation(AB.stats("b").field("bytes"))]
    _both(engine, aggs, shards=2, filters=[QB.rangeQuery("bytes").gte(512)])


def test_more_than_four_clauses(engine):
    """Six query clauses (bool.filter) plus three of a filter aggregation: more than the four a collect kernel evaluates
    itself, so each pipeline folds its clauses (and the accept bits) into one doc bitset first (set_preds); terms,
    histograms, metrics and a cardinality leaf all read that bitset."""
    q = [QB.rangeQuery("bytes").gte(100), QB.rangeQuery("bytes").lt(900_000), QB.rangeQuery("response_time_ms").gte(5),
         QB.rangeQuery("response_time_ms").lte(990), QB.rangeQuery("price").gt(1.0), QB.termQuery("status", 200)]
    aggs = [AB.terms("hosts").field("host").size(6).subAggregation(AB.stats("rt").field("response_time_ms"))
            .subAggregation(AB.cardinality("ips").field("client_ip.hash")),
            AB.filter("f", [QB.rangeQuery("bytes").gte(5000), QB.rangeQuery("response_time_ms").lt(500),
                            QB.rangeQuery("price").lt(400.0)])
            .subAggregation(AB.dateHistogram("d").field("@timestamp").interval("1d")
                            .subAggregation(AB.avg("b").field("bytes"))),
            AB.extendedStats("all").field("bytes")]
    red = _both(engine, aggs, shards=2, filters=q, exact=False)
    assert red["f"]["doc_count"] > 0


@pytest.mark.parametrize("asc,thr", [(False, 50), (True, 50), (False, 3000)])
def test_terms_ordered_by_cardinality(engine, asc, thr):
    """InternalOrder.Aggregation over a cardinality child (CardinalityAggregator.metric = counts.cardinality(bucketOrd)):
    shard selection by every ordinal's sketch estimate (LINEAR_COUNTING sizes at threshold 3000, HLL++ estimates at
    50), the reduce by the merged sketches' values; under a top-level filter too."""
    card = AB.cardinality("ips").field("client_ip.hash").precisionThreshold(thr)
    aggs = [AB.terms("hosts").field("host").size(6).order(Order.aggregation("ips", asc)).subAggregation(card)
            .subAggregation(AB.avg("rt").field("response_time_ms")),
            AB.filter("f", [QB.rangeQuery("bytes").gte(5000)]).subAggregation(
                AB.terms("h2").field("host").size(4).order(Order.aggregation("ips2.value", not asc))
                .subAggregation(AB.cardinality("ips2").field("client_ip.hash").precisionThreshold(thr)))]
    _both(engine, aggs, n=300_000, shards=2)


def test_terms_min_doc_count_0_under_empty_filter(engine):
    """Sub-aggregators are wrapped by asMultiBucketAggregator (AggregatorFactories.java:75): a filter that collected no
    doc in the shard never created its bucket-0 terms aggregator, so the shard's terms is first.buildEmptyAggregation()
    (AggregatorFactory.java:215-227) -- no zero-count terms even with min_doc_count 0 -- while a filter that matched
    lists every term; beside a histogram with min_doc_count 0 and extended bounds, and stats, under the empty one."""
    aggs = [AB.filter("none", QB.rangeQuery("bytes").lt(0))
            .subAggregation(AB.terms("t0").field("host").size(20).minDocCount(0)
                            .subAggregation(AB.avg("rt").field("response_time_ms")))
            .subAggregation(AB.histogram("h0").field("response_time_ms").interval(250).minDocCount(0).extendedBounds(0, 1000))
            .subAggregation(AB.stats("s0").field("bytes")),
            AB.filter("some", QB.termQuery("status", 200))
            .subAggregation(AB.terms("t1").field("host").size(20).minDocCount(0))]
    red = _both(engine, aggs, n=200_000, shards=2)
    assert red["none"]["doc_count"] == 0 and red["none"]["t0"]["buckets"] == []
    assert red["some"]["doc_count"] > 0 and len(red["some"]["t1"]["buckets"]) > 0


def test_filter_under_terms(engine):
    """FilterAggregator below the top level (A/bucket/filter/FilterAggregator.java:57-70): per term bucket the docs
    matching its clauses and its metric children over them; beside an unfiltered metric and a histogram child, and a
    filter with no children (doc_count only), under query clauses."""
    aggs = [AB.terms("hosts").field("host").size(7)
            .subAggregation(AB.filter("ok", QB.termQuery("status", 200))
                            .subAggregation(AB.avg("rt").field("response_time_ms"))
                            .subAggregation(AB.stats("b").field("bytes"))
                            .subAggregation(AB.cardinality("ips").field("client_ip.hash").precisionThreshold(100)))
            .subAggregation(AB.filter("big", [QB.rangeQuery("bytes").gte(500_000), QB.rangeQuery("price").lt(300.0)]))
            .subAggregation(AB.extendedStats("all_rt").field("response_time_ms"))
            .subAggregation(AB.dateHistogram("d").field("@timestamp").interval("1d"))]
    _both(engine, aggs, n=400_000, shards=2, filters=[QB.rangeQuery("response_time_ms").gte(3)])


@pytest.mark.parametrize("first", [True, False])
def test_filter_under_histogram(engine, first):
    """Filter children of a (date_)histogram, with min_doc_count 0 (empty buckets carry the filter's prototype); the
    filter as the first child (the outer counts then come from the histogram's own pipeline)."""
    f = AB.filter("slow", QB.rangeQuery("response_time_ms").gte(900)).subAggregation(AB.avg("b").field("bytes"))
    h = AB.histogram("rt").field("response_time_ms").interval(100).minDocCount(0).extendedBounds(-200, 1200)
    if first:
        h.subAggregation(f).subAggregation(AB.stats("p").field("price"))
    else:
        h.subAggregation(AB.stats("p").field("price")).subAggregation(f)
    aggs = [h, AB.dateHistogram("day").field("@timestamp").interval("1d").subAggregation(
        AB.filter("s200", QB.termQuery("status", 200)))]
    _both(engine, aggs, n=300_000, shards=2, exact=False)


def test_nested_filter_aggregations(engine):
    """Filter aggregations inside filter aggregations (FilterAggregator.java:57-70 at every level: a doc reaches the
    inner filter's sub-aggregations only if it matches every enclosing filter's clauses), three deep; a filter under a
    terms aggregation that is itself inside a filter; terms ordered by a cardinality child inside two filters; beside
    query clauses."""
    card = AB.cardinality("ips").field("client_ip.hash").precisionThreshold(200)
    aggs = [AB.filter("ok", QB.termQuery("status", 200))
            .subAggregation(AB.filter("big", QB.rangeQuery("bytes").gte(5000))
                            .subAggregation(AB.terms("hosts").field("host").size(5).subAggregation(AB.avg("rt").field("response_time_ms")))
                            .subAggregation(AB.filter("cheap", [QB.rangeQuery("price").lt(300.0), QB.rangeQuery("response_time_ms").lt(700)])
                                            .subAggregation(AB.stats("b").field("bytes"))
                                            .subAggregation(AB.dateHistogram("d").field("@timestamp").interval("1d")))
                            .subAggregation(AB.filter("empty", QB.rangeQuery("bytes").lt(0))))
            .subAggregation(AB.extendedStats("p").field("price")),
            AB.filter("any", QB.rangeQuery("response_time_ms").gte(10))
            .subAggregation(AB.terms("h2").field("host").size(4)
                            .subAggregation(AB.filter("slow", QB.rangeQuery("response_time_ms").gte(800))
                                            .subAggregation(AB.avg("b2").field("bytes"))))
            .subAggregation(AB.filter("f2", QB.rangeQuery("bytes").gte(1000))
                            .subAggregation(AB.terms("h3").field("host").size(3).order(Order.aggregation("ips", False))
                                            .subAggregation(card)))]
    red = _both(engine, aggs, n=300_000, shards=2, filters=[QB.rangeQuery("price").gte(2.0)], exact=False)
    assert red["ok"]["big"]["empty"]["doc_count"] == 0
    assert 0 < red["ok"]["big"]["cheap"]["doc_count"] < red["ok"]["big"]["doc_count"] < red["ok"]["doc_count"]


@pytest.mark.parametrize("asc", [False, True])
def test_terms_ordered_by_cardinality_below_the_top(engine, asc):
    """InternalOrder.Aggregation over a cardinality child of terms nested in another bucket aggregation: terms under a
    date_histogram, terms under terms, and the middle terms of terms{terms{date_histogram}} -- each candidate cell's
    sketch estimate (CardinalityAggregator.metric(bucketOrd)) from the sketches gathered beside the cells (refused
    before round 4)."""
    rng = np.random.default_rng(77)
    n = 250_000
    cols = {
        "g": {"type": N.COL_ORD_U32, "values": rng.integers(0, 3, size=n).astype(np.uint32), "terms": ["g0", "g1", "g2"]},
        "k": {"type": N.COL_ORD_U32, "values": np.minimum(rng.zipf(1.3, size=n) - 1, 59).astype(np.uint32),
              "terms": ["k%02d" % i for i in range(60)]},
        "ip": {"type": N.COL_I64, "values": (rng.integers(0, 400, size=n) * rng.integers(1, 5, size=n)).astype(np.int64)},
        "@timestamp": {"type": N.COL_I64, "values": np.sort(rng.integers(1441065600000, 1441065600000 + 3 * 86_400_000,
                                                                         size=n)).astype(np.int64)},
        "rt": {"type": N.COL_I64, "values": rng.integers(0, 1000, size=n).astype(np.int64)},
    }
    card = lambda nm: AB.cardinality(nm).field("ip").precisionThreshold(100)  # noqa: E731
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("1d").subAggregation(
                AB.terms("h").field("k").size(3).order(Order.aggregation("ips", asc)).subAggregation(card("ips"))),
            AB.terms("o").field("g").size(2).subAggregation(
                AB.terms("i").field("k").size(4).order(Order.aggregation("c2.value", asc)).subAggregation(card("c2"))
                .subAggregation(AB.avg("a").field("rt"))),
            AB.terms("t1").field("g").size(2).subAggregation(
                AB.terms("t2").field("k").size(3).order(Order.aggregation("c3", not asc)).subAggregation(card("c3"))
                .subAggregation(AB.dateHistogram("d3").field("@timestamp").interval("1d")))]
    lookups = {f: {t: i for i, t in enumerate(cols[f]["terms"])} for f in ("g", "k")}
    ord_lookup = lambda f, t: lookups.get(f, {}).get(t, -1)  # noqa: E731
    want = O.run([(cols, n)], aggs, ord_lookup=ord_lookup)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs, ord_lookup=ord_lookup)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")
    plan.close()
    seg.close()
