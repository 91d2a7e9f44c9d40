"""GPU parity over multi-valued doc values (SortedSetDocValues / SortedNumericDocValues as CSR columns), SURVEY §8(a)
a7 (every ordinal of a doc is a bucket), a11 (a doc's equal consecutive keys are collected once), a13/a14/a16 (count +=
valueCount, sums of the doc's local sum), a18 (every value hashed), a22 (a doc matches if any value matches).
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, QueryBuilders as QB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same

pytestmark = pytest.mark.gpu

T0 = 1441065600000


def csr_sorted(counts, values, dtype, type_, unique=False):
    """CSR column from per-doc value counts and a flat value array: values sorted within each doc (SortedNumeric /
    SortedSet order), duplicates within a doc dropped for SortedSet."""
    n = len(counts)
    doc = np.repeat(np.arange(n), counts)
    order = np.lexsort((values, doc))
    doc, values = doc[order], values[order]
    if unique and len(values):
        keep = np.ones(len(values), dtype=bool)
        keep[1:] = (doc[1:] != doc[:-1]) | (values[1:] != values[:-1])
        doc, values = doc[keep], values[keep]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(np.bincount(doc, minlength=n), out=offs[1:])
    return {"type": type_, "values": values.astype(dtype), "offsets": offs}


def segment(n, seed, lo=T0):
    rng = np.random.default_rng(seed)
    nt = 300
    tc = rng.integers(0, 5, size=n)
    base = np.sort(rng.integers(lo, lo + 10 * 86_400_000, size=n)).astype(np.int64)
    dc = rng.integers(0, 4, size=n)
    pc = rng.integers(0, 4, size=n)
    cc = rng.integers(0, 3, size=n)
    return {
        "tags": {**csr_sorted(tc, rng.integers(0, nt, size=tc.sum()), np.uint32, N.COL_ORD_U32, unique=True),
                 "terms": ["tag-%03d" % i for i in range(nt)]},
        "dates": csr_sorted(dc, np.repeat(base, dc) + rng.integers(0, 3 * 3_600_000, size=dc.sum()), np.int64, N.COL_I64),
        "prices": csr_sorted(pc, np.round(rng.random(pc.sum()) * 1000, 2), np.float64, N.COL_F64),
        "codes": csr_sorted(cc, rng.integers(0, 500, size=cc.sum()), np.int64, N.COL_I64),
        "@timestamp": {"type": N.COL_I64, "values": base},
        "host": {"type": N.COL_ORD_U32, "values": rng.integers(0, 40, size=n).astype(np.uint32),
                 "terms": ["host-%02d" % i for i in range(40)]},
        "response_time_ms": {"type": N.COL_I64, "values": rng.integers(0, 1000, size=n).astype(np.int64)},
    }


def check(engine, aggs, cols, n, filters=None, exact=False):
    lookup = {t: i for i, t in enumerate(cols["tags"]["terms"])}
    ord_lookup = lambda f, t: lookup.get(t, -1)  # noqa: E731
    want = O.run([(cols, n)], aggs, filters=filters, ord_lookup=ord_lookup)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs, filters=filters, ord_lookup=ord_lookup)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard", exact)
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced", exact)
    plan.close()
    seg.close()
    return want["reduced"]


N_DOCS = 400_000


def test_multi_valued_terms_and_metrics(engine):
    aggs = [AB.terms("tags").field("tags").size(25).subAggregation(AB.stats("p").field("prices")),
            AB.terms("tags_by_term").field("tags").size(10).order(Order.term(False))
            .subAggregation(AB.extendedStats("c").field("codes")),
            AB.extendedStats("all_prices").field("prices"),
            AB.avg("all_codes").field("codes")]
    check(engine, aggs, segment(N_DOCS, 1), N_DOCS)


def test_multi_valued_histograms(engine):
    aggs = [AB.dateHistogram("d").field("dates").interval("1d").subAggregation(AB.extendedStats("p").field("prices")),
            AB.histogram("codes").field("codes").interval(10).minDocCount(0).subAggregation(AB.avg("rt").field("response_time_ms")),
            AB.dateHistogram("m").field("dates").interval("month").timeZone("America/Chicago")]
    check(engine, aggs, segment(N_DOCS, 2), N_DOCS)


def test_multi_valued_nested(engine):
    aggs = [AB.terms("tags").field("tags").size(15).subAggregation(
                AB.dateHistogram("h").field("dates").interval("1h").subAggregation(AB.avg("rt").field("response_time_ms"))),
            AB.dateHistogram("d").field("@timestamp").interval("1d").subAggregation(
                AB.terms("tags").field("tags").size(5).subAggregation(AB.stats("p").field("prices"))),
            AB.terms("host").field("host").size(40).subAggregation(
                AB.dateHistogram("h").field("dates").interval("6h").subAggregation(AB.stats("c").field("codes")))]
    check(engine, aggs, segment(N_DOCS, 3), N_DOCS)


def test_multi_valued_filters(engine):
    """bool.filter over multi-valued fields (any value matches) feeding single- and multi-valued aggregations."""
    aggs = [AB.terms("host").field("host").size(10).subAggregation(AB.stats("rt").field("response_time_ms")),
            AB.dateHistogram("d").field("@timestamp").interval("1d"),
            AB.cardinality("tag_card").field("tags"),
            AB.cardinality("code_card").field("codes").precisionThreshold(100)]
    filters = [QB.rangeQuery("codes").gte(100).lt(300), QB.termQuery("tags", "tag-007")]
    check(engine, aggs, segment(N_DOCS, 4), N_DOCS, filters=filters)


@pytest.mark.parametrize("threshold", [50, 40000])
def test_multi_valued_cardinality(engine, threshold):
    aggs = [AB.cardinality("tags").field("tags").precisionThreshold(threshold),
            AB.cardinality("codes").field("codes").precisionThreshold(threshold),
            AB.cardinality("prices").field("prices").precisionThreshold(threshold)]
    check(engine, aggs, segment(N_DOCS, 5), N_DOCS)


def test_multi_valued_accept_bits_and_global_ordinals(engine):
    """Two multi-valued keyword segments with different dictionaries under one ordinal map, plus an accept bitset."""
    a, b = segment(150_000, 6), segment(120_000, 7)
    b["tags"]["terms"] = ["tag-%03d" % (i + 100) for i in range(300)]  # overlapping, shifted dictionary
    rng = np.random.default_rng(8)
    acc = [rng.random(150_000) < 0.7, rng.random(120_000) < 0.7]
    from helpers import bits_from_mask
    gdict = sorted(set(a["tags"]["terms"]) | set(b["tags"]["terms"]))
    gi = {t: i for i, t in enumerate(gdict)}
    # the oracle sees one segment with the merged dictionary over the concatenated docs
    tag_cols, price_cols = [], []
    for sc in (a, b):
        remap = np.array([gi[t] for t in sc["tags"]["terms"]], dtype=np.uint32)
        counts = np.diff(sc["tags"]["offsets"].astype(np.int64))
        tag_cols.append((counts, remap[sc["tags"]["values"]]))
        price_cols.append((np.diff(sc["prices"]["offsets"].astype(np.int64)), sc["prices"]["values"]))
    one = {"tags": {**csr_sorted(np.concatenate([c for c, _ in tag_cols]), np.concatenate([v for _, v in tag_cols]),
                                 np.uint32, N.COL_ORD_U32, unique=True), "terms": gdict},
           "prices": csr_sorted(np.concatenate([c for c, _ in price_cols]), np.concatenate([v for _, v in price_cols]),
                                np.float64, N.COL_F64)}
    aggs = [AB.terms("tags").field("tags").size(30).subAggregation(AB.avg("p").field("prices"))]
    want = O.run([(one, 270_000)], aggs, accept=[bits_from_mask(np.concatenate(acc))])
    segs = [engine.upload_segment({k: a[k] for k in ("tags", "prices")}, 150_000),
            engine.upload_segment({k: b[k] for k in ("tags", "prices")}, 120_000)]
    omap = engine.ordinal_map(segs, "tags")
    plan = engine.plan(aggs)
    for sg, m in zip(segs, acc):
        plan.collect(sg, accept_bits=bits_from_mask(m))
    assert_same(plan.build().to_dict(), want["shards"][0], "shard", False)
    plan.close()
    omap.close()
    for sg in segs:
        sg.close()


def test_multi_valued_double_histogram(engine):
    aggs = [AB.histogram("p").field("prices").interval(50).subAggregation(AB.avg("c").field("codes")),
            AB.terms("tags").field("tags").size(5).subAggregation(AB.histogram("p").field("prices").interval(250))]
    check(engine, aggs, segment(N_DOCS, 12), N_DOCS)


def test_multi_valued_keyword_range(engine):  # a doc matches if any of its terms is in the range
    aggs = [AB.terms("host").field("host").size(10), AB.cardinality("c").field("codes")]
    check(engine, aggs, segment(N_DOCS, 13), N_DOCS, filters=[QB.rangeQuery("tags").gte("tag-050").lt("tag-060")])


def test_filter_aggregation_over_multi_valued_fields(engine):  # FilterAggregator on CSR columns (a doc matches if any value does)
    cols = segment(N_DOCS, 11)
    aggs = [AB.filter("tagged", [QB.termQuery("tags", "tag-007"), QB.rangeQuery("codes").gte(100).lt(300)])
            .subAggregation(AB.terms("tags").field("tags").size(10).subAggregation(AB.avg("p").field("prices")))
            .subAggregation(AB.dateHistogram("d").field("dates").interval("1d"))
            .subAggregation(AB.cardinality("c").field("codes").precisionThreshold(200)),
            AB.stats("all_prices").field("prices")]
    got = check(engine, aggs, cols, N_DOCS, filters=[QB.rangeQuery("response_time_ms").lt(700)])
    assert got["tagged"]["doc_count"] > 0


def test_multi_valued_terms_under_terms(engine):
    """terms under terms with a multi-valued outer or inner keyword field (the CSR kernel with the inner field's
    ordinals as the key dimension): every (outer ordinal, inner ordinal) pair of a doc is one cell."""
    aggs = [AB.terms("tags").field("tags").size(8).subAggregation(
                AB.terms("hosts").field("host").size(5).subAggregation(AB.stats("rt").field("response_time_ms"))),
            AB.terms("hosts").field("host").size(6).order(Order.term(True)).subAggregation(
                AB.terms("tags").field("tags").size(4).order(Order.count(True))),
            AB.terms("pairs").field("tags").size(5).subAggregation(AB.terms("co").field("tags").size(3).minDocCount(0))]
    check(engine, aggs, segment(N_DOCS, 11), N_DOCS, exact=True)
    check(engine, aggs[:1], segment(N_DOCS, 12), N_DOCS, filters=[QB.rangeQuery("codes").gte(100).lte(300)], exact=True)
