"""Terms under terms beyond the dense grid, collected breadth-first: the outer terms' doc counts while collecting, then at
build the inner terms replayed over the retained segments for the surviving outer buckets only (TermsAggregator's
breadth_first mode: A/bucket/terms/TermsAggregator.java:161 shouldDefer, A/bucket/BestBucketsDeferringCollector.java
:127-166 prepareSelectedBuckets, replayed from GlobalOrdinalsStringTermsAggregator.buildAggregation :195-196).  The
reference's results do not depend on the collect mode, so every case is compared with the oracle's depth-first
restatement.  ESGPU_DEFER_CELLS forces the replay on small grids; the real case is 1,000 hosts x 10M urls (10^10
cells, refused before this path existed)."""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, QueryBuilders as QB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same, bits_from_mask, synthetic_columns

pytestmark = pytest.mark.gpu


def _segment(seed, n, t_a=300, t_b=2000, uniform_b=False):
    rng = np.random.default_rng(seed)
    a = ((np.minimum(rng.zipf(1.3, size=n) - 1, t_a - 1) * 7919 + 13) % t_a).astype(np.uint32)
    a[rng.random(n) < 0.03] = 0xFFFFFFFF
    b = ((np.minimum(rng.zipf(1.1, size=n) - 1, t_b - 1) * 104729 + 7) % t_b).astype(np.uint32)
    if uniform_b:
        b = rng.integers(0, t_b, size=n).astype(np.uint32)
    b[rng.random(n) < 0.05] = 0xFFFFFFFF
    num = rng.integers(0, 1000, size=n).astype(np.int64)
    present = rng.random(n) >= 0.1
    return {
        "a": {"type": N.COL_ORD_U32, "values": a, "terms": ["a%04d" % i for i in range(t_a)]},
        "b": {"type": N.COL_ORD_U32, "values": b, "terms": ["b%06d" % i for i in range(t_b)]},
        "num": {"type": N.COL_I64, "values": np.where(present, num, 0), "present": bits_from_mask(present)},
        "status": {"type": N.COL_I64, "values": rng.choice([200, 304, 404, 500], size=n).astype(np.int64)},
    }


def _concat(segs):
    """one shard's segments as one column set for the oracle (the reference's results do not depend on the split)"""
    out = {}
    for f, c in segs[0].items():
        out[f] = dict(c, values=np.concatenate([s[f]["values"] for s in segs]))
        if "present" in c:
            n0 = [len(s[f]["values"]) for s in segs]
            mask = np.concatenate([np.unpackbits(s[f]["present"].view(np.uint8), bitorder="little")[:k] > 0
                                   for s, k in zip(segs, n0)])
            out[f]["present"] = bits_from_mask(mask)
    return out


def _run(engine, aggs, segs_per_shard=1, shards=2, n=120_000, t_b=2000, filters=None, deletes=0.0, close_early=False,
         replayed=True, uniform_b=False):
    cols = [[_segment(70 + 10 * s + j, n, t_b=t_b, uniform_b=uniform_b) for j in range(segs_per_shard)]
            for s in range(shards)]
    masks = [[np.random.default_rng(900 + 10 * s + j).random(n) >= deletes for j in range(segs_per_shard)]
             for s in range(shards)]
    lookups = {f: {t: i for i, t in enumerate(cols[0][0][f]["terms"])} for f in ("a", "b")}
    ord_lookup = lambda f, t: lookups.get(f, {}).get(t, -1)  # noqa: E731
    accept = [bits_from_mask(np.concatenate(masks[s])) for s in range(shards)] if deletes > 0 else None
    want = O.run([(_concat(cols[s]), n * segs_per_shard) for s in range(shards)], aggs, filters=filters, accept=accept,
                 ord_lookup=ord_lookup, number_of_shards=shards, streams=True)
    plan = engine.plan(aggs, filters=filters, ord_lookup=ord_lookup, number_of_shards=shards)
    results = []
    for s in range(shards):
        plan.reset()
        segs = [engine.upload_segment(cols[s][j], n) for j in range(segs_per_shard)]
        for j, seg in enumerate(segs):
            plan.collect(seg, accept_bits=bits_from_mask(masks[s][j]) if deletes > 0 else None)
        assert plan.deferred_segments() == (segs_per_shard if replayed else 0)
        if close_early:  # the plan keeps the segments it replays (their destroy carried out at its reset)
            for seg in segs:
                seg.close()
        r = plan.build()
        assert_same(r.to_dict(), want["shards"][s], f"shard{s}")
        assert r.to_stream() == want["streams"][s], f"shard{s} transport bytes"
        results.append(r)
        if not close_early:
            for seg in segs:
                seg.close()
    assert_same(reduce(results).to_dict(), want["reduced"], "reduced")
    plan.close()
    return results


@pytest.fixture
def forced(monkeypatch):
    monkeypatch.setenv("ESGPU_DEFER_CELLS", "1000")


@pytest.mark.parametrize("order", ["count", "count_asc", "term", "term_desc", "agg"])
def test_replayed_inner_terms_orders(engine, forced, order):
    inner = AB.terms("B").field("b").size(4).subAggregation(AB.avg("n").field("num")).subAggregation(
        AB.stats("s").field("num"))
    if order == "count_asc":
        inner.order(Order.count(True))
    elif order == "term":
        inner.order(Order.term(True))
    elif order == "term_desc":
        inner.order(Order.term(False))
    elif order == "agg":
        inner.order(Order.aggregation("s.max", True))
    aggs = [AB.terms("A").field("a").size(6).subAggregation(inner).subAggregation(AB.avg("na").field("num"))]
    _run(engine, aggs)


def test_replayed_min_doc_count_zero_and_outer_metric_order(engine, forced):
    aggs = [AB.terms("A").field("a").size(5).order(Order.aggregation("x", False)).subAggregation(
        AB.avg("x").field("num")).subAggregation(
        AB.terms("B").field("b").size(3).minDocCount(0).order(Order.count(True)))]
    _run(engine, aggs, t_b=40)


def test_replayed_with_query_filter_and_live_docs(engine, forced):
    aggs = [AB.terms("A").field("a").size(4).subAggregation(
        AB.terms("B").field("b").size(5).subAggregation(AB.extendedStats("x").field("num")))]
    _run(engine, aggs, filters=[QB.termQuery("status", 200)], deletes=0.02)


def test_replayed_under_top_level_filter(engine, forced):
    aggs = [AB.filter("f", QB.rangeQuery("num").gte(100).lt(800)).subAggregation(
        AB.terms("A").field("a").size(4).subAggregation(AB.terms("B").field("b").size(3)))]
    _run(engine, aggs)


def test_replayed_over_two_segments_closed_before_build(engine, forced):
    """a shard of two segments; the caller destroys them after collecting and the replay still reads them"""
    aggs = [AB.terms("A").field("a").size(5).subAggregation(AB.terms("B").field("b").size(4).subAggregation(
        AB.avg("n").field("num")))]
    _run(engine, aggs, segs_per_shard=2, shards=1, close_early=True)


def test_replayed_gpu_topk_rows(engine, forced):
    """inner rows over 65,536 terms: each winner's inner terms picked by the GPU top-k (count and term orders)"""
    for order, metric in ((Order.count(False), False), (Order.term(True), True), (Order.count(True), False)):
        inner = AB.terms("B").field("b").size(5).order(order)
        if metric:  # leaves: the generic grid (u64 counts); none: the partitioned counting path (u32 counts)
            inner.subAggregation(AB.stats("s").field("num"))
        _run(engine, [AB.terms("A").field("a").size(3).subAggregation(inner)], t_b=100_000, n=200_000, shards=1)


def test_dense_grid_when_within_budget(engine):
    """the same shape under the default budget: the dense [outer x inner] grid, nothing retained"""
    aggs = [AB.terms("A").field("a").size(6).subAggregation(AB.terms("B").field("b").size(4))]
    _run(engine, aggs, replayed=False)


def test_hosts_by_urls_10m(engine):
    """terms(host){terms(url)}: 1,000 x 10M ordinals, over the 2^31-cell dense budget -- replayed, no forcing.  A keyword
    range query keeps the oracle's per-bucket inner aggregators (10M counters each, as the reference's) to 12 hosts"""
    n = 4_000_000
    fields = ("host", "url")
    aggs = [AB.terms("hosts").field("host").size(5).subAggregation(AB.terms("urls").field("url").size(3))]
    filters = [QB.rangeQuery("host").gte("host-0000").lt("host-0012")]
    want = O.run([(synthetic_columns(fields, n), n)], aggs, filters=filters, number_of_shards=1)
    seg = engine.synthetic_segment(n, fields=fields)
    plan = engine.plan(aggs, filters=filters)
    plan.collect(seg)
    assert plan.deferred_segments() == 1
    got = plan.build().to_dict()
    assert_same(got, want["shards"][0], "shard")
    assert got["hosts"]["buckets"][0]["urls"]["buckets"]
    plan.close()
    seg.close()


@pytest.mark.parametrize("batch", ["2", "3"])
@pytest.mark.parametrize("order", ["count", "term", "count_asc"])
def test_replayed_batches_compacted(engine, forced, monkeypatch, order, batch):
    """Count-only inner terms over 100,000 ordinals replayed in batches of 2 or 3 winners (ESGPU_REPLAY_BATCH; 17
    winners: 9 batches take the compaction's scattered appends, 6 its per-block sort by batch in LDS): the winners' docs
    are compacted once per retained segment into per-batch regions -- under a query filter and live docs, over two
    segments -- and each batch is counted from its region (ReplayCompactParams)."""
    monkeypatch.setenv("ESGPU_REPLAY_BATCH", batch)
    inner = AB.terms("B").field("b").size(4)
    inner.order(Order.count(False) if order == "count" else Order.term(True) if order == "term" else Order.count(True))
    aggs = [AB.terms("A").field("a").size(5).subAggregation(inner)]
    _run(engine, aggs, t_b=100_000, n=150_000, shards=1, segs_per_shard=2, filters=[QB.termQuery("status", 200)],
         deletes=0.03)


@pytest.mark.parametrize("order", ["count", "term", "count_asc"])
def test_replayed_inner_shard_size_over_1024(engine, forced, order):
    """An inner shard_size above the GPU top-k's final sort (1,100 of 100,000 inner terms): count orders take the GPU's
    threshold candidates and sort them on the host, term orders select from the fetched rows (refused before round 4)."""
    inner = AB.terms("B").field("b").size(1100)
    inner.order(Order.count(False) if order == "count" else Order.term(True) if order == "term" else Order.count(True))
    aggs = [AB.terms("A").field("a").size(3).subAggregation(inner)]
    _run(engine, aggs, t_b=100_000, n=200_000, shards=1)


@pytest.mark.parametrize("size,min_doc", [(3, 1), (10, 1), (60, 1), (5, 40)])
def test_replayed_over_hot_inner_terms(engine, forced, size, min_doc):
    """A count-ordered, count-only inner terms over 150,000 Zipf ordinals in one retained segment (the forced replay at
    its real shape): each winner's inner terms come from one pass over the inner field's hot slots whenever its k-th
    count is above every colder term's count in the segment (replay_hot), else from the full replay -- under a query
    filter and live docs, with inner min_doc_count, against the oracle."""
    inner = AB.terms("B").field("b").size(size).minDocCount(min_doc)
    aggs = [AB.terms("A").field("a").size(4).subAggregation(inner)]
    _run(engine, aggs, t_b=150_000, n=300_000, shards=2)
    _run(engine, aggs, t_b=150_000, n=300_000, shards=1, filters=[QB.termQuery("status", 200)], deletes=0.05)


def test_replayed_hot_inner_terms_unsettled(engine, forced):
    """Uniform inner terms: the hot slots do not settle the winners' inner top-k (their counts tie with colder terms),
    so the full replay runs -- the same result."""
    aggs = [AB.terms("A").field("a").size(3).subAggregation(AB.terms("B").field("b").size(4))]
    _run(engine, aggs, t_b=120_000, n=250_000, shards=1, uniform_b=True)
