"""GPU parity of the hot/cold partitioned terms counting (esgpu_hotcold.hip) against the oracle.

valueCount > 65536 ordinals takes the high-cardinality path (GlobalOrdinalsStringTermsAggregator.java:107-135 with a
LongArray of valueCount counters): the segment's statistics (hot set, partition capacities) are built on the first
request and reused.  Each case stresses one part of that design: ordinals clustered by doc id (every workgroup's
share of a partition is far from its static region: overflow chunks), a flat distribution (no hot table), a cold
ordinal with more than 65535 docs (32-bit counters in the counting pass), filters and accept bitsets (requests that
use a fraction of the capacities), several segments into one plan, and reuse of the statistics across requests.
Requests without predicates or accept bits take the postings form (path 7: hot slots from the recoded column, the cold
docs counted from the segment's partition-ordered cold lists); the others scatter the cold docs per request (path 6).
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, QueryBuilders as QB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same, bits_from_mask

pytestmark = pytest.mark.gpu

def _cols(ords, T, rng):
    n = len(ords)
    return {"kw": {"type": N.COL_ORD_U32, "values": ords.astype(np.uint32), "terms": ["u%07d" % i for i in range(T)]},
            "status": {"type": N.COL_I64, "values": rng.integers(0, 4, size=n).astype(np.int64)}}


def _check(engine, cols, n, aggs, filters=None, accept=None, reps=1, path_want=None):
    want = O.run([(cols, n)], aggs, filters=filters, accept=[accept] if accept is not None else None)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs, filters=filters)
    for rep in range(reps):  # the second request reuses the segment statistics built by the first
        plan.collect(seg, accept_bits=accept)
        _, _, path = plan.last_collect_stats()
        assert path == (path_want or (7 if not filters and accept is None else 6)), path
        res = plan.build()
        assert_same(res.to_dict(), want["shards"][0], f"shard rep{rep}")
        assert_same(reduce([res]).to_dict(), want["reduced"], f"reduced rep{rep}")
        plan.reset()
    plan.close()
    seg.close()


def test_zipf_terms_orders_reused_stats(engine):
    """Zipf(1.1) over 300,000 ordinals (hot table on), every terms order, two requests over one segment."""
    rng = np.random.default_rng(101)
    n, T = 2_000_000, 300_000
    ranks = np.minimum(rng.zipf(1.1, size=n) - 1, T - 1)
    ords = (ranks * 7919 + 17) % T
    ords[rng.random(n) < 0.02] = 0xFFFFFFFF
    cols = _cols(ords, T, rng)
    aggs = [AB.terms("c").field("kw").size(20),
            AB.terms("a").field("kw").size(9).order(Order.count(True)),
            AB.terms("t").field("kw").size(11).order(Order.term(False)).minDocCount(0)]
    _check(engine, cols, n, aggs, reps=2)


def test_clustered_ordinals_overflow(engine):
    """Ordinals sorted by doc id: each partition's docs sit in a few workgroups' ranges, so almost every append goes
    through overflow chunks; a term range filter keeps about half of them."""
    rng = np.random.default_rng(102)
    n, T = 3_000_000, 250_000
    ords = np.sort(rng.integers(0, T, size=n))
    ords[rng.random(n) < 0.01] = 0xFFFFFFFF
    cols = _cols(ords, T, rng)
    aggs = [AB.terms("c").field("kw").size(30), AB.terms("t").field("kw").size(5).order(Order.term(True))]
    _check(engine, cols, n, aggs)
    _check(engine, cols, n, aggs, filters=[QB.rangeQuery("status").gte(2)])


def test_flat_distribution_accept_bits(engine):
    """Uniform over 200,000 ordinals with an accept bitset (the top 16,384 hold ~15 % of the docs: a hot set)."""
    rng = np.random.default_rng(103)
    n, T = 1_500_000, 200_000
    ords = rng.integers(0, T, size=n)
    cols = _cols(ords, T, rng)
    accept = rng.random(n) < 0.7
    _check(engine, cols, n, [AB.terms("c").field("kw").size(40)], accept=bits_from_mask(accept))


def test_cold_ordinal_over_16_bits(engine):
    """4M ordinals, one doc each on average, plus one ordinal with 70,000 docs: the 16,384 most frequent hold under
    5 % of the docs, so there is no hot set and the heavy ordinal is cold -- the counting pass keeps 32-bit counters and
    splits the heavy partition over several workgroups."""
    rng = np.random.default_rng(104)
    T = 4_000_000
    n = 4_000_000
    ords = rng.integers(0, T, size=n)
    ords[rng.choice(n, size=70_000, replace=False)] = 777
    cols = _cols(ords, T, rng)
    _check(engine, cols, n, [AB.terms("c").field("kw").size(10)], filters=[QB.rangeQuery("status").lte(2)])
    _check(engine, cols, n, [AB.terms("c").field("kw").size(10)], reps=2)


@pytest.mark.parametrize("filtered", [True, False])
def test_two_segments_one_plan(engine, filtered):
    """Two segments with their own statistics counted into one plan (same dictionary, no ordinal map); unfiltered, the
    second segment's cold lists add to the first's counts."""
    rng = np.random.default_rng(105)
    T = 180_000
    sizes = [700_001, 1_100_000]
    parts = []
    for k, n in enumerate(sizes):
        ranks = np.minimum(rng.zipf(1.05 + 0.2 * k, size=n) - 1, T - 1)
        parts.append(((ranks * 104729 + 11 * k) % T).astype(np.uint32))
    cols = [_cols(o, T, rng) for o in parts]
    allc = {"kw": dict(cols[0]["kw"], values=np.concatenate(parts)),
            "status": {"type": N.COL_I64, "values": np.concatenate([c["status"]["values"] for c in cols])}}
    aggs = [AB.terms("c").field("kw").size(25), AB.terms("t").field("kw").size(6).order(Order.term(False))]
    flt = [QB.rangeQuery("status").gte(1)] if filtered else None
    want = O.run([(allc, sum(sizes))], aggs, filters=flt)
    segs = [engine.upload_segment(c, n) for c, n in zip(cols, sizes)]
    plan = engine.plan(aggs, filters=flt)
    for s in segs:
        plan.collect(s)
        assert plan.last_collect_stats()[2] == (6 if filtered else 7)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    plan.close()
    for s in segs:
        s.close()


def test_capacity_overrun_in_first_segment_is_reported(engine, monkeypatch):
    """A partition overrun in segment 1 of a two-segment plan must survive segment 2's collect and fail the request
    with ESGPU_ERR_DEVICE (the flag accumulates over the request's segments and is cleared after each check).  The test
    knob ESGPU_DEBUG_HC_NO_OVERFLOW removes the overflow pools while a segment's statistics are built, so clustered
    ordinals (each partition's docs in a few workgroups' ranges) overrun their static regions; the evenly spread second
    segment does not.  The same plan then serves a clean request."""
    rng = np.random.default_rng(106)
    T = 150_000
    clustered = np.sort(rng.integers(0, T, size=2_000_000)).astype(np.uint32)
    spread = rng.integers(0, T, size=1_000_000).astype(np.uint32)
    c1, c2 = _cols(clustered, T, rng), _cols(spread, T, rng)
    aggs = [AB.terms("c").field("kw").size(10)]
    flt = [QB.rangeQuery("status").gte(0)]  # predicates: the scatter form (path 6), which allocates overflow chunks
    monkeypatch.setenv("ESGPU_DEBUG_HC_NO_OVERFLOW", "1")
    s1 = engine.upload_segment(c1, len(clustered))
    s2 = engine.upload_segment(c2, len(spread))
    plan = engine.plan(aggs, filters=flt)
    try:
        plan.collect(s1)
        monkeypatch.delenv("ESGPU_DEBUG_HC_NO_OVERFLOW")
        plan.collect(s2)
        with pytest.raises(N.EsGpuError) as ei:
            plan.build()
        assert ei.value.code == N.ERR_DEVICE, ei.value
        plan.reset()
        plan.collect(s2)  # the error word was cleared by the check
        want = O.run([(c2, len(spread))], aggs, filters=flt)
        assert_same(plan.build().to_dict(), want["shards"][0], "clean request")
    finally:
        plan.close()
        s1.close()
        s2.close()


def test_live_docs_few_deletions_postings(engine):
    """A live-docs bitset clearing ~2 % of the docs keeps the postings form (path 7): the hot pass tests the accept
    bits, the cold lists count every doc and the dead cold docs are taken back out (hc_cold_sub_kernel); two requests
    over one segment, every terms order."""
    rng = np.random.default_rng(106)
    n, T = 2_000_000, 300_000
    ranks = np.minimum(rng.zipf(1.1, size=n) - 1, T - 1)
    ords = (ranks * 7919 + 17) % T
    ords[rng.random(n) < 0.02] = 0xFFFFFFFF
    cols = _cols(ords, T, rng)
    accept = bits_from_mask(rng.random(n) >= 0.02)
    aggs = [AB.terms("c").field("kw").size(20),
            AB.terms("a").field("kw").size(9).order(Order.count(True)),
            AB.terms("t").field("kw").size(11).order(Order.term(False)).minDocCount(0)]
    _check(engine, cols, n, aggs, accept=accept, reps=2, path_want=7)


def test_live_docs_two_segments_postings(engine):
    """Two segments, each with its own live docs (3 % and 1 % deleted), counted into one plan on the postings form:
    the second segment's cold lists add to the first's counts and each subtracts its own dead cold docs."""
    rng = np.random.default_rng(107)
    T = 180_000
    sizes = [900_000, 1_300_000]
    parts, masks = [], []
    for k, n in enumerate(sizes):
        ranks = np.minimum(rng.zipf(1.1, size=n) - 1, T - 1)
        parts.append(((ranks * 104729 + 7 * k) % T).astype(np.uint32))
        masks.append(rng.random(n) >= (0.03, 0.01)[k])
    cols = [_cols(o, T, rng) for o in parts]
    allc = {"kw": dict(cols[0]["kw"], values=np.concatenate(parts)),
            "status": {"type": N.COL_I64, "values": np.concatenate([c["status"]["values"] for c in cols])}}
    aggs = [AB.terms("c").field("kw").size(25)]
    want = O.run([(allc, sum(sizes))], aggs, accept=[bits_from_mask(np.concatenate(masks))])
    segs = [engine.upload_segment(c, n) for c, n in zip(cols, sizes)]
    plan = engine.plan(aggs)
    for seg, m in zip(segs, masks):
        plan.collect(seg, accept_bits=bits_from_mask(m))
        assert plan.last_collect_stats()[2] == 7
    assert_same(plan.build().to_dict(), want["shards"][0], "shard")
    plan.close()
    for seg in segs:
        seg.close()
