"""GPU parity of the hot/cold partitioned terms counting (esgpu_hotcold.hip) against the oracle.

valueCount > 65536 ordinals takes the high-cardinality path (GlobalOrdinalsStringTermsAggregator.java:107-135 with a
LongArray of valueCount counters): the segment's statistics (hot set, partition capacities) are built on the first
request and reused.  Each case stresses one part of that design: ordinals clustered by doc id (every workgroup's
share of a partition is far from its static region: overflow chunks), a flat distribution (no hot table), a cold
ordinal with more than 65535 docs (32-bit counters in the counting pass), filters and accept bitsets (requests that
use a fraction of the capacities), several segments into one plan, and reuse of the statistics across requests.
Requests without predicates or accept bits take the postings form (path 7: hot slots from the recoded column, the cold
docs counted from the segment's partition-ordered cold lists); the others scatter the cold docs per request (path 6).
A lone terms aggregation in count order over one segment defers the cold lists to its top-k (path 8), which counts
them only when the hot slots' k-th count does not exceed the segment's largest cold count; filtered (query clauses or
accept bits) it counts the hot slots and one total of the passing cold docs from the hot-slot column (path 9) and
scatters the cold docs only when the top-k needs them.
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
        # (7 or 8 unfiltered: a lone count-ordered terms aggregation defers the cold lists to its top-k)
        # (a lone count-ordered terms aggregation filtered: 9, the hot slots from the hot-slot column first)
        assert path in ((path_want,) if path_want else (7, 8) if not filters and accept is None else (6, 9)), path
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
    for k, (seg, m) in enumerate(zip(segs, masks)):
        plan.collect(seg, accept_bits=bits_from_mask(m))
        # (the first segment defers to the top-k, path 9; the second segment's collect counts it first)
        assert plan.last_collect_stats()[2] == (9 if k == 0 else 7)
    assert_same(plan.build().to_dict(), want["shards"][0], "shard")
    plan.close()
    for seg in segs:
        seg.close()


def _csr(counts, values):
    offs = np.zeros(len(counts) + 1, dtype=np.uint64)
    np.cumsum(counts, out=offs[1:])
    return values, offs


@pytest.mark.parametrize("multi_field", ["kw", "status"])
@pytest.mark.parametrize("multi_first", [False, True])
def test_count_width_across_single_and_multi_segments(engine, multi_field, multi_first):
    """One request over two segments of a 200,000-term field, the terms field (or the filter field) multi-valued in only
    one of them: the single-valued segment counts into u32 counters (hot/cold path), the multi-valued one through the
    CSR kernel's u64 atomics, so the grid's count width changes between the two collects -- in both orders."""
    rng = np.random.default_rng(108 + multi_first)
    T = 200_000
    n1, n2 = 800_000, 600_000
    # single-valued segment
    ranks = np.minimum(rng.zipf(1.1, size=n1) - 1, T - 1)
    o1 = ((ranks * 7919 + 5) % T).astype(np.uint32)
    o1[rng.random(n1) < 0.02] = 0xFFFFFFFF
    st1 = rng.integers(0, 4, size=n1).astype(np.int64)
    terms = ["u%07d" % i for i in range(T)]
    single = {"kw": {"type": N.COL_ORD_U32, "values": o1, "terms": terms},
              "status": {"type": N.COL_I64, "values": st1}}
    # the other segment: `multi_field` multi-valued (CSR, values sorted and unique per doc for the keyword field)
    if multi_field == "kw":
        cnt = rng.integers(0, 4, size=n2)
        vals = np.minimum(rng.zipf(1.1, size=int(cnt.sum())) - 1, T - 1)
        vals = ((vals * 7919 + 5) % T).astype(np.uint32)
        doc = np.repeat(np.arange(n2), cnt)
        order = np.lexsort((vals, doc))
        doc, vals = doc[order], vals[order]
        keep = np.ones(len(vals), dtype=bool)
        keep[1:] = (doc[1:] != doc[:-1]) | (vals[1:] != vals[:-1])
        doc, vals = doc[keep], vals[keep]
        cnt = np.bincount(doc, minlength=n2)
        v, offs = _csr(cnt, vals)
        other = {"kw": {"type": N.COL_ORD_U32, "values": v, "offsets": offs, "terms": terms},
                 "status": {"type": N.COL_I64, "values": rng.integers(0, 4, size=n2).astype(np.int64)}}
        # the whole shard in CSR form for the oracle: the single-valued docs have 0 or 1 value
        c1 = (o1 != 0xFFFFFFFF).astype(np.int64)
        v1 = o1[o1 != 0xFFFFFFFF]
        seqs = [(c1, v1), (cnt, v)] if not multi_first else [(cnt, v), (c1, v1)]
        allv, alloffs = _csr(np.concatenate([s[0] for s in seqs]), np.concatenate([s[1] for s in seqs]))
        st = [st1, other["status"]["values"]] if not multi_first else [other["status"]["values"], st1]
        allc = {"kw": {"type": N.COL_ORD_U32, "values": allv, "offsets": alloffs, "terms": terms},
                "status": {"type": N.COL_I64, "values": np.concatenate(st)}}
    else:
        ranks2 = np.minimum(rng.zipf(1.1, size=n2) - 1, T - 1)
        o2 = ((ranks2 * 7919 + 5) % T).astype(np.uint32)
        cnt = rng.integers(0, 3, size=n2)
        sv = np.sort(rng.integers(0, 4, size=(n2, 2)), axis=1)
        # values of doc d: the first cnt[d] of its two sorted draws (SortedNumeric order)
        vals = sv[np.arange(2)[None, :] < cnt[:, None]].astype(np.int64)
        v, offs = _csr(cnt, vals)
        other = {"kw": {"type": N.COL_ORD_U32, "values": o2, "terms": terms},
                 "status": {"type": N.COL_I64, "values": v, "offsets": offs}}
        parts = [(o1, np.ones(n1, dtype=np.int64), st1), (o2, cnt, vals)]
        if multi_first:
            parts = parts[::-1]
        allv, alloffs = _csr(np.concatenate([p[1] for p in parts]), np.concatenate([p[2] for p in parts]))
        allc = {"kw": {"type": N.COL_ORD_U32, "values": np.concatenate([p[0] for p in parts]), "terms": terms},
                "status": {"type": N.COL_I64, "values": allv, "offsets": alloffs}}
    aggs = [AB.terms("c").field("kw").size(25), AB.terms("t").field("kw").size(7).order(Order.term(False))]
    flt = [QB.rangeQuery("status").gte(1)] if multi_field == "status" else None
    want = O.run([(allc, n1 + n2)], aggs, filters=flt)
    segs = [engine.upload_segment(single, n1), engine.upload_segment(other, n2)]
    if multi_first:
        segs = segs[::-1]
    plan = engine.plan(aggs, filters=flt)
    try:
        for rep in range(2):  # the second request starts from the width the first one ended with
            for s in segs:
                plan.collect(s)
            assert_same(plan.build().to_dict(), want["shards"][0], f"shard rep{rep}")
            plan.reset()
    finally:
        plan.close()
        for s in segs:
            s.close()


def _zipf_cols(seed, n, T, a=1.1):
    rng = np.random.default_rng(seed)
    ranks = np.minimum(rng.zipf(a, size=n) - 1, T - 1)
    ords = (ranks * 7919 + 17) % T
    ords[rng.random(n) < 0.02] = 0xFFFFFFFF
    return _cols(ords, T, rng)


@pytest.mark.parametrize("size", [1, 10, 200])
def test_deferred_cold_lists_settled_by_hot_slots(engine, size):
    """Zipf(1.1) over 400,000 ordinals, one terms aggregation in count order (the config-3 request): the hot slots'
    top-k is above every cold ordinal's count, so the cold counting and the full top-k are skipped on the device
    (path 8); the other doc count is the segment's total minus the winners'."""
    n, T = 2_000_000, 400_000
    cols = _zipf_cols(106, n, T)
    _check(engine, cols, n, [AB.terms("c").field("kw").size(size)], reps=2, path_want=8)


def test_deferred_cold_lists_counted_when_needed(engine):
    """Uniform over 200,000 ordinals (the hot set's counts tie with cold ones): the k-th hot count does not exceed
    the largest cold count, so the deferred cold lists are counted before the full top-k (path 8, same result)."""
    rng = np.random.default_rng(107)
    n, T = 1_500_000, 200_000
    cols = _cols(rng.integers(0, T, size=n), T, rng)
    _check(engine, cols, n, [AB.terms("c").field("kw").size(40)], reps=2, path_want=8)
    _check(engine, cols, n, [AB.terms("c").field("kw").size(1000).shardSize(1000)], path_want=8)


def test_deferred_cold_lists_second_segment_and_reset(engine):
    """The first segment defers its cold lists; a second segment's collect counts them first (then adds its own,
    path 7); a request reset before its build drops them (the next request counts from scratch)."""
    T = 300_000
    sizes = [900_000, 1_300_000]
    cols = [_zipf_cols(108 + k, n, T, 1.1 + 0.1 * k) for k, n in enumerate(sizes)]
    allc = {"kw": dict(cols[0]["kw"], values=np.concatenate([c["kw"]["values"] for c in cols])),
            "status": {"type": N.COL_I64, "values": np.concatenate([c["status"]["values"] for c in cols])}}
    aggs = [AB.terms("c").field("kw").size(15)]
    want = O.run([(allc, sum(sizes))], aggs)
    want0 = O.run([(cols[0], sizes[0])], aggs)
    segs = [engine.upload_segment(c, n) for c, n in zip(cols, sizes)]
    plan = engine.plan(aggs)
    plan.collect(segs[0])
    assert plan.last_collect_stats()[2] == 8
    plan.reset()
    for k, s in enumerate(segs):
        plan.collect(s)
        assert plan.last_collect_stats()[2] == (8 if k == 0 else 7)
    assert_same(plan.build().to_dict(), want["shards"][0], "two segments")
    plan.reset()
    plan.collect(segs[0])
    assert_same(plan.build().to_dict(), want0["shards"][0], "one segment after reset")
    plan.close()
    for s in segs:
        s.close()


@pytest.mark.parametrize("size", [3, 10, 100])
def test_filtered_deferred_settled(engine, size):
    """Config 3 under a range filter keeping ~75 % and under a live-docs bitset clearing 20 %: Zipf(1.1) head terms
    settle the top-k from the hot slots (path 9); the other doc count is the passing hot docs plus the passing cold
    docs counted beside them."""
    n, T = 2_000_000, 400_000
    cols = _zipf_cols(109, n, T)
    aggs = [AB.terms("c").field("kw").size(size)]
    _check(engine, cols, n, aggs, filters=[QB.rangeQuery("status").gte(1)], reps=2, path_want=9)
    rng = np.random.default_rng(110)
    _check(engine, cols, n, aggs, accept=bits_from_mask(rng.random(n) >= 0.2), reps=2, path_want=9)
    _check(engine, cols, n, aggs, filters=[QB.rangeQuery("status").lte(2)],
           accept=bits_from_mask(rng.random(n) >= 0.3), path_want=9)


def test_filtered_deferred_fallback(engine):
    """A filter whose passing docs are mostly cold: the hot slots' k-th count does not exceed the largest cold count,
    so the scatter form counts the request (path 9's fallback, decided on the device); and a filter that keeps no doc."""
    rng = np.random.default_rng(111)
    n, T = 1_500_000, 200_000
    cols = _cols(rng.integers(0, T, size=n), T, rng)
    _check(engine, cols, n, [AB.terms("c").field("kw").size(25)], filters=[QB.rangeQuery("status").gte(2)], reps=2,
           path_want=9)
    zcols = _zipf_cols(112, n, T)
    _check(engine, zcols, n, [AB.terms("c").field("kw").size(5)], filters=[QB.rangeQuery("status").gte(9)], path_want=9)
    _check(engine, zcols, n, [AB.terms("c").field("kw").size(5).minDocCount(50_000)],
           filters=[QB.rangeQuery("status").gte(1)], path_want=9)
