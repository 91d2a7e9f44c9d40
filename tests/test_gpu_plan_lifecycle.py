"""GPU: plan lifecycle across segments and requests.

A plan is one shard request's aggregator tree (AggregatorBase.getLeafCollector once per segment, AggregatorBase.java:129-133)
and may be reset for the next request.  These cases pin the state that must NOT leak between segments or requests:
  * two segments whose dictionaries number terms differently cannot be counted into one grid without an ordinal map
    (the reference always collects global ordinals, GlobalOrdinalsStringTermsAggregator.java:90-105);
  * a reset plan resolves the next request's terms through that request's dictionary, even with equal term counts;
  * a later segment that widens the histogram key range keeps the cardinality sketches' non-zero register counts;
  * a metric field that turns sparse, a histogram field that turns sparse, and a first segment without histogram
    values all give the oracle's result over the concatenated docs.
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same, bits_from_mask

pytestmark = pytest.mark.gpu

T0 = 1441065600000


def _concat(parts):
    """Oracle input for several uploaded segments of one shard: their columns concatenated (same dictionaries)."""
    out = {}
    for name in parts[0]:
        cols = [p[name] for p in parts]
        c = dict(cols[0])
        c["values"] = np.concatenate([x["values"] for x in cols])
        if any(x.get("present") is not None for x in cols):
            mask = np.concatenate([_mask(x) for x in cols])
            c["present"] = bits_from_mask(mask)
        out[name] = c
    return out


def _mask(c):
    n = len(c["values"])
    if c.get("present") is None:
        return np.ones(n, dtype=bool)
    words = np.asarray(c["present"], dtype=np.uint64)
    bits = ((words[np.arange(n) // 64] >> (np.arange(n) % 64).astype(np.uint64)) & np.uint64(1)).astype(bool)
    return bits


def test_segments_with_different_dictionaries_need_an_ordinal_map(engine):
    n = 50_000
    rng = np.random.default_rng(1)
    a = {"kw": {"type": N.COL_ORD_U32, "values": rng.integers(0, 3, n, dtype=np.uint32), "terms": ["a", "b", "c"]}}
    b = {"kw": {"type": N.COL_ORD_U32, "values": rng.integers(0, 3, n, dtype=np.uint32), "terms": ["b", "c", "d"]}}
    sa, sb = engine.upload_segment(a, n), engine.upload_segment(b, n)
    plan = engine.plan([AB.terms("t").field("kw")])
    plan.collect(sa)
    with pytest.raises(N.EsGpuError) as e:
        plan.collect(sb)
    assert e.value.code == N.ERR_INVALID and "ordinal map" in str(e.value)
    plan.close()
    # the same two segments under an ordinal map: global ordinals, one grid
    omap = engine.ordinal_map([sa, sb], "kw")
    plan = engine.plan([AB.terms("t").field("kw").size(10)])
    plan.collect(sa)
    plan.collect(sb)
    got = {x["key"]: x["doc_count"] for x in plan.build().to_dict()["t"]["buckets"]}
    va, vb = a["kw"]["values"], b["kw"]["values"]
    want = {}
    for terms, v in ((a["kw"]["terms"], va), (b["kw"]["terms"], vb)):
        for o, c in zip(*np.unique(v, return_counts=True)):
            want[terms[o]] = want.get(terms[o], 0) + int(c)
    assert got == want
    plan.close()
    omap.close()
    sa.close()
    sb.close()


def test_reset_plan_takes_the_next_requests_dictionary(engine):
    n = 40_000
    rng = np.random.default_rng(2)
    aggs = [AB.terms("t").field("kw").size(5)]
    plan = engine.plan(aggs)
    for terms in (["apple", "berry", "cherry", "date"], ["w", "x", "y", "z"]):
        cols = {"kw": {"type": N.COL_ORD_U32, "values": rng.integers(0, 4, n, dtype=np.uint32), "terms": terms}}
        seg = engine.upload_segment(cols, n)
        plan.reset()
        plan.collect(seg)
        seg.close()  # the plan keeps the dictionary it resolves winners through
        assert_same(plan.build().to_dict(), O.run([(cols, n)], aggs)["shards"][0], "shard")
    plan.close()


def test_later_segment_widens_keys_without_cardinality_field(engine):
    """Segment 1 holds the cardinality field (one bucket ends in HYPERLOGLOG); segment 2 lacks it and extends the
    histogram range: the sketches move with the regrid, their non-zero register counts included."""
    rng = np.random.default_rng(3)
    n1, n2 = 120_000, 30_000
    day = 86_400_000
    s1 = {"@timestamp": {"type": N.COL_I64, "values": np.sort(rng.integers(T0, T0 + 2 * day, n1)).astype(np.int64)},
          "ip": {"type": N.COL_U64, "values": rng.integers(0, 2**63, n1, dtype=np.uint64)}}
    s2 = {"@timestamp": {"type": N.COL_I64, "values": np.sort(rng.integers(T0 - 3 * day, T0 + 5 * day, n2)).astype(np.int64)}}
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("1d").subAggregation(
        AB.cardinality("c").field("ip").precisionThreshold(100))]
    segs = [engine.upload_segment(s1, n1), engine.upload_segment(s2, n2)]
    plan = engine.plan(aggs)
    for s in segs:
        plan.collect(s)
    got = plan.build().to_dict()
    # oracle: the same docs in one segment, the ip field missing on segment 2's docs
    ip = np.concatenate([s1["ip"]["values"], np.zeros(n2, np.uint64)])
    one = {"@timestamp": {"type": N.COL_I64, "values": np.concatenate([s1["@timestamp"]["values"], s2["@timestamp"]["values"]])},
           "ip": {"type": N.COL_U64, "values": ip, "present": bits_from_mask(np.arange(n1 + n2) < n1)}}
    want = O.run([(one, n1 + n2)], aggs)["shards"][0]
    assert_same(got, want, "shard")
    modes = {b["c"]["_internal"].get("mode") for b in got["d"]["buckets"]}
    assert "hll" in modes
    plan.close()


def test_sparsity_changes_across_segments(engine):
    """Segment 1: dense metric and histogram columns; segment 2: both sparse; segment 0 (first): no histogram values at
    all.  terms{date_histogram{stats}} over the three == the oracle over their concatenation."""
    rng = np.random.default_rng(4)
    terms = ["h%02d" % i for i in range(20)]

    def seg(n, ts_present, rt_present):
        c = {"kw": {"type": N.COL_ORD_U32, "values": rng.integers(0, 20, n, dtype=np.uint32), "terms": terms},
             "@timestamp": {"type": N.COL_I64, "values": np.sort(rng.integers(T0, T0 + 86_400_000, n)).astype(np.int64)},
             "rt": {"type": N.COL_I64, "values": rng.integers(0, 1000, n).astype(np.int64)}}
        if ts_present is not None:
            c["@timestamp"]["present"] = bits_from_mask(rng.random(n) < ts_present)
        if rt_present is not None:
            c["rt"]["present"] = bits_from_mask(rng.random(n) < rt_present)
        return c, n

    parts = [seg(20_000, 0.0, None), seg(60_000, None, None), seg(50_000, 0.6, 0.5)]
    aggs = [AB.terms("t").field("kw").size(20).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("rt"))),
        AB.dateHistogram("h2").field("@timestamp").interval("3h").subAggregation(AB.avg("a").field("rt"))]
    segs = [engine.upload_segment(c, n) for c, n in parts]
    plan = engine.plan(aggs)
    for rep in range(2):  # and again after a reset, the buffers reused
        for s in segs:
            plan.collect(s)
        res = plan.build()
        one = _concat([c for c, _ in parts])
        want = O.run([(one, sum(n for _, n in parts))], aggs)
        assert_same(res.to_dict(), want["shards"][0], f"shard rep{rep}")
        assert_same(reduce([res]).to_dict(), want["reduced"], f"reduced rep{rep}")
        plan.reset()
    plan.close()
