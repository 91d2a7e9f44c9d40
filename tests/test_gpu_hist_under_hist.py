"""GPU parity for histogram under histogram (a5; e.g. the latency heat map date_histogram{histogram}): the outer
histogram is the key dimension of the cell grid, the inner histogram's key indices -- derived per segment from its field
with its affine rounding -- are the ordinal dimension (HistogramAggregator under asMultiBucketAggregator,
A/AggregatorFactory.java:107-200; buckets per owning bucket in key order, HistogramAggregator.java:110-133), reduced by
InternalHistogram.doReduce at both levels (empty-bucket fill included)."""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same, bits_from_mask, synthetic_columns

pytestmark = pytest.mark.gpu

FIELDS = ("@timestamp", "response_time_ms", "bytes", "price", "client_ip.hash")


def _both(engine, aggs, n=300_000, shards=2, exact=True):
    data = [(synthetic_columns(FIELDS, n, shard=s), n) for s in range(shards)]
    want = O.run(data, aggs, number_of_shards=shards)
    plan = engine.plan(aggs, number_of_shards=shards)
    results = []
    for s, (cols, _) in enumerate(data):
        seg = engine.upload_segment(cols, n)
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


def test_latency_heat_map(engine):
    aggs = [AB.dateHistogram("per_hour").field("@timestamp").interval("1h").minDocCount(1).subAggregation(
        AB.histogram("latency").field("response_time_ms").interval(100).minDocCount(1)
        .subAggregation(AB.avg("b").field("bytes")))]
    red = _both(engine, aggs)
    assert len(red["per_hour"]["buckets"]) > 10 and len(red["per_hour"]["buckets"][0]["latency"]["buckets"]) > 3


def test_inner_empty_buckets_bounds_and_stats(engine):
    """inner min_doc_count 0 with extended bounds (EmptyBucketInfo at both levels), an offset, extended_stats leaves"""
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("1d").subAggregation(
        AB.histogram("rt").field("response_time_ms").interval(250).offset(10).extendedBounds(-500, 1500)
        .subAggregation(AB.extendedStats("x").field("response_time_ms")))]
    _both(engine, aggs)


def test_inner_date_histogram_fixed_zone_and_double_field(engine):
    """outer histogram over a double field, inner date_histogram with a fixed time zone (affine) and cardinality"""
    aggs = [AB.histogram("p").field("price").interval(50).minDocCount(1).subAggregation(
        AB.dateHistogram("days").field("@timestamp").interval("1d").timeZone("+02:00").minDocCount(1)
        .subAggregation(AB.cardinality("ips").field("client_ip.hash"))
        .subAggregation(AB.stats("s").field("bytes")))]
    _both(engine, aggs, exact=False)


@pytest.mark.parametrize("interval,zone,shift_days", [("month", None, 0), ("week", "Europe/Berlin", 50),
                                                      ("1h", "America/New_York", 55), ("quarter", "+05:30", 15),
                                                      ("day", "Australia/Lord_Howe", 20), ("1h", "Europe/Berlin", 50)])
def test_inner_calendar_and_dst_rounding(engine, interval, zone, shift_days):
    """A calendar unit or a DST zone is not affine: the inner date_histogram's key index comes from a bucket table over
    the request's values (Rounding.key_table: step starts, sorted keys, a DST fall-back's repeated local hour mapped to
    its first bucket), each doc's step found by binary search -- against the oracle, with min_doc_count 0 and stats;
    the timestamps shifted so the month spans the zone's transition (Berlin and New York fall back in late October /
    early November 2015, Lord Howe moves 30 min forward on October 4)."""
    dh = AB.dateHistogram("m").field("@timestamp").interval(interval).minDocCount(0)
    if zone:
        dh.timeZone(zone)
    aggs = [AB.histogram("b").field("bytes").interval(250000).subAggregation(dh.subAggregation(
        AB.stats("s").field("response_time_ms")))]
    n, shards = 200_000, 2
    data = []
    for sh in range(shards):
        cols = synthetic_columns(FIELDS, n, shard=sh)
        cols["@timestamp"]["values"] = cols["@timestamp"]["values"] + shift_days * 86_400_000
        data.append((cols, n))
    want = O.run(data, aggs, number_of_shards=shards)
    plan = engine.plan(aggs, number_of_shards=shards)
    results = []
    for sh, (cols, _) in enumerate(data):
        seg = engine.upload_segment(cols, n)
        plan.reset()
        plan.collect(seg)
        r = plan.build()
        assert_same(r.to_dict(), want["shards"][sh], f"shard{sh}")
        results.append(r)
        seg.close()
    assert_same(reduce(results).to_dict(), want["reduced"], "reduced")
    plan.close()


def test_inner_calendar_rounding_two_segments_widen_table(engine):
    """A later segment whose timestamps lie before and after the first's: the inner bucket table grows on both sides and
    the grid's columns move to the new keys' positions."""
    n = 150_000
    c0 = synthetic_columns(FIELDS, n, shard=0)
    c1 = synthetic_columns(FIELDS, n, shard=1)
    c0["@timestamp"]["values"] = c0["@timestamp"]["values"] + 40 * 86_400_000  # a later month range
    c1["@timestamp"]["values"] = c1["@timestamp"]["values"] - 20 * 86_400_000
    aggs = [AB.histogram("b").field("bytes").interval(500000).subAggregation(
        AB.dateHistogram("m").field("@timestamp").interval("month").timeZone("Europe/Berlin").subAggregation(
            AB.avg("a").field("response_time_ms")))]
    allc = {f: dict(c0[f], values=np.concatenate([c0[f]["values"], c1[f]["values"]])) for f in FIELDS}
    want = O.run([(allc, 2 * n)], aggs)
    plan = engine.plan(aggs)
    segs = [engine.upload_segment(c, n) for c in (c0, c1)]
    for sg in segs:
        plan.collect(sg)
    assert_same(plan.build().to_dict(), want["shards"][0], "two segments")
    plan.close()
    for sg in segs:
        sg.close()


def test_inner_field_missing_in_a_segment(engine):
    """the second segment lacks the inner field: its docs count in the outer buckets only"""
    n = 200_000
    c0 = synthetic_columns(FIELDS, n, shard=0)
    c1 = synthetic_columns(FIELDS, n, shard=1)
    del c1["response_time_ms"]
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("6h").subAggregation(
        AB.histogram("rt").field("response_time_ms").interval(200))]
    both = {k: v for k, v in c0.items()}
    for k in c0:
        if k != "response_time_ms":
            both[k] = {"type": c0[k]["type"], "values": np.concatenate([c0[k]["values"], c1[k]["values"]])}
    both["response_time_ms"] = {"type": c0["response_time_ms"]["type"],
                                "values": np.concatenate([c0["response_time_ms"]["values"], np.zeros(n, np.int64)]),
                                "present": np.concatenate([np.full(n // 64, ~np.uint64(0), np.uint64),
                                                           np.zeros(n // 64, np.uint64)])}
    want = O.run([(both, 2 * n)], aggs)
    plan = engine.plan(aggs)
    segs = [engine.upload_segment(c0, n), engine.upload_segment(c1, n)]
    for s in segs:
        plan.collect(s)
    assert_same(plan.build().to_dict(), want["shards"][0], "shard")
    plan.close()
    for s in segs:
        s.close()


def test_fused_inner_key_double_sparse_and_negative(engine):
    """the collect loader derives the inner key index (no cardinality leaf, single-valued): a sparse double inner field,
    and a long inner field with negative values and an offset (keys below zero, floor division)"""
    n = 250_000
    rng = np.random.default_rng(5)
    data = []
    for s in range(2):
        cols = synthetic_columns(FIELDS, n, shard=s)
        keep = rng.random(n) >= 0.2
        cols["price"]["values"] = np.where(keep, cols["price"]["values"], 0.0)
        cols["price"]["present"] = bits_from_mask(keep)
        cols["delta"] = {"type": N.COL_I64, "values": rng.integers(-5000, 5000, size=n).astype(np.int64)}
        data.append((cols, n))
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("12h").subAggregation(
                AB.histogram("p").field("price").interval(25).minDocCount(1).subAggregation(AB.avg("b").field("bytes"))),
            AB.histogram("r").field("response_time_ms").interval(200).subAggregation(
                AB.histogram("dl").field("delta").interval(700).offset(-33).minDocCount(1))]
    want = O.run(data, aggs, number_of_shards=2)
    plan = engine.plan(aggs, number_of_shards=2)
    results = []
    for s, (cols, _) in enumerate(data):
        seg = engine.upload_segment(cols, n)
        plan.reset()
        plan.collect(seg)
        r = plan.build()
        assert_same(r.to_dict(), want["shards"][s], f"shard{s}", False)
        results.append(r)
        seg.close()
    assert_same(reduce(results).to_dict(), want["reduced"], "reduced", False)
    plan.close()


@pytest.mark.parametrize("first", ["narrow", "missing"])
def test_later_segment_widens_inner_keys(engine, first):
    """a later segment's inner values fall outside the key range the first segment fixed (or the first segment has no
    inner values at all): the grid's ordinal columns move over to the wider range (strided copies of every cell array,
    cardinality sketches included) and the request stays on the GPU"""
    n = 200_000
    c0 = synthetic_columns(FIELDS, n, shard=0)
    c1 = synthetic_columns(FIELDS, n, shard=1)
    rt0 = c0["response_time_ms"]["values"]
    if first == "narrow":
        c0["response_time_ms"]["values"] = np.clip(rt0, 300, 599)
    else:
        c0["response_time_ms"]["values"] = np.zeros_like(rt0)
        c0["response_time_ms"]["present"] = np.zeros(n // 64, np.uint64)
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("6h").subAggregation(
        AB.histogram("rt").field("response_time_ms").interval(100)
        .subAggregation(AB.stats("b").field("bytes"))
        .subAggregation(AB.cardinality("ips").field("client_ip.hash").precisionThreshold(50)))]
    both = {}
    for k in c0:
        both[k] = {"type": c0[k]["type"], "values": np.concatenate([c0[k]["values"], c1[k]["values"]])}
        if "present" in c0[k] or "present" in c1[k]:
            full = np.full(n // 64, ~np.uint64(0), np.uint64)
            both[k]["present"] = np.concatenate([c0[k].get("present", full), c1[k].get("present", full)])
    want = O.run([(both, 2 * n)], aggs)
    plan = engine.plan(aggs)
    segs = [engine.upload_segment(c0, n), engine.upload_segment(c1, n)]
    for s in segs:
        plan.collect(s)
    assert_same(plan.build().to_dict(), want["shards"][0], "shard")
    plan.close()
    for s in segs:
        s.close()


def _multi_values(rng, n, lo, hi, f64=False, max_per_doc=3):
    """a SortedNumeric field: 0..max_per_doc values per doc, sorted within the doc"""
    per = rng.integers(0, max_per_doc + 1, size=n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(per)
    vals = rng.integers(lo, hi, size=int(offs[-1])).astype(np.int64)
    order = np.lexsort((vals, np.repeat(np.arange(n), per)))  # each doc's values sorted (SortedNumericDocValues)
    vals = vals[order]
    if f64:
        vals = (vals.astype(np.float64) + 0.25)
    return vals, offs


@pytest.mark.parametrize("f64", [False, True])
def test_multi_valued_inner_histogram(engine, f64):
    """A multi-valued inner histogram field (SortedNumeric, several latencies per doc): each value's key, a doc's
    repeated keys once (HistogramAggregator.collect over sorted values), counted in the CSR collect kernel from a key
    index per value -- doc counts, avg / extended_stats leaves and inner empty buckets against the oracle."""
    rng = np.random.default_rng(77)
    n = 200_000
    cols = synthetic_columns(("@timestamp", "bytes"), n)
    vals, offs = _multi_values(rng, n, 0, 2000, f64=f64)
    cols["lat"] = {"type": N.COL_F64 if f64 else N.COL_I64, "values": vals, "offsets": offs}
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("1d").minDocCount(1).subAggregation(
                AB.histogram("lat").field("lat").interval(250).minDocCount(0)
                .subAggregation(AB.avg("b").field("bytes")).subAggregation(AB.extendedStats("x").field("bytes")))]
    want = O.run([(cols, n)], aggs)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs)
    plan.collect(seg)
    assert_same(plan.build().to_dict(), want["shards"][0], "shard")
    plan.close()
    seg.close()
