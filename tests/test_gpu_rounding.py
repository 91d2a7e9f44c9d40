"""GPU parity of date_histogram roundings that are not affine: calendar units (month / quarter / year) and time zones
with DST transitions (TimeZoneRounding.TimeUnitRounding / TimeIntervalRounding over a joda zone).

The kernel buckets these through a per-segment table of bucket start instants built on the host
(es_rounding.hpp key_table); the oracle evaluates the reference's roundKey per value.  Timestamps span two years so
every zone crosses several transitions; sorted data exercises the LDS window, shuffled data the global-atomic path.
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same

pytestmark = pytest.mark.gpu

T0 = 1388534400000  # 2014-01-01T00:00:00Z
SPAN = 2 * 365 * 86_400_000


def columns(n, seed, sorted_ts=True, lo=T0, span=SPAN):
    rng = np.random.default_rng(seed)
    ts = rng.integers(lo, lo + span, size=n).astype(np.int64)
    if sorted_ts:
        ts.sort()
    host = np.minimum(rng.zipf(1.5, size=n) - 1, 199).astype(np.uint32)
    rt = rng.integers(0, 1000, size=n).astype(np.int64)
    return {"@timestamp": {"type": N.COL_I64, "values": ts},
            "host": {"type": N.COL_ORD_U32, "values": host, "terms": ["h%03d" % i for i in range(200)]},
            "response_time_ms": {"type": N.COL_I64, "values": rt}}


def check(engine, aggs, cols, n):
    want = O.run([(cols, n)], aggs)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")
    plan.close()
    seg.close()
    return want["reduced"]


CALENDAR = [
    AB.dateHistogram("month").field("@timestamp").interval("month").subAggregation(AB.stats("rt").field("response_time_ms")),
    AB.dateHistogram("quarter").field("@timestamp").interval("quarter"),
    AB.dateHistogram("year").field("@timestamp").interval("1y").subAggregation(AB.extendedStats("rt").field("response_time_ms")),
    AB.dateHistogram("month_off").field("@timestamp").interval("1M").offset("6h").timeZone("-03:00"),
]

ZONED = [
    AB.dateHistogram("day_chicago").field("@timestamp").interval("1d").timeZone("America/Chicago")
    .subAggregation(AB.avg("rt").field("response_time_ms")),
    AB.dateHistogram("hour_berlin").field("@timestamp").interval("1h").timeZone("Europe/Berlin"),
    AB.dateHistogram("m90_jerusalem").field("@timestamp").interval("90m").timeZone("Asia/Jerusalem"),
    AB.dateHistogram("week_lord_howe").field("@timestamp").interval("week").timeZone("Australia/Lord_Howe"),
    AB.dateHistogram("month_sao_paulo").field("@timestamp").interval("month").timeZone("America/Sao_Paulo").offset("1h"),
]


@pytest.mark.parametrize("sorted_ts", [True, False])
def test_calendar_units(engine, sorted_ts):
    r = check(engine, CALENDAR, columns(1_500_000, 1, sorted_ts), 1_500_000)
    assert len(r["month"]["buckets"]) == 24 and len(r["quarter"]["buckets"]) == 8 and len(r["year"]["buckets"]) == 2


@pytest.mark.parametrize("sorted_ts", [True, False])
def test_dst_zones(engine, sorted_ts):
    check(engine, ZONED, columns(1_500_000, 2, sorted_ts), 1_500_000)


def test_dst_nested_under_terms_and_over_terms(engine):
    aggs = [AB.terms("hosts").field("host").size(20).subAggregation(
                AB.dateHistogram("d").field("@timestamp").interval("day").timeZone("Europe/Berlin")
                .subAggregation(AB.stats("rt").field("response_time_ms"))),
            AB.dateHistogram("m").field("@timestamp").interval("month").timeZone("America/Chicago")
            .subAggregation(AB.terms("hosts").field("host").size(5))]
    check(engine, aggs, columns(1_000_000, 3), 1_000_000)


def test_calendar_extended_bounds_empty_buckets(engine):
    """min_doc_count 0 with extended_bounds outside the data: ExtendedBounds.round and the empty-bucket fill both use
    the zoned calendar rounding (nextRoundingValue across DST)."""
    lo, hi = T0 + 100 * 86_400_000, T0 + 160 * 86_400_000
    cols = columns(200_000, 4, lo=lo, span=hi - lo)
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("day").timeZone("America/Chicago").minDocCount(0)
            .extendedBounds(T0 + 60 * 86_400_000, T0 + 200 * 86_400_000),
            AB.dateHistogram("m").field("@timestamp").interval("month").timeZone("Europe/Berlin").minDocCount(0)
            .extendedBounds(T0, T0 + 300 * 86_400_000)]
    r = check(engine, aggs, cols, 200_000)
    assert len(r["m"]["buckets"]) == 10


def test_table_grows_across_segments(engine):
    """Two segments whose time ranges do not overlap: the second one extends the bucket table on both sides' union
    and the grid rows of the first are shifted, not lost."""
    n1, n2 = 300_000, 200_000
    a = columns(n1, 5, lo=T0 + 400 * 86_400_000, span=100 * 86_400_000)
    b = columns(n2, 6, lo=T0, span=90 * 86_400_000)
    one = {k: {**a[k], "values": np.concatenate([a[k]["values"], b[k]["values"]])} for k in a}
    aggs = [AB.dateHistogram("m").field("@timestamp").interval("month").timeZone("America/Chicago")
            .subAggregation(AB.avg("rt").field("response_time_ms")),
            AB.terms("hosts").field("host").size(5).subAggregation(
                AB.dateHistogram("w").field("@timestamp").interval("week").timeZone("Europe/Berlin"))]
    want = O.run([(one, n1 + n2)], aggs)
    segs = [engine.upload_segment(a, n1), engine.upload_segment(b, n2)]
    plan = engine.plan(aggs)
    for s in segs:
        plan.collect(s)
    assert_same(plan.build().to_dict(), want["shards"][0], "shard")
    plan.close()
    for s in segs:
        s.close()


@pytest.mark.parametrize("jitter", [60_000, 3_600_000])
def test_roughly_sorted_timestamps(engine, jitter):
    """Docs displaced by up to +-1 min / +-1 h (merged segments are only roughly time-ordered): blocks span more hour
    keys than the LDS window, the rest go through the global-atomic path; results stay bit-exact."""
    from elasticsearch_amd import reduce
    import oracle as O
    from helpers import assert_same, synthetic_columns
    n = 2_000_000
    fields = ("host", "@timestamp", "response_time_ms")
    aggs = [AB.terms("hosts").field("host").size(10).subAggregation(
                AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("response_time_ms"))),
            AB.dateHistogram("m").field("@timestamp").interval("1m").subAggregation(AB.extendedStats("rt").field("response_time_ms")),
            # a bucket table (DST zone) under terms: multi-pass windows over table keys
            AB.terms("ny").field("host").size(5).subAggregation(
                AB.dateHistogram("h").field("@timestamp").interval("hour").timeZone("America/New_York")
                .subAggregation(AB.avg("rt").field("response_time_ms"))),
            # minute keys under terms: a block spans more than kMaxPasses windows -> the global-atomic path
            AB.terms("mm").field("host").size(3).subAggregation(AB.dateHistogram("m").field("@timestamp").interval("1m"))]
    want = O.run([(synthetic_columns(fields, n, ts_jitter_ms=jitter), n)], aggs)
    seg = engine.synthetic_segment(n, fields=fields, ts_jitter_ms=jitter)
    host_ts = synthetic_columns(("@timestamp",), n, ts_jitter_ms=jitter)["@timestamp"]["values"]
    assert np.array_equal(seg.read_column("@timestamp", 0, n, np.int64), host_ts)  # device generator == host generator
    assert np.any(np.diff(host_ts) < 0)
    plan = engine.plan(aggs)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")
    plan.close()
    seg.close()


def test_multi_pass_blocks_with_missing_timestamps(engine):
    """Multi-pass blocks (+-1 h jitter, hour keys under / over terms) with 15 % of the timestamps missing: the terms'
    doc counts (docs without a timestamp included) are taken in the first pass only, the histogram's per-key counts
    (date_histogram over terms) in the pass whose window holds the key."""
    from elasticsearch_amd import reduce
    import oracle as O
    from helpers import assert_same, bits_from_mask, synthetic_columns
    n = 3_000_000
    cols = synthetic_columns(("host", "@timestamp", "bytes"), n, ts_jitter_ms=3_600_000)
    cols["@timestamp"]["present"] = bits_from_mask(np.random.default_rng(11).random(n) >= 0.15)
    aggs = [AB.terms("hosts").field("host").size(20).subAggregation(
                AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.avg("b").field("bytes"))),
            AB.dateHistogram("d").field("@timestamp").interval("1h").subAggregation(
                AB.terms("t").field("host").size(4).subAggregation(AB.stats("b").field("bytes")))]
    want = O.run([(cols, n)], aggs)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")
    plan.close()
    seg.close()
