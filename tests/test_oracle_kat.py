"""The oracle is pinned against the reference's own known-answer vectors and fixtures (tests/golden/kat.json,
extracted by tests/golden/make_golden.py from the reference test sources; each vector cites file:line)."""
import ctypes

import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order
from elasticsearch_amd import _native as N


def _s64(v):
    return v - (1 << 64) if v >> 63 else v


def test_murmur3_known_values(kat):  # MurmurHash3Tests.java:29-38
    L = O.lib()
    for v in kat["murmur3_x64_128"]:
        b = v["input"].encode("utf-8")
        h1, h2 = ctypes.c_uint64(), ctypes.c_uint64()
        L.oracle_murmur3_128(b, len(b), v["seed"], ctypes.byref(h1), ctypes.byref(h2))
        assert (_s64(h1.value), _s64(h2.value)) == (v["h1"], v["h2"]), v["cite"]


def test_precision_from_threshold(kat):  # HyperLogLogPlusPlusTests.java:126-135
    L = O.lib()
    for v in kat["precision_from_threshold"]:
        assert L.oracle_precision_from_threshold(v["threshold"]) == v["precision"], v["cite"]


def test_hll_encode_decode_identity():  # HyperLogLogPlusPlusTests.encodeDecode (:34-57)
    L = O.lib()
    rng = np.random.default_rng(1234)
    hashes = [int(x) for x in rng.integers(0, 2**63, size=20000, dtype=np.int64)] + [0, 1, 2**64 - 1]
    for i, h in enumerate(hashes):
        for p in (4, 14, 18, 24) if i < 200 else ((i % 21) + 4,):
            enc = L.oracle_encode_hash(h, p)
            assert L.oracle_decode_index(enc, p) == L.oracle_index(h, p)
            assert L.oracle_decode_run_len(enc, p) == L.oracle_run_len(h, p)


def test_hll_fake_hashes():  # HyperLogLogPlusPlusTests.fakeHashes (:109-124): all hashes in one register
    L = O.lib()
    for p in range(4, 19):
        arr = (ctypes.c_uint64 * 2)(0, 1)
        mode = ctypes.c_int32()
        assert L.oracle_hll_collect(p, arr, 1, ctypes.byref(mode), None) == 1
        assert L.oracle_hll_collect(p, arr, 2, ctypes.byref(mode), None) == 2


def test_hll_accuracy_and_upgrade():  # HyperLogLogPlusPlusTests.accuracy (:59-78): within 10 %
    L = O.lib()
    rng = np.random.default_rng(7)
    for p in (14, 16, 18):
        vals = rng.integers(0, 100000, size=100000)
        hashes = np.array([L.oracle_mix64(int(v)) for v in vals], dtype=np.uint64)
        mode = ctypes.c_int32()
        est = L.oracle_hll_collect(p, hashes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(hashes), ctypes.byref(mode), None)
        exact = len(set(vals.tolist()))
        assert abs(est - exact) <= 0.1 * exact


ROUND_KIND = {"histogram": 0, "unit": 1, "interval": 2}
UNITS = {"month": N.UNIT_MONTH, "week": N.UNIT_WEEK, "day": N.UNIT_DAY, "hour": N.UNIT_HOUR}


def test_rounding_known_values(kat):  # RoundingTests / TimeZoneRoundingTests (UTC and fixed offsets)
    L = O.lib()
    for c in kat["rounding"]:
        kind = ROUND_KIND[c["kind"]]
        unit = UNITS.get(c.get("unit"), 0)
        interval = c.get("interval", 1)
        for v, expect in c["round"]:
            assert L.oracle_rounding(kind, unit, interval, c["offset"], 0, v) == expect, c["cite"]
        for v, expect in c["next"]:
            assert L.oracle_rounding(kind, unit, interval, c["offset"], 1, v) == expect, c["cite"]
        for v, expect in c.get("keys", []):
            assert L.oracle_rounding(kind, unit, interval, c["offset"], 2, v) == expect, c["cite"]


TZ_UNITS = {"hour": N.UNIT_HOUR, "day": N.UNIT_DAY, "month": N.UNIT_MONTH, "year": N.UNIT_YEAR, "minute": N.UNIT_MINUTE}


def oracle_round_tz(kind, unit, interval, offset, zone, op, v):
    """The oracle's Rounding with the oracle's own zone table (TZif transitions + POSIX footer, oracle_request.py)."""
    import oracle_request
    starts, offs = oracle_request.zone_table(zone) or ((-(1 << 63),), (0,))
    st = (ctypes.c_int64 * len(starts))(*starts)
    of = (ctypes.c_int64 * len(offs))(*offs)
    return O.lib().oracle_rounding_tz(kind, unit, interval, offset, st, of, len(starts), op, v)


def test_rounding_dst_known_values(kat):  # TimeZoneRoundingTests.testTimeUnitRoundingDST / testAmbiguousHoursAfterDSTSwitch
    cases = kat["rounding_tz"]["cases"]
    assert sum(len(c["round"]) for c in cases) == 19
    for c in cases:
        for v, expect in c["round"]:
            got = oracle_round_tz(1, TZ_UNITS[c["unit"]], 0, 0, c["zone"], 0, v)
            assert got == expect, (c["cite"], v, got, expect)
        for a, b in c.get("same", []):
            assert oracle_round_tz(1, TZ_UNITS[c["unit"]], 0, 0, c["zone"], 0, a) == \
                oracle_round_tz(1, TZ_UNITS[c["unit"]], 0, 0, c["zone"], 0, b), c["cite"]


def test_rounding_dst_lenient_conversion(kat):  # TimeZoneRoundingTests.testLenientConversionDST
    c = kat["rounding_tz"]["lenient"]
    for t in range(c["start"], c["end"], c["step"]):
        assert oracle_round_tz(1, N.UNIT_MINUTE, 0, 0, c["zone"], 1, t) > t, c["cite"]
        assert oracle_round_tz(2, 0, 60000, 0, c["zone"], 1, t) > t, c["cite"]


def test_rounding_tz_random_properties():  # TimeZoneRoundingTests.testTimeZoneRoundingRandom with DST zones
    rng = np.random.default_rng(77)
    for i in range(600):
        zone = ["Europe/Berlin", "America/Chicago", "Asia/Jerusalem", "America/Sao_Paulo", "Australia/Lord_Howe"][i % 5]
        unit = int(rng.integers(1, 9))
        date = int(rng.integers(0, 10**12))
        r = oracle_round_tz(1, unit, 0, 0, zone, 0, date)
        nxt = oracle_round_tz(1, unit, 0, 0, zone, 1, r)
        assert r <= date, (zone, unit, date)
        assert oracle_round_tz(1, unit, 0, 0, zone, 0, r) == r, (zone, unit, date)
        assert nxt > r, (zone, unit, date)


def _i64(vals):
    return {"type": N.COL_I64, "values": np.array(vals, dtype=np.int64)}


def _multi_i64(lists):
    offs = np.zeros(len(lists) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in lists])
    return {"type": N.COL_I64, "values": np.array([v for x in lists for v in sorted(x)], dtype=np.int64), "offsets": offs}


def test_extended_stats_fixture(kat):  # ExtendedStatsTests.testSingleValuedField / multi-valued (AbstractNumericTestCase)
    st = kat["stats"]
    cols = {"value": _i64(st["docs"]["value"]), "values": _multi_i64(st["docs"]["values"])}
    res = O.run([(cols, 10)], [AB.extendedStats("s1").field("value"), AB.extendedStats("s2").field("values")])["reduced"]
    for name, exp in (("s1", st["single"]), ("s2", st["multi"])):
        got = res[name]
        for k in ("count", "sum", "min", "max", "avg", "sum_of_squares", "variance"):
            assert got[k] == exp[k], (name, k)


def test_empty_bucket_extended_stats(kat):  # ExtendedStatsTests.testEmptyAggregation: bucket "1" is empty
    cols = {"value": _i64(kat["stats"]["empty_bucket_docs"])}
    agg = AB.histogram("histo").field("value").interval(1).minDocCount(0).subAggregation(AB.extendedStats("stats"))
    res = O.run([(cols, 2)], [agg])["reduced"]["histo"]["buckets"]
    assert [b["key"] for b in res] == [0, 1, 2]
    s = res[1]["stats"]
    assert s["count"] == 0 and s["_internal"]["min"] == float("inf") and s["_internal"]["max"] == float("-inf")
    assert s["avg"] is None and s["std_deviation"] is None


def _terms_col(keys):
    terms = sorted(set(keys))
    return {"type": N.COL_ORD_U32, "values": np.array([terms.index(k) for k in keys], dtype=np.uint32), "terms": terms}


def test_shard_size_terms(kat):  # ShardSizeTermsIT.noShardSize_string / shardSizeEqualsSize_string
    fx = kat["shard_size_terms"]
    shards = []
    for counts in fx["shards"]:
        keys = [k for k, n in sorted(counts.items()) for _ in range(n)]
        shards.append(({"key": _terms_col(keys)}, len(keys)))
    for case in fx["cases"]:
        b = AB.terms("keys").field("key").size(case["size"]).order(Order.count(False))
        if case["shard_size"] is not None:
            b.shardSize(case["shard_size"])
        res = O.run(shards, [b], number_of_shards=2)["reduced"]["keys"]
        got = {x["key"]: x["doc_count"] for x in res["buckets"]}
        assert got == case["expect"], case["cite"]


def test_histogram_rest_fixture(kat):  # 10_histogram.yaml
    h = kat["rest"]["histogram"]
    res = O.run([({"number": _i64(h["numbers"])}, 4)], [AB.histogram("histo").field("number").interval(h["interval"])])
    b = res["reduced"]["histo"]["buckets"]
    assert [x["key"] for x in b] == h["keys"] and [x["doc_count"] for x in b] == h["doc_counts"]


def test_murmur3_cardinality_rest_fixture(kat):  # mapper_murmur3/10_basic.yaml: cardinality on foo.hash
    L = O.lib()
    fx = kat["rest"]["murmur3_cardinality"]
    hashes = []
    for s in fx["foo"]:
        b = s.encode()
        h1, h2 = ctypes.c_uint64(), ctypes.c_uint64()
        L.oracle_murmur3_128(b, len(b), 0, ctypes.byref(h1), ctypes.byref(h2))
        hashes.append(h1.value)
    empty = O.run([({"foo.hash": {"type": N.COL_U64, "values": np.zeros(1, np.uint64), "present": np.zeros(1, np.uint64)}}, 1)],
                  [AB.cardinality("foo_count").field("foo.hash")])
    assert empty["reduced"]["foo_count"]["value"] == fx["empty_value"]
    cols = {"foo.hash": {"type": N.COL_U64, "values": np.array(hashes, dtype=np.uint64)}}
    res = O.run([(cols, len(hashes))], [AB.cardinality("foo_count").field("foo.hash")])
    assert res["reduced"]["foo_count"]["value"] == fx["value"]


def test_date_histogram_fixture(kat):  # DateHistogramTests.singleValuedField / _WithTimeZone
    fx = kat["date_histogram"]
    cols = {"date": _i64(fx["date"]), "dates": _multi_i64(fx["dates"])}
    res = O.run([(cols, 6)], [AB.dateHistogram("histo").field("date").interval("month")])["reduced"]["histo"]["buckets"]
    assert [b["key"] for b in res] == fx["monthly"]["keys"]
    assert [b["doc_count"] for b in res] == fx["monthly"]["doc_counts"]
    tz = fx["daily_tz_plus1"]
    res = O.run([(cols, 6)], [AB.dateHistogram("histo").field("date").interval("day").minDocCount(1).timeZone("+01:00")])
    b = res["reduced"]["histo"]["buckets"]
    assert [x["key"] for x in b] == tz["keys"] and [x["doc_count"] for x in b] == tz["doc_counts"]


def oracle_routing_hash(s):
    L = O.lib()
    L.oracle_routing_hash.restype = ctypes.c_int32
    L.oracle_routing_hash.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    u = np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16).copy()
    return L.oracle_routing_hash(u.ctypes.data if u.size else None, u.size)


def oracle_shard_id(h, n):
    L = O.lib()
    L.oracle_shard_id.restype = ctypes.c_int32
    L.oracle_shard_id.argtypes = [ctypes.c_int32, ctypes.c_int32]
    return L.oracle_shard_id(h, n)


def test_routing_murmur3_known_values(kat):  # Murmur3HashFunctionTests.testKnownValues
    for v in kat["routing_murmur3_x86_32"]:
        assert oracle_routing_hash(v["input"]) == v["hash"], v["cite"]
    assert oracle_shard_id(-7, 5) == 3 and oracle_shard_id(7, 5) == 2  # MathUtils.mod: floor modulo


@pytest.mark.parametrize("num_docs,num_tag1", [(5, 1), (12, 7), (20, 19)])
def test_filter_aggregation_fixture(num_docs, num_tag1):  # FilterIT.simple / withSubAggregation (FilterIT.java:95-146)
    """FilterIT's index: docs 0..numTag1Docs-1 {value: i+1, tag: tag1}, the rest {value: i, tag: tag2}.
    filter(termQuery(tag, tag1)) has doc_count numTag1Docs and avg(value) = sum(1..numTag1Docs) / numTag1Docs."""
    from elasticsearch_amd import QueryBuilders as QB
    tags = ["tag1" if i < num_tag1 else "tag2" for i in range(num_docs)]
    vals = [i + 1 if i < num_tag1 else i for i in range(num_docs)]
    cols = {"tag": _terms_col(tags), "value": _i64(vals)}
    lookup = {"tag1": 0, "tag2": 1}
    aggs = [AB.filter("tag1", QB.termQuery("tag", "tag1")).subAggregation(AB.avg("avg_value").field("value")),
            AB.filter("plain", QB.termQuery("tag", "tag1"))]
    res = O.run([(cols, num_docs)], aggs, ord_lookup=lambda f, t: lookup.get(t, -1))["reduced"]
    assert res["tag1"]["doc_count"] == num_tag1 and res["plain"]["doc_count"] == num_tag1
    assert res["tag1"]["avg_value"]["value"] == sum(range(1, num_tag1 + 1)) / num_tag1
    assert list(res["plain"].keys()) == ["doc_count"]
