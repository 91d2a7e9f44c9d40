"""Elasticsearch transport bytes of shard results (esgpu_result_to_stream = InternalAggregations.writeTo, SURVEY §8(f)
rank 3), on the CPU.

* Hand-derived bytes: a few results whose bytes follow line by line from the reference's writeTo code and StreamOutput's
  encodings (StreamOutput.java:144-265: big-endian int/long, 7-bit vInt/vLong, writeString = char count + modified
  UTF-8, writeBoolean = 0/1, writeGenericValue(null) = -1) -- no JVM exists here, so these are the pinned vectors.
* Writer parity: the oracle (cpu_ref.cpp's own restatement of every writeTo) and the product's writer, fed the same
  shard-level numbers (the oracle's shard results, rebuilt into product result blocks), must emit identical bytes for
  every request shape of the path except cardinality (whose sketch state JSON cannot carry; the GPU test covers it).
"""
import struct

import pytest

import oracle as O
import es_stream as ES
import result_stream as RS
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import ShardResult
from elasticsearch_amd import _native as N
from elasticsearch_amd.aggs import Order
from helpers import synthetic_columns


def _wire(aggs):
    return ShardResult.deserialize(RS.encode(aggs)).to_stream()


def _d(v):
    return struct.pack(">d", v)


def test_stats_bytes_by_hand():
    # InternalAggregations.writeTo: vInt 1, writeBytesReference("stats"), then InternalStats.writeTo
    got = _wire([{"type": N.AGG_STATS, "name": "s", "count": 2, "sum": 3.0, "min": 1.0, "max": 2.0}])
    want = (b"\x01" + b"\x05stats" + b"\x01s" + b"\xff" + b"\x00"      # name, null metaData, 0 pipeline aggs
            + b"\x01\x01"                                               # formatter present, ValueFormatter.Raw id 1
            + b"\x02" + _d(1.0) + _d(2.0) + _d(3.0))                    # vLong count, min, max, sum
    assert got == want


def test_extended_stats_and_avg_bytes_by_hand():
    got = _wire([{"type": N.AGG_EXTENDED_STATS, "name": "x", "count": 10, "sum": 55.0, "min": 1.0, "max": 10.0,
                  "sumsq": 385.0, "sigma": 3.0},
                 {"type": N.AGG_AVG, "name": "a", "count": 300, "sum": 1.5}])
    want = (b"\x02"
            + b"\x06estats" + b"\x01x\xff\x00" + b"\x01\x01" + b"\x0a" + _d(1.0) + _d(10.0) + _d(55.0)
            + _d(385.0) + _d(3.0)                                       # writeOtherStatsTo: sumOfSqrs, sigma
            + b"\x03avg" + b"\x01a\xff\x00" + b"\x01\x01" + _d(1.5) + b"\xac\x02")  # sum, vLong 300 = ac 02
    assert got == want


def test_string_terms_bytes_by_hand():
    t = RS.string_terms("t", [("b", 5), ("é", 3)], size=2, shard_size=2147483647, other=4)
    got = _wire([t])
    want = (b"\x01" + b"\x06sterms" + b"\x01t\xff\x00"
            + struct.pack(">q", 0)                                      # docCountError
            + b"\xff\x02\x01\x04"                                       # CompoundOrder[_count desc, _term asc]
            + b"\x02" + b"\x00"                                         # requiredSize 2, shardSize MAX_VALUE -> 0
            + b"\x00" + b"\x01" + b"\x04"                               # showTermDocCountError, minDocCount, other
            + b"\x02"                                                   # 2 buckets
            + b"\x01b" + b"\x05" + b"\x00"                              # BytesRef "b", docCount 5, no sub-aggs
            + b"\x02\xc3\xa9" + b"\x03" + b"\x00")                      # UTF-8 term bytes as they are indexed
    assert got == want


def test_date_histogram_bytes_by_hand():
    hour = 3_600_000
    h = {"type": N.AGG_DATE_HISTOGRAM, "name": "h", "order": N.ORDER_KEY_ASC, "min_doc_count": 0, "has_empty_info": 1,
         "date_unit": N.UNIT_HOUR, "offset": -1800000, "has_bmin": 1, "bmin": 0,
         "time_zone": "+01:00", "value_format": N.FORMAT_DATE_TIME, "format": "strict_date_optional_time||epoch_millis",
         "buckets": [{"key": hour, "doc_count": 300}],
         "sub_specs": [], "empty_subs": []}
    got = _wire([h])
    fmt = "strict_date_optional_time||epoch_millis".encode()
    want = (b"\x01" + b"\x06dhisto" + b"\x01h\xff\x00"
            + b"\x0edate_histogram" + b"\x01" + b"\x00"                 # factory type, KEY_ASC id 1, minDocCount 0
            + b"\x08" + b"\x01\x06\x06+01:00" + struct.pack(">q", -1800000)  # OffsetRounding(TimeUnitRounding(HOUR, tz))
            + b"\x00"                                                   # empty sub-aggregations
            + b"\x01" + b"\x01" + struct.pack(">q", 0) + b"\x00"        # ExtendedBounds(min 0, max null)
            + b"\x01\x02" + bytes([len(fmt)]) + fmt + b"\x06+01:00"     # ValueFormatter.DateTime(pattern, zone)
            + b"\x00" + b"\x01" + struct.pack(">q", hour) + b"\xac\x02" + b"\x00")
    assert got == want


def test_cardinality_bytes_by_hand():
    regs = bytes(range(16))
    got = _wire([RS.cardinality("c", 4, registers=regs), RS.cardinality("l", 4, lc=[7, 3]), RS.cardinality("e", 4)])
    want = (b"\x03"
            + b"\x0bcardinality" + b"\x01c\xff\x00" + b"\x01\x01" + b"\x01" + b"\x04" + b"\x01" + regs
            + b"\x0bcardinality" + b"\x01l\xff\x00" + b"\x01\x01" + b"\x01" + b"\x04" + b"\x00" + b"\x02"
            + struct.pack(">ii", 3, 7)
            + b"\x0bcardinality" + b"\x01e\xff\x00" + b"\x01\x01" + b"\x00")
    assert got == want


def test_vlong_and_string_encodings():
    # vLong of 2^35 + 1 and a name outside the BMP (a surrogate pair: two Java chars, 3 bytes each)
    got = _wire([{"type": N.AGG_AVG, "name": "r\U0001F600", "count": (1 << 35) + 1, "sum": 0.0}])
    s = ES.StreamInput(got)
    assert s.vint() == 1 and s.bytes_ref() == b"avg"
    assert s.raw(1) == b"\x03"  # 3 chars: 'r' + two surrogates
    assert s.raw(7) == b"r\xed\xa0\xbd\xed\xb8\x80"
    out = ES.decode(got)
    assert out[0]["name"] == "r\U0001F600" and out[0]["count"] == (1 << 35) + 1


WIRE_SHAPES = {
    "north_star": lambda: [AB.terms("hosts").field("host").size(5).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(
            AB.stats("rt").field("response_time_ms")))],
    "config2_dst": lambda: [AB.dateHistogram("d").field("@timestamp").interval("1d").timeZone("Europe/Amsterdam")
                            .offset("+2h").subAggregation(AB.extendedStats("x").field("response_time_ms").sigma(1.5))],
    "histogram_bounds": lambda: [AB.histogram("b").field("bytes").interval(100000).offset(5)
                                 .extendedBounds(-200000, 1200000).subAggregation(AB.avg("a").field("response_time_ms"))],
    "terms_term_order_err": lambda: [AB.terms("h").field("host").size(3).order(Order.term(False))
                                     .showTermDocCountError(True).subAggregation(AB.avg("a").field("price"))],
    "terms_agg_order": lambda: [AB.terms("h").field("host").size(4).order(Order.aggregation("rt.max", True))
                                .subAggregation(AB.stats("rt").field("response_time_ms"))],
    "fixed_tz_interval": lambda: [AB.dateHistogram("m").field("@timestamp").interval("90m").timeZone("-03:30")
                                  .minDocCount(1).order(N.ORDER_HCOUNT_DESC)],
    "date_format": lambda: [AB.dateHistogram("y").field("@timestamp").interval("month").format("yyyy-MM"),
                            AB.stats("ts").field("@timestamp")],
}


@pytest.mark.parametrize("shape", sorted(WIRE_SHAPES))
def test_writer_matches_oracle_writer(shape):
    aggs = WIRE_SHAPES[shape]()
    fields = ("host", "@timestamp", "response_time_ms", "bytes", "status", "price")
    shards = [(synthetic_columns(fields, 20000, shard=s), 20000) for s in range(2)]
    want = O.run(shards, aggs, streams=True)
    for s in range(2):
        insts = RS.from_shard_json(aggs, want["shards"][s], number_of_shards=2)
        got = ShardResult.deserialize(RS.encode(insts)).to_stream()
        ES.decode(got)  # well-formed, nothing trailing
        assert got == want["streams"][s], (shape, s, ES.decode(got), ES.decode(want["streams"][s]))
