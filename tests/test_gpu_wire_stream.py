"""GPU: the transport bytes of shard results collected on the gfx950 path (esgpu_result_to_stream) against the oracle's
own restatement of InternalAggregations.writeTo over its shard results for the same seeded columns.

Byte-identical for every case without a LINEAR_COUNTING sketch (the metrics here are integer-valued, so their sums are
exact on both sides).  A LINEAR_COUNTING sketch's hashes are written in the reference's hash-table slot order by the
oracle and ascending by the product -- a permutation that HyperLogLogPlusPlus.readFrom turns back into the same set
(HyperLogLogPlusPlus.java:537-547) -- so those cases compare the decoded streams with the hash lists sorted.
"""
import pytest

import oracle as O
import es_stream as ES
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import QueryBuilders as QB
from helpers import synthetic_columns

pytestmark = pytest.mark.gpu


def _compare(engine, aggs, fields, n, filters=None, shard=0):
    cols = synthetic_columns(fields, n, shard=shard)
    want = O.run([(cols, n)], aggs, filters=filters, streams=True)["streams"][0]
    seg = engine.synthetic_segment(n, fields=fields, shard=shard)
    plan = engine.plan(aggs, filters=filters)
    plan.collect(seg)
    got = plan.build().to_stream()
    plan.close()
    seg.close()
    g, w = ES.decode(got), ES.decode(want)
    assert got == want, (g, w)  # LINEAR_COUNTING hash lists in the reference's Hashset slot order
    return g


def test_wire_north_star(engine):
    aggs = [AB.terms("hosts").field("host").size(10).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("response_time_ms")))]
    out = _compare(engine, aggs, ("host", "@timestamp", "response_time_ms"), 1_000_000)
    assert out[0]["stream_type"] == "sterms" and out[0]["buckets"][0]["aggs"][0]["stream_type"] == "dhisto"


def test_wire_config4_hll_and_lc(engine):
    aggs = [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000),
            AB.cardinality("st").field("status").precisionThreshold(100)]
    out = _compare(engine, aggs, ("client_ip.hash", "status"), 2_000_000)
    assert out[0]["mode"] == "hll" and out[0]["precision"] == 18
    assert out[1]["mode"] == "lc" and len(out[1]["lc"]) == 10


def test_wire_cardinality_under_terms(engine):
    aggs = [AB.terms("hosts").field("host").size(5).subAggregation(AB.cardinality("ips").field("client_ip.hash"))]
    _compare(engine, aggs, ("host", "client_ip.hash"), 400_000)


def test_wire_config5_filters_dst(engine):
    aggs = [AB.terms("hosts").field("host").subAggregation(
        AB.dateHistogram("d").field("@timestamp").interval("1d").timeZone("America/New_York").subAggregation(
            AB.avg("rt").field("response_time_ms")))]
    filters = [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)]
    _compare(engine, aggs, ("host", "@timestamp", "response_time_ms", "status", "bytes"), 600_000, filters=filters)


def test_wire_filter_aggregation(engine):
    # response_time_ms < 1000: every sum of squares stays below 2^53, exact in any order (bytes' would not)
    aggs = [AB.filter("ok", QB.termQuery("status", 200)).subAggregation(AB.extendedStats("b").field("response_time_ms")),
            AB.histogram("rt").field("response_time_ms").interval(50).extendedBounds(0, 2000)]
    _compare(engine, aggs, ("status", "bytes", "response_time_ms"), 500_000)


def test_wire_config3_high_cardinality(engine):
    aggs = [AB.terms("urls").field("url").size(10)]
    _compare(engine, aggs, ("url",), 2_000_000, shard=1)
