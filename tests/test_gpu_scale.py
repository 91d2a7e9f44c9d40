"""GPU parity at the scales the bench claims ("parity at scale").

Every case runs the full synthetic workload shape through the C-ABI and through the oracle on the same seeded columns,
generated on the host with all the job's threads:
  * config 4: cardinality(client_ip.hash, precision_threshold 40000) at 160M docs.  At p = 18 the register kernel's
    phases after the first run with a non-zero register floor, i.e. the zero-mask rejection + LDS nibble snapshot path
    that does the work at 1B docs; registers (FNV-1a over 2^18 bytes), mode and estimate must be bit-exact.
  * config 3: terms(url, 10M global ordinals) at its BASELINE shard size, 125M docs, shard_size 80 (8 shards).
  * north star and config 5 at 200M / 120M docs (the LDS key window slides over ~720 hours).
"""
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import QueryBuilders as QB
from elasticsearch_amd import reduce
from helpers import assert_same, synthetic_columns

pytestmark = pytest.mark.gpu


def _compare(engine, aggs, fields, n, filters=None, number_of_shards=1, shard=0):
    cols = synthetic_columns(fields, n, shard=shard)
    want = O.run([(cols, n)], aggs, filters=filters, number_of_shards=number_of_shards)
    del cols
    seg = engine.synthetic_segment(n, fields=fields, shard=shard)
    plan = engine.plan(aggs, filters=filters, number_of_shards=number_of_shards)
    plan.collect(seg)
    res = plan.build()
    got = res.to_dict()
    assert_same(got, want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")
    plan.close()
    seg.close()
    return got


def test_config4_cardinality_160m(engine):
    aggs = [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)]
    got = _compare(engine, aggs, ("client_ip.hash",), 160_000_000)
    assert got["ips"]["_internal"]["mode"] == "hll"


def test_config3_terms_125m_per_shard(engine):
    aggs = [AB.terms("urls").field("url").size(10)]
    got = _compare(engine, aggs, ("url",), 125_000_000, number_of_shards=8, shard=3)
    assert len(got["urls"]["buckets"]) == 80


def test_north_star_200m(engine):
    aggs = [AB.terms("hosts").field("host").size(10).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("response_time_ms")))]
    got = _compare(engine, aggs, ("host", "@timestamp", "response_time_ms"), 200_000_000)
    assert sum(b["doc_count"] for b in got["hosts"]["buckets"]) + got["hosts"]["sum_other_doc_count"] == 200_000_000


def test_config5_120m(engine):
    aggs = [AB.terms("hosts").field("host").size(10).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.avg("rt").field("response_time_ms")))]
    filters = [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)]
    _compare(engine, aggs, ("status", "bytes", "host", "@timestamp", "response_time_ms"), 120_000_000, filters=filters,
             number_of_shards=8)


def test_config4_shards_merged_into_one_plan(engine):
    """Config 4 as bench.py --shards runs it on one GPU: 4 shards of 40M docs collected into one plan.  From the second
    segment on the register kernel continues the phase sequence with the floor the earlier segments left (no floor-0
    phase); the merged registers must equal the reduce of the per-shard sketches."""
    n, shards = 40_000_000, 4
    fields = ("client_ip.hash",)
    aggs = [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)]
    want = O.run([(synthetic_columns(fields, n, shard=s), n) for s in range(shards)], aggs, number_of_shards=shards)
    plan = engine.plan(aggs, number_of_shards=shards)
    assert plan.shard_mergeable()
    segs = [engine.synthetic_segment(n, fields=fields, shard=s) for s in range(shards)]
    for seg in segs:
        plan.collect(seg)
    got = reduce([plan.build()]).to_dict()
    assert_same(got, want["reduced"], "merged shards")
    assert got["ips"]["_internal"]["mode"] == "hll"
    plan.close()
    for seg in segs:
        seg.close()
