"""GPU parity of cardinality under bucket aggregations (CardinalityAggregator with one HyperLogLogPlusPlus sketch per
bucket ordinal, default precision 14 - 5 per multi-bucket ancestor, CardinalityAggregatorFactory.java:65-78; SURVEY
§8(a) a17-a20).  Each bucket independently ends in LINEAR_COUNTING (exact set of encoded hashes) or HYPERLOGLOG
(registers); both are compared bit-exactly, as is the reduced value.
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import QueryBuilders as QB
from elasticsearch_amd import reduce
from helpers import assert_same, synthetic_columns
from test_gpu_multivalued import segment

pytestmark = pytest.mark.gpu


def check_synthetic(engine, aggs, fields, n, filters=None):
    cols = synthetic_columns(fields, n)
    want = O.run([(cols, n)], aggs, filters=filters)
    seg = engine.synthetic_segment(n, fields=fields)
    plan = engine.plan(aggs, filters=filters)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")
    plan.close()
    seg.close()
    return want["reduced"]


def test_terms_cardinality_default_precision(engine):  # p = 9 under one bucket level: head hosts HLL, tail hosts LC
    aggs = [AB.terms("hosts").field("host").size(1000).subAggregation(AB.cardinality("ips").field("client_ip.hash"))]
    r = check_synthetic(engine, aggs, ("host", "client_ip.hash"), 1_000_000)
    modes = {b["ips"]["_internal"]["mode"] for b in r["hosts"]["buckets"]}
    assert modes == {"lc", "hll"}


def test_date_histogram_cardinality_and_stats(engine):
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("1d")
            .subAggregation(AB.cardinality("ips").field("client_ip.hash").precisionThreshold(3000))
            .subAggregation(AB.stats("rt").field("response_time_ms"))
            .subAggregation(AB.cardinality("hosts").field("host"))]
    check_synthetic(engine, aggs, ("@timestamp", "client_ip.hash", "response_time_ms", "host"), 1_200_000)


def test_nested_two_levels_with_filter(engine):  # p = 4 default two bucket levels down
    aggs = [AB.terms("hosts").field("host").size(8).subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("6h").subAggregation(AB.cardinality("ips").field("client_ip.hash")))]
    check_synthetic(engine, aggs, ("host", "@timestamp", "client_ip.hash", "status"), 800_000,
                    filters=[QB.termQuery("status", 200)])


def test_multi_valued_bucket_cardinality(engine):
    cols = segment(300_000, 9)
    lookup = {t: i for i, t in enumerate(cols["tags"]["terms"])}
    aggs = [AB.terms("tags").field("tags").size(30).subAggregation(AB.cardinality("codes").field("codes")),
            AB.dateHistogram("d").field("dates").interval("1d").subAggregation(
                AB.cardinality("p").field("prices").precisionThreshold(200)).subAggregation(AB.cardinality("t").field("tags"))]
    want = O.run([(cols, 300_000)], aggs, ord_lookup=lambda f, t: lookup.get(t, -1))
    seg = engine.upload_segment(cols, 300_000)
    plan = engine.plan(aggs)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard", False)
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced", False)
    plan.close()
    seg.close()


def test_bucket_cardinality_across_segments_and_shards(engine):
    """Two segments into one plan (sketches accumulate per bucket across segments; a bucket that passes the threshold
    in the second segment upgrades) and a two-shard reduce (InternalCardinality.doReduce merges per bucket)."""
    fields = ("host", "client_ip.hash")
    n = 400_000
    aggs = [AB.terms("hosts").field("host").size(50).subAggregation(AB.cardinality("ips").field("client_ip.hash"))]
    parts = [synthetic_columns(fields, n, shard=k) for k in (0, 1)]
    one = {f: {**parts[0][f], "values": np.concatenate([parts[0][f]["values"], parts[1][f]["values"]])} for f in fields}
    want_one = O.run([(one, 2 * n)], aggs)
    segs = [engine.synthetic_segment(n, fields=fields, shard=k) for k in (0, 1)]
    plan = engine.plan(aggs)
    for sg in segs:
        plan.collect(sg)
    assert_same(plan.build().to_dict(), want_one["shards"][0], "two segments")
    plan.close()
    want = O.run([(parts[0], n), (parts[1], n)], aggs)
    shards = []
    for sg in segs:
        pl = engine.plan(aggs, number_of_shards=2)
        pl.collect(sg)
        shards.append(pl.build())
        pl.close()
    assert_same(reduce(shards).to_dict(), want["reduced"], "two shards")
    for sg in segs:
        sg.close()
