"""GPU parity for terms under a histogram in count orders (date_histogram{terms}, Kibana's split-series chart): each
outer key's terms are selected on the GPU at build (row_topk_kernel: GlobalOrdinalsStringTermsAggregator.buildAggregation
:146-208 once per owning bucket) and only the picks reach the host.  Compared with the oracle at the shard and reduced
levels: count desc / asc, shard_size / size around the term count, min_doc_count 0, shard_min_doc_count, sub-metrics
beside the picks, over the Zipf host field (1,000 terms) and a 3,000-term field with a large shard_size."""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same, synthetic_columns

pytestmark = pytest.mark.gpu

FIELDS = ("@timestamp", "host", "response_time_ms")


def _both(engine, aggs, n=250_000, shards=2, extra=None):
    data = []
    for s in range(shards):
        cols = synthetic_columns(FIELDS, n, shard=s)
        if extra:
            cols.update(extra(s, n))
        data.append((cols, n))
    want = O.run(data, aggs, number_of_shards=shards)
    plan = engine.plan(aggs, number_of_shards=shards)
    results = []
    for s, (cols, _) in enumerate(data):
        seg = engine.upload_segment(cols, n)
        plan.reset()
        plan.collect(seg)
        r = plan.build()
        assert_same(r.to_dict(), want["shards"][s], f"shard{s}")
        results.append(r)
        seg.close()
    assert_same(reduce(results).to_dict(), want["reduced"], "reduced")
    plan.close()


def _dh(inner, interval="1h"):
    return [AB.dateHistogram("t").field("@timestamp").interval(interval).subAggregation(inner)]


@pytest.mark.parametrize("size,shard_size", [(10, None), (1, None), (3, 3), (50, 200), (2000, None)])
def test_count_desc_sizes(engine, size, shard_size):
    t = AB.terms("hosts").field("host").size(size)
    if shard_size:
        t.shardSize(shard_size)
    _both(engine, _dh(t))


def test_count_asc_with_min_doc_counts(engine):
    _both(engine, _dh(AB.terms("hosts").field("host").size(5).order(Order.count(True))
                      .minDocCount(2).shardMinDocCount(3)))


def test_min_doc_count_zero_and_sub_metrics(engine):
    """zero-count terms are candidates (ties by ascending ordinal); the picks' metric cells are gathered beside them"""
    _both(engine, _dh(AB.terms("hosts").field("host").size(20).minDocCount(0)
                      .subAggregation(AB.stats("rt").field("response_time_ms")), interval="6h"))


def test_many_terms_large_shard_size(engine):
    """3,000 terms, shard_size 900: picks far beyond one lane's share of the row"""
    def extra(s, n):
        rng = np.random.default_rng(77 + s)
        v = np.minimum(rng.zipf(1.2, size=n) - 1, 2999).astype(np.uint32)
        return {"kw": {"type": N.COL_ORD_U32, "values": v, "terms": ["w%05d" % i for i in range(3000)]}}
    _both(engine, _dh(AB.terms("w").field("kw").size(600).shardSize(900), interval="1d"), extra=extra)
