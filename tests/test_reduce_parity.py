"""CPU parity of the product's shard-level reduce (esgpu_reduce) and JSON rendering against the oracle, per request
shape, without a GPU.

The oracle collects several synthetic shards and reduces them the way the coordinating node does
(InternalAggregations.reduce).  Its shard-level results are re-encoded into the library's stream format
(tests/result_stream.py), decoded by esgpu_result_deserialize, rendered back (must equal the oracle's shard JSON),
and reduced by esgpu_reduce (must equal the oracle's reduced JSON).  This covers terms error bounds / other counts,
histogram empty-bucket filling with prototypes, order variants and nested sub-aggregation reduce at every level.
"""
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, ShardResult, reduce
from helpers import assert_same, synthetic_columns
from result_stream import encode, from_shard_json

DOCS = 12_000
DAY = 86_400_000
T0 = 1441065600000


def _ns(metric):
    return [AB.terms("hosts").field("host").size(10).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(metric))]


CASES = {
    "north_star": (_ns(AB.stats("rt").field("response_time_ms")), ("host", "@timestamp", "response_time_ms")),
    "config5_avg": (_ns(AB.avg("rt").field("response_time_ms")), ("host", "@timestamp", "response_time_ms")),
    "config2_ext_bounds": ([AB.dateHistogram("h").field("@timestamp").interval("1h").minDocCount(0)
                            .extendedBounds(T0 - DAY, T0 + 2 * DAY)
                            .subAggregation(AB.extendedStats("rt").field("response_time_ms").sigma(3.0))],
                           ("@timestamp", "response_time_ms")),
    "hist_terms_mdc0": ([AB.histogram("b").field("bytes").interval(50_000).minDocCount(0)
                         .subAggregation(AB.terms("st").field("status").size(3)
                                         .subAggregation(AB.avg("rt").field("response_time_ms")))],
                        ("bytes", "status", "response_time_ms")),
    "terms_small_shard_size": ([AB.terms("hosts").field("host").size(5).shardSize(6)
                                .showTermDocCountError(True)], ("host",)),
    "terms_count_asc": ([AB.terms("hosts").field("host").size(7).order(Order.count(True))], ("host",)),
    "terms_term_desc": ([AB.terms("hosts").field("host").size(7).order(Order.term(False))], ("host",)),
    "hist_key_desc": ([AB.histogram("rt").field("response_time_ms").interval(25).order(Order.KEY_DESC)
                       .subAggregation(AB.stats("b").field("bytes"))], ("response_time_ms", "bytes")),
    "hist_count_asc": ([AB.histogram("rt").field("response_time_ms").interval(100).order(Order.COUNT_ASC)],
                       ("response_time_ms",)),
    "day_hist_terms": ([AB.dateHistogram("d").field("@timestamp").interval("1d")
                        .subAggregation(AB.terms("hosts").field("host").size(4))], ("@timestamp", "host")),
    # lattice merge (dense slots) vs k-way merge fallbacks: calendar months (gaps of 28-31 days: a 1-day lattice too
    # sparse for the slot array), a sparse wide histogram, and an offset histogram with a non-integer-valued metric
    "month_hist_stats": ([AB.dateHistogram("m").field("@timestamp").interval("month")
                          .subAggregation(AB.stats("rt").field("response_time_ms"))], ("@timestamp", "response_time_ms")),
    "sparse_wide_hist": ([AB.histogram("b").field("bytes").interval(7).minDocCount(1)
                          .subAggregation(AB.avg("rt").field("response_time_ms"))], ("bytes", "response_time_ms")),
    "offset_hist_price": ([AB.histogram("p").field("price").interval(10).offset(3)
                           .subAggregation(AB.extendedStats("x").field("price"))], ("price",)),
    # lattice reduce with metric leaves streamed per shard run: a count order permutes the emitted buckets, and
    # min_doc_count >= 2 drops slots, so a shard's run of slots may map to non-consecutive buckets
    "hist_count_desc_stats": ([AB.histogram("rt").field("response_time_ms").interval(50).order(Order.COUNT_DESC)
                               .subAggregation(AB.stats("b").field("bytes"))], ("response_time_ms", "bytes")),
    "hist_count_asc_ext": ([AB.histogram("b").field("bytes").interval(20_000).order(Order.COUNT_ASC)
                            .subAggregation(AB.extendedStats("rt").field("response_time_ms"))],
                           ("bytes", "response_time_ms")),
    "sparse_hist_mdc2_stats": ([AB.histogram("b").field("bytes").interval(7).minDocCount(2)
                                .subAggregation(AB.stats("rt").field("response_time_ms"))], ("bytes", "response_time_ms")),
    "sparse_hist_mdc3_avg_desc": ([AB.histogram("b").field("bytes").interval(11).minDocCount(3).order(Order.KEY_DESC)
                                   .subAggregation(AB.avg("rt").field("response_time_ms"))],
                                  ("bytes", "response_time_ms")),
    "top_metrics": ([AB.stats("s").field("response_time_ms"), AB.extendedStats("e").field("bytes"),
                     AB.avg("a").field("response_time_ms")], ("response_time_ms", "bytes")),
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("nshards", [1, 3])
def test_reduce_matches_oracle(name, nshards):
    aggs, fields = CASES[name]
    shards = [(synthetic_columns(fields, DOCS + 997 * s, shard=s), DOCS + 997 * s) for s in range(nshards)]
    want = O.run(shards, aggs, number_of_shards=nshards)
    results = []
    for s, sj in enumerate(want["shards"]):
        r = ShardResult.deserialize(encode(from_shard_json(aggs, sj, nshards)))
        assert_same(r.to_dict(), sj, f"shard{s}")  # columnar blocks render the reference's shard JSON
        results.append(r)
    assert_same(reduce(results).to_dict(), want["reduced"], "reduced")
    # the reduce consumed the shard results read-only: reducing again gives the same answer
    assert reduce(results).to_json() == reduce(results).to_json()


def test_reduce_rejects_mismatched_trees():
    a = encode(from_shard_json([AB.stats("x").field("f")], {"x": {"_internal": {"count": 1, "sum": 2.0, "min": 2.0,
                                                                                  "max": 2.0}}}))
    b = encode([{"type": 1, "name": "x", "buckets": []}])
    from elasticsearch_amd import _native as N
    with pytest.raises(N.EsGpuError):
        reduce([ShardResult.deserialize(a), ShardResult.deserialize(b)])


@pytest.mark.parametrize("path,asc", [("rt.avg", False), ("a", True), ("x.std_upper", True), ("x.count", False),
                                      ("rt.min", True)])
def test_reduce_terms_ordered_by_a_metric(path, asc):
    """InternalTerms.doReduce with InternalOrder.Aggregation: the reduced sub-aggregation's value orders the merged
    buckets (NaN last), ties by term; doc_count_error is -1 (not a count-desc order).  Shard results come from the
    oracle (its shard-level GlobalOrdinalsStringTermsAggregator selection by metric(name, bucketOrd))."""
    from elasticsearch_amd import Order
    from helpers import synthetic_columns
    from result_stream import from_shard_json
    aggs = [AB.terms("hosts").field("host").size(6).order(Order.aggregation(path, asc))
            .subAggregation(AB.stats("rt").field("response_time_ms")).subAggregation(AB.avg("a").field("bytes"))
            .subAggregation(AB.extendedStats("x").field("response_time_ms"))]
    fields = ("host", "response_time_ms", "bytes")
    shards = [(synthetic_columns(fields, 100_000, shard=s), 100_000) for s in range(3)]
    want = O.run(shards, aggs, number_of_shards=3)
    blobs = [encode(from_shard_json(aggs, want["shards"][s], 3)) for s in range(3)]
    got = reduce([ShardResult.deserialize(b) for b in blobs]).to_dict()
    assert_same(got, want["reduced"], "reduced")
    assert got["hosts"]["doc_count_error_upper_bound"] == -1


def _cols(b, rt):
    from elasticsearch_amd import _native as N
    import numpy as np
    return {"bytes": {"type": N.COL_I64, "values": np.asarray(b, dtype=np.int64)},
            "response_time_ms": {"type": N.COL_I64, "values": np.asarray(rt, dtype=np.int64)}}


@pytest.mark.parametrize("shape", ["mdc2_gap", "count_desc", "count_asc_gap"])
def test_lattice_reduce_runs_with_permuted_or_dropped_slots(shape):
    """A shard's run of histogram slots streamed into its buckets (the lattice reduce's metric leaves) must land on the
    right buckets when the ends of the run are len - 1 buckets apart but its middle is not: a slot dropped by
    min_doc_count (shard A holds keys 0, 7, 21; key 7 totals 1 doc) or a count order that permutes the emitted buckets."""
    if shape == "mdc2_gap":
        a = _cols([0, 0, 7, 21, 21], [1, 2, 1000, 5, 6])
        b = _cols([0, 14, 14, 21], [3, 40, 50, 7])
        agg = AB.histogram("b").field("bytes").interval(7).minDocCount(2)
    elif shape == "count_desc":
        # totals: key 0 -> 6, key 7 -> 2, key 14 -> 4, key 21 -> 1: count-desc order 0, 14, 7, 21 (out = 0, 2, 1, 3)
        a = _cols([0, 0, 0, 7, 14, 14, 21], [1, 2, 3, 1000, 9, 8, 77])
        b = _cols([0, 0, 0, 7, 14, 14], [4, 5, 6, 2000, 10, 11])
        agg = AB.histogram("b").field("bytes").interval(7).order(Order.COUNT_DESC)
    else:
        a = _cols([0, 7, 7, 7, 21, 21], [1, 500, 600, 700, 5, 6])
        b = _cols([0, 14, 14, 21, 28, 28, 28, 28], [3, 40, 50, 7, 1, 1, 1, 1])
        agg = AB.histogram("b").field("bytes").interval(7).order(Order.COUNT_ASC)
    aggs = [agg.subAggregation(AB.stats("s").field("response_time_ms"))
            .subAggregation(AB.extendedStats("x").field("response_time_ms"))]
    shards = [(a, 5 if shape == "mdc2_gap" else len(a["bytes"]["values"])), (b, len(b["bytes"]["values"]))]
    want = O.run(shards, aggs, number_of_shards=2)
    blobs = [encode(from_shard_json(aggs, want["shards"][s], 2)) for s in range(2)]
    assert_same(reduce([ShardResult.deserialize(x) for x in blobs]).to_dict(), want["reduced"], "reduced")
