"""GPU boundary: error behaviour of the C-ABI (include/esgpu.h status codes) on a real device.

The plugin's contract: a request shape the GPU path does not handle fails with
ESGPU_ERR_UNSUPPORTED at plan create / collect time so the stock Java aggregator runs instead (never a CPU fallback
inside the library), and an allocation over the context's HBM budget fails with ESGPU_ERR_OOM, the analogue of the
REQUEST breaker's CircuitBreakingException (C/common/util/BigArrays.java:393-395).
"""
import pytest

from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Engine, Order
from elasticsearch_amd import _native as N

pytestmark = pytest.mark.gpu


def _plan_and_collect(engine, aggs, fields, n=100_000):
    seg = engine.synthetic_segment(n, fields=fields)
    try:
        plan = engine.plan(aggs)
        try:
            plan.collect(seg)
            plan.build()
        finally:
            plan.close()
    finally:
        seg.close()


@pytest.mark.parametrize("case", ["metric_ordered_terms_under_high_cardinality_terms", "four_bucket_levels",
                                  "three_bucket_levels"])
def test_unsupported_shapes_raise(engine, case):
    if case == "metric_ordered_terms_under_high_cardinality_terms":
        # 1,000 x 10M cells: no dense grid, and a metric order over 10M inner terms is not selected by the replay
        aggs = [AB.terms("hosts").field("host").subAggregation(AB.terms("urls").field("url").order(
            Order.aggregation("rt", True)).subAggregation(AB.avg("rt").field("response_time_ms")))]
        fields = ("host", "url", "response_time_ms")
    elif case == "four_bucket_levels":  # (a calendar inner histogram is collected since round 6: bucket table)
        aggs = [AB.terms("hosts").field("host").subAggregation(AB.terms("urls").field("url").subAggregation(
            AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(
                AB.histogram("b").field("bytes").interval(1024))))]
        fields = ("host", "url", "@timestamp", "bytes")
    else:
        aggs = [AB.terms("hosts").field("host").subAggregation(
            AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(
                AB.histogram("b").field("bytes").interval(1024)))]
        fields = ("host", "@timestamp", "bytes")
    with pytest.raises(N.UnsupportedOnGpu):
        _plan_and_collect(engine, aggs, fields)


def test_engine_usable_after_unsupported(engine):
    with pytest.raises(N.UnsupportedOnGpu):
        _plan_and_collect(engine, [AB.terms("hosts").field("host").subAggregation(
            AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(
                AB.histogram("b").field("bytes").interval(1024)))], ("host", "@timestamp", "bytes"))
    aggs = [AB.terms("hosts").field("host").subAggregation(AB.stats("rt").field("response_time_ms"))]
    seg = engine.synthetic_segment(50_000, fields=("host", "response_time_ms"))
    plan = engine.plan(aggs)
    plan.collect(seg)
    d = plan.build().to_dict()
    assert sum(b["doc_count"] for b in d["hosts"]["buckets"]) + d["hosts"]["sum_other_doc_count"] == 50_000
    plan.close()
    seg.close()


def test_hbm_budget_breaker():
    small = Engine(0, hbm_budget_bytes=1 << 20)  # 1 MB: a 1M-doc segment (4+ MB per column) cannot fit
    try:
        with pytest.raises(N.CircuitBreakingError):
            seg = small.synthetic_segment(1_000_000, fields=("host", "response_time_ms"))
            seg.close()
    finally:
        small.close()
