"""XContent rendering of shard / reduced results: esgpu_result_to_xcontent writes the search
response's "aggregations" object the way Elasticsearch's XContentBuilder (Jackson, compact) does.

Pinned against the reference where its tests hold the strings:
  * date_histogram key_as_string in the request's time zone -- DateHistogramTests.testDSTBoundaryIssue9491 (year in
    Asia/Jerusalem: "2014-01-01T00:00:00.000+02:00") and testIssue8209 (months in CET across the DST change,
    min_doc_count 0: "+01:00" x 3 then "+02:00"), plugins/lang-groovy/src/test/java/org/elasticsearch/messy/tests/
    DateHistogramTests.java:1335-1372;
  * the ExtendedStats values of AbstractNumericTestCase (1..10): count 10, sum 55, min 1, max 10, avg 5.5,
    sum_of_squares 385, variance 8.25 (ExtendedStatsTests.java:128);
  * the field order of each class's doXContentBody (InternalTerms.java:220-229, StringTerms.java:138-148,
    InternalHistogram.java:152-173 / 526-541, InternalStats.java:206-221, InternalExtendedStats.java:192-213,
    InternalAvg.java:109-115, InternalCardinality.java:129-136).
Double.toString layout (plain decimal for 1e-3 <= |v| < 1e7, else d.dddE<n>) is pinned by the JDK's documented
examples; the digit strings are the shortest round-trip ones (JDK 19+ exactly).
"""
import json

import pytest

from elasticsearch_amd import ShardResult
from elasticsearch_amd import _native as N
from elasticsearch_amd.aggs import tz_history
import result_stream as RS


def _render(aggs):
    return ShardResult.deserialize(RS.encode(aggs)).to_xcontent()


def _stats(name, count, sum_, mn, mx, sumsq=0.0, ext=False, sigma=2.0):
    return {"type": N.AGG_EXTENDED_STATS if ext else N.AGG_STATS, "name": name, "count": count, "sum": sum_, "min": mn,
            "max": mx, "sumsq": sumsq, "sigma": sigma}


@pytest.mark.parametrize("v, java", [
    (1.0, "1.0"), (100.0, "100.0"), (5.5, "5.5"), (0.1, "0.1"), (0.001, "0.001"), (1.0e-4, "1.0E-4"),
    (1234567.0, "1234567.0"), (9999999.0, "9999999.0"), (1.0e7, "1.0E7"), (12345678.9, "1.23456789E7"),
    (-2.5, "-2.5"), (-0.0, "-0.0"), (1.0 / 3.0, "0.3333333333333333"), (2.0 / 3.0, "0.6666666666666666"),
    (1.0e21, "1.0E21"), (1.7976931348623157e308, "1.7976931348623157E308"), (4.9e-324, "4.9E-324"),
    (123.456, "123.456"), (0.00123, "0.00123"), (3.0e-3, "0.003"),
])
def test_double_layout(v, java):
    out = _render([_stats("s", 1, v, v, v)])
    assert out == '{"s":{"count":1,"min":%s,"max":%s,"avg":%s,"sum":%s}}' % (java, java, java, java)


def test_extended_stats_of_the_reference_fixture():
    vals = list(range(1, 11))
    out = json.loads(_render([_stats("x", 10, 55.0, 1.0, 10.0, float(sum(v * v for v in vals)), ext=True)]))["x"]
    assert list(out) == ["count", "min", "max", "avg", "sum", "sum_of_squares", "variance", "std_deviation",
                         "std_deviation_bounds"]
    assert (out["count"], out["sum"], out["min"], out["max"], out["avg"]) == (10, 55.0, 1.0, 10.0, 5.5)
    assert (out["sum_of_squares"], out["variance"]) == (385.0, 8.25)
    assert list(out["std_deviation_bounds"]) == ["upper", "lower"]


def test_empty_metrics_render_null():
    out = _render([_stats("s", 0, 0.0, float("inf"), float("-inf"), ext=True),
                   {"type": N.AGG_AVG, "name": "a", "count": 0, "sum": 0.0}])
    assert out == ('{"s":{"count":0,"min":null,"max":null,"avg":null,"sum":null,"sum_of_squares":null,"variance":null,'
                   '"std_deviation":null,"std_deviation_bounds":{"upper":null,"lower":null}},"a":{"value":null}}')


def test_terms_with_sub_aggregations_field_order():
    agg = {"type": N.AGG_TERMS, "name": "hosts", "other_doc_count": 7, "doc_count_error": 0, "show_err": 1,
           "buckets": [{"term": "a\"b\n", "key": 0, "doc_count": 5, "doc_count_error": 2,
                        "subs": [{"type": N.AGG_AVG, "name": "rt", "count": 2, "sum": 3.0}]}]}
    assert _render([agg]) == ('{"hosts":{"doc_count_error_upper_bound":0,"sum_other_doc_count":7,"buckets":'
                              '[{"key":"a\\"b\\n","doc_count":5,"doc_count_error_upper_bound":2,"rt":{"value":1.5}}]}}')


def _date_histogram(keys, counts, zone, keyed=0, name="histo"):
    starts, offs = zone
    return {"type": N.AGG_DATE_HISTOGRAM, "name": name, "keyed": keyed, "date_unit": N.UNIT_MONTH,
            "tz_starts": list(starts), "tz_offs": list(offs),
            "buckets": [{"key": k, "doc_count": c} for k, c in zip(keys, counts)]}


def test_key_as_string_in_the_request_time_zone_dst_boundary_issue_9491():
    # 2014-01-01T00:00:00+02:00 (Asia/Jerusalem) = 2013-12-31T22:00:00Z
    out = json.loads(_render([_date_histogram([1388527200000], [2], tz_history("Asia/Jerusalem"))]))
    assert out["histo"]["buckets"][0]["key_as_string"] == "2014-01-01T00:00:00.000+02:00"


def test_key_as_string_across_a_dst_change_issue_8209():
    keys = [1388530800000, 1391209200000, 1393628400000, 1396303200000]  # 2014-01/02/03/04-01T00:00 in CET
    out = json.loads(_render([_date_histogram(keys, [1, 0, 0, 2], tz_history("CET"))]))
    assert [b["key_as_string"] for b in out["histo"]["buckets"]] == [
        "2014-01-01T00:00:00.000+01:00", "2014-02-01T00:00:00.000+01:00", "2014-03-01T00:00:00.000+01:00",
        "2014-04-01T00:00:00.000+02:00"]
    assert [b["doc_count"] for b in out["histo"]["buckets"]] == [1, 0, 0, 2]


def test_utc_fixed_offset_and_keyed_histograms():
    utc = _date_histogram([1441065600000], [3], ((), ()), name="u")
    fixed = _date_histogram([1441062000000], [3], ((0,), (3600000,)), name="f")
    keyed = {"type": N.AGG_HISTOGRAM, "name": "h", "keyed": 1, "buckets": [{"key": 50, "doc_count": 1}]}
    out = _render([utc, fixed, keyed])
    assert out == ('{"u":{"buckets":[{"key_as_string":"2015-09-01T00:00:00.000Z","key":1441065600000,"doc_count":3}]},'
                   '"f":{"buckets":[{"key_as_string":"2015-09-01T00:00:00.000+01:00","key":1441062000000,"doc_count":3}]},'
                   '"h":{"buckets":{"50":{"key":50,"doc_count":1}}}}')


def test_fixed_zone_is_kept_for_printing():
    """aggs.py passes a fixed zone as a one-entry table (folded into the rounding offset by the library), so the
    result still knows the zone for key_as_string."""
    from elasticsearch_amd import AggregationBuilders as AB
    from elasticsearch_amd.aggs import flatten
    arr, n, _keep = flatten([AB.dateHistogram("d").field("t").interval("1d").timeZone("+01:00")])
    assert arr[0].tz_count == 1 and arr[0].tz_offsets_ms[0] == 3600000 and arr[0].offset == 0
