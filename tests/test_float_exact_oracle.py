"""The oracle's exact-sum shadow (oracle.run(..., exact=True)) pinned against math.fsum, and the parity helper that
uses it (helpers.assert_same_exact).

SURVEY §7 "Float parity": the reference adds doubles in doc order, so its sums of non-integer values (and of integers
past 2^53) carry its own rounding error, which grows like sqrt(n) * 2^-53.  The GPU's compensated sums are checked
against the exact value (and the oracle's own error recorded) rather than against that rounding.  The shadow is a
double-double accumulation; here it must agree with math.fsum (correctly rounded) on every bucket, including
cancellation, subnormals, sums of squares past 2^53 and non-finite values (IEEE: NaN, or +Inf with -Inf, is NaN).
"""
import math

import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import _native as N
from helpers import FloatReport, assert_same_exact, strip_exact

DISTS = ["uniform", "cancel", "subnormal", "bigint", "lognormal"]


def _values(kind, n, rng):
    if kind == "uniform":
        return rng.random(n) * 1e3
    if kind == "cancel":  # large opposite values and small ones: sum |v| >> |sum|
        v = rng.standard_normal(n) * 1e10
        v[1::2] = -v[0::2][: n // 2] + rng.random(n // 2) * 1e-3
        return v
    if kind == "subnormal":
        return (rng.random(n) - 0.25) * 2.0 ** -1030
    if kind == "bigint":  # squares up to 1e14, sums of squares past 2^53
        return rng.integers(0, 10_000_000, size=n).astype(np.float64)
    return np.exp(rng.standard_normal(n) * 3.0)


@pytest.mark.parametrize("kind", DISTS)
def test_shadow_matches_fsum(kind):
    rng = np.random.default_rng(DISTS.index(kind) + 7)
    n = 200_000
    v = _values(kind, n, rng)
    keys = rng.integers(0, 37, size=n) * 10
    cols = {"price": {"type": N.COL_F64, "values": v}, "k": {"type": N.COL_I64, "values": keys.astype(np.int64)}}
    aggs = [AB.extendedStats("x").field("price"),
            AB.histogram("h").field("k").interval(10).subAggregation(AB.extendedStats("e").field("price"))]
    r = O.run([(cols, n)], aggs, exact=True)["reduced"]
    ex = r["x"]["_exact"]
    assert ex["sum"] == math.fsum(v)
    assert ex["sum_of_squares"] == math.fsum(v * v)
    for b in r["h"]["buckets"]:
        sel = v[keys == b["key"]]
        assert b["e"]["_exact"]["sum"] == math.fsum(sel), b["key"]
        assert b["e"]["_exact"]["sum_of_squares"] == math.fsum(sel * sel), b["key"]
        assert b["e"]["_exact"]["avg"] == math.fsum(sel) / len(sel)


def test_shadow_non_finite():
    def run(vals):
        v = np.array(vals, dtype=np.float64)
        cols = {"price": {"type": N.COL_F64, "values": v}}
        return O.run([(cols, len(v))], [AB.stats("s").field("price")], exact=True)["reduced"]["s"]["_exact"]["sum"]
    assert run([1.0, math.inf, 2.0]) == math.inf
    assert run([1.0, -math.inf]) == -math.inf
    assert math.isnan(run([math.inf, 3.0, -math.inf]))
    assert math.isnan(run([1.0, math.nan, 2.0]))
    assert run([2.0 ** -1074] * 5) == 5 * 2.0 ** -1074


def test_shadow_reduce_is_exact_over_shards():
    """The reduce merges the shards' shadows exactly (the reference reduce adds the shards' rounded sums in order)."""
    rng = np.random.default_rng(3)
    shards, allv = [], []
    for s in range(3):
        v = _values("lognormal", 50_000 + s, rng)
        allv.append(v)
        shards.append(({"price": {"type": N.COL_F64, "values": v}}, len(v)))
    r = O.run(shards, [AB.avg("a").field("price")], exact=True)
    assert r["reduced"]["a"]["_exact"]["_internal"]["sum"] == math.fsum(np.concatenate(allv))


def test_assert_same_exact_rules():
    rng = np.random.default_rng(5)
    v = rng.random(100_000) * 1e3
    cols = {"price": {"type": N.COL_F64, "values": v}}
    want = O.run([(cols, len(v))], [AB.extendedStats("x").field("price")], exact=True)["reduced"]
    exact_tree = {"x": dict(strip_exact(want)["x"])}
    for k, val in want["x"]["_exact"].items():
        if not isinstance(val, dict):
            exact_tree["x"][k] = val
    exact_tree["x"]["_internal"] = dict(exact_tree["x"]["_internal"], **want["x"]["_exact"]["_internal"])
    rep = FloatReport()
    # a result equal to the exact values passes, and the oracle's own error is recorded
    assert_same_exact(exact_tree, want, "x", exact_floats=False, report=rep)
    assert rep.as_dict()["max_rel_err_gpu_vs_exact"]["sum"] == 0.0
    assert rep.as_dict()["max_rel_err_oracle_vs_exact"]["sum"] > 0.0
    # a sum 1e-11 off the exact value fails
    bad = {"x": dict(exact_tree["x"], sum=exact_tree["x"]["sum"] * (1 + 1e-11))}
    with pytest.raises(AssertionError):
        assert_same_exact(bad, want, "x", exact_floats=False)
