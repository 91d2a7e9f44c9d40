"""Shared test utilities: synthetic host columns for the oracle, and the parity comparison rules.

Parity bar (BASELINE.json north_star): bucket keys / counts / ordinals / HLL registers bit-exact; floating sums
and averages within 1e-12 relative.  For integer-valued metrics (the synthetic response_time_ms, bytes) every
partial sum is exact, so those comparisons are bit-exact too (`exact_floats=True`).
"""
import math

import numpy as np

from elasticsearch_amd import _native as N
from elasticsearch_amd import synthetic_host_column

REL_TOL = 1e-12
# variance / std_deviation / std_deviation_bounds are derived as (sum_of_squares - sum^2 / count) / count: the subtraction
# cancels, amplifying the 1e-12 relative differences of the two sums (order-dependent rounding of non-integer doubles)
# by sum_of_squares / (count * variance).  They are compared at 1e-9; the sums they come from stay at 1e-12.
DERIVED_TOL = 1e-9
DERIVED_KEYS = ("variance", "std_deviation", "std_deviation_bounds", "upper", "lower")
# Sums past 2^53 (sum_of_squares of a long field such as bytes, sums of a metric with a 10^12 base) and sums of
# non-integer doubles round on every addition, in the reference's doc order and in the GPU's partial sums alike.  Such
# results are checked with an oracle run with exact=True (assert_same_exact): its "_exact" values are the exact sums the
# reference approximates, and the GPU's compensated sums must lie within 1e-12 of them (as of the oracle, unless the
# oracle's own doc-order error is the larger).


def synthetic_dict(field):
    """Term dictionary blob/offsets of a synthetic keyword field (host-%04d / /p/%08x)."""
    if field == "host":
        terms = [b"host-%04d" % i for i in range(1000)]
        blob = np.frombuffer(b"".join(terms), dtype=np.uint8).copy()
        offs = np.arange(0, 9 * 1001, 9, dtype=np.uint64)
        return blob, offs
    if field == "url":
        n = 10_000_000
        ids = np.arange(n, dtype=np.uint64)
        digits = (ids[:, None] >> (np.arange(7, -1, -1, dtype=np.uint64) * 4)) & 15
        hexchars = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)[digits.astype(np.int64)]
        out = np.empty((n, 11), dtype=np.uint8)
        out[:, 0] = ord("/")
        out[:, 1] = ord("p")
        out[:, 2] = ord("/")
        out[:, 3:] = hexchars
        return out.reshape(-1), np.arange(0, 11 * (n + 1), 11, dtype=np.uint64)
    raise KeyError(field)


def _host_column(field, num_docs, shard, seed, threads, ts_jitter_ms=0):
    """synthetic_host_column in `threads` concurrent chunks (the C generator releases the GIL)."""
    if threads <= 1 or num_docs < (1 << 22):
        return synthetic_host_column(field, num_docs, shard=shard, seed=seed, ts_jitter_ms=ts_jitter_ms)
    from concurrent.futures import ThreadPoolExecutor
    bounds = [num_docs * i // threads for i in range(threads + 1)]
    first = synthetic_host_column(field, num_docs, start=0, count=1, shard=shard, seed=seed)
    out = np.empty(num_docs, dtype=first.dtype)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda i: synthetic_host_column(field, num_docs, start=bounds[i], count=bounds[i + 1] - bounds[i],
                                                    shard=shard, seed=seed, ts_jitter_ms=ts_jitter_ms,
                                                    out=out[bounds[i]:bounds[i + 1]]), range(threads)))
    return out


def host_threads():
    """Host threads this job may use: its CPU affinity, capped by OMP_NUM_THREADS (the GPU box allots 16)."""
    import os
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, omp) if omp > 0 else n)


def synthetic_columns(fields, num_docs, shard=0, seed=0x5EEDE1A5, threads=None, ts_jitter_ms=0):
    """Host copies of a synthetic shard, in the column-dict format of Engine.upload_segment / oracle.run."""
    threads = host_threads() if threads is None else threads
    cols = {}
    for f in fields:
        c = {"type": N.SYNTH_TYPES[f], "values": _host_column(f, num_docs, shard, seed, threads, ts_jitter_ms)}
        if f in ("host", "url"):
            c["terms_blob"] = synthetic_dict(f)
        cols[f] = c
    return cols


def _num_equal(a, b, exact, tol=REL_TOL):
    if isinstance(a, bool) or isinstance(b, bool) or a is None or b is None:
        return a == b
    if isinstance(a, int) and isinstance(b, int):
        return a == b
    fa, fb = float(a), float(b)
    if math.isnan(fa) or math.isnan(fb):
        return math.isnan(fa) and math.isnan(fb)
    if math.isinf(fa) or math.isinf(fb) or exact:
        return fa == fb
    return abs(fa - fb) <= tol * max(abs(fa), abs(fb)) or fa == fb


def assert_same(got, want, path="", exact_floats=True):
    """Deep comparison of two parsed result trees with the parity rules above (a metric from an oracle run with
    exact=True is compared through assert_same_exact)."""
    if isinstance(want, dict) and "_exact" in want:
        assert_same_exact(got, want, path, exact_floats)
        return
    if isinstance(want, dict):
        assert isinstance(got, dict), f"{path}: expected object, got {type(got).__name__}"
        assert set(got) == set(want), f"{path}: keys differ: {sorted(set(got) ^ set(want))}"
        for k in want:
            assert_same(got[k], want[k], f"{path}.{k}", exact_floats)
    elif isinstance(want, list):
        assert isinstance(got, list), f"{path}: expected list"
        assert len(got) == len(want), f"{path}: length {len(got)} != {len(want)}"
        for i, (g, w) in enumerate(zip(got, want)):
            assert_same(g, w, f"{path}[{i}]", exact_floats)
    elif isinstance(want, str):
        assert got == want, f"{path}: {got!r} != {want!r}"
    else:
        derived = any(("." + k) in path for k in DERIVED_KEYS)
        tol = DERIVED_TOL if derived else REL_TOL
        ok = _num_equal(got, want, exact_floats, tol)
        if not ok and derived and not exact_floats and isinstance(want, float) and isinstance(got, float):
            # avg +- sigma * std_deviation near zero: the subtraction cancels, so the operands' rounding (relative to
            # their own magnitude, >= 1 here) is what the result carries -- compared against a unit scale
            ok = abs(got - want) <= tol * max(abs(got), abs(want), 1.0)
        assert ok, f"{path}: {got!r} != {want!r}"


def _rel(a, b):
    """Relative difference of two floats (0 when equal, NaN-equal or the same infinity; inf when only one is finite)."""
    fa, fb = float(a), float(b)
    if fa == fb or (math.isnan(fa) and math.isnan(fb)):
        return 0.0
    if not (math.isfinite(fa) and math.isfinite(fb)):
        return math.inf
    return abs(fa - fb) / max(abs(fa), abs(fb))


class FloatReport:
    """Largest relative errors against the exact sums seen by assert_same_exact, per rendered key: the oracle's
    (the reference's doc-order rounding) and the GPU's."""

    def __init__(self):
        self.oracle, self.got, self.n = {}, {}, 0

    def add(self, key, oracle_err, got_err):
        self.n += 1
        self.oracle[key] = max(self.oracle.get(key, 0.0), oracle_err)
        self.got[key] = max(self.got.get(key, 0.0), got_err)

    def as_dict(self):
        return {"values_checked": self.n, "max_rel_err_oracle_vs_exact": self.oracle,
                "max_rel_err_gpu_vs_exact": self.got}


def _exact_leaf(got, want, exact, path, key, exact_floats, report, strict):
    derived = any(("." + k) in path for k in DERIVED_KEYS)
    tol = DERIVED_TOL if derived else REL_TOL
    if exact is None or not isinstance(want, float) or not isinstance(got, (int, float)):
        # no exact counterpart: counts, and min / max (order-independent: always bit-exact)
        assert _num_equal(got, want, exact_floats or key in ("min", "max"), tol), f"{path}: {got!r} != {want!r}"
        return
    eg, ew = _rel(got, exact), _rel(want, exact)
    if report is not None:
        report.add(key, ew, eg)
    if _rel(got, want) == 0.0 and not (strict and eg > tol and not derived):
        return  # the reference's own double, bit for bit
    if exact_floats and ew == 0.0:
        # the reference's sum is exact (integer data below 2^53): the GPU's must be the same double
        assert False, f"{path}: {got!r} != {want!r} (exact {exact!r})"
    # within the bar of the oracle, or -- where the oracle's doc-order rounding is the larger error -- of the exact
    # value; strict: always within the bar of the exact value (a derived statistic, whose subtraction cancels, may
    # instead match the oracle's)
    ok = eg <= tol or (not strict and _num_equal(got, want, False, tol)) or (derived and _num_equal(got, want, False, tol))
    if not ok and derived and math.isfinite(float(got)) and math.isfinite(float(exact)):
        ok = abs(float(got) - float(exact)) <= tol * max(abs(float(got)), abs(float(exact)), 1.0)
    assert ok, f"{path}: {got!r} vs exact {exact!r} (oracle {want!r}; rel err gpu {eg:.3g}, oracle {ew:.3g})"


def assert_same_exact(got, want, path="", exact_floats=True, report=None, _exact=None, _key="", strict=False):
    """assert_same against an oracle run with exact=True: a metric's floating values are compared with its "_exact"
    values (the exact sums the reference's doc-order additions approximate, and the statistics derived from them by the
    reference's formulas).  The GPU must be within REL_TOL (DERIVED_TOL for variance / std_deviation / bounds) of the
    exact value or of the oracle's (strict: of the exact value); with exact_floats, a value the oracle computed exactly
    must be bit-identical.  `report` (FloatReport) collects the oracle's and the GPU's largest errors."""
    if isinstance(want, dict):
        if "_exact" in want:
            want = dict(want)
            ex = want.pop("_exact")
            assert isinstance(got, dict), f"{path}: expected object"
            assert set(got) == set(want), f"{path}: keys differ: {sorted(set(got) ^ set(want))}"
            for k in want:
                assert_same_exact(got[k], want[k], f"{path}.{k}", exact_floats, report, ex.get(k), k, strict)
            return
        assert isinstance(got, dict), f"{path}: expected object, got {type(got).__name__}"
        assert set(got) == set(want), f"{path}: keys differ: {sorted(set(got) ^ set(want))}"
        for k in want:
            sub = _exact.get(k) if isinstance(_exact, dict) else None
            assert_same_exact(got[k], want[k], f"{path}.{k}", exact_floats, report, sub, k, strict)
    elif isinstance(want, list):
        assert isinstance(got, list), f"{path}: expected list"
        assert len(got) == len(want), f"{path}: length {len(got)} != {len(want)}"
        for i, (g, w) in enumerate(zip(got, want)):
            assert_same_exact(g, w, f"{path}[{i}]", exact_floats, report, strict=strict)
    elif isinstance(want, str):
        assert got == want, f"{path}: {got!r} != {want!r}"
    else:
        _exact_leaf(got, want, _exact, path, _key, exact_floats, report, strict)


def strip_exact(tree):
    """An oracle result run with exact=True, without its "_exact" objects (for assert_same)."""
    if isinstance(tree, dict):
        return {k: strip_exact(v) for k, v in tree.items() if k != "_exact"}
    if isinstance(tree, list):
        return [strip_exact(v) for v in tree]
    return tree


def bits_from_mask(mask):
    """bool array -> u64 bitset words (bit d of word d // 64 set = doc d), the layout of include/esgpu.h."""
    mask = np.asarray(mask, dtype=bool)
    words = np.zeros(max((len(mask) + 63) // 64, 1), dtype=np.uint64)
    idx = np.nonzero(mask)[0].astype(np.uint64)
    np.bitwise_or.at(words, (idx // np.uint64(64)).astype(np.int64), np.left_shift(np.uint64(1), idx % np.uint64(64)))
    return words
