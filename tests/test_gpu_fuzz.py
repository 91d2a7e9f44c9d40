"""GPU parity over seeded random requests: request trees drawn from everything the GPU path accepts (terms over low- /
mid- / high-cardinality and multi-valued keyword fields, histogram, date_histogram with calendar and fixed intervals,
offsets, fixed and DST time zones, min_doc_count 0 with extended bounds, every terms order including metric-path
orders, stats / extended_stats / avg / cardinality leaves, terms under terms, filter aggregations, query term / range
clauses, histogram under histogram) over random columns (missing values, unsorted timestamps, ragged sizes).  Each case compares the shard-level
and the reduced results with the oracle (tests/helpers.assert_same) and, when every metric is integer-valued, the
transport bytes of the shard result with the oracle's writer.

A case the GPU plan reports as ESGPU_ERR_UNSUPPORTED is counted and skipped (the plugin keeps the stock aggregator);
the test fails if more than a third of the cases are refused, so the generator keeps exercising the GPU path.
"""
import numpy as np
import pytest

import oracle as O
import es_stream as ES
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, QueryBuilders as QB
from elasticsearch_amd import _native as N
from elasticsearch_amd.aggs import TermsBuilder
from elasticsearch_amd import reduce
from helpers import assert_same, bits_from_mask

pytestmark = pytest.mark.gpu

T0 = 1441065600000  # 2015-09-01T00:00:00Z
DAY = 86_400_000


def _zipf_ords(rng, n, T, s):
    r = np.minimum(rng.zipf(s, size=n) - 1, T - 1)
    return ((r * 7919 + 13) % T).astype(np.uint32)


def make_segment(rng, n):
    span = int(rng.choice([6 * 3_600_000, 3 * DAY, 40 * DAY]))
    ts = T0 + np.sort(rng.integers(0, span, size=n)).astype(np.int64)
    jitter = int(rng.choice([0, 0, 600_000, 5 * 3_600_000]))
    if jitter:
        ts = ts + rng.integers(-jitter, jitter + 1, size=n)
    T_kw = int(rng.choice([9, 400, 6000, 150_000]))
    kw = _zipf_ords(rng, n, T_kw, float(rng.choice([1.05, 1.3, 2.0])))
    kw[rng.random(n) < 0.04] = 0xFFFFFFFF
    kw2 = rng.integers(0, 40, size=n).astype(np.uint32)
    ts_present = rng.random(n) >= (0.1 if rng.random() < 0.5 else 0.0)
    cols = {
        "kw": {"type": N.COL_ORD_U32, "values": kw, "terms": ["k%06d" % i for i in range(T_kw)]},
        "kw2": {"type": N.COL_ORD_U32, "values": kw2, "terms": ["q%02d" % i for i in range(40)]},
        "@timestamp": {"type": N.COL_I64, "values": np.where(ts_present, ts, 0),
                       "present": bits_from_mask(ts_present) if not ts_present.all() else None},
        "num": {"type": N.COL_I64, "values": rng.integers(0, 1000, size=n).astype(np.int64)},
        "price": {"type": N.COL_F64, "values": np.round(rng.random(n) * 500.0, 3)},
        "h": {"type": N.COL_U64, "values": rng.integers(0, 1 << 62, size=n, dtype=np.int64).astype(np.uint64)
              % np.uint64(int(rng.choice([50, 5000, 1 << 40])))},
        "status": {"type": N.COL_I64, "values": rng.choice([200, 200, 200, 304, 404, 500], size=n).astype(np.int64)},
    }
    # multi-valued keyword field (SortedSet CSR: unique, ascending per doc)
    cnt = rng.integers(0, 4, size=n)
    doc = np.repeat(np.arange(n), cnt)
    vals = rng.integers(0, 60, size=cnt.sum())
    order = np.lexsort((vals, doc))
    doc, vals = doc[order], vals[order]
    keep = np.ones(len(vals), dtype=bool)
    keep[1:] = (doc[1:] != doc[:-1]) | (vals[1:] != vals[:-1])
    doc, vals = doc[keep], vals[keep]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(np.bincount(doc, minlength=n), out=offs[1:])
    cols["tags"] = {"type": N.COL_ORD_U32, "values": vals.astype(np.uint32), "offsets": offs,
                    "terms": ["t%02d" % i for i in range(60)]}
    return cols, T_kw


class Gen:
    def __init__(self, rng, T_kw, rng2=None, rng3=None):
        self.r = rng
        # shapes added later draw from their own stream, so the earlier shapes of every seed stay what they were
        self.r2 = rng2 if rng2 is not None else np.random.default_rng(0)
        self.r3 = rng3 if rng3 is not None else np.random.default_rng(1)  # round 4: nested filter aggregations
        self.T_kw = T_kw
        self.k = 0
        self.inexact = False

    def name(self, p):
        self.k += 1
        return "%s%d" % (p, self.k)

    def metric(self):
        r = self.r
        kind = r.choice(["stats", "extended_stats", "avg", "cardinality"])
        field = "price" if r.random() < 0.25 else "num"
        if kind == "cardinality":
            m = AB.cardinality(self.name("c")).field(str(r.choice(["h", "num", "kw"])))
            if r.random() < 0.5:
                m.precisionThreshold(int(r.choice([100, 3000, 40000])))
            return m, None
        if field == "price":
            self.inexact = True
        if kind == "stats":
            m = AB.stats(self.name("s")).field(field)
            return m, str(r.choice([".count", ".max", ".min", ".avg", ".sum"]))
        if kind == "extended_stats":
            m = AB.extendedStats(self.name("x")).field(field)
            if r.random() < 0.3:
                m.sigma(float(r.choice([0.5, 1.0, 3.0])))
            return m, str(r.choice([".variance", ".sum_of_squares", ".std_upper", ".max"]))
        return AB.avg(self.name("a")).field(field), ""

    def terms(self, inner):
        r = self.r
        field = "kw2" if inner else str(r.choice(["kw", "kw", "kw2", "tags"]))
        t = AB.terms(self.name("t")).field(field).size(int(r.choice([1, 3, 10, 25])))
        small = field != "kw" or self.T_kw <= 6000
        if r.random() < 0.3:
            t.shardSize(int(r.choice([0, 5, 50])))
        if small and r.random() < 0.15:
            t.minDocCount(0)
        elif r.random() < 0.2:
            t.minDocCount(int(r.choice([2, 50])))
        if r.random() < 0.2:
            t.showTermDocCountError(True)
        return t

    def date_histogram(self, affine=False):
        r = self.r
        interval = str(r.choice(["1h", "30m", "3h", "1d"] if affine else ["1h", "1h", "30m", "3h", "1d", "day", "week", "month"]))
        d = AB.dateHistogram(self.name("d")).field("@timestamp").interval(interval)
        tz = r.choice([None, "+01:00", "-05:30"] if affine else [None, None, "+01:00", "-05:30", "Europe/Berlin", "America/New_York"])
        if tz is not None:
            d.timeZone(str(tz))
        if r.random() < 0.3:
            d.offset(str(r.choice(["+15m", "-2h", "+1h"])))
        if r.random() < 0.5:
            d.minDocCount(1)
        elif r.random() < 0.3:
            d.extendedBounds(T0 - DAY, T0 + 5 * DAY)
        if r.random() < 0.15:
            d.order(N.ORDER_KEY_DESC)
        return d

    def histogram(self):
        r = self.r
        h = AB.histogram(self.name("h")).field("num").interval(int(r.choice([7, 50, 250])))
        if r.random() < 0.3:
            h.offset(int(r.choice([3, 20])))
        if r.random() < 0.5:
            h.minDocCount(1)
        elif r.random() < 0.3:
            h.extendedBounds(-100, 1500)
        if r.random() < 0.15:
            h.order(int(r.choice([N.ORDER_KEY_DESC, N.ORDER_HCOUNT_DESC, N.ORDER_HCOUNT_ASC])))
        return h

    def bucket(self, depth):
        r = self.r
        kind = r.choice(["terms", "date_histogram", "histogram"], p=[0.5, 0.3, 0.2])
        b = self.terms(False) if kind == "terms" else self.date_histogram() if kind == "date_histogram" else self.histogram()
        order_targets = []
        for _ in range(int(r.integers(0, 3))):
            m, key = self.metric()
            b.subAggregation(m)
            if key is not None:
                order_targets.append(m.name + key)
            elif self.r2.random() < 0.5:  # a cardinality child as the terms order (its single value)
                order_targets.append(m.name)
        if (depth == 0 and self.r2.random() < 0.25) or (depth == 1 and self.r3.random() < 0.3):
            # a filter aggregation under the bucket (a first-level bucket: at the top, or inside a top-level filter)
            r_main, self.r = self.r, self.r2
            f = AB.filter(self.name("g"), QB.termQuery("status", int(self.r2.choice([200, 404]))) if self.r2.random() < 0.6
                          else QB.rangeQuery("num").gte(int(self.r2.integers(0, 600))))
            for _ in range(int(self.r2.integers(0, 3))):
                f.subAggregation(self.metric()[0])
            self.r = r_main
            b.subAggregation(f)
        if depth == 0 and r.random() < 0.5:
            inner = self.terms(True) if kind == "terms" and r.random() < 0.5 else (
                self.date_histogram() if kind == "terms" else self.terms(True))
            if kind != "terms" and r.random() < 0.4:  # histogram under histogram (affine inner rounding)
                inner = self.histogram() if kind == "date_histogram" or r.random() < 0.5 else self.date_histogram(affine=True)
            for _ in range(int(r.integers(0, 2))):
                inner.subAggregation(self.metric()[0])
            root_t, inner_t = kind == "terms", isinstance(inner, TermsBuilder)
            if (root_t or inner_t) and self.r2.random() < 0.3:  # a third level: two terms and one histogram
                r_main, self.r = self.r, self.r2
                third = self.terms(True) if not (root_t and inner_t) else (
                    self.date_histogram(affine=True) if self.r2.random() < 0.6 else self.histogram())
                for _ in range(int(self.r2.integers(0, 2))):
                    third.subAggregation(self.metric()[0])
                self.r = r_main
                inner.subAggregation(third)
            if kind != "terms" and isinstance(inner, TermsBuilder) and r.random() < 0.4:
                # terms under a histogram: count orders select per row on the GPU, term orders on the host
                inner.order(Order.count(bool(r.random() < 0.5)) if r.random() < 0.7 else Order.term(bool(r.random() < 0.5)))
            b.subAggregation(inner)
        if kind == "terms":
            c = r.random()
            if order_targets and c < 0.3:
                b.order(Order.aggregation(str(r.choice(order_targets)), bool(r.random() < 0.5)))
            elif c < 0.5:
                b.order(Order.count(True) if r.random() < 0.5 else Order.term(bool(r.random() < 0.5)))
        return b

    def request(self):
        r = self.r
        aggs = []
        for _ in range(int(r.integers(1, 3))):
            c = r.random()
            if c < 0.7:
                aggs.append(self.bucket(0))
            elif c < 0.85:
                f = AB.filter(self.name("f"), QB.termQuery("status", int(r.choice([200, 404]))))
                f.subAggregation(self.metric()[0] if r.random() < 0.5 else self.bucket(1))
                if self.r3.random() < 0.4:  # a filter inside the filter (nested FilterAggregators intersect)
                    g = AB.filter(self.name("n"), QB.rangeQuery("num").gte(int(self.r3.integers(0, 700))))
                    r_main, self.r = self.r, self.r3
                    g.subAggregation(self.metric()[0] if self.r3.random() < 0.5 else self.bucket(1))
                    self.r = r_main
                    f.subAggregation(g)
                aggs.append(f)
            else:
                aggs.append(self.metric()[0])
        filters = []
        if r.random() < 0.4:
            filters.append(QB.termQuery("status", int(r.choice([200, 304, 500]))))
        if r.random() < 0.3:
            filters.append(QB.rangeQuery("num").gte(int(r.integers(0, 500))).lt(int(r.integers(500, 1100))))
        return aggs, filters or None


SEEDS = list(range(160))
_stats = {"ran": 0, "refused": 0}


@pytest.mark.parametrize("seed", SEEDS)
def test_random_request(engine, seed, monkeypatch):
    if seed % 3 == 0:  # terms under terms collected breadth-first (replayed at build) whatever the grid size
        monkeypatch.setenv("ESGPU_DEFER_CELLS", "1")
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(30_000, 300_000))
    cols, T_kw = make_segment(rng, n)
    gen = Gen(rng, T_kw, np.random.default_rng(50_000 + seed), np.random.default_rng(90_000 + seed))
    aggs, filters = gen.request()
    lookups = {f: {t: i for i, t in enumerate(cols[f]["terms"])} for f in ("kw", "kw2", "tags")}
    ord_lookup = lambda f, t: lookups.get(f, {}).get(t, -1)  # noqa: E731
    seg = engine.upload_segment(cols, n)
    try:
        plan = engine.plan(aggs, filters=filters, ord_lookup=ord_lookup)
        plan.collect(seg)
    except N.UnsupportedOnGpu as e:
        _stats["refused"] += 1
        seg.close()
        pytest.skip("shape refused by the GPU plan: %s" % e)
    _stats["ran"] += 1
    res = plan.build()
    want = O.run([(cols, n)], aggs, filters=filters, ord_lookup=ord_lookup, streams=True)
    exact = not gen.inexact
    assert_same(res.to_dict(), want["shards"][0], "shard", exact)
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced", exact)
    if exact:
        got_w, want_w = res.to_stream(), want["streams"][0]
        # byte for byte, LINEAR_COUNTING hash lists included (the reference's Hashset slot order)
        if got_w != want_w:
            g, w = ES.decode(got_w), ES.decode(want_w)
            d = ES.first_diff(g, w)
            msg = f"stream differs at {d[0] if d else '?'}: got {d[1] if d else ''} want {d[2] if d else ''}"
            if d and ".lc[" in d[0]:  # the whole hash lists of that sketch
                path = d[0][:d[0].rindex("[")]
                def at(tree, pth):
                    import re
                    x = tree
                    for tok in re.findall(r"\.(\w+)|\[(\d+)\]", pth[len("aggs"):]):
                        x = x[tok[0]] if tok[0] else x[int(tok[1])]
                    return x
                gl, wl = at(g, path), at(w, path)
                msg += f"; lists {len(gl)} / {len(wl)}, same set {sorted(gl) == sorted(wl)}, got {gl[:6]} want {wl[:6]}"
            raise AssertionError(msg)
    plan.close()
    seg.close()


DENSE_SEEDS = list(range(48))


@pytest.mark.parametrize("seed", DENSE_SEEDS)
def test_random_request_dense_timestamps(engine, seed, monkeypatch):
    """The same random requests over segments whose timestamps are dense enough for the block-delta layout (every run of
    2,048 docs spans < 2^16 ms: 30 minutes to 4 hours of docs, displaced by up to 5 s): the raw-load kernels read 16-bit
    timestamp deltas, take single-key zone blocks' key without reading them, and step 8 docs per thread."""
    if seed % 3 == 0:
        monkeypatch.setenv("ESGPU_DEFER_CELLS", "1")
    rng = np.random.default_rng(7000 + seed)
    n = int(rng.integers(30_000, 300_000))
    cols, T_kw = make_segment(rng, n)
    r = np.random.default_rng(9000 + seed)
    span = int(r.choice([1_800_000, 3_600_000, 4 * 3_600_000]))
    span = min(span, n * 30)  # < 2^16 ms per 2,048-doc run
    ts = T0 + np.sort(r.integers(0, span, size=n)).astype(np.int64)
    if r.random() < 0.5:
        ts = ts + r.integers(-5000, 5001, size=n)
    cols["@timestamp"] = {"type": N.COL_I64, "values": ts}
    gen = Gen(rng, T_kw, np.random.default_rng(60_000 + seed), np.random.default_rng(95_000 + seed))
    aggs, filters = gen.request()
    lookups = {f: {t: i for i, t in enumerate(cols[f]["terms"])} for f in ("kw", "kw2", "tags")}
    ord_lookup = lambda f, t: lookups.get(f, {}).get(t, -1)  # noqa: E731
    seg = engine.upload_segment(cols, n)
    try:
        plan = engine.plan(aggs, filters=filters, ord_lookup=ord_lookup)
        plan.collect(seg)
    except N.UnsupportedOnGpu as e:
        seg.close()
        pytest.skip("shape refused by the GPU plan: %s" % e)
    res = plan.build()
    want = O.run([(cols, n)], aggs, filters=filters, ord_lookup=ord_lookup)
    exact = not gen.inexact
    assert_same(res.to_dict(), want["shards"][0], "shard", exact)
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced", exact)
    plan.close()
    seg.close()


def test_fuzz_mostly_on_gpu():
    """runs after the cases above (file order): most random requests must have run on the GPU path"""
    total = _stats["ran"] + _stats["refused"]
    if total == 0:
        pytest.skip("no fuzz case ran in this session")
    assert _stats["refused"] * 3 <= total, _stats
