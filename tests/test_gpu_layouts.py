"""GPU parity of every collect-kernel column layout ("parity leg for the upload-width kernels").

The single-valued collect kernel reads, per segment, the narrowest layout the data allows:
  * upload width: u32 ordinals, i64 timestamps / filter values / metric (compact columns off);
  * compact: u16 ordinals (dictionaries under 65,535 terms), u32 deltas of long columns spanning < 2^32 (u16 deltas
    for filter columns spanning < 2^16);
  * compact + packed integer metric cells: a dense long metric under terms read as its u32 deltas (u16 when its values
    span < 2^16) and accumulated as count << shift | sum of deltas in one u64 LDS word;
  * + block deltas: a dense time-sorted key column whose every run of 2,048 docs spans < 2^16 ms, read by the raw-load
    kernels as 16-bit deltas over each run's minimum (2 B per timestamp, plus 8 B per run).
Real indices take each of them: timestamps over more than 2^32 ms (49.7 days) keep i64 keys, sparse or double metrics
keep f64 cells.  The layout is a per-context option (Engine.set_option), so one session runs them all against the same
oracle result; the algorithmic bytes the plan reports name the layout that ran (north star: 20 / 14 / 8 / 6 B per doc).
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, QueryBuilders as QB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce
from helpers import assert_same, assert_same_exact, bits_from_mask, synthetic_columns

pytestmark = pytest.mark.gpu

# name -> (compact columns, packed metric, block deltas)
LAYOUTS = {"upload": (0, 0, 0), "compact": (1, 0, 0), "packed": (1, 1, 0), "block": (1, 1, 1)}


class layout:
    """Context options for the duration of a block (the session's engine is shared by every GPU test)."""

    def __init__(self, engine, name):
        self.e, self.v = engine, LAYOUTS[name]

    def __enter__(self):
        self.e.set_option("compact_columns", self.v[0])
        self.e.set_option("packed_metric", self.v[1])
        self.e.set_option("block_deltas", self.v[2])

    def __exit__(self, *a):
        self.e.set_option("compact_columns", 1)
        self.e.set_option("packed_metric", 1)
        self.e.set_option("block_deltas", 1)


def run_bytes(n):
    """The block-delta layout's per-run words (8 B per 2,048 docs)."""
    return (n + 2047) // 2048 * 8


def check_bytes(name, nbytes, bpd, n, skips=("packed", "block")):
    """The bytes the plan reports for its layout.  The raw-load kernels (packed cells, and on the block layout every
    grid over the timestamp deltas) read no timestamp in a zone block whose docs all round to one key: bpd B per doc
    (and the run words of block deltas), less the 2 B (block deltas) or 4 B (32-bit deltas) timestamps of those blocks --
    at 100M docs over 30 days a block spans ~212 s, so ~94 % of the blocks hold one hour."""
    if name not in skips:
        assert nbytes == bpd * n, (name, nbytes / n)
        return
    ts = 2 if name == "block" else 4
    full = bpd * n + (run_bytes(n) if name == "block" else 0)
    assert full - ts * n <= nbytes < full - ts * n // 2, (name, nbytes / n)


def _run(engine, seg, aggs, filters=None, number_of_shards=1, segs=None):
    plan = engine.plan(aggs, filters=filters, number_of_shards=number_of_shards)
    nbytes = 0
    for s in (segs or [seg]):
        plan.collect(s)
        nbytes += plan.last_collect_stats()[1]
    res = plan.build()
    plan.close()
    return res, nbytes


NS_FIELDS = ("host", "@timestamp", "response_time_ms")
NS_AGGS = [AB.terms("hosts").field("host").size(10).subAggregation(
    AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("response_time_ms")))]
C5_FIELDS = ("status", "bytes", "host", "@timestamp", "response_time_ms")
C5_AGGS = [AB.terms("hosts").field("host").size(10).subAggregation(
    AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.avg("rt").field("response_time_ms")))]
C5_FILTERS = [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)]


@pytest.fixture(scope="module")
def ns_100m():
    n = 100_000_000
    cols = synthetic_columns(NS_FIELDS, n)
    want = O.run([(cols, n)], NS_AGGS)
    return n, want


@pytest.fixture(scope="module")
def c5_100m():
    n = 100_000_000
    cols = synthetic_columns(C5_FIELDS, n, shard=2)
    want = O.run([(cols, n)], C5_AGGS, filters=C5_FILTERS, number_of_shards=8)
    return n, want


@pytest.mark.parametrize("name,bpd", [("upload", 20), ("compact", 14), ("packed", 8), ("block", 6)])
def test_north_star_100m_every_layout(engine, ns_100m, name, bpd):
    n, want = ns_100m
    with layout(engine, name):
        seg = engine.synthetic_segment(n, fields=NS_FIELDS)  # a fresh segment: its compact copies are built by this layout
        res, nbytes = _run(engine, seg, NS_AGGS)
        seg.close()
    check_bytes(name, nbytes, bpd, n)
    assert_same(res.to_dict(), want["shards"][0], f"{name} shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], f"{name} reduced")


@pytest.mark.parametrize("name,bpd", [("upload", 36), ("compact", 20), ("packed", 14), ("block", 12)])
def test_config5_100m_every_layout(engine, c5_100m, name, bpd):
    n, want = c5_100m
    with layout(engine, name):
        seg = engine.synthetic_segment(n, fields=C5_FIELDS, shard=2)
        res, nbytes = _run(engine, seg, C5_AGGS, filters=C5_FILTERS, number_of_shards=8)
        seg.close()
    check_bytes(name, nbytes, bpd, n)
    assert_same(res.to_dict(), want["shards"][0], f"{name} shard")


C2_FIELDS = ("@timestamp", "response_time_ms")
C2_AGGS = [AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(
    AB.extendedStats("rt").field("response_time_ms"))]


@pytest.fixture(scope="module")
def c2_100m():
    n = 100_000_000
    cols = synthetic_columns(C2_FIELDS, n, shard=3)
    want = O.run([(cols, n)], C2_AGGS)
    return n, want


@pytest.mark.parametrize("name", ["upload", "compact", "packed", "block"])
def test_config2_100m_every_layout(engine, c2_100m, name):
    """Config 2 (date_histogram{extended_stats}) on every layout: upload-width f64 runs
    (16 B per doc), the 32-bit timestamp deltas with the metric's 16-bit deltas in integer runs (6 B), and block deltas
    (4 B + the run words)."""
    n, want = c2_100m
    with layout(engine, name):
        seg = engine.synthetic_segment(n, fields=C2_FIELDS, shard=3)
        res, nbytes = _run(engine, seg, C2_AGGS)
        seg.close()
    # (the histogram-only raw-load kernels read the 32-bit deltas on the compact layout already)
    check_bytes(name, nbytes, {"upload": 16, "compact": 6, "packed": 6, "block": 4}[name], n,
                skips=("compact", "packed", "block"))
    assert_same(res.to_dict(), want["shards"][0], f"{name} shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], f"{name} reduced")


def _dense_ts(rng, n, t0, per_run_span):
    """Sorted timestamps whose runs of 2,048 docs span about per_run_span ms."""
    step = per_run_span / 2048.0
    return (t0 + np.floor(np.arange(n) * step) + rng.integers(0, max(int(step), 1), size=n)).astype(np.int64)


@pytest.mark.parametrize("t0,per_run,layout,jitter", [
    (1_441_065_600_000, 30_000, "b16", 0),      # dense logs
    (-3_600_000 * 5, 30_000, "b16", 0),          # before the epoch: negative keys and bases
    (1_441_065_600_000, 66_000, "b24", 0),      # some run spans >= 2^16 ms: 24-bit runs (a zone block spans < 5 min)
    (1_441_065_600_000, 2_000_000, "d32", 0),   # runs < 2^24 ms but every zone block spans several keys: 32-bit deltas
    (1_441_065_600_000, 20_000, "b16", 20_000),  # merged-segment order: docs displaced by up to 20 s, runs still < 2^16
    (1_441_065_600_000, 20_000, "b24", 60_000),  # ... by up to 1 min: 24-bit runs, most zone blocks still single-key
])
def test_block_delta_keys(engine, t0, per_run, layout, jitter):
    """Block-delta timestamps on every raw-load kernel that takes them -- packed cells (terms{date_histogram{stats}},
    unfiltered and through a folded filter), integer runs (date_histogram{extended_stats}), counting grids
    (date_histogram, terms{date_histogram}) -- over a ragged last run (n not a multiple of 2,048), against the oracle;
    16-bit runs, 24-bit runs (a high-byte plane) and the 32-bit deltas where the zone blocks span several keys; then the
    upload-width timestamps released and rebuilt from the block deltas (a calendar histogram reads them)."""
    rng = np.random.default_rng(50 + per_run)
    n = 2_000_000 + 777
    cols = _log_segment(rng, n, 0, 1)
    cols["@timestamp"]["values"] = _dense_ts(rng, n, t0, per_run)
    if jitter:  # unsorted inside and across blocks; blocks straddling key boundaries take the per-doc keys
        cols["@timestamp"]["values"] = cols["@timestamp"]["values"] + rng.integers(-jitter, jitter + 1, size=n)
    cols["rt"]["values"] = rng.integers(0, 5000, size=n).astype(np.int64)
    aggs = [AB.terms("h").field("host").size(6).subAggregation(
                AB.dateHistogram("d").field("@timestamp").interval("1h").minDocCount(0).subAggregation(AB.stats("s").field("rt"))),
            AB.dateHistogram("x").field("@timestamp").interval("1h").subAggregation(AB.extendedStats("e").field("rt")),
            AB.dateHistogram("c").field("@timestamp").interval("5m"),
            AB.terms("hc").field("host").size(4).subAggregation(AB.dateHistogram("d").field("@timestamp").interval("1h"))]
    want = O.run([(cols, n)], aggs)
    seg = engine.upload_segment(cols, n)
    got = {}
    for a in aggs:
        r, nbytes = _run(engine, seg, [a])
        got.update(r.to_dict())
    assert_same(got, want["shards"][0], "block deltas")
    # the key column's bytes: 2 B (3 B with the high-byte plane) per doc + the run words on the block-delta layouts (less
    # the single-key zone blocks' timestamps: a block spans ~120 s in the dense case, 60 % of them within one 5-minute
    # key), else 4 B
    r, nbytes = _run(engine, seg, [aggs[2]])
    if layout == "b24":  # 3 B per doc of the multi-key zone blocks
        assert run_bytes(n) + 0.5 * n < nbytes <= run_bytes(n) + 3 * n, nbytes / n
    elif layout == "d32":
        assert 3.9 * n < nbytes <= 4 * n + 64, nbytes / n
    elif layout == "b16":
        assert run_bytes(n) < nbytes <= run_bytes(n) + 2 * n, nbytes / n
        if not jitter:
            assert run_bytes(n) + 0.4 * n < nbytes < run_bytes(n) + 1.2 * n, nbytes / n
    accept = bits_from_mask(rng.random(n) >= 0.25)
    fw = O.run([(cols, n)], aggs[:1], accept=[accept])
    plan = engine.plan(aggs[:1])
    plan.collect(seg, accept_bits=accept)
    assert_same(plan.build().to_dict(), fw["shards"][0], "folded filter")
    plan.close()
    freed = seg.release_wide()
    assert freed >= 8 * n
    month = [AB.dateHistogram("m").field("@timestamp").interval("month").subAggregation(AB.stats("s").field("rt"))]
    r, _ = _run(engine, seg, month)
    assert_same(r.to_dict(), O.run([(cols, n)], month)["shards"][0], "rebuilt from block deltas")
    seg.close()


@pytest.mark.parametrize("jitter", [60_000, 3_600_000])
def test_jittered_timestamps(engine, jitter):
    """Roughly time-ordered data (merged segments: docs displaced by up to +-1 min / +-1 h; one day, 3M docs): every run
    of 2,048 docs then spans >= 2^16 ms.  At +-1 min most zone blocks still round to one hour: the key column is read as
    24-bit block deltas (the high-byte plane) with the single-key blocks skipped, one integer run per thread; at +-1 h
    they span three keys: the 32-bit deltas, the histogram-only integer grids' window accumulators (kWin4) and the
    packed-cell grids' per-doc path -- every leaf against the oracle, 1 h and 5 min keys."""
    rng = np.random.default_rng(61)
    n = 3_000_000 + 333
    cols = _log_segment(rng, n, 1_441_065_600_000, 86_400_000)
    cols["@timestamp"]["values"] = cols["@timestamp"]["values"] + rng.integers(-jitter, jitter + 1, size=n)
    dh = lambda i: AB.dateHistogram("d").field("@timestamp").interval(i)  # noqa: E731
    aggs = [dh("1h").subAggregation(AB.extendedStats("e").field("rt")),
            dh("1h").subAggregation(AB.stats("s").field("rt")),
            dh("1h").subAggregation(AB.avg("a").field("rt")),
            dh("5m").subAggregation(AB.extendedStats("e").field("rt")),
            AB.terms("h").field("host").size(5).subAggregation(dh("1h").subAggregation(AB.stats("s").field("rt"))),
            AB.terms("h").field("host").size(5).subAggregation(dh("1h").subAggregation(AB.avg("a").field("rt")))]
    seg = engine.upload_segment(cols, n)
    for k, a in enumerate(aggs):
        want = O.run([(cols, n)], [a])
        r, _ = _run(engine, seg, [a])
        assert_same(r.to_dict(), want["shards"][0], f"jitter {jitter} agg {k}")
    seg.close()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_window_accumulators_fuzz(engine, seed):
    """Window accumulators (kWin4: histogram-only integer grids over roughly time-ordered data, four key slots per
    thread) under displacement that moves a thread's keys both ways: ±1 h to ±3 h jitter, 0.1 % of the docs thrown
    days away (each one a re-base below or above the window and back), metric deltas up to the 16-bit edge, a ragged
    last block -- extended_stats / stats / avg per key against the oracle, 1 h and 20 min keys."""
    rng = np.random.default_rng(700 + seed)
    n = 1_500_000 + 4099 * seed + 13
    t0 = 1_441_065_600_000
    ts = np.sort(rng.integers(t0, t0 + 3 * 86_400_000, size=n)).astype(np.int64)
    ts += rng.integers(-(1 + seed) * 3_600_000, (1 + seed) * 3_600_000 + 1, size=n)
    far = rng.random(n) < 0.001
    ts[far] += rng.integers(-2 * 86_400_000, 2 * 86_400_000 + 1, size=int(far.sum()))
    cols = _log_segment(rng, n, 0, 1, metric=rng.integers(0, 65536, size=n))
    cols["@timestamp"]["values"] = ts
    dh = lambda i: AB.dateHistogram("d").field("@timestamp").interval(i)  # noqa: E731
    aggs = [dh("1h").subAggregation(AB.extendedStats("e").field("rt")),
            dh("20m").subAggregation(AB.stats("s").field("rt")),
            dh("1h").subAggregation(AB.avg("a").field("rt"))]
    seg = engine.upload_segment(cols, n)
    for k, a in enumerate(aggs):
        r, _ = _run(engine, seg, [a])
        assert_same(r.to_dict(), O.run([(cols, n)], [a])["shards"][0], f"seed {seed} agg {k}")
    seg.close()


def _log_segment(rng, n, t0, span_ms, nterms=300, metric=None):
    ranks = np.minimum(rng.zipf(1.2, size=n) - 1, nterms - 1)
    cols = {
        "host": {"type": N.COL_ORD_U32, "values": ((ranks * 37 + 11) % nterms).astype(np.uint32),
                 "terms": ["h%04d" % i for i in range(nterms)]},
        "@timestamp": {"type": N.COL_I64, "values": np.sort(rng.integers(t0, t0 + span_ms, size=n)).astype(np.int64)},
        "rt": {"type": N.COL_I64, "values": (rng.integers(0, 1000, size=n) if metric is None else metric).astype(np.int64)},
    }
    return cols


@pytest.mark.parametrize("name", ["upload", "compact", "packed"])
def test_timestamps_over_2_32_ms(engine, name):
    """Timestamps spanning 60 days (5.2e9 ms > 2^32): the key column stays i64 on every layout (u16 ordinals and the
    packed metric still apply where they can: terms{stats} without a key takes packed cells, the daily and hourly
    histograms i64 keys)."""
    rng = np.random.default_rng(41)
    n = 3_000_000
    cols = _log_segment(rng, n, 1_420_070_400_000, 60 * 86_400_000)
    aggs = [AB.terms("h").field("host").size(8).subAggregation(
                AB.dateHistogram("d").field("@timestamp").interval("1h").subAggregation(AB.stats("s").field("rt"))),
            AB.terms("hs").field("host").size(12).order(Order.aggregation("s.max", False)).subAggregation(AB.stats("s").field("rt")),
            AB.dateHistogram("days").field("@timestamp").interval("1d").subAggregation(
                AB.terms("t").field("host").size(3).subAggregation(AB.avg("a").field("rt")))]
    want = O.run([(cols, n)], aggs)
    with layout(engine, name):
        seg = engine.upload_segment(cols, n)
        res, _ = _run(engine, seg, aggs)
        seg.close()
    assert_same(res.to_dict(), want["shards"][0], f"{name} shard")


@pytest.mark.parametrize("name", ["compact", "packed"])
def test_packed_metric_edge_values(engine, name):
    """Packed cells decode count * base + sum of deltas: negative metrics, a base far from zero (sums beyond 2^53:
    compensated into the grid, checked against the exact sums; values spanning < 2^16, read as u16 deltas), deltas near
    2^32, and two segments whose metric bases differ -- each decoded with its own base; stats, avg and extended_stats
    (the latter never packed) side by side."""
    rng = np.random.default_rng(42)
    t0 = 1_441_065_600_000
    segs_cols = []
    for k, (lo, hi) in enumerate([(-500_000, 500_000), (1_000_000_000_000, 1_000_000_000_999), (0, (1 << 32) - 1)]):
        n = 700_000 + 100_000 * k
        cols = _log_segment(rng, n, t0 + k * 86_400_000, 86_400_000, metric=rng.integers(lo, hi + 1, size=n))
        segs_cols.append((cols, n))
    allc = {f: dict(segs_cols[0][0][f], values=np.concatenate([c[f]["values"] for c, _ in segs_cols])) for f in segs_cols[0][0]}
    ntot = sum(n for _, n in segs_cols)
    aggs = [AB.terms("h").field("host").size(6).subAggregation(
                AB.dateHistogram("d").field("@timestamp").interval("1h").minDocCount(0).subAggregation(AB.stats("s").field("rt"))),
            AB.terms("a").field("host").size(9).subAggregation(AB.avg("m").field("rt")),
            AB.terms("x").field("host").size(4).subAggregation(AB.extendedStats("e").field("rt"))]
    want = O.run([(allc, ntot)], aggs, exact=True)
    with layout(engine, name):
        segs = [engine.upload_segment(c, n) for c, n in segs_cols]
        res, _ = _run(engine, None, aggs, segs=segs)
        for s in segs:
            s.close()
    assert_same_exact(res.to_dict(), want["shards"][0], f"{name} shard", exact_floats=True)


def test_packed_then_sparse_metric_segment(engine):
    """The first segment's metric is dense (packed cells), the second's sparse (a present bitset: value counts split
    from doc counts mid-request, f64 cells for that segment)."""
    rng = np.random.default_rng(43)
    t0 = 1_441_065_600_000
    c1 = _log_segment(rng, 900_000, t0, 86_400_000)
    c2 = _log_segment(rng, 600_000, t0 + 86_400_000, 86_400_000)
    pres = rng.random(600_000) < 0.8
    c2["rt"]["present"] = bits_from_mask(pres)
    aggs = [AB.terms("h").field("host").size(7).subAggregation(
        AB.dateHistogram("d").field("@timestamp").interval("1h").subAggregation(AB.stats("s").field("rt")))]
    vals2 = c2["rt"]["values"].copy()
    vals2[~pres] = 0
    c2["rt"]["values"] = vals2
    allc = {f: dict(c1[f], values=np.concatenate([c1[f]["values"], c2[f]["values"]])) for f in c1}
    allc["rt"]["present"] = bits_from_mask(np.concatenate([np.ones(900_000, dtype=bool), pres]))
    want = O.run([(allc, 1_500_000)], aggs)
    segs = [engine.upload_segment(c1, 900_000), engine.upload_segment(c2, 600_000)]
    res, _ = _run(engine, None, aggs, segs=segs)
    for s in segs:
        s.close()
    assert_same(res.to_dict(), want["shards"][0], "shard")


@pytest.mark.parametrize("name", ["compact", "packed"])
@pytest.mark.parametrize("dead", [0.0, 0.3])
def test_packed_cells_through_folded_filters(engine, name, dead):
    """Packed cells under a filter read one accept bitset into which the host folds the request's clauses and the live
    docs first (VK bit 512): config 5's clauses (a 16-bit status range, a 32-bit bytes range) with and without 30 % of the
    docs deleted, terms{date_histogram{avg}} and terms{stats}, against the oracle; the compact layout (f64 cells,
    clauses evaluated in the loader) runs the same request."""
    n = 6_000_000
    cols = synthetic_columns(C5_FIELDS, n, shard=4)
    rng = np.random.default_rng(44)
    accept = None
    if dead:
        accept = bits_from_mask(rng.random(n) >= dead)
    aggs = C5_AGGS + [AB.terms("hs").field("host").size(15).subAggregation(AB.stats("s").field("response_time_ms"))]
    want = O.run([(cols, n)], aggs, filters=C5_FILTERS, number_of_shards=8, accept=[accept] if accept is not None else None)
    with layout(engine, name):
        seg = engine.synthetic_segment(n, fields=C5_FIELDS, shard=4)
        plan = engine.plan(aggs, filters=C5_FILTERS, number_of_shards=8)
        plan.collect(seg, accept_bits=accept)
        res = plan.build()
        plan.close()
        seg.close()
    assert_same(res.to_dict(), want["shards"][0], f"{name} dead {dead}")


def test_released_wide_columns_rebuilt_on_demand(engine):
    """esgpu_segment_release_wide (HBM footprint): after the north star built the segment's compact
    copies, the upload-width timestamp and metric columns are freed (16 B per doc); the north star runs again from the
    copies alone (no rebuild: the HBM in use stays down), then requests whose kernels read the upload-width values -- a
    monthly calendar histogram (bucket-start table over the raw timestamps), cardinality of a long field, terms with
    extended_stats (the metric's 32-bit deltas, rebuilt from the 16-bit ones through the wide column) -- rebuild them from
    the deltas and still match the oracle."""
    n = 3_000_000
    fields = ("host", "@timestamp", "response_time_ms", "bytes")
    cols = synthetic_columns(fields, n, shard=6)
    seg = engine.synthetic_segment(n, fields=fields, shard=6)
    res, _ = _run(engine, seg, NS_AGGS)
    want = O.run([(cols, n)], NS_AGGS)
    assert_same(res.to_dict(), want["shards"][0], "before release")
    used0 = engine.hbm_used()
    freed = seg.release_wide()
    assert freed >= 16 * n, freed  # timestamps and response times (bytes has no compact copy yet)
    assert engine.hbm_used() <= used0 - freed
    res, _ = _run(engine, seg, NS_AGGS)
    assert_same(res.to_dict(), want["shards"][0], "after release")
    assert engine.hbm_used() <= used0 - freed  # the compact copies sufficed
    wide_aggs = [AB.dateHistogram("m").field("@timestamp").interval("month").subAggregation(AB.stats("s").field("response_time_ms")),
                 AB.terms("h").field("host").size(5).subAggregation(AB.extendedStats("x").field("response_time_ms")),
                 AB.cardinality("c").field("response_time_ms"),
                 AB.histogram("rt").field("response_time_ms").interval(100).subAggregation(AB.avg("b").field("bytes"))]
    res, _ = _run(engine, seg, wide_aggs)
    assert_same(res.to_dict(), O.run([(cols, n)], wide_aggs)["shards"][0], "rebuilt")
    seg.close()
