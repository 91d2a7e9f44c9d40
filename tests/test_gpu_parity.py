"""GPU parity: the gfx950 path (through the C-ABI) against the CPU oracle on the same seeded inputs.

Each case builds one request with the reference's builder API, runs it on the GPU (device-generated or uploaded
segment) and through the oracle (host-generated copies of the same columns), and compares the shard-level and the
reduced InternalAggregations with tests/helpers.assert_same (counts/keys/registers bit-exact, floats bit-exact for
integer-valued metrics, 1e-12 relative otherwise).
"""
import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, QueryBuilders as QB
from elasticsearch_amd import _native as N
from elasticsearch_amd import reduce, synthetic_host_column
from helpers import assert_same, bits_from_mask, synthetic_columns

pytestmark = pytest.mark.gpu


def run_both(engine, aggs, fields, num_docs, shard=0, filters=None, exact=True, upload=False, accept=None):
    cols = synthetic_columns(fields, num_docs, shard=shard)
    want = O.run([(cols, num_docs)], aggs, filters=filters, accept=[accept] if accept is not None else None)
    if upload:
        seg = engine.upload_segment(cols, num_docs)
    else:
        seg = engine.synthetic_segment(num_docs, fields=fields, shard=shard)
    plan = engine.plan(aggs, filters=filters)
    plan.collect(seg, accept_bits=accept)
    shard_res = plan.build()
    got_shard = shard_res.to_dict()
    got_red = reduce([shard_res]).to_dict()
    assert_same(got_shard, want["shards"][0], "shard", exact)
    assert_same(got_red, want["reduced"], "reduced", exact)
    plan.close()
    seg.close()
    return got_red


def test_device_generator_matches_host(engine):
    n = 300_000
    fields = ("@timestamp", "host", "status", "response_time_ms", "bytes", "client_ip.hash", "price")
    seg = engine.synthetic_segment(n, fields=fields, shard=3)
    for f in fields:
        host = synthetic_host_column(f, n, shard=3)
        dev = seg.read_column(f, 0, n, host.dtype)
        assert np.array_equal(dev.view(np.uint8), host.view(np.uint8)), f
    ts = synthetic_host_column("@timestamp", n, shard=3)
    assert np.all(np.diff(ts) >= 0)


def test_config1_terms_stats(engine):  # terms(host){stats(response_time_ms)} on 1M docs
    aggs = [AB.terms("hosts").field("host").subAggregation(AB.stats("rt").field("response_time_ms"))]
    run_both(engine, aggs, ("host", "response_time_ms"), 1_000_000)


def test_config2_date_histogram_extended_stats(engine):  # date_histogram(1h){extended_stats}
    aggs = [AB.dateHistogram("per_hour").field("@timestamp").interval("1h")
            .subAggregation(AB.extendedStats("rt").field("response_time_ms"))]
    r = run_both(engine, aggs, ("@timestamp", "response_time_ms"), 2_000_000)
    assert len(r["per_hour"]["buckets"]) == 720


def test_north_star_terms_date_histogram_stats(engine):  # terms(host){date_histogram(1h){stats}}
    aggs = [AB.terms("hosts").field("host").size(10).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("response_time_ms")))]
    run_both(engine, aggs, ("host", "@timestamp", "response_time_ms"), 3_000_000)


def test_north_star_windowed_many_terms(engine):  # shard_size 1000: every host, forces the LDS key window
    aggs = [AB.terms("hosts").field("host").size(1000).subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(
            AB.extendedStats("rt").field("response_time_ms")))]
    run_both(engine, aggs, ("host", "@timestamp", "response_time_ms"), 1_500_000)


def test_config5_filtered_nested_avg(engine):  # bool.filter[term, range] -> terms{date_histogram{avg}}
    aggs = [AB.terms("hosts").field("host").subAggregation(
        AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.avg("rt").field("response_time_ms")))]
    filters = [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)]
    run_both(engine, aggs, ("host", "@timestamp", "response_time_ms", "status", "bytes"), 2_000_000, filters=filters)


def test_config3_high_cardinality_terms(engine):  # terms(url) over 10M global ordinals, shard_size 80
    aggs = [AB.terms("urls").field("url").size(10)]
    cols = synthetic_columns(("url",), 3_000_000)
    want = O.run([(cols, 3_000_000)], aggs, number_of_shards=8)
    seg = engine.synthetic_segment(3_000_000, fields=("url",))
    plan = engine.plan(aggs, number_of_shards=8)
    plan.collect(seg)
    got = plan.build().to_dict()
    assert_same(got, want["shards"][0], "shard")


@pytest.mark.parametrize("n", [1_000, 40_000, 2_000_000])
def test_config4_cardinality(engine, n):  # cardinality(client_ip.hash, precision_threshold 40000): LC and HLL modes
    aggs = [AB.cardinality("ips").field("client_ip.hash").precisionThreshold(40000)]
    r = run_both(engine, aggs, ("client_ip.hash",), n)
    assert r["ips"]["_internal"]["mode"] == ("lc" if n <= 40_000 else "hll")


def test_cardinality_default_precision_keyword(engine):  # cardinality on a keyword field (murmur3 of term bytes)
    run_both(engine, [AB.cardinality("hosts").field("host")], ("host",), 500_000)


def test_float_stress_sums(engine):  # non-integer doubles: sums compared at 1e-12 relative
    aggs = [AB.dateHistogram("d").field("@timestamp").interval("1d").subAggregation(AB.extendedStats("p").field("price")),
            AB.terms("hosts").field("host").subAggregation(AB.stats("p").field("price"))]
    run_both(engine, aggs, ("@timestamp", "host", "price"), 1_000_000, exact=False)


def test_histogram_interval_offset_and_orders(engine):
    aggs = [AB.histogram("rt_hist").field("response_time_ms").interval(50).offset(7).subAggregation(AB.avg("b").field("bytes")),
            AB.terms("hosts_asc").field("host").size(7).order(Order.count(True)),
            AB.terms("hosts_term").field("host").size(5).order(Order.term(False)),
            AB.dateHistogram("tz").field("@timestamp").interval("1d").timeZone("+05:30").minDocCount(1)]
    run_both(engine, aggs, ("host", "@timestamp", "response_time_ms", "bytes"), 800_000)


def test_date_histogram_then_terms(engine):  # date_histogram(1d){terms(host){stats}}
    aggs = [AB.dateHistogram("days").field("@timestamp").interval("1d").subAggregation(
        AB.terms("hosts").field("host").size(3).subAggregation(AB.stats("rt").field("response_time_ms")))]
    run_both(engine, aggs, ("host", "@timestamp", "response_time_ms"), 1_000_000)


def test_missing_values_min_doc_count_zero_and_accept_bits(engine):
    n = 200_003  # ragged: not a multiple of the 8192-doc block
    rng = np.random.default_rng(11)
    cols = synthetic_columns(("host", "@timestamp", "response_time_ms"), n)
    host = cols["host"]["values"].copy()
    host[rng.random(n) < 0.1] = 0xFFFFFFFF  # missing keyword values
    cols["host"]["values"] = host
    cols["@timestamp"]["present"] = bits_from_mask(rng.random(n) >= 0.05)
    cols["response_time_ms"]["present"] = bits_from_mask(rng.random(n) >= 0.2)
    accept = bits_from_mask(rng.random(n) < 0.7)
    aggs = [AB.terms("hosts").field("host").size(20).minDocCount(0).subAggregation(
                AB.dateHistogram("h").field("@timestamp").interval("6h").subAggregation(AB.stats("rt").field("response_time_ms"))),
            AB.dateHistogram("days").field("@timestamp").interval("1d").extendedBounds(1440000000000, 1444000000000)
            .subAggregation(AB.terms("hosts").field("host").size(2)),
            AB.extendedStats("all_rt").field("response_time_ms"),
            AB.cardinality("card").field("host")]
    want = O.run([(cols, n)], aggs, accept=[accept])
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs)
    plan.collect(seg, accept_bits=accept)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")


def test_empty_segment_and_unmapped_fields(engine):
    cols = {"host": {"type": N.COL_ORD_U32, "values": np.zeros(0, np.uint32), "terms": []}}
    aggs = [AB.terms("t").field("host"), AB.terms("unmapped").field("nope"), AB.stats("s").field("nope"),
            AB.dateHistogram("d").field("nope").interval("1h"), AB.cardinality("c").field("nope")]
    want = O.run([(cols, 0)], aggs)
    seg = engine.upload_segment(cols, 0)
    plan = engine.plan(aggs)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")


def test_multi_shard_reduce_matches_oracle(engine):  # 4 shards, one plan per shard, host-side coordinator reduce
    n = 250_000
    fields = ("host", "@timestamp", "response_time_ms", "client_ip.hash")
    aggs = [AB.terms("hosts").field("host").size(5).subAggregation(
                AB.dateHistogram("h").field("@timestamp").interval("1d").subAggregation(AB.stats("rt").field("response_time_ms"))),
            AB.cardinality("ips").field("client_ip.hash").precisionThreshold(1000)]
    shards = [(synthetic_columns(fields, n, shard=s), n) for s in range(4)]
    want = O.run(shards, aggs, number_of_shards=4)
    results = []
    for s in range(4):
        seg = engine.synthetic_segment(n, fields=fields, shard=s)
        plan = engine.plan(aggs, number_of_shards=4)
        plan.collect(seg)
        r = plan.build()
        assert_same(r.to_dict(), want["shards"][s], f"shard{s}")
        results.append(r)
    assert_same(reduce(results).to_dict(), want["reduced"], "reduced")


def test_plan_reset_reuse_and_multi_segment(engine):  # two segments into one plan == oracle over the concatenation
    n = 300_000
    fields = ("host", "@timestamp", "response_time_ms")
    cols = synthetic_columns(fields, 2 * n)
    halves = []
    for h in range(2):
        part = {}
        for f, c in cols.items():
            d = dict(c)
            d["values"] = c["values"][h * n:(h + 1) * n]
            part[f] = d
        halves.append(part)
    aggs = [AB.terms("hosts").field("host").subAggregation(
        AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("response_time_ms")))]
    want = O.run([(cols, 2 * n)], aggs)
    plan = engine.plan(aggs)
    for rep in range(2):
        segs = [engine.upload_segment(halves[h], n) for h in range(2)]
        for s in segs:
            plan.collect(s)
        assert_same(plan.build().to_dict(), want["shards"][0], f"rep{rep}")
        plan.reset()


@pytest.mark.parametrize("order", [Order.count(False), Order.count(True), Order.term(True), Order.term(False)])
def test_high_cardinality_partitioned_orders(engine, order):
    """valueCount 70,000 (> LDS): partitioned counting + GPU top-k; a 40 % hot term spans several counting chunks."""
    n, T = 3_000_000, 70_000
    rng = np.random.default_rng(5)
    ords = rng.integers(0, T, size=n, dtype=np.uint32)
    ords[rng.random(n) < 0.4] = 5
    ords[rng.random(n) < 0.05] = 0xFFFFFFFF  # missing
    terms = ["t%06d" % i for i in range(T)]
    status = rng.integers(0, 3, size=n).astype(np.int64)
    cols = {"kw": {"type": N.COL_ORD_U32, "values": ords, "terms": terms},
            "status": {"type": N.COL_I64, "values": status}}
    aggs = [AB.terms("kw").field("kw").size(25).order(order),
            AB.terms("kw0").field("kw").size(7).minDocCount(0).order(order)]
    flt = [QB.rangeQuery("status").gte(1)]
    want = O.run([(cols, n)], aggs, filters=flt)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs, filters=flt)
    plan.collect(seg)
    _, _, path = plan.last_collect_stats()
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard")
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced")


def test_multi_segment_global_ordinals(engine):
    """Three segments with different term dictionaries (GlobalOrdinalsBuilder / OrdinalMap): the
    GPU-remapped global ordinals give the same shard result as one segment over the concatenated docs with the
    merged dictionary; a keyword term filter resolves its term through the global dictionary."""
    rng = np.random.default_rng(11)
    universe = sorted("kw-%05d-%s" % (i, "x" * (i % 3)) for i in range(4000))
    sizes = [200_000, 150_001, 250_003]
    segs_cols, dicts, concat = [], [], {"kw": [], "@timestamp": [], "response_time_ms": []}
    t0 = 1441065600000
    for k, n in enumerate(sizes):
        d = sorted(rng.choice(universe, size=1500 + 400 * k, replace=False).tolist())
        ranks = np.minimum(rng.zipf(1.3, size=n) - 1, len(d) - 1).astype(np.uint32)
        ords = rng.permutation(len(d)).astype(np.uint32)[ranks]
        ords[rng.random(n) < 0.03] = 0xFFFFFFFF  # missing
        ts = np.sort(rng.integers(t0, t0 + 3 * 86_400_000, size=n)).astype(np.int64)
        rt = rng.integers(0, 1000, size=n).astype(np.int64)
        segs_cols.append({"kw": {"type": N.COL_ORD_U32, "values": ords, "terms": d},
                          "@timestamp": {"type": N.COL_I64, "values": ts},
                          "response_time_ms": {"type": N.COL_I64, "values": rt}})
        dicts.append(d)
        concat["kw"].append([d[o] if o != 0xFFFFFFFF else None for o in ords])
        concat["@timestamp"].append(ts)
        concat["response_time_ms"].append(rt)
    gdict = sorted(set().union(*dicts))
    gindex = {t: i for i, t in enumerate(gdict)}
    gords = np.array([gindex[t] if t is not None else 0xFFFFFFFF for part in concat["kw"] for t in part], dtype=np.uint32)
    total = sum(sizes)
    one = {"kw": {"type": N.COL_ORD_U32, "values": gords, "terms": gdict},
           "@timestamp": {"type": N.COL_I64, "values": np.concatenate(concat["@timestamp"])},
           "response_time_ms": {"type": N.COL_I64, "values": np.concatenate(concat["response_time_ms"])}}
    segs = [engine.upload_segment(c, n) for c, n in zip(segs_cols, sizes)]
    omap = engine.ordinal_map(segs, "kw")
    assert omap.value_count == len(gdict)
    probe = dicts[1][7]
    assert omap.lookup(probe) == gindex[probe] and omap.lookup("no-such-term") == -1
    requests = [
        ([AB.terms("t").field("kw").size(15).subAggregation(
            AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.stats("rt").field("response_time_ms")))],
         None),
        ([AB.terms("t").field("kw").size(5).order(Order.term(False)).subAggregation(AB.avg("a").field("response_time_ms"))],
         None),
        ([AB.dateHistogram("h").field("@timestamp").interval("6h").subAggregation(AB.terms("t").field("kw").size(3))],
         [QB.termQuery("kw", probe)]),
    ]
    for aggs, flt in requests:
        want = O.run([(one, total)], aggs, filters=flt, ord_lookup=lambda f, t: gindex.get(t, -1))
        plan = engine.plan(aggs, filters=flt, ord_lookup=lambda f, t: omap.lookup(t))
        for s in segs:
            plan.collect(s)
        shard = plan.build()
        assert_same(shard.to_dict(), want["shards"][0], "shard")
        assert_same(reduce([shard]).to_dict(), want["reduced"], "reduced")
        plan.close()
    omap.close()
    for s in segs:
        s.close()


def test_histogram_over_double_field(engine):
    """HistogramAggregator over a double field buckets (long) value (ValuesSource.Numeric.longValues ->
    FieldData.castToLong): truncation toward zero, NaN -> 0."""
    n = 400_000
    rng = np.random.default_rng(21)
    x = (rng.standard_normal(n) * 300.0).astype(np.float64)
    x[rng.random(n) < 0.001] = np.nan
    x[:3] = [-0.5, 0.5, -99.99]
    present = rng.random(n) < 0.9
    cols = {"x": {"type": N.COL_F64, "values": x, "present": bits_from_mask(present)},
            "rt": {"type": N.COL_I64, "values": rng.integers(0, 1000, size=n).astype(np.int64)}}
    aggs = [AB.histogram("hx").field("x").interval(25).offset(3).subAggregation(AB.stats("rt").field("rt")),
            AB.histogram("hx0").field("x").interval(100).minDocCount(0).subAggregation(AB.extendedStats("x").field("x"))]
    want = O.run([(cols, n)], aggs)
    seg = engine.upload_segment(cols, n)
    plan = engine.plan(aggs)
    plan.collect(seg)
    res = plan.build()
    assert_same(res.to_dict(), want["shards"][0], "shard", False)
    assert_same(reduce([res]).to_dict(), want["reduced"], "reduced", False)
    plan.close()
    seg.close()


def test_keyword_range_filters(engine):
    """RangeQuery on a keyword field (TermRangeQuery over BytesRef order) becomes an ordinal range of the sorted
    dictionary: inclusive / exclusive / open bounds, bounds that are not terms, an empty range, and the partitioned
    high-cardinality path."""
    n = 600_000
    fields = ("host", "@timestamp", "response_time_ms", "url")
    cases = [
        [QB.rangeQuery("host").gte("host-0100").lt("host-0500")],
        [QB.rangeQuery("host").gt("host-0100").lte("host-0500x")],
        [QB.rangeQuery("host").gt("host-09")],
        [QB.rangeQuery("host").lt("host-0002"), QB.termQuery("host", "host-0001")],
        [QB.rangeQuery("host").gte("zzz")],
        [QB.rangeQuery("url").gte("/p/00100000").lt("/p/00800000")],
    ]
    aggs = [AB.terms("hosts").field("host").size(20).subAggregation(AB.stats("rt").field("response_time_ms")),
            AB.dateHistogram("d").field("@timestamp").interval("1d"),
            AB.terms("urls").field("url").size(10)]
    cols = synthetic_columns(fields, n)
    hosts = ["host-%04d" % i for i in range(1000)]
    lookup = lambda f, t: hosts.index(t) if f == "host" and t in hosts else -1  # noqa: E731
    seg = engine.synthetic_segment(n, fields=fields)
    for flt in cases:
        want = O.run([(cols, n)], aggs, filters=flt, ord_lookup=lookup)
        plan = engine.plan(aggs, filters=flt, ord_lookup=lookup)
        plan.collect(seg)
        assert_same(plan.build().to_dict(), want["shards"][0], "shard")
        plan.close()
    seg.close()


def test_index_time_hashing(engine):
    """Bulk ingest helpers on the GPU: shard routing of _ids (Murmur3HashFunction + MathUtils.mod) against the oracle,
    and murmur3 field values against MurmurHash3.hash128(...).h1 -- the device-generated client_ip.hash column is the
    murmur3 field of the generated IP strings."""
    import ctypes
    from test_oracle_kat import oracle_routing_hash, oracle_shard_id
    rng = np.random.default_rng(17)
    ids = ["doc-%d-%s" % (i, "x" * int(rng.integers(0, 9))) for i in range(20_000)] + ["", "é中\U0001F600"]
    for nshards in (1, 5, 8):
        shards, hashes = engine.route_shards(ids, nshards, with_hashes=True)
        for i in range(0, len(ids), 97):
            h = oracle_routing_hash(ids[i])
            assert hashes[i] == h and shards[i] == oracle_shard_id(h, nshards), ids[i]
        assert shards.min() >= 0 and shards.max() < nshards
    vals = ["10.%d.%d.%d" % tuple(rng.integers(0, 256, size=3)) for _ in range(5000)] + ["", "a" * 37]
    got = engine.murmur3_field(vals)
    L = O.lib()
    for i, v in enumerate(vals):
        b = v.encode()
        h1, h2 = ctypes.c_uint64(), ctypes.c_uint64()
        L.oracle_murmur3_128(b, len(b), 0, ctypes.byref(h1), ctypes.byref(h2))
        assert int(got[i]) == h1.value, v


def test_rccl_gather_reduce_single_rank(engine):  # the bench's N > 1 exchange (esgpu_comm_*) on a one-rank communicator
    from elasticsearch_amd import Communicator
    n = 200_000
    fields = ("host", "@timestamp", "response_time_ms", "client_ip.hash")
    aggs = [AB.terms("hosts").field("host").size(5).subAggregation(
                AB.dateHistogram("h").field("@timestamp").interval("1d").subAggregation(AB.stats("rt").field("response_time_ms"))),
            AB.cardinality("ips").field("client_ip.hash").precisionThreshold(1000)]
    want = O.run([(synthetic_columns(fields, n), n)], aggs)
    comm = Communicator(engine, 1, 0, Communicator.unique_id())
    seg = engine.synthetic_segment(n, fields=fields)
    plan = engine.plan(aggs)
    for _ in range(2):  # communicator buffers are reused across requests
        plan.reset()
        plan.collect(seg)
        got = comm.gather_reduce(plan.build()).to_dict()
        assert_same(got, want["reduced"], "rccl reduced")
    plan.close()
    seg.close()
    # esgpu_comm_reduce over RCCL with two local shards: all-reduce for the fixed-shape aggregations (histogram with
    # metrics, top-level stats, cardinality), all-gather for terms; == the oracle's two-shard coordinator reduce
    aggs2 = aggs + [AB.dateHistogram("days").field("@timestamp").interval("1d").minDocCount(0).subAggregation(
        AB.extendedStats("rt").field("response_time_ms")), AB.stats("all").field("response_time_ms")]
    want2 = O.run([(synthetic_columns(fields, n, shard=s), n) for s in range(2)], aggs2, number_of_shards=2)
    plan = engine.plan(aggs2, number_of_shards=2)
    locals_ = []
    for s in range(2):
        seg = engine.synthetic_segment(n, fields=fields, shard=s)
        plan.reset()
        plan.collect(seg)
        locals_.append(plan.build())
        seg.close()
    got = comm.reduce(locals_).to_dict()
    assert_same(got, want2["reduced"], "rccl comm reduce")
    ar_bytes, _, _ = comm.last_exchange()
    assert ar_bytes >= (1 << 10)  # the registers went through ncclAllReduce(max)
    plan.close()
    comm.close()


def test_filter_aggregation(engine):  # FilterAggregator: top-level filter{...} beside unfiltered siblings, under a query
    n = 300_001
    fields = ("host", "@timestamp", "response_time_ms", "status", "bytes", "client_ip.hash")
    aggs = [AB.filter("ok_small", [QB.termQuery("status", 200), QB.rangeQuery("bytes").gte(1024).lte(65536)]).subAggregation(
                AB.terms("hosts").field("host").size(5).subAggregation(
                    AB.dateHistogram("h").field("@timestamp").interval("1d").subAggregation(AB.avg("rt").field("response_time_ms")))
            ).subAggregation(AB.stats("rt_all").field("response_time_ms")).subAggregation(
                AB.cardinality("ips").field("client_ip.hash").precisionThreshold(100)),
            AB.filter("errors", QB.rangeQuery("status").gte(500)),
            AB.terms("all_hosts").field("host").size(3)]
    run_both(engine, aggs, fields, n, filters=[QB.rangeQuery("response_time_ms").lt(900)])
    run_both(engine, aggs, fields, n)  # no query clauses: only the filters' own


def test_fixed_shape_shards_collected_into_one_plan(engine):
    """esgpu_plan_shard_mergeable: a request without terms may collect several shards into one plan (bench.py
    --shards S on fewer GPUs); its one shard result reduces to what the reduce of the separate shard results gives."""
    n = 300_000
    fields = ("@timestamp", "response_time_ms", "client_ip.hash")
    aggs = [AB.dateHistogram("h").field("@timestamp").interval("1h").minDocCount(3).subAggregation(
                AB.extendedStats("rt").field("response_time_ms")).subAggregation(
                AB.cardinality("ips").field("client_ip.hash").precisionThreshold(200)),
            AB.cardinality("all_ips").field("client_ip.hash").precisionThreshold(40000),
            AB.avg("rt").field("response_time_ms")]
    shards = [(synthetic_columns(fields, n, shard=s), n) for s in range(3)]
    want = O.run(shards, aggs, number_of_shards=3)
    plan = engine.plan(aggs, number_of_shards=3)
    assert plan.shard_mergeable()
    assert not engine.plan([AB.terms("t").field("host")]).shard_mergeable()
    segs = [engine.synthetic_segment(n, fields=fields, shard=s) for s in range(3)]
    for s in segs:
        plan.collect(s)
    assert_same(reduce([plan.build()]).to_dict(), want["reduced"], "merged shards")
    plan.close()
    for s in segs:
        s.close()
