"""CPU tests of the product library without a GPU: the C-ABI loads and exports every declared symbol, the parser
helpers follow the reference, and the shard-level reduce (stream -> esgpu_reduce) matches the oracle, also when the
shard results travel between two processes (world_size 2, gloo)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as O
from elasticsearch_amd import AggregationBuilders as AB
from elasticsearch_amd import Order, ShardResult
from elasticsearch_amd import _native as N
from elasticsearch_amd import precision_from_threshold, reduce, synthetic_host_column, synthetic_terms
from elasticsearch_amd.aggs import thresholds
from helpers import assert_same
from result_stream import cardinality, encode, string_terms

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    with open(os.path.join(REPO, "include", "esgpu.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*int\s+(esgpu_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    names = declared_functions()
    assert len(names) >= 30
    for name in names:
        assert hasattr(lib, name), name
    assert {n for n, _, _ in N.SIGNATURES} == set(names)
    assert lib.esgpu_abi_version() == 7


def test_no_silent_cpu_fallback():
    """Without a GPU the product path refuses to run (ESGPU_ERR_NO_DEVICE), it never computes on the CPU."""
    import elasticsearch_amd as ea
    if ea.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(ea.NoDeviceError):
        ea.Engine(0)


def test_precision_and_murmur3_kats(kat):
    for v in kat["precision_from_threshold"]:
        assert precision_from_threshold(v["threshold"]) == v["precision"], v["cite"]
    out = (ctypes.c_uint64 * 2)()
    for v in kat["murmur3_x64_128"]:
        b = v["input"].encode()
        N.check(N.lib().esgpu_murmur3_x64_128(b, len(b), v["seed"], out))
        s64 = [x - (1 << 64) if x >> 63 else x for x in out]
        assert s64 == [v["h1"], v["h2"]], v["cite"]


def test_terms_thresholds_follow_reference():
    # TermsParser + BucketUtils.suggestShardSideQueueSize + BucketCountThresholds.ensureValidity
    assert thresholds(10, -1, -1, -1, N.ORDER_COUNT_DESC, 1) == (10, 10, 1, 0)
    assert thresholds(10, -1, -1, -1, N.ORDER_COUNT_DESC, 8) == (10, 80, 1, 0)
    assert thresholds(3, -1, -1, -1, N.ORDER_COUNT_DESC, 2) == (3, 10, 1, 0)
    assert thresholds(10, -1, -1, -1, N.ORDER_COUNT_DESC, 20) == (10, 100, 1, 0)
    assert thresholds(3, 3, -1, -1, N.ORDER_COUNT_DESC, 2) == (3, 3, 1, 0)
    assert thresholds(5, -1, -1, -1, N.ORDER_TERM_ASC, 4) == (5, 5, 1, 0)
    assert thresholds(0, 0, 2, 5, N.ORDER_COUNT_DESC, 1) == (2**31 - 1, 2**31 - 1, 2, 2)
    assert thresholds(10, 4, 0, -1, N.ORDER_COUNT_DESC, 3) == (10, 10, 0, 0)


def test_synthetic_generator_host_properties():
    n = 200_000
    ts = synthetic_host_column("@timestamp", n)
    assert np.all(np.diff(ts) >= 0) and ts[0] >= 1441065600000 and ts[-1] < 1441065600000 + 30 * 86400000
    host = synthetic_host_column("host", n)
    assert host.max() < 1000
    st = synthetic_host_column("status", n)
    assert abs(np.mean(st == 200) - 0.70) < 0.01
    rt = synthetic_host_column("response_time_ms", n)
    assert rt.min() >= 0 and rt.max() <= 999
    assert np.array_equal(synthetic_host_column("host", n, start=1000, count=50), host[1000:1050])
    assert synthetic_terms("host", 3) == ["host-0000", "host-0001", "host-0002"]
    import ctypes
    buf = ctypes.create_string_buffer(64)
    for o in (0, 7, 999, 9999, 10000, 123456, 2**32 - 1):  # the hand formatter against printf's "%04u" / "%08x"
        assert N.lib().esgpu_synthetic_term(N.SYNTH_FIELDS["host"], o, buf, 64) == len("host-%04u" % o)
        assert buf.value.decode() == "host-%04u" % o
        N.lib().esgpu_synthetic_term(N.SYNTH_FIELDS["url"], o, buf, 64)
        assert buf.value.decode() == "/p/%08x" % o
    ip = synthetic_host_column("client_ip.hash", 1000)
    assert len(np.unique(ip)) > 990


def _shard_size_results(kat, size, shard_size, nshards=2):
    """ShardSizeTestCase fixture: each shard's StringTerms, built from the oracle's shard-level output."""
    fx = kat["shard_size_terms"]
    shards = []
    for counts in fx["shards"]:
        keys = sorted(counts)
        vals = np.array([keys.index(k) for k in keys for _ in range(counts[k])], dtype=np.uint32)
        shards.append(({"key": {"type": N.COL_ORD_U32, "values": vals, "terms": keys}}, len(vals)))
    b = AB.terms("keys").field("key").size(size).order(Order.count(False))
    if shard_size is not None:
        b.shardSize(shard_size)
    want = O.run(shards, [b], number_of_shards=nshards)
    results = []
    for sh in want["shards"]:
        t = sh["keys"]
        sz, ssz, _, _ = thresholds(size, shard_size if shard_size is not None else -1, -1, -1, N.ORDER_COUNT_DESC, nshards)
        results.append(encode([string_terms("keys", [(x["key"], x["doc_count"]) for x in t["buckets"]], size=sz,
                                            shard_size=ssz, other=t["sum_other_doc_count"])]))
    return results, want


@pytest.mark.parametrize("case", [0, 1])
def test_reduce_shard_size_terms_matches_reference(kat, case):
    c = kat["shard_size_terms"]["cases"][case]
    blobs, want = _shard_size_results(kat, c["size"], c["shard_size"])
    red = reduce([ShardResult.deserialize(b) for b in blobs]).to_dict()
    assert_same(red, want["reduced"], "reduced")
    assert {x["key"]: x["doc_count"] for x in red["keys"]["buckets"]} == c["expect"], c["cite"]


def _hll_parts(p, hashes):
    """registers / encoded LC set of a hash list, computed with the oracle's HyperLogLogPlusPlus helpers."""
    L = O.lib()
    regs = np.zeros(1 << p, dtype=np.uint8)
    enc = set()
    for h in hashes:
        idx = L.oracle_index(int(h), p)
        regs[idx] = max(regs[idx], L.oracle_run_len(int(h), p))
        enc.add(L.oracle_encode_hash(int(h), p) & 0xFFFFFFFF)
    return regs, enc


@pytest.mark.parametrize("sizes", [(300, 500), (40_000, 35_000), (3_000, 120_000)])
def test_reduce_cardinality_merge_matches_single(sizes):
    """HyperLogLogPlusPlusTests.merge: merging shard sketches == one sketch over all values (LC/LC, LC->HLL, LC+HLL)."""
    L = O.lib()
    p = 14
    rng = np.random.default_rng(sum(sizes))
    vals = [rng.integers(0, 2**40, size=n) for n in sizes]
    hashes = [np.array([L.oracle_mix64(int(v)) for v in vs], dtype=np.uint64) for vs in vals]
    thr = int((1 << p) / 4 * 0.75)
    blobs = []
    for h in hashes:
        regs, enc = _hll_parts(p, h)
        blobs.append(encode([cardinality("c", p, lc=enc) if len(enc) <= thr else cardinality("c", p, registers=regs)]))
    red = reduce([ShardResult.deserialize(b) for b in blobs])
    allh = np.concatenate(hashes)
    mode = ctypes.c_int32()
    fnv = ctypes.c_uint64()
    want = L.oracle_hll_collect(p, allh.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(allh), ctypes.byref(mode),
                                ctypes.byref(fnv))
    got = red.to_dict()["c"]
    assert got["value"] == want
    assert got["_internal"]["mode"] == ("hll" if mode.value else "lc")
    if mode.value:
        assert int(got["_internal"]["registers_fnv1a64"], 16) == fnv.value


def _gloo_worker(rank, world, port, blobs, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    gathered = [None] * world
    dist.all_gather_object(gathered, blobs[rank])  # the shard results cross the process boundary as streams
    red = reduce([ShardResult.deserialize(b) for b in gathered])
    q.put((rank, red.to_json()))
    dist.destroy_process_group()


def test_two_rank_gloo_gather_reduce(kat):
    """N>1 path on CPU: two ranks exchange shard results (gloo stands in for the RCCL all-gather) and reduce in shard
    order; both ranks must agree with the oracle's coordinator reduce."""
    import json
    import socket

    import torch.multiprocessing as mp
    blobs, want = _shard_size_results(kat, 3, None)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, blobs, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for r in range(2):
        assert_same(json.loads(out[r]), want["reduced"], f"rank{r}")


def test_stream_roundtrip_and_json():
    blob = encode([string_terms("t", [("a", 5), ("b", 3)]), cardinality("c", 14)])
    r = ShardResult.deserialize(blob)
    assert r.serialize() == blob
    d = r.to_dict()
    assert [b["key"] for b in d["t"]["buckets"]] == ["a", "b"]
    assert d["c"]["value"] == 0 and d["c"]["_internal"]["present"] == 0
    with pytest.raises(N.EsGpuError):
        ShardResult.deserialize(b"garbage!")


# ---- date rounding (esgpu_date_rounding: Rounding / TimeZoneRounding with joda zone arithmetic) ----
def _date_spec(unit, interval=0, offset=0, zone=None):
    from elasticsearch_amd.aggs import tz_history
    sp = N.AggSpec()
    sp.type = N.AGG_DATE_HISTOGRAM
    sp.date_unit = unit
    sp.interval = interval
    sp.offset = offset
    keep = []
    if zone and zone != "UTC":
        starts, offs = tz_history(zone)
        st = (ctypes.c_int64 * len(starts))(*starts)
        of = (ctypes.c_int64 * len(offs))(*offs)
        keep += [st, of]
        sp.tz_starts = ctypes.cast(st, ctypes.POINTER(ctypes.c_int64))
        sp.tz_offsets_ms = ctypes.cast(of, ctypes.POINTER(ctypes.c_int64))
        sp.tz_count = len(starts)
    return sp, keep


def product_round(sp, op, v):
    out = ctypes.c_int64()
    N.check(N.lib().esgpu_date_rounding(ctypes.byref(sp), op, v, ctypes.byref(out)))
    return out.value


UNITS_BY_NAME = {"hour": N.UNIT_HOUR, "day": N.UNIT_DAY, "month": N.UNIT_MONTH, "year": N.UNIT_YEAR, "minute": N.UNIT_MINUTE,
                 "week": N.UNIT_WEEK}


def test_date_rounding_known_values(kat):  # the product's rounding on TimeZoneRoundingTests' UTC, fixed and DST KATs
    for c in kat["rounding"]:
        if c["kind"] == "histogram":
            continue
        unit = UNITS_BY_NAME[c["unit"]] if c["kind"] == "unit" else N.UNIT_NONE
        sp, _ = _date_spec(unit, c.get("interval", 0), c["offset"])
        for v, expect in c["round"]:
            assert product_round(sp, 0, v) == expect, c["cite"]
        for v, expect in c["next"]:
            assert product_round(sp, 1, v) == expect, c["cite"]
    for c in kat["rounding_tz"]["cases"]:
        sp, keep = _date_spec(UNITS_BY_NAME[c["unit"]], zone=c["zone"])
        for v, expect in c["round"]:
            assert product_round(sp, 0, v) == expect, c["cite"]
        for a, b in c.get("same", []):
            assert product_round(sp, 0, a) == product_round(sp, 0, b), c["cite"]
    c = kat["rounding_tz"]["lenient"]
    sp, keep = _date_spec(N.UNIT_MINUTE, zone=c["zone"])
    sp2, keep2 = _date_spec(N.UNIT_NONE, 60000, zone=c["zone"])
    for t in range(c["start"], c["end"], c["step"]):
        assert product_round(sp, 1, t) > t and product_round(sp2, 1, t) > t, c["cite"]


def test_date_rounding_matches_oracle_across_zones():
    """Product Rounding (es_rounding.hpp) == oracle Rounding (cpu_ref.cpp), two independent restatements, on random
    instants around DST transitions, for every unit, fixed intervals and offsets."""
    from test_oracle_kat import oracle_round_tz
    rng = np.random.default_rng(5)
    zones = ["Europe/Berlin", "America/Chicago", "Asia/Jerusalem", "America/Sao_Paulo", "Australia/Lord_Howe",
             "Asia/Kolkata", "UTC"]
    for i in range(1500):
        zone = zones[i % len(zones)]
        if i % 3 == 2:
            kind, unit, interval = 2, N.UNIT_NONE, int(rng.choice([60000, 900000, 5400000, 3600000 * 7, 86400000]))
        else:
            kind, unit, interval = 1, int(rng.integers(1, 9)), 0
        offset = int(rng.choice([0, 0, 3600000, -1800000]))
        base = int(rng.integers(0, 2 * 10**12))
        sp, keep = _date_spec(unit, interval, offset, zone)
        for v in (base, base - base % 3600000, base - base % 86400000 + 3600000 * int(rng.integers(0, 4))):
            for op in (0, 1, 2):
                assert product_round(sp, op, v) == oracle_round_tz(kind, unit, interval, offset, zone, op, v), \
                    (zone, kind, unit, interval, offset, op, v)


def test_routing_hash_matches_kats_and_oracle(kat):
    """Product Murmur3HashFunction (host path) == the reference's KATs, and == the oracle on random strings including
    odd lengths, non-ASCII and surrogate pairs (UTF-16 code units, as Java's String.charAt)."""
    from elasticsearch_amd import routing_hash
    from test_oracle_kat import oracle_routing_hash
    for v in kat["routing_murmur3_x86_32"]:
        assert routing_hash(v["input"]) == v["hash"], v["cite"]
    rng = np.random.default_rng(3)
    alphabet = list("abcdefghijklmnopqrstuvwxyz0123456789-_") + ["é", "ß", "中", "文", "\U0001F600"]
    for i in range(400):
        s = "".join(rng.choice(alphabet, size=int(rng.integers(0, 40))))
        assert routing_hash(s) == oracle_routing_hash(s), s


def test_filter_aggregation_plan_validation():
    """Filter aggregations compile on the GPU path at the top level only; clause owners must name filter specs."""
    from elasticsearch_amd import AggregationBuilders as AB
    from elasticsearch_amd import QueryBuilders as QB
    from elasticsearch_amd.aggs import flatten, flatten_filters
    aggs = [AB.filter("f", [QB.termQuery("status", 200)]).subAggregation(AB.avg("a").field("x")),
            AB.terms("t").field("host")]
    specs, n, _k1 = flatten(aggs)
    flt, nf, _k2 = flatten_filters([QB.rangeQuery("bytes").gte(1)], None, aggs)
    assert n == 3 and nf == 2
    assert [flt[i].owner for i in range(nf)] == [0, 1]  # query clause, then the clause of spec 0
    assert specs[0].type == N.AGG_FILTER and specs[1].parent == 0
    with pytest.raises(ValueError):
        flatten_filters(None, None, [AB.filter("nofilter")])
