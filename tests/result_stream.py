"""Test-side encoder of the libesgpu shard-result stream (esgpu_result_serialize format, version 5, esgpu_results.cpp).

Lets CPU tests hand-build shard-level InternalAggregations (the way the reference's unit tests construct
StringTerms / InternalHistogram / InternalCardinality objects) and push them through esgpu_result_deserialize +
esgpu_reduce without a GPU.  Aggregations are written row-wise here (one dict per instance, buckets carrying their
sub-aggregations) and turned into the library's columnar blocks (one block per spec, arrays over all instances).
"""
import struct

from elasticsearch_amd import _native as N

MAGIC = 0x45534750
VERSION = 5
BUCKET_TYPES = (N.AGG_TERMS, N.AGG_HISTOGRAM, N.AGG_DATE_HISTOGRAM)


def _str(b, s):
    data = s.encode("utf-8") if isinstance(s, str) else bytes(s)
    b += struct.pack("<Q", len(data)) + data


def _vec(b, fmt, xs):
    xs = list(xs)
    b += struct.pack("<Q", len(xs)) + (struct.pack("<%d%s" % (len(xs), fmt), *xs) if xs else b"")


def _fmt(b, a):
    """time zone id, ESGPU_FORMAT_* and pattern (version 5)"""
    _str(b, a.get("time_zone", "UTC"))
    b += struct.pack("<i", a.get("value_format", N.FORMAT_RAW))
    _str(b, a.get("format", ""))


def _block(b, insts):
    """One block from a non-empty list of same-spec instance dicts (the first one supplies the parameters)."""
    a = insts[0]
    t = a["type"]
    b += struct.pack("<ii", t, a.get("order", 0))
    _str(b, a["name"])
    b += struct.pack("<iiqii", a.get("required_size", 10), a.get("shard_size", 10), a.get("min_doc_count", 1),
                     a.get("show_err", 0), a.get("keyed", 0))
    b += struct.pack("<Biqq", a.get("has_empty_info", 0), a.get("date_unit", 0), a.get("interval", 1), a.get("offset", 0))
    _vec(b, "q", a.get("tz_starts", []))
    _vec(b, "q", a.get("tz_offs", []))
    b += struct.pack("<BBqq", a.get("has_bmin", 0), a.get("has_bmax", 0), a.get("bmin", 0), a.get("bmax", 0))
    b += struct.pack("<di", a.get("sigma", 2.0), a.get("precision", 14))
    _str(b, a.get("order_path", ""))
    _fmt(b, a)
    b += struct.pack("<Q", len(insts))
    bucket = t in BUCKET_TYPES
    buckets = [bk for x in insts for bk in x.get("buckets", [])] if bucket else []
    _vec(b, "q", [x.get("doc_count_error", 0) for x in insts] if bucket else [])
    _vec(b, "q", [x.get("other_doc_count", 0) for x in insts] if bucket else [])
    offs = [0]
    for x in insts:
        offs.append(offs[-1] + len(x.get("buckets", [])))
    _vec(b, "Q", offs if bucket else [])
    _vec(b, "q", [bk.get("key", 0) for bk in buckets])
    terms = [bk.get("term", b"") for bk in buckets]
    terms = [s.encode("utf-8") if isinstance(s, str) else bytes(s) for s in terms]
    toff = [0]
    for s in terms:
        toff.append(toff[-1] + len(s))
    _vec(b, "Q", toff if bucket else [])
    _str(b, b"".join(terms))
    _vec(b, "q", [bk["doc_count"] for bk in buckets])
    _vec(b, "q", [bk.get("doc_count_error", 0) for bk in buckets])
    # sub-aggregations: spec j of every bucket forms one block (all buckets carry the same spec list)
    nsubs = len(a.get("sub_specs", buckets[0].get("subs", []) if buckets else []))
    b += struct.pack("<I", nsubs)
    for j in range(nsubs):
        rows = [bk["subs"][j] for bk in buckets]
        _block(b, rows) if rows else _empty_block(b, a["sub_specs"][j])
    empty = a.get("empty_subs", [])
    b += struct.pack("<I", len(empty))
    for e in empty:
        _block(b, [e])
    metric = t in (N.AGG_STATS, N.AGG_EXTENDED_STATS, N.AGG_AVG)
    _vec(b, "q", [x.get("count", 0) for x in insts] if metric else [])
    _vec(b, "d", [x.get("sum", 0.0) for x in insts] if metric else [])
    _vec(b, "d", [x.get("min", float("inf")) for x in insts] if metric else [])
    _vec(b, "d", [x.get("max", float("-inf")) for x in insts] if metric else [])
    _vec(b, "d", [x.get("sumsq", 0.0) for x in insts] if metric else [])
    card = t == N.AGG_CARDINALITY
    _vec(b, "B", [x.get("hll_present", 0) for x in insts] if card else [])
    _vec(b, "i", [x.get("hll_mode", 0) for x in insts] if card else [])
    b += struct.pack("<Q", len(insts) if card else 0)
    for x in insts if card else []:
        _vec(b, "B", bytes(x.get("registers", b"")))
    b += struct.pack("<Q", len(insts) if card else 0)
    for x in insts if card else []:
        _vec(b, "I", sorted(x.get("lc", [])))


def _empty_block(b, spec):
    """A block with zero instances (a sub-aggregation of a bucket aggregation that has no buckets)."""
    s = dict(spec)
    t = s["type"]
    b += struct.pack("<ii", t, s.get("order", 0))
    _str(b, s["name"])
    b += struct.pack("<iiqii", s.get("required_size", 10), s.get("shard_size", 10), s.get("min_doc_count", 1),
                     s.get("show_err", 0), s.get("keyed", 0))
    b += struct.pack("<Biqq", s.get("has_empty_info", 0), s.get("date_unit", 0), s.get("interval", 1), s.get("offset", 0))
    _vec(b, "q", s.get("tz_starts", []))
    _vec(b, "q", s.get("tz_offs", []))
    b += struct.pack("<BBqq", s.get("has_bmin", 0), s.get("has_bmax", 0), s.get("bmin", 0), s.get("bmax", 0))
    b += struct.pack("<di", s.get("sigma", 2.0), s.get("precision", 14))
    _str(b, s.get("order_path", ""))
    _fmt(b, s)
    b += struct.pack("<Q", 0)
    bucket = t in BUCKET_TYPES
    _vec(b, "q", [])
    _vec(b, "q", [])
    _vec(b, "Q", [0] if bucket else [])
    _vec(b, "q", [])
    _vec(b, "Q", [0] if bucket else [])
    _str(b, b"")
    _vec(b, "q", [])
    _vec(b, "q", [])
    subs = s.get("sub_specs", [])
    b += struct.pack("<I", len(subs))
    for sub in subs:
        _empty_block(b, sub)
    empty = s.get("empty_subs", [])
    b += struct.pack("<I", len(empty))
    for e in empty:
        _block(b, [e])
    for _ in range(5):
        _vec(b, "q", [])
    _vec(b, "B", [])
    _vec(b, "i", [])
    b += struct.pack("<QQ", 0, 0)


def encode(aggs):
    b = bytearray(struct.pack("<II", MAGIC, VERSION))
    b += struct.pack("<I", len(aggs))
    for a in aggs:
        _block(b, [a])
    return bytes(b)


def string_terms(name, buckets, size=10, shard_size=10, order=N.ORDER_COUNT_DESC, min_doc_count=1, other=0):
    """Shard-level StringTerms as GlobalOrdinalsStringTermsAggregator.buildAggregation emits it (docCountError 0)."""
    return {"type": N.AGG_TERMS, "name": name, "order": order, "required_size": size, "shard_size": shard_size,
            "min_doc_count": min_doc_count, "other_doc_count": other,
            "buckets": [{"key": i, "term": t, "doc_count": c} for i, (t, c) in enumerate(buckets)]}


def cardinality(name, precision, registers=None, lc=None):
    if registers is None and lc is None:
        return {"type": N.AGG_CARDINALITY, "name": name, "precision": precision}
    if registers is not None:
        return {"type": N.AGG_CARDINALITY, "name": name, "precision": precision, "hll_present": 1, "hll_mode": 1,
                "registers": bytes(registers)}
    return {"type": N.AGG_CARDINALITY, "name": name, "precision": precision, "hll_present": 1, "hll_mode": 0,
            "lc": list(lc)}


def from_shard_json(aggs, shard_json, number_of_shards=1):
    """Shard-level JSON (the oracle's / esgpu_result_to_json schema) of a builder tree -> instance dicts for encode().

    Needs the `_internal` state the schema carries for metrics; cardinality sketches are not recoverable from JSON
    (only their fingerprints are), so trees containing cardinality are rejected."""
    from elasticsearch_amd.aggs import flatten
    arr, n, _keep = flatten(aggs, number_of_shards)
    specs = [arr[i] for i in range(n)]
    children = {i: [j for j in range(n) if specs[j].parent == i] for i in range(-1, n)}

    def params(i):
        s = specs[i]
        hist = s.type in (N.AGG_HISTOGRAM, N.AGG_DATE_HISTOGRAM)
        p = {"type": s.type, "name": s.name.decode(), "order": s.order, "sigma": s.sigma,
             "time_zone": (s.time_zone or b"UTC").decode(), "value_format": s.value_format,
             "format": (s.format or b"").decode()}
        if s.type == N.AGG_TERMS:
            p.update(required_size=s.size, shard_size=s.shard_size, min_doc_count=s.min_doc_count,
                     show_err=s.show_term_doc_count_error, order_path=(s.order_path or b"").decode())
        if hist:
            p.update(min_doc_count=s.min_doc_count, keyed=s.keyed, interval=s.interval, offset=s.offset,
                     date_unit=s.date_unit if s.type == N.AGG_DATE_HISTOGRAM else 0)
            if s.min_doc_count == 0:
                p.update(has_empty_info=1, has_bmin=s.has_extended_bounds_min, has_bmax=s.has_extended_bounds_max,
                         bmin=s.extended_bounds_min, bmax=s.extended_bounds_max,
                         empty_subs=[empty(c) for c in children[i]])
        if s.type == N.AGG_CARDINALITY:
            raise ValueError("cardinality state is not recoverable from JSON")
        if s.type in BUCKET_TYPES:
            p["sub_specs"] = [spec_tree(c) for c in children[i]]
        return p

    def spec_tree(i):
        return params(i)

    def empty(i):
        return params(i)  # no buckets / zero metrics == buildEmptyAggregation

    def inst(i, js):
        s = specs[i]
        p = params(i)
        if s.type == N.AGG_TERMS:
            p["doc_count_error"] = js["doc_count_error_upper_bound"]
            p["other_doc_count"] = js["sum_other_doc_count"]
        if s.type in BUCKET_TYPES:
            bks = []
            for k, b in enumerate(js["buckets"]):
                bk = {"doc_count": b["doc_count"], "doc_count_error": b.get("doc_count_error_upper_bound", 0),
                      "subs": [inst(c, b[specs[c].name.decode()]) for c in children[i]]}
                if s.type == N.AGG_TERMS:
                    bk.update(key=k, term=b["key"])
                else:
                    bk["key"] = b["key"]
                bks.append(bk)
            p["buckets"] = bks
        else:
            st = js["_internal"]
            p.update(count=st["count"], sum=st["sum"], min=st.get("min", float("inf")),
                     max=st.get("max", float("-inf")), sumsq=st.get("sum_of_squares", 0.0))
        return p

    return [inst(i, shard_json[specs[i].name.decode()]) for i in children[-1]]
