"""Test-side decoder of Elasticsearch's transport bytes for shard-level aggregations: the readFrom side of
InternalAggregations (A/InternalAggregations.java:190-212) and of each class esgpu_result_to_stream writes, over
StreamInput's encodings (C/common/io/stream/StreamInput.java).  A = core/src/main/java/org/elasticsearch/search/
aggregations, C = core/src/main/java/org/elasticsearch.

decode(bytes) -> list of dicts, one per aggregation, in stream order; raises on trailing or missing bytes.
normalized(aggs) -> the same with every LINEAR_COUNTING hash list sorted (diagnostics: the set regardless of slot
order, a permutation; HyperLogLogPlusPlus.readFrom re-adds them to a set, HyperLogLogPlusPlus.java:537-547).
"""
import struct


class StreamInput:
    def __init__(self, data):
        self.b = bytes(data)
        self.i = 0

    def byte(self):
        if self.i >= len(self.b):
            raise EOFError("stream ends early")
        v = self.b[self.i]
        self.i += 1
        return v

    def sbyte(self):
        v = self.byte()
        return v - 256 if v > 127 else v

    def boolean(self):
        v = self.byte()
        if v not in (0, 1):
            raise ValueError("bad boolean %d" % v)
        return v == 1

    def vint(self):  # readVInt: at most 5 bytes
        v, shift = 0, 0
        for _ in range(5):
            b = self.byte()
            v |= (b & 0x7F) << shift
            if not b & 0x80:
                return v - (1 << 32) if v >= 1 << 31 else v
            shift += 7
        raise ValueError("vint too long")

    def vlong(self):  # readVLong: at most 9 bytes for non-negative values
        v, shift = 0, 0
        for _ in range(10):
            b = self.byte()
            v |= (b & 0x7F) << shift
            if not b & 0x80:
                return v - (1 << 64) if v >= 1 << 63 else v
            shift += 7
        raise ValueError("vlong too long")

    def raw(self, n):
        if self.i + n > len(self.b):
            raise EOFError("stream ends early")
        v = self.b[self.i:self.i + n]
        self.i += n
        return v

    def i32(self):
        return struct.unpack(">i", self.raw(4))[0]

    def i64(self):
        return struct.unpack(">q", self.raw(8))[0]

    def f64(self):
        return struct.unpack(">d", self.raw(8))[0]

    def bytes_ref(self):
        return self.raw(self.vint())

    def string(self):  # readString: char count, then each char in 1-3 bytes
        n = self.vint()
        chars = []
        for _ in range(n):
            c = self.byte()
            if c >> 4 in (0xC, 0xD):
                c = ((c & 0x1F) << 6) | (self.byte() & 0x3F)
            elif c >> 4 == 0xE:
                c = ((c & 0x0F) << 12) | ((self.byte() & 0x3F) << 6) | (self.byte() & 0x3F)
            chars.append(c)
        return struct.pack("<%dH" % len(chars), *chars).decode("utf-16-le", errors="surrogatepass")


def _formatter(s):  # ValueFormatterStreams.readOptional
    if not s.boolean():
        return None
    fid = s.byte()
    if fid == 1:
        return ("raw",)
    if fid == 2:
        return ("date_time", s.string(), s.string())
    if fid == 4:
        return ("number", s.string())
    raise ValueError("formatter id %d" % fid)


def _rounding(s):  # Rounding.Streams.read
    rid = s.byte()
    if rid == 0:
        return ("interval", s.vlong())
    if rid == 1:
        return ("time_unit", s.byte(), s.string())
    if rid == 2:
        return ("time_interval", s.vlong(), s.string())
    if rid == 8:
        inner = _rounding(s)
        return ("offset", inner, s.i64())
    raise ValueError("rounding id %d" % rid)


def _terms_order(s):  # InternalOrder.Streams.readOrder
    oid = s.sbyte()
    if oid in (1, 2, 3, 4):
        return {1: "_count desc", 2: "_count asc", 3: "_term desc", 4: "_term asc"}[oid]
    if oid == 0:
        asc = s.boolean()
        return ("agg", s.string(), asc)
    if oid == -1:
        return ("compound", [_terms_order(s) for _ in range(s.vint())])
    raise ValueError("terms order id %d" % oid)


def _aggs(s):
    out = []
    for _ in range(s.vint()):
        typ = s.bytes_ref().decode()
        out.append(_agg(s, typ))
    return out


def _agg(s, typ):  # InternalAggregation.readFrom, then doReadFrom
    a = {"stream_type": typ, "name": s.string()}
    meta = s.sbyte()
    if meta != -1:
        raise ValueError("metadata is not null")
    if s.vint() != 0:
        raise ValueError("pipeline aggregators present")
    if typ == "sterms":  # StringTerms.doReadFrom (:185-200)
        a["doc_count_error"] = s.i64()
        a["order"] = _terms_order(s)
        a["required_size"] = s.vint()
        a["shard_size"] = s.vint()
        a["show_term_doc_count_error"] = s.boolean()
        a["min_doc_count"] = s.vlong()
        a["other_doc_count"] = s.vlong()
        bks = []
        for _ in range(s.vint()):
            bk = {"key": s.bytes_ref(), "doc_count": s.vlong()}
            if a["show_term_doc_count_error"]:
                bk["doc_count_error"] = s.i64()
            bk["aggs"] = _aggs(s)
            bks.append(bk)
        a["buckets"] = bks
    elif typ in ("histo", "dhisto"):  # InternalHistogram.doReadFrom (:479-495)
        a["factory"] = s.string()
        a["order"] = s.byte()
        a["min_doc_count"] = s.vlong()
        if a["min_doc_count"] == 0:
            a["rounding"] = _rounding(s)
            a["empty_aggs"] = _aggs(s)
            if s.boolean():
                lo = s.i64() if s.boolean() else None
                hi = s.i64() if s.boolean() else None
                a["bounds"] = (lo, hi)
        a["formatter"] = _formatter(s)
        a["keyed"] = s.boolean()
        a["buckets"] = [{"key": s.i64(), "doc_count": s.vlong(), "aggs": _aggs(s)} for _ in range(s.vint())]
    elif typ in ("stats", "estats"):  # InternalStats.doReadFrom (:169-176), InternalExtendedStats.readOtherStatsFrom
        a["formatter"] = _formatter(s)
        a["count"] = s.vlong()
        a["min"], a["max"], a["sum"] = s.f64(), s.f64(), s.f64()
        if typ == "estats":
            a["sum_of_squares"], a["sigma"] = s.f64(), s.f64()
    elif typ == "avg":  # InternalAvg.doReadFrom (:95-99)
        a["formatter"] = _formatter(s)
        a["sum"] = s.f64()
        a["count"] = s.vlong()
    elif typ == "cardinality":  # InternalCardinality.doReadFrom (:82-90), HyperLogLogPlusPlus.readFrom (:537-555)
        a["formatter"] = _formatter(s)
        a["present"] = s.boolean()
        if a["present"]:
            a["precision"] = s.vint()
            if s.boolean():
                a["mode"] = "hll"
                a["registers"] = s.raw(1 << a["precision"])
            else:
                a["mode"] = "lc"
                a["lc"] = [s.i32() & 0xFFFFFFFF for _ in range(s.vlong())]
    elif typ == "filter":  # InternalSingleBucketAggregation.doReadFrom (:118-122)
        a["doc_count"] = s.vlong()
        a["aggs"] = _aggs(s)
    else:
        raise ValueError("unknown stream type %r" % typ)
    return a


def decode(data):
    s = StreamInput(data)
    out = _aggs(s)
    if s.i != len(s.b):
        raise ValueError("%d trailing bytes" % (len(s.b) - s.i))
    return out


def normalized(aggs):
    def fix(x):
        if isinstance(x, dict):
            y = {k: fix(v) for k, v in x.items()}
            if y.get("mode") == "lc":
                y["lc"] = sorted(y["lc"])
            return y
        if isinstance(x, list):
            return [fix(v) for v in x]
        return x
    return fix(aggs)


def has_lc(aggs):
    return any(a.get("mode") == "lc" for a in _walk(aggs))


def _walk(aggs):
    for a in aggs:
        yield a
        for bk in a.get("buckets", []):
            yield from _walk(bk["aggs"])
        yield from _walk(a.get("aggs", []))
        yield from _walk(a.get("empty_aggs", []))


def first_diff(a, b, path="aggs"):
    """Path and values of the first difference between two decoded trees (diagnostics)."""
    if isinstance(a, dict) and isinstance(b, dict):
        for k in sorted(set(a) | set(b), key=str):
            if k not in a or k not in b:
                return f"{path}.{k}", a.get(k), b.get(k)
            d = first_diff(a[k], b[k], f"{path}.{k}")
            if d:
                return d
        return None
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        if len(a) != len(b):
            return f"{path}[len]", len(a), len(b)
        for i, (x, y) in enumerate(zip(a, b)):
            d = first_diff(x, y, f"{path}[{i}]")
            if d:
                return d
        return None
    return None if a == b else (path, a, b)
