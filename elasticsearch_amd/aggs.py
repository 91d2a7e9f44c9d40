"""Request builders mirroring the reference's Java API for this path.

    AggregationBuilders.terms("keys").field("key").size(3).shardSize(3).order(Terms.Order.count(False))
    AggregationBuilders.dateHistogram("histo").field("date").interval("1h").minDocCount(0)
    QueryBuilders.termQuery("status", 200), QueryBuilders.rangeQuery("bytes").gte(1024).lte(65536)

(core/src/main/java/org/elasticsearch/search/aggregations/AggregationBuilders.java and
core/src/main/java/org/elasticsearch/index/query/QueryBuilders.java).  `flatten()` applies the parser defaults
the reference applies before an AggregatorFactory exists (TermsParser.java:46-77 + BucketCountThresholds,
DateHistogramParser.java:85-193, CardinalityParser.java:48-71, ExtendedStatsParser.java:57) and produces the
flattened esgpu_agg_spec array of include/esgpu.h.
"""
import ctypes
import functools
import re

from . import _native as N

# ---- DateHistogramParser.DATE_FIELD_UNITS (DateHistogramParser.java:50-69) ----
DATE_FIELD_UNITS = {
    "year": N.UNIT_YEAR, "1y": N.UNIT_YEAR, "quarter": N.UNIT_QUARTER, "1q": N.UNIT_QUARTER,
    "month": N.UNIT_MONTH, "1M": N.UNIT_MONTH, "week": N.UNIT_WEEK, "1w": N.UNIT_WEEK,
    "day": N.UNIT_DAY, "1d": N.UNIT_DAY, "hour": N.UNIT_HOUR, "1h": N.UNIT_HOUR,
    "minute": N.UNIT_MINUTE, "1m": N.UNIT_MINUTE, "second": N.UNIT_SECOND, "1s": N.UNIT_SECOND,
}

_TIME_UNITS_MS = {"ms": 1, "s": 1000, "m": 60000, "h": 3600000, "d": 86400000, "w": 7 * 86400000}


def parse_time_value(text):
    """TimeValue.parseTimeValue (common/unit/TimeValue.java:232-272): the lower-cased text's suffix picks the unit
    (ms, s, m, h, d, w in that order of tests), a bare number is milliseconds.  As in Java, seconds truncate the
    number before scaling ((long) 1.5 * 1000 = 1000); the other units scale, then truncate."""
    t = str(text).lower().strip()
    m = re.fullmatch(r"(-?\d+(?:\.\d*)?|-?\.\d+)(ms|s|m|h|d|w)?", t)
    if not m:
        raise ValueError(f"Failed to parse [{text}]")
    num, unit = m.group(1), m.group(2)
    if unit is None:
        if "." in num:
            raise ValueError(f"Failed to parse [{text}]")
        return int(num)
    if unit == "s":
        return int(float(num)) * 1000
    return int(float(num) * _TIME_UNITS_MS[unit])


def parse_offset(text):
    """DateHistogramParser.parseOffset: "-" negates, "+" is dropped, the rest is a TimeValue."""
    t = str(text)
    if t.startswith("-"):
        return -parse_time_value(t[1:])
    return parse_time_value(t[1:] if t.startswith("+") else t)


def parse_time_zone(tz):
    """DateTimeZone.forID: fixed offsets ("UTC", "+01:00", "-08:00", "-2") -> offset in ms; a region id
    ("Europe/Berlin", "America/Chicago", "CET") -> its offset history (tz_history)."""
    if tz is None or tz in ("UTC", "Z", "utc"):
        return 0
    m = re.fullmatch(r"([+-])?(\d{1,2})(?::?(\d{2}))?", tz)
    if not m:
        return tz_history(tz)
    sign = -1 if m.group(1) == "-" else 1
    return sign * (int(m.group(2)) * 3600000 + int(m.group(3) or 0) * 60000)


@functools.lru_cache(maxsize=64)
def tz_history(name, first_year=1900, last_year=2100):
    """Offset history of an IANA zone as the C-ABI takes it (esgpu_agg_spec.tz_starts / tz_offsets_ms): offset
    offs[i] applies from UTC instant starts[i] on (starts[0] = -infinity).  What a JNI caller reads from joda's
    DateTimeZone (getOffset / nextTransition), read here from the IANA database behind Python's zoneinfo: the offset
    is sampled every 6 hours over [first_year, last_year) and each change is bisected to the second."""
    import datetime as _dt
    import zoneinfo
    try:
        z = zoneinfo.ZoneInfo(name)
    except (zoneinfo.ZoneInfoNotFoundError, ValueError) as e:
        raise ValueError(f"The datetime zone id '{name}' is not recognised") from e
    epoch = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)

    def off(sec):
        return int((epoch + _dt.timedelta(seconds=sec)).astimezone(z).utcoffset().total_seconds() * 1000)

    lo = int((_dt.datetime(first_year, 1, 1, tzinfo=_dt.timezone.utc) - epoch).total_seconds())
    hi = int((_dt.datetime(last_year, 1, 1, tzinfo=_dt.timezone.utc) - epoch).total_seconds())
    step = 6 * 3600
    starts, offs = [-(1 << 63)], [off(lo)]
    prev = offs[0]
    t = lo
    while t < hi:
        nxt = t + step
        o = off(nxt)
        if o != prev:
            a, b = t, nxt  # off(a) == prev != off(b): the transition instant is in (a, b]
            while b - a > 1:
                mid = (a + b) // 2
                if off(mid) == prev:
                    a = mid
                else:
                    b = mid
            starts.append(b * 1000)
            offs.append(off(b))
            prev = offs[-1]
            if o != prev:  # two changes inside one step: rescan from the transition
                t = b
                continue
        t = nxt
    return tuple(starts), tuple(offs)


class AggOrder:
    def __init__(self, path, asc):
        self.path, self.asc = path, bool(asc)


def order_code(o):
    """-> (ESGPU_ORDER_*, order path or None)"""
    if isinstance(o, AggOrder):
        return (N.ORDER_AGG_ASC if o.asc else N.ORDER_AGG_DESC), o.path
    return o, None


class Order:
    """Terms.Order (InternalOrder.java) and Histogram.Order."""

    @staticmethod
    def count(asc):
        return N.ORDER_COUNT_ASC if asc else N.ORDER_COUNT_DESC

    @staticmethod
    def term(asc):
        return N.ORDER_TERM_ASC if asc else N.ORDER_TERM_DESC

    @staticmethod
    def aggregation(path, asc):
        """Terms.Order.aggregation: order by a metric sub-aggregation, "avg_rt" or "rt.max" (InternalOrder.Aggregation)."""
        return AggOrder(path, asc)

    KEY_ASC = N.ORDER_KEY_ASC
    KEY_DESC = N.ORDER_KEY_DESC
    COUNT_ASC = N.ORDER_HCOUNT_ASC
    COUNT_DESC = N.ORDER_HCOUNT_DESC


class _Builder:
    type = 0

    def __init__(self, name):
        self.name = name
        self._field = None
        self._format = None
        self.subs = []

    def field(self, f):
        self._field = f
        return self

    def format(self, pattern):
        """the request's "format" (ValuesSourceParser formattable aggregations): a date pattern on a date field, a
        DecimalFormat pattern on a numeric one"""
        self._format = pattern
        return self

    def subAggregation(self, sub):  # noqa: N802 - mirrors the Java API
        self.subs.append(sub)
        return self

    sub_aggregation = subAggregation


class TermsBuilder(_Builder):
    type = N.AGG_TERMS

    def __init__(self, name):
        super().__init__(name)
        self._size, self._shard_size, self._min, self._shard_min = 10, -1, -1, -1
        self._order = N.ORDER_COUNT_DESC
        self._show_err = False

    def size(self, n):
        self._size = n
        return self

    def shardSize(self, n):  # noqa: N802
        self._shard_size = n
        return self

    def minDocCount(self, n):  # noqa: N802
        self._min = n
        return self

    def shardMinDocCount(self, n):  # noqa: N802
        self._shard_min = n
        return self

    def order(self, o):
        self._order = o
        return self

    def showTermDocCountError(self, b):  # noqa: N802
        self._show_err = bool(b)
        return self

    shard_size = shardSize
    min_doc_count = minDocCount


class HistogramBuilder(_Builder):
    type = N.AGG_HISTOGRAM

    def __init__(self, name):
        super().__init__(name)
        self._interval = None
        self._offset = 0
        self._min = 0  # HistogramParser / DateHistogramParser: min_doc_count default 0
        self._order = N.ORDER_KEY_ASC
        self._keyed = False
        self._bounds = (None, None)

    def interval(self, i):
        self._interval = i
        return self

    def offset(self, o):
        self._offset = o
        return self

    def minDocCount(self, n):  # noqa: N802
        self._min = n
        return self

    def order(self, o):
        self._order = o
        return self

    def keyed(self, k):
        self._keyed = bool(k)
        return self

    def extendedBounds(self, lo, hi):  # noqa: N802
        self._bounds = (lo, hi)
        return self

    min_doc_count = minDocCount


class DateHistogramBuilder(HistogramBuilder):
    type = N.AGG_DATE_HISTOGRAM

    def __init__(self, name):
        super().__init__(name)
        self._tz = None

    def timeZone(self, tz):  # noqa: N802
        self._tz = tz
        return self

    time_zone = timeZone


class _MetricBuilder(_Builder):
    def subAggregation(self, sub):  # noqa: N802
        raise ValueError("Aggregator [%s] of type [%d] cannot accept sub-aggregations" % (self.name, self.type))


class StatsBuilder(_MetricBuilder):
    type = N.AGG_STATS


class ExtendedStatsBuilder(_MetricBuilder):
    type = N.AGG_EXTENDED_STATS

    def __init__(self, name):
        super().__init__(name)
        self._sigma = 2.0

    def sigma(self, s):
        if s < 0:
            raise ValueError("[sigma] must not be negative")
        self._sigma = float(s)
        return self


class AvgBuilder(_MetricBuilder):
    type = N.AGG_AVG


class CardinalityBuilder(_MetricBuilder):
    type = N.AGG_CARDINALITY

    def __init__(self, name):
        super().__init__(name)
        self._threshold = -1

    def precisionThreshold(self, t):  # noqa: N802
        self._threshold = int(t)
        return self

    precision_threshold = precisionThreshold


class FilterBuilder(_Builder):
    """filter aggregation (FilterAggregator / InternalFilter): one bucket of the docs matching `query` -- a TermQuery,
    a RangeQuery or a list of them (bool.filter conjunction) -- with sub-aggregations.  On the GPU path at the top level
    (any sub-aggregations) or directly under a top-level bucket aggregation (metric sub-aggregations)."""
    type = N.AGG_FILTER

    def __init__(self, name, query=None):
        super().__init__(name)
        self._query = query

    def filter(self, query):
        self._query = query
        return self

    def clauses(self):
        q = self._query
        if q is None:
            raise ValueError("[filter] aggregation [%s] requires a filter" % self.name)
        return list(q) if isinstance(q, (list, tuple)) else [q]


class AggregationBuilders:
    terms = TermsBuilder
    filter = FilterBuilder
    histogram = HistogramBuilder
    dateHistogram = DateHistogramBuilder
    date_histogram = DateHistogramBuilder
    stats = StatsBuilder
    extendedStats = ExtendedStatsBuilder
    extended_stats = ExtendedStatsBuilder
    avg = AvgBuilder
    cardinality = CardinalityBuilder


# ---- queries (bool.filter conjunction of term / range) ----
class TermQuery:
    def __init__(self, field, value):
        self.field, self.value = field, value


class RangeQuery:
    def __init__(self, field):
        self.field = field
        self.lo = self.hi = None
        self.include_lower = self.include_upper = True

    def gte(self, v):
        self.lo, self.include_lower = v, True
        return self

    def gt(self, v):
        self.lo, self.include_lower = v, False
        return self

    def lte(self, v):
        self.hi, self.include_upper = v, True
        return self

    def lt(self, v):
        self.hi, self.include_upper = v, False
        return self

    def from_(self, v, include=True):
        self.lo, self.include_lower = v, include
        return self

    def to(self, v, include=True):
        self.hi, self.include_upper = v, include
        return self


class QueryBuilders:
    @staticmethod
    def termQuery(field, value):  # noqa: N802
        return TermQuery(field, value)

    @staticmethod
    def rangeQuery(field):  # noqa: N802
        return RangeQuery(field)

    term_query = termQuery
    range_query = rangeQuery


# ---- flattening -------------------------------------------------------------------------------------------------
def _rounding_params(b):
    """-> (date_unit, interval, offset, zone) with a fixed time-zone offset folded into OffsetRounding; zone is None
    or the (starts, offsets) history of a region zone (DateHistogramParser.java:178-187)."""
    if b.type == N.AGG_HISTOGRAM:
        if b._interval is None or int(b._interval) < 1:
            raise ValueError("[interval] must be 1 or greater for histogram aggregation [%s]" % b.name)
        return N.UNIT_NONE, int(b._interval), int(b._offset), None
    if b._interval is None:
        raise ValueError("Missing required field [interval] for histogram aggregation [%s]" % b.name)
    off = b._offset if isinstance(b._offset, int) else parse_offset(b._offset)
    tz = parse_time_zone(b._tz)
    zone = None
    if isinstance(tz, tuple):
        zone = tz
    elif tz != 0:  # a fixed zone as a one-entry table: Rounding.from_spec folds it into the offset, and the result
        zone = ((0,), (tz,))  # keeps it for printing the keys (key_as_string "...+01:00")
    unit = DATE_FIELD_UNITS.get(str(b._interval))
    if unit is not None:
        return unit, 0, off, zone
    return N.UNIT_NONE, parse_time_value(b._interval), off, zone


# The index mapping behind the synthetic log documents: "@timestamp" is a date field with the
# default date format; every other numeric field is a long / double / murmur3 (NumberFieldType).  A JNI caller reads
# both from the field's MappedFieldType instead.
DATE_FIELDS = {"@timestamp": "strict_date_optional_time||epoch_millis"}  # DateFieldMapper.Defaults.DATE_TIME_FORMATTER


def time_zone_id(tz):
    """DateTimeZone.forID(tz).getID(): "UTC" for a zero offset, "+hh:mm" / "-hh:mm" for a fixed one, a region id as
    given.  None = UTC (ValuesSourceParser's default)."""
    if tz is None:
        return "UTC"
    off = parse_time_zone(tz)
    if isinstance(off, tuple):
        return str(tz)
    if off == 0:
        return "UTC"
    a = abs(off)
    return "%s%02d:%02d" % ("-" if off < 0 else "+", a // 3600000, a // 60000 % 60)


def _value_format(b):
    """ValuesSourceParser.resolveFormat (ValuesSourceParser.java:244-257): (ESGPU_FORMAT_*, pattern)"""
    if b._field in DATE_FIELDS:
        return N.FORMAT_DATE_TIME, b._format or DATE_FIELDS[b._field]
    if b._format is not None:
        return N.FORMAT_NUMBER, b._format
    return N.FORMAT_RAW, None


def _round_bound(spec, v):
    """ExtendedBounds.round: the bound is rounded with the aggregation's own Rounding (esgpu_date_rounding)."""
    if v is None:
        return None
    out = ctypes.c_int64()
    N.check(N.lib().esgpu_date_rounding(ctypes.byref(spec), 0, int(v), ctypes.byref(out)))
    return out.value


def thresholds(size, shard_size, min_doc_count, shard_min_doc_count, order, number_of_shards):
    out = [ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()]
    N.check(N.lib().esgpu_terms_thresholds(size, shard_size, min_doc_count, shard_min_doc_count, order,
                                           number_of_shards, *[ctypes.byref(x) for x in out]))
    return tuple(x.value for x in out)


def flatten(aggs, number_of_shards=1):
    """Builders -> ctypes array of AggSpec (parents before children, parser defaults applied)."""
    specs = []
    keep = []  # keep the encoded names alive

    def enc(s):
        b = s.encode("utf-8") if s is not None else None
        keep.append(b)
        return b

    def visit(b, parent):
        sp = N.AggSpec()
        sp.type = b.type
        sp.parent = parent
        sp.name = enc(b.name)
        sp.field = enc(b._field)
        sp.sigma = 2.0
        sp.precision_threshold = -1
        if b.type != N.AGG_FILTER:
            fmt, pattern = _value_format(b)
            sp.value_format = fmt
            sp.format = enc(pattern)
            # the request time zone reaches the formatter through ValuesSourceParser.Input.timezone: date_histogram only
            sp.time_zone = enc(time_zone_id(b._tz) if b.type == N.AGG_DATE_HISTOGRAM else "UTC")
        if b.type == N.AGG_TERMS:
            code, path = order_code(b._order)
            size, ssize, mn, smn = thresholds(b._size, b._shard_size, b._min, b._shard_min, code, number_of_shards)
            sp.size, sp.shard_size, sp.min_doc_count, sp.shard_min_doc_count = size, ssize, mn, smn
            sp.order = code
            if path is not None:
                sp.order_path = enc(path)
            sp.show_term_doc_count_error = int(b._show_err)
        elif b.type in (N.AGG_HISTOGRAM, N.AGG_DATE_HISTOGRAM):
            unit, interval, off, zone = _rounding_params(b)
            sp.date_unit, sp.interval, sp.offset = unit, interval, off
            if zone is not None:
                starts = (ctypes.c_int64 * len(zone[0]))(*zone[0])
                offs = (ctypes.c_int64 * len(zone[1]))(*zone[1])
                keep.extend([starts, offs])
                sp.tz_starts = ctypes.cast(starts, ctypes.POINTER(ctypes.c_int64))
                sp.tz_offsets_ms = ctypes.cast(offs, ctypes.POINTER(ctypes.c_int64))
                sp.tz_count = len(zone[0])
            sp.min_doc_count = b._min
            sp.order = b._order
            sp.keyed = int(b._keyed)
            lo, hi = b._bounds
            if lo is not None:
                sp.has_extended_bounds_min = 1
                sp.extended_bounds_min = _round_bound(sp, lo)
            if hi is not None:
                sp.has_extended_bounds_max = 1
                sp.extended_bounds_max = _round_bound(sp, hi)
        elif b.type == N.AGG_EXTENDED_STATS:
            sp.sigma = b._sigma
        elif b.type == N.AGG_CARDINALITY:
            sp.precision_threshold = b._threshold
        idx = len(specs)
        specs.append(sp)
        for s in b.subs:
            visit(s, idx)

    for a in aggs:
        visit(a, -1)
    arr = (N.AggSpec * max(len(specs), 1))(*specs)
    return arr, len(specs), keep


def _preorder(aggs):
    """(builder, spec index) in flatten()'s order (parents before children, depth first)."""
    out = []

    def visit(b):
        out.append(b)
        for s in b.subs:
            visit(s)

    for a in aggs or []:
        visit(a)
    return [(b, i) for i, b in enumerate(out)]


def flatten_filters(queries, ord_lookup=None, aggs=None):
    """Queries -> ctypes array of Filter.  `ord_lookup(field, term) -> ordinal or -1` resolves keyword terms.  With
    `aggs`, the clauses of every filter aggregation follow, each tagged with its owner (spec index + 1)."""
    out, keep = [], []
    tagged = [(q, 0) for q in queries or []]
    for b, i in _preorder(aggs):
        if b.type == N.AGG_FILTER:
            tagged += [(q, i + 1) for q in b.clauses()]
    for q, owner in tagged:
        f = N.Filter()
        f.owner = owner
        b = q.field.encode("utf-8")
        keep.append(b)
        f.field = b
        if isinstance(q, TermQuery):
            f.type = N.FILTER_TERM
            v = q.value
            if isinstance(v, str):
                if ord_lookup is None:
                    raise ValueError("keyword term filters need an ordinal lookup")
                v = ord_lookup(q.field, v)
            f.term = int(v)
        else:
            f.type = N.FILTER_RANGE
            if q.lo is not None:
                f.has_lower, f.include_lower = 1, int(q.include_lower)
                if isinstance(q.lo, (str, bytes)):  # TermRangeQuery on a keyword field
                    b = q.lo.encode("utf-8") if isinstance(q.lo, str) else bytes(q.lo)
                    keep.append(b)
                    f.lo_term, f.lo_term_len = b, len(b)
                else:
                    f.lo_i, f.lo_d = int(q.lo), float(q.lo)
            if q.hi is not None:
                f.has_upper, f.include_upper = 1, int(q.include_upper)
                if isinstance(q.hi, (str, bytes)):
                    b = q.hi.encode("utf-8") if isinstance(q.hi, str) else bytes(q.hi)
                    keep.append(b)
                    f.hi_term, f.hi_term_len = b, len(b)
                else:
                    f.hi_i, f.hi_d = int(q.hi), float(q.hi)
        out.append(f)
    arr = (N.Filter * max(len(out), 1))(*out)
    return arr, len(out), keep
