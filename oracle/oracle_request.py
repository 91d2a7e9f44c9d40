"""The oracle's own request lowering: raw builder requests -> esgpu_agg_spec / esgpu_filter structs.  TEST
INFRASTRUCTURE ONLY (see oracle.py).

Independent of the product: nothing here calls libesgpu.so or elasticsearch_amd.aggs; the only thing taken from the
product package is the ctypes struct LAYOUT of include/esgpu.h (elasticsearch_amd._native), which is the boundary both
sides speak.  Every parser default and rounding step is restated from the reference here:

  terms thresholds ........ TermsParser.parse (A/bucket/terms/TermsParser.java:46-77): compound order, the
                            suggestShardSideQueueSize heuristic when shard_size was not given and the order is not a
                            term order (A/bucket/BucketUtils.java:36-47), then BucketCountThresholds.ensureValidity
                            (A/bucket/terms/TermsAggregator.java:63-85); defaults size 10, shard_size -1,
                            min_doc_count 1, shard_min_doc_count 0 (TermsParametersParser.java:35)
  histogram ............... HistogramParser.parse: interval >= 1, Rounding.Interval + OffsetRounding
  date_histogram .......... DateHistogramParser.parse (:85-193): DATE_FIELD_UNITS (:50-69), else
                            TimeValue.parseTimeValue; offset "+1h"/"-30m" (parseOffset); the time zone goes into
                            TimeZoneRounding as a zone -- here ALWAYS as an offset table, fixed offsets included (the
                            product instead folds a fixed offset into OffsetRounding; both must round alike)
  time zones .............. joda DateTimeZone.forID: fixed "+hh:mm" / "-hh" offsets, or a region id whose offset
                            history is read from the IANA TZif file (RFC 8536) plus its POSIX TZ footer rule, expanded
                            to 2100 (the product samples Python's zoneinfo instead)
  extended_bounds ......... ExtendedBounds.round(rounding) = rounding.round(bound) with the aggregation's full
                            Rounding, evaluated by the oracle's own Rounding (cpu_ref.cpp, oracle_rounding_tz)
  cardinality ............. precision_threshold passed through; precision derived inside cpu_ref.cpp
"""
import ctypes
import datetime as _dt
import functools
import importlib.resources
import re
import struct

from elasticsearch_amd import _native as N  # struct layouts only

INT_MAX = 2**31 - 1
NEG_INF_MS = -(1 << 63)

# ---- DateHistogramParser.DATE_FIELD_UNITS (A/bucket/histogram/DateHistogramParser.java:50-69) ----
_UNITS = {"year": N.UNIT_YEAR, "1y": N.UNIT_YEAR, "quarter": N.UNIT_QUARTER, "1q": N.UNIT_QUARTER,
          "month": N.UNIT_MONTH, "1M": N.UNIT_MONTH, "week": N.UNIT_WEEK, "1w": N.UNIT_WEEK,
          "day": N.UNIT_DAY, "1d": N.UNIT_DAY, "hour": N.UNIT_HOUR, "1h": N.UNIT_HOUR,
          "minute": N.UNIT_MINUTE, "1m": N.UNIT_MINUTE, "second": N.UNIT_SECOND, "1s": N.UNIT_SECOND}

_TIME_MS = {"ms": 1, "s": 1000, "m": 60_000, "h": 3_600_000, "d": 86_400_000, "w": 604_800_000}


def time_value_ms(text):
    """TimeValue.parseTimeValue (common/unit/TimeValue.java:232-272), suffix tests in its order; note "s" casts
    before it multiplies ((long) 1.5 * 1000 = 1000) and a bare number is lenient milliseconds."""
    t = str(text).lower().strip()
    try:
        if t.endswith("ms"):
            return int(float(t[:-2]))
        if t.endswith("s"):
            return int(float(t[:-1])) * 1000
        for suffix in ("m", "h", "d", "w"):
            if t.endswith(suffix):
                return int(float(t[:-1]) * _TIME_MS[suffix])
        return int(str(text).strip())
    except ValueError:
        raise ValueError("Failed to parse [%s]" % text) from None


def parse_offset(text):
    """DateHistogramParser.parseOffset: optional sign, then a TimeValue."""
    if isinstance(text, int):
        return text
    t = str(text)
    if t.startswith("-"):
        return -time_value_ms(t[1:])
    return time_value_ms(t[1:] if t.startswith("+") else t)


# ---- terms (TermsParser / BucketUtils / BucketCountThresholds) ----
def suggest_shard_side_queue_size(final_size, number_of_shards):
    if number_of_shards == 1:
        return final_size
    sample = final_size * min(10, number_of_shards)
    return int(min(INT_MAX, max(10, sample)))


def terms_thresholds(size, shard_size, min_doc_count, shard_min_doc_count, order, number_of_shards):
    """-> (size, shard_size, min_doc_count, shard_min_doc_count) as the TermsAggregatorFactory receives them."""
    size = 10 if size is None or size < 0 else size                    # TermsParametersParser defaults (1, 0, 10, -1)
    min_doc_count = 1 if min_doc_count is None or min_doc_count < 0 else min_doc_count
    shard_min_doc_count = 0 if shard_min_doc_count is None or shard_min_doc_count < 0 else shard_min_doc_count
    shard_size = -1 if shard_size is None else shard_size
    term_order = order in (N.ORDER_TERM_ASC, N.ORDER_TERM_DESC)
    if not term_order and shard_size == -1:
        shard_size = suggest_shard_side_queue_size(size, number_of_shards)
    # ensureValidity
    if shard_size == 0:
        shard_size = INT_MAX
    if size == 0:
        size = INT_MAX
    if shard_size < size:
        shard_size = size
    if shard_min_doc_count > min_doc_count:
        shard_min_doc_count = min_doc_count
    if size < 0 or min_doc_count < 0:
        raise ValueError("parameters [requiredSize] and [minDocCount] must be >=0 in terms aggregation.")
    return size, shard_size, min_doc_count, shard_min_doc_count


# ---- time zones (joda DateTimeZone.forID) ----
def _posix_offset(s):
    """POSIX TZ offset "[+-]hh[:mm[:ss]]" -> seconds EAST of UTC (POSIX counts west)."""
    m = re.fullmatch(r"([+-]?)(\d{1,3})(?::(\d{1,2}))?(?::(\d{1,2}))?", s)
    sign = -1 if m.group(1) == "-" else 1
    secs = int(m.group(2)) * 3600 + int(m.group(3) or 0) * 60 + int(m.group(4) or 0)
    return -sign * secs


def _rule_day(year, rule):
    """POSIX date rule -> day ordinal (datetime.date.toordinal) in `year`: Mm.w.d, Jn (1..365, no Feb 29) or n."""
    if rule.startswith("M"):
        m, w, d = (int(x) for x in rule[1:].split("."))
        first = _dt.date(year, m, 1)
        delta = (d - (first.isoweekday() % 7)) % 7       # first weekday d (0 = Sunday) of the month
        day = first.toordinal() + delta + 7 * (w - 1)
        nxt = _dt.date(year + (m == 12), m % 12 + 1, 1).toordinal()
        while day >= nxt:                                 # week 5 = the last such weekday
            day -= 7
        return day
    if rule.startswith("J"):
        n = int(rule[1:])
        day = _dt.date(year, 1, 1).toordinal() + n - 1
        if n >= 60 and year % 4 == 0 and (year % 100 != 0 or year % 400 == 0):
            day += 1
        return day
    return _dt.date(year, 1, 1).toordinal() + int(rule)


def _posix_transitions(footer, first_year, last_year):
    """Expand a POSIX TZ string into (utc_seconds, utc_offset_seconds) transitions, plus its standard offset."""
    name = r"(?:<[^>]*>|[A-Za-z]{3,})"
    off = r"[+-]?\d{1,3}(?::\d{1,2}){0,2}"
    m = re.fullmatch(rf"({name})({off})(?:({name})({off})?(?:,([^,/]+)(?:/({off}))?,([^,/]+)(?:/({off}))?)?)?", footer)
    if not m:
        raise ValueError("unsupported POSIX TZ string %r" % footer)
    std = _posix_offset(m.group(2))
    if not m.group(3):
        return [], std
    dst = _posix_offset(m.group(4)) if m.group(4) else std + 3600
    start_rule, start_time = m.group(5) or "M3.2.0", m.group(6) or "2"
    end_rule, end_time = m.group(7) or "M11.1.0", m.group(8) or "2"
    epoch = _dt.date(1970, 1, 1).toordinal()
    out = []
    for y in range(first_year, last_year + 1):
        # the start time is standard local time, the end time daylight local time (POSIX)
        s = (_rule_day(y, start_rule) - epoch) * 86400 - _posix_offset(start_time) - std
        e = (_rule_day(y, end_rule) - epoch) * 86400 - _posix_offset(end_time) - dst
        out += [(s, dst), (e, std)]
    out.sort()
    return out, std


@functools.lru_cache(maxsize=64)
def zone_table(tz):
    """-> ((starts_ms...), (offsets_ms...)) for the C side (starts[0] = -infinity), or None for UTC."""
    if tz is None or tz in ("UTC", "utc", "Z", "Etc/UTC"):
        return None
    m = re.fullmatch(r"([+-])?(\d{1,2})(?::?(\d{2}))?", tz)
    if m:  # DateTimeZone.forID("+01:00") / forOffsetHours: a fixed zone
        sign = -1 if m.group(1) == "-" else 1
        return (NEG_INF_MS,), (sign * (int(m.group(2)) * 3_600_000 + int(m.group(3) or 0) * 60_000),)
    try:
        data = importlib.resources.files("tzdata.zoneinfo").joinpath(*tz.split("/")).read_bytes()
    except (FileNotFoundError, ModuleNotFoundError, IsADirectoryError) as e:
        raise ValueError("The datetime zone id '%s' is not recognised" % tz) from e
    if data[:4] != b"TZif":
        raise ValueError("not a TZif file: %s" % tz)
    # RFC 8536: skip the v1 block, read the 64-bit v2+ block and the footer
    isut, isstd, leap, timecnt, typecnt, charcnt = struct.unpack(">6l", data[20:44])
    p = 44 + timecnt * 4 + timecnt + typecnt * 6 + charcnt + leap * 8 + isstd + isut
    isut, isstd, leap, timecnt, typecnt, charcnt = struct.unpack(">6l", data[p + 20:p + 44])
    q = p + 44
    times = struct.unpack(">%dq" % timecnt, data[q:q + 8 * timecnt])
    q += 8 * timecnt
    idx = data[q:q + timecnt]
    q += timecnt
    types = [struct.unpack(">lBB", data[q + 6 * i:q + 6 * i + 6]) for i in range(typecnt)]
    q += 6 * typecnt + charcnt + leap * 12 + isstd + isut
    footer = data[q:].strip(b"\n").decode()
    trans = [(t, types[i][0]) for t, i in zip(times, idx)]
    initial = types[0][0]  # local time type 0 applies before the first transition
    if footer:
        last = trans[-1][0] if trans else -(1 << 62)
        first_year = _dt.datetime.fromtimestamp(max(last, -2**31), _dt.timezone.utc).year if trans else 1900
        extra, std = _posix_transitions(footer, first_year, 2100)
        trans += [x for x in extra if x[0] > last]
        if not trans:
            initial = std
    starts, offs = [NEG_INF_MS], [initial * 1000]
    for t, o in trans:
        if o * 1000 != offs[-1]:
            starts.append(t * 1000)
            offs.append(o * 1000)
    return tuple(starts), tuple(offs)


# ---- value formatter and time zone id (wire stream) ----
# The test index mapping (SURVEY §8(d) synthetic log documents): "@timestamp" is a date field with the mapper's default
# format, DateFieldMapper.Defaults.DATE_TIME_FORMATTER (C/index/mapper/core/DateFieldMapper.java:75); every other field
# is a NumberFieldType (long / double / murmur3) or a string.
_DATE_FIELD_FORMATS = {"@timestamp": "strict_date_optional_time||epoch_millis"}


def _resolve_format(field, fmt):
    """ValuesSourceParser.resolveFormat(format, timezone, fieldType) (ValuesSourceParser.java:244-257)"""
    if field in _DATE_FIELD_FORMATS:  # ValueFormat.DateTime.format(format, tz) / .mapper(fieldType, tz)
        return N.FORMAT_DATE_TIME, fmt if fmt is not None else _DATE_FIELD_FORMATS[field]
    if fmt is not None:               # NumberFieldType with a pattern: ValueFormat.Number.format(format)
        return N.FORMAT_NUMBER, fmt
    return N.FORMAT_RAW, None         # ValueFormat.RAW


def zone_id(tz):
    """joda DateTimeZone.forID(tz).getID(): UTC for "UTC" and for a zero offset (forOffsetMillis(0) == UTC), the offset
    printed as [+-]hh:mm for a fixed zone (DateTimeZone.printOffset), a region id as named."""
    if tz is None or tz in ("UTC", "utc", "Z", "Etc/UTC"):
        return "UTC"
    m = re.fullmatch(r"([+-])?(\d{1,2})(?::?(\d{2}))?", tz)
    if not m:
        return tz
    ms = int(m.group(2)) * 3_600_000 + int(m.group(3) or 0) * 60_000
    if ms == 0:
        return "UTC"
    return "%s%02d:%02d" % ("-" if m.group(1) == "-" else "+", ms // 3_600_000, ms // 60_000 % 60)


# ---- lowering ----
def _zone_arrays(zone, keep):
    starts = (ctypes.c_int64 * len(zone[0]))(*zone[0])
    offs = (ctypes.c_int64 * len(zone[1]))(*zone[1])
    keep += [starts, offs]
    return ctypes.cast(starts, ctypes.POINTER(ctypes.c_int64)), ctypes.cast(offs, ctypes.POINTER(ctypes.c_int64))


def _round(lib, sp, kind, v):
    """ExtendedBounds.round through the oracle's Rounding (cpu_ref.cpp oracle_rounding_tz, op 0 = round)."""
    return lib.oracle_rounding_tz(kind, sp.date_unit, sp.interval, sp.offset, sp.tz_starts, sp.tz_offsets_ms,
                                  sp.tz_count, 0, int(v))


def lower(lib, aggs, number_of_shards=1):
    """Builders -> (ctypes AggSpec array, count, keep-alive list); parents precede children (depth first)."""
    specs, keep = [], []

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
            fmt, pattern = _resolve_format(b._field, getattr(b, "_format", None))
            sp.value_format = fmt
            sp.format = enc(pattern)
            sp.time_zone = enc(zone_id(b._tz) if b.type == N.AGG_DATE_HISTOGRAM else "UTC")
        if b.type == N.AGG_TERMS:
            order = b._order
            if hasattr(order, "path"):  # Terms.Order.aggregation(path, asc)
                sp.order = N.ORDER_AGG_ASC if order.asc else N.ORDER_AGG_DESC
                sp.order_path = enc(order.path)
            else:
                sp.order = order
            sp.size, sp.shard_size, sp.min_doc_count, sp.shard_min_doc_count = terms_thresholds(
                b._size, b._shard_size, b._min, b._shard_min, sp.order, number_of_shards)
            sp.show_term_doc_count_error = int(b._show_err)
        elif b.type == N.AGG_HISTOGRAM:
            if b._interval is None or int(b._interval) < 1:
                raise ValueError("Missing required field [interval] for histogram aggregation [%s]" % b.name)
            sp.date_unit, sp.interval, sp.offset = N.UNIT_NONE, int(b._interval), int(b._offset)
        elif b.type == N.AGG_DATE_HISTOGRAM:
            if b._interval is None:
                raise ValueError("Missing required field [interval] for histogram aggregation [%s]" % b.name)
            unit = _UNITS.get(str(b._interval))
            sp.date_unit = unit if unit is not None else N.UNIT_NONE
            sp.interval = 0 if unit is not None else time_value_ms(b._interval)
            sp.offset = parse_offset(b._offset)
            zone = zone_table(b._tz)
            if zone is not None:
                sp.tz_starts, sp.tz_offsets_ms = _zone_arrays(zone, keep)
                sp.tz_count = len(zone[0])
        if b.type in (N.AGG_HISTOGRAM, N.AGG_DATE_HISTOGRAM):
            kind = 0 if b.type == N.AGG_HISTOGRAM else (1 if sp.date_unit != N.UNIT_NONE else 2)
            sp.min_doc_count = b._min
            sp.order = b._order
            sp.keyed = int(b._keyed)
            lo, hi = b._bounds
            if lo is not None:
                sp.has_extended_bounds_min = 1
                sp.extended_bounds_min = _round(lib, sp, kind, lo)
            if hi is not None:
                sp.has_extended_bounds_max = 1
                sp.extended_bounds_max = _round(lib, sp, kind, hi)
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
    return (N.AggSpec * max(len(specs), 1))(*specs), len(specs), keep


def lower_filters(queries, ord_lookup=None, aggs=None):
    """Query clauses (owner 0), then every filter aggregation's clauses (owner = its spec index + 1)."""
    tagged = [(q, 0) for q in queries or []]
    order = []

    def walk(b):
        order.append(b)
        for s in b.subs:
            walk(s)

    for a in aggs or []:
        walk(a)
    for i, b in enumerate(order):
        if b.type == N.AGG_FILTER:
            q = b._query
            if q is None:
                raise ValueError("[filter] aggregation [%s] requires a filter" % b.name)
            tagged += [(c, i + 1) for c in (q if isinstance(q, (list, tuple)) else [q])]
    out, keep = [], []
    for q, owner in tagged:
        f = N.Filter()
        f.owner = owner
        fb = q.field.encode("utf-8")
        keep.append(fb)
        f.field = fb
        if hasattr(q, "value"):  # TermQuery
            f.type = N.FILTER_TERM
            v = q.value
            if isinstance(v, str):
                if ord_lookup is None:
                    raise ValueError("keyword term filters need an ordinal lookup")
                v = ord_lookup(q.field, v)
            f.term = int(v)
        else:  # RangeQuery
            f.type = N.FILTER_RANGE
            for side, val, incl in (("lo", q.lo, q.include_lower), ("hi", q.hi, q.include_upper)):
                if val is None:
                    continue
                setattr(f, "has_lower" if side == "lo" else "has_upper", 1)
                setattr(f, "include_lower" if side == "lo" else "include_upper", int(incl))
                if isinstance(val, (str, bytes)):
                    tb = val.encode("utf-8") if isinstance(val, str) else bytes(val)
                    keep.append(tb)
                    setattr(f, side + "_term", tb)
                    setattr(f, side + "_term_len", len(tb))
                else:
                    setattr(f, side + "_i", int(val))
                    setattr(f, side + "_d", float(val))
        out.append(f)
    return (N.Filter * max(len(out), 1))(*out), len(out), keep
