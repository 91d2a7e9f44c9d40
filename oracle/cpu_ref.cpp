/*
 * cpu_ref.cpp — CPU ORACLE for the per-shard aggregation path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only as
 * the checker / the timed CPU baseline.  The product (libesgpu.so) never links or calls it.
 *
 * It is a line-by-line restatement, in C++, of the reference Java collect loops, buildAggregation and
 * InternalAggregation.doReduce for the aggregations named in SURVEY.md §8(a).  Iteration order is the
 * reference's (segment -> doc -> value); double arithmetic is strict IEEE (compiled -ffp-contract=off,
 * no fast-math) and Math.min/max follow Java semantics.  Each function cites the Java it restates
 * (paths relative to /root/reference/core/src/main/java/org/elasticsearch/, "A/" = search/aggregations/).
 *
 * Pinning: the restatement is checked against the reference's own known-answer vectors and fixtures in
 * tests/golden/kat.json (MurmurHash3Tests, HyperLogLogPlusPlusTests.precisionFromThreshold, RoundingTests,
 * TimeZoneRoundingTests, ExtendedStatsTests, ShardSizeTermsIT, DateHistogramTests, 10_histogram.yaml,
 * mapper_murmur3/10_basic.yaml).  hppc BitMixer.mix64 (third-party, hppc 0.7.1) has no reference KAT:
 * its use here is "parity unpinned" (DESIGN.md §Oracle).
 */
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../include/esgpu.h"

namespace oracle {

#include "hllpp_tables.inc"

// ------------------------------------------------------------------------------------------------------------
// Java semantics helpers
// ------------------------------------------------------------------------------------------------------------
static inline double java_min(double a, double b) {  // java.lang.Math.min(double,double)
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && std::signbit(b)) return b;  // -0.0 < +0.0
    return a <= b ? a : b;
}
static inline double java_max(double a, double b) {  // java.lang.Math.max(double,double)
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && std::signbit(a)) return b;
    return a >= b ? a : b;
}
static inline int64_t java_round(double a) {  // java.lang.Math.round(double): closest long, ties toward +inf
    if (a != a) return 0;
    if (a >= 9.2233720368547758e18) return INT64_MAX;
    if (a <= -9.2233720368547758e18) return INT64_MIN;
    double f = std::floor(a);
    return (int64_t)f + ((a - f) >= 0.5 ? 1 : 0);
}
static inline int64_t java_cast_long(double v) {  // (long) v
    if (v != v) return 0;
    if (v >= 9.2233720368547758e18) return INT64_MAX;
    if (v <= -9.2233720368547758e18) return INT64_MIN;
    return (int64_t)v;
}
static inline int nlz64(uint64_t x) { return x == 0 ? 64 : __builtin_clzll(x); }
static inline int nlz32(uint32_t x) { return x == 0 ? 32 : __builtin_clz(x); }
static inline int64_t floor_div(int64_t a, int64_t b) {  // Rounding.Interval.roundKey semantics (Rounding.java:92-98)
    if (a < 0) return (a - b + 1) / b;
    return a / b;
}

// hppc 0.7.1 com.carrotsearch.hppc.BitMixer.mix64 — third-party, not in /root/reference (parity unpinned).
// Call sites: A/metrics/cardinality/CardinalityAggregator.java:368,392; common/util/AbstractPagedHashMap.java:37
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 32)) * 0x4cd6944c5cc20b6dULL;
    z = (z ^ (z >> 29)) * 0xfc12c5b19d3259e9ULL;
    return z ^ (z >> 32);
}

// common/hash/MurmurHash3.java:38-157 (hash128, MurmurHash3_x64_128)
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}
static inline uint64_t read_le64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}
static void murmur3_128(const uint8_t* key, int length, int64_t seed, uint64_t* o1, uint64_t* o2) {
    const uint64_t C1 = 0x87c37b91114253d5ULL, C2 = 0x4cf5ad432745937fULL;
    uint64_t h1 = (uint64_t)seed, h2 = (uint64_t)seed;
    int offset = 0;
    if (length >= 16) {
        const int len16 = length & 0xFFFFFFF0;
        for (int i = 0; i < len16; i += 16) {
            uint64_t k1 = read_le64(key + i), k2 = read_le64(key + i + 8);
            k1 *= C1; k1 = rotl64(k1, 31); k1 *= C2; h1 ^= k1;
            h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
            k2 *= C2; k2 = rotl64(k2, 33); k2 *= C1; h2 ^= k2;
            h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
        }
        offset = len16;
    }
    uint64_t k1 = 0, k2 = 0;
    const uint8_t* t = key + offset;
    switch (length & 15) {
        case 15: k2 ^= (uint64_t)t[14] << 48;  // fallthrough
        case 14: k2 ^= (uint64_t)t[13] << 40;  // fallthrough
        case 13: k2 ^= (uint64_t)t[12] << 32;  // fallthrough
        case 12: k2 ^= (uint64_t)t[11] << 24;  // fallthrough
        case 11: k2 ^= (uint64_t)t[10] << 16;  // fallthrough
        case 10: k2 ^= (uint64_t)t[9] << 8;    // fallthrough
        case 9:
            k2 ^= (uint64_t)t[8];
            k2 *= C2; k2 = rotl64(k2, 33); k2 *= C1; h2 ^= k2;
            // fallthrough
        case 8: k1 ^= (uint64_t)t[7] << 56;  // fallthrough
        case 7: k1 ^= (uint64_t)t[6] << 48;  // fallthrough
        case 6: k1 ^= (uint64_t)t[5] << 40;  // fallthrough
        case 5: k1 ^= (uint64_t)t[4] << 32;  // fallthrough
        case 4: k1 ^= (uint64_t)t[3] << 24;  // fallthrough
        case 3: k1 ^= (uint64_t)t[2] << 16;  // fallthrough
        case 2: k1 ^= (uint64_t)t[1] << 8;   // fallthrough
        case 1:
            k1 ^= (uint64_t)t[0];
            k1 *= C1; k1 = rotl64(k1, 31); k1 *= C2; h1 ^= k1;
    }
    h1 ^= (uint64_t)(int64_t)length;
    h2 ^= (uint64_t)(int64_t)length;
    h1 += h2; h2 += h1;
    h1 = fmix(h1); h2 = fmix(h2);
    h1 += h2; h2 += h1;
    *o1 = h1; *o2 = h2;
}

// ------------------------------------------------------------------------------------------------------------
// Calendar arithmetic for joda ISOChronology UTC (proleptic Gregorian) — DateTimeUnit.java:36-43
// ------------------------------------------------------------------------------------------------------------
static int64_t days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
static void civil_from_days(int64_t z, int64_t* y, int* m, int* d) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    *d = (int)(doy - (153 * mp + 2) / 5 + 1);
    *m = (int)(mp < 10 ? mp + 3 : mp - 9);
    *y = yoe + era * 400 + (*m <= 2);
}
static const int64_t MS_DAY = 86400000LL;

// ------------------------------------------------------------------------------------------------------------
// joda-time 2.8.2 DateTimeZone (third-party, not in /root/reference): getOffset / nextTransition over an offset
// history (offs[i] from UTC instant starts[i] on), convertUTCToLocal, and both convertLocalToUTC overloads, restated
// from joda's published DateTimeZone.java.  Pinned by TimeZoneRoundingTests' DST cases (kat.json "rounding_tz").
// An empty table is UTC.
// ------------------------------------------------------------------------------------------------------------
struct Zone {
    std::vector<int64_t> starts, offs;
    int64_t getOffset(int64_t instant) const {  // starts[0] is -infinity
        if (starts.empty()) return 0;
        size_t lo = 0, hi = starts.size();  // last i with starts[i] <= instant (i = 0 always qualifies)
        while (hi - lo > 1) {
            const size_t mid = (lo + hi) / 2;
            if (starts[mid] <= instant) lo = mid; else hi = mid;
        }
        return offs[lo];
    }
    int64_t nextTransition(int64_t instant) const {
        for (size_t lo = 1, hi = starts.size(); lo < hi;) {  // first i >= 1 with starts[i] > instant
            const size_t mid = (lo + hi) / 2;
            if (starts[mid] > instant) hi = mid; else lo = mid + 1;
            if (lo == hi) return lo < starts.size() ? starts[lo] : instant;
        }
        return instant;
    }
    int64_t convertUTCToLocal(int64_t utc) const { return utc + getOffset(utc); }
    int64_t convertLocalToUTC(int64_t instantLocal, bool strict) const {
        const int64_t offsetLocal = getOffset(instantLocal);
        int64_t offset = getOffset(instantLocal - offsetLocal);
        if (offsetLocal != offset) {
            if (strict || offsetLocal < 0) {
                int64_t nextLocal = nextTransition(instantLocal - offsetLocal);
                if (nextLocal == (instantLocal - offsetLocal)) nextLocal = INT64_MAX;
                int64_t nextAdjusted = nextTransition(instantLocal - offset);
                if (nextAdjusted == (instantLocal - offset)) nextAdjusted = INT64_MAX;
                if (nextLocal != nextAdjusted) {
                    if (strict) throw std::runtime_error("IllegalInstantException");
                    offset = offsetLocal;
                }
            }
        }
        return instantLocal - offset;
    }
    int64_t convertLocalToUTC(int64_t instantLocal, bool strict, int64_t originalInstantUTC) const {
        const int64_t offsetOriginal = getOffset(originalInstantUTC);
        const int64_t instantUTC = instantLocal - offsetOriginal;
        const int64_t offsetLocalFromOriginal = getOffset(instantUTC);
        if (offsetLocalFromOriginal == offsetOriginal) return instantUTC;
        return convertLocalToUTC(instantLocal, strict);
    }
};

// ------------------------------------------------------------------------------------------------------------
// Rounding (common/rounding/Rounding.java, TimeZoneRounding.java:101-217).  A fixed time-zone offset given without a
// zone table is folded into OffsetRounding by the caller (see include/esgpu.h esgpu_agg_spec.offset).
// ------------------------------------------------------------------------------------------------------------
struct Rounding {
    int kind = 0;       // 0 = Interval (histogram), 1 = TimeUnitRounding, 2 = TimeIntervalRounding
    int unit = 0;       // ESGPU_UNIT_*
    int64_t interval = 1;
    int64_t offset = 0; // OffsetRounding (Rounding.java:205-236); 0 = not wrapped
    Zone tz;            // TimeZoneRounding's timeZone (empty = UTC)

    int64_t inner_round_key(int64_t v) const {
        switch (kind) {
            case 0: return floor_div(v, interval);                  // Rounding.Interval.roundKey
            case 2: {                                               // TimeIntervalRounding.roundKey
                const int64_t timeLocal = tz.convertUTCToLocal(v);
                const int64_t rounded = floor_div(timeLocal, interval) * interval;
                return tz.convertLocalToUTC(rounded, false);
            }
            default: {                                              // TimeUnitRounding.roundKey
                const int64_t timeLocal = tz.convertUTCToLocal(v);
                const int64_t rounded = unit_floor(timeLocal);
                return tz.convertLocalToUTC(rounded, false, v);
            }
        }
    }
    int64_t inner_value_for_key(int64_t k) const { return kind == 0 ? k * interval : k; }
    int64_t inner_next(int64_t v) const {
        switch (kind) {
            case 0: return v + interval;
            case 2: return tz.convertLocalToUTC(tz.convertUTCToLocal(v) + interval, false);
            default: return tz.convertLocalToUTC(unit_add(tz.convertUTCToLocal(v)), false);
        }
    }
    int64_t unit_floor(int64_t t) const {  // joda DateTimeField.roundFloor in ISOChronology UTC
        switch (unit) {
            case ESGPU_UNIT_SECOND: return floor_div(t, 1000) * 1000;
            case ESGPU_UNIT_MINUTE: return floor_div(t, 60000) * 60000;
            case ESGPU_UNIT_HOUR: return floor_div(t, 3600000) * 3600000;
            case ESGPU_UNIT_DAY: return floor_div(t, MS_DAY) * MS_DAY;
            case ESGPU_UNIT_WEEK: {  // Monday 00:00; 1970-01-01 is a Thursday
                int64_t days = floor_div(t, MS_DAY);
                int64_t monday = days - ((days + 3) % 7 + 7) % 7;
                return monday * MS_DAY;
            }
            default: {
                int64_t y; int m, d;
                civil_from_days(floor_div(t, MS_DAY), &y, &m, &d);
                if (unit == ESGPU_UNIT_MONTH) return days_from_civil(y, m, 1) * MS_DAY;
                if (unit == ESGPU_UNIT_QUARTER) return days_from_civil(y, ((m - 1) / 3) * 3 + 1, 1) * MS_DAY;
                if (unit == ESGPU_UNIT_YEAR) return days_from_civil(y, 1, 1) * MS_DAY;
                throw std::runtime_error("bad date unit");
            }
        }
    }
    int64_t unit_add(int64_t t) const {  // DurationField.add(t, 1)
        switch (unit) {
            case ESGPU_UNIT_SECOND: return t + 1000;
            case ESGPU_UNIT_MINUTE: return t + 60000;
            case ESGPU_UNIT_HOUR: return t + 3600000;
            case ESGPU_UNIT_DAY: return t + MS_DAY;
            case ESGPU_UNIT_WEEK: return t + 7 * MS_DAY;
            default: {
                int64_t days = floor_div(t, MS_DAY);
                int64_t rem = t - days * MS_DAY;
                int64_t y; int m, d;
                civil_from_days(days, &y, &m, &d);
                int add = unit == ESGPU_UNIT_MONTH ? 1 : unit == ESGPU_UNIT_QUARTER ? 3 : 12;
                int64_t mm = (int64_t)(m - 1) + add;
                y += mm / 12; m = (int)(mm % 12) + 1;
                static const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
                int dim = mdays[m - 1] + ((m == 2 && ((y % 4 == 0 && y % 100 != 0) || y % 400 == 0)) ? 1 : 0);
                if (d > dim) d = dim;
                return days_from_civil(y, m, d) * MS_DAY + rem;
            }
        }
    }
    // OffsetRounding wrapper semantics
    int64_t round_key(int64_t v) const { return inner_round_key(v - offset); }
    int64_t value_for_key(int64_t k) const { return offset + inner_value_for_key(k); }
    int64_t next_rounding_value(int64_t v) const { return inner_next(v - offset) + offset; }
    int64_t round(int64_t v) const { return value_for_key(round_key(v)); }
};

static Rounding make_rounding(const esgpu_agg_spec& s) {
    Rounding r;
    if (s.type == ESGPU_AGG_HISTOGRAM) {
        r.kind = 0;
        r.interval = s.interval;
    } else if (s.date_unit != ESGPU_UNIT_NONE) {
        r.kind = 1;
        r.unit = s.date_unit;
    } else {
        r.kind = 2;
        r.interval = s.interval;
    }
    r.offset = s.offset;
    if (r.kind != 0 && s.tz_count > 0) {
        r.tz.starts.assign(s.tz_starts, s.tz_starts + s.tz_count);
        r.tz.offs.assign(s.tz_offsets_ms, s.tz_offsets_ms + s.tz_count);
    }
    if (r.kind != 1 && r.interval < 1) throw std::invalid_argument("interval must be >= 1");
    return r;
}

// ------------------------------------------------------------------------------------------------------------
// Column access (SortedNumericDocValues / SortedSetDocValues contract)
// ------------------------------------------------------------------------------------------------------------
struct Column {
    const esgpu_column_desc* d = nullptr;
    int count(uint32_t doc) const {
        if (d->offsets) return (int)(d->offsets[doc + 1] - d->offsets[doc]);
        if (d->type == ESGPU_COL_ORD_U32) return ((const uint32_t*)d->values)[doc] == 0xFFFFFFFFu ? 0 : 1;
        if (d->present) return (int)((d->present[doc >> 6] >> (doc & 63)) & 1);
        return 1;
    }
    uint64_t idx(uint32_t doc, int i) const { return d->offsets ? d->offsets[doc] + i : doc; }
    int64_t long_at(uint32_t doc, int i) const {  // ValuesSource.Numeric.longValues
        uint64_t k = idx(doc, i);
        if (d->type == ESGPU_COL_F64) return java_cast_long(((const double*)d->values)[k]);  // FieldData.castToLong
        if (d->type == ESGPU_COL_ORD_U32) return ((const uint32_t*)d->values)[k];
        return ((const int64_t*)d->values)[k];
    }
    double double_at(uint32_t doc, int i) const {  // ValuesSource.Numeric.doubleValues (FieldData.castToDouble)
        uint64_t k = idx(doc, i);
        if (d->type == ESGPU_COL_F64) return ((const double*)d->values)[k];
        if (d->type == ESGPU_COL_ORD_U32) return (double)((const uint32_t*)d->values)[k];
        return (double)((const int64_t*)d->values)[k];
    }
    uint32_t ord_at(uint32_t doc, int i) const { return ((const uint32_t*)d->values)[idx(doc, i)]; }
    std::string term(uint64_t ord) const {
        if (!d->dict_bytes || !d->dict_offsets) return std::to_string(ord);
        return std::string((const char*)d->dict_bytes + d->dict_offsets[ord],
                           (size_t)(d->dict_offsets[ord + 1] - d->dict_offsets[ord]));
    }
};

struct Segment {
    uint32_t max_doc = 0;
    std::map<std::string, Column> cols;
    const Column* col(const char* name) const {
        if (!name) return nullptr;
        auto it = cols.find(name);
        return it == cols.end() ? nullptr : &it->second;  // unmapped field => null values source
    }
};

// ------------------------------------------------------------------------------------------------------------
// HyperLogLogPlusPlus (A/metrics/cardinality/HyperLogLogPlusPlus.java) — restated with its LC hash set living
// inside the runLens byte array.
// ------------------------------------------------------------------------------------------------------------
static const int P2 = 25;
static const int BIAS_K = 6;

static int precision_from_threshold(int64_t count) {  // HyperLogLogPlusPlus.java:68-74
    const int64_t entries = (int64_t)std::ceil((double)((float)count / 0.75f));
    const int64_t v = entries * 4;
    int precision = v == 0 ? 1 : std::max(1, 64 - nlz64((uint64_t)v));  // PackedInts.bitsRequired
    precision = std::max(precision, 4);
    precision = std::min(precision, 18);
    return precision;
}
static int encode_hash(uint64_t hash, int p) {  // :335-347
    const uint64_t e = hash >> (64 - P2);
    uint64_t encoded;
    if ((e & ((1ULL << (P2 - p)) - 1)) == 0) {
        const int runLen = 1 + std::min(nlz64(hash << P2), 64 - P2);
        encoded = (e << 7) | ((uint64_t)runLen << 1) | 1;
    } else {
        encoded = e << 1;
    }
    return (int)(uint32_t)encoded;
}
static int decode_run_len(int encoded, int p) {  // :349-357
    if ((encoded & 1) == 1) return (((uint32_t)encoded >> 1) & 0x3F) + (P2 - p);
    const uint32_t bits = (uint32_t)encoded << (31 + p - P2);
    return 1 + nlz32(bits);
}
static int decode_index(int encoded, int p) {  // :359-367
    uint64_t index = (encoded & 1) == 1 ? ((uint32_t)encoded >> 7) : ((uint32_t)encoded >> 1);
    return (int)(index >> (P2 - p));
}
static int64_t hll_index(uint64_t hash, int p) { return (int64_t)(hash >> (64 - p)); }
static int run_len(uint64_t hash, int p) { return 1 + std::min(nlz64(hash << p), 64 - p); }
static int64_t linear_counting(int64_t m, int64_t v) { return java_round((double)m * std::log((double)m / (double)v)); }

struct HLLPP {
    int p, m;
    double alphaMM;
    std::vector<uint8_t> runLens;
    std::vector<bool> algorithm;  // false = LINEAR_COUNTING, true = HYPERLOGLOG
    std::vector<int> sizes;
    int capacity, threshold, mask;

    HLLPP(int precision, int64_t initialBuckets) : p(precision), m(1 << precision) {
        if (precision < 4 || precision > 18) throw std::invalid_argument("precision");
        runLens.assign((size_t)initialBuckets << p, 0);
        double alpha = p == 4 ? 0.673 : p == 5 ? 0.697 : 0.7213 / (1 + 1.079 / m);
        alphaMM = alpha * m * m;
        capacity = m / 4;
        threshold = (int)((float)capacity * 0.75f);
        mask = capacity - 1;
    }
    int64_t max_bucket() const { return (int64_t)(runLens.size() >> p); }
    void ensure(int64_t nb) {
        if ((int64_t)runLens.size() < (nb << p)) runLens.resize((size_t)nb << p, 0);
        if ((int64_t)sizes.size() < nb) sizes.resize((size_t)nb, 0);
        if ((int64_t)algorithm.size() < nb) algorithm.resize((size_t)nb, false);
    }
    bool algo(int64_t b) const { return b < (int64_t)algorithm.size() ? algorithm[b] : false; }
    // Hashset (:428-517)
    int hs_get(int64_t b, int i) const {
        size_t o = ((size_t)b << p) + ((size_t)i << 2);
        return (int)((uint32_t)runLens[o] | ((uint32_t)runLens[o + 1] << 8) | ((uint32_t)runLens[o + 2] << 16) |
                     ((uint32_t)runLens[o + 3] << 24));
    }
    void hs_set(int64_t b, int i, int v) {
        size_t o = ((size_t)b << p) + ((size_t)i << 2);
        runLens[o] = (uint8_t)v; runLens[o + 1] = (uint8_t)(v >> 8);
        runLens[o + 2] = (uint8_t)(v >> 16); runLens[o + 3] = (uint8_t)(v >> 24);
    }
    int hs_size(int64_t b) const { return b < (int64_t)sizes.size() ? sizes[b] : 0; }
    int hs_add(int64_t b, int k) {
        ensure(b + 1);
        for (int i = k & mask;; i = (i + 1) & mask) {
            const int v = hs_get(b, i);
            if (v == 0) { hs_set(b, i, k); return ++sizes[b]; }
            if (v == k) return -1;
        }
    }
    std::vector<int> hs_values(int64_t b) const {
        std::vector<int> out;
        if (hs_size(b) == 0) return out;
        for (int j = 0; j < capacity; ++j) {
            int k = hs_get(b, j);
            if (k != 0) out.push_back(k);
        }
        return out;
    }
    void collect(int64_t b, uint64_t hash) {  // :232-239
        ensure(b + 1);
        if (!algo(b)) collect_lc_encoded(b, encode_hash(hash, p));
        else collect_hll(b, hll_index(hash, p), run_len(hash, p));
    }
    void collect_lc_encoded(int64_t b, int enc) {
        const int newSize = hs_add(b, enc);
        if (newSize > threshold) upgrade_to_hll(b);
    }
    void collect_hll_encoded(int64_t b, int enc) { collect_hll(b, decode_index(enc, p), decode_run_len(enc, p)); }
    void collect_hll(int64_t b, int64_t index, int rl) {
        const size_t bi = ((size_t)b << p) + (size_t)index;
        runLens[bi] = (uint8_t)std::max(rl, (int)(int8_t)runLens[bi]);
    }
    void upgrade_to_hll(int64_t b) {  // :309-322
        ensure(b + 1);
        std::vector<int> values = hs_values(b);
        std::fill(runLens.begin() + ((size_t)b << p), runLens.begin() + (((size_t)b << p) + m), 0);
        for (int enc : values) collect_hll_encoded(b, enc);
        algorithm[b] = true;
    }
    void merge(int64_t thisBucket, const HLLPP& other, int64_t otherBucket) {  // :201-230
        if (p != other.p) throw std::invalid_argument("precision mismatch");
        ensure(thisBucket + 1);
        if (!other.algo(otherBucket)) {
            for (int enc : other.hs_values(otherBucket)) {
                if (!algo(thisBucket)) collect_lc_encoded(thisBucket, enc);
                else collect_hll_encoded(thisBucket, enc);
            }
        } else {
            if (!algo(thisBucket)) upgrade_to_hll(thisBucket);
            const size_t ts = (size_t)thisBucket << p, os = (size_t)otherBucket << p;
            for (int i = 0; i < m; ++i) runLens[ts + i] = std::max(runLens[ts + i], other.runLens[os + i]);
        }
    }
    double estimate_bias(double e) const {  // :378-405
        const double* raw = HLLPP_RAW[p - 4];
        const double* bias = HLLPP_BIAS[p - 4];
        const int n = HLLPP_TABLE_LEN[p - 4];
        double weights[BIAS_K] = {0, 0, 0, 0, 0, 0};
        int index = n - BIAS_K;
        for (int i = 0; i < n; ++i) {
            const double w = 1.0 / std::fabs(raw[i] - e);
            const int j = i % BIAS_K;
            if (std::isinf(w)) return bias[i];
            else if (weights[j] >= w) { index = i - BIAS_K; break; }
            weights[j] = w;
        }
        double weightSum = 0.0, biasSum = 0.0;
        for (int i = 0, j = index; i < BIAS_K; ++i, ++j) {
            biasSum += weights[i] * bias[j];
            weightSum += weights[i];
        }
        return biasSum / weightSum;
    }
    int64_t cardinality(int64_t b) const {  // :270-307
        if (!algo(b)) return linear_counting(1LL << P2, (1LL << P2) - hs_size(b));
        double inverseSum = 0;
        int zeros = 0;
        for (size_t i = (size_t)b << p, end = i + m; i < end; ++i) {
            const int rl = (int)(int8_t)runLens[i];
            inverseSum += 1. / (double)(1LL << rl);
            if (rl == 0) ++zeros;
        }
        double e1 = alphaMM / inverseSum;
        double e2 = e1 <= 5 * m ? e1 - estimate_bias(e1) : e1;
        int64_t h = zeros != 0 ? linear_counting(m, zeros) : java_round(e2);
        if (h <= HLLPP_THRESHOLDS[p - 4]) return h;
        return java_round(e2);
    }
};

// ------------------------------------------------------------------------------------------------------------
// Internal aggregation results (StringTerms, InternalHistogram, InternalStats, InternalExtendedStats,
// InternalAvg, InternalCardinality)
// ------------------------------------------------------------------------------------------------------------
struct Internal;
using InternalPtr = std::shared_ptr<Internal>;
using InternalList = std::vector<InternalPtr>;

struct Bucket {
    std::string term;        // terms key bytes
    int64_t key = 0;         // histogram key
    int64_t doc_count = 0;
    int64_t doc_count_error = 0;
    InternalList aggs;
};

// Exact shadow of a floating sum (checker only, off unless oracle_set_exact_shadow(1)): the value the reference's
// doc-order double additions approximate, so tests can tell the reference's own rounding error from the GPU's (SURVEY §7
// "Float parity").  Double-double accumulation (Knuth TwoSum into hi, the rounding errors summed into lo; relative error
// about n * 2^-104 of sum |v|); non-finite addends tracked apart with IEEE semantics (NaN, or +Inf with -Inf, give NaN).
struct XSum {
    double hi = 0.0, lo = 0.0;
    bool pinf = false, ninf = false, nan = false;
    void add(double v) {
        if (!std::isfinite(v)) {
            if (v != v) nan = true; else if (v > 0) pinf = true; else ninf = true;
            return;
        }
        const double s = hi + v, bp = s - hi, e = (hi - (s - bp)) + (v - bp);
        hi = s;
        lo += e;
    }
    void merge(const XSum& o) {
        add(o.hi);
        lo += o.lo;
        pinf |= o.pinf; ninf |= o.ninf; nan |= o.nan;
    }
    double value() const {
        if (nan || (pinf && ninf)) return NAN;
        if (pinf) return INFINITY;
        if (ninf) return -INFINITY;
        return hi + lo;
    }
};
static bool g_exact_shadow = false;

struct Internal {
    int type = 0;
    std::string name;
    // terms
    int order = ESGPU_ORDER_COUNT_DESC;
    std::string order_path;  // InternalOrder.Aggregation path
    int required_size = 10, shard_size = 10;
    int64_t min_doc_count = 1;
    bool show_err = false;
    int64_t doc_count_error = 0, other_doc_count = 0;
    std::vector<Bucket> buckets;
    // histogram
    bool keyed = false, date = false;
    bool has_empty_info = false;
    Rounding rounding;
    bool has_bmin = false, has_bmax = false;
    int64_t bmin = 0, bmax = 0;
    InternalList empty_subs;
    // metrics
    int64_t count = 0;
    double sum = 0, min = INFINITY, max = -INFINITY, sumsq = 0, sigma = 2.0;
    XSum xsum, xsq;  // exact shadows of sum / sumsq (g_exact_shadow)
    // cardinality
    std::shared_ptr<HLLPP> hll;
    // filter (InternalSingleBucketAggregation): doc_count in `count`, sub-aggregations here
    InternalList subs;
    // the ValueFormatter of the aggregation's ValuesSourceConfig and the request time zone (wire stream only)
    int value_format = ESGPU_FORMAT_RAW;
    std::string format, tz_id = "UTC";
    void set_format(const esgpu_agg_spec& sp) {
        value_format = sp.value_format;
        format = sp.format ? sp.format : "";
        tz_id = sp.time_zone && *sp.time_zone ? sp.time_zone : "UTC";
    }
};

// ---- comparators (A/bucket/terms/InternalOrder.java:47-76, CompoundOrder with _term asc tie-break) ----
static int term_compare(const std::string& a, const std::string& b) {  // BytesRef.compareTo (unsigned bytes)
    int c = std::memcmp(a.data(), b.data(), std::min(a.size(), b.size()));
    if (c != 0) return c < 0 ? -1 : 1;
    return a.size() < b.size() ? -1 : a.size() > b.size() ? 1 : 0;
}
template <class KeyCmp>
static int terms_compare(int order, int64_t ca, int64_t cb, KeyCmp keycmp) {
    switch (order) {
        case ESGPU_ORDER_COUNT_DESC: { int c = cb < ca ? -1 : cb > ca ? 1 : 0; return c != 0 ? c : keycmp(); }
        case ESGPU_ORDER_COUNT_ASC: { int c = ca < cb ? -1 : ca > cb ? 1 : 0; return c != 0 ? c : keycmp(); }
        case ESGPU_ORDER_TERM_ASC: return keycmp();
        case ESGPU_ORDER_TERM_DESC: return -keycmp();
    }
    throw std::invalid_argument("order");
}

// ---- InternalOrder.Aggregation (A/bucket/terms/InternalOrder.java:149-225) ----
// AggregationPath.parse of a one-element path (A/support/AggregationPath.java:68-113): "name", "name.key", "name[key]"
static void split_path(const std::string& path, std::string* name, std::string* key) {
    const size_t br = path.rfind('[');
    if (br != std::string::npos && path.back() == ']') { *name = path.substr(0, br); *key = path.substr(br + 1, path.size() - br - 2); return; }
    const size_t dot = path.rfind('.');
    if (dot == std::string::npos) { *name = path; key->clear(); return; }
    *name = path.substr(0, dot);
    *key = path.substr(dot + 1);
}
// InternalAvg.value / InternalStats.value(name) / InternalExtendedStats.value(name) (and the aggregators' metric(name,
// bucket), the same formulas)
static double metric_of(int type, const std::string& key, int64_t count, double sum, double mn, double mx, double sq, double sigma) {
    const double avg = sum / (double)count;
    if (type == ESGPU_AGG_AVG) return avg;
    if (key == "count") return (double)count;
    if (key == "sum") return sum;
    if (key == "min") return mn;
    if (key == "max") return mx;
    if (key == "avg") return avg;
    const double variance = (sq - ((sum * sum) / (double)count)) / (double)count;  // InternalExtendedStats.getVariance
    if (key == "sum_of_squares") return sq;
    if (key == "variance") return variance;
    if (key == "std_deviation") return std::sqrt(variance);
    if (key == "std_upper") return avg + (std::sqrt(variance) * sigma);
    if (key == "std_lower") return avg - (std::sqrt(variance) * sigma);
    throw std::invalid_argument("Unknown value [" + key + "] in common stats aggregation");
}
// Comparators.compareDiscardNaN (common/util/Comparators.java): NaN last, Double.compare otherwise
static int compare_discard_nan(double a, double b, bool asc) {
    if (a != a) return b != b ? 0 : 1;
    if (b != b) return -1;
    auto dcmp = [](double x, double y) {  // Double.compare
        if (x < y) return -1;
        if (x > y) return 1;
        uint64_t bx, by;
        std::memcpy(&bx, &x, 8);
        std::memcpy(&by, &y, 8);
        return bx == by ? 0 : ((int64_t)bx < (int64_t)by ? -1 : 1);
    };
    return asc ? dcmp(a, b) : dcmp(b, a);
}

// Lucene PriorityQueue.insertWithOverflow + pop-into-array, with lessThan(a,b) = cmp(a,b) > 0
// (BucketPriorityQueue.java:30-38).  Returns the top `size` elements in comparator order and the overflowed ones.
template <class T, class Cmp>
static std::vector<T> top_k(std::vector<T> cands, size_t size, Cmp cmp, std::vector<T>* overflow) {
    std::stable_sort(cands.begin(), cands.end(), [&](const T& a, const T& b) { return cmp(a, b) < 0; });
    if (overflow && cands.size() > size) overflow->assign(cands.begin() + size, cands.end());
    if (cands.size() > size) cands.resize(size);
    return cands;
}

// ------------------------------------------------------------------------------------------------------------
// Aggregators (collect + buildAggregation)
// ------------------------------------------------------------------------------------------------------------
struct Factory;
struct Aggregator {
    const Factory* f = nullptr;
    std::vector<std::unique_ptr<Aggregator>> subs;
    virtual ~Aggregator() {}
    virtual void set_leaf(const Segment& seg) { for (auto& s : subs) s->set_leaf(seg); }
    virtual void collect(uint32_t doc, int64_t bucket) = 0;
    virtual void post_collection() { for (auto& s : subs) s->post_collection(); }
    virtual InternalPtr build(int64_t bucket) = 0;
    virtual InternalPtr build_empty() = 0;
    void collect_subs(uint32_t doc, int64_t bucket) { for (auto& s : subs) s->collect(doc, bucket); }
    InternalList bucket_aggs(int64_t bucket) {  // BucketsAggregator.bucketAggregations
        InternalList out;
        for (auto& s : subs) out.push_back(s->build(bucket));
        return out;
    }
    InternalList bucket_empty_aggs() {
        InternalList out;
        for (auto& s : subs) out.push_back(s->build_empty());
        return out;
    }
};

struct Factory {
    esgpu_agg_spec spec;
    std::string name, field;
    std::vector<esgpu_filter> clauses;  // filter aggregation: its query (conjunction of term / range clauses)
    std::vector<std::unique_ptr<Factory>> children;
    const Factory* parent = nullptr;
    int precision = 14;
    std::unique_ptr<Aggregator> create(bool collectsFromSingleBucket) const;
    std::unique_ptr<Aggregator> create_one() const;
    bool is_bucket() const {
        return spec.type == ESGPU_AGG_TERMS || spec.type == ESGPU_AGG_HISTOGRAM || spec.type == ESGPU_AGG_DATE_HISTOGRAM;
    }
};

// AggregatorFactory.asMultiBucketAggregator (A/AggregatorFactory.java:118-235)
struct MultiBucketWrapper : Aggregator {
    std::vector<std::unique_ptr<Aggregator>> aggs;
    const Segment* seg = nullptr;
    std::vector<bool> leaf_set;
    std::unique_ptr<Aggregator> first;
    explicit MultiBucketWrapper(const Factory* fac) { f = fac; first = fac->create_one(); }
    void set_leaf(const Segment& s) override {
        seg = &s;
        leaf_set.assign(aggs.size(), false);
        if (first) { /* aggregator 0 is `first` */ }
    }
    Aggregator* get(int64_t b) {
        if ((int64_t)aggs.size() <= b) { aggs.resize((size_t)b + 1); leaf_set.resize((size_t)b + 1, false); }
        if (!aggs[b]) {
            if (b == 0 && first) aggs[0] = std::move(first);
            else aggs[b] = f->create_one();
        }
        if (!leaf_set[b]) { aggs[b]->set_leaf(*seg); leaf_set[b] = true; }
        return aggs[b].get();
    }
    void collect(uint32_t doc, int64_t bucket) override { get(bucket)->collect(doc, 0); }
    void post_collection() override { for (auto& a : aggs) if (a) a->post_collection(); }
    InternalPtr build(int64_t bucket) override {
        if (bucket < (int64_t)aggs.size() && aggs[bucket]) return aggs[bucket]->build(0);
        return build_empty();
    }
    InternalPtr build_empty() override {
        if (first) return first->build_empty();
        auto tmp = f->create_one();
        return tmp->build_empty();
    }
};

// the shard-level metric(name, bucketOrd) of a metrics sub-aggregator (defined after StatsAgg)
static double sub_metric(Aggregator* a, const std::string& key, int64_t bucket);

// GlobalOrdinalsStringTermsAggregator (A/bucket/terms/GlobalOrdinalsStringTermsAggregator.java:90-224)
struct TermsAgg : Aggregator {
    const Column* ords = nullptr;
    std::vector<int32_t> docCounts;  // BucketsAggregator.docCounts (IntArray)
    bool have_ctx = false;
    void set_leaf(const Segment& seg) override {
        ords = seg.col(f->field.c_str());
        if (ords) {
            have_ctx = true;
            if (docCounts.size() < ords->d->value_count) docCounts.resize(ords->d->value_count, 0);  // grow(valueCount)
        }
        Aggregator::set_leaf(seg);
    }
    void collect(uint32_t doc, int64_t bucket) override {
        if (!ords) return;
        const int n = ords->count(doc);
        for (int i = 0; i < n; ++i) {
            const uint32_t ord = ords->ord_at(doc, i);
            if (ord == 0xFFFFFFFFu) continue;  // ord < 0: missing
            if (docCounts.size() <= ord) docCounts.resize(ord + 1, 0);
            docCounts[ord] += 1;               // collectExistingBucket
            collect_subs(doc, ord);
        }
    }
    InternalPtr make(std::vector<Bucket> buckets, int64_t other) const {
        auto r = std::make_shared<Internal>();
        r->type = ESGPU_AGG_TERMS;
        r->name = f->name;
        r->order = f->spec.order;
        if (f->spec.order_path) r->order_path = f->spec.order_path;
        r->required_size = f->spec.size;
        r->shard_size = f->spec.shard_size;
        r->min_doc_count = f->spec.min_doc_count;
        r->show_err = f->spec.show_term_doc_count_error != 0;
        r->buckets = std::move(buckets);
        r->doc_count_error = 0;
        r->other_doc_count = other;
        return r;
    }
    InternalPtr build(int64_t bucket) override {  // buildAggregation (:146-208)
        if (!have_ctx) return build_empty();
        const esgpu_agg_spec& s = f->spec;
        const uint64_t valueCount = ords->d->value_count;
        struct OB { uint64_t ord; int64_t count; };
        std::vector<OB> cands;
        int64_t other = 0;
        for (uint64_t g = 0; g < valueCount; ++g) {
            const int64_t c = g < docCounts.size() ? docCounts[g] : 0;
            if (s.min_doc_count > 0 && c == 0) continue;
            other += c;
            if (s.shard_min_doc_count <= c) cands.push_back({g, c});
        }
        size_t size = s.min_doc_count == 0 ? (size_t)std::min<uint64_t>(valueCount, (uint64_t)s.shard_size)
                                           : (size_t)std::min<uint64_t>(std::max<uint64_t>(valueCount, docCounts.size()),
                                                                        (uint64_t)s.shard_size);
        std::vector<OB> top;
        if (s.order == ESGPU_ORDER_AGG_ASC || s.order == ESGPU_ORDER_AGG_DESC) {
            // CompoundOrder(Aggregation(path), TERM_ASC) with the sub-aggregator's metric(key, bucketOrd)
            std::string name, key;
            split_path(s.order_path ? s.order_path : "", &name, &key);
            Aggregator* sub = nullptr;
            for (auto& a : subs) if (a->f->name == name) sub = a.get();
            if (!sub) throw std::invalid_argument("Invalid term-aggregator order path [" + std::string(s.order_path) + "]");
            std::unordered_map<uint64_t, double> v;
            for (const OB& c : cands) v[c.ord] = sub_metric(sub, key, (int64_t)c.ord);
            top = top_k(cands, size, [&](const OB& a, const OB& b) {
                const int c = compare_discard_nan(v[a.ord], v[b.ord], s.order == ESGPU_ORDER_AGG_ASC);
                return c != 0 ? c : (a.ord < b.ord ? -1 : a.ord > b.ord ? 1 : 0);
            }, (std::vector<OB>*)nullptr);
        } else {
            top = top_k(cands, size, [&](const OB& a, const OB& b) {
                return terms_compare(s.order, a.count, b.count, [&] { return a.ord < b.ord ? -1 : a.ord > b.ord ? 1 : 0; });
            }, (std::vector<OB>*)nullptr);
        }
        std::vector<Bucket> list;
        for (auto& ob : top) {
            Bucket b;
            b.term = ords->term(ob.ord);
            b.key = (int64_t)ob.ord;
            b.doc_count = ob.count;
            other -= ob.count;
            b.aggs = ob.count == 0 ? bucket_empty_aggs() : bucket_aggs((int64_t)ob.ord);
            b.doc_count_error = 0;
            list.push_back(std::move(b));
        }
        return make(std::move(list), other);
    }
    InternalPtr build_empty() override { return make({}, 0); }
};

// HistogramAggregator (A/bucket/histogram/HistogramAggregator.java:84-133)
struct HistogramAgg : Aggregator {
    Rounding rounding;
    const Column* values = nullptr;
    std::unordered_map<int64_t, int64_t> bucketOrds;  // LongHash: key -> ord in first-seen order
    std::vector<int64_t> keys;                         // ord -> key
    std::vector<int32_t> docCounts;
    void set_leaf(const Segment& seg) override {
        values = seg.col(f->field.c_str());
        Aggregator::set_leaf(seg);
    }
    void collect(uint32_t doc, int64_t bucket) override {
        if (!values) return;
        const int n = values->count(doc);
        int64_t previousKey = INT64_MIN;
        for (int i = 0; i < n; ++i) {
            const int64_t v = values->long_at(doc, i);
            const int64_t key = rounding.round_key(v);
            if (key == previousKey) continue;
            auto it = bucketOrds.find(key);
            int64_t ord;
            if (it == bucketOrds.end()) {
                ord = (int64_t)keys.size();
                bucketOrds.emplace(key, ord);
                keys.push_back(key);
                docCounts.push_back(0);
            } else {
                ord = it->second;
            }
            docCounts[ord] += 1;
            collect_subs(doc, ord);
            previousKey = key;
        }
    }
    InternalPtr base() {
        auto r = std::make_shared<Internal>();
        r->type = f->spec.type;
        r->name = f->name;
        r->date = f->spec.type == ESGPU_AGG_DATE_HISTOGRAM;
        r->set_format(f->spec);
        r->order = f->spec.order;
        r->keyed = f->spec.keyed != 0;
        r->min_doc_count = f->spec.min_doc_count;
        r->rounding = rounding;
        if (f->spec.min_doc_count == 0) {  // EmptyBucketInfo
            r->has_empty_info = true;
            r->has_bmin = f->spec.has_extended_bounds_min != 0;
            r->has_bmax = f->spec.has_extended_bounds_max != 0;
            r->bmin = f->spec.extended_bounds_min;
            r->bmax = f->spec.extended_bounds_max;
            r->empty_subs = bucket_empty_aggs();
        }
        return r;
    }
    InternalPtr build(int64_t bucket) override {
        auto r = base();
        for (size_t i = 0; i < keys.size(); ++i) {
            Bucket b;
            b.key = rounding.value_for_key(keys[i]);
            b.doc_count = docCounts[i];
            b.aggs = bucket_aggs((int64_t)i);
            r->buckets.push_back(std::move(b));
        }
        std::stable_sort(r->buckets.begin(), r->buckets.end(), [](const Bucket& a, const Bucket& b) { return a.key < b.key; });
        return r;
    }
    InternalPtr build_empty() override { return base(); }
};

// StatsAggegator / ExtendedStatsAggregator / AvgAggregator (A/metrics/stats/StatsAggegator.java:88-118,
// A/metrics/stats/extended/ExtendedStatsAggregator.java:91-127, A/metrics/avg/AvgAggregator.java:80-95)
struct StatsAgg : Aggregator {
    const Column* values = nullptr;
    std::vector<int64_t> counts;
    std::vector<double> sums, mins, maxes, sumsqs;
    std::vector<XSum> xsums, xsqs;  // exact shadows (g_exact_shadow only)
    bool ext = false, avg = false;
    void set_leaf(const Segment& seg) override { values = seg.col(f->field.c_str()); }
    void grow(int64_t b) {
        if ((int64_t)counts.size() > b) return;
        size_t n = (size_t)b + 1;
        counts.resize(n, 0); sums.resize(n, 0.0); sumsqs.resize(n, 0.0);
        mins.resize(n, INFINITY); maxes.resize(n, -INFINITY);
        if (g_exact_shadow) { xsums.resize(n); xsqs.resize(n); }
    }
    void collect(uint32_t doc, int64_t bucket) override {
        if (!values) return;
        grow(bucket);
        const int n = values->count(doc);
        counts[bucket] += n;
        double sum = 0, sumOfSqr = 0;
        double mn = mins[bucket], mx = maxes[bucket];
        for (int i = 0; i < n; ++i) {
            const double v = values->double_at(doc, i);
            sum += v;
            if (ext) sumOfSqr += v * v;
            if (!avg) { mn = java_min(mn, v); mx = java_max(mx, v); }
            if (g_exact_shadow) {
                xsums[bucket].add(v);
                if (ext) xsqs[bucket].add(v * v);  // the reference's rounded products, summed exactly
            }
        }
        sums[bucket] += sum;
        if (ext) sumsqs[bucket] += sumOfSqr;
        if (!avg) { mins[bucket] = mn; maxes[bucket] = mx; }
    }
    InternalPtr make(int64_t c, double s, double mn, double mx, double sq) {
        auto r = std::make_shared<Internal>();
        r->type = f->spec.type;
        r->name = f->name;
        r->count = c; r->sum = s; r->min = mn; r->max = mx; r->sumsq = sq;
        r->sigma = f->spec.sigma;
        r->set_format(f->spec);
        return r;
    }
    InternalPtr build(int64_t b) override {
        if (!values || b >= (int64_t)counts.size()) return build_empty();
        InternalPtr r = make(counts[b], sums[b], mins[b], maxes[b], sumsqs[b]);
        if (g_exact_shadow) { r->xsum = xsums[b]; r->xsq = xsqs[b]; }
        return r;
    }
    InternalPtr build_empty() override { return make(0, 0.0, INFINITY, -INFINITY, 0.0); }
};

static double card_metric(Aggregator* a, const std::string& key, int64_t b);
static double sub_metric(Aggregator* a, const std::string& key, int64_t b) {  // StatsAggegator / AvgAggregator .metric
    if (a->f->spec.type == ESGPU_AGG_CARDINALITY) return card_metric(a, key, b);
    StatsAgg* sa = dynamic_cast<StatsAgg*>(a);
    if (!sa) throw std::invalid_argument("terms order path must name a metrics aggregation");
    const bool have = sa->values && b < (int64_t)sa->counts.size();
    const int64_t cnt = have ? sa->counts[b] : 0;
    return metric_of(sa->f->spec.type, key, cnt, have ? sa->sums[b] : 0.0, have ? sa->mins[b] : INFINITY,
                     have ? sa->maxes[b] : -INFINITY, have ? sa->sumsqs[b] : 0.0, sa->f->spec.sigma);
}

// CardinalityAggregator (A/metrics/cardinality/CardinalityAggregator.java:80-150,186-294)
struct CardinalityAgg : Aggregator {
    std::unique_ptr<HLLPP> counts;
    const Column* values = nullptr;
    std::vector<std::vector<bool>> visited;  // OrdinalsCollector per-bucket FixedBitSet
    bool ords_mode = false;
    void set_leaf(const Segment& seg) override {
        post_leaf();
        values = seg.col(f->field.c_str());
        ords_mode = false;
        if (values && values->d->type == ESGPU_COL_ORD_U32) {
            const int64_t maxOrd = (int64_t)values->d->value_count;
            const int64_t ordinalsMemory = 8 + 32 + (maxOrd + 7) / 8;  // OrdinalsCollector.memoryOverhead
            const int64_t countsMemory = 1LL << f->precision;
            ords_mode = maxOrd > 0 && ordinalsMemory < countsMemory / 4;
            visited.clear();
        }
        if (values && !counts) counts.reset(new HLLPP(f->precision, 1));
    }
    uint64_t hash_of(uint32_t doc, int i) const {
        switch (values->d->type) {
            case ESGPU_COL_F64: {  // MurmurHash3Values.Double: mix64(doubleToLongBits(v))
                double v = values->double_at(doc, i);
                uint64_t bits;
                if (v != v) bits = 0x7ff8000000000000ULL;
                else std::memcpy(&bits, &v, 8);
                return mix64(bits);
            }
            case ESGPU_COL_ORD_U32: {  // MurmurHash3Values.Bytes: hash128(bytes, 0).h1
                std::string t = values->term(values->ord_at(doc, i));
                uint64_t h1, h2;
                murmur3_128((const uint8_t*)t.data(), (int)t.size(), 0, &h1, &h2);
                return h1;
            }
            default: return mix64((uint64_t)values->long_at(doc, i));  // MurmurHash3Values.Long
        }
    }
    void collect(uint32_t doc, int64_t bucket) override {
        if (!values) return;
        const int n = values->count(doc);
        if (ords_mode) {
            if ((int64_t)visited.size() <= bucket) visited.resize((size_t)bucket + 1);
            auto& bits = visited[bucket];
            if (bits.empty()) bits.assign(values->d->value_count, false);
            for (int i = 0; i < n; ++i) {
                uint32_t o = values->ord_at(doc, i);
                if (o != 0xFFFFFFFFu) bits[o] = true;
            }
            return;
        }
        for (int i = 0; i < n; ++i) counts->collect(bucket, hash_of(doc, i));
    }
    void post_leaf() {  // OrdinalsCollector.postCollect (:259-282)
        if (!ords_mode || !values) return;
        const uint64_t maxOrd = values->d->value_count;
        std::vector<bool> all(maxOrd, false);
        for (auto& b : visited) for (uint64_t o = 0; o < b.size(); ++o) if (b[o]) all[o] = true;
        std::vector<uint64_t> hashes(maxOrd, 0);
        for (uint64_t o = 0; o < maxOrd; ++o) {
            if (!all[o]) continue;
            std::string t = values->term(o);
            uint64_t h1, h2;
            murmur3_128((const uint8_t*)t.data(), (int)t.size(), 0, &h1, &h2);
            hashes[o] = h1;
        }
        for (int64_t b = (int64_t)visited.size() - 1; b >= 0; --b)
            for (uint64_t o = 0; o < visited[b].size(); ++o)
                if (visited[b][o]) counts->collect(b, hashes[o]);
        visited.clear();
        ords_mode = false;
    }
    void post_collection() override { post_leaf(); }
    InternalPtr make(std::shared_ptr<HLLPP> h) {
        auto r = std::make_shared<Internal>();
        r->type = ESGPU_AGG_CARDINALITY;
        r->name = f->name;
        r->set_format(f->spec);
        r->hll = std::move(h);
        return r;
    }
    InternalPtr build(int64_t b) override {
        if (!counts || b >= counts->max_bucket() || counts->cardinality(b) == 0) return build_empty();
        auto copy = std::make_shared<HLLPP>(f->precision, 1);
        copy->merge(0, *counts, b);
        return make(copy);
    }
    InternalPtr build_empty() override { return make(nullptr); }
};

// CardinalityAggregator.metric (:136-138): counts.cardinality(bucketOrd), a single-value metric (InternalOrder.Aggregation
// accepts no other key than "value"); the collectors have posted their hashes before buildAggregation asks
static double card_metric(Aggregator* a, const std::string& key, int64_t b) {
    if (!key.empty() && key != "value")
        throw std::invalid_argument("Ordering on a single-value metrics aggregation can only be done on its value.");
    CardinalityAgg* ca = dynamic_cast<CardinalityAgg*>(a);
    if (!ca || !ca->counts || b >= ca->counts->max_bucket()) return 0.0;
    return (double)ca->counts->cardinality(b);
}

// FilterAggregator (A/bucket/filter/FilterAggregator.java:57-81): a SingleBucketAggregator; collect(doc, bucket) counts
// the doc into docCounts[bucket] and collects the sub-aggregators iff the doc matches the filter's query.  Not wrapped
// by asMultiBucketAggregator (it keeps one doc count per owning bucket itself).
struct FilterAgg : Aggregator {
    const Segment* seg = nullptr;
    std::vector<int64_t> docCounts;
    void set_leaf(const Segment& s) override { seg = &s; Aggregator::set_leaf(s); }
    void collect(uint32_t doc, int64_t bucket) override;
    InternalPtr make(int64_t bucket, bool empty) {
        auto r = std::make_shared<Internal>();
        r->type = ESGPU_AGG_FILTER;
        r->name = f->name;
        r->count = (!empty && bucket < (int64_t)docCounts.size()) ? docCounts[bucket] : 0;
        r->subs = empty ? bucket_empty_aggs() : bucket_aggs(bucket);
        return r;
    }
    InternalPtr build(int64_t bucket) override { return make(bucket, false); }
    InternalPtr build_empty() override { return make(0, true); }
};

static bool doc_matches(const Segment& seg, uint32_t doc, const esgpu_filter* flt, int nf, const uint64_t* accept);

void FilterAgg::collect(uint32_t doc, int64_t bucket) {
    if (!doc_matches(*seg, doc, f->clauses.data(), (int)f->clauses.size(), nullptr)) return;
    if ((int64_t)docCounts.size() <= bucket) docCounts.resize((size_t)bucket + 1, 0);
    ++docCounts[bucket];  // collectBucket
    collect_subs(doc, bucket);
}

std::unique_ptr<Aggregator> Factory::create_one() const {
    std::unique_ptr<Aggregator> a;
    switch (spec.type) {
        case ESGPU_AGG_TERMS: a.reset(new TermsAgg()); break;
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM: {
            auto* h = new HistogramAgg();
            h->rounding = make_rounding(spec);
            a.reset(h);
            break;
        }
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS:
        case ESGPU_AGG_AVG: {
            auto* s = new StatsAgg();
            s->ext = spec.type == ESGPU_AGG_EXTENDED_STATS;
            s->avg = spec.type == ESGPU_AGG_AVG;
            a.reset(s);
            break;
        }
        case ESGPU_AGG_CARDINALITY: a.reset(new CardinalityAgg()); break;
        case ESGPU_AGG_FILTER: a.reset(new FilterAgg()); break;
        default: throw std::invalid_argument("unsupported aggregation type " + std::to_string(spec.type));
    }
    a->f = this;
    for (auto& c : children) a->subs.push_back(c->create(false));  // createSubAggregators: collectsFromSingleBucket=false
    return a;
}
std::unique_ptr<Aggregator> Factory::create(bool single) const {
    if (!single && is_bucket()) return std::unique_ptr<Aggregator>(new MultiBucketWrapper(this));
    return create_one();
}

// ------------------------------------------------------------------------------------------------------------
// Reduce (A/InternalAggregations.java:133-161 and each doReduce)
// ------------------------------------------------------------------------------------------------------------
static InternalList reduce_list(const std::vector<InternalList>& lists);

static InternalPtr reduce_one(const InternalList& aggs) {
    const Internal& first = *aggs[0];
    auto r = std::make_shared<Internal>(first);
    switch (first.type) {
        case ESGPU_AGG_FILTER: {  // InternalSingleBucketAggregation.doReduce (A/bucket/InternalSingleBucketAggregation.java:85-95)
            int64_t dc = 0;
            std::vector<InternalList> lists;
            for (auto& a : aggs) { dc += a->count; lists.push_back(a->subs); }
            r->count = dc;
            r->subs = reduce_list(lists);
            return r;
        }
        case ESGPU_AGG_TERMS: {  // InternalTerms.doReduce (A/bucket/terms/InternalTerms.java:165-246)
            std::map<std::string, std::vector<const Bucket*>> groups;  // iteration order irrelevant (strict order)
            std::vector<std::string> key_order;
            int64_t sumDocCountError = 0, otherDocCount = 0;
            std::vector<int64_t> aggErr(aggs.size());
            for (size_t a = 0; a < aggs.size(); ++a) {
                const Internal& t = *aggs[a];
                otherDocCount += t.other_doc_count;
                int64_t thisErr;
                if ((int64_t)t.buckets.size() < first.shard_size || first.order == ESGPU_ORDER_TERM_ASC ||
                    first.order == ESGPU_ORDER_TERM_DESC) thisErr = 0;
                else if (first.order == ESGPU_ORDER_COUNT_DESC) thisErr = t.buckets.back().doc_count;
                else thisErr = -1;
                if (sumDocCountError != -1) sumDocCountError = thisErr == -1 ? -1 : sumDocCountError + thisErr;
                aggErr[a] = thisErr;
                for (const Bucket& b : t.buckets) {
                    auto it = groups.find(b.term);
                    if (it == groups.end()) { key_order.push_back(b.term); groups[b.term] = {}; }
                    groups[b.term].push_back(&b);
                }
            }
            std::vector<Bucket> reduced;
            for (const std::string& k : key_order) {
                const auto& same = groups[k];
                Bucket nb;  // Bucket.reduce (:91-108)
                nb.term = k;
                nb.key = same[0]->key;
                int64_t docCount = 0, docCountError = 0;
                std::vector<InternalList> subl;
                for (const Bucket* b : same) {
                    docCount += b->doc_count;
                    // bucket.docCountError was set to the owning shard's thisAggDocCountError
                    int64_t be = 0;
                    for (size_t a = 0; a < aggs.size(); ++a)
                        if (b >= aggs[a]->buckets.data() && b < aggs[a]->buckets.data() + aggs[a]->buckets.size()) be = aggErr[a];
                    if (docCountError != -1) docCountError = be == -1 ? -1 : docCountError + be;
                    subl.push_back(b->aggs);
                }
                nb.doc_count = docCount;
                nb.doc_count_error = docCountError;
                nb.aggs = reduce_list(subl);
                if (nb.doc_count_error != -1)
                    nb.doc_count_error = sumDocCountError == -1 ? -1 : sumDocCountError - nb.doc_count_error;
                if (nb.doc_count >= first.min_doc_count) reduced.push_back(std::move(nb));
            }
            const size_t size = std::min<size_t>((size_t)first.required_size, key_order.size());
            std::vector<Bucket> overflow;
            std::vector<Bucket> top;
            if (first.order == ESGPU_ORDER_AGG_ASC || first.order == ESGPU_ORDER_AGG_DESC) {
                // SubAggregationComparator: AggregationPath.resolveValue on the reduced bucket, then _term asc
                std::string name, key;
                split_path(first.order_path, &name, &key);
                auto value = [&](const Bucket& b) {
                    for (const InternalPtr& a : b.aggs) {
                        if (a->name != name) continue;
                        if (a->type == ESGPU_AGG_CARDINALITY) return (double)(a->hll ? a->hll->cardinality(0) : 0);  // .value()
                        return metric_of(a->type, key, a->count, a->sum, a->min, a->max, a->sumsq, a->sigma);
                    }
                    throw std::invalid_argument("Invalid order path [" + first.order_path + "]");
                };
                std::vector<double> vals(reduced.size());
                for (size_t i = 0; i < reduced.size(); ++i) { vals[i] = value(reduced[i]); reduced[i].key = (int64_t)i; }
                top = top_k(std::move(reduced), size, [&](const Bucket& a, const Bucket& b) {
                    const int c = compare_discard_nan(vals[a.key], vals[b.key], first.order == ESGPU_ORDER_AGG_ASC);
                    return c != 0 ? c : term_compare(a.term, b.term);
                }, &overflow);
            } else {
                top = top_k(std::move(reduced), size, [&](const Bucket& a, const Bucket& b) {
                    return terms_compare(first.order, a.doc_count, b.doc_count, [&] { return term_compare(a.term, b.term); });
                }, &overflow);
            }
            for (auto& o : overflow) otherDocCount += o.doc_count;
            r->buckets = std::move(top);
            r->doc_count_error = sumDocCountError == -1 ? -1 : (aggs.size() == 1 ? 0 : sumDocCountError);
            r->other_doc_count = otherDocCount;
            return r;
        }
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM: {  // InternalHistogram.doReduce (A/bucket/histogram/InternalHistogram.java:338-476)
            std::map<int64_t, std::vector<const Bucket*>> byKey;  // k-way merge by key; shard order within a key
            for (auto& a : aggs) for (const Bucket& b : a->buckets) byKey[b.key].push_back(&b);
            std::vector<Bucket> list;
            for (auto& kv : byKey) {
                Bucket nb;
                nb.key = kv.first;
                std::vector<InternalList> subl;
                for (const Bucket* b : kv.second) { nb.doc_count += b->doc_count; subl.push_back(b->aggs); }
                nb.aggs = reduce_list(subl);
                if (nb.doc_count >= first.min_doc_count) list.push_back(std::move(nb));
            }
            if (first.min_doc_count == 0 && first.has_empty_info) {  // addEmptyBuckets (:395-449)
                const Rounding& rd = first.rounding;
                std::vector<Bucket> out;
                auto empty = [&](int64_t key) {
                    Bucket e; e.key = key; e.doc_count = 0; e.aggs = first.empty_subs; return e;
                };
                if (list.empty()) {
                    if (first.has_bmin && first.has_bmax)
                        for (int64_t key = first.bmin; key <= first.bmax; key = rd.next_rounding_value(key)) out.push_back(empty(key));
                } else {
                    if (first.has_bmin)
                        for (int64_t key = first.bmin; key < list[0].key; key = rd.next_rounding_value(key)) out.push_back(empty(key));
                    const Bucket* last = nullptr;
                    for (Bucket& b : list) {
                        if (last) for (int64_t key = rd.next_rounding_value(last->key); key < b.key; key = rd.next_rounding_value(key))
                            out.push_back(empty(key));
                        out.push_back(b);
                        last = &b;
                    }
                    if (first.has_bmax && first.bmax > out.back().key) {
                        int64_t lastKey = out.back().key;
                        for (int64_t key = rd.next_rounding_value(lastKey); key <= first.bmax; key = rd.next_rounding_value(key))
                            out.push_back(empty(key));
                    }
                }
                list = std::move(out);
            }
            if (first.order == ESGPU_ORDER_KEY_DESC) std::reverse(list.begin(), list.end());
            else if (first.order == ESGPU_ORDER_HCOUNT_ASC || first.order == ESGPU_ORDER_HCOUNT_DESC) {
                const bool asc = first.order == ESGPU_ORDER_HCOUNT_ASC;
                std::stable_sort(list.begin(), list.end(), [&](const Bucket& a, const Bucket& b) {
                    if (a.doc_count != b.doc_count) return asc ? a.doc_count < b.doc_count : a.doc_count > b.doc_count;
                    return a.key < b.key;
                });
            }
            r->buckets = std::move(list);
            return r;
        }
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS:
        case ESGPU_AGG_AVG: {  // InternalStats/InternalExtendedStats/InternalAvg.doReduce
            int64_t count = 0;
            double mn = INFINITY, mx = -INFINITY, sum = 0, sq = 0;
            r->xsum = XSum();
            r->xsq = XSum();
            for (auto& a : aggs) {
                count += a->count;
                mn = java_min(mn, a->min);
                mx = java_max(mx, a->max);
                sum += a->sum;
                sq += a->sumsq;
                r->xsum.merge(a->xsum);
                r->xsq.merge(a->xsq);
            }
            r->count = count; r->min = mn; r->max = mx; r->sum = sum; r->sumsq = sq;
            return r;
        }
        case ESGPU_AGG_CARDINALITY: {  // InternalCardinality.doReduce (A/metrics/cardinality/InternalCardinality.java:103-121)
            std::shared_ptr<HLLPP> reduced;
            for (auto& a : aggs) {
                if (!a->hll) continue;
                if (!reduced) reduced = std::make_shared<HLLPP>(a->hll->p, 1);
                reduced->merge(0, *a->hll, 0);
            }
            if (!reduced) return aggs[0];
            r->hll = reduced;
            return r;
        }
    }
    throw std::invalid_argument("reduce: type");
}

static InternalList reduce_list(const std::vector<InternalList>& lists) {
    InternalList out;
    if (lists.empty()) return out;
    for (size_t i = 0; i < lists[0].size(); ++i) {
        InternalList same;
        for (auto& l : lists) same.push_back(l[i]);
        out.push_back(reduce_one(same));
    }
    return out;
}

// ------------------------------------------------------------------------------------------------------------
// JSON (XContent-like, lossless)
// ------------------------------------------------------------------------------------------------------------
struct Json {
    std::string s;
    void raw(const char* t) { s += t; }
    void str(const std::string& v) {
        s += '"';
        for (unsigned char c : v) {
            if (c == '"' || c == '\\') { s += '\\'; s += (char)c; }
            else if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); s += b; }
            else s += (char)c;
        }
        s += '"';
    }
    void i64(int64_t v) { s += std::to_string(v); }
    void dbl(double v) {
        if (v != v) { s += "NaN"; return; }
        if (std::isinf(v)) { s += v > 0 ? "Infinity" : "-Infinity"; return; }
        char b[40];
        snprintf(b, sizeof b, "%.17g", v);
        s += b;
        if (!strpbrk(b, ".eE")) s += ".0";
    }
    void key(const char* k) { str(k); s += ':'; }
};

static std::string iso8601(int64_t ms) {
    int64_t days = floor_div(ms, MS_DAY);
    int64_t rem = ms - days * MS_DAY;
    int64_t y; int m, d;
    civil_from_days(days, &y, &m, &d);
    char b[64];
    snprintf(b, sizeof b, "%04lld-%02d-%02dT%02d:%02d:%02d.%03dZ", (long long)y, m, d, (int)(rem / 3600000),
             (int)(rem / 60000 % 60), (int)(rem / 1000 % 60), (int)(rem % 1000));
    return b;
}

static uint64_t fnv1a(const uint8_t* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ULL; }
    return h;
}

static void write_list(Json& j, const InternalList& aggs);

// g_exact_shadow: ,"_exact":{...} -- the metric's rendered values recomputed from the exact sums with the same formulas
// (InternalStats / InternalExtendedStats / InternalAvg getters), so a test can compare either value against either
static void write_exact(Json& j, const Internal& a) {
    const double sum = a.xsum.value(), sq = a.xsq.value();
    j.raw(","); j.key("_exact"); j.raw("{");
    if (a.type == ESGPU_AGG_AVG) {
        j.key("value"); if (a.count != 0) j.dbl(sum / (double)a.count); else j.raw("null");
        j.raw(","); j.key("_internal"); j.raw("{"); j.key("sum"); j.dbl(sum); j.raw("}");
    } else {
        const bool c = a.count != 0;
        const double avg = sum / (double)a.count;
        j.key("avg"); if (c) j.dbl(avg); else j.raw("null"); j.raw(",");
        j.key("sum"); if (c) j.dbl(sum); else j.raw("null");
        if (a.type == ESGPU_AGG_EXTENDED_STATS) {
            const double var = (sq - ((sum * sum) / (double)a.count)) / (double)a.count;
            const double sd = std::sqrt(var);
            j.raw(","); j.key("sum_of_squares"); if (c) j.dbl(sq); else j.raw("null");
            j.raw(","); j.key("variance"); if (c) j.dbl(var); else j.raw("null");
            j.raw(","); j.key("std_deviation"); if (c) j.dbl(sd); else j.raw("null");
            j.raw(","); j.key("std_deviation_bounds"); j.raw("{");
            j.key("upper"); if (c) j.dbl(avg + (sd * a.sigma)); else j.raw("null"); j.raw(",");
            j.key("lower"); if (c) j.dbl(avg - (sd * a.sigma)); else j.raw("null"); j.raw("}");
        }
        j.raw(","); j.key("_internal"); j.raw("{"); j.key("sum"); j.dbl(sum);
        if (a.type == ESGPU_AGG_EXTENDED_STATS) { j.raw(","); j.key("sum_of_squares"); j.dbl(sq); }
        j.raw("}");
    }
    j.raw("}");
}

static void write_agg(Json& j, const Internal& a) {
    j.raw("{");
    switch (a.type) {
        case ESGPU_AGG_FILTER:  // InternalSingleBucketAggregation.doXContentBody (:130-134)
            j.key("doc_count"); j.i64(a.count);
            if (!a.subs.empty()) { j.raw(","); write_list(j, a.subs); }
            break;
        case ESGPU_AGG_TERMS: {
            j.key("doc_count_error_upper_bound"); j.i64(a.doc_count_error); j.raw(",");
            j.key("sum_other_doc_count"); j.i64(a.other_doc_count); j.raw(",");
            j.key("buckets"); j.raw("[");
            for (size_t i = 0; i < a.buckets.size(); ++i) {
                const Bucket& b = a.buckets[i];
                if (i) j.raw(",");
                j.raw("{"); j.key("key"); j.str(b.term); j.raw(",");
                j.key("doc_count"); j.i64(b.doc_count);
                if (a.show_err) { j.raw(","); j.key("doc_count_error_upper_bound"); j.i64(b.doc_count_error); }
                if (!b.aggs.empty()) { j.raw(","); write_list(j, b.aggs); }
                j.raw("}");
            }
            j.raw("]");
            break;
        }
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM: {
            j.key("buckets"); j.raw("[");
            for (size_t i = 0; i < a.buckets.size(); ++i) {
                const Bucket& b = a.buckets[i];
                if (i) j.raw(",");
                j.raw("{");
                if (a.date) { j.key("key_as_string"); j.str(iso8601(b.key)); j.raw(","); }
                j.key("key"); j.i64(b.key); j.raw(",");
                j.key("doc_count"); j.i64(b.doc_count);
                if (!b.aggs.empty()) { j.raw(","); write_list(j, b.aggs); }
                j.raw("}");
            }
            j.raw("]");
            break;
        }
        case ESGPU_AGG_AVG: {
            j.key("value");
            if (a.count != 0) j.dbl(a.sum / (double)a.count); else j.raw("null");
            j.raw(","); j.key("_internal"); j.raw("{"); j.key("count"); j.i64(a.count); j.raw(",");
            j.key("sum"); j.dbl(a.sum); j.raw("}");
            if (g_exact_shadow) write_exact(j, a);
            break;
        }
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS: {
            const bool c = a.count != 0;
            const double avg = a.sum / (double)a.count;
            j.key("count"); j.i64(a.count); j.raw(",");
            j.key("min"); if (c) j.dbl(a.min); else j.raw("null"); j.raw(",");
            j.key("max"); if (c) j.dbl(a.max); else j.raw("null"); j.raw(",");
            j.key("avg"); if (c) j.dbl(avg); else j.raw("null"); j.raw(",");
            j.key("sum"); if (c) j.dbl(a.sum); else j.raw("null");
            if (a.type == ESGPU_AGG_EXTENDED_STATS) {  // InternalExtendedStats.java getVariance/getStdDeviation
                const double var = (a.sumsq - ((a.sum * a.sum) / (double)a.count)) / (double)a.count;
                const double sd = std::sqrt(var);
                j.raw(","); j.key("sum_of_squares"); if (c) j.dbl(a.sumsq); else j.raw("null");
                j.raw(","); j.key("variance"); if (c) j.dbl(var); else j.raw("null");
                j.raw(","); j.key("std_deviation"); if (c) j.dbl(sd); else j.raw("null");
                j.raw(","); j.key("std_deviation_bounds"); j.raw("{");
                j.key("upper"); if (c) j.dbl(avg + (sd * a.sigma)); else j.raw("null"); j.raw(",");
                j.key("lower"); if (c) j.dbl(avg - (sd * a.sigma)); else j.raw("null"); j.raw("}");
            }
            j.raw(","); j.key("_internal"); j.raw("{");
            j.key("count"); j.i64(a.count); j.raw(",");
            j.key("sum"); j.dbl(a.sum); j.raw(",");
            j.key("min"); j.dbl(a.min); j.raw(",");
            j.key("max"); j.dbl(a.max);
            if (a.type == ESGPU_AGG_EXTENDED_STATS) { j.raw(","); j.key("sum_of_squares"); j.dbl(a.sumsq); }
            j.raw("}");
            if (g_exact_shadow) write_exact(j, a);
            break;
        }
        case ESGPU_AGG_CARDINALITY: {
            j.key("value"); j.i64(a.hll ? a.hll->cardinality(0) : 0);
            j.raw(","); j.key("_internal"); j.raw("{");
            j.key("present"); j.i64(a.hll ? 1 : 0);
            if (a.hll) {
                const HLLPP& h = *a.hll;
                j.raw(","); j.key("precision"); j.i64(h.p);
                j.raw(","); j.key("mode"); j.str(h.algo(0) ? "hll" : "lc");
                if (h.algo(0)) {
                    char b[32];
                    snprintf(b, sizeof b, "%016llx", (unsigned long long)fnv1a(h.runLens.data(), (size_t)h.m));
                    j.raw(","); j.key("registers_fnv1a64"); j.str(b);
                } else {
                    std::vector<int> v = h.hs_values(0);
                    std::vector<uint32_t> u(v.begin(), v.end());
                    std::sort(u.begin(), u.end());
                    j.raw(","); j.key("lc_size"); j.i64((int64_t)u.size());
                    j.raw(","); j.key("lc_fnv1a64");
                    char b[32];
                    snprintf(b, sizeof b, "%016llx", (unsigned long long)fnv1a((const uint8_t*)u.data(), u.size() * 4));
                    j.str(b);
                }
            }
            j.raw("}");
            break;
        }
    }
    j.raw("}");
}

static void write_list(Json& j, const InternalList& aggs) {
    for (size_t i = 0; i < aggs.size(); ++i) {
        if (i) j.raw(",");
        j.key(aggs[i]->name.c_str());
        write_agg(j, *aggs[i]);
    }
}

// ------------------------------------------------------------------------------------------------------------
// Transport bytes of a shard result: InternalAggregations.writeTo (A/InternalAggregations.java:215-222), restated
// from each class's writeTo / doWriteTo over org.elasticsearch.common.io.stream.StreamOutput (C/common/io/stream/
// StreamOutput.java).  The LINEAR_COUNTING hashes come out in the hash table's slot order, as HyperLogLogPlusPlus
// .writeTo iterates hashSet.values(bucket) (HyperLogLogPlusPlus.java:519-528).
// ------------------------------------------------------------------------------------------------------------
struct StreamOutput {
    std::string b;
    void writeByte(int v) { b.push_back((char)(uint8_t)v); }
    void writeBoolean(bool v) { writeByte(v ? 1 : 0); }
    void writeInt(int32_t i) { writeByte(i >> 24); writeByte(i >> 16); writeByte(i >> 8); writeByte(i); }
    void writeLong(int64_t i) { writeInt((int32_t)(i >> 32)); writeInt((int32_t)i); }
    void writeVInt(int32_t i) {
        while ((i & ~0x7F) != 0) { writeByte((i & 0x7F) | 0x80); i = (int32_t)((uint32_t)i >> 7); }
        writeByte(i);
    }
    void writeVLong(int64_t i) {
        while ((i & ~0x7FLL) != 0) { writeByte((int)((i & 0x7F) | 0x80)); i = (int64_t)((uint64_t)i >> 7); }
        writeByte((int)i);
    }
    void writeDouble(double v) {  // Double.doubleToLongBits: NaN canonical
        int64_t bits;
        if (v != v) bits = 0x7ff8000000000000LL; else std::memcpy(&bits, &v, 8);
        writeLong(bits);
    }
    void writeString(const std::string& utf8) {  // String.length() chars, then each char as 1-3 bytes
        std::vector<uint32_t> chars;
        size_t i = 0;
        while (i < utf8.size()) {
            uint32_t c = (uint8_t)utf8[i], n = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
            if (i + n > utf8.size()) n = 1;
            uint32_t cp = n == 1 ? c : n == 2 ? (c & 0x1F) : n == 3 ? (c & 0x0F) : (c & 0x07);
            for (uint32_t k = 1; k < n; ++k) cp = (cp << 6) | ((uint8_t)utf8[i + k] & 0x3F);
            i += n;
            if (cp > 0xFFFF) { chars.push_back(0xD800 + ((cp - 0x10000) >> 10)); chars.push_back(0xDC00 + ((cp - 0x10000) & 0x3FF)); }
            else chars.push_back(cp);
        }
        writeVInt((int32_t)chars.size());
        for (uint32_t c : chars) {
            if (c <= 0x007F) writeByte((int)c);
            else if (c > 0x07FF) { writeByte(0xE0 | ((c >> 12) & 0x0F)); writeByte(0x80 | ((c >> 6) & 0x3F)); writeByte(0x80 | (c & 0x3F)); }
            else { writeByte(0xC0 | ((c >> 6) & 0x1F)); writeByte(0x80 | (c & 0x3F)); }
        }
    }
    void writeBytes(const std::string& bytes) { writeVInt((int32_t)bytes.size()); b += bytes; }  // writeBytesRef / Reference
};

static void writeSize(int size, StreamOutput& out) { out.writeVInt(size == INT32_MAX ? 0 : size); }  // InternalAggregation.java:181-186

static void writeFormatter(const Internal& a, StreamOutput& out) {  // ValueFormatterStreams.writeOptional / write
    out.writeBoolean(true);  // ValuesSourceParser.resolveFormat never yields null for a field
    if (a.value_format == ESGPU_FORMAT_DATE_TIME) { out.writeByte(2); out.writeString(a.format); out.writeString(a.tz_id); }
    else if (a.value_format == ESGPU_FORMAT_NUMBER) { out.writeByte(4); out.writeString(a.format); }
    else out.writeByte(1);  // ValueFormatter.Raw: writeTo writes nothing
}

static void writeRounding(const Internal& a, StreamOutput& out) {  // Rounding.Streams.write: id, then writeTo
    const Rounding& r = a.rounding;
    if (r.offset != 0) out.writeByte(8);  // OffsetRounding.writeTo: the inner rounding, then writeLong(offset)
    if (r.kind == 0) { out.writeByte(0); out.writeVLong(r.interval); }                            // Rounding.Interval
    else if (r.kind == 1) { out.writeByte(1); out.writeByte(r.unit); out.writeString(a.tz_id); }  // TimeUnitRounding
    else { out.writeByte(2); out.writeVLong(r.interval); out.writeString(a.tz_id); }              // TimeIntervalRounding
    if (r.offset != 0) out.writeLong(r.offset);
}

static void writeTermsOrder(const Internal& a, StreamOutput& out) {  // InternalOrder.Streams.writeOrder
    if (a.order == ESGPU_ORDER_TERM_ASC) { out.writeByte(4); return; }   // TermsParser: a lone term order stays itself
    if (a.order == ESGPU_ORDER_TERM_DESC) { out.writeByte(3); return; }
    out.writeByte(-1);  // CompoundOrder(user order, _term asc)
    out.writeVInt(2);
    if (a.order == ESGPU_ORDER_COUNT_DESC) out.writeByte(1);
    else if (a.order == ESGPU_ORDER_COUNT_ASC) out.writeByte(2);
    else { out.writeByte(0); out.writeBoolean(a.order == ESGPU_ORDER_AGG_ASC); out.writeString(a.order_path); }
    out.writeByte(4);
}

static void writeAggregations(const InternalList& aggs, StreamOutput& out);

static const char* streamType(int type) {
    switch (type) {
        case ESGPU_AGG_TERMS: return "sterms";
        case ESGPU_AGG_HISTOGRAM: return "histo";
        case ESGPU_AGG_DATE_HISTOGRAM: return "dhisto";
        case ESGPU_AGG_STATS: return "stats";
        case ESGPU_AGG_EXTENDED_STATS: return "estats";
        case ESGPU_AGG_AVG: return "avg";
        case ESGPU_AGG_CARDINALITY: return "cardinality";
        default: return "filter";
    }
}

static void writeAggregation(const Internal& a, StreamOutput& out) {  // InternalAggregation.writeTo (:212-221)
    out.writeString(a.name);
    out.writeByte(-1);  // writeGenericValue(null)
    out.writeVInt(0);   // pipelineAggregators.size()
    switch (a.type) {
        case ESGPU_AGG_TERMS:  // StringTerms.doWriteTo (:205-217)
            out.writeLong(a.doc_count_error);
            writeTermsOrder(a, out);
            writeSize(a.required_size, out);
            writeSize(a.shard_size, out);
            out.writeBoolean(a.show_err);
            out.writeVLong(a.min_doc_count);
            out.writeVLong(a.other_doc_count);
            out.writeVInt((int32_t)a.buckets.size());
            for (const Bucket& bk : a.buckets) {  // StringTerms.Bucket.writeTo (:128-136)
                out.writeBytes(bk.term);
                out.writeVLong(bk.doc_count);
                if (a.show_err) out.writeLong(bk.doc_count_error);
                writeAggregations(bk.aggs, out);
            }
            break;
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM:  // InternalHistogram.doWriteTo (:510-523)
            out.writeString(a.date ? "date_histogram" : "histogram");
            out.writeByte(a.order == ESGPU_ORDER_KEY_ASC ? 1 : a.order == ESGPU_ORDER_KEY_DESC ? 2 :
                          a.order == ESGPU_ORDER_HCOUNT_ASC ? 3 : 4);
            out.writeVLong(a.min_doc_count);
            if (a.min_doc_count == 0) {  // EmptyBucketInfo.writeTo (:223-230)
                writeRounding(a, out);
                writeAggregations(a.empty_subs, out);
                out.writeBoolean(a.has_bmin || a.has_bmax);
                if (a.has_bmin || a.has_bmax) {  // ExtendedBounds.writeTo
                    out.writeBoolean(a.has_bmin);
                    if (a.has_bmin) out.writeLong(a.bmin);
                    out.writeBoolean(a.has_bmax);
                    if (a.has_bmax) out.writeLong(a.bmax);
                }
            }
            writeFormatter(a, out);
            out.writeBoolean(a.keyed);
            out.writeVInt((int32_t)a.buckets.size());
            for (const Bucket& bk : a.buckets) {  // InternalHistogram.Bucket.writeTo (:183-187)
                out.writeLong(bk.key);
                out.writeVLong(bk.doc_count);
                writeAggregations(bk.aggs, out);
            }
            break;
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS:  // InternalStats.doWriteTo (:182-189), InternalExtendedStats.writeOtherStatsTo
            writeFormatter(a, out);
            out.writeVLong(a.count);
            out.writeDouble(a.min);
            out.writeDouble(a.max);
            out.writeDouble(a.sum);
            if (a.type == ESGPU_AGG_EXTENDED_STATS) { out.writeDouble(a.sumsq); out.writeDouble(a.sigma); }
            break;
        case ESGPU_AGG_AVG:  // InternalAvg.doWriteTo (:102-106)
            writeFormatter(a, out);
            out.writeDouble(a.sum);
            out.writeVLong(a.count);
            break;
        case ESGPU_AGG_CARDINALITY:  // InternalCardinality.doWriteTo (:92-100), HyperLogLogPlusPlus.writeTo(0, out)
            writeFormatter(a, out);
            out.writeBoolean(a.hll != nullptr);
            if (a.hll) {
                const HLLPP& h = *a.hll;
                out.writeVInt(h.p);
                if (!h.algo(0)) {
                    out.writeBoolean(false);
                    const std::vector<int> v = h.hs_values(0);
                    out.writeVLong((int64_t)v.size());
                    for (int e : v) out.writeInt(e);
                } else {
                    out.writeBoolean(true);
                    for (int i = 0; i < h.m; ++i) out.writeByte(h.runLens[(size_t)i]);
                }
            }
            break;
        case ESGPU_AGG_FILTER:  // InternalSingleBucketAggregation.doWriteTo (:124-127)
            out.writeVLong(a.count);
            writeAggregations(a.subs, out);
            break;
    }
}

static void writeAggregations(const InternalList& aggs, StreamOutput& out) {  // InternalAggregations.writeTo
    out.writeVInt((int32_t)aggs.size());
    for (const InternalPtr& a : aggs) {
        out.writeBytes(streamType(a->type));
        writeAggregation(*a, out);
    }
}

static int g_emit_streams = 0;

// ------------------------------------------------------------------------------------------------------------
// Driver: AggregationPhase.preProcess -> QueryPhase collection loop -> postCollection -> buildAggregation(0)
// (A/AggregationPhase.java:69-168; C/search/query/QueryPhase.java:254-258,312-314) and the coordinator reduce
// (C/search/controller/SearchPhaseController.java:401-411).
// ------------------------------------------------------------------------------------------------------------
static std::vector<std::unique_ptr<Factory>> build_factories(const esgpu_agg_spec* specs, int n, std::vector<Factory*>& top,
                                                             const esgpu_filter* flt, int nf) {
    std::vector<std::unique_ptr<Factory>> owned;
    std::vector<Factory*> all(n, nullptr);
    for (int i = 0; i < n; ++i) {
        std::unique_ptr<Factory> f(new Factory());
        f->spec = specs[i];
        f->name = specs[i].name ? specs[i].name : "";
        f->field = specs[i].field ? specs[i].field : "";
        all[i] = f.get();
        if (specs[i].parent < 0) { top.push_back(f.get()); owned.push_back(std::move(f)); }
        else {
            if (specs[i].parent >= i) throw std::invalid_argument("parent must precede child");
            f->parent = all[specs[i].parent];
            all[specs[i].parent]->children.push_back(std::move(f));
        }
    }
    // filter aggregations own the clauses whose owner names them (esgpu_filter.owner = spec index + 1)
    for (int k = 0; k < nf; ++k) {
        const int o = flt[k].owner - 1;
        if (o < 0) continue;
        if (o >= n || all[o]->spec.type != ESGPU_AGG_FILTER) throw std::invalid_argument("filter clause owner is not a filter aggregation");
        all[o]->clauses.push_back(flt[k]);
    }
    // cardinality precision: CardinalityAggregatorFactory.precision / defaultPrecision (:43-77)
    for (int i = 0; i < n; ++i) {
        Factory* f = all[i];
        if (f->spec.type != ESGPU_AGG_CARDINALITY) continue;
        if (f->spec.precision_threshold >= 0) f->precision = precision_from_threshold(f->spec.precision_threshold);
        else {
            int p = 14;
            for (const Factory* q = f->parent; q; q = q->parent) if (q->is_bucket()) p -= 5;
            f->precision = std::max(p, 4);
        }
    }
    return owned;
}

static bool doc_matches(const Segment& seg, uint32_t doc, const esgpu_filter* flt, int nf, const uint64_t* accept) {
    if (accept && !((accept[doc >> 6] >> (doc & 63)) & 1)) return false;
    for (int k = 0; k < nf; ++k) {
        const Column* c = seg.col(flt[k].field);
        if (!c) return false;  // unmapped field matches nothing
        const int n = c->count(doc);
        bool any = false;
        for (int i = 0; i < n && !any; ++i) {
            if (flt[k].type == ESGPU_FILTER_TERM) {
                any = c->d->type == ESGPU_COL_ORD_U32 ? (int64_t)c->ord_at(doc, i) == flt[k].term : c->long_at(doc, i) == flt[k].term;
            } else if (c->d->type == ESGPU_COL_ORD_U32) {  // TermRangeQuery: BytesRef (unsigned byte) order
                const uint32_t o = c->ord_at(doc, i);
                if (o == 0xFFFFFFFFu) continue;
                const std::string t = c->term(o);
                const std::string lo((const char*)flt[k].lo_term, flt[k].lo_term ? (size_t)flt[k].lo_term_len : 0);
                const std::string hi((const char*)flt[k].hi_term, flt[k].hi_term ? (size_t)flt[k].hi_term_len : 0);
                const bool lo_ok = !flt[k].has_lower || (flt[k].include_lower ? term_compare(t, lo) >= 0 : term_compare(t, lo) > 0);
                const bool hi_ok = !flt[k].has_upper || (flt[k].include_upper ? term_compare(t, hi) <= 0 : term_compare(t, hi) < 0);
                any = lo_ok && hi_ok;
            } else if (c->d->type == ESGPU_COL_F64) {
                const double v = c->double_at(doc, i);
                bool lo = !flt[k].has_lower || (flt[k].include_lower ? v >= flt[k].lo_d : v > flt[k].lo_d);
                bool hi = !flt[k].has_upper || (flt[k].include_upper ? v <= flt[k].hi_d : v < flt[k].hi_d);
                any = lo && hi;
            } else {
                const int64_t v = c->long_at(doc, i);
                bool lo = !flt[k].has_lower || (flt[k].include_lower ? v >= flt[k].lo_i : v > flt[k].lo_i);
                bool hi = !flt[k].has_upper || (flt[k].include_upper ? v <= flt[k].hi_i : v < flt[k].hi_i);
                any = lo && hi;
            }
        }
        if (!any) return false;
    }
    return true;
}

}  // namespace oracle

// ------------------------------------------------------------------------------------------------------------
// C API (loaded with ctypes by tests/ and bench.py only)
// ------------------------------------------------------------------------------------------------------------
extern "C" {

typedef struct oracle_shard {
    const esgpu_column_desc* cols;
    int32_t ncols;
    uint32_t max_doc;
    const uint64_t* accept_bits;
} oracle_shard;

static thread_local std::string g_oracle_err;

const char* oracle_last_error(void) { return g_oracle_err.c_str(); }

/* Runs the request over every shard (one segment per shard), returns JSON
 * {"shards":[{aggs of shard 0}, ...], "reduced":{aggs}}.  Free with oracle_free. */
int oracle_run(const oracle_shard* shards, int32_t nshards, const esgpu_agg_spec* specs, int32_t nspecs,
               const esgpu_filter* filters, int32_t nfilters, char** json_out, double* collect_seconds) {
    using namespace oracle;
    try {
        std::vector<InternalList> shard_results;
        double secs = 0;
        for (int s = 0; s < nshards; ++s) {
            Segment seg;
            seg.max_doc = shards[s].max_doc;
            for (int c = 0; c < shards[s].ncols; ++c) seg.cols[shards[s].cols[c].name].d = &shards[s].cols[c];
            std::vector<Factory*> top;
            auto owned = build_factories(specs, nspecs, top, filters, nfilters);
            std::vector<esgpu_filter> query;  // bool.filter clauses (owner 0); the rest belong to filter aggregations
            for (int k = 0; k < nfilters; ++k) if (filters[k].owner == 0) query.push_back(filters[k]);
            std::vector<std::unique_ptr<Aggregator>> aggs;
            for (Factory* f : top) aggs.push_back(f->create(true));
            struct timespec t0, t1;
            clock_gettime(CLOCK_MONOTONIC, &t0);
            for (auto& a : aggs) a->set_leaf(seg);
            for (uint32_t doc = 0; doc < seg.max_doc; ++doc) {
                if (!doc_matches(seg, doc, query.data(), (int)query.size(), shards[s].accept_bits)) continue;
                for (auto& a : aggs) a->collect(doc, 0);
            }
            for (auto& a : aggs) a->post_collection();
            InternalList res;
            for (auto& a : aggs) res.push_back(a->build(0));
            clock_gettime(CLOCK_MONOTONIC, &t1);
            secs += (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
            shard_results.push_back(std::move(res));
        }
        Json j;
        j.raw("{\"shards\":[");
        for (size_t s = 0; s < shard_results.size(); ++s) {
            if (s) j.raw(",");
            j.raw("{"); write_list(j, shard_results[s]); j.raw("}");
        }
        j.raw("],\"reduced\":{");
        if (!shard_results.empty()) write_list(j, reduce_list(shard_results));
        j.raw("}");
        if (g_emit_streams) {  // per shard, hex of InternalAggregations.writeTo
            j.raw(",\"streams\":[");
            for (size_t s = 0; s < shard_results.size(); ++s) {
                StreamOutput out;
                writeAggregations(shard_results[s], out);
                static const char* hx = "0123456789abcdef";
                std::string h;
                h.reserve(out.b.size() * 2);
                for (unsigned char c : out.b) { h.push_back(hx[c >> 4]); h.push_back(hx[c & 15]); }
                if (s) j.raw(",");
                j.raw("\""); j.raw(h.c_str()); j.raw("\"");
            }
            j.raw("]");
        }
        j.raw("}");
        *json_out = strdup(j.s.c_str());
        if (collect_seconds) *collect_seconds = secs;
        return 0;
    } catch (const std::exception& e) {
        g_oracle_err = e.what();
        return 1;
    }
}

void oracle_free(char* p) { free(p); }
/* 1: oracle_run's JSON also carries "streams": per shard, the hex of InternalAggregations.writeTo */
void oracle_set_emit_streams(int32_t on) { oracle::g_emit_streams = on; }
/* 1: stats / extended_stats / avg results also carry "_exact": their values recomputed from the exact sums that the
   reference's doc-order double additions approximate (double-double shadow accumulators) */
void oracle_set_exact_shadow(int32_t on) { oracle::g_exact_shadow = on != 0; }

/* known-answer helpers */
void oracle_murmur3_128(const uint8_t* key, int32_t len, int64_t seed, uint64_t* h1, uint64_t* h2) {
    oracle::murmur3_128(key, len, seed, h1, h2);
}
uint64_t oracle_mix64(uint64_t v) { return oracle::mix64(v); }
int32_t oracle_precision_from_threshold(int64_t c) { return oracle::precision_from_threshold(c); }
int32_t oracle_encode_hash(uint64_t h, int32_t p) { return oracle::encode_hash(h, p); }
int32_t oracle_decode_run_len(int32_t e, int32_t p) { return oracle::decode_run_len(e, p); }
int32_t oracle_decode_index(int32_t e, int32_t p) { return oracle::decode_index(e, p); }
int64_t oracle_index(uint64_t h, int32_t p) { return oracle::hll_index(h, p); }
int32_t oracle_run_len(uint64_t h, int32_t p) { return oracle::run_len(h, p); }

/* Rounding KATs: kind 0 histogram Interval, 1 date unit, 2 date interval; returns round(v) / next(v) / roundKey(v) */
/* Lucene StringHelper.murmurhash3_x86_32 (third-party, Lucene 5.4) over the UTF-16LE bytes of a Java string, as
 * Murmur3HashFunction.hash (cluster/routing/Murmur3HashFunction.java:31-41); pinned by Murmur3HashFunctionTests. */
int32_t oracle_routing_hash(const uint16_t* chars, int32_t n) {
    std::vector<uint8_t> b((size_t)n * 2);
    for (int32_t i = 0; i < n; ++i) { b[2 * i] = (uint8_t)chars[i]; b[2 * i + 1] = (uint8_t)(chars[i] >> 8); }
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h1 = 0;
    const int len = (int)b.size(), rounded = len & ~3;
    for (int i = 0; i < rounded; i += 4) {
        uint32_t k1 = (b[i] & 0xff) | ((b[i + 1] & 0xff) << 8) | ((b[i + 2] & 0xff) << 16) | ((uint32_t)b[i + 3] << 24);
        k1 *= c1; k1 = (k1 << 15) | (k1 >> 17); k1 *= c2;
        h1 ^= k1; h1 = (h1 << 13) | (h1 >> 19); h1 = h1 * 5 + 0xe6546b64u;
    }
    uint32_t k1 = 0;
    const int tail = len & 3;
    if (tail == 3) k1 = (uint32_t)(b[rounded + 2] & 0xff) << 16;
    if (tail >= 2) k1 |= (uint32_t)(b[rounded + 1] & 0xff) << 8;
    if (tail >= 1) {
        k1 |= (b[rounded] & 0xff);
        k1 *= c1; k1 = (k1 << 15) | (k1 >> 17); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint32_t)len;
    h1 ^= h1 >> 16; h1 *= 0x85ebca6bu; h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u; h1 ^= h1 >> 16;
    return (int32_t)h1;
}
/* OperationRouting.shardId (indices created on or after 2.0): MathUtils.mod(hash, numberOfShards) */
int32_t oracle_shard_id(int32_t hash, int32_t nshards) {
    int32_t r = hash % nshards;
    if (r < 0) r += nshards;
    return r;
}

int64_t oracle_rounding_tz(int32_t kind, int32_t unit, int64_t interval, int64_t offset, const int64_t* tz_starts,
                           const int64_t* tz_offs, int32_t tz_count, int32_t op, int64_t v) {
    oracle::Rounding r;
    r.kind = kind; r.unit = unit; r.interval = interval; r.offset = offset;
    if (tz_count > 0) {
        r.tz.starts.assign(tz_starts, tz_starts + tz_count);
        r.tz.offs.assign(tz_offs, tz_offs + tz_count);
    }
    if (op == 0) return r.round(v);
    if (op == 1) return r.next_rounding_value(v);
    return r.round_key(v);
}

int64_t oracle_rounding(int32_t kind, int32_t unit, int64_t interval, int64_t offset, int32_t op, int64_t v) {
    oracle::Rounding r;
    r.kind = kind; r.unit = unit; r.interval = interval; r.offset = offset;
    if (op == 0) return r.round(v);
    if (op == 1) return r.next_rounding_value(v);
    return r.round_key(v);
}

/* HLL++ driver for property tests: collect `n` hashes into bucket 0, return cardinality and mode. */
int64_t oracle_hll_collect(int32_t p, const uint64_t* hashes, int64_t n, int32_t* mode_out, uint64_t* fnv_out) {
    oracle::HLLPP h(p, 1);
    for (int64_t i = 0; i < n; ++i) h.collect(0, hashes[i]);
    if (mode_out) *mode_out = h.algo(0) ? 1 : 0;
    if (fnv_out) *fnv_out = h.algo(0) ? oracle::fnv1a(h.runLens.data(), (size_t)h.m) : 0;
    return h.cardinality(0);
}

}  // extern "C"
