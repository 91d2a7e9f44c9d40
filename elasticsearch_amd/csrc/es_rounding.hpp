// es_rounding.hpp — host-side roundings of histogram / date_histogram keys (common/rounding/*), with the
// joda-time 2.8.2 DateTimeZone arithmetic they call (third-party, not in /root/reference; restated from its
// published algorithm and pinned by TimeZoneRoundingTests' DST cases, tests/golden/kat.json "rounding_tz").
//
//   Rounding.Interval ............ common/rounding/Rounding.java:92-118      (histogram; kind KIND_INTERVAL)
//   TimeZoneRounding.TimeUnitRounding       TimeZoneRounding.java:101-160    (calendar units; KIND_UNIT)
//   TimeZoneRounding.TimeIntervalRounding   TimeZoneRounding.java:162-217    (fixed intervals; KIND_TIME_INTERVAL)
//   Rounding.OffsetRounding ..... Rounding.java:205-236                      (offset wrapper)
//   DateTimeUnit fields ......... common/rounding/DateTimeUnit.java:36-43   (ISOChronology UTC roundFloor / add)
//
// The GPU never evaluates a time zone: an affine rounding (numeric histogram, or a unit / interval in UTC or a
// fixed-offset zone) is evaluated in the kernel as floor((v - offset) / interval); every other rounding (calendar
// months / quarters / years, DST zones) is turned here into a table of bucket start instants over the segment's value
// range (key_table), and the kernel finds a value's bucket in that table.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "../../include/esgpu.h"

namespace esgpu {

// ---- proleptic Gregorian calendar (joda ISOChronology) ----
inline int64_t r_floor_div(int64_t a, int64_t b) {
    const int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}
inline int64_t r_days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
inline void r_civil_from_days(int64_t z, int64_t* y, int* m, int* d) {
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
constexpr int64_t kMsDay = 86400000LL;

// DateTimeZone as an offset history: offs[i] (ms) applies from UTC instant starts[i] on; starts[0] == INT64_MIN.
// A fixed zone has one entry.  The JNI shim fills it from the request's joda zone (getOffset / nextTransition over the
// index's time range), the Python mirror from the IANA database (elasticsearch_amd.aggs.tz_history).
struct TimeZone {
    std::vector<int64_t> starts{INT64_MIN};
    std::vector<int64_t> offs{0};

    bool fixed() const { return starts.size() <= 1; }
    int64_t offset(int64_t t) const {  // getOffset(instant)
        if (starts.size() == 1) return offs[0];
        const size_t i = (size_t)(std::upper_bound(starts.begin(), starts.end(), t) - starts.begin());
        return offs[i ? i - 1 : 0];
    }
    int64_t next_transition(int64_t t) const {  // nextTransition(instant): the instant itself when there is none
        auto it = std::upper_bound(starts.begin(), starts.end(), t);
        return it == starts.end() ? t : *it;
    }
    int64_t utc_to_local(int64_t t) const { return t + offset(t); }  // convertUTCToLocal
    int64_t local_to_utc(int64_t local) const {  // convertLocalToUTC(instantLocal, strict = false)
        if (starts.size() == 1) return local - offs[0];
        const int64_t offset_local = offset(local);
        int64_t off = offset(local - offset_local);
        if (offset_local != off && offset_local < 0) {  // Western hemisphere: is instantLocal in a DST gap?
            int64_t next_local = next_transition(local - offset_local);
            if (next_local == local - offset_local) next_local = INT64_MAX;
            int64_t next_adjusted = next_transition(local - off);
            if (next_adjusted == local - off) next_adjusted = INT64_MAX;
            if (next_local != next_adjusted) off = offset_local;  // in the gap: keep the pre-cutover offset
        }
        return local - off;
    }
    int64_t local_to_utc(int64_t local, int64_t original) const {  // convertLocalToUTC(local, false, originalUTC)
        const int64_t off_orig = offset(original);
        const int64_t utc = local - off_orig;
        if (offset(utc) == off_orig) return utc;
        return local_to_utc(local);
    }
};

struct Rounding {
    enum { KIND_INTERVAL = 0, KIND_UNIT = 1, KIND_TIME_INTERVAL = 2 };
    int kind = KIND_INTERVAL;
    int unit = ESGPU_UNIT_NONE;
    int64_t interval = 1;
    int64_t offset = 0;  // OffsetRounding (a fixed zone offset z is folded in as -z by the caller)
    TimeZone tz;

    static Rounding from_spec(const esgpu_agg_spec& s) {
        Rounding r;
        if (s.type == ESGPU_AGG_HISTOGRAM) {
            r.kind = KIND_INTERVAL;
            r.interval = s.interval;
        } else if (s.date_unit != ESGPU_UNIT_NONE) {
            r.kind = KIND_UNIT;
            r.unit = s.date_unit;
            if (r.unit < ESGPU_UNIT_WEEK || r.unit > ESGPU_UNIT_SECOND) throw std::invalid_argument("unknown date unit");
        } else {
            r.kind = KIND_TIME_INTERVAL;
            r.interval = s.interval;
        }
        if (r.kind != KIND_UNIT && r.interval < 1) throw std::invalid_argument("[interval] must be 1 or greater");
        r.offset = s.offset;
        if (s.type != ESGPU_AGG_HISTOGRAM && s.tz_count > 0) {
            if (!s.tz_starts || !s.tz_offsets_ms) throw std::invalid_argument("time zone table without arrays");
            r.tz.starts.assign(s.tz_starts, s.tz_starts + s.tz_count);
            r.tz.offs.assign(s.tz_offsets_ms, s.tz_offsets_ms + s.tz_count);
            r.tz.starts[0] = INT64_MIN;
            for (int i = 1; i < s.tz_count; ++i)
                if (r.tz.starts[i] <= r.tz.starts[i - 1]) throw std::invalid_argument("time zone transitions not ascending");
            if (r.tz.fixed()) {  // a fixed zone is OffsetRounding(-z) of the UTC rounding
                r.offset -= r.tz.offs[0];
                r.tz = TimeZone();
            }
        }
        return r;
    }

    // floor / step of the unit's ISOChronology UTC field (DateTimeField.roundFloor, DurationField.add(t, 1))
    int64_t unit_floor(int64_t t) const {
        switch (unit) {
            case ESGPU_UNIT_SECOND: return r_floor_div(t, 1000) * 1000;
            case ESGPU_UNIT_MINUTE: return r_floor_div(t, 60000) * 60000;
            case ESGPU_UNIT_HOUR: return r_floor_div(t, 3600000) * 3600000;
            case ESGPU_UNIT_DAY: return r_floor_div(t, kMsDay) * kMsDay;
            case ESGPU_UNIT_WEEK: {  // weekOfWeekyear: Monday 00:00 (1970-01-01 was a Thursday)
                const int64_t days = r_floor_div(t, kMsDay);
                return (days - ((days + 3) % 7 + 7) % 7) * kMsDay;
            }
            default: {
                int64_t y; int m, d;
                r_civil_from_days(r_floor_div(t, kMsDay), &y, &m, &d);
                if (unit == ESGPU_UNIT_MONTH) return r_days_from_civil(y, m, 1) * kMsDay;
                if (unit == ESGPU_UNIT_QUARTER) return r_days_from_civil(y, ((m - 1) / 3) * 3 + 1, 1) * kMsDay;
                return r_days_from_civil(y, 1, 1) * kMsDay;  // YEAR_OF_CENTURY
            }
        }
    }
    int64_t unit_add(int64_t t) const {
        switch (unit) {
            case ESGPU_UNIT_SECOND: return t + 1000;
            case ESGPU_UNIT_MINUTE: return t + 60000;
            case ESGPU_UNIT_HOUR: return t + 3600000;
            case ESGPU_UNIT_DAY: return t + kMsDay;
            case ESGPU_UNIT_WEEK: return t + 7 * kMsDay;
            default: {  // months: day-of-month clamped to the target month's length (ISO month arithmetic)
                const int64_t days = r_floor_div(t, kMsDay);
                const int64_t rem = t - days * kMsDay;
                int64_t y; int m, d;
                r_civil_from_days(days, &y, &m, &d);
                const int add = unit == ESGPU_UNIT_MONTH ? 1 : unit == ESGPU_UNIT_QUARTER ? 3 : 12;
                const int64_t mm = (int64_t)(m - 1) + add;
                y += r_floor_div(mm, 12);
                m = (int)(mm - r_floor_div(mm, 12) * 12) + 1;
                static const int md[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
                const int dim = md[m - 1] + ((m == 2 && ((y % 4 == 0 && y % 100 != 0) || y % 400 == 0)) ? 1 : 0);
                if (d > dim) d = dim;
                return r_days_from_civil(y, m, d) * kMsDay + rem;
            }
        }
    }

    // ---- the inner rounding (without the offset wrapper) ----
    int64_t inner_round_key(int64_t t) const {
        switch (kind) {
            case KIND_INTERVAL: return r_floor_div(t, interval);
            case KIND_UNIT: {  // TimeUnitRounding.roundKey
                const int64_t local = tz.utc_to_local(t);
                return tz.local_to_utc(unit_floor(local), t);
            }
            default: {  // TimeIntervalRounding.roundKey
                const int64_t local = tz.utc_to_local(t);
                return tz.local_to_utc(r_floor_div(local, interval) * interval);
            }
        }
    }
    int64_t inner_value_for_key(int64_t k) const { return kind == KIND_INTERVAL ? k * interval : k; }
    int64_t inner_next(int64_t t) const {
        switch (kind) {
            case KIND_INTERVAL: return t + interval;
            case KIND_UNIT: return tz.local_to_utc(unit_add(tz.utc_to_local(t)));
            default: return tz.local_to_utc(tz.utc_to_local(t) + interval);
        }
    }
    // ---- OffsetRounding wrapper ----
    int64_t round_key(int64_t v) const { return inner_round_key(v - offset); }
    int64_t value_for_key(int64_t k) const { return offset + inner_value_for_key(k); }
    int64_t next_rounding_value(int64_t v) const { return inner_next(v - offset) + offset; }
    int64_t round(int64_t v) const { return value_for_key(round_key(v)); }

    // An affine rounding is evaluated on the GPU as key = floor((v - aff_offset) / aff_interval) * aff_interval + aff_offset.
    bool affine(int64_t* aff_interval, int64_t* aff_offset) const {
        if (kind == KIND_INTERVAL || (tz.fixed() && kind == KIND_TIME_INTERVAL)) {
            *aff_interval = interval;
            *aff_offset = offset;
            return true;
        }
        if (!tz.fixed()) return false;
        switch (unit) {
            case ESGPU_UNIT_SECOND: *aff_interval = 1000; break;
            case ESGPU_UNIT_MINUTE: *aff_interval = 60000; break;
            case ESGPU_UNIT_HOUR: *aff_interval = 3600000; break;
            case ESGPU_UNIT_DAY: *aff_interval = kMsDay; break;
            case ESGPU_UNIT_WEEK: *aff_interval = 7 * kMsDay; *aff_offset = offset - 3 * kMsDay; return true;  // Monday
            default: return false;  // month / quarter / year
        }
        *aff_offset = offset;
        return true;
    }

    // Bucket table of a non-affine rounding over the values [lo, hi].  round_key is a step function whose steps can only
    // sit at a zone transition or at a local-time unit / interval boundary, so walking those points visits every step:
    //   starts[j]  first value of step j (ascending)          keys[b]  distinct bucket keys, ascending
    //   slot[j]    bucket of step j (empty when step j == bucket j, i.e. the keys rise with the value)
    // TimeIntervalRounding maps the repeated local hour of a DST fall-back to its first occurrence
    // (convertLocalToUTC without the original instant), so there a later step can return to an earlier bucket.
    // Returns false when the table would exceed max_steps.
    bool key_table(int64_t lo, int64_t hi, size_t max_steps, std::vector<int64_t>& starts, std::vector<int64_t>& keys,
                   std::vector<uint32_t>& slot) const {
        starts.clear();
        keys.clear();
        slot.clear();
        if (lo > hi) return true;
        std::vector<int64_t> step_key;
        bool monotone = true;
        int64_t u = lo - offset;
        const int64_t uhi = hi - offset;
        for (;;) {
            const int64_t k = inner_round_key(u) + offset;
            if (step_key.empty() || k != step_key.back()) {
                if (!step_key.empty() && k < step_key.back()) monotone = false;
                if (step_key.size() >= max_steps) return false;
                starts.push_back(u + offset);
                step_key.push_back(k);
            }
            const int64_t o = tz.offset(u);
            const int64_t local = u + o;
            const int64_t fl = kind == KIND_UNIT ? unit_floor(local) : r_floor_div(local, interval) * interval;
            int64_t cand = (kind == KIND_UNIT ? unit_add(fl) : fl + interval) - o;
            const int64_t tn = tz.next_transition(u);
            if (tn > u && tn < cand) cand = tn;
            if (cand <= u) return false;
            if (cand > uhi) break;
            u = cand;
        }
        if (monotone) {
            keys = std::move(step_key);
            return true;
        }
        keys = step_key;
        std::sort(keys.begin(), keys.end());
        keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
        slot.resize(step_key.size());
        for (size_t j = 0; j < step_key.size(); ++j)
            slot[j] = (uint32_t)(std::lower_bound(keys.begin(), keys.end(), step_key[j]) - keys.begin());
        return true;
    }
};

}  // namespace esgpu
