// esgpu_results.cpp — InternalAggregation reduce / JSON / stream formats for libesgpu.so (host C++).
//
// The reduce follows the reference's doReduce implementations (paths relative to
// /root/reference/core/src/main/java/org/elasticsearch/search/aggregations/):
//   InternalTerms.doReduce + Bucket.reduce ..... bucket/terms/InternalTerms.java:91-108,165-246
//   InternalHistogram.doReduce/addEmptyBuckets . bucket/histogram/InternalHistogram.java:338-476
//   InternalStats/ExtendedStats/Avg.doReduce .... metrics/stats/InternalStats.java:153-166,
//                                                 metrics/stats/extended/InternalExtendedStats.java:147-156,
//                                                 metrics/avg/InternalAvg.java:84-92
//   InternalCardinality.doReduce / HLL++ merge .. metrics/cardinality/InternalCardinality.java:103-126,
//                                                 metrics/cardinality/HyperLogLogPlusPlus.java:201-307
#include "esgpu_results.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <unordered_map>

namespace esgpu {

#include "hllpp_tables.inc"

// ------------------------------------------------------------------------------------------------------------
// Java double semantics
// ------------------------------------------------------------------------------------------------------------
static inline double jmin(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && std::signbit(b)) return b;
    return a <= b ? a : b;
}
static inline double jmax(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && std::signbit(a)) return b;
    return a >= b ? a : b;
}
static inline int64_t jround(double a) {
    if (a != a) return 0;
    if (a >= 9.2233720368547758e18) return INT64_MAX;
    if (a <= -9.2233720368547758e18) return INT64_MIN;
    const double f = std::floor(a);
    return (int64_t)f + ((a - f) >= 0.5 ? 1 : 0);
}
static inline int64_t fdiv(int64_t a, int64_t b) { return a < 0 ? (a - b + 1) / b : a / b; }

// ------------------------------------------------------------------------------------------------------------
// calendar (joda ISOChronology UTC) for EmptyBucketInfo.rounding.nextRoundingValue
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
static const int64_t kDay = 86400000LL;

int64_t rounding_next(int32_t type, int32_t unit, int64_t interval, int64_t offset, int64_t v) {
    if (type == ESGPU_AGG_HISTOGRAM || unit == ESGPU_UNIT_NONE) return v + interval;  // Interval / TimeIntervalRounding
    const int64_t t = v - offset;  // OffsetRounding.nextRoundingValue
    int64_t r;
    switch (unit) {
        case ESGPU_UNIT_SECOND: r = t + 1000; break;
        case ESGPU_UNIT_MINUTE: r = t + 60000; break;
        case ESGPU_UNIT_HOUR: r = t + 3600000; break;
        case ESGPU_UNIT_DAY: r = t + kDay; break;
        case ESGPU_UNIT_WEEK: r = t + 7 * kDay; break;
        default: {
            const int64_t days = fdiv(t, kDay);
            const int64_t rem = t - days * kDay;
            int64_t y; int m, d;
            civil_from_days(days, &y, &m, &d);
            const int add = unit == ESGPU_UNIT_MONTH ? 1 : unit == ESGPU_UNIT_QUARTER ? 3 : 12;
            const int64_t mm = (int64_t)(m - 1) + add;
            y += mm / 12;
            m = (int)(mm % 12) + 1;
            static const int md[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
            const int dim = md[m - 1] + ((m == 2 && ((y % 4 == 0 && y % 100 != 0) || y % 400 == 0)) ? 1 : 0);
            if (d > dim) d = dim;
            r = days_from_civil(y, m, d) * kDay + rem;
        }
    }
    return r + offset;
}

// ------------------------------------------------------------------------------------------------------------
// HyperLogLog++ (A/metrics/cardinality/HyperLogLogPlusPlus.java)
// ------------------------------------------------------------------------------------------------------------
static const int kP2 = 25;

int hll_precision_from_threshold(int64_t count) {  // :68-74 (float division as in Java: count / 0.75f)
    const int64_t entries = (int64_t)std::ceil((double)((float)count / 0.75f));
    const uint64_t v = (uint64_t)(entries * 4);
    int bits = v == 0 ? 1 : 64 - __builtin_clzll(v);  // PackedInts.bitsRequired
    if (bits < 4) bits = 4;
    if (bits > 18) bits = 18;
    return bits;
}

static int64_t linear_counting(int64_t m, int64_t v) { return jround((double)m * std::log((double)m / (double)v)); }

static double estimate_bias(int p, double e) {  // :378-405
    const double* raw = HLLPP_RAW[p - 4];
    const double* bias = HLLPP_BIAS[p - 4];
    const int n = HLLPP_TABLE_LEN[p - 4];
    double w6[6] = {0, 0, 0, 0, 0, 0};
    int index = n - 6;
    for (int i = 0; i < n; ++i) {
        const double w = 1.0 / std::fabs(raw[i] - e);
        const int j = i % 6;
        if (std::isinf(w)) return bias[i];
        if (w6[j] >= w) { index = i - 6; break; }
        w6[j] = w;
    }
    double ws = 0.0, bs = 0.0;
    for (int i = 0, j = index; i < 6; ++i, ++j) {
        bs += w6[i] * bias[j];
        ws += w6[i];
    }
    return bs / ws;
}

int64_t hll_cardinality(const RAgg& a) {  // :270-307
    if (!a.hll_present) return 0;
    const int p = a.precision;
    if (a.hll_mode == 0) return linear_counting(1LL << kP2, (1LL << kP2) - (int64_t)a.lc.size());
    const int m = 1 << p;
    const double alpha = p == 4 ? 0.673 : p == 5 ? 0.697 : 0.7213 / (1 + 1.079 / m);
    const double alphaMM = alpha * m * m;
    double inv = 0;
    int zeros = 0;
    for (int i = 0; i < m; ++i) {
        const int rl = a.registers[i];
        inv += 1. / (double)(1LL << rl);
        if (rl == 0) ++zeros;
    }
    const double e1 = alphaMM / inv;
    const double e2 = e1 <= 5 * m ? e1 - estimate_bias(p, e1) : e1;
    const int64_t h = zeros != 0 ? linear_counting(m, zeros) : jround(e2);
    if (h <= HLLPP_THRESHOLDS[p - 4]) return h;
    return jround(e2);
}

static uint32_t dec_run_len(uint32_t enc, int p) {
    if (enc & 1) return ((enc >> 1) & 0x3F) + (uint32_t)(kP2 - p);
    const uint32_t bits = enc << (31 + p - kP2);
    return 1u + (uint32_t)__builtin_clz(bits);
}
static uint32_t dec_index(uint32_t enc, int p) {
    const uint32_t idx = (enc & 1) ? (enc >> 7) : (enc >> 1);
    return idx >> (kP2 - p);
}
static void upgrade_to_hll(RAgg& a) {  // :309-322
    a.registers.assign((size_t)1 << a.precision, 0);
    for (uint32_t e : a.lc) {
        uint8_t& r = a.registers[dec_index(e, a.precision)];
        r = (uint8_t)std::max<uint32_t>(r, dec_run_len(e, a.precision));
    }
    a.lc.clear();
    a.hll_mode = 1;
}

void hll_merge(RAgg& into, const RAgg& other) {  // HyperLogLogPlusPlus.merge (:201-230)
    if (!other.hll_present) return;
    if (into.precision != other.precision) throw std::invalid_argument("cardinality precision mismatch");
    const int m = 1 << into.precision;
    const size_t threshold = (size_t)((float)(m / 4) * 0.75f);
    if (other.hll_mode == 0) {
        for (uint32_t e : other.lc) {
            if (into.hll_mode == 0) {
                auto it = std::lower_bound(into.lc.begin(), into.lc.end(), e);
                if (it == into.lc.end() || *it != e) {
                    into.lc.insert(it, e);
                    if (into.lc.size() > threshold) upgrade_to_hll(into);
                }
            } else {
                uint8_t& r = into.registers[dec_index(e, into.precision)];
                r = (uint8_t)std::max<uint32_t>(r, dec_run_len(e, into.precision));
            }
        }
    } else {
        if (into.hll_mode == 0) upgrade_to_hll(into);
        for (int i = 0; i < m; ++i) into.registers[i] = std::max(into.registers[i], other.registers[i]);
    }
}

// ------------------------------------------------------------------------------------------------------------
// reduce
// ------------------------------------------------------------------------------------------------------------
static int terms_cmp(int order, const RBucket& a, const RBucket& b) {
    auto keycmp = [&]() {
        const int c = std::memcmp(a.term.data(), b.term.data(), std::min(a.term.size(), b.term.size()));
        if (c != 0) return c < 0 ? -1 : 1;
        return a.term.size() < b.term.size() ? -1 : a.term.size() > b.term.size() ? 1 : 0;
    };
    switch (order) {
        case ESGPU_ORDER_COUNT_DESC: if (a.doc_count != b.doc_count) return a.doc_count > b.doc_count ? -1 : 1; return keycmp();
        case ESGPU_ORDER_COUNT_ASC: if (a.doc_count != b.doc_count) return a.doc_count < b.doc_count ? -1 : 1; return keycmp();
        case ESGPU_ORDER_TERM_DESC: return -keycmp();
        default: return keycmp();
    }
}

static RAgg reduce_one(const std::vector<const RAgg*>& aggs);

std::vector<RAgg> reduce_lists(const std::vector<const std::vector<RAgg>*>& lists) {
    std::vector<RAgg> out;
    if (lists.empty()) return out;
    const size_t n = lists[0]->size();
    for (size_t i = 0; i < n; ++i) {
        std::vector<const RAgg*> same;
        for (auto* l : lists) {
            if (l->size() != n) throw std::invalid_argument("shard results have different aggregation lists");
            same.push_back(&(*l)[i]);
        }
        out.push_back(reduce_one(same));
    }
    return out;
}

static RAgg reduce_one(const std::vector<const RAgg*>& aggs) {
    const RAgg& first = *aggs[0];
    RAgg r;  // header of the first aggregation (InternalX carries its request parameters); buckets rebuilt below
    r.type = first.type; r.order = first.order; r.name = first.name;
    r.doc_count_error = first.doc_count_error; r.other_doc_count = first.other_doc_count;
    r.required_size = first.required_size; r.shard_size = first.shard_size; r.min_doc_count = first.min_doc_count;
    r.show_err = first.show_err; r.keyed = first.keyed;
    r.has_empty_info = first.has_empty_info; r.date_unit = first.date_unit; r.interval = first.interval;
    r.offset = first.offset; r.has_bmin = first.has_bmin; r.has_bmax = first.has_bmax; r.bmin = first.bmin; r.bmax = first.bmax;
    r.empty_subs = first.empty_subs;
    r.count = first.count; r.sum = first.sum; r.min = first.min; r.max = first.max; r.sumsq = first.sumsq;
    r.sigma = first.sigma;
    r.hll_present = first.hll_present; r.precision = first.precision; r.hll_mode = first.hll_mode;
    switch (first.type) {
        case ESGPU_AGG_TERMS: {
            int64_t sumErr = 0, other = 0;
            std::unordered_map<std::string, size_t> index;
            std::vector<std::vector<std::pair<const RBucket*, int64_t>>> groups;  // (bucket, its shard's error)
            for (const RAgg* t : aggs) {
                other += t->other_doc_count;
                int64_t thisErr;
                if ((int64_t)t->buckets.size() < first.shard_size || first.order == ESGPU_ORDER_TERM_ASC ||
                    first.order == ESGPU_ORDER_TERM_DESC) thisErr = 0;
                else if (first.order == ESGPU_ORDER_COUNT_DESC) thisErr = t->buckets.back().doc_count;
                else thisErr = -1;
                if (sumErr != -1) sumErr = thisErr == -1 ? -1 : sumErr + thisErr;
                for (const RBucket& b : t->buckets) {
                    auto it = index.find(b.term);
                    if (it == index.end()) { index.emplace(b.term, groups.size()); groups.push_back({}); it = index.find(b.term); }
                    groups[it->second].push_back({&b, thisErr});
                }
            }
            std::vector<RBucket> cands;
            for (auto& g : groups) {
                RBucket nb;
                nb.term = g[0].first->term;
                nb.key = g[0].first->key;
                int64_t err = 0;
                std::vector<const std::vector<RAgg>*> subl;
                for (auto& pr : g) {
                    nb.doc_count += pr.first->doc_count;
                    if (err != -1) err = pr.second == -1 ? -1 : err + pr.second;
                    subl.push_back(&pr.first->subs);
                }
                nb.subs = reduce_lists(subl);
                nb.doc_count_error = err;
                if (nb.doc_count_error != -1) nb.doc_count_error = sumErr == -1 ? -1 : sumErr - nb.doc_count_error;
                if (nb.doc_count >= first.min_doc_count) cands.push_back(std::move(nb));
            }
            const size_t size = std::min<size_t>((size_t)std::max(first.required_size, 0), groups.size());
            std::stable_sort(cands.begin(), cands.end(),
                             [&](const RBucket& a, const RBucket& b) { return terms_cmp(first.order, a, b) < 0; });
            for (size_t i = size; i < cands.size(); ++i) other += cands[i].doc_count;
            if (cands.size() > size) cands.resize(size);
            r.buckets = std::move(cands);
            r.doc_count_error = sumErr == -1 ? -1 : (aggs.size() == 1 ? 0 : sumErr);
            r.other_doc_count = other;
            return r;
        }
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM: {
            std::map<int64_t, std::vector<const RBucket*>> byKey;
            for (const RAgg* a : aggs) for (const RBucket& b : a->buckets) byKey[b.key].push_back(&b);
            std::vector<RBucket> list;
            for (auto& kv : byKey) {
                RBucket nb;
                nb.key = kv.first;
                std::vector<const std::vector<RAgg>*> subl;
                for (const RBucket* b : kv.second) { nb.doc_count += b->doc_count; subl.push_back(&b->subs); }
                nb.subs = reduce_lists(subl);
                if (nb.doc_count >= first.min_doc_count) list.push_back(std::move(nb));
            }
            if (first.min_doc_count == 0 && first.has_empty_info) {
                auto next = [&](int64_t k) { return rounding_next(first.type, first.date_unit, first.interval, first.offset, k); };
                auto empty = [&](int64_t k) { RBucket e; e.key = k; e.subs = first.empty_subs; return e; };
                std::vector<RBucket> out;
                if (list.empty()) {
                    if (first.has_bmin && first.has_bmax)
                        for (int64_t k = first.bmin; k <= first.bmax; k = next(k)) out.push_back(empty(k));
                } else {
                    if (first.has_bmin)
                        for (int64_t k = first.bmin; k < list[0].key; k = next(k)) out.push_back(empty(k));
                    for (size_t i = 0; i < list.size(); ++i) {
                        if (i > 0) for (int64_t k = next(list[i - 1].key); k < list[i].key; k = next(k)) out.push_back(empty(k));
                        out.push_back(list[i]);
                    }
                    if (first.has_bmax && first.bmax > list.back().key)
                        for (int64_t k = next(list.back().key); k <= first.bmax; k = next(k)) out.push_back(empty(k));
                }
                list = std::move(out);
            }
            if (first.order == ESGPU_ORDER_KEY_DESC) std::reverse(list.begin(), list.end());
            else if (first.order == ESGPU_ORDER_HCOUNT_ASC || first.order == ESGPU_ORDER_HCOUNT_DESC) {
                const bool asc = first.order == ESGPU_ORDER_HCOUNT_ASC;
                std::stable_sort(list.begin(), list.end(), [&](const RBucket& a, const RBucket& b) {
                    if (a.doc_count != b.doc_count) return asc ? a.doc_count < b.doc_count : a.doc_count > b.doc_count;
                    return a.key < b.key;
                });
            }
            r.buckets = std::move(list);
            return r;
        }
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS:
        case ESGPU_AGG_AVG: {
            int64_t count = 0;
            double mn = INFINITY, mx = -INFINITY, sum = 0, sq = 0;
            for (const RAgg* a : aggs) {
                count += a->count;
                mn = jmin(mn, a->min);
                mx = jmax(mx, a->max);
                sum += a->sum;
                sq += a->sumsq;
            }
            r.count = count; r.min = mn; r.max = mx; r.sum = sum; r.sumsq = sq;
            return r;
        }
        case ESGPU_AGG_CARDINALITY: {
            bool any = false;
            for (const RAgg* a : aggs) {
                if (!a->hll_present) continue;
                if (!any) {
                    any = true;
                    r.hll_present = true;
                    r.precision = a->precision;
                    r.hll_mode = 0;
                    r.lc.clear();
                    r.registers.clear();
                }
                hll_merge(r, *a);
            }
            if (!any) return first;
            return r;
        }
    }
    throw std::invalid_argument("reduce: unknown aggregation type");
}

// ------------------------------------------------------------------------------------------------------------
// JSON
// ------------------------------------------------------------------------------------------------------------
namespace {
struct J {
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
    void key(const std::string& k) { str(k); s += ':'; }
    void opt(bool c, double v) { if (c) dbl(v); else raw("null"); }
};
std::string iso8601(int64_t ms) {
    const int64_t days = fdiv(ms, kDay);
    const int64_t rem = ms - days * kDay;
    int64_t y; int m, d;
    civil_from_days(days, &y, &m, &d);
    char b[64];
    snprintf(b, sizeof b, "%04lld-%02d-%02dT%02d:%02d:%02d.%03dZ", (long long)y, m, d, (int)(rem / 3600000),
             (int)(rem / 60000 % 60), (int)(rem / 1000 % 60), (int)(rem % 1000));
    return b;
}
uint64_t fnv1a(const uint8_t* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ULL; }
    return h;
}
void write_list(J& j, const std::vector<RAgg>& aggs);
void write_agg(J& j, const RAgg& a) {
    j.raw("{");
    switch (a.type) {
        case ESGPU_AGG_TERMS:
            j.key("doc_count_error_upper_bound"); j.i64(a.doc_count_error); j.raw(",");
            j.key("sum_other_doc_count"); j.i64(a.other_doc_count); j.raw(",");
            j.key("buckets"); j.raw("[");
            for (size_t i = 0; i < a.buckets.size(); ++i) {
                const RBucket& b = a.buckets[i];
                if (i) j.raw(",");
                j.raw("{"); j.key("key"); j.str(b.term); j.raw(",");
                j.key("doc_count"); j.i64(b.doc_count);
                if (a.show_err) { j.raw(","); j.key("doc_count_error_upper_bound"); j.i64(b.doc_count_error); }
                if (!b.subs.empty()) { j.raw(","); write_list(j, b.subs); }
                j.raw("}");
            }
            j.raw("]");
            break;
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM:
            j.key("buckets"); j.raw("[");
            for (size_t i = 0; i < a.buckets.size(); ++i) {
                const RBucket& b = a.buckets[i];
                if (i) j.raw(",");
                j.raw("{");
                if (a.type == ESGPU_AGG_DATE_HISTOGRAM) { j.key("key_as_string"); j.str(iso8601(b.key)); j.raw(","); }
                j.key("key"); j.i64(b.key); j.raw(",");
                j.key("doc_count"); j.i64(b.doc_count);
                if (!b.subs.empty()) { j.raw(","); write_list(j, b.subs); }
                j.raw("}");
            }
            j.raw("]");
            break;
        case ESGPU_AGG_AVG:
            j.key("value"); j.opt(a.count != 0, a.sum / (double)a.count);
            j.raw(","); j.key("_internal"); j.raw("{"); j.key("count"); j.i64(a.count); j.raw(",");
            j.key("sum"); j.dbl(a.sum); j.raw("}");
            break;
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS: {
            const bool c = a.count != 0;
            const double avg = a.sum / (double)a.count;
            j.key("count"); j.i64(a.count); j.raw(",");
            j.key("min"); j.opt(c, a.min); j.raw(",");
            j.key("max"); j.opt(c, a.max); j.raw(",");
            j.key("avg"); j.opt(c, avg); j.raw(",");
            j.key("sum"); j.opt(c, a.sum);
            if (a.type == ESGPU_AGG_EXTENDED_STATS) {
                const double var = (a.sumsq - ((a.sum * a.sum) / (double)a.count)) / (double)a.count;
                const double sd = std::sqrt(var);
                j.raw(","); j.key("sum_of_squares"); j.opt(c, a.sumsq);
                j.raw(","); j.key("variance"); j.opt(c, var);
                j.raw(","); j.key("std_deviation"); j.opt(c, sd);
                j.raw(","); j.key("std_deviation_bounds"); j.raw("{");
                j.key("upper"); j.opt(c, avg + (sd * a.sigma)); j.raw(",");
                j.key("lower"); j.opt(c, avg - (sd * a.sigma)); j.raw("}");
            }
            j.raw(","); j.key("_internal"); j.raw("{");
            j.key("count"); j.i64(a.count); j.raw(",");
            j.key("sum"); j.dbl(a.sum); j.raw(",");
            j.key("min"); j.dbl(a.min); j.raw(",");
            j.key("max"); j.dbl(a.max);
            if (a.type == ESGPU_AGG_EXTENDED_STATS) { j.raw(","); j.key("sum_of_squares"); j.dbl(a.sumsq); }
            j.raw("}");
            break;
        }
        case ESGPU_AGG_CARDINALITY: {
            j.key("value"); j.i64(hll_cardinality(a));
            j.raw(","); j.key("_internal"); j.raw("{");
            j.key("present"); j.i64(a.hll_present ? 1 : 0);
            if (a.hll_present) {
                char b[32];
                j.raw(","); j.key("precision"); j.i64(a.precision);
                j.raw(","); j.key("mode"); j.str(a.hll_mode ? "hll" : "lc");
                if (a.hll_mode) {
                    snprintf(b, sizeof b, "%016llx", (unsigned long long)fnv1a(a.registers.data(), a.registers.size()));
                    j.raw(","); j.key("registers_fnv1a64"); j.str(b);
                } else {
                    j.raw(","); j.key("lc_size"); j.i64((int64_t)a.lc.size());
                    snprintf(b, sizeof b, "%016llx", (unsigned long long)fnv1a((const uint8_t*)a.lc.data(), a.lc.size() * 4));
                    j.raw(","); j.key("lc_fnv1a64"); j.str(b);
                }
            }
            j.raw("}");
            break;
        }
    }
    j.raw("}");
}
void write_list(J& j, const std::vector<RAgg>& aggs) {
    for (size_t i = 0; i < aggs.size(); ++i) {
        if (i) j.raw(",");
        j.key(aggs[i].name);
        write_agg(j, aggs[i]);
    }
}
}  // namespace

std::string to_json(const std::vector<RAgg>& aggs) {
    J j;
    j.raw("{");
    write_list(j, aggs);
    j.raw("}");
    return j.s;
}

// ------------------------------------------------------------------------------------------------------------
// stream format (AggregationStreams analogue): little-endian, length-prefixed, versioned
// ------------------------------------------------------------------------------------------------------------
namespace {
struct W {
    std::string& o;
    template <class T> void pod(const T& v) { o.append((const char*)&v, sizeof v); }
    void str(const std::string& s) { pod<uint32_t>((uint32_t)s.size()); o.append(s); }
};
struct R {
    const uint8_t* p;
    size_t n, i = 0;
    template <class T> T pod() {
        if (i + sizeof(T) > n) throw std::runtime_error("truncated stream");
        T v;
        std::memcpy(&v, p + i, sizeof v);
        i += sizeof v;
        return v;
    }
    std::string str() {
        const uint32_t len = pod<uint32_t>();
        if (i + len > n) throw std::runtime_error("truncated stream");
        std::string s((const char*)p + i, len);
        i += len;
        return s;
    }
};
void w_list(W& w, const std::vector<RAgg>& l);
void w_agg(W& w, const RAgg& a) {
    w.pod(a.type); w.pod(a.order); w.str(a.name);
    w.pod(a.doc_count_error); w.pod(a.other_doc_count); w.pod(a.required_size); w.pod(a.shard_size);
    w.pod(a.min_doc_count); w.pod(a.show_err); w.pod(a.keyed);
    w.pod<uint8_t>(a.has_empty_info); w.pod(a.date_unit); w.pod(a.interval); w.pod(a.offset);
    w.pod<uint8_t>(a.has_bmin); w.pod<uint8_t>(a.has_bmax); w.pod(a.bmin); w.pod(a.bmax);
    w_list(w, a.empty_subs);
    w.pod(a.count); w.pod(a.sum); w.pod(a.min); w.pod(a.max); w.pod(a.sumsq); w.pod(a.sigma);
    w.pod<uint8_t>(a.hll_present); w.pod(a.precision); w.pod(a.hll_mode);
    w.pod<uint64_t>(a.registers.size()); w.o.append((const char*)a.registers.data(), a.registers.size());
    w.pod<uint64_t>(a.lc.size()); w.o.append((const char*)a.lc.data(), a.lc.size() * 4);
    w.pod<uint64_t>(a.buckets.size());
    for (const RBucket& b : a.buckets) {
        w.pod(b.key); w.str(b.term); w.pod(b.doc_count); w.pod(b.doc_count_error);
        w_list(w, b.subs);
    }
}
void w_list(W& w, const std::vector<RAgg>& l) {
    w.pod<uint32_t>((uint32_t)l.size());
    for (const RAgg& a : l) w_agg(w, a);
}
void r_list(R& r, std::vector<RAgg>& l);
void r_agg(R& r, RAgg& a) {
    a.type = r.pod<int32_t>(); a.order = r.pod<int32_t>(); a.name = r.str();
    a.doc_count_error = r.pod<int64_t>(); a.other_doc_count = r.pod<int64_t>();
    a.required_size = r.pod<int32_t>(); a.shard_size = r.pod<int32_t>();
    a.min_doc_count = r.pod<int64_t>(); a.show_err = r.pod<int32_t>(); a.keyed = r.pod<int32_t>();
    a.has_empty_info = r.pod<uint8_t>(); a.date_unit = r.pod<int32_t>(); a.interval = r.pod<int64_t>();
    a.offset = r.pod<int64_t>();
    a.has_bmin = r.pod<uint8_t>(); a.has_bmax = r.pod<uint8_t>(); a.bmin = r.pod<int64_t>(); a.bmax = r.pod<int64_t>();
    r_list(r, a.empty_subs);
    a.count = r.pod<int64_t>(); a.sum = r.pod<double>(); a.min = r.pod<double>(); a.max = r.pod<double>();
    a.sumsq = r.pod<double>(); a.sigma = r.pod<double>();
    a.hll_present = r.pod<uint8_t>(); a.precision = r.pod<int32_t>(); a.hll_mode = r.pod<int32_t>();
    const uint64_t nr = r.pod<uint64_t>();
    if (r.i + nr > r.n) throw std::runtime_error("truncated stream");
    a.registers.assign(r.p + r.i, r.p + r.i + nr); r.i += nr;
    const uint64_t nl = r.pod<uint64_t>();
    if (r.i + nl * 4 > r.n) throw std::runtime_error("truncated stream");
    a.lc.resize(nl); std::memcpy(a.lc.data(), r.p + r.i, nl * 4); r.i += nl * 4;
    const uint64_t nb = r.pod<uint64_t>();
    a.buckets.resize(nb);
    for (RBucket& b : a.buckets) {
        b.key = r.pod<int64_t>(); b.term = r.str(); b.doc_count = r.pod<int64_t>(); b.doc_count_error = r.pod<int64_t>();
        r_list(r, b.subs);
    }
}
void r_list(R& r, std::vector<RAgg>& l) {
    const uint32_t n = r.pod<uint32_t>();
    l.resize(n);
    for (RAgg& a : l) r_agg(r, a);
}
const uint32_t kStreamMagic = 0x45534750;  // "ESGP"
}  // namespace

void serialize(const std::vector<RAgg>& aggs, std::string& out) {
    out.clear();
    W w{out};
    w.pod(kStreamMagic);
    w.pod<uint32_t>(ESGPU_ABI_VERSION);
    w_list(w, aggs);
}

bool deserialize(const uint8_t* p, size_t n, std::vector<RAgg>& out) {
    R r{p, n};
    if (r.pod<uint32_t>() != kStreamMagic) return false;
    if (r.pod<uint32_t>() != ESGPU_ABI_VERSION) return false;
    r_list(r, out);
    return true;
}

// ------------------------------------------------------------------------------------------------------------
// C view export
// ------------------------------------------------------------------------------------------------------------
ResultHolder* holder_of(const esgpu_result* r) { return reinterpret_cast<ResultHolder*>(const_cast<esgpu_result*>(r)); }

static void export_list(ResultHolder& h, std::vector<RAgg>& src, esgpu_agg_result** out, int32_t* n);

static void export_agg(ResultHolder& h, RAgg& a, esgpu_agg_result& o) {
    std::memset(&o, 0, sizeof o);
    o.type = a.type;
    o.order = a.order;
    o.name = a.name.c_str();
    o.doc_count_error = a.doc_count_error;
    o.other_doc_count = a.other_doc_count;
    o.required_size = a.required_size;
    o.shard_size = a.shard_size;
    o.min_doc_count = a.min_doc_count;
    o.show_term_doc_count_error = a.show_err;
    o.keyed = a.keyed;
    o.has_empty_bucket_info = a.has_empty_info;
    o.date_unit = a.date_unit;
    o.interval = a.interval;
    o.offset = a.offset;
    o.has_extended_bounds_min = a.has_bmin;
    o.has_extended_bounds_max = a.has_bmax;
    o.extended_bounds_min = a.bmin;
    o.extended_bounds_max = a.bmax;
    export_list(h, a.empty_subs, &o.empty_subs, &o.nempty_subs);
    o.count = a.count;
    o.sum = a.sum;
    o.min = a.min;
    o.max = a.max;
    o.sum_of_squares = a.sumsq;
    o.sigma = a.sigma;
    o.hll_present = a.hll_present;
    o.precision = a.precision;
    o.hll_mode = a.hll_mode;
    o.registers = a.registers.empty() ? nullptr : a.registers.data();
    o.lc_hashes = a.lc.empty() ? nullptr : a.lc.data();
    o.lc_size = (int64_t)a.lc.size();
    o.nbuckets = (int64_t)a.buckets.size();
    if (!a.buckets.empty()) {
        std::unique_ptr<esgpu_bucket[]> bb(new esgpu_bucket[a.buckets.size()]);
        for (size_t i = 0; i < a.buckets.size(); ++i) {
            RBucket& b = a.buckets[i];
            esgpu_bucket& ob = bb[i];
            std::memset(&ob, 0, sizeof ob);
            ob.key = b.key;
            ob.key_bytes = (const uint8_t*)b.term.data();
            ob.key_len = (int32_t)b.term.size();
            ob.doc_count = b.doc_count;
            ob.doc_count_error = b.doc_count_error;
            export_list(h, b.subs, &ob.subs, &ob.nsubs);
        }
        o.buckets = bb.get();
        h.bucket_blocks.push_back(std::move(bb));
    }
}

static void export_list(ResultHolder& h, std::vector<RAgg>& src, esgpu_agg_result** out, int32_t* n) {
    *n = (int32_t)src.size();
    *out = nullptr;
    if (src.empty()) return;
    std::unique_ptr<esgpu_agg_result[]> blk(new esgpu_agg_result[src.size()]);
    for (size_t i = 0; i < src.size(); ++i) export_agg(h, src[i], blk[i]);
    *out = blk.get();
    h.agg_blocks.push_back(std::move(blk));
}

void ResultHolder::export_view() {
    agg_blocks.clear();
    bucket_blocks.clear();
    std::memset(&pub, 0, sizeof pub);
    export_list(*this, aggs, &pub.aggs, &pub.naggs);
}

}  // namespace esgpu
