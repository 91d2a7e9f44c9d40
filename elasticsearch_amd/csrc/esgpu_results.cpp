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
#include "java_double.hpp"

#include <algorithm>
#include <iterator>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string_view>
#include <numeric>
#include <unordered_map>
#include <unordered_set>

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
// the same as jmin / jmax without branches (the reduce's contiguous runs vectorise): a NaN operand wins, and of two
// zeros min takes -0.0 / max +0.0 if either operand is one
static inline double jmin_v(double a, double b) {
    uint64_t ua, ub, uz;
    std::memcpy(&ua, &a, 8);
    std::memcpy(&ub, &b, 8);
    uz = ua | ub;
    double z;
    std::memcpy(&z, &uz, 8);
    double r = a <= b ? a : b;
    r = (a == 0.0 && b == 0.0) ? z : r;
    return a != a ? a : r;
}
static inline double jmax_v(double a, double b) {
    uint64_t ua, ub, uz;
    std::memcpy(&ua, &a, 8);
    std::memcpy(&ub, &b, 8);
    uz = ua & ub;
    double z;
    std::memcpy(&z, &uz, 8);
    double r = a >= b ? a : b;
    r = (a == 0.0 && b == 0.0) ? z : r;
    return a != a ? a : r;
}
static inline int64_t jround(double a) {
    if (a != a) return 0;
    if (a >= 9.2233720368547758e18) return INT64_MAX;
    if (a <= -9.2233720368547758e18) return INT64_MIN;
    const double f = std::floor(a);
    return (int64_t)f + ((a - f) >= 0.5 ? 1 : 0);
}
static inline int64_t fdiv(int64_t a, int64_t b) { return a < 0 ? (a - b + 1) / b : a / b; }

bool parse_order_path(const std::string& path, std::string* name, std::string* key) {  // AggregationPath.java:68-113
    if (path.empty() || path.find('>') != std::string::npos) return false;
    const size_t br = path.rfind('[');
    if (br != std::string::npos) {
        if (br == 0 || br > path.size() - 3 || path.back() != ']') return false;
        *name = path.substr(0, br);
        *key = path.substr(br + 1, path.size() - br - 2);
        return true;
    }
    const size_t dot = path.rfind('.');
    if (dot == std::string::npos) { *name = path; key->clear(); return true; }
    if (dot == 0 || dot > path.size() - 2) return false;
    *name = path.substr(0, dot);
    *key = path.substr(dot + 1);
    return true;
}

bool metric_value(int type, const std::string& key, int64_t count, double sum, double min, double max, double sumsq,
                  double sigma, double* out) {
    const double avg = sum / (double)count;
    if (type == ESGPU_AGG_AVG) {
        if (!key.empty() && key != "value") return false;
        *out = avg;
        return true;
    }
    if (key == "count") *out = (double)count;
    else if (key == "sum") *out = sum;
    else if (key == "min") *out = min;
    else if (key == "max") *out = max;
    else if (key == "avg") *out = avg;
    else if (type == ESGPU_AGG_EXTENDED_STATS) {  // InternalExtendedStats.value / ExtendedStatsAggregator.metric
        const double variance = (sumsq - ((sum * sum) / (double)count)) / (double)count;
        if (key == "sum_of_squares") *out = sumsq;
        else if (key == "variance") *out = variance;
        else if (key == "std_deviation") *out = std::sqrt(variance);
        else if (key == "std_upper") *out = avg + (std::sqrt(variance) * sigma);
        else if (key == "std_lower") *out = avg - (std::sqrt(variance) * sigma);
        else return false;
    } else {
        return false;
    }
    return true;
}

// EmptyBucketInfo.rounding (InternalHistogram.java:395-449): the spec's Rounding, time zone included
Rounding Block::rounding() const {
    esgpu_agg_spec sp{};
    sp.type = type;
    sp.date_unit = date_unit;
    sp.interval = interval;
    sp.offset = offset;
    sp.tz_count = (int32_t)tz_starts.size();
    sp.tz_starts = tz_starts.data();
    sp.tz_offsets_ms = tz_offs.data();
    return Rounding::from_spec(sp);
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

int64_t hll_cardinality(int p, bool present, int mode, const uint8_t* regs, size_t nlc) {  // :270-307
    if (!present) return 0;
    if (mode == 0) return linear_counting(1LL << kP2, (1LL << kP2) - (int64_t)nlc);
    const int m = 1 << p;
    const double alpha = p == 4 ? 0.673 : p == 5 ? 0.697 : 0.7213 / (1 + 1.079 / m);
    const double alphaMM = alpha * m * m;
    double inv = 0;
    int zeros = 0;
    for (int i = 0; i < m; ++i) {
        const int rl = regs[i];
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
// HyperLogLogPlusPlus (:161-330) for one bucket: LINEAR_COUNTING keeps the Hashset (:428-498) -- m / 4 int slots, linear
// probing from (k & mask), 0 = empty -- so its values come out in the reference's slot order (writeTo :519-528 and
// merge :201-230 iterate hashSet.values(bucket) in slot order, and the layout depends on the insertion order).
struct HllState {
    int p = 14;
    bool present = false;
    int mode = 0;
    std::vector<uint8_t> regs;
    std::vector<uint32_t> table;  // LINEAR_COUNTING: the Hashset slots
    size_t size = 0;
    size_t threshold() const { return (size_t)((float)((1u << p) / 4) * 0.75f); }  // (int) (capacity * MAX_LOAD_FACTOR)
    void collect_hll(uint32_t e) {  // collectHllEncoded
        uint8_t& r = regs[dec_index(e, p)];
        r = (uint8_t)std::max<uint32_t>(r, dec_run_len(e, p));
    }
    std::vector<uint32_t> lc() const {  // hashSet.values(bucket): slot order
        std::vector<uint32_t> v;
        v.reserve(size);
        for (uint32_t k : table) if (k) v.push_back(k);
        return v;
    }
    void upgrade() {  // upgradeToHll (:309-322)
        regs.assign((size_t)1 << p, 0);
        for (uint32_t k : table) if (k) collect_hll(k);
        table.clear();
        size = 0;
        mode = 1;
    }
    void add(uint32_t k) {  // collectLcEncoded: Hashset.add, upgrade once the size passes the threshold
        if (mode) { collect_hll(k); return; }
        const uint32_t cap = (1u << p) / 4, mask = cap - 1;
        if (table.empty()) table.assign(cap, 0);
        for (uint32_t i = k & mask;; i = (i + 1) & mask) {
            if (table[i] == 0) {
                table[i] = k;
                if (++size > threshold()) upgrade();
                return;
            }
            if (table[i] == k) return;
        }
    }
    void merge(int op, int omode, const std::vector<uint8_t>& oregs, const std::vector<uint32_t>& olc) {
        if (p != op) throw std::invalid_argument("cardinality precision mismatch");
        if (omode == 0) {
            for (uint32_t e : olc) add(e);  // the other sketch's values in its slot order
        } else {
            if (mode == 0) upgrade();
            const int m = 1 << p;
            for (int i = 0; i < m; ++i) regs[i] = std::max(regs[i], oregs[i]);
        }
    }
};

// ------------------------------------------------------------------------------------------------------------
// Block structure helpers
// ------------------------------------------------------------------------------------------------------------
Block Block::like() const {
    Block b;
    b.type = type; b.order = order; b.name = name;
    b.required_size = required_size; b.shard_size = shard_size; b.min_doc_count = min_doc_count;
    b.show_err = show_err; b.keyed = keyed;
    b.has_empty_info = has_empty_info; b.date_unit = date_unit; b.interval = interval; b.offset = offset;
    b.tz_starts = tz_starts; b.tz_offs = tz_offs;
    b.has_bmin = has_bmin; b.has_bmax = has_bmax; b.bmin = bmin; b.bmax = bmax;
    b.sigma = sigma; b.precision = precision; b.order_path = order_path;
    b.time_zone = time_zone; b.value_format = value_format; b.format = format;
    b.n = 0;
    if (is_bucket()) {
        b.boff.assign(1, 0);
        b.term_off.assign(1, 0);
        for (const Block& s : subs) b.subs.push_back(s.like());
        b.empty_subs = empty_subs;
    } else if (type == ESGPU_AGG_FILTER) {
        for (const Block& s : subs) b.subs.push_back(s.like());
    }
    return b;
}

void Block::append_instance(const Block& src, uint64_t i) {
    ++n;
    if (is_bucket()) {
        doc_count_error.push_back(src.doc_count_error[i]);
        other_doc_count.push_back(src.other_doc_count[i]);
        const uint64_t b0 = src.boff[i], b1 = src.boff[i + 1];
        for (uint64_t k = b0; k < b1; ++k) {
            key.push_back(src.key[k]);
            term_pool.append(src.term_pool, src.term_off[k], src.term_off[k + 1] - src.term_off[k]);
            term_off.push_back(term_pool.size());
            bcount.push_back(src.bcount[k]);
            berr.push_back(src.berr[k]);
        }
        boff.push_back(boff.back() + (b1 - b0));
        for (size_t j = 0; j < subs.size(); ++j)
            for (uint64_t k = b0; k < b1; ++k) subs[j].append_instance(src.subs[j], k);
    } else if (type == ESGPU_AGG_FILTER) {
        count.push_back(src.count[i]);
        for (size_t j = 0; j < subs.size(); ++j) subs[j].append_instance(src.subs[j], i);
    } else if (type == ESGPU_AGG_CARDINALITY) {
        hll_present.push_back(src.hll_present[i]);
        hll_mode.push_back(src.hll_mode[i]);
        regs.push_back(src.regs[i]);
        lc.push_back(src.lc[i]);
    } else {
        count.push_back(src.count[i]);
        sum.push_back(src.sum[i]);
        min.push_back(src.min[i]);
        max.push_back(src.max[i]);
        sumsq.push_back(src.sumsq[i]);
    }
}

void Block::append_empty() {  // buildEmptyAggregation
    ++n;
    if (is_bucket()) {
        doc_count_error.push_back(0);
        other_doc_count.push_back(0);
        boff.push_back(boff.back());
    } else if (type == ESGPU_AGG_FILTER) {
        count.push_back(0);
        for (Block& s : subs) s.append_empty();
    } else if (type == ESGPU_AGG_CARDINALITY) {
        hll_present.push_back(0);
        hll_mode.push_back(0);
        regs.emplace_back();
        lc.emplace_back();
    } else {
        count.push_back(0);
        sum.push_back(0.0);
        min.push_back(INFINITY);
        max.push_back(-INFINITY);
        sumsq.push_back(0.0);
    }
}

// ------------------------------------------------------------------------------------------------------------
// reduce: one output instance per group of input instances (shard order inside a group)
//
// All bookkeeping is flat: a level's groups are ranges into one Ref pool, so a reduce allocates O(depth) vectors,
// not O(buckets).
// ------------------------------------------------------------------------------------------------------------
namespace {

struct Ref {
    const Block* b;
    uint64_t i;
};
struct Group {
    uint32_t begin, end;    // range in the level's Ref pool
    bool verbatim = false;  // an empty histogram bucket's prototype sub-aggregation: copied, not reduced
};
struct Level {
    std::vector<Ref> pool;
    std::vector<Group> groups;
    void add(const Ref* r, size_t n, bool verbatim) {
        Group g{(uint32_t)pool.size(), (uint32_t)(pool.size() + n), verbatim};
        pool.insert(pool.end(), r, r + n);
        groups.push_back(g);
    }
};

void reduce_level(const Level& lv, Block& out);

inline std::string_view term_of(const Block& b, uint64_t k) {
    return std::string_view(b.term_pool.data() + b.term_off[k], b.term_off[k + 1] - b.term_off[k]);
}

int cmp_terms(int order, int64_t ca, int64_t cb, std::string_view ta, std::string_view tb) {
    switch (order) {
        case ESGPU_ORDER_COUNT_DESC: if (ca != cb) return ca > cb ? -1 : 1; return ta.compare(tb);
        case ESGPU_ORDER_COUNT_ASC: if (ca != cb) return ca < cb ? -1 : 1; return ta.compare(tb);
        case ESGPU_ORDER_TERM_DESC: return -ta.compare(tb);
        default: return ta.compare(tb);
    }
}

// emitted bucket: its contributing (block, bucket) pairs are contrib[c0, c1) of the group's scratch
struct OutBucket {
    int64_t key;
    const Block* tb;  // where the term bytes live (terms)
    uint64_t tk;
    int64_t count;
    int64_t err;
    uint32_t c0, c1;
    bool empty;
    uint32_t val = 0;   // terms ordered by a sub-aggregation: index of the bucket's value
    uint32_t slot = 0;  // histogram keys on a lattice: the key's slot (DenseKeys)
};

// a histogram reduce whose keys lie on one lattice kmin + j * step: every contribution's slot j, in input order
struct DenseKeys {
    const Ref* refs = nullptr;
    size_t nrefs = 0;
    int64_t kmin = 0;
    uint64_t step = 1;
    uint32_t span = 0;
    std::vector<uint32_t> slot;      // [contributions] in input (shard, bucket) order
    std::vector<int64_t> count;      // [span] summed doc counts
    std::vector<uint32_t> n;         // [span] contributions
    std::vector<int32_t> out;        // [span] position of the slot's bucket among the emitted ones, -1: none
};

struct Scratch {
    std::vector<double> vals;
    std::vector<Ref> contrib;
    std::vector<OutBucket> buckets, filled;
    std::vector<uint32_t> ids, start;
    std::unordered_map<std::string_view, uint32_t> index;
    std::vector<Ref> child;
    DenseKeys dense;
};

// numeric metric sub-aggregations of a bucket reduce are reduced as their bucket is emitted (no child level): their
// reduce reads nothing but the contributions' partials, and instances are appended in emission order either way
inline bool fused_leaf(const Block& b) {
    return b.type == ESGPU_AGG_STATS || b.type == ESGPU_AGG_EXTENDED_STATS || b.type == ESGPU_AGG_AVG;
}

// InternalStats / InternalExtendedStats / InternalAvg .doReduce of sub-aggregation j over contributions [c0, c1) (shard
// order): sums in that order from 0, Math.min / Math.max
void reduce_leaf(Block& m, const Scratch& sc, size_t j, uint32_t c0, uint32_t c1) {
    int64_t count = 0;
    double mn = INFINITY, mx = -INFINITY, sum = 0, sq = 0;
    for (uint32_t c = c0; c < c1; ++c) {
        const Block& b = sc.contrib[c].b->subs[j];
        const uint64_t i = sc.contrib[c].i;
        count += b.count[i];
        mn = jmin(mn, b.min[i]);
        mx = jmax(mx, b.max[i]);
        sum += b.sum[i];
        sq += b.sumsq[i];
    }
    ++m.n;
    m.count.push_back(count);
    m.min.push_back(mn);
    m.max.push_back(mx);
    m.sum.push_back(sum);
    m.sumsq.push_back(sq);
}

// fused metric sub-aggregation j of a lattice histogram reduce: the emitted buckets' instances initialised (an empty
// bucket's from its prototype), then every shard's partials streamed in shard order into their bucket's instance --
// the same additions in the same order as reduce_leaf, without a contribution list
void stream_leaf(Block& m, const Block* proto, const std::vector<OutBucket>& buckets, const DenseKeys& dk, size_t j) {
    const size_t base = m.count.size(), nb = buckets.size();
    m.n += nb;
    m.count.resize(base + nb, 0);
    m.sum.resize(base + nb, 0.0);
    m.min.resize(base + nb, INFINITY);
    m.max.resize(base + nb, -INFINITY);
    m.sumsq.resize(base + nb, 0.0);
    for (size_t q = 0; q < nb; ++q)
        if (buckets[q].empty) {  // only with EmptyBucketInfo: proto = its prototype
            m.count[base + q] = proto->count[0];
            m.sum[base + q] = proto->sum[0];
            m.min[base + q] = proto->min[0];
            m.max[base + q] = proto->max[0];
            m.sumsq[base + q] = proto->sumsq[0];
        }
    int64_t* cnt = m.count.data() + base;
    double *sum = m.sum.data() + base, *mn = m.min.data() + base, *mx = m.max.data() + base, *sq = m.sumsq.data() + base;
    size_t e = 0;
    for (size_t x = 0; x < dk.nrefs; ++x) {
        const Block& h = *dk.refs[x].b;
        const Block& L = h.subs[j];
        const uint64_t b0 = h.boff[dk.refs[x].i], b1 = h.boff[dk.refs[x].i + 1];
        const uint64_t len = b1 - b0;
        if (len > 1) {  // the shard's run lands on consecutive emitted buckets (a complete time series): one vector pass
            // every position checked, not only the ends: a count-ordered histogram permutes out[], and min_doc_count
            // drops slots (out = -1), so a run whose ends are len - 1 apart may still map its middle elsewhere
            const int32_t o0 = dk.out[dk.slot[e]];
            bool run = o0 >= 0;
            for (uint64_t t = 1; run && t < len; ++t) run = dk.out[dk.slot[e + t]] == o0 + (int32_t)t;
            if (run) {
                // one loop per array (two streams each, no aliasing between output arrays to disprove): each vectorises
                {
                    int64_t* __restrict__ o = cnt + o0;
                    const int64_t* __restrict__ in = L.count.data() + b0;
                    for (uint64_t t = 0; t < len; ++t) o[t] += in[t];
                }
                {
                    double* __restrict__ o = mn + o0;
                    const double* __restrict__ in = L.min.data() + b0;
                    for (uint64_t t = 0; t < len; ++t) o[t] = jmin_v(o[t], in[t]);
                }
                {
                    double* __restrict__ o = mx + o0;
                    const double* __restrict__ in = L.max.data() + b0;
                    for (uint64_t t = 0; t < len; ++t) o[t] = jmax_v(o[t], in[t]);
                }
                {
                    double* __restrict__ o = sum + o0;
                    const double* __restrict__ in = L.sum.data() + b0;
                    for (uint64_t t = 0; t < len; ++t) o[t] += in[t];
                }
                {
                    double* __restrict__ o = sq + o0;
                    const double* __restrict__ in = L.sumsq.data() + b0;
                    for (uint64_t t = 0; t < len; ++t) o[t] += in[t];
                }
                e += len;
                continue;
            }
        }
        for (uint64_t k = b0; k < b1; ++k) {
            const int32_t o = dk.out[dk.slot[e++]];
            if (o < 0) continue;
            cnt[o] += L.count[k];
            mn[o] = jmin(mn[o], L.min[k]);
            mx[o] = jmax(mx[o], L.max[k]);
            sum[o] += L.sum[k];
            sq[o] += L.sumsq[k];
        }
    }
}

void emit_buckets(Block& out, const std::vector<OutBucket>& buckets, const Scratch& sc, std::vector<Level>& child,
                  DenseKeys* dk = nullptr) {
    const size_t nb = buckets.size();
    // the bucket arrays sized once and written by index; then each sub-aggregation's instances in bucket order (every
    // sub-block is independent of the others, so per-sub passes append exactly what the per-bucket loop did)
    const size_t k0 = out.key.size(), t0 = out.term_off.size();
    out.key.resize(k0 + nb);
    out.bcount.resize(k0 + nb);
    out.berr.resize(k0 + nb);
    out.term_off.resize(t0 + nb);
    for (size_t q = 0; q < nb; ++q) {
        const OutBucket& ob = buckets[q];
        out.key[k0 + q] = ob.key;
        if (ob.tb) {
            const std::string_view t = term_of(*ob.tb, ob.tk);
            out.term_pool.append(t.data(), t.size());
        }
        out.term_off[t0 + q] = out.term_pool.size();
        out.bcount[k0 + q] = ob.count;
        out.berr[k0 + q] = ob.err;
    }
    for (size_t j = 0; j < out.subs.size(); ++j) {
        Block& m = out.subs[j];
        if (fused_leaf(m)) {
            if (dk) continue;  // streamed below
            for (auto* v : {&m.sum, &m.min, &m.max, &m.sumsq}) v->reserve(v->size() + nb);
            m.count.reserve(m.count.size() + nb);
            for (const OutBucket& ob : buckets) {
                if (ob.empty) m.append_instance(out.empty_subs[j], 0);
                else reduce_leaf(m, sc, j, ob.c0, ob.c1);
            }
            continue;
        }
        Level& lv = child[j];
        for (const OutBucket& ob : buckets) {
            if (ob.empty) {
                const Ref r{&out.empty_subs[j], 0};
                lv.add(&r, 1, true);
                continue;
            }
            Group g{(uint32_t)lv.pool.size(), 0, false};
            for (uint32_t c = ob.c0; c < ob.c1; ++c) lv.pool.push_back({&sc.contrib[c].b->subs[j], sc.contrib[c].i});
            g.end = (uint32_t)lv.pool.size();
            lv.groups.push_back(g);
        }
    }
    out.boff.push_back(out.boff.back() + buckets.size());
    if (dk) {
        bool any = false;
        for (const Block& m : out.subs) any |= fused_leaf(m);
        if (any) {
            dk->out.assign(dk->span, -1);
            for (size_t q = 0; q < nb; ++q)
                if (!buckets[q].empty) dk->out[buckets[q].slot] = (int32_t)q;
            for (size_t j = 0; j < out.subs.size(); ++j)
                if (fused_leaf(out.subs[j]))
                    stream_leaf(out.subs[j], j < out.empty_subs.size() ? &out.empty_subs[j] : nullptr, buckets, *dk, j);
        }
    }
}

void reduce_terms(const Ref* refs, size_t nrefs, Block& out, Scratch& sc, std::vector<Level>& child) {  // InternalTerms.doReduce
    int64_t sumErr = 0, other = 0;
    sc.buckets.clear();
    sc.contrib.clear();
    sc.ids.clear();
    sc.index.clear();
    std::vector<Ref>& entries = sc.child;  // (block, bucket) in shard order
    entries.clear();
    for (size_t x = 0; x < nrefs; ++x) {
        const Ref& r = refs[x];
        const Block& t = *r.b;
        other += t.other_doc_count[r.i];
        const uint64_t b0 = t.boff[r.i], b1 = t.boff[r.i + 1];
        int64_t thisErr;
        if ((int64_t)(b1 - b0) < out.shard_size || out.order == ESGPU_ORDER_TERM_ASC || out.order == ESGPU_ORDER_TERM_DESC) thisErr = 0;
        else if (out.order == ESGPU_ORDER_COUNT_DESC) thisErr = t.bcount[b1 - 1];
        else thisErr = -1;
        if (sumErr != -1) sumErr = thisErr == -1 ? -1 : sumErr + thisErr;
        for (uint64_t k = b0; k < b1; ++k) {
            uint32_t id;
            if (nrefs == 1) {  // one shard: its terms are distinct
                id = (uint32_t)sc.buckets.size();
                sc.buckets.push_back(OutBucket{t.key[k], &t, k, 0, 0, 0, 0, false});
            } else {
                auto ins = sc.index.try_emplace(term_of(t, k), (uint32_t)sc.buckets.size());
                if (ins.second) sc.buckets.push_back(OutBucket{t.key[k], &t, k, 0, 0, 0, 0, false});
                id = ins.first->second;
            }
            OutBucket& ob = sc.buckets[id];
            ob.count += t.bcount[k];
            if (ob.err != -1) ob.err = thisErr == -1 ? -1 : ob.err + thisErr;  // Bucket.reduce of per-shard errors
            ob.c1++;  // contribution count for now
            sc.ids.push_back(id);
            entries.push_back({&t, k});
        }
    }
    // contributions grouped by bucket, shard order kept (counting sort)
    const uint32_t nb = (uint32_t)sc.buckets.size();
    sc.start.assign(nb + 1, 0);
    for (uint32_t id = 0; id < nb; ++id) sc.start[id + 1] = sc.start[id] + sc.buckets[id].c1;
    for (uint32_t id = 0; id < nb; ++id) { sc.buckets[id].c0 = sc.start[id]; sc.buckets[id].c1 = sc.start[id]; }
    sc.contrib.resize(entries.size());
    for (size_t e = 0; e < entries.size(); ++e) sc.contrib[sc.buckets[sc.ids[e]].c1++] = entries[e];
    // per-bucket error relative to the summed shard error, min_doc_count filter (in place)
    size_t m = 0;
    for (uint32_t id = 0; id < nb; ++id) {
        OutBucket ob = sc.buckets[id];
        if (ob.err != -1) ob.err = sumErr == -1 ? -1 : sumErr - ob.err;
        if (ob.count >= out.min_doc_count) sc.buckets[m++] = ob;
    }
    sc.buckets.resize(m);
    const size_t size = std::min<size_t>((size_t)std::max(out.required_size, 0), nb);
    // InternalOrder.Aggregation: the reduced sub-aggregation's value (AggregationPath.resolveValue on the reduced
    // bucket), from the metric partials of the bucket's contributions reduced in shard order
    const bool agg_order = out.order == ESGPU_ORDER_AGG_ASC || out.order == ESGPU_ORDER_AGG_DESC;
    std::vector<double>& vals = sc.vals;
    if (agg_order) {
        std::string name, key;
        int j = -1;
        if (parse_order_path(out.order_path, &name, &key))
            for (size_t x = 0; x < out.subs.size(); ++x) if (out.subs[x].name == name) j = (int)x;
        if (j < 0) throw std::invalid_argument("Invalid order path [" + out.order_path + "]");
        vals.resize(sc.buckets.size());
        for (size_t b = 0; b < sc.buckets.size(); ++b) {
            const OutBucket& ob = sc.buckets[b];
            sc.buckets[b].val = (uint32_t)b;
            if (out.subs[j].type == ESGPU_AGG_CARDINALITY) {  // InternalCardinality.doReduce, then .value()
                if (!key.empty() && key != "value") throw std::invalid_argument("Invalid order path [" + out.order_path + "]");
                HllState st;
                for (uint32_t c = ob.c0; c < ob.c1; ++c) {
                    const Block& m = sc.contrib[c].b->subs[j];
                    const uint64_t i = sc.contrib[c].i;
                    if (!m.hll_present[i]) continue;
                    if (!st.present) { st.present = true; st.p = m.precision; st.mode = 0; }
                    st.merge(m.precision, m.hll_mode[i], m.regs[i], m.lc[i]);
                }
                vals[b] = (double)(st.present ? hll_cardinality(st.p, true, st.mode, st.regs.data(), st.mode ? 0 : st.lc().size()) : 0);
                continue;
            }
            int64_t cnt = 0;
            double sum = 0, mn = INFINITY, mx = -INFINITY, sq = 0;
            for (uint32_t c = ob.c0; c < ob.c1; ++c) {
                const Block& m = sc.contrib[c].b->subs[j];
                const uint64_t i = sc.contrib[c].i;
                cnt += m.count[i];
                sum += m.sum[i];
                mn = jmin(mn, m.min[i]);
                mx = jmax(mx, m.max[i]);
                sq += m.sumsq[i];
            }
            if (!metric_value(out.subs[j].type, key, cnt, sum, mn, mx, sq, out.subs[j].sigma, &vals[b]))
                throw std::invalid_argument("Invalid order path [" + out.order_path + "]");
            sc.buckets[b].val = (uint32_t)b;
        }
    }
    auto less = [&](const OutBucket& a, const OutBucket& b) {
        if (agg_order) {
            const int c = compare_discard_nan(vals[a.val], vals[b.val], out.order == ESGPU_ORDER_AGG_ASC);
            if (c != 0) return c < 0;
            return term_of(*a.tb, a.tk).compare(term_of(*b.tb, b.tk)) < 0;
        }
        return cmp_terms(out.order, a.count, b.count, term_of(*a.tb, a.tk), term_of(*b.tb, b.tk)) < 0;
    };
    if (sc.buckets.size() > size) {
        std::partial_sort(sc.buckets.begin(), sc.buckets.begin() + size, sc.buckets.end(), less);
        for (size_t i = size; i < sc.buckets.size(); ++i) other += sc.buckets[i].count;
        sc.buckets.resize(size);
    } else {
        std::sort(sc.buckets.begin(), sc.buckets.end(), less);
    }
    ++out.n;
    out.doc_count_error.push_back(sumErr == -1 ? -1 : (nrefs == 1 ? 0 : sumErr));
    out.other_doc_count.push_back(other);
    emit_buckets(out, sc.buckets, sc, child);
}

// InternalHistogram.reduceBuckets' merge when every key lies on one lattice kmin + j * step (step = the gcd of the key
// gaps: a fixed interval or a fixed-length date unit): a contribution's slot is its key's position on the lattice, so the
// merged buckets are the non-empty slots in slot order -- exactly the k-way merge by (key, shard) -- and their doc
// counts are summed by streaming each shard.  Returns false (nothing usable) when the keys are off one lattice or span
// more than ~4 slots per contribution.
bool dense_slots(const Ref* refs, size_t nrefs, size_t total, DenseKeys& dk) {
    int64_t kmin = INT64_MAX, kmax = INT64_MIN;
    uint64_t step = 0;
    for (size_t x = 0; x < nrefs; ++x) {
        const Block& h = *refs[x].b;
        const uint64_t b0 = h.boff[refs[x].i], b1 = h.boff[refs[x].i + 1];
        if (b0 == b1) continue;
        kmin = std::min(kmin, h.key[b0]);
        kmax = std::max(kmax, h.key[b1 - 1]);
        for (uint64_t k = b0 + 1; k < b1; ++k) {
            const uint64_t d = (uint64_t)h.key[k] - (uint64_t)h.key[k - 1];
            if (d != step) step = std::gcd(step, d);  // consecutive keys one step apart: nothing to do
        }
    }
    if (kmin > kmax) return false;
    const uint64_t range = (uint64_t)kmax - (uint64_t)kmin;  // kmin <= kmax: exact in two's complement
    if (step == 0) step = range ? range : 1;
    if (range / step + 1 > 4 * (uint64_t)total + 64) return false;
    dk.refs = refs;
    dk.nrefs = nrefs;
    dk.kmin = kmin;
    dk.step = step;
    dk.span = (uint32_t)(range / step + 1);
    dk.slot.resize(total);
    dk.count.assign(dk.span, 0);
    dk.n.assign(dk.span, 0);
    size_t e = 0;
    for (size_t x = 0; x < nrefs; ++x) {
        const Block& h = *refs[x].b;
        const uint64_t b0 = h.boff[refs[x].i], b1 = h.boff[refs[x].i + 1];
        if (b0 == b1) continue;
        const uint64_t off0 = (uint64_t)h.key[b0] - (uint64_t)kmin;
        if (off0 % step) return false;  // this shard's keys are off the lattice (its gaps are multiples of step)
        uint32_t j = (uint32_t)(off0 / step);
        if ((uint64_t)h.key[b1 - 1] - (uint64_t)h.key[b0] == (b1 - b0 - 1) * step) {
            // strictly increasing keys whose gaps (multiples of step) sum to (n - 1) steps: every gap is one step
            const int64_t* bc = h.bcount.data() + b0;
            uint32_t* sl = dk.slot.data() + e;
            int64_t* dc = dk.count.data() + j;
            uint32_t* dn = dk.n.data() + j;
            const uint64_t len = b1 - b0;
            for (uint64_t t = 0; t < len; ++t) {
                sl[t] = j + (uint32_t)t;
                dc[t] += bc[t];
                dn[t] += 1;
            }
            e += len;
            continue;
        }
        for (uint64_t k = b0; k < b1; ++k) {
            if (k > b0) {  // one division per gap longer than a step
                const uint64_t d = (uint64_t)h.key[k] - (uint64_t)h.key[k - 1];
                j += d == step ? 1u : (uint32_t)(d / step);
            }
            dk.slot[e++] = j;
            dk.count[j] += h.bcount[k];
            ++dk.n[j];
        }
    }
    return true;
}

void reduce_histogram(const Ref* refs, size_t nrefs, Block& out, Scratch& sc, std::vector<Level>& child) {  // InternalHistogram.doReduce
    std::vector<OutBucket>& list = sc.buckets;
    list.clear();
    sc.contrib.clear();
    DenseKeys* dense = nullptr;
    if (nrefs == 1) {  // one shard: already key-sorted, nothing to merge
        const Block& h = *refs[0].b;
        const uint64_t i = refs[0].i;
        for (uint64_t k = h.boff[i]; k < h.boff[i + 1]; ++k) {
            if (h.bcount[k] < out.min_doc_count) continue;
            const uint32_t c = (uint32_t)sc.contrib.size();
            sc.contrib.push_back({&h, k});
            list.push_back(OutBucket{h.key[k], nullptr, 0, h.bcount[k], 0, c, c + 1, false});
        }
    } else {
        // InternalHistogram.reduceBuckets: every shard's buckets are key-ascending, so a k-way merge by (key, shard)
        // orders them (equal keys in shard order); inputs not in key order (a reduced result with another order)
        // take a stable sort instead
        std::vector<Ref>& all = sc.contrib;
        all.clear();
        bool sorted = true;
        size_t total = 0;
        for (size_t x = 0; x < nrefs; ++x) {
            const Block& h = *refs[x].b;
            const uint64_t b0 = h.boff[refs[x].i], b1 = h.boff[refs[x].i + 1];
            total += b1 - b0;
            for (uint64_t k = b0 + 1; k < b1 && sorted; ++k) sorted = h.key[k - 1] < h.key[k];
        }
        DenseKeys& dk = sc.dense;
        if (sorted && total && dense_slots(refs, nrefs, total, dk)) {
            bool need_contrib = false;  // contributions grouped by slot only for sub-aggregations that are not streamed
            for (const Block& m : out.subs) need_contrib |= !fused_leaf(m);
            std::vector<uint32_t>& start = sc.start;
            if (need_contrib) {
                start.assign((size_t)dk.span + 1, 0);
                for (uint32_t j = 0; j < dk.span; ++j) start[j + 1] = start[j] + dk.n[j];
            }
            for (uint32_t j = 0; j < dk.span; ++j) {
                if (!dk.n[j] || dk.count[j] < out.min_doc_count) continue;
                OutBucket ob{dk.kmin + (int64_t)((uint64_t)j * dk.step), nullptr, 0, dk.count[j], 0, 0, 0, false};
                if (need_contrib) { ob.c0 = start[j]; ob.c1 = start[j + 1]; }
                ob.slot = j;
                list.push_back(ob);
            }
            if (need_contrib) {  // counting sort by slot, shard order kept within a slot
                all.resize(total);
                size_t e = 0;
                for (size_t x = 0; x < nrefs; ++x) {
                    const Block& h = *refs[x].b;
                    for (uint64_t k = h.boff[refs[x].i]; k < h.boff[refs[x].i + 1]; ++k) all[start[dk.slot[e++]]++] = Ref{&h, k};
                }
            }
            dense = &dk;
        } else if (sorted && nrefs <= 16) {
            // few shards: the next key is the minimum of the heads; every head at that key contributes, in shard
            // order -- one scan of the heads per output key, the buckets of a key landing together
            uint64_t pos[16], end[16];
            for (size_t x = 0; x < nrefs; ++x) {
                pos[x] = refs[x].b->boff[refs[x].i];
                end[x] = refs[x].b->boff[refs[x].i + 1];
            }
            for (;;) {
                int64_t key = INT64_MAX;
                bool any = false;
                for (size_t x = 0; x < nrefs; ++x)
                    if (pos[x] < end[x]) {
                        const int64_t k = refs[x].b->key[pos[x]];
                        if (!any || k < key) key = k;
                        any = true;
                    }
                if (!any) break;
                for (size_t x = 0; x < nrefs; ++x)
                    if (pos[x] < end[x] && refs[x].b->key[pos[x]] == key) all.push_back({refs[x].b, pos[x]++});
            }
        } else if (sorted) {
            struct Head { int64_t key; uint32_t x; uint64_t k, end; };
            std::vector<Head> heap;
            heap.reserve(nrefs);
            auto later = [](const Head& a, const Head& b) { return a.key != b.key ? a.key > b.key : a.x > b.x; };
            for (size_t x = 0; x < nrefs; ++x) {
                const Block& h = *refs[x].b;
                const uint64_t b0 = h.boff[refs[x].i], b1 = h.boff[refs[x].i + 1];
                if (b0 < b1) heap.push_back({h.key[b0], (uint32_t)x, b0, b1});
            }
            std::make_heap(heap.begin(), heap.end(), later);
            while (!heap.empty()) {
                std::pop_heap(heap.begin(), heap.end(), later);
                Head& t = heap.back();
                const Block* b = refs[t.x].b;
                all.push_back({b, t.k});
                if (++t.k < t.end) {
                    t.key = b->key[t.k];
                    std::push_heap(heap.begin(), heap.end(), later);
                } else {
                    heap.pop_back();
                }
            }
        } else {
            for (size_t x = 0; x < nrefs; ++x)
                for (uint64_t k = refs[x].b->boff[refs[x].i]; k < refs[x].b->boff[refs[x].i + 1]; ++k) all.push_back({refs[x].b, k});
            std::stable_sort(all.begin(), all.end(), [](const Ref& a, const Ref& b) { return a.b->key[a.i] < b.b->key[b.i]; });
        }
        for (size_t x = 0; !dense && x < all.size();) {
            const int64_t key = all[x].b->key[all[x].i];
            OutBucket ob{key, nullptr, 0, 0, 0, (uint32_t)x, 0, false};
            size_t y = x;
            for (; y < all.size() && all[y].b->key[all[y].i] == key; ++y) ob.count += all[y].b->bcount[all[y].i];
            ob.c1 = (uint32_t)y;
            if (ob.count >= out.min_doc_count) list.push_back(ob);
            x = y;
        }
    }
    if (out.min_doc_count == 0 && out.has_empty_info) {  // addEmptyBuckets (InternalHistogram.java:395-449)
        const Rounding rnd = out.rounding();
        // an affine rounding's next bucket key is the key plus its interval (no time-zone arithmetic per bucket)
        int64_t ai = 0, ao = 0;
        const bool aff = rnd.affine(&ai, &ao);
        auto next = [&](int64_t k) {
            int64_t n;
            if (aff && !__builtin_add_overflow(k, ai, &n)) return n;
            return rnd.next_rounding_value(k);
        };
        auto empty = [](int64_t k) { return OutBucket{k, nullptr, 0, 0, 0, 0, 0, true}; };
        std::vector<OutBucket>& filled = sc.filled;
        filled.clear();
        if (list.empty()) {
            if (out.has_bmin && out.has_bmax)
                for (int64_t k = out.bmin; k <= out.bmax; k = next(k)) filled.push_back(empty(k));
        } else {
            if (out.has_bmin)
                for (int64_t k = out.bmin; k < list[0].key; k = next(k)) filled.push_back(empty(k));
            for (size_t i = 0; i < list.size(); ++i) {
                if (i > 0)
                    for (int64_t k = next(list[i - 1].key); k < list[i].key; k = next(k)) filled.push_back(empty(k));
                filled.push_back(list[i]);
            }
            const int64_t last = filled.back().key;
            if (out.has_bmax && out.bmax > last)
                for (int64_t k = next(last); k <= out.bmax; k = next(k)) filled.push_back(empty(k));
        }
        list.swap(filled);
    }
    if (out.order == ESGPU_ORDER_KEY_DESC) std::reverse(list.begin(), list.end());
    else if (out.order == ESGPU_ORDER_HCOUNT_ASC || out.order == ESGPU_ORDER_HCOUNT_DESC) {
        const bool asc = out.order == ESGPU_ORDER_HCOUNT_ASC;
        std::stable_sort(list.begin(), list.end(), [&](const OutBucket& a, const OutBucket& b) {
            if (a.count != b.count) return asc ? a.count < b.count : a.count > b.count;
            return a.key < b.key;
        });
    }
    ++out.n;
    out.doc_count_error.push_back(0);
    out.other_doc_count.push_back(0);
    emit_buckets(out, list, sc, child, dense);
}

// copy a prototype instance; its sub-aggregations stay verbatim too (queued in bucket order)
void copy_verbatim(const Ref& r, Block& out, std::vector<Level>& child) {
    const Block& src = *r.b;
    const uint64_t i = r.i;
    ++out.n;
    out.doc_count_error.push_back(src.doc_count_error[i]);
    out.other_doc_count.push_back(src.other_doc_count[i]);
    for (uint64_t k = src.boff[i]; k < src.boff[i + 1]; ++k) {
        out.key.push_back(src.key[k]);
        const std::string_view t = term_of(src, k);
        out.term_pool.append(t.data(), t.size());
        out.term_off.push_back(out.term_pool.size());
        out.bcount.push_back(src.bcount[k]);
        out.berr.push_back(src.berr[k]);
        for (size_t j = 0; j < out.subs.size(); ++j) {
            if (fused_leaf(out.subs[j])) { out.subs[j].append_instance(src.subs[j], k); continue; }
            const Ref c{&src.subs[j], k};
            child[j].add(&c, 1, true);
        }
    }
    out.boff.push_back(out.boff.back() + (src.boff[i + 1] - src.boff[i]));
}

void reduce_level(const Level& lv, Block& out) {
    if (out.is_bucket()) {
        std::vector<Level> child(out.subs.size());
        Scratch sc;
        for (const Group& g : lv.groups) {
            const Ref* refs = lv.pool.data() + g.begin;
            const size_t n = g.end - g.begin;
            if (g.verbatim) copy_verbatim(refs[0], out, child);
            else if (out.type == ESGPU_AGG_TERMS) reduce_terms(refs, n, out, sc, child);
            else reduce_histogram(refs, n, out, sc, child);
        }
        for (size_t j = 0; j < out.subs.size(); ++j)
            if (!fused_leaf(out.subs[j])) reduce_level(child[j], out.subs[j]);
        return;
    }
    if (out.type == ESGPU_AGG_FILTER) {  // InternalFilter (InternalSingleBucketAggregation.doReduce): Σ doc_count, subs
        std::vector<Level> child(out.subs.size());
        std::vector<Ref> rs;
        for (const Group& g : lv.groups) {
            const Ref* refs = lv.pool.data() + g.begin;
            const size_t n = g.end - g.begin;
            int64_t dc = 0;
            for (size_t x = 0; x < n; ++x) dc += refs[x].b->count[refs[x].i];
            ++out.n;
            out.count.push_back(dc);
            for (size_t j = 0; j < out.subs.size(); ++j) {
                rs.clear();
                for (size_t x = 0; x < n; ++x) rs.push_back({&refs[x].b->subs[j], refs[x].i});
                child[j].add(rs.data(), rs.size(), g.verbatim);
            }
        }
        for (size_t j = 0; j < out.subs.size(); ++j) reduce_level(child[j], out.subs[j]);
        return;
    }
    for (const Group& g : lv.groups) {
        const Ref* refs = lv.pool.data() + g.begin;
        const size_t n = g.end - g.begin;
        if (g.verbatim) {
            out.append_instance(*refs[0].b, refs[0].i);
            continue;
        }
        if (out.type == ESGPU_AGG_CARDINALITY) {  // InternalCardinality.doReduce (:103-121)
            HllState st;
            bool any = false;
            for (size_t x = 0; x < n; ++x) {
                const Ref& r = refs[x];
                if (!r.b->hll_present[r.i]) continue;
                if (!any) { any = true; st.present = true; st.p = r.b->precision; st.mode = 0; }
                st.merge(r.b->precision, r.b->hll_mode[r.i], r.b->regs[r.i], r.b->lc[r.i]);
            }
            if (!any) { out.append_instance(*refs[0].b, refs[0].i); continue; }  // all empty: the first one
            ++out.n;
            out.hll_present.push_back(1);
            out.hll_mode.push_back(st.mode);
            out.regs.push_back(std::move(st.regs));
            out.lc.push_back(st.mode ? std::vector<uint32_t>() : st.lc());
            continue;
        }
        // InternalStats / InternalExtendedStats / InternalAvg .doReduce: sums in shard order, Math.min / Math.max
        int64_t count = 0;
        double mn = INFINITY, mx = -INFINITY, sum = 0, sq = 0;
        for (size_t x = 0; x < n; ++x) {
            const Ref& r = refs[x];
            count += r.b->count[r.i];
            mn = jmin(mn, r.b->min[r.i]);
            mx = jmax(mx, r.b->max[r.i]);
            sum += r.b->sum[r.i];
            sq += r.b->sumsq[r.i];
        }
        ++out.n;
        out.count.push_back(count);
        out.min.push_back(mn);
        out.max.push_back(mx);
        out.sum.push_back(sum);
        out.sumsq.push_back(sq);
    }
}

}  // namespace

// shard results of one request share the aggregation tree (types, sub-aggregation lists, sketch precision)
bool same_shape(const Block& a, const Block& b) {
    if (a.type != b.type || a.subs.size() != b.subs.size() || a.empty_subs.size() != b.empty_subs.size()) return false;
    if (a.type == ESGPU_AGG_CARDINALITY && a.precision != b.precision) return false;
    for (size_t j = 0; j < a.subs.size(); ++j) if (!same_shape(a.subs[j], b.subs[j])) return false;
    return true;
}

std::vector<Block> reduce_lists(const std::vector<const std::vector<Block>*>& lists) {
    std::vector<Block> out;
    if (lists.empty()) return out;
    const size_t n = lists[0]->size();
    for (size_t a = 0; a < n; ++a) {
        Level lv;
        for (auto* l : lists) {
            if (l->size() != n) throw std::invalid_argument("shard results have different aggregation lists");
            if (!same_shape((*l)[a], (*lists[0])[a])) throw std::invalid_argument("aggregation trees differ across shards");
            lv.pool.push_back({&(*l)[a], 0});
        }
        lv.groups.push_back(Group{0, (uint32_t)lv.pool.size(), false});
        Block b = (*lists[0])[a].like();
        reduce_level(lv, b);
        out.push_back(std::move(b));
    }
    return out;
}

// ------------------------------------------------------------------------------------------------------------
// JSON
// ------------------------------------------------------------------------------------------------------------
namespace {
struct J {
    std::string s;
    void raw(const char* t) { s += t; }
    void str(const char* p, size_t n) {
        s += '"';
        for (size_t i = 0; i < n; ++i) {
            const unsigned char c = (unsigned char)p[i];
            if (c == '"' || c == '\\') { s += '\\'; s += (char)c; }
            else if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); s += b; }
            else s += (char)c;
        }
        s += '"';
    }
    void str(const std::string& v) { str(v.data(), v.size()); }
    void i64(int64_t v) { char b[24]; snprintf(b, sizeof b, "%lld", (long long)v); s += b; }
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
    const int64_t days = fdiv(ms, kMsDay);
    const int64_t rem = ms - days * kMsDay;
    int64_t y; int m, d;
    r_civil_from_days(days, &y, &m, &d);
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

void write_instance(J& j, const Block& a, uint64_t i);

void write_subs(J& j, const Block& a, uint64_t k) {
    for (const Block& s : a.subs) {
        j.raw(",");
        j.key(s.name);
        write_instance(j, s, k);
    }
}

void write_instance(J& j, const Block& a, uint64_t i) {
    j.raw("{");
    switch (a.type) {
        case ESGPU_AGG_TERMS:
            j.key("doc_count_error_upper_bound"); j.i64(a.doc_count_error[i]); j.raw(",");
            j.key("sum_other_doc_count"); j.i64(a.other_doc_count[i]); j.raw(",");
            j.key("buckets"); j.raw("[");
            for (uint64_t k = a.boff[i]; k < a.boff[i + 1]; ++k) {
                if (k != a.boff[i]) j.raw(",");
                j.raw("{"); j.key("key"); j.str(a.term_pool.data() + a.term_off[k], a.term_off[k + 1] - a.term_off[k]); j.raw(",");
                j.key("doc_count"); j.i64(a.bcount[k]);
                if (a.show_err) { j.raw(","); j.key("doc_count_error_upper_bound"); j.i64(a.berr[k]); }
                write_subs(j, a, k);
                j.raw("}");
            }
            j.raw("]");
            break;
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM:
            j.key("buckets"); j.raw("[");
            for (uint64_t k = a.boff[i]; k < a.boff[i + 1]; ++k) {
                if (k != a.boff[i]) j.raw(",");
                j.raw("{");
                if (a.type == ESGPU_AGG_DATE_HISTOGRAM) { j.key("key_as_string"); j.str(iso8601(a.key[k])); j.raw(","); }
                j.key("key"); j.i64(a.key[k]); j.raw(",");
                j.key("doc_count"); j.i64(a.bcount[k]);
                write_subs(j, a, k);
                j.raw("}");
            }
            j.raw("]");
            break;
        case ESGPU_AGG_FILTER:  // InternalSingleBucketAggregation.doXContentBody: doc_count, then the sub-aggregations
            j.key("doc_count"); j.i64(a.count[i]);
            write_subs(j, a, i);
            break;
        case ESGPU_AGG_AVG:
            j.key("value"); j.opt(a.count[i] != 0, a.sum[i] / (double)a.count[i]);
            j.raw(","); j.key("_internal"); j.raw("{"); j.key("count"); j.i64(a.count[i]); j.raw(",");
            j.key("sum"); j.dbl(a.sum[i]); j.raw("}");
            break;
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS: {
            const int64_t cnt = a.count[i];
            const double sum = a.sum[i], mn = a.min[i], mx = a.max[i], sq = a.sumsq[i];
            const bool c = cnt != 0;
            const double avg = sum / (double)cnt;
            j.key("count"); j.i64(cnt); j.raw(",");
            j.key("min"); j.opt(c, mn); j.raw(",");
            j.key("max"); j.opt(c, mx); j.raw(",");
            j.key("avg"); j.opt(c, avg); j.raw(",");
            j.key("sum"); j.opt(c, sum);
            if (a.type == ESGPU_AGG_EXTENDED_STATS) {  // InternalExtendedStats.getVariance / getStdDeviationBound
                const double var = (sq - ((sum * sum) / (double)cnt)) / (double)cnt;
                const double sd = std::sqrt(var);
                j.raw(","); j.key("sum_of_squares"); j.opt(c, sq);
                j.raw(","); j.key("variance"); j.opt(c, var);
                j.raw(","); j.key("std_deviation"); j.opt(c, sd);
                j.raw(","); j.key("std_deviation_bounds"); j.raw("{");
                j.key("upper"); j.opt(c, avg + (sd * a.sigma)); j.raw(",");
                j.key("lower"); j.opt(c, avg - (sd * a.sigma)); j.raw("}");
            }
            j.raw(","); j.key("_internal"); j.raw("{");
            j.key("count"); j.i64(cnt); j.raw(",");
            j.key("sum"); j.dbl(sum); j.raw(",");
            j.key("min"); j.dbl(mn); j.raw(",");
            j.key("max"); j.dbl(mx);
            if (a.type == ESGPU_AGG_EXTENDED_STATS) { j.raw(","); j.key("sum_of_squares"); j.dbl(sq); }
            j.raw("}");
            break;
        }
        case ESGPU_AGG_CARDINALITY: {
            const bool present = a.hll_present[i];
            const int mode = a.hll_mode[i];
            j.key("value"); j.i64(hll_cardinality(a.precision, present, mode, a.regs[i].data(), a.lc[i].size()));
            j.raw(","); j.key("_internal"); j.raw("{");
            j.key("present"); j.i64(present ? 1 : 0);
            if (present) {
                char b[32];
                j.raw(","); j.key("precision"); j.i64(a.precision);
                j.raw(","); j.key("mode"); j.str(mode ? "hll" : "lc");
                if (mode) {
                    snprintf(b, sizeof b, "%016llx", (unsigned long long)fnv1a(a.regs[i].data(), a.regs[i].size()));
                    j.raw(","); j.key("registers_fnv1a64"); j.str(b);
                } else {
                    j.raw(","); j.key("lc_size"); j.i64((int64_t)a.lc[i].size());
                    std::vector<uint32_t> u(a.lc[i].begin(), a.lc[i].end());  // fingerprint of the set (order-free)
                    std::sort(u.begin(), u.end());
                    snprintf(b, sizeof b, "%016llx", (unsigned long long)fnv1a((const uint8_t*)u.data(), u.size() * 4));
                    j.raw(","); j.key("lc_fnv1a64"); j.str(b);
                }
            }
            j.raw("}");
            break;
        }
    }
    j.raw("}");
}
}  // namespace

std::string to_json(const std::vector<Block>& aggs) {
    J j;
    j.raw("{");
    for (size_t i = 0; i < aggs.size(); ++i) {
        if (i) j.raw(",");
        j.key(aggs[i].name);
        write_instance(j, aggs[i], 0);
    }
    j.raw("}");
    return j.s;
}

// ------------------------------------------------------------------------------------------------------------
// XContent: the REST response body of the aggregations as Elasticsearch renders it (Jackson, compact), field by
// field after each class's doXContentBody -- InternalTerms/StringTerms (A/bucket/terms/InternalTerms.java:220-229,
// StringTerms.java:138-148), InternalHistogram (A/bucket/histogram/InternalHistogram.java:152-173,526-541),
// InternalStats (A/metrics/stats/InternalStats.java:206-221), InternalExtendedStats (:192-213), InternalAvg (:109-115),
// InternalCardinality (:129-136), InternalSingleBucketAggregation (filter).  Numeric fields use the RAW value
// formatter (no *_as_string); date_histogram keys print with the date field's default printer
// (strict_date_optional_time: yyyy-MM-dd'T'HH:mm:ss.SSSZZ) in the request's time zone.
// ------------------------------------------------------------------------------------------------------------
namespace {
// Double.toString: java_double.hpp (JDK 8 FloatingDecimal)

// strict_date_optional_time printer in the zone of the table (offset offs[i] from UTC instant starts[i]; empty = UTC)
std::string es_date(int64_t ms, const std::vector<int64_t>& starts, const std::vector<int64_t>& offs) {
    int64_t off = 0;
    if (!offs.empty()) {
        size_t i = (size_t)(std::upper_bound(starts.begin() + 1, starts.end(), ms) - starts.begin());
        off = offs[i - 1];
    }
    const int64_t local = ms + off;
    const int64_t days = fdiv(local, kMsDay);
    const int64_t rem = local - days * kMsDay;
    int64_t y; int m, d;
    r_civil_from_days(days, &y, &m, &d);
    char b[64];
    int n = snprintf(b, sizeof b, "%04lld-%02d-%02dT%02d:%02d:%02d.%03d", (long long)y, m, d, (int)(rem / 3600000),
                     (int)(rem / 60000 % 60), (int)(rem / 1000 % 60), (int)(rem % 1000));
    if (off == 0) {
        snprintf(b + n, sizeof b - n, "Z");
    } else {
        const int64_t a = off < 0 ? -off : off;
        snprintf(b + n, sizeof b - n, "%c%02d:%02d", off < 0 ? '-' : '+', (int)(a / 3600000), (int)(a / 60000 % 60));
    }
    return b;
}

struct X {
    std::string s;
    void raw(const char* t) { s += t; }
    void str(const char* p, size_t n) {  // Jackson: short escapes for \b \t \n \f \r, \uXXXX for other controls
        s += '"';
        for (size_t i = 0; i < n; ++i) {
            const unsigned char c = (unsigned char)p[i];
            switch (c) {
                case '"': s += "\\\""; break;
                case '\\': s += "\\\\"; break;
                case '\b': s += "\\b"; break;
                case '\t': s += "\\t"; break;
                case '\n': s += "\\n"; break;
                case '\f': s += "\\f"; break;
                case '\r': s += "\\r"; break;
                default:
                    if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04X", c); s += b; }
                    else s += (char)c;
            }
        }
        s += '"';
    }
    void str(const std::string& v) { str(v.data(), v.size()); }
    void key(const std::string& k) { str(k); s += ':'; }
    void i64(int64_t v) { s += std::to_string(v); }
    void dbl(double v) { s += java_double(v); }
    void opt(bool c, double v) { if (c) dbl(v); else raw("null"); }
};

void x_instance(X& x, const Block& a, uint64_t i);

void x_subs(X& x, const Block& a, uint64_t k) {
    for (const Block& sb : a.subs) {
        x.raw(",");
        x.key(sb.name);
        x_instance(x, sb, k);
    }
}

void x_instance(X& x, const Block& a, uint64_t i) {
    x.raw("{");
    switch (a.type) {
        case ESGPU_AGG_TERMS:
            x.key("doc_count_error_upper_bound"); x.i64(a.doc_count_error[i]); x.raw(",");
            x.key("sum_other_doc_count"); x.i64(a.other_doc_count[i]); x.raw(",");
            x.key("buckets"); x.raw("[");
            for (uint64_t k = a.boff[i]; k < a.boff[i + 1]; ++k) {
                if (k != a.boff[i]) x.raw(",");
                x.raw("{"); x.key("key"); x.str(a.term_pool.data() + a.term_off[k], a.term_off[k + 1] - a.term_off[k]); x.raw(",");
                x.key("doc_count"); x.i64(a.bcount[k]);
                if (a.show_err) { x.raw(","); x.key("doc_count_error_upper_bound"); x.i64(a.berr[k]); }
                x_subs(x, a, k);
                x.raw("}");
            }
            x.raw("]");
            break;
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM: {
            const bool date = a.type == ESGPU_AGG_DATE_HISTOGRAM;
            x.key("buckets"); x.raw(a.keyed ? "{" : "[");
            for (uint64_t k = a.boff[i]; k < a.boff[i + 1]; ++k) {
                if (k != a.boff[i]) x.raw(",");
                const std::string ks = date ? es_date(a.key[k], a.tz_starts, a.tz_offs) : std::string();
                if (a.keyed) x.key(date ? ks : std::to_string(a.key[k]));
                x.raw("{");
                if (date) { x.key("key_as_string"); x.str(ks); x.raw(","); }
                x.key("key"); x.i64(a.key[k]); x.raw(",");
                x.key("doc_count"); x.i64(a.bcount[k]);
                x_subs(x, a, k);
                x.raw("}");
            }
            x.raw(a.keyed ? "}" : "]");
            break;
        }
        case ESGPU_AGG_FILTER:
            x.key("doc_count"); x.i64(a.count[i]);
            x_subs(x, a, i);
            break;
        case ESGPU_AGG_AVG:
            x.key("value"); x.opt(a.count[i] != 0, a.sum[i] / (double)a.count[i]);
            break;
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS: {
            const int64_t cnt = a.count[i];
            const double sum = a.sum[i], sq = a.sumsq[i];
            const bool c = cnt != 0;
            const double avg = sum / (double)cnt;
            x.key("count"); x.i64(cnt); x.raw(",");
            x.key("min"); x.opt(c, a.min[i]); x.raw(",");
            x.key("max"); x.opt(c, a.max[i]); x.raw(",");
            x.key("avg"); x.opt(c, avg); x.raw(",");
            x.key("sum"); x.opt(c, sum);
            if (a.type == ESGPU_AGG_EXTENDED_STATS) {
                const double var = (sq - ((sum * sum) / (double)cnt)) / (double)cnt;
                const double sd = std::sqrt(var);
                x.raw(","); x.key("sum_of_squares"); x.opt(c, sq);
                x.raw(","); x.key("variance"); x.opt(c, var);
                x.raw(","); x.key("std_deviation"); x.opt(c, sd);
                x.raw(","); x.key("std_deviation_bounds"); x.raw("{");
                x.key("upper"); x.opt(c, avg + (sd * a.sigma)); x.raw(",");
                x.key("lower"); x.opt(c, avg - (sd * a.sigma)); x.raw("}");
            }
            break;
        }
        case ESGPU_AGG_CARDINALITY:
            x.key("value"); x.i64(hll_cardinality(a.precision, a.hll_present[i], a.hll_mode[i], a.regs[i].data(), a.lc[i].size()));
            break;
    }
    x.raw("}");
}
}  // namespace

std::string to_xcontent(const std::vector<Block>& aggs) {
    X x;
    x.raw("{");
    for (size_t i = 0; i < aggs.size(); ++i) {
        if (i) x.raw(",");
        x.key(aggs[i].name);
        x_instance(x, aggs[i], 0);
    }
    x.raw("}");
    return x.s;
}

// ------------------------------------------------------------------------------------------------------------
// Elasticsearch's transport bytes: InternalAggregations.writeTo(StreamOutput) (A/InternalAggregations.java:215-222)
// ------------------------------------------------------------------------------------------------------------
namespace {
struct JavaOut {  // org.elasticsearch.common.io.stream.StreamOutput encodings (C/common/io/stream/StreamOutput.java)
    std::string& o;
    void byte(uint8_t b) { o.push_back((char)b); }
    void boolean(bool b) { byte(b ? 1 : 0); }                        // :263-265
    void vint(int32_t i) {                                           // :157-163 (i >>>= 7)
        uint32_t u = (uint32_t)i;
        while (u & ~0x7Fu) { byte((uint8_t)((u & 0x7F) | 0x80)); u >>= 7; }
        byte((uint8_t)u);
    }
    void vlong(int64_t i) {                                          // :178-185
        uint64_t u = (uint64_t)i;
        while (u & ~0x7Full) { byte((uint8_t)((u & 0x7F) | 0x80)); u >>= 7; }
        byte((uint8_t)u);
    }
    void i32(int32_t i) { for (int s = 24; s >= 0; s -= 8) byte((uint8_t)((uint32_t)i >> s)); }  // :144-149
    void i64(int64_t i) { i32((int32_t)(i >> 32)); i32((int32_t)i); }                           // :168-171
    void f64(double v) {                                             // :251-253, Double.doubleToLongBits
        uint64_t b;
        std::memcpy(&b, &v, 8);
        if (v != v) b = 0x7ff8000000000000ULL;
        i64((int64_t)b);
    }
    void bytes_ref(const char* p, size_t n) { vint((int32_t)n); o.append(p, n); }  // writeBytesRef / writeBytesReference
    // writeString (:228-245): the String's UTF-16 code units, each in 1-3 bytes (modified UTF-8; surrogates separately)
    void str(const std::string& utf8) {
        std::vector<uint16_t> u;
        for (size_t i = 0; i < utf8.size();) {
            const uint8_t c = (uint8_t)utf8[i];
            uint32_t cp = c, len = 1;
            if (c >= 0xF0) { cp = c & 0x07; len = 4; }
            else if (c >= 0xE0) { cp = c & 0x0F; len = 3; }
            else if (c >= 0xC0) { cp = c & 0x1F; len = 2; }
            if (i + len > utf8.size()) { len = 1; cp = c; }
            for (uint32_t k = 1; k < len; ++k) cp = (cp << 6) | ((uint8_t)utf8[i + k] & 0x3F);
            i += len;
            if (cp >= 0x10000) {
                cp -= 0x10000;
                u.push_back((uint16_t)(0xD800 + (cp >> 10)));
                u.push_back((uint16_t)(0xDC00 + (cp & 0x3FF)));
            } else {
                u.push_back((uint16_t)cp);
            }
        }
        vint((int32_t)u.size());
        for (uint16_t c : u) {
            if (c <= 0x007F) byte((uint8_t)c);
            else if (c > 0x07FF) { byte((uint8_t)(0xE0 | ((c >> 12) & 0x0F))); byte((uint8_t)(0x80 | ((c >> 6) & 0x3F))); byte((uint8_t)(0x80 | (c & 0x3F))); }
            else { byte((uint8_t)(0xC0 | ((c >> 6) & 0x1F))); byte((uint8_t)(0x80 | (c & 0x3F))); }
        }
    }
    void size(int32_t s) { vint(s == INT32_MAX ? 0 : s); }  // InternalAggregation.writeSize (A/InternalAggregation.java:181-186)
};

const char* stream_type(int32_t type) {  // InternalAggregation.Type stream names (each class's TYPE)
    switch (type) {
        case ESGPU_AGG_TERMS: return "sterms";               // StringTerms.java:43
        case ESGPU_AGG_HISTOGRAM: return "histo";            // InternalHistogram.java:55
        case ESGPU_AGG_DATE_HISTOGRAM: return "dhisto";      // InternalDateHistogram.java:33
        case ESGPU_AGG_STATS: return "stats";                // InternalStats.java:41
        case ESGPU_AGG_EXTENDED_STATS: return "estats";      // InternalExtendedStats.java:41
        case ESGPU_AGG_AVG: return "avg";                    // InternalAvg.java:40
        case ESGPU_AGG_CARDINALITY: return "cardinality";    // InternalCardinality.java:39
        case ESGPU_AGG_FILTER: return "filter";              // InternalFilter.java:36
    }
    throw std::invalid_argument("aggregation type without a stream");
}

// ValueFormatterStreams.writeOptional (A/support/format/ValueFormatterStreams.java:54-64) of the field's formatter;
// ValuesSourceParser.resolveFormat never leaves it null for a field (RAW at worst, ValuesSourceParser.java:233-257)
void write_formatter(JavaOut& w, const Block& a) {
    w.boolean(true);
    switch (a.value_format) {
        case ESGPU_FORMAT_DATE_TIME: w.byte(2); w.str(a.format); w.str(a.time_zone); break;  // ValueFormatter.java:155-158
        case ESGPU_FORMAT_NUMBER: w.byte(4); w.str(a.format); break;                       // ValueFormatter.java:208-211
        default: w.byte(1); break;                                                         // Raw: no payload (:93-94)
    }
}

// Rounding.Streams.write (C/common/rounding/Rounding.java:229-234) of the histogram's rounding:
// HistogramParser.java:128-131 (Interval, OffsetRounding) and TimeZoneRounding.Builder.build (TimeZoneRounding.java:84-98)
void write_rounding(JavaOut& w, const Block& a) {
    if (a.offset != 0) { w.byte(8); }  // OffsetRounding: the wrapped rounding, then the offset (Rounding.java:223-226)
    if (a.type == ESGPU_AGG_HISTOGRAM) {
        w.byte(0);                     // Rounding.Interval (:126-128)
        w.vlong(a.interval);
    } else if (a.date_unit != ESGPU_UNIT_NONE) {
        w.byte(1);                     // TimeUnitRounding: DateTimeUnit id (DateTimeUnit.java:30-37) + zone id (:156-159)
        w.byte((uint8_t)a.date_unit);
        w.str(a.time_zone);
    } else {
        w.byte(2);                     // TimeIntervalRounding: vLong interval + zone id (:213-216)
        w.vlong(a.interval);
        w.str(a.time_zone);
    }
    if (a.offset != 0) w.i64(a.offset);
}

// InternalOrder.Streams.writeOrder (A/bucket/terms/InternalOrder.java:289-306) of the order TermsParser builds: a single
// term order as itself, every other order as CompoundOrder(order, _term asc) (TermsParser.java:57-67, :233-241)
void write_terms_order(JavaOut& w, const Block& a) {
    switch (a.order) {
        case ESGPU_ORDER_TERM_ASC: w.byte(4); return;
        case ESGPU_ORDER_TERM_DESC: w.byte(3); return;
    }
    w.byte(0xFF);  // CompoundOrder.ID = -1
    w.vint(2);
    switch (a.order) {
        case ESGPU_ORDER_COUNT_DESC: w.byte(1); break;
        case ESGPU_ORDER_COUNT_ASC: w.byte(2); break;
        case ESGPU_ORDER_AGG_ASC:
        case ESGPU_ORDER_AGG_DESC:  // InternalOrder.Aggregation: id 0, asc, AggregationPath.toString
            w.byte(0);
            w.boolean(a.order == ESGPU_ORDER_AGG_ASC);
            w.str(a.order_path);
            break;
        default: throw std::invalid_argument("unknown terms order");
    }
    w.byte(4);  // _term asc tie-break
}

uint8_t hist_order_id(int32_t order) {  // Histogram.Order ids (A/bucket/histogram/Histogram.java:51-77)
    switch (order) {
        case ESGPU_ORDER_KEY_ASC: return 1;
        case ESGPU_ORDER_KEY_DESC: return 2;
        case ESGPU_ORDER_HCOUNT_ASC: return 3;
        case ESGPU_ORDER_HCOUNT_DESC: return 4;
    }
    throw std::invalid_argument("unknown histogram order");
}

void es_list(JavaOut& w, const std::vector<Block>& l, uint64_t i);

// InternalAggregation.writeTo (A/InternalAggregation.java:212-221) of instance i, then the class's doWriteTo
void es_instance(JavaOut& w, const Block& a, uint64_t i) {
    w.str(a.name);
    w.byte(0xFF);  // writeGenericValue(null metaData)
    w.vint(0);     // no pipeline aggregators
    switch (a.type) {
        case ESGPU_AGG_TERMS: {  // StringTerms.doWriteTo (:205-217), Bucket.writeTo (:128-136)
            w.i64(a.doc_count_error[i]);
            write_terms_order(w, a);
            w.size(a.required_size);
            w.size(a.shard_size);
            w.boolean(a.show_err != 0);
            w.vlong(a.min_doc_count);
            w.vlong(a.other_doc_count[i]);
            const uint64_t b0 = a.boff[i], b1 = a.boff[i + 1];
            w.vint((int32_t)(b1 - b0));
            for (uint64_t b = b0; b < b1; ++b) {
                w.bytes_ref(a.term_pool.data() + a.term_off[b], a.term_off[b + 1] - a.term_off[b]);
                w.vlong(a.bcount[b]);
                if (a.show_err) w.i64(a.berr[b]);
                es_list(w, a.subs, b);
            }
            break;
        }
        case ESGPU_AGG_HISTOGRAM:
        case ESGPU_AGG_DATE_HISTOGRAM: {  // InternalHistogram.doWriteTo (:510-523), Bucket.writeTo (:183-187)
            w.str(a.type == ESGPU_AGG_DATE_HISTOGRAM ? "date_histogram" : "histogram");  // factory.type()
            w.byte(hist_order_id(a.order));
            w.vlong(a.min_doc_count);
            if (a.min_doc_count == 0) {  // EmptyBucketInfo.writeTo (:223-230)
                write_rounding(w, a);
                es_list(w, a.empty_subs, 0);
                const bool bounds = a.has_bmin || a.has_bmax;
                w.boolean(bounds);
                if (bounds) {  // ExtendedBounds.writeTo (A/bucket/histogram/ExtendedBounds.java:67-80)
                    w.boolean(a.has_bmin);
                    if (a.has_bmin) w.i64(a.bmin);
                    w.boolean(a.has_bmax);
                    if (a.has_bmax) w.i64(a.bmax);
                }
            }
            write_formatter(w, a);
            w.boolean(a.keyed != 0);
            const uint64_t b0 = a.boff[i], b1 = a.boff[i + 1];
            w.vint((int32_t)(b1 - b0));
            for (uint64_t b = b0; b < b1; ++b) {
                w.i64(a.key[b]);
                w.vlong(a.bcount[b]);
                es_list(w, a.subs, b);
            }
            break;
        }
        case ESGPU_AGG_STATS:
        case ESGPU_AGG_EXTENDED_STATS:  // InternalStats.doWriteTo (:182-189) + InternalExtendedStats.writeOtherStatsTo (:169-174)
            write_formatter(w, a);
            w.vlong(a.count[i]);
            w.f64(a.min[i]);
            w.f64(a.max[i]);
            w.f64(a.sum[i]);
            if (a.type == ESGPU_AGG_EXTENDED_STATS) {
                w.f64(a.sumsq[i]);
                w.f64(a.sigma);
            }
            break;
        case ESGPU_AGG_AVG:  // InternalAvg.doWriteTo (:102-106)
            write_formatter(w, a);
            w.f64(a.sum[i]);
            w.vlong(a.count[i]);
            break;
        case ESGPU_AGG_CARDINALITY:  // InternalCardinality.doWriteTo (:92-100), HyperLogLogPlusPlus.writeTo (:519-535)
            write_formatter(w, a);
            w.boolean(a.hll_present[i] != 0);
            if (a.hll_present[i]) {
                w.vint(a.precision);
                if (a.hll_mode[i] == 0) {  // LINEAR_COUNTING = false
                    w.boolean(false);
                    w.vlong((int64_t)a.lc[i].size());
                    for (uint32_t e : a.lc[i]) w.i32((int32_t)e);
                } else {
                    w.boolean(true);
                    const std::vector<uint8_t>& r = a.regs[i];
                    if (r.size() != ((size_t)1 << a.precision)) throw std::runtime_error("register array size");
                    w.o.append((const char*)r.data(), r.size());
                }
            }
            break;
        case ESGPU_AGG_FILTER:  // InternalSingleBucketAggregation.doWriteTo (:124-127)
            w.vlong(a.count[i]);
            es_list(w, a.subs, i);
            break;
        default: throw std::invalid_argument("aggregation type without a stream");
    }
}

// InternalAggregations.writeTo: count, then per aggregation its stream type and writeTo
void es_list(JavaOut& w, const std::vector<Block>& l, uint64_t i) {
    w.vint((int32_t)l.size());
    for (const Block& a : l) {
        const char* t = stream_type(a.type);
        w.bytes_ref(t, std::strlen(t));
        es_instance(w, a, i);
    }
}
}  // namespace

void to_es_stream(const std::vector<Block>& aggs, std::string& out) {
    out.clear();
    JavaOut w{out};
    es_list(w, aggs, 0);
}

// ------------------------------------------------------------------------------------------------------------
// stream format (AggregationStreams analogue): little-endian, versioned, one record per block
// ------------------------------------------------------------------------------------------------------------
namespace {
struct W {
    std::string& o;
    template <class T> void pod(const T& v) { o.append((const char*)&v, sizeof v); }
    void str(const std::string& s) { pod<uint64_t>(s.size()); o.append(s); }
    template <class T> void vec(const std::vector<T>& v) {
        pod<uint64_t>(v.size());
        if (!v.empty()) o.append((const char*)v.data(), v.size() * sizeof(T));
    }
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
        const uint64_t len = pod<uint64_t>();
        if (len > n - i) throw std::runtime_error("truncated stream");
        std::string s((const char*)p + i, (size_t)len);
        i += len;
        return s;
    }
    template <class T> void vec(std::vector<T>& v) {
        const uint64_t len = pod<uint64_t>();
        if (len > (n - i) / sizeof(T)) throw std::runtime_error("truncated stream");
        v.resize(len);
        if (len) std::memcpy(v.data(), p + i, len * sizeof(T));
        i += len * sizeof(T);
    }
};
void w_blocks(W& w, const std::vector<Block>& l);
void w_block(W& w, const Block& a) {
    w.pod(a.type); w.pod(a.order); w.str(a.name);
    w.pod(a.required_size); w.pod(a.shard_size); w.pod(a.min_doc_count); w.pod(a.show_err); w.pod(a.keyed);
    w.pod<uint8_t>(a.has_empty_info); w.pod(a.date_unit); w.pod(a.interval); w.pod(a.offset);
    w.vec(a.tz_starts); w.vec(a.tz_offs);
    w.pod<uint8_t>(a.has_bmin); w.pod<uint8_t>(a.has_bmax); w.pod(a.bmin); w.pod(a.bmax);
    w.pod(a.sigma); w.pod(a.precision); w.str(a.order_path);
    w.str(a.time_zone); w.pod(a.value_format); w.str(a.format); w.pod(a.n);
    w.vec(a.doc_count_error); w.vec(a.other_doc_count); w.vec(a.boff); w.vec(a.key); w.vec(a.term_off);
    w.str(a.term_pool); w.vec(a.bcount); w.vec(a.berr);
    w_blocks(w, a.subs);
    w_blocks(w, a.empty_subs);
    w.vec(a.count); w.vec(a.sum); w.vec(a.min); w.vec(a.max); w.vec(a.sumsq);
    w.vec(a.hll_present); w.vec(a.hll_mode);
    w.pod<uint64_t>(a.regs.size());
    for (auto& r : a.regs) w.vec(r);
    w.pod<uint64_t>(a.lc.size());
    for (auto& l : a.lc) w.vec(l);
}
void w_blocks(W& w, const std::vector<Block>& l) {
    w.pod<uint32_t>((uint32_t)l.size());
    for (const Block& a : l) w_block(w, a);
}
void r_blocks(R& r, std::vector<Block>& l, int depth);
void r_block(R& r, Block& a, int depth) {
    if (depth > 64) throw std::runtime_error("stream nests too deep");
    a.type = r.pod<int32_t>(); a.order = r.pod<int32_t>(); a.name = r.str();
    a.required_size = r.pod<int32_t>(); a.shard_size = r.pod<int32_t>(); a.min_doc_count = r.pod<int64_t>();
    a.show_err = r.pod<int32_t>(); a.keyed = r.pod<int32_t>();
    a.has_empty_info = r.pod<uint8_t>(); a.date_unit = r.pod<int32_t>(); a.interval = r.pod<int64_t>();
    a.offset = r.pod<int64_t>();
    r.vec(a.tz_starts); r.vec(a.tz_offs);
    if (a.tz_starts.size() != a.tz_offs.size()) throw std::runtime_error("bad time zone table");
    a.has_bmin = r.pod<uint8_t>(); a.has_bmax = r.pod<uint8_t>(); a.bmin = r.pod<int64_t>(); a.bmax = r.pod<int64_t>();
    a.sigma = r.pod<double>(); a.precision = r.pod<int32_t>(); a.order_path = r.str();
    a.time_zone = r.str(); a.value_format = r.pod<int32_t>(); a.format = r.str(); a.n = r.pod<uint64_t>();
    r.vec(a.doc_count_error); r.vec(a.other_doc_count); r.vec(a.boff); r.vec(a.key); r.vec(a.term_off);
    a.term_pool = r.str(); r.vec(a.bcount); r.vec(a.berr);
    r_blocks(r, a.subs, depth + 1);
    r_blocks(r, a.empty_subs, depth + 1);
    r.vec(a.count); r.vec(a.sum); r.vec(a.min); r.vec(a.max); r.vec(a.sumsq);
    r.vec(a.hll_present); r.vec(a.hll_mode);
    a.regs.resize(r.pod<uint64_t>());
    for (auto& x : a.regs) r.vec(x);
    a.lc.resize(r.pod<uint64_t>());
    for (auto& x : a.lc) r.vec(x);
    // structural validation: a corrupt record must not produce out-of-bounds views
    const bool bucket = a.is_bucket();
    if (bucket) {
        const uint64_t nb = a.boff.empty() ? 0 : a.boff.back();
        if (a.boff.size() != a.n + 1 || a.key.size() != nb || a.bcount.size() != nb || a.berr.size() != nb ||
            a.term_off.size() != nb + 1 || a.doc_count_error.size() != a.n || a.other_doc_count.size() != a.n ||
            (nb && a.term_off.back() != a.term_pool.size()))
            throw std::runtime_error("inconsistent bucket block");
        for (size_t k = 0; k + 1 < a.boff.size(); ++k) if (a.boff[k] > a.boff[k + 1]) throw std::runtime_error("bad offsets");
        for (size_t k = 0; k + 1 < a.term_off.size(); ++k) if (a.term_off[k] > a.term_off[k + 1]) throw std::runtime_error("bad offsets");
        for (const Block& s : a.subs) if (s.n != nb) throw std::runtime_error("sub-aggregation instance count mismatch");
        if (a.has_empty_info && a.empty_subs.size() != a.subs.size()) throw std::runtime_error("missing empty-bucket prototypes");
        for (size_t j = 0; j < a.empty_subs.size(); ++j)
            if (a.empty_subs[j].n != 1 || a.empty_subs[j].type != a.subs[j].type) throw std::runtime_error("bad empty-bucket prototype");
    } else if (a.type == ESGPU_AGG_FILTER) {
        if (a.count.size() != a.n) throw std::runtime_error("inconsistent filter block");
        for (const Block& s : a.subs) if (s.n != a.n) throw std::runtime_error("sub-aggregation instance count mismatch");
    } else if (a.type == ESGPU_AGG_CARDINALITY) {
        if (a.hll_present.size() != a.n || a.hll_mode.size() != a.n || a.regs.size() != a.n || a.lc.size() != a.n)
            throw std::runtime_error("inconsistent cardinality block");
        if (a.precision < 4 || a.precision > 18) throw std::runtime_error("bad precision");
        // every value the reduce decodes must stay in range: unflagged encoded hashes carry a 25-bit index
        // (dec_index < 2^p), flagged ones a run length of at most 64 - 25 + 1, registers at most 64 - p + 1
        const uint32_t max_rl = (uint32_t)(64 - a.precision + 1);
        for (uint64_t i = 0; i < a.n; ++i) {
            if (a.hll_present[i] && a.hll_mode[i] && a.regs[i].size() != ((size_t)1 << a.precision))
                throw std::runtime_error("bad register array");
            for (uint8_t r : a.regs[i]) if (r > max_rl) throw std::runtime_error("bad register value");
            for (uint32_t e : a.lc[i]) {
                if (e & 1) { if (((e >> 1) & 0x3F) > 64 - kP2 + 1) throw std::runtime_error("bad encoded hash"); }
                else if (e >= (1u << (kP2 + 1))) throw std::runtime_error("bad encoded hash");
            }
        }
    } else if (a.count.size() != a.n || a.sum.size() != a.n || a.min.size() != a.n || a.max.size() != a.n ||
               a.sumsq.size() != a.n) {
        throw std::runtime_error("inconsistent metric block");
    }
}
void r_blocks(R& r, std::vector<Block>& l, int depth) {
    const uint32_t n = r.pod<uint32_t>();
    if (n > 4096) throw std::runtime_error("too many aggregations");
    l.resize(n);
    for (Block& a : l) r_block(r, a, depth);
}
const uint32_t kStreamMagic = 0x45534750;  // "ESGP"
const uint32_t kStreamVersion = 5;
}  // namespace

void serialize(const std::vector<Block>& aggs, std::string& out) {
    out.clear();
    W w{out};
    w.pod(kStreamMagic);
    w.pod(kStreamVersion);
    w_blocks(w, aggs);
}

bool deserialize(const uint8_t* p, size_t n, std::vector<Block>& out) {
    R r{p, n};
    if (n < 8 || r.pod<uint32_t>() != kStreamMagic) return false;
    if (r.pod<uint32_t>() != kStreamVersion) return false;
    r_blocks(r, out, 0);
    for (const Block& b : out) if (b.n != 1) throw std::runtime_error("top-level aggregations carry one instance");
    return true;
}

// ------------------------------------------------------------------------------------------------------------
// C view export
// ------------------------------------------------------------------------------------------------------------
ResultHolder* holder_of(const esgpu_result* r) { return reinterpret_cast<ResultHolder*>(const_cast<esgpu_result*>(r)); }

namespace {
template <class T> const T* ptr(const std::vector<T>& v) { return v.empty() ? nullptr : v.data(); }

const esgpu_agg_block* export_blocks(ResultHolder& h, const std::vector<Block>& src);

void export_block(ResultHolder& h, const Block& a, esgpu_agg_block& o) {
    std::memset(&o, 0, sizeof o);
    o.type = a.type;
    o.order = a.order;
    o.name = a.name.c_str();
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
    o.sigma = a.sigma;
    o.precision = a.precision;
    o.order_path = a.order_path.c_str();
    o.time_zone = a.time_zone.c_str();
    o.value_format = a.value_format;
    o.format = a.format.c_str();
    o.nsubs = (int32_t)a.subs.size();
    o.n_instances = a.n;
    o.doc_count_error = ptr(a.doc_count_error);
    o.other_doc_count = ptr(a.other_doc_count);
    o.bucket_offsets = ptr(a.boff);
    o.n_buckets = a.nbuckets();
    o.keys = ptr(a.key);
    o.term_offsets = ptr(a.term_off);
    o.term_bytes = (const uint8_t*)a.term_pool.data();
    o.doc_counts = ptr(a.bcount);
    o.bucket_doc_count_errors = ptr(a.berr);
    o.subs = export_blocks(h, a.subs);
    o.empty_subs = export_blocks(h, a.empty_subs);
    o.count = ptr(a.count);
    o.sum = ptr(a.sum);
    o.min = ptr(a.min);
    o.max = ptr(a.max);
    o.sum_of_squares = ptr(a.sumsq);
    if (a.type == ESGPU_AGG_CARDINALITY && a.n) {
        std::unique_ptr<int32_t[]> pres(new int32_t[a.n]);
        std::unique_ptr<const uint8_t*[]> rp(new const uint8_t*[a.n]);
        std::unique_ptr<const uint32_t*[]> lp(new const uint32_t*[a.n]);
        std::unique_ptr<int64_t[]> ls(new int64_t[a.n]);
        for (uint64_t i = 0; i < a.n; ++i) {
            pres[i] = a.hll_present[i];
            rp[i] = a.regs[i].empty() ? nullptr : a.regs[i].data();
            lp[i] = a.lc[i].empty() ? nullptr : a.lc[i].data();
            ls[i] = (int64_t)a.lc[i].size();
        }
        o.hll_present = pres.get();
        o.hll_mode = ptr(a.hll_mode);
        o.registers = rp.get();
        o.lc_hashes = lp.get();
        o.lc_sizes = ls.get();
        h.present32.push_back(std::move(pres));
        h.reg_ptrs.push_back(std::move(rp));
        h.lc_ptrs.push_back(std::move(lp));
        h.lc_sizes.push_back(std::move(ls));
    }
}

const esgpu_agg_block* export_blocks(ResultHolder& h, const std::vector<Block>& src) {
    if (src.empty()) return nullptr;
    std::unique_ptr<esgpu_agg_block[]> blk(new esgpu_agg_block[src.size()]);
    for (size_t i = 0; i < src.size(); ++i) export_block(h, src[i], blk[i]);
    const esgpu_agg_block* p = blk.get();
    h.views.push_back(std::move(blk));
    return p;
}
}  // namespace

void ResultHolder::export_view() {
    views.clear();
    reg_ptrs.clear();
    lc_ptrs.clear();
    lc_sizes.clear();
    present32.clear();
    std::memset(&pub, 0, sizeof pub);
    pub.aggs = export_blocks(*this, aggs);
    pub.naggs = (int32_t)aggs.size();
}


// ------------------------------------------------------------------------------------------------------------
// reduce across ranks: all-reduce for fixed-shape partials, all-gather of shard records for the rest
// ------------------------------------------------------------------------------------------------------------
namespace {

// order-preserving image of a double (Java Math.min / Math.max order: -0.0 < +0.0); NaN wins both reductions
inline uint64_t enc_dbl(double x) {
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
inline double dec_dbl(uint64_t e) {
    const uint64_t b = (e >> 63) ? (e & 0x7FFFFFFFFFFFFFFFULL) : ~e;
    double x;
    std::memcpy(&x, &b, 8);
    return x;
}
inline uint64_t enc_min(double x) { return x != x ? 0 : enc_dbl(x); }
inline uint64_t enc_max(double x) { return x != x ? ~0ULL : enc_dbl(x); }
inline double dec_min(uint64_t e) { return e == 0 ? NAN : dec_dbl(e); }
inline double dec_max(uint64_t e) { return e == ~0ULL ? NAN : dec_dbl(e); }

bool is_numeric_metric(int t) { return t == ESGPU_AGG_STATS || t == ESGPU_AGG_EXTENDED_STATS || t == ESGPU_AGG_AVG; }

// a top-level aggregation whose shard partials have a fixed shape once the bucket keys are agreed on
bool fixed_shape(const Block& b) {
    if (is_numeric_metric(b.type) || b.type == ESGPU_AGG_CARDINALITY) return true;
    if (b.type == ESGPU_AGG_HISTOGRAM || b.type == ESGPU_AGG_DATE_HISTOGRAM) {
        for (const Block& s : b.subs) if (!is_numeric_metric(s.type)) return false;
        return true;
    }
    return false;
}

// all-gather of one variable-size byte message per rank: sizes first, then padded records
std::vector<std::string> gather_messages(Collective& c, const std::string& mine) {
    std::vector<uint64_t> sizes(c.nranks);
    const uint64_t my = mine.size();
    c.allgather(&my, sizes.data(), 8);
    const uint64_t rec = (std::max<uint64_t>(*std::max_element(sizes.begin(), sizes.end()), 8) + 15) & ~15ull;
    std::string padded(mine);
    padded.resize(rec, '\0');
    std::string all((size_t)(rec * c.nranks), '\0');
    c.allgather(padded.data(), &all[0], rec);
    std::vector<std::string> out(c.nranks);
    for (int r = 0; r < c.nranks; ++r) out[r] = all.substr((size_t)(rec * r), (size_t)sizes[r]);
    return out;
}

std::string pack_lists(const std::vector<std::vector<Block>>& lists) {
    std::string out;
    const uint32_t n = (uint32_t)lists.size();
    out.append((const char*)&n, 4);
    for (const auto& l : lists) {
        std::string rec;
        serialize(l, rec);
        const uint64_t len = rec.size();
        out.append((const char*)&len, 8);
        out += rec;
    }
    return out;
}

void unpack_lists(const std::string& msg, std::vector<std::vector<Block>>& out) {
    size_t i = 0;
    auto need = [&](size_t k) { if (i + k > msg.size()) throw std::runtime_error("corrupt shard message"); };
    need(4);
    uint32_t n;
    std::memcpy(&n, msg.data(), 4);
    i = 4;
    if (n > 65536) throw std::runtime_error("corrupt shard message");
    for (uint32_t k = 0; k < n; ++k) {
        need(8);
        uint64_t len;
        std::memcpy(&len, msg.data() + i, 8);
        i += 8;
        need((size_t)len);
        out.emplace_back();
        if (!deserialize((const uint8_t*)msg.data() + i, (size_t)len, out.back())) throw std::runtime_error("corrupt shard record");
        i += (size_t)len;
    }
}

// a one-instance terms result with its buckets' sub-aggregations as empty instances (the two-phase terms exchange)
Block terms_skeleton(const Block& t) {
    Block s = t.like();
    s.n = t.n;
    s.doc_count_error = t.doc_count_error;
    s.other_doc_count = t.other_doc_count;
    s.boff = t.boff;
    s.key = t.key;
    s.term_off = t.term_off;
    s.term_pool = t.term_pool;
    s.bcount = t.bcount;
    s.berr = t.berr;
    for (Block& sub : s.subs)
        for (uint64_t k = 0; k < t.nbuckets(); ++k) sub.append_empty();
    return s;
}

// the shard's terms result with the sub-aggregations of the buckets whose term is not in `keep` emptied
Block terms_pruned(const Block& t, const std::unordered_set<std::string>& keep) {
    Block s = terms_skeleton(t);
    for (Block& sub : s.subs) sub = sub.like();
    for (uint64_t k = 0; k < t.nbuckets(); ++k) {
        const bool kept = keep.count(t.term(k)) != 0;
        for (size_t j = 0; j < s.subs.size(); ++j) {
            if (kept) s.subs[j].append_instance(t.subs[j], k);
            else s.subs[j].append_empty();
        }
    }
    return s;
}

}  // namespace

std::vector<Block> reduce_across(Collective& c, const std::vector<const std::vector<Block>*>& locals, bool gather_only) {
    if (locals.empty()) throw std::invalid_argument("every rank reduces at least one local shard result");
    c.allreduce_bytes = c.allgather_bytes = 0;
    c.collectives = 0;
    c.exchange_ms = 0;
    const std::vector<Block>& first = *locals[0];
    const size_t naggs = first.size();
    for (auto* l : locals) {
        if (l->size() != naggs) throw std::invalid_argument("shard results have different aggregation lists");
        for (size_t a = 0; a < naggs; ++a)
            if (!same_shape((*l)[a], first[a])) throw std::invalid_argument("aggregation trees differ across shards");
    }
    std::vector<int> fixed, gathered;
    for (size_t a = 0; a < naggs; ++a) (!gather_only && fixed_shape(first[a]) ? fixed : gathered).push_back((int)a);
    std::vector<Block> out(naggs);

    // ---- all-gather path: every rank's shard records, reduced in global shard order (rank-major) ----
    if (!gathered.empty()) {
        // Top-level terms in a count or term order reduce their sub-aggregations only for the buckets that survive the
        // reduce (InternalTerms.doReduce: the top `size` merged buckets), and which survive depends on the terms-level
        // records alone.  So the records travel first without sub-aggregations (skeletons), every rank reduces them to
        // the same winners, and the shard records then carry the sub-aggregations of the winners' buckets only -- the
        // other buckets' sub-aggregations are empty instances the reduce never reads.  Same result, the sub-trees of
        // shard_size - size buckets per shard (70 of the north star's 80 at 8 shards) off the wire.
        std::vector<std::unordered_set<std::string>> winners(naggs);
        std::vector<char> two(naggs, 0);
        bool any_two = false;
        for (int a : gathered) {
            const Block& b = first[a];
            two[a] = c.nranks > 1 && b.type == ESGPU_AGG_TERMS && !b.subs.empty() && b.order != ESGPU_ORDER_AGG_ASC &&
                     b.order != ESGPU_ORDER_AGG_DESC;
            any_two |= two[a] != 0;
        }
        if (any_two) {
            std::vector<std::vector<Block>> skel;
            for (auto* l : locals) {
                skel.emplace_back();
                for (int a : gathered) if (two[a]) skel.back().push_back(terms_skeleton((*l)[a]));
            }
            std::vector<std::string> msgs = gather_messages(c, pack_lists(skel));
            std::vector<std::vector<Block>> all;
            for (const std::string& m : msgs) unpack_lists(m, all);
            std::vector<const std::vector<Block>*> lists;
            for (auto& s : all) lists.push_back(&s);
            const std::vector<Block> red = reduce_lists(lists);
            size_t q = 0;
            for (int a : gathered) {
                if (!two[a]) continue;
                const Block& r = red[q++];
                for (uint64_t b = 0; b < r.nbuckets(); ++b) winners[a].insert(r.term(b));
            }
        }
        std::vector<std::vector<Block>> mine;
        for (auto* l : locals) {
            mine.emplace_back();
            for (int a : gathered) mine.back().push_back(two[a] ? terms_pruned((*l)[a], winners[a]) : (*l)[a]);
        }
        std::vector<std::string> msgs = gather_messages(c, pack_lists(mine));
        std::vector<std::vector<Block>> shards;
        for (const std::string& m : msgs) unpack_lists(m, shards);
        std::vector<const std::vector<Block>*> lists;
        for (auto& s : shards) lists.push_back(&s);
        std::vector<Block> red = reduce_lists(lists);
        for (size_t k = 0; k < gathered.size(); ++k) out[gathered[k]] = std::move(red[k]);
    }

    // ---- fixed-shape path ----
    // (1) bucket keys of the top-level histograms: the union over every rank's shards (all-gather of the key lists)
    std::vector<int> hists, metrics, cards;
    for (int a : fixed) {
        const int t = first[a].type;
        if (t == ESGPU_AGG_CARDINALITY) cards.push_back(a);
        else if (t == ESGPU_AGG_HISTOGRAM || t == ESGPU_AGG_DATE_HISTOGRAM) hists.push_back(a);
        else metrics.push_back(a);
    }
    std::vector<std::vector<int64_t>> keys(naggs);
    if (!hists.empty()) {
        std::vector<int64_t> msg;  // [count per histogram] [keys of histogram 0] ...
        std::vector<std::vector<int64_t>> local(hists.size());
        for (size_t h = 0; h < hists.size(); ++h) {
            for (auto* l : locals) {
                const Block& b = (*l)[hists[h]];
                local[h].insert(local[h].end(), b.key.begin() + (int64_t)b.boff[0], b.key.begin() + (int64_t)b.boff[1]);
            }
            std::sort(local[h].begin(), local[h].end());
            local[h].erase(std::unique(local[h].begin(), local[h].end()), local[h].end());
            msg.push_back((int64_t)local[h].size());
        }
        for (auto& v : local) msg.insert(msg.end(), v.begin(), v.end());
        const std::vector<std::string> msgs = gather_messages(c, std::string((const char*)msg.data(), msg.size() * 8));
        for (const std::string& m : msgs) {
            const int64_t* p = (const int64_t*)m.data();
            const size_t n = m.size() / 8;
            if (n < hists.size()) throw std::runtime_error("corrupt key message");
            size_t pos = hists.size();
            for (size_t h = 0; h < hists.size(); ++h) {
                const size_t cnt = (size_t)p[h];
                if (pos + cnt > n) throw std::runtime_error("corrupt key message");
                keys[hists[h]].insert(keys[hists[h]].end(), p + pos, p + pos + cnt);
                pos += cnt;
            }
        }
        for (int a : hists) {
            std::sort(keys[a].begin(), keys[a].end());
            keys[a].erase(std::unique(keys[a].begin(), keys[a].end()), keys[a].end());
        }
    }
    // (2) dense partials: per slot (histogram bucket, or the one metric instance) the doc count, and per numeric metric
    //     its value count (u64 sums), sum and sum of squares (f64 sums), min and max (u64 min / max of encodings)
    struct Layout { int agg; size_t slots, nmet, u64, f64, mn, mx; };
    std::vector<Layout> lay;
    size_t nu = 0, nf = 0, nmn = 0, nmx = 0;
    for (int a : fixed) {
        const Block& b = first[a];
        if (b.type == ESGPU_AGG_CARDINALITY) continue;
        const bool hist = b.is_bucket();
        Layout L{a, hist ? keys[a].size() : 1, hist ? b.subs.size() : 1, nu, nf, nmn, nmx};
        nu += L.slots * ((hist ? 1 : 0) + L.nmet);
        nf += L.slots * L.nmet * 2;
        nmn += L.slots * L.nmet;
        nmx += L.slots * L.nmet;
        lay.push_back(L);
    }
    if (!lay.empty()) {
        // integer counts and the order-preserving extrema are exact under any combination order: all-reduced.  The f64
        // sums are not: each shard's (sum, sum of squares) partials are all-gathered and added in global shard order,
        // the order of the shard-order reduce (InternalStats.doReduce), so the result is bit-identical to it.
        std::vector<uint64_t> U(nu, 0), MN(nmn, ~0ULL), MX(nmx, 0);
        std::vector<double> FS(nf * locals.size(), 0.0);  // [local shard][nf]
        for (const Layout& L : lay) {
            const bool hist = first[L.agg].is_bucket();
            const size_t du = hist ? 1 : 0;
            for (size_t li = 0; li < locals.size(); ++li) {  // local shards in shard order
                const Block& b = (*locals[li])[L.agg];
                double* F = FS.data() + li * nf;
                const uint64_t k0 = hist ? b.boff[0] : 0, k1 = hist ? b.boff[1] : 1;
                for (uint64_t k = k0; k < k1; ++k) {
                    size_t slot = 0;
                    if (hist) {
                        slot = (size_t)(std::lower_bound(keys[L.agg].begin(), keys[L.agg].end(), b.key[k]) - keys[L.agg].begin());
                        U[L.u64 + slot * (du + L.nmet)] += (uint64_t)b.bcount[k];
                    }
                    for (size_t j = 0; j < L.nmet; ++j) {
                        const Block& m = hist ? b.subs[j] : b;
                        const uint64_t i = hist ? k : 0;
                        U[L.u64 + slot * (du + L.nmet) + du + j] += (uint64_t)m.count[i];
                        F[L.f64 + (slot * L.nmet + j) * 2] += m.sum[i];
                        F[L.f64 + (slot * L.nmet + j) * 2 + 1] += m.sumsq[i];
                        uint64_t& mn = MN[L.mn + slot * L.nmet + j];
                        uint64_t& mx = MX[L.mx + slot * L.nmet + j];
                        mn = std::min(mn, enc_min(m.min[i]));
                        mx = std::max(mx, enc_max(m.max[i]));
                    }
                }
            }
        }
        if (nu) c.allreduce(U.data(), nu, ESGPU_DT_U64, ESGPU_RED_SUM);
        std::vector<double> F(nf, 0.0);
        if (nf) {
            const std::vector<std::string> msgs = gather_messages(c, std::string((const char*)FS.data(), FS.size() * 8));
            for (const std::string& m : msgs) {  // ranks in order, each rank's shards in order
                if (m.size() % (nf * 8)) throw std::runtime_error("corrupt partial-sum message");
                const double* v = (const double*)m.data();
                for (size_t sh = 0; sh < m.size() / (nf * 8); ++sh)
                    for (size_t i = 0; i < nf; ++i) F[i] += v[sh * nf + i];
            }
        }
        if (nmn) c.allreduce(MN.data(), nmn, ESGPU_DT_U64, ESGPU_RED_MIN);
        if (nmx) c.allreduce(MX.data(), nmx, ESGPU_DT_U64, ESGPU_RED_MAX);
        // (3) one merged shard result per aggregation, then the reference's own single-shard reduce on it (min_doc_count,
        //     empty-bucket fill, order)
        for (const Layout& L : lay) {
            const Block& proto = first[L.agg];
            const bool hist = proto.is_bucket();
            const size_t du = hist ? 1 : 0;
            Block m = proto.like();
            auto put_metric = [&](Block& dst, size_t slot, size_t j) {
                ++dst.n;
                dst.count.push_back((int64_t)U[L.u64 + slot * (du + L.nmet) + du + j]);
                dst.sum.push_back(F[L.f64 + (slot * L.nmet + j) * 2]);
                dst.sumsq.push_back(F[L.f64 + (slot * L.nmet + j) * 2 + 1]);
                dst.min.push_back(dec_min(MN[L.mn + slot * L.nmet + j]));
                dst.max.push_back(dec_max(MX[L.mx + slot * L.nmet + j]));
            };
            if (!hist) {
                put_metric(m, 0, 0);
            } else {
                ++m.n;
                m.doc_count_error.push_back(0);
                m.other_doc_count.push_back(0);
                for (size_t slot = 0; slot < L.slots; ++slot) {
                    const uint64_t dc = U[L.u64 + slot * (du + L.nmet)];
                    if (dc == 0) continue;
                    m.key.push_back(keys[L.agg][slot]);
                    m.term_off.push_back(m.term_pool.size());
                    m.bcount.push_back((int64_t)dc);
                    m.berr.push_back(0);
                    for (size_t j = 0; j < L.nmet; ++j) put_metric(m.subs[j], slot, j);
                }
                m.boff.push_back(m.key.size());
            }
            std::vector<Block> one;
            one.push_back(std::move(m));
            out[L.agg] = std::move(reduce_lists({&one})[0]);
        }
    }
    // (4) cardinality: local merge (shard order), then register max over the ranks -- or, while every rank is still in
    //     LINEAR_COUNTING, the union of the encoded-hash sets (HyperLogLogPlusPlus.merge, :201-230; the merged state
    //     depends only on the union of encoded hashes and the register maxima)
    if (!cards.empty()) {
        std::vector<HllState> st(cards.size());
        std::vector<uint64_t> flags(cards.size() * 2, 0);  // present, hll mode
        for (size_t k = 0; k < cards.size(); ++k) {
            for (auto* l : locals) {
                const Block& b = (*l)[cards[k]];
                if (!b.hll_present[0]) continue;
                if (!st[k].present) { st[k].present = true; st[k].p = b.precision; st[k].mode = 0; }
                st[k].merge(b.precision, b.hll_mode[0], b.regs[0], b.lc[0]);
            }
            flags[2 * k] = st[k].present;
            flags[2 * k + 1] = st[k].mode;
        }
        c.allreduce(flags.data(), flags.size(), ESGPU_DT_U64, ESGPU_RED_MAX);
        std::vector<int> to_union;
        for (size_t k = 0; k < cards.size(); ++k) {
            const Block& proto = first[cards[k]];
            if (!flags[2 * k]) {  // no rank collected a value: the empty sketch
                Block m = proto.like();
                m.append_empty();
                out[cards[k]] = std::move(m);
                continue;
            }
            if (!flags[2 * k + 1]) { to_union.push_back((int)k); continue; }
            HllState& s = st[k];
            s.p = proto.precision;
            if (!s.present) s.regs.assign((size_t)1 << s.p, 0);
            else if (s.mode == 0) s.upgrade();
            c.allreduce(s.regs.data(), s.regs.size(), ESGPU_DT_U8, ESGPU_RED_MAX);
            Block m = proto.like();
            ++m.n;
            m.hll_present.push_back(1);
            m.hll_mode.push_back(1);
            m.regs.push_back(std::move(s.regs));
            m.lc.emplace_back();
            out[cards[k]] = std::move(m);
        }
        if (!to_union.empty()) {
            // every rank in LINEAR_COUNTING: the shards' hash lists are all-gathered and merged in global shard order
            // into one Hashset -- the insertion order of the shard-order reduce, so the slots (and the hashes' order on
            // the wire) come out as the reference's coordinator lays them out
            std::string msg;
            for (int k : to_union) {
                for (auto* l : locals) {
                    const Block& b = (*l)[cards[k]];
                    const uint64_t n = b.hll_present[0] && !b.hll_mode[0] ? b.lc[0].size() : 0;
                    msg.append((const char*)&n, 8);
                    if (n) msg.append((const char*)b.lc[0].data(), n * 4);
                }
            }
            const uint64_t nl = locals.size();
            const std::vector<std::string> msgs = gather_messages(c, std::string((const char*)&nl, 8) + msg);
            std::vector<HllState> merged(to_union.size());
            for (size_t u = 0; u < to_union.size(); ++u) {
                merged[u].p = first[cards[to_union[u]]].precision;
                merged[u].present = true;
            }
            for (const std::string& mm : msgs) {  // ranks in order, each rank's shards in order
                size_t pos = 0;
                auto take = [&](size_t n) {
                    if (pos + n > mm.size()) throw std::runtime_error("corrupt set message");
                    const char* q = mm.data() + pos;
                    pos += n;
                    return q;
                };
                uint64_t nsh;
                std::memcpy(&nsh, take(8), 8);
                for (size_t u = 0; u < to_union.size(); ++u)
                    for (uint64_t sh = 0; sh < nsh; ++sh) {
                        uint64_t n;
                        std::memcpy(&n, take(8), 8);
                        std::vector<uint32_t> lc(n);
                        if (n) std::memcpy(lc.data(), take(n * 4), n * 4);
                        merged[u].merge(merged[u].p, 0, {}, lc);
                    }
            }
            for (size_t u = 0; u < to_union.size(); ++u) {
                HllState& s = merged[u];
                Block m = first[cards[to_union[u]]].like();
                ++m.n;
                m.hll_present.push_back(1);
                m.hll_mode.push_back(s.mode);
                m.lc.push_back(s.mode ? std::vector<uint32_t>() : s.lc());
                m.regs.push_back(std::move(s.regs));
                out[cards[to_union[u]]] = std::move(m);
            }
        }
    }
    return out;
}

}  // namespace esgpu
