// esgpu_results.hpp — columnar InternalAggregations of libesgpu.so and their reduce / JSON / stream formats.
//
// A Block holds ONE aggregation (one spec of the request) for `n` parent buckets at once: instance i is the
// InternalAggregation that the reference would build for parent bucket i (StringTerms, InternalHistogram,
// InternalStats, InternalExtendedStats, InternalAvg, InternalCardinality).  Bucket aggregations keep their buckets
// in flat arrays ([boff[i], boff[i+1]) belong to instance i) and every sub-aggregation is again a Block with one
// instance per bucket.  The north-star result (10 terms x 720 hours x stats) is 3 blocks of flat arrays instead of
// ~7,200 objects, which keeps build / reduce / transport in the tens of microseconds.
#pragma once

#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/esgpu.h"
#include "es_rounding.hpp"

namespace esgpu {

struct Block {
    // ---- request parameters (shared by every instance of the spec) ----
    int32_t type = 0;
    int32_t order = 0;
    std::string name;
    int32_t required_size = 10;
    int32_t shard_size = 10;
    int64_t min_doc_count = 1;
    int32_t show_err = 0;
    int32_t keyed = 0;
    bool has_empty_info = false;  // histogram EmptyBucketInfo (min_doc_count == 0)
    int32_t date_unit = 0;
    int64_t interval = 1;
    int64_t offset = 0;
    std::vector<int64_t> tz_starts, tz_offs;  // date_histogram time zone (empty = UTC / folded fixed offset)
    bool has_bmin = false, has_bmax = false;
    int64_t bmin = 0, bmax = 0;
    double sigma = 2.0;
    int32_t precision = 14;
    std::string order_path;  // terms ordered by a metric sub-aggregation (ESGPU_ORDER_AGG_*)
    std::string time_zone = "UTC";  // request time zone id (wire stream: TimeZoneRounding, ValueFormatter.DateTime)
    int32_t value_format = 0;       // ESGPU_FORMAT_* of the field (ValuesSourceParser.resolveFormat)
    std::string format;             // its pattern

    uint64_t n = 0;  // instances

    // ---- bucket aggregations ----
    std::vector<int64_t> doc_count_error;  // [n]
    std::vector<int64_t> other_doc_count;  // [n]
    std::vector<uint64_t> boff;            // [n + 1]
    std::vector<int64_t> key;              // [nb] histogram key / terms ordinal in the producing shard
    std::vector<uint64_t> term_off;        // [nb + 1] (terms)
    std::string term_pool;
    std::vector<int64_t> bcount;           // [nb] doc_count
    std::vector<int64_t> berr;             // [nb] bucket doc_count_error
    std::vector<Block> subs;               // each with n == nb
    std::vector<Block> empty_subs;         // prototypes, n == 1

    // ---- numeric metrics [n] ----
    std::vector<int64_t> count;
    std::vector<double> sum, min, max, sumsq;

    // ---- cardinality [n] ----
    std::vector<uint8_t> hll_present;
    std::vector<int32_t> hll_mode;
    std::vector<std::vector<uint8_t>> regs;
    std::vector<std::vector<uint32_t>> lc;  // encoded hashes in the Hashset's slot order (HyperLogLogPlusPlus.java:428-498)

    Rounding rounding() const;  // histogram specs: the request's Rounding (EmptyBucketInfo)
    bool is_bucket() const { return type == ESGPU_AGG_TERMS || type == ESGPU_AGG_HISTOGRAM || type == ESGPU_AGG_DATE_HISTOGRAM; }
    uint64_t nbuckets() const { return boff.empty() ? 0 : boff.back(); }
    std::string term(uint64_t b) const { return term_pool.substr(term_off[b], term_off[b + 1] - term_off[b]); }

    // an empty block with this block's parameters and sub-structure (no instances)
    Block like() const;
    // append instance `i` of `src` (same spec) to this block, deep (sub-blocks included)
    void append_instance(const Block& src, uint64_t i);
    // append an empty instance (buildEmptyAggregation) of this spec
    void append_empty();
};


// ---- terms ordered by a metric sub-aggregation (InternalOrder.Aggregation) ----
// AggregationPath.parse of a one-element path: "name", "name.key" or "name[key]" (key empty when absent)
bool parse_order_path(const std::string& path, std::string* name, std::string* key);
// the metric the path's key names, with Java double arithmetic: InternalAvg.value / InternalStats.value(name) /
// InternalExtendedStats.value(name), equal to the shard-level AvgAggregator.metric / StatsAggegator.metric /
// ExtendedStatsAggregator.metric(name, bucket); returns false for a key the metric does not have
bool metric_value(int type, const std::string& key, int64_t count, double sum, double min, double max, double sumsq,
                  double sigma, double* out);
// Comparators.compareDiscardNaN: NaN sorts last in both directions
inline int compare_discard_nan(double a, double b, bool asc) {
    if (a != a) return b != b ? 0 : 1;
    if (b != b) return -1;
    const int c = a < b ? -1 : a > b ? 1 : 0;  // Double.compare on non-NaN values, except -0.0 vs 0.0 below
    if (c != 0) return asc ? c : -c;
    if (a == 0.0 && b == 0.0) {  // Double.compare orders -0.0 before 0.0
        const bool na = __builtin_signbit(a), nb = __builtin_signbit(b);
        const int z = na == nb ? 0 : (na ? -1 : 1);
        return asc ? z : -z;
    }
    return 0;
}

// HyperLogLogPlusPlus
int hll_precision_from_threshold(int64_t count);
int64_t hll_cardinality(int precision, bool present, int mode, const uint8_t* regs, size_t nlc);

// InternalAggregations.reduce over shard lists in shard order
std::vector<Block> reduce_lists(const std::vector<const std::vector<Block>*>& lists);

// ---- the shard reduce across ranks (one process per GPU) ----
// Host-memory collectives among the ranks of one reduce; RCCL over xGMI (esgpu_comm_init) or a caller transport
// (esgpu_comm_init_host).  dtype / op values are include/esgpu.h's ESGPU_DT_* / ESGPU_RED_*.
struct Collective {
    int nranks = 1, rank = 0;
    uint64_t allreduce_bytes = 0, allgather_bytes = 0;  // per reduce call (statistics)
    int32_t collectives = 0;
    double exchange_ms = 0;                             // wall time inside the collectives of the last reduce
    int32_t last_path = 0;                              // esgpu_comm_build_reduce: 1 device-resident, 0 builds + reduce
    double last_host_ms = 0;                            // ... and its host time once the local collects had finished
    virtual ~Collective() {}
    virtual void allreduce(void* buf, uint64_t count, int dtype, int op) = 0;  // in place
    virtual void allgather(const void* in, void* out, uint64_t bytes) = 0;     // out: nranks * bytes, rank order
    // device operands, enqueued on `stream` (a hipStream_t): RCCL gathers device to device; a host transport stages
    // through pinned memory
    virtual void allgather_dev(const void* d_in, void* d_out, uint64_t bytes, void* stream) = 0;
    // in place on a device buffer, enqueued on `stream`: RCCL reduces device to device (ncclAllReduce); the in-process
    // transport reduces the ranks' buffers in rank order with one kernel; a host transport stages through pinned memory
    virtual void allreduce_dev(void* d_buf, uint64_t count, int dtype, int op, void* stream) = 0;
};
// InternalAggregations.reduce over every rank's shard results, the shards in rank-major order (rank r's `locals` are
// global shards r * n_local ...).  Fixed-shape partials are combined by all-reduce: top-level histograms with numeric
// metric sub-aggregations (bucket keys all-gathered, then sum of doc counts / metric counts / sums / sums of squares,
// min / max of order-preserving encodings), top-level numeric metrics, and top-level cardinality (register max over
// 2^p bytes, or the union of the linear-counting sets while every rank is still in LINEAR_COUNTING).  Everything
// else (terms at any level: per-shard top-k then merge) is all-gathered as shard records and reduced in shard order.
std::vector<Block> reduce_across(Collective& c, const std::vector<const std::vector<Block>*>& locals,
                                 bool gather_only = false);
bool same_shape(const Block& a, const Block& b);

std::string to_json(const std::vector<Block>& aggs);
// the aggregations object of an Elasticsearch search response, byte for byte as its XContent renders it
std::string to_xcontent(const std::vector<Block>& aggs);
void serialize(const std::vector<Block>& aggs, std::string& out);
// InternalAggregations.writeTo(StreamOutput): Elasticsearch's transport bytes of these aggregations
void to_es_stream(const std::vector<Block>& aggs, std::string& out);
bool deserialize(const uint8_t* p, size_t n, std::vector<Block>& out);

// owning wrapper behind the public esgpu_result (pub must stay the first member)
struct ResultHolder {
    esgpu_result pub;
    std::vector<Block> aggs;
    std::vector<std::unique_ptr<esgpu_agg_block[]>> views;
    std::vector<std::unique_ptr<const uint8_t*[]>> reg_ptrs;
    std::vector<std::unique_ptr<const uint32_t*[]>> lc_ptrs;
    std::vector<std::unique_ptr<int64_t[]>> lc_sizes;
    std::vector<std::unique_ptr<int32_t[]>> present32;
    std::string json;  // rendered on first esgpu_result_to_json
    bool json_valid = false;
    void export_view();
};

ResultHolder* holder_of(const esgpu_result* r);

}  // namespace esgpu
