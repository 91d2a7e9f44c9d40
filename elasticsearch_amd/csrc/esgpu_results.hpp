// esgpu_results.hpp — host-side InternalAggregation model of libesgpu.so (StringTerms, InternalHistogram,
// InternalStats, InternalExtendedStats, InternalAvg, InternalCardinality), its reduce, JSON and stream formats.
#pragma once

#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/esgpu.h"

namespace esgpu {

struct RAgg;

struct RBucket {
    int64_t key = 0;          // histogram key / terms ordinal in its shard
    std::string term;         // terms key bytes
    int64_t doc_count = 0;
    int64_t doc_count_error = 0;
    std::vector<RAgg> subs;
};

struct RAgg {
    int32_t type = 0;
    int32_t order = 0;
    std::string name;
    // bucket aggregations
    std::vector<RBucket> buckets;
    int64_t doc_count_error = 0;
    int64_t other_doc_count = 0;
    int32_t required_size = 10;
    int32_t shard_size = 10;
    int64_t min_doc_count = 1;
    int32_t show_err = 0;
    int32_t keyed = 0;
    // histogram EmptyBucketInfo
    bool has_empty_info = false;
    int32_t date_unit = 0;
    int64_t interval = 1;
    int64_t offset = 0;
    bool has_bmin = false, has_bmax = false;
    int64_t bmin = 0, bmax = 0;
    std::vector<RAgg> empty_subs;
    // metrics
    int64_t count = 0;
    double sum = 0.0, min = 0.0, max = 0.0, sumsq = 0.0, sigma = 2.0;
    // cardinality
    bool hll_present = false;
    int32_t precision = 14;
    int32_t hll_mode = 0;            // 0 linear counting, 1 hyperloglog
    std::vector<uint8_t> registers;  // 2^precision
    std::vector<uint32_t> lc;        // distinct encoded hashes, ascending
};

// rounding helpers for EmptyBucketInfo (common/rounding/*)
int64_t rounding_next(int32_t type, int32_t date_unit, int64_t interval, int64_t offset, int64_t value);

// HyperLogLogPlusPlus
int hll_precision_from_threshold(int64_t count);
int64_t hll_cardinality(const RAgg& a);
void hll_merge(RAgg& into, const RAgg& other);  // InternalCardinality.merge (into has hll_present)

// InternalAggregations.reduce over shard lists in shard order
std::vector<RAgg> reduce_lists(const std::vector<const std::vector<RAgg>*>& lists);

std::string to_json(const std::vector<RAgg>& aggs);
void serialize(const std::vector<RAgg>& aggs, std::string& out);
bool deserialize(const uint8_t* p, size_t n, std::vector<RAgg>& out);

// owning wrapper behind the public esgpu_result (pub must stay the first member)
struct ResultHolder {
    esgpu_result pub;
    std::vector<RAgg> aggs;
    // storage for the exported C view
    std::vector<std::unique_ptr<esgpu_agg_result[]>> agg_blocks;
    std::vector<std::unique_ptr<esgpu_bucket[]>> bucket_blocks;
    void export_view();
};

ResultHolder* holder_of(const esgpu_result* r);

}  // namespace esgpu
