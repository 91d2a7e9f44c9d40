// esgpu_kernels.hpp — launch interfaces between the host runtime (esgpu_runtime.cpp) and the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace esgpu {

struct SynthParams {
    uint64_t seed;
    uint32_t shard;
    uint32_t pad0;
    uint64_t n;       // live docs
    uint64_t n_pad;   // allocated (multiple of kBlockDocs)
    int64_t ts_jitter;  // @timestamp displacement bound in ms (0 = sorted)
    int64_t* ts;
    uint32_t* host;
    uint32_t* url;
    int64_t* status;
    int64_t* rt;
    int64_t* bytes;
    uint64_t* ip;
    double* price;
    const double* host_cdf;
    const double* url_cdf;
    const double* rt_cdf;
};

#ifndef ESGPU_GROUP_BLOCKS  // collect: blocks per multi-pass group (and per dynamically claimed chunk)
#define ESGPU_GROUP_BLOCKS 4
#endif
constexpr uint32_t kGroupBlocks = ESGPU_GROUP_BLOCKS;
#ifndef ESGPU_DYN_CLAIM  // collect: claim chunks dynamically (1) or split the blocks statically (0); env ESGPU_DYN overrides
#define ESGPU_DYN_CLAIM 0
#endif
constexpr int kMaxPreds = 4;  // clauses a collect kernel evaluates itself (more: folded into a doc bitset first)
// PRED_D32_RANGE / PRED_D16_RANGE: an I64 range over the column's compact copy (u32 / u16 deltas over `base`)
enum PredKind : int32_t {
    PRED_ORD_EQ = 0, PRED_I64_RANGE = 1, PRED_F64_RANGE = 2, PRED_ORD_RANGE = 3, PRED_D32_RANGE = 4, PRED_D16_RANGE = 5
};

struct PredDev {
    const void* col;
    const uint64_t* present;
    const uint64_t* offsets;   // multi-valued column: CSR offsets [n_docs + 1] (doc matches if any value matches)
    int32_t kind;
    int32_t lo_incl, hi_incl, pad;
    int64_t lo, hi;    // ORD_EQ: lo = ordinal; I64_RANGE / ORD_RANGE: inclusive [lo, hi]
    double dlo, dhi;   // F64_RANGE with include flags
    int64_t base;      // D32_RANGE / D16_RANGE: value = base + delta
};

// separate outer-level doc counts: TERMS / HIST = counted per doc (the inner column has missing values);
// TERMS_DERIVED = terms outer over a dense histogram column: the per-term totals are summed from the LDS window at
// flush time (no per-doc cost) and counted per doc only on the global-atomic path.
enum OcntMode : int32_t { OCNT_NONE = 0, OCNT_TERMS = 1, OCNT_HIST = 2, OCNT_TERMS_DERIVED = 3 };

struct CollectParams {
    uint32_t n_docs, n_blocks, blocks_per_wg;
    int32_t lds_mode;    // 1: LDS-privatised cells, 0: global atomics only
    // terms dimension
    const uint32_t* ord;
    uint32_t T;
    // compact columns (loader VK bits 16 / 32): the ordinals as u16 (0xFFFF missing), the histogram column's long values
    // as u32 deltas over hv_base (a missing value's delta is 0; hv_present still decides)
    const uint16_t* ord16;
    const uint32_t* hv32;
    int64_t hv_base;
    // block-delta key column (loader VK bit 8192, raw-load kernels only): a dense long column whose every run of
    // 2^kB16Shift docs spans < 2^16, as the run's minimum (hv16_base) plus a 16-bit delta per doc -- 2 B per timestamp
    const uint16_t* hv16;
    const int64_t* hv16_base;
    // ... runs spanning < 2^24 (roughly time-ordered data): bits 16..23 of each delta in a byte plane (hv8, hv8_mask
    // ~0, hv8_and 0xFF); a column of 16-bit runs has no plane: hv8 = any readable word, hv8_mask = hv8_and = 0
    const uint8_t* hv8;
    uint32_t hv8_mask, hv8_and;
    // histogram under histogram, fused (loader VK bit 8): the terms dimension is the inner histogram's key index,
    // derived from its i64 / f64 column as t = (v - ord_base) / ord_div when 0 <= v - ord_base < ord_span (a 32-bit
    // magic division; ord_span = keys x interval < 2^32), else missing -- no materialised ordinal column
    const int64_t* ord_src;
    const uint64_t* ord_src_present;
    int32_t ord_src_f64;
    int64_t ord_base;
    uint32_t ord_span, ord_div, omg_m, omg_s1, omg_s2;
    // histogram dimension
    uint32_t H, W;
    int32_t windowed;    // 1: W < H, slide a W-slot window using the zone maps
    const int64_t* hv;               // histogram field values (i64, or f64 bits when hv_f64)
    const uint64_t* hv_present;
    int32_t hv_f64;                  // double field: keys from (long) value (ValuesSource.Numeric.longValues, castToLong)
    int64_t interval, offset, key0;  // key index k of a value v: floor((v - offset) / interval) - key0
    const int64_t* kstart;           // non-affine roundings: step start instants [nsteps] (step = last start <= v)
    const uint32_t* kslot;           // bucket of each step (null: step j is bucket j)
    uint32_t nsteps;
    const int64_t* zmin;
    const int64_t* zmax;
    const int64_t* zkey;             // windowed / block-delta collects: per-block key range [kmn, kmx] (launch_zone_keys)
    int32_t hord;                    // the key dimension is a second terms aggregation: hv holds u32 ordinals, H of them
    uint32_t mg_m, mg_s1, mg_s2;
    int32_t fast32;
    // metric
    const void* mv;
    const uint64_t* mv_present;
    int32_t mv_f64;
    // packed integer metric cells (loader VK bit 64): a dense single-valued long metric read as u32 deltas over mv_base
    // (the column's compact copy); an LDS cell is one u64 word, count << pk_shift | sum of deltas, plus a u32 (min, max)
    // delta pair -- one LDS atomic per doc for count + sum instead of two.  The host picks pk_shift so that neither field
    // can overflow within one workgroup's range of docs.
    const uint32_t* mv32;
    const uint16_t* mv16;  // the same deltas in 16 bits when the values span < 2^16 (loader VK bit 256)
    int64_t mv_base;
    uint32_t pk_shift;
    uint32_t hot_t[4];   // the segment's most frequent ordinals (a sampled hint; kMissingOrd: none): the packed cells'
                         // register runs (ESGPU_PI_NHOT of them)
    int32_t raw_dense;   // histogram-only grid over dense compact columns, no filter: the raw-load kernels (VK bit 1024)
    int32_t runs1;       // integer runs over time-sorted data: one run accumulator per thread (VK bit 4096)
    int32_t hdirect;     // histogram-only integer-run grids over roughly time-ordered data (no runs1): every doc straight
                         // into its key's LDS cells, lane-rotated copies (ncopies) instead of three thrashing runs
    int32_t dot16;       // ... whose metric deltas stay below 46,341 (a pair's squares fit 32 bits): single-key zone
                         // blocks update the run from the raw 16-bit words with packed dot / min / max instructions
    int32_t ukey32;      // raw-load kernels over 32-bit timestamp deltas skip single-key zone blocks (VK bit 16384:
                         // roughly time-ordered data whose blocks mostly hold one key; block deltas always do)
    int32_t vcnt_mode;   // separate value counts (metric column has missing values)
    int32_t ocnt_mode;   // separate outer-level doc counts (inner dimension column has missing values)
    uint32_t ncopies;    // terms-only LDS grids: copies of the additive cells (count, value count, sum, sum of squares);
                         // lane l adds into copy l % ncopies, so hot terms collide on ncopies addresses, not one
    int32_t npred;
    PredDev pred[4];
    const uint64_t* accept;
    // multi-valued columns (collect_multi_kernel): CSR offsets [n_docs + 1], null = single valued
    const uint64_t* ord_off;
    const uint64_t* hv_off;
    const uint64_t* mv_off;
    // global cell grid [H][T]
    unsigned long long* g_cnt;
    unsigned long long* g_ocnt;
    unsigned long long* g_vcnt;
    double* g_sum;
    unsigned long long* g_min;
    unsigned long long* g_max;
    double* g_sq;
    // compensated sums (DESIGN §5 "Float parity"; null: plain f64 adds, exact for the request's data): the low parts of
    // g_sum / g_sq as double-doubles -- zero between collects (launch_dd_fold adds them into g_sum / g_sq and clears them)
    double* g_sum_lo;
    double* g_sq_lo;
    // dynamic chunk claiming (null: static ranges of blocks_per_wg blocks): the grid is the resident workgroup slots,
    // workgroup g starts on chunk g (kGroup blocks) and claims later chunks from claim[0]; claim[1] counts finished
    // workgroups, and the last one resets both, so the pair is zero again for the next launch on the plan's stream
    unsigned int* claim;
    uint32_t n_chunks;
};

enum HllKind : int32_t { HLL_I64 = 0, HLL_F64 = 1, HLL_ORD = 2 };

struct HllParams {
    uint32_t n_docs;
    int32_t p;
    int32_t kind;
    int32_t npred;
    const void* col;
    const uint64_t* present;
    const uint64_t* ord_hash;   // HLL_ORD: murmur3 h1 of each term
    uint64_t n_ords;            // HLL_ORD: entries of ord_hash (ordinals >= n_ords are treated as missing)
    const uint64_t* accept;
    PredDev pred[4];
    unsigned int* regs;         // 2^p u32 registers
    unsigned int* lc_set;       // open-addressing set of encoded hashes (0 = empty)
    unsigned int* lc_count;
    unsigned int* nonzero;      // written by the register pass: registers != 0
    unsigned int* floor;        // scratch: min register after a phase
    unsigned char* gfloor;      // scratch: min register of each group of 64 registers after a phase ([max(m / 64, 1)])
    unsigned char* snap;        // scratch: registers as 4-bit lower bounds over the floor ([2^p / 2], 16-byte aligned)
    unsigned int* nz_part;      // [2] refresh / phase-0 gather: partial non-zero count and finished blocks (self-resetting)
    uint32_t lc_mask;
    uint32_t lc_threshold;
    uint64_t seen;              // values the registers already hold from earlier segments of this request
    // LINEAR_COUNTING insertion order: lc_first[slot] = min over the slot's hash occurrences of pos_base + (pos_ord ?
    // the ordinal : the value index) -- the order the reference's collector adds the hash to its Hashset (DirectCollector:
    // doc / value order; OrdinalsCollector.postCollect: ordinal order), pos_base = the segment's sequence << 40
    unsigned long long* lc_first;
    uint64_t pos_base;
    int32_t pos_ord;
    // phase 0 by register range (hll_p0_*): per-range fill counters [p0_ranges] (zero between requests) and the
    // entries (run length << 24 | register index) of each range, p0_cap per range; null: no partitioned phase 0
    unsigned int* p0_cnt;
    unsigned int* p0_buf;
    uint32_t p0_cap;
    uint32_t cut0;              // phase 0 spans the request's first cut0 * 2^p values (ESGPU_HLL_CUT0)
    int32_t log_raises;         // LDS phases log their register raises and leave them, partitioned by range, in p0_buf
                                // for the gather kernel (instead of one global atomicMax per raise); needs p0_cnt
    // floored stream (hll_fs_*, one pass instead of the phases): only hashes with run length >= fs_f are kept, logged
    // by register range into fs_buf (fs_cap per range) and maxed by one gather; a register still below fs_f afterwards
    // ("unresolved", counted into *unres by the gather) is finished by the tail pass over this segment's hashes with
    // run length < fs_f.  fs_f = 0: the phases.
    uint32_t fs_f;
    uint32_t fs_cap;
    unsigned int* fs_buf;
    unsigned int* unres;
    // the floored stream's input in 4 bytes per doc instead of the 8-byte values (null: hash the values): per doc its
    // hash's top kP2 = 25 bits and min(nlz(hash << 25), 39) -- the quantities HyperLogLogPlusPlus.encodeHash keeps
    // (HyperLogLogPlusPlus.java:335-346), from which index and run length follow exactly for any p <= 25 (hll_enc32)
    const uint32_t* enc32;
    // the group floors and snapshot already hold lower bounds of the registers as they stand (this request's previous
    // segment ended with a gather, which writes them; later raises keep them lower bounds): a warm segment skips its
    // refresh launch
    int32_t snap_ok;
};
// floored stream: the floor F (kept hashes have run length >= F, a fraction 2^-(F-1) of the stream) for a request whose
// registers will have seen `total` values when this segment is done: the largest F for which the expected number of
// registers ending below F, m * exp(-(total / m) * 2^-(F-1)), stays under 5e-3 (then a tail pass finishes them).
// 0 = too few values per register for a floor worth a pass (the phases instead).
uint32_t hll_fs_floor(uint64_t total, int p, uint32_t min_f);
uint32_t hll_fs_cap(uint64_t n, int p, uint32_t f);  // entries per register range for n values at floor f
#ifndef ESGPU_HLL_CUT0  // HLL phase 0 spans the request's first ESGPU_HLL_CUT0 * 2^p values
#define ESGPU_HLL_CUT0 4  // measured: 4 beats 16 by 3-4 % (phase 0 reads and raises registers for every hash)
#endif
// partitioned phase 0: ranges of registers (each whole groups of 64) and the entries a range holds
__host__ __device__ constexpr uint32_t hll_p0_ranges(uint32_t m) { return m >= 256u * 64u ? 256u : m / 64u; }
__host__ __device__ constexpr uint32_t hll_p0_cap(uint32_t m, uint32_t cut0) {  // mean + mean / 8 + 256 (> 8 sigma)
    return (cut0 * (m / hll_p0_ranges(m)) * 9u / 8u + 256u + 3u) & ~3u;
}

struct GatherParams {
    const uint32_t* rows;
    uint32_t k, H, T;
    int32_t narrays;
    const unsigned long long* src[6];
    unsigned long long* dst[6];
    int32_t cnt32;   // src[0] holds u32 counts (widened to u64 in dst[0])
};

// build: the winners' histogram rows compacted on the GPU into the result's columnar arrays (HistogramAggregator
// .buildAggregation per winner: the non-empty key slots ascending, each with its metric leaves decoded the way the
// host's metric_cell does), written straight into pinned host memory -- the host copies whole arrays instead of
// visiting k x H cells
struct CompactLeaf {
    const unsigned long long* cnt;   // the leaf's value counts ([H][T]: the value-count grid, or the doc-count grid)
    const double* sum;               // null: avg-less leaves never happen (every numeric metric keeps a sum)
    const unsigned long long* mn;    // order-preserving encodings; null: no min / max (avg)
    const unsigned long long* mx;
    const double* sq;                // null: no sum of squares (avg, stats)
    // [cap] outputs (pinned, device-mapped); o_count null: the leaf counts every doc of its bucket (the host copies the
    // bucket counts), o_min / o_max / o_sq null: not collected (the host fills the empty-leaf values)
    uint32_t* o_count;
    double *o_sum, *o_min, *o_max, *o_sq;
};
constexpr int kCompactLeaves = 4;
struct CompactParams {
    const uint32_t* rows;            // [k] winners' ordinals
    uint32_t k, H, T;
    const unsigned long long* cnt;   // bucket doc counts [H][T]
    uint32_t* nnz;                   // [k] non-empty slots per row (device scratch)
    uint32_t* o_nnz;                 // [k] the same, pinned
    uint32_t* o_slot;                // [cap] bucket key slots (the host maps them to keys)
    uint32_t* o_count;               // [cap] bucket doc counts (a shard's max_doc < 2^31)
    int32_t nleaves;
    CompactLeaf leaf[kCompactLeaves];
};
void launch_compact_rows(const CompactParams& p, hipStream_t s);

// co-located reduce (esgpu_plans_build_reduce): the final terms buckets' histogram rows merged over the shards of one
// device, in shard order (InternalHistogram.doReduce per key, InternalStats / InternalAvg / InternalExtendedStats.doReduce
// per bucket), into dense [R][Hm] rows over the union of the shards' key ranges
constexpr int kColoMaxShards = 64;  // shards one co-located reduce merges on the device (descriptors in LDS)
constexpr size_t kColoMergeBytes = 256ull << 20;  // the merge's pinned [R][Hm] rows at most (else builds + reduce)
constexpr size_t kColoKeepBytes = 32ull << 20;    // a merge buffer above this is released after the request
struct ColoShard {
    const unsigned long long* cnt;   // bucket doc counts [H][T] (u32 when cnt32)
    int32_t cnt32;
    uint32_t H, T;
    int64_t key0;
    const unsigned long long* lcnt[kCompactLeaves];  // leaf value counts (null: the bucket counts)
    const double* lsum[kCompactLeaves];
    const unsigned long long* lmn[kCompactLeaves];   // null: no extrema (avg)
    const unsigned long long* lmx[kCompactLeaves];
    const double* lsq[kCompactLeaves];               // null: no sum of squares
};
static_assert(sizeof(ColoShard) % 8 == 0, "ColoShard is copied as 8-byte words");
struct ColoParams {
    const ColoShard* shards;  // [nsh] (pinned, device-mapped; 8-byte multiple)
    const int32_t* rows;      // [R][nsh]: the final bucket's ordinal in each shard, -1 when the shard did not return it
    uint32_t nsh, R, Hm;
    int64_t kmin;
    int32_t nleaves;
    unsigned long long* o_cnt;  // [R][Hm] (pinned, device-mapped)
    unsigned long long* o_lcnt; // [nleaves][R][Hm]
    double *o_sum, *o_min, *o_max, *o_sq;  // [nleaves][R][Hm]
};
void launch_colo_merge(const ColoParams& p, hipStream_t s);
// the co-located reduce across ranks (esgpu_comm_build_reduce): each local shard's rows of the final terms packed as
// [F][Hmax][R] 8-byte words (F = 1 + 5 leaves: the bucket counts, then per leaf its value counts, sums, min, max and sums
// of squares), which colo_merge_kernel reads as a grid with T = R (the final bucket index as the ordinal)
struct ColoPackParams {
    const ColoShard* shards;  // [n] the local shards (pinned, device-mapped)
    const int32_t* rows;      // [R][n]: the final bucket's ordinal in local shard i, -1 when the shard did not return it
    uint32_t n, R, Hmax;
    int32_t nleaves;
    unsigned long long* out;  // [n][1 + 5 * nleaves][Hmax][R]
};
void launch_colo_pack(const ColoPackParams& p, hipStream_t s);
// the in-process transport's all-gather on one device: rank r's `bytes` (a multiple of 8) from srcs[r] into dst + r * bytes,
// one launch for every rank (n <= kColoMaxShards)
void launch_gather_bufs(const void* const* srcs, int n, size_t bytes, void* dst, hipStream_t s);
// dst = the n buffers (count elements of dtype ESGPU_DT_*) combined element-wise by op ESGPU_RED_*, in rank order
void launch_reduce_bufs(const void* const* srcs, int n, uint64_t count, int dt, int op, void* dst, hipStream_t s);
// the reduce across ranks of a top-level cardinality (esgpu_comm_build_reduce): the local plans' u32 registers maxed into
// out[0, m) as bytes, then a kXrCardTail-byte tail (present / HYPERLOGLOG flags, the shape hash and its complement) that
// the all-reduce (max) carries; every plan's two counters (LC hashes inserted, non-zero registers) to lc_out[2 * s ...]
constexpr uint32_t kXrCardTail = 64;
struct XrCardPack {
    const unsigned int* regs[kColoMaxShards];  // null: the plan collected nothing
    const unsigned int* cnt[kColoMaxShards];   // Pipeline.lc_count: [0] LC hashes, [1] non-zero registers
    uint32_t n, m, thr;
    unsigned long long hash;
    uint8_t* out;                              // device, m + kXrCardTail bytes
    uint32_t* lc_out;                          // pinned (device-mapped), 2 * n words
};
void launch_xr_card_pack(const XrCardPack& K, hipStream_t s);
// the all-reduced bytes (m + kXrCardTail) copied to dst (pinned, device-mapped) and the non-zero registers added to *nz
void launch_xr_card_finish(const uint8_t* regs, uint32_t m, unsigned long long* dst, uint32_t* nz, hipStream_t s);
// a shard's GPU top-k keys (k_req wanted of kk slots, then the sum of all counts at keys[kk]) as the selection record
// {picks, other-doc count, count << 32 | ordinal ...} (2 + K words)
void launch_xr_terms_record(const unsigned long long* keys, uint32_t kk, uint32_t k_req, int order, unsigned long long* rec,
                            uint32_t K, hipStream_t s);
// the co-located reduce's selection input: every shard's per-ordinal doc counts, summed over the [H][T] grid rows,
// written to out[shard][Tmax] (pinned, device-mapped) by one launch over all the shards
struct ColoTotals {
    const void* cnt;  // [H][T] u64 counts (u32 when cnt32)
    uint32_t H, T;
    uint32_t cnt32;
    uint32_t vc;      // the terms' value count (ordinals >= vc are not terms of the field)
};
static_assert(sizeof(ColoTotals) % 8 == 0, "ColoTotals is copied as 8-byte words");
void launch_colo_totals(const ColoTotals* d, uint32_t n, uint32_t Tmax, unsigned long long* out, hipStream_t s);
// each shard's terms selection on the device (build_terms_root's select_terms, count and term orders, value count <=
// kColoSelMax): one workgroup per shard sorts its candidates in LDS; out[shard][2 + K]: the number of picks, the
// other-doc count, then the picks in order as count << 32 | ordinal
constexpr uint32_t kColoSelMax = 4096;
struct ColoSelect {
    int32_t order;
    uint32_t K;  // picks per shard at most (the row stride is 2 + K)
    int64_t min_doc_count, shard_min_doc_count, shard_size;
};
void launch_colo_select(const unsigned long long* tot, const ColoTotals* d, uint32_t n, uint32_t Tmax, const ColoSelect& S,
                        unsigned long long* out, hipStream_t s);

// per-8192-doc-block min / max; f64 = the column holds doubles, taken as (long) casts (FieldData.castToLong)
void launch_zone_map(const int64_t* v, const uint64_t* present, uint32_t n, int64_t* zmin, int64_t* zmax, bool f64,
                     hipStream_t s);
void launch_synth(const SynthParams& p, hipStream_t s);
// wide: 1024-thread workgroups (histogram grids whose LDS window exceeds the two-per-CU budget), else 512
void launch_collect(const CollectParams& p, bool ord, bool hist, int met, bool wide, uint32_t grid, size_t lds, hipStream_t s);
// per-block key ranges of the zone maps under the request's rounding (out: 2 x n_blocks)
void launch_zone_keys(const CollectParams& p, int64_t* out, hipStream_t s, unsigned long long* udocs = nullptr);
// pi: packed integer metric cells (CollectParams.pk_shift): 8 B per cell copy + an 8 B (min, max) pair per cell
size_t collect_lds_bytes(uint32_t T, uint32_t W, int met, int vcnt_mode, int ocnt_mode, uint32_t ncopies = 1, bool pi = false);
// resident workgroups per CU (hk: 0 none, 1 affine, 2 table; vk: bit 0 double histogram column, bit 1 double metric)
int collect_occupancy(bool ord, int hk, int met, size_t lds, int vk, bool wide = false);
// returns whether the group floors and snapshot are left as lower bounds of the registers (HllParams.snap_ok for the
// request's next segment)
bool launch_hll(const HllParams& p, uint32_t cus, hipStream_t s);
// the HllParams.enc32 form of a dense long / double column (n_pad entries: the column's padding included)
void launch_hll_enc32(const void* col, int kind, uint32_t n_pad, uint32_t* out, hipStream_t s);

// ---- multi-valued (CSR) columns, esgpu_kernels_multi.hip ----
// K1/K4/K5/K6/K7 for SortedSet / SortedNumeric doc values: one doc per thread, every (ordinal x deduplicated key)
// pair of the doc is a cell update, metrics aggregate all of the doc's values once (StatsAggegator's local sum).
void launch_collect_multi(const CollectParams& p, bool ord, bool hist, int met, uint32_t grid, size_t lds, hipStream_t s);
// doc bitset of (accept AND every predicate); multi-valued predicate columns match if any value matches
void launch_filter_bits4(uint32_t n_docs, const uint64_t* accept, const PredDev* preds, int npred, uint64_t* out,
                         hipStream_t st);  // single-valued clauses only (no offsets)
void launch_filter_bits(uint32_t n_docs, const uint64_t* accept, const PredDev* preds, int npred, uint64_t* out,
                        hipStream_t s);
// per-value bitset from a doc bitset over a CSR column (out zeroed by the launcher, words for n_values)
void launch_expand_bits(uint32_t n_docs, const uint64_t* doc_bits, const uint64_t* offsets, uint64_t n_values,
                        uint64_t* out, hipStream_t s);
// ---- cardinality under a bucket aggregation (HyperLogLogPlusPlus with one sketch per bucket ordinal) ----
// The buckets are the cells of the parent grid (cell = key slot * T + ordinal).  Pass 0 raises the u8 run-length
// registers [B][m]; nonzero counts them per bucket; pass 1 inserts the encoded hashes of the buckets that can still end
// in LINEAR_COUNTING (nonzero <= threshold) into per-bucket open-addressing sets [B][cap].
struct CardParams {
    CollectParams G;             // bucket dimensions: ord / hv columns, key mapping, T, H, accept (filters folded in)
    const void* col;             // the cardinality field
    const uint64_t* off;         // CSR offsets (multi-valued) or null
    const uint64_t* present;
    int32_t kind;                // HLL_I64 / HLL_F64 / HLL_ORD
    int32_t p;
    const uint64_t* ord_hash;    // HLL_ORD: murmur3 h1 per term
    uint64_t n_ords;
    uint8_t* regs;               // [B][2^p]
    uint32_t* sets;              // [B][cap]
    uint32_t* set_cnt;           // [B]
    uint32_t* nonzero;           // [B]
    uint32_t cap, thr;
    unsigned long long* first;   // [B][cap] insertion order of each set entry (HllParams.lc_first)
    uint64_t pos_base;
    int32_t pos_ord;
};
void launch_card(const CardParams& c, bool ord, bool hist, int pass, uint32_t grid, hipStream_t s);
void launch_card_nonzero(const uint8_t* regs, uint64_t n_buckets, int p, uint32_t* nonzero, hipStream_t s);
// out[i*row ... ] = src[cells[i]*row ...] (bytes), for the cells of the emitted buckets
void launch_gather_bytes(const uint32_t* cells, uint32_t n, uint32_t row_bytes, const uint8_t* src, uint8_t* dst, hipStream_t s);

// ---- index-time hashing (bulk ingest helpers) ----
// shard of each _id / routing value: MathUtils.mod(murmur3_x86_32(UTF-16LE(id)), nshards) (OperationRouting.java:238-258)
void launch_route(const uint16_t* chars, const uint64_t* offsets, uint64_t n, int32_t nshards, int32_t* hash_out,
                  int32_t* shard_out, hipStream_t s);
// murmur3 field values: MurmurHash3.hash128(utf8 bytes, seed 0).h1 per value (Murmur3FieldMapper.java:152-165)
void launch_murmur3_field(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1_out, hipStream_t s);

// min / max over a value array (multi-valued i64 columns: key range of a histogram), out[0] = min, out[1] = max
void launch_minmax_i64(const int64_t* v, uint64_t n, int64_t* out, bool f64, hipStream_t s);
void launch_widen_u32(const unsigned int* src, size_t n, unsigned long long* dst, hipStream_t st);
void launch_narrow_u64(const unsigned long long* src, size_t n, unsigned int* dst, hipStream_t st);
void launch_pack_ord16(const uint32_t* src, uint32_t n, uint16_t* out, hipStream_t st);
void launch_delta16(const int64_t* v, uint32_t n, int64_t base, uint16_t* out, hipStream_t st);
void launch_delta32(const int64_t* v, uint32_t n, int64_t base, uint32_t* out, hipStream_t st);
// breadth-first replay, compacted: one pass over a retained segment appends, for every doc whose outer bucket survived
// (slot_map) and that has an inner term, its replay-grid ordinal (winner w % wb) * stride + inner into the region of
// its batch of wb winners; the batches are then counted from their regions alone (the ordinal columns are read once for
// all batches instead of once per batch).  An append past a region's capacity is dropped and sets *overflow.
struct ReplayCompactParams {
    uint32_t n_docs;
    const uint32_t* a;           // outer (global) ordinals
    const uint16_t* a16;         // ... or their 16-bit copy (0xFFFF missing; null: read a)
    const uint32_t* b;           // inner (global) ordinals
    // outer ordinal -> its winner's batch << kReplayBatchShift | index in the batch (kMissingOrd: the bucket did not
    // survive) -- the per-doc batch arithmetic done once per ordinal on the host
    const uint32_t* slot_map;
    uint32_t slot_map_n;
    uint32_t vcB;                // inner ordinals (b >= vcB: missing)
    uint32_t wb, stride, nbatch;
    int32_t npred;
    PredDev pred[4];
    const uint64_t* accept;
    uint32_t* out;
    const uint64_t* region;      // [nbatch] first element of each batch's region in out
    const uint32_t* cap;         // [nbatch] its capacity (elements)
    uint32_t* fill;              // [nbatch] elements appended so far, kReplayFillStride words apart (zeroed before the
                                 // first segment; one cache line each: the workgroups' reservations do not queue on one)
    uint32_t* overflow;          // set to 1 when an append did not fit
};
constexpr uint32_t kReplayMaxBatches = 1024, kReplayBatchShift = 20, kReplayFillStride = 64;
void launch_replay_compact(const ReplayCompactParams& p, hipStream_t s);
// The breadth-first replay of a count-ordered terms child over its segment's hot inner terms (replay_hot): one pass
// counts, per outer winner, its docs on each of the inner field's Hh most frequent terms (the statistics' hot slots,
// most frequent first) in LDS, and the docs whose inner term is missing; a per-workgroup slab row is summed after.
struct ReplayHotParams {
    uint32_t n_docs, n_blocks, blocks_per_wg, G;
    const uint16_t* a16;         // outer ordinals, 16 bits (0xFFFF missing)
    const uint16_t* hot16;       // inner hot slot (0xFFFE a colder term, 0xFFFF missing)
    const uint8_t* slot_map;     // [slot_map_n] outer ordinal -> winner index (0xFF: not a winner)
    uint32_t slot_map_n;
    const uint64_t* accept;      // the request's folded clauses and live docs (null: every doc)
    uint32_t k, Hh;              // winners (< 255), hot slots counted per winner
    uint32_t* slab;              // [G][stride]: k * Hh counts, then k missing-term counts
    uint32_t* out;               // [stride] the sums
};
__host__ __device__ inline uint32_t replay_hot_stride(uint32_t k, uint32_t Hh) { return ((k * Hh + k) + 3u) & ~3u; }  // slab row words
size_t replay_hot_lds(uint32_t k, uint32_t Hh, uint32_t slot_map_n);
void launch_replay_hot(const ReplayHotParams& p, hipStream_t s);
void launch_comp_ords(const uint32_t* a, const uint32_t* b, uint32_t n_pad, uint32_t na, uint32_t nb, const uint32_t* amap,
                      uint32_t amap_n, uint32_t* out, hipStream_t st);
// ... with a calendar / DST rounding: each value's step in the bucket table (starts ascending), its key slot (slot[step],
// or the step itself when null); single-valued (offsets null: one per doc, padded docs included) or CSR
void launch_hist_ords_table(const int64_t* v, const uint64_t* present, const uint64_t* offsets, uint32_t n_docs, uint32_t n_pad,
                            bool f64, const int64_t* starts, uint32_t nsteps, const uint32_t* slot, uint32_t nkeys,
                            uint32_t* out, hipStream_t st);
// ... over a multi-valued field: one key index per value (CSR, the source's offsets), a doc's repeated keys kMissingOrd
void launch_hist_ords_multi(const int64_t* v, const uint64_t* offsets, uint32_t n_docs, bool f64, int64_t interval,
                            int64_t offset, int64_t key0, uint32_t nkeys, uint32_t* out, hipStream_t st);
void launch_hist_ords(const int64_t* v, const uint64_t* present, uint32_t n_docs, uint32_t n_pad, bool f64, int64_t interval,
                      int64_t offset, int64_t key0, uint32_t nkeys, uint32_t* out, hipStream_t s);
void launch_remap_ords(const uint32_t* in, uint32_t n, const uint32_t* map, uint32_t map_n, uint32_t* out, hipStream_t s);
void launch_pack_u8(const unsigned int* src, uint32_t n, uint8_t* dst, hipStream_t s);
void launch_term_totals(const unsigned long long* cnt, uint32_t H, uint32_t T, unsigned long long* out, hipStream_t s);
// n u64 words device -> device-visible pinned host memory
void launch_copy_u64(const unsigned long long* src, unsigned long long* dst, size_t n, hipStream_t s);
void launch_gather_rows(const GatherParams& p, hipStream_t s);
// a long column's upload-width values rebuilt from its compact deltas (value = base + delta)
void launch_expand_d32(const uint32_t* d, uint32_t n, int64_t base, int64_t* out, hipStream_t s);
void launch_expand_d16(const uint16_t* d, uint32_t n, int64_t base, int64_t* out, hipStream_t s);
// block-delta columns (CollectParams.hv16): runs of kB16Docs docs, each the run's minimum plus 16-bit deltas, and with a
// high-byte plane (hi, may be null) bits 16..23 of each delta.  The build ORs into *bad 1 when a run spans 2^16 or more
// (the plane is needed) and 2 when one spans 2^24 or more (the caller then keeps the 32-bit deltas); docs >= n_docs get
// delta 0
constexpr uint32_t kB16Shift = 11, kB16Docs = 1u << kB16Shift;
void launch_block_delta16(const int64_t* v, uint32_t n_docs, uint32_t n_pad, uint16_t* d, uint8_t* hi, int64_t* base,
                          unsigned int* bad, hipStream_t st);
void launch_expand_b16(const uint16_t* d, const uint8_t* hi, const int64_t* base, uint32_t n_docs, uint32_t n_pad, int64_t* out,
                       hipStream_t st);
// g_sum / g_sq += their compensated low parts, which are cleared (after every collect launch that used them)
void launch_dd_fold(double* hi, double* lo, size_t n, hipStream_t s);
void launch_fill_u64(unsigned long long* p, size_t n, unsigned long long v, hipStream_t s);
// several u64 arrays filled by one launch (a plan reset: counts, sums, min / max identities)
constexpr int kFillSpans = 8;
struct FillList {
    unsigned long long* p[kFillSpans];
    uint64_t n[kFillSpans];
    unsigned long long v[kFillSpans];
    int32_t count;
};
void launch_fill_multi(const FillList& l, hipStream_t s);
// several device -> pinned-host copies in one launch (the build's grid arrays: one launch instead of one per array)
struct CopyList {
    const unsigned long long* src[kFillSpans];
    unsigned long long* dst[kFillSpans];
    uint64_t n[kFillSpans];
    int32_t count;
};
void launch_copy_multi(const CopyList& l, hipStream_t s);

}  // namespace esgpu

namespace esgpu {

// ---- high-cardinality terms: radix-partitioned counting (T ordinals >> LDS) ----
struct PartParams {
    uint32_t n_docs, n_blocks, blocks_per_wg, G;   // G = workgroups of the histogram / scatter passes
    const uint32_t* ord;
    uint32_t T;
    uint32_t shift;          // partition of an ordinal = ord >> shift
    uint32_t P;              // number of partitions
    int32_t npred;
    PredDev pred[4];
    const uint64_t* accept;
    uint32_t* wg_counts;     // [P][G] docs of partition p seen by workgroup g (pass 1), exclusive offsets after the scan
    uint32_t* part_begin;    // [P + 1] start of each partition in pbuf
    uint16_t* pbuf;          // partitioned ordinals as partition-local offsets (ord & (2^shift - 1))
    unsigned int* counts;    // [T] output doc counts, u32 (BucketsAggregator's IntArray; max_doc < 2^31)
    uint32_t chunk;          // partitioned elements per counting workgroup
    uint32_t* tile_sums;     // scratch of the scan: part_scan_tiles(P * G) entries
};
#ifndef ESGPU_PART_SHIFT
#define ESGPU_PART_SHIFT 15  // measured: 5 % faster than 14 on config 3 (fewer, longer partition runs)
#endif
constexpr uint32_t kPartShift = ESGPU_PART_SHIFT;  // 32768 ordinals per partition (128 KB of LDS counters)
constexpr uint32_t kPartMaxStaged = 2048;  // partitions the LDS-staged scatter handles (2^25 ordinals at shift 14)
void launch_part_hist(const PartParams& p, hipStream_t s);
void launch_part_scan(const PartParams& p, hipStream_t s);
void launch_part_scatter(const PartParams& p, hipStream_t s);
void launch_part_count(const PartParams& p, hipStream_t s);
size_t part_scatter_lds_bytes(uint32_t n_parts);
uint32_t part_wg_per_cu();  // workgroups per CU of the histogram / scatter passes
uint32_t part_scan_tiles(uint32_t n);

// ---- high-cardinality terms, hot/cold partitioned counting (esgpu_hotcold.hip) ----
constexpr uint32_t kHcTile = 16384;     // upper bound of the docs of one scatter tile (spare elements of pbuf)
constexpr uint32_t kHcMaxParts = 1024;  // partitions the scatter handles: T <= 2^25 ordinals
constexpr uint32_t kHcHotBit = 0x80000000u;  // recoded column: kHcHotBit | hot slot
constexpr uint32_t kHcHotCopies = 64;   // the 64 most frequent hot slots keep 4 lane-rotated LDS counters each
struct HcPart {            // one partition's layout in pbuf (elements), fixed per segment by its HcStats
    uint32_t sbase;        // static regions: workgroup g owns [sbase + g * chunk, sbase + (g + 1) * chunk)
    uint32_t chunk;        // multiple of 64
    uint32_t ovf_base;     // overflow pool [ovf_base, cap_end): chunks of >= ovf_chunk elements
    uint32_t cap_end;
    uint32_t ovf_chunk;
    uint32_t pad[3];
};
struct HcPiece {           // a counting workgroup's share: region elements [lo, hi) of partition p (static ++ overflow)
    uint32_t p, lo, hi, whole;  // whole: the piece is the partition's only one (stores its counters, no atomics)
};
struct HcParams {
    uint32_t n_docs, n_blocks, blocks_per_wg, G;   // G = scatter workgroups (the segment statistics' layout)
    const uint32_t* rc;                // recoded ordinal column: cold ordinal | kHcHotBit | hot slot | 0xFFFFFFFF missing
    const uint16_t* rc16;              // postings hot pass: the hot slot of each doc, 0xFFFF for a cold / missing one
    uint32_t T, P;
    int32_t npred;
    PredDev pred[4];
    const uint64_t* accept;
    uint32_t hot_n;                    // hot slots (0 = none), most frequent first
    const uint32_t* hot_ord;           // [hot_n] ordinal of each hot slot
    const HcPart* part;                // [P]
    const HcPiece* piece;              // [n_pieces]
    uint32_t n_pieces;
    uint32_t* ovf_cur;                 // [P] next free element of each overflow pool
    uint32_t* used;                    // [P][G] elements written into each workgroup's static region
    uint32_t* hot_slab;                // [G][hc_hot_counters(hot_n)] per-workgroup hot counters
    uint16_t* pbuf;                    // partition-local offsets (ord & 32767); 0xFFFF = unused overflow element
    uint32_t trash;                    // kHcTile spare elements at the end of pbuf (capacity violation sink)
    unsigned int* counts;              // [T] u32 doc counts (IntArray: a shard's max_doc is below 2^31)
    uint32_t* err;                     // set to 1 on a capacity violation (device-visible host word)
    int32_t u16_counters;              // every cold ordinal's count in the segment < 65536: packed LDS counters
    int32_t overwrite;                 // store the counts instead of adding (the plan's first segment)
    uint32_t* slot_tot;                // postings hot pass, deferred cold lists: [hot_n] hot slot totals instead of
                                       // atomics onto counts[hot_ord] (esgpu_runtime.cpp hc_pending)
    const uint32_t* skip;              // non-null and set: the cold counting, the fold and (a filtered request's fallback)
                                       // the scatter form return at once
    uint32_t* cold_tot;                // hot16 pass with accept bits: the passing docs of cold ordinals, one total
};
__host__ __device__ inline uint32_t hc_hot_counters(uint32_t hot_n) { return hot_n + 3 * (hot_n < kHcHotCopies ? hot_n : kHcHotCopies); }
// per-workgroup hot slab row: the counters padded to 16 bytes (the reduce reads them as uint4)
__host__ __device__ inline uint32_t hc_slab_stride(uint32_t hot_n) { return (hc_hot_counters(hot_n) + 3u) & ~3u; }
size_t hc_scatter_lds_bytes(uint32_t n_parts, uint32_t hot_n);
constexpr uint32_t kHcScatterWG = 512;  // threads of a scatter workgroup (esgpu_hotcold.hip kHcWG)
void launch_hotcold(const HcParams& p, hipStream_t s);
// Requests without predicates or accept bits over a segment whose cold docs are also stored in partition order
// (HcStats' cold lists): `hot` streams the recoded column and counts only the hot slots (G = hot.G workgroups), `cold`
// counts the cold lists (one static region per partition, G = 1) with the scatter path's counting pass.
void launch_hotcold_postings(const HcParams& hot, const HcParams& cold, hipStream_t s);
// ... in two halves, for a request whose top-k the hot slots may settle alone (count order, the segment's largest cold
// count below the k-th hot one): the hot pass with its slot totals into hot.slot_tot, and later -- unless *cold.skip --
// the cold lists counted and the slot totals folded onto their ordinals
void launch_hot_postings(const HcParams& hot, hipStream_t s);
void launch_cold_postings(const HcParams& hot, const HcParams& cold, hipStream_t s);
// the hot slots' top-k settles the request: skip = the k keys all present and the k-th count above max_cold; then the
// final keys and the count sum (docs) are written where the full top-k would write them
// (cold_tot non-null: a filtered request, whose count sum is the hot slot totals plus *cold_tot instead of docs)
void launch_hot_topk_check(const unsigned long long* hot_keys, uint32_t k, uint32_t k_req, uint64_t max_cold, uint64_t docs,
                           int order, uint32_t* skip, unsigned long long* out_keys, unsigned long long* out_sum,
                           const uint32_t* slot_tot, uint32_t hot_n, const uint32_t* cold_tot, hipStream_t s);
// stats time: the dense partition-ordered cold offsets -> one list per partition starting at pad_begin[p] (a multiple
// of 64 elements), 0xFFFF between lists
void launch_hc_pad(const uint16_t* dense, const uint32_t* dense_begin, const uint32_t* pad_begin, uint32_t P,
                   uint16_t* out, hipStream_t s);
// stats time: out[d] = kHcHotBit | slot for the hot ordinals (open-addressing table keys -> vals, 2^log2 entries,
// 0xFFFFFFFF = empty key), the ordinal itself otherwise
void launch_hc_recode(const uint32_t* ord, uint32_t n, const uint32_t* keys, const uint32_t* vals, uint32_t log2,
                      uint32_t* out, hipStream_t s);
// stats time: the 16-bit hot-slot column of the postings hot pass from the recoded column (0xFFFF: cold or missing)
void launch_hc_hot16(const uint32_t* rc, uint32_t n, uint16_t* out, hipStream_t s);
// stats time: per partition of 2^shift ordinals the summed counts of its cold ordinals and the largest one
void launch_hc_part_stats(const unsigned int* counts, uint32_t T, uint32_t shift, uint32_t P, const uint64_t* hot_bits,
                          unsigned long long* part_sum, unsigned int* part_max, hipStream_t st);

// ---- GPU top-k over a count vector (BucketPriorityQueue replacement for large T) ----
struct TopkParams {
    const unsigned long long* counts;
    const unsigned int* counts32;  // non-null: u32 counts (the partitioned / hot-cold paths), read instead of counts
    uint32_t T;
    int32_t order;           // ESGPU_ORDER_COUNT_DESC / COUNT_ASC / TERM_ASC / TERM_DESC
    int64_t min_doc_count, shard_min_doc_count;
    uint32_t k;              // <= kTopkMax
    unsigned long long* cand;    // candidate keys: [n_wg][k] (term orders) or up to T (count orders)
    uint32_t* hist;              // count orders: [2048] count histogram
    uint32_t* sel;               // count orders: [2] threshold bin, candidate counter
    uint32_t n_wg;
    unsigned long long* out_keys;    // [k] winners (0 = none), best first
    unsigned long long* out_sum;     // [1] sum of counts over min_doc_count-eligible terms
    const uint32_t* ord_of;          // count orders: counts[i] is ordinal ord_of[i]'s (null: ordinal i) -- hot slots
    const uint32_t* skip;            // non-null and set: every kernel of this top-k returns at once (decided on the device)
};
constexpr uint32_t kTopkMax = 1024;
void launch_topk(const TopkParams& p, hipStream_t s);
void launch_topk_candidates(const TopkParams& p, hipStream_t s);  // count orders: cand[0, sel[1]) unsorted, out_sum
// terms under a histogram, count orders: per row r of the [H][T] count grid, the row's total (total[r]) and its top S
// candidates (count >= min_count) as u64 keys in selection order, count-major (asc: complemented), ties by ascending
// ordinal -- out[r * S + i], 0 past the last candidate.  S <= kRowTopkMax.
constexpr uint32_t kRowTopkMax = 1024;
void launch_row_topk(const unsigned long long* cnt, uint32_t T, uint32_t H, uint32_t S, bool asc, int64_t min_count,
                     unsigned long long* out, unsigned long long* total, hipStream_t st);
uint64_t topk_key(int order, uint64_t count, uint32_t ord);   // host mirror of the device key (for tests)

}  // namespace esgpu
