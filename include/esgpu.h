/*
 * esgpu.h — C-ABI of libesgpu.so, the MI355X-native replacement for Elasticsearch's per-shard
 * aggregation collection path (global-ordinal terms, histogram/date_histogram, stats/extended_stats/avg,
 * HyperLogLog++ cardinality, term/range filters) and the shard-level InternalAggregation.reduce.
 *
 * Reference interfaces (paths relative to /root/reference/core/src/main/java/org/elasticsearch/):
 *   AggregatorFactory.createInternal ............ search/aggregations/AggregatorFactory.java:88-103
 *   Aggregator / BucketCollector ................. search/aggregations/Aggregator.java:38-107,
 *                                                  search/aggregations/BucketCollector.java:34-117
 *   getLeafCollector + LeafBucketCollector.collect search/aggregations/AggregatorBase.java:129-133,
 *                                                  search/aggregations/LeafBucketCollector.java:78-83
 *   postCollection / buildAggregation ............ search/aggregations/AggregatorBase.java:239-243
 *   InternalAggregation.doReduce ................. search/aggregations/InternalAggregation.java:152-160,
 *                                                  search/aggregations/InternalAggregations.java:133-161
 *   AggregationStreams (writeTo / readFrom) ...... search/aggregations/AggregationStreams.java
 *
 * A JNI shim maps each Java call onto exactly one entry point below.  Every function
 * returns an int status (ESGPU_OK = 0); esgpu_last_error() returns the thread-local message, which the
 * shim turns into IOException / AggregationExecutionException / CircuitBreakingException.
 *
 * Nothing here takes or returns a torch/HIP type: plain pointers and sizes only.
 */
#ifndef ESGPU_H
#define ESGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ESGPU_ABI_VERSION 7

/* ---------------------------------------------------------------------------------------------------------
 * Status codes.  Mapping used by the JNI shim (SURVEY §8(b) "Errors"):
 *   ESGPU_ERR_INVALID     -> IllegalArgumentException / AggregationInitializationException (AggregationPhase.java:90-91)
 *   ESGPU_ERR_UNSUPPORTED -> the plugin keeps the stock Java aggregator for this request (no GPU attempt made)
 *   ESGPU_ERR_DEVICE      -> IOException from collect/build => QueryPhaseExecutionException => shard failure
 *   ESGPU_ERR_OOM         -> CircuitBreakingException (BigArrays.java:393-395 accounting, here: HBM budget)
 *   ESGPU_ERR_STATE       -> IllegalStateException (calls out of order)
 * ------------------------------------------------------------------------------------------------------- */
enum {
    ESGPU_OK = 0,
    ESGPU_ERR_INVALID = 1,
    ESGPU_ERR_UNSUPPORTED = 2,
    ESGPU_ERR_DEVICE = 3,
    ESGPU_ERR_OOM = 4,
    ESGPU_ERR_STATE = 5,
    ESGPU_ERR_NO_DEVICE = 6
};

/* Copies the calling thread's last error message (NUL-terminated, truncated to cap). Returns its length. */
int esgpu_last_error(char* buf, size_t cap);
int esgpu_abi_version(void);

/* ---------------------------------------------------------------------------------------------------------
 * Device context: one per GPU, owns the HBM budget (REQUEST/FIELDDATA breaker analogue) and the streams.
 * Thread-safe for segment upload.  A plan is used by one thread at a time (one SEARCH thread per shard request,
 * SURVEY §8(b) "Threading"); distinct plans -- each with its own stream -- may run on different threads at once,
 * over the same segments.
 * ------------------------------------------------------------------------------------------------------- */
typedef struct esgpu_ctx esgpu_ctx;

/* device: HIP ordinal. hbm_budget_bytes: 0 = 90% of device memory. */
int esgpu_ctx_create(int device, uint64_t hbm_budget_bytes, esgpu_ctx** out);
int esgpu_ctx_destroy(esgpu_ctx* ctx);
int esgpu_ctx_hbm_used(const esgpu_ctx* ctx, uint64_t* bytes);
int esgpu_device_count(int* count);

/* Per-context layout options (no reference counterpart: they choose between equivalent GPU layouts, the results are
 * identical).  Defaults come from the environment (ESGPU_COMPACT / ESGPU_PI = 0 turn them off), else on; a change
 * applies from the next collect of any plan of the context.
 *   ESGPU_OPT_COMPACT_COLUMNS: the single-valued collect kernels read the segments' compact copies -- u16 ordinals
 *                              (dictionaries under 65,535 terms) and u32 deltas of long columns spanning < 2^32 --
 *                              instead of the upload-width columns
 *   ESGPU_OPT_PACKED_METRIC:   avg / stats under terms over a dense long metric accumulate in packed integer LDS cells
 *                              (count and sum of deltas in one u64 word; needs compact columns)
 *   ESGPU_OPT_HLL_FLOOR:       cardinality register passes over a dense numeric column take the floored stream when
 *                              the request's values per register allow it: 0 = the register phases
 *                              instead, 1 = on (default), 2..8 = on with the floor raised by value - 1 (a test leg:
 *                              registers left below the floor are finished by the tail pass)
 *   ESGPU_OPT_BLOCK_DELTAS:    a dense time-sorted key column whose every run of 2,048 docs spans < 2^16 is read by
 *                              the raw-load collect kernels as 16-bit deltas over each run's minimum (2 B per doc
 *                              instead of 4; needs compact columns; ESGPU_B16=0 turns the default off) */
enum { ESGPU_OPT_COMPACT_COLUMNS = 1, ESGPU_OPT_PACKED_METRIC = 2, ESGPU_OPT_HLL_FLOOR = 3, ESGPU_OPT_BLOCK_DELTAS = 4 };
int esgpu_ctx_set_option(esgpu_ctx* ctx, int32_t option, int64_t value);
int esgpu_ctx_get_option(const esgpu_ctx* ctx, int32_t option, int64_t* value);

/* ---------------------------------------------------------------------------------------------------------
 * Segment = one Lucene LeafReaderContext exported from doc values (K11).
 * Replaces ValuesSource.*Values(ctx) (search/aggregations/support/ValuesSource.java:60-152, 380-398).
 *
 * Column types (natural widths of SURVEY §8(d)):
 *   ESGPU_COL_ORD_U32 : SORTED / SORTED_SET doc values as u32 global ordinals, 0xFFFFFFFF = missing
 *                       (GlobalOrdinalsStringTermsAggregator.java:113-118; ord < 0 == missing)
 *   ESGPU_COL_I64     : SORTED_NUMERIC longs / dates as epoch millis (DateFieldMapper.java:539)
 *   ESGPU_COL_F64     : doubles (DoubleFieldMapper sortable-long already decoded to double)
 *   ESGPU_COL_U64     : murmur3 field hashes (Murmur3FieldMapper.java:160-162), stored as the signed long bits
 * Multi-valued columns are CSR: offsets[max_doc + 1] into values, values of one doc sorted ascending
 * (SortedNumericDocValues / SortedSetDocValues contract).  Single-valued numerics may carry a
 * `present` bitset (bit d set = doc d has a value); NULL = every doc has exactly one value.
 * ------------------------------------------------------------------------------------------------------- */
enum {
    ESGPU_COL_ORD_U32 = 1,
    ESGPU_COL_I64 = 2,
    ESGPU_COL_F64 = 3,
    ESGPU_COL_U64 = 4
};

typedef struct esgpu_column_desc {
    const char* name;            /* field name as used by esgpu_agg_spec.field / esgpu_filter.field */
    int32_t type;                /* ESGPU_COL_* */
    int32_t reserved;
    const void* values;          /* host memory (pinned recommended): max_doc entries, or offsets[max_doc] for CSR */
    const uint64_t* offsets;     /* NULL = single valued; else max_doc+1 CSR offsets */
    const uint64_t* present;     /* NULL = dense; else ceil(max_doc/64) words */
    /* ORD_U32 only: the segment's term dictionary, terms sorted by unsigned bytes (Lucene BytesRef order).
     * term i = dict_bytes[dict_offsets[i] .. dict_offsets[i+1]).  value_count = number of terms. */
    const uint8_t* dict_bytes;
    const uint64_t* dict_offsets;
    uint64_t value_count;
} esgpu_column_desc;

typedef struct esgpu_segment esgpu_segment;

/* Page-locked host memory for the export side of K11 (ValuesSource doc values decoded into flat arrays by the JNI
 * shim, A/support/ValuesSource.java:148-152, 391-398): esgpu_segment_upload copies from such buffers by DMA at the
 * host link's rate; from pageable memory the HIP runtime stages every copy through a bounce buffer. */
int esgpu_host_alloc(size_t bytes, void** out);
int esgpu_host_free(void* p);

/* K11: copies each column once into HBM (hipMemcpyAsync from the caller's buffers), builds per-block
 * min/max zone maps for numeric columns, keeps the term dictionaries host-side for lookupOrd. */
int esgpu_segment_upload(esgpu_ctx* ctx, const esgpu_column_desc* cols, int32_t ncols, uint32_t max_doc,
                         esgpu_segment** out);
int esgpu_segment_destroy(esgpu_segment* seg);
int esgpu_segment_max_doc(const esgpu_segment* seg, uint32_t* max_doc);

/* Synthetic log-style shard generated directly in HBM (bench/test data).
 * fields_mask: bit set of ESGPU_SYNTH_* columns to materialise. */
enum {
    ESGPU_SYNTH_TIMESTAMP = 1 << 0,   /* "@timestamp"       I64  */
    ESGPU_SYNTH_HOST = 1 << 1,        /* "host"             ORD  (1,000 terms, Zipf 1.1) */
    ESGPU_SYNTH_URL = 1 << 2,         /* "url"              ORD  (10,000,000 terms, Zipf 1.0) */
    ESGPU_SYNTH_STATUS = 1 << 3,      /* "status"           I64  */
    ESGPU_SYNTH_RESPONSE = 1 << 4,    /* "response_time_ms" I64  in [0,999] */
    ESGPU_SYNTH_BYTES = 1 << 5,       /* "bytes"            I64  in [0,1e6) */
    ESGPU_SYNTH_CLIENT_IP = 1 << 6,   /* "client_ip.hash"   U64  murmur3 h1 of a dotted quad */
    ESGPU_SYNTH_PRICE = 1 << 7        /* "price"            F64  non-integer doubles (float-stress) */
};
/* ts_jitter_ms: 0 = "@timestamp" non-decreasing in doc order; > 0 = each doc displaced by up to +-ts_jitter_ms
 * (roughly time-ordered docs, as merged segments hold them). */
int esgpu_segment_synthetic(esgpu_ctx* ctx, uint64_t seed, uint32_t shard, uint32_t num_docs, uint32_t fields_mask,
                            int64_t ts_jitter_ms, esgpu_segment** out);
/* Host-side generation of the same values (doc range [start, start+count)), for the CPU oracle/baseline.
 * out must hold count entries of the column's natural width (u32 for ORD columns, 8 bytes otherwise). */
int esgpu_synthetic_fill_host(uint64_t seed, uint32_t shard, uint32_t num_docs, uint32_t field_bit, int64_t ts_jitter_ms,
                              uint64_t start, uint64_t count, void* out);
/* Term bytes of a synthetic dictionary term (host / url).  Returns length, writes at most cap bytes. */
int esgpu_synthetic_term(uint32_t field_bit, uint64_t ord, char* buf, size_t cap);
/* Copy a device column range back to host (tests compare device vs host generator). */
int esgpu_segment_read_column(const esgpu_segment* seg, const char* field, uint64_t start, uint64_t count, void* out);
/* Frees the upload-width values of every single-valued long column that has a compact copy (its u32 / u16 deltas over
 * the segment minimum, built by an earlier request): those kernels read only the copy.  A later request whose kernel
 * reads the upload-width values (a calendar / DST rounding, cardinality of the field, a range filter over a wide
 * span ...) rebuilds them from the deltas -- losslessly -- and they stay (charged to the context's budget, like every
 * segment product).  No request may be collecting the segment during the call.  *released: the bytes freed. */
int esgpu_segment_release_wide(esgpu_segment* seg, uint64_t* released);

/* Global ordinals over the segments of one reader = GlobalOrdinalsBuilder.build / Lucene OrdinalMap
 * (core/.../index/fielddata/ordinals/GlobalOrdinalsBuilder.java:45-70, GlobalOrdinalMapping.java:51-58).
 * Merges the segments' term dictionaries of `field` (each sorted by unsigned bytes, as Lucene stores them) into
 * global ordinals and remaps every segment's ordinal column on the GPU.  From then on, terms aggregations and
 * keyword term filters on these segments use global ordinals and resolve terms through the global dictionary
 * (until a segment is destroyed or remapped by another map).  Segments without the field are skipped. */
typedef struct esgpu_ordinal_map esgpu_ordinal_map;
int esgpu_ordinal_map_build(esgpu_ctx* ctx, esgpu_segment* const* segs, int32_t nsegs, const char* field,
                            esgpu_ordinal_map** out);
int esgpu_ordinal_map_value_count(const esgpu_ordinal_map* map, uint64_t* count);
/* global ordinal of a term, or -1 (TermQuery resolution for keyword term filters) */
int esgpu_ordinal_map_lookup(const esgpu_ordinal_map* map, const uint8_t* term, size_t len, int64_t* ord);
int esgpu_ordinal_map_destroy(esgpu_ordinal_map* map);

/* ---------------------------------------------------------------------------------------------------------
 * Aggregation plan = one AggregatorFactory tree for one shard request (AggregatorFactories.java:68-90).
 * Specs are a flattened tree: spec[i].parent is the index of the enclosing bucket aggregation (-1 = top
 * level); parents precede children.  Parameters already carry the parser defaults (a1, a10, a17):
 *   terms:          size 10, shard_size from BucketUtils.suggestShardSideQueueSize, min_doc_count 1,
 *                   shard_min_doc_count 0, order count desc (+ term asc tie-break)
 *   date_histogram: min_doc_count 0, order key asc, unit/interval + offset (UTC or fixed tz offset folded in)
 *   cardinality:    precision_threshold -1 = default precision (14, -5 per multi-bucket ancestor)
 * esgpu_terms_thresholds() applies TermsParser + BucketCountThresholds.ensureValidity for callers that
 * only have the raw request values.
 * ------------------------------------------------------------------------------------------------------- */
enum {
    ESGPU_AGG_TERMS = 1,
    ESGPU_AGG_HISTOGRAM = 2,
    ESGPU_AGG_DATE_HISTOGRAM = 3,
    ESGPU_AGG_STATS = 4,
    ESGPU_AGG_EXTENDED_STATS = 5,
    ESGPU_AGG_AVG = 6,
    ESGPU_AGG_CARDINALITY = 7,
    ESGPU_AGG_SUM = 8,
    ESGPU_AGG_MIN = 9,
    ESGPU_AGG_MAX = 10,
    ESGPU_AGG_VALUE_COUNT = 11,
    ESGPU_AGG_FILTER = 12         /* FilterAggregator: single bucket of the docs matching its clauses (esgpu_filter.owner);
                                     top level only; result block: count[i] = doc_count, subs = its sub-aggregations */
};

/* terms order (InternalOrder.java:47-76; compound with _term asc tie-break for the count orders) */
enum {
    ESGPU_ORDER_COUNT_DESC = 0,
    ESGPU_ORDER_COUNT_ASC = 1,
    ESGPU_ORDER_TERM_ASC = 2,
    ESGPU_ORDER_TERM_DESC = 3,
    /* histogram orders (bucket/histogram/InternalOrder.java) */
    ESGPU_ORDER_KEY_ASC = 4,
    ESGPU_ORDER_KEY_DESC = 5,
    ESGPU_ORDER_HCOUNT_ASC = 6,
    ESGPU_ORDER_HCOUNT_DESC = 7,
    /* terms ordered by a metric sub-aggregation (InternalOrder.Aggregation, A/bucket/terms/InternalOrder.java:149-225;
     * compound with _term asc tie-break; NaN values last, Comparators.compareDiscardNaN): esgpu_agg_spec.order_path
     * names a direct stats / extended_stats / avg child, "<name>" or "<name>.value" for avg, "<name>.<metric>" for
     * stats (count, sum, min, max, avg) and extended_stats (+ sum_of_squares, variance, std_deviation, std_upper,
     * std_lower) -- AggregationPath.parse / validate (A/support/AggregationPath.java:68-113, 289-347) */
    ESGPU_ORDER_AGG_ASC = 8,
    ESGPU_ORDER_AGG_DESC = 9
};

/* date_histogram calendar units (DateTimeUnit.java:36-43); ESGPU_UNIT_NONE = fixed interval in ms */
enum {
    ESGPU_UNIT_NONE = 0,
    ESGPU_UNIT_WEEK = 1,
    ESGPU_UNIT_YEAR = 2,
    ESGPU_UNIT_QUARTER = 3,
    ESGPU_UNIT_MONTH = 4,
    ESGPU_UNIT_DAY = 5,
    ESGPU_UNIT_HOUR = 6,
    ESGPU_UNIT_MINUTE = 7,
    ESGPU_UNIT_SECOND = 8
};

typedef struct esgpu_agg_spec {
    int32_t type;                 /* ESGPU_AGG_* */
    int32_t parent;               /* index of parent bucket agg, -1 = top level */
    const char* name;
    const char* field;
    /* terms (TermsAggregator.BucketCountThresholds, TermsAggregator.java:63-85) */
    int32_t size;
    int32_t shard_size;
    int64_t min_doc_count;
    int64_t shard_min_doc_count;
    int32_t order;                /* ESGPU_ORDER_* */
    int32_t show_term_doc_count_error;
    /* histogram / date_histogram (HistogramAggregator.java:60-75, DateHistogramParser.java:85-193) */
    int32_t date_unit;            /* ESGPU_UNIT_*; NONE => `interval` in field units */
    int32_t keyed;
    int64_t interval;
    int64_t offset;               /* OffsetRounding offset; a fixed time-zone offset is passed as -tz_offset_ms */
    int32_t has_extended_bounds_min;
    int32_t has_extended_bounds_max;
    int64_t extended_bounds_min;  /* already rounded (ExtendedBounds.round) */
    int64_t extended_bounds_max;
    /* extended_stats (ExtendedStatsParser.java:57) */
    double sigma;
    /* cardinality (CardinalityParser.java:60-61) */
    int64_t precision_threshold;
    /* date_histogram time zone (ValuesSourceParser timezone -> TimeZoneRounding.Builder.timeZone,
     * DateHistogramParser.java:185-187).  tz_count == 0: UTC, or a fixed offset already folded into `offset`.
     * Otherwise the zone's offset history as joda's DateTimeZone reports it: offset tz_offsets_ms[i] applies from the
     * UTC instant tz_starts[i] on (tz_starts[0] is taken as -infinity), ascending, covering the field's value range.
     * Calendar units (month / quarter / year) and zones with transitions are bucketed through a per-segment table of
     * bucket start instants (es_rounding.hpp); everything else is affine on the GPU. */
    const int64_t* tz_starts;
    const int64_t* tz_offsets_ms;
    int32_t tz_count;
    int32_t reserved_tz;
    /* terms order ESGPU_ORDER_AGG_*: the sub-aggregation path (NUL-terminated) */
    const char* order_path;
    /* What the shard result's wire stream (esgpu_result_to_stream) carries besides the numbers:
     *   time_zone:    DateTimeZone.getID() of the request's time_zone ("UTC", "+01:00", "Europe/Berlin"); NULL = "UTC".
     *                 Written by TimeZoneRounding.TimeUnitRounding/TimeIntervalRounding.writeTo (TimeZoneRounding.java:
     *                 156-159, 213-216) and by the date formatter.
     *   value_format: the ValueFormatter ValuesSourceParser.resolveFormat picks for the field (ValuesSourceParser.java:
     *                 233-257): ESGPU_FORMAT_RAW (numeric field, no "format"), ESGPU_FORMAT_DATE_TIME (date field: the
     *                 mapping's date format, or the request's "format", with the request time zone), ESGPU_FORMAT_NUMBER
     *                 (numeric field with a "format" pattern); `format` holds the pattern. */
    const char* time_zone;
    int32_t value_format;
    int32_t reserved_fmt;
    const char* format;
} esgpu_agg_spec;

enum {
    ESGPU_FORMAT_RAW = 0,         /* ValueFormatter.Raw, stream id 1 */
    ESGPU_FORMAT_DATE_TIME = 1,   /* ValueFormatter.DateTime, stream id 2 (pattern, time zone id) */
    ESGPU_FORMAT_NUMBER = 2       /* ValueFormatter.Number.Pattern, stream id 4 (pattern) */
};

/* Query filters: bool{filter:[...]} conjunction of term / range clauses. */
enum {
    ESGPU_FILTER_TERM = 1,        /* doc matches if any value == term (numeric: TermQuery on the prefix-coded long;
                                     keyword: the term's ordinal; -1 = term not in dictionary => no match) */
    ESGPU_FILTER_RANGE = 2        /* doc matches if any value in [lo,hi] with include flags (NumericRangeQuery; on a
                                     keyword field TermRangeQuery over the term bytes lo_term / hi_term) */
};
typedef struct esgpu_filter {
    int32_t type;
    int32_t include_lower;
    int32_t include_upper;
    int32_t has_lower;
    int32_t has_upper;
    int32_t owner;                /* 0 = query clause (applies to every aggregation); k + 1 = clause of the filter
                                     aggregation spec[k] (FilterAggregator: conjunction of its clauses) */
    const char* field;
    int64_t term;                 /* TERM on I64 / ORD columns */
    int64_t lo_i, hi_i;           /* RANGE on I64 / U64 columns */
    double lo_d, hi_d;            /* RANGE on F64 columns */
    const uint8_t* lo_term;       /* RANGE on ORD columns: bounds as term bytes, compared as unsigned bytes (BytesRef) */
    const uint8_t* hi_term;
    uint64_t lo_term_len, hi_term_len;
} esgpu_filter;

int esgpu_terms_thresholds(int32_t size, int32_t shard_size, int64_t min_doc_count, int64_t shard_min_doc_count,
                           int32_t order, int32_t number_of_shards, int32_t* out_size, int32_t* out_shard_size,
                           int64_t* out_min_doc_count, int64_t* out_shard_min_doc_count);
int esgpu_precision_from_threshold(int64_t count, int32_t* precision);
/* The histogram / date_histogram spec's Rounding (Rounding.java, TimeZoneRounding.java incl. its time zone):
 * op 0 = round(value), 1 = nextRoundingValue(value), 2 = roundKey(value).  Callers use it for ExtendedBounds.round
 * (ExtendedBounds.java) before filling esgpu_agg_spec.extended_bounds_*. */
int esgpu_date_rounding(const esgpu_agg_spec* spec, int32_t op, int64_t value, int64_t* out);
/* MurmurHash3_x64_128 (common/hash/MurmurHash3.java:62-157): the murmur3 field's index-time hash is out[0] (h1)
 * (plugins/mapper-murmur3/.../Murmur3FieldMapper.java:152-165). */
int esgpu_murmur3_x64_128(const uint8_t* bytes, size_t len, int64_t seed, uint64_t* out2);
/* Double.toString(v) as the reference's JVM (Java 8, sun.misc.FloatingDecimal) prints it -- the digits every double of
 * esgpu_result_to_xcontent carries (XContentBuilder.value(double) -> Jackson -> Double.toString).  NUL-terminated into
 * buf (at most cap bytes incl. the NUL); returns ESGPU_ERR_INVALID when cap < 26. */
int esgpu_java_double(double v, char* buf, size_t cap);

/* ---------------------------------------------------------------------------------------------------------
 * Index-time hashing for bulk ingest: the shard a document routes to, and the murmur3 field value
 * stored for it, so that shards built outside Elasticsearch match the ones it would build from the same _ids / values.
 *   esgpu_routing_hash: Murmur3HashFunction.hash(routing) = StringHelper.murmurhash3_x86_32 over the UTF-16LE bytes of
 *                       the string (cluster/routing/Murmur3HashFunction.java:31-41); chars = Java UTF-16 code units.
 *   esgpu_route_shards: for n strings (CSR over UTF-16 units, host memory) the shard
 *                       MathUtils.mod(hash, number_of_shards) (cluster/routing/OperationRouting.java:238-258), on the GPU;
 *                       hashes_out may be NULL.
 *   esgpu_murmur3_field: for n values (CSR over UTF-8 bytes, host memory) MurmurHash3.hash128(bytes, 0).h1, the long
 *                       the murmur3 field mapper indexes (plugins/mapper-murmur3/.../Murmur3FieldMapper.java:152-165).
 * ------------------------------------------------------------------------------------------------------- */
int esgpu_routing_hash(const uint16_t* chars, size_t nchars, int32_t* hash);
int esgpu_route_shards(esgpu_ctx* ctx, const uint16_t* chars, const uint64_t* offsets, uint64_t n, int32_t number_of_shards,
                       int32_t* hashes_out, int32_t* shards_out);
int esgpu_murmur3_field(esgpu_ctx* ctx, const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1_out);

typedef struct esgpu_plan esgpu_plan;

/* = AggregationPhase.preProcess + AggregatorFactories.createTopLevelAggregators (AggregationPhase.java:69-94). */
int esgpu_plan_create(esgpu_ctx* ctx, const esgpu_agg_spec* specs, int32_t nspecs, const esgpu_filter* filters,
                      int32_t nfilters, esgpu_plan** out);
/* = getLeafCollector(ctx) + every collect(doc) of that segment.  accept_bits: optional live-docs / external
 * query bitset (host memory, ceil(max_doc/64) words, bit d = doc d matches), AND-ed with the plan filters.
 * Asynchronous on the plan's stream. */
int esgpu_plan_collect_segment(esgpu_plan* plan, const esgpu_segment* seg, const uint64_t* accept_bits);
/* = postCollection (AggregatorBase.java:239-243): LowCardinality remap, HLL LC/HLL decision; synchronises. */
int esgpu_plan_post_collection(esgpu_plan* plan);
/* = buildAggregation(0) on every top-level aggregator: returns the shard-level InternalAggregations. */
typedef struct esgpu_result esgpu_result;
int esgpu_plan_build(esgpu_plan* plan, esgpu_result** out);
/* Zero the accumulators so the plan (and its compiled launch configuration) is reused for another request. */
int esgpu_plan_reset(esgpu_plan* plan);
int esgpu_plan_destroy(esgpu_plan* plan);
/* Timing of the last collect_segment's dominant kernel (HIP events on the plan's stream), in milliseconds,
 * and the algorithmic bytes it read (SURVEY §8(d) formula).  path: the collect form -- 0 grid in global memory,
 * 1 LDS grid, 2 LDS key window, 3 HLL registers, 4 partitioned terms counting, 5 multi-valued (CSR) columns, 6 hot/cold
 * terms scatter form, 7 hot/cold postings form, 8 hot slots only (cold lists deferred to the top-k), 9 hot slots of a
 * filtered request (the scatter form deferred to the top-k). */
int esgpu_plan_last_collect_stats(const esgpu_plan* plan, double* kernel_ms, uint64_t* algorithmic_bytes,
                                  int32_t* path);
/* Wall time of the last esgpu_plan_build and the part of it spent waiting on the plan's stream (gathers and copies of
 * the winners' cells); the rest is host assembly of the result blocks.  Milliseconds. */
int esgpu_plan_last_build_stats(const esgpu_plan* plan, double* total_ms, double* wait_ms);
/* 1 if the plan's shard results are fixed-shape (no terms aggregation at any level): several shards of one GPU may
 * then be collected into one plan -- their doc counts, sums, extrema and sketches add up exactly as the reduce of their
 * separate results would (HistogramAggregator / metrics / HyperLogLogPlusPlus.merge; min_doc_count and empty buckets
 * apply at reduce) -- while terms need one build per shard (per-shard top-k, InternalTerms.doReduce). */
int esgpu_plan_shard_mergeable(const esgpu_plan* plan, int32_t* mergeable);
/* Segments the plan retains for a breadth-first replay at build (TermsAggregator breadth_first collect mode,
 * BestBucketsDeferringCollector.java:96-166): a terms-under-terms child whose [outer x inner] grid is over the dense
 * budget counts only the outer buckets while collecting and is collected again at build over the retained segments for
 * the surviving outer buckets.  A retained segment stays valid until the plan's reset / destroy even if
 * esgpu_segment_destroy is called on it first (its destroy is then carried out at that point). */
int esgpu_plan_deferred_segments(const esgpu_plan* plan, int32_t* segments);

/* ---------------------------------------------------------------------------------------------------------
 * Results: columnar InternalAggregations, owned by the library.
 * An esgpu_agg_block holds ONE aggregation of the request for n_instances parent buckets: instance i is the
 * InternalAggregation the reference builds for parent bucket i (StringTerms, InternalHistogram / InternalDateHistogram,
 * InternalStats, InternalExtendedStats, InternalAvg, InternalCardinality).  Top-level blocks have one instance.
 * A bucket aggregation's instance i owns buckets [bucket_offsets[i], bucket_offsets[i+1]); each sub-aggregation is a
 * block with one instance per bucket.  A JNI shim builds the Java objects from these arrays with bulk copies.
 * ------------------------------------------------------------------------------------------------------- */
typedef struct esgpu_agg_block esgpu_agg_block;

struct esgpu_agg_block {
    int32_t type;                 /* ESGPU_AGG_* */
    int32_t order;
    const char* name;
    /* request parameters shared by all instances */
    int32_t required_size;
    int32_t shard_size;
    int64_t min_doc_count;
    int32_t show_term_doc_count_error;
    int32_t keyed;
    int32_t has_empty_bucket_info;          /* histogram EmptyBucketInfo (InternalHistogram.java) */
    int32_t date_unit;
    int64_t interval;
    int64_t offset;
    int32_t has_extended_bounds_min;
    int32_t has_extended_bounds_max;
    int64_t extended_bounds_min;
    int64_t extended_bounds_max;
    double sigma;
    int32_t precision;
    int32_t nsubs;
    uint64_t n_instances;
    /* bucket aggregations */
    const int64_t* doc_count_error;         /* [n_instances] InternalTerms.docCountError */
    const int64_t* other_doc_count;         /* [n_instances] InternalTerms.otherDocCount */
    const uint64_t* bucket_offsets;         /* [n_instances + 1] */
    uint64_t n_buckets;
    const int64_t* keys;                    /* [n_buckets] histogram key; terms: ordinal in the producing shard */
    const uint64_t* term_offsets;           /* [n_buckets + 1] terms key bytes in term_bytes */
    const uint8_t* term_bytes;
    const int64_t* doc_counts;              /* [n_buckets] */
    const int64_t* bucket_doc_count_errors; /* [n_buckets] */
    const esgpu_agg_block* subs;            /* nsubs blocks, each with n_instances == n_buckets */
    const esgpu_agg_block* empty_subs;      /* nsubs prototypes (n_instances == 1) for empty histogram buckets */
    /* numeric metrics [n_instances] */
    const int64_t* count;
    const double* sum;
    const double* min;
    const double* max;
    const double* sum_of_squares;
    /* cardinality [n_instances] (HyperLogLogPlusPlus state, HyperLogLogPlusPlus.java:519-555) */
    const int32_t* hll_present;             /* 0 = InternalCardinality with counts == null */
    const int32_t* hll_mode;                /* 0 = linear counting, 1 = hyperloglog */
    const uint8_t* const* registers;        /* 2^precision run lengths (hll_mode 1) */
    const uint32_t* const* lc_hashes;       /* encoded hashes in Hashset slot order (hll_mode 0) */
    const int64_t* lc_sizes;
    const char* order_path;                 /* terms ordered by ESGPU_ORDER_AGG_*: the sub-aggregation path, else "" */
    const char* time_zone;                  /* the spec's time_zone id ("UTC" when none) */
    int32_t value_format;                   /* ESGPU_FORMAT_* */
    int32_t reserved_fmt;
    const char* format;                     /* pattern of DATE_TIME / NUMBER formats, else "" */
};

struct esgpu_result {
    const esgpu_agg_block* aggs;
    int32_t naggs;
    int32_t reserved;
};

int esgpu_result_free(esgpu_result* r);
/* InternalAggregations.reduce over shard results in shard order (InternalAggregations.java:133-161). */
int esgpu_reduce(const esgpu_result* const* shard_results, int32_t n, esgpu_result** out);
/* The same reduce over the shards of one request whose plans live on one device, built and reduced in one call:
 * identical to esgpu_reduce over esgpu_plan_build(plans[i]) in order.  For a top-level terms aggregation whose only
 * child is a histogram (affine rounding, key order, any min_doc_count / extended bounds) with numeric metric children
 * (at most 4, 2 to 64 shards), each plan builds only its
 * terms selection, the reference reduce runs over those, and the surviving terms' histogram rows are merged on the
 * device (no shard result is materialised); a top-level terms aggregation without sub-aggregations builds its plans
 * side by side (their device selections overlap); any other request builds every plan and reduces. */
int esgpu_plans_build_reduce(esgpu_plan* const* plans, int32_t n, esgpu_result** out);
/* *merged = 1 if the request's shape is one esgpu_plans_build_reduce merges on the device (the shards' data may still
 * send a request down the build-and-reduce path, e.g. an unmapped shard), 0 if it always builds and reduces. */
int esgpu_plans_colocated(esgpu_plan* const* plans, int32_t n, int32_t* merged);
/* Cardinality value of instance i of a cardinality block (HyperLogLogPlusPlus.cardinality(0)). */
int esgpu_cardinality_value(const esgpu_agg_block* block, uint64_t instance, int64_t* value);
/* XContent-style JSON ({"<name>": {...}}), full double precision, Infinity/NaN as JSON tokens.
 * Writes at most cap bytes (NUL-terminated) and returns the full length in *needed. */
int esgpu_result_to_json(const esgpu_result* r, char* buf, size_t cap, size_t* needed);
/* The "aggregations" object of the REST response as Elasticsearch's XContent writes it (compact Jackson JSON, field
 * order of each class's doXContentBody, Double.toString numbers, null metrics for empty buckets, date keys printed
 * with strict_date_optional_time in the request's time zone).  Same buffer contract as esgpu_result_to_json. */
int esgpu_result_to_xcontent(const esgpu_result* r, char* buf, size_t cap, size_t* needed);
/* Elasticsearch's transport wire format of a shard result: the bytes InternalAggregations.writeTo(StreamOutput) writes
 * (InternalAggregations.java:215-222) -- per aggregation its AggregationStreams type ("sterms", "dhisto", "histo",
 * "stats", "estats", "avg", "cardinality", "filter"), InternalAggregation.writeTo (name, null metadata, no pipeline
 * aggregators, InternalAggregation.java:212-221) and the class's doWriteTo (StringTerms.java:205-217 + Bucket.writeTo
 * :128-136, InternalHistogram.java:510-523 + Bucket.writeTo :183-187 + EmptyBucketInfo :223-230, InternalStats.java:
 * 182-189, InternalExtendedStats.java:169-174, InternalAvg.java:102-106, InternalCardinality.java:92-100 +
 * HyperLogLogPlusPlus.writeTo :519-535, InternalSingleBucketAggregation.java:124-127), with StreamOutput's encodings
 * (vInt/vLong, big-endian long/int, writeString as Java chars in modified UTF-8, StreamOutput.java:118-270).
 * A JNI shim hands these bytes to StreamInput and InternalAggregations.readAggregations to get the Java objects.
 * A LINEAR_COUNTING cardinality writes its hashes in the slot order of the reference's Hashset (HyperLogLogPlusPlus
 * .java:428-528): the collect records where each hash first occurred (the order its collector -- DirectCollector or
 * OrdinalsCollector -- adds it) and the build re-adds them in that order into a restated Hashset.
 * Same buffer contract as esgpu_result_to_json. */
int esgpu_result_to_stream(const esgpu_result* r, uint8_t* buf, size_t cap, size_t* needed);
/* Stream (AggregationStreams writeTo / readFrom analogue) for moving shard results between processes. */
int esgpu_result_serialize(const esgpu_result* r, uint8_t* buf, size_t cap, size_t* needed);
int esgpu_result_deserialize(const uint8_t* buf, size_t len, esgpu_result** out);

/* ---------------------------------------------------------------------------------------------------------
 * Shard reduce across ranks (one process per GPU; S shards per job, S / nranks per GPU); the
 * coordinating reduce of SearchPhaseController.merge (C/search/controller/SearchPhaseController.java:401-411) done by
 * every rank over a collective instead of a gather to one node.
 *   esgpu_comm_init:      RCCL communicator over xGMI; the unique id (ESGPU_COMM_ID_BYTES bytes) is created on rank 0
 *                         (esgpu_comm_unique_id) and broadcast by the caller.
 *   esgpu_comm_init_host: the same reduce over a caller-supplied host transport (cross-node: the node's own transport,
 *                         TransportService in the reference; tests: gloo).  Callbacks run on the calling thread and
 *                         return 0 on success.
 *   esgpu_comm_reduce:    InternalAggregations.reduce over every rank's shard results, the shards in rank-major order
 *                         (rank r passes its n_local results in its shard order).  Fixed-shape partials are combined by
 *                         all-reduce: top-level histograms with numeric metric sub-aggregations (bucket keys all-gathered,
 *                         then ncclAllReduce sum of doc counts / value counts / sums / sums of squares, min / max of the
 *                         order-preserving u64 image of the doubles), top-level stats / extended_stats / avg, and
 *                         top-level cardinality (ncclAllReduce max over the 2^p u8 registers, or the union of the
 *                         linear-counting sets while every rank is still in LINEAR_COUNTING); their f64 sums are
 *                         all-gathered per shard and added in global shard order.  Everything else -- terms at any
 *                         level, whose reduce is per-shard top-k then merge (InternalTerms.doReduce) -- is all-gathered
 *                         as shard records and reduced in shard order; top-level terms in a count or term order in two
 *                         phases (terms-level records first, then only the surviving buckets' sub-aggregations).  The
 *                         result is bit-identical to esgpu_reduce over every shard in shard order.
 *   esgpu_comm_gather_reduce: every aggregation through the all-gather path (one local shard).
 *   esgpu_comm_build_reduce: the reduce of one request straight from the ranks' collected shard plans (each rank passes
 *                         its n_local plans, global shard order rank-major), device-resident for the co-located shape
 *                         (esgpu_plans_colocated: terms{histogram{stats / extended_stats / avg}} in a count or term order,
 *                         one term dictionary on every rank): each device selects its shards' top shard_size terms, the
 *                         {count, ordinal} records are all-gathered from device memory, InternalTerms.doReduce
 *                         (A/bucket/terms/InternalTerms.java:165-246) runs on every rank over the shards' skeletons, and
 *                         only the surviving terms' histogram rows are all-gathered device to device and merged in global
 *                         shard order on the device (InternalHistogram.java:338-476 and the metric reduces) -- no shard
 *                         result is built.  The result is produced on rank `root` (an empty result elsewhere; every rank
 *                         when root < 0).  Other shapes build every local shard and run esgpu_comm_reduce (the result
 *                         on every rank).  Either way it equals esgpu_reduce over the shards' builds in shard order.
 *   esgpu_comm_init_local: an in-process communicator: nranks ranks of this process (one thread each, each with its own
 *                         context, on one or several devices) that name the same group; collectives are barriers among
 *                         the threads, device operands copied device to device on each rank's stream.
 *   esgpu_comm_last_build_reduce: the last build_reduce's path (1: device-resident, 0: builds + reduce) and its host
 *                         milliseconds once the rank's collects had finished (exchanges and the root's merge included).
 *   esgpu_comm_last_exchange: bytes moved by the last reduce on this communicator.
 *   esgpu_comm_destroy:   an RCCL communicator holds device buffers of its context: destroy it before esgpu_ctx_destroy.
 * ------------------------------------------------------------------------------------------------------- */
#define ESGPU_COMM_ID_BYTES 128
typedef struct esgpu_comm esgpu_comm;
enum { ESGPU_DT_U8 = 0, ESGPU_DT_I64 = 1, ESGPU_DT_U64 = 2, ESGPU_DT_F64 = 3 };
enum { ESGPU_RED_SUM = 0, ESGPU_RED_MIN = 1, ESGPU_RED_MAX = 2 };
typedef struct esgpu_host_transport {
    void* user;
    /* in place over `count` elements of dtype ESGPU_DT_*, op ESGPU_RED_* */
    int (*allreduce)(void* user, void* buf, uint64_t count, int32_t dtype, int32_t op);
    /* every rank contributes `bytes` bytes; `out` receives nranks * bytes in rank order */
    int (*allgather)(void* user, const void* in, void* out, uint64_t bytes);
} esgpu_host_transport;
int esgpu_comm_unique_id(uint8_t* id_out);
int esgpu_comm_init(esgpu_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* id, esgpu_comm** out);
int esgpu_comm_init_host(int32_t nranks, int32_t rank, const esgpu_host_transport* transport, esgpu_comm** out);
int esgpu_comm_destroy(esgpu_comm* comm);
int esgpu_comm_reduce(esgpu_comm* comm, const esgpu_result* const* locals, int32_t n_local, esgpu_result** out);
int esgpu_comm_gather_reduce(esgpu_comm* comm, const esgpu_result* local, esgpu_result** out);
int esgpu_comm_last_exchange(const esgpu_comm* comm, uint64_t* allreduce_bytes, uint64_t* allgather_bytes,
                             int32_t* collectives);
/* wall-clock milliseconds the last reduce spent inside its collectives (staging copies included) */
int esgpu_comm_last_exchange_ms(const esgpu_comm* comm, double* ms);
int esgpu_comm_build_reduce(esgpu_comm* comm, esgpu_plan* const* plans, int32_t n_local, int32_t root, esgpu_result** out);
int esgpu_comm_init_local(const char* group, int32_t nranks, int32_t rank, esgpu_comm** out);
int esgpu_comm_last_build_reduce(const esgpu_comm* comm, int32_t* path, double* host_ms);

#ifdef __cplusplus
}
#endif

#endif /* ESGPU_H */
