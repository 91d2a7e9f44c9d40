// esgpu_runtime.cpp — the C-ABI of libesgpu.so (include/esgpu.h): device contexts, HBM-resident segments,
// aggregation plans compiled to gfx950 kernel launches, shard-level build, and the RCCL shard reduce.
//
// The plan mirrors the reference operator lifecycle (paths relative to
// /root/reference/core/src/main/java/org/elasticsearch/search/aggregations/):
//   esgpu_plan_create           AggregationPhase.preProcess / AggregatorFactories.createTopLevelAggregators
//                               (AggregationPhase.java:69-94, AggregatorFactories.java:68-90)
//   esgpu_plan_collect_segment  getLeafCollector + LeafBucketCollector.collect for every matching doc
//                               (AggregatorBase.java:129-133, LeafBucketCollector.java:78-83)
//   esgpu_plan_post_collection  postCollection (AggregatorBase.java:239-243)
//   esgpu_plan_build            buildAggregation(0) (GlobalOrdinalsStringTermsAggregator.java:146-208,
//                               HistogramAggregator.java:120-133, StatsAggegator.java:140-152, ...)
#include <hip/hip_runtime.h>
#include <malloc.h>

#include <algorithm>
#include <functional>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <queue>
#include <string_view>
#include <unordered_map>
#include <memory>
#include <mutex>
#include <condition_variable>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/esgpu.h"
#include "es_common.hpp"
#include "es_rounding.hpp"
#include "esgpu_kernels.hpp"
#include "esgpu_results.hpp"
#include "esgpu_internal.hpp"
#include "java_double.hpp"

using namespace esgpu;

extern "C" int esgpu_last_error(char* buf, size_t cap) {
    if (buf && cap) {
        const size_t n = std::min(cap - 1, g_err.size());
        std::memcpy(buf, g_err.data(), n);
        buf[n] = 0;
    }
    return (int)g_err.size();
}
extern "C" int esgpu_abi_version(void) { return ESGPU_ABI_VERSION; }

extern "C" int esgpu_device_count(int* count) {
    return guarded([&] {
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess) n = 0;
        *count = n;
    });
}

void tune_host_heap() {
    static std::once_flag once;
    std::call_once(once, [] {
        // opt-in: the settings are the whole host process's (a JVM embedding the library keeps its own allocator
        // behaviour unless the operator asks for this)
        const char* e = std::getenv("ESGPU_MALLOC_TUNE");
        if (!(e && *e == '1')) return;
        mallopt(M_MMAP_THRESHOLD, 32 << 20);
        mallopt(M_TRIM_THRESHOLD, 256 << 20);
    });
}

extern "C" int esgpu_ctx_set_option(esgpu_ctx* c, int32_t option, int64_t value) {
    return guarded([&] {
        require(c, ESGPU_ERR_INVALID, "null context");
        if (option == ESGPU_OPT_HLL_FLOOR) {
            require(value >= 0 && value <= 8, ESGPU_ERR_INVALID, "hll floor option must be 0..8");
            c->opt_hll_fs = (int)value;
            return;
        }
        require(value == 0 || value == 1, ESGPU_ERR_INVALID, "option value must be 0 or 1");
        if (option == ESGPU_OPT_COMPACT_COLUMNS) c->opt_compact = (int)value;
        else if (option == ESGPU_OPT_PACKED_METRIC) c->opt_pi = (int)value;
        else if (option == ESGPU_OPT_BLOCK_DELTAS) c->opt_b16 = (int)value;
        else throw EsError(ESGPU_ERR_INVALID, "unknown context option");
    });
}

extern "C" int esgpu_ctx_get_option(const esgpu_ctx* c, int32_t option, int64_t* value) {
    return guarded([&] {
        require(c && value, ESGPU_ERR_INVALID, "null argument");
        if (option == ESGPU_OPT_COMPACT_COLUMNS) *value = c->opt_compact;
        else if (option == ESGPU_OPT_PACKED_METRIC) *value = c->opt_pi;
        else if (option == ESGPU_OPT_HLL_FLOOR) *value = c->opt_hll_fs;
        else if (option == ESGPU_OPT_BLOCK_DELTAS) *value = c->opt_b16;
        else throw EsError(ESGPU_ERR_INVALID, "unknown context option");
    });
}

extern "C" int esgpu_ctx_create(int device, uint64_t budget, esgpu_ctx** out) {
    tune_host_heap();
    return guarded([&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
            throw EsError(ESGPU_ERR_NO_DEVICE, "no HIP device visible (libesgpu requires an MI355X / gfx950 GPU)");
        require(device >= 0 && device < n, ESGPU_ERR_INVALID, "device ordinal out of range");
        HIPX(hipSetDevice(device));
        hipDeviceProp_t prop;
        HIPX(hipGetDeviceProperties(&prop, device));
        std::unique_ptr<esgpu_ctx> c(new esgpu_ctx());
        c->device = device;
        c->budget = budget ? budget : (uint64_t)(prop.totalGlobalMem * 0.9);
        c->cus = prop.multiProcessorCount;
        auto env_on = [](const char* name) { const char* e = std::getenv(name); return !(e && *e == '0'); };
        c->opt_compact = env_on("ESGPU_COMPACT") ? 1 : 0;
        c->opt_pi = env_on("ESGPU_PI") ? 1 : 0;
        c->opt_hll_fs = env_on("ESGPU_HLL_FS") ? 1 : 0;
        c->opt_b16 = env_on("ESGPU_B16") ? 1 : 0;
        HIPX(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        *out = c.release();
    });
}

extern "C" int esgpu_ctx_destroy(esgpu_ctx* c) {
    return guarded([&] {
        if (!c) return;
        (void)hipSetDevice(c->device);
        if (c->d_host_cdf) (void)hipFree(c->d_host_cdf);
        if (c->d_rt_cdf) (void)hipFree(c->d_rt_cdf);
        if (c->d_url_cdf) (void)hipFree(c->d_url_cdf);
        if (c->stream) (void)hipStreamDestroy(c->stream);
        delete c;
    });
}

extern "C" int esgpu_ctx_hbm_used(const esgpu_ctx* c, uint64_t* bytes) {
    return guarded([&] { *bytes = c->used.load(); });
}

// ------------------------------------------------------------------------------------------------------------
// synthetic data tables (host-computed once, identical for the host and device generators)
// ------------------------------------------------------------------------------------------------------------
static std::once_flag g_tables_once, g_url_once;
static std::vector<double> g_host_cdf, g_rt_cdf, g_url_cdf;

static void zipf_cdf(std::vector<double>& cdf, uint32_t n, double s) {
    cdf.resize(n);
    double total = 0;
    for (uint32_t k = 1; k <= n; ++k) total += std::pow((double)k, -s);
    double acc = 0;
    for (uint32_t k = 1; k <= n; ++k) {
        acc += std::pow((double)k, -s);
        cdf[k - 1] = acc / total;
    }
    cdf[n - 1] = 1.0;
}
static void ensure_tables() {
    std::call_once(g_tables_once, [] {
        zipf_cdf(g_host_cdf, kHostTerms, 1.1);
        g_rt_cdf.resize(kRtValues);
        // response_time_ms: floor(lognormal(mu=4, sigma=1)) clamped to [0, 999]
        for (uint32_t k = 0; k < kRtValues; ++k)
            g_rt_cdf[k] = 0.5 * std::erfc(-(std::log((double)k + 1.0) - 4.0) / std::sqrt(2.0));
        g_rt_cdf[kRtValues - 1] = 1.0;
    });
}
static void ensure_url_table() {
    std::call_once(g_url_once, [] { zipf_cdf(g_url_cdf, kUrlTerms, 1.0); });
}

static const char* synth_name(uint32_t bit) {
    switch (bit) {
        case ESGPU_SYNTH_TIMESTAMP: return "@timestamp";
        case ESGPU_SYNTH_HOST: return "host";
        case ESGPU_SYNTH_URL: return "url";
        case ESGPU_SYNTH_STATUS: return "status";
        case ESGPU_SYNTH_RESPONSE: return "response_time_ms";
        case ESGPU_SYNTH_BYTES: return "bytes";
        case ESGPU_SYNTH_CLIENT_IP: return "client_ip.hash";
        case ESGPU_SYNTH_PRICE: return "price";
    }
    return nullptr;
}

extern "C" int esgpu_synthetic_term(uint32_t field_bit, uint64_t ord, char* buf, size_t cap) {
    // formatted by hand ("host-%04u" / "/p/%08x"): builds resolve every winning ordinal of a synthetic field here
    char tmp[32];
    int n = 0;
    const uint32_t o = (uint32_t)ord;
    if (field_bit == ESGPU_SYNTH_HOST) {
        char d[10];
        int k = 0;
        for (uint32_t v = o; v || k < 4; v /= 10) d[k++] = (char)('0' + v % 10);
        std::memcpy(tmp, "host-", 5);
        n = 5;
        while (k) tmp[n++] = d[--k];
    } else if (field_bit == ESGPU_SYNTH_URL) {
        std::memcpy(tmp, "/p/", 3);
        for (int i = 0; i < 8; ++i) tmp[3 + i] = "0123456789abcdef"[(o >> (28 - 4 * i)) & 15];
        n = 11;
    } else {
        return -1;
    }
    tmp[n] = 0;
    if (buf && cap) {
        const size_t c = std::min((size_t)n, cap - 1);
        std::memcpy(buf, tmp, c);
        buf[c] = 0;
    }
    return n;
}

extern "C" int esgpu_synthetic_fill_host(uint64_t seed, uint32_t shard, uint32_t num_docs, uint32_t field_bit,
                                         int64_t ts_jitter_ms, uint64_t start, uint64_t count, void* out) {
    return guarded([&] {
        ensure_tables();
        if (field_bit == ESGPU_SYNTH_URL) ensure_url_table();
        const uint64_t ss = shard_seed(seed, shard);
        for (uint64_t i = 0; i < count; ++i) {
            const uint64_t d = start + i;
            switch (field_bit) {
                case ESGPU_SYNTH_TIMESTAMP: ((int64_t*)out)[i] = synth_timestamp(ss, d, num_docs, ts_jitter_ms); break;
                case ESGPU_SYNTH_HOST: ((uint32_t*)out)[i] = synth_host(ss, d, g_host_cdf.data()); break;
                case ESGPU_SYNTH_URL: ((uint32_t*)out)[i] = synth_url(ss, d, g_url_cdf.data()); break;
                case ESGPU_SYNTH_STATUS: ((int64_t*)out)[i] = synth_status(ss, d); break;
                case ESGPU_SYNTH_RESPONSE: ((int64_t*)out)[i] = synth_rt(ss, d, g_rt_cdf.data()); break;
                case ESGPU_SYNTH_BYTES: ((int64_t*)out)[i] = synth_bytes(ss, d); break;
                case ESGPU_SYNTH_CLIENT_IP: ((uint64_t*)out)[i] = synth_ip_hash(ss, d); break;
                case ESGPU_SYNTH_PRICE: ((double*)out)[i] = synth_price(ss, d); break;
                default: throw EsError(ESGPU_ERR_INVALID, "unknown synthetic field");
            }
        }
    });
}

// ------------------------------------------------------------------------------------------------------------
// segments
// ------------------------------------------------------------------------------------------------------------
// An immutable term dictionary (ordinal -> term bytes, sorted by unsigned bytes): a segment's own SortedSet dictionary,
// the synthetic formula, or the reader-wide global dictionary of an ordinal map (Lucene OrdinalMap).  Shared by the
// segments that use it and by the plans that resolve winners through it, so a plan never copies a dictionary and a
// destroyed segment never invalidates a plan's terms.  `identity` is a content hash: two dictionaries with equal
// identity number their terms the same way, so their ordinals may be counted into one grid.
struct TermDict {
    uint32_t synth_bit = 0;          // synthetic formula (esgpu_synthetic_term)
    bool numbered = false;           // no term bytes given: term(ord) = decimal ordinal
    uint64_t n = 0;
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offsets;   // n + 1 (explicit dictionaries)
    uint64_t identity = 0;
    uint64_t count() const { return n; }
    std::string_view view(uint64_t o, std::string& scratch) const {
        if (synth_bit) {
            char b[32];
            esgpu_synthetic_term(synth_bit, o, b, sizeof b);
            scratch = b;
            return scratch;
        }
        if (numbered) {
            scratch = std::to_string(o);
            return scratch;
        }
        return std::string_view((const char*)bytes.data() + offsets[o], (size_t)(offsets[o + 1] - offsets[o]));
    }
    std::string term(uint64_t o) const {
        std::string s;
        return std::string(view(o, s));
    }
    void seal() {  // FNV-1a over (kind, count, offsets, bytes)
        uint64_t h = 0xcbf29ce484222325ULL;
        auto mix = [&](const void* p, size_t len) {
            const uint8_t* b = (const uint8_t*)p;
            for (size_t i = 0; i < len; ++i) { h ^= b[i]; h *= 0x100000001b3ULL; }
        };
        const uint32_t kind = synth_bit ? synth_bit : numbered ? 0x80000000u : 0x40000000u;
        mix(&kind, sizeof kind);
        mix(&n, sizeof n);
        if (!offsets.empty()) mix(offsets.data(), offsets.size() * 8);
        if (!bytes.empty()) mix(bytes.data(), bytes.size());
        identity = h;
    }
};

static bool same_dict(const std::shared_ptr<const TermDict>& a, const std::shared_ptr<const TermDict>& b) {
    return a == b || (a && b && a->n == b->n && a->identity == b->identity);
}

struct HcStats;  // hot set + partition capacities of a high-cardinality ordinal column (collect_hotcold)

struct DevColumn {
    std::string name;
    int32_t type = 0;
    bool multi = false;
    DevBuf values;   // padded to a multiple of kBlockDocs entries
    DevBuf present;  // optional
    DevBuf offsets;  // multi-valued: CSR offsets [max_doc + 1] (values hold n_values entries, padded)
    const uint64_t* off_view = nullptr;  // a derived multi-valued column: its source's offsets (not owned)
    uint64_t n_values = 0;
    DevBuf zmin, zmax;
    int64_t vmin = INT64_MAX, vmax = INT64_MIN;  // over present values (I64 columns)
    int64_t zspan = 0;  // 90th percentile of a block's value range (zmax - zmin): how far the data is from sorted
    uint64_t value_count = 0;
    std::shared_ptr<const TermDict> dict;   // ORD: the segment's own dictionary (value_count terms)
    DevBuf ord_hash;  // murmur3 h1 per term (built lazily for cardinality on keyword fields)
    // global ordinals (esgpu_ordinal_map_build): the segment's ordinals remapped into the reader-wide dictionary
    std::shared_ptr<const TermDict> gdict;
    DevBuf gvalues;
    // statistics of ords() for high-cardinality terms, built on first use (ensure_hc_stats); rebuilt when ords() is
    // replaced by a remap into another global dictionary
    std::shared_ptr<const HcStats> hc;
    // compact copies the collect kernel's loader reads instead (ensure_ord16 / ensure_d32, built on first use and cached
    // with the column): ords() in 16 bits (0xFFFF missing) while the dictionary has fewer than 65,535 terms -- keyed by
    // the ords() buffer it was made from -- and a long column's values as 32-bit deltas over vmin while vmax - vmin < 2^32
    DevBuf ord16, d32, d16;  // d16: the same deltas in 16 bits while vmax - vmin < 2^16 (ensure_d16)
    // block deltas of a dense key column (ensure_b16): per run of kB16Docs docs its minimum (b16_base) and a 16-bit delta
    // per doc, when every run spans < 2^16 -- time-sorted timestamps at any density above ~1 doc per 32 ms -- and, when
    // some run spans 2^16 or more but none 2^24 (roughly time-ordered data: ±1 h of displacement), bits 16..23 of every
    // delta in a byte plane (b16_hi): 3 B per timestamp (Lucene's per-block bit packing, at 16 or 24 bits)
    DevBuf b16, b16_base, b16_hi;
    // esgpu_segment_release_wide: the upload-width values of a single-valued long column with a compact copy were
    // released; wide_i64 rebuilds them (losslessly, from the deltas) for a kernel that reads them, and keeps them
    // released by esgpu_segment_release_wide, rebuilt on first use (wide_i64): written under the context lock, read
    // without it by the collect path -- an atomic so that a rebuilt column's pointer is published before the flag clears
    std::atomic<bool> wide_released{false};
    const void* ord16_src = nullptr;
    bool d32_done = false, d16_done = false, b16_done = false;
    // the floored HLL stream's 4-byte words of a dense long / double column (ensure_hll_enc32, HllParams.enc32)
    DevBuf hll32;
    bool hll32_done = false;
    // distinct values of the column, estimated from the HLL registers of an earlier request that collected this segment
    // alone and unfiltered (-1: none yet) -- picks the floored stream's floor (collect_hll); any value is correct
    // (shared: a plan that collected the segment keeps it alive for its build, whatever happens to the segment meanwhile)
    std::shared_ptr<std::atomic<double>> hll_distinct = std::make_shared<std::atomic<double>>(-1.0);
    // the most frequent ordinal of ords() in a sample (a hint for the packed cells' register run; any value is correct)
    uint32_t hot_ord[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    const void* hot_src = nullptr;

    const DevBuf& ords() const { return gdict ? gvalues : values; }       // what terms aggregations count by
    uint64_t ord_count() const { return gdict ? gdict->count() : value_count; }
    const std::shared_ptr<const TermDict>& ord_dict() const { return gdict ? gdict : dict; }
    std::string ord_term(uint64_t ord) const { return ord_dict()->term(ord); }
    std::string term(uint64_t ord) const { return dict->term(ord); }
};

struct esgpu_segment {
    esgpu_ctx* ctx = nullptr;
    uint32_t max_doc = 0;
    uint32_t n_pad = 0;
    // plans that will read the segment again at build (breadth-first replay, the way BestBucketsDeferringCollector keeps
    // each LeafReaderContext until prepareSelectedBuckets): a destroy while pinned is carried out at the last unpin
    int pins = 0;
    bool doomed = false;
    std::map<std::string, std::unique_ptr<DevColumn>> cols;
    const DevColumn* col(const char* name) const {
        if (!name) return nullptr;
        auto it = cols.find(name);
        return it == cols.end() ? nullptr : it->second.get();
    }
};

static const void* wide_i64(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st);

// the synthetic dictionaries (host-%04d / /p/%08x) are formulas: one shared instance per field
static std::shared_ptr<const TermDict> synth_dict(uint32_t bit, uint64_t n) {
    static std::mutex mu;
    static std::map<uint32_t, std::shared_ptr<const TermDict>> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto& d = cache[bit];
    if (!d) {
        auto td = std::make_shared<TermDict>();
        td->synth_bit = bit;
        td->n = n;
        td->seal();
        d = td;
    }
    return d;
}

static uint32_t pad_docs(uint32_t n) { return (uint32_t)(((uint64_t)n + kBlockDocs - 1) / kBlockDocs * kBlockDocs); }

static void build_zone_map(esgpu_ctx* c, DevColumn& col, uint32_t n) {
    const uint32_t nb = (n + kBlockDocs - 1) / kBlockDocs;
    col.zmin.alloc(c, (size_t)std::max(nb, 1u) * 8);
    col.zmax.alloc(c, (size_t)std::max(nb, 1u) * 8);
    launch_zone_map(col.values.as<int64_t>(), col.present.as<uint64_t>(), n, col.zmin.as<int64_t>(), col.zmax.as<int64_t>(),
                    col.type == ESGPU_COL_F64,
                    c->stream);
    HIPX(hipGetLastError());
    std::vector<int64_t> mn(nb), mx(nb);
    if (nb) {
        HIPX(hipMemcpyAsync(mn.data(), col.zmin.p, nb * 8, hipMemcpyDeviceToHost, c->stream));
        HIPX(hipMemcpyAsync(mx.data(), col.zmax.p, nb * 8, hipMemcpyDeviceToHost, c->stream));
    }
    HIPX(hipStreamSynchronize(c->stream));
    std::vector<int64_t> range;
    range.reserve(nb);
    for (uint32_t b = 0; b < nb; ++b) {
        col.vmin = std::min(col.vmin, mn[b]);
        col.vmax = std::max(col.vmax, mx[b]);
        if (mn[b] <= mx[b]) range.push_back((int64_t)std::min<uint64_t>((uint64_t)mx[b] - (uint64_t)mn[b], INT64_MAX));
    }
    if (!range.empty()) {
        const size_t q = range.size() * 9 / 10;
        std::nth_element(range.begin(), range.begin() + q, range.end());
        col.zspan = range[q];
    }
}

extern "C" int esgpu_host_alloc(size_t bytes, void** out) {
    return guarded([&] {
        require(out != nullptr, ESGPU_ERR_INVALID, "null argument");
        *out = nullptr;
        if (!bytes) return;
        HIPX(hipHostMalloc(out, bytes, hipHostMallocDefault));
    });
}

extern "C" int esgpu_host_free(void* p) {
    return guarded([&] { if (p) HIPX(hipHostFree(p)); });
}

extern "C" int esgpu_segment_upload(esgpu_ctx* c, const esgpu_column_desc* cols, int32_t ncols, uint32_t max_doc,
                                    esgpu_segment** out) {
    return guarded([&] {
        require(c && out && (ncols == 0 || cols), ESGPU_ERR_INVALID, "null argument");
        require(max_doc <= 0x7FFFFFFFu, ESGPU_ERR_INVALID, "max_doc exceeds Lucene's int doc id space");
        std::lock_guard<std::mutex> lk(c->mu);
        HIPX(hipSetDevice(c->device));
        std::unique_ptr<esgpu_segment> s(new esgpu_segment());
        s->ctx = c;
        s->max_doc = max_doc;
        s->n_pad = pad_docs(max_doc);
        for (int i = 0; i < ncols; ++i) {
            const esgpu_column_desc& d = cols[i];
            require(d.name && d.type >= ESGPU_COL_ORD_U32 && d.type <= ESGPU_COL_U64, ESGPU_ERR_INVALID, "bad column descriptor");
            require(s->cols.find(d.name) == s->cols.end(), ESGPU_ERR_INVALID, std::string("duplicate column ") + d.name);
            std::unique_ptr<DevColumn> col(new DevColumn());
            col->name = d.name;
            col->type = d.type;
            col->value_count = d.value_count;
            const size_t w = d.type == ESGPU_COL_ORD_U32 ? 4 : 8;
            if (d.offsets) {
                // multi-valued (SortedNumeric / SortedSet): CSR on the device, values padded like a doc column
                col->multi = true;
                require(d.offsets[0] == 0, ESGPU_ERR_INVALID, "CSR offsets must start at 0");
                for (uint32_t k = 0; k < max_doc; ++k)
                    require(d.offsets[k] <= d.offsets[k + 1], ESGPU_ERR_INVALID, "CSR offsets must be non-decreasing");
                const uint64_t nv = d.offsets[max_doc];
                require(nv < 0xFFFFFFFFull - kBlockDocs, ESGPU_ERR_UNSUPPORTED, "more than 2^32 values in one segment");
                col->n_values = nv;
                const uint64_t nv_pad = pad_docs((uint32_t)nv);
                col->values.alloc(c, std::max<uint64_t>(nv_pad, kBlockDocs) * w);
                HIPX(hipMemsetAsync(col->values.p, d.type == ESGPU_COL_ORD_U32 ? 0xFF : 0, col->values.bytes, c->stream));
                if (nv) HIPX(hipMemcpyAsync(col->values.p, d.values, nv * w, hipMemcpyHostToDevice, c->stream));
                col->offsets.alloc(c, ((size_t)max_doc + 1) * 8);
                HIPX(hipMemcpyAsync(col->offsets.p, d.offsets, ((size_t)max_doc + 1) * 8, hipMemcpyHostToDevice, c->stream));
                if ((d.type == ESGPU_COL_I64 || d.type == ESGPU_COL_F64) && nv) {  // key range of a histogram over the field
                    DevBuf mm;
                    mm.alloc(c, 16);
                    const int64_t init[2] = {INT64_MAX, INT64_MIN};
                    HIPX(hipMemcpyAsync(mm.p, init, 16, hipMemcpyHostToDevice, c->stream));
                    launch_minmax_i64(col->values.as<int64_t>(), nv, mm.as<int64_t>(), d.type == ESGPU_COL_F64, c->stream);
                    HIPX(hipGetLastError());
                    int64_t r[2];
                    HIPX(hipMemcpyAsync(r, mm.p, 16, hipMemcpyDeviceToHost, c->stream));
                    HIPX(hipStreamSynchronize(c->stream));
                    col->vmin = r[0];
                    col->vmax = r[1];
                }
            } else {
                col->values.alloc(c, (size_t)s->n_pad * w);
                if (max_doc) HIPX(hipMemcpyAsync(col->values.p, d.values, (size_t)max_doc * w, hipMemcpyHostToDevice, c->stream));
                if (s->n_pad > max_doc) {
                    if (d.type == ESGPU_COL_ORD_U32)
                        HIPX(hipMemsetAsync(col->values.as<uint8_t>() + (size_t)max_doc * w, 0xFF, (size_t)(s->n_pad - max_doc) * w, c->stream));
                    else
                        HIPX(hipMemsetAsync(col->values.as<uint8_t>() + (size_t)max_doc * w, 0, (size_t)(s->n_pad - max_doc) * w, c->stream));
                }
                if (d.present && d.type != ESGPU_COL_ORD_U32) {
                    const size_t words = s->n_pad / 64;
                    col->present.alloc(c, words * 8);
                    HIPX(hipMemsetAsync(col->present.p, 0, words * 8, c->stream));
                    HIPX(hipMemcpyAsync(col->present.p, d.present, ((size_t)max_doc + 63) / 64 * 8, hipMemcpyHostToDevice, c->stream));
                }
                if (d.type == ESGPU_COL_I64 || d.type == ESGPU_COL_F64) build_zone_map(c, *col, max_doc);
            }
            if (d.type == ESGPU_COL_ORD_U32) {
                auto td = std::make_shared<TermDict>();
                td->n = d.value_count;
                if (d.dict_bytes && d.dict_offsets) {
                    require(d.dict_offsets[0] == 0, ESGPU_ERR_INVALID, "dictionary offsets must start at 0");
                    for (uint64_t k = 0; k < d.value_count; ++k)
                        require(d.dict_offsets[k] <= d.dict_offsets[k + 1], ESGPU_ERR_INVALID, "dictionary offsets must be non-decreasing");
                    td->offsets.assign(d.dict_offsets, d.dict_offsets + d.value_count + 1);
                    td->bytes.assign(d.dict_bytes, d.dict_bytes + d.dict_offsets[d.value_count]);
                } else {
                    td->numbered = true;
                }
                td->seal();
                col->dict = std::move(td);
            }
            s->cols[d.name] = std::move(col);
        }
        HIPX(hipStreamSynchronize(c->stream));
        *out = s.release();
    });
}

extern "C" int esgpu_segment_synthetic(esgpu_ctx* c, uint64_t seed, uint32_t shard, uint32_t num_docs, uint32_t mask,
                                       int64_t ts_jitter_ms, esgpu_segment** out) {
    return guarded([&] {
        require(c && out, ESGPU_ERR_INVALID, "null argument");
        require(num_docs <= 0x7FFFFFFFu, ESGPU_ERR_INVALID, "num_docs exceeds Lucene's int doc id space");
        std::lock_guard<std::mutex> lk(c->mu);
        HIPX(hipSetDevice(c->device));
        ensure_tables();
        if (!c->d_host_cdf) {
            HIPX(hipMalloc(&c->d_host_cdf, kHostTerms * 8));
            HIPX(hipMalloc(&c->d_rt_cdf, kRtValues * 8));
            HIPX(hipMemcpy(c->d_host_cdf, g_host_cdf.data(), kHostTerms * 8, hipMemcpyHostToDevice));
            HIPX(hipMemcpy(c->d_rt_cdf, g_rt_cdf.data(), kRtValues * 8, hipMemcpyHostToDevice));
        }
        if ((mask & ESGPU_SYNTH_URL) && !c->d_url_cdf) {
            ensure_url_table();
            HIPX(hipMalloc(&c->d_url_cdf, (size_t)kUrlTerms * 8));
            HIPX(hipMemcpy(c->d_url_cdf, g_url_cdf.data(), (size_t)kUrlTerms * 8, hipMemcpyHostToDevice));
        }
        std::unique_ptr<esgpu_segment> s(new esgpu_segment());
        s->ctx = c;
        s->max_doc = num_docs;
        s->n_pad = pad_docs(num_docs);
        SynthParams p{};
        p.seed = seed;
        p.shard = shard;
        p.n = num_docs;
        p.n_pad = s->n_pad;
        require(ts_jitter_ms >= 0, ESGPU_ERR_INVALID, "negative timestamp jitter");
        p.ts_jitter = ts_jitter_ms;
        p.host_cdf = c->d_host_cdf;
        p.rt_cdf = c->d_rt_cdf;
        p.url_cdf = c->d_url_cdf;
        for (uint32_t bit = 1; bit <= ESGPU_SYNTH_PRICE; bit <<= 1) {
            if (!(mask & bit)) continue;
            std::unique_ptr<DevColumn> col(new DevColumn());
            col->name = synth_name(bit);
            const bool ord = bit == ESGPU_SYNTH_HOST || bit == ESGPU_SYNTH_URL;
            col->type = ord ? ESGPU_COL_ORD_U32 : bit == ESGPU_SYNTH_CLIENT_IP ? ESGPU_COL_U64
                                                : bit == ESGPU_SYNTH_PRICE ? ESGPU_COL_F64 : ESGPU_COL_I64;
            col->values.alloc(c, (size_t)s->n_pad * (ord ? 4 : 8));
            if (ord) {
                col->value_count = bit == ESGPU_SYNTH_HOST ? kHostTerms : kUrlTerms;
                col->dict = synth_dict(bit, col->value_count);
            }
            switch (bit) {
                case ESGPU_SYNTH_TIMESTAMP: p.ts = col->values.as<int64_t>(); break;
                case ESGPU_SYNTH_HOST: p.host = col->values.as<uint32_t>(); break;
                case ESGPU_SYNTH_URL: p.url = col->values.as<uint32_t>(); break;
                case ESGPU_SYNTH_STATUS: p.status = col->values.as<int64_t>(); break;
                case ESGPU_SYNTH_RESPONSE: p.rt = col->values.as<int64_t>(); break;
                case ESGPU_SYNTH_BYTES: p.bytes = col->values.as<int64_t>(); break;
                case ESGPU_SYNTH_CLIENT_IP: p.ip = col->values.as<uint64_t>(); break;
                case ESGPU_SYNTH_PRICE: p.price = col->values.as<double>(); break;
            }
            s->cols[col->name] = std::move(col);
        }
        launch_synth(p, c->stream);
        HIPX(hipGetLastError());
        HIPX(hipStreamSynchronize(c->stream));
        for (auto& kv : s->cols)
            if (kv.second->type == ESGPU_COL_I64 || kv.second->type == ESGPU_COL_F64) build_zone_map(c, *kv.second, num_docs);
        *out = s.release();
    });
}

static std::mutex g_pin_mu;
static void pin_segment(const esgpu_segment* cs) {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    ++const_cast<esgpu_segment*>(cs)->pins;
}
static void unpin_segment(const esgpu_segment* cs) {
    esgpu_segment* s = const_cast<esgpu_segment*>(cs);
    bool drop = false;
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        drop = --s->pins == 0 && s->doomed;
    }
    if (drop) delete s;
}

extern "C" int esgpu_segment_destroy(esgpu_segment* s) {
    return guarded([&] {
        if (!s) return;
        {
            std::lock_guard<std::mutex> lk(g_pin_mu);
            if (s->pins > 0) { s->doomed = true; return; }
        }
        delete s;
    });
}

extern "C" int esgpu_segment_max_doc(const esgpu_segment* s, uint32_t* max_doc) {
    return guarded([&] { *max_doc = s->max_doc; });
}

extern "C" int esgpu_segment_release_wide(esgpu_segment* s, uint64_t* released) {
    return guarded([&] {
        require(s != nullptr, ESGPU_ERR_INVALID, "null segment");
        esgpu_ctx* c = s->ctx;
        HIPX(hipSetDevice(c->device));
        HIPX(hipDeviceSynchronize());  // no kernel still reads a buffer released below
        std::lock_guard<std::mutex> lk(c->mu);
        uint64_t n = 0;
        for (auto& kv : s->cols) {
            DevColumn& col = *kv.second;
            if (col.type != ESGPU_COL_I64 || col.multi || !col.values.p || !(col.d32.p || col.d16.p || col.b16.p)) continue;
            n += col.values.bytes;
            col.values.release();
            col.wide_released = true;
        }
        if (released) *released = n;
    });
}

extern "C" int esgpu_segment_read_column(const esgpu_segment* s, const char* field, uint64_t start, uint64_t count, void* out) {
    return guarded([&] {
        const DevColumn* col = s->col(field);
        require(col != nullptr, ESGPU_ERR_INVALID, std::string("no such column: ") + (field ? field : "(null)"));
        require(!col->multi && start + count <= s->max_doc, ESGPU_ERR_INVALID, "range out of bounds");
        const size_t w = col->type == ESGPU_COL_ORD_U32 ? 4 : 8;
        HIPX(hipSetDevice(s->ctx->device));
        const uint8_t* v = (const uint8_t*)(col->type == ESGPU_COL_I64 ? wide_i64(s->ctx, col, s, s->ctx->stream) : col->values.p);
        HIPX(hipMemcpy(out, v + start * w, count * w, hipMemcpyDeviceToHost));
    });
}

// ------------------------------------------------------------------------------------------------------------
// Global ordinals across the segments of a reader (GlobalOrdinalsBuilder.build -> Lucene OrdinalMap,
// GlobalOrdinalsBuilder.java:45-70, GlobalOrdinalMapping.java:51-58).  Segment dictionaries are sorted by unsigned
// bytes; their union in that order defines the global ordinals.  The dictionaries are merged on the host (once per
// reader, as Lucene does), then every segment's ordinal column is remapped on the GPU.
// ------------------------------------------------------------------------------------------------------------
struct esgpu_ordinal_map {
    std::shared_ptr<const TermDict> dict;
};

static std::string_view dict_view(const DevColumn* c, uint64_t o, std::string& scratch) { return c->dict->view(o, scratch); }

extern "C" int esgpu_ordinal_map_build(esgpu_ctx* ctx, esgpu_segment* const* segs, int32_t nsegs, const char* field,
                                       esgpu_ordinal_map** out) {
    return guarded([&] {
        require(ctx && segs && nsegs >= 1 && field && out, ESGPU_ERR_INVALID, "bad ordinal map arguments");
        HIPX(hipSetDevice(ctx->device));
        std::vector<DevColumn*> cols;
        for (int i = 0; i < nsegs; ++i) {
            require(segs[i] != nullptr, ESGPU_ERR_INVALID, "null segment");
            auto it = segs[i]->cols.find(field);
            if (it == segs[i]->cols.end()) { cols.push_back(nullptr); continue; }  // unmapped in this segment
            DevColumn* c = it->second.get();
            require(c->type == ESGPU_COL_ORD_U32, ESGPU_ERR_INVALID, "ordinal maps cover keyword columns");
            require(c->dict && !c->dict->numbered, ESGPU_ERR_INVALID, std::string("no term dictionary for ") + field);
            cols.push_back(c);
        }
        // k-way merge of the sorted segment dictionaries (unsigned byte order, BytesRef.compareTo)
        auto g = std::make_shared<TermDict>();
        g->offsets.push_back(0);
        std::vector<std::vector<uint32_t>> maps(cols.size());
        std::vector<uint64_t> pos(cols.size(), 0);
        std::vector<std::string> cur(cols.size()), scratch(cols.size());
        using Item = std::pair<std::string_view, int>;
        auto cmp = [](const Item& a, const Item& b) { return b.first < a.first || (a.first == b.first && b.second < a.second); };
        std::priority_queue<Item, std::vector<Item>, decltype(cmp)> heap(cmp);
        for (size_t k = 0; k < cols.size(); ++k) {
            if (!cols[k]) continue;
            maps[k].resize(cols[k]->value_count);
            if (cols[k]->value_count) heap.push({dict_view(cols[k], 0, scratch[k]), (int)k});
        }
        std::string last;
        bool have_last = false;
        while (!heap.empty()) {
            const auto [term, k] = heap.top();
            heap.pop();
            if (!have_last || term != std::string_view(last)) {
                last.assign(term.data(), term.size());
                have_last = true;
                g->bytes.insert(g->bytes.end(), last.begin(), last.end());
                g->offsets.push_back(g->bytes.size());
                g->n++;
                require(g->count() < 0xFFFFFFFFull, ESGPU_ERR_UNSUPPORTED, "more than 2^32-1 global ordinals");
            }
            const uint64_t o = pos[k]++;
            maps[k][o] = (uint32_t)(g->count() - 1);
            if (pos[k] < cols[k]->value_count) {
                const std::string_view nx = dict_view(cols[k], pos[k], scratch[k]);  // last == this segment's term
                require(std::string_view(last) < nx, ESGPU_ERR_INVALID, "segment dictionary not strictly sorted");
                heap.push({nx, k});
            }
        }
        g->seal();
        // remap every segment's column on the GPU: gvalues[d] = map[values[d]] (missing stays missing)
        for (size_t k = 0; k < cols.size(); ++k) {
            DevColumn* c = cols[k];
            if (!c) continue;
            DevBuf dmap;
            dmap.alloc(ctx, std::max<size_t>(maps[k].size(), 1) * 4);
            if (!maps[k].empty()) HIPX(hipMemcpy(dmap.p, maps[k].data(), maps[k].size() * 4, hipMemcpyHostToDevice));
            DevBuf gv;
            gv.alloc(ctx, c->values.bytes);
            launch_remap_ords(c->values.as<uint32_t>(), (uint32_t)(c->values.bytes / 4), dmap.as<uint32_t>(),
                              (uint32_t)maps[k].size(), gv.as<uint32_t>(), nullptr);
            HIPX(hipGetLastError());
            HIPX(hipDeviceSynchronize());
            {  // the 16-bit copy of the old ords() goes with it (a new buffer may reuse the old address)
                std::lock_guard<std::mutex> lk(ctx->mu);
                c->ord16.release();
                c->ord16_src = nullptr;
            }
            c->gvalues = std::move(gv);
            c->gdict = g;
        }
        std::unique_ptr<esgpu_ordinal_map> m(new esgpu_ordinal_map());
        m->dict = g;
        *out = m.release();
    });
}

extern "C" int esgpu_ordinal_map_value_count(const esgpu_ordinal_map* m, uint64_t* count) {
    return guarded([&] {
        require(m && count, ESGPU_ERR_INVALID, "null argument");
        *count = m->dict->count();
    });
}

extern "C" int esgpu_ordinal_map_lookup(const esgpu_ordinal_map* m, const uint8_t* term, size_t len, int64_t* ord) {
    return guarded([&] {
        require(m && ord && (term || len == 0), ESGPU_ERR_INVALID, "null argument");
        const TermDict& d = *m->dict;
        const std::string_view key((const char*)term, len);
        uint64_t lo = 0, hi = d.count();
        while (lo < hi) {  // lower bound in unsigned byte order
            const uint64_t mid = (lo + hi) / 2;
            const std::string_view t((const char*)d.bytes.data() + d.offsets[mid], (size_t)(d.offsets[mid + 1] - d.offsets[mid]));
            if (t < key) lo = mid + 1; else hi = mid;
        }
        *ord = -1;
        if (lo < d.count()) {
            const std::string_view t((const char*)d.bytes.data() + d.offsets[lo], (size_t)(d.offsets[lo + 1] - d.offsets[lo]));
            if (t == key) *ord = (int64_t)lo;
        }
    });
}

extern "C" int esgpu_ordinal_map_destroy(esgpu_ordinal_map* m) {
    return guarded([&] { delete m; });  // segments keep the dictionary they were remapped into
}

// ------------------------------------------------------------------------------------------------------------
// parser helpers (TermsParser + BucketCountThresholds.ensureValidity, TermsAggregator.java:63-85,
// BucketUtils.suggestShardSideQueueSize, bucket/BucketUtils.java:36-47)
// ------------------------------------------------------------------------------------------------------------
extern "C" int esgpu_terms_thresholds(int32_t size, int32_t shard_size, int64_t min_doc_count, int64_t shard_min_doc_count,
                                      int32_t order, int32_t nshards, int32_t* o_size, int32_t* o_shard_size,
                                      int64_t* o_min, int64_t* o_shard_min) {
    return guarded([&] {
        require(nshards >= 1, ESGPU_ERR_INVALID, "number_of_shards must be >= 1");
        if (size < 0) size = 10;                    // TermsParametersParser.java:35 defaults
        if (min_doc_count < 0) min_doc_count = 1;
        if (shard_min_doc_count < 0) shard_min_doc_count = 0;
        const bool term_order = order == ESGPU_ORDER_TERM_ASC || order == ESGPU_ORDER_TERM_DESC;
        if (shard_size < 0) {
            if (!term_order) {
                if (nshards == 1) shard_size = size;
                else {
                    const int64_t sample = (int64_t)size * std::min(10, nshards);
                    shard_size = (int32_t)std::min<int64_t>(INT32_MAX, std::max<int64_t>(10, sample));
                }
            } else {
                shard_size = size;  // default shard_size (-1) with term order keeps -1 -> size below
            }
        }
        if (shard_size == 0) shard_size = INT32_MAX;
        if (size == 0) size = INT32_MAX;
        if (shard_size < size) shard_size = size;
        if (shard_min_doc_count > min_doc_count) shard_min_doc_count = min_doc_count;
        require(size >= 0 && min_doc_count >= 0, ESGPU_ERR_INVALID,
                "parameters [requiredSize] and [minDocCount] must be >=0 in terms aggregation.");
        *o_size = size;
        *o_shard_size = shard_size;
        *o_min = min_doc_count;
        *o_shard_min = shard_min_doc_count;
    });
}

extern "C" int esgpu_murmur3_x64_128(const uint8_t* bytes, size_t len, int64_t seed, uint64_t* out2) {
    return guarded([&] {
        require(out2 && (bytes || len == 0), ESGPU_ERR_INVALID, "null argument");
        murmur3_x64_128(bytes, (int)len, (uint64_t)seed, &out2[0], &out2[1]);
    });
}

extern "C" int esgpu_java_double(double v, char* buf, size_t cap) {
    return guarded([&] {
        require(buf && cap >= 26, ESGPU_ERR_INVALID, "buffer under 26 bytes");
        const std::string s = java_double(v);
        std::memcpy(buf, s.c_str(), s.size() + 1);
    });
}

extern "C" int esgpu_date_rounding(const esgpu_agg_spec* spec, int32_t op, int64_t value, int64_t* out) {
    return guarded([&] {
        require(spec && out && op >= 0 && op <= 2, ESGPU_ERR_INVALID, "bad rounding arguments");
        require(spec->type == ESGPU_AGG_HISTOGRAM || spec->type == ESGPU_AGG_DATE_HISTOGRAM, ESGPU_ERR_INVALID,
                "not a histogram spec");
        Rounding r;
        try {
            r = Rounding::from_spec(*spec);
        } catch (const std::invalid_argument& e) {
            throw EsError(ESGPU_ERR_INVALID, e.what());
        }
        *out = op == 0 ? r.round(value) : op == 1 ? r.next_rounding_value(value) : r.round_key(value);
    });
}

// ------------------------------------------------------------------------------------------------------------
// index-time hashing (bulk ingest helpers)
// ------------------------------------------------------------------------------------------------------------
extern "C" int esgpu_routing_hash(const uint16_t* chars, size_t nchars, int32_t* hash) {
    return guarded([&] {
        require(hash && (chars || nchars == 0), ESGPU_ERR_INVALID, "null argument");
        require(nchars < (1u << 30), ESGPU_ERR_INVALID, "routing value too long");
        *hash = (int32_t)murmur3_x86_32_utf16(chars, (int)nchars, 0);
    });
}

// host CSR arrays -> device, kernel, results -> host (one synchronous round trip per batch)
template <class In, class Out, class Launch>
static void batch_hash(esgpu_ctx* c, const In* data, const uint64_t* offsets, uint64_t n, Out* out, Out* out2, Launch&& launch) {
    require(offsets && out && (data || n == 0), ESGPU_ERR_INVALID, "null argument");
    require(offsets[0] == 0, ESGPU_ERR_INVALID, "CSR offsets must start at 0");
    for (uint64_t i = 0; i < n; ++i) {
        require(offsets[i] <= offsets[i + 1], ESGPU_ERR_INVALID, "CSR offsets must be non-decreasing");
        require(offsets[i + 1] - offsets[i] < (1u << 30), ESGPU_ERR_INVALID, "value too long");
    }
    if (n == 0) return;
    HIPX(hipSetDevice(c->device));
    const uint64_t units = offsets[n];
    DevBuf d_data, d_off, d_out, d_out2;
    d_data.alloc(c, std::max<uint64_t>(units, 1) * sizeof(In));
    d_off.alloc(c, (n + 1) * 8);
    d_out.alloc(c, n * sizeof(Out));
    if (out2) d_out2.alloc(c, n * sizeof(Out));
    if (units) HIPX(hipMemcpyAsync(d_data.p, data, units * sizeof(In), hipMemcpyHostToDevice, c->stream));
    HIPX(hipMemcpyAsync(d_off.p, offsets, (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    launch(d_data.as<In>(), d_off.as<uint64_t>(), d_out.as<Out>(), out2 ? d_out2.as<Out>() : nullptr);
    HIPX(hipGetLastError());
    HIPX(hipMemcpyAsync(out, d_out.p, n * sizeof(Out), hipMemcpyDeviceToHost, c->stream));
    if (out2) HIPX(hipMemcpyAsync(out2, d_out2.p, n * sizeof(Out), hipMemcpyDeviceToHost, c->stream));
    HIPX(hipStreamSynchronize(c->stream));
}

extern "C" int esgpu_route_shards(esgpu_ctx* c, const uint16_t* chars, const uint64_t* offsets, uint64_t n, int32_t nshards,
                                  int32_t* hashes_out, int32_t* shards_out) {
    return guarded([&] {
        require(c != nullptr && nshards >= 1, ESGPU_ERR_INVALID, "bad routing arguments");
        std::lock_guard<std::mutex> lk(c->mu);
        batch_hash<uint16_t, int32_t>(c, chars, offsets, n, shards_out, hashes_out,
                                      [&](const uint16_t* d, const uint64_t* o, int32_t* shards, int32_t* hashes) {
                                          launch_route(d, o, n, nshards, hashes, shards, c->stream);
                                      });
    });
}

extern "C" int esgpu_murmur3_field(esgpu_ctx* c, const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1_out) {
    return guarded([&] {
        require(c != nullptr, ESGPU_ERR_INVALID, "null context");
        std::lock_guard<std::mutex> lk(c->mu);
        batch_hash<uint8_t, uint64_t>(c, bytes, offsets, n, h1_out, (uint64_t*)nullptr,
                                      [&](const uint8_t* d, const uint64_t* o, uint64_t* h1, uint64_t*) {
                                          launch_murmur3_field(d, o, n, h1, c->stream);
                                      });
    });
}

extern "C" int esgpu_precision_from_threshold(int64_t count, int32_t* precision) {
    return guarded([&] { *precision = hll_precision_from_threshold(count); });
}

// ------------------------------------------------------------------------------------------------------------
// plans
// ------------------------------------------------------------------------------------------------------------
static bool is_bucket(int t) { return t == ESGPU_AGG_TERMS || t == ESGPU_AGG_HISTOGRAM || t == ESGPU_AGG_DATE_HISTOGRAM; }
static bool is_metric(int t) { return t == ESGPU_AGG_STATS || t == ESGPU_AGG_EXTENDED_STATS || t == ESGPU_AGG_AVG; }

struct SpecNode {
    esgpu_agg_spec s;
    std::string name, field;
    std::string order_path;            // terms ordered by a sub-aggregation: the path, its child spec and metric key
    int order_child = -1;
    std::string order_key;
    std::vector<int> children;
    int precision = 14;
    std::vector<int64_t> tz_starts, tz_offs;  // owned copy of the spec's time zone table
    std::string time_zone = "UTC", format;    // wire-stream parameters (esgpu_agg_spec.time_zone / format)
    Rounding rounding() const {               // histogram specs (Rounding.java / TimeZoneRounding.java)
        esgpu_agg_spec sp = s;
        sp.tz_count = (int32_t)tz_starts.size();
        sp.tz_starts = tz_starts.data();
        sp.tz_offsets_ms = tz_offs.data();
        return Rounding::from_spec(sp);
    }
};

// cardinality under a bucket aggregation: one HyperLogLogPlusPlus sketch per bucket cell of the pipeline's grid
struct CardState {
    int spec = -1;
    int p = 9;
    std::string field;
    uint32_t m = 0, cap = 0, thr = 0;
    DevBuf regs, sets, cnt, nonzero;  // [B][m] u8, [B][cap] u32, [B], [B]
    DevBuf first;                     // [B][cap] u64: insertion order of each set entry (CardParams.first)
    // gathered rows of the emitted buckets (build)
    std::vector<uint8_t> h_regs;
    std::vector<uint32_t> h_sets, h_cnt, h_nz;
    std::vector<uint64_t> h_first;
};

// host views of one pipeline's cells (its pinned staging buffers), gathered rows or the whole grid
struct HostCells {
    const unsigned long long* cnt = nullptr;
    const unsigned long long* vcnt = nullptr;
    const unsigned long long* mn = nullptr;
    const unsigned long long* mx = nullptr;
    const double* sum = nullptr;
    const double* sq = nullptr;
};

// One cell grid ([H][T]: outer / inner bucket dimensions) with its leaf metrics, collected by one kernel launch.
struct Pipeline {
    int root = -1;             // spec index of the top-level aggregation (for a filter's children: the child)
    int kind = 0;              // 0 = cell grid (bucket / metric), 1 = cardinality
    int fspec = -1;            // enclosing filter aggregation (FilterAggregator): its clauses apply too; -1 = none
    bool count_only = false;   // the filter aggregation's own doc_count (one cell, no metric)
    // cell grid shape
    int outer = -1, inner = -1;      // bucket spec indices (inner may be -1)
    int term_spec = -1, hist_spec = -1;
    std::vector<int> metrics;        // leaf specs at the deepest level, in request order (numeric metrics + cardinality)
    std::vector<CardState> cards;    // cardinality leaves (spec order)
    std::string ord_field, hist_field, metric_field;
    // histogram under histogram: the inner histogram's key indices are the ordinal dimension (ord_field = its field),
    // derived per segment into ord_col (affine rounding ord_interval / ord_offset; keys ord_key0 .. + ord_keys - 1, fixed
    // by the request's first segment)
    bool ord_hist = false;
    int64_t ord_interval = 1, ord_offset = 0, ord_key0 = 0;
    uint32_t ord_keys = 0;
    // ... or a calendar / DST rounding (ord_table): the bucket table over the request's inner values (key_table: step
    // starts, sorted keys, step -> key slot), the key index being the slot of the value's step
    bool ord_table = false;
    Rounding ord_rnd;
    int64_t ot_lo = 0, ot_hi = -1;
    std::vector<int64_t> ot_start, ot_key;
    std::vector<uint32_t> ot_slot;
    DevBuf d_ostart, d_oslot;
    std::shared_ptr<DevColumn> ord_col;
    int met = 0;                     // 0 none, 1 avg, 2 stats, 3 extended
    int64_t interval = 1, offset = 0;  // affine roundings: key = floor((v - offset) / interval) * interval + offset
    Rounding rnd;                    // the histogram spec's rounding
    bool ktable = false;             // non-affine rounding: bucket start table instead of the affine map
    int64_t kt_lo = 0, kt_hi = -1;   // value range the table covers
    std::vector<int64_t> kt_start, kt_key;  // step start instants, [H] bucket keys (es_rounding.hpp key_table)
    std::vector<uint32_t> kt_slot;   // bucket of each step (empty: steps are buckets)
    DevBuf d_kstart, d_kslot;        // device copies
    // device state
    bool allocated = false;
    uint32_t T = 1, H = 1;
    uint64_t value_count = 1;        // terms: the global ordinal count (T is max(value_count, 1))
    int64_t key0 = 0;
    bool keyed = false;              // the key range has been taken from a segment's values (else H == 1, key0 == 0)
    bool inner_terms = false;        // terms under terms: the key dimension is the inner terms field's ordinals
    std::shared_ptr<const TermDict> tdict2;  // inner terms: the dictionary its keys resolve through
    // three bucket levels (two terms and one histogram): the ordinal dimension is the pair of the two terms fields,
    // ord = a * vcB + b (ord_field = a's field, ord_field2 = b's), derived per segment into ord_col
    bool cnt32 = false;              // g_cnt holds u32 counts (written by the partitioned / hot-cold terms paths)
    bool zero_pending = false;       // g_cnt not zeroed since the plan's reset yet (zero_counts)
    bool comp = false;
    int comp_spec2 = -1;
    // terms under terms whose [outer x inner] grid is over the dense budget (ESGPU_DEFER_CELLS, default 2^31 cells):
    // `deferred` -- this inner-terms pipeline counts only the outer doc counts while collecting, and its bucket child is
    // collected again at build over the surviving outer buckets (TermsAggregator's breadth_first mode,
    // BestBucketsDeferringCollector.prepareSelectedBuckets) by the companion `replay` pipelines: a composite grid over
    // (winner slot, inner ordinal), ord = slot * vcB + b, derived per retained segment through `slot_map`
    bool can_defer = false, deferred = false, replay = false;
    std::string ord_field2;
    std::shared_ptr<const TermDict> tdictB;
    uint64_t vcA = 0, vcB = 0;
    uint64_t value_count2 = 0;       // inner terms: its global ordinal count (H is max(value_count2, 1))
    int vcnt_mode = 0, ocnt_mode = OCNT_NONE;
    DevBuf g_cnt, g_ocnt, g_vcnt, g_sum, g_min, g_max, g_sq;
    // compensated sums (CollectParams.g_sum_lo): on once the request's metric partial sums can round -- a double metric,
    // or |values| x values (x |values| for sums of squares) reaching 2^53 over the segments collected so far
    DevBuf g_sum_lo, g_sq_lo;        // zero between collects
    bool dd = false;
    uint64_t dd_vals = 0, dd_amax = 0;
    // cardinality state
    int p = 14;
    DevBuf regs, lc_set, lc_count;
    DevBuf fs_buf;                   // floored-stream HLL: entries by register range (grown on demand)
    DevBuf lc_first;                 // [lc_mask + 1] u64: insertion order of each LC set entry (HllParams.lc_first)
    uint32_t lc_mask = 0, lc_threshold = 0;
    uint64_t hll_seen = 0;           // values hashed into the registers by earlier segments of this request
    bool hll_snap_ok = false;        // the last launch_hll left the group floors and snapshot as register lower bounds
    // the request's first segment, when it was collected dense (its registers alone then estimate its distinct values at
    // build), the segments collected, and the largest distinct estimate among them
    std::shared_ptr<std::atomic<double>> hll_d1;
    // the registers right after that first segment, kept when more segments may follow and its distinct count is not
    // known yet: estimated at build, so the segment's next request can take the floored stream
    DevBuf hll_r1;
    bool hll_r1_pending = false;
    int hll_nseg = 0;
    double hll_dmax = 0.0;
    bool lc_dirty = true;            // lc_set / lc_first may hold entries (cleared at reset only then)
    // post_collection products
    std::vector<uint8_t> h_regs;
    std::vector<uint32_t> h_lc;
    int hll_mode = 0;
    bool any_value = false;
    // the term dictionary the terms keys resolve through (the first collected segment's; every later segment must
    // number its terms the same way) -- shared, so it outlives the segments
    std::shared_ptr<const TermDict> tdict;
    bool fresh = true;               // no segment collected since create / reset: the grid shape is (re)derived
    // timing of this pipeline's collect launch on the plan stream
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool timed = false;
    uint64_t occ_key = ~0ull;   // cached occupancy of the last launch configuration
    int occ = 1;
    // build: the pipeline's cells on the host (gathered winner rows or the whole grid) and their staging buffers
    HostCells hc;
    PinnedBuf h_cells[6], h_ocnt;
    PinnedBuf h_picks, h_rowtot;     // terms under a histogram: per-row picks and totals (row_topk_kernel)
};

// One aggregation subtree (a top-level aggregation, or a child of a top-level filter aggregation) compiled to one or
// more pipelines.  A bucket aggregation's children are split over pipelines so that each pipeline's grid has at most
// one inner bucket dimension and one metric field: its metric children grouped by field, each bucket child (with its
// own metric children grouped by field) in pipelines of its own -- the way AggregatorFactories.createSubAggregators
// (A/AggregatorFactories.java:68-79) gives every child its own aggregator behind BucketCollector.wrap
// (A/BucketCollector.java:59).  Every pipeline counts the outer buckets alike; pipes[0]'s counts pick the buckets.
struct LeafRef { int pipe = -1, leaf = -1; };  // a metric / cardinality spec: its pipeline and index in pl.metrics
struct ChildSrc {
    int spec = -1;
    bool bucket = false;
    bool filter = false;             // a filter aggregation (FilterAggregator): pipes = its doc counts per outer bucket
                                     // (pipes[0]) and its metric children (grand), all under its clauses
    LeafRef leaf;                    // metric / cardinality child
    std::vector<int> pipes;          // bucket child: pipelines carrying it (pipes[0]'s counts define its buckets)
    std::vector<LeafRef> grand;      // bucket child: its children in request order (a deep child excluded)
    // a bucket child X whose last child is a bucket aggregation Y (three levels): Y's spec, the shape (1: terms{terms{
    // histogram}}, 2: terms{histogram{terms}}, 3: histogram{terms{terms}}), Y's composite pipelines and leaf refs
    int deep = -1, deep_shape = 0;
    std::vector<int> dpipes;
    std::vector<LeafRef> dgrand;
    // terms under terms: the breadth-first replay pipelines (parallel to pipes) and the leaves' refs into them
    std::vector<int> rpipes;
    std::vector<LeafRef> rgrand;
};
struct Group {
    int root = -1, fspec = -1;
    std::vector<int> pipes;          // pipes[0] holds the outer doc counts
    std::vector<ChildSrc> kids;      // bucket root: its children in request order
};

constexpr uint32_t kZuSlots = 64;  // zone-skip counters per collect call (esgpu_plan.s_zu)
constexpr uint32_t kZuMaxWG = 2048;  // ... each one word per zone-keys workgroup (a segment has < 2^19 blocks)

struct esgpu_plan {
    esgpu_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::vector<SpecNode> specs;
    std::vector<esgpu_filter> filters;
    std::vector<std::string> filter_fields;
    std::vector<int> filter_owner;             // -1 = query clause (bool.filter); k = clause of filter aggregation spec k
    std::vector<std::string> filter_lo, filter_hi;  // owned copies of keyword range bounds (the caller's may not outlive create)
    std::vector<int> tops;                     // top-level spec indices in request order
    std::vector<Pipeline> pipes;
    std::vector<Group> groups;                 // top-level subtrees (and filter aggregations' children) in request order
    bool collected = false, posted = false;
    double last_ms = 0;
    uint64_t last_bytes = 0;
    double b_wait = 0, b_total = 0;  // last build: stream waits / whole call (ms)
    bool b_trace = false;
    std::vector<std::pair<const char*, double>> b_marks;
    // co-located reduce (esgpu_plans_build_reduce): the build stops after the terms selection (buckets with empty
    // sub-aggregations) and keeps the winners' ordinals for the device merge of their rows
    bool skeleton = false;
    std::vector<uint32_t> sk_ords;
    PinnedBuf h_colo;   // the merged rows (pinned, device-mapped)
    PinnedBuf h_colo_meta;  // shard descriptors + the rows table (pinned, device-mapped: read once per workgroup)
    PinnedBuf h_colo_tot;   // every shard's per-ordinal doc counts, or its picks (pinned, device-mapped)
    Scratch s_colo_tot;     // every shard's per-ordinal doc counts (device selection)
    // the co-located reduce across ranks (esgpu_comm_build_reduce): local and all-gathered selection records, the packed
    // rows sent and received, the records on the host, the pack's descriptors; the event other local plans wait on
    Scratch s_xr_picks, s_xr_allpicks, s_xr_send, s_xr_recv;
    PinnedBuf h_xr_picks, h_xr_meta, h_xr_hdr;
    hipEvent_t ev_xr = nullptr;
    int32_t last_path = 0;
    // per-request scratch, reused across requests
    Scratch s_accept, s_tcnt, s_rows, s_dst[6];
    Scratch s_wgc, s_pbeg, s_pbuf, s_tiles, s_cand, s_keys, s_hist;  // partitioned counting + GPU top-k
    Scratch s_fbits, s_vbits;  // doc bitset of multi-valued filters, per-value bitset of a multi-valued HLL field
    Scratch s_cells;           // cell list of a cardinality gather
    Scratch s_zkey;            // per-block key ranges of a windowed collect
    // block-delta collects: the docs of zone blocks whose timestamps the kernel did not read (one key per block), one
    // device word per launch of the current collect call, copied into zu_host; taken off last_bytes by the stats call
    Scratch s_zu;
    PinnedBuf zu_host;
    uint32_t zu_n = 0;
    uint8_t zu_w[kZuSlots] = {};  // ... and the timestamp bytes per doc of each launch (2: block deltas, 4: 32-bit deltas)
    uint32_t zu_g[kZuSlots] = {};  // ... and its zone-keys workgroups (words written)
    DevBuf d_claim;            // collect kernel's chunk-claim counter pair (zeroed once; every launch leaves it zero)
    Scratch s_hcur, s_hused, s_hslab;  // hot/cold counting: overflow cursors, static-region fills, hot slabs
    PinnedBuf h_hcerr;         // hot/cold counting: capacity-violation word (written by the scatter kernel)
    bool hc_check = false;     // a hot/cold collect ran since the last post_collection
    // a single-segment plain terms request in count order on the postings form: the cold lists' counting deferred to
    // the top-k, which runs it only when the hot slots do not settle the winners (collect_hotcold, hc_topk_launch)
    struct HcPending {
        bool on = false;
        bool filtered = false;  // a filter / accept bits: `cold` is the scatter form's parameters (the fallback)
        int pipe = -1;
        HcParams hot{}, cold{};
        std::shared_ptr<const HcStats> hs;  // keeps the segment statistics' buffers the two passes read
    } hc_pend;
    Scratch s_slot_tot, s_hcand, s_hhist, s_hkeys, s_hskip, s_cold_tot, s_hbits;
    PinnedBuf h_keys;
    hipEvent_t ev_mid = nullptr;
    PinnedBuf h_tcnt, h_rows, h_dst[6];
    Scratch s_nnz;                     // build: non-empty slots per winner row (compact_rows)
    Scratch s_drows;                   // build: composite ordinals a three-level child reads (fetch_rows)
    bool sparse_dead = false;          // the current segment's accept bitset clears few docs (host sample, <= 10 %)
    Scratch s_xbits;                   // doc bitset of a pipeline with more than kMaxPreds clauses
    uint32_t seg_seq = 0;              // segments collected since create / reset (cardinality insertion order)
    uint64_t docs_seen = 0;            // max_doc summed over those segments (u32 terms counts need it below 2^32)
    std::vector<PinnedBuf> h_compact;  // build: per bucket child, its GPU-compacted buckets and leaves (pinned)
    // breadth-first replay: the segments collected while a pipeline was deferred (pinned until reset / destroy) with a
    // device copy of each one's accept bits, and the outer ordinal -> winner slot map of the replay being run
    struct DeferredSeg { const esgpu_segment* s; int accept; };
    std::vector<DeferredSeg> dsegs;
    std::vector<DevBuf> d_daccept;
    Scratch s_slotmap;
    const uint32_t* slot_map = nullptr;
    uint32_t slot_map_n = 0, slot_k = 0;
    Scratch s_rkeys;                   // replay: per winner, the GPU top-k's keys and row total
    PinnedBuf h_rkeys;
    Scratch s_rregion, s_rmeta;        // compacted replay: the batches' regions; region offsets, capacities, fills
    Scratch s_rkeys2;                  // replay rows selected batch by batch (term orders, large shard sizes)
    PinnedBuf h_rfill, h_rcand;        // compacted replay fills; large inner top-k: row sum + candidates
    void unpin_all() {
        for (const DeferredSeg& d : dsegs) unpin_segment(d.s);
        dsegs.clear();
    }
};

static int metric_level(int t) { return t == ESGPU_AGG_AVG ? 1 : t == ESGPU_AGG_STATS ? 2 : 3; }

static int64_t key_value(const Pipeline& pl, uint32_t slot) {
    return pl.ktable ? pl.kt_key[slot] : (pl.key0 + (int64_t)slot) * pl.interval + pl.offset;
}

// a pipeline over the outer (and optional inner) bucket spec with the given leaves (metric specs of one field and/or
// cardinality specs), appended to p->pipes; returns its index
static int add_pipeline(esgpu_plan* p, int root, int fspec, int outer, int inner, const std::vector<int>& leaves) {
    Pipeline pl;
    pl.root = root;
    pl.fspec = fspec;
    pl.outer = outer;
    pl.inner = inner;
    pl.metrics = leaves;
    for (int b : {outer, inner}) {
        if (b < 0) continue;
        const SpecNode& n = p->specs[b];
        if (n.s.type == ESGPU_AGG_TERMS && b == inner && outer >= 0 && p->specs[outer].s.type == ESGPU_AGG_TERMS) {
            // terms under terms: the inner field's ordinals are the key dimension (key = ordinal)
            pl.hist_spec = b;
            pl.hist_field = n.field;
            pl.inner_terms = true;
            pl.interval = 1;
            pl.offset = 0;
        } else if (n.s.type == ESGPU_AGG_TERMS) { pl.term_spec = b; pl.ord_field = n.field; }
        else if (b == inner && outer >= 0 && p->specs[outer].s.type != ESGPU_AGG_TERMS) {
            // histogram under histogram: the inner histogram's key indices take the ordinal dimension of the grid
            pl.term_spec = b;
            pl.ord_field = n.field;
            pl.ord_hist = true;
            Rounding r;
            try {
                r = n.rounding();
            } catch (const std::invalid_argument& e) {
                throw EsError(ESGPU_ERR_INVALID, std::string(e.what()) + " for histogram aggregation [" + n.name + "]");
            }
            if (!r.affine(&pl.ord_interval, &pl.ord_offset)) {  // calendar units, DST zones: a bucket table
                pl.ord_table = true;
                pl.ord_rnd = r;
                pl.ord_interval = 0;
            }
        } else {
            pl.hist_spec = b;
            pl.hist_field = n.field;
            try {
                pl.rnd = n.rounding();
            } catch (const std::invalid_argument& e) {
                throw EsError(ESGPU_ERR_INVALID, std::string(e.what()) + " for histogram aggregation [" + n.name + "]");
            }
            pl.ktable = !pl.rnd.affine(&pl.interval, &pl.offset);
        }
    }
    for (int m : leaves) {
        const SpecNode& n = p->specs[m];
        if (n.s.type == ESGPU_AGG_CARDINALITY) {
            CardState cs;
            cs.spec = m;
            cs.p = n.precision;
            cs.field = n.field;
            cs.m = 1u << cs.p;
            cs.thr = (uint32_t)((float)(cs.m / 4) * 0.75f);  // Hashset threshold (HyperLogLogPlusPlus.java:437-440)
            cs.cap = 16;
            while (cs.cap < 4 * (cs.thr + 1)) cs.cap <<= 1;
            pl.cards.push_back(std::move(cs));
            continue;
        }
        if (pl.metric_field.empty()) pl.metric_field = n.field;
        pl.met = std::max(pl.met, metric_level(n.s.type));
    }
    p->pipes.push_back(std::move(pl));
    return (int)p->pipes.size() - 1;
}

// leaves grouped into pipelines: one per metric field (first-appearance order), cardinality leaves with the first;
// `refs` gets each leaf's (pipeline, index); a bucket with no leaves still gets one pipeline for its counts
static std::vector<int> add_leaf_pipelines(esgpu_plan* p, int root, int fspec, int outer, int inner, const std::vector<int>& leaves,
                                           std::vector<LeafRef>* refs) {
    std::vector<std::string> fields;
    std::vector<std::vector<int>> by;
    std::vector<int> cards;
    for (int m : leaves) {
        if (p->specs[m].s.type == ESGPU_AGG_CARDINALITY) { cards.push_back(m); continue; }
        const std::string& f = p->specs[m].field;
        size_t k = std::find(fields.begin(), fields.end(), f) - fields.begin();
        if (k == fields.size()) { fields.push_back(f); by.emplace_back(); }
        by[k].push_back(m);
    }
    if (by.empty()) by.emplace_back();
    by[0].insert(by[0].end(), cards.begin(), cards.end());
    std::vector<int> idx;
    for (const auto& g : by) idx.push_back(add_pipeline(p, root, fspec, outer, inner, g));
    refs->assign(leaves.size(), LeafRef{});
    for (size_t j = 0; j < leaves.size(); ++j)
        for (int pi : idx) {
            const auto& ms = p->pipes[pi].metrics;
            const auto it = std::find(ms.begin(), ms.end(), leaves[j]);
            if (it != ms.end()) (*refs)[j] = LeafRef{pi, (int)(it - ms.begin())};
        }
    return idx;
}

// x is -1 or a filter aggregation whose ancestors are all filter aggregations (a chain of filters from the top)
static bool filter_chain_to_top(const esgpu_plan* p, int x) {
    for (; x >= 0; x = p->specs[x].s.parent)
        if (p->specs[x].s.type != ESGPU_AGG_FILTER) return false;
    return true;
}

static Group compile_group(esgpu_plan* p, int r, int fspec) {
    Group g;
    g.root = r;
    g.fspec = fspec;
    const SpecNode& root = p->specs[r];
    if (root.s.type == ESGPU_AGG_CARDINALITY) {
        Pipeline pl;
        pl.root = r;
        pl.fspec = fspec;
        pl.kind = 1;
        pl.p = root.precision;
        pl.metric_field = root.field;
        p->pipes.push_back(std::move(pl));
        g.pipes.push_back((int)p->pipes.size() - 1);
        return g;
    }
    if (is_metric(root.s.type)) {
        g.pipes.push_back(add_pipeline(p, r, fspec, -1, -1, {r}));
        return g;
    }
    require(is_bucket(root.s.type), ESGPU_ERR_UNSUPPORTED, "aggregation type not on the GPU path");
    std::vector<int> leaves;
    for (int ch : root.children) {
        const int t = p->specs[ch].s.type;
        if (is_metric(t) || t == ESGPU_AGG_CARDINALITY) leaves.push_back(ch);
        else if (t == ESGPU_AGG_FILTER) continue;  // its own pipelines below (under the enclosing filters' clauses too)
        else if (!is_bucket(t)) throw EsError(ESGPU_ERR_UNSUPPORTED, "aggregation type not on the GPU path");
    }
    std::vector<LeafRef> leaf_refs;
    bool have_bucket_child = false, have_filter_child = false;
    for (int ch : root.children) {
        have_bucket_child |= is_bucket(p->specs[ch].s.type);
        have_filter_child |= p->specs[ch].s.type == ESGPU_AGG_FILTER;
    }
    // the outer level's own pipelines (also: a bucket with no children, and one with a filter child, whose pipelines
    // count only the filter's docs -- pipes[0] must count every doc of the outer buckets)
    if (!leaves.empty() || !have_bucket_child || have_filter_child)
        for (int pi : add_leaf_pipelines(p, r, fspec, r, -1, leaves, &leaf_refs)) g.pipes.push_back(pi);
    size_t li = 0;
    for (int ch : root.children) {
        ChildSrc cs;
        cs.spec = ch;
        if (p->specs[ch].s.type == ESGPU_AGG_FILTER) {
            // FilterAggregator under a bucket aggregation (A/bucket/filter/FilterAggregator.java:57-70): per outer bucket,
            // the docs matching its clauses counted, and its metric children collected over them -- outer-level pipelines
            // carrying the filter's clauses (a filter with no children still gets one for its doc counts)
            cs.filter = true;
            std::vector<int> fl;
            for (int gc : p->specs[ch].children) {
                const int t = p->specs[gc].s.type;
                require(is_metric(t) || t == ESGPU_AGG_CARDINALITY, ESGPU_ERR_UNSUPPORTED,
                        "bucket aggregations under a filter aggregation under a bucket aggregation run on the CPU path");
                fl.push_back(gc);
            }
            cs.pipes = add_leaf_pipelines(p, r, ch, r, -1, fl, &cs.grand);
            for (int pi : cs.pipes) g.pipes.push_back(pi);
        } else if (!is_bucket(p->specs[ch].s.type)) {
            cs.leaf = leaf_refs[li++];
        } else {
            cs.bucket = true;
            std::vector<int> inner_leaves;
            const std::vector<int>& xc = p->specs[ch].children;
            for (size_t q = 0; q < xc.size(); ++q) {
                const int t = p->specs[xc[q]].s.type;
                if (is_bucket(t) && q + 1 == xc.size()) { cs.deep = xc[q]; continue; }
                require(is_metric(t) || t == ESGPU_AGG_CARDINALITY, ESGPU_ERR_UNSUPPORTED,
                        "a bucket aggregation three levels deep other than the last sub-aggregation runs on the CPU path");
                inner_leaves.push_back(xc[q]);
            }
            cs.pipes = add_leaf_pipelines(p, r, fspec, r, ch, inner_leaves, &cs.grand);
            for (int pi : cs.pipes) g.pipes.push_back(pi);
            if (cs.deep >= 0) {  // three levels: two terms and one histogram (the histogram at any level)
                const SpecNode& Y = p->specs[cs.deep];
                std::vector<int> yl;
                for (int gc : Y.children) {
                    const int t = p->specs[gc].s.type;
                    require(is_metric(t) || t == ESGPU_AGG_CARDINALITY, ESGPU_ERR_UNSUPPORTED, "bucket aggregations nested four levels deep");
                    yl.push_back(gc);
                }
                const bool rt = root.s.type == ESGPU_AGG_TERMS, xt = p->specs[ch].s.type == ESGPU_AGG_TERMS,
                           yt = Y.s.type == ESGPU_AGG_TERMS;
                require((int)rt + (int)xt + (int)yt == 2, ESGPU_ERR_UNSUPPORTED,
                        "three bucket levels other than two terms and one histogram run on the CPU path");
                cs.deep_shape = rt && xt ? 1 : rt ? 2 : 3;
                // the composite pipelines: shape 1 [Y keys][R x X], shape 2 [X keys][R x Y], shape 3 [R keys][X x Y]
                const int outer_b = cs.deep_shape == 1 ? cs.deep : ch;
                cs.dpipes = add_leaf_pipelines(p, r, fspec, r, outer_b, yl, &cs.dgrand);
                for (int pi : cs.dpipes) {
                    Pipeline& D = p->pipes[pi];
                    D.comp = true;
                    D.comp_spec2 = cs.deep_shape == 1 ? ch : cs.deep;
                    D.ord_field2 = p->specs[D.comp_spec2].field;
                    g.pipes.push_back(pi);
                }
            }
            // terms under terms with numeric-metric leaves: replay pipelines for a grid over the dense budget
            // (collected at build over the surviving outer buckets only; not in g.pipes, so never collected per segment)
            bool defer_ok = root.s.type == ESGPU_AGG_TERMS && p->specs[ch].s.type == ESGPU_AGG_TERMS && cs.deep < 0;
            for (int m : inner_leaves) defer_ok = defer_ok && is_metric(p->specs[m].s.type);
            if (defer_ok) {
                cs.rpipes = add_leaf_pipelines(p, r, fspec, ch, -1, inner_leaves, &cs.rgrand);
                for (int pi : cs.rpipes) {
                    Pipeline& R = p->pipes[pi];
                    R.comp = true;
                    R.replay = true;
                    R.comp_spec2 = ch;
                    R.ord_field = p->specs[r].field;
                    R.ord_field2 = p->specs[ch].field;
                }
                for (int pi : cs.pipes) p->pipes[pi].can_defer = true;
            }
        }
        g.kids.push_back(std::move(cs));
    }
    // a terms aggregation ordered by a metric child: that child's pipeline must hold the selection (it is a direct
    // child, so its pipeline is an outer-level one)
    return g;
}

extern "C" int esgpu_plan_create(esgpu_ctx* c, const esgpu_agg_spec* specs, int32_t nspecs, const esgpu_filter* filters,
                                 int32_t nfilters, esgpu_plan** out) {
    return guarded([&] {
        require(c && out && (nspecs == 0 || specs), ESGPU_ERR_INVALID, "null argument");
        require(nfilters >= 0, ESGPU_ERR_INVALID, "negative filter count");
        std::unique_ptr<esgpu_plan> p(new esgpu_plan());
        p->ctx = c;
        p->specs.resize(nspecs);
        std::vector<int> tops;
        for (int i = 0; i < nspecs; ++i) {
            SpecNode& n = p->specs[i];
            n.s = specs[i];
            n.name = specs[i].name ? specs[i].name : "";
            n.field = specs[i].field ? specs[i].field : "";
            n.s.name = nullptr;
            n.s.field = nullptr;
            if (is_bucket(n.s.type) && n.s.type != ESGPU_AGG_TERMS && specs[i].tz_count > 0) {
                require(specs[i].tz_starts && specs[i].tz_offsets_ms, ESGPU_ERR_INVALID, "time zone table without arrays");
                n.tz_starts.assign(specs[i].tz_starts, specs[i].tz_starts + specs[i].tz_count);
                n.tz_offs.assign(specs[i].tz_offsets_ms, specs[i].tz_offsets_ms + specs[i].tz_count);
            }
            n.s.tz_starts = nullptr;
            n.s.tz_offsets_ms = nullptr;
            n.s.tz_count = 0;
            if (specs[i].time_zone && *specs[i].time_zone) n.time_zone = specs[i].time_zone;
            require(n.s.value_format >= ESGPU_FORMAT_RAW && n.s.value_format <= ESGPU_FORMAT_NUMBER, ESGPU_ERR_INVALID,
                    "unknown value format");
            if (n.s.value_format != ESGPU_FORMAT_RAW) {
                require(specs[i].format != nullptr, ESGPU_ERR_INVALID, "value format without a pattern");
                n.format = specs[i].format;
            }
            n.s.time_zone = nullptr;
            n.s.format = nullptr;
            require(n.s.type >= ESGPU_AGG_TERMS && n.s.type <= ESGPU_AGG_FILTER, ESGPU_ERR_INVALID, "unknown aggregation type");
            if (n.s.type == ESGPU_AGG_FILTER && n.s.parent >= 0) {
                // a chain of filter aggregations from the top (each one's docs: its clauses and its ancestors'), or a
                // filter directly under a bucket aggregation of the first bucket level (compile_group)
                require(n.s.parent < i, ESGPU_ERR_INVALID, "parent must precede child");
                const SpecNode& par = p->specs[n.s.parent];
                require((par.s.type == ESGPU_AGG_FILTER && filter_chain_to_top(p.get(), n.s.parent)) ||
                            (is_bucket(par.s.type) && filter_chain_to_top(p.get(), par.s.parent)),
                        ESGPU_ERR_UNSUPPORTED, "a filter aggregation below the first bucket level runs on the CPU path");
            }
            if (n.s.parent < 0) tops.push_back(i);
            else {
                require(n.s.parent < i, ESGPU_ERR_INVALID, "parent must precede child");
                const int pt = p->specs[n.s.parent].s.type;
                require(is_bucket(pt) || pt == ESGPU_AGG_FILTER, ESGPU_ERR_INVALID, "metrics aggregations cannot have sub-aggregations");
                p->specs[n.s.parent].children.push_back(i);
            }
            if (n.s.type >= ESGPU_AGG_SUM && n.s.type <= ESGPU_AGG_VALUE_COUNT)
                throw EsError(ESGPU_ERR_UNSUPPORTED, "sum/min/max/value_count run on the CPU path");
            if (n.s.type == ESGPU_AGG_TERMS) {
                require(n.s.size >= 0 && n.s.min_doc_count >= 0, ESGPU_ERR_INVALID,
                        "parameters [requiredSize] and [minDocCount] must be >=0 in terms aggregation.");
                require((n.s.order >= ESGPU_ORDER_COUNT_DESC && n.s.order <= ESGPU_ORDER_TERM_DESC) ||
                            n.s.order == ESGPU_ORDER_AGG_ASC || n.s.order == ESGPU_ORDER_AGG_DESC,
                        ESGPU_ERR_INVALID, "unknown terms order");
                if (n.s.order == ESGPU_ORDER_AGG_ASC || n.s.order == ESGPU_ORDER_AGG_DESC) {
                    require(specs[i].order_path != nullptr, ESGPU_ERR_INVALID, "terms order by sub-aggregation without a path");
                    n.order_path = specs[i].order_path;
                }
            }
            n.s.order_path = nullptr;
            if (n.s.type == ESGPU_AGG_CARDINALITY) {
                if (n.s.precision_threshold >= 0) n.precision = hll_precision_from_threshold(n.s.precision_threshold);
                else {
                    int pr = 14;  // CardinalityAggregatorFactory.defaultPrecision
                    for (int q = n.s.parent; q >= 0; q = p->specs[q].s.parent) if (is_bucket(p->specs[q].s.type)) pr -= 5;
                    n.precision = std::max(pr, 4);
                }
            }
        }
        p->filter_lo.resize(nfilters);
        p->filter_hi.resize(nfilters);
        for (int k = 0; k < nfilters; ++k) {
            require(filters[k].field != nullptr, ESGPU_ERR_INVALID, "filter without field");
            const int owner = filters[k].owner - 1;  // 0 = query clause, k + 1 = clause of filter aggregation spec k
            require(owner >= -1 && owner < nspecs && (owner < 0 || p->specs[owner].s.type == ESGPU_AGG_FILTER), ESGPU_ERR_INVALID,
                    "filter clause owner is not a filter aggregation");
            p->filters.push_back(filters[k]);
            p->filter_fields.push_back(filters[k].field);
            p->filter_owner.push_back(owner);
            esgpu_filter& f = p->filters.back();
            if (f.lo_term) { p->filter_lo[k].assign((const char*)f.lo_term, (size_t)f.lo_term_len); f.lo_term = (const uint8_t*)p->filter_lo[k].data(); }
            if (f.hi_term) { p->filter_hi[k].assign((const char*)f.hi_term, (size_t)f.hi_term_len); f.hi_term = (const uint8_t*)p->filter_hi[k].data(); }
            f.field = nullptr;  // filter_fields[k] holds it
        }
        // every pipeline evaluates the query clauses plus those of its filter aggregation (set_preds folds more than
        // kMaxPreds of them into a doc bitset)
        for (int r = 0; r < nspecs; ++r) {
            if (p->specs[r].s.type != ESGPU_AGG_FILTER) continue;
            int own = 0;
            for (int o : p->filter_owner) own += o == r;
            require(own >= 1, ESGPU_ERR_INVALID, "filter aggregation without a filter clause");
            for (int ch : p->specs[r].children)  // filters under a filter: only on a chain of filters from the top
                require(p->specs[ch].s.type != ESGPU_AGG_FILTER || filter_chain_to_top(p.get(), r), ESGPU_ERR_UNSUPPORTED,
                        "a filter aggregation below the first bucket level runs on the CPU path");
        }
        p->tops = tops;
        // terms ordered by a sub-aggregation: AggregationPath.validate (A/support/AggregationPath.java:289-347)
        for (SpecNode& n : p->specs) {
            if (n.s.type != ESGPU_AGG_TERMS || (n.s.order != ESGPU_ORDER_AGG_ASC && n.s.order != ESGPU_ORDER_AGG_DESC)) continue;
            std::string name, key;
            require(parse_order_path(n.order_path, &name, &key), ESGPU_ERR_INVALID,
                    "Invalid path element in path [" + n.order_path + "]");
            for (int ch : n.children) if (p->specs[ch].name == name) n.order_child = ch;
            require(n.order_child >= 0, ESGPU_ERR_INVALID, "Invalid term-aggregator order path [" + n.order_path +
                    "]. Unknown aggregation [" + name + "]");
            const int t = p->specs[n.order_child].s.type;
            if (t == ESGPU_AGG_CARDINALITY) {
                // CardinalityAggregator.metric(bucketOrd) = counts.cardinality(bucketOrd) (a single-value metric): every
                // candidate ordinal's sketch estimate, derived at build from the sketches gathered beside the cells
                // (order_value), at the top level or under other bucket levels
                require(key.empty() || key == "value", ESGPU_ERR_INVALID, "Invalid terms aggregation order path [" + n.order_path +
                        "]. Ordering on a single-value metrics aggregation can only be done on its value.");
                n.order_key = key;
                continue;
            }
            require(is_metric(t), ESGPU_ERR_INVALID, "Invalid terms aggregation order path [" + n.order_path +
                    "]. Terms buckets can only be sorted on a sub-aggregator path that is built out of zero or more "
                    "single-bucket aggregations within the path and a final single-bucket or a metrics aggregation at the path end.");
            double probe;
            if (t == ESGPU_AGG_AVG) {
                require(key.empty() || key == "value", ESGPU_ERR_INVALID, "Invalid terms aggregation order path [" + n.order_path +
                        "]. Ordering on a single-value metrics aggregation can only be done on its value.");
            } else {
                require(!key.empty(), ESGPU_ERR_INVALID, "Invalid terms aggregation order path [" + n.order_path +
                        "]. When ordering on a multi-value metrics aggregation a metric name must be specified");
                require(metric_value(t, key, 1, 0, 0, 0, 0, 2.0, &probe), ESGPU_ERR_INVALID, "Invalid terms aggregation order path [" +
                        n.order_path + "]. Unknown metric name [" + key + "] on multi-value metrics aggregation [" + name + "]");
            }
            n.order_key = key;
        }
        // compile each top-level subtree into a group of pipelines (one cell grid each, one kernel launch each);
        // a filter aggregation (FilterAggregator) becomes one counting pipeline for its doc_count plus one group per
        // sub-aggregation, all under its clauses
        std::function<void(int)> compile_filter = [&](int r) {  // a filter, its children (nested filters: recursively)
            Pipeline cnt;
            cnt.root = r;
            cnt.fspec = r;
            cnt.count_only = true;
            p->pipes.push_back(std::move(cnt));
            for (int ch : p->specs[r].children) {
                if (p->specs[ch].s.type == ESGPU_AGG_FILTER) compile_filter(ch);
                else p->groups.push_back(compile_group(p.get(), ch, r));
            }
        };
        for (int r : tops) {
            if (p->specs[r].s.type != ESGPU_AGG_FILTER) { p->groups.push_back(compile_group(p.get(), r, -1)); continue; }
            compile_filter(r);
        }
        HIPX(hipSetDevice(c->device));
        HIPX(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
        HIPX(hipEventCreate(&p->ev0));
        HIPX(hipEventCreate(&p->ev1));
        HIPX(hipEventCreateWithFlags(&p->ev_mid, hipEventDisableTiming));
        for (Pipeline& pl : p->pipes) {
            HIPX(hipEventCreate(&pl.e0));
            HIPX(hipEventCreate(&pl.e1));
        }
        *out = p.release();
    });
}

// The grid's doc counts are zeroed lazily after a reset: a request whose first segment takes a hot / cold path stores
// every counter (HcParams::overwrite) -- or, settled by its hot slots, never reads them -- and needs no zeroing pass
// (80 MB at 10M ordinals, 28 us per config-3 shard request); every other path, and a build with no collect, zeroes
// them first.
// ESGPU_EAGER_ZERO=0: a small grid's counts are zeroed at the first collect too (A/B)
static bool eager_zero_on() {
    static const bool on = [] {
        const char* e = std::getenv("ESGPU_EAGER_ZERO");
        return !(e && e[0] == '0');
    }();
    return on;
}
static void zero_counts(esgpu_plan* p, Pipeline& pl) {
    if (!pl.zero_pending) return;
    pl.zero_pending = false;
    if (!pl.allocated || !pl.g_cnt.p) return;
    HIPX(hipMemsetAsync(pl.g_cnt.p, 0, (size_t)pl.T * pl.H * 8, p->stream));
}
static void zero_all_counts(esgpu_plan* p) {
    for (Pipeline& pl : p->pipes) zero_counts(p, pl);
}

static void alloc_grid(esgpu_plan* p, Pipeline& pl) {
    esgpu_ctx* c = p->ctx;
    const size_t cells = (size_t)pl.T * pl.H;
    // arrays the shape uses keep their allocation when it is large enough (a reset plan whose next request's first
    // segment spans a slightly different key range: no hipFree, which would synchronise the whole device and stall
    // the other plan's collect), grown with 25 % headroom otherwise; arrays it does not use are released
    auto need = [&](DevBuf& b, bool used, size_t n) {
        if (!used) { b.release(); return; }
        if (!b.p || b.bytes < n) b.alloc(c, n + n / 4);
    };
    need(pl.g_cnt, true, cells * 8);
    HIPX(hipMemsetAsync(pl.g_cnt.p, 0, cells * 8, p->stream));
    pl.zero_pending = false;
    const size_t no = pl.ocnt_mode == OCNT_HIST ? pl.H : pl.T;
    need(pl.g_ocnt, pl.ocnt_mode != OCNT_NONE, no * 8);
    if (pl.ocnt_mode != OCNT_NONE) HIPX(hipMemsetAsync(pl.g_ocnt.p, 0, pl.g_ocnt.bytes, p->stream));
    need(pl.g_vcnt, pl.met > 0 && pl.vcnt_mode, cells * 8);
    if (pl.g_vcnt.p) HIPX(hipMemsetAsync(pl.g_vcnt.p, 0, cells * 8, p->stream));
    need(pl.g_sum, pl.met > 0, cells * 8);
    if (pl.g_sum.p) HIPX(hipMemsetAsync(pl.g_sum.p, 0, cells * 8, p->stream));
    need(pl.g_min, pl.met >= 2, cells * 8);
    need(pl.g_max, pl.met >= 2, cells * 8);
    if (pl.met >= 2) {
        launch_fill_u64(pl.g_min.as<unsigned long long>(), cells, kMinInit, p->stream);
        launch_fill_u64(pl.g_max.as<unsigned long long>(), cells, kMaxInit, p->stream);
    }
    need(pl.g_sq, pl.met >= 3, cells * 8);
    if (pl.g_sq.p) HIPX(hipMemsetAsync(pl.g_sq.p, 0, cells * 8, p->stream));
    for (CardState& cs : pl.cards) {
        require((double)cells * (cs.m + 12.0 * cs.cap) <= 4.0 * (1ull << 30), ESGPU_ERR_UNSUPPORTED,
                "cardinality sketches for every bucket exceed the 4 GiB per-request budget");
        need(cs.regs, true, cells * cs.m);
        need(cs.sets, true, cells * cs.cap * 4);
        need(cs.first, true, cells * cs.cap * 8);
        HIPX(hipMemsetAsync(cs.first.p, 0xFF, cs.first.bytes, p->stream));
        need(cs.cnt, true, cells * 4);
        need(cs.nonzero, true, cells * 4);
        HIPX(hipMemsetAsync(cs.regs.p, 0, cs.regs.bytes, p->stream));
        HIPX(hipMemsetAsync(cs.sets.p, 0, cs.sets.bytes, p->stream));
        HIPX(hipMemsetAsync(cs.cnt.p, 0, cs.cnt.bytes, p->stream));
        HIPX(hipMemsetAsync(cs.nonzero.p, 0, cs.nonzero.bytes, p->stream));
    }
    pl.allocated = true;
}

// re-shape an allocated grid to newH key rows, the old rows landing at row `shift` ([H][T] rows are contiguous, so a
// key-range extension is one copy per array)
static void regrid(esgpu_plan* p, Pipeline& pl, uint32_t newH, int64_t shift) {
    const uint32_t oldH = pl.H;
    std::vector<CardState> old_cards(pl.cards.size());
    for (size_t i = 0; i < pl.cards.size(); ++i) {
        old_cards[i].regs = std::move(pl.cards[i].regs);
        old_cards[i].sets = std::move(pl.cards[i].sets);
        old_cards[i].first = std::move(pl.cards[i].first);
        old_cards[i].cnt = std::move(pl.cards[i].cnt);
        old_cards[i].nonzero = std::move(pl.cards[i].nonzero);
    }
    struct { DevBuf g_cnt, g_ocnt, g_vcnt, g_sum, g_min, g_max, g_sq; } old;
    old.g_cnt = std::move(pl.g_cnt);
    old.g_ocnt = std::move(pl.g_ocnt);
    old.g_vcnt = std::move(pl.g_vcnt);
    old.g_sum = std::move(pl.g_sum);
    old.g_min = std::move(pl.g_min);
    old.g_max = std::move(pl.g_max);
    old.g_sq = std::move(pl.g_sq);
    pl.H = newH;
    alloc_grid(p, pl);
    const size_t row = (size_t)pl.T * 8;
    auto cp = [&](DevBuf& dst, DevBuf& src, size_t rowb) {
        if (src.p) HIPX(hipMemcpyAsync(dst.as<uint8_t>() + shift * rowb, src.p, (size_t)oldH * rowb, hipMemcpyDeviceToDevice, p->stream));
    };
    cp(pl.g_cnt, old.g_cnt, row);
    cp(pl.g_vcnt, old.g_vcnt, row);
    cp(pl.g_sum, old.g_sum, row);
    cp(pl.g_min, old.g_min, row);
    cp(pl.g_max, old.g_max, row);
    cp(pl.g_sq, old.g_sq, row);
    if (pl.ocnt_mode == OCNT_HIST) cp(pl.g_ocnt, old.g_ocnt, 8);
    if ((pl.ocnt_mode == OCNT_TERMS || pl.ocnt_mode == OCNT_TERMS_DERIVED) && old.g_ocnt.p)
        HIPX(hipMemcpyAsync(pl.g_ocnt.p, old.g_ocnt.p, (size_t)pl.T * 8, hipMemcpyDeviceToDevice, p->stream));
    for (size_t i = 0; i < pl.cards.size(); ++i) {
        CardState& cs = pl.cards[i];
        cp(cs.regs, old_cards[i].regs, (size_t)pl.T * cs.m);
        cp(cs.sets, old_cards[i].sets, (size_t)pl.T * cs.cap * 4);
        cp(cs.first, old_cards[i].first, (size_t)pl.T * cs.cap * 8);
        cp(cs.cnt, old_cards[i].cnt, (size_t)pl.T * 4);
        cp(cs.nonzero, old_cards[i].nonzero, (size_t)pl.T * 4);
    }
    HIPX(hipStreamSynchronize(p->stream));
}

// grow the key range of an allocated affine grid to cover key indices [kmin, kmax]
static void grow_keys(esgpu_plan* p, Pipeline& pl, int64_t kmin, int64_t kmax) {
    const int64_t nk0 = std::min(pl.key0, kmin);
    const int64_t nk1 = std::max(pl.key0 + (int64_t)pl.H - 1, kmax);
    if (nk0 == pl.key0 && nk1 == pl.key0 + (int64_t)pl.H - 1) return;
    require(nk1 - nk0 + 1 <= 64 * 1024 * 1024, ESGPU_ERR_UNSUPPORTED, "histogram key range too large for a dense grid");
    const int64_t shift = pl.key0 - nk0;
    pl.key0 = nk0;
    regrid(p, pl, (uint32_t)(nk1 - nk0 + 1), shift);
}

// (re)build the bucket table of a non-affine rounding so that it covers [lo, hi]; returns the row shift of the
// previous table's buckets (0 on first build)
static constexpr size_t kMaxTableBuckets = 16u << 20;
static int64_t build_key_table(esgpu_plan* p, Pipeline& pl, int64_t lo, int64_t hi) {
    if (pl.kt_lo <= pl.kt_hi) {
        if (lo >= pl.kt_lo && hi <= pl.kt_hi) return 0;
        lo = std::min(lo, pl.kt_lo);
        hi = std::max(hi, pl.kt_hi);
    }
    std::vector<int64_t> starts, keys;
    std::vector<uint32_t> slot;
    require(pl.rnd.key_table(lo, hi, kMaxTableBuckets, starts, keys, slot), ESGPU_ERR_UNSUPPORTED,
            "date_histogram rounding produces too many buckets for a dense grid");
    int64_t shift = 0;
    if (!pl.kt_key.empty()) {
        auto it = std::lower_bound(keys.begin(), keys.end(), pl.kt_key.front());
        require(it != keys.end() && *it == pl.kt_key.front(), ESGPU_ERR_DEVICE, "bucket table is not a superset");
        shift = it - keys.begin();
    }
    pl.kt_lo = lo;
    pl.kt_hi = hi;
    pl.kt_start = std::move(starts);
    pl.kt_key = std::move(keys);
    pl.kt_slot = std::move(slot);
    pl.d_kstart.alloc(p->ctx, std::max<size_t>(pl.kt_start.size(), 1) * 8);
    if (!pl.kt_start.empty())
        HIPX(hipMemcpyAsync(pl.d_kstart.p, pl.kt_start.data(), pl.kt_start.size() * 8, hipMemcpyHostToDevice, p->stream));
    pl.d_kslot.release();
    if (!pl.kt_slot.empty()) {
        pl.d_kslot.alloc(p->ctx, pl.kt_slot.size() * 4);
        HIPX(hipMemcpyAsync(pl.d_kslot.p, pl.kt_slot.data(), pl.kt_slot.size() * 4, hipMemcpyHostToDevice, p->stream));
    }
    return shift;
}

// the query clauses and those of the pipeline's filter aggregation
// a clause applies to a pipeline when it is a query clause or belongs to a filter aggregation enclosing the pipeline's
// (its own filter, and every filter aggregation above it: nested filters intersect, FilterAggregator.java:57-70 per level)
static bool applies(const esgpu_plan* p, const Pipeline& pl, size_t k) {
    const int owner = p->filter_owner[k];
    if (owner < 0) return true;
    for (int x = pl.fspec; x >= 0; x = p->specs[x].s.parent)
        if (x == owner) return true;
    return false;
}

static bool compact_cols(const esgpu_ctx* c);
static bool dyn_claim_on();
static bool replay_compaction();
static bool d16_on();
static bool raw_hist_on();
static bool dd_forced();
static bool int_runs_on();
static bool dot16_on();
static uint32_t hdirect_copies();
static bool runs1_on();
static bool b16_on(const esgpu_ctx* c);
static bool pi_cells(const esgpu_ctx* c);
static uint32_t pi_copies(int met);
static const uint16_t* ensure_ord16(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st);
static const uint32_t* ensure_d32(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st);
static const uint16_t* ensure_d16(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st);
static const DevColumn* ensure_b16(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st);
static int b24_mode();
static const void* wide_i64(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st);
static void sampled_hot_ords(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, uint32_t (&out)[4]);

// The pipeline's clauses as device predicates: up to kMaxPreds of them are evaluated inside the collect kernels; with
// more, all of them (and the accept bitset) are folded first into one doc bitset -- chained filter_bits passes of four
// clauses each -- which replaces *accept, and no predicate is left for the kernel.
static void set_preds(esgpu_plan* p, const Pipeline& pl, const esgpu_segment* s, PredDev* out, int32_t* npred,
                      uint64_t* bytes_per_doc, const uint64_t** accept) {
    std::vector<PredDev> all;
    *npred = 0;
    for (size_t k = 0; k < p->filters.size(); ++k) {
        if (!applies(p, pl, k)) continue;
        const esgpu_filter& f = p->filters[k];
        const DevColumn* col = s->col(p->filter_fields[k].c_str());
        PredDev q{};
        require(col != nullptr, ESGPU_ERR_UNSUPPORTED, "filter on a field missing from the segment");
        q.col = col->type == ESGPU_COL_ORD_U32 ? col->ords().p : col->type == ESGPU_COL_F64 ? col->values.p : nullptr;
        q.present = col->present.as<uint64_t>();
        q.offsets = col->multi ? col->offsets.as<uint64_t>() : nullptr;
        if (col->type == ESGPU_COL_ORD_U32) {
            if (f.type == ESGPU_FILTER_TERM) {
                q.kind = PRED_ORD_EQ;
                q.lo = q.hi = f.term;
            } else {  // TermRangeQuery: the dictionary is sorted by unsigned bytes, so the range is an ordinal range
                q.kind = PRED_ORD_RANGE;
                const uint64_t n = col->ord_count();
                auto bound = [&](const uint8_t* t, uint64_t len, bool upper) {  // first ord with term > t (upper) / >= t
                    const std::string key((const char*)t, (size_t)len);
                    uint64_t lo = 0, hi = n;
                    while (lo < hi) {
                        const uint64_t mid = (lo + hi) / 2;
                        const std::string m = col->ord_term(mid);
                        if (upper ? !(key < m) : m < key) lo = mid + 1; else hi = mid;
                    }
                    return (int64_t)lo;
                };
                q.lo = 0;
                q.hi = (int64_t)n - 1;
                if (f.has_lower) {
                    require(f.lo_term || f.lo_term_len == 0, ESGPU_ERR_INVALID, "keyword range without lower term bytes");
                    q.lo = bound(f.lo_term, f.lo_term_len, !f.include_lower);
                }
                if (f.has_upper) {
                    require(f.hi_term || f.hi_term_len == 0, ESGPU_ERR_INVALID, "keyword range without upper term bytes");
                    q.hi = bound(f.hi_term, f.hi_term_len, f.include_upper) - 1;
                }
            }
            *bytes_per_doc += 4;
        } else if (col->type == ESGPU_COL_F64) {
            q.kind = PRED_F64_RANGE;
            if (f.type == ESGPU_FILTER_TERM) { q.dlo = q.dhi = (double)f.term; q.lo_incl = q.hi_incl = 1; }
            else {
                q.dlo = f.has_lower ? f.lo_d : -INFINITY;
                q.dhi = f.has_upper ? f.hi_d : INFINITY;
                q.lo_incl = f.has_lower ? f.include_lower : 1;
                q.hi_incl = f.has_upper ? f.include_upper : 1;
            }
            *bytes_per_doc += 8;
        } else {
            q.kind = PRED_I64_RANGE;
            if (f.type == ESGPU_FILTER_TERM) { q.lo = q.hi = f.term; }
            else {
                int64_t lo = INT64_MIN, hi = INT64_MAX;
                bool empty = false;
                if (f.has_lower) {
                    if (f.include_lower) lo = f.lo_i;
                    else if (f.lo_i == INT64_MAX) empty = true;
                    else lo = f.lo_i + 1;
                }
                if (f.has_upper) {
                    if (f.include_upper) hi = f.hi_i;
                    else if (f.hi_i == INT64_MIN) empty = true;
                    else hi = f.hi_i - 1;
                }
                if (empty) { lo = 1; hi = 0; }
                q.lo = lo;
                q.hi = hi;
            }
            // single-valued: the compact copy of the column (u16 / u32 deltas) when its values span < 2^16 / 2^32
            if (compact_cols(p->ctx) && d16_on() && !col->multi && col->vmin <= col->vmax &&
                (uint64_t)col->vmax - (uint64_t)col->vmin < (1ull << 16)) {
                if (const uint16_t* d = ensure_d16(p->ctx, col, s, p->stream)) {
                    q.col = d;
                    q.kind = PRED_D16_RANGE;
                    q.base = col->vmin;
                }
            }
            if (q.kind != PRED_D16_RANGE && compact_cols(p->ctx) && !col->multi && col->vmin <= col->vmax &&
                (uint64_t)col->vmax - (uint64_t)col->vmin < (1ull << 32)) {
                if (const uint32_t* d = ensure_d32(p->ctx, col, s, p->stream)) {
                    q.col = d;
                    q.kind = PRED_D32_RANGE;
                    q.base = col->vmin;
                }
            }
            if (q.kind == PRED_I64_RANGE) q.col = wide_i64(p->ctx, col, s, p->stream);  // the upload-width values
            *bytes_per_doc += q.kind == PRED_D16_RANGE ? 2 : q.kind == PRED_D32_RANGE ? 4 : 8;
        }
        all.push_back(q);
    }
    if (all.size() <= (size_t)kMaxPreds) {
        for (const PredDev& q : all) out[(*npred)++] = q;
        return;
    }
    uint64_t* bits = (uint64_t*)p->s_xbits.ensure(p->ctx, std::max<size_t>(s->n_pad / 64, 1) * 8);
    const uint64_t* in = *accept;
    for (size_t k = 0; k < all.size(); k += kMaxPreds) {
        launch_filter_bits(s->max_doc, in, all.data() + k, (int)std::min<size_t>(kMaxPreds, all.size() - k), bits, p->stream);
        HIPX(hipGetLastError());
        in = bits;  // in place: each thread reads and rewrites its own word
    }
    *accept = bits;
    *bytes_per_doc += 0;  // the clause columns were counted above; the bitset the kernel then reads is 1 bit per doc
}

// The terms doc counts in g_cnt are u32 on the partitioned / hot-cold paths (BucketsAggregator's IntArray,
// A/bucket/BucketsAggregator.java:44-50) and u64 for every other kernel (LDS flushes, the CSR kernel, global atomics).
// Which kernel runs can change from one segment of a request to the next (a field multi-valued in only some segments),
// so the width is settled per segment before the launch: the grid is zero at a request's first segment (either width),
// later ones convert the counts in place through a scratch copy.  u32 counts need the request's docs below 2^32 --
// a shard holds at most IndexWriter.MAX_DOCS = 2^31 - 128 docs over all its segments, so only a caller collecting more
// than a shard into one plan can reach that.
static void count_width(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, bool want32, bool first_segment) {
    if (want32)
        require(p->docs_seen + (uint64_t)s->max_doc <= 0xFFFFFFFFull, ESGPU_ERR_UNSUPPORTED,
                "a terms request over more than 2^32 docs (a shard holds at most 2^31 - 128): runs on the CPU path");
    if (first_segment || want32 == pl.cnt32) { pl.cnt32 = want32; return; }
    const size_t cells = (size_t)pl.T * pl.H;
    if (cells) {
        void* tmp = p->s_tcnt.ensure(p->ctx, cells * 8);
        if (want32) {  // u64 -> u32: the scratch takes the narrow copy, then it goes back over the grid's head
            launch_narrow_u64(pl.g_cnt.as<unsigned long long>(), cells, (unsigned int*)tmp, p->stream);
            HIPX(hipGetLastError());
            HIPX(hipMemcpyAsync(pl.g_cnt.p, tmp, cells * 4, hipMemcpyDeviceToDevice, p->stream));
        } else {
            launch_widen_u32(pl.g_cnt.as<unsigned int>(), cells, (unsigned long long*)tmp, p->stream);
            HIPX(hipGetLastError());
            HIPX(hipMemcpyAsync(pl.g_cnt.p, tmp, cells * 8, hipMemcpyDeviceToDevice, p->stream));
        }
    }
    pl.cnt32 = want32;
}

// K1 for valueCount >> LDS (e.g. 10M url ordinals): radix-partitioned counting instead of global atomics, which
// serialise on the Zipf head terms.  Reads the ordinal column twice (4 + 4 B/doc), writes and re-reads a 2 B/doc
// partition-local copy: 12 B/doc of traffic for the 4 B/doc algorithmic stream.  Fully asynchronous.
static bool count_partitioned(esgpu_plan* p, Pipeline& pl, const uint32_t* ords, uint32_t n_docs, uint32_t n_blocks,
                              const uint64_t* d_accept, const PredDev* pred, int npred);
static bool collect_partitioned(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, const DevColumn* oc,
                                const uint64_t* d_accept, const PredDev* pred, int npred) {
    return count_partitioned(p, pl, oc->ords().as<uint32_t>(), s->max_doc, s->n_pad / kBlockDocs, d_accept, pred, npred);
}
// the counting core over any u32 ordinal list of n_docs entries, readable up to n_blocks * kBlockDocs (a segment's
// column, or a compacted replay region)
static bool count_partitioned(esgpu_plan* p, Pipeline& pl, const uint32_t* ords, uint32_t n_docs, uint32_t n_blocks,
                              const uint64_t* d_accept, const PredDev* pred, int npred) {
    esgpu_ctx* c = p->ctx;
    hipStream_t st = p->stream;
    PartParams Q{};
    Q.n_docs = n_docs;
    Q.n_blocks = n_blocks;
    const uint32_t target = (uint32_t)c->cus * part_wg_per_cu();
    Q.blocks_per_wg = std::max(1u, (Q.n_blocks + target - 1) / target);
    Q.G = (Q.n_blocks + Q.blocks_per_wg - 1) / Q.blocks_per_wg;
    Q.ord = ords;
    Q.T = pl.T;
    Q.shift = kPartShift;  // 32768 ordinals per partition: 128 KB of LDS counters in the counting pass
    Q.P = (uint32_t)(((uint64_t)pl.T + (1u << Q.shift) - 1) >> Q.shift);
    require(Q.P >= 1 && Q.P <= kPartMaxStaged, ESGPU_ERR_INVALID, "partition count out of range");
    Q.npred = npred;
    for (int k = 0; k < npred; ++k) Q.pred[k] = pred[k];
    Q.accept = d_accept;
    Q.wg_counts = (uint32_t*)p->s_wgc.ensure(c, (size_t)Q.P * Q.G * 4);
    Q.part_begin = (uint32_t*)p->s_pbeg.ensure(c, (size_t)(Q.P + 1) * 4);
    const uint32_t ntiles = part_scan_tiles(Q.P * Q.G);
    require(ntiles <= 4096, ESGPU_ERR_INVALID, "partition scan too large");
    Q.tile_sums = (uint32_t*)p->s_tiles.ensure(c, (size_t)ntiles * 4);
    Q.pbuf = (uint16_t*)p->s_pbuf.ensure(c, (std::max<size_t>(n_docs, 1) + 8) * 2);
    Q.counts = pl.g_cnt.as<unsigned int>();
    // counting workgroups (one resident per CU at 128 KB of LDS counters); each covers `chunk` partitioned elements
    // (a multiple of 8: 16-byte loads).  Every partition piece a workgroup counts ends in a flush of its 32768
    // counters (256 KB of global adds), so the workgroup count is capped at one per 512K elements -- the flushes stay
    // within a quarter of the 2-byte reads -- between 1 and 4 per CU.  Measured: 4 per CU is best at 1B docs (3.16 vs
    // 3.47 ms for 1 per CU), 1 per CU at 125M (0.55 vs 0.62 ms).
    const uint64_t want = std::min<uint64_t>((uint64_t)c->cus * 4,
                                             std::max<uint64_t>((uint64_t)c->cus, (uint64_t)n_docs >> 19));
    Q.chunk = (uint32_t)std::max<uint64_t>(1u << 16, (((uint64_t)n_docs + want - 1) / want + 7) & ~7ull);
    HIPX(hipEventRecord(pl.e0, st));
    launch_part_hist(Q, st);
    launch_part_scan(Q, st);
    launch_part_scatter(Q, st);
    launch_part_count(Q, st);
    HIPX(hipGetLastError());
    HIPX(hipEventRecord(pl.e1, st));
    p->last_path = 4;
    return true;
}

// ------------------------------------------------------------------------------------------------------------
// K1 for valueCount >> LDS, hot/cold form (esgpu_hotcold.hip): one read of the ordinal column instead of two, the
// most frequent ordinals counted in LDS and never written out, the rest appended to partitions whose capacities come
// from the segment's statistics (no histogram pass).  The statistics are the segment's, built on the first request
// over the column and kept beside it, the way Elasticsearch builds a field's global ordinals on first use and caches
// them (GlobalOrdinalsBuilder.build via IndexFieldDataService's cache, C/index/fielddata/ordinals/
// GlobalOrdinalsBuilder.java:46-70).
// ------------------------------------------------------------------------------------------------------------
#ifndef ESGPU_HOTCOLD
#define ESGPU_HOTCOLD 1
#endif
#ifndef ESGPU_HOT_MAX
#define ESGPU_HOT_MAX 16384  // hot slots at most (LDS counters of the scatter)
#endif
#ifndef ESGPU_HOT_PER_CU
#define ESGPU_HOT_PER_CU 2  // hot-pass workgroups per CU (postings path; 4 measured 13 % slower)
#endif
#ifndef ESGPU_HC_POSTINGS
#define ESGPU_HC_POSTINGS 1  // cold lists for requests without predicates / accept bits (0: always the scatter path)
#endif
#ifndef ESGPU_NO_HOT
#define ESGPU_NO_HOT 0  // timing experiments: no hot set
#endif

// the postings hot pass reads the 16-bit hot-slot column (ESGPU_HOT16=0: the 32-bit recoded column, for A/B runs)
static bool hc_hot16() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_HOT16"); return !(e && *e == '0'); }();
    return on;
}
static_assert(ESGPU_HOT_MAX <= 0xFFFF, "hot slots must fit the 16-bit column");

struct HcStats {
    const void* src = nullptr;   // the ordinal buffer described (DevColumn::ords())
    uint64_t T = 0;
    uint32_t G = 0, P = 0, hot_n = 0, trash = 0, n_pieces = 0;
    bool u16 = false;            // every cold ordinal's count < 65536: packed 16-bit counters in the counting pass
    uint64_t pbuf_elems = 0;     // partition regions + kHcTile spare elements
    uint64_t hot_docs = 0, docs = 0;
    std::vector<uint32_t> hot_cnt;  // each hot slot's count in the segment (most frequent first)
    uint64_t max_cold = 0;       // the largest count of a cold ordinal in the segment (unfiltered): a request's top-k
                                 // in count order is settled by the hot slots alone when its k-th count is above it
    bool refused = false;        // outside what the hot/cold kernels handle (cached: the check counts the column)
    // recoded ordinal column (hot ordinals as kHcHotBit | slot); empty: no hot set, or released once the postings form is
    // ready (the hot16 column and the cold lists serve unfiltered requests) and rebuilt from the hot table on the first
    // request that needs it (predicates, live docs: ensure_rc)
    mutable DevBuf d_rc;
    DevBuf d_rc_keys, d_rc_vals;  // the hot ordinals' open-addressing table (hc_recode)
    uint32_t rc_log2 = 0;
    DevBuf d_hot16;              // the hot slot of each doc in 16 bits (0xFFFF: cold / missing) for the postings hot pass
    DevBuf d_hot_ord, d_part, d_piece;
    // cold lists: the cold docs' partition-local offsets grouped by partition (postings of the cold ordinals, 64-element
    // aligned per partition), read by requests without predicates or accept bits instead of scattering the cold docs
    bool cold_lists = false;
    uint32_t cold_pieces = 0;
    DevBuf d_cold, d_cold_part, d_cold_piece, d_cold_used, d_cold_ovf;
};

static uint32_t hc_hash_host(uint32_t o, uint32_t log2) { return (uint32_t)(o * 0x9E3779B1u) >> (32 - log2); }

// doc count of every ordinal of a column (no filters), by the radix-partitioned passes (collect_partitioned's kernels)
static void count_all_ordinals(esgpu_ctx* c, const uint32_t* ord, uint32_t max_doc, uint32_t n_pad, uint32_t T,
                               DevBuf& counts, hipStream_t st) {
    counts.alloc(c, (size_t)std::max<uint32_t>(T, 1) * 4);
    HIPX(hipMemsetAsync(counts.p, 0, counts.bytes, st));
    if (max_doc == 0) return;
    PartParams Q{};
    Q.n_docs = max_doc;
    Q.n_blocks = n_pad / kBlockDocs;
    const uint32_t target = (uint32_t)c->cus * part_wg_per_cu();
    Q.blocks_per_wg = std::max(1u, (Q.n_blocks + target - 1) / target);
    Q.G = (Q.n_blocks + Q.blocks_per_wg - 1) / Q.blocks_per_wg;
    Q.ord = ord;
    Q.T = T;
    Q.shift = kPartShift;
    Q.P = (uint32_t)(((uint64_t)T + (1u << Q.shift) - 1) >> Q.shift);
    DevBuf wgc, pbeg, tiles, pbuf;
    wgc.alloc(c, (size_t)Q.P * Q.G * 4);
    pbeg.alloc(c, (size_t)(Q.P + 1) * 4);
    const uint32_t ntiles = part_scan_tiles(Q.P * Q.G);
    require(ntiles <= 4096, ESGPU_ERR_INVALID, "partition scan too large");
    tiles.alloc(c, (size_t)ntiles * 4);
    pbuf.alloc(c, ((size_t)max_doc + 8) * 2);
    Q.wg_counts = wgc.as<uint32_t>();
    Q.part_begin = pbeg.as<uint32_t>();
    Q.tile_sums = tiles.as<uint32_t>();
    Q.pbuf = pbuf.as<uint16_t>();
    Q.counts = counts.as<unsigned int>();
    const uint64_t want = std::min<uint64_t>((uint64_t)c->cus * 4, std::max<uint64_t>((uint64_t)c->cus, (uint64_t)max_doc >> 19));
    Q.chunk = (uint32_t)std::max<uint64_t>(1u << 16, (((uint64_t)max_doc + want - 1) / want + 7) & ~7ull);
    launch_part_hist(Q, st);
    launch_part_scan(Q, st);
    launch_part_scatter(Q, st);
    launch_part_count(Q, st);
    HIPX(hipGetLastError());
    HIPX(hipStreamSynchronize(st));  // the scratch buffers are released on return
}

// The column's hot set and partition capacities (built once per ordinal buffer, under the context lock).  Returns null
// when the column is outside what the hot/cold kernels handle (more than kHcMaxParts partitions, or a buffer beyond
// 32-bit element offsets): the caller keeps the histogram-pass form.
static std::shared_ptr<const HcStats> ensure_hc_stats(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s,
                                                     uint32_t T, hipStream_t st) {
    DevColumn* mcol = const_cast<DevColumn*>(col);
    std::lock_guard<std::mutex> lk(c->mu);  // plans on different threads may share the segment
    const void* src = col->ords().p;
    if (mcol->hc && mcol->hc->src == src && mcol->hc->T == T) return mcol->hc->refused ? nullptr : mcol->hc;
    const uint32_t P = (uint32_t)(((uint64_t)T + (1u << kPartShift) - 1) >> kPartShift);
    if (P == 0 || P > kHcMaxParts || c->cus <= 0) return nullptr;
    auto hs = std::make_shared<HcStats>();
    hs->src = src;
    hs->T = T;
    hs->P = P;
    auto refuse = [&]() -> std::shared_ptr<const HcStats> {  // remembered for this (buffer, T): not counted again
        auto r = std::make_shared<HcStats>();
        r->src = src;
        r->T = T;
        r->refused = true;
        mcol->hc = r;
        return nullptr;
    };
    // the segment's counts per ordinal on the GPU; the hot set from the GPU top-k's threshold candidates (sorted on the
    // host: a few times H keys), the cold totals per partition from one more pass over the counts -- the T counts never
    // leave the device (a 10M-ordinal column: 40 MB of counts, an nth_element over 10M on the host before)
    DevBuf dcnt;
    count_all_ordinals(c, (const uint32_t*)src, s->max_doc, s->n_pad, T, dcnt, st);
    // scatter workgroups and hot slots: two workgroups per CU while their LDS layouts fit with >= 2048 hot counters
    const size_t kLdsCu = 160 * 1024 - 512;
    auto hot_fit = [&](size_t budget) -> int64_t {
        const int64_t room = ((int64_t)budget - (int64_t)hc_scatter_lds_bytes(P, 0)) / 4 - 3 * (int64_t)kHcHotCopies - 4;
        return std::min<int64_t>(ESGPU_HOT_MAX, room) & ~63ll;
    };
    uint32_t H;
    if (hot_fit(kLdsCu / 2) >= 2048) {
        hs->G = (uint32_t)c->cus * 2;
        H = (uint32_t)hot_fit(kLdsCu / 2);
    } else {
        hs->G = (uint32_t)c->cus;
        H = (uint32_t)std::max<int64_t>(0, hot_fit(kLdsCu));
    }
    // hot set: the H most frequent ordinals (ties by ordinal), slot 0 the most frequent
    std::vector<uint32_t> hot, hot_cnt;
    uint64_t hot_total = 0, total = 0;
    {
        DevBuf dcand, dmeta;
        dcand.alloc(c, (size_t)std::max<uint32_t>(T, 1) * 8);
        dmeta.alloc(c, (2048 + 2) * 4 + 16);
        HIPX(hipMemsetAsync(dmeta.p, 0, dmeta.bytes, st));
        TopkParams K{};
        K.counts32 = dcnt.as<unsigned int>();
        K.T = T;
        K.order = ESGPU_ORDER_COUNT_DESC;
        K.min_doc_count = 1;
        K.shard_min_doc_count = 0;
        K.k = std::max<uint32_t>(std::min<uint32_t>(H, T), 1);
        K.n_wg = std::min<uint32_t>(512, (T + 4095) / 4096);
        K.cand = dcand.as<unsigned long long>();
        K.hist = dmeta.as<uint32_t>();
        K.sel = K.hist + 2048;
        K.out_sum = (unsigned long long*)(dmeta.as<unsigned char>() + (2048 + 2) * 4);  // 8,200: 8-byte aligned
        launch_topk_candidates(K, st);
        HIPX(hipGetLastError());
        uint32_t sel[2];
        HIPX(hipMemcpyAsync(sel, K.sel, 8, hipMemcpyDeviceToHost, st));
        HIPX(hipMemcpyAsync(&total, K.out_sum, 8, hipMemcpyDeviceToHost, st));
        HIPX(hipStreamSynchronize(st));
        if (H && !ESGPU_NO_HOT && sel[1]) {
            std::vector<unsigned long long> keys(sel[1]);
            HIPX(hipMemcpyAsync(keys.data(), dcand.p, keys.size() * 8, hipMemcpyDeviceToHost, st));
            HIPX(hipStreamSynchronize(st));
            const size_t take = std::min<size_t>(keys.size(), H);
            std::partial_sort(keys.begin(), keys.begin() + take, keys.end(), std::greater<unsigned long long>());
            for (size_t i = 0; i < take; ++i) {  // key: flag | count << 32 | ~ordinal (make_topk_key, _count desc)
                const uint64_t cntv = (keys[i] >> 32) & 0x7FFFFFFFull;
                if (cntv == 0) break;
                hot.push_back(0xFFFFFFFFu - (uint32_t)keys[i]);
                hot_cnt.push_back((uint32_t)cntv);
                hot_total += cntv;
            }
        }
        if (hot_total * 20 < total) {  // under 5 % of the docs: the recoded copy would not pay for itself
            hot.clear();
            hot_cnt.clear();
            hot_total = 0;
        }
    }
    hs->docs = total;
    hs->hot_n = (uint32_t)hot.size();
    hs->hot_cnt = hot_cnt;
    hs->hot_docs = hot_total;
    std::vector<uint64_t> cold(P, 0);
    uint64_t max_cold = 0;
    {
        std::vector<uint64_t> bits(((size_t)T + 63) / 64, 0);
        for (uint32_t o : hot) bits[o >> 6] |= 1ull << (o & 63);
        DevBuf dbits, dsum, dmax;
        dbits.alloc(c, std::max<size_t>(bits.size(), 1) * 8);
        dsum.alloc(c, (size_t)P * 8);
        dmax.alloc(c, (size_t)P * 4);
        HIPX(hipMemcpyAsync(dbits.p, bits.data(), bits.size() * 8, hipMemcpyHostToDevice, st));
        launch_hc_part_stats(dcnt.as<unsigned int>(), T, kPartShift, P, dbits.as<uint64_t>(), dsum.as<unsigned long long>(),
                             dmax.as<unsigned int>(), st);
        HIPX(hipGetLastError());
        std::vector<uint32_t> pmax(P);
        HIPX(hipMemcpyAsync(cold.data(), dsum.p, (size_t)P * 8, hipMemcpyDeviceToHost, st));
        HIPX(hipMemcpyAsync(pmax.data(), dmax.p, (size_t)P * 4, hipMemcpyDeviceToHost, st));
        HIPX(hipStreamSynchronize(st));  // `bits` is read by the copy above
        for (uint32_t m : pmax) max_cold = std::max<uint64_t>(max_cold, m);
    }
    hs->u16 = max_cold < 65536;
    hs->max_cold = max_cold;
    // layout: per partition, G static regions of `chunk` (its expected share per workgroup) then an overflow pool that
    // covers every way the docs can be spread over the workgroups: a workgroup allocates a new overflow chunk only when
    // its current one is full, so what it leaves unused is under one chunk (sizes: DESIGN.md §5)
    std::vector<HcPart> parts(P);
    std::vector<uint64_t> cap(P);
    uint64_t acc = 0;
    const uint64_t G = hs->G;
    for (uint32_t p = 0; p < P; ++p) {
        HcPart& q = parts[p];
        // static region: the expected share x 1.125 (+64): overflow allocations (a returning global atomic that the
        // whole workgroup waits for) stay rare on evenly spread data
        const uint64_t share = (cold[p] + G - 1) / G;
        const uint64_t chunk = cold[p] ? ((share + share / 8 + 64 + 63) & ~63ull) : 0;
        const uint64_t ovf = std::max<uint64_t>(64, ((chunk / 4) + 63) & ~63ull);
        q.sbase = (uint32_t)acc;
        q.chunk = (uint32_t)chunk;
        q.ovf_base = (uint32_t)(acc + G * chunk);
        acc += G * chunk + cold[p] + G * ovf;
        q.cap_end = (uint32_t)acc;
        q.ovf_chunk = (uint32_t)ovf;
        cap[p] = acc - q.sbase;
        if (acc + kHcTile + 64 >= 0xFFFFFFFFull) return refuse();
    }
    if (const char* e = std::getenv("ESGPU_DEBUG_HC_NO_OVERFLOW"); e && *e == '1')  // tests only: no overflow pools,
        for (HcPart& q : parts) q.cap_end = q.ovf_base;                          // so an uneven spread overruns
    hs->trash = (uint32_t)acc;
    hs->pbuf_elems = acc + kHcTile;
    // counting pieces: a partition far above the average region (a heavy cold ordinal) is split so that no counting
    // workgroup serialises the pass; the pieces of a split partition add their counters atomically
    const uint64_t piece_len = std::max<uint64_t>(1ull << 20, (4 * acc / P + 63) & ~63ull);
    std::vector<HcPiece> pieces;
    for (uint32_t p = 0; p < P; ++p) {
        const uint32_t n = (uint32_t)std::max<uint64_t>(1, (cap[p] + piece_len - 1) / piece_len);
        for (uint32_t k = 0; k < n; ++k)
            pieces.push_back(HcPiece{p, (uint32_t)(k * piece_len), (uint32_t)std::min<uint64_t>((k + 1) * piece_len, cap[p]),
                                     n == 1 ? 1u : 0u});
    }
    hs->n_pieces = (uint32_t)pieces.size();
    hs->d_part.alloc(c, parts.size() * sizeof(HcPart));
    hs->d_piece.alloc(c, pieces.size() * sizeof(HcPiece));
    HIPX(hipMemcpy(hs->d_part.p, parts.data(), parts.size() * sizeof(HcPart), hipMemcpyHostToDevice));
    HIPX(hipMemcpy(hs->d_piece.p, pieces.data(), pieces.size() * sizeof(HcPiece), hipMemcpyHostToDevice));
    if (!hot.empty()) {
        // the recoded column: an open-addressing table (load <= 1/4) of the hot ordinals, probed once per doc here
        uint32_t log2 = 2;
        while ((1u << log2) < 4 * hot.size()) ++log2;
        std::vector<uint32_t> keys(1u << log2, kMissingOrd), vals(1u << log2, 0);
        for (uint32_t sl = 0; sl < hot.size(); ++sl) {
            uint32_t h = hc_hash_host(hot[sl], log2);
            while (keys[h] != kMissingOrd) h = (h + 1) & ((1u << log2) - 1);
            keys[h] = hot[sl];
            vals[h] = sl;
        }
        DevBuf& dk = hs->d_rc_keys;
        DevBuf& dv = hs->d_rc_vals;
        hs->rc_log2 = log2;
        dk.alloc(c, keys.size() * 4);
        dv.alloc(c, vals.size() * 4);
        HIPX(hipMemcpy(dk.p, keys.data(), keys.size() * 4, hipMemcpyHostToDevice));
        HIPX(hipMemcpy(dv.p, vals.data(), vals.size() * 4, hipMemcpyHostToDevice));
        hs->d_rc.alloc(c, (size_t)s->n_pad * 4);
        launch_hc_recode((const uint32_t*)src, s->n_pad, dk.as<uint32_t>(), dv.as<uint32_t>(), log2, hs->d_rc.as<uint32_t>(), st);
        HIPX(hipGetLastError());
        if (ESGPU_HC_POSTINGS && hc_hot16()) {  // slots < ESGPU_HOT_MAX (16,384) fit 16 bits beside the 0xFFFF sentinel
            hs->d_hot16.alloc(c, (size_t)s->n_pad * 2);
            launch_hc_hot16(hs->d_rc.as<uint32_t>(), s->n_pad, hs->d_hot16.as<uint16_t>(), st);
            HIPX(hipGetLastError());
        }
        hs->d_hot_ord.alloc(c, hot.size() * 4);
        HIPX(hipMemcpy(hs->d_hot_ord.p, hot.data(), hot.size() * 4, hipMemcpyHostToDevice));
        HIPX(hipStreamSynchronize(st));  // the table buffers are released on return
    }
    if (ESGPU_HC_POSTINGS) {
        // cold lists: the radix-partition passes over the recoded column (hot and missing values are >= T and skipped)
        // give the cold docs' offsets partition by partition; each partition's list is then copied to a 64-aligned start
        const uint32_t* col = hot.empty() ? (const uint32_t*)src : hs->d_rc.as<uint32_t>();
        std::vector<uint32_t> pad(P + 1, 0);
        for (uint32_t p = 0; p < P; ++p) pad[p + 1] = pad[p] + (uint32_t)((cold[p] + 63) & ~63ull);
        if ((uint64_t)pad[P] + (uint64_t)64 * P < 0xFFFFFFF0ull) {
            DevBuf dense, wgc, pbeg, tiles, dpad;
            PartParams Q{};
            Q.n_docs = s->max_doc;
            Q.n_blocks = s->n_pad / kBlockDocs;
            const uint32_t target = (uint32_t)c->cus * part_wg_per_cu();
            Q.blocks_per_wg = std::max(1u, (Q.n_blocks + target - 1) / target);
            Q.G = (Q.n_blocks + Q.blocks_per_wg - 1) / Q.blocks_per_wg;
            Q.ord = col;
            Q.T = T;
            Q.shift = kPartShift;
            Q.P = P;
            wgc.alloc(c, (size_t)Q.P * Q.G * 4);
            pbeg.alloc(c, (size_t)(Q.P + 1) * 4);
            const uint32_t ntiles = part_scan_tiles(Q.P * Q.G);
            require(ntiles <= 4096, ESGPU_ERR_INVALID, "partition scan too large");
            tiles.alloc(c, (size_t)ntiles * 4);
            dense.alloc(c, ((size_t)total + 8) * 2);
            Q.wg_counts = wgc.as<uint32_t>();
            Q.part_begin = pbeg.as<uint32_t>();
            Q.tile_sums = tiles.as<uint32_t>();
            Q.pbuf = dense.as<uint16_t>();
            if (s->max_doc) {
                launch_part_hist(Q, st);
                launch_part_scan(Q, st);
                launch_part_scatter(Q, st);
            } else {
                HIPX(hipMemsetAsync(pbeg.p, 0, pbeg.bytes, st));
            }
            dpad.alloc(c, pad.size() * 4);
            HIPX(hipMemcpyAsync(dpad.p, pad.data(), pad.size() * 4, hipMemcpyHostToDevice, st));
            hs->d_cold.alloc(c, ((size_t)pad[P] + 8) * 2);
            launch_hc_pad(dense.as<uint16_t>(), pbeg.as<uint32_t>(), dpad.as<uint32_t>(), P, hs->d_cold.as<uint16_t>(), st);
            HIPX(hipGetLastError());
            std::vector<HcPart> cparts(P);
            std::vector<uint32_t> used(P);
            std::vector<HcPiece> cpieces;
            const uint64_t cpiece_len = std::max<uint64_t>(1ull << 20, (4 * (uint64_t)pad[P] / P + 63) & ~63ull);
            for (uint32_t p = 0; p < P; ++p) {
                HcPart& q = cparts[p];
                q.sbase = pad[p];
                q.chunk = pad[p + 1] - pad[p];
                q.ovf_base = q.cap_end = pad[p + 1];
                q.ovf_chunk = 64;
                used[p] = (uint32_t)cold[p];
                const uint32_t n = (uint32_t)std::max<uint64_t>(1, (q.chunk + cpiece_len - 1) / cpiece_len);
                for (uint32_t k = 0; k < n; ++k)  // at least one piece per partition: the first segment's counts are stored
                    cpieces.push_back(HcPiece{p, (uint32_t)(k * cpiece_len),
                                              (uint32_t)std::min<uint64_t>((k + 1) * cpiece_len, q.chunk), n == 1 ? 1u : 0u});
            }
            hs->cold_pieces = (uint32_t)cpieces.size();
            hs->d_cold_part.alloc(c, cparts.size() * sizeof(HcPart));
            hs->d_cold_piece.alloc(c, cpieces.size() * sizeof(HcPiece));
            hs->d_cold_used.alloc(c, used.size() * 4);
            std::vector<uint32_t> ovf(P);
            for (uint32_t p = 0; p < P; ++p) ovf[p] = cparts[p].ovf_base;  // no overflow pool: fill 0 for every request
            hs->d_cold_ovf.alloc(c, ovf.size() * 4);
            HIPX(hipMemcpyAsync(hs->d_cold_ovf.p, ovf.data(), ovf.size() * 4, hipMemcpyHostToDevice, st));
            HIPX(hipMemcpyAsync(hs->d_cold_part.p, cparts.data(), cparts.size() * sizeof(HcPart), hipMemcpyHostToDevice, st));
            HIPX(hipMemcpyAsync(hs->d_cold_piece.p, cpieces.data(), cpieces.size() * sizeof(HcPiece), hipMemcpyHostToDevice, st));
            HIPX(hipMemcpyAsync(hs->d_cold_used.p, used.data(), used.size() * 4, hipMemcpyHostToDevice, st));
            HIPX(hipStreamSynchronize(st));  // the scratch buffers and host vectors are released on return
            hs->cold_lists = true;
        }
    }
    // the postings form is complete: the 32-bit recoded column (2 B per doc more than the hot16 column) is released and
    // rebuilt only for a request that scatters or subtracts dead docs (ESGPU_HC_KEEP_RC=1 keeps it)
    if (hs->cold_lists && hs->d_hot16.p && hs->d_rc.p) {
        static const bool keep = [] { const char* e = std::getenv("ESGPU_HC_KEEP_RC"); return e && *e == '1'; }();
        if (!keep) hs->d_rc.release();
    }
    mcol->hc = hs;
    return hs;
}

// the recoded column of a segment's statistics, rebuilt from the hot table when it was released (under the context
// lock: plans on other threads may share the segment)
static const uint32_t* ensure_rc(esgpu_ctx* c, const HcStats& hs, const DevColumn* col, const esgpu_segment* s, hipStream_t st) {
    if (!hs.hot_n) return col->ords().as<uint32_t>();
    std::lock_guard<std::mutex> lk(c->mu);
    if (!hs.d_rc.p) {
        hs.d_rc.alloc(c, (size_t)s->n_pad * 4);
        launch_hc_recode(col->ords().as<uint32_t>(), s->n_pad, hs.d_rc_keys.as<uint32_t>(), hs.d_rc_vals.as<uint32_t>(), hs.rc_log2,
                         hs.d_rc.as<uint32_t>(), st);
        HIPX(hipGetLastError());
        HIPX(hipStreamSynchronize(st));
    }
    return hs.d_rc.as<uint32_t>();
}

// config 3's deferred cold lists (collect_hotcold / hc_topk_launch; ESGPU_HC_PRUNE=0: always counted, for A/B runs)
static bool hc_prune_on() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_HC_PRUNE"); return !(e && *e == '0'); }();
    return on;
}
// the request shape whose cold docs may wait for the top-k: one terms aggregation and nothing else (no other reader of
// these counts), in count order descending, shard_size within the hot set and the GPU top-k
static bool hc_defer_shape(const esgpu_plan* p, const Pipeline& pl, const HcStats& hs) {
    const int pipe = (int)(&pl - p->pipes.data());
    const SpecNode& tn = p->specs[pl.root];
    const bool plain = p->pipes.size() == 1 && p->groups.size() == 1 && p->groups[0].pipes.size() == 1 &&
                       p->groups[0].pipes[0] == pipe && p->groups[0].kids.empty();
    return hc_prune_on() && plain && hs.hot_n && hs.d_hot16.p && tn.s.type == ESGPU_AGG_TERMS &&
           tn.s.order == ESGPU_ORDER_COUNT_DESC && tn.s.shard_size >= 1 &&
           (uint64_t)tn.s.shard_size <= std::min<uint64_t>(hs.hot_n, kTopkMax) && pl.value_count > 65536 && pl.H == 1 &&
           pl.ocnt_mode == OCNT_NONE;
}
static bool collect_hotcold(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, const DevColumn* oc,
                            const uint64_t* d_accept, const PredDev* pred, int npred, bool first_segment) {
    esgpu_ctx* c = p->ctx;
    hipStream_t st = p->stream;
    std::shared_ptr<const HcStats> hs = ensure_hc_stats(c, oc, s, pl.T, st);
    if (!hs) return false;
    HcParams H{};
    H.n_docs = s->max_doc;
    H.n_blocks = s->n_pad / kBlockDocs;
    H.G = hs->G;
    H.blocks_per_wg = std::max(1u, (H.n_blocks + H.G - 1) / H.G);
    // the recoded column: read by the scatter form and the dead-doc subtraction; an unfiltered request on the postings
    // form reads only the hot16 column and the cold lists
    const bool clean_postings = hs->cold_lists && npred == 0 && !d_accept && hs->d_hot16.p && hc_hot16();
    H.rc = clean_postings ? nullptr : ensure_rc(c, *hs, oc, s, st);
    H.T = pl.T;
    H.P = hs->P;
    H.npred = npred;
    for (int k = 0; k < npred; ++k) H.pred[k] = pred[k];
    H.accept = d_accept;
    H.hot_n = hs->hot_n;
    H.hot_ord = hs->d_hot_ord.as<uint32_t>();
    H.part = hs->d_part.as<HcPart>();
    H.piece = hs->d_piece.as<HcPiece>();
    H.n_pieces = hs->n_pieces;
    H.ovf_cur = (uint32_t*)p->s_hcur.ensure(c, (size_t)H.P * 4);
    H.used = (uint32_t*)p->s_hused.ensure(c, (size_t)H.P * H.G * 4);
    H.hot_slab = H.hot_n ? (uint32_t*)p->s_hslab.ensure(c, (size_t)hc_slab_stride(H.hot_n) * H.G * 4) : nullptr;
    H.pbuf = (uint16_t*)p->s_pbuf.ensure(c, hs->pbuf_elems * 2);
    H.trash = hs->trash;
    H.counts = pl.g_cnt.as<unsigned int>();
    if (!p->h_hcerr.bytes) {  // zeroed once here and after each check: overruns of every segment accumulate
        p->h_hcerr.ensure(8);
        *p->h_hcerr.as<volatile uint32_t>() = 0;
    }
    H.err = (uint32_t*)p->h_hcerr.dev();
    p->hc_check = true;
    H.u16_counters = hs->u16 ? 1 : 0;
    H.overwrite = first_segment ? 1 : 0;  // every counter is stored by the counting pass: no read of the zeroed grid
    // every doc counts (or all but a few: a live-docs bitset with few deletions, sampled on the host at collect) -- hot
    // slots from the column (testing the accept bits), the cold lists, then the dead cold docs taken back out
    const bool live_docs_only = d_accept && d_accept == (const uint64_t*)p->s_accept.buf.p && p->sparse_dead;
    // the hot pass over the 16-bit hot-slot column: ESGPU_HOT_PER_CU 512-thread workgroups per CU
    auto hot_params = [&](HcParams& Hh) {
        const size_t hot_lds = (size_t)hc_hot_counters(Hh.hot_n) * 4;
        require(hot_lds <= 160 * 1024, ESGPU_ERR_STATE, "hot counters beyond LDS");
        Hh.G = (uint32_t)c->cus * (uint32_t)std::max<size_t>(1, std::min<size_t>(ESGPU_HOT_PER_CU, 160 * 1024 / (hot_lds + 1024)));
        Hh.blocks_per_wg = std::max(1u, (Hh.n_blocks + Hh.G - 1) / Hh.G);
        Hh.G = std::max(1u, (Hh.n_blocks + Hh.blocks_per_wg - 1) / Hh.blocks_per_wg);
        Hh.rc16 = hs->d_hot16.p ? hs->d_hot16.as<uint16_t>() : nullptr;
    };
    const int pipe = (int)(&pl - p->pipes.data());
    if (first_segment && (npred > 0 || d_accept) && hc_hot16() && hc_defer_shape(p, pl, *hs) &&
        hc_scatter_lds_bytes(H.P, H.hot_n) <= 160 * 1024 - 256) {
        // a lone count-ordered terms aggregation under a query filter or accept bits (config 3 filtered, deleted
        // docs): the request's clauses folded into one accept bitset, then only the hot slots (and one total of the
        // passing cold docs) counted from the 16-bit hot-slot column; the cold docs are scattered and counted (the
        // scatter form, from the folded bitset) only if the top-k needs them (hc_topk_launch) -- a cold ordinal's
        // filtered count is at most its count in the segment, HcStats::max_cold
        HIPX(hipEventRecord(pl.e0, st));
        const uint64_t* bits = d_accept;
        if (npred > 0) {
            uint64_t* xb = (uint64_t*)p->s_hbits.ensure(c, std::max<size_t>(s->n_pad / 64, 1) * 8);
            launch_filter_bits4(s->max_doc, d_accept, pred, npred, xb, st);
            HIPX(hipGetLastError());
            bits = xb;
        }
        HcParams Hh = H;
        hot_params(Hh);
        Hh.accept = bits;
        Hh.npred = 0;
        Hh.rc = nullptr;
        const size_t slab = (size_t)hc_slab_stride(H.hot_n) * std::max(H.G, Hh.G) * 4;
        Hh.hot_slab = H.hot_slab = (uint32_t*)p->s_hslab.ensure(c, slab);
        Hh.slot_tot = (uint32_t*)p->s_slot_tot.ensure(c, (size_t)hs->hot_n * 4);
        Hh.cold_tot = (uint32_t*)p->s_cold_tot.ensure(c, 16);
        HIPX(hipMemsetAsync(Hh.cold_tot, 0, 4, st));
        launch_hot_postings(Hh, st);
        HIPX(hipGetLastError());
        HIPX(hipEventRecord(pl.e1, st));
        H.accept = bits;  // the fallback: the scatter form from the folded bitset (no clause reads the segment later)
        H.npred = 0;
        p->hc_pend.on = true;
        p->hc_pend.filtered = true;
        p->hc_pend.pipe = pipe;
        p->hc_pend.hot = Hh;
        p->hc_pend.cold = H;
        p->hc_pend.hs = hs;
        // bytes: 2 per doc of hot slots instead of 4 of ordinals, the folded bitset read (and written by the fold)
        p->last_bytes = p->last_bytes - 2ull * s->max_doc + s->n_pad / 8 + (npred > 0 ? s->n_pad / 8 : 0);
        p->last_path = 9;
        return true;
    }
    if (hs->cold_lists && npred == 0 && (!d_accept || live_docs_only)) {
        HcParams K = H;                                 // the cold lists: one static region per partition
        K.accept = nullptr;
        K.G = 1;
        K.part = hs->d_cold_part.as<HcPart>();
        K.piece = hs->d_cold_piece.as<HcPiece>();
        K.n_pieces = hs->cold_pieces;
        K.used = hs->d_cold_used.as<uint32_t>();
        K.pbuf = hs->d_cold.as<uint16_t>();
        K.ovf_cur = hs->d_cold_ovf.as<uint32_t>();
        K.hot_n = 0;
        HcParams Hh = H;
        hot_params(Hh);
        Hh.hot_slab = Hh.hot_n ? (uint32_t*)p->s_hslab.ensure(c, (size_t)hc_slab_stride(Hh.hot_n) * Hh.G * 4) : nullptr;
        // a plain terms request in count order over one segment: the cold lists wait for the top-k (hc_topk_launch),
        // which needs them only if some cold ordinal can reach the k-th count
        const bool defer = first_segment && Hh.rc16 && !d_accept && hc_defer_shape(p, pl, *hs);
        if (Hh.rc16) {  // the bytes this form moves: 2 B per doc of hot slots plus 2 B per listed cold doc (not 4 B per doc)
            p->last_bytes = p->last_bytes - 2ull * s->max_doc + (defer ? 0ull : 2ull * (hs->docs - hs->hot_docs));
        }
        HIPX(hipEventRecord(pl.e0, st));
        if (defer) {
            Hh.slot_tot = (uint32_t*)p->s_slot_tot.ensure(c, (size_t)hs->hot_n * 4);
            launch_hot_postings(Hh, st);
            p->hc_pend.on = true;
            p->hc_pend.pipe = pipe;
            p->hc_pend.hot = Hh;
            p->hc_pend.cold = K;
            p->hc_pend.hs = hs;
        } else {
            launch_hotcold_postings(Hh, K, st);
        }
        HIPX(hipGetLastError());
        HIPX(hipEventRecord(pl.e1, st));
        p->last_path = defer ? 8 : 7;
        return true;
    }
    require(hc_scatter_lds_bytes(H.P, H.hot_n) <= 160 * 1024 - 256, ESGPU_ERR_STATE, "hot/cold LDS layout");
    HIPX(hipEventRecord(pl.e0, st));
    launch_hotcold(H, st);
    HIPX(hipGetLastError());
    HIPX(hipEventRecord(pl.e1, st));
    p->last_path = 6;
    return true;
}

// after a sync of the plan's stream: a partition overran the capacity the segment statistics promised (a bug, never data)
static void hc_check_err(esgpu_plan* p) {
    if (!p->hc_check) return;
    p->hc_check = false;
    volatile uint32_t* err = p->h_hcerr.as<volatile uint32_t>();
    const uint32_t e = *err;
    *err = 0;
    require(e == 0, ESGPU_ERR_DEVICE, "hot/cold counting: partition capacity exceeded");
}

// the deferred cold lists counted and folded (every reader of the counts but the top-k below: a second segment, a
// host selection, the co-located reduce)
static void hc_flush(esgpu_plan* p) {
    if (!p->hc_pend.on) return;
    if (p->hc_pend.filtered) launch_hotcold(p->hc_pend.cold, p->stream);  // the scatter form, hot slots included
    else launch_cold_postings(p->hc_pend.hot, p->hc_pend.cold, p->stream);
    HIPX(hipGetLastError());
    p->hc_pend = esgpu_plan::HcPending{};
    p->hc_check = true;  // (the cold counting writes the capacity word)
}

// K3 over a pipeline's counts (build_terms_root, xr_terms).  With the cold lists deferred: the top-k of the hot slot
// totals first; when its k-th count is above every cold ordinal's count in the segment (HcStats::max_cold), those are
// the request's winners and the cold counting, the fold and the full top-k return at once (a device flag, no host
// round trip); otherwise they run as without the deferral.
static void hc_topk_launch(esgpu_plan* p, const Pipeline& P0, TopkParams K, uint32_t k_req, hipStream_t st) {
    const int pipe = (int)(&P0 - p->pipes.data());
    if (!p->hc_pend.on || p->hc_pend.pipe != pipe) {
        hc_flush(p);
        launch_topk(K, st);
        return;
    }
    esgpu_ctx* c = p->ctx;
    const esgpu_plan::HcPending pend = p->hc_pend;
    p->hc_pend = esgpu_plan::HcPending{};
    require(st == p->stream, ESGPU_ERR_STATE, "deferred cold lists on another stream");
    const uint32_t hot_n = pend.hot.hot_n;
    TopkParams Hk = K;
    Hk.counts = nullptr;
    Hk.counts32 = pend.hot.slot_tot;
    Hk.ord_of = pend.hot.hot_ord;
    Hk.T = hot_n;
    Hk.n_wg = std::min<uint32_t>(512, (hot_n + 4095) / 4096);
    Hk.cand = (unsigned long long*)p->s_hcand.ensure(c, (size_t)hot_n * 8);
    uint32_t* hh = (uint32_t*)p->s_hhist.ensure(c, (2048 + 2) * 4);
    Hk.hist = hh;
    Hk.sel = hh + 2048;
    unsigned long long* hk = (unsigned long long*)p->s_hkeys.ensure(c, ((size_t)K.k + 1) * 8);
    Hk.out_keys = hk;
    Hk.out_sum = hk + K.k;
    Hk.skip = nullptr;
    HIPX(hipMemsetAsync(Hk.out_sum, 0, 8, st));
    launch_topk(Hk, st);
    HIPX(hipGetLastError());
    uint32_t* skip = (uint32_t*)p->s_hskip.ensure(c, 16);
    launch_hot_topk_check(hk, K.k, k_req, pend.hs->max_cold, pend.hs->docs, K.order, skip, K.out_keys, K.out_sum,
                          pend.hot.slot_tot, hot_n, pend.filtered ? pend.hot.cold_tot : nullptr, st);
    HIPX(hipGetLastError());
    HcParams hot = pend.hot, cold = pend.cold;
    hot.skip = skip;
    cold.skip = skip;
    if (pend.filtered) launch_hotcold(cold, st);  // (every kernel of the scatter form returns at once when settled)
    else launch_cold_postings(hot, cold, st);
    HIPX(hipGetLastError());
    p->hc_check = true;
    K.skip = skip;
    launch_topk(K, st);
}

// algorithmic bytes of one referenced column over a segment: natural width per value, plus the CSR
// offsets (8 B per doc) of a multi-valued column
static uint64_t column_bytes(const DevColumn* c, uint32_t max_doc) {
    if (!c) return 0;
    const uint64_t w = c->type == ESGPU_COL_ORD_U32 ? 4 : 8;
    return c->multi ? w * c->n_values + 8ull * max_doc : w * max_doc;
}

// K1/K4-K7 over multi-valued columns: collect_multi_kernel (one doc per thread, CSR), filters folded into a doc bitset
static bool collect_multi(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, CollectParams& P, const DevColumn* oc,
                          const DevColumn* hc, const DevColumn* mc, int met_launch, const uint64_t* d_accept) {
    esgpu_ctx* c = p->ctx;
    const bool ORD = oc != nullptr, HIST = hc != nullptr;
    uint64_t bytes = column_bytes(oc, s->max_doc) + column_bytes(hc, s->max_doc) + column_bytes(mc, s->max_doc);
    if (d_accept) bytes += ((uint64_t)s->max_doc + 7) / 8;
    for (size_t k = 0; k < p->filter_fields.size(); ++k)
        if (applies(p, pl, k)) bytes += column_bytes(s->col(p->filter_fields[k].c_str()), s->max_doc);
    HIPX(hipEventRecord(pl.e0, p->stream));
    if (P.npred > 0) {
        uint64_t* bits = (uint64_t*)p->s_fbits.ensure(c, std::max<size_t>(s->n_pad / 64, 1) * 8);
        launch_filter_bits(s->max_doc, d_accept, P.pred, P.npred, bits, p->stream);
        HIPX(hipGetLastError());
        P.accept = bits;
        P.npred = 0;
    }
    P.ord_off = (oc && oc->multi) ? (oc->off_view ? oc->off_view : oc->offsets.as<uint64_t>()) : nullptr;
    P.hv_off = (hc && hc->multi) ? hc->offsets.as<uint64_t>() : nullptr;
    P.mv_off = (mc && mc->multi) ? mc->offsets.as<uint64_t>() : nullptr;
    if (P.ocnt_mode == OCNT_TERMS_DERIVED) P.ocnt_mode = OCNT_TERMS;  // outer counts per doc, never from the cells
    P.W = P.H;
    P.windowed = 0;
    size_t lds = collect_lds_bytes(P.T, P.H, met_launch, P.vcnt_mode, P.ocnt_mode);
    P.lds_mode = lds <= 64 * 1024 ? 1 : 0;
    if (!P.lds_mode) lds = 0;
    const uint32_t want = (s->max_doc + 511) / 512;
    const uint32_t grid = std::max(1u, std::min(want, (uint32_t)c->cus * 4));
    launch_collect_multi(P, ORD, HIST, met_launch, grid, lds, p->stream);
    HIPX(hipGetLastError());
    HIPX(hipEventRecord(pl.e1, p->stream));
    p->last_bytes += bytes;
    p->last_path = 5;
    return true;
}

static void ensure_ord_hash(esgpu_ctx* c, const DevColumn* col, hipStream_t st);

// re-shape an allocated grid to newT ordinal columns, the old columns landing at column `shift` (histogram under
// histogram: a later segment widens the inner key range).  Rows are [T] cells, so every array moves as a strided 2D
// copy; the new cells start from the arrays' initial values (alloc_grid).
static void regrid_cols(esgpu_plan* p, Pipeline& pl, uint32_t newT, int64_t shift) {
    const uint32_t oldT = pl.T;
    std::vector<CardState> old_cards(pl.cards.size());
    for (size_t i = 0; i < pl.cards.size(); ++i) {
        old_cards[i].regs = std::move(pl.cards[i].regs);
        old_cards[i].sets = std::move(pl.cards[i].sets);
        old_cards[i].first = std::move(pl.cards[i].first);
        old_cards[i].cnt = std::move(pl.cards[i].cnt);
        old_cards[i].nonzero = std::move(pl.cards[i].nonzero);
    }
    struct { DevBuf g_cnt, g_ocnt, g_vcnt, g_sum, g_min, g_max, g_sq; } old;
    old.g_cnt = std::move(pl.g_cnt);
    old.g_ocnt = std::move(pl.g_ocnt);
    old.g_vcnt = std::move(pl.g_vcnt);
    old.g_sum = std::move(pl.g_sum);
    old.g_min = std::move(pl.g_min);
    old.g_max = std::move(pl.g_max);
    old.g_sq = std::move(pl.g_sq);
    pl.T = newT;
    alloc_grid(p, pl);
    auto cp = [&](DevBuf& dst, DevBuf& src, size_t esz) {  // [H][oldT] cells of esz bytes -> [H][newT] at column shift
        if (!src.p) return;
        HIPX(hipMemcpy2DAsync(dst.as<uint8_t>() + (size_t)shift * esz, (size_t)newT * esz, src.p, (size_t)oldT * esz,
                              (size_t)oldT * esz, pl.H, hipMemcpyDeviceToDevice, p->stream));
    };
    cp(pl.g_cnt, old.g_cnt, 8);
    cp(pl.g_vcnt, old.g_vcnt, 8);
    cp(pl.g_sum, old.g_sum, 8);
    cp(pl.g_min, old.g_min, 8);
    cp(pl.g_max, old.g_max, 8);
    cp(pl.g_sq, old.g_sq, 8);
    if (pl.ocnt_mode == OCNT_HIST && old.g_ocnt.p)
        HIPX(hipMemcpyAsync(pl.g_ocnt.p, old.g_ocnt.p, (size_t)pl.H * 8, hipMemcpyDeviceToDevice, p->stream));
    require(pl.ocnt_mode == OCNT_HIST || pl.ocnt_mode == OCNT_NONE, ESGPU_ERR_DEVICE, "ordinal regrid of per-term counts");
    for (size_t i = 0; i < pl.cards.size(); ++i) {
        CardState& cs = pl.cards[i];
        cp(cs.regs, old_cards[i].regs, cs.m);
        cp(cs.sets, old_cards[i].sets, (size_t)cs.cap * 4);
        cp(cs.first, old_cards[i].first, (size_t)cs.cap * 8);
        cp(cs.cnt, old_cards[i].cnt, 4);
        cp(cs.nonzero, old_cards[i].nonzero, 4);
    }
    HIPX(hipStreamSynchronize(p->stream));
}

// histogram under histogram: this segment's inner key indices as a u32 ordinal column (pl.ord_col), or null when the
// segment lacks the inner field.  The key range is taken from the request's first segment that has values; a later
// segment whose values fall outside it widens the range (up to 65536 keys): the grid's ordinal columns move over.
// materialize = false: only the key range is checked / taken; pl.ord_col describes the dimension (T) and its values
// are written later by materialize_hist_ords when the launch cannot derive the keys in its loader.
static void materialize_hist_ords(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s);
static const DevColumn* derive_hist_ords(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, bool materialize = true) {
    const DevColumn* src = s->col(pl.ord_field.c_str());
    if (!src) return nullptr;
    require(src->type == ESGPU_COL_I64 || src->type == ESGPU_COL_F64, ESGPU_ERR_UNSUPPORTED,
            "histogram over a keyword field runs on the CPU path");
    // a multi-valued inner field: one key index per value, in the source's CSR layout (collect_multi_kernel)
    require(!src->multi || pl.cards.empty(), ESGPU_ERR_UNSUPPORTED,
            "cardinality under a multi-valued inner histogram runs on the CPU path");
    const bool has = src->vmin <= src->vmax;
    if (pl.ord_table) {  // the bucket table grows to cover every segment's values; the grid's columns follow its keys
        if (pl.fresh) {
            pl.ot_lo = 0;
            pl.ot_hi = -1;
            pl.ot_start.clear();
            pl.ot_key.clear();
            pl.ot_slot.clear();
            pl.ord_keys = 0;
        }
        if (has && !(pl.ot_lo <= pl.ot_hi && src->vmin >= pl.ot_lo && src->vmax <= pl.ot_hi)) {
            int64_t lo = src->vmin, hi = src->vmax;
            if (pl.ot_lo <= pl.ot_hi) { lo = std::min(lo, pl.ot_lo); hi = std::max(hi, pl.ot_hi); }
            std::vector<int64_t> starts, keys;
            std::vector<uint32_t> slot;
            require(pl.ord_rnd.key_table(lo, hi, 65536, starts, keys, slot) && keys.size() <= 65536, ESGPU_ERR_UNSUPPORTED,
                    "an inner histogram over 65536 keys runs on the CPU path");
            int64_t shift = 0;
            if (!pl.ot_key.empty()) {
                auto it = std::lower_bound(keys.begin(), keys.end(), pl.ot_key.front());
                require(it != keys.end() && *it == pl.ot_key.front(), ESGPU_ERR_DEVICE, "inner bucket table is not a superset");
                shift = it - keys.begin();
            }
            const uint32_t old = pl.ord_keys;
            pl.ot_lo = lo;
            pl.ot_hi = hi;
            pl.ot_start = std::move(starts);
            pl.ot_key = std::move(keys);
            pl.ot_slot = std::move(slot);
            pl.ord_keys = (uint32_t)pl.ot_key.size();
            pl.d_ostart.alloc(p->ctx, std::max<size_t>(pl.ot_start.size(), 1) * 8);
            HIPX(hipMemcpyAsync(pl.d_ostart.p, pl.ot_start.data(), pl.ot_start.size() * 8, hipMemcpyHostToDevice, p->stream));
            pl.d_oslot.release();
            if (!pl.ot_slot.empty()) {
                pl.d_oslot.alloc(p->ctx, pl.ot_slot.size() * 4);
                HIPX(hipMemcpyAsync(pl.d_oslot.p, pl.ot_slot.data(), pl.ot_slot.size() * 4, hipMemcpyHostToDevice, p->stream));
            }
            HIPX(hipStreamSynchronize(p->stream));  // (the host tables are replaced by the next widening)
            // earlier segments of the request: their columns move to the new keys' positions
            if (!pl.fresh && pl.allocated && (old ? (shift != 0 || pl.ord_keys != old) : pl.T != pl.ord_keys))
                regrid_cols(p, pl, pl.ord_keys, old ? shift : 0);
        }
    } else {
    const int64_t kmin = has ? floor_div64(src->vmin - pl.ord_offset, pl.ord_interval) : 0;
    const int64_t kmax = has ? floor_div64(src->vmax - pl.ord_offset, pl.ord_interval) : -1;
    if (pl.fresh || pl.ord_keys == 0) {
        if (has) {
            require(kmax - kmin + 1 <= 65536, ESGPU_ERR_UNSUPPORTED, "an inner histogram over 65536 keys runs on the CPU path");
            pl.ord_key0 = kmin;
            pl.ord_keys = (uint32_t)(kmax - kmin + 1);
            // earlier segments of the request had no inner values: their grid has one empty ordinal column
            if (!pl.fresh && pl.allocated && pl.T != pl.ord_keys) regrid_cols(p, pl, pl.ord_keys, 0);
        } else if (pl.fresh) {
            pl.ord_key0 = 0;
            pl.ord_keys = 0;
        }
    } else if (has && (kmin < pl.ord_key0 || kmax >= pl.ord_key0 + (int64_t)pl.ord_keys)) {
        const int64_t nk0 = std::min(kmin, pl.ord_key0), nk1 = std::max(kmax, pl.ord_key0 + (int64_t)pl.ord_keys - 1);
        require(nk1 - nk0 + 1 <= 65536, ESGPU_ERR_UNSUPPORTED, "an inner histogram over 65536 keys runs on the CPU path");
        const int64_t shift = pl.ord_key0 - nk0;
        pl.ord_key0 = nk0;
        pl.ord_keys = (uint32_t)(nk1 - nk0 + 1);
        if (pl.allocated) regrid_cols(p, pl, pl.ord_keys, shift);
    }
    }
    if (!pl.ord_col) pl.ord_col = std::make_shared<DevColumn>();
    DevColumn& d = *pl.ord_col;
    d.name = pl.ord_field;
    d.type = ESGPU_COL_ORD_U32;
    d.multi = src->multi;
    d.n_values = src->multi ? src->n_values : 0;
    d.off_view = src->multi ? src->offsets.as<uint64_t>() : nullptr;
    d.value_count = std::max<uint32_t>(pl.ord_keys, 1);
    if (materialize) materialize_hist_ords(p, pl, s);
    return &d;
}
// three bucket levels: this segment's composite ordinals of the two terms fields (a * vcB + b) as pl.ord_col, or null
// when the segment lacks either field (its docs then fall in no bucket of the deepest level; the levels above count them
// through their own pipelines).  Both fields single-valued keyword fields numbered by the request's dictionaries.
// replay grids: each winner's row of inner ordinals padded to a multiple of 4 cells (16-byte aligned row starts for the
// top-k's vector loads)
static uint64_t replay_stride(uint64_t vcB) { return (std::max<uint64_t>(vcB, 1) + 3) & ~3ull; }

static const DevColumn* derive_comp_ords(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s) {
    const DevColumn* a = s->col(pl.ord_field.c_str());
    const DevColumn* b = s->col(pl.ord_field2.c_str());
    if (!a || !b) return nullptr;
    require(a->type == ESGPU_COL_ORD_U32 && b->type == ESGPU_COL_ORD_U32, ESGPU_ERR_UNSUPPORTED,
            "terms on numeric fields run on the CPU path");
    require(!a->multi && !b->multi, ESGPU_ERR_UNSUPPORTED, "multi-valued terms fields three bucket levels deep run on the CPU path");
    if (pl.fresh || !pl.tdict) {
        pl.tdict = a->ord_dict();
        pl.tdictB = b->ord_dict();
        pl.vcA = pl.replay ? p->slot_k : a->ord_count();  // replay: the surviving outer buckets' slots
        pl.vcB = b->ord_count();
    } else {
        require(same_dict(a->ord_dict(), pl.tdict) && same_dict(b->ord_dict(), pl.tdictB), ESGPU_ERR_INVALID,
                "segments number the terms of [" + pl.ord_field + "] or [" + pl.ord_field2 + "] differently: build an "
                "ordinal map (esgpu_ordinal_map_build) over the reader's segments first");
    }
    const uint64_t na = std::max<uint64_t>(pl.vcA, 1), nb = pl.replay ? replay_stride(pl.vcB) : std::max<uint64_t>(pl.vcB, 1);
    require(na * nb < 0xFFFFFFFFull, ESGPU_ERR_UNSUPPORTED, "three bucket levels over more than 2^32 term pairs");
    if (!pl.ord_col) pl.ord_col = std::make_shared<DevColumn>();
    DevColumn& d = *pl.ord_col;
    d.name = pl.ord_field;
    d.type = ESGPU_COL_ORD_U32;
    d.multi = false;
    d.value_count = na * nb;
    if (d.values.bytes < (size_t)s->n_pad * 4) d.values.alloc(p->ctx, (size_t)s->n_pad * 4);
    require(!pl.replay || p->slot_map, ESGPU_ERR_STATE, "replay outside a build");
    launch_comp_ords(a->ords().as<uint32_t>(), b->ords().as<uint32_t>(), (uint32_t)s->n_pad, (uint32_t)pl.vcA, (uint32_t)nb,
                     pl.replay ? p->slot_map : nullptr, p->slot_map_n, d.values.as<uint32_t>(), p->stream);
    HIPX(hipGetLastError());
    return &d;
}

static void materialize_hist_ords(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s) {
    const DevColumn* src = s->col(pl.ord_field.c_str());
    DevColumn& d = *pl.ord_col;
    if (pl.ord_table) {  // each value's step in the bucket table, its key slot
        const size_t nv = src->multi ? std::max<size_t>(src->n_values, 1) : (size_t)s->n_pad;
        if (d.values.bytes < nv * 4) d.values.alloc(p->ctx, nv * 4);
        launch_hist_ords_table((const int64_t*)wide_i64(p->ctx, src, s, p->stream), src->present.as<uint64_t>(),
                               src->multi ? src->offsets.as<uint64_t>() : nullptr, s->max_doc, s->n_pad,
                               src->type == ESGPU_COL_F64, pl.d_ostart.as<int64_t>(), (uint32_t)pl.ot_start.size(),
                               pl.d_oslot.p ? pl.d_oslot.as<uint32_t>() : nullptr, pl.ord_keys, d.values.as<uint32_t>(), p->stream);
        HIPX(hipGetLastError());
        return;
    }
    if (src->multi) {  // HistogramAggregator.collect: each value's key, a doc's repeated keys once (values are sorted)
        const size_t nv = std::max<size_t>(src->n_values, 1);
        if (d.values.bytes < nv * 4) d.values.alloc(p->ctx, nv * 4);
        launch_hist_ords_multi((const int64_t*)wide_i64(p->ctx, src, s, p->stream), src->offsets.as<uint64_t>(), s->max_doc,
                               src->type == ESGPU_COL_F64, pl.ord_interval, pl.ord_offset, pl.ord_key0, pl.ord_keys,
                               d.values.as<uint32_t>(), p->stream);
        HIPX(hipGetLastError());
        return;
    }
    if (d.values.bytes < (size_t)s->n_pad * 4) d.values.alloc(p->ctx, (size_t)s->n_pad * 4);
    launch_hist_ords((const int64_t*)wide_i64(p->ctx, src, s, p->stream), src->present.as<uint64_t>(), s->max_doc, s->n_pad,
                     src->type == ESGPU_COL_F64,
                     pl.ord_interval, pl.ord_offset, pl.ord_key0, pl.ord_keys, d.values.as<uint32_t>(), p->stream);
    HIPX(hipGetLastError());
}

// cardinality leaves of a bucket pipeline: register pass, nonzero recount, linear-counting pass (per segment, in
// order, so a bucket's set holds every encoded hash of every segment while it can still end in LINEAR_COUNTING)
// CardinalityAggregator.pickCollector (:86-108): a keyword field whose segment has few ordinals takes the
// OrdinalsCollector (hashes added per segment in ordinal order at postCollect), every other field the DirectCollector
// (hashes added in doc / value order).  memoryOverhead = object reference + FixedBitSet shell (8 + 32 bytes, the
// oracle's figures for a 64-bit JVM) + one bit per ordinal, against HyperLogLogPlusPlus.memoryUsage = 2^p.
static int ordinals_collector(uint64_t max_ord, int p) {
    return max_ord > 0 && (int64_t)(8 + 32 + (max_ord + 7) / 8) < ((int64_t)1 << p) / 4 ? 1 : 0;
}

// HyperLogLogPlusPlus.Hashset (:428-498) as the reference fills it: the distinct encoded hashes, each with the position
// at which its collector first added it, added in that order into m / 4 slots by linear probing from (k & mask).
// CardinalityAggregator.buildAggregation (:145-149) then copies the bucket's sketch into a fresh one by merge, which
// re-adds the values in slot order (a wrapped probe run lands elsewhere the second time); returns the copy's
// hashSet.values() -- the slot order writeTo and the coordinator's merge iterate (:519-528, :201-230)
static std::vector<uint32_t> hashset_values(std::vector<std::pair<uint64_t, uint32_t>>& added, int p) {
    std::sort(added.begin(), added.end());
    const uint32_t cap = (1u << p) / 4, mask = cap - 1;
    std::vector<uint32_t> t(cap, 0), copy(cap, 0);
    auto put = [&](std::vector<uint32_t>& tab, uint32_t k) {
        uint32_t i = k & mask;
        while (tab[i] != 0 && tab[i] != k) i = (i + 1) & mask;
        tab[i] = k;
    };
    for (const auto& e : added) put(t, e.second);
    for (uint32_t k : t) if (k) put(copy, k);
    std::vector<uint32_t> out;
    out.reserve(added.size());
    for (uint32_t k : copy) if (k) out.push_back(k);
    return out;
}

static void collect_cards(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, const uint64_t* d_accept) {
    const bool ORD = pl.term_spec >= 0, HIST = pl.hist_spec >= 0;
    const DevColumn* oc = ORD ? (pl.ord_hist || pl.comp ? pl.ord_col.get() : s->col(pl.ord_field.c_str())) : nullptr;
    const DevColumn* hc = HIST ? s->col(pl.hist_field.c_str()) : nullptr;
    CollectParams G{};
    G.n_docs = s->max_doc;
    G.ord = oc ? oc->ords().as<uint32_t>() : nullptr;
    G.ord_off = (oc && oc->multi) ? oc->offsets.as<uint64_t>() : nullptr;
    G.T = pl.T;
    G.H = pl.H;
    G.hv = hc && !pl.inner_terms ? (const int64_t*)wide_i64(p->ctx, hc, s, p->stream) : nullptr;
    G.hv_present = hc ? hc->present.as<uint64_t>() : nullptr;
    G.hv_off = (hc && hc->multi) ? hc->offsets.as<uint64_t>() : nullptr;
    G.hv_f64 = hc && hc->type == ESGPU_COL_F64;
    G.interval = pl.interval;
    G.offset = pl.offset;
    G.key0 = pl.key0;
    G.kstart = (HIST && pl.ktable) ? pl.d_kstart.as<int64_t>() : nullptr;
    G.kslot = G.kstart ? pl.d_kslot.as<uint32_t>() : nullptr;
    G.nsteps = (uint32_t)pl.kt_start.size();
    if (hc && pl.inner_terms) {  // terms under terms: the inner field's (global) ordinals are the keys
        G.hv = (const int64_t*)hc->ords().p;
        G.hv_present = nullptr;
        G.hv_f64 = 0;
        G.hord = 1;
    }
    G.accept = d_accept;
    PredDev pred[4];
    int npred = 0;
    uint64_t fbytes = 0;
    set_preds(p, pl, s, pred, &npred, &fbytes, &G.accept);
    if (npred > 0) {
        uint64_t* bits = (uint64_t*)p->s_fbits.ensure(p->ctx, std::max<size_t>(s->n_pad / 64, 1) * 8);
        launch_filter_bits(s->max_doc, G.accept, pred, npred, bits, p->stream);
        HIPX(hipGetLastError());
        G.accept = bits;
    }
    const uint64_t B = (uint64_t)pl.T * pl.H;
    const uint32_t grid = std::max(1u, std::min((s->max_doc + 255) / 256, (uint32_t)p->ctx->cus * 8));
    for (CardState& cs : pl.cards) {
        const DevColumn* col = s->col(cs.field.c_str());
        if (!col || s->max_doc == 0) continue;  // unmapped in this segment: no values
        CardParams C{};
        C.G = G;
        C.col = wide_i64(p->ctx, col, s, p->stream);  // (any column type: only a released long is rebuilt)
        C.off = col->multi ? col->offsets.as<uint64_t>() : nullptr;
        C.present = col->present.as<uint64_t>();
        C.p = cs.p;
        if (col->type == ESGPU_COL_ORD_U32) {
            C.kind = HLL_ORD;
            ensure_ord_hash(p->ctx, col, p->stream);
            C.ord_hash = col->ord_hash.as<uint64_t>();
            C.n_ords = col->value_count;
            C.pos_ord = ordinals_collector(col->value_count, cs.p);
        } else {
            C.kind = col->type == ESGPU_COL_F64 ? HLL_F64 : HLL_I64;
        }
        C.regs = cs.regs.as<uint8_t>();
        C.sets = cs.sets.as<uint32_t>();
        C.set_cnt = cs.cnt.as<uint32_t>();
        C.nonzero = cs.nonzero.as<uint32_t>();
        C.cap = cs.cap;
        C.thr = cs.thr;
        C.first = cs.first.as<unsigned long long>();
        C.pos_base = (uint64_t)p->seg_seq << 40;
        launch_card(C, ORD, HIST, 0, grid, p->stream);
        launch_card_nonzero(C.regs, B, cs.p, C.nonzero, p->stream);
        launch_card(C, ORD, HIST, 1, grid, p->stream);
        HIPX(hipGetLastError());
        p->last_bytes += column_bytes(col, s->max_doc);
    }
    HIPX(hipEventRecord(pl.e1, p->stream));
}

// 0 = nothing collected, 1 = the grid, 2 = only the outer doc counts (the segment lacks the inner dimension's field)
static int collect_grid_cells(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, const uint64_t* d_accept);

static bool collect_grid(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, const uint64_t* d_accept) {
    const int done = collect_grid_cells(p, pl, s, d_accept);
    if (done == 1 && !pl.cards.empty()) collect_cards(p, pl, s, d_accept);
    return done != 0;
}

#ifndef ESGPU_TERMS_COPIES
#define ESGPU_TERMS_COPIES 4
#endif
#ifndef ESGPU_COPIES_HIST
#define ESGPU_COPIES_HIST 0  // terms x histogram grids: copies measured within noise
#endif
#ifndef ESGPU_ROW_TOPK
#define ESGPU_ROW_TOPK 1  // terms under a histogram, count orders: per-row selection on the GPU at build
#endif
#ifndef ESGPU_FUSE_HIST_ORDS
#define ESGPU_FUSE_HIST_ORDS 1  // histogram under histogram: inner key index derived in the collect kernel's loader
#endif
static constexpr uint32_t kTermsCopies = ESGPU_TERMS_COPIES;
#ifndef ESGPU_COMPACT_ROWS
#define ESGPU_COMPACT_ROWS 1  // build: histogram children of terms compacted on the GPU (0: host assembly, for A/B)
#endif

// cells of a terms-under-terms grid above which the inner buckets are collected breadth-first (ESGPU_DEFER_CELLS
// overrides: tests force the replay on small grids)
static uint64_t defer_cells() {
    const char* e = std::getenv("ESGPU_DEFER_CELLS");
    if (e && *e) return std::strtoull(e, nullptr, 10);
    return 1ull << 31;
}

static int collect_grid_cells(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, const uint64_t* d_accept) {
    const bool ORD = pl.term_spec >= 0, HIST = pl.hist_spec >= 0;
    const DevColumn* oc = !ORD ? nullptr : pl.ord_hist ? derive_hist_ords(p, pl, s, false)
                        : pl.comp ? derive_comp_ords(p, pl, s) : s->col(pl.ord_field.c_str());
    if (pl.comp && !oc) return 0;
    const DevColumn* hc = HIST ? s->col(pl.hist_field.c_str()) : nullptr;
    const DevColumn* mc = pl.met > 0 ? s->col(pl.metric_field.c_str()) : nullptr;
    const bool terms_outer = pl.outer == pl.term_spec;
    if (pl.inner_terms && pl.fresh) pl.deferred = false;
    if (pl.inner_terms && pl.can_defer && pl.fresh && oc && hc && oc->type == ESGPU_COL_ORD_U32 && hc->type == ESGPU_COL_ORD_U32 &&
        !oc->multi && !hc->multi) {
        // terms under terms over the dense budget: breadth-first (TermsAggregator.shouldDefer / BestBucketsDeferringCollector)
        // -- the outer doc counts now, the inner buckets replayed at build for the outer winners; the replay grid (winners x
        // inner ordinals) must fit, and an inner order by a metric selects on the host (rows of at most 65,536 terms)
        const uint64_t T = std::max<uint64_t>(oc->ord_count(), 1), H = std::max<uint64_t>(hc->ord_count(), 1);
        const SpecNode& to = p->specs[pl.outer];
        const SpecNode& ti = p->specs[pl.hist_spec];
        const uint64_t W = std::max<uint64_t>(1, std::min<uint64_t>(T, (uint64_t)std::max<int64_t>(to.s.shard_size, 0)));
        const bool agg2 = ti.s.order == ESGPU_ORDER_AGG_ASC || ti.s.order == ESGPU_ORDER_AGG_DESC;
        pl.deferred = T * H > defer_cells() && W * replay_stride(H) <= (1ull << 31) && (!agg2 || H <= 65536);
    }
    if (pl.deferred && oc) {
        require(!oc->multi && !(hc && hc->multi), ESGPU_ERR_UNSUPPORTED,
                "a breadth-first replay over multi-valued terms fields runs on the CPU path");
    }
    // unmapped fields: a bucket aggregation over a missing field collects nothing (ValuesSource null); when only the
    // inner bucket aggregation's field is missing, the outer buckets still count the segment's docs and the inner
    // aggregation of those docs is empty.  A deferred pipeline collects the same way: only the outer doc counts.
    const bool inner_missing = ORD && HIST && ((pl.deferred && oc) || (terms_outer ? (oc && !hc) : (hc && !oc)));
    if (((ORD && !oc) || (HIST && !hc)) && !inner_missing) return 0;
    if (oc) require(oc->type == ESGPU_COL_ORD_U32, ESGPU_ERR_UNSUPPORTED, "terms on numeric fields run on the CPU path");
    if (hc && pl.inner_terms) {  // multi-valued outer / inner fields take the CSR kernel (inner ordinals as keys)
        require(hc->type == ESGPU_COL_ORD_U32, ESGPU_ERR_UNSUPPORTED, "terms on numeric fields run on the CPU path");
    } else if (hc) {
        require(hc->type == ESGPU_COL_I64 || hc->type == ESGPU_COL_F64, ESGPU_ERR_UNSUPPORTED,
                "histogram over a keyword field runs on the CPU path");
    }
    if (mc) require(mc->type == ESGPU_COL_I64 || mc->type == ESGPU_COL_F64, ESGPU_ERR_UNSUPPORTED, "metric over non-numeric field");
    // any multi-valued column (aggregated field or filter field) takes the CSR kernel
    bool multi = (oc && oc->multi) || (hc && hc->multi) || (mc && mc->multi);
    for (size_t k = 0; k < p->filter_fields.size(); ++k) {
        const DevColumn* fc = applies(p, pl, k) ? s->col(p->filter_fields[k].c_str()) : nullptr;
        if (fc && fc->multi) multi = true;
    }
    // histogram under histogram: the collect kernel's loader derives the inner key index from the field (no ordinal
    // column written and re-read) unless a kernel that reads the materialised column runs on this segment (the CSR
    // kernel, cardinality leaves) or the key span does not fit the loader's 32-bit division
    const DevColumn* osrc = pl.ord_hist && oc ? s->col(pl.ord_field.c_str()) : nullptr;
    int64_t ord_base = 0;
    const bool fuse_ords = osrc && ESGPU_FUSE_HIST_ORDS && !multi && pl.cards.empty() && pl.ord_interval > 0 &&
                           pl.ord_interval < (1ll << 32) && (uint64_t)pl.ord_keys * (uint64_t)pl.ord_interval < (1ull << 32) &&
                           !__builtin_mul_overflow(pl.ord_key0, pl.ord_interval, &ord_base) &&
                           !__builtin_add_overflow(ord_base, pl.ord_offset, &ord_base);
    if (osrc && !fuse_ords) materialize_hist_ords(p, pl, s);
    // an unmapped metric field collects nothing (ValuesSource null => NO_OP collector); counts stay separate
    const int met_launch = mc ? pl.met : 0;
    const bool first_segment = pl.fresh;
    if (!first_segment) zero_counts(p, pl);  // (a first segment that launched nothing left them pending)
    // ---- shape the grid ----
    if (pl.fresh) {  // first segment since create / reset: the grid shape and the dictionary are taken from it
        pl.kt_lo = 0;
        pl.kt_hi = -1;
        pl.kt_start.clear();
        pl.kt_key.clear();
        pl.kt_slot.clear();
    }
    int64_t kmin = 0, kmax = 0;
    bool has_keys = false;
    int64_t table_shift = 0;
    const uint32_t H_before = pl.H;
    if (HIST && hc && pl.inner_terms) {  // one key per inner ordinal (deferred: none, the grid is the outer counts)
        if (!pl.deferred) {
            kmin = 0;
            kmax = (int64_t)std::max<uint64_t>(hc->ord_count(), 1) - 1;
            has_keys = true;
        }
    } else if (HIST && hc && hc->vmin <= hc->vmax) {
        if (pl.ktable) {
            table_shift = build_key_table(p, pl, hc->vmin, hc->vmax);
            kmin = 0;
            kmax = (int64_t)pl.kt_key.size() - 1;
        } else {
            kmin = floor_div64(hc->vmin - pl.offset, pl.interval);
            kmax = floor_div64(hc->vmax - pl.offset, pl.interval);
        }
        has_keys = true;
    }
    const bool sparse_metric = pl.met > 0 && (!mc || mc->present.p || mc->multi);
    // ords may be missing; a doc may have several keys: then the outer counts cannot be summed from the cells
    const bool inner_sparse = ORD && HIST && (inner_missing || pl.inner_terms ||
                                              (terms_outer ? (hc->present.p != nullptr || hc->multi) : true));
    if (!pl.allocated || pl.fresh) {
        const uint32_t T = oc ? (uint32_t)std::max<uint64_t>(oc->ord_count(), 1) : 1;
        const int64_t key0 = has_keys ? kmin : 0;
        require(!HIST || !has_keys || kmax - kmin + 1 <= 64 * 1024 * 1024, ESGPU_ERR_UNSUPPORTED,
                "histogram key range too large for a dense grid");
        const uint32_t H = HIST ? (uint32_t)(has_keys ? kmax - kmin + 1 : 1) : 1;
        require((uint64_t)T * H <= (1ull << 31), ESGPU_ERR_UNSUPPORTED, "bucket grid too large");
        const int vcnt = sparse_metric ? 1 : 0;
        int ocnt = OCNT_NONE;
        if (ORD && HIST) ocnt = inner_sparse ? (terms_outer ? OCNT_TERMS : OCNT_HIST) : OCNT_TERMS_DERIVED;
        // a reset plan keeps its buffers (already zeroed) when the new request's first segment has the same shape
        const bool same = pl.allocated && T == pl.T && H == pl.H && key0 == pl.key0 && vcnt == pl.vcnt_mode &&
                          ocnt == pl.ocnt_mode;
        pl.T = T;
        pl.H = H;
        pl.key0 = key0;
        pl.vcnt_mode = vcnt;
        pl.ocnt_mode = ocnt;
        pl.keyed = has_keys;
        pl.value_count = oc ? oc->ord_count() : (ORD ? 0 : 1);
        if (!pl.comp) pl.tdict = oc ? oc->ord_dict() : nullptr;
        pl.tdict2 = pl.inner_terms && hc ? hc->ord_dict() : nullptr;
        pl.value_count2 = pl.inner_terms && hc ? hc->ord_count() : 0;
        if (!same) alloc_grid(p, pl);
        pl.fresh = false;
    } else {
        if (oc && !pl.tdict && !pl.ord_hist && !pl.comp)
            throw EsError(ESGPU_ERR_UNSUPPORTED, "terms field [" + pl.ord_field + "] unmapped in the first segment under a histogram");
        if (oc && pl.ord_hist)
            require(pl.T == std::max<uint32_t>(pl.ord_keys, 1), ESGPU_ERR_UNSUPPORTED,
                    "the inner histogram had no values in the request's first segment: runs on the CPU path");
        if (oc && !pl.ord_hist && !pl.comp) require(same_dict(oc->ord_dict(), pl.tdict), ESGPU_ERR_INVALID,
                         "segments number the terms of [" + pl.ord_field + "] differently: build an ordinal map "
                         "(esgpu_ordinal_map_build) over the reader's segments first");
        if (pl.inner_terms && hc) {
            if (!pl.tdict2) { pl.tdict2 = hc->ord_dict(); pl.value_count2 = hc->ord_count(); }
            require(same_dict(hc->ord_dict(), pl.tdict2), ESGPU_ERR_INVALID,
                    "segments number the terms of [" + pl.hist_field + "] differently: build an ordinal map "
                    "(esgpu_ordinal_map_build) over the reader's segments first");
        }
        if (HIST && has_keys && !pl.keyed) {
            // the earlier segments had no histogram values: their single placeholder row is empty
            require(kmax - kmin + 1 <= 64 * 1024 * 1024, ESGPU_ERR_UNSUPPORTED, "histogram key range too large for a dense grid");
            pl.key0 = kmin;
            regrid(p, pl, (uint32_t)(kmax - kmin + 1), 0);
            pl.keyed = true;
        } else if (HIST && has_keys) {
            if (!pl.ktable) grow_keys(p, pl, kmin, kmax);
            else if ((uint32_t)pl.kt_key.size() != H_before || table_shift != 0) regrid(p, pl, (uint32_t)pl.kt_key.size(), table_shift);
        }
        if (sparse_metric && !pl.vcnt_mode) {
            // the metric field turns sparse in this segment: value counts split from doc counts, which they equalled
            // so far (every earlier doc had exactly one value)
            const size_t cells = (size_t)pl.T * pl.H;
            pl.g_vcnt.alloc(p->ctx, cells * 8);
            HIPX(hipMemcpyAsync(pl.g_vcnt.p, pl.g_cnt.p, cells * 8, hipMemcpyDeviceToDevice, p->stream));
            pl.vcnt_mode = 1;
        }
        // the histogram field turns sparse / multi-valued: outer counts are counted per doc from here on (the derived
        // counts of the earlier segments are already in g_ocnt)
        if (inner_sparse && pl.ocnt_mode == OCNT_TERMS_DERIVED) pl.ocnt_mode = OCNT_TERMS;
    }
    // ---- launch configuration ----
    // what this launch collects: the grid, or -- the segment lacking the inner dimension's field -- only the outer doc
    // counts, as a one-dimensional grid over g_ocnt
    const bool L_ORD = ORD && (!inner_missing || terms_outer), L_HIST = HIST && (!inner_missing || !terms_outer);
    const uint32_t LT = L_ORD ? pl.T : 1, LH = L_HIST ? pl.H : 1;
    const int L_met = inner_missing ? 0 : met_launch;
    const int L_vcnt = inner_missing ? 0 : pl.vcnt_mode, L_ocnt = inner_missing ? (int)OCNT_NONE : pl.ocnt_mode;
    CollectParams P{};
    P.n_docs = s->max_doc;
    P.n_blocks = s->n_pad / kBlockDocs;
    for (uint32_t& h : P.hot_t) h = kMissingOrd;
    if (P.n_blocks == 0) return 0;
    P.ord = oc ? oc->ords().as<uint32_t>() : nullptr;
    if (fuse_ords && L_ORD) {
        P.ord = nullptr;
        P.ord_src = osrc->values.as<int64_t>();
        P.ord_src_present = osrc->present.as<uint64_t>();
        P.ord_src_f64 = osrc->type == ESGPU_COL_F64;
        P.ord_base = ord_base;
        P.ord_span = (uint32_t)((uint64_t)pl.ord_keys * (uint64_t)pl.ord_interval);
        P.ord_div = (uint32_t)pl.ord_interval;
        const MagicU32 mg = make_magic(P.ord_div);
        P.omg_m = mg.m; P.omg_s1 = mg.s1; P.omg_s2 = mg.s2;
    }
    P.T = LT;
    P.H = LH;
    P.hv = hc ? hc->values.as<int64_t>() : nullptr;
    P.hv_present = hc ? hc->present.as<uint64_t>() : nullptr;
    P.hv_f64 = hc && hc->type == ESGPU_COL_F64;
    if (hc && pl.inner_terms) {  // u32 (global) ordinals of the inner terms field
        P.hv = (const int64_t*)hc->ords().p;
        P.hv_present = nullptr;
        P.hv_f64 = 0;
        P.hord = L_HIST ? 1 : 0;
    }
    P.interval = pl.interval;
    P.offset = pl.offset;
    P.key0 = pl.key0;
    P.kstart = (HIST && pl.ktable) ? pl.d_kstart.as<int64_t>() : nullptr;
    P.kslot = P.kstart ? pl.d_kslot.as<uint32_t>() : nullptr;
    P.nsteps = (uint32_t)pl.kt_start.size();
    P.zmin = hc ? hc->zmin.as<int64_t>() : nullptr;
    P.zmax = hc ? hc->zmax.as<int64_t>() : nullptr;
    P.mv = mc ? mc->values.p : nullptr;
    P.mv_present = mc ? mc->present.as<uint64_t>() : nullptr;
    P.mv_f64 = mc && mc->type == ESGPU_COL_F64;
    P.vcnt_mode = L_vcnt;
    P.ocnt_mode = L_ocnt;
    P.accept = d_accept;
    if (inner_missing) { P.mv = nullptr; P.mv_present = nullptr; P.mv_f64 = 0; }
    uint64_t bytes_per_doc = (oc ? (pl.ord_hist ? 8 : 4) : 0) + (hc && !pl.deferred ? (pl.inner_terms ? 4 : 8) : 0) +
                             (mc && !inner_missing ? 8 : 0);
    set_preds(p, pl, s, P.pred, &P.npred, &bytes_per_doc, &P.accept);
    d_accept = P.accept;  // the clauses folded into a bitset when there are more than kMaxPreds
    P.g_cnt = inner_missing ? pl.g_ocnt.as<unsigned long long>() : pl.g_cnt.as<unsigned long long>();
    P.g_ocnt = pl.g_ocnt.as<unsigned long long>();
    P.g_vcnt = pl.g_vcnt.as<unsigned long long>();
    P.g_sum = pl.g_sum.as<double>();
    P.g_min = pl.g_min.as<unsigned long long>();
    P.g_max = pl.g_max.as<unsigned long long>();
    P.g_sq = pl.g_sq.as<double>();
    // compensated sums (DESIGN §5 "Float parity"): while every partial sum of the request's metric values is an integer
    // below 2^53 the grid's f64 adds are exact in any order; otherwise (a double metric, or long values whose magnitude
    // times their number -- squared for sums of squares -- reaches 2^53) the flushes add double-doubles, folded back into
    // the grid after the launch (dd_fold below)
    if (first_segment) {
        pl.dd = false;
        pl.dd_vals = 0;
        pl.dd_amax = 0;
    }
    if (L_met > 0 && mc && !inner_missing) {
        pl.dd_vals += mc->multi ? mc->n_values : (uint64_t)s->max_doc;
        if (mc->type == ESGPU_COL_F64 || dd_forced()) {
            pl.dd = true;
        } else if (mc->vmin <= mc->vmax) {
            auto mag = [](int64_t v) { return v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v; };
            pl.dd_amax = std::max(pl.dd_amax, std::max(mag(mc->vmin), mag(mc->vmax)));
            const long double n = (long double)pl.dd_vals, a = (long double)pl.dd_amax, lim = 9007199254740992.0L;
            if (n * a >= lim || (pl.met >= 3 && n * a * a >= lim)) pl.dd = true;
        }
    }
    const size_t dd_cells = (size_t)pl.T * pl.H;
    if (pl.dd && L_met > 0 && !inner_missing) {
        auto lo = [&](DevBuf& b) {
            if (b.p && b.bytes >= dd_cells * 8) return b.as<double>();
            b.alloc(p->ctx, dd_cells * 8 + dd_cells * 2);
            HIPX(hipMemsetAsync(b.p, 0, b.bytes, p->stream));
            return b.as<double>();
        };
        P.g_sum_lo = lo(pl.g_sum_lo);
        if (pl.met >= 3 && P.g_sq) P.g_sq_lo = lo(pl.g_sq_lo);
    }
    // upload-width values the launch reads, rebuilt if released (esgpu_segment_release_wide): the CSR kernel reads them
    // all; the single-valued kernel the ones no compact copy replaces
    auto need_wide = [&](bool all) {
        if (P.ord_src && osrc && osrc->wide_released) P.ord_src = (const int64_t*)wide_i64(p->ctx, osrc, s, p->stream);
        if (L_HIST && hc && !pl.inner_terms && hc->wide_released && (all || !(P.hv32 || P.hv16)))
            P.hv = (const int64_t*)wide_i64(p->ctx, hc, s, p->stream);
        if (L_met > 0 && mc && mc->wide_released && (all || (!P.mv32 && !P.mv16))) P.mv = wide_i64(p->ctx, mc, s, p->stream);
    };
    auto dd_fold = [&] {
        if (P.g_sum_lo) launch_dd_fold(P.g_sum, P.g_sum_lo, dd_cells, p->stream);
        if (P.g_sq_lo) launch_dd_fold(P.g_sq, P.g_sq_lo, dd_cells, p->stream);
        HIPX(hipGetLastError());
    };
    const int ret = inner_missing ? 2 : 1;
    if (multi && !inner_missing) count_width(p, pl, s, false, first_segment);
    if (multi) {
        need_wide(true);
        zero_counts(p, pl);
        const bool ok = collect_multi(p, pl, s, P, L_ORD ? oc : nullptr, L_HIST ? hc : nullptr, inner_missing ? nullptr : mc,
                                      L_met, d_accept);
        dd_fold();
        return ok ? ret : 0;
    }
    // compact columns: 2 B per ordinal instead of 4, 4 B per timestamp instead of 8 -- the reported (algorithmic) bytes
    // are the bytes this layout must move (SURVEY §8(d)'s upload-width figure would put config 5 above the HBM peak)
    const DevColumn* t16 = nullptr;  // the key column's block deltas (ensure_b16)
    bool tcomp = false;              // the key column is read as compact deltas (32-bit, or block deltas)
    if (compact_cols(p->ctx)) {
        const bool plain_ord = oc && !pl.comp && !pl.ord_hist && oc == s->col(pl.ord_field.c_str());
        if (L_ORD && P.ord && plain_ord && !oc->multi && oc->ord_count() < 0xFFFFu) {
            P.ord16 = ensure_ord16(p->ctx, oc, s, p->stream);
            if (P.ord16) bytes_per_doc -= 2;
            // counting terms x histogram grids: the hot ordinal the kernel counts in registers in single-key zone blocks
            // (ESGPU_ORDH_HOT; the packed-cell grids take theirs below)
            if (P.ord16 && L_HIST && L_met == 0) sampled_hot_ords(p->ctx, oc, s, P.hot_t);
        }
        if (L_HIST && hc && !pl.inner_terms && !P.kstart && hc->type == ESGPU_COL_I64 && !hc->multi && hc->vmin <= hc->vmax &&
            (uint64_t)hc->vmax - (uint64_t)hc->vmin < (1ull << 32)) {
            // a dense time-sorted column has block deltas (2 B per doc), which the raw-load kernels read: taken below once
            // the launch is known to be one of them -- no 32-bit copy is built for it then
            if (b16_on(p->ctx) && !hc->present.p) t16 = ensure_b16(p->ctx, hc, s, p->stream);
            if (t16) {
                P.hv_base = hc->vmin;
                tcomp = true;
            } else {
                P.hv32 = ensure_d32(p->ctx, hc, s, p->stream);
                if (P.hv32) {
                    P.hv_base = hc->vmin;
                    bytes_per_doc -= 4;
                    tcomp = true;
                }
            }
        }
    }
    // packed integer metric cells (CollectParams.pk_shift): terms grids with avg / stats over a dense
    // single-valued long metric whose values span < 2^32, read as the column's u32 deltas -- the kernel instantiations
    // exist for no key and for an affine key over the compact timestamps (with_vk); confirmed below once the workgroup
    // ranges are known (neither packed field may overflow)
    bool pi = false;
    const int hk_launch = L_HIST ? (P.hord ? 3 : P.kstart ? 2 : 1) : 0;
    if (pi_cells(p->ctx) && compact_cols(p->ctx) && L_ORD && !P.ord_src && (L_met == 1 || L_met == 2) && mc && mc->type == ESGPU_COL_I64 &&
        !mc->multi && !mc->present.p && !L_vcnt && mc->vmin <= mc->vmax && (uint64_t)mc->vmax - (uint64_t)mc->vmin < (1ull << 32) &&
        (hk_launch == 0 || (hk_launch == 1 && tcomp && !P.hv_f64)) && !dyn_claim_on()) {
        // values spanning < 2^16 (a latency in ms, a status code): the 16-bit deltas, 2 B per doc (instantiated with
        // 16-bit ordinals; those kernels load raw words and unpack them when the docs are processed: dense timestamps
        // only).  Only the copy the kernel reads is built -- no 32-bit copy beside the 16-bit one (HBM per segment)
        const bool span16 = P.ord16 && d16_on() && (uint64_t)mc->vmax - (uint64_t)mc->vmin < (1ull << 16) &&
                            !(hk_launch == 1 && P.hv_present);
        const uint16_t* d16 = span16 ? ensure_d16(p->ctx, mc, s, p->stream) : nullptr;
        const uint32_t* d32 = d16 ? nullptr : ensure_d32(p->ctx, mc, s, p->stream);
        if (d16 || d32) {
            P.mv32 = d32;
            P.mv16 = d16;
            P.mv_base = mc->vmin;
            sampled_hot_ords(p->ctx, oc, s, P.hot_t);
            pi = true;
            // a filtered request (clauses or live docs) takes the packed cells through one folded accept bitset, which
            // is instantiated with the 16-bit columns only (with_vk)
            if ((P.npred > 0 || P.accept) && !(P.ord16 && P.mv16)) {
                pi = false;
                P.mv32 = nullptr;
                P.mv16 = nullptr;
            }
        }
    }
    auto pi_fits = [&](uint32_t bpw) {  // docs of one workgroup range: count field and sum-of-deltas field both fit
        const uint64_t docs = std::min<uint64_t>((uint64_t)bpw * kBlockDocs, (uint64_t)s->max_doc);
        const uint32_t cbits = 64 - __builtin_clzll(docs | 1);
        const uint32_t sh = 64 - cbits;
        const unsigned __int128 maxsum = (unsigned __int128)docs * (uint64_t)((uint64_t)mc->vmax - (uint64_t)mc->vmin);
        // the decoded sum count * base + deltas must stay a long as well
        const unsigned __int128 mag = (unsigned __int128)docs *
                                      (uint64_t)std::max<int64_t>(mc->vmax < 0 ? -(mc->vmax + 1) : mc->vmax, mc->vmin < 0 ? -(mc->vmin + 1) : mc->vmin);
        P.pk_shift = sh;
        return sh < 64 && (maxsum >> sh) == 0 && (mag >> 62) == 0;
    };
  relaunch:
    // otherwise a long metric spanning < 2^32 is still read as its compact u32 deltas where a kernel instantiation reads
    // them (VK bit 128, with_vk): date_histogram{stats / extended_stats / avg} over compact timestamps, extended_stats
    // under terms over compact columns -- 4 B per doc instead of 8, the values restored exactly in the loader
    bool m32 = false;
    if (!pi && compact_cols(p->ctx) && L_met > 0 && mc && mc->type == ESGPU_COL_I64 && !mc->multi && mc->vmin <= mc->vmax &&
        (uint64_t)mc->vmax - (uint64_t)mc->vmin < (1ull << 32) && !P.mv_f64 && !inner_missing &&
        ((!L_ORD && hk_launch == 1 && tcomp && !P.hv_f64) ||
         (L_ORD && L_met == 3 && !P.ord_src && P.ord16 && (hk_launch == 0 || (hk_launch == 1 && tcomp && !P.hv_f64))))) {
        // histogram-only grids over a dense metric spanning < 2^16 with |values| < 2^26 (v * v exact, as the reference's
        // rounded products then are), read without a filter by the raw-load kernels: the 16-bit deltas and integer run
        // accumulators (VK bit 2048), 6 B per doc -- and no 32-bit copy
        const bool int_runs = !L_ORD && int_runs_on() && d16_on() && raw_hist_on() && !P.accept && P.npred == 0 &&
                              !mc->present.p && !P.hv_present && (uint64_t)mc->vmax - (uint64_t)mc->vmin < (1ull << 16) &&
                              mc->vmin > -(1ll << 26) && mc->vmax < (1ll << 26);
        const uint16_t* d16 = int_runs ? ensure_d16(p->ctx, mc, s, p->stream) : nullptr;
        const uint32_t* d32 = d16 ? nullptr : ensure_d32(p->ctx, mc, s, p->stream);
        if (d16 || d32) {
            P.mv32 = d32;
            P.mv16 = d16;
            P.mv_base = mc->vmin;
            P.pk_shift = 0;
            m32 = true;
        }
    }

    // LDS sizing: the whole grid if it fits, else a sliding window over the key dimension (time-sorted data)
#ifndef ESGPU_LDS_PAIR  // LDS budget of a window that keeps two workgroups per CU
#define ESGPU_LDS_PAIR (64 * 1024)
#endif
#ifndef ESGPU_LDS_PI  // packed cells: a window that keeps three 512-thread workgroups per CU (24 waves: more loads in flight)
#define ESGPU_LDS_PI (52 * 1024)
#endif
    const size_t kLdsPair = pi ? (size_t)ESGPU_LDS_PI : (size_t)ESGPU_LDS_PAIR, kLdsMax = 150 * 1024;
    uint32_t W = LH;
    size_t lds = collect_lds_bytes(LT, W, L_met, L_vcnt, L_ocnt, 1, pi);
    P.lds_mode = 1;
    P.windowed = 0;
    if (lds > kLdsPair) {
        if (L_HIST && !P.kslot && !P.hord) {  // the key window needs buckets that rise with the value (zone-map ranges)
            uint32_t w = LH;
            while (w > 1 && collect_lds_bytes(LT, w, L_met, L_vcnt, L_ocnt, 1, pi) > kLdsPair) w = (w + 1) / 2;
            if (collect_lds_bytes(LT, w, L_met, L_vcnt, L_ocnt, 1, pi) > kLdsPair) w = 1;
            W = w;
            P.windowed = 1;
            lds = collect_lds_bytes(LT, W, L_met, L_vcnt, L_ocnt, 1, pi);
        }
        if (lds > kLdsMax) {
            P.lds_mode = 0;
            P.windowed = 0;
            lds = 0;
            W = LH;
        }
    }
    // Roughly time-ordered data (merged segments: docs displaced by up to an hour or so) has blocks spanning more keys
    // than a two-per-CU window holds; each such block is then read once per W keys (multi-pass groups).  When the
    // segment's blocks typically span more keys (90th percentile of the zone-map ranges), widen the window instead:
    // one 1024-thread workgroup per CU with up to kLdsMax of LDS (the same 16 waves per CU).
    bool wide = false;
#ifndef ESGPU_WIDE_WINDOW
#define ESGPU_WIDE_WINDOW 1
#endif
#ifndef ESGPU_WIDE_MIN  // widen to at least this many keys whenever the two-per-CU window is narrower (A/B knob)
#define ESGPU_WIDE_MIN 0
#endif
    if (ESGPU_WIDE_WINDOW && P.lds_mode && P.windowed && !P.kstart && hc && pl.interval > 0) {
        const int64_t need = std::min<int64_t>(std::max<int64_t>(hc->zspan / pl.interval + 2, ESGPU_WIDE_MIN), (int64_t)LH);
        if (need > (int64_t)W) {
            uint32_t w2 = W;
            while ((int64_t)w2 < need && collect_lds_bytes(LT, w2 + 1, L_met, L_vcnt, L_ocnt, 1, pi) <= kLdsMax) ++w2;
            if (w2 > W) {
                W = w2;
                wide = true;
                if (W >= LH) { W = LH; P.windowed = 0; }
                lds = collect_lds_bytes(LT, W, L_met, L_vcnt, L_ocnt, 1, pi);
            }
        }
    }
    P.W = W;
    // grids with a terms dimension: lane-rotated copies of the additive cells while they still fit two workgroups per
    // CU (the Zipf-head terms otherwise serialise a wave's LDS atomics on one address)
    P.ncopies = 1;
    if (P.lds_mode && L_ORD && (!L_HIST || ESGPU_COPIES_HIST)) {
        for (uint32_t nc = kTermsCopies; nc > 1; nc /= 2) {
            const size_t b = collect_lds_bytes(LT, W, L_met, L_vcnt, L_ocnt, nc, pi);
            if (b <= kLdsPair) { P.ncopies = nc; lds = b; break; }
        }
    } else if (pi && P.lds_mode && L_HIST && pi_copies(L_met) > 1 && !wide) {
        // packed cells are 16 B instead of 28: a time-sorted window of 2 keys leaves room for lane-rotated copies of the
        // count + sum words (the Zipf-head terms of a wave otherwise queue on one LDS address)
        if (P.windowed && W > 2) {
            W = 2;
            P.W = W;
            lds = collect_lds_bytes(LT, W, L_met, L_vcnt, L_ocnt, 1, pi);
        }
        for (uint32_t nc = pi_copies(L_met); nc > 1; --nc) {
            const size_t b = collect_lds_bytes(LT, W, L_met, L_vcnt, L_ocnt, nc, pi);
            if (b <= kLdsPair) { P.ncopies = nc; lds = b; break; }
        }
    }
    if (!P.lds_mode && L_ORD && !L_HIST && L_met == 0 && !L_vcnt && L_ocnt == OCNT_NONE && !inner_missing &&
        (((uint64_t)pl.T + (1u << kPartShift) - 1) >> kPartShift) <= kPartMaxStaged) {
        p->last_bytes += bytes_per_doc * (uint64_t)s->max_doc + (d_accept ? ((uint64_t)s->max_doc + 7) / 8 : 0);
        count_width(p, pl, s, true, first_segment);
        // (the hot/cold form keeps statistics per ordinal column: not for a column derived per request)
        if (ESGPU_HOTCOLD && !pl.comp && collect_hotcold(p, pl, s, oc, d_accept, P.pred, P.npred, first_segment)) {
            if (first_segment) pl.zero_pending = false;  // (every counter stored, or never read: HcParams::overwrite)
            else zero_counts(p, pl);
            return 1;
        }
        zero_counts(p, pl);
        return collect_partitioned(p, pl, s, oc, d_accept, P.pred, P.npred) ? 1 : 0;
    }
    if (!inner_missing) count_width(p, pl, s, false, first_segment);
    const uint64_t span = (uint64_t)pl.interval * (uint64_t)W;
    P.fast32 =!P.kstart && !P.hord && pl.interval < (1ll << 32) && span < (1ull << 32);
    if (P.fast32) {
        const MagicU32 mg = make_magic((uint32_t)pl.interval);
        P.mg_m = mg.m; P.mg_s1 = mg.s1; P.mg_s2 = mg.s2;
    }
    const int hk = L_HIST ? (P.hord ? 3 : P.kstart ? 2 : 1) : 0;
    // packed cells under a filter: the clauses (and live docs) folded into one accept bitset before the collect
    const bool fold = pi && (P.npred > 0 || P.accept);
    // grids over dense compact columns without a filter -- histogram-only over the timestamp deltas (and a dense compact
    // metric), counting terms grids over 16-bit ordinals (and the timestamp deltas): raw-load kernels (VK bit 1024)
    const bool raw_hist = hk_launch == 1 && tcomp && !P.hv_f64 && !P.hv_present;
    P.raw_dense = raw_hist_on() && !pi && !P.accept && P.npred == 0 &&
                  ((!L_ORD && raw_hist && (L_met == 0 || (m32 && !P.mv_present))) ||
                   (L_ORD && L_met == 0 && P.ord16 && !P.ord_src && (hk_launch == 0 || raw_hist))) ? 1 : 0;
    // the integer runs' 16-bit deltas are read only by the raw-load kernels (no 32-bit copy was built for them)
    require(!(m32 && P.mv16 && !P.raw_dense), ESGPU_ERR_DEVICE, "internal: 16-bit metric deltas outside the raw-load kernels");
    // the key column: its block deltas where the launch is a raw-load kernel (packed cells over 16-bit columns, or the
    // dense unfiltered grids), else the 32-bit deltas
    if (t16) {
        P.hv16 = nullptr;
        P.hv16_base = nullptr;
        P.hv32 = nullptr;
        // 24-bit runs where most zone blocks hold one key (their timestamps are not read: ±1 min of displacement, north
        // star 1.28 -> 1.05 ms at 1B, r6ab); with wider displacement every block is multi-key, the kernel is bound by its
        // per-doc work rather than by the bytes, and the 32-bit deltas' simpler unpack measured faster (±1 h: 2.12
        // against 2.27 ms)
        const bool b24_fits = !t16->b16_hi.p || b24_mode() == 2 || (pl.interval > 0 && !P.kstart && hc->zspan < pl.interval);
        if (((pi && P.ord16 && P.mv16) || (P.raw_dense && hk_launch == 1)) && b24_fits) {
            P.hv16 = t16->b16.as<uint16_t>();
            P.hv16_base = t16->b16_base.as<int64_t>();
            const bool b24 = t16->b16_hi.p != nullptr;
            P.hv8 = b24 ? t16->b16_hi.as<uint8_t>() : (const uint8_t*)t16->b16.p;
            P.hv8_mask = b24 ? 0xFFFFFFFFu : 0u;
            P.hv8_and = b24 ? 0xFFu : 0u;
        } else {
            P.hv32 = ensure_d32(p->ctx, hc, s, p->stream);
            require(P.hv32 != nullptr, ESGPU_ERR_DEVICE, "out of device memory for the key column's deltas");
        }
    }
    // integer runs over time-sorted data (90 % of the blocks span less than one interval): one run per thread; roughly
    // time-ordered data alternates between neighbouring keys and keeps three
    P.runs1 = m32 && P.mv16 && hc && pl.interval > 0 && hc->zspan < pl.interval && runs1_on() ? 1 : 0;
    P.dot16 = P.runs1 && mc && (uint64_t)mc->vmax - (uint64_t)mc->vmin <= 46340 && dot16_on() ? 1 : 0;
    // ... and without runs1 (roughly time-ordered data), each doc straight into its key's LDS cells, in lane-rotated
    // copies while they fit two workgroups per CU (ESGPU_HDIRECT=0: the three integer runs, for A/B runs)
    P.hdirect = 0;
    if (m32 && P.mv16 && !L_ORD && L_HIST && L_met > 0 && P.lds_mode && !P.runs1 && hdirect_copies() > 0) {
        P.hdirect = 1;
        for (uint32_t nc = hdirect_copies(); nc > 1; nc /= 2) {
            const size_t b = collect_lds_bytes(LT, P.W, L_met, L_vcnt, L_ocnt, nc, pi);
            if (b <= kLdsPair) { P.ncopies = nc; lds = b; break; }
        }
    }
    // raw-load kernels over 32-bit timestamp deltas (block deltas did not apply: runs spanning 2^16 ms or more) skip the
    // single-key zone blocks' deltas where most blocks hold one key (90 % of the blocks span less than one interval:
    // roughly time-ordered data displaced by minutes); with wider displacement the skip's conditional load costs more
    // than it saves (north star at +-1 h: 2.06 -> 2.40 ms, r6c)
    P.ukey32 = L_HIST && !P.hv16 && P.hv32 && ((pi && P.ord16 && P.mv16) || P.raw_dense) && !P.kstart && hc &&
               pl.interval > 0 && hc->zspan < pl.interval ? 1 : 0;
    const int vk = (P.hv_f64 ? 1 : 0) | (P.mv_f64 ? 2 : 0) | (P.ord_src ? 8 : 0) | (P.ord16 ? 16 : 0) | (P.hv32 ? 32 : 0) |
                   (pi ? 64 : 0) | (m32 ? 128 : 0) | (P.mv16 ? 256 : 0) | (fold ? 512 : 0) | (P.raw_dense ? 1024 : 0) |
                   (P.runs1 ? 4096 : 0) | (P.hv16 ? 8192 : 0) | (P.ukey32 ? 16384 : 0) |
                   (P.ocnt_mode != OCNT_TERMS && P.ocnt_mode != OCNT_HIST ? 32768 : 0);
    const uint64_t occ_key = ((uint64_t)lds << 24) | ((uint64_t)wide << 23) | ((uint64_t)vk << 8) | ((uint64_t)L_met << 4) |
                             ((uint64_t)hk << 1) | (L_ORD ? 1 : 0);
    if (pl.occ_key != occ_key) {
        pl.occ = std::max(1, collect_occupancy(L_ORD, hk, L_met, lds, vk, wide));
        pl.occ_key = occ_key;
    }
    const uint32_t wg_per_cu = (uint32_t)pl.occ;
#ifndef ESGPU_WG_WAVES
#define ESGPU_WG_WAVES 8  // measured: 1-7 % faster than 1 on the collect shapes (8 and 16 alike, 32 slower)
#endif
    // ESGPU_WG_WAVES > 1: more, shorter workgroup ranges than resident slots (tail balancing vs per-workgroup setup)
    static const uint32_t wg_waves = [] {  // (ESGPU_WG_WAVES_ENV: A/B runs)
        const char* e = std::getenv("ESGPU_WG_WAVES_ENV");
        return (uint32_t)std::max(1, e && *e ? std::atoi(e) : ESGPU_WG_WAVES);
    }();
    const uint32_t target = (uint32_t)p->ctx->cus * wg_per_cu * wg_waves;
    const uint32_t bpw = (P.n_blocks + target - 1) / target;
#ifndef ESGPU_MIN_BPW
#define ESGPU_MIN_BPW 32  // measured at 125M docs: terms(host) 0.19 -> 0.10 ms, terms{stats} -16 %, config 5 -8 %
#endif
    // a workgroup flushes its LDS cells once; with a terms dimension that is ~T x W global atomics, so keep at least
    // ESGPU_MIN_BPW blocks per workgroup (fewer, longer ranges than the tail-balancing target) -- small segments
    // otherwise pay about one global atomic per 30 docs.  Histogram-only grids flush only the keys they touched.
    const uint32_t slots = (uint32_t)p->ctx->cus * wg_per_cu;
    // Histogram-only grids: at least ESGPU_HIST_MIN_BPW (16) blocks per workgroup too -- a workgroup's setup and run
    // flushes against one 8,192-doc block left config 2 at 100M docs at 0.119 ms; 8 blocks: 0.090 ms (r5, kbench)
    static const uint32_t hist_min_bpw = [] {
        const char* e = std::getenv("ESGPU_HIST_MIN_BPW");
        return (uint32_t)std::max(1, e && *e ? std::atoi(e) : 16);  // (16: config 2 at 100M 0.0799 -> 0.0754 ms, r6l)
    }();
    static const uint32_t ord_min_bpw = [] {  // (ESGPU_MIN_BPW_ENV: A/B runs)
        const char* e = std::getenv("ESGPU_MIN_BPW_ENV");
        return (uint32_t)std::max(1, e && *e ? std::atoi(e) : ESGPU_MIN_BPW);
    }();
    const uint32_t min_bpw = std::min<uint32_t>(L_ORD ? ord_min_bpw : hist_min_bpw, (P.n_blocks + slots - 1) / slots);
    P.blocks_per_wg = std::max(std::max(1u, bpw), min_bpw);
    if (pi && P.lds_mode && !pi_fits(P.blocks_per_wg)) {  // a packed field could overflow: the f64 cells instead
        pi = false;
        P.mv32 = nullptr;
        P.mv16 = nullptr;
        P.pk_shift = 0;
        P.ncopies = 1;
        goto relaunch;
    }
    if (pi || m32) bytes_per_doc -= P.mv16 ? 6 : 4;
    if (P.hv16) bytes_per_doc -= P.hv8_and ? 5 : 6;  // (+ one 8-byte base per run, below)
    else if (t16 && P.hv32) bytes_per_doc -= 4;
    uint32_t grid = (P.n_blocks + P.blocks_per_wg - 1) / P.blocks_per_wg;
    // dynamic chunk claiming: one resident wave of workgroups, each flushing its LDS cells once, taking chunks of
    // kGroup blocks until none are left (ESGPU_DYN=0/1 overrides the build default for A/B runs)
    P.claim = nullptr;
    P.n_chunks = (P.n_blocks + kGroupBlocks - 1) / kGroupBlocks;
    if (dyn_claim_on() && P.n_chunks > slots) {
        if (!p->d_claim.p) {
            p->d_claim.alloc(p->ctx, 16);
            HIPX(hipMemsetAsync(p->d_claim.p, 0, 16, p->stream));
        }
        P.claim = (unsigned int*)p->d_claim.p;
        grid = slots;
    }
    // the raw-load kernels over block deltas or 32-bit deltas read the timestamps of multi-key zone blocks only
    const bool raw_keys = L_HIST && (P.hv16 || P.ukey32);
    if ((P.lds_mode && P.windowed) || raw_keys) {
        P.zkey = (const int64_t*)p->s_zkey.ensure(p->ctx, (size_t)std::max(P.n_blocks, 1u) * 16);
        unsigned long long* ud = nullptr;
        if (raw_keys && p->zu_n < kZuSlots && (P.n_blocks + 255) / 256 <= kZuMaxWG) {
            ud = (unsigned long long*)p->s_zu.ensure(p->ctx, (size_t)kZuSlots * kZuMaxWG * 8) + (size_t)p->zu_n * kZuMaxWG;
            p->zu_g[p->zu_n] = (P.n_blocks + 255) / 256;  // (every workgroup writes its word: no zeroing)
        }
        launch_zone_keys(P, const_cast<int64_t*>(P.zkey), p->stream, ud);
        HIPX(hipGetLastError());
        if (ud) {
            // (read by esgpu_plan_last_collect_stats: no per-collect copy to the host on the request's path)
            p->zu_w[p->zu_n] = P.hv16 ? (P.hv8_and ? 3 : 2) : 4;  // timestamp bytes per doc the skipped blocks did not read
            ++p->zu_n;
        }
    }
    need_wide(false);
    HIPX(hipEventRecord(pl.e0, p->stream));
    if (fold && P.npred > 0) {  // (inside the timed region: part of the collect)
        uint64_t* bits = (uint64_t*)p->s_xbits.ensure(p->ctx, std::max<size_t>(s->n_pad / 64, 1) * 8);
        launch_filter_bits4(s->max_doc, P.accept, P.pred, P.npred, bits, p->stream);
        HIPX(hipGetLastError());
        P.accept = bits;
        P.npred = 0;
    }
    zero_counts(p, pl);
    launch_collect(P, L_ORD, L_HIST, L_met, wide, grid, lds, p->stream);
    HIPX(hipGetLastError());
    HIPX(hipEventRecord(pl.e1, p->stream));
    dd_fold();
    p->last_bytes += bytes_per_doc * (uint64_t)s->max_doc + (d_accept ? ((uint64_t)s->max_doc + 7) / 8 : 0) +
                     (P.hv16 ? (((uint64_t)s->max_doc + kB16Docs - 1) >> kB16Shift) * 8 : 0);
    p->last_path = P.lds_mode ? (P.windowed ? 2 : 1) : 0;
    return ret;
}

// raw-load histogram-only kernels (VK bit 1024; ESGPU_RAW_HIST=0: the converting loader, for A/B runs)
static bool raw_hist_on() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_RAW_HIST"); return !(e && *e == '0'); }();
    return on;
}
// 16-bit deltas of long columns spanning < 2^16 (the packed cells' metric, range predicates); ESGPU_D16=0: the 32-bit
// deltas instead (A/B runs)
static bool d16_on() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_D16"); return !(e && *e == '0'); }();
    return on;
}
// the compacted replay (ESGPU_REPLAY_COMPACT=0: one pass over the segments per batch of winners, for A/B runs)
static bool replay_compaction() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_REPLAY_COMPACT"); return !(e && *e == '0'); }();
    return on;
}
// integer run accumulators of histogram-only grids (VK bit 2048; ESGPU_INT_RUNS=0: the f64 runs, for A/B runs)
// per-doc LDS cells for histogram-only integer-run grids over roughly time-ordered data (CollectParams.hdirect):
// ESGPU_HDIRECT = the lane-rotated copies to try (0: off, the three integer runs).  Off: measured slower (config 2 at
// +-1 h jitter, 1B docs: 2.96 ms with the runs, 4.76 ms with 2 or 4 copies, r6p -- the wave's docs land on ~3 keys, and
// its f64 LDS atomics on those few addresses serialise)
static uint32_t hdirect_copies() {
    static const uint32_t n = [] { const char* e = std::getenv("ESGPU_HDIRECT"); return (uint32_t)(e && *e ? std::atoi(e) : 0); }();
    return n;
}
// packed run updates for single-key zone blocks (CollectParams.dot16; ESGPU_DOT16=0: the unpacked update, for A/B runs)
static bool dot16_on() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_DOT16"); return !(e && *e == '0'); }();
    return on;
}
static bool int_runs_on() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_INT_RUNS"); return !(e && *e == '0'); }();
    return on;
}
// one integer run per thread over time-sorted data (VK bit 4096; ESGPU_RUNS1=0: three, for A/B runs)
static bool runs1_on() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_RUNS1"); return !(e && *e == '0'); }();
    return on;
}
// block-delta timestamps on the raw-load kernels (ensure_b16; ESGPU_OPT_BLOCK_DELTAS)
static bool b16_on(const esgpu_ctx* c) { return c->opt_b16.load() != 0; }
// ESGPU_B24=0: a column with a run spanning 2^16 or more keeps the 32-bit deltas (no 24-bit runs; A/B); 2: the 24-bit
// runs whatever the zone span (A/B of the gate below)
static int b24_mode() {
    static const int m = [] {
        const char* e = std::getenv("ESGPU_B24");
        return e && e[0] == '0' ? 0 : e && e[0] == '2' ? 2 : 1;
    }();
    return m;
}
static bool b24_on() { return b24_mode() != 0; }
// ESGPU_DD=1: every metric grid takes the compensated flushes, exact data or not (tests of those paths on integer data)
static bool dd_forced() {
    static const bool on = [] { const char* e = std::getenv("ESGPU_DD"); return e && *e == '1'; }();
    return on;
}
static bool dyn_claim_on() {
    static const int dyn_claim = [] {
        const char* e = std::getenv("ESGPU_DYN");
        return e && *e ? (*e == '1' ? 1 : 0) : ESGPU_DYN_CLAIM;
    }();
    return dyn_claim != 0;
}
// packed integer metric cells (CollectParams.pk_shift; ESGPU_PI=0: the f64 cells, for A/B runs) and the lane-rotated
// copies of their count + sum words under a time window (ESGPU_PI_COPIES, 1 = none; default: 2 for avg leaves -- the
// Zipf-head terms' adds on one LDS word are their limit, terms{dh{avg}} 0.843 -> 0.790 ms at 1B, config 5 1.998 -> 1.928
// ms, r6f -- and 1 with min / max, where the hot term's register run takes those adds instead)
#ifndef ESGPU_PI_COPIES
#define ESGPU_PI_COPIES 0
#endif
static bool pi_cells(const esgpu_ctx* c) { return c->opt_pi.load() != 0; }
static uint32_t pi_copies(int met) {
    static const int v = [] {
        const char* e = std::getenv("ESGPU_PI_COPIES");
        return e && *e ? std::atoi(e) : ESGPU_PI_COPIES;
    }();
    return v > 0 ? (uint32_t)std::min(v, 4) : met == 1 ? 2u : 1u;
}

// Compact columns: a segment's ordinals and timestamps need fewer bits than their upload width -- Lucene
// stores them bit-packed / delta-coded for the same reason -- and the collect loop is HBM-bound, so the single-valued
// collect kernel reads 16-bit ordinals and 32-bit timestamp deltas when the segment's values fit (ESGPU_COMPACT=0: the
// upload-width columns, for A/B runs).  Built once per column under the context lock (plans on other threads may share
// the segment); an allocation over the HBM budget leaves the column as it is.
static bool compact_cols(const esgpu_ctx* c) { return c->opt_compact.load() != 0; }
static const uint16_t* ensure_ord16(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st) {
    DevColumn* m = const_cast<DevColumn*>(col);
    std::lock_guard<std::mutex> lk(c->mu);
    if (m->ord16.p && m->ord16_src == col->ords().p) return m->ord16.as<uint16_t>();
    if (m->ord16_src == col->ords().p) return nullptr;  // tried: over the budget
    m->ord16_src = col->ords().p;
    try {
        m->ord16.alloc(c, (size_t)s->n_pad * 2);
    } catch (const EsError&) {
        m->ord16.release();
        return nullptr;
    }
    launch_pack_ord16(col->ords().as<uint32_t>(), s->n_pad, m->ord16.as<uint16_t>(), st);
    HIPX(hipGetLastError());
    HIPX(hipStreamSynchronize(st));
    return m->ord16.as<uint16_t>();
}
// the 4 most frequent ordinals among 64 evenly spaced runs of 4,096 docs, most frequent first (cached with the ordinal
// buffer; kMissingOrd where fewer ordinals occur)
static void sampled_hot_ords(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, uint32_t (&out)[4]) {
    DevColumn* m = const_cast<DevColumn*>(col);
    std::lock_guard<std::mutex> lk(c->mu);
    auto give = [&] { for (int k = 0; k < 4; ++k) out[k] = m->hot_ord[k]; };
    if (m->hot_src == col->ords().p) return give();
    m->hot_src = col->ords().p;
    for (uint32_t& h : m->hot_ord) h = kMissingOrd;
    const uint64_t T = col->ord_count();
    if (!T || T > (1u << 24) || s->max_doc == 0) return give();
    const uint32_t run = std::min<uint32_t>(4096, s->max_doc), nrun = s->max_doc >= 64u * run ? 64u : 1u;
    std::vector<uint32_t> buf((size_t)run * nrun), hist(T, 0);
    for (uint32_t r = 0; r < nrun; ++r) {
        const uint64_t at = nrun == 1 ? 0 : (uint64_t)(s->max_doc - run) * r / (nrun - 1);
        HIPX(hipMemcpyAsync(buf.data() + (size_t)r * run, col->ords().as<uint32_t>() + at, (size_t)run * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIPX(hipStreamSynchronize(c->stream));
    for (uint32_t o : buf) if (o < T) ++hist[o];
    for (int k = 0; k < 4; ++k) {
        uint32_t best = 0;
        for (uint64_t o = 1; o < T; ++o) if (hist[o] > hist[best]) best = (uint32_t)o;
        if (!hist[best]) break;
        m->hot_ord[k] = best;
        hist[best] = 0;
    }
    give();
}

// the upload-width values of a long column whose wide buffer esgpu_segment_release_wide released, rebuilt from its compact
// deltas (value = vmin + delta: lossless for every present value) on the first kernel that reads them, and kept
// (the caller holds c->mu)
static const void* wide_i64_locked(esgpu_ctx* c, DevColumn* m, const esgpu_segment* s, hipStream_t st) {
    if (!m->wide_released.load(std::memory_order_relaxed) || m->values.p) return m->values.p;
    m->values.alloc(c, (size_t)s->n_pad * 8);
    if (m->d32.p) launch_expand_d32(m->d32.as<uint32_t>(), s->n_pad, m->vmin, m->values.as<int64_t>(), st);
    else if (m->b16.p) launch_expand_b16(m->b16.as<uint16_t>(), m->b16_hi.as<uint8_t>(), m->b16_base.as<int64_t>(), s->max_doc, s->n_pad,
                                         m->values.as<int64_t>(), st);
    else launch_expand_d16(m->d16.as<uint16_t>(), s->n_pad, m->vmin, m->values.as<int64_t>(), st);
    HIPX(hipGetLastError());
    HIPX(hipStreamSynchronize(st));
    m->wide_released.store(false, std::memory_order_release);  // (after values.p is set)
    return m->values.p;
}
static const void* wide_i64(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st) {
    if (!col) return nullptr;
    if (!col->wide_released.load(std::memory_order_acquire)) return col->values.p;
    std::lock_guard<std::mutex> lk(c->mu);
    return wide_i64_locked(c, const_cast<DevColumn*>(col), s, st);
}

static const uint32_t* ensure_d32(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st) {
    DevColumn* m = const_cast<DevColumn*>(col);
    std::lock_guard<std::mutex> lk(c->mu);
    if (m->d32_done) return m->d32.as<uint32_t>();
    m->d32_done = true;
    try {
        m->d32.alloc(c, (size_t)s->n_pad * 4);
    } catch (const EsError&) {
        m->d32.release();
        return nullptr;
    }
    launch_delta32((const int64_t*)wide_i64_locked(c, m, s, st), s->n_pad, col->vmin, m->d32.as<uint32_t>(), st);
    HIPX(hipGetLastError());
    HIPX(hipStreamSynchronize(st));
    return m->d32.as<uint32_t>();
}

// the block deltas of a dense single-valued long column (null when some run of kB16Docs docs spans 2^24 or more, or 2^16
// with ESGPU_B24=0: the column is not sorted enough; the verdict is cached)
static const DevColumn* ensure_b16(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st) {
    DevColumn* m = const_cast<DevColumn*>(col);
    std::lock_guard<std::mutex> lk(c->mu);
    if (m->b16_done) return m->b16.p ? m : nullptr;
    m->b16_done = true;
    if (col->type != ESGPU_COL_I64 || col->multi || col->present.p || s->n_pad % kB16Docs) return nullptr;
    const uint32_t runs = s->n_pad >> kB16Shift;
    const bool b24 = b24_on();
    try {
        m->b16.alloc(c, (size_t)s->n_pad * 2);
        m->b16_base.alloc(c, (size_t)std::max<uint32_t>(runs, 1) * 8);
        if (b24) m->b16_hi.alloc(c, (size_t)s->n_pad);
    } catch (const EsError&) {
        m->b16.release();
        m->b16_base.release();
        m->b16_hi.release();
        return nullptr;
    }
    DevBuf flag;
    flag.alloc(c, 4);
    HIPX(hipMemsetAsync(flag.p, 0, 4, st));
    launch_block_delta16((const int64_t*)wide_i64_locked(c, m, s, st), s->max_doc, s->n_pad, m->b16.as<uint16_t>(),
                         m->b16_hi.as<uint8_t>(), m->b16_base.as<int64_t>(), flag.as<unsigned int>(), st);
    HIPX(hipGetLastError());
    unsigned int bad = 0;
    HIPX(hipMemcpyAsync(&bad, flag.p, 4, hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));
    if ((bad & 2) || (bad && !b24)) {
        m->b16.release();
        m->b16_base.release();
        m->b16_hi.release();
        return nullptr;
    }
    if (!bad) m->b16_hi.release();  // (every run spans < 2^16: no plane)
    return m;
}

// the enc32 words of a dense single-valued long / double column for the floored HLL stream (null: over the budget; cached
// with the column like the compact columns, built once under the context lock)
static const uint32_t* ensure_hll_enc32(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st) {
    DevColumn* m = const_cast<DevColumn*>(col);
    std::lock_guard<std::mutex> lk(c->mu);
    if (m->hll32_done) return m->hll32.as<uint32_t>();
    m->hll32_done = true;
    if (col->type == ESGPU_COL_ORD_U32 || col->multi || col->present.p) return nullptr;  // longs, unsigned longs, doubles
    try {
        m->hll32.alloc(c, (size_t)s->n_pad * 4);
    } catch (const EsError&) {
        m->hll32.release();
        return nullptr;
    }
    const void* v = col->type == ESGPU_COL_F64 ? col->values.p : wide_i64_locked(c, m, s, st);
    launch_hll_enc32(v, col->type == ESGPU_COL_F64 ? HLL_F64 : HLL_I64, s->n_pad, m->hll32.as<uint32_t>(), st);
    HIPX(hipGetLastError());
    HIPX(hipStreamSynchronize(st));
    return m->hll32.as<uint32_t>();
}

static const uint16_t* ensure_d16(esgpu_ctx* c, const DevColumn* col, const esgpu_segment* s, hipStream_t st) {
    DevColumn* m = const_cast<DevColumn*>(col);
    std::lock_guard<std::mutex> lk(c->mu);
    if (m->d16_done) return m->d16.as<uint16_t>();
    m->d16_done = true;
    try {
        m->d16.alloc(c, (size_t)s->n_pad * 2);
    } catch (const EsError&) {
        m->d16.release();
        return nullptr;
    }
    launch_delta16((const int64_t*)wide_i64_locked(c, m, s, st), s->n_pad, col->vmin, m->d16.as<uint16_t>(), st);
    HIPX(hipGetLastError());
    HIPX(hipStreamSynchronize(st));
    return m->d16.as<uint16_t>();
}

static void ensure_ord_hash(esgpu_ctx* c, const DevColumn* col, hipStream_t st) {
    DevColumn* mcol = const_cast<DevColumn*>(col);
    std::lock_guard<std::mutex> lk(c->mu);  // plans on different threads may share the segment
    if (mcol->ord_hash.p) return;
    std::vector<uint64_t> h(std::max<uint64_t>(col->value_count, 1));
    for (uint64_t o = 0; o < col->value_count; ++o) {
        const std::string t = col->term(o);
        uint64_t h1, h2;
        murmur3_x64_128((const uint8_t*)t.data(), (int)t.size(), 0, &h1, &h2);
        h[o] = h1;
    }
    mcol->ord_hash.alloc(c, h.size() * 8);
    HIPX(hipMemcpyAsync(mcol->ord_hash.p, h.data(), h.size() * 8, hipMemcpyHostToDevice, st));
    HIPX(hipStreamSynchronize(st));
}

static size_t hll_snap_offset(uint32_t m) { return (32 + std::max<size_t>(m / 64, 1) + 15) & ~(size_t)15; }
// HLL phase 0 length in registers' worth of values (ESGPU_HLL_CUT0 env overrides the build default for A/B runs)
static uint32_t hll_cut0() {
    static const uint32_t c = [] {
        const char* e = std::getenv("ESGPU_HLL_CUT0");
        const int v = e && *e ? std::atoi(e) : 0;
        return v >= 1 && v <= 256 ? (uint32_t)v : (uint32_t)ESGPU_HLL_CUT0;
    }();
    return c;
}
static size_t hll_p0_offset(uint32_t m) { return (hll_snap_offset(m) + std::max<size_t>(m / 2, 16) + 15) & ~(size_t)15; }

static bool collect_hll(esgpu_plan* p, Pipeline& pl, const esgpu_segment* s, const uint64_t* d_accept) {
    const DevColumn* col = s->col(pl.metric_field.c_str());
    if (!col) return false;
    if (!pl.allocated) {
        const uint32_t m = 1u << pl.p;
        pl.regs.alloc(p->ctx, (size_t)m * 4);
        HIPX(hipMemsetAsync(pl.regs.p, 0, (size_t)m * 4, p->stream));
        pl.lc_threshold = (uint32_t)((float)(m / 4) * 0.75f);  // Hashset threshold (HyperLogLogPlusPlus.java:437-440)
        uint32_t cap = 1024;  // load factor <= 1/16 while the set is within the threshold
        while (cap < 16 * (pl.lc_threshold + 1)) cap <<= 1;
        pl.lc_mask = cap - 1;
        pl.lc_set.alloc(p->ctx, (size_t)cap * 4);
        HIPX(hipMemsetAsync(pl.lc_set.p, 0, (size_t)cap * 4, p->stream));
        pl.lc_first.alloc(p->ctx, (size_t)cap * 8);
        HIPX(hipMemsetAsync(pl.lc_first.p, 0xFF, (size_t)cap * 8, p->stream));
        // counters (32 bytes), then the group floors, then the packed register snapshot (16-byte aligned), then (p >= 12) the
        // partitioned phase 0's range counters (zero between requests) and entries
        const size_t p0_off = hll_p0_offset(m);
        const size_t p0_bytes = pl.p >= 12 ? 16 * (((size_t)hll_p0_ranges(m) * 4 + 15) / 16) +
                                                 (size_t)hll_p0_ranges(m) * hll_p0_cap(m, hll_cut0()) * 4 : 0;
        pl.lc_count.alloc(p->ctx, p0_off + p0_bytes);
        HIPX(hipMemsetAsync(pl.lc_count.p, 0, 32, p->stream));
        if (p0_bytes) HIPX(hipMemsetAsync(pl.lc_count.as<unsigned char>() + p0_off, 0, (size_t)hll_p0_ranges(m) * 4, p->stream));
        pl.allocated = true;
    }
    HllParams H{};
    H.n_docs = s->max_doc;
    H.p = pl.p;
    H.col = wide_i64(p->ctx, col, s, p->stream);
    H.present = col->present.as<uint64_t>();
    H.accept = d_accept;
    uint64_t bytes_per_doc = col->type == ESGPU_COL_ORD_U32 ? 4 : 8;
    if (col->type == ESGPU_COL_ORD_U32) {
        H.kind = HLL_ORD;
        ensure_ord_hash(p->ctx, col, p->stream);
        H.ord_hash = col->ord_hash.as<uint64_t>();
        H.n_ords = col->value_count;
        H.pos_ord = ordinals_collector(col->value_count, pl.p);
    } else {
        H.kind = col->type == ESGPU_COL_F64 ? HLL_F64 : HLL_I64;
    }
    set_preds(p, pl, s, H.pred, &H.npred, &bytes_per_doc, &H.accept);
    d_accept = H.accept;
    bool multi_pred = false;
    for (int k = 0; k < H.npred; ++k) multi_pred |= H.pred[k].offsets != nullptr;
    uint64_t bytes = bytes_per_doc * (uint64_t)s->max_doc;
    if (col->multi || multi_pred) {
        // MurmurHash3Values iterates every value of an accepted doc: fold accept + filters into a doc bitset, then
        // (multi-valued field) expand it to a per-value bitset and run the register passes over the value array
        bytes = column_bytes(col, s->max_doc) + (d_accept ? ((uint64_t)s->max_doc + 7) / 8 : 0);
        for (size_t k = 0; k < p->filter_fields.size(); ++k)
        if (applies(p, pl, k)) bytes += column_bytes(s->col(p->filter_fields[k].c_str()), s->max_doc);
        const uint64_t* doc_bits = d_accept;
        if (H.npred > 0) {
            uint64_t* b = (uint64_t*)p->s_fbits.ensure(p->ctx, std::max<size_t>(s->n_pad / 64, 1) * 8);
            launch_filter_bits(s->max_doc, d_accept, H.pred, H.npred, b, p->stream);
            HIPX(hipGetLastError());
            doc_bits = b;
            H.npred = 0;
        }
        H.accept = doc_bits;
        if (col->multi) {
            H.n_docs = (uint32_t)col->n_values;
            H.present = nullptr;
            if (doc_bits) {
                uint64_t* vb = (uint64_t*)p->s_vbits.ensure(p->ctx, (col->values.bytes / (col->type == ESGPU_COL_ORD_U32 ? 4 : 8) + 63) / 64 * 8);
                launch_expand_bits(s->max_doc, doc_bits, col->offsets.as<uint64_t>(), col->n_values, vb, p->stream);
                HIPX(hipGetLastError());
                H.accept = vb;
            }
        }
    }
    H.regs = pl.regs.as<unsigned int>();
    H.lc_set = pl.lc_set.as<unsigned int>();
    H.lc_count = pl.lc_count.as<unsigned int>();
    H.nonzero = pl.lc_count.as<unsigned int>() + 1;
    H.floor = pl.lc_count.as<unsigned int>() + 2;
    H.nz_part = pl.lc_count.as<unsigned int>() + 4;
    H.cut0 = hll_cut0();
    H.gfloor = pl.lc_count.as<unsigned char>() + 32;
    H.snap = pl.lc_count.as<unsigned char>() + hll_snap_offset(1u << pl.p);
    if (pl.p >= 12) {
        const uint32_t m = 1u << pl.p;
        H.p0_cnt = (unsigned int*)(pl.lc_count.as<unsigned char>() + hll_p0_offset(m));
        H.p0_buf = H.p0_cnt + 4 * (((size_t)hll_p0_ranges(m) * 4 + 15) / 16);
        H.p0_cap = hll_p0_cap(m, hll_cut0());
        // the register phases log their raises for a gather instead of raising each with a scattered global atomic
        // (which run at the memory side at ~20 G/s); ESGPU_HLL_LOG=0 keeps the atomics (A/B runs)
        static const int log_raises = [] { const char* e = std::getenv("ESGPU_HLL_LOG"); return e && *e == '0' ? 0 : 1; }();
        H.log_raises = log_raises;
        // the floored stream (one pass) when the request's values per register allow a floor F >= 4 (the
        // pass keeps 1/8 of the hashes or fewer); ESGPU_HLL_FS_MINF overrides the minimum (A/B runs), the context
        // option ESGPU_OPT_HLL_FLOOR turns it off or raises the floor (test leg for the tail pass)
        static const uint32_t fs_minf = [] {
            const char* e = std::getenv("ESGPU_HLL_FS_MINF");
            return e && *e ? std::max(2u, (uint32_t)std::atoi(e)) : 4u;
        }();
        // The floor is chosen from the distinct values the registers will have seen -- not the doc count: values
        // repeat (2^27 synthetic IPs over 1B docs: ~7 docs per value), and a floor picked from the docs would leave
        // registers below it for the tail pass.  The segment's distinct count comes from an earlier request's registers
        // (DevColumn::hll_distinct, a cached statistic like the compact columns); the first request on a segment takes
        // the register phases.  Over several segments the largest estimate is a lower bound of the union's.
        const int fs_mode = p->ctx->opt_hll_fs.load();
        const bool dense = !H.accept && H.npred == 0 && !H.present && !col->multi && H.kind != HLL_ORD;
        const double dseg = col->hll_distinct->load();
        const double dknown = dseg >= 0 ? std::max(dseg, pl.hll_dmax) : -1.0;
        // Measured at p = 18 (profiles/r4_hll_floor_ab.jsonl): the stream wins over the phases on a 125M-doc segment
        // (0.233 vs 0.290 ms) and loses on 1B (1.77 vs 1.60 ms) -- the phases' cost beyond streaming is a fixed ~0.1 ms
        // (their gathers and snapshot loads), the stream's grows with the entries it logs -- so it takes segments of up
        // to 1,024 values per register
        static const uint64_t fs_max_per_reg = [] {
            const char* e = std::getenv("ESGPU_HLL_FS_MAXPR");
            return e && *e ? (uint64_t)std::atoll(e) : (uint64_t)1024;
        }();
        const bool fs_size = (uint64_t)H.n_docs <= fs_max_per_reg * m;
        // a warm segment (a later segment of the request, the registers past the first cut) takes the one LDS phase
        // that remains: 0.098 ms + its gather at 125M docs against the stream's 0.135 ms + its gather
        // (profiles/r5/hll32); a raised floor (fs_mode > 1, the tail pass's test leg) keeps the stream
        const bool fs_warm_ok = pl.hll_seen < (uint64_t)m * H.cut0 || fs_mode > 1;
        uint32_t F = fs_mode && dense && fs_size && fs_warm_ok && dknown >= 0 ? hll_fs_floor((uint64_t)dknown, pl.p, fs_minf) : 0u;
        if (F && fs_mode > 1) F = std::min<uint32_t>(F + (uint32_t)fs_mode - 1, 64u - (uint32_t)pl.p);
        if (F) {
            const uint32_t cap = hll_fs_cap(H.n_docs, pl.p, F);
            const size_t need = (size_t)hll_p0_ranges(m) * cap * 4;
            if (pl.fs_buf.bytes < need) pl.fs_buf.alloc(p->ctx, need);
            H.fs_f = F;
            H.fs_cap = cap;
            H.fs_buf = pl.fs_buf.as<unsigned int>();
            H.unres = pl.lc_count.as<unsigned int>() + 6;
        }
        // the floored stream and the LDS register phases read 4 bytes per doc (HllParams.enc32); phase 0 of a request's
        // first 4 * 2^p values and the LC / tail pass still hash the values.  ESGPU_HLL_E32=0: the values (A/B runs)
        static const bool e32_on = [] { const char* e = std::getenv("ESGPU_HLL_E32"); return !(e && *e == '0'); }();
        if (e32_on && dense && pl.p <= kP2) H.enc32 = ensure_hll_enc32(p->ctx, col, s, p->stream);
        if (H.enc32) {
            const uint64_t n = s->max_doc, cold = F || pl.hll_seen >= (uint64_t)m * H.cut0 ? 0 : (uint64_t)m * H.cut0 - pl.hll_seen;
            bytes = 4 * n + 4 * std::min(n, cold);  // phase 0's values are 8 bytes
        }
    }
    H.lc_mask = pl.lc_mask;
    H.lc_threshold = pl.lc_threshold;
    H.lc_first = pl.lc_first.as<unsigned long long>();
    H.pos_base = (uint64_t)p->seg_seq << 40;
    H.seen = pl.hll_seen;
    H.snap_ok = pl.hll_seen > 0 && pl.hll_snap_ok;
    if (H.n_docs == 0) return false;
    if (pl.hll_seen == 0) {
        const bool dense1 = !H.accept && H.npred == 0 && !H.present && !col->multi && H.kind != HLL_ORD;
        pl.hll_d1 = dense1 ? col->hll_distinct : nullptr;
        pl.hll_nseg = 0;
        pl.hll_dmax = 0.0;
    }
    ++pl.hll_nseg;
    if (col->hll_distinct->load() >= 0) pl.hll_dmax = std::max(pl.hll_dmax, col->hll_distinct->load());
    pl.hll_seen += H.n_docs;
    pl.lc_dirty = true;
    HIPX(hipEventRecord(pl.e0, p->stream));
    pl.hll_snap_ok = launch_hll(H, (uint32_t)p->ctx->cus, p->stream);
    HIPX(hipGetLastError());
    if (pl.hll_nseg == 1 && pl.hll_d1 && pl.hll_d1->load() < 0 && pl.p >= 12) {
        const size_t rb = (size_t)4 << pl.p;
        if (pl.hll_r1.bytes < rb) pl.hll_r1.alloc(p->ctx, rb);
        HIPX(hipMemcpyAsync(pl.hll_r1.p, pl.regs.p, rb, hipMemcpyDeviceToDevice, p->stream));
        pl.hll_r1_pending = true;
    }
    HIPX(hipEventRecord(pl.e1, p->stream));
    p->last_bytes += bytes;
    p->last_path = 3;
    return true;
}

extern "C" int esgpu_plan_collect_segment(esgpu_plan* p, const esgpu_segment* s, const uint64_t* accept_bits) {
    return guarded([&] {
        require(p && s, ESGPU_ERR_INVALID, "null argument");
        require(!p->posted, ESGPU_ERR_STATE, "collect after postCollection");
        require(s->ctx == p->ctx, ESGPU_ERR_INVALID, "segment belongs to another device context");
        HIPX(hipSetDevice(p->ctx->device));
        hc_flush(p);  // (a second segment adds to the counts)
        const uint64_t* d_accept = nullptr;
        p->sparse_dead = false;
        if (accept_bits) {
            const size_t words = std::max<size_t>(s->n_pad / 64, 1);
            {  // how many docs the bitset clears, from up to 1,024 evenly spaced words (picks the hot/cold form)
                const size_t nw = ((size_t)s->max_doc + 63) / 64, step = std::max<size_t>(1, nw / 1024);
                uint64_t dead = 0, seen = 0;
                for (size_t w = 0; w + 1 < nw; w += step, seen += 64) dead += 64 - __builtin_popcountll(accept_bits[w]);
                p->sparse_dead = seen == 0 || dead * 10 <= seen;
            }
            void* a = p->s_accept.ensure(p->ctx, words * 8);
            HIPX(hipMemsetAsync(a, 0, words * 8, p->stream));
            HIPX(hipMemcpyAsync(a, accept_bits, ((size_t)s->max_doc + 63) / 64 * 8, hipMemcpyHostToDevice, p->stream));
            // the caller may reuse its buffer as soon as we return
            HIPX(hipStreamSynchronize(p->stream));
            d_accept = (const uint64_t*)a;
        }
        p->last_bytes = 0;
        p->last_ms = -1;
        p->zu_n = 0;
        bool deferred = false;
        for (Pipeline& pl : p->pipes) {
            if (pl.replay) { pl.timed = false; continue; }
            pl.timed = pl.kind == 1 ? collect_hll(p, pl, s, d_accept) : collect_grid(p, pl, s, d_accept);
            deferred |= pl.timed && pl.deferred;
        }
        if (deferred) {  // BestBucketsDeferringCollector: the segment (and its accept bits) kept for the replay at build
            esgpu_plan::DeferredSeg d{s, -1};
            if (d_accept) {
                const size_t bytes = std::max<size_t>(s->n_pad / 64, 1) * 8;
                size_t slot = 0;
                while (slot < p->d_daccept.size() && std::any_of(p->dsegs.begin(), p->dsegs.end(),
                                                                 [&](const esgpu_plan::DeferredSeg& x) { return x.accept == (int)slot; }))
                    ++slot;
                if (slot == p->d_daccept.size()) p->d_daccept.emplace_back();
                DevBuf& b = p->d_daccept[slot];
                if (b.bytes < bytes) b.alloc(p->ctx, bytes);
                HIPX(hipMemcpyAsync(b.p, d_accept, bytes, hipMemcpyDeviceToDevice, p->stream));
                d.accept = (int)slot;
            }
            pin_segment(s);
            p->dsegs.push_back(d);
        }
        p->collected = true;
        ++p->seg_seq;
        p->docs_seen += s->max_doc;
    });
}

extern "C" int esgpu_plan_shard_mergeable(const esgpu_plan* p, int32_t* mergeable) {
    return guarded([&] {
        require(p && mergeable, ESGPU_ERR_INVALID, "null argument");
        int32_t m = 1;
        for (const SpecNode& n : p->specs) if (n.s.type == ESGPU_AGG_TERMS) m = 0;
        *mergeable = m;
    });
}

extern "C" int esgpu_plan_deferred_segments(const esgpu_plan* p, int32_t* n) {
    return guarded([&] {
        require(p && n, ESGPU_ERR_INVALID, "null argument");
        *n = (int32_t)p->dsegs.size();
    });
}

extern "C" int esgpu_plan_last_collect_stats(const esgpu_plan* cp, double* kernel_ms, uint64_t* bytes, int32_t* path) {
    return guarded([&] {
        esgpu_plan* p = const_cast<esgpu_plan*>(cp);
        if (p->last_ms < 0) {  // resolve the HIP events of the last collect (synchronises with it)
            float total = 0;
            for (Pipeline& pl : p->pipes) {
                if (!pl.timed) continue;
                HIPX(hipEventSynchronize(pl.e1));
                float ms = 0;
                HIPX(hipEventElapsedTime(&ms, pl.e0, pl.e1));
                total += ms;
            }
            p->last_ms = total;
            if (p->zu_n) {  // the timestamps of single-key zone blocks were not read
                p->zu_host.ensure((size_t)kZuSlots * kZuMaxWG * 8);
                for (uint32_t i = 0; i < p->zu_n; ++i)
                    launch_copy_u64(p->s_zu.as<unsigned long long>() + (size_t)i * kZuMaxWG,
                                    (unsigned long long*)p->zu_host.dev() + (size_t)i * kZuMaxWG, p->zu_g[i], p->stream);
                HIPX(hipGetLastError());
                HIPX(hipStreamSynchronize(p->stream));
                uint64_t ud = 0;
                for (uint32_t i = 0; i < p->zu_n; ++i) {
                    uint64_t w = 0;
                    for (uint32_t g = 0; g < p->zu_g[i]; ++g) w += ((const uint64_t*)p->zu_host.p)[(size_t)i * kZuMaxWG + g];
                    ud += w * p->zu_w[i];
                }
                p->last_bytes -= std::min<uint64_t>(p->last_bytes, ud);
                p->zu_n = 0;
            }
        }
        if (kernel_ms) *kernel_ms = p->last_ms;
        if (bytes) *bytes = p->last_bytes;
        if (path) *path = p->last_path;
    });
}

// n u64 words from the device into pinned host memory (asynchronous): small transfers by a kernel writing through
// the buffer's device mapping, large ones by DMA
static void d2h_u64(esgpu_plan* p, PinnedBuf& dst, const void* src, size_t n) {
    dst.ensure(std::max<size_t>(n, 1) * 8);
    if (n == 0) return;
    if (n * 8 <= (4u << 20)) {
        launch_copy_u64((const unsigned long long*)src, (unsigned long long*)dst.dev(), n, p->stream);
        HIPX(hipGetLastError());
    } else {
        HIPX(hipMemcpyAsync(dst.p, src, n * 8, hipMemcpyDeviceToHost, p->stream));
    }
}
// build-phase stream waits, timed (esgpu_plan_last_build_stats: device wait vs host assembly)
static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void bsync(esgpu_plan* p) {
    const double t0 = now_ms();
    HIPX(hipStreamSynchronize(p->stream));
    p->b_wait += now_ms() - t0;
}
// ESGPU_TRACE_BUILD=1: per-phase marks of each build on stderr (diagnostics only)
static void bmark(esgpu_plan* p, const char* what) {
    if (p->b_trace) p->b_marks.emplace_back(what, now_ms());
}

extern "C" int esgpu_plan_last_build_stats(const esgpu_plan* p, double* total_ms, double* wait_ms) {
    return guarded([&] {
        require(p && total_ms && wait_ms, ESGPU_ERR_INVALID, "null argument");
        *total_ms = p->b_total;
        *wait_ms = p->b_wait;
    });
}

extern "C" int esgpu_plan_post_collection(esgpu_plan* p) {
    return guarded([&] {
        require(p != nullptr, ESGPU_ERR_INVALID, "null plan");
        HIPX(hipSetDevice(p->ctx->device));
        bsync(p);
        hc_check_err(p);
        for (Pipeline& pl : p->pipes) {
            if (pl.kind != 1 || !pl.allocated) continue;
            // [0] = distinct encoded hashes inserted (LC pass), [1] = non-zero registers (register pass)
            d2h_u64(p, p->h_tcnt, pl.lc_count.p, 1);
            const uint32_t* cnt = p->h_tcnt.as<uint32_t>();
            bsync(p);
            const uint32_t m = 1u << pl.p;
            pl.any_value = cnt[0] > 0 || cnt[1] > 0;
            pl.lc_dirty = cnt[0] > 0;  // the LC pass inserted nothing: its set is still clear
            if (cnt[1] <= pl.lc_threshold && cnt[0] <= pl.lc_threshold) {  // LINEAR_COUNTING: the distinct encoded hashes
                pl.hll_mode = 0;
                const size_t cap = (size_t)pl.lc_mask + 1;
                d2h_u64(p, p->h_dst[0], pl.lc_set.p, cap / 2);  // cap is a power of two >= 1024
                d2h_u64(p, p->h_dst[1], pl.lc_first.p, cap);
                const uint32_t* set = p->h_dst[0].as<uint32_t>();
                const uint64_t* first = p->h_dst[1].as<uint64_t>();
                bsync(p);
                std::vector<std::pair<uint64_t, uint32_t>> added;
                for (size_t i = 0; i < cap; ++i) if (set[i]) added.emplace_back(first[i], set[i]);
                pl.h_lc = hashset_values(added, pl.p);
                if (pl.hll_nseg == 1 && pl.hll_d1 && pl.hll_d1->load() < 0) pl.hll_d1->store((double)added.size());
            } else {  // HYPERLOGLOG
                pl.hll_mode = 1;
                // registers are u32 on the device (atomicMax); pack to the reference's byte array before the copy
                uint8_t* d8 = (uint8_t*)p->s_dst[0].ensure(p->ctx, m);
                launch_pack_u8(pl.regs.as<unsigned int>(), m, d8, p->stream);
                HIPX(hipGetLastError());
                d2h_u64(p, p->h_dst[0], d8, std::max<size_t>(m / 8, 1));  // m = 2^p >= 16
                const uint8_t* r = p->h_dst[0].as<uint8_t>();
                bsync(p);
                pl.h_regs.assign(r, r + m);
                if (pl.hll_nseg == 1 && pl.hll_d1 && pl.hll_d1->load() < 0) {
                    // the raw HyperLogLog estimate of the segment's distinct values (once per segment: the floored
                    // stream's floor on later requests)
                    double z = 0.0;
                    for (uint32_t i = 0; i < m; ++i) z += std::ldexp(1.0, -(int)r[i]);
                    const double alpha = 0.7213 / (1.0 + 1.079 / m);
                    pl.hll_d1->store(alpha * (double)m * (double)m / z);
                }
            }
            if (pl.hll_r1_pending) {  // a merged request: the first segment's own registers estimate its distinct values
                pl.hll_r1_pending = false;
                if (pl.hll_nseg > 1 && pl.hll_d1 && pl.hll_d1->load() < 0) {
                    d2h_u64(p, p->h_dst[0], pl.hll_r1.p, (size_t)m / 2);
                    const uint32_t* r = p->h_dst[0].as<uint32_t>();
                    bsync(p);
                    double z = 0.0;
                    for (uint32_t i = 0; i < m; ++i) z += std::ldexp(1.0, -(int)r[i]);
                    const double alpha = 0.7213 / (1.0 + 1.079 / m);
                    pl.hll_d1->store(alpha * (double)m * (double)m / z);
                }
            }
        }
        p->posted = true;
    });
}

// ---- build ----------------------------------------------------------------------------------------------------
static std::string plan_term(const esgpu_plan*, const Pipeline& pl, uint64_t ord) {
    return pl.tdict ? pl.tdict->term(ord) : std::to_string(ord);
}

// ---- result blocks (columnar InternalAggregations, see esgpu_results.hpp) ----
static void set_format(Block& r, const SpecNode& n) {
    r.time_zone = n.time_zone;
    r.value_format = n.s.value_format;
    r.format = n.format;
}

static Block metric_shell(const SpecNode& n) {
    Block r;
    r.type = n.s.type;
    r.name = n.name;
    r.sigma = n.s.sigma;
    set_format(r, n);
    return r;
}

// histogram spec with the given sub-aggregation prototypes (each an n == 1 empty instance)
static Block hist_shell(const esgpu_plan* p, int spec, const std::vector<Block>& protos) {
    const SpecNode& n = p->specs[spec];
    Block r;
    r.type = n.s.type;
    r.name = n.name;
    r.order = n.s.order;
    r.keyed = n.s.keyed;
    r.min_doc_count = n.s.min_doc_count;
    r.date_unit = n.s.type == ESGPU_AGG_DATE_HISTOGRAM ? n.s.date_unit : 0;
    r.interval = n.s.interval;
    r.offset = n.s.offset;
    r.tz_starts = n.tz_starts;
    r.tz_offs = n.tz_offs;
    set_format(r, n);
    r.boff.assign(1, 0);
    r.term_off.assign(1, 0);
    for (const Block& b : protos) r.subs.push_back(b.like());
    if (n.s.min_doc_count == 0) {  // EmptyBucketInfo
        r.has_empty_info = true;
        r.has_bmin = n.s.has_extended_bounds_min;
        r.has_bmax = n.s.has_extended_bounds_max;
        r.bmin = n.s.extended_bounds_min;
        r.bmax = n.s.extended_bounds_max;
        r.empty_subs = protos;
    }
    return r;
}

static Block terms_shell(const esgpu_plan* p, int spec, const std::vector<Block>& protos) {
    const SpecNode& n = p->specs[spec];
    Block r;
    r.type = ESGPU_AGG_TERMS;
    r.name = n.name;
    r.order = n.s.order;
    r.required_size = n.s.size;
    r.shard_size = n.s.shard_size;
    r.min_doc_count = n.s.min_doc_count;
    r.order_path = n.order_path;
    r.show_err = n.s.show_term_doc_count_error;
    r.boff.assign(1, 0);
    r.term_off.assign(1, 0);
    for (const Block& b : protos) r.subs.push_back(b.like());
    return r;
}

static void begin_instance(Block& b, int64_t other) {
    ++b.n;
    b.doc_count_error.push_back(0);
    b.other_doc_count.push_back(other);
}
static void end_instance(Block& b) { b.boff.push_back(b.key.size()); }
static void push_bucket(Block& b, int64_t key, std::string_view term, int64_t count) {
    b.key.push_back(key);
    b.term_pool += term;
    b.term_off.push_back(b.term_pool.size());
    b.bcount.push_back(count);
    b.berr.push_back(0);
}
static void push_bucket(Block& b, int64_t key, const std::string* term, int64_t count) {
    b.key.push_back(key);
    if (term) b.term_pool += *term;
    b.term_off.push_back(b.term_pool.size());
    b.bcount.push_back(count);
    b.berr.push_back(0);
}

// the cardinality sketches of the given bucket cells, gathered to the host in that order (rows index like HostCells)
static void gather_cards(esgpu_plan* p, Pipeline& pl, const std::vector<uint32_t>& cells) {
    if (pl.cards.empty()) return;
    hipStream_t st = p->stream;
    const uint32_t n = (uint32_t)cells.size();
    uint32_t* dcells = nullptr;
    if (n) {
        dcells = (uint32_t*)p->s_cells.ensure(p->ctx, (size_t)n * 4);
        HIPX(hipMemcpyAsync(dcells, cells.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    }
    for (CardState& cs : pl.cards) {
        cs.h_regs.resize((size_t)n * cs.m);
        cs.h_sets.resize((size_t)n * cs.cap);
        cs.h_cnt.resize(n);
        cs.h_nz.resize(n);
        cs.h_first.resize((size_t)n * cs.cap);
        if (!n) continue;
        struct { const DevBuf* src; uint32_t row; void* host; } parts[5] = {
            {&cs.regs, cs.m, cs.h_regs.data()}, {&cs.sets, cs.cap * 4, cs.h_sets.data()},
            {&cs.cnt, 4, cs.h_cnt.data()}, {&cs.nonzero, 4, cs.h_nz.data()}, {&cs.first, cs.cap * 8, cs.h_first.data()}};
        for (auto& pt : parts) {
            uint8_t* d = (uint8_t*)p->s_dst[5].ensure(p->ctx, (size_t)n * pt.row);
            launch_gather_bytes(dcells, n, pt.row, pt.src->as<uint8_t>(), d, st);
            HIPX(hipGetLastError());
            HIPX(hipMemcpyAsync(pt.host, d, (size_t)n * pt.row, hipMemcpyDeviceToHost, st));
            bsync(p);  // s_dst[5] is reused by the next part
        }
    }
}

// one instance of cardinality leaf `cs` from gathered row c (CardinalityAggregator.buildAggregation: a sketch whose
// cardinality is 0 is reported as "no counts"; HYPERLOGLOG iff more than threshold distinct encoded hashes)
static void append_card(const CardState& cs, size_t c, Block& r) {
    const uint32_t nz = cs.h_nz[c], cnt = cs.h_cnt[c];
    r.append_empty();
    if (nz == 0 && cnt == 0) return;
    const size_t i = r.n - 1;
    r.hll_present[i] = 1;
    if (nz > cs.thr || cnt > cs.thr) {
        r.hll_mode[i] = 1;
        r.regs[i].assign(cs.h_regs.begin() + c * cs.m, cs.h_regs.begin() + (c + 1) * cs.m);
    } else {
        r.hll_mode[i] = 0;
        std::vector<std::pair<uint64_t, uint32_t>> added;
        for (size_t k = 0; k < cs.cap; ++k) {
            const uint32_t e = cs.h_sets[c * cs.cap + k];
            if (e) added.emplace_back(cs.h_first[c * cs.cap + k], e);
        }
        r.lc[i] = hashset_values(added, cs.p);
        if (r.lc[i].empty()) r.hll_present[i] = 0;
    }
}

// the estimate of gathered row c's sketch (CardinalityAggregator.metric -> HyperLogLogPlusPlus.cardinality :270-282:
// LINEAR_COUNTING over the set's size, else the HLL++ estimate; a sketch that saw no value counts 0)
static int64_t card_estimate(const CardState& cs, size_t c) {
    const uint32_t nz = cs.h_nz[c], cnt = cs.h_cnt[c];
    if (nz == 0 && cnt == 0) return 0;
    if (nz > cs.thr || cnt > cs.thr) return hll_cardinality(cs.p, true, 1, cs.h_regs.data() + c * cs.m, 0);
    size_t n = 0;
    for (size_t k = 0; k < cs.cap; ++k) n += cs.h_sets[c * cs.cap + k] != 0;
    return n ? hll_cardinality(cs.p, true, 0, nullptr, n) : 0;
}

// the numeric partials of leaf j of a pipeline at host cell c: (count, sum, min, max, sum of squares)
struct MetricCell { int64_t count; double sum, min, max, sq; };
static MetricCell metric_cell(const esgpu_plan* p, const Pipeline& pl, int j, size_t c) {
    const int32_t type = p->specs[pl.metrics[j]].s.type;
    const HostCells& h = pl.hc;
    const uint64_t vc = pl.vcnt_mode ? h.vcnt[c] : h.cnt[c];
    MetricCell m{(int64_t)vc, 0.0, INFINITY, -INFINITY, 0.0};
    if (vc > 0) {
        m.sum = h.sum[c];
        if (pl.met >= 2 && type != ESGPU_AGG_AVG) {
            const uint64_t emn = h.mn[c], emx = h.mx[c];
            if (emn < kEncNegInf || emx > kEncPosInf) { m.min = NAN; m.max = NAN; }  // a NaN value was collected
            else { m.min = unsortable(emn); m.max = unsortable(emx); }
        }
        if (pl.met >= 3 && type == ESGPU_AGG_EXTENDED_STATS) m.sq = h.sq[c];
    }
    return m;
}

// one instance of leaf j (metric or cardinality) of a pipeline, from its host cell c
static void append_leaf(const esgpu_plan* p, const Pipeline& pl, int j, size_t c, Block& r) {
    if (p->specs[pl.metrics[j]].s.type == ESGPU_AGG_CARDINALITY) {
        size_t card = 0;
        for (int q = 0; q < j; ++q) card += p->specs[pl.metrics[q]].s.type == ESGPU_AGG_CARDINALITY;
        append_card(pl.cards[card], c, r);
        return;
    }
    const MetricCell m = metric_cell(p, pl, j, c);
    ++r.n;
    r.count.push_back(m.count);
    r.sum.push_back(m.sum);
    r.min.push_back(m.min);
    r.max.push_back(m.max);
    r.sumsq.push_back(m.sq);
}

// instances of leaf j of a pipeline for the given host cells, appended in order (columnar: one resize per array)
static void append_leaves(const esgpu_plan* p, const Pipeline& pl, int j, const std::vector<uint32_t>& cells, Block& r) {
    const int32_t type = p->specs[pl.metrics[j]].s.type;
    if (type == ESGPU_AGG_CARDINALITY) {
        for (uint32_t c : cells) append_leaf(p, pl, j, c, r);
        return;
    }
    const size_t n0 = r.count.size(), m = cells.size();
    r.n += m;
    r.count.resize(n0 + m);
    r.sum.resize(n0 + m);
    r.min.resize(n0 + m);
    r.max.resize(n0 + m);
    r.sumsq.resize(n0 + m);
    for (size_t i = 0; i < m; ++i) {
        const MetricCell mc = metric_cell(p, pl, j, cells[i]);
        r.count[n0 + i] = mc.count;
        r.sum[n0 + i] = mc.sum;
        r.min[n0 + i] = mc.min;
        r.max[n0 + i] = mc.max;
        r.sumsq[n0 + i] = mc.sq;
    }
}

static void reserve_buckets(Block& b, size_t buckets, size_t instances) {
    b.key.reserve(b.key.size() + buckets);
    b.bcount.reserve(b.bcount.size() + buckets);
    b.berr.reserve(b.berr.size() + buckets);
    b.term_off.reserve(b.term_off.size() + buckets);
    b.boff.reserve(b.boff.size() + instances);
    b.doc_count_error.reserve(b.doc_count_error.size() + instances);
    b.other_doc_count.reserve(b.other_doc_count.size() + instances);
}
static void reserve_leaves(Block& b, size_t n) {
    if (b.type == ESGPU_AGG_CARDINALITY) return;
    for (auto* v : {&b.sum, &b.min, &b.max, &b.sumsq}) v->reserve(v->size() + n);
    b.count.reserve(b.count.size() + n);
}

// histogram buckets of the given key slots (host cells `cells`, counts `counts[i]`), appended to the open instance
static void append_hist_buckets(const Pipeline& B, const std::vector<uint32_t>& slots, const std::vector<int64_t>& counts,
                                Block& r) {
    const size_t n0 = r.key.size(), m = slots.size();
    r.key.resize(n0 + m);
    r.bcount.resize(n0 + m);
    r.berr.resize(n0 + m, 0);
    r.term_off.resize(r.term_off.size() + m, r.term_pool.size());
    for (size_t i = 0; i < m; ++i) {
        r.key[n0 + i] = key_value(B, slots[i]);
        r.bcount[n0 + i] = counts[i];
    }
}

static Block leaf_proto(const esgpu_plan* p, int spec) {
    Block b = metric_shell(p->specs[spec]);
    if (p->specs[spec].s.type == ESGPU_AGG_CARDINALITY) b.precision = p->specs[spec].precision;
    b.append_empty();
    return b;
}

// device arrays of a pipeline's grid, in HostCells order (null: absent in its metric level)
static void grid_arrays(const Pipeline& pl, const void* src[6]) {
    src[0] = pl.g_cnt.p;
    src[1] = pl.vcnt_mode ? pl.g_vcnt.p : nullptr;
    src[2] = pl.met > 0 ? pl.g_sum.p : nullptr;
    src[3] = pl.met >= 2 ? pl.g_min.p : nullptr;
    src[4] = pl.met >= 2 ? pl.g_max.p : nullptr;
    src[5] = pl.met >= 3 ? pl.g_sq.p : nullptr;
}
static void point_cells(Pipeline& pl, const void* const src[6]) {
    auto h = [&](int a) { return src[a] ? pl.h_cells[a].p : nullptr; };
    pl.hc.cnt = (const unsigned long long*)h(0);
    pl.hc.vcnt = (const unsigned long long*)h(1);
    pl.hc.sum = (const double*)h(2);
    pl.hc.mn = (const unsigned long long*)h(3);
    pl.hc.mx = (const unsigned long long*)h(4);
    pl.hc.sq = (const double*)h(5);
}
// the rows [k][H] of the given ordinals, gathered on the GPU straight into the pipeline's pinned cells (asynchronous)
static void fetch_rows(esgpu_plan* p, Pipeline& pl, const uint32_t* drows, uint32_t k) {
    const void* src[6];
    grid_arrays(pl, src);
    GatherParams G{};
    G.rows = drows;
    G.k = k; G.H = pl.H; G.T = pl.T;
    G.cnt32 = pl.cnt32 ? 1 : 0;
    const size_t bytes = std::max<size_t>((size_t)k * pl.H, 1) * 8;
    for (int a = 0; a < 6; ++a) {
        if (!src[a]) continue;
        pl.h_cells[a].ensure(bytes);
        G.src[G.narrays] = (const unsigned long long*)src[a];
        G.dst[G.narrays] = (unsigned long long*)pl.h_cells[a].dev();
        G.narrays++;
    }
    if (k) {
        launch_gather_rows(G, p->stream);
        HIPX(hipGetLastError());
    }
    point_cells(pl, src);
}
// the whole grid into the pipeline's pinned cells (asynchronous)
static void fetch_grid(esgpu_plan* p, Pipeline& pl) {
    const void* src[6];
    grid_arrays(pl, src);
    const size_t cells = (size_t)pl.T * pl.H;
    if (pl.cnt32) {  // u32 counts widened on the device first
        unsigned long long* w = (unsigned long long*)p->s_tcnt.ensure(p->ctx, std::max<size_t>(cells, 1) * 8);
        launch_widen_u32(pl.g_cnt.as<unsigned int>(), cells, w, p->stream);
        HIPX(hipGetLastError());
        src[0] = w;
    }
    // the small arrays in one copy launch (config 2: five 721-cell arrays), large ones by DMA
    CopyList cl{};
    for (int a = 0; a < 6; ++a) {
        if (!src[a]) continue;
        if (cells * 8 > (4u << 20) || cells == 0) { d2h_u64(p, pl.h_cells[a], src[a], cells); continue; }
        pl.h_cells[a].ensure(cells * 8);
        cl.src[cl.count] = (const unsigned long long*)src[a];
        cl.dst[cl.count] = (unsigned long long*)pl.h_cells[a].dev();
        cl.n[cl.count] = cells;
        ++cl.count;
    }
    if (cl.count) {
        launch_copy_multi(cl, p->stream);
        HIPX(hipGetLastError());
    }
    point_cells(pl, src);
}

// GlobalOrdinalsStringTermsAggregator.buildAggregation candidate selection + PQ (:146-208); `value` is the
// InternalOrder.Aggregation metric of an ordinal (terms ordered by a sub-aggregation)
struct TermPick { uint32_t ord; int64_t count; };
template <class Value>
static std::vector<TermPick> select_terms(const esgpu_agg_spec& s, const unsigned long long* counts, uint32_t T, int64_t* other,
                                          Value&& value) {
    std::vector<TermPick> cands;
    int64_t oth = 0;
    for (uint32_t g = 0; g < T; ++g) {
        const int64_t c = (int64_t)counts[g];
        if (s.min_doc_count > 0 && c == 0) continue;
        oth += c;
        if (s.shard_min_doc_count <= c) cands.push_back({g, c});
    }
    const size_t size = (size_t)std::min<int64_t>((int64_t)T, (int64_t)s.shard_size);
    std::vector<double> vals;
    const bool agg = s.order == ESGPU_ORDER_AGG_ASC || s.order == ESGPU_ORDER_AGG_DESC;
    if (agg) {
        vals.resize(T);
        for (const TermPick& t : cands) vals[t.ord] = value(t.ord);
    }
    auto cmp = [&](const TermPick& a, const TermPick& b) {
        switch (s.order) {
            case ESGPU_ORDER_COUNT_DESC: if (a.count != b.count) return a.count > b.count; return a.ord < b.ord;
            case ESGPU_ORDER_COUNT_ASC: if (a.count != b.count) return a.count < b.count; return a.ord < b.ord;
            case ESGPU_ORDER_TERM_DESC: return a.ord > b.ord;
            case ESGPU_ORDER_AGG_ASC:
            case ESGPU_ORDER_AGG_DESC: {  // CompoundOrder(Aggregation, TERM_ASC) over the sub-aggregator's metric(bucketOrd)
                const int c = compare_discard_nan(vals[a.ord], vals[b.ord], s.order == ESGPU_ORDER_AGG_ASC);
                if (c != 0) return c < 0;
                return a.ord < b.ord;
            }
            default: return a.ord < b.ord;
        }
    };
    if (cands.size() > size) {
        std::partial_sort(cands.begin(), cands.begin() + size, cands.end(), cmp);
        cands.resize(size);
    } else {
        std::sort(cands.begin(), cands.end(), cmp);
    }
    for (auto& t : cands) oth -= t.count;
    *other = oth;
    return cands;
}

// Three bucket levels: one instance of the deepest aggregation Y of bucket child `kid` from its composite pipelines'
// host cells.  Terms: its candidates are the cells base + y * stride for every Y ordinal y (the same selection and
// comparators as a two-level terms, GlobalOrdinalsStringTermsAggregator.buildAggregation); histogram: the cells base + s
// for every key slot s, non-empty ones ascending (HistogramAggregator.buildAggregation).
static double order_value(const esgpu_plan* p, const SpecNode& t, const Pipeline& pl, int leaf, size_t c);
static void emit_deep(const esgpu_plan* p, const ChildSrc& kid, size_t base, size_t stride, Block& yb) {
    const Pipeline& C0 = p->pipes[kid.dpipes[0]];
    if (!C0.allocated) { yb.append_empty(); return; }
    const SpecNode& tn = p->specs[kid.deep];
    if (tn.s.type != ESGPU_AGG_TERMS) {
        begin_instance(yb, 0);
        std::vector<uint32_t> slots, cells;
        std::vector<int64_t> counts;
        for (uint32_t s2 = 0; s2 < C0.H; ++s2) {
            const unsigned long long c = C0.hc.cnt[base + s2];
            if (c == 0) continue;
            slots.push_back(s2);
            cells.push_back((uint32_t)(base + s2));
            counts.push_back((int64_t)c);
        }
        append_hist_buckets(C0, slots, counts, yb);
        for (size_t gj = 0; gj < kid.dgrand.size(); ++gj)
            append_leaves(p, p->pipes[kid.dgrand[gj].pipe], kid.dgrand[gj].leaf, cells, yb.subs[gj]);
        end_instance(yb);
        return;
    }
    const uint32_t Ty = (uint32_t)C0.vcB;
    std::vector<unsigned long long> cnt(std::max<uint32_t>(Ty, 1), 0);
    for (uint32_t y = 0; y < Ty; ++y) cnt[y] = C0.hc.cnt[base + (size_t)y * stride];
    LeafRef ordr;
    if (tn.s.order == ESGPU_ORDER_AGG_ASC || tn.s.order == ESGPU_ORDER_AGG_DESC)
        for (size_t gj = 0; gj < tn.children.size(); ++gj) if (tn.children[gj] == tn.order_child) ordr = kid.dgrand[gj];
    int64_t other = 0;
    const std::vector<TermPick> top = select_terms(tn.s, cnt.data(), Ty, &other, [&](uint32_t ord) {
        return order_value(p, tn, p->pipes[ordr.pipe], ordr.leaf, base + (size_t)ord * stride);
    });
    begin_instance(yb, other);
    std::string scratch;
    for (const TermPick& tp : top) {
        push_bucket(yb, tp.ord, C0.tdictB->view(tp.ord, scratch), tp.count);
        if (tp.count == 0) { for (Block& sb : yb.subs) sb.append_empty(); continue; }
        for (size_t gj = 0; gj < kid.dgrand.size(); ++gj)
            append_leaf(p, p->pipes[kid.dgrand[gj].pipe], kid.dgrand[gj].leaf, base + (size_t)tp.ord * stride, yb.subs[gj]);
    }
    end_instance(yb);
}

// one InternalFilter instance of filter child `kid` at host cell c of its outer-level pipelines
// (FilterAggregator.buildAggregation: bucketDocCount(owningBucketOrdinal), bucketAggregations(owningBucketOrdinal))
static void append_filter(const esgpu_plan* p, const ChildSrc& kid, size_t c, Block& sub) {
    const Pipeline& F0 = p->pipes[kid.pipes[0]];
    ++sub.n;
    sub.count.push_back(F0.allocated ? (int64_t)F0.hc.cnt[c] : 0);
    for (size_t gj = 0; gj < kid.grand.size(); ++gj) {
        const Pipeline& L = p->pipes[kid.grand[gj].pipe];
        if (!L.allocated) sub.subs[gj].append_empty();
        else append_leaf(p, L, kid.grand[gj].leaf, c, sub.subs[gj]);
    }
}

// prototypes (n == 1 empty instances) of a bucket aggregation's children, in request order
static std::vector<Block> child_protos(const esgpu_plan* p, const Group& g) {
    std::vector<Block> out;
    for (const ChildSrc& k : g.kids) {
        if (k.filter) {  // InternalFilter: doc_count + its metric children
            Block f;
            f.type = ESGPU_AGG_FILTER;
            f.name = p->specs[k.spec].name;
            for (int gc : p->specs[k.spec].children) f.subs.push_back(leaf_proto(p, gc));
            f.append_empty();
            out.push_back(std::move(f));
            continue;
        }
        if (!k.bucket) { out.push_back(leaf_proto(p, k.spec)); continue; }
        std::vector<Block> grand;
        for (int gc : p->specs[k.spec].children) {
            if (gc != k.deep) { grand.push_back(leaf_proto(p, gc)); continue; }
            std::vector<Block> yl;  // the third level's prototype: its (empty) instance over its own leaf prototypes
            for (int gy : p->specs[gc].children) yl.push_back(leaf_proto(p, gy));
            Block yb = p->specs[gc].s.type == ESGPU_AGG_TERMS ? terms_shell(p, gc, yl) : hist_shell(p, gc, yl);
            yb.append_empty();
            grand.push_back(std::move(yb));
        }
        Block in = p->specs[k.spec].s.type == ESGPU_AGG_TERMS ? terms_shell(p, k.spec, grand) : hist_shell(p, k.spec, grand);
        in.append_empty();
        out.push_back(std::move(in));
    }
    return out;
}

// the InternalOrder.Aggregation value of terms spec `t` for ordinal cell c of the pipeline holding its order child
static double order_value(const esgpu_plan* p, const SpecNode& t, const Pipeline& pl, int leaf, size_t c) {
    const SpecNode& mn = p->specs[t.order_child];
    if (mn.s.type == ESGPU_AGG_CARDINALITY) {
        // CardinalityAggregator.metric(bucketOrd) = counts.cardinality(bucketOrd): the estimate of the cell's sketch,
        // gathered to the host beside the cells (the same host-cell layout at every nesting level)
        for (const CardState& cs : pl.cards)
            if (cs.spec == t.order_child) return (double)card_estimate(cs, c);
        return 0.0;
    }
    const MetricCell m = metric_cell(p, pl, leaf, c);
    double v = NAN;
    metric_value(mn.s.type, t.order_key, m.count, m.sum, m.min, m.max, m.sq, mn.s.sigma, &v);
    return v;
}

static Block build_metric_root(esgpu_plan* p, const Group& g) {
    Pipeline& pl = p->pipes[g.pipes[0]];
    Block r = leaf_proto(p, g.root).like();
    if (!pl.allocated) { r.append_empty(); return r; }
    fetch_grid(p, pl);
    bsync(p);
    append_leaf(p, pl, 0, 0, r);
    return r;
}

// The replayed inner terms of a deferred terms-under-terms child: per outer winner i, the selected inner terms, the
// instance's other-doc count, and each pick's host cell in the replay pipelines (append_leaf / order_value index)
struct ReplaySel {
    std::vector<std::vector<TermPick>> picks;
    std::vector<int64_t> other;
    std::vector<std::vector<size_t>> cell;
};

// TermsAggregator breadth_first (A/bucket/terms/TermsAggregator.java:161 shouldDefer; BestBucketsDeferringCollector
// .prepareSelectedBuckets :127-166, replayed from GlobalOrdinalsStringTermsAggregator.buildAggregation :195-196): the
// child's collectors run again over the retained segments, each doc counted in its outer bucket's winner slot when that
// bucket survived (the replay grid [slot][inner ordinal], rows padded to replay_stride); then the inner terms of every
// winner are selected -- on the GPU per row (count / term orders) or from the fetched rows on the host (metric orders,
// rows of at most 65,536 terms), with the same comparators as the dense grid's select_terms
// One replay pass: outer winners [b0, b0 + kb) take slots 0 .. kb - 1 and the replay pipelines collect every retained
// segment into their [slot][inner ordinal] grid; false when no retained segment had both fields
static bool replay_pass(esgpu_plan* p, const ChildSrc& kid, const std::vector<TermPick>& top, uint32_t b0, uint32_t kb,
                        uint64_t T_outer) {
    hipStream_t st = p->stream;
    std::vector<uint32_t> map(std::max<uint64_t>(T_outer, 1), kMissingOrd);
    for (uint32_t i = 0; i < kb; ++i) if (top[b0 + i].ord < map.size()) map[top[b0 + i].ord] = i;
    uint32_t* dmap = (uint32_t*)p->s_slotmap.ensure(p->ctx, map.size() * 4);
    HIPX(hipMemcpyAsync(dmap, map.data(), map.size() * 4, hipMemcpyHostToDevice, st));
    p->slot_map = dmap;
    p->slot_map_n = (uint32_t)map.size();
    p->slot_k = kb;
    bool any = false;
    try {
        for (int pi : kid.rpipes) {
            Pipeline& R = p->pipes[pi];
            if (b0 > 0 && R.allocated) {  // a later pass over the same buffers: the grid starts from zero again
                R.fresh = true;
                HIPX(hipMemsetAsync(R.g_cnt.p, 0, R.g_cnt.bytes, st));
            }
            R.fresh = true;
        }
        for (const esgpu_plan::DeferredSeg& d : p->dsegs) {
            const uint64_t* acc = d.accept >= 0 ? p->d_daccept[d.accept].as<uint64_t>() : nullptr;
            for (size_t j = 0; j < kid.rpipes.size(); ++j) {
                const bool done = collect_grid(p, p->pipes[kid.rpipes[j]], d.s, acc);
                if (j == 0) any |= done;
            }
        }
        HIPX(hipStreamSynchronize(st));  // `map` is read by the copy above
    } catch (...) {
        p->slot_map = nullptr;
        throw;
    }
    p->slot_map = nullptr;
    return any;
}

// The compacted replay of a count-only child in batches of wb winners (ReplayCompactParams): one pass over every retained
// segment writes each surviving doc's replay ordinal into its batch's region -- capacity from the winners' outer doc
// counts, which bound the docs that can land there -- so each batch is counted from its region alone instead of
// re-reading both ordinal columns of every segment per batch.  False (nothing changed) when it does not apply: more
// batches than the kernel stages, a region budget over the context's HBM, or an append that did not fit.
struct ReplayRegions {
    std::vector<uint32_t> n;      // elements per batch
    std::vector<uint64_t> off;    // first element of each batch's region
    uint64_t vcB = 0;
    bool any = false;             // some retained segment had both fields
    std::shared_ptr<const TermDict> da, db;
};
static bool replay_compact(esgpu_plan* p, const ChildSrc& kid, const std::vector<TermPick>& top, uint32_t wb, uint64_t T_outer,
                           ReplayRegions& rr) {
    hipStream_t st = p->stream;
    Pipeline& R0 = p->pipes[kid.rpipes[0]];
    const uint32_t k = (uint32_t)top.size();
    const uint32_t nbatch = (k + wb - 1) / wb;
    if (nbatch > kReplayMaxBatches || wb > (1u << kReplayBatchShift) || dyn_claim_on()) return false;
    // the inner dictionary: the first retained segment with both fields (every later one must number alike)
    for (const esgpu_plan::DeferredSeg& d : p->dsegs) {
        const DevColumn* a = d.s->col(R0.ord_field.c_str());
        const DevColumn* b = d.s->col(R0.ord_field2.c_str());
        if (!a || !b) continue;
        if (!rr.db) { rr.da = a->ord_dict(); rr.db = b->ord_dict(); rr.vcB = b->ord_count(); }
        else require(same_dict(a->ord_dict(), rr.da) && same_dict(b->ord_dict(), rr.db), ESGPU_ERR_INVALID,
                     "segments number the terms of [" + R0.ord_field + "] or [" + R0.ord_field2 + "] differently: build an "
                     "ordinal map (esgpu_ordinal_map_build) over the reader's segments first");
        require(!a->multi && !b->multi, ESGPU_ERR_UNSUPPORTED, "a breadth-first replay over multi-valued terms fields runs on the CPU path");
        rr.any = true;
    }
    rr.n.assign(nbatch, 0);
    rr.off.assign(nbatch + 1, 0);
    if (!rr.any) return true;
    const uint64_t stride = replay_stride(rr.vcB);
    if ((uint64_t)wb * stride >= 0xFFFFFFFFull) return false;
    std::vector<uint32_t> cap(nbatch);
    for (uint32_t bi = 0; bi < nbatch; ++bi) {
        uint64_t c = 0;
        for (uint32_t w = bi * wb; w < std::min(k, (bi + 1) * wb); ++w) {
            if (top[w].count < 0) return false;  // a count not gathered yet (GPU top-k in a term order): no capacity known
            c += (uint64_t)top[w].count;
        }
        if (c >= 0x7FFFFFFFull) return false;
        cap[bi] = (uint32_t)c;
        rr.off[bi + 1] = rr.off[bi] + ((c + kBlockDocs - 1) / kBlockDocs + 1) * kBlockDocs;  // + one block: the loads past n
    }
    uint32_t* region;
    try {
        region = (uint32_t*)p->s_rregion.ensure(p->ctx, rr.off[nbatch] * 4);
    } catch (const EsError& e) {
        if (e.code != ESGPU_ERR_OOM) throw;
        return false;
    }
    // outer ordinal -> its winner's batch and index in the batch (ReplayCompactParams.slot_map)
    std::vector<uint32_t> map(std::max<uint64_t>(T_outer, 1), kMissingOrd);
    for (uint32_t w = 0; w < k; ++w)
        if (top[w].ord < map.size()) map[top[w].ord] = (w / wb) << kReplayBatchShift | (w % wb);
    // device metadata: [slot map][region offsets (u64)][capacities][fills, one cache line each][overflow]
    const size_t moff = ((map.size() * 4 + 15) & ~(size_t)15), coff = moff + (size_t)nbatch * 8,
                 foff = (coff + (size_t)nbatch * 4 + 255) & ~(size_t)255, fbytes = (size_t)nbatch * kReplayFillStride * 4;
    unsigned char* meta = (unsigned char*)p->s_rmeta.ensure(p->ctx, foff + fbytes + 16);
    HIPX(hipMemcpyAsync(meta, map.data(), map.size() * 4, hipMemcpyHostToDevice, st));
    HIPX(hipMemcpyAsync(meta + moff, rr.off.data(), (size_t)nbatch * 8, hipMemcpyHostToDevice, st));
    HIPX(hipMemcpyAsync(meta + coff, cap.data(), (size_t)nbatch * 4, hipMemcpyHostToDevice, st));
    HIPX(hipMemsetAsync(meta + foff, 0, fbytes + 16, st));
    for (const esgpu_plan::DeferredSeg& d : p->dsegs) {
        const DevColumn* a = d.s->col(R0.ord_field.c_str());
        const DevColumn* b = d.s->col(R0.ord_field2.c_str());
        if (!a || !b) continue;
        ReplayCompactParams C{};
        C.n_docs = d.s->max_doc;
        C.a = a->ords().as<uint32_t>();
        // the outer ordinals' 16-bit copy when the request's collect built it (2 B per doc instead of 4)
        if (a->ord16.p && a->ord16_src == a->ords().p) C.a16 = a->ord16.as<uint16_t>();
        C.b = b->ords().as<uint32_t>();
        C.slot_map = (const uint32_t*)meta;
        C.slot_map_n = (uint32_t)map.size();
        C.vcB = (uint32_t)std::min<uint64_t>(rr.vcB, 0xFFFFFFFFull);
        C.wb = wb;
        C.stride = (uint32_t)stride;
        C.nbatch = nbatch;
        const uint64_t* acc = d.accept >= 0 ? p->d_daccept[d.accept].as<uint64_t>() : nullptr;
        uint64_t bytes = 0;
        set_preds(p, R0, d.s, C.pred, &C.npred, &bytes, &acc);
        C.accept = acc;
        C.out = region;
        C.region = (const uint64_t*)(meta + moff);
        C.cap = (const uint32_t*)(meta + coff);
        C.fill = (uint32_t*)(meta + foff);
        C.overflow = (uint32_t*)(meta + foff + fbytes);
        launch_replay_compact(C, st);
        HIPX(hipGetLastError());
    }
    uint32_t* hf = (uint32_t*)p->h_rfill.ensure(fbytes + 16);
    HIPX(hipMemcpyAsync(hf, meta + foff, fbytes + 16, hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));  // also keeps `map` / `cap` alive for the copies
    if (hf[(size_t)nbatch * kReplayFillStride] != 0) return false;  // an append past its capacity: the per-pass replay instead
    for (uint32_t bi = 0; bi < nbatch; ++bi) rr.n[bi] = hf[(size_t)bi * kReplayFillStride];
    return true;
}

// The replay of a count-only child in count order over the inner field's hot terms (ReplayHotParams): with one retained
// segment, the inner field's statistics (HcStats: hot slots most frequent first, each slot's count, the largest cold
// count) bound every term outside the first Hh hot slots by the count of slot Hh (or the largest cold count).  One pass
// counts each winner's docs on those Hh slots (in LDS) and its docs without an inner term; per winner the GPU top-k
// (K3) over its Hh slots, mapped to ordinals, gives the winners' inner terms whenever its k-th count is above that bound
// -- no other term can reach it (ties go to the smaller ordinal, which may be outside: strictly above) -- and the other
// doc count is the winner's doc count less its missing-term docs and its picks.  False when it does not apply or some
// winner is not settled: the full replay then runs (ESGPU_REPLAY_HOT=0: always).
static bool replay_hot(esgpu_plan* p, const ChildSrc& kid, const std::vector<TermPick>& top, uint64_t T_outer, ReplaySel& rs) {
    static const bool on = [] { const char* e = std::getenv("ESGPU_REPLAY_HOT"); return !(e && *e == '0'); }();
    if (!on || kid.rpipes.size() != 1 || !kid.rgrand.empty() || p->dsegs.size() != 1) return false;
    const SpecNode& tn2 = p->specs[kid.spec];
    Pipeline& R0 = p->pipes[kid.rpipes[0]];
    if (tn2.s.order != ESGPU_ORDER_COUNT_DESC || R0.met != 0 || !R0.cards.empty() || tn2.s.shard_size < 1) return false;
    const uint32_t k = (uint32_t)top.size();
    if (k == 0 || k >= 255) return false;
    for (const TermPick& tp : top) if (tp.count < 0) return false;
    esgpu_ctx* c = p->ctx;
    hipStream_t st = p->stream;
    const esgpu_plan::DeferredSeg& d = p->dsegs[0];
    const DevColumn* a = d.s->col(R0.ord_field.c_str());
    const DevColumn* b = d.s->col(R0.ord_field2.c_str());
    if (!a || !b || a->multi || b->multi || T_outer > 65535 || a->ord_count() > 65535 || b->ord_count() <= 65536) return false;
    const uint16_t* a16 = ensure_ord16(c, a, d.s, st);
    if (!a16) return false;
    std::shared_ptr<const HcStats> hs = ensure_hc_stats(c, b, d.s, (uint32_t)b->ord_count(), st);
    if (!hs || !hs->hot_n || !hs->d_hot16.p || hs->hot_cnt.size() != hs->hot_n) return false;
    const uint32_t kk = (uint32_t)std::min<uint64_t>(b->ord_count(), (uint64_t)tn2.s.shard_size);
    // the hot slots per winner that fit LDS beside the outer ordinal -> winner map
    const size_t budget = 156 * 1024;
    const uint32_t nmap = (uint32_t)std::max<uint64_t>(T_outer, 1);
    uint32_t Hh = std::min<uint32_t>(hs->hot_n, 65534);
    while (Hh > 0 && replay_hot_lds(k, Hh, nmap) > budget) Hh = Hh > 64 ? Hh - 64 : 0;
    if (Hh < kk || kk > kTopkMax) return false;
    const uint64_t bound = Hh < hs->hot_n ? (uint64_t)hs->hot_cnt[Hh] : hs->max_cold;
    // the request's clauses (as the collect applied them) and live docs, folded into one bitset
    const uint64_t* acc = d.accept >= 0 ? p->d_daccept[d.accept].as<uint64_t>() : nullptr;
    PredDev pred[4];
    int32_t npred = 0;
    uint64_t bytes = 0;
    set_preds(p, R0, d.s, pred, &npred, &bytes, &acc);
    if (npred > 0) {
        uint64_t* xb = (uint64_t*)p->s_hbits.ensure(c, std::max<size_t>(d.s->n_pad / 64, 1) * 8);
        launch_filter_bits4(d.s->max_doc, acc, pred, npred, xb, st);
        HIPX(hipGetLastError());
        acc = xb;
    }
    std::vector<uint8_t> map(nmap, 0xFF);
    for (uint32_t w = 0; w < k; ++w) if (top[w].ord < nmap) map[top[w].ord] = (uint8_t)w;
    ReplayHotParams Q{};
    Q.n_docs = d.s->max_doc;
    Q.n_blocks = d.s->n_pad / kBlockDocs;
    Q.G = std::max(1u, std::min<uint32_t>((uint32_t)c->cus, Q.n_blocks));
    Q.blocks_per_wg = (Q.n_blocks + Q.G - 1) / Q.G;
    Q.G = std::max(1u, (Q.n_blocks + Q.blocks_per_wg - 1) / Q.blocks_per_wg);
    Q.a16 = a16;
    Q.hot16 = hs->d_hot16.as<uint16_t>();
    Q.slot_map_n = nmap;
    Q.accept = acc;
    Q.k = k;
    Q.Hh = Hh;
    const uint32_t stride = replay_hot_stride(k, Hh);
    unsigned char* meta = (unsigned char*)p->s_rmeta.ensure(c, (((size_t)nmap + 15) & ~(size_t)15) + (size_t)stride * 4);
    Q.slot_map = meta;
    Q.out = (uint32_t*)(meta + (((size_t)nmap + 15) & ~(size_t)15));
    Q.slab = (uint32_t*)p->s_rregion.ensure(c, (size_t)Q.G * stride * 4);
    HIPX(hipMemcpyAsync(meta, map.data(), nmap, hipMemcpyHostToDevice, st));
    launch_replay_hot(Q, st);
    HIPX(hipGetLastError());
    // per winner: K3 over its Hh slot counts, keys mapped to the inner ordinals
    unsigned long long* dk = (unsigned long long*)p->s_rkeys.ensure(c, (size_t)k * (kk + 1) * 8);
    HIPX(hipMemsetAsync(dk, 0, (size_t)k * (kk + 1) * 8, st));
    const uint32_t n_wg = std::min<uint32_t>(512, (Hh + 4095) / 4096);
    unsigned long long* cand = (unsigned long long*)p->s_cand.ensure(c, (size_t)Hh * 8);
    uint32_t* hh = (uint32_t*)p->s_hist.ensure(c, (2048 + 2) * 4);
    for (uint32_t w = 0; w < k; ++w) {
        TopkParams K{};
        K.counts32 = Q.out + (size_t)w * Hh;
        K.ord_of = hs->d_hot_ord.as<uint32_t>();
        K.T = Hh;
        K.order = tn2.s.order;
        K.min_doc_count = tn2.s.min_doc_count;
        K.shard_min_doc_count = tn2.s.shard_min_doc_count;
        K.k = kk;
        K.n_wg = n_wg;
        K.cand = cand;
        K.hist = hh;
        K.sel = hh + 2048;
        K.out_keys = dk + (size_t)w * (kk + 1);
        K.out_sum = K.out_keys + kk;
        launch_topk(K, st);
        HIPX(hipGetLastError());
    }
    d2h_u64(p, p->h_rkeys, dk, (size_t)k * (kk + 1));
    uint32_t* hmiss = (uint32_t*)p->h_rfill.ensure((size_t)k * 4 + 16);
    HIPX(hipMemcpyAsync(hmiss, Q.out + (size_t)k * Hh, (size_t)k * 4, hipMemcpyDeviceToHost, st));
    bsync(p);
    const unsigned long long* hk = p->h_rkeys.as<unsigned long long>();
    for (uint32_t w = 0; w < k; ++w) {
        const unsigned long long last = hk[(size_t)w * (kk + 1) + kk - 1];
        if (last == 0 || ((last >> 32) & 0x7FFFFFFFull) <= bound) return false;  // not settled: the full replay
    }
    for (uint32_t w = 0; w < k; ++w) {
        const unsigned long long* ki = hk + (size_t)w * (kk + 1);
        rs.other[w] = top[w].count - (int64_t)hmiss[w];
        for (uint32_t j = 0; j < kk; ++j) {
            TermPick tp;
            tp.ord = 0xFFFFFFFFu - (uint32_t)ki[j];
            tp.count = (int64_t)((ki[j] >> 32) & 0x7FFFFFFFull);
            rs.other[w] -= tp.count;
            rs.cell[w].push_back(0);  // (no gather: the counts came with the keys)
            rs.picks[w].push_back(tp);
        }
    }
    return true;
}

// TermsAggregator breadth_first (A/bucket/terms/TermsAggregator.java:161 shouldDefer; BestBucketsDeferringCollector
// .prepareSelectedBuckets :127-166, replayed from GlobalOrdinalsStringTermsAggregator.buildAggregation :195-196): the
// child's collectors run again over the retained segments, each doc counted in its outer bucket's winner slot when that
// bucket survived (the replay grid [slot][inner ordinal], rows padded to replay_stride); then the inner terms of every
// winner are selected -- on the GPU per row (count / term orders) or from the fetched rows on the host (metric orders,
// rows of at most 65,536 terms), with the same comparators as the dense grid's select_terms.  A count-only child whose
// grid is over what the partitioned counting path stages (kPartMaxStaged partitions) replays the winners in batches, so
// every pass counts in LDS partitions instead of one global atomic per doc (hot inner terms serialise those).
static ReplaySel replay_child(esgpu_plan* p, const ChildSrc& kid, const std::vector<TermPick>& top, uint64_t T_outer) {
    ReplaySel rs;
    const uint32_t k = (uint32_t)top.size();
    rs.picks.resize(k);
    rs.other.assign(k, 0);
    rs.cell.resize(k);
    if (!k || kid.rpipes.empty()) return rs;
    if (replay_hot(p, kid, top, T_outer, rs)) return rs;
    hipStream_t st = p->stream;
    const SpecNode& tn2 = p->specs[kid.spec];
    const Pipeline& B0 = p->pipes[kid.pipes[0]];
    Pipeline& R0 = p->pipes[kid.rpipes[0]];
    const bool agg2 = tn2.s.order == ESGPU_ORDER_AGG_ASC || tn2.s.order == ESGPU_ORDER_AGG_DESC;
    const bool host_sel = agg2 || B0.value_count2 <= 65536;
    uint32_t wb = k;
    if (!host_sel && kid.rpipes.size() == 1 && R0.met == 0 && R0.cards.empty()) {
        const uint64_t part_cells = (uint64_t)kPartMaxStaged << kPartShift;
        wb = (uint32_t)std::min<uint64_t>(k, std::max<uint64_t>(1, part_cells / replay_stride(B0.value_count2)));
        if (const char* e = std::getenv("ESGPU_REPLAY_BATCH")) {  // tests: smaller batches on small grids
            const int v = std::atoi(e);
            if (v >= 1) wb = std::min<uint32_t>(wb, (uint32_t)v);
        }
    }
    LeafRef ord2;
    if (agg2)
        for (size_t gj = 0; gj < tn2.children.size(); ++gj) if (tn2.children[gj] == tn2.order_child) ord2 = kid.rgrand[gj];
    // count-only children in batches: compact the winners' docs once, then count each batch from its region
    ReplayRegions rr;
    const bool compact = wb < k && replay_compaction() && replay_compact(p, kid, top, wb, T_outer, rr);
    // count orders selected on the GPU: every batch's rows go to one key array, fetched once after the last batch (the
    // counts are in the keys: no gather, no wait per batch)
    std::vector<uint8_t> deferred(k, 0);
    unsigned long long* dk_all = nullptr;
    uint32_t kk_all = 0;
    for (uint32_t b0 = 0; b0 < k; b0 += wb) {
        const uint32_t kb = std::min(wb, k - b0);
        bool any;
        if (compact) {
            const uint32_t bi = b0 / wb;
            any = rr.any && rr.n[bi] > 0;
            if (any) {  // the batch's replay grid, counted from its region (the partitioned path's u32 counters)
                Pipeline& R = R0;
                R.vcA = kb;
                R.vcB = rr.vcB;
                R.tdict = rr.da;
                R.tdictB = rr.db;
                R.T = (uint32_t)(kb * replay_stride(rr.vcB));
                R.H = 1;
                R.key0 = 0;
                R.keyed = false;
                R.value_count = R.T;
                R.vcnt_mode = 0;
                R.ocnt_mode = OCNT_NONE;
                alloc_grid(p, R);
                R.allocated = true;
                R.fresh = false;
                R.cnt32 = true;  // the grid was just zeroed: either width
                const uint32_t* reg = p->s_rregion.as<uint32_t>() + rr.off[bi];
                count_partitioned(p, R, reg, rr.n[bi], (rr.n[bi] + kBlockDocs - 1) / kBlockDocs, nullptr, nullptr, 0);
            }
        } else {
            any = replay_pass(p, kid, top, b0, kb, T_outer);
        }
        const uint64_t nb = any ? R0.vcB : B0.value_count2;
        const uint64_t stride = replay_stride(nb);
        if (!any) {  // no doc of these winners has an inner term: every row is empty (min_doc_count 0 still lists terms)
            std::vector<unsigned long long> zero(std::max<uint64_t>(nb, 1), 0ull);
            for (uint32_t i = b0; i < b0 + kb; ++i) {
                rs.picks[i] = select_terms(tn2.s, zero.data(), (uint32_t)nb, &rs.other[i], [](uint32_t) { return NAN; });
                rs.cell[i].assign(rs.picks[i].size(), 0);
            }
            continue;
        }
        const bool count_order = tn2.s.order == ESGPU_ORDER_COUNT_DESC || tn2.s.order == ESGPU_ORDER_COUNT_ASC;
        const uint32_t kk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nb, (uint64_t)std::max<int64_t>(tn2.s.shard_size, 0)));
        // an inner shard_size beyond the GPU top-k's final sort: count orders select their candidates on the GPU and
        // sort them on the host (below); term orders select from the batch's rows on the host
        if (host_sel || (kk > kTopkMax && !count_order)) {  // the winners' rows on the host
            for (int pi : kid.rpipes) fetch_grid(p, p->pipes[pi]);
            bsync(p);
            for (uint32_t r = 0; r < kb; ++r) {
                const size_t row = (size_t)r * stride;
                rs.picks[b0 + r] = select_terms(tn2.s, R0.hc.cnt + row, (uint32_t)nb, &rs.other[b0 + r], [&](uint32_t ord) {
                    return order_value(p, tn2, p->pipes[ord2.pipe], ord2.leaf, row + ord);
                });
                for (const TermPick& tp : rs.picks[b0 + r]) rs.cell[b0 + r].push_back(row + tp.ord);
            }
            continue;
        }
        // per winner row: the GPU top-k (K3) over its inner ordinals, then one gather of the picked cells of every array
        require(p->docs_seen < (1ull << 31), ESGPU_ERR_UNSUPPORTED,
                "a breadth-first terms request over more than 2^31 - 1 docs (more than one Lucene shard): runs on the CPU path");
        const bool big = kk > kTopkMax;
        const bool defer = count_order && !big && kid.rgrand.empty();  // (grandchildren read the gathered cells)
        unsigned long long* dk;
        if (defer) {
            if (!dk_all) {
                dk_all = (unsigned long long*)p->s_rkeys.ensure(p->ctx, (size_t)k * (kk + 1) * 8);
                HIPX(hipMemsetAsync(dk_all, 0, (size_t)k * (kk + 1) * 8, st));
                kk_all = kk;
            }
            dk = dk_all + (size_t)b0 * (kk + 1);
        } else {
            dk = (unsigned long long*)p->s_rkeys2.ensure(p->ctx, (size_t)kb * (kk + 1) * 8);
            HIPX(hipMemsetAsync(dk, 0, (size_t)kb * (kk + 1) * 8, st));
        }
        std::vector<unsigned long long> big_keys;
        const uint32_t n_wg = std::min<uint32_t>(512, (uint32_t)((nb + 4095) / 4096));
        unsigned long long* cand = (unsigned long long*)p->s_cand.ensure(p->ctx, (count_order ? (size_t)nb : (size_t)n_wg * kk) * 8);
        uint32_t* hs = (uint32_t*)p->s_hist.ensure(p->ctx, (2048 + 2) * 4);
        for (uint32_t r = 0; r < kb; ++r) {
            TopkParams K{};
            if (R0.cnt32) K.counts32 = R0.g_cnt.as<unsigned int>() + (size_t)r * stride;
            else K.counts = R0.g_cnt.as<unsigned long long>() + (size_t)r * stride;
            K.T = (uint32_t)nb;
            K.order = tn2.s.order;
            K.min_doc_count = tn2.s.min_doc_count;
            K.shard_min_doc_count = tn2.s.shard_min_doc_count;
            K.k = kk;
            K.n_wg = n_wg;
            K.cand = cand;
            K.hist = hs;
            K.sel = hs + 2048;
            K.out_keys = dk + (size_t)r * (kk + 1);
            K.out_sum = K.out_keys + kk;
            if (!big) {
                launch_topk(K, st);
                HIPX(hipGetLastError());
                continue;
            }
            // the histogram threshold and the candidates at or above it on the GPU; their sort on the host
            launch_topk_candidates(K, st);
            HIPX(hipGetLastError());
            uint32_t* hsel = (uint32_t*)p->h_rfill.ensure(16);
            HIPX(hipMemcpyAsync(hsel, K.sel, 8, hipMemcpyDeviceToHost, st));
            HIPX(hipMemcpyAsync(hsel + 2, K.out_sum, 8, hipMemcpyDeviceToHost, st));
            bsync(p);
            const uint32_t nc = hsel[1];
            uint64_t row_sum;
            std::memcpy(&row_sum, hsel + 2, 8);
            d2h_u64(p, p->h_rcand, cand, nc);
            bsync(p);
            std::vector<unsigned long long> ck(p->h_rcand.as<unsigned long long>(), p->h_rcand.as<unsigned long long>() + nc);
            const size_t take = std::min<size_t>(kk, ck.size());
            std::partial_sort(ck.begin(), ck.begin() + take, ck.end(), std::greater<unsigned long long>());
            big_keys.resize((size_t)kb * (kk + 1), 0ull);
            std::copy(ck.begin(), ck.begin() + take, big_keys.begin() + (size_t)r * (kk + 1));
            big_keys[(size_t)r * (kk + 1) + kk] = row_sum;
        }
        if (defer) {
            std::fill(deferred.begin() + b0, deferred.begin() + b0 + kb, 1);
            continue;
        }
        const unsigned long long* hk;
        if (big) {
            hk = big_keys.data();
        } else {
            d2h_u64(p, p->h_rkeys, dk, (size_t)kb * (kk + 1));
            bsync(p);
            hk = p->h_rkeys.as<unsigned long long>();
        }
        std::vector<uint32_t> cells;
        for (uint32_t r = 0; r < kb; ++r) {
            const unsigned long long* ki = hk + (size_t)r * (kk + 1);
            rs.other[b0 + r] = (int64_t)ki[kk];
            for (uint32_t j = 0; j < kk; ++j) {
                const unsigned long long key = ki[j];
                if (key == 0) break;
                TermPick tp;
                const uint32_t lo = (uint32_t)key;
                tp.ord = tn2.s.order == ESGPU_ORDER_TERM_DESC ? lo : 0xFFFFFFFFu - lo;
                const uint64_t hi = (key >> 32) & 0x7FFFFFFFull;
                tp.count = tn2.s.order == ESGPU_ORDER_COUNT_DESC ? (int64_t)hi
                         : tn2.s.order == ESGPU_ORDER_COUNT_ASC ? (int64_t)(0x7FFFFFFFull - hi) : -1;
                rs.cell[b0 + r].push_back(cells.size());
                cells.push_back((uint32_t)((size_t)r * stride + tp.ord));
                rs.picks[b0 + r].push_back(tp);
            }
        }
        uint32_t* dc = (uint32_t*)p->s_cells.ensure(p->ctx, std::max<size_t>(cells.size(), 1) * 4);
        if (!cells.empty()) HIPX(hipMemcpyAsync(dc, cells.data(), cells.size() * 4, hipMemcpyHostToDevice, st));
        for (int pi : kid.rpipes) {  // H == 1: the gather of rows is a gather of cells
            Pipeline& R = p->pipes[pi];
            require(R.H == 1, ESGPU_ERR_DEVICE, "replay grid with a key dimension");
            fetch_rows(p, R, dc, (uint32_t)cells.size());
        }
        bsync(p);  // also keeps `cells` alive for the copy
        for (uint32_t r = 0; r < kb; ++r)
            for (size_t j = 0; j < rs.picks[b0 + r].size(); ++j) {
                TermPick& tp = rs.picks[b0 + r][j];
                if (tp.count < 0) tp.count = (int64_t)R0.hc.cnt[rs.cell[b0 + r][j]];  // term orders: count from the gather
                rs.other[b0 + r] -= tp.count;
            }
    }
    if (dk_all) {  // the deferred rows (count orders: count and ordinal in each key)
        d2h_u64(p, p->h_rkeys, dk_all, (size_t)k * (kk_all + 1));
        bsync(p);
        const unsigned long long* hk = p->h_rkeys.as<unsigned long long>();
        for (uint32_t w = 0; w < k; ++w) {
            if (!deferred[w]) continue;
            const unsigned long long* ki = hk + (size_t)w * (kk_all + 1);
            rs.other[w] = (int64_t)ki[kk_all];
            for (uint32_t j = 0; j < kk_all; ++j) {
                const unsigned long long key = ki[j];
                if (key == 0) break;
                TermPick tp;
                tp.ord = 0xFFFFFFFFu - (uint32_t)key;
                const uint64_t hi = (key >> 32) & 0x7FFFFFFFull;
                tp.count = tn2.s.order == ESGPU_ORDER_COUNT_DESC ? (int64_t)hi : (int64_t)(0x7FFFFFFFull - hi);
                rs.other[w] -= tp.count;
                rs.cell[w].push_back(0);  // (no gather: the counts came with the keys)
                rs.picks[w].push_back(tp);
            }
        }
    }
    return rs;
}

static Block build_terms_root(esgpu_plan* p, const Group& g) {
    hipStream_t st = p->stream;
    const SpecNode& tn = p->specs[g.root];
    Block r = terms_shell(p, g.root, child_protos(p, g));
    Pipeline& P0 = p->pipes[g.pipes[0]];
    if (!P0.allocated) { r.append_empty(); return r; }  // unmapped: buildEmptyAggregation
    const uint32_t T = P0.T;
    // the pipeline of the child the terms are ordered by (an outer-level pipeline: one cell per ordinal)
    const bool agg_order = tn.s.order == ESGPU_ORDER_AGG_ASC || tn.s.order == ESGPU_ORDER_AGG_DESC;
    LeafRef ord_ref;
    if (agg_order)
        for (const ChildSrc& k : g.kids) if (k.spec == tn.order_child) ord_ref = k.leaf;
    // outer doc counts per ordinal (term_totals over the [H][T] grid unless counted separately)
    const unsigned long long* dcnt = P0.g_cnt.as<unsigned long long>();
    if (P0.ocnt_mode == OCNT_TERMS || P0.ocnt_mode == OCNT_TERMS_DERIVED) dcnt = P0.g_ocnt.as<unsigned long long>();
    else if (P0.H > 1) {
        unsigned long long* tmp = (unsigned long long*)p->s_tcnt.ensure(p->ctx, (size_t)T * 8);
        launch_term_totals(P0.g_cnt.as<unsigned long long>(), P0.H, T, tmp, st);
        HIPX(hipGetLastError());
        dcnt = tmp;
    }
    int64_t other = 0;
    std::vector<TermPick> top;
    const uint64_t k_req = std::min<uint64_t>(P0.value_count, (uint64_t)std::max(tn.s.shard_size, 0));
    const bool count_order = tn.s.order == ESGPU_ORDER_COUNT_DESC || tn.s.order == ESGPU_ORDER_COUNT_ASC;
    // (the GPU top-k's keys hold a count in 31 bits: a request over at most 2^31 - 1 docs, i.e. one Lucene shard)
    const bool gpu_topk = !agg_order && P0.value_count > 65536 && k_req <= kTopkMax && (P0.H == 1 || count_order) &&
                          p->docs_seen < (1ull << 31);
    if (!gpu_topk) hc_flush(p);
    if (P0.cnt32 && !gpu_topk) {  // u32 counts (partitioned / hot-cold paths) widened for the host selection
        unsigned long long* w = (unsigned long long*)p->s_tcnt.ensure(p->ctx, (size_t)T * 8);
        launch_widen_u32(P0.g_cnt.as<unsigned int>(), T, w, st);
        HIPX(hipGetLastError());
        dcnt = w;
    }
    if (gpu_topk) {
        // K3 on the GPU: only the k winners (and the count total) cross PCIe
        const uint32_t kk = (uint32_t)std::max<uint64_t>(k_req, 1);
        TopkParams K{};
        K.counts = dcnt;
        K.counts32 = P0.cnt32 ? P0.g_cnt.as<unsigned int>() : nullptr;  // the top-k reads 4 B per ordinal
        K.T = (uint32_t)P0.value_count;
        K.order = tn.s.order;
        K.min_doc_count = tn.s.min_doc_count;
        K.shard_min_doc_count = tn.s.shard_min_doc_count;
        K.k = kk;
        K.n_wg = std::min<uint32_t>(512, (K.T + 4095) / 4096);
        K.cand = (unsigned long long*)p->s_cand.ensure(p->ctx, (count_order ? (size_t)K.T : (size_t)K.n_wg * kk) * 8);
        uint32_t* hs = (uint32_t*)p->s_hist.ensure(p->ctx, (2048 + 2) * 4);
        K.hist = hs;
        K.sel = hs + 2048;
        unsigned long long* dk = (unsigned long long*)p->s_keys.ensure(p->ctx, ((size_t)kk + 1) * 8);
        K.out_keys = dk;
        K.out_sum = dk + kk;
        HIPX(hipMemsetAsync(K.out_sum, 0, 8, st));
        hc_topk_launch(p, P0, K, (uint32_t)k_req, st);
        HIPX(hipGetLastError());
        d2h_u64(p, p->h_keys, dk, (size_t)kk + 1);
        const unsigned long long* hk = p->h_keys.as<unsigned long long>();
        bsync(p);
        hc_check_err(p);
        other = (int64_t)hk[kk];
        for (uint32_t i = 0; i < (uint32_t)k_req; ++i) {
            const unsigned long long key = hk[i];
            if (key == 0) break;
            TermPick tp;
            const uint32_t lo = (uint32_t)key;
            tp.ord = (tn.s.order == ESGPU_ORDER_TERM_DESC) ? lo : 0xFFFFFFFFu - lo;
            const uint64_t hi = (key >> 32) & 0x7FFFFFFFull;
            tp.count = tn.s.order == ESGPU_ORDER_COUNT_DESC ? (int64_t)hi
                     : tn.s.order == ESGPU_ORDER_COUNT_ASC ? (int64_t)(0x7FFFFFFFull - hi) : -1;  // term orders: gathered below
            top.push_back(tp);
        }
    } else {
        d2h_u64(p, p->h_tcnt, dcnt, T);
        const unsigned long long* tcnt = p->h_tcnt.as<unsigned long long>();
        const bool card_order = agg_order && p->specs[tn.order_child].s.type == ESGPU_AGG_CARDINALITY;
        std::vector<double> card_vals;
        if (card_order) {  // every ordinal's sketch, gathered, and its estimate (HyperLogLogPlusPlus.cardinality)
            Pipeline& OPc = p->pipes[ord_ref.pipe];
            std::vector<uint32_t> all(T);
            for (uint32_t o = 0; o < T; ++o) all[o] = o;
            gather_cards(p, OPc, all);
            card_vals.assign(T, 0.0);
            for (const CardState& cs : OPc.cards)
                if (cs.spec == tn.order_child)
                    for (uint32_t o = 0; o < T; ++o) card_vals[o] = (double)card_estimate(cs, o);
        } else if (agg_order) {
            fetch_grid(p, p->pipes[ord_ref.pipe]);  // every ordinal's metric partials
        }
        bsync(p);
        const Pipeline* OP = agg_order ? &p->pipes[ord_ref.pipe] : nullptr;
        top = select_terms(tn.s, tcnt, (uint32_t)P0.value_count, &other, [&](uint32_t ord) {
            return card_order ? card_vals[ord] : order_value(p, tn, *OP, ord_ref.leaf, ord);
        });
    }
    bmark(p, "selected");
    if (p->skeleton) {  // esgpu_plans_build_reduce: the winners and their counts; the children's rows merge on the device
        p->sk_ords.clear();
        begin_instance(r, other);
        for (const TermPick& tp : top) {
            const std::string term = plan_term(p, P0, tp.ord);
            push_bucket(r, tp.ord, &term, tp.count);
            p->sk_ords.push_back(tp.ord);
            for (Block& sb : r.subs) sb.append_empty();
        }
        end_instance(r);
        return r;
    }
    const uint32_t k = (uint32_t)top.size();
    uint32_t* rows = (uint32_t*)p->h_rows.ensure(std::max<size_t>(k, 1) * 4);
    for (uint32_t i = 0; i < k; ++i) rows[i] = top[i].ord;
    uint32_t* drows = (uint32_t*)p->s_rows.ensure(p->ctx, std::max<size_t>(k, 1) * 4);
    if (k) HIPX(hipMemcpyAsync(drows, rows, (size_t)k * 4, hipMemcpyHostToDevice, st));
    // histogram children whose own children are numeric metrics are compacted on the GPU (compact_rows): the host
    // receives their buckets as whole columnar arrays; every other child reads the winners' rows [k][H] on the host
    std::vector<char> fast(g.kids.size(), 0), need_rows(p->pipes.size(), 0);
    need_rows[g.pipes[0]] = gpu_topk;  // term orders read the winners' counts from P0's rows
    p->h_compact.resize(g.kids.size());
    std::vector<std::vector<CompactLeaf>> leaf_of(g.kids.size());  // what each compacted child's transfer holds
    for (size_t ki = 0; ki < g.kids.size(); ++ki) {
        const ChildSrc& kid = g.kids[ki];
        if (kid.filter) { for (int pi : kid.pipes) need_rows[pi] = 1; continue; }
        if (!kid.bucket) { need_rows[kid.leaf.pipe] = 1; continue; }
        const Pipeline& B0 = p->pipes[kid.pipes[0]];
        bool ok = ESGPU_COMPACT_ROWS && B0.allocated && !B0.inner_terms && !B0.ord_hist && B0.cards.empty() &&
                  kid.grand.size() <= (size_t)kCompactLeaves && kid.deep < 0;
        for (const LeafRef& l : kid.grand) {  // the leaves' grids index like B0's (the kernel reads one cell of each)
            const Pipeline& L = p->pipes[l.pipe];
            ok = ok && L.allocated && L.H == B0.H && L.T == B0.T && L.key0 == B0.key0 &&
                 is_metric(p->specs[L.metrics[l.leaf]].s.type);
        }
        fast[ki] = ok;
        if (ok) continue;
        for (int pi : kid.pipes) need_rows[pi] = 1;
        for (const LeafRef& l : kid.grand) need_rows[l.pipe] = 1;
    }
    for (int pi : g.pipes) {
        Pipeline& pl = p->pipes[pi];
        if (pl.allocated && !pl.comp && (need_rows[pi] || !pl.cards.empty())) fetch_rows(p, pl, drows, k);
    }
    for (size_t ki = 0; ki < g.kids.size(); ++ki) {
        if (!fast[ki] || !k) continue;
        const ChildSrc& kid = g.kids[ki];
        const Pipeline& B0 = p->pipes[kid.pipes[0]];
        const size_t cap = (size_t)k * B0.H, nl = kid.grand.size();
        PinnedBuf& hb = p->h_compact[ki];
        const size_t nnz_bytes = ((size_t)k * 4 + 63) & ~(size_t)63;
        char* base = (char*)hb.ensure(nnz_bytes + cap * 8 * (2 + 5 * nl));
        char* dbase = (char*)hb.dev();
        auto dev_at = [&](size_t a) { return dbase + nnz_bytes + a * cap * 8; };
        CompactParams C{};
        C.rows = drows;
        C.k = k; C.H = B0.H; C.T = B0.T;
        C.cnt = B0.g_cnt.as<unsigned long long>();
        C.nnz = (uint32_t*)p->s_nnz.ensure(p->ctx, (size_t)k * 4);
        C.o_nnz = (uint32_t*)dbase;
        // the narrowest transfer the host can expand: u32 slots (keys computed on the host) and counts, leaf counts only
        // where a leaf's value count differs from its bucket's doc count, extrema and sums of squares only where collected
        C.o_slot = (uint32_t*)dev_at(0);
        C.o_count = (uint32_t*)dev_at(1);
        C.nleaves = (int32_t)nl;
        for (size_t gj = 0; gj < nl; ++gj) {
            const Pipeline& L = p->pipes[kid.grand[gj].pipe];
            const int32_t type = p->specs[L.metrics[kid.grand[gj].leaf]].s.type;
            CompactLeaf& o = C.leaf[gj];
            o.cnt = (L.vcnt_mode ? L.g_vcnt : L.g_cnt).as<unsigned long long>();
            o.sum = L.g_sum.as<double>();
            o.mn = L.met >= 2 && type != ESGPU_AGG_AVG ? L.g_min.as<unsigned long long>() : nullptr;
            o.mx = o.mn ? L.g_max.as<unsigned long long>() : nullptr;
            o.sq = L.met >= 3 && type == ESGPU_AGG_EXTENDED_STATS ? L.g_sq.as<double>() : nullptr;
            o.o_count = o.cnt == C.cnt ? nullptr : (uint32_t*)dev_at(2 + 5 * gj);
            o.o_sum = (double*)dev_at(3 + 5 * gj);
            o.o_min = o.mn ? (double*)dev_at(4 + 5 * gj) : nullptr;
            o.o_max = o.mn ? (double*)dev_at(5 + 5 * gj) : nullptr;
            o.o_sq = o.sq ? (double*)dev_at(6 + 5 * gj) : nullptr;
        }
        leaf_of[ki].assign(C.leaf, C.leaf + nl);
        launch_compact_rows(C, st);
        HIPX(hipGetLastError());
        (void)base;
    }
    bmark(p, "fetch_issued");
    bsync(p);
    bmark(p, "fetched");
    for (int pi : g.pipes) {
        Pipeline& pl = p->pipes[pi];
        if (!pl.allocated || pl.cards.empty() || pl.comp) continue;
        std::vector<uint32_t> cells((size_t)k * pl.H);
        for (uint32_t i = 0; i < k; ++i)
            for (uint32_t s2 = 0; s2 < pl.H; ++s2) cells[(size_t)i * pl.H + s2] = s2 * pl.T + top[i].ord;
        gather_cards(p, pl, cells);
    }
    // deferred terms-under-terms children: their breadth-first replay over the surviving outer buckets
    std::vector<ReplaySel> replays(g.kids.size());
    for (size_t ki = 0; ki < g.kids.size(); ++ki) {
        const ChildSrc& kid = g.kids[ki];
        if (!kid.bucket || kid.rpipes.empty() || !p->pipes[kid.pipes[0]].deferred || !p->pipes[kid.pipes[0]].allocated) continue;
        replays[ki] = replay_child(p, kid, top, P0.value_count);
    }
    bmark(p, "replayed");
    // three-level children: the composite ordinals their emission reads, gathered as rows [r][H] -- shape 1 (terms{terms
    // {histogram}}): (winner, each X term it selects), shape 2 (terms{histogram{terms}}): (winner, every Y term)
    std::vector<std::vector<uint32_t>> deep_off(g.kids.size());
    for (size_t ki = 0; ki < g.kids.size(); ++ki) {
        const ChildSrc& kid = g.kids[ki];
        if (kid.deep < 0) continue;
        const Pipeline& B0 = p->pipes[kid.pipes[0]];
        Pipeline& C0 = p->pipes[kid.dpipes[0]];
        if (!C0.allocated || !B0.allocated) continue;
        const uint64_t nb = C0.vcB;
        std::vector<uint32_t> rows;
        deep_off[ki].assign(k + 1, 0);
        for (uint32_t i = 0; i < k; ++i) {
            deep_off[ki][i] = (uint32_t)rows.size();
            if (top[i].count == 0) continue;
            if (kid.deep_shape == 1) {
                if (!B0.tdict2) continue;
                const SpecNode& tn2 = p->specs[kid.spec];
                LeafRef ord2;
                if (tn2.s.order == ESGPU_ORDER_AGG_ASC || tn2.s.order == ESGPU_ORDER_AGG_DESC)
                    for (size_t gj = 0; gj < tn2.children.size(); ++gj) if (tn2.children[gj] == tn2.order_child) ord2 = kid.grand[gj];
                const size_t row = (size_t)i * B0.H;
                int64_t other2 = 0;
                for (const TermPick& tp : select_terms(tn2.s, B0.hc.cnt + row, (uint32_t)B0.value_count2, &other2,
                         [&](uint32_t ord) { return order_value(p, tn2, p->pipes[ord2.pipe], ord2.leaf, row + ord); }))
                    rows.push_back((uint32_t)(top[i].ord * nb + tp.ord));
            } else {
                for (uint64_t y = 0; y < nb; ++y) rows.push_back((uint32_t)(top[i].ord * nb + y));
            }
        }
        deep_off[ki][k] = (uint32_t)rows.size();
        const uint32_t nr = (uint32_t)rows.size();
        uint32_t* dr = (uint32_t*)p->s_drows.ensure(p->ctx, std::max<size_t>(nr, 1) * 4);
        if (nr) HIPX(hipMemcpyAsync(dr, rows.data(), (size_t)nr * 4, hipMemcpyHostToDevice, st));
        for (int pi : kid.dpipes) {
            Pipeline& D = p->pipes[pi];
            if (!D.allocated) continue;
            require(D.H == C0.H && D.T == C0.T && D.key0 == C0.key0, ESGPU_ERR_DEVICE, "sibling pipelines disagree on the key grid");
            fetch_rows(p, D, dr, nr);
            if (!D.cards.empty()) {
                std::vector<uint32_t> cells((size_t)nr * D.H);
                for (uint32_t r2 = 0; r2 < nr; ++r2)
                    for (uint32_t s2 = 0; s2 < D.H; ++s2) cells[(size_t)r2 * D.H + s2] = s2 * D.T + rows[r2];
                gather_cards(p, D, cells);
            }
        }
        bsync(p);  // s_drows is reused by the next three-level child
    }
    if (gpu_topk) {  // otherDocCount = (sum of all counts) - (sum of the winners' counts)
        for (uint32_t i = 0; i < k; ++i) {
            if (top[i].count < 0) top[i].count = (int64_t)P0.hc.cnt[i];  // term orders (H == 1): count from the row
            other -= top[i].count;
        }
    }
    for (size_t ki = 0; ki < g.kids.size(); ++ki) {  // compacted children: k instances appended as whole arrays
        if (!fast[ki]) continue;
        const ChildSrc& kid = g.kids[ki];
        const Pipeline& B0 = p->pipes[kid.pipes[0]];
        Block& sub = r.subs[ki];
        if (!k) continue;
        const size_t cap = (size_t)k * B0.H, nl = kid.grand.size();
        const char* hb = (const char*)p->h_compact[ki].p;
        const size_t nnz_bytes = ((size_t)k * 4 + 63) & ~(size_t)63;
        auto host_at = [&](size_t a) { return hb + nnz_bytes + a * cap * 8; };
        const uint32_t* nnz = (const uint32_t*)hb;
        size_t total = 0;
        sub.n += k;
        sub.doc_count_error.insert(sub.doc_count_error.end(), k, 0);
        sub.other_doc_count.insert(sub.other_doc_count.end(), k, 0);
        sub.boff.reserve(sub.boff.size() + k);
        for (uint32_t i = 0; i < k; ++i) {
            total += nnz[i];
            sub.boff.push_back(sub.boff.back() + nnz[i]);
        }
        const uint32_t* slots = (const uint32_t*)host_at(0);
        const size_t n0 = sub.key.size();
        sub.key.resize(n0 + total);
        int64_t* kd = sub.key.data() + n0;
        if (B0.ktable) {  // slots: the bucket-start table's keys
            for (size_t q = 0; q < total; ++q) kd[q] = B0.kt_key[slots[q]];
        } else {
            const int64_t k0 = B0.key0, iv = B0.interval, off = B0.offset;
            for (size_t q = 0; q < total; ++q) kd[q] = (k0 + (int64_t)slots[q]) * iv + off;
        }
        const uint32_t* cnts = (const uint32_t*)host_at(1);
        const size_t c0 = sub.bcount.size();
        sub.bcount.resize(c0 + total);
        int64_t* cd = sub.bcount.data() + c0;
        for (size_t q = 0; q < total; ++q) cd[q] = (int64_t)cnts[q];
        sub.berr.insert(sub.berr.end(), total, 0);
        sub.term_off.insert(sub.term_off.end(), total, sub.term_pool.size());
        for (size_t gj = 0; gj < nl; ++gj) {
            Block& gb = sub.subs[gj];
            const CompactLeaf& o = leaf_of[ki][gj];
            gb.n += total;
            if (o.o_count) {
                const uint32_t* c = (const uint32_t*)host_at(2 + 5 * gj);
                const size_t g0 = gb.count.size();
                gb.count.resize(g0 + total);
                for (size_t q = 0; q < total; ++q) gb.count[g0 + q] = (int64_t)c[q];
            } else {
                gb.count.insert(gb.count.end(), cd, cd + total);
            }
            const double* sm = (const double*)host_at(3 + 5 * gj);
            gb.sum.insert(gb.sum.end(), sm, sm + total);
            if (o.o_min) {
                const double* mn = (const double*)host_at(4 + 5 * gj);
                const double* mx = (const double*)host_at(5 + 5 * gj);
                gb.min.insert(gb.min.end(), mn, mn + total);
                gb.max.insert(gb.max.end(), mx, mx + total);
            } else {  // not collected (avg): the empty leaf's values
                gb.min.insert(gb.min.end(), total, __builtin_inf());
                gb.max.insert(gb.max.end(), total, -__builtin_inf());
            }
            if (o.o_sq) {
                const double* sq = (const double*)host_at(6 + 5 * gj);
                gb.sumsq.insert(gb.sumsq.end(), sq, sq + total);
            } else {
                gb.sumsq.insert(gb.sumsq.end(), total, 0.0);
            }
        }
    }
    bmark(p, "kids_appended");
    for (const ChildSrc& kid : g.kids) {  // every pipeline of a bucket child shares its key grid
        if (!kid.bucket) continue;
        const Pipeline& B0 = p->pipes[kid.pipes[0]];
        for (const LeafRef& l : kid.grand) {
            const Pipeline& L = p->pipes[l.pipe];
            require(!B0.allocated || (L.H == B0.H && L.key0 == B0.key0), ESGPU_ERR_DEVICE,
                    "sibling pipelines disagree on the key grid");
        }
    }
    // one allocation per array: the bucket children's total bucket count over the winners, reserved up front
    for (size_t ki = 0; ki < g.kids.size(); ++ki) {
        const ChildSrc& kid = g.kids[ki];
        if (kid.filter) continue;
        const Pipeline& B0 = kid.bucket ? p->pipes[kid.pipes[0]] : p->pipes[kid.leaf.pipe];
        if (!B0.allocated || fast[ki]) continue;
        size_t nb = k;
        if (kid.bucket) {
            nb = 0;
            for (size_t c = 0; c < (size_t)k * B0.H; ++c) nb += B0.hc.cnt[c] != 0;
            reserve_buckets(r.subs[ki], nb, k);
            for (Block& gb : r.subs[ki].subs) reserve_leaves(gb, nb);
        } else {
            reserve_leaves(r.subs[ki], nb);
        }
    }
    bmark(p, "reserved");
    std::vector<uint32_t> slots, cells;
    std::vector<int64_t> counts;
    begin_instance(r, other);
    for (uint32_t i = 0; i < k; ++i) {
        const std::string term = plan_term(p, P0, top[i].ord);
        push_bucket(r, top[i].ord, &term, top[i].count);
        if (top[i].count == 0) {  // bucketEmptyAggregations (a compacted child's row is empty too: appended above)
            for (size_t ki = 0; ki < g.kids.size(); ++ki) if (!fast[ki]) r.subs[ki].append_empty();
            continue;
        }
        for (size_t ki = 0; ki < g.kids.size(); ++ki) {
            const ChildSrc& kid = g.kids[ki];
            Block& sub = r.subs[ki];
            if (fast[ki]) continue;
            if (kid.filter) {
                append_filter(p, kid, i, sub);
                continue;
            }
            if (!kid.bucket) {
                const Pipeline& L = p->pipes[kid.leaf.pipe];
                if (!L.allocated) sub.append_empty(); else append_leaf(p, L, kid.leaf.leaf, i, sub);
                continue;
            }
            const Pipeline& B0 = p->pipes[kid.pipes[0]];
            if (!B0.allocated) { sub.append_empty(); continue; }
            if (B0.inner_terms && B0.deferred) {  // replayed breadth-first: the picks of replay_child
                if (!B0.tdict2) { sub.append_empty(); continue; }
                const ReplaySel& rs = replays[ki];
                begin_instance(sub, rs.other[i]);
                for (size_t j = 0; j < rs.picks[i].size(); ++j) {
                    const TermPick& tp = rs.picks[i][j];
                    const std::string term2 = B0.tdict2->term(tp.ord);
                    push_bucket(sub, tp.ord, &term2, tp.count);
                    if (tp.count == 0) { for (Block& sb : sub.subs) sb.append_empty(); continue; }
                    for (size_t gj = 0; gj < kid.rgrand.size(); ++gj)
                        append_leaf(p, p->pipes[kid.rgrand[gj].pipe], kid.rgrand[gj].leaf, rs.cell[i][j], sub.subs[gj]);
                }
                end_instance(sub);
                continue;
            }
            if (B0.inner_terms) {  // terms under terms: the inner buckets are the top terms of the winner's row
                if (!B0.tdict2) { sub.append_empty(); continue; }
                const SpecNode& tn2 = p->specs[kid.spec];
                LeafRef ord2;
                if (tn2.s.order == ESGPU_ORDER_AGG_ASC || tn2.s.order == ESGPU_ORDER_AGG_DESC)
                    for (size_t gj = 0; gj < tn2.children.size(); ++gj) if (tn2.children[gj] == tn2.order_child) ord2 = kid.grand[gj];
                const size_t row = (size_t)i * B0.H;
                int64_t other2 = 0;
                const std::vector<TermPick> top2 = select_terms(tn2.s, B0.hc.cnt + row, (uint32_t)B0.value_count2, &other2,
                    [&](uint32_t ord) { return order_value(p, tn2, p->pipes[ord2.pipe], ord2.leaf, row + ord); });
                begin_instance(sub, other2);
                uint32_t dj = kid.deep >= 0 && !deep_off[ki].empty() ? deep_off[ki][i] : 0;
                for (const TermPick& tp : top2) {
                    const std::string term2 = B0.tdict2->term(tp.ord);
                    push_bucket(sub, tp.ord, &term2, tp.count);
                    if (tp.count == 0) { for (Block& sb : sub.subs) sb.append_empty(); ++dj; continue; }
                    for (size_t gj = 0; gj < kid.grand.size(); ++gj)
                        append_leaf(p, p->pipes[kid.grand[gj].pipe], kid.grand[gj].leaf, row + tp.ord, sub.subs[gj]);
                    if (kid.deep >= 0) {  // terms{terms{histogram}}: the histogram of composite row dj
                        if (deep_off[ki].empty()) sub.subs.back().append_empty();
                        else emit_deep(p, kid, (size_t)dj * p->pipes[kid.dpipes[0]].H, 1, sub.subs.back());
                        ++dj;
                    }
                }
                end_instance(sub);
                continue;
            }
            begin_instance(sub, 0);
            const unsigned long long* crow = B0.hc.cnt + (size_t)i * B0.H;
            slots.clear();
            cells.clear();
            counts.clear();
            for (uint32_t s = 0; s < B0.H; ++s) {
                if (crow[s] == 0) continue;
                slots.push_back(s);
                cells.push_back(i * B0.H + s);
                counts.push_back((int64_t)crow[s]);
            }
            append_hist_buckets(B0, slots, counts, sub);
            for (size_t gj = 0; gj < kid.grand.size(); ++gj)
                append_leaves(p, p->pipes[kid.grand[gj].pipe], kid.grand[gj].leaf, cells, sub.subs[gj]);
            if (kid.deep >= 0) {  // terms{histogram{terms}}: per key slot, Y's candidates in the winner's composite rows
                const Pipeline& C0 = p->pipes[kid.dpipes[0]];
                for (uint32_t s2 : slots) {
                    if (deep_off[ki].empty()) { sub.subs.back().append_empty(); continue; }
                    emit_deep(p, kid, (size_t)deep_off[ki][i] * C0.H + s2, C0.H, sub.subs.back());
                }
            }
            end_instance(sub);
        }
    }
    end_instance(r);
    return r;
}

static Block build_hist_root(esgpu_plan* p, const Group& g) {
    hipStream_t st = p->stream;
    Block r = hist_shell(p, g.root, child_protos(p, g));
    Pipeline& P0 = p->pipes[g.pipes[0]];
    if (!P0.allocated) { r.append_empty(); return r; }
    const bool p0_terms = P0.term_spec >= 0;
    // terms children in a count order select each outer key's terms on the GPU (row_topk_kernel, picks written into
    // pinned memory); the whole grid reaches the host only for pipelines whose cells the build still reads
    std::vector<uint32_t> pick_s(g.kids.size(), 0);
    std::vector<char> need(p->pipes.size(), 0);
    if (!p0_terms) need[g.pipes[0]] = 1;
    for (size_t ki = 0; ki < g.kids.size(); ++ki) {
        const ChildSrc& kid = g.kids[ki];
        if (kid.filter) { for (int pi : kid.pipes) need[pi] = 1; continue; }
        if (!kid.bucket) { need[kid.leaf.pipe] = 1; continue; }
        for (const LeafRef& gr : kid.grand) need[gr.pipe] = 1;
        for (int pi : kid.dpipes) need[pi] = 1;  // histogram{terms{terms}}: the whole composite grid
        Pipeline& B0 = p->pipes[kid.pipes[0]];
        const SpecNode& tn = p->specs[kid.spec];
        const bool count_order = tn.s.order == ESGPU_ORDER_COUNT_DESC || tn.s.order == ESGPU_ORDER_COUNT_ASC;
        const uint64_t S = std::min<uint64_t>(B0.value_count, (uint64_t)std::max<int64_t>(tn.s.shard_size, 0));
        if (ESGPU_ROW_TOPK && !B0.ord_hist && B0.allocated && B0.tdict && count_order && B0.value_count == B0.T && S > 0 &&
            S <= kRowTopkMax) {
            pick_s[ki] = (uint32_t)S;
            B0.h_picks.ensure((size_t)B0.H * S * 8);
            B0.h_rowtot.ensure((size_t)B0.H * 8);
            const int64_t min_count = std::max<int64_t>(tn.s.shard_min_doc_count, tn.s.min_doc_count > 0 ? 1 : 0);
            launch_row_topk(B0.g_cnt.as<unsigned long long>(), B0.T, B0.H, (uint32_t)S, tn.s.order == ESGPU_ORDER_COUNT_ASC,
                            min_count, (unsigned long long*)B0.h_picks.dev(), (unsigned long long*)B0.h_rowtot.dev(), st);
            HIPX(hipGetLastError());
        } else {
            need[kid.pipes[0]] = 1;
        }
    }
    for (int pi : g.pipes) {
        Pipeline& pl = p->pipes[pi];
        if (pl.allocated && (need[pi] || !pl.cards.empty() || !ESGPU_ROW_TOPK)) fetch_grid(p, pl);
    }
    bmark(p, "hist_issued");
    unsigned long long* ocnt = nullptr;
    if (p0_terms) {  // histogram doc counts counted per doc beside the [H][T] cells (OCNT_HIST)
        d2h_u64(p, P0.h_ocnt, P0.g_ocnt.p, P0.H);
        ocnt = P0.h_ocnt.as<unsigned long long>();
    }
    bsync(p);
    bmark(p, "hist_synced");
    for (int pi : g.pipes) {
        Pipeline& pl = p->pipes[pi];
        if (!pl.allocated || pl.cards.empty()) continue;
        std::vector<uint32_t> cells((size_t)pl.T * pl.H);
        for (size_t i = 0; i < cells.size(); ++i) cells[i] = (uint32_t)i;
        gather_cards(p, pl, cells);
    }
    // the buckets: key slots with a doc count (columnar fill), then each child over those slots
    std::vector<uint32_t> slots;
    std::vector<int64_t> counts;
    for (uint32_t s = 0; s < P0.H; ++s) {
        const uint64_t dc = p0_terms ? ocnt[s] : P0.hc.cnt[s];
        if (dc == 0) continue;
        slots.push_back(s);
        counts.push_back((int64_t)dc);
    }
    begin_instance(r, 0);
    append_hist_buckets(P0, slots, counts, r);
    for (size_t ki = 0; ki < g.kids.size(); ++ki) {
        const ChildSrc& kid = g.kids[ki];
        Block& sub = r.subs[ki];
        if (kid.filter) {
            for (int pi : kid.pipes) {
                const Pipeline& L = p->pipes[pi];
                require(!L.allocated || (L.H == P0.H && L.key0 == P0.key0), ESGPU_ERR_DEVICE, "sibling pipelines disagree on the key grid");
            }
            for (uint32_t s : slots) append_filter(p, kid, s, sub);  // one cell per key (T == 1): cell == slot
            continue;
        }
        if (!kid.bucket) {
            const Pipeline& L = p->pipes[kid.leaf.pipe];
            require(L.H == P0.H && L.key0 == P0.key0, ESGPU_ERR_DEVICE, "sibling pipelines disagree on the key grid");
            append_leaves(p, L, kid.leaf.leaf, slots, sub);  // one cell per key (T == 1): cell == slot
            continue;
        }
        const Pipeline& B0 = p->pipes[kid.pipes[0]];
        if (B0.ord_hist) {  // histogram under histogram: each outer key's row holds the inner histogram's key cells
            require(!B0.allocated || (B0.H == P0.H && B0.key0 == P0.key0), ESGPU_ERR_DEVICE, "sibling pipelines disagree on the key grid");
            for (uint32_t s : slots) {
                begin_instance(sub, 0);
                if (B0.allocated && B0.ord_keys) {
                    const size_t row = (size_t)s * B0.T;
                    for (uint32_t t = 0; t < B0.T; ++t) {  // HistogramAggregator.buildAggregation: keys ascending
                        const int64_t c = (int64_t)B0.hc.cnt[row + t];
                        if (c == 0) continue;
                        push_bucket(sub, B0.ord_table ? B0.ot_key[t] : (B0.ord_key0 + (int64_t)t) * B0.ord_interval + B0.ord_offset,
                                    nullptr, c);
                        for (size_t gj = 0; gj < kid.grand.size(); ++gj)
                            append_leaf(p, p->pipes[kid.grand[gj].pipe], kid.grand[gj].leaf, row + t, sub.subs[gj]);
                    }
                }
                end_instance(sub);
            }
            continue;
        }
        require(!B0.allocated || B0.tdict == nullptr || (B0.H == P0.H && B0.key0 == P0.key0), ESGPU_ERR_DEVICE,
                "sibling pipelines disagree on the key grid");
        std::string term_scratch;
        for (uint32_t s : slots) {
            if (!B0.allocated || B0.tdict == nullptr) { sub.append_empty(); continue; }
            const SpecNode& tn = p->specs[kid.spec];
            LeafRef ord_ref;
            if (tn.s.order == ESGPU_ORDER_AGG_ASC || tn.s.order == ESGPU_ORDER_AGG_DESC) {
                const auto& ch = tn.children;
                for (size_t gj = 0; gj < ch.size(); ++gj) if (ch[gj] == tn.order_child) ord_ref = kid.grand[gj];
            }
            int64_t other = 0;
            const size_t row = (size_t)s * B0.T;
            std::vector<TermPick> top;
            if (const uint32_t S = pick_s[ki]) {  // the GPU's picks: count-major keys in the order's sequence
                const unsigned long long* pk = B0.h_picks.as<unsigned long long>() + (size_t)s * S;
                const bool asc = tn.s.order == ESGPU_ORDER_COUNT_ASC;
                other = (int64_t)B0.h_rowtot.as<unsigned long long>()[s];
                for (uint32_t i = 0; i < S && pk[i]; ++i) {
                    const uint64_t hi = pk[i] >> 32;
                    const int64_t c = (int64_t)(asc ? 0xFFFFFFFFull - hi : hi);
                    top.push_back({0xFFFFFFFFu - (uint32_t)pk[i], c});
                    other -= c;
                }
            } else {
                top = select_terms(tn.s, B0.hc.cnt + row, (uint32_t)B0.value_count, &other, [&](uint32_t ord) {
                    return order_value(p, tn, p->pipes[ord_ref.pipe], ord_ref.leaf, row + ord);
                });
            }
            begin_instance(sub, other);
            for (auto& tp : top) {
                push_bucket(sub, tp.ord, B0.tdict->view(tp.ord, term_scratch), tp.count);
                if (tp.count == 0) { for (Block& sb : sub.subs) sb.append_empty(); continue; }
                for (size_t gj = 0; gj < kid.grand.size(); ++gj)
                    append_leaf(p, p->pipes[kid.grand[gj].pipe], kid.grand[gj].leaf, row + tp.ord, sub.subs[gj]);
                if (kid.deep >= 0) {  // histogram{terms{terms}}: Y's candidates at (slot, X term) in the composite grid
                    const Pipeline& C0 = p->pipes[kid.dpipes[0]];
                    if (!C0.allocated) { sub.subs.back().append_empty(); continue; }
                    require(C0.H == P0.H && C0.key0 == P0.key0, ESGPU_ERR_DEVICE, "sibling pipelines disagree on the key grid");
                    emit_deep(p, kid, (size_t)s * C0.T + (size_t)tp.ord * C0.vcB, 1, sub.subs.back());
                }
            }
            end_instance(sub);
        }
    }
    end_instance(r);
    return r;
}

static Block build_cardinality(esgpu_plan* p, Pipeline& pl);

static Block build_group(esgpu_plan* p, const Group& g) {
    Pipeline& P0 = p->pipes[g.pipes[0]];
    if (P0.kind == 1) return build_cardinality(p, P0);
    const int t = p->specs[g.root].s.type;
    if (is_metric(t)) return build_metric_root(p, g);
    if (t == ESGPU_AGG_TERMS) return build_terms_root(p, g);
    return build_hist_root(p, g);
}

static Block build_cardinality(esgpu_plan* p, Pipeline& pl) {
    const SpecNode& n = p->specs[pl.root];
    Block r;
    r.type = ESGPU_AGG_CARDINALITY;
    r.name = n.name;
    set_format(r, n);
    r.precision = pl.p;
    r.append_empty();  // counts == null
    if (!pl.allocated || !pl.any_value) return r;
    // CardinalityAggregator:141-143 — a sketch whose cardinality is 0 is reported as "no counts".  That is exactly
    // an empty linear-counting set: HYPERLOGLOG mode implies more than threshold distinct hashes.
    if (pl.hll_mode == 0 && pl.h_lc.empty()) return r;
    r.hll_present[0] = 1;
    r.hll_mode[0] = pl.hll_mode;
    r.lc[0] = pl.h_lc;
    r.regs[0] = pl.h_regs;
    return r;
}

extern "C" int esgpu_plan_build(esgpu_plan* p, esgpu_result** out) {
    return guarded([&] {
        require(p && out, ESGPU_ERR_INVALID, "null argument");
        zero_all_counts(p);  // (a pipeline no segment reached since the reset)
        const double t0 = now_ms();
        p->b_wait = 0;
        p->b_trace = std::getenv("ESGPU_TRACE_BUILD") != nullptr;
        p->b_marks.clear();
        bmark(p, "start");
        if (!p->posted) {
            int rc = esgpu_plan_post_collection(p);
            if (rc != ESGPU_OK) throw EsError(rc, g_err);
        }
        bmark(p, "posted");
        HIPX(hipSetDevice(p->ctx->device));
        std::unique_ptr<ResultHolder> h(new ResultHolder());
        // top-level aggregations in request order; a filter aggregation (InternalFilter, FilterAggregator.java:72-80)
        // is its counting pipeline's doc_count plus its sub-aggregations' groups, in the order create made them
        size_t gi = 0;
        std::function<Block(int)> build_filter = [&](int r) {  // InternalFilter: doc_count, then its sub-aggregations
            Pipeline* cnt = nullptr;
            for (Pipeline& pl : p->pipes) if (pl.count_only && pl.root == r) cnt = &pl;
            Block fb;
            fb.type = ESGPU_AGG_FILTER;
            fb.name = p->specs[r].name;
            fb.n = 1;
            uint64_t dc = 0;
            if (cnt && cnt->allocated) {
                d2h_u64(p, p->h_tcnt, cnt->g_cnt.p, 1);
                const uint64_t* hc = p->h_tcnt.as<uint64_t>();
                bsync(p);
                dc = hc[0];
            }
            fb.count.push_back((int64_t)dc);
            for (int ch : p->specs[r].children) {
                if (p->specs[ch].s.type == ESGPU_AGG_FILTER) { fb.subs.push_back(build_filter(ch)); continue; }
                const Group& g = p->groups[gi++];
                // a terms child of a filter that matched no doc builds empty: bucket 0 of the asMultiBucketAggregator
                // wrapper holds `first` (AggregatorFactory.java:129), whose leaf collector is created only when a doc is
                // collected into the bucket, so GlobalOrdinalsStringTermsAggregator never set globalOrds and its
                // buildAggregation returns buildEmptyAggregation() (GlobalOrdinalsStringTermsAggregator.java:147-149)
                // -- with min_doc_count 0 it lists no zero-count terms.  The GPU plan's terms are always that
                // aggregator (keyword fields through global ordinals: terms over numeric fields are refused at create);
                // the map-mode StringTermsAggregator would instead list zero-count terms from every leaf (:110).
                if (dc == 0 && p->specs[g.root].s.type == ESGPU_AGG_TERMS) {
                    Block e = terms_shell(p, g.root, child_protos(p, g));
                    e.append_empty();
                    fb.subs.push_back(std::move(e));
                    continue;
                }
                fb.subs.push_back(build_group(p, g));
            }
            return fb;
        };
        for (int r : p->tops) {
            if (p->specs[r].s.type != ESGPU_AGG_FILTER) { h->aggs.push_back(build_group(p, p->groups[gi++])); continue; }
            h->aggs.push_back(build_filter(r));
        }
        bmark(p, "assembled");
        h->export_view();
        *out = &h.release()->pub;
        p->b_total = now_ms() - t0;
        bmark(p, "exported");
        if (p->b_trace) {
            std::string line = "esgpu build:";
            char buf[64];
            for (size_t i = 1; i < p->b_marks.size(); ++i) {
                std::snprintf(buf, sizeof buf, " %s +%.3f", p->b_marks[i].first, p->b_marks[i].second - p->b_marks[i - 1].second);
                line += buf;
            }
            std::snprintf(buf, sizeof buf, " (wait %.3f ms)\n", p->b_wait);
            line += buf;
            std::fputs(line.c_str(), stderr);
        }
    });
}

extern "C" int esgpu_plan_reset(esgpu_plan* p) {
    return guarded([&] {
        require(p != nullptr, ESGPU_ERR_INVALID, "null plan");
        HIPX(hipSetDevice(p->ctx->device));
        p->hc_pend = esgpu_plan::HcPending{};  // (a request reset before its build: its cold lists are not needed)
        for (Pipeline& pl : p->pipes) {
            // the next request takes its grid shape and term dictionary from its own first segment
            pl.fresh = true;
            pl.tdict.reset();
            pl.tdict2.reset();
            if (!pl.allocated) continue;
            if (pl.kind == 1) {
                HIPX(hipMemsetAsync(pl.regs.p, 0, pl.regs.bytes, p->stream));
                if (pl.lc_dirty) {  // the LC pass inserted hashes in the last request (12 MB at p = 18 otherwise skipped)
                    HIPX(hipMemsetAsync(pl.lc_set.p, 0, pl.lc_set.bytes, p->stream));
                    HIPX(hipMemsetAsync(pl.lc_first.p, 0xFF, pl.lc_first.bytes, p->stream));
                    pl.lc_dirty = false;
                }
                // the counters (the group floors, snapshot and phase-0 entries are rewritten before they are read)
                HIPX(hipMemsetAsync(pl.lc_count.p, 0, 32, p->stream));
                if (pl.p >= 12)
                    HIPX(hipMemsetAsync(pl.lc_count.as<unsigned char>() + hll_p0_offset(1u << pl.p), 0,
                                        (size_t)hll_p0_ranges(1u << pl.p) * 4, p->stream));
                pl.h_lc.clear();
                pl.h_regs.clear();
                pl.any_value = false;
                pl.hll_seen = 0;
                pl.hll_snap_ok = false;
                pl.hll_r1_pending = false;
                pl.hll_d1.reset();
                pl.hll_nseg = 0;
                continue;
            }
            const size_t cells = (size_t)pl.T * pl.H;
            for (CardState& cs : pl.cards) {
                HIPX(hipMemsetAsync(cs.regs.p, 0, cs.regs.bytes, p->stream));
                HIPX(hipMemsetAsync(cs.sets.p, 0, cs.sets.bytes, p->stream));
                HIPX(hipMemsetAsync(cs.first.p, 0xFF, cs.first.bytes, p->stream));
                HIPX(hipMemsetAsync(cs.cnt.p, 0, cs.cnt.bytes, p->stream));
                HIPX(hipMemsetAsync(cs.nonzero.p, 0, cs.nonzero.bytes, p->stream));
            }
            // the grid's arrays in one launch (one per pipeline instead of one per array: a multi-shard request resets
            // every shard's plan, and each launch costs host time)
            FillList fl{};
            auto span = [&](void* ptr, size_t n, unsigned long long v) {
                if (!ptr || n == 0) return;
                fl.p[fl.count] = (unsigned long long*)ptr;
                fl.n[fl.count] = n;
                fl.v[fl.count] = v;
                if (++fl.count == kFillSpans) { launch_fill_multi(fl, p->stream); fl.count = 0; }
            };
            // the counts: with the other arrays in this launch where the grid is small (the north star's 5.8 MB: one
            // launch fewer ahead of the next collect), else at the request's first collect or build (zero_counts: a
            // high-cardinality terms grid's first hot/cold segment writes its counts itself)
            pl.zero_pending = pl.g_cnt.p != nullptr;
            if (pl.zero_pending && eager_zero_on() && !pl.cnt32 && (size_t)pl.T * pl.H * 8 <= (16u << 20)) {
                span(pl.g_cnt.p, (size_t)pl.T * pl.H, 0ull);
                pl.zero_pending = false;
            }
            if (pl.g_ocnt.p) {
                if (pl.g_ocnt.bytes % 8 == 0) span(pl.g_ocnt.p, pl.g_ocnt.bytes / 8, 0ull);
                else HIPX(hipMemsetAsync(pl.g_ocnt.p, 0, pl.g_ocnt.bytes, p->stream));
            }
            span(pl.g_vcnt.p, cells, 0ull);
            span(pl.g_sum.p, cells, 0ull);
            span(pl.g_min.p, cells, kMinInit);
            span(pl.g_max.p, cells, kMaxInit);
            span(pl.g_sq.p, cells, 0ull);
            if (fl.count) launch_fill_multi(fl, p->stream);
            HIPX(hipGetLastError());
        }
        p->posted = false;
        p->collected = false;
        p->seg_seq = 0;
        p->docs_seen = 0;
        p->unpin_all();
    });
}

extern "C" int esgpu_plan_destroy(esgpu_plan* p) {
    return guarded([&] {
        if (!p) return;
        (void)hipSetDevice(p->ctx->device);
        (void)hipStreamSynchronize(p->stream);
        p->unpin_all();
        for (Pipeline& pl : p->pipes) {
            if (pl.e0) (void)hipEventDestroy(pl.e0);
            if (pl.e1) (void)hipEventDestroy(pl.e1);
        }
        p->pipes.clear();
        if (p->ev_mid) (void)hipEventDestroy(p->ev_mid);
        if (p->ev_xr) (void)hipEventDestroy(p->ev_xr);
        if (p->ev0) (void)hipEventDestroy(p->ev0);
        if (p->ev1) (void)hipEventDestroy(p->ev1);
        if (p->stream) (void)hipStreamDestroy(p->stream);
        delete p;
    });
}

// ------------------------------------------------------------------------------------------------------------
// results
// ------------------------------------------------------------------------------------------------------------
extern "C" int esgpu_result_free(esgpu_result* r) {
    return guarded([&] { delete holder_of(r); });
}

// ---- co-located reduce ----------------------------------------------------------------------------------------
// The shards of one request that live on one device, reduced without materialising their results: each plan's build
// stops after its terms selection (the buckets and counts of its top shard_size terms, children empty), the reference
// reduce runs over those skeletons (InternalTerms.doReduce: the final terms, their counts, errors and other-doc count
// are exactly the full reduce's -- a bucket's children never affect which terms survive), and the surviving terms'
// histogram rows are merged over the shards on the device in shard order (colo_merge_kernel: the per-key
// InternalHistogram / stats reduce) and expanded once.  Shape: a top-level terms aggregation (a count-ordered or term-
// ordered host selection) whose only child is a histogram / date_histogram over an affine rounding with
// min_doc_count >= 1 and numeric metric children.  Anything else builds every shard and reduces (esgpu_reduce).
static bool colo_eligible(esgpu_plan* const* plans, int n, bool shape_only = false, bool cross = false) {
    // (across ranks a rank may hold one shard of the request)
    if (n < (cross ? 1 : 2) || n > kColoMaxShards) return false;
    const esgpu_plan* p0 = plans[0];
    for (int i = 0; i < n; ++i) {
        const esgpu_plan* p = plans[i];
        if (!p || p->ctx != p0->ctx || p->tops.size() != 1 || p->groups.size() != 1 || p->specs.size() != p0->specs.size())
            return false;
        const Group& g = p->groups[0];
        const SpecNode& tn = p->specs[g.root];
        if (tn.s.type != ESGPU_AGG_TERMS || tn.s.order == ESGPU_ORDER_AGG_ASC || tn.s.order == ESGPU_ORDER_AGG_DESC)
            return false;
        if (g.pipes.empty()) return false;
        if (g.kids.empty()) continue;  // terms without sub-aggregations: the shards' builds run side by side, then reduce
        if (g.kids.size() != 1) return false;
        const ChildSrc& kid = g.kids[0];
        if (!kid.bucket || kid.filter || kid.deep >= 0 || !kid.rpipes.empty() || kid.grand.empty() ||
            kid.grand.size() > (size_t)kCompactLeaves)
            return false;
        const SpecNode& hn = p->specs[kid.spec];
        if ((hn.s.type != ESGPU_AGG_HISTOGRAM && hn.s.type != ESGPU_AGG_DATE_HISTOGRAM) || hn.s.min_doc_count < 0 ||
            !hn.tz_starts.empty() || (hn.s.order != ESGPU_ORDER_KEY_ASC && hn.s.order != ESGPU_ORDER_KEY_DESC))
            return false;
        for (const LeafRef& l : kid.grand)
            if (!is_metric(p->specs[p->pipes[l.pipe].metrics[l.leaf]].s.type)) return false;
        if (shape_only) continue;
        const Pipeline& P0 = p->pipes[g.pipes[0]];
        const Pipeline& B0 = p->pipes[kid.pipes[0]];
        if (!P0.allocated || !B0.allocated || P0.value_count > 65536 || P0.comp) return false;
        if (B0.inner_terms || B0.ord_hist || !B0.cards.empty() || B0.ktable || B0.deferred || B0.comp) return false;
        for (const LeafRef& l : kid.grand) {
            const Pipeline& L = p->pipes[l.pipe];
            if (!L.allocated || L.H != B0.H || L.T != B0.T || L.key0 != B0.key0) return false;
        }
        if (B0.interval != plans[0]->pipes[plans[0]->groups[0].kids[0].pipes[0]].interval ||
            B0.offset != plans[0]->pipes[plans[0]->groups[0].kids[0].pipes[0]].offset)
            return false;
    }
    if (!shape_only && !p0->groups[0].kids.empty()) {
        // the merge writes dense [R x Hm] rows into pinned host memory: R <= the terms size, Hm the union of the
        // shards' key ranges (shards far apart in time inflate it); over the budget the shards build and reduce instead
        int64_t kmin = INT64_MAX, kmax = INT64_MIN;
        for (int i = 0; i < n; ++i) {
            const Pipeline& B0 = plans[i]->pipes[plans[i]->groups[0].kids[0].pipes[0]];
            kmin = std::min<int64_t>(kmin, B0.key0);
            kmax = std::max<int64_t>(kmax, B0.key0 + (int64_t)B0.H - 1);
        }
        const SpecNode& tn = p0->specs[p0->groups[0].root];
        const double R = (double)std::max<int64_t>(std::min<int64_t>(tn.s.size, 65536), 1);
        const double nl = (double)p0->groups[0].kids[0].grand.size();
        if (kmax >= kmin && R * (double)(kmax - kmin + 1) * 8.0 * (1.0 + 5.0 * nl) > (double)kColoMergeBytes) return false;
    }
    return true;
}

// A few host threads for esgpu_plans_build_reduce's per-shard skeleton builds: each build is mostly waits on its own
// stream (the collect's end, one device-to-host copy of the ordinal counts), so the shards' round trips overlap instead
// of adding up.  The caller runs jobs too; one batch at a time.
class HostPool {
public:
    static HostPool& get() {
        static HostPool pool;
        return pool;
    }
    void run(int n, const std::function<void(int)>& f) {
        std::lock_guard<std::mutex> one(run_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (threads_.empty())
                for (int i = 0; i < kThreads; ++i) threads_.emplace_back([this] { loop(); });
            job_ = &f;
            next_ = 0;
            n_ = n;
            left_ = n;
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::exception_ptr err;
        {
            std::unique_lock<std::mutex> lk(mu_);
            done_.wait(lk, [&] { return left_ == 0; });
            job_ = nullptr;
            err = err_;
            err_ = nullptr;
        }
        // every job has returned (no worker still reads f or the caller's locals): the first failure goes to the caller
        if (err) std::rethrow_exception(err);
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : threads_) t.join();
    }

private:
    static constexpr int kThreads = 7;
    void work() {
        for (;;) {
            int i;
            const std::function<void(int)>* f;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (!job_ || next_ >= n_) return;
                i = next_++;
                f = job_;
            }
            std::exception_ptr e;
            try {
                (*f)(i);
            } catch (...) {  // a throw must neither terminate a worker nor unwind run() while other jobs still run
                e = std::current_exception();
            }
            std::lock_guard<std::mutex> lk(mu_);
            if (e && !err_) err_ = e;
            if (--left_ == 0) done_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> threads_;
    const std::function<void(int)>* job_ = nullptr;
    std::exception_ptr err_;
    int next_ = 0, n_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

extern "C" int esgpu_plans_colocated(esgpu_plan* const* plans, int32_t n, int32_t* merged) {
    return guarded([&] {
        require(plans && merged && n >= 1, ESGPU_ERR_INVALID, "null argument");
        *merged = colo_eligible(plans, n, true) ? 1 : 0;
    });
}

// ---- co-located reduce building blocks (esgpu_plans_build_reduce, esgpu_comm_build_reduce) --------------------
// every plan's outer doc counts as a ColoTotals descriptor, in p0's pinned h_colo_meta, after each plan's collects (a
// query of its stream, then one wait), and whether the terms selection can run on the device (colo_select_kernel:
// value counts <= kColoSelMax, a count or term order, doc counts below 2^31)
struct ColoSelection {
    std::vector<ColoTotals> d;
    ColoSelect S{};
    uint32_t Tmax = 0;
    bool dev = false;
};
static ColoSelection colo_selection(esgpu_plan* const* plans, int n) {
    ColoSelection r;
    esgpu_plan* p0 = plans[0];
    r.d.resize(n);
    static const bool dev_sel_on = [] { const char* e = std::getenv("ESGPU_COLO_DEVSEL"); return !(e && *e == '0'); }();
    r.dev = dev_sel_on;
    for (int i = 0; i < n; ++i) {
        esgpu_plan* p = plans[i];
        const Pipeline& P0 = p->pipes[p->groups[0].pipes[0]];
        // this plan's collects (an event wait measured slower; a query is cheaper than a wait on an idle stream)
        if (p != p0 && hipStreamQuery(p->stream) != hipSuccess) HIPX(hipStreamSynchronize(p->stream));
        ColoTotals& c = r.d[i];
        const bool oc = P0.ocnt_mode == OCNT_TERMS || P0.ocnt_mode == OCNT_TERMS_DERIVED;
        c.cnt = oc ? (const void*)P0.g_ocnt.p : (const void*)P0.g_cnt.p;
        c.H = oc ? 1u : P0.H;
        c.T = P0.T;
        c.cnt32 = !oc && P0.cnt32 ? 1u : 0u;
        c.vc = (uint32_t)P0.value_count;
        r.Tmax = std::max(r.Tmax, P0.T);
        r.dev = r.dev && P0.value_count <= kColoSelMax && p->docs_seen < (1ull << 31);
    }
    const SpecNode& tn0 = p0->specs[p0->groups[0].root];
    r.dev = r.dev && tn0.s.order >= ESGPU_ORDER_COUNT_DESC && tn0.s.order <= ESGPU_ORDER_TERM_DESC;
    r.S.order = tn0.s.order;
    r.S.K = (uint32_t)std::min<int64_t>(std::max<int64_t>(tn0.s.shard_size, 0), kColoSelMax);
    r.S.min_doc_count = tn0.s.min_doc_count;
    r.S.shard_min_doc_count = tn0.s.shard_min_doc_count;
    r.S.shard_size = tn0.s.shard_size;
    std::memcpy(p0->h_colo_meta.ensure(sizeof(ColoTotals) * n), r.d.data(), sizeof(ColoTotals) * n);
    return r;
}

// a shard's terms skeleton from its device selection record o = {picks, other-doc count, count << 32 | ordinal ...}:
// build_terms_root's buckets and counts with empty sub-aggregations, terms resolved through plan tp's dictionary
static Block colo_skeleton(esgpu_plan* tp, const unsigned long long* o, std::vector<uint32_t>* ords) {
    const Group& g = tp->groups[0];
    const Pipeline& P0 = tp->pipes[g.pipes[0]];
    Block r = terms_shell(tp, g.root, {});
    begin_instance(r, (int64_t)o[1]);
    for (uint64_t j = 0; j < o[0]; ++j) {
        const uint32_t ord = (uint32_t)o[2 + j];
        const std::string term = plan_term(tp, P0, ord);
        push_bucket(r, ord, &term, (int64_t)(o[2 + j] >> 32));
        if (ords) ords->push_back(ord);
    }
    end_instance(r);
    return r;
}

// the device descriptor of a plan's histogram child grid and its metric leaves (colo_merge_kernel / colo_pack_kernel)
static ColoShard colo_shard_desc(const esgpu_plan* p, int nl) {
    const ChildSrc& kid = p->groups[0].kids[0];
    const Pipeline& B0 = p->pipes[kid.pipes[0]];
    ColoShard c{};
    c.cnt = B0.g_cnt.as<unsigned long long>();
    c.cnt32 = B0.cnt32 ? 1 : 0;
    c.H = B0.H;
    c.T = B0.T;
    c.key0 = B0.key0;
    for (int l = 0; l < nl; ++l) {
        const Pipeline& L = p->pipes[kid.grand[l].pipe];
        const int32_t type = p->specs[L.metrics[kid.grand[l].leaf]].s.type;
        const unsigned long long* lc = (L.vcnt_mode ? L.g_vcnt : L.g_cnt).as<unsigned long long>();
        c.lcnt[l] = lc == c.cnt && !c.cnt32 ? nullptr : lc;
        c.lsum[l] = L.g_sum.as<double>();
        c.lmn[l] = L.met >= 2 && type != ESGPU_AGG_AVG ? L.g_min.as<unsigned long long>() : nullptr;
        c.lmx[l] = c.lmn[l] ? L.g_max.as<unsigned long long>() : nullptr;
        c.lsq[l] = L.met >= 3 && type == ESGPU_AGG_EXTENDED_STATS ? L.g_sq.as<double>() : nullptr;
    }
    return c;
}

// the terms block's histogram child, rebuilt from the merged rows [R][Hm] at hbase (count; per leaf value count, sum,
// min, max, sum of squares): keys with at least min_doc_count docs, and for min_doc_count 0 the empty buckets of
// addEmptyBuckets (InternalHistogram.java:395-449) -- every grid key between a row's first and last non-empty key, and the
// extended bounds' keys outside them
static void colo_rebuild(Block& tb, const Block& proto, int64_t iv, int64_t off, int64_t kmin, uint64_t Hm, int nl,
                         const char* hbase) {
    const uint64_t R = tb.nbuckets();
    const size_t cells = (size_t)R * Hm;
    Block hist = proto.like();
    const int64_t mdc = proto.min_doc_count;
    const bool fill = mdc == 0 && proto.has_empty_info, desc = proto.order == ESGPU_ORDER_KEY_DESC;
    const unsigned long long* oc = (const unsigned long long*)hbase;
    const unsigned long long* olc = (const unsigned long long*)(hbase + cells * 8);
    const double* osum = (const double*)(hbase + cells * 8 * (1 + (size_t)nl));
    const double* omin = (const double*)(hbase + cells * 8 * (1 + 2 * (size_t)nl));
    const double* omax = (const double*)(hbase + cells * 8 * (1 + 3 * (size_t)nl));
    const double* osq = (const double*)(hbase + cells * 8 * (1 + 4 * (size_t)nl));
    struct Out { int64_t key; int64_t at; };  // at < 0: an empty bucket
    std::vector<Out> list;
    {
        const size_t guess = (size_t)R * Hm;
        hist.key.reserve(guess);
        hist.term_off.reserve(guess + 1);
        hist.bcount.reserve(guess);
        hist.berr.reserve(guess);
        for (int l = 0; l < nl; ++l) {
            Block& gb = hist.subs[l];
            gb.count.reserve(guess);
            for (auto* v : {&gb.sum, &gb.min, &gb.max, &gb.sumsq}) v->reserve(guess);
        }
    }
    for (uint64_t b = 0; b < R; ++b) {
        list.clear();
        int64_t first = -1, last = -1;
        for (uint64_t m = 0; m < Hm; ++m)
            if (oc[(size_t)b * Hm + m]) { if (first < 0) first = (int64_t)m; last = (int64_t)m; }
        auto key_of = [&](int64_t m) { return (kmin + m) * iv + off; };
        if (!fill) {
            for (int64_t m = first; first >= 0 && m <= last; ++m) {
                const size_t at = (size_t)b * Hm + (size_t)m;
                if (oc[at] && (int64_t)oc[at] >= mdc) list.push_back({key_of(m), (int64_t)at});
            }
        } else if (first < 0) {
            if (proto.has_bmin && proto.has_bmax)
                for (int64_t k = proto.bmin; k <= proto.bmax; k += iv) list.push_back({k, -1});
        } else {
            if (proto.has_bmin)
                for (int64_t k = proto.bmin; k < key_of(first); k += iv) list.push_back({k, -1});
            for (int64_t m = first; m <= last; ++m) {
                const size_t at = (size_t)b * Hm + (size_t)m;
                list.push_back({key_of(m), oc[at] ? (int64_t)at : -1});
            }
            if (proto.has_bmax && proto.bmax > key_of(last))
                for (int64_t k = key_of(last) + iv; k <= proto.bmax; k += iv) list.push_back({k, -1});
        }
        if (desc) std::reverse(list.begin(), list.end());
        begin_instance(hist, 0);
        // the instance's buckets written by index (no per-bucket push_back); an empty bucket's leaves are the
        // prototypes' empty instances (addEmptyBuckets' emptyBucketInfo.subAggregations)
        const size_t L = list.size(), k0 = hist.key.size();
        hist.key.resize(k0 + L);
        hist.term_off.resize(k0 + 1 + L, hist.term_pool.size());
        hist.bcount.resize(k0 + L);
        hist.berr.resize(k0 + L, 0);
        for (size_t q = 0; q < L; ++q) {
            hist.key[k0 + q] = list[q].key;
            hist.bcount[k0 + q] = list[q].at < 0 ? 0 : (int64_t)oc[list[q].at];
        }
        for (int l = 0; l < nl; ++l) {
            Block& gb = hist.subs[l];
            const Block& eb = hist.empty_subs.empty() ? gb : hist.empty_subs[l];
            const size_t m0 = gb.count.size();
            gb.n += L;
            gb.count.resize(m0 + L);
            gb.sum.resize(m0 + L);
            gb.min.resize(m0 + L);
            gb.max.resize(m0 + L);
            gb.sumsq.resize(m0 + L);
            const size_t lo = (size_t)l * cells;
            for (size_t q = 0; q < L; ++q) {
                const int64_t at = list[q].at;
                if (at < 0) {
                    gb.count[m0 + q] = eb.count[0];
                    gb.sum[m0 + q] = eb.sum[0];
                    gb.min[m0 + q] = eb.min[0];
                    gb.max[m0 + q] = eb.max[0];
                    gb.sumsq[m0 + q] = eb.sumsq[0];
                    continue;
                }
                gb.count[m0 + q] = (int64_t)olc[lo + at];
                gb.sum[m0 + q] = osum[lo + at];
                gb.min[m0 + q] = omin[lo + at];
                gb.max[m0 + q] = omax[lo + at];
                gb.sumsq[m0 + q] = osq[lo + at];
            }
        }
        end_instance(hist);
    }
    tb.subs.push_back(std::move(hist));
}

extern "C" int esgpu_plans_build_reduce(esgpu_plan* const* plans, int32_t n, esgpu_result** out) {
    tune_host_heap();
    return guarded([&] {
        require(plans && out && n >= 1, ESGPU_ERR_INVALID, "build_reduce needs at least one plan");
        for (int i = 0; i < n; ++i) if (plans[i]) zero_all_counts(plans[i]);
        std::vector<std::unique_ptr<ResultHolder, void (*)(ResultHolder*)>> parts;
        const bool colo = colo_eligible(plans, n) && std::getenv("ESGPU_COLO") == nullptr;
        const bool merged_shape = colo && !plans[0]->groups[0].kids.empty();
        std::vector<esgpu_result*> built(n, nullptr);
        std::vector<int> rcs(n, ESGPU_OK);
        std::vector<std::string> errs(n);
        auto one = [&](int i) {
            plans[i]->skeleton = merged_shape;
            rcs[i] = esgpu_plan_build(plans[i], &built[i]);
            plans[i]->skeleton = false;
            if (rcs[i] != ESGPU_OK) errs[i] = g_err;
        };
        const bool trace = std::getenv("ESGPU_TRACE_BUILD") != nullptr;
        std::vector<std::pair<const char*, double>> marks{{"start", now_ms()}};
        auto mark = [&](const char* w) { if (trace) marks.emplace_back(w, now_ms()); };
        // the merged shape: the skeletons' histogram instances are empty placeholders, replaced below -- the terms are
        // reduced without them (the rebuild starts from the histogram's prototype)
        Block hproto;
        // terms{histogram{metrics}}: every shard's selection from one launch and one wait (no per-plan build), the rows
        // merged on the device; plain terms: the shards' own builds, side by side on the host pool (their top-k launches
        // overlap on the plans' streams)
        bool direct = merged_shape;
        for (int i = 0; direct && i < n; ++i) {
            direct = !plans[i]->hc_check;
            for (const Pipeline& pl : plans[i]->pipes) direct = direct && pl.kind != 1;
        }
        if (direct) {
            esgpu_plan* p0 = plans[0];
            hipStream_t st = p0->stream;
            HIPX(hipSetDevice(p0->ctx->device));
            ColoSelection sel = colo_selection(plans, n);
            const bool dev_select = sel.dev;
            const ColoSelect& S = sel.S;
            const uint32_t Tmax = sel.Tmax;
            PinnedBuf& mb = p0->h_colo_meta;
            PinnedBuf& tb = p0->h_colo_tot;
            if (dev_select) tb.ensure((size_t)n * (2 + S.K) * 8);
            else tb.ensure(std::max<size_t>((size_t)n * Tmax * 8, 8));
            mark("waited");
            if (dev_select) {  // totals in device scratch, the selection on the device, only the picks to the host
                unsigned long long* dtot = (unsigned long long*)p0->s_colo_tot.ensure(p0->ctx, std::max<size_t>((size_t)n * Tmax * 8, 8));
                launch_colo_totals((const ColoTotals*)mb.dev(), (uint32_t)n, Tmax, dtot, st);
                HIPX(hipGetLastError());
                launch_colo_select(dtot, (const ColoTotals*)mb.dev(), (uint32_t)n, Tmax, S, (unsigned long long*)tb.dev(), st);
            } else {
                launch_colo_totals((const ColoTotals*)mb.dev(), (uint32_t)n, Tmax, (unsigned long long*)tb.dev(), st);
            }
            HIPX(hipGetLastError());
            HIPX(hipStreamSynchronize(st));
            mark("totals");
            const unsigned long long* tot = tb.as<unsigned long long>();
            {
                const Group& g0 = p0->groups[0];
                hproto = child_protos(p0, g0)[0].like();
            }
            std::vector<std::unique_ptr<ResultHolder>> sk(n);
            auto select = [&](int i) {  // build_terms_root's host selection (select_terms), its winners only
                esgpu_plan* p = plans[i];
                p->sk_ords.clear();
                sk[i].reset(new ResultHolder());
                if (dev_select) {
                    sk[i]->aggs.push_back(colo_skeleton(p, tot + (size_t)i * (2 + S.K), &p->sk_ords));
                } else {
                    const Group& g = p->groups[0];
                    const Pipeline& P0 = p->pipes[g.pipes[0]];
                    const SpecNode& tn = p->specs[g.root];
                    int64_t other = 0;
                    const std::vector<TermPick> top = select_terms(tn.s, tot + (size_t)i * Tmax, (uint32_t)P0.value_count,
                                                                   &other, [](uint32_t) { return 0.0; });
                    Block r = terms_shell(p, g.root, {});
                    begin_instance(r, other);
                    for (const TermPick& tp : top) {
                        const std::string term = plan_term(p, P0, tp.ord);
                        push_bucket(r, tp.ord, &term, tp.count);
                        p->sk_ords.push_back(tp.ord);
                    }
                    end_instance(r);
                    sk[i]->aggs.push_back(std::move(r));
                }
                p->posted = true;
            };
            mark("protos");
            // measured at 8 x 1,000 terms: 0.05 ms on the pool, 0.10 ms one after the other (ESGPU_COLO_POOL=0)
            static const bool pool = [] { const char* e = std::getenv("ESGPU_COLO_POOL"); return !(e && *e == '0'); }();
            if (pool && !dev_select) HostPool::get().run(n, select);
            else for (int i = 0; i < n; ++i) select(i);
            mark("selected");
            for (int i = 0; i < n; ++i) parts.emplace_back(sk[i].release(), +[](ResultHolder* x) { delete x; });
        } else {
            if (colo) HostPool::get().run(n, one);  // skeletons: selection only, their waits overlapped
            else for (int i = 0; i < n; ++i) one(i);
            for (int i = 0; i < n; ++i)
                if (built[i]) parts.emplace_back(holder_of(built[i]), +[](ResultHolder* h) { delete h; });
            for (int i = 0; i < n; ++i)
                if (rcs[i] != ESGPU_OK) throw EsError(rcs[i], errs[i]);
            if (merged_shape && !parts[0]->aggs.empty() && parts[0]->aggs[0].type == ESGPU_AGG_TERMS &&
                parts[0]->aggs[0].subs.size() == 1) {
                hproto = parts[0]->aggs[0].subs[0].like();
                for (auto& h : parts) h->aggs[0].subs.clear();
            }
        }
        std::vector<const std::vector<Block>*> lists;
        for (auto& h : parts) lists.push_back(&h->aggs);
        std::unique_ptr<ResultHolder> res(new ResultHolder());
        mark("skeletons");
        res->aggs = reduce_lists(lists);
        mark("reduced");
        if (colo && !res->aggs.empty() && res->aggs[0].type == ESGPU_AGG_TERMS && res->aggs[0].subs.empty() &&
            hproto.type != 0) {
            Block& tb = res->aggs[0];
            const uint64_t R = tb.nbuckets();
            esgpu_plan* p0 = plans[0];
            hipStream_t st = p0->stream;
            HIPX(hipSetDevice(p0->ctx->device));
            // rows: each final term's ordinal in each shard that returned it
            std::vector<int32_t> rows((size_t)R * n, -1);
            // one term dictionary for every shard (global ordinals, or the same segment dictionary): a final term's
            // ordinal is its skeleton key in any shard, so membership is a search of each shard's winners
            bool same_dict = true;
            {
                const Pipeline& A = p0->pipes[p0->groups[0].pipes[0]];
                for (int i = 0; i < n && same_dict; ++i) {
                    const Pipeline& B = plans[i]->pipes[plans[i]->groups[0].pipes[0]];
                    same_dict = A.tdict && B.tdict && ::same_dict(A.tdict, B.tdict);
                }
            }
            for (int i = 0; same_dict && i < n; ++i) {
                std::vector<uint32_t> won(plans[i]->sk_ords);
                std::sort(won.begin(), won.end());
                for (uint64_t b = 0; b < R; ++b) {
                    const uint32_t o = (uint32_t)tb.key[b];
                    if (std::binary_search(won.begin(), won.end(), o)) rows[(size_t)b * n + i] = (int32_t)o;
                }
            }
            for (int i = 0; !same_dict && i < n; ++i) {
                const Block& sb = parts[i]->aggs[0];
                std::unordered_map<std::string_view, uint32_t> at;
                for (uint64_t b = 0; b < sb.nbuckets(); ++b)
                    at.emplace(std::string_view(sb.term_pool).substr(sb.term_off[b], sb.term_off[b + 1] - sb.term_off[b]),
                               plans[i]->sk_ords[b]);
                for (uint64_t b = 0; b < R; ++b) {
                    auto it = at.find(std::string_view(tb.term_pool).substr(tb.term_off[b], tb.term_off[b + 1] - tb.term_off[b]));
                    if (it != at.end()) rows[(size_t)b * n + i] = (int32_t)it->second;
                }
            }
            // shard descriptors and the union of the key ranges
            const ChildSrc& kid0 = p0->groups[0].kids[0];
            const int nl = (int)kid0.grand.size();
            std::vector<ColoShard> sh(n);
            int64_t kmin = INT64_MAX, kmax = INT64_MIN;
            for (int i = 0; i < n; ++i) {
                sh[i] = colo_shard_desc(plans[i], nl);
                kmin = std::min<int64_t>(kmin, sh[i].key0);
                kmax = std::max<int64_t>(kmax, sh[i].key0 + (int64_t)sh[i].H - 1);
            }
            const uint64_t Hm = R ? (uint64_t)(kmax - kmin + 1) : 0;
            require(Hm <= (1ull << 26), ESGPU_ERR_UNSUPPORTED, "co-located reduce over a key range beyond 64M buckets");
            const size_t cells = (size_t)R * Hm;
            PinnedBuf& hb = p0->h_colo;
            const size_t o_bytes = cells * 8 * (1 + 5 * (size_t)std::max(nl, 1));
            char* hbase = (char*)hb.ensure(std::max<size_t>(o_bytes, 8));
            char* dbase = (char*)hb.dev();
            // the descriptors in pinned memory the kernel reads directly (no pageable staging copy on the stream)
            PinnedBuf& mb = p0->h_colo_meta;
            char* hmeta = (char*)mb.ensure(sizeof(ColoShard) * n + rows.size() * 4 + 16);
            std::memcpy(hmeta, sh.data(), sizeof(ColoShard) * n);
            if (!rows.empty()) std::memcpy(hmeta + sizeof(ColoShard) * n, rows.data(), rows.size() * 4);
            ColoParams C{};
            C.shards = (const ColoShard*)mb.dev();
            C.rows = (const int32_t*)((const char*)mb.dev() + sizeof(ColoShard) * n);
            C.nsh = (uint32_t)n;
            C.R = (uint32_t)R;
            C.Hm = (uint32_t)Hm;
            C.kmin = kmin;
            C.nleaves = nl;
            C.o_cnt = (unsigned long long*)dbase;
            C.o_lcnt = (unsigned long long*)(dbase + cells * 8);
            C.o_sum = (double*)(dbase + cells * 8 * (1 + (size_t)nl));
            C.o_min = (double*)(dbase + cells * 8 * (1 + 2 * (size_t)nl));
            C.o_max = (double*)(dbase + cells * 8 * (1 + 3 * (size_t)nl));
            C.o_sq = (double*)(dbase + cells * 8 * (1 + 4 * (size_t)nl));
            // the other plans' streams must have finished their collects (each build synchronised its own stream)
            mark("rows");
            launch_colo_merge(C, st);
            HIPX(hipGetLastError());
            HIPX(hipStreamSynchronize(st));
            mark("merged");
            const Pipeline& B00 = p0->pipes[kid0.pipes[0]];
            colo_rebuild(tb, hproto, B00.interval, B00.offset, kmin, Hm, nl, hbase);
            // a large merge buffer is not kept with the plan (pinned memory outside the context's budget)
            if (hb.bytes > kColoKeepBytes) hb.release();
            mark("rebuilt");
        }
        res->export_view();
        mark("exported");
        if (trace) {
            std::string line = "build_reduce";
            char buf[64];
            for (size_t i = 1; i < marks.size(); ++i) {
                std::snprintf(buf, sizeof buf, " %s +%.3f", marks[i].first, marks[i].second - marks[i - 1].second);
                line += buf;
            }
            std::fprintf(stderr, "%s\n", line.c_str());
        }
        *out = &res.release()->pub;
    });
}

// ---- the co-located reduce across ranks -----------------------------------------------------------------------
// esgpu_comm_build_reduce: the co-located reduce (above) with the shards spread over the ranks of a communicator
// (the coordinating reduce SearchPhaseController.java:401-411 over InternalTerms.doReduce,
// InternalTerms.java:165-246, and InternalHistogram.doReduce, InternalHistogram.java:338-476).  Per request:
//   1. every rank selects its shards' top shard_size terms on its device (colo_totals + colo_select), and the ranks
//      all-gather a small header (shape, dictionary identity, each shard's key range) and then the selection records
//      {picks, other-doc count, count << 32 | ordinal ...} straight from device memory;
//   2. every rank runs InternalTerms.doReduce over the skeletons of all shards (the same answer everywhere): the final
//      terms, their counts, errors and other-doc count;
//   3. every rank packs its shards' rows of the final terms on its device (colo_pack_kernel: [F][Hmax][R] words per
//      shard) and the ranks all-gather them device to device;
//   4. the root merges every shard's rows in global shard order (colo_merge_kernel, the rows read as grids with T = R)
//      and rebuilds the histogram child on the host, as the single-device co-located reduce does.
// Shapes the co-located reduce does not take (or dictionaries that differ between ranks) build every local shard and
// reduce through reduce_across (esgpu_comm_reduce) -- on every rank.
// InternalTerms.doReduce (A/bucket/terms/InternalTerms.java:165-246) over the shards' device selection records, for shards
// that number their terms through one dictionary (an ordinal names the same term on every shard, and ordinal order is
// the dictionary's byte order): the buckets, counts, errors and other-doc count reduce_terms computes from the shards'
// skeletons (esgpu_results.cpp), without building them -- only the surviving terms are resolved to bytes.  won[s]: the
// ordinals shard s returned, sorted.
static Block xr_reduce_terms(esgpu_plan* p0, const unsigned long long* recs, int S, uint32_t rec, uint32_t T,
                             std::vector<std::vector<uint32_t>>& won) {
    const Group& g = p0->groups[0];
    const Pipeline& P0 = p0->pipes[g.pipes[0]];
    Block out = terms_shell(p0, g.root, {});
    int64_t sumErr = 0, other = 0;
    // the shards' picks as (ordinal, shard) entries, grouped by ordinal: sparse in the S x K picks, not dense in the
    // dictionary (10M ordinals for config 3)
    struct Pick { uint32_t ord, shard; int64_t count; };
    std::vector<Pick> picks;
    std::vector<int64_t> shardErr(S, 0);
    won.assign(S, {});
    for (int s = 0; s < S; ++s) {
        const unsigned long long* o = recs + (size_t)s * rec;
        const uint64_t np = o[0];
        require(np <= rec - 2, ESGPU_ERR_DEVICE, "internal: selection record overflows its row");
        other += (int64_t)o[1];
        int64_t thisErr;  // InternalTerms: the shard's doc count error
        if ((int64_t)np < out.shard_size || out.order == ESGPU_ORDER_TERM_ASC || out.order == ESGPU_ORDER_TERM_DESC) thisErr = 0;
        else if (out.order == ESGPU_ORDER_COUNT_DESC) thisErr = (int64_t)(o[2 + np - 1] >> 32);  // its last bucket's count
        else thisErr = -1;
        shardErr[s] = thisErr;
        if (sumErr != -1) sumErr = thisErr == -1 ? -1 : sumErr + thisErr;
        won[s].resize(np);
        for (uint64_t j = 0; j < np; ++j) {
            const uint32_t ord = (uint32_t)o[2 + j];
            require(ord < T, ESGPU_ERR_DEVICE, "internal: selection record ordinal out of range");
            won[s][j] = ord;
            picks.push_back({ord, (uint32_t)s, (int64_t)(o[2 + j] >> 32)});
        }
        std::sort(won[s].begin(), won[s].end());
    }
    std::sort(picks.begin(), picks.end(), [](const Pick& a, const Pick& b) { return a.ord != b.ord ? a.ord < b.ord : a.shard < b.shard; });
    std::vector<uint32_t> ords;
    std::vector<int64_t> tcnt, terr;  // per distinct ordinal (parallel to ords)
    for (size_t i = 0; i < picks.size();) {
        const uint32_t ord = picks[i].ord;
        int64_t c = 0, e = 0;
        for (; i < picks.size() && picks[i].ord == ord; ++i) {
            c += picks[i].count;
            const int64_t te = shardErr[picks[i].shard];
            if (e != -1) e = te == -1 ? -1 : e + te;  // Bucket.reduce
        }
        ords.push_back(ord);
        tcnt.push_back(c);
        terr.push_back(e);
    }
    const size_t nb = ords.size();
    std::vector<uint32_t> keep;  // indices into ords
    keep.reserve(nb);
    for (size_t i = 0; i < nb; ++i) {
        if (terr[i] != -1) terr[i] = sumErr == -1 ? -1 : sumErr - terr[i];
        if (tcnt[i] >= out.min_doc_count) keep.push_back((uint32_t)i);
    }
    const size_t size = std::min<size_t>((size_t)std::max(out.required_size, 0), nb);
    const int32_t order = out.order;
    auto less = [&](uint32_t x, uint32_t y) {  // cmp_terms with the ordinal as the term
        const uint32_t a = ords[x], b = ords[y];
        switch (order) {
            case ESGPU_ORDER_COUNT_DESC: return tcnt[x] != tcnt[y] ? tcnt[x] > tcnt[y] : a < b;
            case ESGPU_ORDER_COUNT_ASC: return tcnt[x] != tcnt[y] ? tcnt[x] < tcnt[y] : a < b;
            case ESGPU_ORDER_TERM_DESC: return a > b;
            default: return a < b;
        }
    };
    if (keep.size() > size) {
        std::partial_sort(keep.begin(), keep.begin() + size, keep.end(), less);
        for (size_t i = size; i < keep.size(); ++i) other += tcnt[keep[i]];
        keep.resize(size);
    } else {
        std::sort(keep.begin(), keep.end(), less);
    }
    ++out.n;
    out.doc_count_error.push_back(sumErr == -1 ? -1 : (S == 1 ? 0 : sumErr));
    out.other_doc_count.push_back(other);
    for (uint32_t i : keep) {
        const std::string term = plan_term(p0, P0, ords[i]);
        push_bucket(out, ords[i], &term, tcnt[i]);
        out.berr.back() = terr[i];
    }
    end_instance(out);
    return out;
}

constexpr int kXrHeader = 8 + 2 * kColoMaxShards;  // header words per rank

static uint64_t fnv64(uint64_t h, uint64_t v) {
    for (int i = 0; i < 8; ++i) {
        h ^= (v >> (8 * i)) & 0xFF;
        h *= 0x100000001b3ULL;
    }
    return h;
}
// p0's stream waits for the other local plans' streams (their collects) without a host wait
static void xr_join_streams(esgpu_plan* const* plans, int n) {
    for (int i = 1; i < n; ++i) {
        esgpu_plan* p = plans[i];
        if (!p->ev_xr) HIPX(hipEventCreateWithFlags(&p->ev_xr, hipEventDisableTiming));
        HIPX(hipEventRecord(p->ev_xr, p->stream));
        HIPX(hipStreamWaitEvent(plans[0]->stream, p->ev_xr, 0));
    }
}
// ... and the other way round: the local plans' next collects wait for p0's stream (which read their grids)
static void xr_release_streams(esgpu_plan* const* plans, int n) {
    esgpu_plan* p0 = plans[0];
    if (!p0->ev_xr) HIPX(hipEventCreateWithFlags(&p0->ev_xr, hipEventDisableTiming));
    HIPX(hipEventRecord(p0->ev_xr, p0->stream));
    for (int i = 1; i < n; ++i) HIPX(hipStreamWaitEvent(plans[i]->stream, p0->ev_xr, 0));
}

// ---- top-level cardinality across ranks (config 4) ----
// A request whose only aggregation is a top-level cardinality: InternalCardinality.doReduce over every shard
// (InternalCardinality.java:103-126; HyperLogLogPlusPlus.merge, HyperLogLogPlusPlus.java:201-230) is a register max
// whenever the merged sketch ends in HYPERLOGLOG -- any shard in HYPERLOGLOG, or more non-zero merged registers than the
// linear-counting threshold (every distinct encoded hash raises one register, so the union of the shards' hash sets is
// at least that large).  The device registers of a shard in LINEAR_COUNTING hold every hash too, which is what the
// merge's upgradeToHll re-collects.  One all-reduce (max, u8) of [registers | tail] straight from device memory on p0's
// stream, no host staging: the tail carries the present / HYPERLOGLOG flags and the request's shape hash (as h and ~h:
// after a max over the ranks they read back as each other's complement only if every rank sent the same hash).  Only
// a request that ends in LINEAR_COUNTING (every shard in it, a small union) goes to the builds and reduce_across.
static bool xr_card_shape(esgpu_plan* const* plans, int n) {
    for (int i = 0; i < n; ++i) {
        const esgpu_plan* p = plans[i];
        if (p->tops.size() != 1 || p->groups.size() != 1 || p->specs[p->tops[0]].s.type != ESGPU_AGG_CARDINALITY) return false;
        const Group& g = p->groups[0];
        if (g.pipes.size() != 1 || p->pipes[g.pipes[0]].kind != 1) return false;
    }
    return true;
}
// returns false when the merged sketch may end in LINEAR_COUNTING (every rank decides alike from the reduced bytes)
static bool xr_card(Collective& C, esgpu_plan* const* plans, int n, int32_t root, ResultHolder& res) {
    esgpu_plan* p0 = plans[0];
    hipStream_t st = p0->stream;
    const int spec = p0->tops[0];
    const uint32_t pr = (uint32_t)p0->specs[spec].precision;
    require(pr >= 4 && pr <= 18, ESGPU_ERR_INVALID, "precision out of range");
    const uint32_t m = 1u << pr;
    const uint32_t thr = (uint32_t)((float)(m / 4) * 0.75f);  // Hashset threshold (HyperLogLogPlusPlus.java:437-440)
    // a fresh segment's one-time distinct estimate (post_collection: its later requests' floored-stream floor) reads that
    // plan's own registers on the host -- such a plan takes its post_collection first, once per segment
    for (int i = 0; i < n; ++i) {
        Pipeline& pl = plans[i]->pipes[plans[i]->groups[0].pipes[0]];
        if (pl.allocated && pl.hll_d1 && pl.hll_d1->load() < 0 && (pl.hll_nseg == 1 || pl.hll_r1_pending)) {
            const int rc = esgpu_plan_post_collection(plans[i]);
            if (rc != ESGPU_OK) throw EsError(rc, g_err);
        }
    }
    xr_join_streams(plans, n);
    XrCardPack K{};
    uint64_t h = fnv64(fnv64(fnv64(0xcbf29ce484222325ULL, 0xCA4D), pr), (uint64_t)n);
    for (int i = 0; i < n; ++i) {
        Pipeline& pl = plans[i]->pipes[plans[i]->groups[0].pipes[0]];
        if (!pl.allocated) continue;
        require(pl.p == (int)pr, ESGPU_ERR_DEVICE, "internal: cardinality precision differs between plans");
        K.regs[i] = pl.regs.as<unsigned int>();
        K.cnt[i] = pl.lc_count.as<unsigned int>();
    }
    K.n = (uint32_t)n;
    K.m = m;
    K.thr = thr;
    K.hash = h;
    const size_t bytes = (size_t)m + kXrCardTail;
    K.out = (uint8_t*)p0->s_xr_send.ensure(p0->ctx, bytes);
    PinnedBuf& hp = p0->h_xr_picks;  // [registers | tail] [non-zero count, pad] [2 counters per local plan]
    char* hbase = (char*)hp.ensure(bytes + 8 + 8 * (size_t)n);
    K.lc_out = (uint32_t*)((char*)hp.dev() + bytes + 8);
    uint32_t* dnz = (uint32_t*)p0->s_xr_picks.ensure(p0->ctx, 8);
    HIPX(hipMemsetAsync(dnz, 0, 8, st));
    launch_xr_card_pack(K, st);
    HIPX(hipGetLastError());
    C.allreduce_dev(K.out, bytes, ESGPU_DT_U8, ESGPU_RED_MAX, st);
    launch_xr_card_finish(K.out, m, (unsigned long long*)hp.dev(), dnz, st);
    HIPX(hipGetLastError());
    launch_copy_u64((const unsigned long long*)dnz, (unsigned long long*)((char*)hp.dev() + bytes), 1, st);
    HIPX(hipGetLastError());
    xr_release_streams(plans, n);
    HIPX(hipStreamSynchronize(st));
    const uint8_t* regs = (const uint8_t*)hbase;
    const uint8_t* tail = regs + m;
    uint64_t hmax = 0, cmax = 0;
    for (int k = 0; k < 8; ++k) {
        hmax |= (uint64_t)tail[8 + k] << (8 * k);
        cmax |= (uint64_t)tail[16 + k] << (8 * k);
    }
    require(cmax == ~hmax, ESGPU_ERR_INVALID, "reduce across ranks: the ranks run different requests");
    const uint32_t* lc = (const uint32_t*)(hbase + bytes + 8);
    for (int i = 0; i < n; ++i) {  // the next reset clears a plan's LC set only where its pass inserted hashes
        Pipeline& pl = plans[i]->pipes[plans[i]->groups[0].pipes[0]];
        if (pl.allocated) pl.lc_dirty = pl.lc_dirty || lc[2 * i] > 0;
    }
    const uint32_t nz = *(const uint32_t*)(hbase + bytes);
    const bool present = tail[0] != 0, hll = tail[1] != 0 || nz > thr;
    if (present && !hll) return false;
    if (root >= 0 && root != C.rank) return true;  // the result on the root only
    const SpecNode& sn = p0->specs[spec];
    Block r;
    r.type = ESGPU_AGG_CARDINALITY;
    r.name = sn.name;
    set_format(r, sn);
    r.precision = (int32_t)pr;
    if (!present) {  // no shard collected a value: the empty sketch
        r.append_empty();
    } else {
        ++r.n;
        r.hll_present.push_back(1);
        r.hll_mode.push_back(1);
        r.regs.emplace_back(regs, regs + m);
        r.lc.emplace_back();
    }
    res.aggs.push_back(std::move(r));
    return true;
}

// ---- a plain terms aggregation across ranks (config 3) ----
// terms without sub-aggregations in a count or term order (InternalTerms.doReduce, InternalTerms.java:165-246): every
// local shard's selection record {picks, other-doc count, count << 32 | ordinal ...} is made on its own stream -- the GPU
// top-k (K3, count orders over more than 65,536 ordinals: build_terms_root's selection) or colo_select (up to
// kColoSelMax ordinals) -- and the ranks all-gather [header | records] from device memory in one collective; the
// doReduce then runs once per rank over the records (xr_reduce_terms).  Ranks that cannot make a record (another
// dictionary, an order or size outside both selections) say so in the header, and every rank then builds and reduces.
constexpr int kXrTermsHdr = 8;
static bool xr_terms_shape(esgpu_plan* const* plans, int n) {
    for (int i = 0; i < n; ++i) {
        const esgpu_plan* p = plans[i];
        if (p->tops.size() != 1 || p->groups.size() != 1) return false;
        const Group& g = p->groups[0];
        if (p->specs[g.root].s.type != ESGPU_AGG_TERMS || !g.kids.empty() || g.pipes.size() != 1 || g.fspec >= 0) return false;
        const int32_t o = p->specs[g.root].s.order;
        if (o < ESGPU_ORDER_COUNT_DESC || o > ESGPU_ORDER_TERM_DESC) return false;
    }
    return true;
}
static bool xr_terms(Collective& C, esgpu_plan* const* plans, int n, int32_t root, ResultHolder& res) {
    esgpu_plan* p0 = plans[0];
    hipStream_t st = p0->stream;
    const int W = C.nranks, S = W * n;
    const SpecNode& tn = p0->specs[p0->groups[0].root];
    const uint32_t K = (uint32_t)std::min<int64_t>(std::max<int64_t>(tn.s.shard_size, 0), kTopkMax);  // request-level
    const uint32_t rec = 2 + K, words = kXrTermsHdr + (uint32_t)n * rec;
    const bool count_order = tn.s.order == ESGPU_ORDER_COUNT_DESC || tn.s.order == ESGPU_ORDER_COUNT_ASC;
    unsigned long long* send = (unsigned long long*)p0->s_xr_send.ensure(p0->ctx, (size_t)words * 8);
    PinnedBuf& hh = p0->h_xr_meta;
    uint64_t* hdr = (uint64_t*)hh.ensure(kXrTermsHdr * 8);
    std::memset(hdr, 0, kXrTermsHdr * 8);
    const Pipeline& A = p0->pipes[p0->groups[0].pipes[0]];
    bool ok = tn.s.shard_size >= 1 && (int64_t)K == tn.s.shard_size;
    ok = ok && A.allocated && A.tdict != nullptr && A.H == 1;
    for (int i = 0; ok && i < n; ++i) {
        const Pipeline& B = plans[i]->pipes[plans[i]->groups[0].pipes[0]];
        ok = B.allocated && B.H == 1 && B.value_count == A.value_count && same_dict(A.tdict, B.tdict) &&
             plans[i]->docs_seen < (1ull << 31);
    }
    const bool topk = ok && count_order && A.value_count > 65536;
    ok = ok && (topk || A.value_count <= kColoSelMax);
    if (ok && topk) {
        for (int i = 0; i < n; ++i) {  // each shard's K3 on its own stream, its record into p0's send buffer
            esgpu_plan* p = plans[i];
            const Pipeline& P0 = p->pipes[p->groups[0].pipes[0]];
            const uint64_t k_req = std::min<uint64_t>(P0.value_count, (uint64_t)std::max<int64_t>(tn.s.shard_size, 0));
            const uint32_t kk = (uint32_t)std::max<uint64_t>(k_req, 1);
            TopkParams T{};  // (build_terms_root's K3 parameters)
            T.counts = P0.ocnt_mode == OCNT_TERMS || P0.ocnt_mode == OCNT_TERMS_DERIVED ? P0.g_ocnt.as<unsigned long long>()
                                                                                         : P0.g_cnt.as<unsigned long long>();
            T.counts32 = P0.cnt32 ? P0.g_cnt.as<unsigned int>() : nullptr;
            T.T = (uint32_t)P0.value_count;
            T.order = tn.s.order;
            T.min_doc_count = tn.s.min_doc_count;
            T.shard_min_doc_count = tn.s.shard_min_doc_count;
            T.k = kk;
            T.n_wg = std::min<uint32_t>(512, (T.T + 4095) / 4096);
            T.cand = (unsigned long long*)p->s_cand.ensure(p->ctx, (size_t)T.T * 8);
            uint32_t* hs = (uint32_t*)p->s_hist.ensure(p->ctx, (2048 + 2) * 4);
            T.hist = hs;
            T.sel = hs + 2048;
            unsigned long long* dk = (unsigned long long*)p->s_keys.ensure(p->ctx, ((size_t)kk + 1) * 8);
            T.out_keys = dk;
            T.out_sum = dk + kk;
            HIPX(hipMemsetAsync(T.out_sum, 0, 8, p->stream));
            hc_topk_launch(p, P0, T, (uint32_t)k_req, p->stream);
            HIPX(hipGetLastError());
            if (p != p0) {  // the record is written on p0's stream once this shard's top-k is done
                if (!p->ev_xr) HIPX(hipEventCreateWithFlags(&p->ev_xr, hipEventDisableTiming));
                HIPX(hipEventRecord(p->ev_xr, p->stream));
                HIPX(hipStreamWaitEvent(st, p->ev_xr, 0));
            }
            launch_xr_terms_record(dk, kk, (uint32_t)k_req, tn.s.order, send + kXrTermsHdr + (size_t)i * rec, K, st);
            HIPX(hipGetLastError());
        }
    } else if (ok) {  // up to kColoSelMax ordinals: the co-located reduce's device selection
        ColoSelection sel = colo_selection(plans, n);  // (waits for the local collects)
        ok = sel.dev && sel.S.K == K;
        if (ok) {
            unsigned long long* dtot = (unsigned long long*)p0->s_colo_tot.ensure(p0->ctx, std::max<size_t>((size_t)n * sel.Tmax * 8, 8));
            launch_colo_totals((const ColoTotals*)p0->h_colo_meta.dev(), (uint32_t)n, sel.Tmax, dtot, st);
            HIPX(hipGetLastError());
            launch_colo_select(dtot, (const ColoTotals*)p0->h_colo_meta.dev(), (uint32_t)n, sel.Tmax, sel.S, send + kXrTermsHdr, st);
            HIPX(hipGetLastError());
        }
    }
    hdr[0] = ok ? 1 : 0;
    hdr[1] = (uint64_t)n;
    hdr[2] = ok ? A.tdict->identity : 0;
    hdr[3] = ok ? A.value_count : 0;
    hdr[4] = K;
    HIPX(hipMemcpyAsync(send, hh.p, kXrTermsHdr * 8, hipMemcpyHostToDevice, st));
    unsigned long long* dall = (unsigned long long*)p0->s_xr_allpicks.ensure(p0->ctx, (size_t)words * W * 8);
    C.allgather_dev(send, dall, (uint64_t)words * 8, st);
    PinnedBuf& hp = p0->h_xr_picks;
    hp.ensure((size_t)words * W * 8);
    launch_copy_u64(dall, (unsigned long long*)hp.dev(), (size_t)words * W, st);
    HIPX(hipGetLastError());
    xr_release_streams(plans, n);
    HIPX(hipStreamSynchronize(st));
    for (int i = 0; i < n; ++i) {  // the hot/cold counting's capacity word (a bug, never data), as post_collection checks it
        esgpu_plan* p = plans[i];
        if (!p->hc_check) continue;
        if (p != p0) HIPX(hipStreamSynchronize(p->stream));
        p->hc_check = false;
        volatile uint32_t* err = p->h_hcerr.as<volatile uint32_t>();
        const uint32_t e = *err;
        *err = 0;
        require(e == 0, ESGPU_ERR_DEVICE, "hot/cold counting: partition capacity exceeded");
    }
    const uint64_t* all = hp.as<uint64_t>();
    bool dev = true;
    for (int r = 0; r < W && dev; ++r) {
        const uint64_t* h = all + (size_t)r * words;
        dev = h[0] == 1 && h[1] == (uint64_t)n && h[2] == all[2] && h[3] == all[3] && h[4] == K;
    }
    if (!dev) return false;
    if (root >= 0 && root != C.rank) return true;
    std::vector<unsigned long long> recs((size_t)S * rec);
    for (int s = 0; s < S; ++s)
        std::memcpy(recs.data() + (size_t)s * rec, all + (size_t)(s / n) * words + kXrTermsHdr + (size_t)(s % n) * rec, (size_t)rec * 8);
    std::vector<std::vector<uint32_t>> won;
    res.aggs.push_back(xr_reduce_terms(p0, recs.data(), S, rec, (uint32_t)all[3], won));
    return true;
}

extern "C" int esgpu_comm_build_reduce(esgpu_comm* cm, esgpu_plan* const* plans, int32_t n, int32_t root,
                                       esgpu_result** out) {
    tune_host_heap();
    return guarded([&] {
        require(cm && plans && out && n >= 1 && n <= kColoMaxShards, ESGPU_ERR_INVALID, "build_reduce needs 1..64 local plans");
        for (int i = 0; i < n; ++i) require(plans[i] != nullptr, ESGPU_ERR_INVALID, "null plan");
        for (int i = 0; i < n; ++i) zero_all_counts(plans[i]);
        Collective& C = comm_collective(cm);
        require(root < C.nranks, ESGPU_ERR_INVALID, "build_reduce root is not a rank of the communicator");
        const double t_start = now_ms();
        C.allreduce_bytes = C.allgather_bytes = 0;
        C.collectives = 0;
        C.exchange_ms = 0;
        const int W = C.nranks, S = W * n;
        esgpu_plan* p0 = plans[0];
        hipStream_t st = p0->stream;
        HIPX(hipSetDevice(p0->ctx->device));
        // shapes with a device exchange of their own (decided from the request alone: every rank takes the same branch)
        {
            std::unique_ptr<ResultHolder> res(new ResultHolder());
            bool done = false;
            if (S <= kColoMaxShards && xr_card_shape(plans, n)) done = xr_card(C, plans, n, root, *res);
            else if (S <= kColoMaxShards && xr_terms_shape(plans, n)) done = xr_terms(C, plans, n, root, *res);
            if (done) {
                C.last_path = 1;
                C.last_host_ms = now_ms() - t_start;
                res->export_view();
                *out = &res.release()->pub;
                return;
            }
        }
        // ---- this rank's header and selection records, all-gathered in one collective from device memory ----
        // (the record size is the request's: every rank sends the same number of words, eligible or not)
        std::vector<uint64_t> hdr(kXrHeader, 0);
        bool ok = S <= kColoMaxShards && colo_eligible(plans, n, false, true) && !p0->groups[0].kids.empty();
        for (int i = 0; ok && i < n; ++i) {
            ok = !plans[i]->hc_check;
            for (const Pipeline& pl : plans[i]->pipes) ok = ok && pl.kind != 1;
        }
        const SpecNode& tn_root = p0->specs[p0->groups[0].root];
        const uint32_t K = tn_root.s.type == ESGPU_AGG_TERMS
                               ? (uint32_t)std::min<int64_t>(std::max<int64_t>(tn_root.s.shard_size, 0), kColoSelMax) : 0u;
        const uint32_t rec = 2 + K, words = kXrHeader + (uint32_t)n * rec;
        ColoSelection sel;
        double t_host = t_start;  // the device path's host time is counted once this rank's collects have finished
        if (ok) {
            sel = colo_selection(plans, n);  // waits for the other local plans' collects
            HIPX(hipStreamSynchronize(st));  // ... and p0's
            t_host = now_ms();
            ok = sel.dev && sel.S.K == K;
        }
        int nl = 0;
        if (ok) {
            const Pipeline& A = p0->pipes[p0->groups[0].pipes[0]];
            ok = A.tdict != nullptr;
            for (int i = 1; ok && i < n; ++i) ok = same_dict(A.tdict, plans[i]->pipes[plans[i]->groups[0].pipes[0]].tdict);
            if (ok) {
                nl = (int)p0->groups[0].kids[0].grand.size();
                hdr[2] = A.tdict->identity;
                hdr[3] = A.tdict->n;
                hdr[4] = sel.S.K;
                hdr[5] = (uint64_t)nl;
                hdr[6] = sel.Tmax;
                for (int i = 0; i < n; ++i) {
                    const Pipeline& B0 = plans[i]->pipes[plans[i]->groups[0].kids[0].pipes[0]];
                    hdr[8 + 2 * i] = (uint64_t)B0.key0;
                    hdr[9 + 2 * i] = B0.H;
                }
            }
        }
        hdr[0] = ok ? 1 : 0;
        hdr[1] = (uint64_t)n;
        static const bool trace = std::getenv("ESGPU_TRACE_XR") != nullptr;
        std::vector<std::pair<const char*, double>> marks{{"host", t_host}};
        auto mark = [&](const char* w) { if (trace) marks.emplace_back(w, now_ms()); };
        unsigned long long* dsend = (unsigned long long*)p0->s_xr_picks.ensure(p0->ctx, (size_t)words * 8);
        if (ok) {  // ---- 1. the local selections on the device, into the send buffer behind the header ----
            unsigned long long* dtot = (unsigned long long*)p0->s_colo_tot.ensure(p0->ctx, std::max<size_t>((size_t)n * sel.Tmax * 8, 8));
            launch_colo_totals((const ColoTotals*)p0->h_colo_meta.dev(), (uint32_t)n, sel.Tmax, dtot, st);
            HIPX(hipGetLastError());
            launch_colo_select(dtot, (const ColoTotals*)p0->h_colo_meta.dev(), (uint32_t)n, sel.Tmax, sel.S, dsend + kXrHeader, st);
            HIPX(hipGetLastError());
        }
        PinnedBuf& hh = p0->h_xr_hdr;
        std::memcpy(hh.ensure(kXrHeader * 8), hdr.data(), kXrHeader * 8);
        HIPX(hipMemcpyAsync(dsend, hh.p, kXrHeader * 8, hipMemcpyHostToDevice, st));
        unsigned long long* dall = (unsigned long long*)p0->s_xr_allpicks.ensure(p0->ctx, (size_t)words * W * 8);
        C.allgather_dev(dsend, dall, (uint64_t)words * 8, st);
        PinnedBuf& hp = p0->h_xr_picks;
        hp.ensure((size_t)words * W * 8);
        launch_copy_u64(dall, (unsigned long long*)hp.dev(), (size_t)words * W, st);
        HIPX(hipGetLastError());
        HIPX(hipStreamSynchronize(st));
        mark("records");
        const uint64_t* all = hp.as<uint64_t>();
        // ---- one decision on every rank: the device path, or builds + reduce_across ----
        bool dev = true;
        for (int r = 0; r < W && dev; ++r) {
            const uint64_t* h = all + (size_t)r * words;
            dev = h[0] == 1 && h[1] == (uint64_t)n && h[2] == all[2] && h[3] == all[3] && h[4] == all[4] && h[5] == all[5];
        }
        int64_t kmin = INT64_MAX, kmax = INT64_MIN;
        uint32_t Hmax = 1;
        std::vector<int64_t> skey0(S);
        std::vector<uint32_t> sH(S);
        if (dev) {
            for (int s = 0; s < S; ++s) {
                const uint64_t* h = all + (size_t)(s / n) * words + 8 + 2 * (s % n);
                skey0[s] = (int64_t)h[0];
                sH[s] = (uint32_t)h[1];
                kmin = std::min<int64_t>(kmin, skey0[s]);
                kmax = std::max<int64_t>(kmax, skey0[s] + (int64_t)sH[s] - 1);
                Hmax = std::max(Hmax, sH[s]);
            }
            const SpecNode& tn = p0->specs[p0->groups[0].root];
            const double Rb = (double)std::max<int64_t>(std::min<int64_t>(tn.s.size, 65536), 1);
            dev = kmax >= kmin && kmax - kmin < (1ll << 26) &&
                  Rb * (double)(kmax - kmin + 1) * 8.0 * (1.0 + 5.0 * nl) <= (double)kColoMergeBytes &&
                  (double)S * Rb * Hmax * 8.0 * (1.0 + 5.0 * nl) <= (double)kColoMergeBytes;
        }
        std::unique_ptr<ResultHolder> res(new ResultHolder());
        if (!dev) {  // every local shard built, then the reduce across ranks (its collectives on every rank)
            std::vector<std::unique_ptr<ResultHolder, void (*)(ResultHolder*)>> parts;
            for (int i = 0; i < n; ++i) {
                esgpu_result* r = nullptr;
                const int rc = esgpu_plan_build(plans[i], &r);
                if (rc != ESGPU_OK) throw EsError(rc, g_err);
                parts.emplace_back(holder_of(r), +[](ResultHolder* h) { delete h; });
            }
            std::vector<const std::vector<Block>*> lists;
            for (auto& h : parts) lists.push_back(&h->aggs);
            res->aggs = reduce_across(C, lists);
            C.last_path = 0;
            C.last_host_ms = now_ms() - t_start;
            res->export_view();
            *out = &res.release()->pub;
            return;
        }
        std::vector<unsigned long long> recs((size_t)S * rec);
        for (int s = 0; s < S; ++s)
            std::memcpy(recs.data() + (size_t)s * rec, all + (size_t)(s / n) * words + kXrHeader + (size_t)(s % n) * rec,
                        (size_t)rec * 8);
        const uint64_t dict_n = all[3];
        // ---- 2. InternalTerms.doReduce over every shard's skeleton ----
        std::vector<std::vector<uint32_t>> won;
        res->aggs.push_back(xr_reduce_terms(p0, recs.data(), S, rec, (uint32_t)dict_n, won));
        for (int i = 0; i < n; ++i) plans[i]->posted = true;
        Block& tb = res->aggs[0];
        const uint32_t R = (uint32_t)tb.nbuckets();
        const bool here = root < 0 || root == C.rank;
        mark("skeleton_reduce");
        // ---- 3. this rank's rows of the final terms, packed and all-gathered ----
        const uint32_t F = 1 + 5 * (uint32_t)nl;
        const size_t HR = (size_t)Hmax * R, blk = (size_t)F * HR;
        std::vector<ColoShard> loc(n);
        for (int i = 0; i < n; ++i) loc[i] = colo_shard_desc(plans[i], nl);
        if (R > 0) {
            std::vector<int32_t> rows((size_t)R * n, -1);
            for (uint32_t b = 0; b < R; ++b) {
                const uint32_t o = (uint32_t)tb.key[b];
                for (int i = 0; i < n; ++i) {
                    const std::vector<uint32_t>& w = won[C.rank * n + i];
                    if (std::binary_search(w.begin(), w.end(), o)) rows[(size_t)b * n + i] = (int32_t)o;
                }
            }
            PinnedBuf& pm = p0->h_xr_meta;
            char* pmeta = (char*)pm.ensure(sizeof(ColoShard) * n + rows.size() * 4 + 16);
            std::memcpy(pmeta, loc.data(), sizeof(ColoShard) * n);
            std::memcpy(pmeta + sizeof(ColoShard) * n, rows.data(), rows.size() * 4);
            ColoPackParams K2{};
            K2.shards = (const ColoShard*)pm.dev();
            K2.rows = (const int32_t*)((const char*)pm.dev() + sizeof(ColoShard) * n);
            K2.n = (uint32_t)n;
            K2.R = R;
            K2.Hmax = Hmax;
            K2.nleaves = nl;
            K2.out = (unsigned long long*)p0->s_xr_send.ensure(p0->ctx, (size_t)n * blk * 8);
            launch_colo_pack(K2, st);
            HIPX(hipGetLastError());
            unsigned long long* drecv = (unsigned long long*)p0->s_xr_recv.ensure(p0->ctx, (size_t)S * blk * 8);
            C.allgather_dev(K2.out, drecv, (uint64_t)n * blk * 8, st);
        }
        mark("rows");
        // ---- 4. the root merges every shard's rows in global shard order ----
        if (here) {
            const Block hproto = child_protos(p0, p0->groups[0])[0].like();
            const uint64_t Hm = (uint64_t)(kmax - kmin + 1);
            const Pipeline& B00 = p0->pipes[p0->groups[0].kids[0].pipes[0]];
            PinnedBuf& hb = p0->h_colo;
            const char* hbase = nullptr;
            if (R > 0) {
                const unsigned long long* drecv = (const unsigned long long*)p0->s_xr_recv.buf.p;
                std::vector<ColoShard> vs(S);
                for (int s = 0; s < S; ++s) {
                    ColoShard& c = vs[s];
                    c = ColoShard{};
                    const unsigned long long* base = drecv + (size_t)s * blk;
                    c.cnt = base;
                    c.cnt32 = 0;
                    c.H = sH[s];
                    c.T = R;
                    c.key0 = skey0[s];
                    for (int l = 0; l < nl; ++l) {
                        const unsigned long long* f = base + (size_t)(1 + 5 * l) * HR;
                        c.lcnt[l] = f;
                        c.lsum[l] = (const double*)(f + HR);
                        c.lmn[l] = loc[0].lmn[l] ? f + 2 * HR : nullptr;
                        c.lmx[l] = loc[0].lmx[l] ? f + 3 * HR : nullptr;
                        c.lsq[l] = loc[0].lsq[l] ? (const double*)(f + 4 * HR) : nullptr;
                    }
                }
                std::vector<int32_t> vrows((size_t)R * S, -1);
                for (uint32_t b = 0; b < R; ++b) {
                    const uint32_t o = (uint32_t)tb.key[b];
                    for (int s = 0; s < S; ++s)
                        if (std::binary_search(won[s].begin(), won[s].end(), o)) vrows[(size_t)b * S + s] = (int32_t)b;
                }
                const size_t cells = (size_t)R * Hm;
                PinnedBuf& vm = p0->h_colo_meta;  // (its selection descriptors are consumed)
                char* vmeta = (char*)vm.ensure(sizeof(ColoShard) * S + vrows.size() * 4 + 16);
                std::memcpy(vmeta, vs.data(), sizeof(ColoShard) * S);
                std::memcpy(vmeta + sizeof(ColoShard) * S, vrows.data(), vrows.size() * 4);
                hbase = (const char*)hb.ensure(std::max<size_t>(cells * 8 * (1 + 5 * (size_t)std::max(nl, 1)), 8));
                char* dbase = (char*)hb.dev();
                ColoParams M{};
                M.shards = (const ColoShard*)vm.dev();
                M.rows = (const int32_t*)((const char*)vm.dev() + sizeof(ColoShard) * S);
                M.nsh = (uint32_t)S;
                M.R = R;
                M.Hm = (uint32_t)Hm;
                M.kmin = kmin;
                M.nleaves = nl;
                M.o_cnt = (unsigned long long*)dbase;
                M.o_lcnt = (unsigned long long*)(dbase + cells * 8);
                M.o_sum = (double*)(dbase + cells * 8 * (1 + (size_t)nl));
                M.o_min = (double*)(dbase + cells * 8 * (1 + 2 * (size_t)nl));
                M.o_max = (double*)(dbase + cells * 8 * (1 + 3 * (size_t)nl));
                M.o_sq = (double*)(dbase + cells * 8 * (1 + 4 * (size_t)nl));
                launch_colo_merge(M, st);
                HIPX(hipGetLastError());
                HIPX(hipStreamSynchronize(st));
                mark("merged");
            }
            colo_rebuild(tb, hproto, B00.interval, B00.offset, kmin, Hm, nl, hbase);
            mark("rebuilt");
            if (hb.bytes > kColoKeepBytes) hb.release();
        }
        // the other local plans' next collects (on their own streams) must not rewrite their grids before the pack read them
        if (!p0->ev_xr) HIPX(hipEventCreateWithFlags(&p0->ev_xr, hipEventDisableTiming));
        HIPX(hipEventRecord(p0->ev_xr, st));
        for (int i = 1; i < n; ++i) HIPX(hipStreamWaitEvent(plans[i]->stream, p0->ev_xr, 0));
        if (!here) res->aggs.clear();
        C.last_path = 1;
        C.last_host_ms = now_ms() - t_host;
        res->export_view();
        mark("exported");
        if (trace && C.rank == 0) {
            std::string line = "comm_build_reduce";
            char buf[64];
            for (size_t k = 1; k < marks.size(); ++k) {
                std::snprintf(buf, sizeof buf, " %s +%.3f", marks[k].first, marks[k].second - marks[k - 1].second);
                line += buf;
            }
            std::fprintf(stderr, "%s\n", line.c_str());
        }
        *out = &res.release()->pub;
    });
}

extern "C" int esgpu_reduce(const esgpu_result* const* shards, int32_t n, esgpu_result** out) {
    tune_host_heap();
    return guarded([&] {
        require(out && n >= 1 && shards, ESGPU_ERR_INVALID, "reduce needs at least one shard result");
        std::vector<const std::vector<Block>*> lists;
        for (int i = 0; i < n; ++i) lists.push_back(&holder_of(shards[i])->aggs);
        std::unique_ptr<ResultHolder> h(new ResultHolder());
        h->aggs = reduce_lists(lists);
        h->export_view();
        *out = &h.release()->pub;
    });
}

extern "C" int esgpu_cardinality_value(const esgpu_agg_block* b, uint64_t instance, int64_t* value) {
    return guarded([&] {
        require(b && value && b->type == ESGPU_AGG_CARDINALITY && instance < b->n_instances, ESGPU_ERR_INVALID,
                "not a cardinality block instance");
        require(b->precision >= 4 && b->precision <= 18, ESGPU_ERR_INVALID, "precision out of range");
        const bool present = b->hll_present && b->hll_present[instance];
        const int mode = b->hll_mode ? b->hll_mode[instance] : 0;
        const uint8_t* regs = b->registers ? b->registers[instance] : nullptr;
        const size_t nlc = b->lc_sizes ? (size_t)b->lc_sizes[instance] : 0;
        require(!(present && mode && !regs), ESGPU_ERR_INVALID, "missing registers");
        *value = hll_cardinality(b->precision, present, mode, regs, nlc);
    });
}

extern "C" int esgpu_result_to_xcontent(const esgpu_result* r, char* buf, size_t cap, size_t* needed) {
    return guarded([&] {
        require(r != nullptr, ESGPU_ERR_INVALID, "null result");
        const std::string s = to_xcontent(holder_of(r)->aggs);
        if (needed) *needed = s.size() + 1;
        if (buf && cap) {
            const size_t c = std::min(cap - 1, s.size());
            std::memcpy(buf, s.data(), c);
            buf[c] = 0;
        }
    });
}

extern "C" int esgpu_result_to_stream(const esgpu_result* r, uint8_t* buf, size_t cap, size_t* needed) {
    return guarded([&] {
        require(r != nullptr, ESGPU_ERR_INVALID, "null result");
        std::string s;
        to_es_stream(holder_of(r)->aggs, s);
        if (needed) *needed = s.size();
        if (buf) {
            require(cap >= s.size(), ESGPU_ERR_INVALID, "buffer too small");
            std::memcpy(buf, s.data(), s.size());
        }
    });
}

extern "C" int esgpu_result_to_json(const esgpu_result* r, char* buf, size_t cap, size_t* needed) {
    return guarded([&] {
        require(r != nullptr, ESGPU_ERR_INVALID, "null result");
        ResultHolder* h = holder_of(r);
        if (!h->json_valid) {  // results are immutable: render once (callers size the buffer, then fill it)
            h->json = to_json(h->aggs);
            h->json_valid = true;
        }
        const std::string& s = h->json;
        if (needed) *needed = s.size() + 1;
        if (buf && cap) {
            const size_t c = std::min(cap - 1, s.size());
            std::memcpy(buf, s.data(), c);
            buf[c] = 0;
        }
    });
}

extern "C" int esgpu_result_serialize(const esgpu_result* r, uint8_t* buf, size_t cap, size_t* needed) {
    return guarded([&] {
        std::string s;
        serialize(holder_of(r)->aggs, s);
        if (needed) *needed = s.size();
        if (buf) {
            require(cap >= s.size(), ESGPU_ERR_INVALID, "buffer too small");
            std::memcpy(buf, s.data(), s.size());
        }
    });
}

extern "C" int esgpu_result_deserialize(const uint8_t* buf, size_t len, esgpu_result** out) {
    return guarded([&] {
        std::unique_ptr<ResultHolder> h(new ResultHolder());
        require(deserialize(buf, len, h->aggs), ESGPU_ERR_INVALID, "not an esgpu result stream");
        h->export_view();
        *out = &h.release()->pub;
    });
}

