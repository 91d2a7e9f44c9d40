// esgpu_collect.hpp — the collect kernel (K1/K4-K7 over single-valued columns) and its device helpers, shared by the
// translation units that instantiate it (esgpu_collect_inst.hip, one object per (ORD, HK)) and by the other kernels
// of esgpu_kernels.hip that reuse the doc loaders, predicates and LDS accumulators.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "es_common.hpp"
#include "esgpu_kernels.hpp"

namespace esgpu {

// ------------------------------------------------------------------------------------------------------------
// collect
// ------------------------------------------------------------------------------------------------------------
constexpr int kWG = 512;                         // threads per workgroup (8 waves)
constexpr int kVec = 4;                          // consecutive docs per thread per iteration
constexpr int kIterDocs = kWG * kVec;            // 2048
constexpr int kItersPerBlock = kBlockDocs / kIterDocs;  // 4
#ifndef ESGPU_MAX_PASSES  // passes over a block whose keys span more than the LDS window, before global atomics
#define ESGPU_MAX_PASSES 8
#endif
constexpr int kMaxPasses = ESGPU_MAX_PASSES;
constexpr uint32_t kGroup = kGroupBlocks;  // blocks per multi-pass group (esgpu_kernels.hpp)
#ifndef ESGPU_NBUF_NARROW  // load buffers in flight per thread for shapes reading one narrow column
#define ESGPU_NBUF_NARROW 2  // measured: 4 no faster for terms(host), 4 % slower for date_histogram
#endif
#ifndef ESGPU_MINMAX_CHECK
#define ESGPU_MINMAX_CHECK 1
#endif
#ifndef ESGPU_NBUF_COMPACT  // load buffers of the metric / two-dimension shapes over compact columns
#define ESGPU_NBUF_COMPACT 2
#endif
#ifndef ESGPU_NBUF_HIST  // load buffers of the raw-load counting histogram grids (VK bit 1024: timestamp deltas)
#define ESGPU_NBUF_HIST 4  // with 6 waves per SIMD: date_histogram at 1B docs 0.92 -> 0.84 ms (r5c)
#endif
#ifndef ESGPU_NBUF_HIST_MET  // ... and of those with a metric (their run accumulators take the registers)
#define ESGPU_NBUF_HIST_MET 2
#endif
#ifndef ESGPU_NBUF_PI  // load buffers with packed integer metric cells (all columns compact)
#define ESGPU_NBUF_PI 2
#endif
#ifndef ESGPU_NBUF_PI_RAW  // ... the unfiltered raw-load packed-cell kernels (north star 1.39 -> 1.34 ms at 1B, r5ab2; the
#define ESGPU_NBUF_PI_RAW 4  // folded-accept ones spill at 4)
#endif

struct Doc4 {
    // raw-loaded packed-cell kernels (kRawPI): the loads' words as they arrive, unpacked only when the docs are processed
    // (a conversion right after the load would wait for it there, a full memory latency per buffer reload)
    uint32_t raw[11];  // ([10]: the block-delta key column's high bytes, 4 docs)
    uint64_t racc;
    uint32_t doc0;
    // block-delta kernels (VK bit 8192): the grid key every doc of this buffer's zone block has (its zone-map range
    // rounds to one key; kNoUKey: per-doc keys) -- the block's timestamps were then not read (zone_ukey)
    uint32_t ukey;
    uint32_t ord[kVec];
    int64_t hv[kVec];
    double mv[kVec];
    uint32_t mvd[kVec];  // VK bit 64: the metric's u32 deltas over P.mv_base
    uint32_t ok;      // bit j: doc j passes filters / accept / bounds
    uint32_t hpres;   // bit j: hist value present
    uint32_t mpres;   // bit j: metric value present
};

__device__ __forceinline__ uint32_t bits4(const uint64_t* bm, uint32_t doc0) {
    return (uint32_t)(bm[doc0 >> 6] >> (doc0 & 63)) & 0xFu;
}

// Column streams are read once per request: ESGPU_NT=1 marks them non-temporal (nt) so they do not displace the
// cell grid and the zone maps in L2 / MALL.
#ifndef ESGPU_NT
#define ESGPU_NT 0
#endif
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4_t load16(const void* p) {
#if ESGPU_NT
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
#else
    return *reinterpret_cast<const u32x4_t*>(p);
#endif
}
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2_t load8(const void* p) {
#if ESGPU_NT
    return __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(p));
#else
    return *reinterpret_cast<const u32x2_t*>(p);
#endif
}
__device__ __forceinline__ uint64_t join64(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }
__device__ __forceinline__ void load_i64x4(const int64_t* p, uint32_t doc0, int64_t out[4]) {
    const u32x4_t a = load16(p + doc0), b = load16(p + doc0 + 2);
    out[0] = (int64_t)join64(a.x, a.y); out[1] = (int64_t)join64(a.z, a.w);
    out[2] = (int64_t)join64(b.x, b.y); out[3] = (int64_t)join64(b.z, b.w);
}
__device__ __forceinline__ void load_f64x4(const double* p, uint32_t doc0, double out[4]) {
    const u32x4_t a = load16(p + doc0), b = load16(p + doc0 + 2);
    out[0] = bits_dbl(join64(a.x, a.y)); out[1] = bits_dbl(join64(a.z, a.w));
    out[2] = bits_dbl(join64(b.x, b.y)); out[3] = bits_dbl(join64(b.z, b.w));
}
__device__ __forceinline__ void load_u32x4(const uint32_t* p, uint32_t doc0, uint32_t out[4]) {
    const u32x4_t a = load16(p + doc0);
    out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
}

__device__ __forceinline__ uint32_t eval_pred(const PredDev& q, uint32_t doc0) {
    uint32_t m = 0;
    if (q.kind == PRED_ORD_EQ || q.kind == PRED_ORD_RANGE) {  // a term is the range [ord, ord]
        uint32_t o[4];
        load_u32x4((const uint32_t*)q.col, doc0, o);
#pragma unroll
        for (int j = 0; j < 4; ++j) m |= (uint32_t)((int64_t)o[j] >= q.lo && (int64_t)o[j] <= q.hi && o[j] != kMissingOrd) << j;
    } else if (q.kind == PRED_F64_RANGE) {
        double v[4];
        load_f64x4((const double*)q.col, doc0, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool lo = q.lo_incl ? v[j] >= q.dlo : v[j] > q.dlo;
            const bool hi = q.hi_incl ? v[j] <= q.dhi : v[j] < q.dhi;
            m |= (uint32_t)(lo && hi) << j;
        }
    } else if (q.kind == PRED_D16_RANGE) {
        const u32x2_t w = load8((const uint16_t*)q.col + doc0);
        const uint32_t o[4] = {w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t v = q.base + (int64_t)o[j];
            m |= (uint32_t)(v >= q.lo && v <= q.hi) << j;
        }
    } else if (q.kind == PRED_D32_RANGE) {
        uint32_t o[4];
        load_u32x4((const uint32_t*)q.col, doc0, o);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t v = q.base + (int64_t)o[j];
            m |= (uint32_t)(v >= q.lo && v <= q.hi) << j;
        }
    } else {  // PRED_I64_RANGE (term on a long is the degenerate range [t, t])
        int64_t v[4];
        load_i64x4((const int64_t*)q.col, doc0, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) m |= (uint32_t)(v[j] >= q.lo && v[j] <= q.hi) << j;
    }
    if (q.present) m &= bits4(q.present, doc0);
    return m;
}

// VK (value kinds, compile time): bit 0 = the histogram column holds doubles (keys are (long) casts), bit 1 = the
// metric column holds doubles (else longs cast to double).  A runtime branch on these cost the north-star kernel ~6 %.
// Compact columns (segment products built on first use): bit 16 = the terms dimension is read from the
// 16-bit ordinal column (0xFFFF missing), bit 32 = the histogram column from its 32-bit deltas over hv_base.
// packed-cell kernels over the 16-bit ordinals and metric deltas (and, with a key, the 32-bit timestamp deltas of a dense
// timestamp column): loads only, no use of a loaded word until unpack_docs
template <int MET, int VK, bool HIST>
constexpr bool kRawPI = MET > 0 && (VK & 64) != 0 && (VK & 16) != 0 && (VK & 256) != 0 && (!HIST || (VK & (32 | 8192)) != 0);
#ifndef ESGPU_B16_NOLOAD
#define ESGPU_B16_NOLOAD 0
#endif
#ifndef ESGPU_B16_BRANCH  // single-key blocks skip the timestamp and base loads (a wave-uniform branch; with ESGPU_DOCS8
#define ESGPU_B16_BRANCH 1  // measured level with the dummy loads on the north star, 3 % better on config 5)
#endif
#ifndef ESGPU_B16_SCALAR  // block-delta bases as scalar loads (1) or per-lane vector loads (0)
#define ESGPU_B16_SCALAR 0
#endif
// VK bit 8192 (raw-load kernels only, instead of bit 32): the key column as block deltas -- 16 bits per doc over the
// minimum of its run of 2^kB16Shift docs (one 8-byte word per run, the same for all 4 docs of a thread)
constexpr uint32_t kNoUKey = 0xFFFFFFFFu, kOutUKey = 0xFFFFFFFEu;  // per-doc keys / one key outside the grid
template <int VK>
__device__ __forceinline__ void load_keys_raw(const CollectParams& P, uint32_t doc0, uint32_t (&raw)[11], uint32_t uk) {
    if constexpr ((VK & 8192) != 0) {
        // a block whose docs all round to one key reads no timestamp: every lane loads the column's first word (one
        // cache line per wave, in place of a branch around the load -- a load under a branch makes the compiler wait
        // for the other buffers' loads)
#if ESGPU_B16_NOLOAD  // timing experiment only (wrong keys in multi-key blocks): no timestamp or base loads at all
        raw[2] = doc0; raw[3] = doc0; raw[4] = 0; raw[5] = 0; raw[10] = 0;
        return;
#endif
#if ESGPU_B16_BRANCH  // (A/B) the single-key blocks' loads skipped under a wave-uniform branch
        if (uk != kNoUKey) {
            raw[2] = 0; raw[3] = 0; raw[4] = 0; raw[5] = 0; raw[10] = 0;
            return;
        }
#endif
        const u32x2_t t = load8(P.hv16 + (uk == kNoUKey ? doc0 : 0u));
        raw[2] = t.x; raw[3] = t.y;
        // bits 16..23 of the deltas (24-bit runs): the high-byte plane, or -- for a column whose every run spans < 2^16 --
        // the column's first word for all lanes (hv8_mask 0; the bytes are masked off by hv8_and = 0)
        raw[10] = *reinterpret_cast<const uint32_t*>(P.hv8 + (doc0 & P.hv8_mask));
#if ESGPU_B16_SCALAR
        // a wave's 256 docs lie in one run: its base is a scalar load
        const int64_t b = P.hv16_base[__builtin_amdgcn_readfirstlane(doc0 >> kB16Shift)];
        raw[4] = (uint32_t)b; raw[5] = (uint32_t)((uint64_t)b >> 32);
#else
        const u32x2_t b = load8(P.hv16_base + (doc0 >> kB16Shift));
        raw[4] = b.x; raw[5] = b.y;
#endif
    } else {
        if constexpr ((VK & 16384) != 0) {  // single-key zone blocks read no 32-bit delta either (VK bit 16384)
            if (uk != kNoUKey) {
                raw[2] = 0; raw[3] = 0; raw[4] = 0; raw[5] = 0;
                return;
            }
        }
        const u32x4_t t = load16(P.hv32 + doc0);
        raw[2] = t.x; raw[3] = t.y; raw[4] = t.z; raw[5] = t.w;
    }
}
template <int VK>
__device__ __forceinline__ void unpack_keys_raw(const CollectParams& P, const uint32_t (&raw)[11], int64_t (&hv)[4]) {
    if constexpr ((VK & 8192) != 0) {
        const int64_t b = (int64_t)join64(raw[4], raw[5]);
        const uint32_t h = raw[10] & (P.hv8_and * 0x01010101u);
        hv[0] = b + (int64_t)((raw[2] & 0xFFFFu) | ((h & 0xFFu) << 16));
        hv[1] = b + (int64_t)((raw[2] >> 16) | ((h & 0xFF00u) << 8));
        hv[2] = b + (int64_t)((raw[3] & 0xFFFFu) | ((h >> 16 & 0xFFu) << 16));
        hv[3] = b + (int64_t)((raw[3] >> 16) | ((h >> 24) << 16));
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) hv[j] = P.hv_base + (int64_t)raw[2 + j];
    }
}
// VK bit 1024: grids over dense compact columns without a filter -- 16-bit ordinals (counting terms grids), timestamp
// deltas, a histogram-only grid's u32 metric deltas -- the same raw loads, unpacked when processed
template <bool ORD, int MET, int VK>
constexpr bool kRawH = (VK & 1024) != 0;
// VK bit 2048 (with 1024): a histogram-only grid over a dense long metric whose values span < 2^16 and stay below 2^26 in
// magnitude -- the metric read as its 16-bit deltas and the run accumulators kept as integers (count, sum of deltas, sum
// of squared deltas, min / max delta): exact, and a third of the VALU work of the f64 runs; decoded at the run's flush
template <bool ORD, int MET, int VK>
constexpr bool kIntRuns = !ORD && MET > 0 && (VK & 2048) != 0;
// raw-load kernels whose key column is block deltas (VK bit 8192) or 32-bit deltas (bit 32): single-key zone blocks take
// their key from the zone map (zone_ukey) and read no timestamp
template <bool ORD, bool HIST, int MET, int VK>
constexpr bool kUKeyK = HIST && ((VK & 8192) != 0 || (VK & (32 | 16384)) == (32 | 16384)) &&
                        (kRawPI<MET, VK, HIST> || kRawH<ORD, MET, VK>);

template <bool ORD, bool HIST, int MET, int VK>
__device__ __forceinline__ void load_docs(const CollectParams& P, uint32_t doc0, Doc4& d, uint32_t uk = kNoUKey) {
    d.ukey = uk;
    if constexpr (kRawPI<MET, VK, HIST>) {
        const u32x2_t o = load8(P.ord16 + doc0);
        d.raw[0] = o.x; d.raw[1] = o.y;
        if constexpr (HIST) load_keys_raw<VK>(P, doc0, d.raw, uk);
        const u32x2_t m = load8(P.mv16 + doc0);
        d.raw[6] = m.x; d.raw[7] = m.y;
        if constexpr ((VK & 512) != 0) d.racc = P.accept[doc0 >> 6];
        d.doc0 = doc0;
        return;
    }
    if constexpr (kRawH<ORD, MET, VK>) {
        if constexpr (ORD) {
            const u32x2_t o = load8(P.ord16 + doc0);
            d.raw[0] = o.x; d.raw[1] = o.y;
        }
        if constexpr (HIST) load_keys_raw<VK>(P, doc0, d.raw, uk);
        if constexpr (MET > 0 && (VK & 2048) != 0) {
            const u32x2_t m = load8(P.mv16 + doc0);
            d.raw[6] = m.x; d.raw[7] = m.y;
        } else if constexpr (MET > 0) {
            const u32x4_t m = load16(P.mv32 + doc0);
            d.raw[6] = m.x; d.raw[7] = m.y; d.raw[8] = m.z; d.raw[9] = m.w;
        }
        d.doc0 = doc0;
        return;
    }
    uint32_t ok = 0xF;
    if (doc0 + 4 > P.n_docs) ok = doc0 >= P.n_docs ? 0u : ((1u << (P.n_docs - doc0)) - 1u);
    if constexpr (MET > 0 && (VK & 64)) {
        // packed-cell kernels read no clause and no conditional bitset: the host folds the request's clauses and live
        // docs into one accept bitset first (VK bit 512: loaded unconditionally) -- a load under a runtime branch makes
        // the compiler wait for every load in flight at each later use, i.e. for the other buffer's prefetch
        if constexpr ((VK & 512) != 0) ok &= bits4(P.accept, doc0);
    } else {
        if (P.accept) ok &= bits4(P.accept, doc0);
        for (int k = 0; k < P.npred; ++k) ok &= eval_pred(P.pred[k], doc0);
    }
    d.ok = ok;
    if (ORD && (VK & 8)) {  // inner histogram key index, derived in registers (HistogramAggregator under a histogram)
        int64_t v[4];
        load_i64x4(P.ord_src, doc0, v);
        const uint32_t pres = P.ord_src_present ? bits4(P.ord_src_present, doc0) : 0xFu;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t x = P.ord_src_f64 ? java_long(bits_dbl((uint64_t)v[j])) : v[j];  // longValues of a double
            const uint64_t u = (uint64_t)x - (uint64_t)P.ord_base;
            d.ord[j] = ((pres >> j) & 1) && u < P.ord_span ? magic_div((uint32_t)u, P.omg_m, P.omg_s1, P.omg_s2, P.ord_div)
                                                           : kMissingOrd;
        }
    } else if (ORD && (VK & 16)) {
        const u32x2_t w = load8(P.ord16 + doc0);
        const uint32_t x[4] = {w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16};
#pragma unroll
        for (int j = 0; j < 4; ++j) d.ord[j] = x[j] == 0xFFFFu ? kMissingOrd : x[j];
    } else if (ORD) {
        load_u32x4(P.ord, doc0, d.ord);
    }
    if (HIST && (VK & 4)) {  // the key dimension is a second terms aggregation: u32 ordinals, missing = kMissingOrd
        uint32_t o[4];
        load_u32x4((const uint32_t*)P.hv, doc0, o);
        uint32_t pres = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            d.hv[j] = o[j];
            pres |= (uint32_t)(o[j] < P.H) << j;
        }
        d.hpres = pres;
    } else if (HIST && (VK & 32)) {
        uint32_t o[4];
        load_u32x4(P.hv32, doc0, o);
#pragma unroll
        for (int j = 0; j < 4; ++j) d.hv[j] = P.hv_base + (int64_t)o[j];
        d.hpres = P.hv_present ? bits4(P.hv_present, doc0) : 0xFu;
    } else if (HIST) {
        load_i64x4(P.hv, doc0, d.hv);
        if (VK & 1) {
#pragma unroll
            for (int j = 0; j < 4; ++j) d.hv[j] = java_long(bits_dbl((uint64_t)d.hv[j]));
        }
        d.hpres = P.hv_present ? bits4(P.hv_present, doc0) : 0xFu;
    }
    if (MET > 0 && (VK & 64) && (VK & 256)) {  // packed integer cells over the 16-bit deltas (values span < 2^16)
        const u32x2_t w = load8(P.mv16 + doc0);
        d.mvd[0] = w.x & 0xFFFFu; d.mvd[1] = w.x >> 16; d.mvd[2] = w.y & 0xFFFFu; d.mvd[3] = w.y >> 16;
        d.mpres = 0xFu;
    } else if (MET > 0 && (VK & 64)) {  // packed integer cells: a dense long metric as its compact u32 deltas
        load_u32x4(P.mv32, doc0, d.mvd);
        d.mpres = 0xFu;
    } else if (MET > 0 && (VK & 128)) {  // a long metric read as its compact u32 deltas, the values restored exactly
        uint32_t t[4];
        load_u32x4(P.mv32, doc0, t);
#pragma unroll
        for (int j = 0; j < 4; ++j) d.mv[j] = (double)(P.mv_base + (int64_t)t[j]);  // FieldData.castToDouble of the long
        d.mpres = P.mv_present ? bits4(P.mv_present, doc0) : 0xFu;
    } else if (MET > 0) {
        if (VK & 2) {
            load_f64x4((const double*)P.mv, doc0, d.mv);
        } else {
            int64_t t[4];
            load_i64x4((const int64_t*)P.mv, doc0, t);
#pragma unroll
            for (int j = 0; j < 4; ++j) d.mv[j] = (double)t[j];  // FieldData.castToDouble
        }
        d.mpres = P.mv_present ? bits4(P.mv_present, doc0) : 0xFu;
    }
}

// Packed-cell raw-load kernels with 8 docs per thread per step (ESGPU_DOCS8): one 16-byte load per column for 8 docs
// instead of an 8-byte load per 4, the step's loop, prefetch and zone work shared by twice the docs; processed as two
// Doc4 halves (docs doc0 .. doc0 + 3 and doc0 + 4 .. doc0 + 7)
#ifndef ESGPU_DOCS8  // (r5ab7, 1B docs: north star 1.21 -> 1.19 ms, terms{dh{avg}} 1.09 -> 0.96, config 5 2.36 -> 2.12)
#define ESGPU_DOCS8 1
#endif
#ifndef ESGPU_DOCS8_HI  // ... and the histogram-only integer-run grids over time-sorted data (VK bits 2048 | 4096), whose
#define ESGPU_DOCS8_HI 1  // single-key blocks' packed run updates (CollectParams.dot16): level at 4 waves per SIMD (r6m),
#endif                    // with 6 (ESGPU_HIST_RUNS1_WAVES) config 2 0.622 -> 0.523 ms at 1B (r6ag)
#ifndef ESGPU_DOCS8_H  // ... the raw-load counting grids with a terms dimension (VK bit 1024; r5ab8: terms{date_histogram}
#define ESGPU_DOCS8_H 1  // 0.96 -> 0.88 ms at 1B; the histogram-only grids measured 7 % slower at 8 and keep 4)
#endif
#ifndef ESGPU_B16_BRANCH8  // ... single-key blocks' timestamp loads skipped under a branch, else a dummy load (r5ab8:
#define ESGPU_B16_BRANCH8 1  // north star 1.196 -> 1.165 ms)
#endif
struct Doc8 {
    Doc4 a, b;
};
template <bool ORD, bool HIST, int MET, int VK>
__device__ __forceinline__ void load_docs8(const CollectParams& P, uint32_t doc0, Doc8& d, uint32_t uk = kNoUKey) {
    static_assert(kRawPI<MET, VK, HIST> || kRawH<ORD, MET, VK>, "8 docs per thread: raw-load kernels only");
    d.a.ukey = uk;
    d.b.ukey = uk;
    if constexpr (ORD) {
        const u32x4_t o = load16(P.ord16 + doc0);
        d.a.raw[0] = o.x; d.a.raw[1] = o.y; d.b.raw[0] = o.z; d.b.raw[1] = o.w;
    }
    if constexpr (HIST) {
        if constexpr ((VK & 8192) != 0) {
            bool skip = false;
#if ESGPU_B16_BRANCH8
            skip = uk != kNoUKey;  // a single-key block: no timestamp is read (wave-uniform branch)
#endif
            if (skip) {
                d.a.raw[2] = d.a.raw[3] = d.a.raw[4] = d.a.raw[5] = d.a.raw[10] = 0u;
                d.b.raw[2] = d.b.raw[3] = d.b.raw[4] = d.b.raw[5] = d.b.raw[10] = 0u;
            } else {
                const u32x4_t t = load16(P.hv16 + (uk == kNoUKey ? doc0 : 0u));
                const u32x2_t bs = load8(P.hv16_base + (doc0 >> kB16Shift));  // (8 docs never straddle a run)
                const u32x2_t h = load8(P.hv8 + (doc0 & P.hv8_mask));          // (see load_keys_raw)
                d.a.raw[2] = t.x; d.a.raw[3] = t.y; d.b.raw[2] = t.z; d.b.raw[3] = t.w;
                d.a.raw[10] = h.x; d.b.raw[10] = h.y;
                d.a.raw[4] = bs.x; d.a.raw[5] = bs.y; d.b.raw[4] = bs.x; d.b.raw[5] = bs.y;
            }
        } else {
            bool skip = false;
            if constexpr ((VK & 16384) != 0) skip = uk != kNoUKey;  // a single-key block (VK bit 16384): no delta read
            if (skip) {
                d.a.raw[2] = d.a.raw[3] = d.a.raw[4] = d.a.raw[5] = 0u;
                d.b.raw[2] = d.b.raw[3] = d.b.raw[4] = d.b.raw[5] = 0u;
            } else {
                const u32x4_t t0 = load16(P.hv32 + doc0), t1 = load16(P.hv32 + doc0 + 4);
                d.a.raw[2] = t0.x; d.a.raw[3] = t0.y; d.a.raw[4] = t0.z; d.a.raw[5] = t0.w;
                d.b.raw[2] = t1.x; d.b.raw[3] = t1.y; d.b.raw[4] = t1.z; d.b.raw[5] = t1.w;
            }
        }
    }
    if constexpr (MET > 0 && (kRawPI<MET, VK, HIST> || (VK & 2048) != 0)) {  // 16-bit metric deltas
        const u32x4_t m = load16(P.mv16 + doc0);
        d.a.raw[6] = m.x; d.a.raw[7] = m.y; d.b.raw[6] = m.z; d.b.raw[7] = m.w;
    } else if constexpr (MET > 0) {  // u32 metric deltas
        const u32x4_t m0 = load16(P.mv32 + doc0), m1 = load16(P.mv32 + doc0 + 4);
        d.a.raw[6] = m0.x; d.a.raw[7] = m0.y; d.a.raw[8] = m0.z; d.a.raw[9] = m0.w;
        d.b.raw[6] = m1.x; d.b.raw[7] = m1.y; d.b.raw[8] = m1.z; d.b.raw[9] = m1.w;
    }
    if constexpr (kRawPI<MET, VK, HIST> && (VK & 512) != 0) {  // (both halves in one 64-doc word)
        d.a.racc = P.accept[doc0 >> 6];
        d.b.racc = d.a.racc;
    }
    d.a.doc0 = doc0;
    d.b.doc0 = doc0 + 4;
}

// Accumulator views: either the workgroup's LDS window or the global cell grid.
struct Acc {
    uint32_t* cnt32;                // LDS
    unsigned long long* cnt64;      // global
    uint32_t* vcnt32;
    unsigned long long* vcnt64;
    double* sum;
    unsigned long long* mn;         // LDS min / max: interleaved (mx == mn + 1, stride 2) or two arrays (stride 1)
    unsigned long long* mx;
    double* sq;
    uint32_t* ocnt32;
    unsigned long long* ocnt64;
    uint32_t mstride;               // LDS min/max stride; 1 in the global grid
    uint32_t coff;                  // this lane's copy of the additive LDS cells (CollectParams.ncopies); 0 in the grid
    unsigned long long* pk;         // LDS, packed integer cells (VK bit 64): count << pk_shift | sum of deltas [C][ncopies]
    uint32_t* mm;                   // LDS, packed integer cells: (min, max) delta pair per cell [C][2]
    unsigned long long* pkd;        // LDS, packed integer cells: this thread's spare word (the adds of docs that hit nothing)
    double* sum_lo;                 // global, compensated sums (CollectParams.g_sum_lo): null = plain
    double* sq_lo;
};

// Compensated accumulation into the global grid (DESIGN §5 "Float parity"): the grid word is the high part of a
// double-double and `lo` collects every addition's rounding error.  The returning atomic yields the value it added to,
// so the error of that addition is TwoSum's -- exact as long as the atomic rounds like a VALU add (round to nearest
// even, subnormals kept: tools/fpatomic_probe.hip on gfx950).  `xl` is the addend's own low part (a double-double
// addend); a non-finite sum carries no error term (Inf / NaN propagate through the high part alone, as in Java).
__device__ __forceinline__ void dd_atomic_add(double* hi, double* lo, double x, double xl = 0.0) {
    if (!lo) {
        atomicAdd(hi, x);
        return;
    }
    const double old = atomicAdd(hi, x);
    const double s = old + x;
    const double bp = s - old;
    const double e = ((old - (s - bp)) + (x - bp)) + xl;
    if (e != 0.0 && __builtin_isfinite(s)) atomicAdd(lo, e);
}
// an exact long as a double-double (its high and low 32 bits are exact doubles; TwoSum of them)
__device__ __forceinline__ void i64_to_dd(long long v, double& hi, double& lo) {
    const double a = (double)(v >> 32) * 4294967296.0, b = (double)(unsigned long long)(v & 0xFFFFFFFFll);
    hi = a + b;
    const double bp = hi - a;
    lo = (a - (hi - bp)) + (b - bp);
}

template <int MET, bool LDS, int MS>
__device__ __forceinline__ void add_value(const Acc& a, uint32_t c, double x, bool has_vcnt) {
    const uint32_t ca = LDS ? c + a.coff : c;  // additive cell (lane copy)
    if (LDS) {
        if (has_vcnt) atomicAdd(&a.vcnt32[ca], 1u);
    } else {
        if (has_vcnt) atomicAdd(&a.vcnt64[c], 1ull);
    }
    if (LDS) atomicAdd(&a.sum[ca], x);
    else dd_atomic_add(&a.sum[c], a.sum_lo ? a.sum_lo + c : nullptr, x);
    if (MET >= 2) {
        const bool nan = x != x;
        const unsigned long long e = sortable(x);
        const unsigned long long emn = nan ? 0ull : e;
        const unsigned long long emx = nan ? ~0ull : e;
        // read-check before the atomic: reads of one address broadcast, and min/max converge quickly
        // (ESGPU_MINMAX_CHECK=0: unconditional no-return atomics -- no LDS read to wait on -- for A/B runs)
        constexpr uint32_t st = LDS ? MS : 1;
#if ESGPU_MINMAX_CHECK
        const unsigned long long cmn = a.mn[c * st], cmx = a.mx[c * st];
        if (emn < cmn) atomicMin(&a.mn[c * st], emn);
        if (emx > cmx) atomicMax(&a.mx[c * st], emx);
#else
        atomicMin(&a.mn[c * st], emn);
        atomicMax(&a.mx[c * st], emx);
#endif
    }
    if (MET >= 3) {  // ExtendedStatsAggregator: sumOfSqr += value * value (no FMA)
        if (LDS) atomicAdd(&a.sq[ca], x * x);
        else dd_atomic_add(&a.sq[c], a.sq_lo ? a.sq_lo + c : nullptr, x * x);
    }
}

// Per-doc update.  `slot` is the key index relative to the accumulator's first slot (window or grid).
// `outer` = false in the extra passes over a multi-pass block (its docs' terms were counted in the first pass).
template <bool ORD, bool HIST, int MET, bool LDS, int MS>
__device__ __forceinline__ void update_doc(const CollectParams& P, const Acc& a, uint32_t T, bool has_t, uint32_t t,
                                           bool has_h, uint32_t slot, bool mpres, double x, bool outer) {
    if (P.ocnt_mode == OCNT_TERMS) {
        if (has_t && outer) {
            if (LDS) atomicAdd(&a.ocnt32[t], 1u); else atomicAdd(&a.ocnt64[t], 1ull);
        }
    } else if (!LDS && P.ocnt_mode == OCNT_TERMS_DERIVED && has_t && has_h) {
        atomicAdd(&a.ocnt64[t], 1ull);
    } else if (P.ocnt_mode == OCNT_HIST && has_h) {
        if (LDS) atomicAdd(&a.ocnt32[slot], 1u); else atomicAdd(&a.ocnt64[slot], 1ull);
    }
    if (!(has_t && has_h)) return;
    const uint32_t c = slot * T + t;
    if (LDS) atomicAdd(&a.cnt32[c + a.coff], 1u); else atomicAdd(&a.cnt64[c], 1ull);
    if (MET > 0 && mpres) add_value<MET, LDS, MS>(a, c, x, P.vcnt_mode != 0);
}

// Wave-level pre-aggregation for a cell shared by the whole wave (time-sorted data without a terms dimension):
// one LDS atomic per quantity per wave instead of 256 conflicting ones.
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

// grid key index of a value: affine roundings divide, table roundings (calendar units, DST zones) search the bucket
// start instants; values outside the grid give an index outside [0, H)
template <bool KT>
__device__ __forceinline__ int64_t key_index(const CollectParams& P, int64_t v) {
    if (!KT) return floor_div64(v - P.offset, P.interval) - P.key0;
    if (v < P.kstart[0]) return -1;
    uint32_t lo = 0, hi = P.nsteps;  // kstart[lo] <= v < kstart[hi] (kstart[nsteps] = +inf)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (P.kstart[mid] <= v) lo = mid; else hi = mid;
    }
    return P.kslot ? P.kslot[lo] : lo;
}

// key slot of a value relative to `base` (= value of the first slot); 32-bit magic division fast path
__device__ __forceinline__ uint32_t slot_of(const CollectParams& P, int64_t v, int64_t base) {
    if (P.fast32) return magic_div((uint32_t)((uint64_t)v - (uint64_t)base), P.mg_m, P.mg_s1, P.mg_s2, (uint32_t)P.interval);
    return (uint32_t)(floor_div64(v - P.offset, P.interval) - floor_div64(base - P.offset, P.interval));
}

// Per-thread run accumulator for histogram-only plans over time-sorted data: a thread's consecutive docs share a
// key slot, so their count / sum / min / max / sum-of-squares are combined in registers and reach LDS only when
// the slot changes (an hour boundary) or at a window flush -- no per-doc LDS traffic.
struct Run {
    uint32_t slot;  // 0xFFFFFFFF = empty
    uint32_t cnt, vc;
    double sum, sq;
    unsigned long long mn, mx;
    // integer runs (kIntRuns): sum of deltas, sum of squared deltas, min / max delta (a thread's run holds at most one
    // workgroup range of docs, < 2^19: the sums cannot overflow)
    uint32_t isd, imn, imx;
    unsigned long long isq;
    uint32_t pmn, pmx;  // ... and the extrema of the packed updates (runs_add_pk) as two 16-bit lanes each
};

__device__ __forceinline__ void run_reset(Run& r) {
    r.slot = 0xFFFFFFFFu;
    r.cnt = 0;
    r.vc = 0;
    r.sum = 0.0;
    r.sq = 0.0;
    r.mn = kMinInit;
    r.mx = kMaxInit;
    r.isd = 0;
    r.isq = 0;
    r.imn = ~0u;
    r.imx = 0;
    r.pmn = ~0u;
    r.pmx = 0;
}

// an integer run into its LDS cell: the values are v = mv_base + d, so sum = cnt * base + sum d and sum of squares =
// cnt * base^2 + 2 * base * sum d + sum d^2 -- exact in 128 bits, one rounding to double (exact while the request's sums
// stay below 2^53, the plan's compensated flushes past it); extrema are the casts of base + the delta extrema
template <int MET, int MS>
__device__ __forceinline__ void run_flush_i(const CollectParams& P, const Acc& a, Run& r) {
    if (r.slot != 0xFFFFFFFFu) {
        const uint32_t c = r.slot;
        atomicAdd(&a.cnt32[c], r.cnt);
        const long long base = P.mv_base;
        atomicAdd(&a.sum[c], (double)((long long)r.cnt * base + (long long)r.isd));
        if (MET >= 2) {
            const uint32_t imn = min(r.imn, min(r.pmn & 0xFFFFu, r.pmn >> 16));
            const uint32_t imx = max(r.imx, max(r.pmx & 0xFFFFu, r.pmx >> 16));
            const unsigned long long emn = sortable((double)(base + (long long)imn));
            const unsigned long long emx = sortable((double)(base + (long long)imx));
            const unsigned long long cmn = a.mn[MS * c], cmx = a.mx[MS * c];
            if (emn < cmn) atomicMin(&a.mn[MS * c], emn);
            if (emx > cmx) atomicMax(&a.mx[MS * c], emx);
        }
        if (MET >= 3) {
            const __int128 b = base;
            const __int128 q = (__int128)r.cnt * b * b + 2 * b * (__int128)r.isd + (__int128)r.isq;
            atomicAdd(&a.sq[c], (double)q);
        }
    }
    run_reset(r);
}

template <int MET, int MS>
__device__ __forceinline__ void run_flush(const CollectParams& P, const Acc& a, Run& r) {
    if (r.slot != 0xFFFFFFFFu) {
        const uint32_t c = r.slot;  // T == 1: cell == slot
        atomicAdd(&a.cnt32[c], r.cnt);
        if (MET > 0 && r.vc) {
            if (P.vcnt_mode) atomicAdd(&a.vcnt32[c], r.vc);
            atomicAdd(&a.sum[c], r.sum);
            if (MET >= 2) {
                const unsigned long long cmn = a.mn[MS * c], cmx = a.mx[MS * c];  // LDS
                if (r.mn < cmn) atomicMin(&a.mn[MS * c], r.mn);
                if (r.mx > cmx) atomicMax(&a.mx[MS * c], r.mx);
            }
            if (MET >= 3) atomicAdd(&a.sq[c], r.sq);
        }
    }
    run_reset(r);
}

// Several run accumulators per thread (runs_for<MET>): roughly time-ordered data (a doc displaced by up to an hour) alternates between
// neighbouring keys, which a single run would flush to LDS on almost every doc (conflicting LDS atomics on ~3
// addresses per wave).  A miss replaces the runs round-robin.
#ifndef ESGPU_RUNS  // run accumulators with a metric (measured: 3 takes config 2 at +-1 h jitter from 4.6 to 3.0 ms)
#define ESGPU_RUNS 3
#endif
// counting only (MET 0): one run -- a count flush is a single LDS add, and the run array would go to scratch
#ifndef ESGPU_INT_RUNS_NR  // integer run accumulators (VK bit 2048) per thread
#define ESGPU_INT_RUNS_NR 3
#endif
// VK bit 4096 (with 2048): time-sorted data (a block's keys span less than one interval: CollectParams.runs1) -- one integer
// run per thread, a third of the registers and no run lookup (config 2 at 1B docs: 1.46 -> 1.12 ms, r5d)
// Integer runs over roughly time-ordered data (VK bit 2048 without 4096): the docs go to four window accumulators per
// thread instead of three runs (ESGPU_WIN4=0: the runs, for A/B) -- see win_add
#ifndef ESGPU_WIN4
#define ESGPU_WIN4 1
#endif
template <int MET, int VK> constexpr bool kWin4 = ESGPU_WIN4 != 0 && MET > 0 && (VK & 2048) != 0 && (VK & 4096) == 0;
#ifndef ESGPU_WIN_MK  // ... and the multi-key zone blocks of the one-run grids with single-key blocks (kWinMK): off --
#define ESGPU_WIN_MK 0  // the accumulators' registers spill those kernels at 6 waves per SIMD (config 2 sorted 0.53 ->
#endif                  // 3.66 ms with four slots, r6aw; 2.59 ms with two, r6ay)
template <bool ORD, bool HIST, int MET, int VK>
constexpr bool kWinMK = ESGPU_WIN_MK != 0 && !ORD && MET > 0 && (VK & 2048) != 0 && (VK & 4096) != 0 &&
                        kUKeyK<ORD, HIST, MET, VK>;
#ifndef ESGPU_WIN_MK_SLOTS  // key slots of the multi-key-block windows (kWinMK): 2 (an hour boundary inside a block)
#define ESGPU_WIN_MK_SLOTS 2
#endif
template <bool ORD, bool HIST, int MET, int VK>
constexpr int kWinSlots = kWinMK<ORD, HIST, MET, VK> ? ESGPU_WIN_MK_SLOTS : 4;
template <int MET, int VK = 0> constexpr int runs_for() {
    return MET == 0 ? 1 : (VK & 4096) != 0 ? 1 : kWin4<MET, VK> ? 1 : (VK & 2048) != 0 ? ESGPU_INT_RUNS_NR : ESGPU_RUNS;
}
#ifndef ESGPU_PI_NHOT  // hot ordinals with register runs in the packed-cell kernels (CollectParams.hot_t, up to 4)
#define ESGPU_PI_NHOT 1
#endif
constexpr int kNHot = ESGPU_PI_NHOT;
template <int NR>
struct Runs {
    Run r[NR];
    uint32_t victim;
    // packed integer cells (VK bit 64): the segment's most frequent ordinals (CollectParams.hot_t) accumulated in
    // registers for the current key slot -- the Zipf head's docs leave the LDS atomics, whose same-address conflicts they
    // caused (ESGPU_PI_HOTU in the uniform-key path, ESGPU_PI_HOT per doc)
    uint32_t hslot, hlo[kNHot], hhi[kNHot];
    uint32_t hcnt[kNHot], hsum[kNHot];  // docs and their delta sum (a lane holds < 65,536 docs of a workgroup range)
    // window accumulators (kWin4): key slots wb .. wb + 3 -- per slot the docs, delta sum and squared-delta sum, and the
    // delta extrema as 16-bit pairs (slots 0/1 in wmn[0] / wmx[0], 2/3 in [1]); wb = kWinEmpty: none
    uint32_t wb, wc[4], ws[4], wmn[2], wmx[2];
    unsigned long long wq[4];
};
constexpr uint32_t kWinEmpty = 0x80000000u;  // (slots are < 2^31: slot - kWinEmpty is never a window offset)
template <int NR>
__device__ __forceinline__ void runs_reset(Runs<NR>& R) {
#pragma unroll
    for (int k = 0; k < NR; ++k) run_reset(R.r[k]);
    R.victim = 0;
    R.hslot = ~0u;
    R.wb = kWinEmpty;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        R.wc[k] = 0u;
        R.ws[k] = 0u;
        R.wq[k] = 0ull;
    }
    R.wmn[0] = R.wmn[1] = ~0u;
    R.wmx[0] = R.wmx[1] = 0u;
#pragma unroll
    for (int k = 0; k < kNHot; ++k) {
        R.hlo[k] = ~0u;
        R.hhi[k] = 0u;
        R.hcnt[k] = 0u;
        R.hsum[k] = 0u;
    }
}
#ifndef ESGPU_PI_HOT
#define ESGPU_PI_HOT 0
#endif
#ifndef ESGPU_PI_MMCHECK  // packed cells: (min, max) pairs read first, atomics only where they change -- 2: one divergent
                          // region per doc (NS 1.324 -> 1.29 ms, r5ab3), 1: one per bound, 0: unconditional (1.9x slower)
#define ESGPU_PI_MMCHECK 2
#endif
#ifndef ESGPU_PI_NOATOM
#define ESGPU_PI_NOATOM 0
#endif
#ifndef ESGPU_PI_STRAIGHT  // packed cells: straight-line reads and adds (1), or under the hit mask (0, for A/B runs)
#define ESGPU_PI_STRAIGHT 1
#endif
// the hot ordinal's run into its LDS cell (before a window moves, and at the end)
template <int MET, int NR>
__device__ __forceinline__ void pi_hot_flush(const CollectParams& P, const Acc& a, Runs<NR>& R, uint32_t T) {
#pragma unroll
    for (int k = 0; k < kNHot; ++k) {
        if (R.hslot != ~0u && R.hcnt[k]) {
            const uint32_t c = R.hslot * T + P.hot_t[k];
            atomicAdd(&a.pk[c + a.coff], ((unsigned long long)R.hcnt[k] << P.pk_shift) + R.hsum[k]);
            if (MET >= 2) {
                if (R.hlo[k] < a.mm[2 * c]) atomicMin(&a.mm[2 * c], R.hlo[k]);
                if (R.hhi[k] > a.mm[2 * c + 1]) atomicMax(&a.mm[2 * c + 1], R.hhi[k]);
            }
        }
        R.hlo[k] = ~0u;
        R.hhi[k] = 0u;
        R.hcnt[k] = 0u;
        R.hsum[k] = 0u;
    }
    R.hslot = ~0u;
}
// the window accumulators into their LDS cells (each slot with docs as one integer run), then emptied
template <int MET, int MS, int NR, int S = 4>
__device__ __forceinline__ void win_flush(const CollectParams& P, const Acc& a, Runs<NR>& R) {
#pragma unroll
    for (int k = 0; k < S; ++k) {
        if (R.wc[k]) {
            Run r;
            run_reset(r);
            r.slot = R.wb + (uint32_t)k;
            r.cnt = R.wc[k];
            r.isd = R.ws[k];
            r.isq = R.wq[k];
            r.imn = (R.wmn[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
            r.imx = (R.wmx[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
            run_flush_i<MET, MS>(P, a, r);
        }
        R.wc[k] = 0u;
        R.ws[k] = 0u;
        R.wq[k] = 0ull;
    }
    R.wmn[0] = R.wmn[1] = ~0u;
    R.wmx[0] = R.wmx[1] = 0u;
    R.wb = kWinEmpty;
}
template <int MET, int MS, int NR, bool INT = false, bool WIN = false, int WS = 4>
__device__ __forceinline__ void runs_flush(const CollectParams& P, const Acc& a, Runs<NR>& R) {
    if constexpr (WIN) win_flush<MET, MS, NR, WS>(P, a, R);
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        if constexpr (INT) run_flush_i<MET, MS>(P, a, R.r[k]);
        else run_flush<MET, MS>(P, a, R.r[k]);
    }
}
// n docs of one key slot into the integer run of `slot` (n = 1: one doc; 4: a thread's 4 docs that share the slot,
// combined first): sd / sq / mn / mx are the docs' delta sum, squared-delta sum and extrema
template <int MET, int MS, int NR>
__device__ __forceinline__ void runs_add_i(const CollectParams& P, const Acc& a, Runs<NR>& R, uint32_t slot, uint32_t n,
                                           uint32_t sd, unsigned long long sq, uint32_t mn, uint32_t mx) {
    int hit = -1;
#pragma unroll
    for (int k = 0; k < NR; ++k) hit = R.r[k].slot == slot ? k : hit;
    if (hit < 0) {
        hit = NR == 1 ? 0 : (int)R.victim;
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (k == hit) {
                run_flush_i<MET, MS>(P, a, R.r[k]);
                R.r[k].slot = slot;
            }
        if (NR > 1) R.victim = R.victim + 1 == (uint32_t)NR ? 0u : R.victim + 1;
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const bool h = hit == k;
        R.r[k].cnt += h ? n : 0u;
        R.r[k].isd += h ? sd : 0u;
        if (MET >= 3) R.r[k].isq += h ? sq : 0ull;
        if (MET >= 2) {
            R.r[k].imn = h && mn < R.r[k].imn ? mn : R.r[k].imn;
            R.r[k].imx = h && mx > R.r[k].imx ? mx : R.r[k].imx;
        }
    }
}
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
// a thread's 4 docs of a single-key zone block into its one integer run, straight from the two raw words of 16-bit
// metric deltas: v_dot2_u32_u16 sums the deltas (and, below 46,341, their squares: CollectParams.dot16), v_pk_min/max_u16
// keep two extrema per word until the flush -- 9 VALU per 4 docs where unpacked they took ~25
template <int MET, int MS, int NR>
__device__ __forceinline__ void runs_add_pk(const CollectParams& P, const Acc& a, Runs<NR>& R, uint32_t slot, uint32_t w0,
                                            uint32_t w1) {
    static_assert(NR == 1, "one run per thread (VK bit 4096)");
    Run& r = R.r[0];
    if (r.slot != slot) {
        run_flush_i<MET, MS>(P, a, r);
        r.slot = slot;
    }
    const u16x2_t x0 = __builtin_bit_cast(u16x2_t, w0), x1 = __builtin_bit_cast(u16x2_t, w1);
    const u16x2_t one = {1, 1};
    r.cnt += 4u;
    r.isd = __builtin_amdgcn_udot2(x0, one, __builtin_amdgcn_udot2(x1, one, r.isd, false), false);
    if (MET >= 3)
        r.isq += (unsigned long long)__builtin_amdgcn_udot2(x0, x0, 0u, false) +
                 (unsigned long long)__builtin_amdgcn_udot2(x1, x1, 0u, false);
    if (MET >= 2) {
        r.pmn = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2_t, r.pmn),
                                                                        __builtin_elementwise_min(x0, x1)));
        r.pmx = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, r.pmx),
                                                                        __builtin_elementwise_max(x0, x1)));
    }
}
// one doc (v: it passes and has a key) into window slot o = slot - wb (o < 4 when v): the slot's 0/1 weight e multiplies
// the delta into each sum (v_mad), so a doc costs ~30 VALU where the three runs' hit search and predicated updates took
// ~110 (config 2 at ±1 h, SQ counters r6ac: 446 VALU per wave per 256 docs)
template <int MET, int NR, int S = 4>
__device__ __forceinline__ void win_add(Runs<NR>& R, uint32_t o, uint32_t x, bool v) {
    const uint32_t oh = v ? 1u << ((o & 3u) << 3) : 0u;  // one-hot byte of the slot
    const uint32_t xx = x * x;                              // (x < 2^16)
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const uint32_t e = (oh >> (8 * k)) & 0xFFu;
        R.wc[k] += e;
        R.ws[k] += x * e;
        if (MET >= 3) R.wq[k] += (unsigned long long)xx * e;
    }
    if (MET >= 2) {
        const uint32_t sh = (o & 1u) << 4;
        const uint32_t xm = (x << sh) | (0xFFFF0000u >> sh), xM = x << sh;  // the other half: min / max identities
        const bool h0 = v && o < 2u, h1 = S > 2 && v && o >= 2u;
        const u16x2_t m = __builtin_bit_cast(u16x2_t, xm), M = __builtin_bit_cast(u16x2_t, xM);
        const uint32_t n0 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2_t, R.wmn[0]), m));
        const uint32_t n1 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2_t, R.wmn[1]), m));
        const uint32_t x0 = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, R.wmx[0]), M));
        const uint32_t x1 = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, R.wmx[1]), M));
        R.wmn[0] = h0 ? n0 : R.wmn[0];
        R.wmn[1] = h1 ? n1 : R.wmn[1];
        R.wmx[0] = h0 ? x0 : R.wmx[0];
        R.wmx[1] = h1 ? x1 : R.wmx[1];
    }
}
// a doc whose slot is outside the window: flush it and re-base -- new keys above put the slot at the top (the keys of
// roughly time-ordered data drift upwards), below at the bottom, a first doc one above the bottom
template <int MET, int MS, int NR, int S = 4>
__device__ __forceinline__ void win_rebase(const CollectParams& P, const Acc& a, Runs<NR>& R, uint32_t slot) {
    const uint32_t old = R.wb;
    win_flush<MET, MS, NR, S>(P, a, R);
    constexpr uint32_t top = S - 1;
    R.wb = old == kWinEmpty ? (S > 2 && slot ? slot - 1u : slot) : slot > old ? (slot >= top ? slot - top : 0u) : slot;
}
template <int MET, int MS, int NR>
__device__ __forceinline__ void runs_add(const CollectParams& P, const Acc& a, Runs<NR>& R, uint32_t slot, bool mpres, double x) {
    int hit = -1;
#pragma unroll
    for (int k = 0; k < NR; ++k) hit = R.r[k].slot == slot ? k : hit;
    if (hit < 0) {
        hit = NR == 1 ? 0 : (int)R.victim;
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (k == hit) {
                run_flush<MET, MS>(P, a, R.r[k]);
                R.r[k].slot = slot;
            }
        if (NR > 1) R.victim = R.victim + 1 == (uint32_t)NR ? 0u : R.victim + 1;
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        if (k != hit) continue;
        Run& run = R.r[k];
        ++run.cnt;
        if (MET > 0 && mpres) {
            ++run.vc;
            run.sum += x;
            if (MET >= 3) run.sq += x * x;
            if (MET >= 2) {
                const bool nan = x != x;
                const unsigned long long e = sortable(x);
                const unsigned long long emn = nan ? 0ull : e, emx = nan ? ~0ull : e;
                run.mn = emn < run.mn ? emn : run.mn;
                run.mx = emx > run.mx ? emx : run.mx;
            }
        }
    }
}

// n docs at once into the run of `slot` (a thread's 4 docs that share a key slot, combined in registers first): the run
// lookup and its predicated per-run updates once per 4 docs instead of once per doc
template <int MET, int MS, int NR>
__device__ __forceinline__ void runs_add_n(const CollectParams& P, const Acc& a, Runs<NR>& R, uint32_t slot, uint32_t n,
                                           uint32_t vc, double sum, double sq, unsigned long long mn, unsigned long long mx) {
    int hit = -1;
#pragma unroll
    for (int k = 0; k < NR; ++k) hit = R.r[k].slot == slot ? k : hit;
    if (hit < 0) {
        hit = NR == 1 ? 0 : (int)R.victim;
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (k == hit) {
                run_flush<MET, MS>(P, a, R.r[k]);
                R.r[k].slot = slot;
            }
        if (NR > 1) R.victim = R.victim + 1 == (uint32_t)NR ? 0u : R.victim + 1;
    }
    // the hit run's fields selected into registers, updated once, and selected back (indexing R.r by `hit`, or
    // updating under `k == hit`, lets the compiler turn the runs into a dynamically indexed array in scratch)
    Run c = R.r[0];
#pragma unroll
    for (int k = 1; k < NR; ++k) {
        const bool h = hit == k;
        c.cnt = h ? R.r[k].cnt : c.cnt;
        c.vc = h ? R.r[k].vc : c.vc;
        c.sum = h ? R.r[k].sum : c.sum;
        c.sq = h ? R.r[k].sq : c.sq;
        c.mn = h ? R.r[k].mn : c.mn;
        c.mx = h ? R.r[k].mx : c.mx;
    }
    c.cnt += n;
    if (MET > 0) {
        c.vc += vc;
        c.sum += sum;
        if (MET >= 3) c.sq += sq;
        if (MET >= 2) {
            c.mn = mn < c.mn ? mn : c.mn;
            c.mx = mx > c.mx ? mx : c.mx;
        }
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const bool h = hit == k;
        R.r[k].cnt = h ? c.cnt : R.r[k].cnt;
        if (MET > 0) {
            R.r[k].vc = h ? c.vc : R.r[k].vc;
            R.r[k].sum = h ? c.sum : R.r[k].sum;
            if (MET >= 3) R.r[k].sq = h ? c.sq : R.r[k].sq;
            if (MET >= 2) {
                R.r[k].mn = h ? c.mn : R.r[k].mn;
                R.r[k].mx = h ? c.mx : R.r[k].mx;
            }
        }
    }
}
#ifndef ESGPU_RUN4  // histogram-only grids: a thread's 4 docs with one key slot combined before the run update; measured
#define ESGPU_RUN4 0  // slower (config 2 at 1B docs 2.15 -> 2.62 ms, date_histogram 1.03 -> 1.14 ms): off, kept for A/B
#endif

#ifndef ESGPU_ORDH_HOT  // counting ORD x histogram raw-load grids: the segment's most frequent ordinal counted in a
#define ESGPU_ORDH_HOT 0  // register in single-key zone blocks (cnt_hot_flush), its docs off the LDS atomics -- measured
#endif                    // slower (terms{date_histogram} 0.885 -> 1.046 ms at 1B, r6am): A/B option, off
#ifndef ESGPU_COMBINE4  // counting ORD x histogram grids: combine a thread's equal keys before the LDS atomics
#define ESGPU_COMBINE4 1
#endif
// calls emit(key, multiplicity) once per distinct key of k[0..3] (~0u = none)
template <class F>
__device__ __forceinline__ void combine4(uint32_t (&k)[kVec], F emit) {
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
        if (k[j] == ~0u) continue;
        uint32_t n = 1;
#pragma unroll
        for (int i = j + 1; i < kVec; ++i)
            if (k[i] == k[j]) { ++n; k[i] = ~0u; }
        emit(k[j], n);
    }
}

// kRawPI: the raw words of a buffer turned into the docs' fields (ordinals, key values, metric deltas, pass mask)
template <bool HIST, int MET, int VK>
__device__ __forceinline__ void unpack_docs(const CollectParams& P, Doc4& d) {
    const uint32_t doc0 = d.doc0;
    uint32_t ok = doc0 + 4 <= P.n_docs ? 0xFu : doc0 >= P.n_docs ? 0u : ((1u << (P.n_docs - doc0)) - 1u);
    if constexpr ((VK & 512) != 0) ok &= (uint32_t)(d.racc >> (doc0 & 63)) & 0xFu;
    d.ok = ok;
    // a missing ordinal stays 0xFFFF: the packed-cell path tests t < T, and a 16-bit ordinal column exists only while T
    // is below 0xFFFF
    d.ord[0] = d.raw[0] & 0xFFFFu; d.ord[1] = d.raw[0] >> 16; d.ord[2] = d.raw[1] & 0xFFFFu; d.ord[3] = d.raw[1] >> 16;
    if constexpr (HIST) {
        if (d.ukey == kNoUKey) unpack_keys_raw<VK>(P, d.raw, d.hv);  // (zone_ukey: kNoUKey on the other kernels)
        d.hpres = 0xFu;
    }
    d.mvd[0] = d.raw[6] & 0xFFFFu; d.mvd[1] = d.raw[6] >> 16; d.mvd[2] = d.raw[7] & 0xFFFFu; d.mvd[3] = d.raw[7] >> 16;
    d.mpres = 0xFu;
}

// counting ORD x histogram raw-load grids with single-key zone blocks: the hot ordinal's register count (ESGPU_ORDH_HOT)
template <bool ORD, bool HIST, int MET, int VK>
constexpr bool kOrdHHot = ESGPU_ORDH_HOT != 0 && ORD && HIST && MET == 0 && kUKeyK<ORD, HIST, MET, VK>;
template <int NR>
__device__ __forceinline__ void cnt_hot_flush(const Acc& a, Runs<NR>& R, uint32_t T, uint32_t ht) {
    if (R.hslot != ~0u && R.hcnt[0]) atomicAdd(&a.cnt32[R.hslot * T + ht + a.coff], R.hcnt[0]);
    R.hcnt[0] = 0u;
    R.hslot = ~0u;
}
template <bool ORD, bool HIST, int MET, bool LDS, bool KT, int MS, bool HORD = false, int VK = 0>
__device__ __forceinline__ void process4(const CollectParams& P, const Acc& a, const Doc4& d_in, uint32_t T, int64_t base,
                                         uint32_t win0, Runs<runs_for<MET, VK>()>& run, uint32_t mw = 0, bool outer = true) {
    if constexpr (LDS && kIntRuns<ORD, MET, VK> && kUKeyK<ORD, HIST, MET, VK> && (VK & 4096) != 0) {
        // a single-key zone block's whole quad (every doc but the segment's last few): the packed run update, no unpack
        if (d_in.ukey != kNoUKey && P.dot16 && d_in.doc0 + 4 <= P.n_docs) {
            const uint32_t k = d_in.ukey, sl = k - win0;  // (kOutUKey: outside the grid, no doc counts)
            if (k < P.H && sl < (mw ? mw : P.W)) runs_add_pk<MET, MS>(P, a, run, sl, d_in.raw[6], d_in.raw[7]);
            return;
        }
    }
    Doc4 du;
    if constexpr (kRawPI<MET, VK, HIST>) {
        du = d_in;
        unpack_docs<HIST, MET, VK>(P, du);
    } else if constexpr (kRawH<ORD, MET, VK>) {
        du = d_in;
        const uint32_t doc0 = du.doc0;
        du.ok = doc0 + 4 <= P.n_docs ? 0xFu : doc0 >= P.n_docs ? 0u : ((1u << (P.n_docs - doc0)) - 1u);
        if constexpr (ORD) {
            const uint32_t x[4] = {du.raw[0] & 0xFFFFu, du.raw[0] >> 16, du.raw[1] & 0xFFFFu, du.raw[1] >> 16};
#pragma unroll
            for (int j = 0; j < 4; ++j) du.ord[j] = x[j] == 0xFFFFu ? kMissingOrd : x[j];
        }
        if constexpr (HIST) {
            if (du.ukey == kNoUKey) unpack_keys_raw<VK>(P, du.raw, du.hv);
            du.hpres = 0xFu;
        }
        if constexpr (MET > 0 && (VK & 2048) != 0) {  // integer runs: the 16-bit deltas as they are
            du.mvd[0] = du.raw[6] & 0xFFFFu; du.mvd[1] = du.raw[6] >> 16; du.mvd[2] = du.raw[7] & 0xFFFFu; du.mvd[3] = du.raw[7] >> 16;
            du.mpres = 0xFu;
        } else if constexpr (MET > 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) du.mv[j] = (double)(P.mv_base + (int64_t)du.raw[6 + j]);  // FieldData.castToDouble of the long
            du.mpres = 0xFu;
        }
    }
    const Doc4& d = kRawPI<MET, VK, HIST> || kRawH<ORD, MET, VK> ? du : d_in;
    uint32_t slot[kVec];
    bool hv_ok[kVec];
    // raw-load kernels over block deltas or 32-bit deltas: a zone block whose docs all share one key takes it for every
    // doc (wave-uniform branch)
    const bool ublock = kUKeyK<ORD, HIST, MET, VK> && d.ukey != kNoUKey;
    if (ublock) {
        const uint32_t k = d.ukey;  // grid key index, or kOutUKey (outside the grid: no doc counts)
        const uint32_t sl = LDS ? k - win0 : k;
        const bool in = k < P.H && (!LDS || sl < (mw ? mw : P.W));
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
            slot[j] = sl;
            hv_ok[j] = in;
        }
    }
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
        if (ublock) break;
        hv_ok[j] = true;
        slot[j] = 0;
        if (HIST && HORD) {  // ordinal keys: the slot is the ordinal (never windowed)
            hv_ok[j] = (d.hpres >> j) & 1;
            slot[j] = (uint32_t)d.hv[j];
        } else if (HIST) {
            hv_ok[j] = (d.hpres >> j) & 1;
            if (LDS) {
                if (KT) {
                    const int64_t k = key_index<KT>(P, d.hv[j]) - (int64_t)win0;
                    slot[j] = (uint32_t)k;
                    if (mw) hv_ok[j] = hv_ok[j] && k >= 0 && k < (int64_t)mw;
                } else {
                    slot[j] = slot_of(P, d.hv[j], base);
                    // 64-bit range test: slot_of's 32-bit fast path wraps for values 2^32 past the window
                    if (mw) hv_ok[j] = hv_ok[j] && (uint64_t)d.hv[j] - (uint64_t)base < (uint64_t)mw * (uint64_t)P.interval;
                }
            } else {
                const int64_t k = key_index<KT>(P, d.hv[j]);
                hv_ok[j] = hv_ok[j] && k >= 0 && k < (int64_t)P.H;
                slot[j] = (uint32_t)k;
            }
        }
    }
    if constexpr (LDS && kIntRuns<ORD, MET, VK> && (VK & 4096) == 0) {
        // roughly time-ordered data (the blocks span more than one key: no runs1): a thread's consecutive docs alternate
        // between neighbouring keys and its three runs thrash -- each doc goes straight to its key's LDS cells instead,
        // in the lane's rotated copy (CollectParams.hdirect, ncopies); the values are exact integers, so the cells'
        // f64 sums equal the runs' (and the reference's sequential additions below 2^53)
        if (P.hdirect) {
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                if (!((d.ok >> j) & 1) || !hv_ok[j]) continue;
                const uint32_t c = slot[j] + a.coff;
                const double x = (double)(P.mv_base + (int64_t)d.mvd[j]);
                atomicAdd(&a.cnt32[c], 1u);
                atomicAdd(&a.sum[c], x);
                if (MET >= 3) atomicAdd(&a.sq[c], x * x);
                if (MET >= 2) {
                    const unsigned long long e = sortable(x);
                    if (e < a.mn[MS * slot[j]]) atomicMin(&a.mn[MS * slot[j]], e);
                    if (e > a.mx[MS * slot[j]]) atomicMax(&a.mx[MS * slot[j]], e);
                }
            }
            return;
        }
    }
    // one-run grids over time-sorted data with single-key zone blocks (kWinMK): a multi-key block's quads (an hour
    // boundary inside the block) go to the window accumulators too -- the one run flushed on every key change there, a
    // wave's flushes on two LDS addresses
    bool winq = kWin4<MET, VK>;
    constexpr int WS = kWinSlots<ORD, HIST, MET, VK>;
    if constexpr (kWinMK<ORD, HIST, MET, VK>) winq = !ublock;
    if constexpr (LDS && kIntRuns<ORD, MET, VK> && (kWin4<MET, VK> || kWinMK<ORD, HIST, MET, VK>)) if (winq) {
        uint32_t vm = 0;
        bool miss = false;
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
            const bool v = ((d.ok >> j) & 1) && hv_ok[j];
            vm |= (uint32_t)v << j;
            miss = miss || (v && slot[j] - run.wb >= (uint32_t)WS);
        }
        if (miss) {  // (rare: a lane's keys left its window) one doc at a time, re-basing where needed
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                if (!((vm >> j) & 1)) continue;
                if (slot[j] - run.wb >= (uint32_t)WS) win_rebase<MET, MS, runs_for<MET, VK>(), WS>(P, a, run, slot[j]);
                win_add<MET, runs_for<MET, VK>(), WS>(run, slot[j] - run.wb, d.mvd[j], true);
            }
        } else {
#pragma unroll
            for (int j = 0; j < kVec; ++j) win_add<MET, runs_for<MET, VK>(), WS>(run, slot[j] - run.wb, d.mvd[j], (vm >> j) & 1);
        }
        return;
    }
    if constexpr (LDS && kIntRuns<ORD, MET, VK>) {
        // integer runs: a thread's 4 docs that all pass and share one slot (time-sorted data: nearly always) are combined
        // into one run update; otherwise one update per doc
        const bool all4 = d.ok == 0xFu && hv_ok[0] && hv_ok[1] && hv_ok[2] && hv_ok[3] && slot[0] == slot[1] &&
                          slot[0] == slot[2] && slot[0] == slot[3];
        if (all4) {
            const uint32_t x0 = d.mvd[0], x1 = d.mvd[1], x2 = d.mvd[2], x3 = d.mvd[3];
            const unsigned long long q = MET >= 3 ? (unsigned long long)(x0 * x0) + (x1 * x1) + (unsigned long long)(x2 * x2) +
                                                        (x3 * x3)
                                                  : 0ull;
            runs_add_i<MET, MS>(P, a, run, slot[0], 4u, x0 + x1 + x2 + x3, q, min(min(x0, x1), min(x2, x3)),
                                max(max(x0, x1), max(x2, x3)));
        } else {
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                if (!((d.ok >> j) & 1) || !hv_ok[j]) continue;
                const uint32_t x = d.mvd[j];
                runs_add_i<MET, MS>(P, a, run, slot[j], 1u, x, (unsigned long long)(x * x), x, x);
            }
        }
        return;
    }
    if (LDS && !ORD) {  // ocnt_mode is OCNT_NONE without a terms dimension; without HIST the slot is always 0
        if (ESGPU_RUN4) {
            uint32_t okm = 0, first = ~0u;
#pragma unroll
            for (int j = 0; j < kVec; ++j) okm |= (((d.ok >> j) & 1) && hv_ok[j] ? 1u : 0u) << j;
            bool same = true;
#pragma unroll
            for (int j = 0; j < kVec; ++j)
                if ((okm >> j) & 1) {
                    if (first == ~0u) first = slot[j];
                    same = same && slot[j] == first;
                }
            // groups of docs with one key slot: all of them (time-sorted data: nearly always, a thread's 4 docs are
            // consecutive), else one doc each; one run update per group (a rolled loop: one inlined copy of the update)
            uint32_t rest = okm;
#pragma unroll
            for (int it = 0; it < kVec; ++it) {
                if (!rest) break;
                const uint32_t g = same ? rest : (rest & (0u - rest));
                rest &= ~g;
                uint32_t gs = first;
#pragma unroll
                for (int j = kVec - 1; j >= 0; --j)
                    if (!same && ((g >> j) & 1)) gs = slot[j];
                uint32_t vc = 0;
                double sum = 0.0, sq = 0.0;
                unsigned long long mn = kMinInit, mx = kMaxInit;
                if (MET > 0) {
#pragma unroll
                    for (int j = 0; j < kVec; ++j) {
                        const bool m = ((g >> j) & 1) && ((d.mpres >> j) & 1);
                        const double x = m ? d.mv[j] : 0.0;
                        vc += m ? 1u : 0u;
                        sum += x;
                        if (MET >= 3) sq += x * x;
                        if (MET >= 2) {
                            const bool nan = x != x;
                            const unsigned long long e = sortable(x);
                            const unsigned long long emn = !m ? kMinInit : nan ? 0ull : e, emx = !m ? kMaxInit : nan ? ~0ull : e;
                            mn = emn < mn ? emn : mn;
                            mx = emx > mx ? emx : mx;
                        }
                    }
                }
                runs_add_n<MET, MS>(P, a, run, gs, (uint32_t)__builtin_popcount(g), vc, sum, sq, mn, mx);
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
            if (!((d.ok >> j) & 1) || !hv_ok[j]) continue;
            runs_add<MET, MS>(P, a, run, slot[j], MET > 0 && ((d.mpres >> j) & 1), MET > 0 ? d.mv[j] : 0.0);
        }
        return;
    }
    if constexpr (LDS && ORD && MET > 0 && (VK & 64)) {
        // packed integer cells: one ds_add_u64 per doc carries count and sum; the 4 docs' (min, max) pairs are read
        // first with one wait for all four (the read-check is only a filter: a stale pair costs an extra atomic), so the
        // thread waits once per 4 docs instead of once per doc behind the queued atomics
        uint32_t cell[kVec], hit = 0;
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
            const uint32_t t = d.ord[j];
            const bool ok = (d.ok >> j) & 1, has_t = t < T;  // (kMissingOrd, and a raw 16-bit 0xFFFF, are >= T)
            hit |= (uint32_t)(ok && hv_ok[j] && has_t) << j;
            cell[j] = slot[j] * T + t;
        }
        // separate outer counts: one wave-uniform branch per 4 docs (inside the doc loop the compiler kept each doc's
        // masked atomic and its exec bookkeeping even when the mode counts nothing: ~10 scalar instructions per doc)
        if ((VK & 32768) != 0) {  // (no per-doc outer counts: VK bit 32768)
        } else if (P.ocnt_mode == OCNT_TERMS) {
            if (outer)
#pragma unroll
                for (int j = 0; j < kVec; ++j)
                    if (((d.ok >> j) & 1) && d.ord[j] < T) atomicAdd(&a.ocnt32[d.ord[j]], 1u);
        } else if (P.ocnt_mode == OCNT_HIST) {
#pragma unroll
            for (int j = 0; j < kVec; ++j)
                if (((d.ok >> j) & 1) && hv_ok[j]) atomicAdd(&a.ocnt32[slot[j]], 1u);
        }
        const unsigned long long one = 1ull << P.pk_shift;
#if ESGPU_PI_HOT
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
            if (!((hit >> j) & 1) || d.ord[j] != P.hot_t[0]) continue;
            if (slot[j] != run.hslot) {
                pi_hot_flush<MET>(P, a, run, T);
                run.hslot = slot[j];
            }
            run.hcnt[0] += 1u;
            run.hsum[0] += d.mvd[j];
            run.hlo[0] = min(run.hlo[0], d.mvd[j]);
            run.hhi[0] = max(run.hhi[0], d.mvd[j]);
            hit &= ~(1u << j);
        }
#endif
        // straight-line LDS traffic, so the compiler can count the one wait below (lgkmcnt(4): the reads, not the adds
        // queued behind them): every lane reads a (min, max) pair (a doc that hits nothing reads cell 0 and ignores it)
        // and adds to a cell (a miss adds 0 to the lane's own spare word)
        uint32_t mlo[kVec], mhi[kVec];
#if ESGPU_PI_NOATOM  // diagnostic only (A/B builds; wrong results): no LDS cell traffic, the docs folded into registers
#pragma unroll
        for (int j = 0; j < kVec; ++j) run.hpk += ((hit >> j) & 1) ? one + d.mvd[j] + cell[j] : 0ull;
        *a.pkd = run.hpk;
        return;
#endif
#if ESGPU_PI_STRAIGHT
        if (MET >= 2) {
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                const u32x2_t m = *reinterpret_cast<const u32x2_t*>(a.mm + 2 * (((hit >> j) & 1) ? cell[j] : 0u));
                mlo[j] = m.x;
                mhi[j] = m.y;
            }
        }
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
            const bool h = (hit >> j) & 1;
            atomicAdd(h ? &a.pk[cell[j] + a.coff] : a.pkd, one + d.mvd[j]);  // (a miss: into the lane's spare word)
        }
#else  // (A/B) reads and adds under the hit mask: the compiler then waits for every queued LDS op before the checks
        if (MET >= 2) {
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                mlo[j] = 0u;
                mhi[j] = ~0u;
                if ((hit >> j) & 1) {
                    const u32x2_t m = *reinterpret_cast<const u32x2_t*>(a.mm + 2 * cell[j]);
                    mlo[j] = m.x;
                    mhi[j] = m.y;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < kVec; ++j)
            if ((hit >> j) & 1) atomicAdd(&a.pk[cell[j] + a.coff], one + d.mvd[j]);
#endif
        if (MET >= 2) {
#if ESGPU_PI_MMCHECK == 4
            // one divergent loop over the lane's moving bounds (ESGPU_PI_MMU 4)
            uint32_t need = 0;
#pragma unroll
            for (int j = 0; j < kVec; ++j)
                need |= (uint32_t)(((hit >> j) & 1) && (d.mvd[j] < mlo[j] || d.mvd[j] > mhi[j])) << j;
            while (need) {
                const uint32_t j0 = (uint32_t)__builtin_ctz(need);
                need &= need - 1u;
                uint32_t c = 0, x = 0;
#pragma unroll
                for (int j = 0; j < kVec; ++j) {
                    c = j0 == (uint32_t)j ? cell[j] : c;
                    x = j0 == (uint32_t)j ? d.mvd[j] : x;
                }
                atomicMin(&a.mm[2 * c], x);
                atomicMax(&a.mm[2 * c + 1], x);
            }
#elif ESGPU_PI_MMCHECK == 2
            // one divergent region per doc: both atomics where either bound moves (the other is then a no-op)
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                const bool mv = ((hit >> j) & 1) && (d.mvd[j] < mlo[j] || d.mvd[j] > mhi[j]);
                if (mv) {
                    atomicMin(&a.mm[2 * cell[j]], d.mvd[j]);
                    atomicMax(&a.mm[2 * cell[j] + 1], d.mvd[j]);
                }
            }
#elif ESGPU_PI_MMCHECK
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                if (!((hit >> j) & 1)) continue;
                if (d.mvd[j] < mlo[j]) atomicMin(&a.mm[2 * cell[j]], d.mvd[j]);
                if (d.mvd[j] > mhi[j]) atomicMax(&a.mm[2 * cell[j] + 1], d.mvd[j]);
            }
#else  // (A/B) unconditional min / max atomics, a miss on the lane's spare word: no branches
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                const bool h = (hit >> j) & 1;
                uint32_t* w = h ? &a.mm[2 * cell[j]] : reinterpret_cast<uint32_t*>(a.pkd);
                atomicMin(w, h ? d.mvd[j] : ~0u);
                atomicMax(w + 1, h ? d.mvd[j] : 0u);
            }
#endif
        }
        return;
    }
    if constexpr (LDS && ORD && HIST && MET == 0 && ESGPU_COMBINE4) if (P.ocnt_mode != OCNT_TERMS) {
        // counting grids: a thread's 4 docs usually share the outer key (time-sorted data) and often the cell (skewed
        // inner keys): equal keys are combined in registers, and an outer key shared by the whole wave takes one LDS
        // atomic for the wave instead of 64 on one address
        uint32_t hk[kVec], cell[kVec];
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
            const bool hit = ((d.ok >> j) & 1) && hv_ok[j];
            const uint32_t t = d.ord[j];
            hk[j] = hit ? slot[j] : ~0u;
            cell[j] = hit && t != kMissingOrd && t < T ? slot[j] * T + t : ~0u;
        }
        if constexpr (kOrdHHot<ORD, HIST, MET, VK>) {
            // a single-key zone block (wave-uniform): the hot ordinal's docs into the lane's register count for the key
            // -- the Zipf head's same-address LDS atomics were the grid's conflicts
            const uint32_t ht = P.hot_t[0];
            if (ublock && ht < T) {
                if (slot[0] != run.hslot) {
                    cnt_hot_flush(a, run, T, ht);
                    run.hslot = slot[0];
                }
#pragma unroll
                for (int j = 0; j < kVec; ++j) {
                    const bool h = cell[j] != ~0u && d.ord[j] == ht;
                    run.hcnt[0] += h ? 1u : 0u;
                    cell[j] = h ? ~0u : cell[j];
                }
            }
        }
        if (P.ocnt_mode == OCNT_HIST) {
            uint32_t key = ~0u, n = 0;
            bool single = true;
#pragma unroll
            for (int j = 0; j < kVec; ++j) {
                if (hk[j] == ~0u) continue;
                if (n == 0) key = hk[j];
                single = single && hk[j] == key;
                ++n;
            }
            const uint64_t live = __ballot(n > 0);
            if (live) {
                const int src = __ffsll((unsigned long long)live) - 1;
                const uint32_t k0 = __shfl(key, src, 64);
                if (__all(n == 0 || (single && key == k0))) {
                    const uint32_t tot = wave_sum_u32(n);
                    if ((int)(threadIdx.x & 63) == src) atomicAdd(&a.ocnt32[k0], tot);
                } else {
                    combine4(hk, [&](uint32_t k, uint32_t m) { atomicAdd(&a.ocnt32[k], m); });
                }
            }
        }
        combine4(cell, [&](uint32_t c, uint32_t m) { atomicAdd(&a.cnt32[c + a.coff], m); });
        return;
    }
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
        if (!((d.ok >> j) & 1)) continue;
        const uint32_t t = ORD ? d.ord[j] : 0u;
        const bool has_t = ORD ? (t != kMissingOrd && t < T) : true;
        const double x = MET > 0 ? ((VK & 64) ? (double)(P.mv_base + (int64_t)d.mvd[j]) : d.mv[j]) : 0.0;
        update_doc<ORD, HIST, MET, LDS, MS>(P, a, T, has_t, t, hv_ok[j], slot[j], MET > 0 && ((d.mpres >> j) & 1), x, outer);
    }
}

// Packed-cell raw-load kernels over block-delta keys (VK bits 64 | 8192), a full zone block whose docs all round to one
// key (99.4 % of the north star's blocks at 1B docs): the key slot is wave-uniform, so a doc's cell is slot * T + its
// ordinal and nothing else is computed per doc -- no key arithmetic, no per-doc slot selects, no tail mask (the caller
// takes this path for full blocks only), and the packed add's high word is a constant: pk_shift >= 33 (pi_fits: a
// workgroup range holds < 2^31 docs), so `one + delta` is the pair {delta, one >> 32}.  NH = 1 or 2 Doc4 halves of one
// step, processed together (their LDS reads issued before the adds).
#ifndef ESGPU_PI_UFAST  // (A/B) 0: the general per-doc path for these blocks too
#define ESGPU_PI_UFAST 1
#endif
#ifndef ESGPU_PI_HOTU  // the segment's most frequent ordinal counted and summed in registers in uniform blocks: 2 = with
#define ESGPU_PI_HOTU 2  // (min, max) leaves only (north star 1.104 -> 1.046 ms at 1B, r6f: its LDS adds were the kernel's
#endif                   // limit; avg grids, which are not LDS-bound, measured 5 % slower with it), 1 = always, 0 = never
#ifndef ESGPU_PI_HOTMM  // (A/B) the hot ordinal's register run keeps its (min, max) too (no LDS read for its docs)
#define ESGPU_PI_HOTMM 0  // (measured slower: north star 1.081 -> 1.133 ms at 1B, r6h -- its VALU cost; 2 or 3 hot ordinals 1.54 / 1.91)
#endif
#ifndef ESGPU_PI_HOTPK  // the hot ordinal's count and sum by packed 16-bit compares and v_dot2 (0: per-doc selects, A/B)
#define ESGPU_PI_HOTPK 1
#endif
#ifndef ESGPU_PI_MMU  // (A/B) uniform blocks' (min, max) updates: 2 = one divergent region per doc (as ESGPU_PI_MMCHECK 2),
#define ESGPU_PI_MMU 2  // 3 = branch-free -- every lane issues both atomics, lanes whose bounds do not move on a spare word;
#endif                  // 4 = one divergent loop per lane over its moving bounds (north star 1.03 -> 1.06 ms, r6aj);
                        // 5 = one region per pair of docs, four unconditional atomics (0.99-1.02 -> 1.03-1.04 ms, r6au)
template <int MET, int VK, int NH, int NR>
__device__ __forceinline__ void pi_uniform(const CollectParams& P, const Acc& a, const Doc4& h0, const Doc4& h1, uint32_t T,
                                           uint32_t win0, Runs<NR>& run, uint32_t mw, bool outer) {
    constexpr int N = 4 * NH;
    const uint32_t k = h0.ukey;  // wave-uniform (zone_ukey: scalar loads)
    const uint32_t sl = k - win0;
    const bool in = k < P.H && sl < (mw ? mw : P.W);
    uint32_t t[N], dv[N];
    uint32_t okm = (1u << N) - 1u;  // bit j: doc j passes the folded accept bitset (VK bit 512)
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
        const Doc4& h = hh == 0 ? h0 : h1;
        t[4 * hh + 0] = h.raw[0] & 0xFFFFu; t[4 * hh + 1] = h.raw[0] >> 16;
        t[4 * hh + 2] = h.raw[1] & 0xFFFFu; t[4 * hh + 3] = h.raw[1] >> 16;
        dv[4 * hh + 0] = h.raw[6] & 0xFFFFu; dv[4 * hh + 1] = h.raw[6] >> 16;
        dv[4 * hh + 2] = h.raw[7] & 0xFFFFu; dv[4 * hh + 3] = h.raw[7] >> 16;
        if constexpr ((VK & 512) != 0) okm &= ~((~(uint32_t)(h.racc >> (h.doc0 & 63)) & 0xFu) << (4 * hh));
    }
    // outer counts (wave-uniform mode): per-term counts need every doc; a per-key count is the wave's passing docs
    // (VK bit 32768: the plan's outer counts are not counted per doc -- derived from the cells at the flush)
    if ((VK & 32768) != 0) {
    } else if (P.ocnt_mode == OCNT_TERMS) {
        if (outer)
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (((okm >> j) & 1) && t[j] < T) atomicAdd(&a.ocnt32[t[j]], 1u);
    } else if (P.ocnt_mode == OCNT_HIST) {
        if (in) {
            const uint32_t tot = wave_sum_u32((uint32_t)__builtin_popcount(okm));
            if ((threadIdx.x & 63) == 0 && tot) atomicAdd(&a.ocnt32[sl], tot);
        }
    }
    if (!in) return;
    const uint32_t cb = sl * T;  // the block's row of cells
    const uint32_t onehi = (uint32_t)(1ull << (P.pk_shift - 32));
    bool hit[N], hpk[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        hit[j] = (((okm >> j) & 1) != 0) & (t[j] < T);  // (a missing ordinal, 0xFFFF, is >= T)
        hpk[j] = hit[j];
    }
    constexpr bool kHot = ESGPU_PI_HOTU == 1 || (ESGPU_PI_HOTU == 2 && MET >= 2);
    if constexpr (kHot) {
    if (sl != run.hslot) {  // (uniform) the hot ordinal's register run moves to this key
        pi_hot_flush<MET>(P, a, run, T);
        run.hslot = sl;
    }
    if constexpr (ESGPU_PI_HOTPK && NH == 1 && kNHot == 1 && !ESGPU_PI_HOTMM && (VK & 512) == 0) {
        // packed: the hot ordinal's docs among the 4 found as zero 16-bit halves of (ordinals ^ hot), their count and
        // delta sum by v_dot2_u32_u16 (a doc equal to the hot ordinal is below T: no hit test needed without a bitset)
        // (no hot ordinal, kMissingOrd: 0xFFFE halves, which no 16-bit ordinal or missing value (0xFFFF) equals)
        const uint32_t ht = P.hot_t[0], htp = ht < T ? (ht | (ht << 16)) : 0xFFFEFFFEu;
        const u16x2_t one = {1, 1};
        const u16x2_t e0 = one - __builtin_elementwise_min(__builtin_bit_cast(u16x2_t, h0.raw[0] ^ htp), one);
        const u16x2_t e1 = one - __builtin_elementwise_min(__builtin_bit_cast(u16x2_t, h0.raw[1] ^ htp), one);
        run.hcnt[0] = __builtin_amdgcn_udot2(e0, one, __builtin_amdgcn_udot2(e1, one, run.hcnt[0], false), false);
        run.hsum[0] = __builtin_amdgcn_udot2(e0, __builtin_bit_cast(u16x2_t, h0.raw[6]),
                                             __builtin_amdgcn_udot2(e1, __builtin_bit_cast(u16x2_t, h0.raw[7]), run.hsum[0], false),
                                             false);
#pragma unroll
        for (int j = 0; j < N; ++j) hpk[j] = hpk[j] & (t[j] != ht);
    } else {
#pragma unroll
        for (int k = 0; k < kNHot; ++k) {
            const uint32_t ht = P.hot_t[k];
            uint32_t hc = run.hcnt[k], hs = run.hsum[k], hl = run.hlo[k], hh = run.hhi[k];
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const bool ho = hit[j] & (t[j] == ht);
                hc += ho ? 1u : 0u;
                hs += ho ? dv[j] : 0u;
                if (MET >= 2 && ESGPU_PI_HOTMM) {  // ... and its extrema: the hot docs leave the (min, max) reads too
                    hl = min(hl, ho ? dv[j] : ~0u);
                    hh = max(hh, ho ? dv[j] : 0u);
                    hit[j] = hit[j] & !ho;
                }
                hpk[j] = hpk[j] & !ho;
            }
            run.hcnt[k] = hc;
            run.hsum[k] = hs;
            run.hlo[k] = hl;
            run.hhi[k] = hh;
        }
    }
    }
    uint32_t mlo[N], mhi[N];
    if (MET >= 2) {
#pragma unroll
        for (int j = 0; j < N; ++j) {  // (a doc that hits nothing reads cell 0: one broadcast address)
            const u32x2_t m = *reinterpret_cast<const u32x2_t*>(hit[j] ? a.mm + 2 * (cb + t[j]) : a.mm);
            mlo[j] = m.x;
            mhi[j] = m.y;
        }
    }
#pragma unroll
    for (int j = 0; j < N; ++j)  // (a miss adds into the lane's spare word)
        atomicAdd(hpk[j] ? &a.pk[cb + t[j] + a.coff] : a.pkd, join64(dv[j], onehi));
    if (MET >= 2) {
#if ESGPU_PI_MMU == 5
        // one divergent region per pair of docs, its four atomics unconditional (a doc whose bounds stay on the lane's
        // spare word)
        uint32_t* spare = reinterpret_cast<uint32_t*>(a.pkd);
#pragma unroll
        for (int j = 0; j < N; j += 2) {
            const bool m0 = hit[j] & ((dv[j] < mlo[j]) | (dv[j] > mhi[j]));
            const bool m1 = hit[j + 1] & ((dv[j + 1] < mlo[j + 1]) | (dv[j + 1] > mhi[j + 1]));
            if (m0 | m1) {
                uint32_t* w0 = m0 ? &a.mm[2 * (cb + t[j])] : spare;
                uint32_t* w1 = m1 ? &a.mm[2 * (cb + t[j + 1])] : spare;
                atomicMin(w0, dv[j]);
                atomicMax(w0 + 1, dv[j]);
                atomicMin(w1, dv[j + 1]);
                atomicMax(w1 + 1, dv[j + 1]);
            }
        }
#elif ESGPU_PI_MMU == 4
        // one divergent loop over the lane's moving bounds (most lanes have none: ~1 iteration where the per-doc regions
        // issued the two atomics for up to N docs)
        uint32_t need = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) need |= (uint32_t)(hit[j] & ((dv[j] < mlo[j]) | (dv[j] > mhi[j]))) << j;
        while (need) {
            const uint32_t j0 = (uint32_t)__builtin_ctz(need);
            need &= need - 1u;
            uint32_t c = 0, x = 0;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                c = j0 == (uint32_t)j ? t[j] : c;
                x = j0 == (uint32_t)j ? dv[j] : x;
            }
            atomicMin(&a.mm[2 * (cb + c)], x);
            atomicMax(&a.mm[2 * (cb + c) + 1], x);
        }
#elif ESGPU_PI_MMU == 3
        uint32_t* spare = reinterpret_cast<uint32_t*>(a.pkd);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const bool mv = hit[j] & ((dv[j] < mlo[j]) | (dv[j] > mhi[j]));
            uint32_t* w = mv ? &a.mm[2 * (cb + t[j])] : spare;
            atomicMin(w, dv[j]);
            atomicMax(w + 1, dv[j]);
        }
#else
#pragma unroll
        for (int j = 0; j < N; ++j) {
            // (bitwise: one divergent region per doc -- a short-circuit && nests a second one around the comparisons)
            const bool mv = hit[j] & ((dv[j] < mlo[j]) | (dv[j] > mhi[j]));
            if (mv) {
                atomicMin(&a.mm[2 * (cb + t[j])], dv[j]);
                atomicMax(&a.mm[2 * (cb + t[j]) + 1], dv[j]);
            }
        }
#endif
    }
}

// packed integer cells (VK bit 64): decoded into the grid's u64 counts, f64 sums (the exact integer sum of the cell's
// values, count * base + sum of deltas) and order-preserving extrema of (double) values -- (double) is monotonic on
// longs, so the min / max of the casts are the casts of the min / max
template <int MET, int WGS>
__device__ void flush_window_pi(const CollectParams& P, const Acc& s, uint32_t T, uint32_t W, uint32_t win0, uint32_t ncp) {
    __syncthreads();
    const uint32_t C = T * W;
    const uint32_t sh = P.pk_shift;
    const unsigned long long mask = (1ull << sh) - 1ull;
    if (P.ocnt_mode == OCNT_TERMS_DERIVED) {
        for (uint32_t t = threadIdx.x; t < T; t += WGS) {
            unsigned long long tot = 0;
            for (uint32_t k = 0; k < ncp; ++k)
                for (uint32_t l = 0; l < W; ++l) tot += s.pk[k * C + l * T + t];
            tot >>= sh;
            if (tot) atomicAdd(&P.g_ocnt[t], tot);
        }
        __syncthreads();
    }
    for (uint32_t c = threadIdx.x; c < C; c += WGS) {
        unsigned long long n = 0;
        for (uint32_t k = 0; k < ncp; ++k) n += s.pk[k * C + c];
        if (n == 0) continue;
        const uint32_t local = c / T;
        const uint32_t t = c - local * T;
        const uint32_t slot = win0 + local;
        if (slot >= P.H) continue;
        const size_t g = (size_t)slot * T + t;
        const unsigned long long cnt = n >> sh;
        atomicAdd(&P.g_cnt[g], cnt);
        for (uint32_t k = 0; k < ncp; ++k) s.pk[k * C + c] = 0;
        // the cell's exact integer sum; compensated into the grid when its partial sums could pass 2^53
        const long long isum = (long long)(n & mask) + (long long)cnt * P.mv_base;
        if (P.g_sum_lo) {
            double xh, xl;
            i64_to_dd(isum, xh, xl);
            dd_atomic_add(&P.g_sum[g], P.g_sum_lo + g, xh, xl);
        } else {
            atomicAdd(&P.g_sum[g], (double)isum);
        }
        if (MET >= 2) {
            const uint32_t lo = s.mm[2 * c], hi = s.mm[2 * c + 1];
            atomicMin(&P.g_min[g], sortable((double)(P.mv_base + (int64_t)lo)));
            atomicMax(&P.g_max[g], sortable((double)(P.mv_base + (int64_t)hi)));
            s.mm[2 * c] = ~0u;
            s.mm[2 * c + 1] = 0u;
        }
    }
    if (P.ocnt_mode == OCNT_TERMS) {
        for (uint32_t t = threadIdx.x; t < T; t += WGS) {
            const uint32_t n = s.ocnt32[t];
            if (n) { atomicAdd(&P.g_ocnt[t], (unsigned long long)n); s.ocnt32[t] = 0; }
        }
    } else if (P.ocnt_mode == OCNT_HIST) {
        for (uint32_t l = threadIdx.x; l < W; l += WGS) {
            const uint32_t n = s.ocnt32[l];
            if (n && win0 + l < P.H) { atomicAdd(&P.g_ocnt[win0 + l], (unsigned long long)n); }
            s.ocnt32[l] = 0;
        }
    }
    __syncthreads();
}

template <int MET, int MS, int WGS>
__device__ void flush_window(const CollectParams& P, const Acc& s, uint32_t T, uint32_t W, uint32_t win0, uint32_t ncp = 1) {
    __syncthreads();
    const uint32_t C = T * W;
    if (P.ocnt_mode == OCNT_TERMS_DERIVED) {  // per-term totals of this window (one atomic per term)
        for (uint32_t t = threadIdx.x; t < T; t += WGS) {
            uint32_t tot = 0;
            for (uint32_t k = 0; k < ncp; ++k)
                for (uint32_t l = 0; l < W; ++l) tot += s.cnt32[k * C + l * T + t];
            if (tot) atomicAdd(&P.g_ocnt[t], (unsigned long long)tot);
        }
        __syncthreads();
    }
    for (uint32_t c = threadIdx.x; c < C; c += WGS) {
        uint32_t n = 0;
        for (uint32_t k = 0; k < ncp; ++k) n += s.cnt32[k * C + c];
        if (n == 0) continue;
        const uint32_t local = c / T;
        const uint32_t t = c - local * T;
        const uint32_t slot = win0 + local;
        if (slot >= P.H) continue;
        const size_t g = (size_t)slot * T + t;
        atomicAdd(&P.g_cnt[g], (unsigned long long)n);
        for (uint32_t k = 0; k < ncp; ++k) s.cnt32[k * C + c] = 0;
        if (MET > 0) {
            if (P.vcnt_mode) {
                uint32_t vc = 0;
                for (uint32_t k = 0; k < ncp; ++k) { vc += s.vcnt32[k * C + c]; s.vcnt32[k * C + c] = 0; }
                atomicAdd(&P.g_vcnt[g], (unsigned long long)vc);
            }
            double sum = 0.0;
            for (uint32_t k = 0; k < ncp; ++k) { sum += s.sum[k * C + c]; s.sum[k * C + c] = 0.0; }
            dd_atomic_add(&P.g_sum[g], P.g_sum_lo ? P.g_sum_lo + g : nullptr, sum);
            if (MET >= 2) {
                const unsigned long long mn = s.mn[MS * c], mx = s.mx[MS * c];
                if (mn != kMinInit) atomicMin(&P.g_min[g], mn);
                if (mx != kMaxInit) atomicMax(&P.g_max[g], mx);
                s.mn[MS * c] = kMinInit;
                s.mx[MS * c] = kMaxInit;
            }
            if (MET >= 3) {
                double sq = 0.0;
                for (uint32_t k = 0; k < ncp; ++k) { sq += s.sq[k * C + c]; s.sq[k * C + c] = 0.0; }
                dd_atomic_add(&P.g_sq[g], P.g_sq_lo ? P.g_sq_lo + g : nullptr, sq);
            }
        }
    }
    if (P.ocnt_mode == OCNT_TERMS) {
        for (uint32_t t = threadIdx.x; t < T; t += WGS) {
            const uint32_t n = s.ocnt32[t];
            if (n) { atomicAdd(&P.g_ocnt[t], (unsigned long long)n); s.ocnt32[t] = 0; }
        }
    } else if (P.ocnt_mode == OCNT_HIST) {
        for (uint32_t l = threadIdx.x; l < W; l += WGS) {
            const uint32_t n = s.ocnt32[l];
            if (n && win0 + l < P.H) { atomicAdd(&P.g_ocnt[win0 + l], (unsigned long long)n); }
            s.ocnt32[l] = 0;
        }
    }
    __syncthreads();
}

// next chunk of a dynamically claimed collect (thread 0 only).  The counter address goes through an opaque VGPR zero:
// with a provably uniform address the atomic optimizer broadcasts the returned value at once (v_readfirstlane right
// after the atomic, i.e. a vmcnt(0) wait that drains the wave's prefetched loads); this way the value is first used a
// chunk later, when the claim is published.
__device__ __forceinline__ uint32_t claim_chunk(unsigned int* claim) {
    uint32_t zero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    return atomicAdd(claim + zero, 1u);  // chunks claimed past the grid's first gridDim.x
}

// HK: 0 = no histogram dimension, 1 = affine rounding, 2 = bucket table (calendar units / DST zones)
// WGS: threads per workgroup -- 512 (two resident per CU, each with an LDS window of <= 64 KB), or 1024 for
// histogram grids whose data needs a wider window than 64 KB holds (one workgroup per CU with up to 150 KB of LDS,
// the same 16 waves per CU)
#ifndef ESGPU_PI_WAVES  // packed-cell kernels: waves per SIMD the register budget must allow (6: three 512-thread workgroups per CU)
#define ESGPU_PI_WAVES 6
#endif
// 4 waves per SIMD (16 per CU): <= 128 VGPRs; packed-cell kernels ESGPU_PI_WAVES (6: <= 80 VGPRs, 24 waves per CU with the
// runtime's ESGPU_LDS_PI window budget -- the stream's bytes in flight scale with the waves)
#ifndef ESGPU_HIST_WAVES  // raw-load counting histogram grids (VK bit 1024): waves per SIMD
#define ESGPU_HIST_WAVES 6
#endif
#ifndef ESGPU_HIST_MET_WAVES  // raw-load histogram-only grids with a metric: waves per SIMD
#define ESGPU_HIST_MET_WAVES 4
#endif
#ifndef ESGPU_HIST_RUNS1_WAVES  // ... of them the one-run integer grids over time-sorted data (VK bits 2048 | 4096): the
#define ESGPU_HIST_RUNS1_WAVES 6  // stream's bytes in flight scale with the waves (6 with 8 docs per thread: config 2
#endif                            // 0.622 -> 0.523 ms at 1B, 0.0816 -> 0.0703 ms at 100M; the ±1 h window kernels at 6:
                                  // 2.35 -> 4.49 ms, r6ag -- they keep 4)
#ifndef ESGPU_ORDH_WAVES  // raw-load counting grids with a terms dimension (terms{date_histogram}, VK bit 1024): waves per SIMD
#define ESGPU_ORDH_WAVES 4
#endif
template <bool ORD, int MET, int VK, int WGS> constexpr int collect_min_waves() {
    return (VK & 64) && WGS == 512                    ? ESGPU_PI_WAVES
           : ORD && (VK & 1024) && WGS == 512 && MET == 0 ? ESGPU_ORDH_WAVES
           : !ORD && (VK & 1024) && WGS == 512 && MET == 0 ? ESGPU_HIST_WAVES
           : !ORD && (VK & 1024) && WGS == 512 && MET > 0 && (VK & 2048) && (VK & 4096) ? ESGPU_HIST_RUNS1_WAVES
           : !ORD && (VK & 1024) && WGS == 512        ? ESGPU_HIST_MET_WAVES
                                                     : 4;
}
template <bool ORD, int HK, int MET, int VK, int WGS>
__global__ __launch_bounds__(WGS, (collect_min_waves<ORD, MET, VK, WGS>())) void collect_kernel(CollectParams P) {
    constexpr bool WIDE8 = (ESGPU_DOCS8 != 0 && kRawPI<MET, VK, (HK != 0)>) ||  // 8 docs per thread per step (Doc8)
                           (ESGPU_DOCS8_H != 0 && kRawH<ORD, MET, VK> && ORD) ||
                           (ESGPU_DOCS8_HI != 0 && kIntRuns<ORD, MET, VK> && (VK & 4096) != 0 && (HK != 0));
    constexpr int kIterDocsW = WGS * (WIDE8 ? 2 * kVec : kVec);
    constexpr int kItersPerBlockW = kBlockDocs / kIterDocsW;
    constexpr bool HIST = HK != 0;
    constexpr bool KT = HK == 2;
    constexpr bool HORD = HK == 3;  // terms under terms: the inner ordinal column is the key dimension
    constexpr int VKL = HORD ? (VK | 4) : VK;
    // min/max LDS layout: interleaved (one paired read per check) with a key dimension, two arrays without one
    // (terms{stats}: measured 11 % faster with separate arrays, the interleaved pairs conflict on fewer banks)
    constexpr int kMS = HIST ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t T = ORD ? P.T : 1u;
    const uint32_t W = HIST ? P.W : 1u;
    const uint32_t C = T * W;

    Acc g;  // global grid view
    g.cnt32 = nullptr; g.vcnt32 = nullptr; g.ocnt32 = nullptr;
    g.cnt64 = P.g_cnt; g.vcnt64 = P.g_vcnt; g.sum = P.g_sum; g.mn = P.g_min; g.mx = P.g_max; g.sq = P.g_sq;
    g.sum_lo = P.g_sum_lo; g.sq_lo = P.g_sq_lo;
    g.mstride = 1;
    g.coff = 0;
    g.ocnt64 = P.g_ocnt;
    g.pk = nullptr; g.mm = nullptr; g.pkd = nullptr;
    // additive cell copies: grids with a terms dimension, and the per-doc integer-run grids (CollectParams.hdirect)
    const uint32_t ncp = (ORD || (kIntRuns<ORD, MET, VK> && (VK & 4096) == 0)) ? max(P.ncopies, 1u) : 1u;

    // LDS window view.  Every pointer is derived from `smem` alone -- never merged with a global pointer -- so the
    // compiler keeps them in the LDS address space (ds_* instructions).  A generic pointer would compile to flat_*
    // accesses, and each flat load waits for vmcnt(0): the prefetched loads of the next iteration.
    constexpr bool PI = MET > 0 && (VK & 64) != 0;  // packed integer cells
    // ... over block-delta keys: full single-key zone blocks take pi_uniform
    constexpr bool kPIU = ESGPU_PI_UFAST != 0 && PI && HIST && !HORD && kUKeyK<ORD, HIST, MET, VKL> && kRawPI<MET, VKL, HIST>;
    Acc s;
    s.sum_lo = nullptr; s.sq_lo = nullptr;
    if constexpr (PI) {  // collect_lds_bytes(pi = true) mirrors this carve
        size_t off = 0;
        auto carve = [&](size_t bytes) { unsigned char* p = smem + off; off += (bytes + 15) & ~(size_t)15; return p; };
        s.cnt64 = nullptr; s.vcnt64 = nullptr; s.ocnt64 = nullptr;
        s.cnt32 = nullptr; s.vcnt32 = nullptr; s.sum = nullptr; s.sq = nullptr; s.mn = nullptr; s.mx = nullptr;
        s.mstride = 1;
        s.pk = (unsigned long long*)carve(8 * C * ncp);
        s.mm = (uint32_t*)carve(MET >= 2 ? 8 * C : 0);
        s.coff = ((threadIdx.x & 63) % ncp) * C;
        s.ocnt32 = (uint32_t*)carve(P.ocnt_mode == OCNT_TERMS ? sizeof(uint32_t) * T
                                    : P.ocnt_mode == OCNT_HIST ? sizeof(uint32_t) * W : 0);
        s.pkd = (unsigned long long*)carve(8 * WGS) + threadIdx.x;
    } else {
        size_t off = 0;
        auto carve = [&](size_t bytes) { unsigned char* p = smem + off; off += (bytes + 15) & ~(size_t)15; return p; };
        s.pk = nullptr; s.mm = nullptr; s.pkd = nullptr;
        s.cnt64 = nullptr; s.vcnt64 = nullptr; s.ocnt64 = nullptr;
        s.cnt32 = (uint32_t*)carve(sizeof(uint32_t) * C * ncp);
        s.vcnt32 = (uint32_t*)carve(P.vcnt_mode ? sizeof(uint32_t) * C * ncp : 0);
        s.sum = (double*)carve(MET > 0 ? sizeof(double) * C * ncp : 0);
        s.mn = (unsigned long long*)carve(MET >= 2 ? 16 * C : 0);
        s.mx = s.mn + (kMS == 2 ? 1 : C);
        s.mstride = kMS;
        s.sq = (double*)carve(MET >= 3 ? sizeof(double) * C * ncp : 0);
        s.coff = ((threadIdx.x & 63) % ncp) * C;
        s.ocnt32 = (uint32_t*)carve(P.ocnt_mode == OCNT_TERMS ? sizeof(uint32_t) * T
                                    : P.ocnt_mode == OCNT_HIST ? sizeof(uint32_t) * W : 0);
    }
    if (PI && P.lds_mode) {
        for (uint32_t c = threadIdx.x; c < C * ncp; c += WGS) s.pk[c] = 0;
        if (MET >= 2)
            for (uint32_t c = threadIdx.x; c < C; c += WGS) { s.mm[2 * c] = ~0u; s.mm[2 * c + 1] = 0u; }
        if (P.ocnt_mode == OCNT_TERMS || P.ocnt_mode == OCNT_HIST)
            for (uint32_t c = threadIdx.x; c < (P.ocnt_mode == OCNT_TERMS ? T : W); c += WGS) s.ocnt32[c] = 0;
        __syncthreads();
    } else if (P.lds_mode) {
        for (uint32_t c = threadIdx.x; c < C * ncp; c += WGS) {
            s.cnt32[c] = 0;
            if (P.vcnt_mode) s.vcnt32[c] = 0;
            if (MET > 0) s.sum[c] = 0.0;
            if (MET >= 3) s.sq[c] = 0.0;
        }
        for (uint32_t c = threadIdx.x; c < C; c += WGS)
            if (MET >= 2) { s.mn[kMS * c] = kMinInit; s.mx[kMS * c] = kMaxInit; }
        if (P.ocnt_mode == OCNT_TERMS || P.ocnt_mode == OCNT_HIST)
            for (uint32_t c = threadIdx.x; c < (P.ocnt_mode == OCNT_TERMS ? T : W); c += WGS) s.ocnt32[c] = 0;
        __syncthreads();
    }

    // dynamic claiming: a workgroup's blocks are chunks of kGroup blocks (= the multi-pass groups) taken from a
    // counter while they last, so the workgroups that run faster (a CU holding one workgroup, an idle XCD) take more
    // and the single wave of resident workgroups ends together.  Thread 0 claims one chunk ahead: the claim issued
    // at the start of chunk k is published (LDS + the barrier) at the start of chunk k + 1, and names chunk k + 2,
    // so its latency hides behind a chunk of loads and the prefetch into the next chunk knows where to go.
    const bool dyn = P.claim != nullptr;
    __shared__ uint32_t claim_lds[2];
    uint32_t claim_pend = 0, claim_k = 0, nxt_c = ~0u;
    uint32_t b_begin, b_end;
    if (dyn) {
        b_begin = blockIdx.x * kGroup;
        b_end = P.n_blocks;
        if (threadIdx.x == 0) claim_pend = claim_chunk(P.claim);
    } else {
        b_begin = blockIdx.x * P.blocks_per_wg;
        b_end = b_begin + P.blocks_per_wg;
        if (b_end > P.n_blocks) b_end = P.n_blocks;
        if (b_begin >= b_end) return;
    }

    // window state (only meaningful with HIST && lds_mode)
    uint32_t win0 = 0;
    bool win_set = !(HIST && P.windowed);   // un-windowed: slot 0 of LDS == grid slot 0
    bool dirty = false;
    int64_t base = HIST ? P.key0 * P.interval + P.offset : 0;  // value of the first LDS slot

    Runs<runs_for<MET, VKL>()> run;
    runs_reset(run);
    // software pipeline over two buffers: each is reloaded (iteration i + 2) right after it is processed, so one
    // buffer's loads are in flight while the other is processed.  Loads are unconditional (past the end: the last
    // block's docs again, never processed) and no loaded register is copied: a conditional load or a register
    // copy of a load's result makes the compiler wait vmcnt(0), which drains the other buffer's loads as well.
    //
    // Multi-pass groups (roughly time-ordered data whose blocks span more keys than the window): the blocks are taken
    // in groups of kGroup; a group holding a block that spans more than W keys is replayed once per W keys of the
    // group's key range, each pass accumulating only the docs whose key falls in its window (replays re-read the
    // group from L2 / MALL).  One window flush per pass of a group instead of one per pass of every block: with
    // +-1 h jitter the flushes (T x W cells of global atomics) cost 4x the column read when taken per block.  The
    // replay is part of the schedule the prefetches follow -- the pass count is known at the group's first
    // iteration, before any replayed iteration is prefetched -- so it costs no extra load buffers.  Groups whose
    // blocks each fit the window are taken block by block, the window sliding as before.
    const uint32_t tid4 = threadIdx.x * (WIDE8 ? 2 * kVec : kVec);
    // shapes that read few bytes per doc (one ordinal or one key column) keep 4 buffers in flight, the rest 2 (their
    // buffers are 5x larger; 4 would cost occupancy).  kItersPerBlockW (4) is a multiple of either.
    constexpr int kBuf = (kRawH<ORD, MET, VK> && !ORD && MET == 0) ? (ESGPU_NBUF_HIST <= kItersPerBlockW ? ESGPU_NBUF_HIST : kItersPerBlockW)
                         : (kRawH<ORD, MET, VK> && !ORD) ? (ESGPU_NBUF_HIST_MET <= kItersPerBlockW ? ESGPU_NBUF_HIST_MET : kItersPerBlockW)
                         : (MET == 0 && !(ORD && HIST)) ? ESGPU_NBUF_NARROW
                         : ((VK & 64) && kRawPI<MET, VK, HIST> && !(VK & 512))
                             ? (ESGPU_NBUF_PI_RAW <= kItersPerBlockW ? ESGPU_NBUF_PI_RAW : kItersPerBlockW)
                         : (VK & 64) ? (ESGPU_NBUF_PI <= kItersPerBlockW ? ESGPU_NBUF_PI : kItersPerBlockW)
                         : ((VK & 176) ? (ESGPU_NBUF_COMPACT <= kItersPerBlockW ? ESGPU_NBUF_COMPACT : kItersPerBlockW) : 2);
    static_assert(kItersPerBlockW % kBuf == 0, "buffers per block");
    // block-delta kernels: the zone block's key when all its docs share one (zone_keys ranges, two scalar loads per
    // block and wave), the block's timestamps then left unread
    auto zone_ukey = [&](uint32_t blk) -> uint32_t {
        if constexpr (!kUKeyK<ORD, HIST, MET, VKL>) {
            return kNoUKey;
        } else {
            const uint32_t b = __builtin_amdgcn_readfirstlane(blk);
            const int64_t kmn = P.zkey[2 * b], kmx = P.zkey[2 * b + 1];
            if (kmn != kmx) return kNoUKey;
            return kmn >= 0 && kmn < (int64_t)P.H ? (uint32_t)kmn : kOutUKey;
        }
    };
    uint32_t pf_blk = b_begin, pf_uk = zone_ukey(b_begin);  // the block the prefetches read, and its key
    using Buf = std::conditional_t<WIDE8, Doc8, Doc4>;
    auto load_buf = [&](uint32_t doc0, Buf& d, uint32_t uk) {
        if constexpr (WIDE8) load_docs8<ORD, HIST, MET, VKL>(P, doc0, d, uk);
        else load_docs<ORD, HIST, MET, VKL>(P, doc0, d, uk);
    };
    Buf q[kBuf];
#pragma unroll
    for (int k = 0; k < kBuf; ++k) load_buf(b_begin * kBlockDocs + k * kIterDocsW + tid4, q[k], pf_uk);

    bool use_lds = P.lds_mode != 0;
    uint32_t cb = b_begin;                               // block being processed
    uint32_t gb = b_begin, ge = min(b_begin + kGroup, b_end);  // its group
    uint32_t pass = 0, npass = 1;                        // npass > 1: a multi-pass group
    auto slide_to = [&](uint32_t k0) {
        if (dirty) {
            if (!ORD) runs_flush<MET, kMS, runs_for<MET, VKL>(), kIntRuns<ORD, MET, VKL>, kWin4<MET, VKL> || kWinMK<ORD, HIST, MET, VKL>, kWinSlots<ORD, HIST, MET, VKL>>(P, s, run);
            if constexpr (PI && (ESGPU_PI_HOT != 0 || ESGPU_PI_HOTU != 0)) pi_hot_flush<MET>(P, s, run, T);
            if constexpr (kOrdHHot<ORD, HIST, MET, VKL>) cnt_hot_flush(s, run, T, P.hot_t[0]);
            if constexpr (PI) flush_window_pi<MET, WGS>(P, s, T, W, win0, ncp);
            else flush_window<MET, kMS, WGS>(P, s, T, W, win0, ncp);
        }
        dirty = false;
        win0 = k0;
        win_set = true;
        base = (P.key0 + (int64_t)win0) * P.interval + P.offset;
    };
    auto step = [&](uint32_t it, Buf& q) {
        if (it == 0) {
            // ---- per-group / per-block decisions (wave-uniform: every lane reads the same zone-map words) ----
            // readfirstlane: the zone-map words become scalar loads (lgkmcnt), not vector loads whose vmcnt wait
            // would drain the prefetched buffers
            const uint32_t b = __builtin_amdgcn_readfirstlane(cb);
            if (cb == gb && pass == 0) {
                if (dyn) {  // publish the pending claim (the chunk after this one), then claim the one after that
                    if (threadIdx.x == 0) claim_lds[claim_k & 1] = gridDim.x + claim_pend;
                    __syncthreads();
                    nxt_c = __builtin_amdgcn_readfirstlane(claim_lds[claim_k & 1]);
                    if (threadIdx.x == 0 && nxt_c < P.n_chunks) claim_pend = claim_chunk(P.claim);
                    ++claim_k;
                }
                use_lds = P.lds_mode != 0;
                npass = 1;
                if (use_lds && HIST && P.windowed) {
                    int64_t gmn = INT64_MAX, gmx = INT64_MIN, maxspan = 0;
                    for (uint32_t x = b; x < ge; ++x) {
                        const int64_t kmn = P.zkey[2 * x], kmx = P.zkey[2 * x + 1];
                        if (kmn > kmx) continue;  // no timestamp in the block
                        gmn = kmn < gmn ? kmn : gmn;
                        gmx = kmx > gmx ? kmx : gmx;
                        maxspan = kmx - kmn + 1 > maxspan ? kmx - kmn + 1 : maxspan;
                    }
                    if (maxspan > (int64_t)W) {
                        const int64_t span = gmx - gmn + 1;
                        if (span > (int64_t)W * kMaxPasses) {
                            use_lds = false;  // the group spans too many keys: global atomics for it
                        } else {
                            npass = (uint32_t)((span + W - 1) / W);
                            if (!win_set || (uint32_t)gmn != win0) slide_to((uint32_t)gmn);
                        }
                    }
                }
            } else if (HIST && npass > 1 && cb == gb) {  // next pass over a multi-pass group: the window moves up W keys
                slide_to(win0 + W);
            }
            if (HIST && use_lds && P.windowed && npass == 1) {  // block by block: slide the window when it must
                const int64_t kmn = P.zkey[2 * b], kmx = P.zkey[2 * b + 1];
                if (kmn <= kmx) {
                    if (!win_set || kmn < (int64_t)win0 || kmx >= (int64_t)win0 + (int64_t)W) slide_to((uint32_t)kmn);
                }
            }
        }
        bool uni = false;  // packed cells, a full zone block of one key (wave-uniform test): the uniform-slot path
        if constexpr (kPIU) {
            const Doc4* qa;
            const Doc4* qz;
            if constexpr (WIDE8) { qa = &q.a; qz = &q.b; } else { qa = &q; qz = &q; }
            uni = use_lds && qa->ukey != kNoUKey && (uint32_t)__builtin_amdgcn_readlane((int)qz->doc0, 63) + 4u <= P.n_docs;
            if (uni) {
                if constexpr (WIDE8 && MET >= 2) {  // (the (min, max) regions: one half at a time -- registers)
                    pi_uniform<MET, VKL, 1>(P, s, *qa, *qa, T, win0, run, npass > 1 ? W : 0u, pass == 0);
                    pi_uniform<MET, VKL, 1>(P, s, *qz, *qz, T, win0, run, npass > 1 ? W : 0u, pass == 0);
                } else {
                    pi_uniform<MET, VKL, WIDE8 ? 2 : 1>(P, s, *qa, *qz, T, win0, run, npass > 1 ? W : 0u, pass == 0);
                }
                dirty = true;
            }
        }
        if (uni) {
        } else if (use_lds) {
            if constexpr (WIDE8) {
                process4<ORD, HIST, MET, true, KT, kMS, HORD, VKL>(P, s, q.a, T, base, win0, run, npass > 1 ? W : 0u, pass == 0);
                process4<ORD, HIST, MET, true, KT, kMS, HORD, VKL>(P, s, q.b, T, base, win0, run, npass > 1 ? W : 0u, pass == 0);
            } else {
                process4<ORD, HIST, MET, true, KT, kMS, HORD, VKL>(P, s, q, T, base, win0, run, npass > 1 ? W : 0u, pass == 0);
            }
            dirty = true;
        } else {
            if constexpr (WIDE8) {
                process4<ORD, HIST, MET, false, KT, kMS, HORD, VKL>(P, g, q.a, T, base, win0, run);
                process4<ORD, HIST, MET, false, KT, kMS, HORD, VKL>(P, g, q.b, T, base, win0, run);
            } else {
                process4<ORD, HIST, MET, false, KT, kMS, HORD, VKL>(P, g, q, T, base, win0, run);
            }
        }
        // prefetch kBuf iterations ahead along the schedule (next block of the group, the group's next pass, or the
        // next group)
        uint32_t nit = it + kBuf, nb = cb;
        if (nit >= (uint32_t)kItersPerBlockW) {
            nit -= kItersPerBlockW;
            nb = cb + 1;
            if (nb == ge && pass + 1 < npass) nb = gb;
            else if (dyn && nb == ge) nb = nxt_c < P.n_chunks ? nxt_c * kGroup : cb;
            nb = min(nb, b_end - 1);
        }
        if (nb != pf_blk) {
            pf_blk = nb;
            pf_uk = zone_ukey(nb);
        }
        load_buf(nb * kBlockDocs + nit * kIterDocsW + tid4, q, pf_uk);
    };
    while (cb < b_end) {
        for (uint32_t it = 0; it < (uint32_t)kItersPerBlockW; it += kBuf) {
#pragma unroll
            for (int k = 0; k < kBuf; ++k) step(it + k, q[k]);
        }
        if (++cb == ge) {
            if (++pass < npass) {
                cb = gb;
            } else {
                pass = 0;
                npass = 1;
                if (dyn) {
                    if (nxt_c >= P.n_chunks) break;
                    gb = cb = nxt_c * kGroup;
                } else {
                    gb = ge;
                }
                ge = min(gb + kGroup, b_end);
            }
        }
    }
#ifndef ESGPU_FLUSH_DIAG  // timing experiment only (wrong results): 1 = no final window flush
#define ESGPU_FLUSH_DIAG 0
#endif
    if (P.lds_mode && (dirty || !(HIST && P.windowed)) && !ESGPU_FLUSH_DIAG) {
        if (!ORD) runs_flush<MET, kMS, runs_for<MET, VKL>(), kIntRuns<ORD, MET, VKL>, kWin4<MET, VKL> || kWinMK<ORD, HIST, MET, VKL>, kWinSlots<ORD, HIST, MET, VKL>>(P, s, run);
        if constexpr (PI && (ESGPU_PI_HOT != 0 || ESGPU_PI_HOTU != 0)) pi_hot_flush<MET>(P, s, run, T);
        if constexpr (kOrdHHot<ORD, HIST, MET, VKL>) cnt_hot_flush(s, run, T, P.hot_t[0]);
        if constexpr (PI) flush_window_pi<MET, WGS>(P, s, T, W, win0, ncp);
        else flush_window<MET, kMS, WGS>(P, s, T, W, win0, ncp);
    }
    if (dyn && threadIdx.x == 0) {  // the last workgroup to finish re-arms the counter pair (vector atomics only)
        __threadfence();
        if (atomicAdd(&P.claim[1], 1u) == gridDim.x - 1) {
            atomicExch(&P.claim[0], 0u);
            atomicExch(&P.claim[1], 0u);
        }
    }
}

// per-block key range [kmn, kmx] of a windowed collect (the zone maps mapped through the request's rounding once, so
// the collect kernel's per-block window decisions are two scalar loads instead of two 64-bit divisions or table
// searches per block); a block without values gets (1, 0)
// udocs (optional): the docs of the blocks whose range rounds to one key, summed -- the block-delta kernels read no
// timestamp of those blocks (zone_ukey), and the plan's byte count leaves them out
template <bool KT>
__global__ __launch_bounds__(256) void zone_keys_kernel(CollectParams P, int64_t* __restrict__ out,
                                                        unsigned long long* __restrict__ udocs) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long ud = 0;
    if (b < P.n_blocks) {
        const int64_t zmn = P.zmin[b], zmx = P.zmax[b];
        int64_t kmn = 1, kmx = 0;
        if (zmn <= zmx) {
            kmn = key_index<KT>(P, zmn);
            kmx = key_index<KT>(P, zmx);
        }
        out[2 * (size_t)b] = kmn;
        out[2 * (size_t)b + 1] = kmx;
        const uint64_t d0 = (uint64_t)b * kBlockDocs;
        if (kmn == kmx && d0 < P.n_docs) ud = min((uint64_t)kBlockDocs, (uint64_t)P.n_docs - d0);
    }
    if (udocs) {  // the workgroup's single-key docs into its own word (no shared counter: one atomic per wave on one
                  // address had made this kernel 26 us at 1B docs)
        __shared__ unsigned long long wsum[4];
        for (int o = 32; o > 0; o >>= 1) ud += __shfl_xor(ud, o, 64);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = ud;
        __syncthreads();
        if (threadIdx.x == 0) udocs[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    }
}

// calls f(std::integral_constant<int, VK>) for the value kinds the plan uses; bits that cannot matter (no histogram
// dimension, no metric) are never instantiated
template <int HK, int MET, class F>
static auto with_vk0(bool hv_f64, bool mv_f64, F f) {
    const bool hf = HK != 0 && hv_f64, mf = MET > 0 && mv_f64;
    if constexpr (HK == 3) {  // ordinal keys: only the metric's kind varies
        if constexpr (MET > 0) {
            if (mf) return f(std::integral_constant<int, 2>{});
        }
        return f(std::integral_constant<int, 0>{});
    } else if constexpr (HK != 0 && MET > 0) {
        if (hf && mf) return f(std::integral_constant<int, 3>{});
        if (hf) return f(std::integral_constant<int, 1>{});
        if (mf) return f(std::integral_constant<int, 2>{});
        return f(std::integral_constant<int, 0>{});
    } else if constexpr (HK != 0) {
        if (hf) return f(std::integral_constant<int, 1>{});
        return f(std::integral_constant<int, 0>{});
    } else if constexpr (MET > 0) {
        if (mf) return f(std::integral_constant<int, 2>{});
        return f(std::integral_constant<int, 0>{});
    } else {
        return f(std::integral_constant<int, 0>{});
    }
}
// VK bit 8: the terms dimension is a derived histogram key index (CollectParams.ord_src); only for ORD x histogram grids.
// Bits 16 / 32 (compact ordinal / histogram columns): terms dimensions without a derived key index, affine histograms
// over a long column.
template <bool ORD, int HK, int MET, class F>
static auto with_vk(bool hv_f64, bool mv_f64, bool dord, bool c16, bool t32, bool t16, bool pi, bool m32, bool m16, bool acc,
                    bool raw, bool runs1, bool uk32, bool noc, F f) {
    // t16: the key column is read as block deltas (VK bit 8192 in place of 32) -- by the raw-load kernels only; the host
    // picks it only for a launch that takes one of them (t32 is then set as well)
    // VK bit 128, a compact long metric (u32 deltas, values restored in the loader): histogram-only grids over compact
    // timestamps (date_histogram{stats / extended_stats / avg}) and extended_stats under terms over compact columns
    if constexpr (MET > 0 && !ORD && HK == 1) {
        if (m32 && !pi && !mv_f64 && t32 && !hv_f64) {
            if (raw && m16 && runs1 && t16) return f(std::integral_constant<int, 8192 | 128 | 1024 | 2048 | 4096>{});
            if (raw && m16 && t16) return f(std::integral_constant<int, 8192 | 128 | 1024 | 2048>{});
            if (raw && t16) return f(std::integral_constant<int, 8192 | 128 | 1024>{});
            if (raw && uk32) {  // (32-bit deltas skipping single-key zone blocks)
                if (m16 && runs1) return f(std::integral_constant<int, 16384 | 32 | 128 | 1024 | 2048 | 4096>{});
                if (m16) return f(std::integral_constant<int, 16384 | 32 | 128 | 1024 | 2048>{});
                return f(std::integral_constant<int, 16384 | 32 | 128 | 1024>{});
            }
            if (raw && m16 && runs1) return f(std::integral_constant<int, 32 | 128 | 1024 | 2048 | 4096>{});
            if (raw && m16) return f(std::integral_constant<int, 32 | 128 | 1024 | 2048>{});
            if (raw) return f(std::integral_constant<int, 32 | 128 | 1024>{});
            return f(std::integral_constant<int, 32 | 128>{});
        }
    }
    if constexpr (MET == 0 && !ORD && HK == 1) {
        if (raw && t16 && !hv_f64) return f(std::integral_constant<int, 8192 | 1024>{});
        if (raw && t32 && uk32 && !hv_f64) return f(std::integral_constant<int, 16384 | 32 | 1024>{});
        if (raw && t32 && !hv_f64) return f(std::integral_constant<int, 32 | 1024>{});
    }
    if constexpr (MET == 0 && ORD && (HK == 0 || HK == 1)) {  // counting terms grids over 16-bit ordinals
        if (raw && c16 && !dord) {
            if constexpr (HK == 1) {
                if (t16 && !hv_f64) return f(std::integral_constant<int, 16 | 8192 | 1024>{});
                if (t32 && uk32 && !hv_f64) return f(std::integral_constant<int, 16384 | 48 | 1024>{});
                if (t32 && !hv_f64) return f(std::integral_constant<int, 48 | 1024>{});
            } else {
                return f(std::integral_constant<int, 16 | 1024>{});
            }
        }
    }
    if constexpr (MET == 3 && ORD && (HK == 0 || HK == 1)) {
        if (m32 && !pi && !mv_f64 && !dord && c16) {
            if constexpr (HK == 1) {
                if (t32 && !hv_f64) return f(std::integral_constant<int, 48 | 128>{});
            } else {
                return f(std::integral_constant<int, 16 | 128>{});
            }
        }
    }
    // VK bit 64, packed integer metric cells: terms grids (no key, or an affine key over the compact timestamps) with
    // avg / stats over a dense long metric
    // (+ bit 256: the 16-bit deltas, with 16-bit ordinals only; + bit 512: filtered through one accept bitset, with the
    // 16-bit deltas only -- the host keeps the f64 cells for other filtered shapes)
    if constexpr (ORD && (HK == 0 || HK == 1) && (MET == 1 || MET == 2)) {
        if (pi && !mv_f64 && !dord) {
            if constexpr (HK == 1) {
                if (t32 && !hv_f64) {
                    // (+ bit 32768: the plan's outer counts are derived at the flush, none counted per doc)
                    if (c16 && m16 && acc && t16 && noc) return f(std::integral_constant<int, 32768 | 16 | 8192 | 64 | 256 | 512>{});
                    if (c16 && m16 && t16 && noc) return f(std::integral_constant<int, 32768 | 16 | 8192 | 64 | 256>{});
                    if (c16 && m16 && acc && uk32 && noc) return f(std::integral_constant<int, 32768 | 16384 | 48 | 64 | 256 | 512>{});
                    if (c16 && m16 && uk32 && noc) return f(std::integral_constant<int, 32768 | 16384 | 48 | 64 | 256>{});
                    if (c16 && m16 && acc && t16) return f(std::integral_constant<int, 16 | 8192 | 64 | 256 | 512>{});
                    if (c16 && m16 && t16) return f(std::integral_constant<int, 16 | 8192 | 64 | 256>{});
                    if (c16 && m16 && acc && uk32) return f(std::integral_constant<int, 16384 | 48 | 64 | 256 | 512>{});
                    if (c16 && m16 && uk32) return f(std::integral_constant<int, 16384 | 48 | 64 | 256>{});
                    if (c16 && m16 && acc) return f(std::integral_constant<int, 48 | 64 | 256 | 512>{});
                    if (c16 && m16) return f(std::integral_constant<int, 48 | 64 | 256>{});
                    if (c16) return f(std::integral_constant<int, 48 | 64>{});
                    return f(std::integral_constant<int, 32 | 64>{});
                }
            } else {
                if (c16 && m16 && acc) return f(std::integral_constant<int, 16 | 64 | 256 | 512>{});
                if (c16 && m16) return f(std::integral_constant<int, 16 | 64 | 256>{});
                if (c16) return f(std::integral_constant<int, 16 | 64>{});
                return f(std::integral_constant<int, 64>{});
            }
        }
    }
    if constexpr (ORD && (HK == 1 || HK == 2)) {
        if (dord)
            return with_vk0<HK, MET>(hv_f64, mv_f64, [&](auto vk) { return f(std::integral_constant<int, decltype(vk)::value | 8>{}); });
    }
    if constexpr (HK == 1) {
        if (t32 && !hv_f64) {
            if constexpr (ORD) {
                if (c16)
                    return with_vk0<HK, MET>(false, mv_f64, [&](auto vk) { return f(std::integral_constant<int, decltype(vk)::value | 48>{}); });
            }
            return with_vk0<HK, MET>(false, mv_f64, [&](auto vk) { return f(std::integral_constant<int, decltype(vk)::value | 32>{}); });
        }
    }
    if constexpr (ORD && (HK == 0 || HK == 1)) {
        if (c16)
            return with_vk0<HK, MET>(hv_f64, mv_f64, [&](auto vk) { return f(std::integral_constant<int, decltype(vk)::value | 16>{}); });
    }
    return with_vk0<HK, MET>(hv_f64, mv_f64, f);
}

// wide = 1024-thread workgroups (instantiated for histogram grids only)
template <bool ORD, int HK, int MET, class F>
static auto with_wg(bool wide, F f) {
    if constexpr (HK == 1 || HK == 2) {
        if (wide) return f(std::integral_constant<int, 1024>{});
    }
    return f(std::integral_constant<int, kWG>{});
}

template <bool ORD, int HK, int MET>
static void launch_t(const CollectParams& p, bool wide, uint32_t grid, size_t lds, hipStream_t st) {
    with_vk<ORD, HK, MET>(p.hv_f64 != 0, p.mv_f64 != 0, p.ord_src != nullptr, p.ord16 != nullptr,
                          p.hv32 != nullptr || p.hv16 != nullptr, p.hv16 != nullptr, (p.mv32 || p.mv16) && p.pk_shift != 0, (p.mv32 || p.mv16) && p.pk_shift == 0, p.mv16 != nullptr,
                          p.accept != nullptr, p.raw_dense != 0, p.runs1 != 0, p.ukey32 != 0,
                          p.ocnt_mode != OCNT_TERMS && p.ocnt_mode != OCNT_HIST, [&](auto vk) {
        return with_wg<ORD, HK, MET>(wide, [&](auto wg) {
            hipLaunchKernelGGL((collect_kernel<ORD, HK, MET, decltype(vk)::value, decltype(wg)::value>), dim3(grid),
                               dim3(decltype(wg)::value), lds, st, p);
            return 0;
        });
    });
}

template <bool ORD, int HK>
static void launch_m(const CollectParams& p, int met, bool wide, uint32_t grid, size_t lds, hipStream_t st) {
    switch (met) {
        case 0: launch_t<ORD, HK, 0>(p, wide, grid, lds, st); break;
        case 1: launch_t<ORD, HK, 1>(p, wide, grid, lds, st); break;
        case 2: launch_t<ORD, HK, 2>(p, wide, grid, lds, st); break;
        default: launch_t<ORD, HK, 3>(p, wide, grid, lds, st); break;
    }
}

template <bool ORD, int HK, int MET>
static int occ_t(size_t lds, int vkbits, bool wide) {
    return with_vk<ORD, HK, MET>((vkbits & 1) != 0, (vkbits & 2) != 0, (vkbits & 8) != 0, (vkbits & 16) != 0,
                                 (vkbits & (32 | 8192)) != 0, (vkbits & 8192) != 0, (vkbits & 64) != 0, (vkbits & 128) != 0, (vkbits & 256) != 0,
                                 (vkbits & 512) != 0, (vkbits & 1024) != 0, (vkbits & 4096) != 0, (vkbits & 16384) != 0,
                                 (vkbits & 32768) != 0, [&](auto vk) {
        return with_wg<ORD, HK, MET>(wide, [&](auto wg) {
            int n = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &n, collect_kernel<ORD, HK, MET, decltype(vk)::value, decltype(wg)::value>, decltype(wg)::value, lds) !=
                hipSuccess)
                n = 1;
            return n;
        });
    });
}
template <bool ORD, int HK>
static int occ_m(int met, size_t lds, int vk, bool wide) {
    switch (met) {
        case 0: return occ_t<ORD, HK, 0>(lds, vk, wide);
        case 1: return occ_t<ORD, HK, 1>(lds, vk, wide);
        case 2: return occ_t<ORD, HK, 2>(lds, vk, wide);
        default: return occ_t<ORD, HK, 3>(lds, vk, wide);
    }
}
// explicit instantiations live in esgpu_collect_inst.hip (one object per ORD x HK x MET)
template <bool ORD, int HK, int MET>
void launch_collect_met(const CollectParams& p, bool wide, uint32_t grid, size_t lds, hipStream_t st);
template <bool ORD, int HK, int MET>
int collect_occ_met(size_t lds, int vk, bool wide);
template <bool ORD, int HK>
void launch_collect_inst(const CollectParams& p, int met, bool wide, uint32_t grid, size_t lds, hipStream_t st) {
    switch (met) {
        case 0: launch_collect_met<ORD, HK, 0>(p, wide, grid, lds, st); break;
        case 1: launch_collect_met<ORD, HK, 1>(p, wide, grid, lds, st); break;
        case 2: launch_collect_met<ORD, HK, 2>(p, wide, grid, lds, st); break;
        default: launch_collect_met<ORD, HK, 3>(p, wide, grid, lds, st); break;
    }
}
template <bool ORD, int HK>
int collect_occ_inst(int met, size_t lds, int vk, bool wide) {
    switch (met) {
        case 0: return collect_occ_met<ORD, HK, 0>(lds, vk, wide);
        case 1: return collect_occ_met<ORD, HK, 1>(lds, vk, wide);
        case 2: return collect_occ_met<ORD, HK, 2>(lds, vk, wide);
        default: return collect_occ_met<ORD, HK, 3>(lds, vk, wide);
    }
}

}  // namespace esgpu
