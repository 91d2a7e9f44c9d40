// esgpu_hotcold.hip — K1 for high-cardinality terms (valueCount >> LDS, e.g. 10M url ordinals), hot/cold partitioned
// counting.  Replaces GlobalOrdinalsStringTermsAggregator.collect's `docCounts.increment(globalOrd)` over a BigArrays
// LongArray of valueCount counters (A/bucket/terms/GlobalOrdinalsStringTermsAggregator.java:107-135) for the request
// shapes whose counters cannot be privatised in LDS.
//
// Three facts of the segment, gathered once per ordinal column and cached beside it the way Elasticsearch caches a
// field's global ordinals (HcStats in esgpu_runtime.cpp, built on first use):
//   * the hot set: the most frequent ordinals (Zipf-like term distributions put most docs on a few thousand), numbered
//     by frequency (hot slots);
//   * a recoded copy of the ordinal column in which a hot ordinal reads kHcHotBit | its slot: telling hot from cold is
//     one bit test, and a hot doc is one LDS add at its slot (no lookup);
//   * per partition (32768 ordinals) the number of docs whose ordinal is not hot, which bounds what any request over
//     the segment (any filter, any accept bitset) can write into that partition: the capacities of the partitioned
//     buffer are therefore known before the request runs, and no histogram pass over the docs is needed.
// Request passes:
//   hc_init      reset the overflow cursors and the capacity flag
//   hc_scatter   ONE read of the recoded column (4 B/doc): hot slots counted in LDS, cold ordinals through per-partition
//                LDS rings out to the workgroup's static region of the partition as whole 64-byte segments of 16-bit
//                partition-local offsets (overflow: 64-element-aligned chunks from the partition's overflow pool, one
//                global atomic per chunk)
//   hc_count     one workgroup per piece of a partition (one piece unless the partition is far above the average): the
//                static regions (holes masked by the per-workgroup fill) and the overflow pool counted into LDS (two
//                16-bit counters per word when the segment's cold counts fit), then one coalesced pass over the counters
//   hc_hot_reduce  the per-workgroup hot counters summed per slot and added to their ordinals
// Scatter workgroups: 512 threads, two per CU when the LDS layout fits, so one workgroup's barrier phases overlap the
// other's loads.
// Traffic: 4 B/doc + 2 x 2 B per cold doc (~43 % of docs on the Zipf(1) url field) + 8-16 B per ordinal (counters).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "es_common.hpp"
#include "esgpu_collect.hpp"
#include "esgpu_kernels.hpp"

namespace esgpu {

constexpr int kHcWG = 512;                           // scatter: 8 waves, two workgroups per CU (P <= 512)
constexpr int kHcIt = 4;                             // 16-byte loads per thread per tile
constexpr uint32_t kHcTileDocs = kHcWG * kHcIt * 4;  // 8192 docs per tile (<= kHcTile, the spare elements of pbuf)
constexpr uint32_t kHcNone = 0xFFFFFFFFu;
constexpr int kHcCountWG = 1024;                     // counting: 16 waves, 4 vectors in flight per thread

__device__ __forceinline__ uint32_t hc_hash(uint32_t o, uint32_t log2) { return (o * 0x9E3779B1u) >> (32 - log2); }

__global__ void hc_recode_kernel(const uint32_t* ord, uint32_t n, const uint32_t* keys, const uint32_t* vals,
                                 uint32_t log2, uint32_t* out) {
    const uint32_t mask = (1u << log2) - 1u;
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < n; d += gridDim.x * blockDim.x) {
        const uint32_t o = ord[d];
        uint32_t r = o;
        if (o != kMissingOrd)
            for (uint32_t h = hc_hash(o, log2);; h = (h + 1) & mask) {
                const uint32_t k = keys[h];
                if (k == o) { r = kHcHotBit | vals[h]; break; }
                if (k == kMissingOrd) break;
            }
        out[d] = r;
    }
}
void launch_hc_recode(const uint32_t* ord, uint32_t n, const uint32_t* keys, const uint32_t* vals, uint32_t log2,
                      uint32_t* out, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(hc_recode_kernel, dim3(std::min<uint32_t>(8192, (n + 255) / 256)), dim3(256), 0, s, ord, n, keys,
                       vals, log2, out);
}

__global__ void hc_hot16_kernel(const uint32_t* rc, uint32_t n, uint16_t* out) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < n; d += gridDim.x * blockDim.x) {
        const uint32_t v = rc[d];
        // hot slot, 0xFFFE for a cold ordinal (counted as one total by a filtered request's hot pass), 0xFFFF missing
        out[d] = v == kMissingOrd ? (uint16_t)0xFFFFu : (v & kHcHotBit) ? (uint16_t)(v & ~kHcHotBit) : (uint16_t)0xFFFEu;
    }
}
void launch_hc_hot16(const uint32_t* rc, uint32_t n, uint16_t* out, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(hc_hot16_kernel, dim3(std::min<uint32_t>(8192, (n + 255) / 256)), dim3(256), 0, s, rc, n, out);
}

__global__ void hc_init_kernel(HcParams P) {
    if (P.skip && *P.skip) return;  // (the hot slots settled the request's top-k: hc_topk_launch)
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < P.P; p += gridDim.x * blockDim.x)
        P.ovf_cur[p] = P.part[p].ovf_base;
}  // P.err is zeroed by the host (after each check), so overruns of every segment of a request accumulate

// Cold ordinals leave the workgroup only as whole, aligned 64-byte segments (32 offsets; every region and chunk is a
// multiple of 64 elements).  Each partition owns a 64-slot ring in LDS: a cold doc's single LDS atomic on the
// partition's word returns its sequence number c since the last flush and the ring half in use, so the doc is written
// straight into its ring slot; after the tile every full 32-offset half goes out as one 64-byte store from four lanes.
// A partition that receives more than 64 - pending offsets in one tile (clustered data) writes the excess straight to
// memory from registers.  (Appending each tile's few offsets per partition to memory left lines partly written in L2:
// WRITE_SIZE 3x the cold bytes; an LDS counting sort of the tile cost twice the LDS instructions of the ring.)
#ifndef ESGPU_HC_NT
#define ESGPU_HC_NT 1
#endif
#ifndef ESGPU_HC_EXP  // timing experiments only: 1 = classify alone (steps 2-5 and the flush skipped), 2 = loads alone
#define ESGPU_HC_EXP 0
#endif
constexpr uint32_t kSeg = 32;
constexpr uint32_t kRing = 2 * kSeg;
constexpr uint32_t kCnt = (1u << 26) - 1u;  // word: ring base (0 or 32) << 26 | offsets since the last flush
// ring slot k of partition p in LDS (u16 units): the 16-byte granules of a partition's ring are XOR-swizzled by p, so the
// same slot of different partitions falls on different banks (rows are 128 B = exactly the 32 banks of a dword store;
// slots advance in step across partitions, so an unswizzled ring write is a many-way bank conflict)
__device__ __forceinline__ uint32_t ring_idx(uint32_t p, uint32_t k) {
    return p * kRing + ((((k >> 3) ^ p) & 7u) << 3) + (k & 7u);
}

size_t hc_scatter_lds_bytes(uint32_t n_parts, uint32_t hot_n) {
    // hot counters | rings (u16 x 64) | stp (16 B) + word, cpos, cend
    return (((size_t)hc_hot_counters(hot_n) * 4 + 15) & ~(size_t)15) + (size_t)n_parts * (kRing * 2 + 16 + 3 * 4);
}

template <bool HOT>
__global__ __launch_bounds__(kHcWG) void hc_scatter_kernel(HcParams P) {
    if (P.skip && *P.skip) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t NH = HOT ? hc_hot_counters(P.hot_n) : 0u;
    uint32_t* hot = (uint32_t*)smem;                        // [NH] hot counters (slot s < 64: 4 s + lane % 4)
    uint16_t* ring = (uint16_t*)(smem + ((NH * 4 + 15) & ~15u));  // [P][64] (16-byte aligned: read as uint4)
    uint4* stp = (uint4*)(ring + (size_t)P.P * kRing);      // [P] this tile: {split, base A, base B, ring base | L << 8}
    uint32_t* word = (uint32_t*)(stp + P.P);                // [P] ring base << 26 | offsets since the last flush
    uint32_t* cpos = word + P.P;                            // [P] next element of the workgroup's current chunk
    uint32_t* cend = cpos + P.P;                            // [P] end of that chunk
    const uint32_t word_off = (uint32_t)((unsigned char*)word - smem);
    const uint32_t w = blockIdx.x;
    constexpr uint32_t kMask = (1u << kPartShift) - 1u;
    for (uint32_t i = threadIdx.x; i < NH; i += kHcWG) hot[i] = 0u;
    for (uint32_t p = threadIdx.x; p < P.P; p += kHcWG) {
        const HcPart q = P.part[p];
        word[p] = 0u;
        cpos[p] = q.sbase + w * q.chunk;
        cend[p] = cpos[p] + q.chunk;
    }
    __syncthreads();
    // destination of `len` more elements of partition p: the rest of the current chunk, then a fresh overflow chunk
    // (a returning global atomic; 64-element aligned); returns {split, base A, base B}: element i -> i < split ? A + i
    // : B + i.  `avail` and every length reserved during the tiles are multiples of 32, so a segment never straddles.
    auto reserve = [&](uint32_t p, uint32_t len) -> uint3 {
        const uint32_t a = cpos[p], avail = cend[p] - a;
        if (len <= avail) {
            cpos[p] = a + len;
            return make_uint3(len, a, a);
        }
        const HcPart q = P.part[p];
        const uint32_t need = len - avail;
        const uint32_t sz = max(q.ovf_chunk, (need + 63u) & ~63u);
        uint32_t nb = atomicAdd(&P.ovf_cur[p], sz);
        uint32_t end = nb + sz;
        if (end > q.cap_end || end < nb) {  // cannot happen by construction of the capacities
            *P.err = 1u;
            nb = P.trash;                   // keep every write inside pbuf (kHcTile spare elements)
            end = nb + need;
        }
        cpos[p] = nb + need;
        cend[p] = end;
        return make_uint3(avail, a, nb - avail);
    };
    const uint32_t b_begin = min(w * P.blocks_per_wg, P.n_blocks);
    const uint32_t b_end = min(b_begin + P.blocks_per_wg, P.n_blocks);
    const uint32_t d_begin = b_begin * kBlockDocs;
    const uint32_t d_end = min(b_end * kBlockDocs, P.n_docs);
    // loads past the range re-read the workgroup's own last quad (an L2 hit), not the next workgroup's docs from HBM
    const uint32_t d_last = (b_end > b_begin ? b_end : P.n_blocks) * kBlockDocs - 4;
    const uint32_t tid4 = threadIdx.x * 4;
    auto load = [&](uint32_t t0, uint32_t o[kHcIt][4]) {
#pragma unroll
        for (int k = 0; k < kHcIt; ++k) {
            const uint32_t d = min(t0 + k * (kHcWG * 4) + tid4, d_last);
#if ESGPU_HC_NT  // the column is read once: non-temporal loads keep L2 for the partitions' open segments (5 % faster)
            const u32x4_t a = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(P.rc + d));
            o[k][0] = a.x; o[k][1] = a.y; o[k][2] = a.z; o[k][3] = a.w;
#else
            load_u32x4(P.rc, d, o[k]);
#endif
        }
    };
    auto process = [&](uint32_t t0, const uint32_t o[kHcIt][4]) {
        // 1. classify: hot -> LDS counter; cold -> sequence number in the partition's ring (written when it fits).
        //    Straight-line phases over the thread's 16 docs, so each phase's LDS operations issue back to back and
        //    their latencies overlap (hot adds + returning adds on the partition words; ring writes).
        constexpr int kD = kHcIt * 4;
        uint32_t rk[kHcIt][4];
        uint32_t okm = 0;  // bit d: doc d counts
#pragma unroll
        for (int k = 0; k < kHcIt; ++k) {
            const uint32_t doc0 = t0 + k * (kHcWG * 4) + tid4;
            uint32_t ok = 0u;
            if (doc0 < d_end) ok = doc0 + 4 <= d_end ? 0xFu : ((1u << (d_end - doc0)) - 1u);
            if (ok && P.accept) ok &= bits4(P.accept, doc0);
            for (int q = 0; q < P.npred && ok; ++q) ok &= eval_pred(P.pred[q], doc0);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t v = o[k][j];
                const bool c = (v & kHcHotBit) ? v != kMissingOrd : v < P.T;
                okm |= (((ok >> j) & 1u) && c ? 1u : 0u) << (k * 4 + j);
            }
        }
#if ESGPU_HC_EXP == 2
        {
            uint32_t acc = 0;
#pragma unroll
            for (int d = 0; d < kD; ++d) acc += ((okm >> d) & 1u) ? o[d / 4][d % 4] : 0u;
            if (acc == 0x12345678u) hot[0] = acc;
            return;
        }
#endif
        // one LDS atomic per doc: a hot doc adds at its slot's counter (the 64 most frequent slots spread over 4 lane-
        // rotated copies), a cold doc at its partition's word and keeps the returned sequence number; one
        // ds_add_rtn_u32 with per-lane addresses serves both (two instructions cost twice: LDS atomics are issue-bound)
        uint32_t old[kD];
#pragma unroll
        for (int d = 0; d < kD; ++d) {
            const uint32_t v = o[d / 4][d % 4];
            const bool hb = (v & kHcHotBit) != 0u;
            const uint32_t sl = v & ~kHcHotBit;
            // one LDS address (a byte offset from smem: a select between two pointers compiles to flat atomics)
            const uint32_t off = hb ? (sl < kHcHotCopies ? 4 * sl + (threadIdx.x & 3) : 3 * kHcHotCopies + sl) * 4u
                                    : word_off + (v >> kPartShift) * 4u;
            old[d] = ((okm >> d) & 1u) ? atomicAdd((uint32_t*)(smem + off), 1u) : kHcNone;
            if (hb) old[d] = kHcNone;
        }
        bool burst = false;
#pragma unroll
        for (int d = 0; d < kD; ++d) {
            const uint32_t v = o[d / 4][d % 4];
            const uint32_t r = old[d] == kHcNone ? kHcNone : (old[d] & kCnt);
            if (r < kRing) ring[ring_idx(v >> kPartShift, ((old[d] >> 26) + r) & (kRing - 1))] = (uint16_t)(v & kMask);
            burst |= r != kHcNone && r >= kRing;
            rk[d / 4][d % 4] = r;
        }
        const bool any_burst = __syncthreads_or(burst);
#if ESGPU_HC_EXP == 1
        return;
#endif
        // 2. per partition: whole segments to flush (L), their destination, the ring state after the flush
        for (uint32_t p = threadIdx.x; p < P.P; p += kHcWG) {
            const uint32_t wd = word[p], C = wd & kCnt, rb = wd >> 26;
            const uint32_t L = C & ~(kSeg - 1);
            if (L) {
                const uint3 d = reserve(p, L);
                stp[p] = make_uint4(d.x, d.y, d.z, rb | (L << 8));
                word[p] = (((rb + L) & (kRing - 1)) << 26) | (C - L);
            } else {
                stp[p].w = rb;  // bursts need the ring base only when L > 0; keep w coherent for step 5
            }
        }
        __syncthreads();
        // 3. offsets beyond the ring that are flushed this tile: straight to memory (clustered data only)
        if (any_burst) {
#pragma unroll
            for (int k = 0; k < kHcIt; ++k)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t r = rk[k][j];
                    if (r != kHcNone && r >= kRing) {
                        const uint32_t p = o[k][j] >> kPartShift;
                        const uint4 st = stp[p];
                        if (r < (st.w >> 8)) P.pbuf[r < st.x ? st.y + r : st.z + r] = (uint16_t)(o[k][j] & kMask);
                    }
                }
        }
        // 4. ring halves out: four lanes per 64-byte segment, 16 bytes each (partition p -> lane group p % (WG / 4))
        {
            const uint32_t grp = threadIdx.x >> 2, qt = threadIdx.x & 3;
            for (uint32_t p = grp; p < P.P; p += kHcWG / 4) {
                const uint4 st = stp[p];
                const uint32_t L = st.w >> 8, rb = st.w & 0xFFu;
                const uint32_t nseg = min(L, kRing) / kSeg;
                for (uint32_t sgi = 0; sgi < nseg; ++sgi) {
                    const uint32_t i0 = sgi * kSeg;  // sequence index of the segment's first offset
                    const uint32_t half = (rb + i0) & (kRing - 1);
                    const uint4 v = *reinterpret_cast<const uint4*>(ring + ring_idx(p, half + qt * 8));
                    *reinterpret_cast<uint4*>(P.pbuf + (i0 < st.x ? st.y + i0 : st.z + i0) + qt * 8) = v;
                }
            }
        }
        __syncthreads();
        // 5. burst offsets that stay pending: into the ring slots the flush freed
        if (any_burst) {
#pragma unroll
            for (int k = 0; k < kHcIt; ++k)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t r = rk[k][j];
                    if (r != kHcNone && r >= kRing) {
                        const uint32_t p = o[k][j] >> kPartShift;
                        const uint4 st = stp[p];
                        if (r >= (st.w >> 8)) ring[ring_idx(p, ((st.w & 0xFFu) + r) & (kRing - 1))] = (uint16_t)(o[k][j] & kMask);
                    }
                }
        }
        // the next tile's classify writes ring slots past the pending ones (step 2 set the words before two barriers);
        // step 5's slots are the pending ones, so no barrier is needed here
    };
    const uint32_t span = b_end > b_begin ? (b_end - b_begin) * kBlockDocs : 0u;
    if (span) {
        uint32_t A[kHcIt][4], B[kHcIt][4];
        // A's loads must issue before B's, as they do on the loop's back edge: the wait counts at the loop head are
        // merged over both paths, and with B issued first the head waited vmcnt(0), draining the prefetch every tile
        load(d_begin, A);
        __builtin_amdgcn_sched_barrier(0);
        load(d_begin + kHcTileDocs, B);
        for (uint32_t t0 = d_begin; t0 < d_begin + span; t0 += 2 * kHcTileDocs) {
            process(t0, A);
            load(t0 + 2 * kHcTileDocs, A);
            if (t0 + kHcTileDocs < d_begin + span) process(t0 + kHcTileDocs, B);
            load(t0 + 3 * kHcTileDocs, B);
        }
    }
    __syncthreads();
    // the partitions' pending offsets (one partial segment); static-region fill; sentinel tail of an overflow chunk
    for (uint32_t p = threadIdx.x; p < P.P && ESGPU_HC_EXP == 0; p += kHcWG) {
        const HcPart q = P.part[p];
        const uint32_t wd = word[p], f = wd & kCnt, rb = wd >> 26;
        if (f) {
            const uint3 d = reserve(p, f);
            for (uint32_t i = 0; i < f; ++i) P.pbuf[i < d.x ? d.y + i : d.z + i] = ring[ring_idx(p, (rb + i) & (kRing - 1))];
        }
        const uint32_t s0 = q.sbase + w * q.chunk;
        uint32_t used = q.chunk;
        if (cend[p] == s0 + q.chunk) {
            used = cpos[p] - s0;
        } else if (cpos[p] < cend[p] && cend[p] <= q.cap_end) {
            for (uint32_t e = cpos[p]; e < cend[p]; ++e) P.pbuf[e] = 0xFFFFu;
        }
        P.used[(size_t)p * P.G + w] = used;
    }
    if (HOT)
        for (uint32_t i = threadIdx.x; i < hc_slab_stride(P.hot_n); i += kHcWG)
            P.hot_slab[(size_t)w * hc_slab_stride(P.hot_n) + i] = i < NH ? hot[i] : 0u;
}

// one workgroup per piece: region elements [lo, hi) of partition p, where the region is the G static regions
// (element g * chunk + i, valid while i < used[g]) followed by the overflow pool (0xFFFF = unused)
template <bool U16>
__global__ __launch_bounds__(kHcCountWG) void hc_count_kernel(HcParams P) {
    if (P.skip && *P.skip) return;  // (the hot slots settled the request's top-k)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* cnt = (uint32_t*)smem;  // U16: [16384] two 16-bit counters per word, else [32768]
    uint32_t* used = cnt + (U16 ? (1u << kPartShift) / 2 : (1u << kPartShift));  // [G]
    const HcPiece pc = P.piece[blockIdx.x];
    const uint32_t p = pc.p;
    const HcPart q = P.part[p];
    const uint32_t nwords = U16 ? (1u << kPartShift) / 2 : (1u << kPartShift);
    for (uint32_t i = threadIdx.x; i < nwords; i += kHcCountWG) cnt[i] = 0u;
    for (uint32_t i = threadIdx.x; i < P.G; i += kHcCountWG) used[i] = P.used[(size_t)p * P.G + i];
    __syncthreads();
    auto add = [&](uint32_t v) {
        if (U16) atomicAdd(&cnt[v >> 1], 1u << ((v & 1u) * 16));
        else atomicAdd(&cnt[v], 1u);
    };
    // static regions: 8 elements per 16-byte vector (chunk is a multiple of 64: a vector never straddles two regions)
    const uint32_t cv = q.chunk / 8;  // vectors per region
    const uint32_t nstat = cv * P.G;  // vectors of the static part
    {
        const uint32_t k0 = pc.lo / 8, k1 = min(pc.hi / 8, nstat);
        if (k1 > k0) {
            const uint4* src = reinterpret_cast<const uint4*>(P.pbuf + q.sbase);
            auto count_vec = [&](uint32_t k, const uint4 v) {
                const uint32_t g = k / cv;
                const uint32_t r0 = (k - g * cv) * 8;
                const uint32_t u = used[g];
                const uint32_t m = u > r0 ? min(u - r0, 8u) : 0u;
                const uint32_t wds[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (2 * t < (int)m) add(wds[t] & 0xFFFFu);
                    if (2 * t + 1 < (int)m) add(wds[t] >> 16);
                }
            };
            // four vectors in flight per thread, each reloaded right after it is counted (loads unconditional, clamped)
            constexpr uint32_t S = kHcCountWG;
            const uint32_t t = k0 + threadIdx.x, last = k1 - 1;
            uint4 v0 = src[min(t, last)], v1 = src[min(t + S, last)];
            uint4 v2 = src[min(t + 2 * S, last)], v3 = src[min(t + 3 * S, last)];
            for (uint32_t k = t; k < k1; k += 4 * S) {
                count_vec(k, v0);
                v0 = src[min(k + 4 * S, last)];
                if (k + S < k1) count_vec(k + S, v1);
                v1 = src[min(k + 5 * S, last)];
                if (k + 2 * S < k1) count_vec(k + 2 * S, v2);
                v2 = src[min(k + 6 * S, last)];
                if (k + 3 * S < k1) count_vec(k + 3 * S, v3);
                v3 = src[min(k + 7 * S, last)];
            }
        }
    }
    // overflow pool (chunks of 64-element multiples; unused tails hold the 0xFFFF sentinel)
    {
        const uint32_t sn = nstat * 8;  // region index of the pool's first element
        const uint32_t fill = min(P.ovf_cur[p], q.cap_end) - q.ovf_base;
        const uint32_t e0 = max(pc.lo, sn) - sn, e1 = min(pc.hi, sn + fill);
        if (e1 > sn + e0) {
            const uint4* src = reinterpret_cast<const uint4*>(P.pbuf + q.ovf_base);
            for (uint32_t k = e0 / 8 + threadIdx.x; k < (e1 - sn) / 8; k += kHcCountWG) {
                const uint4 v = src[k];
                const uint32_t wds[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t lo = wds[t] & 0xFFFFu, hi = wds[t] >> 16;
                    if (lo != 0xFFFFu) add(lo);
                    if (hi != 0xFFFFu) add(hi);
                }
            }
        }
    }
    __syncthreads();
    const uint32_t base = p << kPartShift;
    const uint32_t S = min(1u << kPartShift, P.T - base);
    auto get = [&](uint32_t j) { return U16 ? (cnt[j >> 1] >> ((j & 1u) * 16)) & 0xFFFFu : cnt[j]; };
    if (!pc.whole) {  // one of several pieces of a heavy partition: add the non-zero counters
        for (uint32_t j = threadIdx.x; j < S; j += kHcCountWG) {
            const uint32_t c = get(j);
            if (c) atomicAdd(&P.counts[base + j], c);
        }
    } else if (P.overwrite) {
        for (uint32_t j = threadIdx.x; j < S; j += kHcCountWG) P.counts[base + j] = get(j);
    } else {  // later segments: read-modify-write, four counters in flight per thread
        for (uint32_t j = threadIdx.x; j < S; j += 4 * kHcCountWG) {
            uint32_t g[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) g[u] = j + u * kHcCountWG < S ? P.counts[base + j + u * kHcCountWG] : 0u;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (j + u * kHcCountWG < S) P.counts[base + j + u * kHcCountWG] = g[u] + get(j + u * kHcCountWG);
        }
    }
}

// hot slot totals in two steps.  hc_hot_reduce: block (x, y) sums counters [1024 x, 1024 x + 1024) of the slabs
// g = y (mod gridDim.y) -- four counters per thread as one 16-byte load, eight slab rows in flight -- and stores the
// partial sums over slab row y (only this block reads those columns of that row).  hc_hot_final: the gridDim.y partial
// rows summed, one atomic per slot onto its ordinal.  Counters 0..255 are the four lane-rotated copies of slots 0..63
// (one thread's four), counter i >= 256 is slot i - 192.
constexpr uint32_t kHotSplit = 16;
__global__ __launch_bounds__(256) void hc_hot_reduce_kernel(HcParams P) {
    if (P.skip && *P.skip) return;
    const uint32_t NH = hc_hot_counters(P.hot_n), stride = hc_slab_stride(P.hot_n);
    const uint32_t base = blockIdx.x * 1024 + threadIdx.x * 4;
    if (base >= NH) return;
    uint4* src = reinterpret_cast<uint4*>(P.hot_slab + base);
    const size_t row = stride / 4;  // uint4 per slab row
    uint4 acc = make_uint4(0, 0, 0, 0);
    const uint32_t Y = gridDim.y;
    uint32_t g = blockIdx.y;
    for (; g + 7 * Y < P.G; g += 8 * Y) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = src[(size_t)(g + k * Y) * row];
#pragma unroll
        for (int k = 0; k < 8; ++k) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
    }
    for (; g < P.G; g += Y) {
        const uint4 v = src[(size_t)g * row];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    src[(size_t)blockIdx.y * row] = acc;
}
__global__ __launch_bounds__(256) void hc_hot_final_kernel(HcParams P, uint32_t Y) {
    if (P.skip && *P.skip) return;
    const uint32_t NH = hc_hot_counters(P.hot_n), stride = hc_slab_stride(P.hot_n);
    const uint32_t base = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (base >= NH) return;
    const uint4* src = reinterpret_cast<const uint4*>(P.hot_slab + base);
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint32_t y = 0;
    for (; y + 8 <= Y; y += 8) {  // eight partial rows in flight
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = src[(size_t)(y + k) * (stride / 4)];
#pragma unroll
        for (int k = 0; k < 8; ++k) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
    }
    for (; y < Y; ++y) {
        const uint4 v = src[(size_t)y * (stride / 4)];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    auto add = [&](uint32_t slot, uint32_t t) {
        if (slot >= P.hot_n) return;
        if (P.slot_tot) {  // deferred cold lists: the slot's total (every slot written), folded onto its ordinal later
            P.slot_tot[slot] = t;
            return;
        }
        if (!t) return;
        const uint32_t o = P.hot_ord[slot];
        if (o < P.T) atomicAdd(&P.counts[o], t);
    };
    if (base < 4 * kHcHotCopies) {
        add(base / 4, acc.x + acc.y + acc.z + acc.w);
    } else {
        const uint32_t t[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (base + k < NH) add(base + k - 3 * kHcHotCopies, t[k]);
    }
}
static void launch_hot_reduce(const HcParams& p, hipStream_t s) {
    const uint32_t Y = std::max(1u, std::min(std::min(kHotSplit, p.G), std::max(1u, p.G / 8)));
    const uint32_t nh = hc_hot_counters(p.hot_n);
    hipLaunchKernelGGL(hc_hot_reduce_kernel, dim3((nh + 1023) / 1024, Y), dim3(256), 0, s, p);
    hipLaunchKernelGGL(hc_hot_final_kernel, dim3((nh + 1023) / 1024), dim3(256), 0, s, p, Y);
}

void launch_hotcold(const HcParams& p, hipStream_t s) {
    hipLaunchKernelGGL(hc_init_kernel, dim3((p.P + 255) / 256), dim3(256), 0, s, p);
    const size_t lds = hc_scatter_lds_bytes(p.P, p.hot_n);
    if (p.hot_n) hipLaunchKernelGGL(hc_scatter_kernel<true>, dim3(p.G), dim3(kHcWG), lds, s, p);
    else hipLaunchKernelGGL(hc_scatter_kernel<false>, dim3(p.G), dim3(kHcWG), lds, s, p);
    const size_t clds = (p.u16_counters ? (1u << kPartShift) / 2 : (1u << kPartShift)) * 4 + (size_t)p.G * 4;
    if (p.u16_counters) hipLaunchKernelGGL(hc_count_kernel<true>, dim3(p.n_pieces), dim3(kHcCountWG), clds, s, p);
    else hipLaunchKernelGGL(hc_count_kernel<false>, dim3(p.n_pieces), dim3(kHcCountWG), clds, s, p);
    if (p.hot_n) launch_hot_reduce(p, s);
}

// Hot slots only (postings path): the recoded column streamed with no barrier and no LDS return value in the loop; a
// cold or missing doc costs its bit test.  Three load buffers of 4 x 16 bytes per thread keep 96 KB per workgroup in
// flight; two workgroups per CU (measured: 0.155 ms for 125M docs against 0.175 ms with four, whose 2x hot slabs cost
// more in the reduce than the extra waves gain).
constexpr int kHotWG = 512;
constexpr uint32_t kHotTileDocs = kHotWG * kHcIt * 4;
// ACC: an accept bitset (live docs) -- its word loaded beside each 16-byte column load and tested at counting time
template <bool ACC>
__global__ __launch_bounds__(kHotWG) void hc_hot_kernel(HcParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* hot = (uint32_t*)smem;
    const uint32_t NH = hc_hot_counters(P.hot_n);
    for (uint32_t i = threadIdx.x; i < NH; i += kHotWG) hot[i] = 0u;
    __syncthreads();
    const uint32_t w = blockIdx.x;
    const uint32_t b_begin = min(w * P.blocks_per_wg, P.n_blocks);
    const uint32_t b_end = min(b_begin + P.blocks_per_wg, P.n_blocks);
    const uint32_t d_begin = b_begin * kBlockDocs;
    const uint32_t d_end = min(b_end * kBlockDocs, P.n_docs);
    const uint32_t span = b_end > b_begin ? (b_end - b_begin) * kBlockDocs : 0u;
    const uint32_t d_last = (b_end > b_begin ? b_end : P.n_blocks) * kBlockDocs - 4;  // (the workgroup's own last quad)
    const uint32_t tid4 = threadIdx.x * 4;
    auto load = [&](uint32_t t0, uint32_t o[kHcIt][4], uint64_t aw[kHcIt]) {
#pragma unroll
        for (int k = 0; k < kHcIt; ++k) {
            const uint32_t d = min(t0 + k * (kHotWG * 4) + tid4, d_last);
            const u32x4_t a = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(P.rc + d));
            o[k][0] = a.x; o[k][1] = a.y; o[k][2] = a.z; o[k][3] = a.w;
            if (ACC) aw[k] = P.accept[d >> 6];  // the raw word: shifted only when counted (no early wait on it)
        }
    };
    auto count = [&](uint32_t t0, const uint32_t o[kHcIt][4], const uint64_t aw[kHcIt]) {
        if (t0 >= d_begin + span) return;
#pragma unroll
        for (int k = 0; k < kHcIt; ++k) {
            const uint32_t doc0 = t0 + k * (kHotWG * 4) + tid4;
            const uint32_t live = ACC ? (uint32_t)(aw[k] >> (doc0 & 63)) & 0xFu : 0xFu;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t v = o[k][j];
                if ((v & kHcHotBit) && v != kMissingOrd && doc0 + j < d_end && ((live >> j) & 1u)) {
                    const uint32_t sl = v & ~kHcHotBit;
                    atomicAdd(&hot[sl < kHcHotCopies ? 4 * sl + (threadIdx.x & 3) : 3 * kHcHotCopies + sl], 1u);
                }
            }
        }
    };
    if (span) {
        uint32_t A[kHcIt][4], B[kHcIt][4], C[kHcIt][4];
        uint64_t Aw[kHcIt], Bw[kHcIt], Cw[kHcIt];
        load(d_begin, A, Aw);
        __builtin_amdgcn_sched_barrier(0);
        load(d_begin + kHotTileDocs, B, Bw);
        __builtin_amdgcn_sched_barrier(0);
        load(d_begin + 2 * kHotTileDocs, C, Cw);
        for (uint32_t t0 = d_begin; t0 < d_begin + span; t0 += 3 * kHotTileDocs) {
            count(t0, A, Aw);
            load(t0 + 3 * kHotTileDocs, A, Aw);
            count(t0 + kHotTileDocs, B, Bw);
            load(t0 + 4 * kHotTileDocs, B, Bw);
            count(t0 + 2 * kHotTileDocs, C, Cw);
            load(t0 + 5 * kHotTileDocs, C, Cw);
        }
    }
    __syncthreads();
    const uint32_t stride = hc_slab_stride(P.hot_n);
    for (uint32_t i = threadIdx.x; i < stride; i += kHotWG) P.hot_slab[(size_t)w * stride + i] = i < NH ? hot[i] : 0u;
}

// The same pass over the 16-bit hot-slot column (the segment statistics' compressed copy, like Lucene's bit-packed
// ordinals): 8 docs per 16-byte load, half the bytes of the recoded column
constexpr uint32_t kHot16TileDocs = kHotWG * kHcIt * 8;
// CT: the docs of cold ordinals that pass are counted too (one total, P.cold_tot: a filtered request's other doc count
// when the hot slots settle its top-k)
template <bool ACC, bool CT = false>
__global__ __launch_bounds__(kHotWG) void hc_hot16_count_kernel(HcParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* hot = (uint32_t*)smem;
    const uint32_t NH = hc_hot_counters(P.hot_n);
    for (uint32_t i = threadIdx.x; i < NH; i += kHotWG) hot[i] = 0u;
    __syncthreads();
    const uint32_t w = blockIdx.x;
    const uint32_t b_begin = min(w * P.blocks_per_wg, P.n_blocks);
    const uint32_t b_end = min(b_begin + P.blocks_per_wg, P.n_blocks);
    const uint32_t d_begin = b_begin * kBlockDocs;
    const uint32_t d_end = min(b_end * kBlockDocs, P.n_docs);
    const uint32_t span = b_end > b_begin ? (b_end - b_begin) * kBlockDocs : 0u;
    const uint32_t d_last = (b_end > b_begin ? b_end : P.n_blocks) * kBlockDocs - 8;  // (the workgroup's own last 8 docs)
    const uint32_t tid8 = threadIdx.x * 8;
    auto load = [&](uint32_t t0, uint32_t o[kHcIt][4], uint64_t aw[kHcIt]) {
#pragma unroll
        for (int k = 0; k < kHcIt; ++k) {
            const uint32_t d = min(t0 + k * (kHotWG * 8) + tid8, d_last);
            const u32x4_t a = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(P.rc16 + d));
            o[k][0] = a.x; o[k][1] = a.y; o[k][2] = a.z; o[k][3] = a.w;
            if (ACC) aw[k] = P.accept[d >> 6];
        }
    };
    uint32_t ncold = 0;
    auto count = [&](uint32_t t0, const uint32_t o[kHcIt][4], const uint64_t aw[kHcIt]) {
        if (t0 >= d_begin + span) return;
#pragma unroll
        for (int k = 0; k < kHcIt; ++k) {
            const uint32_t doc0 = t0 + k * (kHotWG * 8) + tid8;
            const uint32_t live = ACC ? (uint32_t)(aw[k] >> (doc0 & 63)) & 0xFFu : 0xFFu;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t sl = (o[k][j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                const bool in = doc0 + j < d_end && ((live >> j) & 1u);
                if (sl < 0xFFFEu && in)
                    atomicAdd(&hot[sl < kHcHotCopies ? 4 * sl + (threadIdx.x & 3) : 3 * kHcHotCopies + sl], 1u);
                if (CT) ncold += (sl == 0xFFFEu && in) ? 1u : 0u;
            }
        }
    };
    if (span) {
        uint32_t A[kHcIt][4], B[kHcIt][4], C[kHcIt][4];
        uint64_t Aw[kHcIt], Bw[kHcIt], Cw[kHcIt];
        load(d_begin, A, Aw);
        __builtin_amdgcn_sched_barrier(0);
        load(d_begin + kHot16TileDocs, B, Bw);
        __builtin_amdgcn_sched_barrier(0);
        load(d_begin + 2 * kHot16TileDocs, C, Cw);
        for (uint32_t t0 = d_begin; t0 < d_begin + span; t0 += 3 * kHot16TileDocs) {
            count(t0, A, Aw);
            load(t0 + 3 * kHot16TileDocs, A, Aw);
            count(t0 + kHot16TileDocs, B, Bw);
            load(t0 + 4 * kHot16TileDocs, B, Bw);
            count(t0 + 2 * kHot16TileDocs, C, Cw);
            load(t0 + 5 * kHot16TileDocs, C, Cw);
        }
    }
    if (CT) {  // one global add per wave
        const uint32_t wsum = wave_sum_u32(ncold);
        if ((threadIdx.x & 63) == 0 && wsum) atomicAdd(P.cold_tot, wsum);
    }
    __syncthreads();
    const uint32_t stride = hc_slab_stride(P.hot_n);
    for (uint32_t i = threadIdx.x; i < stride; i += kHotWG) P.hot_slab[(size_t)w * stride + i] = i < NH ? hot[i] : 0u;
}

__global__ __launch_bounds__(256) void hc_pad_kernel(const uint16_t* dense, const uint32_t* dense_begin,
                                                     const uint32_t* pad_begin, uint16_t* out) {
    const uint32_t p = blockIdx.x;
    const uint32_t b = dense_begin[p], n = dense_begin[p + 1] - b, o = pad_begin[p], cap = pad_begin[p + 1] - o;
    for (uint32_t i = threadIdx.x; i < cap; i += 256) out[o + i] = i < n ? dense[b + i] : (uint16_t)0xFFFFu;
}
void launch_hc_pad(const uint16_t* dense, const uint32_t* dense_begin, const uint32_t* pad_begin, uint32_t P,
                   uint16_t* out, hipStream_t s) {
    if (P) hipLaunchKernelGGL(hc_pad_kernel, dim3(P), dim3(256), 0, s, dense, dense_begin, pad_begin, out);
}

// live docs under the postings form: the cold lists hold every doc of the segment, so the cold docs the accept bitset
// clears are taken back out -- each dead doc's recoded value read, a cold one's counter decremented (one scattered
// atomic per dead cold doc: cheap while deletions are few, the hot ones were never counted)
__global__ __launch_bounds__(256) void hc_cold_sub_kernel(const uint32_t* rc, const uint64_t* accept, uint32_t n_docs, uint32_t T,
                                                          unsigned int* counts) {
    const uint32_t nw = (n_docs + 63) / 64;
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
        uint64_t dead = ~accept[w];
        if (w == nw - 1 && (n_docs & 63)) dead &= (1ull << (n_docs & 63)) - 1ull;
        while (dead) {
            const uint32_t d = w * 64 + (uint32_t)__builtin_ctzll(dead);
            dead &= dead - 1ull;
            const uint32_t v = rc[d];
            if (!(v & kHcHotBit) && v < T) atomicSub(&counts[v], 1u);
        }
    }
}

// ---- replay over the hot inner terms (ReplayHotParams) ----
size_t replay_hot_lds(uint32_t k, uint32_t Hh, uint32_t slot_map_n) {
    return (size_t)replay_hot_stride(k, Hh) * 4 + (((size_t)slot_map_n + 15) & ~(size_t)15);
}
constexpr int kRhWG = 512;
constexpr int kRhIt = 2;  // 16-byte loads of each column per thread per tile
constexpr uint32_t kRhTileDocs = kRhWG * kRhIt * 8;
__global__ __launch_bounds__(kRhWG) void replay_hot_kernel(ReplayHotParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t stride = replay_hot_stride(P.k, P.Hh);
    uint32_t* cnt = (uint32_t*)smem;                 // [k][Hh], then [k] missing-term counts
    uint8_t* map = smem + (size_t)stride * 4;        // [slot_map_n]
    for (uint32_t i = threadIdx.x; i < stride; i += kRhWG) cnt[i] = 0u;
    for (uint32_t i = threadIdx.x; i < P.slot_map_n; i += kRhWG) map[i] = P.slot_map[i];
    __syncthreads();
    const uint32_t w = blockIdx.x;
    const uint32_t b_begin = min(w * P.blocks_per_wg, P.n_blocks);
    const uint32_t b_end = min(b_begin + P.blocks_per_wg, P.n_blocks);
    const uint32_t d_begin = b_begin * kBlockDocs;
    const uint32_t d_end = min(b_end * kBlockDocs, P.n_docs);
    const uint32_t span = b_end > b_begin ? (b_end - b_begin) * kBlockDocs : 0u;
    const uint32_t d_last = (b_end > b_begin ? b_end : P.n_blocks) * kBlockDocs - 8;  // (the workgroup's own last 8 docs)
    const uint32_t tid8 = threadIdx.x * 8;
    const uint32_t Hh = P.Hh, nmap = P.slot_map_n, k = P.k;
    const bool acc = P.accept != nullptr;
    auto load = [&](uint32_t t0, u32x4_t a[kRhIt], u32x4_t h[kRhIt], uint64_t aw[kRhIt]) {
#pragma unroll
        for (int it = 0; it < kRhIt; ++it) {
            const uint32_t d = min(t0 + it * (kRhWG * 8) + tid8, d_last);
            a[it] = load16(P.a16 + d);
            h[it] = load16(P.hot16 + d);
            aw[it] = acc ? P.accept[d >> 6] : ~0ull;
        }
    };
    auto count = [&](uint32_t t0, const u32x4_t a[kRhIt], const u32x4_t h[kRhIt], const uint64_t aw[kRhIt]) {
        if (t0 >= d_begin + span) return;
#pragma unroll
        for (int it = 0; it < kRhIt; ++it) {
            const uint32_t doc0 = t0 + it * (kRhWG * 8) + tid8;
            const uint32_t live = (uint32_t)(aw[it] >> (doc0 & 63)) & 0xFFu;
            const uint32_t aw4[4] = {a[it].x, a[it].y, a[it].z, a[it].w}, hw4[4] = {h[it].x, h[it].y, h[it].z, h[it].w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t o = (aw4[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                const uint32_t sl = (hw4[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                const uint32_t s = o < nmap ? map[o] : 0xFFu;
                if (s < k && doc0 + j < d_end && ((live >> j) & 1u)) {
                    if (sl < Hh) atomicAdd(&cnt[s * Hh + sl], 1u);
                    else if (sl == 0xFFFFu) atomicAdd(&cnt[k * Hh + s], 1u);
                }
            }
        }
    };
    if (span) {
        u32x4_t A[kRhIt], Ah[kRhIt], B[kRhIt], Bh[kRhIt];
        uint64_t Aw[kRhIt], Bw[kRhIt];
        load(d_begin, A, Ah, Aw);
        load(d_begin + kRhTileDocs, B, Bh, Bw);
        for (uint32_t t0 = d_begin; t0 < d_begin + span; t0 += 2 * kRhTileDocs) {
            count(t0, A, Ah, Aw);
            load(t0 + 2 * kRhTileDocs, A, Ah, Aw);
            count(t0 + kRhTileDocs, B, Bh, Bw);
            load(t0 + 3 * kRhTileDocs, B, Bh, Bw);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < stride; i += kRhWG) P.slab[(size_t)w * stride + i] = cnt[i];
}
__global__ __launch_bounds__(256) void replay_hot_sum_kernel(ReplayHotParams P) {
    const uint32_t stride = replay_hot_stride(P.k, P.Hh);
    const uint32_t i = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (i >= stride) return;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t g = 0; g < P.G; ++g) {
        const uint4 v = *reinterpret_cast<const uint4*>(P.slab + (size_t)g * stride + i);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *reinterpret_cast<uint4*>(P.out + i) = acc;
}
void launch_replay_hot(const ReplayHotParams& p, hipStream_t s) {
    hipLaunchKernelGGL(replay_hot_kernel, dim3(p.G), dim3(kRhWG), replay_hot_lds(p.k, p.Hh, p.slot_map_n), s, p);
    const uint32_t stride = replay_hot_stride(p.k, p.Hh);
    hipLaunchKernelGGL(replay_hot_sum_kernel, dim3((stride / 4 + 255) / 256), dim3(256), 0, s, p);
}

// the deferred cold lists' fold: the hot slot totals onto their ordinals (after the overwriting cold count)
__global__ __launch_bounds__(256) void hc_slot_fold_kernel(HcParams P) {
    if (P.skip && *P.skip) return;
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= P.hot_n) return;
    const uint32_t t = P.slot_tot[s], o = P.hot_ord[s];
    if (t && o < P.T) atomicAdd(&P.counts[o], t);
}
void launch_hot_postings(const HcParams& hot, hipStream_t s) {
    const size_t hlds = (size_t)hc_hot_counters(hot.hot_n) * 4;
    if (hot.accept) hipLaunchKernelGGL((hc_hot16_count_kernel<true, true>), dim3(hot.G), dim3(kHotWG), hlds, s, hot);
    else hipLaunchKernelGGL(hc_hot16_count_kernel<false>, dim3(hot.G), dim3(kHotWG), hlds, s, hot);
    launch_hot_reduce(hot, s);
}
void launch_cold_postings(const HcParams& hot, const HcParams& cold, hipStream_t s) {
    if (cold.n_pieces) {
        const size_t clds = (cold.u16_counters ? (1u << kPartShift) / 2 : (1u << kPartShift)) * 4 + (size_t)cold.G * 4;
        if (cold.u16_counters) hipLaunchKernelGGL(hc_count_kernel<true>, dim3(cold.n_pieces), dim3(kHcCountWG), clds, s, cold);
        else hipLaunchKernelGGL(hc_count_kernel<false>, dim3(cold.n_pieces), dim3(kHcCountWG), clds, s, cold);
    }
    hipLaunchKernelGGL(hc_slot_fold_kernel, dim3((hot.hot_n + 255) / 256), dim3(256), 0, s, hot);
}
__global__ void hot_topk_check_kernel(const unsigned long long* hot_keys, uint32_t k, uint32_t k_req, uint64_t max_cold,
                                      uint64_t docs, int order, uint32_t* skip, unsigned long long* out_keys,
                                      unsigned long long* out_sum, const uint32_t* slot_tot, uint32_t hot_n,
                                      const uint32_t* cold_tot) {
    __shared__ uint32_t ok;
    __shared__ unsigned long long tot;
    if (threadIdx.x == 0) {
        // count order descending: the k-th pick present and above every cold ordinal's count (ties go to the smaller
        // ordinal, which may be cold: strictly above)
        const unsigned long long last = k_req ? hot_keys[k_req - 1] : 0ull;
        ok = order == 0 && k_req >= 1 && last != 0 && ((last >> 32) & 0x7FFFFFFFull) > max_cold;
        *skip = ok;
    }
    __syncthreads();
    if (!ok) return;
    for (uint32_t i = threadIdx.x; i < k; i += blockDim.x) out_keys[i] = hot_keys[i];
    if (!cold_tot) {
        if (threadIdx.x == 0) *out_sum = docs;  // the sum of every ordinal's count: the segment's docs with a value
        return;
    }
    // a filtered request: its docs with a value that pass = the hot slots' totals + the passing cold docs
    if (threadIdx.x == 0) tot = *cold_tot;
    __syncthreads();
    unsigned long long part = 0;
    for (uint32_t i = threadIdx.x; i < hot_n; i += blockDim.x) part += slot_tot[i];
    atomicAdd(&tot, part);
    __syncthreads();
    if (threadIdx.x == 0) *out_sum = tot;
}
void launch_hot_topk_check(const unsigned long long* hot_keys, uint32_t k, uint32_t k_req, uint64_t max_cold, uint64_t docs,
                           int order, uint32_t* skip, unsigned long long* out_keys, unsigned long long* out_sum,
                           const uint32_t* slot_tot, uint32_t hot_n, const uint32_t* cold_tot, hipStream_t s) {
    hipLaunchKernelGGL(hot_topk_check_kernel, dim3(1), dim3(256), 0, s, hot_keys, k, k_req, max_cold, docs, order, skip,
                       out_keys, out_sum, slot_tot, hot_n, cold_tot);
}

void launch_hotcold_postings(const HcParams& hot, const HcParams& cold, hipStream_t s) {
    const size_t hlds = (size_t)hc_hot_counters(hot.hot_n) * 4;
    if (hot.hot_n && hot.rc16 && hot.accept)
        hipLaunchKernelGGL(hc_hot16_count_kernel<true>, dim3(hot.G), dim3(kHotWG), hlds, s, hot);
    else if (hot.hot_n && hot.rc16)
        hipLaunchKernelGGL(hc_hot16_count_kernel<false>, dim3(hot.G), dim3(kHotWG), hlds, s, hot);
    else if (hot.hot_n && hot.accept)
        hipLaunchKernelGGL(hc_hot_kernel<true>, dim3(hot.G), dim3(kHotWG), (size_t)hc_hot_counters(hot.hot_n) * 4, s, hot);
    else if (hot.hot_n)
        hipLaunchKernelGGL(hc_hot_kernel<false>, dim3(hot.G), dim3(kHotWG), (size_t)hc_hot_counters(hot.hot_n) * 4, s, hot);
    if (cold.n_pieces) {  // the cold lists never use overflow chunks: their cursors were set once (HcStats)
        const size_t clds = (cold.u16_counters ? (1u << kPartShift) / 2 : (1u << kPartShift)) * 4 + (size_t)cold.G * 4;
        if (cold.u16_counters) hipLaunchKernelGGL(hc_count_kernel<true>, dim3(cold.n_pieces), dim3(kHcCountWG), clds, s, cold);
        else hipLaunchKernelGGL(hc_count_kernel<false>, dim3(cold.n_pieces), dim3(kHcCountWG), clds, s, cold);
    }
    if (hot.hot_n) launch_hot_reduce(hot, s);
    if (hot.accept) {
        const uint32_t nw = (hot.n_docs + 63) / 64;
        hipLaunchKernelGGL(hc_cold_sub_kernel, dim3(std::max(1u, std::min(4096u, (nw + 255) / 256))), dim3(256), 0, s, hot.rc,
                           hot.accept, hot.n_docs, hot.T, hot.counts);
    }
}

}  // namespace esgpu
