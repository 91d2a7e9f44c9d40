// esgpu_kernels.hip — hand-written gfx950 kernels for the per-shard aggregation collection path.
//
//   zone_map_kernel      per-8192-doc-block min/max of an i64 column (segment upload, K11)
//   synth_kernel         synthetic log-style shard generated in HBM (bench/test data)
//   collect_kernel<...>  K1/K4/K5/K6/K7/K10 fused: filter predicates -> (term ord x rounded key) cell ->
//                        doc count + stats/extended_stats/avg accumulators, LDS-privatised per workgroup with a
//                        sliding key window over time-sorted blocks, flushed to HBM with coalesced atomics
//   hll_kernel           K8: mix64 / murmur3-ord hashing, HLL++ register max + exact linear-counting set
//   term_totals_kernel   outer-level doc counts from the [H][T] cell grid
//   gather_rows_kernel   copies the surviving terms' rows (top shard_size) for the D2H build
//
// No MFMA: nothing on this path is a dense contraction.  Every kernel is an HBM stream; the per-doc work is
// integer/LDS-atomic bound.  See DESIGN.md for the roofline accounting.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "es_common.hpp"
#include "esgpu_kernels.hpp"

namespace esgpu {

// ------------------------------------------------------------------------------------------------------------
// zone maps
// ------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void zone_map_kernel(const int64_t* __restrict__ v, const uint64_t* __restrict__ present,
                                                       uint32_t n, int64_t* __restrict__ zmin, int64_t* __restrict__ zmax,
                                                       int f64) {
    const uint32_t block = blockIdx.x;
    const uint32_t begin = block * kBlockDocs;
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    for (uint32_t i = begin + threadIdx.x; i < begin + kBlockDocs && i < n; i += blockDim.x) {
        if (present && !((present[i >> 6] >> (i & 63)) & 1)) continue;
        const int64_t x = f64 ? java_long(bits_dbl((uint64_t)v[i])) : v[i];
        mn = x < mn ? x : mn;
        mx = x > mx ? x : mx;
    }
    __shared__ int64_t smn[256], smx[256];
    smn[threadIdx.x] = mn;
    smx[threadIdx.x] = mx;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            smn[threadIdx.x] = smn[threadIdx.x] < smn[threadIdx.x + s] ? smn[threadIdx.x] : smn[threadIdx.x + s];
            smx[threadIdx.x] = smx[threadIdx.x] > smx[threadIdx.x + s] ? smx[threadIdx.x] : smx[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        zmin[block] = smn[0];
        zmax[block] = smx[0];
    }
}

void launch_zone_map(const int64_t* v, const uint64_t* present, uint32_t n, int64_t* zmin, int64_t* zmax, bool f64,
                     hipStream_t stream) {
    const uint32_t nb = (n + kBlockDocs - 1) / kBlockDocs;
    if (nb == 0) return;
    hipLaunchKernelGGL(zone_map_kernel, dim3(nb), dim3(256), 0, stream, v, present, n, zmin, zmax, f64 ? 1 : 0);
}

// ------------------------------------------------------------------------------------------------------------
// synthetic shard
// ------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void synth_kernel(SynthParams P) {
    const uint64_t sseed = shard_seed(P.seed, P.shard);
    for (uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; d < P.n_pad; d += (uint64_t)gridDim.x * blockDim.x) {
        const bool live = d < P.n;
        if (P.ts) P.ts[d] = live ? synth_timestamp(sseed, d, P.n, P.ts_jitter) : 0;
        if (P.host) P.host[d] = live ? synth_host(sseed, d, P.host_cdf) : kMissingOrd;
        if (P.url) P.url[d] = live ? synth_url(sseed, d, P.url_cdf) : kMissingOrd;
        if (P.status) P.status[d] = live ? synth_status(sseed, d) : 0;
        if (P.rt) P.rt[d] = live ? synth_rt(sseed, d, P.rt_cdf) : 0;
        if (P.bytes) P.bytes[d] = live ? synth_bytes(sseed, d) : 0;
        if (P.ip) P.ip[d] = live ? synth_ip_hash(sseed, d) : 0;
        if (P.price) P.price[d] = live ? synth_price(sseed, d) : 0.0;
    }
}

void launch_synth(const SynthParams& p, hipStream_t stream) {
    hipLaunchKernelGGL(synth_kernel, dim3(4096), dim3(256), 0, stream, p);
}

}  // namespace esgpu

#include "esgpu_collect.hpp"

namespace esgpu {

void launch_zone_keys(const CollectParams& p, int64_t* out, hipStream_t st, unsigned long long* udocs) {
    if (p.n_blocks == 0) return;
    const uint32_t g = (p.n_blocks + 255) / 256;
    if (p.kstart) hipLaunchKernelGGL(zone_keys_kernel<true>, dim3(g), dim3(256), 0, st, p, out, udocs);
    else hipLaunchKernelGGL(zone_keys_kernel<false>, dim3(g), dim3(256), 0, st, p, out, udocs);
}

// the collect kernels are instantiated in esgpu_collect_inst.hip, compiled once per (ORD, HK) so the variants build
// in parallel
void launch_collect(const CollectParams& p, bool ord, bool hist, int met, bool wide, uint32_t grid, size_t lds, hipStream_t st) {
    const int hk = hist ? (p.hord ? 3 : p.kstart ? 2 : 1) : 0;
    if (ord) {
        if (hk == 3) launch_collect_inst<true, 3>(p, met, false, grid, lds, st);
        else if (hk == 2) launch_collect_inst<true, 2>(p, met, wide, grid, lds, st);
        else if (hk == 1) launch_collect_inst<true, 1>(p, met, wide, grid, lds, st);
        else launch_collect_inst<true, 0>(p, met, false, grid, lds, st);
    } else {
        if (hk == 2) launch_collect_inst<false, 2>(p, met, wide, grid, lds, st);
        else if (hk == 1) launch_collect_inst<false, 1>(p, met, wide, grid, lds, st);
        else launch_collect_inst<false, 0>(p, met, false, grid, lds, st);
    }
}

int collect_occupancy(bool ord, int hk, int met, size_t lds, int vk, bool wide) {
    if (ord && hk == 3) return collect_occ_inst<true, 3>(met, lds, vk, false);
    if (ord)
        return hk == 2 ? collect_occ_inst<true, 2>(met, lds, vk, wide) : hk == 1 ? collect_occ_inst<true, 1>(met, lds, vk, wide)
                                                                                : collect_occ_inst<true, 0>(met, lds, vk, false);
    return hk == 2 ? collect_occ_inst<false, 2>(met, lds, vk, wide) : hk == 1 ? collect_occ_inst<false, 1>(met, lds, vk, wide)
                                                                             : collect_occ_inst<false, 0>(met, lds, vk, false);
}


size_t collect_lds_bytes(uint32_t T, uint32_t W, int met, int vcnt_mode, int ocnt_mode, uint32_t ncopies, bool pi) {
    const size_t C = (size_t)T * W;
    const size_t n = std::max(ncopies, 1u);
    auto r = [](size_t b) { return (b + 15) & ~(size_t)15; };
    if (pi) {  // must match collect_kernel's carve order
        size_t bytes = r(8 * C * n) + (met >= 2 ? r(8 * C) : 0);
        if (ocnt_mode == OCNT_TERMS) bytes += r(4 * (size_t)T);
        if (ocnt_mode == OCNT_HIST) bytes += r(4 * (size_t)W);
        return bytes + 8 * 1024;  // a spare word per thread (1024-thread workgroups at most)
    }
    size_t bytes = r(4 * C * n);
    if (vcnt_mode) bytes += r(4 * C * n);
    if (met > 0) bytes += r(8 * C * n);
    if (met >= 2) bytes += r(16 * C);
    if (met >= 3) bytes += r(8 * C * n);
    if (ocnt_mode == OCNT_TERMS) bytes += r(4 * (size_t)T);
    if (ocnt_mode == OCNT_HIST) bytes += r(4 * (size_t)W);
    return bytes;
}

// ------------------------------------------------------------------------------------------------------------
// HLL++ (K8)
// ------------------------------------------------------------------------------------------------------------
// hashes of 4 consecutive docs (MurmurHash3Values.Long/Double: mix64; Bytes/ordinals: murmur3 h1 per term)

// pass 1: HLL registers (max runLen per index).  Registers only grow, so a stale read-check costs at most an extra
// atomic; after warm-up almost every doc is a read that finds a register already >= its run length.
// `floor` is a lower bound of every register (min over registers after the previous phase): a hash whose run
// length is <= floor cannot raise any register, so it needs no register read at all.
// Each workgroup owns a contiguous doc range and prefetches the next 1024 docs' raw words while it hashes the
// current ones (mix64 runs at processing time, so the prefetch is never drained early).
constexpr int kHllWG = 256;
constexpr uint32_t kHllIter = kHllWG * 4;

__device__ __forceinline__ void hll_load_raw(const HllParams& P, uint32_t i0, uint64_t raw[4]) {
    if (P.kind == HLL_ORD) {
        uint32_t o[4];
        load_u32x4((const uint32_t*)P.col, i0, o);
#pragma unroll
        for (int j = 0; j < 4; ++j) raw[j] = o[j];
    } else {
        load_i64x4((const int64_t*)P.col, i0, (int64_t*)raw);
    }
}

__device__ __forceinline__ uint32_t hll_hash_raw(const HllParams& P, uint32_t i0, const uint64_t raw[4], uint64_t hv[4]) {
    uint32_t ok = 0xF;
    if (i0 + 4 > P.n_docs) ok = i0 >= P.n_docs ? 0u : (1u << (P.n_docs - i0)) - 1u;
    if (P.accept) ok &= bits4(P.accept, i0);
    for (int k = 0; k < P.npred; ++k) ok &= eval_pred(P.pred[k], i0);
    if (P.kind == HLL_ORD) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t o = (uint32_t)raw[j];
            const bool valid = o != kMissingOrd && o < P.n_ords;
            if (!valid) ok &= ~(1u << j);
            hv[j] = valid ? P.ord_hash[o] : 0;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint64_t bits = raw[j];
            if (P.kind == HLL_F64) {  // doubleToLongBits canonicalises NaN
                const double x = bits_dbl(bits);
                if (x != x) bits = 0x7ff8000000000000ULL;
            }
            hv[j] = mix64(bits);
        }
        if (P.present) ok &= bits4(P.present, i0);
    }
    return ok;
}

__global__ __launch_bounds__(kHllWG) void hll_registers_kernel(HllParams P, uint32_t d_begin, uint32_t d_end,
                                                               uint32_t per_wg, const unsigned int* floor_ptr) {
    const uint32_t floor = floor_ptr ? *floor_ptr : 0u;
    const uint32_t w0 = d_begin + blockIdx.x * per_wg;
    const uint32_t w1 = min(d_end, w0 + per_wg);
    if (w0 >= w1) return;
    const uint32_t t4 = threadIdx.x * 4;
    uint64_t cur_raw[4] = {0, 0, 0, 0};
    if (w0 + t4 < w1) hll_load_raw(P, w0 + t4, cur_raw);
    for (uint32_t base = w0; base < w1; base += kHllIter) {
        const uint32_t i0 = base + t4, nx = i0 + kHllIter;
        uint64_t nxt_raw[4] = {0, 0, 0, 0};
        if (nx < w1) hll_load_raw(P, nx, nxt_raw);
        if (i0 < w1) {
            uint64_t hv[4];
            uint32_t ok = hll_hash_raw(P, i0, cur_raw, hv);
            if (i0 + 4 > w1) ok &= (1u << (w1 - i0)) - 1u;
            // all register reads first, then the atomics: registers only grow, so a read that races with another
            // thread's atomicMax can only cause a redundant atomic, never a missed one
            uint32_t rl[4], idx[4], cur[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                rl[j] = ((ok >> j) & 1) ? hll_run_len(hv[j], P.p) : 0u;
                idx[j] = hll_index(hv[j], P.p);
                cur[j] = rl[j] > floor ? P.regs[idx[j]] : 0xFFu;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (rl[j] > cur[j]) atomicMax(&P.regs[idx[j]], rl[j]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) cur_raw[j] = nxt_raw[j];
    }
}

// Unfiltered dense columns (no accept bits, no predicates, no present bitset): the register pass without the generic
// per-doc branches.  A hash can raise a register only if its run length exceeds the floor, i.e. only if the `floor`
// bits below the index bits are all zero -- one 64-bit AND decides that before any clz / index / register read.
template <int KIND>
__device__ __forceinline__ uint64_t hll_fast_hash(const HllParams& P, uint64_t raw) {
    if (KIND == HLL_ORD) {
        const uint32_t o = (uint32_t)raw;
        return (o != kMissingOrd && o < P.n_ords) ? P.ord_hash[o] : 0ull;
    }
    uint64_t bits = raw;
    if (KIND == HLL_F64) {  // doubleToLongBits canonicalises NaN
        const double x = bits_dbl(bits);
        if (x != x) bits = 0x7ff8000000000000ULL;
    }
    return mix64(bits);
}

constexpr uint32_t kHllGroup = 64;       // registers per group floor
constexpr uint32_t kHllMaxGroups = 4096;  // 2^18 / 64

template <int KIND>
__global__ __launch_bounds__(kHllWG) void hll_registers_fast_kernel(HllParams P, uint32_t d_begin, uint32_t d_end,
                                                                    uint32_t per_wg, const unsigned int* floor_ptr) {
    const uint32_t floor = floor_ptr ? min(*floor_ptr, 64u - (uint32_t)P.p) : 0u;
    // rl > floor  <=>  bits [64 - p - floor, 64 - p) of the hash are zero
    const uint64_t zmask = floor == 0 ? 0ull : (((1ull << floor) - 1ull) << (64 - P.p - floor));
    // per-group floors (min of 64 registers) rise faster than the global one: most survivors of the mask test stop here
    __shared__ unsigned char gf[kHllMaxGroups];
    const uint32_t m = 1u << P.p;
    const uint32_t ngroups = m >= kHllGroup ? m / kHllGroup : 1u;
    const uint32_t gshift = m >= kHllGroup ? 6u : (uint32_t)P.p;
    for (uint32_t i = threadIdx.x; i < ngroups; i += kHllWG) gf[i] = floor_ptr ? P.gfloor[i] : 0;
    __syncthreads();
    const uint32_t w0 = d_begin + blockIdx.x * per_wg;
    const uint32_t w1 = min(d_end, w0 + per_wg);
    if (w0 >= w1) return;
    const uint32_t t4 = threadIdx.x * 4;
    uint64_t cur_raw[4] = {0, 0, 0, 0};
    if (w0 + t4 < w1) hll_load_raw(P, w0 + t4, cur_raw);
    for (uint32_t base = w0; base < w1; base += kHllIter) {
        const uint32_t i0 = base + t4, nx = i0 + kHllIter;
        uint64_t nxt_raw[4] = {0, 0, 0, 0};
        if (nx < w1) hll_load_raw(P, nx, nxt_raw);
        if (i0 < w1) {
            const uint32_t lim = w1 - i0;  // docs of this thread inside the range (>= 1)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t h = hll_fast_hash<KIND>(P, cur_raw[j]);
                bool live = (uint32_t)j < lim && (h & zmask) == 0;
                if (KIND == HLL_ORD) live = live && (uint32_t)cur_raw[j] != kMissingOrd && (uint32_t)cur_raw[j] < P.n_ords;
                if (live) {
                    const uint32_t rl = hll_run_len(h, P.p);
                    const uint32_t idx = hll_index(h, P.p);
                    if (rl > gf[idx >> gshift] && rl > P.regs[idx]) atomicMax(&P.regs[idx], rl);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) cur_raw[j] = nxt_raw[j];
    }
}

// Register pass over a numeric column (phases after the first), with a per-workgroup LDS copy of the registers as
// 4-bit lower bounds: register >= F + nibble, F = the floor (min register) when the phase started.  A hash reads
// only LDS; when it beats its bound it raises the global register with a no-return atomicMax and its nibble.  The
// kernel issues no global load between a prefetch and its use, so two 16-byte loads per thread stay in flight
// across the hashing of the previous 4 docs (a global register read-check waits for vmcnt(0), i.e. for the
// prefetch).  Nibble writes are plain read-modify-writes of a byte: a lost update leaves an older nibble, which is
// still a lower bound (registers only grow, and every nibble written came with an atomicMax of at least its value).
constexpr uint32_t kHllLdsWG = 1024;
#ifndef ESGPU_HLL_NBUF
#define ESGPU_HLL_NBUF 2  // load buffers in flight per thread (2 or 3)
#endif
constexpr uint32_t kHllLdsIter = kHllLdsWG * 4;
#ifndef ESGPU_HLL_BITS
#define ESGPU_HLL_BITS 4
#endif
constexpr uint32_t kHllBits = ESGPU_HLL_BITS;            // bits per register bound in the snapshot (4: 128 KB at p = 18)
constexpr uint32_t kHllPerByte = 8 / kHllBits;
constexpr uint32_t kHllMaxDelta = (1u << kHllBits) - 1;
__host__ __device__ constexpr uint32_t hll_snap_bytes(uint32_t m) { return m / kHllPerByte; }
// raises a phase workgroup logs in LDS (more: straight to the registers with an atomicMax); expected about
// (growth - 1) * m / workgroups = 3,072 per workgroup and phase at p = 18
constexpr uint32_t kHllLog = 4096;
// the phase kernel's LDS: the nibbles, then one group floor byte per group of kHllGroup registers (16-byte multiple),
// then (logging) the raise log, per-range counters and cursors, bases, and the log length
__host__ __device__ constexpr uint32_t hll_lds_bytes(uint32_t m, bool logm = false) {
    return hll_snap_bytes(m) + (((m >= 64u ? m / 64u : 1u) + 15u) & ~15u) + (logm ? kHllLog * 4u + 3u * 256u * 4u + 16u : 0u);
}

__device__ __forceinline__ uint32_t hll_enc32_entry(uint32_t v, int p);

// E32: the enc32 words (HllParams.enc32, 4 bytes per doc) instead of the values, 8 docs per thread and buffer
template <int KIND, bool E32>
__global__ __launch_bounds__(kHllLdsWG) void hll_registers_lds_kernel(HllParams P, uint32_t d_begin, uint32_t d_end,
                                                                       uint32_t per_wg, const unsigned int* floor_ptr) {
    // LDS: [2^p / 2] packed nibbles, then the group floors [ngroups] (one byte per group of 64 registers)
    extern __shared__ __attribute__((aligned(16))) unsigned char nib[];
    const uint32_t m = 1u << P.p;
    const uint32_t nbytes = hll_snap_bytes(m);
    const uint32_t ngroups = m >= kHllGroup ? m / kHllGroup : 1u;
    const uint32_t gshift = m >= kHllGroup ? 6u : (uint32_t)P.p;
    unsigned char* gfl = nib + nbytes;
    const bool logm = P.log_raises != 0;
    uint32_t* rlog = (uint32_t*)(gfl + ((ngroups + 15u) & ~15u));  // [kHllLog] (rl << 24 | idx)
    uint32_t* lcnt = rlog + kHllLog;                                 // [256] entries per register range
    uint32_t* lcur = lcnt + 256;                                     // [256] their write cursors
    uint32_t* lbase = lcur + 256;                                    // [256] reserved base in the range's slots
    uint32_t* nlog = lbase + 256;                                    // [1]
    if (logm && threadIdx.x == 0) *nlog = 0;
    if ((nbytes & 15u) == 0) {
        for (uint32_t i = threadIdx.x * 16; i < nbytes; i += kHllLdsWG * 16)
            *reinterpret_cast<u32x4_t*>(nib + i) = load16(P.snap + i);
    } else {
        for (uint32_t i = threadIdx.x; i < nbytes; i += kHllLdsWG) nib[i] = P.snap[i];
    }
    // the floor F (min register) is the min of the group floors, derived here rather than by a separate kernel
    __shared__ uint32_t wmin[kHllLdsWG / 64];
    uint32_t f = 0xFFFFFFFFu;
    for (uint32_t i = threadIdx.x; i < ngroups; i += kHllLdsWG) {
        const uint32_t g = P.gfloor[i];
        gfl[i] = (unsigned char)g;
        f = min(f, g);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f = min(f, (uint32_t)__shfl_xor((int)f, o, 64));
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = f;
    __syncthreads();
    f = wmin[0];
#pragma unroll
    for (uint32_t w = 1; w < kHllLdsWG / 64; ++w) f = min(f, wmin[w]);
    const uint32_t F = min(f, 64u - (uint32_t)P.p);
    (void)floor_ptr;
    const uint64_t zmask = F == 0 ? 0ull : (((1ull << F) - 1ull) << (64 - P.p - F));  // rl > F <=> these bits are 0
    const uint32_t w0 = d_begin + blockIdx.x * per_wg;
    const uint32_t w1 = min(d_end, w0 + per_wg);
    if (w0 >= w1) return;  // workgroup-uniform: no docs, nothing logged
    constexpr uint32_t kPer = E32 ? 8u : 4u;  // docs per thread and buffer
    constexpr uint32_t kIt = kHllLdsWG * kPer;
    const uint32_t t4 = threadIdx.x * kPer;
    // unconditional loads (past the range: the range's last 4 docs again, never hashed), so the compiler can count
    // them: a conditional load makes every later wait a vmcnt(0), which drains the other buffer's prefetch too
    const uint32_t last4 = (w1 - 1) & ~3u;
    auto load = [&](uint32_t i0, uint64_t raw[4]) {
        if (E32) {  // two words per 64-bit slot: docs i0 + 2k and i0 + 2k + 1 in the low / high half of raw[k]
            uint32_t w[8];
            load_u32x4(P.enc32, min(i0, last4), w);
            load_u32x4(P.enc32, min(i0 + 4, last4), w + 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) raw[k] = (uint64_t)w[2 * k] | (uint64_t)w[2 * k + 1] << 32;
        } else {
            load_i64x4((const int64_t*)P.col, min(i0, last4), (int64_t*)raw);
        }
    };
    auto hash4 = [&](uint32_t i0, const uint64_t raw[4], int half) {
        if (i0 >= w1) return;
        const uint32_t lim = w1 - i0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t rl = 0, idx = 0;
            bool t;
            if (E32) {
                const uint32_t e = hll_enc32_entry((uint32_t)(raw[(half * 4 + j) >> 1] >> (32 * (j & 1))), P.p);
                rl = e >> 24;
                idx = e & 0xFFFFFFu;
                t = (uint32_t)j < lim && rl > F;
            } else {
                const uint64_t h = hll_fast_hash<KIND>(P, raw[j]);
                t = (uint32_t)j < lim && (h & zmask) == 0;
                if (t) {
                    rl = hll_run_len(h, P.p);
                    idx = hll_index(h, P.p);
                }
            }
            if (t) {
                const uint32_t bi = idx / kHllPerByte;
                const uint32_t byte = nib[bi];
                const uint32_t sh = (idx % kHllPerByte) * kHllBits;
                const uint32_t gf = gfl[idx >> gshift];
                if (rl > gf + ((byte >> sh) & kHllMaxDelta)) {
                    // logged (a lost nibble write only repeats a log entry: the log holds the values, the nibbles
                    // only filter), or past the log's end an atomicMax straight on the register
                    const uint32_t k = logm ? atomicAdd(nlog, 1u) : kHllLog;
                    if (k < kHllLog) rlog[k] = (rl << 24) | idx;
                    else atomicMax(&P.regs[idx], rl);
                    nib[bi] = (unsigned char)((byte & ~(kHllMaxDelta << sh)) | (min(rl - gf, kHllMaxDelta) << sh));
                }
            }
        }
    };
    // ESGPU_HLL_NBUF buffers, each reloaded right after it is hashed: no register copies (which would wait for the
    // loads); the prologue issues them in the loop's order (the loop head's wait counts merge both paths)
    auto take = [&](uint32_t i0, const uint64_t raw[4]) {
        hash4(i0, raw, 0);
        if (E32) hash4(i0 + 4, raw, 1);
    };
    uint64_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    load(w0 + t4, a);
    __builtin_amdgcn_sched_barrier(0);
    load(w0 + kIt + t4, b);
#if ESGPU_HLL_NBUF == 3
    uint64_t c[4] = {0, 0, 0, 0};
    __builtin_amdgcn_sched_barrier(0);
    load(w0 + 2 * kIt + t4, c);
    for (uint32_t base = w0; base < w1; base += 3 * kIt) {
        take(base + t4, a);
        load(base + 3 * kIt + t4, a);
        take(base + kIt + t4, b);
        load(base + 4 * kIt + t4, b);
        take(base + 2 * kIt + t4, c);
        load(base + 5 * kIt + t4, c);
    }
#else
    for (uint32_t base = w0; base < w1; base += 2 * kIt) {
        take(base + t4, a);
        load(base + 2 * kIt + t4, a);
        take(base + kIt + t4, b);
        load(base + 3 * kIt + t4, b);
    }
#endif
    if (!logm) return;
    // the log out, partitioned by register range like hll_p0_scatter: per range a count, one global reservation, then
    // each entry at its range's base + its cursor (past the range's capacity: an atomicMax straight on the register)
    __syncthreads();
    const uint32_t n = min(*nlog, kHllLog);
    const uint32_t R = hll_p0_ranges(m);
    const uint32_t rshift = (uint32_t)P.p - (31u - (uint32_t)__builtin_clz(R));
    for (uint32_t i = threadIdx.x; i < R; i += kHllLdsWG) { lcnt[i] = 0; lcur[i] = 0; }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += kHllLdsWG) atomicAdd(&lcnt[(rlog[i] & 0xFFFFFFu) >> rshift], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < R; i += kHllLdsWG) lbase[i] = lcnt[i] ? atomicAdd(&P.p0_cnt[i], lcnt[i]) : 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += kHllLdsWG) {
        const uint32_t e = rlog[i], idx = e & 0xFFFFFFu, r = idx >> rshift;
        const uint32_t slot = lbase[r] + atomicAdd(&lcur[r], 1u);
        if (slot < P.p0_cap) P.p0_buf[(size_t)r * P.p0_cap + slot] = e;
        else atomicMax(&P.regs[idx], e >> 24);
    }
}

// Floored stream (one pass over the segment instead of phase 0 + the LDS phases, when the request's values per register
// are many): a register that will hold at least F is decided only by hashes with run length >= F, i.e. those whose F - 1
// bits below the index bits are zero -- one 64-bit AND per hash.  Those (a fraction 2^-(F-1)) are logged in LDS and
// flushed, partitioned by register range, into fs_buf for one gather (hll_p0_gather_kernel); the host picks F so that
// a register ending below F is a ~5e-3 event per request, and the tail pass (hll_lc_kernel) finishes such registers
// from the hashes below F.  No snapshot, no phase structure: the pass streams the column at the HBM rate.
#ifndef ESGPU_HLL_FS_WG
#define ESGPU_HLL_FS_WG 1024
#endif
#ifndef ESGPU_HLL_FS_NBUF  // load buffers per thread (2 or 3)
#define ESGPU_HLL_FS_NBUF 2
#endif
constexpr uint32_t kHllFsWG = ESGPU_HLL_FS_WG;
constexpr uint32_t kHllFsIter = kHllFsWG * 4;
// LDS log entries; the count is checked every ~kHllFsLog / 4 expected entries and the log flushed once it is over half
// full (measured at 125M docs: 0.231 ms; a fixed flush schedule with 18,432 / 19,456 entries 0.248 / 0.240 ms)
#ifndef ESGPU_HLL_FS_LOG
#define ESGPU_HLL_FS_LOG 16384
#endif
constexpr uint32_t kHllFsLog = ESGPU_HLL_FS_LOG;
constexpr uint32_t hll_fs_lds_bytes() { return kHllFsLog * 4u + 3u * 256u * 4u + 16u; }

// one workgroup's log out, partitioned by register range (as the LDS phase kernel's end does); the callers barrier
// before (the log is complete) and this barriers before returning (the log may be reused)
__device__ __forceinline__ void hll_fs_flush(const HllParams& P, uint32_t* rlog, uint32_t* lcnt, uint32_t* lcur,
                                             uint32_t* lbase, uint32_t* nlog) {
    const uint32_t m = 1u << P.p;
    const uint32_t n = min(*nlog, kHllFsLog);
    const uint32_t R = hll_p0_ranges(m);
    const uint32_t rshift = (uint32_t)P.p - (31u - (uint32_t)__builtin_clz(R));
    for (uint32_t i = threadIdx.x; i < R; i += kHllFsWG) { lcnt[i] = 0; lcur[i] = 0; }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += kHllFsWG) atomicAdd(&lcnt[(rlog[i] & 0xFFFFFFu) >> rshift], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < R; i += kHllFsWG) lbase[i] = lcnt[i] ? atomicAdd(&P.p0_cnt[i], lcnt[i]) : 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += kHllFsWG) {
        const uint32_t e = rlog[i], idx = e & 0xFFFFFFu, r = idx >> rshift;
        const uint32_t slot = lbase[r] + atomicAdd(&lcur[r], 1u);
        if (slot < P.fs_cap) P.fs_buf[(size_t)r * P.fs_cap + slot] = e;
        else atomicMax(&P.regs[idx], e >> 24);
    }
    __syncthreads();
    if (threadIdx.x == 0) *nlog = 0;
    __syncthreads();
}

// the enc32 form of one hash (HllParams.enc32): its top kP2 bits and min(nlz(h << kP2), 64 - kP2)
__device__ __forceinline__ uint32_t hll_enc32(uint64_t h) {
    const uint32_t z = (uint32_t)clz64(h << kP2);
    return (uint32_t)(h >> (64 - kP2)) << 7 | min(z, 64u - kP2);
}
// index and run length of an enc32 word, as hll_index / hll_run_len of its hash (p <= kP2): the kP2 - p bits below the
// index decide the run length if any is set (decodeRunLen's even case, HyperLogLogPlusPlus.java:349-357), else it is
// kP2 - p plus the stored count plus one (the odd case; the count is clamped at 64 - kP2 as runLen clamps at 64 - p)
__device__ __forceinline__ uint32_t hll_enc32_entry(uint32_t v, int p) {
    const uint32_t e = v >> 7, s = (uint32_t)(kP2 - p);
    const uint32_t low = s ? (e & ((1u << s) - 1u)) : 0u;
    const uint32_t rl = low ? (uint32_t)__builtin_clz(low) - (32u - s) + 1u : s + (v & 127u) + 1u;
    return rl << 24 | (e >> s);
}

template <int KIND>
__global__ __launch_bounds__(256) void hll_enc32_kernel(const void* col, uint32_t n, uint32_t* out) {
    HllParams P{};
    const uint32_t i0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (i0 >= n) return;  // n is a multiple of 4 (the column's padding)
    int64_t raw[4];
    load_i64x4((const int64_t*)col, i0, raw);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = hll_enc32(hll_fast_hash<KIND>(P, (uint64_t)raw[j]));
    *(uint4*)(out + i0) = make_uint4(o[0], o[1], o[2], o[3]);
}

void launch_hll_enc32(const void* col, int kind, uint32_t n_pad, uint32_t* out, hipStream_t st) {
    const dim3 g((n_pad / 4 + 255) / 256);
    if (n_pad == 0) return;
    if (kind == HLL_F64) hipLaunchKernelGGL(hll_enc32_kernel<HLL_F64>, g, dim3(256), 0, st, col, n_pad, out);
    else hipLaunchKernelGGL(hll_enc32_kernel<HLL_I64>, g, dim3(256), 0, st, col, n_pad, out);
}

// E32: the enc32 words (4 bytes per doc) instead of the values, 8 docs per thread and buffer (the same bytes in flight)
template <int KIND, bool E32>
__global__ __launch_bounds__(kHllFsWG) void hll_fs_kernel(HllParams P, uint32_t per_wg, uint32_t check_iters) {
    extern __shared__ __attribute__((aligned(16))) uint32_t fs_lds[];
    uint32_t* rlog = fs_lds;                // [kHllFsLog] (rl << 24 | idx)
    uint32_t* lcnt = rlog + kHllFsLog;      // [256]
    uint32_t* lcur = lcnt + 256;            // [256]
    uint32_t* lbase = lcur + 256;           // [256]
    uint32_t* nlog = lbase + 256;           // [1]
    if (threadIdx.x == 0) *nlog = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *P.unres = 0;  // counted by the gather that follows this launch
    const uint32_t G = P.fs_f - 1;          // kept: run length > G <=> the G bits below the index bits are zero
    const uint64_t zmask = G == 0 ? 0ull : (((1ull << G) - 1ull) << (64 - P.p - G));
    const uint32_t w0 = blockIdx.x * per_wg;
    const uint32_t w1 = min(P.n_docs, w0 + per_wg);
    __syncthreads();
    if (w0 >= w1) return;  // workgroup-uniform
    constexpr uint32_t kPer = E32 ? 8u : 4u;  // docs per thread and buffer
    constexpr uint32_t kIt = kHllFsWG * kPer;
    const uint32_t t4 = threadIdx.x * kPer;
    const uint32_t last4 = (w1 - 1) & ~3u;  // unconditional loads (see hll_registers_lds_kernel)
    auto load = [&](uint32_t i0, uint64_t raw[4]) {
        if (E32) {  // two words per 64-bit slot: docs i0 + 2k and i0 + 2k + 1 in the low / high half of raw[k]
            uint32_t w[8];
            load_u32x4(P.enc32, min(i0, last4), w);
            load_u32x4(P.enc32, min(i0 + 4, last4), w + 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) raw[k] = (uint64_t)w[2 * k] | (uint64_t)w[2 * k + 1] << 32;
        } else {
            load_i64x4((const int64_t*)P.col, min(i0, last4), (int64_t*)raw);
        }
    };
    // the thread's 4 hashes, then ONE log reservation per wave for all of the wave's entries (one returning LDS atomic
    // and one wait per 256 docs instead of one per doc slot); called by every thread of the workgroup
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
    auto hash4 = [&](uint32_t i0, const uint64_t raw[4], int half) {
        const uint32_t lim = i0 < w1 ? w1 - i0 : 0u;
        uint32_t e[4], hit = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bool t;
            if (E32) {
                const uint32_t v = (uint32_t)(raw[(half * 4 + j) >> 1] >> (32 * (j & 1)));
                e[j] = hll_enc32_entry(v, P.p);
                t = (uint32_t)j < lim && (e[j] >> 24) > G;
            } else {
                const uint64_t h = hll_fast_hash<KIND>(P, raw[j]);
                t = (uint32_t)j < lim && (h & zmask) == 0;
                e[j] = (hll_run_len(h, P.p) << 24) | hll_index(h, P.p);
            }
            hit |= (t ? 1u : 0u) << j;
        }
        const uint64_t m0 = __ballot(hit & 1u), m1 = __ballot(hit & 2u), m2 = __ballot(hit & 4u), m3 = __ballot(hit & 8u);
        const uint32_t c0 = (uint32_t)__popcll(m0), c1 = (uint32_t)__popcll(m1), c2 = (uint32_t)__popcll(m2);
        const uint32_t tot = c0 + c1 + c2 + (uint32_t)__popcll(m3);
        if (tot == 0) return;  // wave-uniform
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(nlog, tot);
        base = __shfl(base, 0, 64);
        const uint32_t off[4] = {(uint32_t)__popcll(m0 & lt), c0 + (uint32_t)__popcll(m1 & lt),
                                 c0 + c1 + (uint32_t)__popcll(m2 & lt), c0 + c1 + c2 + (uint32_t)__popcll(m3 & lt)};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!((hit >> j) & 1u)) continue;
            const uint32_t k = base + off[j];
            if (k < kHllFsLog) rlog[k] = e[j];
            else atomicMax(&P.regs[e[j] & 0xFFFFFFu], e[j] >> 24);  // never expected: flushed at half full
        }
    };
    // one buffer's docs: 4 (values) or 8 (enc32 words, two hash4 rounds)
    auto take = [&](uint32_t i0, const uint64_t raw[4]) {
        hash4(i0, raw, 0);
        if (E32) hash4(i0 + 4, raw, 1);
    };
    uint64_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    load(w0 + t4, a);
    __builtin_amdgcn_sched_barrier(0);
    load(w0 + kIt + t4, b);
    uint32_t it = 0;
#if ESGPU_HLL_FS_NBUF == 3
    uint64_t c[4] = {0, 0, 0, 0};
    __builtin_amdgcn_sched_barrier(0);
    load(w0 + 2 * kIt + t4, c);
    for (uint32_t base = w0; base < w1; base += 3 * kIt) {
        take(base + t4, a);
        load(base + 3 * kIt + t4, a);
        take(base + kIt + t4, b);
        load(base + 4 * kIt + t4, b);
        take(base + 2 * kIt + t4, c);
        load(base + 5 * kIt + t4, c);
#else
    for (uint32_t base = w0; base < w1; base += 2 * kIt) {
        take(base + t4, a);
        load(base + 2 * kIt + t4, a);
        take(base + kIt + t4, b);
        load(base + 3 * kIt + t4, b);
#endif
        if (++it == check_iters) {  // workgroup-uniform: every thread runs the same iterations
            it = 0;
            __syncthreads();
            const uint32_t n = *nlog;
            __syncthreads();
            if (n > kHllFsLog / 2) hll_fs_flush(P, rlog, lcnt, lcur, lbase, nlog);
        }
    }
    __syncthreads();
    hll_fs_flush(P, rlog, lcnt, lcur, lbase, nlog);
}

// the refresh (or the phase-0 gather) counts the non-zero registers as it reads them: each block adds its count to
// nz_part[0]; the last block to finish raises *nonzero to the total and re-arms the pair.  Registers only grow, so
// the count is a lower bound on the registers at the end of the segment, which is all the LINEAR_COUNTING decision
// needs (a lower bound above the threshold proves HYPERLOGLOG; otherwise the LC pass counts exactly)
__device__ __forceinline__ void hll_count_nonzero(const HllParams& P, uint32_t nz, uint32_t* wsum) {
    nz = wave_sum_u32(nz);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = nz;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; ++w) t += wsum[w];
        if (t) atomicAdd(&P.nz_part[0], t);
        __threadfence();
        if (atomicAdd(&P.nz_part[1], 1u) == gridDim.x - 1) {
            atomicMax(P.nonzero, atomicExch(&P.nz_part[0], 0u));
            atomicExch(&P.nz_part[1], 0u);
        }
    }
}

// one refresh between register phases: per group of 64 registers (one wave) its floor (min register) and each
// register's 4-bit lower bound over that floor, nibble = min(reg - group floor, 15), packed two per byte.  The phase
// kernel derives the global floor from the group floors itself, so no second kernel, memset or atomic is needed.
__global__ __launch_bounds__(1024) void hll_refresh_kernel(HllParams P) {
    static_assert(kHllBits == 4, "two nibbles per snapshot byte");
    __shared__ uint32_t wsum[16];
    const uint32_t m = 1u << P.p;
    const uint32_t gsz = m >= kHllGroup ? kHllGroup : m;
    const uint32_t g = blockIdx.x * 16 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const bool live = g * gsz < m && lane < gsz;
    const uint32_t r = live ? P.regs[g * gsz + lane] : 0xFFFFFFFFu;
    uint32_t v = r;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    const uint32_t d = live ? min(r - v, kHllMaxDelta) : 0u;
    const uint32_t hi = (uint32_t)__shfl_down((int)d, 1, 64);  // the odd neighbour's nibble
    if (g * gsz < m) {
        if (lane == 0) P.gfloor[g] = (unsigned char)min(v, 255u);
        if (live && (lane & 1) == 0) P.snap[(g * gsz + lane) / 2] = (unsigned char)(d | (lane + 1 < gsz ? hi << 4 : 0u));
    }
    hll_count_nonzero(P, live && r != 0 ? 1u : 0u, wsum);
}

// Phase 0 by register range (a fresh request's first cut0 * m values, when every hash finds an empty or low
// register): instead of one scattered global atomicMax per hash (~4 per register, the atomic rate bounds it), the
// entries are partitioned by register range and each range's owner maxes them in LDS and stores its registers once.
// hll_p0_scatter: 16 docs per thread, a slot per entry reserved in LDS per range, one global reservation per (workgroup,
// range); an entry past its range's capacity raises its register with an atomicMax directly (never expected: the
// capacity is ~8 sigma above the mean).
constexpr uint32_t kP0WG = 256, kP0Docs = 16;
template <int KIND>
__global__ __launch_bounds__(kP0WG) void hll_p0_scatter_kernel(HllParams P, uint32_t d_end) {
    __shared__ uint32_t lcnt[256], lbase[256];
    const uint32_t m = 1u << P.p, R = hll_p0_ranges(m);
    const uint32_t rshift = (uint32_t)P.p - (31u - (uint32_t)__builtin_clz(R));  // log2(m / R)
    for (uint32_t i = threadIdx.x; i < R; i += kP0WG) lcnt[i] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kP0WG * kP0Docs;
    const uint32_t last4 = (d_end - 1) & ~3u;
    uint64_t raw[kP0Docs];
#pragma unroll
    for (uint32_t k = 0; k < kP0Docs / 4; ++k)
        load_i64x4((const int64_t*)P.col, min(base + (k * kP0WG + threadIdx.x) * 4, last4), (int64_t*)&raw[4 * k]);
    uint32_t ent[kP0Docs], pos[kP0Docs];
#pragma unroll
    for (uint32_t k = 0; k < kP0Docs; ++k) {
        const uint32_t d = base + ((k / 4) * kP0WG + threadIdx.x) * 4 + (k & 3);
        const uint64_t h = hll_fast_hash<KIND>(P, raw[k]);
        const uint32_t idx = hll_index(h, P.p);
        ent[k] = (hll_run_len(h, P.p) << 24) | idx;
        pos[k] = d < d_end ? atomicAdd(&lcnt[idx >> rshift], 1u) : ~0u;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < R; i += kP0WG) lbase[i] = lcnt[i] ? atomicAdd(&P.p0_cnt[i], lcnt[i]) : 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kP0Docs; ++k) {
        if (pos[k] == ~0u) continue;
        const uint32_t idx = ent[k] & 0xFFFFFFu, r = idx >> rshift;
        const uint32_t slot = lbase[r] + pos[k];
        if (slot < P.p0_cap) P.p0_buf[(size_t)r * P.p0_cap + slot] = ent[k];
        else atomicMax(&P.regs[idx], ent[k] >> 24);
    }
}
// hll_p0_gather: one workgroup per range: its registers maxed with its entries in LDS, stored once, and the range's
// group floors and nibble snapshot written as hll_refresh_kernel would (the first LDS phase needs no refresh launch);
// the range's fill counter is re-armed for the next request
__global__ __launch_bounds__(1024) void hll_p0_gather_kernel(HllParams P, int count) {
    static_assert(kHllBits == 4, "two nibbles per snapshot byte");
    __shared__ uint32_t reg[1024];
    const uint32_t m = 1u << P.p, per = m / hll_p0_ranges(m);  // 64 .. 1024 registers (p <= 18)
    const uint32_t b = blockIdx.x, r0 = b * per;
    for (uint32_t i = threadIdx.x; i < per; i += 1024) reg[i] = P.regs[r0 + i];
    __syncthreads();
    const uint32_t cap = P.fs_f ? P.fs_cap : P.p0_cap;
    const uint32_t n = min(P.p0_cnt[b], cap);
    const uint32_t* src = (P.fs_f ? P.fs_buf : P.p0_buf) + (size_t)b * cap;
    // eight entries' loads issued before their LDS maxes (a range holds ~30K entries at 125M docs: one dependent load
    // per entry left the gather latency-bound)
    uint32_t i = threadIdx.x;
    for (; i + 7 * 1024 < n; i += 8 * 1024) {
        uint32_t e[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = src[i + k * 1024];
#pragma unroll
        for (int k = 0; k < 8; ++k) atomicMax(&reg[(e[k] & 0xFFFFFFu) - r0], e[k] >> 24);
    }
    for (; i < n; i += 1024) {
        const uint32_t e = src[i];
        atomicMax(&reg[(e & 0xFFFFFFu) - r0], e >> 24);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < per; i += 1024) P.regs[r0 + i] = reg[i];
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t gl = threadIdx.x >> 6; gl < per / kHllGroup; gl += 16) {
        const uint32_t v0 = reg[gl * kHllGroup + lane];
        uint32_t v = v0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
        if (lane == 0) P.gfloor[r0 / kHllGroup + gl] = (unsigned char)min(v, 255u);
        const uint32_t d = min(v0 - v, kHllMaxDelta);
        const uint32_t hi = (uint32_t)__shfl_down((int)d, 1, 64);
        if ((lane & 1) == 0) P.snap[(r0 + gl * kHllGroup + lane) / 2] = (unsigned char)(d | (hi << 4));
    }
    if (threadIdx.x == 0) atomicExch(&P.p0_cnt[b], 0u);
    if (P.fs_f) {  // floored stream: registers below the floor are finished by the tail pass
        uint32_t u = 0;
        for (uint32_t i = threadIdx.x; i < per; i += 1024) u += reg[i] < P.fs_f;
        u = wave_sum_u32(u);
        if ((threadIdx.x & 63) == 0 && u) atomicAdd(P.unres, u);
    }
    if (!count) return;  // only the segment's last gather counts (the LC decision reads the final registers)
    uint32_t nz = 0;
    for (uint32_t i = threadIdx.x; i < per; i += 1024) nz += reg[i] != 0;
    __shared__ uint32_t wsum[16];
    hll_count_nonzero(P, nz, wsum);
}

// group floors: one wave per group of 64 registers; with `out`, the global floor is their min (*out initialised to ~0),
// one atomic per workgroup of 16 groups
__global__ __launch_bounds__(1024) void hll_group_floor_kernel(const unsigned int* regs, uint32_t m, unsigned char* gfloor,
                                                               unsigned int* out) {
    __shared__ uint32_t wmin[16];
    const uint32_t gsz = m >= kHllGroup ? kHllGroup : m;
    const uint32_t g = blockIdx.x * 16 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t v = (g * gsz < m && lane < gsz) ? regs[g * gsz + lane] : 0xFFFFFFFFu;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    if (lane == 0) {
        if (g * gsz < m) gfloor[g] = (unsigned char)min(v, 255u);
        wmin[threadIdx.x >> 6] = v;
    }
    if (!out) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = wmin[0];
        for (int w = 1; w < 16; ++w) t = min(t, wmin[w]);
        atomicMin(out, t);
    }
}

// min over the registers -> *out (initialised to ~0 by the launcher); one read of the 2^p words by 64 workgroups
__global__ __launch_bounds__(1024) void hll_floor_kernel(const unsigned int* regs, uint32_t m, unsigned int* out) {
    uint32_t mn = 0xFFFFFFFFu;
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < m; i += gridDim.x * 1024) mn = min(mn, regs[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    __shared__ uint32_t part[16];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = part[0];
        for (int w = 1; w < 16; ++w) t = min(t, part[w]);
        atomicMin(out, t);
    }
}

// number of non-zero registers: a lower bound on the number of distinct encoded hashes (distinct register indices
// come from distinct encodeHash values), so nonzero > threshold proves the reference ends in HYPERLOGLOG mode.
__global__ __launch_bounds__(1024) void hll_nonzero_kernel(const unsigned int* regs, uint32_t m, unsigned int* out) {
    uint32_t n = 0;
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < m; i += gridDim.x * 1024) n += regs[i] != 0;
    __shared__ uint32_t part[16];
    n = wave_sum_u32(n);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < 16; ++w) t += part[w];
        if (t) atomicAdd(out, t);  // *out is zeroed with the plan's accumulators
    }
}

// pass 2 (only while nonzero <= threshold): the exact LINEAR_COUNTING set of encodeHash values.  Open addressing,
// probes bounded by threshold+1 (a longer run proves > threshold distinct values), stops once the count passes
// the threshold.  Final mode = LC iff count <= threshold, exactly as Hashset.add/upgradeToHll decide.
// With the floored stream the same launch is its tail pass: while the gather left registers below the floor F
// (*unres, a ~5e-3 event), every hash with run length < F raises its register if it is still below -- registers at or
// above F are exact already and are only read.
__global__ __launch_bounds__(256) void hll_lc_kernel(HllParams P) {
    const bool fix = P.fs_f && *P.unres != 0;
    bool lc = *P.nonzero <= P.lc_threshold;  // else already proven HYPERLOGLOG
    if (!lc && !fix) return;
    const uint32_t gsz = gridDim.x * blockDim.x;
    for (uint32_t i0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4; i0 < P.n_docs; i0 += gsz * 4) {
        if (lc && __hip_atomic_load(P.lc_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > P.lc_threshold) {
            if (!fix) return;
            lc = false;
        }
        uint64_t raw[4], hv[4];
        hll_load_raw(P, i0, raw);
        const uint32_t ok = hll_hash_raw(P, i0, raw, hv);
        if (fix) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t rl = hll_run_len(hv[j], P.p), idx = hll_index(hv[j], P.p);
                if (((ok >> j) & 1) && rl < P.fs_f && P.regs[idx] < rl) atomicMax(&P.regs[idx], rl);
            }
        }
        if (!lc) continue;
        uint32_t added = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!((ok >> j) & 1)) continue;
            const uint32_t enc = hll_encode(hv[j], P.p);
            const unsigned long long pos = P.pos_base + (P.pos_ord ? raw[j] : (uint64_t)(i0 + j));
            uint32_t slot = (uint32_t)(mix64(enc) & P.lc_mask);
            for (uint32_t probe = 0; probe <= P.lc_threshold + 1; ++probe) {
                const uint32_t cur = __hip_atomic_load(&P.lc_set[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                bool found = cur == enc;
                if (!found && cur == 0) {
                    const uint32_t prev = atomicCAS(&P.lc_set[slot], 0u, enc);
                    if (prev == 0) ++added;
                    found = prev == 0 || prev == enc;
                }
                if (found) {
                    atomicMin(&P.lc_first[slot], pos);
                    break;
                }
                if (probe == P.lc_threshold + 1) { added = P.lc_threshold + 1; break; }  // run longer than the set
                slot = (slot + 1) & P.lc_mask;
            }
        }
        if (added) atomicAdd(P.lc_count, added);
    }
}

uint32_t hll_fs_floor(uint64_t total, int p, uint32_t min_f) {
    const double m = (double)(1u << p);
    const double lam = (double)total / m, need = std::log(m) + 5.3;  // m * exp(-lam * 2^-(F-1)) <= 5e-3
    if (lam < need * 2.0) return 0;
    const uint32_t f = 1u + (uint32_t)std::floor(std::log2(lam / need));
    const uint32_t fmax = 64u - (uint32_t)p;  // run lengths top out at 64 - p + 1
    const uint32_t F = std::min(f, fmax);
    return F >= min_f ? F : 0u;
}
uint32_t hll_fs_cap(uint64_t n, int p, uint32_t f) {
    const uint32_t R = hll_p0_ranges(1u << p);
    const double e = (double)n / std::ldexp(1.0, (int)f - 1) / R;  // mean entries per range
    const double c = e + e / 8 + 8 * std::sqrt(e) + 256;
    return (uint32_t)std::min(c, 4.0e9) & ~3u;
}

bool launch_hll(const HllParams& p, uint32_t cus, hipStream_t st) {
    const uint32_t n = p.n_docs;
    const uint32_t m = 1u << p.p;
    // phases [0, 4m), then x4 each: every register has seen ~4 hashes after the first cut, so the floor (min
    // register) starts to rise, and each later phase reads registers only for hashes longer than the floor.  The cuts
    // are positions in the request's whole value stream: a later segment (p.seen values already in the registers)
    // continues the sequence -- its first phase refreshes the floor and snapshot and runs the LDS pass at once,
    // instead of restarting with a floor-0 phase that reads a register for every hash.
    std::vector<uint32_t> cuts{0};
#ifndef ESGPU_HLL_GROW
#define ESGPU_HLL_GROW 4
#endif
    const uint32_t cut0 = p.cut0 ? p.cut0 : ESGPU_HLL_CUT0;
    uint64_t c = (uint64_t)m * cut0;
    while (c <= p.seen) c *= ESGPU_HLL_GROW;
    while (c < p.seen + n) {
        cuts.push_back((uint32_t)(c - p.seen) & ~3u);
        c *= ESGPU_HLL_GROW;
    }
    cuts.push_back(n);
    const uint32_t wgs_max = cus * 8;  // 8 workgroups of 256 threads per CU
    const bool fast = !p.accept && p.npred == 0 && !p.present;
#ifndef ESGPU_HLL_LDS
#define ESGPU_HLL_LDS 1
#endif
    const bool lds = ESGPU_HLL_LDS && fast && p.snap && (p.kind == HLL_I64 || p.kind == HLL_F64) && p.p >= 4;
    const uint32_t floor_grid = std::max(1u, std::min(64u, m / 4096));
    // floor (and group floors + LDS snapshot) of the registers as they stand
    auto refresh = [&]() {
        const uint32_t ng = m >= kHllGroup ? m / kHllGroup : 1u;
        if (lds) {  // group floors and the nibble snapshot in one pass
            hipLaunchKernelGGL(hll_refresh_kernel, dim3((ng + 15) / 16), dim3(1024), 0, st, p);
            return;
        }
        (void)hipMemsetAsync(p.floor, 0xFF, 4, st);
        if (fast)
            hipLaunchKernelGGL(hll_group_floor_kernel, dim3((ng + 15) / 16), dim3(1024), 0, st, (const unsigned int*)p.regs, m,
                               p.gfloor, p.floor);
        else
            hipLaunchKernelGGL(hll_floor_kernel, dim3(floor_grid), dim3(1024), 0, st, (const unsigned int*)p.regs, m, p.floor);
    };
    // LC / tail pass: mostly a launch whose blocks see *nonzero above the threshold and return at once; 2048 blocks
    // loop over the docs when it does run
    auto tail = [&](const HllParams& t) {
        uint32_t grid = (n + 1023) / 1024;
        if (grid > 2048) grid = 2048;
        if (grid == 0) grid = 1;
        hipLaunchKernelGGL(hll_lc_kernel, dim3(grid), dim3(256), 0, st, t);
    };
    if (p.fs_f && lds && p.p0_cnt && p.p >= 12 && n > 0) {
        // floored stream: one resident wave of workgroups, contiguous ranges; the log is checked every ~kHllFsLog / 4
        // expected entries (2^(F-1) docs per entry)
        static int per_cu = 0;
        if (!per_cu) {
            int b = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, hll_fs_kernel<HLL_I64, false>, kHllFsWG, hll_fs_lds_bytes()) != hipSuccess || b < 1)
                b = 1;
            per_cu = b;
        }
        const uint64_t docs_per_check = ((uint64_t)kHllFsLog / 4) << (p.fs_f - 1);
        const bool e32 = p.enc32 != nullptr && p.p <= kP2;
        const uint32_t it_docs = kHllFsIter * (e32 ? 2u : 1u);  // docs per buffer and workgroup
        uint32_t wgs = std::max(1u, std::min(cus * (uint32_t)per_cu, n / (it_docs * ESGPU_HLL_FS_NBUF)));
        const uint32_t per = ((n + wgs - 1) / wgs + 3) & ~3u;
        wgs = (n + per - 1) / per;
        const uint32_t check = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1u << 20, docs_per_check / (ESGPU_HLL_FS_NBUF * it_docs)));
        if (e32)
            hipLaunchKernelGGL((hll_fs_kernel<HLL_I64, true>), dim3(wgs), dim3(kHllFsWG), hll_fs_lds_bytes(), st, p, per, check);
        else if (p.kind == HLL_I64)
            hipLaunchKernelGGL((hll_fs_kernel<HLL_I64, false>), dim3(wgs), dim3(kHllFsWG), hll_fs_lds_bytes(), st, p, per, check);
        else
            hipLaunchKernelGGL((hll_fs_kernel<HLL_F64, false>), dim3(wgs), dim3(kHllFsWG), hll_fs_lds_bytes(), st, p, per, check);
        hipLaunchKernelGGL(hll_p0_gather_kernel, dim3(hll_p0_ranges(m)), dim3(1024), 0, st, p, 1);
        tail(p);  // its raises (registers below the floor) keep the gather's floors and snapshot lower bounds
        return true;
    }
    HllParams q = p;  // the phases (fs_f = 0 for their gathers)
    q.fs_f = 0;
    const bool warm = p.seen >= (uint64_t)m * cut0;  // the registers already passed the first cut
    if (warm && !p.snap_ok) refresh();
#ifndef ESGPU_HLL_P0
#define ESGPU_HLL_P0 1
#endif
    // phase 0 partitioned by register range (the LDS phases' kinds, p >= 12: at least 64 ranges of whole groups)
    const bool p0 = ESGPU_HLL_P0 && lds && !warm && p.p >= 12 && p.p0_cnt && cuts.size() > 1 && cuts[1] > 0;
    // LDS phases log their raises and a gather applies them (p.log_raises, set by the host when p0_cnt is there)
    const bool logr = lds && p.log_raises && p.p0_cnt && p.p >= 12;
    bool counted = false;  // the last launch that touched the registers was a gather: *nonzero is exact
    for (size_t ph = 0; ph + 1 < cuts.size(); ++ph) {
        const uint32_t span = cuts[ph + 1] - cuts[ph];
        if (span == 0) continue;
        if (ph == 0 && p0) {
            const dim3 g1((span + kP0WG * kP0Docs - 1) / (kP0WG * kP0Docs));
            if (p.kind == HLL_I64) hipLaunchKernelGGL(hll_p0_scatter_kernel<HLL_I64>, g1, dim3(kP0WG), 0, st, q, span);
            else hipLaunchKernelGGL(hll_p0_scatter_kernel<HLL_F64>, g1, dim3(kP0WG), 0, st, q, span);
            hipLaunchKernelGGL(hll_p0_gather_kernel, dim3(hll_p0_ranges(m)), dim3(1024), 0, st, q, ph + 2 >= cuts.size() ? 1 : 0);
            counted = ph + 2 >= cuts.size();
            continue;  // the gather left the registers' group floors and snapshot behind: no refresh
        }
        const bool floored = warm || ph > 0;
        // contiguous range per workgroup, a multiple of 4 docs, at least 4 iterations of 1024 docs (the first phase is
        // small and latency-bound: every hash reads a register there, so it needs the whole chip)
        uint32_t wgs = std::max(1u, std::min(wgs_max, span / (kHllIter * 4)));
        const uint32_t per = ((span + wgs - 1) / wgs + 3) & ~3u;
        wgs = (span + per - 1) / per;
        const unsigned int* fl = floored ? (const unsigned int*)p.floor : (const unsigned int*)nullptr;
        if (lds && floored) {
            // one 1024-thread workgroup per CU (128 KB of nibbles at p = 18), more for smaller p
            const uint32_t per_cu = std::max(1u, std::min(4u, (uint32_t)(160u * 1024u / (hll_lds_bytes(m, logr) + 1024u))));
            uint32_t lw = std::max(1u, std::min(cus * per_cu, span / (kHllLdsIter * 4)));
            const uint32_t lper = ((span + lw - 1) / lw + 3) & ~3u;
            lw = (span + lper - 1) / lper;
            if (q.enc32 && q.p <= kP2)
                hipLaunchKernelGGL((hll_registers_lds_kernel<HLL_I64, true>), dim3(lw), dim3(kHllLdsWG), hll_lds_bytes(m, logr), st, q, cuts[ph], cuts[ph + 1], lper, fl);
            else if (p.kind == HLL_I64)
                hipLaunchKernelGGL((hll_registers_lds_kernel<HLL_I64, false>), dim3(lw), dim3(kHllLdsWG), hll_lds_bytes(m, logr), st, q, cuts[ph], cuts[ph + 1], lper, fl);
            else
                hipLaunchKernelGGL((hll_registers_lds_kernel<HLL_F64, false>), dim3(lw), dim3(kHllLdsWG), hll_lds_bytes(m, logr), st, q, cuts[ph], cuts[ph + 1], lper, fl);
        } else if (fast && p.kind == HLL_I64)
            hipLaunchKernelGGL(hll_registers_fast_kernel<HLL_I64>, dim3(wgs), dim3(kHllWG), 0, st, q, cuts[ph], cuts[ph + 1], per, fl);
        else if (fast && p.kind == HLL_F64)
            hipLaunchKernelGGL(hll_registers_fast_kernel<HLL_F64>, dim3(wgs), dim3(kHllWG), 0, st, q, cuts[ph], cuts[ph + 1], per, fl);
        else if (fast)
            hipLaunchKernelGGL(hll_registers_fast_kernel<HLL_ORD>, dim3(wgs), dim3(kHllWG), 0, st, q, cuts[ph], cuts[ph + 1], per, fl);
        else
            hipLaunchKernelGGL(hll_registers_kernel, dim3(wgs), dim3(kHllWG), 0, st, q, cuts[ph], cuts[ph + 1], per, fl);
        if (lds && floored && logr) {  // the phase's logged raises applied; floors, snapshot and count refreshed
            hipLaunchKernelGGL(hll_p0_gather_kernel, dim3(hll_p0_ranges(m)), dim3(1024), 0, st, q, ph + 2 >= cuts.size() ? 1 : 0);
            counted = ph + 2 >= cuts.size();
            continue;
        }
        counted = false;
        if (ph + 2 < cuts.size()) refresh();
    }
    if (!counted) {  // after a gather *nonzero is already the count of the final registers (hll_count_nonzero)
        (void)hipMemsetAsync(p.nonzero, 0, 4, st);  // recount over the registers (they accumulate across segments)
        hipLaunchKernelGGL(hll_nonzero_kernel, dim3(floor_grid), dim3(1024), 0, st, (const unsigned int*)p.regs, m, p.nonzero);
    }
    tail(q);  // fs_f = 0: reads the registers only
    return counted;  // the last phase's gather wrote the floors and snapshot of the final registers
}

// ------------------------------------------------------------------------------------------------------------
// build helpers
// ------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void term_totals_kernel(const unsigned long long* __restrict__ cnt, uint32_t H, uint32_t T,
                                                          unsigned long long* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    unsigned long long s = 0;
    for (uint32_t h = 0; h < H; ++h) s += cnt[(size_t)h * T + t];
    out[t] = s;
}

void launch_term_totals(const unsigned long long* cnt, uint32_t H, uint32_t T, unsigned long long* out, hipStream_t st) {
    hipLaunchKernelGGL(term_totals_kernel, dim3((T + 255) / 256), dim3(256), 0, st, cnt, H, T, out);
}

// out[r][h] = src[h][rows[r]] for every column array (k rows x H slots)
__global__ __launch_bounds__(256) void gather_rows_kernel(GatherParams P) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.k * P.H) return;
    const uint32_t r = i / P.H, h = i - r * P.H;
    const size_t src = (size_t)h * P.T + P.rows[r];
    for (int a = 0; a < P.narrays; ++a)
        P.dst[a][i] = (a == 0 && P.cnt32) ? (unsigned long long)((const unsigned int*)P.src[0])[src] : P.src[a][src];
}

// compact_rows, pass 1: non-empty key slots of each winner's row (one workgroup per row)
__global__ __launch_bounds__(256) void row_nnz_kernel(CompactParams P) {
    __shared__ uint32_t part[4];
    const uint32_t r = blockIdx.x, ord = P.rows[r];
    uint32_t n = 0;
    for (uint32_t s = threadIdx.x; s < P.H; s += 256) n += P.cnt[(size_t)s * P.T + ord] != 0ull;
    for (int o = 32; o > 0; o >>= 1) n += (uint32_t)__shfl_xor((int)n, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = part[0] + part[1] + part[2] + part[3];
        P.nnz[r] = t;
        P.o_nnz[r] = t;
    }
}

// compact_rows, pass 2: row r's non-empty slots written from position sum(nnz[0..r)), key-ascending, with every leaf's
// partials decoded (vc == 0: sum 0, min +inf, max -inf, sum of squares 0; a NaN collected: min = max = NaN)
__global__ __launch_bounds__(256) void compact_rows_kernel(CompactParams P) {
    __shared__ uint32_t part[4];
    __shared__ uint32_t wsum[4];
    const uint32_t r = blockIdx.x, ord = P.rows[r];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t b = 0;
    for (uint32_t j = threadIdx.x; j < r; j += 256) b += P.nnz[j];
    for (int o = 32; o > 0; o >>= 1) b += (uint32_t)__shfl_xor((int)b, o, 64);
    if (lane == 0) part[wave] = b;
    __syncthreads();
    uint64_t pos = (uint64_t)part[0] + part[1] + part[2] + part[3];
    for (uint32_t s0 = 0; s0 < P.H; s0 += 256) {
        const uint32_t s = s0 + threadIdx.x;
        const size_t cell = (size_t)s * P.T + ord;
        const unsigned long long c = s < P.H ? P.cnt[cell] : 0ull;
        const unsigned long long m = __ballot(c != 0ull);
        __syncthreads();  // wsum of the previous chunk consumed
        if (lane == 0) wsum[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint64_t at = pos + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        for (uint32_t w = 0; w < wave; ++w) at += wsum[w];
        pos += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (c == 0ull) continue;
        P.o_slot[at] = s;
        P.o_count[at] = (uint32_t)c;
        for (int l = 0; l < P.nleaves; ++l) {
            const CompactLeaf& L = P.leaf[l];
            const unsigned long long vc = L.o_count ? L.cnt[cell] : c;
            double sum = 0.0, mn = __builtin_inf(), mx = -__builtin_inf(), sq = 0.0;
            if (vc) {
                sum = L.sum[cell];
                if (L.mn) {
                    const uint64_t emn = L.mn[cell], emx = L.mx[cell];
                    if (emn < kEncNegInf || emx > kEncPosInf) { mn = __builtin_nan(""); mx = __builtin_nan(""); }
                    else { mn = unsortable(emn); mx = unsortable(emx); }
                }
                if (L.sq) sq = L.sq[cell];
            }
            if (L.o_count) L.o_count[at] = (uint32_t)vc;
            L.o_sum[at] = sum;
            if (L.o_min) {
                L.o_min[at] = mn;
                L.o_max[at] = mx;
            }
            if (L.o_sq) L.o_sq[at] = sq;
        }
    }
}

void launch_compact_rows(const CompactParams& p, hipStream_t st) {
    if (p.k == 0) return;
    hipLaunchKernelGGL(row_nnz_kernel, dim3(p.k), dim3(256), 0, st, p);
    hipLaunchKernelGGL(compact_rows_kernel, dim3(p.k), dim3(256), 0, st, p);
}

__global__ __launch_bounds__(256) void colo_merge_kernel(ColoParams P) {
    // the descriptors live in pinned host memory: each workgroup reads them once, over the link, into LDS
    __shared__ ColoShard shs[kColoMaxShards];
    __shared__ int32_t srow[kColoMaxShards];
    const uint32_t m = blockIdx.x * 256 + threadIdx.x, r = blockIdx.y;
    {
        const uint32_t words = P.nsh * (uint32_t)(sizeof(ColoShard) / 8);
        const unsigned long long* src = (const unsigned long long*)P.shards;
        unsigned long long* dst = (unsigned long long*)shs;
        for (uint32_t i = threadIdx.x; i < words; i += 256) dst[i] = src[i];
        for (uint32_t i = threadIdx.x; i < P.nsh; i += 256) srow[i] = P.rows[(size_t)r * P.nsh + i];
    }
    __syncthreads();
    if (m >= P.Hm) return;
    unsigned long long c = 0;
    unsigned long long vc[kCompactLeaves] = {0, 0, 0, 0}, mn[kCompactLeaves], mx[kCompactLeaves];
    double sum[kCompactLeaves] = {0.0, 0.0, 0.0, 0.0}, sq[kCompactLeaves] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int l = 0; l < kCompactLeaves; ++l) { mn[l] = kMinInit; mx[l] = kMaxInit; }
    // shard order: the reference reduce's addition order.  Eight shards at a time: every load of the eight is issued
    // before the first add (an absent shard reads cell 0 and adds nothing), so their latencies overlap
    constexpr int kC = 8;
    for (uint32_t sh0 = 0; sh0 < P.nsh; sh0 += kC) {
        size_t cell[kC];
        unsigned long long cs[kC];
#pragma unroll
        for (int k = 0; k < kC; ++k) {
            const uint32_t sh = sh0 + k;
            bool ok = sh < P.nsh;
            const ColoShard& S = shs[ok ? sh : 0];
            const int32_t ord = ok ? srow[sh] : -1;
            const int64_t slot = P.kmin + (int64_t)m - S.key0;
            ok = ok && ord >= 0 && slot >= 0 && slot < (int64_t)S.H && (uint32_t)ord < S.T;
            cell[k] = ok ? (size_t)slot * S.T + (uint32_t)ord : 0;
            const unsigned long long x = S.cnt32 ? ((const unsigned int*)S.cnt)[cell[k]] : S.cnt[cell[k]];
            cs[k] = ok ? x : 0ull;  // 0: the shard has no bucket at this key
        }
#pragma unroll
        for (int k = 0; k < kC; ++k) c += cs[k];
        for (int l = 0; l < P.nleaves; ++l) {
            unsigned long long v[kC], a[kC], b[kC];
            double su[kC], q[kC];
#pragma unroll
            for (int k = 0; k < kC; ++k) {
                const ColoShard& S = shs[sh0 + k < P.nsh ? sh0 + k : 0];
                v[k] = S.lcnt[l] ? S.lcnt[l][cell[k]] : cs[k];
                v[k] = cs[k] ? v[k] : 0ull;
                su[k] = S.lsum[l][cell[k]];
                a[k] = S.lmn[l] ? S.lmn[l][cell[k]] : kMinInit;
                b[k] = S.lmx[l] ? S.lmx[l][cell[k]] : kMaxInit;
                q[k] = S.lsq[l] ? S.lsq[l][cell[k]] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < kC; ++k) {
                if (!cs[k]) continue;
                vc[l] += v[k];
                sum[l] += v[k] ? su[k] : 0.0;  // an empty shard stats adds its 0.0 sum
                if (v[k]) {
                    mn[l] = min(mn[l], a[k]);  // order-preserving encodings: Java Math.min / max
                    mx[l] = max(mx[l], b[k]);
                    sq[l] += q[k];
                }
            }
        }
    }
    const size_t at = (size_t)r * P.Hm + m, stride = (size_t)P.R * P.Hm;
    P.o_cnt[at] = c;
    for (int l = 0; l < P.nleaves; ++l) {
        double dmn = __builtin_inf(), dmx = -__builtin_inf();
        if (vc[l]) {
            if (mn[l] < kEncNegInf || mx[l] > kEncPosInf) { dmn = __builtin_nan(""); dmx = __builtin_nan(""); }
            else { dmn = unsortable(mn[l]); dmx = unsortable(mx[l]); }
        }
        P.o_lcnt[l * stride + at] = vc[l];
        P.o_sum[l * stride + at] = sum[l];
        P.o_min[l * stride + at] = dmn;
        P.o_max[l * stride + at] = dmx;
        P.o_sq[l * stride + at] = sq[l];
    }
}
__global__ __launch_bounds__(256) void colo_totals_kernel(const ColoTotals* __restrict__ d, uint32_t Tmax,
                                                          unsigned long long* __restrict__ out) {
    __shared__ ColoTotals c;  // the descriptor from pinned host memory, once per workgroup
    if (threadIdx.x < sizeof(ColoTotals) / 8)
        ((unsigned long long*)&c)[threadIdx.x] = ((const unsigned long long*)(d + blockIdx.y))[threadIdx.x];
    __syncthreads();
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= c.T) return;
    unsigned long long s = 0;
    if (c.cnt32)
        for (uint32_t h = 0; h < c.H; ++h) s += ((const unsigned int*)c.cnt)[(size_t)h * c.T + t];
    else
        for (uint32_t h = 0; h < c.H; ++h) s += ((const unsigned long long*)c.cnt)[(size_t)h * c.T + t];
    out[(size_t)blockIdx.y * Tmax + t] = s;
}
void launch_colo_totals(const ColoTotals* d, uint32_t n, uint32_t Tmax, unsigned long long* out, hipStream_t st) {
    if (n == 0 || Tmax == 0) return;
    hipLaunchKernelGGL(colo_totals_kernel, dim3((Tmax + 255) / 256, n), dim3(256), 0, st, d, Tmax, out);
}

__device__ __forceinline__ unsigned long long wg_sum_u64(unsigned long long v, unsigned long long* ws) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned long long t = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; ++w) t += ws[w];
    return t;
}

// terms orders (include/esgpu.h ESGPU_ORDER_*): 0 count desc, 1 count asc, 2 term asc, 3 term desc
constexpr int32_t kOrdCountDesc = 0, kOrdCountAsc = 1, kOrdTermDesc = 3;
__global__ __launch_bounds__(1024) void colo_select_kernel(const unsigned long long* __restrict__ tot,
                                                           const ColoTotals* __restrict__ d, uint32_t Tmax, ColoSelect S,
                                                           unsigned long long* __restrict__ out) {
    __shared__ unsigned long long key[kColoSelMax];
    __shared__ unsigned long long ws[16];
    __shared__ uint32_t vcs;
    const uint32_t i = blockIdx.x;
    if (threadIdx.x == 0) vcs = d[i].vc;  // from pinned host memory, once
    __syncthreads();
    const uint32_t V = vcs;
    uint32_t N2 = 2;
    while (N2 < V) N2 <<= 1;
    const unsigned long long* ti = tot + (size_t)i * Tmax;
    // candidates (select_terms: min_doc_count drops empty terms, shard_min_doc_count bounds the candidates) as sort keys,
    // descending = the selection order; bit 63 marks a candidate
    unsigned long long oth = 0, nc = 0;
    for (uint32_t t = threadIdx.x; t < N2; t += blockDim.x) {
        unsigned long long k = 0;
        if (t < V) {
            const unsigned long long c = ti[t];
            if (!(S.min_doc_count > 0 && c == 0)) {
                oth += c;
                if (S.shard_min_doc_count <= (long long)c) {
                    const unsigned long long lo = S.order == kOrdTermDesc ? t : 0xFFFFFFFFull - t;
                    const unsigned long long hi = S.order == kOrdCountDesc ? c
                                                : S.order == kOrdCountAsc ? 0x7FFFFFFFull - c : 0ull;
                    k = (1ull << 63) | (hi << 32) | lo;
                    ++nc;
                }
            }
        }
        key[t] = k;
    }
    oth = wg_sum_u64(oth, ws);
    nc = wg_sum_u64(nc, ws);
    __syncthreads();
    for (uint32_t k = 2; k <= N2; k <<= 1)  // bitonic sort, descending
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < N2; t += blockDim.x) {
                const uint32_t u = t ^ j;
                if (u > t) {
                    const unsigned long long a = key[t], b = key[u];
                    if (((t & k) == 0) ? a < b : a > b) { key[t] = b; key[u] = a; }
                }
            }
            __syncthreads();
        }
    const unsigned long long size = (unsigned long long)min((long long)V, max(S.shard_size, 0ll));
    const unsigned long long np = min(size, nc);
    unsigned long long* o = out + (size_t)i * (2 + S.K);
    unsigned long long picked = 0;
    for (uint32_t j = threadIdx.x; j < np; j += blockDim.x) {
        const unsigned long long k = key[j];
        const uint32_t lo = (uint32_t)k;
        const uint32_t ord = S.order == kOrdTermDesc ? lo : 0xFFFFFFFFu - lo;
        const unsigned long long c = ti[ord];
        picked += c;
        o[2 + j] = (c << 32) | ord;
    }
    picked = wg_sum_u64(picked, ws);
    if (threadIdx.x == 0) {
        o[0] = np;
        o[1] = oth - picked;
    }
}
void launch_colo_select(const unsigned long long* tot, const ColoTotals* d, uint32_t n, uint32_t Tmax, const ColoSelect& S,
                        unsigned long long* out, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(colo_select_kernel, dim3(n), dim3(1024), 0, st, tot, d, Tmax, S, out);
}

// the cross-rank co-located reduce: one local shard's rows of the final terms as [F][Hmax][R] words (F = 1 + 5 leaves),
// which colo_merge_kernel reads as a grid with T = R (the final bucket index as the ordinal); an absent row is zeros
__global__ __launch_bounds__(256) void colo_pack_kernel(ColoPackParams P) {
    __shared__ ColoShard S;  // the descriptor from pinned host memory, once per workgroup
    const uint32_t i = blockIdx.y;
    if (threadIdx.x < sizeof(ColoShard) / 8)
        ((unsigned long long*)&S)[threadIdx.x] = ((const unsigned long long*)(P.shards + i))[threadIdx.x];
    __syncthreads();
    const size_t HR = (size_t)P.Hmax * P.R;
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= HR) return;
    const uint32_t m = (uint32_t)(e / P.R), b = (uint32_t)(e - (size_t)m * P.R);
    const int32_t ord = P.rows[(size_t)b * P.n + i];
    const bool ok = ord >= 0 && m < S.H && (uint32_t)ord < S.T;
    const size_t cell = ok ? (size_t)m * S.T + (uint32_t)ord : 0;
    unsigned long long* o = P.out + (size_t)i * (1 + 5 * (size_t)P.nleaves) * HR + e;
    const unsigned long long c = !ok ? 0ull : S.cnt32 ? ((const unsigned int*)S.cnt)[cell] : S.cnt[cell];
    o[0] = c;
    for (int l = 0; l < P.nleaves; ++l) {
        unsigned long long* f = o + (size_t)(1 + 5 * l) * HR;
        f[0] = !ok ? 0ull : S.lcnt[l] ? S.lcnt[l][cell] : c;
        f[HR] = ok ? dbl_bits(S.lsum[l][cell]) : 0ull;
        if (S.lmn[l]) {
            f[2 * HR] = ok ? S.lmn[l][cell] : kMinInit;
            f[3 * HR] = ok ? S.lmx[l][cell] : kMaxInit;
        }
        if (S.lsq[l]) f[4 * HR] = ok ? dbl_bits(S.lsq[l][cell]) : 0ull;
    }
}
void launch_colo_pack(const ColoPackParams& p, hipStream_t st) {
    const size_t HR = (size_t)p.Hmax * p.R;
    if (HR == 0 || p.n == 0) return;
    hipLaunchKernelGGL(colo_pack_kernel, dim3((uint32_t)((HR + 255) / 256), p.n), dim3(256), 0, st, p);
}

struct GatherBufs {
    const unsigned long long* src[kColoMaxShards];
    unsigned long long* dst;
    uint64_t words;  // per rank
    uint32_t n;
};
__global__ __launch_bounds__(256) void gather_bufs_kernel(GatherBufs G) {
    const uint64_t total = G.words * G.n;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256) {
        const uint32_t r = (uint32_t)(i / G.words);
        G.dst[i] = G.src[r][i - (uint64_t)r * G.words];
    }
}
void launch_gather_bufs(const void* const* srcs, int n, size_t bytes, void* dst, hipStream_t st) {
    if (n <= 0 || bytes == 0) return;
    GatherBufs G{};
    for (int r = 0; r < n && r < kColoMaxShards; ++r) G.src[r] = (const unsigned long long*)srcs[r];
    G.dst = (unsigned long long*)dst;
    G.words = bytes / 8;
    G.n = (uint32_t)std::min(n, kColoMaxShards);
    const uint64_t total = G.words * G.n;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(gather_bufs_kernel, dim3(grid), dim3(256), 0, st, G);
}

// the in-process transport's all-reduce: dst[i] = src[0][i] (op) src[1][i] (op) ... in rank order (dtype: 0 u8, 1 i64,
// 2 u64, 3 f64; op: 0 sum, 1 min, 2 max -- include/esgpu.h ESGPU_DT_* / ESGPU_RED_*)
struct ReduceBufs {
    const void* src[kColoMaxShards];
    void* dst;
    uint64_t count;
    uint32_t n;
    int dt, op;
};
template <class T>
__device__ __forceinline__ T red_op(T a, T b, int op) {
    return op == 0 ? (T)(a + b) : op == 1 ? (b < a ? b : a) : (b > a ? b : a);
}
template <class T>
__device__ void reduce_bufs_t(const ReduceBufs& R) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < R.count; i += (uint64_t)gridDim.x * 256) {
        T a = ((const T*)R.src[0])[i];
        for (uint32_t r = 1; r < R.n; ++r) a = red_op(a, ((const T*)R.src[r])[i], R.op);
        ((T*)R.dst)[i] = a;
    }
}
__global__ __launch_bounds__(256) void reduce_bufs_kernel(ReduceBufs R) {
    switch (R.dt) {
        case 0: reduce_bufs_t<uint8_t>(R); break;
        case 1: reduce_bufs_t<long long>(R); break;
        case 2: reduce_bufs_t<unsigned long long>(R); break;
        default: reduce_bufs_t<double>(R); break;
    }
}
void launch_reduce_bufs(const void* const* srcs, int n, uint64_t count, int dt, int op, void* dst, hipStream_t st) {
    if (n <= 0 || count == 0) return;
    ReduceBufs R{};
    for (int r = 0; r < n && r < kColoMaxShards; ++r) R.src[r] = srcs[r];
    R.dst = dst;
    R.count = count;
    R.n = (uint32_t)std::min(n, kColoMaxShards);
    R.dt = dt;
    R.op = op;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((count + 255) / 256, 2048);
    hipLaunchKernelGGL(reduce_bufs_kernel, dim3(grid), dim3(256), 0, st, R);
}

// ---- the reduce across ranks of a top-level cardinality (esgpu_comm_build_reduce) --------------------------------
// this rank's local shard plans' u32 registers maxed into one u8 array (HyperLogLogPlusPlus.merge's register max,
// HyperLogLogPlusPlus.java:223-228) followed by the 64-byte tail the all-reduce (max) carries: [0] some local shard
// collected a value, [1] some local shard is in HYPERLOGLOG (post_collection's decision from its counters), bytes 8-15 /
// 16-23 the request's shape hash and its complement (after a max over the ranks, equal hashes read back as h and ~h);
// and every local plan's two counters copied to pinned memory (lc_out[2 * i ...]).
__global__ __launch_bounds__(256) void xr_card_pack_kernel(XrCardPack K) {
    const uint32_t m = K.m;
    if (blockIdx.x == 0 && threadIdx.x < 2 * K.n) {
        const uint32_t s = threadIdx.x / 2;
        K.lc_out[threadIdx.x] = K.cnt[s] ? K.cnt[s][threadIdx.x % 2] : 0u;
    }
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < m + kXrCardTail; i += gridDim.x * 256) {
        if (i < m) {
            uint32_t v = 0;
            for (uint32_t s = 0; s < K.n; ++s)
                if (K.regs[s]) v = max(v, K.regs[s][i]);
            K.out[i] = (uint8_t)v;
        } else {
            const uint32_t t = i - m;
            uint8_t b = 0;
            if (t == 0 || t == 1) {
                for (uint32_t s = 0; s < K.n; ++s) {
                    if (!K.cnt[s]) continue;
                    const uint32_t c0 = K.cnt[s][0], c1 = K.cnt[s][1];
                    if (t == 0 && (c0 > 0 || c1 > 0)) b = 1;
                    if (t == 1 && !(c1 <= K.thr && c0 <= K.thr)) b = 1;
                }
            } else if (t >= 8 && t < 16) {
                b = (uint8_t)(K.hash >> (8 * (t - 8)));
            } else if (t >= 16 && t < 24) {
                b = (uint8_t)(~K.hash >> (8 * (t - 16)));
            }
            K.out[i] = b;
        }
    }
}
void launch_xr_card_pack(const XrCardPack& K, hipStream_t st) {
    const uint32_t total = K.m + kXrCardTail;
    hipLaunchKernelGGL(xr_card_pack_kernel, dim3(std::min<uint32_t>(1024, (total + 255) / 256)), dim3(256), 0, st, K);
}
// the all-reduced registers + tail into pinned memory, and the non-zero registers counted into nz (zeroed before)
__global__ __launch_bounds__(256) void xr_card_finish_kernel(const uint8_t* regs, uint32_t m, unsigned long long* dst,
                                                              uint32_t* nz) {
    const uint32_t words = (m + kXrCardTail) / 8;
    uint32_t c = 0;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < words; i += gridDim.x * 256) {
        const unsigned long long w = reinterpret_cast<const unsigned long long*>(regs)[i];
        dst[i] = w;
        if (i < m / 8)
#pragma unroll
            for (int k = 0; k < 8; ++k) c += ((w >> (8 * k)) & 0xFF) != 0;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(nz, c);
}
void launch_xr_card_finish(const uint8_t* regs, uint32_t m, unsigned long long* dst, uint32_t* nz, hipStream_t st) {
    const uint32_t words = (m + kXrCardTail) / 8;
    hipLaunchKernelGGL(xr_card_finish_kernel, dim3(std::min<uint32_t>(256, (words + 255) / 256)), dim3(256), 0, st, regs, m,
                       dst, nz);
}

// ---- the reduce across ranks of a plain terms aggregation (config 3) ----------------------------------------------
// a shard's GPU top-k output (K3: k keys, count << 32 | ~ordinal for count-descending order, then the sum of every
// ordinal's count) turned into the selection record the other ranks all-gather: {picks, other-doc count,
// count << 32 | ordinal ...} -- what build_terms_root makes of the same keys on the host (picks end at the first zero
// key; other = the sum minus the picks' counts)
__global__ void xr_terms_record_kernel(const unsigned long long* keys, uint32_t kk, uint32_t k_req, int order,
                                       unsigned long long* rec, uint32_t K) {
    if (threadIdx.x != 0) return;
    unsigned long long picks = 0, taken = 0;
    for (uint32_t i = 0; i < k_req && i < K; ++i) {
        const unsigned long long key = keys[i];
        if (key == 0) break;
        const uint32_t lo = (uint32_t)key;
        const uint32_t ord = order == 3 /* ESGPU_ORDER_TERM_DESC */ ? lo : 0xFFFFFFFFu - lo;
        const unsigned long long hi = (key >> 32) & 0x7FFFFFFFull;
        const unsigned long long cnt = order == 1 /* ESGPU_ORDER_COUNT_ASC */ ? 0x7FFFFFFFull - hi : hi;
        rec[2 + picks] = (cnt << 32) | ord;
        taken += cnt;
        ++picks;
    }
    for (uint32_t i = (uint32_t)picks; i < K; ++i) rec[2 + i] = 0;
    rec[0] = picks;
    rec[1] = keys[kk] - taken;
}
void launch_xr_terms_record(const unsigned long long* keys, uint32_t kk, uint32_t k_req, int order, unsigned long long* rec,
                            uint32_t K, hipStream_t st) {
    hipLaunchKernelGGL(xr_terms_record_kernel, dim3(1), dim3(64), 0, st, keys, kk, k_req, order, rec, K);
}

void launch_colo_merge(const ColoParams& p, hipStream_t st) {
    if (p.R == 0 || p.Hm == 0) return;
    hipLaunchKernelGGL(colo_merge_kernel, dim3((p.Hm + 255) / 256, p.R), dim3(256), 0, st, p);
}

// device -> pinned host memory for the build's small transfers: a kernel writing over the link beats a DMA copy,
// whose setup measured ~130 us per 144 KB transfer
__global__ __launch_bounds__(256) void copy_u64_kernel(const unsigned long long* __restrict__ src,
                                                       unsigned long long* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

void launch_copy_u64(const unsigned long long* src, unsigned long long* dst, size_t n, hipStream_t st) {
    if (n == 0) return;
    const size_t g = std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(copy_u64_kernel, dim3((uint32_t)g), dim3(256), 0, st, src, dst, n);
}

void launch_gather_rows(const GatherParams& p, hipStream_t st) {
    const uint32_t n = p.k * p.H;
    if (n == 0) return;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, st, p);
}

template <class D>
__global__ __launch_bounds__(256) void expand_delta_kernel(const D* __restrict__ d, uint32_t n, int64_t base,
                                                           int64_t* __restrict__ out) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        out[i] = (int64_t)((uint64_t)base + (uint64_t)d[i]);
}
void launch_expand_d32(const uint32_t* d, uint32_t n, int64_t base, int64_t* out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(expand_delta_kernel<uint32_t>, dim3(std::min<uint32_t>((n + 255) / 256, 8192)), dim3(256), 0, s,
                              d, n, base, out);
}
void launch_expand_d16(const uint16_t* d, uint32_t n, int64_t base, int64_t* out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(expand_delta_kernel<uint16_t>, dim3(std::min<uint32_t>((n + 255) / 256, 8192)), dim3(256), 0, s,
                              d, n, base, out);
}

// one workgroup per run of kB16Docs docs: the run's minimum over its live docs, and every doc's delta over it
__global__ __launch_bounds__(256) void block_delta16_kernel(const int64_t* __restrict__ v, uint32_t n_docs, uint16_t* __restrict__ d,
                                                            uint8_t* __restrict__ hi, int64_t* __restrict__ base,
                                                            unsigned int* __restrict__ bad) {
    __shared__ long long smn[4], smx[4];
    const uint32_t c0 = blockIdx.x << kB16Shift;
    long long mn = 0x7FFFFFFFFFFFFFFFll, mx = -0x7FFFFFFFFFFFFFFFll - 1;
    for (uint32_t i = c0 + threadIdx.x; i < c0 + kB16Docs; i += 256)
        if (i < n_docs) {
            const long long x = v[i];
            mn = min(mn, x);
            mx = max(mx, x);
        }
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, __shfl_xor(mn, o));
        mx = max(mx, __shfl_xor(mx, o));
    }
    if ((threadIdx.x & 63) == 0) { smn[threadIdx.x >> 6] = mn; smx[threadIdx.x >> 6] = mx; }
    __syncthreads();
    mn = min(min(smn[0], smn[1]), min(smn[2], smn[3]));
    mx = max(max(smx[0], smx[1]), max(smx[2], smx[3]));
    const bool any = c0 < n_docs;
    if (threadIdx.x == 0) {
        base[blockIdx.x] = any ? mn : 0;
        const unsigned long long span = (unsigned long long)mx - (unsigned long long)mn;
        if (any && span >= 65536ull) atomicOr(bad, span >= (1ull << 24) ? 3u : 1u);
    }
    for (uint32_t i = c0 + threadIdx.x; i < c0 + kB16Docs; i += 256) {
        const uint32_t x = i < n_docs ? (uint32_t)((unsigned long long)v[i] - (unsigned long long)mn) : 0u;
        d[i] = (uint16_t)x;
        if (hi) hi[i] = (uint8_t)(x >> 16);
    }
}
void launch_block_delta16(const int64_t* v, uint32_t n_docs, uint32_t n_pad, uint16_t* d, uint8_t* hi, int64_t* base,
                          unsigned int* bad, hipStream_t st) {
    const uint32_t runs = n_pad >> kB16Shift;
    if (runs) hipLaunchKernelGGL(block_delta16_kernel, dim3(runs), dim3(256), 0, st, v, n_docs, d, hi, base, bad);
}
__global__ __launch_bounds__(256) void expand_b16_kernel(const uint16_t* __restrict__ d, const uint8_t* __restrict__ hi,
                                                         const int64_t* __restrict__ base, uint32_t n_docs, uint32_t n,
                                                         int64_t* __restrict__ out) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint64_t x = (uint64_t)d[i] | (hi ? (uint64_t)hi[i] << 16 : 0ull);
        out[i] = i < n_docs ? (int64_t)((uint64_t)base[i >> kB16Shift] + x) : 0;  // the upload pads with 0
    }
}
void launch_expand_b16(const uint16_t* d, const uint8_t* hi, const int64_t* base, uint32_t n_docs, uint32_t n_pad, int64_t* out,
                       hipStream_t st) {
    if (n_pad) hipLaunchKernelGGL(expand_b16_kernel, dim3(std::min<uint32_t>((n_pad + 255) / 256, 8192)), dim3(256), 0, st,
                                  d, hi, base, n_docs, n_pad, out);
}

__global__ __launch_bounds__(256) void dd_fold_kernel(double* __restrict__ hi, double* __restrict__ lo, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const double l = lo[i];
        if (l != 0.0) {
            const double h = hi[i];
            if (__builtin_isfinite(h)) hi[i] = h + l;  // a non-finite sum keeps its Inf / NaN
            lo[i] = 0.0;
        }
    }
}
void launch_dd_fold(double* hi, double* lo, size_t n, hipStream_t s) {
    if (!n) return;
    const uint32_t grid = (uint32_t)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(dd_fold_kernel, dim3(grid), dim3(256), 0, s, hi, lo, n);
}

__global__ void fill_u64_kernel(unsigned long long* p, size_t n, unsigned long long v) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void widen_u32_kernel(const unsigned int* src, size_t n, unsigned long long* dst) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}
void launch_widen_u32(const unsigned int* src, size_t n, unsigned long long* dst, hipStream_t st) {
    if (n) hipLaunchKernelGGL(widen_u32_kernel, dim3((uint32_t)std::min<size_t>(4096, (n + 255) / 256)), dim3(256), 0, st, src, n, dst);
}
__global__ void narrow_u64_kernel(const unsigned long long* src, size_t n, unsigned int* dst) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = (unsigned int)src[i];
}
void launch_narrow_u64(const unsigned long long* src, size_t n, unsigned int* dst, hipStream_t st) {
    if (n) hipLaunchKernelGGL(narrow_u64_kernel, dim3((uint32_t)std::min<size_t>(4096, (n + 255) / 256)), dim3(256), 0, st, src, n, dst);
}
// global ordinals: out[d] = map[in[d]] (ordinals outside the segment dictionary, incl. missing, stay missing)
__global__ void remap_ords_kernel(const uint32_t* in, uint32_t n, const uint32_t* map, uint32_t map_n, uint32_t* out) {
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += gridDim.x * blockDim.x * 4) {
        uint32_t o[4];
        load_u32x4(in, i, o);  // n is a multiple of kBlockDocs
        uint4 r;
        r.x = o[0] < map_n ? map[o[0]] : kMissingOrd;
        r.y = o[1] < map_n ? map[o[1]] : kMissingOrd;
        r.z = o[2] < map_n ? map[o[2]] : kMissingOrd;
        r.w = o[3] < map_n ? map[o[3]] : kMissingOrd;
        *reinterpret_cast<uint4*>(out + i) = r;
    }
}
void launch_remap_ords(const uint32_t* in, uint32_t n, const uint32_t* map, uint32_t map_n, uint32_t* out, hipStream_t st) {
    if (n == 0) return;
    const uint32_t grid = std::min<uint32_t>(4096, (n / 4 + 255) / 256);
    hipLaunchKernelGGL(remap_ords_kernel, dim3(grid), dim3(256), 0, st, in, n, map, map_n, out);
}

// compact columns: ordinals in 16 bits (kMissingOrd -> 0xFFFF; only for dictionaries under 65,535 terms) and long
// values as 32-bit deltas over the column's minimum (a missing value's delta is never read: the present bits decide)
__global__ void pack_ord16_kernel(const uint32_t* src, uint32_t n, uint16_t* out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t o = src[i];
        out[i] = o == kMissingOrd ? (uint16_t)0xFFFFu : (uint16_t)o;
    }
}
void launch_pack_ord16(const uint32_t* src, uint32_t n, uint16_t* out, hipStream_t st) {
    if (n) hipLaunchKernelGGL(pack_ord16_kernel, dim3(std::min<uint32_t>(8192, (n + 255) / 256)), dim3(256), 0, st, src, n, out);
}
__global__ void delta32_kernel(const int64_t* v, uint32_t n, int64_t base, uint32_t* out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[i] = (uint32_t)((uint64_t)v[i] - (uint64_t)base);
}
void launch_delta32(const int64_t* v, uint32_t n, int64_t base, uint32_t* out, hipStream_t st) {
    if (n) hipLaunchKernelGGL(delta32_kernel, dim3(std::min<uint32_t>(8192, (n + 255) / 256)), dim3(256), 0, st, v, n, base, out);
}

__global__ void delta16_kernel(const int64_t* v, uint32_t n, int64_t base, uint16_t* out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[i] = (uint16_t)((uint64_t)v[i] - (uint64_t)base);
}
void launch_delta16(const int64_t* v, uint32_t n, int64_t base, uint16_t* out, hipStream_t st) {
    if (n) hipLaunchKernelGGL(delta16_kernel, dim3(std::min<uint32_t>(8192, (n + 255) / 256)), dim3(256), 0, st, v, n, base, out);
}

__global__ void pack_u8_kernel(const unsigned int* src, uint32_t n, uint8_t* dst) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = (uint8_t)src[i];
}
void launch_pack_u8(const unsigned int* src, uint32_t n, uint8_t* dst, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(pack_u8_kernel, dim3(std::min<uint32_t>(1024, (n + 255) / 256)), dim3(256), 0, st, src, n, dst);
}

__global__ __launch_bounds__(256) void fill_multi_kernel(FillList L) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    for (int k = 0; k < L.count; ++k) {
        unsigned long long* p = L.p[k];
        const unsigned long long v = L.v[k];
        const size_t n = L.n[k];
        if (((uintptr_t)p & 15) == 0) {  // 16-byte stores (the grid arrays are 256-byte aligned), then the odd tail word
            const uint4 w = make_uint4((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)v, (uint32_t)(v >> 32));
            for (size_t i = g; i < n / 2; i += stride) reinterpret_cast<uint4*>(p)[i] = w;
            if (g == 0 && (n & 1)) p[n - 1] = v;
        } else {
            for (size_t i = g; i < n; i += stride) p[i] = v;
        }
    }
}
void launch_fill_multi(const FillList& l, hipStream_t st) {
    uint64_t total = 0;
    for (int k = 0; k < l.count; ++k) total += l.n[k];
    if (total == 0) return;
    // a few workgroups per CU looping over the spans (one thread per pair of words, per span, had spent more on
    // dispatching ~2,800 workgroups than on the stores: 13 us for the north star's 29 MB)
    size_t grid = (total / (uint64_t)l.count / 2 + 255) / 256;
    if (grid > 1024) grid = 1024;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(fill_multi_kernel, dim3((uint32_t)grid), dim3(256), 0, st, l);
}

__global__ __launch_bounds__(256) void copy_multi_kernel(CopyList L) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    for (int k = 0; k < L.count; ++k) {
        const unsigned long long* __restrict__ s = L.src[k];
        unsigned long long* __restrict__ d = L.dst[k];
        for (size_t i = g; i < L.n[k]; i += stride) d[i] = s[i];
    }
}
void launch_copy_multi(const CopyList& l, hipStream_t st) {
    uint64_t mx = 0;
    for (int k = 0; k < l.count; ++k) mx = l.n[k] > mx ? l.n[k] : mx;
    if (mx == 0) return;
    size_t grid = (mx + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(copy_multi_kernel, dim3((uint32_t)grid), dim3(256), 0, st, l);
}

void launch_fill_u64(unsigned long long* p, size_t n, unsigned long long v, hipStream_t st) {
    if (n == 0) return;
    size_t grid = (n + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(fill_u64_kernel, dim3((uint32_t)grid), dim3(256), 0, st, p, n, v);
}

}  // namespace esgpu

// ------------------------------------------------------------------------------------------------------------
// K1 for high-cardinality terms (valueCount >> LDS): radix-partitioned counting.
//   pass 1  part_hist     per-workgroup histogram of partitions (ord >> shift) in LDS
//   pass 2  part_scan     exclusive scan of the [P][G] histogram -> per-(partition, workgroup) write cursors
//   pass 3  part_scatter  each workgroup re-reads its docs and appends ordinals to its slice of every partition
//   pass 4  part_count    one workgroup per (partition, <= chunk elements): LDS counters for the 2^shift ordinals of
//                         the partition, flushed once -> no global atomic contention on hot (Zipf head) terms
// ------------------------------------------------------------------------------------------------------------
namespace esgpu {

// pass 1: per-workgroup partition histogram
__global__ __launch_bounds__(kWG) void part_hist_kernel(PartParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* lds = (uint32_t*)smem;  // [P]
    const uint32_t g = blockIdx.x;
    for (uint32_t p = threadIdx.x; p < P.P; p += kWG) lds[p] = 0u;
    __syncthreads();
    const uint32_t b_begin = g * P.blocks_per_wg;
    const uint32_t b_end = min(b_begin + P.blocks_per_wg, P.n_blocks);
    for (uint32_t b = b_begin; b < b_end; ++b) {
        uint32_t o[kItersPerBlock][4], ok[kItersPerBlock];
#pragma unroll
        for (int it = 0; it < kItersPerBlock; ++it) {  // all 16 loads in flight before the first atomic
            const uint32_t doc0 = b * kBlockDocs + it * kIterDocs + threadIdx.x * kVec;
            load_u32x4(P.ord, doc0, o[it]);
            ok[it] = 0xF;
            if (doc0 + 4 > P.n_docs) ok[it] = doc0 >= P.n_docs ? 0u : ((1u << (P.n_docs - doc0)) - 1u);
            if (P.accept) ok[it] &= bits4(P.accept, doc0);
            for (int k = 0; k < P.npred; ++k) ok[it] &= eval_pred(P.pred[k], doc0);
        }
#pragma unroll
        for (int it = 0; it < kItersPerBlock; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (((ok[it] >> j) & 1) && o[it][j] < P.T) atomicAdd(&lds[o[it][j] >> P.shift], 1u);
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < P.P; p += kWG) P.wg_counts[(size_t)p * P.G + g] = lds[p];
}

// exclusive scan of v[0, n) in LDS by one workgroup (n <= kPartMaxStaged); returns the total
__device__ uint32_t block_exclusive_scan(uint32_t* v, uint32_t n, uint32_t* wave_tot) {
    const uint32_t per = (n + kWG - 1) / kWG;
    const uint32_t b = threadIdx.x * per, e = min(b + per, n);
    uint32_t local = 0;
    for (uint32_t i = b; i < e; ++i) local += v[i];
    // inclusive scan of `local` across the wave (wave64), then across the 8 waves
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = local;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wave_tot[wave] = x;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kWG / 64; ++w) {
        const uint32_t t = wave_tot[w];
        if (w < wave) before += t;
        total += t;
    }
    uint32_t run = before + x - local;
    for (uint32_t i = b; i < e; ++i) {
        const uint32_t c = v[i];
        v[i] = run;
        run += c;
    }
    return total;
}

// pass 3: scatter through an LDS-staged tile.  Every tile (kScatterTB 8192-doc blocks) is counting-sorted by
// partition in LDS first, so the global writes are runs of consecutive 16-bit partition-local offsets instead of
// scattered words; the larger the tile, the longer the runs and the fewer partially written lines leave L2.
#ifndef ESGPU_SCATTER_TB
#define ESGPU_SCATTER_TB 4
#endif
constexpr int kScatterTB = ESGPU_SCATTER_TB;
constexpr uint32_t kScatterTile = kScatterTB * kBlockDocs;

__global__ __launch_bounds__(kWG) void part_scatter_kernel(PartParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* cursor = (uint32_t*)smem;      // [P] next write position of (partition, this workgroup)
    uint32_t* tcnt = cursor + P.P;           // [P] elements of the tile per partition
    uint32_t* toff = tcnt + P.P;             // [P] their exclusive offsets inside the tile
    uint32_t* stage = toff + P.P;            // [kScatterTile] the tile, sorted by partition
    __shared__ uint32_t wave_tot[kWG / 64];
    const uint32_t g = blockIdx.x;
    const uint32_t mask = (1u << P.shift) - 1u;
    constexpr int kIt = kScatterTB * kItersPerBlock;
    for (uint32_t p = threadIdx.x; p < P.P; p += kWG) {
        cursor[p] = P.wg_counts[(size_t)p * P.G + g];
        tcnt[p] = 0u;
    }
    __syncthreads();
    const uint32_t b_begin = g * P.blocks_per_wg;
    const uint32_t b_end = min(b_begin + P.blocks_per_wg, P.n_blocks);
    for (uint32_t b = b_begin; b < b_end; b += kScatterTB) {
        uint32_t o[kIt][4], ok[kIt], rank[kIt][4];
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const uint32_t blk = b + it / kItersPerBlock;
            const uint32_t doc0 = blk * kBlockDocs + (it % kItersPerBlock) * kIterDocs + threadIdx.x * kVec;
            ok[it] = 0u;
            o[it][0] = o[it][1] = o[it][2] = o[it][3] = 0u;
            if (blk < b_end) {
                load_u32x4(P.ord, doc0, o[it]);
                ok[it] = 0xF;
                if (doc0 + 4 > P.n_docs) ok[it] = doc0 >= P.n_docs ? 0u : ((1u << (P.n_docs - doc0)) - 1u);
                if (P.accept) ok[it] &= bits4(P.accept, doc0);
                for (int k = 0; k < P.npred; ++k) ok[it] &= eval_pred(P.pred[k], doc0);
            }
        }
#pragma unroll
        for (int it = 0; it < kIt; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool v = ((ok[it] >> j) & 1) && o[it][j] < P.T;
                rank[it][j] = v ? atomicAdd(&tcnt[o[it][j] >> P.shift], 1u) : 0xFFFFFFFFu;
            }
        __syncthreads();
        for (uint32_t p = threadIdx.x; p < P.P; p += kWG) toff[p] = tcnt[p];
        __syncthreads();
        const uint32_t n_tile = block_exclusive_scan(toff, P.P, wave_tot);
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kIt; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (rank[it][j] != 0xFFFFFFFFu) stage[toff[o[it][j] >> P.shift] + rank[it][j]] = o[it][j];
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < n_tile; i += kWG) {
            const uint32_t v = stage[i];
            const uint32_t p = v >> P.shift;
            P.pbuf[cursor[p] + (i - toff[p])] = (uint16_t)(v & mask);
        }
        __syncthreads();
        for (uint32_t p = threadIdx.x; p < P.P; p += kWG) {
            cursor[p] += tcnt[p];
            tcnt[p] = 0u;
        }
        __syncthreads();
    }
}

void launch_part_hist(const PartParams& p, hipStream_t s) {
    hipLaunchKernelGGL(part_hist_kernel, dim3(p.G), dim3(kWG), (size_t)p.P * 4, s, p);
}
void launch_part_scatter(const PartParams& p, hipStream_t s) {
    hipLaunchKernelGGL(part_scatter_kernel, dim3(p.G), dim3(kWG), part_scatter_lds_bytes(p.P), s, p);
}
size_t part_scatter_lds_bytes(uint32_t n_parts) { return ((size_t)n_parts * 3 + kScatterTile) * 4; }
uint32_t part_wg_per_cu() {  // the staged tile takes most of the LDS: one scatter workgroup per CU
#ifdef ESGPU_PART_WG_PER_CU
    return ESGPU_PART_WG_PER_CU;
#else
    return 1;
#endif
}

// exclusive scan of wg_counts[P*G] (partition-major) in place; part_begin[p] = offset of (p, g = 0), [P] = total.
// Three launches over 4096-element tiles (tile sums, scan of the tile sums, tile-local scans), all coalesced.
constexpr uint32_t kScanTile = kWG * 8;

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

__global__ __launch_bounds__(kWG) void scan_tile_sums_kernel(const uint32_t* v, uint32_t n, uint32_t* tile_sums) {
    const uint32_t base = blockIdx.x * kScanTile;
    uint32_t local = 0;
    for (uint32_t i = base + threadIdx.x; i < min(n, base + kScanTile); i += kWG) local += v[i];
    local = wave_sum_u32(local);
    __shared__ uint32_t part[kWG / 64];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = local;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kWG / 64; ++w) t += part[w];
        tile_sums[blockIdx.x] = t;
    }
}

// one workgroup: exclusive scan of the tile sums (ntiles <= kScanTile)
__global__ __launch_bounds__(kWG) void scan_tile_offsets_kernel(uint32_t* tile_sums, uint32_t ntiles) {
    __shared__ uint32_t wave_tot[kWG / 64];
    __shared__ uint32_t buf[kScanTile];
    for (uint32_t i = threadIdx.x; i < kScanTile; i += kWG) buf[i] = i < ntiles ? tile_sums[i] : 0u;
    __syncthreads();
    block_exclusive_scan(buf, kScanTile, wave_tot);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < ntiles; i += kWG) tile_sums[i] = buf[i];
}

__global__ __launch_bounds__(kWG) void scan_tiles_kernel(PartParams P, const uint32_t* tile_offsets, uint32_t n) {
    __shared__ uint32_t wave_tot[kWG / 64];
    __shared__ uint32_t buf[kScanTile];
    const uint32_t base = blockIdx.x * kScanTile;
    const uint32_t cnt = min(kScanTile, n - base);
    for (uint32_t i = threadIdx.x; i < kScanTile; i += kWG) buf[i] = i < cnt ? P.wg_counts[base + i] : 0u;
    __syncthreads();
    const uint32_t tile_total = block_exclusive_scan(buf, kScanTile, wave_tot);
    __syncthreads();
    const uint32_t off = tile_offsets[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < cnt; i += kWG) {
        const uint32_t gi = base + i;
        const uint32_t x = off + buf[i];
        P.wg_counts[gi] = x;
        if (gi % P.G == 0) P.part_begin[gi / P.G] = x;
    }
    if (base + cnt == n && threadIdx.x == 0) P.part_begin[P.P] = off + tile_total;
}

void launch_part_scan(const PartParams& p, hipStream_t s) {
    const uint32_t n = p.P * p.G;
    const uint32_t ntiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(scan_tile_sums_kernel, dim3(ntiles), dim3(kWG), 0, s, (const uint32_t*)p.wg_counts, n, p.tile_sums);
    hipLaunchKernelGGL(scan_tile_offsets_kernel, dim3(1), dim3(kWG), 0, s, p.tile_sums, ntiles);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(ntiles), dim3(kWG), 0, s, p, (const uint32_t*)p.tile_sums, n);
}
uint32_t part_scan_tiles(uint32_t n) { return (n + kScanTile - 1) / kScanTile; }

// pass 4: workgroup w counts the partitioned elements [w*chunk, (w+1)*chunk) — hot partitions are thereby split
// across many workgroups, and no host round trip is needed.  Each partition piece is counted in 2^shift LDS
// counters; a thread merges runs of equal offsets in registers first (the Zipf head term dominates its partition).
__device__ __forceinline__ void count_run(uint32_t* cnt, uint32_t& cur, uint32_t& n, uint32_t v) {
    if (v == cur) { ++n; return; }
    if (n) atomicAdd(&cnt[cur], n);
    cur = v;
    n = 1;
}

#ifndef ESGPU_COUNT_WG
#define ESGPU_COUNT_WG 512
#endif
constexpr int kCountWG = ESGPU_COUNT_WG;  // one counting workgroup per CU at 128 KB of LDS counters

__global__ __launch_bounds__(kCountWG) void part_count_kernel(PartParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* cnt = (uint32_t*)smem;
    const uint32_t S = 1u << P.shift;
    const uint32_t total = P.part_begin[P.P];
    const uint64_t e0l = (uint64_t)blockIdx.x * P.chunk;
    if (e0l >= total) return;
    const uint32_t e0 = (uint32_t)e0l, e1 = (uint32_t)min<uint64_t>(e0l + P.chunk, total);
    // first partition with part_begin[q + 1] > e0
    uint32_t lo = 0, hi = P.P - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (P.part_begin[mid + 1] <= e0) lo = mid + 1;
        else hi = mid;
    }
    for (uint32_t q = lo; q < P.P; ++q) {
        const uint32_t qb = P.part_begin[q], qe = P.part_begin[q + 1];
        if (qb >= e1) break;
        const uint32_t s0 = max(e0, qb), s1 = min(e1, qe);
        if (s0 >= s1) continue;
        for (uint32_t i = threadIdx.x; i < S; i += kCountWG) cnt[i] = 0;
        __syncthreads();
        uint32_t cur = 0, n = 0;
        uint32_t i0 = s0;
        const uint32_t a0 = min(s1, (s0 + 7u) & ~7u);  // head up to a 16-byte boundary
        for (uint32_t i = i0 + threadIdx.x; i < a0; i += kCountWG) count_run(cnt, cur, n, P.pbuf[i]);
        const uint32_t nvec = (s1 - a0) / 8;
        const uint4* v8 = reinterpret_cast<const uint4*>(P.pbuf + a0);
        // two buffers of 2 x 16 bytes (16 offsets), each reloaded right after it is counted; loads are unconditional
        // (clamped to the last vector, counted only when in range) so the compiler waits with counted vmcnt
        if (nvec > 0) {
            auto ld = [&](uint32_t k, uint4 v[2]) {
                v[0] = v8[min(k, nvec - 1)];
                v[1] = v8[min(k + kCountWG, nvec - 1)];
            };
            auto count8 = [&](uint32_t k, const uint4 v[2]) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (k + h * kCountWG >= nvec) break;
                    const uint32_t w[4] = {v[h].x, v[h].y, v[h].z, v[h].w};
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        count_run(cnt, cur, n, w[t] & 0xFFFFu);
                        count_run(cnt, cur, n, w[t] >> 16);
                    }
                }
            };
            uint4 va[2], vb[2];
            ld(threadIdx.x, va);
            ld(threadIdx.x + 2 * kCountWG, vb);
            for (uint32_t k = threadIdx.x; k < nvec; k += 4 * kCountWG) {
                count8(k, va);
                ld(k + 4 * kCountWG, va);
                count8(k + 2 * kCountWG, vb);
                ld(k + 6 * kCountWG, vb);
            }
        }
        for (uint32_t i = a0 + nvec * 8 + threadIdx.x; i < s1; i += kCountWG) count_run(cnt, cur, n, P.pbuf[i]);
        if (n) atomicAdd(&cnt[cur], n);
        __syncthreads();
        const bool whole = s0 == qb && s1 == qe;  // the only writer of this partition in this launch
        const uint32_t base = q << P.shift;
        for (uint32_t j = threadIdx.x; j < S; j += kCountWG) {
            const uint32_t c = cnt[j];
            if (c == 0 || base + j >= P.T) continue;
            if (whole) P.counts[base + j] += c;
            else atomicAdd(&P.counts[base + j], c);
        }
        __syncthreads();
    }
}

void launch_part_count(const PartParams& p, hipStream_t s) {
    const uint32_t grid = (uint32_t)(((uint64_t)p.n_docs + p.chunk - 1) / p.chunk);
    if (grid == 0) return;
    hipLaunchKernelGGL(part_count_kernel, dim3(grid), dim3(kCountWG), (size_t)4 << p.shift, s, p);
}

// ------------------------------------------------------------------------------------------------------------
// K3: top shard_size of a count vector on the GPU (replaces BucketPriorityQueue over valueCount ordinals).
// A candidate's key orders exactly like InternalOrder's comparator with the _term asc tie-break (larger = better);
// key 0 = no candidate.  Pass 1: each workgroup keeps its best k keys (bitonic sort of 4096-key chunks in LDS +
// bitonic merge with the running best); pass 2: one workgroup merges the candidates.
// ------------------------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ unsigned long long make_topk_key(int order, unsigned long long count, uint32_t ord) {
    const unsigned long long flag = 1ull << 63;
    switch (order) {
        case 0: return flag | (count << 32) | (0xFFFFFFFFull - ord);                  // _count desc, _term asc
        case 1: return flag | ((0x7FFFFFFFull - count) << 32) | (0xFFFFFFFFull - ord);  // _count asc, _term asc
        case 2: return flag | (0xFFFFFFFFull - ord);                                  // _term asc
        default: return flag | (unsigned long long)ord;                                // _term desc
    }
}
uint64_t topk_key(int order, uint64_t count, uint32_t ord) { return make_topk_key(order, count, ord); }

constexpr int kTopkChunk = 4096;

// one atomic per workgroup (1024 threads): a per-wave atomic on one word serialises ~8k arrivals (~12 ns each)
__device__ __forceinline__ void block_add_u64(unsigned long long* out, unsigned long long v) {
    __shared__ unsigned long long part[16];
    v = wave_sum_u64(v);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; ++w) t += part[w];
        if (t) atomicAdd(out, t);
    }
}

// sort s[0..n) descending, n a power of two, 1024 threads
__device__ void bitonic_sort_desc(unsigned long long* s, uint32_t n) {
    for (uint32_t size = 2; size <= n; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (uint32_t t = threadIdx.x; t < n / 2; t += 1024) {
                const uint32_t i = 2 * t - (t & (stride - 1));
                const uint32_t j = i + stride;
                const bool desc = (i & size) == 0;
                const unsigned long long a = s[i], b = s[j];
                if ((a < b) == desc) { s[i] = b; s[j] = a; }
            }
        }
    }
    __syncthreads();
}
// s[0..n) holds a bitonic sequence; merge it into descending order
__device__ void bitonic_merge_desc(unsigned long long* s, uint32_t n) {
    for (uint32_t stride = n >> 1; stride > 0; stride >>= 1) {
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < n / 2; t += 1024) {
            const uint32_t i = 2 * t - (t & (stride - 1));
            const uint32_t j = i + stride;
            const unsigned long long a = s[i], b = s[j];
            if (a < b) { s[i] = b; s[j] = a; }
        }
    }
    __syncthreads();
}

template <bool FROM_COUNTS>
__global__ __launch_bounds__(1024) void topk_kernel(TopkParams P, const unsigned long long* src, uint32_t n, uint32_t per_wg,
                                                    unsigned long long* out) {
    __shared__ unsigned long long chunk[kTopkChunk];
    __shared__ unsigned long long best[2 * kTopkMax];
    uint32_t kp = 1;
    while (kp < P.k) kp <<= 1;
    for (uint32_t i = threadIdx.x; i < kp; i += 1024) best[i] = 0;
    const uint32_t b = blockIdx.x * per_wg, e = min(b + per_wg, n);
    unsigned long long sum = 0;
    for (uint32_t c0 = b; c0 < e; c0 += kTopkChunk) {
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < kTopkChunk; t += 1024) {
            const uint32_t i = c0 + t;
            unsigned long long key = 0;
            if (i < e) {
                if (FROM_COUNTS) {
                    const unsigned long long c = P.counts32 ? (unsigned long long)P.counts32[i] : src[i];
                    sum += c;
                    const bool eligible = !(P.min_doc_count > 0 && c == 0) && (long long)c >= P.shard_min_doc_count;
                    key = eligible ? make_topk_key(P.order, c, i) : 0ull;
                } else {
                    key = src[i];
                }
            }
            chunk[t] = key;
        }
        bitonic_sort_desc(chunk, kTopkChunk);
        // best (desc) ++ reverse(chunk[0..kp)) is bitonic; merge and keep the top kp
        for (uint32_t t = threadIdx.x; t < kp; t += 1024) best[kp + t] = chunk[kp - 1 - t];
        bitonic_merge_desc(best, 2 * kp);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < P.k; i += 1024) out[(size_t)blockIdx.x * P.k + i] = best[i];
    if (FROM_COUNTS) {
        block_add_u64(P.out_sum, sum);
    }
}

// Count-ordered top-k by selection instead of sorting every ordinal (10M counts -> two streaming passes):
//   topk_hist      log-scale histogram of the eligible counts (32 sub-bins per power of two, 2048 bins, monotone in
//                  the key) + the sum of all counts
//   topk_thresh    one workgroup: the highest bin b* such that bins >= b* hold at least k candidates
//   topk_compact   every eligible ordinal whose bin >= b* -> candidate keys (wave-aggregated append)
//   topk_final     one workgroup: chunked bitonic top-k over the candidates (usually a few hundred)
constexpr uint32_t kTopkBins = 2048;

__device__ __forceinline__ uint32_t count_bin(int order, unsigned long long c) {
    uint32_t b;
    if (c < 32) {
        b = (uint32_t)c;
    } else {
        const uint32_t e = 63u - (uint32_t)__clzll((long long)c);  // >= 5
        b = (e - 4) * 32 + (uint32_t)((c >> (e - 5)) & 31u);       // 32 sub-bins per octave, >= 32
    }
    b = min(b, kTopkBins - 1);
    return order == 0 ? b : kTopkBins - 1 - b;  // COUNT_ASC: fewer docs = better
}

__device__ __forceinline__ bool topk_eligible(const TopkParams& P, unsigned long long c) {
    return !(P.min_doc_count > 0 && c == 0) && (long long)c >= P.shard_min_doc_count;
}

// 4 consecutive counts per thread per step (two 16-byte loads): a single 8-byte load per thread left the pass
// latency-bound at ~0.7 TB/s over the 10M-ordinal count vector
__device__ __forceinline__ void load_counts4(const unsigned long long* c, uint32_t T, uint32_t i, unsigned long long v[4]) {
    if (i + 4 <= T) {
        const u32x4_t a = load16(c + i), b = load16(c + i + 2);
        v[0] = join64(a.x, a.y); v[1] = join64(a.z, a.w); v[2] = join64(b.x, b.y); v[3] = join64(b.z, b.w);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = i + j < T ? c[i + j] : 0ull;
    }
}

__device__ __forceinline__ void load_counts4(const TopkParams& P, uint32_t i, unsigned long long v[4]) {
    if (!P.counts32) { load_counts4(P.counts, P.T, i, v); return; }
    if (i + 4 <= P.T) {  // u32 counts: one 16-byte load per 4 ordinals
        const u32x4_t a = load16(P.counts32 + i);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = i + j < P.T ? P.counts32[i + j] : 0ull;
    }
}

__global__ __launch_bounds__(1024) void topk_hist_kernel(TopkParams P) {
    if (P.skip && *P.skip) return;
    __shared__ uint32_t hist[kTopkBins];
    for (uint32_t i = threadIdx.x; i < kTopkBins; i += 1024) hist[i] = 0;
    __syncthreads();
    unsigned long long sum = 0;
    for (uint32_t i = (blockIdx.x * 1024 + threadIdx.x) * 4; i < P.T; i += gridDim.x * 1024 * 4) {
        unsigned long long c[4];
        load_counts4(P, i, c);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sum += c[j];
            if (i + j < P.T && topk_eligible(P, c[j])) atomicAdd(&hist[count_bin(P.order, c[j])], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kTopkBins; i += 1024)
        if (hist[i]) atomicAdd(&P.hist[i], hist[i]);
    block_add_u64(P.out_sum, sum);
}

// one workgroup: suffix sums of the histogram (bins are in key order) -> the highest bin b* whose suffix holds >= k
// candidates, or 0 when fewer than k are eligible
__global__ __launch_bounds__(kWG) void topk_thresh_kernel(TopkParams P) {
    if (P.skip && *P.skip) return;
    __shared__ uint32_t v[kTopkBins];
    __shared__ uint32_t wave_tot[kWG / 64];
    __shared__ uint32_t first;
    for (uint32_t i = threadIdx.x; i < kTopkBins; i += kWG) v[i] = P.hist[kTopkBins - 1 - i];  // reversed
    if (threadIdx.x == 0) first = kTopkBins;
    __syncthreads();
    block_exclusive_scan(v, kTopkBins, wave_tot);  // v[i] = candidates in bins > kTopkBins-1-i
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kTopkBins; i += kWG)
        if (v[i] + P.hist[kTopkBins - 1 - i] >= P.k) atomicMin(&first, i);
    __syncthreads();
    if (threadIdx.x == 0) {
        P.sel[0] = first == kTopkBins ? 0u : kTopkBins - 1 - first;  // bins >= b hold >= k candidates (or all)
        P.sel[1] = 0;  // candidate counter for topk_compact
    }
}

__global__ __launch_bounds__(1024) void topk_compact_kernel(TopkParams P) {
    if (P.skip && *P.skip) return;
    const uint32_t tb = P.sel[0];
    const int lane = threadIdx.x & 63;
    for (uint32_t i0 = blockIdx.x * 1024 * 4; i0 < P.T; i0 += gridDim.x * 1024 * 4) {
        const uint32_t i = i0 + threadIdx.x * 4;
        unsigned long long c[4] = {0, 0, 0, 0};
        if (i < P.T) load_counts4(P, i, c);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool take = i + j < P.T && topk_eligible(P, c[j]) && count_bin(P.order, c[j]) >= tb;
            const unsigned long long m = __ballot(take);
            if (m == 0) continue;
            uint32_t base = 0;
            if (lane == __ffsll((long long)m) - 1) base = atomicAdd(&P.sel[1], (uint32_t)__popcll(m));
            base = __shfl(base, __ffsll((long long)m) - 1, 64);
            if (take)
                P.cand[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] =
                    make_topk_key(P.order, c[j], P.ord_of ? P.ord_of[i + j] : i + j);
        }
    }
}

// one workgroup: best k of the n = sel[1] candidate keys, chunked bitonic sort + merge (chunk = pow2 >= n, <= 4096)
__global__ __launch_bounds__(1024) void topk_final_kernel(TopkParams P) {
    if (P.skip && *P.skip) return;
    __shared__ unsigned long long chunk[kTopkChunk];
    __shared__ unsigned long long best[2 * kTopkMax];
    const uint32_t n = P.sel[1];
    uint32_t kp = 1;
    while (kp < P.k) kp <<= 1;
    uint32_t cs = 64;
    while (cs < n && cs < kTopkChunk) cs <<= 1;
    if (cs < kp) cs = kp;
    for (uint32_t i = threadIdx.x; i < kp; i += 1024) best[i] = 0;
    for (uint32_t c0 = 0; c0 < max(n, 1u); c0 += cs) {
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < cs; t += 1024) chunk[t] = c0 + t < n ? P.cand[c0 + t] : 0ull;
        bitonic_sort_desc(chunk, cs);
        for (uint32_t t = threadIdx.x; t < kp; t += 1024) best[kp + t] = chunk[kp - 1 - t];
        bitonic_merge_desc(best, 2 * kp);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < P.k; i += 1024) P.out_keys[i] = best[i];
}

// segment statistics of a high-cardinality column: per partition of 2^shift ordinals, the docs of its cold (not hot)
// ordinals and their largest count -- one workgroup per partition, the hot ordinals as a bitset
__global__ __launch_bounds__(1024) void hc_part_stats_kernel(const unsigned int* counts, uint32_t T, uint32_t shift,
                                                             const uint64_t* hot_bits, unsigned long long* part_sum,
                                                             unsigned int* part_max) {
    const uint32_t p = blockIdx.x;
    const uint32_t o0 = p << shift, o1 = min(T, (p + 1) << shift);
    unsigned long long sum = 0;
    uint32_t mx = 0;
    for (uint32_t o = o0 + threadIdx.x; o < o1; o += 1024) {
        const uint32_t c = counts[o];
        if ((hot_bits[o >> 6] >> (o & 63)) & 1) continue;
        sum += c;
        mx = max(mx, c);
    }
    sum = wave_sum_u64(sum);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    __shared__ unsigned long long ws[16];
    __shared__ uint32_t wm[16];
    if ((threadIdx.x & 63) == 0) { ws[threadIdx.x >> 6] = sum; wm[threadIdx.x >> 6] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        uint32_t m = 0;
        for (int w = 0; w < 16; ++w) { t += ws[w]; m = max(m, wm[w]); }
        part_sum[p] = t;
        part_max[p] = m;
    }
}
void launch_hc_part_stats(const unsigned int* counts, uint32_t T, uint32_t shift, uint32_t P, const uint64_t* hot_bits,
                          unsigned long long* part_sum, unsigned int* part_max, hipStream_t st) {
    if (P) hipLaunchKernelGGL(hc_part_stats_kernel, dim3(P), dim3(1024), 0, st, counts, T, shift, hot_bits, part_sum, part_max);
}

// count orders, k beyond the final sort: the count histogram, its threshold and the candidates at or above it (sel[1]
// of them in cand, in no order; the caller sorts them)
void launch_topk_candidates(const TopkParams& p, hipStream_t s) {
    const uint32_t g = std::max(1u, std::min(p.n_wg, (p.T + 4095) / 4096));
    (void)hipMemsetAsync(p.hist, 0, kTopkBins * 4, s);
    hipLaunchKernelGGL(topk_hist_kernel, dim3(g), dim3(1024), 0, s, p);
    hipLaunchKernelGGL(topk_thresh_kernel, dim3(1), dim3(kWG), 0, s, p);
    hipLaunchKernelGGL(topk_compact_kernel, dim3(g), dim3(1024), 0, s, p);
}

void launch_topk(const TopkParams& p, hipStream_t s) {
    if (p.order == 0 || p.order == 1) {  // count orders: select, then sort the few candidates
        const uint32_t g = std::max(1u, std::min(p.n_wg, (p.T + 4095) / 4096));
        // (with p.skip the histogram is cleared even when the kernels return at once: harmless)
        (void)hipMemsetAsync(p.hist, 0, kTopkBins * 4, s);
        hipLaunchKernelGGL(topk_hist_kernel, dim3(g), dim3(1024), 0, s, p);
        hipLaunchKernelGGL(topk_thresh_kernel, dim3(1), dim3(kWG), 0, s, p);
        hipLaunchKernelGGL(topk_compact_kernel, dim3(g), dim3(1024), 0, s, p);
        hipLaunchKernelGGL(topk_final_kernel, dim3(1), dim3(1024), 0, s, p);
        return;
    }
    const uint32_t per1 = (uint32_t)(((uint64_t)p.T + p.n_wg - 1) / p.n_wg);
    hipLaunchKernelGGL((topk_kernel<true>), dim3(p.n_wg), dim3(1024), 0, s, p, p.counts, p.T, per1, p.cand);
    const uint32_t nc = p.n_wg * p.k;
    hipLaunchKernelGGL((topk_kernel<false>), dim3(1), dim3(1024), 0, s, p, (const unsigned long long*)p.cand, nc, nc,
                       p.out_keys);
}

// K3 per owning bucket for terms under a histogram (GlobalOrdinalsStringTermsAggregator.buildAggregation :146-208 once
// per outer key, count orders): one wave per row.  Each lane keeps the best key of its strided share of the row; the
// wave's maximum is a pick, and only the lane that held it rescans its share for the best key below it -- S picks cost
// S wave reductions plus S rescans of T / 64 cells, where the host spent a pass over all T cells and a partial sort.
__device__ __forceinline__ unsigned long long row_key(unsigned long long c, uint32_t t, bool asc, int64_t min_count) {
    if ((int64_t)c < min_count) return 0ull;
    const unsigned long long hi = asc ? (0xFFFFFFFFull - c) : c;  // counts < 2^32 (docs per shard)
    return (hi << 32) | (unsigned long long)(0xFFFFFFFFu - t);   // never 0: t < 2^32 - 1
}
// the row's keys are staged in LDS when they fit (the rescans then read LDS, not L2 at ~1 us a dependent round), and the
// picks are staged in LDS and written out coalesced at the end
constexpr uint32_t kRowTopkLdsKeys = 4096;  // 32 KB of keys
template <bool LROW>
__global__ __launch_bounds__(64) void row_topk_kernel(const unsigned long long* cnt, uint32_t T, uint32_t S, int asc,
                                                      int64_t min_count, unsigned long long* out,
                                                      unsigned long long* total) {
    __shared__ unsigned long long picks[kRowTopkMax];
    extern __shared__ unsigned long long rowk[];
    const uint32_t row = blockIdx.x;
    const unsigned long long* r = cnt + (size_t)row * T;
    const uint32_t lane = threadIdx.x;
    unsigned long long tot = 0, best = 0;
    for (uint32_t t = lane; t < T; t += 64) {
        const unsigned long long c = r[t];
        tot += c;
        const unsigned long long k = row_key(c, t, asc != 0, min_count);
        if (LROW) rowk[t] = k;
        best = k > best ? k : best;
    }
    tot = wave_sum_u64(tot);
    uint32_t n = 0;
    for (; n < S; ++n) {
        const unsigned long long m = wave_max_u64(best);
        if (m == 0ull) break;
        if (lane == 0) picks[n] = m;
        if (best == m) {
            unsigned long long nb = 0;
            for (uint32_t t = lane; t < T; t += 64) {
                const unsigned long long k = LROW ? rowk[t] : row_key(r[t], t, asc != 0, min_count);
                nb = (k < m && k > nb) ? k : nb;
            }
            best = nb;
        }
    }
    __syncthreads();
    for (uint32_t i = lane; i < S; i += 64) out[(size_t)row * S + i] = i < n ? picks[i] : 0ull;
    if (lane == 0) total[row] = tot;
}
void launch_row_topk(const unsigned long long* cnt, uint32_t T, uint32_t H, uint32_t S, bool asc, int64_t min_count,
                     unsigned long long* out, unsigned long long* total, hipStream_t st) {
    if (H == 0) return;
    if (T <= kRowTopkLdsKeys)
        hipLaunchKernelGGL(row_topk_kernel<true>, dim3(H), dim3(64), (size_t)T * 8, st, cnt, T, S, asc ? 1 : 0, min_count, out, total);
    else
        hipLaunchKernelGGL(row_topk_kernel<false>, dim3(H), dim3(64), 0, st, cnt, T, S, asc ? 1 : 0, min_count, out, total);
}

}  // namespace esgpu

// ------------------------------------------------------------------------------------------------------------
// Multi-valued doc values (SortedSetDocValues / SortedNumericDocValues as CSR: offsets[doc] .. offsets[doc+1]).
//   GlobalOrdinalsStringTermsAggregator (multi-valued ords, :100-112): every ordinal of the doc is a bucket
//   HistogramAggregator.collect (:95-117): keys of the doc's sorted values, equal consecutive keys collected once
//   StatsAggegator / ExtendedStats / Avg collect: count += valueCount, sums[b] += (local sum of the doc's values)
// One doc per thread; the cells of the doc are the cross product of its ordinals and its deduplicated keys.  The grid
// lives in LDS when it fits (flushed like the single-valued kernel), else updates go to HBM with global atomics.
// ------------------------------------------------------------------------------------------------------------
namespace esgpu {

__device__ __forceinline__ bool bit_at(const uint64_t* bm, uint32_t d) { return (bm[d >> 6] >> (d & 63)) & 1; }

// histogram field value i as a long (a double field is cast, ValuesSource.Numeric.longValues)
__device__ __forceinline__ int64_t hv_at(const CollectParams& P, uint64_t i) {
    const int64_t x = P.hv[i];
    return P.hv_f64 ? java_long(bits_dbl((uint64_t)x)) : x;
}

// key slot of histogram value i: a rounded / table-looked-up key, or (HK 3, terms under terms) the inner field's ordinal
// itself (u32 column; missing = 0xFFFFFFFF lands outside [0, H) and is skipped)
template <int HK>
__device__ __forceinline__ int64_t multi_key(const CollectParams& P, uint64_t i) {
    if constexpr (HK == 3) return (int64_t)((const uint32_t*)P.hv)[i];
    else return key_index<HK == 2>(P, hv_at(P, i));
}

// values [b, e) of doc d in a column (single valued: [d, d+1) when present)
__device__ __forceinline__ void value_range(const uint64_t* off, const uint64_t* present, uint32_t d, uint64_t& b,
                                            uint64_t& e) {
    if (off) {
        b = off[d];
        e = off[d + 1];
    } else {
        b = d;
        e = (uint64_t)d + ((present && !bit_at(present, d)) ? 0 : 1);
    }
}

__device__ bool pred_doc(const PredDev& q, uint32_t d) {
    uint64_t b, e;
    value_range(q.offsets, q.present, d, b, e);
    for (uint64_t i = b; i < e; ++i) {
        bool m;
        if (q.kind == PRED_ORD_EQ || q.kind == PRED_ORD_RANGE) {
            const uint32_t o = ((const uint32_t*)q.col)[i];
            m = o != kMissingOrd && (int64_t)o >= q.lo && (int64_t)o <= q.hi;
        } else if (q.kind == PRED_F64_RANGE) {
            const double v = ((const double*)q.col)[i];
            m = (q.lo_incl ? v >= q.dlo : v > q.dlo) && (q.hi_incl ? v <= q.dhi : v < q.dhi);
        } else if (q.kind == PRED_D32_RANGE || q.kind == PRED_D16_RANGE) {
            const int64_t v = q.base + (q.kind == PRED_D16_RANGE ? (int64_t)((const uint16_t*)q.col)[i] : (int64_t)((const uint32_t*)q.col)[i]);
            m = v >= q.lo && v <= q.hi;
        } else {
            const int64_t v = ((const int64_t*)q.col)[i];
            m = v >= q.lo && v <= q.hi;
        }
        if (m) return true;
    }
    return false;
}

template <bool ORD, int HK, int MET>
__global__ __launch_bounds__(kWG) void collect_multi_kernel(CollectParams P) {
    constexpr bool HIST = HK != 0;
    constexpr bool KT = HK == 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t T = ORD ? P.T : 1u;
    const uint32_t H = HIST ? P.H : 1u;
    const uint32_t C = T * H;
    Acc g;
    g.cnt32 = nullptr; g.vcnt32 = nullptr; g.ocnt32 = nullptr;
    g.cnt64 = P.g_cnt; g.vcnt64 = P.g_vcnt; g.sum = P.g_sum; g.mn = P.g_min; g.mx = P.g_max; g.sq = P.g_sq;
    g.sum_lo = P.g_sum_lo; g.sq_lo = P.g_sq_lo;
    g.mstride = 1;
    g.coff = 0;
    g.ocnt64 = P.g_ocnt;
    Acc s;
    s.sum_lo = nullptr; s.sq_lo = nullptr;
    {
        size_t off = 0;
        auto carve = [&](size_t bytes) { unsigned char* p = smem + off; off += (bytes + 15) & ~(size_t)15; return p; };
        s.cnt64 = nullptr; s.vcnt64 = nullptr; s.ocnt64 = nullptr;
        s.cnt32 = (uint32_t*)carve(sizeof(uint32_t) * C);
        s.vcnt32 = (uint32_t*)carve(P.vcnt_mode ? sizeof(uint32_t) * C : 0);
        s.sum = (double*)carve(MET > 0 ? sizeof(double) * C : 0);
        s.mn = (unsigned long long*)carve(MET >= 2 ? 16 * C : 0);
        s.mx = s.mn + 1;
        s.mstride = 2;
        s.coff = 0;
        s.sq = (double*)carve(MET >= 3 ? sizeof(double) * C : 0);
        s.ocnt32 = (uint32_t*)carve(P.ocnt_mode == OCNT_TERMS ? sizeof(uint32_t) * T : P.ocnt_mode == OCNT_HIST ? sizeof(uint32_t) * H : 0);
    }
    if (P.lds_mode) {
        for (uint32_t c = threadIdx.x; c < C; c += kWG) {
            s.cnt32[c] = 0;
            if (P.vcnt_mode) s.vcnt32[c] = 0;
            if (MET > 0) s.sum[c] = 0.0;
            if (MET >= 2) { s.mn[2 * c] = kMinInit; s.mx[2 * c] = kMaxInit; }
            if (MET >= 3) s.sq[c] = 0.0;
        }
        if (P.ocnt_mode == OCNT_TERMS || P.ocnt_mode == OCNT_HIST)
            for (uint32_t c = threadIdx.x; c < (P.ocnt_mode == OCNT_TERMS ? T : H); c += kWG) s.ocnt32[c] = 0;
        __syncthreads();
    }
    for (uint32_t d = blockIdx.x * kWG + threadIdx.x; d < P.n_docs; d += gridDim.x * kWG) {
        if (P.accept && !bit_at(P.accept, d)) continue;
        // the doc's metric values, aggregated once (StatsAggegator.collect: local sum, then sums[b] += sum)
        uint32_t nm = 0;
        double msum = 0.0, msq = 0.0;
        unsigned long long emn = kMinInit, emx = kMaxInit;
        if (MET > 0) {
            uint64_t b, e;
            value_range(P.mv_off, P.mv_present, d, b, e);
            for (uint64_t i = b; i < e; ++i) {
                const double x = P.mv_f64 ? ((const double*)P.mv)[i] : (double)((const int64_t*)P.mv)[i];
                msum += x;
                if (MET >= 3) msq += x * x;
                if (MET >= 2) {
                    const bool nan = x != x;
                    const unsigned long long en = sortable(x);
                    const unsigned long long a = nan ? 0ull : en, z = nan ? ~0ull : en;
                    emn = a < emn ? a : emn;
                    emx = z > emx ? z : emx;
                }
                ++nm;
            }
        }
        uint64_t ob = 0, oe = 1, hb = 0, he = 1;
        if (ORD) value_range(P.ord_off, nullptr, d, ob, oe);
        if (HIST) value_range(P.hv_off, P.hv_present, d, hb, he);
        if (HIST && P.ocnt_mode == OCNT_HIST) {  // outer histogram doc counts: once per distinct key
            bool first = true;
            int64_t prev = 0;
            for (uint64_t h = hb; h < he; ++h) {
                const int64_t k = multi_key<HK>(P, h);
                if (!first && k == prev) continue;
                first = false;
                prev = k;
                if (k < 0 || k >= (int64_t)H) continue;
                if (P.lds_mode) atomicAdd(&s.ocnt32[k], 1u); else atomicAdd(&g.ocnt64[k], 1ull);
            }
        }
        for (uint64_t o = ob; o < oe; ++o) {
            const uint32_t t = ORD ? P.ord[o] : 0u;
            if (ORD && (t == kMissingOrd || t >= T)) continue;
            if (ORD && P.ocnt_mode == OCNT_TERMS) {
                if (P.lds_mode) atomicAdd(&s.ocnt32[t], 1u); else atomicAdd(&g.ocnt64[t], 1ull);
            }
            bool first = true;
            int64_t prev = 0;
            for (uint64_t h = hb; h < he; ++h) {
                uint32_t slot = 0;
                if (HIST) {
                    const int64_t k = multi_key<HK>(P, h);
                    if (!first && k == prev) continue;
                    first = false;
                    prev = k;
                    if (k < 0 || k >= (int64_t)H) continue;
                    slot = (uint32_t)k;
                }
                const uint32_t c = slot * T + t;
                const Acc& a = P.lds_mode ? s : g;
                if (P.lds_mode) atomicAdd(&s.cnt32[c], 1u); else atomicAdd(&g.cnt64[c], 1ull);
                if (MET > 0 && nm) {
                    if (P.vcnt_mode) {
                        if (P.lds_mode) atomicAdd(&s.vcnt32[c], nm); else atomicAdd(&g.vcnt64[c], (unsigned long long)nm);
                    }
                    if (P.lds_mode) atomicAdd(&s.sum[c], msum);
                    else dd_atomic_add(&g.sum[c], g.sum_lo ? g.sum_lo + c : nullptr, msum);
                    if (MET >= 2) {
                        if (emn < a.mn[c * a.mstride]) atomicMin(&a.mn[c * a.mstride], emn);
                        if (emx > a.mx[c * a.mstride]) atomicMax(&a.mx[c * a.mstride], emx);
                    }
                    if (MET >= 3) {
                        if (P.lds_mode) atomicAdd(&s.sq[c], msq);
                        else dd_atomic_add(&g.sq[c], g.sq_lo ? g.sq_lo + c : nullptr, msq);
                    }
                }
            }
        }
    }
    if (P.lds_mode) flush_window<MET, 2, kWG>(P, s, T, H, 0);
}

template <bool ORD, int HK, int MET>
static void launch_multi_t(const CollectParams& p, uint32_t grid, size_t lds, hipStream_t st) {
    hipLaunchKernelGGL((collect_multi_kernel<ORD, HK, MET>), dim3(grid), dim3(kWG), lds, st, p);
}
template <bool ORD, int HK>
static void launch_multi_m(const CollectParams& p, int met, uint32_t grid, size_t lds, hipStream_t st) {
    switch (met) {
        case 0: launch_multi_t<ORD, HK, 0>(p, grid, lds, st); break;
        case 1: launch_multi_t<ORD, HK, 1>(p, grid, lds, st); break;
        case 2: launch_multi_t<ORD, HK, 2>(p, grid, lds, st); break;
        default: launch_multi_t<ORD, HK, 3>(p, grid, lds, st); break;
    }
}
void launch_collect_multi(const CollectParams& p, bool ord, bool hist, int met, uint32_t grid, size_t lds, hipStream_t st) {
    const int hk = hist ? (p.hord ? 3 : p.kstart ? 2 : 1) : 0;
    if (ord) {
        if (hk == 3) launch_multi_m<true, 3>(p, met, grid, lds, st);
        else if (hk == 2) launch_multi_m<true, 2>(p, met, grid, lds, st);
        else if (hk == 1) launch_multi_m<true, 1>(p, met, grid, lds, st);
        else launch_multi_m<true, 0>(p, met, grid, lds, st);
    } else {
        if (hk == 2) launch_multi_m<false, 2>(p, met, grid, lds, st);
        else if (hk == 1) launch_multi_m<false, 1>(p, met, grid, lds, st);
        else launch_multi_m<false, 0>(p, met, grid, lds, st);
    }
}

struct FilterBitsArgs {
    uint32_t n_docs;
    int32_t npred;
    const uint64_t* accept;
    uint64_t* out;
    PredDev pred[4];
};
// one thread per 64-doc word: no atomics
__global__ __launch_bounds__(256) void filter_bits_kernel(FilterBitsArgs A) {
    const uint32_t nw = (A.n_docs + 63) / 64;
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
        uint64_t bits = A.accept ? A.accept[w] : ~0ull;
        const uint32_t d0 = w * 64;
        if (d0 + 64 > A.n_docs) bits &= (1ull << (A.n_docs - d0)) - 1ull;
        for (int j = 0; j < 64; ++j) {
            if (!((bits >> j) & 1)) continue;
            for (int k = 0; k < A.npred; ++k)
                if (!pred_doc(A.pred[k], d0 + j)) { bits &= ~(1ull << j); break; }
        }
        A.out[w] = bits;
    }
}
void launch_filter_bits(uint32_t n_docs, const uint64_t* accept, const PredDev* preds, int npred, uint64_t* out,
                        hipStream_t st) {
    FilterBitsArgs A{};
    A.n_docs = n_docs;
    A.npred = npred;
    A.accept = accept;
    A.out = out;
    for (int k = 0; k < npred && k < 4; ++k) A.pred[k] = preds[k];
    const uint32_t nw = (n_docs + 63) / 64;
    if (nw == 0) return;
    hipLaunchKernelGGL(filter_bits_kernel, dim3(std::min<uint32_t>(4096, (nw + 255) / 256)), dim3(256), 0, st, A);
}

// the request's clauses over single-valued columns folded into a doc bitset at the streaming rate (4 docs per thread,
// the collect loader's quad predicates; 16 lanes' 4-bit masks OR-ed into each 64-doc word), for the collect kernels
// that read one accept bitset instead of evaluating clauses (VK bit 512)
__global__ __launch_bounds__(256) void filter_bits4_kernel(FilterBitsArgs A, uint32_t n_quads) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t q0 = blockIdx.x * 256; q0 < n_quads; q0 += gridDim.x * 256) {  // block-uniform trip count
        const uint32_t q = q0 + threadIdx.x, doc0 = q * 4;
        uint64_t m = 0;
        if (q < n_quads) {
            uint32_t ok = doc0 + 4 <= A.n_docs ? 0xFu : doc0 >= A.n_docs ? 0u : (1u << (A.n_docs - doc0)) - 1u;
            if (A.accept) ok &= (uint32_t)(A.accept[doc0 >> 6] >> (doc0 & 63)) & 0xFu;
            for (int k = 0; k < A.npred; ++k) ok &= eval_pred(A.pred[k], doc0);
            m = (uint64_t)ok << ((lane & 15) * 4);
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) m |= (uint64_t)__shfl_xor((long long)m, o, 64);
        if ((lane & 15) == 0 && q < n_quads) A.out[doc0 >> 6] = m;
    }
}
void launch_filter_bits4(uint32_t n_docs, const uint64_t* accept, const PredDev* preds, int npred, uint64_t* out,
                         hipStream_t st) {
    FilterBitsArgs A{};
    A.n_docs = n_docs;
    A.npred = npred;
    A.accept = accept;
    A.out = out;
    for (int k = 0; k < npred && k < 4; ++k) A.pred[k] = preds[k];
    const uint32_t nq = ((n_docs + 63) / 64) * 16;  // whole words
    if (nq == 0) return;
    hipLaunchKernelGGL(filter_bits4_kernel, dim3(std::min<uint32_t>(8192, (nq + 255) / 256)), dim3(256), 0, st, A, nq);
}

__global__ __launch_bounds__(256) void expand_bits_kernel(uint32_t n_docs, const uint64_t* doc_bits, const uint64_t* off,
                                                         uint64_t* out) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < n_docs; d += gridDim.x * blockDim.x) {
        if (!bit_at(doc_bits, d)) continue;
        for (uint64_t i = off[d]; i < off[d + 1]; ++i) atomicOr(&out[i >> 6], 1ull << (i & 63));
    }
}
void launch_expand_bits(uint32_t n_docs, const uint64_t* doc_bits, const uint64_t* offsets, uint64_t n_values,
                        uint64_t* out, hipStream_t st) {
    (void)hipMemsetAsync(out, 0, (n_values + 63) / 64 * 8, st);
    if (n_docs == 0) return;
    hipLaunchKernelGGL(expand_bits_kernel, dim3(std::min<uint32_t>(4096, (n_docs + 255) / 256)), dim3(256), 0, st, n_docs,
                       doc_bits, offsets, out);
}

// ---- cardinality per bucket ----
__device__ __forceinline__ void reg_max_u8(uint8_t* regs, size_t idx, uint32_t rl) {
    uint32_t* w = (uint32_t*)(regs + (idx & ~(size_t)3));
    const int sh = (int)(idx & 3) * 8;
    uint32_t old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (((old >> sh) & 0xFFu) < rl) {
        const uint32_t nw = (old & ~(0xFFu << sh)) | (rl << sh);
        const uint32_t prev = atomicCAS(w, old, nw);
        if (prev == old) break;
        old = prev;
    }
}

__device__ __forceinline__ bool card_hash(const CardParams& C, uint64_t i, uint64_t& h) {
    if (C.kind == HLL_ORD) {
        const uint32_t o = ((const uint32_t*)C.col)[i];
        if (o == kMissingOrd || o >= C.n_ords) return false;
        h = C.ord_hash[o];
        return true;
    }
    uint64_t bits = ((const uint64_t*)C.col)[i];
    if (C.kind == HLL_F64) {  // MurmurHash3Values.Double: doubleToLongBits (canonical NaN)
        const double x = bits_dbl(bits);
        if (x != x) bits = 0x7ff8000000000000ULL;
    }
    h = mix64(bits);
    return true;
}

template <bool ORD, int HK>
__global__ __launch_bounds__(256) void card_kernel(CardParams C, int pass) {
    constexpr bool HIST = HK != 0;
    constexpr bool KT = HK == 2;
    const CollectParams& P = C.G;
    const uint32_t T = ORD ? P.T : 1u;
    const uint32_t H = HIST ? P.H : 1u;
    const uint32_t m = 1u << C.p;
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < P.n_docs; d += gridDim.x * blockDim.x) {
        if (P.accept && !bit_at(P.accept, d)) continue;
        uint64_t vb, ve;
        value_range(C.off, C.present, d, vb, ve);
        if (vb == ve) continue;
        uint64_t ob = 0, oe = 1, hb = 0, he = 1;
        if (ORD) value_range(P.ord_off, nullptr, d, ob, oe);
        if (HIST) value_range(P.hv_off, P.hv_present, d, hb, he);
        for (uint64_t o = ob; o < oe; ++o) {
            const uint32_t t = ORD ? P.ord[o] : 0u;
            if (ORD && (t == kMissingOrd || t >= T)) continue;
            bool first = true;
            int64_t prev = 0;
            for (uint64_t hh = hb; hh < he; ++hh) {
                uint32_t slot = 0;
                if (HIST) {
                    const int64_t k = multi_key<HK>(P, hh);
                    if (!first && k == prev) continue;
                    first = false;
                    prev = k;
                    if (k < 0 || k >= (int64_t)H) continue;
                    slot = (uint32_t)k;
                }
                const size_t b = (size_t)slot * T + t;
                if (pass == 1 && (C.nonzero[b] > C.thr ||
                                  __hip_atomic_load(&C.set_cnt[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > C.thr))
                    continue;  // this bucket already ends in HYPERLOGLOG
                for (uint64_t i = vb; i < ve; ++i) {
                    uint64_t h;
                    if (!card_hash(C, i, h)) continue;
                    if (pass == 0) {
                        reg_max_u8(C.regs, b * m + hll_index(h, C.p), hll_run_len(h, C.p));
                        continue;
                    }
                    const uint32_t enc = hll_encode(h, C.p);
                    const unsigned long long pos = C.pos_base + (C.pos_ord ? (uint64_t)((const uint32_t*)C.col)[i] : i);
                    uint32_t* set = C.sets + b * C.cap;
                    uint32_t sl = (uint32_t)(mix64(enc) & (C.cap - 1));
                    uint32_t probe = 0;
                    for (; probe < C.cap; ++probe) {
                        const uint32_t cur = __hip_atomic_load(&set[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        bool found = cur == enc;
                        if (!found && cur == 0) {
                            const uint32_t was = atomicCAS(&set[sl], 0u, enc);
                            if (was == 0) atomicAdd(&C.set_cnt[b], 1u);
                            found = was == 0 || was == enc;
                        }
                        if (found) {
                            atomicMin(&C.first[b * C.cap + sl], pos);
                            break;
                        }
                        sl = (sl + 1) & (C.cap - 1);
                    }
                    if (probe == C.cap) atomicAdd(&C.set_cnt[b], C.cap);  // full: more than cap distinct hashes
                }
            }
        }
    }
}

void launch_card(const CardParams& c, bool ord, bool hist, int pass, uint32_t grid, hipStream_t st) {
    const int hk = hist ? (c.G.hord ? 3 : c.G.kstart ? 2 : 1) : 0;
    if (ord) {
        if (hk == 3) hipLaunchKernelGGL((card_kernel<true, 3>), dim3(grid), dim3(256), 0, st, c, pass);
        else if (hk == 2) hipLaunchKernelGGL((card_kernel<true, 2>), dim3(grid), dim3(256), 0, st, c, pass);
        else if (hk == 1) hipLaunchKernelGGL((card_kernel<true, 1>), dim3(grid), dim3(256), 0, st, c, pass);
        else hipLaunchKernelGGL((card_kernel<true, 0>), dim3(grid), dim3(256), 0, st, c, pass);
    } else {
        if (hk == 2) hipLaunchKernelGGL((card_kernel<false, 2>), dim3(grid), dim3(256), 0, st, c, pass);
        else if (hk == 1) hipLaunchKernelGGL((card_kernel<false, 1>), dim3(grid), dim3(256), 0, st, c, pass);
        else hipLaunchKernelGGL((card_kernel<false, 0>), dim3(grid), dim3(256), 0, st, c, pass);
    }
}

__global__ __launch_bounds__(256) void card_nonzero_kernel(const uint32_t* regs, uint64_t n_words, uint32_t words_per_bucket,
                                                          uint32_t* nonzero) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_words; w += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = regs[w];
        const uint32_t n = ((v & 0xFFu) != 0) + ((v & 0xFF00u) != 0) + ((v & 0xFF0000u) != 0) + ((v & 0xFF000000u) != 0);
        if (n) atomicAdd(&nonzero[w / words_per_bucket], n);
    }
}
void launch_card_nonzero(const uint8_t* regs, uint64_t n_buckets, int p, uint32_t* nonzero, hipStream_t st) {
    (void)hipMemsetAsync(nonzero, 0, n_buckets * 4, st);
    const uint32_t wpb = (1u << p) / 4;
    const uint64_t n_words = n_buckets * wpb;
    if (n_words == 0) return;
    hipLaunchKernelGGL(card_nonzero_kernel, dim3((uint32_t)std::min<uint64_t>(8192, (n_words + 255) / 256)), dim3(256), 0, st,
                       (const uint32_t*)regs, n_words, wpb, nonzero);
}

__global__ __launch_bounds__(256) void gather_bytes_kernel(const uint32_t* cells, uint32_t n, uint32_t row, const uint8_t* src,
                                                          uint8_t* dst) {
    const uint32_t wpr = row / 4;  // rows are multiples of 4 bytes
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)n * wpr; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = i / wpr, w = i - r * wpr;
        ((uint32_t*)dst)[i] = ((const uint32_t*)(src + (size_t)cells[r] * row))[w];
    }
}
void launch_gather_bytes(const uint32_t* cells, uint32_t n, uint32_t row_bytes, const uint8_t* src, uint8_t* dst, hipStream_t st) {
    const uint64_t total = (uint64_t)n * (row_bytes / 4);
    if (total == 0) return;
    hipLaunchKernelGGL(gather_bytes_kernel, dim3((uint32_t)std::min<uint64_t>(8192, (total + 255) / 256)), dim3(256), 0, st, cells,
                       n, row_bytes, src, dst);
}

// ---- index-time hashing: one value per thread ----
__global__ __launch_bounds__(256) void route_kernel(const uint16_t* chars, const uint64_t* off, uint64_t n, int32_t nshards,
                                                   int32_t* hash_out, int32_t* shard_out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t h = (int32_t)murmur3_x86_32_utf16(chars + off[i], (int)(off[i + 1] - off[i]), 0);
        if (hash_out) hash_out[i] = h;
        shard_out[i] = routing_shard(h, nshards);
    }
}
void launch_route(const uint16_t* chars, const uint64_t* offsets, uint64_t n, int32_t nshards, int32_t* hash_out,
                  int32_t* shard_out, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(route_kernel, dim3((uint32_t)std::min<uint64_t>(8192, (n + 255) / 256)), dim3(256), 0, st, chars, offsets, n,
                       nshards, hash_out, shard_out);
}
__global__ __launch_bounds__(256) void murmur3_field_kernel(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint64_t* h1_out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h1, h2;
        murmur3_x64_128(bytes + off[i], (int)(off[i + 1] - off[i]), 0, &h1, &h2);
        h1_out[i] = h1;
    }
}
void launch_murmur3_field(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1_out, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(murmur3_field_kernel, dim3((uint32_t)std::min<uint64_t>(8192, (n + 255) / 256)), dim3(256), 0, st, bytes,
                       offsets, n, h1_out);
}

__global__ __launch_bounds__(256) void minmax_i64_kernel(const int64_t* v, uint64_t n, int64_t* out, int f64) {
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t x = f64 ? java_long(bits_dbl((uint64_t)v[i])) : v[i];
        mn = x < mn ? x : mn;
        mx = x > mx ? x : mx;
    }
    atomicMin((long long*)&out[0], (long long)mn);
    atomicMax((long long*)&out[1], (long long)mx);
}
// histogram under histogram: the inner histogram's key index of every doc as a u32 "ordinal" (affine rounding;
// 0xFFFFFFFF = no value, or a key outside [key0, key0 + nkeys)), padded docs included
__global__ __launch_bounds__(256) void hist_ords_kernel(const int64_t* v, const uint64_t* present, uint32_t n_docs,
                                                        uint32_t n_pad, int f64, int64_t interval, int64_t offset,
                                                        int64_t key0, uint32_t nkeys, uint32_t* out) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < n_pad; d += gridDim.x * blockDim.x) {
        uint32_t o = 0xFFFFFFFFu;
        if (d < n_docs && (!present || ((present[d >> 6] >> (d & 63)) & 1))) {
            const int64_t x = f64 ? java_long(bits_dbl((uint64_t)v[d])) : v[d];  // ValuesSource.Numeric.longValues
            const int64_t k = floor_div64(x - offset, interval) - key0;         // Rounding.Interval.roundKey
            if (k >= 0 && k < (int64_t)nkeys) o = (uint32_t)k;
        }
        out[d] = o;
    }
}
__global__ __launch_bounds__(256) void hist_ords_multi_kernel(const int64_t* v, const uint64_t* off, uint32_t n_docs, int f64,
                                                              int64_t interval, int64_t offset, int64_t key0, uint32_t nkeys,
                                                              uint32_t* out) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < n_docs; d += gridDim.x * blockDim.x) {
        int64_t prev = 0;
        bool first = true;
        for (uint64_t i = off[d]; i < off[d + 1]; ++i) {
            const int64_t x = f64 ? java_long(bits_dbl((uint64_t)v[i])) : v[i];
            const int64_t k = floor_div64(x - offset, interval) - key0;
            const bool dup = !first && k == prev;  // (a doc's values are sorted: its keys are too)
            first = false;
            prev = k;
            out[i] = !dup && k >= 0 && k < (int64_t)nkeys ? (uint32_t)k : 0xFFFFFFFFu;
        }
    }
}
__device__ __forceinline__ uint32_t table_key(const int64_t* starts, uint32_t nsteps, const uint32_t* slot, uint32_t nkeys,
                                              int64_t x) {
    if (nsteps == 0 || x < starts[0]) return 0xFFFFFFFFu;
    uint32_t lo = 0, hi = nsteps;  // starts[lo] <= x < starts[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (starts[mid] <= x) lo = mid; else hi = mid;
    }
    const uint32_t k = slot ? slot[lo] : lo;
    return k < nkeys ? k : 0xFFFFFFFFu;
}
__global__ __launch_bounds__(256) void hist_ords_table_kernel(const int64_t* v, const uint64_t* present, const uint64_t* off,
                                                              uint32_t n_docs, uint32_t n_pad, int f64, const int64_t* starts,
                                                              uint32_t nsteps, const uint32_t* slot, uint32_t nkeys,
                                                              uint32_t* out) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < (off ? n_docs : n_pad); d += gridDim.x * blockDim.x) {
        if (!off) {
            uint32_t o = 0xFFFFFFFFu;
            if (d < n_docs && (!present || ((present[d >> 6] >> (d & 63)) & 1)))
                o = table_key(starts, nsteps, slot, nkeys, f64 ? java_long(bits_dbl((uint64_t)v[d])) : v[d]);
            out[d] = o;
            continue;
        }
        uint32_t prev = 0xFFFFFFFFu;
        for (uint64_t i = off[d]; i < off[d + 1]; ++i) {  // a doc's repeated keys once (HistogramAggregator.collect)
            const uint32_t k = table_key(starts, nsteps, slot, nkeys, f64 ? java_long(bits_dbl((uint64_t)v[i])) : v[i]);
            const bool dup = i > off[d] && k == prev;
            prev = k;
            out[i] = dup ? 0xFFFFFFFFu : k;
        }
    }
}
void launch_hist_ords_table(const int64_t* v, const uint64_t* present, const uint64_t* offsets, uint32_t n_docs, uint32_t n_pad,
                            bool f64, const int64_t* starts, uint32_t nsteps, const uint32_t* slot, uint32_t nkeys,
                            uint32_t* out, hipStream_t st) {
    const uint32_t n = offsets ? n_docs : n_pad;
    if (n == 0) return;
    hipLaunchKernelGGL(hist_ords_table_kernel, dim3(std::min<uint32_t>(8192, (n + 255) / 256)), dim3(256), 0, st, v, present,
                       offsets, n_docs, n_pad, f64 ? 1 : 0, starts, nsteps, slot, nkeys, out);
}
void launch_hist_ords_multi(const int64_t* v, const uint64_t* offsets, uint32_t n_docs, bool f64, int64_t interval,
                            int64_t offset, int64_t key0, uint32_t nkeys, uint32_t* out, hipStream_t st) {
    if (n_docs == 0) return;
    hipLaunchKernelGGL(hist_ords_multi_kernel, dim3(std::min<uint32_t>(8192, (n_docs + 255) / 256)), dim3(256), 0, st, v,
                       offsets, n_docs, f64 ? 1 : 0, interval, offset, key0, nkeys, out);
}
void launch_hist_ords(const int64_t* v, const uint64_t* present, uint32_t n_docs, uint32_t n_pad, bool f64, int64_t interval,
                      int64_t offset, int64_t key0, uint32_t nkeys, uint32_t* out, hipStream_t st) {
    if (n_pad == 0) return;
    hipLaunchKernelGGL(hist_ords_kernel, dim3(std::min<uint32_t>(8192, (n_pad + 255) / 256)), dim3(256), 0, st, v, present, n_docs,
                       n_pad, f64 ? 1 : 0, interval, offset, key0, nkeys, out);
}

// three bucket levels: the pair of two single-valued ordinal columns as one composite ordinal a * nb + b (missing when
// either is missing or out of its dictionary); 16-byte loads and stores, n_pad is a multiple of kBlockDocs
// composite ordinals a * nb + b (missing when either is); with `amap`, a is first mapped through it (breadth-first
// replay: the outer ordinal's winner slot, kMissingOrd for the ordinals that did not survive)
__global__ __launch_bounds__(256) void comp_ords_kernel(const uint32_t* a, const uint32_t* b, uint32_t n_pad, uint32_t na,
                                                        uint32_t nb, const uint32_t* amap, uint32_t amap_n, uint32_t* out) {
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n_pad; i += gridDim.x * blockDim.x * 4) {
        uint32_t x[4], y[4];
        load_u32x4(a, i, x);
        load_u32x4(b, i, y);
        if (amap) {
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = x[j] < amap_n ? amap[x[j]] : kMissingOrd;
        }
        u32x4_t o;
        o.x = x[0] < na && y[0] < nb ? x[0] * nb + y[0] : kMissingOrd;
        o.y = x[1] < na && y[1] < nb ? x[1] * nb + y[1] : kMissingOrd;
        o.z = x[2] < na && y[2] < nb ? x[2] * nb + y[2] : kMissingOrd;
        o.w = x[3] < na && y[3] < nb ? x[3] * nb + y[3] : kMissingOrd;
        *reinterpret_cast<u32x4_t*>(out + i) = o;
    }
}
void launch_comp_ords(const uint32_t* a, const uint32_t* b, uint32_t n_pad, uint32_t na, uint32_t nb, const uint32_t* amap,
                      uint32_t amap_n, uint32_t* out, hipStream_t st) {
    if (n_pad == 0) return;
    hipLaunchKernelGGL(comp_ords_kernel, dim3(std::min<uint32_t>(8192, (n_pad / 4 + 255) / 256)), dim3(256), 0, st, a, b, n_pad,
                       na, nb, amap, amap_n, out);
}

// one 8192-doc block per workgroup: each doc's batch and replay ordinal (the slot map carries the batch, no per-doc
// division), then the appends.  Up to kReplayFastBatches batches: the block's appends are sorted by batch in LDS -- a
// thread's per-batch counts packed as 16-bit fields of two u64 words, one wave scan of each, the waves' totals combined
// per batch -- and leave as one contiguous, coalesced run per batch after one global reservation per (workgroup, batch)
// on its own cache line.  More batches: a position per wave round of each distinct batch, scattered appends.
constexpr uint32_t kReplayFastBatches = 8;
#ifndef ESGPU_RC_EXP  // timing experiments only (wrong results): 1 = no appends, 2 = no global reservations, 3 = loads alone
#define ESGPU_RC_EXP 0
#endif
// the block's docs (16 per thread): each one's batch and replay ordinal (the slot map carries the batch: no per-doc
// division); bid = kMissingOrd when the doc does not survive
constexpr uint32_t kReplayLdsMap = 4096;  // outer ordinals whose slot map the sort kernel stages in LDS (16 KB)
__device__ __forceinline__ void replay_classify(const ReplayCompactParams& P, const uint32_t* __restrict__ smap,
                                                uint32_t (&val)[kItersPerBlock][4], uint32_t (&bid)[kItersPerBlock][4]) {
    constexpr uint32_t kRMask = (1u << kReplayBatchShift) - 1u;
#pragma unroll
    for (int it = 0; it < kItersPerBlock; ++it) {
        const uint32_t doc0 = blockIdx.x * kBlockDocs + it * kIterDocs + threadIdx.x * kVec;
        uint32_t x[4], y[4];
        if (P.a16) {
            const u32x2_t w = load8(P.a16 + doc0);
            const uint32_t h[4] = {w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16};
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = h[j] == 0xFFFFu ? kMissingOrd : h[j];
        } else {
            load_u32x4(P.a, doc0, x);
        }
        load_u32x4(P.b, doc0, y);
        uint32_t ok = 0xF;
        if (doc0 + 4 > P.n_docs) ok = doc0 >= P.n_docs ? 0u : ((1u << (P.n_docs - doc0)) - 1u);
        if (P.accept) ok &= bits4(P.accept, doc0);
        for (int k = 0; k < P.npred; ++k) ok &= eval_pred(P.pred[k], doc0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t m = ((ok >> j) & 1) && x[j] < P.slot_map_n ? smap[x[j]] : kMissingOrd;
            const bool live = m != kMissingOrd && y[j] < P.vcB;
            bid[it][j] = live ? m >> kReplayBatchShift : kMissingOrd;
            val[it][j] = live ? (m & kRMask) * P.stride + y[j] : 0u;
        }
    }
}

// up to kReplayFastBatches batches (the usual case): the block's appends are sorted by batch in LDS -- a thread's
// per-batch counts packed as 16-bit fields of two u64 words, one wave scan of each, the waves' totals combined per
// batch by one thread each -- and leave as one contiguous, coalesced run per batch after one global reservation per
// (workgroup, batch) on its own cache line.  A doc's batch is kept in 4 bits and its rank among the thread's docs of
// that batch recounted when it is staged, so the kernel holds few registers (a block's 16 docs per thread).
__global__ __launch_bounds__(kWG, 2) void replay_compact_sort_kernel(ReplayCompactParams P) {
    __shared__ uint32_t stage[kBlockDocs];                       // the block's appends, batch by batch
    __shared__ uint32_t wtot[kWG / 64][kReplayFastBatches];      // per wave and batch: appends
    __shared__ uint32_t wpos[kWG / 64][kReplayFastBatches];      // ... and their first staging position
    __shared__ uint32_t boff[kReplayFastBatches + 1], glim[kReplayFastBatches];
    __shared__ unsigned long long gdst[kReplayFastBatches];
    // the slot map in LDS when it is small (the outer terms of a breadth-first request: hosts, statuses): 16 gathers per
    // thread from a global table queue on the texture unit, tens of cycles per wave each
    __shared__ uint32_t lmap[kReplayLdsMap];
    const uint32_t* smap = P.slot_map;
    if (P.slot_map_n <= kReplayLdsMap) {
        for (uint32_t i = threadIdx.x; i < P.slot_map_n; i += kWG) lmap[i] = P.slot_map[i];
        __syncthreads();
        smap = lmap;
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t val[kItersPerBlock][4];
    unsigned long long bits = 0;  // doc k's batch in bits 4k..4k+3 (15: none)
    unsigned long long c[2] = {0ull, 0ull};
    {
        uint32_t bid[kItersPerBlock][4];
        replay_classify(P, smap, val, bid);
#if ESGPU_RC_EXP == 3
        uint32_t acc = 0;
#pragma unroll
        for (int it = 0; it < kItersPerBlock; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc += val[it][j] + bid[it][j];
        if (acc == 0x12345u) *P.overflow = acc;
        return;
#endif
#pragma unroll
        for (int it = 0; it < kItersPerBlock; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t b = bid[it][j] < kReplayFastBatches ? bid[it][j] : 15u;
                bits |= (unsigned long long)b << (4 * (it * 4 + j));
                const unsigned long long one = b < kReplayFastBatches ? 1ull << (16u * (b & 3u)) : 0ull;
                if (b < 4u) c[0] += one; else c[1] += one;
            }
    }
    // wave exclusive scan of both words (a wave holds at most 1,024 docs of a batch: no field overflows)
    unsigned long long e[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        unsigned long long incl = c[h];
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const unsigned long long t = __shfl_up(incl, off, 64);
            if ((int)lane >= off) incl += t;
        }
        e[h] = incl - c[h];
        if (lane == 63)
#pragma unroll
            for (int q = 0; q < 4; ++q) wtot[wave][4 * h + q] = (uint32_t)(incl >> (16 * q)) & 0xFFFFu;
    }
    __syncthreads();
    if (threadIdx.x < kReplayFastBatches) {
        // thread b: batch b's start in the staging array (the totals of the batches before it) and each wave's start
        // inside the batch, the batch's global reservation
        const uint32_t b = threadIdx.x;
        uint32_t before = 0, t = 0;
#pragma unroll 1
        for (int w = 0; w < kWG / 64; ++w) {  // (rolled: 64 LDS words in flight would hold 64 registers)
            wpos[w][b] = t;  // the wave's start inside the batch, made absolute below
#pragma unroll
            for (uint32_t q = 0; q < kReplayFastBatches; ++q) {
                const uint32_t x = wtot[w][q];
                before += q < b ? x : 0u;
                t += q == b ? x : 0u;
            }
        }
#if ESGPU_RC_EXP == 2
        const uint32_t g = blockIdx.x * 2048u;
#else
        const uint32_t g = b < P.nbatch && t ? atomicAdd(&P.fill[(size_t)b * kReplayFillStride], t) : 0u;
#endif
        const uint32_t cap = b < P.nbatch ? P.cap[b] : 0u;
        gdst[b] = (b < P.nbatch ? P.region[b] : 0ull) + g;  // where the batch's run goes, and how much of it fits
        glim[b] = cap > g ? cap - g : 0u;
        boff[b] = before;
        if (b == kReplayFastBatches - 1) boff[kReplayFastBatches] = before + t;
#pragma unroll
        for (int w = 0; w < kWG / 64; ++w) wpos[w][b] += before;
    }
    __syncthreads();
    // stage: the thread's docs in order, each at its wave's start + the lanes before it + its rank among the thread's
    // docs of its batch (the running count, rebuilt)
    unsigned long long r[2] = {e[0], e[1]};
#pragma unroll
    for (int k = 0; k < kItersPerBlock * 4; ++k) {
        const uint32_t b = (uint32_t)(bits >> (4 * k)) & 15u;
        if (b >= kReplayFastBatches) continue;
        const unsigned long long rh = b < 4u ? r[0] : r[1];
        const uint32_t sh = 16u * (b & 3u);
        stage[wpos[wave][b] + ((uint32_t)(rh >> sh) & 0xFFFFu)] = val[k / 4][k % 4];
        if (b < 4u) r[0] += 1ull << sh; else r[1] += 1ull << sh;
    }
    __syncthreads();
    const uint32_t total = ESGPU_RC_EXP == 1 ? 0u : boff[kReplayFastBatches];
    if (ESGPU_RC_EXP == 1 && threadIdx.x == 0 && stage[boff[1]] == 0x12345u) *P.overflow = 1u;
    for (uint32_t i = threadIdx.x; i < total; i += kWG) {
        uint32_t b = 0;
#pragma unroll
        for (uint32_t q = 1; q < kReplayFastBatches; ++q) b += i >= boff[q] ? 1u : 0u;
        const uint32_t k = i - boff[b];
        if (k < glim[b]) P.out[gdst[b] + k] = stage[i];
        else *P.overflow = 1u;
    }
}

// more batches: a position per wave round of each distinct batch, scattered appends
__global__ __launch_bounds__(kWG) void replay_compact_kernel(ReplayCompactParams P) {
    __shared__ uint32_t cnt[kReplayMaxBatches], base[kReplayMaxBatches];
    const uint32_t lane = threadIdx.x & 63;
    uint32_t val[kItersPerBlock][4], bid[kItersPerBlock][4];
    replay_classify(P, P.slot_map, val, bid);
    for (uint32_t i = threadIdx.x; i < P.nbatch; i += kWG) cnt[i] = 0;
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t pos[kItersPerBlock][4];
#pragma unroll
    for (int it = 0; it < kItersPerBlock; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t mine = bid[it][j];
            uint64_t todo = __ballot(mine != kMissingOrd);
            uint32_t p = 0;
            while (todo) {  // one round per distinct batch among the wave's live lanes
                const int leader = __ffsll((unsigned long long)todo) - 1;
                const uint32_t bl = __shfl(mine, leader, 64);
                const uint64_t same = __ballot(mine == bl);
                uint32_t b0 = 0;
                if ((int)lane == leader) b0 = atomicAdd(&cnt[bl], (uint32_t)__popcll(same));
                b0 = __shfl(b0, leader, 64);
                if (mine == bl) p = b0 + (uint32_t)__popcll(same & lt);
                todo &= ~same;
            }
            pos[it][j] = p;
        }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < P.nbatch; i += kWG)
        base[i] = cnt[i] ? atomicAdd(&P.fill[(size_t)i * kReplayFillStride], cnt[i]) : 0u;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kItersPerBlock; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t bb = bid[it][j];
            if (bb == kMissingOrd) continue;
            const uint32_t q = base[bb] + pos[it][j];
            if (q < P.cap[bb]) P.out[P.region[bb] + q] = val[it][j];
            else *P.overflow = 1u;
        }
}
void launch_replay_compact(const ReplayCompactParams& p, hipStream_t st) {
    const uint32_t blocks = (p.n_docs + kBlockDocs - 1) / kBlockDocs;
    if (!blocks) return;
    if (p.nbatch <= kReplayFastBatches) hipLaunchKernelGGL(replay_compact_sort_kernel, dim3(blocks), dim3(kWG), 0, st, p);
    else hipLaunchKernelGGL(replay_compact_kernel, dim3(blocks), dim3(kWG), 0, st, p);
}

void launch_minmax_i64(const int64_t* v, uint64_t n, int64_t* out, bool f64, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(minmax_i64_kernel, dim3((uint32_t)std::min<uint64_t>(1024, (n + 255) / 256)), dim3(256), 0, st, v, n, out,
                       f64 ? 1 : 0);
}

}  // namespace esgpu
