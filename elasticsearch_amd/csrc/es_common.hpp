// es_common.hpp — primitives shared by the gfx950 kernels and the host runtime of libesgpu.so.
//
// Everything here is __host__ __device__ so the synthetic shard generator produces identical values on
// the CPU (for the oracle / CPU baseline) and in HBM (for the GPU path).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define ES_HD __host__ __device__ __forceinline__

namespace esgpu {

constexpr uint32_t kMissingOrd = 0xFFFFFFFFu;
constexpr uint32_t kBlockDocs = 8192;  // zone-map granularity and the unit of work of one collect iteration set

// ---- hashing -------------------------------------------------------------------------------------------------
// hppc 0.7.1 BitMixer.mix64 (third-party; called at A/metrics/cardinality/CardinalityAggregator.java:368,392)
ES_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 32)) * 0x4cd6944c5cc20b6dULL;
    z = (z ^ (z >> 29)) * 0xfc12c5b19d3259e9ULL;
    return z ^ (z >> 32);
}

ES_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

ES_HD uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

// MurmurHash3_x64_128 as used by common/hash/MurmurHash3.java:62-157 (seed 0 for the murmur3 field and for
// string cardinality).  Writes h1/h2.
ES_HD void murmur3_x64_128(const uint8_t* key, int len, uint64_t seed, uint64_t* out_h1, uint64_t* out_h2) {
    const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    uint64_t h1 = seed, h2 = seed;
    const int nblocks = len / 16;
    for (int b = 0; b < nblocks; ++b) {
        uint64_t k1 = 0, k2 = 0;
        for (int i = 7; i >= 0; --i) k1 = (k1 << 8) | key[16 * b + i];
        for (int i = 7; i >= 0; --i) k2 = (k2 << 8) | key[16 * b + 8 + i];
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t* tail = key + 16 * nblocks;
    const int rem = len & 15;
    uint64_t k1 = 0, k2 = 0;
    for (int i = rem - 1; i >= 8; --i) k2 = (k2 << 8) | tail[i];
    if (rem > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
    for (int i = (rem < 8 ? rem : 8) - 1; i >= 0; --i) k1 = (k1 << 8) | tail[i];
    if (rem > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
    h1 ^= (uint64_t)(int64_t)len;
    h2 ^= (uint64_t)(int64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    *out_h1 = h1;
    *out_h2 = h2;
}

// MurmurHash3_x86_32 as Lucene's StringHelper.murmurhash3_x86_32 (third-party, Lucene 5.4; seed 0 for routing):
// little-endian 4-byte blocks, tail of 1-3 bytes, fmix32.  Murmur3HashFunction.hash(routing) feeds it the UTF-16LE
// bytes of the routing string (cluster/routing/Murmur3HashFunction.java:31-41).
ES_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
ES_HD uint32_t murmur3_x86_32(const uint8_t* data, int len, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h1 = seed;
    const int rounded = len & ~3;
    for (int i = 0; i < rounded; i += 4) {
        uint32_t k1 = (uint32_t)data[i] | ((uint32_t)data[i + 1] << 8) | ((uint32_t)data[i + 2] << 16) | ((uint32_t)data[i + 3] << 24);
        k1 *= c1;
        k1 = rotl32(k1, 15);
        k1 *= c2;
        h1 ^= k1;
        h1 = rotl32(h1, 13);
        h1 = h1 * 5 + 0xe6546b64u;
    }
    uint32_t k1 = 0;
    switch (len & 3) {
        case 3: k1 = (uint32_t)data[rounded + 2] << 16;  // fallthrough
        case 2: k1 |= (uint32_t)data[rounded + 1] << 8;  // fallthrough
        case 1:
            k1 |= data[rounded];
            k1 *= c1;
            k1 = rotl32(k1, 15);
            k1 *= c2;
            h1 ^= k1;
    }
    h1 ^= (uint32_t)len;
    h1 ^= h1 >> 16;
    h1 *= 0x85ebca6bu;
    h1 ^= h1 >> 13;
    h1 *= 0xc2b2ae35u;
    h1 ^= h1 >> 16;
    return h1;
}
// the same over the UTF-16LE bytes of n UTF-16 code units (a Java String's chars): two chars per 4-byte block
ES_HD uint32_t murmur3_x86_32_utf16(const uint16_t* c, int n, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h1 = seed;
    for (int i = 0; i + 1 < n; i += 2) {
        uint32_t k1 = (uint32_t)c[i] | ((uint32_t)c[i + 1] << 16);
        k1 *= c1;
        k1 = rotl32(k1, 15);
        k1 *= c2;
        h1 ^= k1;
        h1 = rotl32(h1, 13);
        h1 = h1 * 5 + 0xe6546b64u;
    }
    if (n & 1) {  // two tail bytes
        uint32_t k1 = c[n - 1];
        k1 *= c1;
        k1 = rotl32(k1, 15);
        k1 *= c2;
        h1 ^= k1;
    }
    h1 ^= (uint32_t)(2 * n);
    h1 ^= h1 >> 16;
    h1 *= 0x85ebca6bu;
    h1 ^= h1 >> 13;
    h1 *= 0xc2b2ae35u;
    h1 ^= h1 >> 16;
    return h1;
}
// OperationRouting.shardId for indices created on or after 2.0: MathUtils.mod(hash, numberOfShards)
ES_HD int32_t routing_shard(int32_t hash, int32_t nshards) {
    const int32_t r = hash % nshards;
    return r < 0 ? r + nshards : r;
}

// ---- HyperLogLog++ register math (A/metrics/cardinality/HyperLogLogPlusPlus.java:335-375) ----------------------
constexpr int kP2 = 25;
ES_HD int clz64(uint64_t x) {
#ifdef __HIP_DEVICE_COMPILE__
    return x == 0 ? 64 : __clzll((long long)x);
#else
    return x == 0 ? 64 : __builtin_clzll(x);
#endif
}
ES_HD uint32_t hll_index(uint64_t h, int p) { return (uint32_t)(h >> (64 - p)); }
ES_HD uint32_t hll_run_len(uint64_t h, int p) {
    const int z = clz64(h << p);
    return 1u + (uint32_t)(z < 64 - p ? z : 64 - p);
}
ES_HD uint32_t hll_encode(uint64_t h, int p) {
    const uint64_t e = h >> (64 - kP2);
    if ((e & ((1ULL << (kP2 - p)) - 1)) == 0) {
        const int z = clz64(h << kP2);
        const uint32_t rl = 1u + (uint32_t)(z < 64 - kP2 ? z : 64 - kP2);
        return (uint32_t)((e << 7) | ((uint64_t)rl << 1) | 1);
    }
    return (uint32_t)(e << 1);
}

// ---- order-preserving u64 encoding of doubles (Java Math.min/max semantics via integer atomics) ----------------
// enc(-0.0) < enc(+0.0); NaN is tracked separately: min slot gets 0, max slot gets ~0 (both outside the range
// of any non-NaN encoding), which decode_min/decode_max turn back into NaN.
ES_HD uint64_t dbl_bits(double x) {
    union { double d; uint64_t u; } c;
    c.d = x;
    return c.u;
}
ES_HD double bits_dbl(uint64_t u) {
    union { double d; uint64_t u; } c;
    c.u = u;
    return c.d;
}
ES_HD uint64_t sortable(double x) {
    const uint64_t b = dbl_bits(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
ES_HD double unsortable(uint64_t e) { return bits_dbl((e >> 63) ? (e & 0x7FFFFFFFFFFFFFFFULL) : ~e); }
constexpr uint64_t kEncNegInf = 0x000FFFFFFFFFFFFFULL;  // sortable(-inf)
constexpr uint64_t kEncPosInf = 0xFFF0000000000000ULL;  // sortable(+inf)
constexpr uint64_t kMinInit = ~0ULL;                     // "no value yet" for min (decodes to +inf)
constexpr uint64_t kMaxInit = 0ULL;                      // "no value yet" for max (decodes to -inf)

// ---- 32-bit unsigned division by a runtime-invariant divisor (Granlund–Montgomery "round-up + add") -----------
struct MagicU32 {
    uint32_t m;
    uint32_t s1, s2;
    uint32_t d;
};
inline MagicU32 make_magic(uint32_t d) {
    MagicU32 r;
    r.d = d;
    if (d == 1) { r.m = 0; r.s1 = 0; r.s2 = 0; return r; }
    int l = 0;
    while ((1ULL << l) < d) ++l;  // l = ceil(log2 d)
    const uint64_t m = ((1ULL << 32) * ((1ULL << l) - d)) / d + 1;
    r.m = (uint32_t)m;
    r.s1 = 1;
    r.s2 = (uint32_t)(l - 1);
    return r;
}
ES_HD uint32_t magic_div(uint32_t n, uint32_t m, uint32_t s1, uint32_t s2, uint32_t d) {
    if (d == 1) return n;
    const uint32_t t = (uint32_t)(((uint64_t)m * n) >> 32);
    return (t + ((n - t) >> s1)) >> s2;
}

// Java (long) of a double (FieldData.castToLong / JLS 5.1.3): NaN -> 0, saturating, truncation toward zero
ES_HD int64_t java_long(double v) {
    if (v != v) return 0;
    if (v >= 9.2233720368547758e18) return INT64_MAX;
    if (v <= -9.2233720368547758e18) return INT64_MIN;
    return (int64_t)v;
}

ES_HD int64_t floor_div64(int64_t a, int64_t b) {  // Rounding.Interval.roundKey (common/rounding/Rounding.java:92-98)
    return a < 0 ? (a - b + 1) / b : a / b;
}

// ---- synthetic log-style documents ------------------------------------------
constexpr uint64_t kSynthSeed = 0x5EEDE1A5ULL;
constexpr int64_t kSynthT0 = 1441065600000LL;  // 2015-09-01T00:00:00Z
constexpr int64_t kSynthSpan = 30LL * 86400000LL;
constexpr uint32_t kHostTerms = 1000;
constexpr uint32_t kUrlTerms = 10000000;
constexpr uint32_t kRtValues = 1000;

ES_HD uint64_t splitmix_at(uint64_t seed, uint64_t k) {  // the k-th output of a splitmix64 stream seeded at `seed`
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
ES_HD uint64_t shard_seed(uint64_t seed, uint32_t shard) { return seed ^ (0xA0761D6478BD642FULL * ((uint64_t)shard + 1)); }
ES_HD uint64_t synth_rand(uint64_t sseed, uint64_t doc, uint32_t field) { return splitmix_at(sseed, doc * 8 + field); }
ES_HD double unit_double(uint64_t r) { return (double)(r >> 11) * (1.0 / 9007199254740992.0); }

// first k with u < cdf[k] (cdf[n-1] == 1.0)
ES_HD uint32_t cdf_search(const double* cdf, uint32_t n, double u) {
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
}

enum SynthField : uint32_t { F_TS = 0, F_HOST = 1, F_URL = 2, F_STATUS = 3, F_RT = 4, F_BYTES = 5, F_IP = 6, F_PRICE = 7,
                              F_TS_JITTER = 8 };

// non-decreasing in doc order; jitter_ms > 0 displaces each doc by a uniform offset in [-jitter_ms, +jitter_ms] (docs
// roughly time-ordered, as merged segments are, instead of sorted)
ES_HD int64_t synth_timestamp(uint64_t sseed, uint64_t doc, uint64_t n, int64_t jitter_ms = 0) {
    const uint64_t base = (doc * (uint64_t)kSynthSpan) / n;
    const uint64_t next = ((doc + 1) * (uint64_t)kSynthSpan) / n;
    const uint64_t gap = next - base;
    const uint64_t r = synth_rand(sseed, doc, F_TS);
    int64_t t = kSynthT0 + (int64_t)(base + (gap ? r % gap : 0));
    if (jitter_ms > 0) t += (int64_t)(synth_rand(sseed, doc, F_TS_JITTER) % (uint64_t)(2 * jitter_ms + 1)) - jitter_ms;
    return t;
}
ES_HD uint32_t synth_host(uint64_t sseed, uint64_t doc, const double* cdf) {
    const uint32_t rank = cdf_search(cdf, kHostTerms, unit_double(synth_rand(sseed, doc, F_HOST)));
    return (rank * 619u + 17u) % kHostTerms;
}
ES_HD uint32_t synth_url(uint64_t sseed, uint64_t doc, const double* cdf) {
    const uint32_t rank = cdf_search(cdf, kUrlTerms, unit_double(synth_rand(sseed, doc, F_URL)));
    return (uint32_t)(((uint64_t)rank * 7919u + 12345u) % kUrlTerms);
}
ES_HD int64_t synth_status(uint64_t sseed, uint64_t doc) {
    const uint32_t r = (uint32_t)(synth_rand(sseed, doc, F_STATUS) % 1000u);
    // permille thresholds: 200:70% 304:10% 404:8% 301:4% 500:3% 302:2% 401:1% 403:1% 502:0.5% 503:0.5%
    if (r < 700) return 200;
    if (r < 800) return 304;
    if (r < 880) return 404;
    if (r < 920) return 301;
    if (r < 950) return 500;
    if (r < 970) return 302;
    if (r < 980) return 401;
    if (r < 990) return 403;
    if (r < 995) return 502;
    return 503;
}
ES_HD int64_t synth_rt(uint64_t sseed, uint64_t doc, const double* cdf) {
    return (int64_t)cdf_search(cdf, kRtValues, unit_double(synth_rand(sseed, doc, F_RT)));
}
ES_HD int64_t synth_bytes(uint64_t sseed, uint64_t doc) { return (int64_t)(synth_rand(sseed, doc, F_BYTES) % 1000000u); }
ES_HD double synth_price(uint64_t sseed, uint64_t doc) { return unit_double(synth_rand(sseed, doc, F_PRICE)) * 1000.0; }
ES_HD int synth_ip_string(uint64_t sseed, uint64_t doc, uint8_t* buf) {  // dotted quad from a 2^27 pool
    const uint32_t j = (uint32_t)(synth_rand(sseed, doc, F_IP) >> 37);
    const uint32_t oct[4] = {10u + (j >> 24), (j >> 16) & 255u, (j >> 8) & 255u, j & 255u};
    int n = 0;
    for (int o = 0; o < 4; ++o) {
        const uint32_t v = oct[o];
        if (v >= 100) buf[n++] = (uint8_t)('0' + v / 100);
        if (v >= 10) buf[n++] = (uint8_t)('0' + (v / 10) % 10);
        buf[n++] = (uint8_t)('0' + v % 10);
        if (o < 3) buf[n++] = '.';
    }
    return n;
}
ES_HD uint64_t synth_ip_hash(uint64_t sseed, uint64_t doc) {
    uint8_t buf[16];
    const int n = synth_ip_string(sseed, doc, buf);
    uint64_t h1, h2;
    murmur3_x64_128(buf, n, 0, &h1, &h2);
    return h1;  // Murmur3FieldMapper stores h1 (plugins/mapper-murmur3/.../Murmur3FieldMapper.java:160-162)
}

}  // namespace esgpu
