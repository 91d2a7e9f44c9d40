// java_double.hpp — Double.toString(double) exactly as the reference's JVM prints it.
//
// The reference is built for Java 1.8 (pom.xml:40-41), whose Double.toString is sun.misc.FloatingDecimal
// (OpenJDK 8: BinaryToASCIIBuffer.dtoa + getChars, getBinaryToASCIIConverter, estimateDecExp, developLongDigits,
// roundup, insignificantDigitsForPow2).  The JDK is a dependency absent from /root/reference; this restates its
// published algorithm.  It is NOT the shortest round-trip conversion (JDK 19+): it stops generating digits by a
// symmetric, strict test against half an ULP, prints integers below 2^63 digit for digit, and forces two digits in
// E-form, so it sometimes emits more digits than needed (2e23 -> "1.9999999999999998E23", 8.41e21 ->
// "8.409999999999999E21", 2.82879384806159e17 -> "2.82879384806159008E17").  Those digit strings are what an
// Elasticsearch 2.x node writes into a search response, so the XContent rendering reproduces them.
//
// Arithmetic follows the three paths of dtoa: Java int (32-bit, wrapping) and long (64-bit, wrapping) when the scaled
// values fit, otherwise exact big integers.  The wrapping of the int / long paths is kept (the m > 0 overflow test).
#pragma once

#include <stdint.h>

#include <cstring>
#include <string>
#include <vector>

namespace esgpu {
namespace jfd {

constexpr int kExpShift = 52;
constexpr uint64_t kFractHob = 1ull << kExpShift;
constexpr uint64_t kSignifMask = kFractHob - 1;
constexpr int kMaxSmallBinExp = 62;
constexpr int kMinSmallBinExp = -(63 / 3);

inline uint64_t pow5(int i) {  // FDBigInteger.LONG_5_POW / SMALL_5_POW (i <= 26)
    uint64_t v = 1;
    for (int k = 0; k < i; ++k) v *= 5;
    return v;
}
inline int n5bits(int i) {  // N_5_BITS: bit length of 5^i (0 for i == 0)
    if (i == 0) return 0;
    const uint64_t v = pow5(i);
    return 64 - __builtin_clzll(v);
}
inline int insignificant_digits_pow2(int p2) {  // insignificantDigitsForPow2: digits of 2^p2 minus one, for 1 < p2 < 64
    if (p2 <= 1 || p2 >= 64) return 0;
    uint64_t v = 1ull << p2;
    int i = 0;
    while (v >= 10) { v /= 10; ++i; }
    return i;
}
inline int32_t wrap32(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }
inline int64_t wrap64(unsigned __int128 v) { return (int64_t)(uint64_t)v; }

// minimal unsigned big integer (little-endian 32-bit limbs) for the FDBigInteger path
struct Big {
    std::vector<uint32_t> d;
    static Big of(uint64_t v) { Big b; while (v) { b.d.push_back((uint32_t)v); v >>= 32; } return b; }
    void trim() { while (!d.empty() && d.back() == 0) d.pop_back(); }
    void mul_small(uint32_t m) {
        uint64_t c = 0;
        for (uint32_t& x : d) { const uint64_t t = (uint64_t)x * m + c; x = (uint32_t)t; c = t >> 32; }
        if (c) d.push_back((uint32_t)c);
    }
    void shl(int n) {
        if (d.empty() || n == 0) return;
        const int w = n / 32, b = n % 32;
        std::vector<uint32_t> r(d.size() + w + 1, 0);
        for (size_t i = 0; i < d.size(); ++i) {
            r[i + w] |= d[i] << b;
            if (b) r[i + w + 1] |= d[i] >> (32 - b);
        }
        d.swap(r);
        trim();
    }
    static Big pow52(int p5, int p2, uint64_t mul = 1) {  // mul * 5^p5 * 2^p2
        Big b = of(mul);
        for (int k = 0; k < p5; ++k) b.mul_small(5);
        b.shl(p2);
        return b;
    }
    static int cmp(const Big& a, const Big& b) {
        if (a.d.size() != b.d.size()) return a.d.size() < b.d.size() ? -1 : 1;
        for (size_t i = a.d.size(); i-- > 0;)
            if (a.d[i] != b.d[i]) return a.d[i] < b.d[i] ? -1 : 1;
        return 0;
    }
    void sub(const Big& o) {  // *this >= o
        int64_t br = 0;
        for (size_t i = 0; i < d.size(); ++i) {
            int64_t t = (int64_t)d[i] - br - (i < o.d.size() ? (int64_t)o.d[i] : 0);
            br = t < 0;
            d[i] = (uint32_t)(t + (br << 32));
        }
        trim();
    }
    static Big add(const Big& a, const Big& b) {
        Big r;
        uint64_t c = 0;
        for (size_t i = 0; i < std::max(a.d.size(), b.d.size()); ++i) {
            const uint64_t t = (uint64_t)(i < a.d.size() ? a.d[i] : 0) + (i < b.d.size() ? b.d[i] : 0) + c;
            r.d.push_back((uint32_t)t);
            c = t >> 32;
        }
        if (c) r.d.push_back((uint32_t)c);
        return r;
    }
    bool zero() const { return d.empty(); }
    int quo_rem10(const Big& s) {  // FDBigInteger.quoRemIteration: q = this / s, this = (this % s) * 10
        int q = 0;
        while (cmp(*this, s) >= 0) { sub(s); ++q; }
        mul_small(10);
        return q;
    }
};

struct Digits {
    char dig[24];
    int first = 0, n = 0, dec_exp = 0;
    void roundup() {  // BinaryToASCIIBuffer.roundup
        int i = first + n - 1;
        char q = dig[i];
        if (q == '9') {
            while (q == '9' && i > first) { dig[i] = '0'; q = dig[--i]; }
            if (q == '9') { dec_exp += 1; dig[first] = '1'; return; }
        }
        dig[i] = (char)(q + 1);
    }
    void develop_long(int dexp, int64_t lvalue, int insignificant) {  // developLongDigits
        if (insignificant != 0) {
            const int64_t pow10 = (int64_t)(pow5(insignificant) << insignificant);
            const int64_t residue = lvalue % pow10;
            lvalue /= pow10;
            dexp += insignificant;
            if (residue >= (pow10 >> 1)) lvalue++;
        }
        int digitno = 23;
        int64_t v = lvalue;
        int c = (int)(v % 10);
        v /= 10;
        while (c == 0) { dexp++; c = (int)(v % 10); v /= 10; }
        while (v != 0) { dig[digitno--] = (char)(c + '0'); dexp++; c = (int)(v % 10); v /= 10; }
        dig[digitno] = (char)(c + '0');
        dec_exp = dexp + 1;
        first = digitno;
        n = 24 - digitno;
    }
};

inline int estimate_dec_exp(uint64_t fract, int bin_exp) {  // estimateDecExp (floor of the log10 estimate)
    const uint64_t bits = 0x3FF0000000000000ull | (fract & kSignifMask);
    double d2;
    std::memcpy(&d2, &bits, 8);
    const double d = (d2 - 1.5) * 0.289529654 + 0.176091259 + (double)bin_exp * 0.301029995663981;
    double f = (double)(int64_t)d;
    if (f > d) f -= 1.0;
    return (int)f;
}

// BinaryToASCIIBuffer.dtoa(binExp, fractBits, nSignificantBits, isCompatibleFormat = true)
inline void dtoa(int bin_exp, uint64_t fract, int nsig, Digits& o) {
    const int tail = __builtin_ctzll(fract);
    const int nfract = kExpShift + 1 - tail;
    int ntiny = std::max(0, nfract - bin_exp - 1);
    if (bin_exp <= kMaxSmallBinExp && bin_exp >= kMinSmallBinExp) {
        if (ntiny < 27 && nfract + n5bits(ntiny) < 64 && ntiny == 0) {
            const int insig = bin_exp > nsig ? insignificant_digits_pow2(bin_exp - nsig - 1) : 0;
            if (bin_exp >= kExpShift) fract <<= (bin_exp - kExpShift);
            else fract >>= (kExpShift - bin_exp);
            o.develop_long(0, (int64_t)fract, insig);
            return;
        }
    }
    int dec_exp = estimate_dec_exp(fract, bin_exp);
    int B5 = std::max(0, -dec_exp);
    int B2 = B5 + ntiny + bin_exp;
    int S5 = std::max(0, dec_exp);
    int S2 = S5 + ntiny;
    int M5 = B5;
    int M2 = B2 - nsig;
    fract >>= tail;
    B2 -= nfract - 1;
    const int common2 = std::min(B2, S2);
    B2 -= common2;
    S2 -= common2;
    M2 -= common2;
    if (nfract == 1) M2 -= 1;  // exact power of two
    if (M2 < 0) { B2 -= M2; S2 -= M2; M2 = 0; }
    int nd = 0;
    bool low, high;
    int64_t low_diff = 0;
    const int Bbits = nfract + B2 + (B5 < 27 ? n5bits(B5) : B5 * 3);
    const int tenSbits = S2 + 1 + ((S5 + 1) < 27 ? n5bits(S5 + 1) : (S5 + 1) * 3);
    auto e_form = [&] { return dec_exp < -3 || dec_exp >= 8; };
    if (Bbits < 64 && tenSbits < 64) {
        if (Bbits < 32 && tenSbits < 32) {  // Java int arithmetic (wrapping)
            int32_t b = wrap32((int64_t)(int32_t)(uint32_t)fract * (int64_t)pow5(B5));
            b = wrap32((int64_t)((uint64_t)(uint32_t)b << B2));
            const int32_t s = wrap32((int64_t)(pow5(S5) << S2));
            int32_t m = wrap32((int64_t)(pow5(M5) << M2));
            const int32_t tens = wrap32((int64_t)s * 10);
            int q = b / s;
            b = wrap32((int64_t)10 * (b % s));
            m = wrap32((int64_t)m * 10);
            low = b < m;
            high = wrap32((int64_t)b + m) > tens;
            if (q == 0 && !high) dec_exp--;
            else o.dig[nd++] = (char)('0' + q);
            if (e_form()) high = low = false;
            while (!low && !high) {
                q = b / s;
                b = wrap32((int64_t)10 * (b % s));
                m = wrap32((int64_t)m * 10);
                if (m > 0) {
                    low = b < m;
                    high = wrap32((int64_t)b + m) > tens;
                } else {
                    low = high = true;
                }
                o.dig[nd++] = (char)('0' + q);
            }
            low_diff = (int64_t)wrap32((int64_t)((uint32_t)b << 1) - tens);
        } else {  // Java long arithmetic (wrapping)
            int64_t b = wrap64((unsigned __int128)fract * pow5(B5));
            b = (int64_t)((uint64_t)b << B2);
            const int64_t s = (int64_t)(pow5(S5) << S2);
            int64_t m = (int64_t)(pow5(M5) << M2);
            const int64_t tens = wrap64((unsigned __int128)(uint64_t)s * 10);
            int q = (int)(b / s);
            b = wrap64((unsigned __int128)(uint64_t)(b % s) * 10);
            m = wrap64((unsigned __int128)(uint64_t)m * 10);
            low = b < m;
            high = (int64_t)((uint64_t)b + (uint64_t)m) > tens;
            if (q == 0 && !high) dec_exp--;
            else o.dig[nd++] = (char)('0' + q);
            if (e_form()) high = low = false;
            while (!low && !high) {
                q = (int)(b / s);
                b = wrap64((unsigned __int128)(uint64_t)(b % s) * 10);
                m = wrap64((unsigned __int128)(uint64_t)m * 10);
                if (m > 0) {
                    low = b < m;
                    high = (int64_t)((uint64_t)b + (uint64_t)m) > tens;
                } else {
                    low = high = true;
                }
                o.dig[nd++] = (char)('0' + q);
            }
            low_diff = (int64_t)(((uint64_t)b << 1) - (uint64_t)tens);
        }
    } else {  // FDBigInteger arithmetic (exact; the normalisation shift scales B, S, M alike and changes nothing)
        const Big S = Big::pow52(S5, S2);
        Big B = Big::pow52(B5, B2, fract);
        Big M = Big::pow52(M5 + 1, M2 + 1);
        const Big tenS = Big::pow52(S5 + 1, S2 + 1);
        int q = B.quo_rem10(S);
        low = Big::cmp(B, M) < 0;
        high = Big::cmp(Big::add(B, M), tenS) > 0;
        if (q == 0 && !high) dec_exp--;
        else o.dig[nd++] = (char)('0' + q);
        if (e_form()) high = low = false;
        while (!low && !high) {
            q = B.quo_rem10(S);
            M.mul_small(10);
            low = Big::cmp(B, M) < 0;
            high = Big::cmp(Big::add(B, M), tenS) > 0;
            o.dig[nd++] = (char)('0' + q);
        }
        if (high && low) {
            B.shl(1);
            low_diff = Big::cmp(B, tenS);
        }
    }
    o.dec_exp = dec_exp + 1;
    o.first = 0;
    o.n = nd;
    if (high) {
        if (low) {
            if (low_diff == 0) {
                if ((o.dig[o.first + o.n - 1] & 1) != 0) o.roundup();
            } else if (low_diff > 0) {
                o.roundup();
            }
        } else {
            o.roundup();
        }
    }
}

}  // namespace jfd

// Double.toString(v) (FloatingDecimal.toJavaFormatString: getBinaryToASCIIConverter + getChars)
inline std::string java_double(double v) {
    uint64_t bits;
    std::memcpy(&bits, &v, 8);
    const bool neg = (bits >> 63) != 0;
    uint64_t fract = bits & jfd::kSignifMask;
    int bin_exp = (int)((bits >> jfd::kExpShift) & 0x7FF);
    if (bin_exp == 0x7FF) return fract ? "NaN" : (neg ? "-Infinity" : "Infinity");
    int nsig;
    if (bin_exp == 0) {
        if (fract == 0) return neg ? "-0.0" : "0.0";
        const int lz = __builtin_clzll(fract);
        const int shift = lz - (63 - jfd::kExpShift);
        fract <<= shift;
        bin_exp = 1 - shift;
        nsig = 64 - lz;
    } else {
        fract |= jfd::kFractHob;
        nsig = jfd::kExpShift + 1;
    }
    bin_exp -= 1023;
    jfd::Digits d;
    jfd::dtoa(bin_exp, fract, nsig, d);
    std::string out = neg ? "-" : "";
    const char* dig = d.dig + d.first;
    const int n = d.n, e = d.dec_exp;
    if (e > 0 && e < 8) {
        const int cl = std::min(n, e);
        out.append(dig, cl);
        if (cl < e) {
            out.append((size_t)(e - cl), '0');
            out += ".0";
        } else {
            out += '.';
            if (cl < n) out.append(dig + cl, n - cl);
            else out += '0';
        }
    } else if (e <= 0 && e > -3) {
        out += "0.";
        out.append((size_t)(-e), '0');
        out.append(dig, n);
    } else {
        out += dig[0];
        out += '.';
        if (n > 1) out.append(dig + 1, n - 1);
        else out += '0';
        out += 'E';
        int x;
        if (e <= 0) { out += '-'; x = -e + 1; }
        else x = e - 1;
        out += std::to_string(x);
    }
    return out;
}

}  // namespace esgpu
