"""Double.toString(double) of Java 8 (sun.misc.FloatingDecimal) restated in Python.  TEST INFRASTRUCTURE ONLY.

The reference is built for Java 1.8 (/root/reference/pom.xml:40-41); every double of a search response's XContent is
printed by Jackson through Double.toString.  The JDK is a dependency absent from /root/reference, so this restates its
published algorithm (OpenJDK 8 FloatingDecimal: getBinaryToASCIIConverter, BinaryToASCIIBuffer.dtoa with its int, long
and FDBigInteger paths, estimateDecExp, developLongDigits, insignificantDigitsForPow2, roundup, getChars) on Python
integers, emulating Java's 32-bit / 64-bit wrap-around where dtoa relies on it.  Written independently of the product's
C++ (elasticsearch_amd/csrc/java_double.hpp): tests/test_java_double.py compares the two on KATs and random doubles.
Only tests/ import this module.
"""
import math
import struct

EXP_SHIFT = 52
FRACT_HOB = 1 << EXP_SHIFT
MAX_SMALL_BIN_EXP = 62
MIN_SMALL_BIN_EXP = -(63 // 3)
LONG_5_POW = [5 ** i for i in range(27)]
N_5_BITS = [0] + [(5 ** i).bit_length() for i in range(1, 27)]
INSIGNIFICANT = [0, 0] + [len(str(1 << p)) - 1 for p in range(2, 64)]


def _i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def _i64(v):
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= 1 << 63 else v


def _jdiv(a, b):  # Java integer division truncates toward zero
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _jmod(a, b):
    return a - _jdiv(a, b) * b


def _estimate_dec_exp(fract, bin_exp):
    d2 = struct.unpack("<d", struct.pack("<Q", 0x3FF0000000000000 | (fract & (FRACT_HOB - 1))))[0]
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + float(bin_exp) * 0.301029995663981
    return math.floor(d)


class _Buf:
    def __init__(self):
        self.digits = []
        self.dec_exponent = 0

    def roundup(self):
        i = len(self.digits) - 1
        q = self.digits[i]
        if q == 9:
            while q == 9 and i > 0:
                self.digits[i] = 0
                i -= 1
                q = self.digits[i]
            if q == 9:
                self.dec_exponent += 1
                self.digits[0] = 1
                return
        self.digits[i] = q + 1

    def develop_long(self, dec_exponent, lvalue, insignificant):
        if insignificant:
            pow10 = LONG_5_POW[insignificant] << insignificant
            residue = lvalue % pow10
            lvalue //= pow10
            dec_exponent += insignificant
            if residue >= pow10 >> 1:
                lvalue += 1
        s = str(lvalue)
        stripped = s.rstrip("0")
        dec_exponent += len(s) - 1  # one per digit after the first (trailing zeros included)
        self.digits = [int(c) for c in stripped]
        self.dec_exponent = dec_exponent + 1

    def dtoa(self, bin_exp, fract, nsig):
        tail = (fract & -fract).bit_length() - 1
        nfract = EXP_SHIFT + 1 - tail
        ntiny = max(0, nfract - bin_exp - 1)
        if MIN_SMALL_BIN_EXP <= bin_exp <= MAX_SMALL_BIN_EXP and ntiny < len(LONG_5_POW) and \
                nfract + N_5_BITS[ntiny] < 64 and ntiny == 0:
            insig = INSIGNIFICANT[bin_exp - nsig - 1] if bin_exp > nsig and 1 < bin_exp - nsig - 1 < 64 else 0
            lv = fract << (bin_exp - EXP_SHIFT) if bin_exp >= EXP_SHIFT else fract >> (EXP_SHIFT - bin_exp)
            self.develop_long(0, lv, insig)
            return
        dec_exp = _estimate_dec_exp(fract, bin_exp)
        b5 = max(0, -dec_exp)
        b2 = b5 + ntiny + bin_exp
        s5 = max(0, dec_exp)
        s2 = s5 + ntiny
        m5 = b5
        m2 = b2 - nsig
        fract >>= tail
        b2 -= nfract - 1
        common = min(b2, s2)
        b2 -= common
        s2 -= common
        m2 -= common
        if nfract == 1:
            m2 -= 1
        if m2 < 0:
            b2 -= m2
            s2 -= m2
            m2 = 0
        bbits = nfract + b2 + (N_5_BITS[b5] if b5 < len(N_5_BITS) else b5 * 3)
        tens_bits = s2 + 1 + (N_5_BITS[s5 + 1] if s5 + 1 < len(N_5_BITS) else (s5 + 1) * 3)
        digits = []
        low_diff = 0

        def e_form():
            return dec_exp < -3 or dec_exp >= 8

        if bbits < 64 and tens_bits < 64:
            wrap = _i32 if (bbits < 32 and tens_bits < 32) else _i64
            b = wrap(wrap(fract * LONG_5_POW[b5]) << b2)
            s = wrap(LONG_5_POW[s5] << s2)
            m = wrap(LONG_5_POW[m5] << m2)
            tens = wrap(s * 10)
            q = _jdiv(b, s)
            b = wrap(10 * _jmod(b, s))
            m = wrap(m * 10)
            low = b < m
            high = wrap(b + m) > tens
            if q == 0 and not high:
                dec_exp -= 1
            else:
                digits.append(q)
            if e_form():
                low = high = False
            while not low and not high:
                q = _jdiv(b, s)
                b = wrap(10 * _jmod(b, s))
                m = wrap(m * 10)
                if m > 0:
                    low = b < m
                    high = wrap(b + m) > tens
                else:
                    low = high = True
                digits.append(q)
            low_diff = wrap(wrap(b << 1) - tens)
        else:
            S = LONG_5_POW[0] * 5 ** s5 << s2
            B = fract * 5 ** b5 << b2
            M = 5 ** (m5 + 1) << (m2 + 1)
            tenS = 5 ** (s5 + 1) << (s2 + 1)
            q, B = B // S, (B % S) * 10
            low = B < M
            high = B + M > tenS
            if q == 0 and not high:
                dec_exp -= 1
            else:
                digits.append(q)
            if e_form():
                low = high = False
            while not low and not high:
                q, B = B // S, (B % S) * 10
                M *= 10
                low = B < M
                high = B + M > tenS
                digits.append(q)
            if high and low:
                low_diff = (B << 1) - tenS
        self.digits = digits
        self.dec_exponent = dec_exp + 1
        if high:
            if low:
                if low_diff == 0:
                    if digits[-1] & 1:
                        self.roundup()
                elif low_diff > 0:
                    self.roundup()
            else:
                self.roundup()


def java_double_to_string(v):
    bits = struct.unpack("<Q", struct.pack("<d", v))[0]
    neg = bits >> 63
    fract = bits & (FRACT_HOB - 1)
    bin_exp = (bits >> EXP_SHIFT) & 0x7FF
    if bin_exp == 0x7FF:
        return "NaN" if fract else ("-Infinity" if neg else "Infinity")
    if bin_exp == 0:
        if fract == 0:
            return "-0.0" if neg else "0.0"
        lz = 64 - fract.bit_length()
        shift = lz - (63 - EXP_SHIFT)
        fract <<= shift
        bin_exp = 1 - shift
        nsig = 64 - lz
    else:
        fract |= FRACT_HOB
        nsig = EXP_SHIFT + 1
    bin_exp -= 1023
    buf = _Buf()
    buf.dtoa(bin_exp, fract, nsig)
    d = "".join(str(x) for x in buf.digits)
    e = buf.dec_exponent
    out = "-" if neg else ""
    if 0 < e < 8:
        cl = min(len(d), e)
        out += d[:cl]
        if cl < e:
            out += "0" * (e - cl) + ".0"
        else:
            out += "." + (d[cl:] if cl < len(d) else "0")
    elif -3 < e <= 0:
        out += "0." + "0" * (-e) + d
    else:
        out += d[0] + "." + (d[1:] if len(d) > 1 else "0") + "E"
        out += ("-" + str(-e + 1)) if e <= 0 else str(e - 1)
    return out
