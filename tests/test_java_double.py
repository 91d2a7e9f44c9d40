"""Double.toString of the reference's JVM (Java 8 FloatingDecimal) -- the digits of every double in the XContent
rendering (esgpu_result_to_xcontent, esgpu_java_double) -- against the oracle's independent Python restatement
(oracle/java_double.py) and known answers.

Known answers: Java 8 prints some doubles with more digits than the shortest round trip, because its digit loop stops
on a strict half-ULP test, prints integers below 2^63 digit for digit, and forces two digits in E-form.  The values below
are the documented anomalies of that algorithm (OpenJDK JDK-4511638, fixed only in JDK 19), plus the layout examples of
Double.toString's specification.  No JVM is available here to generate more: the remaining cases are "parity pinned
to the restatement" (two independent implementations of the published algorithm agree)."""
import ctypes
import math
import struct

import numpy as np
import pytest

from elasticsearch_amd import _native as N
from java_double import java_double_to_string

KATS = [
    # JDK-4511638 anomalies (Java <= 18): more digits than the shortest round trip
    (2e23, "1.9999999999999998E23"), (1e23, "9.999999999999999E22"), (8.41e21, "8.409999999999999E21"),
    (2.82879384806159e17, "2.82879384806159008E17"),
    # Double.toString layout: plain decimal for 1e-3 <= |v| < 1e7, d.dddE<n> otherwise, at least one fraction digit
    (1.0, "1.0"), (100.0, "100.0"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1e7, "1.0E7"), (9999999.0, "9999999.0"),
    (12345678.9, "1.23456789E7"), (-0.0, "-0.0"), (4.9e-324, "4.9E-324"), (1.7976931348623157e308, "1.7976931348623157E308"),
    (float("nan"), "NaN"), (float("inf"), "Infinity"), (float("-inf"), "-Infinity"), (0.1, "0.1"), (5.5, "5.5"),
    (2.2250738585072014e-308, "2.2250738585072014E-308"),
]


def product(v):
    buf = ctypes.create_string_buffer(32)
    N.check(N.lib().esgpu_java_double(v, buf, 32))
    return buf.value.decode()


@pytest.mark.parametrize("v, java", KATS)
def test_known_answers(v, java):
    assert java_double_to_string(v) == java, "oracle"
    assert product(v) == java, "product"


def _sample():
    rng = np.random.default_rng(20261017)
    vals = list(rng.integers(0, 1 << 64, 6000, dtype=np.uint64).view(np.float64))  # every exponent
    vals += list(rng.integers(1, 10**6, 3000) / rng.integers(1, 10**4, 3000))   # averages of integer metrics
    vals += list(rng.random(2000) * 10.0 ** rng.integers(-12, 25, 2000))        # decades around both layouts
    vals += [float(k) * 10.0**e for k in (1, 2, 3, 5, 7, 9) for e in range(-30, 31)]  # decimal midpoints
    vals += [math.ldexp(1.0, e) for e in range(-1074, 1024, 7)]                  # powers of two (asymmetric ULP)
    vals += list(rng.integers(1, 1 << 62, 2000).astype(np.float64))             # integers (developLongDigits)
    return [float(v) for v in vals]


def test_product_matches_the_oracle_restatement():
    bad = []
    for v in _sample():
        a, b = product(v), java_double_to_string(v)
        if a != b:
            bad.append((v.hex(), a, b))
    assert not bad, bad[:10]


def test_output_reads_back_as_the_same_double():
    """Double.toString's contract (and Double.parseDouble reading it back) holds for every sampled value."""
    for v in _sample():
        if math.isfinite(v):
            assert float(product(v)) == v, v.hex()
