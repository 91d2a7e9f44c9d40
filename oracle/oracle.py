"""ctypes wrapper of the CPU oracle (oracle/libesoracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module - as the checker or
the timed CPU baseline, never as part of the product path.  See oracle/cpu_ref.cpp for what it restates.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(_HERE))
sys.path.insert(0, _HERE)

from elasticsearch_amd import _native as N  # noqa: E402  (struct layouts of include/esgpu.h)

import oracle_request  # noqa: E402  (the oracle's own request lowering: no product code)

LIB_PATH = os.path.join(_HERE, "libesoracle.so")


class OracleShard(ctypes.Structure):
    _fields_ = [("cols", ctypes.POINTER(N.ColumnDesc)), ("ncols", ctypes.c_int32), ("max_doc", ctypes.c_uint32),
                ("accept_bits", ctypes.c_void_p)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_run.restype = ctypes.c_int
        L.oracle_run.argtypes = [ctypes.POINTER(OracleShard), ctypes.c_int32, ctypes.POINTER(N.AggSpec), ctypes.c_int32,
                                 ctypes.POINTER(N.Filter), ctypes.c_int32, ctypes.POINTER(ctypes.c_char_p),
                                 ctypes.POINTER(ctypes.c_double)]
        L.oracle_free.argtypes = [ctypes.c_char_p]
        L.oracle_set_emit_streams.argtypes = [ctypes.c_int32]
        L.oracle_set_exact_shadow.argtypes = [ctypes.c_int32]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_murmur3_128.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_mix64.restype = ctypes.c_uint64
        L.oracle_mix64.argtypes = [ctypes.c_uint64]
        L.oracle_precision_from_threshold.restype = ctypes.c_int32
        L.oracle_precision_from_threshold.argtypes = [ctypes.c_int64]
        L.oracle_encode_hash.restype = ctypes.c_int32
        L.oracle_encode_hash.argtypes = [ctypes.c_uint64, ctypes.c_int32]
        L.oracle_decode_run_len.restype = ctypes.c_int32
        L.oracle_decode_run_len.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.oracle_decode_index.restype = ctypes.c_int32
        L.oracle_decode_index.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.oracle_index.restype = ctypes.c_int64
        L.oracle_index.argtypes = [ctypes.c_uint64, ctypes.c_int32]
        L.oracle_run_len.restype = ctypes.c_int32
        L.oracle_run_len.argtypes = [ctypes.c_uint64, ctypes.c_int32]
        L.oracle_rounding.restype = ctypes.c_int64
        L.oracle_rounding.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_int64]
        L.oracle_rounding_tz.restype = ctypes.c_int64
        L.oracle_rounding_tz.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int64]
        L.oracle_hll_collect.restype = ctypes.c_int64
        L.oracle_hll_collect.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint64)]
        _lib = L
    return _lib


def _columns(columns):
    """Same column dict format as elasticsearch_amd.Engine.upload_segment."""
    descs, keep = [], []
    for name, c in columns.items():
        d = N.ColumnDesc()
        b = name.encode()
        keep.append(b)
        d.name = b
        d.type = c["type"]
        dtype = {N.COL_ORD_U32: np.uint32, N.COL_I64: np.int64, N.COL_F64: np.float64, N.COL_U64: np.uint64}[c["type"]]
        vals = np.ascontiguousarray(c["values"], dtype=dtype)
        keep.append(vals)
        d.values = vals.ctypes.data if vals.size else None
        if c.get("offsets") is not None:
            o = np.ascontiguousarray(c["offsets"], dtype=np.uint64)
            keep.append(o)
            d.offsets = o.ctypes.data
        if c.get("present") is not None:
            p = np.ascontiguousarray(c["present"], dtype=np.uint64)
            keep.append(p)
            d.present = p.ctypes.data
        terms = c.get("terms")
        if c.get("terms_blob") is not None:
            blob, offs = c["terms_blob"]
            blob = np.ascontiguousarray(blob, dtype=np.uint8)
            offs = np.ascontiguousarray(offs, dtype=np.uint64)
            keep += [blob, offs]
            d.dict_bytes = blob.ctypes.data
            d.dict_offsets = offs.ctypes.data
            d.value_count = len(offs) - 1
        elif terms is not None:
            tb = [t.encode() if isinstance(t, str) else bytes(t) for t in terms]
            blob = np.frombuffer(b"".join(tb) or b"\0", dtype=np.uint8).copy()
            offs = np.zeros(len(tb) + 1, dtype=np.uint64)
            if tb:
                offs[1:] = np.cumsum([len(t) for t in tb])
            keep += [blob, offs]
            d.dict_bytes = blob.ctypes.data
            d.dict_offsets = offs.ctypes.data
            d.value_count = len(tb)
        else:
            d.value_count = int(c.get("value_count", 0))
        descs.append(d)
    arr = (N.ColumnDesc * max(len(descs), 1))(*descs)
    return arr, len(descs), keep


# oracle runs carry the exact-sum shadow unless told otherwise (tests/conftest.py turns it on for the test session)
EXACT_DEFAULT = False


def run(shards, aggs, filters=None, number_of_shards=None, accept=None, ord_lookup=None, return_seconds=False,
        streams=False, exact=None):
    """shards: list of (columns_dict, max_doc).  Returns {"shards": [...], "reduced": {...}} (parsed JSON); with
    streams=True also "streams": per shard the bytes of InternalAggregations.writeTo; with exact=True every stats /
    extended_stats / avg result also carries "_exact": its rendered values recomputed from the exact sums that the
    reference's doc-order double additions approximate (tests/helpers.assert_same_exact)."""
    L = lib()
    L.oracle_set_emit_streams(1 if streams else 0)
    L.oracle_set_exact_shadow(1 if (EXACT_DEFAULT if exact is None else exact) else 0)
    number_of_shards = number_of_shards or len(shards)
    specs, nspecs, k1 = oracle_request.lower(L, aggs, number_of_shards)
    flt, nf, k2 = oracle_request.lower_filters(filters, ord_lookup, aggs)
    oshards, keep = [], [k1, k2]
    for i, (cols, max_doc) in enumerate(shards):
        arr, n, k = _columns(cols)
        keep += [arr, k]
        s = OracleShard()
        s.cols = arr
        s.ncols = n
        s.max_doc = max_doc
        if accept is not None and accept[i] is not None:
            a = np.ascontiguousarray(accept[i], dtype=np.uint64)
            keep.append(a)
            s.accept_bits = a.ctypes.data
        oshards.append(s)
    sarr = (OracleShard * max(len(oshards), 1))(*oshards)
    out = ctypes.c_char_p()
    secs = ctypes.c_double()
    rc = L.oracle_run(sarr, len(oshards), specs, nspecs, flt, nf, ctypes.byref(out), ctypes.byref(secs))
    L.oracle_set_exact_shadow(0)
    if rc != 0:
        raise RuntimeError("oracle: " + L.oracle_last_error().decode())
    res = json.loads(out.value.decode("utf-8"))
    L.oracle_free(out)
    L.oracle_set_emit_streams(0)
    if streams:
        res["streams"] = [bytes.fromhex(h) for h in res["streams"]]
    if return_seconds:
        return res, secs.value
    return res
