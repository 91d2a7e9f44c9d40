"""ctypes binding of libesgpu.so (include/esgpu.h).

The structures below mirror include/esgpu.h field for field.  The library is built in-tree
(elasticsearch_amd/libesgpu.so, see __graft_entry__.build()); importing this module fails loudly when it is
missing - there is no CPU fallback for the product path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ESGPU_LIBRARY selects an alternative build of the same library (kernel-variant experiments, tools/kbench.py)
LIB_PATH = os.environ.get("ESGPU_LIBRARY") or os.path.join(_HERE, "libesgpu.so")

# ---- constants (include/esgpu.h) ----
OK, ERR_INVALID, ERR_UNSUPPORTED, ERR_DEVICE, ERR_OOM, ERR_STATE, ERR_NO_DEVICE = range(7)
COL_ORD_U32, COL_I64, COL_F64, COL_U64 = 1, 2, 3, 4
SYNTH_TIMESTAMP, SYNTH_HOST, SYNTH_URL, SYNTH_STATUS = 1, 2, 4, 8
SYNTH_RESPONSE, SYNTH_BYTES, SYNTH_CLIENT_IP, SYNTH_PRICE = 16, 32, 64, 128
SYNTH_FIELDS = {
    "@timestamp": SYNTH_TIMESTAMP, "host": SYNTH_HOST, "url": SYNTH_URL, "status": SYNTH_STATUS,
    "response_time_ms": SYNTH_RESPONSE, "bytes": SYNTH_BYTES, "client_ip.hash": SYNTH_CLIENT_IP, "price": SYNTH_PRICE,
}
SYNTH_TYPES = {
    "@timestamp": COL_I64, "host": COL_ORD_U32, "url": COL_ORD_U32, "status": COL_I64,
    "response_time_ms": COL_I64, "bytes": COL_I64, "client_ip.hash": COL_U64, "price": COL_F64,
}
AGG_TERMS, AGG_HISTOGRAM, AGG_DATE_HISTOGRAM, AGG_STATS, AGG_EXTENDED_STATS, AGG_AVG, AGG_CARDINALITY = 1, 2, 3, 4, 5, 6, 7
AGG_SUM, AGG_MIN, AGG_MAX, AGG_VALUE_COUNT, AGG_FILTER = 8, 9, 10, 11, 12
ORDER_COUNT_DESC, ORDER_COUNT_ASC, ORDER_TERM_ASC, ORDER_TERM_DESC = 0, 1, 2, 3
ORDER_KEY_ASC, ORDER_KEY_DESC, ORDER_HCOUNT_ASC, ORDER_HCOUNT_DESC = 4, 5, 6, 7
ORDER_AGG_ASC, ORDER_AGG_DESC = 8, 9
FORMAT_RAW, FORMAT_DATE_TIME, FORMAT_NUMBER = 0, 1, 2
UNIT_NONE, UNIT_WEEK, UNIT_YEAR, UNIT_QUARTER, UNIT_MONTH, UNIT_DAY, UNIT_HOUR, UNIT_MINUTE, UNIT_SECOND = range(9)
FILTER_TERM, FILTER_RANGE = 1, 2
COMM_ID_BYTES = 128
DT_U8, DT_I64, DT_U64, DT_F64 = 0, 1, 2, 3
RED_SUM, RED_MIN, RED_MAX = 0, 1, 2


class ColumnDesc(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char_p), ("type", ctypes.c_int32), ("reserved", ctypes.c_int32),
        ("values", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("present", ctypes.c_void_p),
        ("dict_bytes", ctypes.c_void_p), ("dict_offsets", ctypes.c_void_p), ("value_count", ctypes.c_uint64),
    ]


class AggSpec(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int32), ("parent", ctypes.c_int32), ("name", ctypes.c_char_p), ("field", ctypes.c_char_p),
        ("size", ctypes.c_int32), ("shard_size", ctypes.c_int32), ("min_doc_count", ctypes.c_int64),
        ("shard_min_doc_count", ctypes.c_int64), ("order", ctypes.c_int32), ("show_term_doc_count_error", ctypes.c_int32),
        ("date_unit", ctypes.c_int32), ("keyed", ctypes.c_int32), ("interval", ctypes.c_int64), ("offset", ctypes.c_int64),
        ("has_extended_bounds_min", ctypes.c_int32), ("has_extended_bounds_max", ctypes.c_int32),
        ("extended_bounds_min", ctypes.c_int64), ("extended_bounds_max", ctypes.c_int64),
        ("sigma", ctypes.c_double), ("precision_threshold", ctypes.c_int64),
        ("tz_starts", ctypes.POINTER(ctypes.c_int64)), ("tz_offsets_ms", ctypes.POINTER(ctypes.c_int64)),
        ("tz_count", ctypes.c_int32), ("reserved_tz", ctypes.c_int32), ("order_path", ctypes.c_char_p),
        ("time_zone", ctypes.c_char_p), ("value_format", ctypes.c_int32), ("reserved_fmt", ctypes.c_int32),
        ("format", ctypes.c_char_p),
    ]


class Filter(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int32), ("include_lower", ctypes.c_int32), ("include_upper", ctypes.c_int32),
        ("has_lower", ctypes.c_int32), ("has_upper", ctypes.c_int32), ("owner", ctypes.c_int32),
        ("field", ctypes.c_char_p), ("term", ctypes.c_int64), ("lo_i", ctypes.c_int64), ("hi_i", ctypes.c_int64),
        ("lo_d", ctypes.c_double), ("hi_d", ctypes.c_double),
        ("lo_term", ctypes.c_char_p), ("hi_term", ctypes.c_char_p), ("lo_term_len", ctypes.c_uint64),
        ("hi_term_len", ctypes.c_uint64),
    ]


class AggBlock(ctypes.Structure):
    """esgpu_agg_block: one aggregation spec for n_instances parent buckets, columnar (include/esgpu.h)."""


_I32, _I64, _U64, _F64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
AggBlock._fields_ = [
    ("type", _I32), ("order", _I32), ("name", ctypes.c_char_p),
    ("required_size", _I32), ("shard_size", _I32), ("min_doc_count", _I64),
    ("show_term_doc_count_error", _I32), ("keyed", _I32),
    ("has_empty_bucket_info", _I32), ("date_unit", _I32), ("interval", _I64), ("offset", _I64),
    ("has_extended_bounds_min", _I32), ("has_extended_bounds_max", _I32),
    ("extended_bounds_min", _I64), ("extended_bounds_max", _I64),
    ("sigma", _F64), ("precision", _I32), ("nsubs", _I32), ("n_instances", _U64),
    ("doc_count_error", ctypes.POINTER(_I64)), ("other_doc_count", ctypes.POINTER(_I64)),
    ("bucket_offsets", ctypes.POINTER(_U64)), ("n_buckets", _U64),
    ("keys", ctypes.POINTER(_I64)), ("term_offsets", ctypes.POINTER(_U64)), ("term_bytes", ctypes.POINTER(ctypes.c_uint8)),
    ("doc_counts", ctypes.POINTER(_I64)), ("bucket_doc_count_errors", ctypes.POINTER(_I64)),
    ("subs", ctypes.POINTER(AggBlock)), ("empty_subs", ctypes.POINTER(AggBlock)),
    ("count", ctypes.POINTER(_I64)), ("sum", ctypes.POINTER(_F64)), ("min", ctypes.POINTER(_F64)),
    ("max", ctypes.POINTER(_F64)), ("sum_of_squares", ctypes.POINTER(_F64)),
    ("hll_present", ctypes.POINTER(_I32)), ("hll_mode", ctypes.POINTER(_I32)),
    ("registers", ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))),
    ("lc_hashes", ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32))), ("lc_sizes", ctypes.POINTER(_I64)),
    ("order_path", ctypes.c_char_p),
    ("time_zone", ctypes.c_char_p), ("value_format", _I32), ("reserved_fmt", _I32), ("format", ctypes.c_char_p),
]


class Result(ctypes.Structure):
    _fields_ = [("aggs", ctypes.POINTER(AggBlock)), ("naggs", ctypes.c_int32), ("reserved", ctypes.c_int32)]


ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32,
                                ctypes.c_int32)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)


class HostTransport(ctypes.Structure):
    """esgpu_host_transport: a caller's collectives for esgpu_comm_init_host."""
    _fields_ = [("user", ctypes.c_void_p), ("allreduce", ALLREDUCE_FN), ("allgather", ALLGATHER_FN)]


# every entry point declared in include/esgpu.h: (name, restype, argtypes)
_VP = ctypes.c_void_p
_PP = ctypes.POINTER(ctypes.c_void_p)
SIGNATURES = [
    ("esgpu_last_error", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    ("esgpu_abi_version", ctypes.c_int, []),
    ("esgpu_ctx_create", ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, _PP]),
    ("esgpu_ctx_destroy", ctypes.c_int, [_VP]),
    ("esgpu_ctx_hbm_used", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint64)]),
    ("esgpu_ctx_set_option", ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_int64]),
    ("esgpu_ctx_get_option", ctypes.c_int, [_VP, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
    ("esgpu_device_count", ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ("esgpu_host_alloc", ctypes.c_int, [ctypes.c_size_t, _PP]),
    ("esgpu_host_free", ctypes.c_int, [_VP]),
    ("esgpu_segment_upload", ctypes.c_int, [_VP, ctypes.POINTER(ColumnDesc), ctypes.c_int32, ctypes.c_uint32, _PP]),
    ("esgpu_segment_destroy", ctypes.c_int, [_VP]),
    ("esgpu_segment_max_doc", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint32)]),
    ("esgpu_segment_synthetic", ctypes.c_int, [_VP, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_int64, _PP]),
    ("esgpu_synthetic_fill_host", ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64, _VP]),
    ("esgpu_synthetic_term", ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_size_t]),
    ("esgpu_segment_read_column", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, _VP]),
    ("esgpu_ordinal_map_build", ctypes.c_int, [_VP, ctypes.POINTER(_VP), ctypes.c_int32, ctypes.c_char_p,
                                               ctypes.POINTER(_VP)]),
    ("esgpu_ordinal_map_value_count", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint64)]),
    ("esgpu_ordinal_map_lookup", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64)]),
    ("esgpu_ordinal_map_destroy", ctypes.c_int, [_VP]),
    ("esgpu_terms_thresholds", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                              ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    ("esgpu_precision_from_threshold", ctypes.c_int, [ctypes.c_int64, ctypes.POINTER(ctypes.c_int32)]),
    ("esgpu_date_rounding", ctypes.c_int, [ctypes.POINTER(AggSpec), ctypes.c_int32, ctypes.c_int64,
                                           ctypes.POINTER(ctypes.c_int64)]),
    ("esgpu_routing_hash", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32)]),
    ("esgpu_route_shards", ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, ctypes.c_int32, _VP, _VP]),
    ("esgpu_murmur3_field", ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, _VP]),
    ("esgpu_java_double", ctypes.c_int, [ctypes.c_double, ctypes.c_char_p, ctypes.c_size_t]),
    ("esgpu_murmur3_x64_128", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64)]),
    ("esgpu_plan_create", ctypes.c_int, [_VP, ctypes.POINTER(AggSpec), ctypes.c_int32, ctypes.POINTER(Filter),
                                         ctypes.c_int32, _PP]),
    ("esgpu_plan_collect_segment", ctypes.c_int, [_VP, _VP, _VP]),
    ("esgpu_plan_post_collection", ctypes.c_int, [_VP]),
    ("esgpu_plan_build", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.POINTER(Result))]),
    ("esgpu_plan_reset", ctypes.c_int, [_VP]),
    ("esgpu_plan_destroy", ctypes.c_int, [_VP]),
    ("esgpu_plan_last_collect_stats", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64),
                                                     ctypes.POINTER(ctypes.c_int32)]),
    ("esgpu_plan_last_build_stats", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    ("esgpu_plan_shard_mergeable", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_int32)]),
    ("esgpu_plan_deferred_segments", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_int32)]),
    ("esgpu_result_free", ctypes.c_int, [ctypes.POINTER(Result)]),
    ("esgpu_reduce", ctypes.c_int, [ctypes.POINTER(ctypes.POINTER(Result)), ctypes.c_int32,
                                    ctypes.POINTER(ctypes.POINTER(Result))]),
    ("esgpu_plans_build_reduce", ctypes.c_int, [ctypes.POINTER(_VP), ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Result))]),
    ("esgpu_plans_colocated", ctypes.c_int, [ctypes.POINTER(_VP), ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    ("esgpu_cardinality_value", ctypes.c_int, [ctypes.POINTER(AggBlock), ctypes.c_uint64, ctypes.POINTER(ctypes.c_int64)]),
    ("esgpu_result_to_json", ctypes.c_int, [ctypes.POINTER(Result), ctypes.c_char_p, ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.c_size_t)]),
    ("esgpu_result_to_xcontent", ctypes.c_int, [ctypes.POINTER(Result), ctypes.c_char_p, ctypes.c_size_t,
                                                ctypes.POINTER(ctypes.c_size_t)]),
    ("esgpu_result_to_stream", ctypes.c_int, [ctypes.POINTER(Result), _VP, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    ("esgpu_result_serialize", ctypes.c_int, [ctypes.POINTER(Result), _VP, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    ("esgpu_result_deserialize", ctypes.c_int, [_VP, ctypes.c_size_t, ctypes.POINTER(ctypes.POINTER(Result))]),
    ("esgpu_comm_unique_id", ctypes.c_int, [_VP]),
    ("esgpu_comm_init", ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_int32, _VP, _PP]),
    ("esgpu_comm_init_host", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(HostTransport), _PP]),
    ("esgpu_segment_release_wide", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint64)]),
    ("esgpu_comm_init_local", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, _PP]),
    ("esgpu_comm_build_reduce", ctypes.c_int, [_VP, ctypes.POINTER(_VP), ctypes.c_int32, ctypes.c_int32,
                                               ctypes.POINTER(ctypes.POINTER(Result))]),
    ("esgpu_comm_last_build_reduce", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)]),
    ("esgpu_comm_destroy", ctypes.c_int, [_VP]),
    ("esgpu_comm_reduce", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.POINTER(Result)), ctypes.c_int32,
                                         ctypes.POINTER(ctypes.POINTER(Result))]),
    ("esgpu_comm_gather_reduce", ctypes.c_int, [_VP, ctypes.POINTER(Result), ctypes.POINTER(ctypes.POINTER(Result))]),
    ("esgpu_comm_last_exchange_ms", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    ("esgpu_comm_last_exchange", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_int32)]),
]


class EsGpuError(RuntimeError):
    """Maps the C status codes onto the exceptions the reference raises (SURVEY.md §8(b) "Errors")."""

    def __init__(self, code, message):
        super().__init__(f"[{code}] {message}")
        self.code = code


class UnsupportedOnGpu(EsGpuError):
    """ESGPU_ERR_UNSUPPORTED: the request shape stays on the stock Java (CPU) aggregator."""


class CircuitBreakingError(EsGpuError):
    """ESGPU_ERR_OOM: HBM budget exceeded (CircuitBreakingException)."""


class NoDeviceError(EsGpuError):
    """ESGPU_ERR_NO_DEVICE: no HIP device; the GPU path refuses to run instead of silently falling back."""


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(handle, name, None)
            if fn is None and os.environ.get("ESGPU_LIBRARY"):  # an older variant build for A/B timing
                continue
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc):
    if rc == OK:
        return
    buf = ctypes.create_string_buffer(4096)
    lib().esgpu_last_error(buf, len(buf))
    msg = buf.value.decode("utf-8", "replace")
    cls = {ERR_UNSUPPORTED: UnsupportedOnGpu, ERR_OOM: CircuitBreakingError, ERR_NO_DEVICE: NoDeviceError}.get(rc, EsGpuError)
    raise cls(rc, msg)
