"""elasticsearch_amd — MI355X-native per-shard aggregation collection for Elasticsearch.

The product path is libesgpu.so (hand-written gfx950 HIP kernels + C-ABI, include/esgpu.h); this package is the
host-side driver mirroring the reference's Aggregator / AggregationBuilders surface.  There is no CPU fallback:
without the built library or without a GPU the calls raise.
"""
from ._native import (CircuitBreakingError, EsGpuError, NoDeviceError, UnsupportedOnGpu)  # noqa: F401
from .aggs import AggregationBuilders, Order, QueryBuilders  # noqa: F401
from .engine import (Communicator, Engine, Plan, Segment, ShardResult, device_count, pinned_empty, precision_from_threshold,  # noqa: F401
                     build_reduce, colocated, reduce, routing_hash, synthetic_host_column, synthetic_terms)

__all__ = [
    "AggregationBuilders", "QueryBuilders", "Order", "Engine", "Plan", "Segment", "ShardResult", "Communicator",
    "reduce", "build_reduce", "colocated", "routing_hash", "device_count", "precision_from_threshold", "synthetic_host_column", "synthetic_terms",
    "EsGpuError", "UnsupportedOnGpu", "CircuitBreakingError", "NoDeviceError",
]
