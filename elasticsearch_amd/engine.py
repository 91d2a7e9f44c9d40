"""Host-side driver of libesgpu.so: the Aggregator lifecycle of the reference, one shard per GPU.

    engine = Engine(device=0)
    seg = engine.synthetic_segment(num_docs=1 << 24, fields=("host", "@timestamp", "response_time_ms"))
    plan = engine.plan([AggregationBuilders.terms("hosts").field("host")
                        .subAggregation(AggregationBuilders.dateHistogram("h").field("@timestamp").interval("1h")
                                        .subAggregation(AggregationBuilders.stats("rt").field("response_time_ms")))])
    plan.collect(seg)                 # getLeafCollector + collect(doc) for every doc of the segment
    shard = plan.build()              # postCollection + buildAggregation(0)
    final = reduce([shard])           # InternalAggregations.reduce on the coordinating node
    final.to_dict()

Mirrors AggregationPhase / QueryPhase (core/src/main/java/org/elasticsearch/search/aggregations/AggregationPhase.java:69-168,
core/src/main/java/org/elasticsearch/search/query/QueryPhase.java:254-258,312-314) and the coordinator reduce
(core/src/main/java/org/elasticsearch/search/controller/SearchPhaseController.java:401-411).
"""
import ctypes
import json

import numpy as np

from . import _native as N
from .aggs import flatten, flatten_filters


class ShardResult:
    """An esgpu_result: the shard-level (or reduced) InternalAggregations."""

    def __init__(self, ptr):
        self._ptr = ptr

    @property
    def ptr(self):
        return self._ptr

    def __del__(self):
        if getattr(self, "_ptr", None):
            try:
                N.lib().esgpu_result_free(self._ptr)
            except Exception:
                pass
            self._ptr = None

    def to_json(self):
        needed = ctypes.c_size_t()
        N.check(N.lib().esgpu_result_to_json(self._ptr, None, 0, ctypes.byref(needed)))
        buf = ctypes.create_string_buffer(needed.value + 1)
        N.check(N.lib().esgpu_result_to_json(self._ptr, buf, len(buf), ctypes.byref(needed)))
        return buf.value.decode("utf-8")

    def to_xcontent(self):
        """the search response's "aggregations" object, as Elasticsearch renders it (esgpu_result_to_xcontent)"""
        needed = ctypes.c_size_t()
        N.check(N.lib().esgpu_result_to_xcontent(self._ptr, None, 0, ctypes.byref(needed)))
        buf = ctypes.create_string_buffer(needed.value + 1)
        N.check(N.lib().esgpu_result_to_xcontent(self._ptr, buf, len(buf), ctypes.byref(needed)))
        return buf.value.decode("utf-8")

    def to_dict(self):
        return json.loads(self.to_json())

    def to_stream(self):
        """the bytes InternalAggregations.writeTo(StreamOutput) sends over Elasticsearch's transport
        (esgpu_result_to_stream)"""
        needed = ctypes.c_size_t()
        N.check(N.lib().esgpu_result_to_stream(self._ptr, None, 0, ctypes.byref(needed)))
        buf = (ctypes.c_uint8 * max(needed.value, 1))()
        N.check(N.lib().esgpu_result_to_stream(self._ptr, buf, needed.value, ctypes.byref(needed)))
        return bytes(buf[: needed.value])

    def serialize(self):
        needed = ctypes.c_size_t()
        N.check(N.lib().esgpu_result_serialize(self._ptr, None, 0, ctypes.byref(needed)))
        buf = (ctypes.c_uint8 * max(needed.value, 1))()
        N.check(N.lib().esgpu_result_serialize(self._ptr, buf, needed.value, ctypes.byref(needed)))
        return bytes(buf[: needed.value])

    @staticmethod
    def deserialize(data):
        out = ctypes.POINTER(N.Result)()
        buf = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data if data else b"\0")
        N.check(N.lib().esgpu_result_deserialize(buf, len(data), ctypes.byref(out)))
        return ShardResult(out)

    def aggregation(self, i=0):
        return self._ptr.contents.aggs[i]

    def registers(self, i=0):
        """HLL registers of top-level cardinality aggregation i (None unless it is in hyperloglog mode)."""
        a = self.aggregation(i)
        if a.type != N.AGG_CARDINALITY or not a.hll_present[0] or not a.hll_mode[0]:
            return None
        return np.ctypeslib.as_array(a.registers[0], shape=(1 << a.precision,)).copy()

    def cardinality(self, i=0):
        v = ctypes.c_int64()
        N.check(N.lib().esgpu_cardinality_value(ctypes.byref(self.aggregation(i)), 0, ctypes.byref(v)))
        return v.value


def reduce(results):
    """InternalAggregations.reduce over shard results in shard order (runs on the host, no GPU needed)."""
    arr = (ctypes.POINTER(N.Result) * len(results))(*[r.ptr for r in results])
    out = ctypes.POINTER(N.Result)()
    N.check(N.lib().esgpu_reduce(arr, len(results), ctypes.byref(out)))
    return ShardResult(out)


def build_reduce(plans):
    """The reduce of one request's shard plans that live on one device, built and reduced in one call: the same result
    as reduce([p.build() for p in plans]); terms{histogram{metrics}} requests merge the surviving terms' rows on the
    device instead of building every shard's result (esgpu_plans_build_reduce)."""
    arr = (N._VP * len(plans))(*[p._ptr for p in plans])
    out = ctypes.POINTER(N.Result)()
    N.check(N.lib().esgpu_plans_build_reduce(arr, len(plans), ctypes.byref(out)))
    return ShardResult(out)


def colocated(plans):
    """True if build_reduce merges this request's shards on the device (esgpu_plans_colocated)."""
    arr = (N._VP * len(plans))(*[p._ptr for p in plans])
    v = ctypes.c_int32()
    N.check(N.lib().esgpu_plans_colocated(arr, len(plans), ctypes.byref(v)))
    return bool(v.value)


class OrdinalMap:
    """Global ordinals of one keyword field over a reader's segments (GlobalOrdinalsBuilder / Lucene OrdinalMap)."""

    def __init__(self, ptr):
        self._ptr = ptr

    @property
    def value_count(self):
        v = ctypes.c_uint64()
        N.check(N.lib().esgpu_ordinal_map_value_count(self._ptr, ctypes.byref(v)))
        return v.value

    def lookup(self, term):
        """global ordinal of `term` (str or bytes), -1 if no segment holds it"""
        b = term.encode("utf-8") if isinstance(term, str) else bytes(term)
        v = ctypes.c_int64()
        N.check(N.lib().esgpu_ordinal_map_lookup(self._ptr, b, len(b), ctypes.byref(v)))
        return v.value

    def close(self):
        if self._ptr:
            N.check(N.lib().esgpu_ordinal_map_destroy(self._ptr))
            self._ptr = None


class Segment:
    def __init__(self, engine, ptr, dictionaries=None):
        self.engine = engine
        self._ptr = ptr
        self.dictionaries = dictionaries or {}

    @property
    def ptr(self):
        return self._ptr

    @property
    def max_doc(self):
        v = ctypes.c_uint32()
        N.check(N.lib().esgpu_segment_max_doc(self._ptr, ctypes.byref(v)))
        return v.value

    def release_wide(self):
        """Frees the upload-width values of the long columns that have compact copies (esgpu_segment_release_wide);
        returns the bytes freed.  A later kernel that reads them rebuilds them from the deltas."""
        v = ctypes.c_uint64()
        N.check(N.lib().esgpu_segment_release_wide(self._ptr, ctypes.byref(v)))
        return v.value

    def read_column(self, field, start, count, dtype):
        out = np.empty(count, dtype=dtype)
        N.check(N.lib().esgpu_segment_read_column(self._ptr, field.encode(), start, count, out.ctypes.data))
        return out

    def ord_of(self, field, term):
        d = self.dictionaries.get(field)
        if d is None:
            return -1
        try:
            return d.index(term)
        except ValueError:
            return -1

    def close(self):
        if self._ptr:
            N.check(N.lib().esgpu_segment_destroy(self._ptr))
            self._ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Plan:
    def __init__(self, engine, aggs, filters=None, number_of_shards=1, ord_lookup=None):
        self.engine = engine
        self._specs, n, self._keep = flatten(aggs, number_of_shards)
        self._filters, nf, self._fkeep = flatten_filters(filters, ord_lookup, aggs)
        ptr = ctypes.c_void_p()
        N.check(N.lib().esgpu_plan_create(engine.ptr, self._specs, n, self._filters, nf, ctypes.byref(ptr)))
        self._ptr = ptr

    def collect(self, segment, accept_bits=None):
        bits = None
        if accept_bits is not None:
            bits = np.ascontiguousarray(accept_bits, dtype=np.uint64)
        N.check(N.lib().esgpu_plan_collect_segment(self._ptr, segment.ptr, bits.ctypes.data if bits is not None else None))
        return self

    def post_collection(self):
        N.check(N.lib().esgpu_plan_post_collection(self._ptr))

    def build(self):
        out = ctypes.POINTER(N.Result)()
        N.check(N.lib().esgpu_plan_build(self._ptr, ctypes.byref(out)))
        return ShardResult(out)

    def reset(self):
        N.check(N.lib().esgpu_plan_reset(self._ptr))

    def last_collect_stats(self):
        ms, nbytes, path = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_int32()
        N.check(N.lib().esgpu_plan_last_collect_stats(self._ptr, ctypes.byref(ms), ctypes.byref(nbytes), ctypes.byref(path)))
        return ms.value, nbytes.value, path.value

    def last_build_stats(self):
        """(total_ms, stream_wait_ms) of the last build()"""
        tot, wait = ctypes.c_double(), ctypes.c_double()
        N.check(N.lib().esgpu_plan_last_build_stats(self._ptr, ctypes.byref(tot), ctypes.byref(wait)))
        return tot.value, wait.value

    def shard_mergeable(self):
        """True if several shards may be collected into this one plan (no terms aggregation, see include/esgpu.h)."""
        v = ctypes.c_int32()
        N.check(N.lib().esgpu_plan_shard_mergeable(self._ptr, ctypes.byref(v)))
        return bool(v.value)

    def deferred_segments(self):
        """Segments retained for a breadth-first replay at build (terms under terms over the dense budget)."""
        v = ctypes.c_int32()
        N.check(N.lib().esgpu_plan_deferred_segments(self._ptr, ctypes.byref(v)))
        return v.value

    def close(self):
        if self._ptr:
            N.check(N.lib().esgpu_plan_destroy(self._ptr))
            self._ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    """One device context (one GPU); shards map one-per-GPU."""

    def __init__(self, device=0, hbm_budget_bytes=0):
        ptr = ctypes.c_void_p()
        N.check(N.lib().esgpu_ctx_create(device, hbm_budget_bytes, ctypes.byref(ptr)))
        self._ptr = ptr
        self.device = device
        self._comms = []  # communicators over this context: destroyed before it (they use its device and budget)

    @property
    def ptr(self):
        return self._ptr

    def hbm_used(self):
        v = ctypes.c_uint64()
        N.check(N.lib().esgpu_ctx_hbm_used(self._ptr, ctypes.byref(v)))
        return v.value

    OPTIONS = {"compact_columns": 1, "packed_metric": 2, "hll_floor": 3, "block_deltas": 4}  # include/esgpu.h ESGPU_OPT_*

    def set_option(self, name, value):
        """Layout option of this context (esgpu_ctx_set_option): 'compact_columns' / 'packed_metric' / 'block_deltas', 0 or 1;
        'hll_floor' 0..8 (include/esgpu.h ESGPU_OPT_HLL_FLOOR)."""
        N.check(N.lib().esgpu_ctx_set_option(self._ptr, self.OPTIONS[name], int(value)))

    def get_option(self, name):
        v = ctypes.c_int64()
        N.check(N.lib().esgpu_ctx_get_option(self._ptr, self.OPTIONS[name], ctypes.byref(v)))
        return v.value

    def synthetic_segment(self, num_docs, fields=("host", "@timestamp", "response_time_ms"), shard=0,
                          seed=0x5EEDE1A5, ts_jitter_ms=0):
        mask = 0
        for f in fields:
            mask |= N.SYNTH_FIELDS[f]
        ptr = ctypes.c_void_p()
        N.check(N.lib().esgpu_segment_synthetic(self._ptr, seed, shard, num_docs, mask, ts_jitter_ms, ctypes.byref(ptr)))
        return Segment(self, ptr)

    def ordinal_map(self, segments, field):
        """Build global ordinals of `field` over `segments` and remap their ordinal columns on the GPU."""
        arr = (ctypes.c_void_p * len(segments))(*[sg.ptr for sg in segments])
        out = ctypes.c_void_p()
        N.check(N.lib().esgpu_ordinal_map_build(self._ptr, arr, len(segments), field.encode(), ctypes.byref(out)))
        return OrdinalMap(out)

    def upload_segment(self, columns, max_doc):
        """columns: {name: dict(type=COL_*, values=np.array, offsets=None|np.uint64, present=None|np.uint64 bits,
        terms=None|list[str|bytes])}.  Host arrays are copied once into HBM."""
        descs, keep, dicts = [], [], {}
        for name, c in columns.items():
            d = N.ColumnDesc()
            bname = name.encode("utf-8")
            keep.append(bname)
            d.name = bname
            d.type = c["type"]
            dtype = {N.COL_ORD_U32: np.uint32, N.COL_I64: np.int64, N.COL_F64: np.float64, N.COL_U64: np.uint64}[c["type"]]
            vals = np.ascontiguousarray(c["values"], dtype=dtype)
            keep.append(vals)
            d.values = vals.ctypes.data if vals.size else None
            if c.get("offsets") is not None:
                offs = np.ascontiguousarray(c["offsets"], dtype=np.uint64)
                keep.append(offs)
                d.offsets = offs.ctypes.data
            if c.get("present") is not None:
                pres = np.ascontiguousarray(c["present"], dtype=np.uint64)
                keep.append(pres)
                d.present = pres.ctypes.data
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
                tb = [t.encode("utf-8") if isinstance(t, str) else bytes(t) for t in terms]
                blob = np.frombuffer(b"".join(tb), dtype=np.uint8) if tb and sum(map(len, tb)) else np.zeros(1, np.uint8)
                offs = np.zeros(len(tb) + 1, dtype=np.uint64)
                offs[1:] = np.cumsum([len(t) for t in tb]) if tb else []
                blob = np.ascontiguousarray(blob)
                keep += [blob, offs]
                d.dict_bytes = blob.ctypes.data
                d.dict_offsets = offs.ctypes.data
                d.value_count = len(tb)
                dicts[name] = [t.decode("utf-8", "replace") for t in tb]
            else:
                d.value_count = int(c.get("value_count", 0))
            descs.append(d)
        arr = (N.ColumnDesc * max(len(descs), 1))(*descs)
        ptr = ctypes.c_void_p()
        N.check(N.lib().esgpu_segment_upload(self._ptr, arr, len(descs), max_doc, ctypes.byref(ptr)))
        return Segment(self, ptr, dicts)

    def plan(self, aggs, filters=None, number_of_shards=1, ord_lookup=None):
        return Plan(self, aggs, filters, number_of_shards, ord_lookup)

    def route_shards(self, ids, number_of_shards, with_hashes=False):
        """Shard of each _id / routing string (OperationRouting.shardId, Murmur3HashFunction), computed on the GPU."""
        units = [np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16) for s in ids]
        offs = np.zeros(len(ids) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(u) for u in units]) if units else []
        chars = np.ascontiguousarray(np.concatenate(units) if units else np.zeros(1, np.uint16))
        shards = np.zeros(max(len(ids), 1), dtype=np.int32)
        hashes = np.zeros(max(len(ids), 1), dtype=np.int32)
        N.check(N.lib().esgpu_route_shards(self._ptr, chars.ctypes.data, offs.ctypes.data, len(ids), number_of_shards,
                                           hashes.ctypes.data if with_hashes else None, shards.ctypes.data))
        return (shards[:len(ids)], hashes[:len(ids)]) if with_hashes else shards[:len(ids)]

    def murmur3_field(self, values):
        """The murmur3 field's indexed long of each string value (MurmurHash3.hash128(utf8, 0).h1), on the GPU."""
        b = [v.encode("utf-8") if isinstance(v, str) else bytes(v) for v in values]
        offs = np.zeros(len(b) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(x) for x in b]) if b else []
        blob = np.frombuffer(b"".join(b) or b"\0", dtype=np.uint8).copy()
        out = np.zeros(max(len(b), 1), dtype=np.uint64)
        N.check(N.lib().esgpu_murmur3_field(self._ptr, blob.ctypes.data, offs.ctypes.data, len(b), out.ctypes.data))
        return out[:len(b)]

    def close(self):
        if self._ptr:
            for c in self._comms:
                c.close()
            self._comms = []
            N.check(N.lib().esgpu_ctx_destroy(self._ptr))
            self._ptr = None


class PinnedArray(np.ndarray):
    """A numpy array over page-locked host memory (esgpu_host_alloc); freed with the array."""

    def __array_finalize__(self, obj):
        pass


def pinned_empty(count, dtype):
    """numpy array of `count` elements in page-locked host memory, for K11 exports (esgpu_segment_upload)."""
    dtype = np.dtype(dtype)
    nbytes = max(int(count) * dtype.itemsize, 1)
    ptr = ctypes.c_void_p()
    N.check(N.lib().esgpu_host_alloc(nbytes, ctypes.byref(ptr)))
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr.value)
    arr = np.frombuffer(buf, dtype=np.uint8, count=int(count) * dtype.itemsize).view(dtype)
    import weakref
    holder = arr.view(PinnedArray)
    weakref.finalize(holder, N.lib().esgpu_host_free, ptr.value)
    holder._pin_buf = buf  # noqa: SLF001 -- keeps the ctypes view alive with the array
    return holder


def device_count():
    n = ctypes.c_int()
    N.check(N.lib().esgpu_device_count(ctypes.byref(n)))
    return n.value


def synthetic_host_column(field, num_docs, start=0, count=None, shard=0, seed=0x5EEDE1A5, ts_jitter_ms=0, out=None):
    """The same synthetic values the device generator writes, computed on the CPU (oracle / CPU baseline input)."""
    count = num_docs - start if count is None else count
    dtype = {N.COL_ORD_U32: np.uint32, N.COL_I64: np.int64, N.COL_F64: np.float64, N.COL_U64: np.uint64}[N.SYNTH_TYPES[field]]
    if out is None:
        out = np.empty(count, dtype=dtype)
    N.check(N.lib().esgpu_synthetic_fill_host(seed, shard, num_docs, N.SYNTH_FIELDS[field], ts_jitter_ms, start, count,
                                              out.ctypes.data))
    return out


def synthetic_terms(field, n):
    buf = ctypes.create_string_buffer(64)
    out = []
    for o in range(n):
        N.lib().esgpu_synthetic_term(N.SYNTH_FIELDS[field], o, buf, 64)
        out.append(buf.value.decode())
    return out


def routing_hash(routing):
    """Murmur3HashFunction.hash(routing): murmur3_x86_32 of the string's UTF-16LE bytes (host, no GPU needed)."""
    u = np.frombuffer(routing.encode("utf-16-le"), dtype=np.uint16).copy()
    out = ctypes.c_int32()
    N.check(N.lib().esgpu_routing_hash(u.ctypes.data if u.size else None, u.size, ctypes.byref(out)))
    return out.value


def precision_from_threshold(t):
    p = ctypes.c_int32()
    N.check(N.lib().esgpu_precision_from_threshold(t, ctypes.byref(p)))
    return p.value


class Communicator:
    """The shard reduce across ranks (include/esgpu.h "Shard reduce across ranks"): RCCL over xGMI between the GPUs of a
    node, or the same reduce over a torch.distributed process group on the host (gloo: cross-node, CPU tests)."""

    def __init__(self, engine, nranks, rank, unique_id):
        ptr = ctypes.c_void_p()
        idbuf = (ctypes.c_uint8 * N.COMM_ID_BYTES).from_buffer_copy(unique_id)
        N.check(N.lib().esgpu_comm_init(engine.ptr, nranks, rank, idbuf, ctypes.byref(ptr)))
        self._ptr = ptr
        self._keep = engine  # the context outlives the communicator (esgpu_comm_destroy frees device buffers in it)
        engine._comms.append(self)

    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * N.COMM_ID_BYTES)()
        N.check(N.lib().esgpu_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def over_process_group(cls, group=None):
        """The reduce's collectives over torch.distributed (the default group, or `group`) in host memory."""
        import numpy as _np
        import torch
        import torch.distributed as dist
        nranks, rank = dist.get_world_size(group), dist.get_rank(group)
        np_types = {N.DT_U8: _np.uint8, N.DT_I64: _np.int64, N.DT_U64: _np.uint64, N.DT_F64: _np.float64}
        ops = {N.RED_SUM: dist.ReduceOp.SUM, N.RED_MIN: dist.ReduceOp.MIN, N.RED_MAX: dist.ReduceOp.MAX}

        def allreduce(_user, buf, count, dt, op):
            try:
                a = _np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(_np.ctypeslib.as_ctypes_type(np_types[dt]))),
                                           shape=(count,))
                if dt == N.DT_U64:  # unsigned order through signed int64: flip the sign bit around min / max
                    x = a.view(_np.int64).copy()
                    if op != N.RED_SUM:
                        x ^= _np.int64(-(1 << 63))
                    t = torch.from_numpy(x)
                    dist.all_reduce(t, op=ops[op], group=group)
                    y = t.numpy()
                    if op != N.RED_SUM:
                        y ^= _np.int64(-(1 << 63))
                    a.view(_np.int64)[:] = y
                else:
                    t = torch.from_numpy(a.copy())
                    dist.all_reduce(t, op=ops[op], group=group)
                    a[:] = t.numpy()
                return 0
            except Exception:  # noqa: BLE001 -- a C caller cannot take a Python exception
                return 1

        def allgather(_user, src, dst, nbytes):
            try:
                x = torch.from_numpy(_np.frombuffer(ctypes.string_at(src, nbytes), dtype=_np.uint8).copy())
                outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(nranks)]
                dist.all_gather(outs, x, group=group)
                joined = torch.cat(outs).numpy()  # keep a reference while copying out of it
                ctypes.memmove(dst, joined.ctypes.data, nbytes * nranks)
                return 0
            except Exception:  # noqa: BLE001
                return 1

        t = N.HostTransport(None, N.ALLREDUCE_FN(allreduce), N.ALLGATHER_FN(allgather))
        ptr = ctypes.c_void_p()
        N.check(N.lib().esgpu_comm_init_host(nranks, rank, ctypes.byref(t), ctypes.byref(ptr)))
        self = cls.__new__(cls)
        self._ptr = ptr
        self._keep = t  # the callbacks must outlive the communicator
        return self

    @classmethod
    def local(cls, group, nranks, rank):
        """An in-process communicator: `nranks` ranks of this process (one thread each, each with its own Engine, on one
        or several devices) that share the name `group`.  Collectives are barriers among the threads; device operands are
        copied device to device.  Every rank's thread must make the same calls in the same order."""
        ptr = ctypes.c_void_p()
        N.check(N.lib().esgpu_comm_init_local(group.encode(), nranks, rank, ctypes.byref(ptr)))
        self = cls.__new__(cls)
        self._ptr = ptr
        self._keep = None
        return self

    def build_reduce(self, plans, root=-1):
        """The device-resident reduce across ranks (esgpu_comm_build_reduce): this rank's collected shard plans (its
        shards in global order rank-major).  The reduced result is returned on rank `root` (every rank when root < 0;
        an empty result elsewhere)."""
        arr = (N._VP * len(plans))(*[p._ptr for p in plans])
        out = ctypes.POINTER(N.Result)()
        N.check(N.lib().esgpu_comm_build_reduce(self._ptr, arr, len(plans), root, ctypes.byref(out)))
        return ShardResult(out)

    def last_build_reduce(self):
        """(path, host ms) of the last build_reduce: path 1 = device-resident exchange, 0 = builds + reduce."""
        path, ms = ctypes.c_int32(), ctypes.c_double()
        N.check(N.lib().esgpu_comm_last_build_reduce(self._ptr, ctypes.byref(path), ctypes.byref(ms)))
        return path.value, ms.value

    def reduce(self, shard_results):
        """InternalAggregations.reduce over every rank's shard results (this rank's in its shard order)."""
        arr = (ctypes.POINTER(N.Result) * len(shard_results))(*[r.ptr for r in shard_results])
        out = ctypes.POINTER(N.Result)()
        N.check(N.lib().esgpu_comm_reduce(self._ptr, arr, len(shard_results), ctypes.byref(out)))
        return ShardResult(out)

    def gather_reduce(self, shard_result):
        out = ctypes.POINTER(N.Result)()
        N.check(N.lib().esgpu_comm_gather_reduce(self._ptr, shard_result.ptr, ctypes.byref(out)))
        return ShardResult(out)

    def last_exchange(self):
        """(all-reduce bytes, all-gather bytes, collectives) of the last reduce."""
        ar, ag, n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int32()
        N.check(N.lib().esgpu_comm_last_exchange(self._ptr, ctypes.byref(ar), ctypes.byref(ag), ctypes.byref(n)))
        return ar.value, ag.value, n.value

    def last_exchange_ms(self):
        """wall-clock ms the last reduce spent inside its collectives"""
        v = ctypes.c_double()
        N.check(N.lib().esgpu_comm_last_exchange_ms(self._ptr, ctypes.byref(v)))
        return v.value

    def close(self):
        if self._ptr:
            N.check(N.lib().esgpu_comm_destroy(self._ptr))
            self._ptr = None
