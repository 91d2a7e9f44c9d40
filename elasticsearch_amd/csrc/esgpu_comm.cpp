// esgpu_comm.cpp — the shard reduce across ranks (include/esgpu.h "Shard reduce across ranks"): collectives over
// RCCL / xGMI (one process per GPU) or over a caller's host transport, driving reduce_across (esgpu_results.cpp).
//
// Reference: the coordinating reduce SearchPhaseController.merge -> InternalAggregations.reduce
// (core/src/main/java/org/elasticsearch/search/controller/SearchPhaseController.java:401-411) over shard results
// that travel as AggregationStreams records; here fixed-shape partials travel as ncclAllReduce operands instead.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/esgpu.h"
#include "esgpu_internal.hpp"
#include "esgpu_kernels.hpp"
#include "esgpu_results.hpp"

using namespace esgpu;

#define NCCLX(expr)                                                                                           \
    do {                                                                                                      \
        ncclResult_t r_ = (expr);                                                                             \
        if (r_ != ncclSuccess) throw EsError(ESGPU_ERR_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

namespace {

size_t dt_size(int dt) { return dt == ESGPU_DT_U8 ? 1 : 8; }

// adds the lifetime of the scope to a collective's exchange time
struct Clock {
    Collective& c;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit Clock(Collective& col) : c(col) {}
    ~Clock() { c.exchange_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
};

// RCCL over xGMI: host operands staged through pinned memory into a device buffer, reduced in place on the
// communicator's stream.  The operands are small (KB for histograms, 2^p bytes of registers, shard records).
struct RcclCollective : Collective {
    esgpu_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    Scratch d_in, d_out;
    PinnedBuf h_in, h_out;
    ~RcclCollective() override {
        if (ctx) (void)hipSetDevice(ctx->device);
        if (comm) ncclCommDestroy(comm);
        if (stream) (void)hipStreamDestroy(stream);
    }
    void allreduce(void* buf, uint64_t count, int dt, int op) override {
        if (!count) return;
        Clock clk(*this);
        const size_t bytes = count * dt_size(dt);
        HIPX(hipSetDevice(ctx->device));
        void* h = h_in.ensure(bytes);
        std::memcpy(h, buf, bytes);
        void* d = d_in.ensure(ctx, bytes);
        HIPX(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream));
        const ncclDataType_t t = dt == ESGPU_DT_U8 ? ncclUint8 : dt == ESGPU_DT_I64 ? ncclInt64 : dt == ESGPU_DT_U64 ? ncclUint64 : ncclFloat64;
        const ncclRedOp_t o = op == ESGPU_RED_SUM ? ncclSum : op == ESGPU_RED_MIN ? ncclMin : ncclMax;
        NCCLX(ncclAllReduce(d, d, count, t, o, comm, stream));
        HIPX(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, stream));
        HIPX(hipStreamSynchronize(stream));
        std::memcpy(buf, h, bytes);
        allreduce_bytes += bytes;
        ++collectives;
    }
    void allgather(const void* in, void* out, uint64_t bytes) override {
        Clock clk(*this);
        HIPX(hipSetDevice(ctx->device));
        const size_t total = (size_t)bytes * nranks;
        void* hi = h_in.ensure(std::max<size_t>(bytes, 1));
        std::memcpy(hi, in, bytes);
        uint8_t* di = (uint8_t*)d_in.ensure(ctx, std::max<size_t>(bytes, 1));
        uint8_t* dout = (uint8_t*)d_out.ensure(ctx, std::max<size_t>(total, 1));
        HIPX(hipMemcpyAsync(di, hi, bytes, hipMemcpyHostToDevice, stream));
        NCCLX(ncclAllGather(di, dout, bytes, ncclUint8, comm, stream));
        void* ho = h_out.ensure(std::max<size_t>(total, 1));
        HIPX(hipMemcpyAsync(ho, dout, total, hipMemcpyDeviceToHost, stream));
        HIPX(hipStreamSynchronize(stream));
        std::memcpy(out, ho, total);
        allgather_bytes += total;
        ++collectives;
    }
    void allgather_dev(const void* d_in, void* d_out, uint64_t bytes, void* stream) override {
        Clock clk(*this);
        HIPX(hipSetDevice(ctx->device));
        NCCLX(ncclAllGather(d_in, d_out, bytes, ncclUint8, comm, (hipStream_t)stream));  // no host round trip
        allgather_bytes += bytes * nranks;
        ++collectives;
    }
    void allreduce_dev(void* d_buf, uint64_t count, int dt, int op, void* stream) override {
        if (!count) return;
        Clock clk(*this);
        HIPX(hipSetDevice(ctx->device));
        const ncclDataType_t t = dt == ESGPU_DT_U8 ? ncclUint8 : dt == ESGPU_DT_I64 ? ncclInt64 : dt == ESGPU_DT_U64 ? ncclUint64 : ncclFloat64;
        const ncclRedOp_t o = op == ESGPU_RED_SUM ? ncclSum : op == ESGPU_RED_MIN ? ncclMin : ncclMax;
        NCCLX(ncclAllReduce(d_buf, d_buf, count, t, o, comm, (hipStream_t)stream));  // in place, on the caller's stream
        allreduce_bytes += count * dt_size(dt);
        ++collectives;
    }
};

// a caller's transport (esgpu_comm_init_host)
struct HostCollective : Collective {
    esgpu_host_transport t{};
    void allreduce(void* buf, uint64_t count, int dt, int op) override {
        if (!count) return;
        Clock clk(*this);
        require(t.allreduce(t.user, buf, count, dt, op) == 0, ESGPU_ERR_DEVICE, "host transport all-reduce failed");
        allreduce_bytes += count * dt_size(dt);
        ++collectives;
    }
    void allgather(const void* in, void* out, uint64_t bytes) override {
        Clock clk(*this);
        require(t.allgather(t.user, in, out, bytes) == 0, ESGPU_ERR_DEVICE, "host transport all-gather failed");
        allgather_bytes += bytes * nranks;
        ++collectives;
    }
    PinnedBuf h_in, h_out;
    void allgather_dev(const void* d_in, void* d_out, uint64_t bytes, void* stream) override {
        // the caller's transport moves host memory: the operand staged through pinned buffers
        hipStream_t st = (hipStream_t)stream;
        void* hi = h_in.ensure(std::max<size_t>(bytes, 1));
        void* ho = h_out.ensure(std::max<size_t>(bytes * nranks, 1));
        HIPX(hipMemcpyAsync(hi, d_in, bytes, hipMemcpyDeviceToHost, st));
        HIPX(hipStreamSynchronize(st));
        allgather(hi, ho, bytes);
        HIPX(hipMemcpyAsync(d_out, ho, bytes * nranks, hipMemcpyHostToDevice, st));
        HIPX(hipStreamSynchronize(st));  // the staging buffer is reused by the next call
    }
    void allreduce_dev(void* d_buf, uint64_t count, int dt, int op, void* stream) override {
        if (!count) return;
        hipStream_t st = (hipStream_t)stream;
        const size_t bytes = count * dt_size(dt);
        void* h = h_in.ensure(bytes);
        HIPX(hipMemcpyAsync(h, d_buf, bytes, hipMemcpyDeviceToHost, st));
        HIPX(hipStreamSynchronize(st));
        allreduce(h, count, dt, op);
        HIPX(hipMemcpyAsync(d_buf, h, bytes, hipMemcpyHostToDevice, st));
        HIPX(hipStreamSynchronize(st));
    }
};

// a device buffer of the in-process transport (no context: its ranks' contexts are their own), grown on demand
struct RawDev {
    void* p = nullptr;
    size_t bytes = 0;
    int dev = 0;
    void* ensure_raw(size_t n) {
        if (n > bytes) {
            if (p) HIPX(hipFree(p));
            p = nullptr;
            HIPX(hipGetDevice(&dev));
            HIPX(hipMalloc(&p, n));
            bytes = n;
        }
        return p;
    }
    ~RawDev() {
        if (p) {
            (void)hipSetDevice(dev);
            (void)hipFree(p);
        }
    }
};

// in-process ranks (esgpu_comm_init_local): the threads of one process, one context each, meet at barriers; host
// operands are copied between their buffers, device operands device to device on each rank's stream
struct LocalGroup {
    std::mutex mu;
    std::condition_variable cv;
    int n = 0, arrived = 0;
    uint64_t gen = 0;
    std::vector<const void*> src;
    std::vector<hipEvent_t> ready;
    std::vector<int> dev;
    bool broken = false;
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        require(!broken, ESGPU_ERR_DEVICE, "in-process communicator: a rank failed");
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; }) || broken) {
            broken = true;  // a rank that never arrives (it failed): every waiting rank fails instead of hanging
            cv.notify_all();
            throw EsError(ESGPU_ERR_DEVICE, "in-process communicator: a rank did not reach the collective");
        }
    }
};
std::mutex g_local_mu;
std::map<std::string, std::weak_ptr<LocalGroup>> g_local_groups;

struct LocalCollective : Collective {
    std::shared_ptr<LocalGroup> g;
    hipEvent_t ready = nullptr;
    std::vector<uint8_t> tmp;
    ~LocalCollective() override {
        if (ready) (void)hipEventDestroy(ready);
    }
    void allreduce(void* buf, uint64_t count, int dt, int op) override {
        if (!count) return;
        Clock clk(*this);
        const size_t bytes = count * dt_size(dt);
        g->src[rank] = buf;
        g->barrier();
        tmp.assign((const uint8_t*)g->src[0], (const uint8_t*)g->src[0] + bytes);  // rank order: rank 0 first
        for (int r = 1; r < nranks; ++r) {
            const void* s = g->src[r];
            for (uint64_t i = 0; i < count; ++i) {
                switch (dt) {
                    case ESGPU_DT_U8: red(((uint8_t*)tmp.data())[i], ((const uint8_t*)s)[i], op); break;
                    case ESGPU_DT_I64: red(((int64_t*)tmp.data())[i], ((const int64_t*)s)[i], op); break;
                    case ESGPU_DT_U64: red(((uint64_t*)tmp.data())[i], ((const uint64_t*)s)[i], op); break;
                    default: red(((double*)tmp.data())[i], ((const double*)s)[i], op); break;
                }
            }
        }
        g->barrier();  // every rank has read every operand
        std::memcpy(buf, tmp.data(), bytes);
        allreduce_bytes += bytes;
        ++collectives;
    }
    template <class T> static void red(T& a, T b, int op) {
        if (op == ESGPU_RED_SUM) a = a + b;
        else if (op == ESGPU_RED_MIN) a = b < a ? b : a;
        else a = b > a ? b : a;
    }
    void allgather(const void* in, void* out, uint64_t bytes) override {
        Clock clk(*this);
        g->src[rank] = in;
        g->barrier();
        for (int r = 0; r < nranks; ++r) std::memcpy((uint8_t*)out + (size_t)r * bytes, g->src[r], bytes);
        g->barrier();
        allgather_bytes += bytes * nranks;
        ++collectives;
    }
    void allgather_dev(const void* d_in, void* d_out, uint64_t bytes, void* stream) override {
        Clock clk(*this);
        hipStream_t st = (hipStream_t)stream;
        if (!ready) HIPX(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        HIPX(hipEventRecord(ready, st));  // this rank's operand is written once its stream reaches here
        int d = 0;
        HIPX(hipGetDevice(&d));
        g->src[rank] = d_in;
        g->ready[rank] = ready;
        g->dev[rank] = d;
        g->barrier();
        bool one_device = bytes % 8 == 0 && nranks <= esgpu::kColoMaxShards;
        for (int r = 0; r < nranks; ++r) {
            one_device = one_device && g->dev[r] == d;
            if (r != rank) HIPX(hipStreamWaitEvent(st, g->ready[r], 0));
        }
        if (one_device) {  // every operand on this device: one gather launch instead of a DMA copy per rank
            launch_gather_bufs(g->src.data(), nranks, bytes, d_out, st);
            HIPX(hipGetLastError());
        } else {
            for (int r = 0; r < nranks; ++r)
                HIPX(hipMemcpyAsync((uint8_t*)d_out + (size_t)r * bytes, g->src[r], bytes, hipMemcpyDeviceToDevice, st));
        }
        // every rank has finished reading every operand before any rank goes on: a rank may rewrite, reallocate or free
        // its operand buffer as soon as the call returns (the next request, or the plan's destruction)
        HIPX(hipStreamSynchronize(st));
        g->barrier();
        allgather_bytes += bytes * nranks;
        ++collectives;
    }
    RawDev d_stage, d_red;
    void allreduce_dev(void* d_buf, uint64_t count, int dt, int op, void* stream) override {
        if (!count) return;
        Clock clk(*this);
        hipStream_t st = (hipStream_t)stream;
        const size_t bytes = count * dt_size(dt);
        if (!ready) HIPX(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        HIPX(hipEventRecord(ready, st));
        int d = 0;
        HIPX(hipGetDevice(&d));
        g->src[rank] = d_buf;
        g->ready[rank] = ready;
        g->dev[rank] = d;
        g->barrier();
        bool one_device = nranks <= esgpu::kColoMaxShards;
        for (int r = 0; r < nranks; ++r) {
            one_device = one_device && g->dev[r] == d;
            if (r != rank) HIPX(hipStreamWaitEvent(st, g->ready[r], 0));
        }
        // every rank reduces all operands (rank order, as the host transport does) into its own scratch, and writes its
        // buffer only after every rank has read every operand
        void* red = d_red.ensure_raw(bytes);
        std::vector<const void*> srcs(g->src.begin(), g->src.end());
        if (!one_device) {  // operands on other devices: copied here first
            uint8_t* stage = (uint8_t*)d_stage.ensure_raw(bytes * nranks);
            for (int r = 0; r < nranks; ++r) {
                HIPX(hipMemcpyAsync(stage + (size_t)r * bytes, g->src[r], bytes, hipMemcpyDeviceToDevice, st));
                srcs[r] = stage + (size_t)r * bytes;
            }
        }
        launch_reduce_bufs(srcs.data(), nranks, count, dt, op, red, st);
        HIPX(hipGetLastError());
        HIPX(hipStreamSynchronize(st));
        g->barrier();
        HIPX(hipMemcpyAsync(d_buf, red, bytes, hipMemcpyDeviceToDevice, st));
        allreduce_bytes += bytes;
        ++collectives;
    }
};

}  // namespace

struct esgpu_comm {
    std::unique_ptr<Collective> coll;
};

extern "C" int esgpu_comm_unique_id(uint8_t* id_out) {
    return guarded([&] {
        static_assert(sizeof(ncclUniqueId) == ESGPU_COMM_ID_BYTES, "ncclUniqueId size");
        require(id_out != nullptr, ESGPU_ERR_INVALID, "null argument");
        ncclUniqueId id;
        NCCLX(ncclGetUniqueId(&id));
        std::memcpy(id_out, &id, sizeof id);
    });
}

extern "C" int esgpu_comm_init(esgpu_ctx* c, int32_t nranks, int32_t rank, const uint8_t* id, esgpu_comm** out) {
    return guarded([&] {
        require(c && id && out && nranks >= 1 && rank >= 0 && rank < nranks, ESGPU_ERR_INVALID, "bad communicator arguments");
        HIPX(hipSetDevice(c->device));
        std::unique_ptr<RcclCollective> r(new RcclCollective());
        r->ctx = c;
        r->nranks = nranks;
        r->rank = rank;
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof uid);
        NCCLX(ncclCommInitRank(&r->comm, nranks, uid, rank));
        HIPX(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
        std::unique_ptr<esgpu_comm> cm(new esgpu_comm());
        cm->coll = std::move(r);
        *out = cm.release();
    });
}

extern "C" int esgpu_comm_init_host(int32_t nranks, int32_t rank, const esgpu_host_transport* t, esgpu_comm** out) {
    tune_host_heap();
    return guarded([&] {
        require(t && t->allreduce && t->allgather && out && nranks >= 1 && rank >= 0 && rank < nranks, ESGPU_ERR_INVALID,
                "bad communicator arguments");
        std::unique_ptr<HostCollective> h(new HostCollective());
        h->t = *t;
        h->nranks = nranks;
        h->rank = rank;
        std::unique_ptr<esgpu_comm> cm(new esgpu_comm());
        cm->coll = std::move(h);
        *out = cm.release();
    });
}

extern "C" int esgpu_comm_init_local(const char* group, int32_t nranks, int32_t rank, esgpu_comm** out) {
    return guarded([&] {
        require(group && out && nranks >= 1 && rank >= 0 && rank < nranks, ESGPU_ERR_INVALID, "bad communicator arguments");
        std::shared_ptr<LocalGroup> g;
        {
            std::lock_guard<std::mutex> lk(g_local_mu);
            std::weak_ptr<LocalGroup>& w = g_local_groups[group];
            g = w.lock();
            bool broken = false;
            if (g) {
                std::lock_guard<std::mutex> glk(g->mu);
                broken = g->broken;
            }
            if (g && !broken) {
                // the ranks of one live group must agree on its size: replacing it would strand the ranks already in it
                require(g->n == nranks, ESGPU_ERR_INVALID, "in-process communicator: the group is alive with another rank count");
            } else {
                // a new group, or a name whose group broke (a rank timed out; its ranks all fail): the name is reusable
                g = std::make_shared<LocalGroup>();
                g->n = nranks;
                g->src.assign(nranks, nullptr);
                g->ready.assign(nranks, nullptr);
                g->dev.assign(nranks, 0);
                w = g;
            }
        }
        std::unique_ptr<LocalCollective> c(new LocalCollective());
        c->g = g;
        c->nranks = nranks;
        c->rank = rank;
        std::unique_ptr<esgpu_comm> cm(new esgpu_comm());
        cm->coll = std::move(c);
        *out = cm.release();
    });
}

namespace esgpu {
Collective& comm_collective(esgpu_comm* c) { return *c->coll; }
}  // namespace esgpu

extern "C" int esgpu_comm_last_build_reduce(const esgpu_comm* cm, int32_t* path, double* host_ms) {
    return guarded([&] {
        require(cm != nullptr, ESGPU_ERR_INVALID, "null communicator");
        if (path) *path = cm->coll->last_path;
        if (host_ms) *host_ms = cm->coll->last_host_ms;
    });
}

extern "C" int esgpu_comm_destroy(esgpu_comm* cm) {
    return guarded([&] { delete cm; });
}

static int comm_reduce(esgpu_comm* cm, const esgpu_result* const* locals, int32_t n, esgpu_result** out, bool gather_only) {
    return guarded([&] {
        require(cm && locals && n >= 1 && out, ESGPU_ERR_INVALID, "comm reduce needs at least one local shard result");
        std::vector<const std::vector<Block>*> lists;
        for (int i = 0; i < n; ++i) {
            require(locals[i] != nullptr, ESGPU_ERR_INVALID, "null shard result");
            lists.push_back(&holder_of(locals[i])->aggs);
        }
        std::unique_ptr<ResultHolder> h(new ResultHolder());
        h->aggs = reduce_across(*cm->coll, lists, gather_only);
        h->export_view();
        *out = &h.release()->pub;
    });
}

extern "C" int esgpu_comm_reduce(esgpu_comm* cm, const esgpu_result* const* locals, int32_t n, esgpu_result** out) {
    return comm_reduce(cm, locals, n, out, false);
}

extern "C" int esgpu_comm_gather_reduce(esgpu_comm* cm, const esgpu_result* local, esgpu_result** out) {
    return comm_reduce(cm, &local, 1, out, true);
}

extern "C" int esgpu_comm_last_exchange_ms(const esgpu_comm* cm, double* ms) {
    return guarded([&] {
        require(cm && ms, ESGPU_ERR_INVALID, "null argument");
        *ms = cm->coll->exchange_ms;
    });
}

extern "C" int esgpu_comm_last_exchange(const esgpu_comm* cm, uint64_t* ar, uint64_t* ag, int32_t* n) {
    return guarded([&] {
        require(cm != nullptr, ESGPU_ERR_INVALID, "null communicator");
        if (ar) *ar = cm->coll->allreduce_bytes;
        if (ag) *ag = cm->coll->allgather_bytes;
        if (n) *n = cm->coll->collectives;
    });
}
