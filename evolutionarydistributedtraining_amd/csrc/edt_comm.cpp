// edt_comm.cpp — RCCL (over xGMI) behind the C ABI of include/edt_comm.h, and the bucketed
// DiLoCo schedules in C (distributed.py mode="reduce", "reduce_ordered" and "exact"): host code
// only, the kernels are libedt_sync's edt_delta_partial / edt_sgd_apply / edt_sgd_apply_sum /
// edt_outer_step.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "edt_comm.h"
#include "edt_sync.h"

namespace {

thread_local char g_err[512];

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define EDT_RCCL(call)                                                                        \
    do {                                                                                      \
        ncclResult_t r_ = (call);                                                             \
        if (r_ != ncclSuccess) return fail(EDT_COMM_ERR_RCCL, "%s: %s", #call, ncclGetErrorString(r_)); \
    } while (0)
#define EDT_HIP(call)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) return fail(EDT_COMM_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)

// One rank's communicator: the RCCL comm, a stream of its own for the collectives of the
// sharded step (so they overlap the kernels on the caller's stream), and an event pool.
struct Comm {
    ncclComm_t nccl = nullptr;
    int rank = 0, nranks = 1;
    hipStream_t side = nullptr;
    std::vector<hipEvent_t> events;
    bool aborted = false;        // edt_comm_abort (or a timeout) tore the RCCL communicator down
    double timeout_s = 0.0;      // > 0: edt_outer_step_sharded waits for its work, bounded by this
};

Comm* as_comm(void* c) { return static_cast<Comm*>(c); }

// Every entry point first: a torn-down communicator, or an asynchronous RCCL error a peer's
// failure left behind, fails the call instead of enqueueing work that can never complete.
int usable(Comm* c) {
    if (!c) return fail(EDT_COMM_ERR_ARG, "null communicator");
    if (c->aborted) return fail(EDT_COMM_ERR_ABORTED, "communicator of rank %d was aborted", c->rank);
    ncclResult_t async = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(c->nccl, &async);
    if (r != ncclSuccess) return fail(EDT_COMM_ERR_RCCL, "ncclCommGetAsyncError: %s", ncclGetErrorString(r));
    if (async != ncclSuccess && async != ncclInProgress)
        return fail(EDT_COMM_ERR_RCCL, "asynchronous RCCL error on rank %d: %s", c->rank, ncclGetErrorString(async));
    return 0;
}

void abort_comm(Comm* c) {
    if (c && !c->aborted) {
        (void)ncclCommAbort(c->nccl);
        c->nccl = nullptr;
        c->aborted = true;
    }
}

// Host wait for `ev` (recorded after the work to wait for), polling the event and RCCL's async
// error; past timeout_s (<= 0: none) the communicator is aborted so the stuck collectives end.
int wait_event(Comm* c, hipEvent_t ev, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return 0;
        if (q != hipErrorNotReady) return fail(EDT_COMM_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(q));
        if (int rc = usable(c)) {
            abort_comm(c);
            return rc;
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (timeout_s > 0 && el > timeout_s) {
            abort_comm(c);
            return fail(EDT_COMM_ERR_TIMEOUT, "rank %d: collectives not done after %.3f s; communicator aborted",
                        c->rank, el);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

bool nccl_type(int dt, ncclDataType_t* t, uint64_t* size) {
    if (dt == EDT_F32) { *t = ncclFloat32; *size = 4; return true; }
    if (dt == EDT_BF16) { *t = ncclBfloat16; *size = 2; return true; }
    return false;
}

int ensure_events(Comm* c, size_t n) {
    while (c->events.size() < n) {
        hipEvent_t e;
        EDT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->events.push_back(e);
    }
    return 0;
}

}  // namespace

extern "C" {

uint64_t edt_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

int edt_comm_unique_id(void* id_out) {
    if (!id_out) return fail(EDT_COMM_ERR_ARG, "id_out is null");
    ncclUniqueId id;
    EDT_RCCL(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

int edt_comm_init(void** comm, const void* id, int nranks, int rank) {
    if (!comm || !id) return fail(EDT_COMM_ERR_ARG, "comm / id is null");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return fail(EDT_COMM_ERR_ARG, "rank %d of %d ranks", rank, nranks);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    Comm* c = new Comm;
    c->rank = rank;
    c->nranks = nranks;
    ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(EDT_COMM_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    hipError_t e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
    if (e != hipSuccess) {
        (void)ncclCommDestroy(c->nccl);
        delete c;
        return fail(EDT_COMM_ERR_HIP, "hipStreamCreateWithFlags: %s", hipGetErrorString(e));
    }
    *comm = c;
    return 0;
}

int edt_comm_destroy(void* comm) {
    Comm* c = as_comm(comm);
    if (!c) return 0;
    if (c->side) (void)hipStreamSynchronize(c->side);
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    if (c->side) (void)hipStreamDestroy(c->side);
    ncclResult_t r = c->aborted ? ncclSuccess : ncclCommDestroy(c->nccl);   // abort already freed it
    delete c;
    if (r != ncclSuccess) return fail(EDT_COMM_ERR_RCCL, "ncclCommDestroy: %s", ncclGetErrorString(r));
    return 0;
}

int edt_comm_rank(const void* comm) { return comm ? static_cast<const Comm*>(comm)->rank : -1; }
int edt_comm_size(const void* comm) { return comm ? static_cast<const Comm*>(comm)->nranks : -1; }

int edt_comm_abort(void* comm) {
    Comm* c = as_comm(comm);
    if (!c) return fail(EDT_COMM_ERR_ARG, "null communicator");
    abort_comm(c);
    return 0;
}

int edt_comm_poll(void* comm) { return usable(as_comm(comm)); }

int edt_comm_set_timeout(void* comm, double seconds) {
    Comm* c = as_comm(comm);
    if (!c) return fail(EDT_COMM_ERR_ARG, "null communicator");
    if (!(seconds >= 0)) return fail(EDT_COMM_ERR_ARG, "timeout %g s", seconds);
    c->timeout_s = seconds;
    return 0;
}

int edt_comm_wait(void* comm, void* stream, double timeout_s) {
    Comm* c = as_comm(comm);
    if (int rc = usable(c)) return rc;
    if (int rc = ensure_events(c, 1)) return rc;
    hipEvent_t ev = c->events[0];
    EDT_HIP(hipEventRecord(ev, static_cast<hipStream_t>(stream)));
    if (int rc = wait_event(c, ev, timeout_s)) return rc;
    EDT_HIP(hipEventRecord(ev, c->side));                  // and the communicator's own stream
    return wait_event(c, ev, timeout_s);
}

int edt_comm_reduce_scatter_f32(void* comm, const float* send, float* recv, uint64_t count_per_rank,
                                void* stream) {
    Comm* c = as_comm(comm);
    if (int rc = usable(c)) return rc;
    if (count_per_rank && (!send || !recv)) return fail(EDT_COMM_ERR_ARG, "null buffer");
    EDT_RCCL(ncclReduceScatter(send, recv, count_per_rank, ncclFloat32, ncclSum, c->nccl,
                               static_cast<hipStream_t>(stream)));
    return 0;
}

int edt_comm_all_gather(void* comm, const void* send, void* recv, uint64_t count_per_rank, int dt,
                        void* stream) {
    Comm* c = as_comm(comm);
    ncclDataType_t t;
    uint64_t sz;
    if (int rc = usable(c)) return rc;
    if (count_per_rank && (!send || !recv)) return fail(EDT_COMM_ERR_ARG, "null buffer");
    if (!nccl_type(dt, &t, &sz)) return fail(EDT_COMM_ERR_ARG, "dtype %d", dt);
    EDT_RCCL(ncclAllGather(send, recv, count_per_rank, t, c->nccl, static_cast<hipStream_t>(stream)));
    return 0;
}

int edt_comm_all_to_all(void* comm, const void* send, void* recv, uint64_t count_per_rank, int dt,
                        void* stream) {
    Comm* c = as_comm(comm);
    ncclDataType_t t;
    uint64_t sz;
    if (int rc = usable(c)) return rc;
    if (count_per_rank && (!send || !recv)) return fail(EDT_COMM_ERR_ARG, "null buffer");
    if (!nccl_type(dt, &t, &sz)) return fail(EDT_COMM_ERR_ARG, "dtype %d", dt);
    EDT_RCCL(ncclAllToAll(send, recv, count_per_rank, t, c->nccl, static_cast<hipStream_t>(stream)));
    return 0;
}

int edt_comm_exchange(void* comm, const int32_t* send_to, const int32_t* recv_from,
                      const void* const* sendbufs, void* const* recvbufs, const uint64_t* bytes,
                      int nops, void* stream) {
    Comm* c = as_comm(comm);
    if (int rc = usable(c)) return rc;
    if (nops < 0 || (nops && (!send_to || !recv_from || !bytes)))
        return fail(EDT_COMM_ERR_ARG, "null op arrays");
    for (int i = 0; i < nops; ++i) {
        if (send_to[i] >= c->nranks || recv_from[i] >= c->nranks)
            return fail(EDT_COMM_ERR_ARG, "op %d names a rank outside [0, %d)", i, c->nranks);
        if ((send_to[i] >= 0 && (!sendbufs || !sendbufs[i])) || (recv_from[i] >= 0 && (!recvbufs || !recvbufs[i])))
            return fail(EDT_COMM_ERR_ARG, "op %d has no buffer", i);
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    EDT_RCCL(ncclGroupStart());
    for (int i = 0; i < nops; ++i) {
        if (send_to[i] >= 0) {
            ncclResult_t r = ncclSend(sendbufs[i], bytes[i], ncclUint8, send_to[i], c->nccl, s);
            if (r != ncclSuccess) { (void)ncclGroupEnd(); return fail(EDT_COMM_ERR_RCCL, "ncclSend op %d: %s", i, ncclGetErrorString(r)); }
        }
        if (recv_from[i] >= 0) {
            ncclResult_t r = ncclRecv(recvbufs[i], bytes[i], ncclUint8, recv_from[i], c->nccl, s);
            if (r != ncclSuccess) { (void)ncclGroupEnd(); return fail(EDT_COMM_ERR_RCCL, "ncclRecv op %d: %s", i, ncclGetErrorString(r)); }
        }
    }
    EDT_RCCL(ncclGroupEnd());
    return 0;
}

int edt_outer_step_sharded(void* comm, void* theta_g, int gdt, const void* const* theta_k, int wdt,
                           int K_local, void* momentum_shard, int has_momentum, uint64_t n_pad,
                           uint64_t bucket_elems, double lr, double momentum_coef, int nesterov,
                           float* acc, void* stream) {
    Comm* c = as_comm(comm);
    ncclDataType_t gt, wt;
    uint64_t gsz, wsz;
    if (int rc = usable(c)) return rc;
    if (!theta_g || !theta_k || !acc) return fail(EDT_COMM_ERR_ARG, "null buffer");
    if (!nccl_type(gdt, &gt, &gsz) || !nccl_type(wdt, &wt, &wsz)) return fail(EDT_COMM_ERR_ARG, "dtype pair %d/%d", gdt, wdt);
    if (K_local < 1 || K_local > EDT_MAX_WORKERS) return fail(EDT_COMM_ERR_ARG, "K_local %d", K_local);
    const uint64_t unit = (uint64_t)c->nranks * 64;
    if (n_pad % unit) return fail(EDT_COMM_ERR_ARG, "n_pad %llu is not a multiple of nranks x 64",
                                  (unsigned long long)n_pad);
    if (momentum_coef != 0 && !momentum_shard) return fail(EDT_COMM_ERR_ARG, "momentum shard is null");
    uint64_t bucket = bucket_elems / unit * unit;
    if (bucket < unit) bucket = unit;
    if (bucket > n_pad) bucket = n_pad;
    const uint64_t nb = n_pad ? (n_pad + bucket - 1) / bucket : 0;
    if (int rc = ensure_events(c, 2 * nb + 1)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int K_total = K_local * c->nranks;
    char* th = static_cast<char*>(theta_g);
    std::vector<const void*> wb(K_local);
    // phase 1: partial sums per bucket on `stream`; each bucket's reduce-scatter on the side
    // stream as soon as its partial is done
    for (uint64_t i = 0; i < nb; ++i) {
        const uint64_t b = i * bucket, e = b + bucket < n_pad ? b + bucket : n_pad, per = (e - b) / c->nranks;
        for (int k = 0; k < K_local; ++k) wb[k] = static_cast<const char*>(theta_k[k]) + b * wsz;
        int rc = edt_delta_partial(th + b * gsz, gdt, wb.data(), wdt, K_local, K_total, e - b, acc + b, 0, s);
        if (rc) return fail(EDT_COMM_ERR_ARG, "edt_delta_partial: %s", edt_last_error());
        EDT_HIP(hipEventRecord(c->events[2 * i], s));
        EDT_HIP(hipStreamWaitEvent(c->side, c->events[2 * i], 0));
        EDT_RCCL(ncclReduceScatter(acc + b, acc + b + (uint64_t)c->rank * per, per, ncclFloat32, ncclSum,
                                   c->nccl, c->side));
        EDT_HIP(hipEventRecord(c->events[2 * i + 1], c->side));
    }
    // phase 2: as each bucket's sum lands, SGD on the owned shard, then its all-gather
    uint64_t mom_off = 0;
    for (uint64_t i = 0; i < nb; ++i) {
        const uint64_t b = i * bucket, e = b + bucket < n_pad ? b + bucket : n_pad, per = (e - b) / c->nranks;
        const uint64_t s0 = b + (uint64_t)c->rank * per;
        EDT_HIP(hipStreamWaitEvent(s, c->events[2 * i + 1], 0));
        void* mom = momentum_shard ? static_cast<char*>(momentum_shard) + mom_off * gsz : nullptr;
        int rc = edt_sgd_apply(th + s0 * gsz, gdt, acc + s0, momentum_coef != 0 ? mom : nullptr, has_momentum,
                               per, lr, momentum_coef, nesterov, s);
        if (rc) return fail(EDT_COMM_ERR_ARG, "edt_sgd_apply: %s", edt_last_error());
        mom_off += per;
        EDT_HIP(hipEventRecord(c->events[2 * i], s));
        EDT_HIP(hipStreamWaitEvent(c->side, c->events[2 * i], 0));
        EDT_RCCL(ncclAllGather(th + s0 * gsz, th + b * gsz, per, gt, c->nccl, c->side));
    }
    // the caller's stream sees the gathered theta
    EDT_HIP(hipEventRecord(c->events[2 * nb], c->side));
    EDT_HIP(hipStreamWaitEvent(s, c->events[2 * nb], 0));
    // edt_comm_set_timeout > 0: wait here, polling RCCL's async error; a dead or stalled peer
    // aborts the communicator after the timeout and the step returns EDT_COMM_ERR_TIMEOUT
    // (the reference's master gives up on workers it stops hearing from, EDT_LM/diloco.py:46-71)
    if (c->timeout_s > 0) return wait_event(c, c->events[2 * nb], c->timeout_s);
    return 0;
}

int edt_outer_step_sharded_ordered(void* comm, void* theta_g, int gdt, const void* const* theta_k, int wdt,
                                   int K_local, void* momentum_shard, int has_momentum, uint64_t n_pad,
                                   uint64_t bucket_elems, double lr, double momentum_coef, int nesterov,
                                   float* acc, float* recv, void* stream) {
    Comm* c = as_comm(comm);
    ncclDataType_t gt, wt;
    uint64_t gsz, wsz;
    if (int rc = usable(c)) return rc;
    if (!theta_g || !theta_k || !acc || !recv) return fail(EDT_COMM_ERR_ARG, "null buffer");
    if (recv == acc) return fail(EDT_COMM_ERR_ARG, "recv must not alias acc (the all-to-all is out of place)");
    if (!nccl_type(gdt, &gt, &gsz) || !nccl_type(wdt, &wt, &wsz)) return fail(EDT_COMM_ERR_ARG, "dtype pair %d/%d", gdt, wdt);
    if (K_local < 1 || K_local > EDT_MAX_WORKERS) return fail(EDT_COMM_ERR_ARG, "K_local %d", K_local);
    if (c->nranks > EDT_MAX_WORKERS) return fail(EDT_COMM_ERR_ARG, "%d ranks: at most %d partials per shard", c->nranks,
                                                 EDT_MAX_WORKERS);
    const uint64_t unit = (uint64_t)c->nranks * 64;
    if (n_pad % unit) return fail(EDT_COMM_ERR_ARG, "n_pad %llu is not a multiple of nranks x 64",
                                  (unsigned long long)n_pad);
    if (momentum_coef != 0 && !momentum_shard) return fail(EDT_COMM_ERR_ARG, "momentum shard is null");
    uint64_t bucket = bucket_elems / unit * unit;
    if (bucket < unit) bucket = unit;
    if (bucket > n_pad) bucket = n_pad;
    const uint64_t nb = n_pad ? (n_pad + bucket - 1) / bucket : 0;
    if (int rc = ensure_events(c, 2 * nb + 1)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int K_total = K_local * c->nranks;
    char* th = static_cast<char*>(theta_g);
    std::vector<const void*> wb(K_local);
    // phase 1: per bucket the local fp32 partial on `stream` (laid out [dest rank][shard]), then
    // its all-to-all on the side stream: recv[b, e) arrives as [src rank][shard]
    for (uint64_t i = 0; i < nb; ++i) {
        const uint64_t b = i * bucket, e = b + bucket < n_pad ? b + bucket : n_pad, per = (e - b) / c->nranks;
        for (int k = 0; k < K_local; ++k) wb[k] = static_cast<const char*>(theta_k[k]) + b * wsz;
        int rc = edt_delta_partial(th + b * gsz, gdt, wb.data(), wdt, K_local, K_total, e - b, acc + b, 0, s);
        if (rc) return fail(EDT_COMM_ERR_ARG, "edt_delta_partial: %s", edt_last_error());
        EDT_HIP(hipEventRecord(c->events[2 * i], s));
        EDT_HIP(hipStreamWaitEvent(c->side, c->events[2 * i], 0));
        EDT_RCCL(ncclAllToAll(acc + b, recv + b, per, ncclFloat32, c->nccl, c->side));
        EDT_HIP(hipEventRecord(c->events[2 * i + 1], c->side));
    }
    // phase 2: the owned shard's N partials summed in rank order + SGD (edt_sgd_apply_sum), then
    // the shard's all-gather — the cross-rank sum has one order whatever RCCL's algorithm
    std::vector<const float*> parts(c->nranks);
    uint64_t mom_off = 0;
    for (uint64_t i = 0; i < nb; ++i) {
        const uint64_t b = i * bucket, e = b + bucket < n_pad ? b + bucket : n_pad, per = (e - b) / c->nranks;
        const uint64_t s0 = b + (uint64_t)c->rank * per;
        for (int r = 0; r < c->nranks; ++r) parts[r] = recv + b + (uint64_t)r * per;
        EDT_HIP(hipStreamWaitEvent(s, c->events[2 * i + 1], 0));
        void* mom = momentum_shard ? static_cast<char*>(momentum_shard) + mom_off * gsz : nullptr;
        int rc = edt_sgd_apply_sum(th + s0 * gsz, gdt, parts.data(), c->nranks, momentum_coef != 0 ? mom : nullptr,
                                   has_momentum, per, lr, momentum_coef, nesterov, s);
        if (rc) return fail(EDT_COMM_ERR_ARG, "edt_sgd_apply_sum: %s", edt_last_error());
        mom_off += per;
        EDT_HIP(hipEventRecord(c->events[2 * i], s));
        EDT_HIP(hipStreamWaitEvent(c->side, c->events[2 * i], 0));
        EDT_RCCL(ncclAllGather(th + s0 * gsz, th + b * gsz, per, gt, c->nccl, c->side));
    }
    EDT_HIP(hipEventRecord(c->events[2 * nb], c->side));
    EDT_HIP(hipStreamWaitEvent(s, c->events[2 * nb], 0));
    if (c->timeout_s > 0) return wait_event(c, c->events[2 * nb], c->timeout_s);
    return 0;
}

int edt_outer_step_sharded_exact(void* comm, void* theta_g, int gdt, const void* const* theta_k, int wdt,
                                 int K_local, void* momentum_shard, int has_momentum, uint64_t n_pad,
                                 uint64_t bucket_elems, double lr, double momentum_coef, int nesterov,
                                 void* const* recv, void* stream) {
    Comm* c = as_comm(comm);
    ncclDataType_t gt, wt;
    uint64_t gsz, wsz;
    if (int rc = usable(c)) return rc;
    if (!theta_g || !theta_k || !recv) return fail(EDT_COMM_ERR_ARG, "null buffer");
    if (!nccl_type(gdt, &gt, &gsz) || !nccl_type(wdt, &wt, &wsz)) return fail(EDT_COMM_ERR_ARG, "dtype pair %d/%d", gdt, wdt);
    if (K_local < 1 || (int64_t)K_local * c->nranks > EDT_MAX_WORKERS)
        return fail(EDT_COMM_ERR_ARG, "K_local %d x %d ranks: the fused step takes at most %d workers", K_local,
                    c->nranks, EDT_MAX_WORKERS);
    for (int j = 0; j < K_local; ++j)
        if (!theta_k[j] || !recv[j]) return fail(EDT_COMM_ERR_ARG, "worker %d: null arena or receive buffer", j);
    const uint64_t unit = (uint64_t)c->nranks * 64;
    if (n_pad % unit) return fail(EDT_COMM_ERR_ARG, "n_pad %llu is not a multiple of nranks x 64",
                                  (unsigned long long)n_pad);
    if (momentum_coef != 0 && !momentum_shard) return fail(EDT_COMM_ERR_ARG, "momentum shard is null");
    uint64_t bucket = bucket_elems / unit * unit;
    if (bucket < unit) bucket = unit;
    if (bucket > n_pad) bucket = n_pad;
    const uint64_t nb = n_pad ? (n_pad + bucket - 1) / bucket : 0;
    if (int rc = ensure_events(c, 2 * nb + 2)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int K_total = K_local * c->nranks;
    char* th = static_cast<char*>(theta_g);
    // phase 1 (side stream, after the caller's work on the arenas): every bucket's all-to-all, one
    // per local worker, straight from the arenas — a worker's bucket is already laid out
    // [dest rank][shard] and arrives in recv[j] as [src rank][shard]
    EDT_HIP(hipEventRecord(c->events[2 * nb + 1], s));
    EDT_HIP(hipStreamWaitEvent(c->side, c->events[2 * nb + 1], 0));
    for (uint64_t i = 0; i < nb; ++i) {
        const uint64_t b = i * bucket, e = b + bucket < n_pad ? b + bucket : n_pad, per = (e - b) / c->nranks;
        EDT_RCCL(ncclGroupStart());
        for (int j = 0; j < K_local; ++j) {
            ncclResult_t r = ncclAllToAll(static_cast<const char*>(theta_k[j]) + b * wsz,
                                          static_cast<char*>(recv[j]) + b * wsz, per, wt, c->nccl, c->side);
            if (r != ncclSuccess) {
                (void)ncclGroupEnd();
                return fail(EDT_COMM_ERR_RCCL, "ncclAllToAll worker %d: %s", j, ncclGetErrorString(r));
            }
        }
        EDT_RCCL(ncclGroupEnd());
        EDT_HIP(hipEventRecord(c->events[2 * i + 1], c->side));
    }
    // phase 2: as each bucket lands, the single-GPU fused step on the owned shard with the K_total
    // workers in the reference's order (global worker k = src rank x K_local + j): bit-exact with
    // edt_outer_step over the whole population; then the shard's all-gather into theta
    std::vector<const void*> shards(K_total);
    uint64_t mom_off = 0;
    for (uint64_t i = 0; i < nb; ++i) {
        const uint64_t b = i * bucket, e = b + bucket < n_pad ? b + bucket : n_pad, per = (e - b) / c->nranks;
        const uint64_t s0 = b + (uint64_t)c->rank * per;
        for (int src = 0; src < c->nranks; ++src)
            for (int j = 0; j < K_local; ++j)
                shards[src * K_local + j] = static_cast<const char*>(recv[j]) + (b + (uint64_t)src * per) * wsz;
        EDT_HIP(hipStreamWaitEvent(s, c->events[2 * i + 1], 0));
        void* mom = momentum_shard ? static_cast<char*>(momentum_shard) + mom_off * gsz : nullptr;
        int rc = edt_outer_step(th + s0 * gsz, gdt, shards.data(), wdt, K_total, momentum_coef != 0 ? mom : nullptr,
                                has_momentum, per, lr, momentum_coef, nesterov, s);
        if (rc) return fail(EDT_COMM_ERR_ARG, "edt_outer_step: %s", edt_last_error());
        mom_off += per;
        EDT_HIP(hipEventRecord(c->events[2 * i], s));
        EDT_HIP(hipStreamWaitEvent(c->side, c->events[2 * i], 0));
        EDT_RCCL(ncclAllGather(th + s0 * gsz, th + b * gsz, per, gt, c->nccl, c->side));
    }
    EDT_HIP(hipEventRecord(c->events[2 * nb], c->side));
    EDT_HIP(hipStreamWaitEvent(s, c->events[2 * nb], 0));
    if (c->timeout_s > 0) return wait_event(c, c->events[2 * nb], c->timeout_s);
    return 0;
}

const char* edt_comm_last_error(void) { return g_err; }

}  // extern "C"
