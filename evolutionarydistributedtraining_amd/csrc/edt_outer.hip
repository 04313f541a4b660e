// edt_outer.hip — the DiLoCo outer step (EDT_LM/diloco.py:238-289): the fused kernel over flat
// arenas or tensor lists, its sharded halves (partial sums, SGD on a shard) and the stream-ceiling
// probe, with their C ABI entries (include/edt_sync.h).
#include "edt_common.h"

namespace {

// ---------------------------------------------------------------------------------------
// DiLoCo outer step

struct Workers {
    const void* p[EDT_MAX_WORKERS];
};

struct OuterArgs {
    void* theta;
    void* mom;
    float* acc_out;      // partial mode
    uint64_t n;
    int K;               // workers in this launch
    float kdiv;          // divisor (K_total)
    float kinv;          // 1/K_total when K_total is a power of two
    int div_exact;       // 1: true division, 0: multiply by kinv (identical for powers of two)
    int accumulate;      // partial mode: add into acc_out
    void* acc_ws;        // chain mode: running sum in theta's dtype between launches
    int acc_in;          // chain mode: start from acc_ws
    int acc_store;       // chain mode: store the running sum to acc_ws (no SGD)
    SgdScalars sgd;
    Workers w;
    Workers bc;          // broadcast mode: round_w(theta_new) stored to these (worker dtype)
    int nbc;
    __device__ __forceinline__ const void* wp(int k) const { return w.p[k]; }
};

// One tensor of a tensor-list launch (outer_list_kernel), seen through outer_elems: the same
// fields, worker pointers read from the device-resident table (theta_k[k * T + t]).
struct TensorArgs {
    void* theta;
    void* mom;
    float* acc_out;
    int K;
    float kdiv;
    float kinv;
    int accumulate;
    void* acc_ws;
    int acc_in;
    int acc_store;
    SgdScalars sgd;
    const void* const* w;
    uint64_t T;
    uint64_t t;
    __device__ __forceinline__ const void* wp(int k) const { return w[(uint64_t)k * T + t]; }
};

// MODE_CHAIN = MODE_FUSED for populations above EDT_MAX_WORKERS: launches of <= 64 workers
// carry the running sum in theta's dtype (lossless: it is rounded to that dtype after every add).
enum { MODE_FUSED = 0, MODE_PARTIAL = 1, MODE_CHAIN = 2 };

// Per-element accumulation acc = sum_k round(round(w_k - g) / K) in the precision of GDT
// (worker-major order, EDT_LM/diloco.py:243-246). MODE_PARTIAL sums the rounded quotients
// in fp32 instead (the cross-rank sum is then an fp32 RCCL reduction).
template <int GDT, int WDT, int KC, int DIV, int MODE, int N, class A, int H2 = 4, bool BC = false>
__device__ __forceinline__ void outer_elems(const A& a, uint64_t i) {
    float g[N], acc[N], b_in[N];
    ld<GDT, N, (EDT_NT_RMW != 0), H2>(a.theta, i, g);
    if constexpr (MODE != MODE_PARTIAL) ld_momentum<GDT, N, H2>(a.mom, i, a.sgd, b_in);
    if (MODE == MODE_PARTIAL && a.accumulate) {
        ld<EDT_F32, N, false, H2>(a.acc_out, i, acc);      // continue the running sum in worker order
    } else if (MODE == MODE_CHAIN && a.acc_in) {
        ld<GDT, N, false, H2>(a.acc_ws, i, acc);
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) acc[j] = 0.f;
    }
    const int K = KC > 0 ? KC : a.K;
    auto body = [&](int k) {
        float w[N];
        ld<WDT, N, nt_worker_loads<WDT, H2>(), H2>(a.wp(k), i, w);
#pragma unroll
        for (int j = 0; j < N; ++j) w[j] = w[j] - g[j];              // trained - base
        rnd<GDT>(w);
        if constexpr (DIV) {
#pragma unroll
            for (int j = 0; j < N; ++j) w[j] = w[j] / a.kdiv;        // delta / num_models
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) w[j] = w[j] * a.kinv;
        }
        rnd<GDT>(w);
#pragma unroll
        for (int j = 0; j < N; ++j) acc[j] = acc[j] + w[j];          // acc += delta / K
        if constexpr (MODE != MODE_PARTIAL) rnd<GDT>(acc);
    };
    if constexpr (KC > 0) {
#pragma unroll
        for (int k = 0; k < KC; ++k) body(k);
    } else {
#pragma unroll 4
        for (int k = 0; k < K; ++k) body(k);
    }
    if constexpr (MODE == MODE_PARTIAL) {
        st<EDT_F32, N, (EDT_NT_STORES != 0), H2>(a.acc_out, i, acc);
    } else if (MODE == MODE_CHAIN && a.acc_store) {
        st<GDT, N, (EDT_NT_STORES != 0), H2>(a.acc_ws, i, acc);
    } else {
        float grad[N];
#pragma unroll
        for (int j = 0; j < N; ++j) grad[j] = -acc[j];               // p.grad = -avg_delta
        sgd_update<GDT, N, H2>(g, grad, a.mom, i, a.sgd, b_in);
        st<GDT, N, (EDT_NT_STORES != 0), H2>(a.theta, i, g);
        if constexpr (BC) {
            // the broadcast of EDT_LM/diloco.py:302-308 fused in: every destination starts the
            // next inner loop from theta_new rounded to the worker dtype (torch copy_: RNE). A
            // destination may be a worker this thread just read (same elements, same thread).
#pragma unroll 4
            for (int k = 0; k < a.nbc; ++k) st<WDT, N, (EDT_NT_STORES != 0), H2>(const_cast<void*>(a.bc.p[k]), i, g);
        }
    }
}

// DIV = 1: true division by K (torch CPU `delta / num_models`); DIV = 0: multiply by 1/K,
// bit-identical when K is a power of two.
// BC: also store round_w(theta_new) into a.bc (edt_outer_step_bcast).
template <int GDT, int WDT, int KC, int DIV, int MODE, int N, bool BC = false>
__global__ __launch_bounds__(kBlock, EDT_MIN_WAVES) void outer_kernel(OuterArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = xcd_block(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    if constexpr (N == kVec && split_halves<GDT, WDT>()) {
        // tiles of kBlock x 8 elements; thread t owns [4t, 4t+4) and [4(kBlock+t), +4) of a tile
        constexpr int H2 = 4 * kBlock;
        const uint64_t nv = a.n / (kVec * kBlock) * kBlock;
        for (uint64_t v = tid; v < nv; v += stride)
            outer_elems<GDT, WDT, KC, DIV, MODE, kVec, OuterArgs, H2, BC>(a, v * kVec - 4 * threadIdx.x);
        for (uint64_t e = nv * kVec + tid; e < a.n; e += stride)     // scalar tail (< 8 x kBlock)
            outer_elems<GDT, WDT, KC, DIV, MODE, 1, OuterArgs, 4, BC>(a, e);
    } else if constexpr (N == kVec) {
        const uint64_t nv = a.n / kVec;
        for (uint64_t v = tid; v < nv; v += stride)
            outer_elems<GDT, WDT, KC, DIV, MODE, kVec, OuterArgs, 4, BC>(a, v * kVec);
        const uint64_t t = nv * kVec + tid;      // scalar tail (< 8 elements)
        if (t < a.n) outer_elems<GDT, WDT, KC, DIV, MODE, 1, OuterArgs, 4, BC>(a, t);
    } else {
        for (uint64_t e = tid; e < a.n; e += stride) outer_elems<GDT, WDT, KC, DIV, MODE, 1, OuterArgs, 4, BC>(a, e);
    }
}

// Tensor-list form: the parameters are T separate allocations (HF models loaded straight to
// the GPU), described by a table in device memory. The flat index space is cut into chunks of
// kListChunk elements that never cross a tensor; a grid-stride loop (as outer_kernel's) hands
// chunk b to a workgroup, which finds its tensor t by a binary search over the chunk prefix
// sums (uniform across the workgroup) and runs the same per-thread 8-element body as
// outer_kernel on it. Tensors whose operands are not all 16-byte aligned take the scalar body.
#ifndef EDT_LIST_ITERS          // 8-element iterations per thread per chunk
#define EDT_LIST_ITERS 2        // measured: 2-4 with the grid-stride loop beat 1 and 8-64
#endif
constexpr uint64_t kListChunk = (uint64_t)kBlock * kVec * EDT_LIST_ITERS;   // 4096 elements
constexpr uint64_t kVecFlag = 1ull << 63;                          // numel[t] bit: vector body ok

struct ListArgs {
    const uint64_t* prefix;     // T + 1 chunk prefix sums
    const uint64_t* numel;      // T, kVecFlag | numel
    void* const* theta;         // T
    void* const* mom;           // T (unused without momentum)
    const void* const* w;       // K * T, worker-major
    uint64_t T;
    uint64_t chunks;            // prefix[T]
    int K;
    float kdiv;
    float kinv;
    SgdScalars sgd;
    const uint8_t* tail;        // nullable: bf16 scalar-tail bits, tensor t's from byte tail_off[t]
    const uint64_t* tail_off;   // T
};

template <int GDT, int WDT, int KC, int DIV>
__device__ __forceinline__ void outer_list_chunk(const ListArgs& L, const uint64_t* prefix, uint64_t b) {
    uint64_t lo = 0, hi = L.T;                       // last t with prefix[t] <= b
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (prefix[mid] <= b) lo = mid;
        else hi = mid;
    }
    const uint64_t t = lo;
    const uint64_t nf = L.numel[t];
    const uint64_t n = nf & ~kVecFlag;
    const uint64_t c0 = (b - prefix[t]) * kListChunk;
    const uint64_t c1 = c0 + kListChunk < n ? c0 + kListChunk : n;
    TensorArgs a;
    a.theta = L.theta[t];
    a.mom = L.sgd.use_momentum ? L.mom[t] : nullptr;
    a.acc_out = nullptr;
    a.K = L.K;
    a.kdiv = L.kdiv;
    a.kinv = L.kinv;
    a.accumulate = 0;
    a.acc_ws = nullptr;
    a.acc_in = 0;
    a.acc_store = 0;
    a.sgd = L.sgd;
    if (L.tail) a.sgd.tail = L.tail + L.tail_off[t];     // the tensor's own bits, indexed locally
    a.w = L.w;
    a.T = L.T;
    a.t = t;
    if ((nf & kVecFlag) && split_halves<GDT, WDT>()) {
        // tiles of kBlock x 8 elements in split-halves order (as outer_kernel), then a scalar tail
        constexpr uint64_t tile = (uint64_t)kBlock * kVec;
        const uint64_t vend = c0 + (c1 - c0) / tile * tile;
        for (uint64_t i = c0 + 4ull * threadIdx.x; i < vend; i += tile)
            outer_elems<GDT, WDT, KC, DIV, MODE_FUSED, kVec, TensorArgs, 4 * kBlock>(a, i);
        for (uint64_t i = vend + threadIdx.x; i < c1; i += kBlock)
            outer_elems<GDT, WDT, KC, DIV, MODE_FUSED, 1>(a, i);
    } else if (nf & kVecFlag) {
        const uint64_t vend = c0 + (c1 - c0) / kVec * kVec;
        for (uint64_t i = c0 + (uint64_t)threadIdx.x * kVec; i < vend; i += (uint64_t)kBlock * kVec)
            outer_elems<GDT, WDT, KC, DIV, MODE_FUSED, kVec>(a, i);
        const uint64_t i = vend + threadIdx.x;
        if (i < c1) outer_elems<GDT, WDT, KC, DIV, MODE_FUSED, 1>(a, i);
    } else {
        for (uint64_t i = c0 + threadIdx.x; i < c1; i += kBlock)
            outer_elems<GDT, WDT, KC, DIV, MODE_FUSED, 1>(a, i);
    }
}

// LDS = true: the chunk prefix sums are staged in LDS once per workgroup (dynamic shared
// memory, (T + 1) x 8 bytes), so the per-chunk tensor search costs LDS reads, not a chain of
// dependent global loads; LDS = false (very long tensor lists) searches the global table.
template <int GDT, int WDT, int KC, int DIV, bool LDS>
__global__ __launch_bounds__(kBlock, EDT_MIN_WAVES) void outer_list_kernel(ListArgs L) {
    extern __shared__ uint64_t s_prefix[];
    const uint64_t* prefix = L.prefix;
    if constexpr (LDS) {
        for (uint64_t i = threadIdx.x; i <= L.T; i += kBlock) s_prefix[i] = L.prefix[i];
        __syncthreads();
        prefix = s_prefix;
    }
    for (uint64_t b = blockIdx.x; b < L.chunks; b += gridDim.x) outer_list_chunk<GDT, WDT, KC, DIV>(L, prefix, b);
}

// SGD from a reduced fp32 sum (sharded multi-GPU step).
template <int GDT, int N>
__global__ __launch_bounds__(kBlock) void sgd_apply_kernel(void* theta, const float* acc, void* mom,
                                                           uint64_t n, SgdScalars s) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    auto elems = [&](auto tagN, uint64_t i) {
        constexpr int M = decltype(tagN)::value;
        float g[M], a[M], grad[M], b_in[M];
        ld<GDT, M>(theta, i, g);
        ld<EDT_F32, M>(acc, i, a);
        ld_momentum<GDT, M>(mom, i, s, b_in);
        rnd<GDT>(a);
#pragma unroll
        for (int j = 0; j < M; ++j) grad[j] = -a[j];
        sgd_update<GDT, M>(g, grad, mom, i, s, b_in);
        st<GDT, M>(theta, i, g);
    };
    using V8 = std::integral_constant<int, kVec>;
    using V1 = std::integral_constant<int, 1>;
    if constexpr (N == kVec) {
        const uint64_t nv = n / kVec;
        for (uint64_t v = tid; v < nv; v += stride) elems(V8{}, v * kVec);
        const uint64_t t = nv * kVec + tid;
        if (t < n) elems(V1{}, t);
    } else {
        for (uint64_t e = tid; e < n; e += stride) elems(V1{}, e);
    }
}


// SGD from N per-rank fp32 partial sums of the same shard, summed in rank order (the sharded
// step's "reduce_ordered" schedule: an all-to-all delivers every rank's partial of the owned
// shard, so the cross-rank sum has one fixed order whatever the collective library does).
struct Partials {
    const float* p[EDT_MAX_WORKERS];
};

template <int GDT, int N>
__global__ __launch_bounds__(kBlock) void sgd_apply_sum_kernel(void* theta, Partials P, int np, void* mom,
                                                               uint64_t n, SgdScalars s) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    auto elems = [&](auto tagN, uint64_t i) {
        constexpr int M = decltype(tagN)::value;
        float g[M], a[M], grad[M], b_in[M];
        ld<GDT, M>(theta, i, g);
        ld_momentum<GDT, M>(mom, i, s, b_in);
        ld<EDT_F32, M>(P.p[0], i, a);
        for (int r = 1; r < np; ++r) {              // rank order
            float x[M];
            ld<EDT_F32, M>(P.p[r], i, x);
#pragma unroll
            for (int j = 0; j < M; ++j) a[j] = a[j] + x[j];
        }
        rnd<GDT>(a);
#pragma unroll
        for (int j = 0; j < M; ++j) grad[j] = -a[j];
        sgd_update<GDT, M>(g, grad, mom, i, s, b_in);
        st<GDT, M>(theta, i, g);
    };
    using V8 = std::integral_constant<int, kVec>;
    using V1 = std::integral_constant<int, 1>;
    if constexpr (N == kVec) {
        const uint64_t nv = n / kVec;
        for (uint64_t v = tid; v < nv; v += stride) elems(V8{}, v * kVec);
        const uint64_t t = nv * kVec + tid;
        if (t < n) elems(V1{}, t);
    } else {
        for (uint64_t e = tid; e < n; e += stride) elems(V1{}, e);
    }
}


// ---------------------------------------------------------------------------------------
// Diagnostic: the fused step's access pattern (same operands, loads, stores, cache policy, grid)
// with a trivial body. Its time is the memory-system ceiling of the step on the device at hand:
// the fused kernel's time over it says how much of the step is anything but HBM traffic.

template <int GDT, int WDT, int KC, int N, int H2 = 4>
__device__ __forceinline__ void probe_elems(const OuterArgs& a, uint64_t i) {
    float g[N], b[N], acc[N];
    ld<GDT, N, false, H2>(a.theta, i, g);
    ld<GDT, N, false, H2>(a.mom, i, b);
#pragma unroll
    for (int j = 0; j < N; ++j) acc[j] = 0.f;
    const int K = KC > 0 ? KC : a.K;
#pragma unroll 8
    for (int k = 0; k < K; ++k) {
        float w[N];
        ld<WDT, N, nt_worker_loads<WDT, H2>(), H2>(a.wp(k), i, w);
#pragma unroll
        for (int j = 0; j < N; ++j) acc[j] += w[j];
    }
#pragma unroll
    for (int j = 0; j < N; ++j) { g[j] += acc[j] * 1e-30f; b[j] += acc[j] * 1e-30f; }
    st<GDT, N, (EDT_NT_STORES != 0), H2>(a.theta, i, g);
    st<GDT, N, (EDT_NT_STORES != 0), H2>(a.mom, i, b);
}

template <int GDT, int WDT, int KC>
__global__ __launch_bounds__(kBlock, EDT_MIN_WAVES) void probe_kernel(OuterArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if constexpr (split_halves<GDT, WDT>()) {
        constexpr int H2 = 4 * kBlock;
        const uint64_t nv = a.n / (kVec * kBlock) * kBlock;
        for (uint64_t v = tid; v < nv; v += stride) probe_elems<GDT, WDT, KC, kVec, H2>(a, v * kVec - 4 * threadIdx.x);
        for (uint64_t e = nv * kVec + tid; e < a.n; e += stride) probe_elems<GDT, WDT, KC, 1>(a, e);
    } else {
        const uint64_t nv = a.n / kVec;
        for (uint64_t v = tid; v < nv; v += stride) probe_elems<GDT, WDT, KC, kVec>(a, v * kVec);
        const uint64_t t = nv * kVec + tid;
        if (t < a.n) probe_elems<GDT, WDT, KC, 1>(a, t);
    }
}


// ---------------------------------------------------------------------------------------
// launch helpers

template <int GDT, int WDT, int MODE, bool BC = false>
int launch_outer_k(const OuterArgs& a, bool vec, hipStream_t s) {
    const unsigned g = grid_for(a.n, vec);
#define EDT_LAUNCH_K(KC, DIV)                                                                    \
    do {                                                                                         \
        if (vec) outer_kernel<GDT, WDT, KC, DIV, MODE, kVec, BC><<<g, kBlock, 0, s>>>(a);        \
        else outer_kernel<GDT, WDT, KC, DIV, MODE, 1, BC><<<g, kBlock, 0, s>>>(a);               \
    } while (0)
    // compile-time worker counts for the common populations; the divisor is K_total
    if constexpr (MODE == MODE_CHAIN) {
        if (a.div_exact) EDT_LAUNCH_K(0, 1);
        else EDT_LAUNCH_K(0, 0);
        return check_launch("outer_kernel");
    }
    if (a.K == 1 && !a.div_exact) EDT_LAUNCH_K(1, 0);
    else if (a.K == 2 && !a.div_exact) EDT_LAUNCH_K(2, 0);
    else if (a.K == 3 && a.div_exact) EDT_LAUNCH_K(3, 1);
    else if (a.K == 4 && !a.div_exact) EDT_LAUNCH_K(4, 0);
    else if (a.K == 8 && !a.div_exact) EDT_LAUNCH_K(8, 0);
    else if (a.div_exact) EDT_LAUNCH_K(0, 1);
    else EDT_LAUNCH_K(0, 0);
#undef EDT_LAUNCH_K
    return check_launch("outer_kernel");
}

template <int MODE, bool BC = false>
int launch_outer(int gdt, int wdt, const OuterArgs& a, bool vec, hipStream_t s) {
    if (gdt == EDT_F32 && wdt == EDT_F32) return launch_outer_k<EDT_F32, EDT_F32, MODE, BC>(a, vec, s);
    if (gdt == EDT_F32 && wdt == EDT_BF16) return launch_outer_k<EDT_F32, EDT_BF16, MODE, BC>(a, vec, s);
    return launch_outer_k<EDT_BF16, EDT_BF16, MODE, BC>(a, vec, s);
}

constexpr uint64_t kListLdsMaxTensors = 8191;          // (T + 1) x 8 B <= 64 KiB of LDS

template <int GDT, int WDT>
int launch_list_k(const ListArgs& L, int div_exact, unsigned grid, hipStream_t s) {
    const bool lds = L.T <= kListLdsMaxTensors;
    const size_t shm = lds ? (size_t)(L.T + 1) * sizeof(uint64_t) : 0;
#define EDT_LAUNCH_L(KC, DIV)                                                                    \
    do {                                                                                         \
        if (lds) outer_list_kernel<GDT, WDT, KC, DIV, true><<<grid, kBlock, shm, s>>>(L);        \
        else outer_list_kernel<GDT, WDT, KC, DIV, false><<<grid, kBlock, 0, s>>>(L);             \
    } while (0)
    if (L.K == 1 && !div_exact) EDT_LAUNCH_L(1, 0);
    else if (L.K == 2 && !div_exact) EDT_LAUNCH_L(2, 0);
    else if (L.K == 3 && div_exact) EDT_LAUNCH_L(3, 1);
    else if (L.K == 4 && !div_exact) EDT_LAUNCH_L(4, 0);
    else if (L.K == 8 && !div_exact) EDT_LAUNCH_L(8, 0);
    else if (div_exact) EDT_LAUNCH_L(0, 1);
    else EDT_LAUNCH_L(0, 0);
#undef EDT_LAUNCH_L
    return check_launch("outer_list_kernel");
}


int fill_outer(OuterArgs& a, const void* theta, const void* const* theta_k, int K, int K_total, uint64_t n) {
    memset(&a, 0, sizeof(a));
    if (!theta && n) return fail(EDT_ERR_ARG, "theta_g is null");
    if (K < 1 || K > EDT_MAX_WORKERS)
        return fail(EDT_ERR_ARG, "worker count %d out of range [1, %d]", K, EDT_MAX_WORKERS);
    if (K_total < 1) return fail(EDT_ERR_ARG, "total worker count %d < 1", K_total);
    if (!theta_k) return fail(EDT_ERR_ARG, "theta_k is null");
    for (int k = 0; k < K; ++k) {
        if (!theta_k[k] && n) return fail(EDT_ERR_ARG, "theta_k[%d] is null", k);
        a.w.p[k] = theta_k[k];
    }
    a.theta = const_cast<void*>(theta);
    a.n = n;
    a.K = K;
    a.kdiv = (float)K_total;
    a.kinv = 1.0f / (float)K_total;
    a.div_exact = is_pow2(K_total) ? 0 : 1;
    return EDT_OK;
}


}  // namespace

extern "C" {

int edt_probe_stream(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K, void* momentum,
                     uint64_t n, void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    OuterArgs a;
    int rc = fill_outer(a, theta_g, theta_k, K, K, n);
    if (rc) return rc;
    if (!momentum) return fail(EDT_ERR_ARG, "momentum is null");
    a.mom = momentum;
    bool vec = aligned16(theta_g) && aligned16(momentum);
    for (int k = 0; k < K; ++k) vec = vec && aligned16(theta_k[k]);
    if (!vec) return fail(EDT_ERR_ARG, "the probe needs 16-byte aligned operands");
    if (n == 0) return EDT_OK;
    const unsigned g = grid_for(n, true);
    hipStream_t s = (hipStream_t)stream;
    if (gdt == EDT_F32 && wdt == EDT_BF16) {
        if (K == 8) probe_kernel<EDT_F32, EDT_BF16, 8><<<g, kBlock, 0, s>>>(a);
        else probe_kernel<EDT_F32, EDT_BF16, 0><<<g, kBlock, 0, s>>>(a);
    } else if (gdt == EDT_F32) {
        if (K == 8) probe_kernel<EDT_F32, EDT_F32, 8><<<g, kBlock, 0, s>>>(a);
        else probe_kernel<EDT_F32, EDT_F32, 0><<<g, kBlock, 0, s>>>(a);
    } else {
        if (K == 8) probe_kernel<EDT_BF16, EDT_BF16, 8><<<g, kBlock, 0, s>>>(a);
        else probe_kernel<EDT_BF16, EDT_BF16, 0><<<g, kBlock, 0, s>>>(a);
    }
    return check_launch("probe_kernel");
}

int edt_outer_step_bytes_per_elem(int gdt, int wdt, int K, int with_momentum) {
    const int bg = gdt == EDT_BF16 ? 2 : 4, bw = wdt == EDT_BF16 ? 2 : 4;
    return K * bw + 2 * bg + (with_momentum ? 2 * bg : 0);
}

int edt_outer_step(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K,
                   void* momentum, int has_momentum, uint64_t n, double lr, double momentum_coef,
                   int nesterov, void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    OuterArgs a;
    int rc = fill_outer(a, theta_g, theta_k, K, K, n);
    if (rc) return rc;
    a.sgd = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (a.sgd.use_momentum && !momentum && n) return fail(EDT_ERR_ARG, "momentum buffer is null");
    a.mom = momentum;
    if (n == 0) return EDT_OK;
    bool vec = aligned16(theta_g) && (!a.sgd.use_momentum || aligned16(momentum));
    for (int k = 0; k < K; ++k) vec = vec && aligned16(theta_k[k]);
    return launch_outer<MODE_FUSED>(gdt, wdt, a, vec, (hipStream_t)stream);
}

int edt_outer_step_tail(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K,
                        void* momentum, int has_momentum, uint64_t n, double lr, double momentum_coef,
                        int nesterov, const uint8_t* tail_bits, void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    OuterArgs a;
    int rc = fill_outer(a, theta_g, theta_k, K, K, n);
    if (rc) return rc;
    a.sgd = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (a.sgd.use_momentum && !momentum && n) return fail(EDT_ERR_ARG, "momentum buffer is null");
    a.mom = momentum;
    if (gdt == EDT_BF16) a.sgd.tail = tail_bits;    // fp32: torch's tails are FMAs too, nothing to emulate
    if (n == 0) return EDT_OK;
    bool vec = aligned16(theta_g) && (!a.sgd.use_momentum || aligned16(momentum));
    for (int k = 0; k < K; ++k) vec = vec && aligned16(theta_k[k]);
    return launch_outer<MODE_FUSED>(gdt, wdt, a, vec, (hipStream_t)stream);
}

int edt_outer_step_bcast(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K,
                         void* momentum, int has_momentum, uint64_t n, double lr, double momentum_coef,
                         int nesterov, void* const* bcast, int nbcast, void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    if (nbcast < 0 || nbcast > EDT_MAX_WORKERS)
        return fail(EDT_ERR_ARG, "broadcast count %d out of range [0, %d]", nbcast, EDT_MAX_WORKERS);
    if (nbcast == 0)
        return edt_outer_step(theta_g, gdt, theta_k, wdt, K, momentum, has_momentum, n, lr, momentum_coef, nesterov,
                              stream);
    OuterArgs a;
    int rc = fill_outer(a, theta_g, theta_k, K, K, n);
    if (rc) return rc;
    a.sgd = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (a.sgd.use_momentum && !momentum && n) return fail(EDT_ERR_ARG, "momentum buffer is null");
    a.mom = momentum;
    if (!bcast) return fail(EDT_ERR_ARG, "bcast is null");
    const uintptr_t t0 = reinterpret_cast<uintptr_t>(theta_g), t1 = t0 + n * (gdt == EDT_BF16 ? 2 : 4);
    for (int k = 0; k < nbcast; ++k) {
        if (!bcast[k] && n) return fail(EDT_ERR_ARG, "bcast[%d] is null", k);
        const uintptr_t b0 = reinterpret_cast<uintptr_t>(bcast[k]), b1 = b0 + n * (wdt == EDT_BF16 ? 2 : 4);
        if (n && b0 < t1 && t0 < b1) return fail(EDT_ERR_ARG, "bcast[%d] overlaps theta_g", k);
        a.bc.p[k] = bcast[k];
    }
    a.nbc = nbcast;
    if (n == 0) return EDT_OK;
    bool vec = aligned16(theta_g) && (!a.sgd.use_momentum || aligned16(momentum));
    for (int k = 0; k < K; ++k) vec = vec && aligned16(theta_k[k]);
    for (int k = 0; k < nbcast; ++k) vec = vec && aligned16(bcast[k]);
    return launch_outer<MODE_FUSED, true>(gdt, wdt, a, vec, (hipStream_t)stream);
}

int edt_outer_step_ws(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K, void* momentum,
                      int has_momentum, uint64_t n, double lr, double momentum_coef, int nesterov, void* workspace,
                      void* stream) {
    if (K <= EDT_MAX_WORKERS)
        return edt_outer_step(theta_g, gdt, theta_k, wdt, K, momentum, has_momentum, n, lr, momentum_coef, nesterov,
                              stream);
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    if (!workspace && n) return fail(EDT_ERR_ARG, "K = %d > %d needs a workspace of n elements of theta's dtype",
                                     K, EDT_MAX_WORKERS);
    if (!theta_k) return fail(EDT_ERR_ARG, "theta_k is null");
    const SgdScalars sg = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (sg.use_momentum && !momentum && n) return fail(EDT_ERR_ARG, "momentum buffer is null");
    if (n == 0) return EDT_OK;
    bool vec = aligned16(theta_g) && aligned16(workspace) && (!sg.use_momentum || aligned16(momentum));
    for (int k = 0; k < K; ++k) vec = vec && theta_k[k] && aligned16(theta_k[k]);
    for (int k0 = 0; k0 < K; k0 += EDT_MAX_WORKERS) {       // worker order preserved across launches
        const int kc = K - k0 < EDT_MAX_WORKERS ? K - k0 : EDT_MAX_WORKERS;
        OuterArgs a;
        int rc = fill_outer(a, theta_g, theta_k + k0, kc, K, n);
        if (rc) return rc;
        a.sgd = sg;
        a.mom = momentum;
        a.acc_ws = workspace;
        a.acc_in = k0 > 0;
        a.acc_store = k0 + kc < K;
        rc = launch_outer<MODE_CHAIN>(gdt, wdt, a, vec, (hipStream_t)stream);
        if (rc) return rc;
    }
    return EDT_OK;
}

uint64_t edt_outer_list_workspace_bytes(int T, int K) {
    if (T < 0 || K < 1) return 0;
    return (uint64_t)(5 * (uint64_t)T + 1 + (uint64_t)K * T) * sizeof(uint64_t);
}

}   // extern "C"

static int outer_step_list_impl(void* const* theta_t, int gdt, const void* const* theta_k, int wdt, int K,
                                void* const* momentum_t, int has_momentum, const uint64_t* numel, int T,
                                double lr, double momentum_coef, int nesterov, const uint8_t* tail,
                                const uint64_t* tail_off, void* workspace, uint64_t workspace_bytes, void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    if (K < 1 || K > EDT_MAX_WORKERS)
        return fail(EDT_ERR_ARG, "worker count %d out of range [1, %d]", K, EDT_MAX_WORKERS);
    if (T < 0) return fail(EDT_ERR_ARG, "tensor count %d < 0", T);
    if (T == 0) return EDT_OK;
    if (!theta_t || !theta_k || !numel) return fail(EDT_ERR_ARG, "null tensor table");
    const SgdScalars sg = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (sg.use_momentum && !momentum_t) return fail(EDT_ERR_ARG, "momentum table is null");
    const uint64_t need = edt_outer_list_workspace_bytes(T, K);
    if (!workspace || workspace_bytes < need)
        return fail(EDT_ERR_ARG, "workspace of %llu bytes needed", (unsigned long long)need);
    if (reinterpret_cast<uintptr_t>(workspace) & 7u) return fail(EDT_ERR_ARG, "workspace must be 8-byte aligned");
    if (tail && (gdt != EDT_BF16 || !tail_off)) return fail(EDT_ERR_ARG, "tail bits need a bf16 master and byte offsets");
    // table: prefix[T+1] | numel[T] | theta[T] | mom[T] | w[K*T] | tail_off[T]   (all 8-byte words)
    thread_local std::vector<uint64_t> h;
    h.assign(need / sizeof(uint64_t), 0);
    uint64_t* prefix = h.data();
    uint64_t* nflag = prefix + T + 1;
    uint64_t* pth = nflag + T;
    uint64_t* pmo = pth + T;
    uint64_t* pw = pmo + T;
    uint64_t* ptail = pw + (uint64_t)K * T;
    if (tail)
        for (int t = 0; t < T; ++t) ptail[t] = tail_off[t];
    for (int t = 0; t < T; ++t) {
        const uint64_t n = numel[t];
        if (n >= kVecFlag) return fail(EDT_ERR_ARG, "tensor %d too large", t);
        bool vec = true;
        if (n) {
            if (!theta_t[t]) return fail(EDT_ERR_ARG, "theta_t[%d] is null", t);
            vec = aligned16(theta_t[t]);
            if (sg.use_momentum) {
                if (!momentum_t[t]) return fail(EDT_ERR_ARG, "momentum_t[%d] is null", t);
                vec = vec && aligned16(momentum_t[t]);
            }
            for (int k = 0; k < K; ++k) {
                const void* p = theta_k[(uint64_t)k * T + t];
                if (!p) return fail(EDT_ERR_ARG, "theta_k[%d][%d] is null", k, t);
                vec = vec && aligned16(p);
            }
        }
        prefix[t + 1] = prefix[t] + (n + kListChunk - 1) / kListChunk;
        nflag[t] = n | (vec ? kVecFlag : 0);
        pth[t] = reinterpret_cast<uintptr_t>(theta_t[t]);
        pmo[t] = sg.use_momentum ? reinterpret_cast<uintptr_t>(momentum_t[t]) : 0;
        for (int k = 0; k < K; ++k) pw[(uint64_t)k * T + t] = reinterpret_cast<uintptr_t>(theta_k[(uint64_t)k * T + t]);
    }
    const uint64_t chunks = prefix[T];
    if (chunks == 0) return EDT_OK;
    if (chunks > 0x7fffffffull) return fail(EDT_ERR_ARG, "too many elements for one launch");
    hipStream_t st = (hipStream_t)stream;
    // pageable source: the copy is staged before hipMemcpyAsync returns, stream-ordered on the device
    hipError_t e = hipMemcpyAsync(workspace, h.data(), need, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return fail(EDT_ERR_LAUNCH, "tensor table upload failed: %s", hipGetErrorString(e));
    const uint64_t* d = static_cast<const uint64_t*>(workspace);
    ListArgs L;
    L.prefix = d;
    L.numel = d + T + 1;
    L.theta = reinterpret_cast<void* const*>(d + 2 * (uint64_t)T + 1);
    L.mom = reinterpret_cast<void* const*>(d + 3 * (uint64_t)T + 1);
    L.w = reinterpret_cast<const void* const*>(d + 4 * (uint64_t)T + 1);
    L.T = (uint64_t)T;
    L.chunks = chunks;
    L.K = K;
    L.kdiv = (float)K;
    L.kinv = 1.0f / (float)K;
    L.sgd = sg;
    L.tail = tail;
    L.tail_off = d + 4 * (uint64_t)T + 1 + (uint64_t)K * T;
    const int div_exact = is_pow2(K) ? 0 : 1;
    const unsigned grid = chunks > kMaxBlocks ? (unsigned)kMaxBlocks : (unsigned)chunks;   // grid-stride
    if (gdt == EDT_F32 && wdt == EDT_F32) return launch_list_k<EDT_F32, EDT_F32>(L, div_exact, grid, st);
    if (gdt == EDT_F32) return launch_list_k<EDT_F32, EDT_BF16>(L, div_exact, grid, st);
    return launch_list_k<EDT_BF16, EDT_BF16>(L, div_exact, grid, st);
}

extern "C" {

int edt_outer_step_list(void* const* theta_t, int gdt, const void* const* theta_k, int wdt, int K,
                        void* const* momentum_t, int has_momentum, const uint64_t* numel, int T,
                        double lr, double momentum_coef, int nesterov, void* workspace,
                        uint64_t workspace_bytes, void* stream) {
    return outer_step_list_impl(theta_t, gdt, theta_k, wdt, K, momentum_t, has_momentum, numel, T, lr,
                                momentum_coef, nesterov, nullptr, nullptr, workspace, workspace_bytes, stream);
}

int edt_outer_step_list_tail(void* const* theta_t, int gdt, const void* const* theta_k, int wdt, int K,
                             void* const* momentum_t, int has_momentum, const uint64_t* numel, int T,
                             double lr, double momentum_coef, int nesterov, const uint8_t* tail_bits,
                             const uint64_t* tail_byte_offset, void* workspace, uint64_t workspace_bytes,
                             void* stream) {
    return outer_step_list_impl(theta_t, gdt, theta_k, wdt, K, momentum_t, has_momentum, numel, T, lr,
                                momentum_coef, nesterov, tail_bits, tail_byte_offset, workspace, workspace_bytes,
                                stream);
}

int edt_delta_partial(const void* theta_g, int gdt, const void* const* theta_k, int wdt, int K_local,
                      int K_total, uint64_t n, float* acc_f32, int accumulate, void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    OuterArgs a;
    int rc = fill_outer(a, theta_g, theta_k, K_local, K_total, n);
    if (rc) return rc;
    if (!acc_f32 && n) return fail(EDT_ERR_ARG, "acc_f32 is null");
    a.acc_out = acc_f32;
    a.accumulate = accumulate;
    if (n == 0) return EDT_OK;
    bool vec = aligned16(theta_g) && aligned16(acc_f32);
    for (int k = 0; k < K_local; ++k) vec = vec && aligned16(theta_k[k]);
    return launch_outer<MODE_PARTIAL>(gdt, wdt, a, vec, (hipStream_t)stream);
}

int edt_sgd_apply_sum(void* theta_g, int gdt, const float* const* acc_f32, int nacc, void* momentum,
                      int has_momentum, uint64_t n, double lr, double momentum_coef, int nesterov, void* stream) {
    g_err[0] = 0;
    if (gdt != EDT_F32 && gdt != EDT_BF16) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nacc < 1 || nacc > EDT_MAX_WORKERS) return fail(EDT_ERR_ARG, "partial count %d out of range [1, %d]", nacc,
                                                         EDT_MAX_WORKERS);
    if (n == 0) return EDT_OK;
    if (!theta_g || !acc_f32) return fail(EDT_ERR_ARG, "null buffer");
    SgdScalars s = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (s.use_momentum && !momentum) return fail(EDT_ERR_ARG, "momentum buffer is null");
    Partials P;
    memset(&P, 0, sizeof(P));
    bool vec = aligned16(theta_g) && (!s.use_momentum || aligned16(momentum));
    for (int r = 0; r < nacc; ++r) {
        if (!acc_f32[r]) return fail(EDT_ERR_ARG, "acc_f32[%d] is null", r);
        P.p[r] = acc_f32[r];
        vec = vec && aligned16(acc_f32[r]);
    }
    const unsigned g = grid_for(n, vec);
    hipStream_t st = (hipStream_t)stream;
    if (gdt == EDT_F32) {
        if (vec) sgd_apply_sum_kernel<EDT_F32, kVec><<<g, kBlock, 0, st>>>(theta_g, P, nacc, momentum, n, s);
        else sgd_apply_sum_kernel<EDT_F32, 1><<<g, kBlock, 0, st>>>(theta_g, P, nacc, momentum, n, s);
    } else {
        if (vec) sgd_apply_sum_kernel<EDT_BF16, kVec><<<g, kBlock, 0, st>>>(theta_g, P, nacc, momentum, n, s);
        else sgd_apply_sum_kernel<EDT_BF16, 1><<<g, kBlock, 0, st>>>(theta_g, P, nacc, momentum, n, s);
    }
    return check_launch("sgd_apply_sum_kernel");
}

int edt_sgd_apply(void* theta_g, int gdt, const float* acc_f32, void* momentum, int has_momentum,
                  uint64_t n, double lr, double momentum_coef, int nesterov, void* stream) {
    g_err[0] = 0;
    if (gdt != EDT_F32 && gdt != EDT_BF16) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (n == 0) return EDT_OK;
    if (!theta_g || !acc_f32) return fail(EDT_ERR_ARG, "null buffer");
    SgdScalars s = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (s.use_momentum && !momentum) return fail(EDT_ERR_ARG, "momentum buffer is null");
    const bool vec = aligned16(theta_g) && aligned16(acc_f32) && (!s.use_momentum || aligned16(momentum));
    const unsigned g = grid_for(n, vec);
    hipStream_t st = (hipStream_t)stream;
    if (gdt == EDT_F32) {
        if (vec) sgd_apply_kernel<EDT_F32, kVec><<<g, kBlock, 0, st>>>(theta_g, acc_f32, momentum, n, s);
        else sgd_apply_kernel<EDT_F32, 1><<<g, kBlock, 0, st>>>(theta_g, acc_f32, momentum, n, s);
    } else {
        if (vec) sgd_apply_kernel<EDT_BF16, kVec><<<g, kBlock, 0, st>>>(theta_g, acc_f32, momentum, n, s);
        else sgd_apply_kernel<EDT_BF16, 1><<<g, kBlock, 0, st>>>(theta_g, acc_f32, momentum, n, s);
    }
    return check_launch("sgd_apply_kernel");
}


}  // extern "C"
