// edt_sync.hip — CDNA4 (gfx950) kernels for the outer-loop sync hot path and their C ABI
// (declared in include/edt_sync.h).
//
// Everything here is element-wise and HBM-bound: no MFMA. Each thread moves 8 elements per
// iteration with 16-byte loads (one bf16 x8 or two fp32 x4 per operand), a grid-stride loop
// keeps ~2k workgroups resident, and every operand is read once and written once.
//
// Numerics mirror the reference's PyTorch-CPU / numpy kernels bit for bit:
//  * fp32 regime: each torch op is one IEEE fp32 op; `add(x, y, alpha=a)` is fmaf(a, y, x)
//    (torch's vectorised CPU add is an FMA, tails included); true division by K.
//  * bf16 regime: each torch op is computed in fp32 and rounded to bf16 (RNE); `mul_(s)` uses
//    the fp32 scalar, `add(..., alpha=a)` first rounds alpha to bf16.
// The file must be compiled with -ffp-contract=off so that no unintended FMA is formed.

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include "edt_sync.h"

namespace {

// Tunables (overridable at build time for the variant sweep in scripts/kernel_variants.py).
// Measured on MI355X, 1.3B params x 8 bf16 workers (profiles/r01_variants.txt): 256 blocks per
// CU (short grid-stride runs, no tail of late blocks) + non-temporal worker loads is fastest,
// 6.78 ms = 6.21 TB/s vs 7.36 ms for 8 blocks per CU with default-policy loads.
#ifndef EDT_BLOCKS_PER_CU
#define EDT_BLOCKS_PER_CU 256
#endif
#ifndef EDT_NT_LOADS          // non-temporal loads for the once-read bf16 worker streams
#define EDT_NT_LOADS 1        // (fp32 streams: measured 1.6x SLOWER with nt, 17.5 vs 11.2 ms)
#endif
#ifndef EDT_NT_STORES         // non-temporal stores for theta / momentum
#define EDT_NT_STORES 0
#endif

#ifndef EDT_NT_LERP             // non-temporal loads of lerp's two (read-once) inputs
#define EDT_NT_LERP 0
#endif
// SLERP of two Qwen2.5-7B bodies (bf16, profiles/r01_slerp_variants.json, two boxes): non-temporal
// parent loads + one workgroup per segment for the chunk-sum reduction + 64 Ki-element chunks
// 11.23 / 11.41 ms, against 12.14 / 12.27 ms for default loads, one wave per segment and 16 Ki
// chunks. The population form (edt_slerp_population) keeps default-policy loads (2 % faster).
#ifndef EDT_NT_SLERP            // non-temporal loads of the SLERP parents (stats and blend passes)
#define EDT_NT_SLERP 1
#endif
#ifndef EDT_SLERP_BPC           // workgroups per CU for the chunk-looping SLERP passes
#define EDT_SLERP_BPC 256
#endif
#ifndef EDT_SLERP_COEF_BLOCK    // 1: one workgroup per segment for the chunk-sum reduction (else one wave)
#define EDT_SLERP_COEF_BLOCK 1
#endif
// outer_kernel / probe_kernel element mapping (see ld()): 0 = 8 consecutive elements per thread,
// 1 = wave-contiguous "split halves", 2 = split halves when workers and theta are fp32. Same speed
// in every regime (profiles/r01_split_halves.json), but with 8 fp32 worker streams the 32-B-strided
// pairs of 16-B loads fetch ~20 % more than the algorithmic bytes (FETCH_SIZE; served mostly by
// the Infinity Cache) while split halves fetch exactly them (profiles/pmc_traffic.json).
#ifndef EDT_SPLIT_HALVES
#define EDT_SPLIT_HALVES 2
#endif
// Non-temporal loads for the once-read worker streams: bf16 always (EDT_NT_LOADS); fp32 with the
// split-halves mapping (EDT_NT_F32: 10.61 vs 11.03 ms on 1.3B x 8 fp32, profiles/r01_f32_variants.json;
// with the 8-consecutive mapping nt was 1.6x slower, so it never applies there).
#ifndef EDT_NT_F32
#define EDT_NT_F32 1
#endif
template <int WDT, int H2>
constexpr bool nt_worker_loads() {
    return EDT_NT_LOADS != 0 && (WDT == EDT_BF16 || (EDT_NT_F32 != 0 && H2 != 4));
}

template <int GDT, int WDT>
constexpr bool split_halves() {
    return EDT_SPLIT_HALVES == 1 || (EDT_SPLIT_HALVES == 2 && GDT == EDT_F32 && WDT == EDT_F32);
}
#ifndef EDT_MIN_WAVES           // __launch_bounds__ minimum waves per SIMD for the stream kernels
#define EDT_MIN_WAVES 1
#endif

constexpr int kBlock = 256;                         // 4 waves
constexpr int kVec = 8;                             // elements per thread per iteration
// grid cap for the grid-stride loops: 256 CUs x workgroups per CU (0 = one pass, no cap)
constexpr uint64_t kMaxBlocks = EDT_BLOCKS_PER_CU > 0 ? 256ull * EDT_BLOCKS_PER_CU : (1ull << 31) - 1;

constexpr uint64_t kSlerpMaxBlocks = 256ull * EDT_SLERP_BPC;
inline unsigned slerp_grid(int64_t nchunks) {
    return (unsigned)((uint64_t)nchunks < kSlerpMaxBlocks ? (uint64_t)nchunks : kSlerpMaxBlocks);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

thread_local char g_err[512];

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(EDT_ERR_LAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e));
    return EDT_OK;
}

// ---------------------------------------------------------------------------------------
// bf16 helpers: a bf16 is the top half of an fp32; conversion f32->bf16 is v_cvt_pk_bf16_f32
// (round-to-nearest-even, as c10::BFloat16).

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf(float lo, float hi) {
    bf16x2 r = __builtin_convertvector((f32x2){lo, hi}, bf16x2);
    return __builtin_bit_cast(uint32_t, r);
}
__host__ __device__ inline float host_round_bf16(float x) {   // used for scalars on the host
    uint32_t u;
    memcpy(&u, &x, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return x;
    u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
    float r;
    memcpy(&r, &u, 4);
    return r;
}

// Round each of the N values to the precision of dtype DT (no-op for fp32).
template <int DT, int N>
__device__ __forceinline__ void rnd(float (&x)[N]) {
    if constexpr (DT == EDT_BF16) {
        if constexpr (N % 2 == 0) {
#pragma unroll
            for (int j = 0; j < N; j += 2) {
                uint32_t p = pack_bf(x[j], x[j + 1]);
                x[j] = bf_lo(p);
                x[j + 1] = bf_hi(p);
            }
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) x[j] = bf_lo(pack_bf(x[j], 0.f));
        }
    }
}

// Load / store N (= 8 or 1) consecutive elements of a buffer of dtype DT as fp32.
// Index `i` is the element index of the first element (a multiple of 8 when N == 8).
template <typename V, bool NT>
__device__ __forceinline__ V vload(const V* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <typename V, bool NT>
__device__ __forceinline__ void vstore(V* p, V v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// An 8-element group is elements [i, i+4) and [i+H2, i+H2+4): H2 = 4 is 8 consecutive elements
// (one 16-B access per bf16 operand, two per fp32 operand, 32 B apart across lanes); H2 = 4 x
// workgroup size ("split halves") makes every access of a wave contiguous across its lanes (fp32:
// 16 B per lane; bf16: 8 B per lane, twice).
template <int DT, int N, bool NT = false, int H2 = 4>
__device__ __forceinline__ void ld(const void* __restrict__ p, uint64_t i, float (&x)[N]) {
    if constexpr (DT == EDT_F32) {
        const float* q = static_cast<const float*>(p) + i;
        if constexpr (N == 8) {
            f32x4 a = vload<f32x4, NT>(reinterpret_cast<const f32x4*>(q));
            f32x4 b = vload<f32x4, NT>(reinterpret_cast<const f32x4*>(q + H2));
            x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
            x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) x[j] = q[j];
        }
    } else {
        const uint16_t* q = static_cast<const uint16_t*>(p) + i;
        if constexpr (N == 8 && H2 == 4) {
            u32x4 w = vload<u32x4, NT>(reinterpret_cast<const u32x4*>(q));
            x[0] = bf_lo(w.x); x[1] = bf_hi(w.x); x[2] = bf_lo(w.y); x[3] = bf_hi(w.y);
            x[4] = bf_lo(w.z); x[5] = bf_hi(w.z); x[6] = bf_lo(w.w); x[7] = bf_hi(w.w);
        } else if constexpr (N == 8) {
            u32x2 w0 = vload<u32x2, NT>(reinterpret_cast<const u32x2*>(q));
            u32x2 w1 = vload<u32x2, NT>(reinterpret_cast<const u32x2*>(q + H2));
            x[0] = bf_lo(w0.x); x[1] = bf_hi(w0.x); x[2] = bf_lo(w0.y); x[3] = bf_hi(w0.y);
            x[4] = bf_lo(w1.x); x[5] = bf_hi(w1.x); x[6] = bf_lo(w1.y); x[7] = bf_hi(w1.y);
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) x[j] = __uint_as_float(uint32_t(q[j]) << 16);
        }
    }
}

// Stores round-to-nearest-even into DT (values are already DT-exact in the bf16 regime).
template <int DT, int N, bool NT = (EDT_NT_STORES != 0), int H2 = 4>
__device__ __forceinline__ void st(void* __restrict__ p, uint64_t i, const float (&x)[N]) {
    if constexpr (DT == EDT_F32) {
        float* q = static_cast<float*>(p) + i;
        if constexpr (N == 8) {
            vstore<f32x4, NT>(reinterpret_cast<f32x4*>(q), (f32x4){x[0], x[1], x[2], x[3]});
            vstore<f32x4, NT>(reinterpret_cast<f32x4*>(q + H2), (f32x4){x[4], x[5], x[6], x[7]});
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) q[j] = x[j];
        }
    } else {
        uint16_t* q = static_cast<uint16_t*>(p) + i;
        if constexpr (N == 8 && H2 == 4) {
            u32x4 w;
            w.x = pack_bf(x[0], x[1]); w.y = pack_bf(x[2], x[3]);
            w.z = pack_bf(x[4], x[5]); w.w = pack_bf(x[6], x[7]);
            vstore<u32x4, NT>(reinterpret_cast<u32x4*>(q), w);
        } else if constexpr (N == 8) {
            u32x2 w0, w1;
            w0.x = pack_bf(x[0], x[1]); w0.y = pack_bf(x[2], x[3]);
            w1.x = pack_bf(x[4], x[5]); w1.y = pack_bf(x[6], x[7]);
            vstore<u32x2, NT>(reinterpret_cast<u32x2*>(q), w0);
            vstore<u32x2, NT>(reinterpret_cast<u32x2*>(q + H2), w1);
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) q[j] = uint16_t(pack_bf(x[j], 0.f) & 0xffffu);
        }
    }
}

// ---------------------------------------------------------------------------------------
// SGD scalars, rounded on the host exactly as torch rounds them.

struct SgdScalars {
    float mul_mu;      // buf.mul_(momentum): fp32 scalar
    float alpha_mu;    // grad.add(buf, alpha=momentum): alpha in the tensor dtype
    float alpha_nlr;   // param.add_(grad, alpha=-lr): alpha in the tensor dtype
    int use_momentum;  // momentum != 0
    int has_buf;       // momentum buffer carried from a previous step
    int nesterov;
};

SgdScalars make_sgd(int gdt, double lr, double mu, int has_buf, int nesterov) {
    SgdScalars s;
    s.mul_mu = (float)mu;
    s.alpha_mu = gdt == EDT_BF16 ? host_round_bf16((float)mu) : (float)mu;
    s.alpha_nlr = gdt == EDT_BF16 ? host_round_bf16((float)(-lr)) : (float)(-lr);
    s.use_momentum = mu != 0.0;
    s.has_buf = has_buf;
    s.nesterov = nesterov;
    return s;
}

// torch.optim.sgd._single_tensor_sgd for one group of N elements, in regime GDT.
// grad is the pseudo-gradient (already in GDT precision); theta is updated in registers,
// the momentum buffer is read from / written to `mom` at element i.
// Loads the carried momentum buffer (issued together with the other operand loads).
template <int GDT, int N, int H2 = 4>
__device__ __forceinline__ void ld_momentum(const void* mom, uint64_t i, const SgdScalars& s, float (&b)[N]) {
    if (s.use_momentum && s.has_buf) ld<GDT, N, false, H2>(mom, i, b);
}

template <int GDT, int N, int H2 = 4>
__device__ __forceinline__ void sgd_update(float (&theta)[N], const float (&grad)[N], void* mom,
                                           uint64_t i, const SgdScalars& s, const float (&b_in)[N]) {
    float u[N];
    if (s.use_momentum) {
        float b[N];
        if (s.has_buf) {
#pragma unroll
            for (int j = 0; j < N; ++j) b[j] = b_in[j] * s.mul_mu;   // buf.mul_(momentum)
            rnd<GDT>(b);
#pragma unroll
            for (int j = 0; j < N; ++j) b[j] = b[j] + grad[j];       // .add_(grad, alpha=1)
            rnd<GDT>(b);
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) b[j] = grad[j];              // buf = grad.clone()
        }
        st<GDT, N, (EDT_NT_STORES != 0), H2>(mom, i, b);
        if (s.nesterov) {
#pragma unroll
            for (int j = 0; j < N; ++j) u[j] = __builtin_fmaf(s.alpha_mu, b[j], grad[j]);
            rnd<GDT>(u);
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) u[j] = b[j];
        }
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) u[j] = grad[j];
    }
#pragma unroll
    for (int j = 0; j < N; ++j) theta[j] = __builtin_fmaf(s.alpha_nlr, u[j], theta[j]);
    rnd<GDT>(theta);
}

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

// MODE_CHAIN = MODE_FUSED for populations above EDT_MAX_WORKERS: launches of <= 32 workers
// carry the running sum in theta's dtype (lossless: it is rounded to that dtype after every add).
enum { MODE_FUSED = 0, MODE_PARTIAL = 1, MODE_CHAIN = 2 };

// Per-element accumulation acc = sum_k round(round(w_k - g) / K) in the precision of GDT
// (worker-major order, EDT_LM/diloco.py:243-246). MODE_PARTIAL sums the rounded quotients
// in fp32 instead (the cross-rank sum is then an fp32 RCCL reduction).
template <int GDT, int WDT, int KC, int DIV, int MODE, int N, class A, int H2 = 4>
__device__ __forceinline__ void outer_elems(const A& a, uint64_t i) {
    float g[N], acc[N], b_in[N];
    ld<GDT, N, false, H2>(a.theta, i, g);
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
    }
}

// DIV = 1: true division by K (torch CPU `delta / num_models`); DIV = 0: multiply by 1/K,
// bit-identical when K is a power of two.
template <int GDT, int WDT, int KC, int DIV, int MODE, int N>
__global__ __launch_bounds__(kBlock, EDT_MIN_WAVES) void outer_kernel(OuterArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if constexpr (N == kVec && split_halves<GDT, WDT>()) {
        // tiles of kBlock x 8 elements; thread t owns [4t, 4t+4) and [4(kBlock+t), +4) of a tile
        constexpr int H2 = 4 * kBlock;
        const uint64_t nv = a.n / (kVec * kBlock) * kBlock;
        for (uint64_t v = tid; v < nv; v += stride)
            outer_elems<GDT, WDT, KC, DIV, MODE, kVec, OuterArgs, H2>(a, v * kVec - 4 * threadIdx.x);
        for (uint64_t e = nv * kVec + tid; e < a.n; e += stride)     // scalar tail (< 8 x kBlock)
            outer_elems<GDT, WDT, KC, DIV, MODE, 1>(a, e);
    } else if constexpr (N == kVec) {
        const uint64_t nv = a.n / kVec;
        for (uint64_t v = tid; v < nv; v += stride) outer_elems<GDT, WDT, KC, DIV, MODE, kVec>(a, v * kVec);
        const uint64_t t = nv * kVec + tid;      // scalar tail (< 8 elements)
        if (t < a.n) outer_elems<GDT, WDT, KC, DIV, MODE, 1>(a, t);
    } else {
        for (uint64_t e = tid; e < a.n; e += stride) outer_elems<GDT, WDT, KC, DIV, MODE, 1>(a, e);
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

// ---------------------------------------------------------------------------------------
// EDT pair merge: child = SGD step of lerp(0.5, b1, b2) towards the parents' trained weights.

struct PairArgs {
    const void* b1;
    const void* b2;
    const void* m1;
    const void* m2;
    void* out;
    const void* mom_in;   // carried buffer read (the donor parent's); may equal mom
    void* mom;            // the child's buffer written
    uint64_t n;
    SgdScalars sgd;
};

template <int GDT, int WDT, int N, bool NT = (EDT_NT_LOADS != 0 && WDT == EDT_BF16)>
__device__ __forceinline__ void pair_elems(const PairArgs& a, uint64_t i) {
    float base[N], b_in[N];
    ld_momentum<GDT, N>(a.mom_in, i, a.sgd, b_in);
    if (a.b2) {                        // run_linear_merge_5050: lerp(0.5, b1, b2) in the model dtype
        float x[N], y[N];
        ld<WDT, N, NT>(a.b1, i, x);
        ld<WDT, N, NT>(a.b2, i, y);
#pragma unroll
        for (int j = 0; j < N; ++j) { x[j] = x[j] * 0.5f; y[j] = y[j] * 0.5f; }   // (1-.5)*v0, .5*v1
        rnd<WDT>(x);
        rnd<WDT>(y);
#pragma unroll
        for (int j = 0; j < N; ++j) base[j] = x[j] + y[j];
        rnd<WDT>(base);
    } else {                           // run_sgd on an already merged base model (dtype GDT)
        ld<GDT, N>(a.b1, i, base);
    }
    rnd<GDT>(base);                    // load_state_dict into the base model's dtype
    float d1[N], d2[N];
    ld<WDT, N, NT>(a.m1, i, d1);
    ld<WDT, N, NT>(a.m2, i, d2);
#pragma unroll
    for (int j = 0; j < N; ++j) { d1[j] = d1[j] - base[j]; d2[j] = d2[j] - base[j]; }
    rnd<GDT>(d1);
    rnd<GDT>(d2);
#pragma unroll
    for (int j = 0; j < N; ++j) d1[j] = d1[j] + d2[j];
    rnd<GDT>(d1);
#pragma unroll
    for (int j = 0; j < N; ++j) d1[j] = d1[j] * 0.5f;              // / num_models (= 2)
    rnd<GDT>(d1);
    float grad[N];
#pragma unroll
    for (int j = 0; j < N; ++j) grad[j] = -(0.f + d1[j]);           // acc = zeros + delta
    sgd_update<GDT, N>(base, grad, a.mom, i, a.sgd, b_in);
    st<GDT, N>(a.out, i, base);
}

template <int GDT, int WDT, int N>
__global__ __launch_bounds__(kBlock) void pair_kernel(PairArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if constexpr (N == kVec) {
        const uint64_t nv = a.n / kVec;
        for (uint64_t v = tid; v < nv; v += stride) pair_elems<GDT, WDT, kVec>(a, v * kVec);
        const uint64_t t = nv * kVec + tid;
        if (t < a.n) pair_elems<GDT, WDT, 1>(a, t);
    } else {
        for (uint64_t e = tid; e < a.n; e += stride) pair_elems<GDT, WDT, 1>(a, e);
    }
}

// EDT-LM children of a resident population in ONE launch (EDT_LM/edt_sim.py:244-256 builds one
// child per machine from the selected pairs). A parent feeds ~2 children; the workgroups of every
// child for the same chunk of elements carry the same blockIdx % 8 (they share an XCD, hence an
// L2) and are dispatched together, and the parents are read with default-policy loads, so a
// parent chunk crosses HBM once and its other readers hit the L2 / Infinity Cache. Per child the
// element math is pair_elems' (bit-identical to edt_pair_merge_to).
constexpr int kPopMaxChildren = 16;
constexpr uint64_t kPopChunk = (uint64_t)kBlock * kVec * 4;     // 8192 elements per workgroup

struct PopPairArgs {
    PairArgs c[kPopMaxChildren];
    int nchildren;
    uint64_t nchunks;
};

template <int GDT, int WDT, bool VEC>
__global__ __launch_bounds__(kBlock) void pair_population_kernel(PopPairArgs P) {
    const uint64_t bid = blockIdx.x;
    const uint64_t per_group = 8ull * (uint64_t)P.nchildren;
    const uint64_t r = bid % per_group;
    const int child = (int)(r / 8);
    const uint64_t chunk = (bid / per_group) * 8 + (r % 8);
    if (chunk >= P.nchunks) return;
    const PairArgs& a = P.c[child];
    const uint64_t c0 = chunk * kPopChunk;
    const uint64_t c1 = c0 + kPopChunk < a.n ? c0 + kPopChunk : a.n;
    if constexpr (VEC) {
        const uint64_t vend = c0 + (c1 - c0) / kVec * kVec;
        for (uint64_t i = c0 + (uint64_t)threadIdx.x * kVec; i < vend; i += (uint64_t)kBlock * kVec)
            pair_elems<GDT, WDT, kVec, false>(a, i);
        const uint64_t i = vend + threadIdx.x;
        if (i < c1) pair_elems<GDT, WDT, 1, false>(a, i);
    } else {
        for (uint64_t i = c0 + threadIdx.x; i < c1; i += kBlock) pair_elems<GDT, WDT, 1, false>(a, i);
    }
}

// ---------------------------------------------------------------------------------------
// lerp with a scalar t: out = round(round(c0*v0) + round(c1*v1)) in compute dtype CDT.

template <int IDT, int ODT, int CDT, int N, bool NTL = false, bool NTS = (EDT_NT_STORES != 0)>
__device__ __forceinline__ void lerp_elems(const void* v0, const void* v1, void* out, uint64_t i,
                                           float c0, float c1) {
    float x[N], y[N];
    ld<IDT, N, NTL>(v0, i, x);
    ld<IDT, N, NTL>(v1, i, y);
#pragma unroll
    for (int j = 0; j < N; ++j) { x[j] = c0 * x[j]; y[j] = c1 * y[j]; }
    rnd<CDT>(x);
    rnd<CDT>(y);
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] = x[j] + y[j];
    rnd<CDT>(x);
    st<ODT, N, NTS>(out, i, x);
}

template <int IDT, int ODT, int CDT, int N>
__global__ __launch_bounds__(kBlock) void lerp_kernel(const void* v0, const void* v1, void* out,
                                                      uint64_t n, float c0, float c1) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if constexpr (N == kVec) {
        const uint64_t nv = n / kVec;
        for (uint64_t v = tid; v < nv; v += stride)
            lerp_elems<IDT, ODT, CDT, kVec, EDT_NT_LERP != 0>(v0, v1, out, v * kVec, c0, c1);
        const uint64_t t = nv * kVec + tid;
        if (t < n) lerp_elems<IDT, ODT, CDT, 1>(v0, v1, out, t, c0, c1);
    } else {
        for (uint64_t e = tid; e < n; e += stride) lerp_elems<IDT, ODT, CDT, 1>(v0, v1, out, e, c0, c1);
    }
}

// ---------------------------------------------------------------------------------------
// SLERP. chunk_desc[3c .. 3c+2] = {start, length, segment}; chunks never cross a segment.

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// Block-wide sums {v0.v0, v1.v1, v0.v1} over one chunk [start, start+len), fp64 per thread,
// fixed reduction order (wave shuffles, then waves in order). Valid in thread 0. EMIT = true also
// writes the lerp-branch output l0 v0 + l1 v1 of the chunk (two rounded fp32 products, one
// rounded sum: lerp_elems' math) in the same pass — the speculative forms; every caller forms
// the sums with this one loop, so their sums are bit-identical.
template <int IDT, bool NT, bool EMIT = false, int ODT = EDT_F32>
__device__ __forceinline__ void chunk_pass(const void* v0, const void* v1, void* out, uint64_t start, uint64_t len,
                                           float l0, float l1, double (*red)[kBlock / 64], double (&sums)[3]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t end = start + len;
    double s00 = 0.0, s11 = 0.0, s01 = 0.0;
    const uint64_t a = (start + kVec - 1) / kVec * kVec;      // aligned body [a, b)
    const uint64_t b = end / kVec * kVec;
    auto elems = [&](auto tagN, uint64_t i) {
        constexpr int N = decltype(tagN)::value;
        float x[N], y[N];
        ld<IDT, N, NT && N == kVec>(v0, i, x);
        ld<IDT, N, NT && N == kVec>(v1, i, y);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const double dx = x[j], dy = y[j];
            s00 = __builtin_fma(dx, dx, s00);
            s11 = __builtin_fma(dy, dy, s11);
            s01 = __builtin_fma(dx, dy, s01);
        }
        if constexpr (EMIT) {
            float o[N];
#pragma unroll
            for (int j = 0; j < N; ++j) o[j] = l0 * x[j] + l1 * y[j];
            st<ODT, N>(out, i, o);
        }
    };
    if (a < b) {
        for (uint64_t i = a + (uint64_t)threadIdx.x * kVec; i < b; i += (uint64_t)kBlock * kVec)
            elems(std::integral_constant<int, kVec>{}, i);
    }
    // head [start, min(a, end)) and tail [max(b, a), end): fewer than 16 elements
    const uint64_t h_end = a < end ? a : end;
    const uint64_t t_beg = b > a ? b : h_end;
    const uint64_t nh = h_end - start, nt = end - t_beg;
    if ((uint64_t)threadIdx.x < nh + nt)
        elems(std::integral_constant<int, 1>{}, threadIdx.x < nh ? start + threadIdx.x : t_beg + (threadIdx.x - nh));
    s00 = wave_sum(s00);
    s11 = wave_sum(s11);
    s01 = wave_sum(s01);
    if (lane == 0) { red[0][wave] = s00; red[1][wave] = s11; red[2][wave] = s01; }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            double acc = 0.0;
#pragma unroll
            for (int w = 0; w < kBlock / 64; ++w) acc += red[q][w];
            sums[q] = acc;
        }
    }
    __syncthreads();
}

template <int IDT>
__device__ __forceinline__ void chunk_sums(const void* v0, const void* v1, uint64_t start, uint64_t len,
                                           double (*red)[kBlock / 64], double (&out)[3]) {
    chunk_pass<IDT, EDT_NT_SLERP != 0 && IDT == EDT_BF16>(v0, v1, nullptr, start, len, 0.f, 0.f, red, out);
}

// The reference's scalar SLERP math (EDT_RL/crossover.py:24-45) from the three sums, in fp32 as
// numpy does it for float32 scalars (NEP 50: python floats enter as fp32).
__device__ __forceinline__ void slerp_coefficients(double s00, double s11, double s01, double t, float thr,
                                                   float eps, float& c0, float& c1, float& dot) {
    const float n0 = (float)sqrt(s00), n1 = (float)sqrt(s11);      // np.linalg.norm (fp32)
    const double d0 = n0 > eps ? (double)n0 : 1.0;                  // normalize() divides only if > eps
    const double d1 = n1 > eps ? (double)n1 : 1.0;
    dot = (float)(s01 / (d0 * d1));
    if (fabsf(dot) > thr) {                                         // lerp on the originals
        c0 = (float)(1.0 - t);
        c1 = (float)t;
    } else {
        const float th0 = acosf(dot);
        const float s0 = sinf(th0);
        const float tht = th0 * (float)t;
        c0 = sinf(th0 - tht) / s0;
        c1 = sinf(tht) / s0;
    }
}

// seg_ptrs (tensor-list form, may be null): per segment {v0, v1, out} device pointers; chunk
// starts are then relative to their segment. Null: v0 / v1 / out are flat arenas.
template <int IDT>
__global__ __launch_bounds__(kBlock) void slerp_stats_kernel(const void* v0, const void* v1,
                                                             const uint64_t* chunks, int64_t nchunks,
                                                             double* partial, const uint64_t* seg_ptrs) {
    __shared__ double red[3][kBlock / 64];
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        double sums[3];
        const void* a = v0;
        const void* b = v1;
        if (seg_ptrs) {
            const uint64_t seg = chunks[3 * c + 2];
            a = reinterpret_cast<const void*>(seg_ptrs[3 * seg]);
            b = reinterpret_cast<const void*>(seg_ptrs[3 * seg + 1]);
        }
        chunk_sums<IDT>(a, b, chunks[3 * c], chunks[3 * c + 1], red, sums);
        if (threadIdx.x == 0) {
            partial[3 * c] = sums[0];
            partial[3 * c + 1] = sums[1];
            partial[3 * c + 2] = sums[2];
        }
    }
}

// Speculative first pass (edt_slerp_merge_speculative): the chunk sums exactly as
// slerp_stats_kernel forms them (same element order per thread, same FMAs, same reductions), and
// in the same pass the lerp-branch output (1-t) v0 + t v1 (lerp_elems with the coefficients
// slerp_coefficients gives that branch). Parents of one lineage (fine-tunes of a common base)
// mostly have |dot| > 0.9995, where this output is final; the other segments are blended again.
template <int IDT, int ODT>
__global__ __launch_bounds__(kBlock) void slerp_stats_lerp_kernel(const void* v0, const void* v1, void* out,
                                                                  const uint64_t* chunks, int64_t nchunks,
                                                                  double* partial, const double* tvals) {
    __shared__ double red[3][kBlock / 64];
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const uint64_t seg = chunks[3 * c + 2];
        double sums[3];
        chunk_pass<IDT, EDT_NT_SLERP != 0 && IDT == EDT_BF16, true, ODT>(
            v0, v1, out, chunks[3 * c], chunks[3 * c + 1], (float)(1.0 - tvals[seg]), (float)tvals[seg], red, sums);
        if (threadIdx.x == 0) {
            partial[3 * c] = sums[0];
            partial[3 * c + 1] = sums[1];
            partial[3 * c + 2] = sums[2];
        }
    }
}

// Fixed-order reduction of a segment's chunk sums: column q of rows [c0, c1) of a row-major table
// with `stride` doubles per row, for the three columns (q0, q1, q2). EDT_SLERP_COEF_BLOCK = 0: one
// wave per segment (lane-strided, then a wave sum); 1: one workgroup per segment (thread-strided,
// wave sums, then the waves in order). Every coefficient kernel uses this one order.
constexpr int kCoefThreads = EDT_SLERP_COEF_BLOCK ? kBlock : 64;

__device__ __forceinline__ bool segment_sums(const double* tab, int stride, int q0, int q1, int q2, int c0,
                                             int c1, double (&out)[3]) {
    const int tid = EDT_SLERP_COEF_BLOCK ? (int)threadIdx.x : (int)(threadIdx.x & 63);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int c = c0 + tid; c < c1; c += kCoefThreads) {
        s0 += tab[(uint64_t)c * stride + q0];
        s1 += tab[(uint64_t)c * stride + q1];
        s2 += tab[(uint64_t)c * stride + q2];
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if constexpr (EDT_SLERP_COEF_BLOCK) {
        __shared__ double red[3][kBlock / 64];
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if (lane == 0) { red[0][wave] = s0; red[1][wave] = s1; red[2][wave] = s2; }
        __syncthreads();
        if (threadIdx.x != 0) return false;
        s0 = s1 = s2 = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) { s0 += red[0][w]; s1 += red[1][w]; s2 += red[2][w]; }
    } else {
        if ((threadIdx.x & 63) != 0) return false;
    }
    out[0] = s0;
    out[1] = s1;
    out[2] = s2;
    return true;
}

__device__ __forceinline__ int coef_segment() {
    return EDT_SLERP_COEF_BLOCK ? (int)blockIdx.x : (int)(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6));
}

inline unsigned coef_grid(int nseg) {
    return EDT_SLERP_COEF_BLOCK ? (unsigned)nseg : (unsigned)((nseg + kBlock / 64 - 1) / (kBlock / 64));
}

// Per segment: the reduction above, then the coefficients.
__global__ __launch_bounds__(kBlock) void slerp_coef_kernel(const double* partial, const int32_t* first,
                                                            int nseg, const double* tvals,
                                                            float thr, float eps, float* coef,
                                                            float* dot_out, int32_t* redo = nullptr) {
    const int seg = coef_segment();
    if (seg >= nseg) return;
    double sums[3];
    if (!segment_sums(partial, 3, 0, 1, 2, first[seg], first[seg + 1], sums)) return;
    float c0, c1, dot;
    slerp_coefficients(sums[0], sums[1], sums[2], tvals[seg], thr, eps, c0, c1, dot);
    coef[2 * seg] = c0;
    coef[2 * seg + 1] = c1;
    if (dot_out) dot_out[seg] = dot;
    if (redo) redo[seg] = fabsf(dot) > thr ? 0 : 1;   // the speculative lerp output stands or not
}

template <int IDT, int ODT, bool NT = (EDT_NT_SLERP != 0 && IDT == EDT_BF16)>
__global__ __launch_bounds__(kBlock) void slerp_blend_kernel(const void* v0, const void* v1, void* out,
                                                             const uint64_t* chunks, int64_t nchunks,
                                                             const float* coef, const uint64_t* seg_ptrs,
                                                             const int32_t* redo = nullptr) {
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const uint64_t start = chunks[3 * c], len = chunks[3 * c + 1], seg = chunks[3 * c + 2];
        if (redo && !redo[seg]) continue;         // speculative lerp output already final
        if (seg_ptrs) {
            v0 = reinterpret_cast<const void*>(seg_ptrs[3 * seg]);
            v1 = reinterpret_cast<const void*>(seg_ptrs[3 * seg + 1]);
            out = reinterpret_cast<void*>(seg_ptrs[3 * seg + 2]);
        }
        const uint64_t end = start + len;
        const float c0 = coef[2 * seg], c1 = coef[2 * seg + 1];
        const uint64_t a = (start + kVec - 1) / kVec * kVec;
        const uint64_t b = end / kVec * kVec;
        if (a < b) {
            for (uint64_t i = a + (uint64_t)threadIdx.x * kVec; i < b; i += (uint64_t)kBlock * kVec)
                lerp_elems<IDT, ODT, EDT_F32, kVec, NT>(v0, v1, out, i, c0, c1);
        }
        const uint64_t h_end = a < end ? a : end;
        const uint64_t t_beg = b > a ? b : h_end;
        const uint64_t nh = h_end - start, nt = end - t_beg;
        if ((uint64_t)threadIdx.x < nh + nt) {
            const uint64_t i = threadIdx.x < nh ? start + threadIdx.x : t_beg + (threadIdx.x - nh);
            lerp_elems<IDT, ODT, EDT_F32, 1>(v0, v1, out, i, c0, c1);
        }
    }
}

// ---------------------------------------------------------------------------------------
// SLERP for a resident population (EDT_RL/edt.py:286-299 merges every selected pair of one
// generation): ONE pass over the M <= 8 members per chunk forms every member's squared norm and
// every pair's dot — the upper triangle of the Gram matrix, M(M+1)/2 fp64 sums per chunk — where
// per-child stats passes would read each child's two parents. A child's (|vi|^2, |vj|^2, vi.vj)
// are then read out of it. Every sum is bit-identical to chunk_sums() on (vi, vj): the same
// per-thread FMA sequence in element order (an FMA's product is exact, so vi*vj == vj*vi), the
// same wave and block reductions; the coefficients therefore equal edt_slerp_merge's.

constexpr int kGramMaxMembers = 8;
struct Members {
    const void* p[kGramMaxMembers];
};

__host__ __device__ constexpr int tri_index(int a, int b, int M) {   // a <= b < M
    return a * M - a * (a - 1) / 2 + (b - a);
}

template <int IDT, int M, int N>
__device__ __forceinline__ void gram_accumulate(const Members& mem, uint64_t i, double (&g)[M * (M + 1) / 2]) {
    float x[M][N];
#pragma unroll
    for (int m = 0; m < M; ++m) ld<IDT, N>(mem.p[m], i, x[m]);   // default policy: measured faster here
#pragma unroll
    for (int j = 0; j < N; ++j) {
#pragma unroll
        for (int a = 0; a < M; ++a) {
            const double da = x[a][j];
#pragma unroll
            for (int b = a; b < M; ++b) {
                const double db = x[b][j];
                g[tri_index(a, b, M)] = __builtin_fma(da, db, g[tri_index(a, b, M)]);
            }
        }
    }
}

template <int IDT, int M>
__global__ __launch_bounds__(kBlock) void slerp_gram_kernel(Members mem, const uint64_t* chunks, int64_t nchunks,
                                                            double* gram) {
    constexpr int NT = M * (M + 1) / 2;
    __shared__ double red[NT][kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const uint64_t start = chunks[3 * c], end = start + chunks[3 * c + 1];
        double g[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) g[q] = 0.0;
        const uint64_t a = (start + kVec - 1) / kVec * kVec;
        const uint64_t b = end / kVec * kVec;
        if (a < b) {
            for (uint64_t i = a + (uint64_t)threadIdx.x * kVec; i < b; i += (uint64_t)kBlock * kVec)
                gram_accumulate<IDT, M, kVec>(mem, i, g);
        }
        const uint64_t h_end = a < end ? a : end;
        const uint64_t t_beg = b > a ? b : h_end;
        const uint64_t nh = h_end - start, nt = end - t_beg;
        if ((uint64_t)threadIdx.x < nh + nt) {
            const uint64_t i = threadIdx.x < nh ? start + threadIdx.x : t_beg + (threadIdx.x - nh);
            gram_accumulate<IDT, M, 1>(mem, i, g);
        }
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            const double v = wave_sum(g[q]);
            if (lane == 0) red[q][wave] = v;
        }
        __syncthreads();
        if (threadIdx.x < NT) {
            double acc = 0.0;
#pragma unroll
            for (int w = 0; w < kBlock / 64; ++w) acc += red[threadIdx.x][w];
            gram[(uint64_t)c * NT + threadIdx.x] = acc;
        }
        __syncthreads();
    }
}

// The blends of every child in one launch, with pair_population_kernel's placement: the
// workgroups of all children for one chunk carry the same blockIdx % 8 (one XCD, one L2) and run
// together, so a member that is a parent of several children is read from HBM once per chunk.
// Same per-element math as slerp_blend_kernel (lerp_elems with the child's coefficients).
constexpr int kBlendMaxChildren = 16;
struct BlendChildren {
    const void* v0[kBlendMaxChildren];
    const void* v1[kBlendMaxChildren];
    void* out[kBlendMaxChildren];
    const float* coef[kBlendMaxChildren];     // [nseg][2] of the child
    const int32_t* redo[kBlendMaxChildren];   // [nseg] of the child, or null: blend every segment
    double* partial[kBlendMaxChildren];       // [nchunks][3] of the child (speculative stats pass)
    int nchildren;
};

template <int IDT, int ODT>
__global__ __launch_bounds__(kBlock) void slerp_blend_population_kernel(BlendChildren B, const uint64_t* chunks,
                                                                        int64_t nchunks) {
    const uint64_t per_group = 8ull * (uint64_t)B.nchildren;
    const uint64_t r = blockIdx.x % per_group;
    const int child = (int)(r / 8);
    const int64_t c = (int64_t)((blockIdx.x / per_group) * 8 + (r % 8));
    if (c >= nchunks) return;
    const uint64_t start = chunks[3 * c], len = chunks[3 * c + 1], seg = chunks[3 * c + 2];
    if (B.redo[child] && !B.redo[child][seg]) return;      // speculative lerp output stands
    const void* v0 = B.v0[child];
    const void* v1 = B.v1[child];
    void* out = B.out[child];
    const float c0 = B.coef[child][2 * seg], c1 = B.coef[child][2 * seg + 1];
    const uint64_t end = start + len;
    const uint64_t a = (start + kVec - 1) / kVec * kVec;
    const uint64_t b = end / kVec * kVec;
    if (a < b) {
        for (uint64_t i = a + (uint64_t)threadIdx.x * kVec; i < b; i += (uint64_t)kBlock * kVec)
            lerp_elems<IDT, ODT, EDT_F32, kVec, false>(v0, v1, out, i, c0, c1);
    }
    const uint64_t h_end = a < end ? a : end;
    const uint64_t t_beg = b > a ? b : h_end;
    const uint64_t nh = h_end - start, nt = end - t_beg;
    if ((uint64_t)threadIdx.x < nh + nt) {
        const uint64_t i = threadIdx.x < nh ? start + threadIdx.x : t_beg + (threadIdx.x - nh);
        lerp_elems<IDT, ODT, EDT_F32, 1>(v0, v1, out, i, c0, c1);
    }
}

// Speculative population pass: block (chunk, child) with the co-located placement above; each
// forms its child's chunk sums exactly as chunk_sums() does and writes the lerp-branch output in
// the same pass (as slerp_stats_lerp_kernel). Shared parents cross HBM once for all children.
template <int IDT, int ODT>
__global__ __launch_bounds__(kBlock) void slerp_pop_stats_lerp_kernel(BlendChildren B, const uint64_t* chunks,
                                                                      int64_t nchunks, const double* tvals) {
    __shared__ double red[3][kBlock / 64];
    const uint64_t per_group = 8ull * (uint64_t)B.nchildren;
    const uint64_t r = blockIdx.x % per_group;
    const int child = (int)(r / 8);
    const int64_t c = (int64_t)((blockIdx.x / per_group) * 8 + (r % 8));
    if (c >= nchunks) return;
    const uint64_t seg = chunks[3 * c + 2];
    double sums[3];
    // default-policy loads: a parent's chunk is re-read by its other children from L2
    chunk_pass<IDT, false, true, ODT>(B.v0[child], B.v1[child], B.out[child], chunks[3 * c], chunks[3 * c + 1],
                                      (float)(1.0 - tvals[seg]), (float)tvals[seg], red, sums);
    if (threadIdx.x == 0) {
        double* pc = B.partial[child] + 3 * c;
        pc[0] = sums[0];
        pc[1] = sums[1];
        pc[2] = sums[2];
    }
}

// Per segment for the pair (i, j): slerp_coef_kernel's reduction over the chunks, reading the
// three Gram columns of the pair.
__global__ __launch_bounds__(kBlock) void slerp_gram_coef_kernel(const double* gram, int NT, int qi, int qj, int qd,
                                                                 const int32_t* first, int nseg,
                                                                 const double* tvals, float thr, float eps,
                                                                 float* coef, float* dot_out) {
    const int seg = coef_segment();
    if (seg >= nseg) return;
    double sums[3];
    if (!segment_sums(gram, NT, qi, qj, qd, first[seg], first[seg + 1], sums)) return;
    float c0, c1, dot;
    slerp_coefficients(sums[0], sums[1], sums[2], tvals[seg], thr, eps, c0, c1, dot);
    coef[2 * seg] = c0;
    coef[2 * seg + 1] = c1;
    if (dot_out) dot_out[seg] = dot;
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
// host-side dispatch helpers

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

unsigned grid_for(uint64_t n, bool vec) {
    const uint64_t per = vec ? (uint64_t)kBlock * kVec : (uint64_t)kBlock;
    uint64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    if (g > kMaxBlocks) g = kMaxBlocks;
    return (unsigned)g;
}

bool valid_pair(int gdt, int wdt) {
    return (gdt == EDT_F32 && (wdt == EDT_F32 || wdt == EDT_BF16)) || (gdt == EDT_BF16 && wdt == EDT_BF16);
}

template <int GDT, int WDT, int MODE>
int launch_outer_k(const OuterArgs& a, bool vec, hipStream_t s) {
    const unsigned g = grid_for(a.n, vec);
#define EDT_LAUNCH_K(KC, DIV)                                                                    \
    do {                                                                                         \
        if (vec) outer_kernel<GDT, WDT, KC, DIV, MODE, kVec><<<g, kBlock, 0, s>>>(a);            \
        else outer_kernel<GDT, WDT, KC, DIV, MODE, 1><<<g, kBlock, 0, s>>>(a);                   \
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

template <int MODE>
int launch_outer(int gdt, int wdt, const OuterArgs& a, bool vec, hipStream_t s) {
    if (gdt == EDT_F32 && wdt == EDT_F32) return launch_outer_k<EDT_F32, EDT_F32, MODE>(a, vec, s);
    if (gdt == EDT_F32 && wdt == EDT_BF16) return launch_outer_k<EDT_F32, EDT_BF16, MODE>(a, vec, s);
    return launch_outer_k<EDT_BF16, EDT_BF16, MODE>(a, vec, s);
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

bool is_pow2(int k) { return k > 0 && (k & (k - 1)) == 0; }

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

// =========================================================================================
// C ABI

extern "C" {

const char* edt_last_error(void) { return g_err; }
const char* edt_version(void) { return "edt_sync 0.1.0 gfx950"; }

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
    return (uint64_t)(4 * (uint64_t)T + 1 + (uint64_t)K * T) * sizeof(uint64_t);
}

int edt_outer_step_list(void* const* theta_t, int gdt, const void* const* theta_k, int wdt, int K,
                        void* const* momentum_t, int has_momentum, const uint64_t* numel, int T,
                        double lr, double momentum_coef, int nesterov, void* workspace,
                        uint64_t workspace_bytes, void* stream) {
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
    // table: prefix[T+1] | numel[T] | theta[T] | mom[T] | w[K*T]   (all 8-byte words)
    thread_local std::vector<uint64_t> h;
    h.assign(need / sizeof(uint64_t), 0);
    uint64_t* prefix = h.data();
    uint64_t* nflag = prefix + T + 1;
    uint64_t* pth = nflag + T;
    uint64_t* pmo = pth + T;
    uint64_t* pw = pmo + T;
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
    const int div_exact = is_pow2(K) ? 0 : 1;
    const unsigned grid = chunks > kMaxBlocks ? (unsigned)kMaxBlocks : (unsigned)chunks;   // grid-stride
    if (gdt == EDT_F32 && wdt == EDT_F32) return launch_list_k<EDT_F32, EDT_F32>(L, div_exact, grid, st);
    if (gdt == EDT_F32) return launch_list_k<EDT_F32, EDT_BF16>(L, div_exact, grid, st);
    return launch_list_k<EDT_BF16, EDT_BF16>(L, div_exact, grid, st);
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

int edt_pair_merge(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                   void* theta_out, int gdt, void* momentum, int has_momentum, uint64_t n, double lr,
                   double momentum_coef, int nesterov, void* stream) {
    return edt_pair_merge_to(b1, b2, m1, m2, wdt, theta_out, gdt, momentum, momentum, has_momentum, n, lr,
                             momentum_coef, nesterov, stream);
}

int edt_pair_merge_to(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                      void* theta_out, int gdt, const void* momentum_in, void* momentum, int has_momentum,
                      uint64_t n, double lr, double momentum_coef, int nesterov, void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    if (n == 0) return EDT_OK;
    if (!b1 || !m1 || !m2 || !theta_out) return fail(EDT_ERR_ARG, "null buffer");
    PairArgs a;
    a.b1 = b1; a.b2 = b2; a.m1 = m1; a.m2 = m2; a.out = theta_out; a.mom = momentum; a.n = n;
    a.mom_in = momentum_in;
    a.sgd = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (a.sgd.use_momentum && !momentum) return fail(EDT_ERR_ARG, "momentum buffer is null");
    if (a.sgd.use_momentum && has_momentum && !momentum_in) return fail(EDT_ERR_ARG, "carried momentum is null");
    const bool vec = aligned16(b1) && (!b2 || aligned16(b2)) && aligned16(m1) && aligned16(m2) &&
                     aligned16(theta_out) && (!a.sgd.use_momentum || aligned16(momentum)) &&
                     (!a.sgd.use_momentum || !has_momentum || aligned16(momentum_in));
    const unsigned g = grid_for(n, vec);
    hipStream_t s = (hipStream_t)stream;
    if (gdt == EDT_F32 && wdt == EDT_F32) {
        if (vec) pair_kernel<EDT_F32, EDT_F32, kVec><<<g, kBlock, 0, s>>>(a);
        else pair_kernel<EDT_F32, EDT_F32, 1><<<g, kBlock, 0, s>>>(a);
    } else if (gdt == EDT_F32) {
        if (vec) pair_kernel<EDT_F32, EDT_BF16, kVec><<<g, kBlock, 0, s>>>(a);
        else pair_kernel<EDT_F32, EDT_BF16, 1><<<g, kBlock, 0, s>>>(a);
    } else {
        if (vec) pair_kernel<EDT_BF16, EDT_BF16, kVec><<<g, kBlock, 0, s>>>(a);
        else pair_kernel<EDT_BF16, EDT_BF16, 1><<<g, kBlock, 0, s>>>(a);
    }
    return check_launch("pair_kernel");
}

int edt_pair_merge_population(const void* const* b1, const void* const* b2, const void* const* m1,
                              const void* const* m2, int wdt, void* const* out, int gdt,
                              const void* const* momentum_in, void* const* momentum_out,
                              const int32_t* has_momentum, int nchildren, uint64_t n, double lr,
                              double momentum_coef, int nesterov, void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    if (nchildren < 1 || nchildren > kPopMaxChildren)
        return fail(EDT_ERR_ARG, "child count %d out of range [1, %d]", nchildren, kPopMaxChildren);
    if (!b1 || !b2 || !m1 || !m2 || !out) return fail(EDT_ERR_ARG, "null pointer table");
    if (n == 0) return EDT_OK;
    PopPairArgs P;
    memset(&P, 0, sizeof(P));
    P.nchildren = nchildren;
    P.nchunks = (n + kPopChunk - 1) / kPopChunk;
    bool vec = true;
    for (int c = 0; c < nchildren; ++c) {
        PairArgs& a = P.c[c];
        const int has = has_momentum ? has_momentum[c] : 0;
        a.b1 = b1[c]; a.b2 = b2[c]; a.m1 = m1[c]; a.m2 = m2[c]; a.out = out[c]; a.n = n;
        a.mom = momentum_out ? momentum_out[c] : nullptr;
        a.mom_in = momentum_in ? momentum_in[c] : nullptr;
        a.sgd = make_sgd(gdt, lr, momentum_coef, has, nesterov);
        if (!a.b1 || !a.b2 || !a.m1 || !a.m2 || !a.out) return fail(EDT_ERR_ARG, "child %d: null buffer", c);
        if (a.sgd.use_momentum && !a.mom) return fail(EDT_ERR_ARG, "child %d: momentum buffer is null", c);
        if (a.sgd.use_momentum && has && !a.mom_in) return fail(EDT_ERR_ARG, "child %d: carried momentum is null", c);
        for (int d = 0; d < c; ++d)
            if (P.c[d].out == a.out || (a.mom && P.c[d].mom == a.mom))
                return fail(EDT_ERR_ARG, "children %d and %d write the same buffer", d, c);
        for (int d = 0; d < nchildren; ++d) {           // outputs never alias an input of any child
            const bool reads_mom = momentum_in && has_momentum && has_momentum[d];
            const void* ins[5] = {b1[d], b2[d], m1[d], m2[d], reads_mom ? momentum_in[d] : nullptr};
            for (const void* q : ins)
                if (q && (q == a.out || q == a.mom))
                    return fail(EDT_ERR_ARG, "child %d writes an input of child %d", c, d);
        }
        vec = vec && aligned16(a.b1) && aligned16(a.b2) && aligned16(a.m1) && aligned16(a.m2) && aligned16(a.out) &&
              (!a.sgd.use_momentum || (aligned16(a.mom) && (!has || aligned16(a.mom_in))));
    }
    const uint64_t groups = (P.nchunks + 7) / 8;
    const uint64_t blocks = groups * 8ull * (uint64_t)nchildren;
    if (blocks > 0x7fffffffull) return fail(EDT_ERR_ARG, "too many elements for one launch");
    const unsigned g = (unsigned)blocks;
    hipStream_t s = (hipStream_t)stream;
#define EDT_POP(G, W)                                                                   \
    do {                                                                                \
        if (vec) pair_population_kernel<G, W, true><<<g, kBlock, 0, s>>>(P);            \
        else pair_population_kernel<G, W, false><<<g, kBlock, 0, s>>>(P);               \
    } while (0)
    if (gdt == EDT_F32 && wdt == EDT_F32) EDT_POP(EDT_F32, EDT_F32);
    else if (gdt == EDT_F32) EDT_POP(EDT_F32, EDT_BF16);
    else EDT_POP(EDT_BF16, EDT_BF16);
#undef EDT_POP
    return check_launch("pair_population_kernel");
}

int edt_lerp(const void* v0, const void* v1, int in_dt, void* out, int out_dt, int cdt, uint64_t n,
             double t, void* stream) {
    g_err[0] = 0;
    if ((in_dt | out_dt | cdt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (in_dt == EDT_F32 && cdt == EDT_BF16) return fail(EDT_ERR_ARG, "bf16 compute of fp32 inputs unsupported");
    if (n == 0) return EDT_OK;
    if (!v0 || !v1 || !out) return fail(EDT_ERR_ARG, "null buffer");
    const float c0 = (float)(1.0 - t), c1 = (float)t;
    const bool vec = aligned16(v0) && aligned16(v1) && aligned16(out);
    const unsigned g = grid_for(n, vec);
    hipStream_t s = (hipStream_t)stream;
#define EDT_LERP(I, O, C)                                                                  \
    do {                                                                                   \
        if (vec) lerp_kernel<I, O, C, kVec><<<g, kBlock, 0, s>>>(v0, v1, out, n, c0, c1);   \
        else lerp_kernel<I, O, C, 1><<<g, kBlock, 0, s>>>(v0, v1, out, n, c0, c1);          \
    } while (0)
    if (in_dt == EDT_F32) {
        if (out_dt == EDT_F32) EDT_LERP(EDT_F32, EDT_F32, EDT_F32);
        else EDT_LERP(EDT_F32, EDT_BF16, EDT_F32);
    } else if (cdt == EDT_F32) {
        if (out_dt == EDT_F32) EDT_LERP(EDT_BF16, EDT_F32, EDT_F32);
        else EDT_LERP(EDT_BF16, EDT_BF16, EDT_F32);
    } else {
        if (out_dt == EDT_F32) EDT_LERP(EDT_BF16, EDT_F32, EDT_BF16);
        else EDT_LERP(EDT_BF16, EDT_BF16, EDT_BF16);
    }
#undef EDT_LERP
    return check_launch("lerp_kernel");
}

int64_t edt_slerp_make_chunks(const uint64_t* seg_offsets, int nseg, uint32_t chunk_elems,
                              uint64_t* chunk_desc, int64_t max_chunks, int32_t* seg_first_chunk) {
    g_err[0] = 0;
    if (nseg < 0 || !seg_offsets || chunk_elems == 0) return fail(EDT_ERR_ARG, "bad segment table");
    int64_t c = 0;
    for (int s = 0; s < nseg; ++s) {
        if (seg_first_chunk) seg_first_chunk[s] = (int32_t)c;
        const uint64_t a = seg_offsets[s], b = seg_offsets[s + 1];
        if (b < a) return fail(EDT_ERR_ARG, "segment offsets decrease at segment %d", s);
        for (uint64_t x = a; x < b; x += chunk_elems) {
            if (c < max_chunks && chunk_desc) {
                chunk_desc[3 * c] = x;
                chunk_desc[3 * c + 1] = (b - x) < chunk_elems ? (b - x) : chunk_elems;
                chunk_desc[3 * c + 2] = (uint64_t)s;
            }
            ++c;
        }
    }
    if (seg_first_chunk) seg_first_chunk[nseg] = (int32_t)c;
    if (c > max_chunks) return -c - 1;
    return c;
}

}  // extern "C"

namespace {

int slerp_stats_impl(const void* v0, const void* v1, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                     double* partial, const uint64_t* seg_ptrs, void* stream) {
    if (in_dt & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nchunks == 0) return EDT_OK;
    if (!chunk_desc || !partial) return fail(EDT_ERR_ARG, "null buffer");
    const unsigned g = slerp_grid(nchunks);
    hipStream_t s = (hipStream_t)stream;
    if (in_dt == EDT_F32) slerp_stats_kernel<EDT_F32><<<g, kBlock, 0, s>>>(v0, v1, chunk_desc, nchunks, partial, seg_ptrs);
    else slerp_stats_kernel<EDT_BF16><<<g, kBlock, 0, s>>>(v0, v1, chunk_desc, nchunks, partial, seg_ptrs);
    return check_launch("slerp_stats_kernel");
}

int slerp_blend_impl(const void* v0, const void* v1, int in_dt, void* out, int out_dt, const uint64_t* chunk_desc,
                     int64_t nchunks, const float* coef, const uint64_t* seg_ptrs, void* stream, bool nt = true) {
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nchunks == 0) return EDT_OK;
    if (!chunk_desc || !coef) return fail(EDT_ERR_ARG, "null buffer");
    const unsigned g = slerp_grid(nchunks);
    hipStream_t s = (hipStream_t)stream;
    if (in_dt == EDT_F32 && out_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_F32><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs);
    else if (in_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_BF16><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs);
    else if (out_dt == EDT_F32 && nt)
        slerp_blend_kernel<EDT_BF16, EDT_F32><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs);
    else if (out_dt == EDT_F32)
        slerp_blend_kernel<EDT_BF16, EDT_F32, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs);
    else if (nt)
        slerp_blend_kernel<EDT_BF16, EDT_BF16><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs);
    else
        slerp_blend_kernel<EDT_BF16, EDT_BF16, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs);
    return check_launch("slerp_blend_kernel");
}

}  // namespace

extern "C" {

int edt_slerp_stats(const void* v0, const void* v1, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                    double* partial, void* stream) {
    g_err[0] = 0;
    if (nchunks == 0) return EDT_OK;
    if (!v0 || !v1) return fail(EDT_ERR_ARG, "null buffer");
    if (!aligned16(v0) || !aligned16(v1)) return fail(EDT_ERR_ARG, "slerp inputs must be 16-byte aligned");
    return slerp_stats_impl(v0, v1, in_dt, chunk_desc, nchunks, partial, nullptr, stream);
}

int edt_slerp_coef(const double* partial, const int32_t* seg_first_chunk, int nseg, const double* t,
                   double dot_threshold, double eps, float* coef, float* dot_out, void* stream) {
    g_err[0] = 0;
    if (nseg == 0) return EDT_OK;
    if (!partial || !seg_first_chunk || !t || !coef) return fail(EDT_ERR_ARG, "null buffer");
    const unsigned g = coef_grid(nseg);
    slerp_coef_kernel<<<g, kBlock, 0, (hipStream_t)stream>>>(partial, seg_first_chunk, nseg, t,
                                                            (float)dot_threshold, (float)eps, coef, dot_out);
    return check_launch("slerp_coef_kernel");
}

int edt_slerp_blend(const void* v0, const void* v1, int in_dt, void* out, int out_dt, const uint64_t* chunk_desc,
                    int64_t nchunks, const float* coef, void* stream) {
    g_err[0] = 0;
    if (nchunks == 0) return EDT_OK;
    if (!v0 || !v1 || !out) return fail(EDT_ERR_ARG, "null buffer");
    if (!aligned16(v0) || !aligned16(v1) || !aligned16(out))
        return fail(EDT_ERR_ARG, "slerp buffers must be 16-byte aligned");
    return slerp_blend_impl(v0, v1, in_dt, out, out_dt, chunk_desc, nchunks, coef, nullptr, stream);
}

int edt_slerp_merge(const void* v0, const void* v1, int in_dt, void* out, int out_dt, const uint64_t* chunk_desc,
                    int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t, double dot_threshold,
                    double eps, double* partial, float* coef, float* dot_out, void* stream) {
    int rc = edt_slerp_stats(v0, v1, in_dt, chunk_desc, nchunks, partial, stream);
    if (rc) return rc;
    rc = edt_slerp_coef(partial, seg_first_chunk, nseg, t, dot_threshold, eps, coef, dot_out, stream);
    if (rc) return rc;
    return edt_slerp_blend(v0, v1, in_dt, out, out_dt, chunk_desc, nchunks, coef, stream);
}

uint64_t edt_slerp_population_gram_doubles(int nmembers, int64_t nchunks) {
    if (nmembers < 1 || nmembers > kGramMaxMembers || nchunks < 0) return 0;
    return (uint64_t)nchunks * (uint64_t)(nmembers * (nmembers + 1) / 2);
}

int edt_slerp_population(const void* const* members, int nmembers, int in_dt, const int32_t* pairs, int npairs,
                         void* const* outs, int out_dt, const uint64_t* chunk_desc, int64_t nchunks,
                         const int32_t* seg_first_chunk, int nseg, const double* t, double dot_threshold,
                         double eps, double* gram, float* coef, float* dot_out, void* stream) {
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nmembers < 1 || nmembers > kGramMaxMembers)
        return fail(EDT_ERR_ARG, "member count %d out of range [1, %d]", nmembers, kGramMaxMembers);
    if (npairs < 0 || nseg < 0 || nchunks < 0) return fail(EDT_ERR_ARG, "negative count");
    if (npairs == 0 || nseg == 0 || nchunks == 0) return EDT_OK;
    if (!members || !pairs || !outs || !chunk_desc || !seg_first_chunk || !t || !gram || !coef)
        return fail(EDT_ERR_ARG, "null buffer");
    Members mem;
    memset(&mem, 0, sizeof(mem));
    for (int m = 0; m < nmembers; ++m) {
        if (!aligned16(members[m]) || !members[m]) return fail(EDT_ERR_ARG, "member %d is null or not 16-byte aligned", m);
        mem.p[m] = members[m];
    }
    for (int q = 0; q < npairs; ++q) {
        const int i = pairs[2 * q], j = pairs[2 * q + 1];
        if (i < 0 || j < 0 || i >= nmembers || j >= nmembers) return fail(EDT_ERR_ARG, "pair %d: member out of range", q);
        if (!outs[q] || !aligned16(outs[q])) return fail(EDT_ERR_ARG, "output %d is null or not 16-byte aligned", q);
        for (int m = 0; m < nmembers; ++m)
            if (outs[q] == members[m]) return fail(EDT_ERR_ARG, "output %d aliases member %d", q, m);
    }
    hipStream_t s = (hipStream_t)stream;
    const unsigned g = slerp_grid(nchunks);
#define EDT_GRAM(M)                                                                                  \
    case M:                                                                                          \
        if (in_dt == EDT_F32) slerp_gram_kernel<EDT_F32, M><<<g, kBlock, 0, s>>>(mem, chunk_desc, nchunks, gram); \
        else slerp_gram_kernel<EDT_BF16, M><<<g, kBlock, 0, s>>>(mem, chunk_desc, nchunks, gram);              \
        break;
    switch (nmembers) {
        EDT_GRAM(1) EDT_GRAM(2) EDT_GRAM(3) EDT_GRAM(4) EDT_GRAM(5) EDT_GRAM(6) EDT_GRAM(7) EDT_GRAM(8)
    }
#undef EDT_GRAM
    int rc = check_launch("slerp_gram_kernel");
    if (rc) return rc;
    const int M = nmembers, NT = M * (M + 1) / 2;
    const unsigned gc = coef_grid(nseg);
    for (int q = 0; q < npairs; ++q) {
        const int i = pairs[2 * q], j = pairs[2 * q + 1];
        const int lo = i < j ? i : j, hi = i < j ? j : i;
        slerp_gram_coef_kernel<<<gc, kBlock, 0, s>>>(gram, NT, tri_index(i, i, M), tri_index(j, j, M),
                                                     tri_index(lo, hi, M), seg_first_chunk, nseg, t,
                                                     (float)dot_threshold, (float)eps, coef + 2 * (size_t)nseg * q,
                                                     dot_out ? dot_out + (size_t)nseg * q : nullptr);
        rc = check_launch("slerp_gram_coef_kernel");
        if (rc) return rc;
    }
    // the blends: every child in one co-located launch (groups of <= 16 children)
    for (int q0 = 0; q0 < npairs; q0 += kBlendMaxChildren) {
        BlendChildren B;
        memset(&B, 0, sizeof(B));
        B.nchildren = npairs - q0 < kBlendMaxChildren ? npairs - q0 : kBlendMaxChildren;
        for (int k = 0; k < B.nchildren; ++k) {
            const int q = q0 + k;
            B.v0[k] = members[pairs[2 * q]];
            B.v1[k] = members[pairs[2 * q + 1]];
            B.out[k] = outs[q];
            B.coef[k] = coef + 2 * (size_t)nseg * q;
        }
        const uint64_t blocks = ((uint64_t)nchunks + 7) / 8 * 8ull * (uint64_t)B.nchildren;
        if (blocks > 0x7fffffffull) return fail(EDT_ERR_ARG, "too many chunks for one launch");
        const unsigned gb = (unsigned)blocks;
        if (in_dt == EDT_F32 && out_dt == EDT_F32)
            slerp_blend_population_kernel<EDT_F32, EDT_F32><<<gb, kBlock, 0, s>>>(B, chunk_desc, nchunks);
        else if (in_dt == EDT_F32)
            slerp_blend_population_kernel<EDT_F32, EDT_BF16><<<gb, kBlock, 0, s>>>(B, chunk_desc, nchunks);
        else if (out_dt == EDT_F32)
            slerp_blend_population_kernel<EDT_BF16, EDT_F32><<<gb, kBlock, 0, s>>>(B, chunk_desc, nchunks);
        else
            slerp_blend_population_kernel<EDT_BF16, EDT_BF16><<<gb, kBlock, 0, s>>>(B, chunk_desc, nchunks);
        rc = check_launch("slerp_blend_population_kernel");
        if (rc) return rc;
    }
    return EDT_OK;
}

int edt_slerp_merge_speculative(const void* v0, const void* v1, int in_dt, void* out, int out_dt,
                                const uint64_t* chunk_desc, int64_t nchunks, const int32_t* seg_first_chunk,
                                int nseg, const double* t, double dot_threshold, double eps, double* partial,
                                float* coef, float* dot_out, int32_t* redo, uint64_t n, void* stream) {
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nseg == 0 || nchunks == 0) return EDT_OK;
    if (!v0 || !v1 || !out || !chunk_desc || !seg_first_chunk || !t || !partial || !coef || !redo)
        return fail(EDT_ERR_ARG, "null buffer");
    if (!aligned16(v0) || !aligned16(v1) || !aligned16(out))
        return fail(EDT_ERR_ARG, "slerp buffers must be 16-byte aligned");
    // the first pass writes `out` while the second may still need both parents
    const uintptr_t o0 = reinterpret_cast<uintptr_t>(out), o1 = o0 + n * (out_dt == EDT_BF16 ? 2 : 4);
    const uint64_t isz = in_dt == EDT_BF16 ? 2 : 4;
    for (const void* p : {v0, v1}) {
        const uintptr_t p0 = reinterpret_cast<uintptr_t>(p), p1 = p0 + n * isz;
        if (p0 < o1 && o0 < p1) return fail(EDT_ERR_ARG, "speculative SLERP needs an output apart from the parents");
    }
    hipStream_t s = (hipStream_t)stream;
    const unsigned g = slerp_grid(nchunks);
    if (in_dt == EDT_F32 && out_dt == EDT_F32)
        slerp_stats_lerp_kernel<EDT_F32, EDT_F32><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, partial, t);
    else if (in_dt == EDT_F32)
        slerp_stats_lerp_kernel<EDT_F32, EDT_BF16><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, partial, t);
    else if (out_dt == EDT_F32)
        slerp_stats_lerp_kernel<EDT_BF16, EDT_F32><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, partial, t);
    else
        slerp_stats_lerp_kernel<EDT_BF16, EDT_BF16><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, partial, t);
    int rc = check_launch("slerp_stats_lerp_kernel");
    if (rc) return rc;
    slerp_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(partial, seg_first_chunk, nseg, t, (float)dot_threshold,
                                                         (float)eps, coef, dot_out, redo);
    rc = check_launch("slerp_coef_kernel");
    if (rc) return rc;
    if (in_dt == EDT_F32 && out_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_F32><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo);
    else if (in_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_BF16><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo);
    else if (out_dt == EDT_F32)
        slerp_blend_kernel<EDT_BF16, EDT_F32><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo);
    else
        slerp_blend_kernel<EDT_BF16, EDT_BF16><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo);
    return check_launch("slerp_blend_kernel");
}

int edt_slerp_population_speculative(const void* const* members, int nmembers, int in_dt, const int32_t* pairs,
                                     int npairs, void* const* outs, int out_dt, const uint64_t* chunk_desc,
                                     int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t,
                                     double dot_threshold, double eps, double* partial, float* coef,
                                     float* dot_out, int32_t* redo, uint64_t n, void* stream) {
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nmembers < 1 || npairs < 0 || nseg < 0 || nchunks < 0) return fail(EDT_ERR_ARG, "bad count");
    if (npairs == 0 || nseg == 0 || nchunks == 0) return EDT_OK;
    if (!members || !pairs || !outs || !chunk_desc || !seg_first_chunk || !t || !partial || !coef || !redo)
        return fail(EDT_ERR_ARG, "null buffer");
    const uint64_t isz = in_dt == EDT_BF16 ? 2 : 4, osz = out_dt == EDT_BF16 ? 2 : 4;
    for (int m = 0; m < nmembers; ++m)
        if (!members[m] || !aligned16(members[m])) return fail(EDT_ERR_ARG, "member %d is null or not 16-byte aligned", m);
    for (int q = 0; q < npairs; ++q) {
        const int i = pairs[2 * q], j = pairs[2 * q + 1];
        if (i < 0 || j < 0 || i >= nmembers || j >= nmembers) return fail(EDT_ERR_ARG, "pair %d: member out of range", q);
        if (!outs[q] || !aligned16(outs[q])) return fail(EDT_ERR_ARG, "output %d is null or not 16-byte aligned", q);
        const uintptr_t o0 = reinterpret_cast<uintptr_t>(outs[q]), o1 = o0 + n * osz;
        for (int m = 0; m < nmembers; ++m) {           // outputs are written before the redo pass
            const uintptr_t p0 = reinterpret_cast<uintptr_t>(members[m]), p1 = p0 + n * isz;
            if (p0 < o1 && o0 < p1) return fail(EDT_ERR_ARG, "output %d overlaps member %d", q, m);
        }
    }
    hipStream_t s = (hipStream_t)stream;
    for (int pass = 0; pass < 2; ++pass) {
        for (int q0 = 0; q0 < npairs; q0 += kBlendMaxChildren) {
            BlendChildren B;
            memset(&B, 0, sizeof(B));
            B.nchildren = npairs - q0 < kBlendMaxChildren ? npairs - q0 : kBlendMaxChildren;
            for (int k = 0; k < B.nchildren; ++k) {
                const int q = q0 + k;
                B.v0[k] = members[pairs[2 * q]];
                B.v1[k] = members[pairs[2 * q + 1]];
                B.out[k] = outs[q];
                B.coef[k] = coef + 2 * (size_t)nseg * q;
                B.redo[k] = redo + (size_t)nseg * q;
                B.partial[k] = partial + 3 * (size_t)nchunks * q;
            }
            const uint64_t blocks = ((uint64_t)nchunks + 7) / 8 * 8ull * (uint64_t)B.nchildren;
            if (blocks > 0x7fffffffull) return fail(EDT_ERR_ARG, "too many chunks for one launch");
            const unsigned gb = (unsigned)blocks;
#define EDT_SPEC_POP(KERNEL, ...)                                                                   \
    do {                                                                                            \
        if (in_dt == EDT_F32 && out_dt == EDT_F32) KERNEL<EDT_F32, EDT_F32><<<gb, kBlock, 0, s>>>(__VA_ARGS__);   \
        else if (in_dt == EDT_F32) KERNEL<EDT_F32, EDT_BF16><<<gb, kBlock, 0, s>>>(__VA_ARGS__);                  \
        else if (out_dt == EDT_F32) KERNEL<EDT_BF16, EDT_F32><<<gb, kBlock, 0, s>>>(__VA_ARGS__);                 \
        else KERNEL<EDT_BF16, EDT_BF16><<<gb, kBlock, 0, s>>>(__VA_ARGS__);                                       \
    } while (0)
            if (pass == 0) EDT_SPEC_POP(slerp_pop_stats_lerp_kernel, B, chunk_desc, nchunks, t);
            else EDT_SPEC_POP(slerp_blend_population_kernel, B, chunk_desc, nchunks);
#undef EDT_SPEC_POP
            int rc = check_launch(pass == 0 ? "slerp_pop_stats_lerp_kernel" : "slerp_blend_population_kernel");
            if (rc) return rc;
        }
        if (pass == 0) {
            for (int q = 0; q < npairs; ++q) {
                slerp_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(
                    partial + 3 * (size_t)nchunks * q, seg_first_chunk, nseg, t, (float)dot_threshold, (float)eps,
                    coef + 2 * (size_t)nseg * q, dot_out ? dot_out + (size_t)nseg * q : nullptr, redo + (size_t)nseg * q);
                int rc = check_launch("slerp_coef_kernel");
                if (rc) return rc;
            }
        }
    }
    return EDT_OK;
}

int edt_slerp_merge_list(const void* const* v0_t, const void* const* v1_t, int in_dt, void* const* out_t,
                         int out_dt, const uint64_t* chunk_desc, int64_t nchunks, const int32_t* seg_first_chunk,
                         int nseg, const double* t, double dot_threshold, double eps, double* partial, float* coef,
                         float* dot_out, void* workspace, uint64_t workspace_bytes, void* stream) {
    g_err[0] = 0;
    if (nseg < 0) return fail(EDT_ERR_ARG, "segment count %d < 0", nseg);
    if (nseg == 0 || nchunks == 0) return EDT_OK;
    if (!v0_t || !v1_t || !out_t) return fail(EDT_ERR_ARG, "null tensor table");
    const uint64_t need = 3ull * sizeof(uint64_t) * (uint64_t)nseg;
    if (!workspace || workspace_bytes < need)
        return fail(EDT_ERR_ARG, "workspace of %llu bytes needed", (unsigned long long)need);
    if (reinterpret_cast<uintptr_t>(workspace) & 7u) return fail(EDT_ERR_ARG, "workspace must be 8-byte aligned");
    thread_local std::vector<uint64_t> h;
    h.assign(3 * (size_t)nseg, 0);
    for (int i = 0; i < nseg; ++i) {
        // a null pointer is only valid for an empty segment (it has no chunks, so it is never read)
        if (!aligned16(v0_t[i]) || !aligned16(v1_t[i]) || !aligned16(out_t[i]))
            return fail(EDT_ERR_ARG, "tensor %d is not 16-byte aligned", i);
        h[3 * i] = reinterpret_cast<uintptr_t>(v0_t[i]);
        h[3 * i + 1] = reinterpret_cast<uintptr_t>(v1_t[i]);
        h[3 * i + 2] = reinterpret_cast<uintptr_t>(out_t[i]);
    }
    // pageable source: staged before hipMemcpyAsync returns, stream-ordered on the device
    hipError_t e = hipMemcpyAsync(workspace, h.data(), need, hipMemcpyHostToDevice, (hipStream_t)stream);
    if (e != hipSuccess) return fail(EDT_ERR_LAUNCH, "tensor table upload failed: %s", hipGetErrorString(e));
    const uint64_t* seg_ptrs = static_cast<const uint64_t*>(workspace);
    int rc = slerp_stats_impl(nullptr, nullptr, in_dt, chunk_desc, nchunks, partial, seg_ptrs, stream);
    if (rc) return rc;
    rc = edt_slerp_coef(partial, seg_first_chunk, nseg, t, dot_threshold, eps, coef, dot_out, stream);
    if (rc) return rc;
    return slerp_blend_impl(nullptr, nullptr, in_dt, nullptr, out_dt, chunk_desc, nchunks, coef, seg_ptrs, stream);
}

}  // extern "C"
