// edt_common.h — what every kernel translation unit of libedt_sync.so shares: the build-time
// tunables, vector types, bf16 rounding, the 8-element load/store addressing, torch's SGD update
// restated per element, lerp_elems, the error plumbing and host-side launch helpers. The kernels
// live in edt_outer.hip (DiLoCo), edt_merge.hip (pair merge, lerp), edt_slerp.hip (SLERP) and
// their C ABI (include/edt_sync.h) beside them; edt_abi.hip holds the error message and version.
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
#pragma once

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include "edt_sync.h"

// edt_last_error(): one thread-local message for the whole library (defined in edt_abi.hip).
namespace edt {
extern thread_local char g_err[512];
}

namespace {
using edt::g_err;


// Tunables (overridable at build time for the variant sweep in scripts/kernel_variants.py).
// Grid: one pass (EDT_BLOCKS_PER_CU 0: one 2048-element tile per workgroup, dispatched in address
// order, so the chip's in-flight window stays one contiguous stretch of every stream). With the
// momentum placed by measurement (placement.py) it beats 256 grid-stride blocks per CU on every
// 1.3B regime and op (profiles/r01_oneshot.json): outer step fp32 10.74 -> 10.48 ms, bf16
// workers 6.85 -> 6.74, all bf16 5.44 -> 5.24, pair merge 3.50 -> 3.13, lerp 1.53 -> 1.31 ms;
// 125M equal. (Before the placement search the two were within noise, profiles/r01_variants.txt,
// which is why 256 per CU shipped first: 6.78 ms vs 7.36 ms for 8 per CU.)
#ifndef EDT_BLOCKS_PER_CU
#define EDT_BLOCKS_PER_CU 0
#endif
#ifndef EDT_NT_LOADS          // non-temporal loads for the once-read bf16 worker streams
#define EDT_NT_LOADS 1        // (fp32 streams: measured 1.6x SLOWER with nt, 17.5 vs 11.2 ms)
#endif
#ifndef EDT_NT_RMW            // non-temporal loads for theta / momentum (read, then rewritten)
#define EDT_NT_RMW 0
#endif
#ifndef EDT_NT_STORES         // non-temporal stores for theta / momentum
#define EDT_NT_STORES 0
#endif

#ifndef EDT_NT_LERP             // non-temporal loads of lerp's two (read-once) inputs
#define EDT_NT_LERP 0
#endif
#ifndef EDT_NT_LERP_STORES      // non-temporal stores of lerp's child (written once, never re-read by
#define EDT_NT_LERP_STORES 1    // the merge): r6, interleaved on the same buffers, bits identical —
#endif                          // 1.3B 1.323 vs 1.340 ms, 7B body 6.957 vs 7.053 ms; the pair merge
                                // measured no gain (3.05 vs 3.00 ms at 1.3B, equal at 7B) and keeps
                                // ordinary stores (profiles/r06_store_kind_probe.jsonl)
// SLERP of two Qwen2.5-7B bodies (bf16, profiles/r01_slerp_variants.json, two boxes): non-temporal
// parent loads + one workgroup per segment for the chunk-sum reduction + 64 Ki-element chunks
// 11.23 / 11.41 ms, against 12.14 / 12.27 ms for default loads, one wave per segment and 16 Ki
// chunks. The population form (edt_slerp_population) keeps default-policy loads (2 % faster).
#ifndef EDT_NT_SLERP_STORES     // non-temporal stores of the pair SLERP's children (the speculative
#define EDT_NT_SLERP_STORES 1   // pass's lerp outputs, the blends): r5, 7B lineage 6.63 vs 7.16 ms,
#endif                          // blend 6.44 vs 6.84 (profiles/r05_nt_stores_variants.log)
#ifndef EDT_NT_SLERP            // non-temporal loads of the SLERP parents (stats and blend passes)
#define EDT_NT_SLERP 1
#endif
// 512-element tiles per wave in the read-only chunk-sum pass (4, 8 or 16; the sums' order is the
// same for every value, edt_slerp.hip). 7B body, bf16, one box (profiles/r03_slerp_stats_tpw.jsonl):
// 4.44 / 4.21 / 4.09 ms for 4 / 8 / 16 — a read-only stream wants many bytes in flight per wave
// (16: 142 VGPRs, 3 waves per SIMD, 256 B per lane outstanding).
#ifndef EDT_SLERP_STATS_TPW
#define EDT_SLERP_STATS_TPW 16
#endif
// Speculative passes (pair and co-located population): 1 = the four waves' tile sums combined
// through LDS into one level-2 row per workgroup (a quarter of the row bytes, one barrier); 0 = a
// level-0 row per wave, no barrier. 7B lineage merge, one box, interleaved (profiles/
// r03_spec_wg_rows.jsonl): 7.01-7.03 ms against 7.14-7.17, lerp 6.96.
// Population stats passes (the needed / triangle sums, edt_slerp.hip): non-temporal member loads
// (each member is read once; r4, 8 x 7B two-pass generation: nt alone 57.7 / 57.9 ms against 58.0
// / 58.3 without, profiles/r04_gram_variants.json)
#ifndef EDT_GRAM_NT
#define EDT_GRAM_NT 1
#endif
// Needed-sums pass (r5, edt_slerp.hip): elements converted to fp64 per group before the dot
// slots' switches (4: two groups per lane vector; 2: four).
#ifndef EDT_NEED_GROUP
#define EDT_NEED_GROUP 8
#endif
#ifndef EDT_NEED_MIN_WAVES      // needed-sums pass: __launch_bounds__ minimum waves per SIMD
#define EDT_NEED_MIN_WAVES 1
#endif
#ifndef EDT_NEED_GLDS           // needed-sums pass: the next tile staged in LDS by DMA (bf16 members)
#define EDT_NEED_GLDS 1
#endif
#ifndef EDT_SLERP_SPEC_WG_ROWS
#define EDT_SLERP_SPEC_WG_ROWS 1
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
// HIP's dispatch limit: at most 2^32 - 1 work-items per grid dimension, i.e. 16,777,215 workgroups
// of kBlock threads. Every grid below is capped there and the kernels grid-stride past it.
constexpr uint64_t kGridBlockCap = 0xffffffffull / kBlock;
// grid cap for the grid-stride loops: 256 CUs x workgroups per CU (0 = one pass up to the dispatch cap)
constexpr uint64_t kMaxBlocks = EDT_BLOCKS_PER_CU > 0 ? 256ull * EDT_BLOCKS_PER_CU : kGridBlockCap;

// XCD-aware block order for the one-pass stream kernels (outer_kernel, pair_kernel). Workgroups
// are dispatched round-robin over the 8 XCDs (block b on XCD b % 8), so by default the XCDs
// interleave at one tile. EDT_XCD_RUN = M > 0 permutes the blocks so each XCD streams runs of M
// consecutive tiles (M = -1: one contiguous 1/8 of the arena per XCD). A permutation of
// [0, gridDim): every tile is still processed exactly once, by one workgroup.
#ifndef EDT_XCD_RUN
#define EDT_XCD_RUN 0
#endif
__device__ __forceinline__ uint64_t xcd_block(uint64_t b, uint64_t G) {
    if constexpr (EDT_XCD_RUN == 0) {
        return b;
    } else {
        const uint64_t M = EDT_XCD_RUN > 0 ? (uint64_t)EDT_XCD_RUN : G / 8;
        const uint64_t span = 8 * M;                 // blocks per group: M tiles on each XCD
        if (M == 0 || b >= G / span * span) return b;    // the ragged last group keeps its order
        const uint64_t g = b / span, x = b % 8, j = (b / 8) % M;
        return g * span + x * M + j;
    }
}

// the passes that skip most chunks (the speculative redo blends) or hold several parents' tiles in
// registers (the member-major blends) stay grid-stride over chunks, EDT_SLERP_SPEC_BPC per CU
#ifndef EDT_SLERP_SPEC_BPC
#define EDT_SLERP_SPEC_BPC 256
#endif
inline unsigned slerp_spec_grid(int64_t nchunks) {
    const uint64_t cap = 256ull * EDT_SLERP_SPEC_BPC;
    return (unsigned)((uint64_t)nchunks < cap ? (uint64_t)nchunks : cap);
}
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));



inline int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

inline int check_launch(const char* what) {
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
    // bf16 only, may be null: 1 bit per element (bit i & 7 of byte i >> 3, flat-arena index) set
    // where the reference's torch CPU kernels take their scalar tail, whose add(x, y, alpha) rounds
    // twice: round(x + round(alpha * y)) instead of one FMA (edt_outer_step_tail, edt_pair_merge_tail)
    const uint8_t* tail;
};

inline SgdScalars make_sgd(int gdt, double lr, double mu, int has_buf, int nesterov) {
    SgdScalars s;
    s.mul_mu = (float)mu;
    s.alpha_mu = gdt == EDT_BF16 ? host_round_bf16((float)mu) : (float)mu;
    s.alpha_nlr = gdt == EDT_BF16 ? host_round_bf16((float)(-lr)) : (float)(-lr);
    s.use_momentum = mu != 0.0;
    s.has_buf = has_buf;
    s.nesterov = nesterov;
    s.tail = nullptr;
    return s;
}

// torch.optim.sgd._single_tensor_sgd for one group of N elements, in regime GDT.
// grad is the pseudo-gradient (already in GDT precision); theta is updated in registers,
// the momentum buffer is read from / written to `mom` at element i.
// Loads the carried momentum buffer (issued together with the other operand loads).
template <int GDT, int N, int H2 = 4>
__device__ __forceinline__ void ld_momentum(const void* mom, uint64_t i, const SgdScalars& s, float (&b)[N]) {
    if (s.use_momentum && s.has_buf) ld<GDT, N, (EDT_NT_RMW != 0), H2>(mom, i, b);
}

// add(x, y, alpha) in bf16 where the tail bit is set: torch CPU's scalar form, alpha * y rounded
// to bf16 before the add (the vectorised form is one fp32 FMA; the caller rounds the sum)
__device__ __forceinline__ float tail_add(float x, float a, float y) {
    float p[1] = {a * y};
    rnd<EDT_BF16>(p);
    return x + p[0];
}

template <int GDT, int N, int H2 = 4>
__device__ __forceinline__ void sgd_update(float (&theta)[N], const float (&grad)[N], void* mom,
                                           uint64_t i, const SgdScalars& s, const float (&b_in)[N]) {
    uint32_t tb = 0;                   // scalar-tail bits of elements i .. i + N - 1
    if constexpr (GDT == EDT_BF16 && H2 == 4 && (N == 8 || N == 1)) {
        if (s.tail) tb = N == 8 ? (uint32_t)s.tail[i >> 3] : ((uint32_t)s.tail[i >> 3] >> (i & 7)) & 1u;
    }
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
            for (int j = 0; j < N; ++j)
                u[j] = (tb >> j) & 1u ? tail_add(grad[j], s.alpha_mu, b[j]) : __builtin_fmaf(s.alpha_mu, b[j], grad[j]);
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
    for (int j = 0; j < N; ++j)
        theta[j] = (tb >> j) & 1u ? tail_add(theta[j], s.alpha_nlr, u[j]) : __builtin_fmaf(s.alpha_nlr, u[j], theta[j]);
    rnd<GDT>(theta);
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


// ---------------------------------------------------------------------------------------
// host-side dispatch helpers

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline unsigned grid_for(uint64_t n, bool vec) {
    const uint64_t per = vec ? (uint64_t)kBlock * kVec : (uint64_t)kBlock;
    uint64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    if (g > kMaxBlocks) g = kMaxBlocks;
    return (unsigned)g;
}

inline bool valid_pair(int gdt, int wdt) {
    return (gdt == EDT_F32 && (wdt == EDT_F32 || wdt == EDT_BF16)) || (gdt == EDT_BF16 && wdt == EDT_BF16);
}


inline bool is_pow2(int k) { return k > 0 && (k & (k - 1)) == 0; }

}  // namespace
