// edt_merge.hip — the EDT-LM pair merge (EDT_LM/train/crossover.py:150-232), its population
// form, and lerp, with their C ABI entries (include/edt_sync.h).
#include "edt_common.h"

namespace {

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

// The merge of one child from its already-loaded inputs (lerp base from x = b1, y = b2; trained
// weights d1 = m1, d2 = m2; carried buffer b_in).
template <int GDT, int WDT, int N>
__device__ __forceinline__ void pair_core(const PairArgs& a, uint64_t i, float (&x)[N], float (&y)[N],
                                          float (&d1)[N], float (&d2)[N], const float (&b_in)[N]) {
    float base[N];
#pragma unroll
    for (int j = 0; j < N; ++j) { x[j] = x[j] * 0.5f; y[j] = y[j] * 0.5f; }   // (1-.5)*v0, .5*v1
    rnd<WDT>(x);
    rnd<WDT>(y);
#pragma unroll
    for (int j = 0; j < N; ++j) base[j] = x[j] + y[j];
    rnd<WDT>(base);
    rnd<GDT>(base);                    // load_state_dict into the base model's dtype
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

template <int GDT, int WDT, int N, bool NT = (EDT_NT_LOADS != 0 && WDT == EDT_BF16)>
__device__ __forceinline__ void pair_elems(const PairArgs& a, uint64_t i) {
    float b_in[N];
    ld_momentum<GDT, N>(a.mom_in, i, a.sgd, b_in);
    if (a.b2) {                        // run_linear_merge_5050: lerp(0.5, b1, b2) in the model dtype
        float x[N], y[N], d1[N], d2[N];
        ld<WDT, N, NT>(a.b1, i, x);
        ld<WDT, N, NT>(a.b2, i, y);
        ld<WDT, N, NT>(a.m1, i, d1);
        ld<WDT, N, NT>(a.m2, i, d2);
        pair_core<GDT, WDT, N>(a, i, x, y, d1, d2, b_in);
        return;
    }
    float base[N];                     // run_sgd on an already merged base model (dtype GDT)
    ld<GDT, N>(a.b1, i, base);
    rnd<GDT>(base);
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
    for (int j = 0; j < N; ++j) d1[j] = d1[j] * 0.5f;
    rnd<GDT>(d1);
    float grad[N];
#pragma unroll
    for (int j = 0; j < N; ++j) grad[j] = -(0.f + d1[j]);
    sgd_update<GDT, N>(base, grad, a.mom, i, a.sgd, b_in);
    st<GDT, N>(a.out, i, base);
}

template <int GDT, int WDT, int N>
__global__ __launch_bounds__(kBlock) void pair_kernel(PairArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = xcd_block(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
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
#ifndef EDT_POP_ITERS             // 8-element iterations per thread per population chunk
#define EDT_POP_ITERS 4
#endif
constexpr uint64_t kPopChunk = (uint64_t)kBlock * kVec * EDT_POP_ITERS;   // 8192 elements per workgroup

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


// Closed by measurement (profiles/HISTORY.md §C): a member-major form (each thread loads every distinct
// parent's tiles once and runs the children from its registers: 17.2-17.7 ms r4, 20.4 / 26.9 ms
// r5 on rank-selected pairs, against 15.7-16.7 co-located) and a child loop inside the thread
// (parents re-read from L1): both removed.

// ---------------------------------------------------------------------------------------
// lerp with a scalar t (lerp_elems in edt_common.h)

template <int IDT, int ODT, int CDT, int N>
__global__ __launch_bounds__(kBlock) void lerp_kernel(const void* v0, const void* v1, void* out,
                                                      uint64_t n, float c0, float c1) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if constexpr (N == kVec) {
        const uint64_t nv = n / kVec;
        for (uint64_t v = tid; v < nv; v += stride)
            lerp_elems<IDT, ODT, CDT, kVec, EDT_NT_LERP != 0, EDT_NT_LERP_STORES != 0>(v0, v1, out, v * kVec, c0, c1);
        const uint64_t t = nv * kVec + tid;
        if (t < n) lerp_elems<IDT, ODT, CDT, 1>(v0, v1, out, t, c0, c1);
    } else {
        for (uint64_t e = tid; e < n; e += stride) lerp_elems<IDT, ODT, CDT, 1>(v0, v1, out, e, c0, c1);
    }
}


}  // namespace

extern "C" {

int edt_pair_merge(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                   void* theta_out, int gdt, void* momentum, int has_momentum, uint64_t n, double lr,
                   double momentum_coef, int nesterov, void* stream) {
    return edt_pair_merge_to(b1, b2, m1, m2, wdt, theta_out, gdt, momentum, momentum, has_momentum, n, lr,
                             momentum_coef, nesterov, stream);
}

int edt_pair_merge_tail(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                        void* theta_out, int gdt, const void* momentum_in, void* momentum, int has_momentum,
                        uint64_t n, double lr, double momentum_coef, int nesterov, const uint8_t* tail_bits,
                        void* stream);

int edt_pair_merge_to(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                      void* theta_out, int gdt, const void* momentum_in, void* momentum, int has_momentum,
                      uint64_t n, double lr, double momentum_coef, int nesterov, void* stream) {
    return edt_pair_merge_tail(b1, b2, m1, m2, wdt, theta_out, gdt, momentum_in, momentum, has_momentum, n, lr,
                               momentum_coef, nesterov, nullptr, stream);
}

int edt_pair_merge_tail(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                        void* theta_out, int gdt, const void* momentum_in, void* momentum, int has_momentum,
                        uint64_t n, double lr, double momentum_coef, int nesterov, const uint8_t* tail_bits,
                        void* stream) {
    g_err[0] = 0;
    if (!valid_pair(gdt, wdt)) return fail(EDT_ERR_ARG, "unsupported dtype pair (gdt/wdt)");
    if (n == 0) return EDT_OK;
    if (!b1 || !m1 || !m2 || !theta_out) return fail(EDT_ERR_ARG, "null buffer");
    PairArgs a;
    a.b1 = b1; a.b2 = b2; a.m1 = m1; a.m2 = m2; a.out = theta_out; a.mom = momentum; a.n = n;
    a.mom_in = momentum_in;
    a.sgd = make_sgd(gdt, lr, momentum_coef, has_momentum, nesterov);
    if (gdt == EDT_BF16) a.sgd.tail = tail_bits;    // fp32: nothing to emulate
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
    if (blocks > kGridBlockCap) return fail(EDT_ERR_ARG, "too many elements for one launch");
    const unsigned g = (unsigned)blocks;
    hipStream_t s = (hipStream_t)stream;
#define EDT_POP(G, W)                                                                   \
    do {                                                                                \
        if (vec) pair_population_kernel<G, W, true><<<g, kBlock, 0, s>>>(P);            \
        else pair_population_kernel<G, W, false><<<g, kBlock, 0, s>>>(P);              \
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


}  // extern "C"
