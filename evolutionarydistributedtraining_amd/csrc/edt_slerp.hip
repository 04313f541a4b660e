// edt_slerp.hip — the SLERP crossover (EDT_RL/crossover.py:11-135,
// EDT_EVOMERGE/train/crossover.py:14-146): chunk sums, coefficients, blends, the speculative
// and population forms, with their C ABI entries (include/edt_sync.h).
#include "edt_common.h"

namespace {

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

// The element ranges a blend workgroup owns, as body(start, end, segment). TILES: one kTile of its
// chunk (tiles kTilesPerChunk apart for longer chunks; grid slerp_tile_grid) — the full blends.
// Else whole chunks, grid-stride (grid slerp_spec_grid) — the speculative redo blends, where most
// segments are skipped and a workgroup per tile would cost more to dispatch than it saves (7B
// lineage merge: 3.45 M empty workgroups = +1.1 ms). Tiles assume the plans' 64 Ki chunks: shorter
// chunks stay correct, with idle workgroups.
template <bool TILES, typename F>
__device__ __forceinline__ void for_blend_ranges(const uint64_t* chunks, int64_t nchunks, F&& body) {
    if constexpr (TILES && EDT_SLERP_GRID) {
        const uint64_t b = EDT_SLERP_BLEND_REV ? gridDim.x - 1 - blockIdx.x : blockIdx.x;
        const int64_t c = (int64_t)(b / kTilesPerChunk);
        if (c >= nchunks) return;
        const uint64_t start = chunks[3 * c], len = chunks[3 * c + 1], seg = chunks[3 * c + 2];
        for (uint64_t off = (b % kTilesPerChunk) * kTile; off < len;
             off += (uint64_t)kTilesPerChunk * kTile)
            body(start + off, start + (off + kTile < len ? off + kTile : len), seg);
    } else {
        for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x)
            body(chunks[3 * c], chunks[3 * c] + chunks[3 * c + 1], chunks[3 * c + 2]);
    }
}

// f(N, i) over [start, end): the 16-B-aligned body in 8-element vectors (workgroup-strided), then
// the < 16 head / tail elements one per thread.
template <typename F>
__device__ __forceinline__ void for_range_elems(uint64_t start, uint64_t end, F&& f) {
    const uint64_t a = (start + kVec - 1) / kVec * kVec;
    const uint64_t b = end / kVec * kVec;
    if (a < b) {
        for (uint64_t i = a + (uint64_t)threadIdx.x * kVec; i < b; i += (uint64_t)kBlock * kVec)
            f(std::integral_constant<int, kVec>{}, i);
    }
    const uint64_t h_end = a < end ? a : end;
    const uint64_t t_beg = b > a ? b : h_end;
    const uint64_t nh = h_end - start, nt = end - t_beg;
    if ((uint64_t)threadIdx.x < nh + nt)
        f(std::integral_constant<int, 1>{}, threadIdx.x < nh ? start + threadIdx.x : t_beg + (threadIdx.x - nh));
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
    // EDT_SLERP_SPEC_CONTIG = k > 0: workgroup b takes chunks [b k, b k + k) (address order);
    // 0: grid-stride. Either way each chunk's sums come from one workgroup in the same order.
    const int64_t c_first = EDT_SLERP_SPEC_CONTIG > 0 ? (int64_t)blockIdx.x * EDT_SLERP_SPEC_CONTIG : (int64_t)blockIdx.x;
    const int64_t c_step = EDT_SLERP_SPEC_CONTIG > 0 ? 1 : (int64_t)gridDim.x;
    const int64_t c_end = EDT_SLERP_SPEC_CONTIG > 0 ? (c_first + EDT_SLERP_SPEC_CONTIG < nchunks
                                                        ? c_first + EDT_SLERP_SPEC_CONTIG : nchunks) : nchunks;
    for (int64_t c = c_first; c < c_end; c += c_step) {
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

template <int IDT, int ODT, bool NT = (EDT_NT_SLERP != 0 && IDT == EDT_BF16), bool TILES = true>
__global__ __launch_bounds__(kBlock) void slerp_blend_kernel(const void* v0, const void* v1, void* out,
                                                             const uint64_t* chunks, int64_t nchunks,
                                                             const float* coef, const uint64_t* seg_ptrs,
                                                             const int32_t* redo = nullptr) {
    for_blend_ranges<TILES>(chunks, nchunks, [&](uint64_t start, uint64_t end, uint64_t seg) {
        if (redo && !redo[seg]) return;           // speculative lerp output already final
        const void* a = v0;
        const void* b = v1;
        void* o = out;
        if (seg_ptrs) {
            a = reinterpret_cast<const void*>(seg_ptrs[3 * seg]);
            b = reinterpret_cast<const void*>(seg_ptrs[3 * seg + 1]);
            o = reinterpret_cast<void*>(seg_ptrs[3 * seg + 2]);
        }
        const float c0 = coef[2 * seg], c1 = coef[2 * seg + 1];
        for_range_elems(start, end, [&](auto tagN, uint64_t i) {
            constexpr int N = decltype(tagN)::value;
            lerp_elems<IDT, ODT, EDT_F32, N, NT && N == kVec>(a, b, o, i, c0, c1);
        });
    });
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
                                                                 float* coef, float* dot_out, int32_t* redo = nullptr) {
    const int seg = coef_segment();
    if (seg >= nseg) return;
    double sums[3];
    if (!segment_sums(gram, NT, qi, qj, qd, first[seg], first[seg + 1], sums)) return;
    float c0, c1, dot;
    slerp_coefficients(sums[0], sums[1], sums[2], tvals[seg], thr, eps, c0, c1, dot);
    coef[2 * seg] = c0;
    coef[2 * seg + 1] = c1;
    if (dot_out) dot_out[seg] = dot;
    if (redo) redo[seg] = fabsf(dot) > thr ? 0 : 1;   // as slerp_coef_kernel
}

// The speculative population pass in member-major form: per chunk, every distinct parent's tile
// is loaded ONCE into registers; from it the thread accumulates the Gram sums (gram_accumulate's
// exact FMA order, so every child's sums equal chunk_sums' on its two parents) and writes every
// child's lerp-branch output (chunk_pass' EMIT math). A shared parent crosses HBM once for all
// its children regardless of cache residency.
struct PopLerp {
    void* out[kBlendMaxChildren];
    int32_t a[kBlendMaxChildren], b[kBlendMaxChildren];   // compact member indices of the parents
    int n;
};

template <int M, int N>
__device__ __forceinline__ void pick(const float (&x)[M][N], int idx, float (&y)[N]) {
#pragma unroll
    for (int m = 0; m < M; ++m)
        if (m == idx) {                 // idx is uniform across the workgroup: no divergence
#pragma unroll
            for (int j = 0; j < N; ++j) y[j] = x[m][j];
        }
}

template <int IDT, int ODT, int M, int N>
__device__ __forceinline__ void gram_lerp_elems(const Members& mem, const PopLerp& po, uint64_t i, float l0, float l1,
                                                double (&g)[M * (M + 1) / 2]) {
    float x[M][N];
#pragma unroll
    for (int m = 0; m < M; ++m) ld<IDT, N>(mem.p[m], i, x[m]);
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
    for (int q = 0; q < po.n; ++q) {
        float u[N], v[N], o[N];
        pick<M, N>(x, po.a[q], u);
        pick<M, N>(x, po.b[q], v);
#pragma unroll
        for (int j = 0; j < N; ++j) o[j] = l0 * u[j] + l1 * v[j];
        st<ODT, N>(po.out[q], i, o);
    }
}

template <int IDT, int ODT, int M>
__global__ __launch_bounds__(kBlock) void slerp_gram_lerp_kernel(Members mem, PopLerp po, const uint64_t* chunks,
                                                                 int64_t nchunks, const double* tvals, double* gram) {
    constexpr int NT = M * (M + 1) / 2;
    __shared__ double red[NT][kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const uint64_t start = chunks[3 * c], end = start + chunks[3 * c + 1], seg = chunks[3 * c + 2];
        const float l0 = (float)(1.0 - tvals[seg]), l1 = (float)tvals[seg];
        double g[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) g[q] = 0.0;
        const uint64_t a = (start + kVec - 1) / kVec * kVec;
        const uint64_t b = end / kVec * kVec;
        if (a < b) {
            for (uint64_t i = a + (uint64_t)threadIdx.x * kVec; i < b; i += (uint64_t)kBlock * kVec)
                gram_lerp_elems<IDT, ODT, M, kVec>(mem, po, i, l0, l1, g);
        }
        const uint64_t h_end = a < end ? a : end;
        const uint64_t t_beg = b > a ? b : h_end;
        const uint64_t nh = h_end - start, nt = end - t_beg;
        if ((uint64_t)threadIdx.x < nh + nt) {
            const uint64_t i = threadIdx.x < nh ? start + threadIdx.x : t_beg + (threadIdx.x - nh);
            gram_lerp_elems<IDT, ODT, M, 1>(mem, po, i, l0, l1, g);
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

// The blends of every child in member-major form (the two-pass Gram form's second pass and the
// speculative form's redo pass, <= 8 distinct parents): per chunk each distinct parent's tile is
// loaded once and every child whose segment needs blending writes c0 v_i + c1 v_j from the same
// registers (lerp_elems' math with the child's coefficients, as slerp_blend_kernel).
struct PopBlend {
    void* out[kBlendMaxChildren];
    const float* coef[kBlendMaxChildren];     // [nseg][2] of the child
    const int32_t* redo[kBlendMaxChildren];   // [nseg] of the child, or null: blend every segment
    int32_t a[kBlendMaxChildren], b[kBlendMaxChildren];
    int n;
};

template <int IDT, int ODT, int M, int N>
__device__ __forceinline__ void blend_mm_elems(const Members& mem, const PopBlend& pb, uint64_t i, uint64_t seg,
                                               uint32_t need) {
    float x[M][N];
#pragma unroll
    for (int m = 0; m < M; ++m) ld<IDT, N>(mem.p[m], i, x[m]);
    for (int q = 0; q < pb.n; ++q) {
        if (!(need & (1u << q))) continue;
        float u[N], v[N], o[N];
        pick<M, N>(x, pb.a[q], u);
        pick<M, N>(x, pb.b[q], v);
        const float c0 = pb.coef[q][2 * seg], c1 = pb.coef[q][2 * seg + 1];
#pragma unroll
        for (int j = 0; j < N; ++j) o[j] = c0 * u[j] + c1 * v[j];
        st<ODT, N>(pb.out[q], i, o);
    }
}

template <int IDT, int ODT, int M, bool TILES>
__global__ __launch_bounds__(kBlock) void slerp_blend_mm_kernel(Members mem, PopBlend pb, const uint64_t* chunks,
                                                                int64_t nchunks) {
    for_blend_ranges<TILES>(chunks, nchunks, [&](uint64_t start, uint64_t end, uint64_t seg) {
        uint32_t need = 0;                   // children whose output this segment still needs
        for (int q = 0; q < pb.n; ++q)
            if (!pb.redo[q] || pb.redo[q][seg]) need |= 1u << q;
        if (!need) return;                   // every child keeps its speculative lerp output
        for_range_elems(start, end, [&](auto tagN, uint64_t i) {
            blend_mm_elems<IDT, ODT, M, decltype(tagN)::value>(mem, pb, i, seg, need);
        });
    });
}

// host: launch slerp_blend_mm_kernel over D compact parents. Grid-stride over chunks for both the
// Gram form's blends and the speculative redo: one tile per workgroup measured 11.46-11.51 ms
// against 10.83 ms for a 1.3B x 8 generation (the member-major body holds D parent tiles in
// registers; profiles/r02_slerp_pop_grid.json).
inline int launch_blend_mm(const Members& mem, int D, const PopBlend& pb, int in_dt, int out_dt,
                           const uint64_t* chunk_desc, int64_t nchunks, hipStream_t s) {
    const unsigned g = slerp_spec_grid(nchunks);
#define EDT_BMM(M)                                                                                            \
    case M:                                                                                                   \
        if (in_dt == EDT_F32 && out_dt == EDT_F32)                                                            \
            slerp_blend_mm_kernel<EDT_F32, EDT_F32, M, false><<<g, kBlock, 0, s>>>(mem, pb, chunk_desc, nchunks);   \
        else if (in_dt == EDT_F32)                                                                            \
            slerp_blend_mm_kernel<EDT_F32, EDT_BF16, M, false><<<g, kBlock, 0, s>>>(mem, pb, chunk_desc, nchunks);  \
        else if (out_dt == EDT_F32)                                                                           \
            slerp_blend_mm_kernel<EDT_BF16, EDT_F32, M, false><<<g, kBlock, 0, s>>>(mem, pb, chunk_desc, nchunks);  \
        else                                                                                                  \
            slerp_blend_mm_kernel<EDT_BF16, EDT_BF16, M, false><<<g, kBlock, 0, s>>>(mem, pb, chunk_desc, nchunks); \
        break;
    switch (D) {
        EDT_BMM(1) EDT_BMM(2) EDT_BMM(3) EDT_BMM(4) EDT_BMM(5) EDT_BMM(6) EDT_BMM(7) EDT_BMM(8)
        default: return fail(EDT_ERR_ARG, "member-major blend over %d parents", D);
    }
#undef EDT_BMM
    return check_launch("slerp_blend_mm_kernel");
}

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
    const unsigned g = slerp_tile_grid(nchunks);
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



int edt_slerp_stats(const void* v0, const void* v1, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                    double* partial, void* stream) {
    g_err[0] = 0;
    if (nchunks < 0) return fail(EDT_ERR_ARG, "negative chunk count");
    if (nchunks == 0) return EDT_OK;
    if (!v0 || !v1) return fail(EDT_ERR_ARG, "null buffer");
    if (!aligned16(v0) || !aligned16(v1)) return fail(EDT_ERR_ARG, "slerp inputs must be 16-byte aligned");
    return slerp_stats_impl(v0, v1, in_dt, chunk_desc, nchunks, partial, nullptr, stream);
}

int edt_slerp_coef(const double* partial, const int32_t* seg_first_chunk, int nseg, const double* t,
                   double dot_threshold, double eps, float* coef, float* dot_out, void* stream) {
    g_err[0] = 0;
    if (nseg < 0) return fail(EDT_ERR_ARG, "negative segment count");
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
    if (nchunks < 0) return fail(EDT_ERR_ARG, "negative chunk count");
    if (nchunks == 0) return EDT_OK;
    if (!v0 || !v1 || !out) return fail(EDT_ERR_ARG, "null buffer");
    if (!aligned16(v0) || !aligned16(v1) || !aligned16(out))
        return fail(EDT_ERR_ARG, "slerp buffers must be 16-byte aligned");
    return slerp_blend_impl(v0, v1, in_dt, out, out_dt, chunk_desc, nchunks, coef, nullptr, stream);
}

int edt_slerp_merge(const void* v0, const void* v1, int in_dt, void* out, int out_dt, const uint64_t* chunk_desc,
                    int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t, double dot_threshold,
                    double eps, double* partial, float* coef, float* dot_out, void* stream) {
    // every argument of the three passes checked before the first launch: a rejected call does nothing
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nchunks < 0 || nseg < 0) return fail(EDT_ERR_ARG, "negative count");
    if (nchunks > 0 && (!v0 || !v1 || !out || !chunk_desc || !partial || !coef))
        return fail(EDT_ERR_ARG, "null buffer");
    if (nseg > 0 && (!seg_first_chunk || !t || !partial || !coef)) return fail(EDT_ERR_ARG, "null buffer");
    if (nchunks > 0 && (!aligned16(v0) || !aligned16(v1) || !aligned16(out)))
        return fail(EDT_ERR_ARG, "slerp buffers must be 16-byte aligned");
    int rc = edt_slerp_stats(v0, v1, in_dt, chunk_desc, nchunks, partial, stream);
    if (rc) return rc;
    rc = edt_slerp_coef(partial, seg_first_chunk, nseg, t, dot_threshold, eps, coef, dot_out, stream);
    if (rc) return rc;
    return edt_slerp_blend(v0, v1, in_dt, out, out_dt, chunk_desc, nchunks, coef, stream);
}

uint64_t edt_slerp_population_speculative_doubles(int npairs, int64_t nchunks) {
    if (npairs < 0 || nchunks < 0) return 0;
    const uint64_t per = 3ull * (uint64_t)npairs > 36ull ? 3ull * (uint64_t)npairs : 36ull;   // 36: 8 x 9 / 2
    return (uint64_t)nchunks * per;
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
    // the Gram pass and the blends run over the distinct parents only (compact indices)
    int compact[kGramMaxMembers];
    int D = 0;
    for (int m = 0; m < nmembers; ++m) compact[m] = -1;
    memset(&mem, 0, sizeof(mem));
    for (int q = 0; q < npairs; ++q)
        for (int e = 0; e < 2; ++e) {
            const int m = pairs[2 * q + e];
            if (compact[m] < 0) {
                compact[m] = D;
                mem.p[D++] = members[m];
            }
        }
    // the Gram pass (M(M+1)/2 fp64 sums per thread, low occupancy) stays grid-stride unless
    // EDT_SLERP_GRAM_GRID: 1.3B x 8 generation 10.83 ms grid-stride vs 11.46 ms one per chunk
    const unsigned g = EDT_SLERP_GRAM_GRID ? slerp_grid(nchunks) : slerp_spec_grid(nchunks);
#define EDT_GRAM(M)                                                                                  \
    case M:                                                                                          \
        if (in_dt == EDT_F32) slerp_gram_kernel<EDT_F32, M><<<g, kBlock, 0, s>>>(mem, chunk_desc, nchunks, gram); \
        else slerp_gram_kernel<EDT_BF16, M><<<g, kBlock, 0, s>>>(mem, chunk_desc, nchunks, gram);              \
        break;
    switch (D) {
        EDT_GRAM(1) EDT_GRAM(2) EDT_GRAM(3) EDT_GRAM(4) EDT_GRAM(5) EDT_GRAM(6) EDT_GRAM(7) EDT_GRAM(8)
    }
#undef EDT_GRAM
    int rc = check_launch("slerp_gram_kernel");
    if (rc) return rc;
    const int M = D, NT = M * (M + 1) / 2;
    const unsigned gc = coef_grid(nseg);
    for (int q = 0; q < npairs; ++q) {
        const int i = compact[pairs[2 * q]], j = compact[pairs[2 * q + 1]];
        const int lo = i < j ? i : j, hi = i < j ? j : i;
        slerp_gram_coef_kernel<<<gc, kBlock, 0, s>>>(gram, NT, tri_index(i, i, M), tri_index(j, j, M),
                                                     tri_index(lo, hi, M), seg_first_chunk, nseg, t,
                                                     (float)dot_threshold, (float)eps, coef + 2 * (size_t)nseg * q,
                                                     dot_out ? dot_out + (size_t)nseg * q : nullptr);
        rc = check_launch("slerp_gram_coef_kernel");
        if (rc) return rc;
    }
    // the blends: member-major when the children fit one launch, else co-located groups of <= 16
    if (npairs <= kBlendMaxChildren) {
        PopBlend pb;
        memset(&pb, 0, sizeof(pb));
        pb.n = npairs;
        for (int q = 0; q < npairs; ++q) {
            pb.out[q] = outs[q];
            pb.coef[q] = coef + 2 * (size_t)nseg * q;
            pb.a[q] = compact[pairs[2 * q]];
            pb.b[q] = compact[pairs[2 * q + 1]];
        }
        return launch_blend_mm(mem, D, pb, in_dt, out_dt, chunk_desc, nchunks, s);
    }
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

// ---- the three passes of edt_slerp_population as separate entries (the link-balanced sharded
// population, distributed.ShardedSlerpPopulation: Gram sums over a rank's chunk range, then the
// coefficients from the all-gathered table, then the blends of the rank's range) ----

int edt_slerp_gram(const void* const* members, int nmembers, int in_dt, const uint64_t* chunk_desc,
                   int64_t nchunks, double* gram, void* stream) {
    g_err[0] = 0;
    if (in_dt & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nmembers < 1 || nmembers > kGramMaxMembers)
        return fail(EDT_ERR_ARG, "member count %d out of range [1, %d]", nmembers, kGramMaxMembers);
    if (nchunks < 0) return fail(EDT_ERR_ARG, "negative chunk count");
    if (nchunks == 0) return EDT_OK;
    if (!members || !chunk_desc || !gram) return fail(EDT_ERR_ARG, "null buffer");
    Members mem;
    memset(&mem, 0, sizeof(mem));
    for (int m = 0; m < nmembers; ++m) {
        if (!members[m] || !aligned16(members[m])) return fail(EDT_ERR_ARG, "member %d is null or not 16-byte aligned", m);
        mem.p[m] = members[m];
    }
    hipStream_t s = (hipStream_t)stream;
    const unsigned g = EDT_SLERP_GRAM_GRID ? slerp_grid(nchunks) : slerp_spec_grid(nchunks);
#define EDT_GRAM1(M)                                                                                 \
    case M:                                                                                          \
        if (in_dt == EDT_F32) slerp_gram_kernel<EDT_F32, M><<<g, kBlock, 0, s>>>(mem, chunk_desc, nchunks, gram); \
        else slerp_gram_kernel<EDT_BF16, M><<<g, kBlock, 0, s>>>(mem, chunk_desc, nchunks, gram);              \
        break;
    switch (nmembers) {
        EDT_GRAM1(1) EDT_GRAM1(2) EDT_GRAM1(3) EDT_GRAM1(4) EDT_GRAM1(5) EDT_GRAM1(6) EDT_GRAM1(7) EDT_GRAM1(8)
    }
#undef EDT_GRAM1
    return check_launch("slerp_gram_kernel");
}

int edt_slerp_gram_coef(const double* gram, int nmembers, const int32_t* pairs, int npairs,
                        const int32_t* seg_first_chunk, int nseg, const double* t, double dot_threshold,
                        double eps, float* coef, float* dot_out, void* stream) {
    g_err[0] = 0;
    if (nmembers < 1 || nmembers > kGramMaxMembers)
        return fail(EDT_ERR_ARG, "member count %d out of range [1, %d]", nmembers, kGramMaxMembers);
    if (npairs < 0 || nseg < 0) return fail(EDT_ERR_ARG, "negative count");
    if (npairs == 0 || nseg == 0) return EDT_OK;
    if (!gram || !pairs || !seg_first_chunk || !t || !coef) return fail(EDT_ERR_ARG, "null buffer");
    const int M = nmembers, NT = M * (M + 1) / 2;
    hipStream_t s = (hipStream_t)stream;
    for (int q = 0; q < npairs; ++q) {
        const int i = pairs[2 * q], j = pairs[2 * q + 1];
        if (i < 0 || j < 0 || i >= M || j >= M) return fail(EDT_ERR_ARG, "pair %d: member out of range", q);
        const int lo = i < j ? i : j, hi = i < j ? j : i;
        slerp_gram_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(gram, NT, tri_index(i, i, M), tri_index(j, j, M),
                                                                  tri_index(lo, hi, M), seg_first_chunk, nseg, t,
                                                                  (float)dot_threshold, (float)eps,
                                                                  coef + 2 * (size_t)nseg * q,
                                                                  dot_out ? dot_out + (size_t)nseg * q : nullptr);
        int rc = check_launch("slerp_gram_coef_kernel");
        if (rc) return rc;
    }
    return EDT_OK;
}

int edt_slerp_blend_children(const void* const* members, int nmembers, int in_dt, const int32_t* pairs,
                             int npairs, void* const* outs, int out_dt, const uint64_t* chunk_desc,
                             int64_t nchunks, const float* coef, int nseg, void* stream) {
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nmembers < 1 || nmembers > kGramMaxMembers)
        return fail(EDT_ERR_ARG, "member count %d out of range [1, %d]", nmembers, kGramMaxMembers);
    if (npairs < 0 || npairs > kBlendMaxChildren)
        return fail(EDT_ERR_ARG, "child count %d out of range [0, %d]", npairs, kBlendMaxChildren);
    if (nchunks < 0 || nseg < 0) return fail(EDT_ERR_ARG, "negative count");
    if (npairs == 0 || nchunks == 0) return EDT_OK;
    if (!members || !pairs || !outs || !chunk_desc || !coef) return fail(EDT_ERR_ARG, "null buffer");
    Members mem;
    memset(&mem, 0, sizeof(mem));
    for (int m = 0; m < nmembers; ++m) {
        if (!members[m] || !aligned16(members[m])) return fail(EDT_ERR_ARG, "member %d is null or not 16-byte aligned", m);
        mem.p[m] = members[m];
    }
    PopBlend pb;
    memset(&pb, 0, sizeof(pb));
    pb.n = npairs;
    for (int q = 0; q < npairs; ++q) {
        const int i = pairs[2 * q], j = pairs[2 * q + 1];
        if (i < 0 || j < 0 || i >= nmembers || j >= nmembers) return fail(EDT_ERR_ARG, "pair %d: member out of range", q);
        if (!outs[q] || !aligned16(outs[q])) return fail(EDT_ERR_ARG, "output %d is null or not 16-byte aligned", q);
        for (int m = 0; m < nmembers; ++m)
            if (outs[q] == members[m]) return fail(EDT_ERR_ARG, "output %d aliases member %d", q, m);
        pb.out[q] = outs[q];
        pb.coef[q] = coef + 2 * (size_t)nseg * q;
        pb.a[q] = i;
        pb.b[q] = j;
    }
    return launch_blend_mm(mem, nmembers, pb, in_dt, out_dt, chunk_desc, nchunks, (hipStream_t)stream);
}

int edt_slerp_merge_speculative(const void* v0, const void* v1, int in_dt, void* out, int out_dt,
                                const uint64_t* chunk_desc, int64_t nchunks, const int32_t* seg_first_chunk,
                                int nseg, const double* t, double dot_threshold, double eps, double* partial,
                                float* coef, float* dot_out, int32_t* redo, uint64_t n, void* stream) {
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nseg < 0 || nchunks < 0) return fail(EDT_ERR_ARG, "negative count");
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
    const unsigned g = EDT_SLERP_SPEC_CONTIG > 0 ? (unsigned)((nchunks + EDT_SLERP_SPEC_CONTIG - 1) / EDT_SLERP_SPEC_CONTIG)
                                                 : slerp_spec_grid(nchunks);
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
    // the redo blends: grid-stride over chunks (most segments are skipped)
    constexpr bool kNtB = EDT_NT_SLERP != 0;
    if (in_dt == EDT_F32 && out_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_F32, false, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo);
    else if (in_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_BF16, false, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo);
    else if (out_dt == EDT_F32)
        slerp_blend_kernel<EDT_BF16, EDT_F32, kNtB, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo);
    else
        slerp_blend_kernel<EDT_BF16, EDT_BF16, kNtB, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo);
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
    // member-major first pass when the distinct parents fit one Gram tile (<= 8) and the children
    // one launch (<= 16): every distinct parent read once per chunk, whatever the caches do
    int compact[256];
    int D = 0;
    Members mem;
    memset(&mem, 0, sizeof(mem));
    bool fused = npairs <= kBlendMaxChildren && nmembers <= 256;
    if (fused) {
        for (int m = 0; m < nmembers; ++m) compact[m] = -1;
        for (int q = 0; q < npairs && fused; ++q)
            for (int e = 0; e < 2; ++e) {
                const int m = pairs[2 * q + e];
                if (compact[m] < 0) {
                    if (D == kGramMaxMembers) { fused = false; break; }
                    compact[m] = D;
                    mem.p[D++] = members[m];
                }
            }
    }
    if (fused) {
        PopLerp po;
        memset(&po, 0, sizeof(po));
        po.n = npairs;
        for (int q = 0; q < npairs; ++q) {
            po.out[q] = outs[q];
            po.a[q] = compact[pairs[2 * q]];
            po.b[q] = compact[pairs[2 * q + 1]];
        }
        const unsigned g = slerp_spec_grid(nchunks);
#define EDT_GL(M)                                                                                             \
    case M:                                                                                                   \
        if (in_dt == EDT_F32 && out_dt == EDT_F32)                                                            \
            slerp_gram_lerp_kernel<EDT_F32, EDT_F32, M><<<g, kBlock, 0, s>>>(mem, po, chunk_desc, nchunks, t, partial); \
        else if (in_dt == EDT_F32)                                                                            \
            slerp_gram_lerp_kernel<EDT_F32, EDT_BF16, M><<<g, kBlock, 0, s>>>(mem, po, chunk_desc, nchunks, t, partial); \
        else if (out_dt == EDT_F32)                                                                           \
            slerp_gram_lerp_kernel<EDT_BF16, EDT_F32, M><<<g, kBlock, 0, s>>>(mem, po, chunk_desc, nchunks, t, partial); \
        else                                                                                                  \
            slerp_gram_lerp_kernel<EDT_BF16, EDT_BF16, M><<<g, kBlock, 0, s>>>(mem, po, chunk_desc, nchunks, t, partial); \
        break;
        switch (D) {
            EDT_GL(1) EDT_GL(2) EDT_GL(3) EDT_GL(4) EDT_GL(5) EDT_GL(6) EDT_GL(7) EDT_GL(8)
        }
#undef EDT_GL
        int rc = check_launch("slerp_gram_lerp_kernel");
        if (rc) return rc;
        const int NT = D * (D + 1) / 2;
        for (int q = 0; q < npairs; ++q) {
            const int i = compact[pairs[2 * q]], j = compact[pairs[2 * q + 1]];
            const int lo = i < j ? i : j, hi = i < j ? j : i;
            slerp_gram_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(
                partial, NT, tri_index(i, i, D), tri_index(j, j, D), tri_index(lo, hi, D), seg_first_chunk, nseg, t,
                (float)dot_threshold, (float)eps, coef + 2 * (size_t)nseg * q,
                dot_out ? dot_out + (size_t)nseg * q : nullptr, redo + (size_t)nseg * q);
            rc = check_launch("slerp_gram_coef_kernel");
            if (rc) return rc;
        }
    }
    if (fused) {                             // the redo blends, member-major over the same D parents
        PopBlend pb;
        memset(&pb, 0, sizeof(pb));
        pb.n = npairs;
        for (int q = 0; q < npairs; ++q) {
            pb.out[q] = outs[q];
            pb.coef[q] = coef + 2 * (size_t)nseg * q;
            pb.redo[q] = redo + (size_t)nseg * q;
            pb.a[q] = compact[pairs[2 * q]];
            pb.b[q] = compact[pairs[2 * q + 1]];
        }
        return launch_blend_mm(mem, D, pb, in_dt, out_dt, chunk_desc, nchunks, s);
    }
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
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nseg < 0 || nchunks < 0) return fail(EDT_ERR_ARG, "negative count (segments %d, chunks %lld)", nseg, (long long)nchunks);
    if (nseg == 0 || nchunks == 0) return EDT_OK;
    if (!v0_t || !v1_t || !out_t) return fail(EDT_ERR_ARG, "null tensor table");
    if (!chunk_desc || !seg_first_chunk || !t || !partial || !coef) return fail(EDT_ERR_ARG, "null buffer");
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
