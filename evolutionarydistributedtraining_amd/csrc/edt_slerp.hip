// edt_slerp.hip — the SLERP crossover (EDT_RL/crossover.py:11-135,
// EDT_EVOMERGE/train/crossover.py:14-146): chunk sums, coefficients, blends, the speculative
// and population forms, with their C ABI entries (include/edt_sync.h).
#include "edt_common.h"

#include <algorithm>
#include <string>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------
// SLERP. chunk_desc[3c .. 3c+2] = {start, length, segment}; chunks never cross a segment.

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// ---- the tile butterfly without LDS ------------------------------------------------------------
// wave_sum's descending xor butterfly (x_l += x_{l ^ o}, o = 32 .. 1) bit for bit, on the VALU:
// __shfl_xor is a ds_bpermute through the LDS crossbar (two per double and level), which on the
// Gram pass (36 sums per tile) cost more than streaming its members. Levels 32 / 16 use gfx950's
// v_permlane32_swap / v_permlane16_swap, levels 8 .. 1 DPP moves (row_ror:8; half-mirror after a
// quad reverse = xor 4; quad_perm xor 2 / xor 1). fp64 addition is commutative, so a lane forming
// partner + self instead of self + partner gets the same bits.
//
// Several values at once are TRANSPOSED at levels 32 and 16 (the swap exchanges half the values):
// for values A = v[k], B = v[h + k] a lane whose level bit is clear keeps A's pair sum, the other
// lane B's — the same pair sums the per-value butterfly forms, one swap + one add per pair instead
// of per value. After both levels, row r = lane / 16 holds N2 of the N values (index: red_index),
// and the remaining levels run on those alone.
__device__ __forceinline__ double join_d(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

template <int LVL>
__device__ __forceinline__ double swap_sum(double x, double y) {
    const uint64_t bx = (uint64_t)__double_as_longlong(x), by = (uint64_t)__double_as_longlong(y);
    if constexpr (LVL == 32) {
        const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)bx, (uint32_t)by, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(bx >> 32), (uint32_t)(by >> 32), false, false);
        return join_d(lo[0], hi[0]) + join_d(lo[1], hi[1]);
    } else {
        static_assert(LVL == 16, "swap levels are 32 and 16");
        const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)bx, (uint32_t)by, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(bx >> 32), (uint32_t)(by >> 32), false, false);
        return join_d(lo[0], hi[0]) + join_d(lo[1], hi[1]);
    }
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return join_d((uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xf, 0xf, false));
}

// levels 8, 4, 2, 1 of the butterfly (within each row of 16 lanes)
__device__ __forceinline__ double row_butterfly(double x) {
    x += dpp_d<0x128>(x);                 // row_ror:8       = lane ^ 8
    x += dpp_d<0x141>(dpp_d<0x1B>(x));    // half-mirror (lane ^ 7) of quad_perm [3,2,1,0] (lane ^ 3)
    x += dpp_d<0x4E>(x);                  // quad_perm [2,3,0,1] = lane ^ 2
    x += dpp_d<0xB1>(x);                  // quad_perm [1,0,3,2] = lane ^ 1
    return x;
}

template <int N>
struct Red {
    static constexpr int H1 = N / 2, N1 = H1 + (N & 1);       // after level 32
    static constexpr int H2 = N1 / 2, N2 = H2 + (N1 & 1);     // after level 16: values per row
};

// N tile sums at once: r[s] on lane l = the butterfly total of value red_index<N>(s, l)
template <int N>
__device__ __forceinline__ void tile_reduce(const double (&v)[N], double (&r)[Red<N>::N2]) {
    constexpr int H1 = Red<N>::H1, N1 = Red<N>::N1, H2 = Red<N>::H2, N2 = Red<N>::N2;
    double r1[N1];
#pragma unroll
    for (int k = 0; k < H1; ++k) r1[k] = swap_sum<32>(v[k], v[H1 + k]);
    if constexpr (N & 1) r1[H1] = swap_sum<32>(v[N - 1], v[N - 1]);
#pragma unroll
    for (int k = 0; k < H2; ++k) r[k] = swap_sum<16>(r1[k], r1[H2 + k]);
    if constexpr (N1 & 1) r[H2] = swap_sum<16>(r1[N1 - 1], r1[N1 - 1]);
#pragma unroll
    for (int s = 0; s < N2; ++s) r[s] = row_butterfly(r[s]);
}

// tile_reduce's swap levels (32 and 16) alone: r[s] on lane l = the level-16 partial of value
// red_index<N>(s, l), i.e. of the 16-lane row l / 16, position l % 16 in it.
template <int N>
__device__ __forceinline__ void tile_swap_levels(const double (&v)[N], double (&r)[Red<N>::N2]) {
    constexpr int H1 = Red<N>::H1, N1 = Red<N>::N1, H2 = Red<N>::H2;
    double r1[N1];
#pragma unroll
    for (int k = 0; k < H1; ++k) r1[k] = swap_sum<32>(v[k], v[H1 + k]);
    if constexpr (N & 1) r1[H1] = swap_sum<32>(v[N - 1], v[N - 1]);
#pragma unroll
    for (int k = 0; k < H2; ++k) r[k] = swap_sum<16>(r1[k], r1[H2 + k]);
    if constexpr (N1 & 1) r[H2] = swap_sum<16>(r1[N1 - 1], r1[N1 - 1]);
}

// row_butterfly's total (levels 8, 4, 2, 1 of the xor butterfly) of one row's 16 level-16
// partials p[i] (i = position in the row), formed serially by one lane in the butterfly's own
// pairing — lane 0's sums: (p0 + p8), then + (p4 + p12), ... — so bit-identical to it (fp64
// addition is commutative: a lane forming partner + self gets the same bits).
__device__ __forceinline__ double row_tree16(const double (&p)[16]) {
    double q8[8], q4[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) q8[i] = p[i] + p[i + 8];
#pragma unroll
    for (int i = 0; i < 4; ++i) q4[i] = q8[i] + q8[i + 4];
    return (q4[0] + q4[2]) + (q4[1] + q4[3]);
}

// Which value slot s of lane `lane` holds after tile_reduce<N>, and whether this lane is the one
// writer of it (a leftover value at an odd level is held by both halves).
template <int N>
__device__ __forceinline__ int red_index(int s, int lane, bool& owner) {
    constexpr int H1 = Red<N>::H1, N1 = Red<N>::N1, H2 = Red<N>::H2;
    const bool b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
    owner = true;
    int s1;
    if (s < H2) {
        s1 = b4 ? H2 + s : s;
    } else {
        s1 = N1 - 1;
        owner = !b4;
    }
    if (s1 < H1) return b5 ? H1 + s1 : s1;
    owner = owner && !b5;
    return N - 1;
}

// Lane l writes, when it owns one, the value slot (l % 16) holds: store(index, value). One
// predicated store per slot (a register chosen by lane would be an indexed private array: scratch).
template <int N, typename Store>
__device__ __forceinline__ void red_store(const double (&r)[Red<N>::N2], Store&& store) {
    const int lane = threadIdx.x & 63, s = lane & 15;
#pragma unroll
    for (int q = 0; q < Red<N>::N2; ++q) {
        if (s == q) {
            bool owner;
            const int idx = red_index<N>(q, lane, owner);
            if (owner) store(idx, r[q]);
        }
    }
}

// ---- the chunk sums' canonical order (every form: pair, speculative, Gram, sharded) --------------
// A chunk [start, start + len) (len <= 64 Ki) is cut into kTileSlots = 128 tiles of its 16-B-aligned
// body [a, b): tile j holds, on lane l, the 8 elements at a + 512 j + 8 l (when below b); tile 0's
// lanes also take the < 16 head / tail elements (lane l the l-th of them) after their vector. Per
// lane the products are accumulated in element order by fp64 FMAs; the wave's xor butterfly
// (wave_sum's order, formed on the VALU by tile_reduce) gives the TILE SUM; the chunk's sum is the perfect binary tree over its 128 tile sums
// in order, adjacent pairs first ((t0 + t1) + (t2 + t3)) + ..., empty tiles 0.0. Every kernel forms
// complete subtrees — one tile per wave (the speculative passes: the workgroup's four combined
// through LDS into a level-2 row, kSpecWgRows; else a level-0 row), kStatsTPW tiles per wave combined in
// registers (the read-only stats pass), sixteen per workgroup combined in LDS (level 4) — and
// writes them as rows;
// tree_reduce_kernel finishes each chunk's tree from its rows. So every form's per-chunk sums are
// bit-identical whatever the work split (the read-only pass needs no workgroup barrier; the
// speculative passes take one: a quarter of the row bytes measured faster, EDT_SLERP_SPEC_WG_ROWS).
//
// Why this shape (profiles/r03_spec_probe_{a,b,c}.json, scripts/spec_probe.hip on the 7B body): the
// speculative pass is lerp's stream (2 reads + 1 write per element) plus the sums; one tile per wave
// in address order — lerp's own grid — costs little for the fp64 math and butterflies (6.91-7.02 ms
// vs lerp 6.80-6.92 with the row store removed); what does cost is the rows' second write stream:
// 24-B rows scattered over the table +11 %, rows padded to whole lines +3-7 %, rows placed XCD-major
// (each XCD's workgroups write one contiguous stretch, so its L2 writes back whole lines) +1.3 %.
// The previous form (one workgroup per 64 Ki chunk, grid-stride, an LDS block reduction per chunk)
// ran 7.1-8.3 ms depending on the allocation.
constexpr int kTileElems = 64 * kVec;                         // 512
constexpr int kTileSlots = 128;                               // tiles per chunk: chunks <= 64 Ki
constexpr uint32_t kMaxChunkElems = (uint32_t)kTileSlots * kTileElems;
constexpr int kWavesPerBlock = kBlock / 64;
// the row levels the kernels write: pair passes one tile per wave (level 0; the read-only stats
// pass kStatsTPW per wave, level log2 kStatsTPW), the Gram passes sixteen per workgroup (level 4)
constexpr int kPairRows = kTileSlots;                         // rows per chunk, level 0
constexpr int kGramRows = kTileSlots / 16;                    // rows per chunk, level 4
constexpr int kStatsTPW = EDT_SLERP_STATS_TPW;                // tiles per wave of the read-only pass
constexpr bool kSpecWgRows = EDT_SLERP_SPEC_WG_ROWS != 0;     // speculative pass: one row per workgroup

// One-pass grids of `units` workgroups in address order (a unit = a fixed set of a chunk's tiles);
// past the dispatch cap (a multiple of 8, so blockIdx % 8 stays the unit's XCD) they stride.
constexpr uint64_t kUnitGridCap = kGridBlockCap / 8 * 8;
inline unsigned unit_grid(uint64_t units) {
    return (unsigned)(units < kUnitGridCap ? (units ? units : 1) : kUnitGridCap);
}

// Where unit u's rows go: XCD-major — the units one XCD runs (u % 8 equal) are contiguous, so each
// XCD's L2 fills whole lines of the row table before writing them back.
__host__ __device__ __forceinline__ uint64_t unit_slot(uint64_t u, uint64_t units) {
    const uint64_t per = (units + 7) / 8;
    return (u % 8) * per + u / 8;
}

// The lane's share of tile j of chunk [start, start + len): vec(i) for its 8-element vector (when
// inside the aligned body), then (tile 0) elem(i) for its head / tail element.
template <typename Vec, typename Elem>
__device__ __forceinline__ void for_tile(uint64_t start, uint64_t len, int j, Vec&& vec, Elem&& elem) {
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t end = start + len;
    const uint64_t a = (start + kVec - 1) / kVec * kVec;      // aligned body [a, b)
    const uint64_t b = end / kVec * kVec;
    const uint64_t i = a + (uint64_t)j * kTileElems + lane * kVec;
    if (a < b && i < b) vec(i);
    if (j == 0) {
        const uint64_t h_end = a < end ? a : end;
        const uint64_t t_beg = b > a ? b : h_end;
        const uint64_t nh = h_end - start, nt = end - t_beg;
        if (lane < nh + nt) elem(lane < nh ? start + lane : t_beg + (lane - nh));
    }
}

// Per chunk, one wave: the chunk's W sums from its `nrows` rows (level log2(128 / nrows)), as the
// perfect tree's upper levels — each lane combines its consecutive rows, then the ascending xor
// butterfly (1, 2, 4, ...) pairs adjacent subtrees level by level. Rows of chunk c: unit
// u = c * upc + r / rpu at row table slot unit_slot(u, nchunks * upc) * rpu + r % rpu.
__global__ __launch_bounds__(kBlock) void tree_reduce_kernel(const double* __restrict__ rows, int W, int nrows,
                                                             int upc, int rpu, int64_t nchunks,
                                                             double* __restrict__ out) {
    const uint64_t c = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= (uint64_t)nchunks) return;
    const uint64_t units = (uint64_t)nchunks * (uint64_t)upc;
    const int per_lane = nrows > 64 ? nrows / 64 : 1;
    const int lanes = nrows > 64 ? 64 : nrows;
    for (int q = 0; q < W; ++q) {
        double x = 0.0;
        if (lane < lanes) {
            for (int k = 0; k < per_lane; ++k) {              // per_lane is 1 or 2: a pair's sum
                const int r = lane * per_lane + k;
                const uint64_t u = c * (uint64_t)upc + (uint64_t)(r / rpu);
                const double v = rows[(unit_slot(u, units) * (uint64_t)rpu + (uint64_t)(r % rpu)) * (uint64_t)W + q];
                x = k == 0 ? v : x + v;
            }
        }
        for (int o = 1; o < lanes; o <<= 1) x += __shfl_xor(x, o, 64);
        if (lane == 0) out[c * (uint64_t)W + q] = x;
    }
}

inline int launch_tree_reduce(const double* rows, int W, int nrows, int upc, int rpu, int64_t nchunks, double* out,
                              hipStream_t s) {
    if (nchunks <= 0) return EDT_OK;
    const uint64_t g = ((uint64_t)nchunks + kWavesPerBlock - 1) / kWavesPerBlock;
    if (g > kGridBlockCap) return fail(EDT_ERR_ARG, "too many chunks for one launch");
    tree_reduce_kernel<<<(unsigned)g, kBlock, 0, s>>>(rows, W, nrows, upc, rpu, nchunks, out);
    return check_launch("tree_reduce_kernel");
}

// 8 consecutive elements held as loaded (bf16: one 16-B word, unpacked per element on use), so a
// wave keeps several vectors in flight on few registers.
template <int IDT>
struct Raw8;
template <>
struct Raw8<EDT_BF16> {
    u32x4 w;
    __device__ __forceinline__ float operator[](int j) const {
        const uint32_t x = (j >> 1) == 0 ? w.x : (j >> 1) == 1 ? w.y : (j >> 1) == 2 ? w.z : w.w;
        return (j & 1) ? bf_hi(x) : bf_lo(x);
    }
};
template <>
struct Raw8<EDT_F32> {
    f32x4 lo, hi;
    __device__ __forceinline__ float operator[](int j) const {
        const f32x4& v = j < 4 ? lo : hi;
        return (j & 3) == 0 ? v.x : (j & 3) == 1 ? v.y : (j & 3) == 2 ? v.z : v.w;
    }
};

struct Raw1 {                                        // one element, the same indexing
    float v[1];
    __device__ __forceinline__ float operator[](int) const { return v[0]; }
};

template <int IDT, bool NT>
__device__ __forceinline__ Raw8<IDT> ld_raw(const void* p, uint64_t i) {
    Raw8<IDT> r;
    if constexpr (IDT == EDT_BF16) {
        r.w = vload<u32x4, NT>(reinterpret_cast<const u32x4*>(static_cast<const uint16_t*>(p) + i));
    } else {
        const float* q = static_cast<const float*>(p) + i;
        r.lo = vload<f32x4, NT>(reinterpret_cast<const f32x4*>(q));
        r.hi = vload<f32x4, NT>(reinterpret_cast<const f32x4*>(q + 4));
    }
    return r;
}

// The fp64 FMAs of a pair's sums {v0.v0, v1.v1, v0.v1} over N elements (canonical per-lane order).
template <int N, typename X, typename Y>
__device__ __forceinline__ void pair_fma(const X& x, const Y& y, double& s00, double& s11, double& s01) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double dx = x[j], dy = y[j];
        s00 = __builtin_fma(dx, dx, s00);
        s11 = __builtin_fma(dy, dy, s11);
        s01 = __builtin_fma(dx, dy, s01);
    }
}

// Tile 0's head / tail element of this lane, if any: elem(i).
template <typename Elem>
__device__ __forceinline__ void tile0_edge(uint64_t start, uint64_t len, Elem&& elem) {
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t end = start + len;
    const uint64_t a = (start + kVec - 1) / kVec * kVec;
    const uint64_t b = end / kVec * kVec;
    const uint64_t h_end = a < end ? a : end;
    const uint64_t t_beg = b > a ? b : h_end;
    const uint64_t nh = h_end - start, nt = end - t_beg;
    if (lane < nh + nt) elem(lane < nh ? start + lane : t_beg + (lane - nh));
}

// Tile j's pair sums, stored as the row {v0.v0, v1.v1, v0.v1} at `row` (level 0). EMIT = true also
// writes the lerp-branch output l0 v0 + l1 v1 of the tile (two rounded fp32 products, one rounded
// sum: lerp_elems' math) — the speculative forms.
template <int IDT, bool NT, bool EMIT, int ODT>
__device__ __forceinline__ void pair_tile(const void* v0, const void* v1, void* out, uint64_t start, uint64_t len,
                                          int j, float l0, float l1, double* row) {
    double s00 = 0.0, s11 = 0.0, s01 = 0.0;
    const uint64_t a = (start + kVec - 1) / kVec * kVec, b = (start + len) / kVec * kVec;
    const uint64_t i = a + (uint64_t)j * kTileElems + (uint64_t)(threadIdx.x & 63) * kVec;
    if (a < b && i < b) {
        const Raw8<IDT> x = ld_raw<IDT, NT>(v0, i), y = ld_raw<IDT, NT>(v1, i);
        pair_fma<kVec>(x, y, s00, s11, s01);
        if constexpr (EMIT) {
            float o[kVec];
#pragma unroll
            for (int e = 0; e < kVec; ++e) o[e] = l0 * x[e] + l1 * y[e];
            st<ODT, kVec, (EDT_NT_SLERP_STORES != 0)>(out, i, o);
        }
    }
    if (j == 0)
        tile0_edge(start, len, [&](uint64_t e) {
            float x[1], y[1];
            ld<IDT, 1>(v0, e, x);
            ld<IDT, 1>(v1, e, y);
            pair_fma<1>(x, y, s00, s11, s01);
            if constexpr (EMIT) {
                float o[1] = {l0 * x[0] + l1 * y[0]};
                st<ODT, 1>(out, e, o);
            }
        });
    const double v[3] = {s00, s11, s01};
    double r[Red<3>::N2];
    tile_reduce<3>(v, r);
    red_store<3>(r, [&](int q, double x) { row[q] = x; });
}

// Tiles T m .. T m + T - 1 of a chunk by one wave, read-only (the two-pass stats; T = 4, 8, 16):
// the T tiles' loads issued together, each tile's sums and butterfly as pair_tile's (the 3 T values
// transposed together: row r of the wave ends with tiles K r .. K r + K - 1, K = T / 4), then the
// tree over the T tile sums in registers — within a row, then rows 0 + 1 and 2 + 3 by the level-16
// swap, then the two halves by the level-32 swap — stored as one row of level log2 T.
// The lane's vectors of tiles T m .. T m + T - 1 (ZERO: out-of-range tiles set to 0, so a caller
// holding them across phases owns defined registers).
template <int IDT, bool NT, int T, bool ZERO = false>
__device__ __forceinline__ void tiles_load(const void* v0, const void* v1, uint64_t start, uint64_t len, int m,
                                           Raw8<IDT> (&x)[T], Raw8<IDT> (&y)[T]) {
    const uint64_t a = (start + kVec - 1) / kVec * kVec, b = (start + len) / kVec * kVec;
    const uint64_t i0 = a + (uint64_t)(T * m) * kTileElems + (uint64_t)(threadIdx.x & 63) * kVec;
#pragma unroll
    for (int k = 0; k < T; ++k) {
        const uint64_t i = i0 + (uint64_t)k * kTileElems;
        if (a < b && i < b) {
            x[k] = ld_raw<IDT, NT>(v0, i);
            y[k] = ld_raw<IDT, NT>(v1, i);
        } else if constexpr (ZERO) {
            x[k] = Raw8<IDT>{};
            y[k] = Raw8<IDT>{};
        }
    }
}

// The row of level log2 T from the loaded vectors (pair_tiles' arithmetic): store(q, value) is
// called by lanes 0 .. 2 for the sums {v0.v0, v1.v1, v0.v1}.
template <int IDT, int T, typename Store>
__device__ __forceinline__ void tiles_sums(const void* v0, const void* v1, uint64_t start, uint64_t len, int m,
                                           const Raw8<IDT> (&x)[T], const Raw8<IDT> (&y)[T], Store&& store) {
    static_assert(T == 4 || T == 8 || T == 16, "tiles per wave");
    constexpr int K = T / 4;
    const uint64_t a = (start + kVec - 1) / kVec * kVec, b = (start + len) / kVec * kVec;
    const uint64_t i0 = a + (uint64_t)(T * m) * kTileElems + (uint64_t)(threadIdx.x & 63) * kVec;
    double t[3 * T];                                 // tile-major: t[3 k + q]
#pragma unroll
    for (int k = 0; k < T; ++k) {
        double s00 = 0.0, s11 = 0.0, s01 = 0.0;
        if (a < b && i0 + (uint64_t)k * kTileElems < b) pair_fma<kVec>(x[k], y[k], s00, s11, s01);
        if (T * m + k == 0)
            tile0_edge(start, len, [&](uint64_t e) {
                float xe[1], ye[1];
                ld<IDT, 1>(v0, e, xe);
                ld<IDT, 1>(v1, e, ye);
                pair_fma<1>(xe, ye, s00, s11, s01);
            });
        t[3 * k] = s00;
        t[3 * k + 1] = s11;
        t[3 * k + 2] = s01;
    }
    static_assert(Red<3 * T>::N2 == 3 * K, "row layout");
    double r[3 * K];                                 // row r: tiles K r + j at r[3 j + q] (red_index)
    tile_reduce<3 * T>(t, r);
    auto total = [&](int q) {                        // q is a constant after inlining
        double v;
        if constexpr (K == 1) v = r[q];
        else if constexpr (K == 2) v = r[q] + r[3 + q];
        else v = (r[q] + r[3 + q]) + (r[6 + q] + r[9 + q]);
        const double p = swap_sum<16>(v, v);              // rows 0 / 2: the first / second quarter pairs
        return swap_sum<32>(p, p);                        // the two halves
    };
    const double s0 = total(0), s1 = total(1), s2 = total(2);
    const int lane = threadIdx.x & 63;
    const double x0 = lane == 0 ? s0 : lane == 1 ? s1 : s2;
    if (lane < 3) store(lane, x0);
}

template <int IDT, bool NT, int T>
__device__ __forceinline__ void pair_tiles(const void* v0, const void* v1, uint64_t start, uint64_t len, int m,
                                           double* row) {
    Raw8<IDT> x[T], y[T];
    tiles_load<IDT, NT, T>(v0, v1, start, len, m, x, y);
    tiles_sums<IDT, T>(v0, v1, start, len, m, x, y, [&](int q, double v) { row[q] = v; });
}

// The reference's branch and coefficients (EDT_RL/crossover.py:31-45) for an fp32 dot, in fp32 as
// numpy does it for float32 scalars (NEP 50: python floats enter as fp32).
__device__ __forceinline__ void coefficients_from_dot(float dot, double t, float thr, float& c0, float& c1) {
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

// The reference's scalar SLERP math (EDT_RL/crossover.py:24-45) from the three sums.
__device__ __forceinline__ void slerp_coefficients(double s00, double s11, double s01, double t, float thr,
                                                   float eps, float& c0, float& c1, float& dot) {
    const float n0 = (float)sqrt(s00), n1 = (float)sqrt(s11);      // np.linalg.norm (fp32)
    const double d0 = n0 > eps ? (double)n0 : 1.0;                  // normalize() divides only if > eps
    const double d1 = n1 > eps ? (double)n1 : 1.0;
    dot = (float)(s01 / (d0 * d1));
    coefficients_from_dot(dot, t, thr, c0, c1);
}

// The element ranges a blend workgroup owns, as body(start, end, segment): whole chunks,
// grid-stride (grid slerp_spec_grid) — the speculative redo blends and the member-major blends,
// where most segments may be skipped and a workgroup per tile would cost more to dispatch than it
// saves (7B lineage merge: 3.45 M empty workgroups = +1.1 ms). The full blends run on the unit
// grid of slerp_blend_tile_kernel.
template <typename F>
__device__ __forceinline__ void for_blend_ranges(const uint64_t* chunks, int64_t nchunks, F&& body) {
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x)
        body(chunks[3 * c], chunks[3 * c] + chunks[3 * c + 1], chunks[3 * c + 2]);
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

// The pair sums' rows, one workgroup per unit in address order (unit_slot: XCD-major rows).
// EMIT (the speculative first pass, edt_slerp_merge_speculative): unit = 4 tiles, one per wave
// (a level-2 row per workgroup, or level-0 rows per wave), lerp's own grid; the lerp-branch
// output (1-t) v0 + t v1 with the coefficients
// slerp_coefficients gives that branch is written in the same pass. Parents of one lineage
// (fine-tunes of a common base) mostly have |dot| > 0.9995, where this output is final; the other
// segments are blended again. Read-only (the two-pass stats): unit = 4 kStatsTPW tiles,
// kStatsTPW per wave (rows of level log2 kStatsTPW). seg_ptrs (tensor-list form, may be null): per segment {v0, v1, out} device
// pointers; chunk starts are then relative to their segment. Null: flat arenas.
template <int IDT, bool EMIT, int ODT>
__global__ __launch_bounds__(kBlock) void pair_sums_kernel(const void* v0, const void* v1, void* out,
                                                           const uint64_t* chunks, int64_t nchunks, double* rows,
                                                           const double* tvals, const uint64_t* seg_ptrs, uint64_t u0,
                                                           int32_t* zero_word) {
    constexpr bool NT = EDT_NT_SLERP != 0 && IDT == EDT_BF16;
    if (zero_word && u0 == 0 && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;   // the any-redo flag
    constexpr int upc = EMIT ? kTileSlots / 4 : kTileSlots / (4 * kStatsTPW);   // units per chunk
    const int wave = threadIdx.x >> 6;
    const uint64_t units = (uint64_t)nchunks * upc;
    {   // one unit per workgroup (no grid-stride loop: it costs registers, i.e. occupancy)
        const uint64_t u = u0 + blockIdx.x;
        if (u >= units) return;
        const uint64_t c = u / upc;
        const int g = (int)(u % upc);
        const uint64_t seg = chunks[3 * c + 2];
        const void* a = v0;
        const void* b = v1;
        void* o = out;
        if (seg_ptrs) {
            a = reinterpret_cast<const void*>(seg_ptrs[3 * seg]);
            b = reinterpret_cast<const void*>(seg_ptrs[3 * seg + 1]);
            o = reinterpret_cast<void*>(seg_ptrs[3 * seg + 2]);
        }
        double* row = rows + (unit_slot(u, units) * kWavesPerBlock + wave) * 3;
        if constexpr (EMIT && kSpecWgRows) {
            // one level-2 row per workgroup: the four waves' tile sums through LDS, combined as
            // the tree does ((t0 + t1) + (t2 + t3)) — a quarter of the row bytes, one barrier
            __shared__ double part[kWavesPerBlock][3];
            pair_tile<IDT, NT, true, ODT>(a, b, o, chunks[3 * c], chunks[3 * c + 1], 4 * g + wave,
                                          (float)(1.0 - tvals[seg]), (float)tvals[seg], &part[wave][0]);
            __syncthreads();
            if (threadIdx.x < 3) {
                const int q = threadIdx.x;
                rows[unit_slot(u, units) * 3 + q] = (part[0][q] + part[1][q]) + (part[2][q] + part[3][q]);
            }
        } else if constexpr (EMIT) {
            pair_tile<IDT, NT, true, ODT>(a, b, o, chunks[3 * c], chunks[3 * c + 1], 4 * g + wave,
                                          (float)(1.0 - tvals[seg]), (float)tvals[seg], row);
        } else {
            pair_tiles<IDT, NT, kStatsTPW>(a, b, chunks[3 * c], chunks[3 * c + 1], 4 * g + wave, row);
        }
    }
}

// host: the pair sums into partial (chunk rows [nchunks][3], then the row scratch), EMIT optional
int pair_sums(const void* v0, const void* v1, int in_dt, void* out, int out_dt, bool emit,
              const uint64_t* chunk_desc, int64_t nchunks, double* partial, const double* t,
              const uint64_t* seg_ptrs, hipStream_t s, int32_t* zero_word = nullptr) {
    double* rows = partial + 3 * (uint64_t)nchunks;
    const int upc = emit ? kTileSlots / 4 : kTileSlots / (4 * kStatsTPW);
    const uint64_t units = (uint64_t)nchunks * upc;
    for (uint64_t u0 = 0; u0 < units; u0 += kUnitGridCap) {       // > 16.7M units: several launches
        const unsigned g = unit_grid(units - u0);
#define EDT_PS(I, E, O) pair_sums_kernel<I, E, O><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, rows, t, seg_ptrs, u0, zero_word)
        if (!emit) {
            if (in_dt == EDT_F32) EDT_PS(EDT_F32, false, EDT_F32);
            else EDT_PS(EDT_BF16, false, EDT_F32);
        } else if (in_dt == EDT_F32 && out_dt == EDT_F32) EDT_PS(EDT_F32, true, EDT_F32);
        else if (in_dt == EDT_F32) EDT_PS(EDT_F32, true, EDT_BF16);
        else if (out_dt == EDT_F32) EDT_PS(EDT_BF16, true, EDT_F32);
        else EDT_PS(EDT_BF16, true, EDT_BF16);
#undef EDT_PS
        int rc = check_launch(emit ? "pair_sums_kernel (speculative)" : "pair_sums_kernel");
        if (rc) return rc;
    }
    // rows per chunk: 128 (level 0, one per unit's wave), 32 (level 2, one per unit) or 128 / kStatsTPW
    if (emit && kSpecWgRows) return launch_tree_reduce(rows, 3, upc, upc, 1, nchunks, partial, s);
    return launch_tree_reduce(rows, 3, upc * kWavesPerBlock, upc, kWavesPerBlock, nchunks, partial, s);
}

// Fixed-order reduction of a segment's chunk sums: column q of rows [c0, c1) of a row-major table
// with `stride` doubles per row, for the three columns (q0, q1, q2). EDT_SLERP_COEF_BLOCK = 0: one
// wave per segment (lane-strided, then a wave sum); 1: one workgroup per segment (thread-strided,
// wave sums, then the waves in order). Every coefficient kernel uses this one order.
constexpr int kCoefThreads = EDT_SLERP_COEF_BLOCK ? kBlock : 64;

__device__ __forceinline__ bool segment_sums(const double* tab, int stride, int q0, int q1, int q2, int c0,
                                             int c1, double (&out)[3]) {
    const int tid = EDT_SLERP_COEF_BLOCK ? (int)threadIdx.x : (int)(threadIdx.x & 63);
    auto at = [&](uint64_t k) { return tab[k]; };
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int c = c0 + tid; c < c1; c += kCoefThreads) {
        s0 += at((uint64_t)c * stride + q0);
        s1 += at((uint64_t)c * stride + q1);
        s2 += at((uint64_t)c * stride + q2);
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
                                                            float* dot_out, int32_t* redo = nullptr,
                                                            int32_t* any_redo = nullptr) {
    const int seg = coef_segment();
    if (seg >= nseg) return;
    double sums[3];
    if (!segment_sums(partial, 3, 0, 1, 2, first[seg], first[seg + 1], sums)) return;
    float c0, c1, dot;
    slerp_coefficients(sums[0], sums[1], sums[2], tvals[seg], thr, eps, c0, c1, dot);
    coef[2 * seg] = c0;
    coef[2 * seg + 1] = c1;
    if (dot_out) dot_out[seg] = dot;
    if (redo) {                                       // the speculative lerp output stands or not
        const int32_t r = fabsf(dot) > thr ? 0 : 1;
        redo[seg] = r;
        if (r && any_redo) *any_redo = 1;             // every writer stores the same 1
    }
}

template <int IDT, int ODT, bool NT = (EDT_NT_SLERP != 0 && IDT == EDT_BF16)>
__global__ __launch_bounds__(kBlock) void slerp_blend_kernel(const void* v0, const void* v1, void* out,
                                                             const uint64_t* chunks, int64_t nchunks,
                                                             const float* coef, const uint64_t* seg_ptrs,
                                                             const int32_t* redo = nullptr,
                                                             const int32_t* any_redo = nullptr) {
    if (any_redo && *any_redo == 0) return;       // no segment to blend again: the whole grid exits
    for_blend_ranges(chunks, nchunks, [&](uint64_t start, uint64_t end, uint64_t seg) {
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
            lerp_elems<IDT, ODT, EDT_F32, N, NT && N == kVec, (EDT_NT_SLERP_STORES != 0)>(a, b, o, i, c0, c1);
        });
    });
}

// The full blend (the two-pass form's second pass) on the speculative pass's grid: one workgroup
// per unit of 4 tiles in address order (one-shot, no grid-stride loop), wave w the unit's tile
// j = 4 g + w (for_tile's lane mapping; tile 0 also takes the head / tail elements). The chunk row
// is read once, the parents' vectors are loaded before the segment's coefficients, so the data
// loads wait on one dependent read, not three (slerp_blend_kernel's tile form: 7.52 ms against
// lerp's 7.04 on the 7B body, r3 counters — 36 % more wave-cycles, 2.5x the VMEM reads).
// lerp_elems' math: two rounded fp32 products, one rounded sum.
template <int IDT, int ODT, bool NT>
__global__ __launch_bounds__(kBlock) void slerp_blend_tile_kernel(const void* __restrict__ v0,
                                                                  const void* __restrict__ v1,
                                                                  void* __restrict__ out,
                                                                  const uint64_t* __restrict__ chunks, int64_t nchunks,
                                                                  const float* __restrict__ coef,
                                                                  const uint64_t* __restrict__ seg_ptrs, uint64_t u0) {
    constexpr int upc = kTileSlots / kWavesPerBlock;
    const uint64_t u = u0 + blockIdx.x;
    if (u >= (uint64_t)nchunks * upc) return;
    const uint64_t c = u / upc;
    const int j = (int)(u % upc) * kWavesPerBlock + (int)(threadIdx.x >> 6);
    const uint64_t start = chunks[3 * c], len = chunks[3 * c + 1], seg = chunks[3 * c + 2];
    const void* a = v0;
    const void* b = v1;
    void* o = out;
    if (seg_ptrs) {
        a = reinterpret_cast<const void*>(seg_ptrs[3 * seg]);
        b = reinterpret_cast<const void*>(seg_ptrs[3 * seg + 1]);
        o = reinterpret_cast<void*>(seg_ptrs[3 * seg + 2]);
    }
    const uint64_t A = (start + kVec - 1) / kVec * kVec, B = (start + len) / kVec * kVec;
    const uint64_t i = A + (uint64_t)j * kTileElems + (uint64_t)(threadIdx.x & 63) * kVec;
    if (A < B && i < B) {
        const Raw8<IDT> x = ld_raw<IDT, NT>(a, i), y = ld_raw<IDT, NT>(b, i);
        const float c0 = coef[2 * seg], c1 = coef[2 * seg + 1];
        float r[kVec];
#pragma unroll
        for (int e = 0; e < kVec; ++e) r[e] = c0 * x[e] + c1 * y[e];
        st<ODT, kVec, (EDT_NT_SLERP_STORES != 0)>(o, i, r);
    }
    if (j == 0)
        tile0_edge(start, len, [&](uint64_t e) {
            lerp_elems<IDT, ODT, EDT_F32, 1>(a, b, o, e, coef[2 * seg], coef[2 * seg + 1]);
        });
}

// ---------------------------------------------------------------------------------------
// SLERP for a resident population (EDT_RL/edt.py:286-299 merges every selected pair of one
// generation): ONE pass over the M <= 8 members per chunk forms the squared norms and the dots the
// children need (slerp_need_kernel below) where per-child stats passes would read each child's two
// parents. A child's (|vi|^2, |vj|^2, vi.vj) are then read out of its component's sums. Every sum
// is bit-identical to pair_slot() on (vi, vj): the same per-lane FMA sequence in element order (an
// FMA's product is exact, so vi*vj == vj*vi), the same butterfly and tree; the coefficients
// therefore equal edt_slerp_merge's.

constexpr int kGramMaxMembers = 8;
struct Members {
    const void* p[kGramMaxMembers];
};

__host__ __device__ constexpr int tri_index(int a, int b, int M) {   // a <= b < M
    return a * M - a * (a - 1) / 2 + (b - a);
}

template <int M, int N>
__device__ __forceinline__ void pick(const float (&x)[M][N], int idx, float (&y)[N]) {
#pragma unroll
    for (int m = 0; m < M; ++m)
        if (m == idx) {                 // idx is uniform across the workgroup: no divergence
#pragma unroll
            for (int j = 0; j < N; ++j) y[j] = x[m][j];
        }
}

__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

// ---- the needed-sums layout (r5): any pair graph --------------------------------------------------
// A generation needs each distinct parent's norm and each distinct dot its children use — at most
// D + 8 sums for 8 children, against the triangle's D(D+1)/2 (36 at D = 8). EDT_RL's roulette
// selection (EDT_RL/edt.py:231-240, 268-269: 8 pairs drawn with replacement) gives graphs with a
// parent in >= 3 pairs in most generations, so r4's ring (paths / cycles only) does not cover
// them. The host lists a component's D members in the cyclic order that puts the most of its dots
// on consecutive members (a search over the orders: at most 5,040 at D = 8); those dots are RING
// dots (c, c + 1 mod D) whose operands are registers named at compile time (a uniform mask skips
// the unused ones), the rest CHORDS (<= 4; in 3,000 roulette-drawn generations, 99.4 % need <= 3)
// whose member pair is picked per slot by a uniform switch — its arms are the FMAs on the members'
// registers, so no register is indexed at run time (r3's member-major pass lost to scratch that
// way) and the selection costs scalar branches only. Layout of a component: sums [0, D) = |v_m|^2,
// [D, D + NR) = ring dot c, [D + NR, NT) = chord e. Same per-lane chains in element order, same
// butterfly and tree as every other form: each sum is bit-identical to pair_slot() on its two
// members, so every child's coefficients are edt_slerp_merge's.
//
// r6: a component whose dots do not fit the ring + chord slots (dense graphs: K5 and up, a hub in
// more than the slots' pairs) takes the TRIANGLE layout of the same pass (TRI): the upper triangle
// of its Gram matrix, D(D+1)/2 sums at tri_index(a, b, D) in compact member order, each dot formed
// only when a child needs it (a uniform mask; its operands are registers named at compile time, so
// no switch) and the norms always. It replaced the separate Gram kernel (slerp_gram_kernel and its
// edt_slerp_gram / _gram_coef entries): one stats kernel for every pair graph, the same canonical
// per-chunk order, the same rows.
constexpr int kNeedChords = 4;                // chord dot slots (D >= 5)
constexpr int kNeedChordEmits = 8;            // children on chords (distinct ordered pairs)
constexpr int kNeedMaxOut = 16;               // duplicate children per component

template <int D, bool TRI = false>
struct NeedLayout {
    static constexpr int NR = D >= 3 ? D : D - 1;                           // ring dots
    static constexpr int NC = D <= 3 ? 0 : D == 4 ? 2 : kNeedChords;        // chord slots
    static constexpr int NT = TRI ? D * (D + 1) / 2 : D + NR + NC;
};
inline int need_nr(int D) { return D >= 3 ? D : D - 1; }
inline int need_nc(int D) { return D <= 3 ? 0 : D == 4 ? 2 : kNeedChords; }
inline int need_nt(int D) { return D + need_nr(D) + need_nc(D); }

// What one needed-sums pass forms (and, EMIT, writes). Passed by value: every field is uniform.
struct NeedSpec {
    uint32_t ring;                            // ring dot c (members c, c + 1 mod D) in use: bit c
    int32_t nchord;
    int32_t code[kNeedChords];                // chord e: members u * 8 + v (u < v)
    // EMIT: children on ring edge c: (c, c + 1) -> out_fwd[c] (bit c of fwd), (c + 1, c) -> out_rev[c]
    uint32_t fwd, rev;
    void* out_fwd[kGramMaxMembers];
    void* out_rev[kGramMaxMembers];
    int32_t nemit;                            // children off the ring (chords, self-pairs): distinct
    int32_t ea[kNeedChordEmits], eb[kNeedChordEmits];   // ordered pairs v0 = ea[e], v1 = eb[e]
    void* out[kNeedChordEmits];
    int32_t nextra;                           // further children of an emitted pair: slot c (fwd),
    int32_t xslot[kNeedMaxOut];               // 8 + c (rev), 16 + e (chord pair e)
    void* xout[kNeedMaxOut];
    const double* t;                          // per segment
    int32_t* zero_word;                       // the any-redo word, zeroed by block 0 of the first launch
    uint64_t tri;                             // TRI layout: bit tri_index(a, b, D) = dot (a, b) formed
};

// acc += the dot of members (code / 8, code % 8) over N elements: one switch arm per pair, the
// operands registers named at compile time (pairs with a member >= D have no arm). Each arm ends
// with an empty asm statement carrying its own immediate: LLVM cannot merge arms whose last
// instructions differ in an inline-asm immediate, so it neither sinks the FMAs out of the arms
// (PHIs of the operands = register copies per FMA) nor turns the switch into an indexed load.
template <int D, int N>
__device__ __forceinline__ void need_dot(const double (&d)[D][N], int code, double& acc) {
#define EDT_ND(U, V)                                                                        \
    case U * 8 + V:                                                                         \
        if constexpr (V < D) {                                                              \
            _Pragma("unroll") for (int j = 0; j < N; ++j) acc = __builtin_fma(d[U][j], d[V][j], acc); \
            asm volatile("; need dot %1" : "+v"(acc) : "n"(U * 8 + V));                     \
        }                                                                                   \
        break;
    switch (code) {
        EDT_ND(0, 1) EDT_ND(0, 2) EDT_ND(0, 3) EDT_ND(0, 4) EDT_ND(0, 5) EDT_ND(0, 6) EDT_ND(0, 7)
        EDT_ND(1, 2) EDT_ND(1, 3) EDT_ND(1, 4) EDT_ND(1, 5) EDT_ND(1, 6) EDT_ND(1, 7)
        EDT_ND(2, 3) EDT_ND(2, 4) EDT_ND(2, 5) EDT_ND(2, 6) EDT_ND(2, 7)
        EDT_ND(3, 4) EDT_ND(3, 5) EDT_ND(3, 6) EDT_ND(3, 7)
        EDT_ND(4, 5) EDT_ND(4, 6) EDT_ND(4, 7)
        EDT_ND(5, 6) EDT_ND(5, 7)
        EDT_ND(6, 7)
        default: break;
    }
#undef EDT_ND
}

// The sums of N elements of every member (the lane's vector: N = 8; its head / tail element:
// N = 1), continuing each chain: the members' fp64 values per group of EDT_NEED_GROUP elements,
// the norms, the ring dots in use, the chords (TRI: the norms and the masked triangle dots).
template <int D, int N, bool TRI = false, typename X>
__device__ __forceinline__ void need_fma(const X (&x)[D], const NeedSpec& S, double (&g)[NeedLayout<D, TRI>::NT]) {
    constexpr int NR = NeedLayout<D, TRI>::NR, NC = NeedLayout<D, TRI>::NC;
    constexpr int H = N < EDT_NEED_GROUP ? N : EDT_NEED_GROUP;
#pragma unroll
    for (int h = 0; h < N / H; ++h) {
        double d[D][H];
#pragma unroll
        for (int m = 0; m < D; ++m)
#pragma unroll
            for (int j = 0; j < H; ++j) d[m][j] = x[m][H * h + j];
        if constexpr (TRI) {                      // the norms, and the dots the mask names
#pragma unroll
            for (int u = 0; u < D; ++u)
#pragma unroll
                for (int v = u; v < D; ++v)
                    if (u == v || ((S.tri >> tri_index(u, v, D)) & 1u)) {
#pragma unroll
                        for (int j = 0; j < H; ++j)
                            g[tri_index(u, v, D)] = __builtin_fma(d[u][j], d[v][j], g[tri_index(u, v, D)]);
                    }
        } else {
#pragma unroll
            for (int m = 0; m < D; ++m)
#pragma unroll
                for (int j = 0; j < H; ++j) g[m] = __builtin_fma(d[m][j], d[m][j], g[m]);
#pragma unroll
            for (int c = 0; c < NR; ++c)
                if ((S.ring >> c) & 1u) {
#pragma unroll
                    for (int j = 0; j < H; ++j) g[D + c] = __builtin_fma(d[c][j], d[(c + 1) % D][j], g[D + c]);
                }
#pragma unroll
            for (int e = 0; e < NC; ++e)
                if (e < S.nchord) need_dot<D, H>(d, S.code[e], g[D + NR + e]);
        }
    }
}

// member `idx` of x (uniform): a scalar switch, one copy of the member's registers per arm (the
// arms' asm immediates keep LLVM from turning the switch into an indexed private array: scratch)
template <int M>
__device__ __forceinline__ void need_pin(Raw8<EDT_BF16>& r) { asm volatile("; pick %1" : "+v"(r.w) : "n"(M)); }
template <int M>
__device__ __forceinline__ void need_pin(Raw8<EDT_F32>& r) { asm volatile("; pick %2" : "+v"(r.lo), "+v"(r.hi) : "n"(M)); }
template <int M>
__device__ __forceinline__ void need_pin(Raw1& r) { asm volatile("; pick %1" : "+v"(r.v[0]) : "n"(M)); }

template <int D, typename X>
__device__ __forceinline__ X need_pick(const X (&x)[D], int idx) {
    X r;
    switch (idx) {
#define EDT_NP(M) case M: if constexpr (M < D) { r = x[M]; need_pin<M>(r); } break;
        EDT_NP(0) EDT_NP(1) EDT_NP(2) EDT_NP(3) EDT_NP(4) EDT_NP(5) EDT_NP(6) EDT_NP(7)
#undef EDT_NP
        default: r = x[0]; break;
    }
    return r;
}

// Global-memory access through a pointer built from a uniform integer: the address space is
// stated (global_* instructions, not flat_*: a flat access also counts on lgkmcnt and retires out
// of order, so every LDS wait would drain it), the base stays in scalar registers.
typedef __attribute__((address_space(1))) const char gcchar;
typedef __attribute__((address_space(1))) char gchar;

__device__ __forceinline__ gcchar* global_ptr(const void* p, uint64_t byte_off) {
    return reinterpret_cast<gcchar*>(uniform_u64(reinterpret_cast<uint64_t>(p) + byte_off));
}

template <int IDT, bool NT>
__device__ __forceinline__ Raw8<IDT> ld_raw_g(gcchar* p) {
    typedef __attribute__((address_space(1))) const u32x4 gu4;
    typedef __attribute__((address_space(1))) const f32x4 gf4;
    Raw8<IDT> r;
    if constexpr (IDT == EDT_BF16) {
        if constexpr (NT) r.w = __builtin_nontemporal_load(reinterpret_cast<gu4*>(p));
        else r.w = *reinterpret_cast<gu4*>(p);
    } else {
        if constexpr (NT) {
            r.lo = __builtin_nontemporal_load(reinterpret_cast<gf4*>(p));
            r.hi = __builtin_nontemporal_load(reinterpret_cast<gf4*>(p + 16));
        } else {
            r.lo = *reinterpret_cast<gf4*>(p);
            r.hi = *reinterpret_cast<gf4*>(p + 16);
        }
    }
    return r;
}

template <int IDT>
__device__ __forceinline__ float ld1_g(gcchar* p) {
    if constexpr (IDT == EDT_BF16) return __uint_as_float((uint32_t)*reinterpret_cast<__attribute__((address_space(1))) const uint16_t*>(p) << 16);
    else return *reinterpret_cast<__attribute__((address_space(1))) const float*>(p);
}

// st<ODT, N>'s rounding and packing, stored through a global pointer
template <int ODT, int N>
__device__ __forceinline__ void st_g(gchar* p, const float (&x)[N]) {
    if constexpr (ODT == EDT_F32) {
        typedef __attribute__((address_space(1))) f32x4 gf4;
        if constexpr (N == 8) {
            *reinterpret_cast<gf4*>(p) = (f32x4){x[0], x[1], x[2], x[3]};
            *reinterpret_cast<gf4*>(p + 16) = (f32x4){x[4], x[5], x[6], x[7]};
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) reinterpret_cast<__attribute__((address_space(1))) float*>(p)[j] = x[j];
        }
    } else {
        if constexpr (N == 8) {
            typedef __attribute__((address_space(1))) u32x4 gu4;
            u32x4 w;
            w.x = pack_bf(x[0], x[1]); w.y = pack_bf(x[2], x[3]);
            w.z = pack_bf(x[4], x[5]); w.w = pack_bf(x[6], x[7]);
            *reinterpret_cast<gu4*>(p) = w;
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j)
                reinterpret_cast<__attribute__((address_space(1))) uint16_t*>(p)[j] = uint16_t(pack_bf(x[j], 0.f) & 0xffffu);
        }
    }
}

// EMIT: every child's lerp-branch output l0 v0 + l1 v1 (pair_tile's math: two rounded fp32
// products, one rounded sum) — ring-edge children from registers named at compile time, the others
// through need_pick — each distinct ordered pair computed once and stored to every child of it. A
// lane's vector (N = 8) is stored through a uniform base (the tile's start, scalar registers) + the
// lane's byte offset; its head / tail element (N = 1) at element i0.
template <int ODT, int D, int N, typename X>
__device__ __forceinline__ void need_emit(const X (&x)[D], const NeedSpec& S, uint64_t i0, uint32_t lane,
                                          float l0, float l1) {
    constexpr uint64_t osz = ODT == EDT_BF16 ? 2 : 4;
    constexpr int NR = NeedLayout<D>::NR;
    auto store = [&](void* out, const float (&o)[N]) {
        if constexpr (N == kVec) {                // uniform tile start + the lane's offset
            gchar* base = const_cast<gchar*>(global_ptr(out, i0 * osz));
            st_g<ODT, N>(base + lane * (kVec * osz), o);
        } else {                                  // i0: this lane's own element
            st_g<ODT, N>(reinterpret_cast<gchar*>(reinterpret_cast<uint64_t>(out)) + i0 * osz, o);
        }
    };
    auto emit = [&](const X& a, const X& b, void* out, int slot) {
        float o[N];
#pragma unroll
        for (int j = 0; j < N; ++j) o[j] = l0 * a[j] + l1 * b[j];
        store(out, o);
        for (int k = 0; k < S.nextra; ++k)
            if (S.xslot[k] == slot) store(S.xout[k], o);
    };
#pragma unroll
    for (int c = 0; c < NR; ++c) {
        if ((S.fwd >> c) & 1u) emit(x[c], x[(c + 1) % D], S.out_fwd[c], c);
        if ((S.rev >> c) & 1u) emit(x[(c + 1) % D], x[c], S.out_rev[c], 8 + c);
    }
#pragma unroll
    for (int e = 0; e < kNeedChordEmits; ++e) {
        if (e >= S.nemit) break;
        emit(need_pick<D>(x, S.ea[e]), need_pick<D>(x, S.eb[e]), S.out[e], 16 + e);
    }
}

// The needed sums as rows of level 4, one workgroup per unit of 16 tiles in address order (the
// Gram kernel's grid, reduction and row format; tiles past the chunk's aligned body load zeros,
// which leave every chain's bits unchanged). bf16 members: the next tiles land in LDS by DMA while
// this tile is summed from registers (below; a two-register-set prefetch measured slower: its
// VGPRs cost a wave per SIMD).
template <int IDT, int D, bool EMIT = false, int ODT = EDT_BF16, bool TRI = false>
__global__ __launch_bounds__(kBlock, EDT_NEED_MIN_WAVES) void slerp_need_kernel(Members mem, NeedSpec S,
                                                                                 const uint64_t* chunks,
                                                                                 int64_t nchunks, double* rows,
                                                                                 uint64_t u0) {
    static_assert(!(EMIT && TRI), "the triangle layout is a stats pass only");
    constexpr int NT = NeedLayout<D, TRI>::NT, N2 = Red<NT>::N2;
    constexpr bool kGlds = EDT_NEED_GLDS != 0 && IDT == EDT_BF16;
    // LDS-DMA stages per wave: two (two tiles in flight besides the one in registers) where the
    // registers already limit the pass to 2 waves per SIMD (the emitting form, D = 8), else one
    // (3 waves per SIMD fit the LDS with one stage, not with two; the triangle's larger partials
    // table leaves room for one)
    constexpr int kStages = kGlds ? ((EMIT || D == 8) && !TRI ? 2 : 1) : 1;
    __shared__ u32x4 stage[kStages][kGlds ? kWavesPerBlock : 1][kGlds ? D : 1][64];
    if constexpr (EMIT)
        if (S.zero_word && u0 == 0 && blockIdx.x == 0 && threadIdx.x == 0) *S.zero_word = 0;
    constexpr int upc = kTileSlots / 16;
    constexpr int kPad = 17;
    __shared__ double part[kWavesPerBlock][4 * N2 * kPad];
    __shared__ double ts2[kWavesPerBlock][NT];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t units = (uint64_t)nchunks * upc;
    const uint64_t u = u0 + blockIdx.x;
    if (u >= units) return;
    const uint64_t c = u / upc;
    const int g = (int)(u % upc);
    const uint64_t start = uniform_u64(chunks[3 * c]), len = uniform_u64(chunks[3 * c + 1]);
    float l0 = 0.f, l1 = 0.f;
    if constexpr (EMIT) {
        const double tv = S.t[chunks[3 * c + 2]];
        l0 = (float)(1.0 - tv);
        l1 = (float)tv;
    }
    int pos = 0;
#pragma unroll
    for (int row = 0; row < 4; ++row)
#pragma unroll
        for (int sl = 0; sl < N2; ++sl) {
            bool owner;
            if (red_index<NT>(sl, row * 16, owner) == lane) pos = row * N2 + sl;
        }
    const double* mine = &part[wave][pos * kPad];
    double* put = &part[wave][(lane >> 4) * N2 * kPad + (lane & 15)];
    const uint64_t a = (start + kVec - 1) / kVec * kVec, b = (start + len) / kVec * kVec;
    double n01 = 0.0, n23 = 0.0;
    // a member's tile: a uniform base (scalar registers, readfirstlane so LLVM cannot fold the lane
    // offset into a per-member 64-bit address held in vector registers) + the lane's byte offset
    constexpr uint32_t esz = IDT == EDT_BF16 ? 2 : 4;
    auto member_base = [&](int m, uint64_t e0) { return global_ptr(mem.p[m], e0 * esz); };
    auto load_tile = [&](int k, Raw8<IDT> (&x)[D]) {
        const uint64_t t0 = a + (uint64_t)(16 * g + 4 * wave + k) * kTileElems;     // uniform
        const uint32_t off = (uint32_t)lane * (kVec * esz);
        if (t0 + kTileElems <= b) {                    // the whole tile inside the aligned body
#pragma unroll
            for (int m = 0; m < D; ++m) x[m] = ld_raw_g<IDT, EDT_GRAM_NT != 0>(member_base(m, t0) + off);
        } else {
#pragma unroll
            for (int m = 0; m < D; ++m) x[m] = Raw8<IDT>{};
            if (a < b && t0 + (uint64_t)lane * kVec < b) {
#pragma unroll
                for (int m = 0; m < D; ++m) x[m] = ld_raw_g<IDT, EDT_GRAM_NT != 0>(member_base(m, t0) + off);
            }
        }
    };
    // `mid()` runs right after the tile's lerp-branch stores (the staged loop issues the next DMA
    // there, so a counted vmcnt can leave it in flight past those stores)
    auto tile = [&](int k, const Raw8<IDT> (&x)[D], auto&& mid) {
        const int j = 16 * g + 4 * wave + k;
        const uint64_t i = a + (uint64_t)j * kTileElems + (uint64_t)lane * kVec;
        double gs[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) gs[q] = 0.0;
        if constexpr (EMIT)               // first: the members' registers are all it needs
            if (a < b && i < b) need_emit<ODT, D, kVec>(x, S, a + (uint64_t)j * kTileElems, (uint32_t)lane, l0, l1);
        mid();
        need_fma<D, kVec, TRI>(x, S, gs);
        if (j == 0)
            tile0_edge(start, len, [&](uint64_t e) {
                Raw1 y[D];
#pragma unroll
                for (int m = 0; m < D; ++m) y[m].v[0] = ld1_g<IDT>(member_base(m, start) + (uint32_t)(e - start) * esz);
                need_fma<D, 1, TRI>(y, S, gs);
                if constexpr (EMIT) need_emit<ODT, D, 1>(y, S, e, 0, l0, l1);
            });
        double r[N2];
        tile_swap_levels<NT>(gs, r);
#pragma unroll
        for (int sl = 0; sl < N2; ++sl) put[sl * kPad] = r[sl];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double p[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) p[t] = mine[t];
        const double tsum = row_tree16(p);
        if (k == 0) n01 = tsum;
        else if (k == 1) n01 = n01 + tsum;
        else if (k == 2) n23 = tsum;
        else n23 = n23 + tsum;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    bool staged = false;
    if constexpr (kGlds) if (a + (uint64_t)(16 * g + 16) * kTileElems <= b) {
        staged = true;
        // the unit's tiles are whole: tile k + 1 lands in the wave's LDS stage by DMA
        // (global_load_lds, no registers) while tile k is summed from registers — two tiles of
        // loads in flight per wave at the registers of one. vmcnt(0) before reading the stage
        // (the wave's own DMA; its stores count too on gfx9), lgkmcnt(0) before the next DMA.
        // Vector-memory operations retire in issue order (loads, stores and LDS-DMA alike), so
        // with two stages the wait for tile k's DMA is vmcnt(D): only tile k + 1's D DMA
        // operations, issued after every older load and store, may stay in flight.
        auto issue = [&](int k) {
            const uint64_t t0 = a + (uint64_t)(16 * g + 4 * wave + k) * kTileElems;
#pragma unroll
            for (int m = 0; m < D; ++m)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(member_base(m, t0) + lane * (kVec * esz)),
                    (__attribute__((address_space(3))) void*)&stage[k % kStages][wave][m][0], 16, 0, EDT_GRAM_NT ? 2 : 0);
        };
        auto fetch = [&](int k, Raw8<IDT> (&x)[D]) {
            if (kStages == 2 && k + 1 < 4) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(D) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // the stage read in asm: the compiler's own wait before an LDS read after an LDS-DMA
            // is vmcnt(0), which would drain the next tile's DMA too
            const uint32_t sa = (uint32_t)(uintptr_t)&stage[k % kStages][wave][0][lane];
#pragma unroll
            for (int m = 0; m < D; ++m)
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x[m].w) : "v"(sa), "n"(m * 1024) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        };
        issue(0);
        if constexpr (kStages == 2) issue(1);
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {
            Raw8<IDT> x[D];
            fetch(k, x);
            if constexpr (kStages == 2) tile(k, x, [&] { if (k + 2 < 4) issue(k + 2); });
            else {
                if (k < 3) issue(k + 1);
                tile(k, x, [] {});
            }
        }
    }
    if (!staged) {
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {
            Raw8<IDT> x[D];
            load_tile(k, x);
            tile(k, x, [] {});
        }
    }
    if (lane < NT) ts2[wave][lane] = n01 + n23;
    __syncthreads();
    if (wave == 0 && lane < NT)
        rows[unit_slot(u, units) * NT + lane] = (ts2[0][lane] + ts2[1][lane]) + (ts2[2][lane] + ts2[3][lane]);
}

// host: one needed-sums pass over the D members of `mem` (their order is the layout's) into sums
// ([nchunks][need_nt(D)]; `rows`: the level-4 row scratch, nchunks x 8 x need_nt(D) doubles);
// emit: also every child's lerp-branch output (S.out, S.t, S.zero_word).
inline int need_sums(const Members& mem, int D, const NeedSpec& S, int in_dt, int out_dt, bool emit,
                     const uint64_t* chunk_desc, int64_t nchunks, double* sums, double* rows, hipStream_t s,
                     bool tri = false) {
    if (D < 1 || D > kGramMaxMembers) return fail(EDT_ERR_ARG, "needed-sums pass over %d members", D);
    if (tri && emit) return fail(EDT_ERR_ARG, "the triangle layout is a stats pass only");
    if (!tri && (S.nchord < 0 || S.nchord > need_nc(D))) return fail(EDT_ERR_ARG, "%d chords over %d members", S.nchord, D);
    if (S.nemit < 0 || S.nemit > kNeedChordEmits || S.nextra < 0 || S.nextra > kNeedMaxOut)
        return fail(EDT_ERR_ARG, "bad emit table");
    constexpr int upc = kTileSlots / 16;
    const uint64_t units = (uint64_t)nchunks * upc;
    for (uint64_t u0 = 0; u0 < units; u0 += kUnitGridCap) {
        const unsigned g = unit_grid(units - u0);
#define EDT_NK(M)                                                                                          \
    case M:                                                                                                \
        if (tri) {                                                                                         \
            if (in_dt == EDT_F32) slerp_need_kernel<EDT_F32, M, false, EDT_BF16, true><<<g, kBlock, 0, s>>>(mem, S, chunk_desc, nchunks, rows, u0); \
            else slerp_need_kernel<EDT_BF16, M, false, EDT_BF16, true><<<g, kBlock, 0, s>>>(mem, S, chunk_desc, nchunks, rows, u0); \
        } else if (!emit) {                                                                                \
            if (in_dt == EDT_F32) slerp_need_kernel<EDT_F32, M><<<g, kBlock, 0, s>>>(mem, S, chunk_desc, nchunks, rows, u0); \
            else slerp_need_kernel<EDT_BF16, M><<<g, kBlock, 0, s>>>(mem, S, chunk_desc, nchunks, rows, u0);    \
        } else if (in_dt == EDT_F32 && out_dt == EDT_F32) {                                                \
            slerp_need_kernel<EDT_F32, M, true, EDT_F32><<<g, kBlock, 0, s>>>(mem, S, chunk_desc, nchunks, rows, u0); \
        } else if (in_dt == EDT_F32) {                                                                     \
            slerp_need_kernel<EDT_F32, M, true, EDT_BF16><<<g, kBlock, 0, s>>>(mem, S, chunk_desc, nchunks, rows, u0); \
        } else if (out_dt == EDT_F32) {                                                                    \
            slerp_need_kernel<EDT_BF16, M, true, EDT_F32><<<g, kBlock, 0, s>>>(mem, S, chunk_desc, nchunks, rows, u0); \
        } else {                                                                                           \
            slerp_need_kernel<EDT_BF16, M, true, EDT_BF16><<<g, kBlock, 0, s>>>(mem, S, chunk_desc, nchunks, rows, u0); \
        }                                                                                                  \
        break;
        switch (D) {
            EDT_NK(1) EDT_NK(2) EDT_NK(3) EDT_NK(4) EDT_NK(5) EDT_NK(6) EDT_NK(7) EDT_NK(8)
            default: break;
        }
#undef EDT_NK
        int rc = check_launch(emit ? "slerp_need_kernel (speculative)" : "slerp_need_kernel");
        if (rc) return rc;
    }
    return launch_tree_reduce(rows, tri ? D * (D + 1) / 2 : need_nt(D), kGramRows, upc, 1, nchunks, sums, s);
}

// How edt_slerp_population lays out its sums: the distinct parents split into the connected
// components of the "needs a dot" graph (an edge per child with two different parents). r5: a
// component takes the NEEDED layout (its norms + its dots: ring dots along the cyclic order that
// covers the most of them, the rest chords) when its chords fit their slots, else the triangle
// (every pair). Every member belongs to one component, so each parent is still read once in the
// whole pass. (r4's ring layout — paths and cycles only, a compile-time ring kernel — was measured
// against it on roulette-drawn generations and removed: profiles/r05_pop_roulette_*.json.)
enum { kTri = 0, kNeed = 2 };

struct GramPlan {
    int ncomp = 0;
    int comp_of[kGramMaxMembers];          // compact member -> component
    int pos[kGramMaxMembers];              // compact member -> position in its component's list
    int size[kGramMaxMembers];
    int kind[kGramMaxMembers];
    int list[kGramMaxMembers][kGramMaxMembers];   // component -> members (compact), in layout order
    NeedSpec need[kGramMaxMembers];        // kNeed: the component's ring mask and chords
    uint64_t off[kGramMaxMembers];         // component's chunk rows in gram (doubles)
    int nt(int k) const {
        return kind[k] == kNeed ? need_nt(size[k]) : size[k] * (size[k] + 1) / 2;
    }
    int norm_index(int c) const {
        const int k = comp_of[c], p = pos[c];
        return kind[k] == kTri ? tri_index(p, p, size[k]) : p;
    }
    // ring edge of positions (p1, p2) in a component of M members, or -1
    static int ring_edge(int p1, int p2, int M) {
        if (M == 2) return p1 != p2 ? 0 : -1;
        if (M < 3) return -1;
        if ((p1 + 1) % M == p2) return p1;
        if ((p2 + 1) % M == p1) return p2;
        return -1;
    }
    int dot_index(int c1, int c2) const {            // same component
        const int k = comp_of[c1], M = size[k];
        int p1 = pos[c1], p2 = pos[c2];
        if (c1 == c2) return norm_index(c1);
        if (kind[k] == kNeed) {
            const int e = ring_edge(p1, p2, M);
            if (e >= 0) return M + e;
            if (p1 > p2) { const int t = p1; p1 = p2; p2 = t; }
            for (int c = 0; c < need[k].nchord; ++c)
                if (need[k].code[c] == p1 * 8 + p2) return M + need_nr(M) + c;
            return -1;
        }
        if (p1 > p2) { const int t = p1; p1 = p2; p2 = t; }
        return tri_index(p1, p2, M);
    }
};

// The cyclic order of a component's n members (compact ids, sorted) that puts the most of its
// dots on consecutive members: members[0] first, every order of the rest (n <= 8: <= 5,040), the
// first best in lexicographic order kept (deterministic); stops early when every dot is covered.
inline void need_cyclic_order(const int* members, int n, const bool (&adj)[kGramMaxMembers][kGramMaxMembers],
                              int nedges, int* order) {
    for (int x = 0; x < n; ++x) order[x] = members[x];
    if (n <= 3) return;                               // every dot is a ring dot
    int perm[kGramMaxMembers], best = -1;
    for (int x = 0; x < n; ++x) perm[x] = members[x];
    do {
        int cov = 0;
        for (int c = 0; c < n; ++c) cov += adj[perm[c]][perm[(c + 1) % n]];
        if (cov > best) {
            best = cov;
            for (int x = 0; x < n; ++x) order[x] = perm[x];
            if (cov == nedges) return;
        }
    } while (std::next_permutation(perm + 1, perm + n));
}

inline void plan_gram(int D, const int* a, const int* b, int npairs, int64_t nchunks, GramPlan& G) {
    bool adj[kGramMaxMembers][kGramMaxMembers] = {};
    int deg[kGramMaxMembers] = {};
    for (int q = 0; q < npairs; ++q)
        if (a[q] != b[q] && !adj[a[q]][b[q]]) {
            adj[a[q]][b[q]] = adj[b[q]][a[q]] = true;
            ++deg[a[q]];
            ++deg[b[q]];
        }
    for (int c = 0; c < D; ++c) G.comp_of[c] = -1;
    for (int c0 = 0; c0 < D; ++c0) {
        if (G.comp_of[c0] >= 0) continue;
        const int k = G.ncomp++;
        memset(&G.need[k], 0, sizeof(NeedSpec));
        int members[kGramMaxMembers], n = 0, stack[kGramMaxMembers], top = 0;
        stack[top++] = c0;
        G.comp_of[c0] = k;
        int nedge2 = 0;
        while (top) {                                 // the component, in compact order below
            const int c = stack[--top];
            members[n++] = c;
            nedge2 += deg[c];
            for (int o = 0; o < D; ++o)
                if (adj[c][o] && G.comp_of[o] < 0) {
                    G.comp_of[o] = k;
                    stack[top++] = o;
                }
        }
        for (int x = 1; x < n; ++x)                   // sort: compact order
            for (int y = x; y > 0 && members[y] < members[y - 1]; --y) {
                const int t = members[y]; members[y] = members[y - 1]; members[y - 1] = t;
            }
        G.size[k] = n;
        need_cyclic_order(members, n, adj, nedge2 / 2, G.list[k]);
        G.kind[k] = kNeed;                            // checked against the chord slots below
        for (int x = 0; x < n; ++x) G.pos[G.list[k][x]] = x;
    }
    // the needed components' ring masks and chords (chords in the order the children first use them)
    for (int q = 0; q < npairs; ++q) {
        if (a[q] == b[q]) continue;
        const int k = G.comp_of[a[q]];
        if (G.kind[k] != kNeed) continue;
        NeedSpec& S = G.need[k];
        int p1 = G.pos[a[q]], p2 = G.pos[b[q]];
        const int e = GramPlan::ring_edge(p1, p2, G.size[k]);
        if (e >= 0) {
            S.ring |= 1u << e;
            continue;
        }
        if (p1 > p2) { const int t = p1; p1 = p2; p2 = t; }
        bool seen = false;
        for (int c = 0; c < S.nchord; ++c) seen = seen || S.code[c] == p1 * 8 + p2;
        if (seen) continue;
        if (S.nchord == need_nc(G.size[k])) {         // more chords than slots: the triangle
            G.kind[k] = kTri;
            for (int x = 1; x < G.size[k]; ++x) {      // compact order again
                int* L = G.list[k];
                for (int y = x; y > 0 && L[y] < L[y - 1]; --y) { const int t = L[y]; L[y] = L[y - 1]; L[y - 1] = t; }
            }
            for (int x = 0; x < G.size[k]; ++x) G.pos[G.list[k][x]] = x;
            continue;
        }
        S.code[S.nchord++] = p1 * 8 + p2;
    }
    // the triangle components' masks: the dots their children use, at compact positions
    for (int q = 0; q < npairs; ++q) {
        if (a[q] == b[q]) continue;
        const int k = G.comp_of[a[q]];
        if (G.kind[k] != kTri) continue;
        int p1 = G.pos[a[q]], p2 = G.pos[b[q]];
        if (p1 > p2) { const int t = p1; p1 = p2; p2 = t; }
        G.need[k].tri |= 1ull << tri_index(p1, p2, G.size[k]);
    }
    uint64_t off = 0;
    for (int k = 0; k < G.ncomp; ++k) {
        G.off[k] = off;
        off += (uint64_t)nchunks * G.nt(k);
    }
}

// The row scratch a plan's passes need after its chunk rows (doubles): the largest component's
// level-4 rows (one component's pass at a time on one stream).
inline uint64_t plan_row_scratch(const GramPlan& G, int64_t nchunks) {
    uint64_t m = 0;
    for (int k = 0; k < G.ncomp; ++k) {
        const uint64_t r = (uint64_t)nchunks * kGramRows * G.nt(k);
        m = r > m ? r : m;
    }
    return m;
}

// One component's stats pass (no outputs), whichever layout it took.
inline int plan_component_sums(const GramPlan& G, int k, const void* const* dm, int in_dt, const uint64_t* chunk_desc,
                               int64_t nchunks, double* gram, double* rows, hipStream_t s) {
    Members gm;
    memset(&gm, 0, sizeof(gm));
    for (int x = 0; x < G.size[k]; ++x) gm.p[x] = dm[G.list[k][x]];
    return need_sums(gm, G.size[k], G.need[k], in_dt, EDT_F32, false, chunk_desc, nchunks, gram + G.off[k], rows, s,
                     G.kind[k] == kTri);
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
    double* slots[kBlendMaxChildren];         // the child's row table (speculative stats pass)
    int nchildren;
};

template <int IDT, int ODT>
__global__ __launch_bounds__(kBlock) void slerp_blend_population_kernel(BlendChildren B, const uint64_t* chunks,
                                                                        int64_t nchunks, uint64_t cbase,
                                                                        const int32_t* any_redo = nullptr) {
    if (any_redo && *any_redo == 0) return;       // no child needs a segment blended again
    const uint64_t per_group = 8ull * (uint64_t)B.nchildren;
    const uint64_t r = blockIdx.x % per_group;
    const int child = (int)(r / 8);
    const int64_t c = (int64_t)(cbase + (blockIdx.x / per_group) * 8 + (r % 8));
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

// Co-located launches (block -> (unit, child), all children of 8 consecutive units on the XCDs of
// those units): `units` split into launches of whole groups of 8 units under the dispatch cap.
template <typename F>
inline int colocated_launches(uint64_t units, int nchildren, F&& launch) {
    const uint64_t per_launch = kGridBlockCap / (8ull * (uint64_t)nchildren) * 8ull;   // units, a multiple of 8
    for (uint64_t u0 = 0; u0 < units; u0 += per_launch) {
        const uint64_t n = units - u0 < per_launch ? units - u0 : per_launch;
        launch(u0, (unsigned)((n + 7) / 8 * 8ull * (uint64_t)nchildren));
        int rc = check_launch("co-located population kernel");
        if (rc) return rc;
    }
    return EDT_OK;
}

// Speculative population pass for more than 8 distinct parents: block (unit, child) with the
// co-located placement above, a unit being 4 tiles of a chunk (one per wave): the blocks of every
// child for one unit carry the same blockIdx % 8 (one XCD, one L2). Each forms its child's tile
// sums exactly as pair_sums_kernel does (the child's own row table) and writes the
// lerp-branch output in the same pass. Shared parents cross HBM once for all children.
template <int IDT, int ODT>
__global__ __launch_bounds__(kBlock) void slerp_pop_stats_lerp_kernel(BlendChildren B, const uint64_t* chunks,
                                                                      int64_t nchunks, const double* tvals, uint64_t u0,
                                                                      int32_t* zero_word) {
    if (zero_word && u0 == 0 && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;   // the any-redo flag
    constexpr int upc = kTileSlots / 4;
    const uint64_t per_group = 8ull * (uint64_t)B.nchildren;
    const uint64_t r = blockIdx.x % per_group;
    const int child = (int)(r / 8);
    const uint64_t u = u0 + (blockIdx.x / per_group) * 8 + (r % 8);
    const uint64_t units = (uint64_t)nchunks * upc;
    if (u >= units) return;
    const uint64_t c = u / upc;
    const int wave = (int)(threadIdx.x >> 6);
    const uint64_t seg = chunks[3 * c + 2];
    // default-policy loads: a parent's chunk is re-read by its other children from L2
    if constexpr (kSpecWgRows) {                      // one level-2 row per block, as pair_sums_kernel
        __shared__ double part[kWavesPerBlock][3];
        pair_tile<IDT, false, true, ODT>(B.v0[child], B.v1[child], B.out[child], chunks[3 * c], chunks[3 * c + 1],
                                         (int)(u % upc) * kWavesPerBlock + wave, (float)(1.0 - tvals[seg]),
                                         (float)tvals[seg], &part[wave][0]);
        __syncthreads();
        if (threadIdx.x < 3) {
            const int q = threadIdx.x;
            B.slots[child][unit_slot(u, units) * 3 + q] = (part[0][q] + part[1][q]) + (part[2][q] + part[3][q]);
        }
    } else {
        pair_tile<IDT, false, true, ODT>(B.v0[child], B.v1[child], B.out[child], chunks[3 * c], chunks[3 * c + 1],
                                         (int)(u % upc) * kWavesPerBlock + wave, (float)(1.0 - tvals[seg]),
                                         (float)tvals[seg],
                                         B.slots[child] + (unit_slot(u, units) * kWavesPerBlock + wave) * 3);
    }
}

// Per segment for the pair (i, j): slerp_coef_kernel's reduction over the chunks, reading the
// three Gram columns of the pair.
__global__ __launch_bounds__(kBlock) void slerp_gram_coef_kernel(const double* gram, int NT, int qi, int qj, int qd,
                                                                 const int32_t* first, int nseg,
                                                                 const double* tvals, float thr, float eps,
                                                                 float* coef, float* dot_out, int32_t* redo = nullptr,
                                                                 int32_t* any_redo = nullptr) {
    const int seg = coef_segment();
    if (seg >= nseg) return;
    double sums[3];
    if (!segment_sums(gram, NT, qi, qj, qd, first[seg], first[seg + 1], sums)) return;
    float c0, c1, dot;
    slerp_coefficients(sums[0], sums[1], sums[2], tvals[seg], thr, eps, c0, c1, dot);
    coef[2 * seg] = c0;
    coef[2 * seg + 1] = c1;
    if (dot_out) dot_out[seg] = dot;
    if (redo) {                                       // as slerp_coef_kernel
        const int32_t r = fabsf(dot) > thr ? 0 : 1;
        redo[seg] = r;
        if (r && any_redo) *any_redo = 1;
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
    const int32_t* any;                       // nullable: the any-redo word (clear: nothing to blend)
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

template <int IDT, int ODT, int M>
__global__ __launch_bounds__(kBlock) void slerp_blend_mm_kernel(Members mem, PopBlend pb, const uint64_t* chunks,
                                                                int64_t nchunks) {
    if (pb.any && *pb.any == 0) return;      // no child needs a SLERP-branch segment
    for_blend_ranges(chunks, nchunks, [&](uint64_t start, uint64_t end, uint64_t seg) {
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
            slerp_blend_mm_kernel<EDT_F32, EDT_F32, M><<<g, kBlock, 0, s>>>(mem, pb, chunk_desc, nchunks);   \
        else if (in_dt == EDT_F32)                                                                            \
            slerp_blend_mm_kernel<EDT_F32, EDT_BF16, M><<<g, kBlock, 0, s>>>(mem, pb, chunk_desc, nchunks);  \
        else if (out_dt == EDT_F32)                                                                           \
            slerp_blend_mm_kernel<EDT_BF16, EDT_F32, M><<<g, kBlock, 0, s>>>(mem, pb, chunk_desc, nchunks);  \
        else                                                                                                  \
            slerp_blend_mm_kernel<EDT_BF16, EDT_BF16, M><<<g, kBlock, 0, s>>>(mem, pb, chunk_desc, nchunks); \
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
    return pair_sums(v0, v1, in_dt, nullptr, EDT_F32, false, chunk_desc, nchunks, partial, nullptr, seg_ptrs,
                     (hipStream_t)stream);
}

int slerp_blend_impl(const void* v0, const void* v1, int in_dt, void* out, int out_dt, const uint64_t* chunk_desc,
                     int64_t nchunks, const float* coef, const uint64_t* seg_ptrs, void* stream, bool nt = true) {
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nchunks == 0) return EDT_OK;
    if (!chunk_desc || !coef) return fail(EDT_ERR_ARG, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    constexpr bool kNt = EDT_NT_SLERP != 0;
    const uint64_t units = (uint64_t)nchunks * (kTileSlots / kWavesPerBlock);
    for (uint64_t u0 = 0; u0 < units; u0 += kUnitGridCap) {
        const unsigned g = unit_grid(units - u0);
#define EDT_BT(I, O, N) slerp_blend_tile_kernel<I, O, N><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs, u0)
        if (in_dt == EDT_F32 && out_dt == EDT_F32) EDT_BT(EDT_F32, EDT_F32, false);
        else if (in_dt == EDT_F32) EDT_BT(EDT_F32, EDT_BF16, false);
        else if (out_dt == EDT_F32 && nt) EDT_BT(EDT_BF16, EDT_F32, kNt);
        else if (out_dt == EDT_F32) EDT_BT(EDT_BF16, EDT_F32, false);
        else if (nt) EDT_BT(EDT_BF16, EDT_BF16, kNt);
        else EDT_BT(EDT_BF16, EDT_BF16, false);
#undef EDT_BT
        int rc = check_launch("slerp_blend_tile_kernel");
        if (rc) return rc;
    }
    return EDT_OK;
}

// ---------------------------------------------------------------------------------------
// Reference-dot mode (opt-in): the reference's own fp32 dot of EDT_RL/crossover.py:20-29 restated
// bit for bit on the device (oracle/edt_oracle.c, pinned on numpy 2.2 / OpenBLAS 0.3.29 SkylakeX):
//   norm  = sqrt(sdot(v, v)): `threads` OpenBLAS level-1 chunks (ceil(rest / threads left)), each
//           64 fp32 FMA chains over 64-element blocks (chain L takes elements 64k + L), folded to
//           32, the 32-element remainder block, ((a0 + a1) + a2) + a3, the halves and two hadds,
//           then the < 32 tail in double; chunks added in order in double, rounded each time;
//   dot   = np.sum((v0 / n0) * (v1 / n1)): 8192-element buffers, each summed pairwise (blocks of
//           <= 128 with 8 accumulators, else halves cut at a multiple of 8), added in order to a
//           float starting at 0.
// The fp64 dot of the chunk sums stays the default; this mode replaces it where the caller's
// flags say so (e.g. segments whose fp64 dot lies near DOT_THRESHOLD, where the two can take
// different branches). The FMA chains are sequential by definition, so one workgroup streams a
// segment chunk through LDS to one compute wave: a parity mode, not a fast path.

constexpr int kRefThreads = 1024;                      // workgroup of the norm pass
constexpr int kRefPer = 16;                            // elements staged per thread per stage
constexpr int kRefStage = kRefThreads * kRefPer;       // 16,384 elements (64 KiB of fp32)
constexpr int kRefBuf = 8192;                          // numpy's ufunc buffer

// segment s of a chunk table: [start, end) (relative to the segment's buffers when seg_ptrs)
__device__ __forceinline__ void ref_segment(const uint64_t* chunks, const int32_t* first, int s, uint64_t& a,
                                            uint64_t& e) {
    const int c0 = first[s], c1 = first[s + 1];
    a = e = 0;
    if (c1 > c0) {
        a = chunks[3 * (uint64_t)c0];
        e = chunks[3 * (uint64_t)(c1 - 1)] + chunks[3 * (uint64_t)(c1 - 1) + 1];
    }
}

// OpenBLAS's level-1 split: chunk t of `threads` over n elements -> [off, off + len)
__device__ __forceinline__ void ref_split(uint64_t n, int threads, int t, uint64_t& off, uint64_t& len) {
    uint64_t rest = n;
    off = 0;
    len = 0;
    for (int c = 0; c <= t && rest > 0; ++c) {
        uint64_t w = (rest + (uint64_t)(threads - c) - 1) / (uint64_t)(threads - c);
        if (w > rest) w = rest;
        if (c == t) {
            len = w;
            return;
        }
        off += w;
        rest -= w;
    }
}

template <int IDT>
__device__ __forceinline__ float ref_load(const void* p, uint64_t i) {
    float x[1];
    ld<IDT, 1>(p, i, x);
    return x[0];
}

// Pass 1: block -> (segment s, vector w in {v0, v1}, thread chunk t); part[(2 s + w) threads + t] =
// that chunk's sdot(v, v) as OpenBLAS returns it to its combiner (double).
template <int IDT>
__global__ __launch_bounds__(kRefThreads) void refdot_norm_kernel(const void* v0, const void* v1,
                                                                  const uint64_t* chunks, const int32_t* first,
                                                                  int nseg, const int32_t* flag, int threads,
                                                                  const uint64_t* seg_ptrs, double* part) {
    const int s = (int)(blockIdx.x / (2u * (unsigned)threads));
    const int w = (int)((blockIdx.x / (unsigned)threads) % 2u);
    const int t = (int)(blockIdx.x % (unsigned)threads);
    if (s >= nseg || (flag && !flag[s])) return;
    uint64_t a, e;
    ref_segment(chunks, first, s, a, e);
    const void* v = w ? v1 : v0;
    if (seg_ptrs) v = reinterpret_cast<const void*>(seg_ptrs[3 * (uint64_t)s + w]);
    uint64_t off, len;
    ref_split(e - a, threads, t, off, len);
    const uint64_t base = a + off;
    const uint64_t n1 = len & ~(uint64_t)31, n64 = n1 & ~(uint64_t)63;
    __shared__ float buf[2][kRefStage];
    __shared__ float red[64];
    const int tid = threadIdx.x, lane = tid & 63;
    float acc = 0.f;                                     // wave 0: chain `lane`
    const uint64_t nst = (n64 + kRefStage - 1) / kRefStage;
    float r[kRefPer];
    auto fetch = [&](uint64_t st) {
#pragma unroll
        for (int q = 0; q < kRefPer; ++q) {
            const uint64_t i = st * kRefStage + (uint64_t)q * kRefThreads + (uint64_t)tid;
            r[q] = i < n64 ? ref_load<IDT>(v, base + i) : 0.f;
        }
    };
    auto put = [&](int b) {
#pragma unroll
        for (int q = 0; q < kRefPer; ++q) buf[b][q * kRefThreads + tid] = r[q];
    };
    if (nst > 0) {
        fetch(0);
        put(0);
    }
    __syncthreads();
    for (uint64_t st = 0; st < nst; ++st) {
        if (st + 1 < nst) fetch(st + 1);                 // the next stage's loads in flight ...
        if (tid < 64) {                                  // ... while wave 0 runs this stage's chains
            const uint64_t m = (n64 - st * kRefStage < (uint64_t)kRefStage ? n64 - st * kRefStage : kRefStage) / 64;
            const float* bb = buf[st & 1];
            for (uint64_t k = 0; k < m; ++k) {
                const float x = bb[k * 64 + lane];
                acc = __builtin_fmaf(x, x, acc);
            }
        }
        if (st + 1 < nst) put((int)((st + 1) & 1));      // buffer last read in stage st - 1
        __syncthreads();
    }
    if (tid < 64) red[lane] = acc;
    __syncthreads();
    if (tid == 0) {
        double d = 0.0;
        if (n1) {
            float a8[4][8];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int l = 0; l < 8; ++l) a8[j][l] = red[16 * j + l] + red[16 * j + l + 8];
            if (n1 > n64)                                // the 32-element remainder block
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int l = 0; l < 8; ++l) {
                        const float x = ref_load<IDT>(v, base + n64 + 8 * j + l);
                        a8[j][l] = __builtin_fmaf(x, x, a8[j][l]);
                    }
            float sl[8], h[4];
#pragma unroll
            for (int l = 0; l < 8; ++l) sl[l] = ((a8[0][l] + a8[1][l]) + a8[2][l]) + a8[3][l];
#pragma unroll
            for (int l = 0; l < 4; ++l) h[l] = sl[l] + sl[l + 4];
            d = (double)((h[0] + h[1]) + (h[2] + h[3]));
        }
        for (uint64_t i = n1; i < len; ++i) {
            const float x = ref_load<IDT>(v, base + i);
            d += (double)(x * x);
        }
        part[(2 * (uint64_t)s + w) * (uint64_t)threads + t] = d;
    }
}

// IEEE sqrt rounded to nearest (numpy's float32 sqrt). This toolchain emits sqrtf as the bare
// hardware v_sqrt_f32 (not correctly rounded), so the result is moved to the nearest float by
// comparing x with the squared midpoints to its neighbours, exactly, in double (a midpoint has 25
// significant bits, its square 50). Checked on the host against sqrtf for starts up to 2 ulps off
// over the whole positive float range.
__device__ __forceinline__ float sqrt_rn(float x) {
    if (!(x > 0.f) || x == __builtin_inff()) return __builtin_sqrtf(x);
    float r = __builtin_sqrtf(x);
    const double xd = x;
    for (int it = 0; it < 2; ++it) {
        const float up = __uint_as_float(__float_as_uint(r) + 1u), dn = __uint_as_float(__float_as_uint(r) - 1u);
        const double hi = ((double)r + (double)up) * 0.5, lo = ((double)r + (double)dn) * 0.5;
        if (xd > hi * hi) r = up;
        else if (xd < lo * lo) r = dn;
        else break;
    }
    return r;
}

// The norm of (segment s, vector w) from the chunk results, as np.linalg.norm returns it.
__device__ __forceinline__ float ref_norm(const double* part, int s, int w, int threads) {
    const double* p = part + (2 * (uint64_t)s + w) * (uint64_t)threads;
    float dot;
    if (threads <= 1) {
        dot = (float)p[0];
    } else {
        dot = 0.f;
        for (int t = 0; t < threads; ++t) dot = (float)((double)dot + p[t]);
    }
    return sqrt_rn(dot);
}

template <int IDT>
struct RefProd {                                         // element i of (v0 / n0) * (v1 / n1)
    const void* a;
    const void* b;
    float n0, n1;
    bool d0, d1;                                         // normalize() divides only if norm > eps
    __device__ __forceinline__ float operator()(uint64_t i) const {
        float x = ref_load<IDT>(a, i), y = ref_load<IDT>(b, i);
        if (d0) x = __fdiv_rn(x, n0);
        if (d1) y = __fdiv_rn(y, n1);
        return x * y;
    }
};

template <typename P>
__device__ __forceinline__ float np_leaf(const P& p, uint64_t o, uint64_t n) {
    if (n < 8) {
        float r = 0.f;
        for (uint64_t i = 0; i < n; ++i) r += p(o + i);
        return r;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = p(o + j);
    uint64_t i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += p(o + i + j);
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += p(o + i);
    return res;
}

// numpy's pairwise_sum over [o, o + n), n <= 8192, on one lane (explicit stack, depth <= 7).
template <typename P>
__device__ float np_pairwise_serial(const P& p, uint64_t o, uint64_t n) {
    uint64_t so[12], sn[12];
    float sl[12];
    int stage[12];
    int sp = 0;
    so[0] = o;
    sn[0] = n;
    stage[0] = 0;
    float ret = 0.f;
    for (;;) {
        const uint64_t fo = so[sp], fn = sn[sp];
        uint64_t h = fn / 2;
        h -= h % 8;
        bool done = false;
        if (stage[sp] == 0) {
            if (fn <= 128) {
                ret = np_leaf(p, fo, fn);
                done = true;
            } else {
                stage[sp] = 1;
                so[sp + 1] = fo;
                sn[sp + 1] = h;
                stage[sp + 1] = 0;
                ++sp;
            }
        } else if (stage[sp] == 1) {
            sl[sp] = ret;
            stage[sp] = 2;
            so[sp + 1] = fo + h;
            sn[sp + 1] = fn - h;
            stage[sp + 1] = 0;
            ++sp;
        } else {
            ret = sl[sp] + ret;
            done = true;
        }
        if (done) {
            if (sp == 0) return ret;
            --sp;
        }
    }
}

// Pass 2: one wave per 8192-element buffer of a flagged segment (buffer q of chunk c; chunks are
// whole multiples of it inside their segment): a full buffer is numpy's perfect pairwise tree —
// lane L the 128-element leaf L, the xor butterfly the levels above it in order — a partial one
// (the segment's last) runs the recursion on lane 0. bsum[c * bpc + q] = the buffer's sum.
template <int IDT>
__global__ __launch_bounds__(kBlock) void refdot_sum_kernel(const void* v0, const void* v1, const uint64_t* chunks,
                                                            int64_t nchunks, const int32_t* first, const int32_t* flag,
                                                            int threads, float eps, const uint64_t* seg_ptrs,
                                                            const double* part, int bpc, float* bsum) {
    const uint64_t u = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (u >= (uint64_t)nchunks * (uint64_t)bpc) return;
    const uint64_t c = u / (uint64_t)bpc, q = u % (uint64_t)bpc;
    const int s = (int)chunks[3 * c + 2];
    if (flag && !flag[s]) return;
    const uint64_t cs = chunks[3 * c], cl = chunks[3 * c + 1];
    if (q * kRefBuf >= cl) return;
    const uint64_t o = cs + q * kRefBuf;
    const uint64_t n = cl - q * kRefBuf < (uint64_t)kRefBuf ? cl - q * kRefBuf : (uint64_t)kRefBuf;
    RefProd<IDT> p;
    p.a = seg_ptrs ? reinterpret_cast<const void*>(seg_ptrs[3 * (uint64_t)s]) : v0;
    p.b = seg_ptrs ? reinterpret_cast<const void*>(seg_ptrs[3 * (uint64_t)s + 1]) : v1;
    p.n0 = ref_norm(part, s, 0, threads);
    p.n1 = ref_norm(part, s, 1, threads);
    p.d0 = p.n0 > eps;
    p.d1 = p.n1 > eps;
    if (n == (uint64_t)kRefBuf) {
        float x = np_leaf(p, o + 128 * (uint64_t)lane, 128);
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) x += __shfl_xor(x, m, 64);
        if (lane == 0) bsum[u] = x;
    } else if (lane == 0) {
        bsum[u] = np_pairwise_serial(p, o, n);
    }
}

// Pass 3: per flagged segment, the buffers' sums added in order to a float starting at 0.
__global__ __launch_bounds__(kBlock) void refdot_total_kernel(const uint64_t* chunks, const int32_t* first, int nseg,
                                                              const int32_t* flag, int bpc, const float* bsum,
                                                              float* ref_dot) {
    const int s = (int)(blockIdx.x * kBlock + threadIdx.x);
    if (s >= nseg || (flag && !flag[s])) return;
    float r = 0.f;
    for (int c = first[s]; c < first[s + 1]; ++c) {
        const uint64_t cl = chunks[3 * (uint64_t)c + 1];
        for (int q = 0; q < bpc && (uint64_t)q * kRefBuf < cl; ++q) r += bsum[(uint64_t)c * bpc + q];
    }
    ref_dot[s] = r;
}

// Flags: segments whose dot lies within `band` of the threshold (|dot| in [thr - band, thr + band]);
// band < 0: every segment.
__global__ __launch_bounds__(kBlock) void refdot_flag_kernel(const float* dots, int nseg, float thr, float band,
                                                             int32_t* flag) {
    const int s = (int)(blockIdx.x * kBlock + threadIdx.x);
    if (s >= nseg) return;
    flag[s] = band < 0.f || fabsf(fabsf(dots[s]) - thr) <= band ? 1 : 0;
}

// Coefficients of the flagged segments from the reference dot (slerp_coefficients' scalar math).
__global__ __launch_bounds__(kBlock) void refdot_coef_kernel(const float* ref_dot, const int32_t* flag, int nseg,
                                                             const double* tvals, float thr, float* coef,
                                                             float* dot_out) {
    const int s = (int)(blockIdx.x * kBlock + threadIdx.x);
    if (s >= nseg || (flag && !flag[s])) return;
    const float dot = ref_dot[s];
    float c0, c1;
    coefficients_from_dot(dot, tvals[s], thr, c0, c1);
    coef[2 * s] = c0;
    coef[2 * s + 1] = c1;
    if (dot_out) dot_out[s] = dot;
}

}  // namespace

extern "C" {

int64_t edt_slerp_make_chunks(const uint64_t* seg_offsets, int nseg, uint32_t chunk_elems,
                              uint64_t* chunk_desc, int64_t max_chunks, int32_t* seg_first_chunk) {
    g_err[0] = 0;
    if (nseg < 0 || !seg_offsets || chunk_elems == 0) return fail(EDT_ERR_ARG, "bad segment table");
    if (chunk_elems > kMaxChunkElems)       // the sums' canonical tree spans 128 tiles of 512
        return fail(EDT_ERR_ARG, "chunk_elems %u above %u", chunk_elems, kMaxChunkElems);
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

uint64_t edt_slerp_sums_doubles(int width, int64_t nchunks) {
    // the chunk rows + the largest row scratch a pass writes for this width: level-0 rows (one per
    // tile) for the pair passes (width 3), level-4 rows for the Gram passes
    // (width 3: plus one double at the end, the speculative pass's any-redo flag)
    if (width < 1 || nchunks < 0) return 0;
    const uint64_t rows = width <= 3 ? kPairRows : kGramRows;
    return (uint64_t)nchunks * (uint64_t)width * (1ull + rows) + (width <= 3 ? 1 : 0);
}

uint64_t edt_slerp_population_speculative_doubles(int npairs, int64_t nchunks) {
    if (npairs < 0 || nchunks < 0) return 0;
    // each child's chunk rows + its row scratch (level-0 rows), + the any-redo word
    return (uint64_t)nchunks * 3ull * (uint64_t)npairs * (1ull + kPairRows) + 1;
}

uint64_t edt_slerp_population_gram_doubles(int nmembers, int64_t nchunks) {
    if (nmembers < 1 || nmembers > kGramMaxMembers || nchunks < 0) return 0;
    return edt_slerp_sums_doubles(nmembers * (nmembers + 1) / 2, nchunks);
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
    // the sums per component of the pair graph (GramPlan): the needed layout where it applies
    // (r5); the chunk rows of every component first, one shared level-4 row scratch after them
    // (each component's pass has finished with it before the next one starts: one stream)
    GramPlan G;
    int rc = EDT_OK;
    {
        std::vector<int> A(npairs), B(npairs);
        for (int q = 0; q < npairs; ++q) { A[q] = compact[pairs[2 * q]]; B[q] = compact[pairs[2 * q + 1]]; }
        plan_gram(D, A.data(), B.data(), npairs, nchunks, G);
    }
    uint64_t scratch = 0;
    for (int k = 0; k < G.ncomp; ++k) scratch += (uint64_t)nchunks * G.nt(k);
    for (int k = 0; k < G.ncomp; ++k) {
        rc = plan_component_sums(G, k, mem.p, in_dt, chunk_desc, nchunks, gram, gram + scratch, s);
        if (rc) return rc;
    }
    const unsigned gc = coef_grid(nseg);
    for (int q = 0; q < npairs; ++q) {
        const int i = compact[pairs[2 * q]], j = compact[pairs[2 * q + 1]];
        const int k = G.comp_of[i];                   // i and j share a component
        slerp_gram_coef_kernel<<<gc, kBlock, 0, s>>>(gram + G.off[k], G.nt(k), G.norm_index(i), G.norm_index(j),
                                                     G.dot_index(i, j), seg_first_chunk, nseg, t,
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
        rc = colocated_launches((uint64_t)nchunks, B.nchildren, [&](uint64_t c0, unsigned gb) {
            if (in_dt == EDT_F32 && out_dt == EDT_F32)
                slerp_blend_population_kernel<EDT_F32, EDT_F32><<<gb, kBlock, 0, s>>>(B, chunk_desc, nchunks, c0);
            else if (in_dt == EDT_F32)
                slerp_blend_population_kernel<EDT_F32, EDT_BF16><<<gb, kBlock, 0, s>>>(B, chunk_desc, nchunks, c0);
            else if (out_dt == EDT_F32)
                slerp_blend_population_kernel<EDT_BF16, EDT_F32><<<gb, kBlock, 0, s>>>(B, chunk_desc, nchunks, c0);
            else
                slerp_blend_population_kernel<EDT_BF16, EDT_BF16><<<gb, kBlock, 0, s>>>(B, chunk_desc, nchunks, c0);
        });
        if (rc) return rc;
    }
    return EDT_OK;
}

// ---- the member-major blends of edt_slerp_population as a separate entry (the link-balanced
// sharded population, distributed.ShardedPopulationCrossover: the blends of a rank's chunk range
// after the needed sums' table rows were all-gathered; the sums and coefficients are
// edt_slerp_needed_sums / _coef below) ----

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
    // the any-redo flag: the last double of the workspace (edt_slerp_sums_doubles), zeroed by the
    // first pass, set by the coefficient kernel when some segment takes the SLERP branch
    int32_t* any = reinterpret_cast<int32_t*>(partial + edt_slerp_sums_doubles(3, nchunks) - 1);
    int rc = pair_sums(v0, v1, in_dt, out, out_dt, true, chunk_desc, nchunks, partial, t, nullptr, s, any);
    if (rc) return rc;
    slerp_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(partial, seg_first_chunk, nseg, t, (float)dot_threshold,
                                                         (float)eps, coef, dot_out, redo, any);
    rc = check_launch("slerp_coef_kernel");
    if (rc) return rc;
    // the redo blends: grid-stride over chunks (most segments are skipped)
    const unsigned g = slerp_spec_grid(nchunks);
    constexpr bool kNtB = EDT_NT_SLERP != 0;
    if (in_dt == EDT_F32 && out_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_F32, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo, any);
    else if (in_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_BF16, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo, any);
    else if (out_dt == EDT_F32)
        slerp_blend_kernel<EDT_BF16, EDT_F32, kNtB><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo, any);
    else
        slerp_blend_kernel<EDT_BF16, EDT_BF16, kNtB><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, nullptr, redo, any);
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
    // the any-redo word (the workspace's last double): zeroed by the first pass, set by any child's
    // coefficient kernel that sends a segment to the SLERP branch; clear, the redo grid exits at once
    int32_t* any = reinterpret_cast<int32_t*>(partial + edt_slerp_population_speculative_doubles(npairs, nchunks) - 1);
    // member-major form (r5: the needed layout; r4: the ring, EDT_POP_LAYOUT=ring): per component of
    // the children's pair graph one pass reads each of its parents once, forms the component's
    // needed sums (its norms + the dots its children use) AND writes every child's lerp-branch
    // output from the members' registers (each distinct ordered pair computed once, stored to
    // every child of it); then the children's coefficients from those sums and one member-major
    // redo blend per component (which exits at once when no segment of any child needs the SLERP
    // branch). Any pair graph over <= 8 distinct parents whose components fit their dot slots
    // (every graph of <= 8 children) takes it; others the co-located pass below.
    {
        std::vector<int> compact(nmembers, -1), A(npairs), B(npairs);
        const void* dm[kGramMaxMembers];
        int D = 0;
        bool fits = npairs <= kBlendMaxChildren;
        for (int q = 0; q < npairs && fits; ++q)
            for (int e = 0; e < 2 && fits; ++e) {
                const int m = pairs[2 * q + e];
                if (compact[m] < 0) {
                    if (D == kGramMaxMembers) { fits = false; break; }
                    compact[m] = D;
                    dm[D++] = members[m];
                }
                (e ? B : A)[q] = compact[m];
            }
        GramPlan G;
        if (fits) {
            plan_gram(D, A.data(), B.data(), npairs, nchunks, G);
            for (int k = 0; k < G.ncomp && fits; ++k) fits = G.kind[k] == kNeed;
        }
        if (fits) {                                     // each child onto its component's emit table
            for (int q = 0; q < npairs && fits; ++q) {
                const int k = G.comp_of[A[q]], n = G.size[k];
                NeedSpec& S = G.need[k];
                const int pa = G.pos[A[q]], pb = G.pos[B[q]];
                int slot = -1;
                void** first = nullptr;
                uint32_t* bits = nullptr;
                if (pa != pb && pb == (pa + 1) % n && (n >= 3 || pa == 0)) {
                    slot = pa;
                    bits = &S.fwd;
                    first = &S.out_fwd[pa];
                } else if (pa != pb && pa == (pb + 1) % n && (n >= 3 || pb == 0)) {
                    slot = 8 + pb;
                    bits = &S.rev;
                    first = &S.out_rev[pb];
                }
                if (bits) {
                    const uint32_t bit = 1u << (slot & 7);
                    if (!(*bits & bit)) {
                        *bits |= bit;
                        *first = outs[q];
                        continue;
                    }
                } else {                                // a chord or a self-pair: a picked pair
                    int e = 0;
                    while (e < S.nemit && !(S.ea[e] == pa && S.eb[e] == pb)) ++e;
                    if (e == S.nemit) {
                        if (e == kNeedChordEmits) { fits = false; break; }
                        S.ea[e] = pa;
                        S.eb[e] = pb;
                        S.out[e] = outs[q];
                        ++S.nemit;
                        continue;
                    }
                    slot = 16 + e;
                }
                if (S.nextra == kNeedMaxOut) { fits = false; break; }   // a duplicate: same registers
                S.xslot[S.nextra] = slot;
                S.xout[S.nextra++] = outs[q];
            }
            for (int k = 0; k < G.ncomp; ++k) G.need[k].t = t;
        }
        if (fits) {
            uint64_t scratch = 0;
            for (int k = 0; k < G.ncomp; ++k) scratch += (uint64_t)nchunks * G.nt(k);
            Members gm[kGramMaxMembers];
            for (int k = 0; k < G.ncomp; ++k) {           // the passes first: only the first zeroes `any`
                memset(&gm[k], 0, sizeof(Members));
                for (int x = 0; x < G.size[k]; ++x) gm[k].p[x] = dm[G.list[k][x]];
                G.need[k].zero_word = k == 0 ? any : nullptr;
                int rc = need_sums(gm[k], G.size[k], G.need[k], in_dt, out_dt, true, chunk_desc, nchunks,
                                   partial + G.off[k], partial + scratch, s);
                if (rc) return rc;
            }
            for (int q = 0; q < npairs; ++q) {
                const int k = G.comp_of[A[q]];
                const int qd = G.dot_index(A[q], B[q]);
                slerp_gram_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(
                    partial + G.off[k], G.nt(k), G.norm_index(A[q]), G.norm_index(B[q]), qd, seg_first_chunk, nseg, t,
                    (float)dot_threshold, (float)eps, coef + 2 * (size_t)nseg * q,
                    dot_out ? dot_out + (size_t)nseg * q : nullptr, redo + (size_t)nseg * q, any);
                int rc = check_launch("slerp_gram_coef_kernel");
                if (rc) return rc;
            }
            for (int k = 0; k < G.ncomp; ++k) {
                PopBlend pb;
                memset(&pb, 0, sizeof(pb));
                pb.any = any;
                for (int q = 0; q < npairs; ++q) {
                    if (G.comp_of[A[q]] != k) continue;
                    pb.out[pb.n] = outs[q];
                    pb.coef[pb.n] = coef + 2 * (size_t)nseg * q;
                    pb.redo[pb.n] = redo + (size_t)nseg * q;
                    pb.a[pb.n] = G.pos[A[q]];
                    pb.b[pb.n] = G.pos[B[q]];
                    ++pb.n;
                }
                int rc = launch_blend_mm(gm[k], G.size[k], pb, in_dt, out_dt, chunk_desc, nchunks, s);
                if (rc) return rc;
            }
            return EDT_OK;
        }
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
                B.slots[k] = partial + 3 * (size_t)nchunks * npairs + 3 * (size_t)kPairRows * nchunks * q;
            }
            // pass 0: one block per (unit = 4 tiles of a chunk, child); pass 1: per (chunk, child)
            const uint64_t units = pass == 0 ? (uint64_t)nchunks * (kTileSlots / 4) : (uint64_t)nchunks;
#define EDT_SPEC_POP(KERNEL, ...)                                                                   \
    do {                                                                                            \
        if (in_dt == EDT_F32 && out_dt == EDT_F32) KERNEL<EDT_F32, EDT_F32><<<gb, kBlock, 0, s>>>(__VA_ARGS__);   \
        else if (in_dt == EDT_F32) KERNEL<EDT_F32, EDT_BF16><<<gb, kBlock, 0, s>>>(__VA_ARGS__);                  \
        else if (out_dt == EDT_F32) KERNEL<EDT_BF16, EDT_F32><<<gb, kBlock, 0, s>>>(__VA_ARGS__);                 \
        else KERNEL<EDT_BF16, EDT_BF16><<<gb, kBlock, 0, s>>>(__VA_ARGS__);                                       \
    } while (0)
            int rc = colocated_launches(units, B.nchildren, [&](uint64_t u0, unsigned gb) {
                if (pass == 0) EDT_SPEC_POP(slerp_pop_stats_lerp_kernel, B, chunk_desc, nchunks, t, u0, any);
                else EDT_SPEC_POP(slerp_blend_population_kernel, B, chunk_desc, nchunks, u0, any);
            });
#undef EDT_SPEC_POP
            if (rc) return rc;
        }
        if (pass == 0) {
            for (int q = 0; q < npairs; ++q) {
                int rc = launch_tree_reduce(partial + 3 * (size_t)nchunks * npairs + 3 * (size_t)kPairRows * nchunks * q, 3,
                                            kSpecWgRows ? kTileSlots / 4 : kPairRows, kTileSlots / 4,
                                            kSpecWgRows ? 1 : kWavesPerBlock, nchunks,
                                            partial + 3 * (size_t)nchunks * q, s);
                if (rc) return rc;
                slerp_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(
                    partial + 3 * (size_t)nchunks * q, seg_first_chunk, nseg, t, (float)dot_threshold, (float)eps,
                    coef + 2 * (size_t)nseg * q, dot_out ? dot_out + (size_t)nseg * q : nullptr, redo + (size_t)nseg * q,
                    any);
                rc = check_launch("slerp_coef_kernel");
                if (rc) return rc;
            }
        }
    }
    return EDT_OK;
}

// ---- the needed-sums passes as separate entries (r5: the sharded population,
// distributed.ShardedPopulationCrossover — each rank forms the needed sums of its chunk range,
// the table's rows are all-gathered, every rank forms every child's coefficients) ----

namespace {
// The distinct parents of `pairs` in first-use order (compact ids) and the GramPlan of the pair
// graph: the same planning as edt_slerp_population, so a table row equals that pass's sums.
struct NeededPlan {
    int D = 0;
    int orig[kGramMaxMembers];                 // compact -> member index
    std::vector<int> A, B;                     // children's compact parents
    GramPlan G;
};

int needed_plan(const int32_t* pairs, int npairs, int nmembers, int64_t nchunks, NeededPlan& P) {
    if (nmembers < 1 || nmembers > kGramMaxMembers)
        return fail(EDT_ERR_ARG, "member count %d out of range [1, %d]", nmembers, kGramMaxMembers);
    if (npairs < 1 || !pairs) return fail(EDT_ERR_ARG, "no pairs");
    if (nchunks < 0) return fail(EDT_ERR_ARG, "negative chunk count");
    int compact[kGramMaxMembers];
    for (int m = 0; m < nmembers; ++m) compact[m] = -1;
    P.A.assign(npairs, 0);
    P.B.assign(npairs, 0);
    for (int q = 0; q < npairs; ++q)
        for (int e = 0; e < 2; ++e) {
            const int m = pairs[2 * q + e];
            if (m < 0 || m >= nmembers) return fail(EDT_ERR_ARG, "pair %d: member out of range", q);
            if (compact[m] < 0) {
                compact[m] = P.D;
                P.orig[P.D++] = m;
            }
            (e ? P.B : P.A)[q] = compact[m];
        }
    plan_gram(P.D, P.A.data(), P.B.data(), npairs, nchunks, P.G);
    return EDT_OK;
}

// the two members (member indices) each column of block k holds the sum of
void needed_columns(const NeededPlan& P, int k, int32_t* cols) {
    const GramPlan& G = P.G;
    const int M = G.size[k];
    const int* L = G.list[k];
    if (G.kind[k] == kTri) {                           // dots no child uses are not formed
        for (int i = 0; i < M; ++i)
            for (int j = i; j < M; ++j) {
                const int c = tri_index(i, j, M);
                const bool used = i == j || ((G.need[k].tri >> c) & 1u);
                cols[2 * c] = used ? P.orig[L[i]] : -1;
                cols[2 * c + 1] = used ? P.orig[L[j]] : -1;
            }
        return;
    }
    int c = 0;
    for (int x = 0; x < M; ++x, ++c) { cols[2 * c] = P.orig[L[x]]; cols[2 * c + 1] = P.orig[L[x]]; }
    for (int e = 0; e < need_nr(M); ++e, ++c) { cols[2 * c] = P.orig[L[e]]; cols[2 * c + 1] = P.orig[L[(e + 1) % M]]; }
    for (int e = 0; e < need_nc(M); ++e, ++c) {
        if (e < G.need[k].nchord) {
            const int code = G.need[k].code[e];
            cols[2 * c] = P.orig[L[code / 8]];
            cols[2 * c + 1] = P.orig[L[code % 8]];
        } else {                                       // an unused chord slot (its sum is not formed)
            cols[2 * c] = cols[2 * c + 1] = -1;
        }
    }
}
}   // namespace

int edt_slerp_needed_table(const int32_t* pairs, int npairs, int nmembers, int64_t nchunks, uint64_t* block_off,
                           int32_t* block_nt, int32_t* ncomp, int32_t* col_members, uint64_t* table_doubles,
                           uint64_t* scratch_doubles) {
    g_err[0] = 0;
    if (!block_off || !block_nt || !ncomp || !table_doubles || !scratch_doubles) return fail(EDT_ERR_ARG, "null output");
    NeededPlan P;
    int rc = needed_plan(pairs, npairs, nmembers, nchunks, P);
    if (rc) return rc;
    *ncomp = P.G.ncomp;
    uint64_t tot = 0;
    int col = 0;
    for (int k = 0; k < P.G.ncomp; ++k) {
        block_off[k] = P.G.off[k];
        block_nt[k] = P.G.nt(k);
        tot += (uint64_t)nchunks * P.G.nt(k);
        if (col_members) needed_columns(P, k, col_members + 2 * col);
        col += P.G.nt(k);
    }
    *table_doubles = tot;
    *scratch_doubles = plan_row_scratch(P.G, nchunks);
    return EDT_OK;
}

int edt_slerp_needed_sums(const void* const* members, int nmembers, int in_dt, const int32_t* pairs, int npairs,
                          const uint64_t* chunk_desc, int64_t nchunks, int64_t table_chunks, int64_t row0,
                          double* table, double* scratch, uint64_t scratch_doubles, void* stream) {
    g_err[0] = 0;
    if (in_dt & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    NeededPlan P;
    int rc = needed_plan(pairs, npairs, nmembers, table_chunks, P);
    if (rc) return rc;
    if (nchunks < 0 || row0 < 0 || row0 + nchunks > table_chunks)
        return fail(EDT_ERR_ARG, "rows [%lld, %lld) outside the table's %lld chunks", (long long)row0,
                    (long long)(row0 + nchunks), (long long)table_chunks);
    if (nchunks == 0) return EDT_OK;
    if (!members || !chunk_desc || !table || !scratch) return fail(EDT_ERR_ARG, "null buffer");
    if (scratch_doubles < plan_row_scratch(P.G, nchunks))
        return fail(EDT_ERR_ARG, "scratch of %llu doubles, the passes need %llu", (unsigned long long)scratch_doubles,
                    (unsigned long long)plan_row_scratch(P.G, nchunks));
    Members mem;
    memset(&mem, 0, sizeof(mem));
    for (int d = 0; d < P.D; ++d) {
        const void* m = members[P.orig[d]];
        if (!m || !aligned16(m)) return fail(EDT_ERR_ARG, "member %d is null or not 16-byte aligned", P.orig[d]);
        mem.p[d] = m;
    }
    for (int k = 0; k < P.G.ncomp; ++k) {
        // rows [row0, row0 + nchunks) of the component's block (plan_component_sums adds the
        // block's offset)
        rc = plan_component_sums(P.G, k, mem.p, in_dt, chunk_desc, nchunks, table + (uint64_t)row0 * P.G.nt(k),
                                 scratch, (hipStream_t)stream);
        if (rc) return rc;
    }
    return EDT_OK;
}

int edt_slerp_needed_coef(const double* table, int64_t table_chunks, const int32_t* pairs, int npairs, int nmembers,
                          const int32_t* seg_first_chunk, int nseg, const double* t, double dot_threshold, double eps,
                          float* coef, float* dot_out, void* stream) {
    g_err[0] = 0;
    NeededPlan P;
    int rc = needed_plan(pairs, npairs, nmembers, table_chunks, P);
    if (rc) return rc;
    if (nseg < 0) return fail(EDT_ERR_ARG, "negative count");
    if (nseg == 0) return EDT_OK;
    if (!table || !seg_first_chunk || !t || !coef) return fail(EDT_ERR_ARG, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    for (int q = 0; q < npairs; ++q) {
        const int i = P.A[q], j = P.B[q];
        const int k = P.G.comp_of[i];
        slerp_gram_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(
            table + P.G.off[k], P.G.nt(k), P.G.norm_index(i), P.G.norm_index(j), P.G.dot_index(i, j), seg_first_chunk,
            nseg, t, (float)dot_threshold, (float)eps, coef + 2 * (size_t)nseg * q,
            dot_out ? dot_out + (size_t)nseg * q : nullptr);
        rc = check_launch("slerp_gram_coef_kernel");
        if (rc) return rc;
    }
    return EDT_OK;
}

int edt_slerp_population_layout(const int32_t* pairs, int npairs, int nmembers, int speculate, char* buf,
                                int buflen) {
    // the plan edt_slerp_population(_speculative) makes for these pairs, as JSON (host only)
    g_err[0] = 0;
    if (!buf || buflen < 2) return fail(EDT_ERR_ARG, "null or short buffer");
    if (npairs < 0 || nmembers < 1) return fail(EDT_ERR_ARG, "bad count");
    if (npairs > 0 && !pairs) return fail(EDT_ERR_ARG, "null pairs");
    std::vector<int> compact(nmembers, -1), orig, A(npairs), B(npairs);
    for (int q = 0; q < npairs; ++q)
        for (int e = 0; e < 2; ++e) {
            const int m = pairs[2 * q + e];
            if (m < 0 || m >= nmembers) return fail(EDT_ERR_ARG, "pair %d: member out of range", q);
            if (compact[m] < 0) {
                compact[m] = (int)orig.size();
                orig.push_back(m);
            }
            (e ? B : A)[q] = compact[m];
        }
    const int D = (int)orig.size();
    std::string js = "{\"distinct_parents\": " + std::to_string(D) + ", \"children\": " + std::to_string(npairs);
    if (D > kGramMaxMembers) {
        js += std::string(", \"form\": \"") + (speculate ? "co-located" : "unsupported") + "\", \"components\": []}";
    } else {
        GramPlan G;
        plan_gram(D, A.data(), B.data(), npairs, 1, G);
        bool mm = npairs <= kBlendMaxChildren;
        std::string comps;
        for (int k = 0; k < G.ncomp; ++k) {
            const int n = G.size[k];
            int nemit = 0, picked = 0, ea[64], eb[64];
            for (int q = 0; q < npairs; ++q) {        // distinct ordered pairs; those off the ring
                if (G.comp_of[A[q]] != k) continue;
                int e = 0;
                while (e < nemit && !(ea[e] == A[q] && eb[e] == B[q])) ++e;
                if (e < nemit || nemit == 64) continue;
                ea[nemit] = A[q];
                eb[nemit++] = B[q];
                const int pa = G.pos[A[q]], pb = G.pos[B[q]];
                picked += !(G.kind[k] == kNeed && pa != pb && GramPlan::ring_edge(pa, pb, n) >= 0);
            }
            int dupes = 0;
            for (int q = 0; q < npairs; ++q) dupes += G.comp_of[A[q]] == k;
            dupes -= nemit;
            mm = mm && G.kind[k] == kNeed && picked <= kNeedChordEmits && dupes <= kNeedMaxOut;
            int ndots = 0;
            for (int q = 0; q < npairs; ++q) {     // distinct unordered dots of the component
                if (G.comp_of[A[q]] != k || A[q] == B[q]) continue;
                bool seen = false;
                for (int r = 0; r < q; ++r)
                    seen = seen || (G.comp_of[A[r]] == k && ((A[r] == A[q] && B[r] == B[q]) || (A[r] == B[q] && B[r] == A[q])));
                ndots += !seen;
            }
            std::string mem;
            for (int x = 0; x < G.size[k]; ++x) mem += (x ? ", " : "") + std::to_string(orig[G.list[k][x]]);
            const char* kind = G.kind[k] == kNeed ? "needed" : "triangle";
            const int chords = G.kind[k] == kNeed ? G.need[k].nchord : 0;
            comps += std::string(k ? ", " : "") + "{\"members\": [" + mem + "], \"dots\": " + std::to_string(ndots) +
                     ", \"chords\": " + std::to_string(chords) + ", \"sums\": " + std::to_string(G.nt(k)) +
                     ", \"stats_layout\": \"" + kind + "\", \"emit_pairs\": " + std::to_string(nemit) +
                     ", \"picked_pairs\": " + std::to_string(picked) + "}";
        }
        const char* form = speculate ? (mm ? "member-major" : "co-located") : "two-pass";
        js += std::string(", \"form\": \"") + form + "\", \"components\": [" + comps + "]}";
    }
    if ((int)js.size() + 1 > buflen) return fail(EDT_ERR_ARG, "buffer of %d bytes too short (%d)", buflen, (int)js.size() + 1);
    memcpy(buf, js.c_str(), js.size() + 1);
    return EDT_OK;
}

}   // extern "C"

static int seg_table_impl(const void* const* v0_t, const void* const* v1_t, void* const* out_t, int nseg,
                          const uint64_t* seg_numel, int in_dt, int out_dt, int apart, uint64_t* table_host);

namespace {
// The tensor-list forms: segment s is its own tensor triple {v0, v1, out}, read through a DEVICE
// table of 3 x nseg uint64 pointers (edt_slerp_seg_table validates and writes its host image; the
// caller uploads it once and reuses it while the tensors stay where they are).

struct Span {
    uintptr_t a, e;
    bool out;
};

// No output span overlaps a parent span: spans sorted by start, each checked against the
// furthest end of the other kind before it (empty spans ignored).
bool spans_apart(std::vector<Span>& sp) {
    std::sort(sp.begin(), sp.end(), [](const Span& x, const Span& y) { return x.a < y.a; });
    uintptr_t far_in = 0, far_out = 0;
    for (const Span& x : sp) {
        if (x.out ? x.a < far_in : x.a < far_out) return false;
        uintptr_t& f = x.out ? far_out : far_in;
        if (x.e > f) f = x.e;
    }
    return true;
}

// the redo blends / any table blend with a redo mask: grid-stride over chunks (most are skipped)
int blend_redo(const void* v0, const void* v1, int in_dt, void* out, int out_dt, const uint64_t* chunk_desc,
               int64_t nchunks, const float* coef, const uint64_t* seg_ptrs, const int32_t* redo,
               const int32_t* any, hipStream_t s) {
    const unsigned g = slerp_spec_grid(nchunks);
    constexpr bool kNtB = EDT_NT_SLERP != 0;
    if (in_dt == EDT_F32 && out_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_F32, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs, redo, any);
    else if (in_dt == EDT_F32)
        slerp_blend_kernel<EDT_F32, EDT_BF16, false><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs, redo, any);
    else if (out_dt == EDT_F32)
        slerp_blend_kernel<EDT_BF16, EDT_F32, kNtB><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs, redo, any);
    else
        slerp_blend_kernel<EDT_BF16, EDT_BF16, kNtB><<<g, kBlock, 0, s>>>(v0, v1, out, chunk_desc, nchunks, coef, seg_ptrs, redo, any);
    return check_launch("slerp_blend_kernel");
}

int table_args(const uint64_t* table, int in_dt, int out_dt, int64_t nchunks, int nseg) {
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nseg < 0 || nchunks < 0) return fail(EDT_ERR_ARG, "negative count (segments %d, chunks %lld)", nseg, (long long)nchunks);
    if (nchunks > 0 && !table) return fail(EDT_ERR_ARG, "null tensor table");
    if (reinterpret_cast<uintptr_t>(table) & 7u) return fail(EDT_ERR_ARG, "tensor table must be 8-byte aligned");
    return EDT_OK;
}

// the pointer-array entries: validate, then upload the table into `workspace` by a stream-ordered
// copy (pageable source: staged before hipMemcpyAsync returns)
int upload_seg_table(const void* const* v0_t, const void* const* v1_t, void* const* out_t, int nseg,
                     const uint64_t* seg_numel, int in_dt, int out_dt, int apart, void* workspace,
                     uint64_t workspace_bytes, hipStream_t s) {
    const uint64_t need = 3ull * sizeof(uint64_t) * (uint64_t)nseg;
    if (!workspace || workspace_bytes < need)
        return fail(EDT_ERR_ARG, "workspace of %llu bytes needed", (unsigned long long)need);
    if (reinterpret_cast<uintptr_t>(workspace) & 7u) return fail(EDT_ERR_ARG, "workspace must be 8-byte aligned");
    thread_local std::vector<uint64_t> h;
    h.assign(3 * (size_t)nseg, 0);
    int rc = seg_table_impl(v0_t, v1_t, out_t, nseg, seg_numel, in_dt, out_dt, apart, h.data());
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(workspace, h.data(), need, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return fail(EDT_ERR_LAUNCH, "tensor table upload failed: %s", hipGetErrorString(e));
    return EDT_OK;
}
}   // namespace

// apart = 0 (the two-pass form): an output may be exactly one of its own parents (written in place
// after the stats pass read it), never overlap another tensor's parent or output. Spans grouped by
// identical byte range, then swept in address order: a group holding an output must belong to one
// segment and overlap no other group; input-only groups may overlap each other.
struct SegSpan {
    uintptr_t a, e;
    int seg;
    bool out;
};

inline bool in_place_safe(std::vector<SegSpan>& sp) {
    std::sort(sp.begin(), sp.end(), [](const SegSpan& x, const SegSpan& y) {
        return x.a != y.a ? x.a < y.a : x.e < y.e;
    });
    uintptr_t far_any = 0, far_out = 0;
    for (size_t i = 0; i < sp.size();) {
        size_t j = i;
        bool out = false, one_seg = true;
        for (; j < sp.size() && sp[j].a == sp[i].a && sp[j].e == sp[i].e; ++j) {
            out = out || sp[j].out;
            one_seg = one_seg && sp[j].seg == sp[i].seg;
        }
        if (out && !one_seg) return false;                 // an output shared with another tensor's span
        if (sp[i].a < far_out || (out && sp[i].a < far_any)) return false;   // a partial overlap with an output
        far_any = sp[i].e > far_any ? sp[i].e : far_any;
        if (out) far_out = sp[i].e > far_out ? sp[i].e : far_out;
        i = j;
    }
    return true;
}

// seg_numel may be NULL only here, for edt_slerp_merge_list (its ABI carries no sizes: the
// in-place rule is its caller's, as the header says); the public entry requires the sizes.
static int seg_table_impl(const void* const* v0_t, const void* const* v1_t, void* const* out_t, int nseg,
                          const uint64_t* seg_numel, int in_dt, int out_dt, int apart, uint64_t* table_host) {
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nseg < 0) return fail(EDT_ERR_ARG, "negative segment count");
    if (nseg == 0) return EDT_OK;
    if (!v0_t || !v1_t || !out_t || !table_host) return fail(EDT_ERR_ARG, "null tensor table");
    if (apart && !seg_numel) return fail(EDT_ERR_ARG, "the overlap check needs the segment sizes");
    const uint64_t isz = in_dt == EDT_BF16 ? 2 : 4, osz = out_dt == EDT_BF16 ? 2 : 4;
    std::vector<Span> sp;
    if (apart) sp.reserve(3 * (size_t)nseg);
    for (int i = 0; i < nseg; ++i) {
        // a null pointer is only valid for an empty segment (it has no chunks, so it is never read)
        if (!aligned16(v0_t[i]) || !aligned16(v1_t[i]) || !aligned16(out_t[i]))
            return fail(EDT_ERR_ARG, "tensor %d is not 16-byte aligned", i);
        if (seg_numel && seg_numel[i] > 0 && (!v0_t[i] || !v1_t[i] || !out_t[i]))
            return fail(EDT_ERR_ARG, "tensor %d is null", i);
        table_host[3 * (size_t)i] = reinterpret_cast<uintptr_t>(v0_t[i]);
        table_host[3 * (size_t)i + 1] = reinterpret_cast<uintptr_t>(v1_t[i]);
        table_host[3 * (size_t)i + 2] = reinterpret_cast<uintptr_t>(out_t[i]);
        if (apart && seg_numel[i] > 0) {
            const uintptr_t p0 = reinterpret_cast<uintptr_t>(v0_t[i]), p1 = reinterpret_cast<uintptr_t>(v1_t[i]);
            const uintptr_t po = reinterpret_cast<uintptr_t>(out_t[i]);
            sp.push_back({p0, p0 + seg_numel[i] * isz, false});
            sp.push_back({p1, p1 + seg_numel[i] * isz, false});
            sp.push_back({po, po + seg_numel[i] * osz, true});
        }
    }
    if (apart && !spans_apart(sp))
        return fail(EDT_ERR_ARG, "an output overlaps a parent tensor: the single-pass form needs outputs apart");
    if (!apart && seg_numel) {
        std::vector<SegSpan> ss;
        ss.reserve(3 * (size_t)nseg);
        for (int i = 0; i < nseg; ++i) {
            if (!seg_numel[i]) continue;
            const uintptr_t p0 = reinterpret_cast<uintptr_t>(v0_t[i]), p1 = reinterpret_cast<uintptr_t>(v1_t[i]);
            const uintptr_t po = reinterpret_cast<uintptr_t>(out_t[i]);
            ss.push_back({p0, p0 + seg_numel[i] * isz, i, false});
            ss.push_back({p1, p1 + seg_numel[i] * isz, i, false});
            ss.push_back({po, po + seg_numel[i] * osz, i, true});
        }
        if (!in_place_safe(ss))
            return fail(EDT_ERR_ARG, "an output overlaps another tensor's parent or output (only its own parent, "
                                     "exactly, may be written in place)");
    }
    return EDT_OK;
}

extern "C" {

int edt_slerp_seg_table(const void* const* v0_t, const void* const* v1_t, void* const* out_t, int nseg,
                        const uint64_t* seg_numel, int in_dt, int out_dt, int apart, uint64_t* table_host) {
    if (nseg > 0 && !seg_numel) {
        g_err[0] = 0;
        return fail(EDT_ERR_ARG, "the overlap checks need the segment sizes (seg_numel)");
    }
    return seg_table_impl(v0_t, v1_t, out_t, nseg, seg_numel, in_dt, out_dt, apart, table_host);
}

int edt_slerp_stats_table(const uint64_t* seg_table, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                          double* partial, void* stream) {
    g_err[0] = 0;
    int rc = table_args(seg_table, in_dt, EDT_F32, nchunks, 0);
    if (rc) return rc;
    return slerp_stats_impl(nullptr, nullptr, in_dt, chunk_desc, nchunks, partial, seg_table, stream);
}

int edt_slerp_blend_table(const uint64_t* seg_table, int in_dt, int out_dt, const uint64_t* chunk_desc,
                          int64_t nchunks, const float* coef, const int32_t* redo, void* stream) {
    g_err[0] = 0;
    int rc = table_args(seg_table, in_dt, out_dt, nchunks, 0);
    if (rc) return rc;
    if (nchunks == 0) return EDT_OK;
    if (!chunk_desc || !coef) return fail(EDT_ERR_ARG, "null buffer");
    if (!redo) return slerp_blend_impl(nullptr, nullptr, in_dt, nullptr, out_dt, chunk_desc, nchunks, coef, seg_table, stream);
    return blend_redo(nullptr, nullptr, in_dt, nullptr, out_dt, chunk_desc, nchunks, coef, seg_table, redo, nullptr,
                      (hipStream_t)stream);
}

int edt_slerp_blend_segments(const void* v0, const void* v1, int in_dt, void* out, int out_dt,
                             const uint64_t* chunk_desc, int64_t nchunks, const float* coef, const int32_t* redo,
                             void* stream) {
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nchunks < 0) return fail(EDT_ERR_ARG, "negative chunk count");
    if (nchunks == 0) return EDT_OK;
    if (!v0 || !v1 || !out || !chunk_desc || !coef || !redo) return fail(EDT_ERR_ARG, "null buffer");
    if (!aligned16(v0) || !aligned16(v1) || !aligned16(out))
        return fail(EDT_ERR_ARG, "slerp buffers must be 16-byte aligned");
    return blend_redo(v0, v1, in_dt, out, out_dt, chunk_desc, nchunks, coef, nullptr, redo, nullptr, (hipStream_t)stream);
}

int edt_slerp_merge_table(const uint64_t* seg_table, int in_dt, int out_dt, const uint64_t* chunk_desc,
                          int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t,
                          double dot_threshold, double eps, double* partial, float* coef, float* dot_out,
                          void* stream) {
    g_err[0] = 0;
    int rc = table_args(seg_table, in_dt, out_dt, nchunks, nseg);
    if (rc) return rc;
    if (nseg == 0 || nchunks == 0) return EDT_OK;
    if (!chunk_desc || !seg_first_chunk || !t || !partial || !coef) return fail(EDT_ERR_ARG, "null buffer");
    rc = slerp_stats_impl(nullptr, nullptr, in_dt, chunk_desc, nchunks, partial, seg_table, stream);
    if (rc) return rc;
    rc = edt_slerp_coef(partial, seg_first_chunk, nseg, t, dot_threshold, eps, coef, dot_out, stream);
    if (rc) return rc;
    return slerp_blend_impl(nullptr, nullptr, in_dt, nullptr, out_dt, chunk_desc, nchunks, coef, seg_table, stream);
}

int edt_slerp_merge_table_speculative(const uint64_t* seg_table, int in_dt, int out_dt, const uint64_t* chunk_desc,
                                      int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t,
                                      double dot_threshold, double eps, double* partial, float* coef,
                                      float* dot_out, int32_t* redo, void* stream) {
    g_err[0] = 0;
    int rc = table_args(seg_table, in_dt, out_dt, nchunks, nseg);
    if (rc) return rc;
    if (nseg == 0 || nchunks == 0) return EDT_OK;
    if (!chunk_desc || !seg_first_chunk || !t || !partial || !coef || !redo) return fail(EDT_ERR_ARG, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    // the any-redo word: the last double of the workspace, as edt_slerp_merge_speculative's
    int32_t* any = reinterpret_cast<int32_t*>(partial + edt_slerp_sums_doubles(3, nchunks) - 1);
    rc = pair_sums(nullptr, nullptr, in_dt, nullptr, out_dt, true, chunk_desc, nchunks, partial, t, seg_table, s, any);
    if (rc) return rc;
    slerp_coef_kernel<<<coef_grid(nseg), kBlock, 0, s>>>(partial, seg_first_chunk, nseg, t, (float)dot_threshold,
                                                         (float)eps, coef, dot_out, redo, any);
    rc = check_launch("slerp_coef_kernel");
    if (rc) return rc;
    return blend_redo(nullptr, nullptr, in_dt, nullptr, out_dt, chunk_desc, nchunks, coef, seg_table, redo, any, s);
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
    int rc = upload_seg_table(v0_t, v1_t, out_t, nseg, nullptr, in_dt, out_dt, 0, workspace, workspace_bytes,
                              (hipStream_t)stream);
    if (rc) return rc;
    return edt_slerp_merge_table(static_cast<const uint64_t*>(workspace), in_dt, out_dt, chunk_desc, nchunks,
                                 seg_first_chunk, nseg, t, dot_threshold, eps, partial, coef, dot_out, stream);
}

int edt_slerp_merge_list_speculative(const void* const* v0_t, const void* const* v1_t, int in_dt, void* const* out_t,
                                     int out_dt, const uint64_t* seg_numel, const uint64_t* chunk_desc,
                                     int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t,
                                     double dot_threshold, double eps, double* partial, float* coef, float* dot_out,
                                     int32_t* redo, void* workspace, uint64_t workspace_bytes, void* stream) {
    g_err[0] = 0;
    if ((in_dt | out_dt) & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nseg < 0 || nchunks < 0) return fail(EDT_ERR_ARG, "negative count (segments %d, chunks %lld)", nseg, (long long)nchunks);
    if (nseg == 0 || nchunks == 0) return EDT_OK;
    if (!v0_t || !v1_t || !out_t) return fail(EDT_ERR_ARG, "null tensor table");
    if (!seg_numel) return fail(EDT_ERR_ARG, "null segment sizes");
    if (!chunk_desc || !seg_first_chunk || !t || !partial || !coef || !redo) return fail(EDT_ERR_ARG, "null buffer");
    int rc = upload_seg_table(v0_t, v1_t, out_t, nseg, seg_numel, in_dt, out_dt, 1, workspace, workspace_bytes,
                              (hipStream_t)stream);
    if (rc) return rc;
    return edt_slerp_merge_table_speculative(static_cast<const uint64_t*>(workspace), in_dt, out_dt, chunk_desc,
                                             nchunks, seg_first_chunk, nseg, t, dot_threshold, eps, partial, coef,
                                             dot_out, redo, stream);
}


// ---- reference-dot mode (include/edt_sync.h) ----

uint64_t edt_slerp_refdot_workspace_bytes(int nseg, int64_t nchunks, uint32_t chunk_elems, int threads) {
    if (nseg < 0 || nchunks < 0 || threads < 1 || chunk_elems == 0 || chunk_elems % kRefBuf) return 0;
    const uint64_t bpc = chunk_elems / kRefBuf;
    return 8ull * 2 * (uint64_t)(nseg > 0 ? nseg : 1) * (uint64_t)threads + 4ull * (uint64_t)(nchunks > 0 ? nchunks : 1) * bpc;
}

int edt_slerp_refdot_flags(const float* dots, int nseg, double dot_threshold, double band, int32_t* flag,
                           void* stream) {
    g_err[0] = 0;
    if (nseg < 0) return fail(EDT_ERR_ARG, "negative segment count");
    if (nseg == 0) return EDT_OK;
    if (!dots || !flag) return fail(EDT_ERR_ARG, "null buffer");
    refdot_flag_kernel<<<(unsigned)((nseg + kBlock - 1) / kBlock), kBlock, 0, (hipStream_t)stream>>>(
        dots, nseg, (float)dot_threshold, (float)band, flag);
    return check_launch("refdot_flag_kernel");
}

static int refdot_impl(const void* v0, const void* v1, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                       const int32_t* seg_first_chunk, int nseg, uint32_t chunk_elems, const int32_t* flag,
                       int threads, double eps, float* ref_dot, void* workspace, uint64_t workspace_bytes,
                       const uint64_t* seg_ptrs, void* stream) {
    if (in_dt & ~1) return fail(EDT_ERR_ARG, "unsupported dtype");
    if (nseg < 0 || nchunks < 0) return fail(EDT_ERR_ARG, "negative count");
    if (threads < 1 || threads > 256) return fail(EDT_ERR_ARG, "BLAS thread count %d out of range [1, 256]", threads);
    if (chunk_elems == 0 || chunk_elems % kRefBuf)
        return fail(EDT_ERR_ARG, "reference-dot mode needs chunks of a multiple of %d elements (got %u)", kRefBuf,
                    chunk_elems);
    if (nseg == 0) return EDT_OK;
    if (!seg_first_chunk || !ref_dot || !workspace) return fail(EDT_ERR_ARG, "null buffer");
    // no chunks: nothing is read (every flagged segment's dot is the empty sum, 0)
    if (nchunks > 0 && (!chunk_desc || (!seg_ptrs && (!v0 || !v1)))) return fail(EDT_ERR_ARG, "null buffer");
    const uint64_t need = edt_slerp_refdot_workspace_bytes(nseg, nchunks, chunk_elems, threads);
    if (workspace_bytes < need) return fail(EDT_ERR_ARG, "workspace of %llu bytes needed", (unsigned long long)need);
    if (reinterpret_cast<uintptr_t>(workspace) & 7u) return fail(EDT_ERR_ARG, "workspace must be 8-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    double* part = static_cast<double*>(workspace);
    float* bsum = reinterpret_cast<float*>(part + 2 * (uint64_t)nseg * (uint64_t)threads);
    const int bpc = (int)(chunk_elems / kRefBuf);
    const uint64_t gn = 2ull * (uint64_t)nseg * (uint64_t)threads;
    if (gn > kGridBlockCap) return fail(EDT_ERR_ARG, "too many segments x threads");
    if (in_dt == EDT_F32)
        refdot_norm_kernel<EDT_F32><<<(unsigned)gn, kRefThreads, 0, s>>>(v0, v1, chunk_desc, seg_first_chunk, nseg, flag,
                                                                         threads, seg_ptrs, part);
    else
        refdot_norm_kernel<EDT_BF16><<<(unsigned)gn, kRefThreads, 0, s>>>(v0, v1, chunk_desc, seg_first_chunk, nseg,
                                                                          flag, threads, seg_ptrs, part);
    int rc = check_launch("refdot_norm_kernel");
    if (rc) return rc;
    if (nchunks > 0) {
        const uint64_t waves = (uint64_t)nchunks * (uint64_t)bpc;
        const uint64_t gs = (waves + kBlock / 64 - 1) / (kBlock / 64);
        if (gs > kGridBlockCap) return fail(EDT_ERR_ARG, "too many chunks for one launch");
        if (in_dt == EDT_F32)
            refdot_sum_kernel<EDT_F32><<<(unsigned)gs, kBlock, 0, s>>>(v0, v1, chunk_desc, nchunks, seg_first_chunk, flag,
                                                                        threads, (float)eps, seg_ptrs, part, bpc, bsum);
        else
            refdot_sum_kernel<EDT_BF16><<<(unsigned)gs, kBlock, 0, s>>>(v0, v1, chunk_desc, nchunks, seg_first_chunk,
                                                                         flag, threads, (float)eps, seg_ptrs, part, bpc,
                                                                         bsum);
        rc = check_launch("refdot_sum_kernel");
        if (rc) return rc;
    }
    refdot_total_kernel<<<(unsigned)((nseg + kBlock - 1) / kBlock), kBlock, 0, s>>>(chunk_desc, seg_first_chunk, nseg,
                                                                                    flag, bpc, bsum, ref_dot);
    return check_launch("refdot_total_kernel");
}

int edt_slerp_refdot(const void* v0, const void* v1, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                     const int32_t* seg_first_chunk, int nseg, uint32_t chunk_elems, const int32_t* flag, int threads,
                     double eps, float* ref_dot, void* workspace, uint64_t workspace_bytes, void* stream) {
    g_err[0] = 0;
    return refdot_impl(v0, v1, in_dt, chunk_desc, nchunks, seg_first_chunk, nseg, chunk_elems, flag, threads, eps,
                       ref_dot, workspace, workspace_bytes, nullptr, stream);
}

int edt_slerp_refdot_table(const uint64_t* seg_table, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                           const int32_t* seg_first_chunk, int nseg, uint32_t chunk_elems, const int32_t* flag,
                           int threads, double eps, float* ref_dot, void* workspace, uint64_t workspace_bytes,
                           void* stream) {
    g_err[0] = 0;
    int rc = table_args(seg_table, in_dt, EDT_F32, nchunks, nseg);
    if (rc) return rc;
    if (nseg > 0 && !seg_table) return fail(EDT_ERR_ARG, "null tensor table");
    return refdot_impl(nullptr, nullptr, in_dt, chunk_desc, nchunks, seg_first_chunk, nseg, chunk_elems, flag, threads,
                       eps, ref_dot, workspace, workspace_bytes, seg_table, stream);
}

int edt_slerp_refdot_coef(const float* ref_dot, const int32_t* flag, int nseg, const double* t, double dot_threshold,
                          float* coef, float* dot_out, void* stream) {
    g_err[0] = 0;
    if (nseg < 0) return fail(EDT_ERR_ARG, "negative segment count");
    if (nseg == 0) return EDT_OK;
    if (!ref_dot || !t || !coef) return fail(EDT_ERR_ARG, "null buffer");
    refdot_coef_kernel<<<(unsigned)((nseg + kBlock - 1) / kBlock), kBlock, 0, (hipStream_t)stream>>>(
        ref_dot, flag, nseg, t, (float)dot_threshold, coef, dot_out);
    return check_launch("refdot_coef_kernel");
}

}  // extern "C"
