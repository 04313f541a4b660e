// Speculative-SLERP pass probe (standalone, not part of the library): what does the single pass
// of edt_slerp_merge_speculative — read two bf16 parents, write their lerp, and form fp64 sums
// {x.x, y.y, x.y} — cost beyond lerp's identical stream, and where? Every kernel is a one-pass grid
// (one workgroup per tile, address order) over the 7.07B-element Qwen2.5-7B body, 256 threads:
//
//   lerp        lerp only (the library's lerp_kernel shape: 8 bf16 per lane, one 16-B load each)
//   w1          + fp64 sums per lane, wave butterfly, 3 doubles per wave stored (512 el / wave)
//   w4          + the same with 4 vectors per lane (2,048 el / wave)
//   w1f         w1 with fp32 sums (what the fp64 FMAs cost)
//   w1nb        w1 without the butterfly: lane 0 stores its own sums (what the reduction costs)
//   w1tab       w1 with the tile's start read from a 24-B-per-chunk table first (the chunk lookup)
//   s1 / s4     read-only sums (the two-pass stats), 1 or 4 vectors per lane
//   w1ns        w1 with the row store skipped (stored only if a sum were NaN): the second write stream
//   w1lo        fp64 sums per lane, no butterfly, no store (NaN-guarded): the per-lane math alone
//   lerp4       lerp with 4 vectors per lane
//   w4plain     w4 with default-policy loads
//   w1p128 / w4p128 / w4p64   the row padded to a whole 128-B (64-B) line, written by one wave
//   w4p128nt    the same with a non-temporal row store
//   w1x / w4x   rows placed XCD-major (the rows of the workgroups one XCD runs are contiguous, so
//               its L2 fills whole lines before writing back)
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o scripts/_spec_probe scripts/spec_probe.hip
//   scripts/_spec_probe [n_elements] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pk(float a, float b) {
    const uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
    const uint32_t ra = (ua + 0x7fffu + ((ua >> 16) & 1u)) >> 16, rb = (ub + 0x7fffu + ((ub >> 16) & 1u)) >> 16;
    return ra | (rb << 16);
}
__device__ __forceinline__ void unpack(u4 w, float (&x)[8]) {
    x[0] = lo(w.x); x[1] = hi(w.x); x[2] = lo(w.y); x[3] = hi(w.y);
    x[4] = lo(w.z); x[5] = hi(w.z); x[6] = lo(w.w); x[7] = hi(w.w);
}
__device__ __forceinline__ double wsum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
__device__ __forceinline__ float wsumf(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// MODE: 0 lerp, 1 fp64 sums + butterfly, 2 fp32 sums + butterfly, 3 fp64 no butterfly, 4 = 1 + table,
// 5 = 1 with the row store NaN-guarded, 6 = per-lane fp64 sums NaN-guarded (no butterfly),
// 7 / 8 = 1 with the row padded to 16 / 8 doubles (a whole 128-B / 64-B line per wave), 9 = 7 + nt store,
// 10 = 1 with XCD-major row placement
// EMIT: write the lerp output; IT: vectors per lane; NTL: non-temporal loads
template <int MODE, bool EMIT, int IT, bool NTL = true>
__global__ __launch_bounds__(256) void k(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                         uint16_t* __restrict__ o, uint64_t n, const uint64_t* __restrict__ tab,
                                         double* __restrict__ rows) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t base = (uint64_t)blockIdx.x * (256 * 8 * IT);
    if constexpr (MODE == 4) base = tab[3 * blockIdx.x];        // the tile start from a table
    const uint64_t wbase = base + (uint64_t)wave * (64 * 8 * IT) + (uint64_t)lane * 8;
    u4 wa[IT], wb[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const uint64_t i = wbase + (uint64_t)k * 512;
        if (i + 8 <= n) {
            if constexpr (NTL) {
                wa[k] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(a + i));
                wb[k] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(b + i));
            } else {
                wa[k] = *reinterpret_cast<const u4*>(a + i);
                wb[k] = *reinterpret_cast<const u4*>(b + i);
            }
        } else {
            wa[k] = wb[k] = (u4){0, 0, 0, 0};
        }
    }
    double s00 = 0, s11 = 0, s01 = 0;
    float f00 = 0, f11 = 0, f01 = 0;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        float x[8], y[8];
        unpack(wa[k], x);
        unpack(wb[k], y);
        if constexpr (MODE == 2) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                f00 = __builtin_fmaf(x[j], x[j], f00);
                f11 = __builtin_fmaf(y[j], y[j], f11);
                f01 = __builtin_fmaf(x[j], y[j], f01);
            }
        } else if constexpr (MODE != 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const double dx = x[j], dy = y[j];
                s00 = __builtin_fma(dx, dx, s00);
                s11 = __builtin_fma(dy, dy, s11);
                s01 = __builtin_fma(dx, dy, s01);
            }
        }
        if constexpr (EMIT) {
            const uint64_t i = wbase + (uint64_t)k * 512;
            if (i + 8 <= n) {
                float r[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = 0.57f * x[j] + 0.43f * y[j];
                u4 w;
                w.x = pk(r[0], r[1]); w.y = pk(r[2], r[3]); w.z = pk(r[4], r[5]); w.w = pk(r[6], r[7]);
                *reinterpret_cast<u4*>(o + i) = w;
            }
        }
    }
    if constexpr (MODE == 0) return;
    const uint64_t row = ((uint64_t)blockIdx.x * 4 + wave) * 3;
    if constexpr (MODE == 3) {
        if (lane == 0) { rows[row] = s00; rows[row + 1] = s11; rows[row + 2] = s01; }
        return;
    }
    if constexpr (MODE == 6) {
        if (s00 != s00 || s11 != s11 || s01 != s01) rows[row] = s00;
        return;
    }
    double v;
    if constexpr (MODE == 2) {
        const float a0 = wsumf(f00), a1 = wsumf(f11), a2 = wsumf(f01);
        v = lane == 0 ? a0 : lane == 1 ? a1 : a2;
    } else {
        const double a0 = wsum(s00), a1 = wsum(s11), a2 = wsum(s01);
        v = lane == 0 ? a0 : lane == 1 ? a1 : a2;
    }
    if constexpr (MODE == 5) {
        if (v != v) rows[row + lane] = v;
        return;
    }
    if constexpr (MODE == 7 || MODE == 8 || MODE == 9) {
        constexpr int W = MODE == 8 ? 8 : 16;
        const uint64_t prow = ((uint64_t)blockIdx.x * 4 + wave) * W;
        const double pv = lane < 3 ? v : 0.0;
        if (lane < W) {
            if constexpr (MODE == 9) __builtin_nontemporal_store(pv, rows + prow + lane);
            else rows[prow + lane] = pv;
        }
        return;
    }
    if constexpr (MODE == 10) {
        const uint64_t G = gridDim.x, b = blockIdx.x, per = (G + 7) / 8;
        const uint64_t xrow = ((b % 8) * per + b / 8) * 4 + wave;
        if (lane < 3) rows[xrow * 3 + lane] = v;
        return;
    }
    if (lane < 3) rows[row + lane] = v;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 7070619136ull;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    uint16_t *a, *b, *o;
    double* rows;
    uint64_t* tab;
    CHECK(hipMalloc(&a, n * 2));
    CHECK(hipMalloc(&b, n * 2));
    CHECK(hipMalloc(&o, n * 2));
    CHECK(hipMemset(a, 0x3c, n * 2));
    CHECK(hipMemset(b, 0x3d, n * 2));
    const uint64_t tiles1 = (n + 2047) / 2048, tiles4 = (n + 8191) / 8192;
    CHECK(hipMalloc(&rows, tiles1 * 4 * 16 * 8));
    std::vector<uint64_t> ht(3 * tiles1);
    for (uint64_t t = 0; t < tiles1; ++t) { ht[3 * t] = t * 2048; ht[3 * t + 1] = 2048; ht[3 * t + 2] = 0; }
    CHECK(hipMalloc(&tab, ht.size() * 8));
    CHECK(hipMemcpy(tab, ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
    struct Case { std::string name; double bytes_per_el; std::function<void()> f; };
    auto g1 = (unsigned)tiles1, g4 = (unsigned)tiles4;
    std::vector<Case> cs = {
        {"lerp", 6, [&] { k<0, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"w1", 6, [&] { k<1, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"w4", 6, [&] { k<1, true, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"w1f", 6, [&] { k<2, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"w1nb", 6, [&] { k<3, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"w1tab", 6, [&] { k<4, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"s1", 4, [&] { k<1, false, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"s4", 4, [&] { k<1, false, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"w1ns", 6, [&] { k<5, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"w1lo", 6, [&] { k<6, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"lerp4", 6, [&] { k<0, true, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"w4plain", 6, [&] { k<1, true, 4, false><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"lerp_plain", 6, [&] { k<0, true, 1, false><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"w1p128", 6, [&] { k<7, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"w4p128", 6, [&] { k<7, true, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"w4p64", 6, [&] { k<8, true, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"w4p128nt", 6, [&] { k<9, true, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"s4p128", 4, [&] { k<7, false, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"w1x", 6, [&] { k<10, true, 1><<<g1, 256>>>(a, b, o, n, tab, rows); }},
        {"w4x", 6, [&] { k<10, true, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
        {"w2x", 6, [&] { k<10, true, 2><<<(unsigned)((n + 4095) / 4096), 256>>>(a, b, o, n, tab, rows); }},
        {"s4x", 4, [&] { k<10, false, 4><<<g4, 256>>>(a, b, o, n, tab, rows); }},
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (auto& c : cs) c.f();
    CHECK(hipDeviceSynchronize());
    std::vector<std::vector<float>> ms(cs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < cs.size(); ++i) {
            CHECK(hipEventRecord(e0));
            cs[i].f();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float t;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t);
        }
    std::printf("{\"probe\": \"spec_probe\", \"elements\": %llu, \"results\": {", (unsigned long long)n);
    for (size_t i = 0; i < cs.size(); ++i) {
        auto v = ms[i];
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2];
        std::printf("%s\"%s\": {\"median_ms\": %.4f, \"min_ms\": %.4f, \"TBps\": %.3f}", i ? ", " : "", cs[i].name.c_str(),
                    med, v[0], cs[i].bytes_per_el * (double)n / med / 1e9);
    }
    std::printf("}}\n");
    return 0;
}
