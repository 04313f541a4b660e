// Stream roofline probe (standalone, not part of the library): what HBM rate do plain streaming
// kernels of a given read / write mix reach on this MI355X, independent of the library's kernels?
// DiLoCo's fp32 step moves 8 worker reads + theta and momentum read and rewritten (40 B read, 8 B
// written per element); the library's kernel and its access-pattern probe run at ~5.9 TB/s.
//
//   copy        1 read stream  -> 1 write stream
//   read8       8 read streams -> one float per workgroup (writes negligible)
//   read8w1     8 read streams -> 1 write stream (the reduce schedule's partial)
//   step10      8 read streams + 2 streams read and rewritten in place (the fused step's mix)
// each with plain or non-temporal loads, one 2,048-element tile per 256-thread workgroup
// (8 floats per thread as two float4), grid in address order.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/_stream_roofline scripts/stream_roofline.hip
//   scripts/_stream_roofline [n_floats]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4 ld4(const float* p) {
    const f4* q = reinterpret_cast<const f4*>(p);
    if constexpr (NT) return __builtin_nontemporal_load(q);
    return *q;
}

struct Ptrs {
    const float* in[8];
};

// tile = blockIdx.x: elements [tile * 2048, +2048); thread t handles [base + 4t, +4) and
// [base + 1024 + 4t, +4) (wave-contiguous halves)
__device__ __forceinline__ uint64_t idx(int h) {
    return (uint64_t)blockIdx.x * 2048 + (uint64_t)h * 1024 + (uint64_t)threadIdx.x * 4;
}

template <bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const float* in, float* out, uint64_t n) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t i = idx(h);
        if (i + 4 <= n) *reinterpret_cast<f4*>(out + i) = ld4<NT>(in + i);
    }
}

template <bool NT, bool WRITE>
__global__ __launch_bounds__(256) void read8_kernel(Ptrs p, float* out, uint64_t n) {
    f4 acc[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        acc[h] = f4{0.f, 0.f, 0.f, 0.f};
        const uint64_t i = idx(h);
        if (i + 4 > n) continue;
        f4 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = ld4<NT>(p.in[k] + i);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[h] += x[k];
        if constexpr (WRITE) *reinterpret_cast<f4*>(out + i) = acc[h];
    }
    if constexpr (!WRITE) {
        __shared__ float red[256];
        red[threadIdx.x] = acc[0].x + acc[0].y + acc[0].z + acc[0].w + acc[1].x + acc[1].y + acc[1].z + acc[1].w;
        __syncthreads();
        if (threadIdx.x == 0) {
            float s = 0.f;
            for (int t = 0; t < 256; ++t) s += red[t];
            out[blockIdx.x] = s;
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void step10_kernel(Ptrs p, float* theta, float* mom, uint64_t n) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t i = idx(h);
        if (i + 4 > n) continue;
        f4 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = ld4<NT>(p.in[k] + i);
        f4 th = *reinterpret_cast<const f4*>(theta + i);
        f4 m = *reinterpret_cast<const f4*>(mom + i);
        f4 d = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k) d += x[k] - th;
        m = 0.9f * m + d * 0.125f;
        *reinterpret_cast<f4*>(mom + i) = m;
        *reinterpret_cast<f4*>(theta + i) = th + 0.7f * m;
    }
}

// theta and momentum interleaved per tile in ONE buffer (tile t: 2,048 theta floats then 2,048
// momentum floats): the two read-modify-write streams always sit side by side in HBM, whatever
// the allocation — does that make the step's rate independent of placement?
template <bool NT>
__global__ __launch_bounds__(256) void step10_il_kernel(Ptrs p, float* tm, uint64_t n) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t i = idx(h);
        if (i + 4 > n) continue;
        const uint64_t j = (uint64_t)blockIdx.x * 4096 + (uint64_t)h * 1024 + (uint64_t)threadIdx.x * 4;
        f4 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = ld4<NT>(p.in[k] + i);
        f4 th = *reinterpret_cast<const f4*>(tm + j);
        f4 m = *reinterpret_cast<const f4*>(tm + j + 2048);
        f4 d = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k) d += x[k] - th;
        m = 0.9f * m + d * 0.125f;
        *reinterpret_cast<f4*>(tm + j + 2048) = m;
        *reinterpret_cast<f4*>(tm + j) = th + 0.7f * m;
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1315723264ull;
    const uint64_t bytes = n * 4;
    // argv[2]: MiB of spacer allocated between theta and momentum (shifts their relative placement)
    const uint64_t spacer = argc > 2 ? std::strtoull(argv[2], nullptr, 10) << 20 : 0;
    const bool only_step = argc > 3;       // argv[3] present: only the two step kernels
    std::vector<float*> bufs(11);
    float* gap = nullptr;
    for (int q = 0; q < 11; ++q) {
        if (q == 9 && spacer) CHECK(hipMalloc(&gap, spacer));
        CHECK(hipMalloc(&bufs[q], bytes));
        CHECK(hipMemset(bufs[q], 0, bytes));
    }
    float* tm = nullptr;
    const uint64_t grid_tiles = (n + 2047) / 2048;
    CHECK(hipMalloc(&tm, grid_tiles * 4096 * 4));
    CHECK(hipMemset(tm, 0, grid_tiles * 4096 * 4));
    Ptrs p;
    for (int k = 0; k < 8; ++k) p.in[k] = bufs[k];
    float* theta = bufs[8];
    float* mom = bufs[9];
    float* out = bufs[10];
    const unsigned grid = (unsigned)((n + 2047) / 2048);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto time = [&](const char* name, double moved, auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        std::vector<float> ms;
        for (int r = 0; r < 10; ++r) {
            CHECK(hipEventRecord(a, 0));
            launch();
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float t;
            CHECK(hipEventElapsedTime(&t, a, b));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f, \"bytes\": %.0f}\n", name, med,
                    moved / (med / 1e3) / 1e12, moved);
        std::fflush(stdout);
    };
    const double B = (double)bytes;
    if (only_step) {
        for (int r = 0; r < 3; ++r) {
            time("step10", 12 * B, [&] { step10_kernel<false><<<grid, 256>>>(p, theta, mom, n); });
            time("step10_il", 12 * B, [&] { step10_il_kernel<false><<<grid, 256>>>(p, tm, n); });
        }
        return 0;
    }
    time("copy", 2 * B, [&] { copy_kernel<false><<<grid, 256>>>(bufs[0], out, n); });
    time("copy_nt", 2 * B, [&] { copy_kernel<true><<<grid, 256>>>(bufs[0], out, n); });
    time("read8", 8 * B, [&] { read8_kernel<false, false><<<grid, 256>>>(p, out, n); });
    time("read8_nt", 8 * B, [&] { read8_kernel<true, false><<<grid, 256>>>(p, out, n); });
    time("read8w1", 9 * B, [&] { read8_kernel<false, true><<<grid, 256>>>(p, out, n); });
    time("read8w1_nt", 9 * B, [&] { read8_kernel<true, true><<<grid, 256>>>(p, out, n); });
    time("step10", 12 * B, [&] { step10_kernel<false><<<grid, 256>>>(p, theta, mom, n); });
    time("step10_nt", 12 * B, [&] { step10_kernel<true><<<grid, 256>>>(p, theta, mom, n); });
    time("step10_il", 12 * B, [&] { step10_il_kernel<false><<<grid, 256>>>(p, tm, n); });
    CHECK(hipGetLastError());
    for (auto& x : bufs) CHECK(hipFree(x));
    CHECK(hipFree(tm));
    if (gap) CHECK(hipFree(gap));
    return 0;
}
