// In-place vs out-of-place probe (standalone, not part of the library): is the fp32 DiLoCo step's
// sensitivity to where its operands sit in HBM (10.3–11.7 ms for the same launch on
// different allocations) a property of its two read-modify-write streams? The step's mix — 8
// worker streams read (non-temporal), theta and the momentum read — written three ways:
//
//   inplace   theta and momentum rewritten in place (the library's step)
//   mom_out   theta in place, the new momentum into a second buffer (a ping-pong momentum)
//   both_out  theta and momentum both into second buffers (ping-pong theta and momentum)
//
// per allocation draw: fresh theta / momentum / second buffers behind a held spacer that grows by
// 1.375 GiB per draw (the workers allocated once), every variant timed 5 times interleaved, the
// median reported. One 2,048-element tile per 256-thread workgroup (8 floats per thread as two
// float4 halves, wave-contiguous), grid in address order; the SGD body of the library's step
// (Nesterov, lr 0.7, mu 0.9) in fp32.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/_rmw_probe scripts/rmw_probe.hip
//   scripts/_rmw_probe [draws] [n_floats]
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

struct Ops {
    const float* w[8];
    const float* th;
    const float* m;
    float* th_out;
    float* m_out;
};

__global__ __launch_bounds__(256) void step_kernel(Ops p, uint64_t n) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t i = (uint64_t)blockIdx.x * 2048 + (uint64_t)h * 1024 + (uint64_t)threadIdx.x * 4;
        if (i + 4 > n) continue;
        const f4 t = *reinterpret_cast<const f4*>(p.th + i);
        const f4 m = *reinterpret_cast<const f4*>(p.m + i);
        f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const f4 w = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p.w[k] + i));
            acc += (w - t) / 8.0f;
        }
        const f4 g = -acc;
        const f4 mn = m * 0.9f + g;
        const f4 u = g + mn * 0.9f;
        *reinterpret_cast<f4*>(p.m_out + i) = mn;
        *reinterpret_cast<f4*>(p.th_out + i) = t - u * 0.7f;
    }
}

static float time_ms(const Ops& o, uint64_t n, hipEvent_t a, hipEvent_t b) {
    const unsigned grid = (unsigned)((n + 2047) / 2048);
    hipLaunchKernelGGL(step_kernel, dim3(grid), dim3(256), 0, 0, o, n);
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(step_kernel, dim3(grid), dim3(256), 0, 0, o, n);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main(int argc, char** argv) {
    const int draws = argc > 1 ? std::atoi(argv[1]) : 6;
    const uint64_t n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1315723264ull;
    if (n % 4 || draws < 1 || draws > 16) {
        std::fprintf(stderr, "n must be a multiple of 4, draws in [1, 16]\n");
        return 2;
    }
    const size_t bytes = n * sizeof(float);
    std::vector<float*> w(8);
    for (auto& p : w) {
        CHECK(hipMalloc(&p, bytes));
        CHECK(hipMemset(p, 0, bytes));
    }
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<void*> spacers;
    const double algo = 48.0 * (double)n;                 // 40 B read + 8 B written per element
    for (int d = 0; d < draws; ++d) {
        if (d) {
            void* s = nullptr;
            CHECK(hipMalloc(&s, (size_t)d * (11ull << 27)));
            spacers.push_back(s);
        }
        float *th, *m, *th2, *m2;
        CHECK(hipMalloc(&th, bytes));
        CHECK(hipMalloc(&m, bytes));
        CHECK(hipMalloc(&th2, bytes));
        CHECK(hipMalloc(&m2, bytes));
        CHECK(hipMemset(th, 0, bytes));
        CHECK(hipMemset(m, 0, bytes));
        Ops base{};
        for (int k = 0; k < 8; ++k) base.w[k] = w[k];
        Ops v[3] = {base, base, base};
        const char* names[3] = {"inplace", "mom_out", "both_out"};
        v[0].th = th; v[0].m = m; v[0].th_out = th; v[0].m_out = m;
        v[1].th = th; v[1].m = m; v[1].th_out = th; v[1].m_out = m2;
        v[2].th = th; v[2].m = m; v[2].th_out = th2; v[2].m_out = m2;
        std::vector<float> t[3];
        for (int r = 0; r < 5; ++r)
            for (int k = 0; k < 3; ++k) t[k].push_back(time_ms(v[k], n, a, b));
        std::printf("{\"draw\": %d, \"n\": %llu", d, (unsigned long long)n);
        for (int k = 0; k < 3; ++k) {
            std::sort(t[k].begin(), t[k].end());
            const float med = t[k][2];
            std::printf(", \"%s_ms\": %.4f, \"%s_TBps\": %.3f", names[k], med, names[k], algo / (med * 1e-3) / 1e12);
        }
        std::printf(", \"va\": {\"th\": \"%p\", \"m\": \"%p\", \"th2\": \"%p\", \"m2\": \"%p\", \"w0\": \"%p\", \"w7\": \"%p\"}}\n",
                    (void*)th, (void*)m, (void*)th2, (void*)m2, (void*)w[0], (void*)w[7]);
        std::fflush(stdout);
        CHECK(hipFree(th));
        CHECK(hipFree(m));
        CHECK(hipFree(th2));
        CHECK(hipFree(m2));
    }
    for (void* s : spacers) CHECK(hipFree(s));
    for (auto p : w) CHECK(hipFree(p));
    return 0;
}
