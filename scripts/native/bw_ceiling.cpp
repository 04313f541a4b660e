// bw_ceiling: what does this box's HBM deliver for the fused outer step's exact access mix?
// Times, on one allocation of the 1.3B / K = 8 bf16-worker / fp32 theta+momentum operand set:
//   step   edt_outer_step from libedt_sync.so (the product kernel)
//   mix    the same 12 streams (read theta, momentum, 8 workers; write theta, momentum) with a
//          trivial body: the memory ceiling of the access mix itself
//   read10 the 10 reads only (one 4-byte store per thread at the end)
//   copy   float4 copy theta -> momentum (read 1, write 1)
// all with 256-thread workgroups, 16-byte accesses, grid-stride with G workgroups per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/native/bw_ceiling.cpp -ldl -o bw_ceiling
//   ./bw_ceiling path/to/libedt_sync.so
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "edt_sync.h"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

typedef int (*step_fn)(void*, int, const void* const*, int, int, void*, int, uint64_t, double, double, int, void*);
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct W8 { const u32x4* p[8]; };

template <bool NT>
__global__ __launch_bounds__(256) void mix_kernel(f32x4* th, f32x4* mo, W8 w, uint64_t nv8) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < nv8; v += stride) {
        f32x4 a0 = th[2 * v], a1 = th[2 * v + 1], b0 = mo[2 * v], b1 = mo[2 * v + 1];
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u32x4 x = NT ? __builtin_nontemporal_load(w.p[k] + v) : w.p[k][v];
            s ^= x.x ^ x.y ^ x.z ^ x.w;
        }
        float f = __uint_as_float(s & 0x3f7fffffu) * 1e-30f;
        a0 += f; a1 += f; b0 += f; b1 += f;
        th[2 * v] = a0; th[2 * v + 1] = a1; mo[2 * v] = b0; mo[2 * v + 1] = b1;
    }
}

__global__ __launch_bounds__(256) void read10_kernel(const f32x4* th, const f32x4* mo, W8 w, uint64_t nv8, uint32_t* sink) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint32_t s = 0;
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < nv8; v += stride) {
        f32x4 a0 = th[2 * v], a1 = th[2 * v + 1], b0 = mo[2 * v], b1 = mo[2 * v + 1];
        s ^= __float_as_uint(a0.x + a1.y + b0.z + b1.w);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u32x4 x = __builtin_nontemporal_load(w.p[k] + v);
            s ^= x.x ^ x.y ^ x.z ^ x.w;
        }
    }
    if (s == 0x12345678u) sink[0] = s;
}

__global__ __launch_bounds__(256) void copy_kernel(const f32x4* src, f32x4* dst, uint64_t nv) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < nv; v += stride) dst[v] = src[v];
}

int main(int argc, char** argv) {
    const uint64_t P = 1315723264ull;    // multiple of 8
    const int K = 8, iters = 10;
    step_fn step = nullptr;
    if (argc > 1) {
        void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
        if (!h) { fprintf(stderr, "dlopen %s: %s\n", argv[1], dlerror()); return 4; }
        step = (step_fn)dlsym(h, "edt_outer_step");
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float *th, *mo;
    uint16_t* w[K];
    uint32_t* sink;
    CK(hipMalloc(&th, P * 4));
    CK(hipMalloc(&mo, P * 4));
    for (int k = 0; k < K; ++k) CK(hipMalloc(&w[k], P * 2));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(th, 0, P * 4));
    CK(hipMemset(mo, 0, P * 4));
    for (int k = 0; k < K; ++k) CK(hipMemset(w[k], 0x3c, P * 2));
    W8 w8;
    for (int k = 0; k < K; ++k) w8.p[k] = reinterpret_cast<const u32x4*>(w[k]);
    const void* wp[K];
    for (int k = 0; k < K; ++k) wp[k] = w[k];

    auto time_it = [&](auto&& launch) {
        launch();
        CK(hipStreamSynchronize(s));
        std::vector<float> ms;
        for (int i = 0; i < iters; ++i) {
            CK(hipEventRecord(a, s));
            launch();
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float t;
            CK(hipEventElapsedTime(&t, a, b));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        return ms[iters / 2];
    };
    const double mix_bytes = 32.0 * P, read_bytes = 24.0 * P, copy_bytes = 8.0 * P;
    printf("{\"P\": %llu, \"results\": [\n", (unsigned long long)P);
    bool first = true;
    auto emit = [&](const char* name, int g, double bytes, float ms) {
        printf("%s {\"kernel\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"TBps\": %.3f}", first ? "" : ",\n",
               name, g, ms, bytes / (ms * 1e-3) / 1e12);
        first = false;
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        if (step) {
            float t = time_it([&] {
                if (step(th, 0, wp, 1, K, mo, 1, P, 0.7, 0.9, 1, s) != 0) { fprintf(stderr, "step failed\n"); exit(3); }
            });
            emit("step", 256, mix_bytes, t);
        }
        for (int g : {8, 32, 256}) {
            const int grid = 256 * g;
            emit("mix_nt", g, mix_bytes, time_it([&] { mix_kernel<true><<<grid, 256, 0, s>>>((f32x4*)th, (f32x4*)mo, w8, P / 8); }));
            emit("mix", g, mix_bytes, time_it([&] { mix_kernel<false><<<grid, 256, 0, s>>>((f32x4*)th, (f32x4*)mo, w8, P / 8); }));
            emit("read10", g, read_bytes, time_it([&] { read10_kernel<<<grid, 256, 0, s>>>((const f32x4*)th, (const f32x4*)mo, w8, P / 8, sink); }));
            emit("copy", g, copy_bytes, time_it([&] { copy_kernel<<<grid, 256, 0, s>>>((const f32x4*)th, (f32x4*)mo, P / 4); }));
        }
    }
    printf("\n]}\n");
    CK(hipGetLastError());
    return 0;
}
