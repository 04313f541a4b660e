// pair_ceiling: the access-pattern ceilings of the EDT-LM pair merge and of lerp / the single-pass
// SLERP on this box, beside the product kernels (r5).
//   pair   edt_pair_merge_to from libedt_sync.so: 1.3B bf16, four parents + the carried momentum
//          read, the child and its momentum written (14 B per element)
//   pmix   the same 7 streams (5 reads, 2 writes, 16-byte accesses) with a trivial body
//   lerp   edt_lerp from libedt_sync.so: 7.07B bf16 (the SLERP lineage pass's stream, 6 B per element)
//   lmix   its 3 streams with a trivial body
// grid: one-shot (one 2,048-element tile per workgroup, address order) and grid-stride at 32 / 256
// workgroups per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/native/pair_ceiling.cpp -ldl -o pair_ceiling
//   ./pair_ceiling path/to/libedt_sync.so
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

typedef int (*pair_fn)(const void*, const void*, const void*, const void*, int, void*, int, const void*, void*, int,
                       uint64_t, double, double, int, void*);
typedef int (*lerp_fn)(const void*, const void*, int, void*, int, int, uint64_t, double, void*);
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct S7 { const u32x4* r[5]; u32x4* w[2]; };

__global__ __launch_bounds__(256) void pmix_kernel(S7 s, uint64_t nv) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < nv; v += stride) {
        u32x4 x = s.r[0][v];
#pragma unroll
        for (int k = 1; k < 5; ++k) x ^= s.r[k][v];
        s.w[0][v] = x;
        s.w[1][v] = x + 1u;
    }
}

__global__ __launch_bounds__(256) void lmix_kernel(const u32x4* a, const u32x4* b, u32x4* o, uint64_t nv) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < nv; v += stride) o[v] = a[v] ^ b[v];
}

int main(int argc, char** argv) {
    const uint64_t P = 1315723264ull, Q = 7070619136ull;     // multiples of 8
    const int iters = 10;
    pair_fn pair = nullptr;
    lerp_fn lerp = nullptr;
    if (argc > 1) {
        void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
        if (!h) { fprintf(stderr, "dlopen %s: %s\n", argv[1], dlerror()); return 4; }
        pair = (pair_fn)dlsym(h, "edt_pair_merge_to");
        lerp = (lerp_fn)dlsym(h, "edt_lerp");
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    uint16_t* bufs[7];
    for (int k = 0; k < 7; ++k) {
        CK(hipMalloc(&bufs[k], P * 2));
        CK(hipMemset(bufs[k], 0x3c, P * 2));
    }
    uint16_t *l0, *l1, *lo;
    CK(hipMalloc(&l0, Q * 2));
    CK(hipMalloc(&l1, Q * 2));
    CK(hipMalloc(&lo, Q * 2));
    CK(hipMemset(l0, 0x3c, Q * 2));
    CK(hipMemset(l1, 0x3c, Q * 2));
    S7 s7;
    for (int k = 0; k < 5; ++k) s7.r[k] = reinterpret_cast<const u32x4*>(bufs[k]);
    for (int k = 0; k < 2; ++k) s7.w[k] = reinterpret_cast<u32x4*>(bufs[5 + k]);
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
    printf("{\"P\": %llu, \"Q\": %llu, \"results\": [\n", (unsigned long long)P, (unsigned long long)Q);
    bool first = true;
    auto emit = [&](const char* name, const char* grid, double bytes, float ms) {
        printf("%s {\"kernel\": \"%s\", \"grid\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}", first ? "" : ",\n", name, grid,
               ms, bytes / (ms * 1e-3) / 1e12);
        first = false;
        fflush(stdout);
    };
    const double pb = 14.0 * P, lb = 6.0 * Q;
    for (int rep = 0; rep < 2; ++rep) {
        if (pair)
            emit("pair", "product", pb, time_it([&] {
                if (pair(bufs[0], bufs[1], bufs[2], bufs[3], 1, bufs[5], 1, bufs[4], bufs[6], 1, P, 0.7, 0.9, 1, s))
                    exit(3);
            }));
        if (lerp)
            emit("lerp", "product", lb, time_it([&] {
                if (lerp(l0, l1, 1, lo, 1, 1, Q, 0.5, s)) exit(3);
            }));
        const uint64_t pnv = P / 8, lnv = Q / 8;
        for (int g : {0, 32, 256}) {
            const unsigned pg = g ? 256u * g : (unsigned)((pnv + 255) / 256);
            const unsigned lg = g ? 256u * g : (unsigned)std::min<uint64_t>((lnv + 255) / 256, 0x7fffffffull);
            char name[32];
            snprintf(name, sizeof(name), g ? "%d/CU" : "one-shot", g);
            emit("pmix", name, pb, time_it([&] { pmix_kernel<<<pg, 256, 0, s>>>(s7, pnv); }));
            emit("lmix", name, lb, time_it([&] {
                lmix_kernel<<<lg, 256, 0, s>>>((const u32x4*)l0, (const u32x4*)l1, (u32x4*)lo, lnv);
            }));
        }
    }
    printf("\n]}\n");
    CK(hipGetLastError());
    return 0;
}
