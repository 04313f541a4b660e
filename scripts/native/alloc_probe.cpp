// alloc_probe: does the physical placement of the arenas change the fused outer step's speed,
// and which kernel variant is robust to it?
// Allocates the 1.3B / K = 8 bf16-worker / fp32 theta+momentum operand set (10 arenas, 31.6 GB)
// several times, with hipMalloc and with hipExtMallocWithFlags(hipDeviceMallocContiguous), and on
// each allocation times edt_outer_step of every library given (dlopen; HIP events, median of 10).
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -I include alloc_probe.cpp -ldl -o alloc_probe
//   ./alloc_probe REPS lib1.so[,lib2.so...]
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
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

__global__ void fill_f32(float* p, uint64_t n, float v) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        p[i] = v * (float)((i * 2654435761ull) % 1000) * 1e-3f;
}
__global__ void fill_bf16(uint16_t* p, uint64_t n, uint16_t v) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) p[i] = v;
}

int main(int argc, char** argv) {
    const uint64_t P = 1315723264ull;
    const int K = 8, iters = 10;
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    std::vector<std::string> names;
    std::vector<step_fn> fns;
    if (argc > 2) {
        std::string all = argv[2];
        size_t q = 0;
        while (q <= all.size()) {
            size_t e = all.find(',', q);
            if (e == std::string::npos) e = all.size();
            std::string path = all.substr(q, e - q);
            void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
            if (!h) { fprintf(stderr, "dlopen %s: %s\n", path.c_str(), dlerror()); return 4; }
            fns.push_back((step_fn)dlsym(h, "edt_outer_step"));
            names.push_back(path);
            q = e + 1;
        }
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::string out = "{";
    for (int mode = 0; mode < 2; ++mode) {
        for (int r = 0; r < reps; ++r) {
            std::vector<void*> p(2 + K, nullptr);
            bool ok = true;
            for (int j = 0; j < 2 + K; ++j) {
                const size_t nb = P * (j < 2 ? 4 : 2);
                hipError_t e = mode ? hipExtMallocWithFlags(&p[j], nb, hipDeviceMallocContiguous) : hipMalloc(&p[j], nb);
                if (e != hipSuccess) { ok = false; fprintf(stderr, "alloc %d failed: %s\n", j, hipGetErrorString(e)); break; }
            }
            if (!ok) {
                for (void* q : p) if (q) (void)hipFree(q);
                (void)hipGetLastError();
                continue;
            }
            fill_f32<<<4096, 256, 0, s>>>((float*)p[0], P, 0.02f);
            CK(hipMemsetAsync(p[1], 0, P * 4, s));
            for (int k = 0; k < K; ++k) fill_bf16<<<4096, 256, 0, s>>>((uint16_t*)p[2 + k], P, 0x3c00 + k);
            const void* w[K];
            for (int k = 0; k < K; ++k) w[k] = p[2 + k];
            char key[96];
            snprintf(key, sizeof(key), "\"%s_%d\": {", mode ? "contiguous" : "hipMalloc", r);
            out += key;
            for (size_t f = 0; f < fns.size(); ++f) {
                if (fns[f](p[0], EDT_F32, w, EDT_BF16, K, p[1], 1, P, 0.7, 0.9, 1, s)) return 3;
                std::vector<float> ts;
                for (int i = 0; i < iters; ++i) {
                    CK(hipEventRecord(a, s));
                    fns[f](p[0], EDT_F32, w, EDT_BF16, K, p[1], 1, P, 0.7, 0.9, 1, s);
                    CK(hipEventRecord(b, s));
                    CK(hipEventSynchronize(b));
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, b));
                    ts.push_back(ms);
                }
                std::sort(ts.begin(), ts.end());
                char buf[256];
                snprintf(buf, sizeof(buf), "\"%s\": %.4f%s", names[f].c_str(), ts[ts.size() / 2],
                         f + 1 < fns.size() ? ", " : "");
                out += buf;
            }
            out += "}, ";
            for (void* q : p) CK(hipFree(q));
        }
    }
    if (out.size() > 2 && out.substr(out.size() - 2) == ", ") out.resize(out.size() - 2);
    out += "}";
    printf("%s\n", out.c_str());
    return 0;
}
