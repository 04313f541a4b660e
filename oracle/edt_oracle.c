/*
 * edt_oracle.c — CPU restatement of the reference's outer-loop sync arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY. This is the checker the parity tests, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg compare the HIP kernels against; the product library never links
 * or calls it. It is pinned against golden vectors produced by the reference's own code
 * (tests/golden/gen_golden.py -> tests/test_oracle_golden.py).
 *
 * Each function restates, element by element and in the same op order, what the reference's
 * PyTorch CPU ops compute:
 *   oracle_outer_step   EDT_LM/diloco.py:238-289 (== EDT_LM/diloco_sim.py:233-299)
 *                       + torch/optim/sgd.py _single_tensor_sgd (momentum, nesterov)
 *   oracle_pair_merge   EDT_LM/train/crossover.py:150-163 (lerp .5) + 166-230 (run_sgd)
 *   oracle_lerp         EDT_LM/train/crossover.py:50-51 on torch tensors / EDT_RL/crossover.py:46-47
 * Rounding model (verified against the goldens):
 *   fp32  : one IEEE op per torch op; add(x, y, alpha=a) == fmaf(a, y, x); x / K true division.
 *   bf16  : every op computed in fp32, then rounded to bf16 RNE (c10::BFloat16); the alpha of
 *           add(..., alpha=a) is first rounded to bf16; mul_(s) uses the fp32 scalar.
 *           torch's CPU add(x, y, alpha) is vectorised: x + alpha*y is ONE fp32 fma rounded to
 *           bf16 -- except on the scalar tail of each contiguous run its vectorised loop handles
 *           (the last numel % 32 elements of a tensor, per parallel chunk, on an AVX-512 host),
 *           where it is BFloat16 arithmetic: round(x + round(alpha*y)). `tail` (nullable, one
 *           byte per element, 1 = scalar-tail element) selects that form, so the oracle can
 *           reproduce the reference bit for bit; tail = NULL is the vectorised semantics the HIP
 *           kernels implement on every element.
 * Build: see oracle/Makefile (gcc -O3 -march=x86-64-v3 -ffp-contract=off: the only FMAs are the
 * explicit fmaf() calls, which x86-64-v3 executes as one vfmadd instead of a libm call).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { OR_F32 = 0, OR_BF16 = 1 };

static inline float bf2f(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static inline uint16_t f2bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;        /* NaN, as c10 */
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

/* value of x rounded to dtype dt, as fp32 */
static inline float rnd(int dt, float x) { return dt == OR_BF16 ? bf2f(f2bf(x)) : x; }

static inline float load(const void* p, int dt, uint64_t i) {
    return dt == OR_BF16 ? bf2f(((const uint16_t*)p)[i]) : ((const float*)p)[i];
}

static inline void store(void* p, int dt, uint64_t i, float x) {
    if (dt == OR_BF16) ((uint16_t*)p)[i] = f2bf(x);
    else ((float*)p)[i] = x;
}

typedef struct {
    float mul_mu, alpha_mu, alpha_nlr;
    int use_mom, has_buf, nesterov;
} sgd_t;

static sgd_t make_sgd(int gdt, double lr, double mu, int has_buf, int nesterov) {
    sgd_t s;
    s.mul_mu = (float)mu;                         /* buf.mul_(momentum): fp32 opmath scalar */
    s.alpha_mu = rnd(gdt, (float)mu);             /* alpha cast to the tensor dtype */
    s.alpha_nlr = rnd(gdt, (float)(-lr));
    s.use_mom = mu != 0.0;
    s.has_buf = has_buf;
    s.nesterov = nesterov;
    return s;
}

/* add(x, y, alpha=a) in dtype dt: vectorised form, or BFloat16 scalar-tail form */
static inline float add_alpha(int dt, float x, float a, float y, int scalar_tail) {
    if (dt == OR_BF16 && scalar_tail) return rnd(dt, x + rnd(dt, a * y));
    return rnd(dt, fmaf(a, y, x));
}

/* torch.optim.SGD single-tensor step on one element; returns the new parameter. */
static inline float sgd_elem(int gdt, const sgd_t* s, float theta, float grad, void* mom, uint64_t i,
                             int tail) {
    float u = grad;
    if (s->use_mom) {
        float b;
        if (s->has_buf) {
            b = rnd(gdt, load(mom, gdt, i) * s->mul_mu);  /* buf.mul_(momentum) */
            b = rnd(gdt, b + grad);                       /* .add_(grad, alpha=1 - dampening) */
        } else {
            b = grad;                                     /* buf = grad.clone() */
        }
        store(mom, gdt, i, b);
        u = s->nesterov ? add_alpha(gdt, grad, s->alpha_mu, b, tail) : b;   /* grad.add(buf, alpha=mu) */
    }
    return add_alpha(gdt, theta, s->alpha_nlr, u, tail);                   /* param.add_(grad, alpha=-lr) */
}

/* DiLoCo outer step, in place on theta (gdt) and mom (gdt). One loop body per dtype regime
 * (GDT/WDT compile-time constants) so gcc vectorises the per-element chain. */
#define OB 512   /* elements per block: the worker loop runs inside, vectorised over the block */
#define OUTER_LOOP(GDT, WDT)                                                                      \
    _Pragma("omp parallel for schedule(static)")                                                  \
    for (int64_t bb = 0; bb < ((int64_t)n + OB - 1) / OB; ++bb) {                                 \
        const uint64_t i0 = (uint64_t)bb * OB;                                                    \
        const int m = (int)((n - i0) < OB ? (n - i0) : OB);                                       \
        float g[OB], acc[OB];                                                                     \
        for (int e = 0; e < m; ++e) {                                                             \
            g[e] = load(theta, GDT, i0 + e);                                                      \
            acc[e] = 0.0f;                                         /* zeros_like(base) */         \
        }                                                                                         \
        for (int k = 0; k < K; ++k) {                              /* worker-major, as :243 */    \
            const void* w = workers[k];                                                           \
            for (int e = 0; e < m; ++e) {                                                         \
                float d = rnd(GDT, load(w, WDT, i0 + e) - g[e]);   /* trained - base */           \
                d = rnd(GDT, pow2 ? d * kinv : d / kf);            /* delta / num_models */       \
                acc[e] = rnd(GDT, acc[e] + d);                     /* acc += ... */               \
            }                                                                                     \
        }                                                                                         \
        for (int e = 0; e < m; ++e) {                                                             \
            const uint64_t i = i0 + e;                                                            \
            store(theta, GDT, i, sgd_elem(GDT, &s, g[e], -acc[e], mom, i, tail ? tail[i] : 0));   \
        }                                                                                         \
    }

int oracle_outer_step(void* theta, int gdt, const void* const* workers, int wdt, int K, void* mom,
                      int has_buf, uint64_t n, double lr, double mu, int nesterov,
                      const uint8_t* tail) {
    if (K < 1) return -1;
    if (gdt == OR_BF16 && wdt != OR_BF16) return -1;
    const sgd_t s = make_sgd(gdt, lr, mu, has_buf, nesterov);
    const float kf = (float)K;
    const int pow2 = (K & (K - 1)) == 0;          /* x * (1/K) == x / K exactly for K = 2^j */
    const float kinv = 1.0f / kf;
    if (gdt == OR_BF16) {
        OUTER_LOOP(OR_BF16, OR_BF16)
    } else if (wdt == OR_BF16) {
        OUTER_LOOP(OR_F32, OR_BF16)
    } else {
        OUTER_LOOP(OR_F32, OR_F32)
    }
    return 0;
}

/* Sharded form, part 1: acc (+)= sum_k round_g(round_g(w_k - g) / K_total), fp32 running sum
 * (accumulate = 1 continues from acc). Restates EDT_LM/diloco.py:243-246 over a worker subset. */
int oracle_delta_partial(const void* theta, int gdt, const void* const* workers, int wdt, int K,
                         int K_total, uint64_t n, float* acc, int accumulate) {
    if (gdt == OR_BF16 && wdt != OR_BF16) return -1;
    const float kf = (float)K_total;
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
        const uint64_t i = (uint64_t)ii;
        const float g = load(theta, gdt, i);
        float a = accumulate ? acc[i] : 0.0f;
        for (int k = 0; k < K; ++k) {
            float d = rnd(gdt, load(workers[k], wdt, i) - g);
            d = rnd(gdt, d / kf);
            a = a + d;
        }
        acc[i] = a;
    }
    return 0;
}

/* Sharded form, part 2: grad = -round_g(acc); SGD step (diloco.py:248-289). */
int oracle_sgd_apply(void* theta, int gdt, const float* acc, void* mom, int has_buf, uint64_t n,
                     double lr, double mu, int nesterov) {
    const sgd_t s = make_sgd(gdt, lr, mu, has_buf, nesterov);
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
        const uint64_t i = (uint64_t)ii;
        const float g = load(theta, gdt, i);
        store(theta, gdt, i, sgd_elem(gdt, &s, g, -rnd(gdt, acc[i]), mom, i, 0));
    }
    return 0;
}

/* EDT pair merge for one child: base = lerp(.5, b1, b2) in wdt (b2 == NULL: b1 is the base, gdt),
 * d = ((m1-B)+(m2-B))/2 in gdt, SGD; writes theta_out (gdt) and mom (gdt). */
int oracle_pair_merge(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                      void* theta_out, int gdt, void* mom, int has_buf, uint64_t n, double lr,
                      double mu, int nesterov, const uint8_t* tail) {
    if (gdt == OR_BF16 && wdt != OR_BF16) return -1;
    const sgd_t s = make_sgd(gdt, lr, mu, has_buf, nesterov);
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
        const uint64_t i = (uint64_t)ii;
        float base;
        if (b2) {
            const float x = rnd(wdt, 0.5f * load(b1, wdt, i));     /* (1 - 0.5) * v0 */
            const float y = rnd(wdt, 0.5f * load(b2, wdt, i));     /* 0.5 * v1 */
            base = rnd(wdt, x + y);
        } else {
            base = load(b1, gdt, i);                                /* merged base, dtype gdt */
        }
        base = rnd(gdt, base);                                      /* load_state_dict copy */
        const float d1 = rnd(gdt, load(m1, wdt, i) - base);
        const float d2 = rnd(gdt, load(m2, wdt, i) - base);
        float d = rnd(gdt, d1 + d2);
        d = rnd(gdt, d / 2.0f);                                     /* / num_models */
        const float acc = rnd(gdt, 0.0f + d);                       /* zeros + delta */
        store(theta_out, gdt, i, sgd_elem(gdt, &s, base, -acc, mom, i, tail ? tail[i] : 0));
    }
    return 0;
}

/* (1-t)*v0 + t*v1 with three rounded ops in compute dtype cdt, stored as out_dt. */
int oracle_lerp(const void* v0, const void* v1, int in_dt, void* out, int out_dt, int cdt,
                uint64_t n, double t) {
    const float c0 = (float)(1.0 - t), c1 = (float)t;
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
        const uint64_t i = (uint64_t)ii;
        const float x = rnd(cdt, c0 * load(v0, in_dt, i));
        const float y = rnd(cdt, c1 * load(v1, in_dt, i));
        store(out, out_dt, i, rnd(cdt, x + y));
    }
    return 0;
}

/* Threads the OpenMP loops above may use (for the bench's cpu_baseline report). */
int oracle_max_threads(void) {
#ifdef _OPENMP
    extern int omp_get_max_threads(void);
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* The OpenMP team size of the loops above (bench.py's cpu_baseline: the host's CPU share). */
int oracle_set_threads(int n) {
#ifdef _OPENMP
    extern void omp_set_num_threads(int);
    if (n > 0) omp_set_num_threads(n);
#endif
    return oracle_max_threads();
}

/* ---- the reference's SLERP dot (EDT_RL/crossover.py:20-29), restated bit for bit ------------
 * dot = np.sum(normalize(v0) * normalize(v1)) on float32 arrays, normalize(v) = v / ||v|| when
 * ||v|| > eps (:57-61), ||v|| = np.linalg.norm = sqrt(v.ravel().dot(v.ravel())):
 *   * v.dot(v) is BLAS sdot. numpy 2.2's wheel bundles OpenBLAS 0.3.29 (scipy-openblas, DYNAMIC_ARCH),
 *     which on this host runs its SkylakeX kernel (threadpoolctl: architecture "SkylakeX"): for the
 *     first n1 = n & -32 elements, 4 x 16 fp32 lanes accumulate with FMA over 64-element blocks
 *     (lane L takes elements 64k + L), fold to 4 x 8 lanes (acc[L] + acc[L + 8] per zmm), the
 *     32-element remainder block (if any) into those with FMA, then ((a0 + a1) + a2) + a3 per lane,
 *     the two 128-bit halves added and two hadds; the n - n1 tail elements are added one by one
 *     as fp32 products into a double accumulator, and the result is returned as float. With
 *     `threads` > 1 the vector is cut into OpenBLAS's level-1 chunks (ceil(rest / threads left))
 *     and the chunk results are added in order in double, rounding to float after each add.
 *     Pinned on this host (tests/test_refdot_cpu.py): threads = 1 at every size tested (up to 67M
 *     elements) reproduces x.dot(x) bit for bit; threads > 1 is the library's published split,
 *     unpinned here.
 *   * np.sum over a contiguous float32 array: the ufunc reduction walks it in buffers of 8192
 *     elements; each buffer is summed pairwise (numpy's pairwise_sum: blocks of <= 128 with 8
 *     accumulators, else halves cut at a multiple of 8) and added to a float running sum that
 *     starts at 0 (the add identity). Pinned the same way.
 * The reference's threshold test `np.abs(dot) > 0.9995` compares in float32 (NEP 50). */
static float sdot_k16(int64_t n, const float* x, const float* y) {
    float a5[4][16], a[4][8];
    memset(a5, 0, sizeof(a5));
    int64_t i = 0;
    const int64_t n64 = n & ~(int64_t)63;
    for (; i < n64; i += 64)
        for (int j = 0; j < 4; ++j)
            for (int l = 0; l < 16; ++l) a5[j][l] = fmaf(x[i + 16 * j + l], y[i + 16 * j + l], a5[j][l]);
    for (int j = 0; j < 4; ++j)
        for (int l = 0; l < 8; ++l) a[j][l] = a5[j][l] + a5[j][l + 8];
    for (; i < n; i += 32)
        for (int j = 0; j < 4; ++j)
            for (int l = 0; l < 8; ++l) a[j][l] = fmaf(x[i + 8 * j + l], y[i + 8 * j + l], a[j][l]);
    float s[8], h[4];
    for (int l = 0; l < 8; ++l) s[l] = ((a[0][l] + a[1][l]) + a[2][l]) + a[3][l];
    for (int l = 0; l < 4; ++l) h[l] = s[l] + s[l + 4];
    return (h[0] + h[1]) + (h[2] + h[3]);
}

static double sdot_chunk(int64_t n, const float* x, const float* y) {
    const int64_t n1 = n & ~(int64_t)31;
    double d = n1 ? (double)sdot_k16(n1, x, y) : 0.0;
    for (int64_t i = n1; i < n; ++i) d += (double)(y[i] * x[i]);
    return d;
}

float oracle_ref_sdot(const float* x, const float* y, int64_t n, int threads) {
    if (n <= 0) return 0.f;
    if (threads <= 1) return (float)sdot_chunk(n, x, y);
    float dot = 0.f;
    int64_t rest = n, off = 0;
    for (int c = 0; rest > 0; ++c) {
        int64_t w = (rest + threads - c - 1) / (threads - c);
        if (w > rest) w = rest;
        dot = (float)((double)dot + sdot_chunk(w, x + off, y + off));
        rest -= w;
        off += w;
    }
    return dot;
}

static float np_pairwise(const float* a, int64_t n) {
    if (n < 8) {
        float r = 0.f;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
}

float oracle_np_sum_f32(const float* a, int64_t n) {
    float r = 0.f;
    for (int64_t o = 0; o < n; o += 8192) r += np_pairwise(a + o, n - o < 8192 ? n - o : 8192);
    return r;
}

/* The whole dot of EDT_RL/crossover.py:20-29 for inputs of dtype dt (bf16 widened to fp32 first,
 * as `.float().numpy()`); also returns the two fp32 norms. */
int oracle_ref_slerp_dot(const void* v0, const void* v1, int dt, int64_t n, int threads, float eps, float* dot,
                         float* norm0, float* norm1) {
    float* a = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    float* b = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    if (!a || !b) {
        free(a);
        free(b);
        return -1;
    }
    for (int64_t i = 0; i < n; ++i) {
        a[i] = load(v0, dt, (uint64_t)i);
        b[i] = load(v1, dt, (uint64_t)i);
    }
    const float n0 = sqrtf(oracle_ref_sdot(a, a, n, threads));
    const float n1 = sqrtf(oracle_ref_sdot(b, b, n, threads));
    for (int64_t i = 0; i < n; ++i) {
        const float x = n0 > eps ? a[i] / n0 : a[i];
        const float y = n1 > eps ? b[i] / n1 : b[i];
        a[i] = x * y;
    }
    *dot = oracle_np_sum_f32(a, n);
    if (norm0) *norm0 = n0;
    if (norm1) *norm1 = n1;
    free(a);
    free(b);
    return 0;
}
