/* A plain-C consumer of the drop-in boundary (include/edt_sync.h), with no Python and no torch:
 * what a cgo / JNI / N-API binding of the reference's DiLoCo step would do.
 * Device buffers come from hipMalloc; two outer steps (first: no carried buffer, second: carried)
 * run on the null stream through edt_outer_step, and theta and the momentum are compared bit for
 * bit with the CPU oracle's restatement of EDT_LM/diloco.py:238-289 (oracle/_build/liboracle.so,
 * test infrastructure). Then the error convention: a bad dtype code returns a negative EDT_ERR_*
 * and edt_last_error() says why. Then the SLERP crossover over separate tensors as a binding of
 * EDT_RL/crossover.py:84-135 would drive it (edt_slerp_make_chunks -> relative chunk starts ->
 * edt_slerp_merge_list, and the single-pass edt_slerp_merge_list_speculative): parents of one
 * lineage, so every tensor takes the lerp branch, whose output is compared bit for bit with the
 * oracle's lerp, and the two forms with each other (outputs and dots). Then a resident
 * population (population_check). Prints "abi consumer ok" and exits 0 on success. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "edt_sync.h"

/* oracle/edt_oracle.c */
int oracle_outer_step(void* theta, int gdt, const void* const* workers, int wdt, int K, void* mom,
                      int has_buf, uint64_t n, double lr, double mu, int nesterov, const uint8_t* tail);
int oracle_lerp(const void* v0, const void* v1, int in_dt, void* out, int out_dt, int cdt, uint64_t n, double t);

#define K 3
#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 2;                                                          \
        }                                                                      \
    } while (0)

static uint64_t lcg = 0x9E3779B97F4A7C15ull;
static float uniform(void) { /* in (-1, 1) */
    lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
    return (float)((int64_t)(lcg >> 11) - (1ll << 52)) / (float)(1ll << 52);
}

#define NSEG 4
/* The tensor-list SLERP of three ragged tensors (+ an empty one) through the C ABI, both forms. */
static int slerp_list_check(void) {
    const uint64_t sizes[NSEG] = {70001, 0, 131073, 4099};
    uint64_t offs[NSEG + 1] = {0};
    for (int s = 0; s < NSEG; ++s) offs[s + 1] = offs[s] + sizes[s];
    int32_t first[NSEG + 1];
    /* sizing call: no table given, so the count comes back as -(count) - 1 */
    const int64_t need = edt_slerp_make_chunks(offs, NSEG, 1u << 16, NULL, 0, first);
    const int64_t nchunks = need < 0 ? -need - 1 : need;
    if (nchunks <= 0) {
        fprintf(stderr, "edt_slerp_make_chunks: %lld %s\n", (long long)nchunks, edt_last_error());
        return 1;
    }
    uint64_t* desc = malloc(3 * nchunks * sizeof(uint64_t));
    if (edt_slerp_make_chunks(offs, NSEG, 1u << 16, desc, nchunks, first) != nchunks) return 1;
    for (int64_t c = 0; c < nchunks; ++c) desc[3 * c] -= offs[desc[3 * c + 2]];    /* relative starts */
    const double tv[NSEG] = {0.5, 0.3, 0.43, 0.9};
    void *d_v0[NSEG], *d_v1[NSEG], *d_a[NSEG], *d_b[NSEG];
    float *h0[NSEG], *h1[NSEG], *want[NSEG], *got = malloc(sizes[2] * sizeof(float) + 16);
    for (int s = 0; s < NSEG; ++s) {
        const size_t nb = sizes[s] * sizeof(float);
        h0[s] = malloc(nb + 16);
        h1[s] = malloc(nb + 16);
        want[s] = malloc(nb + 16);
        for (uint64_t i = 0; i < sizes[s]; ++i) {
            h0[s][i] = 0.02f * uniform();
            h1[s][i] = h0[s][i] * (1.0f + 1e-3f * uniform());      /* one lineage: |dot| > 0.9995 */
        }
        oracle_lerp(h0[s], h1[s], EDT_F32, want[s], EDT_F32, EDT_F32, sizes[s], tv[s]);
        d_v0[s] = d_v1[s] = d_a[s] = d_b[s] = NULL;
        if (!nb) continue;
        CK(hipMalloc(&d_v0[s], nb));
        CK(hipMalloc(&d_v1[s], nb));
        CK(hipMalloc(&d_a[s], nb));
        CK(hipMalloc(&d_b[s], nb));
        CK(hipMemcpy(d_v0[s], h0[s], nb, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_v1[s], h1[s], nb, hipMemcpyHostToDevice));
    }
    void *d_desc, *d_first, *d_t, *d_partial, *d_coef, *d_dots_a, *d_dots_b, *d_redo, *d_ws;
    const uint64_t nd = edt_slerp_sums_doubles(3, nchunks);
    CK(hipMalloc(&d_desc, 3 * nchunks * sizeof(uint64_t)));
    CK(hipMalloc(&d_first, sizeof(first)));
    CK(hipMalloc(&d_t, sizeof(tv)));
    CK(hipMalloc(&d_partial, nd * sizeof(double)));
    CK(hipMalloc(&d_coef, 2 * NSEG * sizeof(float)));
    CK(hipMalloc(&d_dots_a, NSEG * sizeof(float)));
    CK(hipMalloc(&d_dots_b, NSEG * sizeof(float)));
    CK(hipMalloc(&d_redo, NSEG * sizeof(int32_t)));
    CK(hipMalloc(&d_ws, 3 * NSEG * sizeof(uint64_t)));
    CK(hipMemcpy(d_desc, desc, 3 * nchunks * sizeof(uint64_t), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_first, first, sizeof(first), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_t, tv, sizeof(tv), hipMemcpyHostToDevice));
    int rc = edt_slerp_merge_list((const void* const*)d_v0, (const void* const*)d_v1, EDT_F32, d_a, EDT_F32, d_desc,
                                  nchunks, d_first, NSEG, d_t, 0.9995, 1e-8, d_partial, d_coef, d_dots_a, d_ws,
                                  3 * NSEG * sizeof(uint64_t), NULL);
    if (rc == 0)
        rc = edt_slerp_merge_list_speculative((const void* const*)d_v0, (const void* const*)d_v1, EDT_F32, d_b,
                                              EDT_F32, sizes, d_desc, nchunks, d_first, NSEG, d_t, 0.9995, 1e-8,
                                              d_partial, d_coef, d_dots_b, d_redo, d_ws, 3 * NSEG * sizeof(uint64_t),
                                              NULL);
    if (rc != 0) {
        fprintf(stderr, "slerp list: %d %s\n", rc, edt_last_error());
        return 1;
    }
    /* an output that is its own parent: the speculative form refuses it, nothing launched */
    rc = edt_slerp_merge_list_speculative((const void* const*)d_v0, (const void* const*)d_v1, EDT_F32, d_v0,
                                          EDT_F32, sizes, d_desc, nchunks, d_first, NSEG, d_t, 0.9995, 1e-8,
                                          d_partial, d_coef, d_dots_b, d_redo, d_ws, 3 * NSEG * sizeof(uint64_t),
                                          NULL);
    if (rc >= 0) {
        fprintf(stderr, "speculative list form accepted an output aliasing its parent\n");
        return 1;
    }
    CK(hipDeviceSynchronize());
    float da[NSEG], db[NSEG];
    CK(hipMemcpy(da, d_dots_a, sizeof(da), hipMemcpyDeviceToHost));
    CK(hipMemcpy(db, d_dots_b, sizeof(db), hipMemcpyDeviceToHost));
    for (int s = 0; s < NSEG; ++s) {
        if (!sizes[s]) continue;
        if (memcmp(&da[s], &db[s], sizeof(float)) != 0 || !(da[s] > 0.9995f)) {
            fprintf(stderr, "tensor %d: dots %.9g / %.9g\n", s, da[s], db[s]);
            return 1;
        }
        for (int form = 0; form < 2; ++form) {
            CK(hipMemcpy(got, form ? d_b[s] : d_a[s], sizes[s] * sizeof(float), hipMemcpyDeviceToHost));
            if (memcmp(got, want[s], sizes[s] * sizeof(float)) != 0) {
                fprintf(stderr, "tensor %d (%s form) differs from the oracle's lerp\n", s,
                        form ? "speculative" : "two-pass");
                return 1;
            }
        }
        hipFree(d_v0[s]);
        hipFree(d_v1[s]);
        hipFree(d_a[s]);
        hipFree(d_b[s]);
    }
    printf("slerp list (two-pass and speculative): %lld chunks, bit-exact with the oracle's lerp branch\n",
           (long long)nchunks);
    return 0;
}

/* A resident population through the C ABI (BASELINE configs[4], EDT_RL/edt.py:286-299): 6 members
 * of 5 ragged tensors in flat arenas, 8 children on a roulette-like pair graph (a hub parent, a
 * repeated pair, a reversed pair, a self-pair), lineage members so most tensors take the lerp
 * branch and two far members the SLERP branch. Three routes, every child bit for bit:
 *   edt_slerp_population_speculative (the one-pass form) against edt_slerp_merge per child;
 *   the sharded stages at one rank — edt_slerp_needed_table, edt_slerp_needed_sums over two chunk
 *   ranges (rows written where they belong), edt_slerp_needed_coef, edt_slerp_blend_children —
 *   against the same. */
#define PM 6
#define PQ 8
#define PSEG 5
static int population_check(void) {
    const uint64_t sizes[PSEG] = {70001, 9, 131072, 4099, 1};
    uint64_t offs[PSEG + 1] = {0};
    for (int s = 0; s < PSEG; ++s) offs[s + 1] = offs[s] + sizes[s];
    const uint64_t n = offs[PSEG];
    int32_t first[PSEG + 1];
    const int64_t need = edt_slerp_make_chunks(offs, PSEG, 8192u, NULL, 0, first);
    const int64_t nchunks = need < 0 ? -need - 1 : need;
    uint64_t* desc = malloc(3 * nchunks * sizeof(uint64_t));
    if (nchunks <= 0 || edt_slerp_make_chunks(offs, PSEG, 8192u, desc, nchunks, first) != nchunks) return 1;
    const int32_t pairs[2 * PQ] = {0, 5, 5, 2, 0, 1, 5, 3, 2, 5, 4, 4, 1, 0, 5, 2};
    const double tv[PSEG] = {0.5, 0.3, 0.43, 0.9, 0.5};
    float* base = malloc(n * sizeof(float));
    for (uint64_t i = 0; i < n; ++i) base[i] = 0.02f * uniform();
    void *d_mem[PM], *d_out[PQ], *d_out2[PQ], *d_want;
    float* h = malloc(n * sizeof(float));
    for (int m = 0; m < PM; ++m) {
        const float rel = (m == 3 || m == 4) ? 0.5f : 1e-3f;          /* members 3, 4 far from the lineage */
        for (uint64_t i = 0; i < n; ++i) h[i] = base[i] + 0.02f * rel * uniform();
        CK(hipMalloc(&d_mem[m], n * sizeof(float)));
        CK(hipMemcpy(d_mem[m], h, n * sizeof(float), hipMemcpyHostToDevice));
    }
    for (int q = 0; q < PQ; ++q) {
        CK(hipMalloc(&d_out[q], n * sizeof(float)));
        CK(hipMalloc(&d_out2[q], n * sizeof(float)));
    }
    CK(hipMalloc(&d_want, n * sizeof(float)));
    void *d_desc, *d_first, *d_t, *d_partial, *d_coef, *d_dots, *d_redo, *d_pcoef, *d_pdots;
    const uint64_t spec = edt_slerp_population_speculative_doubles(PQ, nchunks);
    const uint64_t pair_nd = edt_slerp_sums_doubles(3, nchunks);
    CK(hipMalloc(&d_desc, 3 * nchunks * sizeof(uint64_t)));
    CK(hipMalloc(&d_first, sizeof(first)));
    CK(hipMalloc(&d_t, sizeof(tv)));
    CK(hipMalloc(&d_partial, (spec > pair_nd ? spec : pair_nd) * sizeof(double)));
    CK(hipMalloc(&d_coef, 2 * PQ * PSEG * sizeof(float)));
    CK(hipMalloc(&d_dots, PQ * PSEG * sizeof(float)));
    CK(hipMalloc(&d_redo, PQ * PSEG * sizeof(int32_t)));
    CK(hipMalloc(&d_pcoef, 2 * PSEG * sizeof(float)));
    CK(hipMalloc(&d_pdots, PSEG * sizeof(float)));
    CK(hipMemcpy(d_desc, desc, 3 * nchunks * sizeof(uint64_t), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_first, first, sizeof(first), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_t, tv, sizeof(tv), hipMemcpyHostToDevice));
    int rc = edt_slerp_population_speculative((const void* const*)d_mem, PM, EDT_F32, pairs, PQ, d_out, EDT_F32, d_desc,
                                              nchunks, d_first, PSEG, d_t, 0.9995, 1e-8, d_partial, d_coef, d_dots,
                                              d_redo, n, NULL);
    if (rc != 0) {
        fprintf(stderr, "edt_slerp_population_speculative: %d %s\n", rc, edt_last_error());
        return 1;
    }
    /* the sharded stages at one rank: the needed table, its rows in two chunk ranges */
    uint64_t boff[8], tdoubles = 0, sdoubles = 0;
    int32_t bnt[8], ncomp = 0;
    rc = edt_slerp_needed_table(pairs, PQ, PM, nchunks, boff, bnt, &ncomp, NULL, &tdoubles, &sdoubles);
    void *d_table, *d_scratch, *d_desc2;
    CK(hipMalloc(&d_table, tdoubles * sizeof(double)));
    CK(hipMalloc(&d_scratch, sdoubles * sizeof(double)));
    const int64_t cut = nchunks / 3;
    CK(hipMalloc(&d_desc2, 3 * nchunks * sizeof(uint64_t)));
    CK(hipMemcpy(d_desc2, desc, 3 * nchunks * sizeof(uint64_t), hipMemcpyHostToDevice));
    if (rc == 0)
        rc = edt_slerp_needed_sums((const void* const*)d_mem, PM, EDT_F32, pairs, PQ, d_desc2, cut, nchunks, 0,
                                   d_table, d_scratch, sdoubles, NULL);
    if (rc == 0)
        rc = edt_slerp_needed_sums((const void* const*)d_mem, PM, EDT_F32, pairs, PQ,
                                   (const uint64_t*)d_desc2 + 3 * cut, nchunks - cut, nchunks, cut, d_table,
                                   d_scratch, sdoubles, NULL);
    if (rc == 0)
        rc = edt_slerp_needed_coef(d_table, nchunks, pairs, PQ, PM, d_first, PSEG, d_t, 0.9995, 1e-8, d_coef, NULL,
                                   NULL);
    if (rc == 0)
        rc = edt_slerp_blend_children((const void* const*)d_mem, PM, EDT_F32, pairs, PQ, d_out2, EDT_F32, d_desc,
                                      nchunks, d_coef, PSEG, NULL);
    if (rc != 0) {
        fprintf(stderr, "needed-sums stages: %d %s\n", rc, edt_last_error());
        return 1;
    }
    float *a = malloc(n * sizeof(float)), *b = malloc(n * sizeof(float)), *w = malloc(n * sizeof(float));
    int slerp_branch = 0;
    for (int q = 0; q < PQ; ++q) {
        rc = edt_slerp_merge(d_mem[pairs[2 * q]], d_mem[pairs[2 * q + 1]], EDT_F32, d_want, EDT_F32, d_desc, nchunks,
                             d_first, PSEG, d_t, 0.9995, 1e-8, d_partial, d_pcoef, d_pdots, NULL);
        if (rc != 0) {
            fprintf(stderr, "edt_slerp_merge: %d %s\n", rc, edt_last_error());
            return 1;
        }
        CK(hipDeviceSynchronize());
        float pd[PSEG];
        CK(hipMemcpy(pd, d_pdots, sizeof(pd), hipMemcpyDeviceToHost));
        for (int s = 0; s < PSEG; ++s) slerp_branch += !(pd[s] > 0.9995f || pd[s] < -0.9995f);
        CK(hipMemcpy(w, d_want, n * sizeof(float), hipMemcpyDeviceToHost));
        CK(hipMemcpy(a, d_out[q], n * sizeof(float), hipMemcpyDeviceToHost));
        CK(hipMemcpy(b, d_out2[q], n * sizeof(float), hipMemcpyDeviceToHost));
        if (memcmp(a, w, n * sizeof(float)) != 0 || memcmp(b, w, n * sizeof(float)) != 0) {
            fprintf(stderr, "child %d (%d, %d) differs from edt_slerp_merge (speculative %d, stages %d)\n", q,
                    pairs[2 * q], pairs[2 * q + 1], memcmp(a, w, n * sizeof(float)) != 0,
                    memcmp(b, w, n * sizeof(float)) != 0);
            return 1;
        }
    }
    if (slerp_branch == 0) {
        fprintf(stderr, "no child segment took the SLERP branch\n");
        return 1;
    }
    for (int m = 0; m < PM; ++m) hipFree(d_mem[m]);
    for (int q = 0; q < PQ; ++q) {
        hipFree(d_out[q]);
        hipFree(d_out2[q]);
    }
    printf("population (%d children over %d members, %d components): one-pass form and needed-sums stages "
           "bit-identical to edt_slerp_merge per child (%d SLERP-branch segments)\n", PQ, PM, ncomp, slerp_branch);
    return 0;
}

int main(void) {
    if (edt_abi_version() != EDT_ABI_VERSION) {     /* workspace sizes and signatures follow the header */
        fprintf(stderr, "library ABI %d, header ABI %d: rebuild\n", edt_abi_version(), EDT_ABI_VERSION);
        return 1;
    }
    const uint64_t n = 1000003; /* odd: exercises the scalar tail */
    const size_t nb = n * sizeof(float);
    float *theta = malloc(nb), *mom = malloc(nb), *w[K];
    float *theta_ref = malloc(nb), *mom_ref = malloc(nb), *back = malloc(nb);
    for (uint64_t i = 0; i < n; ++i) theta[i] = 0.02f * uniform();
    for (int k = 0; k < K; ++k) {
        w[k] = malloc(nb);
        for (uint64_t i = 0; i < n; ++i) w[k][i] = theta[i] + 1e-3f * uniform();
    }
    memset(mom, 0, nb);
    memcpy(theta_ref, theta, nb);
    memcpy(mom_ref, mom, nb);

    void *d_theta, *d_mom, *d_w[K];
    CK(hipMalloc(&d_theta, nb));
    CK(hipMalloc(&d_mom, nb));
    CK(hipMemcpy(d_theta, theta, nb, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_mom, mom, nb, hipMemcpyHostToDevice));
    for (int k = 0; k < K; ++k) {
        CK(hipMalloc(&d_w[k], nb));
        CK(hipMemcpy(d_w[k], w[k], nb, hipMemcpyHostToDevice));
    }
    const void* dw[K] = {d_w[0], d_w[1], d_w[2]};
    const void* hw[K] = {w[0], w[1], w[2]};
    for (int step = 0; step < 2; ++step) {
        int rc = edt_outer_step(d_theta, EDT_F32, dw, EDT_F32, K, d_mom, step, n, 0.7, 0.9, 1, NULL);
        if (rc != 0) {
            fprintf(stderr, "edt_outer_step: %d %s\n", rc, edt_last_error());
            return 1;
        }
        if (oracle_outer_step(theta_ref, EDT_F32, hw, EDT_F32, K, mom_ref, step, n, 0.7, 0.9, 1, NULL) != 0) {
            fprintf(stderr, "oracle_outer_step failed\n");
            return 1;
        }
    }
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(back, d_theta, nb, hipMemcpyDeviceToHost));
    if (memcmp(back, theta_ref, nb) != 0) {
        fprintf(stderr, "theta differs from the oracle\n");
        return 1;
    }
    CK(hipMemcpy(back, d_mom, nb, hipMemcpyDeviceToHost));
    if (memcmp(back, mom_ref, nb) != 0) {
        fprintf(stderr, "momentum differs from the oracle\n");
        return 1;
    }
    /* error convention: nothing launched, a negative code and a message */
    int rc = edt_outer_step(d_theta, 7, dw, EDT_F32, K, d_mom, 1, n, 0.7, 0.9, 1, NULL);
    if (rc >= 0 || edt_last_error() == NULL || edt_last_error()[0] == '\0') {
        fprintf(stderr, "bad dtype accepted (rc %d)\n", rc);
        return 1;
    }
    printf("edt %s: bad dtype -> %d (%s)\n", edt_version(), rc, edt_last_error());
    for (int k = 0; k < K; ++k) hipFree(d_w[k]);
    hipFree(d_theta);
    hipFree(d_mom);
    if (slerp_list_check() || population_check()) return 1;
    printf("abi consumer ok\n");
    return 0;
}
