/* Host-side code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only, no GPU needed):
 *   1. the CPU oracle (oracle/edt_oracle.c, compiled into this binary with the sanitizers) over
 *      randomised inputs in every dtype regime, K = 1..9, with and without torch's tail mask; the
 *      sharded split (delta_partial + sgd_apply) must equal the fused step bit for bit (fp32 master);
 *   2. the host logic of libedt_sync (built host-only with the sanitizers: argument validation,
 *      the chunk table, the tensor-list table, overlap checks) through the C ABI's error paths;
 *   3. libedt_comm's argument validation.
 * SURVEY.md §5 asked for this build (the reference's own race: EDT_LM/train/runner.py:9,23-28).
 * Prints "host checks ok" and exits 0; any sanitizer report aborts with a non-zero status. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "edt_comm.h"
#include "edt_sync.h"

int oracle_outer_step(void* theta, int gdt, const void* const* workers, int wdt, int K, void* mom,
                      int has_buf, uint64_t n, double lr, double mu, int nesterov, const uint8_t* tail);
int oracle_delta_partial(const void* theta, int gdt, const void* const* workers, int wdt, int K,
                         int K_total, uint64_t n, float* acc, int accumulate);
int oracle_sgd_apply(void* theta, int gdt, const float* acc, void* mom, int has_buf, uint64_t n,
                     double lr, double mu, int nesterov);
int oracle_pair_merge(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                      void* theta_out, int gdt, void* mom, int has_buf, uint64_t n, double lr,
                      double mu, int nesterov, const uint8_t* tail);
int oracle_lerp(const void* v0, const void* v1, int in_dt, void* out, int out_dt, int cdt, uint64_t n,
                double t);

static int failures = 0;
#define EXPECT(c)                                                               \
    do {                                                                        \
        if (!(c)) {                                                             \
            fprintf(stderr, "%s:%d: expected %s\n", __FILE__, __LINE__, #c);    \
            ++failures;                                                         \
        }                                                                       \
    } while (0)
#define EXPECT_FAIL(rc) EXPECT((rc) < 0 && edt_last_error()[0] != 0)

static uint64_t lcg = 0x9E3779B97F4A7C15ull;
static float uniform(void) {
    lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
    return (float)((int64_t)(lcg >> 11) - (1ll << 52)) / (float)(1ll << 52);
}
static uint16_t to_bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static void* fill(uint64_t n, int dt, float scale, const float* base) {
    void* p = malloc(n * (dt ? 2 : 4));
    for (uint64_t i = 0; i < n; ++i) {
        float v = (base ? base[i] : 0.f) + scale * uniform();
        if (dt) ((uint16_t*)p)[i] = to_bf(v);
        else ((float*)p)[i] = v;
    }
    return p;
}

static void oracle_checks(void) {
    const int regimes[3][2] = {{0, 0}, {0, 1}, {1, 1}};
    for (int r = 0; r < 3; ++r)
        for (int K = 1; K <= 9; ++K) {
            const uint64_t n = 4099 + 37 * K;
            const int gdt = regimes[r][0], wdt = regimes[r][1];
            float* base = malloc(n * 4);
            for (uint64_t i = 0; i < n; ++i) base[i] = 0.02f * uniform();
            void* th = fill(n, gdt, 0.f, base);
            void* th2 = fill(n, gdt, 0.f, base);
            void* mom = fill(n, gdt, 1e-3f, NULL);
            void* mom2 = malloc(n * (gdt ? 2 : 4));
            memcpy(mom2, mom, n * (gdt ? 2 : 4));
            const void* w[9];
            for (int k = 0; k < K; ++k) w[k] = fill(n, wdt, 1e-3f, base);
            uint8_t* tail = calloc(n, 1);
            for (uint64_t i = n - 31; i < n; ++i) tail[i] = 1;
            EXPECT(oracle_outer_step(th, gdt, w, wdt, K, mom, 1, n, 0.7, 0.9, 1, (K & 1) ? tail : NULL) == 0);
            if (gdt == 0) {    /* fp32 master: the sharded split is the fused step, bit for bit */
                float* acc = malloc(n * 4);
                EXPECT(oracle_delta_partial(th2, gdt, w, wdt, K, K, n, acc, 0) == 0);
                EXPECT(oracle_sgd_apply(th2, gdt, acc, mom2, 1, n, 0.7, 0.9, 1) == 0);
                if (!(K & 1)) EXPECT(memcmp(th, th2, n * 4) == 0 && memcmp(mom, mom2, n * 4) == 0);
                free(acc);
            }
            void* out = malloc(n * (gdt ? 2 : 4));
            if (K >= 2) {
                EXPECT(oracle_pair_merge(w[0], w[1], w[0], w[1], wdt, out, gdt, mom, 1, n, 0.7, 0.9, 1, tail) == 0);
                EXPECT(oracle_pair_merge(th, NULL, w[0], w[1], wdt, out, gdt, mom, 0, n, 0.7, 0.0, 0, NULL) == 0);
            }
            EXPECT(oracle_lerp(w[0], w[K - 1], wdt, out, gdt, gdt, n, 0.5) == 0);
            for (int k = 0; k < K; ++k) free((void*)w[k]);
            free(base); free(th); free(th2); free(mom); free(mom2); free(tail); free(out);
        }
}

static void sync_host_paths(void) {
    EXPECT(edt_outer_step_bytes_per_elem(0, 1, 8, 1) == 32);
    EXPECT(strncmp(edt_version(), "edt_sync", 8) == 0);
    /* chunk table: count query, exact fill, truncated fill, decreasing offsets */
    const uint64_t offs[6] = {0, 5, 5, 70000, 200001, 200009};
    const int nseg = 5;
    int32_t first[6];
    int64_t need = edt_slerp_make_chunks(offs, nseg, 65536, NULL, 0, first);
    EXPECT(need < 0);
    const int64_t nc = -need - 1;
    uint64_t* desc = malloc(3 * sizeof(uint64_t) * (size_t)nc);
    EXPECT(edt_slerp_make_chunks(offs, nseg, 65536, desc, nc, first) == nc);
    uint64_t at = 0;
    for (int64_t c = 0; c < nc; ++c) {
        EXPECT(desc[3 * c] == at && desc[3 * c + 1] > 0 && desc[3 * c + 1] <= 65536);
        EXPECT(offs[desc[3 * c + 2]] <= desc[3 * c] && desc[3 * c] + desc[3 * c + 1] <= offs[desc[3 * c + 2] + 1]);
        at += desc[3 * c + 1];
    }
    EXPECT(at == offs[nseg] && first[nseg] == nc && first[1] == first[2]);
    uint64_t* small = malloc(3 * sizeof(uint64_t) * 2);
    EXPECT(edt_slerp_make_chunks(offs, nseg, 65536, small, 2, first) == -nc - 1);   /* no overflow */
    const uint64_t bad[3] = {0, 10, 4};
    EXPECT_FAIL(edt_slerp_make_chunks(bad, 2, 16, NULL, 0, NULL));
    free(desc); free(small);

    /* argument validation of the launches (fails before any HIP call) */
    _Alignas(16) static float dummy[64 * 64];
    void* d = dummy;
    const void* w65[65];
    for (int k = 0; k < 65; ++k) w65[k] = d;
    EXPECT_FAIL(edt_outer_step(NULL, 0, w65, 0, 2, d, 0, 100, 0.7, 0.9, 1, NULL));
    EXPECT_FAIL(edt_outer_step(d, 0, w65, 0, 0, d, 0, 100, 0.7, 0.9, 1, NULL));
    EXPECT_FAIL(edt_outer_step(d, 0, w65, 0, 65, d, 0, 100, 0.7, 0.9, 1, NULL));
    EXPECT_FAIL(edt_outer_step(d, 1, w65, 0, 2, d, 0, 100, 0.7, 0.9, 1, NULL));      /* bf16 master, fp32 workers */
    EXPECT_FAIL(edt_outer_step(d, 0, w65, 0, 2, NULL, 0, 100, 0.7, 0.9, 1, NULL));   /* momentum needed */
    void* b65[65];
    for (int k = 0; k < 65; ++k) b65[k] = dummy + 64 * (k % 60);
    EXPECT_FAIL(edt_outer_step_bcast(d, 0, w65, 0, 2, d, 0, 100, 0.7, 0.9, 1, b65, 65, NULL));
    void* over[1] = {dummy + 10};
    EXPECT_FAIL(edt_outer_step_bcast(d, 0, w65, 0, 2, dummy + 2000, 0, 100, 0.7, 0.9, 1, over, 1, NULL));
    EXPECT_FAIL(edt_outer_step_ws(d, 0, w65, 0, 65, d, 0, 100, 0.7, 0.9, 1, NULL, NULL));
    void* tt[2] = {d, d};
    const uint64_t numel[2] = {100, 0};
    EXPECT(edt_outer_list_workspace_bytes(2, 3) == (5 * 2 + 1 + 3 * 2) * 8);   /* r5: + the tail offsets */
    EXPECT_FAIL(edt_outer_step_list(tt, 0, w65, 0, 3, tt, 1, numel, 2, 0.7, 0.9, 1, NULL, 0, NULL));
    EXPECT_FAIL(edt_outer_step_list(tt, 0, w65, 0, 3, tt, 1, numel, 2, 0.7, 0.9, 1, d, 8, NULL));
    const void* nullw[6] = {d, NULL, d, d, d, d};
    EXPECT_FAIL(edt_outer_step_list(tt, 0, nullw, 0, 3, tt, 1, numel, 2, 0.7, 0.9, 1, d, 1024, NULL));
    EXPECT_FAIL(edt_delta_partial(d, 0, w65, 0, 2, 4, 100, NULL, 0, NULL));
    EXPECT_FAIL(edt_sgd_apply(d, 3, (const float*)d, d, 0, 100, 0.7, 0.9, 1, NULL));
    EXPECT_FAIL(edt_lerp(d, d, 2, d, 0, 0, 100, 0.5, NULL));
    void* outs17[17];
    int32_t has17[17] = {0};
    for (int k = 0; k < 17; ++k) outs17[k] = d;
    EXPECT_FAIL(edt_pair_merge_population(w65, w65, w65, w65, 1, outs17, 1, w65, outs17, has17, 17, 100,
                                          0.7, 0.9, 1, NULL));
    const int32_t pairs[4] = {0, 1, 0, 7};
    const void* mem2[2] = {dummy, dummy + 512};
    void* out2[2] = {dummy + 1024, dummy + 1536};
    double tv[2] = {0.5, 0.5};
    float coef[8];
    EXPECT_FAIL(edt_slerp_population(mem2, 9, 1, pairs, 1, out2, 1, (const uint64_t*)d, 1, first, 1, tv, 0.9995,
                                     1e-8, (double*)d, coef, NULL, NULL));
    EXPECT_FAIL(edt_slerp_population(mem2, 2, 1, pairs, 2, out2, 1, (const uint64_t*)d, 1, first, 1, tv, 0.9995,
                                     1e-8, (double*)d, coef, NULL, NULL));   /* member 7 out of range */
    void* alias[2] = {dummy, dummy + 1536};
    EXPECT_FAIL(edt_slerp_population(mem2, 2, 1, pairs, 1, alias, 1, (const uint64_t*)d, 1, first, 1, tv, 0.9995,
                                     1e-8, (double*)d, coef, NULL, NULL));   /* output aliases a member */
    EXPECT_FAIL(edt_slerp_merge_list((const void* const*)tt, (const void* const*)tt, 1, tt, 1, (const uint64_t*)d, 1,
                                     first, 2, tv, 0.9995, 1e-8, (double*)d, coef, NULL, d, 8, NULL));
    EXPECT_FAIL(edt_slerp_needed_sums(mem2, 9, 1, pairs, 1, (const uint64_t*)d, 1, 1, 0, (double*)d, (double*)d, 64,
                                      NULL));                                 /* 9 members */
    EXPECT_FAIL(edt_slerp_needed_coef((const double*)d, 1, pairs, 2, 2, first, 1, tv, 0.9995, 1e-8, coef, NULL,
                                      NULL));                                 /* member 7 of 2 */
    EXPECT_FAIL(edt_slerp_blend_children(mem2, 2, 1, pairs, 17, outs17, 1, (const uint64_t*)d, 1, coef, 1, NULL));
    EXPECT_FAIL(edt_slerp_merge_speculative(d, dummy + 8, 1, dummy + 4, 1, (const uint64_t*)d, 1, first, 1, tv,
                                            0.9995, 1e-8, (double*)d, coef, NULL, (int32_t*)d, 100, NULL));
    /* r5: the list step's tail masks need a bf16 master and byte offsets */
    const uint64_t toff[2] = {0, 13};
    EXPECT_FAIL(edt_outer_step_list_tail(tt, 0, w65, 0, 3, tt, 1, numel, 2, 0.7, 0.9, 1, (const uint8_t*)d, toff,
                                         d, 1024, NULL));
    EXPECT_FAIL(edt_outer_step_list_tail(tt, 1, w65, 1, 3, tt, 1, numel, 2, 0.7, 0.9, 1, (const uint8_t*)d, NULL,
                                         d, 1024, NULL));
    /* r5: the population planner (host only) — roulette-like graphs, the fallbacks, bad input */
    char buf[4096];
    const int32_t rl[16] = {0, 5, 5, 2, 0, 1, 5, 2, 6, 3, 6, 7, 5, 3, 7, 2};
    EXPECT(edt_slerp_population_layout(rl, 8, 8, 1, buf, (int)sizeof(buf)) == 0);
    EXPECT(strstr(buf, "\"member-major\"") != NULL && strstr(buf, "\"needed\"") != NULL);
    int32_t k5[20];
    int nk = 0;
    for (int a = 0; a < 5; ++a)
        for (int b = a + 1; b < 5; ++b) { k5[2 * nk] = a; k5[2 * nk + 1] = b; ++nk; }
    EXPECT(edt_slerp_population_layout(k5, nk, 5, 1, buf, (int)sizeof(buf)) == 0);
    EXPECT(strstr(buf, "\"co-located\"") != NULL && strstr(buf, "\"triangle\"") != NULL);
    EXPECT_FAIL(edt_slerp_population_layout(rl, 8, 4, 1, buf, (int)sizeof(buf)));   /* member 5 of 4 */
    EXPECT_FAIL(edt_slerp_population_layout(rl, 8, 8, 1, buf, 16));                  /* short buffer */
    EXPECT_FAIL(edt_slerp_population_layout(rl, 8, 8, 1, NULL, 16));
    /* r5: the needed-sums table of the sharded population (host only) */
    uint64_t boff[8], tdoubles = 0, sdoubles = 0;
    int32_t bnt[8], ncomp = 0, cols[2 * 36 * 8];
    EXPECT(edt_slerp_needed_table(rl, 8, 8, 100, boff, bnt, &ncomp, cols, &tdoubles, &sdoubles) == 0);
    EXPECT(ncomp >= 1 && boff[0] == 0 && tdoubles >= 100ull * (uint64_t)bnt[0] && sdoubles > 0);
    EXPECT(cols[0] >= 0 && cols[0] == cols[1]);                          /* column 0: a norm */
    EXPECT_FAIL(edt_slerp_needed_table(rl, 8, 4, 100, boff, bnt, &ncomp, cols, &tdoubles, &sdoubles));
    EXPECT_FAIL(edt_slerp_needed_table(rl, 0, 8, 100, boff, bnt, &ncomp, cols, &tdoubles, &sdoubles));
    EXPECT_FAIL(edt_slerp_needed_table(rl, 8, 8, 100, NULL, bnt, &ncomp, cols, &tdoubles, &sdoubles));
    const void* mem8[8] = {d, d, d, d, d, d, d, d};
    EXPECT_FAIL(edt_slerp_needed_sums(mem8, 8, 1, rl, 8, (const uint64_t*)d, 10, 100, 95, (double*)d, (double*)d,
                                      sdoubles, NULL));                  /* rows past the table */
    EXPECT_FAIL(edt_slerp_needed_sums(mem8, 8, 1, rl, 8, (const uint64_t*)d, 10, 100, 0, (double*)d, (double*)d,
                                      0, NULL));                         /* scratch too small */
    EXPECT_FAIL(edt_slerp_needed_coef((const double*)d, 100, rl, 8, 9, first, 1, tv, 0.9995, 1e-8, coef, NULL, NULL));
    /* r5: edt_slerp_seg_table's in-place rule (apart = 0 with sizes): an output may be exactly its
     * own parent, never overlap another tensor's parent or output */
    uint64_t host[6];
    const uint64_t n2[2] = {16, 16};
    const void* v0s[2] = {dummy, dummy + 64};
    const void* v1s[2] = {dummy + 128, dummy + 192};
    void* own[2] = {dummy, dummy + 192};                      /* in place: tensor 0 into v0, 1 into v1 */
    EXPECT(edt_slerp_seg_table(v0s, v1s, own, 2, n2, 0, 0, 0, host) == 0);
    void* other[2] = {dummy + 64, dummy + 256};               /* tensor 0 written over tensor 1's parent */
    EXPECT_FAIL(edt_slerp_seg_table(v0s, v1s, other, 2, n2, 0, 0, 0, host));
    void* partial[2] = {dummy + 8, dummy + 256};              /* across its own parent, not exactly it */
    EXPECT_FAIL(edt_slerp_seg_table(v0s, v1s, partial, 2, n2, 0, 0, 0, host));
    void* same[2] = {dummy + 256, dummy + 256};               /* two outputs on one buffer */
    EXPECT_FAIL(edt_slerp_seg_table(v0s, v1s, same, 2, n2, 0, 0, 0, host));
    EXPECT_FAIL(edt_slerp_seg_table(v0s, v1s, other, 2, NULL, 0, 0, 0, host));   /* r6: sizes required */
}

static void comm_host_paths(void) {
    EXPECT(edt_comm_id_bytes() == 128);
    EXPECT(edt_comm_poll(NULL) == EDT_COMM_ERR_ARG);
    EXPECT(edt_comm_abort(NULL) == EDT_COMM_ERR_ARG);
    EXPECT(edt_comm_set_timeout(NULL, 1.0) == EDT_COMM_ERR_ARG);
    EXPECT(edt_comm_wait(NULL, NULL, 1.0) == EDT_COMM_ERR_ARG);
    EXPECT(edt_comm_reduce_scatter_f32(NULL, NULL, NULL, 4, NULL) == EDT_COMM_ERR_ARG);
    EXPECT(edt_outer_step_sharded(NULL, NULL, 0, NULL, 0, 1, NULL, 0, 64, 64, 0.7, 0.9, 1, NULL, NULL) ==
           EDT_COMM_ERR_ARG);
    EXPECT(edt_outer_step_sharded_ordered(NULL, NULL, 0, NULL, 0, 1, NULL, 0, 64, 64, 0.7, 0.9, 1, NULL, NULL,
                                          NULL) == EDT_COMM_ERR_ARG);
    EXPECT(edt_outer_step_sharded_exact(NULL, NULL, 0, NULL, 0, 1, NULL, 0, 64, 64, 0.7, 0.9, 1, NULL, NULL) ==
           EDT_COMM_ERR_ARG);
    EXPECT(edt_comm_last_error()[0] != 0);
    char id[128];
    void* comm = NULL;
    EXPECT(edt_comm_init(&comm, id, 0, 0) == EDT_COMM_ERR_ARG);
    EXPECT(edt_comm_init(&comm, id, 2, 2) == EDT_COMM_ERR_ARG);
    EXPECT(edt_comm_destroy(NULL) == 0);
}

int main(void) {
    oracle_checks();
    sync_host_paths();
    comm_host_paths();
    if (failures) {
        fprintf(stderr, "%d host checks failed\n", failures);
        return 1;
    }
    printf("host checks ok\n");
    return 0;
}
