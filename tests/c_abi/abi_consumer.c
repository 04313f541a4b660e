/* A plain-C consumer of the drop-in boundary (include/edt_sync.h), with no Python and no torch:
 * what a cgo / JNI / N-API binding of the reference's DiLoCo step would do.
 * Device buffers come from hipMalloc; two outer steps (first: no carried buffer, second: carried)
 * run on the null stream through edt_outer_step, and theta and the momentum are compared bit for
 * bit with the CPU oracle's restatement of EDT_LM/diloco.py:238-289 (oracle/_build/liboracle.so,
 * test infrastructure). Then the error convention: a bad dtype code returns a negative EDT_ERR_*
 * and edt_last_error() says why. Prints "abi consumer ok" and exits 0 on success. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "edt_sync.h"

/* oracle/edt_oracle.c */
int oracle_outer_step(void* theta, int gdt, const void* const* workers, int wdt, int K, void* mom,
                      int has_buf, uint64_t n, double lr, double mu, int nesterov, const uint8_t* tail);

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

int main(void) {
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
    printf("abi consumer ok\n");
    return 0;
}
