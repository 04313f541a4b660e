/* A plain-C multi-GPU master over the drop-in boundary (include/edt_comm.h + include/edt_sync.h),
 * with no Python and no torch: what a cgo / JNI / N-API binding of the reference's DiLoCo master
 * (EDT_LM/diloco.py:238-289) would do with libedt_comm. Run at world size 1
 * (the one-GPU box): unique id -> init -> two outer steps (first: no carried buffer, second:
 * carried) with each of the three sharded schedules (edt_outer_step_sharded = reduce,
 * _ordered = reduce_ordered, _exact = exact), theta and the momentum compared bit for bit with the
 * CPU oracle's restatement (oracle/_build/liboracle.so, test infrastructure); then the failure
 * path: after edt_comm_abort every call returns EDT_COMM_ERR_ABORTED with a message.
 * Prints "comm consumer ok" and exits 0 on success. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "edt_comm.h"
#include "edt_sync.h"

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

static uint64_t lcg = 0x2545F4914F6CDD1Dull;
static float uniform(void) { /* in (-1, 1) */
    lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
    return (float)((int64_t)(lcg >> 11) - (1ll << 52)) / (float)(1ll << 52);
}

int main(void) {
    const uint64_t n = 100003, n_pad = 100032; /* n_pad: a multiple of nranks x 64 */
    const size_t nb = n_pad * sizeof(float);
    float *theta0 = calloc(n_pad, 4), *w[K], *back = malloc(nb);
    for (uint64_t i = 0; i < n; ++i) theta0[i] = 0.02f * uniform();
    for (int k = 0; k < K; ++k) {
        w[k] = calloc(n_pad, 4);
        for (uint64_t i = 0; i < n; ++i) w[k][i] = theta0[i] + 1e-3f * uniform();
    }
    /* the oracle's two steps over the padded arrays (the padding stays zero) */
    float *theta_ref = malloc(nb), *mom_ref = calloc(n_pad, 4);
    memcpy(theta_ref, theta0, nb);
    const void* hw[K] = {w[0], w[1], w[2]};
    for (int step = 0; step < 2; ++step)
        if (oracle_outer_step(theta_ref, EDT_F32, hw, EDT_F32, K, mom_ref, step, n_pad, 0.7, 0.9, 1, NULL) != 0) {
            fprintf(stderr, "oracle_outer_step failed\n");
            return 1;
        }

    void *d_theta, *d_mom, *d_w[K], *d_recv[K];
    float *d_acc, *d_acc_recv;
    CK(hipMalloc(&d_theta, nb));
    CK(hipMalloc(&d_mom, nb));
    CK(hipMalloc((void**)&d_acc, nb));
    CK(hipMalloc((void**)&d_acc_recv, nb));
    for (int k = 0; k < K; ++k) {
        CK(hipMalloc(&d_w[k], nb));
        CK(hipMalloc(&d_recv[k], nb));
        CK(hipMemcpy(d_w[k], w[k], nb, hipMemcpyHostToDevice));
    }
    const void* dw[K] = {d_w[0], d_w[1], d_w[2]};

    char id[128];
    if (edt_comm_id_bytes() > sizeof(id) || edt_comm_unique_id(id) != 0) {
        fprintf(stderr, "edt_comm_unique_id: %s\n", edt_comm_last_error());
        return 1;
    }
    void* comm = NULL;
    if (edt_comm_init(&comm, id, 1, 0) != 0) {
        fprintf(stderr, "edt_comm_init: %s\n", edt_comm_last_error());
        return 1;
    }
    const char* names[3] = {"reduce", "reduce_ordered", "exact"};
    for (int sched = 0; sched < 3; ++sched) {
        CK(hipMemcpy(d_theta, theta0, nb, hipMemcpyHostToDevice));
        CK(hipMemset(d_mom, 0, nb));
        for (int step = 0; step < 2; ++step) {
            int rc;
            if (sched == 0)
                rc = edt_outer_step_sharded(comm, d_theta, EDT_F32, dw, EDT_F32, K, d_mom, step, n_pad, 16384, 0.7,
                                            0.9, 1, d_acc, NULL);
            else if (sched == 1)
                rc = edt_outer_step_sharded_ordered(comm, d_theta, EDT_F32, dw, EDT_F32, K, d_mom, step, n_pad, 16384,
                                                    0.7, 0.9, 1, d_acc, d_acc_recv, NULL);
            else
                rc = edt_outer_step_sharded_exact(comm, d_theta, EDT_F32, dw, EDT_F32, K, d_mom, step, n_pad, 16384,
                                                  0.7, 0.9, 1, d_recv, NULL);
            if (rc != 0) {
                fprintf(stderr, "%s step %d: %d %s\n", names[sched], step, rc, edt_comm_last_error());
                return 1;
            }
        }
        if (edt_comm_wait(comm, NULL, 60.0) != 0) {
            fprintf(stderr, "edt_comm_wait: %s\n", edt_comm_last_error());
            return 1;
        }
        CK(hipMemcpy(back, d_theta, nb, hipMemcpyDeviceToHost));
        if (memcmp(back, theta_ref, nb) != 0) {
            fprintf(stderr, "%s: theta differs from the oracle\n", names[sched]);
            return 1;
        }
        CK(hipMemcpy(back, d_mom, nb, hipMemcpyDeviceToHost));
        if (memcmp(back, mom_ref, nb) != 0) {
            fprintf(stderr, "%s: momentum differs from the oracle\n", names[sched]);
            return 1;
        }
        printf("%s: bit-exact with the oracle\n", names[sched]);
    }
    /* failure path: an aborted communicator fails every later call with a message */
    if (edt_comm_abort(comm) != 0) return 1;
    int rc = edt_outer_step_sharded_exact(comm, d_theta, EDT_F32, dw, EDT_F32, K, d_mom, 1, n_pad, 16384, 0.7, 0.9, 1,
                                          d_recv, NULL);
    if (rc != EDT_COMM_ERR_ABORTED || edt_comm_last_error()[0] == '\0') {
        fprintf(stderr, "aborted communicator accepted a step (rc %d)\n", rc);
        return 1;
    }
    printf("after abort -> %d (%s)\n", rc, edt_comm_last_error());
    edt_comm_destroy(comm);
    for (int k = 0; k < K; ++k) {
        hipFree(d_w[k]);
        hipFree(d_recv[k]);
    }
    hipFree(d_theta);
    hipFree(d_mom);
    hipFree(d_acc);
    hipFree(d_acc_recv);
    printf("comm consumer ok\n");
    return 0;
}
