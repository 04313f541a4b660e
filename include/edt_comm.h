/* edt_comm.h — the cross-GPU half of the outer-loop sync behind a C ABI (libedt_comm.so):
 * RCCL over xGMI, one communicator per rank, for hosts that do not have torch.distributed.
 *
 * The reference has no collectives: its gather is K x from_pretrained of the workers' checkpoints
 * on a shared disk and its broadcast K x save_pretrained (EDT_LM/diloco.py:231-235, 302-308), and
 * its EDT children fetch their parents' checkpoint dirs (EDT_LM/train/crossover.py:255-258).
 * These entry points are the device-resident replacements (edt_comm_*); the
 * Python package reaches the same RCCL through torch.distributed (distributed.py) instead.
 *
 * Conventions as edt_sync.h: the caller owns every buffer (device pointers), all calls are
 * stream-ordered and asynchronous on `stream` (a hipStream_t; NULL = the null stream), and return
 * 0 or a negative EDT_COMM_ERR_*; edt_comm_last_error() (thread-local) says why. A communicator
 * is used by one host thread at a time.
 */
#ifndef EDT_COMM_H
#define EDT_COMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EDT_COMM_ERR_ARG (-1)
#define EDT_COMM_ERR_RCCL (-2)
#define EDT_COMM_ERR_HIP (-3)
#define EDT_COMM_ERR_ABORTED (-4)   /* the communicator was aborted (edt_comm_abort or a timeout) */
#define EDT_COMM_ERR_TIMEOUT (-5)   /* a bounded wait expired; the communicator is now aborted */

/* Bytes of the opaque communicator id (ncclUniqueId): rank 0 makes it, every rank passes the
 * same bytes to edt_comm_init (the host moves them, e.g. over its own control channel). */
uint64_t edt_comm_id_bytes(void);
int edt_comm_unique_id(void* id_out);

/* One communicator per rank: nranks ranks, this one `rank`, on the current HIP device. */
int edt_comm_init(void** comm, const void* id, int nranks, int rank);
int edt_comm_destroy(void* comm);
int edt_comm_rank(const void* comm);
int edt_comm_size(const void* comm);

/* Failure handling (the reference's master polls its workers over HTTP and gives up on the ones
 * that stop answering, EDT_LM/diloco.py:46-71, diloco_sim.py:65-68; here a dead rank would
 * otherwise leave its peers inside a collective forever):
 *   edt_comm_abort        tear the RCCL communicator down (ncclCommAbort): outstanding collectives
 *                         end, every later call on it returns EDT_COMM_ERR_ABORTED;
 *                         edt_comm_destroy still frees the handle.
 *   edt_comm_poll         0, or the asynchronous RCCL error a peer's failure left (every entry
 *                         point checks this first and refuses to enqueue on a failed communicator).
 *   edt_comm_wait         host wait until the work enqueued on `stream` and on the communicator's
 *                         own stream is done, polling the async error; after timeout_s seconds
 *                         (<= 0: no limit) the communicator is aborted -> EDT_COMM_ERR_TIMEOUT.
 *   edt_comm_set_timeout  > 0: edt_outer_step_sharded ends with edt_comm_wait(comm, stream, s)
 *                         (the step then returns when done, or fails after s seconds); 0 (the
 *                         default): it returns as soon as the work is enqueued. */
int edt_comm_abort(void* comm);
int edt_comm_poll(void* comm);
int edt_comm_wait(void* comm, void* stream, double timeout_s);
int edt_comm_set_timeout(void* comm, double seconds);

/* Collectives (dt: EDT_F32 = 0, EDT_BF16 = 1 as in edt_sync.h).
 * reduce_scatter_f32: recv[0, count) = sum over ranks of send[rank * count, +count).
 *   In place when recv == send + rank * count.
 * all_gather:  recv[r * count, +count) = rank r's send[0, count). In place when
 *   send == recv + rank * count.
 * all_to_all:  recv[r * count, +count) = rank r's send[this rank * count, +count). */
int edt_comm_reduce_scatter_f32(void* comm, const float* send, float* recv, uint64_t count_per_rank,
                                void* stream);
int edt_comm_all_gather(void* comm, const void* send, void* recv, uint64_t count_per_rank, int dt,
                        void* stream);
int edt_comm_all_to_all(void* comm, const void* send, void* recv, uint64_t count_per_rank, int dt,
                        void* stream);

/* Grouped point-to-point (the parents of each child to the rank that builds it,
 * schedule.exchange_plan): op i sends bytes[i] from sendbufs[i] to rank send_to[i] when
 * send_to[i] >= 0, and receives bytes[i] into recvbufs[i] from rank recv_from[i] when
 * recv_from[i] >= 0; all nops operations form one group (no ordering deadlock). */
int edt_comm_exchange(void* comm, const int32_t* send_to, const int32_t* recv_from,
                      const void* const* sendbufs, void* const* recvbufs, const uint64_t* bytes,
                      int nops, void* stream);

/* The DiLoCo outer step across ranks, reduce schedule (distributed.py mode="reduce"), with the
 * collectives on the communicator's own stream overlapping the kernels on `stream`. Per bucket
 * [b, e) of the padded flat arena (buckets of bucket_elems, rounded to multiples of nranks * 64;
 * n_pad a multiple of nranks * 64):
 *   edt_delta_partial over the K_local local workers into acc[b, e)  (fp32, K_total = K_local x nranks)
 *   reduce-scatter of acc[b, e) in place -> this rank's shard s = [b + rank*per, +per)
 *   edt_sgd_apply on theta[s] with the momentum shard (per elements of momentum_shard, buckets
 *   in order: the shard of rank r is n_pad / nranks elements of theta's dtype)
 *   all-gather of theta[s] in place -> theta[b, e) on every rank.
 * acc: n_pad fp32 elements of workspace. Returns when the work is enqueued on `stream`. */
int edt_outer_step_sharded(void* comm, void* theta_g, int gdt, const void* const* theta_k, int wdt,
                           int K_local, void* momentum_shard, int has_momentum, uint64_t n_pad,
                           uint64_t bucket_elems, double lr, double momentum_coef, int nesterov,
                           float* acc, void* stream);

/* The same step, reduce_ordered schedule (distributed.py mode="reduce_ordered"): per bucket the
 * local fp32 partial into acc[b, e) (laid out [dest rank][shard]), an all-to-all into recv[b, e)
 * ([src rank][shard]), then edt_sgd_apply_sum on the owned shard with the nranks partials in rank
 * order, then the all-gather. The cross-rank sum has one fixed order whatever RCCL's algorithm
 * or topology: the result is reproducible run to run. Same wire bytes as the reduce schedule.
 * recv: n_pad fp32 elements of workspace, distinct from acc. nranks <= EDT_MAX_WORKERS.
 * Replaces the same block as edt_outer_step_sharded (EDT_LM/diloco.py:238-289). */
int edt_outer_step_sharded_ordered(void* comm, void* theta_g, int gdt, const void* const* theta_k, int wdt,
                                   int K_local, void* momentum_shard, int has_momentum, uint64_t n_pad,
                                   uint64_t bucket_elems, double lr, double momentum_coef, int nesterov,
                                   float* acc, float* recv, void* stream);

/* The same step, exact schedule (distributed.py mode="exact", broadcast="theta"): per bucket one
 * all-to-all per local worker straight from the worker arenas into recv[j] (a worker's bucket is
 * already laid out [dest rank][shard]; it arrives as [src rank][shard]), then edt_outer_step on
 * the owned shard with the K_local x nranks workers in the reference's order (global worker
 * k = src rank x K_local + j) — bit-exact with edt_outer_step over the whole population — then
 * the shard's all-gather into theta_g. Wire bytes per rank (nranks-1)/nranks x n_pad x
 * (K_local x wdt + gdt bytes): fewer than the reduce schedules when K_local x wdt bytes < 4.
 * recv: K_local device buffers of n_pad elements of wdt. K_local x nranks <= EDT_MAX_WORKERS. */
int edt_outer_step_sharded_exact(void* comm, void* theta_g, int gdt, const void* const* theta_k, int wdt,
                                 int K_local, void* momentum_shard, int has_momentum, uint64_t n_pad,
                                 uint64_t bucket_elems, double lr, double momentum_coef, int nesterov,
                                 void* const* recv, void* stream);

const char* edt_comm_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* EDT_COMM_H */
