/*
 * edt_sync.h — C ABI of the MI355X (gfx950) outer-loop sync library `libedt_sync.so`.
 *
 * The reference (BarryFutureman/EvolutionaryDistributedTraining) has no FFI: its hot path is
 * Python/PyTorch-CPU code. Each entry point below replaces one piece of that code; the
 * reference location it replaces is cited on the declaration (paths relative to the reference
 * root). The Python shim `evolutionarydistributedtraining_amd` binds these with ctypes and keeps
 * the reference's call surfaces.
 *
 * Conventions
 *  - Every pointer argument named *device* is HBM memory owned by the caller (PyTorch tensors,
 *    `data_ptr()`); the library never allocates device memory and never synchronises.
 *  - `stream` is a hipStream_t (NULL = the legacy default stream). All work is stream-ordered
 *    and asynchronous; every call is hipGraph-capturable.
 *  - Element counts are uint64_t; buffers are flat, parameters laid out back to back in
 *    `model.parameters()` order (the index order the reference's optimizer state uses).
 *  - Scalars arrive as doubles and are rounded exactly as the reference's torch/numpy code
 *    rounds them (fp32 scalar for `mul_`, tensor-dtype `alpha` for `add(..., alpha=)`).
 *  - Return 0 on success or a negative EDT_ERR_* code; edt_last_error() then holds a
 *    thread-local message.
 */
#ifndef EDT_SYNC_H
#define EDT_SYNC_H

#include <stdint.h>

/* ABI revision. 6 (round 6): edt_slerp_gram / edt_slerp_gram_coef removed (the population's
 * triangle layout is a mode of the needed-sums pass; the sharded population uses
 * edt_slerp_needed_*), edt_slerp_seg_table requires the segment sizes. 5 (round 5): the
 * tensor-list outer step's workspace grew (per-tensor tail-mask
 * offsets; edt_outer_list_workspace_bytes), edt_outer_step_list_tail and
 * edt_slerp_population_layout added, edt_slerp_seg_table refuses in-place outputs that overlap
 * another tensor. 4 (round 4): the tensor-list SLERP reads a device pointer table
 * (edt_slerp_seg_table + the *_table entries), edt_slerp_merge_list_speculative takes the segment
 * sizes (full byte-range overlap check), edt_slerp_blend_segments / _blend_table / _refdot_table
 * added, the on-chip-hold form removed. Workspace sizes come from the *_doubles / *_bytes functions
 * of THIS build: a consumer compiled against another revision must be rebuilt
 * (edt_abi_version() != EDT_ABI_VERSION: refuse to run). */
#define EDT_ABI_VERSION 6

#ifdef __cplusplus
extern "C" {
#endif

/* EDT_ABI_VERSION of the loaded library. */
int edt_abi_version(void);

typedef enum { EDT_F32 = 0, EDT_BF16 = 1 } edt_dtype_t;

enum {
    EDT_OK = 0,
    EDT_ERR_ARG = -1,      /* bad argument (null pointer, unsupported dtype pair, K out of range) */
    EDT_ERR_LAUNCH = -2,   /* kernel launch failed (hipGetLastError) */
};

#define EDT_MAX_WORKERS 64   /* workers consumed by one fused launch */

/* ---- DiLoCo outer step ------------------------------------------------------------------
 * Replaces EDT_LM/diloco.py:238-289 (== EDT_LM/diloco_sim.py:233-299):
 *   acc = 0; for k: acc += (theta_k - theta_g) / K      (worker-major, true division by K)
 *   grad = -acc; torch.optim.SGD(lr, momentum, nesterov).step()  (single-tensor CPU path)
 * fused in one pass over HBM. theta_g and momentum are updated in place.
 * dtype pairs (gdt, wdt): (F32,F32), (F32,BF16) [torch promotion: math in fp32], (BF16,BF16)
 * [every op rounded to bf16 as torch's CPU kernels do]. momentum has dtype gdt and is only
 * touched when momentum_coef != 0; has_momentum = 0 reproduces the first step
 * (`buf = grad.clone()`), 1 the carried buffer (`load_state_dict` carry, diloco.py:258-286).
 * theta_k: host array of K device pointers, 1 <= K <= EDT_MAX_WORKERS. */
int edt_outer_step(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K,
                   void* momentum, int has_momentum, uint64_t n,
                   double lr, double momentum_coef, int nesterov, void* stream);

/* edt_outer_step fused with the broadcast of EDT_LM/diloco.py:302-308 (the new global model saved
 * to every worker dir, from which the next inner loops start): the same step, and in the same pass
 * theta_new rounded to the worker dtype (RNE, torch copy_) is stored into the nbcast device
 * buffers bcast[0..nbcast) (n elements of wdt each; a buffer may be one of the theta_k, which are
 * read before they are overwritten, element by element; none may overlap theta_g).
 * Replaces edt_outer_step + nbcast device copies (each re-reading theta). 0 <= nbcast <= 64;
 * nbcast = 0 is edt_outer_step. */
int edt_outer_step_bcast(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K,
                         void* momentum, int has_momentum, uint64_t n, double lr, double momentum_coef,
                         int nesterov, void* const* bcast, int nbcast, void* stream);

/* Bit-exact with the reference on a given host: torch's CPU kernels run add(x, y, alpha) as one
 * FMA on their vectorised path but as round(x + round(alpha * y)) on the scalar tail of every
 * contiguous run (the last numel % Vec::size() elements of each at::parallel_for chunk; Vec::size()
 * = 32 bf16 on AVX-512, 16 on AVX2), which differ in bf16 (EDT_LM/diloco.py:252-289's SGD:
 * grad.add(buf, alpha=mu), param.add_(grad, alpha=-lr)). edt_outer_step / edt_pair_merge_to compute
 * the vectorised form on every element; these variants take the tail elements of the reference's
 * host as a bitmask (device, 1 bit per element of the flat arena, bit i & 7 of byte i >> 3; built
 * from the layout, the host's vector width and its thread count) and round those twice. Ignored
 * for fp32 (torch's fp32 tails are FMAs too). tail_bits NULL = the plain functions. */
int edt_outer_step_tail(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K,
                        void* momentum, int has_momentum, uint64_t n, double lr, double momentum_coef,
                        int nesterov, const uint8_t* tail_bits, void* stream);
int edt_pair_merge_tail(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                        void* theta_out, int gdt, const void* momentum_in, void* momentum_out,
                        int has_momentum, uint64_t n, double lr, double momentum_coef, int nesterov,
                        const uint8_t* tail_bits, void* stream);

/* The same step for any population size: K > EDT_MAX_WORKERS runs as consecutive launches of
 * <= 64 workers (the reference's worker order), the running sum carried in `workspace` (n
 * elements of theta's dtype: lossless, the sum is rounded to that dtype after every add).
 * K <= 64: identical to edt_outer_step (workspace unused, may be NULL). */
int edt_outer_step_ws(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K,
                      void* momentum, int has_momentum, uint64_t n, double lr, double momentum_coef,
                      int nesterov, void* workspace, void* stream);

/* Tensor-list form of edt_outer_step, for parameters that are T separate device allocations
 * (`list(model.parameters())` of models loaded straight to the GPU, the reference's own objects at
 * EDT_LM/diloco.py:231-246): one launch over all tensors, no packing into a flat buffer.
 *   theta_t[T], momentum_t[T]   host arrays of device pointers (momentum_t unused, may be NULL,
 *                               when momentum == 0)
 *   theta_k[K * T]              worker-major: theta_k[k * T + t] is tensor t of worker k
 *   numel[T]                    element count of each tensor (0 allowed)
 * The per-tensor math is exactly edt_outer_step's. The tensor table (pointers, sizes, chunk
 * offsets) is copied into `workspace` (device memory, 8-byte aligned, at least
 * edt_outer_list_workspace_bytes(T, K)) by a stream-ordered copy, so the workspace must not be
 * reused before the launch has run. 1 <= K <= EDT_MAX_WORKERS. */
uint64_t edt_outer_list_workspace_bytes(int T, int K);
int edt_outer_step_list(void* const* theta_t, int gdt, const void* const* theta_k, int wdt, int K,
                        void* const* momentum_t, int has_momentum, const uint64_t* numel, int T,
                        double lr, double momentum, int nesterov, void* workspace,
                        uint64_t workspace_bytes, void* stream);
/* edt_outer_step_list with the reference host's bf16 scalar tails (edt_outer_step_tail's rule, r5;
 * replaces EDT_LM/diloco.py:238-289 run on a master whose torch CPU kernels round bf16 tails
 * separately, over `model.parameters()` lists):
 * tail_bits (device, nullable) holds each tensor's 1-bit-per-element mask from byte
 * tail_byte_offset[t] (host array, T entries), indexed by the element's index inside its tensor.
 * gdt must be EDT_BF16 when tail_bits is given. */
int edt_outer_step_list_tail(void* const* theta_t, int gdt, const void* const* theta_k, int wdt, int K,
                             void* const* momentum_t, int has_momentum, const uint64_t* numel, int T,
                             double lr, double momentum, int nesterov, const uint8_t* tail_bits,
                             const uint64_t* tail_byte_offset, void* workspace, uint64_t workspace_bytes,
                             void* stream);

/* Partial delta sum for the sharded multi-GPU step (EDT_LM/diloco.py:243-246 restricted to the
 * workers resident on this rank): acc_f32[i] (+)= sum_{k<K_local} round_g((theta_k - theta_g)/K_total).
 * accumulate = 0 starts from zero, 1 continues the running fp32 sum already in acc_f32 (so two
 * launches over workers [0,a) and [a,K) add in the same order as one launch over [0,K)).
 * The cross-rank sum then goes over RCCL. */
int edt_delta_partial(const void* theta_g, int gdt, const void* const* theta_k, int wdt,
                      int K_local, int K_total, uint64_t n, float* acc_f32, int accumulate,
                      void* stream);

/* SGD on a shard from a reduced fp32 pseudo-gradient sum: grad = -round_g(acc_f32), then the
 * torch.optim.SGD single-tensor update of EDT_LM/diloco.py:252-289. */
int edt_sgd_apply(void* theta_g, int gdt, const float* acc_f32, void* momentum, int has_momentum,
                  uint64_t n, double lr, double momentum_coef, int nesterov, void* stream);

/* SGD on a shard from nacc per-rank fp32 partial sums of it (acc_f32[0..nacc), device pointers,
 * n elements each), summed in that order: grad = -round_g(((acc_0 + acc_1) + ...) + acc_{nacc-1}).
 * The sharded step's reduce_ordered schedule (all-to-all of the partials, then this): the
 * cross-rank sum has one fixed order, independent of the collective library's algorithm. */
int edt_sgd_apply_sum(void* theta_g, int gdt, const float* const* acc_f32, int nacc, void* momentum,
                      int has_momentum, uint64_t n, double lr, double momentum_coef, int nesterov, void* stream);

/* ---- EDT pairwise merge -------------------------------------------------------------------
 * Replaces EDT_LM/train/crossover.py:150-163 + 166-230 for one child:
 *   B = lerp(0.5, b1, b2)                         (run_linear_merge_5050, in the model dtype wdt)
 *   d = ((m1 - B) + (m2 - B)) / 2 ; grad = -d      (run_sgd, in the base dtype gdt)
 *   SGD(lr, momentum, nesterov).step() with the parent's momentum when has_momentum = 1.
 * Writes the child parameters to theta_out (gdt) and the new momentum buffer in place.
 * The parents' bases b1/b2 and trained weights m1/m2 have dtype wdt. b2 may be NULL: b1 is
 * then the already merged base of dtype gdt (run_sgd called on a given base_model). */
int edt_pair_merge(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                   void* theta_out, int gdt, void* momentum, int has_momentum, uint64_t n,
                   double lr, double momentum_coef, int nesterov, void* stream);

/* edt_pair_merge with the inherited momentum read from `momentum_in` (the donor parent's
 * outer_optim.pt buffer, EDT_LM/train/crossover.py:183-219) and the child's written to
 * `momentum_out`: the donor stays intact for the other children it feeds, and no copy of it is
 * made first. momentum_in == momentum_out is edt_pair_merge. */
int edt_pair_merge_to(const void* b1, const void* b2, const void* m1, const void* m2, int wdt,
                      void* theta_out, int gdt, const void* momentum_in, void* momentum_out,
                      int has_momentum, uint64_t n, double lr, double momentum_coef, int nesterov,
                      void* stream);

/* Every EDT-LM child of a resident population in ONE launch (EDT_LM/edt_sim.py:244-256: one child
 * per machine from the selected pairs): child c is edt_pair_merge_to(b1[c], b2[c], m1[c], m2[c],
 * out[c], momentum_in[c] -> momentum_out[c], has_momentum[c]) — host arrays of nchildren (<= 16)
 * device pointers; parents repeat across children (a parent feeds ~2). The workgroups of all
 * children for one chunk of elements share an XCD (blockIdx % 8) and run together, so each parent
 * chunk is fetched from HBM once and served from L2 / the Infinity Cache to its other readers.
 * Results are bit-identical to the per-child calls. Outputs must not alias any input. */
int edt_pair_merge_population(const void* const* b1, const void* const* b2, const void* const* m1,
                              const void* const* m2, int wdt, void* const* out, int gdt,
                              const void* const* momentum_in, void* const* momentum_out,
                              const int32_t* has_momentum, int nchildren, uint64_t n, double lr,
                              double momentum_coef, int nesterov, void* stream);

/* lerp(t, v0, v1) = (1-t)*v0 + t*v1 as three rounded ops in compute dtype cdt (= the tensors'
 * dtype for torch, F32 for numpy), stored as out_dt.
 * Replaces EDT_LM/train/crossover.py:50-51 / EDT_RL/crossover.py:46-47 when applied per tensor. */
int edt_lerp(const void* v0, const void* v1, int in_dt, void* out, int out_dt, int cdt,
             uint64_t n, double t, void* stream);

/* ---- SLERP crossover (EDT_RL/crossover.py:11-43, EDT_EVOMERGE/train/crossover.py:14-46) ------
 * Multi-tensor: the parents v0, v1 are flat buffers holding `nseg` tensors; segment s spans
 * [seg_offsets[s], seg_offsets[s+1]). Work is cut into chunks that never cross a segment.
 *
 * edt_slerp_make_chunks (HOST function): fills chunk_desc (3 uint64 per chunk:
 *   start, length, segment) and seg_first_chunk (nseg+1) for chunk length `chunk_elems`
 *   (<= 65536: a chunk's sums are a fixed tree over at most 128 tiles of 512 elements);
 *   returns the chunk count, or the required count (negated - 1) if max_chunks is too small. */
int64_t edt_slerp_make_chunks(const uint64_t* seg_offsets_host, int nseg, uint32_t chunk_elems,
                              uint64_t* chunk_desc_host, int64_t max_chunks,
                              int32_t* seg_first_chunk_host);

/* Chunk-sum tables. Every chunk's fp64 sums are formed in one canonical order (edt_slerp.hip:
 * per-lane FMA chains over 512-element tiles, the wave butterfly, a perfect binary tree over the
 * tiles), written as partial-tree rows: a table of W sums per chunk
 * therefore needs edt_slerp_sums_doubles(W, nchunks) doubles — the chunk rows [nchunks][W] first
 * (what the coefficient passes read and what a caller may copy or all-gather), then the row
 * scratch the sum pass fills and folds into the rows (W = 3: and one flag word at the end). Every
 * `partial` of the pair forms below holds edt_slerp_sums_doubles(3, nchunks) doubles. */
uint64_t edt_slerp_sums_doubles(int width, int64_t nchunks);

/* Pass 1: per-chunk sums  partial[c] = { sum v0^2, sum v1^2, sum v0*v1 }  (fp64). */
int edt_slerp_stats(const void* v0, const void* v1, int in_dt, const uint64_t* chunk_desc,
                    int64_t nchunks, double* partial, void* stream);

/* Per segment: reduce the chunk sums in a fixed order, form the norms, the normalised dot and
 * the blend coefficients coef[2s], coef[2s+1] exactly as the reference's branch does:
 *   |dot| > dot_threshold -> (1-t, t) (lerp);  else (sin((1-t)th)/sin th, sin(t th)/sin th).
 * t: device array of nseg doubles (interpolate_t / global t per key). dot_out (nullable): the
 * fp32 dot per segment. */
int edt_slerp_coef(const double* partial, const int32_t* seg_first_chunk, int nseg,
                   const double* t, double dot_threshold, double eps, float* coef,
                   float* dot_out, void* stream);

/* Pass 2: out = coef0*v0 + coef1*v1 in fp32 (numpy: two rounded products, one rounded sum),
 * stored as out_dt (RN to bf16 when the merged model is bf16, EDT_EVOMERGE/train/crossover.py:142). */
int edt_slerp_blend(const void* v0, const void* v1, int in_dt, void* out, int out_dt,
                    const uint64_t* chunk_desc, int64_t nchunks, const float* coef, void* stream);

/* The three passes above in one call (stats -> coef -> blend), stream-ordered. A
 * segment-grouped variant that re-reads each group from the Infinity Cache measured slower on
 * MI355X (launch count; 87 % of a 7B body's bytes sit in tensors larger than the cache), so the
 * whole-arena form is the one shipped. */
int edt_slerp_merge(const void* v0, const void* v1, int in_dt, void* out, int out_dt,
                    const uint64_t* chunk_desc, int64_t nchunks, const int32_t* seg_first_chunk, int nseg,
                    const double* t, double dot_threshold, double eps, double* partial, float* coef,
                    float* dot_out, void* stream);

/* edt_slerp_merge with a speculative first pass: the chunk sums and, in the same pass, the
 * lerp-branch output (1-t) v0 + t v1 of every segment; the coefficients then flag (redo[s] = 1,
 * nseg int32 of device workspace) the segments whose |dot| <= dot_threshold, and only their
 * chunks are blended again with the SLERP coefficients. Parents of one lineage (fine-tunes of a
 * common base: |dot| > 0.9995 on most tensors, EDT_RL/crossover.py:31-32) are merged in ONE pass
 * over them (2 b_in + b_out per element instead of 4 b_in + b_out); segments that take the SLERP
 * branch cost a second full pass. Outputs, sums and dots are bit-identical to edt_slerp_merge.
 * `out` must not overlap the parents (n elements each). */
int edt_slerp_merge_speculative(const void* v0, const void* v1, int in_dt, void* out, int out_dt,
                                const uint64_t* chunk_desc, int64_t nchunks, const int32_t* seg_first_chunk,
                                int nseg, const double* t, double dot_threshold, double eps, double* partial,
                                float* coef, float* dot_out, int32_t* redo, uint64_t n, void* stream);

/* Tensor-list form of edt_slerp_merge: segment i is its own tensor pair v0_t[i], v1_t[i] and is
 * written to out_t[i] (host arrays of nseg device pointers, each 16-byte aligned; NULL only for
 * empty segments), e.g. two models' state-dict tensors merged straight into a third model's
 * parameters (EDT_EVOMERGE/train/crossover.py:104-146 without the state-dict copies). chunk_desc
 * holds starts RELATIVE to their segment (edt_slerp_make_chunks output minus
 * seg_offsets[segment]). The kernels read the tensors through a DEVICE table of 3 x nseg uint64
 * {v0, v1, out} pointers:
 *   edt_slerp_seg_table   (HOST) validates the arrays (alignment; with `apart`, no output byte
 *                         range [out, out + n*osize) overlaps any parent range — a sorted-span
 *                         check over every tensor, seg_numel = the nseg sizes; r5: without
 *                         `apart` but with seg_numel, an output may be exactly one of its OWN
 *                         parents and must overlap no other tensor's parent or output — the
 *                         two-pass blend would race; r6: seg_numel is required whenever
 *                         nseg > 0 — the checks need the sizes) and writes the
 *                         table's host image (3 x nseg uint64). The caller uploads it once and
 *                         reuses it while the tensors stay where they are: the *_table entries
 *                         below then cost no per-tensor host work per call.
 *   edt_slerp_merge_table / _speculative   edt_slerp_merge / _speculative over the table (the
 *                         speculative one needs a table validated with apart = 1)
 *   edt_slerp_stats_table / edt_slerp_blend_table   the passes alone; blend: redo (nseg int32,
 *                         nullable) restricts it to segments with redo[s] != 0
 *   edt_slerp_merge_list / _list_speculative   the same from host pointer arrays: the table is
 *                         validated and copied into `workspace` (24 bytes per segment, device,
 *                         8-byte aligned) by a stream-ordered copy on every call. edt_slerp_merge_list
 *                         takes no sizes, so its in-place rule (an output exactly its own parent
 *                         or apart from every other tensor) is the caller's to keep; the
 *                         speculative form checks its rule over seg_numel. */
int edt_slerp_seg_table(const void* const* v0_t, const void* const* v1_t, void* const* out_t, int nseg,
                        const uint64_t* seg_numel, int in_dt, int out_dt, int apart, uint64_t* table_host);
int edt_slerp_stats_table(const uint64_t* seg_table, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                          double* partial, void* stream);
int edt_slerp_blend_table(const uint64_t* seg_table, int in_dt, int out_dt, const uint64_t* chunk_desc,
                          int64_t nchunks, const float* coef, const int32_t* redo, void* stream);
int edt_slerp_merge_table(const uint64_t* seg_table, int in_dt, int out_dt, const uint64_t* chunk_desc,
                          int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t,
                          double dot_threshold, double eps, double* partial, float* coef, float* dot_out,
                          void* stream);
int edt_slerp_merge_table_speculative(const uint64_t* seg_table, int in_dt, int out_dt, const uint64_t* chunk_desc,
                                      int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t,
                                      double dot_threshold, double eps, double* partial, float* coef,
                                      float* dot_out, int32_t* redo, void* stream);
int edt_slerp_merge_list(const void* const* v0_t, const void* const* v1_t, int in_dt,
                         void* const* out_t, int out_dt, const uint64_t* chunk_desc, int64_t nchunks,
                         const int32_t* seg_first_chunk, int nseg, const double* t,
                         double dot_threshold, double eps, double* partial, float* coef,
                         float* dot_out, void* workspace, uint64_t workspace_bytes, void* stream);

/* edt_slerp_merge_list with edt_slerp_merge_speculative's first pass: the chunk sums and the
 * lerp-branch output of every tensor in one pass over the tensors where they lie; only tensors
 * whose |dot| <= dot_threshold (redo[s] = 1, nseg int32 of device workspace) are blended again.
 * Parents of one lineage cost one pass instead of two. Outputs, sums and dots are bit-identical
 * to edt_slerp_merge_list. No output may overlap any parent tensor (checked over the byte ranges
 * from seg_numel, the nseg sizes on the host: EDT_ERR_ARG, and the two-pass list form takes
 * that case); `partial` as edt_slerp_merge_speculative's (its last double holds the any-redo
 * word). */
int edt_slerp_merge_list_speculative(const void* const* v0_t, const void* const* v1_t, int in_dt,
                                     void* const* out_t, int out_dt, const uint64_t* seg_numel,
                                     const uint64_t* chunk_desc, int64_t nchunks,
                                     const int32_t* seg_first_chunk, int nseg, const double* t,
                                     double dot_threshold, double eps, double* partial, float* coef,
                                     float* dot_out, int32_t* redo, void* workspace, uint64_t workspace_bytes,
                                     void* stream);

/* out = coef0*v0 + coef1*v1 (edt_slerp_blend's math) over the chunks whose segment has
 * redo[s] != 0 only (nseg int32, device): the flat-arena re-blend of selected segments. */
int edt_slerp_blend_segments(const void* v0, const void* v1, int in_dt, void* out, int out_dt,
                             const uint64_t* chunk_desc, int64_t nchunks, const float* coef, const int32_t* redo,
                             void* stream);

/* SLERP children of a resident population (EDT_RL/edt.py:286-299: every selected pair of one
 * generation, EDT_RL/crossover.py:84-135 per child): ONE stats pass over the nmembers (<= 8) flat
 * member arenas forms every parent's squared norm and the dots the children need per chunk, then
 * per child the coefficients (from pairs[2q], pairs[2q+1] = member indices, host array) and the
 * blend into outs[q] (host array of device pointers; no output may alias a member). The stats pass
 * runs per connected component of the children's pair graph (r5, any graph the reference's
 * roulette selection draws): a component of D <= 8 parents forms its D norms and only the dots its
 * children use — the edges of the best cyclic order of the parents (the ring) plus up to 4 chord
 * slots (2 at D = 4, none below) — or, when the children need more dots than that, the same pass
 * in the triangle layout (its Gram upper triangle: the norms and the dots used); each parent is
 * read once either way. `gram`: edt_slerp_population_gram_doubles(nmembers, nchunks) doubles of
 * device workspace (layout internal to this call). Each child's sums,
 * coefficients and output are bit-identical to edt_slerp_merge on (members[i], members[j]).
 * coef: [npairs][nseg][2] floats; dot_out (nullable): [npairs][nseg]. */
uint64_t edt_slerp_population_gram_doubles(int nmembers, int64_t nchunks);
int edt_slerp_population(const void* const* members, int nmembers, int in_dt, const int32_t* pairs, int npairs,
                         void* const* outs, int out_dt, const uint64_t* chunk_desc, int64_t nchunks,
                         const int32_t* seg_first_chunk, int nseg, const double* t, double dot_threshold,
                         double eps, double* gram, float* coef, float* dot_out, void* stream);

/* edt_slerp_population with edt_slerp_merge_speculative's first pass, which also writes every
 * child's lerp-branch output: when every component takes the needed-sums layout and npairs <= 16,
 * one member-major launch per component (each parent read once, every child emitted from the
 * parents' registers: ring-edge children directly, the others from a chord slot or a copy);
 * otherwise — the fallback for graphs the reference's 8-pair selection does not draw: more than 16
 * children, more than 8 distinct parents, a component on the triangle layout, or more distinct
 * chord children than the emit slots — one co-located launch (every child of a chunk on one XCD,
 * shared parents read once).
 * Per child the coefficients flag (redo: [npairs][nseg] int32) the SLERP-branch segments, which
 * one launch blends again (it exits at once when no child needs any).
 * partial: edt_slerp_population_speculative_doubles(npairs, nchunks) doubles of workspace.
 * Outputs must not overlap any member (n elements each). Bit-identical to edt_slerp_merge per
 * child either way. */
uint64_t edt_slerp_population_speculative_doubles(int npairs, int64_t nchunks);
int edt_slerp_population_speculative(const void* const* members, int nmembers, int in_dt, const int32_t* pairs,
                                     int npairs, void* const* outs, int out_dt, const uint64_t* chunk_desc,
                                     int64_t nchunks, const int32_t* seg_first_chunk, int nseg, const double* t,
                                     double dot_threshold, double eps, double* partial, float* coef,
                                     float* dot_out, int32_t* redo, uint64_t n, void* stream);

/* The needed-sums passes of edt_slerp_population as separate entries (r5: the link-balanced sharded
 * population — each rank forms the sums of its chunk range, the table rows are all-gathered, every
 * rank forms every child's coefficients; distributed.ShardedPopulationCrossover). Replaces, across
 * the node's GPUs, the RL master's generation EDT_RL/edt.py:286-299 -> EDT_RL/crossover.py:84-135
 * per child (the dots of EDT_RL/crossover.py:20-29). The table of a
 * generation (pairs over nmembers <= 8 members, nchunks chunks) is ncomp blocks, one per connected
 * component of the children's pair graph: block k at block_off[k] doubles, nchunks rows of
 * block_nt[k] sums (the component's norms and the dots its children use, or its Gram triangle
 * when they need more dots than the slots: D(D+1)/2 columns, the dots no child uses not formed).
 * col_members (nullable, 2 x sum(block_nt) int32): the two members of each column, block after
 * block (-1, -1: an unused slot, its sum not formed). scratch_doubles: the
 * row scratch a pass over up to nchunks chunks needs.
 *   edt_slerp_needed_sums  rows [row0, row0 + nchunks) of every block, over a chunk table of those
 *                          nchunks chunks (starts relative to the member buffers), table_chunks =
 *                          the table's row count; a row is bit-identical to edt_slerp_population's
 *                          sums of that chunk, wherever the chunk's elements lie (16-byte aligned)
 *   edt_slerp_needed_coef  every child's coefficients [npairs][nseg][2] and dots [npairs][nseg]
 *                          (nullable) from the complete table
 *   edt_slerp_blend_children (below) then blends a rank's chunks of every child. */
int edt_slerp_needed_table(const int32_t* pairs, int npairs, int nmembers, int64_t nchunks, uint64_t* block_off,
                           int32_t* block_nt, int32_t* ncomp, int32_t* col_members, uint64_t* table_doubles,
                           uint64_t* scratch_doubles);
int edt_slerp_needed_sums(const void* const* members, int nmembers, int in_dt, const int32_t* pairs, int npairs,
                          const uint64_t* chunk_desc, int64_t nchunks, int64_t table_chunks, int64_t row0,
                          double* table, double* scratch, uint64_t scratch_doubles, void* stream);
int edt_slerp_needed_coef(const double* table, int64_t table_chunks, const int32_t* pairs, int npairs, int nmembers,
                          const int32_t* seg_first_chunk, int nseg, const double* t, double dot_threshold, double eps,
                          float* coef, float* dot_out, void* stream);

/* The plan the two population entries above make for a pair graph (the pairs of
 * EDT_RL/edt.py:268-269's selection), as JSON text into buf (host only, no device work): distinct parents, the form (speculative: "member-major" or "co-located";
 * "two-pass"), and per connected component of the children's pair graph its members, distinct
 * dots, sums per element and stats layout ("needed": the members' norms + the dots the children
 * use; "triangle": every pair). For benches and logs. */
int edt_slerp_population_layout(const int32_t* pairs, int npairs, int nmembers, int speculate, char* buf,
                                int buflen);

/* ---- reference-dot mode (opt-in; EDT_RL/crossover.py:20-31 on the reference host) -------------
 * The default coefficients come from an fp64 dot of the chunk sums (within ~3e-7 of the true
 * cosine). The reference decides its branch from an fp32 dot whose error grows with the tensor
 * (BLAS sdot norms, then numpy's pairwise sum of the normalised products), so near
 * DOT_THRESHOLD the two can take different branches. This mode recomputes, for the flagged
 * segments, the reference's own fp32 dot bit for bit (restated and pinned in oracle/edt_oracle.c:
 * numpy 2.2 with OpenBLAS 0.3.29's SkylakeX sdot; `threads` = OpenBLAS's thread count for sdot
 * on the reference host, 1 on the pinned host) and the coefficients from it:
 *   edt_slerp_refdot_flags  flag[s] = 1 where | |dots[s]| - dot_threshold | <= band (band < 0: all)
 *   edt_slerp_refdot        ref_dot[s] for every flagged segment (flag NULL: all); chunks of the
 *                           plan (chunk_elems, a multiple of 8192); workspace (device, 8-byte
 *                           aligned): edt_slerp_refdot_workspace_bytes(...)
 *   edt_slerp_refdot_coef   coef / dot_out of the flagged segments from ref_dot (the branch and the
 *                           fp32 SLERP coefficients of edt_slerp_coef)
 * Order: edt_slerp_stats -> edt_slerp_coef -> flags -> refdot -> refdot_coef -> edt_slerp_blend.
 * The norms are sequential FMA chains by definition (one workgroup per segment and BLAS thread):
 * a parity mode, tens of ms for a 545M-element tensor. */
uint64_t edt_slerp_refdot_workspace_bytes(int nseg, int64_t nchunks, uint32_t chunk_elems, int threads);
int edt_slerp_refdot_flags(const float* dots, int nseg, double dot_threshold, double band, int32_t* flag,
                           void* stream);
int edt_slerp_refdot(const void* v0, const void* v1, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                     const int32_t* seg_first_chunk, int nseg, uint32_t chunk_elems, const int32_t* flag, int threads,
                     double eps, float* ref_dot, void* workspace, uint64_t workspace_bytes, void* stream);
/* edt_slerp_refdot over a tensor-list device table (edt_slerp_seg_table; chunk starts relative). */
int edt_slerp_refdot_table(const uint64_t* seg_table, int in_dt, const uint64_t* chunk_desc, int64_t nchunks,
                           const int32_t* seg_first_chunk, int nseg, uint32_t chunk_elems, const int32_t* flag,
                           int threads, double eps, float* ref_dot, void* workspace, uint64_t workspace_bytes,
                           void* stream);
int edt_slerp_refdot_coef(const float* ref_dot, const int32_t* flag, int nseg, const double* t, double dot_threshold,
                          float* coef, float* dot_out, void* stream);

/* ---- the population SLERP's blends, separately (link-balanced sharded population) -----------
 * edt_slerp_population = edt_slerp_needed_sums (every block, all chunks) + edt_slerp_needed_coef +
 * edt_slerp_blend_children. Split so that the sums of a rank's range of whole chunks (its
 * parameter-index shard of all members, EDT_RL/edt.py:286-299's population spread over the node)
 * can be all-gathered before the coefficients: each chunk's sums are formed by the same kernel in
 * the same order wherever the chunk lives, so the coefficients — and every child — equal
 * edt_slerp_merge's bit for bit.
 *   edt_slerp_blend_children  outs[q] = c0 v_a + c1 v_b over the chunks of chunk_desc (starts
 *                         relative to the member buffers), the segment of each chunk selecting
 *                         coef[q][seg] (nseg = the row length of coef); <= 8 members, <= 16
 *                         children, member-major (each member's tile read once per chunk). */
int edt_slerp_blend_children(const void* const* members, int nmembers, int in_dt, const int32_t* pairs,
                             int npairs, void* const* outs, int out_dt, const uint64_t* chunk_desc,
                             int64_t nchunks, const float* coef, int nseg, void* stream);

/* ---- misc ---- */
const char* edt_last_error(void);
const char* edt_version(void);
/* Diagnostic (not a reference surface): edt_outer_step's exact access pattern on the same
 * operands (theta and momentum read and written, K workers read with the same loads, cache policy
 * and grid) with a trivial body that perturbs theta and momentum by ~1e-30 relative. Its time is
 * the memory-system ceiling of the fused step on the device at hand (bench.py reports both).
 * Operands must be 16-byte aligned. */
int edt_probe_stream(void* theta_g, int gdt, const void* const* theta_k, int wdt, int K, void* momentum,
                     uint64_t n, void* stream);

/* bytes of device memory the kernels above may touch per element, for roofline accounting */
int edt_outer_step_bytes_per_elem(int gdt, int wdt, int K, int with_momentum);

#ifdef __cplusplus
}
#endif
#endif /* EDT_SYNC_H */
