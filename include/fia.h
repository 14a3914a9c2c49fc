/*
 * fia.h — C ABI of the MI355X-native FIA (fast influence analysis) library.
 *
 * One shared library (libfia.so, gfx950) replaces the TensorFlow/scipy steps
 * of the reference's per-test-rating influence path:
 *
 *   reference (zz9tf/FIA-KDD-19, src/influence/)        replaced by
 *   -------------------------------------------------   ------------------------
 *   MF.__init__ / NCF.__init__ variables                 fia_set_params
 *     (matrix_factorization.py:89-116, NCF.py:102-145)
 *   DataSet train.x scanned per query                    fia_build_index (once)
 *     (dataset.py:14, matrix_factorization.py:320-321)
 *   get_train_indices_of_test_case                       fia_count_related + fia_related
 *     (matrix_factorization.py:315-322, NCF.py:344-351)
 *   hessian_vector_product_test + minibatch_hessian_     fia_prepare (entity Gram caches)
 *     vector_val (mf:288-308, 324-351; ncf:317-380)       + fia_query_batch (assembly)
 *   get_inverse_hvp -> get_inverse_hvp_cg / fmin_ncg     fia_query_batch (exact fp64 LDL^T)
 *     (genericNeuralNet.py:503-508, mf:419-433, ncf:448-462)
 *   scoring loop of get_influence_on_test_loss           fia_query_batch (influence)
 *     (mf:237-246, ncf:266-274)
 *   top-K of experiments.test_retraining                 fia_query_batch (top-K)
 *     (experiments.py:46-48)
 *
 * Conventions
 *   - All array arguments are DEVICE pointers owned by the caller (PyTorch).
 *     The context owns only its index, caches and scratch.
 *   - Every call is ordered on `stream` (a hipStream_t passed as void*; NULL =
 *     the null stream).  Use one stream per context.  A context is not
 *     thread-safe; use one context per GPU / process.  A call on a new stream first
 *     synchronises the previous one -- except when the new stream is being captured
 *     into a HIP graph (no synchronisation is legal there): finish the previous
 *     stream's work (e.g. an eager warm-up) before the capture begins.  An eager
 *     fia_prepare / fia_prepare_for may run its Gram pass on the context's own aux
 *     stream, joined by the next fia_query_batch / fia_prepare; a capture may only
 *     start once that join has happened (the aux stream is idle to the capture):
 *     otherwise the first call on the capturing stream returns FIA_ERR_STATE.
 *   - Every entry point returns FIA_OK (0) or an error code; no exception
 *     crosses the ABI.  fia_last_error() describes the last failure.
 *   - Ids are int32 in [0, num_users) / [0, num_items); ratings are float32.
 *   - Parameters are float32 device tables in the reference's flat layout.
 *     The math (Hessian assembly, solve, scoring) runs in fp64.
 */
#ifndef FIA_H_
#define FIA_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FIA_OK 0
#define FIA_ERR_INVALID 1      /* bad argument (null pointer, size, id range)   */
#define FIA_ERR_HIP 2          /* HIP runtime error                             */
#define FIA_ERR_STATE 3        /* call order: params/index/prepare missing      */
#define FIA_ERR_UNSUPPORTED 4  /* model / embedding size not built into library */
#define FIA_ERR_NOMEM 5

#define FIA_MODEL_MF 0
#define FIA_MODEL_NCF 1

#define FIA_MAX_TOPK 64

typedef struct fia_ctx fia_ctx;

/* Library version (major*10000 + minor*100 + patch). */
int fia_version(void);

/* Create a context bound to HIP device `device`. */
int fia_create(int device, fia_ctx** out);
/* Waits for the context's own work (its aux stream and the stream of its last call, not the
 * whole device), frees its buffers in order on that stream and destroys it. */
int fia_destroy(fia_ctx* ctx);
/* Message of the last failing call on ctx ("" if none).  ctx may be NULL. */
const char* fia_last_error(const fia_ctx* ctx);

/* Register the model parameters (device float32 tables, kept by pointer).
 *   MF  (matrix_factorization.py:30-36), nptrs = 5:
 *     [0] embedding_users [U*k]  [1] embedding_items [I*k]
 *     [2] bias_users [U]         [3] bias_items [I]        [4] global_bias [1]
 *   NCF (NCF.py:29-41, 85-145), nptrs = 10:
 *     [0] mlp/embedding_users [U*k]  [1] mlp/embedding_items [I*k]
 *     [2] gmf/embedding_users [U*k]  [3] gmf/embedding_items [I*k]
 *     [4] h1/weights [2k*k] [5] h1/biases [k] [6] h2/weights [k*k/2]
 *     [7] h2/biases [k/2]  [8] h3/weights [3k/2] [9] h3/biases [1]
 * weight_decay: the reference's wd (variable_with_weight_decay,
 * genericNeuralNet.py:40-65); damping: lambda added to every HVP (mf:306). */
int fia_set_params(fia_ctx* ctx, int model, int k, int64_t num_users, int64_t num_items,
                   const float* const* tables, int nptrs, double weight_decay, double damping);

/* Build the user-major (CSR) and item-major (CSC) rating index from the
 * training ratings (row j = (user[j], item[j], rating[j])).  Inside a user's
 * or an item's list rows keep ascending train-row order, so the related set of
 * (u,i) is exactly np.where(x[:,0]==u) ++ np.where(x[:,1]==i) (mf:320-322).
 * Synchronises `stream` (one-time setup). */
int fia_build_index(fia_ctx* ctx, int64_t n_train, int64_t num_users, int64_t num_items,
                    const int32_t* user, const int32_t* item, const float* rating, void* stream);

/* Per-entity Hessian caches for the current params + index: for every user u
 * the Gram sum over R_u of the restricted prediction gradients, likewise for
 * every item (the rank-1 updates of H_t).  Call after set_params/build_index
 * and again whenever the parameter VALUES change.
 * Ordering: the caches are ready for every later call on the context.  For small k
 * (except MF k <= 16) the pass runs on the context's own stream, forked from `stream`, and
 * the next fia_* call on the context joins it (the query-side scans of fia_query_batch
 * overlap it); until then it still READS the parameter tables and the index, so keep the
 * tables alive and unchanged until the next call on the context -- fia_set_params (which
 * waits for the pass on the host), fia_build_index, fia_prepare*, fia_query_batch* or
 * fia_destroy -- rather than only until `stream` is synchronised. */
int fia_prepare(fia_ctx* ctx, void* stream);

/* Like fia_prepare, but the per-entity caches are built only for the users and items
 * referenced by the Q queries (q_user / q_item, device int32): one GPU's query shard needs
 * its own users and items, not the whole table.  Later fia_count_related calls (with
 * total_out) reject queries outside that set (FIA_ERR_STATE).
 *   large k (MF k >= 128, NCF k >= 64): compacted caches (20M ratings, NCF k=256: 1 MB per
 *     entity); synchronises `stream` (the cache size is decided on the host);
 *   small k: the entities are marked on the device and only their caches are computed (the
 *     layout stays dense); stream-ordered, no synchronisation.
 * Results for covered queries are bitwise identical to those after fia_prepare. */
int fia_prepare_for(fia_ctx* ctx, int64_t num_queries, const int32_t* q_user, const int32_t* q_item, void* stream);

/* offsets[q] = sum_{q'<q} n_q', offsets[Q] = total, with n_q = |R_u| + |C_i|
 * (device int64[Q+1]).  If total_out is non-NULL the total is copied to the
 * host and the stream is synchronised; out-of-range query ids are then
 * reported as FIA_ERR_INVALID. */
int fia_count_related(fia_ctx* ctx, int64_t num_queries, const int32_t* q_user, const int32_t* q_item,
                      int64_t* offsets, int64_t* total_out, void* stream);

/* rel_idx[offsets[q] + p] = p-th train row of the related list of query q (device
 * int32: fia_build_index limits n_train to < 2^31, so every train row fits; the reference's
 * np.where gives int64 -- the Python facade widens on the copy to the host, and the
 * device writes 4 B instead of 8 B per related rating). */
int fia_related(fia_ctx* ctx, int64_t num_queries, const int32_t* q_user, const int32_t* q_item,
                const int64_t* offsets, int32_t* rel_idx, void* stream);

/* Batched FIA: for every query q = (q_user[q], q_item[q]):
 *   H_t x = v solved exactly (fp64 LDL^T), then for every related rating p:
 *   influence[offsets[q]+p] = x . grad L_p / n_q   (mf:237-246),
 *   rel_idx[offsets[q]+p]   = its train row (int32, see fia_related).
 * x_out (nullable): device double[Q * D] in the reference theta order
 *   (MF [p_u, q_i, b_u, b_i], D = 2k+2; NCF [Pm_u, Qm_i, Pg_u, Qg_i], D = 4k).
 * rel_idx / influence may be NULL to skip writing the full vectors.
 * topk (K in [0, FIA_MAX_TOPK]; 0 = off): per query the K related ratings of
 * largest |influence| (ties: lower related position first), as related
 * position (topk_pos), train row (topk_idx) and signed influence (topk_val),
 * device arrays [Q*K]; unused slots hold -1 / NaN (n_q < K).
 * total_rel must equal offsets[Q].  Queries with n_q = 0 produce no ratings
 * and a NaN x (TF's mean over an empty batch). */
int fia_query_batch(fia_ctx* ctx, int64_t num_queries, const int32_t* q_user, const int32_t* q_item,
                    const int64_t* offsets, int64_t total_rel,
                    int32_t* rel_idx, double* influence, double* x_out,
                    int K, int64_t* topk_pos, int64_t* topk_idx, double* topk_val, void* stream);

/* fia_query_batch with a GIVEN inverse HVP instead of the solve: x_in (device double[Q * D],
 * the reference theta order, as fia_query_batch's x_out) replaces H_t^-1 v; the related sets,
 * influence and top-K follow from it exactly as in fia_query_batch.  Replaces the reference's
 * cached-inverse-HVP branch of get_influence_on_test_loss (force_refresh=False and an existing
 * <model>-cg-normal_loss-test-[t].npz, matrix_factorization.py:210-214).  Every built model:
 * small k records from x directly (k_record_x); large k (MF k >= 128, NCF k >= 64) skips the
 * batched LDL^T panels and writes the padded solution and records from x (k_big_record_x). */
int fia_query_batch_x(fia_ctx* ctx, int64_t num_queries, const int32_t* q_user, const int32_t* q_item,
                      const int64_t* offsets, int64_t total_rel, const double* x_in,
                      int32_t* rel_idx, double* influence,
                      int K, int64_t* topk_pos, int64_t* topk_idx, double* topk_val, void* stream);

/* Number of restricted parameters D of the registered model (0 if none). */
int fia_num_params(const fia_ctx* ctx);

/* Phase timing with HIP events recorded on the call's stream (for the
 * roofline figures of bench.py).  phase_mask bit p enables phase p (0 = off,
 * FIA_PROFILE_ALL = every phase): every fia_prepare / fia_query_batch then
 * records one event pair per enabled phase; fia_profile_read synchronises
 * them, returns per-phase sums (ms) and counts, and clears them.
 * Phases: 0 prepare, 1 solve, 2 score (the dominant gather/scoring kernel),
 * 3 topk merge, 4 chunk build + scan.  Each pair costs a little stream time,
 * so timed runs enable only the phase they price. */
#define FIA_NUM_PHASES 5
#define FIA_PROFILE_ALL 0x1f
int fia_set_profiling(fia_ctx* ctx, int phase_mask);
int fia_profile_read(fia_ctx* ctx, double* ms_sum /*[FIA_NUM_PHASES]*/, int64_t* counts /*[FIA_NUM_PHASES]*/);

#ifdef __cplusplus
}
#endif
#endif /* FIA_H_ */
