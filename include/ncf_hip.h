/*
 * ncf_hip.h — C-ABI of libncf_hip.so, the MI355X (gfx950) AdvancedNCF hot path.
 *
 * The reference (ethanshenley/Neural-Collaborative-Filtering-Demo) is pure Python; its hot path
 * is AdvancedNCF.forward / backward + torch.optim.Adam.step (src/model/architecture.py:258-381,
 * src/model/trainer.py:253-285), executed by ATen and torchrec kernels.  Each entry point below
 * replaces the implicit kernel(s) of one stage of that path; the host side (Python,
 * neural-collaborative-filtering-demo_amd/) binds them with ctypes.
 *
 * Conventions
 *   - plain device pointers, int64 sizes, fp32 data, int64 ids (KeyedJaggedTensor values);
 *   - every call is asynchronous on `stream` (a hipStream_t), never synchronises the host,
 *     never allocates: scratch comes from a caller-provided workspace (size queries below);
 *   - return 0 on success, a negative NCF_ERR_* code otherwise; ncf_last_error() gives a
 *     thread-local message.  Stateless and re-entrant; ordering is by stream.
 *   - ids outside [0, rows) never read out of bounds: they read row 0 and set bit 0 of the
 *     caller's device `err_flag` (the host raises IndexError, like nn.EmbeddingBag).
 */
#ifndef NCF_HIP_H
#define NCF_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NCF_OK 0
#define NCF_ERR_ARG (-1)
#define NCF_ERR_LAUNCH (-2)
#define NCF_ERR_WORKSPACE (-3)

/* Step clock: the per-step values of a training step kept on the device, so a whole step can be
 * captured once as a hipGraph and replayed (nothing step-dependent in any kernel argument).
 * t = steps completed; seed = this step's dropout stream.  Kernels that take a clock read it;
 * ncf_step_clock_advance() closes a step (t += 1, next seed = splitmix64(base_seed + t)).   */
typedef struct ncf_step_clock {
  int32_t t;
  int32_t reserved;   /* 0; used by ncf_adam_flat_clock_close during its launch */
  uint64_t seed;
} ncf_step_clock;
int ncf_step_clock_advance(ncf_step_clock* clock, uint64_t base_seed, void* stream);
/* Sets *clock = {t, 0, seed} on `stream` (a side stream's own copy of the step clock, set from the
 * host's step counter: kernels queued there read their step targets from it while the step's
 * stream advances the live clock without waiting for them). */
int ncf_step_clock_set(ncf_step_clock* clock, int32_t t, uint64_t seed, void* stream);

/* One wavefront waiting `microseconds` (<= 1e6) of wall-clock time on `stream`: the overlap
 * probe of a step's side streams (two spins on two streams finish in about one span when the
 * streams reach the GPU through different hardware queues).                                   */
int ncf_stream_spin(int64_t microseconds, void* stream);
/* A stream restricted to `keep_per8` of every 8 compute units (hipExtStreamCreateWithCUMask;
 * its own hardware queue), and its destruction.  Side-stream placement knob.                   */
int ncf_stream_create_cu_mask(int32_t keep_per8, void** out);
/* Blocks per CU the rolling table sweep launches at most (grid-stride beyond; default 16).
 * per_cu <= 0 queries.  Returns the previous value.  (A/B: the overlapped sweep's footprint.) */
int64_t ncf_adam_sweep_set_blocks(int64_t per_cu);
int ncf_stream_destroy(void* stream);
int ncf_version(void);
const char* ncf_last_error(void);
int ncf_device_count(void);
/* Build identity: "abi=<16 hex> src=<16 hex>", the hash of the ctypes table the library was built
 * against (_lib.SIGNATURES) and of the kernel sources it was compiled from (_abi.py).  The
 * loader refuses a library whose hashes differ from the Python side and sources beside it.
 * (Packaging plumbing: the reference is pure Python and has no compiled library to match.)   */
const char* ncf_build_info(void);

/* Cross-stream ordering (hipEventRecord / hipStreamWaitEvent, events created without timing).
 * Replaces: the torch.cuda.Event record / wait_event pairs of the step's fork / join points
 * (this port's own plumbing: the reference runs one stream).  As entry points they are part of
 * a recorded launch sequence (launch tapes) and replay in order with it.     */
int ncf_event_create(void** event);
/* scope 0: as ncf_event_create (a system-scope release when recorded: host waits see every
 * write before it); 1: a device-scope release (hipEventReleaseToDevice: enough for another
 * stream of this device to wait on; no host reads behind it); 2: no fence of the event's own
 * (hipEventDisableSystemFence: the preceding kernels' own releases only)                     */
int ncf_event_create_scoped(void** event, int32_t scope);
int ncf_event_destroy(void* event);
int ncf_event_record(void* event, void* stream);
int ncf_stream_wait_event(void* stream, void* event);
int ncf_event_synchronize(void* event);   /* host wait */
/* stream-ordered hipMemcpyAsync (hipMemcpyDefault): the sharded step's count copies */
int ncf_memcpy_async(void* dst, const void* src, int64_t bytes, void* stream);

/* ---- a2+a3+a4: EBC lookups x4 + mf_norm/mlp_norm + GMF dot --------------------------------
 * Replaces: EmbeddingBagCollection fwd (architecture.py:286-287), LayerNorms (:305-306,
 * :311-312), mf_vector/mf_output (:307-308).  Writes mf_pred[n], LN'd MLP rows [n,dim] (the
 * attention inputs) and, when non-NULL, LN'd GMF rows (kept for the backward).            */
int ncf_gather_ln_gmf_fwd(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                          const float* mf_user, const float* mf_item, const float* mlp_user,
                          const float* mlp_item, int64_t num_users, int64_t num_items,
                          int64_t dim, const float* mf_gamma, const float* mf_beta,
                          const float* mlp_gamma, const float* mlp_beta, const float* mf_out_w,
                          const float* mf_out_b, float eps, float* mf_pred, float* mlp_user_ln,
                          float* mlp_item_ln, float* mf_user_ln, float* mf_item_ln,
                          int* err_flag, void* stream);

/* forward_simple(hour=h) variant (architecture.py:432-458): the LN'd item rows of both paths are
 * multiplied by (1 + scale_factor * item_scale[row]) before the GMF dot product and before
 * they are stored; item_scale [n, dim] = the call's projection of hour_E[h] (or hour_E[h] when
 * T == D), scale_factor = 0.3 in the reference.                                               */
int ncf_gather_ln_gmf_scaled_fwd(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                                 const float* mf_user, const float* mf_item,
                                 const float* mlp_user, const float* mlp_item, int64_t num_users,
                                 int64_t num_items, int64_t dim, const float* mf_gamma,
                                 const float* mf_beta, const float* mlp_gamma,
                                 const float* mlp_beta, const float* mf_out_w,
                                 const float* mf_out_b, float eps, const float* item_scale,
                                 float scale_factor, int64_t group_rows, float* mf_pred,
                                 float* mlp_user_ln, float* mlp_item_ln, float* mf_user_ln,
                                 float* mf_item_ln, int* err_flag, void* stream);
/* group_rows = G > 1 (training, SURVEY fact 6: a group's rows hold one user): the LN'd user rows
 * (mlp_user_ln, mf_user_ln) are written only for a group's first row and for rows whose user
 * differs from that row's; every other row's are the first row's (readers: ncf_attn_block_* and
 * ncf_mlp_bwd's head with the same user_ids / group_rows).  0 or 1: every row written. */

/* Row gather (+ optional LayerNorm): EBC forward as read by callers (app.py:156-184) and
 * get_user_embeddings / get_product_embeddings (architecture.py:383-407).                   */
/* bf16-table configuration: the training gather over bf16 table rows (fp32 outputs). */
/* ncf_gather_ln_gmf_fwd over tables whose rows are table_ld floats apart (>= dim; the
 * row-sharded step's received rows read in place: [mf | mlp] halves, table_ld = 2 D). */
int ncf_gather_ln_gmf_ld_fwd(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                             const float* mf_user, const float* mf_item, const float* mlp_user,
                             const float* mlp_item, int64_t num_users, int64_t num_items,
                             int64_t dim, int64_t table_ld, const float* mf_gamma,
                             const float* mf_beta, const float* mlp_gamma, const float* mlp_beta,
                             const float* mf_out_w, const float* mf_out_b, float eps,
                             int64_t group_rows, float* mf_pred, float* mlp_user_ln,
                             float* mlp_item_ln, float* mf_user_ln, float* mf_item_ln,
                             int* err_flag, void* stream);
int ncf_gather_ln_gmf_bf16_fwd(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                               const uint16_t* mf_user, const uint16_t* mf_item,
                               const uint16_t* mlp_user, const uint16_t* mlp_item,
                               int64_t num_users, int64_t num_items, int64_t dim,
                               const float* mf_gamma, const float* mf_beta, const float* mlp_gamma,
                               const float* mlp_beta, const float* mf_out_w, const float* mf_out_b,
                               float eps, int64_t group_rows, float* mf_pred, float* mlp_user_ln,
                               float* mlp_item_ln, float* mf_user_ln, float* mf_item_ln,
                               int* err_flag, void* stream);
int ncf_gather_rows(const int64_t* ids, int64_t n, const float* table, int64_t rows,
                    int64_t dim, const float* ln_gamma, const float* ln_beta, float eps,
                    float* out, int* err_flag, void* stream);
/* 8f rank 2, ANN feed (generate_embeddings.py:201-221): ncf_gather_rows + each row divided by
 * its L2 norm when l2_normalize != 0 (the product "mlp" vectors for the JSONL export). */
int ncf_embedding_export(const int64_t* ids, int64_t n, const float* table, int64_t rows,
                         int64_t dim, const float* ln_gamma, const float* ln_beta, float eps,
                         int l2_normalize, float* out, int* err_flag, void* stream);

/* ---- dense layers: fp32 MFMA GEMM (v_mfma_f32_32x32x2_f32) --------------------------------
 * Replaces the addmm/mm of the attention projections (architecture.py:40-42, :57) and the MLP
 * tower Linear layers (:230-246) fwd and bwd.  C = act(A·B + bias); A(i,k) = a_trans ?
 * A[k*lda+i] : A[i*lda+k]; B(k,j) = b_trans ? B[j*ldb+k] : B[k*ldb+j]; flags bit0 = ReLU,
 * bit1 = accumulate into C.                                                                */
int ncf_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int a_trans,
                 const float* B, int64_t ldb, int b_trans, float* C, int64_t ldc,
                 const float* bias, int flags, void* stream);
/* LDS-free variant for the square DxD attention projections: one wave per 32x32 tile, MFMA
 * operands loaded straight from global memory (k permuted per 64-chunk so contiguous operands
 * are float4 runs and strided ones are coalesced per step).  Same convention as ncf_gemm_f32. */
int ncf_gemm_direct(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int a_trans,
                    const float* B, int64_t ldb, int b_trans, float* C, int64_t ldc,
                    const float* bias, int flags, void* stream);

/* Weights-resident streaming variant (row-major A only; K, N in {64,128,256}, N*K <= 32768):
 * B is staged once per workgroup into LDS, waves stream 32-row tiles of A with all N output
 * columns each (A read from HBM exactly once).  Same B / flags convention as ncf_gemm_f32.   */
int ncf_gemm_rows(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
                  int64_t ldb, int b_trans, float* C, int64_t ldc, const float* bias, int flags,
                  void* stream);

/* ---- deferred reductions --------------------------------------------------------------------
 * Every backward call that produces a parameter gradient as a sum over batch rows writes
 * per-block partial rows and reduces them in a fixed order (bitwise reproducible, no float
 * atomics).  Given a non-NULL `defer` list such a call APPENDS its reduction(s) to the list
 * instead of launching them — its workspace then holds the partials and must stay untouched
 * until ncf_reduce_batch() has run every listed reduction (two launches for the whole list).
 * The weight/bias gradients are off the backward's critical path, so a training step pays two
 * launches for all of them instead of ~40.                                                   */
typedef struct ncf_reduce_desc {
  const float* part;  /* P partial rows, row p at part + p*stride, L floats each               */
  float* out;         /* element i -> out[(i / cols) * ldo + i % cols]                        */
  int64_t stride;
  int64_t ldo;
  int32_t L, cols, P, accumulate;
  float scale;        /* out = scale * sum (+ previous out when accumulate)                  */
  int32_t reserved;
} ncf_reduce_desc;
#define NCF_REDUCE_LIST_MAX 64
typedef struct ncf_reduce_list {
  int32_t count;
  int32_t reserved;
  ncf_reduce_desc d[NCF_REDUCE_LIST_MAX];
} ncf_reduce_list;
int64_t ncf_reduce_batch_scratch(const ncf_reduce_list* list);
/* Stage lanes of 16 bytes (four adjacent columns per lane) for descriptors whose L, stride and
 * partial base allow it (default on; same bits either way).  on < 0 queries.  Returns the
 * previous setting.  (Round 6: the batch's reductions' loads widened.)                       */
int64_t ncf_reduce_set_vec(int64_t on);
int ncf_reduce_batch(const ncf_reduce_list* list, float* scratch, int64_t scratch_floats,
                     void* stream);

int64_t ncf_gemm_splitk_workspace(int64_t M, int64_t N, int splits);
/* Long-K GEMM for weight gradients (dW = dYᵀ·X over the batch): K split into `splits` slabs
 * reduced in slab order.  row_sums (nullable) receives sum_k A(i,k) from the same pass — the
 * bias gradient when A = dYᵀ.  defer: see above.                                            */
int ncf_gemm_f32_splitk(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                        int a_trans, const float* B, int64_t ldb, int b_trans, float* C,
                        int64_t ldc, int accumulate, float* row_sums, int splits,
                        float* workspace, int64_t workspace_floats, ncf_reduce_list* defer,
                        void* stream);
/* Grouped weight gradients (all dW = dYᵀ·X of a step in one launch, + bias gradients = column
 * sums of dY when dbias != NULL).  dY [n, m_out] (ld ldy), X [n, k_in] (ld ldx), dW [m_out, k_in]
 * (ld ldw, accumulate or overwrite); the batch rows are split into `slabs` row slabs whose
 * partials are summed in slab order (deferred to `defer` when non-NULL).                      */
typedef struct ncf_wgrad_desc {
  const float* dy;
  const float* x;
  float* dw;
  float* dbias;
  int64_t ldy, ldx, ldw;
  int32_t m_out, k_in, n, slabs, accumulate, reserved;
} ncf_wgrad_desc;
#define NCF_WGRAD_GROUP_MAX 8
int64_t ncf_wgrad_grouped_workspace(const ncf_wgrad_desc* descs, int count);
int ncf_wgrad_grouped(const ncf_wgrad_desc* descs, int count, float* workspace,
                      int64_t workspace_floats, ncf_reduce_list* defer, void* stream);
int64_t ncf_colsum_workspace(int64_t rows, int64_t cols);
/* Bias gradients: out[c] (+)= sum_r X[r*ld+c]. */
int ncf_colsum(const float* X, int64_t rows, int64_t cols, int64_t ld, float* out,
               int accumulate, float* workspace, int64_t workspace_floats, void* stream);

/* p[r*ld + c] = value (zero the gradient columns of mlp.0.weight that see the all-zero
 * temporal features, architecture.py:329-340). */
int ncf_fill_2d(float* p, int64_t rows, int64_t cols, int64_t ld, float value, void* stream);

/* ---- a5: MultiHeadAttention core over each group of `group_len` rows ----------------------
 * Replaces MultiHeadAttention.forward's bmm/softmax/dropout/bmm (architecture.py:45-55) as
 * called at :319-323.  q,k,v,out: [groups*group_len, dim]; probs: [groups, heads, L, L]
 * (pre-dropout softmax, saved for backward).  group_len <= 64, head dim in {8,16,32,64}.   */
/* Dropout masks depend on seed + (clock ? clock->seed : 0).                                */
int ncf_attention_fwd(const float* q, const float* k, const float* v, int64_t groups,
                      int64_t group_len, int64_t heads, int64_t dim, float dropout_p,
                      uint64_t seed, const ncf_step_clock* clock, float* probs, float* out,
                      void* stream);
/* The same with MultiHeadAttention.forward's mask (architecture.py:36, 47-48: scores.masked_fill(
 * mask == 0, -inf)): mask [groups, heads, L, L] bytes (0 = masked; a broadcast mask expanded by
 * the caller).  Masked probabilities are exactly 0, so ncf_attention_bwd applies unchanged; a
 * fully masked row is NaN, as the reference's softmax over all -inf makes it.               */
int ncf_attention_fwd_masked(const float* q, const float* k, const float* v, int64_t groups,
                             int64_t group_len, int64_t heads, int64_t dim, float dropout_p,
                             uint64_t seed, const ncf_step_clock* clock, const uint8_t* mask,
                             float* probs, float* out, void* stream);
int ncf_attention_bwd(const float* q, const float* k, const float* v, const float* probs,
                      const float* grad_out, int64_t groups, int64_t group_len, int64_t heads,
                      int64_t dim, float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                      float* grad_scores, float* grad_q, float* grad_k, float* grad_v,
                      void* stream);
/* The whole a5 block in one launch per direction (D = 64 or 128, M <= 6; ncf_attn_block_supported):
 * forward  q,k,v = LN rows x W^T + b, the core above (same P layout and dropout stream), y =
 *          o Wo^T + bo.  q = k = NULL: nothing is stashed (with M == 1 and no dropout this is
 *          the eval form, o = v; otherwise the core runs in LDS only, for ncf_attn_block_bwd_rc);
 *          probs required when q is given; o may be NULL (not stashed: ncf_attn_block_bwd
 *          given o = NULL recomputes it from probs and v with the forward's arithmetic).
 * backward from dY: dO = dY Wo, the core backward, dXu = dQ Wq, dXi = dK Wk + dV Wv, and the
 *          four Linear gradients (below).                                                     */
int ncf_attn_block_supported(int64_t dim, int64_t heads, int64_t group_len);
/* user_ids (may be NULL): the user id of every row.  A workgroup whose groups each hold one user
 * (the reference's collate, data_prep.py:201) projects Q once per group (the same
 * bits as per row) and stashes it once per group, at the group's first row of q (the other rows
 * of q are not written); ncf_attn_block_bwd given the same user_ids reads it there.           */
int ncf_attn_block_fwd(const float* xu, const float* xi, int64_t groups, int64_t group_len,
                       int64_t heads, int64_t dim, const float* wq, const float* bq,
                       const float* wk, const float* bk, const float* wv, const float* bv,
                       const float* wo, const float* bo, float dropout_p, uint64_t seed,
                       const ncf_step_clock* clock, float* q, float* k, float* v, float* probs,
                       float* o, float* y, const int64_t* user_ids, void* stream);
/* Fused weight gradients: grad_params = {q.weight, q.bias, k.weight, k.bias, v.weight, v.bias,
 * out.weight, out.bias} (written, not accumulated) from per-workgroup partials in `workspace`
 * (ncf_attn_block_bwd_workspace floats), reduced now or deferred into `defer`; then grad_q/k/v
 * may be NULL.  grad_params = NULL: no weight gradients, grad_q/k/v written for a separate
 * weight-gradient pass (o/xu/xi/workspace unused). */
int64_t ncf_attn_block_bwd_workspace(int64_t groups);
int ncf_attn_block_bwd(const float* grad_y, const float* q, const float* k, const float* v,
                       const float* probs, int64_t groups, int64_t group_len, int64_t heads,
                       int64_t dim, const float* wq, const float* wk, const float* wv,
                       const float* wo, float dropout_p, uint64_t seed,
                       const ncf_step_clock* clock, const float* o, const float* xu,
                       const float* xi, float* const* grad_params, float* workspace,
                       int64_t workspace_floats, ncf_reduce_list* defer, float* grad_q,
                       float* grad_k, float* grad_v, float* grad_xu, float* grad_xi,
                       const int64_t* user_ids, void* stream);
/* The same backward (fused weight gradients) after a forward that stashed nothing: q, k, v are
 * re-projected from xu / xi (+ the biases) and the core forward (probabilities, o) is re-run in
 * LDS with the forward's own arithmetic (same bits), instead of reading q/k/v/o/probs from HBM.
 * ncf_attn_block_rc_supported: the shapes whose recomputed probabilities fit in LDS beside dS. */
int ncf_attn_block_rc_supported(int64_t dim, int64_t heads, int64_t group_len);
int ncf_attn_block_bwd_rc(const float* grad_y, const float* xu, const float* xi, int64_t groups,
                          int64_t group_len, int64_t heads, int64_t dim, const float* wq,
                          const float* bq, const float* wk, const float* bk, const float* wv,
                          const float* bv, const float* wo, float dropout_p, uint64_t seed,
                          const ncf_step_clock* clock, float* const* grad_params,
                          float* workspace, int64_t workspace_floats, ncf_reduce_list* defer,
                          float* grad_xu, float* grad_xi, const int64_t* user_ids, void* stream);

/* ---- a7 + a8 fused: the MLP tower in one launch per direction (input 64, hidden [256,128,64];
 * ncf_mlp_fused_supported).  Layer l = mlp.{4l} Linear (w [N_l][ldw], first K_l columns used:
 * mlp.0's temporal columns see zeros), mlp.{4l+2} LayerNorm (gamma, beta); dropout seed of layer
 * l = (seed + 0x9E37*(l+1)) & (2^63-1) (+ clock), the unfused path's stream.
 * Forward: r = relu(x W^T + b), mean/rstd, a = dropout(LN(r)) per layer (r/a/mean/rstd may be
 *   NULL: not saved), then mlp_pred = a_2 . mlp_out_w + mlp_out_b and
 *   prob = sigmoid(final_w[0] mf_pred + final_w[1] mlp_pred + final_b) (the ncf_head_fwd math).
 * Backward: from dL/da_2 (ncf_head_bwd's grad_mlp_last) -> dlin per layer (written when
 *   non-NULL: the weight gradients' dY; required unless the dw are set), grad_x = dL/dx [n,64];
 *   dbias/dgamma/dbeta per layer through the workspace (deferred into `defer` when given).
 *   r/mean/rstd are required; where `a` is NULL the backward recomputes a = dropout(LN(r))
 *   bit-identically from r/mean/rstd and the dropout stream (so the forward need not save it). */
typedef struct ncf_mlp_layer {
  const float* w;
  int64_t ldw;
  const float* b;
  const float* gamma;
  const float* beta;
  float* r;
  float* a;
  float* mean;
  float* rstd;
  float* dlin;
  float* dbias;
  float* dgamma;
  float* dbeta;
  float* dw;     /* weight gradient [N_l][ldw] (first K_l columns written); all three set:
                  * the backward computes them too (per-workgroup partials, deferred) */
} ncf_mlp_layer;
int ncf_mlp_fused_supported(int64_t dim, int64_t n_layers, const int64_t* hidden);
int ncf_mlp_fwd(const float* x, int64_t n, int64_t dim, const ncf_mlp_layer* layers,
                int64_t n_layers, const int64_t* hidden, float eps, float dropout_p, uint64_t seed,
                const ncf_step_clock* clock, const float* mlp_out_w, const float* mlp_out_b,
                const float* mf_pred, const float* final_w, const float* final_b, float* mlp_pred,
                float* prob, void* stream);
/* Fused head backward (the ncf_head_bwd math, W3 = D = 64): with `head` given, the tower's
 * backward starts from the loss instead of grad_a_last (which may be NULL): dL/dprob from
 * grad_prob or the mean BCE of targets (loss_denominator as in ncf_head_bwd), the GMF row
 * gradients, and the six head parameter gradients + loss through the same workspace / defer list.
 * Needs layers[2].a (the forward's last activation).                                           */
typedef struct ncf_head_args {
  const float* prob;
  const float* grad_prob;
  const float* targets;
  const float* mf_pred;
  const float* mlp_pred;
  const float* mf_user_ln;
  const float* mf_item_ln;
  const float* mlp_out_w;
  const float* final_w;
  const float* mf_out_w;
  float* grad_mf_user_ln;
  float* grad_mf_item_ln;
  float* grad_mlp_out_w;
  float* grad_mlp_out_b;
  float* grad_mf_out_w;
  float* grad_mf_out_b;
  float* grad_final_w;
  float* grad_final_b;
  float* loss;
  double loss_denominator;
  /* optional: the batch's user ids and group size (the gather's group_rows): a row whose user is
   * its group's first row's user reads mf_user_ln at that first row (NULL / <= 1: its own) */
  const int64_t* user_ids;
  int64_t group_rows;
} ncf_head_args;
int64_t ncf_mlp_bwd_workspace(int64_t n);
int ncf_mlp_bwd(const float* grad_a_last, int64_t n, int64_t dim, const float* x,
                const ncf_mlp_layer* layers,
                int64_t n_layers, const int64_t* hidden, float dropout_p, uint64_t seed,
                const ncf_step_clock* clock, const ncf_head_args* head, float* grad_x,
                float* workspace, int64_t workspace_floats, ncf_reduce_list* defer, void* stream);

/* bf16 configuration: the tower with its Linears on bf16 MFMA (operands rounded to bf16, fp32
 * accumulate, v_mfma_f32_16x16x32_bf16 / 16x16x16_bf16); same arguments as the fp32 forms.   */
int ncf_mlp_fwd_bf16(const float* x, int64_t n, int64_t dim, const ncf_mlp_layer* layers,
                     int64_t n_layers, const int64_t* hidden, float eps, float dropout_p,
                     uint64_t seed, const ncf_step_clock* clock, const float* mlp_out_w,
                     const float* mlp_out_b, const float* mf_pred, const float* final_w,
                     const float* final_b, float* mlp_pred, float* prob, void* stream);
int ncf_mlp_bwd_bf16(const float* grad_a_last, int64_t n, int64_t dim, const float* x,
                     const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                     float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                     const ncf_head_args* head, float* grad_x, float* workspace,
                     int64_t workspace_floats, ncf_reduce_list* defer, void* stream);

/* fp32 tower on bf16 matrix cores through split operands: every fp32 operand x = h + m + l
 * (three bf16 terms, round to nearest), a product accumulated from the six bf16 products of
 * order >= 2^-16 (v_mfma_f32_16x16x32_bf16, fp32 accumulate; the dropped terms are below 2^-24
 * of it, fp32's own rounding level); row ops fp32.  Same arguments as ncf_mlp_fwd / _bwd.     */
int ncf_mlp_fwd_split(const float* x, int64_t n, int64_t dim, const ncf_mlp_layer* layers,
                      int64_t n_layers, const int64_t* hidden, float eps, float dropout_p,
                      uint64_t seed, const ncf_step_clock* clock, const float* mlp_out_w,
                      const float* mlp_out_b, const float* mf_pred, const float* final_w,
                      const float* final_b, float* mlp_pred, float* prob, void* stream);
int ncf_mlp_bwd_split(const float* grad_a_last, int64_t n, int64_t dim, const float* x,
                      const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                      float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                      const ncf_head_args* head, float* grad_x, float* workspace,
                      int64_t workspace_floats, ncf_reduce_list* defer, void* stream);

/* a5 + a7 + a8 forward fused (C2 training geometry: D = 64, groups of M = 5 rows, hidden
 * [256,128,64]): ncf_attn_block_fwd (training stash q/k/v/probs, no o) then ncf_mlp_fwd on its
 * output y in ONE launch, the attention output handed to the tower in LDS (y still written for
 * the backward's layer-0 weight gradient).  tower_mode: 0 fp32 MFMA, 1 bf16, 3 split operands.
 * Same results as the two launches.                                                           */
int ncf_attn_mlp_fused_supported(int64_t dim, int64_t heads, int64_t group_len, int64_t n_layers,
                                 const int64_t* hidden);
int ncf_attn_mlp_fwd(const float* xu, const float* xi, int64_t groups, int64_t heads,
                     const float* wq, const float* bq, const float* wk, const float* bk,
                     const float* wv, const float* bv, const float* wo, const float* bo,
                     float dropout_p, uint64_t seed, const ncf_step_clock* clock, float* q,
                     float* k, float* v, float* probs, float* y, const int64_t* user_ids,
                     const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                     float eps, const float* mlp_out_w, const float* mlp_out_b,
                     const float* mf_pred, const float* final_w, const float* final_b,
                     float* mlp_pred, float* prob, int32_t tower_mode, void* stream);
/* ... and the backward: ncf_mlp_bwd (head fused, weight gradients fused, x = y) then
 * ncf_attn_block_bwd on its input gradient in ONE launch, that gradient handed over in LDS
 * (never written to HBM).  The tower's partials in tower_workspace (ncf_mlp_bwd_workspace(n)),
 * the attention's in attn_workspace (ncf_attn_block_bwd_workspace(groups)); both deferred into
 * `defer` (required).  Same results as the two launches.                                       */
int ncf_attn_mlp_bwd(int64_t groups, int64_t heads, const float* y, const ncf_mlp_layer* layers,
                     int64_t n_layers, const int64_t* hidden, float dropout_p, uint64_t seed,
                     const ncf_step_clock* clock, const ncf_head_args* head,
                     float* tower_workspace, int64_t tower_workspace_floats, const float* q,
                     const float* k, const float* v, const float* probs, const float* wq,
                     const float* wk, const float* wv, const float* wo, const float* xu,
                     const float* xi, float* const* attn_grad_params, float* attn_workspace,
                     int64_t attn_workspace_floats, float* grad_xu, float* grad_xi,
                     const int64_t* user_ids, ncf_reduce_list* defer, int32_t tower_mode,
                     void* stream);
/* Partial floats of the fused backward for `groups` groups: the tower's (which = 0) and the
 * attention block's (which = 1) workspaces; at least ncf_mlp_bwd_workspace(5 groups) /
 * ncf_attn_block_bwd_workspace(groups) ask for.                                              */
int64_t ncf_attn_mlp_bwd_workspace(int64_t groups, int32_t which);
/* The same three entry points (and the workspace query) in small-batch tiles: 3 groups (15 rows)
 * per workgroup instead of 16 (tower_fused_small.hip).  The reference's default batch of 256
 * groups (config.yaml:65) then fills 86 workgroups instead of 16.  Forward outputs and input
 * gradients are the same bits as the 80-row tiles'; the weight gradients are the same sums
 * grouped per workgroup differently (fp32 rounding).  Workspaces from
 * ncf_attn_mlp_bwd_workspace_small (more partial sets than the 80-row tiles leave).         */
int ncf_attn_mlp_fused_supported_small(int64_t dim, int64_t heads, int64_t group_len,
                                       int64_t n_layers, const int64_t* hidden);
int ncf_attn_mlp_fwd_small(const float* xu, const float* xi, int64_t groups, int64_t heads,
                           const float* wq, const float* bq, const float* wk, const float* bk,
                           const float* wv, const float* bv, const float* wo, const float* bo,
                           float dropout_p, uint64_t seed, const ncf_step_clock* clock, float* q,
                           float* k, float* v, float* probs, float* y, const int64_t* user_ids,
                           const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                           float eps, const float* mlp_out_w, const float* mlp_out_b,
                           const float* mf_pred, const float* final_w, const float* final_b,
                           float* mlp_pred, float* prob, int32_t tower_mode, void* stream);
int ncf_attn_mlp_bwd_small(int64_t groups, int64_t heads, const float* y,
                           const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                           float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                           const ncf_head_args* head, float* tower_workspace,
                           int64_t tower_workspace_floats, const float* q, const float* k,
                           const float* v, const float* probs, const float* wq, const float* wk,
                           const float* wv, const float* wo, const float* xu, const float* xi,
                           float* const* attn_grad_params, float* attn_workspace,
                           int64_t attn_workspace_floats, float* grad_xu, float* grad_xi,
                           const int64_t* user_ids, ncf_reduce_list* defer, int32_t tower_mode,
                           void* stream);
int64_t ncf_attn_mlp_bwd_workspace_small(int64_t groups, int32_t which);

/* ---- 8f rank 1: device-side training batches (data_prep.py:95-161, 181-313) --------------
 * ncf_alias_build (HOST function, once per dataset): Walker/Vose alias table of the
 *   inverse-popularity weights.
 * ncf_sample_negatives: per interaction b, rows b*(1+k) .. b*(1+k)+k of the KJT batch:
 *   out_users = user, out_items = [pos, k negatives], out_targets = [1, 0, ...].  A negative is
 *   an alias-table draw rejected when it is the positive or in the user's history (CSR:
 *   hist_items[hist_offsets[u] .. hist_offsets[u+1]) sorted ascending; NULL offsets = no
 *   history), up to max_attempts draws, then uniform over the items outside history + {pos}
 *   (any item but pos when that set is empty).  Deterministic in (inputs, seed). */
int ncf_alias_build(const double* weights, int64_t n, float* prob, int32_t* alias);
int ncf_sample_negatives(const int64_t* users, const int64_t* pos_items, int64_t batch,
                         int64_t negatives, const float* alias_prob, const int32_t* alias_idx,
                         int64_t n_items, const int64_t* hist_offsets, const int32_t* hist_items,
                         int64_t n_users, uint64_t seed, int64_t max_attempts, int64_t* out_users,
                         int64_t* out_items, float* out_targets, int* err_flag, void* stream);

/* ---- 8f rank 4: ranking metrics over [groups, group_len] (src/utils/metrics.py) -----------
 * ncf_group_metrics: out[4j + {0,1,2,3}] = sums over groups of hit@k, ndcg@k, mrr@k, map@k for
 *   k = ks[j] (clamped to group_len); out[4nk + {0..4}] = #correct, #positives,
 *   #correct positives, #negatives, #correct negatives at `threshold`.  Rank order per group:
 *   prediction desc, column asc.  group_len <= 64, nk <= 16.
 * ncf_auc_count: *sum_2u = sum over positives (targets == 1) of (#neg < s) + (#neg <= s), with
 *   neg_sorted = the negatives' predictions ascending; AUC = sum_2u / (2 P N). */
int64_t ncf_group_metrics_workspace(int64_t groups, int64_t nk);
int ncf_group_metrics(const float* pred, const float* targets, int64_t groups, int64_t group_len,
                      const int32_t* ks, int64_t nk, float threshold, double* out,
                      void* workspace, int64_t workspace_bytes, void* stream);
int ncf_auc_count(const float* pred, const float* targets, int64_t n, const float* neg_sorted,
                  int64_t n_neg, unsigned long long* sum_2u, void* stream);

/* ---- a6: TemporalEncoding (architecture.py:59-94): hour/day/month rows + pe[days mod P] -- */
int ncf_temporal_fwd(const int64_t* hour, const int64_t* day, const int64_t* month,
                     const int64_t* days_since, int64_t n, const float* hour_embed,
                     const float* day_embed, const float* month_embed, const float* pe,
                     int64_t max_period, int64_t dim, float* out, int* err_flag, void* stream);
int ncf_temporal_bwd(const int64_t* hour, const int64_t* day, const int64_t* month, int64_t n,
                     const float* grad_out, int64_t dim, float* grad_hour, float* grad_day,
                     float* grad_month, void* stream);

/* ---- a7: MLP tower row ops (ReLU -> LayerNorm -> Dropout), architecture.py:233-239 --------
 * Backward also returns grad_bias = column sums of grad_lin (the bias gradient of the Linear
 * that feeds the ReLU; nullable).                                                            */
/* out[r, c] = x[r, c] * keep-scale of (r, c / group) from the package's dropout stream (seed);
 * the keep-scales optionally to scales[rows][cols / group].  group = 1: nn.Dropout per element;
 * group = head dim: attention-weight dropout over a single key (CategoryHierarchy in training
 * mode, architecture.py:45-51, 114-117).  In place allowed.                                    */
int ncf_dropout_rows(const float* x, int64_t rows, int64_t cols, int64_t group, float dropout_p,
                     uint64_t seed, float* out, float* scales, void* stream);
int ncf_relu_ln_dropout_fwd(float* relu_in, int64_t n, int64_t width, const float* gamma,
                            const float* beta, float eps, float dropout_p, uint64_t seed,
                            const ncf_step_clock* clock, float* out, float* mean, float* rstd,
                            void* stream);
int64_t ncf_relu_ln_dropout_bwd_workspace(int64_t n, int64_t width);
int ncf_relu_ln_dropout_bwd(const float* grad_out, const float* relu_in, const float* mean,
                            const float* rstd, const float* gamma, int64_t n, int64_t width,
                            float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                            float* grad_lin, float* grad_gamma,
                            float* grad_beta, float* grad_bias, float* workspace,
                            int64_t workspace_floats, ncf_reduce_list* defer, void* stream);

/* ---- a8 + a12: mlp_output + final Linear(2,1) + Sigmoid (+ fused BCELoss) -----------------
 * Replaces architecture.py:345, :353-354 and nn.BCELoss (trainer.py:78, :271).  With fused
 * BCE the mean is over loss_denominator samples (> 0; the global batch under DP) or n.      */
int ncf_head_fwd(const float* mlp_last, int64_t n, int64_t width, const float* mlp_out_w,
                 const float* mlp_out_b, const float* mf_pred, const float* final_w,
                 const float* final_b, float* mlp_pred, float* prob, void* stream);
int64_t ncf_head_bwd_workspace(int64_t n, int64_t width, int64_t dim);
int ncf_head_bwd(const float* prob, const float* grad_prob, const float* targets,
                 const float* mf_pred, const float* mlp_pred, const float* mlp_last, int64_t n,
                 int64_t width, const float* mlp_out_w, const float* final_w,
                 const float* mf_user_ln, const float* mf_item_ln, int64_t dim,
                 const float* mf_out_w, float* grad_mlp_last, float* grad_mf_user_ln,
                 float* grad_mf_item_ln, float* grad_mlp_out_w, float* grad_mlp_out_b,
                 float* grad_mf_out_w, float* grad_mf_out_b, float* grad_final_w,
                 float* grad_final_b, float* loss, double loss_denominator, float* workspace,
                 int64_t workspace_floats, ncf_reduce_list* defer, void* stream);

/* ---- a2/a3 backward: sparse segment-reduce + LayerNorm backward ----------------------------
 * Replaces _embedding_bag_dense_backward (+ sort) of the four EBC tables and the mf_norm /
 * mlp_norm backward.  Produces compact per-unique-id gradients and slot maps (slot[id] = c);
 * the dense [rows, D] gradient is never materialised.                                       */
int64_t ncf_embedding_bwd_workspace(int64_t n, int64_t dim);
/* The largest per-kind id count ncf_dedup_ids sorts in its one-launch form (bitonic sort in LDS,
 * one workgroup per kind; larger batches take the multi-launch radix sort).  Returns the previous
 * value; n < 0 only reads it, n is capped at 2048.  The two forms leave the same workspace
 * contents (tested); the setter exists for that A/B.                                        */
int64_t ncf_dedup_set_small_max(int64_t n);
int ncf_embedding_bwd(const int64_t* user_ids, const int64_t* item_ids, int64_t n, int64_t dim,
                      int64_t num_users, int64_t num_items, const float* dy_mf_user,
                      const float* dy_mlp_user, const float* dy_mf_item, const float* dy_mlp_item,
                      const float* mf_user, const float* mlp_user, const float* mf_item,
                      const float* mlp_item, const float* mf_gamma, const float* mlp_gamma,
                      float eps, float* grad_mf_user, float* grad_mlp_user, float* grad_mf_item,
                      float* grad_mlp_item, int64_t* uniq_users, int64_t* uniq_items,
                      int32_t* slot_users, int32_t* slot_items, uint32_t* num_unique,
                      float* grad_mf_gamma, float* grad_mf_beta, float* grad_mlp_gamma,
                      float* grad_mlp_beta, void* workspace, int64_t workspace_bytes,
                      void* stream);
/* Deduplication of two id lists of different lengths (kind 0 / kind 1); ncf_dedup_ids is the
 * n0 == n1 case. */
int ncf_dedup_ids2(const int64_t* ids0, int64_t n0, int64_t rows0, const int64_t* ids1,
                   int64_t n1, int64_t rows1, int64_t dim, int64_t* uniq0, int64_t* uniq1,
                   int32_t* slot0, int32_t* slot1, uint32_t* num_unique, void* workspace,
                   int64_t workspace_bytes, void* stream);
/* inv[position] = compact index of its id, for the dedup held in `workspace`. */
int ncf_dedup_inverse(int64_t n0, int64_t n1, int64_t rows0, int64_t rows1, int64_t dim,
                      int64_t* inv0, int64_t* inv1, void* workspace, int64_t workspace_bytes,
                      void* stream);

/* The two phases of ncf_embedding_bwd, separable so the dedup can run BEFORE the forward
 * (the deferred Adam catches up exactly the batch's rows before they are gathered):
 *   ncf_dedup_ids: stable radix sort + segment heads -> uniq ids, num_unique, optional slots;
 *   ncf_embedding_bwd_reduce: segment-reduce + LN backward using the same workspace.        */
int ncf_dedup_ids(const int64_t* user_ids, const int64_t* item_ids, int64_t n, int64_t dim,
                  int64_t num_users, int64_t num_items, int64_t* uniq_users, int64_t* uniq_items,
                  int32_t* slot_users, int32_t* slot_items, uint32_t* num_unique, void* workspace,
                  int64_t workspace_bytes, void* stream);
int ncf_embedding_bwd_reduce(int64_t n, int64_t dim, int64_t num_users, int64_t num_items,
                             const float* dy_mf_user, const float* dy_mlp_user,
                             const float* dy_mf_item, const float* dy_mlp_item,
                             const float* mf_user, const float* mlp_user, const float* mf_item,
                             const float* mlp_item, const float* mf_gamma, const float* mlp_gamma,
                             float eps, float* grad_mf_user, float* grad_mlp_user,
                             float* grad_mf_item, float* grad_mlp_item, const int64_t* uniq_users,
                             const int64_t* uniq_items, float* grad_mf_gamma, float* grad_mf_beta,
                             float* grad_mlp_gamma, float* grad_mlp_beta, void* workspace,
                             int64_t workspace_bytes, ncf_reduce_list* defer, void* stream);
/* The same reduce writing unique row c's two gradient rows at row out_rows_*[c] (stride out_ld
 * floats) of the four gradient pointers: the row-sharded step hands its send buffer ([mf | mlp]
 * halves of 2 D floats per row: grad_mf_* = buf, grad_mlp_* = buf + D, out_ld = 2 D) instead of
 * compact rows it then re-orders (ncf_shard_rows); the four table pointers' rows are table_ld
 * floats apart (its received rows read in place: 2 D). */
int ncf_embedding_bwd_reduce_rows(int64_t n, int64_t dim, int64_t num_users, int64_t num_items,
                                  const float* dy_mf_user, const float* dy_mlp_user,
                                  const float* dy_mf_item, const float* dy_mlp_item,
                                  const float* mf_user, const float* mlp_user,
                                  const float* mf_item, const float* mlp_item,
                                  const float* mf_gamma, const float* mlp_gamma, float eps,
                                  float* grad_mf_user, float* grad_mlp_user, float* grad_mf_item,
                                  float* grad_mlp_item, const int64_t* uniq_users,
                                  const int64_t* uniq_items, const int32_t* out_rows_users,
                                  const int32_t* out_rows_items, int64_t out_ld,
                                  int64_t table_ld, float* grad_mf_gamma, float* grad_mf_beta,
                                  float* grad_mlp_gamma, float* grad_mlp_beta, void* workspace,
                                  int64_t workspace_bytes, ncf_reduce_list* defer, void* stream);
/* bf16-table configuration: the same reduce with bf16 table rows (uint16 bit patterns). */
int ncf_embedding_bwd_reduce_bf16(int64_t n, int64_t dim, int64_t num_users, int64_t num_items,
                                  const float* dy_mf_user, const float* dy_mlp_user,
                                  const float* dy_mf_item, const float* dy_mlp_item,
                                  const uint16_t* mf_user, const uint16_t* mlp_user,
                                  const uint16_t* mf_item, const uint16_t* mlp_item,
                                  const float* mf_gamma, const float* mlp_gamma, float eps,
                                  float* grad_mf_user, float* grad_mlp_user, float* grad_mf_item,
                                  float* grad_mlp_item, const int64_t* uniq_users,
                                  const int64_t* uniq_items, float* grad_mf_gamma,
                                  float* grad_mf_beta, float* grad_mlp_gamma, float* grad_mlp_beta,
                                  void* workspace, int64_t workspace_bytes, ncf_reduce_list* defer,
                                  void* stream);
int ncf_slot_reset(const int64_t* uniq, const uint32_t* num_unique, int kind, int32_t* slot,
                   int64_t max_n, void* stream);
/* dense[uniq[c]] = grad_compact[c] (materialise a dense table gradient for non-Adam users). */
int ncf_scatter_compact_rows(float* dense_grad, int64_t dim, const int64_t* uniq,
                             const uint32_t* num_unique, int kind, const float* grad_compact,
                             int64_t max_n, void* stream);

/* ---- C5: batch candidate scoring (app.py:44-75 forward_simple over all products + nlargest) ---
 * Factorised eval logit(u, i) = q_u . p_i + bias_i (score.hip header); results ordered by
 * (logit desc, item id asc).  dim must be 64, except ncf_score_queries: its table rows may be 16,
 * 32 or 64 wide and its query rows are always 64 floats (zero-padded; the item rows of an index
 * over a narrower table are padded the same way).  Pipeline: queries -> sample logits (ncf_gemm_f32
 * with a strided B) -> ncf_score_kth thresholds -> ncf_score_collect candidates ->
 * ncf_score_select top-K (overflow[slot] = 1: re-run 3-4 for those slots with the returned thr). */
int ncf_score_queries(const int64_t* user_ids, int64_t n, const float* mf_user, int64_t rows,
                      int64_t dim, const float* mf_gamma, const float* mf_beta, float eps,
                      const float* mf_out_w, const float* final_w, float* queries, int* err_flag,
                      void* stream);
int ncf_score_item_bias(const float* mlp_item, int64_t n, const float* final_w,
                        const float* final_b, const float* mf_out_b, float* bias, void* stream);
/* ncf_score_kth: logit(u, j) = logits[u*S + j] + item_bias[j*stride]; item_bias may be NULL
 * when the sample logits already include the bias (the sample GEMM's column bias). */
int ncf_score_kth(const float* logits, int64_t n_users, int64_t S, int K, const float* item_bias,
                  int64_t stride, float* thr, void* stream);
/* The threshold sample on bf16 matrix cores: out[u*S + j] = fp16, rounded toward -inf, of the
 * two-term split logit q_u . p_(j*stride) + sample_bias[j] (items3: the ncf_score_split_items
 * planes of the n_items rows), within 1e-4 |q_u| max|p| of the fp32 logit; then its k-th per
 * user (S <= 38912).  A valid threshold is the k-th lowered by that bound (ncf_score_margin with
 * c = 1e-4): replaces ncf_gemm_f32 + ncf_score_kth with half the bytes and 16x the MFMA rate.
 * group = 8: out holds rows of Sg = ceil(S / 8), out[u*Sg + g] = the largest of the fp16 values of
 * sample items 8g .. 8g + 7 (the K-th largest group maximum is <= the K-th largest sample logit:
 * the same bound, 8x fewer bytes written and selected over); group = 1: rows of S. */
int ncf_score_sample_split16(const float* queries, int64_t n_users, const uint16_t* items3,
                             int64_t n_items, int64_t dim, int64_t stride,
                             const float* sample_bias, int64_t S, int64_t group, uint16_t* out,
                             void* stream);
int ncf_score_kth16(const uint16_t* logits, int64_t n_users, int64_t S, int K, float* thr,
                    void* stream);
/* A candidate of a user's list: its scan logit and item (shard-local index).  One 8-byte record
 * per candidate, [n_users][cap] of them: a run of one user's candidates lands in one contiguous
 * span (two 4-byte arrays put every run in two).                                             */
typedef struct __attribute__((aligned(8))) ncf_score_cand {
  float logit;
  int32_t item;
} ncf_score_cand;   /* (8-byte aligned: one 64-bit store per candidate) */
int ncf_score_collect(const float* queries, const int32_t* user_list, int64_t n_users,
                      const float* items, const float* item_bias, int64_t n_items, int64_t dim,
                      const float* thr, int64_t cap, uint32_t* count, ncf_score_cand* cand,
                      void* stream);
/* ncf_score_collect on the bf16 matrix cores at fp32 accuracy: every operand split into three
 * bf16 terms (24 significant bits), six products per logit accumulated in fp32.  items3: the
 * three bf16 planes [3][n_items][dim] of `items` (ncf_score_split_items).  Same candidate sets
 * (the logits differ from the fp32 scan's by accumulation rounding only, far inside the
 * threshold's margin). */
int ncf_score_split_items(const float* items, int64_t n_items, int64_t dim, uint16_t* items3,
                          void* stream);
int ncf_score_collect_split(const float* queries, const int32_t* user_list, int64_t n_users,
                            const uint16_t* items3, const float* item_bias, int64_t n_items,
                            int64_t dim, const float* thr, int64_t cap, uint32_t* count,
                            ncf_score_cand* cand, int terms, int64_t expected_per_user,
                            void* stream);
/* expected_per_user: the candidates per user the thresholds aim at (0: unknown); sizes the item
 * split so a wave's candidates fit its LDS slice (fewer, grouped global writes).
 * terms = 2: the scan takes only x0 + x1 of each operand (three products a0b0 + a0b1 + a1b0):
 * its logits are within 1e-4 * |q_u| * max_i |p_i| of fp32, so the thresholds are first lowered
 * by that (ncf_score_margin, with max_i |p_i| from ncf_score_item_norm_max) and the candidates'
 * logits recomputed in fp32 by ncf_score_select_rescored. */
int ncf_score_item_norm_max(const float* items, int64_t n_items, int64_t dim, uint32_t* out_bits,
                            void* stream);
int ncf_score_margin(const float* queries, const int32_t* user_list, int64_t n_users, int64_t dim,
                     const uint32_t* item_norm_max, float c, float* thr, void* stream);
int ncf_score_select_rescored(const int32_t* user_list, int64_t n_users, const uint32_t* count,
                              const ncf_score_cand* cand, int64_t cap, int K, const float* queries, const float* items,
                              const float* item_bias, int64_t dim, const uint32_t* item_norm_max,
                              float c, float* out_score, int64_t* out_item, float* thr,
                              uint32_t* overflow, const float* thr_check, void* stream);
/* thr_check (may be NULL): per user, a threshold T the collect was run below (its rank-j sample
 * logit, j < K, before the margins) that is not a guaranteed bound of the K-th logit.  Every item
 * with fp32 logit >= T was collected, so the K selected are exact iff K were found and the K-th
 * re-scored logit is >= T; otherwise overflow[slot] = 2 and the caller re-runs the user from a
 * guaranteed threshold (the sample's K-th). */
int ncf_score_select(const int32_t* user_list, int64_t n_users, const uint32_t* count,
                     const ncf_score_cand* cand, int64_t cap, int K,
                     float* out_score, int64_t* out_item, float* thr, uint32_t* overflow,
                     void* stream);
/* Item-sharded scoring: merge per-user lists of L = W*K (score, global item id)
 * gathered from W item shards into the top-K by (score desc, item id asc); id < 0 = empty slot
 * (an empty output slot is (0, -1)).  L, K <= 8192; item ids < 2^32 - 1. */
int ncf_score_merge(const float* cand_score, const int64_t* cand_item, int64_t n_users, int64_t L,
                    int K, float* out_score, int64_t* out_item, void* stream);

/* ---- a13: torch.optim.Adam step (trainer.py:71-75, :285) ----------------------------------
 * Dense-exact over a whole table via the slot map (every row decays every step).            */
int ncf_adam_table(float* param, float* exp_avg, float* exp_avg_sq, int64_t rows, int64_t dim,
                   const int32_t* slot, const float* grad_compact, double lr, double beta1,
                   double beta2, double eps, double weight_decay, double step, void* stream);
int ncf_adam_flat(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                  double lr, double beta1, double beta2, double eps, double weight_decay,
                  double step, void* stream);
/* One Adam step over a table given its dense gradient (n = rows * dim elements): elements whose
 * gradient is exactly zero take the zero-gradient form of the row-sparse schedules (adam.hip). */
int ncf_adam_table_dense_grad(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              int64_t n, double lr, double beta1, double beta2, double eps,
                              double weight_decay, double step, void* stream);

/* ---- (e) row sharding over W ranks: owner(id) = id mod W, local row = id div W ------------
 * The per-rank kernels of the row-sharded step (exchange.hip; the protocol and the RCCL
 * all-to-alls are in distributed.py).  R = ceil(rows / W) local rows per shard.
 *
 * ncf_shard_plan (requester): keys = (id mod W) * R + id div W, deduplicated (the radix dedup of
 *   ncf_dedup_ids2, whose segments stay in `workspace` for ncf_embedding_bwd_reduce); compact
 *   index c = rank of the row's key, so compact order = owner order.  Writes uniq keys,
 *   num_unique[2], inv (position -> compact index), counts[W][2] (rows per destination: users,
 *   items), send[] = the local rows in destination-major order (per destination: its user rows,
 *   then its item rows; exactly the all-to-all input), spos0/1[c] = send position of compact c.
 *   bounds: scratch of 3 * (W + 1) int32.  err_flag |= 1 / 2 for an out-of-range user / item id.
 * ncf_shard_recv: layout of a received buffer (per source s: kind-0 entries at
 *   [start[s], start[s] + n0[s]), kind-1 entries up to start[s + 1]).
 * ncf_shard_owner_prepare (owner): deduplicates the received local rows without a sort (a row
 *   occurs at most once per source): uniq0/1 (count[2]), uidx0/1 (row -> unique index; per local
 *   row), mark0/1 (per local row, claim tokens; zero-initialised, token > 0 new every call),
 *   pos0/1[u * W + s] = received position of row u from source s, -1 if none.  err |= 4 on an
 *   out-of-range row.
 * ncf_shard_owner_gather: out[j] = (t?0[row] | t?1[row]) for received entry j ([total][2 dim]).
 * ncf_shard_owner_gradsum: g?0[u] / g?1[u] = sum over s = 0..W-1 of the halves of got[pos[u][s]]
 *   (fixed rank order: deterministic).
 * ncf_shard_rows: requester rows in (dir 0: mini tables m?0/m?1 [c] = halves of buf[spos?[c]])
 *   and gradients out (dir 1: buf[spos?[c]] = (m?0[c] | m?1[c])).                            */
#define NCF_SHARD_MAX_WORLD 64
typedef struct ncf_shard_plan_out {
  int64_t* keys0;
  int64_t* keys1;
  int64_t* uniq0;
  int64_t* uniq1;
  uint32_t* num_unique;
  int64_t* inv0;
  int64_t* inv1;
  int64_t* counts;
  int32_t* send;
  int32_t* spos0;
  int32_t* spos1;
  int32_t* bounds;
  /* optional (NULL: not written): spos as int64, and each row's send position
   * rows0/1[r] = spos0/1[inv0/1[r]] — the row-sharded step reads its received rows in place */
  int64_t* spos64_0;
  int64_t* spos64_1;
  int64_t* rows0;
  int64_t* rows1;
} ncf_shard_plan_out;
typedef struct ncf_shard_recv {
  int32_t world;
  int32_t start[NCF_SHARD_MAX_WORLD + 1];
  int32_t n0[NCF_SHARD_MAX_WORLD];
} ncf_shard_recv;
int ncf_shard_plan(const int64_t* user_ids, const int64_t* item_ids, int64_t n, int world,
                   int64_t num_users, int64_t num_items, int64_t dim, const ncf_shard_plan_out* out,
                   void* workspace, int64_t workspace_bytes, int* err_flag, void* stream);
int ncf_shard_owner_prepare(const int32_t* recv, const ncf_shard_recv* layout, int32_t token,
                            int32_t* mark0, int32_t* mark1, int32_t* uidx0, int32_t* uidx1,
                            int64_t rows0, int64_t rows1, int64_t* uniq0, int64_t* uniq1,
                            uint32_t* count, int32_t* pos0, int32_t* pos1, int* err_flag,
                            void* stream);
int ncf_shard_owner_gather(const int32_t* recv, const ncf_shard_recv* layout, const float* t00,
                           const float* t01, int64_t rows0, const float* t10, const float* t11,
                           int64_t rows1, int64_t dim, float* out, void* stream);
int ncf_shard_owner_gradsum(const float* got, const int32_t* pos0, const int32_t* pos1,
                            const uint32_t* count, int64_t max_unique, int world, int64_t dim,
                            float* g00, float* g01, float* g10, float* g11, void* stream);
int ncf_shard_rows(float* buf, const int32_t* spos0, const int32_t* spos1,
                   const uint32_t* num_unique, int64_t max_n, int64_t dim, float* m00, float* m01,
                   float* m10, float* m11, int dir, void* stream);

/* RCCL communicators and the collectives of the row-sharded step on the caller's stream
 * (replace torch.distributed.all_to_all_single(out, in, recv_splits, send_splits) and
 * all_reduce(SUM) of the exchange phases; no c10d layer in between).  RCCL is resolved from the
 * librccl.so.1 already loaded in the process (ncf_comm_available() == 0 when there is none).
 * ncf_comm_unique_id (one rank) -> the same 128 bytes to every rank -> ncf_comm_init on all of
 * them (collective).  ncf_comm_alltoallv: send_rows / recv_rows are HOST arrays of `world`
 * per-peer row counts; peer p's rows sit at the prefix-sum offsets; a row is row_bytes bytes. */
int ncf_comm_available(void);
int ncf_comm_unique_id(uint8_t* id, int64_t bytes);
int ncf_comm_init(const uint8_t* id, int64_t bytes, int world, int rank, void** comm);
int ncf_comm_destroy(void* comm);
int ncf_comm_alltoallv(void* comm, const void* send, const int64_t* send_rows, void* recv,
                       const int64_t* recv_rows, int64_t row_bytes, void* stream);
int ncf_comm_allreduce_sum_f32(void* comm, float* buf, int64_t n, void* stream);

/* Deferred dense-exact schedule (bit-identical to ncf_adam_table, see adam.hip): rows carry
 * stamp[row] = last step reflected; step_table[4s .. 4s+3] = fp32 scalars of step s
 * (-lr/(1-b1^s), 1/sqrt(1-b2^s) for a gradient step; their ratio and eps / (-lr/(1-b1^s)) for
 * the folded zero-gradient step of untouched rows) (ncf_adam_step_scalars, `count` steps from
 * `first`, 4 floats each).  Two tables (GMF + MLP) sharing one id space go in one call
 * (p1/m1/v1 nullable).                                                                      */
int ncf_adam_step_scalars(double lr, double beta1, double beta2, double eps, int64_t first,
                          int64_t count, float* out_host);
int ncf_adam_rows_catchup(float* p0, float* m0, float* v0, float* p1, float* m1, float* v1,
                          int64_t dim, const int64_t* row_ids, const uint32_t* count, int kind,
                          int64_t max_n, int32_t* stamp, int32_t target, const float* step_table,
                          double beta1, double beta2, double eps, double weight_decay,
                          void* stream);
int ncf_adam_rows_apply(float* p0, float* m0, float* v0, const float* g0, float* p1, float* m1,
                        float* v1, const float* g1, int64_t dim, const int64_t* row_ids,
                        const uint32_t* count, int kind, int64_t max_n, int32_t* stamp,
                        int32_t step, const float* step_table, double beta1, double beta2,
                        double eps, double weight_decay, void* stream);
int ncf_adam_sweep(float* p0, float* m0, float* v0, float* p1, float* m1, float* v1,
                   int64_t row0, int64_t rows, int64_t dim, int32_t* stamp, int32_t target,
                   const float* step_table, double beta1, double beta2, double eps,
                   double weight_decay, void* stream);
/* Clock-driven forms (hipGraph-capturable): catch-up target = clock->t + target_rel; apply step
 * = clock->t + step_rel; the rolling sweep closes step s = clock->t + step_rel and brings slice
 * (s mod sweep_every) of `slice` rows current through s; the flat Adam applies step
 * clock->t + step_rel with the scalars of step_table (bit-identical to ncf_adam_flat).       */
int ncf_adam_rows_catchup_clock(float* p0, float* m0, float* v0, float* p1, float* m1, float* v1,
                                int64_t dim, const int64_t* row_ids, const uint32_t* count,
                                int kind, int64_t max_n, int32_t* stamp, int32_t target_rel,
                                const ncf_step_clock* clock, const float* step_table,
                                double beta1, double beta2, double eps, double weight_decay,
                                void* stream);
int ncf_adam_rows_apply_clock(float* p0, float* m0, float* v0, const float* g0, float* p1,
                              float* m1, float* v1, const float* g1, int64_t dim,
                              const int64_t* row_ids, const uint32_t* count, int kind,
                              int64_t max_n, int32_t* stamp, int32_t step_rel,
                              const ncf_step_clock* clock, const float* step_table, double beta1,
                              double beta2, double eps, double weight_decay, void* stream);
int ncf_adam_sweep_rolling(float* p0, float* m0, float* v0, float* p1, float* m1, float* v1,
                           int64_t total_rows, int64_t slice, int32_t sweep_every, int64_t dim,
                           int32_t* stamp, int32_t step_rel, const ncf_step_clock* clock,
                           const float* step_table, double beta1, double beta2, double eps,
                           double weight_decay, void* stream);
/* Both id kinds in one launch each (blockIdx.y = kind): pairs[k] holds kind k's GMF + MLP
 * tables (sharing the row index), their moments, compact gradients (apply), the step's unique
 * rows and the stamps; count[k] = unique rows of kind k (ncf_dedup_ids).                      */
/* param_dtype: NCF_DTYPE_F32, or NCF_DTYPE_BF16 when p0 / p1 point at bf16 rows (the moments stay
 * fp32; the parameter is rounded to bf16, nearest even, after every step it takes).           */
#define NCF_DTYPE_F32 0
#define NCF_DTYPE_BF16 1
typedef struct ncf_table_pair {
  float *p0, *m0, *v0, *p1, *m1, *v1;
  const float *g0, *g1;
  const int64_t* row_ids;
  int32_t* stamp;
  int64_t rows;
  int64_t param_dtype;
} ncf_table_pair;
/* The reduce with the deferred table Adam's apply of the step fused in (FusedTrainStep): each
 * unique row's two gradient rows, once complete (in the reduce for a segment of one piece, in
 * the fix-up for longer ones), step that row as ncf_adam_pairs_apply_clock(pairs, 2, dim,
 * num_unique, n, step_rel, ...) would, and stamp it; the compact gradients are still written.
 * pairs[k] (k = users, items): the two tables (p0 GMF, p1 MLP; the rows the reduce reads), their
 * moments and stamps.  Same bits as the reduce followed by the apply (trainer.py:285's
 * Adam.step on the touched rows, fused into the backward of :282). */
int ncf_embedding_bwd_reduce_apply_clock(
    int64_t n, int64_t dim, int64_t num_users, int64_t num_items, const float* dy_mf_user,
    const float* dy_mlp_user, const float* dy_mf_item, const float* dy_mlp_item,
    const float* mf_gamma, const float* mlp_gamma, float eps, float* grad_mf_user,
    float* grad_mlp_user, float* grad_mf_item, float* grad_mlp_item, const int64_t* uniq_users,
    const int64_t* uniq_items, float* grad_mf_gamma, float* grad_mf_beta, float* grad_mlp_gamma,
    float* grad_mlp_beta, void* workspace, int64_t workspace_bytes, ncf_reduce_list* defer,
    const ncf_table_pair* pairs, int32_t step_rel, const ncf_step_clock* clock,
    const float* step_table, double beta1, double beta2, double eps_adam, double weight_decay,
    void* stream);
int ncf_adam_pairs_catchup_clock(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                 const uint32_t* count, int64_t max_n, int32_t target_rel,
                                 const ncf_step_clock* clock, const float* step_table,
                                 double beta1, double beta2, double eps, double weight_decay,
                                 void* stream);
/* Stamps at or above NCF_STAMP_LOCK (0x40000000) compare above any target: the catch-up kernels
 * leave such rows alone.  ncf_adam_pairs_catchup_lock_clock with lock = 1 sets it on the listed
 * rows (caught up through the target, their gradient step of this step still to come; the
 * apply writes the plain stamp back); with lock = 0 and target_rel = 1 it is the early catch-up
 * of the NEXT batch's rows through the step now running, on a side stream beside its backward
 * (rows of this step's batch are locked and skipped).  The reference's Adam.step over every row
 * (src/model/trainer.py:285) gives the same values: the skipped step of an unlisted row is a
 * zero-gradient one. */
#define NCF_STAMP_LOCK 0x40000000
int ncf_adam_pairs_catchup_lock_clock(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                      const uint32_t* count, int64_t max_n, int32_t target_rel,
                                      int32_t lock, const ncf_step_clock* clock,
                                      const float* step_table, double beta1, double beta2,
                                      double eps, double weight_decay, void* stream);
/* The catch-up of the rows named by RAW id lists (ids0 for pairs[0], ids1 for pairs[1], n
 * occurrences each, duplicates allowed): the first occurrence of a row to raise its stamp to the
 * target (atomicMax) replays it, the others skip: the same rows, bit-identical, with no dedup
 * before the forward (the id sort can then run beside it on another stream).  Replaces the
 * dedup + ncf_adam_pairs_catchup_clock pair before the gathers of the reference call pattern
 * (src/model/trainer.py:258, the forward of a train step). */
int ncf_adam_pairs_catchup_claim_clock(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                       const int64_t* ids0, const int64_t* ids1, int64_t n,
                                       int32_t target_rel, const ncf_step_clock* clock,
                                       const float* step_table, double beta1, double beta2,
                                       double eps, double weight_decay, void* stream);
/* The owner side of the row-sharded step (distributed.py): ncf_shard_owner_gradsum (the W
 * requesters' gradient rows of each unique row, summed in rank order: got[pos[c][s]], -1 = not
 * sent) and ncf_adam_pairs_apply_clock in ONE launch, the same bits; pairs' g0 / g1 unused.
 * Replaces the sharded EBC's gradient exchange + Adam.step of torchrec's pipeline (the
 * reference's single-process trainer.py:285). */
int ncf_adam_pairs_apply_gsum_clock(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                    const uint32_t* count, int64_t max_n, int32_t step_rel,
                                    const float* got, const int32_t* pos0, const int32_t* pos1,
                                    int world, const ncf_step_clock* clock,
                                    const float* step_table, double beta1, double beta2,
                                    double eps, double weight_decay, void* stream);
int ncf_adam_pairs_apply_clock(const ncf_table_pair* pairs, int npairs, int64_t dim,
                               const uint32_t* count, int64_t max_n, int32_t step_rel,
                               const ncf_step_clock* clock, const float* step_table, double beta1,
                               double beta2, double eps, double weight_decay, void* stream);
int ncf_adam_pairs_sweep_rolling(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                 int32_t sweep_every, int32_t step_rel,
                                 const ncf_step_clock* clock, const float* step_table,
                                 double beta1, double beta2, double eps, double weight_decay,
                                 void* stream);
/* Part `part` of `nparts` (consecutive row ranges) of that slice: the parts of one step may run at
 * different points of it, on any stream, before the clock advances (the overlapped sweep). */
int ncf_adam_pairs_sweep_rolling_part(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                      int32_t sweep_every, int32_t step_rel, int32_t part,
                                      int32_t nparts, const ncf_step_clock* clock,
                                      const float* step_table, double beta1, double beta2,
                                      double eps, double weight_decay, void* stream);
/* bf16 parameter rows (C2 "bf16": tables bf16, Adam moments fp32): ncf_adam_table and
 * ncf_adam_sweep with the parameter rounded to bf16 after every step.                        */
int ncf_adam_table_bf16(uint16_t* param, float* exp_avg, float* exp_avg_sq, int64_t rows,
                        int64_t dim, const int32_t* slot, const float* grad_compact, double lr,
                        double beta1, double beta2, double eps, double weight_decay, double step,
                        void* stream);
int ncf_adam_sweep_bf16(uint16_t* p0, float* m0, float* v0, uint16_t* p1, float* m1, float* v1,
                        int64_t row0, int64_t rows, int64_t dim, int32_t* stamp, int32_t target,
                        const float* step_table, double beta1, double beta2, double eps,
                        double weight_decay, void* stream);
int ncf_adam_flat_clock(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        int64_t n, const float* step_table, int32_t step_rel,
                        const ncf_step_clock* clock, double beta1, double beta2, double eps,
                        double weight_decay, void* stream);
/* ncf_adam_flat_clock, then ncf_step_clock_advance(clock, base_seed), in one launch (the last
 * block to finish closes the step; clock->reserved is its block counter, 0 between launches). */
int ncf_adam_flat_clock_close(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              int64_t n, const float* step_table, int32_t step_rel,
                              ncf_step_clock* clock, double beta1, double beta2, double eps,
                              double weight_decay, uint64_t base_seed, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NCF_HIP_H */
