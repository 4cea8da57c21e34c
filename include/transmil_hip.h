/* C ABI of libtransmil_hip.so -- the MI355X (gfx950) TransMIL hot path.
 *
 * The reference has no native boundary: its plugin surface is Python
 * (`models.TransMIL` imported by ModelInterface.load_model,
 * code/models/model_interface.py:1256-1293, and the third-party
 * `nystrom_attention.NystromAttention`, code/models/TransMIL.py:5,26-34,47).
 * This ABI is what the drop-in Python module (transmil_deepgraft_amd/models/
 * TransMIL.py and transmil_deepgraft_amd/nystrom_attention.py) binds through
 * ctypes; each entry point below names the reference op it replaces.
 *
 * Conventions (all entry points):
 *   - device pointers are caller-owned; nothing is allocated inside;
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream);
 *   - no host synchronisation, so every call is hipGraph-capturable -- with ONE documented
 *     exception, tm_conv1x1_tune (a host-timed algorithm search, refused during capture);
 *   - deterministic: no float atomics, fixed reduction orders -- every result is a function of
 *     the inputs alone, with ONE documented exception: tm_conv1x1 after tm_conv1x1_tune runs the
 *     algorithm the tune call timed fastest IN THIS PROCESS, so two processes that tuned may
 *     round the C5 encoder features differently (the Python encoder skips the tune under
 *     torch.use_deterministic_algorithms(True) or TM_CONV1X1_TUNE=0: heuristic first choice);
 *   - return 0 on success, 1 on a bad argument, 2 on a launch error;
 *     tm_last_error() returns the thread-local message.
 *   - dtype enum: TM_F32 = 0, TM_BF16 = 1 (activations / MFMA operands).
 */
#ifndef TRANSMIL_HIP_H
#define TRANSMIL_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- errors / build info ---------------------------------------------- */
const char* tm_last_error(void);
const char* tm_build_info(void);

/* ---- dense GEMM with fused epilogues (gemm.hip) -----------------------
 * C[m,n] = epi(alpha * sum_k A(m,k) B(k,n)),
 *   A(m,k) = a_trans ? A[k*lda+m] : A[m*lda+k];  B(k,n) = b_kn ? B[k*ldb+n] : B[n*ldb+k].
 * Replaces the nn.Linear call sites of _fc1 (code/models/TransMIL.py:128-133),
 * NystromAttention.to_qkv / to_out (SURVEY.md App. A eq. 2, 10) and their
 * backward products. */
enum { TM_EPI_PLAIN = 0, TM_EPI_QKV = 1, TM_EPI_SPLITK = 2 };
typedef struct tm_gemm_args {
  int M, N, K;
  int lda, ldb, ldc;
  int a_trans, b_kn;
  int ab_dtype, c_dtype;
  int splits, k_per_split;
  int mode;            /* TM_EPI_* */
  float alpha;
  const float* bias;   /* [N] fp32 or NULL */
  int gelu;            /* exact erf GELU after bias */
  void* pre;           /* pre-activation store (c_dtype), row m, ld_pre; or NULL */
  int ld_pre;
  float drop_p, drop_scale;
  uint64_t seed;
  const float* resid;  /* fp32 residual added last, indexed like C; or NULL */
  int accumulate;      /* C += result */
  /* output row map (grp_in > 0): bag = m / grp_in, t = m % grp_in - skip;
   * t < 0 -> not stored; row = bag*grp_out + out_off + t; if t < dup_n also
   * stored at bag*grp_out + dup_off + t (TransMIL grid padding, :177-180) */
  int grp_in, skip, grp_out, out_off, dup_n, dup_off;
  /* TM_EPI_QKV: m = bag*seq + t, n = which*(nh*dh) + head*dh + d ->
   * C[((which*nbags + bag)*nh + head)*seq + t][d]; q (which==0) scaled by qscale */
  int nbags, nh, dh, seq;
  float qscale;
  /* dropout seed read from device memory when non-NULL: seed = *seed_ptr * 0x9E3779B97F4A7C15 + seed
   * (keeps a hipGraph replay drawing a fresh mask every step) */
  const uint64_t* seed_ptr;
  /* bf16 weight-gradient split-K (a_trans = 1, TM_EPI_SPLITK, K and k_per_split multiples of 64)
   * only, else NULL: colsum[z][m] = sum over split z's k of A[k][m] (the bias gradient of the same
   * dY, summed by the workgroups of the first column tile while they stage A) -- [splits][M] fp32 */
  float* colsum;
  /* 1: the pre-activation store (pre) is bf16 whatever c_dtype (the bf16 step's _fc1: the GELU
   * backward reads it back in bf16, tm_fc1_gelu_bwd with TM_BF16); 0: c_dtype */
  int pre_bf16;
  /* TM_EPI_SPLITK with bf16 operands: 1 = the split slabs are written bf16 (each split's partial
   * rounded once; tm_splitk_reduce_bf16 sums them in fp32); 0: fp32 slabs (c_dtype TM_F32) */
  int slab_bf16;
} tm_gemm_args;

int tm_gemm(const void* A, const void* B, void* C, const tm_gemm_args* args, void* stream);
/* Deferred parameter-gradient reductions.  A tm_reduce_queue is a caller-owned host object
 * (no device memory, no stream): every entry point below that ends in a split-K / slab sum takes
 * `tm_reduce_queue* rq`.  rq == NULL launches the sum now on `stream`; otherwise the (slab, out)
 * pair is only appended to *rq, and tm_reduce_flush(rq, stream) sums every queued pair in ONE
 * launch (same fixed split order, so bit-identical to the immediate form).  The library keeps no
 * deferral state of its own: two engines on two streams, or two threads, each pass their own
 * queue.  A queue must not be used by two threads at once; nothing may read a queued output (or
 * free its slab) before the flush.  A full queue (48 entries) is flushed on the appending call's
 * stream.  Replaces the DDP-reducer-era fixed-bucket gradient pass (code/train.py:184). */
typedef struct tm_reduce_queue tm_reduce_queue;
tm_reduce_queue* tm_reduce_queue_create(void);          /* NULL + tm_last_error() on failure */
void tm_reduce_queue_destroy(tm_reduce_queue* rq);      /* entries still queued are dropped */
int tm_reduce_queue_pending(const tm_reduce_queue* rq); /* queued entries, -1 if rq is invalid */
int tm_reduce_flush(tm_reduce_queue* rq, void* stream);
int tm_splitk_reduce(const float* slab, float* out, int splits, long long count, float alpha,
                     int accumulate, tm_reduce_queue* rq, void* stream);
/* the same over bf16 slabs (tm_gemm_args.slab_bf16): the splits summed in fp32 in index order */
int tm_splitk_reduce_bf16(const void* slab, float* out, int splits, long long count, float alpha,
                          int accumulate, tm_reduce_queue* rq, void* stream);
long long tm_colsum_workspace(int rows, int cols, int rows_per_chunk);
int tm_colsum(const void* X, int dtype, int rows, int cols, int ld, int rows_per_chunk,
              float* work, float* out, int accumulate, tm_reduce_queue* rq, void* stream);

/* ---- LayerNorm / head (layernorm.hip) ----------------------------------
 * TransLayer.norm (code/models/TransMIL.py:23,47) and the final norm + _fc
 * head (:154-155, 202-204).  x rows are [B*S, D] fp32; y is written into the
 * front-padded [B, n_pad, D] layout (rows b*n_pad + pad + i; pad rows zeroed). */
int tm_layernorm_fwd(const float* x, const float* gamma, const float* beta, float eps, int rows, int D,
                     int S, int n_pad, int pad, int dtype, void* y, float* mean, float* rstd, void* stream);
long long tm_layernorm_bwd_workspace(int rows, int D, int rows_per_block);
/* dx_accum[r] += LN'(dy) (dy read from the padded layout); dgamma/dbeta written */
/* resid_cls_only != 0: dx_accum holds the residual gradient only at the class rows (row % S == 0);
 * the other rows are written (=) without being read (the last layer's dL/dH, clsrow.hip) */
int tm_layernorm_bwd(const void* dy, int dtype, const float* x, const float* gamma, const float* mean,
                     const float* rstd, int rows, int D, int S, int n_pad, int pad, int rows_per_block,
                     int resid_cls_only, float* dx_accum, float* work, float* dgamma, float* dbeta,
                     tm_reduce_queue* rq, void* stream);
/* tm_layernorm_bwd with a per-segment addend on dy: row t of bag b reads dy + seg_add[b][(pad + t) /
 * seg_len] (+ seg_add[b][nseg] at t = 0, the class row); seg_add is [B][seg_rows][D] fp32 (the
 * scale * Aq Wq rows of tm_cls_q_rows' products, seg_rows = 288, nseg = 256) */
int tm_layernorm_bwd_seg(const void* dy, int dtype, const float* x, const float* gamma, const float* mean,
                         const float* rstd, int rows, int D, int S, int n_pad, int pad, int rows_per_block,
                         int resid_cls_only, const float* seg_add, int seg_len, int nseg, int seg_rows,
                         float* dx_accum, float* work, float* dgamma, float* dbeta, tm_reduce_queue* rq,
                         void* stream);
int tm_head_fwd(const float* h, int B, int S, int D, const float* gamma, const float* beta, float eps,
                const float* W, const float* bias, int C, float* logits, float* xhat, float* rstd,
                void* stream);
/* writes dh[b*S*D + :D] (row 0 of each bag); other rows untouched */
int tm_head_bwd(const float* dlogits, int B, int C, int S, int D, const float* xhat, const float* rstd,
                const float* gamma, const float* beta, const float* W, float* dW, float* dbias,
                float* dgamma, float* dbeta, float* dh, void* stream);
/* The training step's head and loss in one launch each way (replaces tm_head_fwd + tm_ce_fwd and
 * tm_ce_bwd + tm_head_bwd on the fused TransMILTask path): forward = tm_head_fwd, then
 * CrossEntropyLoss(logits, one_hot(label).float()) / Y_prob / Y_hat / class stats as tm_ce_fwd
 * (code/models/model_interface.py:339-356); backward: dlogits = gloss (prob - one_hot) / B
 * (+ dlogits_in, nullable), then tm_head_bwd.  scratch: B*C floats (may be null if B == 1, C <= 4). */
int tm_head_ce_fwd(const float* h, int B, int S, int D, const float* gamma, const float* beta, float eps,
                   const float* W, const float* bias, int C, const long long* label, float* logits, float* xhat,
                   float* rstd, float* loss, float* prob, long long* yhat, int* class_stats, void* stream);
int tm_head_ce_bwd(const float* prob, const long long* label, const float* gloss, const float* dlogits_in, int B,
                   int C, int S, int D, const float* xhat, const float* rstd, const float* gamma,
                   const float* beta, const float* W, float* dW, float* dbias, float* dgamma, float* dbeta,
                   float* dh, float* scratch, void* stream);

/* ---- NystromAttention core (nystrom.hip) --------------------------------
 * SURVEY.md App. A eq. 4-9 of the third-party nystrom_attention package
 * (call site code/models/TransMIL.py:47).  dim_head = 64, 256 landmarks.
 * q/k/v: [B*h, n, 64] (T), n a multiple of 256; landmarks [B*h, 256, 64]. */
int tm_nys_landmarks(int dtype, const void* q, const void* k, int nbh, int n, float* ql, float* kl,
                     void* ql_t, void* kl_t, void* stream);
int tm_nys_sim2_softmax(const float* ql, const float* kl, int nbh, float* a2, void* stream);
int tm_softmax_bwd_rows256(const float* a, const float* da, float* ds, int rows, void* stream);
long long tm_nys_a3_workspace(int nbh, int n);
/* W = softmax(ql k^T) v  [B*h,256,64] fp32, lse3 [B*h,256] */
/* bf16: w = lse3 = NULL leaves the tm_nys_a3_partials(nbh, n) key-split partials in work for
 * tm_pinv_fwd_split_a3 to combine */
long long tm_nys_a3_partials(int nbh, int n);
int tm_nys_a3_fwd(int dtype, const float* ql, const void* k, const void* v, int nbh, int n, float* work,
                  float* w, float* lse3, void* stream);
/* bf16 only: tm_nys_a3_fwd(TM_BF16, ..., w = NULL, lse3 = NULL) and tm_nys_sim2_softmax_split(ql, kl,
 * nbh, a2, a2s) in ONE launch (the A3 workgroups also write the A2 rows, bit-identical to the
 * separate kernel; two launches where the key split does not tile the 256 rows).  Both replace
 * NystromAttention.forward's attn2 / attn3 softmaxes (code/models/TransMIL.py:47; App. A eq. 5-6). */
int tm_nys_a3_fwd_sim2(const float* ql, const float* kl, const void* k, const void* v, int nbh, int n,
                       float* work, float* a2, void* a2s, void* stream);
/* merged[b][t][head*64+d] = softmax(q kl^T) y + conv33(v); lse1 [B*h, n]; kl_t, y_t: T copies */
int tm_nys_a1_fwd(int dtype, const void* q, const void* v, const void* kl_t, const void* y_t,
                  const float* wconv, int nbh, int nh, int n, void* merged, float* lse1, void* stream);
int tm_nys_rowdot_cast(int dtype, const float* dw, const float* w, int rows, float* dd, void* dw_t, void* stream);
int tm_cast_f32(int dtype, const float* x, void* y, long long count, void* stream);
long long tm_nys_conv_bwd_workspace(int nbags, int nh, int n);
/* dv [B*h, n, 64] in the step's dtype T (bf16 in the bf16 mode: the fused A3 backward reads it once) */
int tm_nys_conv_bwd(int dtype, const void* dmerged, const void* merged, const void* v, const float* wconv,
                    int nbh, int nh, int n, void* dv, float* d1, float* work, float* dwconv,
                    tm_reduce_queue* rq, void* stream);
long long tm_nys_a1_bwd_workspace(int nbh, int n, int queries_per_wg);
int tm_nys_a1_bwd(int dtype, const void* q, const void* dmerged, const void* kl_t, const void* y_t,
                  const float* lse1, const float* d1, int nbh, int nh, int n, int queries_per_wg,
                  float* dq, float* work, float* dkl, float* dy, int accumulate, tm_reduce_queue* rq,
                  void* stream);
/* bf16 only: tm_nys_a1_bwd with dq written as bf16(dq_scale * dq) into the q part of dqkv
 * ([B][n][3*nh*64], bf16, the columns of each head) instead of fp32 [B*h][n][64] rows (half the
 * bytes, no fp32 round trip); tm_nys_assemble_q_slab_inplace then adds the landmark term there. */
int tm_nys_a1_bwd_dqkv(const void* q, const void* dmerged, const void* kl_t, const void* y_t, const float* lse1,
                       const float* d1, int nbh, int nh, int n, void* dqkv, float dq_scale, float* work, float* dkl,
                       float* dy, tm_reduce_queue* rq, void* stream);
long long tm_nys_a3_bwd_workspace(int nbh, int n);
/* d3 (here and in tm_nys_a3_bwd_fused): D = rowsum(dW o W) as [2][B*h][256] partials, the two
 * 32-column halves of dW (tm_bmm_job.Rd of the dW = Z^T dY product); the kernels sum them */
int tm_nys_a3_bwd(int dtype, const void* ql_t, const void* dw_t, const void* k, const void* v,
                  const float* lse3, const float* d3, int nbh, int nh, int n, float* dk, float* dv,
                  float* work, float* dql, int accumulate, tm_reduce_queue* rq, void* stream);
/* Row `row` of the return_attn product attn1 Z attn3 (App. A eq. 11; read by
 * code/visualize_mil.py:580-581 as cls_attention[0,:,padding+1,...]) for every bag and
 * head, without the [n, n] matrix: out [B*h, n] fp32 from the forward's q, k (T, q
 * pre-scaled), ql / kl [B*h,256,64], Z [B*h,256,256] and lse3 [B*h,256] (fp32). */
int tm_nys_attn_row(int dtype, const void* q, const void* k, const float* ql, const float* kl, const float* z,
                    const float* lse3, int nbh, int n, int row, float* out, void* stream);
int tm_nys_assemble_dqkv(int dtype, const float* dq, const float* dql, const float* dk, const float* dkl,
                         const float* dv, int nbags, int nh, int n, float scale, void* dqkv, void* stream);
/* bf16 mode, fused key side: the A3 backward writes the final bf16 k / v parts of dqkv
 * (k = dK + dk~[t/l]/l, v = dv_conv + dV) and dql (=) from its slabs; then tm_nys_assemble_q
 * writes the q part, scale * (dq + (dql_a + dql_b)[t/l]/l).  dv_conv (bf16, as tm_nys_conv_bwd /
 * tm_cls_a1_row_bwd write it in the bf16 mode) is read only for rows
 * [dv_lo, dv_hi) (zero elsewhere; 0, n = dense); dq_row >= 0: dq is zero outside that row.
 * dql = NULL: the dq~ partial slab is left in work ([tm_nys_a3_bwd_slabs][B*h][256][64] bf16, each
 * partial rounded once; the consumers sum them in fp32) for tm_nys_assemble_q_slab, which reduces it
 * while writing the q part (one launch fewer). */
int tm_nys_a3_bwd_fused(const void* ql_t, const void* dw_t, const void* k, const void* v, const float* lse3,
                        const float* d3, int nbh, int nh, int n, const void* dv_conv, int dv_lo, int dv_hi,
                        const float* dkl, float* work, float* dql, void* dqkv, tm_reduce_queue* rq,
                        void* stream);
int tm_nys_assemble_q(int dtype, const float* dq, int dq_row, const float* dql_a, const float* dql_b, int nbags,
                      int nh, int n, float scale, void* dqkv, void* stream);
/* partial slabs the bf16 A3 backward writes (tm_nys_a3_bwd_fused's work) */
int tm_nys_a3_bwd_slabs(int nbh, int n);
/* q part of dqkv, scale * (dq + (dql + sum_p slab[p])[t/l]/l), the slab sum in the same launch
 * (nh <= 8; slab [slabs][nbags*nh][256][64] bf16 as tm_nys_a3_bwd_fused(dql = NULL) leaves it) */
int tm_nys_assemble_q_slab(int dtype, const float* dq, int dq_row, const float* dql, const void* slab, int slabs,
                           int nbags, int nh, int n, float scale, void* dqkv, void* stream);
/* bf16, after tm_nys_a1_bwd_dqkv: q += scale * (dql + sum_p slab[p])[t/l]/l in place in dqkv */
int tm_nys_assemble_q_slab_inplace(const float* dql, const void* slab, int slabs, int nbags, int nh, int n,
                                   float scale, void* dqkv, void* stream);

/* ---- pseudo-inverse + small fp32 batched products (pinv.hip) -------------
 * moore_penrose_iter_pinv of nystrom_attention (App. A eq. 7).
 * C = diag*I + alpha*(op(A) op(B) [+ op(A2) op(B2)]) + e1*E1 + e2*E2, batched;
 * op(X) = X^T when the t-flag is set; E1/E2 share C's layout. */
typedef struct tm_bmm_job {
  const float* A; const float* B; int ta, tb; int lda, ldb; long long sa, sb;
  const float* A2; const float* B2; int ta2, tb2; int lda2, ldb2; long long sa2, sb2;
  const float* E1; float e1; const float* E2; float e2;
  float alpha, diag;
  float* C; int ldc; long long sc;
  int M, N, K;
  /* optional second output of the same product (C's layout): C2 = c2_alpha*(products)
   * + c2_diag*I + c2_e1*E1 (null: none) */
  float* C2; float c2_alpha, c2_diag, c2_e1;
  /* optional bf16 form of C (C's layout, written beside it): ct_mode 1 = bf16(C) at Ct,
   * 2 = split planes hi = bf16(C) at Ct and lo = bf16(C - hi) at Ct + ct_plane elements
   * (the operand format of tm_pinv_bwd_split), 0 = none */
  void* Ct; long long ct_plane; int ct_mode; int ct_reserved;
  /* optional partial row dots of C with Rw (C's layout), one per 32-column tile:
   * Rd[(n / 32) * nbatch + b][m] = sum over that tile's columns of C[b][m][n] * Rw[b][m][n]
   * (null: none).  D = rowsum(dW o W) of the A3 backward as N / 32 = 2 partials. */
  float* Rd; const float* Rw;
} tm_bmm_job;
/* prec 0: exact fp32 MFMA; prec 1: bf16x3 (hi/lo split, ~16-bit operands, fp32 accumulate) */
int tm_bmm(const tm_bmm_job* jobs, int njobs, int nbatch, int prec, void* stream);
long long tm_pinv_saved_floats(int nbh, int iters);
int tm_pinv_fwd(const float* X, int nbh, int iters, int prec, float* saved, void* stream);
long long tm_pinv_bwd_workspace_floats(int nbh);
int tm_pinv_bwd(const float* X, int nbh, int iters, int prec, const float* saved, float* dZ, float* work,
                float* dX, void* stream);

/* ---- pseudo-inverse on split operands, bf16 (bench) mode (pinv_split.hip) --
 * Same function as tm_pinv_fwd / tm_pinv_bwd with prec 1, restructured for MI355X: every chain
 * matrix is kept as bf16 hi / lo planes (hi = bf16(M), lo = bf16(M - hi); the lo plane follows the
 * hi plane at + nbh*256*256 elements), products are hi*hi + hi*lo + lo*hi on the bf16 MFMA with
 * fp32 accumulation, 64x64 output tiles fed by LDS-DMA; 14 launches forward.
 * A2 = softmax(ql kl^T) with its split planes (replaces tm_nys_sim2_softmax on this path): */
int tm_nys_sim2_softmax_split(const float* ql, const float* kl, int nbh, float* a2, void* a2s, void* stream);
/* saved: Z_iters fp32 at saved[0 .. nbh*65536), then the split chain matrices, sums and maxima */
long long tm_pinv_split_saved_floats(int nbh, int iters);
int tm_pinv_fwd_split(const float* X, const void* Xs, int nbh, int iters, float* saved, void* stream);
/* tm_pinv_fwd_split with the A3 forward's partial combine in the chain's last launch (its idle CUs):
 * a3_work / a3_parts = the partials tm_nys_a3_fwd(TM_BF16, ..., w = NULL, lse3 = NULL) left,
 * a3_parts = tm_nys_a3_partials(nbh, n); writes W [B*h,256,64] and lse3 [B*h,256] as tm_nys_a3_fwd. */
int tm_pinv_fwd_split_a3(const float* X, const void* Xs, int nbh, int iters, float* saved, const float* a3_work,
                         int a3_parts, float* w, float* lse3, void* stream);
/* work: the gradient w.r.t. Z_iters as split planes at work[0 .. nbh*65536) on entry (tm_split_f32);
 * out = dL/dX (softmax == 0) or the backward of A2 = softmax(.) through X (softmax != 0), fp32 */
long long tm_pinv_bwd_split_workspace_floats(int nbh);
int tm_pinv_bwd_split(const float* X, const void* Xs, int nbh, int iters, const float* saved, float* work,
                      int softmax, float* out, void* stream);
/* fp32 -> split planes: y[i] = bf16(x[i]), y[count + i] = bf16(x[i] - y[i]); count % 8 == 0 */
int tm_split_f32(const float* x, void* y, long long count, void* stream);

/* ---- PPEG (ppeg.hip) -- code/models/TransMIL.py:60-75 -------------------- *
 * wfold [49][D] tap-major (the three depthwise kernels + identity folded into one 7x7), bfold [D] */
int tm_ppeg_fold(const float* w7, const float* b7, const float* w5, const float* b5, const float* w3,
                 const float* b3, int D, float* wfold, float* bfold, void* stream);
int tm_ppeg_fwd(const float* x, int B, int G, int D, const float* wfold, const float* bfold, float* y,
                void* stream);
long long tm_ppeg_bwd_workspace(int B, int G, int D);
/* dout (nullable): also writes the padded to_out-dropout gradient of the TransLayer below from dx
 * (as tm_dropout_bwd_pad with the same dtype / n_pad / pad / p / seed / seed_ptr).  The weight
 * gradients (=) are summed from the workspace's slabs by tm_splitk_reduce: deferred into rq when
 * it is non-null (final after tm_reduce_flush), else summed before return */
int tm_ppeg_bwd(const float* x, const float* dy, int B, int G, int D, const float* wfold, float* dx,
                float* work, float* dw7, float* db7, float* dw5, float* db5, float* dw3, float* db3,
                int dtype, void* dout, int n_pad, int pad, float p, uint64_t seed,
                const uint64_t* seed_ptr, tm_reduce_queue* rq, void* stream);

/* ---- AttMIL gated attention pooling (attmil.hip) -- code/models/AttMIL.py:88-110 ----
 * Z [N, 2D] = H [Wv;Wu]^T + [bv;bu] (caller's GEMM), H [N, L], w [D] / b [1] = attention_weights,
 * Wc [C, L] / bc [C] = classifier.  Forward writes a [N] scores, p [N] softmax weights, M [L] pooled
 * bag and logits [C]; backward writes dZ [N, 2D], dH [N, L] = p dM (the caller's GEMM then adds
 * dZ [Wv;Wu]), dM [L], dw [D], db [1], dWc [C, L], dbc [C].  fp32; work sized by the queries. */
long long tm_attmil_fwd_workspace(int N, int L);
int tm_attmil_fwd(const float* Z, const float* H, const float* w, const float* b, const float* Wc,
                  const float* bc, int N, int L, int D, int C, float* work, float* a, float* p, float* M,
                  float* logits, void* stream);
long long tm_attmil_bwd_workspace(int N, int L, int D);
int tm_attmil_bwd(const float* Z, const float* H, const float* w, const float* p, const float* M,
                  const float* Wc, const float* dlogits, int N, int L, int D, int C, float* work,
                  float* dZ, float* dH, float* dM, float* dw, float* db, float* dWc, float* dbc, void* stream);

/* ---- feature-bag sampling (bags.hip) -- code/datasets/feature_dataloader.py:335-431 ----
 * dst[r] = src[i0[r]] (i1 NULL or i1[r] < 0), (src[i0[r]] * wa[r]) + (src[i1[r]] * wb[r]) (mixup),
 * or 0 (i0[r] < 0); src [*, F] and dst [nrows, F] of dtype TM_F32 / TM_BF16, i0/i1 int64 row
 * ids into src (device), nrows <= 65535.  Replaces the per-item indexing of
 * FeatureBagLoader.__getitem__ (:346-362) and data_interface.simple_collate's stack (:238-246). */
int tm_gather_rows(int dtype, const void* src, int F, const long long* i0, const long long* i1,
                   const float* wa, const float* wb, int nrows, void* dst, void* stream);

/* ---- glue (glue.hip) -- code/models/TransMIL.py:177-186 ------------------ */
int tm_put_cls(const float* cls, int B, int S, int D, float* H, void* stream);
/* CrossEntropyLoss(logits, one_hot(label).float()) mean over B rows + softmax + argmax in one
 * launch (code/models/model_interface.py:339-347); backward dlogits = g[0] (prob - one_hot) / B.
 * label int64 [B] on the device, values in [0, C); an out-of-range label makes the loss NaN and is
 * left out of class_stats (no out-of-bounds access).  class_stats
 * (nullable, int32 [C][2]) accumulates per-class count / correct (:350-356). */
int tm_ce_fwd(const float* logits, const long long* label, int B, int C, float* loss, float* prob,
              long long* yhat, int* class_stats, void* stream);
int tm_ce_bwd(const float* prob, const long long* label, int B, int C, const float* g, float* dlogits,
              void* stream);
int tm_dropout_bwd_pad(int dtype, const float* dH, int B, int S, int n_pad, int pad, int D, float p,
                       uint64_t seed, const uint64_t* seed_ptr, void* out, void* stream);
/* NystromAttention eq. 1 for a raw input: [B*S, D] fp32 -> front-padded [B, n_pad, D] T */
int tm_pad_rows(int dtype, const float* x, int B, int S, int n_pad, int pad, int D, void* y, void* stream);
/* _fc1 GELU backward + grid-pad fold: dpre (dtype T) = (dH[token] + dH[dup]) * GELU'(pre); `pre` is the
 * forward's pre-activation in the same T (fp32 for TM_F32, bf16 for TM_BF16: tm_gemm_args.pre_bf16) */
int tm_fc1_gelu_bwd(int dtype, const float* dH, const void* pre, int B, int N, int S, int add, int D,
                    void* dpre, float* dcls, void* stream);
/* dpre = dy * GELU'(pre) elementwise (fp32 dy / pre, dpre in dtype): the backward of the inner
 * Linear + GELU of the in_features = 2048 _fc1 branch (code/models/TransMIL.py:100-111) */
int tm_gelu_bwd(int dtype, const float* dy, const float* pre, long long count, void* dpre, void* stream);
/* y = max(a + b, 0) elementwise (the C5 encoder's residual add + ReLU, Bottleneck.forward,
 * code/models/ResNet.py:97-124); 16-B aligned, y may alias a */
int tm_add_relu(int dtype, const void* a, const void* b, void* y, long long count, void* stream);
/* y[r, c] = act(y[r, c] + bias[c]) in place over rows x C channels-last (C % 8 == 0; act = ReLU
 * when relu != 0): a 3x3 convolution's folded conv+BN bias + ReLU (ResNet.py:95-104) in one pass */
int tm_bias_act(int dtype, void* y, const void* bias, long long rows, int C, int relu, void* stream);
/* ResNet stem tail (ResNet.py:240-245, BN folded into the convolution's bias): out[N, OH, OW, C] =
 * maxpool3x3/2 pad 1 (relu(y + bias)) over the raw channels-last bf16 stem output y[N, H, W, C],
 * OH = (H - 1) / 2 + 1; one pass instead of the in-place bias + ReLU and a max-pool launch */
int tm_bias_relu_maxpool(const void* y, const void* bias, void* out, int N, int H, int W, int C, void* stream);
/* the same with train-mode BatchNorm: each tap bf16(relu(y * scale + shift)) (tm_bn_apply's
 * arithmetic, scale / shift fp32 [C] from tm_bn_train_stats), then the window max */
int tm_bn_relu_maxpool(const void* y, const float* scale, const float* shift, void* out, int N, int H, int W, int C,
                       void* stream);
/* The whole eval-mode stem in one pass (code/models/ResNet.py:240-245, BN folded): out[N, PH, PW, 64]
 * = maxpool3x3/2 pad 1(relu(conv7x7/2 pad 3(x, w) + bias)), x bf16 [N, 3, H, W] at element strides
 * (sn, sc, sh, sw) (NCHW or channels-last),
 * wp the folded weights packed bf16 [64][7][8][4] (w[o, c, ky, kx] at [o][ky][kx][c]; kx = 7 and
 * c = 3 zero), bias bf16 [64]; CH = (H - 1) / 2 + 1, PH = (CH - 1) / 2 + 1 (same for W).  fp32
 * accumulation, one bf16 rounding after the ReLU; the convolution output never reaches HBM. */
int tm_stem_conv_pool(const void* x, const void* wp, const void* bias, void* out, int N, int H, int W, long long sn,
                      long long sc, long long sh, long long sw, void* stream);
/* The train-mode stem (batch-statistics bn1, code/models/model_interface.py:303-309 feeding the
 * frozen encoder in train mode) in two passes over the tiles, the convolution recomputed instead of
 * stored: tm_stem_bn_stats runs the convolution and reduces its bf16-rounded outputs per channel
 * (per-workgroup count / mean / M2, merged in workgroup order in fp64: deterministic), then writes
 * scale = gamma / sqrt(var + eps), shift = beta - mean * scale (biased variance) and updates the
 * running statistics with the unbiased variance and the momentum (nn.BatchNorm2d);
 * workspace >= tm_stem_bn_stats_workspace() doubles.  tm_stem_conv_pool_bn then writes
 * maxpool(bf16(relu(bf16(conv) * scale + shift))) (tm_bn_apply's arithmetic).  N may be the whole
 * bag: tiles are addressed with 64-bit bases. */
long long tm_stem_bn_stats_workspace(void);
int tm_stem_bn_stats(const void* x, const void* wp, int N, int H, int W, long long sn, long long sc, long long sh,
                     long long sw, const float* gamma, const float* beta, float* running_mean, float* running_var,
                     float momentum, float eps, float* scale, float* shift, double* workspace, long long ws_doubles,
                     void* stream);
int tm_stem_conv_pool_bn(const void* x, const void* wp, const float* scale, const float* shift, void* out, int N,
                         int H, int W, long long sn, long long sc, long long sh, long long sw, void* stream);
/* out[n, i, j, :] = x[n, s*i, s*j, :] for channels-last x [N, H, W, C] (bf16 / fp32, C * elem % 16
 * == 0): the input of a stride-s 1x1 downsample convolution (code/models/ResNet.py:130-135). */
int tm_subsample2d(int dtype, const void* x, void* out, int N, int H, int W, int C, int stride, void* stream);
/* C5 encoder 1x1 convolution over channels-last rows (code/models/ResNet.py:95-117 conv1 / conv3
 * / downsample with BN folded): y[rows, cout] = act(x[rows, cin] . w[cout, cin]^T (+ bias[cout])
 * (+ residual[rows, cout])), one hipBLASLt GEMM with the bias / residual / ReLU epilogue.
 * bias / residual may be NULL; residual must not alias y.  workspace: caller-owned device scratch
 * of ws_bytes, stream-ordered on `stream` (NULL / 0: workspace-free algorithms only; up to
 * tm_conv1x1_workspace_bytes() is used).  Library state: a per-device hipBLASLt handle and a
 * per-shape plan cache (host objects behind a mutex, immutable once built -- no device scratch is
 * shared between calls).  No host synchronisation.  Returns 3 on a hipBLASLt error. */
long long tm_conv1x1_workspace_bytes(void);
int tm_conv1x1(int dtype, const void* x, const void* w, const void* bias, const void* residual, void* y,
               long long rows, int cin, int cout, int relu, void* workspace, long long ws_bytes, void* stream);
/* THE EXCEPTION to "no host synchronisation": times every hipBLASLt heuristic candidate for this
 * shape on the given operands (y is overwritten) and waits on timing events, then keeps the fastest
 * for later tm_conv1x1 calls of the shape (the hipBLASLt analogue of MIOpen find).  Call once per
 * shape, outside stream capture (refused with status 1 while `stream` is capturing); without it
 * tm_conv1x1 uses the heuristic's first choice. */
int tm_conv1x1_tune(int dtype, const void* x, const void* w, const void* bias, const void* residual, void* y,
                    long long rows, int cin, int cout, int relu, void* workspace, long long ws_bytes,
                    void* stream);
/* Train-mode BatchNorm2d over a channels-last activation given as npieces (1..64) row pieces
 * xs[p] of [rows[p], C] (host arrays; C a power of two, 8..2048; nn.BatchNorm2d.forward in
 * training, code/models/ResNet.py:95-117 under model.train()): batch statistics over all pieces
 * (biased variance for the normalisation) -> scale = gamma / sqrt(var + eps), shift = beta -
 * mean * scale (fp32 [C]); running_mean / running_var (may be NULL) updated with the unbiased
 * variance and momentum.  workspace >= tm_bn_train_workspace(C) floats. */
long long tm_bn_train_workspace(int C);
int tm_bn_train_stats(int dtype, const void* const* xs, const long long* rows, int npieces, int C,
                      const float* gamma, const float* beta, float* running_mean, float* running_var,
                      float momentum, float eps, float* scale, float* shift, float* workspace, long long ws_floats,
                      void* stream);
/* y = act(y * scale[c] + shift[c] (+ residual | + residual * rscale[c] + rshift[c])) in place over
 * rows x C channels-last (C % 8 == 0): BN apply + ReLU, or bn3 + (BN'd) identity + ReLU, one pass */
int tm_bn_apply(int dtype, void* y, const float* scale, const float* shift, const void* residual,
                const float* rscale, const float* rshift, long long rows, int C, int relu, void* stream);

/* ---- class-row specialisation of the last TransLayer (clsrow.hip) -- code/models/TransMIL.py:195-203 ----
 * The logits read layer 2 only through the class token (norm(h)[:, 0]), which sits at row r = pad of
 * the front-padded attention input.  Forward: merged[b][r] = A1 row + conv33 (lse1[bh][r] written),
 * then H3[b*S] = H2[b*S] + dropout(merged[b][r] Wo^T + bo) (other H3 rows are not written).
 * Backward (dL/dH3 zero outside the class rows): dWo, dbo (=), dmerged [B][D] (dtype) rows; then
 * dq row r (the caller zero-fills dq), dk~ / dY (=) [nbh][256][64], the conv33 dv window rows
 * r-16..r+16 (caller zero-fills dv) and dwconv (=) [nh][33]. */
int tm_cls_a1_row_fwd(int dtype, const void* q, const void* v, const void* kl_t, const void* y_t, const float* wconv,
                      int nbh, int nh, int n, int r, void* merged, float* lse1, void* stream);
int tm_cls_out_fwd(int dtype, const void* merged, const void* wo, const float* bo, const float* H2, int B, int n, int r,
                   int S, int D, float p, uint64_t seed, const uint64_t* seed_ptr, float* H3, void* stream);
int tm_cls_out_bwd(int dtype, const float* dH, const void* merged, const void* wo, int B, int n, int r, int S, int D,
                   float p, uint64_t seed, const uint64_t* seed_ptr, float* dwo, float* dbo, void* dmerged,
                   void* stream);
/* tm_head_ce_bwd's one-bag fast path (B = 1, C <= 4, D = 512, no extra logits gradient) folded
 * into tm_cls_out_bwd: every block recomputes dL/dH3 at the class row from the saved softmax, x^
 * and rstd; dH's class row and the head / norm gradients are written as tm_head_ce_bwd writes
 * them.  One launch instead of two on the training step's tail (code/models/TransMIL.py:202-204,
 * model_interface.py:346-347 backward). */
int tm_cls_head_out_bwd(int dtype, const float* prob, const long long* label, const float* gloss, int C,
                        const float* xhat, const float* rstd, const float* gamma, const float* beta, const float* W,
                        float* dW, float* dbias, float* dgamma, float* dbeta, float* dH, const void* merged,
                        const void* wo, int n, int r, int S, int D, float p, uint64_t seed, const uint64_t* seed_ptr,
                        float* dwo, float* dbo, void* dmerged, void* stream);
int tm_cls_a1_row_bwd(int dtype, const void* dmerged, const void* q, const void* v, const void* kl_t, const void* y_t,
                      const float* lse1, const float* wconv, int B, int nh, int n, int r, float* dq, float* dkl,
                      float* dy, void* dv, float* dwconv, void* stream);   /* dv: the 33-row window, in T */
/* bf16 mode: layer 2's q enters the loss only through its landmark means q~ (App. A eq. 4) and the
 * class row r, so dL/dq = dq~[t / l] / l on every row t plus the class row's own term, and the q
 * part of to_qkv's backward is two small products instead of a dense q block in dqkv:
 *   dWq = scale * Aq^T Xs,   dxn[t] += scale * (Aq Wq)[t / l] (+ row NL at t = r)
 * (tm_bmm, then tm_layernorm_bwd_seg).  This writes their operands, [B][288][nh*64] fp32 each:
 *   Aq rows j < 256: (dql + sum_p slab[p])[b*nh + h][j][d] / l at column h*64 + d (slab: the
 *   nslabs [B*nh][256][64] partials tm_nys_a3_bwd_fused leaves in its work), row 256: dq[b*nh+h][r][d];
 *   Xs rows j < 256: sum over the segment's rows of xn[b] (bf16 [B][n][nh*64], pad rows zero),
 *   row 256: xn[b][r]; rows 257..287 of both: zeros (operand rows to a multiple of 32). */
int tm_cls_q_rows(const float* dql, const void* slab, int nslabs, const float* dq, const void* xn, int B, int nh,
                  int n, int r, float* Aq, float* Xs, void* stream);

/* fp32 -> dtype copies of up to 8 tensors (per-step bf16 GEMM weight operands) in one launch;
 * offset[] = prefix sums of the element counts, offset[0] = 0 */
#define TM_CAST_MAX 8
typedef struct tm_cast_table {
  int count;
  int reserved;
  const float* src[TM_CAST_MAX];
  void* dst[TM_CAST_MAX];
  long long offset[TM_CAST_MAX + 1];
} tm_cast_table;
int tm_cast_f32_many(int dtype, const tm_cast_table* table, void* stream);
/* One launch per forward: the cast table (as tm_cast_f32_many, 0..8 tensors), the PPEG fold
 * (as tm_ppeg_fold; skipped when w7 is NULL), when counter is non-NULL counter[0] += 1 with the
 * new value written to seed_out[0] (the dropout stream of a captured step), and when cls is
 * non-NULL the class-token rows H[b*S][0..D) = cls (as tm_put_cls). */
int tm_step_prepare(int dtype, const tm_cast_table* table, const float* w7, const float* b7,
                    const float* w5, const float* b5, const float* w3, const float* b3, int D,
                    float* wfold, float* bfold, long long* counter, long long* seed_out,
                    const float* cls, float* H, int B, int S, void* stream);

/* ---- optimizer step (optim.hip) ----------------------------------------
 * torch.optim.RAdam (L2 decay, code/MyOptimizer/optim_factory.py:77-79) + the
 * Lookahead sync (code/MyOptimizer/lookahead.py, wrapped at optim_factory.py:118-121)
 * over up to 40 parameter tensors in one launch.  exp_avg / exp_avg_sq / slow are
 * flat 16-B aligned fp32 buffers indexed by the table's offsets (prefix sums of numel, each
 * rounded up to a multiple of 4); counters (int32[tm_radam_counters_len(total)], device,
 * zero-initialised; total = the table's last offset) hold one (RAdam step, Lookahead step) pair per
 * workgroup of the launch, each advanced by its workgroup in the same launch (no tick launch);
 * the pairs stay equal as long as the table's total is fixed, and pair 0 is the one to checkpoint.
 * lookahead_k == 0 disables the sync (plain RAdam). */
#define TM_OPTIM_MAX_TENSORS 40
typedef struct tm_optim_tensor {
  float* param;
  const float* grad;
  long long numel;
  float lr;
  float weight_decay;
} tm_optim_tensor;
typedef struct tm_optim_table {
  int count;
  int reserved;
  long long offset[TM_OPTIM_MAX_TENSORS + 1];
  tm_optim_tensor t[TM_OPTIM_MAX_TENSORS];
  /* device [count][2] fp32 (lr, weight_decay) read by the kernel in place of t[i].lr /
   * t[i].weight_decay, or NULL.  A captured hipGraph replays the kernel arguments it was captured
   * with; reading the hyper-parameters from device memory lets an LR scheduler (ReduceLROnPlateau,
   * model_interface.py:862-877) act on a replayed step (the caller rewrites the buffer). */
  const float* hyper;
} tm_optim_table;
long long tm_radam_counters_len(long long total_elements);
int tm_radam_lookahead_step(const tm_optim_table* table, float* exp_avg, float* exp_avg_sq, float* slow,
                            int* counters, float beta1, float beta2, float eps, int lookahead_k,
                            float lookahead_alpha, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TRANSMIL_HIP_H */
