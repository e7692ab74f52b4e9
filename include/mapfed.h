/*
 * mapfed.h — C ABI of the MI355X-native federated MaPLe hot path (libmapfed.so, gfx950).
 *
 * The reference (tahaspc82442/federated_multi_modal) is pure Python on PyTorch: its "kernels" are
 * implicit torch ops and it has no FFI below Python.  Each entry point
 * below replaces the torch op(s) the reference calls at the cited file:line; INTEGRATION.md shows
 * the ctypes binding and the Python module API (trainers/maple.py, trainers/maple_fed.py mirror)
 * that sit on top.
 *
 * Conventions
 *   - All pointers are DEVICE pointers owned by the caller (kernels never allocate or free).
 *   - `stream` is a hipStream_t (void* so the header needs no HIP include); all work is enqueued
 *     asynchronously on it; nothing synchronises the host.  Safe to capture in a hipGraph.
 *   - fp16 tensors are IEEE binary16, row-major; `ld*` are leading dimensions in elements.
 *   - Return value: 0 on success, non-zero on argument or launch error; the message is in
 *     mf_last_error() (thread-local).
 */
#ifndef MAPFED_H_
#define MAPFED_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* mf_last_error(void);
int mf_abi_version(void);

/* ---- dense projections (GEMM, MFMA) ------------------------------------------------------
 * C[M,N] = epilogue(A[M,K] . B[N,K]^T), fp32 accumulate.  K % 64 == 0, N % 4 == 0.
 * epilogue: 0 none | 1 +bias | 2 +bias then +aux_in residual | 3 +bias, aux_out = pre-activation (the
 *           backward's operand; null: not stored, the forward-only eval engine), C = QuickGELU | 4 C = QuickGELU'(fp16(acc), aux_in) | 5 fp32 store | 6 +aux_in residual
 * tile: 0 auto (latency picks), -1 auto for a product of the tower off the step's critical path (tiles chosen for
 *       work per CU-second; the engine passes it for the text tower at c4, the vision tower at C5), 1 128x128,
 *       2 128x64, 3 64x64, 10 160x128, 15 96x128, 16 160x64, 20 256x256 8-wave, 26 96x64, 40 256x256 8-wave
 *       full-line (gemm8f).
 * Replaces: nn.Linear / addmm inside nn.MultiheadAttention in_proj + out_proj, mlp.c_fc, QuickGELU,
 * mlp.c_proj and the residual adds (clip/model.py:274-280,303-305,350-351), the patch-embed conv as
 * im2col GEMM (clip/model.py:514), the tower heads (clip/model.py:570, trainers/maple.py:76) and all
 * of their autograd dX/dW products.                                                             */
int mf_gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
               const void* bias, const void* aux_in, void* aux_out, int64_t ld_aux, int epilogue, int tile,
               void* stream);
/* General layouts: C[M,N] = epilogue(op(A) . op(B)^T) with
 *   a_kmajor = 0: A[m][k] at A[m*lda + k]  |  1: A[k*lda + m]   (e.g. dY^T of a weight gradient)
 *   b_kmajor = 0: B[n][k] at B[n*ldb + k]  |  1: B[k*ldb + n]   (e.g. nn.Linear W [out][in] in dX = dY . W)
 * K-major operands need rows % 8 == 0; K % 64 == 0 unless both operands are K-major (then any K: the
 * tail reads as zero).  Replaces the autograd dX / dW products of every nn.Linear on the path
 * (torch.mm(grad, W), torch.mm(grad^T, X)) without materialising a transpose.                      */
int mf_gemm(const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb, int b_kmajor, void* C, int64_t ldc,
            int M, int N, int K, const void* bias, const void* aux_in, void* aux_out, int64_t ld_aux, int epilogue,
            int tile, void* stream);
/* Split-K plain product (no epilogue) for few output tiles and a long K, e.g. the weight gradients
 * dW = dY^T X with K = tokens (autograd's torch.mm(grad.t(), x) of nn.Linear, clip/model.py:274-280):
 * `splits` 128x128-tile workgroups per tile each reduce a K slice into an fp32 plane of ws, then the
 * planes are summed in a fixed order into C (fp16 if out_f16, else fp32).  splits <= 0: automatic.
 * ws: mf_gemm_splitk_ws_floats(M, N, K, splits) floats.  Layout flags as mf_gemm; N % 8 == 0.     */
int mf_gemm_splitk(const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb, int b_kmajor, void* C,
                   int64_t ldc, int M, int N, int K, float* ws, int64_t ws_floats, int splits, int out_f16,
                   void* stream);
int mf_gemm_splitk_ws_floats(int M, int N, int K, int splits);

/* ---- LayerNorm (fp16 io, fp32 math; clip/model.py:153-159) --------------------------------
 * row_index (optional, int32): output row i normalises input row row_index[i]
 * (ln_post on class tokens clip/model.py:567, ln_final + EOT gather trainers/maple.py:72-76).    */
int mf_layernorm_fwd(const void* x, int64_t ldx, const int* row_index, const float* gamma, const float* beta,
                     void* y, int64_t ldy, float* mean, float* rstd, int rows, int D, void* stream);
/* mf_prompt_inject_fwd(x, prompt, rows / L, L, row0, nrows, D) then mf_layernorm_fwd(x, ...), in one
 * pass (bit-identical): the deep prompts injected at the start of a block and that block's ln_1
 * (clip/model.py:320-349, 153-159).  x is written (the injected rows).                            */
int mf_layernorm_fwd_inject(void* x, int64_t ldx, const float* gamma, const float* beta, void* y, int64_t ldy,
                            float* mean, float* rstd, int rows, int D, const float* prompt, int L, int row0,
                            int nrows, void* stream);
/* dx = fp16(dres + fp16(LN'(dy)))  (dres optional; dx may alias dres); dgamma/dbeta written or
 * accumulated (accumulate != 0).  workspace: 2 * mf_layernorm_bwd_blocks(rows) * D floats.        */
int mf_layernorm_bwd_blocks(int rows);
int mf_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const int* row_index,
                     const float* gamma, const float* mean, const float* rstd, const void* dres, int64_t ldres,
                     void* dx, int64_t lddx, float* dgamma, float* dbeta, float* workspace, int rows, int D,
                     int accumulate, void* stream);

/* Partials-only LayerNorm backward with the deep-prompt injection backward fused in: rows row0..row0+
 * nrows-1 of each L-row sequence store their dx as fp32 partials inj_part[rows/L][nrows][D] (the prompt
 * gradient = their sum over sequences, via mf_col_reduce_batch) and a zero dx row.  Replaces
 * mf_layernorm_bwd + mf_prompt_inject_bwd(zero_rows) on the same rows (clip/model.py:153-159,320-349). */
int mf_layernorm_bwd_inject(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* gamma,
                            const float* mean, const float* rstd, const void* dres, int64_t ldres, void* dx,
                            int64_t lddx, float* workspace, int rows, int D, float* inj_part, int L, int row0,
                            int nrows, void* stream);

/* Partials-only LayerNorm backward of a tower stored as the first L_live rows of each of its seqs L_full-row
 * sequences (the EOT-truncated text tower: every later row has exactly zero gradient).  The compact rows are
 * processed as rows t < L_live of the full tower, so the block partials (workspace: 2 *
 * mf_layernorm_bwd_blocks(seqs * L_full) * D floats) -- and dgamma / dbeta -- are bit for bit those of
 * mf_layernorm_bwd over all seqs * L_full rows.  inj_part (optional): the injection backward of
 * mf_layernorm_bwd_inject (L = L_live).  clip/model.py:153-159 under the causal mask of :679-685.        */
int mf_layernorm_bwd_live(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* gamma,
                          const float* mean, const float* rstd, const void* dres, int64_t ldres, void* dx,
                          int64_t lddx, float* workspace, int seqs, int L_live, int L_full, int D, float* inj_part,
                          int row0, int nrows, void* stream);

/* dgamma == dbeta == NULL: write the per-block partials only; their reduction is deferred to one
 * mf_col_reduce_batch over all LayerNorms of a backward pass.  desc = {const float* part; float* out;
 * int nblk, C, accumulate, pad} (mf_col_reduce_desc_bytes() bytes each, device memory):
 * out[c] (=|+=) sum_b part[b*C + c], fixed order.                                                  */
int mf_col_reduce_desc_bytes(void);
int mf_col_reduce_batch(const void* descs, int n, int max_cols, void* stream);

/* ---- attention (head_dim 64, L <= 512: one-pass kernels up to 256 rows, the caption path's growing
 * vision sequences of 257..512 rows on the two-pass forward / dK-dV + dQ backward; SDPA inside
 * nn.MultiheadAttention, clip/model.py:303-305, causal mask clip/model.py:679-685)
 * — qkv [N*L, 3*H*64], out [N*L, H*64], lse [N*H, ld_lse]                                         */
int mf_attention_fwd(const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out, float* lse, int ld_lse, int N,
                     int L, int H, int causal, void* stream);
/* The first q_rows query rows of every head only (K / V of all L <= 256 rows; each computed row bit-identical to
 * mf_attention_fwd's): the forward-only engine's last vision block, whose output ln_post reads only at the class
 * token (clip/model.py:567), attends query row 0 (r06).                                              */
int mf_attention_fwd_rows(const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out, float* lse, int ld_lse, int N,
                          int L, int H, int causal, int q_rows, void* stream);
/* The in-projection and the attention forward in one launch: qkv = fp16(x w^T + bias) (w = in_proj_weight
 * [3D, D], bias [3D]; bit-identical to mf_gemm_nt's EPI_BIAS) is written to qkv [N*L, 3D] and attended
 * as mf_attention_fwd does (bit-identical out / lse).  Shapes: the vision blocks (D = 768, 193..208
 * tokens) and the text blocks (D = 512, causal, 65..80 tokens); x_rows = rows of the x buffer (>= N*L).
 * Replaces the in_proj + SDPA of nn.MultiheadAttention (clip/model.py:303-305).                      */
int mf_qkv_attention_fwd(const void* x, int64_t ld_x, int x_rows, const void* w, const void* bias, void* qkv,
                         int64_t ld_qkv, void* out, int64_t ld_out, float* lse, int ld_lse, int N, int L, int H,
                         int causal, void* stream);
int mf_qkv_attention_supported(int N, int L, int H, int causal);
/* dqkv [N*L, 3*H*64]; dq_dot_ws: N*H*ld_lse floats of workspace                                   */
int mf_attention_bwd(const void* qkv, int64_t ld_qkv, const void* out, int64_t ld_out, const void* dout,
                     int64_t ld_dout, const float* lse, float* dq_dot_ws, int ld_lse, void* dqkv, int64_t ld_dqkv,
                     int N, int L, int H, int causal, void* stream);

/* ---- token assembly / prompt injection (clip/model.py:514-538,320-349; trainers/maple.py:54,152-166) */
int mf_im2col_patch(const void* img, int img_is_f32, void* out, int B, int R, int P, void* stream);
int mf_vision_assemble(const void* patch, const float* cls, const float* pos, const void* shared_ctx, void* x,
                       int B, int G2, int n_ctx, int D, void* stream);
int mf_text_assemble(const void* prefix, const void* ctx, const void* suffix, const float* pos, void* x, int K,
                     int L, int n_ctx, int D, void* stream);
int mf_prompt_inject_fwd(void* x, const float* prompt, int N, int L, int row0, int nrows, int D, void* stream);
/* out[r,:] (=|+=) sum_n dx[n*L+row0+r,:] (fp32 accumulate, fp16 or fp32 out); zero_rows clears them  */
int mf_prompt_inject_bwd(void* dx, int N, int L, int row0, int nrows, int D, void* out, int out_f16, int accumulate,
                         int zero_rows, void* stream);

/* ---- helpers for the backward products ------------------------------------------------------ */
/* ---- caption-conditioned visual prompts (K19; clip/model.py:457-476, 550-561; trainers/maple.py:307-322) */
/* The growing vision sequence of a prompted layer: dst [N, Lp+ncap, D] = src rows 0..Lp-n_ctx-1 | cap    */
/* [ncap, D] (fp16, shared by every sequence) | fp16(prompt [n_ctx, D] fp32); replaces the torch.cat of   */
/* clip/model.py:324-330 fed with cat(projected captions, deep prompt) (:558-559)                          */
int mf_seq_grow(const void* src, void* dst, const void* cap, const float* prompt, int N, int Lp, int ncap, int n_ctx,
                int D, void* stream);
/* its backward into the previous output: dsrc [N, Lp, D] = ddst rows 0..Lp-n_ctx-1, zeros for the dropped */
/* previous prompt rows                                                                                     */
int mf_seq_grow_bwd(const void* ddst, void* dsrc, int N, int Lp, int ncap, int n_ctx, int D, void* stream);
/* AttentionPooling (clip/model.py:464-476) of B captions from their token ids [B, T] (int32), the fp32     */
/* token-embedding table [vocab, D] and the fp16 weight vector w [D]: pooled [B, D] fp16.  An id outside    */
/* [0, vocab) reads nothing and makes its caption's pooled row NaN (the step's loss check then raises)      */
int mf_caption_pool(const int* tokens, int B, int T, const float* table, int vocab, const void* w, int D,
                    void* pooled, void* stream);
int mf_transpose_f16(const void* in, int64_t ld_in, void* out, int64_t ld_out, int R, int C, void* stream);
/* dst row n*L_full + t = src row n*L_live + t (t < L_live; other dst rows untouched), C % 8 == 0 columns: the
 * EOT-truncated text tower's block-11 weight-gradient operands in the full tower's row layout              */
int mf_seq_scatter(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, int N, int L_live, int L_full, int C,
                   void* stream);
int mf_colsum_blocks(int R);
/* out[c] = sum_r in[r,c]; workspace: mf_colsum_blocks(R) * C floats                               */
int mf_colsum_f16(const void* in, int64_t ld, int R, int C, void* out, int out_f16, float* workspace, void* stream);
int mf_cast_f16_f32(const void* in, float* out, int64_t n, void* stream);

/* ---- prompt-learner linears, M <= 16 rows (trainers/maple.py:111-131,194-215) --------------- */
int mf_small_linear_fwd(const void* X, const void* W, const void* b, void* Y, int M, int I, int O, int is_f16,
                        void* stream);
int mf_small_linear_bwd(const void* dY, const void* X, const void* W, void* dX, void* dW, void* db, int M, int I,
                        int O, int is_f16, int accumulate_dx, void* stream);

/* Batched form: every Linear of the prompt learner in one launch per direction.  descs: device array
 * of n descriptors of mf_small_linear_desc_bytes() bytes {const void *X, *W, *b; void *Y; const void* dY;
 * void *dX, *dW, *db; int M, I, O, is_f16, accumulate_dx, pad} (b / dX / dW / db may be null);
 * max_* bound the grid over the descriptors (M*O, M, I, O*I).                                         */
int mf_small_linear_desc_bytes(void);
int mf_small_linear_fwd_batch(const void* descs, int n, int max_mo, void* stream);
int mf_small_linear_bwd_batch(const void* descs, int n, int max_m, int max_i, int max_oi, void* stream);

/* ---- cosine-logit head + loss (trainers/maple.py:325,340-378) -------------------------------- */
int mf_clip_head_fwd(const void* img, const void* txt, int B, int K, int D, const float* logit_scale, void* img_n,
                     void* txt_n, float* norms, void* mm, void* logits, void* stream);
int mf_clip_loss_fwd_bwd(const void* img, const void* txt, const void* img_n, const void* txt_n, const float* norms,
                         const void* logits, const int64_t* label, int B, int K, int D, const float* logit_scale,
                         void* dmm, float* cos_ws, float* loss_out, void* dimg_n, void* dtxt_n, void* dimg,
                         void* dtxt, void* stream);
/* Soft (float) labels q [B,K] fp32 (trainers/maple.py:356-360): KL(q.clamp(1e-8) || softmax) batchmean
 * (fp32) + 0.5 (1 - mean cos(img_n, fp16(q) @ txt_n)); loss_out[0] is the fp32 total.  soft_ws: 2*B*D
 * fp16 of workspace.  The reference's `label @ text_features` multiplies fp32 by fp16 and raises in its
 * fp16 configuration; the label is taken in the features' dtype (what torch.autocast computes).       */
int mf_clip_loss_soft_fwd_bwd(const void* img, const void* txt, const void* img_n, const void* txt_n,
                              const float* norms, const void* logits, const float* label_probs, int B, int K, int D,
                              const float* logit_scale, void* dmm, float* cos_ws, void* soft_ws, float* loss_out,
                              void* dimg_n, void* dtxt_n, void* dimg, void* dtxt, void* stream);

/* eval predictions (trainers/maple.py:674-677): pred[b] = argmax_k logits (first max; NaN is the max);
 * acc[0] += #correct, acc[1] += B (device-side accuracy counters, read once per test pass)           */
int mf_argmax_correct(const void* logits, int B, int K, const int64_t* label, int64_t* pred, float* acc, void* stream);

/* ---- optimizer / federated averaging (trainers/maple.py:592-598; trainers/maple_fed.py:309-325) */
int mf_optim_chunk_bytes(void);
int mf_optim_chunk_elems(void);
int mf_clip_grad_norm(const void* g16, const float* g32, const void* chunks, int nchunks, float max_norm,
                      float* part, float* out, void* stream);
/* coef: the clip output (coef at [1]); hyper (device): {lr, momentum, weight_decay, first_step,    */
/* halt}; halt != 0 skips the update (a non-finite loss, trainers/maple.py:375-376)               */
int mf_sgd_step(void* p, void* g, void* buf, int64_t n, int is16, const float* coef, const float* hyper,
                void* stream);
/* The optimizer step in three launches (clip partial sums, coefficient + halt latch, SGD over both flat
 * buffers): mf_clip_grad_norm + mf_sgd_step(fp16) + mf_sgd_step(fp32), with hyper[4] = max(hyper[4], *halt_src,
 * *input_flag) (the step's non-finite-loss flag and its non-finite-input flag, input_flag nullable) folded into
 * the coefficient launch.  Bit-identical to those calls.                                                     */
int mf_optimizer_step(void* p16, void* g16, void* b16, int64_t n16, float* p32, float* g32, float* b32, int64_t n32,
                      const void* chunks, int nchunks, float max_norm, float* part, float* out, float* hyper,
                      const float* halt_src, const int* input_flag, void* stream);
/* bucket[0:n16+n32] = this client's trainables as fp32 (0 if *invalid_flag), bucket[n16+n32] = its vote
 * (1 valid / 0 invalid); after an all-reduce(SUM) of the n16+n32+1 floats, unpack writes
 * fp16(sum / n_valid) into every trainable and into the global copy g16/g32, n_valid read from
 * bucket[n16+n32] on the device; n_valid == 0 (every client failed) restores the trainables from g16/g32.
 * Replaces: safe_average_weights + broadcast_weights' load_state_dict (trainers/maple_fed.py:309-315,327-331). */
int mf_fedavg_pack(const void* p16, int64_t n16, const float* p32, int64_t n32, const int* invalid_flag,
                   float* bucket, void* stream);
int mf_fedavg_unpack(const float* bucket, void* p16, int64_t n16, float* p32, int64_t n32, void* g16, float* g32,
                     void* stream);
/* FedAvg in client order (trainers/maple_fed.py:311-314: torch.stack over the clients, then mean):   */
/* out[i] = sum_c gathered[c * stride + i] accumulated c = 0, 1, ... in fp32, for i < n; gathered    */
/* holds every client's packed bucket (an all-gather of mf_fedavg_pack outputs)                      */
int mf_fedavg_reduce_ordered(const float* gathered, int nclients, int64_t stride, int64_t n, float* out,
                             void* stream);
int mf_nonfinite_flag(const void* x, int64_t n, int is16, int* flag, void* stream);

/* ---- image transforms (data step before the path) ---------------------
 * Replaces the CPU transform workers the reference builds from configs/trainers/MaPLeFederated/
 * *.yaml:8-13 (Dassl build_transform -> torchvision RandomResizedCrop / RandomHorizontalFlip /
 * Resize + CenterCrop / ToTensor / Normalize on Pillow images, bicubic) and the fp16 cast at
 * trainers/maple.py:336.  Per image b, geom_host[b*11 ..] = {H, W, y0, x0, ch, cw, RH, RW, oy, ox,
 * flip} (HOST memory): crop [y0, y0+ch) x [x0, x0+cw) of the HxWx3 uint8 image at src + src_off[b],
 * resample it Pillow-exactly (interp 0 bicubic, 1 bilinear; 22-bit fixed-point taps, uint8
 * intermediate) to RH x RW, keep the out_h x out_w window at (oy, ox), flip it horizontally when
 * flip != 0, and store (u/255 - mean_c)/std_c as fp16 (out_f16) or fp32, planar [B][3][out_h][out_w].
 * src_off_host / src_off: the same byte offsets on the host (validated) and on the device.
 * ws: device workspace of mf_augment_ws_bytes(B, out_h, out_w, max crop height) bytes.         */
int64_t mf_augment_ws_bytes(int B, int out_h, int out_w, int max_rows);
int mf_augment(const void* src, int64_t src_bytes, const int64_t* src_off_host, const int64_t* src_off,
               const int* geom_host, int B, int out_h, int out_w, int interp, float mean0, float mean1, float mean2,
               float std0, float std1, float std2, void* out, int out_f16, void* ws, int64_t ws_bytes,
               void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAPFED_H_ */
