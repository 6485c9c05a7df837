/* fervit.h — C ABI of libfervit.so, the MI355X (gfx950) kernels behind the
 * FER-ViT training hot path.
 *
 * The reference (yuki-ominato/FER-ViT) is pure PyTorch: its hot-path "ABI" is the
 * set of torch.nn modules its models compose. Each entry point below replaces
 * one of those calls (reference file:line given per function); the Python host
 * (`fer-vit_amd/fervit/`) binds them with ctypes behind the reference's own
 * model constructors (`models_fer_vit/`, `modules/`).
 *
 * Conventions
 *  - Plain pointers to device memory owned by the caller (the PyTorch caching
 *    allocator); the library never allocates or frees caller memory. Optional
 *    pointers may be NULL.
 *  - Activations are row-major [rows][cols]; `dtype` selects FER_BF16 (fast path,
 *    fp32 accumulation) or FER_F32 (exact parity path). Parameters, their
 *    gradients, LayerNorm statistics and logits are always fp32.
 *  - Every call enqueues on `stream` and never synchronises the host.
 *  - Return 0 on success, a negative code on error; fer_last_error() then
 *    returns a thread-local message. No C++ exception crosses the ABI.
 *  - Dropout masks are regenerated from (seed, element index): element i is
 *    dropped iff its 16-bit uniform u16(i) < drop_thresh. Callers pass
 *    drop_thresh = round(p * 65536) clamped to [1, 65535] for 0 < p < 1,
 *    0 = dropout off (p = 0), 65536 = drop everything (p = 1, with drop_scale 0);
 *    drop_scale = 1/(1-p). (fervit/ops.py drop_args is the reference encoder.)
 *  - Gradient all-reduce (DDP) is NOT in this ABI: the Python host issues it through
 *    torch.distributed's "nccl" backend (= RCCL on ROCm) on a side stream, ordered against
 *    these kernels by HIP events (fervit/ddp.py). No fer_rccl_* entry points exist.
 */
#ifndef FERVIT_H
#define FERVIT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* fer_stream_t; /* == hipStream_t */

enum { FER_BF16 = 0, FER_F32 = 1 };
enum { FER_ACT_NONE_ = 0, FER_ACT_GELU_ = 1, FER_ACT_RELU_ = 2, FER_ACT_MUL_ = 3 /* aux_act only */ };
enum { FER_PRE_GATE_ = 16 /* act flag, see fer_epilogue */ };

/* C = epilogue(sum_k A(m,k) B(n,k)); A(m,k) = a_kc ? A[m*lda+k] : A[k*lda+m],
 * B(n,k) = b_kc ? B[n*ldb+k] : B[k*ldb+n].
 * Replaces nn.Linear forward/dgrad/wgrad (`image_vit.py:101-113`, `latent_vit.py:20,24-31`,
 * `hybrid_latent_vit.py:79`) and nn.Conv2d(k=P,s=P) patch embedding (`image_vit.py:27-32`)
 * once the input is in im2col order. ws: optional fp32 split-K workspace. */
typedef struct {
  int dtype;
  const void* A; int64_t lda; int a_kc;
  const void* B; int64_t ldb; int b_kc;
  int M, N, K;
  float* ws; int64_t ws_bytes;
} fer_gemm_desc;

/* Epilogue, applied per element in this order:
 *   v = alpha*acc (+ bias[n]); pre[m][n] = v; v = act(v); v = dropout(v, seed, m*drop_ld+n);
 *   v *= *post_scale; v *= act'(aux[m][n]); v += res[m][n]; c[m][n] (+)= v
 * act | FER_PRE_GATE_: pre[m][n] receives the backward gate act'(v) * keep * drop_scale (the
 * same keep bit as v's dropout) instead of v; the input-gradient GEMM of the next layer then
 * applies act' and the dropout in one multiply with aux_act = FER_ACT_MUL_ (v *= aux[m][n]). */
typedef struct {
  void* c; int64_t ldc; int c_f32; int accumulate; float alpha;
  const float* bias; int act;
  void* pre; int64_t ldp;
  const void* res; int64_t ldr;
  uint32_t drop_thresh; float drop_scale; uint64_t seed; int64_t drop_ld;
  const void* aux; int64_t ldx; int aux_act;
  const float* post_scale;
  /* optional fp32 column sums of the final output (the bias gradient of a layer whose input
   * gradient this GEMM produces, e.g. linear1.bias from the linear2 dgrad): colsum[n] (+)=
   * sum_m c[m][n]. Fused into the tile epilogue (per-tile partials + a fixed-order reduction,
   * deterministic); needs the desc workspace ws (>= fer_gemm_colsum_ws bytes). */
  float* colsum; int colsum_accumulate;
} fer_epilogue;

int fer_gemm(const fer_gemm_desc* d, const fer_epilogue* e, fer_stream_t stream);

/* Grouped weight gradients: dw[n][k] (+)= sum_m dy[m][n] x[m][k] (bf16 dy [M][N] row stride ld_dy,
 * bf16 x [M][K] row stride ld_x, fp32 dw [N][K] row stride ld_dw) for up to 8 nn.Linear weights
 * that share the token count M, in one launch -- the weight-gradient half of nn.Linear's backward
 * (`latent_vit.py:20,24-31`, `image_vit.py:101-113` TransformerEncoderLayer linears) for the
 * small-token configurations, where each weight alone is too few output tiles to fill the GPU.
 * splits: K (token) split per tile, 0 = automatic; a split run needs ws >= fer_wgrad_group_ws
 * bytes (fp32 slabs + tile tickets; the reduction is in-launch, fixed split order). */
typedef struct {
  const void* dy; int64_t ld_dy;
  const void* x; int64_t ld_x;
  float* dw; int64_t ld_dw;
  int M, N, K; int accumulate;
} fer_wgrad_item;
int fer_wgrad_group(const fer_wgrad_item* items, int n, int splits, float* ws, int64_t ws_bytes, fer_stream_t stream);
int64_t fer_wgrad_group_ws(const fer_wgrad_item* items, int n, int splits);

/* Workspace bytes fer_gemm needs for the fused column sums of an M x N output. */
int64_t fer_gemm_colsum_ws(int M, int N);

/* Tuning/testing hook (no reference counterpart): force the bf16 GEMM tile configuration for
 * every later fer_gemm call of the process. -1 = automatic (default); 0..11 = fixed kernel
 * (see csrc/gemm.hip dispatch_tile). Results are identical up to fp32 summation order. */
int fer_gemm_set_config(int cfg);

/* Testing / A/B hook (no reference counterpart): the persistent kernels (8-phase GEMM, persistent
 * attention; one workgroup per CU) take their items from a per-(device, stream) work queue
 * (mode 0, default) or walk a fixed blockIdx stride (mode 1; FERVIT_FIXED_STRIDE=1 sets it at
 * start-up). Results are bit-identical between the modes. */
int fer_set_persistent_mode(int mode);

/* A HIP stream whose kernels run only on the CUs set in mask (nwords 32-bit words, bit i = CU i in
 * the driver's CU numbering; hipExtStreamCreateWithCUMask), or with nwords = 0 an unmasked stream
 * of the given priority. For the weight-gradient side stream of the backward
 * (`train/train_image_vit.py:124` loss.backward(): this path's dgrad / wgrad split over streams);
 * the caller owns the stream (fer_stream_destroy). With a mask the stream is a BLOCKING stream
 * (it serialises with the legacy null stream) at the default priority, and a non-zero priority is
 * an error; without one it is non-blocking. Destroy a stream only once no live tensor of the
 * caller's allocator has it recorded (torch record_stream). */
int fer_stream_create_cu_mask(const uint32_t* mask, int nwords, int priority, fer_stream_t* out);
int fer_stream_destroy(fer_stream_t stream);

/* LayerNorm forward over rows of x [M][D] (nn.LayerNorm, biased variance;
 * post-norm `nn.TransformerEncoderLayer` norm1/norm2, heads `image_vit.py:162-163`,
 * `latent_vit.py:33-36`, timm pre-norm eps 1e-6). gamma/beta are [gamma_rows][D]:
 * row r uses gamma[(r / row_div) % gamma_rows] (gamma_rows=1: shared; LayerWiseNorm
 * `modules/layer_wise_norm.py:35-46` uses gamma_rows=L, row_div=1).
 * Saves mean/rstd [M] (fp32). y may alias nothing. */
int fer_layernorm_fwd(int dtype, const void* x, int64_t ldx, const float* gamma, const float* beta,
                      int gamma_rows, int row_div, void* y, int64_t ldy, float* mean, float* rstd,
                      int M, int D, float eps, fer_stream_t stream);

/* LayerNorm backward. dx = LN'(dy) (+ res), optional dx_drop = dropout_bwd(dx) (mask of
 * the branch feeding the norm's input, post-norm residual `x + Drop(h)`).
 * Column partial sums go to ws ([nblk][3][D] fp32, ws_bytes >= fer_layernorm_bwd_ws(M,D));
 * dgamma/dbeta/dbias (optional, [gamma_rows][D] fp32) receive sum(dy*xhat), sum(dy),
 * sum(dx_drop or dx); accumulate != 0 adds to them. */
int64_t fer_layernorm_bwd_ws(int M, int D);
int fer_layernorm_bwd(int dtype, const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* mean,
                      const float* rstd, const float* gamma, int gamma_rows, int row_div, const void* res,
                      int64_t ldr, void* dx, int64_t lddx, void* dx_drop, uint32_t drop_thresh, float drop_scale,
                      uint64_t seed, float* dgamma, float* dbeta, float* dbias, int accumulate, float* ws,
                      int64_t ws_bytes, int M, int D, fer_stream_t stream);

/* Multi-head self-attention core, softmax(Q K^T * scale) V with dropout on the
 * probabilities (F.multi_head_attention_forward -> scaled_dot_product_attention inside
 * nn.TransformerEncoderLayer; timm Attention for the hybrid). qkv: [B*N][ld_qkv] with
 * q|k|v column blocks of width H*dh (in_proj rows order); out: [B*N][ld_out].
 * `saved` (saved_floats fp32 words, >= fer_attention_saved_floats(...)) is the state kept for the
 * backward: lse [B*H*N] (natural log), padded to a multiple of 64 words, then -- bf16 with dropout,
 * N <= 224, dh <= 64 -- the probability-dropout keep bits, [B*H][NB][NB][32] uint32 (NB = ceil(N/32);
 * word (kb, qb, j) = bits over the 32 queries of block qb for key kb*32 + j; words of padding keys
 * kb*32 + j >= N unspecified), so the backward does not re-hash them. bf16: any N, dh <= 128, dh % 8 == 0 (persistent workgroup per CU walking the
 * (batch, head) units for N <= 256 and dh <= 64, 128-row chunks streamed through LDS otherwise). */
int64_t fer_attention_ws(int dtype, int B, int N, int H);
/* Forward kernel for bf16, N <= 224, dh <= 64: 0 automatic (the occupancy form for N > 96 with
 * dropout on, else the persistent kernel), 1 the persistent producer / consumer kernel, 2 the occupancy form (one workgroup
 * per (batch, head), two per CU). Same results bit for bit. */
int fer_attention_set_fwd_kernel(int k);
int64_t fer_attention_saved_floats(int dtype, int B, int N, int H, int dh, uint32_t drop_thresh);
int fer_attention_fwd(int dtype, const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out, float* saved,
                      int64_t saved_floats, int B, int N, int H, int dh, float scale, uint32_t drop_thresh,
                      float drop_scale, uint64_t seed, float* ws, int64_t ws_bytes, fer_stream_t stream);
/* Backward: dqkv [B*N][ld_dqkv] (dq|dk|dv). Optional colsum [3*H*dh] fp32 (+)= column sums of
 * dqkv over the B*N rows = in_proj.bias gradient, fused into the kernel (per-(batch) partials
 * + fixed-order reduction). ws >= fer_attention_ws bytes (fp32 path scratch / colsum partials). */
int fer_attention_bwd(int dtype, const void* qkv, int64_t ld_qkv, const void* out, int64_t ld_out,
                      const void* dout, int64_t ld_dout, const float* saved, int64_t saved_floats, void* dqkv,
                      int64_t ld_dqkv, float* ws, int64_t ws_bytes, int B, int N, int H, int dh, float scale,
                      uint32_t drop_thresh, float drop_scale, uint64_t seed, float* colsum, int colsum_accumulate,
                      fer_stream_t stream);

/* Column sums: out[n] (+)= scale * sum_m x[m][n]  (bias gradients). ws >= fer_colsum_ws(M,N). */
int64_t fer_colsum_ws(int M, int N);
int fer_colsum(int dtype, const void* x, int64_t ldx, int M, int N, float* out, int accumulate,
               const float* scale_ptr, float* ws, int64_t ws_bytes, fer_stream_t stream);

/* Deferred gradient reductions (the framework's backward pass; no reference counterpart: the
 * reference's bias / LayerNorm gradients come out of torch autograd one kernel each). mode 1
 * opens (or resumes) a window: fer_layernorm_bwd / fer_attention_bwd / fer_colsum / fused GEMM
 * column sums issued on `stream` write their per-block column partials into `arena` and queue the
 * fixed-order partial sum instead of launching it; mode 2 pauses (the queue stays, new calls run
 * immediately); mode 0 flushes and closes. fer_reduce_flush runs every queued sum as ONE launch on
 * that stream (bit-identical to the immediate path). Callers flush before anything reads those
 * gradients. Host state is per process (one window at a time, on one device: opening it from another
 * device while open is an error). Only part_reduce writers (the entry points above) are ordered
 * against the queue -- a queued sum runs first when a later reduction's output range overlaps its
 * own; any OTHER kernel that writes a queued gradient inside the window must flush first. */
int fer_reduce_defer(int mode, void* arena, int64_t arena_bytes, fer_stream_t stream);
int fer_reduce_flush(void);

/* Patch im2col (nn.Conv2d k=P,s=P, `image_vit.py:27-43`): x fp32 NCHW [B][C][Hh][Ww] ->
 * cols [B*gh*gw][ldc] in (c,kh,kw) order, cast to dtype. */
int fer_im2col_patch(int dtype, const float* x, int B, int C, int Hh, int Ww, int P, void* cols, int64_t ldc,
                     fer_stream_t stream);

/* Token assembly: t[b][0] = cls + pos[0]; t[b][1+i] = emb[b*n+i] + pos[1+i] (emb may be
 * dtype; `image_vit.py:151-156`, `latent_vit.py:42-44`, `hybrid_latent_vit.py:218-222`),
 * optional embedding dropout. Backward: dcls += sum_b dt[b][0], dpos += sum_b dt[b],
 * demb[b*n+i] = dt[b][1+i] (dropout-masked). ws >= fer_tokens_bwd_ws(B,N,D). */
int fer_tokens_fwd(int dtype, const void* emb, const float* cls, const float* pos, void* t, int B, int n, int D,
                   uint32_t drop_thresh, float drop_scale, uint64_t seed, fer_stream_t stream);
int64_t fer_tokens_bwd_ws(int B, int N, int D);
int fer_tokens_bwd(int dtype, const void* dt, void* demb, float* dcls, float* dpos, int accumulate, int B, int n,
                   int D, uint32_t drop_thresh, float drop_scale, uint64_t seed, float* ws, int64_t ws_bytes,
                   fer_stream_t stream);

/* Classification head on the CLS rows: logits = LN(t[b*N]) W^T + b (fp32 out), W [C][D].
 * (`image_vit.py:161-164`, `latent_vit.py:33-36,46-47`, `hybrid_latent_vit.py:110-114,236-237`) */
int fer_head_fwd(int dtype, const void* t, int64_t row_stride, const float* ln_w, const float* ln_b, float eps,
                 const float* W, const float* bias, float* logits, float* stats, int B, int D, int C,
                 uint32_t drop_thresh, float drop_scale, uint64_t seed, fer_stream_t stream);
/* Backward: dt rows b*row_stride get d(CLS); all other rows of dt are zeroed when
 * zero_rest != 0. Parameter grads accumulate when accumulate != 0. */
int64_t fer_head_bwd_ws(int B, int D, int C);
int fer_head_bwd(int dtype, const void* t, int64_t row_stride, const float* ln_w, const float* ln_b,
                 const float* W, const float* stats, const float* dlogits, void* dt, int zero_rest, int rows_total,
                 int D_ld, float* dln_w, float* dln_b, float* dW, float* dbias, int accumulate, int B, int D, int C,
                 uint32_t drop_thresh, float drop_scale, uint64_t seed, float* ws, int64_t ws_bytes,
                 fer_stream_t stream);

/* Softmax cross-entropy with label smoothing and optional class weights, mean reduction
 * normalised by sum w[y] (nn.CrossEntropyLoss, `train_image_vit.py:262-267`). Writes the
 * scalar loss and dlogits = grad_scale * dloss/dlogits. */
int fer_cross_entropy(const float* logits, const int64_t* labels, const float* weight, int B, int C,
                      float label_smoothing, float grad_scale, float* loss, float* dlogits, fer_stream_t stream);

/* w+ prologue (LatentViTv2 order SPE -> LWN -> LEAM, `latent_vit_v2.py:82-84`):
 * SemanticPE add (`semantic_pe.py:36-48`), LayerWiseNorm (+ residual gate,
 * `layer_wise_norm.py:35-50`), LEAM scale (`leam.py:31-40`). x,y fp32 [B][L][D]. */
int64_t fer_wplus_ws(int B, int L, int D);
int fer_wplus_fwd(const float* x, float* y, int B, int L, int D, const float* spe_group, const float* spe_layer,
                  const int64_t* groups, const float* lwn_w, const float* lwn_b, const float* lwn_gate,
                  const float* leam_w, float eps, float* saved, fer_stream_t stream);
int fer_wplus_bwd(const float* x, const float* saved, const float* dy, float* dx, int B, int L, int D,
                  const float* spe_group, const float* spe_layer, const int64_t* groups, const float* lwn_w,
                  const float* lwn_b, const float* lwn_gate, const float* leam_w, float eps, float* d_spe_group,
                  float* d_spe_layer, float* d_lwn_w, float* d_lwn_b, float* d_lwn_gate, float* d_leam_w,
                  int accumulate, float* ws, int64_t ws_bytes, fer_stream_t stream);

/* LatentDecomposer (`latent_decomposer.py:82-173`): dirs [C][L*D] (unit rows),
 * output_mode 0 expr_only, 1 id_only, 2 enhanced, 3 concat; decompose_mode 0 all_classes,
 * 1 max_class. y: [B][L or 2L][D] fp32. scores (optional) [B][C]. */
int fer_decompose(const float* w, const float* dirs, int B, int C, int LD, int output_mode, float alpha,
                  int decompose_mode, float* y, float* scores, fer_stream_t stream);

/* Elementwise helpers. */
int fer_cast_f32_bf16(const float* x, void* y, int64_t n, fer_stream_t stream);
int fer_cast_bf16_f32(const void* x, float* y, int64_t n, fer_stream_t stream);
/* y = x + s * t (s = *scale_ptr) over n elements, dtype; dot: out (+)= sum(a*b) fp32. */
int fer_axpy(int dtype, const void* x, const void* t, const float* scale_ptr, void* y, int64_t n,
             fer_stream_t stream);
int fer_dot(int dtype, const void* a, const void* b, int64_t n, float* out, int accumulate, float* ws,
            int64_t ws_bytes, fer_stream_t stream);
/* y = dropout(x) (p encoded by thresh); used for standalone dropout sites. */
int fer_dropout(int dtype, const void* x, void* y, int64_t n, uint32_t drop_thresh, float drop_scale, uint64_t seed,
                fer_stream_t stream);

/* Fused AdamW over a flat fp32 parameter buffer (torch.optim.AdamW semantics,
 * `train_image_vit.py:270-276`), segments with per-group lr / weight decay,
 * grad_scale multiplies the gradient (e.g. 1/world after an all-reduce sum, or a
 * clip factor read from clip_coef if non-NULL). Optionally refreshes the bf16 shadow copy. */
typedef struct {
  int64_t offset, numel;
  float lr, weight_decay, beta1, beta2, eps;
  int step;
} fer_adamw_segment;
int fer_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* param_bf16,
              const fer_adamw_segment* segs_device, int nsegs, int64_t max_seg_numel, float grad_scale,
              const float* clip_coef, const uint64_t* step_add, fer_stream_t stream);

/* Transposed bf16 weight shadow (no reference counterpart: layout only). segs: device int64
 * [nseg][4] = {offset, rows, cols, first_tile} into the flat buffers, first_tile the running
 * count of 64x64 tiles (ceil(rows/64)*ceil(cols/64) per segment), total_tiles their sum:
 * dst[off + c*rows + r] = src[off + r*cols + c]. The dgrad GEMMs read W^T K-contiguous. */
int fer_transpose_bf16_segments(const void* src, void* dst, const int64_t* segs, int nseg, int64_t total_tiles,
                                fer_stream_t stream);

/* LatentAugment (`data/latent_dataset.py:6-49`) on a device batch x fp32 [B][LD], in place:
 * x += N(0, noise_std); x *= U(scale_lo, scale_hi) per sample; x *= (U(0,1) > mask_prob).
 * Counter-based draws keyed by seed (and the step counter below, when set). */
int fer_latent_augment(float* x, int64_t B, int LD, float noise_std, float scale_lo, float scale_hi,
                       float mask_prob, uint64_t seed, fer_stream_t stream);

/* ImageViT input transforms (`data/image_dataset.py:139-173`, torchvision on PIL images) on the
 * device, SURVEY §8(f) row 4. Sources: B decoded uint8 HWC images (C = 1 or 3) packed in one
 * device buffer, image b at src + offsets[b], hwc[3b..3b+2] = H, W, C. Output fp32 NCHW
 * [B][3][S][S] normalised with mean3/std3 (host arrays).
 *   train = 0: Resize((S,S)) -> ToTensor -> Normalize (get_val_transforms)
 *   train = 1: Resize -> HorizontalFlip -> Rotation -> ColorJitter -> Affine -> ... (get_train_transforms)
 * with per-image parameter records params[B][16] (fer_image_aug_draw, or given by the caller):
 * [0] flip, [1] angle deg, [2..5] brightness/contrast/saturation/hue factors, [6..9] jitter op
 * order (0 b, 1 c, 2 s, 3 h), [10] tx, [11] ty (pixels), [12] scale, [13] hue enabled.
 * Every stage follows PIL's own arithmetic (fixed-point resampling and rotation, uint8 blends,
 * 8-bit HSV), so the output equals the reference pipeline's for the same parameters.
 * S <= 1024; any source size (shrinking widens the resize filter, as in PIL). */
typedef struct {
  float flip_p, degrees, brightness, contrast, saturation, hue, translate, scale_lo, scale_hi;
} fer_image_aug;
int fer_image_aug_draw(float* params, int B, int S, const fer_image_aug* aug, uint64_t seed, fer_stream_t stream);
int fer_image_augment(const uint8_t* src, const int64_t* offsets, const int32_t* hwc, int B, int S,
                      const float* params, int train, const float* mean3, const float* std3, float* out,
                      fer_stream_t stream);

/* Graph-replayed training steps (hipGraph capture of a whole step; no reference counterpart,
 * the reference trains eagerly). counter: caller-owned device uint64. After
 * fer_set_step_counter(counter) every dropout kernel mixes *counter into its seed, so a replayed
 * launch with a captured (constant) seed still draws a fresh mask each step; fer_adamw adds
 * *step_add to each segment's step. fer_step_advance(counter) (+1, a 1-thread kernel) is the
 * first node of the captured step. NULL disables (default). */
int fer_set_step_counter(const uint64_t* counter);
int fer_step_advance(uint64_t* counter, fer_stream_t stream);
/* sum of squares of grad (for clip_grad_norm_), out fp32 scalar; ws >= fer_colsum_ws(1, 4096). */
int fer_sumsq(const float* x, int64_t n, float* out, float* ws, int64_t ws_bytes, fer_stream_t stream);
/* clip coefficient: coef = min(1, max_norm / (sqrt(sumsq*sq_scale) + 1e-6)) (torch clip_grad_norm_). */
int fer_clip_coef(const float* sumsq, float sq_scale, float max_norm, float* coef, fer_stream_t stream);

const char* fer_last_error(void);
const char* fer_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FERVIT_H */
