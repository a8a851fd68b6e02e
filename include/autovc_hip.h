/*
 * autovc_hip.h — C-ABI of libautovc_hip.so, the MI355X (gfx950) kernels behind the
 * AutoVC / MetaConv / MetaPool / Discriminator training path.
 *
 * The reference (achyun/Autoformer) has no native code: every op on its hot path is an
 * implicit PyTorch -> cuDNN/cuBLAS call made by nn.Module forwards.  Each entry point
 * below replaces one such family of implicit calls; the reference call site is cited.
 * The Python host layer (autoformer_amd/) binds these with ctypes behind the reference's
 * own plugin API: factory.<Model>(dim_neck, dim_emb, dim_pre, freq), forward(x, c_org,
 * c_trg) (reference train.py:45-47, factory/AutoVC.py:185-211).
 *
 * Conventions
 *   - Activations are frame-major ("channels-last"): row r = b*T + t, C contiguous.
 *   - All device buffers are owned by the caller (PyTorch's caching allocator); the
 *     library never allocates or frees device memory.
 *   - Every launch goes on the hipStream_t passed as `stream`; no implicit syncs, so the
 *     calls are hipGraph-capturable.
 *   - Return 0 on success, a negative code on failure; avc_last_error() gives the
 *     (thread-local) message.
 */
#ifndef AUTOVC_HIP_H
#define AUTOVC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVC_ABI_VERSION 31

enum { AVC_F32 = 0, AVC_BF16 = 1 };
enum { AVC_ACT_NONE = 0, AVC_ACT_RELU = 1, AVC_ACT_TANH = 2, AVC_ACT_LEAKY = 3, AVC_ACT_GELU = 4, AVC_ACT_SIGMOID = 5 };

/* One GEMM operand, logically an R x K matrix (R = M for A, N for B).
 *   kstrided = 0 : element (r, k) at ptr[r*ld + k]   (K contiguous)
 *   kstrided = 1 : element (r, k) at ptr[k*ld + r]   (R contiguous)
 * Frame window (taps > 0): the frame-indexed dimension (r when kstrided = 0, k when
 * kstrided = 1) is a frame f = b*t_out + t; the other dimension is split as
 * tap*chans + c, and the element is src[(b*t_in + t + tap - pad)*ld + c], zero when
 * t + tap - pad is outside [0, t_in).  This expresses Conv1d im2col (taps = kernel size)
 * and the LSTM's h_{t-1} time shift (taps = 1, pad = +-1) without materialising either.
 * batch_stride: element offset between consecutive blockIdx.z batches (0 = shared). */
typedef struct {
  const void* ptr;
  int dtype;
  int kstrided;
  long long ld;
  long long batch_stride;
  int taps, pad, t_out, t_in, chans;
} avc_operand;

/* C[z][m][n] (+)= sum_k A(m,k) B(n,k) (+ bias[n]) ; fp32 C.
 * compute: AVC_BF16 -> bf16 MFMA 16x16x32 with fp32 accumulate; AVC_F32 -> exact fp32 MFMA.
 * split_k > 1 accumulates with fp32 atomics (C is zeroed first unless accumulate); so does a
 * batch > 1 with c_batch_stride == 0 (the output is the SUM over the batch).
 * bn_partial (nullable, split_k == 1, batch == 1): per 128-row tile and column the
 *   pair (sum, M2 about the tile mean) of the stored values, layout [ceil(M/128)][N][2],
 *   the BatchNorm batch-statistics epilogue.  */
typedef struct {
  int M, N, K, batch;
  avc_operand a, b;
  float* c;
  long long ldc, c_batch_stride;
  const float* bias;
  int accumulate;
  int split_k;
  float* bn_partial;
  int compute;
  void* c_bf16;         /* nullable: also store C rounded to bf16 (same ldc), for the next GEMM; with c == NULL
                            (no accumulate / split-K / batch-sum / cperm) C is stored in bf16 only */
  const float* residual; /* nullable: C = A.B + bias + residual (same ldc / batch stride) */
  int cperm;             /* 0, or taps > 1: columns are (tap, channel) pairs, n = tap*(N/taps) + ch, and
                            land at C[m*ldc + ch*taps + tap] -- a Conv1d weight gradient written straight
                            into nn.Conv1d's [Co][Ci][K] layout (no bias / residual / bf16 / BN epilogue) */
  const float* row_bias; /* nullable: per-(utterance, edge class) bias added with `bias` (before the BN
                            statistics): row m = b*rb_t + t adds row_bias[(b*(2 rb_pad + 1) + cls)*N + n],
                            cls = t (t < rb_pad), 2 rb_pad - (rb_t - 1 - t) (t >= rb_t - rb_pad), else
                            rb_pad -- the speaker half of the encoder's first conv folded out of the
                            frames (factory/AutoVC.py:46-51, fold.hip); non-K-strided operands only */
  int rb_t, rb_pad;
  int c_bf16_act;        /* 0, or AVC_ACT_GELU: c_bf16 receives GELU(C) (erf form) instead of C rounded -- the
                            next GEMM's operand (MLPMixer.py:16-23 FeedForward); the pre-activation C goes to
                            c (fp32) and / or c_pre_bf16.  Needs c_bf16 and one of those, ldc == N, no
                            accumulate / split-K / batch sum / cperm */
  const void* act_grad_of; /* nullable: C = (A.B + bias) * GELU'(act_grad_of[m*ldc + n]) (fp32 or bf16 per
                            act_grad_dtype) stored to c and / or c_bf16 -- the GELU backward folded into the
                            data-gradient GEMM.  Same restrictions, no residual */
  float* col_sum;        /* nullable: col_sum[n] += sum over m of the stored C[m][n], n < col_sum_n (0 = N) -- the
                            bias gradient of the layer whose output gradient C is (MLPMixer.py:16-23), without a
                            second pass over C.  Float atomics (order-dependent rounding); no accumulate /
                            split-K / batch sum / cperm */
  int col_sum_n;
  void* c_pre_bf16;      /* nullable, with c_bf16_act: the pre-activation C rounded to bf16 (same ldc) -- the
                            backward's act_grad_of at half the bytes of an fp32 C */
  int act_grad_dtype;    /* AVC_F32 / AVC_BF16: element type of act_grad_of */
  int c_trans_rows;      /* 0, or R > 0 (R % 4 == 0, dividing M of the folded batch): C(m, n) is stored at
                            ((m / R) * N + n) * R + m % R -- each R-row block of C transposed, the per-utterance
                            (D x NP) token-mixing output written straight into the frame-major (NP x D) layout
                            with the residual read in the same layout (MLPMixer.py:80-86).  fp32 C only, ldc == N,
                            bias / residual / accumulate; no bf16 / BN / GELU / col_sum / row-bias epilogue */
} avc_gemm_desc;

int avc_abi_version(void);
const char* avc_last_error(void);
/* Host-only test hook (no device, no HIP call): one reservation of n slots from a ring of
 * `pool` slots (power of two) through *cursor, the allocator behind the library's arrival-counter
 * and zero-slot pools.  Returns the first slot; reserved ranges never overlap across the wrap
 * (ABI 29). */
unsigned avc_ring_reserve_test(unsigned* cursor, unsigned n, unsigned pool);

/* Conv1d / Linear / LSTM-projection / weight-gradient GEMMs.
 * Replaces: nn.Conv1d (factory/Norm.py:21-28 via AutoVC.py:26-41, 79-94, 125-171,
 * Discriminator.py:7-9, MLPMixer.py:53,82), nn.Linear (Norm.py:40-50, MLPMixer.py:70-76),
 * the W_ih products inside nn.LSTM (AutoVC.py:43,77,96) and all their backward GEMMs. */
int avc_gemm(const avc_gemm_desc* d, void* stream);

/* BatchNorm1d BACKWARD reduction fused into a data-gradient GEMM (avc_gemm_bnb).  The GEMM's
 * output C is dL/da of a conv + BatchNorm + activation layer (the layer BEFORE this GEMM's own
 * layer: e.g. the encoder's conv1 -> conv2 chain, AutoVC.py:56-58, postnet :167-170); y is that
 * layer's stored conv output (pre-BN, [M][N] row-major like C), mean / rstd its batch
 * statistics, gamma / beta its affine parameters, act its activation (AVC_ACT_*).  The
 * epilogue recomputes dz = C * act'(z), z = (y - mean)*rstd*gamma + beta, sums dz, dz*yhat and
 * yhat per column and 128-row tile, and the last row tile of each column tile writes the
 * planar apply constants coef[6][N] (16-B aligned; k1 = gamma*rstd, mean(dz), mean(dz*yhat),
 * mean, rstd, beta) and dgamma / dbeta / the conv-bias gradient (accumulated when accumulate
 * != 0; nullable) -- what avc_bn_bwd's reduce + finalize passes compute; avc_bn_bwd_apply
 * then finishes the layer.  ws: avc_gemm_bnb_ws(M, N) floats.  Replaces the statistics half
 * of nn.BatchNorm1d.backward (AutoVC.py:38,91,138,154,169). */
typedef struct {
  const void* y;
  int y_dtype;
  const float* mean;
  const float* rstd;
  const float* gamma;
  const float* beta;
  int act;
  float* coef;
  float* dgamma;
  float* dbeta;
  float* dbias;
  int accumulate;
  float* ws;
  /* nullable (ABI 26): the layer's dy (bf16, avc_bn_bwd_apply's output with these constants) is
   * written too -- by the epilogue itself on the halo conv ring, whose row tiles of a column tile
   * are all resident (a column-tile barrier after the last row tile's finalize), else by an apply
   * pass after the GEMM.  y bf16, N % 8 == 0 on the fused form. */
  void* dy_bf16;
} avc_bnb_args;

size_t avc_gemm_bnb_ws(int M, int N);
int avc_gemm_bnb(const avc_gemm_desc* d, const avc_bnb_args* bnb, void* stream);

/* The apply half of the BatchNorm backward with the constants of avc_gemm_bnb:
 * dy = k1*(dz - mean(dz) - yhat*mean(dz*yhat)), dz from the pre-activation recomputed from y.
 * dy fp32 and/or bf16 (dy_bf16), either nullable but not both. */
int avc_bn_bwd_apply(const void* dA, int dA_dtype, const void* y, int y_dtype, const float* coef, int M, int C,
                     int act, float* dy, void* dy_bf16, void* stream);

/* BatchNorm1d training-mode statistics from avc_gemm's bn_partial: mean/rstd per
 * channel, scale = gamma*rstd, shift = beta - mean*scale, running-stat update with
 * momentum and UNBIASED variance, num_batches_tracked += 1.
 * Replaces nn.BatchNorm1d.forward (train mode) at AutoVC.py:38,91,138,154,169. */
int avc_bn_finalize(const float* partial, int M, int C, const float* gamma, const float* beta,
                    float* running_mean, float* running_var, long long* num_batches_tracked,
                    float momentum, float eps, float* mean, float* rstd, float* scale, float* shift,
                    void* stream);

/* avc_gemm with the train-mode BatchNorm1d finalize of avc_bn_finalize fused in: the GEMM's
 * bn_partial statistics are merged by the last row tile of each column tile (bf16 fast kernels;
 * other paths launch avc_bn_finalize after the GEMM) -- same outputs, running statistics updated
 * nupd times, num_batches_tracked += nupd.  gamma / beta / running stats / nbt are nullable.
 * Replaces nn.BatchNorm1d.forward (train mode) at AutoVC.py:38,91,138,154,169 with its conv. */
typedef struct {
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  long long* num_batches_tracked;
  float momentum, eps;
  int nupd;
  float* mean;
  float* rstd;
  float* scale;
  float* shift;
  /* nullable (ABI 26): act(y*scale + shift) in bf16 (avc_bn_apply without residual, ldc == N) written
   * too -- by the halo conv ring's epilogue behind a column-tile barrier, else by a pass after. */
  void* apply_bf16;
  int apply_act;
} avc_bn_fin;
int avc_gemm_bn(const avc_gemm_desc* d, const avc_bn_fin* f, void* stream);

/* Eval-mode coefficients from the running statistics (nn.BatchNorm1d in .eval()). */
int avc_bn_eval(const float* running_mean, const float* running_var, const float* gamma, const float* beta, int C,
                float eps, float* mean, float* rstd, float* scale, float* shift, void* stream);

/* Per-channel statistics pass for inputs that did not come out of avc_gemm (ld >= C). */
int avc_bn_stats(const float* y, long long ld, int M, int C, float* partial, void* stream);

/* out[r][c] = act(y[r][c]*scale[c] + shift[c]) (+ residual[r][c]); rows of length C.
 * y is fp32 or bf16 (y_dtype = AVC_F32 / AVC_BF16); out (fp32) and out_bf16 are each nullable,
 * not both (bf16 compute mode stores inter-layer activations in bf16 only). */
int avc_bn_apply(const void* y, int y_dtype, const float* scale, const float* shift, const float* residual,
                 float* out, void* out_bf16, int M, int C, int act, void* stream);

/* BatchNorm1d + activation backward.  yhat = (y-mean)*rstd; dz = dA * act'(.), taken from the
 * stored activation output `a` when it is given, else (a == NULL) from the pre-activation
 * yhat*gamma + beta recomputed here (one activation-sized read fewer per pass; also right
 * when a residual was added after the activation).
 * Writes dy = gamma*rstd*(dz - sum(dz)/N - yhat*sum(dz*yhat)/N), and dgamma, dbeta and
 * the (analytically ~0) bias gradient of the producing conv (accumulate != 0: added into them).
 * dA and y are fp32 or bf16 (their dtype arguments); dy (fp32) and dy_bf16 are each nullable, not both.
 * `ws` >= avc_bn_bwd_ws floats. */
size_t avc_bn_bwd_ws(int M, int C);
int avc_bn_bwd(const void* dA, int dA_dtype, const float* a, const void* y, int y_dtype, const float* mean,
               const float* rstd, const float* gamma, const float* beta, int M, int C, int act, float* dy,
               void* dy_bf16, float* dgamma, float* dbeta, float* dbias, int accumulate, float* ws, void* stream);

/* out[n] (+)= sum_m x[m*ld + n] (bias gradients); out2 (nullable) receives the same sums (an
 * LSTM's b_ih and b_hh share one gradient, nn.LSTM AutoVC.py:43,77,96).  ws >= avc_colsum_ws floats. */
size_t avc_colsum_ws(int M, int N);
int avc_colsum(const float* x, long long ld, int M, int N, float* out, float* out2, int accumulate, float* ws,
               void* stream);

/* LSTM layer recurrence (both directions of a bidirectional layer in one call).
 * Replaces the time loop of nn.LSTM (AutoVC.py:43,55 encoder BiLSTM; :77,103 lstm1;
 * :96,110 lstm2).  xproj (B,T,dirs*4H) already holds x W_ih^T + b_ih + b_hh.
 * w_hh: dirs x [4H][H] in `wdtype`; outputs h (B,T,dirs*H) fp32, c (B,T,dirs*H),
 * gates (B,T,dirs*4H) activated.  Small H (<= 64) keeps fp32 weights and state; `compute` ==
 * AVC_BF16 selects its v_exp/v_rcp activation forms (IEEE library forms otherwise).  hbuf (large
 * H, bf16 compute): scratch of at least
 * max(4*dirs*B*H, 8*B*H + 16) bytes.  For dirs == 1, H in {512, 1024} and enough CUs the
 * whole sequence runs as ONE persistent launch (W_hh slices register-resident, h_t handed
 * between workgroups as write-through payload + per-workgroup flags, bounded spins; timeout
 * flag = u32 at byte 0 of hbuf); otherwise one fused kernel per time step.  The small-H and the
 * persistent launches can also write a bf16 copy of h (h_bf16, (B,T,dirs*H), the next GEMMs'
 * operand; else null — the per-step path needs null). */
int avc_lstm_fwd(const float* xproj, const void* w_hh, int wdtype, int B, int T, int H, int dirs,
                 float* h, void* h_bf16, float* c, float* gates, void* hbuf, int compute, void* stream);

/* Backward recurrence.  dh_out (B,T,dirs*H) = dL/dh; writes dgates (B,T,dirs*4H)
 * (pre-activation).  w_hh_t: dirs x [H][4H] transposed copy (large H) or w_hh itself
 * (small H, pass the same layout as avc_lstm_fwd). dcbuf: B*H*dirs fp32.  gbuf (large H,
 * bf16 compute): at least avc_lstm_bwd_scratch_bytes(B, H, dirs) bytes.  For dirs == 1, H in
 * {512, 768, 1024} and enough CUs the whole sequence is ONE persistent launch (W_hh^T slices
 * register-resident; each workgroup gathers the group's bf16 dG_{t+1}, handed over as
 * write-through payload + per-workgroup flags, bounded spins; timeout flag = u32 at byte 0 of
 * gbuf).  The small-H and persistent launches can also write a bf16 copy of dgates (dgates_bf16,
 * else null); the per-step path needs null. */
/* Bytes of the backward scratch gbuf for (B, H, dirs). */
size_t avc_lstm_bwd_scratch_bytes(int B, int H, int dirs);

int avc_lstm_bwd(const float* dh_out, const float* h, const float* c, const float* gates,
                 const void* w_hh, const void* w_hh_t, int wdtype, int B, int T, int H, int dirs,
                 float* dgates, void* dgates_bf16, float* dcbuf, void* gbuf, int compute, void* stream);

/* Decoder lstm1 with the input projection folded per code (ABI 31; AutoVC.py:96,103 on the concat
 * of AutoVC.py:197-204): the persistent forward above reading step t's projection
 * from row b*nc + t/(T/nc) of pcode (B*nc, 4H) fp32 = [code_j ; c_trg_b] . W_ih^T + b_ih + b_hh,
 * without expanding it to B*T rows.  Persistent path only (bf16 compute, avc_lstm_persistent(B, H,
 * 1, AVC_BF16, 0)), T % nc == 0; h_bf16 and hbuf as avc_lstm_fwd.  Replaces avc_expand_codes +
 * avc_lstm_fwd there. */
int avc_lstm_fwd_fold(const float* pcode, int nc, const void* w_hh, int B, int T, int H, float* h,
                      void* h_bf16, float* c, float* gates, void* hbuf, void* stream);
/* Its backward: the persistent backward writing dG's bf16 twin (dgates_bf16, required), dgates
 * fp32 only when non-null, and s_code (B*nc, 4H) = dG summed over each code's T/nc frames (fp32,
 * plus its bf16 twin s_code_bf16 when non-null) -- the fold's segment sum taken inside the
 * recurrence instead of a pass over dG afterwards (avc_segsum).  gbuf as avc_lstm_bwd. */
int avc_lstm_bwd_fold(const float* dh_out, const float* c, const float* gates, const void* w_hh_t,
                      int B, int T, int H, int nc, float* dgates, void* dgates_bf16, float* s_code,
                      void* s_code_bf16, void* gbuf, void* stream);

/* Two stacked unidirectional layers of one nn.LSTM (decoder lstm2, AutoVC.py:96,110: 512 -> 1024,
 * num_layers=2) forward in ONE persistent launch, as a layer wavefront (tick k = layer 0 step k
 * beside layer 1 step k-1; layer 1's input projection inside the recurrence).  xproj0 (B,T,4H) =
 * x W_ih0^T + b_ih0 + b_hh0; w_hh0, w_ih1, w_hh1: [4H][H] bf16; bias1 = b_ih1 + b_hh1 (4H fp32).
 * Outputs per layer as avc_lstm_fwd (h fp32 + bf16 twin, c, activated gates).  buf: at least
 * avc_lstm2_scratch_bytes(B, H) bytes (control words + flags zeroed by the call, then a
 * [2 layers][2][B][H] bf16 payload); timeout flag = u32 at byte 0, fault word as avc_lstm_fwd.
 * Only where avc_lstm2_persistent(B, H, In1 = H, AVC_BF16) is 1 (H = 1024, bf16, whole grid
 * ceil(B/16) * H/16 workgroups resident); the caller runs the layers one by one otherwise. */
int avc_lstm2_persistent(int B, int H, int in1, int compute);
size_t avc_lstm2_scratch_bytes(int B, int H);
int avc_lstm2_fwd(const float* xproj0, const void* w_hh0, const void* w_ih1, const void* w_hh1,
                  const float* bias1, int B, int T, int H, float* h0, void* h0_bf16, float* c0,
                  float* gates0, float* h1, void* h1_bf16, float* c1, float* gates1, void* buf,
                  void* stream);

/* Diagnostics (no reference counterpart): with buf non-null, later persistent LSTM launches
 * record the 100 MHz realtime clock at 4 points of every step of every workgroup into
 * buf[(workgroup*T + step)*4 + j] (j: step start, exchange complete, product reduced,
 * published; u64, caller-sized).  null switches it off (the default). */
int avc_lstm_trace(void* buf);

/* Fault reporting (no reference counterpart; nn.LSTM cannot fail this way).  `word` is a
 * caller-owned device u32 for the CURRENT device (null unregisters).  A persistent LSTM
 * launch whose bounded spin times out -- a workgroup of its grid never became resident, or
 * a member died -- ORs bit 0 into it (as well as into the launch's own ctl[0]) and exits;
 * the host reads the word where it reads the loss and raises.  Sticky until the caller
 * clears it. */
int avc_set_fault_word(void* word);

/* Debug: spin bound of the persistent recurrences' waits (0 = the built-in bound, or the
 * AVC_LSTM_SPIN environment variable when set).  ~0u injects a timeout: every wait fails at
 * once, deterministically (the fault-path tests); a small bound only times out the waits that
 * do not succeed within it. */
int avc_lstm_set_spin(unsigned spins);

/* Benchmarking: configuration of the 8-wave deep-ring GEMMs (gemm_ring.hip) that avc_gemm
 * dispatches bf16 products with K-contiguous operands to.  mode -1 = the measured default policy
 * (256 x 256 tiles for N >= 1024 with a tile per CU, the halo ring for utterance-aligned 5-tap
 * convs), 0 = off (the older kernels), 1 = forced bm x bn tile with nst ring slots; gm = row tiles
 * per tile group (<= 0 keeps the current value); win: 0 = conv window operands never take it,
 * 1 = forced configurations stream them as im2col windows, 2 = 5-tap convs take the halo ring
 * (10 = the same without the one-utterance tile for 128 < T <= 192).
 * Same as the AVC_RING / AVC_RING_WIN environment variables.  Returns 0. */
int avc_gemm_set_ring(int mode, int bm, int bn, int nst, int gm, int win);

/* Decoder lstm2 BACKWARD, both layers in one persistent launch (layer wavefront, lstm.hip
 * lstm2_persist_bwd): tick k runs layer 1 at step T-1-k and layer 0 at step T-k; layer 0's upstream
 * gradient dG1 W_ih1 is formed inside the recurrence.  dh1 = dL/dh of layer 1's output (B,T,H);
 * c0/gates0, c1/gates1 the forward's cell states and activated gates (avc_lstm2_fwd); w_hh0_t,
 * w_ih1_t, w_hh1_t the transposed bf16 weights [H][4H]; outputs dg0 / dg1 = dL/d(pre-activation
 * gates) (B,T,4H) fp32 and / or their bf16 twins (each layer needs one of the two; ABI 28: the fp32
 * form is optional).  db_part (nullable, ABI 28): [2 layers][ceil(B/16) groups][4H] floats, each the
 * layer's dG summed over one 16-utterance group and every step -- the column sums of dG that make
 * the bias gradients (b_ih, b_hh: AutoVC.py:96's nn.LSTM), so the fp32 dG need not be stored for them.
 * buf: avc_lstm2_bwd_scratch_bytes(B, H) bytes.
 * bf16 compute, H = 1024, the whole grid resident (avc_lstm2_bwd_persistent).  Replaces
 * nn.LSTM.backward of AutoVC.py:96,110's two-layer lstm2 (two avc_lstm_bwd + the dX1 GEMM). */
int avc_lstm2_bwd_persistent(int B, int H, int compute);
size_t avc_lstm2_bwd_scratch_bytes(int B, int H);
int avc_lstm2_bwd(const float* dh1, const float* c0, const float* gates0, const float* c1, const float* gates1,
                  const void* w_hh0_t, const void* w_ih1_t, const void* w_hh1_t, int B, int T, int H, float* dg0,
                  void* dg0_bf16, float* dg1, void* dg1_bf16, void* buf, float* db_part, void* stream);

/* Which deep-ring kernel the last avc_gemm on this host thread launched (tests, tools): 0 none (an
 * older kernel), 1 gemm_ring_kernel, 2 the 128-row halo conv (conv_ring_kernel, its BN-backward
 * form included), 3 the one-utterance halo conv (conv_utt_kernel, 128 < T <= 192), 4 the
 * warp-specialised halo conv, 5 the 32-deep-slot ring.  Replaces no reference interface. */
int avc_gemm_ring_last(void);

/* 1 when avc_lstm_fwd (backward = 0) / avc_lstm_bwd (backward = 1) take the one-launch
 * persistent path for this shape on the current device: bf16 compute, dirs == 1, H in
 * {512, 768, 1024}, and the occupancy API admits the whole grid (ceil(B/8) * H/32
 * workgroups of 512 threads) resident at once.  0 otherwise (per-step kernels). */
int avc_lstm_persistent(int B, int H, int dirs, int compute, int backward);
/* 1 when avc_lstm_fwd / avc_lstm_bwd run this small-H shape (H <= 64) on the MFMA BiLSTM kernels
 * (lstm_mfma_fwd / _bwd: bf16 compute, H in {16, 32, 44, 48, 64}; ABI 29), 0 when on the packed-FMA
 * kernels.  avc_lstm_set_small_mfma: 1 selects the MFMA form, 0 the packed-FMA form (the default:
 * measured faster, profiles/r6_bilstm_mfma_ab.txt), -1 back to the AVC_BILSTM_MFMA environment default.
 * Replaces: the recurrent product of nn.LSTM(512, 44, 2, bidirectional) (AutoVC.py:43,54-55). */
int avc_lstm_small_mfma(int H, int compute);
int avc_lstm_set_small_mfma(int mode);

/* Elementwise / layout kernels of the model glue (AutoVC.py:46-48, 56-66, 197-207). */
int avc_enc_concat(const float* mel, long long mel_ld, const float* emb, float* out, int B, int T,
                   int n_mel, int d_emb, void* stream);
int avc_codes_gather(const float* lstm_out, float* codes, int B, int T, int dim_neck, int freq,
                     void* stream);
int avc_codes_scatter(const float* dcodes, float* dlstm_out, int B, int T, int dim_neck, int freq,
                      void* stream);
int avc_dec_concat(const float* codes, const float* emb, float* out, int B, int T, int n_codes,
                   int code_dim, int d_emb, void* stream);
int avc_dec_concat_bwd(const float* dout, float* dcodes, int B, int T, int n_codes, int code_dim,
                       int d_emb, void* stream);

/* Decoder lstm1 input projection folded per code and per utterance:
 * out[b*T+t][:] = pc[b*nc + t/(T/nc)][:] + pe[b][:], pc = codes . W_ih[:, :cd]^T (B*nc x G),
 * pe = c_trg . W_ih[:, cd:]^T + b_ih + b_hh (B x G): the x_t . W_ih^T + b of nn.LSTM at
 * AutoVC.py:96,103 on the concat of AutoVC.py:197-204, without the concat or its (B*T x G x cd+de)
 * GEMM.  G % 4 == 0, 16-B aligned. */
int avc_expand_codes(const float* pc, const float* pe, float* out, int B, int T, int nc, int G, void* stream);
/* The folded lstm1's operand (ABI 31): out[b*nc + j] = [codes[b][j*cd : (j+1)*cd] ; emb[b]] in bf16,
 * (B*nc, cd+de) -- one row per code, so ONE GEMM out . W_ih^T + b gives avc_lstm_fwd_fold's pcode and
 * the weight gradient is s_code^T . out (the per-utterance half sums to s_utt^T . c_trg). */
int avc_code_cat(const float* codes, const float* emb, void* out_bf16, int B, int nc, int cd, int de,
                 void* stream);

/* Weight repacks (and fp32 -> compute dtype).  conv: W[co][ci][k] ->
 *   mode 0: Wf[co][k][ci] (forward im2col order)
 *   mode 1: Wd[ci][k'][co] with k' = K-1-k (data-gradient order)
 * grad_unpack: dWf[co][k][ci] -> dW[co][ci][k] (accumulate optional). */
int avc_conv_pack(const float* w, void* out, int dtype, int Cout, int Cin, int Kw, int mode, void* stream);
int avc_conv_grad_unpack(const float* dwf, float* dw, int Cout, int Cin, int Kw, int accumulate, void* stream);

/* The encoder conv0 fold (fold.hip; factory/AutoVC.py:46-51: cat(mel, c_org broadcast) -> ConvNorm(336,
 * 512, 5)).  pack_slice packs the input channels [ci0, ci0 + cn) of W [Co][Ci][K] (fp32) into `out`
 * (dtype), the channel axis zero-padded to cpad: mode 0 Wf[co][k][cpad] (forward), 1 Wd[cpad][K-1-k][co]
 * (data gradient), 2 We[k][co][cpad] (the speaker term E = c . We^T); mode 3 Wd[cn][K-1-k][cpad] with
 * the OUTPUT channel axis padded (cpad >= Co; the Discriminator's 22-channel conv3 data gradient).
 * edge_table: S[b][cls][co] = sum over the taps k valid at edge class cls (see avc_gemm_desc.row_bias)
 * of E[b][k*Co + co]; T > 2 pad.
 * edge_colsum: out[b][k][c] = sum over the frames t of utterance b with 0 <= t + k - pad < T of
 * dy[b*T + t][c] (dy fp32 or bf16, C % 4 == 0, K <= 16): the speaker half's weight / embedding gradients.
 * grad_unpack_slice: dw[co][ci0 + ci][k] (+)= dwf[co*ld + k*kstride + ci] for ci < cn (dw has Ci channels). */
int avc_conv_pack_slice(const float* w, void* out, int dtype, int Co, int Ci, int K, int ci0, int cn, int cpad,
                        int mode, void* stream);
int avc_conv_edge_table(const float* E, int B, int Co, int K, int T, int pad, float* S, void* stream);
int avc_conv_edge_colsum(const void* dy, int dy_dtype, int B, int T, int C, int K, int pad, float* out, void* stream);
int avc_conv_grad_unpack_slice(const float* dwf, long long ld, int kstride, float* dw, int Co, int Ci, int K, int ci0,
                               int cn, int accumulate, void* stream);
/* Discriminator head (factory/Discriminator.py:28-29, dense1 + sigmoid over the flattened C x L
 * channel-major features) on the bin-major activation a [B][L][C]: p[b] = sigmoid(bias +
 * sum a[b][l*C + c] w[c*L + l]) (logit optional); backward through the sigmoid from dL/dp:
 * da [B][L*C], dw [C*L] (dense1.weight layout), dbias [1] (each optional), B <= 1024. */
int avc_disc_dense_fwd(const float* a, const float* w, const float* bias, int B, int L, int C, float* logit, float* p,
                       void* stream);
int avc_disc_dense_bwd(const float* dp, const float* p, const float* a, const float* w, int B, int L, int C, float* da,
                       float* dw, float* dbias, void* stream);
/* dst = convert(src) (n elements). */
int avc_convert(const float* src, void* dst, int dtype, long long n, void* stream);
/* dst[c * ld_dst + r] = convert(src[r][c]) for a row-major [R][C] fp32 matrix (ld_dst = 0:
 * R, a plain transpose; ld_dst > R: a column block of a wider matrix, e.g. the stacked
 * W_ih^T of a bidirectional LSTM). */
int avc_transpose(const float* src, void* dst, int dtype, int R, int C, long long ld_dst, void* stream);
/* out = a + b elementwise (n), e.g. b_ih + b_hh. */
int avc_add(const float* a, const float* b, float* out, long long n, void* stream);

/* Losses of Solver.train (train.py:85-86, 94) and their gradients. */
int avc_mse_loss(const float* a, const float* b, long long n, float* out, void* stream);
int avc_l1_loss(const float* a, const float* b, long long n, float* out, void* stream);
/* g = scale * dL * (mode 0: 2(a-b)/n ; mode 1: sign(a-b)/n) ; dL = *dloss (device) */
int avc_loss_grad(const float* a, const float* b, long long n, const float* dloss, int mode, float* g,
                  float sign, void* stream);
/* The whole loss block of Solver.train in ONE launch (train.py:84-96): with x = x_real (n1),
 * y1 = x_identic, y2 = x_identic_psnt (n1 each), ca = code_real, cb = code_reconst (n2)
 *   out[0] = mean((x - y1)^2), out[1] = mean((x - y2)^2), out[2] = mean|ca - cb|,
 *   out[3] = out[0] + out[1] + lambda_cd * out[2]
 * Block partials are handed over in-kernel and summed in a fixed order by the last-arriving
 * block (deterministic; no zeroing launch).  Replaces 3 avc_mse_loss/avc_l1_loss + the adds.
 * ws: avc_vc_loss_ws() floats of caller-owned scratch (not shared with a concurrent call). */
size_t avc_vc_loss_ws(void);
int avc_vc_loss(const float* x, const float* y1, const float* y2, long long n1, const float* ca, const float* cb,
                long long n2, float lambda_cd, float* out, float* ws, void* stream);
/* Its gradient, one launch: with the upstream gradients d[0..3] of out[0..3] (device scalars,
 * each pointer may be null = 0) and c_id = d3 + d0, c_psnt = d3 + d1, c_cd = lambda_cd*d3 + d2:
 *   g1 = c_id * 2(y1 - x)/n1, g2 = c_psnt * 2(y2 - x)/n1, ga = c_cd * sign(ca - cb)/n2, gb = -ga
 * (any output pointer may be null: not computed). */
int avc_vc_loss_grad(const float* x, const float* y1, const float* y2, long long n1, const float* ca,
                     const float* cb, long long n2, float lambda_cd, const float* d0, const float* d1,
                     const float* d2, const float* d3, float* g1, float* g2, float* ga, float* gb, void* stream);

/* Activation-only passes (Discriminator's conv -> LeakyReLU -> BN order,
 * factory/Discriminator.py:18-29); the backward takes the activation OUTPUT. */
int avc_act_fwd(const float* x, float* y, long long n, int act, void* stream);
int avc_act_bwd(const float* g, const float* yout, float* dx, long long n, int act, void* stream);

/* nn.BCELoss (mean) against a constant target (train_with_discriminator.py:58-61); the
 * gradient optionally chained through the Sigmoid that produced p. */
int avc_bce_loss(const float* p, long long n, float target, float* out, void* stream);
int avc_bce_grad(const float* p, long long n, float target, const float* dloss, float* g,
                 int through_sigmoid, void* stream);

/* MetaFormer blocks (MetaConv.py:8-76, MetaPool.py:7-77, MLPMixer.py:16-92, Norm.py:53-60).
 * GroupNorm(1, C) over each sample's S = L*C contiguous frame-major elements; LayerNorm
 * over rows of D; backward passes write dx and (accumulate != 0: add into) dgamma/dbeta.
 * ws >= avc_norm_ws(rows, C) floats. */
size_t avc_norm_ws(int rows, int C);
int avc_group_norm_fwd(const float* x, int B, long long S, int C, const float* gamma, const float* beta, float eps,
                       float* y, float* mean, float* rstd, void* stream);
int avc_group_norm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                       int B, long long S, int C, float* dx, float* dgamma, float* dbeta, int accumulate, float* ws,
                       void* stream);
int avc_layer_norm_fwd(const float* x, int R, int D, const float* gamma, const float* beta, float eps, float* y,
                       float* mean, float* rstd, void* stream);
int avc_layer_norm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                       int R, int D, float* dx, float* dgamma, float* dbeta, int accumulate, float* ws, void* stream);
/* The same passes with bf16 outputs: y16 / dx16 (nullable) beside or instead of the fp32 y / dx (GEMM operands
 * only ever read in bf16), and for the LayerNorm backward dres (nullable): dx = dres + the norm's gradient -- the
 * residual add after the norm (MLPMixer.py:80-86) folded into the pass, and row_sum (nullable): each row's sum of dx
 * (the token-mixing bias gradient of the transposed layout, summed per patch).  The bf16 / dres forms need C (D) % 4 == 0,
 * D <= 512 and 16-B aligned rows; the LayerNorm backward then computes dx and the parameter sums in ONE pass.
 * avc_group_norm_fwd2's ws (nullable, >= avc_norm_ws(rows, C) floats) lets the per-sample statistics be split over
 * ~1024 blocks (partials merged by Chan's formula) instead of one block per sample. */
int avc_group_norm_fwd2(const float* x, int B, long long S, int C, const float* gamma, const float* beta, float eps,
                        float* y, void* y16, float* mean, float* rstd, float* ws, void* stream);
int avc_layer_norm_fwd2(const float* x, int R, int D, const float* gamma, const float* beta, float eps, float* y,
                        void* y16, float* mean, float* rstd, void* stream);
int avc_layer_norm_bwd2(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                        int R, int D, const float* dres, float* dx, void* dx16, float* row_sum, float* dgamma,
                        float* dbeta, int accumulate, float* ws, void* stream);
/* exact (erf) GELU backward from the GELU input x; the forward is avc_act_fwd(AVC_ACT_GELU). */
int avc_gelu_bwd(const float* g, const float* x, float* dx, long long n, void* stream);
/* y = AvgPool1d(3,1,1,count_include_pad=False)(x) - x along the frames of (B, L, C);
 * backward != 0 maps dy -> dx instead. */
int avc_pool3_mixer(const float* x, float* y, int B, int L, int C, int backward, void* stream);
/* Rearrange('b c (h p1) (w p2) -> b (h w) (p1 p2 c)') of the (C x L) image held frame-major
 * as (B, L, C) (image rows = channels); backward != 0 scatters a patch gradient back. */
int avc_patchify(const float* src, float* dst, int B, int L, int C, int ps, int backward, void* stream);
/* The forward rearrangement written in bf16 (the patches are read only as the embedding GEMM's operand). */
int avc_patchify16(const float* src, void* dst, int B, int L, int C, int ps, void* stream);
/* dst[b] (+)= src[b]^T for B row-major R x C matrices. */
int avc_transpose_batched(const float* src, float* dst, int B, int R, int C, int accumulate, void* stream);
/* The same transpose of an fp32 or bf16 (src_dtype) source into rows of ld >= R elements (r in [R, ld) written 0),
 * writing dst (fp32, nullable) and / or dst16 (bf16 GEMM operand, nullable) in one pass; accumulate needs dst
 * (MLPMixer.py:58-92 operands with the patch count zero-padded to a multiple of 8). */
int avc_transpose_batched2(const void* src, int src_dtype, float* dst, void* dst16, int B, int R, int C, int ld,
                           int accumulate, void* stream);

/* Batched weight packing: every bf16 / re-laid-out copy of the parameters the kernels read
 * (conv Wf / Wd, the conv0 fold's channel-slice packs, LSTM W_ih / W_hh / W_hh^T / W_ih^T,
 * b_ih + b_hh, linear W and W^T) rebuilt after the optimizer step in ONE launch instead of one
 * small kernel per copy.  `ops` and `prefix` (device memory, caller-owned): op i covers UNITS
 * [prefix[i], prefix[i+1]) of the launch, a unit being one 64 x 64 tile of a transpose
 * (ceil(d0 / 64) * ceil(d1 / 64) units), one LDS-staged conv tile (CONV_F with K <= 16: 4 output x
 * 64 input channels, ceil(d0 / 4) * ceil(d1 / 64) units; CONV_D with K <= 8: 32 x 16,
 * ceil(d0 / 32) * ceil(d1 / 16) units) or 4096 elements of anything else (ceil(n / 4096) units);
 * total = prefix[nops]; nops <= 128. */
enum { AVC_PACK_COPY = 0, AVC_PACK_TRANSPOSE = 1, AVC_PACK_CONV_F = 2, AVC_PACK_CONV_D = 3, AVC_PACK_ADD = 4,
       AVC_PACK_CONV_SLICE = 5 };
typedef struct {
  const float* src;   /* the fp32 parameter */
  const float* src2;  /* AVC_PACK_ADD: second addend (b_hh), else null */
  void* dst;
  int kind;           /* AVC_PACK_* */
  int out_dtype;      /* AVC_F32 / AVC_BF16 */
  int d0, d1, d2;     /* COPY / ADD: n = d0.  TRANSPOSE: src [d0][d1] -> dst[c*ld_out + r].
                         CONV_F: W [d0=Co][d1=Ci][d2=K] -> dst[co][k*Ci + ci];
                         CONV_D: -> dst[ci][(K-1-k)*Co + co] (flipped taps: the data-gradient operand);
                         CONV_SLICE: W [d0=Co][d1=Ci][d2=K] -> avc_conv_pack_slice(ci0, cn, cpad, mode) */
  int pad_;
  long long ld_out;   /* TRANSPOSE: destination row stride (>= d0) */
  int ci0, cn, cpad, mode;  /* CONV_SLICE only (ABI 31) */
} avc_pack_op;
int avc_pack_batch(const avc_pack_op* ops, const long long* prefix, int nops, long long total, void* stream);

/* Fused Adam (torch.optim.Adam defaults, train.py:49,99) over a slice of one flat fp32 buffer.
 * state[0] = step count (float), state[1..2] = this step's bias corrections, updated on device
 * (graph-replayable) when `advance` != 0.  A step split over several slices advances on its
 * first slice only; the later slices run on a stream ordered after it. */
int avc_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
             float beta2, float eps, float* state, int advance, void* stream);
/* avc_adam with at most max_blocks 256-thread workgroups (0 = as avc_adam): a slice that runs
 * BESIDE latency-bound kernels (the decoder-slice Adam next to the encoder backward) takes a
 * smaller share of the memory system. */
int avc_adam_blocks(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                    float beta2, float eps, float* state, int advance, int max_blocks, void* stream);

/* AdaIN / speaker-embedding-adjust variants (variants.hip).
 * Whole-tensor moments of x.mean(), x.std() (unbiased) — factory/AutoVC2.py:58-60,
 * factory/Norm.py:84-91 — as out = [mean, std] (device).  ws >= avc_moments_ws() doubles. */
size_t avc_moments_ws(void);
int avc_moments(const float* x, long long n, double* ws, float* out, void* stream);
/* dx = dmean/n + dstd*(x - mean)/((n-1) std) (+ acc); dmean / dstd / acc nullable (device). */
int avc_moments_bwd(const float* x, long long n, const float* mom, const float* dmean, const float* dstd,
                    const float* acc, float* dx, void* stream);
/* AdaIN (Norm.py:84-91): y = (x - mom[0]) / mom[1] * sigma + mu; mom from avc_moments(x). */
int avc_adain_fwd(const float* x, long long n, const float* mom, const float* mu, const float* sigma, float* y,
                  void* stream);
/* AdaIN backward: dx, dmu = sum g, dsigma = sum g*xhat (sums: 2 floats scratch). */
int avc_adain_bwd(const float* g, const float* x, long long n, const float* mom, const float* sigma, double* ws,
                  float* sums, float* dx, float* dmu, float* dsigma, void* stream);
/* out[b][c] (+)= sum_t x[(b*T + t)*ld + c]: the gradient of a speaker embedding broadcast
 * over time into a concat (AutoVC_Adjust.py:178-189 trains it through Adjust). */
int avc_segsum(const float* x, long long ld, int B, int T, int C, float* out, int accumulate, void* stream);
/* scatter = 0: dst[b][c] = src[(b*T + t)*C + c] (nn.LSTM output [:, t, :], Adjust.py:39);
 * scatter = 1: dst (B*T x C) = that step's gradient, zero elsewhere. */
int avc_step_select(const float* src, float* dst, int B, int T, int t, int C, int scatter, void* stream);
/* Row L2 normalisation (Adjust.py:40-42) and its backward dx = (dy - y (y.dy)) / norm. */
int avc_rownorm_fwd(const float* x, int R, int C, float* y, float* norms, void* stream);
int avc_rownorm_bwd(const float* dy, const float* y, const float* norms, int R, int C, float* dx, void* stream);
/* dst (R x Cd, dtype) = the first min(C, Cd) columns of src (rows lds apart), zero-filled to
 * Cd: pads the MLP-Mixer output convolution's NP channels (1849 / 121 patches) to a multiple
 * of 8 for the bf16 LDS-DMA kernels (MLPMixer.py:88-90) and crops its gradients back. */
int avc_pad_cols(const float* src, long long lds, void* dst, int dtype, int R, int C, int Cd, void* stream);
/* dst[r][c] += src[r*lds + c], c < C (dst rows C apart): the zero-padded token-mixing weight
 * gradients (MLPMixer.py:79-80, NP padded to a multiple of 8) cropped into .grad in one pass. */
int avc_crop_add(const float* src, long long lds, float* dst, int R, int C, void* stream);
/* GELU forward (bwd = 0: y = gelu(x)) or backward (bwd = 1: y = g * gelu'(x)) with the
 * fp32 result and/or its bf16 GEMM-operand twin from one pass (y or y16 may be null):
 * the MLP-Mixer hidden activations (MLPMixer.py:9-14) feed only GEMMs and bias sums. */
int avc_gelu_twin(const float* g, const float* x, float* y, void* y16, long long n, int bwd, void* stream);

/* MelGAN vocoder generator, inference (melgan.hip).  Replaces the forward of
 * melgan/modules.py:88-131 Generator (called by melgan/interface.py:47-53 MelVocoder.inverse,
 * util/evaluate.py:98); the convolutions themselves run on avc_gemm.
 * Gather: out[(b*Lo + t)][k*C + c] = act(x[b][src][c]), src = t + k*dil - pad reflected into
 * [0, L) (reflect = 1, nn.ReflectionPad1d, modules.py:76,95,124) or zero outside (reflect = 0);
 * Lo = L + 2 pad - dil (taps - 1); act = 1: LeakyReLU(slope) (modules.py:75,78,108,123).
 * x / out dtypes AVC_F32 / AVC_BF16; C % 4 == 0. */
int avc_mg_gather(const void* x, int x_dtype, int B, int L, int C, int taps, int dil, int pad, int reflect, int act,
                  float slope, void* out, int out_dtype, void* stream);
/* LeakyReLU(slope) of n floats (n % 4 == 0) into out (fp32) and/or out_bf16 (either nullable). */
int avc_mg_act(const float* x, long long n, float slope, float* out, void* out_bf16, void* stream);
/* weight_norm (torch.nn.utils.weight_norm, dim 0: w = g v / ||v||, modules.py:18-23) folded into a
 * GEMM B operand (N x K rows, dtype out_dtype).  stride = 0: Conv1d v [d0 = Co][d1 = Ci][K] ->
 * out [Co][K*Ci] (tap-major, the avc_mg_gather column order).  stride = r: ConvTranspose1d
 * v [d0 = Ci][d1 = Co][K = 2r], padding `pad` (modules.py:101-108) -> polyphase out [r*Co][3*Ci]
 * over the zero-padded 3-tap window (j-1, j, j+1), and bias_out[p*Co + co] = bias[co].
 * norms: d0 floats of scratch (device). */
int avc_mg_wn_pack(const float* v, const float* g, const float* bias, int d0, int d1, int K, int stride, int pad,
                   float* norms, void* out, int out_dtype, float* bias_out, void* stream);
/* The generator's last layer (modules.py:122-126): LeakyReLU(slope), ReflectionPad1d(3),
 * Conv1d(C -> 1, k 7) with w [7][C] (avc_mg_wn_pack, stride 0, fp32) and device bias[1], Tanh:
 * out[b*L + t] = tanh(bias + sum_k,c w[k][c] act(x[b][reflect(t + k - 3)][c])). */
int avc_mg_conv_out(const float* x, int B, int L, int C, int taps, const float* w, const float* bias, float slope,
                    float* out, void* stream);

/* Host-side event helpers (events.hip): one reusable event (no timing, no system-scope fence),
 * recorded on a raw stream handle, and a stream made to wait for the record current at the time of
 * the call -- the step's cross-stream ordering (weight-gradient side stream, comm stream, pack
 * prefetch) without torch.cuda.Event / current_stream() Python costs.  (ABI 30: the hipGraph split
 * entry points of ABI <= 29 are gone; the recorded replay replaced them.) */
int avc_event_create(void** out);
int avc_event_record(void* ev, void* stream);
int avc_stream_wait_event(void* stream, void* ev);


#ifdef __cplusplus
}
#endif
#endif
