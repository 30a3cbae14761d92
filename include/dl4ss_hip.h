/* dl4ss_hip.h -- C ABI of libdl4ss_hip.so, the MI355X (gfx950) hot path of the
 * DL4SS speech-separation training step.
 *
 * Conventions (every entry point):
 *   - returns int: a hipError_t, 0 = success; never throws, never allocates;
 *   - every buffer is a caller-owned device pointer (fp32 unless stated), with
 *     shapes passed as ints; workspaces are caller-allocated;
 *   - `stream` is a hipStream_t passed as void*; the call is asynchronous on it;
 *   - the only library state is per-kernel constant tables; calls on distinct
 *     streams are thread-safe.
 *
 * The reference (shincling/DL4SS) is Python-2 / torch-0.3 code with no native or
 * plugin interface; each entry point below cites the reference call site whose
 * arithmetic it replaces.  The Python boundary (dl4ss_amd.config / predata_* /
 * myNet / test_multi_labels_speech / bss_test) is what binds them; see
 * INTEGRATION.md.
 */
#ifndef DL4SS_HIP_H
#define DL4SS_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- STFT / iSTFT ------------------------------------------------------ */
enum {
  DL4SS_STFT_COMPLEX = 1, /* write X (n_sig, T, F, 2) [re, im]                     */
  DL4SS_STFT_MAG = 2,     /* write |X| (n_sig, T, F)                              */
  DL4SS_STFT_LOGMAG = 4,  /* write log(|X| + 2.22e-16) into `mag` instead         */
  DL4SS_STFT_CONJ = 8     /* librosa <= 0.5.x convention (conjugated spectrum)    */
};

/* Framed STFT, n_fft = 256, hop = 128, periodic Hann, centre / reflect padding;
 * T = 1 + n_samples / 128, F = 129.  x: (n_sig, n_samples).
 * Replaces np.transpose(librosa.core.spectrum.stft(y, 256, 128)) and its abs /
 * log-abs at Torch_multi/predata_multiAims_dB.py:180,194,209,214 and
 * TDAA_beta/predata_fromList_cRM_123.py:215-255 (convert2 layout = [re, im]). */
int dl4ss_stft_fwd(const float* x, long long n_sig, int n_samples, int n_fft, int hop, int flags,
                   float* X_c64, float* mag, void* stream);
/* dl4ss_stft_fwd that also writes bf16 (round-to-nearest-even) copies of the magnitudes (or log
 * magnitudes) of the first n_sig_bf16 signals: mag_bf16[(sig * T + t) * ld_bf16 + f], ld_bf16 >= 129,
 * columns >= 129 untouched -- the bf16 recurrence's first-layer input rows without a conversion pass.
 * mag_bf16 NULL: dl4ss_stft_fwd. */
int dl4ss_stft_fwd_ex(const float* x, long long n_sig, int n_samples, int n_fft, int hop, int flags, float* X_c64,
                      float* mag, void* mag_bf16, long long ld_bf16, long long n_sig_bf16, void* stream);

/* Overlap-add inverse STFT: S (n_sig, T, 129, 2) -> y (n_sig, 128 * (T - 1)).
 * Replaces librosa.core.spectrum.istft(S.T, 128) at
 * TDAA_beta/main_run_sstune_EvalVer.py:64-65 and main_run_sstune_cRM_EvalVer.py:98-99.
 * flags: DL4SS_STFT_CONJ only. */
int dl4ss_istft(const float* S_c64, long long n_sig, int T, int n_fft, int hop, int flags, float* y,
                void* stream);
/* Mask apply + iSTFT in one pass (eval output path): signal s (n_sig of them) is
 * synthesised from mixture s / k_per_mix.  mode 0: aux = masked magnitude (n_sig,T,129)
 * with the mixture phase (EvalVer.py:56-65); mode 1: aux = complex ratio mask
 * (n_sig,T,129,2) times the mixture spectrum (cRM_EvalVer.py:96-99,720-728).
 * conj: the mixture spectrum is stored conjugated (librosa <= 0.5). */
int dl4ss_istft_apply(const float* X_mix_c64, const float* aux, long long n_sig, int k_per_mix, int T, int mode,
                      int conj, float* y, void* stream);

/* ---- R1 preprocessing / mixing ----------------------------------------- */
/* raw (B, K, N) -> out_src (B, K, N): each source x -> (x - mean) / max|x - mean| * gain;
 * out_mix (B, N): their sum.  stats_ws: 32*B*K floats of workspace (16-B aligned; K <= 16).
 * Replaces Torch_multi/predata_multiAims_dB.py:156-197 (and the _3dB /
 * fromList_cRM_123 gain variants: gains are computed by the caller). */
int dl4ss_mix_sources(const float* raw, const float* gains, int B, int K, int N, float* stats_ws, float* out_src,
                      float* out_mix, void* stream);
/* As dl4ss_mix_sources, with per-source valid lengths (B*K int32; NULL = N): mean and peak
 * over the first lengths[s] samples, zero beyond -- a list-file wav shorter than MAX_LEN
 * (TDAA_beta/predata_fromList_cRM_123.py:186-201: crop, normalise, then zero-pad). */
int dl4ss_mix_sources_ex(const float* raw, const int* lengths, const float* gains, int B, int K, int N,
                         float* stats_ws, float* out_src, float* out_mix, void* stream);
/* As dl4ss_mix_sources_ex, plus the train-split augmentation of the list loaders: source s is
 * rotated by shifts[s] (B*K int32; NULL = none; taken modulo the source's length) after the
 * normalisation and before the zero-padding -- np.append(x[s:], x[:s]) over the source's own
 * length (TDAA_beta/predata_fromList.py:150-151, predata_fromList_cRM_123.py:198-200). */
int dl4ss_mix_sources_rot(const float* raw, const int* lengths, const int* shifts, const float* gains, int B, int K,
                          int N, float* stats_ws, float* out_src, float* out_mix, void* stream);

/* ---- dense contractions (MFMA) ------------------------------------------ */
enum { DL4SS_EPI_NONE = 0, DL4SS_EPI_TANH = 1, DL4SS_EPI_TANH_BF16 = 2 /* tanh, C written as bf16 */,
       DL4SS_EPI_SPLIT_SLABS = 3 /* dl4ss_gemm_bf16_gl split-K only: the S fp32 slabs stay in ws
                                    ([S][batch][M][N], S = dl4ss_gemm_bf16_gl_ws_bytes / (batch M N 4)),
                                    no combine, C not written: their consumer sums them (the
                                    BPTT's DL4SS_RNN_DOUT_SLABS) */ };
enum { DL4SS_PREC_F32 = 0, DL4SS_PREC_BF16 = 1 };
/* C = op(A) op(B) (+ bias[N]) (tanh) (+ beta C); row-major, leading dims in elements.
 * transA: A stored K x M (else M x K); transB: B stored N x K (else K x N).
 * splitk > 1: C += op(A) op(B) with fp32 atomics (epilogue none, beta 1).
 * Replaces the cuDNN input projection inside nn.LSTM/nn.GRU (EvalVer.py:282-293),
 * nn.Linear(600, 6450) + tanh (EvalVer.py:290,298-299) and their autograd GEMMs. */
int dl4ss_gemm(int transA, int transB, int M, int N, int K, const float* A, long long lda, const float* B,
               long long ldb, float* C, long long ldc, const float* bias, int epilogue, float beta, int precision,
               int splitk, void* stream);

/* y[i] = bf16(x[i]) (round to nearest even), n elements; x 16-B aligned, y 8-B aligned. */
int dl4ss_f32_to_bf16(const float* x, void* y, long long n, void* stream);
/* bf16-operand GEMM with LDS-DMA staging (gemm_gl.hip): every GEMM of the bf16 step.  A and B
 * are raw bf16 words already rounded by their producers, C fp32 (or bf16 with the tanh-bf16
 * epilogue); layout, bias and epilogue as dl4ss_gemm.  Strided batch: member i uses
 * A + i*strideA, B + i*strideB, C + i*strideC (elements).  Deterministic split-K (fp32
 * slabs in ws, dl4ss_gemm_bf16_gl_ws_bytes bytes, then a fixed-order reduce; EPI_NONE only).
 * Needs lda / ldb / strides % 8 == 0, 16-B aligned A / B, for a k-major operand a row stride
 * >= its row count rounded up to 8, and for a k-contiguous one a row stride >= K rounded up
 * to 8 with zeros in that padding; hipErrorInvalidValue otherwise. */
long long dl4ss_gemm_bf16_gl_ws_bytes(int M, int N, int K, int splitk, int batch);
/* Tuning knob: tile configuration of dl4ss_gemm_bf16_gl (0 = per shape, 1 = 128 x 128 double
 * buffer, 2 = 256 x 128 three stages, 3 = 128 x 128 three stages, 4 / 5 = 256 x 256 ping-pong,
 * 6 / 7 = 128 x 128 with five / four 32-deep k-tile stages). */
int dl4ss_gemm_gl_set_config(int cfg);
int dl4ss_gemm_bf16_gl(int transA, int transB, int M, int N, int K, const void* A, long long lda, const void* B,
                       long long ldb, float* C, long long ldc, const float* bias, int epilogue, float beta,
                       int splitk, int batch, long long strideA, long long strideB, long long strideC, void* ws,
                       long long ws_bytes, void* stream);
/* Grouped form: n <= 16 independent problems C_i = op(A_i) op(B_i) + beta_i C_i (same transA /
 * transB for all, no bias, EPI_NONE, per-problem split-K factor) as ONE GEMM launch plus one
 * split-K combine launch; each C_i bitwise equal to dl4ss_gemm_bf16_gl with the same split factor.
 * The backward's weight gradients (dW_lin, every layer's dW_ih and both directions' dW_hh), which
 * the reference accumulates in loss.backward() (TDAA_beta/main_run_sstune_EvalVer.py:673).  The
 * arrays are host arrays of n entries; ws holds dl4ss_gemm_bf16_gl_grouped_ws_bytes bytes. */
long long dl4ss_gemm_bf16_gl_grouped_ws_bytes(int n, const int* M, const int* N, const int* K, const int* splitk);
int dl4ss_gemm_bf16_gl_grouped(int n, int transA, int transB, const int* M, const int* N, const int* K,
                               const void* const* A, const long long* lda, const void* const* B, const long long* ldb,
                               float* const* C, const long long* ldc, const float* beta, const int* splitk, void* ws,
                               long long ws_bytes, void* stream);
/* The grouped launch in its persistent form: `grid` workgroups walk the tiles (grid <= 0: one per
 * tile); cfg 1 = 128 x 128 double buffer, 2 = 256 x 128 three stages (one workgroup per CU);
 * one_per_cu pads cfg 1's LDS to one workgroup per CU.  For a side stream on the CUs the persistent
 * recurrence leaves free (its co-residency budget, dl4ss_birnn_plan_info).  rowsum (NULL or n
 * entries, each NULL or M_i floats): rowsum_i[m] = beta_i rowsum_i[m] + sum_k op(A_i)(m, k), for
 * unsplit problems whose operands are both k-major (transA, !transB) -- the Linear's bias gradient
 * sum_rows dPre (EvalVer.py:290, loss.backward() at :673) beside dW_lin. */
int dl4ss_gemm_bf16_gl_grouped_ex(int n, int transA, int transB, const int* M, const int* N, const int* K,
                                  const void* const* A, const long long* lda, const void* const* B,
                                  const long long* ldb, float* const* C, const long long* ldc, const float* beta,
                                  const int* splitk, void* ws, long long ws_bytes, int grid, int cfg, int one_per_cu,
                                  float* const* rowsum, void* stream);
/* Split-precision operand image: x = hi + lo (hi = bf16(x), lo = bf16(x - hi)); segment s of each
 * row of y (width segw >= cols, zero-padded; s < nseg <= 8) holds hi, or lo when bit s of pattern
 * is set; zeros up to ldy.  [x_hi | x_lo | x_hi] against weights [w_hi | w_hi | w_lo] makes one bf16
 * GEMM with K' = 3 K fp32-accurate (~2^-16): the split forward GEMMs of the "bf16s" step, whose
 * masked magnitude meets the 1e-3 bar on the BiGRU nets (EvalVer.py:282-299 nn.LSTM / Linear). */
int dl4ss_f32_to_bf16_hilo(const float* x, long long ldx, int rows, int cols, void* y, long long ldy, int segw,
                           int nseg, unsigned pattern, void* stream);
/* 2-D form with row padding: y[r*ldy + c] = bf16(x[r*ldx + c]) (c < cols), 0 up to ldy. */
int dl4ss_f32_to_bf16_2d(const float* x, long long ldx, int rows, int cols, void* y, long long ldy, void* stream);
/* out[n] += sum_m A[m*lda + n] for a bf16 matrix A (bias gradient from bf16 dPre). */
int dl4ss_colsum_bf16(const void* A, long long lda, int M, int N, float* out, void* stream);
/* Deterministic form: per-256-row-block partials in part (dl4ss_colsum_bf16_part_bytes(M, N)
 * bytes), then a fixed-order reduce into out (bitwise reproducible bias gradients). */
long long dl4ss_colsum_bf16_part_bytes(int M, int N);
int dl4ss_colsum_bf16_det(const void* A, long long lda, int M, int N, float* out, float* part, long long part_bytes,
                          void* stream);
/* dl4ss_colsum_bf16_det with out = beta out + sums (beta 0: out written, not read; beta 1 bitwise _det). */
int dl4ss_colsum_bf16_det_ex(const void* A, long long lda, int M, int N, float* out, float* part,
                             long long part_bytes, float beta, void* stream);
/* n (<= 8) dl4ss_f32_to_bf16_2d conversions in one launch (host arrays of per-segment
 * arguments): the step's bf16 weight copies (W_ih of every layer, the Linear). */
int dl4ss_f32_to_bf16_2d_multi(int n, const float* const* x, const long long* ldx, const int* rows, const int* cols,
                               void* const* y, const long long* ldy, void* stream);

/* ---- persistent bidirectional LSTM / GRU recurrence ---------------------- */
enum { DL4SS_CELL_LSTM = 0, DL4SS_CELL_GRU = 1 };
/* Workspace (bytes) needed by dl4ss_birnn_fwd / _bwd for (cell, B, H); -1 if unsupported: the
 * hand-off granules, then (bf16 BPTT with fused bias gradients) the per-row bias partials that
 * a fixed-order reduce adds into db_ih / db_hh, so the gradients are bitwise reproducible.
 * The launchers zero the workspace themselves (hipMemsetAsync) unless `precision` carries
 * DL4SS_RNN_WS_ZEROED: the caller then guarantees it is zero (e.g. one fill per training
 * step over separate workspaces for every layer and pass) -- or exactly as the previous launch
 * on it left it, when that launch had the same (cell, B, T, H), T >= 4, and completed without a
 * timeout: its stale tags cannot match, and the packed kernels reset their start counters and
 * placement granules themselves (the training step zeroes its workspaces once). */
#define DL4SS_RNN_WS_ZEROED 0x100
/* precision flag of dl4ss_birnn_bwd_ex: dGh_bf16 is laid out (B, T, 2, pad8(NGATE*H)) -- each
 * direction's columns start 16-B aligned (the GRU's 900 gate rows -> 904), so both directions'
 * dW_hh run as one LDS-DMA batched GEMM (gemm_gl).  The unpadded default is (B, T, 2, NGATE*H). */
#define DL4SS_RNN_DGH_PAD8 0x200
/* precision flag of dl4ss_birnn_bwd_ex (bf16 BPTT with fused bias gradients): leave the per-row
 * bias partials in the workspace; dl4ss_birnn_bias_reduce adds those of n launches (n <= 8, their
 * workspaces and bias gradient pointers as host arrays) into db_ih / db_hh in ONE launch, in the
 * same fixed row order (bitwise the per-launch reduce). */
#define DL4SS_RNN_DEFER_BIAS 0x400
/* precision field of dl4ss_birnn_bwd_ex (bits 12-13: S - 1): dOut is not one (B, T, 2H) array but the S
 * (2..4) fp32 split-K slabs dl4ss_gemm_bf16_gl leaves with DL4SS_EPI_SPLIT_SLABS, slab z at dOut + z B T 2H;
 * the BPTT sums them per element in slab order from zero (((0 + s0) + s1) + ...), bitwise the combine
 * launch it replaces.  Packed bf16 BPTT at batch chunks of 4 only (hipErrorInvalidValue otherwise). */
#define DL4SS_RNN_DOUT_SLABS(S) ((((S) - 1) & 3) << 12)
int dl4ss_birnn_bias_reduce(int cell, int B, int H, int n, void* const* workspaces, float* const* db_ih,
                            float* const* db_hh, void* stream);
/* dl4ss_birnn_bias_reduce with db = beta db + sums: beta 0 writes db_ih / db_hh without reading them
 * (the training step then needs no zeroed gradient buffer; beta 1 is bitwise the += form). */
int dl4ss_birnn_bias_reduce_ex(int cell, int B, int H, int n, void* const* workspaces, float* const* db_ih,
                               float* const* db_hh, float beta, void* stream);
long long dl4ss_birnn_workspace_bytes(int cell, int B, int H);
/* The persistent recurrence's plan under a co-residency budget: every workgroup of a launch
 * (2 directions x nchunk batch chunks x NG units groups) must be resident at once, so the
 * batch chunk BC is the smallest in {1, 2, 4, 8} with 2 * nchunk * NG <= max_wg (max_wg <= 0:
 * the current device's CUs minus 1/16, 240 on a full MI355X; env DL4SS_RNN_MAX_WG overrides).
 * info[5] = {BC, NG, J, nchunk, grid}.  Host-only when max_wg > 0.  0, or
 * hipErrorInvalidValue when no plan fits.  Every launch re-checks the grid against the CU
 * count x the kernel's occupancy and fails with hipErrorCooperativeLaunchTooLarge (720)
 * instead of spinning to the hand-off timeout. */
int dl4ss_birnn_plan_info(int cell, int B, int H, int precision, int max_wg, int* info);
/* Test hook: polls before a recurrence hand-off times out (0 = default, ~1 s of polling). */
void dl4ss_debug_set_spin_limit(unsigned limit);
/* Test hook: 1 = the packed (bf16) recurrence kernels write every hand-off granule through
 * (`sc1`), as for a group whose workgroups span XCDs; 0 = by the placement found at launch. */
void dl4ss_debug_set_place_force(int force);
/* Test hook: > 0 replaces the device's co-residency budget (workgroups per persistent launch) in
 * every later recurrence plan -- e.g. 120 gives the B = 32, H = 300 nets batch chunks of 8, the
 * plan of B >= 33 on a full MI355X; 0 restores the default. */
void dl4ss_debug_set_rnn_max_wg(int max_wg);
/* One layer, both directions: G (B,T,2,NG*H) = X W_ih^T + b_ih (NG = 4 LSTM / 3 GRU),
 * W_hh (2, NG*H, H), b_hh (2, NG*H) -> out (B,T,2H) [fwd | reverse], hprev (B,T,2H)
 * (h_{t-1} per step), act (B,T,2,4H) gate activations, cs (B,T,2,H) LSTM cells.  act is
 * gate-major (B,T,2,4H) except where both packed bf16 kernels run the plan at batch chunks >= 4
 * (every C2 / C4 step at B = 32): there it is cell-major (B,T,2,H,4), one 16-B record per cell,
 * written by the forward and read by dl4ss_birnn_bwd[_ex] of the same precision and shape.
 * precision 0: exact fp32 recurrent matvec (VALU); 1: bf16 operands on MFMA with fp32
 * accumulate (cell state, gates and all outputs stay fp32).  A precision-0 plan that does not
 * fit the co-residency budget at B (H = 600: 50 workgroups per group, B <= 16 on a full part)
 * runs as consecutive near-equal sub-batch launches on the same workspace (rows never interact;
 * dl4ss_birnn_workspace_bytes sizes the workspace for the sub-batch plan).
 * *status != 0 after the call means a hand-off timed out (results invalid).
 * Replaces the cuDNN recurrence of nn.LSTM / nn.GRU(batch_first, bidirectional)
 * at TDAA_beta/main_run_sstune_EvalVer.py:282-293, Torch_multi/main_run.py:263-273. */
int dl4ss_birnn_fwd(int cell, int precision, int B, int T, int H, const float* G, const float* W_hh,
                    const float* b_hh, float* out, float* hprev, float* act, float* cs, void* workspace,
                    long long ws_bytes, int* status, void* stream);
/* dl4ss_birnn_fwd with bf16 extras (precision 1, packed-hand-off kernel only):
 * out_bf16 (B*T rows of pad8(2H): [fwd | reverse] adjacent) receives bf16(h), the next
 * layer's / the Linear's GEMM operand; hprev_bf16 (B*T rows of 2 pad8(H): each direction's
 * block 16-B aligned) receives bf16(h_{t-1}), the W_hh weight-gradient operand
 * (pad8(n) = n rounded up to a multiple of 8; pads are not written).  hprev may be NULL
 * for LSTM (only the GRU BPTT reads the fp32 h_{t-1}). */
int dl4ss_birnn_fwd_ex(int cell, int precision, int B, int T, int H, const float* G, const float* W_hh,
                       const float* b_hh, float* out, float* hprev, float* act, float* cs, void* out_bf16,
                       void* hprev_bf16, void* workspace, long long ws_bytes, int* status, void* stream);
/* dl4ss_birnn_fwd_ex with, in the packed kernel (precision 1), the fp32 output optional (out NULL when
 * out_bf16 is given) and h_mean (B, 2H) = the mean over t of the output, summed in step order by each
 * unit's cell lane (NULL: none) -- as dl4ss_birnn_fwd_xw_ex, for the unfused projection. */
int dl4ss_birnn_fwd_mean(int cell, int precision, int B, int T, int H, const float* G, const float* W_hh,
                         const float* b_hh, float* out, float* hprev, float* act, float* cs, void* out_bf16,
                         void* hprev_bf16, float* h_mean, void* workspace, long long ws_bytes, int* status, void* stream);
/* dl4ss_birnn_fwd_ex with the input projection fused into the recurrence (bf16 packed kernel):
 * no G buffer and no separate GEMM -- every workgroup forms x_t W_ih^T + b_ih of its own gate rows
 * with MFMAs while the previous step's hand-off travels.  x_bf16 (B*T, ldx) bf16 layer input rows
 * (read in 16-B chunks: the row padding up to the next multiple of 8 must be finite, e.g. zero), W_ih_bf16 (2*NGATE*H, ldw) bf16, b_ih (2, NGATE*H); ldx, ldw multiples of 8,
 * x_bf16 and W_ih_bf16 16-B aligned.  Bitwise equal to gemm_gl (G = x W_ih^T + b_ih) followed by
 * dl4ss_birnn_fwd_ex.  Replaces the same reference lines as dl4ss_birnn_fwd (the cuDNN LSTM / GRU of
 * TDAA_beta/main_run_sstune_EvalVer.py:282-293, whose input projection is part of that call).
 * ws_zeroed: the caller already zeroed the hand-off area. */
int dl4ss_birnn_fwd_xw(int cell, int B, int T, int H, const void* x_bf16, int Kin, long long ldx,
                       const void* W_ih_bf16, long long ldw, const float* b_ih, const float* W_hh,
                       const float* b_hh, float* out, float* hprev, float* act, float* cs, void* out_bf16,
                       void* hprev_bf16, void* workspace, long long ws_bytes, int* status, void* stream,
                       int ws_zeroed);
/* dl4ss_birnn_fwd_xw with the fp32 layer output optional (out may be NULL when out_bf16 is not)
 * and h_mean (B, 2H) (NULL: none) = the mean over t of the layer output, each (b, direction, unit)
 * summed in step order by the unit's own cell lane -- the time mean of the last layer that ADDJUST
 * (EvalVer.py:363-377) reads, without a pass over the output. */
int dl4ss_birnn_fwd_xw_ex(int cell, int B, int T, int H, const void* x_bf16, int Kin, long long ldx,
                          const void* W_ih_bf16, long long ldw, const float* b_ih, const float* W_hh, const float* b_hh,
                          float* out, float* hprev, float* act, float* cs, void* out_bf16, void* hprev_bf16,
                          float* h_mean, void* workspace, long long ws_bytes, int* status, void* stream, int ws_zeroed);
/* 1 when dl4ss_birnn_fwd_xw applies to (cell, B, T, H, Kin) (the packed bf16 plan exists, Kin <= 640);
 * host-only. */
int dl4ss_birnn_fwd_xw_supported(int cell, int B, int T, int H, int Kin);
/* BPTT of one layer: dOut (B,T,2H) (+ dOut_bcast (B,2H) at every t, may be NULL) ->
 * dG (B,T,2,NG*H) grad of the input projection (pre-activation) and, for GRU, dGh
 * grad of W_hh h + b_hh (for LSTM they coincide; dGh may be NULL). */
int dl4ss_birnn_bwd(int cell, int precision, int B, int T, int H, const float* dOut, const float* dOut_bcast,
                    const float* W_hh, const float* act, const float* cs, const float* hprev, float* dG, float* dGh, void* workspace,
                    long long ws_bytes, int* status, void* stream);

/* dl4ss_birnn_bwd with bf16 extras (precision 1, packed-hand-off kernel only): dG_bf16 /
 * dGh_bf16 (B,T,2,NG*H) receive bf16 copies (the weight-gradient / dX GEMM operands),
 * dG / dGh may then be NULL, and db_ih / db_hh (2, NG*H) are ACCUMULATED with the sums
 * over (b,t) of dG / dGh (the bias gradients; fp32 atomics, one per cell and gate). */
int dl4ss_birnn_bwd_ex(int cell, int precision, int B, int T, int H, const float* dOut, const float* dOut_bcast,
                       const float* W_hh, const float* act, const float* cs, const float* hprev, float* dG,
                       float* dGh, void* dG_bf16, void* dGh_bf16, float* db_ih, float* db_hh, void* workspace,
                       long long ws_bytes, int* status, void* stream);

/* ---- speaker-query mask attention + loss (fused forward/backward) -------- */
/* Blocks per utterance used by the partial-sum buffers. */
int dl4ss_attn_nblk(int T, int F);
/* pass 0 (COST): costs (+ optional mask / pred outputs); pass 1 (GRAD): also
 * dPre (B,T*F,E) = dL/d(h W_lin^T + b) (may alias V: in-place) and dq partials.
 * V (B,T*F,E) = tanh Linear output; q (B,K,QW), QW = E (magnitude) or 2E (cRM).
 * X: magnitude (b*x_bstride + row) or complex [re,im] pairs; Y target k of b at
 * b*y_bstride + k*y_kstride (+ row).  perm (B,K) target per channel (NULL = label
 * order).  s1/s2 scale the MSE and sum-to-one terms.  part_loss (B,nblk,K*K+1),
 * part_dq (B,nblk,K,QW).
 * Replaces EvalVer.py:615-666 (expand + baddbmm + sigmoid + MSE + sum loss) and
 * main_run_sstune_cRM_EvalVer.py:259-271,688,720-743 (cRM branch). */
int dl4ss_mask_attn_loss(int pass, int crm, int B, int K, int T, int F, int E, const float* V, const float* q,
                         const float* X, long long x_bstride, const float* Y, long long y_bstride,
                         long long y_kstride, const int* perm, float s1, float s2, float* dPre, float* part_loss,
                         float* part_dq, float* mask_out, float* pred_out, void* stream);
/* dl4ss_mask_attn_loss with a bf16 GRAD output: dPre_bf16 row (b*T + t) holds the F*E
 * values of frame t at stride dpre_bf16_ld (even, >= F*E: 16-B rows for the Linear's
 * backward GEMMs); dPre may then be NULL.  A non-NULL dPre_bf16 on the magnitude path (also
 * given to the COST pass, which does not write it) selects the quad-per-row kernel for the fp32
 * V as well -- logits summed as quad partials, as the bf16-V kernel does; NULL keeps the
 * row-per-lane kernel of the fp32 parity step. */
int dl4ss_mask_attn_loss_ex(int pass, int crm, int B, int K, int T, int F, int E, const float* V, const float* q,
                            const float* X, long long x_bstride, const float* Y, long long y_bstride,
                            long long y_kstride, const int* perm, float s1, float s2, float* dPre, void* dPre_bf16,
                            long long dpre_bf16_ld, float* part_loss, float* part_dq, float* mask_out,
                            float* pred_out, void* stream);
/* dl4ss_mask_attn_loss_ex with V in bf16 (V_bf16: (B, T*F, E) raw 16-bit words, 4-B aligned):
 * the bf16 path's Linear writes V = tanh(h W^T + b) directly in bf16 (gemm EPI_TANH_BF16),
 * halving the bytes of the Linear's output and of both attention passes' V reads. */
int dl4ss_mask_attn_loss_bf16v(int pass, int crm, int B, int K, int T, int F, int E, const void* V_bf16, const float* q,
                               const float* X, long long x_bstride, const float* Y, long long y_bstride,
                               long long y_kstride, const int* perm, float s1, float s2, float* dPre, void* dPre_bf16,
                               long long dpre_bf16_ld, float* part_loss, float* part_dq, float* mask_out,
                               float* pred_out, void* stream);
/* PIT: per utterance the lowest-index permutation minimising the summed costs. */
int dl4ss_pit_select(const float* part_loss, int B, int K, int nblk, int* perm, void* stream);
/* loss_out[3] = {total, MSE term, weighted sum-to-one term}; dq = sum of partials. */
int dl4ss_loss_finalize(const float* part_loss, int B, int K, int nblk, const int* perm, float s1, float s2,
                        float* loss_out, const float* part_dq, int qw, float* dq, void* stream);

/* ---- speaker queries, reductions, optimizer ------------------------------ */
/* q[b,k] = Emb[idx[b,k]] (+ W_adj [mean_t h[b]; Emb[idx[b,k]]]); h (B,T,D).
 * SPEECH_EMBEDDING + ADDJUST: EvalVer.py:348-377,606-608. w_adj may be NULL; an idx of -1 (no speaker) gives a zero query.
 * mean_out (B,D) receives mean_t h; with h NULL it is instead READ as that mean, formed by the
 * recurrence (dl4ss_birnn_fwd_xw_ex h_mean). */
int dl4ss_query_fwd(const float* h, int B, int T, int D, const int* idx, const float* emb, const float* w_adj, int K,
                    int W, float* q, float* mean_out, void* stream);
/* d_emb (+=, scatter), d_wadj (+=), dh_bcast (B,D) = W_m^T sum_k dq / T. */
int dl4ss_query_bwd(const float* dq, int B, int T, int D, const int* idx, const float* emb, const float* w_adj,
                    const float* mean, int K, int W, float* d_emb, float* d_wadj, float* dh_bcast, void* stream);
/* dl4ss_query_bwd with d_emb / d_wadj = beta (old) + this step's: beta 0 writes them without reading --
 * every d_wadj element, the embedding rows the batch's speakers own, and zeros in the other rows of
 * the n_labels-row d_emb (the step's gradient buffer then needs no zeroing pass); beta 1 is bitwise
 * dl4ss_query_bwd (n_labels unused). */
int dl4ss_query_bwd_ex(const float* dq, int B, int T, int D, const int* idx, const float* emb, const float* w_adj,
                       const float* mean, int K, int W, float* d_emb, float* d_wadj, float* dh_bcast, int n_labels,
                       float beta, void* stream);
/* out[n] += sum_m A[m*lda + n] (bias gradients). */
int dl4ss_colsum(const float* A, long long lda, int M, int N, float* out, void* stream);
/* torch.optim.Adam step on flat fp32 buffers (EvalVer.py:538-544). */
int dl4ss_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
               float eps, int step, void* stream);
/* dl4ss_adam that refuses a step computed from a timed-out recurrence: when status[0] != 0
 * (a BiRNN hand-off of this step timed out) no parameter or moment changes and loss[0] (if not
 * NULL) is set to NaN, so the step's loss read by the caller reports it.  status is ONE int,
 * only read. */
int dl4ss_adam_guarded(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                       float beta2, float eps, int step, int* status, float* loss, void* stream);
/* dl4ss_adam_guarded that also refuses when *dp_flag != 0: the data-parallel form, where
 * dp_flag is the slot behind the flat gradient that dl4ss_status_flag filled from each rank's
 * status and the gradient all-reduce combined, so every rank refuses the same steps.  Here
 * status points at 2 ints: {hand-off word, refused-update count}; the count is incremented on
 * every refusal (the host rolls its Adam step count back by it). */
int dl4ss_adam_guarded_dp(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                          float beta2, float eps, int step, int* status, const float* dp_flag, float* loss,
                          void* stream);
/* dl4ss_adam_guarded_dp on g * gscale: the data-parallel step takes the gradient all-reduced with
 * SUM and applies the 1 / world_size of the mean here (no separate pass over the buffer; gscale =
 * 1 is bitwise the unscaled step).  Replaces optimizer.step() at EvalVer.py:673-675 under DP. */
int dl4ss_adam_guarded_dp_scaled(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                                 float beta2, float eps, int step, int* status, const float* dp_flag, float gscale,
                                 float* loss, void* stream);
/* dl4ss_adam_guarded_dp_scaled that also writes bf16 (round-to-nearest-even) shadow copies of the
 * updated parameters: segment s < nseg (<= 8) maps the flat range [seg_off[s], + rows*cols) row-major
 * onto seg_y[s] (row stride seg_ldy[s] >= cols; columns >= cols untouched).  The bf16 step's weight
 * operands (W_ih of every layer, the Linear) then need no conversion launch before the next forward:
 * bitwise dl4ss_f32_to_bf16_2d_multi of the new parameters; a refused update leaves both untouched. */
int dl4ss_adam_guarded_dp_scaled_bf16(float* p, const float* g, float* m, float* v, long long n, float lr,
                                      float beta1, float beta2, float eps, int step, int* status, const float* dp_flag,
                                      float gscale, float* loss, int nseg, const long long* seg_off,
                                      const int* seg_rows, const int* seg_cols, void* const* seg_y,
                                      const long long* seg_ldy, void* stream);
/* flag[0] = status[0] != 0 ? 1 : 0 (one float, written in front of the flat gradient before its all-reduce). */
int dl4ss_status_flag(const int* status, float* flag, void* stream);

/* ---- kernels behind the reference-API nn.Modules (dl4ss_amd/compat/myNet.py) ---- */
/* dpre = dv * (1 - v^2): backward of MIX_SPEECH's tanh(Linear) (EvalVer.py:298-299). */
int dl4ss_tanh_bwd(const float* v, const float* dv, float* dpre, long long n, void* stream);
/* Row blocks of the ATTENTION 'dot' backward (size of part_dq: Bq * nblk * E). */
int dl4ss_attn_dot_nblk(int R);
/* ATTENTION 'dot': mask (Bq,R) = act(V (Bq,R,E) . q (Bq, row stride q_stride)); act 0 =
 * sigmoid (EvalVer.py:216-226), 1 = 10 tanh, the cRM branch per query half (cRM:259-271). */
int dl4ss_attn_dot_fwd(const float* V, const float* q, int q_stride, int Bq, int R, int E, int act, float* mask,
                       void* stream);
/* Its backward: dV += dE q (may be NULL; accumulates, so both cRM halves add) and
 * dq (Bq,E) = sum_r dE V (deterministic partial sums, part_dq: Bq*nblk*E). */
int dl4ss_attn_dot_bwd(const float* V, const float* q, int q_stride, const float* mask, const float* dmask, int Bq,
                       int R, int E, int act, float* dV, float* part_dq, float* dq, void* stream);
/* top_k_mask (EvalVer.py:390-405, main_run.py:340-355): mask (B,N) of the first
 * min(top_k, #{p > alpha}) entries in descending order (ties: lower index first);
 * idx (B,top_k) the selected ids ascending (-1 padded), count (B); idx/count may be NULL. */
int dl4ss_top_k_mask(const float* prob, int B, int N, float alpha, int top_k, float* mask, int* idx, int* count,
                     void* stream);
/* dl4ss_attn_dot_fwd with an output row stride: mask[b * mask_stride + r] (K queries of one
 * V (B,R,E) write a (B,K,R) mask without expanding V, the 414 MB copy of EvalVer.py:615-617). */
int dl4ss_attn_dot_fwd_ex(const float* V, const float* q, int q_stride, int Bq, int R, int E, int act, float* mask,
                          long long mask_stride, void* stream);

/* ---- recursive extraction / speaker classifier ---- */
/* Speaker choice of one recursion step (Torch_multi/main_run_multi_selfSS_recuReal_GRID.py:
 * 227-244 top_k_mask with sort_index, 391-404 the seen-speaker filter), per row b:
 * prob = sigmoid(logits) (GRID.py:197; may be NULL), sort_index (B,top_k) ids by descending
 * prob (ties: lower id; -1 beyond N; may be NULL), chosen (B) = first id of sort_index not in
 * prev (n_prev,B) (the ids chosen at earlier steps, -1 = none) if any prob > alpha, else -1
 * (may be NULL).  top_k <= 64, N <= 8192. */
int dl4ss_classifier_select(const float* logits, int B, int N, float alpha, int top_k, const int* prev, int n_prev,
                            float* prob, int* sort_index, int* chosen, void* stream);
/* pred = mask * x and resid = (1 - mask) * x, n elements (GRID.py:433-434 predict_multi_map,
 * GRID.py:444 the residual spectrogram); pred or resid may be NULL. */
int dl4ss_mask_split(const float* mask, const float* x, long long n, float* pred, float* resid, void* stream);
/* mean over t of h (B,T,D) -> (B,D): the classifier's torch.mean(x, 1) (GRID.py:196,
 * EvalVer.py:323) and ADDJUST's time mean (EvalVer.py:373). */
int dl4ss_time_mean(const float* h, int B, int T, int D, float* mean_out, void* stream);

/* ---- BSS-eval (replaces the un-vendored separation.bss_eval_sources of
 *      Torch_multi/bss_test.py:5,55 -- BSS_EVAL v3, 512-tap distortion filters) ---- */
/* R (M,P,P,L) fp64: R[m][a][b][l] = sum_n x[m][a][n] x[m][b][n+l], l < L, x (M,P,N) fp32
 * (the K references then the estimates of mixture m). */
int dl4ss_bss_corr(const float* x, int M, int P, int N, int L, double* R, void* stream);
/* From R: the Gram matrix of the delayed references G (M, K L, K L) (may be NULL), its
 * diagonal blocks Gd (M, K, L, L) (may be NULL) and D (M, K L, P-K) = <delayed refs, est>. */
int dl4ss_bss_gram(const double* R, int M, int P, int K, int L, double* G, double* Gd, double* D, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DL4SS_HIP_H */
