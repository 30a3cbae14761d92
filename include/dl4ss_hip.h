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

/* Overlap-add inverse STFT: S (n_sig, T, 129, 2) -> y (n_sig, 128 * (T - 1)).
 * Replaces librosa.core.spectrum.istft(S.T, 128) at
 * TDAA_beta/main_run_sstune_EvalVer.py:64-65 and main_run_sstune_cRM_EvalVer.py:98-99.
 * flags: DL4SS_STFT_CONJ only. */
int dl4ss_istft(const float* S_c64, long long n_sig, int T, int n_fft, int hop, int flags, float* y,
                void* stream);

/* ---- R1 preprocessing / mixing ----------------------------------------- */
/* raw (B, K, N) -> out (B, K+1, N): each source x -> (x - mean) / max|x - mean| * gain,
 * then their sum as channel K.  stats_ws: 2*B*K floats of workspace.
 * Replaces Torch_multi/predata_multiAims_dB.py:156-197 (and the _3dB /
 * fromList_cRM_123 gain variants: gains are computed by the caller). */
int dl4ss_mix_sources(const float* raw, const float* gains, int B, int K, int N, float* stats_ws, float* out,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DL4SS_HIP_H */
