// Framed STFT (n_fft 256, hop 128, periodic Hann, centre/reflect padding) and
// overlap-add iSTFT for gfx950.
//
// Replaces the CPU librosa.core.spectrum.stft calls of the reference data path
// (Torch_multi/predata_multiAims_dB.py:180,194,209,214;
//  TDAA_beta/predata_fromList_cRM_123.py:215-255) and the istft of its eval
// output path (TDAA_beta/main_run_sstune_EvalVer.py:64-65, cRM_EvalVer.py:98-99).
//
// Design (HBM-bound, ~3.7 flop/B):
//  * forward: one 256-thread workgroup = one 32-frame tile of one signal (see the
//    forward section below: paired real-input DFTs); the iSTFT uses 16-frame
//    tiles.  The sample span a tile covers is read once, coalesced, into LDS
//    (reflect padding resolved at load time), so every sample crosses HBM once;
//  * Hann window and the 256 twiddles W256^m live in LDS, computed once per
//    workgroup with accurate sincospif;
//  * each frame is a 256-pt real DFT done as 16 x 16 Cooley-Tukey: 16 lanes per
//    frame, each lane runs two in-register radix-4x4 DFT16s with one LDS
//    transpose (row stride 17 complex -> conflict-free) in between;
//  * complex (interleaved re/im == the reference's convert2 layout) and
//    magnitude / log-magnitude are written in the same pass.
#include "common.h"

namespace {

constexpr int NFFT = 256;
constexpr int HOPL = 128;
constexpr int NBIN = NFFT / 2 + 1;  // 129
constexpr int FPW = 16;             // frames per workgroup
constexpr int SPAN = HOPL * FPW + NFFT;  // 2304 samples
constexpr int YS = 17;              // padded row stride (complex) of the transpose

enum { F_COMPLEX = 1, F_MAG = 2, F_LOGMAG = 4, F_CONJ = 8, F_APPLY_MAG = 16, F_APPLY_CRM = 32 };

// cos / sin of 2*pi*m/16
__device__ constexpr float C16[16] = {1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
                                      0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
                                      -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f,
                                      0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f};
__device__ constexpr float S16[16] = {0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f,
                                      1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
                                      0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
                                      -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f};

// forward 4-point DFT, in place (W4 = -i)
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  float2 s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
  a0 = cadd(s02, s13);
  a2 = csub(s02, s13);
  a1 = make_float2(d02.x + d13.y, d02.y - d13.x);
  a3 = make_float2(d02.x - d13.y, d02.y + d13.x);
}

// forward 16-point DFT of v (natural order in) -> o (natural order out), sign -1.
template <int SIGN>
__device__ __forceinline__ void dft16(const float2 (&v)[16], float2 (&o)[16]) {
  float2 A[4][4];
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
    float2 a0 = v[n2], a1 = v[4 + n2], a2 = v[8 + n2], a3 = v[12 + n2];
    if (SIGN > 0) {  // inverse: conj trick
      a0.y = -a0.y; a1.y = -a1.y; a2.y = -a2.y; a3.y = -a3.y;
    }
    dft4(a0, a1, a2, a3);
    A[n2][0] = a0; A[n2][1] = a1; A[n2][2] = a2; A[n2][3] = a3;
  }
#pragma unroll
  for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1) {
      const int m = n2 * k1;
      A[n2][k1] = cmul(A[n2][k1], make_float2(C16[m], -S16[m]));
    }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    float2 a0 = A[0][k1], a1 = A[1][k1], a2 = A[2][k1], a3 = A[3][k1];
    dft4(a0, a1, a2, a3);
    if (SIGN > 0) {
      a0.y = -a0.y; a1.y = -a1.y; a2.y = -a2.y; a3.y = -a3.y;
    }
    o[k1] = a0; o[k1 + 4] = a1; o[k1 + 8] = a2; o[k1 + 12] = a3;
  }
}

__device__ __forceinline__ int reflect_idx(int i, int n) {
  // numpy 'reflect' (edge sample not repeated), valid for -n < i < 2n-1
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}

// ---------------------------------------------------------------------------
// Forward STFT.  A tile is FPT = 32 consecutive frames of one signal.  Frames are
// transformed in pairs: z = w.x_a + i w.x_b is one complex 256-point DFT and
//   X_a[k] = (Z[k] + conj Z[256-k]) / 2,   X_b[k] = (Z[k] - conj Z[256-k]) / 2i,
// which halves the DFT work of real input.  16 lanes per pair run the 16 x 16
// Cooley-Tukey (two in-register radix-4x4 DFT16 + one LDS transpose); Z is then
// staged in LDS and every thread emits consecutive output bins of the tile (the
// tile is one contiguous range of the (signal, frame, bin) layout), so complex
// and magnitude stores are fully coalesced.  The launch gives every tile its own
// workgroup (3 resident per CU); a workgroup handed several tiles (grid stride)
// keeps the next span's 16-B loads in flight during the current DFT.
// ---------------------------------------------------------------------------
constexpr int FPT = 32;                  // frames per tile
constexpr int SPAN2 = HOPL * FPT + NFFT;  // 4352 samples
constexpr int SPAN2_Q = SPAN2 / 4;        // 1088 float4
constexpr int PFQ = (SPAN2_Q + 255) / 256;  // float4 per thread (5)

struct SpanRegs {
  float4 v[PFQ];
};
__device__ __forceinline__ void load_span(const float* __restrict__ x, int n_samples, int tiles_per_sig, int tile,
                                          int tid, SpanRegs& r) {
  const int sig = tile / tiles_per_sig;
  const int t0 = (tile - sig * tiles_per_sig) * FPT;
  const float* xs = x + (long long)sig * n_samples;
  const int base = HOPL * t0 - NFFT / 2;  // x index of span[0]
  const bool fast = base >= 0 && base + SPAN2 <= n_samples && ((((uintptr_t)(xs + base)) & 15) == 0);
#pragma unroll
  for (int q = 0; q < PFQ; ++q) {
    const int i4 = tid + 256 * q;
    if (i4 < SPAN2_Q) {
      if (fast) {
        r.v[q] = __ldg(reinterpret_cast<const float4*>(xs + base) + i4);
      } else {
        float e[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int xi = base + 4 * i4 + c;
          e[c] = (xi > -n_samples && xi < 2 * n_samples - 1) ? __ldg(xs + reflect_idx(xi, n_samples)) : 0.0f;
        }
        r.v[q] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  }
}

// the output flags are template parameters: the emit loop carries no per-bin branches and
// computes the log only where it is written
template <bool WC, bool WM, bool LOG, bool CONJ>
__global__ __launch_bounds__(256, 3) void stft_fwd_kernel(const float* __restrict__ x, int n_samples, int T,
                                                          int tiles_per_sig, int n_tiles,
                                                          float2* __restrict__ Xc, float* __restrict__ mag,
                                                          unsigned short* __restrict__ mb, long long ldb, int nbsig) {
  __shared__ float sw[NFFT];
  __shared__ float2 stw[NFFT];
  // transpose [pair][row][col ^ row] (XOR swizzle instead of padding), then Z[pair][256]
  __shared__ __attribute__((aligned(16))) float2 sy[FPT / 2][NFFT];
  __shared__ __attribute__((aligned(16))) float sx[SPAN2];
  // (XOR swizzles of sx / sy against the bank aliasing of a wave's four frame pairs,
  // 256 words apart, measured 12 % slower: the index math costs more than the conflicts)

  const int tid = threadIdx.x;
  {
    float s, c;
    sincospif((float)tid / 128.0f, &s, &c);
    stw[tid] = make_float2(c, -s);  // W256^tid = exp(-2 pi i tid / 256)
    const float sh = sinpif((float)tid / 256.0f);
    // periodic Hann 0.5 - 0.5 cos(2 pi n / 256) = sin^2(pi n / 256), times the 1/2 of the
    // pair split (exact: a power-of-two scale of a linear transform)
    sw[tid] = 0.5f * (sh * sh);
  }
  int tile = blockIdx.x;
  SpanRegs pf;
  if (tile < n_tiles) load_span(x, n_samples, tiles_per_sig, tile, tid, pf);
  const int pr = tid >> 4;  // frame pair within the tile
  const int j = tid & 15;
  float2* sz = &sy[0][0];  // Z of pair p at sz[p * 256 + k]

  for (; tile < n_tiles; tile += gridDim.x) {
    __syncthreads();  // previous tile's Z fully read
#pragma unroll
    for (int q = 0; q < PFQ; ++q) {
      const int i4 = tid + 256 * q;
      if (i4 < SPAN2_Q) reinterpret_cast<float4*>(sx)[i4] = pf.v[q];
    }
    __syncthreads();
    const int next = tile + gridDim.x;
    if (next < n_tiles) load_span(x, n_samples, tiles_per_sig, next, tid, pf);  // in flight during the DFT

    // stage 1: lane j = n2; DFT16 over n1 of z[16 n1 + j], twiddle W256^{j k1}
    {
      float2 v[16], o[16];
      const int fa = HOPL * (2 * pr), fb = fa + HOPL;
#pragma unroll
      for (int n1 = 0; n1 < 16; ++n1) {
        const int n = 16 * n1 + j;
        const float wn = sw[n];
        v[n1] = make_float2(sx[fa + n] * wn, sx[fb + n] * wn);
      }
      dft16<-1>(v, o);
#pragma unroll
      for (int k1 = 0; k1 < 16; ++k1) sz[pr * NFFT + k1 * 16 + (j ^ k1)] = cmul(o[k1], stw[(j * k1) & 255]);
    }
    __syncthreads();
    // stage 2: lane j = k1; DFT16 over n2 -> Z[j + 16 k2]
    float2 o[16];
    {
      float2 v[16];
#pragma unroll
      for (int n2 = 0; n2 < 16; ++n2) v[n2] = sz[pr * NFFT + j * 16 + (n2 ^ j)];
      dft16<-1>(v, o);
    }
    // a pair's 16 lanes sit in one wave and have all read their rows above, so Z
    // overwrites the pair's transpose region without a workgroup barrier
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) sz[pr * NFFT + j + 16 * k2] = o[k2];
    __syncthreads();

    const int sig = tile / tiles_per_sig;
    const int t0 = (tile - sig * tiles_per_sig) * FPT;
    const int nfr = min(FPT, T - t0);
    // split the pairs and emit the tile: thread (parity, bin) = (tid >> 7, tid & 127)
    // writes bin k of frames 2 it + parity (waves 0-1 even frames, 2-3 odd: no
    // divergence); a wave stores 64 consecutive bins of one frame.  Bin 128 by 32
    // threads at the end.
    const long long row0 = ((long long)sig * T + t0) * NBIN;
    const int par = tid >> 7, k = tid & 127;
    const int km = (NFFT - k) & (NFFT - 1);
    float2* xc = Xc + row0 + par * NBIN + k;
    float* xm = mag + row0 + par * NBIN + k;
    // the bf16 copy of the magnitudes of signals < nbsig (the recurrence's first-layer input rows,
    // row stride ldb): no conversion pass over the features (round 5)
    unsigned short* xb = (WM && mb && sig < nbsig) ? mb + ((long long)sig * T + t0 + par) * ldb + k : nullptr;
    auto emit = [&](int it, float2 zk, float2 zm) {
      float2 X = par == 0 ? make_float2(zk.x + zm.x, zk.y - zm.y) : make_float2(zk.y + zm.y, zm.x - zk.x);
      if (CONJ) X.y = -X.y;
      if (WC) xc[2 * it * NBIN] = X;
      if (WM) {
        float m = __builtin_amdgcn_sqrtf(X.x * X.x + X.y * X.y);
        if (LOG) m = __logf(m + 2.220446049250313e-16f);
        xm[2 * it * NBIN] = m;
        if (xb) xb[2 * it * ldb] = (unsigned short)bf16_bits_rne(m);
      }
    };
    if (nfr == FPT) {  // full tile: the LDS reads of four frames issued together
#pragma unroll
      for (int i0 = 0; i0 < FPT / 2; i0 += 4) {
        float2 zk[4], zm[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          zk[u] = sz[(i0 + u) * NFFT + k];
          zm[u] = sz[(i0 + u) * NFFT + km];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) emit(i0 + u, zk[u], zm[u]);
      }
    } else {
      for (int it = 0; 2 * it + par < nfr; ++it) emit(it, sz[it * NFFT + k], sz[it * NFFT + km]);
    }
    if (tid < nfr) {  // Nyquist bin: Z[128] pairs with itself
      const int f = tid;
      const float2 z = sz[(f >> 1) * NFFT + 128];  // Z is half-scaled (window): X = 2 Re / 2 Im
      float2 X = (f & 1) == 0 ? make_float2(2.0f * z.x, 0.0f) : make_float2(2.0f * z.y, 0.0f);
      if (CONJ) X.y = -X.y;
      if (WC) Xc[row0 + f * NBIN + 128] = X;
      if (WM) {
        float m = fabsf(X.x);
        if (LOG) m = __logf(m + 2.220446049250313e-16f);
        mag[row0 + f * NBIN + 128] = m;
        if (WM && mb && sig < nbsig) mb[((long long)sig * T + t0 + f) * ldb + 128] = (unsigned short)bf16_bits_rne(m);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// iSTFT: per output sample, overlap-add of (at most) two frames' windowed
// inverse DFTs, divided by the summed squared window (librosa istft restated).
// One workgroup = 16 frames of one signal: inverse 256-pt real DFT of each
// frame (Hermitian extension), staged in LDS, then the workgroup writes the
// 128*16 output samples it owns: trimmed sample m sits at padded index
// p = m + 128 and needs frames p/128 and p/128 - 1, so the workgroup owning
// m in [128 t0, 128 t0 + 2048) needs frames t0 .. t0+16 (one recomputed).
// ---------------------------------------------------------------------------
// aux (mask-apply modes): signal `sig` is synthesised from mixture sig / k_per_ref:
//   F_APPLY_MAG: S_hat = aux_mag[sig] * exp(i angle X_mix)        (EvalVer.py:56-65)
//   F_APPLY_CRM: S_hat = aux_cplx[sig] (x) X_mix, complex product  (cRM_EvalVer.py:96-99, 720-728)
__global__ __launch_bounds__(256) void istft_kernel(const float2* __restrict__ S, const float* __restrict__ aux,
                                                    int k_per_ref, int T, int flags, float* __restrict__ y,
                                                    int out_len, int tiles) {
  // frames t0 .. t0+16 (17 frames), each 256 real samples after irfft*window
  __shared__ float2 stw[NFFT];
  __shared__ float sw[NFFT];
  __shared__ float2 sy[FPW + 1][16 * YS];
  __shared__ float sf[FPW + 1][NFFT];

  const int tid = threadIdx.x;
  const long long sig = blockIdx.x / tiles;
  const int t0 = (blockIdx.x % tiles) * FPW;
  {
    float s, c;
    sincospif((float)tid / 128.0f, &s, &c);
    stw[tid] = make_float2(c, s);  // inverse twiddle exp(+2 pi i tid/256)
    const float sh = sinpif((float)tid / 256.0f);
    sw[tid] = sh * sh;
  }
  __syncthreads();
  const bool conj = flags & F_CONJ;
  // 17 frames x 16 lanes = 272 tasks over 256 threads
  for (int task = tid; task < (FPW + 1) * 16; task += 256) {
    const int fr = task >> 4, j = task & 15;
    const int t = t0 + fr;
    // inverse 256-pt DFT x[n] = (1/256) sum_k Z[k] e^{+2 pi i nk/256} with
    // k = 16 k1 + k2, n = n1 + 16 n2; stage 1: lane j = k2, DFT16 over k1
    float2 v[16], o[16];
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) {
      const int k = 16 * k1 + j;
      float2 z = make_float2(0.f, 0.f);
      if (t >= 0 && t < T) {
        const long long ref = (flags & (F_APPLY_MAG | F_APPLY_CRM)) ? sig / k_per_ref : sig;
        const int kk = k < NBIN ? k : NFFT - k;
        z = S[(ref * T + t) * (long long)NBIN + kk];
        const long long arow = (sig * T + t) * (long long)NBIN + kk;
        if (flags & F_APPLY_MAG) {
          const float m = aux[arow], a = sqrtf(z.x * z.x + z.y * z.y);
          z = a > 0.0f ? make_float2(z.x * (m / a), z.y * (m / a)) : make_float2(m, 0.0f);
        } else if (flags & F_APPLY_CRM) {
          float2 mk = reinterpret_cast<const float2*>(aux)[arow];
          if (conj) mk.y = -mk.y;  // S holds conj(X): conj(M X) = conj(M) conj(X)
          z = cmul(mk, z);
        }
        if (k < NBIN) {
          if (conj) z.y = -z.y;
        } else {
          if (!conj) z.y = -z.y;  // Hermitian: Z[256-k] = conj(Z[k])
        }
        if (k == 0 || k == 128) z.y = 0.0f;  // irfft ignores imag of DC/Nyquist
      }
      v[k1] = z;
    }
    dft16<+1>(v, o);  // over k1 -> index n1
#pragma unroll
    for (int n1 = 0; n1 < 16; ++n1) sy[fr][n1 * YS + j] = cmul(o[n1], stw[(j * n1) & 255]);
  }
  __syncthreads();
  for (int task = tid; task < (FPW + 1) * 16; task += 256) {
    const int fr = task >> 4, j = task & 15;  // j = n1
    float2 v[16], o[16];
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) v[k2] = sy[fr][j * YS + k2];
    dft16<+1>(v, o);  // over k2 -> n2
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) {
      const int n = j + 16 * n2;
      sf[fr][n] = o[n2].x * (1.0f / 256.0f) * sw[n];
    }
  }
  __syncthreads();
  // output sample m (after trimming 128): padded index p = m + 128,
  // frames covering p: t = p/128 (offset p%128) and t-1 (offset p%128 + 128)
  for (int i = tid; i < FPW * HOPL; i += 256) {
    const int m = t0 * HOPL + i;
    if (m >= out_len) break;
    const int p = m + HOPL;
    const int fa = p / HOPL - t0;  // frame p/128 (local index 1..16); frame fa-1 also covers p
    const int off = p % HOPL;
    const float acc = sf[fa][off] + sf[fa - 1][off + HOPL];
    const float wss = sw[off] * sw[off] + sw[off + HOPL] * sw[off + HOPL];
    y[sig * (long long)out_len + m] = (wss > 1.17549435e-38f) ? acc / wss : acc;
  }
}

}  // namespace

DL4SS_API int dl4ss_stft_fwd_ex(const float* x, long long n_sig, int n_samples, int n_fft, int hop, int flags,
                                float* X_c64, float* mag, void* mag_bf16, long long ld_bf16, long long n_sig_bf16,
                                void* stream) {
  DL4SS_REQUIRE(n_fft == NFFT && hop == HOPL && n_samples > NFFT / 2 && n_sig >= 0);
  if (n_sig == 0) return 0;  // empty batch: no-op (an empty tensor's pointer may be null)
  DL4SS_REQUIRE(x);
  DL4SS_REQUIRE(!((flags & F_COMPLEX) && !X_c64));
  DL4SS_REQUIRE(!((flags & (F_MAG | F_LOGMAG)) && !mag));
  DL4SS_REQUIRE(!mag_bf16 || ((flags & (F_MAG | F_LOGMAG)) && ld_bf16 >= NBIN && n_sig_bf16 >= 0 && n_sig_bf16 <= n_sig));
  const int T = 1 + n_samples / HOPL;
  const int tiles = (T + FPT - 1) / FPT;
  // one workgroup per tile: measured on MI355X (2048 x 4 s signals, complex + magnitude)
  // 4.2-4.3 TB/s against 3.8-3.9 for a grid-stride launch sized to the resident
  // capacity (768 workgroups walking 21 tiles each); the kernel still accepts any grid
  const long long n_tiles = n_sig * tiles;
  DL4SS_REQUIRE(n_tiles < (1LL << 31));
  const long long grid = n_tiles;
  using K = void (*)(const float*, int, int, int, int, float2*, float*, unsigned short*, long long, int);
  static const K kern[16] = {
      stft_fwd_kernel<0, 0, 0, 0>, stft_fwd_kernel<1, 0, 0, 0>, stft_fwd_kernel<0, 1, 0, 0>, stft_fwd_kernel<1, 1, 0, 0>,
      stft_fwd_kernel<0, 0, 1, 0>, stft_fwd_kernel<1, 0, 1, 0>, stft_fwd_kernel<0, 1, 1, 0>, stft_fwd_kernel<1, 1, 1, 0>,
      stft_fwd_kernel<0, 0, 0, 1>, stft_fwd_kernel<1, 0, 0, 1>, stft_fwd_kernel<0, 1, 0, 1>, stft_fwd_kernel<1, 1, 0, 1>,
      stft_fwd_kernel<0, 0, 1, 1>, stft_fwd_kernel<1, 0, 1, 1>, stft_fwd_kernel<0, 1, 1, 1>, stft_fwd_kernel<1, 1, 1, 1>};
  const int sel = ((flags & F_COMPLEX) ? 1 : 0) | ((flags & (F_MAG | F_LOGMAG)) ? 2 : 0) |
                  ((flags & F_LOGMAG) ? 4 : 0) | ((flags & F_CONJ) ? 8 : 0);
  hipLaunchKernelGGL(kern[sel], dim3((unsigned)grid), dim3(256), 0, as_stream(stream), x, n_samples, T, tiles,
                     (int)n_tiles, reinterpret_cast<float2*>(X_c64), mag, static_cast<unsigned short*>(mag_bf16), ld_bf16,
                     (int)(mag_bf16 ? n_sig_bf16 : 0));
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_stft_fwd(const float* x, long long n_sig, int n_samples, int n_fft, int hop, int flags,
                             float* X_c64, float* mag, void* stream) {
  return dl4ss_stft_fwd_ex(x, n_sig, n_samples, n_fft, hop, flags, X_c64, mag, nullptr, 0, 0, stream);
}

DL4SS_API int dl4ss_istft(const float* S_c64, long long n_sig, int T, int n_fft, int hop, int flags, float* y,
                          void* stream) {
  DL4SS_REQUIRE(n_fft == NFFT && hop == HOPL && T >= 2 && n_sig >= 0);
  if (n_sig == 0) return 0;
  DL4SS_REQUIRE(S_c64 && y);
  const int out_len = HOPL * (T - 1);
  const int tiles = (T - 1 + FPW - 1) / FPW;
  hipLaunchKernelGGL(istft_kernel, dim3((unsigned)(n_sig * tiles)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float2*>(S_c64), nullptr, 1, T, flags & F_CONJ, y, out_len, tiles);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

// Mask apply + overlap-add iSTFT in one pass (eval path, SURVEY R12 + R16): n_sig
// output signals, signal s from mixture s / k_per_mix.  mode 0: aux = masked
// magnitude (n_sig, T, 129) with the mixture phase; mode 1: aux = complex ratio
// mask (n_sig, T, 129, 2) multiplied with the mixture spectrum.
DL4SS_API int dl4ss_istft_apply(const float* X_mix_c64, const float* aux, long long n_sig, int k_per_mix, int T,
                                int mode, int conj, float* y, void* stream) {
  DL4SS_REQUIRE(T >= 2 && n_sig >= 0 && k_per_mix >= 1 && (mode == 0 || mode == 1));
  if (n_sig == 0) return 0;
  DL4SS_REQUIRE(X_mix_c64 && aux && y);
  const int out_len = HOPL * (T - 1);
  const int tiles = (T - 1 + FPW - 1) / FPW;
  const int flags = (mode == 0 ? F_APPLY_MAG : F_APPLY_CRM) | (conj ? F_CONJ : 0);
  hipLaunchKernelGGL(istft_kernel, dim3((unsigned)(n_sig * tiles)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float2*>(X_mix_c64), aux, k_per_mix, T, flags, y, out_len, tiles);
  DL4SS_CHECK_LAUNCH();
  return 0;
}
