// Framed STFT (n_fft 256, hop 128, periodic Hann, centre/reflect padding) and
// overlap-add iSTFT for gfx950.
//
// Replaces the CPU librosa.core.spectrum.stft calls of the reference data path
// (Torch_multi/predata_multiAims_dB.py:180,194,209,214;
//  TDAA_beta/predata_fromList_cRM_123.py:215-255) and the istft of its eval
// output path (TDAA_beta/main_run_sstune_EvalVer.py:64-65, cRM_EvalVer.py:98-99).
//
// Design (HBM-bound, ~3.7 flop/B):
//  * one 256-thread workgroup = 16 consecutive frames of one signal; the
//    2304-sample span they cover is read once, coalesced, into LDS (reflect
//    padding resolved at load time), so every sample crosses HBM once;
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

enum { F_COMPLEX = 1, F_MAG = 2, F_LOGMAG = 4, F_CONJ = 8 };

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

// Copy n floats LDS -> global with 16-B stores for the aligned body (the tile of
// 16 consecutive frames is one contiguous range of the (sig, t, bin) output).
__device__ __forceinline__ void store_tile(float* __restrict__ dst, const float* src, int n, int tid) {
  const int h = min((int)(((16 - ((uintptr_t)dst & 15)) & 15) >> 2), n);  // floats before 16-B alignment
  if (tid < h) dst[tid] = src[tid];
  const int nv = (n - h) >> 2;
  float4* d4 = reinterpret_cast<float4*>(dst + h);
  const float* s = src + h;
  for (int i = tid; i < nv; i += 256) d4[i] = make_float4(s[4 * i], s[4 * i + 1], s[4 * i + 2], s[4 * i + 3]);
  const int t0 = h + 4 * nv;
  if (tid < n - t0) dst[t0 + tid] = src[t0 + tid];
}

// Span of tile `tile` into registers: thread owns span[4 (tid + 256 r) .. +3], r < 3.
// Interior tiles: one 16-B load per piece; the two edge tiles of a signal resolve
// the reflect padding per sample.
struct SpanRegs {
  float4 v[3];
};
__device__ __forceinline__ void load_span(const float* __restrict__ x, int n_samples, int frames_tiles, long long tile,
                                          int tid, SpanRegs& r) {
  const long long sig = tile / frames_tiles;
  const int t0 = (int)(tile % frames_tiles) * FPW;
  const float* xs = x + sig * (long long)n_samples;
  const int base = HOPL * t0 - NFFT / 2;  // x index of span[0]
  const bool fast = base >= 0 && base + SPAN <= n_samples && ((((uintptr_t)(xs + base)) & 15) == 0);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int i = 4 * (tid + 256 * q);
    if (i < SPAN) {
      if (fast) {
        r.v[q] = __ldg(reinterpret_cast<const float4*>(xs + base + i));
      } else {
        float e[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int xi = base + i + c;
          e[c] = (xi > -n_samples && xi < 2 * n_samples - 1) ? __ldg(xs + reflect_idx(xi, n_samples)) : 0.0f;
        }
        r.v[q] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  }
}

// One workgroup loops over tiles (16 consecutive frames of one signal) in grid
// stride; the next tile's span is loaded into registers while the current one is
// transformed, so HBM latency hides behind the DFT even at 3 workgroups per CU.
__global__ __launch_bounds__(256) void stft_fwd_kernel(const float* __restrict__ x, int n_samples, int T,
                                                       int frames_tiles, long long n_tiles, int flags,
                                                       float* __restrict__ Xc, float* __restrict__ mag) {
  __shared__ __attribute__((aligned(16))) float sx[SPAN];
  __shared__ float sw[NFFT];
  __shared__ float2 stw[NFFT];
  __shared__ __attribute__((aligned(16))) float2 sy[FPW][16 * YS];  // transpose; then the output tile

  const int tid = threadIdx.x;
  // window + twiddles (LDS-resident, accurate), once per workgroup
  {
    float s, c;
    sincospif((float)tid / 128.0f, &s, &c);
    stw[tid] = make_float2(c, -s);  // W256^tid = exp(-2 pi i tid / 256)
    const float sh = sinpif((float)tid / 256.0f);
    sw[tid] = sh * sh;  // periodic Hann: 0.5 - 0.5 cos(2 pi n / 256) = sin^2(pi n / 256)
  }
  long long tile = blockIdx.x;
  SpanRegs pf;
  if (tile < n_tiles) load_span(x, n_samples, frames_tiles, tile, tid, pf);
  const int fr = tid >> 4;  // frame within tile
  const int j = tid & 15;
  const bool conj = flags & F_CONJ;
  float2* tc = reinterpret_cast<float2*>(&sy[0][0]);      // output tile: FPW x NBIN complex
  float* tm = reinterpret_cast<float*>(tc + FPW * NBIN);  // FPW x NBIN magnitude

  for (; tile < n_tiles; tile += gridDim.x) {
    __syncthreads();  // previous tile's output staging fully read
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int i = 4 * (tid + 256 * q);
      if (i < SPAN) *reinterpret_cast<float4*>(sx + i) = pf.v[q];
    }
    __syncthreads();
    const long long next = tile + gridDim.x;
    if (next < n_tiles) load_span(x, n_samples, frames_tiles, next, tid, pf);  // in flight during the DFT

    // stage 1: lane j = n2; DFT16 over n1 of xw[16 n1 + j], twiddle W256^{j k1}
    {
      float2 v[16], o[16];
      const float* fx = sx + HOPL * fr;
#pragma unroll
      for (int n1 = 0; n1 < 16; ++n1) {
        const int n = 16 * n1 + j;
        v[n1] = make_float2(fx[n] * sw[n], 0.0f);
      }
      dft16<-1>(v, o);
#pragma unroll
      for (int k1 = 0; k1 < 16; ++k1) sy[fr][k1 * YS + j] = cmul(o[k1], stw[(j * k1) & 255]);
    }
    __syncthreads();
    // stage 2: lane j = k1; DFT16 over n2 -> X[j + 16 k2]
    float2 o[16];
    {
      float2 v[16];
#pragma unroll
      for (int n2 = 0; n2 < 16; ++n2) v[n2] = sy[fr][j * YS + n2];
      dft16<-1>(v, o);
    }
    __syncthreads();  // sy is reused as the output tile below
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) {
      const int k = j + 16 * k2;
      if (k < NBIN) {
        float2 X = o[k2];
        if (conj) X.y = -X.y;
        tc[fr * NBIN + k] = X;
        float m = sqrtf(X.x * X.x + X.y * X.y);
        if (flags & F_LOGMAG) m = logf(m + 2.220446049250313e-16f);
        tm[fr * NBIN + k] = m;
      }
    }
    __syncthreads();
    const long long sig = tile / frames_tiles;
    const int t0 = (int)(tile % frames_tiles) * FPW;
    const int nfr = min(FPW, T - t0);
    const long long row0 = (sig * T + t0) * (long long)NBIN;
    if (flags & F_COMPLEX) store_tile(Xc + 2 * row0, reinterpret_cast<const float*>(tc), 2 * nfr * NBIN, tid);
    if (flags & (F_MAG | F_LOGMAG)) store_tile(mag + row0, tm, nfr * NBIN, tid);
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
__global__ __launch_bounds__(256) void istft_kernel(const float2* __restrict__ S, int T, int flags,
                                                    float* __restrict__ y, int out_len, int tiles) {
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
        const long long row = (sig * T + t) * (long long)NBIN;
        if (k < NBIN) {
          z = S[row + k];
          if (conj) z.y = -z.y;
        } else {
          z = S[row + (NFFT - k)];
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

DL4SS_API int dl4ss_stft_fwd(const float* x, long long n_sig, int n_samples, int n_fft, int hop, int flags,
                             float* X_c64, float* mag, void* stream) {
  DL4SS_REQUIRE(n_fft == NFFT && hop == HOPL && n_samples > NFFT / 2 && n_sig >= 0);
  DL4SS_REQUIRE(!((flags & F_COMPLEX) && !X_c64));
  DL4SS_REQUIRE(!((flags & (F_MAG | F_LOGMAG)) && !mag));
  if (n_sig == 0) return 0;
  const int T = 1 + n_samples / HOPL;
  const int tiles = (T + FPW - 1) / FPW;
  // grid-stride launch sized to the resident capacity (3 workgroups per CU: LDS and VGPRs)
  const long long n_tiles = n_sig * tiles;
  const long long grid = n_tiles < 256LL * 3 ? n_tiles : 256LL * 3;
  hipLaunchKernelGGL(stft_fwd_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), x, n_samples, T, tiles,
                     n_tiles, flags, X_c64, mag);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_istft(const float* S_c64, long long n_sig, int T, int n_fft, int hop, int flags, float* y,
                          void* stream) {
  DL4SS_REQUIRE(n_fft == NFFT && hop == HOPL && T >= 2 && n_sig >= 0 && S_c64 && y);
  if (n_sig == 0) return 0;
  const int out_len = HOPL * (T - 1);
  const int tiles = (T - 1 + FPW - 1) / FPW;
  hipLaunchKernelGGL(istft_kernel, dim3((unsigned)(n_sig * tiles)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float2*>(S_c64), T, flags, y, out_len, tiles);
  DL4SS_CHECK_LAUNCH();
  return 0;
}
