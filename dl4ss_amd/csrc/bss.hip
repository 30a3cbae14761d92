// BSS-eval building blocks on the GPU: the correlations and the
// Gram systems of the 512-tap distortion-filter projections of BSS_EVAL v3, which the
// reference evaluates on the host per mixture through the un-vendored
// separation.bss_eval_sources (Torch_multi/bss_test.py:5,55).
//
//   dl4ss_bss_corr  R[m][a][b][l] = sum_n x[m][a][n] x[m][b][n + l], l in [0, L), for every
//                   ordered pair of the P signals of mixture m (references then estimates);
//                   fp64 accumulation of exact fp32 x fp32 products.  HBM-light / FMA-bound:
//                   each workgroup stages a 1024-sample chunk of both signals in LDS.
//   dl4ss_bss_gram  the (K L) x (K L) Gram matrix of the delayed references
//                   G[i L + a][j L + b] = <s_i delayed a, s_j delayed b>, its K diagonal
//                   blocks, and the right-hand sides D[i L + a][e] = <s_i delayed a, est_e>.
#include "common.h"

namespace {

constexpr int LT = 64;     // lags per workgroup (one wave-wide lag vector)
constexpr int CH = 1024;   // samples per staged chunk
constexpr int NPH = 4;     // n phases (waves) per workgroup

__global__ __launch_bounds__(256) void bss_corr_kernel(const float* __restrict__ x, int P, int N, int L,
                                                       double* __restrict__ R) {
  __shared__ double sa[CH];
  __shared__ double sb[CH + LT];
  __shared__ double red[NPH][LT];
  const int ltiles = (L + LT - 1) / LT;
  const int tile = blockIdx.x % ltiles;
  const int pair = (blockIdx.x / ltiles) % (P * P);
  const int m = blockIdx.x / (ltiles * P * P);
  const int a = pair / P, b = pair % P;
  const float* xa = x + ((long long)m * P + a) * N;
  const float* xb = x + ((long long)m * P + b) * N;
  const int l0 = tile * LT;
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int lag = l0 + lane;
  double acc = 0.0;
  for (int n0 = 0; n0 < N; n0 += CH) {
    for (int i = threadIdx.x; i < CH; i += 256) {
      const int n = n0 + i;
      sa[i] = n < N ? (double)xa[n] : 0.0;
    }
    for (int i = threadIdx.x; i < CH + LT; i += 256) {
      const int n = n0 + l0 + i;
      sb[i] = n < N ? (double)xb[n] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int i = ph; i < CH; i += NPH) acc = fma(sa[i], sb[i + lane], acc);
    __syncthreads();
  }
  red[ph][lane] = acc;
  __syncthreads();
  if (ph == 0 && lag < L)
    R[(((long long)m * P + a) * P + b) * L + lag] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// G (M, K L, K L), Gd (M, K, L, L), D (M, K L, Ke); one thread per G element (grid-stride)
__global__ __launch_bounds__(256) void bss_gram_kernel(const double* __restrict__ R, int M, int P, int K, int L,
                                                       double* __restrict__ G, double* __restrict__ Gd,
                                                       double* __restrict__ D) {
  const int KL = K * L, Ke = P - K;
  const long long nG = (long long)M * KL * KL;
  const long long nD = (long long)M * KL * Ke;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < nG + nD; e += (long long)gridDim.x * 256) {
    if (e < nG) {
      const int col = (int)(e % KL);
      const int row = (int)((e / KL) % KL);
      const int m = (int)(e / ((long long)KL * KL));
      const int i = row / L, ra = row % L, j = col / L, cb = col % L;
      // <s_i delayed ra, s_j delayed cb> = R[i][j][ra - cb] (ra >= cb) or R[j][i][cb - ra]
      const double v = ra >= cb ? R[(((long long)m * P + i) * P + j) * L + (ra - cb)]
                                : R[(((long long)m * P + j) * P + i) * L + (cb - ra)];
      if (G) G[e] = v;
      if (Gd && i == j) Gd[(((long long)m * K + i) * L + ra) * L + cb] = v;
    } else {
      const long long f = e - nG;  // D[m][i L + a][est]
      const int est = (int)(f % Ke);
      const int row = (int)((f / Ke) % KL);
      const int m = (int)(f / ((long long)Ke * KL));
      const int i = row / L, la = row % L;
      D[f] = R[(((long long)m * P + i) * P + (K + est)) * L + la];  // <s_i delayed la, est>
    }
  }
}

}  // namespace

DL4SS_API int dl4ss_bss_corr(const float* x, int M, int P, int N, int L, double* R, void* stream) {
  DL4SS_REQUIRE(x && R && M >= 0 && P > 0 && N > 0 && L > 0 && L <= N);
  if (M == 0) return 0;
  const long long grid = (long long)M * P * P * ((L + LT - 1) / LT);
  DL4SS_REQUIRE(grid < (1LL << 31));
  hipLaunchKernelGGL(bss_corr_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), x, P, N, L, R);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_bss_gram(const double* R, int M, int P, int K, int L, double* G, double* Gd, double* D,
                             void* stream) {
  DL4SS_REQUIRE(R && D && M >= 0 && K > 0 && P > K && L > 0);
  if (M == 0) return 0;
  const long long n = (long long)M * K * L * (K * L + (P - K));
  const unsigned grid = (unsigned)min(65536LL, cdiv(n, 256));
  hipLaunchKernelGGL(bss_gram_kernel, dim3(grid), dim3(256), 0, as_stream(stream), R, M, P, K, L, G, Gd, D);
  DL4SS_CHECK_LAUNCH();
  return 0;
}
