// EXPERIMENT (not part of the product library): a bf16 GEMM whose MFMA operands go straight from
// global memory into registers -- no LDS, no workgroup barrier -- to measure the "direct-to-register
// operand path" DESIGN.md section 10 names against gemm_gl's LDS-DMA k-loop on the step's shapes.
//
//   C[M][N] (fp32, ldc) = A[M][K] (bf16, lda) * Bt[N][K]^T (bf16, ldb); both operands k-contiguous.
//
// One wave = one WM*16 x WN*16 output tile (a workgroup is WPB independent waves); each lane loads
// its own 16-B fragments (row lane & 15, k 8 (lane >> 4) .. +7 of every 32-k step) STAGES k-steps
// ahead into registers and runs the k-step's WM x WN v_mfma_f32_16x16x32_bf16.  Operand reuse
// between waves goes through L1 / L2 instead of LDS.  K % 32 == 0, lda / ldb % 8 == 0.
// Built by tools/gemm_dr_probe.py into tools/exp/libgemm_dr.so (outside the package).
#include <hip/hip_runtime.h>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

template <int WM, int WN, int STAGES, int WPB>
__global__ __launch_bounds__(64 * WPB) void gemm_dr_kernel(int M, int N, int K, const unsigned short* __restrict__ A,
                                                           long long lda, const unsigned short* __restrict__ Bt,
                                                           long long ldb, float* __restrict__ C, long long ldc,
                                                           int tiles_n, int n_tiles) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * WPB + (threadIdx.x >> 6);
  if (wave >= n_tiles) return;
  // N-fastest tile order within a group of 8 M-tiles (the A panels of a group stay hot in L2)
  constexpr int GM = 8;
  const int tiles_m = (M + WM * 16 - 1) / (WM * 16);
  const int per_group = GM * tiles_n;
  const int grp = wave / per_group, rem = wave % per_group;
  const int gm = min(GM, tiles_m - grp * GM);
  const int tm = grp * GM + rem % gm, tn = rem / gm;
  const int m0 = tm * WM * 16, n0 = tn * WN * 16;
  const int r = lane & 15, kq = 8 * (lane >> 4);
  const unsigned short* ap[WM];
  const unsigned short* bp[WN];
#pragma unroll
  for (int i = 0; i < WM; ++i) ap[i] = A + (long long)min(m0 + 16 * i + r, M - 1) * lda + kq;
#pragma unroll
  for (int j = 0; j < WN; ++j) bp[j] = Bt + (long long)min(n0 + 16 * j + r, N - 1) * ldb + kq;
  f32x4 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[STAGES][WM], b[STAGES][WN];
  const int nks = K / 32;
#pragma unroll
  for (int s = 0; s < STAGES; ++s) {
    if (s < nks) {
#pragma unroll
      for (int i = 0; i < WM; ++i) a[s][i] = *reinterpret_cast<const bf16x8*>(ap[i] + 32 * s);
#pragma unroll
      for (int j = 0; j < WN; ++j) b[s][j] = *reinterpret_cast<const bf16x8*>(bp[j] + 32 * s);
    }
  }
  // k loop unrolled by STAGES: stage indices compile-time
  for (int k0 = 0; k0 < nks; k0 += STAGES) {
#pragma unroll
    for (int s = 0; s < STAGES; ++s) {
      const int ks = k0 + s;
      if (ks < nks) {
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][i], b[s][j], acc[i][j], 0, 0, 0);
        const int kn = ks + STAGES;
        if (kn < nks) {
#pragma unroll
          for (int i = 0; i < WM; ++i) a[s][i] = *reinterpret_cast<const bf16x8*>(ap[i] + 32 * kn);
#pragma unroll
          for (int j = 0; j < WN; ++j) b[s][j] = *reinterpret_cast<const bf16x8*>(bp[j] + 32 * kn);
        }
      }
    }
  }
  // D[4 (lane >> 4) + e][lane & 15] of each 16 x 16 tile
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int col = n0 + 16 * j + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + 16 * i + 4 * (lane >> 4) + e;
        if (row < M && col < N) C[(long long)row * ldc + col] = acc[i][j][e];
      }
    }
}

template <int WM, int WN, int STAGES, int WPB>
int launch(int M, int N, int K, const void* A, long long lda, const void* Bt, long long ldb, float* C, long long ldc,
           hipStream_t st) {
  const int tiles_m = (M + WM * 16 - 1) / (WM * 16), tiles_n = (N + WN * 16 - 1) / (WN * 16);
  const int n_tiles = tiles_m * tiles_n;
  const int grid = (n_tiles + WPB - 1) / WPB;
  hipLaunchKernelGGL((gemm_dr_kernel<WM, WN, STAGES, WPB>), dim3(grid), dim3(64 * WPB), 0, st, M, N, K,
                     static_cast<const unsigned short*>(A), lda, static_cast<const unsigned short*>(Bt), ldb, C, ldc,
                     tiles_n, n_tiles);
  return (int)hipGetLastError();
}

}  // namespace

// variant: (WM, WN, STAGES, WPB) from a small table
extern "C" __attribute__((visibility("default"))) int gemm_dr(int variant, int M, int N, int K, const void* A,
                                                              long long lda, const void* Bt, long long ldb, float* C,
                                                              long long ldc, void* stream) {
  if (K % 32 || lda % 8 || ldb % 8 || M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (variant) {
    case 0: return launch<4, 4, 2, 4>(M, N, K, A, lda, Bt, ldb, C, ldc, st);
    case 1: return launch<4, 4, 3, 4>(M, N, K, A, lda, Bt, ldb, C, ldc, st);
    case 2: return launch<4, 4, 4, 4>(M, N, K, A, lda, Bt, ldb, C, ldc, st);
    case 3: return launch<2, 4, 4, 4>(M, N, K, A, lda, Bt, ldb, C, ldc, st);
    case 4: return launch<4, 2, 4, 4>(M, N, K, A, lda, Bt, ldb, C, ldc, st);
    case 5: return launch<2, 2, 6, 4>(M, N, K, A, lda, Bt, ldb, C, ldc, st);
    case 6: return launch<4, 4, 3, 1>(M, N, K, A, lda, Bt, ldb, C, ldc, st);
    default: return (int)hipErrorInvalidValue;
  }
}
