// LDS-tiled MFMA GEMM for the dense contractions of the separation step:
//   * BiRNN input projection  G = X W_ih^T + b         (EvalVer.py:282-293, cuDNN)
//   * Linear(600 -> F*E) + tanh  V = tanh(h W^T + b)   (EvalVer.py:290,298-299)
//   * their backward products dX = dG W, dW = dG^T X   (autograd in the reference)
//
// C[M,N] (+)= op(A)[M,K] . op(B)[K,N] (+ bias[N]) (tanh), fp32 in HBM.
// Two arithmetic modes:
//   PREC_F32  : v_mfma_f32_32x32x2_f32 -- exact fp32 products, fp32 accumulate
//               (the parity mode: bitwise an fmaf chain per k-slice);
//   PREC_BF16 : operands rounded to bf16 while staged into LDS,
//               v_mfma_f32_32x32x16_bf16, fp32 accumulate (the throughput mode).
// Tile 128x128xBK, 256 threads = 4 waves in 2x2, each wave 64x64 = 2x2 MFMA
// 32x32 accumulators.  Register-prefetched global loads (the next K-tile is in
// flight while the current one is multiplied), double-buffered LDS, one barrier
// per K-tile.  Each operand is staged in the LDS layout that matches its HBM
// contiguity (k-contiguous rows padded to an odd stride, or r-contiguous
// k-rows), so both global reads and fragment reads are conflict-free.
// Split-K (grid.z) accumulates with fp32 atomics into C (used for the weight
// gradients, whose K = B*T is long and whose tile count is small).
#include "common.h"
#include <type_traits>
#include <hip/hip_bf16.h>

namespace {

constexpr int BM = 128, BN = 128;
constexpr int NT = 256;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

enum { EPI_NONE = 0, EPI_TANH = 1 };
enum { PREC_F32 = 0, PREC_BF16 = 1 };

__device__ __forceinline__ unsigned short f2bf(float f) {
  // round-to-nearest-even (NaN-safe enough for activations/weights)
  unsigned u = __float_as_uint(f);
  u += 0x7FFF + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}

// Operand tile staging.  KC = operand is k-contiguous in HBM.
//   KC  : element (r,k) at G[r*ld + k]; LDS [r][k] with row stride BK+1 (fp32) or BK+8 (bf16 packs)
//   !KC : element (r,k) at G[k*ld + r]; LDS [k][r] with row stride R
template <int BK, bool KC, int PREC>
struct Operand {
  static constexpr int ELEMS = 128 * BK;              // per tile
  static constexpr int PER_THREAD = ELEMS / NT;       // elements each thread stages
  static constexpr int LDK = (PREC == PREC_F32) ? (BK + 1) : (BK + 8);  // KC row stride (elements)
  static constexpr int LDS_ELEMS = KC ? 128 * LDK : BK * 128;
  using elem_t = typename std::conditional<PREC == PREC_F32, float, unsigned short>::type;

  float regs[PER_THREAD];

  __device__ __forceinline__ void load(const float* __restrict__ G, long long ld, int r0, int rmax, int k0,
                                       int kmax) {
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int e = threadIdx.x + NT * i;
      int r, k;
      if (KC) { r = e / BK; k = e % BK; } else { k = e / 128; r = e % 128; }
      const int gr = r0 + r, gk = k0 + k;
      float v = 0.0f;
      if (gr < rmax && gk < kmax) v = KC ? G[(long long)gr * ld + gk] : G[(long long)gk * ld + gr];
      regs[i] = v;
    }
  }
  __device__ __forceinline__ void store(elem_t* __restrict__ s) const {
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int e = threadIdx.x + NT * i;
      int r, k;
      if (KC) { r = e / BK; k = e % BK; } else { k = e / 128; r = e % 128; }
      const int idx = KC ? r * LDK + k : k * 128 + r;
      if constexpr (PREC == PREC_F32) s[idx] = regs[i];
      else s[idx] = f2bf(regs[i]);
    }
  }
};

// f32 fragment for 32x32x2: lane l holds (row r0 + (l&31), k kk + (l>>5))
template <int BK, bool KC>
__device__ __forceinline__ float frag_f32(const float* s, int r0, int kk, int lane) {
  constexpr int LDK = BK + 1;
  const int r = r0 + (lane & 31), k = kk + (lane >> 5);
  return KC ? s[r * LDK + k] : s[k * 128 + r];
}

// bf16 fragment for 32x32x16: lane l holds row r0 + (l&31), k = kk + 8*(l>>5) + j, j=0..7
template <int BK, bool KC>
__device__ __forceinline__ bf16x8 frag_bf16(const unsigned short* s, int r0, int kk, int lane) {
  constexpr int LDK = BK + 8;
  const int r = r0 + (lane & 31), kb = kk + 8 * (lane >> 5);
  bf16x8 v;
  if (KC) {
    // 8 contiguous bf16 = 16 B (row stride BK+8 keeps 16-B alignment)
    v = *reinterpret_cast<const bf16x8*>(s + r * LDK + kb);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (short)s[(kb + j) * 128 + r];
  }
  return v;
}

template <bool A_KC, bool B_KC, int PREC, int EPI, bool ATOMIC>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(int M, int N, int K, const float* __restrict__ A, long long lda,
                                                     const float* __restrict__ B, long long ldb,
                                                     float* __restrict__ C, long long ldc,
                                                     const float* __restrict__ bias, float beta, int k_per_split,
                                                     int grid_m) {
  constexpr int BK = (PREC == PREC_F32) ? 16 : 32;
  using OA = Operand<BK, A_KC, PREC>;
  using OB = Operand<BK, B_KC, PREC>;
  using elem_t = typename OA::elem_t;
  __shared__ __attribute__((aligned(16))) elem_t sA[2][OA::LDS_ELEMS];
  __shared__ __attribute__((aligned(16))) elem_t sB[2][OB::LDS_ELEMS];

  // XCD-aware tile order: consecutive blocks along M share a B panel.
  const int bid = blockIdx.x;
  const int tm = bid % grid_m, tn = bid / grid_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  if (kbeg >= kend) return;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  OA oa;
  OB ob;
  // op(A)(m,k): A_KC -> A[m*lda+k] ; else A[k*lda+m].   op(B)(k,n): B_KC -> B[n*ldb+k] ; else B[k*ldb+n]
  oa.load(A, lda, m0, M, kbeg, kend);
  ob.load(B, ldb, n0, N, kbeg, kend);
  oa.store(sA[0]);
  ob.store(sB[0]);
  __syncthreads();

  const int nk = (kend - kbeg + BK - 1) / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      oa.load(A, lda, m0, M, kbeg + (kt + 1) * BK, kend);
      ob.load(B, ldb, n0, N, kbeg + (kt + 1) * BK, kend);
    }
    if constexpr (PREC == PREC_F32) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        float a0 = frag_f32<BK, A_KC>(sA[cur], wm, kk, lane);
        float a1 = frag_f32<BK, A_KC>(sA[cur], wm + 32, kk, lane);
        float b0 = frag_f32<BK, B_KC>(sB[cur], wn, kk, lane);
        float b1 = frag_f32<BK, B_KC>(sB[cur], wn + 32, kk, lane);
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 16) {
        bf16x8 a0 = frag_bf16<BK, A_KC>(sA[cur], wm, kk, lane);
        bf16x8 a1 = frag_bf16<BK, A_KC>(sA[cur], wm + 32, kk, lane);
        bf16x8 b0 = frag_bf16<BK, B_KC>(sB[cur], wn, kk, lane);
        bf16x8 b1 = frag_bf16<BK, B_KC>(sB[cur], wn + 32, kk, lane);
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) {
      oa.store(sA[cur ^ 1]);
      ob.store(sB[cur ^ 1]);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> row (r&3) + 8*(r>>2) + 4*(lane>>5), col lane&31
  const bool add_bias = bias && blockIdx.z == 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn + 32 * j + (lane & 31);
      if (col >= N) continue;
      const float bv = add_bias ? bias[col] : 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= M) continue;
        float v = acc[i][j][r] + bv;
        float* cp = C + (long long)row * ldc + col;
        if constexpr (ATOMIC) {
          atomicAdd(cp, v);
        } else {
          if (beta != 0.0f) v += beta * *cp;
          if (EPI == EPI_TANH) v = tanhf(v);
          *cp = v;
        }
      }
    }
}

// ---------------------------------------------------------------------------
// bf16 throughput kernel.  128x128x64 tiles, 256 threads (2x2 waves of 64x64,
// 2x2 v_mfma_f32_32x32x16_bf16 accumulators).  Both operands live in LDS as
// bf16 [row][k] (k contiguous, row stride 72 elements = 144 B: the 16-lane phases
// of every ds_read_b128 fragment read hit 16 distinct 4-bank groups), whatever
// their HBM layout: k-contiguous operands are read as 2 x float4 per 8-k chunk,
// row-contiguous ones as float4 over 4 rows x 8 k-rows and transposed in
// registers; fp32 -> bf16 by v_cvt_pk_bf16_f32 (RNE) at the LDS store.
// Global loads of tile k+1 (64 KB per workgroup) are in flight during the MFMAs
// of tile k (register prefetch into a single LDS buffer, two barriers per tile).  Tiles are mapped
// XCD-major (blockIdx % 8 = XCD): each XCD owns a contiguous N-major range of
// tiles, so the workgroups sharing an operand panel share an L2.
// ---------------------------------------------------------------------------
constexpr int GB_BK = 64, GB_LDK = GB_BK + 8;  // 144-B LDS rows

__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  __hip_bfloat162 v = __float22bfloat162_rn(make_float2(a, b));
  return *reinterpret_cast<unsigned*>(&v);
}

template <bool KC>
struct GOperand {
  float4 v[8];  // 32 fp32 of the next 128 x 64 k-tile
  // KC : chunks c = tid + 256 i (i < 4): row c >> 3, k 8 (c & 7) .. +8  -> v[2i], v[2i+1]
  // !KC: row group rg = tid & 31 (rows 4 rg..+4), k group kg = tid >> 5 (k 8 kg..+8) -> v[j] = k-row j
  __device__ __forceinline__ void load(const float* __restrict__ G, long long ld, int r0, int rmax, int k0, int kmax,
                                       bool vec) {
    const int t = threadIdx.x;
    if constexpr (KC) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = t + 256 * i;
        const int gr = r0 + (c >> 3), gk = k0 + 8 * (c & 7);
        const float* p = G + (long long)gr * ld + gk;
        if (vec && gr < rmax && gk + 8 <= kmax) {
          v[2 * i] = *reinterpret_cast<const float4*>(p);
          v[2 * i + 1] = *reinterpret_cast<const float4*>(p + 4);
        } else {
          float e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = (gr < rmax && gk + j < kmax) ? p[j] : 0.0f;
          v[2 * i] = make_float4(e[0], e[1], e[2], e[3]);
          v[2 * i + 1] = make_float4(e[4], e[5], e[6], e[7]);
        }
      }
    } else {
      const int gr = r0 + 4 * (t & 31), gk0 = k0 + 8 * (t >> 5);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int gk = gk0 + j;
        const float* p = G + (long long)gk * ld + gr;
        if (vec && gk < kmax && gr + 4 <= rmax) {
          v[j] = *reinterpret_cast<const float4*>(p);
        } else {
          float e[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) e[c] = (gk < kmax && gr + c < rmax) ? p[c] : 0.0f;
          v[j] = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
    }
  }
  __device__ __forceinline__ void store(unsigned short* __restrict__ s) const {
    const int t = threadIdx.x;
    if constexpr (KC) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = t + 256 * i;
        uint4 w;
        w.x = pk_bf16(v[2 * i].x, v[2 * i].y);
        w.y = pk_bf16(v[2 * i].z, v[2 * i].w);
        w.z = pk_bf16(v[2 * i + 1].x, v[2 * i + 1].y);
        w.w = pk_bf16(v[2 * i + 1].z, v[2 * i + 1].w);
        *reinterpret_cast<uint4*>(s + (c >> 3) * GB_LDK + 8 * (c & 7)) = w;
      }
    } else {
      const int r = 4 * (t & 31), k = 8 * (t >> 5);
      uint4 w[4];  // row r + c: k .. k+7
#define GB_ROW(c, f)                                                                          \
  w[c].x = pk_bf16(v[0].f, v[1].f); w[c].y = pk_bf16(v[2].f, v[3].f);                         \
  w[c].z = pk_bf16(v[4].f, v[5].f); w[c].w = pk_bf16(v[6].f, v[7].f);
      GB_ROW(0, x) GB_ROW(1, y) GB_ROW(2, z) GB_ROW(3, w)
#undef GB_ROW
#pragma unroll
      for (int c = 0; c < 4; ++c) *reinterpret_cast<uint4*>(s + (r + c) * GB_LDK + k) = w[c];
    }
  }
};

template <bool A_KC, bool B_KC, int EPI, bool ATOMIC>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(int M, int N, int K, const float* __restrict__ A,
                                                          long long lda, const float* __restrict__ B, long long ldb,
                                                          float* __restrict__ C, long long ldc,
                                                          const float* __restrict__ bias, float beta,
                                                          int k_per_split, int grid_m, int grid_n, int vec) {
  __shared__ __attribute__((aligned(16))) unsigned short sA[BM * GB_LDK];
  __shared__ __attribute__((aligned(16))) unsigned short sB[BN * GB_LDK];

  // XCD-major, then grouped: each XCD owns a contiguous range of the grouped tile
  // order (8 M-tiles x all N-tiles per group, M fastest), so the ~64 workgroups an
  // XCD runs at once cover an 8 x 8 block of tiles: 16 operand panels in its L2.
  const int ntiles = grid_m * grid_n;
  const int per_xcd = (ntiles + 7) / 8;
  const int tile = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  if (tile >= ntiles) return;
  constexpr int GROUP = 8;
  const int gsize = GROUP * grid_n;
  const int first_m = (tile / gsize) * GROUP;
  const int gm_here = min(grid_m - first_m, GROUP);
  const int tm = first_m + (tile % gsize) % gm_here, tn = (tile % gsize) / gm_here;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  if (kbeg >= kend) return;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  GOperand<A_KC> oa;
  GOperand<B_KC> ob;
  const bool va = vec & 1, vb = vec & 2;
  oa.load(A, lda, m0, M, kbeg, kend, va);
  ob.load(B, ldb, n0, N, kbeg, kend, vb);

  // single LDS buffer, register prefetch: tile k+1's global loads are in flight
  // during tile k's MFMAs (64 KB per workgroup, 2 workgroups per CU)
  const int nk = (kend - kbeg + GB_BK - 1) / GB_BK;
  const int fr = lane & 31, fk = 8 * (lane >> 5);
  for (int kt = 0; kt < nk; ++kt) {
    oa.store(sA);
    ob.store(sB);
    __syncthreads();
    if (kt + 1 < nk) {
      oa.load(A, lda, m0, M, kbeg + (kt + 1) * GB_BK, kend, va);
      ob.load(B, ldb, n0, N, kbeg + (kt + 1) * GB_BK, kend, vb);
    }
#pragma unroll
    for (int kk = 0; kk < GB_BK; kk += 16) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(sA + (wm + fr) * GB_LDK + kk + fk);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(sA + (wm + 32 + fr) * GB_LDK + kk + fk);
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(sB + (wn + fr) * GB_LDK + kk + fk);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(sB + (wn + 32 + fr) * GB_LDK + kk + fk);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> row (r&3) + 8*(r>>2) + 4*(lane>>5), col lane&31
  const bool add_bias = bias && blockIdx.z == 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn + 32 * j + (lane & 31);
      if (col >= N) continue;
      const float bv = add_bias ? bias[col] : 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= M) continue;
        float v = acc[i][j][r] + bv;
        float* cp = C + (long long)row * ldc + col;
        if constexpr (ATOMIC) {
          atomicAdd(cp, v);
        } else {
          if (beta != 0.0f) v += beta * *cp;
          if (EPI == EPI_TANH) v = tanhf(v);
          *cp = v;
        }
      }
    }
}

template <bool A_KC, bool B_KC>
int launch_bf16(int M, int N, int K, const float* A, long long lda, const float* B, long long ldb, float* C,
                long long ldc, const float* bias, int epi, float beta, int splitk, hipStream_t st) {
  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  if (splitk < 1) splitk = 1;
  int kps = (K + splitk - 1) / splitk;
  kps = (kps + GB_BK - 1) / GB_BK * GB_BK;
  splitk = (K + kps - 1) / kps;
  const int ntiles = gm * gn;
  dim3 grid(8 * ((ntiles + 7) / 8), 1, splitk);
  // 16-B vector loads need 16-B aligned rows (ld % 4 == 0) and base pointers
  const int vec = ((lda % 4 == 0 && ((uintptr_t)A & 15) == 0) ? 1 : 0) |
                  ((ldb % 4 == 0 && ((uintptr_t)B & 15) == 0) ? 2 : 0);
  if (splitk > 1) {
    if (epi != EPI_NONE || beta != 1.0f) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm_bf16_kernel<A_KC, B_KC, EPI_NONE, true>), grid, dim3(NT), 0, st, M, N, K, A, lda, B,
                       ldb, C, ldc, bias, beta, kps, gm, gn, vec);
  } else if (epi == EPI_TANH) {
    hipLaunchKernelGGL((gemm_bf16_kernel<A_KC, B_KC, EPI_TANH, false>), grid, dim3(NT), 0, st, M, N, K, A, lda, B,
                       ldb, C, ldc, bias, beta, kps, gm, gn, vec);
  } else {
    hipLaunchKernelGGL((gemm_bf16_kernel<A_KC, B_KC, EPI_NONE, false>), grid, dim3(NT), 0, st, M, N, K, A, lda, B,
                       ldb, C, ldc, bias, beta, kps, gm, gn, vec);
  }
  DL4SS_CHECK_LAUNCH();
  return 0;
}

template <bool A_KC, bool B_KC, int PREC>
int launch_prec(int M, int N, int K, const float* A, long long lda, const float* B, long long ldb, float* C,
                long long ldc, const float* bias, int epi, float beta, int splitk, hipStream_t st) {
  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  constexpr int BK = (PREC == PREC_F32) ? 16 : 32;
  if (splitk < 1) splitk = 1;
  int kps = (K + splitk - 1) / splitk;
  kps = (kps + BK - 1) / BK * BK;
  splitk = (K + kps - 1) / kps;
  dim3 grid(gm * gn, 1, splitk);
  if (splitk > 1) {
    // split-K accumulates into C (C += op(A) op(B)); no epilogue
    if (epi != EPI_NONE || beta != 1.0f) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm_kernel<A_KC, B_KC, PREC, EPI_NONE, true>), grid, dim3(NT), 0, st, M, N, K, A, lda, B,
                       ldb, C, ldc, bias, beta, kps, gm);
  } else if (epi == EPI_TANH) {
    hipLaunchKernelGGL((gemm_kernel<A_KC, B_KC, PREC, EPI_TANH, false>), grid, dim3(NT), 0, st, M, N, K, A, lda,
                       B, ldb, C, ldc, bias, beta, kps, gm);
  } else {
    hipLaunchKernelGGL((gemm_kernel<A_KC, B_KC, PREC, EPI_NONE, false>), grid, dim3(NT), 0, st, M, N, K, A, lda,
                       B, ldb, C, ldc, bias, beta, kps, gm);
  }
  DL4SS_CHECK_LAUNCH();
  return 0;
}

template <bool A_KC, bool B_KC>
int launch(int prec, int M, int N, int K, const float* A, long long lda, const float* B, long long ldb, float* C,
           long long ldc, const float* bias, int epi, float beta, int splitk, hipStream_t st) {
  if (prec == PREC_BF16)
    return launch_bf16<A_KC, B_KC>(M, N, K, A, lda, B, ldb, C, ldc, bias, epi, beta, splitk, st);
  return launch_prec<A_KC, B_KC, PREC_F32>(M, N, K, A, lda, B, ldb, C, ldc, bias, epi, beta, splitk, st);
}

}  // namespace

// C = op(A) op(B) (+ bias) (tanh) (+ beta C).  transA: A stored K x M (else M x K);
// transB: B stored N x K (else K x N).  Row-major, leading dimensions in elements.
DL4SS_API int dl4ss_gemm(int transA, int transB, int M, int N, int K, const float* A, long long lda,
                         const float* B, long long ldb, float* C, long long ldc, const float* bias, int epilogue,
                         float beta, int precision, int splitk, void* stream) {
  DL4SS_REQUIRE(M >= 0 && N >= 0 && K >= 0 && A && B && C);
  if (M == 0 || N == 0) return 0;
  hipStream_t st = as_stream(stream);
  const bool a_kc = !transA, b_kc = transB;
  if (a_kc && b_kc) return launch<true, true>(precision, M, N, K, A, lda, B, ldb, C, ldc, bias, epilogue, beta, splitk, st);
  if (a_kc && !b_kc) return launch<true, false>(precision, M, N, K, A, lda, B, ldb, C, ldc, bias, epilogue, beta, splitk, st);
  if (!a_kc && b_kc) return launch<false, true>(precision, M, N, K, A, lda, B, ldb, C, ldc, bias, epilogue, beta, splitk, st);
  return launch<false, false>(precision, M, N, K, A, lda, B, ldb, C, ldc, bias, epilogue, beta, splitk, st);
}
