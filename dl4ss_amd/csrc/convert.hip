// fp32 -> bf16 operand copies and bf16 column sums of the bf16 training step.
//
// The bf16 step's GEMM operands are produced as bf16 in HBM (gemm_gl.hip reads them by LDS-DMA):
// the BiRNN kernels and the attention GRAD pass write theirs directly; the weights (W_ih of every
// layer and the Linear, one launch: dl4ss_f32_to_bf16_2d_multi) and the layer-0 features
// (dl4ss_f32_to_bf16_2d) are converted here once per step, rows zero-padded to a multiple of 8
// elements (16-B rows).  Rounding: nearest even, as every MFMA operand of the step.
// The Linear bias gradient is the column sum of bf16 dPre (dl4ss_colsum_bf16_det: per-256-row-block
// partials + a fixed-order reduce, bitwise reproducible; EvalVer.py:298 Linear.bias).
#include "common.h"

#include <algorithm>
#include <hip/hip_bf16.h>

namespace {

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, unsigned short* __restrict__ y, long long n) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= n) {
    const float4 v = *reinterpret_cast<const float4*>(x + i);
    __hip_bfloat162 lo2 = __float22bfloat162_rn(make_float2(v.x, v.y));
    __hip_bfloat162 hi2 = __float22bfloat162_rn(make_float2(v.z, v.w));
    const unsigned lo = *reinterpret_cast<unsigned*>(&lo2), hi = *reinterpret_cast<unsigned*>(&hi2);
    *reinterpret_cast<uint2*>(y + i) = make_uint2(lo, hi);
  } else {
    for (long long j = i; j < n; ++j) {
      y[j] = (unsigned short)bf16_bits_rne(x[j]);
    }
  }
}

__global__ void f32_to_bf16_2d_kernel(const float* __restrict__ x, long long ldx, int rows, int cols,
                                      unsigned short* __restrict__ y, long long ldy) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)rows * ldy) return;
  const long long r = i / ldy, c = i - r * ldy;
  unsigned short o = 0;
  if (c < cols) {
    o = (unsigned short)bf16_bits_rne(x[r * ldx + c]);
  }
  y[i] = o;
}

// Several row-padded fp32 -> bf16 conversions in one launch (the step's bf16 weight copies):
// segment i converts rows x cols of x[i] (row stride ldx) into y[i] (row stride ldy, zero
// padding beyond cols).
constexpr int CVT_MAX = 8;
struct CvtSegs {
  const float* x[CVT_MAX];
  unsigned short* y[CVT_MAX];
  long long ldx[CVT_MAX], ldy[CVT_MAX];
  int row0[CVT_MAX + 1];  // row prefix over the segments
  int cols[CVT_MAX];
  int vec[CVT_MAX];       // 16-B aligned rows of x and y (8-column chunks)
  int n;
};
// one wave per row (four rows per workgroup, rows of every segment in sequence).  vec segments
// (16-B aligned x and y rows): each lane converts 8-column chunks with two 16-B loads and one 16-B
// store (a workgroup per row with one 4-B pair per thread ran at ~2.8 TB/s); otherwise pairs of
// columns as one 4-B word (ldy even).  Columns >= cols are zero either way.
__device__ __forceinline__ unsigned bf16_bits(float f) { return bf16_bits_rne(f); }
__global__ __launch_bounds__(256) void f32_to_bf16_multi_kernel(CvtSegs sg) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= sg.row0[sg.n]) return;
  int g = 0;
#pragma unroll
  for (int j = 1; j < CVT_MAX; ++j) g += (j < sg.n && row >= sg.row0[j]) ? 1 : 0;
  const long long r = row - sg.row0[g];
  const float* xr = sg.x[g] + r * sg.ldx[g];
  const int cols = sg.cols[g];
  if (sg.vec[g]) {
    uint4* yr = reinterpret_cast<uint4*>(sg.y[g] + r * sg.ldy[g]);
    const int nc = (int)(sg.ldy[g] >> 3);
    for (int q = lane; q < nc; q += 64) {
      const int c = 8 * q;
      float v[8];
      if (c + 8 <= cols) {
        const float4 a = *reinterpret_cast<const float4*>(xr + c), b = *reinterpret_cast<const float4*>(xr + c + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = c + e < cols ? xr[c + e] : 0.0f;
      }
      unsigned w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        w[e] = (c + 2 * e < cols ? bf16_bits(v[2 * e]) : 0u) | ((c + 2 * e + 1 < cols ? bf16_bits(v[2 * e + 1]) : 0u) << 16);
      }
      yr[q] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return;
  }
  unsigned* yr = reinterpret_cast<unsigned*>(sg.y[g] + r * sg.ldy[g]);
  const int np = (int)(sg.ldy[g] >> 1);
  for (int p = lane; p < np; p += 64) {
    const int c = 2 * p;
    const unsigned lo = c < cols ? bf16_bits(xr[c]) : 0u;
    const unsigned hi = c + 1 < cols ? bf16_bits(xr[c + 1]) : 0u;
    yr[p] = lo | (hi << 16);
  }
}

// out[n] += sum_m A[m*lda + n] for bf16 A (bias gradients from bf16 dPre); VEC: 8 columns per
// lane with 16-B loads (lda % 8 == 0, aligned base), a 64-lane row segment covers 512 columns.
// part == nullptr: float atomics into out (order-dependent); else every row block stores its
// sums to part[blockIdx.y][N] and colsum_reduce_kernel adds the blocks in fixed order.
template <bool VEC>
__global__ __launch_bounds__(256) void colsum_bf16_v_kernel(const unsigned short* __restrict__ A, long long lda, int M,
                                                            int N, int rows_per_block, float* __restrict__ out,
                                                            float* __restrict__ part) {
  constexpr int CPL = VEC ? 8 : 1;
  __shared__ float s[4][64 * CPL];
  const int c0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * CPL;
  const int rl = threadIdx.x >> 6;
  const int m0 = blockIdx.y * rows_per_block;
  const int m1 = min(M, m0 + rows_per_block);
  float acc[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) acc[j] = 0.f;
  if (c0 < N) {
    if constexpr (VEC) {
      for (int m = m0 + rl; m < m1; m += 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(A + (long long)m * lda + c0);
        const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[2 * j] += __uint_as_float(w[j] << 16);
          acc[2 * j + 1] += __uint_as_float(w[j] & 0xFFFF0000u);
        }
      }
    } else {
      for (int m = m0 + rl; m < m1; m += 4) acc[0] += __uint_as_float((unsigned)A[(long long)m * lda + c0] << 16);
    }
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j) s[rl][(threadIdx.x & 63) * CPL + j] = acc[j];
  __syncthreads();
  if (rl == 0)
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int l = (threadIdx.x & 63) * CPL + j;
      if (c0 + j >= N) continue;
      const float v = (s[0][l] + s[1][l]) + (s[2][l] + s[3][l]);
      if (part)
        part[(long long)blockIdx.y * N + c0 + j] = v;
      else
        atomicAdd(out + c0 + j, v);
    }
}

// out[n] += sum_{y < nby} part[y][n], y in order (the deterministic colsum's second pass)
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ part, int nby, int N,
                                                            float* __restrict__ out, float beta) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float a = 0.f;
  for (int y = 0; y < nby; ++y) a += part[(long long)y * N + n];
  out[n] = beta != 0.f ? a + beta * out[n] : a;  // beta 0: out is not read (the step's unzeroed gradient)
}

// Split-precision operand images: x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (|lo| <= 2^-9 |x|,
// x - hi - lo <= 2^-17 |x|).  Segment s of a row (width segw >= cols, zero beyond cols) holds hi or lo
// by bit s of `pattern`; one thread per (row, column < segw) writes all nseg segments, then zeros up
// to ldy.  The K-concatenated product [x_hi | x_lo | x_hi] . [w_hi | w_hi | w_lo] = x w - x_lo w_lo
// - (rounding of lo) is fp32-accurate to ~2^-16 relative: one bf16 MFMA GEMM with K' = 3K.
__global__ __launch_bounds__(256) void f32_to_bf16_hilo_kernel(const float* __restrict__ x, long long ldx, int rows,
                                                               int cols, unsigned short* __restrict__ y,
                                                               long long ldy, int segw, int nseg, unsigned pattern) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int wrow = max(segw, (int)(ldy - (long long)(nseg - 1) * segw));  // the last segment also zeroes the tail
  if (i >= (long long)rows * wrow) return;
  const long long r = i / wrow;
  const int c = (int)(i - r * wrow);
  unsigned short hi = 0, lo = 0;
  if (c < cols) {
    const float v = x[r * ldx + c];
    const unsigned hb = bf16_bits_rne(v);
    hi = (unsigned short)hb;
    lo = (unsigned short)bf16_bits_rne(v - __uint_as_float(hb << 16));
  }
  unsigned short* yr = y + r * ldy;
  for (int sg = 0; sg < nseg; ++sg) {
    const long long col = (long long)sg * segw + c;
    if ((c < segw || sg == nseg - 1) && col < ldy) yr[col] = ((pattern >> sg) & 1u) ? lo : hi;
  }
}

}  // namespace

DL4SS_API int dl4ss_f32_to_bf16_hilo(const float* x, long long ldx, int rows, int cols, void* y, long long ldy,
                                     int segw, int nseg, unsigned pattern, void* stream) {
  DL4SS_REQUIRE(x && y && rows >= 0 && cols >= 0 && ldx >= cols && segw >= cols && nseg >= 1 && nseg <= 8);
  DL4SS_REQUIRE(ldy >= (long long)nseg * segw);
  if (rows == 0) return 0;
  const int wrow = (int)std::max<long long>(segw, ldy - (long long)(nseg - 1) * segw);
  const long long n = (long long)rows * wrow;
  hipLaunchKernelGGL(f32_to_bf16_hilo_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), x,
                     ldx, rows, cols, reinterpret_cast<unsigned short*>(y), ldy, segw, nseg, pattern);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

// y[r*ldy + c] = bf16(x[r*ldx + c]) for c < cols, 0 for cols <= c < ldy (row padding for 16-B rows)
DL4SS_API int dl4ss_f32_to_bf16_2d(const float* x, long long ldx, int rows, int cols, void* y, long long ldy,
                                   void* stream) {
  DL4SS_REQUIRE(x && y && rows >= 0 && cols >= 0 && ldx >= cols && ldy >= cols);
  if (rows == 0) return 0;
  const long long n = (long long)rows * ldy;
  hipLaunchKernelGGL(f32_to_bf16_2d_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), x,
                     ldx, rows, cols, reinterpret_cast<unsigned short*>(y), ldy);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

static int colsum_bf16_launch(const void* A, long long lda, int M, int N, float* out, float* part, void* stream,
                              float beta = 1.f) {
  const int rpb = 256;
  const auto* a = reinterpret_cast<const unsigned short*>(A);
  if (lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && lda >= ((N + 7) & ~7))  // 16-B rows, padding readable
    hipLaunchKernelGGL(colsum_bf16_v_kernel<true>, dim3(cdiv(N, 512), cdiv(M, rpb)), dim3(256), 0, as_stream(stream),
                       a, lda, M, N, rpb, out, part);
  else
    hipLaunchKernelGGL(colsum_bf16_v_kernel<false>, dim3(cdiv(N, 64), cdiv(M, rpb)), dim3(256), 0, as_stream(stream),
                       a, lda, M, N, rpb, out, part);
  DL4SS_CHECK_LAUNCH();
  if (part) {
    hipLaunchKernelGGL(colsum_reduce_kernel, dim3(cdiv(N, 256)), dim3(256), 0, as_stream(stream), part, cdiv(M, rpb), N,
                       out, beta);
    DL4SS_CHECK_LAUNCH();
  }
  return 0;
}

DL4SS_API int dl4ss_colsum_bf16(const void* A, long long lda, int M, int N, float* out, void* stream) {
  DL4SS_REQUIRE(A && out && M >= 0 && N >= 0);
  if (M == 0 || N == 0) return 0;
  return colsum_bf16_launch(A, lda, M, N, out, nullptr, stream);
}

// Bytes of the partial-sum workspace dl4ss_colsum_bf16_det needs for an M x N operand.
DL4SS_API long long dl4ss_colsum_bf16_part_bytes(int M, int N) {
  return M > 0 && N > 0 ? (long long)cdiv(M, 256) * N * 4 : 0;
}

// Deterministic dl4ss_colsum_bf16: per-256-row-block partial sums, then a fixed-order reduce
// (the bf16 step's Linear bias gradient: bitwise reproducible run to run).
DL4SS_API int dl4ss_colsum_bf16_det(const void* A, long long lda, int M, int N, float* out, float* part,
                                    long long part_bytes, void* stream) {
  DL4SS_REQUIRE(A && out && M >= 0 && N >= 0);
  if (M == 0 || N == 0) return 0;
  DL4SS_REQUIRE(part && part_bytes >= dl4ss_colsum_bf16_part_bytes(M, N));
  return colsum_bf16_launch(A, lda, M, N, out, part, stream);
}

// dl4ss_colsum_bf16_det with out = beta out + sums (beta 0: out is written without being read)
DL4SS_API int dl4ss_colsum_bf16_det_ex(const void* A, long long lda, int M, int N, float* out, float* part,
                                       long long part_bytes, float beta, void* stream) {
  DL4SS_REQUIRE(A && out && M >= 0 && N >= 0);
  if (N == 0) return 0;
  if (M == 0) {  // an empty sum: out = beta out (beta 0: zeros)
    DL4SS_REQUIRE(beta == 0.f || beta == 1.f);
    return beta == 0.f ? (int)hipMemsetAsync(out, 0, sizeof(float) * (size_t)N, as_stream(stream)) : 0;
  }
  DL4SS_REQUIRE(part && part_bytes >= dl4ss_colsum_bf16_part_bytes(M, N));
  return colsum_bf16_launch(A, lda, M, N, out, part, stream, beta);
}

DL4SS_API int dl4ss_f32_to_bf16_2d_multi(int n, const float* const* x, const long long* ldx, const int* rows,
                                         const int* cols, void* const* y, const long long* ldy, void* stream) {
  DL4SS_REQUIRE(n >= 1 && n <= CVT_MAX && x && ldx && rows && cols && y && ldy);
  CvtSegs sg{};
  sg.n = n;
  sg.row0[0] = 0;
  for (int i = 0; i < n; ++i) {
    DL4SS_REQUIRE(x[i] && y[i] && rows[i] >= 0 && cols[i] >= 0 && ldx[i] >= cols[i] && ldy[i] >= cols[i] && ldy[i] > 0);
    DL4SS_REQUIRE(ldy[i] % 2 == 0 && ((uintptr_t)y[i] & 3) == 0);  // 4-B pair stores
    sg.x[i] = x[i];
    sg.y[i] = reinterpret_cast<unsigned short*>(y[i]);
    sg.ldx[i] = ldx[i];
    sg.ldy[i] = ldy[i];
    sg.cols[i] = cols[i];
    sg.vec[i] = (((uintptr_t)x[i] & 15) == 0 && ldx[i] % 4 == 0 && ((uintptr_t)y[i] & 15) == 0 && ldy[i] % 8 == 0) ? 1 : 0;
    sg.row0[i + 1] = sg.row0[i] + rows[i];
  }
  for (int i = n + 1; i <= CVT_MAX; ++i) sg.row0[i] = sg.row0[n];
  if (sg.row0[n] == 0) return 0;
  hipLaunchKernelGGL(f32_to_bf16_multi_kernel, dim3(cdiv(sg.row0[n], 4)), dim3(256), 0, as_stream(stream), sg);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

// y = bf16(x), round to nearest even (the rounding gemm.hip applies at its LDS store).
DL4SS_API int dl4ss_f32_to_bf16(const float* x, void* y, long long n, void* stream) {
  DL4SS_REQUIRE(n >= 0 && (n == 0 || (x && y)));
  if (n == 0) return 0;
  DL4SS_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 7) == 0);
  const long long threads = (n + 3) / 4;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, as_stream(stream), x,
                     reinterpret_cast<unsigned short*>(y), n);
  DL4SS_CHECK_LAUNCH();
  return 0;
}
