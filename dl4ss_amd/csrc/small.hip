// Small fused kernels of the separation step: speaker queries (embedding gather +
// ADDJUST), their backward, bias column sums and the Adam update.
#include "common.h"

namespace {

// ---------------------------------------------------------------------------
// q[b,k] = Emb[idx[b,k]] (+ W_adj [mean_t h[b] ; Emb[idx[b,k]]])
//   SPEECH_EMBEDDING gather: TDAA_beta/main_run_sstune_EvalVer.py:355-360
//   ADDJUST: EvalVer.py:373-375 and 606-608 (q <- q + adjust(h, q)), no bias
// one workgroup per utterance: mean over T of h (B,T,D) then K tiny matvecs
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void query_fwd_kernel(const float* __restrict__ h, int T, int D,
                                                        const int* __restrict__ idx, const float* __restrict__ emb,
                                                        const float* __restrict__ wadj, int K, int W,
                                                        float* __restrict__ q, float* __restrict__ mean_out) {
  extern __shared__ float sm[];
  float* smean = sm;       // [D]
  float* se = sm + D;      // [K][W]
  const int b = blockIdx.x;
  const float* hb = h + (long long)b * T * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += hb[(long long)t * D + c];
    const float m = s / (float)T;
    smean[c] = m;
    if (mean_out) mean_out[(long long)b * D + c] = m;
  }
  for (int i = threadIdx.x; i < K * W; i += blockDim.x) {
    const int k = i / W, o = i % W;
    se[i] = emb[(long long)idx[b * K + k] * W + o];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * W; i += blockDim.x) {
    const int k = i / W, o = i % W;
    float v = se[i];
    if (wadj) {
      const float* wr = wadj + (long long)o * (D + W);
      float acc = 0.f;
      for (int c = 0; c < D; ++c) acc = fmaf(wr[c], smean[c], acc);
      for (int c = 0; c < W; ++c) acc = fmaf(wr[D + c], se[k * W + c], acc);
      v += acc;
    }
    q[((long long)b * K + k) * W + o] = v;
  }
}

// dEmb[idx] += dq + W_e^T dq ; dmean[b] = sum_k W_m^T dq[b,k] / T (broadcast grad into h)
__global__ __launch_bounds__(256) void query_bwd_rows_kernel(const float* __restrict__ dq, const int* __restrict__ idx,
                                                             const float* __restrict__ wadj, int T, int D, int K,
                                                             int W, float* __restrict__ demb,
                                                             float* __restrict__ dh_bcast) {
  const int b = blockIdx.x;
  extern __shared__ float sdq[];  // [K][W]
  for (int i = threadIdx.x; i < K * W; i += blockDim.x) sdq[i] = dq[(long long)b * K * W + i];
  __syncthreads();
  if (demb) {
    for (int i = threadIdx.x; i < K * W; i += blockDim.x) {
      const int k = i / W, c = i % W;
      float g = sdq[i];
      if (wadj)
        for (int o = 0; o < W; ++o) g = fmaf(wadj[(long long)o * (D + W) + D + c], sdq[k * W + o], g);
      atomicAdd(demb + (long long)idx[b * K + k] * W + c, g);
    }
  }
  if (wadj && dh_bcast) {
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      float g = 0.f;
      for (int k = 0; k < K; ++k)
        for (int o = 0; o < W; ++o) g = fmaf(wadj[(long long)o * (D + W) + c], sdq[k * W + o], g);
      dh_bcast[(long long)b * D + c] = g / (float)T;
    }
  }
}

// dW_adj[o][i] += sum_{b,k} dq[b,k,o] cat[b,k,i], cat = [mean_b ; Emb[idx[b,k]]]  (fixed order)
__global__ __launch_bounds__(256) void query_bwd_w_kernel(const float* __restrict__ dq, const int* __restrict__ idx,
                                                          const float* __restrict__ emb,
                                                          const float* __restrict__ mean, int B, int D, int K, int W,
                                                          float* __restrict__ dwadj) {
  const long long n = (long long)W * (D + W);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int o = (int)(e / (D + W)), i = (int)(e % (D + W));
    float acc = 0.f;
    for (int b = 0; b < B; ++b)
      for (int k = 0; k < K; ++k) {
        const float c = i < D ? mean[(long long)b * D + i] : emb[(long long)idx[b * K + k] * W + (i - D)];
        acc = fmaf(dq[((long long)b * K + k) * W + o], c, acc);
      }
    dwadj[e] += acc;
  }
}

// out[n] (+)= sum_m A[m*lda + n]   (bias gradients); block = 64 columns x 4 row lanes
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ A, long long lda, int M, int N,
                                                     int rows_per_block, float* __restrict__ out) {
  __shared__ float s[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int m0 = blockIdx.y * rows_per_block;
  const int m1 = min(M, m0 + rows_per_block);
  float acc = 0.f;
  if (c < N)
    for (int m = m0 + rl; m < m1; m += 4) acc += A[(long long)m * lda + c];
  s[rl][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rl == 0 && c < N) atomicAdd(out + c, s[0][threadIdx.x] + s[1][threadIdx.x] + s[2][threadIdx.x] + s[3][threadIdx.x]);
}

// torch.optim.Adam (weight_decay 0, amsgrad off; m via lerp as torch) on flat fp32 buffers
// (EvalVer.py:538-544,673-675: Adam(lr=2e-4), betas (0.9, 0.999), eps 1e-8)
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long long n,
                                                   float lr, float b1, float b2, float eps, float bc1, float bc2s) {
  const float step = lr / bc1;
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * blockDim.x * 4) {
    if (i + 3 < n) {
      float4 pp = *reinterpret_cast<float4*>(p + i);
      const float4 gg = *reinterpret_cast<const float4*>(g + i);
      float4 mm = *reinterpret_cast<float4*>(m + i);
      float4 vv = *reinterpret_cast<float4*>(v + i);
#define ADAM1(c)                                              \
  mm.c = mm.c + (1.f - b1) * (gg.c - mm.c);                    \
  vv.c = b2 * vv.c + (1.f - b2) * gg.c * gg.c;                 \
  pp.c -= step * (mm.c / (sqrtf(vv.c) / bc2s + eps));
      ADAM1(x) ADAM1(y) ADAM1(z) ADAM1(w)
#undef ADAM1
      *reinterpret_cast<float4*>(p + i) = pp;
      *reinterpret_cast<float4*>(m + i) = mm;
      *reinterpret_cast<float4*>(v + i) = vv;
    } else {
      for (long long j = i; j < n; ++j) {
        m[j] = m[j] + (1.f - b1) * (g[j] - m[j]);
        v[j] = b2 * v[j] + (1.f - b2) * g[j] * g[j];
        p[j] -= step * (m[j] / (sqrtf(v[j]) / bc2s + eps));
      }
    }
  }
}

}  // namespace

DL4SS_API int dl4ss_query_fwd(const float* h, int B, int T, int D, const int* idx, const float* emb,
                              const float* w_adj, int K, int W, float* q, float* mean_out, void* stream) {
  DL4SS_REQUIRE(h && idx && emb && q && B > 0 && T > 0 && D > 0 && K > 0 && W > 0);
  const size_t smem = sizeof(float) * (D + K * W);
  hipLaunchKernelGGL(query_fwd_kernel, dim3(B), dim3(256), smem, as_stream(stream), h, T, D, idx, emb, w_adj, K, W,
                     q, mean_out);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_query_bwd(const float* dq, int B, int T, int D, const int* idx, const float* emb,
                              const float* w_adj, const float* mean, int K, int W, float* d_emb, float* d_wadj,
                              float* dh_bcast, void* stream) {
  DL4SS_REQUIRE(dq && idx && B > 0 && K > 0 && W > 0);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(query_bwd_rows_kernel, dim3(B), dim3(256), sizeof(float) * K * W, st, dq, idx, w_adj, T, D, K,
                     W, d_emb, dh_bcast);
  DL4SS_CHECK_LAUNCH();
  if (w_adj && d_wadj) {
    DL4SS_REQUIRE(mean && emb);
    const long long n = (long long)W * (D + W);
    hipLaunchKernelGGL(query_bwd_w_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, dq, idx, emb, mean, B, D, K, W,
                       d_wadj);
    DL4SS_CHECK_LAUNCH();
  }
  return 0;
}

DL4SS_API int dl4ss_colsum(const float* A, long long lda, int M, int N, float* out, void* stream) {
  DL4SS_REQUIRE(A && out && M >= 0 && N >= 0);
  if (M == 0 || N == 0) return 0;
  const int rpb = 256;
  hipLaunchKernelGGL(colsum_kernel, dim3(cdiv(N, 64), cdiv(M, rpb)), dim3(256), 0, as_stream(stream), A, lda, M, N,
                     rpb, out);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                         float beta2, float eps, int step, void* stream) {
  DL4SS_REQUIRE(p && g && m && v && n >= 0 && step >= 1);
  if (n == 0) return 0;
  // bias corrections in double on the host, as torch computes them in Python floats
  const float bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, (double)step));
  const unsigned grid = (unsigned)min(8192LL, (n / 4 + 255) / 256 + 1);
  hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(256), 0, as_stream(stream), p, g, m, v, n, lr, beta1, beta2, eps,
                     bc1, bc2s);
  DL4SS_CHECK_LAUNCH();
  return 0;
}
