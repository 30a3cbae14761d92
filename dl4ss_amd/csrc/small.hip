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
// mean_t h[b, :, c]: block = 64 columns x 4 time phases, grid (B, ceil(D/64));
// each thread keeps 4 independent loads in flight, phases combined in fixed order
__global__ __launch_bounds__(256) void time_mean_kernel(const float* __restrict__ h, int T, int D,
                                                        float* __restrict__ mean_out) {
  __shared__ float sp[4][64];
  const int b = blockIdx.x;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  const float* hb = h + (long long)b * T * D + c;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < D) {
    int t = ph;
    for (; t + 12 < T; t += 16) {
      s0 += hb[(long long)t * D];
      s1 += hb[(long long)(t + 4) * D];
      s2 += hb[(long long)(t + 8) * D];
      s3 += hb[(long long)(t + 12) * D];
    }
    for (; t < T; t += 4) s0 += hb[(long long)t * D];
  }
  sp[ph][threadIdx.x & 63] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ph == 0 && c < D) {
    const int l = threadIdx.x;
    mean_out[(long long)b * D + c] = ((sp[0][l] + sp[1][l]) + (sp[2][l] + sp[3][l])) / (float)T;
  }
}

// one workgroup per utterance: K*W outputs, each a (D + W)-long dot product
__global__ __launch_bounds__(256) void query_fwd_kernel(const float* __restrict__ mean, int D,
                                                        const int* __restrict__ idx, const float* __restrict__ emb,
                                                        const float* __restrict__ wadj, int K, int W,
                                                        float* __restrict__ q) {
  extern __shared__ float sm[];
  float* smean = sm;       // [D]
  float* se = sm + D;      // [K][W]
  const int b = blockIdx.x;
  if (wadj)
    for (int c = threadIdx.x; c < D; c += blockDim.x) smean[c] = mean[(long long)b * D + c];
  for (int i = threadIdx.x; i < K * W; i += blockDim.x) {
    const int k = i / W, o = i % W;
    const int id = idx[b * K + k];
    se[i] = id >= 0 ? emb[(long long)id * W + o] : 0.0f;  // id -1: no speaker (zero query)
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * W; i += blockDim.x) {
    const int k = i / W, o = i % W;
    float v = se[i];
    if (wadj) {
      const float* wr = wadj + (long long)o * (D + W);
      float a0 = 0.f, a1 = 0.f;
      int c = 0;
      for (; c + 1 < D; c += 2) {
        a0 = fmaf(wr[c], smean[c], a0);
        a1 = fmaf(wr[c + 1], smean[c + 1], a1);
      }
      for (; c < D; ++c) a0 = fmaf(wr[c], smean[c], a0);
      for (c = 0; c < W; ++c) a1 = fmaf(wr[D + c], se[k * W + c], a1);
      v += a0 + a1;
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
  DL4SS_REQUIRE(!w_adj || mean_out);  // ADJUST needs the time mean (also saved for the backward)
  hipStream_t st = as_stream(stream);
  if (mean_out) {
    hipLaunchKernelGGL(time_mean_kernel, dim3(B, cdiv(D, 64)), dim3(256), 0, st, h, T, D, mean_out);
    DL4SS_CHECK_LAUNCH();
  }
  const size_t smem = sizeof(float) * (D + K * W);
  hipLaunchKernelGGL(query_fwd_kernel, dim3(B), dim3(256), smem, st, mean_out, D, idx, emb, w_adj, K, W, q);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_time_mean(const float* h, int B, int T, int D, float* mean_out, void* stream) {
  DL4SS_REQUIRE(h && mean_out && B >= 0 && T > 0 && D > 0);
  if (B == 0) return 0;
  hipLaunchKernelGGL(time_mean_kernel, dim3(B, cdiv(D, 64)), dim3(256), 0, as_stream(stream), h, T, D, mean_out);
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
