// Kernels behind the reference-API modules (dl4ss_amd/compat/myNet.py): the pieces
// a driver written against the reference's nn.Modules composes with autograd, where
// the fused training step (SepTrainer) keeps them inside larger kernels.
//
//   dl4ss_tanh_bwd      d(tanh(pre)) for MIX_SPEECH's Linear + tanh
//                       (TDAA_beta/main_run_sstune_EvalVer.py:290,298-299)
//   dl4ss_attn_dot_fwd  ATTENTION 'dot': mask = sigmoid(V . q)   (EvalVer.py:216-226), or the
//                       cRM branch's 10 tanh(V . q_half)          (cRM_EvalVer.py:259-271)
//   dl4ss_attn_dot_bwd  its backward: dV = dE q, dq = sum_r dE V, dE = dmask act'(e)
//   dl4ss_top_k_mask    top_k_mask (EvalVer.py:390-405, Torch_multi/main_run.py:340-355)
//                       on device: no sort, no host loop
//   dl4ss_classifier_select  the speaker choice of the recursive extraction loop
//                       (Torch_multi/main_run_multi_selfSS_recuReal_GRID.py:227-244,391-404):
//                       sigmoid of the classifier logits, descending top-k order, first
//                       not-yet-extracted speaker -- on device, no host round trip
//   dl4ss_mask_split    pred = m X and residual (1 - m) X in one pass (GRID.py:433-444)
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void tanh_bwd_kernel(const float* __restrict__ v, const float* __restrict__ dv,
                                                       float* __restrict__ dpre, long long n) {
  for (long long i = (blockIdx.x * 256LL + threadIdx.x) * 4; i < n; i += (long long)gridDim.x * 1024) {
    if (i + 3 < n) {
      const float4 a = *reinterpret_cast<const float4*>(v + i);
      const float4 g = *reinterpret_cast<const float4*>(dv + i);
      *reinterpret_cast<float4*>(dpre + i) =
          make_float4(g.x * (1.f - a.x * a.x), g.y * (1.f - a.y * a.y), g.z * (1.f - a.z * a.z), g.w * (1.f - a.w * a.w));
    } else {
      for (long long j = i; j < n; ++j) dpre[j] = dv[j] * (1.f - v[j] * v[j]);
    }
  }
}

// one thread per row r of V (Bq, R, E): mask[b][r] = sigmoid(sum_e V[b][r][e] q[b][e])
constexpr float CRM_K = 10.0f;  // cRM_EvalVer.py:28

template <int E>
__global__ __launch_bounds__(256) void attn_dot_fwd_kernel(const float* __restrict__ V, const float* __restrict__ q,
                                                           int q_stride, int R, int act, float* __restrict__ mask,
                                                           long long mask_stride) {
  __shared__ float sq[E];
  const int b = blockIdx.y;
  if (threadIdx.x < E) sq[threadIdx.x] = q[(long long)b * q_stride + threadIdx.x];
  __syncthreads();
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const float* vr = V + ((long long)b * R + r) * E;
  float acc = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) acc = fmaf(vr[e], sq[e], acc);
  mask[b * mask_stride + r] = act == 0 ? 1.0f / (1.0f + __expf(-acc)) : CRM_K * tanhf(acc);
}

// dE = dmask m (1-m); dV[b][r][:] = dE q[b]; per-block partial dq (fixed order, no atomics)
template <int E>
__global__ __launch_bounds__(256) void attn_dot_bwd_kernel(const float* __restrict__ V, const float* __restrict__ q,
                                                           int q_stride, const float* __restrict__ mask,
                                                           const float* __restrict__ dmask, int R, int act,
                                                           float* __restrict__ dV, float* __restrict__ part_dq) {
  __shared__ float sq[E];
  __shared__ float sp[4][E];
  const int b = blockIdx.y;
  if (threadIdx.x < E) sq[threadIdx.x] = q[(long long)b * q_stride + threadIdx.x];
  __syncthreads();
  const int r = blockIdx.x * 256 + threadIdx.x;
  float de = 0.f;
  const float* vr = V + ((long long)b * R + r) * E;
  if (r < R) {
    const float m = mask[(long long)b * R + r];
    const float t = m * (1.0f / CRM_K);
    de = dmask[(long long)b * R + r] * (act == 0 ? m * (1.f - m) : CRM_K * (1.f - t * t));
    if (dV) {  // accumulate: the cRM branch's two halves both feed dV
      float* dvr = dV + ((long long)b * R + r) * E;
#pragma unroll
      for (int e = 0; e < E; ++e) dvr[e] = fmaf(de, sq[e], dvr[e]);
    }
  }
  // dq partial over this block's rows: wave sums then fixed-order combine
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int e = 0; e < E; ++e) {
    const float c = wave_sum(r < R ? de * vr[e] : 0.f);
    if (l == 0) sp[w][e] = c;
  }
  __syncthreads();
  if (threadIdx.x < E)
    part_dq[((long long)b * gridDim.x + blockIdx.x) * E + threadIdx.x] =
        (sp[0][threadIdx.x] + sp[1][threadIdx.x]) + (sp[2][threadIdx.x] + sp[3][threadIdx.x]);
}

__global__ __launch_bounds__(256) void attn_dot_dq_kernel(const float* __restrict__ part_dq, int nblk, int E, int Bq,
                                                          float* __restrict__ dq) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Bq * E) return;
  const int b = i / E, e = i % E;
  float s = 0.f;
  for (int k = 0; k < nblk; ++k) s += part_dq[((long long)b * nblk + k) * E + e];
  dq[i] = s;
}

// One workgroup per row of N probabilities.  Element i's descending rank is the
// number of elements larger than it (ties: lower index first, a stable sort).
// Selected: rank < min(top_k, #elements > alpha)  (the reference takes the first
// `count` of the top_k sorted ids).  Also writes the selected ids in ascending
// index order (np.where(line == 1), EvalVer.py:605) and their count.
__global__ __launch_bounds__(256) void top_k_mask_kernel(const float* __restrict__ prob, int N, float alpha, int top_k,
                                                         float* __restrict__ mask, int* __restrict__ idx,
                                                         int* __restrict__ count) {
  extern __shared__ float sp[];  // [N] probabilities, then [N] selection flags as int
  int* ssel = reinterpret_cast<int*>(sp + N);
  __shared__ int s_cnt;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) s_cnt = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) sp[i] = prob[(long long)b * N + i];
  __syncthreads();
  int above = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) above += sp[i] > alpha ? 1 : 0;
  atomicAdd(&s_cnt, above);
  __syncthreads();
  const int lim = min(top_k, s_cnt);
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float pi = sp[i];
    int rank = 0;
    for (int j = 0; j < N; ++j) {
      const float pj = sp[j];
      rank += (pj > pi || (pj == pi && j < i)) ? 1 : 0;
    }
    const int sel = rank < lim ? 1 : 0;
    ssel[i] = sel;
    mask[(long long)b * N + i] = (float)sel;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // ascending id list (N is small: the label count)
    int c = 0;
    for (int i = 0; i < N; ++i)
      if (ssel[i]) {
        if (idx && c < top_k) idx[(long long)b * top_k + c] = i;
        ++c;
      }
    if (idx)
      for (int k = c; k < top_k; ++k) idx[(long long)b * top_k + k] = -1;
    if (count) count[b] = c;
  }
}

// One workgroup per row b: prob = sigmoid(logit) (the classifier head's F.sigmoid,
// GRID.py:197); sort_index[b][0..top_k) = ids by descending prob (ties: lower id first,
// -1 beyond N); chosen[b] = the first of them not in prev[0..n_prev)[b] when at least
// one prob exceeds alpha (GRID.py:237-238: otherwise the loop has nothing to extract),
// else -1.
__global__ __launch_bounds__(256) void classifier_select_kernel(const float* __restrict__ logits, int N, float alpha,
                                                                int top_k, const int* __restrict__ prev, int n_prev,
                                                                float* __restrict__ prob, int* __restrict__ sort_index,
                                                                int* __restrict__ chosen) {
  extern __shared__ float sp[];  // [N] probabilities
  __shared__ int s_cnt;
  __shared__ int s_top[64];
  const int b = blockIdx.x;
  if (threadIdx.x == 0) s_cnt = 0;
  if (threadIdx.x < 64) s_top[threadIdx.x] = -1;
  __syncthreads();
  int above = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float p = 1.0f / (1.0f + expf(-logits[(long long)b * N + i]));
    sp[i] = p;
    above += p > alpha ? 1 : 0;
    if (prob) prob[(long long)b * N + i] = p;
  }
  atomicAdd(&s_cnt, above);
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float pi = sp[i];
    int rank = 0;
    for (int j = 0; j < N; ++j) {
      const float pj = sp[j];
      rank += (pj > pi || (pj == pi && j < i)) ? 1 : 0;
    }
    if (rank < top_k) s_top[rank] = i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int pick = -1;
    for (int r = 0; r < top_k; ++r) {
      const int k = s_top[r];
      if (sort_index) sort_index[(long long)b * top_k + r] = k;
      if (pick >= 0 || k < 0 || s_cnt == 0) continue;
      bool seen = false;
      for (int p = 0; p < n_prev; ++p) seen |= prev[(long long)p * gridDim.x + b] == k;
      if (!seen) pick = k;
    }
    if (chosen) chosen[b] = pick;
  }
}

// pred = m x, resid = (1 - m) x (either output may be null); 4 elements per thread
__global__ __launch_bounds__(256) void mask_split_kernel(const float* __restrict__ m, const float* __restrict__ x,
                                                         long long n, float* __restrict__ pred,
                                                         float* __restrict__ resid, bool vec) {
  for (long long i = (blockIdx.x * 256LL + threadIdx.x) * 4; i < n; i += (long long)gridDim.x * 1024) {
    if (vec && i + 3 < n) {
      const float4 a = *reinterpret_cast<const float4*>(m + i);
      const float4 v = *reinterpret_cast<const float4*>(x + i);
      if (pred) *reinterpret_cast<float4*>(pred + i) = make_float4(a.x * v.x, a.y * v.y, a.z * v.z, a.w * v.w);
      if (resid)
        *reinterpret_cast<float4*>(resid + i) =
            make_float4((1.f - a.x) * v.x, (1.f - a.y) * v.y, (1.f - a.z) * v.z, (1.f - a.w) * v.w);
    } else {
      for (long long j = i; j < n && j < i + 4; ++j) {
        if (pred) pred[j] = m[j] * x[j];
        if (resid) resid[j] = (1.f - m[j]) * x[j];
      }
    }
  }
}

}  // namespace

DL4SS_API int dl4ss_tanh_bwd(const float* v, const float* dv, float* dpre, long long n, void* stream) {
  DL4SS_REQUIRE(v && dv && dpre && n >= 0);
  if (n == 0) return 0;
  const unsigned grid = (unsigned)min(16384LL, cdiv(n, 1024));
  hipLaunchKernelGGL(tanh_bwd_kernel, dim3(grid), dim3(256), 0, as_stream(stream), v, dv, dpre, n);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_attn_dot_nblk(int R) { return (int)cdiv(R, 256); }

DL4SS_API int dl4ss_attn_dot_fwd_ex(const float* V, const float* q, int q_stride, int Bq, int R, int E, int act,
                                    float* mask, long long mask_stride, void* stream) {
  DL4SS_REQUIRE(V && q && mask && Bq >= 0 && R >= 0 && E == 50 && q_stride >= E && (act == 0 || act == 1));
  DL4SS_REQUIRE(mask_stride >= R);
  if (Bq == 0 || R == 0) return 0;
  hipLaunchKernelGGL(attn_dot_fwd_kernel<50>, dim3(cdiv(R, 256), Bq), dim3(256), 0, as_stream(stream), V, q, q_stride,
                     R, act, mask, mask_stride);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_attn_dot_fwd(const float* V, const float* q, int q_stride, int Bq, int R, int E, int act,
                                 float* mask, void* stream) {
  return dl4ss_attn_dot_fwd_ex(V, q, q_stride, Bq, R, E, act, mask, R, stream);
}

DL4SS_API int dl4ss_classifier_select(const float* logits, int B, int N, float alpha, int top_k, const int* prev,
                                      int n_prev, float* prob, int* sort_index, int* chosen, void* stream) {
  DL4SS_REQUIRE(logits && B >= 0 && N > 0 && N <= 8192 && top_k >= 1 && top_k <= 64 && n_prev >= 0);
  DL4SS_REQUIRE(n_prev == 0 || prev);
  if (B == 0) return 0;
  hipLaunchKernelGGL(classifier_select_kernel, dim3(B), dim3(256), sizeof(float) * N, as_stream(stream), logits, N,
                     alpha, top_k, prev, n_prev, prob, sort_index, chosen);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_mask_split(const float* mask, const float* x, long long n, float* pred, float* resid,
                               void* stream) {
  DL4SS_REQUIRE(mask && x && n >= 0 && (pred || resid));
  if (n == 0) return 0;
  const bool vec = ((uintptr_t)mask | (uintptr_t)x | (uintptr_t)pred | (uintptr_t)resid) % 16 == 0;
  const unsigned grid = (unsigned)min(16384LL, cdiv(n, 1024));
  hipLaunchKernelGGL(mask_split_kernel, dim3(grid), dim3(256), 0, as_stream(stream), mask, x, n, pred, resid, vec);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_attn_dot_bwd(const float* V, const float* q, int q_stride, const float* mask, const float* dmask,
                                 int Bq, int R, int E, int act, float* dV, float* part_dq, float* dq, void* stream) {
  DL4SS_REQUIRE(V && q && mask && dmask && part_dq && dq && Bq >= 0 && R >= 0 && E == 50 && q_stride >= E);
  if (Bq == 0 || R == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int nblk = (int)cdiv(R, 256);
  hipLaunchKernelGGL(attn_dot_bwd_kernel<50>, dim3(nblk, Bq), dim3(256), 0, st, V, q, q_stride, mask, dmask, R, act,
                     dV, part_dq);
  DL4SS_CHECK_LAUNCH();
  hipLaunchKernelGGL(attn_dot_dq_kernel, dim3(cdiv((long long)Bq * E, 256)), dim3(256), 0, st, part_dq, nblk, E, Bq,
                     dq);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_top_k_mask(const float* prob, int B, int N, float alpha, int top_k, float* mask, int* idx,
                               int* count, void* stream) {
  DL4SS_REQUIRE(prob && mask && B >= 0 && N > 0 && top_k >= 0 && N <= 8192);
  if (B == 0) return 0;
  hipLaunchKernelGGL(top_k_mask_kernel, dim3(B), dim3(256), sizeof(float) * 2 * N, as_stream(stream), prob, N, alpha,
                     top_k, mask, idx, count);
  DL4SS_CHECK_LAUNCH();
  return 0;
}
