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
// mean_t h[b, :, c]: block = 64 columns x 16 time phases (1024 threads), grid (B, ceil(D/64));
// each thread sums t = ph, ph + 16, ... with 4 independent loads in flight, the 16 phases are
// combined by a fixed tree.  (4 phases of 256 threads kept too few loads in flight per CU: 11.8 us
// for the 19 MB of the C2 step.)
constexpr int TM_PH = 16;
__global__ __launch_bounds__(64 * TM_PH) void time_mean_kernel(const float* __restrict__ h, int T, int D,
                                                               float* __restrict__ mean_out) {
  __shared__ float sp[TM_PH][64];
  const int b = blockIdx.x;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  const float* hb = h + (long long)b * T * D + c;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < D) {
    int t = ph;
    for (; t + 3 * TM_PH < T; t += 4 * TM_PH) {
      s0 += hb[(long long)t * D];
      s1 += hb[(long long)(t + TM_PH) * D];
      s2 += hb[(long long)(t + 2 * TM_PH) * D];
      s3 += hb[(long long)(t + 3 * TM_PH) * D];
    }
    for (; t < T; t += TM_PH) s0 += hb[(long long)t * D];
  }
  sp[ph][threadIdx.x & 63] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ph == 0 && c < D) {
    const int l = threadIdx.x;
    float v[TM_PH];
#pragma unroll
    for (int i = 0; i < TM_PH; ++i) v[i] = sp[i][l];
#pragma unroll
    for (int w = TM_PH / 2; w > 0; w >>= 1)
#pragma unroll
      for (int i = 0; i < w; ++i) v[i] += v[i + w];
    mean_out[(long long)b * D + c] = v[0] / (float)T;
  }
}

// q[b,k,o] = Emb[idx[b,k]][o] (+ sum_c W_adj[o][c] cat[b,k][c]), cat = [mean_t h[b] ; Emb[idx[b,k]]]:
// one 64-lane wave per (o, b) (grid W x B): lanes stride c with coalesced loads of the W_adj
// row and the mean, all K outputs accumulated together, then a wave reduction.  (A thread
// per output walking its 650-long row issued one dependent L2 load per iteration: 26 us.)
__global__ __launch_bounds__(64) void query_fwd_kernel(const float* __restrict__ mean, int D,
                                                       const int* __restrict__ idx, const float* __restrict__ emb,
                                                       const float* __restrict__ wadj, int K, int W,
                                                       float* __restrict__ q) {
  constexpr int KMAX = 4;  // queries per wave; grid.z covers K in groups of 4
  const int o = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
  const int k0 = blockIdx.z * KMAX;
  idx += k0;
  q += (long long)k0 * W;
  const int Kg = min(KMAX, K - k0);
  int id[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) id[k] = k < Kg ? idx[b * K + k] : -1;
  float acc[KMAX] = {0.f, 0.f, 0.f, 0.f};
  if (wadj) {
    const float* wr = wadj + (long long)o * (D + W);
    const float* mb = mean + (long long)b * D;
#pragma unroll 4
    for (int c = lane; c < D; c += 64) {
      const float wv = wr[c] * mb[c];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) acc[k] += wv;  // the mean part is shared by every k
    }
    for (int c = lane; c < W; c += 64) {
      const float wv = wr[D + c];
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < Kg && id[k] >= 0) acc[k] = fmaf(wv, emb[(long long)id[k] * W + c], acc[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k >= Kg) break;
    const float r = wave_sum(acc[k]);
    if (lane == 0) q[((long long)b * K + k) * W + o] = (id[k] >= 0 ? emb[(long long)id[k] * W + o] : 0.0f) + r;
  }
}

// Backward of the queries (thread per output, every sum over <= 64 terms):
//   dh_bcast[b][c] = sum_o W[o][c] u[b][o] / T,   u[b][o] = sum_k dq[b,k,o]   (c < D)
//   dEmb[idx[b,k]][c] += dq[b,k,c] + sum_o W[o][D + c] dq[b,k,o]
//   dW_adj[o][c] += sum_b u[b][o] mean[b][c]  (c < D);  sum_{b,k} dq[b,k,o] Emb[idx[b,k]][c-D]
// Every element has one owner thread and a fixed summation order (no atomics).  Round 6: each role's
// loads of a QCH-term chunk are issued together from clamped addresses and folded by selects (no
// branches): the round-5 loops (five or eight loads at a time, predicated loads compiled to branches)
// left four to ten dependent load rounds per role on this ~14 us launch.
constexpr int QCH = 32;  // terms per load chunk (a multiple of 8: dW_adj's accumulator of term b is b & 7)
__device__ __forceinline__ void query_bwd_dh(int bx, int by, float* su, const float* __restrict__ dq,
                                             const float* __restrict__ wadj, int T, int D, int K, int W,
                                             float* __restrict__ dh_bcast) {
  const int b = by, c = bx * 64 + threadIdx.x;
  const float* dqb = dq + (long long)b * K * W;
  for (int o = threadIdx.x; o < W; o += 64) {  // u[b][o], k in order from zero
    float u = 0.f;
    for (int k = 0; k < K; ++k) u += dqb[k * W + o];
    su[o] = u;
  }
  __syncthreads();
  if (c >= D) return;
  float g0 = 0.f, g1 = 0.f;
  for (int o0 = 0; o0 < W; o0 += QCH) {
    float wv[QCH];
#pragma unroll
    for (int i = 0; i < QCH; ++i) wv[i] = wadj[(long long)min(o0 + i, W - 1) * (D + W) + c];
#pragma unroll
    for (int i = 0; i < QCH; ++i) {
      const int o = o0 + i;
      const float t = wv[i] * su[min(o, W - 1)];
      const bool in = o < W;
      g0 = (in && !(o & 1)) ? g0 + t : g0;
      g1 = (in && (o & 1)) ? g1 + t : g1;
    }
  }
  dh_bcast[(long long)b * D + c] = (g0 + g1) / (float)T;
}

// d_emb[id] += sum over the rows bk with idx[bk] == id, in bk order: the block of the first
// such row owns the label and sums every row of it (no atomics: a speaker drawn twice in a
// batch gets the same bits on every run).  sidx: the batch's speaker ids staged in LDS by the block
// (round 6: the ownership test and the row scan were serial scalar loads of idx); the matching rows
// come from one ballot per 64 ids, visited in order.
__device__ __forceinline__ void query_bwd_emb(int bk, const float* __restrict__ dq, const int* sidx, int BK,
                                              const float* __restrict__ wadj, int D, int W,
                                              float* __restrict__ demb, float beta) {
  const int id = sidx[bk];
  if (id < 0) return;
  for (int j0 = 0; j0 < bk; j0 += 64) {  // an earlier row owns this label
    const int j = j0 + (int)threadIdx.x;
    if (__any(j < bk && sidx[j] == id)) return;
  }
  for (int c0 = 0; c0 < W; c0 += 64) {  // every lane of the wave in each pass (the ballots are wave-wide)
    const int c = c0 + (int)threadIdx.x, cc = min(c, W - 1);
    float acc = 0.f;
    for (int r0 = bk; r0 < BK; r0 += 64) {
      const int rr = r0 + (int)threadIdx.x;
      unsigned long long m = __ballot(rr < BK && sidx[rr] == id);
      while (m) {  // wave-uniform: the rows of this label in order
        const int r = r0 + __builtin_ctzll(m);
        m &= m - 1;
        const float* dqr = dq + (long long)r * W;
        float g = dqr[cc];
        if (wadj) {
          float g1 = 0.f;
          for (int o0 = 0; o0 < W; o0 += QCH) {
            float wv[QCH], dv[QCH];
#pragma unroll
            for (int i = 0; i < QCH; ++i) {
              const int o = min(o0 + i, W - 1);
              wv[i] = wadj[(long long)o * (D + W) + D + cc];
              dv[i] = dqr[o];
            }
#pragma unroll
            for (int i = 0; i < QCH; ++i) g1 = o0 + i < W ? fmaf(wv[i], dv[i], g1) : g1;
          }
          g += g1;
        }
        acc += g;
      }
    }
    if (c < W) {
      float* o = demb + (long long)id * W + c;
      *o = beta != 0.f ? acc + beta * *o : acc;  // beta 0: the row is written without being read
    }
  }
}

__device__ __forceinline__ void query_bwd_w(int bx, int by, float* sm, const float* __restrict__ dq,
                                            const int* __restrict__ idx, const float* __restrict__ emb,
                                            const float* __restrict__ mean, int B, int D, int K, int W,
                                            float* __restrict__ dwadj, float beta) {
  // block (column chunk, o): the o-th dq column (and its per-utterance sums u) and the
  // speaker ids staged in LDS, then QCH loads in flight per thread
  float* sdq = sm;            // [B*K]  dq[bk][o]
  float* su = sdq + B * K;    // [B]    u[b][o]
  int* sid = reinterpret_cast<int*>(su + B);  // [B*K]
  const int o = by, c = bx * 64 + threadIdx.x;
  for (int i = threadIdx.x; i < B * K; i += 64) {
    sdq[i] = dq[(long long)i * W + o];
    sid[i] = idx[i];
  }
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += 64) {
    float u = 0.f;
    for (int k = 0; k < K; ++k) u += sdq[b * K + k];
    su[b] = u;
  }
  __syncthreads();
  if (c >= D + W) return;
  // the sums over b (or b k) in eight interleaved accumulators, acc[j & 7] += term j in order
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    for (int b0 = 0; b0 < B; b0 += QCH) {
      float m[QCH];
#pragma unroll
      for (int j = 0; j < QCH; ++j) m[j] = mean[(long long)min(b0 + j, B - 1) * D + c];
#pragma unroll
      for (int j = 0; j < QCH; ++j)
        acc[j & 7] = b0 + j < B ? fmaf(su[min(b0 + j, B - 1)], m[j], acc[j & 7]) : acc[j & 7];
    }
  } else {
    const int ce = c - D;
    for (int b0 = 0; b0 < B * K; b0 += QCH) {
      float e[QCH];
#pragma unroll
      for (int j = 0; j < QCH; ++j) e[j] = emb[(long long)max(sid[min(b0 + j, B * K - 1)], 0) * W + ce];
#pragma unroll
      for (int j = 0; j < QCH; ++j) {
        const int jj = min(b0 + j, B * K - 1);
        const float ev = sid[jj] >= 0 ? e[j] : 0.f;
        acc[j & 7] = b0 + j < B * K ? fmaf(sdq[jj], ev, acc[j & 7]) : acc[j & 7];
      }
    }
  }
  const float sum = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  float* od = dwadj + (long long)o * (D + W) + c;
  *od = beta != 0.f ? sum + beta * *od : sum;
}

// The three query backward parts as ONE launch (64-thread blocks, role by block range: the
// embedding rows, dh_bcast, dW_adj): one after another they were three ~10-13 us latency-bound
// launches in the step; side by side they overlap.  Each part's arithmetic is unchanged.
struct QbArgs {
  const float* dq;
  const int* idx;
  const float* emb;
  const float* wadj;
  const float* mean;
  int B, T, D, K, W;
  float* demb;
  float* dwadj;
  float* dh;
  int n_emb, n_dh_x, n_dh, n_w_x;
  float beta;       // d_emb / d_wadj = beta (old) + this step's (beta 0: written, not read)
  int n_zero;       // beta 0: embedding rows 0 .. n_zero-1 that no speaker of the batch owns are zeroed
};
__global__ __launch_bounds__(64) void query_bwd_kernel(QbArgs a) {
  extern __shared__ float sm[];
  int blk = blockIdx.x;
  const int BK = a.B * a.K;
  if (blk < a.n_emb + a.n_zero) {  // the embedding roles: the batch's speaker ids in LDS first
    int* sidx = reinterpret_cast<int*>(sm);
    for (int i = threadIdx.x; i < BK; i += 64) sidx[i] = a.idx[i];
    __syncthreads();
    if (blk < a.n_emb) {
      query_bwd_emb(blk, a.dq, sidx, BK, a.wadj, a.D, a.W, a.demb, a.beta);
      return;
    }
    blk -= a.n_emb;  // (beta 0) embedding row blk: zero unless a speaker of the batch owns it
    for (int j0 = 0; j0 < BK; j0 += 64) {
      const int j = j0 + (int)threadIdx.x;
      if (__any(j < BK && sidx[j] == blk)) return;
    }
    for (int c = threadIdx.x; c < a.W; c += 64) a.demb[(long long)blk * a.W + c] = 0.f;
    return;
  }
  blk -= a.n_emb + a.n_zero;
  if (blk < a.n_dh) {
    query_bwd_dh(blk % a.n_dh_x, blk / a.n_dh_x, sm, a.dq, a.wadj, a.T, a.D, a.K, a.W, a.dh);
    return;
  }
  blk -= a.n_dh;
  query_bwd_w(blk % a.n_w_x, blk / a.n_w_x, sm, a.dq, a.idx, a.emb, a.mean, a.B, a.D, a.K, a.W, a.dwadj, a.beta);
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

// bf16 shadow copies written by the Adam update (the bf16 step's GEMM / recurrence operands): segment s
// maps the flat range [off, off + rows*cols) row-major onto y[r * ldy + c] (columns >= cols untouched)
constexpr int SHADOW_MAX = 8;
struct ShadowSegs {
  long long off[SHADOW_MAX], len[SHADOW_MAX], ldy[SHADOW_MAX];
  int cols[SHADOW_MAX];
  unsigned short* y[SHADOW_MAX];
  int n;
};
__device__ __forceinline__ void shadow_store(const ShadowSegs& sh, long long i, float x) {
#pragma unroll
  for (int s = 0; s < SHADOW_MAX; ++s) {
    if (s >= sh.n) break;
    const long long j = i - sh.off[s];
    if (j >= 0 && j < sh.len[s]) {
      const unsigned r = (unsigned)j / (unsigned)sh.cols[s], c = (unsigned)j - r * (unsigned)sh.cols[s];
      sh.y[s][r * sh.ldy[s] + c] = (unsigned short)bf16_bits_rne(x);
      return;
    }
  }
}
// four consecutive flat elements i..i+3: one 8-B store when they sit in one row of one segment at
// an 8-B aligned destination (the 600-column weights: every quad), else element by element
__device__ __forceinline__ void shadow_store4(const ShadowSegs& sh, long long i, float4 x) {
#pragma unroll
  for (int s = 0; s < SHADOW_MAX; ++s) {
    if (s >= sh.n) break;
    const long long j = i - sh.off[s];
    if (j + 3 < 0 || j >= sh.len[s]) continue;
    if (j >= 0 && j + 3 < sh.len[s]) {
      const unsigned r = (unsigned)j / (unsigned)sh.cols[s], c = (unsigned)j - r * (unsigned)sh.cols[s];
      const long long o = r * sh.ldy[s] + c;
      if (c + 3 < (unsigned)sh.cols[s] && (o & 3) == 0) {
        const unsigned lo = bf16_bits_rne(x.x) | (bf16_bits_rne(x.y) << 16);
        const unsigned hi = bf16_bits_rne(x.z) | (bf16_bits_rne(x.w) << 16);
        *reinterpret_cast<uint2*>(sh.y[s] + o) = make_uint2(lo, hi);
        return;
      }
    }
    break;  // a quad across a row or segment boundary
  }
  shadow_store(sh, i, x.x); shadow_store(sh, i + 1, x.y); shadow_store(sh, i + 2, x.z); shadow_store(sh, i + 3, x.w);
}

// torch.optim.Adam (weight_decay 0, amsgrad off; m via lerp as torch) on flat fp32 buffers
// (EvalVer.py:538-544,673-675: Adam(lr=2e-4), betas (0.9, 0.999), eps 1e-8).  SH: also the bf16
// shadow copies of the updated parameters (bitwise dl4ss_f32_to_bf16_2d_multi of the new values)
template <bool SH>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long long n,
                                                   float lr, float b1, float b2, float eps, float bc1, float bc2s,
                                                   const int* __restrict__ status, int* __restrict__ refused,
                                                   const float* __restrict__ dp_flag, float gscale,
                                                   float* __restrict__ loss, ShadowSegs sh) {
  // refuse the update when a recurrence hand-off of this step timed out on this rank
  // (status[0]) or on any data-parallel peer (dp_flag: the all-reduced status flag)
  if ((status && status[0]) || (dp_flag && dp_flag[0] != 0.f)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (loss) loss[0] = __builtin_nanf("");
      if (refused) refused[0] += 1;  // refused-update count: the host rolls its step count back by it
    }
    return;
  }
  const float step = lr / bc1;
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * blockDim.x * 4) {
    if (i + 3 < n) {
      float4 pp = *reinterpret_cast<float4*>(p + i);
      float4 gg = *reinterpret_cast<const float4*>(g + i);
      gg.x *= gscale; gg.y *= gscale; gg.z *= gscale; gg.w *= gscale;  // 1 / world (DP SUM); 1: exact
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
      if constexpr (SH) {
        shadow_store4(sh, i, pp);
      }
    } else {
      for (long long j = i; j < n; ++j) {
        const float gj = g[j] * gscale;
        m[j] = m[j] + (1.f - b1) * (gj - m[j]);
        v[j] = b2 * v[j] + (1.f - b2) * gj * gj;
        p[j] -= step * (m[j] / (sqrtf(v[j]) / bc2s + eps));
        if constexpr (SH) shadow_store(sh, j, p[j]);
      }
    }
  }
}

}  // namespace

DL4SS_API int dl4ss_query_fwd(const float* h, int B, int T, int D, const int* idx, const float* emb,
                              const float* w_adj, int K, int W, float* q, float* mean_out, void* stream) {
  // h NULL: mean_out already holds the time mean (the recurrence formed it, dl4ss_birnn_fwd_xw_ex)
  DL4SS_REQUIRE((h || mean_out) && idx && emb && q && B > 0 && T > 0 && D > 0 && K > 0 && W > 0);
  DL4SS_REQUIRE(!w_adj || mean_out);  // ADJUST needs the time mean (also saved for the backward)
  hipStream_t st = as_stream(stream);
  if (mean_out && h) {
    hipLaunchKernelGGL(time_mean_kernel, dim3(B, cdiv(D, 64)), dim3(64 * TM_PH), 0, st, h, T, D, mean_out);
    DL4SS_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(query_fwd_kernel, dim3(W, B, cdiv(K, 4)), dim3(64), 0, st, mean_out, D, idx, emb, w_adj, K, W,
                     q);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_time_mean(const float* h, int B, int T, int D, float* mean_out, void* stream) {
  DL4SS_REQUIRE(h && mean_out && B >= 0 && T > 0 && D > 0);
  if (B == 0) return 0;
  hipLaunchKernelGGL(time_mean_kernel, dim3(B, cdiv(D, 64)), dim3(64 * TM_PH), 0, as_stream(stream), h, T, D, mean_out);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_query_bwd_ex(const float* dq, int B, int T, int D, const int* idx, const float* emb,
                                 const float* w_adj, const float* mean, int K, int W, float* d_emb, float* d_wadj,
                                 float* dh_bcast, int n_labels, float beta, void* stream) {
  DL4SS_REQUIRE(dq && idx && B > 0 && K > 0 && W > 0 && (beta != 0.f || !d_emb || n_labels > 0));
  hipStream_t st = as_stream(stream);
  QbArgs a{dq, idx, emb, w_adj, mean, B, T, D, K, W, d_emb, d_wadj, dh_bcast, 0, 0, 0, 0, beta, 0};
  a.n_emb = d_emb ? B * K : 0;
  a.n_zero = (d_emb && beta == 0.f) ? n_labels : 0;
  a.n_dh_x = (int)cdiv(D, 64);
  a.n_dh = (w_adj && dh_bcast) ? a.n_dh_x * B : 0;
  a.n_w_x = (int)cdiv(D + W, 64);
  int n_w = 0;
  size_t smem = a.n_emb + a.n_zero > 0 ? sizeof(int) * (size_t)B * K : 0;  // the embedding roles' staged ids
  if (a.n_dh > 0 && sizeof(float) * (size_t)W > smem) smem = sizeof(float) * (size_t)W;  // dh: u[b][o]
  if (w_adj && d_wadj) {
    DL4SS_REQUIRE(mean && emb);
    n_w = a.n_w_x * W;
    const size_t sw = sizeof(float) * (2 * (size_t)B * K + B);
    smem = sw > smem ? sw : smem;
  }
  const int nblk = a.n_emb + a.n_zero + a.n_dh + n_w;
  if (nblk == 0) return 0;
  hipLaunchKernelGGL(query_bwd_kernel, dim3(nblk), dim3(64), smem, st, a);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_query_bwd(const float* dq, int B, int T, int D, const int* idx, const float* emb,
                              const float* w_adj, const float* mean, int K, int W, float* d_emb, float* d_wadj,
                              float* dh_bcast, void* stream) {
  return dl4ss_query_bwd_ex(dq, B, T, D, idx, emb, w_adj, mean, K, W, d_emb, d_wadj, dh_bcast, 0, 1.f, stream);
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

namespace {
int adam_launch(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                float eps, int step, const int* status, int* refused, const float* dp_flag, float gscale,
                float* loss, void* stream, const ShadowSegs* sh = nullptr) {
  DL4SS_REQUIRE(p && g && m && v && n >= 0 && step >= 1);
  if (n == 0) return 0;
  // bias corrections in double on the host, as torch computes them in Python floats
  const float bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, (double)step));
  const unsigned grid = (unsigned)min(8192LL, (n / 4 + 255) / 256 + 1);
  if (sh && sh->n > 0)
    hipLaunchKernelGGL(adam_kernel<true>, dim3(grid), dim3(256), 0, as_stream(stream), p, g, m, v, n, lr, beta1, beta2,
                       eps, bc1, bc2s, status, refused, dp_flag, gscale, loss, *sh);
  else
    hipLaunchKernelGGL(adam_kernel<false>, dim3(grid), dim3(256), 0, as_stream(stream), p, g, m, v, n, lr, beta1,
                       beta2, eps, bc1, bc2s, status, refused, dp_flag, gscale, loss, ShadowSegs{});
  DL4SS_CHECK_LAUNCH();
  return 0;
}
}  // namespace

DL4SS_API int dl4ss_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                         float beta2, float eps, int step, void* stream) {
  return adam_launch(p, g, m, v, n, lr, beta1, beta2, eps, step, nullptr, nullptr, nullptr, 1.0f, nullptr, stream);
}

// status: ONE int (the hand-off word), read only; a refusal shows as loss[0] = NaN
DL4SS_API int dl4ss_adam_guarded(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                                 float beta2, float eps, int step, int* status, float* loss, void* stream) {
  return adam_launch(p, g, m, v, n, lr, beta1, beta2, eps, step, status, nullptr, nullptr, 1.0f, loss, stream);
}

// status: 2 ints {hand-off word, refused-update count}; the count is incremented per refusal
DL4SS_API int dl4ss_adam_guarded_dp(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                                    float beta2, float eps, int step, int* status, const float* dp_flag, float* loss,
                                    void* stream) {
  return adam_launch(p, g, m, v, n, lr, beta1, beta2, eps, step, status, status ? status + 1 : nullptr, dp_flag, 1.0f,
                     loss, stream);
}

// the DP form on the SUM-reduced gradient: g * gscale (gscale = 1 / world) inside the update
DL4SS_API int dl4ss_adam_guarded_dp_scaled(float* p, const float* g, float* m, float* v, long long n, float lr,
                                           float beta1, float beta2, float eps, int step, int* status,
                                           const float* dp_flag, float gscale, float* loss, void* stream) {
  return adam_launch(p, g, m, v, n, lr, beta1, beta2, eps, step, status, status ? status + 1 : nullptr, dp_flag, gscale,
                     loss, stream);
}

__global__ void status_flag_kernel(const int* __restrict__ status, float* __restrict__ flag) {
  if (threadIdx.x == 0) flag[0] = status[0] ? 1.f : 0.f;
}

DL4SS_API int dl4ss_status_flag(const int* status, float* flag, void* stream) {
  DL4SS_REQUIRE(status && flag);
  hipLaunchKernelGGL(status_flag_kernel, dim3(1), dim3(64), 0, as_stream(stream), status, flag);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

// dl4ss_adam_guarded_dp_scaled that also writes bf16 shadow copies of the updated parameters: segment
// s (s < nseg <= 8) maps the flat range [seg_off, seg_off + rows*cols) row-major onto seg_y (row stride
// seg_ldy >= cols bf16; columns >= cols are not written).  The step's bf16 weight operands then need
// no conversion pass before the next forward (bitwise dl4ss_f32_to_bf16_2d_multi of the new values;
// a refused update leaves parameters and shadows untouched).
DL4SS_API int dl4ss_adam_guarded_dp_scaled_bf16(float* p, const float* g, float* m, float* v, long long n, float lr,
                                                float beta1, float beta2, float eps, int step, int* status,
                                                const float* dp_flag, float gscale, float* loss, int nseg,
                                                const long long* seg_off, const int* seg_rows, const int* seg_cols,
                                                void* const* seg_y, const long long* seg_ldy, void* stream) {
  DL4SS_REQUIRE(nseg >= 0 && nseg <= SHADOW_MAX && (nseg == 0 || (seg_off && seg_rows && seg_cols && seg_y && seg_ldy)));
  ShadowSegs sh{};
  sh.n = nseg;
  for (int i = 0; i < nseg; ++i) {
    DL4SS_REQUIRE(seg_y[i] && seg_rows[i] >= 0 && seg_cols[i] > 0 && seg_ldy[i] >= seg_cols[i] && seg_off[i] >= 0 &&
                  seg_off[i] + (long long)seg_rows[i] * seg_cols[i] <= n && (long long)seg_rows[i] * seg_cols[i] < (1LL << 31));
    DL4SS_REQUIRE(((uintptr_t)seg_y[i] & 7) == 0);  // the 8-B quad stores
    sh.off[i] = seg_off[i];
    sh.len[i] = (long long)seg_rows[i] * seg_cols[i];
    sh.cols[i] = seg_cols[i];
    sh.ldy[i] = seg_ldy[i];
    sh.y[i] = reinterpret_cast<unsigned short*>(seg_y[i]);
  }
  return adam_launch(p, g, m, v, n, lr, beta1, beta2, eps, step, status, status ? status + 1 : nullptr, dp_flag, gscale,
                     loss, stream, &sh);
}
