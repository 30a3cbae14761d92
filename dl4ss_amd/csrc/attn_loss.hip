// Fused speaker-query mask attention + separation loss + its backward.
//
// Replaces, for the magnitude path (TDAA_beta/main_run_sstune_EvalVer.py:615-666,
// Torch_multi/main_run.py:478-506):
//     V.expand(B,K,...).contiguous()          (414 MB copy at B=32)
//     baddbmm(V, q) -> sigmoid                 mask (B,K,T,F)
//     predict = mask * |X| ; MSE(predict, Y) + 0.5 * MSE(sum_k mask, 1)
// and for the cRM path (main_run_sstune_cRM_EvalVer.py:259-271, 688, 720-743):
//     Mc = 10 tanh(V.q_{re,im}); M = -1/0.1 log((10 - Mc)/(10 + Mc));
//     P = M (x) X (complex product); MSE(P_re, Y_re) + MSE(P_im, Y_im)
// together with the whole backward down to dPre = dL/d(h W^T + b) of the
// Linear+tanh that produced V, and dq = dL/dq.
//
// One pass reads each V row (E floats) exactly once: a workgroup stages a 256-row
// tile of V with coalesced 16-B loads into LDS, each lane owns one (b,t,f) row
// (8-B LDS reads: conflict-free for E = 50), computes the K logits / masks /
// costs, and in the GRAD pass writes the dPre row back into the same LDS tile
// for a coalesced store.  Loss terms and dq are reduced per workgroup (wave
// shuffles + LDS) into per-block partials that a finalize kernel sums in fixed
// order (bitwise deterministic).  PIT: the COST pass produces the K x K pairwise
// cost matrix per utterance, `pit_select` picks the lowest-index minimising
// permutation, the GRAD pass uses it; label order (the reference) = identity.
#include <cstdlib>
#include "common.h"
#include <hip/hip_bf16.h>

namespace {

constexpr int NT = 256;
constexpr int TILE = 256;  // rows per tile

template <int K>
struct Perms;
template <>
struct Perms<1> { static constexpr int N = 1; static constexpr int P[1][1] = {{0}}; };
template <>
struct Perms<2> { static constexpr int N = 2; static constexpr int P[2][2] = {{0, 1}, {1, 0}}; };
template <>
struct Perms<3> {
  static constexpr int N = 6;
  static constexpr int P[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
};

struct AttnArgs {
  int B, T, F, rows_per_b, nblk;  // rows_per_b = T*F ; nblk = blocks per utterance
  const float* V;                 // (B, T*F, E)
  const unsigned short* Vb;       // the same as bf16 (the fast path's Linear writes V in bf16); V unused then
  const float* q;                 // (B, K, QW)
  const float* X;                 // mag: (b*xs + row) ; cRM: (b*xs + row)*2
  long long xs;
  const float* Y;                 // target k of b: Y + b*ys + k*yks (+row, cRM *2)
  long long ys, yks;
  const int* perm;                // (B, K) target index per channel, null = identity
  float s1, s2;                   // loss scales: MSE term, sum-to-one term
  float* dPre;                    // (B, T*F, E) GRAD pass output (fp32; null when dPreB is given)
  unsigned* dPreB;                // GRAD pass bf16 output: row (b*T + t) of F*E values at stride ldpb (bf16)
  long long ldpb;
  float* part_loss;               // (B, nblk, K*K + 1)
  float* part_dq;                 // (B, nblk, K, QW)
  float* mask_out;                // optional (B, K, T*F) [cRM: x2]
  float* pred_out;                // optional (B, K, T*F) [cRM: x2]
};

template <int E, int K, bool CRM, bool GRAD, bool VB>
__global__ __launch_bounds__(NT) void attn_kernel(AttnArgs a) {
  constexpr int QW = CRM ? 2 * E : E;
  constexpr int NC = CRM ? 2 : 1;  // components per bin
  __shared__ __attribute__((aligned(16))) float sv[TILE * E];
  __shared__ float sq[K * QW];
  __shared__ float sred[NT / 64][K * K + 1];

  const int b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < K * QW; i += NT) sq[i] = a.q[(long long)b * K * QW + i];

  // this block's row range
  const int per = (a.rows_per_b + a.nblk - 1) / a.nblk;
  const int rbeg = blockIdx.x * per;
  const int rend = min(a.rows_per_b, rbeg + per);

  int pm[K];
#pragma unroll
  for (int k = 0; k < K; ++k) pm[k] = a.perm ? a.perm[b * K + k] : k;

  float cost[K * K + 1];
#pragma unroll
  for (int i = 0; i < K * K + 1; ++i) cost[i] = 0.f;
  __shared__ float sdl[GRAD ? TILE * K * NC : 1];  // dL/dlogit per tile row
  float dqa[2] = {0.f, 0.f};  // dq[j] for j = tid, tid + 256 (j < K*QW)
  const float* Vb = a.V + (long long)b * a.rows_per_b * E;
  float* Db = (GRAD && a.dPre) ? a.dPre + (long long)b * a.rows_per_b * E : nullptr;

  for (int r0 = rbeg; r0 < rend; r0 += TILE) {
    const int nr = min(TILE, rend - r0);
    __syncthreads();  // previous tile fully consumed (and sq visible on first pass)
    // coalesced stage of nr rows (nr*E floats, 16-B aligned when r0*E*4 % 16 == 0); bf16 V:
    // 4-B pairs (E even), widened to fp32 in LDS
    if constexpr (VB) {
      const unsigned* src = reinterpret_cast<const unsigned*>(a.Vb + ((long long)b * a.rows_per_b + r0) * E);
      const int n2 = nr * E / 2;
      // every load of the tile issued before the first LDS store (a load -> store loop
      // kept one 4-B load per thread in flight)
      constexpr int NW = (TILE * E / 2 + NT - 1) / NT;
      unsigned w[NW];
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int i = tid + q * NT;
        w[q] = i < n2 ? src[i] : 0u;
      }
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int i = tid + q * NT;
        if (i < n2)
          reinterpret_cast<float2*>(sv)[i] = make_float2(__uint_as_float(w[q] << 16), __uint_as_float(w[q] & 0xFFFF0000u));
      }
    } else {
      const float* src = Vb + (long long)r0 * E;
      const int n = nr * E;
      if ((((long long)r0 * E) & 3) == 0) {
        const int n4 = n >> 2;
        for (int i = tid; i < n4; i += NT) reinterpret_cast<float4*>(sv)[i] = reinterpret_cast<const float4*>(src)[i];
        for (int i = (n4 << 2) + tid; i < n; i += NT) sv[i] = src[i];
      } else {
        for (int i = tid; i < n; i += NT) sv[i] = src[i];
      }
    }
    __syncthreads();
    const int r = tid;
    if (r < nr) {
      const int row = r0 + r;
      const float* v = sv + r * E;
      float lg[K * NC];
#pragma unroll
      for (int i = 0; i < K * NC; ++i) lg[i] = 0.f;
#pragma unroll
      for (int e = 0; e < E; e += 2) {
        const float2 vv = *reinterpret_cast<const float2*>(v + e);
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            lg[k * NC + c] = fmaf(vv.x, sq[k * QW + c * E + e], lg[k * NC + c]);
            lg[k * NC + c] = fmaf(vv.y, sq[k * QW + c * E + e + 1], lg[k * NC + c]);
          }
      }
      float dl[K * NC];  // dL/dlogit
      if constexpr (!CRM) {
        const float x = a.X[(long long)b * a.xs + row];
        float m[K], y[K], msum = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          m[k] = sigmoidf_(lg[k]);
          msum += m[k];
          y[k] = a.Y[(long long)b * a.ys + (long long)k * a.yks + row];
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const float dd = m[k] * x - y[j];
            cost[k * K + j] = fmaf(dd, dd, cost[k * K + j]);
          }
        const float ds = msum - 1.0f;
        cost[K * K] = fmaf(ds, ds, cost[K * K]);
        if (a.mask_out || a.pred_out) {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const long long o = ((long long)b * K + k) * a.rows_per_b + row;
            if (a.mask_out) a.mask_out[o] = m[k];
            if (a.pred_out) a.pred_out[o] = m[k] * x;
          }
        }
        if constexpr (GRAD) {
          float yp[K];
#pragma unroll
          for (int k = 0; k < K; ++k) {
            yp[k] = y[0];
#pragma unroll
            for (int j = 1; j < K; ++j) yp[k] = pm[k] == j ? y[j] : yp[k];
          }
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const float dm = 2.f * a.s1 * (m[k] * x - yp[k]) * x + 2.f * a.s2 * ds;
            dl[k] = dm * m[k] * (1.f - m[k]);
          }
        }
      } else {
        const float2 x = *reinterpret_cast<const float2*>(a.X + 2 * ((long long)b * a.xs + row));
        float2 p[K], y[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          // cRM_EvalVer.py:269 (10 tanh) and :688 (inverse compression), fp32 as the reference
          const float mcr = 10.f * tanhf(lg[k * 2]);
          const float mci = 10.f * tanhf(lg[k * 2 + 1]);
          const float mr = -10.f * logf((10.f - mcr) / (10.f + mcr));
          const float mi = -10.f * logf((10.f - mci) / (10.f + mci));
          p[k] = make_float2(mr * x.x - mi * x.y, mr * x.y + mi * x.x);
          y[k] = *reinterpret_cast<const float2*>(a.Y + 2 * ((long long)b * a.ys + (long long)k * a.yks + row));
          if (a.mask_out) {
            const long long o = 2 * (((long long)b * K + k) * a.rows_per_b + row);
            a.mask_out[o] = mr;
            a.mask_out[o + 1] = mi;
          }
          if (a.pred_out) {
            const long long o = 2 * (((long long)b * K + k) * a.rows_per_b + row);
            a.pred_out[o] = p[k].x;
            a.pred_out[o + 1] = p[k].y;
          }
          if constexpr (GRAD) {
            // d(M)/d(logit) through the same fp32 chain: dM/dMc * dMc/dl
            const float dmc_r = 10.f * (1.f / (10.f - mcr) + 1.f / (10.f + mcr));
            const float dmc_i = 10.f * (1.f / (10.f - mci) + 1.f / (10.f + mci));
            dl[k * 2] = dmc_r * (10.f * (1.f - (mcr * 0.1f) * (mcr * 0.1f)));
            dl[k * 2 + 1] = dmc_i * (10.f * (1.f - (mci * 0.1f) * (mci * 0.1f)));
          }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const float dr = p[k].x - y[j].x, di = p[k].y - y[j].y;
            cost[k * K + j] = fmaf(dr, dr, fmaf(di, di, cost[k * K + j]));
          }
        if constexpr (GRAD) {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            float2 yp = y[0];
#pragma unroll
            for (int j = 1; j < K; ++j) yp = pm[k] == j ? y[j] : yp;
            const float gr = 2.f * a.s1 * (p[k].x - yp.x), gi = 2.f * a.s1 * (p[k].y - yp.y);
            // P = M (x) X: dMr = gr xr + gi xi ; dMi = -gr xi + gi xr
            const float dmr = gr * x.x + gi * x.y;
            const float dmi = -gr * x.y + gi * x.x;
            dl[k * 2] *= dmr;
            dl[k * 2 + 1] *= dmi;
          }
        }
      }
      if constexpr (GRAD) {
#pragma unroll
        for (int i = 0; i < K * NC; ++i) sdl[r * K * NC + i] = dl[i];
      }
    } else if (GRAD) {
#pragma unroll
      for (int i = 0; i < K * NC; ++i) sdl[r * K * NC + i] = 0.f;
    }
    if constexpr (GRAD) {
      __syncthreads();
      // dq[k][c*E+e] += sum_r dl[r][k*NC+c] V[r][e]   (lanes along e: conflict-free)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = tid + NT * h;
        if (j < K * QW) {
          const int k = j / QW, ce = j % QW, c = ce / E, e = ce % E;
          float acc = 0.f;
          for (int rr = 0; rr < nr; ++rr) acc = fmaf(sdl[rr * K * NC + k * NC + c], sv[rr * E + e], acc);
          dqa[h] += acc;
        }
      }
      __syncthreads();
      // dV[e] = sum_k dl_k q_k[e] ; dPre = dV (1 - V^2), written in place over the own row
      if (r < nr) {
        float* v = sv + r * E;
        float dl[K * NC];
#pragma unroll
        for (int i = 0; i < K * NC; ++i) dl[i] = sdl[r * K * NC + i];
#pragma unroll
        for (int e = 0; e < E; e += 2) {
          const float2 vv = *reinterpret_cast<const float2*>(v + e);
          float g0 = 0.f, g1 = 0.f;
#pragma unroll
          for (int k = 0; k < K; ++k)
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              const float d = dl[k * NC + c];
              g0 = fmaf(d, sq[k * QW + c * E + e], g0);
              g1 = fmaf(d, sq[k * QW + c * E + e + 1], g1);
            }
          *reinterpret_cast<float2*>(v + e) = make_float2(g0 * (1.f - vv.x * vv.x), g1 * (1.f - vv.y * vv.y));
        }
      }
    }
    if (GRAD && a.dPreB) {
      // bf16 dPre for the Linear's backward GEMMs: pairs (e, e+1) as one 4-B store into
      // row (b*T + t) of the padded bf16 matrix (E, F*E offsets and ldpb are even)
      __syncthreads();
      for (int i = tid; i < nr * E / 2; i += NT) {
        const int rl = (2 * i) / E, e = (2 * i) % E;
        const int row = r0 + rl;
        const int t = row / a.F, f = row - t * a.F;
        __hip_bfloat162 v2 = __float22bfloat162_rn(make_float2(sv[2 * i], sv[2 * i + 1]));
        a.dPreB[(((long long)b * a.T + t) * a.ldpb + (long long)f * E + e) >> 1] = *reinterpret_cast<unsigned*>(&v2);
      }
    } else if constexpr (GRAD) {
      __syncthreads();
      float* dst = Db + (long long)r0 * E;
      const int n = nr * E;
      if ((((long long)r0 * E) & 3) == 0) {
        const int n4 = n >> 2;
        for (int i = tid; i < n4; i += NT) reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(sv)[i];
        for (int i = (n4 << 2) + tid; i < n; i += NT) dst[i] = sv[i];
      } else {
        for (int i = tid; i < n; i += NT) dst[i] = sv[i];
      }
    }
  }

  // ---- block reductions (fixed order: wave shuffle, then waves 0..3)
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K * K + 1; ++i) {
    const float s = wave_sum(cost[i]);
    if (lane == 0) sred[wave][i] = s;
  }
  __syncthreads();
  float* pl = a.part_loss + ((long long)b * a.nblk + blockIdx.x) * (K * K + 1);
  if (tid < K * K + 1) pl[tid] = sred[0][tid] + sred[1][tid] + sred[2][tid] + sred[3][tid];
  if constexpr (GRAD) {
    float* pd = a.part_dq + ((long long)b * a.nblk + blockIdx.x) * K * QW;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (tid + NT * h < K * QW) pd[tid + NT * h] = dqa[h];
  }
}

// The bf16-V magnitude path (the throughput step), one QUAD of lanes per (b,t,f) row.
// attn_kernel gives each lane a whole row (E = 50 values: 100 logit FMAs, 100 dPre FMAs and a
// 256-long serial dq chain per tile on 100 lanes: latency-bound at ~2.5 TB/s); a lane holding
// all K*E dq sums in registers (221 VGPRs, 2 waves per SIMD) was slower still.  Here lane j of a
// quad owns the row's bf16 pairs w = j, j+4, j+8, ... (7 of the 25 at E = 50), so a lane keeps
// only its 14 q values and 14 dq sums per query in registers (~4 waves per SIMD): partial logits
// over its pairs, the quad's sum by two DPP quad permutes (bitwise the same value in all four
// lanes), then dl, the lane's dPre pairs (written back as bf16 over its own V words) and its dq
// terms.  V reaches LDS by LDS-DMA (`global_load_lds_dwordx4`, no staging registers) from the 16-B
// aligned word below the tile (the tile's first word sits `off` words into the LDS image); dPre leaves by coalesced 4-B stores whose
// (t, f) destination changes only at frame boundaries, as 16-B stores from each frame segment's first
// 16-B aligned destination word.  Only the
// logits' summation order differs from attn_kernel (quad partials instead of one serial chain);
// dq is per-lane partials -> wave xor-shuffle tree -> waves 0..3 in order (deterministic).
__device__ __forceinline__ float quad_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
}
__device__ __forceinline__ float quad_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
}

typedef __attribute__((address_space(3))) void attn_lds_void;
__device__ __attribute__((aligned(16))) const unsigned g_attn_zero[4] = {0u, 0u, 0u, 0u};

// VF (round 5): fp32 V (the split-precision "bf16s" steps keep V = tanh(Linear) in fp32): the tile
// arrives as fp32 words (a pair = 8 B, read as one float2), the bf16 dPre pairs go to a separate LDS
// image (sdp) for the same copy-out; everything else -- the quad's arithmetic and summation order,
// the bf16 dPre, dq -- as in the bf16-V form.  The generic attn_kernel ran this step at ~2 TB/s
// (C4 bf16s: 156 us per step for its one GRAD launch).
template <int E, int K, bool GRAD, bool VF = false, bool CRM = false>
__global__ __launch_bounds__(NT, (K == 3 && GRAD) || VF || CRM ? 2 : 4) void attn_q4_kernel(AttnArgs a) {
  static_assert(E % 2 == 0, "bf16 pairs");
  // CRM (round 5): the complex-ratio-mask path (cRM_EvalVer.py:259-271, 688, 720-743) -- each row
  // has NC = 2 logits per query (the re / im halves of the 2E-wide query), the inverse-compressed mask
  // M, the complex prediction P = M (x) X and its squared error, as attn_kernel computes them (the same
  // fp32 tanhf / logf chain) -- on the quad layout; only the logits' summation order differs.
  constexpr int NC = CRM ? 2 : 1;        // logits per (row, query)
  constexpr int QW = NC * E;             // query width
  constexpr int EP = E / 2;              // bf16 pairs per row
  constexpr int NWL = (EP + 3) / 4;      // pairs per lane
  constexpr int NQ = NT / 4;             // quads per block
  constexpr int RPQ = TILE / NQ;         // rows per quad per tile
  constexpr int WPR = VF ? E : EP;       // 4-B words of V per row
  constexpr int NCH = (TILE * WPR + 3) / 4 + 1;  // 16-B chunks of a tile, misaligned start included
  constexpr int NCHP = (NCH + 63) / 64 * 64;     // whole 1-KB DMA instructions
  __shared__ __attribute__((aligned(16))) unsigned sv[NCHP * 4];
  __shared__ __attribute__((aligned(16))) unsigned sdp[VF && GRAD ? TILE * EP : 1];
  __shared__ float sred[NT / 64][K * K + 1];
  __shared__ float sdq[GRAD ? NT / 64 * K * QW : 1];

  const int b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = tid & 3, qd = tid >> 2;
  // this lane's q values (zero for the pair slots past EP)
  float qv[K][NC][NWL][2];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < NWL; ++i) {
        const int w = j + 4 * i;
        const float* qk = a.q + ((long long)b * K + k) * QW + c * E;
        qv[k][c][i][0] = w < EP ? qk[2 * w] : 0.f;
        qv[k][c][i][1] = w < EP ? qk[2 * w + 1] : 0.f;
      }
  const int per = (a.rows_per_b + a.nblk - 1) / a.nblk;
  const int rbeg = blockIdx.x * per;
  const int rend = min(a.rows_per_b, rbeg + per);
  int pm[K];
#pragma unroll
  for (int k = 0; k < K; ++k) pm[k] = a.perm ? a.perm[b * K + k] : k;
  float cost[K * K + 1];
#pragma unroll
  for (int i = 0; i < K * K + 1; ++i) cost[i] = 0.f;
  float dq[GRAD ? K : 1][GRAD ? NC : 1][GRAD ? NWL : 1][2];
  if constexpr (GRAD) {
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < NWL; ++i) dq[k][c][i][0] = dq[k][c][i][1] = 0.f;
  }
  const unsigned* Vw = VF ? reinterpret_cast<const unsigned*>(a.V) : reinterpret_cast<const unsigned*>(a.Vb);
  const long long totw = (long long)a.B * a.rows_per_b * WPR;

  for (int r0 = rbeg; r0 < rend; r0 += TILE) {
    const int nr = min(TILE, rend - r0);
    // issue this tile's loads: X and the targets of the quad's rows (cRM: [re, im]), then V by 16-B chunks
    float xr[RPQ][NC], yr[RPQ][K][NC];
#pragma unroll
    for (int s = 0; s < RPQ; ++s) {
      const int r = qd + NQ * s;
      const int row = r0 + (r < nr ? r : 0);
#pragma unroll
      for (int c = 0; c < NC; ++c) xr[s][c] = a.X[((long long)b * a.xs + row) * NC + c];
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int c = 0; c < NC; ++c) yr[s][k][c] = a.Y[((long long)b * a.ys + (long long)k * a.yks + row) * NC + c];
    }
    const long long w0 = ((long long)b * a.rows_per_b + r0) * WPR;
    const int off = (int)(w0 & 3);  // (VF: even -- E is -- so every pair is an aligned float2)
    const long long wa = w0 - off;
    const int nch = (off + nr * WPR + 3) >> 2;
    __syncthreads();  // the previous tile's rows and dPre copy-out are done with sv
    // V by LDS-DMA: wave instruction p moves chunks 64p .. 64p + 63 (1 KB) into sv + 256p words
    int tail = -1;
    for (int p = wave; p * 64 < nch; p += NT / 64) {
      const int c = p * 64 + lane;
      const long long gw = wa + 4LL * c;
      const bool whole = c < nch && gw + 4 <= totw;
      if (c < nch && !whole) tail = c;
      __builtin_amdgcn_global_load_lds(whole ? (const void*)(Vw + gw) : (const void*)g_attn_zero,
                                       (attn_lds_void*)(sv + 256 * p), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tail >= 0) {  // the buffer's last chunk, partly past its end: the valid words by plain loads
      const long long gw = wa + 4LL * tail;
      for (int q = 0; q < 4 && gw + q < totw; ++q) sv[4 * tail + q] = Vw[gw + q];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < RPQ; ++s) {
      const int r = qd + NQ * s;
      if (r < nr) {  // quad-uniform
        const int row = r0 + r;
        unsigned* v = VF ? sdp + r * EP + j : sv + off + r * EP + j;  // (VF: the dPre pairs' LDS words)
        float vxs[NWL], vys[NWL];
        if constexpr (VF) {
          const float2* vf = reinterpret_cast<const float2*>(sv + off + r * E) + j;
#pragma unroll
          for (int i = 0; i < NWL; ++i) {
            const float2 p = (j + 4 * i < EP) ? vf[4 * i] : make_float2(0.f, 0.f);
            vxs[i] = p.x;
            vys[i] = p.y;
          }
        } else {
#pragma unroll
          for (int i = 0; i < NWL; ++i) {
            const unsigned w = (j + 4 * i < EP) ? v[4 * i] : 0u;
            vxs[i] = __uint_as_float(w << 16);
            vys[i] = __uint_as_float(w & 0xFFFF0000u);
          }
        }
        float lg[K][NC];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
          for (int c = 0; c < NC; ++c) lg[k][c] = 0.f;
#pragma unroll
        for (int i = 0; i < NWL; ++i) {
          const float vx = vxs[i], vy = vys[i];
#pragma unroll
          for (int k = 0; k < K; ++k)
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              lg[k][c] = fmaf(vx, qv[k][c][i][0], lg[k][c]);
              lg[k][c] = fmaf(vy, qv[k][c][i][1], lg[k][c]);
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            lg[k][c] += quad_xor1(lg[k][c]);
            lg[k][c] += quad_xor2(lg[k][c]);
          }
        float dl[K][NC];  // dL/dlogit (GRAD)
        if constexpr (!CRM) {
          const float x = xr[s][0];
          float m[K], msum = 0.f;
#pragma unroll
          for (int k = 0; k < K; ++k) {
            m[k] = sigmoidf_(lg[k][0]);
            msum += m[k];
          }
#pragma unroll
          for (int k = 0; k < K; ++k)
#pragma unroll
            for (int jj = 0; jj < K; ++jj) {
              const float dd = m[k] * x - yr[s][jj][0];
              cost[k * K + jj] = fmaf(dd, dd, cost[k * K + jj]);
            }
          const float ds = msum - 1.0f;
          cost[K * K] = fmaf(ds, ds, cost[K * K]);
          if ((a.mask_out || a.pred_out) && j == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
              const long long o = ((long long)b * K + k) * a.rows_per_b + row;
              if (a.mask_out) a.mask_out[o] = m[k];
              if (a.pred_out) a.pred_out[o] = m[k] * x;
            }
          }
          if constexpr (GRAD) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
              float yp = yr[s][0][0];
#pragma unroll
              for (int jj = 1; jj < K; ++jj) yp = pm[k] == jj ? yr[s][jj][0] : yp;
              const float dm = 2.f * a.s1 * (m[k] * x - yp) * x + 2.f * a.s2 * ds;
              dl[k][0] = dm * m[k] * (1.f - m[k]);
            }
          }
        } else {
          const float2 x = make_float2(xr[s][0], xr[s][1]);
          float2 p[K];
#pragma unroll
          for (int k = 0; k < K; ++k) {
            // cRM_EvalVer.py:269 (10 tanh) and :688 (inverse compression), fp32 as the reference
            const float mcr = 10.f * tanhf(lg[k][0]);
            const float mci = 10.f * tanhf(lg[k][1]);
            const float mr = -10.f * logf((10.f - mcr) / (10.f + mcr));
            const float mi = -10.f * logf((10.f - mci) / (10.f + mci));
            p[k] = make_float2(mr * x.x - mi * x.y, mr * x.y + mi * x.x);
            if (j == 0) {
              const long long o = 2 * (((long long)b * K + k) * a.rows_per_b + row);
              if (a.mask_out) { a.mask_out[o] = mr; a.mask_out[o + 1] = mi; }
              if (a.pred_out) { a.pred_out[o] = p[k].x; a.pred_out[o + 1] = p[k].y; }
            }
            if constexpr (GRAD) {
              // d(M)/d(logit) through the same fp32 chain: dM/dMc * dMc/dl
              const float dmc_r = 10.f * (1.f / (10.f - mcr) + 1.f / (10.f + mcr));
              const float dmc_i = 10.f * (1.f / (10.f - mci) + 1.f / (10.f + mci));
              dl[k][0] = dmc_r * (10.f * (1.f - (mcr * 0.1f) * (mcr * 0.1f)));
              dl[k][1] = dmc_i * (10.f * (1.f - (mci * 0.1f) * (mci * 0.1f)));
            }
          }
#pragma unroll
          for (int k = 0; k < K; ++k)
#pragma unroll
            for (int jj = 0; jj < K; ++jj) {
              const float dr = p[k].x - yr[s][jj][0], di = p[k].y - yr[s][jj][1];
              cost[k * K + jj] = fmaf(dr, dr, fmaf(di, di, cost[k * K + jj]));
            }
          if constexpr (GRAD) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
              float2 yp = make_float2(yr[s][0][0], yr[s][0][1]);
#pragma unroll
              for (int jj = 1; jj < K; ++jj) yp = pm[k] == jj ? make_float2(yr[s][jj][0], yr[s][jj][1]) : yp;
              const float gr = 2.f * a.s1 * (p[k].x - yp.x), gi = 2.f * a.s1 * (p[k].y - yp.y);
              // P = M (x) X: dMr = gr xr + gi xi ; dMi = -gr xi + gi xr
              dl[k][0] *= gr * x.x + gi * x.y;
              dl[k][1] *= -gr * x.y + gi * x.x;
            }
          }
        }
        if constexpr (GRAD) {
          // dV[e] = sum_{k,c} dl_kc q_kc[e]; dPre = dV (1 - V^2) as bf16 over the lane's own words;
          // dq_kc[e] += dl_kc V[e]
#pragma unroll
          for (int i = 0; i < NWL; ++i) {
            const float vx = vxs[i], vy = vys[i];
            float g0 = 0.f, g1 = 0.f;
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
              for (int c = 0; c < NC; ++c) {
                g0 = fmaf(dl[k][c], qv[k][c][i][0], g0);
                g1 = fmaf(dl[k][c], qv[k][c][i][1], g1);
                dq[k][c][i][0] = fmaf(dl[k][c], vx, dq[k][c][i][0]);
                dq[k][c][i][1] = fmaf(dl[k][c], vy, dq[k][c][i][1]);
              }
            __hip_bfloat162 o2 = __float22bfloat162_rn(make_float2(g0 * (1.f - vx * vx), g1 * (1.f - vy * vy)));
            if (j + 4 * i < EP) v[4 * i] = *reinterpret_cast<unsigned*>(&o2);
          }
        }
      }
    }
    if constexpr (GRAD) {
      // bf16 dPre rows (b*T + t) of the padded matrix: the tile's words [s, e) of frame t go to
      // words (r0 - t F) EP + i of that row, one contiguous segment per frame (at most 3 here).
      // Rows start 16-B aligned (ldpb % 8 == 0), so each segment is written as 16-B stores from its
      // first 16-B aligned destination word on (four LDS words each: the source is only 4-B
      // aligned), with its <= 3 head and <= 3 tail words stored singly: a quarter of the store
      // instructions of a word-per-lane copy.
      __syncthreads();
      const int t0 = r0 / a.F;
      const long long rowb = (long long)b * a.T;
      const int ntot = nr * EP;
      for (int t = t0, sw = 0; sw < ntot; ++t) {
        const int ew = min(ntot, ((t + 1) * a.F - r0) * EP);  // end of frame t's words in the tile
        unsigned* dst = a.dPreB + ((rowb + t) * a.ldpb >> 1) + (long long)(r0 - t * a.F) * EP;  // + i
        const int lead = (int)((4 - (((uintptr_t)(dst + sw)) >> 2)) & 3);  // words before the first aligned one
        const int i0 = min(ew, sw + lead);
        const int nq = (ew - i0) >> 2;
        const unsigned* so = VF ? sdp : sv + off;  // the tile's dPre words
        for (int q = tid; q < nq; q += NT) {
          const int i = i0 + 4 * q;
          *reinterpret_cast<uint4*>(dst + i) = make_uint4(so[i], so[i + 1], so[i + 2], so[i + 3]);
        }
        const int te = i0 + 4 * nq;  // tail words [te, ew), head words [sw, i0)
        if (tid < i0 - sw) dst[sw + tid] = so[sw + tid];
        if (tid >= 4 && tid - 4 < ew - te) dst[te + tid - 4] = so[te + tid - 4];
        sw = ew;
      }
    }
  }

  // ---- block reductions (fixed order: lane trees, then waves 0..3); costs from lane 0 of each quad
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K * K + 1; ++i) {
    const float s = wave_sum(j == 0 ? cost[i] : 0.f);
    if (lane == 0) sred[wave][i] = s;
  }
  if constexpr (GRAD) {
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < NWL; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float s = dq[k][c][i][h];
#pragma unroll
            for (int o = 4; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
            const int w = lane + 4 * i;  // lanes 0..3 hold the wave's sums of pairs j + 4i
            if (lane < 4 && w < EP) sdq[(wave * K + k) * QW + c * E + 2 * w + h] = s;
          }
  }
  __syncthreads();
  float* pl = a.part_loss + ((long long)b * a.nblk + blockIdx.x) * (K * K + 1);
  if (tid < K * K + 1) pl[tid] = sred[0][tid] + sred[1][tid] + sred[2][tid] + sred[3][tid];
  if constexpr (GRAD) {
    float* pd = a.part_dq + ((long long)b * a.nblk + blockIdx.x) * K * QW;
    for (int i = tid; i < K * QW; i += NT)
      pd[i] = sdq[0 * K * QW + i] + sdq[1 * K * QW + i] + sdq[2 * K * QW + i] + sdq[3 * K * QW + i];
  }
}

// PIT selection: per utterance, lowest-index permutation minimising sum_k C[k][perm k].  One
// wave per utterance: lane l sums the block partials l, l + 64, ... in order, then a fixed
// butterfly tree over the lanes (deterministic; one thread walking all nblk partials serially
// took ~12 us at C2)
template <int K>
__global__ __launch_bounds__(64) void pit_select_kernel(const float* __restrict__ part, int B, int nblk,
                                                        int* __restrict__ perm) {
  const int b = blockIdx.x, lane = threadIdx.x;
  float C[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) C[i] = 0.f;
  for (int blk = lane; blk < nblk; blk += 64)
#pragma unroll
    for (int i = 0; i < K * K; ++i) C[i] += part[((long long)b * nblk + blk) * (K * K + 1) + i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int i = 0; i < K * K; ++i) C[i] += __shfl_xor(C[i], off);
  if (lane != 0) return;
  int best = 0;
  float bc = 0.f;
  for (int p = 0; p < Perms<K>::N; ++p) {
    float c = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) c += C[k * K + Perms<K>::P[p][k]];
    if (p == 0 || c < bc) { bc = c; best = p; }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) perm[b * K + k] = Perms<K>::P[best][k];
}

constexpr int FIN_CH = 8;      // finalize: loss items per thread loaded together
constexpr int FIN_PMAX = 1024;  // finalize: permutation entries staged in LDS (B K <= this; else direct loads)
// loss = s1 * sum_b sum_k C[b][k][perm k] + s2 * S ; also dq = sum_blk part_dq (fixed order)
template <int K>
__global__ __launch_bounds__(256) void finalize_kernel(const float* __restrict__ part, int B, int nblk,
                                                       const int* __restrict__ perm, float s1, float s2,
                                                       float* __restrict__ loss_out,
                                                       const float* __restrict__ part_dq, int qw,
                                                       float* __restrict__ dq) {
  // block 0: loss, 256 fixed-stride fp64 partial sums + fixed-order tree (deterministic)
  if (blockIdx.x == 0) {
    __shared__ double r1[256], r2[256];
    __shared__ int sperm[FIN_PMAX];
    double l1 = 0.0, l2 = 0.0;
    // the permutations staged in LDS first, then each thread's items loaded in chunks of FIN_CH
    // before they are summed in item order (round 6: a perm load then the cost loads per item was
    // two dependent rounds per item)
    const bool lp = perm && B * K <= FIN_PMAX;
    if (lp)
      for (int i = threadIdx.x; i < B * K; i += 256) sperm[i] = perm[i];
    __syncthreads();
    for (int i0 = threadIdx.x; i0 < B * nblk; i0 += 256 * FIN_CH) {
      float c[FIN_CH][K + 1];
#pragma unroll
      for (int u = 0; u < FIN_CH; ++u) {
        const int i = min(i0 + 256 * u, B * nblk - 1), b = i / nblk;
        const float* p = part + (long long)i * (K * K + 1);
#pragma unroll
        for (int k = 0; k < K; ++k)
          c[u][k] = p[k * K + (perm ? (lp ? sperm[b * K + k] : perm[b * K + k]) : k)];
        c[u][K] = p[K * K];
      }
#pragma unroll
      for (int u = 0; u < FIN_CH; ++u) {
        if (i0 + 256 * u < B * nblk) {
#pragma unroll
          for (int k = 0; k < K; ++k) l1 += c[u][k];
          l2 += c[u][K];
        }
      }
    }
    r1[threadIdx.x] = l1;
    r2[threadIdx.x] = l2;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) {
        r1[threadIdx.x] += r1[threadIdx.x + w];
        r2[threadIdx.x] += r2[threadIdx.x + w];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      loss_out[0] = (float)(s1 * r1[0] + s2 * r2[0]);
      loss_out[1] = (float)(s1 * r1[0]);
      loss_out[2] = (float)(s2 * r2[0]);
    }
    return;
  }
  // blocks 1..: dq = sum over the utterance's blocks, fixed order
  if (dq) {
    const int n = B * K * qw;
    for (int i = (blockIdx.x - 1) * blockDim.x + threadIdx.x; i < n; i += (gridDim.x - 1) * blockDim.x) {
      const int b = i / (K * qw), j = i % (K * qw);
      const float* pd = part_dq + (long long)b * nblk * K * qw + j;
      float a0 = 0.f, a1 = 0.f;
      // even blocks into a0, odd into a1, in block order; the loads of 32 blocks issued together
      for (int b0 = 0; b0 < nblk; b0 += 32) {
        float x[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) x[u] = pd[(long long)min(b0 + u, nblk - 1) * K * qw];
#pragma unroll
        for (int u = 0; u < 32; ++u) {
          const bool in = b0 + u < nblk;
          a0 = (in && !(u & 1)) ? a0 + x[u] : a0;
          a1 = (in && (u & 1)) ? a1 + x[u] : a1;
        }
      }
      dq[i] = a0 + a1;
    }
  }
}

template <int E, int K, bool CRM, bool VB>
int launch_attn(bool grad, const AttnArgs& a, hipStream_t st) {
  dim3 grid(a.nblk, a.B);
  if constexpr (!(CRM && K == 3)) {  // the throughput steps' path (16-B aligned V; bf16 dPre), magnitude and
                                     // cRM (K = 3 cRM: the quad kernel's 2 x 3 query halves spill; attn_kernel)
    // fp32 V or cRM: only for a bf16-dPre caller (which passes dPre_bf16 to its COST pass too, so both
    // passes of a PIT step sum the logits alike); the fp32 parity step keeps attn_kernel
    const bool q4 = (VB && !CRM) ? (a.dPreB || !grad) : a.dPreB != nullptr;
    if (q4 && ((uintptr_t)(VB ? (const void*)a.Vb : (const void*)a.V) & 15) == 0) {
      if (grad)
        hipLaunchKernelGGL((attn_q4_kernel<E, K, true, !VB, CRM>), grid, dim3(NT), 0, st, a);
      else
        hipLaunchKernelGGL((attn_q4_kernel<E, K, false, !VB, CRM>), grid, dim3(NT), 0, st, a);
      DL4SS_CHECK_LAUNCH();
      return 0;
    }
  }
  if (grad)
    hipLaunchKernelGGL((attn_kernel<E, K, CRM, true, VB>), grid, dim3(NT), 0, st, a);
  else
    hipLaunchKernelGGL((attn_kernel<E, K, CRM, false, VB>), grid, dim3(NT), 0, st, a);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

template <bool VB>
int dispatch_v(int E, int K, int crm, bool grad, const AttnArgs& a, hipStream_t st) {
  if (E != 50) return (int)hipErrorInvalidValue;
  if (!crm) {
    if (K == 1) return launch_attn<50, 1, false, VB>(grad, a, st);
    if (K == 2) return launch_attn<50, 2, false, VB>(grad, a, st);
    if (K == 3) return launch_attn<50, 3, false, VB>(grad, a, st);
  } else {
    if (K == 1) return launch_attn<50, 1, true, VB>(grad, a, st);
    if (K == 2) return launch_attn<50, 2, true, VB>(grad, a, st);
    if (K == 3) return launch_attn<50, 3, true, VB>(grad, a, st);
  }
  return (int)hipErrorInvalidValue;
}

int attn_common(int pass, int crm, int B, int K, int T, int F, int E, const float* V, const void* Vb, const float* q,
                const float* X, long long x_bstride, const float* Y, long long y_bstride, long long y_kstride,
                const int* perm, float s1, float s2, float* dPre, void* dPre_bf16, long long dpre_bf16_ld,
                float* part_loss, float* part_dq, float* mask_out, float* pred_out, void* stream);

}  // namespace

DL4SS_API int dl4ss_attn_nblk(int T, int F) {
  // DL4SS_ATTN_TILES tiles per block (default 4: with attn_q4_kernel at C2 -- 32 x 32 blocks, one
  // round at 4 resident per CU -- GRAD 65.8 / 66.7 / 71.1 us at 4 / 2 / 3 tiles, COST + PIT select
  // 25.2 / 25.8 / 27.1 us, profiles/r03_attn_q4.jsonl; round 2's attn_kernel preferred 3)
  static const int tpb = std::getenv("DL4SS_ATTN_TILES") ? std::atoi(std::getenv("DL4SS_ATTN_TILES")) : 4;
  const int rows = T * F;
  int nblk = (rows + tpb * TILE - 1) / (tpb * TILE);
  return nblk < 1 ? 1 : nblk;
}

// pass: 0 = COST (costs / masks only), 1 = GRAD (costs + dPre + dq partials)
DL4SS_API int dl4ss_mask_attn_loss_ex(int pass, int crm, int B, int K, int T, int F, int E, const float* V,
                                      const float* q, const float* X, long long x_bstride, const float* Y,
                                      long long y_bstride, long long y_kstride, const int* perm, float s1, float s2,
                                      float* dPre, void* dPre_bf16, long long dpre_bf16_ld, float* part_loss,
                                      float* part_dq, float* mask_out, float* pred_out, void* stream);

DL4SS_API int dl4ss_mask_attn_loss(int pass, int crm, int B, int K, int T, int F, int E, const float* V,
                                   const float* q, const float* X, long long x_bstride, const float* Y,
                                   long long y_bstride, long long y_kstride, const int* perm, float s1, float s2,
                                   float* dPre, float* part_loss, float* part_dq, float* mask_out,
                                   float* pred_out, void* stream) {
  DL4SS_REQUIRE(pass == 0 || dPre);
  return dl4ss_mask_attn_loss_ex(pass, crm, B, K, T, F, E, V, q, X, x_bstride, Y, y_bstride, y_kstride, perm, s1, s2,
                                 dPre, nullptr, 0, part_loss, part_dq, mask_out, pred_out, stream);
}

DL4SS_API int dl4ss_mask_attn_loss_ex(int pass, int crm, int B, int K, int T, int F, int E, const float* V,
                                      const float* q, const float* X, long long x_bstride, const float* Y,
                                      long long y_bstride, long long y_kstride, const int* perm, float s1, float s2,
                                      float* dPre, void* dPre_bf16, long long dpre_bf16_ld, float* part_loss,
                                      float* part_dq, float* mask_out, float* pred_out, void* stream) {
  DL4SS_REQUIRE(V);
  return attn_common(pass, crm, B, K, T, F, E, V, nullptr, q, X, x_bstride, Y, y_bstride, y_kstride, perm, s1, s2,
                     dPre, dPre_bf16, dpre_bf16_ld, part_loss, part_dq, mask_out, pred_out, stream);
}

DL4SS_API int dl4ss_mask_attn_loss_bf16v(int pass, int crm, int B, int K, int T, int F, int E, const void* V_bf16,
                                         const float* q, const float* X, long long x_bstride, const float* Y,
                                         long long y_bstride, long long y_kstride, const int* perm, float s1,
                                         float s2, float* dPre, void* dPre_bf16, long long dpre_bf16_ld,
                                         float* part_loss, float* part_dq, float* mask_out, float* pred_out,
                                         void* stream) {
  DL4SS_REQUIRE(V_bf16 && ((uintptr_t)V_bf16 & 3) == 0 && E % 2 == 0);
  return attn_common(pass, crm, B, K, T, F, E, nullptr, V_bf16, q, X, x_bstride, Y, y_bstride, y_kstride, perm, s1,
                     s2, dPre, dPre_bf16, dpre_bf16_ld, part_loss, part_dq, mask_out, pred_out, stream);
}

namespace {
int attn_common(int pass, int crm, int B, int K, int T, int F, int E, const float* V, const void* Vb, const float* q,
                const float* X, long long x_bstride, const float* Y, long long y_bstride, long long y_kstride,
                const int* perm, float s1, float s2, float* dPre, void* dPre_bf16, long long dpre_bf16_ld,
                float* part_loss, float* part_dq, float* mask_out, float* pred_out, void* stream) {
  DL4SS_REQUIRE(B > 0 && K >= 1 && K <= 3 && T > 0 && F > 0 && q && X && Y && part_loss);
  DL4SS_REQUIRE(pass == 0 || ((dPre || dPre_bf16) && part_dq));
  DL4SS_REQUIRE(!dPre_bf16 || (E % 2 == 0 && dpre_bf16_ld % 2 == 0 && dpre_bf16_ld >= (long long)F * E &&
                               ((uintptr_t)dPre_bf16 & 3) == 0));
  AttnArgs a{};
  a.B = B; a.T = T; a.F = F; a.rows_per_b = T * F; a.nblk = dl4ss_attn_nblk(T, F);
  a.V = V; a.Vb = reinterpret_cast<const unsigned short*>(Vb);
  a.q = q; a.X = X; a.xs = x_bstride; a.Y = Y; a.ys = y_bstride; a.yks = y_kstride;
  a.perm = perm; a.s1 = s1; a.s2 = s2; a.dPre = dPre; a.part_loss = part_loss; a.part_dq = part_dq;
  a.dPreB = reinterpret_cast<unsigned*>(dPre_bf16); a.ldpb = dpre_bf16_ld;
  a.mask_out = mask_out; a.pred_out = pred_out;
  return Vb ? dispatch_v<true>(E, K, crm, pass == 1, a, as_stream(stream))
            : dispatch_v<false>(E, K, crm, pass == 1, a, as_stream(stream));
}
}  // namespace

DL4SS_API int dl4ss_pit_select(const float* part_loss, int B, int K, int nblk, int* perm, void* stream) {
  DL4SS_REQUIRE(part_loss && perm && B > 0 && K >= 1 && K <= 3);
  hipStream_t st = as_stream(stream);
  dim3 grid(B), blk(64);
  if (K == 1) hipLaunchKernelGGL(pit_select_kernel<1>, grid, blk, 0, st, part_loss, B, nblk, perm);
  if (K == 2) hipLaunchKernelGGL(pit_select_kernel<2>, grid, blk, 0, st, part_loss, B, nblk, perm);
  if (K == 3) hipLaunchKernelGGL(pit_select_kernel<3>, grid, blk, 0, st, part_loss, B, nblk, perm);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

// loss_out[0] = total loss, [1] = MSE term, [2] = weighted sum-to-one term; dq (B,K,qw) = sum of partials
DL4SS_API int dl4ss_loss_finalize(const float* part_loss, int B, int K, int nblk, const int* perm, float s1,
                                  float s2, float* loss_out, const float* part_dq, int qw, float* dq,
                                  void* stream) {
  DL4SS_REQUIRE(part_loss && loss_out && B > 0 && K >= 1 && K <= 3);
  hipStream_t st = as_stream(stream);
  dim3 grid(1 + (dq ? cdiv((long long)B * K * (qw > 0 ? qw : 1), 256) : 0)), blk(256);
  if (K == 1) hipLaunchKernelGGL(finalize_kernel<1>, grid, blk, 0, st, part_loss, B, nblk, perm, s1, s2, loss_out, part_dq, qw, dq);
  if (K == 2) hipLaunchKernelGGL(finalize_kernel<2>, grid, blk, 0, st, part_loss, B, nblk, perm, s1, s2, loss_out, part_dq, qw, dq);
  if (K == 3) hipLaunchKernelGGL(finalize_kernel<3>, grid, blk, 0, st, part_loss, B, nblk, perm, s1, s2, loss_out, part_dq, qw, dq);
  DL4SS_CHECK_LAUNCH();
  return 0;
}
