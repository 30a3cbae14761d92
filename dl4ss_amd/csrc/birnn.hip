// Persistent bidirectional LSTM / GRU recurrence (forward and BPTT) for gfx950.
//
// Replaces the cuDNN recurrence of nn.LSTM(129, 300, 4, bidirectional) at
// TDAA_beta/main_run_sstune_EvalVer.py:282-293 and nn.GRU(129, 300, 2,
// bidirectional) at Torch_multi/main_run.py:263-273 / cRM_EvalVer.py:345-355
// (torch cell equations, gate order i,f,g,o / r,z,n, zero initial state).  The
// input projection X W_ih^T + b_ih is a separate MFMA GEMM (gemm.hip); this
// kernel runs the T dependent steps of one layer, both directions at once.
//
// Decomposition: the batch is cut into chunks of BC utterances; each
// (direction, chunk) is a GROUP of NG workgroups, and workgroup w of a group
// owns J hidden units (all NGATE gates of them: the four LSTM gates are fused
// into ONE matvec per direction per step, so the cell update is local).  Its
// W_hh block (NGATE*J rows x H) lives in REGISTERS for the whole launch; the
// previous hidden state is staged in LDS each step.  Only h (forward) or the
// dh partial sums (backward) cross workgroups, once per step, inside the group.
//
// Hand-off (MI355X_MICROARCH.md, Valid forms / R2 granules): every exchanged
// value is an 8-byte {tag = step+1, fp32 bits} granule written by ONE agent-
// scope relaxed atomic store (global_store sc1) and read by agent-scope
// relaxed loads (sc1) until every tag matches -- no fences, no counter.  Two
// slots alternate by step parity (a slot is rewritten only after every reader
// has consumed it, because producing step s+2 needs all of step s+1).  All
// spins are bounded: a timeout sets *status and the workgroup exits.
// Granule buffers are zeroed by hipMemsetAsync in the launch function.
// Co-residency: grid <= 240 workgroups, resources sized for >= 2 per CU.
#include "common.h"

namespace {

enum { CELL_LSTM = 0, CELL_GRU = 1 };
constexpr int NT = 256;
constexpr int WMAX = 104;   // fwd weights per thread
constexpr int RPLMAX = 20;  // bwd rows per thread
constexpr int KGLMAX = 6;   // bwd k per thread
constexpr unsigned SPIN_LIMIT = 1u << 20;  // ~1 s of polling: a stuck hand-off exits, never hangs

typedef unsigned long long u64;

__device__ __forceinline__ void put_granule(u64* g, unsigned tag, float v) {
  const u64 x = ((u64)tag << 32) | (u64)__float_as_uint(v);
  __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 get_granule(const u64* g) {
  return __hip_atomic_load(const_cast<u64*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct RnnArgs {
  int B, T, H, J, NG, nchunk;
  int KP, KPL, HP;       // fwd: k-parts, k per part (mult of 4), padded H
  int RP, RPL, KG, KGL;  // bwd: row parts, rows per part, k groups, k per group
  const float* G;        // fwd (B,T,2,NGATE*H) input projections (+ b_ih)
  const float* Whh;      // (2, NGATE*H, H)
  const float* bhh;      // (2, NGATE*H)
  float* out;            // (B,T,2H) layer output h
  float* hprev;          // (B,T,2H) h_{t-1} per step (zero at the sequence start)
  float* act;            // (B,T,2,4H) LSTM: i,f,g,o ; GRU: r,z,n,(W_hn h + b_hn)
  float* cs;             // (B,T,2,H) LSTM cell states
  const float* dOut;     // bwd (B,T,2H)
  const float* dOutB;    // bwd optional (B,2H) added to dOut at every t (d mean_t h)
  float* dG;             // bwd (B,T,2,NGATE*H) grad wrt input projection (pre-activation)
  float* dGh;            // bwd GRU: grad wrt W_hh h + b_hh (LSTM: == dG, may be null)
  u64* xbuf;             // granules
  int* status;
};

__device__ __forceinline__ void group_of(int bid, int NG, int ngroups, int& group, int& w) {
  if ((ngroups & 7) == 0) {  // keep a group's workgroups on one XCD (speed only: bid % 8 share an XCD)
    const int x = bid & 7, y = bid >> 3;
    group = x * (ngroups >> 3) + y / NG;
    w = y % NG;
  } else {
    group = bid / NG;
    w = bid % NG;
  }
}

template <int CELL, int BC, int KPL_T>
__global__ __launch_bounds__(NT, 2) void rnn_fwd_kernel(RnnArgs a) {
  constexpr int WN = KPL_T > 0 ? KPL_T : WMAX;  // weights per thread (compile-time)
  constexpr int NGATE = CELL == CELL_LSTM ? 4 : 3;
  const int H = a.H, T = a.T, J = a.J;
  const int R = NGATE * J;
  const int ngroups = 2 * a.nchunk;
  int group, w;
  group_of(blockIdx.x, a.NG, ngroups, group, w);
  const int d = group / a.nchunk, chunk = group % a.nchunk;
  const int b0 = chunk * BC;
  const int j0 = w * J;
  const int tid = threadIdx.x;
  const int GH = NGATE * H;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sh = smem;                    // [BC][HP]
  float* spart = sh + BC * a.HP;       // [KP][BC][R]

  // ---- weights of this workgroup in registers: thread (r, kp) holds W[row(r)][kp*KPL + i]
  float wreg[WN];
  const bool mv = tid < R * a.KP;
  const int r = tid % R, kp = tid / R;
  {
    const int q = r / J, u = r % J;
    const bool rv = mv && (j0 + u < H);
    const float* wrow = a.Whh + ((long long)d * GH + q * H + j0 + u) * H;
#pragma unroll
    for (int i = 0; i < WN; ++i) {
      const int k = kp * a.KPL + i;
      wreg[i] = (rv && i < a.KPL && k < H) ? wrow[k] : 0.0f;
    }
  }
  // zero the LDS h image (padding stays zero)
  for (int i = tid; i < BC * a.HP; i += NT) sh[i] = 0.0f;

  // ---- cell threads: (b, u)
  const bool ct = tid < BC * J;
  const int cb = tid / J, cu = tid % J;
  const int cj = j0 + cu;
  const int bg = b0 + cb;
  const bool cval = ct && cj < H && bg < a.B;
  float bh[NGATE];
#pragma unroll
  for (int q = 0; q < NGATE; ++q) bh[q] = cval ? a.bhh[(long long)d * GH + q * H + cj] : 0.0f;
  float hst = 0.0f, cst = 0.0f;  // h_{t-1}, c_{t-1}

  u64* xg = a.xbuf + (long long)group * 2 * BC * H;
  float gpre[NGATE];
  auto load_g = [&](int s) {
    const int t = d == 0 ? s : T - 1 - s;
#pragma unroll
    for (int q = 0; q < NGATE; ++q)
      gpre[q] = cval ? a.G[(((long long)bg * T + t) * 2 + d) * GH + q * H + cj] : 0.0f;
  };
  load_g(0);
  __syncthreads();

  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    // ---- gather h_{s-1} of the whole group (granules, tag s)
    if (s > 0) {
      const u64* src = xg + (long long)((s - 1) & 1) * BC * H;
      const unsigned tag = (unsigned)s;
      for (int i = tid; i < BC * H; i += NT) {
        u64 v = get_granule(src + i);
        unsigned spins = 0;
        while ((unsigned)(v >> 32) != tag) {
          if (++spins > SPIN_LIMIT) {
            atomicOr(a.status, 1);
            return;
          }
          __builtin_amdgcn_s_sleep(1);
          v = get_granule(src + i);
        }
        const int bb = i / H, k = i % H;
        sh[bb * a.HP + k] = __uint_as_float((unsigned)v);
      }
      __syncthreads();
    }
    // ---- fused-gate matvec partials: spart[kp][b][r] = sum_i W[r][kp*KPL+i] h[b][kp*KPL+i]
    if (mv) {
      float acc[BC];
#pragma unroll
      for (int bb = 0; bb < BC; ++bb) acc[bb] = 0.0f;
      const float* hk = sh + kp * a.KPL;
#pragma unroll
      for (int i = 0; i < WN; i += 4) {
        if (KPL_T > 0 || i < a.KPL) {
#pragma unroll
          for (int bb = 0; bb < BC; ++bb) {
            const float4 hv = *reinterpret_cast<const float4*>(hk + bb * a.HP + i);
            acc[bb] = fmaf(wreg[i], hv.x, acc[bb]);
            acc[bb] = fmaf(wreg[i + 1], hv.y, acc[bb]);
            acc[bb] = fmaf(wreg[i + 2], hv.z, acc[bb]);
            acc[bb] = fmaf(wreg[i + 3], hv.w, acc[bb]);
          }
        }
      }
#pragma unroll
      for (int bb = 0; bb < BC; ++bb) spart[(kp * BC + bb) * R + r] = acc[bb];
    }
    __syncthreads();
    // ---- cell update for (b, u)
    if (ct) {
      float hg[NGATE];
#pragma unroll
      for (int q = 0; q < NGATE; ++q) {
        float sacc = bh[q];
        for (int p = 0; p < a.KP; ++p) sacc += spart[(p * BC + cb) * R + q * J + cu];
        hg[q] = sacc;
      }
      float gx[NGATE];
#pragma unroll
      for (int q = 0; q < NGATE; ++q) gx[q] = gpre[q];
      if (s + 1 < T) load_g(s + 1);  // prefetch next step's input projection
      if (cval) {
        const long long bt = (long long)bg * T + t;
        float hn;
        float* actp = a.act + (bt * 2 + d) * (4 * H) + cj;  // act rows are 4H wide for both cells
        if constexpr (CELL == CELL_LSTM) {
          const float ig = sigmoidf_(gx[0] + hg[0]);
          const float fg = sigmoidf_(gx[1] + hg[1]);
          const float gg = tanhf(gx[2] + hg[2]);
          const float og = sigmoidf_(gx[3] + hg[3]);
          cst = fg * cst + ig * gg;
          hn = og * tanhf(cst);
          actp[0] = ig; actp[H] = fg; actp[2 * H] = gg; actp[3 * H] = og;
          a.cs[(bt * 2 + d) * H + cj] = cst;
        } else {
          const float rg = sigmoidf_(gx[0] + hg[0]);
          const float zg = sigmoidf_(gx[1] + hg[1]);
          const float ng = tanhf(gx[2] + rg * hg[2]);
          hn = (1.0f - zg) * ng + zg * hst;
          actp[0] = rg; actp[H] = zg; actp[2 * H] = ng; actp[3 * H] = hg[2];
        }
        a.hprev[bt * 2 * H + d * H + cj] = hst;
        a.out[bt * 2 * H + d * H + cj] = hn;
        hst = hn;
        put_granule(xg + (long long)(s & 1) * BC * H + cb * H + cj, (unsigned)(s + 1), hn);
      } else if (ct && cj < H) {
        // padded batch rows (bg >= B) still publish so peers never wait on them
        put_granule(xg + (long long)(s & 1) * BC * H + cb * H + cj, (unsigned)(s + 1), 0.0f);
      }
    }
    // spart is rewritten only after the next gather's barrier; sh only after this
    // step's matvec (all threads passed the barrier above) -> no extra barrier.
  }
}

// --------------------------------------------------------------------------
// BPTT.  Step s walks time backwards for the forward direction (t = T-1-s) and
// forwards for the reverse direction.  Thread (b,u) owns dh/dc of its unit;
// the recurrent term dh_rec[b][j] = sum_{rows r} dgh[b][r] W_hh[r][j] is formed
// as per-workgroup partial sums over the workgroup's own rows (registers hold
// W[rows of w][k-group]) published for all j, and each consumer sums the NG
// partials of its own units in fixed order (deterministic).
// --------------------------------------------------------------------------
template <int CELL, int BC>
__global__ __launch_bounds__(NT, 2) void rnn_bwd_kernel(RnnArgs a) {
  constexpr int NGATE = CELL == CELL_LSTM ? 4 : 3;
  const int H = a.H, T = a.T, J = a.J, NG = a.NG;
  const int R = NGATE * J;
  const int ngroups = 2 * a.nchunk;
  int group, w;
  group_of(blockIdx.x, NG, ngroups, group, w);
  const int d = group / a.nchunk, chunk = group % a.nchunk;
  const int b0 = chunk * BC;
  const int j0 = w * J;
  const int tid = threadIdx.x;
  const int GH = NGATE * H;
  const int AH = 4 * H;  // act row width (LSTM i,f,g,o; GRU r,z,n and W_hn h + b_hn)

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sdg = smem;                       // [BC][R]   dgh of this workgroup's rows
  float* spart = sdg + BC * R;             // [RP][BC][KG*KGL]
  const int KW = a.KG * a.KGL;

  // thread (kg, rp): rows [rp*RPL, +RPL), k in [kg*KGL, +KGL)
  const int kg = tid % a.KG, rp = tid / a.KG;
  const bool mv = rp < a.RP;
  float wreg[RPLMAX][KGLMAX];
#pragma unroll
  for (int i = 0; i < RPLMAX; ++i) {
    const int rr = rp * a.RPL + i;
    const int q = rr / J, u = rr % J;
    const bool rv = mv && i < a.RPL && rr < R && j0 + u < H;
    const float* wrow = a.Whh + ((long long)d * GH + q * H + j0 + u) * H;
#pragma unroll
    for (int c = 0; c < KGLMAX; ++c) {
      const int k = kg * a.KGL + c;
      wreg[i][c] = (rv && c < a.KGL && k < H) ? wrow[k] : 0.0f;
    }
  }

  const bool ct = tid < BC * J;
  const int cb = tid / J, cu = tid % J;
  const int cj = j0 + cu;
  const int bg = b0 + cb;
  const bool cval = ct && cj < H && bg < a.B;
  float dc_next = 0.0f;  // LSTM dc carried to the earlier step
  float dh_dir = 0.0f;   // GRU direct dh term carried to the earlier step

  u64* xg = a.xbuf + (long long)group * 2 * NG * BC * H;

  // prefetched per-step operands for the cell thread
  float p_dout = 0.f, p_act[4] = {0.f, 0.f, 0.f, 0.f}, p_c = 0.f, p_cprev = 0.f, p_hprev = 0.f;
  auto load_step = [&](int s) {
    if (!cval) return;
    const int t = d == 0 ? T - 1 - s : s;
    const long long bt = (long long)bg * T + t;
    p_dout = a.dOut[bt * 2 * H + d * H + cj] + (a.dOutB ? a.dOutB[(long long)bg * 2 * H + d * H + cj] : 0.0f);
    const float* ap = a.act + (bt * 2 + d) * AH + cj;
#pragma unroll
    for (int q = 0; q < 4; ++q) p_act[q] = ap[q * H];
    if constexpr (CELL == CELL_LSTM) {
      p_c = a.cs[(bt * 2 + d) * H + cj];
      const int tp = d == 0 ? t - 1 : t + 1;  // the step that ran before t in this direction
      p_cprev = (tp >= 0 && tp < T) ? a.cs[(((long long)bg * T + tp) * 2 + d) * H + cj] : 0.0f;
    } else {
      p_hprev = a.hprev[bt * 2 * H + d * H + cj];
    }
  };
  load_step(0);

  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    // ---- cell backward for (b, u)
    if (ct) {
      float dh_rec = 0.0f;
      if (s > 0 && cj < H) {
        const u64* src = xg + (long long)((s - 1) & 1) * NG * BC * H + cb * H + cj;
        const unsigned tag = (unsigned)s;
        for (int p = 0; p < NG; ++p) {
          const u64* gp = src + (long long)p * BC * H;
          u64 v = get_granule(gp);
          unsigned spins = 0;
          while ((unsigned)(v >> 32) != tag) {
            if (++spins > SPIN_LIMIT) {
              atomicOr(a.status, 2);
              return;
            }
            __builtin_amdgcn_s_sleep(1);
            v = get_granule(gp);
          }
          dh_rec += __uint_as_float((unsigned)v);
        }
      }
      const float dout = p_dout;
      float act[4] = {p_act[0], p_act[1], p_act[2], p_act[3]};
      const float c = p_c, cprev = p_cprev, hprev = p_hprev;
      if (s + 1 < T) load_step(s + 1);
      float dgi[NGATE], dgh[NGATE];
      if (cval) {
        const float dh = dout + dh_rec + dh_dir;
        if constexpr (CELL == CELL_LSTM) {
          const float ig = act[0], fg = act[1], gg = act[2], og = act[3];
          const float tc = tanhf(c);
          const float dc = dc_next + dh * og * (1.0f - tc * tc);
          dgi[0] = dc * gg * ig * (1.0f - ig);
          dgi[1] = dc * cprev * fg * (1.0f - fg);
          dgi[2] = dc * ig * (1.0f - gg * gg);
          dgi[3] = dh * tc * og * (1.0f - og);
          dc_next = dc * fg;
#pragma unroll
          for (int q = 0; q < NGATE; ++q) dgh[q] = dgi[q];
        } else {
          const float rg = act[0], zg = act[1], ng = act[2], hn = act[3];
          const float dn = dh * (1.0f - zg);
          const float dz = dh * (hprev - ng);
          dh_dir = dh * zg;
          const float dnp = dn * (1.0f - ng * ng);
          const float dr = dnp * hn;
          dgi[0] = dr * rg * (1.0f - rg);
          dgi[1] = dz * zg * (1.0f - zg);
          dgi[2] = dnp;
          dgh[0] = dgi[0];
          dgh[1] = dgi[1];
          dgh[2] = dnp * rg;
        }
        const long long bt = (long long)bg * T + t;
        float* dgp = a.dG + (bt * 2 + d) * GH + cj;
#pragma unroll
        for (int q = 0; q < NGATE; ++q) dgp[q * H] = dgi[q];
        if (CELL == CELL_GRU) {
          float* dhp = a.dGh + (bt * 2 + d) * GH + cj;
#pragma unroll
          for (int q = 0; q < NGATE; ++q) dhp[q * H] = dgh[q];
        }
      } else {
#pragma unroll
        for (int q = 0; q < NGATE; ++q) dgh[q] = 0.0f;
      }
#pragma unroll
      for (int q = 0; q < NGATE; ++q) sdg[cb * R + q * J + cu] = dgh[q];
    }
    __syncthreads();
    if (s + 1 == T) break;  // nothing flows past the sequence start
    // ---- partials P[b][k] = sum_{own rows} dgh[b][r] W[r][k]
    if (mv) {
      float acc[BC][KGLMAX];
#pragma unroll
      for (int bb = 0; bb < BC; ++bb)
#pragma unroll
        for (int c = 0; c < KGLMAX; ++c) acc[bb][c] = 0.0f;
#pragma unroll
      for (int i = 0; i < RPLMAX; ++i) {
        if (i < a.RPL) {
          const int rr = rp * a.RPL + i;
#pragma unroll
          for (int bb = 0; bb < BC; ++bb) {
            const float g = rr < R ? sdg[bb * R + rr] : 0.0f;
#pragma unroll
            for (int c = 0; c < KGLMAX; ++c) acc[bb][c] = fmaf(g, wreg[i][c], acc[bb][c]);
          }
        }
      }
#pragma unroll
      for (int bb = 0; bb < BC; ++bb)
#pragma unroll
        for (int c = 0; c < KGLMAX; ++c)
          if (c < a.KGL) spart[(rp * BC + bb) * KW + kg * a.KGL + c] = acc[bb][c];
    }
    __syncthreads();
    // ---- reduce over row parts and publish granules (tag s+1) for every k
    {
      u64* dst = xg + (long long)(s & 1) * NG * BC * H + (long long)w * BC * H;
      for (int i = tid; i < BC * H; i += NT) {
        const int bb = i / H, k = i % H;
        float v = 0.0f;
        for (int p = 0; p < a.RP; ++p) v += spart[(p * BC + bb) * KW + k];
        put_granule(dst + i, (unsigned)(s + 1), v);
      }
    }
    // sdg / spart are rewritten only after barriers every thread has passed
    __syncthreads();
  }
}

struct Plan {
  int BC, NG, J, nchunk;
  int KP, KPL, HP, RP, RPL, KG, KGL;
  size_t smem_fwd, smem_bwd;
};

bool make_plan(int cell, int B, int H, Plan& p) {
  const int ngate = cell == CELL_LSTM ? 4 : 3;
  for (int J = 20; J >= 4; --J) {
    const int R = ngate * J;
    if (R > NT) continue;
    const int KP = NT / R;
    int KPL = (H + KP - 1) / KP;
    KPL = (KPL + 3) / 4 * 4;
    if (KPL > WMAX) continue;
    // bwd: RP row parts x KG k-groups <= 256
    int best_rp = -1, best_kg = 0;
    for (int RP = 1; RP <= 16; ++RP) {
      const int RPL = (R + RP - 1) / RP;
      const int KG = NT / RP;
      const int KGL = (H + KG - 1) / KG;
      if (RPL <= RPLMAX && KGL <= KGLMAX) { best_rp = RP; best_kg = KG; break; }
    }
    if (best_rp < 0) continue;
    const int NG = (H + J - 1) / J;
    int BC = 0;
    for (int bc : {1, 2, 4, 8}) {
      const int nchunk = (B + bc - 1) / bc;
      if (2 * nchunk * NG <= 240) { BC = bc; break; }
    }
    if (!BC) continue;
    p.BC = BC; p.NG = NG; p.J = J; p.nchunk = (B + BC - 1) / BC;
    p.KP = KP; p.KPL = KPL; p.HP = KP * KPL;
    p.RP = best_rp; p.RPL = (R + best_rp - 1) / best_rp; p.KG = best_kg; p.KGL = (H + best_kg - 1) / best_kg;
    p.smem_fwd = sizeof(float) * (BC * p.HP + KP * BC * R);
    p.smem_bwd = sizeof(float) * (BC * R + p.RP * BC * p.KG * p.KGL);
    return true;
  }
  return false;
}

template <int CELL, int BC>
void launch_fwd(const RnnArgs& a, int grid, size_t smem, hipStream_t st) {
  // compile-time k-slice lengths for the shipped H = 300 plans (LSTM J=20: 100, GRU J=20: 76)
  if (a.KPL == 100)
    hipLaunchKernelGGL((rnn_fwd_kernel<CELL, BC, 100>), dim3(grid), dim3(NT), smem, st, a);
  else if (a.KPL == 76)
    hipLaunchKernelGGL((rnn_fwd_kernel<CELL, BC, 76>), dim3(grid), dim3(NT), smem, st, a);
  else
    hipLaunchKernelGGL((rnn_fwd_kernel<CELL, BC, 0>), dim3(grid), dim3(NT), smem, st, a);
}
template <int CELL, int BC>
void launch_bwd(const RnnArgs& a, int grid, size_t smem, hipStream_t st) {
  hipLaunchKernelGGL((rnn_bwd_kernel<CELL, BC>), dim3(grid), dim3(NT), smem, st, a);
}

template <int CELL>
int dispatch(bool fwd, int BC, const RnnArgs& a, int grid, size_t smem, hipStream_t st) {
  switch (BC) {
    case 1: fwd ? launch_fwd<CELL, 1>(a, grid, smem, st) : launch_bwd<CELL, 1>(a, grid, smem, st); break;
    case 2: fwd ? launch_fwd<CELL, 2>(a, grid, smem, st) : launch_bwd<CELL, 2>(a, grid, smem, st); break;
    case 4: fwd ? launch_fwd<CELL, 4>(a, grid, smem, st) : launch_bwd<CELL, 4>(a, grid, smem, st); break;
    case 8: fwd ? launch_fwd<CELL, 8>(a, grid, smem, st) : launch_bwd<CELL, 8>(a, grid, smem, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  DL4SS_CHECK_LAUNCH();
  return 0;
}

void fill_args(RnnArgs& a, const Plan& p, int B, int T, int H) {
  a.B = B; a.T = T; a.H = H; a.J = p.J; a.NG = p.NG; a.nchunk = p.nchunk;
  a.KP = p.KP; a.KPL = p.KPL; a.HP = p.HP;
  a.RP = p.RP; a.RPL = p.RPL; a.KG = p.KG; a.KGL = p.KGL;
}

}  // namespace

DL4SS_API long long dl4ss_birnn_workspace_bytes(int cell, int B, int H) {
  Plan p;
  if (!make_plan(cell, B, H, p)) return -1;
  const long long groups = 2LL * p.nchunk;
  const long long fwd = groups * 2 * p.BC * H * 8;
  const long long bwd = groups * 2 * p.NG * p.BC * H * 8;
  return fwd > bwd ? fwd : bwd;
}

DL4SS_API int dl4ss_birnn_fwd(int cell, int B, int T, int H, const float* G, const float* W_hh, const float* b_hh,
                              float* out, float* hprev, float* act, float* cs, void* workspace,
                              long long ws_bytes, int* status, void* stream) {
  DL4SS_REQUIRE(cell == CELL_LSTM || cell == CELL_GRU);
  DL4SS_REQUIRE(B > 0 && T > 0 && H > 0 && G && W_hh && b_hh && out && hprev && act && workspace && status);
  DL4SS_REQUIRE(cell == CELL_GRU || cs);
  Plan p;
  DL4SS_REQUIRE(make_plan(cell, B, H, p));
  DL4SS_REQUIRE(ws_bytes >= dl4ss_birnn_workspace_bytes(cell, B, H));
  hipStream_t st = as_stream(stream);
  const long long groups = 2LL * p.nchunk;
  hipError_t e = hipMemsetAsync(workspace, 0, groups * 2 * p.BC * H * 8, st);
  if (e != hipSuccess) return (int)e;
  RnnArgs a{};
  fill_args(a, p, B, T, H);
  a.G = G; a.Whh = W_hh; a.bhh = b_hh; a.out = out; a.hprev = hprev; a.act = act; a.cs = cs;
  a.xbuf = reinterpret_cast<unsigned long long*>(workspace);
  a.status = status;
  const int grid = (int)(groups * p.NG);
  return cell == CELL_LSTM ? dispatch<CELL_LSTM>(true, p.BC, a, grid, p.smem_fwd, st)
                           : dispatch<CELL_GRU>(true, p.BC, a, grid, p.smem_fwd, st);
}

DL4SS_API int dl4ss_birnn_bwd(int cell, int B, int T, int H, const float* dOut, const float* dOut_bcast,
                              const float* W_hh,
                              const float* act, const float* cs, const float* hprev, float* dG, float* dGh,
                              void* workspace, long long ws_bytes, int* status, void* stream) {
  DL4SS_REQUIRE(cell == CELL_LSTM || cell == CELL_GRU);
  DL4SS_REQUIRE(B > 0 && T > 0 && H > 0 && dOut && W_hh && act && dG && workspace && status);
  DL4SS_REQUIRE(cell == CELL_GRU ? (dGh && hprev) : (cs != nullptr));
  Plan p;
  DL4SS_REQUIRE(make_plan(cell, B, H, p));
  DL4SS_REQUIRE(ws_bytes >= dl4ss_birnn_workspace_bytes(cell, B, H));
  hipStream_t st = as_stream(stream);
  const long long groups = 2LL * p.nchunk;
  hipError_t e = hipMemsetAsync(workspace, 0, groups * 2 * p.NG * p.BC * H * 8, st);
  if (e != hipSuccess) return (int)e;
  RnnArgs a{};
  fill_args(a, p, B, T, H);
  a.Whh = W_hh; a.act = const_cast<float*>(act); a.cs = const_cast<float*>(cs);
  a.hprev = const_cast<float*>(hprev); a.dOut = dOut; a.dOutB = dOut_bcast; a.dG = dG; a.dGh = dGh;
  a.xbuf = reinterpret_cast<unsigned long long*>(workspace);
  a.status = status;
  const int grid = (int)(groups * p.NG);
  return cell == CELL_LSTM ? dispatch<CELL_LSTM>(false, p.BC, a, grid, p.smem_bwd, st)
                           : dispatch<CELL_GRU>(false, p.BC, a, grid, p.smem_bwd, st);
}
