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
//
// Wave roles (512 threads = 8 waves, 2 per SIMD): a wave's vmcnt retires
// loads and stores in issue order, so a wave that polls granules must not
// carry outstanding stores.  Waves 0-3 do the cell update and ALL global
// stores (granules first, then prefetch loads for the next step, then the
// saved activations); waves 4-7 only poll granules into LDS.  All 8 waves run
// the register-resident matvec (two waves per SIMD keep the VALU issuing).
// The packed bf16 kernels (rnn_fwd_pk_kernel / rnn_bwd_pk_kernel, below) split the roles
// differently: waves 0-3 cell + stores, FWD_NPW / BWD_NPW polling waves from wave 4 (the
// forward's second one is wave 7), the rest MFMA tiles + prefetch (see their comments).
// Co-residency: every workgroup of a launch must be resident at once; the plan keeps the
// grid within the device's CUs minus 1/16 (240 on a full MI355X, wg_limit) and every launch
// re-checks it against CUs x occupancy (launch_resident).
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include "common.h"

namespace {

enum { CELL_LSTM = 0, CELL_GRU = 1 };
constexpr int NT = 512;
constexpr int NROLE = 256;   // [0,256): cell + publish ; [256,512): gather
constexpr int WMAX = 64;     // fwd weights per thread (generic path)
constexpr int RPLMAX = 20;   // bwd rows per thread
constexpr int KGLMAX = 6;    // bwd k per thread
constexpr int HMAX = 320;    // largest hidden size of the training kernels (sizes per-thread offset arrays)
constexpr int HMAX_L = 640;  // largest hidden size of the forward-only (inference) instantiations: the
                             // H = 600 speaker classifier of EvalVer.py:305-326 / GRID.py:178-199
constexpr int DL4SS_RNN_WS_ZEROED = 0x100;  // precision flag: workspace already zero (no memset)
constexpr int DL4SS_RNN_DEFER_BIAS = 0x400;  // BPTT: leave the per-row bias partials for dl4ss_birnn_bias_reduce
constexpr int DL4SS_RNN_DGH_PAD8 = 0x200;  // precision flag (bwd): dGh_bf16 direction stride padded to 8
constexpr int DL4SS_RNN_DOUT_SLABS_MASK = 0x3000;  // precision field (bwd): dOut = (S - 1) << 12 split-K slabs
constexpr unsigned SPIN_LIMIT = 1u << 20;  // ~1 s of polling: a stuck hand-off exits, never hangs

typedef unsigned long long u64;

// Diagnostic build only (-DRNN_STAMPS, tools/build_stamps.py): per-phase s_memtime
// sums for threads 0 (cell/publish role) and 256 (gather role) of every workgroup.
#ifdef RNN_STAMPS
__device__ __forceinline__ u64 stamp_now() {
  u64 t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP_DECL u64 st_prev = stamp_now(), st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define STAMP(i) { const u64 n_ = stamp_now(); st_acc[i] += n_ - st_prev; st_prev = n_; }
#ifndef STAMP_T2
#define STAMP_T2 NROLE  // the second recorded thread (320: the first prefetch wave of the packed forward)
#endif
#define STAMP_FLUSH                                                                   \
  if (a.stamps && (threadIdx.x == 0 || threadIdx.x == STAMP_T2))                     \
    for (int i_ = 0; i_ < 8; ++i_) a.stamps[blockIdx.x * 16 + (threadIdx.x ? 8 : 0) + i_] = st_acc[i_];
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH
#endif
// Diagnostic build only (-DRNN_TRACE): per (workgroup, step) s_memrealtime (100 MHz, chip-wide)
// of the publish (slot 0) and of the completed poll (slot 1) in a.stamps[(bid * T + s) * 2 + slot].
#ifdef RNN_TRACE
__device__ __forceinline__ u64 rtc_now() {
  u64 t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define TRACE(slot, s) do { if (a.stamps && (threadIdx.x & 63) == 0) a.stamps[((long long)blockIdx.x * a.T + (s)) * 4 + (slot)] = rtc_now(); } while (0)
#else
#define TRACE(slot, s) do { } while (0)
#endif

// Gate nonlinearities on the serial critical path: v_exp + v_rcp (1 ulp) instead of
// the IEEE division / ocml tanh sequences (the cell update runs on one wave).
__device__ __forceinline__ float fsig(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// tanh(x) = 2 / (1 + 2^(x (-2 log2 e))) - 1: the constant folded into ONE multiply (-2 log2e is exact in
// fp32, so x * (-2 L) rounds the same product as (-2 x) * L did -- bitwise the two-multiply form, one
// dependent VALU op shorter on the recurrences' critical cell chain)
__device__ __forceinline__ float ftanh(float x) {
  return 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -2.88539008177792681472f)) - 1.0f;
}

typedef short bf16x8 __attribute__((ext_vector_type(8)));

// Sum of the NG producers' dh partials p[i * stride] (BPTT cell phase): for NG <= 16 all
// loads are issued at once and added as a pairwise tree.  (A runtime-bound loop compiled to
// an 8-wide unrolled body plus a remainder loop with one LDS round trip per iteration:
// ~800 of the cell phase's ~1500 cycles per step at NG = 15.)
__device__ __forceinline__ float sum_partials(const float* p, int stride, int NG) {
  if (NG > 16) {
    float a = 0.0f;
    for (int i = 0; i < NG; ++i) a += p[i * stride];
    return a;
  }
  // branch-free: 16 loads from valid addresses (index clamped to NG - 1), then a select --
  // a guarded load per element compiled to a branch and a saved exec mask each
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float x = p[(i < NG ? i : NG - 1) * stride];
    v[i] = i < NG ? x : 0.0f;
  }
#pragma unroll
  for (int w = 8; w > 0; w >>= 1)
#pragma unroll
    for (int i = 0; i < w; ++i) v[i] += v[i + w];
  return v[0];
}
// Sum of 16 producers' dh partials p[i * stride] for the packed BPTT, whose partial buffer
// always holds 16 producer rows (rows >= NG stay zero): no index clamp, no select.  Same
// pairwise tree as sum_partials, so the result is bitwise the same.
__device__ __forceinline__ float sum_partials16(const float* p, int stride) {
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = p[i * stride];
#pragma unroll
  for (int w = 8; w > 0; w >>= 1)
#pragma unroll
    for (int i = 0; i < w; ++i) v[i] += v[i + w];
  return v[0];
}
// Sum of N slot partials p[i * stride], i < N, as a fixed pairwise tree over the next power of two
// (missing leaves are zero): deterministic, and for N = 16 the tree of sum_partials16.
template <int N>
__device__ __forceinline__ float sum_slots(const float* p, int stride) {
  constexpr int P2 = N <= 1 ? 1 : N <= 2 ? 2 : N <= 4 ? 4 : N <= 8 ? 8 : 16;
  static_assert(N >= 1 && N <= 16, "1..16 slots");
  float v[P2];
#pragma unroll
  for (int i = 0; i < P2; ++i) v[i] = i < N ? p[i * stride] : 0.0f;
#pragma unroll
  for (int w = P2 / 2; w > 0; w >>= 1)
#pragma unroll
    for (int i = 0; i < w; ++i) v[i] += v[i + w];
  return v[0];
}
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned short bf16_rne(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFF + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
// The weights are rounded with the same plain RNE when a launch loads its W_hh fragments.  No NaN
// special case here: values formed by arithmetic are canonical quiet NaNs (0x7FC00000 / 0xFFC00000),
// which round to NaN, and the NaN-preserving form (bf16_bits_rne) in the once-per-launch weight
// loads changed the packed kernels' code generation enough to cost 4.3 % of the step (A/B, 20 steps
// x 2 alternating runs: 7768 / 7776 vs 8109 / 8097 mixtures/s, round 4).

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
  const float* dOut;     // bwd (B,T,2H), or dout_ns split-K slabs of it dout_zs floats apart (summed in order)
  int dout_ns;
  long long dout_zs;
  const float* dOutB;    // bwd optional (B,2H) added to dOut at every t (d mean_t h)
  float* dG;             // bwd (B,T,2,NGATE*H) grad wrt input projection (pre-activation)
  float* dGh;            // bwd GRU: grad wrt W_hh h + b_hh (LSTM: == dG, may be null)
  u64* xbuf;             // granules
  int* status;
  unsigned spin_limit;   // polls before a hand-off times out (SPIN_LIMIT; dl4ss_debug_set_spin_limit)
  int place_force;       // packed kernels: 1 = write-through hand-off regardless of placement (test hook)
  u64* stamps;           // diagnostic build only
  // bf16 mode extras (packed kernels only; any may be null)
  unsigned short* outb;    // fwd (B,T,2H) bf16(h)          -- next layer's / Linear's GEMM operand
  unsigned short* hprevb;  // fwd (B,T,2H) bf16(h_{t-1})    -- dW_hh GEMM operand
  unsigned short* dGb;     // bwd (B,T,2,NGATE*H) bf16(dG)  -- dW_ih / dX GEMM operand
  unsigned short* dGhb;    // bwd GRU: bf16(dGh)            -- dW_hh GEMM operand
  int ghb;                 // bwd GRU: dGhb's per-direction column stride (NGATE*H, or padded to a
                           //      multiple of 8 by DL4SS_RNN_DGH_PAD8: 16-B aligned GEMM operand rows)
  float* dbi;              // bwd: += sum_{b,t} dG   (bias_ih gradient, (2, NGATE*H))
  float* dbh;              // bwd: += sum_{b,t} dGh  (bias_hh gradient)
  float* dbpart;           // bwd: per-row bias sums [b][d][ih | hh][NGATE*H] (fixed-order reduce), or
                           //      null: float atomics straight into dbi / dbh
  // fused input projection (packed forward, rnn_fwd_pk_kernel<.., true>): G is not read; each
  // step's x_t W_ih^T + b_ih is formed in the kernel from the bf16 layer input
  const unsigned short* Xb;    // (B*T, ldx) bf16 layer input rows, k < Kin (padding never read)
  const unsigned short* Wihb;  // (2*NGATE*H, ldw) bf16 W_ih rows (direction-major), k < Kin
  const float* bih;            // (2, NGATE*H)
  int Kin;
  long long ldx, ldw;
  // act layout: 0 gate-major (B,T,2,4H); 1 cell-major (B,T,2,H,4) -- the packed kernels at BC >= 4
  // (act_cell_major): the forward stores a cell's four gates as one 16-B store, the BPTT loads them
  // as one 16-B item
  int act_cm;
  float* hmean;  // fwd (packed): (B, 2H) mean over t of h, summed by each cell lane in step order (or null)
  unsigned* gctl;  // packed kernels: the group-formation counters (zeroed with the workspace; group_pk)
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

// Per-timestep operand prefetch, run by the gather waves so that the cell waves
// issue no loads at all (their vmcnt then only ever holds stores): item q is
// p[q][(t + shift[q]) * stride[q]] (0 outside [0, T)), landing in LDS at dst[q].
// Loads for step s+1 are issued during step s and committed to LDS at step s+1
// (by then the granule poll has already waited past them).
// NZ > 1 (the BPTT's dOut, DL4SS_RNN_DOUT_SLABS): an item with zq[q] set is the sum of NZ split-K
// slabs zs floats apart, all loaded at issue and added at commit in slab order from zero -- bitwise the
// gemm_gl split-K combine it replaces (((0 + s0) + s1) + ...).  NZ is the launch's exact slab count (a
// kernel template argument): a runtime count per item (round 6's first form, NZ = 4 in every launch)
// cost ~20 us per BPTT launch even at one slab (profiles/r06_nz_ab.txt).
template <int NQ, int NZ = 1>
struct StepLoader {
  const float* p[NQ];
  int stride[NQ], shift[NQ], dst[NQ];
  float v[NQ];
  bool zq[NQ];
  long long zs;
  float vz[NQ][NZ > 1 ? NZ - 1 : 1];
  __device__ __forceinline__ void issue(int t, int T) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int tt = t + shift[q];
      const bool ok = p[q] != nullptr && tt >= 0 && tt < T;
      v[q] = ok ? p[q][(long long)tt * stride[q]] : 0.0f;
      if constexpr (NZ > 1) {
#pragma unroll
        for (int z = 1; z < NZ; ++z)
          vz[q][z - 1] = (ok && zq[q]) ? p[q][(long long)tt * stride[q] + z * zs] : 0.0f;
      }
    }
  }
  __device__ __forceinline__ void commit(float* lds) const {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (dst[q] < 0) continue;
      float x = v[q];
      if constexpr (NZ > 1) {
        if (zq[q]) {
          x = 0.0f + v[q];
#pragma unroll
          for (int z = 1; z < NZ; ++z) x += vz[q][z - 1];
        }
      }
      lds[dst[q]] = x;
    }
  }
};

// Fused input projection: the step's layer-input rows reach LDS by LDS-DMA (16 B per lane,
// lane-linear 1-KB pieces): item i = b * 80 + c is 16-B chunk c (k = 8c .. 8c + 7) of batch row b
// of the chunk, at element 8 i of a step buffer ([b][640] bf16).  Items past the data (c >= Kin / 8
// rounded up, rows past B, the pad items of the last piece) read a global zero line.
typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __attribute__((aligned(64))) const unsigned g_xzero_line[16] = {0};

// Poll the granules src[off[g]] (off < 0: nothing to read) until every tag == tag;
// returns false on timeout.  Offsets are computed once per launch by the caller;
// all loads of the thread are in flight at once and only stale ones are re-issued.
template <int GM>
__device__ __forceinline__ bool gather(const u64* src, const int (&off)[GM], unsigned tag, u64 (&v)[GM],
                                       unsigned limit) {
  const u64 done = (u64)tag << 32;
#pragma unroll
  for (int g = 0; g < GM; ++g) v[g] = off[g] >= 0 ? get_granule(src + off[g]) : done;
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int g = 0; g < GM; ++g) ok &= (unsigned)(v[g] >> 32) == tag;
    if (ok) return true;
    if (++spins > limit) return false;
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int g = 0; g < GM; ++g)
      if ((unsigned)(v[g] >> 32) != tag) v[g] = get_granule(src + off[g]);
  }
}

// MF = false: exact fp32 matvec on the VALU (the parity mode); W_hh slice in fp32
//      registers, k split over KP thread parts, partial sums combined by the cell thread.
// MF = true: bf16 MFMA matvec (v_mfma_f32_16x16x32_bf16, fp32 accumulate; the
//      throughput mode): wave m owns the 16-row tile m of W_hh (bf16 A fragments in
//      registers for all K), h staged in LDS as bf16 [batch][k] (the B operand), one
//      MFMA chain per wave -- no partial sums at all.
template <int CELL, int BC, int KPL_T, bool MF, int HM = HMAX>
__global__ __launch_bounds__(NT, 1) void rnn_fwd_kernel(RnnArgs a) {
  constexpr int WN = MF ? 1 : (KPL_T > 0 ? KPL_T : WMAX);  // fp32 weights per thread (compile-time)
  constexpr int NGATE = CELL == CELL_LSTM ? 4 : 3;
  constexpr int KSMAX = HM / 32;
  const int H = a.H, T = a.T, J = a.J;
  const int R = NGATE * J;
  const int ngroups = 2 * a.nchunk;
  int group, w;
  group_of(blockIdx.x, a.NG, ngroups, group, w);
  const int d = group / a.nchunk, chunk = group % a.nchunk;
  const int b0 = chunk * BC;
  const int j0 = w * J;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int GH = NGATE * H;
  const int MT = (R + 15) / 16;
  constexpr int SHB = KSMAX * 32 + 8;  // bf16 row stride of the MFMA B image (k >= H stays zero)

  extern __shared__ __attribute__((aligned(16))) float smem[];
  // fp32 path: sh [BC][HP], spart [KP][BC][R]; MFMA path: shb bf16 [16][SHB], sgate [BC][MT*16]
  float* sh = smem;
  float* spart = sh + BC * a.HP;
  unsigned short* shb = reinterpret_cast<unsigned short*>(smem);
  float* sgate = smem + 8 * SHB;  // after 16 x SHB bf16
  float* sin = MF ? sgate + BC * MT * 16 : spart + a.KP * BC * R;  // [2][BC*J][4] step inputs (double buffer)

  // ---- weights of this workgroup in registers
  float wreg[WN];
  bf16x8 afrag[MF ? KSMAX : 1];
  const bool mv = MF ? wv < MT : tid < R * a.KP;
  const int r = tid % R, kp = tid / R;
  if constexpr (!MF) {  // thread (r, kp) holds W[row(r)][kp*KPL + i]
    const int q = r / J, u = r % J;
    const bool rv = mv && (j0 + u < H);
    const float* wrow = a.Whh + ((long long)d * GH + q * H + j0 + u) * H;
#pragma unroll
    for (int i = 0; i < WN; ++i) {
      const int k = kp * a.KPL + i;
      wreg[i] = (rv && i < a.KPL && k < H) ? wrow[k] : 0.0f;
    }
    for (int i = tid; i < BC * a.HP; i += NT) sh[i] = 0.0f;  // padding stays zero
  } else {  // lane holds A[row m*16 + (lane&15)][k = ks*32 + 8(lane>>4) + j]
    const int rl = wv * 16 + (lane & 15);
    const int q = rl / J, u = rl % J;
    const bool rv = mv && rl < R && j0 + u < H;
    const float* wrow = a.Whh + ((long long)d * GH + q * H + j0 + u) * H;
#pragma unroll
    for (int ks = 0; ks < KSMAX; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = ks * 32 + 8 * (lane >> 4) + j;
        afrag[ks][j] = (short)bf16_rne((rv && k < H) ? wrow[k] : 0.0f);
      }
    for (int i = tid; i < 8 * SHB; i += NT) smem[i] = 0.0f;  // bf16 image incl. padding rows/cols
  }

  // ---- cell threads (waves 0-3): (b, u)
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
  // gather role: granule offsets and LDS destinations, fixed for the whole launch
  constexpr int GM = (BC * HM + NROLE - 1) / NROLE;
  int goff[GM], gdst[GM];
#pragma unroll
  for (int g = 0; g < GM; ++g) {
    const int i = tid - NROLE + g * NROLE;
    const bool on = tid >= NROLE && i < BC * H;
    goff[g] = on ? i : -1;
    gdst[g] = on ? (i / H) * (MF ? SHB : a.HP) + i % H : 0;
  }
  // gather role: input projection G[b][t][d][q*H + j] of every own (b, unit, gate)
  constexpr int NQ = (BC * 20 * 4 + NROLE - 1) / NROLE;
  StepLoader<NQ> ld;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int i = tid - NROLE + q * NROLE;  // item = gate * (BC*J) + cell
    const int gate = i / (BC * J), cell = i % (BC * J);
    const int ib = b0 + cell / J, ij = j0 + cell % J;
    const bool on = tid >= NROLE && gate < NGATE;
    ld.p[q] = (on && ib < a.B && ij < H) ? a.G + ((long long)ib * T * 2 + d) * GH + gate * H + ij : nullptr;
    ld.stride[q] = 2 * GH;
    ld.shift[q] = 0;
    ld.dst[q] = on ? cell * 4 + gate : -1;
  }
  if (tid >= NROLE) ld.issue(d == 0 ? 0 : T - 1, T);
  __syncthreads();
  STAMP_DECL

  // ---- fused-gate matvec partials: spart[kp][b][r] = sum_i W[r][kp*KPL+i] h[b][kp*KPL+i]
  auto matvec = [&]() {
    if (!mv) return;
    if constexpr (MF) {  // sgate[b][m*16 + row] = sum_k W[row][k] h[b][k]
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const unsigned short* bp = shb + (lane & 15) * SHB + 8 * (lane >> 4);
      bf16x8 bv[KSMAX];  // all B reads in flight before the MFMA chain (zero A/B beyond H)
#pragma unroll
      for (int ks = 0; ks < KSMAX; ++ks) bv[ks] = *reinterpret_cast<const bf16x8*>(bp + ks * 32);
#pragma unroll
      for (int ks = 0; ks < KSMAX; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afrag[ks], bv[ks], acc, 0, 0, 0);
      const int col = lane & 15;
      if (col < BC) {
#pragma unroll
        for (int i = 0; i < 4; ++i) sgate[col * MT * 16 + wv * 16 + (lane >> 4) * 4 + i] = acc[i];
      }
      return;
    }
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
  };

  // Role-split loops with the same barrier sequence per step (B1, B2).  Waves 4-7
  // (gather) issue only loads, waves 0-3 (cell) only stores, so neither loop's
  // waitcnt state ever has to drain the other kind.
  if (tid >= NROLE) {
    for (int s = 0; s < T; ++s) {
      // ---- gather h_{s-1} (granules, tag s) and commit this step's inputs
      if (s > 0) {
        u64 v[GM];
        if (!gather<GM>(xg + (long long)((s - 1) & 1) * BC * H, goff, (unsigned)s, v, a.spin_limit)) {
          atomicOr(a.status, 1);
          return;
        }
#pragma unroll
        for (int g = 0; g < GM; ++g)
          if (goff[g] >= 0) {
            if constexpr (MF)
              shb[gdst[g]] = bf16_rne(__uint_as_float((unsigned)v[g]));
            else
              sh[gdst[g]] = __uint_as_float((unsigned)v[g]);
          }
      }
      ld.commit(sin + (s & 1) * BC * J * 4);
      if (s + 1 < T) ld.issue(d == 0 ? s + 1 : T - 2 - s, T);
      STAMP(0)
      __syncthreads();  // B1
      STAMP(1)
      matvec();
      STAMP(2)
      __syncthreads();  // B2
      STAMP(3)
    }
    STAMP_FLUSH
    return;
  }
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    STAMP(0)
    __syncthreads();  // B1
    STAMP(1)
    matvec();
    STAMP(2)
    __syncthreads();  // B2
    STAMP(3)
    // ---- cell update for (b, u): publish first, then the saved state
    if (ct) {
      float hg[NGATE];
#pragma unroll
      for (int q = 0; q < NGATE; ++q) {
        float sacc = bh[q];
        if constexpr (MF)
          sacc += sgate[cb * MT * 16 + q * J + cu];
        else
          for (int p = 0; p < a.KP; ++p) sacc += spart[(p * BC + cb) * R + q * J + cu];
        hg[q] = sacc;
      }
      float gx[NGATE];
#pragma unroll
      for (int q = 0; q < NGATE; ++q) gx[q] = sin[(s & 1) * BC * J * 4 + tid * 4 + q];
      if (cj < H) {
        float hn = 0.0f, st[4] = {0.f, 0.f, 0.f, 0.f};
        if (cval) {
          if constexpr (CELL == CELL_LSTM) {
            const float ig = fsig(gx[0] + hg[0]);
            const float fg = fsig(gx[1] + hg[1]);
            const float gg = ftanh(gx[2] + hg[2]);
            const float og = fsig(gx[3] + hg[3]);
            cst = fg * cst + ig * gg;
            hn = og * ftanh(cst);
            st[0] = ig; st[1] = fg; st[2] = gg; st[3] = og;
          } else {
            const float rg = fsig(gx[0] + hg[0]);
            const float zg = fsig(gx[1] + hg[1]);
            const float ng = ftanh(gx[2] + rg * hg[2]);
            hn = (1.0f - zg) * ng + zg * hst;
            st[0] = rg; st[1] = zg; st[2] = ng; st[3] = hg[2];
          }
        }
        // padded batch rows (bg >= B) still publish (zeros) so peers never wait on them
        put_granule(xg + (long long)(s & 1) * BC * H + cb * H + cj, (unsigned)(s + 1), hn);
        if (cval) {
          const long long bt = (long long)bg * T + t;
          float* actp = a.act + (bt * 2 + d) * (4 * H) + cj;  // act rows are 4H wide for both cells
          actp[0] = st[0]; actp[H] = st[1]; actp[2 * H] = st[2]; actp[3 * H] = st[3];
          if constexpr (CELL == CELL_LSTM) a.cs[(bt * 2 + d) * H + cj] = cst;
          a.hprev[bt * 2 * H + d * H + cj] = hst;
          a.out[bt * 2 * H + d * H + cj] = hn;
        }
        hst = hn;
      }
    }
    STAMP(4)
    // sh is rewritten only after the next gather's barrier (all matvec reads are
    // behind the barrier above); spart only after that barrier too.
  }
  STAMP_FLUSH
}

// --------------------------------------------------------------------------
// Forward, bf16 MFMA mode with the PACKED hand-off (the throughput path).
//
// Measured on MI355X (tools/rnn_stamps.py, tools/rnn_trace.py; B = 32, H = 300):
// the one-value-granule kernel above spends ~5k of its 6.7k cycles per step in the
// hand-off.  Three changes, each timed:
//  * h crosses workgroups already rounded to bf16 (the consumer rounds it anyway:
//    results are bit-identical), three values per 8-B granule
//      granule = { lo: v0 | v1 << 16, hi: v2 | tag << 16 },  16-bit tag = step + 1,
//    two granules per 16-B store, 8 granules per (batch row, producer);
//  * ONE wave polls, keeping two sweeps in flight (the older one is merged while
//    the newer one travels): hand-off 2.3 -> 1.9 us;
//  * granules written with PLAIN stores and read with `sc1` loads: a plain store
//    lands in the producer XCD's L2, which same-XCD consumers read directly, while an
//    `sc1` store drops the line from L2 and the reader goes to the Infinity Fabric:
//    hand-off 1.9 -> 0.96 us, step 2.68 -> 1.64 us.  A group's workgroups are placed
//    on one XCD (group_of), but placement is speed only, never correctness: at launch
//    start every workgroup of a group publishes its XCC id (group_needs_write_through)
//    and only a group found on ONE XCD uses plain stores; a group that spans XCDs writes
//    every granule `sc1` (the validated write-through form, MI355X_MICROARCH.md, Valid
//    forms R2).  (Round 1 wrote every granule twice, plain + `sc1`, and switched a
//    consumer to the `sc1` copy after a stalled poll: the second store cost ~600 cycles
//    of a BPTT step's publish.)  Every value is validated by its own tag either way.
// Waves (FWD_NPW polling waves, default 2): 0-3 MFMA tiles 0-3 + cell update + publish +
//        saved-state stores; 4 polls, and 7 (FWD_NPW >= 2) and 6 (FWD_NPW == 3) poll too
//        (those waves hold no MFMA tile); the remaining waves of 5-7 run MFMA tiles 4..MT-1
//        and the per-step input prefetch.
// Each MFMA tile runs FWD_MV_CHAINS independent accumulator chains over its k-steps.
// --------------------------------------------------------------------------
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int PKU = 24;     // staged h slots per (row, producer): 8 granules x 3
constexpr int XKMAX = 2 * HMAX / 32;  // fused input projection: k-steps of 32 (Kin <= 2 HMAX)
// bf16 row stride of its B images: 80 16-B chunks of data + 2 pad chunks (656 bf16 = 328 dwords:
// the BC rows and the zero row land on distinct bank quads for every 16-lane ds_read_b128
// group; at 80 chunks every row started on bank 0, a 4-way conflict, tools/lds_banks.py)
constexpr int SXC = XKMAX * 4 + 2;    // 16-B chunks per row
constexpr int SXB = SXC * 8;
// Fused projection in blocks: one MFMA's 16 B-columns are SPB = 16 / BC consecutive steps x BC
// batch rows, so a tile's projection of a whole block of SPB steps is ONE XK-long MFMA chain
// (a quarter of a per-step form's MFMAs at BC = 4); the chain of block k+1 is split into SPB
// parts, one per step of block k.  The layer-input rows sit in a ring of 3 blocks of step slots
// (slot stride XBUF + 16 BC bf16: the 16 columns' rows on distinct bank quads,
// tools/lds_banks.py), DMA'd two blocks ahead of use.
__host__ __device__ constexpr int xw_spb(int bc) { return 16 / bc; }
// Packed forward's per-step input projections, one slab per step slot: [cell = b * J + u][4 gates],
// read by each cell lane as ONE float4; slab stride BC * 128 + 4 floats (= 4 mod 8).  The fused
// projection's block epilogue (xfinal) stores one gate of 16 (step, batch row) columns per
// instruction: with [b * 32 + u][4] records in 512-float slabs all 16 hit ONE bank (a 16-way
// conflict, ~150 conflict cycles per step and workgroup, SQ_LDS_BANK_CONFLICT / IDX_ACTIVE of the
// fused kernels 0.32 / 0.35); dense rows and the odd quad in the slab stride spread them over 8
// banks (tools/lds_banks.py: 600 -> 104 conflict cycles per block).  A gate-major layout (one
// 16-B epilogue store per lane, conflict-free) measured slower: the cell lanes' 4 scalar reads
// instead of one float4 cost the 600-wide layers 9-17 us per launch (round 4)
__host__ __device__ constexpr int sin_slab(int bc) { return bc * 32 * 4 + 4; }
__host__ __device__ constexpr int xw_nxq(int bc) { return (bc * SXC + 127) / 128; }
__host__ __device__ constexpr int xw_slot(int bc) { return xw_nxq(bc) * 128 * 8 + 16 * bc; }  // bf16
__host__ __device__ constexpr int xw_ring_bf16(int bc) { return 3 * xw_spb(bc) * xw_slot(bc); }
constexpr int WPOLL = 4;    // the polling wave (BPTT: the first of BWD_NPW)
#ifndef BWD_NPW
#define BWD_NPW 2  // BPTT polling waves
#endif
constexpr int FWD_MV_CHAINS = 2;  // forward bf16 matvec: accumulator chains per MFMA tile (4: 367 vs 363 us per pass)
#ifndef FWD_XDMA_EARLY
#define FWD_XDMA_EARLY 0  // 1: the fused forward's input-row DMA issued after B1 instead of after B2 (C2: 3.540 vs 3.498 ms per step, A/B x3, round 5: slower)
#endif
#ifndef FWD_NPW
#define FWD_NPW 2  // forward polling waves: 4, and 7 when >= 2, and 6 when 3 (their MFMA tile indices must be >= MT)
#endif
static_assert(FWD_MV_CHAINS >= 1 && FWD_MV_CHAINS <= 8, "FWD_MV_CHAINS: 1..KSMAX accumulator chains");
static_assert(FWD_NPW >= 1 && FWD_NPW <= 3, "FWD_NPW: 1..3 polling waves");
static_assert(BWD_NPW >= 1 && BWD_NPW <= 3, "BWD_NPW: 1..3 polling waves");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t granule_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xFu;
}

// Group formation of the packed kernels by PLACEMENT, not by block index (round 5).  group_of assumes
// blocks b and b + 8 share an XCD -- true when a launch is dispatched alone, but a kernel dispatched
// concurrently on another stream (the side-stream GEMM, RCCL kernels) interleaves its workgroups into the
// XCD round robin, the groups then span XCDs, and every hand-off of the launch goes write-through and
// cross-XCD: the BPTT ran at twice its time (662 vs 336 us per launch).  Here each workgroup takes a slot
// on a per-XCD counter (device-scope atomic, returning): slot s < cap = NG * ngroups / 8 of XCD x is
// member s % NG of group x * ngroups / 8 + s / NG -- every group on one XCD whatever the dispatch order.
// A workgroup past its XCD's cap waits until every workgroup has taken a slot (the sum of the counters
// reaches the grid: all are co-resident, the plan guarantees it), then takes the ov-th unfilled (group,
// member) in XCD order.  Roles never depend on results, so the arithmetic is bitwise the same.
// ctl: 10 zeroed words (8 per-XCD counters, 1 overflow counter, the release_start count); smem: 2
// words of scratch LDS.
__device__ __forceinline__ void group_pk(unsigned* ctl, int NG, int ngroups, unsigned limit, int* status, float* smem,
                                         int& group, int& w) {
  if (ctl == nullptr || (ngroups & 7) != 0) {
    group_of(blockIdx.x, NG, ngroups, group, w);
    return;
  }
  int* sg = reinterpret_cast<int*>(smem);
  if (threadIdx.x == 0) {
    const int per = ngroups >> 3, cap = per * NG, nwg = ngroups * NG;
    const unsigned x = xcc_id() & 7u;
    const int slot = (int)__hip_atomic_fetch_add(ctl + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int g = -1, m = 0;
    if (slot < cap) {
      g = (int)x * per + slot / NG;
      m = slot % NG;
    } else {
      const int ov = (int)__hip_atomic_fetch_add(ctl + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned c[8];
      unsigned spins = 0;
      while (true) {
        int tot = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          c[i] = __hip_atomic_load(ctl + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tot += (int)c[i];
        }
        if (tot >= nwg) break;
        if (++spins > limit) {
          atomicOr(status, 8);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      int k = ov;
      for (int i = 0; i < 8 && g < 0; ++i) {
        const int filled = min((int)c[i], cap), holes = cap - filled;
        if (k < holes) {
          g = i * per + (filled + k) / NG;
          m = (filled + k) % NG;
        }
        k -= holes;
      }
      if (g < 0) group_of(blockIdx.x, NG, ngroups, g, m);  // timed out (status 8): any role, results invalid
    }
    sg[0] = g;
    sg[1] = m;
  }
  __syncthreads();
  group = sg[0];
  w = sg[1];
  __syncthreads();  // the scratch words are reused by the kernel's own LDS
}

// Workspace reuse without a zero fill (round 5).  The packed kernels' hand-off granules need no
// clearing between launches of the same shape: a consumer polls slot (s-1)&1 for tag s at step s
// and a completed launch leaves tags T and T-1 behind, which only steps 1 and 2 could see before
// this launch overwrites them -- never equal for T >= 4 (tags are (step + 1) mod 2^16, T < 65535).
// The group-formation counters and the placement granules {tag 1, XCC id} are what a fill was
// for: the LAST workgroup past the start (all have formed their groups and read the placement by
// then) puts them back to zero.  ctl word 9 counts the workgroups past the start.
// place_stride: u64 between groups' granule blocks; place_off: the placement granules' offset.
__device__ __forceinline__ void release_start(unsigned* ctl, u64* xbuf, int ngroups, int NG, long long place_stride,
                                              long long place_off) {
  if (ctl == nullptr) return;
  // relaxed: this workgroup's reads of the counters and placement granules completed before the
  // startup barrier (their values were used); an acq_rel RMW would write back / invalidate the L2
  const unsigned k = __hip_atomic_fetch_add(ctl + 9, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((int)k != ngroups * NG - 1) return;
  for (int g = 0; g < ngroups; ++g)
    for (int m = 0; m < NG; ++m)
      __hip_atomic_store(xbuf + g * place_stride + place_off + m, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int i = 0; i < 10; ++i) __hip_atomic_store(ctl + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Placement check at launch start (packed kernels).  A group's hand-off granules may be
// written with PLAIN stores only when every workgroup of the group runs on one XCD: a plain
// store stays in that XCD's L2, which serves the peers' `sc1` polls (MI355X_MICROARCH.md,
// stores of each flavour); across XCDs only `sc1` write-through stores are visible.  HIP
// promises no placement (bid % 8 -> XCD is observed, not guaranteed), so every workgroup
// publishes its XCC id as one granule {tag 1, id} and the polling wave gathers the group's NG
// ids.  Every workgroup of the group reads the same NG ids and so picks the same form.
// Called by the polling wave; returns (wave-uniform) true when the granules must be written
// through.  force: 1 = write-through regardless (test hook), 0 = by placement.
__device__ __forceinline__ bool group_needs_write_through(const u64* place, int NG, int lane, unsigned limit,
                                                          int* status, int force) {
  unsigned id = 0;
  bool ok = true;
  if (lane < NG) {
    u64 v = get_granule(place + lane);
    unsigned spins = 0;
    while ((unsigned)(v >> 32) != 1u) {
      if (++spins > limit) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      v = get_granule(place + lane);
    }
    id = (unsigned)v;
  }
  if (!ok) atomicOr(status, 4);
  const unsigned id0 = __shfl(id, 0);
  const bool same = !__any(lane < NG && (id != id0 || !ok));
  return force == 1 || !same;
}

template <int CELL, int BC, int XK = 0>  // XK > 0: fused input projection over XK k-steps of 32
__global__ __launch_bounds__(NT, 1) void rnn_fwd_pk_kernel(RnnArgs a) {
  constexpr bool XW = XK > 0;
  constexpr int NGATE = CELL == CELL_LSTM ? 4 : 3;
  constexpr int KSMAX = HMAX / 32;
  constexpr int SHB = KSMAX * 32 + 8;  // bf16 row stride of the B image (k >= H stays zero)
  const int H = a.H, T = a.T, J = a.J, NG = a.NG;
  const int R = NGATE * J;
  const int MT = (R + 15) / 16;
  const int ngroups = 2 * a.nchunk;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int group, w;
  group_pk(a.gctl, NG, ngroups, a.spin_limit, a.status, smem, group, w);
  const int d = group / a.nchunk, chunk = group % a.nchunk;
  const int b0 = chunk * BC;
  const int j0 = w * J;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int GH = NGATE * H;
  const int tile = wv < WPOLL ? wv : wv - 1;
  // With 5 MFMA tiles (LSTM, J = 20) tile 4 runs as two k-step halves on the polling waves 4 and
  // 7 -- idle from B1 to B2 and on SIMDs 0 and 3 -- instead of whole on wave 5, which shares SIMD 1
  // with wave 1's tile (stamps: every wave waited ~285 cycles at B2 for it).  Wave 4 takes the
  // even k-steps, wave 7 the odd ones: exactly the two accumulator chains of a whole-tile matvec
  // (FWD_MV_CHAINS = 2), summed in the same order by the cell lanes -- bitwise the same gates.
  const bool t4h = MT == 5 && FWD_NPW == 2;
  const bool mv = wv != WPOLL && tile < MT && !(t4h && tile == 4);
  const bool mvh = t4h && (wv == WPOLL || wv == 7);
  const int SGS = MT * 16 + 4;  // sgate row stride (floats): 4 batch rows on 4 distinct bank quads

  // h B image [16][SHB]: rows 0..BC-1 are the gathered h, row BC stays zero and every MFMA lane
  // of a row >= BC reads it (one broadcast address instead of 15 - BC zero rows: the matvec's B
  // reads are conflict-free, tools/lds_banks.py)
  unsigned short* shb = reinterpret_cast<unsigned short*>(smem);
  float* sgate = smem + 8 * SHB;                                                        // [BC][SGS]
  float* sgx = sgate + BC * SGS;  // tile 4's odd-k-step chain (wave 7) [BC][16]; the even one is in sgate
  // per-step input projections [NSIN][sin_slab]: double buffered, or with XW two blocks of SPB steps
  constexpr int SPB = xw_spb(BC);
  constexpr int NSIN = XW ? 2 * SPB : 2;
  constexpr int SINS = sin_slab(BC);
  float* sin = sgx + BC * 16;
  unsigned short* spub = reinterpret_cast<unsigned short*>(sin + NSIN * SINS);   // [BC][PKU]
  // XW: the ring of 3 * SPB step slots of the layer-input rows ([BC][SXB] bf16 + the pad items of
  // the last DMA piece), 256-B aligned (the bank order of its rows)
  static_assert(!XW || FWD_NPW == 2, "the fused projection's DMA pieces assume two prefetch waves of 64 lanes");
  static_assert(16 % BC == 0, "a block fills the MFMA's 16 B-columns");
  constexpr int NXQ = xw_nxq(BC);       // DMA pieces per prefetch wave and step
  constexpr int XSL = xw_slot(BC);      // bf16 per step slot
  constexpr int NSLOT = 3 * SPB;
  // (advanced from spub by element arithmetic, not through an integer cast: the cast lost the LDS
  //  address space and every read of the ring (the projection's B fragments) compiled to a FLAT load,
  //  counted in vmcnt as well as lgkmcnt -- 120 per fused kernel, round 6)
  unsigned short* const sx0 = spub + BC * PKU;
  const unsigned sxpad = (256u - ((unsigned)reinterpret_cast<uintptr_t>(sx0) & 255u)) & 255u;
  unsigned short* sxb = sx0 + sxpad / 2;

  // ---- W_hh tile of this wave as bf16 A fragments: lane holds A[row tile*16 + (lane&15)][k]
  bf16x8 afrag[KSMAX];
  {
    const int rl = tile * 16 + (lane & 15);
    const int q = rl / J, u = rl % J;
    const bool rv = mv && rl < R && j0 + u < H;
    const float* wrow = a.Whh + ((long long)d * GH + q * H + j0 + u) * H;
#pragma unroll
    for (int ks = 0; ks < KSMAX; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = ks * 32 + 8 * (lane >> 4) + j;
        afrag[ks][j] = (short)bf16_rne((rv && k < H) ? wrow[k] : 0.0f);
      }
  }
  for (int i = tid; i < 8 * SHB; i += NT) smem[i] = 0.0f;
  for (int i = tid; i < BC * PKU; i += NT) spub[i] = 0;

  // ---- XW: the fused projection runs off the cell waves, on waves 4-7 (their slack: the free
  //      prefetch wave 6, the DMA wave 5, and the polling waves between B2 and the first
  //      granule that can land): tile 0 on wave 6, tile 1 on wave 5 (one each: their branch also
  //      holds wave 5's matvec fragments), tiles 2 + 2i on wave 4 and 3 + 2i on wave 7 (two each).
  //      Per tile, bf16 A fragments of its W_ih rows, A[row t*16 + (lane&15)][k = ks*32 +
  //      8(lane>>4) + j] (k >= Kin zero), and the b_ih of the lane's four output rows 4(lane>>4) + i;
  //      loaded inside the roles that use them (dead elsewhere: no register pressure on the cell
  //      waves).  Tile counts per role are compile-time (IC<1> / IC<2>) so unused slots stay dead.
  constexpr int XWT = 2;
  int xt[XWT];
  // second tiles on the prefetch waves, 6 first (600-wide layers 351 us per launch, first layer
  // 313 us; on the polling waves instead: 364 / 327 us, round 3)
  xt[0] = !XW ? -1 : wv == 6 ? 0 : wv == 5 ? 1 : wv == WPOLL ? 2 : wv == 7 ? 3 : -1;
  xt[1] = (XW && (wv == 6 || wv == 5) && xt[0] + 4 < MT) ? xt[0] + 4 : -1;
  if (xt[0] >= MT) xt[0] = -1;
  bf16x8 wfr[XWT][XW ? XK : 1];
  float bir[XWT][4];
  f32x4 xacc[XWT];
  auto load_w = [&](auto ntl) {
    constexpr int NTL = decltype(ntl)::value;
#pragma unroll
    for (int i = 0; i < NTL; ++i) {
      const int t = xt[i];
      const int rl = t * 16 + (lane & 15);
      const int q = rl / J, u = rl % J;
      const bool rv = t >= 0 && rl < R && j0 + u < H;
      const unsigned short* wrow = a.Wihb + ((long long)d * GH + q * H + j0 + u) * a.ldw;
      // one 16-B load per fragment (rows 16-B aligned: ldw % 8 == 0); the chunk holding k = Kin
      // element by element, chunks past it zero
#pragma unroll
      for (int ks = 0; ks < XK; ++ks) {
        const int k0 = ks * 32 + 8 * (lane >> 4);
        if (rv && k0 + 8 <= a.Kin) {
          wfr[i][ks] = *reinterpret_cast<const bf16x8*>(wrow + k0);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) wfr[i][ks][j] = (short)((rv && k0 + j < a.Kin) ? wrow[k0 + j] : 0);
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rr = t * 16 + 4 * (lane >> 4) + e;
        const int qq = rr / J, uu = rr % J;
        bir[i][e] = (t >= 0 && rr < R && j0 + uu < H) ? a.bih[(long long)d * GH + qq * H + j0 + uu] : 0.0f;
      }
      xacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  // ---- cell lanes (waves 0-3): row cb = tid / 32, unit cu = tid % 32 (< J)
  const int cb = tid >> 5, cu = tid & 31;
  const bool ct = tid < BC * 32 && cu < J;
  const int cj = j0 + cu;
  const int bg = b0 + cb;
  const bool cval = ct && cj < H && bg < a.B;
  float bh[NGATE];
#pragma unroll
  for (int q = 0; q < NGATE; ++q) bh[q] = cval ? a.bhh[(long long)d * GH + q * H + cj] : 0.0f;
  float hst = 0.0f, cst = 0.0f, hsum = 0.0f;
#ifndef FWD_STORE_WAVES
#define FWD_STORE_WAVES 0
#endif
// The forward's saved gate activations and cell states (read back only by the BPTT, after the
// rest of the forward, the loss and the Linear's backward) leave with non-temporal stores: C2
// 3.438-3.449 vs 3.452-3.472 ms per step (A/B x3 twice, profiles/r05_nt_saves_ab.txt).  Measured
// and not kept: the bf16 layer output / h_{t-1} copies non-temporal too (the next GEMMs read them
// soon: 3.496-3.508 ms), and the BPTT's bf16 dG as well (3.529-3.532 ms).  0: plain stores (A/B).
#ifndef FWD_NT_SAVES
#define FWD_NT_SAVES 1
#endif
// The bf16 h_{t-1} copy (read only by the weight-gradient launch at the end of the backward)
// non-temporal too: 3.440-3.447 vs 3.449-3.454 ms per step (A/B x3, profiles/r05_nt_saves_ab.txt)
#ifndef FWD_NT_HPREVB
#define FWD_NT_HPREVB 1
#endif
#ifndef FWD_EXP_NOXDMA
#define FWD_EXP_NOXDMA 0  // timing experiment only (results wrong): no x-row DMAs after the prologue
#endif
// The packed forward's publish gathers a granule pair's six bf16 h values by DPP wave shifts
// (round 6); 0: through an LDS stage and read-back (the round-2..5 form, A/B)
#ifndef FWD_PUB_DPP
#define FWD_PUB_DPP 1
#endif
#ifndef FWD_POLL3
#define FWD_POLL3 0  // experiment: three granule sweeps in flight in the forward's polling waves (A/B)
#endif
// The BPTT publish at batch chunks of 4: tiles 0-3's quads redistributed over the wave by DPP row shifts
// into one full-wave 16-B store (round 6: bitwise the LDS-transposed form, -35 us per C2 step,
// profiles/r06_bwd_pub_dpp_ab.txt); 0: the LDS transpose for every BC (A/B)
#ifndef BWD_PUB_DPP
#define BWD_PUB_DPP 1
#endif
#ifndef FWD_GATE_LOADS_FIRST
#define FWD_GATE_LOADS_FIRST 0  // experiment (A/B)
#endif
#ifndef FWD_POLL_SLEEP
#define FWD_POLL_SLEEP 0  // experiment: s_sleep (x 64 cycles) before a step's first granule sweep (A/B)
#endif
#ifndef BWD_POLL_SLEEP
#define BWD_POLL_SLEEP 0
#endif
  // FWD_STORE_WAVES (experiment, off): the saved-state stores of step s leave from waves 2-3
  // (matvec-only, idle after B2) during step s+1 instead of from the cell lanes after their publish:
  // the cell lanes stage {act, c, h_{t-1}, h} in LDS (double buffered by step parity), the last step
  // stores directly.  Measured round 5 (A/B x3, gpurun_out/r05sw): 3.522 vs 3.466 ms per step, ~14 us
  // SLOWER per forward launch -- the stores issued right behind the publish pace the polling sweeps
  // (the round-4 observation); moved off the cell lanes they no longer do.
  constexpr bool SW = FWD_STORE_WAVES && BC * 32 <= 128;
  __shared__ float4 s_sta[SW ? 2 * BC * 20 : 1];   // act (4 gates) per cell
  __shared__ float4 s_stb[SW ? 2 * BC * 20 : 1];   // {c, h_{t-1}, h, -} per cell

  // granules of this group: [2 slots][hand-off, spare][BC][NG][8] x 8 B; the spare copy of
  // slot 1 holds the placement granules
  const int slot_g = BC * NG * 8;
  u64* xg = a.xbuf + (long long)group * 4 * slot_g;
  const __amdgpu_buffer_rsrc_t xr = granule_rsrc(xg, (unsigned)(4 * slot_g * 8));
  __shared__ int s_wt;
  if (tid == 0) __hip_atomic_store(xg + 3 * slot_g + w, (1ull << 32) | xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (wv == WPOLL) {
    const bool wt = group_needs_write_through(xg + 3 * slot_g, NG, lane, a.spin_limit, a.status, a.place_force);
    if (lane == 0) s_wt = wt;
  }

  // ---- prefetch waves 5-7 (5-6 with FWD_NPW = 2: wave 7 polls too): input projection
  //      G[b][t][d][q*H + j] of every own (b, unit, gate)
  constexpr int NPF = NT - (WPOLL + FWD_NPW) * 64;  // 192 / 128 prefetch lanes
  const bool pollw = wv == WPOLL || (FWD_NPW >= 2 && wv == 7) || (FWD_NPW == 3 && wv == 6);
  const bool pfw = wv > WPOLL && !pollw;
  constexpr int NQ = (BC * 20 * 4 + NPF - 1) / NPF;
  StepLoader<NQ> ld;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    // item = cell * 4 + gate: consecutive lanes commit consecutive LDS words (conflict-free
    // ds_write_b32; gate-major items were 16 B apart, a 4-way conflict)
    const int i = tid - (WPOLL + 1) * 64 + q * NPF;
    const int gate = i & 3, cell = i >> 2;
    const int ib = b0 + cell / J, iu = cell % J, ij = j0 + iu;
    const bool on = pfw && gate < NGATE && cell < BC * J;
    ld.p[q] = (on && ib < a.B && ij < H) ? a.G + ((long long)ib * T * 2 + d) * GH + gate * H + ij : nullptr;
    ld.stride[q] = 2 * GH;
    ld.shift[q] = 0;
    ld.dst[q] = on ? cell * 4 + gate : -1;
  }
  // XW: per-lane sources of this prefetch wave's DMA pieces (item i = q*128 + (wave-5)*64 + lane)
  const unsigned short* xsrc[NXQ];
  if constexpr (XW) {
#pragma unroll
    for (int q = 0; q < NXQ; ++q) {
      const int i = q * 128 + (wv - WPOLL - 1) * 64 + lane;
      const int b = i / SXC, c = i % SXC;  // chunks c >= 80 of a row are its pad
      const bool on = pfw && b < BC && c < XKMAX * 4 && 8 * c < a.Kin && b0 + b < a.B;
      xsrc[q] = on ? a.Xb + (long long)(b0 + b) * T * a.ldx + 8 * c : nullptr;
    }
  }
  // DMA of step u's rows into ring slot u % NSLOT (prefetch waves only)
  auto xdma = [&](int u) {
    const long long toff = (long long)(d == 0 ? u : T - 1 - u) * a.ldx;
    unsigned short* dst = sxb + (u % NSLOT) * XSL + (wv - WPOLL - 1) * 64 * 8;
#pragma unroll
    for (int q = 0; q < NXQ; ++q) {
      const void* src = xsrc[q] ? (const void*)(xsrc[q] + toff) : (const void*)g_xzero_line;
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(dst + q * 128 * 8), 16, 0, 0);
    }
  };
  // wait until at most `n` steps' pieces (the latest issued) are still in flight (n <= SPB)
  auto xwait = [&](int n) {
    static_assert(!XW || (SPB + FWD_XDMA_EARLY) * NXQ <= 63, "vmcnt range");
#define XW_WAIT(k) \
  case k:          \
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((k) * NXQ <= 63 ? (k) * NXQ : 63) : "memory"); break;
    switch (n) {
      XW_WAIT(0) XW_WAIT(1) XW_WAIT(2) XW_WAIT(3) XW_WAIT(4) XW_WAIT(5) XW_WAIT(6) XW_WAIT(7) XW_WAIT(8)
      XW_WAIT(9) XW_WAIT(10) XW_WAIT(11) XW_WAIT(12) XW_WAIT(13) XW_WAIT(14) XW_WAIT(15)
      default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(16 * NXQ <= 63 ? 16 * NXQ : 63) : "memory");
    }
#undef XW_WAIT
  };
  if (XW && pfw) {
    // blocks 0-2 in flight; blocks 0 and 1 must land before the first barrier (block 0's chain
    // runs before the loop, block 1's first part at step 0)
    for (int u = 0; u < min(T, NSLOT); ++u) xdma(u);
    xwait(max(0, min(T, NSLOT) - 2 * SPB));
  } else if (!XW && pfw) {
    ld.issue(d == 0 ? 0 : T - 1, T);
  }
  __syncthreads();
  const bool wt = __builtin_amdgcn_readfirstlane(s_wt) != 0;  // granules written through (group spans XCDs)
  if (tid == 0) release_start(a.gctl, a.xbuf, ngroups, NG, 4LL * slot_g, 3LL * slot_g);
  STAMP_DECL

  // XW: G of block kb (steps kb*SPB .. +SPB-1) for this wave's tiles' rows: x W_ih^T as one
  // accumulator chain over the k-steps in order, then + b_ih (the separate GEMM's arithmetic:
  // gemm_gl's k-loop and bias epilogue, bitwise).  xpart runs part j of it, the k-steps
  // [j PK, (j+1) PK) (the B fragments, shared by the wave's tiles, read once; every index
  // compile-time through the unrolled part switch); xfinal adds b_ih and writes the block's G to
  // sin.  B column n = o * BC + b: step kb*SPB + o, batch row b.
  constexpr int PK = XW ? (XK + SPB - 1) / SPB : 1;
  auto xpart = [&](auto ntl, int kb, int j) {
    constexpr int NTL = decltype(ntl)::value;
    if (xt[0] < 0) return;
    const int n = lane & 15;
    const unsigned short* bp = sxb + ((kb % 3) * SPB + n / BC) * XSL + (n % BC) * SXB + 8 * (lane >> 4);
#pragma unroll
    for (int jj = 0; jj < SPB; ++jj) {
      if (jj != j || jj * PK >= XK) continue;
      bf16x8 bv[PK];
#pragma unroll
      for (int i = 0; i < PK; ++i)
        if (jj * PK + i < XK) bv[i] = *reinterpret_cast<const bf16x8*>(bp + (jj * PK + i) * 32);
#pragma unroll
      for (int i = 0; i < PK; ++i)
        if (jj * PK + i < XK) {
#pragma unroll
          for (int t = 0; t < NTL; ++t)
            if (xt[t] >= 0)
              xacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[t][jj * PK + i], bv[i], xacc[t], 0, 0, 0);
        }
    }
  };
  auto xfinal = [&](auto ntl, int kb) {
    constexpr int NTL = decltype(ntl)::value;
    const int n = lane & 15, o = n / BC, b = n % BC;
    float* dst = sin + ((kb & 1) * SPB + o) * SINS;
#pragma unroll
    for (int i = 0; i < NTL; ++i) {
      if (xt[i] < 0) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rr = xt[i] * 16 + 4 * (lane >> 4) + e;
        if (rr < R) dst[(b * J + rr % J) * 4 + rr / J] = xacc[i][e] + bir[i][e];
      }
      xacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // this step's part of block kb + 1's chain (steps of block kb = s / SPB); the last part finishes it
  auto xstep = [&](auto ntl, int s) {
    const int kb = s / SPB + 1, j = s % SPB;
    if (kb * SPB >= T) return;
    xpart(ntl, kb, j);
    if (j == SPB - 1 || s == T - 1) xfinal(ntl, kb);
  };
  // a role's start: its W_ih fragments, then block 0 whole (its rows landed before the barrier)
  auto xstart = [&](auto ntl) {
    load_w(ntl);
    for (int j = 0; j < SPB; ++j) xpart(ntl, 0, j);
    xfinal(ntl, 0);
  };
  // compile-time tile slots of the prefetch-wave and polling-wave roles
  using XPF = std::integral_constant<int, 2>;
  using XPL = std::integral_constant<int, 1>;

  // tile 4's half on a polling wave: the even (wave 4, into sgate's tile-4 columns) or odd (wave 7,
  // into sgx) k-steps as one accumulator chain in k order; afh[i] holds k-step 2i + (wave 7), loaded
  // inside the polling role (dead in every other role)
  constexpr int KH = (KSMAX + 1) / 2;
  auto load_half = [&](bf16x8* afh) __attribute__((always_inline)) {
    const int rl = 4 * 16 + (lane & 15);
    const int q = rl / J, u = rl % J;
    const bool rv = mvh && rl < R && j0 + u < H;
    const int kpar = wv == 7 ? 1 : 0;
    const float* wrow = a.Whh + ((long long)d * GH + q * H + j0 + u) * H;
#pragma unroll
    for (int i = 0; i < KH; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = 2 * i + kpar;
        const int k = kk * 32 + 8 * (lane >> 4) + j;
        afh[i][j] = (short)bf16_rne((rv && kk < KSMAX && k < H) ? wrow[k] : 0.0f);
      }
  };
  auto matvec_half = [&](const bf16x8* afh) __attribute__((always_inline)) {
    const int kpar = wv == 7 ? 1 : 0;
    const unsigned short* bp = shb + min(lane & 15, BC) * SHB + 8 * (lane >> 4) + kpar * 32;
    bf16x8 bv[KH];
#pragma unroll
    for (int i = 0; i < KH; ++i)
      if (2 * i + kpar < KSMAX) bv[i] = *reinterpret_cast<const bf16x8*>(bp + i * 64);
    __builtin_amdgcn_sched_barrier(0);  // every B read before the first MFMA (one LDS round trip)
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < KH; ++i)
      if (2 * i + kpar < KSMAX) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afh[i], bv[i], acc, 0, 0, 0);
    const int col = lane & 15;
    if (col < BC) {
      float* dst = wv == 7 ? sgx + col * 16 : sgate + col * SGS + 4 * 16;
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[(lane >> 4) * 4 + i] = acc[i];
    }
  };
  // sgate[b][tile*16 + row] = sum_k W[row][k] h[b][k]
  auto matvec = [&]() __attribute__((always_inline)) {
    if (!mv) return;
    const unsigned short* bp = shb + min(lane & 15, BC) * SHB + 8 * (lane >> 4);
    bf16x8 bv[KSMAX];
#pragma unroll
    for (int ks = 0; ks < KSMAX; ++ks) bv[ks] = *reinterpret_cast<const bf16x8*>(bp + ks * 32);
    // every B read issued before the first MFMA: one LDS round trip instead of one per pair
    // (the scheduler otherwise interleaves reads and waits to save registers)
    __builtin_amdgcn_sched_barrier(0);
    // FWD_MV_CHAINS independent accumulator chains over the k-steps (the chain length is
    // the matvec's latency), summed in fixed order
    f32x4 acc[FWD_MV_CHAINS];
#pragma unroll
    for (int c = 0; c < FWD_MV_CHAINS; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KSMAX; ++ks)
      acc[ks % FWD_MV_CHAINS] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afrag[ks], bv[ks], acc[ks % FWD_MV_CHAINS], 0, 0, 0);
#pragma unroll
    for (int c = 1; c < FWD_MV_CHAINS; ++c) acc[0] += acc[c];
    const int col = lane & 15;
    if (col < BC) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sgate[col * SGS + tile * 16 + (lane >> 4) * 4 + i] = acc[0][i];
    }
  };

  if (pollw) {
    if (XW) xstart(XPL{});
    bf16x8 afh[KH];
    load_half(afh);
    // ---- polling wave(s): 16-B unit idx = (b * NG + producer) * 4 + pair; lane holds
    //      units lane + 64 (g FWD_NPW + pwv) (idle lanes re-read unit 0: every load is
    //      unconditional, so the compiler can keep a sweep in flight behind a counted vmcnt)
    constexpr int GLK = (BC + FWD_NPW - 1) / FWD_NPW;  // BC * NG * 4 <= 64 * BC  (NG <= 16, checked by the plan)
    const int pwv = wv == WPOLL ? 0 : wv == 7 ? 1 : 2;
    const int n16 = BC * NG * 4;
    int loff[GLK], doff[GLK], dlim[GLK];
#pragma unroll
    for (int g = 0; g < GLK; ++g) {
      const int idx = lane + 64 * (g * FWD_NPW + pwv);
      const bool on = idx < n16;
      const int b = idx / (NG * 4), pw = (idx / 4) % NG, pp = idx % 4;
      const int k0 = pw * J + 6 * pp;
      loff[g] = on ? idx * 16 : 0;
      doff[g] = on ? b * SHB + k0 : 0;
      dlim[g] = on ? max(0, min(min(6, J - 6 * pp), H - k0)) : 0;
    }
    for (int s = 0; s < T; ++s) {
      if (s > 0) {
        const unsigned tag = (unsigned)s & 0xFFFFu;
        const int base = ((s - 1) & 1) * 2 * slot_g * 8;  // the slot's hand-off copy (bytes)
        TRACE(2, s);
        // two sweeps in flight: the older one is merged while the newer one travels;
        // a pair is taken from the first sweep that shows both its tags.  One 16-B `sc1`
        // buffer load per granule pair; the empty asm with a memory clobber before each
        // sweep keeps the loads inside the spin loop (the round-1 8-B relaxed agent atomics were
        // 13-16 % slower per step: DESIGN.md section 5).
        u32x4 v[GLK], qa[GLK], qb[GLK];
        unsigned done = 0;
#if FWD_POLL_SLEEP
        // (experiment) the first sweep of the step held back while this CU's own cell phase and publish
        // run: no granule can land before the own publish, and the sweeps sit in the CU's memory queue
        __builtin_amdgcn_s_sleep(FWD_POLL_SLEEP);
#endif
#if FWD_POLL3
        // (experiment) three sweeps in flight: each merge samples a third of a round trip after the last
        u32x4 qc[GLK];
        auto fmerge = [&](const u32x4* q) __attribute__((always_inline)) {
#pragma unroll
          for (int g = 0; g < GLK; ++g) {
            const bool m = ((q[g].y >> 16) == tag) & ((q[g].w >> 16) == tag) & !((done >> g) & 1);
            v[g] = m ? q[g] : v[g];
            done |= (unsigned)m << g;
          }
        };
        asm volatile("" ::: "memory");
#pragma unroll
        for (int g = 0; g < GLK; ++g) qa[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + loff[g], 0, 16);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int g = 0; g < GLK; ++g) qb[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + loff[g], 0, 16);
        unsigned spins = 0;
        while (true) {
          asm volatile("" ::: "memory");
#pragma unroll
          for (int g = 0; g < GLK; ++g) qc[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + loff[g], 0, 16);
          fmerge(qa);
          if (done == (1u << GLK) - 1) break;
          asm volatile("" ::: "memory");
#pragma unroll
          for (int g = 0; g < GLK; ++g) qa[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + loff[g], 0, 16);
          fmerge(qb);
          if (done == (1u << GLK) - 1) break;
          asm volatile("" ::: "memory");
#pragma unroll
          for (int g = 0; g < GLK; ++g) qb[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + loff[g], 0, 16);
          fmerge(qc);
          if (done == (1u << GLK) - 1) break;
          if (++spins > a.spin_limit) {
            atomicOr(a.status, 1);
            return;
          }
        }
#else
        asm volatile("" ::: "memory");
#pragma unroll
        for (int g = 0; g < GLK; ++g) qa[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + loff[g], 0, 16);
        unsigned spins = 0;
        while (true) {
          asm volatile("" ::: "memory");
#pragma unroll
          for (int g = 0; g < GLK; ++g) qb[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + loff[g], 0, 16);
#pragma unroll
          for (int g = 0; g < GLK; ++g) {
            const bool m = ((qa[g].y >> 16) == tag) & ((qa[g].w >> 16) == tag) & !((done >> g) & 1);
            v[g] = m ? qa[g] : v[g];
            done |= (unsigned)m << g;
          }
          if (done == (1u << GLK) - 1) break;
#ifdef RNN_TRACE
          if (spins == 0) TRACE(3, s);
#endif
          asm volatile("" ::: "memory");
#pragma unroll
          for (int g = 0; g < GLK; ++g) qa[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + loff[g], 0, 16);
#pragma unroll
          for (int g = 0; g < GLK; ++g) {
            const bool m = ((qb[g].y >> 16) == tag) & ((qb[g].w >> 16) == tag) & !((done >> g) & 1);
            v[g] = m ? qb[g] : v[g];
            done |= (unsigned)m << g;
          }
          if (done == (1u << GLK) - 1) break;
          if (++spins > a.spin_limit) {
            atomicOr(a.status, 1);
            return;
          }
        }
#endif
#pragma unroll
        for (int g = 0; g < GLK; ++g) {
          const u32x4 x = v[g];
          unsigned* dst = reinterpret_cast<unsigned*>(shb + doff[g]);  // 4-B aligned: J, H, SHB even
          const int nv = dlim[g];
          if (nv > 0) dst[0] = x.x;
          if (nv > 2) dst[1] = (x.y & 0xFFFFu) | (x.z << 16);
          if (nv > 4) dst[2] = (x.z >> 16) | (x.w << 16);
        }
        TRACE(1, s);
      }
      STAMP(0)
      __syncthreads();  // B1
      STAMP(1)
      if (mvh) matvec_half(afh);
      STAMP(2)
      __syncthreads();  // B2
      STAMP(3)
      // XW: this step's part of the next block's projection, before the next gather: no granule of
      // step s+1 can land before the cell phase and publish that follow B2
      if (XW) xstep(XPL{}, s);
    }
    STAMP_FLUSH
    return;
  }
  if (pfw) {
    // Prefetch waves 5-6.  A wave's role is a compile-time pair (its fused-projection tile slots,
    // whether it holds a matvec tile), so no branch keeps the other role's fragments live: wave 6
    // (two projection tiles at H = 300 LSTM, no matvec) and wave 5 (one projection tile + matvec
    // tile 4) -- one shared body for both kept 2 x XK W_ih fragments and the matvec's W_hh / h
    // fragments live together and spilled 45 VGPRs at XK = 20.
    auto pf_loop = [&](auto ntl, auto with_mv) __attribute__((always_inline)) {
      constexpr bool MV = decltype(with_mv)::value;
      if (XW) xstart(ntl);
      for (int s = 0; s < T; ++s) {
        if (!XW) {
          ld.commit(sin + (s & 1) * SINS);
          if (s + 1 < T) ld.issue(d == 0 ? s + 1 : T - 2 - s, T);
        }
        STAMP(0)
        __syncthreads();  // B1
        STAMP(1)
#if FWD_XDMA_EARLY
        // step s + 3 SPB's rows into slot s % NSLOT, issued right after B1: that slot held step s's
        // rows, last read by the chain of block s / SPB, which ended before B1(s).  Here, not after B2,
        // the pieces travel during the matvec and the gate phase instead of sitting in the CU's memory
        // queue beside the next hand-off's polls (the BPTT's BWD_PF_LATE argument)
        if (XW && s + NSLOT < T) xdma(s + NSLOT);
#endif
        if constexpr (MV) matvec();
        // XW: at a block start the rows of the next block (consumed from this step on) landed
        // before B2; the block after it may stay in flight (and, issued early, this step's too)
        if (XW && s % SPB == 0) xwait(max(0, min(SPB + FWD_XDMA_EARLY, T - (s / SPB + 2) * SPB)));
        STAMP(2)
        __syncthreads();  // B2
        STAMP(3)
        if (XW) xstep(ntl, s);
#if !FWD_XDMA_EARLY
        // step s + 3 SPB's rows into slot s % NSLOT, issued after B2 (off the matvec -> B2 path); that
        // slot held step s's rows, last read by the chain of block s / SPB, which ended before B1(s)
        if (XW && !FWD_EXP_NOXDMA && s + NSLOT < T) xdma(s + NSLOT);
#endif
        STAMP(4)
      }
    };
    // (fused projection: wave 6 holds no matvec tile and wave 5 one projection tile --
    // dl4ss_birnn_fwd_xw_supported admits at most 5 MFMA tiles; without it the slot count is moot)
    using XP1 = std::integral_constant<int, 1>;
    if (wv == 6 && !mv)
      pf_loop(XPF{}, std::false_type{});
    else
      pf_loop(XP1{}, std::true_type{});
    STAMP_FLUSH
    return;
  }
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    STAMP(0)
    __syncthreads();  // B1
    STAMP(1)
    matvec();
    STAMP(2)
    __syncthreads();  // B2
    STAMP(3)
    if constexpr (SW) {
      // waves 2-3: step s-1's saved state (staged before B1(s); its slot is rewritten only after B2(s+1))
      const int i = tid - BC * 32;
      if (s > 0 && i >= 0 && i < BC * J) {
        const int sb = (s - 1) & 1, ib = b0 + i / J, ij = j0 + i % J;
        if (ij < H && ib < a.B) {
          const int tp = d == 0 ? s - 1 : T - s;
          const long long bt = (long long)ib * T + tp;
          const float4 ac = s_sta[sb * BC * 20 + i], cb4 = s_stb[sb * BC * 20 + i];
          if (a.act_cm) {
            *reinterpret_cast<float4*>(a.act + ((bt * 2 + d) * H + ij) * 4) = ac;
          } else {
            float* actp = a.act + (bt * 2 + d) * (4 * H) + ij;
            actp[0] = ac.x; actp[H] = ac.y; actp[2 * H] = ac.z; actp[3 * H] = ac.w;
          }
          if constexpr (CELL == CELL_LSTM) a.cs[(bt * 2 + d) * H + ij] = cb4.x;
          const long long ho = bt * 2 * H + d * H + ij;
          if (a.hprev) a.hprev[ho] = cb4.y;
          if (a.out) a.out[ho] = cb4.z;
          const int hp8 = (H + 7) & ~7, op8 = (2 * H + 7) & ~7;
          if (a.outb) a.outb[bt * op8 + d * H + ij] = bf16_rne(cb4.z);
          if (a.hprevb) a.hprevb[bt * 2 * hp8 + d * hp8 + ij] = bf16_rne(cb4.y);
        }
      }
    }
    if (tid < BC * 32) {
      float hn = 0.0f, st[4] = {0.f, 0.f, 0.f, 0.f};
      if (cval) {
        float hg[NGATE], gx[NGATE];
        const int sb = XW ? ((s / SPB) & 1) * SPB + s % SPB : (s & 1);
        const float4 g4 = *reinterpret_cast<const float4*>(sin + sb * SINS + (cb * J + cu) * 4);  // one 16-B read
        const float gxa[4] = {g4.x, g4.y, g4.z, g4.w};
        // tile 4 (rows 64..79: with J = 20 only gate 3's units 4..19): even chain + odd chain, as the
        // whole-tile matvec's acc[0] + acc[1]; read unconditionally (a clamped address) and selected
        const int r3 = (NGATE - 1) * J + cu;
        const float x4 = sgx[cb * 16 + max(r3 - 64, 0)];
        float mqs[NGATE];
#pragma unroll
        for (int q = 0; q < NGATE; ++q) mqs[q] = sgate[cb * SGS + q * J + cu];
#if FWD_GATE_LOADS_FIRST
        // every gate read issued before the first is used (hipcc placed the last gate's read after the
        // first wait: a second LDS round trip on the output gate's chain)
        __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
        for (int q = 0; q < NGATE; ++q) {
          float mq = mqs[q];
          if (q == NGATE - 1) mq = (t4h && r3 >= 64) ? mq + x4 : mq;
          hg[q] = bh[q] + mq;
          gx[q] = gxa[q];
        }
        if constexpr (CELL == CELL_LSTM) {
          const float ig = fsig(gx[0] + hg[0]);
          const float fg = fsig(gx[1] + hg[1]);
          const float gg = ftanh(gx[2] + hg[2]);
          const float og = fsig(gx[3] + hg[3]);
          cst = fg * cst + ig * gg;
          hn = og * ftanh(cst);
          st[0] = ig; st[1] = fg; st[2] = gg; st[3] = og;
        } else {
          const float rg = fsig(gx[0] + hg[0]);
          const float zg = fsig(gx[1] + hg[1]);
          const float ng = ftanh(gx[2] + rg * hg[2]);
          hn = (1.0f - zg) * ng + zg * hst;
          st[0] = rg; st[1] = zg; st[2] = ng; st[3] = hg[2];
        }
      }
      STAMP(5)
#if FWD_PUB_DPP
      // publish: lane cu = 6 k (k < 4) of each row packs the bf16 h of units cu .. cu + 5 (units >=
      // J and padded rows are zeros) into two tagged granules and stores them with one 16-B
      // write-through store.  The neighbours' values arrive by five DPP wave shifts (lane i reads
      // lane i + 1), not through an LDS stage and read-back (round 6: the LDS round trip sat on
      // every step's critical path)
      {
        const int v0 = ct ? (int)bf16_rne(hn) : 0;
        const int v1 = __builtin_amdgcn_mov_dpp(v0, 0x130, 0xF, 0xF, true);  // wave_shl:1
        const int v2 = __builtin_amdgcn_mov_dpp(v1, 0x130, 0xF, 0xF, true);
        const int v3 = __builtin_amdgcn_mov_dpp(v2, 0x130, 0xF, 0xF, true);
        const int v4 = __builtin_amdgcn_mov_dpp(v3, 0x130, 0xF, 0xF, true);
        const int v5 = __builtin_amdgcn_mov_dpp(v4, 0x130, 0xF, 0xF, true);
        const int k6 = cu / 6;
        if (cu == 6 * k6 && k6 < 4) {
          const unsigned tag = (unsigned)(s + 1) & 0xFFFFu;
          const u32x4 x = {(unsigned)v0 | ((unsigned)v1 << 16), (unsigned)v2 | (tag << 16),
                           (unsigned)v3 | ((unsigned)v4 << 16), (unsigned)v5 | (tag << 16)};
          const int off = ((s & 1) * 2 * slot_g + (cb * NG + w) * 8 + 2 * k6) * 8;
          if (wt)
            __builtin_amdgcn_raw_buffer_store_b128(x, xr, off, 0, 16);  // sc1 write-through (group spans XCDs)
          else
            __builtin_amdgcn_raw_buffer_store_b128(x, xr, off, 0, 0);   // plain: stays in the group's L2
        }
      }
#else
      // stage bf16 h (padded rows / units >= H stage zeros) and publish: lanes 0-3 of
      // each row read 6 staged values (LDS is in order within the wave) and store two
      // tagged granules with one 16-B write-through store
      if (ct) spub[cb * PKU + cu] = bf16_rne(hn);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (cu < 4) {
        const unsigned* sp = reinterpret_cast<const unsigned*>(spub + cb * PKU + 6 * cu);
        const unsigned w01 = sp[0], w23 = sp[1], w45 = sp[2];
        const unsigned tag = (unsigned)(s + 1) & 0xFFFFu;
        const u32x4 x = {w01, (w23 & 0xFFFFu) | (tag << 16), (w23 >> 16) | (w45 << 16), (w45 >> 16) | (tag << 16)};
        const int off = ((s & 1) * 2 * slot_g + (cb * NG + w) * 8 + 2 * cu) * 8;
        if (wt)
          __builtin_amdgcn_raw_buffer_store_b128(x, xr, off, 0, 16);  // sc1 write-through (group spans XCDs)
        else
          __builtin_amdgcn_raw_buffer_store_b128(x, xr, off, 0, 0);   // plain: stays in the group's L2
      }
#endif
      STAMP(6)
      if (tid == 0) TRACE(0, s);
#ifndef FWD_EXP_SKIP
#define FWD_EXP_SKIP 0  // timing experiments only (results wrong): skip saved-state stores, bits 1 act, 2 cs, 4 out, 8 outb, 16 hprevb, 32 hprev
#endif
      if (SW && cval && s < T - 1) {  // staged: waves 2-3 store it during step s+1
        const int sb = (s & 1) * BC * 20 + cb * J + cu;
        s_sta[sb] = make_float4(st[0], st[1], st[2], st[3]);
        s_stb[sb] = make_float4(cst, hst, hn, 0.0f);
        hsum += hn;
      } else if (cval) {
        const long long bt = (long long)bg * T + t;
        if (FWD_EXP_SKIP & 1) {
        } else if (a.act_cm) {
#if FWD_NT_SAVES
          typedef float nt_f4 __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(nt_f4{st[0], st[1], st[2], st[3]},
                                      reinterpret_cast<nt_f4*>(a.act + ((bt * 2 + d) * H + cj) * 4));
#else
          *reinterpret_cast<float4*>(a.act + ((bt * 2 + d) * H + cj) * 4) = make_float4(st[0], st[1], st[2], st[3]);
#endif
        } else {
          float* actp = a.act + (bt * 2 + d) * (4 * H) + cj;
          actp[0] = st[0]; actp[H] = st[1]; actp[2 * H] = st[2]; actp[3 * H] = st[3];
        }
#if FWD_NT_SAVES
        if constexpr (CELL == CELL_LSTM) __builtin_nontemporal_store(cst, a.cs + (bt * 2 + d) * H + cj);
#else
        if constexpr (CELL == CELL_LSTM) if (!(FWD_EXP_SKIP & 2)) a.cs[(bt * 2 + d) * H + cj] = cst;
#endif
        const long long ho = bt * 2 * H + d * H + cj;
        if (a.hprev && !(FWD_EXP_SKIP & 32)) a.hprev[ho] = hst;
        if (a.out && !(FWD_EXP_SKIP & 4)) a.out[ho] = hn;
        hsum += hn;
        // bf16 copies, 16-B aligned rows for the GEMMs: out_bf16 (B*T, pad8(2H)) with the
        // directions adjacent (the next layer's K), hprev_bf16 (B*T, 2 pad8(H)) with each
        // direction's block 16-B aligned (the per-direction dW_hh operand)
        const int hp8 = (H + 7) & ~7, op8 = (2 * H + 7) & ~7;
        if (a.outb && !(FWD_EXP_SKIP & 8)) a.outb[bt * op8 + d * H + cj] = bf16_rne(hn);
#if FWD_NT_HPREVB
        if (a.hprevb) __builtin_nontemporal_store((unsigned short)bf16_rne(hst), a.hprevb + bt * 2 * hp8 + d * hp8 + cj);
#else
        if (a.hprevb && !(FWD_EXP_SKIP & 16)) a.hprevb[bt * 2 * hp8 + d * hp8 + cj] = bf16_rne(hst);
#endif
      }
      hst = hn;
    }
    STAMP(4)
  }
  // the layer output's mean over t (the ADDJUST / classifier time mean, EvalVer.py:363-377): each cell
  // lane's own sum in step order -- no separate pass over the (B, T, 2H) output
  if (a.hmean && cval) a.hmean[(long long)bg * 2 * H + d * H + cj] = hsum / (float)T;
  STAMP_FLUSH
}

// --------------------------------------------------------------------------
// BPTT.  Step s walks time backwards for the forward direction (t = T-1-s) and
// forwards for the reverse direction.  Thread (b,u) owns dh/dc of its unit;
// the recurrent term dh_rec[b][j] = sum_{rows r} dgh[b][r] W_hh[r][j] is formed
// as per-workgroup partial sums over the workgroup's own rows (registers hold
// W[rows of w][k-group]) published for all j; each consumer gathers the NG
// partials of its own units (waves 4-7) and sums them in fixed order.
// --------------------------------------------------------------------------
//
// MF = true (bf16 MFMA mode): waves 0-3 hold W_hh^T of the workgroup's rows as bf16
// A fragments (output unit k on the MFMA row, gate row r on its K), dgh is staged
// in LDS as the bf16 B image [batch][r]; each 16-unit tile's D lanes publish their
// granules directly -- no partial-sum buffer, no third barrier.
template <int CELL, int BC, int RPL_T, int KGL_T, bool MF>
__global__ __launch_bounds__(NT, 1) void rnn_bwd_kernel(RnnArgs a) {
  constexpr int NGATE = CELL == CELL_LSTM ? 4 : 3;
  constexpr int RPLN = MF ? 1 : (RPL_T > 0 ? RPL_T : RPLMAX);  // rows per thread (compile-time)
  constexpr int KGLN = MF ? 1 : (KGL_T > 0 ? KGL_T : KGLMAX);  // k per thread (compile-time)
  constexpr int MTWMAX = (HMAX / 16 + 3) / 4;                    // MFMA unit tiles per wave
  constexpr int KSRMAX = (4 * 20 + 31) / 32;                     // MFMA K-steps over gate rows
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
  const int RPAD = a.RP * RPLN;  // padded row count (rows >= R stay zero)
  const int KW = a.KG * KGLN;

  const int lane = tid & 63, wv = tid >> 6;
  constexpr int SDG = KSRMAX * 32 + 8;  // bf16 row stride of the MFMA B image (rows >= R stay zero)
  constexpr int WSPAN = MTWMAX * 16;     // output units per MFMA wave (contiguous)

  extern __shared__ __attribute__((aligned(16))) float smem[];
  // fp32 path: sdg [BC][RPAD] dgh of this workgroup's rows, then sdh, spart [RP][BC][KW]
  // MFMA path: sdgb bf16 [16][SDG], then sdh
  float* sdg = smem;
  unsigned short* sdgb = reinterpret_cast<unsigned short*>(smem);
  float* sdh = MF ? smem + 8 * SDG : sdg + BC * RPAD;  // [NG][BC][J] gathered partials
  float* spart = sdh + ((NG * BC * J + 3) & ~3);        // fp32: [RP][BC][KW]; MFMA: [4 waves][BC][WSPAN]
  float* sop = spart + (MF ? 4 * BC * WSPAN : a.RP * BC * KW);  // [2][BC*J][8] per-step operands
  for (int i = tid; i < (MF ? 8 * SDG : BC * RPAD) + NG * BC * J; i += NT) smem[i] = 0.0f;

  // fp32: thread (kg, rp): rows [rp*RPLN, +RPLN), k in [kg*KGLN, +KGLN)
  const int kg = tid % a.KG, rp = tid / a.KG;
  const bool mv = MF ? wv < 4 : rp < a.RP;
  float wreg[RPLN][KGLN];
  bf16x8 afr[MF ? MTWMAX : 1][MF ? KSRMAX : 1];
  if constexpr (!MF) {
#pragma unroll
    for (int i = 0; i < RPLN; ++i) {
      const int rr = rp * RPLN + i;
      const int q = rr / J, u = rr % J;
      const bool rv = mv && rr < R && j0 + u < H;
      const float* wrow = a.Whh + ((long long)d * GH + q * H + j0 + u) * H;
#pragma unroll
      for (int c = 0; c < KGLN; ++c) {
        const int k = kg * KGLN + c;
        wreg[i][c] = (rv && k < H) ? wrow[k] : 0.0f;
      }
    }
  } else {  // tile m = wv*MTWMAX + t: lane holds A[k = m*16 + (lane&15)][r = ks*32 + 8(lane>>4) + j] = W[row(r)][k]
#pragma unroll
    for (int t = 0; t < MTWMAX; ++t) {
      const int k = (wv * MTWMAX + t) * 16 + (lane & 15);
#pragma unroll
      for (int ks = 0; ks < KSRMAX; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int rr = ks * 32 + 8 * (lane >> 4) + j;
          const int q = rr / J, u = rr % J;
          const bool ok = mv && k < H && rr < R && j0 + u < H;
          afr[t][ks][j] = (short)bf16_rne(ok ? a.Whh[((long long)d * GH + q * H + j0 + u) * H + k] : 0.0f);
        }
    }
  }
  // gather role: offsets of the NG partials of every own (b, unit), fixed per launch
  constexpr int GM = (BC * (HMAX + 20) + NROLE - 1) / NROLE;
  int goff[GM];
#pragma unroll
  for (int g = 0; g < GM; ++g) {
    const int i = tid - NROLE + g * NROLE;
    goff[g] = -1;
    if (tid >= NROLE && i < NG * BC * J) {
      const int p = i / (BC * J), rem = i % (BC * J), bb = rem / J, u = rem % J;
      if (j0 + u < H) goff[g] = p * BC * H + bb * H + j0 + u;
    }
  }
  // publish role: (b, k) of every granule this thread writes, fixed per launch
  constexpr int GP = (BC * HMAX + NROLE - 1) / NROLE;
  int psrc[GP];
#pragma unroll
  for (int g = 0; g < GP; ++g) {
    const int i = tid + g * NROLE;
    psrc[g] = (!MF && tid < NROLE && i < BC * H) ? (i / H) * KW + i % H : -1;
  }

  const bool ct = tid < BC * J;
  const int cb = tid / J, cu = tid % J;
  const int cj = j0 + cu;
  const int bg = b0 + cb;
  const bool cval = ct && cj < H && bg < a.B;
  float dc_next = 0.0f;  // LSTM dc carried to the earlier step
  float dh_dir = 0.0f;   // GRU direct dh term carried to the earlier step

  u64* xg = a.xbuf + (long long)group * 2 * NG * BC * H;
  // d(mean_t h) broadcast term: constant over t, loaded once by the cell thread
  const float doutb = (cval && a.dOutB) ? a.dOutB[(long long)bg * 2 * H + d * H + cj] : 0.0f;

  // gather role: per-step operands of every own (b, unit): 8 slots per cell
  //   0 dOut, 1..4 act, 5 c (LSTM) / h_prev (GRU), 6 c_prev (LSTM), 7 unused
  constexpr int NQ = (BC * 20 * 8 + NROLE - 1) / NROLE;
  StepLoader<NQ> ld;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int i = tid - NROLE + q * NROLE;  // item = slot * (BC*J) + cell
    const int slot = i / (BC * J), cell = i % (BC * J);
    const int ib = b0 + cell / J, ij = j0 + cell % J;
    const bool on = tid >= NROLE && slot < 8;
    const bool valid = on && ib < a.B && ij < H;
    const float* p = nullptr;
    int stride = 2 * H, shift = 0;
    if (valid) {
      if (slot == 0) {
        p = a.dOut + (long long)ib * T * 2 * H + d * H + ij;
      } else if (slot <= 4) {
        p = a.act + ((long long)ib * T * 2 + d) * AH + (slot - 1) * H + ij;
        stride = 2 * AH;
      } else if (CELL == CELL_LSTM && (slot == 5 || slot == 6)) {
        p = a.cs + ((long long)ib * T * 2 + d) * H + ij;
        shift = slot == 6 ? (d == 0 ? -1 : 1) : 0;  // the step that ran before t in this direction
      } else if (CELL == CELL_GRU && slot == 5) {
        p = a.hprev + (long long)ib * T * 2 * H + d * H + ij;
      }
    }
    ld.p[q] = p;
    ld.stride[q] = stride;
    ld.shift[q] = shift;
    ld.dst[q] = on ? cell * 8 + slot : -1;
  }
  if (tid >= NROLE) ld.issue(d == 0 ? T - 1 : 0, T);
  STAMP_DECL

  // ---- partials P[b][k] = sum_{own rows} dgh[b][r] W[r][k]
  auto matvec = [&]() {
    if (!mv) return;
    if constexpr (MF) return;  // MFMA path: mfma_publish below
    float acc[BC][KGLN];
#pragma unroll
    for (int bb = 0; bb < BC; ++bb)
#pragma unroll
      for (int c = 0; c < KGLN; ++c) acc[bb][c] = 0.0f;
    const float* gr = sdg + rp * RPLN;
#pragma unroll
    for (int i = 0; i < RPLN; ++i) {
#pragma unroll
      for (int bb = 0; bb < BC; ++bb) {
        const float g = gr[bb * RPAD + i];  // padded rows are zero
#pragma unroll
        for (int c = 0; c < KGLN; ++c) acc[bb][c] = fmaf(g, wreg[i][c], acc[bb][c]);
      }
    }
#pragma unroll
    for (int bb = 0; bb < BC; ++bb)
#pragma unroll
      for (int c = 0; c < KGLN; ++c) spart[(rp * BC + bb) * KW + kg * KGLN + c] = acc[bb][c];
  };

  // ---- MFMA path: D[k][b] = sum_r W[r][k] dgh[b][r] per 16-unit tile, published
  //      straight from the accumulator lanes (col = batch, 4 consecutive units)
  auto mfma_publish = [&](int s) {
    const unsigned short* bp = sdgb + (lane & 15) * SDG + 8 * (lane >> 4);
    bf16x8 bv[KSRMAX];
#pragma unroll
    for (int ks = 0; ks < KSRMAX; ++ks) bv[ks] = *reinterpret_cast<const bf16x8*>(bp + ks * 32);
    // wave-private transpose: D lanes (4 consecutive units of one batch row) -> [BC][WSPAN]
    float* wsc = spart + wv * BC * WSPAN;
    const int col = lane & 15;
#pragma unroll
    for (int t = 0; t < MTWMAX; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KSRMAX; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[t][ks], bv[ks], acc, 0, 0, 0);
      if (col < BC) *reinterpret_cast<f32x4*>(wsc + col * WSPAN + t * 16 + 4 * (lane >> 4)) = acc;
    }
    __builtin_amdgcn_wave_barrier();  // LDS ops of one wave complete in order
    STAMP(4)
    // coalesced publish of this wave's contiguous unit span (granules, tag s+1)
    u64* dst = xg + (long long)(s & 1) * NG * BC * H + (long long)w * BC * H;
#pragma unroll
    for (int e0 = 0; e0 < BC * WSPAN; e0 += 64) {
      const int e = e0 + lane;
      const int bb = e / WSPAN, k = wv * WSPAN + e % WSPAN;
      if ((BC * WSPAN) % 64 == 0 || e < BC * WSPAN)
        if (k < H) put_granule(dst + bb * H + k, (unsigned)(s + 1), wsc[e]);
    }
  };

  // Role-split loops, same barrier sequence per step (B1, B2, B3 -- no B3 on the
  // MFMA path); see the forward.
  if (tid >= NROLE) {
    for (int s = 0; s < T; ++s) {
      // ---- gather the NG partials of every own unit (tag s) and commit this
      //      step's operands (issued during the previous step)
      if (s > 0) {
        u64 v[GM];
        if (!gather<GM>(xg + (long long)((s - 1) & 1) * NG * BC * H, goff, (unsigned)s, v, a.spin_limit)) {
          atomicOr(a.status, 2);
          return;
        }
#pragma unroll
        for (int g = 0; g < GM; ++g)  // sdh[i] for i = tid-256 + 256 g ; unmapped entries stay 0
          if (goff[g] >= 0) sdh[tid - NROLE + g * NROLE] = __uint_as_float((unsigned)v[g]);
      }
      ld.commit(sop + (s & 1) * BC * J * 8);
      if (s + 1 < T) ld.issue(d == 0 ? T - 2 - s : s + 1, T);
      STAMP(0)
      __syncthreads();  // B1
      STAMP(1)
      __syncthreads();  // B2
      STAMP(3)
      if (s + 1 == T) break;
      if constexpr (!MF) {
        matvec();
        STAMP(4)
        __syncthreads();  // B3
        STAMP(5)
      }
    }
    STAMP_FLUSH
    return;
  }
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    STAMP(0)
    __syncthreads();  // B1
    STAMP(1)
    // ---- cell backward for (b, u): LDS operands only, global stores only
    if (ct) {
      float dh_rec = 0.0f;
      if (s > 0) dh_rec = sum_partials(sdh + cb * J + cu, BC * J, NG);
      const float* op = sop + (s & 1) * BC * J * 8 + tid * 8;
      const float dout = op[0] + doutb;
      const float act[4] = {op[1], op[2], op[3], op[4]};
      const float c = op[5], cprev = op[6], hprev = op[5];
      float dgi[NGATE], dgh[NGATE];
      if (cval) {
        const float dh = dout + dh_rec + dh_dir;
        if constexpr (CELL == CELL_LSTM) {
          const float ig = act[0], fg = act[1], gg = act[2], og = act[3];
          const float tc = ftanh(c);
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
#pragma unroll
        for (int q = 0; q < NGATE; ++q) {
          if constexpr (MF)
            sdgb[cb * SDG + q * J + cu] = bf16_rne(dgh[q]);
          else
            sdg[cb * RPAD + q * J + cu] = dgh[q];
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
        for (int q = 0; q < NGATE; ++q) {
          if constexpr (MF)
            sdgb[cb * SDG + q * J + cu] = 0;
          else
            sdg[cb * RPAD + q * J + cu] = 0.0f;
        }
      }
    }
    STAMP(2)
    __syncthreads();  // B2
    STAMP(3)
    if (s + 1 == T) break;  // nothing flows past the sequence start
    if constexpr (MF) {
      mfma_publish(s);
      STAMP(6)
      continue;
    }
    matvec();
    STAMP(4)
    __syncthreads();  // B3
    STAMP(5)
    // ---- reduce over row parts and publish granules (tag s+1): waves 0-3 only
    {
      u64* dst = xg + (long long)(s & 1) * NG * BC * H + (long long)w * BC * H;
#pragma unroll
      for (int g = 0; g < GP; ++g) {
        if (psrc[g] >= 0) {
          float v = 0.0f;
          for (int p = 0; p < a.RP; ++p) v += spart[p * BC * KW + psrc[g]];
          put_granule(dst + tid + g * NROLE, (unsigned)(s + 1), v);
        }
      }
    }
    STAMP(6)
    // sdg is rewritten after the next gather barrier, spart after the next cell
    // barrier, sdh after this step's barriers: every reader is behind them.
  }
  STAMP_FLUSH
}

// --------------------------------------------------------------------------
// BPTT, bf16 MFMA mode with the packed hand-off (the throughput path; see the
// packed forward above for the measurements behind each choice).  What crosses
// workgroups per step are the partial sums P_w[b][k] = sum_{own rows r} dgh[b][r]
// W[r][k]; they are packed as 24-bit floats (fp32 rounded to 15 mantissa bits,
// relative error <= 2^-16, far below the bf16 rounding of dgh itself), two per
// tagged 8-B granule:
//   granule = { lo: p0 | (p1 & 0xFF) << 24, hi: (p1 >> 8) | tag << 16 }
// one 16-B store per 4 units (two granules), plain or `sc1` by the group's placement,
// buffer [slot][copy][producer][b][HG granules], HG = H/2 rounded up to even.
// Waves: 0-3 cell backward (rows b = tid/32) + MFMA W^T dgh + publish;
//        4 polls the NG producers' partials of the own J units into LDS;
//        5-7 per-step operand prefetch.
// --------------------------------------------------------------------------
// BPTT per-step operand loads (prefetch waves): issued after B1, in the cell phase, not beside the
// polling sweeps in the CU's memory queue (BWD_PF_LATE)
#ifndef BWD_PF_LATE
#define BWD_PF_LATE 1
#endif
// the packed BPTT's prefetch waves keep two steps' operand loads in flight (round 6); 0: one step ahead
#ifndef BWD_PF2
#define BWD_PF2 1
#endif
// ... as straight-line even / odd pairs with the loads issued every step (round 6: hipcc's waitcnt pass
// then keeps the newer step's loads in flight at each commit -- BPTT 331 -> 322 us per launch, bitwise,
// profiles/r06_pf2_unroll_ab.txt); 0: the even / odd branch form
#ifndef BWD_PF2_UNROLL
#define BWD_PF2_UNROLL 1
#endif
// timing experiment only (results wrong): 1 the prefetch waves issue no operand loads in the steps, 2 nor
// form step factors.  Round 6: BPTT 331 -> 289 us per launch at 1 (the loads' price is paid in the
// hand-off: they share the consumer CU's memory queue with the polls); non-temporal operand loads were
// slower (376 us), the last forward layer's act / c saved with plain stores for the top BPTT no faster
#ifndef BWD_EXP_PF
#define BWD_EXP_PF 0
#endif
#if !defined(DL4SS_VARIANT_BUILD) && (BWD_EXP_PF || FWD_EXP_NOXDMA)
#error "BWD_EXP_PF / FWD_EXP_NOXDMA are for tools/variant_lib.py builds only"
#endif
// the cell lanes' dG / dGh stores of step s-1 issued after B1 of step s (before the cell update)
// instead of right after the publish: measured slower, 7994 vs 8085 mixtures/s
// (profiles/r03_dglate.jsonl) -- their issue then sits on the cell phase's critical path
__device__ __forceinline__ unsigned pack24(float v) {
  const unsigned u = __float_as_uint(v);
  return (u + 0x80u) >> 8;  // round to nearest (ties away) on the dropped 8 bits
}
__device__ __forceinline__ float unpack24(unsigned r) { return __uint_as_float(r << 8); }

template <int CELL, int BC, int NZ = 1>
__global__ __launch_bounds__(NT, 1) void rnn_bwd_pk_kernel(RnnArgs a) {
  constexpr int NGATE = CELL == CELL_LSTM ? 4 : 3;
  // partial-sum slots of the gather (polling waves): a lane group of BSL_Q lanes = every (b, quad)
  // of one slot at J <= 20; BSL_G groups per polling wave; BSL_N slots; GLK producers per lane
  constexpr int BSL_Q = BC * 5;
  constexpr int BSL_G = 64 / BSL_Q > 0 ? 64 / BSL_Q : 1;
  constexpr int BSL_N = BWD_NPW * BSL_G < 16 ? BWD_NPW * BSL_G : 16;
  constexpr int GLK = (16 + BSL_N - 1) / BSL_N;  // NG <= 16
  static_assert(BSL_Q <= 64, "one (b, quad) item per lane");
  constexpr int MTWMAX = (HMAX / 16 + 3) / 4;  // MFMA unit tiles per wave (5)
  constexpr int KSRMAX = (4 * 20 + 31) / 32;   // MFMA K-steps over gate rows (3)
  constexpr int SDG = KSRMAX * 32 + 8;         // bf16 row stride of the dgh B image
  constexpr int WSPAN = MTWMAX * 16;           // output units per MFMA wave (80)
  constexpr int WSP = WSPAN + 4;               // transpose row stride (floats): rows on distinct bank quads
  const int H = a.H, T = a.T, J = a.J, NG = a.NG;
  const int R = NGATE * J;
  const int ngroups = 2 * a.nchunk;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int group, w;
  group_pk(a.gctl, NG, ngroups, a.spin_limit, a.status, smem, group, w);
  const int d = group / a.nchunk, chunk = group % a.nchunk;
  const int b0 = chunk * BC;
  const int j0 = w * J;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int GH = NGATE * H;
  const int AH = 4 * H;
  const int HG = ((H + 1) / 2 + 1) & ~1;  // granules per (producer, row), even: 16-B aligned rows

  unsigned short* sdgb = reinterpret_cast<unsigned short*>(smem);  // [16][SDG] bf16 dgh B image
  float* sdh = smem + 8 * SDG;                                      // [16][BC][J] gathered partials (rows >= NG stay 0)
  float* wsc = sdh + ((16 * BC * J + 3) & ~3);                      // [4 waves][BC][WSP]
  // per-step operands, [2 steps][2 planes][cell = b * J + u][4] (slots 0-3 in plane 0, 4-7 in
  // plane 1): the cell lanes read their two 16-B quads conflict-free (16 lanes on 16 consecutive
  // cells), and so is the prefetch commit (below)
  constexpr int SOPP = BC * 32 * 4 + 16;
  float* sop = wsc + 4 * BC * WSP;
  for (int i = tid; i < 8 * SDG + 16 * BC * J; i += NT) smem[i] = 0.0f;

  // ---- W_hh^T tiles (waves 0-3): tile m = wv*MTWMAX + t, lane holds
  //      A[k = m*16 + (lane&15)][r = ks*32 + 8(lane>>4) + j] = W[row(r)][k]
  const bool mv = wv < 4;
  bf16x8 afr[MTWMAX][KSRMAX];
#pragma unroll
  for (int t = 0; t < MTWMAX; ++t) {
    const int k = (wv * MTWMAX + t) * 16 + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < KSRMAX; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int rr = ks * 32 + 8 * (lane >> 4) + j;
        const int q = rr / J, u = rr % J;
        const bool ok = mv && k < H && rr < R && j0 + u < H;
        afr[t][ks][j] = (short)bf16_rne(ok ? a.Whh[((long long)d * GH + q * H + j0 + u) * H + k] : 0.0f);
      }
  }

  // ---- cell lanes: row cb = tid / 32, unit cu = tid % 32 (< J)
  const int cb = tid >> 5, cu = tid & 31;
  const bool ct = tid < BC * 32 && cu < J;
  const int cj = j0 + cu;
  const int bg = b0 + cb;
  const bool cval = ct && cj < H && bg < a.B;
  float dc_next = 0.0f, dh_dir = 0.0f;
  const float doutb = (cval && a.dOutB) ? a.dOutB[(long long)bg * 2 * H + d * H + cj] : 0.0f;

  // partial-sum granules of this group: [2 slots][hand-off, spare][NG][BC][HG] x 8 B; the
  // spare copy of slot 1 holds the placement granules
  const int copy_g = NG * BC * HG;
  u64* xg = a.xbuf + (long long)group * 4 * copy_g;
  const __amdgpu_buffer_rsrc_t xr = granule_rsrc(xg, (unsigned)(4 * copy_g * 8));
  __shared__ int s_wt;
  if (tid == 0) __hip_atomic_store(xg + 3 * copy_g + w, (1ull << 32) | xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (wv == WPOLL) {
    const bool wt = group_needs_write_through(xg + 3 * copy_g, NG, lane, a.spin_limit, a.status, a.place_force);
    if (lane == 0) s_wt = wt;
  }

  // ---- prefetch waves WPF..7: per-step operands of every own (b, unit): 8 slots per cell
  //   0 dOut, 1..4 act, 5 c (LSTM) / h_prev (GRU), 6 c_prev (LSTM), 7 unused
  constexpr int WPF = WPOLL + BWD_NPW;  // waves WPOLL .. WPF-1 poll
  constexpr int NPF = NT - WPF * 64;
  // (round 3 committed the raw operands straight into the cell lanes' record, slot-major: 16-B
  // strided words, a 4-way conflict -- SQ_LDS_BANK_CONFLICT / IDX_ACTIVE 0.036 -> 0.157; cell-major
  // items were conflict-free but touched one cache line per lane octet and held the prefetch waves
  // ~650 cycles past the cell phase, profiles/r03_pfmap_stamps.txt)
  constexpr int NSL = CELL == CELL_LSTM ? 7 : 6;
  // each prefetch wave owns half of the cells (cpw of them) and stages their raw operands
  // slot-major in a wave-private LDS block [NSL][CPWP] (a load instruction's lanes read consecutive
  // units of one operand row; consecutive lanes commit consecutive words), then one lane per cell
  // turns them into the cell's step factors (pf_factors)
  // (BC >= 4 only.  At BC <= 2 the raw operands go straight into the record as slot-major items --
  // 64 consecutive cells of one slot per load instruction, a 4-way commit conflict: there the
  // step is short and the loads' spread decides; 4 slots x 8 cells per half-wave (conflict-free,
  // twice the cache lines per instruction) took the BiGRU C3 BPTT from 325 to 407 us per launch)
  static_assert(NPF == 128, "two prefetch waves");
  constexpr bool PFF = BC >= 4;
  constexpr int CPWP = (BC * 20 + 1) / 2;  // raw staging pitch: cells per prefetch wave at J <= 20
  // PFF: the act slots 1-4 arrive as ONE 16-B item per cell (the cell-major act of the packed
  // forward, a.act_cm, required at BC >= 4 by the launcher); the scalar loader carries dOut and
  // (LSTM) c_prev = c at the step's neighbour t -+ 1, or (GRU) h_prev.  The LSTM's c of a step is
  // the c_prev the previous step loaded: pf_factors keeps it in the slot-5 row for the next step
  // (one scalar load per cell and step fewer; the first step's c is loaded once before the loop)
  constexpr int NSLS = 2;
  constexpr int NQ = PFF ? (NSLS * CPWP + 63) / 64 : (BC * 20 * NSL + NPF - 1) / NPF;
  constexpr int NQA = PFF ? (CPWP + 63) / 64 : 1;
  const int ncell = BC * J, cpw = (ncell + 1) / 2, pwi = wv - WPF;
  float* sraw = sop + 2 * 2 * SOPP + (wv >= WPF ? pwi : 0) * NSL * CPWP;
  StepLoader<NQ, NZ> ld;  // dOut: NZ split-K slabs (DL4SS_RNN_DOUT_SLABS)
  ld.zs = a.dout_zs;
  const float4* ap[NQA];
  float4 av[NQA];
  // BWD_PF2 at batch chunks >= 4 (the step-factor prefetch): two steps in flight, ld2 / av2 the odd
  // steps' operands.  At BC <= 2 (raw operands straight into the record) one step ahead stays: C1's
  // B = 1 step measured 461 vs 468 mixtures/s with two (profiles/r06_cfg_pf2.txt)
  constexpr bool PF2 = BWD_PF2 && PFF;
  StepLoader<NQ, NZ> ld2;
  float4 av2[NQA];
  int ac[NQA];
#pragma unroll
  for (int q = 0; q < NQA; ++q) {
    const int c = lane + 64 * q, cell = pwi * cpw + c;
    const int ib = b0 + cell / J, ij = j0 + cell % J;
    const bool ok = PFF && wv >= WPF && c < cpw && cell < ncell;
    ap[q] = (ok && ib < a.B && ij < H) ? reinterpret_cast<const float4*>(a.act) + ((long long)ib * T * 2 + d) * H + ij
                                       : nullptr;
    ac[q] = ok ? c : -1;
    av[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto act_issue = [&](float4* v, int t) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NQA; ++q)
      v[q] = ap[q] != nullptr ? ap[q][(long long)t * 2 * H] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto act_commit = [&](const float4* v) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NQA; ++q)
      if (ac[q] >= 0) {
        sraw[1 * CPWP + ac[q]] = v[q].x;
        sraw[2 * CPWP + ac[q]] = v[q].y;
        sraw[3 * CPWP + ac[q]] = v[q].z;
        sraw[4 * CPWP + ac[q]] = v[q].w;
      }
  };
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    int slot, c = 0, cell;
    bool on;
    if constexpr (PFF) {
      const int i = lane + 64 * q;
      const int ss = i / cpw;  // scalar slot 0, 1 -> slot 0, and 6 (LSTM c_prev) / 5 (GRU h_prev)
      slot = ss == 0 ? 0 : CELL == CELL_LSTM ? 6 : 5;
      c = i - ss * cpw;
      cell = pwi * cpw + c;
      on = wv >= WPF && ss < NSLS && cell < ncell;
    } else {
      const int i = tid - WPF * 64 + q * NPF;
      slot = i / ncell;
      cell = i - slot * ncell;
      on = wv >= WPF && i >= 0 && slot < NSL;
    }
    const int ib = b0 + cell / J, iu = cell % J, ij = j0 + iu;
    const bool valid = on && ib < a.B && ij < H;
    const float* p = nullptr;
    int stride = 2 * H, shift = 0;
    if (valid) {
      if (slot == 0) {
        p = a.dOut + (long long)ib * T * 2 * H + d * H + ij;
      } else if (slot <= 4) {
        p = a.act + ((long long)ib * T * 2 + d) * AH + (slot - 1) * H + ij;
        stride = 2 * AH;
      } else if (CELL == CELL_LSTM && (slot == 5 || slot == 6)) {
        p = a.cs + ((long long)ib * T * 2 + d) * H + ij;
        shift = slot == 6 ? (d == 0 ? -1 : 1) : 0;
      } else if (CELL == CELL_GRU && slot == 5) {
        p = a.hprev + (long long)ib * T * 2 * H + d * H + ij;
      }
    }
    ld.p[q] = p;
    ld.stride[q] = stride;
    ld.shift[q] = shift;
    ld.dst[q] = !on ? -1 : PFF ? slot * CPWP + c : (slot >> 2) * SOPP + cell * 4 + (slot & 3);
    ld.zq[q] = slot == 0;
  }
  auto tstep = [&](int s) { return d == 0 ? T - 1 - s : s; };  // time index of BPTT step s
  if constexpr (PF2) ld2 = ld;
  if (wv >= WPF) {
    ld.issue(tstep(0), T);
    if constexpr (PFF) act_issue(av, tstep(0));
    if (PF2 && T > 1) {
      ld2.issue(tstep(1), T);
      if constexpr (PFF) act_issue(av2, tstep(1));
    }
    if constexpr (PFF && CELL == CELL_LSTM) {  // the first step's c (later steps reuse c_prev)
      const int t0 = d == 0 ? T - 1 : 0;
      for (int c = lane; c < cpw; c += 64) {
        const int cell = pwi * cpw + c;
        const int ib = b0 + cell / J, ij = j0 + cell % J;
        sraw[5 * CPWP + c] = (cell < ncell && ib < a.B && ij < H) ? a.cs[((long long)(ib * T + t0) * 2 + d) * H + ij]
                                                                     : 0.0f;
      }
    }
  }
  __syncthreads();
  const bool wt = __builtin_amdgcn_readfirstlane(s_wt) != 0;  // granules written through (group spans XCDs)
  if (tid == 0) release_start(a.gctl, a.xbuf, ngroups, NG, 4LL * copy_g, 3LL * copy_g);
  STAMP_DECL

  if (wv >= WPOLL && wv < WPF) {
    // ---- polling waves: a lane owns one (b, quad of 4 units) and BSL_P producers of it -- slot
    //      sl = pw * BSL_G + (lane / (5 BC)), producers sl, sl + BSL_N, ... -- and sums their
    //      partials in registers: the cell lanes then add BSL_N slot partials instead of NG
    //      producer partials (16 LDS reads + a 16-leaf tree cost ~150 cycles of the cell phase,
    //      round-4 stamps).  Lanes of a group read consecutive quads of one producer row (the
    //      sweep touches as many cache lines as a producer-major map).
    const int pw = wv - WPOLL;
    const int JQ = J / 4;
    const int gi = lane / BSL_Q, bq = lane % BSL_Q;
    const int pb_b = bq / 5, qd = bq % 5;
    const int sl = pw * BSL_G + gi;
    const bool lane_on = gi < BSL_G && sl < BSL_N && qd < JQ && pb_b < BC;
    int loff[GLK];
    bool on[GLK];
#pragma unroll
    for (int g = 0; g < GLK; ++g) {
      const int p = sl + BSL_N * g;
      on[g] = lane_on && p < NG;
      loff[g] = on[g] ? (p * BC + pb_b) * HG + (j0 >> 1) + 2 * qd : 0;  // granule offset within a copy
    }
    const int doff = lane_on ? (sl * BC + pb_b) * J + 4 * qd : 0;  // sdh[(slot * BC + b) * J + u]
    for (int s = 0; s < T; ++s) {
      if (s > 0) {
        const unsigned tag = (unsigned)s & 0xFFFFu;
        if (wv == WPOLL) TRACE(2, s);
        // 16-B `sc1` buffer loads, one per granule pair (half the requests of the 8-B atomic
        // loads: BPTT 4800 -> 4153, forward 3302 -> 3111 cycles per step); the empty asm with a
        // memory clobber keeps every sweep inside the loop (the buffer intrinsic is a plain
        // read-only load to the compiler: hoisted out of the spin loop without it)
        const int sb = ((s - 1) & 1) * 2 * copy_g * 8;  // the slot's hand-off copy (bytes)
        u32x4 q[GLK], qa[GLK], qb[GLK];
        unsigned done = 0;
#if BWD_POLL_SLEEP
        __builtin_amdgcn_s_sleep(BWD_POLL_SLEEP);  // (experiment, as FWD_POLL_SLEEP)
#endif
        asm volatile("" ::: "memory");
#pragma unroll
        for (int g = 0; g < GLK; ++g) qa[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, sb + loff[g] * 8, 0, 16);
        unsigned spins = 0;
        while (true) {
          asm volatile("" ::: "memory");
#pragma unroll
          for (int g = 0; g < GLK; ++g) qb[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, sb + loff[g] * 8, 0, 16);
#pragma unroll
          for (int g = 0; g < GLK; ++g) {
            const bool m = ((qa[g].y >> 16) == tag) & ((qa[g].w >> 16) == tag) & !((done >> g) & 1);
            q[g] = m ? qa[g] : q[g];
            done |= (unsigned)m << g;
          }
          if (done == (1u << GLK) - 1) break;
          asm volatile("" ::: "memory");
#pragma unroll
          for (int g = 0; g < GLK; ++g) qa[g] = __builtin_amdgcn_raw_buffer_load_b128(xr, sb + loff[g] * 8, 0, 16);
#pragma unroll
          for (int g = 0; g < GLK; ++g) {
            const bool m = ((qb[g].y >> 16) == tag) & ((qb[g].w >> 16) == tag) & !((done >> g) & 1);
            q[g] = m ? qb[g] : q[g];
            done |= (unsigned)m << g;
          }
          if (done == (1u << GLK) - 1) break;
          if (++spins > a.spin_limit) {
            atomicOr(a.status, 2);
            return;
          }
        }
        float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);  // this lane's producers, summed in order g
#pragma unroll
        for (int g = 0; g < GLK; ++g) {
          if (on[g]) {
            const unsigned l0 = q[g].x, l1 = q[g].y, h0 = q[g].z, h1 = q[g].w;
            acc4.x += unpack24(l0 & 0xFFFFFFu);
            acc4.y += unpack24((l0 >> 24) | ((l1 & 0xFFFFu) << 8));
            acc4.z += unpack24(h0 & 0xFFFFFFu);
            acc4.w += unpack24((h0 >> 24) | ((h1 & 0xFFFFu) << 8));
          }
        }
        if (lane_on) *reinterpret_cast<float4*>(sdh + doff) = acc4;  // 16-B aligned: J % 4 == 0
        if (wv == WPOLL) TRACE(1, s);
      }
      STAMP(0)
      __syncthreads();  // B1
      STAMP(1)
      __syncthreads();  // B2
      STAMP(3)
      if (s + 1 == T) break;
    }
    STAMP_FLUSH
    return;
  }
  if (wv >= WPF) {
    // the step factors of this wave's cells: everything of the cell backward that does not depend
    // on the gathered dh, off the cell lanes' B1 -> B2 path (LSTM: tanh(c) and the gate
    // derivatives; GRU: the z / n / r products), into the record the cell lanes read after B1:
    //   LSTM {dOut, o (1 - tanh^2 c), g i (1 - i), c_prev f (1 - f)} {i (1 - g^2), tanh(c) o (1 - o), f, -}
    //   GRU  {dOut, (1-z)(1-n^2) hn r (1-r), (h_prev - n) z (1-z), (1-z)(1-n^2)} {(1-z)(1-n^2) r, z, -, -}
    auto pf_factors = [&](int s, const StepLoader<NQ, NZ>& L, const float4* A) __attribute__((always_inline)) {
      L.commit(sraw);
      act_commit(A);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      // one lane per cell, in passes of 64: cpw = ceil(BC J / 2) is 80 at BC = 8, J = 20
      for (int c = lane; c < cpw; c += 64) {
        const int cell = pwi * cpw + c;
        if (cell >= ncell) break;
        float v[NSL];
#pragma unroll
        for (int k = 0; k < NSL; ++k) v[k] = sraw[k * CPWP + c];
        float4 p0, p1;
        if constexpr (CELL == CELL_LSTM) {
          const float ig = v[1], fg = v[2], gg = v[3], og = v[4];
          const float tc = ftanh(v[5]);
          p0 = make_float4(v[0], og * (1.0f - tc * tc), gg * ig * (1.0f - ig), v[6] * fg * (1.0f - fg));
          p1 = make_float4(ig * (1.0f - gg * gg), tc * og * (1.0f - og), fg, 0.0f);
        } else {
          const float rg = v[1], zg = v[2], ng = v[3], hn = v[4];
          const float gn = (1.0f - zg) * (1.0f - ng * ng);
          p0 = make_float4(v[0], gn * hn * rg * (1.0f - rg), (v[5] - ng) * zg * (1.0f - zg), gn);
          p1 = make_float4(gn * rg, zg, 0.0f, 0.0f);
        }
        float* rec = sop + (s & 1) * 2 * SOPP + cell * 4;
        *reinterpret_cast<float4*>(rec) = p0;
        *reinterpret_cast<float4*>(rec + SOPP) = p1;
        if constexpr (CELL == CELL_LSTM) sraw[5 * CPWP + c] = v[6];  // the next step's c
      }
    };
    if constexpr (PF2) {
    // two steps in flight: step s's operands were issued in step s - 2 (ld for even s, ld2 for odd), so
    // a load has a whole step more than the cell phase + hand-off window to land before the commit
    // (round 6: with one step ahead the commit waited on them -- two more dOut loads per cell for the
    // split-K slabs cost ~8 us per launch, profiles/r06_nz_ab.txt)
    auto pf_step = [&](int s, StepLoader<NQ, NZ>& L, float4* A) __attribute__((always_inline)) {
#if BWD_EXP_PF < 2
      if constexpr (PFF)
        pf_factors(s, L, A);
      else
        L.commit(sop + (s & 1) * 2 * SOPP);
#endif
      __syncthreads();  // B1
      if (BWD_EXP_PF == 0 && s + 2 < T) {
        L.issue(tstep(s + 2), T);
        if constexpr (PFF) act_issue(A, tstep(s + 2));
      }
      __syncthreads();  // B2
    };
#if BWD_PF2_UNROLL
    // the even / odd pair as straight-line code, the loads issued every step (past the end the last
    // step's again, unused): the same loads in flight at every commit, for hipcc's waitcnt pass
    auto pf_step_u = [&](int s, StepLoader<NQ, NZ>& L, float4* A) __attribute__((always_inline)) {
      if constexpr (PFF)
        pf_factors(s, L, A);
      else
        L.commit(sop + (s & 1) * 2 * SOPP);
      __syncthreads();  // B1
      const int tn = tstep(min(s + 2, T - 1));
      L.issue(tn, T);
      if constexpr (PFF) act_issue(A, tn);
      __syncthreads();  // B2
    };
    int s = 0;
    for (; s + 1 < T; s += 2) {
      pf_step_u(s, ld, av);
      pf_step_u(s + 1, ld2, av2);
    }
    if (s < T) pf_step_u(s, ld, av);
#else
    for (int s = 0; s < T; ++s) {
      if (s & 1)
        pf_step(s, ld2, av2);
      else
        pf_step(s, ld, av);
      if (s + 1 == T) break;
    }
#endif
    } else {
    for (int s = 0; s < T; ++s) {
      if constexpr (PFF)
        pf_factors(s, ld, av);
      else
        ld.commit(sop + (s & 1) * 2 * SOPP);
#if BWD_PF_LATE
      // the next step's operand loads go out after B1, in the cell phase: not in the CU's memory
      // queue beside the polling sweeps (MI355X_MICROARCH.md handoff-1to1: the hand-off price sits
      // in the consumer CU's queue); they still have the cell phase and the next poll window to land
      __syncthreads();  // B1
      if (s + 1 < T) {
        ld.issue(tstep(s + 1), T);
        if constexpr (PFF) act_issue(av, tstep(s + 1));
      }
      __syncthreads();  // B2
#else
      if (s + 1 < T) {
        ld.issue(tstep(s + 1), T);
        if constexpr (PFF) act_issue(av, tstep(s + 1));
      }
      __syncthreads();  // B1
      __syncthreads();  // B2
#endif
      if (s + 1 == T) break;
    }
    }
    return;
  }

  // ---- waves 0-3: cell backward, then MFMA partials and their publish
  float sbi[NGATE], sbh[NGATE];  // this cell's bias-gradient sums over t
  float pgi[NGATE], pgh[NGATE];  // this step's dG / dGh, stored after the publish
  int pt = 0;
#pragma unroll
  for (int q = 0; q < NGATE; ++q) sbi[q] = sbh[q] = pgi[q] = pgh[q] = 0.0f;
  auto store_dg = [&]() {
    if (!cval) return;
    const long long go = (long long)((bg * T + pt) * 2 + d) * GH + cj;
    if (a.dG) {
#pragma unroll
      for (int q = 0; q < NGATE; ++q) a.dG[go + q * H] = pgi[q];
    }
    if (a.dGb) {
#pragma unroll
      for (int q = 0; q < NGATE; ++q) a.dGb[go + q * H] = bf16_rne(pgi[q]);
    }
    if (CELL == CELL_GRU) {
      if (a.dGh) {
#pragma unroll
        for (int q = 0; q < NGATE; ++q) a.dGh[go + q * H] = pgh[q];
      }
      if (a.dGhb) {
        const long long goh = (long long)((bg * T + pt) * 2 + d) * a.ghb + cj;
#pragma unroll
        for (int q = 0; q < NGATE; ++q) a.dGhb[goh + q * H] = bf16_rne(pgh[q]);
      }
    }
  };
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    STAMP(0)
    __syncthreads();  // B1
    STAMP(1)
    if (tid == 0) TRACE(3, s);
    if (tid < BC * 32) {
      float dgi[NGATE], dgh[NGATE];
#pragma unroll
      for (int q = 0; q < NGATE; ++q) dgi[q] = dgh[q] = 0.0f;
      if (cval) {
        // two 16-B reads per lane (the record's two planes), issued first, with the slot
        // partial reads behind them in the same LDS round trip (sdh is zero before the first gather)
        const int rec = (s & 1) * 2 * SOPP + (cb * J + cu) * 4;
        const float4 o0 = *reinterpret_cast<const float4*>(sop + rec);
        const float4 o1 = *reinterpret_cast<const float4*>(sop + rec + SOPP);
        const float dh_rec = sum_slots<BSL_N>(sdh + cb * J + cu, BC * J);
        const float dout = o0.x + doutb;
        const float dh = dout + dh_rec + dh_dir;
        STAMP(7)
        if constexpr (PFF && CELL == CELL_LSTM) {  // the record holds the step factors (pf_factors)
          const float dc = dc_next + dh * o0.y;
          dgi[0] = dc * o0.z;
          dgi[1] = dc * o0.w;
          dgi[2] = dc * o1.x;
          dgi[3] = dh * o1.y;
          dc_next = dc * o1.z;
#pragma unroll
          for (int q = 0; q < NGATE; ++q) dgh[q] = dgi[q];
        } else if constexpr (PFF) {
          dgi[0] = dh * o0.y;
          dgi[1] = dh * o0.z;
          dgi[2] = dh * o0.w;
          dgh[0] = dgi[0];
          dgh[1] = dgi[1];
          dgh[2] = dh * o1.x;
          dh_dir = dh * o1.y;
        } else if constexpr (CELL == CELL_LSTM) {  // raw operands {dOut, i, f, g} {o, c, c_prev, -}
          const float ig = o0.y, fg = o0.z, gg = o0.w, og = o1.x;
          const float tc = ftanh(o1.y);
          const float dc = dc_next + dh * og * (1.0f - tc * tc);
          dgi[0] = dc * gg * ig * (1.0f - ig);
          dgi[1] = dc * o1.z * fg * (1.0f - fg);
          dgi[2] = dc * ig * (1.0f - gg * gg);
          dgi[3] = dh * tc * og * (1.0f - og);
          dc_next = dc * fg;
#pragma unroll
          for (int q = 0; q < NGATE; ++q) dgh[q] = dgi[q];
        } else {  // raw operands {dOut, r, z, n} {hn, h_prev, -, -}
          const float rg = o0.y, zg = o0.z, ng = o0.w, hn = o1.x;
          const float dn = dh * (1.0f - zg);
          const float dz = dh * (o1.y - ng);
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
#pragma unroll
        for (int q = 0; q < NGATE; ++q) {
          sbi[q] += dgi[q];
          sbh[q] += dgh[q];
          pgi[q] = dgi[q];
          pgh[q] = dgh[q];
        }
      }
      if (ct) {
#pragma unroll
        for (int q = 0; q < NGATE; ++q) sdgb[cb * SDG + q * J + cu] = bf16_rne(dgh[q]);
      }
    }
    pt = t;
    STAMP(2)
    __syncthreads();  // B2
    STAMP(3)
    if (s + 1 == T) {  // nothing flows past the sequence start
      store_dg();
      break;
    }
    // ---- D[k][b] = sum_r W[r][k] dgh[b][r] per 16-unit tile, packed four units per 16-B store: at BC = 4
    //      the quads are spread over the wave by DPP row shifts (BWD_PUB_DPP), otherwise transposed through
    //      wave-private LDS to [b][unit].  (Round 4's register-direct form -- five 16-lane stores per wave --
    //      lost to the transpose; the DPP form keeps the transpose's two full stores and drops its LDS trip.)
    {
      // rows >= BC of the dgh B image are zero: read row BC (broadcast, conflict-free B reads)
      const unsigned short* bp = sdgb + min(lane & 15, BC) * SDG + 8 * (lane >> 4);
      bf16x8 bv[KSRMAX];
#pragma unroll
      for (int ks = 0; ks < KSRMAX; ++ks) bv[ks] = *reinterpret_cast<const bf16x8*>(bp + ks * 32);
      float* wsw = wsc + wv * BC * WSP;
      const int col = lane & 15;
      // k-step-major over the wave's tiles: MTWMAX independent chains in flight
      f32x4 acc[MTWMAX];
#pragma unroll
      for (int t2 = 0; t2 < MTWMAX; ++t2) acc[t2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KSRMAX; ++ks)
#pragma unroll
        for (int t2 = 0; t2 < MTWMAX; ++t2)
          acc[t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[t2][ks], bv[ks], acc[t2], 0, 0, 0);
#if BWD_PUB_DPP
      if constexpr (BC == 4 && MTWMAX == 5) {
        // lane 16 g + b (b < 4) holds tile t's four units 16 t + 4 g .. + 3 of batch row b.  Tiles 0-3 go out
        // in ONE full-wave 16-B store: lane 16 g + 4 t + b takes tile t's quad from lane 16 g + b by a DPP row
        // shift of 4 t into bank t (no LDS transpose); tile 4 from its own 16 lanes
        const unsigned tag = (unsigned)(s + 1) & 0xFFFFu;
        f32x4 xq = acc[0];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          int v = __float_as_int(xq[c]);
          v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[1][c]), 0x114, 0xF, 0x2, false);  // row_shr:4
          v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[2][c]), 0x118, 0xF, 0x4, false);  // row_shr:8
          v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[3][c]), 0x11C, 0xF, 0x8, false);  // row_shr:12
          xq[c] = __int_as_float(v);
        }
        const int bb = lane & 3, g = lane >> 4;
        auto put = [&](const f32x4 v, int k) __attribute__((always_inline)) {
          const unsigned r0 = pack24(v[0]), r1 = pack24(v[1]), r2 = pack24(v[2]), r3 = pack24(v[3]);
          const u32x4 x = {r0 | (r1 << 24), (r1 >> 8) | (tag << 16), r2 | (r3 << 24), (r3 >> 8) | (tag << 16)};
          const int off = (((s & 1) * 2 * NG + w) * BC + bb) * HG + (k >> 1);  // granules
          if (wt)
            __builtin_amdgcn_raw_buffer_store_b128(x, xr, off * 8, 0, 16);  // sc1 write-through (group spans XCDs)
          else
            __builtin_amdgcn_raw_buffer_store_b128(x, xr, off * 8, 0, 0);   // plain: stays in the group's L2
        };
        const int k0 = wv * WSPAN + 16 * ((lane >> 2) & 3) + 4 * g;
        if (k0 < H) put(xq, k0);
        const int k4 = wv * WSPAN + 64 + 4 * g;
        if ((lane & 15) < 4 && k4 < H) put(acc[4], k4);
        STAMP(4)
        if (wv == 3) TRACE(0, s);
      } else if constexpr ((BC == 1 || BC == 2) && MTWMAX == 5) {
        // BC <= 2: all five tiles fit one 16-lane row -- tile t's quad of row b into lane BC t + b by a
        // row shift of BC t (bank mask of that lane group; tiles in increasing order, so a lane a shift
        // filled with a neighbour's unused column is rewritten by the later tile that owns it), ONE store
        const unsigned tag = (unsigned)(s + 1) & 0xFFFFu;
        f32x4 xq = acc[0];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          int v = __float_as_int(xq[c]);
          if constexpr (BC == 2) {
            v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[1][c]), 0x112, 0xF, 0x1, false);  // row_shr:2
            v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[2][c]), 0x114, 0xF, 0x2, false);  // row_shr:4
            v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[3][c]), 0x116, 0xF, 0x2, false);  // row_shr:6
            v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[4][c]), 0x118, 0xF, 0x4, false);  // row_shr:8
          } else {
            v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[1][c]), 0x111, 0xF, 0x1, false);  // row_shr:1
            v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[2][c]), 0x112, 0xF, 0x1, false);  // row_shr:2
            v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[3][c]), 0x113, 0xF, 0x1, false);  // row_shr:3
            v = __builtin_amdgcn_update_dpp(v, __float_as_int(acc[4][c]), 0x114, 0xF, 0x2, false);  // row_shr:4
          }
          xq[c] = __int_as_float(v);
        }
        const int p = lane & 15, t = p / BC, bb = p % BC, g = lane >> 4;
        const int k = wv * WSPAN + 16 * t + 4 * g;
        if (p < 5 * BC && k < H) {
          const unsigned r0 = pack24(xq[0]), r1 = pack24(xq[1]), r2 = pack24(xq[2]), r3 = pack24(xq[3]);
          const u32x4 x = {r0 | (r1 << 24), (r1 >> 8) | (tag << 16), r2 | (r3 << 24), (r3 >> 8) | (tag << 16)};
          const int off = (((s & 1) * 2 * NG + w) * BC + bb) * HG + (k >> 1);  // granules
          if (wt)
            __builtin_amdgcn_raw_buffer_store_b128(x, xr, off * 8, 0, 16);  // sc1 write-through (group spans XCDs)
          else
            __builtin_amdgcn_raw_buffer_store_b128(x, xr, off * 8, 0, 0);   // plain: stays in the group's L2
        }
        STAMP(4)
        if (wv == 3) TRACE(0, s);
      } else
#endif
      {
      if (col < BC) {
#pragma unroll
        for (int t2 = 0; t2 < MTWMAX; ++t2)
          *reinterpret_cast<f32x4*>(wsw + col * WSP + t2 * 16 + 4 * (lane >> 4)) = acc[t2];
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      STAMP(4)
      const unsigned tag = (unsigned)(s + 1) & 0xFFFFu;
      constexpr int NQW = BC * WSPAN / 4;  // 16-B quads of this wave
      constexpr int NQI = (NQW + 63) / 64;
      // every quad's LDS read issued before the first is used (one LDS round trip, not one per store:
      // a lane past the wave's quads reads a valid clamped quad and stores nothing)
      float4 vq[NQI];
#pragma unroll
      for (int i = 0; i < NQI; ++i) {
        const int e = min(64 * i + lane, NQW - 1);
        const int bb = e / (WSPAN / 4), kl = 4 * (e % (WSPAN / 4));
        vq[i] = *reinterpret_cast<const float4*>(wsw + bb * WSP + kl);
      }
#pragma unroll
      for (int e0 = 0; e0 < NQW; e0 += 64) {
        const int e = e0 + lane;
        const int bb = e / (WSPAN / 4), k = wv * WSPAN + 4 * (e % (WSPAN / 4));
        if ((NQW % 64 == 0 || e < NQW) && k < H) {
          const float4 v = vq[e0 / 64];
          const unsigned r0 = pack24(v.x), r1 = pack24(v.y), r2 = pack24(v.z), r3 = pack24(v.w);
          const u32x4 x = {r0 | (r1 << 24), (r1 >> 8) | (tag << 16), r2 | (r3 << 24), (r3 >> 8) | (tag << 16)};
          const int off = (((s & 1) * 2 * NG + w) * BC + bb) * HG + (k >> 1);  // granules
          if (wt)
            __builtin_amdgcn_raw_buffer_store_b128(x, xr, off * 8, 0, 16);  // sc1 write-through (group spans XCDs)
          else
            __builtin_amdgcn_raw_buffer_store_b128(x, xr, off * 8, 0, 0);   // plain: stays in the group's L2
        }
      }
      if (wv == 3) TRACE(0, s);
      }
    }
    STAMP(5)
    // this step's dG / dGh, after the publish (off the critical path; issued after B1 of the next
    // step instead they measured slower, 7994 vs 8085 mixtures/s, round 3)
#ifndef BWD_EXP_NO_DG  // timing experiments only (results wrong): the BPTT without its dG stores
    store_dg();
#endif
    STAMP(6)
  }
  // fused bias gradients: this cell's sums over t, one plain store per (row, gate) into the
  // per-row partials (bias_reduce_kernel sums the rows in fixed order: deterministic)
  if (cval && a.dbpart) {
    float* pp = a.dbpart + (long long)(bg * 2 + d) * 2 * GH;
#pragma unroll
    for (int q = 0; q < NGATE; ++q) {
      pp[q * H + cj] = sbi[q];
      pp[GH + q * H + cj] = sbh[q];
    }
  } else if (cval) {
#pragma unroll
    for (int q = 0; q < NGATE; ++q) {
      if (a.dbi) atomicAdd(a.dbi + d * GH + q * H + cj, sbi[q]);
      if (a.dbh) atomicAdd(a.dbh + d * GH + q * H + cj, sbh[q]);
    }
  }
  STAMP_FLUSH
}

// compile-time (rows, k) per thread of the BPTT matvec: the shipped H = 300 plans
// (LSTM R=80: 20 x 3, GRU R=60: 20 x 2) and the generic (guard-free, zero-padded) maxima
void bwd_dims(int rpl, int kgl, int& rpln, int& kgln) {
  if ((rpl == 20 && kgl == 3) || (rpl == 20 && kgl == 2)) {
    rpln = rpl;
    kgln = kgl;
  } else {
    rpln = RPLMAX;
    kgln = KGLMAX;
  }
}

// CUs of the current device (cached per device id); 0 when no device is visible
int device_cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cache[dev] == 0) {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cache[dev] = cu;
  }
  return cache[dev];
}

// Launch-time guard of the co-residency assumption: the grid must not exceed the CUs times
// the kernel's occupancy at this LDS size (a persistent launch whose workgroups cannot all
// be resident would spin to the hand-off timeout on every step).
template <typename K>
bool fits_resident(K kernel, int grid, size_t smem) {
  struct Entry { const void* k; size_t smem; int dev; int occ; };
  static std::mutex mu;
  static Entry cache[64];
  static int n = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const void* kp = reinterpret_cast<const void*>(kernel);
  std::lock_guard<std::mutex> lk(mu);
  int occ = -1;
  for (int i = 0; i < n; ++i)
    if (cache[i].k == kp && cache[i].smem == smem && cache[i].dev == dev) occ = cache[i].occ;
  if (occ < 0) {
    occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, NT, smem) != hipSuccess) occ = 0;
    if (n < 64) cache[n++] = Entry{kp, smem, dev, occ};
  }
  return grid <= occ * device_cu_count();
}

struct Plan {
  int BC, NG, J, nchunk;
  int KP, KPL, HP, RP, RPL, KG, KGL;
  size_t smem_fwd, smem_bwd;        // fp32 VALU matvec
  size_t smem_fwd_mf, smem_bwd_mf;  // bf16 MFMA matvec
  bool fwd_pk;                       // packed hand-off forward (rnn_fwd_pk_kernel) applies
  size_t smem_fwd_pk;
  bool bwd_pk;                       // packed hand-off BPTT (rnn_bwd_pk_kernel) applies
  bool big;                          // H > HMAX: forward-only instantiations (HM = HMAX_L)
  size_t smem_bwd_pk;
};

// mf: plan for the bf16 MFMA matvec (the fp32 VALU forward's per-thread weight limit
// KPL <= WMAX does not apply).  H > HMAX is the forward-only large-H plan (HM = HMAX_L).
// Co-residency budget of one persistent launch (both directions, all batch chunks): every
// workgroup must be resident at once, so the plan keeps 2 * nchunk * NG within the device's
// CU count minus 1/16 of it (240 of 256 on a full MI355X; 30 on a 32-CU CPX partition),
// leaving room for concurrent kernels (RCCL).  DL4SS_RNN_MAX_WG overrides it (experiments).
int g_max_wg = 0;  // dl4ss_debug_set_rnn_max_wg (tests force the wider batch chunks)
int wg_limit() {
  if (g_max_wg > 0) return g_max_wg;
  static const int env = std::getenv("DL4SS_RNN_MAX_WG") ? std::atoi(std::getenv("DL4SS_RNN_MAX_WG")) : 0;
  if (env > 0) return env;
  const int cu = device_cu_count();
  return cu > 0 ? cu - cu / 16 : 240;
}

bool make_plan(int cell, int B, int H, Plan& p, bool mf = true, int max_wg = 0) {
  if (H > HMAX_L) return false;
  if (max_wg <= 0) max_wg = wg_limit();
  p.big = H > HMAX;
  const int ngate = cell == CELL_LSTM ? 4 : 3;
  for (int J = 20; J >= 4; --J) {
    const int R = ngate * J;
    if (R > NT) continue;
    const int KP = NT / R;
    int KPL = (H + KP - 1) / KP;
    KPL = (KPL + 3) / 4 * 4;
    if (KPL > WMAX && !mf) continue;
    // bwd: RP row parts x KG k-groups <= NT
    int best_rp = -1, best_kg = 0;
    for (int RP = 1; RP <= 16; ++RP) {
      const int RPL = (R + RP - 1) / RP;
      const int KG = NT / RP;
      const int KGL = (H + KG - 1) / KG;
      if (RPL <= RPLMAX && KGL <= KGLMAX) { best_rp = RP; best_kg = KG; break; }
    }
    if (best_rp < 0) continue;
    const int NG = (H + J - 1) / J;
    if (J > 20) continue;  // gather/publish offset arrays are sized for J <= 20, H <= HMAX(_L)
    int BC = 0;
    // DL4SS_RNN_MIN_BC (experiments): a wider batch chunk per group, fewer workgroups
    static const int min_bc = std::getenv("DL4SS_RNN_MIN_BC") ? std::atoi(std::getenv("DL4SS_RNN_MIN_BC")) : 1;
    for (int bc : {1, 2, 4, 8}) {
      if (bc < min_bc) continue;
      const int nchunk = (B + bc - 1) / bc;
      if (2 * nchunk * NG <= max_wg && bc * J <= NROLE) {
        BC = bc;
        break;
      }
    }
    if (!BC) continue;
    p.BC = BC; p.NG = NG; p.J = J; p.nchunk = (B + BC - 1) / BC;
    p.KP = KP; p.KPL = KPL; p.HP = KP * KPL;
    p.RP = best_rp; p.RPL = (R + best_rp - 1) / best_rp; p.KG = best_kg; p.KGL = (H + best_kg - 1) / best_kg;
    int rpln, kgln;
    bwd_dims(p.RPL, p.KGL, rpln, kgln);
    p.smem_fwd = sizeof(float) * (BC * p.HP + KP * BC * R + 2 * BC * J * 4);
    p.smem_bwd = sizeof(float) * (BC * p.RP * rpln + NG * BC * J + 3 + p.RP * BC * p.KG * kgln + 2 * BC * J * 8);
    const int SHB = (p.big ? HMAX_L : HMAX) + 8, MT = (R + 15) / 16, SDG = (4 * 20 + 31) / 32 * 32 + 8;
    p.smem_fwd_mf = 2 * 16 * SHB + sizeof(float) * (BC * MT * 16 + 2 * BC * J * 4);
    p.smem_bwd_mf = 2 * 16 * SDG + sizeof(float) * (NG * BC * J + 3 + BC * HMAX + 2 * BC * J * 8);
    p.fwd_pk = !p.big && J % 2 == 0 && H % 2 == 0 && J <= PKU && NG <= 16 && (R + 15) / 16 <= (FWD_NPW == 3 ? 5 : FWD_NPW == 2 ? 6 : 7);
    p.bwd_pk = !p.big && J % 4 == 0 && H % 4 == 0 && NG <= 16;
    p.smem_bwd_pk = 2 * 16 * SDG + sizeof(float) * (((16 * BC * J + 3) & ~3) + 4 * BC * ((HMAX / 16 + 3) / 4 * 16 + 4) +
                                                    2 * 2 * (BC * 32 * 4 + 16) + 2 * 7 * ((BC * 20 + 1) / 2));
    p.smem_fwd_pk = 2 * 16 * SHB + sizeof(float) * (BC * (MT * 16 + 4) + BC * 16 + 2 * sin_slab(BC)) + 2 * BC * PKU;
    return true;
  }
  return false;
}

// act layout of a plan: cell-major (B,T,2,H,4) when both packed kernels run it at BC >= 4 (the
// forward's one 16-B store per cell, the BPTT's one 16-B load; RnnArgs::act_cm), else gate-major
bool act_cell_major(const Plan& p) { return p.fwd_pk && p.bwd_pk && p.BC >= 4; }

// every persistent recurrence launch goes through the co-residency guard
template <typename K>
int launch_resident(K kernel, int grid, size_t smem, hipStream_t st, const RnnArgs& a) {
  if (!fits_resident(kernel, grid, smem)) return (int)hipErrorCooperativeLaunchTooLarge;
  RnnArgs arg = a;
  void* args[] = {&arg};
  return (int)hipLaunchKernel(reinterpret_cast<const void*>(kernel), dim3(grid), dim3(NT), args, smem, st);
}

// RNN_EXP_MINIMAL (experiment variant libraries only, tools/variant_lib.py --minimal): only the packed
// bf16 kernels at BC = 4 are instantiated -- the C2 / C4 training step at B = 32 -- so a variant of
// this file compiles in a fraction of the full build's time; every other plan fails its launch.
template <int CELL, int BC>
int launch_fwd(const RnnArgs& a, bool mf, bool pk, int grid, size_t smem, hipStream_t st) {
#ifdef RNN_EXP_MINIMAL
  if (BC != 4 || !mf || !pk) return (int)hipErrorNotSupported;
  if (a.Xb && a.Kin <= 5 * 32) return launch_resident(rnn_fwd_pk_kernel<CELL, 4, 5>, grid, smem, st, a);
  if (a.Xb) return launch_resident(rnn_fwd_pk_kernel<CELL, 4, XKMAX>, grid, smem, st, a);
  return launch_resident(rnn_fwd_pk_kernel<CELL, 4>, grid, smem, st, a);
#else
  if (a.H > HMAX) {  // forward-only large-H instantiations (the H = 600 classifier)
    if (mf)
      return launch_resident(rnn_fwd_kernel<CELL, BC, 0, true, HMAX_L>, grid, smem, st, a);
    else
      return launch_resident(rnn_fwd_kernel<CELL, BC, 0, false, HMAX_L>, grid, smem, st, a);
  }
  // compile-time k-slice lengths for the shipped H = 300 plans (LSTM J=20: 52, GRU J=20: 40)
  if (mf && pk && a.Xb && a.Kin <= 5 * 32)  // the nets' first layer: 129 features
    return launch_resident(rnn_fwd_pk_kernel<CELL, BC, 5>, grid, smem, st, a);
  if (mf && pk && a.Xb)
    return launch_resident(rnn_fwd_pk_kernel<CELL, BC, XKMAX>, grid, smem, st, a);
  if (mf && pk)
    return launch_resident(rnn_fwd_pk_kernel<CELL, BC>, grid, smem, st, a);
  else if (mf)
    return launch_resident(rnn_fwd_kernel<CELL, BC, 0, true>, grid, smem, st, a);
  else if (a.KPL == 52)
    return launch_resident(rnn_fwd_kernel<CELL, BC, 52, false>, grid, smem, st, a);
  else if (a.KPL == 40)
    return launch_resident(rnn_fwd_kernel<CELL, BC, 40, false>, grid, smem, st, a);
  else
    return launch_resident(rnn_fwd_kernel<CELL, BC, 0, false>, grid, smem, st, a);
#endif
}
template <int CELL, int BC>
int launch_bwd(const RnnArgs& a, bool mf, bool pk, int grid, size_t smem, hipStream_t st) {
  int rpln, kgln;
  bwd_dims(a.RPL, a.KGL, rpln, kgln);
#ifdef RNN_EXP_MINIMAL
  if (BC != 4 || !mf || !pk) return (int)hipErrorNotSupported;
#endif
  if constexpr (BC == 4) {  // the dH GEMM's split-K slabs summed by the top layer (DL4SS_RNN_DOUT_SLABS)
    if (mf && pk && a.dout_ns == 2) return launch_resident(rnn_bwd_pk_kernel<CELL, 4, 2>, grid, smem, st, a);
    if (mf && pk && a.dout_ns == 3) return launch_resident(rnn_bwd_pk_kernel<CELL, 4, 3>, grid, smem, st, a);
    if (mf && pk && a.dout_ns == 4) return launch_resident(rnn_bwd_pk_kernel<CELL, 4, 4>, grid, smem, st, a);
  }
#ifdef RNN_EXP_MINIMAL
  return launch_resident(rnn_bwd_pk_kernel<CELL, 4, 1>, grid, smem, st, a);
#else
  if (mf && pk)
    return launch_resident(rnn_bwd_pk_kernel<CELL, BC>, grid, smem, st, a);
  else if (mf)
    return launch_resident(rnn_bwd_kernel<CELL, BC, 0, 0, true>, grid, smem, st, a);
  else if (rpln == 20 && kgln == 3)
    return launch_resident(rnn_bwd_kernel<CELL, BC, 20, 3, false>, grid, smem, st, a);
  else if (rpln == 20 && kgln == 2)
    return launch_resident(rnn_bwd_kernel<CELL, BC, 20, 2, false>, grid, smem, st, a);
  else
    return launch_resident(rnn_bwd_kernel<CELL, BC, 0, 0, false>, grid, smem, st, a);
#endif
}

template <int CELL>
int dispatch(bool fwd, bool mf, bool pk, int BC, const RnnArgs& a, int grid, size_t smem, hipStream_t st) {
  int e;
  switch (BC) {
    case 1: e = fwd ? launch_fwd<CELL, 1>(a, mf, pk, grid, smem, st) : launch_bwd<CELL, 1>(a, mf, pk, grid, smem, st); break;
    case 2: e = fwd ? launch_fwd<CELL, 2>(a, mf, pk, grid, smem, st) : launch_bwd<CELL, 2>(a, mf, pk, grid, smem, st); break;
    case 4: e = fwd ? launch_fwd<CELL, 4>(a, mf, pk, grid, smem, st) : launch_bwd<CELL, 4>(a, mf, pk, grid, smem, st); break;
    case 8: e = fwd ? launch_fwd<CELL, 8>(a, mf, pk, grid, smem, st) : launch_bwd<CELL, 8>(a, mf, pk, grid, smem, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  if (e) return e;
  DL4SS_CHECK_LAUNCH();
  return 0;
}

#if defined(RNN_STAMPS) || defined(RNN_TRACE)
u64* g_stamps = nullptr;
#endif

unsigned g_spin_limit = SPIN_LIMIT;  // dl4ss_debug_set_spin_limit (tests force a hand-off timeout)
int g_place_force = 0;               // dl4ss_debug_set_place_force (tests force write-through granules)

void fill_args(RnnArgs& a, const Plan& p, int B, int T, int H) {
  a.spin_limit = g_spin_limit;
  a.place_force = g_place_force;
#if defined(RNN_STAMPS) || defined(RNN_TRACE)
  a.stamps = g_stamps;
#endif
  a.B = B; a.T = T; a.H = H; a.J = p.J; a.NG = p.NG; a.nchunk = p.nchunk;
  a.KP = p.KP; a.KPL = p.KPL; a.HP = p.HP;
  a.RP = p.RP; a.RPL = p.RPL; a.KG = p.KG; a.KGL = p.KGL;
}

}  // namespace

#if defined(RNN_STAMPS) || defined(RNN_TRACE)
DL4SS_API void dl4ss_debug_set_stamps(void* p) { g_stamps = reinterpret_cast<unsigned long long*>(p); }
#endif

// dbi[i] += sum_b part[b][d][0][g], dbh[i] += sum_b part[b][d][1][g] for i = d * GH + g, rows
// in order b = 0 .. B-1 (the BPTT kernel's per-row bias sums); blockIdx.y = the job (layer)
constexpr int BIAS_JOBS_MAX = 8;
struct BiasJobs {
  int n, B, GH;
  float beta;  // db = beta db + sums (beta 0: written, not read)
  const float* part[BIAS_JOBS_MAX];
  float* dbi[BIAS_JOBS_MAX];
  float* dbh[BIAS_JOBS_MAX];
};
__global__ __launch_bounds__(256) void bias_reduce_kernel(BiasJobs j) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int B = j.B, GH = j.GH;
  if (i >= 2 * GH) return;
  const float* part = j.part[0];
  float* dbi = j.dbi[0];
  float* dbh = j.dbh[0];
#pragma unroll
  for (int k = 1; k < BIAS_JOBS_MAX; ++k)
    if (k == (int)blockIdx.y) { part = j.part[k]; dbi = j.dbi[k]; dbh = j.dbh[k]; }
  const int d = i / GH, g = i - d * GH;
  float si = 0.0f, sh = 0.0f;
  // rows in chunks of 32 with every load of a chunk issued before its adds (a row-by-row
  // loop paid one dependent L2 round trip per row: 12 us per launch at B = 32; chunks of 8, four
  // rounds: 5.6 us; round 6: one round at B <= 32), the sums in row order
  for (int b0 = 0; b0 < B; b0 += 32) {
    float vi[32], vh[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int b = min(b0 + u, B - 1);
      const float* pp = part + (long long)(b * 2 + d) * 2 * GH + g;
      vi[u] = pp[0];
      vh[u] = pp[GH];
    }
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      si = b0 + u < B ? si + vi[u] : si;
      sh = b0 + u < B ? sh + vh[u] : sh;
    }
  }
  if (dbi) dbi[i] = j.beta != 0.f ? si + j.beta * dbi[i] : si;
  if (dbh) dbh[i] = j.beta != 0.f ? sh + j.beta * dbh[i] : sh;
}

// hand-off area of the BPTT / forward workspace, 256-B aligned
static long long handoff_bytes(const Plan& p, int H);

// per-row bias partials behind the hand-off area (BPTT with fused bias gradients)
static long long bias_part_bytes(const Plan& p, int H) {
  return p.big ? 0 : (long long)p.nchunk * p.BC * 2 * 2 * 4 * H * 4;
}

static long long workspace_bytes(const Plan& p, int H) { return handoff_bytes(p, H) + bias_part_bytes(p, H); }

static long long handoff_bytes(const Plan& p, int H) {
  const long long groups = 2LL * p.nchunk;
  long long fwd = groups * 2 * p.BC * H * 8;
  const long long fwd_pk = groups * 4 * p.BC * p.NG * 8 * 8;
  if (fwd_pk > fwd) fwd = fwd_pk;
  if (p.big) return fwd;  // forward only
  long long bwd = groups * 2 * p.NG * p.BC * H * 8;
  const long long bwd_pk = groups * 4LL * p.NG * p.BC * (((H + 1) / 2 + 1) & ~1) * 8;
  if (bwd_pk > bwd) bwd = bwd_pk;
  const long long n = fwd > bwd ? fwd : bwd;
  return (n + 255) / 256 * 256 + 256;  // + the group-formation counters (ctl_offset)
}

// the packed kernels' group-formation counters: the last 256 B of the hand-off area (group_pk)
static long long ctl_offset(const Plan& p, int H) { return handoff_bytes(p, H) - 256; }

// Polls a hand-off may spin before it times out (sets *status and the polling wave exits;
// the launch still completes).  0 restores the default (SPIN_LIMIT, ~1 s).  Test hook: a
// tiny limit forces the timeout path that the Adam guard (dl4ss_adam_guarded) must catch.
DL4SS_API void dl4ss_debug_set_spin_limit(unsigned limit) { g_spin_limit = limit ? limit : SPIN_LIMIT; }

// 1: the packed kernels write every granule through (`sc1`) as if the group spanned XCDs (test
// hook for the cross-XCD form); 0: plain stores wherever the group was found on one XCD.
DL4SS_API void dl4ss_debug_set_place_force(int force) { g_place_force = force == 1 ? 1 : 0; }

// > 0: the co-residency budget of every later plan (max_wg of dl4ss_birnn_plan_info, in
// workgroups) instead of the device's; 0 restores the default.  Test hook: a budget of 120 makes
// the B = 32, H = 300 nets plan batch chunks of 8 (the plan a B >= 33 batch gets on a full part).
DL4SS_API void dl4ss_debug_set_rnn_max_wg(int max_wg) { g_max_wg = max_wg > 0 ? max_wg : 0; }

// The recurrence plan for (cell, B, H) under a co-residency budget of max_wg workgroups
// (<= 0: the current device's, see wg_limit): info = {BC, NG, J, nchunk, grid}.  Host-only
// (no device call when max_wg > 0).  Returns 0, or hipErrorInvalidValue when no plan fits.
DL4SS_API int dl4ss_birnn_plan_info(int cell, int B, int H, int precision, int max_wg, int* info) {
  DL4SS_REQUIRE(info && (cell == CELL_LSTM || cell == CELL_GRU) && B > 0 && H > 0);
  Plan p;
  if (!make_plan(cell, B, H, p, precision == 1, max_wg)) return (int)hipErrorInvalidValue;
  info[0] = p.BC; info[1] = p.NG; info[2] = p.J; info[3] = p.nchunk; info[4] = 2 * p.nchunk * p.NG;
  return 0;
}

// Sub-batch of a forward whose plan does not fit the co-residency budget at B: the fp32 VALU
// plan of a wide layer (H = 600, the classifier: J <= 12, 50 workgroups per group) fits at most
// B = 16 on a full part.  Rows never interact, so dl4ss_birnn_fwd_mean runs such a batch as
// consecutive launches of (near-)equal sub-batches.  0 when no sub-batch fits either.
static int split_batch(int cell, int B, int H, bool mf, Plan& ps) {
  int fit = 0;
  for (int b = B - 1; b >= 1 && !fit; --b)
    if (make_plan(cell, b, H, ps, mf)) fit = b;
  if (!fit) return 0;
  const int n = (B + fit - 1) / fit;
  const int bs = (B + n - 1) / n;
  return make_plan(cell, bs, H, ps, mf) ? bs : 0;
}

// the larger of the fp32 and bf16 plans' needs (either precision may use the buffer; an fp32
// forward planned as sub-batches counts its sub-batch plan); -1 when neither plan exists
DL4SS_API long long dl4ss_birnn_workspace_bytes(int cell, int B, int H) {
  long long best = -1;
  for (bool mf : {false, true}) {
    Plan p;
    if (!make_plan(cell, B, H, p, mf) && (mf || split_batch(cell, B, H, mf, p) == 0)) continue;
    const long long n = workspace_bytes(p, H);
    if (n > best) best = n;
  }
  return best;
}

DL4SS_API int dl4ss_birnn_fwd_ex(int cell, int precision, int B, int T, int H, const float* G, const float* W_hh,
                                 const float* b_hh, float* out, float* hprev, float* act, float* cs, void* out_bf16,
                                 void* hprev_bf16, void* workspace, long long ws_bytes, int* status, void* stream);

DL4SS_API int dl4ss_birnn_fwd(int cell, int precision, int B, int T, int H, const float* G, const float* W_hh, const float* b_hh,
                              float* out, float* hprev, float* act, float* cs, void* workspace,
                              long long ws_bytes, int* status, void* stream) {
  DL4SS_REQUIRE(hprev);
  return dl4ss_birnn_fwd_ex(cell, precision, B, T, H, G, W_hh, b_hh, out, hprev, act, cs, nullptr, nullptr, workspace,
                            ws_bytes, status, stream);
}

DL4SS_API int dl4ss_birnn_fwd_mean(int cell, int precision, int B, int T, int H, const float* G, const float* W_hh,
                                   const float* b_hh, float* out, float* hprev, float* act, float* cs, void* out_bf16,
                                   void* hprev_bf16, float* h_mean, void* workspace, long long ws_bytes, int* status,
                                   void* stream);

DL4SS_API int dl4ss_birnn_fwd_ex(int cell, int precision, int B, int T, int H, const float* G, const float* W_hh,
                                 const float* b_hh, float* out, float* hprev, float* act, float* cs, void* out_bf16,
                                 void* hprev_bf16, void* workspace, long long ws_bytes, int* status, void* stream) {
  DL4SS_REQUIRE(out);
  return dl4ss_birnn_fwd_mean(cell, precision, B, T, H, G, W_hh, b_hh, out, hprev, act, cs, out_bf16, hprev_bf16,
                              nullptr, workspace, ws_bytes, status, stream);
}

// dl4ss_birnn_fwd_ex with the fp32 output optional (packed kernel: out may be NULL when out_bf16 is
// not) and the time mean of the output formed in the recurrence (h_mean, packed kernel only)
DL4SS_API int dl4ss_birnn_fwd_mean(int cell, int precision, int B, int T, int H, const float* G, const float* W_hh,
                                   const float* b_hh, float* out, float* hprev, float* act, float* cs, void* out_bf16,
                                   void* hprev_bf16, float* h_mean, void* workspace, long long ws_bytes, int* status,
                                   void* stream) {
  DL4SS_REQUIRE(cell == CELL_LSTM || cell == CELL_GRU);
  const bool prezeroed = precision & DL4SS_RNN_WS_ZEROED;  // the caller zeroed the workspace (one fill per step)
  precision &= ~DL4SS_RNN_WS_ZEROED;
  DL4SS_REQUIRE(precision == 0 || precision == 1);
  DL4SS_REQUIRE(B > 0 && T > 0 && H > 0 && G && W_hh && b_hh && (out || out_bf16) && act && workspace && status);
  DL4SS_REQUIRE(cell == CELL_GRU || cs);
  Plan p;
  if (precision == 0 && !make_plan(cell, B, H, p, false)) {
    // the fp32 plan does not fit at this batch: consecutive sub-batch launches (split_batch),
    // each zeroing the shared hand-off workspace itself (stream order keeps them apart)
    const int bs = split_batch(cell, B, H, false, p);
    DL4SS_REQUIRE(bs > 0 && out && !h_mean && !out_bf16 && !hprev_bf16);
    const long long GH = (cell == CELL_LSTM ? 4LL : 3LL) * H;
    for (int b0 = 0; b0 < B; b0 += bs) {
      const long long r = (long long)b0 * T;  // (b, t) rows before the sub-batch
      const int rc = dl4ss_birnn_fwd_mean(cell, 0, B - b0 < bs ? B - b0 : bs, T, H, G + r * 2 * GH, W_hh, b_hh,
                                          out + r * 2 * H, hprev ? hprev + r * 2 * H : nullptr, act + r * 2 * 4 * H,
                                          cs ? cs + r * 2 * H : nullptr, nullptr, nullptr, nullptr, workspace,
                                          ws_bytes, status, stream);
      if (rc) return rc;
    }
    return 0;
  }
  DL4SS_REQUIRE(make_plan(cell, B, H, p, precision == 1));
  DL4SS_REQUIRE(ws_bytes >= workspace_bytes(p, H));
  hipStream_t st = as_stream(stream);
  const long long groups = 2LL * p.nchunk;
  const bool mf = precision == 1;
  const bool pk = mf && p.fwd_pk && T < 65535;
  const bool act_cm = pk && act_cell_major(p);
  DL4SS_REQUIRE(pk || (out && !h_mean));  // the optional output and the fused mean are the packed kernel's
  if (!prezeroed) {
    hipError_t e = hipMemsetAsync(workspace, 0, pk ? groups * 4 * p.BC * p.NG * 8 * 8 : groups * 2 * p.BC * H * 8, st);
    if (e == hipSuccess && pk) e = hipMemsetAsync(static_cast<char*>(workspace) + ctl_offset(p, H), 0, 256, st);
    if (e != hipSuccess) return (int)e;
  }
  // the bf16 copies, and dropping the fp32 h_{t-1} (only the GRU BPTT reads it), need the packed kernel
  DL4SS_REQUIRE(pk || (!out_bf16 && !hprev_bf16 && hprev));
  DL4SS_REQUIRE(hprev || cell == CELL_LSTM);
  RnnArgs a{};
  fill_args(a, p, B, T, H);
  a.G = G; a.Whh = W_hh; a.bhh = b_hh; a.out = out; a.hprev = hprev; a.act = act; a.cs = cs;
  a.act_cm = act_cm ? 1 : 0;
  a.hmean = h_mean;
  a.outb = reinterpret_cast<unsigned short*>(out_bf16);
  a.hprevb = reinterpret_cast<unsigned short*>(hprev_bf16);
  a.xbuf = reinterpret_cast<unsigned long long*>(workspace);
  a.gctl = pk ? reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + ctl_offset(p, H)) : nullptr;
  a.status = status;
  const int grid = (int)(groups * p.NG);
  const size_t smem = pk ? p.smem_fwd_pk : mf ? p.smem_fwd_mf : p.smem_fwd;
  return cell == CELL_LSTM ? dispatch<CELL_LSTM>(true, mf, pk, p.BC, a, grid, smem, st)
                           : dispatch<CELL_GRU>(true, mf, pk, p.BC, a, grid, smem, st);
}

// 1 when the packed bf16 forward (the only one with the fused input projection) applies to
// (cell, B, H, T) and the layer input width Kin: dl4ss_birnn_fwd_xw may be called
DL4SS_API int dl4ss_birnn_fwd_xw_supported(int cell, int B, int T, int H, int Kin) {
  if (!(cell == CELL_LSTM || cell == CELL_GRU) || B <= 0 || T <= 0 || H <= 0 || Kin <= 0) return 0;
  Plan p;
  if (!make_plan(cell, B, H, p, true)) return 0;
  // at most 5 MFMA tiles (R <= 80 gate rows): prefetch wave 6 then holds no matvec tile and wave 5
  // one projection tile, the compile-time roles of rnn_fwd_pk_kernel's prefetch branch
  const int ngate = cell == CELL_LSTM ? 4 : 3;
  return (p.fwd_pk && T < 65535 && Kin <= XKMAX * 32 && (ngate * p.J + 15) / 16 <= 5) ? 1 : 0;
}

// dl4ss_birnn_fwd_ex with the input projection fused into the recurrence (bf16 mode only): instead
// of reading G = X W_ih^T + b_ih from a separate GEMM, every workgroup forms its own gate rows of
// step t+1 with MFMAs while step t's hand-off travels.  x_bf16: (B*T, ldx) bf16 layer input rows
// (16-B chunks: padding up to the next multiple of 8 finite); W_ih_bf16: (2*NGATE*H, ldw) bf16 (direction-major rows, the GEMM's B operand); b_ih
// (2, NGATE*H) fp32.  ldx, ldw multiples of 8 and both bases 16-B aligned.  Same summation order as
// the GEMM path (one k-ordered MFMA chain, then + b_ih): the outputs match it bit for bit.
DL4SS_API int dl4ss_birnn_fwd_xw_ex(int cell, int B, int T, int H, const void* x_bf16, int Kin, long long ldx,
                                    const void* W_ih_bf16, long long ldw, const float* b_ih, const float* W_hh,
                                    const float* b_hh, float* out, float* hprev, float* act, float* cs,
                                    void* out_bf16, void* hprev_bf16, float* h_mean, void* workspace,
                                    long long ws_bytes, int* status, void* stream, int ws_zeroed);

DL4SS_API int dl4ss_birnn_fwd_xw(int cell, int B, int T, int H, const void* x_bf16, int Kin, long long ldx,
                                 const void* W_ih_bf16, long long ldw, const float* b_ih, const float* W_hh,
                                 const float* b_hh, float* out, float* hprev, float* act, float* cs, void* out_bf16,
                                 void* hprev_bf16, void* workspace, long long ws_bytes, int* status, void* stream,
                                 int ws_zeroed) {
  DL4SS_REQUIRE(out);
  return dl4ss_birnn_fwd_xw_ex(cell, B, T, H, x_bf16, Kin, ldx, W_ih_bf16, ldw, b_ih, W_hh, b_hh, out, hprev, act, cs,
                               out_bf16, hprev_bf16, nullptr, workspace, ws_bytes, status, stream, ws_zeroed);
}

DL4SS_API int dl4ss_birnn_fwd_xw_ex(int cell, int B, int T, int H, const void* x_bf16, int Kin, long long ldx,
                                    const void* W_ih_bf16, long long ldw, const float* b_ih, const float* W_hh,
                                    const float* b_hh, float* out, float* hprev, float* act, float* cs,
                                    void* out_bf16, void* hprev_bf16, float* h_mean, void* workspace,
                                    long long ws_bytes, int* status, void* stream, int ws_zeroed) {
  DL4SS_REQUIRE(dl4ss_birnn_fwd_xw_supported(cell, B, T, H, Kin));
  DL4SS_REQUIRE(x_bf16 && W_ih_bf16 && b_ih && W_hh && b_hh && act && workspace && status);
  DL4SS_REQUIRE(out || out_bf16);  // some output of the layer
  DL4SS_REQUIRE(cell == CELL_GRU || cs);
  DL4SS_REQUIRE(hprev || cell == CELL_LSTM);
  DL4SS_REQUIRE(ldx >= Kin && ldw >= Kin && ldx % 8 == 0 && ldw % 8 == 0);
  DL4SS_REQUIRE((reinterpret_cast<uintptr_t>(x_bf16) & 15) == 0 && (reinterpret_cast<uintptr_t>(W_ih_bf16) & 15) == 0);
  Plan p;
  DL4SS_REQUIRE(make_plan(cell, B, H, p, true));
  DL4SS_REQUIRE(ws_bytes >= workspace_bytes(p, H));
  hipStream_t st = as_stream(stream);
  const long long groups = 2LL * p.nchunk;
  if (!ws_zeroed) {
    hipError_t e = hipMemsetAsync(workspace, 0, groups * 4 * p.BC * p.NG * 8 * 8, st);
    if (e == hipSuccess) e = hipMemsetAsync(static_cast<char*>(workspace) + ctl_offset(p, H), 0, 256, st);
    if (e != hipSuccess) return (int)e;
  }
  RnnArgs a{};
  fill_args(a, p, B, T, H);
  a.G = nullptr; a.Whh = W_hh; a.bhh = b_hh; a.out = out; a.hprev = hprev; a.act = act; a.cs = cs;
  a.act_cm = act_cell_major(p) ? 1 : 0;
  a.hmean = h_mean;
  a.outb = reinterpret_cast<unsigned short*>(out_bf16);
  a.hprevb = reinterpret_cast<unsigned short*>(hprev_bf16);
  a.xbuf = reinterpret_cast<unsigned long long*>(workspace);
  a.gctl = reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + ctl_offset(p, H));
  a.status = status;
  a.Xb = reinterpret_cast<const unsigned short*>(x_bf16);
  a.Wihb = reinterpret_cast<const unsigned short*>(W_ih_bf16);
  a.bih = b_ih;
  a.Kin = Kin; a.ldx = ldx; a.ldw = ldw;
  const int grid = (int)(groups * p.NG);
  // + the per-step projections of two blocks instead of two steps, + 256: the ring starts at the
  // next 256-B boundary of the LDS address (bank order of its rows)
  const size_t smem = p.smem_fwd_pk + sizeof(float) * (2 * xw_spb(p.BC) - 2) * sin_slab(p.BC) + 256 +
                      (size_t)xw_ring_bf16(p.BC) * sizeof(unsigned short);
  return cell == CELL_LSTM ? dispatch<CELL_LSTM>(true, true, true, p.BC, a, grid, smem, st)
                           : dispatch<CELL_GRU>(true, true, true, p.BC, a, grid, smem, st);
}

DL4SS_API int dl4ss_birnn_bwd_ex(int cell, int precision, int B, int T, int H, const float* dOut,
                                 const float* dOut_bcast, const float* W_hh, const float* act, const float* cs,
                                 const float* hprev, float* dG, float* dGh, void* dG_bf16, void* dGh_bf16,
                                 float* db_ih, float* db_hh, void* workspace, long long ws_bytes, int* status,
                                 void* stream);

DL4SS_API int dl4ss_birnn_bwd(int cell, int precision, int B, int T, int H, const float* dOut, const float* dOut_bcast,
                              const float* W_hh, const float* act, const float* cs, const float* hprev, float* dG,
                              float* dGh, void* workspace, long long ws_bytes, int* status, void* stream) {
  DL4SS_REQUIRE(dG && (cell == CELL_LSTM || dGh));
  return dl4ss_birnn_bwd_ex(cell, precision, B, T, H, dOut, dOut_bcast, W_hh, act, cs, hprev, dG, dGh, nullptr,
                            nullptr, nullptr, nullptr, workspace, ws_bytes, status, stream);
}

DL4SS_API int dl4ss_birnn_bwd_ex(int cell, int precision, int B, int T, int H, const float* dOut,
                                 const float* dOut_bcast, const float* W_hh, const float* act, const float* cs,
                                 const float* hprev, float* dG, float* dGh, void* dG_bf16, void* dGh_bf16,
                                 float* db_ih, float* db_hh, void* workspace, long long ws_bytes, int* status,
                                 void* stream) {
  DL4SS_REQUIRE(cell == CELL_LSTM || cell == CELL_GRU);
  const bool prezeroed = precision & DL4SS_RNN_WS_ZEROED;
  const bool dgh_pad8 = precision & DL4SS_RNN_DGH_PAD8;
  const bool defer_bias = precision & DL4SS_RNN_DEFER_BIAS;
  const int dout_ns = ((precision & DL4SS_RNN_DOUT_SLABS_MASK) >> 12) + 1;
  precision &= ~(DL4SS_RNN_WS_ZEROED | DL4SS_RNN_DGH_PAD8 | DL4SS_RNN_DEFER_BIAS | DL4SS_RNN_DOUT_SLABS_MASK);
  DL4SS_REQUIRE(precision == 0 || precision == 1);
  DL4SS_REQUIRE(B > 0 && T > 0 && H > 0 && dOut && W_hh && act && workspace && status);
  DL4SS_REQUIRE(dG || dG_bf16);
  DL4SS_REQUIRE(cell == CELL_GRU ? ((dGh || dGh_bf16) && hprev) : (cs != nullptr));
  DL4SS_REQUIRE(H <= HMAX);  // BPTT is built for the mask nets (H <= 320); the large-H plan is forward only
  Plan p;
  DL4SS_REQUIRE(make_plan(cell, B, H, p, precision == 1));
  DL4SS_REQUIRE(ws_bytes >= workspace_bytes(p, H));
  hipStream_t st = as_stream(stream);
  const long long groups = 2LL * p.nchunk;
  const bool mf = precision == 1;
  // the packed BPTT at BC >= 4 reads the cell-major act that only the packed forward writes
  const bool pk = mf && p.bwd_pk && T < 65535 && (p.BC < 4 || act_cell_major(p));
  const long long HG = ((H + 1) / 2 + 1) & ~1;
  if (!prezeroed) {
    hipError_t e =
        hipMemsetAsync(workspace, 0, pk ? groups * 4 * p.NG * p.BC * HG * 8 : groups * 2 * p.NG * p.BC * H * 8, st);
    if (e == hipSuccess && pk) e = hipMemsetAsync(static_cast<char*>(workspace) + ctl_offset(p, H), 0, 256, st);
    if (e != hipSuccess) return (int)e;
  }
  // bf16 gradient copies, dropping the fp32 ones and the fused bias sums need the packed kernel
  DL4SS_REQUIRE(pk || (!dG_bf16 && !dGh_bf16 && !db_ih && !db_hh && dG && (cell == CELL_LSTM || dGh)));
  // split-K dOut slabs: the packed BPTT's step-factor prefetch at batch chunks of 4 sums them
  DL4SS_REQUIRE(dout_ns == 1 || (pk && p.BC == 4));
  RnnArgs a{};
  fill_args(a, p, B, T, H);
  a.Whh = W_hh; a.act = const_cast<float*>(act); a.cs = const_cast<float*>(cs);
  a.hprev = const_cast<float*>(hprev); a.dOut = dOut; a.dOutB = dOut_bcast; a.dG = dG; a.dGh = dGh;
  a.dout_ns = dout_ns;
  a.dout_zs = (long long)B * T * 2 * H;
#ifdef DL4SS_EXP_ZS_PAD
  if (const char* e = getenv("DL4SS_EXP_ZS_PAD")) a.dout_zs += atoll(e);  // probe builds only
#endif
  a.dGb = reinterpret_cast<unsigned short*>(dG_bf16); a.dGhb = reinterpret_cast<unsigned short*>(dGh_bf16);
  const int GHc = (cell == CELL_LSTM ? 4 : 3) * H;
  a.ghb = dgh_pad8 ? (GHc + 7) / 8 * 8 : GHc;
  a.dbi = db_ih; a.dbh = db_hh;
  a.xbuf = reinterpret_cast<unsigned long long*>(workspace);
  a.gctl = pk ? reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + ctl_offset(p, H)) : nullptr;
  const bool bias = pk && (db_ih || db_hh);
  a.dbpart = bias ? reinterpret_cast<float*>(static_cast<char*>(workspace) + handoff_bytes(p, H)) : nullptr;
  a.status = status;
  const int grid = (int)(groups * p.NG);
  const size_t smem = pk ? p.smem_bwd_pk : mf ? p.smem_bwd_mf : p.smem_bwd;
  const int e = cell == CELL_LSTM ? dispatch<CELL_LSTM>(false, mf, pk, p.BC, a, grid, smem, st)
                                  : dispatch<CELL_GRU>(false, mf, pk, p.BC, a, grid, smem, st);
  if (e || !bias || defer_bias) return e;
  const int GH = (cell == CELL_LSTM ? 4 : 3) * H;
  BiasJobs j{};
  j.n = 1; j.B = B; j.GH = GH; j.beta = 1.f; j.part[0] = a.dbpart; j.dbi[0] = db_ih; j.dbh[0] = db_hh;
  hipLaunchKernelGGL(bias_reduce_kernel, dim3((2 * GH + 255) / 256, 1), dim3(256), 0, st, j);
  return (int)hipGetLastError();
}

// The deferred form: the bias partials of n BPTT launches (DL4SS_RNN_DEFER_BIAS) reduced by ONE
// launch after the last of them -- the per-layer reduce was a 5 us latency-bound launch between
// each BPTT and the input-gradient GEMM that the next BPTT waits on.
DL4SS_API int dl4ss_birnn_bias_reduce_ex(int cell, int B, int H, int n, void* const* workspaces,
                                         float* const* db_ih, float* const* db_hh, float beta, void* stream) {
  DL4SS_REQUIRE((cell == CELL_LSTM || cell == CELL_GRU) && B > 0 && H > 0 && n >= 1 && n <= BIAS_JOBS_MAX);
  DL4SS_REQUIRE(workspaces && db_ih && db_hh);
  Plan p;
  if (!make_plan(cell, B, H, p, true)) return (int)hipErrorInvalidValue;  // the bf16 BPTT's plan
  const int GH = (cell == CELL_LSTM ? 4 : 3) * H;
  BiasJobs j{};
  j.n = n; j.B = B; j.GH = GH; j.beta = beta;
  for (int i = 0; i < n; ++i) {
    DL4SS_REQUIRE(workspaces[i] && db_ih[i] && db_hh[i]);
    j.part[i] = reinterpret_cast<const float*>(static_cast<const char*>(workspaces[i]) + handoff_bytes(p, H));
    j.dbi[i] = db_ih[i];
    j.dbh[i] = db_hh[i];
  }
  hipLaunchKernelGGL(bias_reduce_kernel, dim3((2 * GH + 255) / 256, n), dim3(256), 0, as_stream(stream), j);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_birnn_bias_reduce(int cell, int B, int H, int n, void* const* workspaces, float* const* db_ih,
                                      float* const* db_hh, void* stream) {
  return dl4ss_birnn_bias_reduce_ex(cell, B, H, n, workspaces, db_ih, db_hh, 1.f, stream);
}
