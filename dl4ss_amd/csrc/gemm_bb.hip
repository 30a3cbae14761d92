// bf16-operand MFMA GEMM: C[M,N] (fp32) (+)= op(A) . op(B) (+ bias) (tanh), with
// A and B already bf16 in HBM (the throughput path of the separation step).
//
// In bf16 mode every GEMM operand of the step is rounded to bf16 before the MFMA
// anyway (gemm.hip rounds fp32 operands at the LDS store).  Here the PRODUCERS
// write the bf16 copy (the BiRNN kernels write bf16 h / h_{t-1} / dG, the
// attention kernel bf16 dPre, dl4ss_f32_to_bf16 the weights and the layer-0
// features), so the products are bit-identical to gemm.hip's bf16 mode while the
// operand bytes halve and no conversion sits in the load path.
//
// Tile 128 x 128 x 64, 256 threads = 4 waves in 2 x 2, each wave 64 x 64 =
// 2 x 2 v_mfma_f32_32x32x16_bf16 accumulators.  Staging: every thread moves one
// 8 x 8 bf16 block per k-tile (threads 0-127 of A, 128-255 of B): 8 x 16-B global
// loads, and for a k-major operand (element (r,k) at G[k*ld + r]: the transposed
// side of the weight gradients) an 8 x 8 16-bit transpose in registers
// (v_perm_b32), then 8 x 16-B LDS stores into the [row][k] image (row stride 72
// bf16 = 144 B: conflict-free ds_read_b128 fragments).  Pipeline: two LDS
// buffers + a ring of three register blocks, so each k-tile's global loads are in
// flight for two k-tiles of MFMAs before they are stored to LDS.
// Tiles are mapped XCD-major and grouped (8 M-tiles x all N-tiles), as gemm.hip.
// Split-K (grid.z) accumulates with fp32 atomics into C (weight gradients).
#include "common.h"
#include <hip/hip_bf16.h>

namespace {

constexpr int BK = 64, LDK = BK + 8;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
enum { EPI_NONE = 0, EPI_TANH = 1, EPI_TANH_BF16 = 2 };  // 2: tanh, C written as bf16 (raw 16-bit words)

// tanh for the Linear epilogue: 1 - 2 / (1 + e^{2x}) with v_exp + v_rcp (~1e-6 relative;
// saturates cleanly: e^{2x} -> inf gives 1, -> 0 gives -1)
__device__ __forceinline__ float ftanh_fast(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x)); }

// One 8 x 8 block of one operand tile, staged in v[8] (16 B each).  KC: element (r,k)
// at G[r*ld + k] (k contiguous); !KC: at G[k*ld + r].  Block (rb, kb): rows 8rb..+8,
// k 8kb..+8.  Block index bi (tile of ROWS rows): KC -> rb = bi >> 3, kb = bi & 7 (a
// wave's 8 lanes of one rb read 128 contiguous bytes); !KC -> kb = bi / (ROWS/8),
// rb = bi % (ROWS/8) (ROWS/8 lanes of one k-row read 2 ROWS contiguous bytes).
template <bool KC, int ROWS>
__device__ __forceinline__ void block_coords(int bi, int& rb, int& kb) {
  if (KC) { rb = bi >> 3; kb = bi & 7; }
  else { kb = bi / (ROWS / 8); rb = bi % (ROWS / 8); }
}

// mask of dword i of a 16-B chunk whose first n elements (of 8) are valid
__device__ __forceinline__ unsigned chunk_mask(int i, int n) {
  return 2 * i + 1 < n ? 0xFFFFFFFFu : (2 * i < n ? 0x0000FFFFu : 0u);
}

// VEC: every row of the operand is 16-B aligned (ld % 8 == 0, aligned base), so a chunk
// that starts inside the matrix never leaves its row: the eight 16-B loads are issued
// unconditionally (out-of-range rows / k-rows re-read a valid address) and masked
// afterwards -- straight-line code, so the compiler keeps them all in flight.
template <bool KC, bool VEC>
__device__ __forceinline__ void load_block(uint4 (&v)[8], const unsigned short* __restrict__ G, long long ld, int r0,
                                           int rmax, int k0, int kmax, int rb, int kb) {
  if constexpr (VEC) {
    if (KC) {
      const int gk = k0 + 8 * kb;
      const int nk = max(0, min(8, kmax - gk));
      const int gkc = nk > 0 ? gk : 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int gr = r0 + 8 * rb + j;
        const bool rok = gr < rmax;
        v[j] = *reinterpret_cast<const uint4*>(G + (long long)(rok ? gr : 0) * ld + gkc);
        const int n = rok ? nk : 0;
        v[j].x &= chunk_mask(0, n); v[j].y &= chunk_mask(1, n); v[j].z &= chunk_mask(2, n); v[j].w &= chunk_mask(3, n);
      }
    } else {
      const int gr = r0 + 8 * rb;
      const int nr = max(0, min(8, rmax - gr));
      const int grc = nr > 0 ? gr : 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int gk = k0 + 8 * kb + j;
        const bool kok = gk < kmax;
        v[j] = *reinterpret_cast<const uint4*>(G + (long long)(kok ? gk : 0) * ld + grc);
        const int n = kok ? nr : 0;
        v[j].x &= chunk_mask(0, n); v[j].y &= chunk_mask(1, n); v[j].z &= chunk_mask(2, n); v[j].w &= chunk_mask(3, n);
      }
    }
  } else {  // unaligned rows: element-wise (correct, slow; producers pad rows to avoid it)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gr = KC ? r0 + 8 * rb + j : r0 + 8 * rb;
      const int gk = KC ? k0 + 8 * kb : k0 + 8 * kb + j;
      const unsigned short* p = KC ? G + (long long)gr * ld + gk : G + (long long)gk * ld + gr;
      unsigned e[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const bool in = KC ? (gr < rmax && gk + c < kmax) : (gk < kmax && gr + c < rmax);
        e[c] = in ? p[c] : 0u;
      }
      v[j] = make_uint4(e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16));
    }
  }
}

// write the block into the [row][k] LDS image (k-major blocks are transposed 8 x 8 in
// registers: v[k] holds r = 0..7 of k-row k, two per dword)
template <bool KC>
__device__ __forceinline__ void store_block(const uint4 (&v)[8], unsigned short* __restrict__ s, int rb, int kb) {
  if (KC) {
#pragma unroll
    for (int j = 0; j < 8; ++j) *reinterpret_cast<uint4*>(s + (8 * rb + j) * LDK + 8 * kb) = v[j];
  } else {
    const unsigned* w = reinterpret_cast<const unsigned*>(v);  // w[4k + r/2]
#pragma unroll
    for (int r2 = 0; r2 < 4; ++r2) {
      // v_perm_b32 selectors: 0x05040100 = lo16(src1) | lo16(src0) << 16 (even row 2 r2),
      //                       0x07060302 = hi16(src1) | hi16(src0) << 16 (odd row 2 r2 + 1)
      uint4 ev, od;
      ev.x = __builtin_amdgcn_perm(w[4 * 1 + r2], w[4 * 0 + r2], 0x05040100u);
      ev.y = __builtin_amdgcn_perm(w[4 * 3 + r2], w[4 * 2 + r2], 0x05040100u);
      ev.z = __builtin_amdgcn_perm(w[4 * 5 + r2], w[4 * 4 + r2], 0x05040100u);
      ev.w = __builtin_amdgcn_perm(w[4 * 7 + r2], w[4 * 6 + r2], 0x05040100u);
      od.x = __builtin_amdgcn_perm(w[4 * 1 + r2], w[4 * 0 + r2], 0x07060302u);
      od.y = __builtin_amdgcn_perm(w[4 * 3 + r2], w[4 * 2 + r2], 0x07060302u);
      od.z = __builtin_amdgcn_perm(w[4 * 5 + r2], w[4 * 4 + r2], 0x07060302u);
      od.w = __builtin_amdgcn_perm(w[4 * 7 + r2], w[4 * 6 + r2], 0x07060302u);
      *reinterpret_cast<uint4*>(s + (8 * rb + 2 * r2) * LDK + 8 * kb) = ev;
      *reinterpret_cast<uint4*>(s + (8 * rb + 2 * r2 + 1) * LDK + 8 * kb) = od;
    }
  }
}

// Tile configurations (all k-tiles BK = 64, waves of WM x WN = (WM/32) x (WN/32)
// v_mfma_f32_32x32x16_bf16 blocks, WN = 64):
//   TILE_128x128: 4 waves (64 x 64 each), 256 threads, 2 workgroups per CU (73.7 KB LDS)
//   TILE_256x128: 8 waves (64 x 64 each), 512 threads, 1 per CU (110.6 KB)
//   TILE_256x256: 8 waves (128 x 64 each), 512 threads, 1 per CU (147.5 KB)
// The larger tiles halve (256x256) or cut by a quarter (256x128) the operand bytes per
// MFMA that every workgroup pulls through L2 -- the 128 x 128 tile needs ~2x the per-CU
// L2 bandwidth at full MFMA rate.  Staging: threads [0, BM) stage A blocks, [BM, BM+BN)
// B blocks, the rest (256x128: 128 threads) only run MFMAs; all share the barriers.
#ifndef GBB_NS
#define GBB_NS 3  // k-tiles in flight per staging thread, 256-thread tiles
#endif
template <int BM_, int BN_, int WM_, int WN_>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int TI = WM / 32, TJ = WN / 32;
  static constexpr int WAVES_N = BN / WN;
  static constexpr int NT = (BM / WM) * (BN / WN) * 64;
  static constexpr int NS = TI * TJ > 4 ? 2 : GBB_NS;  // register ring depth (VGPR budget at 512 threads)
  static_assert(WN == 64, "the epilogue maps 16 lanes x 4 columns onto a 64-wide wave tile");
};
typedef Tile<128, 128, 64, 64> T128x128;
typedef Tile<256, 128, 64, 64> T256x128;
typedef Tile<256, 256, 128, 64> T256x256;

// The k-loop of one staging role: this thread stages blocks of ONE operand (KC layout,
// ROWS-row tile) -- or none (STAGE false) -- and all threads run the same MFMAs and
// barriers.  Hoisting the (wave-uniform) role out of the loop keeps each loop's loads
// straight-line code.
template <class TC, bool STAGE, bool KC, bool VEC, int ROWS>
__device__ __forceinline__ void kloop(f32x16 (&acc)[TC::TI][TC::TJ], const unsigned short* __restrict__ G, long long ld,
                                      int r0, int rmax, int kbeg, int kend, unsigned short* sOwn,
                                      const unsigned short* sA, const unsigned short* sB, int bi, int lane, int wm,
                                      int wn) {
  constexpr int NS = TC::NS;  // register ring: loads of k-tiles kt+1 .. kt+NS-1 in flight during tile kt
  constexpr int BUF_A = TC::BM * LDK, BUF_B = TC::BN * LDK, BUF_OWN = ROWS * LDK;
  uint4 v[NS][8];
  int rb = 0, kb = 0;
  block_coords<KC, ROWS>(bi, rb, kb);
  const int nk = (kend - kbeg + BK - 1) / BK;
  if constexpr (STAGE) {
#pragma unroll
    for (int u = 0; u < NS; ++u)
      if (u < nk) load_block<KC, VEC>(v[u], G, ld, r0, rmax, kbeg + u * BK, kend, rb, kb);
    store_block<KC>(v[0], sOwn, rb, kb);
  }
  __syncthreads();
  const int fr = lane & 31, fk = 8 * (lane >> 5);
  for (int kt0 = 0; kt0 < nk; kt0 += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int kt = kt0 + u;
      if (kt < nk) {
        const int cur = kt & 1;
        const unsigned short* a = sA + cur * BUF_A;
        const unsigned short* b = sB + cur * BUF_B;
#ifndef GBB_NO_MFMA
#pragma unroll
        for (int kk = 0; kk < BK; kk += 16) {
          bf16x8 af[TC::TI], bfr[TC::TJ];
#pragma unroll
          for (int i = 0; i < TC::TI; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + (wm + 32 * i + fr) * LDK + kk + fk);
#pragma unroll
          for (int j = 0; j < TC::TJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(b + (wn + 32 * j + fr) * LDK + kk + fk);
#pragma unroll
          for (int i = 0; i < TC::TI; ++i)
#pragma unroll
            for (int j = 0; j < TC::TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
#endif
        if constexpr (STAGE) {
          if (kt + 1 < nk) store_block<KC>(v[(u + 1) % NS], sOwn + (cur ^ 1) * BUF_OWN, rb, kb);
          if (kt + NS < nk) load_block<KC, VEC>(v[u], G, ld, r0, rmax, kbeg + (kt + NS) * BK, kend, rb, kb);
        }
        __syncthreads();
      }
    }
  }
}

template <class TC, bool A_KC, bool B_KC, int EPI, bool ATOMIC, bool VEC>
__global__ __launch_bounds__(TC::NT, TC::NT == 256 ? 2 : 1) void gemm_bb_kernel(
    int M, int N, int K, const unsigned short* __restrict__ A, long long lda, const unsigned short* __restrict__ B,
    long long ldb, float* __restrict__ C, long long ldc, const float* __restrict__ bias, float beta, int k_per_split,
    int grid_m, int grid_n, long long sa, long long sb, long long sc) {
  constexpr int BM = TC::BM, BN = TC::BN, TI = TC::TI, TJ = TC::TJ;
  __shared__ __attribute__((aligned(16))) unsigned short sA[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) unsigned short sB[2][BN * LDK];
  // batch member blockIdx.y (strided batch: element offsets sa, sb, sc)
  A += blockIdx.y * sa;
  B += blockIdx.y * sb;
  C += blockIdx.y * sc;

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

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / TC::WAVES_N) * TC::WM, wn = (wave % TC::WAVES_N) * TC::WN;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // threads [0, BM) stage A, [BM, BM + BN) stage B, the rest only compute (wave-uniform)
  if (tid < BM)
    kloop<TC, true, A_KC, VEC, BM>(acc, A, lda, m0, M, kbeg, kend, &sA[0][0], &sA[0][0], &sB[0][0], tid, lane, wm, wn);
  else if (tid < BM + BN)
    kloop<TC, true, B_KC, VEC, BN>(acc, B, ldb, n0, N, kbeg, kend, &sB[0][0], &sA[0][0], &sB[0][0], tid - BM, lane, wm,
                                   wn);
  else
    kloop<TC, false, true, VEC, BM>(acc, A, lda, m0, M, kbeg, kend, &sA[0][0], &sA[0][0], &sB[0][0], 0, lane, wm, wn);

  // epilogue.  acc[i][j][r] holds (row wm + 32i + (r&3) + 8(r>>2) + 4(lane>>5), col
  // wn + 32j + (lane&31)).  Non-atomic: each wave stages one 32-row block (i) of its
  // sub-tile at a time in LDS (the operand buffers are free after the last barrier;
  // 32 x 68 fp32 per wave) and writes it back as 16-B stores, 16 lanes per 256-B row.
  const bool add_bias = bias && blockIdx.z == 0;
  if constexpr (ATOMIC) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = n0 + wn + 32 * j + (lane & 31);
        if (col >= N) continue;
        const float bv = add_bias ? bias[col] : 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < M) atomicAdd(C + (long long)row * ldc + col, acc[i][j][r] + bv);
        }
      }
  } else {
    constexpr int SLD = 68;
    float* stage = reinterpret_cast<float*>(&sA[0][0]) + wave * 32 * SLD;  // 8.7 KB per wave
    const int c4 = 4 * (lane & 15);  // this lane's 4 columns of the wave's 64
    const int col = n0 + wn + c4;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (add_bias) {
      bv.x = col < N ? bias[col] : 0.f;
      bv.y = col + 1 < N ? bias[col + 1] : 0.f;
      bv.z = col + 2 < N ? bias[col + 2] : 0.f;
      bv.w = col + 3 < N ? bias[col + 3] : 0.f;
    }
    const bool vec_c = (ldc % 4 == 0) && ((((uintptr_t)C) & 15) == 0) && col + 4 <= N;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          stage[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * SLD + 32 * j + (lane & 31)] = acc[i][j][r];
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll 4
      for (int rr = 0; rr < 32; rr += 4) {
        const int rl = rr + (lane >> 4);
        const int row = m0 + wm + 32 * i + rl;
        if (row >= M) continue;
        float4 x = *reinterpret_cast<const float4*>(stage + rl * SLD + c4);
        x.x += bv.x; x.y += bv.y; x.z += bv.z; x.w += bv.w;
        if constexpr (EPI == EPI_TANH_BF16) {  // V of the Linear, written directly as bf16 pairs (ldc even)
          unsigned short* cb = reinterpret_cast<unsigned short*>(C) + (long long)row * ldc + col;
          const float xs[4] = {ftanh_fast(x.x), ftanh_fast(x.y), ftanh_fast(x.z), ftanh_fast(x.w)};
          unsigned short hb[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const unsigned u = __float_as_uint(xs[c]);
            hb[c] = (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
          }
          if (col + 4 <= N) {
            *reinterpret_cast<unsigned*>(cb) = hb[0] | ((unsigned)hb[1] << 16);
            *reinterpret_cast<unsigned*>(cb + 2) = hb[2] | ((unsigned)hb[3] << 16);
          } else {
            for (int c = 0; c < 4 && col + c < N; ++c) cb[c] = hb[c];
          }
          continue;
        }
        float* cp = C + (long long)row * ldc + col;
        if (vec_c) {
          if (beta != 0.0f) {
            const float4 o = *reinterpret_cast<const float4*>(cp);
            x.x += beta * o.x; x.y += beta * o.y; x.z += beta * o.z; x.w += beta * o.w;
          }
          if (EPI == EPI_TANH) { x.x = ftanh_fast(x.x); x.y = ftanh_fast(x.y); x.z = ftanh_fast(x.z); x.w = ftanh_fast(x.w); }
          *reinterpret_cast<float4*>(cp) = x;
        } else {
          const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (col + c >= N) break;
            float y = xs[c];
            if (beta != 0.0f) y += beta * cp[c];
            if (EPI == EPI_TANH) y = ftanh_fast(y);
            cp[c] = y;
          }
        }
      }
    }
  }
}

// tile choice: 0 = automatic (gemm_tile_for), else a forced TILE_* (tuning: tools/gemm_bench_bf16.py)
enum { TILE_AUTO = 0, TILE_128x128 = 1, TILE_256x128 = 2, TILE_256x256 = 3 };
int g_tile_override = TILE_AUTO;

int gemm_tile_for(int M, int N, int K, int splitk, int batch) {
  (void)M; (void)N; (void)K; (void)splitk; (void)batch;
  return TILE_128x128;
}

template <class TC, bool A_KC, bool B_KC>
void launch_tile(bool vec, int splitk, int epi, dim3 grid, int M, int N, int K, const unsigned short* A, long long lda,
                 const unsigned short* B, long long ldb, float* C, long long ldc, const float* bias, float beta,
                 int kps, int gm, int gn, long long sa, long long sb, long long sc, hipStream_t st) {
#define GBB_LAUNCH(EPI_, AT_, VEC_)                                                                                 \
  hipLaunchKernelGGL((gemm_bb_kernel<TC, A_KC, B_KC, EPI_, AT_, VEC_>), grid, dim3(TC::NT), 0, st, M, N, K, A, lda, B, \
                     ldb, C, ldc, bias, beta, kps, gm, gn, sa, sb, sc)
  if (vec) {
    if (splitk > 1) GBB_LAUNCH(EPI_NONE, true, true);
    else if (epi == EPI_TANH) GBB_LAUNCH(EPI_TANH, false, true);
    else if (epi == EPI_TANH_BF16) {
      if constexpr (TC::NT == 256) GBB_LAUNCH(EPI_TANH_BF16, false, true);
    } else GBB_LAUNCH(EPI_NONE, false, true);
  } else if constexpr (TC::NT == 256) {  // unaligned operands: the 128 x 128 tile only
    if (splitk > 1) GBB_LAUNCH(EPI_NONE, true, false);
    else if (epi == EPI_TANH) GBB_LAUNCH(EPI_TANH, false, false);
    else GBB_LAUNCH(EPI_NONE, false, false);
  }
#undef GBB_LAUNCH
}

template <bool A_KC, bool B_KC>
int launch(int M, int N, int K, const unsigned short* A, long long lda, const unsigned short* B, long long ldb,
           float* C, long long ldc, const float* bias, int epi, float beta, int splitk, int batch, long long sa,
           long long sb, long long sc, hipStream_t st) {
  if (splitk < 1) splitk = 1;
  // straight-line 16-B loads need 16-B aligned rows (ld % 8 == 0) and base pointers
  const bool vec = lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && ldb % 8 == 0 && ((uintptr_t)B & 15) == 0 &&
                   (batch == 1 || (sa % 8 == 0 && sb % 8 == 0));
  int tc = g_tile_override ? g_tile_override : gemm_tile_for(M, N, K, splitk, batch);
  if (!vec) tc = TILE_128x128;
  if (epi == EPI_TANH_BF16) {  // bf16 output: 128 x 128 tile, aligned operands, even ldc, no accumulation
    if (!vec || beta != 0.0f || (ldc & 1) || ((uintptr_t)C & 3)) return (int)hipErrorInvalidValue;
    tc = TILE_128x128;
  }
  const int BMt = tc == TILE_128x128 ? 128 : 256, BNt = tc == TILE_256x256 ? 256 : 128;
  const int gm = (M + BMt - 1) / BMt, gn = (N + BNt - 1) / BNt;
  int kps = (K + splitk - 1) / splitk;
  kps = (kps + BK - 1) / BK * BK;
  splitk = (K + kps - 1) / kps;
  const int ntiles = gm * gn;
  dim3 grid(8 * ((ntiles + 7) / 8), batch, splitk);
  if (splitk > 1 && (epi != EPI_NONE || beta != 1.0f)) return (int)hipErrorInvalidValue;
#define GBB_ARGS vec, splitk, epi, grid, M, N, K, A, lda, B, ldb, C, ldc, bias, beta, kps, gm, gn, sa, sb, sc, st
  if (tc == TILE_256x256) launch_tile<T256x256, A_KC, B_KC>(GBB_ARGS);
  else if (tc == TILE_256x128) launch_tile<T256x128, A_KC, B_KC>(GBB_ARGS);
  else launch_tile<T128x128, A_KC, B_KC>(GBB_ARGS);
#undef GBB_ARGS
  DL4SS_CHECK_LAUNCH();
  return 0;
}

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
      const unsigned u = __float_as_uint(x[j]);
      y[j] = (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
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
    const unsigned u = __float_as_uint(x[r * ldx + c]);
    o = (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
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
  int n;
};
// one workgroup per row (rows of every segment in sequence); each thread converts pairs of
// columns and stores them as one 4-B word (ldy even)
__global__ __launch_bounds__(256) void f32_to_bf16_multi_kernel(CvtSegs sg) {
  const int row = blockIdx.x;
  int g = 0;
#pragma unroll
  for (int j = 1; j < CVT_MAX; ++j) g += (j < sg.n && row >= sg.row0[j]) ? 1 : 0;
  const long long r = row - sg.row0[g];
  const float* xr = sg.x[g] + r * sg.ldx[g];
  unsigned* yr = reinterpret_cast<unsigned*>(sg.y[g] + r * sg.ldy[g]);
  const int cols = sg.cols[g];
  const int np = (int)(sg.ldy[g] >> 1);
  for (int p = threadIdx.x; p < np; p += 256) {
    const int c = 2 * p;
    unsigned lo = 0, hi = 0;
    if (c < cols) {
      const unsigned u = __float_as_uint(xr[c]);
      lo = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    }
    if (c + 1 < cols) {
      const unsigned u = __float_as_uint(xr[c + 1]);
      hi = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    }
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
                                                            float* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float a = 0.f;
  for (int y = 0; y < nby; ++y) a += part[(long long)y * N + n];
  out[n] += a;
}

}  // namespace

// tuning knob (tools/gemm_bench_bf16.py): force a tile configuration (0 = automatic)
DL4SS_API int dl4ss_gemm_bf16_set_tile(int tile) {
  DL4SS_REQUIRE(tile >= TILE_AUTO && tile <= TILE_256x256);
  g_tile_override = tile;
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

static int colsum_bf16_launch(const void* A, long long lda, int M, int N, float* out, float* part, void* stream) {
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
                       out);
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
    sg.row0[i + 1] = sg.row0[i] + rows[i];
  }
  for (int i = n + 1; i <= CVT_MAX; ++i) sg.row0[i] = sg.row0[n];
  if (sg.row0[n] == 0) return 0;
  hipLaunchKernelGGL(f32_to_bf16_multi_kernel, dim3(sg.row0[n]), dim3(256), 0, as_stream(stream), sg);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

// Strided batch of dl4ss_gemm_bf16: member i uses A + i*strideA, B + i*strideB, C + i*strideC
// (element offsets; the bias, if any, is shared).
DL4SS_API int dl4ss_gemm_bf16_batched(int transA, int transB, int M, int N, int K, const void* A, long long lda,
                                      const void* B, long long ldb, float* C, long long ldc, const float* bias,
                                      int epilogue, float beta, int splitk, int batch, long long strideA,
                                      long long strideB, long long strideC, void* stream) {
  DL4SS_REQUIRE(M >= 0 && N >= 0 && K >= 0 && A && B && C && batch >= 1 && batch <= 65535);
  if (M == 0 || N == 0) return 0;
  hipStream_t st = as_stream(stream);
  const auto* a = reinterpret_cast<const unsigned short*>(A);
  const auto* b = reinterpret_cast<const unsigned short*>(B);
  const bool a_kc = !transA, b_kc = transB;
#define GBB_ARGS M, N, K, a, lda, b, ldb, C, ldc, bias, epilogue, beta, splitk, batch, strideA, strideB, strideC, st
  if (a_kc && b_kc) return launch<true, true>(GBB_ARGS);
  if (a_kc && !b_kc) return launch<true, false>(GBB_ARGS);
  if (!a_kc && b_kc) return launch<false, true>(GBB_ARGS);
  return launch<false, false>(GBB_ARGS);
#undef GBB_ARGS
}

// C = op(A) op(B) (+ bias) (tanh) (+ beta C) with bf16 A, B (raw 16-bit words).
// transA: A stored K x M (else M x K); transB: B stored N x K (else K x N).
DL4SS_API int dl4ss_gemm_bf16(int transA, int transB, int M, int N, int K, const void* A, long long lda,
                              const void* B, long long ldb, float* C, long long ldc, const float* bias, int epilogue,
                              float beta, int splitk, void* stream) {
  return dl4ss_gemm_bf16_batched(transA, transB, M, N, K, A, lda, B, ldb, C, ldc, bias, epilogue, beta, splitk, 1, 0,
                                 0, 0, stream);
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
