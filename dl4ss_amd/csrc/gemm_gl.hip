// bf16-operand MFMA GEMM with LDS-DMA staging (gfx950): C[M,N] (fp32) (+)= op(A) . op(B)
// (+ bias) (tanh / tanh -> bf16), both operands already bf16 in HBM -- every GEMM of the
// bf16 separation step.
//
// Why LDS-DMA: the round-1 kernel (register-staged, since removed) moved operands
// global -> VGPR -> ds_write_b128.  On gfx950 a
// ds_write_b128 moves ~79 B/clk/CU (MI355X_MICROARCH.md, LDS table), so refilling two
// 128 x 64 bf16 tiles per k-tile for two workgroups costs ~810 LDS cycles against 1024
// MFMA cycles, on top of the fragment reads: the 128 x 128 tile was LDS-bound at ~350
// TFLOP/s.  Here the tiles go global -> LDS by `global_load_lds_dwordx4` (LDS-DMA, no
// VGPR round trip, no ds_write), four 1-KB wave instructions per operand per wave and
// k-tile, double-buffered: the next k-tile's DMA is issued before the current tile's
// fragment reads and MFMAs.
//
// Operands are described as A(m, k) and B(n, k) (C = A . B^T in those terms); each is
// either KC (k contiguous: X[row * ld + k]) or KM (k-major: X[k * ld + row]).  LDS images
// (lane-linear, so every swizzle is applied to the per-lane SOURCE address and to the
// read, MI355X rule 21):
//   KC: [128 rows][64 k], 128-B rows; 16-B chunk c of row r stored at c ^ ((r >> 1) & 7):
//       the 16 rows of a ds_read_b128 lane group land on 16 distinct bank slots.
//       Fragment of v_mfma_f32_16x16x32_bf16 (lane l: row l & 15, k 8 (l >> 4) .. +7):
//       one ds_read_b128.
//   KM: [64 k-rows][128 rows], 256-B k-rows; chunk c of k-row k stored at
//       c ^ (((k & 3) << 2) | ((k >> 2) & 3)) (cdna_hip_programming.md T10, image (b)).
//       Fragment: two ds_read_b64_tr_b16 (the hardware transpose read), 4 k each.
// Waves: 4 x (64 x 64), 4 x 4 accumulators of 16 x 16 per wave, 32 MFMAs per k-tile.
// k beyond K reads a zero line (g_zero_line) instead of the operand, so partial k-tiles
// need no masking pass; rows beyond M / N read clamped addresses (their outputs are not
// stored).  Split-K (grid.z) stores fp32 partial slabs that gemm_gl_reduce_kernel adds in
// fixed order (deterministic: no float atomics).
#include "common.h"

#include <algorithm>

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int BN = 128, BK = 64;  // BK: the split-K quantum and the default k-tile depth
constexpr int PAN = 128 * BK;  // bf16 elements of one 128-row operand panel image (16 KB)

// Tile configurations: BM x 128 output tile, BM / 32 waves of 64 x 64, STG LDS stages of KT-deep
// k-tiles (KT 64 or 32), WPC workgroups per CU.
//   Cfg<128, 2>: 256 threads, 64 KB, two workgroups per CU, one k-tile of DMA in flight each
//   Cfg<256, 3>: 512 threads, 144 KB, one workgroup per CU, two k-tiles in flight (a counted
//                vmcnt across a raw s_barrier), 25 % fewer operand bytes per MFMA
//   Cfg<128, 5, 32> (round 6, the deep ring): 32-deep k-tiles, five 16-KB stages = 80 KB, two
//                workgroups per CU (the whole 160 KB), FOUR k-tiles (128 k) in flight during each
//                k-tile's MFMAs -- twice the bytes in flight of Cfg<128, 2> -- behind the same
//                counted-vmcnt raw barrier; the same MFMAs in the same k order (bitwise the same C)
template <int BM_, int STG_, int KT_ = 64>
struct Cfg {
  static constexpr int BM = BM_, STG = STG_, KT = KT_, NT = 2 * BM_, NW = NT / 64;
  static constexpr int PPP = KT_ / 4;  // 1-KB DMA pieces per 128-row panel per k-tile
  static constexpr int CPW_A = BM_ * KT_ / 512 / NW, CPW_B = BN * KT_ / 512 / NW;  // 1-KB DMAs per wave per k-tile
  static constexpr int IMG_A = BM_ * KT_, IMG_B = BN * KT_, STAGE = IMG_A + IMG_B;
  // LDS (bf16 elements): the stages, at least the epilogue's staging (NW waves x 32 rows x 68 fp32)
  static constexpr int SMEM = STG_ * STAGE > NW * 32 * 68 * 2 ? STG_ * STAGE : NW * 32 * 68 * 2;
  static constexpr int WPC = NT > 256 ? 1 : SMEM * 2 <= 40 * 1024 ? 4 : SMEM * 2 <= 53 * 1024 ? 3
                             : SMEM * 2 <= 80 * 1024 ? 2 : 1;  // workgroups per CU
  static_assert(CPW_A >= 1 && CPW_B >= 1, "at least one DMA per wave and operand");
};
enum { EPI_NONE = 0, EPI_TANH = 1, EPI_TANH_BF16 = 2, EPI_SPLIT_SLABS = 3 };

// 64 zero bytes every out-of-range k chunk is loaded from (16 B per lane)
__device__ __attribute__((aligned(64))) const unsigned g_zero_line[16] = {0};

__device__ __forceinline__ float ftanh_fast(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x)); }

__device__ __forceinline__ int km_xor(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
// KC image swizzle: 16-B chunk c of row r at c ^ kc_swz(r).  KT 64 (128-B rows, 8 chunks): the 16
// rows of a ds_read_b128 lane group on 16 distinct bank slots by (r >> 1) & 7; KT 32 (64-B rows, 4
// chunks, four rows per 256-B bank cycle): rows r, r + 4, r + 8, r + 12 apart by (r >> 2) & 3
template <int KT>
__device__ __forceinline__ int kc_swz(int r) { return KT == 64 ? (r >> 1) & 7 : (r >> 2) & 3; }

// Per-lane source pointers of one operand's CPW DMA instructions (this wave's share of a
// ROWS x KT tile, ROWS / 128 panels of PPP = KT / 4 1-KB instructions) at k-tile start kbeg; advanced
// by `step` elements per k-tile.  Instruction j fills panel j / PPP, piece j % PPP.  KC pieces are
// 512 / KT rows of KT k (lanes KT / 8 to a row); KM pieces are 4 k-rows of 128 rows.
template <bool KC, int CPW, int KT = BK>
struct Stager {
  static constexpr int PPP = KT / 4, LPR = KT / 8;
  const unsigned short* src[CPW];
  int kpos[CPW];  // k of this lane's chunk (KC) or k-row (KM) relative to the k-tile start
  long long step;
  __device__ __forceinline__ void init(const unsigned short* G, long long ld, int r0, int rmax, int kbeg, int wave,
                                       int lane) {
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
      const int j = wave * CPW + i, pan = j / PPP, jj = j % PPP;
      if (KC) {
        const int r = (512 / KT) * jj + lane / LPR, cp = lane % LPR;  // row within the panel
        const int c = cp ^ kc_swz<KT>(r);
        const int gr = min(r0 + 128 * pan + r, rmax - 1);
        src[i] = G + (long long)gr * ld + kbeg + 8 * c;
        kpos[i] = 8 * c;
      } else {
        const int k = 4 * jj + (lane >> 4), cp = lane & 15;
        const int c = cp ^ km_xor(k);
        int gc = r0 + 128 * pan + 8 * c;
        if (gc >= rmax) gc = 0;  // a chunk wholly past the last row: any valid address
        src[i] = G + (long long)(kbeg + k) * ld + gc;
        kpos[i] = k;
      }
    }
    step = KC ? KT : (long long)KT * ld;
  }
  // issue this wave's CPW 1-KB DMAs of k-tile t (k0 = kbeg + t * KT) into image dst
  __device__ __forceinline__ void issue(unsigned short* dst, int wave, int t, int k0_rel, int kspan) {
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
      const bool in = k0_rel + kpos[i] < kspan;
      const void* p = in ? (const void*)(src[i] + t * step) : (const void*)g_zero_line;
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(dst + (wave * CPW + i) * 512), 16, 0, 0);
    }
  }
};

// fragment (8 k-values of one row) of k-step kk (0 .. KT / 32 - 1) for tile row `row`
template <bool KC, int KT = BK>
__device__ __forceinline__ bf16x8 frag(const unsigned short* img, int row, int kk, int lane) {
  img += (row >> 7) * (128 * KT);  // 128-row panel
  row &= 127;
  if (KC) {
    const int c = 4 * kk + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * KT + 8 * (c ^ kc_swz<KT>(row)));
  } else {
    // group g = lane >> 4 reads k-rows 32 kk + 8 g + 4 h + q (q = 0..3) for rows c0 .. c0 + 15,
    // lane 4 q + p of the group addressing columns c0 + 4 p .. + 3 (c0 = row - (lane & 15))
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int c0 = row - (lane & 15);
    bf16x4 h[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int k = 32 * kk + 8 * g + 4 * hh + q;
      const int ch = ((c0 >> 3) + (p >> 1)) ^ km_xor(k);
      h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + k * 128 + 8 * ch + 4 * (p & 1)));
    }
    return bf16x8{h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]};
  }
}

// s_waitcnt vmcnt(N) with N a compile-time count; vm_wait_n: the count a * PW for a runtime a < AMAX
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int PW, int AMAX>
__device__ __forceinline__ void vm_wait_n(int a) {
  if constexpr (AMAX > 0) {
    if (a == AMAX - 1) {
      vm_wait<(AMAX - 1) * PW>();
      return;
    }
    vm_wait_n<PW, AMAX - 1>(a);
  } else {
    vm_wait<0>();
  }
}

// One BM x 128 output tile of C (or of split-K slab `slab`, SPLIT) over k in [kbeg, kbeg + kspan):
// the k-loop and the epilogue of gemm_gl_kernel and gemm_gl_grouped_kernel.  smem: the kernel's
// one LDS array (CF::STG * CF::STAGE bf16).
// RS (row sums, the grouped side-stream dW_lin): the tiles of column block 0 also form
// rsum[m] = beta rsum[m] + sum_k A(m, k) -- the Linear's bias gradient, sum over rows of dPre, off the
// same A fragments: the waves of columns 0..63 run one more MFMA per A fragment against an all-ones B
// (bf16 products exact, fp32 accumulation, fixed k order).
template <bool A_KC, bool B_KC, int EPI, bool SPLIT, class CF, bool RS = false>
__device__ __forceinline__ void gl_tile(unsigned short* smem, int M, int N, const unsigned short* __restrict__ A,
                                        long long lda, const unsigned short* __restrict__ B, long long ldb,
                                        float* __restrict__ C, long long ldc, const float* __restrict__ bias,
                                        float beta, int m0, int n0, int kbeg, int kspan, float* __restrict__ slab,
                                        float* __restrict__ rsum = nullptr) {
  constexpr int STG = CF::STG, IMG_A = CF::IMG_A, STAGE = CF::STAGE, KT = CF::KT;
  const int nk = (kspan + KT - 1) / KT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const bool rs = RS && rsum != nullptr && n0 == 0 && wn == 0;  // wave-uniform
  f32x4 accr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) accr[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};

  Stager<A_KC, CF::CPW_A, KT> sa_;
  Stager<B_KC, CF::CPW_B, KT> sb_;
  sa_.init(A, lda, m0, M, kbeg, wave, lane);
  sb_.init(B, ldb, n0, N, kbeg, wave, lane);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const unsigned short* ia) {
    const unsigned short* ib = ia + IMG_A;
#pragma unroll
    for (int kk = 0; kk < KT / 32; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<A_KC, KT>(ia, wm + 16 * i + (lane & 15), kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<B_KC, KT>(ib, wn + 16 * j + (lane & 15), kk, lane);
#ifndef GGL_NO_MFMA  // diagnostic builds: GGL_NO_MFMA (fragments read, no MFMA), GGL_NO_DMA (first tile only)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if constexpr (RS) {
        if (rs) {
#pragma unroll
          for (int i = 0; i < 4; ++i) accr[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, accr[i], 0, 0, 0);
        }
      }
#else
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" :: "v"(af[i]), "v"(bfr[i]));
#endif
    }
  };
  auto dma = [&](int t) {  // this wave's DMAs of k-tile t into LDS stage t % STG
    unsigned short* na = smem + (t % STG) * STAGE;
    sa_.issue(na, wave, t, t * KT, kspan);
    sb_.issue(na + IMG_A, wave, t, t * KT, kspan);
  };
  if constexpr (STG == 2) {
    dma(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
#ifndef GGL_NO_DMA
      if (kt + 1 < nk) dma(kt + 1);  // into the other buffer (last read before the previous barrier)
#endif
      compute(smem + (kt & 1) * STAGE);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMAs of k-tile kt + 1 landed
      __syncthreads();  // ... and every wave's; every wave is done reading buffer kt & 1
    }
  } else {
    // STG - 1 k-tiles issued ahead: at k-tile kt, tiles kt + 1 .. kt + STG - 2 may stay in flight
    // across the wait (a counted vmcnt), then the raw barrier (every wave's tile kt landed, every
    // wave is done reading tile kt - 1's stage), then tile kt + STG - 1 into that stage
    constexpr int PW = CF::CPW_A + CF::CPW_B;  // this wave's DMAs per k-tile
#pragma unroll
    for (int t = 0; t < STG - 1; ++t)
      if (t < nk) dma(t);
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = min(STG - 2, nk - 1 - kt);  // tiles issued after kt (wave-uniform)
      if (ahead >= STG - 2) vm_wait<(STG - 2) * PW>();
      else vm_wait_n<PW, STG - 2>(ahead);
      __builtin_amdgcn_s_barrier();
      if (kt + STG - 1 < nk) dma(kt + STG - 1);  // into the stage tile kt - 1 used
      compute(smem + (kt % STG) * STAGE);
    }
    __syncthreads();  // every wave is done with the stages before the epilogue reuses LDS
  }

  if constexpr (RS) {
    // accr[i][e] = rsum of row wm + 16 i + 4 (lane >> 4) + e in every column; column 0's lanes store
    if (rs && (lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + e;
          if (row < M) rsum[row] = beta != 0.0f ? accr[i][e] + beta * rsum[row] : accr[i][e];
        }
    }
  }
  // epilogue: acc[i][j][e] = C(wm + 16 i + 4 (lane >> 4) + e, wn + 16 j + (lane & 15)).  Each
  // wave stages 32 rows (i = 2h, 2h + 1) of its 64 x 64 sub-tile at a time in LDS (free
  // after the last barrier; 32 x 68 fp32 per wave) and writes rows back as 16-B stores.
  constexpr int SLD = 68;
  float* stage = reinterpret_cast<float*>(smem) + wave * 32 * SLD;
  const int c4 = 4 * (lane & 15);
  const int col = n0 + wn + c4;
  const bool add_bias = !SPLIT && bias != nullptr;
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (add_bias) {
    bv.x = col < N ? bias[col] : 0.f;
    bv.y = col + 1 < N ? bias[col + 1] : 0.f;
    bv.z = col + 2 < N ? bias[col + 2] : 0.f;
    bv.w = col + 3 < N ? bias[col + 3] : 0.f;
  }
  // split-K slab of (batch member y, split z): part[y][z][M][N]
  float* out = SPLIT ? slab : C;
  const long long ldo = SPLIT ? N : ldc;
  const bool vec_c = (ldo % 4 == 0) && ((((uintptr_t)out) & 15) == 0) && col + 4 <= N;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#ifdef GGL_NO_STORE  // diagnostic builds only (results wrong): the k-loop without the epilogue
    if (M > 0) break;
#endif
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          stage[(16 * i2 + 4 * (lane >> 4) + e) * SLD + 16 * j + (lane & 15)] = acc[2 * h + i2][j][e];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll 4
    for (int rr = 0; rr < 32; rr += 4) {
      const int rl = rr + (lane >> 4);
      const int row = m0 + wm + 32 * h + rl;
      if (row >= M) continue;
      float4 x = *reinterpret_cast<const float4*>(stage + rl * SLD + c4);
      x.x += bv.x; x.y += bv.y; x.z += bv.z; x.w += bv.w;
      if constexpr (EPI == EPI_TANH_BF16) {  // V of the Linear, written directly as bf16 pairs (ldc even)
        unsigned short* cb = reinterpret_cast<unsigned short*>(C) + (long long)row * ldc + col;
        const float xs[4] = {ftanh_fast(x.x), ftanh_fast(x.y), ftanh_fast(x.z), ftanh_fast(x.w)};
        unsigned short hb[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          hb[c] = (unsigned short)bf16_bits_rne(xs[c]);
        }
        if (col + 4 <= N) {  // two 4-B stores: ldc is only required even (V rows of F * E = 6450)
          *reinterpret_cast<unsigned*>(cb) = hb[0] | ((unsigned)hb[1] << 16);
          *reinterpret_cast<unsigned*>(cb + 2) = hb[2] | ((unsigned)hb[3] << 16);
        } else {
          for (int c = 0; c < 4 && col + c < N; ++c) cb[c] = hb[c];
        }
        continue;
      }
      float* cp = out + (long long)row * ldo + col;
      if (vec_c) {
        if (!SPLIT && beta != 0.0f) {
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
          if (!SPLIT && beta != 0.0f) y += beta * cp[c];
          if (EPI == EPI_TANH) y = ftanh_fast(y);
          cp[c] = y;
        }
      }
    }
  }
}

template <bool A_KC, bool B_KC, int EPI, bool SPLIT, class CF>
__global__ __launch_bounds__(CF::NT, CF::WPC) void gemm_gl_kernel(
    int M, int N, int K, const unsigned short* __restrict__ A, long long lda, const unsigned short* __restrict__ B,
    long long ldb, float* __restrict__ C, long long ldc, const float* __restrict__ bias, float beta, int k_per_split,
    int grid_m, int grid_n, long long sa, long long sb, long long sc, float* __restrict__ part) {
  constexpr int BM = CF::BM;
  // one LDS array (a second __shared__ object can make hipcc drain vmcnt before every ds_read)
  __shared__ __attribute__((aligned(16))) unsigned short smem[CF::SMEM];
  // XCD-major order over the WHOLE grid (tiles x batch members x k-splits): workgroups are
  // dealt round-robin over the 8 XCDs in dispatch order (x fastest, then y, then z; speed
  // only, never correctness), so the dispatch index L is remapped bijectively to R, giving
  // each XCD a contiguous range of R: mostly one (split, member) and 8 M-tiles x all N-tiles
  // groups of it, whose operand panels then stay in that XCD's L2
  const int ntiles = grid_m * grid_n;
  const int nwg = gridDim.x * gridDim.y * gridDim.z;
  const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xcd = L % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int R = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + L / 8;
  const int zsplit = R / (ntiles * (int)gridDim.y);
  const int ymem = (R / ntiles) % (int)gridDim.y;
  const int tile = R % ntiles;
  A += ymem * sa;
  B += ymem * sb;
  C += ymem * sc;
  constexpr int GROUP = 8;
  const int gsize = GROUP * grid_n;
  const int first_m = (tile / gsize) * GROUP;
  const int gm_here = min(grid_m - first_m, GROUP);
  const int tm = first_m + (tile % gsize) % gm_here, tn = (tile % gsize) / gm_here;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = zsplit * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  if (kbeg >= kend) return;
  gl_tile<A_KC, B_KC, EPI, SPLIT, CF>(smem, M, N, A, lda, B, ldb, C, ldc, bias, beta, m0, n0, kbeg, kend - kbeg,
                                      SPLIT ? part + ((long long)ymem * gridDim.z + zsplit) * M * N : nullptr);
}

// One epilogue store of four consecutive columns col .. col + 3 of output row `row` (row < M
// checked by the caller): + bias, + beta C, tanh, bf16 (EPI_TANH_BF16) or an fp32 split-K slab.
template <int EPI, bool SPLIT>
__device__ __forceinline__ void store4(float4 x, int row, int col, int N, float* C, long long ldc, float* out,
                                       long long ldo, bool vec_c, float beta, const float4& bv) {
  x.x += bv.x; x.y += bv.y; x.z += bv.z; x.w += bv.w;
  if constexpr (EPI == EPI_TANH_BF16) {  // V of the Linear, written directly as bf16 pairs (ldc even)
    unsigned short* cb = reinterpret_cast<unsigned short*>(C) + (long long)row * ldc + col;
    const float xs[4] = {ftanh_fast(x.x), ftanh_fast(x.y), ftanh_fast(x.z), ftanh_fast(x.w)};
    unsigned short hb[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      hb[c] = (unsigned short)bf16_bits_rne(xs[c]);
    }
    if (col + 4 <= N) {  // two 4-B stores: ldc is only required even (V rows of F * E = 6450)
      *reinterpret_cast<unsigned*>(cb) = hb[0] | ((unsigned)hb[1] << 16);
      *reinterpret_cast<unsigned*>(cb + 2) = hb[2] | ((unsigned)hb[3] << 16);
    } else {
      for (int c = 0; c < 4 && col + c < N; ++c) cb[c] = hb[c];
    }
    return;
  }
  float* cp = out + (long long)row * ldo + col;
  if (vec_c) {
    if (!SPLIT && beta != 0.0f) {
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
      if (!SPLIT && beta != 0.0f) y += beta * cp[c];
      if (EPI == EPI_TANH) y = ftanh_fast(y);
      cp[c] = y;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 256 x 256 ping-pong configuration (cfg 4, gemm_pp_kernel).  Why: the 128 x 128 kernel above
// moves 64 KB per k-tile per CU (two workgroups) for 4.2 MFLOP; measured at ~1.3 us per k-tile
// on every shape (4096^3 and the step's), i.e. the per-CU LDS-DMA path (~50-70 GB/s per CU from
// L2, MI355X_MICROARCH.md 'Indexed rows') sets the rate at 0.33 of the MFMA peak.  A 256 x 256
// tile per CU moves the same 64 KB per k-tile for 8.4 MFLOP: the load path and the MFMA pipe
// balance (cdna_hip_programming.md §5 'The 256^2 8-phase template').
//
// Structure (one workgroup of 8 waves per CU, 128 KB LDS):
//  * LDS = 8 half-tile slots of 16 KB: k-tile t (64 deep) lives in slots (t & 1) x {A0, A1, B0,
//    B1}, each one 128-row operand panel in the PAN images of gemm_gl_kernel (same swizzles,
//    same Stager / frag code).
//  * The 256 x 256 C tile is four 128 x 128 quadrants Q(a, b) = A half a x B half b; in phase p
//    of a k-tile EVERY wave works on the same quadrant (wave w: rows 64 (w >> 2), columns
//    32 (w & 3) of it: 4 x 2 tiles of 16 x 16, 16 MFMAs over K = 64), in the order Q00, Q01,
//    Q11, Q10, so each phase reads one new operand half: p0 A0 + B0 (12 ds_read_b128-sized
//    fragments), p1 B1, p2 A1, p3 nothing (B0 kept in registers) -- a half-tile slot is free
//    as soon as its phase has passed.
//  * One half-tile (2 LDS-DMA instructions per wave) is issued per phase: p0 B1(t+1), p1
//    A1(t+1), p2 A0(t+2), p3 B0(t+2) -- each into a slot whose last read is >= 2 phases back.
//    Before the barrier that precedes a phase with reads, every wave retires its own DMAs down
//    to the 4 half-tiles issued after the one that phase reads: `s_waitcnt vmcnt(8)`, never 0
//    in the loop; DMAs past the last k-tile read the zero line, so the count is uniform.
//  * Ping-pong: waves 4-7 run one raw `s_barrier` behind waves 0-3, so on every SIMD one wave
//    issues its fragment reads and DMAs while the other runs its MFMA cluster (s_setprio 1).
//    A group-1 wave's reads of phase p sit between global barriers 2p+1 and 2p+2, group 0's
//    between 2p and 2p+1; every wave's counted wait precedes barrier 2p (group 0: after its
//    MFMAs of p-1, group 1: after its reads of p-1), so the data is in LDS for both groups.
// ---------------------------------------------------------------------------------------------
namespace pp {
constexpr int BM = 256, NT = 512;
constexpr int SLD = 36;  // epilogue staging row stride (floats) of a wave's 64 x 32 block

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
template <int VM>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <bool KC>
__device__ __forceinline__ void read4(bf16x8 (&f)[4][2], const unsigned short* img, int r0, int lane) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i][kk] = frag<KC>(img, r0 + 16 * i + (lane & 15), kk, lane);
}
template <bool KC>
__device__ __forceinline__ void read2(bf16x8 (&f)[2][2], const unsigned short* img, int r0, int lane) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < 2; ++j) f[j][kk] = frag<KC>(img, r0 + 16 * j + (lane & 15), kk, lane);
}
__device__ __forceinline__ void mma(f32x4 (&acc)[4][2], const bf16x8 (&af)[4][2], const bf16x8 (&bf)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], acc[i][j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}
}  // namespace pp

// SL half-tile slots (8: 128 KB, 10: the whole 160 KB).  Half-tiles are numbered in issue order
// n = 4 t + {A0: 0, B0: 1, B1: 2, A1: 3} and live in slot n % SL; phase P = 4 t + p reads up to
// n = P + 1 and issues n = P + AHEAD (AHEAD = SL - 2: the slot it overwrites held n - SL, last
// read in phase <= P - 2), so AHEAD - 2 half-tiles = 2 (AHEAD - 2) DMAs stay in flight at
// every counted wait.
template <bool A_KC, bool B_KC, int EPI, bool SPLIT, int SL>
__global__ __launch_bounds__(pp::NT, 1) void gemm_pp_kernel(
    int M, int N, int K, const unsigned short* __restrict__ A, long long lda, const unsigned short* __restrict__ B,
    long long ldb, float* __restrict__ C, long long ldc, const float* __restrict__ bias, float beta, int k_per_split,
    int grid_m, int grid_n, long long sa, long long sb, long long sc, float* __restrict__ part) {
  constexpr int AHEAD = SL - 2, VM = 2 * (AHEAD - 2);
  __shared__ __attribute__((aligned(16))) unsigned short smem[SL * PAN];  // the only LDS object
  // XCD-major remap of the whole grid, as gemm_gl_kernel
  const int ntiles = grid_m * grid_n;
  const int nwg = gridDim.x * gridDim.y * gridDim.z;
  const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xcd = L % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int R = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + L / 8;
  const int zsplit = R / (ntiles * (int)gridDim.y);
  const int ymem = (R / ntiles) % (int)gridDim.y;
  const int tile = R % ntiles;
  A += ymem * sa;
  B += ymem * sb;
  C += ymem * sc;
  constexpr int GROUP = 4;
  const int gsize = GROUP * grid_n;
  const int first_m = (tile / gsize) * GROUP;
  const int gm_here = min(grid_m - first_m, GROUP);
  const int tm = first_m + (tile % gsize) % gm_here, tn = (tile % gsize) / gm_here;
  const int m0 = tm * pp::BM, n0 = tn * pp::BM;
  const int kbeg = zsplit * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  if (kbeg >= kend) return;  // uniform over the workgroup
  const int kspan = kend - kbeg;
  const int nk = (kspan + BK - 1) / BK;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wave >> 2);
  const int wm = 64 * (wave >> 2), wn = 32 * (wave & 3);

  Stager<A_KC, 2> sa0, sa1;
  Stager<B_KC, 2> sb0, sb1;
  sa0.init(A, lda, m0, M, kbeg, wave, lane);
  sa1.init(A, lda, m0 + 128, M, kbeg, wave, lane);
  sb0.init(B, ldb, n0, N, kbeg, wave, lane);
  sb1.init(B, ldb, n0 + 128, N, kbeg, wave, lane);
  auto slot = [&](int n) { return smem + (n % SL) * PAN; };
  // issue half-tile n (its code n & 3 is a compile-time constant at every call site)
  auto dma = [&](int n) {
    const int t = n >> 2;
    switch (n & 3) {
      case 0: sa0.issue(slot(n), wave, t, t * BK, kspan); break;
      case 1: sb0.issue(slot(n), wave, t, t * BK, kspan); break;
      case 2: sb1.issue(slot(n), wave, t, t * BK, kspan); break;
      default: sa1.issue(slot(n), wave, t, t * BK, kspan); break;
    }
  };

  f32x4 acc[4][4][2];  // [quadrant a * 2 + b][row tile i][column tile j]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bf0[2][2], bf1[2][2];

  // prologue: half-tiles 0 .. AHEAD - 1 (what phases -AHEAD .. -1 would have issued)
#pragma unroll
  for (int n = 0; n < AHEAD; ++n) dma(n);
  pp::wait_vm<VM>();  // half-tiles 0, 1 (A0, B0 of k-tile 0) landed
  pp::bar();          // global barrier 0
  if (grp) pp::bar();  // waves 4-7 one barrier behind
  for (int t = 0; t < nk; ++t) {
    const int P = 4 * t;
    // phase 0: Q00 -- reads A0, B0 of t
    pp::read4<A_KC>(af, slot(P), wm, lane);
    pp::read2<B_KC>(bf0, slot(P + 1), wn, lane);
    dma(P + AHEAD);
    if (grp) pp::wait_vm<VM>();  // B1(t) for phase 1
    pp::bar();
    pp::mma(acc[0], af, bf0);
    if (!grp) pp::wait_vm<VM>();
    pp::bar();
    // phase 1: Q01 -- reads B1 of t
    pp::read2<B_KC>(bf1, slot(P + 2), wn, lane);
    dma(P + 1 + AHEAD);
    if (grp) pp::wait_vm<VM>();  // A1(t) for phase 2
    pp::bar();
    pp::mma(acc[1], af, bf1);
    if (!grp) pp::wait_vm<VM>();
    pp::bar();
    // phase 2: Q11 -- reads A1 of t
    pp::read4<A_KC>(af, slot(P + 3), wm, lane);
    dma(P + 2 + AHEAD);
    pp::bar();
    pp::mma(acc[3], af, bf1);
    pp::bar();
    // phase 3: Q10 -- no reads (B0 still in registers)
    dma(P + 3 + AHEAD);
    if (grp) pp::wait_vm<VM>();  // A0(t+1), B0(t+1) for the next phase 0
    pp::bar();
    pp::mma(acc[2], af, bf0);
    if (!grp) pp::wait_vm<VM>();
    pp::bar();
  }
  if (!grp) pp::bar();  // waves 0-3 catch up with the barrier waves 4-7 spent at the start
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-line DMAs past the last k-tile
  __syncthreads();      // every wave is done with the slots before the epilogue reuses LDS

  // epilogue: per quadrant, the wave's 64 x 32 block (acc[q][i][j][e] = row 16 i + 4 (lane >> 4) + e,
  // column 16 j + (lane & 15)) is staged in its own LDS area and written back 8 rows per pass
  float* stage = reinterpret_cast<float*>(smem) + wave * 64 * pp::SLD;
  float* out = SPLIT ? part + ((long long)ymem * gridDim.z + zsplit) * M * N : C;
  const long long ldo = SPLIT ? N : ldc;
  const bool add_bias = !SPLIT && bias != nullptr;
  const int c4 = 4 * (lane & 7);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int a = q >> 1, b = q & 1;
    const int col = n0 + 128 * b + wn + c4;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (add_bias) {
      bv.x = col < N ? bias[col] : 0.f;
      bv.y = col + 1 < N ? bias[col + 1] : 0.f;
      bv.z = col + 2 < N ? bias[col + 2] : 0.f;
      bv.w = col + 3 < N ? bias[col + 3] : 0.f;
    }
    const bool vec_c = (ldo % 4 == 0) && ((((uintptr_t)out) & 15) == 0) && col + 4 <= N;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) stage[(16 * i + 4 * (lane >> 4) + e) * pp::SLD + 16 * j + (lane & 15)] = acc[q][i][j][e];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll 2
    for (int rr = 0; rr < 64; rr += 8) {
      const int rl = rr + (lane >> 3);
      const int row = m0 + 128 * a + wm + rl;
      if (row >= M) continue;
      const float4 x = *reinterpret_cast<const float4*>(stage + rl * pp::SLD + c4);
      store4<EPI, SPLIT>(x, row, col, N, C, ldc, out, ldo, vec_c, beta, bv);
    }
  }
}

// C[b] = beta C[b] + sum_{z < S} part[b][z] (+ bias), z in order: the split-K combine.  VEC:
// four columns per thread with 16-B loads / stores (N % 4 == 0, ldc % 4 == 0, aligned C), the
// S slab loads of a thread issued together (8 at a time) before they are summed in order.
template <bool VEC>
__global__ __launch_bounds__(256) void gemm_gl_reduce_kernel(int M, int N, int S, const float* __restrict__ part,
                                                             float* __restrict__ C, long long ldc, long long sc,
                                                             const float* __restrict__ bias, float beta) {
  constexpr int W = VEC ? 4 : 1;
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * W;
  const long long mn = (long long)M * N;
  if (i >= mn) return;
  const int b = blockIdx.y;
  const float* p = part + (long long)b * S * mn + i;
  const int r = (int)(i / N), c = (int)(i - (long long)r * N);
  float* cp = C + b * sc + (long long)r * ldc + c;
  if constexpr (VEC) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z0 = 0; z0 < S; z0 += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = z0 + u < S ? *reinterpret_cast<const float4*>(p + (long long)(z0 + u) * mn) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (z0 + u < S) { a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w; }
      }
    }
    if (bias) { a.x += bias[c]; a.y += bias[c + 1]; a.z += bias[c + 2]; a.w += bias[c + 3]; }
    if (beta != 0.0f) {
      const float4 o = *reinterpret_cast<const float4*>(cp);
      a.x += beta * o.x; a.y += beta * o.y; a.z += beta * o.z; a.w += beta * o.w;
    }
    *reinterpret_cast<float4*>(cp) = a;
  } else {
    float a = 0.f;
    for (int z = 0; z < S; ++z) a += p[(long long)z * mn];
    if (bias) a += bias[c];
    *cp = beta != 0.0f ? a + beta * *cp : a;
  }
}

// ---------------------------------------------------------------------------------------------
// Grouped launch: up to GMAXP independent GEMMs (the step's weight gradients: dW_lin and every
// layer's dW_ih / dW_hh, each its own M x N x K and split-K factor) as ONE grid.  One by one they
// under-fill the chip (dW_ih: 95 tiles x 4 splits; dW_hh: 2 x 30 tiles x 8 splits) and each pays its
// own ramp and tail; together they are ~3,000 workgroups of equal-length k-ranges.  The
// workgroup -> (problem, split, tile) map, the per-tile arithmetic and the slabs are those of the
// single launches, so every gradient is bitwise what gemm_gl_kernel + gemm_gl_reduce_kernel
// produce with the same split factors.  Problem parameters travel in the kernel arguments and are
// selected by unrolled compile-time indices (wave-uniform scalar code, no dynamic indexing into
// the argument segment).
// ---------------------------------------------------------------------------------------------
constexpr int GMAXP = 16;
struct GlProb {
  const unsigned short* A;
  const unsigned short* B;
  float* C;
  float* part;  // split-K slabs [nsplit][M][N] (null when nsplit == 1)
  long long lda, ldb, ldc;
  float beta;
  int M, N, K, gm, gn, nsplit, kps;
  int wg0;  // first workgroup (in the XCD-remapped order) of this problem
  int u0;   // first reduce unit (gemm_gl_grouped_reduce_kernel)
  int vec;  // reduce with 16-B accesses (N % 4 == 0, ldc % 4 == 0, C 16-B aligned)
  float* rsum;  // row sums of op(A) (+= beta rsum), formed by column block 0 (unsplit problems, RS kernels)
};
struct GlGroup {
  int n, total_wg, total_units;
  GlProb p[GMAXP];
};

// tile L (dispatch order) of the group: p is its problem (selected by the kernel from the kernel
// argument with compile-time indices: a reference to the argument struct put it in scratch)
template <bool A_KC, bool B_KC, class CF, bool RS>
__device__ __forceinline__ void grouped_tile(const GlProb p, int L, unsigned short* smem) {
  const int ntot = p.gm * p.gn * p.nsplit;
  const int Ll = L - p.wg0;
  const int xcd = Ll % 8, q8 = ntot / 8, r8 = ntot % 8;
  const int local = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + Ll / 8;
  const int ntiles = p.gm * p.gn;
  const int zsplit = local / ntiles, tile = local % ntiles;
  // n fastest: an XCD's contiguous tile range covers whole rows of M-panels, so every A panel
  // (the big operand of these weight gradients: dPre 103.6 MB, each layer's dG 38.6 MB) is fetched
  // into one XCD's L2 once and shared by its gn N-tiles there; the small B operand (layer inputs,
  // h_{t-1}: <= 9.6 MB) is what each XCD re-reads
  // (the single launch's GROUP = 8 m-swizzle here: 8090 vs 8101 mixtures/s, round 4)
  const int tm = tile / p.gn, tn = tile % p.gn;
  const int m0 = tm * CF::BM, n0 = tn * BN;
  const int kbeg = zsplit * p.kps;
  const int kend = min(p.K, kbeg + p.kps);
  if (kbeg >= kend) return;
  if (p.nsplit > 1)
    gl_tile<A_KC, B_KC, EPI_NONE, true, CF>(smem, p.M, p.N, p.A, p.lda, p.B, p.ldb, p.C, p.ldc, nullptr, 0.0f, m0, n0,
                                            kbeg, kend - kbeg, p.part + (long long)zsplit * p.M * p.N);
  else
    gl_tile<A_KC, B_KC, EPI_NONE, false, CF, RS>(smem, p.M, p.N, p.A, p.lda, p.B, p.ldb, p.C, p.ldc, nullptr, p.beta,
                                                 m0, n0, kbeg, kend - kbeg, nullptr, p.rsum);
}

template <bool A_KC, bool B_KC, class CF, bool RS = false>
__global__ __launch_bounds__(CF::NT, CF::WPC) void gemm_gl_grouped_kernel(GlGroup g) {
  __shared__ __attribute__((aligned(16))) unsigned short smem[CF::SMEM];
  // problems by DISPATCH order (so every problem's workgroups are dealt over all 8 XCDs: an
  // XCD-contiguous remap of the whole grid handed one XCD nearly all of dW_lin's long k-ranges,
  // 616 vs ~330 us), then the XCD-major remap inside the problem (L0 = its first dispatch index;
  // L - L0 with equal residues mod 8 share an XCD, whatever L0 % 8 is).  A grid smaller than the
  // tile count (the persistent form, dl4ss_gemm_bf16_gl_grouped_ex) walks the tiles in steps of
  // gridDim.x.
  for (int L = blockIdx.x; L < g.total_wg; L += gridDim.x) {
    if (L != (int)blockIdx.x) __syncthreads();  // the previous tile's epilogue is done with the LDS
    int pi = 0;
#pragma unroll
    for (int k = 1; k < GMAXP; ++k)
      if (k < g.n && L >= g.p[k].wg0) pi = k;
    GlProb p = g.p[0];
#pragma unroll
    for (int k = 1; k < GMAXP; ++k)
      if (k == pi) p = g.p[k];
    grouped_tile<A_KC, B_KC, CF, RS>(p, L, smem);
  }
}

// The split-K combine of every split problem of a group, one launch: unit u of problem p is four
// columns (vec) or one element; the arithmetic of gemm_gl_reduce_kernel<vec> (slabs in order z =
// 0 .. S-1 from zero, then + beta C).
__global__ __launch_bounds__(256) void gemm_gl_grouped_reduce_kernel(GlGroup g) {
  const int u = blockIdx.x * 256 + threadIdx.x;
  if (u >= g.total_units) return;
  int pi = -1;
#pragma unroll
  for (int k = 0; k < GMAXP; ++k)
    if (k < g.n && g.p[k].nsplit > 1 && u >= g.p[k].u0) pi = k;
  if (pi < 0) return;
  GlProb p = g.p[0];
#pragma unroll
  for (int k = 1; k < GMAXP; ++k)
    if (k == pi) p = g.p[k];
  const long long mn = (long long)p.M * p.N;
  const int S = p.nsplit;
  if (p.vec) {
    const long long i = 4LL * (u - p.u0);
    if (i >= mn) return;
    const float* pp = p.part + i;
    const int r = (int)(i / p.N), c = (int)(i - (long long)r * p.N);
    float* cp = p.C + (long long)r * p.ldc + c;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z0 = 0; z0 < S; z0 += 8) {
      float4 v[8];
#pragma unroll
      for (int w = 0; w < 8; ++w)
        v[w] = z0 + w < S ? *reinterpret_cast<const float4*>(pp + (long long)(z0 + w) * mn) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        if (z0 + w < S) { a.x += v[w].x; a.y += v[w].y; a.z += v[w].z; a.w += v[w].w; }
      }
    }
    if (p.beta != 0.0f) {
      const float4 o = *reinterpret_cast<const float4*>(cp);
      a.x += p.beta * o.x; a.y += p.beta * o.y; a.z += p.beta * o.z; a.w += p.beta * o.w;
    }
    *reinterpret_cast<float4*>(cp) = a;
  } else {
    const long long i = u - p.u0;
    if (i >= mn) return;
    const int r = (int)(i / p.N), c = (int)(i - (long long)r * p.N);
    float* cp = p.C + (long long)r * p.ldc + c;
    float a = 0.f;
    for (int z = 0; z < S; ++z) a += p.part[(long long)z * mn + i];
    *cp = p.beta != 0.0f ? a + p.beta * *cp : a;
  }
}

typedef Cfg<128, 2> C128;  // 128 x 128, double buffer, two workgroups per CU (the round-2 default)
typedef Cfg<256, 3> C256;  // 256 x 128, three stages, one workgroup per CU
typedef Cfg<128, 3> C128S3;  // 128 x 128, three stages (measured slower: A/B knob only)
typedef Cfg<128, 5, 32> C128D5;  // 128 x 128, five 32-deep stages (80 KB), two per CU: the deep ring
typedef Cfg<128, 4, 32> C128D4;  // the same with four stages (64 KB): three k-tiles in flight
typedef Cfg<128, 2, 32> C128H2;  // 32-deep double buffer (32 KB): four workgroups per CU
typedef Cfg<64, 2> C64;  // 64 x 128, two waves, double buffer (48 KB): three workgroups per CU
// tile configuration: 0 = per shape (gl_cfg_for), 1 = C128, 2 = C256, 3 = C128S3, 4 / 5 = 256 x 256
// ping-pong with 8 / 10 half-tile slots
int g_gl_cfg = 0;

int gl_cfg_for(int M, int N, int K, int splitk, int batch) {
  (void)M; (void)N; (void)K; (void)splitk; (void)batch;
  return 1;
}

template <bool A_KC, bool B_KC, class CF>
int launch_cfg(int M, int N, int K, const unsigned short* A, long long lda, const unsigned short* B, long long ldb,
               float* C, long long ldc, const float* bias, int epi, float beta, int splitk, int batch, long long sa,
               long long sb, long long sc, float* ws, long long ws_bytes, hipStream_t st) {
  const int gm = (M + CF::BM - 1) / CF::BM, gn = (N + BN - 1) / BN;
  int kps = (K + splitk - 1) / splitk;
  kps = (kps + BK - 1) / BK * BK;
  splitk = (K + kps - 1) / kps;
  const int ntiles = gm * gn;
  dim3 grid(ntiles, batch, splitk);
  if (splitk > 1) {
    if (epi != EPI_NONE && epi != EPI_SPLIT_SLABS) return (int)hipErrorInvalidValue;
    const long long need = (long long)batch * splitk * M * N * 4;
    if (!ws || ws_bytes < need) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm_gl_kernel<A_KC, B_KC, EPI_NONE, true, CF>), grid, dim3(CF::NT), 0, st, M, N, K, A, lda, B,
                       ldb, C, ldc, nullptr, 0.0f, kps, gm, gn, sa, sb, sc, ws);
    DL4SS_CHECK_LAUNCH();
    if (epi == EPI_SPLIT_SLABS) return 0;  // the slabs stay in ws for their consumer
    if (N % 4 == 0 && ldc % 4 == 0 && sc % 4 == 0 && ((uintptr_t)C & 15) == 0)
      hipLaunchKernelGGL(gemm_gl_reduce_kernel<true>, dim3(cdiv((long long)M * N / 4, 256), batch), dim3(256), 0, st, M,
                         N, splitk, ws, C, ldc, sc, bias, beta);
    else
      hipLaunchKernelGGL(gemm_gl_reduce_kernel<false>, dim3(cdiv((long long)M * N, 256), batch), dim3(256), 0, st, M, N,
                         splitk, ws, C, ldc, sc, bias, beta);
    DL4SS_CHECK_LAUNCH();
    return 0;
  }
#define GGL_LAUNCH(EPI_)                                                                                         \
  hipLaunchKernelGGL((gemm_gl_kernel<A_KC, B_KC, EPI_, false, CF>), grid, dim3(CF::NT), 0, st, M, N, K, A, lda, B, \
                     ldb, C, ldc, bias, beta, kps, gm, gn, sa, sb, sc, nullptr)
  if (epi == EPI_TANH) GGL_LAUNCH(EPI_TANH);
  else if (epi == EPI_TANH_BF16) GGL_LAUNCH(EPI_TANH_BF16);
  else GGL_LAUNCH(EPI_NONE);
#undef GGL_LAUNCH
  DL4SS_CHECK_LAUNCH();
  return 0;
}

// split-K slabs + fixed-order reduce of a split launch (any configuration)
int launch_reduce(int M, int N, int splitk, int batch, float* C, long long ldc, long long sc, const float* bias,
                  float beta, float* ws, hipStream_t st) {
  if (N % 4 == 0 && ldc % 4 == 0 && sc % 4 == 0 && ((uintptr_t)C & 15) == 0)
    hipLaunchKernelGGL(gemm_gl_reduce_kernel<true>, dim3(cdiv((long long)M * N / 4, 256), batch), dim3(256), 0, st, M,
                       N, splitk, ws, C, ldc, sc, bias, beta);
  else
    hipLaunchKernelGGL(gemm_gl_reduce_kernel<false>, dim3(cdiv((long long)M * N, 256), batch), dim3(256), 0, st, M, N,
                       splitk, ws, C, ldc, sc, bias, beta);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

// the 256 x 256 ping-pong configuration (gemm_pp_kernel) with SL half-tile slots
template <bool A_KC, bool B_KC, int SL>
int launch_pp(int M, int N, int K, const unsigned short* A, long long lda, const unsigned short* B, long long ldb,
              float* C, long long ldc, const float* bias, int epi, float beta, int splitk, int batch, long long sa,
              long long sb, long long sc, float* ws, long long ws_bytes, hipStream_t st) {
  const int gm = (M + pp::BM - 1) / pp::BM, gn = (N + pp::BM - 1) / pp::BM;
  int kps = (K + splitk - 1) / splitk;
  kps = (kps + BK - 1) / BK * BK;
  splitk = (K + kps - 1) / kps;
  dim3 grid(gm * gn, batch, splitk);
  if (splitk > 1) {
    if (epi != EPI_NONE && epi != EPI_SPLIT_SLABS) return (int)hipErrorInvalidValue;
    const long long need = (long long)batch * splitk * M * N * 4;
    if (!ws || ws_bytes < need) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm_pp_kernel<A_KC, B_KC, EPI_NONE, true, SL>), grid, dim3(pp::NT), 0, st, M, N, K, A, lda, B,
                       ldb, C, ldc, nullptr, 0.0f, kps, gm, gn, sa, sb, sc, ws);
    DL4SS_CHECK_LAUNCH();
    if (epi == EPI_SPLIT_SLABS) return 0;
    return launch_reduce(M, N, splitk, batch, C, ldc, sc, bias, beta, ws, st);
  }
#define GPP_LAUNCH(EPI_)                                                                                            \
  hipLaunchKernelGGL((gemm_pp_kernel<A_KC, B_KC, EPI_, false, SL>), grid, dim3(pp::NT), 0, st, M, N, K, A, lda, B, ldb, \
                     C, ldc, bias, beta, kps, gm, gn, sa, sb, sc, nullptr)
  if (epi == EPI_TANH) GPP_LAUNCH(EPI_TANH);
  else if (epi == EPI_TANH_BF16) GPP_LAUNCH(EPI_TANH_BF16);
  else GPP_LAUNCH(EPI_NONE);
#undef GPP_LAUNCH
  DL4SS_CHECK_LAUNCH();
  return 0;
}

template <bool A_KC, bool B_KC>
int launch(int M, int N, int K, const unsigned short* A, long long lda, const unsigned short* B, long long ldb,
           float* C, long long ldc, const float* bias, int epi, float beta, int splitk, int batch, long long sa,
           long long sb, long long sc, float* ws, long long ws_bytes, hipStream_t st) {
  const int cfg = g_gl_cfg ? g_gl_cfg : gl_cfg_for(M, N, K, splitk, batch);
#define GGL_ARGS M, N, K, A, lda, B, ldb, C, ldc, bias, epi, beta, splitk, batch, sa, sb, sc, ws, ws_bytes, st
  if (cfg == 4) return launch_pp<A_KC, B_KC, 8>(GGL_ARGS);
  if (cfg == 5) return launch_pp<A_KC, B_KC, 10>(GGL_ARGS);
  if (cfg == 2) return launch_cfg<A_KC, B_KC, C256>(GGL_ARGS);
  if (cfg == 3) return launch_cfg<A_KC, B_KC, C128S3>(GGL_ARGS);
  if (cfg == 6) return launch_cfg<A_KC, B_KC, C128D5>(GGL_ARGS);
  if (cfg == 7) return launch_cfg<A_KC, B_KC, C128D4>(GGL_ARGS);
  if (cfg == 8) return launch_cfg<A_KC, B_KC, C128H2>(GGL_ARGS);
  // (64-row A images exist only in the k-contiguous layout: a k-major A runs the 128 x 128 tile)
  if (cfg == 9) return A_KC ? launch_cfg<A_KC, B_KC, C64>(GGL_ARGS) : launch_cfg<A_KC, B_KC, C128>(GGL_ARGS);
  return launch_cfg<A_KC, B_KC, C128>(GGL_ARGS);
#undef GGL_ARGS
}

}  // namespace

// Tuning knob (tools/gemm_gl_bench.py): tile configuration of gemm_gl (0 = per shape, 1 =
// 128 x 128 double buffer, 2 = 256 x 128 three stages, 3 = 128 x 128 three stages, 4 = 256 x
// 256 ping-pong, 128 KB LDS, 5 = the same with the whole 160 KB: six half-tiles in flight, 6 / 7 =
// 128 x 128 deep ring: five / four 32-deep k-tile stages, four / three k-tiles in flight, 8 = 128 x 128
// 32-deep double buffer, four workgroups per CU, 9 = 64 x 128 tiles, three workgroups per CU).
DL4SS_API int dl4ss_gemm_gl_set_config(int cfg) {
  DL4SS_REQUIRE(cfg >= 0 && cfg <= 9);
  g_gl_cfg = cfg;
  return 0;
}

// Workspace bytes dl4ss_gemm_bf16_gl needs for a split-K launch (0 without split-K).
DL4SS_API long long dl4ss_gemm_bf16_gl_ws_bytes(int M, int N, int K, int splitk, int batch) {
  if (splitk <= 1 || M <= 0 || N <= 0 || K <= 0 || batch < 1) return 0;
  int kps = (K + splitk - 1) / splitk;
  kps = (kps + BK - 1) / BK * BK;
  const int s = (K + kps - 1) / kps;
  return s > 1 ? (long long)batch * s * M * N * 4 : 0;
}

// C = op(A) op(B) (+ bias) (epilogue), bf16 operands, the layout conventions of dl4ss_gemm (strided batch)
// (transA: A stored K x M; transB: B stored N x K).  Requires 16-B aligned operand rows (ld %
// 8 == 0, aligned bases, strides % 8 == 0); returns hipErrorInvalidValue otherwise.  k-major
// operands are bounded per k-row (exact for any K); a k-contiguous operand is read in 8-element
// chunks, so with K % 8 != 0 its rows must hold zeros in [K, K rounded up to 8) (ld >= that):
// the producers' zero-padded bf16 rows.  splitk > 1: deterministic split-K through ws
// (dl4ss_gemm_bf16_gl_ws_bytes), EPI_NONE only.
DL4SS_API int dl4ss_gemm_bf16_gl(int transA, int transB, int M, int N, int K, const void* A, long long lda,
                                 const void* B, long long ldb, float* C, long long ldc, const float* bias, int epilogue,
                                 float beta, int splitk, int batch, long long strideA, long long strideB,
                                 long long strideC, void* ws, long long ws_bytes, void* stream) {
  DL4SS_REQUIRE(M >= 0 && N >= 0 && K >= 0 && A && B && C && batch >= 1 && batch <= 65535);
  if (M == 0 || N == 0) return 0;
  DL4SS_REQUIRE(K > 0 && lda % 8 == 0 && ldb % 8 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 &&
                strideA % 8 == 0 && strideB % 8 == 0);
  if (splitk < 1) splitk = 1;
  const bool a_kc = !transA, b_kc = transB;
  const int k8 = (K + 7) & ~7;
  DL4SS_REQUIRE(!a_kc || lda >= k8);
  DL4SS_REQUIRE(!b_kc || ldb >= k8);
  // split points fall on 64-element k boundaries: a chunk straddles K only in the last split
  // a KM operand's rows are read in 16-B chunks: the row stride must cover the chunk past the last row
  DL4SS_REQUIRE(a_kc || lda >= ((M + 7) & ~7));
  DL4SS_REQUIRE(b_kc || ldb >= ((N + 7) & ~7));
  if (epilogue == EPI_TANH_BF16)
    DL4SS_REQUIRE(beta == 0.0f && splitk == 1 && (ldc & 1) == 0 && ((uintptr_t)C & 3) == 0);
  // split slabs only: the effective split (after the 64-k rounding) must still be > 1, no bias / beta
  if (epilogue == EPI_SPLIT_SLABS)
    DL4SS_REQUIRE(bias == nullptr && beta == 0.0f && dl4ss_gemm_bf16_gl_ws_bytes(M, N, K, splitk, batch) > 0);
  DL4SS_REQUIRE(epilogue >= EPI_NONE && epilogue <= EPI_SPLIT_SLABS);
  hipStream_t st = as_stream(stream);
  const auto* a = reinterpret_cast<const unsigned short*>(A);
  const auto* b = reinterpret_cast<const unsigned short*>(B);
  float* w = reinterpret_cast<float*>(ws);
#define GGL_ARGS M, N, K, a, lda, b, ldb, C, ldc, bias, epilogue, beta, splitk, batch, strideA, strideB, strideC, w, ws_bytes, st
  if (a_kc && b_kc) return launch<true, true>(GGL_ARGS);
  if (a_kc && !b_kc) return launch<true, false>(GGL_ARGS);
  if (!a_kc && b_kc) return launch<false, true>(GGL_ARGS);
  return launch<false, false>(GGL_ARGS);
#undef GGL_ARGS
}

// Workspace bytes of dl4ss_gemm_bf16_gl_grouped: the split-K slabs of every problem, each at a
// 256-B aligned offset.
DL4SS_API long long dl4ss_gemm_bf16_gl_grouped_ws_bytes(int n, const int* M, const int* N, const int* K,
                                                         const int* splitk) {
  if (n < 1 || n > GMAXP || !M || !N || !K || !splitk) return -1;
  long long tot = 0;
  for (int i = 0; i < n; ++i) {
    const long long b = dl4ss_gemm_bf16_gl_ws_bytes(M[i], N[i], K[i], splitk[i], 1);
    tot += (b + 255) / 256 * 256;
  }
  return tot;
}

namespace {
// the grouped launch in tile configuration CF over `grid` workgroups (<= 0: one per tile)
template <class CF>
int grouped_launch(int n, bool a_kc, bool b_kc, const int* M, const int* N, const int* K, const void* const* A,
                   const long long* lda, const void* const* B, const long long* ldb, float* const* C,
                   const long long* ldc, const float* beta, const int* splitk, void* ws, long long ws_bytes, int grid,
                   size_t dyn_lds, float* const* rsum, hipStream_t st) {
  GlGroup g{};
  bool any_rs = false;
  long long off = 0;
  int wg = 0, units = 0;
  char* w = reinterpret_cast<char*>(ws);
  for (int i = 0; i < n; ++i) {
    DL4SS_REQUIRE(M[i] > 0 && N[i] > 0 && K[i] > 0 && A[i] && B[i] && C[i]);
    DL4SS_REQUIRE(lda[i] % 8 == 0 && ldb[i] % 8 == 0 && ((uintptr_t)A[i] & 15) == 0 && ((uintptr_t)B[i] & 15) == 0);
    const int k8 = (K[i] + 7) & ~7;
    DL4SS_REQUIRE(!a_kc || lda[i] >= k8);
    DL4SS_REQUIRE(!b_kc || ldb[i] >= k8);
    DL4SS_REQUIRE(a_kc || lda[i] >= ((M[i] + 7) & ~7));
    DL4SS_REQUIRE(b_kc || ldb[i] >= ((N[i] + 7) & ~7));
    GlProb& p = g.p[i];
    p.A = reinterpret_cast<const unsigned short*>(A[i]);
    p.B = reinterpret_cast<const unsigned short*>(B[i]);
    p.C = C[i];
    p.lda = lda[i]; p.ldb = ldb[i]; p.ldc = ldc[i];
    p.beta = beta[i];
    p.M = M[i]; p.N = N[i]; p.K = K[i];
    p.gm = (M[i] + CF::BM - 1) / CF::BM;
    p.gn = (N[i] + BN - 1) / BN;
    int sk = splitk[i] < 1 ? 1 : splitk[i];
    int kps = (K[i] + sk - 1) / sk;
    kps = (kps + BK - 1) / BK * BK;
    sk = (K[i] + kps - 1) / kps;
    p.nsplit = sk;
    p.kps = kps;
    p.wg0 = wg;
    wg += p.gm * p.gn * sk;
    p.part = nullptr;
    p.vec = (N[i] % 4 == 0 && ldc[i] % 4 == 0 && ((uintptr_t)C[i] & 15) == 0) ? 1 : 0;
    p.rsum = rsum ? rsum[i] : nullptr;
    DL4SS_REQUIRE(!p.rsum || sk == 1);  // row sums are formed by unsplit tiles only
    any_rs = any_rs || p.rsum != nullptr;
    p.u0 = units;
    if (sk > 1) {
      const long long b = (long long)sk * M[i] * N[i] * 4;
      DL4SS_REQUIRE(w && off + b <= ws_bytes);
      p.part = reinterpret_cast<float*>(w + off);
      off += (b + 255) / 256 * 256;
      const long long mn = (long long)M[i] * N[i];
      units += (int)(p.vec ? mn / 4 : mn);
    }
  }
  g.n = n;
  g.total_wg = wg;
  g.total_units = units;
  const int nwg = grid > 0 && grid < wg ? grid : wg;
#define GGR(AK, BKC) \
  hipLaunchKernelGGL((gemm_gl_grouped_kernel<AK, BKC, CF>), dim3(nwg), dim3(CF::NT), dyn_lds, st, g)
  if (any_rs) {  // the side-stream dW_lin: A k-major (dPre^T), B k-major (h)
    DL4SS_REQUIRE(!a_kc && !b_kc);
    hipLaunchKernelGGL((gemm_gl_grouped_kernel<false, false, CF, true>), dim3(nwg), dim3(CF::NT), dyn_lds, st, g);
  } else if (a_kc && b_kc) GGR(true, true);
  else if (a_kc) GGR(true, false);
  else if (b_kc) GGR(false, true);
  else GGR(false, false);
#undef GGR
  DL4SS_CHECK_LAUNCH();
  if (units > 0) {
    hipLaunchKernelGGL(gemm_gl_grouped_reduce_kernel, dim3(cdiv(units, 256)), dim3(256), 0, st, g);
    DL4SS_CHECK_LAUNCH();
  }
  return 0;
}
}  // namespace

// Grouped C_i = op(A_i) op(B_i) + beta_i C_i for i < n (n <= 16) in ONE launch (+ one split-K combine
// launch): the backward's weight gradients.  Every problem has the layout rules of
// dl4ss_gemm_bf16_gl with the SAME transA / transB, no bias, EPI_NONE; splitk[i] as there (the
// same slabs and fixed-order sums, so each C_i is bitwise the single launch's).
DL4SS_API int dl4ss_gemm_bf16_gl_grouped(int n, int transA, int transB, const int* M, const int* N, const int* K,
                                         const void* const* A, const long long* lda, const void* const* B,
                                         const long long* ldb, float* const* C, const long long* ldc,
                                         const float* beta, const int* splitk, void* ws, long long ws_bytes,
                                         void* stream) {
  DL4SS_REQUIRE(n >= 1 && n <= GMAXP && M && N && K && A && lda && B && ldb && C && ldc && beta && splitk);
  return grouped_launch<C128>(n, !transA, transB, M, N, K, A, lda, B, ldb, C, ldc, beta, splitk, ws, ws_bytes, 0, 0,
                              nullptr, as_stream(stream));
}

// The persistent form: `grid` workgroups walk the group's tiles (grid <= 0: one per tile, as
// dl4ss_gemm_bf16_gl_grouped), in tile configuration cfg (1 = 128 x 128 double buffer; 2 = 256 x
// 128, three stages, 144 KB LDS: one workgroup per CU; 6 / 7 = 128 x 128 deep ring of five / four
// 32-deep stages, two workgroups per CU); one_per_cu pads cfg 1's LDS so that one
// workgroup fills a CU.  rowsum (NULL, or n pointers, each NULL or M_i floats): rowsum_i[m] =
// beta_i rowsum_i[m] + sum_k op(A_i)(m, k) for unsplit problems with both operands k-major (the
// Linear's bias gradient beside its weight gradient).  For a side stream beside the persistent recurrence, which leaves the CUs
// above its co-residency budget free (dl4ss_birnn_plan_info).
DL4SS_API int dl4ss_gemm_bf16_gl_grouped_ex(int n, int transA, int transB, const int* M, const int* N, const int* K,
                                            const void* const* A, const long long* lda, const void* const* B,
                                            const long long* ldb, float* const* C, const long long* ldc,
                                            const float* beta, const int* splitk, void* ws, long long ws_bytes,
                                            int grid, int cfg, int one_per_cu, float* const* rowsum, void* stream) {
  DL4SS_REQUIRE(n >= 1 && n <= GMAXP && M && N && K && A && lda && B && ldb && C && ldc && beta && splitk);
  DL4SS_REQUIRE(cfg == 1 || cfg == 2 || cfg == 6 || cfg == 7);
  hipStream_t st = as_stream(stream);
  if (cfg == 6)
    return grouped_launch<C128D5>(n, !transA, transB, M, N, K, A, lda, B, ldb, C, ldc, beta, splitk, ws, ws_bytes,
                                  grid, 0, rowsum, st);
  if (cfg == 7)
    return grouped_launch<C128D4>(n, !transA, transB, M, N, K, A, lda, B, ldb, C, ldc, beta, splitk, ws, ws_bytes,
                                  grid, 0, rowsum, st);
  if (cfg == 2)
    return grouped_launch<C256>(n, !transA, transB, M, N, K, A, lda, B, ldb, C, ldc, beta, splitk, ws, ws_bytes, grid,
                                0, rowsum, st);
  // C128 holds 64 KB: 20 KB more dynamic LDS leaves room for only one workgroup per CU
  return grouped_launch<C128>(n, !transA, transB, M, N, K, A, lda, B, ldb, C, ldc, beta, splitk, ws, ws_bytes, grid,
                              one_per_cu ? 20 * 1024 : 0, rowsum, st);
}
