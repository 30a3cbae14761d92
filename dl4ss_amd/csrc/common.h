// Shared helpers for the dl4ss HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DL4SS_API extern "C" __attribute__((visibility("default")))

// Timing-experiment macros that drop stores (results wrong) are accepted only in the experiment
// variant libraries tools/variant_lib.py builds (it defines DL4SS_VARIANT_BUILD): a stray -D in a
// product build stops the compile instead of shipping a library that silently skips work.
#if !defined(DL4SS_VARIANT_BUILD) && (defined(FWD_EXP_SKIP) || defined(BWD_EXP_NO_DG) || defined(GGL_NO_STORE) || \
                                      defined(RNN_EXP_MINIMAL) || defined(DL4SS_EXP_ZS_PAD))
#error "FWD_EXP_SKIP / BWD_EXP_NO_DG / GGL_NO_STORE / RNN_EXP_MINIMAL / DL4SS_EXP_ZS_PAD are for tools/variant_lib.py builds only"
#endif

#define DL4SS_CHECK_LAUNCH()                        \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return (int)_e;           \
  } while (0)

#define DL4SS_REQUIRE(cond)                                   \
  do {                                                        \
    if (!(cond)) return (int)hipErrorInvalidValue;            \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline unsigned cdiv(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// fp32 -> bf16 bits, round to nearest even.  A NaN stays a quiet NaN: the plain rounding add
// carries a NaN with high mantissa bits (e.g. 0x7FFFFFFF) into the exponent / sign (-> -0 or
// inf) and would hide a non-finite weight or feature from the C3 hazard and the guards.
__device__ __forceinline__ unsigned bf16_bits_rne(float f) {
  const unsigned u = __float_as_uint(f);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (u >> 16) | 0x40u;
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// Wave64 reductions (CDNA wavefront is 64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
