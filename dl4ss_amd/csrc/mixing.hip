// Source preprocessing and mixing on device.
//
// Restates, per source: x -= mean(x); x /= max|x|; x *= gain; mixture = sum_k x
// (Torch_multi/predata_multiAims_dB.py:156-197,
//  Torch_multi/predata_multiAims_3dB.py:192-217,
//  TDAA_beta/predata_fromList_cRM_123.py:186-237).  The reference does this in
// float64 numpy; here the mean and peak are reduced in fp64/fp32 and the
// scaled sources are stored fp32 (the STFT's input precision).
//
// Layout: raw (B, K, N) fp32 -> scaled sources (B, K, N) and mixture (B, N), each
// contiguous so that one STFT launch covers all sources and one all mixtures.
//
// Train-time augmentation (config.AUGMENT_DATA): after the normalisation each source is
// rotated by a per-source shift s, signal = np.append(signal[s:], signal[:s]), BEFORE the
// zero-padding, i.e. over the source's own length len (TDAA_beta/predata_fromList.py:150-151,
// TDAA_beta/predata_fromList_cRM_123.py:198-200).  Mean and peak are rotation-invariant, so the
// statistics pass is unchanged and the mixing pass reads x[(i + s) mod len].
#include "common.h"

namespace {

// Statistics of a source over its first len samples (a shorter wav of a list file is
// normalised over its own length, then zero-padded: predata_fromList_cRM_123.py:186-198):
// NSPLIT workgroups per source each reduce one chunk in ONE pass to {fp64 sum, min, max};
// the mixing kernel combines the NSPLIT partials in fixed order.  max|x - m| is taken as
// max(max x - m, m - min x): fp32 subtraction is monotonic, so this equals the per-element
// max of |fl(x - m)| exactly (the previous form re-read the source in a second pass).
constexpr int NSPLIT = 8;
struct SrcPart {
  double sum;
  float mn, mx;
};
static_assert(sizeof(SrcPart) == 16, "16-B partials");

__global__ __launch_bounds__(256) void source_stats_kernel(const float* __restrict__ raw, int NS,
                                                           const int* __restrict__ lens, SrcPart* __restrict__ part) {
  const int src = blockIdx.x, p = blockIdx.y;
  const float* x = raw + (long long)src * NS;
  const int N = lens ? min(max(lens[src], 0), NS) : NS;
  const int chunk = ((N + NSPLIT - 1) / NSPLIT + 3) & ~3;
  const int i0 = min(N, p * chunk), i1 = min(N, i0 + chunk);
  double s = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  const bool vec = (NS & 3) == 0;
  for (int i = i0 + threadIdx.x * 4; i < i1; i += 1024) {
    if (vec && i + 3 < i1) {
      const float4 v = *reinterpret_cast<const float4*>(x + i);
      s += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
      mn = fminf(fminf(mn, fminf(v.x, v.y)), fminf(v.z, v.w));
      mx = fmaxf(fmaxf(mx, fmaxf(v.x, v.y)), fmaxf(v.z, v.w));
    } else {
      for (int k = i; k < i1 && k < i + 4; ++k) {
        s += x[k];
        mn = fminf(mn, x[k]);
        mx = fmaxf(mx, x[k]);
      }
    }
  }
  s = wave_sum_d(s);
  mx = wave_max(mx);
  mn = -wave_max(-mn);
  __shared__ double sd[4];
  __shared__ float smn[4], smx[4];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) { sd[w] = s; smn[w] = mn; smx[w] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    SrcPart r;
    r.sum = (sd[0] + sd[1]) + (sd[2] + sd[3]);
    r.mn = fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3]));
    r.mx = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
    part[src * NSPLIT + p] = r;
  }
}

// grid (ceil(N/1024), B): normalise, gain, write sources and their sum.  fp contraction is off
// here: hipcc fuses (x - m) * g + acc into one fma by default (and __fmul_rn is a plain
// product), which would make the mixture differ in the last bit from the sum of the stored
// sources (the reference's wav_mix = wav_mix + signal, predata_fromList_cRM_123.py:225-229)
__global__ __launch_bounds__(256) void mix_kernel(const float* __restrict__ raw, const SrcPart* __restrict__ part,
                                                  const float* __restrict__ gains, const int* __restrict__ lens,
                                                  const int* __restrict__ shifts, int K, int N,
                                                  float* __restrict__ out_src,
                                                  float* __restrict__ out_mix) {
#pragma clang fp contract(off)
  const int b = blockIdx.y;
  // per-source (mean, 1 / max|x - mean|) from the NSPLIT partials, fixed order; the shift
  // reduced modulo the source's length (0 = no rotation)
  __shared__ float2 sstat[16];
  __shared__ int sshift[16];
  if (threadIdx.x < K) {
    const long long src = (long long)b * K + threadIdx.x;
    const int len = lens ? min(max(lens[src], 0), N) : N;
    double s = 0.0;
    float mn = INFINITY, mx = -INFINITY;
    for (int p = 0; p < NSPLIT; ++p) {
      const SrcPart r = part[src * NSPLIT + p];
      s += r.sum;
      mn = fminf(mn, r.mn);
      mx = fmaxf(mx, r.mx);
    }
    const float meanf = len > 0 ? (float)(s / len) : 0.f;
    const float pk = len > 0 ? fmaxf(mx - meanf, meanf - mn) : 0.f;
    sstat[threadIdx.x] = make_float2(meanf, pk > 0.f ? 1.0f / pk : 0.f);
    int sh = 0;
    if (shifts && len > 0) {
      sh = shifts[src] % len;
      if (sh < 0) sh += len;
    }
    sshift[threadIdx.x] = sh;
  }
  __syncthreads();
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= N) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k = 0; k < K; ++k) {
    const long long src = (long long)b * K + k;
    const float2 st = sstat[k];
    const float g = gains[src] * st.y;
    const float* x = raw + src * N;
    float* o = out_src + ((long long)b * K + k) * N;
    const int len = lens ? min(max(lens[src], 0), N) : N;  // zero beyond the source's own length
    const int sh = sshift[k];
    if (sh != 0) {  // rotated: out[i] = x[(i + sh) mod len] for i < len
      float* a = &acc.x;
      for (int q = 0; q < 4 && i + q < N; ++q) {
        float v = 0.0f;
        if (i + q < len) {
          int j = i + q + sh;
          j -= j >= len ? len : 0;
          v = (x[j] - st.x) * g;
        }
        o[i + q] = v;
        a[q] += v;
      }
    } else if (i + 3 < len && ((N & 3) == 0)) {
      float4 v = *reinterpret_cast<const float4*>(x + i);
      v.x = (v.x - st.x) * g; v.y = (v.y - st.x) * g;
      v.z = (v.z - st.x) * g; v.w = (v.w - st.x) * g;
      *reinterpret_cast<float4*>(o + i) = v;
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    } else {
      float* a = &acc.x;
      for (int q = 0; q < 4 && i + q < N; ++q) {
        const float v = i + q < len ? (x[i + q] - st.x) * g : 0.0f;
        o[i + q] = v;
        a[q] += v;
      }
    }
  }
  float* m = out_mix + (long long)b * N;
  if (i + 3 < N && ((N & 3) == 0)) {
    *reinterpret_cast<float4*>(m + i) = acc;
  } else {
    const float* a = &acc.x;
    for (int q = 0; q < 4 && i + q < N; ++q) m[i + q] = a[q];
  }
}

}  // namespace

DL4SS_API int dl4ss_mix_sources_rot(const float* raw, const int* lengths, const int* shifts, const float* gains,
                                    int B, int K, int N, float* stats_ws, float* out_src, float* out_mix,
                                    void* stream) {
  DL4SS_REQUIRE(B >= 0 && K >= 1 && K <= 16 && N > 0);
  if (B == 0) return 0;  // empty batch: no-op (an empty tensor's pointer may be null)
  DL4SS_REQUIRE(raw && gains && out_src && out_mix && stats_ws);
  DL4SS_REQUIRE(((uintptr_t)stats_ws & 15) == 0);
  SrcPart* part = reinterpret_cast<SrcPart*>(stats_ws);
  hipLaunchKernelGGL(source_stats_kernel, dim3(B * K, NSPLIT), dim3(256), 0, as_stream(stream), raw, N, lengths, part);
  DL4SS_CHECK_LAUNCH();
  hipLaunchKernelGGL(mix_kernel, dim3(cdiv(N, 1024), B), dim3(256), 0, as_stream(stream), raw, part, gains, lengths,
                     shifts, K, N, out_src, out_mix);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_mix_sources_ex(const float* raw, const int* lengths, const float* gains, int B, int K, int N,
                                   float* stats_ws, float* out_src, float* out_mix, void* stream) {
  return dl4ss_mix_sources_rot(raw, lengths, nullptr, gains, B, K, N, stats_ws, out_src, out_mix, stream);
}

DL4SS_API int dl4ss_mix_sources(const float* raw, const float* gains, int B, int K, int N, float* stats_ws,
                                float* out_src, float* out_mix, void* stream) {
  return dl4ss_mix_sources_ex(raw, nullptr, gains, B, K, N, stats_ws, out_src, out_mix, stream);
}
