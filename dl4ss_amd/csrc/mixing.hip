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
#include "common.h"

namespace {

// one workgroup per source: fp64 mean and max|x - mean| over its first len samples (a
// shorter wav of a list file is normalised over its own length, then zero-padded:
// predata_fromList_cRM_123.py:186-198)
__global__ __launch_bounds__(256) void source_stats_kernel(const float* __restrict__ raw, int NS,
                                                           const int* __restrict__ lens, float2* __restrict__ stats) {
  const float* x = raw + (long long)blockIdx.x * NS;
  const int N = lens ? min(max(lens[blockIdx.x], 0), NS) : NS;
  __shared__ double sd[4];
  __shared__ float sm[4];
  double s = 0.0;
  for (int i = threadIdx.x * 4; i < N; i += 1024) {
    if (i + 3 < N && (NS & 3) == 0) {
      const float4 v = *reinterpret_cast<const float4*>(x + i);
      s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
    } else {
      for (int k = i; k < N && k < i + 4; ++k) s += x[k];
    }
  }
  s = wave_sum_d(s);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sd[w] = s;
  __syncthreads();
  const double mean = N > 0 ? (sd[0] + sd[1] + sd[2] + sd[3]) / N : 0.0;
  const float meanf = (float)mean;
  float m = 0.f;
  for (int i = threadIdx.x; i < N; i += 256) m = fmaxf(m, fabsf(x[i] - meanf));
  m = wave_max(m);
  if (l == 0) sm[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float mx = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    stats[blockIdx.x] = make_float2(meanf, mx > 0.f ? 1.0f / mx : 0.f);
  }
}

// grid (ceil(N/1024), B): normalise, gain, write sources and their sum
__global__ __launch_bounds__(256) void mix_kernel(const float* __restrict__ raw, const float2* __restrict__ stats,
                                                  const float* __restrict__ gains, const int* __restrict__ lens,
                                                  int K, int N, float* __restrict__ out_src,
                                                  float* __restrict__ out_mix) {
  const int b = blockIdx.y;
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= N) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k = 0; k < K; ++k) {
    const long long src = (long long)b * K + k;
    const float2 st = stats[src];
    const float g = gains[src] * st.y;
    const float* x = raw + src * N;
    float* o = out_src + ((long long)b * K + k) * N;
    const int len = lens ? min(max(lens[src], 0), N) : N;  // zero beyond the source's own length
    if (i + 3 < len && ((N & 3) == 0)) {
      float4 v = *reinterpret_cast<const float4*>(x + i);
      v.x = (v.x - st.x) * g; v.y = (v.y - st.x) * g; v.z = (v.z - st.x) * g; v.w = (v.w - st.x) * g;
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

DL4SS_API int dl4ss_mix_sources_ex(const float* raw, const int* lengths, const float* gains, int B, int K, int N,
                                   float* stats_ws, float* out_src, float* out_mix, void* stream) {
  DL4SS_REQUIRE(raw && gains && out_src && out_mix && stats_ws && B >= 0 && K >= 1 && N > 0);
  if (B == 0) return 0;
  hipLaunchKernelGGL(source_stats_kernel, dim3(B * K), dim3(256), 0, as_stream(stream), raw, N, lengths,
                     reinterpret_cast<float2*>(stats_ws));
  DL4SS_CHECK_LAUNCH();
  hipLaunchKernelGGL(mix_kernel, dim3(cdiv(N, 1024), B), dim3(256), 0, as_stream(stream), raw,
                     reinterpret_cast<const float2*>(stats_ws), gains, lengths, K, N, out_src, out_mix);
  DL4SS_CHECK_LAUNCH();
  return 0;
}

DL4SS_API int dl4ss_mix_sources(const float* raw, const float* gains, int B, int K, int N, float* stats_ws,
                                float* out_src, float* out_mix, void* stream) {
  return dl4ss_mix_sources_ex(raw, nullptr, gains, B, K, N, stats_ws, out_src, out_mix, stream);
}
