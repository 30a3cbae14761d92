// HBM streaming-ceiling probe (standalone; not part of the library).  Measures what plain,
// perfectly coalesced 16-B-per-lane streams reach on this MI355X for the traffic mixes of the
// step's HBM-bound kernels, so their roofline fractions can be read against a measured ceiling
// as well as the 8 TB/s spec:
//   read      : 1 read stream (sum kept live)
//   write     : 1 write stream
//   copy      : 1 read : 1 write
//   r1w3      : 1 read : 3 writes (the STFT's complex + magnitude mix: 128 KB in, ~388 KB out
//               per 4 s signal)
//   copy_nt   : copy with non-temporal stores
// Each kernel moves ~2.1 GB per launch (the STFT probe's size); grid-stride over 16-B elements,
// 256-thread workgroups, grid = 8 x 256 CUs x 4.  Build: hipcc --offload-arch=gfx950 -O3
// tools/bw_probe.hip -o tools/bw_probe ; run: ./tools/bw_probe  (one JSON line per kernel)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ a, long long n, float* __restrict__ sink) {
  float s = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1.2345f) sink[threadIdx.x] = s;  // keeps the loads live, never true for the fill
}

__global__ __launch_bounds__(256) void k_write(float4* __restrict__ b, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    b[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ a, float4* __restrict__ b, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = a[i];
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy_nt(const f32x4* __restrict__ a, f32x4* __restrict__ b, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    __builtin_nontemporal_store(a[i], b + i);
}

__global__ __launch_bounds__(256) void k_r1w3(const float4* __restrict__ a, float4* __restrict__ b,
                                              float4* __restrict__ c, float4* __restrict__ d, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float4 v = a[i];
    b[i] = v;
    c[i] = make_float4(v.y, v.x, v.w, v.z);
    d[i] = make_float4(v.x * v.x, v.y * v.y, v.z * v.z, v.w * v.w);
  }
}

template <class F>
float time_ms(F launch, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

int main() {
  const long long bytes_stream = 528LL << 20;  // 528 MiB per stream: 2.2 GB for r1w3
  const long long n = bytes_stream / 16;
  float4 *a, *b, *c, *d;
  float* sink;
  CK(hipMalloc(&a, bytes_stream));
  CK(hipMalloc(&b, bytes_stream));
  CK(hipMalloc(&c, bytes_stream));
  CK(hipMalloc(&d, bytes_stream));
  CK(hipMalloc(&sink, 1024));
  CK(hipMemset(a, 0, bytes_stream));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int mult : {4, 8, 16}) {
    const dim3 grid(cus * mult), blk(256);
    const int it = 20;
    struct R { const char* name; int streams; float ms; };
    R rs[5] = {
        {"read", 1, time_ms([&] { hipLaunchKernelGGL(k_read, grid, blk, 0, 0, a, n, sink); }, it)},
        {"write", 1, time_ms([&] { hipLaunchKernelGGL(k_write, grid, blk, 0, 0, b, n); }, it)},
        {"copy", 2, time_ms([&] { hipLaunchKernelGGL(k_copy, grid, blk, 0, 0, a, b, n); }, it)},
        {"copy_nt", 2, time_ms([&] { hipLaunchKernelGGL(k_copy_nt, grid, blk, 0, 0, (const f32x4*)a, (f32x4*)b, n); }, it)},
        {"r1w3", 4, time_ms([&] { hipLaunchKernelGGL(k_r1w3, grid, blk, 0, 0, a, b, c, d, n); }, it)},
    };
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    for (const R& r : rs) {
      const double gbs = (double)r.streams * bytes_stream / (r.ms * 1e-3) / 1e9;
      printf("{\"kernel\": \"%s\", \"wg_per_cu\": %d, \"bytes\": %lld, \"ms\": %.4f, \"GB/s\": %.1f, \"frac_8TBs\": %.3f}\n",
             r.name, mult, (long long)r.streams * bytes_stream, r.ms, gbs, gbs / 8000.0);
    }
  }
  return 0;
}
