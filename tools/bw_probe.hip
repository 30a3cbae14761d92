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
//   write_dword / r1w3_dword : the same streams with one dword per lane (256 B per wave-instruction)
//   write_rows_dword : MI355X_MICROARCH.md's store form -- one dword per lane into random 2,304-B
//               rows of a 302 MB table, each row swept by 9 consecutive wave-instructions
// Each kernel moves ~2.1 GB per launch (the STFT probe's size); grid-stride over 16-B elements,
// 256-thread workgroups, grid = {2, 4, 8, 16} workgroups per CU.  Build: hipcc --offload-arch=gfx950 -O3
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

// one dword per lane: 256 B per wave-instruction, the wave sweeping consecutive 256-B pieces
__global__ __launch_bounds__(256) void k_write_dw(float* __restrict__ b, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = (float)i;
}

// MI355X_MICROARCH.md's store measurement: one dword per lane into random 2,304-B rows of a table,
// each row swept by consecutive wave-instructions (9 x 256 B), one wave per row at a time
__global__ __launch_bounds__(256) void k_write_rows(float* __restrict__ b, long long nrows, int rows_per_wave,
                                                   unsigned seed) {
  const int lane = threadIdx.x & 63;
  const long long w = blockIdx.x * 4LL + (threadIdx.x >> 6);
  for (int r = 0; r < rows_per_wave; ++r) {
    unsigned h = (unsigned)(w * rows_per_wave + r) * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    float* row = b + (long long)(h % (unsigned)nrows) * 576;  // 2,304 B
#pragma unroll
    for (int c = 0; c < 9; ++c) row[c * 64 + lane] = (float)c;
  }
}

// r1w3 with dword-per-lane accesses (the same bytes as k_r1w3)
__global__ __launch_bounds__(256) void k_r1w3_dw(const float* __restrict__ a, float* __restrict__ b,
                                                 float* __restrict__ c, float* __restrict__ d, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float v = a[i];
    b[i] = v;
    c[i] = -v;
    d[i] = v * v;
  }
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
  for (int mult : {2, 4, 8, 16}) {
    const dim3 grid(cus * mult), blk(256);
    const int it = 20;
    const long long nrows = (302LL << 20) / 2304;  // a 302 MB table (beyond the 256 MB Infinity Cache)
    const int rpw = 64;
    const long long rows_bytes = (long long)cus * mult * 4 * rpw * 2304;
    struct R { const char* name; double bytes; float ms; };
    R rs[8] = {
        {"read", 1.0 * bytes_stream, time_ms([&] { hipLaunchKernelGGL(k_read, grid, blk, 0, 0, a, n, sink); }, it)},
        {"write", 1.0 * bytes_stream, time_ms([&] { hipLaunchKernelGGL(k_write, grid, blk, 0, 0, b, n); }, it)},
        {"write_dword", 1.0 * bytes_stream,
         time_ms([&] { hipLaunchKernelGGL(k_write_dw, grid, blk, 0, 0, (float*)b, 4 * n); }, it)},
        {"write_rows_dword", 1.0 * rows_bytes,
         time_ms([&] { hipLaunchKernelGGL(k_write_rows, grid, blk, 0, 0, (float*)c, nrows, rpw, 12345u); }, it)},
        {"copy", 2.0 * bytes_stream, time_ms([&] { hipLaunchKernelGGL(k_copy, grid, blk, 0, 0, a, b, n); }, it)},
        {"copy_nt", 2.0 * bytes_stream, time_ms([&] { hipLaunchKernelGGL(k_copy_nt, grid, blk, 0, 0, (const f32x4*)a, (f32x4*)b, n); }, it)},
        {"r1w3", 4.0 * bytes_stream, time_ms([&] { hipLaunchKernelGGL(k_r1w3, grid, blk, 0, 0, a, b, c, d, n); }, it)},
        {"r1w3_dword", 4.0 * bytes_stream,
         time_ms([&] { hipLaunchKernelGGL(k_r1w3_dw, grid, blk, 0, 0, (const float*)a, (float*)b, (float*)c, (float*)d, 4 * n); }, it)},
    };
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    for (const R& r : rs) {
      const double gbs = r.bytes / (r.ms * 1e-3) / 1e9;
      printf("{\"kernel\": \"%s\", \"wg_per_cu\": %d, \"bytes\": %.0f, \"ms\": %.4f, \"GB/s\": %.1f, \"frac_8TBs\": %.3f}\n",
             r.name, mult, r.bytes, r.ms, gbs, gbs / 8000.0);
    }
  }
  return 0;
}
