// HBM ceiling probe for MI355X: streaming read (reduce) and copy of a 400 MB fp32
// buffer with several launch shapes.  Reports the best achievable GB/s, the
// measured ceiling quoted next to the 8 TB/s spec in DESIGN.md.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_hbm.hip -o probe_hbm && ./probe_hbm
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int U>
__global__ __launch_bounds__(256) void read_grid_stride(const float4* __restrict__ x, long n4, float* out) {
  float acc = 0.f;
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (i + u * 256 < n4) ? x[i + u * 256] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

// one tile per block (like topk_stream): TILE float4 per block, wave-contiguous ranges
template <int U, int TILE4>
__global__ __launch_bounds__(256) void read_tiles(const float4* __restrict__ x, long n4, float* out) {
  float acc = 0.f;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long wbeg = (long)blockIdx.x * TILE4 + w * (TILE4 / 4);
  const long wend = wbeg + TILE4 / 4 < n4 ? wbeg + TILE4 / 4 : n4;
  for (long b = wbeg; b < wend; b += 64 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (b + u * 64 + lane < wend) ? x[b + u * 64 + lane] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

__global__ __launch_bounds__(256) void copy_k(const float4* __restrict__ x, float4* __restrict__ y, long n4) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) y[i] = x[i];
}

template <class F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const long n = 100000000, n4 = n / 4;
  float4 *x, *y;
  float* out;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(x, 0x3c, n * 4));
  const double bytes = n * 4.0;
  int grids[] = {1024, 2048, 4096, 8192, 16384};
  for (int g : grids) {
    float ms = time_ms([&] { hipLaunchKernelGGL(read_grid_stride<4>, dim3(g), dim3(256), 0, 0, x, n4, out); }, 20);
    printf("read grid-stride U=4 grid=%5d : %8.1f us  %7.1f GB/s\n", g, ms * 1e3, bytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL(read_grid_stride<8>, dim3(g), dim3(256), 0, 0, x, n4, out); }, 20);
    printf("read grid-stride U=8 grid=%5d : %8.1f us  %7.1f GB/s\n", g, ms * 1e3, bytes / ms / 1e6);
  }
  {
    const int T4 = 8192;  // 32768 floats per block, as topk_stream
    const int g = (int)((n4 + T4 - 1) / T4);
    float ms = time_ms([&] { hipLaunchKernelGGL((read_tiles<4, T4>), dim3(g), dim3(256), 0, 0, x, n4, out); }, 20);
    printf("read tiles 32K/block U=4      : %8.1f us  %7.1f GB/s\n", ms * 1e3, bytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((read_tiles<8, T4>), dim3(g), dim3(256), 0, 0, x, n4, out); }, 20);
    printf("read tiles 32K/block U=8      : %8.1f us  %7.1f GB/s\n", ms * 1e3, bytes / ms / 1e6);
    const int T4b = 32768;
    const int gb = (int)((n4 + T4b - 1) / T4b);
    ms = time_ms([&] { hipLaunchKernelGGL((read_tiles<8, T4b>), dim3(gb), dim3(256), 0, 0, x, n4, out); }, 20);
    printf("read tiles 128K/block U=8     : %8.1f us  %7.1f GB/s\n", ms * 1e3, bytes / ms / 1e6);
  }
  for (int g : grids) {
    float ms = time_ms([&] { hipLaunchKernelGGL(copy_k, dim3(g), dim3(256), 0, 0, x, y, n4); }, 20);
    printf("copy grid=%5d                 : %8.1f us  %7.1f GB/s (read+write)\n", g, ms * 1e3, 2 * bytes / ms / 1e6);
  }
  return 0;
}
