// Streaming-read shape probe for MI355X: which assignment of a large fp32 buffer
// to waves reaches the HBM ceiling?  Buffer 1.6 GB (>> 256 MB Infinity Cache) and
// 400 MB (the top-k bench size).  All kernels read every byte once and fold it
// into a register that is written only if it hits an impossible value.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_stream.hip -o tools/probe_stream && tools/probe_stream
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__device__ __forceinline__ unsigned fold(float4 v) {
  return __float_as_uint(v.x) ^ __float_as_uint(v.y) ^ __float_as_uint(v.z) ^ __float_as_uint(v.w);
}

// 1. block grid-stride: at every step the grid reads one contiguous window
template <int U>
__global__ __launch_bounds__(256) void k_grid_stride(const float4* __restrict__ x, long n4, unsigned* out) {
  unsigned acc = 0;
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i + (U - 1) * 256 < n4; i += stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= fold(v[u]);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// 2. each wave owns one contiguous region of R float4 (topk_stream's shape)
template <int U, int WPE>
__global__ __launch_bounds__(256, WPE) void k_wave_regions(const float4* __restrict__ x, long n4, long R,
                                                          unsigned* out) {
  unsigned acc = 0;
  const int lane = threadIdx.x & 63;
  const long wg = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long beg = wg * R, end = beg + R < n4 ? beg + R : n4;
  for (long b = beg; b + 64 * U <= end; b += 64 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[b + u * 64 + lane];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= fold(v[u]);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// 3. each block owns a contiguous tile of T float4; its 4 waves interleave U-row
//    chunks, so a block reads one contiguous 4*U KB window per step
template <int U, int WPE>
__global__ __launch_bounds__(256, WPE) void k_block_rows(const float4* __restrict__ x, long n4, long T,
                                                        unsigned* out) {
  unsigned acc = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long beg = (long)blockIdx.x * T, end = beg + T < n4 ? beg + T : n4;
  for (long b = beg + (long)w * 64 * U; b + 64 * U <= end; b += 4 * 64 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[b + u * 64 + lane];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= fold(v[u]);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// 4. persistent waves, 4*U KB chunks dealt round-robin over all waves
template <int U, int WPE>
__global__ __launch_bounds__(256, WPE) void k_wave_chunks(const float4* __restrict__ x, long n4, unsigned* out) {
  unsigned acc = 0;
  const int lane = threadIdx.x & 63;
  const long nw = (long)gridDim.x * 4;
  const long wg = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (long b = wg * 64 * U; b + 64 * U <= n4; b += nw * 64 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[b + u * 64 + lane];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= fold(v[u]);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <class F>
static float time_us(F f, int reps) {
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
  CK(hipGetLastError());
  return ms * 1e3f / reps;
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const long nmax = 400000000;
  float4* x;
  unsigned* out;
  CK(hipMalloc(&x, nmax * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(x, 0x3c, nmax * 4));
  const long sizes[] = {nmax, 100000000};
  for (long n : sizes) {
    const long n4 = n / 4;
    const double gb = n * 4.0 / 1e3;  // bytes / us -> GB/s
    printf("=== %ld floats (%.1f MB), %d CUs\n", n, n * 4.0 / 1e6, cus);
#define REP(label, ...)                                                       \
  do {                                                                        \
    float us = time_us([&] { __VA_ARGS__; }, 10);                             \
    printf("%-44s %9.1f us %8.1f GB/s\n", label, us, gb / us);                \
  } while (0)
    REP("grid-stride U4 g1024", hipLaunchKernelGGL(k_grid_stride<4>, dim3(1024), dim3(256), 0, 0, x, n4, out));
    REP("grid-stride U4 g2048", hipLaunchKernelGGL(k_grid_stride<4>, dim3(2048), dim3(256), 0, 0, x, n4, out));
    REP("grid-stride U8 g2048", hipLaunchKernelGGL(k_grid_stride<8>, dim3(2048), dim3(256), 0, 0, x, n4, out));
    const long regs[] = {1024, 3072, 12288};
    for (long R : regs) {
      const unsigned g = (unsigned)((n4 + 4 * R - 1) / (4 * R));
      char lab[64];
      snprintf(lab, sizeof lab, "wave-regions R=%ldKB U4 wpe8 g%u", R * 16 / 1024, g);
      REP(lab, hipLaunchKernelGGL((k_wave_regions<4, 8>), dim3(g), dim3(256), 0, 0, x, n4, R, out));
      snprintf(lab, sizeof lab, "wave-regions R=%ldKB U8 wpe8 g%u", R * 16 / 1024, g);
      REP(lab, hipLaunchKernelGGL((k_wave_regions<8, 8>), dim3(g), dim3(256), 0, 0, x, n4, R, out));
      snprintf(lab, sizeof lab, "wave-regions R=%ldKB U16 wpe4 g%u", R * 16 / 1024, g);
      REP(lab, hipLaunchKernelGGL((k_wave_regions<16, 4>), dim3(g), dim3(256), 0, 0, x, n4, R, out));
    }
    const long tiles[] = {4096, 12288, 49152};
    for (long T : tiles) {
      const unsigned g = (unsigned)((n4 + T - 1) / T);
      char lab[64];
      snprintf(lab, sizeof lab, "block-rows T=%ldKB U4 wpe8 g%u", T * 16 / 1024, g);
      REP(lab, hipLaunchKernelGGL((k_block_rows<4, 8>), dim3(g), dim3(256), 0, 0, x, n4, T, out));
      snprintf(lab, sizeof lab, "block-rows T=%ldKB U8 wpe8 g%u", T * 16 / 1024, g);
      REP(lab, hipLaunchKernelGGL((k_block_rows<8, 8>), dim3(g), dim3(256), 0, 0, x, n4, T, out));
    }
    const int bpcs[] = {4, 8};
    for (int bpc : bpcs) {
      const unsigned g = (unsigned)(cus * bpc);
      char lab[64];
      snprintf(lab, sizeof lab, "wave-chunks U4 g%u", g);
      REP(lab, hipLaunchKernelGGL((k_wave_chunks<4, 8>), dim3(g), dim3(256), 0, 0, x, n4, out));
      snprintf(lab, sizeof lab, "wave-chunks U8 g%u", g);
      REP(lab, hipLaunchKernelGGL((k_wave_chunks<8, 8>), dim3(g), dim3(256), 0, 0, x, n4, out));
    }
  }
  return 0;
}
