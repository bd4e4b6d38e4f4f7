// Probe: what does one workgroup barrier cost on MI355X in the top-k kernels'
// shape (1024-thread workgroups, one per CU via a large LDS footprint)?  Times
// (s_memrealtime, 100 MHz) the launch skew of the 16 waves, then runs 64
// barriers back to back (with and without a little LDS work between them),
// with and without a global-load flood in flight from every wave.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_barrier.hip -o tools/probe_barrier && tools/probe_barrier
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

template <int FLOOD>
__global__ __launch_bounds__(1024) void k_bar(const float4* __restrict__ x, unsigned long long* t, unsigned* out) {
  __shared__ unsigned big[32768];  // 128 KiB: one workgroup per CU
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const unsigned long long t0 = wall_clock64();
  float4 a[8];
  if (FLOOD) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = x[((size_t)blockIdx.x * 16 + w) * 512 + u * 64 + lane];
  }
  big[tid] = tid;
  __syncthreads();
  const unsigned long long t1 = wall_clock64();
  unsigned acc = 0;
  for (int i = 0; i < 64; ++i) {
    __syncthreads();
  }
  const unsigned long long t2 = wall_clock64();
  for (int i = 0; i < 64; ++i) {
    big[(tid * 7 + i) & 32767] += 1u;
    __syncthreads();
    acc += big[(tid * 13 + i) & 32767];
  }
  const unsigned long long t3 = wall_clock64();
  if (FLOOD) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += __float_as_uint(a[u].x);
  }
  if (lane == 0) {
    t[(blockIdx.x * 16 + w) * 4 + 0] = t0;
    t[(blockIdx.x * 16 + w) * 4 + 1] = t1;
    t[(blockIdx.x * 16 + w) * 4 + 2] = t2;
    t[(blockIdx.x * 16 + w) * 4 + 3] = t3;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const int g = 256;
  float4* x;
  unsigned* out;
  unsigned long long* t;
  CK(hipMalloc(&x, (size_t)g * 16 * 512 * 16));
  CK(hipMemset(x, 0, (size_t)g * 16 * 512 * 16));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&t, g * 16 * 4 * 8));
  static unsigned long long h[g * 16 * 4];
  auto run = [&](auto kern, const char* name) {
    hipLaunchKernelGGL(kern, dim3(g), dim3(1024), 0, 0, x, t, out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost));
    double skew = 0, first = 0, bars = 0, ldsbars = 0;
    for (int b = 0; b < g; ++b) {
      unsigned long long mn = ~0ull, mx = 0;
      for (int w = 0; w < 16; ++w) {
        mn = h[(b * 16 + w) * 4] < mn ? h[(b * 16 + w) * 4] : mn;
        mx = h[(b * 16 + w) * 4] > mx ? h[(b * 16 + w) * 4] : mx;
      }
      skew += (mx - mn);
      first += h[(b * 16) * 4 + 1] - mn;
      bars += h[(b * 16) * 4 + 2] - h[(b * 16) * 4 + 1];
      ldsbars += h[(b * 16) * 4 + 3] - h[(b * 16) * 4 + 2];
    }
    printf("%-8s wave launch skew %6.2f us  first barrier after first wave %6.2f us  64 bare barriers %6.2f us"
           "  64 barriers + LDS rmw %6.2f us\n",
           name, skew / g * 0.01, first / g * 0.01, bars / g * 0.01, ldsbars / g * 0.01);
  };
  for (int it = 0; it < 2; ++it) {
    run(k_bar<0>, "idle");
    run(k_bar<1>, "flood");
  }
  return 0;
}
