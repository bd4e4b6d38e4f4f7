// Probe: cost of executing straight-line code the first time (cold instruction
// cache) vs the second time, on every CU at once (one 1024-thread workgroup per
// CU, like the top-k kernels).  The body is ~kOps dependent VALU ops unrolled
// (several KiB of code); each pass is timed with s_memrealtime (100 MHz).
//   hipcc -O3 --offload-arch=gfx950 tools/probe_icache.hip -o tools/probe_icache && tools/probe_icache
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

template <int kOps>
__global__ __launch_bounds__(1024) void k_code(unsigned* out, unsigned long long* t, unsigned seed) {
  unsigned a = threadIdx.x ^ seed, b = seed * 3u + 1u;
  for (int rep = 0; rep < 3; ++rep) {
    __syncthreads();
    const unsigned long long t0 = wall_clock64();
#pragma unroll
    for (int i = 0; i < kOps; ++i) {
      a = a * 0x9E3779B1u + b;
      b ^= a >> (i & 15);
    }
    __syncthreads();
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) t[(blockIdx.x * 3 + rep)] = t1 - t0;
  }
  if (a == 0x12345678u) out[0] = b;
}

int main() {
  const int g = 256;
  unsigned* out;
  unsigned long long* t;
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&t, g * 3 * 8));
  unsigned long long h[g * 3];
  auto run = [&](auto kern, const char* name) {
    hipLaunchKernelGGL(kern, dim3(g), dim3(1024), 0, 0, out, t, 7u);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost));
    double s[3] = {0, 0, 0};
    for (int b = 0; b < g; ++b)
      for (int r = 0; r < 3; ++r) s[r] += h[b * 3 + r];
    printf("%-10s pass1 %7.2f us  pass2 %7.2f us  pass3 %7.2f us (mean over %d workgroups)\n", name,
           s[0] / g * 0.01, s[1] / g * 0.01, s[2] / g * 0.01, g);
  };
  for (int it = 0; it < 2; ++it) {
    run(k_code<256>, "ops256");
    run(k_code<1024>, "ops1024");
    run(k_code<4096>, "ops4096");
  }
  return 0;
}
