// VALU issue rate on gfx950: every wave of a 1024-thread workgroup (16 waves, 4 per SIMD)
// runs R rounds of 4 INDEPENDENT v_xor_b32 chains (ILP 4) -- the throughput case -- and
// a one-wave workgroup runs the same -- the latency case.  Reports cycles per wave-
// instruction per SIMD (wall_clock64 at 100 MHz, shader clock from the command line).
//   hipcc --offload-arch=gfx950 -O3 tools/probe_valu.hip -o tools/probe_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define R4(x) x x x x
#define R16(x) R4(R4(x))
#define R64(x) R4(R16(x))
#define BODY "v_xor_b32 %0, 1, %0\n v_xor_b32 %1, 1, %1\n v_xor_b32 %2, 1, %2\n v_xor_b32 %3, 1, %3\n"

__global__ void probe(unsigned long long* out, int rounds) {
  unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  __syncthreads();
  unsigned long long t0 = wall_clock64();
  for (int r = 0; r < rounds; ++r) asm volatile(R64(BODY) : "+v"(a), "+v"(b), "+v"(c), "+v"(d));  // 256 instr
  __syncthreads();
  unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if ((a ^ b ^ c ^ d) == 0x12345678u) out[0] = 0;
}

void run(int threads, int nwg, int rounds, double ghz) {
  unsigned long long* d;
  hipMalloc(&d, nwg * 8);
  for (int rep = 0; rep < 3; ++rep) { hipLaunchKernelGGL(probe, dim3(nwg), dim3(threads), 0, 0, d, rounds); hipDeviceSynchronize(); }
  std::vector<unsigned long long> h(nwg);
  hipMemcpy(h.data(), d, nwg * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double us = h[nwg / 2] * 0.01;
  const double waves_per_simd = std::max(1.0, threads / 64 / 4.0);
  const double instr = 256.0 * rounds * waves_per_simd;  // wave-instructions per SIMD
  printf("%4d threads x %4d WGs, %d x 256 instr per wave: %.2f us -> %.2f cycles per wave-instruction per SIMD at %.1f GHz\n",
         threads, nwg, rounds, us, us * 1e3 * ghz / instr, ghz);
  hipFree(d);
}

int main(int argc, char** argv) {
  double ghz = argc > 1 ? atof(argv[1]) : 2.4;
  run(64, 256, 64, ghz);
  run(256, 256, 64, ghz);
  run(1024, 256, 64, ghz);
  run(1024, 512, 64, ghz);
  return 0;
}
