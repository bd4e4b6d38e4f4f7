// Cold instruction-fetch cost on gfx950: one pass over a straight-line block of
// N 4-byte VALU instructions, timed (wall_clock64, 100 MHz) on its first and its
// second execution by every workgroup.  Question it answers: does code that a
// workgroup runs once (the one-launch top-k's select + emission tail) pay an
// instruction-cache miss per line?
//   hipcc --offload-arch=gfx950 -O3 tools/probe_icache.hip -o tools/probe_icache
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define R4(x) x x x x
#define R16(x) R4(R4(x))
#define R256(x) R16(R16(x))
#define R1K(x) R4(R256(x))

template <int KB>
__global__ void probe(unsigned long long* out, int passes) {
  unsigned v = threadIdx.x;
  for (int p = 0; p < passes; ++p) {
    unsigned long long t0 = wall_clock64();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // KB KiB of v_xor_b32 (4 bytes each): 256 instructions per KiB
    if constexpr (KB >= 1) asm volatile(R256("v_xor_b32 %0, 1, %0\n") : "+v"(v));
    if constexpr (KB >= 2) asm volatile(R256("v_xor_b32 %0, 1, %0\n") : "+v"(v));
    if constexpr (KB >= 4) asm volatile(R256("v_xor_b32 %0, 1, %0\n") R256("v_xor_b32 %0, 1, %0\n") : "+v"(v));
    if constexpr (KB >= 8) asm volatile(R1K("v_xor_b32 %0, 1, %0\n") : "+v"(v));
    if constexpr (KB >= 16) asm volatile(R1K("v_xor_b32 %0, 1, %0\n") R1K("v_xor_b32 %0, 1, %0\n") : "+v"(v));
    if constexpr (KB >= 32) asm volatile(R1K("v_xor_b32 %0, 1, %0\n") R1K("v_xor_b32 %0, 1, %0\n") R1K("v_xor_b32 %0, 1, %0\n") R1K("v_xor_b32 %0, 1, %0\n") : "+v"(v));
    asm volatile("s_nop 0" ::: "memory");
    unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) out[blockIdx.x * 4 + p] = t1 - t0;
  }
  if (v == 0xFFFFFFFFu) out[0] = 0;  // keep v live
}

template <int KB>
void run(int nwg) {
  unsigned long long* d;
  hipMalloc(&d, nwg * 4 * 8);
  hipMemset(d, 0, nwg * 32);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe<KB>, dim3(nwg), dim3(64), 0, 0, d, 3);
    hipDeviceSynchronize();
  }
  std::vector<unsigned long long> h(nwg * 4);
  hipMemcpy(h.data(), d, nwg * 32, hipMemcpyDeviceToHost);
  for (int p = 0; p < 3; ++p) {
    std::vector<double> t;
    for (int b = 0; b < nwg; ++b) t.push_back(h[b * 4 + p] * 0.01);
    std::sort(t.begin(), t.end());
    printf("code %2d KiB, %4d workgroups, pass %d: median %.2f us, max %.2f us\n", KB, nwg, p, t[nwg / 2], t.back());
  }
  hipFree(d);
}

int main() {
  run<1>(256); run<4>(256); run<16>(256); run<32>(256);
  run<16>(1); run<16>(8);
  return 0;
}
