// Scattered-access ceiling probe for MI355X: what a sparse accumulate of k sorted
// random indices into 100M-float buffers can cost, independent of the codec.
//   gather1 : v += a[i]                      (one buffer, read only)
//   gather2 : v += a[i] + b[i]               (two buffers, read only)
//   rmw1    : a[i] += v                      (one buffer)
//   rmw2    : a[i] += v; b[i] += w * v       (the CHOCO self accumulate)
//   rmw2_u  : rmw2 with the indices in random (unsorted) order
//   rmw2_ln : rmw2 where each update owns a whole 64-B line (16 floats RMW'd)
// Each at k = 1M, 2M and 4M; the time per touched line gives the HBM
// random-transaction rate the accumulate is bound by.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_scatter.hip -o tools/probe_scatter && tools/probe_scatter
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void gather1(const float* __restrict__ a, const int* __restrict__ idx, int k, float* out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k) return;
  float v = a[idx[t]];
  if (v == 1234.5f) out[0] = v;
}
__global__ void gather2(const float* __restrict__ a, const float* __restrict__ b, const int* __restrict__ idx, int k,
                        float* out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k) return;
  int i = idx[t];
  float v = a[i] + b[i];
  if (v == 1234.5f) out[0] = v;
}
__global__ void rmw1(float* __restrict__ a, const int* __restrict__ idx, const float* __restrict__ val, int k) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k) return;
  int i = idx[t];
  a[i] += val[t];
}
__global__ void rmw2(float* __restrict__ a, float* __restrict__ b, const int* __restrict__ idx,
                     const float* __restrict__ val, int k, float w) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k) return;
  int i = idx[t];
  float v = val[t];
  a[i] += v;
  b[i] += w * v;
}
// whole 64-B line per update: 16 lanes per line, line index = idx[t] / 16
__global__ void rmw2_line(float* __restrict__ a, float* __restrict__ b, const int* __restrict__ idx,
                          const float* __restrict__ val, int k, float w) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long u = t >> 4;
  if (u >= k) return;
  long i = (long)(idx[u] & ~15) + (t & 15);
  float v = val[u];
  a[i] += v;
  b[i] += w * v;
}

int main() {
  const long n = 100000000;
  float *a, *b, *val, *out;
  int* idx;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMemset(a, 0, n * 4));
  CK(hipMemset(b, 0, n * 4));
  const int kmax = 4000000;
  CK(hipMalloc(&val, kmax * 4));
  CK(hipMalloc(&idx, kmax * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(val, 0, kmax * 4));
  // a 512 MB buffer written between repetitions: evicts / dirties the Infinity Cache
  float* junk;
  CK(hipMalloc(&junk, 512l << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::mt19937_64 rng(7);
  for (int k : {1000000, 2000000, 4000000}) {
    // k distinct uniform indices (the top-k of a random buffer), sorted ascending
    std::vector<int> h(k);
    {
      std::vector<uint8_t> seen(n, 0);
      int c = 0;
      while (c < k) {
        long i = (long)(rng() % (uint64_t)n);
        if (!seen[i]) { seen[i] = 1; h[c++] = (int)i; }
      }
    }
    std::sort(h.begin(), h.end());
    std::vector<int> hu(h);
    std::shuffle(hu.begin(), hu.end(), rng);
    long lines = 0;
    for (int j = 0; j < k; ++j) if (j == 0 || h[j] / 16 != h[j - 1] / 16) ++lines;
    for (int mode = 0; mode < 6; ++mode) {
      CK(hipMemcpy(idx, mode == 4 ? hu.data() : h.data(), (size_t)k * 4, hipMemcpyHostToDevice));
      const char* nm[] = {"gather1", "gather2", "rmw1", "rmw2", "rmw2_u", "rmw2_ln"};
      float best = 1e9f, sum = 0.f;
      const int reps = 10;
      for (int r = 0; r < reps + 2; ++r) {
        CK(hipMemsetAsync(junk, r & 1, 512l << 20, 0));
        CK(hipEventRecord(e0, 0));
        const int g = (k + 255) / 256;
        switch (mode) {
          case 0: gather1<<<g, 256>>>(a, idx, k, out); break;
          case 1: gather2<<<g, 256>>>(a, b, idx, k, out); break;
          case 2: rmw1<<<g, 256>>>(a, idx, val, k); break;
          case 3: case 4: rmw2<<<g, 256>>>(a, b, idx, val, k, 0.5f); break;
          case 5: rmw2_line<<<(unsigned)(((long)k * 16 + 255) / 256), 256>>>(a, b, idx, val, k, 0.5f); break;
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) { best = std::min(best, ms); sum += ms; }
      }
      const int nbuf = (mode == 0 || mode == 2) ? 1 : 2;
      const bool rmw = mode >= 2;
      const double us = 1e3 * sum / reps;
      // line transactions: one read per touched line per buffer (+ one write-back for RMW)
      const double tx = (double)lines * nbuf * (rmw ? 2 : 1);
      printf("k=%d lines=%ld %-8s mean %.1f us (best %.1f)  %.1f G line-transactions/s\n", k, lines, nm[mode], us,
             1e3 * best, tx / us * 1e-3);
    }
  }
  return 0;
}
