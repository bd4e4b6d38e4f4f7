// Does a streaming read's per-workgroup time depend on buffer position when the
// same 400 MB buffer is read back to back (Infinity Cache retention)?  Stamps
// every workgroup's start/end (wall_clock64) for a contiguous-tile read (the
// top-k stream kernel's shape) and a tile-interleaved read, reports the median
// duration per eighth of the buffer and the kernel span.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_position.hip -o tools/probe_position
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

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

// tile t = TT float4 (4 waves x TT/4 contiguous); workgroup g processes tiles
// g, g + G, g + 2G, ... (G = gridDim.x); interleave=false => one tile per workgroup
// map: 0 = tile g; 1 = reversed (tile G-1-g); 2 = XCD-local (workgroups of XCD g%8
// read the contiguous eighth g%8 of the tiles)
template <int U>
__global__ __launch_bounds__(256, 8) void k_tiles(const float4* __restrict__ x, long n4, long TT, long ntiles,
                                                  unsigned* out, unsigned long long* st, int map) {
  unsigned acc = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) st[2 * blockIdx.x] = wall_clock64();
  long first = blockIdx.x;
  if (map == 1) first = gridDim.x - 1 - blockIdx.x;
  if (map == 2) first = (long)(blockIdx.x % 8) * ((gridDim.x + 7) / 8) + blockIdx.x / 8;
  for (long t = first; t < ntiles; t += gridDim.x) {
    const long beg = t * TT + w * (TT / 4);
    const long end = beg + TT / 4 < n4 ? beg + TT / 4 : n4;
    for (long b = beg; b + 64 * U <= end; b += 64 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = x[b + u * 64 + lane];
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= fold(v[u]);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) st[2 * blockIdx.x + 1] = wall_clock64();
  if (acc == 0x12345678u) out[0] = acc;
}

static void report(const char* label, const std::vector<unsigned long long>& s, int G, bool by_region) {
  unsigned long long t0 = ~0ull, t1 = 0;
  std::vector<double> all;
  for (int g = 0; g < G; ++g) {
    t0 = std::min(t0, s[2 * g]);
    t1 = std::max(t1, s[2 * g + 1]);
    all.push_back((s[2 * g + 1] - s[2 * g]) * 0.01);
  }
  std::vector<double> srt = all;
  std::sort(srt.begin(), srt.end());
  printf("%-52s span %7.2f us  wg min/med/max %6.1f %6.1f %6.1f", label, (t1 - t0) * 0.01, srt.front(),
         srt[srt.size() / 2], srt.back());
  if (by_region) {
    printf(" | per eighth:");
    for (int q = 0; q < 8; ++q) {
      std::vector<double> d(all.begin() + (long)q * G / 8, all.begin() + (long)(q + 1) * G / 8);
      std::nth_element(d.begin(), d.begin() + d.size() / 2, d.end());
      printf(" %5.1f", d[d.size() / 2]);
    }
  }
  printf("\n");
}

int main() {
  const long n = 100000000, n4 = n / 4;
  float4* x;
  unsigned* out;
  unsigned long long* st;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&st, 2 * 65536 * sizeof(unsigned long long)));
  CK(hipMemset(x, 0x3c, n * 4));
  std::vector<unsigned long long> h(2 * 65536);
  const long TT = 12288;  // 192 KB tiles, one per workgroup (top-k stream shape)
  const long ntiles = (n4 + TT - 1) / TT;
  const int G = (int)ntiles;
  const char* names[3] = {"tile = wg id", "tile = reversed wg id", "XCD-local eighths"};
  for (int map = 0; map < 3; ++map) {
    for (int rep = 0; rep < 4; ++rep) {
      hipLaunchKernelGGL((k_tiles<4>), dim3(G), dim3(256), 0, 0, x, n4, TT, ntiles, out, st, map);
      CK(hipGetLastError());
    }
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), st, 2 * G * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    // per-eighth medians by WORKGROUP id (dispatch order) and by TILE position
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int g = 0; g < G; ++g) { t0 = std::min(t0, h[2 * g]); t1 = std::max(t1, h[2 * g + 1]); }
    printf("%-24s span %7.2f us\n", names[map], (t1 - t0) * 0.01);
    for (int by = 0; by < 3; ++by) {
      printf("   median wg time by %-14s:", by == 0 ? "wg id eighth" : (by == 1 ? "tile eighth" : "XCD (wg%8)"));
      for (int q = 0; q < 8; ++q) {
        std::vector<double> d;
        for (int g = 0; g < G; ++g) {
          long tile = g;
          if (map == 1) tile = G - 1 - g;
          if (map == 2) tile = (long)(g % 8) * ((G + 7) / 8) + g / 8;
          const int key = by == 0 ? (int)((long)g * 8 / G) : (by == 1 ? (int)(tile * 8 / ntiles) : g % 8);
          if (key == q) d.push_back((h[2 * g + 1] - h[2 * g]) * 0.01);
        }
        if (d.empty()) { printf("     -"); continue; }
        std::nth_element(d.begin(), d.begin() + d.size() / 2, d.end());
        printf(" %5.1f", d[d.size() / 2]);
      }
      printf("\n");
    }
  }
  return 0;
}
