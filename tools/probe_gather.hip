// Random-gather / scattered-RMW rate probe for MI355X with a CLEAN cache state:
// k sorted distinct uniform indices into n = 100M floats, sources rotated over
// four 400 MB buffers (1.6 GB >> the 256 MB Infinity Cache) and fresh indices per
// repetition.  Unlike tools/probe_scatter.hip nothing dirties the caches before a
// timed launch, so no write-back of a previous memset is timed with it.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_gather.hip -o tools/probe_gather && tools/probe_gather
//   g<U>     : each thread gathers U indices (strided by the grid), all loads first
//   rmw2<U>  : a[i] += v; b[i] += w v (the CHOCO self accumulate), U per thread
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e = (x);                                         \
    if (e != hipSuccess) {                                      \
      printf("%s: %s\n", #x, hipGetErrorString(e));             \
      exit(1);                                                  \
    }                                                           \
  } while (0)

template <int U>
__global__ __launch_bounds__(256) void gat(const float* __restrict__ a, const int* __restrict__ idx, int k,
                                           float* __restrict__ out) {
  const int t0 = blockIdx.x * 256 * U + threadIdx.x;
  int j[U];
  float v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) j[u] = t0 + u * 256 < k ? idx[t0 + u * 256] : -1;
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = j[u] >= 0 ? a[j[u]] : 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (j[u] >= 0) out[t0 + u * 256] = v[u];
}

template <int U>
__global__ __launch_bounds__(256) void rmw2(float* __restrict__ a, float* __restrict__ b,
                                            const int* __restrict__ idx, const float* __restrict__ val, int k,
                                            float w) {
  const int t0 = blockIdx.x * 256 * U + threadIdx.x;
  int j[U];
  float v[U], x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    j[u] = t0 + u * 256 < k ? idx[t0 + u * 256] : -1;
    v[u] = j[u] >= 0 ? val[t0 + u * 256] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = j[u] >= 0 ? a[j[u]] : 0.f;
    y[u] = j[u] >= 0 ? b[j[u]] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (j[u] >= 0) {
      a[j[u]] = x[u] + v[u];
      b[j[u]] = y[u] + w * v[u];
    }
}

int main() {
  const long n = 100000000;
  float* src[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&src[i], n * 4));
    CK(hipMemset(src[i], 0, n * 4));
  }
  float *a, *b, *out, *val;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMemset(a, 0, n * 4));
  CK(hipMemset(b, 0, n * 4));
  const int kmax = 4000000;
  CK(hipMalloc(&out, kmax * 4));
  CK(hipMalloc(&val, kmax * 4));
  CK(hipMemset(val, 0, kmax * 4));
  const int nsets = 8;
  std::mt19937_64 rng(7);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int k : {1000000, 2000000}) {
    std::vector<int*> sets(nsets);
    for (int s = 0; s < nsets; ++s) {
      std::vector<int> h(k);
      // k distinct sorted uniform indices: Floyd-free -- sort + dedupe a 1.02 k draw, trim
      std::vector<int> d((size_t)(k * 1.02) + 64);
      std::uniform_int_distribution<int> U(0, (int)n - 1);
      for (auto& x : d) x = U(rng);
      std::sort(d.begin(), d.end());
      d.erase(std::unique(d.begin(), d.end()), d.end());
      std::shuffle(d.begin(), d.end(), rng);
      d.resize(k);
      std::sort(d.begin(), d.end());
      CK(hipMalloc(&sets[s], k * 4));
      CK(hipMemcpy(sets[s], d.data(), k * 4, hipMemcpyHostToDevice));
    }
    auto time = [&](const char* nm, auto launch) {
      std::vector<float> ts;
      for (int r = 0; r < 24; ++r) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        launch(r);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 4) ts.push_back(ms * 1000.f);
      }
      std::sort(ts.begin(), ts.end());
      printf("k=%d %-12s min %6.1f med %6.1f us  (%.1f G elem/s)\n", k, nm, ts[0], ts[ts.size() / 2],
             k / (ts[ts.size() / 2] * 1e3));
    };
    time("gather U1", [&](int r) { gat<1><<<(k + 255) / 256, 256>>>(src[r & 3], sets[r % nsets], k, out); });
    time("gather U4", [&](int r) { gat<4><<<(k + 1023) / 1024, 256>>>(src[r & 3], sets[r % nsets], k, out); });
    time("gather U8", [&](int r) { gat<8><<<(k + 2047) / 2048, 256>>>(src[r & 3], sets[r % nsets], k, out); });
    time("rmw2 U1", [&](int r) { rmw2<1><<<(k + 255) / 256, 256>>>(a, b, sets[r % nsets], val, k, 0.5f); });
    time("rmw2 U4", [&](int r) { rmw2<4><<<(k + 1023) / 1024, 256>>>(a, b, sets[r % nsets], val, k, 0.5f); });
    for (auto p : sets) CK(hipFree(p));
  }
  return 0;
}
