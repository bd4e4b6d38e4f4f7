// Probe: what does a trickle of candidate WRITES (or per-flush LDS work) cost a
// saturated streaming read on MI355X?  K2-shaped stream (one 16-wave workgroup
// per CU, 4096-element chunks claimed through an LDS counter, two 8-row register
// batches in flight per wave) over a 100M-fp32 buffer; every `every`-th batch a
// wave runs one "flush" of kind:
//   0 none
//   1 entries : one 16-B + one 4-B store per lane (1.25 KiB, coalesced)
//   2 pairs   : eight dword stores with ~8 active lanes each (scattered expand)
//   3 lds     : the flush's LDS work only (ds_read ring + ds_add histogram)
//   4 entries with sc1 (write-through) stores
//   5 entries with nt stores
//   hipcc -O3 --offload-arch=gfx950 tools/probe_wmix.hip -o tools/probe_wmix && tools/probe_wmix
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

constexpr int kW = 16, kU = 8, kChunk = 4096;

__device__ __forceinline__ unsigned fold(float4 v) {
  return __float_as_uint(v.x) ^ __float_as_uint(v.y) ^ __float_as_uint(v.z) ^ __float_as_uint(v.w);
}

template <int KIND>
__device__ __forceinline__ void flush(float4* ov, unsigned* oi, unsigned pos, unsigned acc, int lane, unsigned* lds,
                                      float4* ring) {
  if (KIND == 1 || KIND == 4 || KIND == 5) {
    float4 v = ring[lane];
    if (KIND == 1) {
      ov[pos + lane] = v;
      oi[pos + lane] = acc + lane;
    } else if (KIND == 4) {
      __hip_atomic_store(reinterpret_cast<unsigned*>(&ov[pos + lane]), __float_as_uint(v.x), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&oi[pos + lane], acc + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __builtin_nontemporal_store(v.x, &ov[pos + lane].x);
      __builtin_nontemporal_store(v.y, &ov[pos + lane].y);
      __builtin_nontemporal_store(v.z, &ov[pos + lane].z);
      __builtin_nontemporal_store(v.w, &ov[pos + lane].w);
      __builtin_nontemporal_store(acc + lane, &oi[pos + lane]);
    }
  } else if (KIND == 2) {
    float* o = reinterpret_cast<float*>(ov);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (((lane + c * 13) & 7) == 0) {
        o[4 * pos + 4 * lane + c] = (float)acc;
        oi[4 * pos + 4 * lane + c] = acc;
      }
    }
  } else if (KIND == 3) {
    float4 v = ring[lane];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned key = (__float_as_uint(c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w) >> 12) & 255u;
      if ((lane + c) & 1) atomicAdd(&lds[key], 1u);
    }
  }
}

template <int KIND>
__global__ __launch_bounds__(1024) void k_stream(const float* __restrict__ x, long n, unsigned tile, int every,
                                                 float4* ov, unsigned* oi, unsigned* out) {
  __shared__ unsigned next, hist[256];
  __shared__ float4 ring[kW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) next = kW;
  if (threadIdx.x < 256) hist[threadIdx.x] = 0;
  ring[w][lane] = make_float4(1.f, 2.f, 3.f, (float)lane);
  __syncthreads();
  const long tb = (long)blockIdx.x * tile;
  const unsigned nchunk = tile / kChunk;
  auto claim = [&]() {
    unsigned c = 0;
    if (lane == 0) c = atomicAdd(&next, 1u);
    return __builtin_amdgcn_readfirstlane(c);
  };
  auto load = [&](float4 (&r)[kU], long base) {
#pragma unroll
    for (int u = 0; u < kU; ++u) r[u] = *reinterpret_cast<const float4*>(x + base + u * 256 + 4 * lane);
  };
  auto b0 = [&](unsigned c) -> long {
    const long cb = tb + (long)c * kChunk;
    return (c < nchunk && cb + kChunk <= n) ? cb : 0;
  };
  unsigned acc = 0, nb = 0, pos = 0;
  unsigned c = w;
  float4 A[kU], B[kU];
  load(A, b0(c));
  unsigned nx = claim();
  while (c < nchunk) {
    const unsigned nn = claim();
    const long cb = tb + (long)c * kChunk;
    if (cb + kChunk <= n) {
      load(B, cb + 2048);
#pragma unroll
      for (int u = 0; u < kU; ++u) acc ^= fold(A[u]);
      if (KIND && ++nb % every == 0) flush<KIND>(ov + cb / 4, oi + cb / 4, (pos++ & 7) * 64, acc, lane, hist, ring[w]);
      load(A, b0(nx));
#pragma unroll
      for (int u = 0; u < kU; ++u) acc ^= fold(B[u]);
      if (KIND && ++nb % every == 0) flush<KIND>(ov + cb / 4, oi + cb / 4, (pos++ & 7) * 64, acc, lane, hist, ring[w]);
    }
    c = nx;
    nx = nn;
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
  float tot = 0.f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  CK(hipGetLastError());
  return tot * 1e3f / reps;
}

int main() {
  const long n = 100000000;
  const unsigned tile = 393216;
  const unsigned g = (unsigned)((n + tile - 1) / tile);
  float* x;
  float4* ov;
  unsigned *oi, *out;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&ov, (size_t)g * tile * 4));
  CK(hipMalloc(&oi, (size_t)g * tile * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(x, 0x3c, n * 4));
  const double gb = n * 4.0 / 1e3;
  const int everys[] = {1, 2, 3, 6};
#define RUN(K, E)                                                                                         \
  do {                                                                                                    \
    float us = time_us([&] { hipLaunchKernelGGL(k_stream<K>, dim3(g), dim3(1024), 0, 0, x, n, tile, E, ov, oi, out); }, \
                       10);                                                                               \
    printf("kind %d every %d batches: %8.1f us %8.1f GB/s read\n", K, E, us, gb / us);                   \
  } while (0)
  RUN(0, 1);
  for (int e : everys) {
    RUN(1, e);
    RUN(2, e);
    RUN(3, e);
    RUN(4, e);
    RUN(5, e);
  }
  RUN(0, 1);
  return 0;
}
