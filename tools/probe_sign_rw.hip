// Access-pattern probe for the fused sign receive (sign_recv_pack1_kernel): read x, x_hat,
// memory and write all three back (24 bytes per element, 345M elements), no sign work.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_sign_rw.hip -o tools/probe_sign_rw && tools/probe_sign_rw [n]
// Shapes:
//   col<RU>   : the kernel's column tiles -- a 256-thread workgroup owns 1024 columns of the
//               (32, N') view, lane l the float4 at its run offset of each row, RU rows per
//               group, two groups in flight, nt loads and stores
//   colh<RU>  : the same with each workgroup covering 16 of the 32 rows (twice the workgroups)
//   flat      : contiguous 4096-element tiles (the QSGD receive's shape), 2 x 8 elements per
//               thread in flight, default-policy loads and stores
// Two sets of arrays alternate (no Infinity-Cache reuse); min / median of 20 launches each.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s: %s\n", #x, hipGetErrorString(e));         \
      exit(1);                                              \
    }                                                       \
  } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldnt(const float* p) {
  const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
  return float4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void stnt(float* p, float4 v) {
  f4v w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(p));
}
__device__ __forceinline__ void upd(float4& x, float4& h, float4& m) {
  x.x += 0.5f * (m.x - h.x); x.y += 0.5f * (m.y - h.y); x.z += 0.5f * (m.z - h.z); x.w += 0.5f * (m.w - h.w);
  h.x += 1e-3f; h.y += 1e-3f; h.z += 1e-3f; h.w += 1e-3f;
  m.x *= 0.999f; m.y *= 0.999f; m.z *= 0.999f; m.w *= 0.999f;
}

// column tiles; rows [r0, r0 + NR) of every column block; only interior blocks (Np a
// multiple of 4 here, every run inside [0, n))
template <int RU, int NR>
__global__ __launch_bounds__(256) void col_kernel(float* x, float* h, float* m, long long n, long long Np) {
  constexpr int RB = 32 / NR;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long cb = blockIdx.x / RB;
  const int r0 = (int)(blockIdx.x % RB) * NR;
  const long long j0 = cb * 1024 + 256 * w;
  if (j0 + 256 > Np || (long long)31 * Np + j0 + 256 > n) return;
  struct G { float4 x[RU], h[RU], m[RU]; };
  auto off = [&](int r) { return (long long)r * Np + j0 + 4 * lane; };
  auto load = [&](int g, G& q) {
#pragma unroll
    for (int u = 0; u < RU; ++u) q.x[u] = ldnt(x + off(r0 + g * RU + u));
#pragma unroll
    for (int u = 0; u < RU; ++u) q.h[u] = ldnt(h + off(r0 + g * RU + u));
#pragma unroll
    for (int u = 0; u < RU; ++u) q.m[u] = ldnt(m + off(r0 + g * RU + u));
  };
  auto proc = [&](int g, G& q) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      upd(q.x[u], q.h[u], q.m[u]);
      const long long o = off(r0 + g * RU + u);
      stnt(x + o, q.x[u]);
      stnt(h + o, q.h[u]);
      stnt(m + o, q.m[u]);
    }
  };
  constexpr int NG = NR / RU;
  G A, B;
  load(0, A);
  load(1, B);
#pragma unroll
  for (int g = 0; g < NG; g += 2) {
    proc(g, A);
    if (g + 2 < NG) load(g + 2, A);
    proc(g + 1, B);
    if (g + 3 < NG) load(g + 3, B);
  }
}

__global__ __launch_bounds__(256) void flat_kernel(float* x, float* h, float* m, long long n) {
  const long long t0 = (long long)blockIdx.x * 4096;
  float4 a[2][2], b[2][2], c[2][2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const long long e = t0 + g * 2048 + threadIdx.x * 8;
    if (e + 8 > n) continue;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      a[g][q] = *reinterpret_cast<const float4*>(x + e + 4 * q);
      b[g][q] = *reinterpret_cast<const float4*>(h + e + 4 * q);
      c[g][q] = *reinterpret_cast<const float4*>(m + e + 4 * q);
    }
  }
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const long long e = t0 + g * 2048 + threadIdx.x * 8;
    if (e + 8 > n) continue;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      upd(a[g][q], b[g][q], c[g][q]);
      *reinterpret_cast<float4*>(x + e + 4 * q) = a[g][q];
      *reinterpret_cast<float4*>(h + e + 4 * q) = b[g][q];
      *reinterpret_cast<float4*>(m + e + 4 * q) = c[g][q];
    }
  }
}

int main(int argc, char** argv) {
  long long n = argc > 1 ? atoll(argv[1]) : 345000000LL;
  long long Np = (n + 31) / 32;
  Np = Np / 4 * 4;  // interior runs only: a multiple of 4 columns
  n = 32 * Np;
  const size_t bytes = (size_t)n * 4;
  float* buf[2][3];
  for (int s = 0; s < 2; ++s)
    for (int a = 0; a < 3; ++a) {
      CK(hipMalloc(&buf[s][a], bytes));
      CK(hipMemset(buf[s][a], 0, bytes));
    }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double mb = 24.0 * (double)n / 1e6;
  printf("n %lld (N' %lld), %.0f MB read + written per launch\n", n, Np, mb);
  auto run = [&](const char* name, auto launch) {
    std::vector<float> t;
    for (int i = 0; i < 22; ++i) {
      float** b = buf[i & 1];
      CK(hipEventRecord(e0));
      launch(b[0], b[1], b[2]);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (i >= 2) t.push_back(ms * 1e3f);
    }
    std::sort(t.begin(), t.end());
    const float med = t[t.size() / 2];
    printf("%-12s min %8.1f us  med %8.1f us  -> %.2f TB/s\n", name, t[0], med, mb / med);
  };
  const unsigned ncb = (unsigned)((Np + 1023) / 1024);
  run("col<4>", [&](float* x, float* h, float* m) { col_kernel<4, 32><<<ncb, 256>>>(x, h, m, n, Np); });
  run("col<8>", [&](float* x, float* h, float* m) { col_kernel<8, 32><<<ncb, 256>>>(x, h, m, n, Np); });
  run("colh<4>", [&](float* x, float* h, float* m) { col_kernel<4, 16><<<ncb * 2, 256>>>(x, h, m, n, Np); });
  run("colq<4>", [&](float* x, float* h, float* m) { col_kernel<4, 8><<<ncb * 4, 256>>>(x, h, m, n, Np); });
  run("flat", [&](float* x, float* h, float* m) { flat_kernel<<<(unsigned)((n + 4095) / 4096), 256>>>(x, h, m, n); });
  run("col<4>", [&](float* x, float* h, float* m) { col_kernel<4, 32><<<ncb, 256>>>(x, h, m, n, Np); });
  run("flat", [&](float* x, float* h, float* m) { flat_kernel<<<(unsigned)((n + 4095) / 4096), 256>>>(x, h, m, n); });
  CK(hipDeviceSynchronize());
  return 0;
}
