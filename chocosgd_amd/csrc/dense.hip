// Element-wise pieces of the CHOCO gossip step on MI355X:
//   * consensus step      x += gamma * (memory - x_hat)   (reference
//                         dl_code/pcode/optim/utils.py:67-72)
//   * sparse accumulate   x_hat[idx] += v ; memory[idx] += w * v
//                         (dl_code/pcode/optim/parallel_choco_v.py:307-310)
//   * gather              x_data[selected_indices]
//                         (dl_code/pcode/utils/sparsification.py:31,52-54)
// All follow the reference's fp32 rounding sequence (no fused multiply-add:
// the library is compiled with -ffp-contract=off).
#include "choco_common.h"

#include <algorithm>

namespace choco {

constexpr int kEwThreads = 256;

__global__ __launch_bounds__(kEwThreads) void gossip_kernel(float* __restrict__ x, const float* __restrict__ mem,
                                                            const float* __restrict__ hat, float gamma, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kEwThreads * 4;
  for (int64_t e = ((int64_t)blockIdx.x * kEwThreads + threadIdx.x) * 4; e < n; e += stride) {
    if (e + 3 < n) {
      float4 a = *reinterpret_cast<const float4*>(x + e);
      const float4 m = *reinterpret_cast<const float4*>(mem + e);
      const float4 h = *reinterpret_cast<const float4*>(hat + e);
      a.x = a.x + gamma * (m.x - h.x);
      a.y = a.y + gamma * (m.y - h.y);
      a.z = a.z + gamma * (m.z - h.z);
      a.w = a.w + gamma * (m.w - h.w);
      *reinterpret_cast<float4*>(x + e) = a;
    } else {
      for (int64_t i = e; i < n; ++i) x[i] = x[i] + gamma * (mem[i] - hat[i]);
    }
  }
}

// Scattered read-modify-write of x_hat and memory at the message's (sorted,
// distinct) indices.  Each thread takes kAccU updates (strided by the block, so
// the index/value reads stay coalesced) and issues all their loads before any
// store.  Default 1: with cold lines (the bench step) the full grid's memory-level
// parallelism wins (U = 16: 82 -> 88 us); with MALL-hot lines U = 16 wins (73 -> 59 us).
#ifndef CHOCO_ACC_U
#define CHOCO_ACC_U 1
#endif
constexpr int kAccU = CHOCO_ACC_U;
__global__ __launch_bounds__(kEwThreads) void sparse_acc_kernel(const float* __restrict__ val,
                                                                const int32_t* __restrict__ idx, int64_t k,
                                                                float* __restrict__ hat, float* __restrict__ mem,
                                                                float w) {
  const int64_t base = (int64_t)blockIdx.x * kEwThreads * kAccU + threadIdx.x;
  if (base + (int64_t)(kAccU - 1) * kEwThreads < k) {
    int64_t j[kAccU];
    float v[kAccU], h[kAccU], m[kAccU];
#pragma unroll
    for (int u = 0; u < kAccU; ++u) {
      j[u] = idx[base + u * kEwThreads];
      v[u] = val[base + u * kEwThreads];
    }
#pragma unroll
    for (int u = 0; u < kAccU; ++u) {
      if (hat) h[u] = hat[j[u]];
      m[u] = mem[j[u]];
    }
#pragma unroll
    for (int u = 0; u < kAccU; ++u) {
      if (hat) hat[j[u]] = h[u] + v[u];
      mem[j[u]] = m[u] + w * v[u];
    }
    return;
  }
  for (int u = 0; u < kAccU; ++u) {
    const int64_t i = base + u * kEwThreads;
    if (i >= k) break;
    const int64_t jj = idx[i];
    const float vv = val[i];
    if (hat) hat[jj] = hat[jj] + vv;
    mem[jj] = mem[jj] + w * vv;
  }
}

__global__ __launch_bounds__(kEwThreads) void gather_kernel(const float* __restrict__ x, const float* __restrict__ xh,
                                                            const int64_t* __restrict__ idx, int64_t k, float scale,
                                                            float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * kEwThreads;
  for (int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x; i < k; i += stride) {
    const int64_t j = idx[i];
    const float d = xh ? x[j] - xh[j] : x[j];
    out[i] = d * scale;
  }
}

static unsigned ew_grid(int64_t work, int per_thread) {
  int64_t g = (work + (int64_t)kEwThreads * per_thread - 1) / ((int64_t)kEwThreads * per_thread);
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 8192));
}

}  // namespace choco

using namespace choco;

CHOCO_API int choco_gossip_step(float* x, const float* memory, const float* xhat, float gamma, int64_t n,
                                void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(x && memory && xhat, "null pointer argument");
  CHOCO_REQUIRE(n > 0, "n must be positive");
  CHOCO_REQUIRE(aligned16(x) && aligned16(memory) && aligned16(xhat), "buffers must be 16-byte aligned");
  profile_begin("gossip_step", st);
  CHOCO_KLAUNCH(gossip_kernel, dim3(ew_grid(n, 4)), dim3(kEwThreads), 0, st, x, memory, xhat, gamma, n);
  profile_end("gossip_step", st);
  CHOCO_LAUNCHED("gossip_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_sparse_accumulate(const float* val, const int32_t* idx, int64_t k, float* xhat_self,
                                      float* memory, float weight, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(val && idx && memory, "null pointer argument");
  if (k <= 0) return CHOCO_OK;
  profile_begin("sparse_accumulate", st);
  CHOCO_KLAUNCH(sparse_acc_kernel, dim3((unsigned)((k + (int64_t)kEwThreads * kAccU - 1) / ((int64_t)kEwThreads * kAccU))),
                dim3(kEwThreads), 0, st, val, idx, k, xhat_self,
                     memory, weight);
  profile_end("sparse_accumulate", st);
  CHOCO_LAUNCHED("sparse_acc_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_gather(const float* x, const float* xhat, const int64_t* idx, int64_t k, float scale,
                           float* out_val, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(x && idx && out_val, "null pointer argument");
  if (k <= 0) return CHOCO_OK;
  CHOCO_KLAUNCH(gather_kernel, dim3(ew_grid(k, 1)), dim3(kEwThreads), 0, st, x, xhat, idx, k, scale, out_val);
  CHOCO_LAUNCHED("gather_kernel");
  return CHOCO_OK;
}
