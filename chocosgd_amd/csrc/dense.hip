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
// An index outside [0, n) (a corrupt message, or a peer with another layout) is
// skipped and counted into *bad (nullable) -- the reference's index_put raises
// IndexError there; the host checks the count lazily (codec.py).
__global__ __launch_bounds__(kEwThreads) void sparse_acc_kernel(const float* __restrict__ val,
                                                                const int32_t* __restrict__ idx, int64_t k,
                                                                float* __restrict__ hat, float* __restrict__ mem,
                                                                int64_t n, float w, uint32_t* __restrict__ bad) {
  const int64_t base = (int64_t)blockIdx.x * kEwThreads * kAccU + threadIdx.x;
  uint32_t nbad = 0;
  if (base + (int64_t)(kAccU - 1) * kEwThreads < k) {
    int64_t j[kAccU];
    float v[kAccU], h[kAccU], m[kAccU];
    bool ok[kAccU];
#pragma unroll
    for (int u = 0; u < kAccU; ++u) {
      j[u] = idx[base + u * kEwThreads];
      v[u] = val[base + u * kEwThreads];
      ok[u] = j[u] >= 0 && j[u] < n;
      nbad += ok[u] ? 0u : 1u;
      if (!ok[u]) j[u] = 0;
    }
#pragma unroll
    for (int u = 0; u < kAccU; ++u) {
      if (hat) h[u] = hat[j[u]];
      m[u] = mem[j[u]];
    }
#pragma unroll
    for (int u = 0; u < kAccU; ++u) {
      if (!ok[u]) continue;
      if (hat) hat[j[u]] = h[u] + v[u];
      mem[j[u]] = m[u] + w * v[u];
    }
  } else {
    for (int u = 0; u < kAccU; ++u) {
      const int64_t i = base + u * kEwThreads;
      if (i >= k) break;
      const int64_t jj = idx[i];
      if (jj < 0 || jj >= n) {
        ++nbad;
        continue;
      }
      const float vv = val[i];
      if (hat) hat[jj] = hat[jj] + vv;
      mem[jj] = mem[jj] + w * vv;
    }
  }
  if (bad && nbad) atomicAdd(bad, nbad);
}

// Segment-owner form (default).  A message's indices are strictly ascending
// (this codec's top-k / random-k wire), so the updates that fall into one
// 64-B segment of x_hat / memory (16 floats) are consecutive in the message.
// One QUAD of lanes per update: the quad of the segment's first update (the
// "leader") loads the whole segment of each target buffer -- lane l4 its
// float4 l4, so one wave instruction covers 16 segments -- applies every
// update of that segment, and writes the whole segment back; the other quads
// idle.  Whole-segment writes: no byte-masked partial writes reach the
// memory side (a 4-B store dirties a sector that must be merged there).
// A non-ascending pair (a corrupt message) is counted into *bad like an
// out-of-range index.  Such a message is applied before the count is seen: with
// indices out of order two leaders can own the same segment (e.g. [20, 3, 21])
// and one whole-segment write overwrites the other's update, so x_hat / memory
// of that step may already be wrong when the host reports the bad count
// (IndexGuard, one step later; INTEGRATION.md "corrupt messages").  Messages
// from this codec are always ascending.
#ifndef CHOCO_ACC_MODE
#define CHOCO_ACC_MODE 1
#endif
#ifndef CHOCO_ACC_SEGF
#define CHOCO_ACC_SEGF 16
#endif
#ifndef CHOCO_ACC_NEXT  // A/B knob: 1 loads the next index and the value with the update's index
#define CHOCO_ACC_NEXT 1
#endif
#ifndef CHOCO_ACC_NT  // cache policy of the owner's segment RMW (A/B): 0 default, 1 nt stores, 2 nt loads + stores
#define CHOCO_ACC_NT 0
#endif
CHOCO_DEV float4 acc_ld4(const float* p) {
  if (CHOCO_ACC_NT >= 2) return ld_nt4(p);
  return *reinterpret_cast<const float4*>(p);
}
CHOCO_DEV void acc_st4(float* p, float4 v) {
  if (CHOCO_ACC_NT >= 1) {
    choco_f32x4 f;
    f.x = v.x; f.y = v.y; f.z = v.z; f.w = v.w;
    __builtin_nontemporal_store(f, reinterpret_cast<choco_f32x4*>(p));
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
constexpr int kSegF = CHOCO_ACC_SEGF;  // floats per owned segment (16: 64 B)
constexpr int kSegL = kSegF / 4;       // lanes per update (one float4 each)
constexpr int kSegShift = kSegF == 32 ? 5 : (kSegF == 16 ? 4 : 3);
static_assert((1 << kSegShift) == kSegF, "segment of 8, 16 or 32 floats");

template <bool HS>
__global__ __launch_bounds__(kEwThreads) void sparse_acc_seg_kernel(const float* __restrict__ val,
                                                                    const int32_t* __restrict__ idx, int64_t k,
                                                                    float* __restrict__ hat,
                                                                    float* __restrict__ mem, int64_t n, float w,
                                                                    uint32_t* __restrict__ bad) {
  const int64_t t = (int64_t)blockIdx.x * kEwThreads + threadIdx.x;
  const int64_t u = t / kSegL;
  const int l4 = (int)(t % kSegL);
  uint32_t nbad = 0;
  if (u < k) {
    const int64_t j = idx[u];
    const int64_t jp = u > 0 ? (int64_t)idx[u - 1] : -1;
    // the next update's index and this update's value in the same round trip: most
    // segments hold one update, so the leader then needs no third round trip to find
    // that the next update is not its segment's
    const int64_t jn = CHOCO_ACC_NEXT && u + 1 < k ? (int64_t)idx[u + 1] : -1;
    const float v0 = CHOCO_ACC_NEXT ? val[u] : 0.f;
    const bool ok = j >= 0 && j < n;
    const int64_t seg = j >> kSegShift;
    if (l4 == 0) nbad += (ok ? 0u : 1u) + ((u > 0 && jp >= j) ? 1u : 0u);
    const bool leader = ok && (u == 0 || jp < 0 || (jp >> kSegShift) != seg);
    if (leader) {
      const int64_t base = seg * kSegF + 4 * l4;
      const bool full = base + 4 <= n;
      float hv[4] = {0.f, 0.f, 0.f, 0.f}, mv[4] = {0.f, 0.f, 0.f, 0.f};
      if (full) {
        const float4 m4 = acc_ld4(mem + base);
        mv[0] = m4.x; mv[1] = m4.y; mv[2] = m4.z; mv[3] = m4.w;
        if (HS) {
          const float4 h4 = acc_ld4(hat + base);
          hv[0] = h4.x; hv[1] = h4.y; hv[2] = h4.z; hv[3] = h4.w;
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (base + c < n) {
            mv[c] = mem[base + c];
            if (HS) hv[c] = hat[base + c];
          }
        }
      }
      int64_t je = j;
      for (int64_t e = u; e < k && e < u + kSegF; ++e) {
        if (e != u) je = (CHOCO_ACC_NEXT && e == u + 1) ? jn : idx[e];
        if (je < 0 || je >= n || (je >> kSegShift) != seg) break;
        const float v = (CHOCO_ACC_NEXT && e == u) ? v0 : val[e];
        const int off = (int)(je - base);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (off == c) {
            if (HS) hv[c] = hv[c] + v;
            mv[c] = mv[c] + w * v;
          }
        }
      }
      if (full) {
        acc_st4(mem + base, make_float4(mv[0], mv[1], mv[2], mv[3]));
        if (HS) acc_st4(hat + base, make_float4(hv[0], hv[1], hv[2], hv[3]));
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (base + c < n) {
            mem[base + c] = mv[c];
            if (HS) hat[base + c] = hv[c];
          }
        }
      }
    }
  }
  if (bad && nbad) atomicAdd(bad, nbad);
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

// ECDSparsificationCompressor.uncompress (ecd_psgd.py:299-303):
//   target[idx] = target[idx].mul(a).add(b, v)  ->  fmaf(b, v, target[idx] * a)
// (torch's vectorized add with alpha fuses).  Indices unique per message.
__global__ __launch_bounds__(kEwThreads) void sparse_extrap_kernel(const float* __restrict__ val,
                                                                   const int32_t* __restrict__ idx, int64_t k,
                                                                   float* __restrict__ target, int64_t n, float a,
                                                                   float b, uint32_t* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x;
  if (i >= k) return;
  const int64_t j = idx[i];
  if (j < 0 || j >= n) {
    if (bad) atomicAdd(bad, 1u);
    return;
  }
  target[j] = fmaf(b, val[i], target[j] * a);
}

static unsigned ew_grid(int64_t work, int per_thread) {
  int64_t g = (work + (int64_t)kEwThreads * per_thread - 1) / ((int64_t)kEwThreads * per_thread);
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 8192));
}

// One-shot form: each thread owns kGossipU float4 of every stream (no grid-stride
// loop), all loads issued before any arithmetic; `nt` policy knob for the A/B.
#ifndef CHOCO_GOSSIP_FORM  // 0: grid-stride gossip_kernel; 1: one-shot gossipu_kernel
#define CHOCO_GOSSIP_FORM 1
#endif
#ifndef CHOCO_GOSSIP_U  // measured at 100M (tools/gossip_probe.py): U=4 + nt 258 us (6.2 TB/s)
#define CHOCO_GOSSIP_U 4    // against 320 us for the grid-stride form and 291 us for U=2 plain
#endif
#ifndef CHOCO_GOSSIP_NT
#define CHOCO_GOSSIP_NT 1
#endif
constexpr int kGossipU = CHOCO_GOSSIP_U;
__global__ __launch_bounds__(kEwThreads) void gossipu_kernel(float* __restrict__ x, const float* __restrict__ mem,
                                                             const float* __restrict__ hat, float gamma, int64_t n) {
  const int64_t e0 = ((int64_t)blockIdx.x * kEwThreads * kGossipU + threadIdx.x) * 4;
  constexpr int64_t kStep = (int64_t)kEwThreads * 4;  // consecutive threads: consecutive float4
  if (e0 + (kGossipU - 1) * kStep + 3 < n) {
    float4 a[kGossipU], m[kGossipU], h[kGossipU];
#pragma unroll
    for (int u = 0; u < kGossipU; ++u) {
      if (CHOCO_GOSSIP_NT) {
        a[u] = ld_nt4(x + e0 + u * kStep);
        m[u] = ld_nt4(mem + e0 + u * kStep);
        h[u] = ld_nt4(hat + e0 + u * kStep);
      } else {
        a[u] = *reinterpret_cast<const float4*>(x + e0 + u * kStep);
        m[u] = *reinterpret_cast<const float4*>(mem + e0 + u * kStep);
        h[u] = *reinterpret_cast<const float4*>(hat + e0 + u * kStep);
      }
    }
#pragma unroll
    for (int u = 0; u < kGossipU; ++u) {
      const float4 v = gossip4(a[u], m[u], h[u], gamma);
      if (CHOCO_GOSSIP_NT) {
        choco_f32x4 f;
        f.x = v.x; f.y = v.y; f.z = v.z; f.w = v.w;
        __builtin_nontemporal_store(f, reinterpret_cast<choco_f32x4*>(x + e0 + u * kStep));
      } else {
        *reinterpret_cast<float4*>(x + e0 + u * kStep) = v;
      }
    }
  } else {
    for (int u = 0; u < kGossipU; ++u)
      for (int c = 0; c < 4; ++c) {
        const int64_t i = e0 + u * kStep + c;
        if (i < n) x[i] = gossip1(x[i], mem[i], hat[i], gamma);
      }
  }
}

// any 4-byte alignment (segments of a flat buffer): one element per thread
__global__ __launch_bounds__(kEwThreads) void gossip1_kernel(float* __restrict__ x, const float* __restrict__ mem,
                                                             const float* __restrict__ hat, float gamma, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kEwThreads;
  for (int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x; i < n; i += stride)
    x[i] = gossip1(x[i], mem[i], hat[i], gamma);
}

int gossip_launch(float* x, const float* mem, const float* xh, float gamma, int64_t n, hipStream_t st) {
  CHOCO_REQUIRE(x && mem && xh, "null pointer argument");
  CHOCO_REQUIRE(n > 0, "n must be positive");
  CHOCO_REQUIRE(aligned4(x) && aligned4(mem) && aligned4(xh), "buffers must be 4-byte aligned");
  profile_begin("gossip_step", st);
  if (aligned16(x) && aligned16(mem) && aligned16(xh)) {
    if (CHOCO_GOSSIP_FORM == 1) {
      const int64_t per = (int64_t)kEwThreads * 4 * kGossipU;
      CHOCO_KLAUNCH(gossipu_kernel, dim3((unsigned)((n + per - 1) / per)), dim3(kEwThreads), 0, st, x, mem, xh,
                    gamma, n);
    } else {
      CHOCO_KLAUNCH(gossip_kernel, dim3(ew_grid(n, 4)), dim3(kEwThreads), 0, st, x, mem, xh, gamma, n);
    }
  } else {
    CHOCO_KLAUNCH(gossip1_kernel, dim3(ew_grid(n, 1)), dim3(kEwThreads), 0, st, x, mem, xh, gamma, n);
  }
  profile_end("gossip_step", st);
  CHOCO_LAUNCHED("gossip_kernel");
  return CHOCO_OK;
}

}  // namespace choco

using namespace choco;

CHOCO_API int choco_gossip_step(float* x, const float* memory, const float* xhat, float gamma, int64_t n,
                                void* stream) {
  return gossip_launch(x, memory, xhat, gamma, n, as_stream(stream));
}


CHOCO_API int choco_sparse_accumulate(const float* val, const int32_t* idx, int64_t k, float* xhat_self,
                                      float* memory, int64_t n, float weight, uint32_t* bad_count, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(val && idx && memory, "null pointer argument");
  CHOCO_REQUIRE(n > 0, "n must be positive");
  if (k <= 0) return CHOCO_OK;
  profile_begin("sparse_accumulate", st);
  if (CHOCO_ACC_MODE == 1 && aligned16(memory) && (!xhat_self || aligned16(xhat_self))) {
    const unsigned g = (unsigned)((kSegL * k + kEwThreads - 1) / kEwThreads);
    if (xhat_self)
      CHOCO_KLAUNCH((sparse_acc_seg_kernel<true>), dim3(g), dim3(kEwThreads), 0, st, val, idx, k, xhat_self, memory,
                    n, weight, bad_count);
    else
      CHOCO_KLAUNCH((sparse_acc_seg_kernel<false>), dim3(g), dim3(kEwThreads), 0, st, val, idx, k, xhat_self,
                    memory, n, weight, bad_count);
  } else {
    CHOCO_KLAUNCH(sparse_acc_kernel,
                  dim3((unsigned)((k + (int64_t)kEwThreads * kAccU - 1) / ((int64_t)kEwThreads * kAccU))),
                  dim3(kEwThreads), 0, st, val, idx, k, xhat_self, memory, n, weight, bad_count);
  }
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

CHOCO_API int choco_sparse_extrapolate(const float* val, const int32_t* idx, int64_t k, float* target, int64_t n,
                                       float a, float b, uint32_t* bad_count, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(val && idx && target, "null pointer argument");
  CHOCO_REQUIRE(n > 0, "n must be positive");
  if (k <= 0) return CHOCO_OK;
  profile_begin("sparse_accumulate", st);
  CHOCO_KLAUNCH(sparse_extrap_kernel, dim3((unsigned)((k + kEwThreads - 1) / kEwThreads)), dim3(kEwThreads), 0, st,
                val, idx, k, target, n, a, b, bad_count);
  profile_end("sparse_accumulate", st);
  CHOCO_LAUNCHED("sparse_extrap_kernel");
  return CHOCO_OK;
}
