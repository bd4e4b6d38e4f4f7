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

// Scattered read-modify-write of x_hat and memory at the message's indices, one
// update per thread: the form for buffers that are not 16-byte aligned (the segment
// form below needs whole float4).  An index outside [0, n) (a corrupt message, or a peer
// with another layout) is skipped and counted into *bad (nullable) -- the reference's
// index_put raises IndexError there; the host checks the count lazily (codec.py).
__global__ __launch_bounds__(kEwThreads) void sparse_acc_kernel(const float* __restrict__ val,
                                                                const int32_t* __restrict__ idx, int64_t k,
                                                                float* __restrict__ hat, float* __restrict__ mem,
                                                                int64_t n, float w, uint32_t* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x;
  if (i >= k) return;
  const int64_t jj = idx[i];
  if (jj < 0 || jj >= n) {
    if (bad) atomicAdd(bad, 1u);
    return;
  }
  const float vv = val[i];
  if (hat) hat[jj] = hat[jj] + vv;
  mem[jj] = mem[jj] + w * vv;
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
// Measured and not kept (same-box A/Bs, r03/r04; git history): owner granules of 32 / 128 B
// and per-element updates (80-99 against 77.5-80 us), non-temporal segment loads / stores;
// r05: one thread per update with return-less float atomics, agent or workgroup scope, 97 /
// 103 us against 77 (top-k / random-k at k = 1M); non-temporal segment stores (whole steps
// within 1 %), loads + stores (+3.5-6 us here; random-k's step -3.6 %, top-k's +3.7 %), or
// loads alone (+3-6 us; the fused top-k step's next stream +30 us): r05_ab_summary.txt 15, 22.
CHOCO_DEV float4 acc_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
CHOCO_DEV void acc_st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
constexpr int kSegF = 16;              // floats per owned segment (64 B)
constexpr int kSegL = kSegF / 4;       // lanes per update (one float4 each)
constexpr int kSegShift = 4;

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
    const int64_t jn = u + 1 < k ? (int64_t)idx[u + 1] : -1;
    const float v0 = val[u];
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
        if (e != u) je = e == u + 1 ? jn : idx[e];
        if (je < 0 || je >= n || (je >> kSegShift) != seg) break;
        const float v = e == u ? v0 : val[e];
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

// (A merged multi-message receive -- one sweep over 8192-element ranges applying every
// neighbour's message to each touched 64-B line of memory once, after a split pass over
// the messages' indices -- was built and measured in r05 (git history): ring-3 loopback at
// k = 1 %, line traffic 477 -> 422 MB per step, but 160 against 156 us per step: the sweep
// ran at the per-message kernels' scattered line rate (~2.9-3.1 TB/s) and the split pass
// cost more than the lines saved.  choco_sparse_accumulate_multi applies the messages with
// the per-message kernels.)
constexpr int kMaxMsgs = 8;

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

// The consensus step x += gamma (memory - x_hat), one-shot form: each thread owns
// kGossipU float4 of every stream (no grid-stride loop), all loads issued before any
// arithmetic, non-temporal loads and stores.  Measured at 100M (tools/gossip_probe.py):
// U = 4 + nt 258 us (6.2 TB/s) against 320 us for a grid-stride form and 291 us for U = 2
// plain.
constexpr int kGossipU = 4;
__global__ __launch_bounds__(kEwThreads) void gossipu_kernel(float* __restrict__ x, const float* __restrict__ mem,
                                                             const float* __restrict__ hat, float gamma, int64_t n) {
  const int64_t e0 = ((int64_t)blockIdx.x * kEwThreads * kGossipU + threadIdx.x) * 4;
  constexpr int64_t kStep = (int64_t)kEwThreads * 4;  // consecutive threads: consecutive float4
  if (e0 + (kGossipU - 1) * kStep + 3 < n) {
    float4 a[kGossipU], m[kGossipU], h[kGossipU];
#pragma unroll
    for (int u = 0; u < kGossipU; ++u) {
      a[u] = ld_nt4(x + e0 + u * kStep);
      m[u] = ld_nt4(mem + e0 + u * kStep);
      h[u] = ld_nt4(hat + e0 + u * kStep);
    }
#pragma unroll
    for (int u = 0; u < kGossipU; ++u) {
      const float4 v = gossip4(a[u], m[u], h[u], gamma);
      choco_f32x4 f;
      f.x = v.x; f.y = v.y; f.z = v.z; f.w = v.w;
      __builtin_nontemporal_store(f, reinterpret_cast<choco_f32x4*>(x + e0 + u * kStep));
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
    const int64_t per = (int64_t)kEwThreads * 4 * kGossipU;
    CHOCO_KLAUNCH(gossipu_kernel, dim3((unsigned)((n + per - 1) / per)), dim3(kEwThreads), 0, st, x, mem, xh,
                  gamma, n);
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
  if (aligned16(memory) && (!xhat_self || aligned16(xhat_self))) {
    const unsigned g = (unsigned)((kSegL * k + kEwThreads - 1) / kEwThreads);
    if (xhat_self)
      CHOCO_KLAUNCH((sparse_acc_seg_kernel<true>), dim3(g), dim3(kEwThreads), 0, st, val, idx, k, xhat_self, memory,
                    n, weight, bad_count);
    else
      CHOCO_KLAUNCH((sparse_acc_seg_kernel<false>), dim3(g), dim3(kEwThreads), 0, st, val, idx, k, xhat_self,
                    memory, n, weight, bad_count);
  } else {
    CHOCO_KLAUNCH(sparse_acc_kernel, dim3((unsigned)((k + kEwThreads - 1) / kEwThreads)), dim3(kEwThreads), 0, st,
                  val, idx, k, xhat_self, memory, n, weight, bad_count);
  }
  profile_end("sparse_accumulate", st);
  CHOCO_LAUNCHED("sparse_acc_kernel");
  return CHOCO_OK;
}

CHOCO_API size_t choco_sparse_accumulate_multi_workspace_size(int64_t n, int32_t nmsg) {
  (void)n;
  (void)nmsg;
  return 0;  // no scratch: the messages are applied by the per-message kernels
}

CHOCO_API int choco_sparse_accumulate_multi(const float* const* vals, const int32_t* const* idxs, const int64_t* ks,
                                            const float* weights, int32_t nmsg, int32_t self_slot, float* xhat_self,
                                            float* memory, int64_t n, void* ws, size_t ws_bytes,
                                            uint32_t* bad_count, void* stream) {
  (void)ws;
  (void)ws_bytes;
  CHOCO_REQUIRE(vals && idxs && ks && weights && memory, "null pointer argument");
  CHOCO_REQUIRE(nmsg >= 1 && nmsg <= kMaxMsgs, "nmsg must be in [1, %d], got %d", kMaxMsgs, (int)nmsg);
  CHOCO_REQUIRE(self_slot >= -1 && self_slot < nmsg, "self_slot out of range");
  CHOCO_REQUIRE(n > 0, "n must be positive");
  // every message is checked before the first launch: a bad message m must not leave
  // messages 0..m-1 applied (a retry would apply them twice)
  for (int m = 0; m < nmsg; ++m) {
    CHOCO_REQUIRE(ks[m] >= 0 && ks[m] < (int64_t)INT32_MAX, "message %d: k out of range", m);
    CHOCO_REQUIRE(ks[m] == 0 || (vals[m] != nullptr && idxs[m] != nullptr), "message %d: null pointer", m);
  }
  for (int m = 0; m < nmsg; ++m) {
    if (ks[m] == 0) continue;  // an empty message changes nothing
    const int rc = choco_sparse_accumulate(vals[m], idxs[m], ks[m], m == self_slot ? xhat_self : nullptr, memory, n,
                                           weights[m], bad_count, stream);
    if (rc) return rc;
  }
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
