// Exact single-workgroup selection, shared by the flat pipeline (topk.hip: small n
// and the segmented fallback) and the batched segmented select (topk_seg.hip: a
// segment whose warm window missed).  Semantics as in topk.hip's header:
//   T = k-th largest key, out = {key > T} U {the lowest-index ties at T}, ascending.
#pragma once

#include "choco_common.h"

namespace choco {

// ----------------------------------------------------------------------------
// key / value sources
// ----------------------------------------------------------------------------
template <int MODE, bool XH>
struct Src {
  const float* __restrict__ x;
  const float* __restrict__ xh;
  uint64_t seed;
  CHOCO_DEV float val(int64_t i) const { return XH ? x[i] - xh[i] : x[i]; }
  // the fused gossip step on one element: x[i] <- x_new, returns x_new - xh[i]
  CHOCO_DEV float val_gossip(int64_t i, const Gossip& g) const {
    const float xn = gossip1(x[i], g.mem[i], xh[i], g.gamma);
    const_cast<float*>(x)[i] = xn;
    return xn - xh[i];
  }
  CHOCO_DEV uint32_t key_of(int64_t i, float v) const {
    if (MODE == kHash) return rank_hash(seed, (uint32_t)i) >> 1;
    return fkey(v);
  }
  CHOCO_DEV uint32_t key(int64_t i) const {
    if (MODE == kHash) return rank_hash(seed, (uint32_t)i) >> 1;
    return fkey(val(i));
  }
};

// ----------------------------------------------------------------------------
// exact single-workgroup select (small n, segments, fallback)
// ----------------------------------------------------------------------------
struct ExactSmem {
  uint32_t hist[2048];
  uint32_t scratch[40];  // block_excl_scan2: 2 words per wave
  uint32_t bc[4];
};

// Returns T (k-th largest key) and the tie quota r via bc[0], bc[1]; bc[2] = #ties at T.
template <class S>
CHOCO_DEV void block_select_T(const S& src, int64_t n, int64_t k, ExactSmem& sm) {
  const int tid = threadIdx.x, B = blockDim.x;
  uint32_t prefix = 0, maskhi = 0;
  uint32_t krem = (uint32_t)k;
  const int shs[3] = {20, 9, 0};
  const int wds[3] = {11, 11, 9};
  for (int rd = 0; rd < 3; ++rd) {
    const int sh = shs[rd];
    const uint32_t dmask = (1u << wds[rd]) - 1u;
    for (int i = tid; i < 2048; i += B) sm.hist[i] = 0;
    __syncthreads();
    for (int64_t i = tid; i < n; i += B) {
      uint32_t key = src.key(i);
      if ((key & maskhi) == prefix) atomicAdd(&sm.hist[(key >> sh) & dmask], 1u);
    }
    __syncthreads();
    const int nbins = (int)dmask + 1;
    const int per = (nbins + B - 1) / B;
    const int b0 = tid * per;
    uint32_t local = 0;
    for (int j = 0; j < per; ++j)
      if (b0 + j < nbins) local += sm.hist[b0 + j];
    uint32_t total;
    uint32_t pre = block_excl_scan(local, sm.scratch, &total);
    uint32_t above = total - pre - local;  // matching keys in bins above my chunk
    if (above < krem && krem <= above + local) {
      uint32_t acc = above;
      for (int j = per - 1; j >= 0; --j) {
        int bin = b0 + j;
        if (bin >= nbins) continue;
        uint32_t c = sm.hist[bin];
        if (acc + c >= krem) {
          sm.bc[0] = (uint32_t)bin;
          sm.bc[1] = krem - acc;
          sm.bc[2] = c;
          break;
        }
        acc += c;
      }
    }
    __syncthreads();
    prefix |= sm.bc[0] << sh;
    maskhi |= dmask << sh;
    krem = sm.bc[1];
    __syncthreads();
  }
  if (tid == 0) { sm.bc[0] = prefix; sm.bc[1] = krem; }
  __syncthreads();
}

// Ordered compaction of the selection defined by (T, r) over [0, n).
template <class S>
CHOCO_DEV void block_emit(const S& src, int64_t n, uint32_t T, uint32_t r, uint32_t ties_total,
                          float scale, float* __restrict__ out_val, int32_t* __restrict__ out_idx,
                          int64_t idx_base, ExactSmem& sm) {
  const int tid = threadIdx.x, B = blockDim.x;
  const bool all_ties = (r == ties_total);
  uint32_t out = 0, tie_run = 0;
  for (int64_t base = 0; base < n; base += B) {
    const int64_t i = base + tid;
    const bool valid = i < n;
    float v = 0.f;
    uint32_t key = 0;
    if (valid) { v = src.val(i); key = src.key_of(i, v); }
    const bool gt = valid && key > T;
    const bool eq = valid && key == T;
    bool sel;
    if (all_ties) {
      sel = gt || eq;
    } else {
      uint32_t ntie;
      uint32_t trank = tie_run + block_excl_scan(eq ? 1u : 0u, sm.scratch, &ntie);
      sel = gt || (eq && trank < r);
      tie_run += ntie;
    }
    uint32_t nsel;
    uint32_t pos = out + block_excl_scan(sel ? 1u : 0u, sm.scratch, &nsel);
    if (sel) {
      out_val[pos] = v * scale;
      out_idx[pos] = (int32_t)(i + idx_base);
    }
    out += nsel;
  }
}

template <class S>
CHOCO_DEV void block_topk_exact(const S& src, int64_t n, int64_t k, float scale,
                                float* out_val, int32_t* out_idx, int64_t idx_base, ExactSmem& sm) {
  if (k >= n) {
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
      out_val[i] = src.val(i) * scale;
      out_idx[i] = (int32_t)(i + idx_base);
    }
    return;
  }
  block_select_T(src, n, k, sm);
  const uint32_t T = sm.bc[0], r = sm.bc[1], ties = sm.bc[2];
  __syncthreads();
  block_emit(src, n, T, r, ties, scale, out_val, out_idx, idx_base, sm);
}

}  // namespace choco
