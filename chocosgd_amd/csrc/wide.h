// Exact radix select over a range shared by a group of workgroups (a ticketed work
// queue), for the selections whose window guess failed:
//   - the flat pipeline's K34 (topk.hip): every K34 workgroup, the whole input;
//   - the segmented warm emission S4w (topk_seg.hip): the tile workgroups of one
//     segment whose carried window missed, that segment only.
// Semantics as in topk.hip's header (the reference's get_top_k, sparsification.py:18-31):
//   T = k-th largest key, out = {key > T} U {the lowest-index ties at T}, ascending.
#pragma once

#include "select.h"

namespace choco {

constexpr uint32_t kStatusPollTimeout = 1u;  // a bounded wait of the exact fallback gave up: output invalid

// Hand-offs between workgroups (bounds, tile tables, side lists, the queue below) use
// the fence-free form of MI355X_MICROARCH.md "Valid forms": every handed-off word is
// stored write-through (relaxed agent-scope atomic store = sc1) and read with sc1
// loads; each storing wave drains (vmcnt(0)) before a workgroup barrier, behind which
// one lane adds to the counter; the consumer polls that counter.  No release fence: a
// buffer_wbl2 writes back the whole XCD L2 and cost 10-30 us per tile in the middle of
// everyone else's stream (measured).
CHOCO_DEV void st_sc1(uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
CHOCO_DEV uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Over hist[2048] in LDS (ascending key order), the bins holding the r0-th and r1-th
// largest entries and the ranks inside them -> out[0..1], out[2..3] (a rank of 0 is
// skipped).  Every thread of the NT-thread workgroup calls it; 2048 / NT consecutive
// bins per thread.
template <int NT = 1024>
CHOCO_DEV void block_find_two(const uint32_t* hist, uint32_t r0, uint32_t r1, uint32_t* scratch, uint32_t* out) {
  constexpr int kB = 2048 / NT;
  static_assert(kB * NT == 2048, "whole bins per thread");
  const int tid = threadIdx.x;
  uint32_t h[kB];
  uint32_t local = 0;
#pragma unroll
  for (int b = 0; b < kB; ++b) {
    h[b] = hist[kB * tid + b];
    local += h[b];
  }
  uint32_t total;
  const uint32_t pre = block_excl_scan(local, scratch, &total);
  const uint32_t above0 = total - pre - local;  // entries in bins above mine
  const uint32_t rs[2] = {r0, r1};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const uint32_t r = rs[q];
    if (r != 0u && above0 < r && r <= above0 + local) {
      uint32_t above = above0;
#pragma unroll
      for (int b = kB - 1; b >= 0; --b) {
        if (above < r && r <= above + h[b]) { out[2 * q] = kB * tid + b; out[2 * q + 1] = r - above; }
        above += h[b];
      }
    }
  }
  __syncthreads();
}

// every wave's stores drained, the workgroup joined, one lane adds
CHOCO_DEV void publish_add(uint32_t* counter) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ----------------------------------------------------------------------------
// The shared exact select.  Instead of one workgroup radix-selecting the whole range,
// every workgroup of the group takes TICKETS from a work queue of 5 * nb items:
//   phases 0-2: histogram of one tile's keys for radix digit 0/1/2 (bits 30..20,
//               19..9, 8..0; only keys matching the digits found so far),
//   phase 3   : one tile's (#key > T, #key == T), from its phase-2 histogram (no pass),
//   phase 4   : one tile's ordered emission at its offset (counts of earlier tiles).
// An item of phase p waits until every item of phase p-1 is done; those are held by
// workgroups that drew earlier tickets and are therefore running, so the queue is
// deadlock-free whatever number of workgroups is resident.  The digits are
// re-derived from the global histograms by whoever needs them (a 2048-bin scan).
// The last workgroup to leave resets the queue and zeroes the histograms, so EXACTLY
// nb workgroups must enter (the caller's group).  Four streaming passes over the range
// by all the group's CUs instead of ~4 by one CU.
// ----------------------------------------------------------------------------
struct WideCtrl {
  uint32_t ticket, exitc, pad0[6];
  uint32_t done[8];  // items completed per phase
  uint32_t pad1[48];
  uint32_t hist[3][2048];
};
constexpr size_t kWideBytes = 4 * (64 + 3 * 2048);
static_assert(sizeof(WideCtrl) == kWideBytes && kWideBytes % 256 == 0, "workspace layouts reserve WideCtrl");
constexpr int kWidePhases = 5;

// Queue hand-offs made by ALL lanes of wave 0 (no lane-divergent region inside the
// ticket loop: with `if (threadIdx.x == 0)` around the atomic and the poll, the
// compiler split the loop so that wave 0 executed extra barriers -- measured hang).
CHOCO_DEV uint32_t wave0_fetch_add(uint32_t* p, uint32_t v) {
  const uint32_t r = __hip_atomic_fetch_add(p, lane_id() == 0 ? v : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane(r);
}
// Bounded: false when the budget ran out (a stuck producer must not hang the GPU;
// the caller flags the call's output invalid in the workspace status word).
#ifndef CHOCO_POLL_BUDGET  // diagnostic builds only (tools/build_variants.py "poll1")
#define CHOCO_POLL_BUDGET (1u << 22)
#endif
CHOCO_DEV bool wave0_poll_ge(const uint32_t* p, uint32_t want) {
  for (uint32_t it = 0; it < (uint32_t)CHOCO_POLL_BUDGET; ++it) {
    if (__builtin_amdgcn_readfirstlane(ld_sc1(p)) >= want) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return __builtin_amdgcn_readfirstlane(ld_sc1(p)) >= want;
}

CHOCO_DEV constexpr int wide_shift(int r) { return r == 0 ? 20 : (r == 1 ? 9 : 0); }
CHOCO_DEV constexpr uint32_t wide_mask(int r) { return r == 2 ? 511u : 2047u; }

// Digits have .. upto-1 from the global histograms, continuing (prefix, maskhi, krem)
// of digits 0 .. have-1 (a workgroup's tickets only move forward through the phases,
// so it derives each digit once).
template <int NT>
CHOCO_DEV void wide_digits(WideCtrl* W, int have, int upto, ExactSmem& es, uint32_t& prefix, uint32_t& maskhi,
                           uint32_t& krem) {
  for (int r = have; r < upto; ++r) {
    for (int i = threadIdx.x; i < 2048; i += NT) es.hist[i] = ld_sc1(&W->hist[r][i]);
    __syncthreads();
    block_find_two<NT>(es.hist, krem, 0u, es.scratch, es.bc);
    const uint32_t bin = es.bc[0];
    krem = es.bc[1];
    prefix |= bin << wide_shift(r);
    maskhi |= wide_mask(r) << wide_shift(r);
    __syncthreads();
  }
}

// The keys (and values) of tile [lo, hi) row by row (a row = 4 consecutive elements
// per thread, NT * 4 per row, U rows' loads in flight):
// fn(i0, n_in, keys[4], vals[4]) for every row, by every thread (block-uniform).
template <int NT, int U, int MODE, bool XH, class F>
CHOCO_DEV void wide_tile(const Src<MODE, XH>& src, int64_t lo, int64_t hi, F&& fn) {
  const uint32_t len = (uint32_t)(hi - lo);
  const __amdgpu_buffer_rsrc_t rx = buf_rsrc(src.x + lo, len * 4u);
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc((XH ? src.xh : src.x) + lo, len * 4u);
  constexpr uint32_t kStep = NT * 4u;
  for (uint32_t b0 = 0; b0 < len; b0 += kStep * U) {
    float4 v[U], h[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t off = (b0 + (uint32_t)u * kStep + 4u * threadIdx.x) * 4u;
      if (MODE == kData) {
        v[u] = ld_buf4<true>(rx, off);
        if (XH) h[u] = ld_buf4<true>(rh, off);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b0 + (uint32_t)u * kStep >= len) break;  // block-uniform
      const uint32_t e0 = b0 + (uint32_t)u * kStep + 4u * threadIdx.x;
      float vv[4] = {0.f, 0.f, 0.f, 0.f};
      uint32_t kk[4];
      if (MODE == kData) {
        const float4 d = XH ? sub4(v[u], h[u]) : v[u];
        vv[0] = d.x; vv[1] = d.y; vv[2] = d.z; vv[3] = d.w;
      }
      const int nin = e0 >= len ? 0 : (int)min(4u, len - e0);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t i = lo + e0 + c;
        if (MODE == kHash && c < nin) vv[c] = src.val(i);
        kk[c] = c < nin ? src.key_of(i, vv[c]) : 0u;
      }
      fn(lo + (int64_t)e0, nin, kk, vv);
    }
  }
}

// A tile reader of wide_select: reader(t, fn) calls fn(n_in, keys[4], vals[4], idx[4]) for
// every row of tile t, by every thread (block-uniform rows); idx is what emit() receives.
// RangeTiles: src[0, n) in tiles of `tile` elements, idx the element index.
template <int NT, int U, int MODE, bool XH>
struct RangeTiles {
  Src<MODE, XH> src;
  int64_t n;
  uint32_t tile;
  template <class F>
  CHOCO_DEV void operator()(uint32_t t, F&& fn) const {
    const int64_t lo = (int64_t)t * tile, hi = min(lo + (int64_t)tile, n);
    wide_tile<NT, U>(src, lo, hi, [&](int64_t i0, int nin, const uint32_t (&kk)[4], const float (&vv)[4]) {
      const int64_t ii[4] = {i0, i0 + 1, i0 + 2, i0 + 3};
      fn(nin, kk, vv, ii);
    });
  }
};

// The shared select over the nb tiles of `reader` (k outputs), by exactly nb workgroups
// of NT threads.  gcnt: 2 words per tile, thist: 512 words per tile (phase 2 -> phase 3
// -> phase 4).
// on_T(T): called by every thread of the workgroup that runs tile 0's phase-3 item,
// once T is known (the caller's next window; W->hist still holds this call's digits).
// emit(pos, idx, v): every selected element, pos its rank in the output (tile order, and
// row order inside a tile: ascending index for both readers).
template <int NT, class Reader, class OnT, class Emit>
CHOCO_DEV void wide_select(const Reader& reader, int64_t k, uint32_t nb, WideCtrl* W, uint32_t* __restrict__ gcnt,
                           uint32_t* __restrict__ thist, ExactSmem& es, uint32_t* s_tk, uint32_t* __restrict__ status,
                           uint32_t* __restrict__ host_status, OnT&& on_T, Emit&& emit) {
  const int tid = threadIdx.x;
  const bool w0 = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;  // wave-uniform
  uint32_t prefix = 0u, maskhi = 0u, krem = (uint32_t)k;  // the digits derived so far
  int have = 0;
  for (;;) {
    if (w0) *s_tk = wave0_fetch_add(&W->ticket, 1u);  // every lane of wave 0 writes the same value
    __syncthreads();
    const uint32_t tk = __builtin_amdgcn_readfirstlane(*s_tk);
    __syncthreads();
    if (tk >= (uint32_t)kWidePhases * nb) break;  // workgroup-uniform
    const int phase = (int)(tk / nb);
    const uint32_t t = tk % nb;
    if (phase > 0) {
      if (w0 && !wave0_poll_ge(&W->done[phase - 1], nb) && lane_id() == 0) {
        atomicOr(status, kStatusPollTimeout);
        // the pinned host mirror: the host sees it at its next call, no copy, no sync
        if (host_status) __hip_atomic_store(host_status, kStatusPollTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __syncthreads();
    }
    const int need = phase < 3 ? phase : 3;
    wide_digits<NT>(W, have, need, es, prefix, maskhi, krem);
    have = max(have, need);
    if (phase < 3) {
      const int sh = wide_shift(phase);
      const uint32_t dm = wide_mask(phase);
      for (int i = tid; i < 2048; i += NT) es.hist[i] = 0u;
      __syncthreads();
      const int lane = lane_id();
      uint32_t above = 0u;  // (phase 2: keys above the first two digits' prefix)
      reader(t, [&](int nin, const uint32_t (&kk)[4], const float (&)[4], const int64_t (&)[4]) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          above += (c < nin && (kk[c] & maskhi) > prefix) ? 1u : 0u;
          // tie-heavy inputs put most lanes in one bin: the lanes of the wave's first
          // bin add with one atomic, the rest one by one
          const bool on = c < nin && (kk[c] & maskhi) == prefix;
          const uint32_t bin = (kk[c] >> sh) & dm;
          const uint64_t live = ballot(on);
          if (live == 0ull) continue;  // wave-uniform
          const int first = __builtin_ctzll(live);
          const uint32_t b0 = __builtin_amdgcn_readlane(bin, first);
          const uint64_t same = ballot(on && bin == b0);
          if (lane == first) atomicAdd(&es.hist[b0], (uint32_t)__popcll(same));
          if (on && bin != b0) atomicAdd(&es.hist[bin], 1u);
        }
      });
      __syncthreads();
      for (int i = tid; i < 2048; i += NT)
        if (es.hist[i]) __hip_atomic_fetch_add(&W->hist[phase][i], es.hist[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (phase == 2) {
        // the tile's last-digit histogram and its count above the prefix: phase 3 takes the
        // tile's (#key > T, #key == T) from them without another pass over the tile
        for (int i = tid; i < 512; i += NT) st_sc1(&thist[512 * (int64_t)t + i], es.hist[i]);
        uint32_t atot;
        block_excl_scan(above, es.scratch, &atot);
        if (w0) st_sc1(&gcnt[2 * t], atot);  // same value from every lane
      }
    } else {
      const uint32_t T = prefix;  // all digits known: T = the k-th largest key, krem = ties to take
      const uint32_t r = krem;
      if (phase == 3 && t == 0) on_T(T);
      if (phase == 3) {
        // #key > T = the keys above the two-digit prefix + the prefix's keys whose last
        // digit is above T's; #key == T = the last-digit bin of T (phase 2's tile histogram)
        const uint32_t d2 = T & 511u;
        uint32_t gt = tid == 0 ? ld_sc1(&gcnt[2 * t]) : 0u, eq = 0u;
        for (int i = tid; i < 512; i += NT) {
          const uint32_t h = ld_sc1(&thist[512 * (int64_t)t + i]);
          gt += (uint32_t)i > d2 ? h : 0u;
          eq += (uint32_t)i == d2 ? h : 0u;
        }
        uint32_t gtot, etot, gp, ep;
        block_excl_scan2(gt, eq, es.scratch, &gp, &ep, &gtot, &etot);
        __syncthreads();  // (every lane read gcnt[2 t] before it is replaced)
        if (w0) { st_sc1(&gcnt[2 * t], gtot); st_sc1(&gcnt[2 * t + 1], etot); }  // same value from every lane
      } else {
        // this tile's output offset and tie start: counts of the tiles before it
        uint32_t gv = 0u, ev = 0u;
        for (uint32_t q = (uint32_t)tid; q < t; q += NT) {
          gv += ld_sc1(&gcnt[2 * q]);
          ev += ld_sc1(&gcnt[2 * q + 1]);
        }
        uint32_t gp, ep, gtot, etot;
        block_excl_scan2(gv, ev, es.scratch, &gp, &ep, &gtot, &etot);
        const uint32_t taken = min(r, etot);  // ties taken by the earlier tiles
        uint32_t out = gtot + taken, tie_run = etot;
        // ordered compaction, row by row: ties by global rank (lowest index first)
        reader(t, [&](int nin, const uint32_t (&kk)[4], const float (&vv)[4], const int64_t (&ii)[4]) {
          uint32_t neq = 0;
#pragma unroll
          for (int c = 0; c < 4; ++c) neq += (c < nin && kk[c] == T) ? 1u : 0u;
          uint32_t tp, tt;
          tp = block_excl_scan(neq, es.scratch, &tt);
          bool sel[4];
          uint32_t ns = 0, q = tie_run + tp;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const bool in = c < nin;
            const bool eqc = in && kk[c] == T;
            sel[c] = (in && kk[c] > T) || (eqc && q < r);
            q += eqc ? 1u : 0u;
            ns += sel[c] ? 1u : 0u;
          }
          uint32_t st;
          uint32_t pos = out + block_excl_scan(ns, es.scratch, &st);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            // (bounded: a wait that gave up leaves the counts unreliable -- the call is flagged
            // invalid, and nothing may be written past the range's k outputs)
            if (sel[c] && pos < (uint64_t)k) emit(pos, ii[c], vv[c]);
            pos += sel[c] ? 1u : 0u;
          }
          out += st;
          tie_run += tt;
        });
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (w0) wave0_fetch_add(&W->done[phase], 1u);
  }
  // the last workgroup out resets the queue for the next call
  if (w0) {
    const uint32_t e = wave0_fetch_add(&W->exitc, 1u);
    *s_tk = e == nb - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (*s_tk) {
    for (int i = tid; i < 3 * 2048; i += NT) st_sc1(&W->hist[0][0] + i, 0u);
    if (tid < 8) st_sc1(&W->done[tid], 0u);
    if (tid == 0) { st_sc1(&W->ticket, 0u); st_sc1(&W->exitc, 0u); }
  }
}

}  // namespace choco
