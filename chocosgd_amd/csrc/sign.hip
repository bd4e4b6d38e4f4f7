// Sign(+norm) compression for the CHOCO gossip step on MI355X.
//
// Replaces SignCompressor.packing/unpacking (reference
// dl_code/pcode/utils/sparsification.py:129-163, including the external
// bit2byte extension) and the norm/sign halves of CHOCOSignCompressor
// (dl_code/pcode/optim/parallel_choco_v.py:476-558).
//
// Layout (the reference's view(32, -1) of the zero-padded flat buffer):
// N' = ceil(n/32) words; word j holds elements e = r*N' + j, r = 0..31, at
// bit r; bit set <=> d < 0.
//
// Work decomposition ("column tiles"): a 256-thread workgroup owns 1024
// consecutive words; each wave owns 256 words and lane l owns words
// j0+4l .. j0+4l+3, so packed words are written once as 16-B stores and every
// element is read exactly once.  For row r the wave's elements are the
// contiguous flat run [r*N' + j0, +256); that run starts at an arbitrary
// alignment m = (r*N' + j0) mod 4 (N' is 2 mod 4 for both BASELINE sign
// configs), so each lane loads the ALIGNED float4 at A + 4l (A = run start
// rounded down to 4), computes its 4 sign bits, and the wave realigns the
// nibbles by one lane shuffle (lane 63 loads one extra float4 for the tail).
// Per-segment L1 norms are accumulated in fp64: a run that lies inside one
// segment is wave-reduced and merged per workgroup (one fp64 atomic per
// segment per workgroup); runs that straddle a segment boundary are reduced
// per segment inside the wave.  The last workgroup (agent-scope ticket)
// rounds the sums to fp32 and zeroes the accumulators for the next call.
#include "choco_common.h"

#include <algorithm>

namespace choco {

constexpr int kSignThreads = 256;
constexpr int kSignCols = 1024;  // words per workgroup

struct SignWs {
  unsigned int ticket;
  unsigned int pad[63];
  // double acc[nseg] follows at offset 256
};

// (16-B stores go through choco_common.h's st_buf4: soffset is always the constant 0.  A
// 16-B buffer store with an SGPR soffset gets no wait state from the compiler before a VALU
// overwrites its data registers, and on gfx950 it can then store the new values -- DESIGN.md
// section 4, "The r5m wrong stores"; tests/test_isa_hazards.py checks the built library.)

CHOCO_DEV void load4g(const float* __restrict__ x, const float* __restrict__ xh, int64_t e, int64_t n,
                      float (&v)[4]) {
  if (e + 3 < n) {
    float4 a = *reinterpret_cast<const float4*>(x + e);
    if (xh) {
      float4 h = *reinterpret_cast<const float4*>(xh + e);
      a.x -= h.x; a.y -= h.y; a.z -= h.z; a.w -= h.w;
    }
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t i = e + c;
      v[c] = (i < n && i >= 0) ? (xh ? x[i] - xh[i] : x[i]) : 0.f;
    }
  }
}

// load4g with the fused gossip step (GS): x_new = x + gamma (memory - xh) for the
// four elements e..e+3, stored back for the elements this wave owns ([own0, own1)
// -- the realigned loads also read neighbours' elements, which are never used),
// v = x_new - xh.
CHOCO_DEV void load4g_gossip(const float* __restrict__ x, const float* __restrict__ xh, const Gossip& gs, int64_t e,
                             int64_t n, int64_t own0, int64_t own1, float (&v)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int64_t i = e + c;
    v[c] = 0.f;
    if (i < n && i >= 0) {
      const float xn = gossip1(x[i], gs.mem[i], xh[i], gs.gamma);
      if (i >= own0 && i < own1) const_cast<float*>(x)[i] = xn;
      v[c] = xn - xh[i];
    }
  }
}

// store x_new of lane-owned elements A+4l+c (c >= m for lane 0) and, for lane 63,
// of the tail A+256+c (c < m): the owned run is [A+m, A+m+256)
CHOCO_DEV void store_owned_gossip(float* __restrict__ x, int64_t A, int m, int lane, float4 a, float4 t) {
  if (lane > 0 || m == 0) {
    *reinterpret_cast<float4*>(x + A + 4 * lane) = a;
  } else {
    const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int c = 1; c < 4; ++c)
      if (c >= m) x[A + c] = av[c];
  }
  if (lane == 63 && m > 0) {
    const float tv[3] = {t.x, t.y, t.z};
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (c < m) x[A + 256 + c] = tv[c];
  }
}

CHOCO_DEV uint32_t neg_bits4(const float (&v)[4]) {
  return (v[0] < 0.f ? 1u : 0u) | (v[1] < 0.f ? 2u : 0u) | (v[2] < 0.f ? 4u : 0u) | (v[3] < 0.f ? 8u : 0u);
}

CHOCO_DEV int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
CHOCO_DEV int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

CHOCO_DEV int seg_walk(const int64_t* __restrict__ seg_off, int nseg, int s0, int64_t e) {
  int s = s0;
  while (s + 1 < nseg && seg_off[s + 1] <= e) ++s;
  return s;
}

// Per-row segment info for this workgroup's 32 row runs.
CHOCO_DEV void row_segments(const int64_t* __restrict__ seg_off, int nseg, int64_t n, int64_t Np, int64_t J0,
                            int* s_lo, int* s_hi) {
  if (threadIdx.x < 32) {
    const int r = threadIdx.x;
    const int64_t jend = std::min<int64_t>(J0 + kSignCols, Np);
    const int64_t e0 = (int64_t)r * Np + J0;
    const int64_t e1 = std::min<int64_t>((int64_t)r * Np + jend, n) - 1;
    if (e0 < n && e1 >= e0) {
      s_lo[r] = nseg > 1 ? seg_of(seg_off, nseg, e0) : 0;
      s_hi[r] = nseg > 1 ? seg_of(seg_off, nseg, e1) : 0;
    } else {
      s_lo[r] = -1;
      s_hi[r] = -1;
    }
  }
}

// GS: the fused gossip step (x_new written back for the wave's own elements).
template <bool XH, bool NORM, bool GS = false>
__global__ __launch_bounds__(kSignThreads) void sign_pack_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, int64_t Np,
    const int64_t* __restrict__ seg_off, int nseg, uint32_t* __restrict__ packed, float* __restrict__ l1_out,
    SignWs* __restrict__ ws, Gossip gs, int64_t blk0, int finish) {
  static_assert(!GS || XH, "the gossip step needs x_hat");
  __shared__ int s_lo[32], s_hi[32];
  __shared__ double s_rows[kSignThreads / 64][32];
  __shared__ unsigned int s_flag;
  double* __restrict__ acc = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + 256);
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int64_t J0 = (blk0 + (int64_t)blockIdx.x) * kSignCols;
  const int64_t j0 = J0 + 256 * w;
  const int ncol = (int)std::max<int64_t>(0, std::min<int64_t>(256, Np - j0));

  uint32_t wd[4] = {0u, 0u, 0u, 0u};
  // Interior workgroups (every row run, incl. the tail float4, inside [0, n)) use
  // UNCONDITIONAL loads so all RU rows stay in flight (a branch around a load makes
  // the compiler wait for it right away); only the last workgroups take the guarded path.
  const bool interior = ncol == 256 && (int64_t)31 * Np + j0 + 260 <= n;
  constexpr int RU = 8;  // rows whose loads are in flight together
  for (int r0 = 0; r0 < 32; r0 += RU) {
  float vr[RU][4], tr[RU][4];
  if (interior) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t A = ((int64_t)(r0 + u) * Np + j0) & ~(int64_t)3;
      float4 a = ld_nt4(x + A + 4 * lane);
      float4 t = *reinterpret_cast<const float4*>(x + A + 256);  // tail (used by lane 63; broadcast)
      if (XH) {
        const float4 h = ld_nt4(xh + A + 4 * lane);
        const float4 ht = *reinterpret_cast<const float4*>(xh + A + 256);
        if (GS) {
          const float4 am = ld_nt4(gs.mem + A + 4 * lane);
          const float4 tm = *reinterpret_cast<const float4*>(gs.mem + A + 256);
          a = gossip4(a, am, h, gs.gamma);
          t = gossip4(t, tm, ht, gs.gamma);
          store_owned_gossip(const_cast<float*>(x), A, (int)(((int64_t)(r0 + u) * Np + j0) & 3), lane, a, t);
        }
        a.x -= h.x; a.y -= h.y; a.z -= h.z; a.w -= h.w;
        t.x -= ht.x; t.y -= ht.y; t.z -= ht.z; t.w -= ht.w;
      }
      vr[u][0] = a.x; vr[u][1] = a.y; vr[u][2] = a.z; vr[u][3] = a.w;
      tr[u][0] = t.x; tr[u][1] = t.y; tr[u][2] = t.z; tr[u][3] = t.w;
    }
  } else {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t s = (int64_t)(r0 + u) * Np + j0;
#pragma unroll
      for (int c = 0; c < 4; ++c) { vr[u][c] = 0.f; tr[u][c] = 0.f; }
      if (ncol > 0 && s < n) {
        const int64_t A = s & ~(int64_t)3;
        if (GS) {
          load4g_gossip(x, xh, gs, A + 4 * lane, n, s, s + ncol, vr[u]);
          if ((s & 3) != 0 && lane == 63) load4g_gossip(x, xh, gs, A + 256, n, s, s + ncol, tr[u]);
        } else {
          load4g(x, XH ? xh : nullptr, A + 4 * lane, n, vr[u]);
          if ((s & 3) != 0 && lane == 63) load4g(x, XH ? xh : nullptr, A + 256, n, tr[u]);
        }
      }
    }
  }
  if (r0 == 0) {
    // the rows' segments, looked up (binary searches) while the first group's loads are in flight
    if (NORM) row_segments(seg_off, nseg, n, Np, J0, s_lo, s_hi);
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    const int r = r0 + u;
    const int64_t s = (int64_t)r * Np + j0;
    double rowpart = 0.0;
    if (ncol > 0 && s < n) {  // wave-uniform
      const int64_t A = s & ~(int64_t)3;
      const int m = (int)(s & 3);
      const int64_t e = A + 4 * lane;
      const float(&v)[4] = vr[u];
      const float(&t)[4] = tr[u];
      const uint32_t b4 = neg_bits4(v);
      uint32_t nb4 = __shfl_down(b4, 1);
      if (lane == 63) nb4 = neg_bits4(t);
      const uint32_t w4 = m ? (((b4 >> m) | (nb4 << (4 - m))) & 15u) : b4;
#pragma unroll
      for (int c = 0; c < 4; ++c) wd[c] |= ((w4 >> c) & 1u) << r;
      if (NORM) {
        const int64_t lim = std::min<int64_t>(s + ncol, n);
        const bool uniform = s_lo[r] == s_hi[r];
        if (uniform) {
          double p = 0.0;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (e + c >= s && e + c < lim) p += (double)fabsf(v[c]);
          if (lane == 63) {
#pragma unroll
            for (int c = 0; c < 3; ++c)
              if (c < m && A + 256 + c < lim) p += (double)fabsf(t[c]);
          }
          rowpart = wave_sum(p);
        } else {
          int sg[4], tg[4];
          int lo = 0x7fffffff, hi = -1;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            sg[c] = -1;
            if (e + c >= s && e + c < lim) {
              sg[c] = seg_walk(seg_off, nseg, s_lo[r], e + c);
              lo = min(lo, sg[c]);
              hi = max(hi, sg[c]);
            }
            tg[c] = -1;
            if (lane == 63 && c < m && A + 256 + c < lim) {
              tg[c] = seg_walk(seg_off, nseg, s_lo[r], A + 256 + c);
              lo = min(lo, tg[c]);
              hi = max(hi, tg[c]);
            }
          }
          lo = wave_min_i(lo);
          hi = wave_max_i(hi);
          for (int q = lo; q <= hi; ++q) {
            double p = 0.0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              if (sg[c] == q) p += (double)fabsf(v[c]);
              if (tg[c] == q) p += (double)fabsf(t[c]);
            }
            p = wave_sum(p);
            if (lane == 0 && p != 0.0) unsafeAtomicAdd(&acc[q], p);
          }
        }
      }
    }
    if (NORM && lane == 0) s_rows[w][r] = rowpart;
  }
  }
  // packed words: 16-B stores where possible
  {
    const int64_t j = j0 + 4 * lane;
    if (j + 3 < Np) {
      *reinterpret_cast<uint4*>(packed + j) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (j + c < Np) packed[j + c] = wd[c];
    }
  }
  if (NORM) {
    __syncthreads();
    if (threadIdx.x == 0) {
      int cur = -1;
      double run = 0.0;
      for (int r = 0; r < 32; ++r) {
        if (s_lo[r] < 0 || s_lo[r] != s_hi[r]) continue;
        double v = 0.0;
#pragma unroll
        for (int ww = 0; ww < kSignThreads / 64; ++ww) v += s_rows[ww][r];
        if (s_lo[r] != cur) {
          if (cur >= 0 && run != 0.0) unsafeAtomicAdd(&acc[cur], run);
          cur = s_lo[r];
          run = 0.0;
        }
        run += v;
      }
      if (cur >= 0 && run != 0.0) unsafeAtomicAdd(&acc[cur], run);
    }
    if (finish && last_block_ticket_atomics(&ws->ticket, gridDim.x, &s_flag)) {
      for (int q = threadIdx.x; q < nseg; q += blockDim.x) l1_out[q] = (float)atomic_exchange_double(&acc[q], 0.0);
      if (threadIdx.x == 0) __hip_atomic_store(&ws->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One-segment pack (nseg == 1: the whole flat buffer has one norm): the same
// column tiles, but each lane loads the float4 at its OWN run offset
// s + 4l -- a dword-aligned (not 16-B aligned) global_load_dwordx4, which
// gfx950 serves directly -- so there is no tail load and no realigning
// shuffle.  Rows go in groups of RU with two groups in flight (A/B register
// double buffer, non-temporal loads), and the L1 norm accumulates per lane in
// fp64 over all 32 rows, with one wave reduction at the end.
// Loads go through a raw buffer resource over the whole input (n * 4 < 2^32
// bytes): the row offset is a wave-uniform SGPR operand and the lane offset
// one VGPR, so the 2 x RU loads in flight need no 64-bit address registers.

// GS: the fused gossip step -- x, memory and xh rows in flight, x_new stored back
// (each lane owns its float4 of every row run: no overlap), d = x_new - xh.
// SEG (per-tensor norms, NORM only): the 32 rows' segments over the workgroup's 1024
// columns are looked up while the first two groups' loads are in flight; a lane keeps one
// running sum while consecutive rows stay in one segment, and a wave sum goes to the
// workgroup's LDS per-segment sums when the segment changes (a row across a boundary: one
// wave sum per segment in it); the workgroup adds its LDS sums to the global ones.
constexpr int kRowRep = 8;  // replicas of the fp64 L1 accumulators (workgroup b -> replica b & 7)
constexpr int kPackSegLds = 1024;  // segments of one workgroup's rows summed in LDS (more: global atomics)
// RS = 2 (small grids): eight waves per workgroup, waves w and w + 4 take rows 0-15 and 16-31
// of the same 256 columns (twice the waves resident per column block); the upper half's
// words are OR-ed in through LDS.
template <bool XH, bool NORM, bool GS = false, bool SEG = false, int RUV = 0, int RS = 1>
__global__ __launch_bounds__(kSignThreads * RS) void sign_pack1_kernel(const float* __restrict__ x,
                                                                  const float* __restrict__ xh, int64_t n,
                                                                  int64_t Np, uint32_t* __restrict__ packed,
                                                                  float* __restrict__ l1_out,
                                                                  SignWs* __restrict__ ws, Gossip gs, int64_t blk0,
                                                                  int finish, const int64_t* __restrict__ seg_off,
                                                                  int nseg) {
  static_assert(!GS || XH, "the gossip step needs x_hat");
  static_assert(!SEG || NORM, "segments only matter to the norms");
  constexpr int RU = RUV ? RUV : (GS ? 8 : (XH ? 4 : 8));  // rows per group (more streams, more registers)
  constexpr int kT = kSignThreads * RS;                     // threads per workgroup
  constexpr int NR = 32 / RS;                               // rows per wave
  constexpr int NG = NR / RU;
  static_assert(NG >= 2 && NG % 2 == 0, "groups go in A/B pairs");
  __shared__ double s_red[kT / 64];
  __shared__ uint4 s_wd[RS > 1 ? 4 : 1][64];
  __shared__ unsigned int s_flag;
  __shared__ int s_lo[SEG ? 32 : 1], s_hi[SEG ? 32 : 1];
  __shared__ double s_sacc[SEG ? kPackSegLds : 1];
  __shared__ int64_t s_so[SEG ? kSegLdsCap : 1];
  double* __restrict__ acc = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + 256);
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int wq = w & 3, rs0 = (w >> 2) * NR;  // the wave's 256 columns and first row
  const int64_t J0 = (blk0 + (int64_t)blockIdx.x) * kSignCols;
  const int64_t j0 = J0 + 256 * wq;
  const int ncol = (int)std::max<int64_t>(0, std::min<int64_t>(256, Np - j0));
  // every row run of the wave (row 31's last float4 included) lies inside [0, n)
  const bool interior = ncol == 256 && (int64_t)31 * Np + j0 + 256 <= n;
  const __amdgpu_buffer_rsrc_t rx = buf_rsrc(x, (uint32_t)(n * 4));
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc(XH ? xh : x, (uint32_t)(n * 4));
  const __amdgpu_buffer_rsrc_t rm = buf_rsrc(GS ? gs.mem : x, (uint32_t)(n * 4));
  const uint32_t voff = 16u * (uint32_t)lane;
  auto row_off = [&](int r) -> uint32_t { return (uint32_t)(((int64_t)r * Np + j0) * 4); };  // wave-uniform
  // A group's raw rows (x; xh; memory) stay in flight until the group is processed:
  // the delta and the gossip step's x_new are formed in proc_group, so the other
  // group's loads are not waited for early.
  struct Group {
    float4 x[RU], h[RU], m[RU];
  };
  auto load_group = [&](int g, Group& G) {
#pragma unroll
    for (int u = 0; u < RU; ++u) G.x[u] = ld_buf4s<true>(rx, voff, row_off(rs0 + g * RU + u));
    if (XH) {
#pragma unroll
      for (int u = 0; u < RU; ++u) G.h[u] = ld_buf4s<true>(rh, voff, row_off(rs0 + g * RU + u));
    }
    if (GS) {
#pragma unroll
      for (int u = 0; u < RU; ++u) G.m[u] = ld_buf4s<true>(rm, voff, row_off(rs0 + g * RU + u));
    }
  };
  uint32_t wd[4] = {0u, 0u, 0u, 0u};
  double p = 0.0;
  // SEG: the rows' segments (s_lo / s_hi), the workgroup's first one and whether its
  // segment span fits the LDS sums; a lane's running sum belongs to segment `cur`
  int sbase = 0;
  bool slds = true;
  int cur = -1;
  int lo_v = 0, hi_v = 0;  // lane l: row (l & 31)'s first and last segment (read back with readlane)
  auto seg_lookup = [&]() {
    if (SEG) {
      row_segments(stage_seg_off(seg_off, nseg, s_so), nseg, n, Np, J0, s_lo, s_hi);
      __syncthreads();
      lo_v = s_lo[lane & 31];
      hi_v = s_hi[lane & 31];
      int lo = s_lo[0] >= 0 ? s_lo[0] : 0, hi = 0;
      for (int r = 31; r >= 0; --r)
        if (s_hi[r] >= 0) { hi = s_hi[r]; break; }
      sbase = lo;
      slds = hi - lo < kPackSegLds;
      if (slds)
        for (int i = threadIdx.x; i <= hi - lo; i += kT) s_sacc[i] = 0.0;
      __syncthreads();
    }
  };
  // the global sums: kRowRep replicas (workgroup b -> replica b & 7), summed by the finish
  double* __restrict__ rep = acc + (size_t)(blockIdx.x & (kRowRep - 1)) * (size_t)(SEG ? nseg : 1);
  auto seg_add = [&](int sg, double v) {  // lane 0 of a wave
    if (v == 0.0) return;
    if (slds) atomicAdd(&s_sacc[sg - sbase], v);
    else unsafeAtomicAdd(&rep[sg], v);
  };
  auto seg_flush = [&]() {  // wave-uniform
    if (cur >= 0) {
      const double t = wave_sum(p);
      if (lane == 0) seg_add(cur, t);
    }
    p = 0.0;
  };
  // one row's |d| (valid elements only) into the norms
  auto seg_row = [&](int r, const float (&v)[4], uint32_t valid) {
    if (!SEG) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if ((valid >> c) & 1u) p += (double)fabsf(v[c]);
      return;
    }
    const int lo = __builtin_amdgcn_readlane(lo_v, r), hi = __builtin_amdgcn_readlane(hi_v, r);
    if (lo < 0) return;  // (a row run past n)
    if (lo == hi) {      // wave-uniform
      if (lo != cur) {
        seg_flush();
        cur = lo;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if ((valid >> c) & 1u) p += (double)fabsf(v[c]);
      return;
    }
    seg_flush();
    cur = -1;
    const int64_t e = (int64_t)r * Np + j0 + 4 * lane;
    int sg[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) sg[c] = ((valid >> c) & 1u) ? seg_walk(seg_off, nseg, lo, e + c) : -1;
    for (int q = lo; q <= hi; ++q) {
      double t = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (sg[c] == q) t += (double)fabsf(v[c]);
      t = wave_sum(t);
      if (lane == 0) seg_add(q, t);
    }
  };
  auto proc_group = [&](int g, Group& G) {
    if (GS) {
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        G.x[u] = gossip4(G.x[u], G.m[u], G.h[u], gs.gamma);
        // non-temporal: x_new is not re-read by this step, and dirty Infinity-Cache
        // lines would be written back in the middle of the receiver's pass.
        // The row offset goes in the VGPR offset, soffset 0: a 16-B buffer store whose
        // soffset is an SGPR gets no wait state from the compiler before a VALU overwrites
        // its data registers, and on gfx950 such a store can write the NEW values (the r5m
        // wrong x / memory stores; DESIGN.md section 4, tests/test_isa_hazards.py).
        st_buf4<true>(rx, voff + row_off(rs0 + g * RU + u), G.x[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = rs0 + g * RU + u;
      const float4 R = XH ? sub4(G.x[u], G.h[u]) : G.x[u];
      const float v[4] = {R.x, R.y, R.z, R.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) wd[c] |= (v[c] < 0.f ? 1u : 0u) << r;
      if (NORM) {
        if (SEG) seg_row(r, v, 15u);
        else p += ((double)fabsf(v[0]) + (double)fabsf(v[1])) + ((double)fabsf(v[2]) + (double)fabsf(v[3]));
      }
      __builtin_amdgcn_sched_barrier(0);  // row by row: hoisted fp64 conversions of a whole group cost registers
    }
  };
  // (sched_barrier: keep each group's loads where they are written -- hoisted,
  // all 32 rows would be live at once)
  if (interior) {
    Group A, B;
    load_group(0, A);
    load_group(1, B);
    seg_lookup();
#pragma unroll
    for (int g = 0; g < NG; g += 2) {
      proc_group(g, A);
      if (g + 2 < NG) load_group(g + 2, A);
      proc_group(g + 1, B);
      if (g + 3 < NG) load_group(g + 3, B);
    }
  } else {
    // the last workgroups: guarded element loads, one row at a time
    seg_lookup();
#pragma unroll 1
    for (int r = rs0; r < rs0 + NR; ++r) {
      const int64_t s = (int64_t)r * Np + j0 + 4 * lane;
      float tt[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t e = s + c;
        if (GS) {
          tt[c] = 0.f;
          if (4 * lane + c < ncol && e < n) {
            const float xn = gossip1(x[e], gs.mem[e], xh[e], gs.gamma);
            const_cast<float*>(x)[e] = xn;
            tt[c] = xn - xh[e];
          }
        } else {
          tt[c] = (4 * lane + c < ncol && e < n) ? (XH ? x[e] - xh[e] : x[e]) : 0.f;
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) wd[c] |= (tt[c] < 0.f ? 1u : 0u) << r;
      if (NORM) {
        if (SEG) {
          uint32_t valid = 0;
#pragma unroll
          for (int c = 0; c < 4; ++c) valid |= (4 * lane + c < ncol && s + c < n ? 1u : 0u) << c;
          seg_row(r, tt, valid);
        } else {
          p += ((double)fabsf(tt[0]) + (double)fabsf(tt[1])) + ((double)fabsf(tt[2]) + (double)fabsf(tt[3]));
        }
      }
    }
  }
  if (RS > 1) {  // the upper rows' bits through LDS
    if (w >= 4) s_wd[wq][lane] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    __syncthreads();
    if (w < 4) {
      const uint4 o = s_wd[wq][lane];
      wd[0] |= o.x; wd[1] |= o.y; wd[2] |= o.z; wd[3] |= o.w;
    }
  }
  if (w < 4) {
    const int64_t j = j0 + 4 * lane;
    if (j + 3 < Np) {
      *reinterpret_cast<uint4*>(packed + j) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (j + c < Np) packed[j + c] = wd[c];
    }
  }
  if (NORM && SEG) {
    seg_flush();
    __syncthreads();
    if (slds) {
      int hi = 0;
      for (int r = 31; r >= 0; --r)
        if (s_hi[r] >= 0) { hi = s_hi[r]; break; }
      for (int i = threadIdx.x; i <= hi - sbase; i += kT)
        if (s_sacc[i] != 0.0) unsafeAtomicAdd(&rep[sbase + i], s_sacc[i]);
    }
    if (finish && last_block_ticket_atomics(&ws->ticket, gridDim.x, &s_flag)) {
      for (int q = threadIdx.x; q < nseg; q += kT) {
        double t = 0.0;
        for (int i = 0; i < kRowRep; ++i) t += atomic_exchange_double(&acc[(size_t)i * nseg + q], 0.0);
        l1_out[q] = (float)t;
      }
      if (threadIdx.x == 0) __hip_atomic_store(&ws->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (NORM) {
    p = wave_sum(p);
    if (lane == 0) s_red[w] = p;
    __syncthreads();
    if (threadIdx.x == 0) {
      double tsum = 0.0;
#pragma unroll
      for (int i = 0; i < kT / 64; ++i) tsum += s_red[i];
      if (tsum != 0.0) unsafeAtomicAdd(&acc[0], tsum);
    }
    if (finish && last_block_ticket_atomics(&ws->ticket, gridDim.x, &s_flag)) {
      if (threadIdx.x == 0) {
        l1_out[0] = (float)atomic_exchange_double(&acc[0], 0.0);
        __hip_atomic_store(&ws->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Decode to +-1 floats (SignCompressor.unpacking).
__global__ __launch_bounds__(kSignThreads) void sign_unpack_kernel(const uint32_t* __restrict__ packed,
                                                                   int64_t n, int64_t Np,
                                                                   float* __restrict__ out) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * kSignCols + 256 * w;
  const int ncol = (int)std::max<int64_t>(0, std::min<int64_t>(256, Np - j0));
  if (ncol == 0) return;
  uint32_t wd[4];
  {
    const int64_t j = j0 + 4 * lane;
#pragma unroll
    for (int c = 0; c < 4; ++c) wd[c] = (j + c < Np) ? packed[j + c] : 0u;
  }
  for (int r = 0; r < 32; ++r) {
    const int64_t s = (int64_t)r * Np + j0;
    if (s >= n) break;
    const int64_t A = s & ~(int64_t)3;
    const int m = (int)(s & 3);
    const int64_t e = A + 4 * lane;
    const int64_t lim = std::min<int64_t>(s + ncol, n);
    uint32_t own4 = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) own4 |= ((wd[c] >> r) & 1u) << c;
    const uint32_t prev4 = __shfl_up(own4, 1);
    const uint32_t x8 = (own4 << 4) | prev4;
    float o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = ((x8 >> (4 + c - m)) & 1u) ? -1.f : 1.f;
    if (e >= s && e + 3 < lim) {
      *reinterpret_cast<float4*>(out + e) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (e + c >= s && e + c < lim) out[e + c] = o[c];
    }
    if (lane == 63)
      for (int c = 0; c < m; ++c)
        if (A + 256 + c < lim) out[A + 256 + c] = ((own4 >> (4 + c - m)) & 1u) ? -1.f : 1.f;
  }
}

// Fused receiver update over up to 8 messages (CHOCOSignCompressor.uncompress).
constexpr int kMaxMsg = 8;
struct SignMsgs {
  const uint32_t* packed[kMaxMsg];
  const float* norms[kMaxMsg];
  float w[kMaxMsg];
  int nmsg;
  int self_slot;
  // memory update: 0 = fmaf(w, u, memory) (torch add_(u, alpha=w)); 1 = memory + (w * u)
  // (add_(w * u)); 2 = (memory * a) + u with u = ((b * norm) / numel) * sign (ECD's
  // extrapolation, ecd_psgd.py:448-454; w unused)
  int mode;
  float a, b;
};

CHOCO_DEV float sign_axpy(const SignMsgs& M, int q, float u, float m) {
  if (M.mode == 2) return m * M.a + u;
  return M.mode == 1 ? m + M.w[q] * u : fmaf(M.w[q], u, m);
}

template <int NM>
CHOCO_DEV void sign_apply(const SignMsgs& M, const float (&sc)[kMaxMsg], const uint32_t (&bits)[kMaxMsg],
                          int shiftbit, float& h, float& mm) {
#pragma unroll
  for (int q = 0; q < NM; ++q) {
    const float u = ((bits[q] >> shiftbit) & 1u) ? -sc[q] : sc[q];  // (norm/numel) * (+-1), exact
    if (q == M.self_slot) h = h + u;
    mm = sign_axpy(M, q, u, mm);  // torch add_(u, alpha=w) fuses on CPU (verified)
  }
}

CHOCO_DEV float seg_scale(const SignMsgs& M, int q, const int64_t* __restrict__ seg_off, int64_t n, int seg) {
  const int64_t numel = seg_off ? seg_off[seg + 1] - seg_off[seg] : n;
  const float nm = M.mode == 2 ? M.b * M.norms[q][seg] : M.norms[q][seg];
  return nm / (float)numel;
}

constexpr int kSAccRU = 4;  // rows per load group in the receiver
// Rows of the (32, N') view one receiver workgroup covers (32 / kSAccRows workgroups
// per 1024-column block).  Block L -> (column block, row block) keeps the row blocks
// of one column block on ONE XCD (linear ids congruent mod 8), so their word loads
// hit that XCD's L2.
constexpr int kSAccRows = 8;
constexpr int kSAccRB = 32 / kSAccRows;  // row blocks per column block
static_assert(kSAccRows % kSAccRU == 0 && 32 % kSAccRows == 0, "row blocking");
CHOCO_DEV void sign_acc_block(uint32_t L, int64_t& cb, int& rb) {
  if (kSAccRB == 1) {
    cb = L;
    rb = 0;
    return;
  }
  const uint32_t rest = L / 8;
  rb = (int)(rest % kSAccRB) * kSAccRows;
  cb = (int64_t)(L % 8) + 8 * (int64_t)(rest / kSAccRB);
}
static unsigned sign_acc_grid(int64_t Np) {
  const int64_t ncb = (Np + kSignCols - 1) / kSignCols;
  return kSAccRB == 1 ? (unsigned)ncb : (unsigned)((ncb + 7) / 8 * 8 * kSAccRB);
}
// NT (large buffers, n >= kSaccNtMin: x_hat and memory far beyond the 256 MB Infinity Cache):
// the interior rows' loads and stores non-temporal, so the receive does not leave dirty lines
// in the cache for the next step's pack to meet.  Same-box A/B (r05_ab_summary.txt item 23):
// `sign` (345M) 1.351-1.370 against 1.415-1.468 ms per step; at ResNet-50's 25.6M, whose x_hat
// and memory fit the cache, non-temporal was 11 % slower (plain kept there).
constexpr int64_t kSaccNtMin = int64_t(1) << 25;
template <bool NT>
CHOCO_DEV float4 sacc_ld4(const float* p) {
  if (NT) return ld_nt4(p);
  return *reinterpret_cast<const float4*>(p);
}
template <bool NT>
CHOCO_DEV void sacc_st4(float* p, float4 v) {
  if (NT) {
    choco_f32x4 f;
    f.x = v.x; f.y = v.y; f.z = v.z; f.w = v.w;
    __builtin_nontemporal_store(f, reinterpret_cast<choco_f32x4*>(p));
    return;
  }
  *reinterpret_cast<float4*>(p) = v;
}
template <int NM, bool HS, bool NT = false>
__global__ __launch_bounds__(kSignThreads) void sign_accumulate_kernel(SignMsgs M, int64_t n, int64_t Np,
                                                                       const int64_t* __restrict__ seg_off,
                                                                       int nseg, float* __restrict__ hat,
                                                                       float* __restrict__ mem) {
  __shared__ int s_lo[32], s_hi[32];
  __shared__ float s_sc[kMaxMsg][32];
  const int lane = lane_id(), w = threadIdx.x >> 6;
  int64_t cb;
  int rb;
  sign_acc_block(blockIdx.x, cb, rb);
  if (cb * kSignCols >= Np) return;  // workgroup-uniform (grid padded to a multiple of 8 column blocks)
  const int64_t J0 = cb * kSignCols;
  const int64_t j0 = J0 + 256 * w;
  const int ncol = (int)std::max<int64_t>(0, std::min<int64_t>(256, Np - j0));
  row_segments(seg_off, nseg, n, Np, J0, s_lo, s_hi);
  __syncthreads();
  // per-row (norm / numel) of every message for rows inside one segment: all global
  // loads of the scales happen here, before the streaming loop
  if (threadIdx.x < NM * 32) {
    const int q = threadIdx.x >> 5, r = threadIdx.x & 31;
    s_sc[q][r] = (s_lo[r] >= 0 && s_lo[r] == s_hi[r]) ? seg_scale(M, q, seg_off, n, s_lo[r]) : 0.f;
  }
  __syncthreads();
  if (ncol == 0) return;
  uint32_t wd[NM][4];
  {
    const int64_t j = j0 + 4 * lane;
#pragma unroll
    for (int q = 0; q < NM; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) wd[q][c] = (j + c < Np) ? M.packed[q][j + c] : 0u;
  }
  // interior workgroups: unconditional loads keep all RU rows in flight
  const bool interior = ncol == 256 && (int64_t)31 * Np + j0 + 260 <= n;
  constexpr int RU = kSAccRU;
  bool all_uniform = true;
#pragma unroll
  for (int r = 0; r < kSAccRows; ++r) all_uniform &= s_lo[rb + r] == s_hi[rb + r];
  // (Buffer loads at each lane's own run offset, as sign_pack1_kernel -- no tail loads, no
  // realigning shuffle -- measured slower here: 1212-1222 against 1153-1155 us at 345M, fused
  // step 1140-1157 against 1065-1066; r05_ab_summary.txt item 20.)
  if (interior && all_uniform) {
    // fast path: no segment lookups, no global memory op besides the prefetch and the stores
    for (int r0 = rb; r0 < rb + kSAccRows; r0 += RU) {
      float4 pm[RU], ph[RU], tm[RU], th[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int64_t A = ((int64_t)(r0 + u) * Np + j0) & ~(int64_t)3;
        pm[u] = sacc_ld4<NT>(mem + A + 4 * lane);
        tm[u] = *reinterpret_cast<const float4*>(mem + A + 256);
        if (HS) {
          ph[u] = sacc_ld4<NT>(hat + A + 4 * lane);
          th[u] = *reinterpret_cast<const float4*>(hat + A + 256);
        }
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int r = r0 + u;
        const int64_t s = (int64_t)r * Np + j0;
        const int64_t A = s & ~(int64_t)3;
        const int m = (int)(s & 3);
        const int64_t e = A + 4 * lane;
        uint32_t x8[kMaxMsg];
        float sc[kMaxMsg];
#pragma unroll
        for (int q = 0; q < NM; ++q) {
          uint32_t own4 = 0;
#pragma unroll
          for (int c = 0; c < 4; ++c) own4 |= ((wd[q][c] >> r) & 1u) << c;
          const uint32_t prev4 = __shfl_up(own4, 1);
          x8[q] = (own4 << 4) | prev4;
          sc[q] = s_sc[q][r];
        }
        float mv[4] = {pm[u].x, pm[u].y, pm[u].z, pm[u].w};
        float hv[4] = {ph[u].x, ph[u].y, ph[u].z, ph[u].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) sign_apply<NM>(M, sc, x8, 4 + c - m, hv[c], mv[c]);
        if (lane != 0 || m == 0) {
          sacc_st4<NT>(mem + e, make_float4(mv[0], mv[1], mv[2], mv[3]));
          if (HS) sacc_st4<NT>(hat + e, make_float4(hv[0], hv[1], hv[2], hv[3]));
        } else {
#pragma unroll
          for (int c = 1; c < 4; ++c) {  // lane 0: elements before the run belong to the previous wave
            if (c >= m) {
              mem[e + c] = mv[c];
              if (HS) hat[e + c] = hv[c];
            }
          }
        }
        if (lane == 63 && m > 0) {
          const float tmv[4] = {tm[u].x, tm[u].y, tm[u].z, tm[u].w};
          const float thv[4] = {th[u].x, th[u].y, th[u].z, th[u].w};
          uint32_t own[kMaxMsg];
#pragma unroll
          for (int q = 0; q < NM; ++q) own[q] = x8[q] >> 4;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            if (c < m) {
              float h1 = thv[c], m1 = tmv[c];
              sign_apply<NM>(M, sc, own, 4 + c - m, h1, m1);
              mem[A + 256 + c] = m1;
              if (HS) hat[A + 256 + c] = h1;
            }
          }
        }
      }
    }
    return;
  }
  for (int r0 = rb; r0 < rb + kSAccRows; r0 += RU) {
    float4 pm[RU], ph[RU], tm[RU], th[RU];
    if (interior) {
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int64_t A = ((int64_t)(r0 + u) * Np + j0) & ~(int64_t)3;
        pm[u] = *reinterpret_cast<const float4*>(mem + A + 4 * lane);
        tm[u] = *reinterpret_cast<const float4*>(mem + A + 256);  // tail float4 (lane 63; broadcast)
        if (HS) {
          ph[u] = *reinterpret_cast<const float4*>(hat + A + 4 * lane);
          th[u] = *reinterpret_cast<const float4*>(hat + A + 256);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int64_t s = (int64_t)(r0 + u) * Np + j0;
        const int64_t e = (s & ~(int64_t)3) + 4 * lane;
        const int64_t lim = std::min<int64_t>(s + ncol, n);
        pm[u] = ph[u] = tm[u] = th[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (s < n && e >= s && e + 3 < lim) {
          pm[u] = *reinterpret_cast<const float4*>(mem + e);
          if (HS) ph[u] = *reinterpret_cast<const float4*>(hat + e);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = r0 + u;
      const int64_t s = (int64_t)r * Np + j0;
      if (s >= n) continue;
      const int64_t A = s & ~(int64_t)3;
      const int m = (int)(s & 3);
      const int64_t e = A + 4 * lane;
      const int64_t lim = std::min<int64_t>(s + ncol, n);
      uint32_t x8[kMaxMsg];
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        uint32_t own4 = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) own4 |= ((wd[q][c] >> r) & 1u) << c;
        const uint32_t prev4 = __shfl_up(own4, 1);
        x8[q] = (own4 << 4) | prev4;
      }
      const bool uniform = s_lo[r] == s_hi[r];
      float sc[kMaxMsg];
#pragma unroll
      for (int q = 0; q < NM; ++q) sc[q] = s_sc[q][r];
      // main float4 of this lane
      const bool full = e >= s && e + 3 < lim;
      float mv[4] = {pm[u].x, pm[u].y, pm[u].z, pm[u].w};
      float hv[4] = {ph[u].x, ph[u].y, ph[u].z, ph[u].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t i = e + c;
        if (!(i >= s && i < lim)) continue;
        if (!interior && !full) {
          mv[c] = mem[i];
          if (HS) hv[c] = hat[i];
        }
        float scl[kMaxMsg];
        if (uniform) {
#pragma unroll
          for (int q = 0; q < NM; ++q) scl[q] = sc[q];
        } else {
          const int sg = seg_walk(seg_off, nseg, s_lo[r], i);
#pragma unroll
          for (int q = 0; q < NM; ++q) scl[q] = seg_scale(M, q, seg_off, n, sg);
        }
        sign_apply<NM>(M, scl, x8, 4 + c - m, hv[c], mv[c]);
      }
      if (full) {
        *reinterpret_cast<float4*>(mem + e) = make_float4(mv[0], mv[1], mv[2], mv[3]);
        if (HS) *reinterpret_cast<float4*>(hat + e) = make_float4(hv[0], hv[1], hv[2], hv[3]);
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int64_t i = e + c;
          if (i >= s && i < lim) {
            mem[i] = mv[c];
            if (HS) hat[i] = hv[c];
          }
        }
      }
      // tail elements of lane 63 (columns 256-m .. 255 of this run)
      if (lane == 63 && m > 0) {
        const float tmv[4] = {tm[u].x, tm[u].y, tm[u].z, tm[u].w};
        const float thv[4] = {th[u].x, th[u].y, th[u].z, th[u].w};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int64_t i = A + 256 + c;
          if (c >= m || i >= lim) continue;
          float h1 = interior ? thv[c] : (HS ? hat[i] : 0.f);
          float m1 = interior ? tmv[c] : mem[i];
          float scl[kMaxMsg];
          if (uniform) {
#pragma unroll
            for (int q = 0; q < NM; ++q) scl[q] = sc[q];
          } else {
            const int sg = seg_walk(seg_off, nseg, s_lo[r], i);
#pragma unroll
            for (int q = 0; q < NM; ++q) scl[q] = seg_scale(M, q, seg_off, n, sg);
          }
          uint32_t own[kMaxMsg];
#pragma unroll
          for (int q = 0; q < NM; ++q) own[q] = x8[q] >> 4;  // this lane's own nibble
          sign_apply<NM>(M, scl, own, 4 + c - m, h1, m1);
          mem[i] = m1;
          if (HS) hat[i] = h1;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- the receive in row runs
// Deferred receive (one segment) over ROW RUNS of the (32, N') view instead of column
// tiles: a workgroup streams 4096 consecutive columns of ONE row -- 16 KiB contiguous of
// x, x_hat and memory each, the access shape of a flat stream -- and needs bit r of 4096
// consecutive words of every message.  Those come from bit PLANES: plane[r][p] bit b =
// word 32 p + b bit r, made from each message by a 32 x 32 bit transpose per 32 words
// (sign_to_planes_kernel), and this step's words are made back from the output planes
// the same way (sign_from_planes_kernel).  The transposes read and write n / 8 bytes per
// message; the row runs save the column tiles' 32 separate row streams per workgroup.
constexpr int kPlaneThreads = 256;
constexpr int kRowRun = 4096;      // columns per workgroup of the row-run receive
static_assert(kRowRun == 4 * 4 * kSignThreads, "four float4 per thread per run");
__host__ __device__ inline int64_t plane_words(int64_t Np) { return (Np + 31) / 32; }

// In place: w[r] bit b <-> w[b] bit r (LSB-first), five rounds of masked block swaps.
CHOCO_DEV void transpose32(uint32_t (&w)[32]) {
  const uint32_t masks[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int m = 16 >> k;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      if ((i & m) == 0) {
        const uint32_t t = ((w[i] >> m) ^ w[i + m]) & masks[k];
        w[i + m] ^= t;
        w[i] ^= t << m;
      }
    }
  }
}

// Both transposes stage a workgroup's 8192 words (256 32-word blocks) through LDS, so the
// word side is read / written as contiguous uint4 rows (a stride-33 layout: the per-block
// accesses are bank-conflict free), and thread t transposes block t in registers; the plane
// side is 32 coalesced rows of 256 words.
constexpr int kPlaneWords = 32 * kPlaneThreads;  // words per transpose workgroup
constexpr int kPlaneLds = 33 * kPlaneThreads;

CHOCO_DEV void words_to_lds(const uint32_t* __restrict__ words, int64_t Np, int64_t base, uint32_t* s) {
  const bool a16 = (reinterpret_cast<uintptr_t>(words) & 15u) == 0;  // (a message may be a view)
#pragma unroll
  for (int i = 0; i < kPlaneWords / 4 / kPlaneThreads; ++i) {
    const int wl = 4 * ((int)threadIdx.x + kPlaneThreads * i);
    uint32_t v[4];
    if (a16 && base + wl + 4 <= Np) {
      const uint4 t = *reinterpret_cast<const uint4*>(words + base + wl);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = base + wl + c < Np ? words[base + wl + c] : 0u;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) s[((wl + c) >> 5) * 33 + ((wl + c) & 31)] = v[c];
  }
}

struct PlaneSrc {
  const uint32_t* words[kMaxMsg];
  uint32_t* planes[kMaxMsg];
  double* acc;  // the receive's fp64 accumulators, zeroed here: their place in the workspace
  int nacc;     // moves with nseg, so an earlier call's planes may lie where they are now
};

// words (Np) -> planes [32][P] of message blockIdx.y
__global__ __launch_bounds__(kPlaneThreads) void sign_to_planes_kernel(PlaneSrc S, int64_t Np) {
  __shared__ uint32_t s[kPlaneLds];
  const int64_t P = plane_words(Np);
  const int64_t base = (int64_t)blockIdx.x * kPlaneWords;
  if (blockIdx.x == 0 && blockIdx.y == 0)
    for (int i = threadIdx.x; i < S.nacc; i += kPlaneThreads) S.acc[i] = 0.0;
  words_to_lds(S.words[blockIdx.y], Np, base, s);
  __syncthreads();
  uint32_t w[32];
#pragma unroll
  for (int b = 0; b < 32; ++b) w[b] = s[threadIdx.x * 33 + b];
  transpose32(w);
  const int64_t p = (int64_t)blockIdx.x * kPlaneThreads + threadIdx.x;
  uint32_t* __restrict__ planes = S.planes[blockIdx.y];
  if (p < P) {
#pragma unroll
    for (int r = 0; r < 32; ++r) planes[(int64_t)r * P + p] = w[r];
  }
}

// planes [32][P] -> words (Np)
__global__ __launch_bounds__(kPlaneThreads) void sign_from_planes_kernel(const uint32_t* __restrict__ planes,
                                                                         int64_t Np, uint32_t* __restrict__ words) {
  __shared__ uint32_t s[kPlaneLds];
  const int64_t P = plane_words(Np);
  const int64_t p = (int64_t)blockIdx.x * kPlaneThreads + threadIdx.x;
  uint32_t w[32];
#pragma unroll
  for (int r = 0; r < 32; ++r) w[r] = p < P ? planes[(int64_t)r * P + p] : 0u;
  transpose32(w);
#pragma unroll
  for (int b = 0; b < 32; ++b) s[threadIdx.x * 33 + b] = w[b];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kPlaneWords;
#pragma unroll
  for (int i = 0; i < kPlaneWords / 4 / kPlaneThreads; ++i) {
    const int wl = 4 * ((int)threadIdx.x + kPlaneThreads * i);
    uint32_t v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = s[((wl + c) >> 5) * 33 + ((wl + c) & 31)];
    if (base + wl + 4 <= Np) {
      *reinterpret_cast<uint4*>(words + base + wl) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (base + wl + c < Np) words[base + wl + c] = v[c];
    }
  }
}

struct PlaneMsgs {
  const uint32_t* planes[kMaxMsg];  // [32][P] per message
  const float* norms[kMaxMsg];
  float w[kMaxMsg];
  int self_slot;
};

constexpr int kRowSegLds = 64;  // a run spanning fewer segments sums them in LDS first
// Workgroup i <-> run i, row-major over the (32, N') view, i.e. the flat element order: row
// r = i / nrun, columns [J, J + 4096) with J = (i % nrun) * 4096.  Thread t takes the float4
// at columns J + 1024 c + 4 t (c = 0..3): every load and store instruction of a wave is one
// contiguous 1 KiB.  Its 4 message bits per float4 are a nibble of a plane word; the 4-bit
// output nibbles of 8 lanes are OR-ed into one plane word (3 xor shuffles).  Every element's
// chain is the unfused sequence's (sign_apply, gossip1, the pack's x_new - x_hat), so x,
// x_hat, memory and the words are bit-identical to sign_accumulate_kernel +
// sign_pack1_kernel<.., GS> (parallel_choco_v.py:548-558, optim/utils.py:67-72, :476-506).
// Same-box A/B at 345M, one message, step_sign --defer-receive (ms per step, two repeats):
// this 1.628 / 1.626; non-temporal loads and stores 1.767 / 1.758; a 2048-workgroup
// grid-stride loop 1.915 / 1.914 (non-temporal 1.994 / 2.036; 1024 workgroups 2.033 /
// 2.030); round 5's column-tile receive (32 rows of a 1024-word block per workgroup,
// non-temporal, 8 rows in flight) 1.983 / 1.984: removed, git history r05.
// SEG (per-tensor layouts, create_optimizer.py:15-24): element e decodes with its segment's
// norm / numel (seg_scale) and adds |d| to its segment's L1 sum.  The run's first and last
// segments are looked up (binary search) while its loads are in flight; a run inside one
// segment (nearly all of them) runs the flat code with that segment's scales, a run across
// boundaries walks them per element and sums per segment (in LDS when it spans fewer than
// kRowSegLds segments).
template <int NM, bool HS, bool SEG>
__global__ __launch_bounds__(kSignThreads) void sign_recv_rows_kernel(PlaneMsgs M, float* __restrict__ x,
                                                                      float* __restrict__ xh,
                                                                      float* __restrict__ mem, float gamma,
                                                                      int64_t n, int64_t Np,
                                                                      const int64_t* __restrict__ seg_off, int nseg,
                                                                      uint32_t* __restrict__ out_planes,
                                                                      float* __restrict__ l1_out,
                                                                      SignWs* __restrict__ ws) {
  __shared__ double s_red[kSignThreads / 64];
  __shared__ double s_sacc[SEG ? kRowSegLds : 1];
  __shared__ int s_seg[2];
  __shared__ unsigned int s_flag;
  double* __restrict__ acc = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + 256);
  double* __restrict__ rep = acc + (size_t)(blockIdx.x & (kRowRep - 1)) * (size_t)(SEG ? nseg : 1);
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int64_t P = plane_words(Np);
  const int64_t nrun = (Np + kRowRun - 1) / kRowRun;
  const uint32_t nib_sh = 4u * (uint32_t)(tid & 7);
  float sc[NM];
  if (!SEG) {
#pragma unroll
    for (int q = 0; q < NM; ++q) sc[q] = M.norms[q][0] / (float)n;
  }
  int s0 = 0, s1 = 0;  // SEG: the run's first and last segments
  bool uni = true;     // the run inside one segment (workgroup-uniform)
  const __amdgpu_buffer_rsrc_t rx = buf_rsrc(x, (uint32_t)(n * 4));
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc(xh, (uint32_t)(n * 4));
  const __amdgpu_buffer_rsrc_t rm = buf_rsrc(mem, (uint32_t)(n * 4));
  double p = 0.0;
  {
    const int64_t i = blockIdx.x;
    const int r = (int)(i / nrun);
    const int64_t J = (i - (int64_t)r * nrun) * kRowRun;
    const int64_t e0 = (int64_t)r * Np + J;  // the run's first element
    const bool full = J + kRowRun <= Np && e0 + kRowRun <= n;
    uint32_t bits[4][NM];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t pw = (J + 1024 * c) / 32 + (tid >> 3);
#pragma unroll
      for (int q = 0; q < NM; ++q) bits[c][q] = pw < P ? M.planes[q][(int64_t)r * P + pw] >> nib_sh : 0u;
    }
    float4 xv[4], hv[4], mv[4];
    if (full) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t off = (uint32_t)((e0 + 1024 * c + 4 * tid) * 4);
        xv[c] = ld_buf4<false>(rx, off);
        hv[c] = ld_buf4<false>(rh, off);
        mv[c] = ld_buf4<false>(rm, off);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float tx[4], th[4], tm[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t jj = J + 1024 * c + 4 * tid + k;
          const bool in = jj < Np && e0 - J + jj < n;
          tx[k] = in ? x[e0 - J + jj] : 0.f;
          th[k] = in ? xh[e0 - J + jj] : 0.f;
          tm[k] = in ? mem[e0 - J + jj] : 0.f;
        }
        xv[c] = make_float4(tx[0], tx[1], tx[2], tx[3]);
        hv[c] = make_float4(th[0], th[1], th[2], th[3]);
        mv[c] = make_float4(tm[0], tm[1], tm[2], tm[3]);
      }
    }
    int64_t s_beg = 0, s_end = n;  // SEG: the current segment's [start, end)
    if (SEG) {
      if (tid == 0) {
        const int64_t elast = std::min<int64_t>(e0 + std::min<int64_t>(kRowRun, Np - J), n) - 1;
        s_seg[0] = e0 < n ? seg_of(seg_off, nseg, e0) : 0;
        s_seg[1] = e0 < n ? seg_of(seg_off, nseg, elast) : 0;
      }
      if (tid < kRowSegLds) s_sacc[tid] = 0.0;
      __syncthreads();
      s0 = s_seg[0];
      s1 = s_seg[1];
      s_beg = seg_off[s0];
      s_end = seg_off[s0 + 1];
#pragma unroll
      for (int q = 0; q < NM; ++q) sc[q] = M.norms[q][s0] / (float)(s_end - s_beg);  // seg_scale
    }
    uni = !SEG || s0 == s1;
    int s = s0, run_s = -1;
    double run_p = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float a[4] = {xv[c].x, xv[c].y, xv[c].z, xv[c].w};
      float h[4] = {hv[c].x, hv[c].y, hv[c].z, hv[c].w};
      float m[4] = {mv[c].x, mv[c].y, mv[c].z, mv[c].w};
      uint32_t nib = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t jj = J + 1024 * c + 4 * tid + k;
        const bool in = full || (jj < Np && e0 - J + jj < n);
        if (SEG && !uni && in && e0 - J + jj >= s_end) {  // the next segment(s) (increasing e)
          do {
            ++s;
            s_beg = s_end;
            s_end = seg_off[s + 1];
          } while (e0 - J + jj >= s_end);
#pragma unroll
          for (int q = 0; q < NM; ++q) sc[q] = M.norms[q][s] / (float)(s_end - s_beg);
        }
#pragma unroll
        for (int q = 0; q < NM; ++q) {
          const float u = ((bits[c][q] >> k) & 1u) ? -sc[q] : sc[q];
          if (HS && q == M.self_slot) h[k] = h[k] + u;
          m[k] = fmaf(M.w[q], u, m[k]);
        }
        a[k] = gossip1(a[k], m[k], h[k], gamma);
        const float d = a[k] - h[k];
        nib |= (in && d < 0.f ? 1u : 0u) << k;
        if (in) {
          if (uni) {
            p += (double)fabsf(d);
          } else {
            if (s != run_s) {
              if (run_s >= 0 && run_p != 0.0) {
                if (s1 - s0 < kRowSegLds) atomicAdd(&s_sacc[run_s - s0], run_p);
                else unsafeAtomicAdd(&rep[run_s], run_p);
              }
              run_s = s;
              run_p = 0.0;
            }
            run_p += (double)fabsf(d);
          }
        }
      }
      xv[c] = make_float4(a[0], a[1], a[2], a[3]);
      hv[c] = make_float4(h[0], h[1], h[2], h[3]);
      mv[c] = make_float4(m[0], m[1], m[2], m[3]);
      uint32_t wd = nib << nib_sh;
      wd |= __shfl_xor(wd, 1);
      wd |= __shfl_xor(wd, 2);
      wd |= __shfl_xor(wd, 4);
      const int64_t pw = (J + 1024 * c) / 32 + (tid >> 3);
      if ((tid & 7) == 0 && pw < P) out_planes[(int64_t)r * P + pw] = wd;
    }
    if (full) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t off = (uint32_t)((e0 + 1024 * c + 4 * tid) * 4);
        st_buf4<false>(rx, off, xv[c]);
        st_buf4<false>(rm, off, mv[c]);
        if (HS) st_buf4<false>(rh, off, hv[c]);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float a[4] = {xv[c].x, xv[c].y, xv[c].z, xv[c].w};
        const float h[4] = {hv[c].x, hv[c].y, hv[c].z, hv[c].w};
        const float m[4] = {mv[c].x, mv[c].y, mv[c].z, mv[c].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t jj = J + 1024 * c + 4 * tid + k;
          if (jj < Np && e0 - J + jj < n) {
            x[e0 - J + jj] = a[k];
            mem[e0 - J + jj] = m[k];
            if (HS) xh[e0 - J + jj] = h[k];
          }
        }
      }
    }
    if (SEG && !uni) {  // workgroup-uniform
      if (run_s >= 0 && run_p != 0.0) {
        if (s1 - s0 < kRowSegLds) atomicAdd(&s_sacc[run_s - s0], run_p);
        else unsafeAtomicAdd(&rep[run_s], run_p);
      }
      __syncthreads();
      if (s1 - s0 < kRowSegLds && tid <= s1 - s0 && s_sacc[tid] != 0.0) unsafeAtomicAdd(&rep[s0 + tid], s_sacc[tid]);
    }
  }
  // the L1 norm: fp64 per thread, per workgroup, into one of kRowRep replicas
  if (uni) {  // workgroup-uniform
    p = wave_sum(p);
    if (lane == 0) s_red[wv] = p;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < kSignThreads / 64; ++i) t += s_red[i];
      if (t != 0.0) unsafeAtomicAdd(&rep[s0], t);
    }
  }
  if (last_block_ticket_atomics(&ws->ticket, gridDim.x, &s_flag)) {
    const int ns = SEG ? nseg : 1;
    for (int q = tid; q < ns; q += kSignThreads) {
      double t = 0.0;
      for (int i = 0; i < kRowRep; ++i) t += atomic_exchange_double(&acc[(size_t)i * ns + q], 0.0);
      l1_out[q] = (float)t;
    }
    if (tid == 0) __hip_atomic_store(&ws->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// DeepSqueezeSignCompressor.compress's local copy of the message
// (deep_squeeze.py:416-422): out = (norm_s * torch.sign(x)) / numel_s -- sign(0) = 0
// and NaN stays NaN, unlike the wire's decode (zero encodes as "+").  One float4
// per thread; the segment is found once per workgroup and walked per element only
// when the workgroup straddles a boundary.
constexpr int kLocalTile = kSignThreads * 4;
__global__ __launch_bounds__(kSignThreads) void sign_local_kernel(const float* __restrict__ x, int64_t n,
                                                                  const int64_t* __restrict__ seg_off, int nseg,
                                                                  const float* __restrict__ norms,
                                                                  float* __restrict__ out) {
  __shared__ int s_seg[2];
  const int64_t t0 = (int64_t)blockIdx.x * kLocalTile;
  const int64_t t1 = std::min<int64_t>(t0 + kLocalTile, n);
  if (threadIdx.x == 0) {
    s_seg[0] = nseg > 1 ? seg_of(seg_off, nseg, t0) : 0;
    s_seg[1] = nseg > 1 ? seg_of(seg_off, nseg, t1 - 1) : 0;
  }
  __syncthreads();
  const int sg0 = s_seg[0];
  const bool uniform = s_seg[1] == sg0;
  const int64_t e0 = t0 + 4 * (int64_t)threadIdx.x;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int64_t e = e0 + c;
    if (e >= n) break;
    int sgi = sg0;
    if (!uniform)
      while (sgi + 1 < nseg && seg_off[sgi + 1] <= e) ++sgi;
    const int64_t numel = nseg > 1 ? seg_off[sgi + 1] - seg_off[sgi] : n;
    const float v = x[e];
    const float sg = v > 0.f ? 1.0f : (v < 0.f ? -1.0f : (v == v ? 0.0f : v));  // torch.sign: NaN -> NaN
    out[e] = (norms[sgi] * sg) / (float)numel;
  }
}

}  // namespace choco

using namespace choco;

CHOCO_API int64_t choco_sign_words(int64_t n) { return (n + 31) / 32; }

CHOCO_API size_t choco_sign_workspace_size(int32_t nseg) {
  // the ticket block, then kRowRep replicas of the per-segment fp64 L1 sums (the one-pass
  // pack's per-tensor form spreads its workgroups' atomics over them)
  return 256 + align_up((size_t)kRowRep * (size_t)(nseg > 0 ? nseg : 1) * sizeof(double), 256);
}

// Same-box A/B, ResNet-50 layout (25.6M, 161 tensors; 780 workgroups), fused step: 4-row groups
// 112.5 / 112.3 us against 135.3 / 134.7 in 8-row groups (profiles/r05_ab_summary.txt item 16)
constexpr int kPackSmallGrid = 2048;
// Row split on those grids, same box (profiles/r05_ab_summary.txt item 18): flat 25.6M pack 35.4 ->
// 26.7 us, fused step 100.8 -> 85.3, ResNet-50's fused step 104 -> 95.6
constexpr int kPackRS = 2;
template <bool XH, bool NORM, bool GS>
static void launch_pack(bool one, unsigned grid, hipStream_t st, const float* x, const float* xhat, int64_t n,
                        int64_t Np, const int64_t* seg_off, int32_t nseg, uint32_t* pk, float* l1, SignWs* w,
                        Gossip gs, int64_t blk0, int finish) {
  // a grid of under kPackSmallGrid workgroups (the ~25M-element buffers of one model) splits each
  // column block's rows over two waves, and runs the fused step in groups of 4 rows: more
  // waves per CU instead of more rows in flight per wave
  const bool small = grid < (unsigned)kPackSmallGrid;
  if (one && small && GS && NORM && nseg > 1)
    CHOCO_KLAUNCH((sign_pack1_kernel<XH, NORM, GS, NORM, 4, kPackRS>), dim3(grid), dim3(kPackRS * kSignThreads), 0, st, x, xhat,
                  n, Np, pk, l1, w, gs, blk0, finish, seg_off, nseg);
  else if (one && small && GS)
    CHOCO_KLAUNCH((sign_pack1_kernel<XH, NORM, GS, false, 4, kPackRS>), dim3(grid), dim3(kPackRS * kSignThreads), 0, st, x, xhat,
                  n, Np, pk, l1, w, gs, blk0, finish, seg_off, nseg);
  else if (one && small && NORM && nseg > 1)
    CHOCO_KLAUNCH((sign_pack1_kernel<XH, NORM, GS, NORM, 0, kPackRS>), dim3(grid), dim3(kPackRS * kSignThreads), 0, st, x, xhat,
                  n, Np, pk, l1, w, gs, blk0, finish, seg_off, nseg);
  else if (one && small)
    CHOCO_KLAUNCH((sign_pack1_kernel<XH, NORM, GS, false, 0, kPackRS>), dim3(grid), dim3(kPackRS * kSignThreads), 0, st, x, xhat,
                  n, Np, pk, l1, w, gs, blk0, finish, seg_off, nseg);
  else if (one && NORM && nseg > 1)
    CHOCO_KLAUNCH((sign_pack1_kernel<XH, NORM, GS, NORM>), dim3(grid), dim3(kSignThreads), 0, st, x, xhat, n, Np, pk,
                  l1, w, gs, blk0, finish, seg_off, nseg);
  else if (one)
    CHOCO_KLAUNCH((sign_pack1_kernel<XH, NORM, GS, false>), dim3(grid), dim3(kSignThreads), 0, st, x, xhat, n, Np, pk,
                  l1, w, gs, blk0, finish, seg_off, nseg);
  else
    CHOCO_KLAUNCH((sign_pack_kernel<XH, NORM, GS>), dim3(grid), dim3(kSignThreads), 0, st, x, xhat, n, Np, seg_off,
                  nseg, pk, l1, w, gs, blk0, finish);
}

// Packs words [w0, w1) (the whole buffer: 0, N').  The per-segment L1 sums of a range
// stay in the workspace's fp64 accumulators; the `finish` launch (issued last) rounds
// them to fp32 into l1_norms and zeroes the accumulators.
static int sign_compress(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                         int32_t* packed, float* l1_norms, void* ws, size_t ws_bytes, hipStream_t st, Gossip gs,
                         int64_t w0 = 0, int64_t w1 = -1, bool finish = true) {
  CHOCO_REQUIRE(x && packed, "null pointer argument");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(aligned16(x) && (!xhat || aligned16(xhat)) && aligned16(packed),
                "x/xhat/packed must be 16-byte aligned");
  CHOCO_REQUIRE(!gs.mem || (xhat && aligned16(gs.mem)), "the gossip step needs x_hat and a 16-byte aligned memory");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  const int64_t Np = choco_sign_words(n);
  if (w1 < 0) w1 = Np;
  CHOCO_REQUIRE(w0 >= 0 && w0 < w1 && w1 <= Np && w0 % kSignCols == 0 && (w1 % kSignCols == 0 || w1 == Np),
                "word range must satisfy 0 <= w0 < w1 <= N', w0 a multiple of 1024, w1 one too or N'");
  const unsigned grid = (unsigned)((w1 - w0 + kSignCols - 1) / kSignCols);
  const int64_t blk0 = w0 / kSignCols;
  uint32_t* pk = reinterpret_cast<uint32_t*>(packed);
  SignWs* w = static_cast<SignWs*>(ws);
  if (l1_norms) {
    CHOCO_REQUIRE(ws && ws_bytes >= choco_sign_workspace_size(nseg), "sign workspace too small");
  }
  const bool one = n < (int64_t(1) << 30);  // the one-pass column kernel: buffer offsets, n * 4 < 2^32 bytes
  const int fin = finish ? 1 : 0;
  profile_begin("sign_pack", st);
  if (gs.mem) {
    if (l1_norms) launch_pack<true, true, true>(one, grid, st, x, xhat, n, Np, seg_off, nseg, pk, l1_norms, w, gs, blk0, fin);
    else launch_pack<true, false, true>(one, grid, st, x, xhat, n, Np, seg_off, nseg, pk, l1_norms, w, gs, blk0, fin);
  } else if (xhat) {
    if (l1_norms) launch_pack<true, true, false>(one, grid, st, x, xhat, n, Np, seg_off, nseg, pk, l1_norms, w, gs, blk0, fin);
    else launch_pack<true, false, false>(one, grid, st, x, xhat, n, Np, seg_off, nseg, pk, l1_norms, w, gs, blk0, fin);
  } else {
    if (l1_norms) launch_pack<false, true, false>(one, grid, st, x, xhat, n, Np, seg_off, nseg, pk, l1_norms, w, gs, blk0, fin);
    else launch_pack<false, false, false>(one, grid, st, x, xhat, n, Np, seg_off, nseg, pk, l1_norms, w, gs, blk0, fin);
  }
  profile_end("sign_pack", st);
  CHOCO_LAUNCHED("sign_pack_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_sign_compress(const float* x, const float* xhat, int64_t n, const int64_t* seg_off,
                                  int32_t nseg, int32_t* packed, float* l1_norms, void* ws, size_t ws_bytes,
                                  void* stream) {
  return sign_compress(x, xhat, n, seg_off, nseg, packed, l1_norms, ws, ws_bytes, as_stream(stream),
                       Gossip{nullptr, 0.f});
}

CHOCO_API int choco_gossip_sign_compress(float* x, const float* memory, const float* xhat, float gamma, int64_t n,
                                         const int64_t* seg_off, int32_t nseg, int32_t* packed, float* l1_norms,
                                         void* ws, size_t ws_bytes, void* stream) {
  CHOCO_REQUIRE(memory != nullptr && xhat != nullptr, "the gossip step needs memory and x_hat");
  return sign_compress(x, xhat, n, seg_off, nseg, packed, l1_norms, ws, ws_bytes, as_stream(stream),
                       Gossip{memory, gamma});
}

CHOCO_API int choco_sign_compress_range(const float* x, const float* xhat, int64_t n, const int64_t* seg_off,
                                        int32_t nseg, int64_t w0, int64_t w1, int32_t finish, int32_t* packed,
                                        float* l1_norms, void* ws, size_t ws_bytes, void* stream) {
  return sign_compress(x, xhat, n, seg_off, nseg, packed, l1_norms, ws, ws_bytes, as_stream(stream),
                       Gossip{nullptr, 0.f}, w0, w1, finish != 0);
}

CHOCO_API int choco_gossip_sign_compress_range(float* x, const float* memory, const float* xhat, float gamma,
                                               int64_t n, const int64_t* seg_off, int32_t nseg, int64_t w0, int64_t w1,
                                               int32_t finish, int32_t* packed, float* l1_norms, void* ws,
                                               size_t ws_bytes, void* stream) {
  CHOCO_REQUIRE(memory != nullptr && xhat != nullptr, "the gossip step needs memory and x_hat");
  return sign_compress(x, xhat, n, seg_off, nseg, packed, l1_norms, ws, ws_bytes, as_stream(stream),
                       Gossip{memory, gamma}, w0, w1, finish != 0);
}

CHOCO_API int choco_sign_unpack(const int32_t* packed, int64_t n, float* out, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed && out && n > 0 && n < (int64_t)INT32_MAX, "bad arguments");
  CHOCO_REQUIRE(aligned16(out), "out must be 16-byte aligned");
  const int64_t Np = choco_sign_words(n);
  const unsigned grid = (unsigned)((Np + kSignCols - 1) / kSignCols);
  CHOCO_KLAUNCH(sign_unpack_kernel, dim3(grid), dim3(kSignThreads), 0, st,
                     reinterpret_cast<const uint32_t*>(packed), n, Np, out);
  CHOCO_LAUNCHED("sign_unpack_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_sign_decompress_accumulate(const int32_t* const* packed_list, const float* const* norms_list,
                                               const float* weights, int32_t nmsg, int32_t self_slot, int64_t n,
                                               const int64_t* seg_off, int32_t nseg, float* xhat_self,
                                               float* memory, void* ws, size_t ws_bytes, void* stream) {
  (void)ws;
  (void)ws_bytes;
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed_list && norms_list && weights && memory, "null pointer argument");
  CHOCO_REQUIRE(nmsg >= 1 && nmsg <= kMaxMsg, "nmsg must be in [1, %d]", kMaxMsg);
  CHOCO_REQUIRE(self_slot >= -1 && self_slot < nmsg, "bad self_slot");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(memory) && (!xhat_self || aligned16(xhat_self)), "buffers must be 16-byte aligned");
  SignMsgs M{};
  for (int q = 0; q < nmsg; ++q) {
    CHOCO_REQUIRE(packed_list[q] && norms_list[q], "null message pointer");
    M.packed[q] = reinterpret_cast<const uint32_t*>(packed_list[q]);
    M.norms[q] = norms_list[q];
    M.w[q] = weights[q];
  }
  M.nmsg = nmsg;
  M.self_slot = self_slot;
  const int64_t Np = choco_sign_words(n);
  const unsigned grid = sign_acc_grid(Np);
  profile_begin("sign_accumulate", st);
#define CHOCO_SIGN_ACC_L(NM, HS, NT)                                                                          \
  CHOCO_KLAUNCH((sign_accumulate_kernel<NM, HS, NT>), dim3(grid), dim3(kSignThreads), 0, st, M, n, Np, seg_off, \
                nseg, xhat_self, memory)
#define CHOCO_SIGN_ACC(NM)                                       \
  case NM:                                                       \
    if (self_slot >= 0 && xhat_self) {                           \
      if (nt)                                                    \
        CHOCO_SIGN_ACC_L(NM, true, true);                        \
      else                                                       \
        CHOCO_SIGN_ACC_L(NM, true, false);                       \
    } else {                                                     \
      if (nt)                                                    \
        CHOCO_SIGN_ACC_L(NM, false, true);                       \
      else                                                       \
        CHOCO_SIGN_ACC_L(NM, false, false);                      \
    }                                                            \
    break;
  const bool nt = n >= kSaccNtMin;
  switch (nmsg) {
    CHOCO_SIGN_ACC(1)
    CHOCO_SIGN_ACC(2)
    CHOCO_SIGN_ACC(3)
    CHOCO_SIGN_ACC(4)
    CHOCO_SIGN_ACC(5)
    CHOCO_SIGN_ACC(6)
    CHOCO_SIGN_ACC(7)
    CHOCO_SIGN_ACC(8)
  }
#undef CHOCO_SIGN_ACC
#undef CHOCO_SIGN_ACC_L
  profile_end("sign_accumulate", st);
  CHOCO_LAUNCHED("sign_accumulate_kernel");
  return CHOCO_OK;
}

// ticket block, kRowRep replicas of the per-segment fp64 L1 sums, then the bit planes of the
// messages and of the output (sign_recv_rows_kernel)
static size_t sign_recv_acc_bytes(int32_t nseg) {
  return 256 + align_up((size_t)kRowRep * (size_t)(nseg > 0 ? nseg : 1) * sizeof(double), 256);
}

CHOCO_API size_t choco_sign_recv_workspace_size(int64_t n, int32_t nseg, int32_t nmsg) {
  if (n >= (int64_t(1) << 30)) return choco_sign_workspace_size(nseg);  // the two-kernel form
  const int64_t Np = choco_sign_words(n > 0 ? n : 1);
  const size_t pb = align_up((size_t)32 * (size_t)plane_words(Np) * 4, 256);
  return sign_recv_acc_bytes(nseg) + (size_t)((nmsg > 0 ? nmsg : 1) + 1) * pb;
}

CHOCO_API int choco_sign_recv_gossip_compress(const int32_t* const* packed_list, const float* const* norms_list,
                                              const float* weights, int32_t nmsg, int32_t self_slot, float* x,
                                              float* memory, float* xhat, float gamma, int64_t n,
                                              const int64_t* seg_off, int32_t nseg, int32_t* packed,
                                              float* l1_norms, void* ws, size_t ws_bytes, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed_list && norms_list && weights && x && memory && xhat && packed && l1_norms,
                "null pointer argument");
  CHOCO_REQUIRE(nmsg >= 1 && nmsg <= kMaxMsg, "nmsg must be in [1, %d]", kMaxMsg);
  CHOCO_REQUIRE(self_slot >= -1 && self_slot < nmsg, "bad self_slot");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(x) && aligned16(memory) && aligned16(xhat) && aligned16(packed),
                "x/memory/xhat/packed must be 16-byte aligned");
  CHOCO_REQUIRE(ws && ws_bytes >= choco_sign_workspace_size(nseg), "sign workspace too small");
  {
    // the output words must not overlap any message's words (the row-run pass reads the
    // message planes while it writes the output): a range test, not a start-pointer test
    const int64_t nw = choco_sign_words(n);
    for (int q = 0; q < nmsg; ++q) {
      CHOCO_REQUIRE(packed_list[q] && norms_list[q], "null message pointer");
      CHOCO_REQUIRE(packed + nw <= packed_list[q] || packed_list[q] + nw <= packed,
                    "the output words alias (overlap) message %d's words", q);
    }
  }
  if (n >= (int64_t(1) << 30)) {  // past 32-bit buffer offsets: the receive, then the fused consensus step + pack
    // (the pack's accumulators may hold an earlier row-run call's planes: zero them)
    CHOCO_HIP(hipMemsetAsync(static_cast<char*>(ws) + 256, 0, (size_t)nseg * sizeof(double), st));
    int rc = choco_sign_decompress_accumulate(packed_list, norms_list, weights, nmsg, self_slot, n, seg_off, nseg,
                                              self_slot >= 0 ? xhat : nullptr, memory, nullptr, 0, stream);
    if (rc != CHOCO_OK) return rc;
    return choco_gossip_sign_compress(x, memory, xhat, gamma, n, seg_off, nseg, packed, l1_norms, ws, ws_bytes,
                                      stream);
  }
  const int64_t Np = choco_sign_words(n);
  uint32_t* pk = reinterpret_cast<uint32_t*>(packed);
  SignWs* w = static_cast<SignWs*>(ws);
  CHOCO_REQUIRE(ws_bytes >= choco_sign_recv_workspace_size(n, nseg, nmsg),
                "sign receive workspace too small: need choco_sign_recv_workspace_size(n, nseg, nmsg) bytes");
  const int64_t P = plane_words(Np);
  const size_t pb = align_up((size_t)32 * (size_t)P * 4, 256);
  char* wb = static_cast<char*>(ws) + sign_recv_acc_bytes(nseg);
  const unsigned gp = (unsigned)((P + kPlaneThreads - 1) / kPlaneThreads);
  PlaneMsgs M{};
  PlaneSrc S{};
  S.acc = reinterpret_cast<double*>(static_cast<char*>(ws) + 256);
  S.nacc = kRowRep * nseg;
  for (int q = 0; q < nmsg; ++q) {
    uint32_t* pl = reinterpret_cast<uint32_t*>(wb + (size_t)q * pb);
    S.words[q] = reinterpret_cast<const uint32_t*>(packed_list[q]);
    S.planes[q] = pl;
    M.planes[q] = pl;
    M.norms[q] = norms_list[q];
    M.w[q] = weights[q];
  }
  profile_begin("sign_planes", st);
  CHOCO_KLAUNCH(sign_to_planes_kernel, dim3(gp, (unsigned)nmsg), dim3(kPlaneThreads), 0, st, S, Np);
  profile_end("sign_planes", st);
  CHOCO_LAUNCHED("sign_to_planes_kernel");
  M.self_slot = self_slot;
  uint32_t* outp = reinterpret_cast<uint32_t*>(wb + (size_t)nmsg * pb);
  const unsigned grid = (unsigned)(32 * ((Np + kRowRun - 1) / kRowRun));  // one workgroup per run
  profile_begin("sign_recv_pack", st);
#define CHOCO_SRR_LAUNCH(NM, HS, SEG)                                                                    \
  CHOCO_KLAUNCH((sign_recv_rows_kernel<NM, HS, SEG>), dim3(grid), dim3(kSignThreads), 0, st, M, x, xhat, memory, \
                gamma, n, Np, seg_off, nseg, outp, l1_norms, w)
#define CHOCO_SRR_CASE(NM)                         \
  case NM:                                         \
    if (nseg > 1) {                                \
      if (self_slot >= 0)                          \
        CHOCO_SRR_LAUNCH(NM, true, true);          \
      else                                         \
        CHOCO_SRR_LAUNCH(NM, false, true);         \
    } else {                                       \
      if (self_slot >= 0)                          \
        CHOCO_SRR_LAUNCH(NM, true, false);         \
      else                                         \
        CHOCO_SRR_LAUNCH(NM, false, false);        \
    }                                              \
    break;
  switch (nmsg) {
    CHOCO_SRR_CASE(1)
    CHOCO_SRR_CASE(2)
    CHOCO_SRR_CASE(3)
    CHOCO_SRR_CASE(4)
    CHOCO_SRR_CASE(5)
    CHOCO_SRR_CASE(6)
    CHOCO_SRR_CASE(7)
    CHOCO_SRR_CASE(8)
  }
#undef CHOCO_SRR_CASE
#undef CHOCO_SRR_LAUNCH
  profile_end("sign_recv_pack", st);
  CHOCO_LAUNCHED("sign_recv_rows_kernel");
  profile_begin("sign_planes", st);
  CHOCO_KLAUNCH(sign_from_planes_kernel, dim3(gp), dim3(kPlaneThreads), 0, st, outp, Np, pk);
  profile_end("sign_planes", st);
  CHOCO_LAUNCHED("sign_from_planes_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_sign_decompress_axpy(const int32_t* const* packed_list, const float* const* norms_list,
                                         const float* weights, int32_t nmsg, int64_t n, const int64_t* seg_off,
                                         int32_t nseg, int32_t two_roundings, float* target, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed_list && norms_list && weights && target, "null pointer argument");
  CHOCO_REQUIRE(nmsg >= 1 && nmsg <= kMaxMsg, "nmsg must be in [1, %d]", kMaxMsg);
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(target), "target must be 16-byte aligned");
  SignMsgs M{};
  for (int q = 0; q < nmsg; ++q) {
    CHOCO_REQUIRE(packed_list[q] && norms_list[q], "null message pointer");
    M.packed[q] = reinterpret_cast<const uint32_t*>(packed_list[q]);
    M.norms[q] = norms_list[q];
    M.w[q] = weights[q];
  }
  M.nmsg = nmsg;
  M.self_slot = -1;
  M.mode = two_roundings ? 1 : 0;
  const int64_t Np = choco_sign_words(n);
  const unsigned grid = sign_acc_grid(Np);
  profile_begin("sign_accumulate", st);
#define CHOCO_SIGN_AXPY(NM)                                                                                 \
  case NM:                                                                                                  \
    CHOCO_KLAUNCH((sign_accumulate_kernel<NM, false>), dim3(grid), dim3(kSignThreads), 0, st, M, n, Np, seg_off, \
                  nseg, nullptr, target);                                                                   \
    break;
  switch (nmsg) {
    CHOCO_SIGN_AXPY(1)
    CHOCO_SIGN_AXPY(2)
    CHOCO_SIGN_AXPY(3)
    CHOCO_SIGN_AXPY(4)
    CHOCO_SIGN_AXPY(5)
    CHOCO_SIGN_AXPY(6)
    CHOCO_SIGN_AXPY(7)
    CHOCO_SIGN_AXPY(8)
  }
#undef CHOCO_SIGN_AXPY
  profile_end("sign_accumulate", st);
  CHOCO_LAUNCHED("sign_accumulate_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_sign_local_decode(const float* x, int64_t n, const int64_t* seg_off, int32_t nseg,
                                      const float* norms, float* out, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(x && norms && out, "null pointer argument");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  const unsigned grid = (unsigned)((n + kLocalTile - 1) / kLocalTile);
  CHOCO_KLAUNCH(sign_local_kernel, dim3(grid), dim3(kSignThreads), 0, st, x, n, seg_off, nseg, norms, out);
  CHOCO_LAUNCHED("sign_local_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_sign_decompress_extrapolate(const int32_t* packed, const float* norms, int64_t n,
                                                const int64_t* seg_off, int32_t nseg, float a, float b, float* target,
                                                void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed && norms && target, "null pointer argument");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(target), "target must be 16-byte aligned");
  SignMsgs M{};
  M.packed[0] = reinterpret_cast<const uint32_t*>(packed);
  M.norms[0] = norms;
  M.w[0] = 1.0f;
  M.nmsg = 1;
  M.self_slot = -1;
  M.mode = 2;
  M.a = a;
  M.b = b;
  const int64_t Np = choco_sign_words(n);
  const unsigned grid = sign_acc_grid(Np);
  profile_begin("sign_accumulate", st);
  CHOCO_KLAUNCH((sign_accumulate_kernel<1, false>), dim3(grid), dim3(kSignThreads), 0, st, M, n, Np, seg_off, nseg,
                nullptr, target);
  profile_end("sign_accumulate", st);
  CHOCO_LAUNCHED("sign_accumulate_kernel");
  return CHOCO_OK;
}
