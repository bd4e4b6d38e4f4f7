// Batched per-tensor (segmented) top-k on MI355X.
//
// Replaces the per-parameter-tensor loop of CHOCOSparsificationCompressor.compress
// (reference dl_code/pcode/optim/parallel_choco_v.py:229-260), which calls
// SparsificationCompressor.get_top_k (sparsification.py:18-31) once per tensor of
// the layout that create_optimizer.py:15-24 defines (one parameter per group: 65
// tensors for ResNet-20, 161 for ResNet-50).  (Per-segment random-k: randk.hip.)
//
// Per segment s the answer is the exact selection of the flat path (topk.hip):
//   T_s = k_s-th largest key, out = {key > T_s} U {the lowest-index ties at T_s},
//   (value, GLOBAL index) in ascending index order, segments concatenated.
//
// Every segment of up to kSegMaxTiles tiles (16M elements) is cut into tiles of
// kSegTile = 16384 elements; ALL tiles of ALL such segments run in the same
// launches.  Two sequences, chosen per call on the host (a workspace's first call
// is cold, later calls warm; include/choco_codec.h "warm start"):
//
// COLD (five launches, two reads of the input):
//   S1 seg_hist     : 2048-bin histogram of key >> 20 -> hist1[s].
//   S2 seg_collect  : coarse bin b1 of the k_s-th key from hist1[s]; candidates
//                     key >= b1 << 20 compacted in index order into the tile's
//                     slots; keys in bin b1 -> hist2[s] (bits 19..9).
//   S3a seg_fine    : bin b2 of the k_s-th key from hist2[s]; bits 8..0 of the
//                     tile's candidates in bin (b1, b2) -> hist3[s].
//   S3b seg_count   : T_s and the tie quota from hist3[s]; the tile's (#> T_s,
//                     #== T_s); tile 0 of the segment writes the NEXT call's window.
//   S4 seg_emit     : offset and tie share from the segment's earlier tiles, then
//                     the ordered compaction of the tile's candidates.
// WARM (three launches, ONE read): each segment carries a window [lo_s, lo_s +
// 2048 << sh_s) from the previous call (around that call's T_s, margins at
// k_s (1 +- m_s) keys), so
//   W2 seg_collect  : candidates key >= lo_s, compacted; their window bin
//                     min((key - lo_s) >> sh_s, 2047) -> hist2[s]  (no S1);
//   S3w seg_bin     : the k_s-th key's window bin b2 from hist2[s]; the tile's
//                     count above b2 and its (few) keys IN b2, kept per tile;
//   S4w seg_emit_w  : T_s from the kept keys, offsets, ordered compaction; one
//                     workgroup per segment writes the next call's window.
//                     A segment whose T_s is not inside its window (fewer than
//                     k_s candidates, or T_s in the clamped top bin) is flagged
//                     in S3w; in S4w its tile workgroups select it exactly
//                     together (wide.h: five per-tile passes through a ticketed
//                     queue, the segment's own WideCtrl), and the workgroup that
//                     learns T re-centres its window; k_s >= len_s segments take
//                     every element.
// Every histogram is reset by the first tile of its segment in the launch after
// its last reader.  Segments over 16M elements take the flat pipeline (topk.hip),
// each in its own workspace (its own warm window).
#include "choco_common.h"
#include "select.h"
#include "wide.h"

#include <math.h>
#include <algorithm>
#include <mutex>
#include <unordered_map>

namespace choco {

// Diagnostic phase stamps (tools/seg_stamps.py; never in the product build): slot t
// (tile t) {dispatched, loads issued}, slot 2048 + t {flags, scanned, stored, exact}.
#ifndef CHOCO_STAMPS
#define CHOCO_STAMPS 0
#endif
#if CHOCO_STAMPS
constexpr int kSgStampSlots = 4096;
__device__ unsigned long long g_sg_stamps[kSgStampSlots][4];
#define SGSTAMP(slot, j)                                                                       \
  do {                                                                                        \
    if (threadIdx.x == 0 && (slot) < kSgStampSlots) g_sg_stamps[(slot)][(j)] = wall_clock64(); \
  } while (0)
#else
#define SGSTAMP(slot, j) \
  do {                   \
  } while (0)
#endif
constexpr int kSegThreads = 1024;  // threads of the tile kernels S1 / S2
// rows of float4 per thread.  Same-box A/B at ResNet-50 (compress us, three passes):
// 4 rows (16384-element tiles) 40.0-40.4, 5 rows 40.0-40.4, 6 rows 42.2-42.6 (spills).
constexpr int kSegRows = 4;
constexpr int kSegTile = kSegRows * 4 * kSegThreads;  // elements per tile
constexpr int kSegMaxTiles = 1024;                    // tiles per batched segment (S3: one per thread)
constexpr int64_t kSegBatchMax = (int64_t)kSegTile * kSegMaxTiles;
constexpr int kRow = 8;                               // plan row width (int64)
constexpr int kH = 2048;                              // histogram bins (S1, S2)
constexpr uint32_t kWinShMax = 9;                     // warm window bin <= 2^9 keys (hist3: 512 bins)
static_assert(kSegRows * 4 * kSegThreads == kSegTile, "tile geometry");

// plan (host + device copies, int64):
//   rows[nseg][8] = {off, len, k, out_off, t0, ntile, 0, 0}; row 0 also carries
//   [6] = total tiles, [7] = batched segments;
//   then tile -> segment map [total tiles]; then batched segment ids [batched];
//   then the random-k tile table (randk.hip).
struct SegRow {
  int64_t off, len, k, out_off, t0, ntile;
};
CHOCO_DEV SegRow seg_row(const int64_t* __restrict__ plan, int s) {
  const int64_t* p = plan + (int64_t)kRow * s;
  return SegRow{p[0], p[1], p[2], p[3], p[4], p[5]};
}

// A segment's warm window: candidates key >= lo, bins of 2^sh keys; and the drift words
// (the exact k-th key of the call that wrote it, and its move from the call before:
// window_drift extrapolates the next window by them).
struct SegWin {
  uint32_t lo, sh, valid, pad;
  uint32_t tprev, dprev, cand, trust;  // cand: the drift window_drift proposed when this window was
                                       // written; trust: the calls in a row it beat the static key
};
CHOCO_DEV SegWin seg_win(uint32_t lo, uint32_t sh, uint32_t T, const SegWin& old, uint32_t cand = 0u,
                         uint32_t trust = 0u) {
  return SegWin{lo, sh, 1u, 0u, T, (old.valid && old.tprev) ? T - old.tprev : 0u, cand, trust};
}

// info[8 s + i]: 0 b1 (cold), 1 rank inside b1 (cold), 2 T, 3 bin of the k-th key
// (S3a), 4 rank inside that bin, 5 ties at T to take, 6 mode (0 select, 1 window
// missed: exact fallback in S4, 2 take every element)
struct SegWs {
  uint32_t *hist1, *hist2, *hist3, *info, *tilecnt, *tcount;
  float* cval;
  uint32_t* cidx;
  SegWin* win;
  uint32_t* misses;     // the workspace's CHOCO_TOPK_FALLBACKS_OFFSET counter
  uint32_t* miss_flag;  // pinned host word of the cold backoff (nullable)
  unsigned long long* shadow;       // device counter of cold calls' window checks (misses << 32 | checks)
  unsigned long long* shadow_host;  // its pinned host copy, written once per cold call by S4 (nullable)
  uint2* blist;         // warm: per tile, its keys in the k-th key's window bin ({key, count} x kTileList)
  WideCtrl* wide;       // per segment: the queue of its shared exact select (S4w, a missed window)
  uint32_t* wcnt;       // per tile: 2 words of that select (phase 2 -> 3 -> 4)
  uint32_t* whist;      // per tile: its 512-bin last-digit histogram (phase 2 -> phase 3)
  uint32_t* status;     // the workspace's sticky status word (CHOCO_TOPK_STATUS_OFFSET)
  uint32_t* host_status;  // its pinned host mirror (choco_topk_host_status)
};

struct SegLayout {
  size_t off_h1, off_h2, off_h3, off_info, off_cnt, off_out, off_cval, off_cidx, off_win, off_blist, off_wide,
      off_wcnt, off_whist, total;
};
constexpr int kTileList = 4;  // warm: a tile's distinct keys in the k-th key's window bin kept for S4w

constexpr size_t kSegShadowOffset = 64;  // in the header: the cold calls' 64-bit window-check counter
static SegLayout seg_layout(int nseg, int64_t ntile) {
  SegLayout L{};
  size_t o = 256;  // [0, 256): the sticky status word (CHOCO_TOPK_STATUS_OFFSET) of the whole call, the
                   // miss counter (CHOCO_TOPK_FALLBACKS_OFFSET), the shadow counter (kSegShadowOffset)
  L.off_h1 = o;   o += align_up((size_t)nseg * kH * 4, 256);
  L.off_h2 = o;   o += align_up((size_t)nseg * kH * 4, 256);
  L.off_h3 = o;   o += align_up((size_t)nseg * 512 * 4, 256);
  L.off_info = o; o += align_up((size_t)nseg * 8 * 4, 256);
  L.off_cnt = o;  o += align_up((size_t)ntile * 4, 256);
  L.off_out = o;  o += align_up((size_t)ntile * 8, 256);
  L.off_cval = o; o += align_up((size_t)ntile * kSegTile * 4, 256);
  L.off_cidx = o; o += align_up((size_t)ntile * kSegTile * 4, 256);
  L.off_win = o;  o += align_up((size_t)nseg * sizeof(SegWin), 256);
  L.off_blist = o; o += align_up((size_t)ntile * kTileList * sizeof(uint2), 256);
  L.off_wide = o; o += (size_t)nseg * kWideBytes;  // (zero between calls: the last workgroup out resets it)
  L.off_wcnt = o; o += align_up((size_t)ntile * 8, 256);
  L.off_whist = o; o += align_up((size_t)ntile * 512 * 4, 256);
  L.total = o;
  return L;
}

// This tile: its segment, the segment's row, its first element and length.
struct TileCtx {
  int s;
  SegRow R;
  int64_t j, start, slot;  // tile number inside the segment, first element, candidate slot base
  int tl;
};
CHOCO_DEV TileCtx tile_ctx(const int64_t* __restrict__ plan, int nseg, int64_t b) {
  TileCtx c;
  c.s = (int)plan[(int64_t)kRow * nseg + b];
  c.R = seg_row(plan, c.s);
  c.j = b - c.R.t0;
  c.start = c.R.off + c.j * kSegTile;
  c.slot = b * kSegTile;
  c.tl = (int)min((int64_t)kSegTile, c.R.len - c.j * kSegTile);
  return c;
}

// The same from the plan's per-tile rows (a copy of the tile's segment row + the segment
// id, 8 int64 per tile): ONE scalar round trip instead of two dependent ones
CHOCO_DEV TileCtx tile_ctx_rows(const int64_t* __restrict__ trows, int64_t b) {
  const int64_t* r = trows + 8 * b;
  TileCtx c;
  c.R = SegRow{r[0], r[1], r[2], r[3], r[4], r[5]};
  c.s = (int)r[6];
  c.j = b - c.R.t0;
  c.start = c.R.off + c.j * kSegTile;
  c.slot = b * kSegTile;
  c.tl = (int)min((int64_t)kSegTile, c.R.len - c.j * kSegTile);
  return c;
}

// The tile's values: row r, thread t <-> elements r * 4096 + 4t .. +3 (dword-
// aligned buffer loads: x + start needs only 4-byte alignment; past the tile
// the loads return zeros and the elements are masked by `valid`).
template <bool XH, bool NT = false>
CHOCO_DEV void tile_load(const float* __restrict__ x, const float* __restrict__ xh, const TileCtx& c,
                         float (&v)[kSegRows][4]) {
  const __amdgpu_buffer_rsrc_t rx = buf_rsrc(x + c.start, (uint32_t)c.tl * 4u);
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc((XH ? xh : x) + c.start, (uint32_t)c.tl * 4u);
  float4 a[kSegRows], h[kSegRows];
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) a[r] = ld_buf4<NT>(rx, (uint32_t)(r * 4 * kSegThreads + 4 * threadIdx.x) * 4u);
  if (XH) {
#pragma unroll
    for (int r = 0; r < kSegRows; ++r) h[r] = ld_buf4<NT>(rh, (uint32_t)(r * 4 * kSegThreads + 4 * threadIdx.x) * 4u);
  }
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    v[r][0] = a[r].x; v[r][1] = a[r].y; v[r][2] = a[r].z; v[r][3] = a[r].w;
    if (XH) { v[r][0] -= h[r].x; v[r][1] -= h[r].y; v[r][2] -= h[r].z; v[r][3] -= h[r].w; }
  }
}

// The first read with the fused gossip step: x, memory and xh of the tile in
// flight together, x_new = x + gamma (memory - xh) stored back (the buffer
// resources end at the tile: nothing past it is read or written), v = x_new - xh.
// NT: the cold sequence re-reads x_new and xh in S2 (keep them in the Infinity
// Cache); the warm one reads them once.
template <bool NT>
CHOCO_DEV void tile_load_gossip(const float* __restrict__ x, const float* __restrict__ xh, const Gossip& gs,
                                const TileCtx& c, float (&v)[kSegRows][4]) {
  const __amdgpu_buffer_rsrc_t rx = buf_rsrc(x + c.start, (uint32_t)c.tl * 4u);
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc(xh + c.start, (uint32_t)c.tl * 4u);
  const __amdgpu_buffer_rsrc_t rm = buf_rsrc(gs.mem + c.start, (uint32_t)c.tl * 4u);
  float4 a[kSegRows], h[kSegRows], m[kSegRows];
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    const uint32_t off = (uint32_t)(r * 4 * kSegThreads + 4 * threadIdx.x) * 4u;
    a[r] = ld_buf4<true>(rx, off);
    m[r] = ld_buf4<true>(rm, off);
    h[r] = ld_buf4<NT>(rh, off);
  }
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    const uint32_t off = (uint32_t)(r * 4 * kSegThreads + 4 * threadIdx.x) * 4u;
    const float4 xn = gossip4(a[r], m[r], h[r], gs.gamma);
    st_buf4<NT>(rx, off, xn);
    v[r][0] = xn.x - h[r].x; v[r][1] = xn.y - h[r].y; v[r][2] = xn.z - h[r].z; v[r][3] = xn.w - h[r].w;
  }
}

CHOCO_DEV int tile_elem(int r, int q) { return r * 4 * kSegThreads + 4 * (int)threadIdx.x + q; }

// Over hist[kH] in LDS or global memory (ascending key order), the bin holding
// the rank-th largest entry and the rank inside it -> out[0], out[1].  kBpt
// consecutive bins per thread of the kSegThreads workgroup (hv[b] = bin kBpt*tid + b);
// ends with a barrier.
constexpr int kBpt = kH / kSegThreads;
static_assert(kBpt * kSegThreads == kH, "whole bins per thread");
CHOCO_DEV void block_find_rank(const uint32_t (&hv)[kBpt], uint32_t rank, uint32_t* scratch, uint32_t* out) {
  const int tid = threadIdx.x;
  uint32_t local = 0;
#pragma unroll
  for (int b = 0; b < kBpt; ++b) local += hv[b];
  uint32_t total;
  const uint32_t pre = block_excl_scan(local, scratch, &total);
  uint32_t above = total - pre - local;  // entries in bins above mine
  if (above < rank && rank <= above + local) {
#pragma unroll
    for (int b = kBpt - 1; b >= 0; --b) {
      if (above < rank && rank <= above + hv[b]) { out[0] = kBpt * tid + b; out[1] = rank - above; }
      above += hv[b];
    }
  }
  __syncthreads();
}
CHOCO_DEV void load_bins(const uint32_t* h, uint32_t (&hv)[kBpt]) {
#pragma unroll
  for (int b = 0; b < kBpt; ++b) hv[b] = h[kBpt * threadIdx.x + b];
}

// ---------------------------------------------------------------- S1: coarse histogram (cold)
template <bool XH, bool GS = false>
__global__ __launch_bounds__(kSegThreads) void seg_hist_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ xh,
                                                               const int64_t* __restrict__ trows, int nseg,
                                                               uint32_t* __restrict__ hist1, Gossip gs) {
  static_assert(!GS || XH, "the gossip step needs x_hat");
  // one LDS histogram (per-wave or per-lane copies measured no faster, r04)
  __shared__ uint32_t h[kH];
  const TileCtx c = tile_ctx_rows(trows, blockIdx.x);
  float v[kSegRows][4] = {};
  if (GS) tile_load_gossip<false>(x, xh, gs, c, v);
  else if (c.R.ntile == 1) return;  // a single-tile segment is selected in S2 (no histogram)
  else tile_load<XH>(x, xh, c, v);
  if (c.R.ntile == 1) return;  // (GS: its consensus step is applied; S2 selects it)
  for (int i = threadIdx.x; i < kH; i += kSegThreads) h[i] = 0u;
  __syncthreads();
  uint32_t* __restrict__ hw = h;
#pragma unroll
  for (int r = 0; r < kSegRows; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tile_elem(r, q);
      if (e < c.tl) atomicAdd(&hw[fkey(v[r][q]) >> 20], 1u);
    }
  __syncthreads();
  uint32_t* __restrict__ g = hist1 + (int64_t)c.s * kH;
  for (int i = threadIdx.x; i < kH; i += kSegThreads) {
    const uint32_t t = h[i];
    if (t) atomicAdd(&g[i], t);
  }
}

// ---------------------------------------------------------------- single-tile segments
// A segment of at most one tile (the many small tensors of a CNN layout: BN scales and
// biases, small convs) is selected EXACTLY by the workgroup that holds it, in S2, from
// its registers: a three-digit radix select (bits 30..20, 19..9, 8..0) in the LDS
// histogram, then the ordered compaction (ties at T by index).  No window, no S3/S4
// work: their k-th key moves by many ranks from call to call, so a warm window would
// miss often.  Exclusive ranks of the set bits of `bits` in row-major order (row r,
// wave, lane, element q) -> base[r] (+ popc of the lane's lower bits); two barriers.
// Wave 0: exclusive scan of the NC (row, wave) counts in rc[0, NC) (row-major), the
// total -> rc[NC]; NC <= 128 (two counts per lane above 64).
template <int NC>
CHOCO_DEV void wave0_scan_counts(uint32_t* rc) {
  static_assert(NC <= 128, "two counts per lane at most");
  const int lane = lane_id();
  if constexpr (NC <= 64) {
    const uint32_t cv = lane < NC ? rc[lane] : 0u;
    const uint32_t inc = wave_incl_scan(cv);
    if (lane < NC) rc[lane] = inc - cv;
    if (lane == 63) rc[NC] = inc;
  } else {
    const int i0 = 2 * lane, i1 = 2 * lane + 1;
    const uint32_t c0 = i0 < NC ? rc[i0] : 0u, c1 = i1 < NC ? rc[i1] : 0u;
    const uint32_t inc = wave_incl_scan(c0 + c1);
    const uint32_t ex = inc - (c0 + c1);
    if (i0 < NC) rc[i0] = ex;
    if (i1 < NC) rc[i1] = ex + c0;
    if (lane == 63) rc[NC] = inc;
  }
}

CHOCO_DEV void tile_ranks(const uint32_t (&bits)[kSegRows], uint32_t (&base)[kSegRows], uint32_t* rc_cnt,
                          uint32_t* total) {
  constexpr int kW = kSegThreads / 64;
  const int lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    const uint32_t cnt = (uint32_t)__popc(bits[r]);
    const uint32_t inc = wave_incl_scan(cnt);
    base[r] = inc - cnt;
    if (lane == 63) rc_cnt[r * kW + w] = inc;
  }
  __syncthreads();
  if (w == 0) wave0_scan_counts<kSegRows * kW>(rc_cnt);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) base[r] += rc_cnt[r * kW + w];
  *total = rc_cnt[kSegRows * kW];
  __syncthreads();  // rc_cnt is reused
}

CHOCO_DEV void seg_exact_tile(const float (&v)[kSegRows][4], const TileCtx& c, uint32_t* h, uint32_t* scratch,
                              uint32_t* bc, uint32_t* rc_cnt, float* __restrict__ out_val,
                              int32_t* __restrict__ out_idx) {
  const int tid = threadIdx.x;
  const uint32_t k = (uint32_t)c.R.k;
  uint32_t key[kSegRows][4];
#pragma unroll
  for (int r = 0; r < kSegRows; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) key[r][q] = fkey(v[r][q]);
  const bool all = k >= (uint32_t)c.tl;
  uint32_t prefix = 0, maskhi = 0, krem = k;
  if (!all) {
    const int shs[3] = {20, 9, 0};
    const uint32_t dms[3] = {2047u, 2047u, 511u};
#pragma unroll
    for (int rd = 0; rd < 3; ++rd) {
      for (int i = tid; i < kH; i += kSegThreads) h[i] = 0u;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kSegRows; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (tile_elem(r, q) < c.tl && (key[r][q] & maskhi) == prefix)
            atomicAdd(&h[(key[r][q] >> shs[rd]) & dms[rd]], 1u);
      __syncthreads();
      uint32_t hv[kBpt];
      load_bins(h, hv);
      block_find_rank(hv, krem, scratch, bc);
      prefix |= bc[0] << shs[rd];
      maskhi |= dms[rd] << shs[rd];
      krem = bc[1];
      __syncthreads();  // bc is rewritten by the next round
    }
  }
  const uint32_t T = prefix, r_take = krem;  // the k-th key and the ties at it to take
  uint32_t eqb[kSegRows], selb[kSegRows], base[kSegRows], tot;
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    eqb[r] = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      eqb[r] |= (!all && tile_elem(r, q) < c.tl && key[r][q] == T) ? (1u << q) : 0u;
  }
  tile_ranks(eqb, base, rc_cnt, &tot);  // tie ranks in index order
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    selb[r] = 0u;
    uint32_t tr = base[r];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool in = tile_elem(r, q) < c.tl;
      const bool eq = (eqb[r] >> q) & 1u;
      selb[r] |= (in && (all || key[r][q] > T || (eq && tr < r_take))) ? (1u << q) : 0u;
      tr += eq ? 1u : 0u;
    }
  }
  tile_ranks(selb, base, rc_cnt, &tot);
  float* __restrict__ ov = out_val + c.R.out_off;
  int32_t* __restrict__ oi = out_idx + c.R.out_off;
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    uint32_t pos = base[r];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if ((selb[r] >> q) & 1u) {
        if (pos < k) {  // (bounded)
          ov[pos] = v[r][q];
          oi[pos] = (int32_t)(c.start + tile_elem(r, q));
        }
        ++pos;
      }
    }
  }
}

// ---------------------------------------------------------------- S2 / W2: candidates
// Cold: the floor is the coarse bin b1 of the k_s-th key (from hist1), keys of bin b1
// feed hist2 by bits 19..9.  Warm: the floor is the window's lo, every candidate
// feeds hist2 by its window bin min((key - lo) >> sh, 2047); GS: the fused gossip
// step happens here (the one read).
// (8 waves per SIMD: <= 64 VGPRs; 2 x 1024 threads per CU.  Fewer workgroups per CU
// measured ~10 us slower at ResNet-50; a looping collect with the next tile's loads in
// flight (one workgroup per CU, 128 VGPRs) 40 against 29.5 us: removed, git history r04.)
// W2's one read of the delta uses non-temporal loads; W2 / S2 take the single-tile
// segments' tiles first (the plan's dispatch records).
constexpr int kSegWpe = kSegThreads == 1024 ? 8 : 6;  // waves per SIMD (VGPR budget 512 / WPE)
template <bool XH, bool WARM, bool GS = false>
__global__ __launch_bounds__(kSegThreads, kSegWpe) void seg_collect_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, const int64_t* __restrict__ plan, int nseg,
    const uint32_t* __restrict__ hist1, uint32_t* __restrict__ hist2, uint32_t* __restrict__ info,
    uint32_t* __restrict__ tilecnt, float* __restrict__ cval, uint32_t* __restrict__ cidx,
    const SegWin* __restrict__ win, Gossip gs, float* __restrict__ out_val, int32_t* __restrict__ out_idx,
    int64_t ntile, const int64_t* __restrict__ order) {
  static_assert(!GS || (XH && WARM), "the gossip step is fused into S2 on the warm path only (S1 on the cold)");
  __shared__ uint32_t h2[kH];
  __shared__ uint32_t scratch[40];
  __shared__ uint32_t bc[4];
  __shared__ uint32_t rc_cnt[kSegRows * (kSegThreads / 64) + 1];
  const int tid = threadIdx.x;
  // `wpre`: the segment's window, read before the tile's loads were issued (warm)
  auto process = [&](const float (&v)[kSegRows][4], const TileCtx& c, int64_t tb, const SegWin& wpre) {
  if (c.R.ntile == 1) {  // workgroup-uniform: the whole segment is here
    seg_exact_tile(v, c, h2, scratch, bc, rc_cnt, out_val, out_idx);
    SGSTAMP(2048 + tb, 3);
    return;
  }
  for (int i = tid; i < kH; i += kSegThreads) h2[i] = 0u;
  uint32_t floor_key, b1 = 0, sh = 0;
  if (WARM) {
    const SegWin w = wpre;
    // no window (never expected after a cold call): no candidates -> S3a flags the miss
    floor_key = w.valid ? w.lo : 0xFFFFFFFFu;
    sh = w.valid ? min(w.sh, kWinShMax) : 0u;
    if (c.R.k >= c.R.len) floor_key = 0u;  // every element
    __syncthreads();
  } else {
    const uint32_t* __restrict__ g1 = hist1 + (int64_t)c.s * kH;
    uint32_t hv[kBpt];
    load_bins(g1, hv);
    block_find_rank(hv, (uint32_t)c.R.k, scratch, bc);
    b1 = bc[0];
    if (c.j == 0 && tid == 0) {
      info[8 * c.s + 0] = b1;
      info[8 * c.s + 1] = bc[1];
    }
    floor_key = b1 << 20;
  }
  // candidate flags of all rows, then ONE scan of the (row, wave) counts places
  // them in index order (row-major: row r, wave w, lane, element)
  constexpr int kW = kSegThreads / 64;
  const int lane = lane_id(), w = tid >> 6;
  uint32_t cm[kSegRows];    // candidate bits of this lane's 4 elements per row
  uint32_t lpre[kSegRows];  // exclusive count of candidates of lower lanes (same row, wave)
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    cm[r] = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tile_elem(r, q);
      const uint32_t key = fkey(v[r][q]);
      const bool cand = e < c.tl && key >= floor_key;
      cm[r] |= cand ? (1u << q) : 0u;
      if (WARM) {
        if (cand) atomicAdd(&h2[min((key - floor_key) >> sh, (uint32_t)(kH - 1))], 1u);
      } else {
        if (cand && (key >> 20) == b1) atomicAdd(&h2[(key >> 9) & (kH - 1)], 1u);
      }
    }
    const uint32_t cnt = (uint32_t)__popc(cm[r]);
    const uint32_t inc = wave_incl_scan(cnt);
    lpre[r] = inc - cnt;
    if (lane == 63) rc_cnt[r * kW + w] = inc;
  }
  SGSTAMP(2048 + tb, 0);
  __syncthreads();
  if (w == 0) wave0_scan_counts<kSegRows * kW>(rc_cnt);  // the (row, wave) counts, row-major
  __syncthreads();
  SGSTAMP(2048 + tb, 1);
#pragma unroll
  for (int r = 0; r < kSegRows; ++r) {
    uint32_t pos = rc_cnt[r * kW + w] + lpre[r];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (cm[r] & (1u << q)) {
        const int e = tile_elem(r, q);
        cval[c.slot + pos] = v[r][q];
        cidx[c.slot + pos] = (uint32_t)(c.start + e);
        ++pos;
      }
    }
  }
  uint32_t* __restrict__ g2 = hist2 + (int64_t)c.s * kH;
  for (int i = tid; i < kH; i += kSegThreads)
    if (h2[i]) atomicAdd(&g2[i], h2[i]);
  if (tid == 0) tilecnt[tb] = rc_cnt[kSegRows * kW];
  SGSTAMP(2048 + tb, 2);
  };
  {
    // the tile this workgroup takes; with the dispatch-order records its loads need only
    // the record (the segment's row is read while they fly)
    int64_t ta;
    TileCtx c;
    if (order) {
      const int64_t* rec = order + 4 * (int64_t)blockIdx.x;
      ta = rec[0];
      c.s = (int)rec[1];
      c.start = rec[2];
      c.tl = (int)rec[3];
      c.slot = ta * kSegTile;
    } else {
      ta = blockIdx.x;
      c = tile_ctx(plan, nseg, ta);
    }
    SGSTAMP(ta, 0);
    float v[kSegRows][4] = {};
    if (GS) tile_load_gossip<true>(x, xh, gs, c, v);  // in flight while the floor is found
    else tile_load<XH, WARM>(x, xh, c, v);  // warm: the only read of the call (non-temporal)
    if (order) {
      c.R = seg_row(plan, c.s);
      c.j = ta - c.R.t0;
    }
    SegWin wpre{};
    if (WARM) wpre = win[c.s];
    SGSTAMP(ta, 1);
    process(v, c, ta, wpre);
  }
}

// ---------------------------------------------------------------- S3: exact T per segment
// Tile-parallel (every tile of every segment in one launch, like S1/S2): a
// per-segment select in ONE workgroup was latency-bound on the largest segment
// (a 2.4M-element conv weight: ~50K candidates walked by 16 waves, a dependent
// load per step).  Both kernels use 256-thread workgroups; every tile derives
// its segment's bins from the complete global histograms of the previous launch.
//   S3a seg_fine : bin of the k-th key from hist2[s]; the low bits of this tile's
//                  candidates in that bin -> hist3[s].
//   S3b seg_count: T_s from hist3[s]; this tile's (#key > T_s, #key == T_s);
//                  tile 0: the next call's window.
// S4 then places each tile from the counts of the tiles before it.
constexpr int kS3Threads = 256;
constexpr int kH3 = 512;  // bits 8..0 (cold) / the low sh <= 9 bits of a window bin (warm)
// kSegMissed: T below the window (fewer candidates than k) or no window: the shared exact
// select reads the segment; kSegMissedHigh: T above the window's top bin -- every key >= T is
// a candidate, so the shared select reads the tiles' candidate lists only.
enum SegMode { kSegSelect = 0, kSegMissed = 1, kSegAll = 2, kSegMissedHigh = 3 };

// Over hist[nb] in global memory (ascending key order), the bin holding the
// rank-th largest entry and the rank inside it -> out[0], out[1], and the
// histogram total -> out[2]; PER bins per thread of a kS3Threads workgroup.
// Ends with a barrier.
template <int PER>
CHOCO_DEV void block_find_rank_g(const uint32_t* __restrict__ hist, uint32_t rank, uint32_t* scratch, uint32_t* out) {
  const int tid = threadIdx.x;
  uint32_t hv[PER];
  uint32_t local = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    hv[j] = hist[tid * PER + j];
    local += hv[j];
  }
  uint32_t total;
  const uint32_t pre = block_excl_scan(local, scratch, &total);
  const uint32_t above = total - pre - local;  // entries in bins above mine
  if (tid == 0) out[2] = total;
  if (above < rank && rank <= above + local) {
    uint32_t acc = above;
#pragma unroll
    for (int j = PER - 1; j >= 0; --j) {
      if (acc < rank && rank <= acc + hv[j]) { out[0] = (uint32_t)(tid * PER + j); out[1] = rank - acc; }
      acc += hv[j];
    }
  }
  __syncthreads();
}

// (cold calls; warm calls take S3w + S4w below)
__global__ __launch_bounds__(kS3Threads) void seg_fine_kernel(
    const int64_t* __restrict__ trows, int nseg, uint32_t* __restrict__ hist1, const uint32_t* __restrict__ hist2,
    uint32_t* __restrict__ hist3, uint32_t* __restrict__ info, const uint32_t* __restrict__ tilecnt,
    const float* __restrict__ cval) {
  __shared__ uint32_t h3[kH3];
  __shared__ uint32_t scratch[40];
  __shared__ uint32_t bc[4];
  const TileCtx c = tile_ctx_rows(trows, blockIdx.x);
  if (c.R.ntile == 1) return;  // selected in S2
  const int tid = threadIdx.x;
  const uint32_t cnt = tilecnt[blockIdx.x];
  for (int i = tid; i < kH3; i += kS3Threads) h3[i] = 0u;
  if (tid < 4) bc[tid] = 0u;
  __syncthreads();
  const uint32_t b1 = info[8 * c.s + 0], rank = info[8 * c.s + 1];
  block_find_rank_g<kH / kS3Threads>(hist2 + (int64_t)c.s * kH, rank, scratch, bc);
  const uint32_t b2 = bc[0];
  if (c.j == 0 && tid == 0) {
    info[8 * c.s + 3] = b2;
    info[8 * c.s + 4] = bc[1];  // rank of the k-th key inside that bin
  }
  if (c.j == 0) {  // every tile of the segment read hist1 in S2: reset it for the next call
    uint32_t* __restrict__ g1 = hist1 + (int64_t)c.s * kH;
    for (int i = tid; i < kH; i += kS3Threads) g1[i] = 0u;
  }
  const uint32_t fmask = (uint32_t)(kH3 - 1);
  constexpr int U = 4;
  for (uint32_t i0 = 0; i0 < cnt; i0 += U * kS3Threads) {  // workgroup-uniform
    uint32_t key[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kS3Threads + tid;
      key[u] = i < cnt ? fkey(cval[c.slot + i]) : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kS3Threads + tid;
      const bool in = key[u] >> 9 == ((b1 << 11) | b2);
      const uint32_t f = key[u] & fmask;
      if (i < cnt && in) atomicAdd(&h3[f], 1u);
    }
  }
  __syncthreads();
  uint32_t* __restrict__ g3 = hist3 + (int64_t)c.s * kH3;
  for (int i = tid; i < kH3; i += kS3Threads)
    if (h3[i]) atomicAdd(&g3[i], h3[i]);
}

// Next call's window of one segment (S3b, tile 0; every thread of the workgroup):
// over hist[kH] of bins of 2^shb keys from `base`, with `above` keys above the
// range, the keys at count levels k + delta and k - delta (delta = 0.03 k +
// 4 sqrt(k) + 8: the k-th key of a small segment moves by many ranks from one
// call to the next), bin-rounded outward; a window wider than 2048 << kWinShMax
// keys is centred on T instead.
constexpr int kWinPer = kH / kS3Threads;  // hist bins per thread of seg_next_window
CHOCO_DEV void seg_next_window_v(const uint32_t (&hv)[kWinPer], uint32_t base, uint32_t shb, uint32_t above,
                                 uint32_t k, uint32_t T, const SegWin& old, SegWin* __restrict__ out,
                                 uint32_t* scratch);
CHOCO_DEV void seg_next_window(const uint32_t* __restrict__ hist, uint32_t base, uint32_t shb, uint32_t above,
                               uint32_t k, uint32_t T, const SegWin& old, SegWin* __restrict__ out,
                               uint32_t* scratch) {
  uint32_t hv[kWinPer];
#pragma unroll
  for (int j = 0; j < kWinPer; ++j) hv[j] = hist[threadIdx.x * kWinPer + j];
  seg_next_window_v(hv, base, shb, above, k, T, old, out, scratch);
}
// the same over bins already in registers (hv[j] = bin tid * kWinPer + j).  `old` is the
// window the call used or the previous call prepared (its drift words; window_drift).
CHOCO_DEV void seg_next_window_v(const uint32_t (&hv)[kWinPer], uint32_t base, uint32_t shb, uint32_t above,
                                 uint32_t k, uint32_t T, const SegWin& old, SegWin* __restrict__ out,
                                 uint32_t* scratch) {
  constexpr int PER = kWinPer;
  const int tid = threadIdx.x;
  const uint64_t delta = (uint64_t)(0.03 * (double)k + 4.0 * sqrt((double)k)) + 8u;
  const uint64_t lo_t = (uint64_t)k + delta, hi_t = (uint64_t)k > delta ? (uint64_t)k - delta : 0u;
  uint32_t local = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) local += hv[j];
  uint32_t total;
  const uint32_t pre = block_excl_scan(local, scratch, &total);
  // C(j) = #keys >= base + (j << shb) = above + total - (keys in bins below j)
  uint32_t nlo = 0, nhi = 0, below = pre;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint64_t C = (uint64_t)above + total - below;
    nlo += C >= lo_t ? 1u : 0u;
    nhi += C > hi_t ? 1u : 0u;
    below += hv[j];
  }
  uint32_t tlo, thi;
  block_excl_scan2(nlo, nhi, scratch, &tlo, &thi, &nlo, &nhi);  // (totals in nlo, nhi)
  if (tid == 0) {
    uint64_t x_lo = (uint64_t)base + ((uint64_t)(nlo ? nlo - 1u : 0u) << shb);
    uint64_t x_hi = (uint64_t)base + ((uint64_t)nhi << shb);
    // trusted drift: applied only when the previous candidate predicted this T better than
    // the key it started from (a steady drift; on a stationary, noisy k-th key the
    // extrapolated noise only widens the misses)
    const int32_t cand = window_drift(T, old.tprev, old.dprev, old.valid != 0u);
    const uint32_t trust = drift_trusted(T, old.tprev, old.cand, old.valid != 0u) ? min(old.trust + 1u, 15u) : 0u;
    const int32_t drift = trust >= kDriftTrust ? cand : 0;
    if (drift != 0) {  // both edges follow the k-th key's steady drift
      const int64_t lo2 = (int64_t)x_lo + drift, hi2 = (int64_t)x_hi + drift;
      x_lo = (uint64_t)(lo2 > 0 ? lo2 : 0);
      x_hi = (uint64_t)(hi2 > (int64_t)x_lo + 1 ? (hi2 < (1ll << 31) ? hi2 : (1ll << 31)) : (int64_t)x_lo + 1);
    }
    uint32_t sh = 0;
    while (((uint64_t)kH << sh) < x_hi - x_lo && sh < kWinShMax) ++sh;
    if (((uint64_t)kH << sh) < x_hi - x_lo) {  // too wide for the finest bins: centre on T
      sh = kWinShMax;
      x_lo = T > (1u << 18) ? (uint64_t)T - (1u << 18) : 0u;
    }
    *out = seg_win((uint32_t)x_lo, sh, T, old, (uint32_t)cand, trust);
  }
}

// (cold calls)
// shadow: on a cold call, tile 0 of each segment also checks whether the window the
// previous call prepared (still in win[s]) would have held this call's T_s, and adds
// (miss << 32) | 1 to a 64-bit device counter; S4 copies it to pinned host memory once per
// call (a system-scope atomic per segment took S3b 5 -> 49 us); the host ends a cold run
// once two calls' worth of checks came without a miss.
__global__ __launch_bounds__(kS3Threads) void seg_count_kernel(
    const int64_t* __restrict__ trows, int nseg, uint32_t* __restrict__ hist2, const uint32_t* __restrict__ hist3,
    uint32_t* __restrict__ info, const uint32_t* __restrict__ tilecnt, const float* __restrict__ cval,
    uint32_t* __restrict__ tcount, SegWin* __restrict__ win, unsigned long long* __restrict__ shadow) {
  __shared__ uint32_t scratch[40];
  __shared__ uint32_t bc[4];
  const TileCtx c = tile_ctx_rows(trows, blockIdx.x);
  if (c.R.ntile == 1) return;  // selected in S2
  const int tid = threadIdx.x;
  const uint32_t cnt = tilecnt[blockIdx.x];
  const uint32_t b2 = info[8 * c.s + 3], kc = info[8 * c.s + 4], b1 = info[8 * c.s + 0];
  block_find_rank_g<kH3 / kS3Threads>(hist3 + (int64_t)c.s * kH3, kc, scratch, bc);
  const uint32_t T = (b1 << 20) | (b2 << 9) | bc[0];
  if (c.j == 0) {
    if (tid == 0) {
      info[8 * c.s + 2] = T;
      info[8 * c.s + 5] = bc[1];  // ties at T to take (>= 1)
    }
    // the next call's window, from this call's hist2 (bits 19..9 inside b1, with the keys
    // of the bins above b1); hist2 was read by every tile in S3a
    uint32_t* __restrict__ g2 = hist2 + (int64_t)c.s * kH;
    const SegWin old = win[c.s];  // the window the previous call prepared (read before it is replaced)
    __syncthreads();
    if (tid == 0 && shadow) {
      const bool hit = old.valid && old.lo <= T && (uint64_t)T < (uint64_t)old.lo + ((uint64_t)(kH - 1) << min(old.sh, kWinShMax));
      __hip_atomic_fetch_add(shadow, (hit ? 0ull : (1ull << 32)) | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    seg_next_window(g2, b1 << 20, 9u, (uint32_t)c.R.k - info[8 * c.s + 1], (uint32_t)c.R.k, T, old, &win[c.s],
                    scratch);
    __syncthreads();
    for (int i = tid; i < kH; i += kS3Threads) g2[i] = 0u;
  }
  uint32_t gt = 0, eq = 0;
  {
    constexpr int U = 4;
    for (uint32_t i0 = 0; i0 < cnt; i0 += U * kS3Threads) {  // workgroup-uniform
      uint32_t key[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * kS3Threads + tid;
        key[u] = i < cnt ? fkey(cval[c.slot + i]) : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * kS3Threads + tid;
        gt += (i < cnt && key[u] > T) ? 1u : 0u;
        eq += (i < cnt && key[u] == T) ? 1u : 0u;
      }
    }
  }
  uint32_t g0, e0, gtot, etot;
  block_excl_scan2(gt, eq, scratch, &g0, &e0, &gtot, &etot);
  if (tid == 0) {
    tcount[2 * blockIdx.x] = gtot;
    tcount[2 * blockIdx.x + 1] = etot;
  }
}

// ---------------------------------------------------------------- S3w: warm bin + list
// Warm calls: the k-th key's window bin b2 and the rank inside it from the complete
// hist2[s] (as S3a), then this tile's candidates ABOVE bin b2 counted and those IN bin b2
// kept: the window's 2048 bins hold ~1-2 keys each near the k-th one, so a tile holds
// none or one or two.  S4w takes T from those kept keys directly: no fine-histogram pass
// over every tile's candidates (S3a) and no per-tile count against T (S3b) -- one launch
// less.  Every load of the tile (its count, the window, its 8 bins of hist2, its first
// 1024 candidates) goes out in ONE round trip; the kept keys go to the tile's own
// kTileList slots as {key, 1} (no atomics) -- or, when the tile has more keys in bin b2
// than slots (ties), as {key, count} of its distinct keys from an LDS histogram of the
// bin's low sh bits -- and tcount[b] = {#above b2, #slots used}.  Tile 0 records the
// window it used (info 0/1: S4w re-writes win[s] for the next call) and b2 / rank / mode
// (info 3/4/6).  A tile with more than kTileList DISTINCT keys in bin b2 sends its
// segment to S4w's exact select (not counted as a window miss).
// Kept over the round-4 sequence S3a + S3b + S4 (same-box A/B, profiles/r05_ab_summary.txt).
template <int PER>
CHOCO_DEV void block_find_rank_v(const uint32_t (&hv)[PER], uint32_t rank, uint32_t* scratch, uint32_t* out) {
  // block_find_rank_g over bins already in registers (hv[j] = bin tid * PER + j)
  const int tid = threadIdx.x;
  uint32_t local = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) local += hv[j];
  uint32_t total;
  const uint32_t pre = block_excl_scan(local, scratch, &total);
  const uint32_t above = total - pre - local;
  if (tid == 0) out[2] = total;
  if (above < rank && rank <= above + local) {
    uint32_t acc = above;
#pragma unroll
    for (int j = PER - 1; j >= 0; --j) {
      if (acc < rank && rank <= acc + hv[j]) { out[0] = (uint32_t)(tid * PER + j); out[1] = rank - acc; }
      acc += hv[j];
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kS3Threads) void seg_bin_kernel(
    const int64_t* __restrict__ trows, const uint32_t* __restrict__ hist2, uint32_t* __restrict__ info,
    const uint32_t* __restrict__ tilecnt, const float* __restrict__ cval, const SegWin* __restrict__ win,
    uint32_t* __restrict__ tcount, uint2* __restrict__ blist) {
  __shared__ uint32_t scratch[40];
  __shared__ uint32_t bc[4];
  __shared__ uint32_t h3[kH3];
  const TileCtx c = tile_ctx_rows(trows, blockIdx.x);
  if (c.R.ntile == 1) return;  // selected in S2
  const int tid = threadIdx.x;
  constexpr int PER = kH / kS3Threads;
  constexpr int U = 4;
  static_assert(PER == 8, "two 16-byte loads of hist2 per thread");
  // ---- every load of the tile in one round trip
  const uint32_t cnt = tilecnt[blockIdx.x];
  const SegWin w = win[c.s];
  uint32_t hv[PER];
  {
    const uint4* h4 = reinterpret_cast<const uint4*>(hist2 + (int64_t)c.s * kH + tid * PER);
    const uint4 a = h4[0], b = h4[1];
    hv[0] = a.x; hv[1] = a.y; hv[2] = a.z; hv[3] = a.w; hv[4] = b.x; hv[5] = b.y; hv[6] = b.z; hv[7] = b.w;
  }
  float cv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) cv[u] = cval[c.slot + u * kS3Threads + tid];  // (inside the tile's slots; masked below)
  if (tid < 4) bc[tid] = 0u;
  __syncthreads();
  const uint32_t lo = w.lo, sh = min(w.sh, kWinShMax);
  const uint32_t rank = (uint32_t)c.R.k;
  block_find_rank_v<PER>(hv, rank, scratch, bc);
  const uint32_t b2 = bc[0];
  uint32_t mode = kSegSelect;
  if (c.R.k >= c.R.len) mode = kSegAll;
  else if (!w.valid || bc[2] < rank) mode = kSegMissed;  // T below the window (or none)
  else if (b2 == (uint32_t)(kH - 1)) mode = kSegMissedHigh;  // T in the window's clamped top bin
  if (c.j == 0 && tid == 0) {
    info[8 * c.s + 0] = lo;
    info[8 * c.s + 1] = sh;
    info[8 * c.s + 3] = b2;
    info[8 * c.s + 4] = bc[1];  // rank of the k-th key inside bin b2
    info[8 * c.s + 6] = mode;
  }
  uint32_t gt = 0, nin = 0;
  if (mode == kSegSelect) {  // workgroup-uniform
    uint2* __restrict__ L = blist + (int64_t)blockIdx.x * kTileList;
    for (uint32_t i0 = 0; i0 < cnt; i0 += U * kS3Threads) {  // workgroup-uniform
      uint32_t key[U], inb = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * kS3Threads + tid;
        key[u] = i0 == 0 ? fkey(cv[u]) : (i < cnt ? fkey(cval[c.slot + i]) : 0u);
        const uint32_t bin = min((key[u] - lo) >> sh, (uint32_t)(kH - 1));  // (every candidate has key >= lo)
        gt += (i < cnt && bin > b2) ? 1u : 0u;
        inb |= (i < cnt && bin == b2) ? (1u << u) : 0u;
      }
      uint32_t nb;
      uint32_t pos = nin + block_excl_scan((uint32_t)__popc(inb), scratch, &nb);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if ((inb >> u) & 1u) {
          if (pos < (uint32_t)kTileList) L[pos] = make_uint2(key[u], 1u);
          ++pos;
        }
      }
      nin += nb;
    }
    if (nin > (uint32_t)kTileList) {  // workgroup-uniform (ties): {key, count} of the distinct keys
      const uint32_t fmask = (1u << sh) - 1u;
      for (int i = tid; i < kH3; i += kS3Threads) h3[i] = 0u;
      __syncthreads();
      for (uint32_t i = tid; i < cnt; i += kS3Threads) {
        const uint32_t key = fkey(cval[c.slot + i]);
        if (min((key - lo) >> sh, (uint32_t)(kH - 1)) == b2) atomicAdd(&h3[(key - lo) & fmask], 1u);
      }
      __syncthreads();
      constexpr int P3 = kH3 / kS3Threads;
      uint32_t hc[P3], nz = 0;
#pragma unroll
      for (int q = 0; q < P3; ++q) {
        hc[q] = h3[tid * P3 + q];
        nz += hc[q] ? 1u : 0u;
      }
      uint32_t nd;
      uint32_t pos = block_excl_scan(nz, scratch, &nd);
#pragma unroll
      for (int q = 0; q < P3; ++q) {
        if (hc[q]) {
          if (pos < (uint32_t)kTileList) L[pos] = make_uint2(lo + (b2 << sh) + (uint32_t)(tid * P3 + q), hc[q]);
          ++pos;
        }
      }
      nin = nd;  // > kTileList: more distinct keys than slots (S4w selects the segment exactly)
    }
  } else if (mode == kSegAll) {
    gt = tid == 0 ? cnt : 0u;
  }
  uint32_t gtot;
  block_excl_scan(gt, scratch, &gtot);
  if (tid == 0) {  // {#candidates above bin b2 (kSegAll: all of them), #slots used}
    tcount[2 * blockIdx.x] = gtot;
    tcount[2 * blockIdx.x + 1] = nin;
  }
}

// ---------------------------------------------------------------- S4: ordered emission
// The tile's output offset and tie share from the counts of the segment's
// earlier tiles (<= kSegMaxTiles - 1: kS4Per per thread), then the ordered
// compaction of its candidates (a few hundred at k = 1 %: one or two rounds).
// Latency-bound like S3: 256-thread workgroups (cheaper block scans, more
// workgroups resident).  (Cold calls; warm calls take S4w below.)
constexpr int kS4Threads = 256;
constexpr int kS4Per = kSegMaxTiles / kS4Threads;
static_assert(kS4Per * kS4Threads == kSegMaxTiles, "S4 tile-count geometry");
__global__ __launch_bounds__(kS4Threads) void seg_emit_kernel(
    const int64_t* __restrict__ trows, const uint32_t* __restrict__ info, const uint32_t* __restrict__ tilecnt,
    const uint32_t* __restrict__ tcount, uint32_t* __restrict__ hist3, const float* __restrict__ cval,
    const uint32_t* __restrict__ cidx, float* __restrict__ out_val, int32_t* __restrict__ out_idx,
    unsigned long long* __restrict__ shadow, unsigned long long* __restrict__ shadow_host) {
  __shared__ uint32_t scratch[40];
  if (blockIdx.x == 0 && threadIdx.x == 0 && shadow_host)  // S3b's checks of this call are complete
    __hip_atomic_store(shadow_host, __hip_atomic_load(shadow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const TileCtx c = tile_ctx_rows(trows, blockIdx.x);
  if (c.R.ntile == 1) return;  // selected in S2
  const int tid = threadIdx.x;
  if (c.j == 0) {  // every tile of the segment read hist3 in S3b: reset it for the next call
    uint32_t* __restrict__ g3 = hist3 + (int64_t)c.s * kH3;
    for (int i = tid; i < kH3; i += kS4Threads) g3[i] = 0u;
  }
  const uint32_t T = info[8 * c.s + 2], r = info[8 * c.s + 5];
  const uint32_t cnt = tilecnt[blockIdx.x];
  const uint32_t ev = tcount[2 * blockIdx.x + 1];
  uint32_t o, quota;
  {
    uint32_t g = 0u, e = 0u;  // over the segment's tiles ahead of this one
#pragma unroll
    for (int q = 0; q < kS4Per; ++q) {
      const int t = q * kS4Threads + tid;
      if (t < c.j) {
        g += tcount[2 * (c.R.t0 + t)];
        e += tcount[2 * (c.R.t0 + t) + 1];
      }
    }
    uint32_t gp, ep, gsum, esum;
    block_excl_scan2(g, e, scratch, &gp, &ep, &gsum, &esum);
    const uint32_t taken = min(r, esum);  // ties taken by earlier tiles (lowest index first)
    o = gsum + taken;
    quota = min(ev, r - taken);
  }
  const bool all_ties = quota == ev;
  float* __restrict__ ov = out_val + c.R.out_off + o;
  int32_t* __restrict__ oi = out_idx + c.R.out_off + o;
  const uint32_t room = (uint32_t)c.R.k - min(o, (uint32_t)c.R.k);  // (bounded: never past the segment's k)
  uint32_t run = 0, tie_run = 0;
  for (uint32_t p0 = 0; p0 < cnt; p0 += kS4Threads) {  // workgroup-uniform
    const uint32_t p = p0 + tid;
    const bool valid = p < cnt;
    const float v = valid ? cval[c.slot + p] : 0.f;
    const uint32_t ix = valid ? cidx[c.slot + p] : 0u;
    const uint32_t key = fkey(v);
    const bool gt = valid && key > T, eq = valid && key == T;
    bool sel;
    if (all_ties || quota == 0u) {
      sel = gt || (eq && all_ties);
    } else {
      uint32_t ntie;
      const uint32_t trank = tie_run + block_excl_scan(eq ? 1u : 0u, scratch, &ntie);
      sel = gt || (eq && trank < quota);
      tie_run += ntie;
    }
    uint32_t nsel;
    const uint32_t pos = run + block_excl_scan(sel ? 1u : 0u, scratch, &nsel);
    if (sel && pos < room) {
      ov[pos] = v;
      oi[pos] = (int32_t)ix;
    }
    run += nsel;
  }
}

// The shared select's reader over the tiles' candidate lists (W2's compaction: values and
// global indices in index order, tilecnt[b] of them at slot b * kSegTile): the missed
// segments whose k-th key lies above the window hold every key >= T among them.
template <int NT, int U>
struct CandTiles {
  const float* __restrict__ cval;
  const uint32_t* __restrict__ cidx;
  const uint32_t* __restrict__ tilecnt;
  int64_t t0;  // the segment's first tile
  template <class F>
  CHOCO_DEV void operator()(uint32_t t, F&& fn) const {
    const int64_t b = t0 + t;
    const uint32_t cnt = tilecnt[b];
    const __amdgpu_buffer_rsrc_t rv = buf_rsrc(cval + b * kSegTile, cnt * 4u);
    const __amdgpu_buffer_rsrc_t ri = buf_rsrc(reinterpret_cast<const float*>(cidx) + b * kSegTile, cnt * 4u);
    constexpr uint32_t kStep = NT * 4u;
    for (uint32_t b0 = 0; b0 < cnt; b0 += kStep * U) {  // workgroup-uniform
      float4 v[U], q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t off = (b0 + (uint32_t)u * kStep + 4u * threadIdx.x) * 4u;
        v[u] = ld_buf4<false>(rv, off);
        q[u] = ld_buf4<false>(ri, off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (b0 + (uint32_t)u * kStep >= cnt) break;  // block-uniform
        const uint32_t e0 = b0 + (uint32_t)u * kStep + 4u * threadIdx.x;
        const int nin = e0 >= cnt ? 0 : (int)min(4u, cnt - e0);
        const float vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        const int64_t ii[4] = {(int64_t)__float_as_uint(q[u].x), (int64_t)__float_as_uint(q[u].y),
                               (int64_t)__float_as_uint(q[u].z), (int64_t)__float_as_uint(q[u].w)};
        uint32_t kk[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) kk[c] = c < nin ? fkey(vv[c]) : 0u;
        fn(nin, kk, vv, ii);
      }
    }
  }
};

// S4w (warm, after S3w): every tile's (#above b2, #in b2) counts and kept keys of its
// segment are loaded in one round trip (with the tile's first 256 candidates), T is taken
// from the kept keys -- histogrammed by their low sh bits in LDS (bins of one key), the
// rank inside bin b2 located -- and the tile's offset is the earlier tiles' counts above
// b2 plus their kept keys above / at T; then the ordered emission as S4.  One extra
// workgroup per segment (the first nseg of the grid, so they start first) derives the
// same T and writes the next call's window from hist2, then zeroes hist2 (every S3w tile
// has read it) -- off the tiles' chains.  Missed windows and tie overflows: tile 0
// selects the segment exactly.
template <bool XH>
__global__ __launch_bounds__(kS4Threads, 7) void seg_emit_w_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, const int64_t* __restrict__ plan,
    const int64_t* __restrict__ trows, uint32_t nseg, const uint32_t* __restrict__ info,
    const uint32_t* __restrict__ tilecnt, const uint32_t* __restrict__ tcount, uint32_t* __restrict__ hist2,
    const float* __restrict__ cval, const uint32_t* __restrict__ cidx, float* __restrict__ out_val,
    int32_t* __restrict__ out_idx, SegWin* __restrict__ win, uint32_t* __restrict__ misses,
    uint32_t* __restrict__ miss_flag, const uint2* __restrict__ blist, WideCtrl* __restrict__ wide,
    uint32_t* __restrict__ wcnt, uint32_t* __restrict__ whist, uint32_t* __restrict__ status,
    uint32_t* __restrict__ host_status) {
  __shared__ uint32_t scratch[40];
  __shared__ uint32_t h3[kH3];
  __shared__ uint32_t bc[4];
  __shared__ uint32_t s_ovf, s_me, s_tk;
  __shared__ ExactSmem es;
  const int tid = threadIdx.x;
  const bool segwg = blockIdx.x < nseg;  // workgroup-uniform: a segment's window workgroup
  const int64_t b = (int64_t)blockIdx.x - nseg;  // the tile (tile workgroups)
  TileCtx c;
  if (segwg) {
    c.s = (int)blockIdx.x;
    c.R = seg_row(plan, c.s);
    if (c.R.ntile <= 1) return;  // single-tile (selected in S2) or flat-pipeline segment
    c.j = -1;
    c.slot = 0;
    c.start = c.R.off;
    c.tl = 0;
  } else {
    c = tile_ctx_rows(trows, b);
    if (c.R.ntile == 1) return;  // selected in S2
  }
  // ---- one round trip: the segment's info, every tile's counts and kept keys, this
  // tile's count and first 256 candidates
  const uint32_t* I = info + 8 * c.s;
  const uint32_t mode = I[6];
  const uint32_t lo = I[0], sh = I[1], b2 = I[3], rb = I[4];
  uint32_t tg[kS4Per], tn[kS4Per];
  uint2 kk[kS4Per][kTileList];  // {key, count}
#pragma unroll
  for (int q = 0; q < kS4Per; ++q) {
    const int t = q * kS4Threads + tid;
    tg[q] = tn[q] = 0u;
#pragma unroll
    for (int i = 0; i < kTileList; ++i) kk[q][i] = make_uint2(0u, 0u);
    if (t < c.R.ntile) {
      const int64_t tb = c.R.t0 + t;
      const uint2 p = reinterpret_cast<const uint2*>(tcount)[tb];
      tg[q] = p.x;
      tn[q] = p.y;
      const uint4* k4 = reinterpret_cast<const uint4*>(blist + tb * kTileList);
      static_assert(kTileList == 4, "two 16-byte loads of kept keys per tile");
      const uint4 a = k4[0], b = k4[1];
      kk[q][0] = make_uint2(a.x, a.y); kk[q][1] = make_uint2(a.z, a.w);
      kk[q][2] = make_uint2(b.x, b.y); kk[q][3] = make_uint2(b.z, b.w);
    }
  }
  const uint32_t cnt = segwg ? 0u : tilecnt[b];
  float v0 = 0.f;
  uint32_t ix0 = 0u;
  uint32_t hv[kWinPer] = {};  // (segment workgroups: hist2 for the next window, in the same trip)
  uint32_t* __restrict__ g2 = hist2 + (int64_t)c.s * kH;
  SegWin old{};  // (segment workgroups and tile 0: the window this call used, for its drift words)
  if (segwg || c.j == 0) old = win[c.s];
  if (!segwg) {
    v0 = cval[c.slot + tid];  // (inside the tile's slots; masked by cnt below)
    ix0 = cidx[c.slot + tid];
  } else {
    static_assert(kWinPer == 8, "two 16-byte loads of hist2 per thread");
    const uint4* h4 = reinterpret_cast<const uint4*>(g2 + tid * kWinPer);
    const uint4 a = h4[0], bb = h4[1];
    hv[0] = a.x; hv[1] = a.y; hv[2] = a.z; hv[3] = a.w; hv[4] = bb.x; hv[5] = bb.y; hv[6] = bb.z; hv[7] = bb.w;
  }
  bool ovf = false;
#pragma unroll
  for (int q = 0; q < kS4Per; ++q) ovf |= tn[q] > (uint32_t)kTileList;
  // (one barrier for the overflow flag, the LDS histogram's reset and bc)
  if (tid == 0) s_ovf = 0u;
  for (int i = tid; i < kH3; i += kS4Threads) h3[i] = 0u;
  if (tid < 4) bc[tid] = 0u;
  __syncthreads();
  if (ovf) s_ovf = 1u;
  __syncthreads();
  const bool overflow = mode == kSegSelect && s_ovf != 0u;
  if (mode == kSegMissed || mode == kSegMissedHigh || overflow) {  // workgroup-uniform: the segment's tiles
    if (segwg) return;                                                // select it exactly together
    if (c.j == 0 && tid == 0 && mode != kSegSelect) {
      atomicAdd(misses, 1u);
      if (miss_flag) __hip_atomic_store(miss_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    auto on_T = [&](uint32_t T) {  // (every thread of the workgroup that learnt T; no other reader of win / hist2 is left)
      const SegWin prev = win[c.s];
      if (overflow) {  // the window held T: the next one from this call's hist2, as usual
        seg_next_window(g2, lo, sh, 0u, (uint32_t)c.R.k, T, prev, &win[c.s], scratch);
      } else {
        // missed: the next window from this select's digit-1 histogram -- the keys of T's
        // coarse bin (key >> 20) in bins of 2^9 keys, with the keys of the coarse bins above
        // it -- at the usual count levels around k (a blind window centred on T with the
        // widest bins overflowed its bin lists on the next call).  (Over candidate lists the
        // counts below the old window's floor are short: the level k + delta then lands at
        // the coarse bin's floor or the old floor, a wider window.)
        const WideCtrl* Wd = wide + c.s;
        const uint32_t d0 = T >> 20;
        uint32_t a = 0u;
        for (int i = tid; i < kH; i += kS4Threads) a += (uint32_t)i > d0 ? ld_sc1(&Wd->hist[0][i]) : 0u;
        uint32_t above;
        block_excl_scan(a, scratch, &above);
        uint32_t hv[kWinPer];
#pragma unroll
        for (int j = 0; j < kWinPer; ++j) hv[j] = ld_sc1(&Wd->hist[1][tid * kWinPer + j]);
        seg_next_window_v(hv, d0 << 20, 9u, above, (uint32_t)c.R.k, T, prev, &win[c.s], scratch);
      }
      __syncthreads();
      for (int i = tid; i < kH; i += kS4Threads) g2[i] = 0u;
    };
    // (2 rows in flight over the segment, 1 over the candidate lists -- a few hundred per
    // tile, one row; the launch bounds hold S4w at 7 waves per SIMD without spills: the
    // shared select is the rare branch of this kernel)
    if (mode == kSegMissed) {
      Src<kData, XH> src{x + c.R.off, XH ? xh + c.R.off : nullptr, 0};
      wide_select<kS4Threads>(RangeTiles<kS4Threads, 2, kData, XH>{src, c.R.len, (uint32_t)kSegTile}, c.R.k,
                              (uint32_t)c.R.ntile, wide + c.s, wcnt + 2 * c.R.t0, whist + 512 * c.R.t0, es, &s_tk,
                              status, host_status, on_T, [&](uint32_t pos, int64_t i, float v) {
                                out_val[c.R.out_off + pos] = v;
                                out_idx[c.R.out_off + pos] = (int32_t)(i + c.R.off);
                              });
    } else {  // every key >= T is among the candidates: select over the tiles' candidate lists
      wide_select<kS4Threads>(CandTiles<kS4Threads, 1>{cval, cidx, tilecnt, c.R.t0}, c.R.k, (uint32_t)c.R.ntile,
                              wide + c.s, wcnt + 2 * c.R.t0, whist + 512 * c.R.t0, es, &s_tk, status, host_status,
                              on_T, [&](uint32_t pos, int64_t ix, float v) {
                                out_val[c.R.out_off + pos] = v;
                                out_idx[c.R.out_off + pos] = (int32_t)ix;
                              });
    }
    return;
  }
  // ---- T and the ties at it to take, from the kept keys (mode kSegAll: every candidate)
  uint32_t T = 0, r = 0;
  if (mode == kSegSelect) {  // workgroup-uniform
    const uint32_t fmask = (1u << sh) - 1u;
#pragma unroll
    for (int q = 0; q < kS4Per; ++q)
#pragma unroll
      for (int i = 0; i < kTileList; ++i)
        if ((uint32_t)i < tn[q]) atomicAdd(&h3[(kk[q][i].x - lo) & fmask], kk[q][i].y);
    __syncthreads();
    block_find_rank_g<kH3 / kS4Threads>(h3, rb, scratch, bc);
    T = lo + (b2 << sh) + bc[0];
    r = bc[1];
  }
  if (segwg) {  // the next call's window (this call's hist2: the window's own bins), then hist2 reset
    if (mode == kSegSelect) {
      seg_next_window_v(hv, lo, sh, 0u, (uint32_t)c.R.k, T, old, &win[c.s], scratch);
      __syncthreads();
    } else if (tid == 0) {
      win[c.s] = SegWin{0u, kWinShMax, 1u, 0u, 0u, 0u, 0u, 0u};
    }
    for (int i = tid; i < kH; i += kS4Threads) g2[i] = 0u;
    return;
  }
  // ---- offsets: the earlier tiles' candidates above bin b2 and their kept keys above / at
  // T; this tile's kept keys at T (its ties)
  uint32_t g = 0u, le = 0u;
#pragma unroll
  for (int q = 0; q < kS4Per; ++q) {
    const int t = q * kS4Threads + tid;
    uint32_t above = 0u, at = 0u;
    if (mode == kSegSelect) {
#pragma unroll
      for (int i = 0; i < kTileList; ++i) {
        above += ((uint32_t)i < tn[q] && kk[q][i].x > T) ? kk[q][i].y : 0u;
        at += ((uint32_t)i < tn[q] && kk[q][i].x == T) ? kk[q][i].y : 0u;
      }
    }
    if (t < c.j) {
      g += tg[q] + above;
      le += at;
    } else if (t == c.j) {
      s_me = at;  // (one thread; read after the scan's barriers)
    }
  }
  uint32_t gp, ep, gsum, lesum;
  block_excl_scan2(g, le, scratch, &gp, &ep, &gsum, &lesum);
  const uint32_t mesum = s_me;
  const uint32_t taken = min(r, lesum);  // ties taken by earlier tiles (lowest index first)
  const uint32_t o = gsum + taken;
  const uint32_t quota = min(mesum, r - taken);
  const bool all_ties = quota == mesum;
  float* __restrict__ ov = out_val + c.R.out_off + o;
  int32_t* __restrict__ oi = out_idx + c.R.out_off + o;
  const uint32_t room = (uint32_t)c.R.k - min(o, (uint32_t)c.R.k);  // (bounded: never past the segment's k)
  uint32_t run = 0, tie_run = 0;
  for (uint32_t p0 = 0; p0 < cnt; p0 += kS4Threads) {  // workgroup-uniform
    const uint32_t p = p0 + tid;
    const bool valid = p < cnt;
    const float v = p0 == 0 ? v0 : (valid ? cval[c.slot + p] : 0.f);
    const uint32_t ix = p0 == 0 ? ix0 : (valid ? cidx[c.slot + p] : 0u);
    const uint32_t key = fkey(v);
    const bool gt = valid && (mode == kSegAll || key > T), eq = valid && mode != kSegAll && key == T;
    bool sel;
    if (all_ties || quota == 0u) {
      sel = gt || (eq && all_ties);
    } else {
      uint32_t ntie;
      const uint32_t trank = tie_run + block_excl_scan(eq ? 1u : 0u, scratch, &ntie);
      sel = gt || (eq && trank < quota);
      tie_run += ntie;
    }
    uint32_t nsel;
    const uint32_t pos = run + block_excl_scan(sel ? 1u : 0u, scratch, &nsel);
    if (sel && pos < room) {
      ov[pos] = v;
      oi[pos] = (int32_t)ix;
    }
    run += nsel;
  }
}

// ---------------------------------------------------------------- host side
static int64_t plan_tiles(const int64_t* plan_host) { return plan_host[6]; }
static int64_t plan_batched(const int64_t* plan_host) { return plan_host[7]; }

// Warm bookkeeping per segmented workspace: whether an earlier call left windows, and a
// cold backoff driven by the device.  S4w raises a flag in pinned host memory (a system-
// scope store, no copy on the stream) when a segment's window missed; the host sees it
// a few calls later (whenever that S4w has run).  A miss seen within kSegMissGap calls of
// the previous one starts the cold sequence (S1 + S2, two reads, never a miss) for a run
// of 64 calls, doubling per run that ends in a new miss, up to 4096.  A stationary delta
// never raises the flag and never pays anything; a delta whose k-th keys keep moving out
// of their windows (x_hat draining the top keys) pays the second read instead of S4w's
// shared exact select of every missed segment.
// A cold run ends early when the windows the cold calls prepare would have held their
// successors' k-th keys: S3b of every cold call checks, per multi-tile segment, the window
// the previous call left (drift-aware, window_drift) against its exact T and counts
// (misses << 32 | checks) in the same pinned page; one cold call's worth of checks with no
// miss ends the run (the drift that caused the miss is followed now).
struct SegState {
  uint64_t calls = 0;
  uint64_t last_flag = 0;  // the call at which the host last saw the miss flag (0: never)
  uint32_t cold_left = 0, backoff = 0;
  uint32_t* flag = nullptr;  // pinned, mapped; word 0: the device writes 1 on a miss; words 2-3: shadow counter
  uint32_t* flag_dev = nullptr;
  uint32_t last_checks = 0, last_misses = 0, clean = 0;
};
constexpr uint32_t kSegShadowExit = 1;  // (2: warm share 0.90 against 0.967, profiles/r06_ab_summary.txt item 10)
// An isolated miss stays warm: S4w's shared exact select handled it (~0.1 ms at ResNet-50's
// largest tensor) and re-centred the window on that select's histogram; only a miss seen
// within kSegMissGap calls of the previous one starts a cold run.  (The host can run many
// calls ahead of the device, so a cold run rarely ends early by the shadow checks: on the
// bench's realistic step every isolated miss cost a whole 64-call run, warm share 0.675
// over 400 steps.)
constexpr uint64_t kSegMissGap = 32;
static uint64_t seg_shadow_read(const SegState& S) {
  return S.flag ? __atomic_load_n(reinterpret_cast<uint64_t*>(S.flag + 2), __ATOMIC_ACQUIRE) : 0ull;
}
static std::mutex g_seg_mu;
static std::unordered_map<const void*, SegState> g_seg;
static bool seg_claim_warm(const void* ws, uint32_t nmulti, uint32_t** flag_dev, unsigned long long** shadow_host) {
  std::lock_guard<std::mutex> g(g_seg_mu);
  SegState& S = g_seg[ws];
  if (!S.flag) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
      S.flag = static_cast<uint32_t*>(h);
      for (int i = 0; i < 16; ++i) __atomic_store_n(S.flag + i, 0u, __ATOMIC_RELEASE);
      void* d = nullptr;
      if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess) S.flag_dev = static_cast<uint32_t*>(d);
    }
  }
  *flag_dev = S.flag_dev;  // (null: no backoff, warm as before)
  *shadow_host = S.flag_dev ? reinterpret_cast<unsigned long long*>(S.flag_dev + 2) : nullptr;
  const bool first = S.calls++ == 0;
  if (S.flag && __atomic_load_n(S.flag, __ATOMIC_ACQUIRE) != 0u) {
    __atomic_store_n(S.flag, 0u, __ATOMIC_RELEASE);
    const bool recurring = S.last_flag != 0u && S.calls - S.last_flag <= kSegMissGap;
    S.last_flag = S.calls;
    if (recurring) {
      S.backoff = std::min<uint32_t>(std::max<uint32_t>(2u * S.backoff, 64u), 4096u);
      S.cold_left = S.backoff;
      const uint64_t v = seg_shadow_read(S);  // checks from before this run do not count
      S.last_checks = (uint32_t)v;
      S.last_misses = (uint32_t)(v >> 32);
      S.clean = 0u;
    }
  }
  if (first) return false;
  if (S.cold_left != 0u) {
    if (S.flag && nmulti > 0u) {
      const uint64_t v = seg_shadow_read(S);
      const uint32_t dc = (uint32_t)v - S.last_checks, dm = (uint32_t)(v >> 32) - S.last_misses;
      if (dc >= nmulti) {  // at least one more cold call's checks have landed
        S.clean = dm == 0u ? S.clean + dc / nmulti : 0u;
        S.last_checks = (uint32_t)v;
        S.last_misses = (uint32_t)(v >> 32);
      }
      if (S.clean >= kSegShadowExit) {
        S.cold_left = 0u;
        S.clean = 0u;
        S.backoff = std::max<uint32_t>(S.backoff / 2u, 64u);
        return topk_warm_enabled();
      }
    }
    --S.cold_left;
    return false;
  }
  return topk_warm_enabled();
}
void seg_forget(const void* ws, size_t bytes) {
  std::lock_guard<std::mutex> g(g_seg_mu);
  const char* lo = static_cast<const char*>(ws);
  for (auto it = g_seg.begin(); it != g_seg.end();) {
    const char* p = static_cast<const char*>(it->first);
    if (p == lo || (p > lo && p < lo + bytes)) {
      if (it->second.flag) (void)hipHostFree(it->second.flag);  // (callers synchronise before a reset)
      it = g_seg.erase(it);
    } else {
      ++it;
    }
  }
}

template <bool XH, bool GS>
static int launch_batched(const float* x, const float* xh, const int64_t* plan_dev, const int64_t* plan_host,
                          int nseg, float* out_val, int32_t* out_idx, const SegWs& W, bool warm, hipStream_t st,
                          Gossip gs) {
  const unsigned ntile = (unsigned)plan_tiles(plan_host);
  // the collect launches' dispatch order (choco_topk_segmented_plan: after the random-k table)
  const int64_t rkb = (int64_t)kRow * nseg + plan_tiles(plan_host) + plan_batched(plan_host);  // (rk_base_of)
  const int64_t* w2_order = plan_dev + rkb + 1 + 4 * plan_host[rkb];
  // the per-tile rows (after the dispatch records): S1 / S3 / S4 look their tile up in one round trip
  const int64_t* trows = plan_dev + rkb + 1 + 4 * plan_host[rkb] + 4 * (int64_t)ntile;
  if (!warm) {
    profile_begin("topk_seg_hist", st);
    CHOCO_KLAUNCH((seg_hist_kernel<XH, GS>), dim3(ntile), dim3(kSegThreads), 0, st, x, xh, trows, nseg, W.hist1,
                  gs);
    profile_end("topk_seg_hist", st);
    CHOCO_LAUNCHED("seg_hist_kernel");
    profile_begin("topk_seg_collect", st);
    CHOCO_KLAUNCH((seg_collect_kernel<XH, false, false>), dim3(ntile), dim3(kSegThreads), 0, st, x, xh, plan_dev,
                  nseg, W.hist1, W.hist2, W.info, W.tilecnt, W.cval, W.cidx, W.win, Gossip{nullptr, 0.f}, out_val,
                  out_idx, (int64_t)ntile, w2_order);
  } else {
    profile_begin("topk_seg_collect", st);
    CHOCO_KLAUNCH((seg_collect_kernel<XH, true, GS>), dim3(ntile), dim3(kSegThreads), 0, st, x, xh, plan_dev, nseg,
                  W.hist1, W.hist2, W.info, W.tilecnt, W.cval, W.cidx, W.win, gs, out_val, out_idx, (int64_t)ntile,
                  w2_order);
  }
  profile_end("topk_seg_collect", st);
  CHOCO_LAUNCHED("seg_collect_kernel");
  if (warm) {
    profile_begin("topk_seg_bin", st);
    CHOCO_KLAUNCH(seg_bin_kernel, dim3(ntile), dim3(kS3Threads), 0, st, trows, W.hist2, W.info, W.tilecnt, W.cval,
                  W.win, W.tcount, W.blist);
    profile_end("topk_seg_bin", st);
    CHOCO_LAUNCHED("seg_bin_kernel");
    profile_begin("topk_seg_emit", st);
    CHOCO_KLAUNCH((seg_emit_w_kernel<XH>), dim3(ntile + (unsigned)nseg), dim3(kS4Threads), 0, st, x, xh, plan_dev,
                  trows, (uint32_t)nseg, W.info, W.tilecnt, W.tcount, W.hist2, W.cval, W.cidx, out_val, out_idx, W.win, W.misses,
                  W.miss_flag, W.blist, W.wide, W.wcnt, W.whist, W.status, W.host_status);
    profile_end("topk_seg_emit", st);
    CHOCO_LAUNCHED("seg_emit_w_kernel");
    return CHOCO_OK;
  }
  // cold calls: S3a, S3b, S4
  profile_begin("topk_seg_fine", st);
  CHOCO_KLAUNCH(seg_fine_kernel, dim3(ntile), dim3(kS3Threads), 0, st, trows, nseg, W.hist1, W.hist2, W.hist3,
                W.info, W.tilecnt, W.cval);
  profile_end("topk_seg_fine", st);
  CHOCO_LAUNCHED("seg_fine_kernel");
  profile_begin("topk_seg_count", st);
  CHOCO_KLAUNCH(seg_count_kernel, dim3(ntile), dim3(kS3Threads), 0, st, trows, nseg, W.hist2, W.hist3, W.info,
                W.tilecnt, W.cval, W.tcount, W.win, W.shadow);
  profile_end("topk_seg_count", st);
  CHOCO_LAUNCHED("seg_count_kernel");
  profile_begin("topk_seg_emit", st);
  CHOCO_KLAUNCH(seg_emit_kernel, dim3(ntile), dim3(kS4Threads), 0, st, trows, W.info, W.tilecnt, W.tcount,
                W.hist3, W.cval, W.cidx, out_val, out_idx, W.shadow, W.shadow_host);
  profile_end("topk_seg_emit", st);
  CHOCO_LAUNCHED("seg_emit_kernel");
  return CHOCO_OK;
}

// Segments over kSegBatchMax elements: one flat-pipeline workspace EACH (after the
// batched one), so each keeps its own warm-start window between calls.
static size_t pipeline_ws(const int64_t* plan_host, int nseg) {
  size_t need = 0;
  for (int s = 0; s < nseg; ++s) {
    const int64_t* p = plan_host + (int64_t)kRow * s;
    if (p[5] == 0) need += align_up(topk_ws_bytes(p[1]), 256);
  }
  return need;
}

// gs.mem != nullptr: the fused gossip step (cold: inside S1; warm: inside S2; the
// flat pipeline: inside its stream).
static int segmented(const float* x, const float* xhat, const int64_t* plan_dev, const int64_t* plan_host,
                     int32_t nseg, float* out_val, int32_t* out_idx, void* ws, size_t ws_bytes, hipStream_t st,
                     Gossip gs = Gossip{nullptr, 0.f}) {
  CHOCO_REQUIRE(x && plan_dev && plan_host && out_val && out_idx && nseg > 0, "null pointer argument");
  CHOCO_REQUIRE(aligned4(x) && (xhat == nullptr || aligned4(xhat)), "x/xhat must be 4-byte aligned");
  const int64_t* last = plan_host + (int64_t)kRow * (nseg - 1);
  CHOCO_REQUIRE(last[0] + last[1] < (int64_t)INT32_MAX, "total length must be < 2^31");
  if (gs.mem) CHOCO_REQUIRE(xhat != nullptr && aligned4(gs.mem), "the gossip step needs x_hat and a 4-byte aligned memory");
  const int64_t ntile = plan_tiles(plan_host);
  const SegLayout L = seg_layout(nseg, ntile);
  const size_t need = L.total + pipeline_ws(plan_host, nseg);
  CHOCO_REQUIRE(ws != nullptr && ws_bytes >= need, "segmented top-k workspace too small: need %zu bytes, got %zu",
                need, ws_bytes);
  char* base = static_cast<char*>(ws);
  if (ntile > 0) {
    SegWs W{reinterpret_cast<uint32_t*>(base + L.off_h1), reinterpret_cast<uint32_t*>(base + L.off_h2),
            reinterpret_cast<uint32_t*>(base + L.off_h3),
            reinterpret_cast<uint32_t*>(base + L.off_info), reinterpret_cast<uint32_t*>(base + L.off_cnt),
            reinterpret_cast<uint32_t*>(base + L.off_out), reinterpret_cast<float*>(base + L.off_cval),
            reinterpret_cast<uint32_t*>(base + L.off_cidx), reinterpret_cast<SegWin*>(base + L.off_win),
            reinterpret_cast<uint32_t*>(base + CHOCO_TOPK_FALLBACKS_OFFSET), nullptr,
            reinterpret_cast<unsigned long long*>(base + kSegShadowOffset), nullptr,
            reinterpret_cast<uint2*>(base + L.off_blist), reinterpret_cast<WideCtrl*>(base + L.off_wide),
            reinterpret_cast<uint32_t*>(base + L.off_wcnt), reinterpret_cast<uint32_t*>(base + L.off_whist),
            reinterpret_cast<uint32_t*>(base + CHOCO_TOPK_STATUS_OFFSET),
            host_status_dev(ws)};
    CHOCO_REQUIRE(W.host_status != nullptr,
                  "top-k: could not map the pinned host mirror of the workspace status word (hipHostMalloc / "
                  "hipHostGetDevicePointer failed), so a failed exact-select wait could not be reported");
    uint32_t nmulti = 0;  // segments with windows (multi-tile, batched): the shadow checks per cold call
    for (int s = 0; s < nseg; ++s) nmulti += plan_host[(int64_t)kRow * s + 5] > 1 ? 1u : 0u;
    const bool warm = seg_claim_warm(base + L.off_win, nmulti, &W.miss_flag, &W.shadow_host);
    int rc;
    if (gs.mem)
      rc = launch_batched<true, true>(x, xhat, plan_dev, plan_host, nseg, out_val, out_idx, W, warm, st, gs);
    else if (xhat)
      rc = launch_batched<true, false>(x, xhat, plan_dev, plan_host, nseg, out_val, out_idx, W, warm, st, gs);
    else
      rc = launch_batched<false, false>(x, xhat, plan_dev, plan_host, nseg, out_val, out_idx, W, warm, st, gs);
    if (rc) return rc;
  }
  // segments over kSegBatchMax elements: the flat pipeline, one after another, each
  // in its own workspace after the batched one (the batched histograms must stay
  // zero); their fallbacks flag this call's status word
  size_t fo = L.total;
  for (int s = 0; s < nseg; ++s) {
    const int64_t* p = plan_host + (int64_t)kRow * s;
    if (p[5] != 0) continue;
    const Gossip gseg{gs.mem ? gs.mem + p[0] : nullptr, gs.gamma};
    const size_t fb = align_up(topk_ws_bytes(p[1]), 256);
    uint32_t* hs = host_status_dev(ws);
    CHOCO_REQUIRE(hs != nullptr,
                  "top-k: could not map the pinned host mirror of the workspace status word (hipHostMalloc / "
                  "hipHostGetDevicePointer failed), so a failed exact-fallback wait could not be reported");
    const int rc = topk_pipeline(kData, x + p[0], xhat ? xhat + p[0] : nullptr, p[1], p[2], 0, 1.0f,
                                 out_val + p[3], out_idx + p[3], p[0], base + fo, fb, st, gseg,
                                 StatusSink{reinterpret_cast<uint32_t*>(base + CHOCO_TOPK_STATUS_OFFSET), hs});
    if (rc) return rc;
    fo += fb;
  }
  return CHOCO_OK;
}

}  // namespace choco

using namespace choco;

static int seg_plan_scan(const int64_t* seg_off_host, int32_t nseg, int64_t* ntile, int64_t* nbat) {
  if (seg_off_host == nullptr || nseg <= 0) return fail(CHOCO_ERR_INVALID, "bad segment table");
  *ntile = 0;
  *nbat = 0;
  for (int s = 0; s < nseg; ++s) {
    const int64_t len = seg_off_host[s + 1] - seg_off_host[s];
    if (len <= 0) return fail(CHOCO_ERR_INVALID, "segment %d has length %lld", s, (long long)len);
    if (len <= kSegBatchMax) {
      *ntile += (len + kSegTile - 1) / kSegTile;
      *nbat += 1;
    }
  }
  return CHOCO_OK;
}

static int64_t rk_plan_tiles(const int64_t* seg_off_host, int32_t nseg) {
  int64_t R = 0;
  for (int s = 0; s < nseg; ++s) R += randk_tiles(seg_off_host[s + 1] - seg_off_host[s]);
  return R;
}

#if CHOCO_STAMPS
// Diagnostic builds only: copy out (and clear) the segmented collect stamps.
CHOCO_API int choco_dbg_seg_stamps(unsigned long long* host, size_t bytes) {
  const size_t all = sizeof(unsigned long long) * kSgStampSlots * 4;
  if (bytes > all) bytes = all;
  if (host) CHOCO_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sg_stamps), bytes, 0, hipMemcpyDeviceToHost));
  static unsigned long long zeros[kSgStampSlots * 4];
  CHOCO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sg_stamps), zeros, all, 0, hipMemcpyHostToDevice));
  return CHOCO_OK;
}
#endif

CHOCO_API int64_t choco_topk_segmented_plan_len(const int64_t* seg_off_host, int32_t nseg) {
  int64_t ntile, nbat;
  const int rc = seg_plan_scan(seg_off_host, nseg, &ntile, &nbat);
  if (rc) return rc;
  return (int64_t)kRow * nseg + ntile + nbat + 1 + 4 * rk_plan_tiles(seg_off_host, nseg) + 4 * ntile + 8 * ntile;
}

CHOCO_API int64_t choco_topk_segmented_plan(const int64_t* seg_off_host, int32_t nseg, double ratio,
                                            int64_t* plan_host) {
  int64_t ntile, nbat;
  const int rc = seg_plan_scan(seg_off_host, nseg, &ntile, &nbat);
  if (rc) return rc;
  CHOCO_REQUIRE(ratio >= 0.0 && ratio < 1.0, "compress ratio must be in [0, 1), got %g", ratio);
  int64_t out = 0, t0 = 0, b = 0;
  for (int s = 0; s < nseg; ++s) {
    const int64_t off = seg_off_host[s], len = seg_off_host[s + 1] - seg_off_host[s];
    const int64_t k = choco_topk_k(len, ratio);
    const int64_t nt = len <= kSegBatchMax ? (len + kSegTile - 1) / kSegTile : 0;
    if (plan_host) {
      int64_t* p = plan_host + (int64_t)kRow * s;
      p[0] = off; p[1] = len; p[2] = k; p[3] = out; p[4] = t0; p[5] = nt; p[6] = 0; p[7] = 0;
      for (int64_t t = 0; t < nt; ++t) plan_host[(int64_t)kRow * nseg + t0 + t] = s;
      if (nt) plan_host[(int64_t)kRow * nseg + ntile + b++] = s;
    }
    t0 += nt;
    out += k;
  }
  if (plan_host) {
    plan_host[6] = ntile;
    plan_host[7] = nbat;
    // the random-k tile table (randk.hip): [R] then R x {segment, tile, first tile, tiles}
    int64_t* rk = plan_host + (int64_t)kRow * nseg + ntile + nbat;
    int64_t r = 0;
    for (int s = 0; s < nseg; ++s) {
      const int64_t nt = randk_tiles(seg_off_host[s + 1] - seg_off_host[s]);
      for (int64_t t = 0; t < nt; ++t) {
        int64_t* e = rk + 1 + 4 * (r + t);
        e[0] = s; e[1] = t; e[2] = r; e[3] = nt;
      }
      r += nt;
    }
    rk[0] = r;
    // The collect launch's dispatch order, one record {tile, segment, first element,
    // length} per workgroup: the tiles of single-tile segments (selected exactly in the
    // collect by a latency-bound three-round radix select) first, so that they overlap
    // the streaming of the large segments' tiles instead of ending the launch; and a
    // workgroup's loads need ONE scalar round trip (r04 stamps: the three dependent plan
    // lookups -- tile -> segment -> row -> start -- took up to 2 us per tile under load)
    int64_t* order = rk + 1 + 4 * r;
    int64_t q = 0;
    for (int pass = 0; pass < 2; ++pass)
      for (int s = 0; s < nseg; ++s) {
        const int64_t* p = plan_host + (int64_t)kRow * s;
        if ((p[5] == 1) != (pass == 0)) continue;
        for (int64_t t = 0; t < p[5]; ++t) {
          int64_t* e = order + 4 * q++;
          e[0] = p[4] + t;
          e[1] = s;
          e[2] = p[0] + t * kSegTile;
          e[3] = std::min<int64_t>(kSegTile, p[1] - t * kSegTile);
        }
      }
    // per tile (tile-id order): its segment's row and the segment id
    int64_t* trows = order + 4 * ntile;
    for (int s = 0; s < nseg; ++s) {
      const int64_t* p = plan_host + (int64_t)kRow * s;
      for (int64_t t = 0; t < p[5]; ++t) {
        int64_t* e = trows + 8 * (p[4] + t);
        for (int i = 0; i < 6; ++i) e[i] = p[i];
        e[6] = s;
        e[7] = 0;
      }
    }
  }
  return out;
}

static int64_t rk_base_of(const int64_t* plan_host, int32_t nseg) {
  return (int64_t)kRow * nseg + plan_tiles(plan_host) + plan_batched(plan_host);
}

CHOCO_API size_t choco_topk_segmented_workspace_size(const int64_t* plan_host, int32_t nseg) {
  if (!plan_host || nseg <= 0) return 256;
  return seg_layout(nseg, plan_tiles(plan_host)).total + pipeline_ws(plan_host, nseg) +
         randk_counts_bytes(plan_host[rk_base_of(plan_host, nseg)]) + 256;
}

// Per-segment random-k (randk.hip): the counts buffer follows the top-k regions.
static int randk_segmented_call(const float* x, const float* xhat, const int64_t* plan_dev, const int64_t* plan_host,
                                int32_t nseg, uint64_t seed, uint64_t offset, int32_t is_biased, float* out_val,
                                int32_t* out_idx, void* ws, size_t ws_bytes, hipStream_t st,
                                Gossip gs = Gossip{nullptr, 0.f}) {
  CHOCO_REQUIRE(x && plan_dev && plan_host && out_val && out_idx && nseg > 0, "null pointer argument");
  CHOCO_REQUIRE(aligned4(x) && (xhat == nullptr || aligned4(xhat)), "x/xhat must be 4-byte aligned");
  const int64_t* last = plan_host + (int64_t)kRow * (nseg - 1);
  const int64_t n = last[0] + last[1];
  CHOCO_REQUIRE(n < (int64_t)INT32_MAX, "total length must be < 2^31");
  const int64_t rk_base = rk_base_of(plan_host, nseg);
  const int64_t R = plan_host[rk_base];
  const size_t off = seg_layout(nseg, plan_tiles(plan_host)).total + pipeline_ws(plan_host, nseg);
  CHOCO_REQUIRE(ws != nullptr && ws_bytes >= off + randk_counts_bytes(R),
                "segmented random-k workspace too small: need %zu bytes, got %zu", off + randk_counts_bytes(R),
                ws_bytes);
  if (gs.mem) {
    // random-k reads only k elements: no full pass to fuse the consensus step into
    CHOCO_REQUIRE(xhat != nullptr && aligned4(gs.mem), "the gossip step needs x_hat and a 4-byte aligned memory");
    const int rc = gossip_launch(const_cast<float*>(x), gs.mem, xhat, gs.gamma, n, st);
    if (rc) return rc;
  }
  return randk_launch(x, xhat, plan_dev, rk_base, R, n, 0, seed, offset, is_biased, out_val, out_idx,
                      static_cast<char*>(ws) + off, ws_bytes - off, st);
}

CHOCO_API int choco_topk_compress_segmented(const float* x, const float* xhat, const int64_t* plan_dev,
                                            const int64_t* plan_host, int32_t nseg, float* out_val,
                                            int32_t* out_idx, void* ws, size_t ws_bytes, void* stream) {
  return segmented(x, xhat, plan_dev, plan_host, nseg, out_val, out_idx, ws, ws_bytes, as_stream(stream));
}

CHOCO_API int choco_randk_compress_segmented(const float* x, const float* xhat, const int64_t* plan_dev,
                                             const int64_t* plan_host, int32_t nseg, uint64_t seed, uint64_t offset,
                                             int32_t is_biased, float* out_val, int32_t* out_idx, void* ws,
                                             size_t ws_bytes, void* stream) {
  return randk_segmented_call(x, xhat, plan_dev, plan_host, nseg, seed, offset, is_biased, out_val, out_idx, ws,
                              ws_bytes, as_stream(stream));
}

CHOCO_API int choco_gossip_topk_compress_segmented(float* x, const float* memory, const float* xhat, float gamma,
                                                   const int64_t* plan_dev, const int64_t* plan_host, int32_t nseg,
                                                   float* out_val, int32_t* out_idx, void* ws, size_t ws_bytes,
                                                   void* stream) {
  CHOCO_REQUIRE(memory != nullptr && xhat != nullptr, "the gossip step needs memory and x_hat");
  return segmented(x, xhat, plan_dev, plan_host, nseg, out_val, out_idx, ws, ws_bytes, as_stream(stream),
                   Gossip{memory, gamma});
}

CHOCO_API int choco_gossip_randk_compress_segmented(float* x, const float* memory, const float* xhat, float gamma,
                                                    const int64_t* plan_dev, const int64_t* plan_host, int32_t nseg,
                                                    uint64_t seed, uint64_t offset, int32_t is_biased,
                                                    float* out_val, int32_t* out_idx, void* ws, size_t ws_bytes,
                                                    void* stream) {
  CHOCO_REQUIRE(memory != nullptr && xhat != nullptr, "the gossip step needs memory and x_hat");
  return randk_segmented_call(x, xhat, plan_dev, plan_host, nseg, seed, offset, is_biased, out_val, out_idx, ws,
                              ws_bytes, as_stream(stream), Gossip{memory, gamma});
}
