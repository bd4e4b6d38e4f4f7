// Top-k / random-k sparsification for the CHOCO gossip step on MI355X.
//
// Replaces SparsificationCompressor.get_top_k / get_random_k
// (reference dl_code/pcode/utils/sparsification.py:18-54) and the per-tensor
// compress loop of CHOCOSparsificationCompressor (parallel_choco_v.py:229-260).
//
// Exact semantics (every path below produces bit-identical results):
//   T  = k-th largest key(d) (key = |d| bits, see choco_common.h)
//   out = { i : key_i > T }  U  { the (k - #{key > T}) lowest i with key_i == T },
//   emitted as (d_i, i) in ascending i.
//
// Fast path for large n ("pipeline"); the delta is read from HBM ONCE:
//   K1 topk_sample  : one workgroup histograms a 64K-element strided sample of
//                     keys (32K bins = key>>16) and picks a candidate floor s_lo
//                     (#{key >= s_lo} >= k with ~6 sigma margin) and a "sure"
//                     ceiling s_hi (#{key >= s_hi} < k); [s_lo, s_hi) is split
//                     into 63 equal key-buckets of width 2^shift.
//   K2 topk_stream  : persistent streaming pass over 32K-element tiles (4 waves,
//                     each a contiguous 8K range).  Loads are double-buffered in
//                     registers; per float4 row the wave ballots candidates
//                     (key >= s_lo), prefix-counts them with bit-sliced ballots
//                     + mbcnt and appends (value, index) in index order to an LDS
//                     stage that is flushed to the wave's slot of the candidate
//                     buffer in coalesced 256-B stores.  "maybe" candidates
//                     (key < s_hi) are also kept in LDS and, at the end of the
//                     tile, counting-sorted by bucket into a per-tile side list;
//                     per-tile bucket suffix counts go to a [64][nb] table and,
//                     by one 256-B wave atomic, to replicated global totals.
//   K3 topk_select  : one workgroup finds the bucket j* holding the k-th key from
//                     the totals, gathers that bucket's keys (a few thousand)
//                     from the side lists into LDS, radix-selects T and the tie
//                     quota exactly and scans per-tile output offsets.
//   K4 topk_emit    : one workgroup per tile compacts the tile's candidates into
//                     the final ascending-index output.
//   If the sample's guess was off (too few candidates, T in the "sure" range,
//   bucket j* larger than LDS, or a wave's maybe-list overflowed), K3 runs an
//   exact single-workgroup radix select over the full input instead (correct,
//   slow, data-dependent only) and K4 exits.
// Small n (<= kSmallN) and every segment of the batched segmented path use
// the same exact radix select (block_topk_exact) in one workgroup.
#include "choco_common.h"

#include <math.h>
#include <algorithm>

namespace choco {

constexpr int kK2Threads = 256;
constexpr int kK2Waves = kK2Threads / 64;
constexpr int kK2Unroll = 4;            // float4 rows per wave per pipeline stage
constexpr int kK2BlocksPerCU = 4;
constexpr int kStage = 512;             // LDS staging entries per wave
constexpr int kNBucket = 64;            // 63 "maybe" buckets + 1 "sure"
constexpr int kMaybeCap = 512;          // maybe keys per wave kept in LDS
constexpr int kSideCap = kK2Waves * kMaybeCap;
constexpr int kNRep = 8;                // replicas of the global totals (per XCD group)
constexpr int kNbMax = 4096;            // max tiles (K3 keeps per-tile arrays in LDS)
constexpr int kMCap = 16384;            // max keys of bucket j* handled in LDS
constexpr int kK3Threads = 1024;
constexpr int kK4Threads = 256;
constexpr int kK1Blocks = 64;           // sample workgroups, 1024 samples each
constexpr int kK1Threads = 256;
constexpr int kK1ListCap = 256;         // per-workgroup tail-list capacity
constexpr int kSampleN = kK1Blocks * kK1Threads * 4;   // 65536
constexpr int kSampleChunk = 256;
constexpr int64_t kSmallN = 65536;
constexpr int kExactThreads = 1024;

enum SrcMode { kData = 0, kHash = 1 };
enum TileMode { kTakeNone = 0, kTakeAll = 1, kTakePartial = 2 };

struct TopkCtrl {
  uint32_t s_lo, s_hi, shift, overflow;
  uint32_t T, r, fallback, k1_ticket;
  uint32_t pad[8];
  uint32_t G[kNRep][kNBucket];
};

struct TopkLayout {
  int64_t n;
  uint32_t tile, nb;
  size_t off_ctrl, off_cum, off_cntw, off_side, off_tile, off_k1, off_cval, off_cidx, total;
};

static TopkLayout topk_layout(int64_t n) {
  TopkLayout L{};
  L.n = n;
  uint32_t tile = 32768;
  while ((int64_t)tile * kNbMax < n) tile <<= 1;
  L.tile = tile;
  L.nb = (uint32_t)((n + tile - 1) / tile);
  size_t o = 0;
  L.off_ctrl = o; o += align_up(sizeof(TopkCtrl), 256);
  L.off_cum = o;  o += align_up((size_t)kNBucket * L.nb * 4, 256);
  L.off_cntw = o; o += align_up((size_t)L.nb * kK2Waves * 4, 256);
  L.off_side = o; o += align_up((size_t)L.nb * kSideCap * 4, 256);
  L.off_tile = o; o += align_up((size_t)L.nb * 3 * 4, 256);   // tile_off | tile_tieb | tile_mode
  L.off_k1 = o;   o += align_up((size_t)(kK1Blocks * kK1ListCap + kK1Blocks) * 4, 256);  // sample tail lists
  L.off_cval = o; o += align_up((size_t)L.nb * tile * 4, 256);
  L.off_cidx = o; o += align_up((size_t)L.nb * tile * 4, 256);
  L.total = o;
  return L;
}

// ----------------------------------------------------------------------------
// key / value sources
// ----------------------------------------------------------------------------
template <int MODE, bool XH>
struct Src {
  const float* __restrict__ x;
  const float* __restrict__ xh;
  uint64_t seed;
  CHOCO_DEV float val(int64_t i) const { return XH ? x[i] - xh[i] : x[i]; }
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
  uint32_t scratch[24];
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

template <int MODE, bool XH>
__global__ __launch_bounds__(kExactThreads) void topk_exact_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, int64_t k, uint64_t seed,
    float scale, float* __restrict__ out_val, int32_t* __restrict__ out_idx, int64_t idx_base) {
  __shared__ ExactSmem sm;
  Src<MODE, XH> src{x, xh, seed};
  block_topk_exact(src, n, k, scale, out_val, out_idx, idx_base, sm);
}

// Segmented: plan rows {off, len, k, out_off}; one workgroup per segment that
// is not routed to the pipeline.
CHOCO_DEV bool seg_uses_pipeline(int64_t off, int64_t len);

template <bool XH>
__global__ __launch_bounds__(kExactThreads) void topk_segmented_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, const int64_t* __restrict__ plan,
    int32_t nseg, float* __restrict__ out_val, int32_t* __restrict__ out_idx) {
  __shared__ ExactSmem sm;
  const int s = blockIdx.x;
  if (s >= nseg) return;
  const int64_t off = plan[4 * s + 0], len = plan[4 * s + 1], k = plan[4 * s + 2], oo = plan[4 * s + 3];
  if (seg_uses_pipeline(off, len) || len == 0) return;
  Src<kData, XH> src{x + off, XH ? xh + off : nullptr, 0};
  block_topk_exact(src, len, k, 1.0f, out_val + oo, out_idx + oo, off, sm);
}

// ----------------------------------------------------------------------------
// K1: sample -> (s_lo, s_hi, shift)
//
// 64 workgroups each take 1024 samples (4 contiguous 256-element chunks spread
// over the buffer).  A workgroup keeps only its local tail -- the keys in the
// coarse (key>>20) bins that hold its top ~4x(expected share) samples -- in a
// global list; the last workgroup (agent-scope ticket) radix-selects the
// R_lo-th / R_hi-th largest keys of the union exactly.  Truncating a list can
// only lower those order statistics, i.e. make s_lo more conservative.
// ----------------------------------------------------------------------------
CHOCO_DEV void write_params(TopkCtrl* ctrl, uint32_t s_lo, uint64_t s_hi_est) {
  uint64_t width = s_hi_est > s_lo ? s_hi_est - s_lo : 1;
  uint32_t shift = 0;
  while ((63ull << shift) < width) ++shift;
  uint64_t s_hi = (uint64_t)s_lo + (63ull << shift);
  if (s_hi > 0xFFFFFFFFull) s_hi = 0xFFFFFFFFull;
  ctrl->s_lo = s_lo;
  ctrl->s_hi = (uint32_t)s_hi;
  ctrl->shift = shift;
}

// rank-th largest (1-based) of keys[0..u) held in LDS; 4 rounds of 8-bit digits.
CHOCO_DEV uint32_t lds_select_kth(const uint32_t* keys, uint32_t u, uint32_t rank, uint32_t* hist, uint32_t* bc) {
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  uint32_t prefix = 0, maskhi = 0, krem = rank;
  const int shs[4] = {23, 15, 7, 0};
  const int wds[4] = {8, 8, 8, 7};
  for (int rd = 0; rd < 4; ++rd) {
    const int sh = shs[rd];
    const uint32_t dmask = (1u << wds[rd]) - 1u;
    for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (uint32_t j = tid; j < u; j += blockDim.x) {
      const uint32_t key = keys[j];
      if ((key & maskhi) == prefix) atomicAdd(&hist[(key >> sh) & dmask], 1u);
    }
    __syncthreads();
    if (w == 0) {
      const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
      const uint32_t loc = h0 + h1 + h2 + h3;
      const uint32_t rv = __shfl(loc, 63 - lane);
      const uint32_t inc = wave_incl_scan(rv);
      const uint32_t suf_incl = __shfl(inc, 63 - lane);
      const uint32_t above = suf_incl - loc;
      if (above < krem && krem <= suf_incl) {
        uint32_t acc = above;
        const uint32_t hs[4] = {h0, h1, h2, h3};
        for (int t = 3; t >= 0; --t) {
          if (acc + hs[t] >= krem) { bc[0] = 4 * lane + t; bc[1] = krem - acc; break; }
          acc += hs[t];
        }
      }
    }
    __syncthreads();
    prefix |= bc[0] << sh;
    maskhi |= dmask << sh;
    krem = bc[1];
    __syncthreads();
  }
  return prefix;
}

struct SampleSmem {
  uint32_t hist[2048];
  uint32_t keys[kK1Blocks * kK1ListCap];
  uint32_t scratch[24];
  uint32_t bc[4];
  uint32_t flag;
};

template <bool XH>
__global__ __launch_bounds__(kK1Threads) void topk_sample_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, int64_t k,
    TopkCtrl* __restrict__ ctrl, uint32_t* __restrict__ lists) {
  __shared__ SampleSmem sm;
  uint32_t* __restrict__ counts = lists + kK1Blocks * kK1ListCap;
  const int tid = threadIdx.x;
  for (int i = tid; i < 2048; i += kK1Threads) sm.hist[i] = 0;
  // this thread's 4 samples: float4 s of chunk s/64 (64 float4 per 256-element chunk)
  constexpr int nchunk = kSampleN / kSampleChunk;
  const int64_t stride4 = ((n - kSampleChunk) / (nchunk - 1)) >> 2;
  const int s = blockIdx.x * kK1Threads + tid;
  const int64_t q = (int64_t)(s / 64) * stride4 + (s % 64);
  float4 v = reinterpret_cast<const float4*>(x)[q];
  if (XH) {
    const float4 h = reinterpret_cast<const float4*>(xh)[q];
    v.x -= h.x; v.y -= h.y; v.z -= h.z; v.w -= h.w;
  }
  const uint32_t kk[4] = {fkey(v.x), fkey(v.y), fkey(v.z), fkey(v.w)};
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 4; ++c) atomicAdd(&sm.hist[kk[c] >> 20], 1u);
  __syncthreads();
  // local cutoff: highest coarse bin whose suffix count reaches m_b
  const double eb = (double)k / (double)n * (double)(kK1Threads * 4);
  const uint32_t m_b = (uint32_t)fmin(4.0 * eb + 16.0, (double)(kK1Threads * 4));
  {
    uint32_t local = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) local += sm.hist[tid * 8 + j];
    uint32_t total;
    const uint32_t pre = block_excl_scan(local, sm.scratch, &total);
    const uint32_t above = total - pre - local;
    if (above < m_b && m_b <= above + local) {
      uint32_t acc = above;
      for (int j = 7; j >= 0; --j) {
        acc += sm.hist[tid * 8 + j];
        if (acc >= m_b) { sm.bc[0] = (uint32_t)(tid * 8 + j); break; }
      }
    }
    __syncthreads();
  }
  const uint32_t cut = sm.bc[0];
  uint32_t mine = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) mine += (kk[c] >> 20) >= cut;
  uint32_t tot;
  uint32_t pos = block_excl_scan(mine, sm.scratch, &tot);
  uint32_t* __restrict__ my = lists + blockIdx.x * kK1ListCap;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if ((kk[c] >> 20) >= cut) {
      if (pos < kK1ListCap) my[pos] = kk[c];
      ++pos;
    }
  }
  if (tid == 0) counts[blockIdx.x] = min(tot, (uint32_t)kK1ListCap);
  if (!last_block_ticket(&ctrl->k1_ticket, gridDim.x, &sm.flag)) return;

  // ---- last workgroup: exact order statistics of the union
  // all counts in parallel, then one independent load per key slot
  const uint32_t myc = tid < kK1Blocks ? counts[tid] : 0u;
  uint32_t u;
  const uint32_t mystart = block_excl_scan(myc, sm.scratch, &u);
  {
    // list starts in LDS (hist reused), then key slot p -> (list, offset) by binary search;
    // G unconditional loads per thread in flight (clamped slot when p >= u)
    if (tid < kK1Blocks) sm.hist[tid] = mystart;
    __syncthreads();
    constexpr int G = 16;
    for (uint32_t base = 0; base < u; base += G * kK1Threads) {
      uint32_t v[G];
      int dst[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const uint32_t p = base + (uint32_t)g * kK1Threads + tid;
        const uint32_t pc = p < u ? p : 0u;
        int lo = 0, hi = kK1Blocks - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (sm.hist[mid] <= pc) lo = mid; else hi = mid - 1;
        }
        v[g] = lists[lo * kK1ListCap + (pc - sm.hist[lo])];
        dst[g] = p < u ? (int)p : -1;
      }
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (dst[g] >= 0) sm.keys[dst[g]] = v[g];
    }
  }
  for (int i = tid; i < kNRep * kNBucket; i += kK1Threads) (&ctrl->G[0][0])[i] = 0;
  __syncthreads();
  const double m = (double)kSampleN;
  const double e = (double)k / (double)n * m;
  const double sd = sqrt(e);
  const double rlo_d = ceil(e + 6.0 * sd + 4.0);
  const double rhi_d = floor(e - 6.0 * sd - 4.0);
  uint32_t s_lo = 0;
  if (rlo_d <= (double)u) s_lo = lds_select_kth(sm.keys, u, (uint32_t)rlo_d, sm.hist, sm.bc);
  uint64_t s_hi_est = 0x80000000ull;  // above every key: nothing is "sure"
  if (rhi_d >= 1.0 && rhi_d <= (double)u) s_hi_est = (uint64_t)lds_select_kth(sm.keys, u, (uint32_t)rhi_d, sm.hist, sm.bc) + 1;
  if (tid == 0) {
    ctrl->overflow = 0;
    write_params(ctrl, s_lo, s_hi_est);
    __hip_atomic_store(&ctrl->k1_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Random-k: keys are uniform on [0, 2^31); thresholds from the binomial tails.
__global__ void topk_set_params_kernel(TopkCtrl* __restrict__ ctrl, uint32_t s_lo, uint64_t s_hi_est) {
  for (int i = threadIdx.x; i < kNRep * kNBucket; i += blockDim.x) (&ctrl->G[0][0])[i] = 0;
  if (threadIdx.x == 0) { ctrl->overflow = 0; write_params(ctrl, s_lo, s_hi_est); }
}

// ----------------------------------------------------------------------------
// K2: persistent streaming candidate compaction
// ----------------------------------------------------------------------------
struct StreamSmem {
  float sv[kK2Waves][kStage];
  uint32_t si[kK2Waves][kStage];
  uint32_t maybe[kK2Waves][kMaybeCap];
  uint32_t hist[kNBucket];
  uint32_t cur[kNBucket];
  uint32_t cnt[kK2Waves];
  uint32_t mcnt[kK2Waves];
};

// Unconditional (branch-free) float4 loads of kK2Unroll rows: keeps the
// compiler's vmcnt accounting exact so the prefetch stays in flight.
template <bool XH>
CHOCO_DEV void load_rows_full(const float* __restrict__ x, const float* __restrict__ xh, int64_t base, int lane,
                              float4 (&r)[kK2Unroll]) {
#pragma unroll
  for (int u = 0; u < kK2Unroll; ++u) r[u] = *reinterpret_cast<const float4*>(x + base + u * 256 + 4 * lane);
  if (XH) {
#pragma unroll
    for (int u = 0; u < kK2Unroll; ++u) {
      const float4 h = *reinterpret_cast<const float4*>(xh + base + u * 256 + 4 * lane);
      r[u].x -= h.x; r[u].y -= h.y; r[u].z -= h.z; r[u].w -= h.w;
    }
  }
}

// Per-wave compaction state (all wave-uniform).
struct WaveAcc {
  uint32_t flushed, staged, mcount;
};

// Flush exactly 256 staged candidates as 4 coalesced 256-B stores per array,
// then move the (< 256) remainder to the front of the stage.
CHOCO_DEV void flush256(StreamSmem& sm, int w, int lane, WaveAcc& a, float* __restrict__ ov,
                        uint32_t* __restrict__ oi) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float fv[4];
  uint32_t fi[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    fv[q] = sm.sv[w][q * 64 + lane];
    fi[q] = sm.si[w][q * 64 + lane];
  }
  const uint32_t rem = a.staged - 256;
  float rv[4];
  uint32_t ri[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t j = q * 64 + lane;
    rv[q] = j < rem ? sm.sv[w][256 + j] : 0.f;
    ri[q] = j < rem ? sm.si[w][256 + j] : 0u;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t j = q * 64 + lane;
    if (j < rem) {
      sm.sv[w][j] = rv[q];
      sm.si[w][j] = ri[q];
    }
    ov[a.flushed + j] = fv[q];
    oi[a.flushed + j] = fi[q];
  }
  a.flushed += 256;
  a.staged = rem;
}

// One float4 row per lane (256 elements per wave): ballot candidates into the stage.
template <int MODE, bool XH, bool GUARD>
CHOCO_DEV void process_row(const Src<MODE, XH>& src, const float4 v4, int64_t i, int64_t wend, uint32_t s_lo,
                           uint32_t s_hi, StreamSmem& sm, int w, int lane, WaveAcc& a, float* __restrict__ ov,
                           uint32_t* __restrict__ oi) {
  const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
  uint32_t kk[4];
  uint32_t cflags = 0, mflags = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const bool valid = !GUARD || i + c < wend;
    const uint32_t key = MODE == kData ? fkey(vv[c]) : (valid ? src.key_of(i + c, 0.f) : 0u);
    kk[c] = key;
    const bool cand = valid && key >= s_lo;
    cflags |= (cand ? 1u : 0u) << c;
    mflags |= ((cand && key < s_hi) ? 1u : 0u) << c;
  }
  const uint32_t cn = __builtin_popcount(cflags);
  const uint64_t b0 = ballot(cn & 1u), b1 = ballot(cn & 2u), b2 = ballot(cn & 4u);
  if ((b0 | b1 | b2) == 0ull) return;  // wave-uniform: no candidate in this row
  uint32_t pos = a.staged + mask_prefix(b0) + 2u * mask_prefix(b1) + 4u * mask_prefix(b2);
  a.staged += (uint32_t)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (cflags & (1u << c)) {
      sm.sv[w][pos] = MODE == kData ? vv[c] : src.val(i + c);
      sm.si[w][pos] = (uint32_t)(i + c);
      ++pos;
    }
  }
  if (ballot(mflags != 0u)) {
    const uint32_t mn = __builtin_popcount(mflags);
    const uint64_t m0 = ballot(mn & 1u), m1 = ballot(mn & 2u), m2 = ballot(mn & 4u);
    uint32_t mpos = a.mcount + mask_prefix(m0) + 2u * mask_prefix(m1) + 4u * mask_prefix(m2);
    a.mcount += (uint32_t)(__popcll(m0) + 2 * __popcll(m1) + 4 * __popcll(m2));
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (mflags & (1u << c)) {
        if (mpos < kMaybeCap) sm.maybe[w][mpos] = kk[c];
        ++mpos;
      }
    }
  }
  if (a.staged >= 256) flush256(sm, w, lane, a, ov, oi);
}

template <int MODE, bool XH>
__global__ __launch_bounds__(kK2Threads) void topk_stream_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, uint32_t tile, uint32_t nb,
    uint64_t seed, TopkCtrl* __restrict__ ctrl, uint32_t* __restrict__ cum_tab,
    uint32_t* __restrict__ cntw, uint32_t* __restrict__ side, float* __restrict__ cval,
    uint32_t* __restrict__ cidx) {
  __shared__ StreamSmem sm;
  const uint32_t s_lo = ctrl->s_lo, s_hi = ctrl->s_hi, shift = ctrl->shift;
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  const int64_t wlen = tile / kK2Waves;
  constexpr int64_t kStep = 256 * kK2Unroll;
  Src<MODE, XH> src{x, xh, seed};

  for (int64_t b = blockIdx.x; b < (int64_t)nb; b += gridDim.x) {
    const int64_t wbeg = b * tile + w * wlen;
    const int64_t wend = min(wbeg + wlen, n);
    float* __restrict__ ov = cval + wbeg;
    uint32_t* __restrict__ oi = cidx + wbeg;
    WaveAcc a{0u, 0u, 0u};
    const int64_t full_end = wend > wbeg ? wbeg + (wend - wbeg) / kStep * kStep : wbeg;

    // main loop: whole kStep blocks, double-buffered unconditional loads
    if (full_end > wbeg) {
      float4 A[kK2Unroll];
      if (MODE == kData) load_rows_full<XH>(x, xh, wbeg, lane, A);
      for (int64_t base = wbeg; base < full_end; base += kStep) {
        float4 B[kK2Unroll];
        if (MODE == kData) {
          const int64_t nxt = base + kStep < full_end ? base + kStep : base;  // clamp: harmless reload
          load_rows_full<XH>(x, xh, nxt, lane, B);
        }
#pragma unroll
        for (int u = 0; u < kK2Unroll; ++u)
          process_row<MODE, XH, false>(src, MODE == kData ? A[u] : make_float4(0.f, 0.f, 0.f, 0.f),
                                       base + u * 256 + 4 * lane, wend, s_lo, s_hi, sm, w, lane, a, ov, oi);
        if (MODE == kData) {
#pragma unroll
          for (int u = 0; u < kK2Unroll; ++u) A[u] = B[u];
        }
      }
    }
    // tail (< kStep elements): guarded loads
    for (int64_t base = full_end; base < wend; base += 256) {
      const int64_t i = base + 4 * lane;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (MODE == kData) {
        float t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) t[c] = (i + c < wend) ? src.val(i + c) : 0.f;
        v = make_float4(t[0], t[1], t[2], t[3]);
      }
      process_row<MODE, XH, true>(src, v, i, wend, s_lo, s_hi, sm, w, lane, a, ov, oi);
    }
    // final partial flush (< 256 entries)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t j = q * 64 + lane;
      if (j < a.staged) {
        ov[a.flushed + j] = sm.sv[w][j];
        oi[a.flushed + j] = sm.si[w][j];
      }
    }
    const uint32_t flushed = a.flushed + a.staged;
    const uint32_t mcount = a.mcount;

    // ---- end of tile: bucket counts, side list, totals
    if (lane == 0) {
      sm.cnt[w] = flushed;
      sm.mcnt[w] = mcount;
      if (mcount > kMaybeCap) atomicOr(&ctrl->overflow, 1u);
    }
    if (threadIdx.x < kNBucket) sm.hist[threadIdx.x] = 0;
    __syncthreads();
    {
      const uint32_t mc = min(sm.mcnt[w], (uint32_t)kMaybeCap);
      for (uint32_t j = lane; j < mc; j += 64) atomicAdd(&sm.hist[(sm.maybe[w][j] - s_lo) >> shift], 1u);
    }
    uint32_t csum = 0, msum = 0;
#pragma unroll
    for (int ww = 0; ww < kK2Waves; ++ww) {
      csum += sm.cnt[ww];
      msum += min(sm.mcnt[ww], (uint32_t)kMaybeCap);
    }
    __syncthreads();
    if (w == 0) {
      // bucket 63 = sure; cum[j] = sum_{i >= j} cnt[i]
      const uint32_t c = (lane == 63) ? (csum - msum) : sm.hist[lane];
      const uint32_t rv = __shfl(c, 63 - lane);
      const uint32_t inc = wave_incl_scan(rv);
      const uint32_t cum = __shfl(inc, 63 - lane);
      cum_tab[(int64_t)lane * nb + b] = cum;
      atomicAdd(&ctrl->G[b & (kNRep - 1)][lane], cum);
      const uint32_t cum_next = __shfl_down(cum, 1);
      const uint32_t sure = __shfl(cum, 63);
      if (lane < 63) sm.cur[lane] = cum_next - sure;   // counting-sort cursor of bucket `lane`
      if (lane < kK2Waves) cntw[b * kK2Waves + lane] = sm.cnt[lane];
    }
    __syncthreads();
    {
      uint32_t* __restrict__ sd = side + b * kSideCap;
      const uint32_t mc = min(sm.mcnt[w], (uint32_t)kMaybeCap);
      for (uint32_t j = lane; j < mc; j += 64) {
        const uint32_t key = sm.maybe[w][j];
        const uint32_t p = atomicAdd(&sm.cur[(key - s_lo) >> shift], 1u);
        sd[p] = key;
      }
    }
    __syncthreads();  // LDS is reused by the next tile
  }
}

// ----------------------------------------------------------------------------
// K3: exact threshold, tie quota and per-tile output offsets (one workgroup)
// ----------------------------------------------------------------------------
struct SelSmem {
  uint32_t keys[kMCap];
  uint32_t A[kNbMax + 1];   // key start per tile (exclusive scan of bucket-j* counts)
  uint32_t Bv[kNbMax];      // side offset of bucket j*, later #keys > T in bucket j*
  uint32_t Cv[kNbMax];      // #candidates in buckets > j* (incl. sure)
  uint32_t Dv[kNbMax];      // #keys == T
  uint32_t G[kNBucket];
  uint32_t hist[256];
  uint32_t scratch[24];
  uint32_t bc[8];
};

template <int MODE, bool XH>
__global__ __launch_bounds__(kK3Threads) void topk_select_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, int64_t k, uint32_t nb,
    uint64_t seed, float scale, TopkCtrl* __restrict__ ctrl, const uint32_t* __restrict__ cum_tab,
    const uint32_t* __restrict__ side, uint32_t* __restrict__ tile_info, float* __restrict__ out_val,
    int32_t* __restrict__ out_idx, int64_t idx_base) {
  __shared__ SelSmem fs;
  __shared__ ExactSmem es;
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint32_t s_lo = ctrl->s_lo, shift = ctrl->shift;
  uint32_t* __restrict__ tile_off = tile_info;
  uint32_t* __restrict__ tile_tieb = tile_info + nb;
  uint32_t* __restrict__ tile_mode = tile_info + 2 * nb;

  if (tid < kNBucket) {
    uint32_t g = 0;
#pragma unroll
    for (int r = 0; r < kNRep; ++r) g += ctrl->G[r][tid];
    fs.G[tid] = g;
  }
  __syncthreads();
  // j* = max{ j <= 62 : G[j] >= k }
  bool fallback = ctrl->overflow != 0 || fs.G[0] < (uint32_t)k || fs.G[63] >= (uint32_t)k;
  uint32_t jstar = 0;
  if (!fallback) {
    for (int j = 62; j >= 0; --j)
      if (fs.G[j] >= (uint32_t)k) { jstar = (uint32_t)j; break; }
    if (fs.G[jstar] - fs.G[jstar + 1] > (uint32_t)kMCap) fallback = true;
  }
  if (fallback) {
    Src<MODE, XH> src{x, xh, seed};
    if (tid == 0) ctrl->fallback = 1u;
    block_topk_exact(src, n, k, scale, out_val, out_idx, idx_base, es);
    return;
  }
  const uint32_t rank_in = (uint32_t)k - fs.G[jstar + 1];  // 1 <= rank_in <= M

  // per tile: bucket-j* count, side offset, count above bucket j*
  const int per = (nb + kK3Threads - 1) / kK3Threads;
  const int b0 = tid * per;
  uint32_t local = 0;
  {
    constexpr int PMAX = (kNbMax + kK3Threads - 1) / kK3Threads;
    uint32_t a[PMAX], c[PMAX], s[PMAX];
#pragma unroll
    for (int q = 0; q < PMAX; ++q) {  // unconditional (clamped) loads: all in flight together
      const int bq = min(b0 + q, (int)nb - 1);
      a[q] = cum_tab[(int64_t)jstar * nb + bq];
      c[q] = cum_tab[(int64_t)(jstar + 1) * nb + bq];
      s[q] = cum_tab[(int64_t)63 * nb + bq];
    }
#pragma unroll
    for (int q = 0; q < PMAX; ++q) {
      const int b = b0 + q;
      if (q < per && b < (int)nb) {
        fs.A[b] = a[q] - c[q];   // temporarily: count
        fs.Bv[b] = c[q] - s[q];  // side offset of bucket j*
        fs.Cv[b] = c[q];
        local += a[q] - c[q];
      }
    }
  }
  uint32_t M;
  uint32_t pre = block_excl_scan(local, fs.scratch, &M);
  for (int q = 0; q < per; ++q) {
    const int b = b0 + q;
    if (b >= (int)nb) break;
    const uint32_t cnt = fs.A[b];
    fs.A[b] = pre;
    pre += cnt;
  }
  if (tid == 0) fs.A[nb] = M;
  __syncthreads();
  // gather bucket-j* keys in tile order: one independent load per key slot
  // (tile of slot p found by binary search over the LDS prefix array A)
  {
    constexpr int G = 8;
    uint32_t v[G];
    int dst[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t p = tid + (uint32_t)g * kK3Threads;
      const uint32_t pc = p < M ? p : 0u;  // clamped: the load below is unconditional
      int lo = 0, hi = (int)nb - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (fs.A[mid] <= pc) lo = mid; else hi = mid - 1;
      }
      v[g] = side[(int64_t)lo * kSideCap + fs.Bv[lo] + (pc - fs.A[lo])];
      dst[g] = p < M ? (int)p : -1;
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (dst[g] >= 0) fs.keys[dst[g]] = v[g];
    for (uint32_t p = tid + G * kK3Threads; p < M; p += kK3Threads) {  // M > 8K: rare
      int lo = 0, hi = (int)nb - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (fs.A[mid] <= p) lo = mid; else hi = mid - 1;
      }
      fs.keys[p] = side[(int64_t)lo * kSideCap + fs.Bv[lo] + (p - fs.A[lo])];
    }
  }
  __syncthreads();
  // radix select inside the bucket: rel = key - base_j in [0, 2^shift), 8-bit digits
  const uint32_t base_j = s_lo + (jstar << shift);
  uint32_t prefix = 0, krem = rank_in;
  int sh = (int)shift;
  while (sh > 0) {
    const int dsh = sh > 8 ? sh - 8 : 0;
    const uint32_t dmask = (1u << (sh - dsh)) - 1u;
    if (tid < 256) fs.hist[tid] = 0;
    __syncthreads();
    for (uint32_t j = tid; j < M; j += kK3Threads) {
      const uint32_t rel = fs.keys[j] - base_j;
      if ((rel >> sh) == (prefix >> sh)) atomicAdd(&fs.hist[(rel >> dsh) & dmask], 1u);
    }
    __syncthreads();
    if (w == 0) {
      const uint32_t h0 = fs.hist[4 * lane], h1 = fs.hist[4 * lane + 1], h2 = fs.hist[4 * lane + 2],
                     h3 = fs.hist[4 * lane + 3];
      const uint32_t loc = h0 + h1 + h2 + h3;
      const uint32_t rv = __shfl(loc, 63 - lane);
      const uint32_t inc = wave_incl_scan(rv);
      const uint32_t suf_incl = __shfl(inc, 63 - lane);  // bins >= 4*lane
      const uint32_t above = suf_incl - loc;
      if (above < krem && krem <= suf_incl) {
        uint32_t acc = above;
        const uint32_t hs[4] = {h0, h1, h2, h3};
        for (int t = 3; t >= 0; --t) {
          if (acc + hs[t] >= krem) { fs.bc[0] = 4 * lane + t; fs.bc[1] = krem - acc; break; }
          acc += hs[t];
        }
      }
    }
    __syncthreads();
    prefix |= fs.bc[0] << dsh;
    krem = fs.bc[1];
    sh = dsh;
    __syncthreads();
  }
  const uint32_t T = base_j + prefix;
  const uint32_t r = krem;  // ties at T to take (>= 1)

  uint32_t eq_local = 0;
  for (int q = 0; q < per; ++q) {
    const int b = b0 + q;
    if (b >= (int)nb) break;
    uint32_t eq = 0, gt = 0;
    for (uint32_t j = fs.A[b]; j < fs.A[b + 1]; ++j) {
      const uint32_t key = fs.keys[j];
      gt += key > T;
      eq += key == T;
    }
    fs.Bv[b] = gt;
    fs.Dv[b] = eq;
    eq_local += eq;
  }
  uint32_t tie_total;
  uint32_t tb = block_excl_scan(eq_local, fs.scratch, &tie_total);
  uint32_t sel_local = 0;
  for (int q = 0; q < per; ++q) {
    const int b = b0 + q;
    if (b >= (int)nb) break;
    const uint32_t eq = fs.Dv[b];
    const uint32_t take = tb >= r ? 0u : min(eq, r - tb);
    const uint32_t sel = fs.Cv[b] + fs.Bv[b] + take;
    tile_tieb[b] = tb;
    tile_mode[b] = take == 0 ? kTakeNone : (take == eq ? kTakeAll : kTakePartial);
    fs.Bv[b] = sel;
    tb += eq;
    sel_local += sel;
  }
  uint32_t sel_total;
  uint32_t sel_pre = block_excl_scan(sel_local, fs.scratch, &sel_total);
  for (int q = 0; q < per; ++q) {
    const int b = b0 + q;
    if (b >= (int)nb) break;
    tile_off[b] = sel_pre;
    sel_pre += fs.Bv[b];
  }
  if (tid == 0) {
    ctrl->T = T;
    ctrl->r = r;
    ctrl->fallback = 0u;
  }
}

// ----------------------------------------------------------------------------
// K4: ordered compaction, one workgroup per tile
// ----------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kK4Threads) void topk_emit_kernel(
    uint32_t tile, uint32_t nb, uint64_t seed, float scale, const TopkCtrl* __restrict__ ctrl,
    const uint32_t* __restrict__ cntw, const uint32_t* __restrict__ tile_info, const float* __restrict__ cval,
    const uint32_t* __restrict__ cidx, float* __restrict__ out_val, int32_t* __restrict__ out_idx,
    int64_t idx_base) {
  __shared__ uint32_t scratch[24];
  const int64_t b = blockIdx.x;
  // every control word is independent: issue all loads before the first use
  const uint32_t fallback = ctrl->fallback, T = ctrl->T, r = ctrl->r;
  uint32_t out = tile_info[b];
  uint32_t tie_run = tile_info[nb + b];
  const uint32_t mode = tile_info[2 * nb + b];
  const uint4 cw4 = *reinterpret_cast<const uint4*>(cntw + b * kK2Waves);
  const uint32_t c0 = cw4.x, c1 = cw4.y, c2 = cw4.z, c3 = cw4.w;
  if (fallback) return;
  const uint32_t e1 = c0, e2 = e1 + c1, e3 = e2 + c2, tot = e3 + c3;
  const int64_t wlen = tile / kK2Waves;
  const int64_t tb = b * tile;
  for (uint32_t p0 = 0; p0 < tot; p0 += kK4Threads) {
    const uint32_t p = p0 + threadIdx.x;
    const bool valid = p < tot;
    float v = 0.f;
    uint32_t idx = 0, key = 0;
    if (valid) {
      // position p of the tile's concatenated wave runs
      const int run = (p >= e1) + (p >= e2) + (p >= e3);
      const uint32_t start = run == 0 ? 0u : (run == 1 ? e1 : (run == 2 ? e2 : e3));
      const int64_t a = tb + run * wlen + (p - start);
      v = cval[a];
      idx = cidx[a];
      key = MODE == kData ? fkey(v) : (rank_hash(seed, idx) >> 1);
    }
    const bool gt = valid && key > T;
    const bool eq = valid && key == T;
    bool sel;
    if (mode == kTakePartial) {
      uint32_t neq;
      const uint32_t rank = tie_run + block_excl_scan(eq ? 1u : 0u, scratch, &neq);
      sel = gt || (eq && rank < r);
      tie_run += neq;
    } else {
      sel = gt || (eq && mode == kTakeAll);
    }
    uint32_t nsel;
    const uint32_t pos = out + block_excl_scan(sel ? 1u : 0u, scratch, &nsel);
    if (sel) {
      out_val[pos] = v * scale;
      out_idx[pos] = (int32_t)((int64_t)idx + idx_base);
    }
    out += nsel;
  }
}

// ----------------------------------------------------------------------------
// host dispatch
// ----------------------------------------------------------------------------
constexpr int64_t kPipeMinSeg = 1 << 20;
CHOCO_DEV bool seg_uses_pipeline(int64_t off, int64_t len) {
  return len >= kPipeMinSeg && (off & 3) == 0;
}
static bool host_seg_uses_pipeline(int64_t off, int64_t len) {
  return len >= kPipeMinSeg && (off & 3) == 0;
}

size_t topk_ws_bytes(int64_t n) { return n > kSmallN ? topk_layout(n).total : 256; }

static int num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                   hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <int MODE, bool XH>
static int launch_topk(const float* x, const float* xh, int64_t n, int64_t k, uint64_t seed, float scale,
                       float* out_val, int32_t* out_idx, int64_t idx_base, void* ws, size_t ws_bytes,
                       hipStream_t st) {
  if (n <= kSmallN || k >= n) {
    hipLaunchKernelGGL((topk_exact_kernel<MODE, XH>), dim3(1), dim3(kExactThreads), 0, st, x, xh, n, k,
                       seed, scale, out_val, out_idx, idx_base);
    CHOCO_LAUNCHED("topk_exact_kernel");
    return CHOCO_OK;
  }
  const TopkLayout L = topk_layout(n);
  CHOCO_REQUIRE(ws != nullptr && ws_bytes >= L.total, "top-k workspace too small: need %zu bytes, got %zu",
                L.total, ws_bytes);
  char* base = static_cast<char*>(ws);
  TopkCtrl* ctrl = reinterpret_cast<TopkCtrl*>(base + L.off_ctrl);
  uint32_t* cum = reinterpret_cast<uint32_t*>(base + L.off_cum);
  uint32_t* cntw = reinterpret_cast<uint32_t*>(base + L.off_cntw);
  uint32_t* side = reinterpret_cast<uint32_t*>(base + L.off_side);
  uint32_t* tinfo = reinterpret_cast<uint32_t*>(base + L.off_tile);
  float* cval = reinterpret_cast<float*>(base + L.off_cval);
  uint32_t* cidx = reinterpret_cast<uint32_t*>(base + L.off_cidx);
  if (MODE == kData) {
    uint32_t* k1 = reinterpret_cast<uint32_t*>(base + L.off_k1);
    hipLaunchKernelGGL((topk_sample_kernel<XH>), dim3(kK1Blocks), dim3(kK1Threads), 0, st, x, xh, n, k, ctrl, k1);
    CHOCO_LAUNCHED("topk_sample_kernel");
  } else {
    // keys uniform on [0, 2^31): P(key >= t) = (2^31 - t) / 2^31
    const double nd = (double)n, kd = (double)k, sd = sqrt(kd);
    const double c_lo = std::min(nd, kd + 6.0 * sd + 16.0);
    const double c_hi = kd - 6.0 * sd - 16.0;
    const double two31 = 2147483648.0;
    uint32_t s_lo = (uint32_t)std::max(0.0, floor(two31 * (1.0 - c_lo / nd)));
    uint64_t s_hi_est = c_hi < 1.0 ? 0x80000000ull : (uint64_t)ceil(two31 * (1.0 - c_hi / nd));
    if (s_hi_est <= s_lo) s_hi_est = (uint64_t)s_lo + 1;
    hipLaunchKernelGGL(topk_set_params_kernel, dim3(1), dim3(256), 0, st, ctrl, s_lo, s_hi_est);
    CHOCO_LAUNCHED("topk_set_params_kernel");
  }
  const unsigned g2 = (unsigned)std::min<int64_t>(L.nb, (int64_t)num_cus() * kK2BlocksPerCU);
  profile_begin("topk_stream", st);
  hipLaunchKernelGGL((topk_stream_kernel<MODE, XH>), dim3(g2), dim3(kK2Threads), 0, st, x, xh, n, L.tile, L.nb,
                     seed, ctrl, cum, cntw, side, cval, cidx);
  profile_end("topk_stream", st);
  CHOCO_LAUNCHED("topk_stream_kernel");
  hipLaunchKernelGGL((topk_select_kernel<MODE, XH>), dim3(1), dim3(kK3Threads), 0, st, x, xh, n, k, L.nb, seed,
                     scale, ctrl, cum, side, tinfo, out_val, out_idx, idx_base);
  CHOCO_LAUNCHED("topk_select_kernel");
  hipLaunchKernelGGL((topk_emit_kernel<MODE>), dim3(L.nb), dim3(kK4Threads), 0, st, L.tile, L.nb, seed, scale,
                     ctrl, cntw, tinfo, cval, cidx, out_val, out_idx, idx_base);
  CHOCO_LAUNCHED("topk_emit_kernel");
  return CHOCO_OK;
}

template <int MODE>
static int dispatch_topk(const float* x, const float* xh, int64_t n, int64_t k, uint64_t seed, float scale,
                         float* out_val, int32_t* out_idx, int64_t idx_base, void* ws, size_t ws_bytes,
                         hipStream_t st) {
  CHOCO_REQUIRE(x != nullptr && out_val != nullptr && out_idx != nullptr, "null pointer argument");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n must be in [1, 2^31-1), got %lld", (long long)n);
  CHOCO_REQUIRE(k >= 1 && k <= n, "k must be in [1, n], got k=%lld n=%lld", (long long)k, (long long)n);
  if (n > kSmallN && k < n) {
    CHOCO_REQUIRE(aligned16(x) && (xh == nullptr || aligned16(xh)),
                  "x/xhat must be 16-byte aligned for n > %lld", (long long)kSmallN);
  }
  if (xh) return launch_topk<MODE, true>(x, xh, n, k, seed, scale, out_val, out_idx, idx_base, ws, ws_bytes, st);
  return launch_topk<MODE, false>(x, xh, n, k, seed, scale, out_val, out_idx, idx_base, ws, ws_bytes, st);
}

}  // namespace choco

using namespace choco;

CHOCO_API int64_t choco_topk_k(int64_t n, double ratio) {
  // identical IEEE-double expression to max(1, int(x_len * (1 - ratio)))
  double v = (double)n * (1.0 - ratio);
  int64_t k = (int64_t)v;  // int() truncates toward zero
  return k < 1 ? 1 : k;
}

CHOCO_API size_t choco_topk_workspace_size(int64_t n) { return topk_ws_bytes(n); }
CHOCO_API size_t choco_randk_workspace_size(int64_t n) { return topk_ws_bytes(n); }

CHOCO_API int choco_topk_compress(const float* x, const float* xhat, int64_t n, int64_t k, float* out_val,
                                  int32_t* out_idx, void* ws, size_t ws_bytes, void* stream) {
  return dispatch_topk<kData>(x, xhat, n, k, 0, 1.0f, out_val, out_idx, 0, ws, ws_bytes, as_stream(stream));
}

CHOCO_API int choco_randk_compress(const float* x, const float* xhat, int64_t n, int64_t k, uint64_t seed,
                                   int32_t is_biased, float* out_val, int32_t* out_idx, void* ws,
                                   size_t ws_bytes, void* stream) {
  const float scale = is_biased ? 1.0f : (float)((double)n / (double)k);
  return dispatch_topk<kHash>(x, xhat, n, k, seed, scale, out_val, out_idx, 0, ws, ws_bytes,
                              as_stream(stream));
}

CHOCO_API int64_t choco_topk_segmented_plan(const int64_t* seg_off_host, int32_t nseg, double ratio,
                                            int64_t* plan_host) {
  if (seg_off_host == nullptr || nseg <= 0) return (int64_t)fail(CHOCO_ERR_INVALID, "bad segment table");
  int64_t out = 0;
  for (int s = 0; s < nseg; ++s) {
    const int64_t off = seg_off_host[s], len = seg_off_host[s + 1] - seg_off_host[s];
    if (len <= 0) return (int64_t)fail(CHOCO_ERR_INVALID, "segment %d has length %lld", s, (long long)len);
    const int64_t k = choco_topk_k(len, ratio);
    if (plan_host) {
      plan_host[4 * s + 0] = off;
      plan_host[4 * s + 1] = len;
      plan_host[4 * s + 2] = k;
      plan_host[4 * s + 3] = out;
    }
    out += k;
  }
  return out;
}

CHOCO_API size_t choco_topk_segmented_workspace_size(const int64_t* plan_host, int32_t nseg) {
  size_t need = 256;
  for (int s = 0; s < nseg; ++s) {
    const int64_t off = plan_host[4 * s], len = plan_host[4 * s + 1];
    if (host_seg_uses_pipeline(off, len)) need = std::max(need, topk_ws_bytes(len));
  }
  return need;
}

CHOCO_API int choco_topk_compress_segmented(const float* x, const float* xhat, const int64_t* plan_dev,
                                            const int64_t* plan_host, int32_t nseg, float* out_val,
                                            int32_t* out_idx, void* ws, size_t ws_bytes, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(x && plan_dev && plan_host && out_val && out_idx && nseg > 0, "null pointer argument");
  CHOCO_REQUIRE(aligned16(x) && (xhat == nullptr || aligned16(xhat)), "x/xhat must be 16-byte aligned");
  const int64_t ntot = plan_host[4 * (nseg - 1)] + plan_host[4 * (nseg - 1) + 1];
  CHOCO_REQUIRE(ntot < (int64_t)INT32_MAX, "total length must be < 2^31");
  // every segment that is not pipelined: one workgroup each, one launch
  if (xhat)
    hipLaunchKernelGGL((topk_segmented_kernel<true>), dim3(nseg), dim3(kExactThreads), 0, st, x, xhat,
                       plan_dev, nseg, out_val, out_idx);
  else
    hipLaunchKernelGGL((topk_segmented_kernel<false>), dim3(nseg), dim3(kExactThreads), 0, st, x, xhat,
                       plan_dev, nseg, out_val, out_idx);
  CHOCO_LAUNCHED("topk_segmented_kernel");
  for (int s = 0; s < nseg; ++s) {
    const int64_t off = plan_host[4 * s], len = plan_host[4 * s + 1], k = plan_host[4 * s + 2],
                  oo = plan_host[4 * s + 3];
    if (!host_seg_uses_pipeline(off, len)) continue;
    int rc = dispatch_topk<kData>(x + off, xhat ? xhat + off : nullptr, len, k, 0, 1.0f, out_val + oo,
                                  out_idx + oo, off, ws, ws_bytes, st);
    if (rc) return rc;
  }
  return CHOCO_OK;
}
