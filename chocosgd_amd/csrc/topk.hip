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
//   K1 topk_sample  : 64 workgroups histogram a 64K-element strided sample and
//                     keep their local tails; the last one picks a candidate
//                     floor s_lo (#{key >= s_lo} >= k with a ~6 sigma margin)
//                     and a "sure" ceiling s_hi (#{key >= s_hi} < k).
//                     [s_lo, s_hi) is split into 255 key-buckets of width 2^shift.
//   K2 topk_stream  : one workgroup per tile (4 waves, each a contiguous range);
//                     per float4 row the wave ballots candidates (key >= s_lo)
//                     and appends (value, index) in index order to an LDS ring
//                     flushed to the wave's slot of the candidate buffer in
//                     256-B stores.  At the end of the tile the "maybe" keys
//                     (key < s_hi) are re-read, bucket-counted and counting-sorted
//                     into a per-tile side list; per-tile bucket suffix counts go
//                     to a [tile][256] table and to 16 replicated global totals.
//   K3 topk_select  : one workgroup finds the bucket j* holding the k-th key
//                     from the totals, copies every tile's bucket-j* keys (a few
//                     thousand) into LDS, radix-selects T and the tie quota r
//                     exactly and scans per-tile output offsets.
//   K4 topk_emit    : one workgroup per tile compacts the tile's candidates into
//                     the final ascending-index output.
//   If the sample's guess was off (too few candidates, T in the "sure" range,
//   bucket j* larger than LDS, or a side list overflowed), K3 runs an exact
//   single-workgroup radix select over the full input instead (correct, slow,
//   data-dependent only) and K4 exits.
// Small n (<= kSmallN) and every segment of the batched segmented path use
// the same exact radix select (block_topk_exact) in one workgroup.
#include "choco_common.h"

#include <math.h>
#include <algorithm>

namespace choco {

constexpr int kK2Threads = 1024;          // 16 waves, each a contiguous range of the tile
constexpr int kK2Waves = kK2Threads / 64;
// Diagnostic knob (tools/build_variants.py): tiles per launch.
#ifndef CHOCO_K2_TARGET  // one workgroup per CU (256 CUs): no two tiles compete on a CU
#define CHOCO_K2_TARGET 256
#endif
constexpr int kK2Unroll = 8;            // float4 rows per wave per load batch (8 KiB in flight)
constexpr int64_t kK2Target = CHOCO_K2_TARGET;
constexpr int64_t kTileQuant = (int64_t)kK2Waves * kK2Unroll * 256;   // 32768 elements
static_assert(kK2Target <= 2048, "K3 keeps at most two tiles per thread");
constexpr int64_t kChunk = 4096;        // elements a wave claims at a time (LDS counter)
static_assert(kTileQuant % kChunk == 0 && kChunk % (256 * kK2Unroll) == 0, "chunk geometry");
static_assert((int64_t(1) << 31) / kK2Target / kChunk <= 2 * 1024, "K4 scans <= 2 chunk counts per thread");
constexpr int kMaybeCap = 16384;        // maybe keys per tile kept in LDS (= side-list capacity)
constexpr int kNBucket = 256;           // 255 "maybe" buckets + 1 "sure"
constexpr int kNMaybe = kNBucket - 1;
constexpr int kNRep = 16;               // replicas of the global bucket totals
constexpr int kMCap = 16384;            // max keys of bucket j* selected in LDS
constexpr int kK3Threads = 1024;
constexpr int kK4Threads = 1024;
constexpr int kK1Blocks = 64;           // sample workgroups, 1024 samples each
constexpr int kK1Threads = 256;
constexpr int kSampleN = kK1Blocks * kK1Threads * 4;   // 65536
constexpr int kSampleChunk = 256;
constexpr int64_t kSmallN = 65536;
constexpr int kExactThreads = 1024;

// Diagnostic phase stamps (tools/stamps.py; never in the product build).
#ifndef CHOCO_STAMPS
#define CHOCO_STAMPS 0
#endif
#if CHOCO_STAMPS
constexpr int kStampSlots = 40960;
__device__ unsigned long long g_stamps[kStampSlots][4];
#define STAMP(slot, j)                                                      \
  do {                                                                      \
    if (threadIdx.x == 0) g_stamps[(slot)][(j)] = wall_clock64();           \
  } while (0)
#else
#define STAMP(slot, j) \
  do {                 \
  } while (0)
#endif

enum SrcMode { kData = 0, kHash = 1 };
enum TileMode { kTakeNone = 0, kTakeAll = 1, kTakePartial = 2 };

struct TopkCtrl {
  uint32_t s_lo, s_hi, shift, overflow;          // K1 -> K2
  uint32_t T, r, fallback, k1_ticket;            // K3 -> K4; K1b's self-resetting ticket
  uint32_t pad[8];
  uint32_t G[kNRep][kNBucket];                   // replicated bucket suffix totals
};

struct TopkLayout {
  int64_t n;
  uint32_t tile, nb, side_cap;
  size_t off_ctrl, off_cum, off_cntw, off_side, off_tile, off_k1, off_cval, off_cidx, total;
};

// Tile = ceil(n / kK2Target) rounded up to 32768 elements: one tile per CU, all
// resident at once (few tiles also keep K3's table reads short).  A tile's side
// list holds its "maybe" keys (kMaybeCap, LDS-staged): the sample's margin is
// ~12 sqrt(k/n / 65536) of the elements (0.5 % at k = 1 %, 1.5 % at k = 10 %,
// 3.3 % at k = 50 % -> 13K of a 390K-element tile).
static TopkLayout topk_layout(int64_t n) {
  TopkLayout L{};
  L.n = n;
  int64_t tile = (n + kK2Target - 1) / kK2Target;
  tile = std::max<int64_t>(kTileQuant, (tile + kTileQuant - 1) / kTileQuant * kTileQuant);
  L.tile = (uint32_t)tile;
  L.nb = (uint32_t)((n + tile - 1) / tile);
  L.side_cap = (uint32_t)std::min<int64_t>(kMaybeCap, tile);
  size_t o = 0;
  L.off_ctrl = o;  o += align_up(sizeof(TopkCtrl), 256);
  L.off_cum = o;   o += align_up((size_t)L.nb * kNBucket * 4, 256);
  L.off_cntw = o;  o += align_up((size_t)L.nb * (tile / kChunk) * 4, 256);   // per-chunk candidate counts
  L.off_side = o;  o += align_up((size_t)L.nb * L.side_cap * 4, 256);
  L.off_tile = o;  o += align_up((size_t)L.nb * 3 * 4, 256);        // tile_off | tile_tieb | tile_mode
  L.off_k1 = o;    o += align_up((size_t)3 * 2048 * 4, 256);           // sample histograms (K1)
  L.off_cval = o;  o += align_up((size_t)L.nb * tile * 4, 256);
  L.off_cidx = o;  o += align_up((size_t)L.nb * tile * 4, 256);
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
// K1: sample -> (s_lo, s_hi, shift), two small kernels
//
// 64 workgroups read a 64K-element strided sample (4 contiguous 256-element
// chunks each).  K1a adds their coarse key histogram (key >> 20, 2048 bins) to
// a global one.  K1b: every workgroup scans it for the coarse bins holding the
// R_lo-th / R_hi-th largest sample keys, re-reads its samples and adds a fine
// histogram (bits 19..9) of the keys in those two bins; the last workgroup
// (fence-free ticket: the payload is atomics only) resolves both ranks to 512
// keys -- s_lo rounded down, s_hi rounded up -- and clears the histograms for
// the next call.  Both bounds are heuristics that K3 verifies (G[0] >= k,
// G[sure] < k); any k/n works.
// ----------------------------------------------------------------------------
CHOCO_DEV void write_params(TopkCtrl* ctrl, uint32_t s_lo, uint64_t s_hi_est) {
  const uint64_t width = s_hi_est > s_lo ? s_hi_est - s_lo : 1;
  uint32_t shift = 0;
  while (((uint64_t)kNMaybe << shift) < width) ++shift;
  uint64_t s_hi = (uint64_t)s_lo + ((uint64_t)kNMaybe << shift);
  if (s_hi > 0xFFFFFFFFull) s_hi = 0xFFFFFFFFull;
  ctrl->s_lo = s_lo;
  ctrl->s_hi = (uint32_t)s_hi;
  ctrl->shift = shift;
}

CHOCO_DEV uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
CHOCO_DEV void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0 of a workgroup: over a 256-bin LDS histogram (ascending value order),
// find the bin holding the rank-th largest entry; returns (bin, rank inside bin)
// via out[0], out[1].  Other waves must not call.
CHOCO_DEV void wave_find_bin(const uint32_t* hist, uint32_t rank, uint32_t* out) {
  const int lane = lane_id();
  const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
  const uint32_t loc = h0 + h1 + h2 + h3;
  const uint32_t rv = __shfl(loc, 63 - lane);
  const uint32_t inc = wave_incl_scan(rv);
  const uint32_t suf_incl = __shfl(inc, 63 - lane);  // entries in bins >= 4*lane
  const uint32_t above = suf_incl - loc;
  if (above < rank && rank <= suf_incl) {
    uint32_t acc = above;
    const uint32_t hs[4] = {h0, h1, h2, h3};
    for (int t = 3; t >= 0; --t) {
      if (acc + hs[t] >= rank) { out[0] = 4 * lane + t; out[1] = rank - acc; break; }
      acc += hs[t];
    }
  }
}

// Workgroup-wide: over hist[2048] in LDS (ascending value order), the bin holding
// the rank-th largest entry and the rank inside it -> out[0], out[1].  Every
// thread of the (kK1Threads) workgroup must call.
CHOCO_DEV void block_find_bin2048(const uint32_t* hist, uint32_t rank, uint32_t* scratch, uint32_t* out) {
  const int tid = threadIdx.x;
  constexpr int per = 2048 / kK1Threads;
  uint32_t hv[per];
  uint32_t local = 0;
#pragma unroll
  for (int j = 0; j < per; ++j) {
    hv[j] = hist[tid * per + j];
    local += hv[j];
  }
  uint32_t total;
  const uint32_t pre = block_excl_scan(local, scratch, &total);
  const uint32_t above = total - pre - local;  // entries in bins above my chunk
  if (above < rank && rank <= above + local) {
    uint32_t acc = above;
#pragma unroll
    for (int j = per - 1; j >= 0; --j) {
      if (acc < rank && rank <= acc + hv[j]) { out[0] = (uint32_t)(tid * per + j); out[1] = rank - acc; }
      acc += hv[j];
    }
  }
  __syncthreads();
}

struct SampleRanks {
  uint32_t lo, hi;  // 1-based ranks from the top; 0 = none
};

// Ranks of the candidate floor / sure ceiling in the 64K sample (~6 sigma margins).
CHOCO_DEV SampleRanks sample_ranks(int64_t n, int64_t k) {
  const double m = (double)kSampleN;
  const double e = (double)k / (double)n * m;
  const double sd = sqrt(e);
  const double rlo = ceil(e + 6.0 * sd + 4.0);
  const double rhi = floor(e - 6.0 * sd - 4.0);
  SampleRanks r;
  r.lo = rlo <= m ? (uint32_t)rlo : 0u;  // 0: every key is a candidate
  r.hi = rhi >= 1.0 ? (uint32_t)rhi : 0u;  // 0: no key is "sure"
  return r;
}

template <bool XH>
CHOCO_DEV void load_sample(const float* __restrict__ x, const float* __restrict__ xh, int64_t n, uint32_t kk[4]) {
  constexpr int nchunk = kSampleN / kSampleChunk;
  const int64_t stride4 = ((n - kSampleChunk) / (nchunk - 1)) >> 2;
  const int s = blockIdx.x * kK1Threads + threadIdx.x;
  const int64_t q = (int64_t)(s / 64) * stride4 + (s % 64);  // float4 s%64 of chunk s/64
  float4 v = reinterpret_cast<const float4*>(x)[q];
  if (XH) {
    const float4 h = reinterpret_cast<const float4*>(xh)[q];
    v.x -= h.x; v.y -= h.y; v.z -= h.z; v.w -= h.w;
  }
  kk[0] = fkey(v.x); kk[1] = fkey(v.y); kk[2] = fkey(v.z); kk[3] = fkey(v.w);
}

// K1a: global coarse histogram of the sample (hist = [coarse 2048 | fine lo 2048 | fine hi 2048]).
template <bool XH>
__global__ __launch_bounds__(kK1Threads) void topk_sample_hist_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[2048];
  const int tid = threadIdx.x;
  STAMP(blockIdx.x, 0);
  for (int i = tid; i < 2048; i += kK1Threads) h[i] = 0;
  uint32_t kk[4];
  load_sample<XH>(x, xh, n, kk);
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 4; ++c) atomicAdd(&h[kk[c] >> 20], 1u);
  __syncthreads();
  for (int i = tid; i < 2048; i += kK1Threads) {
    const uint32_t v = h[i];
    if (v) atomicAdd(&hist[i], v);
  }
  STAMP(blockIdx.x, 1);
}

struct BoundsSmem {
  uint32_t h[2048];
  uint32_t f[2][2048];
  uint32_t scratch[24];
  uint32_t bc[8];
  uint32_t flag;
};

// K1b: fine histograms inside the two coarse bins, then the bounds.
template <bool XH>
__global__ __launch_bounds__(kK1Threads) void topk_sample_bounds_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, int64_t k,
    TopkCtrl* __restrict__ ctrl, uint32_t* __restrict__ hist) {
  __shared__ BoundsSmem sm;
  const int tid = threadIdx.x;
  uint32_t* __restrict__ fine_lo = hist + 2048;
  uint32_t* __restrict__ fine_hi = hist + 4096;
  const SampleRanks R = sample_ranks(n, k);
  uint32_t kk[4];
  load_sample<XH>(x, xh, n, kk);
  {
    constexpr int per = 2048 / kK1Threads;
    uint32_t hv[per];
#pragma unroll
    for (int j = 0; j < per; ++j) hv[j] = hist[tid + j * kK1Threads];  // written by K1a
#pragma unroll
    for (int j = 0; j < per; ++j) sm.h[tid + j * kK1Threads] = hv[j];
  }
  if (tid < 8) sm.bc[tid] = 0;
  __syncthreads();
  if (R.lo) block_find_bin2048(sm.h, R.lo, sm.scratch, sm.bc);
  if (R.hi) block_find_bin2048(sm.h, R.hi, sm.scratch, sm.bc + 2);
  const uint32_t c_lo = sm.bc[0], c_hi = sm.bc[2];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (R.lo && (kk[c] >> 20) == c_lo) atomicAdd(&fine_lo[(kk[c] >> 9) & 2047u], 1u);
    if (R.hi && (kk[c] >> 20) == c_hi) atomicAdd(&fine_hi[(kk[c] >> 9) & 2047u], 1u);
  }
  STAMP(blockIdx.x, 2);
  const bool last = last_block_ticket_atomics(&ctrl->k1_ticket, gridDim.x, &sm.flag);
  STAMP(blockIdx.x, 3);
  if (!last) return;

  // ---- last workgroup: resolve both ranks inside their coarse bins (one load round)
  uint32_t s_lo = 0;
  uint64_t s_hi_est = 0x80000000ull;  // above every key: nothing is "sure"
  {
    constexpr int per = 2048 / kK1Threads;
    uint32_t fa[per], fb[per];
#pragma unroll
    for (int j = 0; j < per; ++j) {
      fa[j] = R.lo ? ld_agent(&fine_lo[tid + j * kK1Threads]) : 0u;
      fb[j] = R.hi ? ld_agent(&fine_hi[tid + j * kK1Threads]) : 0u;
    }
#pragma unroll
    for (int j = 0; j < per; ++j) {
      sm.f[0][tid + j * kK1Threads] = fa[j];
      sm.f[1][tid + j * kK1Threads] = fb[j];
    }
  }
  __syncthreads();
  if (R.lo) {
    block_find_bin2048(sm.f[0], sm.bc[1], sm.scratch, sm.bc + 4);
    s_lo = (c_lo << 20) | (sm.bc[4] << 9);                                  // rounded down
  }
  if (R.hi) {
    block_find_bin2048(sm.f[1], sm.bc[3], sm.scratch, sm.bc + 6);
    s_hi_est = (uint64_t)((c_hi << 20) | (sm.bc[6] << 9)) + 512u;            // rounded up
  }
  STAMP(64, 0);
  // clear the histograms and the bucket totals for K2 / the next call
  for (int i = tid; i < 3 * 2048; i += kK1Threads) hist[i] = 0;
  for (int i = tid; i < kNRep * kNBucket; i += kK1Threads) (&ctrl->G[0][0])[i] = 0;
  if (tid == 0) {
    ctrl->overflow = 0;
    write_params(ctrl, s_lo, s_hi_est);
    st_agent(&ctrl->k1_ticket, 0u);
  }
}

// Random-k: keys are uniform on [0, 2^31); thresholds from the binomial tails.
__global__ void topk_set_params_kernel(TopkCtrl* __restrict__ ctrl, uint32_t s_lo, uint64_t s_hi_est) {
  for (int i = threadIdx.x; i < kNRep * kNBucket; i += blockDim.x) (&ctrl->G[0][0])[i] = 0;
  if (threadIdx.x == 0) { ctrl->overflow = 0; write_params(ctrl, s_lo, s_hi_est); }
}

// ----------------------------------------------------------------------------
// K2: streaming candidate compaction, one 16-wave workgroup per tile, one per CU
//
// Measured (tools/probe_position.hip, probe_balance.hip): when two or more
// workgroups share a CU, the one dispatched first streams first and the last
// ones finish alone with few bytes in flight; with ONE workgroup per CU every
// workgroup finishes within ~10 % of the others.  LDS use (> 80 KiB) enforces
// that placement.  Inside the workgroup the CU's issue arbiter favours older
// waves, so waves claim kChunk-element chunks through an LDS counter.
//
// Two-level compaction, sized for k << n: per float4 row a wave only decides
// which LANES hold a candidate (|v| >= s_lo, one ballot) and appends those lanes'
// float4 + base index to a per-wave LDS entry ring (~3 of 64 lanes per row at
// k = 1 %).  Every 64 entries are expanded to (value, index) pairs with the
// exact integer key test and stored to the chunk's slot range; maybe keys
// (s_lo <= key < s_hi) are binned and staged in LDS on the way, so the end of
// the tile only scans 256 bucket counts and counting-sorts the staged keys.
// ----------------------------------------------------------------------------
constexpr int kEnt = 128;  // entry ring per wave (flush at 64: <= 63 + 64 pending)

struct StreamSmem {
  float4 ent_v[kK2Waves][kEnt];   // staged lanes: the float4 row slice
  uint32_t ent_i[kK2Waves][kEnt]; // ... and the index of its first element
  float4 trash_v[kK2Waves][64];   // per-lane sinks of the branch-free batch writes
  uint32_t trash_i[kK2Waves][64];
  uint32_t maybe[kMaybeCap];      // the tile's maybe keys, in flush order
  uint32_t hist[kNBucket];        // maybe-key bucket counts, then counting-sort cursors
  uint32_t cnt[kK2Waves];
  uint32_t scratch[24];
  uint32_t mcount;
  uint32_t next_chunk;            // the tile's chunk counter (waves claim chunks)
};

// Unconditional float4 loads of kK2Unroll rows (no branch around a load: the
// compiler's vmcnt accounting stays exact and all rows are in flight together).
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

CHOCO_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-wave compaction state of the current chunk (wave-uniform).
struct WaveAcc {
  uint32_t estaged, eflushed;  // entry ring: appended / expanded
  uint32_t staged;             // candidates written to the chunk's slot range
};

// Per-tile bucket geometry, read once from the control block.
struct Buckets {
  uint32_t s_lo, s_hi, shift;
  float s_lo_f;  // s_lo as a float: !(|v| < s_lo_f) is a superset test of key >= s_lo
  uint64_t seed;
};

// Expand entries [eflushed, eflushed + nent) (nent <= 64, one per lane) into
// (value, index) candidates of the chunk [.., cend) in index order.
template <int MODE, bool XH>
CHOCO_DEV void expand_entries(const Src<MODE, XH>& src, StreamSmem& sm, int w, int lane, WaveAcc& a, uint32_t nent,
                              int64_t cend, float* __restrict__ ov, uint32_t* __restrict__ oi, const Buckets& bk) {
  wave_sync();
  const bool have = (uint32_t)lane < nent;
  const uint32_t slot = (a.eflushed + lane) & (kEnt - 1);
  const float4 ev = have ? sm.ent_v[w][slot] : make_float4(0.f, 0.f, 0.f, 0.f);
  const uint32_t ei = have ? sm.ent_i[w][slot] : 0u;
  const float vv[4] = {ev.x, ev.y, ev.z, ev.w};
  uint32_t kk[4];
  bool f[4];
  uint64_t m[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    kk[c] = MODE == kData ? fkey(vv[c]) : (rank_hash(bk.seed, ei + c) >> 1);
    f[c] = have && (int64_t)ei + c < cend && kk[c] >= bk.s_lo;
    m[c] = ballot(f[c]);
  }
  uint32_t pos = a.staged + mask_prefix(m[0]) + mask_prefix(m[1]) + mask_prefix(m[2]) + mask_prefix(m[3]);
  a.staged += (uint32_t)(__popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]) + __popcll(m[3]));
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (m[c] == 0ull) continue;  // wave-uniform
    if (f[c]) {
      ov[pos] = MODE == kData ? vv[c] : src.val((int64_t)ei + c);
      oi[pos] = ei + c;
      ++pos;
    }
    // maybe keys: bin and stage (one LDS atomic per wave for the list slots)
    const bool mb = f[c] && kk[c] < bk.s_hi;
    const uint64_t bm = ballot(mb);
    if (bm != 0ull) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&sm.mcount, (uint32_t)__popcll(bm));
      base = __builtin_amdgcn_readfirstlane(base);
      if (mb) {
        const uint32_t p = base + mask_prefix(bm);
        if (p < (uint32_t)kMaybeCap) sm.maybe[p] = kk[c];
        atomicAdd(&sm.hist[(kk[c] - bk.s_lo) >> bk.shift], 1u);
      }
    }
  }
  a.staged = __builtin_amdgcn_readfirstlane(a.staged);
  a.eflushed += nent;
}

// One float4 row per lane (256 elements per wave): stage the lanes that hold a
// candidate.  The float test !(|v| < s_lo_f) is a superset of key >= s_lo (NaN
// passes); expand_entries applies the exact test.
template <int MODE, bool XH, bool GUARD>
CHOCO_DEV void process_row(const Src<MODE, XH>& src, const float4 v4, int64_t i, int64_t cend, StreamSmem& sm,
                           int w, int lane, WaveAcc& a, float* __restrict__ ov, uint32_t* __restrict__ oi,
                           const Buckets& bk) {
  bool any = false;
  if (MODE == kData) {
    const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) any |= (!GUARD || i + c < cend) && !(fabsf(vv[c]) < bk.s_lo_f);
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) any |= (!GUARD || i + c < cend) && src.key_of(i + c, 0.f) >= bk.s_lo;
  }
  const uint64_t M = ballot(any);
  if (M == 0ull) return;  // wave-uniform: no candidate lane in this row
  if (any) {
    const uint32_t slot = (a.estaged + mask_prefix(M)) & (kEnt - 1);
    sm.ent_v[w][slot] = v4;
    sm.ent_i[w][slot] = (uint32_t)i;
  }
  a.estaged = __builtin_amdgcn_readfirstlane(a.estaged + (uint32_t)__popcll(M));
  if (a.estaged - a.eflushed >= 64u) expand_entries<MODE, XH>(src, sm, w, lane, a, 64u, cend, ov, oi, bk);
}

// Eight full rows (one load batch) as ONE branch-free block, so the compiler can
// interleave the rows' dependent compare -> ballot -> prefix -> LDS-store chains
// (the kernel is otherwise issue-stall bound at 4 waves per SIMD).  Lanes
// without a candidate store to their own trash slot.  If the batch could
// overflow the entry ring (dense inputs), rows take the per-row path instead.
template <bool XH>
CHOCO_DEV void process_batch(const Src<kData, XH>& src, const float4 (&A)[kK2Unroll], int64_t base, int64_t cend,
                             StreamSmem& sm, int w, int lane, WaveAcc& a, float* __restrict__ ov,
                             uint32_t* __restrict__ oi, const Buckets& bk) {
  bool any[kK2Unroll];
  uint64_t M[kK2Unroll];
  uint32_t add = 0;
#pragma unroll
  for (int u = 0; u < kK2Unroll; ++u) {
    any[u] = !(fabsf(A[u].x) < bk.s_lo_f) || !(fabsf(A[u].y) < bk.s_lo_f) || !(fabsf(A[u].z) < bk.s_lo_f) ||
             !(fabsf(A[u].w) < bk.s_lo_f);
    M[u] = ballot(any[u]);
    add += (uint32_t)__popcll(M[u]);
  }
  add = __builtin_amdgcn_readfirstlane(add);
  if (add == 0u) return;
  if (a.estaged - a.eflushed + add <= (uint32_t)kEnt) {
    uint32_t run = a.estaged;
#pragma unroll
    for (int u = 0; u < kK2Unroll; ++u) {
      const uint32_t slot = (run + mask_prefix(M[u])) & (kEnt - 1);
      float4* pv = any[u] ? &sm.ent_v[w][slot] : &sm.trash_v[w][lane];
      uint32_t* pi = any[u] ? &sm.ent_i[w][slot] : &sm.trash_i[w][lane];
      *pv = A[u];
      *pi = (uint32_t)(base + u * 256 + 4 * lane);
      run += (uint32_t)__popcll(M[u]);
    }
    a.estaged = __builtin_amdgcn_readfirstlane(run);
    while (a.estaged - a.eflushed >= 64u) expand_entries<kData, XH>(src, sm, w, lane, a, 64u, cend, ov, oi, bk);
  } else {
#pragma unroll
    for (int u = 0; u < kK2Unroll; ++u)
      process_row<kData, XH, false>(src, A[u], base + u * 256 + 4 * lane, cend, sm, w, lane, a, ov, oi, bk);
  }
}

template <int MODE, bool XH>
__global__ __launch_bounds__(kK2Threads, 4) void topk_stream_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, uint32_t tile, uint32_t nb,
    uint32_t side_cap, uint64_t seed, TopkCtrl* __restrict__ ctrl, uint32_t* __restrict__ cum_tab,
    uint32_t* __restrict__ cntw, uint32_t* __restrict__ side, float* __restrict__ cval,
    uint32_t* __restrict__ cidx) {
  __shared__ StreamSmem sm;
  STAMP(1024 + blockIdx.x, 0);
  Buckets bk;
  bk.s_lo = ctrl->s_lo;
  bk.s_hi = ctrl->s_hi;
  bk.shift = ctrl->shift;
  bk.s_lo_f = __uint_as_float(bk.s_lo);  // NaN when s_lo is a NaN key: then every lane is staged
  bk.seed = seed;
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  const int64_t b = blockIdx.x;
  constexpr int64_t kStep = 256 * kK2Unroll;
  Src<MODE, XH> src{x, xh, seed};
  if (threadIdx.x < kNBucket) sm.hist[threadIdx.x] = 0;
  if (threadIdx.x == 0) { sm.mcount = 0; sm.next_chunk = 0; }
  __syncthreads();

  // Chunk c's candidates go to its own slot range and count, so the tile's
  // output order is the chunk order.
  const uint32_t nchunk = tile / (uint32_t)kChunk;
  uint32_t total = 0;
  uint32_t c = 0;
  if (lane == 0) c = atomicAdd(&sm.next_chunk, 1u);
  c = __builtin_amdgcn_readfirstlane(c);
  while (c < nchunk) {
    uint32_t nx = 0;
    if (lane == 0) nx = atomicAdd(&sm.next_chunk, 1u);  // the next claim, used after this chunk
    const int64_t cbeg = b * (int64_t)tile + (int64_t)c * kChunk;
    const int64_t cend = min(cbeg + kChunk, n);
    float* __restrict__ ov = cval + cbeg;
    uint32_t* __restrict__ oi = cidx + cbeg;
    WaveAcc a{0u, 0u, 0u};
    const int64_t full_end = cend > cbeg ? cbeg + (cend - cbeg) / kStep * kStep : cbeg;
    for (int64_t base = cbeg; base < full_end; base += kStep) {
      float4 A[kK2Unroll];
      if constexpr (MODE == kData) {
        load_rows_full<XH>(x, xh, base, lane, A);
        process_batch<XH>(src, A, base, cend, sm, w, lane, a, ov, oi, bk);
      } else {
#pragma unroll
        for (int u = 0; u < kK2Unroll; ++u)
          process_row<MODE, XH, false>(src, make_float4(0.f, 0.f, 0.f, 0.f), base + u * 256 + 4 * lane, cend, sm,
                                       w, lane, a, ov, oi, bk);
      }
    }
    // tail (< kStep elements, last chunk only): guarded loads
    for (int64_t base = full_end; base < cend; base += 256) {
      const int64_t i = base + 4 * lane;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (MODE == kData) {
        float t[4];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) t[cc] = (i + cc < cend) ? src.val(i + cc) : 0.f;
        v = make_float4(t[0], t[1], t[2], t[3]);
      }
      process_row<MODE, XH, true>(src, v, i, cend, sm, w, lane, a, ov, oi, bk);
    }
    // the chunk's remaining entries (< 64)
    const uint32_t rest = a.estaged - a.eflushed;
    if (rest) expand_entries<MODE, XH>(src, sm, w, lane, a, rest, cend, ov, oi, bk);
    if (lane == 0) cntw[(int64_t)b * nchunk + c] = a.staged;
    total += a.staged;
    c = __builtin_amdgcn_readfirstlane(nx);
  }
  if (lane == 0) sm.cnt[w] = total;
  STAMP(1024 + b, 1);
  __syncthreads();
  STAMP(1024 + b, 2);

  // ---- end of tile: bucket suffix counts, side list
  const uint32_t msum = sm.mcount;
  {
    // thread t <-> maybe bucket jb = 254 - t (t = 255: the "sure" bucket 255);
    // cum[j] = #candidates with bucket >= j, sure included
    const int t = threadIdx.x;
    const int jb = t < kNMaybe ? kNMaybe - 1 - t : kNMaybe;
    const uint32_t hv = t < kNMaybe ? sm.hist[jb] : 0u;
    uint32_t hsum;
    const uint32_t above = block_excl_scan(hv, sm.scratch, &hsum);  // maybe keys in buckets > jb
    uint32_t csum = 0;
#pragma unroll
    for (int ww = 0; ww < kK2Waves; ++ww) csum += sm.cnt[ww];
    const uint32_t sure = csum - hsum;
    if (t == 0 && (msum > side_cap || msum > (uint32_t)kMaybeCap)) atomicOr(&ctrl->overflow, 1u);
    if (t < kNBucket) {
      const uint32_t cum = t < kNMaybe ? sure + above + hv : sure;
      cum_tab[b * kNBucket + jb] = cum;
      atomicAdd(&ctrl->G[b & (kNRep - 1)][jb], cum);
      if (t < kNMaybe) sm.hist[jb] = above;  // counting-sort cursor of bucket jb (hist is dead now)
    }
  }
  __syncthreads();
  {
    uint32_t* __restrict__ sd = side + b * side_cap;
    const uint32_t mc = min(msum, min(side_cap, (uint32_t)kMaybeCap));
    for (uint32_t j = threadIdx.x; j < mc; j += kK2Threads) {
      const uint32_t key = sm.maybe[j];
      const uint32_t p = atomicAdd(&sm.hist[(key - bk.s_lo) >> bk.shift], 1u);
      sd[p] = key;
    }
  }
  STAMP(1024 + b, 3);
}

// ----------------------------------------------------------------------------
// K3: exact threshold T, tie quota r and per-tile output offsets (one workgroup)
//
// Latency-bound, so organised around three dependent global round trips: the
// replicated bucket totals (-> bucket j* of the k-th key), two tiles' table
// words per thread (-> bucket-j* key counts and side offsets), then the keys
// themselves straight into their LDS slots.  T is radix-selected inside the
// bucket in LDS; per-tile (#keys > T, #keys == T) and two block scans give every
// tile's output offset and first-tie rank for K4.
// ----------------------------------------------------------------------------
constexpr int kK3PerThread = (kK2Target + kK3Threads - 1) / kK3Threads;   // tiles per thread

struct SelSmem {
  uint32_t keys[kMCap];
  uint32_t G[kNBucket];
  uint32_t hist[256];
  uint32_t scratch[24];
  uint32_t bc[8];
};

template <int MODE, bool XH>
__global__ __launch_bounds__(kK3Threads) void topk_select_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, int64_t k, uint32_t nb,
    uint32_t side_cap, uint64_t seed, float scale, TopkCtrl* __restrict__ ctrl,
    const uint32_t* __restrict__ cum_tab, const uint32_t* __restrict__ side, uint32_t* __restrict__ tile_info,
    float* __restrict__ out_val, int32_t* __restrict__ out_idx, int64_t idx_base) {
  __shared__ SelSmem fs;
  __shared__ ExactSmem es;
  const int tid = threadIdx.x, w = tid >> 6;
  STAMP(100, 0);
  const uint32_t s_lo = ctrl->s_lo, shift = ctrl->shift, overflow = ctrl->overflow;
  const uint32_t ku = (uint32_t)k;
  if (tid < kNBucket) {
    uint32_t g[kNRep];
#pragma unroll
    for (int r = 0; r < kNRep; ++r) g[r] = ctrl->G[r][tid];
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < kNRep; ++r) s += g[r];
    fs.G[tid] = s;
  }
  if (tid == 0) fs.bc[0] = 0;
  __syncthreads();
  // G[j] = #candidates in buckets >= j is non-increasing; j* = the unique
  // j <= 254 with G[j] >= k > G[j+1]
  bool fallback = overflow != 0 || fs.G[0] < ku || fs.G[kNMaybe] >= ku;
  if (!fallback && tid < kNMaybe && fs.G[tid] >= ku && fs.G[tid + 1] < ku) fs.bc[0] = tid;
  __syncthreads();
  const uint32_t jstar = fs.bc[0];
  if (!fallback && fs.G[jstar] - fs.G[jstar + 1] > (uint32_t)kMCap) fallback = true;
  if (fallback) {
    // the sample's guess was off: exact single-workgroup selection (correct, slow)
    Src<MODE, XH> src{x, xh, seed};
    if (tid == 0) ctrl->fallback = 1u;
    block_topk_exact(src, n, k, scale, out_val, out_idx, idx_base, es);
    return;
  }
  STAMP(100, 1);
  // ---- this thread's tiles: b = tid * kK3PerThread + q (contiguous, so the block
  // scans below run in tile order)
  uint32_t above[kK3PerThread], cb[kK3PerThread], off[kK3PerThread];
#pragma unroll
  for (int q = 0; q < kK3PerThread; ++q) {
    const int64_t b = (int64_t)tid * kK3PerThread + q;
    const int64_t bc = b < (int64_t)nb ? b : 0;  // clamped: the loads below are unconditional
    const uint32_t* row = cum_tab + bc * kNBucket;
    const uint32_t a = row[jstar], c = row[jstar + 1], s = row[kNMaybe];
    above[q] = b < (int64_t)nb ? c : 0u;
    cb[q] = b < (int64_t)nb ? a - c : 0u;  // keys of bucket j* in this tile
    off[q] = c - s;                        // their side-list offset (buckets stored high to low)
  }
  uint32_t mine = 0;
#pragma unroll
  for (int q = 0; q < kK3PerThread; ++q) mine += cb[q];
  STAMP(102, 0);
  uint32_t M;
  const uint32_t kpos = block_excl_scan(mine, fs.scratch, &M);  // M = G[j*] - G[j*+1]
  STAMP(102, 1);
  {
    // this thread's key slots [0, mine) over its tiles; loads in batches of 8
    // issued before any LDS store, so each batch costs one round trip
    const uint32_t* sd[kK3PerThread];
    uint32_t first[kK3PerThread];
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < kK3PerThread; ++q) {
      sd[q] = side + ((int64_t)tid * kK3PerThread + q) * side_cap + off[q];
      first[q] = acc;
      acc += cb[q];
    }
    constexpr int kB = 8;
    for (uint32_t i0 = 0; i0 < mine; i0 += kB) {
      uint32_t v[kB];
#pragma unroll
      for (int g = 0; g < kB; ++g) {
        const uint32_t i = min(i0 + g, mine - 1);  // clamped: the load is unconditional
        int q = 0;
#pragma unroll
        for (int t = 1; t < kK3PerThread; ++t) q += i >= first[t];
        v[g] = sd[q][i - first[q]];
      }
#pragma unroll
      for (int g = 0; g < kB; ++g)
        if (i0 + g < mine) fs.keys[kpos + i0 + g] = v[g];
    }
  }
  STAMP(102, 2);
  __syncthreads();
  STAMP(100, 2);
  // ---- radix select inside bucket j*: rel = key - base_j in [0, 2^shift)
  const uint32_t base_j = s_lo + (jstar << shift);
  uint32_t prefix = 0, krem = ku - fs.G[jstar + 1];  // 1 <= krem <= M
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
    if (w == 0) wave_find_bin(fs.hist, krem, fs.bc + 2);
    __syncthreads();
    prefix |= fs.bc[2] << dsh;
    krem = fs.bc[3];
    sh = dsh;
    __syncthreads();
  }
  const uint32_t T = base_j + prefix;
  const uint32_t r = krem;  // ties at T to take (>= 1)
  STAMP(100, 3);
  // ---- per tile: #keys > T (every key above bucket j* is) and #keys == T
  uint32_t gt[kK3PerThread], eq[kK3PerThread];
  uint32_t gsum = 0, esum = 0;
  {
    uint32_t p = kpos;
#pragma unroll
    for (int q = 0; q < kK3PerThread; ++q) {
      uint32_t g = above[q], e = 0;
      for (uint32_t i = 0; i < cb[q]; ++i) {
        const uint32_t key = fs.keys[p + i];
        g += key > T;
        e += key == T;
      }
      p += cb[q];
      gt[q] = g;
      eq[q] = e;
      gsum += g;
      esum += e;
    }
  }
  uint32_t gtot, etot;
  uint32_t gpre = block_excl_scan(gsum, fs.scratch, &gtot);
  uint32_t epre = block_excl_scan(esum, fs.scratch, &etot);
  uint32_t* __restrict__ tile_off = tile_info;
  uint32_t* __restrict__ tile_tieb = tile_info + nb;
  uint32_t* __restrict__ tile_mode = tile_info + 2 * nb;
#pragma unroll
  for (int q = 0; q < kK3PerThread; ++q) {
    const int64_t b = (int64_t)tid * kK3PerThread + q;
    if (b < (int64_t)nb) {
      const uint32_t taken = min(r, epre);  // ties taken by earlier tiles (lowest index first)
      const uint32_t take = min(eq[q], r - taken);
      tile_off[b] = gpre + taken;
      tile_tieb[b] = epre;
      tile_mode[b] = take == 0 ? kTakeNone : (take == eq[q] ? kTakeAll : kTakePartial);
    }
    gpre += gt[q];
    epre += eq[q];
  }
  if (tid == 0) {
    ctrl->T = T;
    ctrl->r = r;
    ctrl->fallback = 0u;
  }
  STAMP(101, 0);
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
  __shared__ uint32_t run_start[2 * kK4Threads + 1];
  const int64_t b = blockIdx.x;
  STAMP(24576 + b, 0);
  // every control word is independent: issue all loads before the first use
  const uint32_t fallback = ctrl->fallback, T = ctrl->T, r = ctrl->r;
  uint32_t out = tile_info[b];
  uint32_t tie_run = tile_info[nb + b];
  const uint32_t mode = tile_info[2 * nb + b];
  const uint32_t nchunk = tile / (uint32_t)kChunk;  // <= 2 * kK4Threads (tile <= 2^31 / 256)
  const uint32_t j0 = 2 * threadIdx.x, j1 = j0 + 1;
  const uint32_t cw0 = j0 < nchunk ? cntw[b * nchunk + j0] : 0u;
  const uint32_t cw1 = j1 < nchunk ? cntw[b * nchunk + j1] : 0u;
  if (fallback) return;
  {
    // exclusive scan of the tile's per-chunk run lengths -> run_start[0..nchunk]
    uint32_t tot;
    const uint32_t pre = block_excl_scan(cw0 + cw1, scratch, &tot);
    if (j0 < nchunk) run_start[j0] = pre;
    if (j1 < nchunk) run_start[j1] = pre + cw0;
    if (threadIdx.x == 0) run_start[nchunk] = tot;
    __syncthreads();
  }
  const uint32_t tot = run_start[nchunk];
  const int64_t tb = b * tile;
  // Batches of kK4Threads * R candidates; thread t owns R consecutive positions
  // (thread order = index order), loads them all at once, and one block scan of
  // its count places them (two scans only when ties at T are split).
  constexpr int R = 8;
  for (uint32_t p0 = 0; p0 < tot; p0 += kK4Threads * R) {
    const uint32_t pb = p0 + threadIdx.x * R;
    uint32_t lo = 0;
    if (pb < tot) {
      uint32_t hi = nchunk - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (run_start[mid] <= pb) lo = mid; else hi = mid - 1;
      }
    }
    int64_t addr[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const uint32_t p = pb + i;
      if (p < tot)
        while (run_start[lo + 1] <= p) ++lo;  // the run of position p (runs may be empty)
      addr[i] = p < tot ? tb + (int64_t)lo * kChunk + (p - run_start[lo]) : tb;  // clamped: loads are unconditional
    }
    float v[R];
    uint32_t idx[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      v[i] = cval[addr[i]];
      idx[i] = cidx[addr[i]];
    }
    bool gt[R], eq[R];
    uint32_t neq = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const bool valid = pb + i < tot;
      const uint32_t key = MODE == kData ? fkey(v[i]) : (rank_hash(seed, idx[i]) >> 1);
      gt[i] = valid && key > T;
      eq[i] = valid && key == T;
      neq += eq[i] ? 1u : 0u;
    }
    bool sel[R];
    if (mode == kTakePartial) {  // workgroup-uniform
      uint32_t eq_total;
      uint32_t rank = tie_run + block_excl_scan(neq, scratch, &eq_total);
#pragma unroll
      for (int i = 0; i < R; ++i) {
        sel[i] = gt[i] || (eq[i] && rank < r);
        rank += eq[i] ? 1u : 0u;
      }
      tie_run += eq_total;
    } else {
#pragma unroll
      for (int i = 0; i < R; ++i) sel[i] = gt[i] || (eq[i] && mode == kTakeAll);
    }
    uint32_t nmine = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) nmine += sel[i] ? 1u : 0u;
    uint32_t nsel;
    uint32_t pos = out + block_excl_scan(nmine, scratch, &nsel);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (sel[i]) {
        out_val[pos] = v[i] * scale;
        out_idx[pos] = (int32_t)((int64_t)idx[i] + idx_base);
        ++pos;
      }
    }
    out += nsel;
  }
  STAMP(24576 + b, 1);
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

template <int MODE, bool XH>
static int launch_topk(const float* x, const float* xh, int64_t n, int64_t k, uint64_t seed, float scale,
                       float* out_val, int32_t* out_idx, int64_t idx_base, void* ws, size_t ws_bytes,
                       hipStream_t st) {
  if (n <= kSmallN || k >= n) {
    CHOCO_KLAUNCH((topk_exact_kernel<MODE, XH>), dim3(1), dim3(kExactThreads), 0, st, x, xh, n, k,
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
    CHOCO_KLAUNCH((topk_sample_hist_kernel<XH>), dim3(kK1Blocks), dim3(kK1Threads), 0, st, x, xh, n, k1);
    CHOCO_LAUNCHED("topk_sample_hist_kernel");
    CHOCO_KLAUNCH((topk_sample_bounds_kernel<XH>), dim3(kK1Blocks), dim3(kK1Threads), 0, st, x, xh, n, k, ctrl,
                  k1);
    CHOCO_LAUNCHED("topk_sample_bounds_kernel");
  } else {
    // keys uniform on [0, 2^31): P(key >= t) = (2^31 - t) / 2^31
    const double nd = (double)n, kd = (double)k, sd = sqrt(kd);
    const double c_lo = std::min(nd, kd + 6.0 * sd + 16.0);
    const double c_hi = kd - 6.0 * sd - 16.0;
    const double two31 = 2147483648.0;
    uint32_t s_lo = (uint32_t)std::max(0.0, floor(two31 * (1.0 - c_lo / nd)));
    uint64_t s_hi_est = c_hi < 1.0 ? 0x80000000ull : (uint64_t)ceil(two31 * (1.0 - c_hi / nd));
    if (s_hi_est <= s_lo) s_hi_est = (uint64_t)s_lo + 1;
    CHOCO_KLAUNCH(topk_set_params_kernel, dim3(1), dim3(256), 0, st, ctrl, s_lo, s_hi_est);
    CHOCO_LAUNCHED("topk_set_params_kernel");
  }
  profile_begin("topk_stream", st);
  CHOCO_KLAUNCH((topk_stream_kernel<MODE, XH>), dim3(L.nb), dim3(kK2Threads), 0, st, x, xh, n, L.tile, L.nb,
                L.side_cap, seed, ctrl, cum, cntw, side, cval, cidx);
  profile_end("topk_stream", st);
  CHOCO_LAUNCHED("topk_stream_kernel");
  CHOCO_KLAUNCH((topk_select_kernel<MODE, XH>), dim3(1), dim3(kK3Threads), 0, st, x, xh, n, k, L.nb,
                L.side_cap, seed, scale, ctrl, cum, side, tinfo, out_val, out_idx, idx_base);
  CHOCO_LAUNCHED("topk_select_kernel");
  CHOCO_KLAUNCH((topk_emit_kernel<MODE>), dim3(L.nb), dim3(kK4Threads), 0, st, L.tile, L.nb, seed, scale, ctrl,
                cntw, tinfo, cval, cidx, out_val, out_idx, idx_base);
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
    CHOCO_KLAUNCH((topk_segmented_kernel<true>), dim3(nseg), dim3(kExactThreads), 0, st, x, xhat,
                       plan_dev, nseg, out_val, out_idx);
  else
    CHOCO_KLAUNCH((topk_segmented_kernel<false>), dim3(nseg), dim3(kExactThreads), 0, st, x, xhat,
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

#if CHOCO_STAMPS
// Diagnostic builds only: re-launch the stream kernel alone `reps` times back to
// back (after one full choco_topk_compress on the same workspace set its
// thresholds), timed with dispatch-attached events -> *avg_ms.
CHOCO_API int choco_dbg_stream_only(const float* x, int64_t n, void* ws, size_t ws_bytes, int32_t reps,
                                    double* avg_ms, void* stream) {
  hipStream_t st = as_stream(stream);
  const TopkLayout L = topk_layout(n);
  CHOCO_REQUIRE(ws && ws_bytes >= L.total && reps > 0, "bad arguments");
  char* base = static_cast<char*>(ws);
  TopkCtrl* ctrl = reinterpret_cast<TopkCtrl*>(base + L.off_ctrl);
  hipEvent_t a, b;
  CHOCO_HIP(hipEventCreate(&a));
  CHOCO_HIP(hipEventCreate(&b));
  CHOCO_HIP(hipEventRecord(a, st));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((topk_stream_kernel<kData, false>), dim3(L.nb), dim3(kK2Threads), 0, st, x, nullptr, n,
                       L.tile, L.nb, L.side_cap, (uint64_t)0, ctrl, reinterpret_cast<uint32_t*>(base + L.off_cum),
                       reinterpret_cast<uint32_t*>(base + L.off_cntw), reinterpret_cast<uint32_t*>(base + L.off_side),
                       reinterpret_cast<float*>(base + L.off_cval), reinterpret_cast<uint32_t*>(base + L.off_cidx));
  CHOCO_HIP(hipEventRecord(b, st));
  CHOCO_HIP(hipEventSynchronize(b));
  float ms = 0.f;
  CHOCO_HIP(hipEventElapsedTime(&ms, a, b));
  *avg_ms = ms / reps;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return CHOCO_OK;
}

// Diagnostic builds only: copy out (and clear) the phase stamps.
CHOCO_API int choco_dbg_stamps(unsigned long long* host, size_t bytes) {
  const size_t all = sizeof(unsigned long long) * kStampSlots * 4;
  if (bytes > all) bytes = all;
  if (host) CHOCO_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost));
  static unsigned long long zeros[kStampSlots * 4];
  CHOCO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zeros, all, 0, hipMemcpyHostToDevice));
  return CHOCO_OK;
}
#endif
