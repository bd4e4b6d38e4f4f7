// Random-k sparsification on MI355X: a direct sampler.
//
// Replaces SparsificationCompressor.get_random_k (reference
// dl_code/pcode/utils/sparsification.py:40-54: np.random.choice(n, k,
// replace=False), then x_data[selected_indices], scaled by n / k when
// unbiased) and the random_k branch of CHOCOSparsificationCompressor.compress
// (parallel_choco_v.py:229-260, one draw per parameter tensor).
//
// The sample is a uniform k-subset of [0, N) drawn WITHOUT touching the N - k
// unselected elements (round 2 hashed and ranked all N indices):
//   * pi_N(.; K) is a seeded bijection of [0, N): four rounds of
//     (add a_r, multiply by odd m_r, x ^= x >> h) on the B-bit domain
//     (2^B >= N, h = (B + 1) / 2), cycle-walked back into [0, N);
//   * the segment is cut into tiles of 2^18 elements; tile t's count c_t is
//     #{ j < k : pi_N(j; K) >> 18 == t } -- the counts of the first k values of
//     a random permutation, i.e. exactly the multivariate hypergeometric split
//     of a uniform k-subset over the tiles (one pass over k, not N);
//   * inside tile t the c_t positions are pi_{L_t}(j; K_t), j < c_t -- a fresh
//     uniform c_t-subset of the tile (conditioned on its count, a uniform
//     k-subset is uniform inside every tile and independent across tiles), set
//     in a 32 KB LDS bitmap and emitted in ascending order with a gather of
//     x[i] (- xhat[i]) (* n / k).
// Keys: K = derive(qrng_key(seed, offset), s) for segment s (the flat call is
// segment 0), K_t = derive(K, 8 + t), round keys of pi(.; K): a_r = derive(K, 2r),
// m_r = derive(K, 2r + 1) | 1, masked to B bits, derive(K, i) =
// splitmix64_mix(K + (i + 1) * 0x9E3779B97F4A7C15).  oracle/choco_oracle.py
// restates every step (randk_indices, randk_segmented).
//
// Two launches: R1 (tile counts; only for segments of more than one tile) and R2
// (per tile: bitmap sample, ordered emission, gather).  Bytes: 4k gathered (8k
// with xhat) + 8k written; the sampler itself reads nothing.
//
// R1 spreads a segment's k draws over G = min(tiles, 256) workgroups; each writes
// its column of a [tile][256] count matrix (draws per tile, draws in earlier
// tiles) with plain stores, and an R2 tile sums its own row (count and output
// offset) -- no atomics (round 3's per-tile counters, one 128-B line each, took
// 382 device-scope adders per line at 100M: 12-27 us).
#include "choco_common.h"

#include <algorithm>
#include <mutex>
#include <unordered_map>

namespace choco {

// Diagnostic phase stamps (tools/rk_stamps.py; never in the product build).
#ifndef CHOCO_STAMPS
#define CHOCO_STAMPS 0
#endif
#if CHOCO_STAMPS
constexpr int kRkStampSlots = 16384;
__device__ unsigned long long g_rk_stamps[kRkStampSlots][8];
#define RKSTAMP(slot, j)                                                     \
  do {                                                                      \
    if (threadIdx.x == 0 && (slot) < kRkStampSlots) g_rk_stamps[(slot)][(j)] = wall_clock64(); \
  } while (0)
#else
#define RKSTAMP(slot, j) \
  do {                   \
  } while (0)
#endif

constexpr int kRkTileBits = 18;
constexpr int64_t kRkTile = int64_t(1) << kRkTileBits;  // elements per tile: a 32 KB bitmap
constexpr int kRkThreads = 1024;                         // R1
constexpr int kRkWords = (int)(kRkTile / 32);            // 8192 bitmap words per tile
// R2: kRkQ workgroups per tile, each 1 / kRkQ of the tile's bitmap (8: 2^15 bits,
// 4 KB of LDS) with kRkQThreads threads of kRkWpt words each: many small workgroups
// per CU instead of 1-2 large ones (382 tiles on 256 CUs left half the CUs with two
// 1024-thread tiles and set the tail: 44.7 us at 100M).  r04 same-box A/B (three
// passes): R2 itself 41.6-41.7 (4) / 41.1-41.3 (8) / 41.8-43.3 us (16); the sparse
// accumulate after it 78.7-79.3 / 77.4-77.7 / 76.1-76.9 us; step 0.1406-0.1415 /
// 0.1384-0.1405 / 0.1385-0.1391 ms.
constexpr int kRkQ = 8;  // workgroups per tile (4: 41.6 us, 16: no better; r04)
constexpr int kRkQThreads = 256;
constexpr int kRkQWords = kRkWords / kRkQ;               // 1024 at kRkQ = 8
constexpr int kRkWpt = kRkQWords / kRkQThreads;          // 4 words (128 bits) per thread at kRkQ = 8
constexpr int kRkMaxSegTiles = (int)((int64_t(1) << 31) >> kRkTileBits);  // 8192 tiles of one segment
constexpr int kRkGroups = 256;   // R1 workgroups drawing one segment's counts (count-matrix row length)
constexpr int kRkList = 4096;    // R2: positions of a quarter listed in LDS (denser quarters emit per thread)
constexpr int kRkGU = 4;         // R2: list gathers in flight per thread
constexpr int kRkWalkCap = 4096;  // cycle-walk bound (P(walk > 64) < 2^-64 per draw): a GPU loop must end
static_assert(kRkWpt * 32 * kRkQThreads * kRkQ == kRkTile, "bitmap geometry");

CHOCO_DEV __host__ uint64_t rk_derive(uint64_t K, uint64_t i) { return splitmix64_mix(K + (i + 1) * kGoldenGamma); }

// Seeded bijection of [0, N), N in [1, 2^31).
struct RkPerm {
  uint32_t N, mask, h;
  uint32_t a[4], m[4];
  CHOCO_DEV void init(uint64_t K, uint32_t n) {
    N = n;
    uint32_t B = 1;
    while ((1u << B) < n) ++B;
    mask = (1u << B) - 1u;
    h = (B + 1u) / 2u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      a[r] = (uint32_t)rk_derive(K, 2 * r) & mask;
      m[r] = ((uint32_t)rk_derive(K, 2 * r + 1) | 1u) & mask;
    }
  }
  CHOCO_DEV uint32_t rounds(uint32_t x) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x = (x + a[r]) & mask;
      x = (x * m[r]) & mask;
      x ^= x >> h;
    }
    return x;
  }
  CHOCO_DEV uint32_t operator()(uint32_t j) const {
    uint32_t y = rounds(j);
    for (int it = 0; y >= N && it < kRkWalkCap; ++it) y = rounds(y);
    return y;
  }
};

// One tile of one segment: where it is, what its segment is.
struct RkTile {
  int64_t seg_off, seg_len, k, out_off;  // the segment (plan row)
  int64_t t, ntile, first;               // tile index in the segment, its tile count, global id of its tile 0
  uint64_t K;                            // the segment's key
};

// plan (int64): the segmented top-k plan (topk_seg.hip) followed by the random-k
// tile table at rk_base: [R] then R x {segment, tile in segment, first tile of the
// segment, tiles of the segment}.
CHOCO_DEV RkTile rk_tile_seg(const int64_t* __restrict__ plan, int64_t rk_base, uint64_t key, int64_t b) {
  const int64_t* e = plan + rk_base + 1 + 4 * b;
  const int64_t s = e[0];
  const int64_t* row = plan + 8 * s;
  RkTile T;
  T.seg_off = row[0];
  T.seg_len = row[1];
  T.k = row[2];
  T.out_off = row[3];
  T.t = e[1];
  T.first = e[2];
  T.ntile = e[3];
  T.K = rk_derive(key, (uint64_t)s);
  return T;
}
CHOCO_DEV RkTile rk_tile_flat(int64_t n, int64_t k, uint64_t key, int64_t b) {
  RkTile T;
  T.seg_off = 0;
  T.seg_len = n;
  T.k = k;
  T.out_off = 0;
  T.t = b;
  T.ntile = (n + kRkTile - 1) >> kRkTileBits;
  T.first = 0;
  T.K = rk_derive(key, 0);
  return T;
}

// R1: group g < G = min(tiles, kRkGroups) of a multi-tile segment draws j in
// [k g / G, k (g + 1) / G) -> pi_N(j) -> a tile histogram in LDS, and writes its
// column of the segment's count matrix: H[tile][g] (this group's draws in the
// tile) and P[tile][g] (its draws in the segment's earlier tiles).  No atomics:
// an R2 tile sums its own row of H and of P (G contiguous words each).  Workgroup
// b is plan tile b; tiles past their segment's G (and single-tile segments) idle.
template <bool FLAT>
__global__ __launch_bounds__(kRkThreads) void randk_count_kernel(const int64_t* __restrict__ plan, int64_t rk_base,
                                                                 int64_t n, int64_t k, uint64_t key,
                                                                 uint32_t* __restrict__ H, uint32_t* __restrict__ P) {
  __shared__ uint32_t hist[kRkMaxSegTiles];
  __shared__ uint32_t scratch[40];
  const int64_t b = blockIdx.x;
  RKSTAMP(b, 0);
  const RkTile T = FLAT ? rk_tile_flat(n, k, key, b) : rk_tile_seg(plan, rk_base, key, b);
  const int64_t G = std::min<int64_t>(T.ntile, kRkGroups);
  if (T.ntile <= 1 || T.k >= T.seg_len || T.t >= G) return;  // workgroup-uniform
  const int nt = (int)T.ntile;
  for (int i = threadIdx.x; i < nt; i += kRkThreads) hist[i] = 0u;
  __syncthreads();
  RkPerm Pm;
  Pm.init(T.K, (uint32_t)T.seg_len);
  const int64_t j0 = T.k * T.t / G, j1 = T.k * (T.t + 1) / G;
  for (int64_t j = j0 + threadIdx.x; j < j1; j += kRkThreads) atomicAdd(&hist[Pm((uint32_t)j) >> kRkTileBits], 1u);
  __syncthreads();
  RKSTAMP(b, 1);
  // column g of rows first .. first + nt - 1: kRkPer tiles per thread per round
  constexpr int kRkPer = kRkMaxSegTiles / kRkThreads;
  uint32_t c[kRkPer], sum = 0;
#pragma unroll
  for (int q = 0; q < kRkPer; ++q) {
    const int i = (int)threadIdx.x * kRkPer + q;
    c[q] = i < nt ? hist[i] : 0u;
    sum += c[q];
  }
  uint32_t tot;
  uint32_t pre = block_excl_scan(sum, scratch, &tot);
#pragma unroll
  for (int q = 0; q < kRkPer; ++q) {
    const int i = (int)threadIdx.x * kRkPer + q;
    if (i < nt) {
      H[(T.first + i) * kRkGroups + T.t] = c[q];
      P[(T.first + i) * kRkGroups + T.t] = pre;
    }
    pre += c[q];
  }
  RKSTAMP(b, 2);
}

CHOCO_DEV uint32_t pick_word(const uint32_t (&w)[kRkWpt], int q) {  // w[q] by selects (no scratch)
  uint32_t r = w[0];
#pragma unroll
  for (int i = 1; i < kRkWpt; ++i) r = q == i ? w[i] : r;
  return r;
}

// R2: one quarter of a tile ("quarter": the 1 / kRkQ part a workgroup owns) -> the tile's count and output offset (its rows of H
// and P), the quarter's bitmap (every draw of the tile is evaluated; the ones
// below the quarter are counted, which places the quarter inside the tile without
// any exchange between workgroups), the ordered emission with the gather.  Up to
// kRkList positions are listed in LDS in ascending order and gathered by
// consecutive lanes (coalesced stores, kRkGU loads in flight per thread); denser
// quarters emit per thread.
// A gathered element, non-temporal: with default-policy loads the 1M scattered lines of a
// 100M gather allocate in the Infinity Cache and push out the lines the step's accumulate left
// dirty, whose write-back then meets the gather.  Same-box A/B (r05_ab_summary.txt item 19):
// R2 41.0 -> 30.3 us, the random-k step 0.1373 -> 0.1262 ms; ResNet-50 layout unchanged.
CHOCO_DEV float rk_ld(const float* p) { return __builtin_nontemporal_load(p); }

template <bool FLAT, bool XH>
__global__ __launch_bounds__(kRkQThreads) void randk_tile_kernel(const float* __restrict__ x, const float* __restrict__ xh,
                                                                 const int64_t* __restrict__ plan, int64_t rk_base,
                                                                 int64_t n, int64_t k, uint64_t key, int32_t is_biased,
                                                                 const uint32_t* __restrict__ H,
                                                                 const uint32_t* __restrict__ P,
                                                                 float* __restrict__ out_val,
                                                                 int32_t* __restrict__ out_idx) {
  __shared__ uint32_t bm[kRkQWords];
  __shared__ uint32_t list[kRkList];
  __shared__ uint32_t scratch[40];
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x / kRkQ;
  const uint32_t qb = (uint32_t)(blockIdx.x % kRkQ) * (uint32_t)(kRkQWords * 32);  // quarter's first bit
  RKSTAMP(8192 + blockIdx.x, 0);
  const RkTile T = FLAT ? rk_tile_flat(n, k, key, b) : rk_tile_seg(plan, rk_base, key, b);
  const int64_t start = T.t << kRkTileBits;  // within the segment
  const uint32_t L = (uint32_t)std::min<int64_t>(kRkTile, T.seg_len - start);
  const bool all = T.k >= T.seg_len;
  // this tile's count and the draws of the segment's earlier tiles
  uint32_t c, pre;
  if (all) {
    c = L;
    pre = (uint32_t)start;
  } else if (T.ntile == 1) {
    c = (uint32_t)T.k;
    pre = 0u;
  } else {
    const int64_t G = std::min<int64_t>(T.ntile, kRkGroups);
    const int64_t row = (T.first + T.t) * kRkGroups;
    const uint32_t h = tid < G ? H[row + tid] : 0u, p = tid < G ? P[row + tid] : 0u;
    uint32_t x0, x1;
    block_excl_scan2(h, p, scratch, &x0, &x1, &c, &pre);
  }
  RKSTAMP(8192 + blockIdx.x, 1);
  if (qb >= L) return;  // a quarter past the segment's end (workgroup-uniform)
  // the quarter's positions: a bitmap in LDS; `below` = the tile's positions before it
  uint32_t below;
  if (all) {
#pragma unroll
    for (int q = 0; q < kRkWpt; ++q) {
      const uint32_t w0 = qb + (uint32_t)(tid * kRkWpt + q) * 32u;
      bm[tid * kRkWpt + q] = w0 + 32u <= L ? 0xFFFFFFFFu : (w0 >= L ? 0u : ((1u << (L - w0)) - 1u));
    }
    below = qb;
    __syncthreads();
  } else {
#pragma unroll
    for (int q = 0; q < kRkWpt; ++q) bm[tid * kRkWpt + q] = 0u;
    __syncthreads();
    RkPerm Pm;
    Pm.init(rk_derive(T.K, 8 + (uint64_t)T.t), L);
    uint32_t nb = 0;
    for (uint32_t j = tid; j < c; j += kRkQThreads) {
      const uint32_t pos = Pm(j);
      if (pos < qb) {
        ++nb;
      } else if (pos - qb < (uint32_t)(kRkQWords * 32)) {
        const uint32_t p = pos - qb;
        atomicOr(&bm[p >> 5], 1u << (p & 31u));
      }
    }
    block_excl_scan(nb, scratch, &below);  // (ends with a barrier: the bitmap is complete)
  }
  RKSTAMP(8192 + blockIdx.x, 2);
  // thread t owns bits [32 kRkWpt t, 32 kRkWpt (t + 1)) of the quarter: rank of its first set bit
  uint32_t w[kRkWpt];
  uint32_t mine = 0;
#pragma unroll
  for (int q = 0; q < kRkWpt; ++q) {
    w[q] = bm[tid * kRkWpt + q];
    mine += (uint32_t)__popc(w[q]);
  }
  uint32_t cq;
  uint32_t rank = block_excl_scan(mine, scratch, &cq);
  RKSTAMP(8192 + blockIdx.x, 3);
  const float scale = is_biased ? 1.0f : (float)((double)T.seg_len / (double)T.k);
  const int64_t gbase = T.seg_off + start + qb;            // global index of the quarter's first element
  const uint32_t room = c - min(below, c);                 // (bounded: never past the tile's count)
  float* __restrict__ ov = out_val + T.out_off + pre + below;
  int32_t* __restrict__ oi = out_idx + T.out_off + pre + below;
  if (cq <= (uint32_t)kRkList) {  // workgroup-uniform
    // ascending positions -> list[rank ..], then lanes gather consecutive entries
    uint32_t r = rank;
#pragma unroll
    for (int q = 0; q < kRkWpt; ++q) {
      uint32_t wq = w[q];
      while (wq != 0u) {
        list[r] = (uint32_t)(tid * kRkWpt + q) * 32u + (uint32_t)__builtin_ctz(wq);
        ++r;
        wq &= wq - 1u;
      }
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < cq; i0 += kRkQThreads * kRkGU) {
      uint32_t pos[kRkGU];
      float v[kRkGU];
#pragma unroll
      for (int u = 0; u < kRkGU; ++u) {
        const uint32_t i = i0 + (uint32_t)u * kRkQThreads + (uint32_t)tid;
        pos[u] = list[min(i, cq - 1u)];
      }
#pragma unroll
      for (int u = 0; u < kRkGU; ++u) {
        const uint32_t i = i0 + (uint32_t)u * kRkQThreads + (uint32_t)tid;
        const int64_t e = gbase + pos[u];
        v[u] = 0.f;
        if (i < cq) v[u] = XH ? rk_ld(x + e) - rk_ld(xh + e) : rk_ld(x + e);
      }
#pragma unroll
      for (int u = 0; u < kRkGU; ++u) {
        const uint32_t i = i0 + (uint32_t)u * kRkQThreads + (uint32_t)tid;
        if (i < cq && i < room) {
          ov[i] = v[u] * scale;
          oi[i] = (int32_t)(gbase + pos[u]);
        }
      }
    }
  } else {
    // dense quarter: each thread emits its own ascending positions, kG gathers in flight
    constexpr int kG = 8;
    int q = 0;
    uint32_t cur = w[0];
    for (;;) {
      uint32_t pos[kG];
      bool ok[kG];
#pragma unroll
      for (int i = 0; i < kG; ++i) {
        while (cur == 0u && q + 1 < kRkWpt) cur = pick_word(w, ++q);
        ok[i] = cur != 0u;
        pos[i] = ok[i] ? (uint32_t)(tid * kRkWpt + q) * 32u + (uint32_t)__builtin_ctz(cur) : 0u;
        if (ok[i]) cur &= cur - 1u;
      }
      if (!ok[0]) break;
      float v[kG];
#pragma unroll
      for (int i = 0; i < kG; ++i) {
        v[i] = 0.f;
        if (ok[i]) {
          const int64_t e = gbase + pos[i];
          v[i] = XH ? rk_ld(x + e) - rk_ld(xh + e) : rk_ld(x + e);
        }
      }
#pragma unroll
      for (int i = 0; i < kG; ++i) {
        if (ok[i] && rank + (uint32_t)i < room) {
          ov[rank + i] = v[i] * scale;
          oi[rank + i] = (int32_t)(gbase + pos[i]);
        }
      }
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < kG; ++i) m += ok[i] ? 1u : 0u;
      rank += m;
    }
  }
#if CHOCO_STAMPS
  __syncthreads();
  RKSTAMP(8192 + blockIdx.x, 4);
#endif
}

// ---------------------------------------------------------------- host side
void randk_forget(const void*, size_t) {}  // no per-workspace host state

int64_t randk_tiles(int64_t len) { return (len + kRkTile - 1) >> kRkTileBits; }

// counts: [256-B header (status word at 0) | H[R][256] | P[R][256]] (u32); every entry
// an R2 tile reads is written by this call's R1 (no zero-fill needed between calls)
size_t randk_counts_bytes(int64_t R) { return 256 + 2 * align_up((size_t)R * kRkGroups * 4, 256); }

// The flat call (plan == nullptr) or the segmented one (plan_dev / rk_base / R).
int randk_launch(const float* x, const float* xh, const int64_t* plan_dev, int64_t rk_base, int64_t R, int64_t n,
                 int64_t k, uint64_t seed, uint64_t offset, int32_t is_biased, float* out_val, int32_t* out_idx,
                 void* counts, size_t counts_bytes, hipStream_t st) {
  const uint64_t key = qrng_key(seed, offset);
  CHOCO_REQUIRE(counts_bytes >= randk_counts_bytes(R), "random-k counts buffer too small");
  uint32_t* H = reinterpret_cast<uint32_t*>(static_cast<char*>(counts) + 256);
  uint32_t* P = reinterpret_cast<uint32_t*>(static_cast<char*>(counts) + 256 + align_up((size_t)R * kRkGroups * 4, 256));
  const bool flat = plan_dev == nullptr;
  profile_begin("randk_count", st);
  if (flat)
    CHOCO_KLAUNCH((randk_count_kernel<true>), dim3((unsigned)R), dim3(kRkThreads), 0, st, plan_dev, rk_base, n, k,
                  key, H, P);
  else
    CHOCO_KLAUNCH((randk_count_kernel<false>), dim3((unsigned)R), dim3(kRkThreads), 0, st, plan_dev, rk_base, n, k,
                  key, H, P);
  profile_end("randk_count", st);
  CHOCO_LAUNCHED("randk_count_kernel");
  profile_begin("randk_tile", st);
  if (flat && xh)
    CHOCO_KLAUNCH((randk_tile_kernel<true, true>), dim3((unsigned)(R * kRkQ)), dim3(kRkQThreads), 0, st, x, xh, plan_dev,
                  rk_base, n, k, key, is_biased, H, P, out_val, out_idx);
  else if (flat)
    CHOCO_KLAUNCH((randk_tile_kernel<true, false>), dim3((unsigned)(R * kRkQ)), dim3(kRkQThreads), 0, st, x, xh, plan_dev,
                  rk_base, n, k, key, is_biased, H, P, out_val, out_idx);
  else if (xh)
    CHOCO_KLAUNCH((randk_tile_kernel<false, true>), dim3((unsigned)(R * kRkQ)), dim3(kRkQThreads), 0, st, x, xh, plan_dev,
                  rk_base, n, k, key, is_biased, H, P, out_val, out_idx);
  else
    CHOCO_KLAUNCH((randk_tile_kernel<false, false>), dim3((unsigned)(R * kRkQ)), dim3(kRkQThreads), 0, st, x, xh, plan_dev,
                  rk_base, n, k, key, is_biased, H, P, out_val, out_idx);
  profile_end("randk_tile", st);
  CHOCO_LAUNCHED("randk_tile_kernel");
  return CHOCO_OK;
}

}  // namespace choco

using namespace choco;

#if CHOCO_STAMPS
// Diagnostic builds only: copy out (and clear) the random-k phase stamps.
CHOCO_API int choco_dbg_rk_stamps(unsigned long long* host, size_t bytes) {
  const size_t all = sizeof(unsigned long long) * kRkStampSlots * 8;
  if (bytes > all) bytes = all;
  if (host) CHOCO_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rk_stamps), bytes, 0, hipMemcpyDeviceToHost));
  static unsigned long long zeros[kRkStampSlots * 8];
  CHOCO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_rk_stamps), zeros, all, 0, hipMemcpyHostToDevice));
  return CHOCO_OK;
}
#endif

CHOCO_API size_t choco_randk_workspace_size(int64_t n) { return n > 0 ? randk_counts_bytes(randk_tiles(n)) : 256; }

CHOCO_API int choco_randk_compress(const float* x, const float* xhat, int64_t n, int64_t k, uint64_t seed,
                                   uint64_t offset, int32_t is_biased, float* out_val, int32_t* out_idx, void* ws,
                                   size_t ws_bytes, void* stream) {
  CHOCO_REQUIRE(x != nullptr && out_val != nullptr && out_idx != nullptr, "null pointer argument");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n must be in [1, 2^31-1), got %lld", (long long)n);
  CHOCO_REQUIRE(k >= 1 && k <= n, "k must be in [1, n], got k=%lld n=%lld", (long long)k, (long long)n);
  CHOCO_REQUIRE(aligned4(x) && (xhat == nullptr || aligned4(xhat)), "x/xhat must be 4-byte aligned");
  const int64_t R = randk_tiles(n);
  CHOCO_REQUIRE(ws != nullptr && ws_bytes >= randk_counts_bytes(R),
                "random-k workspace too small: need %zu bytes, got %zu", randk_counts_bytes(R), ws_bytes);
  return randk_launch(x, xhat, nullptr, 0, R, n, k, seed, offset, is_biased, out_val, out_idx, ws, ws_bytes,
                      as_stream(stream));
}
