// Floor probe for the north-star top-k (100M fp32, k = 1 %): the best a
// single-pass top-k can do when the threshold T is GIVEN in advance -- one read of
// the 400 MB delta and the ~1M (value, index) pairs written in ascending index
// order, in ONE launch.  Anything the real codec spends beyond this is select
// machinery (VERDICT r03 "Next round" item 1).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/probe_floor.hip -o tools/probe_floor && tools/probe_floor
//
// Input: 4 rotating 400 MB buffers (1.6 GB >> the 256 MB Infinity Cache) of
// uniform [-1, 1) values; T = 0.99 selects ~1 % of them.  Variants:
//   read   : K2's launch shape, read only (255 tiles, 16 waves claiming 2048-element
//            chunks from an LDS counter, 2 x 8 KiB nt loads in flight per wave).
//   static : the same stream, every pair with |v| > T kept in LDS (per-wave regions,
//            per-chunk runs); at the tile end one lane publishes the tile count
//            (sc1) and draws an arrival ticket; the LAST workgroup scans all tile
//            counts and publishes the offsets + a flag; the others poll the flag and
//            emit their pairs from LDS at their offset (no second pass, no second
//            launch).
//   dynamic: the same, but the buffer is cut into 32K-element blocks: every
//            workgroup starts on two static blocks, then claims blocks from a pool
//            of its own XCD (one device-scope head per XCD), stealing from the other
//            XCDs' pools when its own is empty; blocks are ordered by per-block
//            counts scanned by the last workgroup.
// Each variant is checked once (count, strictly ascending indices, |v| > T,
// v == x[i]) and timed over 40 launches (event pairs); one launch per variant
// records per-workgroup phase stamps (s_memrealtime, 100 MHz) with the XCD id.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e = (x);                                         \
    if (e != hipSuccess) {                                      \
      printf("%s: %s\n", #x, hipGetErrorString(e));             \
      exit(1);                                                  \
    }                                                           \
  } while (0)

constexpr int kThreads = 1024, kWaves = 16;
constexpr int kU = 8;            // float4 rows per wave per load batch = one 2048-element chunk
constexpr int kChunk = 256 * kU;
constexpr int kPairCap = 1024;   // pairs per wave region in LDS
constexpr int kBlk = 32768;      // dynamic block: 16 chunks
constexpr int kBlkChunks = kBlk / kChunk;
constexpr int kMaxSlots = 48;    // blocks one workgroup may hold (dynamic)
constexpr int kStampW = 8;

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldnt(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
  const f4v f = __builtin_bit_cast(f4v, v);
  return make_float4(f.x, f.y, f.z, f.w);
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7u;
}
__device__ __forceinline__ void stamp(unsigned long long* st, int slot) {
  if (st != nullptr && threadIdx.x == 0) st[blockIdx.x * kStampW + slot] = wall_clock64();
}

// wave inclusive scan via shuffles (probe: clarity over speed)
__device__ __forceinline__ uint32_t wscan(uint32_t v) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o);
    if (l >= o) v += t;
  }
  return v;
}
__device__ uint32_t block_excl(uint32_t v, uint32_t* scratch, uint32_t* total) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t inc = wscan(v);
  if (l == 63) scratch[w] = inc;
  __syncthreads();
  const uint32_t t = l < kWaves ? scratch[l] : 0u;
  const uint32_t ti = wscan(t);
  const uint32_t base = __shfl(ti - t, w);
  *total = __shfl(ti, kWaves - 1);
  __syncthreads();
  return base + inc - v;
}

// One float4 row per lane: the lanes' |v| > T elements appended to the wave's LDS region.
__device__ __forceinline__ void row_pairs(float4 v, uint32_t i0, float T, uint2* region, uint32_t& fill,
                                          uint32_t& ovf) {
  const bool s0 = fabsf(v.x) > T, s1 = fabsf(v.y) > T, s2 = fabsf(v.z) > T, s3 = fabsf(v.w) > T;
  const uint32_t nc = (uint32_t)s0 + (uint32_t)s1 + (uint32_t)s2 + (uint32_t)s3;
  const uint64_t b0 = ballot(nc & 1u), b1 = ballot(nc & 2u), b2 = ballot(nc & 4u);
  const uint32_t tot = (uint32_t)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
  if (tot == 0u) return;
  if (fill + tot > (uint32_t)kPairCap) { ovf = 1u; return; }
  uint32_t p = fill + mbcnt(b0) + 2 * mbcnt(b1) + 4 * mbcnt(b2);
  if (s0) region[p++] = make_uint2(__float_as_uint(v.x), i0 + 0);
  if (s1) region[p++] = make_uint2(__float_as_uint(v.y), i0 + 1);
  if (s2) region[p++] = make_uint2(__float_as_uint(v.z), i0 + 2);
  if (s3) region[p++] = make_uint2(__float_as_uint(v.w), i0 + 3);
  fill += tot;
}

__device__ __forceinline__ void load8(__amdgpu_buffer_rsrc_t r, uint32_t boff, int lane, float4 (&A)[kU]) {
#pragma unroll
  for (int u = 0; u < kU; ++u) A[u] = ldnt(r, boff + (uint32_t)(u * 256 + 4 * lane) * 4u);
}

// ------------------------------------------------------------------ read only (K2 shape)
__global__ __launch_bounds__(kThreads) void read_only(const float* __restrict__ x, long n, uint32_t tile,
                                                      uint32_t* sink) {
  __shared__ uint32_t next;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long tb = (long)blockIdx.x * tile;
  const uint32_t tlen = (uint32_t)std::min<long>(tile, n - tb);
  const uint32_t nch = (tlen + kChunk - 1) / kChunk;
  const __amdgpu_buffer_rsrc_t r = rsrc(x + tb, tlen * 4u);
  if (threadIdx.x == 0) next = 2 * kWaves;
  __syncthreads();
  uint32_t acc = 0, cA = w, cB = w + kWaves;
  float4 A[kU], B[kU];
  load8(r, cA * kChunk * 4u, lane, A);
  load8(r, cB * kChunk * 4u, lane, B);
  for (;;) {
    if (cA >= nch) break;
    uint32_t nA = 0;
    if (lane == 0) nA = atomicAdd(&next, 1u);
    nA = __builtin_amdgcn_readfirstlane(nA);
#pragma unroll
    for (int u = 0; u < kU; ++u) acc ^= __float_as_uint(A[u].x) ^ __float_as_uint(A[u].w);
    load8(r, nA * kChunk * 4u, lane, A);
    cA = nA;
    if (cB >= nch) break;
    uint32_t nB = 0;
    if (lane == 0) nB = atomicAdd(&next, 1u);
    nB = __builtin_amdgcn_readfirstlane(nB);
#pragma unroll
    for (int u = 0; u < kU; ++u) acc ^= __float_as_uint(B[u].x) ^ __float_as_uint(B[u].w);
    load8(r, nB * kChunk * 4u, lane, B);
    cB = nB;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// ------------------------------------------------------------------ static tiles, in-launch emission
struct StaticSmem {
  uint2 pairs[kWaves * kPairCap];
  uint32_t cmeta[256];   // chunk: abs pair start | count << 16
  uint32_t cpre[257];
  uint32_t scratch[40];
  uint32_t bc[8];
  uint32_t next;
  uint32_t ovf;
};

// ctrl: [0] arrival counter, [32] flag (epoch), [64] overflow
__global__ __launch_bounds__(kThreads) void static_emit(const float* __restrict__ x, long n, uint32_t tile,
                                                        uint32_t nb, float T, uint32_t* __restrict__ cnt_t,
                                                        uint32_t* __restrict__ off_t, uint32_t* __restrict__ ctrl,
                                                        uint32_t epoch, float* __restrict__ ov,
                                                        uint32_t* __restrict__ oi, unsigned long long* stamps) {
  __shared__ StaticSmem sm;
  stamp(stamps, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t b = blockIdx.x;
  const long tb = (long)b * tile;
  const uint32_t tlen = (uint32_t)std::min<long>(tile, n - tb);
  const uint32_t nch = (tlen + kChunk - 1) / kChunk;
  const __amdgpu_buffer_rsrc_t r = rsrc(x + tb, tlen * 4u);
  if (tid == 0) { sm.next = 2 * kWaves; sm.ovf = 0; }
  uint32_t cA = w, cB = w + kWaves;
  float4 A[kU], B[kU];
  load8(r, cA * kChunk * 4u, lane, A);
  load8(r, cB * kChunk * 4u, lane, B);
  __syncthreads();
  uint2* region = sm.pairs + w * kPairCap;
  uint32_t fill = 0, ovf = 0;
  auto chunk = [&](uint32_t c, const float4 (&R)[kU]) {
    const uint32_t f0 = fill;
#pragma unroll
    for (int u = 0; u < kU; ++u) row_pairs(R[u], (uint32_t)(tb + c * kChunk + u * 256 + 4 * lane), T, region, fill, ovf);
    if (lane == 0) sm.cmeta[c] = (w * kPairCap + f0) | ((fill - f0) << 16);
  };
  for (;;) {
    if (cA >= nch) break;
    uint32_t nA = 0;
    if (lane == 0) nA = atomicAdd(&sm.next, 1u);
    nA = __builtin_amdgcn_readfirstlane(nA);
    chunk(cA, A);
    load8(r, nA * kChunk * 4u, lane, A);
    cA = nA;
    if (cB >= nch) break;
    uint32_t nB = 0;
    if (lane == 0) nB = atomicAdd(&sm.next, 1u);
    nB = __builtin_amdgcn_readfirstlane(nB);
    chunk(cB, B);
    load8(r, nB * kChunk * 4u, lane, B);
    cB = nB;
  }
  if (ovf && lane == 0) atomicOr(&sm.ovf, 1u);
  __syncthreads();
  stamp(stamps, 1);
  // tile count and chunk prefix
  uint32_t total;
  const uint32_t cc = (uint32_t)tid < nch ? sm.cmeta[tid] >> 16 : 0u;
  const uint32_t pre = block_excl(cc, sm.scratch, &total);
  if ((uint32_t)tid < nch) sm.cpre[tid] = pre;
  if (tid == 0) {
    st_sc1(&cnt_t[b], total);
    if (sm.ovf) atomicOr(&ctrl[64], 1u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sm.bc[0] = __hip_atomic_fetch_add(&ctrl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  stamp(stamps, 2);
  if (sm.bc[0] == nb - 1) {
    // the last tile: every tile's offset
    const uint32_t v = (uint32_t)tid < nb ? ld_sc1(&cnt_t[tid]) : 0u;
    uint32_t tot;
    const uint32_t o = block_excl(v, sm.scratch, &tot);
    if ((uint32_t)tid < nb) st_sc1(&off_t[tid], o);
    if ((uint32_t)tid == b) sm.bc[1] = o;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      st_sc1(&ctrl[0], 0u);
      st_sc1(&ctrl[32], epoch);
    }
  } else {
    if (w == 0) {
      for (uint32_t it = 0;; ++it) {  // bounded: a missing workgroup must not hang the GPU
        if (__builtin_amdgcn_readfirstlane(ld_sc1(&ctrl[32])) == epoch) break;
        if (it == (1u << 22)) { if (lane == 0) atomicOr(&ctrl[64], 2u); break; }
        __builtin_amdgcn_s_sleep(4);
      }
      const uint32_t o = __builtin_amdgcn_readfirstlane(ld_sc1(&off_t[b]));
      if (lane == 0) sm.bc[1] = o;
    }
    __syncthreads();
  }
  stamp(stamps, 3);
  const uint32_t O = sm.bc[1];
  // emission: a half wave per chunk
  const uint32_t h = lane & 31;
  for (uint32_t c0 = 2u * w; c0 < nch; c0 += 2u * kWaves) {
    const uint32_t c = c0 + (lane >> 5);
    const uint32_t meta = c < nch ? sm.cmeta[c] : 0u;
    const uint32_t st = meta & 0xFFFFu, cnt = meta >> 16;
    const uint32_t base = O + (c < nch ? sm.cpre[c] : 0u);
    for (uint32_t j = h; j < cnt; j += 32) {
      const uint2 pr = sm.pairs[st + j];
      ov[base + j] = __uint_as_float(pr.x);
      oi[base + j] = pr.y;
    }
  }
  stamp(stamps, 4);
  if (tid == 0 && stamps) stamps[b * kStampW + 7] = xcc_id();
}

// ------------------------------------------------------------------ dynamic blocks, in-launch emission
struct DynSmem {
  uint2 pairs[kWaves * kPairCap];
  uint32_t cmeta[kMaxSlots * kBlkChunks];
  uint32_t cpre[kMaxSlots * kBlkChunks];
  int32_t blkq[kMaxSlots];     // block of slot s; -1 pending, -2 none (pools exhausted)
  uint32_t boff[kMaxSlots];
  uint32_t scratch[40];
  uint32_t bc[8];
  uint32_t next;               // WG chunk counter (slot = c / 16)
  uint32_t pool;               // pool this WG claims from (walks 8 pools)
  uint32_t ovf;
  uint32_t nslots;
};

// ctrl: [0] arrival, [32] flag, [64] overflow, [128 + 32 p] pool heads
struct Pools {
  uint32_t D, nblk;  // dynamic blocks [D, nblk), 8 pools
  __device__ uint32_t lo(uint32_t p) const { return D + (uint32_t)(((uint64_t)(nblk - D) * p) / 8u); }
};

// one claim: the next block of the WG's current pool, else of the next pools; -2 when all are empty
__device__ int32_t claim(uint32_t* ctrl, const Pools& P, DynSmem& sm, uint32_t home) {
  for (;;) {
    const uint32_t k = __builtin_amdgcn_readfirstlane(sm.pool);
    if (k >= 8u) return -2;
    const uint32_t p = (home + k) & 7u;
    uint32_t t = 0;
    if ((threadIdx.x & 63) == 0) t = __hip_atomic_fetch_add(&ctrl[128 + 32 * p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __builtin_amdgcn_readfirstlane(t);
    const uint32_t blk = P.lo(p) + t;
    if (blk < P.lo(p + 1)) return (int32_t)blk;
    if ((threadIdx.x & 63) == 0) atomicMax(&sm.pool, k + 1);
  }
}

__global__ __launch_bounds__(kThreads) void dynamic_emit(const float* __restrict__ x, long n, uint32_t nblk,
                                                         float T, uint32_t* __restrict__ cnt_b,
                                                         uint32_t* __restrict__ off_b, uint32_t* __restrict__ ctrl,
                                                         uint32_t epoch, float* __restrict__ ov,
                                                         uint32_t* __restrict__ oi, unsigned long long* stamps) {
  __shared__ DynSmem sm;
  stamp(stamps, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t b = blockIdx.x, nwg = gridDim.x;
  const uint32_t home = xcc_id();
  const Pools P{std::min(2u * nwg, nblk), nblk};
  const __amdgpu_buffer_rsrc_t r = rsrc(x, (uint32_t)(n * 4));
  if (tid < kMaxSlots) sm.blkq[tid] = -1;
  if (tid == 0) {
    sm.blkq[0] = b < nblk ? (int32_t)b : -2;
    sm.blkq[1] = b + nwg < nblk ? (int32_t)(b + nwg) : -2;
    sm.next = 2 * kWaves;
    sm.pool = 0;
    sm.ovf = 0;
  }
  // the first two (static) blocks' chunks: wave w takes chunk w of block b and chunk w of block b + nwg
  auto boff_of = [&](int32_t blk, uint32_t j) -> uint32_t {
    return blk >= 0 ? ((uint32_t)blk * kBlk + j * kChunk) * 4u : 0xFFFFFFF0u;  // out of range: zeros
  };
  uint32_t cA = w, cB = w + kWaves;
  float4 A[kU], B[kU];
  load8(r, boff_of(b < nblk ? (int32_t)b : -2, w), lane, A);
  load8(r, boff_of(b + nwg < nblk ? (int32_t)(b + nwg) : -2, w), lane, B);
  __syncthreads();
  uint2* region = sm.pairs + w * kPairCap;
  uint32_t fill = 0, ovf = 0;
  // block of chunk c (waits while its claim is in flight); -2: past the end
  auto blk_of = [&](uint32_t c) -> int32_t {
    const uint32_t s = c / kBlkChunks;
    if (s >= (uint32_t)kMaxSlots) return -2;
    for (;;) {
      const int32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&sm.blkq[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      if (v != -1) return v;
      __builtin_amdgcn_s_sleep(1);
    }
  };
  auto chunk = [&](uint32_t c, int32_t blk, const float4 (&R)[kU]) {
    const uint32_t f0 = fill;
    const uint32_t e0 = (uint32_t)blk * kBlk + (c % kBlkChunks) * kChunk;
#pragma unroll
    for (int u = 0; u < kU; ++u) row_pairs(R[u], e0 + u * 256 + 4 * lane, T, region, fill, ovf);
    if (lane == 0) sm.cmeta[c] = (w * kPairCap + f0) | ((fill - f0) << 16);
  };
  // slot s >= 2 is claimed by the wave that takes chunk 16 (s - 2), once slot s - 1 is
  // resolved: claims are made in slot order, so a block never follows an exhausted slot
  auto claim_slot = [&](uint32_t s) {
    for (;;) {
      const int32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&sm.blkq[s - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      if (v != -1) break;
      __builtin_amdgcn_s_sleep(1);
    }
    const int32_t v = claim(ctrl, P, sm, home);
    if (lane == 0) __hip_atomic_store(&sm.blkq[s], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto take = [&]() -> uint32_t {
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(&sm.next, 1u);
    c = __builtin_amdgcn_readfirstlane(c);
    if (c % kBlkChunks == 0 && c / kBlkChunks + 2 < (uint32_t)kMaxSlots) claim_slot(c / kBlkChunks + 2);
    return c;
  };
  // chunks 0..31 (the two static blocks) are pre-assigned: slots 2 and 3 are claimed up front
  if (w == 0) {
    claim_slot(2);
    claim_slot(3);
  }
  int32_t bA = blk_of(cA), bB = blk_of(cB);
  for (;;) {
    if (bA < 0) break;
    const uint32_t nA = take();
    chunk(cA, bA, A);
    const int32_t nbA = blk_of(nA);
    load8(r, boff_of(nbA, nA % kBlkChunks), lane, A);
    cA = nA; bA = nbA;
    if (bB < 0) break;
    const uint32_t nB = take();
    chunk(cB, bB, B);
    const int32_t nbB = blk_of(nB);
    load8(r, boff_of(nbB, nB % kBlkChunks), lane, B);
    cB = nB; bB = nbB;
  }
  if (ovf && lane == 0) atomicOr(&sm.ovf, 1u);
  __syncthreads();
  stamp(stamps, 1);
  // slots held: those with a block
  if (tid == 0) {
    uint32_t s = 0;
    while (s < (uint32_t)kMaxSlots && sm.blkq[s] >= 0) ++s;
    sm.nslots = s;
  }
  __syncthreads();
  const uint32_t ns = sm.nslots;
  if ((uint32_t)tid < ns) {
    uint32_t acc = 0;
    for (int j = 0; j < kBlkChunks; ++j) {
      const uint32_t c = tid * kBlkChunks + j;
      sm.cpre[c] = acc;
      acc += sm.cmeta[c] >> 16;
    }
    st_sc1(&cnt_b[sm.blkq[tid]], acc);
  }
  if (tid == 0 && sm.ovf) atomicOr(&ctrl[64], 1u);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) sm.bc[0] = __hip_atomic_fetch_add(&ctrl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  stamp(stamps, 2);
  if (sm.bc[0] == nwg - 1) {
    constexpr int kPer = 4;  // blocks per thread (nblk <= 4096)
    uint32_t v[kPer], s = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const uint32_t i = tid * kPer + q;
      v[q] = i < nblk ? ld_sc1(&cnt_b[i]) : 0u;
      s += v[q];
    }
    uint32_t tot;
    uint32_t o = block_excl(s, sm.scratch, &tot);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const uint32_t i = tid * kPer + q;
      if (i < nblk) st_sc1(&off_b[i], o);
      o += v[q];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      st_sc1(&ctrl[0], 0u);
      for (int p = 0; p < 8; ++p) st_sc1(&ctrl[128 + 32 * p], 0u);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_sc1(&ctrl[32], epoch);
    }
  } else {
    if (w == 0) {
      for (uint32_t it = 0;; ++it) {  // bounded: a missing workgroup must not hang the GPU
        if (__builtin_amdgcn_readfirstlane(ld_sc1(&ctrl[32])) == epoch) break;
        if (it == (1u << 22)) { if (lane == 0) atomicOr(&ctrl[64], 2u); break; }
        __builtin_amdgcn_s_sleep(4);
      }
    }
    __syncthreads();
  }
  if ((uint32_t)tid < ns) sm.boff[tid] = ld_sc1(&off_b[sm.blkq[tid]]);
  __syncthreads();
  stamp(stamps, 3);
  const uint32_t nch = ns * kBlkChunks;
  const uint32_t h = lane & 31;
  for (uint32_t c0 = 2u * w; c0 < nch; c0 += 2u * kWaves) {
    const uint32_t c = c0 + (lane >> 5);
    const uint32_t meta = c < nch ? sm.cmeta[c] : 0u;
    const uint32_t st = meta & 0xFFFFu, cnt = meta >> 16;
    const uint32_t base = c < nch ? sm.boff[c / kBlkChunks] + sm.cpre[c] : 0u;
    for (uint32_t j = h; j < cnt; j += 32) {
      const uint2 pr = sm.pairs[st + j];
      ov[base + j] = __uint_as_float(pr.x);
      oi[base + j] = pr.y;
    }
  }
  stamp(stamps, 4);
  if (tid == 0 && stamps) stamps[b * kStampW + 7] = home | (ns << 8);
}

// ------------------------------------------------------------------ strided static blocks
// Workgroup b streams blocks b, b + nwg, b + 2 nwg, ... (32K elements each): every
// workgroup's bytes are spread over the whole buffer (all address ranges), ordered by
// per-block counts the last workgroup scans.  Tests whether the per-XCD spread of the
// static tiles follows the address ranges (then this evens it out) or the XCD.
struct StrSmem {
  uint2 pairs[kWaves * kPairCap];
  uint32_t cmeta[kMaxSlots * kBlkChunks];
  uint32_t cpre[kMaxSlots * kBlkChunks];
  uint32_t boff[kMaxSlots];
  uint32_t scratch[40];
  uint32_t bc[8];
  uint32_t next;
  uint32_t ovf;
};
__global__ __launch_bounds__(kThreads) void strided_emit(const float* __restrict__ x, long n, uint32_t nblk, float T,
                                                         uint32_t* __restrict__ cnt_b, uint32_t* __restrict__ off_b,
                                                         uint32_t* __restrict__ ctrl, uint32_t epoch,
                                                         float* __restrict__ ov, uint32_t* __restrict__ oi,
                                                         unsigned long long* stamps) {
  __shared__ StrSmem sm;
  stamp(stamps, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t b = blockIdx.x, nwg = gridDim.x;
  const uint32_t ns = (nblk - b + nwg - 1) / nwg;  // blocks of this workgroup
  const uint32_t nch = ns * kBlkChunks;
  const __amdgpu_buffer_rsrc_t r = rsrc(x, (uint32_t)(n * 4));
  auto boff_of = [&](uint32_t c) -> uint32_t {
    if (c >= nch) return 0xFFFFFFF0u;
    const uint32_t blk = b + (c / kBlkChunks) * nwg;
    return (blk * kBlk + (c % kBlkChunks) * kChunk) * 4u;
  };
  if (tid == 0) { sm.next = 2 * kWaves; sm.ovf = 0; }
  uint32_t cA = w, cB = w + kWaves;
  float4 A[kU], B[kU];
  load8(r, boff_of(cA), lane, A);
  load8(r, boff_of(cB), lane, B);
  __syncthreads();
  uint2* region = sm.pairs + w * kPairCap;
  uint32_t fill = 0, ovf = 0;
  auto chunk = [&](uint32_t c, const float4 (&R)[kU]) {
    const uint32_t f0 = fill;
    const uint32_t e0 = (b + (c / kBlkChunks) * nwg) * kBlk + (c % kBlkChunks) * kChunk;
#pragma unroll
    for (int u = 0; u < kU; ++u) row_pairs(R[u], e0 + u * 256 + 4 * lane, T, region, fill, ovf);
    if (lane == 0) sm.cmeta[c] = (w * kPairCap + f0) | ((fill - f0) << 16);
  };
  for (;;) {
    if (cA >= nch) break;
    uint32_t nA = 0;
    if (lane == 0) nA = atomicAdd(&sm.next, 1u);
    nA = __builtin_amdgcn_readfirstlane(nA);
    chunk(cA, A);
    load8(r, boff_of(nA), lane, A);
    cA = nA;
    if (cB >= nch) break;
    uint32_t nB = 0;
    if (lane == 0) nB = atomicAdd(&sm.next, 1u);
    nB = __builtin_amdgcn_readfirstlane(nB);
    chunk(cB, B);
    load8(r, boff_of(nB), lane, B);
    cB = nB;
  }
  if (ovf && lane == 0) atomicOr(&sm.ovf, 1u);
  __syncthreads();
  stamp(stamps, 1);
  if ((uint32_t)tid < ns) {
    uint32_t acc = 0;
    for (int j = 0; j < kBlkChunks; ++j) {
      const uint32_t c = tid * kBlkChunks + j;
      sm.cpre[c] = acc;
      acc += sm.cmeta[c] >> 16;
    }
    st_sc1(&cnt_b[b + tid * nwg], acc);
  }
  if (tid == 0 && sm.ovf) atomicOr(&ctrl[64], 1u);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) sm.bc[0] = __hip_atomic_fetch_add(&ctrl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  stamp(stamps, 2);
  if (sm.bc[0] == nwg - 1) {
    constexpr int kPer = 4;
    uint32_t v[kPer], s = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const uint32_t i = tid * kPer + q;
      v[q] = i < nblk ? ld_sc1(&cnt_b[i]) : 0u;
      s += v[q];
    }
    uint32_t tot;
    uint32_t o = block_excl(s, sm.scratch, &tot);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const uint32_t i = tid * kPer + q;
      if (i < nblk) st_sc1(&off_b[i], o);
      o += v[q];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      st_sc1(&ctrl[0], 0u);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_sc1(&ctrl[32], epoch);
    }
  } else {
    if (w == 0) {
      for (uint32_t it = 0;; ++it) {
        if (__builtin_amdgcn_readfirstlane(ld_sc1(&ctrl[32])) == epoch) break;
        if (it == (1u << 22)) { if (lane == 0) atomicOr(&ctrl[64], 2u); break; }
        __builtin_amdgcn_s_sleep(4);
      }
    }
    __syncthreads();
  }
  if ((uint32_t)tid < ns) sm.boff[tid] = ld_sc1(&off_b[b + tid * nwg]);
  __syncthreads();
  stamp(stamps, 3);
  const uint32_t h = lane & 31;
  for (uint32_t c0 = 2u * w; c0 < nch; c0 += 2u * kWaves) {
    const uint32_t c = c0 + (lane >> 5);
    const uint32_t meta = c < nch ? sm.cmeta[c] : 0u;
    const uint32_t st = meta & 0xFFFFu, cnt = meta >> 16;
    const uint32_t base = c < nch ? sm.boff[c / kBlkChunks] + sm.cpre[c] : 0u;
    for (uint32_t j = h; j < cnt; j += 32) {
      const uint2 pr = sm.pairs[st + j];
      ov[base + j] = __uint_as_float(pr.x);
      oi[base + j] = pr.y;
    }
  }
  stamp(stamps, 4);
  if (tid == 0 && stamps) stamps[b * kStampW + 7] = xcc_id() | (ns << 8);
}

// ------------------------------------------------------------------ input + reference count
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__global__ void fill_uniform(float* x, long n, uint32_t seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = (float)(hash32((uint32_t)i * 2654435761u ^ seed) >> 8) * (1.0f / 8388608.0f) - 1.0f;
}
__global__ void count_gt(const float* x, long n, float T, unsigned long long* c) {
  unsigned long long loc = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    loc += fabsf(x[i]) > T ? 1 : 0;
  atomicAdd(c, loc);
}

static bool verify(const char* name, const float* dx, long n, float T, long want, const float* dov, const uint32_t* doi) {
  std::vector<float> hx(n), hv(want);
  std::vector<uint32_t> hi(want);
  CK(hipMemcpy(hx.data(), dx, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hv.data(), dov, want * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hi.data(), doi, want * 4, hipMemcpyDeviceToHost));
  long bad = 0;
  for (long j = 0; j < want; ++j) {
    const uint32_t i = hi[j];
    const bool ok = i < (uint32_t)n && (j == 0 || i > hi[j - 1]) && fabsf(hx[i]) > T && hx[i] == hv[j];
    if (!ok && bad++ < 5) printf("  %s: bad entry %ld: idx %u val %g\n", name, j, i, hv[j]);
  }
  printf("%-8s verify: %ld entries, %ld bad -> %s\n", name, want, bad, bad ? "FAIL" : "ok");
  return bad == 0;
}

static void timeline(const char* name, const unsigned long long* st, int nwg, bool dyn) {
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < nwg; ++b) t0 = std::min(t0, st[b * kStampW + 0]);
  auto us = [&](unsigned long long t) { return (double)(t - t0) / 100.0; };  // 100 MHz
  const char* names[5] = {"start", "streamed", "ticket", "offsets known", "emitted"};
  printf("%s timeline (us from the first workgroup start)\n", name);
  for (int s = 0; s < 5; ++s) {
    std::vector<double> v;
    for (int b = 0; b < nwg; ++b) v.push_back(us(st[b * kStampW + s]));
    std::sort(v.begin(), v.end());
    printf("  %-14s min %7.2f  med %7.2f  max %7.2f\n", names[s], v[0], v[v.size() / 2], v.back());
  }
  printf("  per-XCD streamed (med / max):");
  for (int xcd = 0; xcd < 8; ++xcd) {
    std::vector<double> v;
    for (int b = 0; b < nwg; ++b)
      if ((st[b * kStampW + 7] & 7) == (unsigned)xcd) v.push_back(us(st[b * kStampW + 1]));
    std::sort(v.begin(), v.end());
    if (!v.empty()) printf(" X%d %.1f/%.1f", xcd, v[v.size() / 2], v.back());
  }
  printf("\n");
  if (dyn) {
    printf("  blocks per XCD:");
    for (int xcd = 0; xcd < 8; ++xcd) {
      unsigned s = 0;
      for (int b = 0; b < nwg; ++b)
        if ((st[b * kStampW + 7] & 7) == (unsigned)xcd) s += (unsigned)(st[b * kStampW + 7] >> 8);
      printf(" X%d %u", xcd, s);
    }
    printf("\n");
  }
}

template <class F>
static void timed(const char* name, F&& launch, double bytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 44; ++r) {
    CK(hipEventRecord(e0));
    launch(r & 3, r);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 4) ts.push_back(ms * 1000.f);
  }
  std::sort(ts.begin(), ts.end());
  const float med = ts[ts.size() / 2];
  printf("%-28s min %7.2f us  med %7.2f us  max %7.2f  -> %5.2f TB/s (%.0f MB algorithmic / med) = %.3f of 8 TB/s\n",
         name, ts[0], med, ts.back(), bytes / (med * 1e-6) / 1e12, bytes / 1e6, bytes / (med * 1e-6) / 8e12);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 100000000;  // r05: any n (cfg 2 = 25M)
  const float T = 0.99f;
  float* bufs[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&bufs[i], n * 4));
    fill_uniform<<<4096, 256>>>(bufs[i], n, 0x1234u + 77u * i);
  }
  unsigned long long* dcnt;
  CK(hipMalloc(&dcnt, 8 * 4));
  CK(hipMemset(dcnt, 0, 32));
  for (int i = 0; i < 4; ++i) count_gt<<<4096, 256>>>(bufs[i], n, T, dcnt + i);
  unsigned long long want[4];
  CK(hipMemcpy(want, dcnt, 32, hipMemcpyDeviceToHost));
  printf("n %ld, T %.2f, selected per buffer: %llu %llu %llu %llu\n", n, T, want[0], want[1], want[2], want[3]);
  const double bytes = 4.0 * n + 8.0 * (double)want[0];

  const uint32_t tileq = 32768;
  uint32_t tile = (uint32_t)((n + 255) / 256);
  tile = (tile + tileq - 1) / tileq * tileq;
  const uint32_t nb = (uint32_t)((n + tile - 1) / tile);
  const uint32_t nblk = (uint32_t)((n + kBlk - 1) / kBlk);
  printf("static: %u tiles of %u; dynamic: %u blocks of %d, 256 workgroups\n", nb, tile, nblk, kBlk);

  uint32_t *cnt, *off, *ctrl, *sink;
  float* ov;
  uint32_t* oi;
  CK(hipMalloc(&cnt, 4096 * 4));
  CK(hipMalloc(&off, 4096 * 4));
  CK(hipMalloc(&ctrl, 4096 * 4));
  CK(hipMemset(ctrl, 0, 4096 * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&ov, 2 * 1000000 * 4 + (1 << 20)));
  CK(hipMalloc(&oi, 2 * 1000000 * 4 + (1 << 20)));
  unsigned long long* st;
  CK(hipMalloc(&st, 1024 * kStampW * 8));
  std::vector<unsigned long long> hst(1024 * kStampW);
  uint32_t epoch = 1;
  uint32_t hctrl[65];

  // correctness once each
  static_emit<<<nb, kThreads>>>(bufs[0], n, tile, nb, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hctrl, ctrl, sizeof(hctrl), hipMemcpyDeviceToHost));
  printf("static overflow flag %u\n", hctrl[64]);
  const bool ok1 = verify("static", bufs[0], n, T, (long)want[0], ov, oi);
  const int nwg = 256;
  dynamic_emit<<<nwg, kThreads>>>(bufs[0], n, nblk, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hctrl, ctrl, sizeof(hctrl), hipMemcpyDeviceToHost));
  printf("dynamic overflow flag %u\n", hctrl[64]);
  const bool ok2 = verify("dynamic", bufs[0], n, T, (long)want[0], ov, oi);
  strided_emit<<<nb, kThreads>>>(bufs[0], n, nblk, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
  CK(hipDeviceSynchronize());
  const bool ok3 = verify("strided", bufs[0], n, T, (long)want[0], ov, oi);
  if (!ok1 || !ok2 || !ok3) return 1;

  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d\n", pass);
    timed("read only (K2 shape)", [&](int i, int) { read_only<<<nb, kThreads>>>(bufs[i], n, tile, sink); }, bytes);
    timed("static: read + emit", [&](int i, int) {
      static_emit<<<nb, kThreads>>>(bufs[i], n, tile, nb, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
    }, bytes);
    timed("dynamic: read + emit", [&](int i, int) {
      dynamic_emit<<<nwg, kThreads>>>(bufs[i], n, nblk, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
    }, bytes);
    timed("strided: read + emit", [&](int i, int) {
      strided_emit<<<nb, kThreads>>>(bufs[i], n, nblk, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
    }, bytes);
  }
  for (int rep = 0; rep < 2; ++rep) {
    // stamped runs (after a warm-up on the other buffers)
    static_emit<<<nb, kThreads>>>(bufs[1], n, tile, nb, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
    static_emit<<<nb, kThreads>>>(bufs[2], n, tile, nb, T, cnt, off, ctrl, epoch++, ov, oi, st);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hst.data(), st, hst.size() * 8, hipMemcpyDeviceToHost));
    timeline("static", hst.data(), (int)nb, false);
    dynamic_emit<<<nwg, kThreads>>>(bufs[3], n, nblk, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
    dynamic_emit<<<nwg, kThreads>>>(bufs[0], n, nblk, T, cnt, off, ctrl, epoch++, ov, oi, st);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hst.data(), st, hst.size() * 8, hipMemcpyDeviceToHost));
    timeline("dynamic", hst.data(), nwg, true);
    strided_emit<<<nb, kThreads>>>(bufs[1], n, nblk, T, cnt, off, ctrl, epoch++, ov, oi, nullptr);
    strided_emit<<<nb, kThreads>>>(bufs[2], n, nblk, T, cnt, off, ctrl, epoch++, ov, oi, st);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hst.data(), st, hst.size() * 8, hipMemcpyDeviceToHost));
    timeline("strided", hst.data(), (int)nb, false);
  }
  return 0;
}
