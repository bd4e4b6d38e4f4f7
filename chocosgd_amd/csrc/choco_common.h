// Shared device/host helpers for the CHOCO codec (gfx950 / CDNA4, wave64).
//
// Everything here is memory-bound per-element work: no MFMA.  Conventions used
// by every kernel in this library:
//   * `key(v)` = IEEE-754 bits of |v| (sign bit cleared).  For non-NaN floats the
//     unsigned order of keys equals the order of magnitudes, so top-k by |v|
//     (reference: torch.topk(x.abs(), k), dl_code/pcode/utils/sparsification.py:28)
//     is top-k by key.  NaN keys sort above +inf, matching torch.topk's NaN order.
//   * indices on the wire are int32 (the reference sends them as fp32 and loses
//     exactness above 2^24: communication.py:69-72, sparsification.py:76).
//   * Every arithmetic step whose rounding is observable follows the reference's
//     fp32 op order; the library is built with -ffp-contract=off so no mul+add is
//     silently fused (fmaf is written explicitly where torch itself fuses).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/choco_codec.h"

#define CHOCO_DEV __device__ __forceinline__
#define CHOCO_API extern "C" __attribute__((visibility("default")))

namespace choco {

// ---------------------------------------------------------------- errors
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);

#define CHOCO_HIP(expr)                                                     \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess)                                                   \
      return ::choco::fail(CHOCO_ERR_HIP, "%s failed: %s", #expr,           \
                           hipGetErrorString(_e));                          \
  } while (0)

#define CHOCO_LAUNCHED(what)                                                \
  do {                                                                      \
    int _rc = ::choco::check_launch(what);                                  \
    if (_rc) return _rc;                                                    \
  } while (0)

#define CHOCO_REQUIRE(cond, ...)                                            \
  do {                                                                      \
    if (!(cond)) return ::choco::fail(CHOCO_ERR_INVALID, __VA_ARGS__);      \
  } while (0)

// Optional per-kernel timing (bench roofline).  profile_begin arms a pair of
// events for the NEXT launch made by this thread; CHOCO_KLAUNCH attaches them to
// the dispatch itself (hipExtLaunchKernelGGL), so they time the kernel and not
// whatever is still queued ahead of it on the stream.  profile_end disarms.
struct ProfArm {
  hipEvent_t a, b;
};
void profile_begin(const char* name, hipStream_t st);
void profile_end(const char* name, hipStream_t st);
ProfArm profile_take();

#define CHOCO_KLAUNCH(kernel, grid, block, shm, st, ...)                                     \
  do {                                                                                      \
    const ::choco::ProfArm _pa = ::choco::profile_take();                                   \
    hipExtLaunchKernelGGL(kernel, grid, block, shm, st, _pa.a, _pa.b, 0u, __VA_ARGS__);     \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ---------------------------------------------------------------- device helpers
CHOCO_DEV uint32_t fkey(float v) { return __float_as_uint(v) & 0x7fffffffu; }

// 16-byte non-temporal load (global_load_dwordx4 ... nt) for bytes a kernel
// reads ONCE: they do not allocate in the Infinity Cache, so the stream neither
// evicts a previous kernel's dirty lines there (their write-back would land in
// the middle of the read stream) nor the data a later pass re-reads.
typedef float choco_f32x4 __attribute__((ext_vector_type(4)));
CHOCO_DEV float4 ld_nt4(const float* p) {
  const choco_f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const choco_f32x4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

// Raw buffer resource over [base, base + bytes) and a 16-byte load through it
// (buffer_load_dwordx4, `nt` when NT).  A load whose offset is out of range
// returns zeros WITHOUT a memory access: a prefetch that has nothing to fetch
// can still be issued unconditionally (exact vmcnt accounting, no branch)
// without costing a round trip.
CHOCO_DEV __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <bool NT>
CHOCO_DEV float4 ld_buf4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, NT ? 2 : 0);
  const choco_f32x4 f = __builtin_bit_cast(choco_f32x4, v);
  return make_float4(f.x, f.y, f.z, f.w);
}

// ... with a wave-uniform SGPR offset added (buffer_load_dwordx4 v, v_off, s[rsrc], s_off)
template <bool NT>
CHOCO_DEV float4 ld_buf4s(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, NT ? 2 : 0);
  const choco_f32x4 f = __builtin_bit_cast(choco_f32x4, v);
  return make_float4(f.x, f.y, f.z, f.w);
}

// 16-byte store through a buffer resource (`nt` when NT); an out-of-range
// offset is dropped without a memory access.
template <bool NT>
CHOCO_DEV void st_buf4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float4 v) {
  choco_f32x4 f;
  f.x = v.x; f.y = v.y; f.z = v.z; f.w = v.w;
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, f), r,
                                         byte_off, 0, NT ? 2 : 0);
}

// ---------------------------------------------------------------- fused gossip step
// The CHOCO consensus step x += gamma * (memory - x_hat) (optim/utils.py:67-72,
// three fp32 roundings as torch does) fused into the FIRST full pass of a
// compressor: that pass reads x, memory and x_hat, writes x_new back in place
// and works on d = x_new - x_hat (parallel_choco_v.py:236); later passes of the
// same call read (x_new, x_hat) like any delta input.
struct Gossip {
  const float* mem;  // nullptr: no gossip step
  float gamma;
};
CHOCO_DEV float gossip1(float x, float m, float h, float g) { return x + g * (m - h); }
CHOCO_DEV float4 gossip4(float4 x, float4 m, float4 h, float g) {
  return make_float4(gossip1(x.x, m.x, h.x, g), gossip1(x.y, m.y, h.y, g), gossip1(x.z, m.z, h.z, g),
                     gossip1(x.w, m.w, h.w, g));
}
CHOCO_DEV float4 sub4(float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
// the standalone step (dense.hip), for paths that have no full first pass to fuse into
int gossip_launch(float* x, const float* mem, const float* xh, float gamma, int64_t n, hipStream_t st);

CHOCO_DEV int lane_id() { return __lane_id(); }

// Drift-aware warm windows (top-k, flat K34 and segmented S3b / S4w): the key drift to
// extrapolate the next call's window by -- the last move T - t_prev when it has the sign
// of the move before it (d_prev), clamped to the smaller of the two.  A steady drift of the
// k-th key (the delta's scale growing or shrinking from step to step, as in a training
// run) is followed; noise, whose moves alternate in sign, is not.  Keys are |v| bits, so a
// key shift is a relative change of the value.
CHOCO_DEV int32_t window_drift(uint32_t T, uint32_t t_prev, uint32_t d_prev_bits, bool valid) {
  if (!valid || t_prev == 0u) return 0;
  const int64_t dn = (int64_t)T - (int64_t)t_prev, dp = (int64_t)(int32_t)d_prev_bits;
  if (dp == 0 || dn == 0 || (dn > 0) != (dp > 0)) return 0;
  const int64_t m = dn > 0 ? (dn < dp ? dn : dp) : (dn > dp ? dn : dp);
  return (int32_t)(m > (1ll << 30) ? (1ll << 30) : (m < -(1ll << 30) ? -(1ll << 30) : m));
}
// Whether the drift the previous call proposed (cand_bits, from its own last two moves) would
// have predicted this call's k-th key T better than the previous key t_prev did: a steady
// drift passes, a stationary noisy key (whose moves revert) does not.
// The caller keeps a streak of such calls and applies the drift from kDriftTrust on.
constexpr uint32_t kDriftTrust = 2;
CHOCO_DEV bool drift_trusted(uint32_t T, uint32_t t_prev, uint32_t cand_bits, bool valid) {
  if (!valid || t_prev == 0u || cand_bits == 0u) return false;
  const int64_t e_static = (int64_t)T - (int64_t)t_prev;
  const int64_t e_drift = e_static - (int64_t)(int32_t)cand_bits;
  return (e_drift < 0 ? -e_drift : e_drift) < (e_static < 0 ? -e_static : e_static);
}

// number of set bits of `mask` strictly below this lane
CHOCO_DEV uint32_t mask_prefix(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

CHOCO_DEV uint64_t ballot(bool p) { return __ballot(p); }

template <typename T>
CHOCO_DEV T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// DPP lane shift of a 32-bit value; lanes whose source is outside the row (or
// whose row is masked off) get 0.
template <int CTRL, int ROW_MASK = 0xf>
CHOCO_DEV uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}

// Inclusive prefix sum across the 64 lanes: Hillis-Steele inside each 16-lane
// row (row_shr 1, 2, 4, 8), then row_bcast:15 / row_bcast:31 carry the row
// totals -- six DPP adds, no LDS traffic (a __shfl_up version costs six
// dependent ds_bpermute round trips).
CHOCO_DEV uint32_t wave_incl_scan(uint32_t v) {
  v += dpp_u32<0x111>(v);
  v += dpp_u32<0x112>(v);
  v += dpp_u32<0x114>(v);
  v += dpp_u32<0x118>(v);
  v += dpp_u32<0x142, 0xa>(v);
  v += dpp_u32<0x143, 0xc>(v);
  return v;
}

CHOCO_DEV uint32_t wave_sum(uint32_t v) { return __builtin_amdgcn_readlane(wave_incl_scan(v), 63); }

// Block-wide exclusive scan of one u32 per thread.  `scratch` must hold
// blockDim.x/64 + 1 words of LDS.  Returns the exclusive prefix; *total gets the
// block sum.  All threads of the block must call it.  Two barriers: every wave
// scans the per-wave totals itself.
CHOCO_DEV uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
  const int l = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = (blockDim.x + 63) >> 6;
  const uint32_t inc = wave_incl_scan(v);
  if (l == 63) scratch[w] = inc;
  __syncthreads();
  const uint32_t t = (l < nw) ? scratch[l] : 0u;
  const uint32_t ti = wave_incl_scan(t);
  const uint32_t base = __builtin_amdgcn_readlane(ti - t, w);
  *total = __builtin_amdgcn_readlane(ti, nw - 1);
  __syncthreads();  // scratch may be reused by the next call
  return base + inc - v;
}

// block_excl_scan for two values at once (one set of barriers); `scratch` must
// hold 2 * blockDim.x/64 words.
CHOCO_DEV void block_excl_scan2(uint32_t v0, uint32_t v1, uint32_t* scratch, uint32_t* pre0, uint32_t* pre1,
                                uint32_t* tot0, uint32_t* tot1) {
  const int l = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = (blockDim.x + 63) >> 6;
  const uint32_t i0 = wave_incl_scan(v0), i1 = wave_incl_scan(v1);
  if (l == 63) { scratch[w] = i0; scratch[nw + w] = i1; }
  __syncthreads();
  const uint32_t t0 = (l < nw) ? scratch[l] : 0u, t1 = (l < nw) ? scratch[nw + l] : 0u;
  const uint32_t s0 = wave_incl_scan(t0), s1 = wave_incl_scan(t1);
  *pre0 = __builtin_amdgcn_readlane(s0 - t0, w) + i0 - v0;
  *pre1 = __builtin_amdgcn_readlane(s1 - t1, w) + i1 - v1;
  *tot0 = __builtin_amdgcn_readlane(s0, nw - 1);
  *tot1 = __builtin_amdgcn_readlane(s1, nw - 1);
  __syncthreads();
}

// 64-bit reinterpret for double atomics through integer exchange
CHOCO_DEV double atomic_exchange_double(double* p, double v) {
  unsigned long long old = atomicExch(reinterpret_cast<unsigned long long*>(p),
                                      (unsigned long long)__double_as_longlong(v));
  return __longlong_as_double((long long)old);
}

// Producer side of a last-block-done ticket (MI355X guide §6 Guideline 16):
// every wave drains its own memory ops, the block joins, one lane releases at
// agent scope and draws a ticket.  Returns true in every thread of the block
// that drew the last ticket; that block then acquires before reading.
CHOCO_DEV bool last_block_ticket(unsigned int* ticket, unsigned int nblocks, unsigned int* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_flag = (t == nblocks - 1) ? 1u : 0u;
  }
  __syncthreads();
  bool last = *lds_flag != 0u;
  if (last) {
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  return last;
}

// Ticket for hand-offs whose payload travels ONLY through device-scope atomics
// (performed at the memory side, coherent across XCDs): each wave waits until
// its atomics are acknowledged, then one lane draws the ticket.  No release
// fence (buffer_wbl2) per workgroup -- with thousands of workgroups that
// write-back is what dominates -- and the last workgroup reads the payload with
// atomic read-modify-writes, so it needs no acquire either.
CHOCO_DEV bool last_block_ticket_atomics(unsigned int* ticket, unsigned int nblocks, unsigned int* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_flag = (t == nblocks - 1) ? 1u : 0u;
  }
  __syncthreads();
  return *lds_flag != 0u;
}

// ---------------------------------------------------------------- segments
// seg_off: int64[nseg+1] monotone, seg_off[0] = 0, seg_off[nseg] = n.
// Returns the segment containing flat element e (binary search, global memory).
CHOCO_DEV int seg_of(const int64_t* __restrict__ seg_off, int nseg, int64_t e) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (seg_off[mid] <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// The workgroup stages seg_off[0 .. nseg] in LDS (`lds`: room for kSegLdsCap entries) when it
// fits, so that its segment lookups are LDS binary searches behind ONE global round trip
// (a search in global memory is ~log2(nseg) dependent ones); returns the table to search.
// Every thread calls it (workgroup-uniform nseg); ends with a barrier.
constexpr int kSegLdsCap = 1024;
CHOCO_DEV const int64_t* stage_seg_off(const int64_t* __restrict__ seg_off, int nseg, int64_t* lds) {
  const bool fits = nseg + 1 <= kSegLdsCap;
  if (fits)
    for (int i = threadIdx.x; i <= nseg; i += blockDim.x) lds[i] = seg_off[i];
  __syncthreads();
  return fits ? lds : seg_off;
}

// ---------------------------------------------------------------- RNG
// SplitMix64 (Steele, Lea & Flood, OOPSLA 2014; passes BigCrush): the output
// function of the splitmix64 generator, used in counter mode -- the value at
// counter c of stream `key` is mix(key + (c + 1) * gamma), exactly the
// generator's own sequence from state `key`.  Integer multiplies are quarter
// rate on CDNA (Philox4x32-10 spends 40 32-bit multiplies per 4 uniforms), so
// SplitMix64 only keys the streams and seeds xoroshiro128+ below.
constexpr uint64_t kGoldenGamma = 0x9E3779B97F4A7C15ull;
CHOCO_DEV __host__ uint64_t splitmix64_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// QSGD uniform stream of (seed, offset): key = mix(seed + (offset + 1) * 0xD1B54A32D192ED03).
CHOCO_DEV __host__ uint64_t qrng_key(uint64_t seed, uint64_t offset) {
  return splitmix64_mix(seed + (offset + 1) * 0xD1B54A32D192ED03ull);
}
CHOCO_DEV float u24(uint32_t b24) { return (float)b24 * 5.9604644775390625e-08f; }

// The uniforms themselves come from xoroshiro128+ (Blackman & Vigna 2018, the
// a=24 b=16 c=37 parameters) run for 8 steps per 16-element STREAM, its state
// seeded by SplitMix64 as its authors prescribe: stream `sid` starts at
// (mix(key + (2 sid + 1) gamma), mix(key + (2 sid + 2) gamma)).  One step (two
// 64-bit adds/xors/rotates, no multiply) yields two uniforms: bits 63..40 and
// 39..16 of s0 + s1, * 2^-24.  Amortising the seeding over 16 elements takes the
// generator from ~20 to ~9 VALU operations per element.  Stream of element e
// (qsgd.hip kQStreamTile, qstream_id): tile T = e >> 13, o = e & 8191, group
// g = o >> 11, sid = (T << 9) | ((g >> 1) << 8) | ((o >> 3) & 255), position
// (g & 1) * 8 + (o & 7).  (Round 4: 16-element streams, so a thread that owns two of a
// slot's four groups starts its own stream instead of stepping past another's.)
CHOCO_DEV __host__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
struct Xoro128 {
  uint64_t s0, s1;
  CHOCO_DEV void seed(uint64_t key, uint64_t sid) {
    const uint64_t z = key + (2 * sid + 1) * kGoldenGamma;
    s0 = splitmix64_mix(z);
    s1 = splitmix64_mix(z + kGoldenGamma);
  }
  // next output; u0/u1 = its two 24-bit uniforms
  CHOCO_DEV void next2(float& u0, float& u1) {
    const uint64_t a = s0, r = a + s1, t = s1 ^ a;
    s0 = rotl64(a, 24) ^ t ^ (t << 16);
    s1 = rotl64(t, 37);
    const uint32_t hi = (uint32_t)(r >> 32), lo = (uint32_t)r;
    u0 = u24(hi >> 8);
    u1 = u24(__builtin_amdgcn_alignbit(hi, lo, 16) & 0xFFFFFFu);
  }
};

// Seeded 32-bit bijective mixer used as the random-k ranking key
// (murmur3 fmix32 of a seeded Weyl sequence).
CHOCO_DEV uint32_t rank_hash(uint64_t seed, uint32_t i) {
  uint32_t h = i * 0x9E3779B1u + (uint32_t)seed;
  h ^= (uint32_t)(seed >> 32);
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Per-segment random-k seed (host and device agree; oracle/choco_oracle.py seg_seed):
// splitmix64 of seed + (s + 1) * golden gamma, so every segment draws an independent
// ranking (the reference calls np.random.choice once per tensor, sparsification.py:48).
CHOCO_DEV __host__ uint64_t seg_seed(uint64_t seed, int64_t s) {
  return splitmix64_mix(seed + (uint64_t)(s + 1) * kGoldenGamma);
}

// ---------------------------------------------------------------- top-k internals
// (topk.hip: the flat multi-workgroup pipeline; topk_seg.hip: the batched
// segmented select).  mode: 0 = data keys |d|, 1 = random-k hash keys.
enum TopkMode { kData = 0, kHash = 1 };
size_t topk_ws_bytes(int64_t n);
// gs.mem != nullptr: the gossip step is applied to x[0, n) first (fused into the
// stream pass where the path has one); x is then written.
// Where a call flags an invalid output (the exact fallback's bounded wait gave up): the
// sticky device status word of a workspace (at CHOCO_TOPK_STATUS_OFFSET) and its pinned
// host mirror (choco_topk_host_status), written with a system-scope store so the host
// sees it without a copy or a synchronisation.  dev == nullptr: the call's own workspace.
struct StatusSink {
  uint32_t* dev;
  uint32_t* host;
};
// the pinned, mapped host mirror of workspace ws's status word (device pointer; nullptr
// if pinned memory is unavailable), allocated on first use
uint32_t* host_status_dev(const void* ws);
int topk_pipeline(int mode, const float* x, const float* xh, int64_t n, int64_t k, uint64_t seed, float scale,
                  float* out_val, int32_t* out_idx, int64_t idx_base, void* ws, size_t ws_bytes, hipStream_t st,
                  Gossip gs = Gossip{nullptr, 0.f}, StatusSink status = StatusSink{nullptr, nullptr});
// forget the warm-start records of the top-k workspaces in [ws, ws + bytes) (include/choco_codec.h)
void topk_warm_forget(const void* ws, size_t bytes);
void seg_forget(const void* ws, size_t bytes);  // ... of the segmented workspaces (topk_seg.hip)
bool topk_warm_enabled();                        // choco_topk_set_warm_start

// random-k (randk.hip): tiles of a segment, the counts buffer, the two launches
// (plan_dev == nullptr: the flat call over [0, n) with k; else the segmented plan's
// random-k table at rk_base with R tiles)
int64_t randk_tiles(int64_t len);
size_t randk_counts_bytes(int64_t R);
int randk_launch(const float* x, const float* xh, const int64_t* plan_dev, int64_t rk_base, int64_t R, int64_t n,
                 int64_t k, uint64_t seed, uint64_t offset, int32_t is_biased, float* out_val, int32_t* out_idx,
                 void* counts, size_t counts_bytes, hipStream_t st);
void randk_forget(const void* ws, size_t bytes);

}  // namespace choco
