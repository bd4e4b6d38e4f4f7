// QSGD random quantization for the CHOCO gossip step on MI355X.
//
// Replaces QuantizationCompressor.get_qsgd / compress / uncompress
// (reference dl_code/pcode/utils/sparsification.py:87-123) as applied per
// parameter tensor by CHOCOQuantizationCompressor
// (dl_code/pcode/optim/parallel_choco_v.py:375-433).
//
// The reference transmits the DEQUANTIZED dense fp32 tensor (4n bytes); here
// the wire carries per-segment fp32 norms + a level plane (cw bits/element,
// cw = the power of two >= q) + a sign plane (1 bit/element).  The receiver
// rebuilds the reference's float bit-for-bit:
//     ((scale * sign) * norm) * level / (float)s
//
// Two passes are unavoidable (the norm of a segment is needed before any of
// its elements can be quantized):
//   qsgd_norm_kernel    : fp64 sum of squares per segment (one fp64 atomic per
//                         workgroup and segment), last workgroup rounds
//                         sqrt() to fp32 and resets the accumulators.
//   qsgd_quant_kernel   : levels + stochastic rounding + packing.  Workgroups
//                         walk the buffer in REVERSE order, so the tail that the
//                         norm pass streamed last is re-read from the 256 MB
//                         Infinity Cache instead of HBM.
#include "choco_common.h"

#include <algorithm>
#include <math.h>

namespace choco {

constexpr int kQThreads = 256;
constexpr int kQPer = 8;                         // elements per thread in the quantize/decode passes
constexpr int kQTile = kQThreads * kQPer;        // 2048
// elements per workgroup in the norm pass (a multiple of 8192): 49152 -> ~2040 workgroups
// at 100M, one round of 8 per CU (r03 A/B: 32768 and 65536 slower); smaller inputs take
// smaller tiles down to 8192, so that the grid still has ~2048 workgroups (norm_tile)
constexpr int kNormTile = 49152;
constexpr int kNormTileMin = 8192;
static int64_t norm_tile(int64_t n) {
  const int64_t t = (n / 2048 + kNormTileMin - 1) / kNormTileMin * kNormTileMin;  // 100M: 49152
  return std::min<int64_t>(kNormTile, std::max<int64_t>(kNormTileMin, t));
}
constexpr int kNormSegLds = 64;  // a tile spanning fewer segments sums them in LDS first
static_assert(kNormTile % kNormTileMin == 0 && kNormTileMin % 8192 == 0, "whole load rounds per norm tile");
constexpr int kQMaxMsg = 8;
constexpr int kAccRep = 8;  // replicas of the fp64 norm accumulators (the fused receive pass)

struct QsgdWs {
  unsigned int ticket;
  unsigned int pad[63];
  // double acc[nseg] at +256
};

static int container_bits(int q) {
  int cw = 1;
  while (cw < q) cw <<= 1;
  return cw;
}

static int64_t plane_bytes(int64_t n, int cw) { return (int64_t)align_up((size_t)((n + 7) / 8) * cw, 16); }

CHOCO_DEV float dval(const float* __restrict__ x, const float* __restrict__ xh, int64_t i) {
  return xh ? x[i] - xh[i] : x[i];
}

// Per-segment quantizer parameters.
struct QParam {
  float norm, scale;
};

CHOCO_DEV QParam qparam(const float* __restrict__ norms, const int64_t* __restrict__ seg_off, int64_t n, int seg,
                        int s_levels, bool biased) {
  QParam p;
  p.norm = norms[seg];
  p.scale = 1.0f;
  if (biased) {
    const double d = (double)(seg_off ? seg_off[seg + 1] - seg_off[seg] : n);
    const double s = (double)s_levels;
    // 1.0 / (min(d / s**2, sqrt(d) / s) + 1.0)  in Python doubles (sparsification.py:96-97)
    p.scale = (float)(1.0 / (fmin(d / (s * s), sqrt(d) / s) + 1.0));
  }
  return p;
}

// Non-temporal loads in the norm pass: they keep the previous decode's dirty
// Infinity-Cache lines from being written back in the middle of this stream (bench
// step: 120 -> 72 us), though the decode then meets them itself.
CHOCO_DEV float4 ld_norm4(const float* p) { return ld_nt4(p); }

// The quantize pass reads with the default policy (non-temporal loads measured: the
// decode after it then runs 270 -> 300 us) and its workgroups walk the tiles in reverse
// (Infinity-Cache hits on the tail the norm pass read last; r03 A/B forward 145-146 vs
// reverse 142-144 us).
CHOCO_DEV float4 ld_quant4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// The fused gossip step's xh loads and x_new stores in the norm pass: non-temporal
// (measured at 100M in the step: norm 343 -> 315 us, step 0.827 -> 0.785 ms; plain lets
// the quantize pass's backward walk hit the Infinity Cache, but the dirty lines cost
// more than that saves).
CHOCO_DEV float4 ld_gs4(const float* p) { return ld_nt4(p); }
CHOCO_DEV void st_gs4(float* p, float4 v) {
  choco_f32x4 f;
  f.x = v.x; f.y = v.y; f.z = v.z; f.w = v.w;
  __builtin_nontemporal_store(f, reinterpret_cast<choco_f32x4*>(p));
}

// ---------------------------------------------------------------- pass 1: norms
// GS: the fused gossip step (x_new = x + gamma (memory - xh) written back, the
// norm is of d = x_new - xh; the quantize pass then reads (x_new, xh)).
// (A flat instantiation without the segment code, as qsgd_decode_kernel's, measured: the
// fused gossip form 145 -> 106 VGPRs but 297-300 -> 304-305 us at 100M, the plain one 69.6-70.2
// -> 69.2-69.5 us; not kept, profiles/r06_ab_summary.txt item 16.)
template <bool XH, bool GS = false>
__global__ __launch_bounds__(kQThreads) void qsgd_norm_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ xh, int64_t n,
                                                              const int64_t* __restrict__ seg_off, int nseg,
                                                              float* __restrict__ norms_out,
                                                              QsgdWs* __restrict__ ws, Gossip gs, int64_t tile) {
  static_assert(!GS || XH, "the gossip step needs x_hat");
  // one element's delta (and, GS, its gossip step)
  auto dv = [&](int64_t i) -> float {
    if (GS) {
      const float xn = gossip1(x[i], gs.mem[i], xh[i], gs.gamma);
      const_cast<float*>(x)[i] = xn;
      return xn - xh[i];
    }
    return dval(x, XH ? xh : nullptr, i);
  };
  __shared__ int s_seg[2];
  __shared__ double s_red[kQThreads / 64];
  __shared__ double s_sacc[kNormSegLds];
  __shared__ unsigned int s_flag;
  double* __restrict__ acc = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + 256);
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = std::min<int64_t>(t0 + tile, n);
  // The tile's first and last segments (binary searches by one thread; a full tile looks them
  // up while its first loads are in flight).  A uniform tile sums per thread; otherwise each
  // thread follows the segment of its current element (its elements ascend) with a running
  // sum, added to the tile's LDS sums (or the global ones) at each boundary.
  int sg0 = 0, sg1 = 0, s = 0;
  bool uniform = true, lds = true;  // workgroup-uniform
  int64_t s_end = t1;
  double p = 0.0, run_p = 0.0;
  auto lookup = [&]() {
    if (tid == 0) {
      s_seg[0] = nseg > 1 ? seg_of(seg_off, nseg, t0) : 0;
      s_seg[1] = nseg > 1 ? seg_of(seg_off, nseg, t1 - 1) : 0;
    }
    if (tid < kNormSegLds) s_sacc[tid] = 0.0;
    __syncthreads();
    sg0 = s_seg[0];
    sg1 = s_seg[1];
    uniform = sg0 == sg1;
    lds = sg1 - sg0 < kNormSegLds;
    s = sg0;
    s_end = uniform ? t1 : seg_off[sg0 + 1];
  };
  auto flush = [&]() {
    if (run_p != 0.0) {
      if (lds) atomicAdd(&s_sacc[s - sg0], run_p);
      else unsafeAtomicAdd(&acc[s], run_p);
    }
    run_p = 0.0;
  };
  auto add4 = [&](int64_t e, const float4& a) {
    if (uniform) {
      p += (double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z + (double)a.w * a.w;
      return;
    }
    const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (e + c >= t1) break;
      if (e + c >= s_end) {
        flush();
        do {
          ++s;
          s_end = seg_off[s + 1];
        } while (e + c >= s_end);
      }
      run_p += (double)av[c] * av[c];
    }
  };
  constexpr int U = 8;  // float4 loads in flight per thread
  if (t1 - t0 == tile) {
    // full tile: unconditional loads (no branch around a load -> all U stay in flight)
    for (int64_t e0 = t0 + 4 * tid; e0 < t1; e0 += 4 * kQThreads * U) {
      float4 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = ld_norm4(x + e0 + (int64_t)u * 4 * kQThreads);
      if (e0 == t0 + 4 * tid) lookup();  // first round (every thread of a full tile runs the same rounds)
      if (GS) {
        float4 h[U], m[U];
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = ld_norm4(gs.mem + e0 + (int64_t)u * 4 * kQThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) h[u] = ld_gs4(xh + e0 + (int64_t)u * 4 * kQThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float4 xn = gossip4(a[u], m[u], h[u], gs.gamma);
          st_gs4(const_cast<float*>(x) + e0 + (int64_t)u * 4 * kQThreads, xn);
          a[u] = sub4(xn, h[u]);
        }
      } else if (XH) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float4 h = ld_norm4(xh + e0 + (int64_t)u * 4 * kQThreads);
          a[u].x -= h.x; a[u].y -= h.y; a[u].z -= h.z; a[u].w -= h.w;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) add4(e0 + (int64_t)u * 4 * kQThreads, a[u]);
    }
  } else {
    lookup();
    for (int64_t e0 = t0 + 4 * tid; e0 < t1; e0 += 4 * kQThreads * U) {
      float4 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e = e0 + (int64_t)u * 4 * kQThreads;
        if (e + 3 < t1 && !GS) {
          a[u] = *reinterpret_cast<const float4*>(x + e);
          if (XH) {
            const float4 h = *reinterpret_cast<const float4*>(xh + e);
            a[u].x -= h.x; a[u].y -= h.y; a[u].z -= h.z; a[u].w -= h.w;
          }
        } else {
          float t[4];
          for (int c = 0; c < 4; ++c) t[c] = (e + c < t1) ? dv(e + c) : 0.f;
          a[u] = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) add4(e0 + (int64_t)u * 4 * kQThreads, a[u]);
    }
  }
  if (uniform) {
    p = wave_sum(p);
    if (lane == 0) s_red[w] = p;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int i = 0; i < kQThreads / 64; ++i) t += s_red[i];
      if (t != 0.0) unsafeAtomicAdd(&acc[sg0], t);
    }
  } else {
    flush();
    if (lds) {
      __syncthreads();
      if (tid <= sg1 - sg0 && s_sacc[tid] != 0.0) unsafeAtomicAdd(&acc[sg0 + tid], s_sacc[tid]);
    }
  }
  if (last_block_ticket_atomics(&ws->ticket, gridDim.x, &s_flag)) {
    for (int q = threadIdx.x; q < nseg; q += blockDim.x)
      norms_out[q] = (float)sqrt(atomic_exchange_double(&acc[q], 0.0));
    if (threadIdx.x == 0) __hip_atomic_store(&ws->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------- pass 2: quantize + pack
template <int CW>
CHOCO_DEV void store_levels(uint8_t* __restrict__ plane, int64_t t, const uint32_t (&lv)[kQPer]) {
  if (CW == 16) {
    uint4 v;
    v.x = lv[0] | (lv[1] << 16);
    v.y = lv[2] | (lv[3] << 16);
    v.z = lv[4] | (lv[5] << 16);
    v.w = lv[6] | (lv[7] << 16);
    reinterpret_cast<uint4*>(plane)[t] = v;
  } else {
    uint64_t acc = 0;
#pragma unroll
    for (int c = 0; c < kQPer; ++c) acc |= (uint64_t)lv[c] << (c * CW);
    if (CW == 8) reinterpret_cast<uint64_t*>(plane)[t] = acc;
    if (CW == 4) reinterpret_cast<uint32_t*>(plane)[t] = (uint32_t)acc;
    if (CW == 2) reinterpret_cast<uint16_t*>(plane)[t] = (uint16_t)acc;
    if (CW == 1) plane[t] = (uint8_t)acc;
  }
}

// A group's packed levels as loaded (CW * 8 bits: 1 to 4 words) and one level of them: the
// fused receive keeps the packed form in registers (8 unpacked levels per message and group
// did not fit).
template <int CW>
struct LevelWords {
  uint32_t w[CW == 16 ? 4 : (CW == 8 ? 2 : 1)];
};
template <int CW>
CHOCO_DEV LevelWords<CW> load_level_words(const uint8_t* __restrict__ plane, int64_t t) {
  LevelWords<CW> r;
  if (CW == 16) {
    const uint4 v = reinterpret_cast<const uint4*>(plane)[t];
    r.w[0] = v.x; r.w[CW == 16 ? 1 : 0] = v.y; r.w[CW == 16 ? 2 : 0] = v.z; r.w[CW == 16 ? 3 : 0] = v.w;
  } else if (CW == 8) {
    const uint2 v = reinterpret_cast<const uint2*>(plane)[t];
    r.w[0] = v.x; r.w[CW == 8 ? 1 : 0] = v.y;
  } else if (CW == 4) {
    r.w[0] = reinterpret_cast<const uint32_t*>(plane)[t];
  } else if (CW == 2) {
    r.w[0] = reinterpret_cast<const uint16_t*>(plane)[t];
  } else {
    r.w[0] = plane[t];
  }
  return r;
}
template <int CW>
CHOCO_DEV uint32_t level_of(const LevelWords<CW>& r, int c) {
  const int bit = c * CW;
  return (r.w[bit >> 5] >> (bit & 31)) & ((CW == 16 ? 0x10000u : (1u << CW)) - 1u);
}

template <int CW>
CHOCO_DEV void load_levels(const uint8_t* __restrict__ plane, int64_t t, uint32_t (&lv)[kQPer]) {
  if (CW == 16) {
    const uint4 v = reinterpret_cast<const uint4*>(plane)[t];
    lv[0] = v.x & 0xFFFFu; lv[1] = v.x >> 16;
    lv[2] = v.y & 0xFFFFu; lv[3] = v.y >> 16;
    lv[4] = v.z & 0xFFFFu; lv[5] = v.z >> 16;
    lv[6] = v.w & 0xFFFFu; lv[7] = v.w >> 16;
  } else {
    uint64_t acc = 0;
    if (CW == 8) acc = reinterpret_cast<const uint64_t*>(plane)[t];
    if (CW == 4) acc = reinterpret_cast<const uint32_t*>(plane)[t];
    if (CW == 2) acc = reinterpret_cast<const uint16_t*>(plane)[t];
    if (CW == 1) acc = plane[t];
    const uint32_t mask = (1u << CW) - 1u;
#pragma unroll
    for (int c = 0; c < kQPer; ++c) lv[c] = (uint32_t)(acc >> (c * CW)) & mask;
  }
}

CHOCO_DEV int tile_seg(const int64_t* __restrict__ seg_off, int nseg, int64_t e0, int64_t e1, int* s_seg) {
  if (threadIdx.x == 0) {
    s_seg[0] = nseg > 1 ? seg_of(seg_off, nseg, e0) : 0;
    s_seg[1] = nseg > 1 ? seg_of(seg_off, nseg, e1 - 1) : 0;
  }
  __syncthreads();
  return s_seg[0];
}

// s * |d| / norm, correctly rounded, without the IEEE division expansion per
// element.  With y = RN(1/norm) (one real division per thread) and q0 = RN(t * y)
// (within one ulp of t / norm), r = fma(-q0, norm, t) is exact and
// RN(q0 + r * y) is RN(t / norm) (Markstein's theorem) as long as nothing
// underflows or overflows: the fast form is taken for norm in [2^-30, 2^96] and
// q0 in [2^-60, 2^7] (then t >= 2^-90 and r stays normal), zeros give +0 as
// 0/norm does, and everything else (tiny quotients, NaN/inf, extreme norms, a
// pinned norm below |d|) takes the real division.  Checked against fp32 division on 3e9 (t, norm) pairs (random over
// the guarded range + exhaustive t for 12 norm mantissas) and bit-exact against
// the oracle in the GPU tests.
struct QDiv {
  float norm, y;
  bool fast;
  uint32_t tlo_m1;  // bits(T_lo) - 1, T_lo = 2^-60 norm (1 + 2^-20): t >= T_lo implies q0 >= 2^-60
  CHOCO_DEV void init(float nrm) {
    norm = nrm;
    y = 1.0f / nrm;
    fast = nrm >= 0x1p-30f && nrm <= 0x1p96f;
    tlo_m1 = __float_as_uint(nrm * 0x1.00001p-60f) - 1u;
  }
  // The guard, per 8-element group: instead of testing every element's q0
  // against [2^-60, 2^7] (three compares and four scalar mask operations per element),
  // the group keeps min(bits(t) - 1) and max(bits(q0)) in two VALU ops per element and
  // tests them once.  Conservative: t != 0 with t < T_lo covers every q0 < 2^-60 (and
  // some above it), bits(q0) > bits(2^7) covers q0 > 2^7, inf and NaN; a flagged group
  // takes the IEEE division for all its elements, so the result is the same as a per-element
  // guard's (q0 in [2^-60, 2^7] or t == 0, norm in range).
  CHOCO_DEV float quot_nocheck(float t, uint32_t& tmin_m1, uint32_t& qmax) const {
    const float q0 = t * y;
    const float r = fmaf(-q0, norm, t);
    tmin_m1 = min(tmin_m1, __float_as_uint(t) - 1u);
    qmax = max(qmax, __float_as_uint(q0));
    return fmaf(r, y, q0);
  }
  CHOCO_DEV bool group_slow(uint32_t tmin_m1, uint32_t qmax) const {
    return !fast || tmin_m1 < tlo_m1 || qmax > 0x43000000u;
  }
};

// The container value of a level: NaN -> 0, levels >= s -> s (a pinned norm below
// |d|), as one branch-free clamp (fmaxf(NaN, 0) = 0); levels are >= 0 and integral.
CHOCO_DEV uint32_t level_code(float lvl, float sf) { return (uint32_t)fminf(fmaxf(lvl, 0.0f), sf); }

// One quantized element: level (clamped container value, 0 for NaN), sign bit.
CHOCO_DEV float qlevel(float lf, float u) {
  const float pl = floorf(lf);                                // previous_level
  return pl + ((u < (lf - pl)) ? 1.0f : 0.0f);                // + is_next_level
}

// Quantize + pack.  A 256-thread workgroup owns an 8192-element tile; thread t
// owns the four 8-element groups t_e0 + g*2048 + 8t (g = 0..3): one 4*CW-bit
// level store and one sign byte per group (the wire of the decode kernel),
// two float4 loads per group, all eight in flight before any arithmetic.  The
// thread's 32 elements are one uniform stream (xoroshiro128+, choco_common.h).
// VALU-bound, not HBM-bound, in its round-1 form (SplitMix64 per pair + the
// IEEE division per element: 123 us at 100M with the tail re-read from the
// Infinity Cache); see DESIGN.md §4 for the measured steps.
constexpr int kQG = 4;                                  // groups per thread
// The uniform stream of thread slot t's groups g, g + 1 (g even) of a tile: 16 uniforms
// each, two streams per slot (choco_common.h Xoro128; oracle qsgd_uniforms_at).
CHOCO_DEV uint64_t qstream_id(int64_t tile, int g, uint32_t t) {
  return ((uint64_t)tile << 9) | ((uint64_t)(g >> 1) << 8) | t;
}
constexpr int kQStreamTile = kQThreads * kQPer * kQG;   // 8192 elements per workgroup
static_assert(kQStreamTile == 8192, "the uniform-stream mapping (choco_common.h) assumes 8192-element tiles");

// A tile that crosses a segment boundary or ends the buffer: element by element,
// in stream order (the same uniforms as the fast path), per-element segment
// parameters and the real division.  Kept out of line: it is rare and would
// otherwise unroll into the hot kernel.
template <int CW>
__device__ __noinline__ void qsgd_quant_tile_slow(const float* __restrict__ x, const float* __restrict__ xh, int64_t n,
                                                  const int64_t* __restrict__ seg_off, int nseg, int s_levels,
                                                  int biased, const float* __restrict__ norms,
                                                  const float* __restrict__ u_in, uint64_t seed, uint64_t offset,
                                                  uint8_t* __restrict__ lvl_plane, uint8_t* __restrict__ sign_plane,
                                                  float* __restrict__ dense_out, int64_t tile, int sg0) {
  const float sf = (float)s_levels;
  const int64_t eb = tile * kQStreamTile + (int64_t)threadIdx.x * kQPer;
  // every delta of the thread first (independent loads, all in flight), then the math
  float dvv[kQG][kQPer];
#pragma unroll
  for (int g = 0; g < kQG; ++g)
#pragma unroll
    for (int c = 0; c < kQPer; ++c) {
      const int64_t e = eb + (int64_t)g * kQThreads * kQPer + c;
      dvv[g][c] = e < n ? dval(x, xh, e) : 0.f;
    }
  Xoro128 rng;
  int s = sg0, qs = -1;
  QParam Q;
#pragma unroll
  for (int g = 0; g < kQG; ++g) {
    if (!u_in && (g & 1) == 0) rng.seed(qrng_key(seed, offset), qstream_id(tile, g, threadIdx.x));
    const int64_t e0 = eb + (int64_t)g * kQThreads * kQPer;
    uint64_t lacc[2] = {0, 0};  // 8 * CW <= 128 level bits
    uint32_t sbits = 0;
#pragma unroll
    for (int c = 0; c < kQPer; c += 2) {
      float uu[2];
      if (!u_in) rng.next2(uu[0], uu[1]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t e = e0 + c + h;
        if (e >= n) continue;
        if (u_in) uu[h] = u_in[e];
        while (s + 1 < nseg && seg_off[s + 1] <= e) ++s;
        if (s != qs) {  // the segment's parameters, once per segment
          Q = qparam(norms, seg_off, n, s, s_levels, biased != 0);
          qs = s;
        }
        const float dv = dvv[g][c + h];
        const float lvl = qlevel((sf * fabsf(dv)) / Q.norm, uu[h]);  // s * x.abs() / norm
        const uint32_t li = level_code(lvl, sf);
        const int bp = (c + h) * CW;
        if (bp < 64) lacc[0] |= (uint64_t)li << bp; else lacc[1] |= (uint64_t)li << (bp - 64);
        sbits |= dv < 0.f ? (1u << (c + h)) : 0u;
        if (dense_out) {
          const float sg = dv > 0.f ? 1.0f : (dv < 0.f ? -1.0f : 0.0f);  // torch.sign (NaN -> 0)
          dense_out[e] = (((Q.scale * sg) * Q.norm) * lvl) / sf;
        }
      }
    }
    if (e0 >= n) break;
    uint32_t lv[kQPer];
#pragma unroll
    for (int c = 0; c < kQPer; ++c)
      lv[c] = (uint32_t)(c * CW < 64 ? lacc[0] >> (c * CW) : lacc[1] >> (c * CW - 64)) & ((1u << CW) - 1u);
    store_levels<CW>(lvl_plane, e0 / kQPer, lv);
    sign_plane[e0 / kQPer] = (uint8_t)sbits;
  }
}

// The math and stores of one full single-segment tile whose deltas d are in registers
// (thread t: its four 8-element groups e = tile * 8192 + g * 2048 + 8 t + c).
// NG groups g0 .. g0 + NG - 1 of thread slot `st` (the one-tile kernel: all four groups
// of slot threadIdx.x, i.e. two streams; the split kernel: two groups, one stream).
// UIN: the uniforms come from u_in (tests pin them) instead of the streams -- a template
// flag, not a runtime test: a runtime branch around the u loads made the compiler wait
// vmcnt(0) before every group's math, draining every load in flight (the prefetch of the
// looping kernel included).
// SEGT: a full tile across tensor boundaries.  Each 8-element group takes its own segment's
// parameters (walked from the tile's first segment through the LDS table `so`: a thread's
// groups ascend); a group that itself straddles a boundary divides per element with its
// element's norm (the same correctly rounded quotients).
struct QSegs {
  const int64_t* so;  // seg_off (LDS copy)
  const float* nm;    // norms (LDS copy)
  int nseg, sg0, s_levels;
  bool biased;
};
template <int CW, int NG, bool UIN, bool SEGT = false>
CHOCO_DEV void quant_tile_math(const float (&d)[NG][kQPer], int64_t tile, int64_t n, const QParam& P0,
                               const QDiv& D0, float sf, const float* __restrict__ u_in, uint64_t seed,
                               uint64_t offset, uint8_t* __restrict__ lvl_plane, uint8_t* __restrict__ sign_plane,
                               float* __restrict__ dense_out, int g0 = 0, int st = -1, const QSegs* SG = nullptr) {
  constexpr int GS = kQThreads * kQPer;  // 2048
  if (st < 0) st = (int)threadIdx.x;
  const int64_t eb = tile * kQStreamTile + (int64_t)st * kQPer + (int64_t)g0 * GS;
  // the thread's uniform stream, drawn group by group in stream order (8 uniforms live at
  // a time, not 32: the registers go to resident waves instead)
  Xoro128 rng;
  const bool dense = dense_out != nullptr;
  QParam P = P0;
  QDiv D = D0;
  int s = SEGT ? SG->sg0 : 0;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if constexpr (!UIN) {
      if (((g0 + g) & 1) == 0) rng.seed(qrng_key(seed, offset), qstream_id(tile, g0 + g, st));
    }
    const int64_t e0 = eb + g * GS;
    bool straddle = false;
    if constexpr (SEGT) {
      const int s_prev = s;
      while (s + 1 < SG->nseg && SG->so[s + 1] <= e0) ++s;
      if (s != s_prev || g == 0) {
        P = qparam(SG->nm, SG->so, n, s, SG->s_levels, SG->biased);
        D.init(P.norm);
      }
      straddle = s + 1 < SG->nseg && SG->so[s + 1] <= e0 + kQPer - 1;
    }
    float lf[kQPer];
    uint32_t tmin_m1 = 0xFFFFFFFFu, qmax = 0u;
#pragma unroll
    for (int c = 0; c < kQPer; ++c) lf[c] = D.quot_nocheck(sf * fabsf(d[g][c]), tmin_m1, qmax);  // s * x.abs() / norm
    const bool gslow = D.group_slow(tmin_m1, qmax);
    if (__builtin_expect(__ballot(gslow) != 0, 0)) {
#pragma unroll
      for (int c = 0; c < kQPer; ++c)
        if (gslow) lf[c] = (sf * fabsf(d[g][c])) / P.norm;
    }
    float escale[SEGT ? kQPer : 1], enorm[SEGT ? kQPer : 1];  // (SEGT, straddling group: per element)
    if constexpr (SEGT) {
      if (straddle) {
        int se = s;
#pragma unroll
        for (int c = 0; c < kQPer; ++c) {
          while (se + 1 < SG->nseg && SG->so[se + 1] <= e0 + c) ++se;
          const QParam Q = qparam(SG->nm, SG->so, n, se, SG->s_levels, SG->biased);
          lf[c] = (sf * fabsf(d[g][c])) / Q.norm;
          escale[c] = Q.scale;
          enorm[c] = Q.norm;
        }
      }
    }
    float u[kQPer];
    if constexpr (UIN) {
      const float4 u0 = *reinterpret_cast<const float4*>(u_in + e0);
      const float4 u1 = *reinterpret_cast<const float4*>(u_in + e0 + 4);
      u[0] = u0.x; u[1] = u0.y; u[2] = u0.z; u[3] = u0.w;
      u[4] = u1.x; u[5] = u1.y; u[6] = u1.z; u[7] = u1.w;
    } else {
#pragma unroll
      for (int c = 0; c < kQPer; c += 2) rng.next2(u[c], u[c + 1]);
    }
    uint32_t lv[kQPer];
    uint32_t sbits = 0;
    float lvlf[kQPer];
#pragma unroll
    for (int c = 0; c < kQPer; ++c) {
      lvlf[c] = qlevel(lf[c], u[c]);
      lv[c] = level_code(lvlf[c], sf);
      sbits |= d[g][c] < 0.f ? (1u << c) : 0u;
    }
    const int64_t t = e0 / kQPer;
    store_levels<CW>(lvl_plane, t, lv);
    sign_plane[t] = (uint8_t)sbits;
    if (dense) {  // one branch per group (a branch per element made the compiler shuffle the group's registers)
      float outv[kQPer];
#pragma unroll
      for (int c = 0; c < kQPer; ++c) {
        const float sg = d[g][c] > 0.f ? 1.0f : (d[g][c] < 0.f ? -1.0f : 0.0f);  // torch.sign (NaN -> 0)
        float sc = P.scale, nr = P.norm;
        if constexpr (SEGT) {
          if (straddle) {
            sc = escale[c];
            nr = enorm[c];
          }
        }
        outv[c] = (((sc * sg) * nr) * lvlf[c]) / sf;
      }
      *reinterpret_cast<float4*>(dense_out + e0) = make_float4(outv[0], outv[1], outv[2], outv[3]);
      *reinterpret_cast<float4*>(dense_out + e0 + 4) = make_float4(outv[4], outv[5], outv[6], outv[7]);
    }
  }
}

// Occupancy of the one-tile quantize kernel (waves per SIMD the compiler must allow).
// r04 same-box A/B at 100M: 4 -> 131 us, 6 -> 132, 8 -> 136 (more waves did not hide
// more latency: the 64-VGPR build spills one float4).
constexpr int kQQWaves = 4;
// H = 2 (the plain delta): a 512-thread workgroup per tile, each stream's four groups
// split over two threads (waves 0-3 take groups 0-1, waves 4-7 groups 2-3 after stepping
// their stream past the first eight uniforms) -- half the registers per thread, twice
// the waves resident, the same uniforms; compiled for 6 waves per SIMD.
constexpr int kQQHWaves = 6;
template <int CW, bool XH, int H, bool UIN>
__global__ __launch_bounds__(kQThreads * H, H == 1 ? kQQWaves : kQQHWaves) void qsgd_quant_kernel(
    const float* __restrict__ x, const float* __restrict__ xh, int64_t n, const int64_t* __restrict__ seg_off,
    int nseg, int s_levels, int biased, const float* __restrict__ norms, const float* __restrict__ u_in,
    uint64_t seed, uint64_t offset, uint8_t* __restrict__ lvl_plane, uint8_t* __restrict__ sign_plane,
    float* __restrict__ dense_out, int64_t tile_lo, int64_t tile_cnt, int64_t pad_e0, int64_t pad_len) {
  __shared__ int s_seg[2];
  __shared__ int64_t s_so[kSegLdsCap];
  __shared__ float s_nm[kSegLdsCap];
  // tiles [tile_lo, tile_lo + tile_cnt) of the buffer, walked in reverse (Infinity-Cache hits)
  const int64_t tile = tile_lo + tile_cnt - 1 - (int64_t)blockIdx.x;
  const int64_t t_e0 = tile * kQStreamTile;
  const int64_t t_e1 = std::min<int64_t>(t_e0 + kQStreamTile, n);
  const bool full = t_e1 - t_e0 == kQStreamTile;
  constexpr int NG = kQG / H;                                // groups per thread
  const int st = (int)(threadIdx.x % kQThreads);             // the thread's uniform stream
  const int g0 = (int)(threadIdx.x / kQThreads) * NG;        // its first group (wave-uniform)
  constexpr int GS = kQThreads * kQPer;                      // 2048
  const int64_t eb = t_e0 + (int64_t)st * kQPer + (int64_t)g0 * GS;  // group g0 + g starts at eb + g * 2048
  // a full tile's loads go out first (the delta's last read: the norm pass read it first);
  // a per-tensor layout's segment lookup then runs while they are in flight
  float4 a[NG][2], hq[XH ? NG : 1][2];
  if (full) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      a[g][0] = ld_quant4(x + eb + g * GS);
      a[g][1] = ld_quant4(x + eb + g * GS + 4);
    }
    if constexpr (XH) {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        hq[g][0] = ld_quant4(xh + eb + g * GS);
        hq[g][1] = ld_quant4(xh + eb + g * GS + 4);
      }
    }
  }
  // (the norms ride along with the table: the tile's parameters then need no further round trip)
  const float* nm = norms;
  if (nseg > 1 && nseg + 1 <= kSegLdsCap) {
    for (int i = threadIdx.x; i < nseg; i += blockDim.x) s_nm[i] = norms[i];
    nm = s_nm;
  }
  const int64_t* so = nseg > 1 ? stage_seg_off(seg_off, nseg, s_so) : seg_off;
  const int sg0 = tile_seg(so, nseg, t_e0, t_e1, s_seg);
  const bool uniform = s_seg[1] == sg0;
  if (blockIdx.x == 0) {
    // the planes of elements [pad_e0, pad_e0 + pad_len) are fully defined: zero their
    // 16-byte padding tails (the planes are indexed by absolute element group)
    const int64_t g0 = pad_e0 / kQPer, groups = (pad_len + kQPer - 1) / kQPer;
    const int64_t lvl_used = (g0 + groups) * CW, lvl_end = g0 * CW + (groups * CW + 15) / 16 * 16;
    const int64_t sgn_used = g0 + groups, sgn_end = g0 + (groups + 15) / 16 * 16;
    for (int64_t b = lvl_used + threadIdx.x; b < lvl_end; b += kQThreads * H) lvl_plane[b] = 0;
    for (int64_t b = sgn_used + threadIdx.x; b < sgn_end; b += kQThreads * H) sign_plane[b] = 0;
  }
  const float sf = (float)s_levels;
  if (!full) {
    if (threadIdx.x < kQThreads)  // (no barrier below: the second half leaves)
      qsgd_quant_tile_slow<CW>(x, xh, n, so, nseg, s_levels, biased, norms, u_in, seed, offset, lvl_plane,
                               sign_plane, dense_out, tile, sg0);
    return;
  }
  // full one-segment tile
  float d[NG][kQPer];
  {
    if constexpr (XH) {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        a[g][0] = sub4(a[g][0], hq[g][0]);
        a[g][1] = sub4(a[g][1], hq[g][1]);
      }
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      d[g][0] = a[g][0].x; d[g][1] = a[g][0].y; d[g][2] = a[g][0].z; d[g][3] = a[g][0].w;
      d[g][4] = a[g][1].x; d[g][5] = a[g][1].y; d[g][6] = a[g][1].z; d[g][7] = a[g][1].w;
    }
  }
  const QParam P = qparam(nm, so, n, sg0, s_levels, biased != 0);
  QDiv D;
  D.init(P.norm);
  if (uniform) {
    quant_tile_math<CW, NG, UIN>(d, tile, n, P, D, sf, u_in, seed, offset, lvl_plane, sign_plane, dense_out, g0, st);
  } else {
    const QSegs SG{so, nm, nseg, sg0, s_levels, biased != 0};
    quant_tile_math<CW, NG, UIN, true>(d, tile, n, P, D, sf, u_in, seed, offset, lvl_plane, sign_plane, dense_out,
                                       g0, st, &SG);
  }
}

// ---------------------------------------------------------------- decode / accumulate
struct QMsgs {
  const uint8_t* lvl[kQMaxMsg];
  const uint8_t* sgn[kQMaxMsg];
  const float* norms[kQMaxMsg];
  float w[kQMaxMsg];
  int nmsg;
  int self_slot;
  int extrap;  // 1: memory = fmaf(w, v, memory * a) (ECD, ecd_psgd.py:421-423)
  float a;
};

CHOCO_DEV float qdecode(uint32_t level, bool neg, const QParam& P, float sf) {
  const float lvl = (P.norm == 0.0f) ? __int_as_float(0x7fc00000) : (float)level;  // ref: 0/0 -> NaN
  const float sg = neg ? -1.0f : 1.0f;
  return (((P.scale * sg) * P.norm) * lvl) / sf;
}

// (non-temporal stores: whole steps within noise, qsgd 0.4735-0.4770 against 0.4735-0.4804 ms;
// loads + stores: the decode 271 -> 300 us, qsgd 0.475-0.480 -> 0.489-0.493 ms; r05_ab_summary.txt
// items 21, 24)
CHOCO_DEV float4 qdec_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
CHOCO_DEV void st_dec4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// MODE 0: out = decode(msg 0); MODE 1: accumulate all messages into hat/mem.
// SEG: a per-tensor layout (nseg > 1); the flat instantiation drops the segment lookups and
// the per-element segment walk (3-message decode 96 -> 59 VGPRs: the ring step's receive
// at 100M 330-333 -> 295 us, profiles/r06_ab_summary.txt item 16).
template <int CW, int NM, int MODE, bool SEG>
__global__ __launch_bounds__(kQThreads) void qsgd_decode_kernel(QMsgs M, int64_t n,
                                                                const int64_t* __restrict__ seg_off, int nseg,
                                                                int s_levels, int biased,
                                                                float* __restrict__ hat, float* __restrict__ mem,
                                                                int64_t blk_lo) {
  __shared__ int s_seg[2];
  const int64_t t_e0 = (blk_lo + (int64_t)blockIdx.x) * kQTile;
  const int64_t t_e1 = std::min<int64_t>(t_e0 + kQTile, n);
  const int sg0 = SEG ? tile_seg(seg_off, nseg, t_e0, t_e1, s_seg) : 0;
  const bool uniform = !SEG || s_seg[1] == sg0;
  const int64_t e0 = t_e0 + (int64_t)threadIdx.x * kQPer;
  if (e0 >= n) return;
  const float sf = (float)s_levels;
  const int64_t t = e0 / kQPer;
  const bool full = e0 + kQPer <= n;
  float mv[kQPer], hv[kQPer];
  const bool has_self = MODE == 1 && M.self_slot >= 0 && hat != nullptr;
  if (MODE == 1) {
    if (full) {
      const float4 a0 = qdec_ld4(mem + e0);
      const float4 a1 = qdec_ld4(mem + e0 + 4);
      mv[0] = a0.x; mv[1] = a0.y; mv[2] = a0.z; mv[3] = a0.w; mv[4] = a1.x; mv[5] = a1.y; mv[6] = a1.z; mv[7] = a1.w;
      if (has_self) {
        const float4 b0 = qdec_ld4(hat + e0);
        const float4 b1 = qdec_ld4(hat + e0 + 4);
        hv[0] = b0.x; hv[1] = b0.y; hv[2] = b0.z; hv[3] = b0.w; hv[4] = b1.x; hv[5] = b1.y; hv[6] = b1.z; hv[7] = b1.w;
      }
    } else {
#pragma unroll
      for (int c = 0; c < kQPer; ++c) {
        mv[c] = (e0 + c < n) ? mem[e0 + c] : 0.f;
        hv[c] = (has_self && e0 + c < n) ? hat[e0 + c] : 0.f;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NM; ++q) {
    uint32_t lv[kQPer];
    load_levels<CW>(M.lvl[q], t, lv);
    const uint32_t sb = M.sgn[q][t];
    QParam P = qparam(M.norms[q], seg_off, n, sg0, s_levels, biased != 0);
#pragma unroll
    for (int c = 0; c < kQPer; ++c) {
      const int64_t e = e0 + c;
      if (!uniform && e < n) {
        int s = sg0;
        while (s + 1 < nseg && seg_off[s + 1] <= e) ++s;
        P = qparam(M.norms[q], seg_off, n, s, s_levels, biased != 0);
      }
      const float v = qdecode(lv[c], (sb >> c) & 1u, P, sf);
      if (MODE == 0) {
        mv[c] = v;
      } else {
        if (has_self && q == M.self_slot) hv[c] = hv[c] + v;  // hat_params.buffer += q_values
        if (M.extrap) {
          mv[c] = fmaf(M.w[q], v, mv[c] * M.a);  // hat.mul_(a).add_(q, alpha=b)
        } else {
          const float wv = M.w[q] * v;                        // weight * q_values (rounded)
          mv[c] = mv[c] + wv;                                  // memory += ...
        }
      }
    }
  }
  float* dst = MODE == 0 ? hat : mem;  // MODE 0 writes the decoded floats to `hat` (= out)
  if (full) {
    st_dec4(dst + e0, make_float4(mv[0], mv[1], mv[2], mv[3]));
    st_dec4(dst + e0 + 4, make_float4(mv[4], mv[5], mv[6], mv[7]));
    if (has_self) {
      st_dec4(hat + e0, make_float4(hv[0], hv[1], hv[2], hv[3]));
      st_dec4(hat + e0 + 4, make_float4(hv[4], hv[5], hv[6], hv[7]));
    }
  } else {
    for (int c = 0; c < kQPer; ++c) {
      if (e0 + c >= n) break;
      dst[e0 + c] = mv[c];
      if (has_self) hat[e0 + c] = hv[c];
    }
  }
}

// ---------------------------------------------------------------- deferred receive, fused
// The previous step's receive (CHOCOQuantizationCompressor.uncompress, parallel_choco_v.py:
// 430-433: x_hat += q_self, memory += w * q per message in neighbors_info order), this
// step's consensus step (update_params_from_neighbor, optim/utils.py:67-72: x += gamma
// (memory - x_hat)) and this step's norm pass (per-segment ||x_new - x_hat||_2, fp64) in
// ONE pass over x, x_hat and memory.  Every step is elementwise, so the results are those of
// the decode, gossip and norm passes run one after the other; the step's SGD update of x
// comes first, as in ParallelCHOCO_V.step (apply_gradient, then the previous gossip's join).
// Thread t: kRG 8-element groups (the planes' groups) t_e0 + g * 2048 + 8 t; every load of
// both groups in flight before any arithmetic.  fp64 sums go to kAccRep replicas of the
// per-segment accumulators (workgroup b -> replica b & 7: 24K workgroups at 100M would
// otherwise queue on one address); the last workgroup sums the replicas.
constexpr int kRG = 2;
constexpr int kRTile = kQTile * kRG;  // 4096 elements per workgroup
template <int CW, int NM, bool SEG>  // (SEG: as qsgd_decode_kernel)
__global__ __launch_bounds__(kQThreads) void qsgd_recv_gossip_norm_kernel(
    QMsgs M, int64_t n, const int64_t* __restrict__ seg_off, int nseg, int s_levels, int biased,
    float* __restrict__ x, float* __restrict__ hat, float* __restrict__ mem, float gamma,
    QsgdWs* __restrict__ ws, float* __restrict__ norms_out) {
  __shared__ int s_seg[2];
  __shared__ double s_red[kQThreads / 64];
  __shared__ unsigned int s_flag;
  double* __restrict__ acc = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + 256);
  double* __restrict__ rep = acc + (size_t)(blockIdx.x & (kAccRep - 1)) * (size_t)nseg;
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int64_t t_e0 = (int64_t)blockIdx.x * kRTile;
  const int64_t t_e1 = std::min<int64_t>(t_e0 + kRTile, n);
  const int sg0 = SEG ? tile_seg(seg_off, nseg, t_e0, t_e1, s_seg) : 0;
  const bool uniform = !SEG || s_seg[1] == sg0;
  const float sf = (float)s_levels;
  const bool has_self = M.self_slot >= 0;
  float xv[kRG][kQPer], hv[kRG][kQPer], mv[kRG][kQPer];
  LevelWords<CW> lw[kRG][NM];
  uint32_t sb[kRG][NM];
  // ---- loads of both groups (a group past n is skipped; the buffer's last group is partial)
#pragma unroll
  for (int g = 0; g < kRG; ++g) {
    const int64_t e0 = t_e0 + (int64_t)g * kQTile + (int64_t)tid * kQPer;
    if (e0 >= n) continue;
    if (e0 + kQPer <= n) {
      const float4 a0 = *reinterpret_cast<const float4*>(x + e0), a1 = *reinterpret_cast<const float4*>(x + e0 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(hat + e0), b1 = *reinterpret_cast<const float4*>(hat + e0 + 4);
      const float4 c0 = *reinterpret_cast<const float4*>(mem + e0), c1 = *reinterpret_cast<const float4*>(mem + e0 + 4);
      xv[g][0] = a0.x; xv[g][1] = a0.y; xv[g][2] = a0.z; xv[g][3] = a0.w;
      xv[g][4] = a1.x; xv[g][5] = a1.y; xv[g][6] = a1.z; xv[g][7] = a1.w;
      hv[g][0] = b0.x; hv[g][1] = b0.y; hv[g][2] = b0.z; hv[g][3] = b0.w;
      hv[g][4] = b1.x; hv[g][5] = b1.y; hv[g][6] = b1.z; hv[g][7] = b1.w;
      mv[g][0] = c0.x; mv[g][1] = c0.y; mv[g][2] = c0.z; mv[g][3] = c0.w;
      mv[g][4] = c1.x; mv[g][5] = c1.y; mv[g][6] = c1.z; mv[g][7] = c1.w;
    } else {
#pragma unroll
      for (int c = 0; c < kQPer; ++c) {
        const bool in = e0 + c < n;
        xv[g][c] = in ? x[e0 + c] : 0.f;
        hv[g][c] = in ? hat[e0 + c] : 0.f;
        mv[g][c] = in ? mem[e0 + c] : 0.f;
      }
    }
    const int64_t t = e0 / kQPer;
#pragma unroll
    for (int q = 0; q < NM; ++q) {
      lw[g][q] = load_level_words<CW>(M.lvl[q], t);
      sb[g][q] = M.sgn[q][t];
    }
  }
  // ---- receive, consensus step, stores, sums of squares
  double p = 0.0;         // uniform tile: this thread's sum
  int run_s = -1;         // otherwise: the current segment run and its sum
  double run_p = 0.0;
#pragma unroll
  for (int g = 0; g < kRG; ++g) {
    const int64_t e0 = t_e0 + (int64_t)g * kQTile + (int64_t)tid * kQPer;
    if (e0 >= n) continue;
    QParam P[NM];
#pragma unroll
    for (int q = 0; q < NM; ++q) P[q] = qparam(M.norms[q], seg_off, n, sg0, s_levels, biased != 0);
    int s = sg0;
#pragma unroll
    for (int c = 0; c < kQPer; ++c) {
      const int64_t e = e0 + c;
      if (!uniform && e < n) {
        while (s + 1 < nseg && seg_off[s + 1] <= e) ++s;
#pragma unroll
        for (int q = 0; q < NM; ++q) P[q] = qparam(M.norms[q], seg_off, n, s, s_levels, biased != 0);
      }
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        const float v = qdecode(level_of<CW>(lw[g][q], c), (sb[g][q] >> c) & 1u, P[q], sf);
        if (has_self && q == M.self_slot) hv[g][c] = hv[g][c] + v;  // hat_params.buffer += q_values
        const float wv = M.w[q] * v;                                  // weight * q_values (rounded)
        mv[g][c] = mv[g][c] + wv;                                     // memory += ...
      }
      xv[g][c] = gossip1(xv[g][c], mv[g][c], hv[g][c], gamma);
      const double d = (double)(xv[g][c] - hv[g][c]);
      if (e < n) {
        if (uniform) {
          p += d * d;
        } else {
          if (s != run_s) {
            if (run_s >= 0 && run_p != 0.0) unsafeAtomicAdd(&rep[run_s], run_p);
            run_s = s;
            run_p = 0.0;
          }
          run_p += d * d;
        }
      }
    }
    if (e0 + kQPer <= n) {
      // (plain stores: non-temporal x / x_hat / memory, or memory alone, measured the same
      // in the deferred step, profiles/r05_ab_summary.txt item 11)
      *reinterpret_cast<float4*>(x + e0) = make_float4(xv[g][0], xv[g][1], xv[g][2], xv[g][3]);
      *reinterpret_cast<float4*>(x + e0 + 4) = make_float4(xv[g][4], xv[g][5], xv[g][6], xv[g][7]);
      *reinterpret_cast<float4*>(mem + e0) = make_float4(mv[g][0], mv[g][1], mv[g][2], mv[g][3]);
      *reinterpret_cast<float4*>(mem + e0 + 4) = make_float4(mv[g][4], mv[g][5], mv[g][6], mv[g][7]);
      if (has_self) {
        *reinterpret_cast<float4*>(hat + e0) = make_float4(hv[g][0], hv[g][1], hv[g][2], hv[g][3]);
        *reinterpret_cast<float4*>(hat + e0 + 4) = make_float4(hv[g][4], hv[g][5], hv[g][6], hv[g][7]);
      }
    } else {
      for (int c = 0; c < kQPer && e0 + c < n; ++c) {
        x[e0 + c] = xv[g][c];
        mem[e0 + c] = mv[g][c];
        if (has_self) hat[e0 + c] = hv[g][c];
      }
    }
  }
  if (uniform) {
    p = wave_sum(p);
    if (lane == 0) s_red[w] = p;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int i = 0; i < kQThreads / 64; ++i) t += s_red[i];
      if (t != 0.0) unsafeAtomicAdd(&rep[sg0], t);
    }
  } else if (run_s >= 0 && run_p != 0.0) {
    unsafeAtomicAdd(&rep[run_s], run_p);
  }
  if (last_block_ticket_atomics(&ws->ticket, gridDim.x, &s_flag)) {
    for (int q = threadIdx.x; q < nseg; q += blockDim.x) {
      double t = 0.0;
      for (int r = 0; r < kAccRep; ++r) t += atomic_exchange_double(&acc[(size_t)r * nseg + q], 0.0);
      norms_out[q] = (float)sqrt(t);
    }
    if (threadIdx.x == 0) __hip_atomic_store(&ws->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int CW>
static void launch_recv_gossip(const QMsgs& M, int64_t n, const int64_t* seg_off, int nseg, int s_levels,
                               int biased, float* x, float* hat, float* mem, float gamma, QsgdWs* ws, float* norms,
                               hipStream_t st) {
  const unsigned grid = (unsigned)((n + kRTile - 1) / kRTile);
#define CHOCO_RG(NMV)                                                                                      \
  case NMV:                                                                                                \
    if (nseg > 1)                                                                                          \
      CHOCO_KLAUNCH((qsgd_recv_gossip_norm_kernel<CW, NMV, true>), dim3(grid), dim3(kQThreads), 0, st, M, n, \
                    seg_off, nseg, s_levels, biased, x, hat, mem, gamma, ws, norms);                       \
    else                                                                                                   \
      CHOCO_KLAUNCH((qsgd_recv_gossip_norm_kernel<CW, NMV, false>), dim3(grid), dim3(kQThreads), 0, st, M,   \
                    n, seg_off, nseg, s_levels, biased, x, hat, mem, gamma, ws, norms);                    \
    break;
  switch (M.nmsg) {
    CHOCO_RG(1)
    CHOCO_RG(2)
    CHOCO_RG(3)
    CHOCO_RG(4)
    CHOCO_RG(5)
    CHOCO_RG(6)
    CHOCO_RG(7)
    CHOCO_RG(8)
  }
#undef CHOCO_RG
}

// Elements [e0, e1) (e0 a multiple of kQTile; e1 a multiple of it or n).
template <int CW, int NM, int MODE>
static void launch_decode(const QMsgs& M, int64_t n, const int64_t* seg_off, int nseg, int s_levels, int biased,
                          float* hat, float* mem, hipStream_t st, int64_t e0, int64_t e1) {
  const unsigned grid = (unsigned)((e1 - e0 + kQTile - 1) / kQTile);
  if (nseg > 1)
    CHOCO_KLAUNCH((qsgd_decode_kernel<CW, NM, MODE, true>), dim3(grid), dim3(kQThreads), 0, st, M, n, seg_off, nseg,
                  s_levels, biased, hat, mem, e0 / kQTile);
  else
    CHOCO_KLAUNCH((qsgd_decode_kernel<CW, NM, MODE, false>), dim3(grid), dim3(kQThreads), 0, st, M, n, seg_off, nseg,
                  s_levels, biased, hat, mem, e0 / kQTile);
}

template <int CW, int MODE>
static void launch_decode_nm(const QMsgs& M, int64_t n, const int64_t* seg_off, int nseg, int s_levels,
                             int biased, float* hat, float* mem, hipStream_t st, int64_t e0, int64_t e1) {
  switch (M.nmsg) {
    case 1: launch_decode<CW, 1, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 2: launch_decode<CW, 2, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 3: launch_decode<CW, 3, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 4: launch_decode<CW, 4, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 5: launch_decode<CW, 5, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 6: launch_decode<CW, 6, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 7: launch_decode<CW, 7, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    default: launch_decode<CW, 8, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
  }
}

template <int MODE>
static void launch_decode_cw(int cw, const QMsgs& M, int64_t n, const int64_t* seg_off, int nseg, int s_levels,
                             int biased, float* hat, float* mem, hipStream_t st, int64_t e0 = 0, int64_t e1 = -1) {
  if (e1 < 0) e1 = n;
  switch (cw) {
    case 1: launch_decode_nm<1, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 2: launch_decode_nm<2, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 4: launch_decode_nm<4, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    case 8: launch_decode_nm<8, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
    default: launch_decode_nm<16, MODE>(M, n, seg_off, nseg, s_levels, biased, hat, mem, st, e0, e1); break;
  }
}

}  // namespace choco

using namespace choco;

CHOCO_API int64_t choco_qsgd_packed_bytes(int64_t n, int32_t q) {
  if (n <= 0 || q < 1 || q > 16) return 0;
  return plane_bytes(n, container_bits(q)) + plane_bytes(n, 1);
}

CHOCO_API size_t choco_qsgd_workspace_size(int32_t nseg) {
  // the ticket, then kAccRep replicas of the per-segment fp64 accumulators (the norm pass
  // uses replica 0; the fused receive pass all of them)
  return 256 + align_up((size_t)kAccRep * (size_t)(nseg > 0 ? nseg : 1) * sizeof(double), 256);
}

static int qsgd_check(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg) {
  CHOCO_REQUIRE(x, "null pointer argument");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(x) && (!xhat || aligned16(xhat)), "buffers must be 16-byte aligned");
  return CHOCO_OK;
}

// The norm pass (per-segment ||d||_2, fp64, rounded once); gs: the fused gossip step.
static int qsgd_norms_launch(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                             float* norms_out, void* ws, size_t ws_bytes, hipStream_t st, Gossip gs) {
  CHOCO_REQUIRE(!gs.mem || (xhat && aligned16(gs.mem)), "the gossip step needs x_hat and a 16-byte aligned memory");
  CHOCO_REQUIRE(norms_out, "norms_out is required when norm_in is NULL");
  CHOCO_REQUIRE(ws && ws_bytes >= choco_qsgd_workspace_size(nseg), "qsgd workspace too small");
  const int64_t tile = norm_tile(n);
  const unsigned g1 = (unsigned)((n + tile - 1) / tile);
  QsgdWs* w = static_cast<QsgdWs*>(ws);
  profile_begin("qsgd_norm", st);
if (gs.mem)
    CHOCO_KLAUNCH((qsgd_norm_kernel<true, true>), dim3(g1), dim3(kQThreads), 0, st, x, xhat, n, seg_off, nseg,
                  norms_out, w, gs, tile);
  else if (xhat)
    CHOCO_KLAUNCH((qsgd_norm_kernel<true>), dim3(g1), dim3(kQThreads), 0, st, x, xhat, n, seg_off, nseg,
                  norms_out, w, gs, tile);
  else
    CHOCO_KLAUNCH((qsgd_norm_kernel<false>), dim3(g1), dim3(kQThreads), 0, st, x, xhat, n, seg_off, nseg,
                  norms_out, w, gs, tile);
  profile_end("qsgd_norm", st);
  CHOCO_LAUNCHED("qsgd_norm_kernel");
  return CHOCO_OK;
}

// The quantize pass over elements [e0, e1) into planes indexed by ABSOLUTE element
// group (lvl_plane / sign_plane point at element 0's group; a range call writes
// only the groups of its elements, plus the 16-byte padding of a plane that ends
// at e1).
// split streams for the plain delta only: with x_hat (the gossip form) the one-stream
// threads measured faster (r4u2: 151.5-153.4 against 154.8-157.6 us).  Measured slower and
// removed from the source (git history: r04): a looping kernel with the next tile's loads
// in flight (141-147 us, also with its prefetch as asm loads), an LDS-DMA ring (149-156 us)
// -- against 122-128 us for this one-tile kernel.
constexpr int kQH = 2;
static int qsgd_quant_launch(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                             int32_t q, int32_t is_biased, const float* norms, const float* u_in, uint64_t seed,
                             uint64_t offset, uint8_t* lvl_plane, uint8_t* sign_plane, float* dense_out,
                             int64_t e0, int64_t e1, int64_t pad_e0, hipStream_t st) {
  const int cw = container_bits(q);
  const int s_levels = (1 << q) - 1;
  const int64_t tile_lo = e0 / kQStreamTile;
  const int64_t tile_cnt = (e1 - e0 + kQStreamTile - 1) / kQStreamTile;
  profile_begin("qsgd_quantize", st);
#define CHOCO_Q1(CWV, XHV, UINV)                                                                              \
  CHOCO_KLAUNCH((qsgd_quant_kernel<CWV, XHV, XHV ? 1 : kQH, UINV>), dim3((unsigned)tile_cnt),                  \
                dim3(kQThreads * (XHV ? 1 : kQH)), 0,                                                          \
                st, x, xhat, n, seg_off, nseg, s_levels, is_biased, norms, u_in, seed, offset, lvl_plane,      \
                sign_plane, dense_out, tile_lo, tile_cnt, pad_e0, e1 - pad_e0)
#define CHOCO_Q(CWV)                                                                                          \
  case CWV:                                                                                                   \
    if (xhat) {                                                                                               \
      if (u_in) CHOCO_Q1(CWV, true, true); else CHOCO_Q1(CWV, true, false);                                   \
    } else {                                                                                                  \
      if (u_in) CHOCO_Q1(CWV, false, true); else CHOCO_Q1(CWV, false, false);                                 \
    }                                                                                                         \
    break;
  switch (cw) {
    CHOCO_Q(1)
    CHOCO_Q(2)
    CHOCO_Q(4)
    CHOCO_Q(8)
    CHOCO_Q(16)
  }
#undef CHOCO_Q
#undef CHOCO_Q1
  profile_end("qsgd_quantize", st);
  CHOCO_LAUNCHED("qsgd_quant_kernel");
  return CHOCO_OK;
}

static int qsgd_compress(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                         int32_t q, int32_t is_biased, const float* norm_in, const float* u_in, uint64_t seed,
                         uint64_t offset, uint8_t* packed, float* norms_out, float* dense_out, void* ws,
                         size_t ws_bytes, hipStream_t st, Gossip gs) {
  CHOCO_REQUIRE(x && packed, "null pointer argument");
  CHOCO_REQUIRE(q >= 1 && q <= 16, "quantize level q must be in [1, 16] (q = 32 is a passthrough), got %d", q);
  if (int rc = qsgd_check(x, xhat, n, seg_off, nseg)) return rc;
  CHOCO_REQUIRE(aligned16(packed) && (!dense_out || aligned16(dense_out)), "buffers must be 16-byte aligned");
  const int cw = container_bits(q);
  const float* norms = norm_in;
  if (!norms) {
    if (int rc = qsgd_norms_launch(x, xhat, n, seg_off, nseg, norms_out, ws, ws_bytes, st, gs)) return rc;
    norms = norms_out;
  } else {
    // pinned norms (parity mode): no norm pass to fuse the gossip step into
    CHOCO_REQUIRE(!gs.mem || (xhat && aligned16(gs.mem)), "the gossip step needs x_hat and a 16-byte aligned memory");
    if (gs.mem) {
      const int rc = gossip_launch(const_cast<float*>(x), gs.mem, xhat, gs.gamma, n, st);
      if (rc) return rc;
    }
    if (norms_out && norms_out != norm_in)
      CHOCO_HIP(hipMemcpyAsync(norms_out, norm_in, sizeof(float) * nseg, hipMemcpyDeviceToDevice, st));
  }
  return qsgd_quant_launch(x, xhat, n, seg_off, nseg, q, is_biased, norms, u_in, seed, offset, packed,
                           packed + plane_bytes(n, cw), dense_out, 0, n, 0, st);
}

// A range [e0, e1) of a chunked wire: e0 a multiple of kQStreamTile, e1 one too or n.
static int qsgd_range_ok(int64_t n, int64_t e0, int64_t e1) {
  CHOCO_REQUIRE(e0 >= 0 && e0 < e1 && e1 <= n && e0 % kQStreamTile == 0 && (e1 % kQStreamTile == 0 || e1 == n),
                "range [%lld, %lld) of n=%lld: e0 must be a multiple of %d, e1 one too or n", (long long)e0,
                (long long)e1, (long long)n, kQStreamTile);
  return CHOCO_OK;
}

// The planes of a range message (packed_range = [level plane | sign plane] of e1 - e0
// elements, choco_qsgd_packed_bytes(e1 - e0, q) bytes) as absolute-group pointers.
static void range_planes(const uint8_t* packed_range, int64_t e0, int64_t len, int cw, const uint8_t** lvl,
                         const uint8_t** sgn) {
  const uintptr_t base = reinterpret_cast<uintptr_t>(packed_range);
  *lvl = reinterpret_cast<const uint8_t*>(base - (uintptr_t)((e0 / kQPer) * cw));
  *sgn = reinterpret_cast<const uint8_t*>(base + (uintptr_t)plane_bytes(len, cw) - (uintptr_t)(e0 / kQPer));
}

CHOCO_API int choco_qsgd_compress(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                                  int32_t q, int32_t is_biased, const float* norm_in, const float* u_in,
                                  uint64_t seed, uint64_t offset, uint8_t* packed, float* norms_out,
                                  float* dense_out, void* ws, size_t ws_bytes, void* stream) {
  return qsgd_compress(x, xhat, n, seg_off, nseg, q, is_biased, norm_in, u_in, seed, offset, packed, norms_out,
                       dense_out, ws, ws_bytes, as_stream(stream), Gossip{nullptr, 0.f});
}

CHOCO_API int choco_gossip_qsgd_compress(float* x, const float* memory, const float* xhat, float gamma, int64_t n,
                                         const int64_t* seg_off, int32_t nseg, int32_t q, int32_t is_biased,
                                         uint64_t seed, uint64_t offset, uint8_t* packed, float* norms_out,
                                         float* dense_out, void* ws, size_t ws_bytes, void* stream) {
  CHOCO_REQUIRE(memory != nullptr && xhat != nullptr, "the gossip step needs memory and x_hat");
  return qsgd_compress(x, xhat, n, seg_off, nseg, q, is_biased, nullptr, nullptr, seed, offset, packed, norms_out,
                       dense_out, ws, ws_bytes, as_stream(stream), Gossip{memory, gamma});
}

CHOCO_API int choco_qsgd_norms(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                               float* norms_out, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = qsgd_check(x, xhat, n, seg_off, nseg)) return rc;
  return qsgd_norms_launch(x, xhat, n, seg_off, nseg, norms_out, ws, ws_bytes, as_stream(stream),
                           Gossip{nullptr, 0.f});
}

CHOCO_API int choco_gossip_qsgd_norms(float* x, const float* memory, const float* xhat, float gamma, int64_t n,
                                      const int64_t* seg_off, int32_t nseg, float* norms_out, void* ws,
                                      size_t ws_bytes, void* stream) {
  CHOCO_REQUIRE(memory != nullptr && xhat != nullptr, "the gossip step needs memory and x_hat");
  if (int rc = qsgd_check(x, xhat, n, seg_off, nseg)) return rc;
  return qsgd_norms_launch(x, xhat, n, seg_off, nseg, norms_out, ws, ws_bytes, as_stream(stream),
                           Gossip{memory, gamma});
}

CHOCO_API int choco_qsgd_quantize_range(const float* x, const float* xhat, int64_t n, const int64_t* seg_off,
                                        int32_t nseg, int32_t q, int32_t is_biased, const float* norms,
                                        uint64_t seed, uint64_t offset, int64_t e0, int64_t e1,
                                        uint8_t* packed_range, void* stream) {
  CHOCO_REQUIRE(norms && packed_range, "null pointer argument");
  CHOCO_REQUIRE(q >= 1 && q <= 16, "quantize level q must be in [1, 16], got %d", q);
  if (int rc = qsgd_check(x, xhat, n, seg_off, nseg)) return rc;
  if (int rc = qsgd_range_ok(n, e0, e1)) return rc;
  CHOCO_REQUIRE(aligned16(packed_range), "packed_range must be 16-byte aligned");
  const int cw = container_bits(q);
  const uint8_t *lvl, *sgn;
  range_planes(packed_range, e0, e1 - e0, cw, &lvl, &sgn);
  return qsgd_quant_launch(x, xhat, n, seg_off, nseg, q, is_biased, norms, nullptr, seed, offset,
                           const_cast<uint8_t*>(lvl), const_cast<uint8_t*>(sgn), nullptr, e0, e1, e0,
                           as_stream(stream));
}

CHOCO_API int choco_qsgd_decompress_accumulate_range(const uint8_t* const* packed_list,
                                                     const float* const* norms_list, const float* weights,
                                                     int32_t nmsg, int32_t self_slot, int64_t n,
                                                     const int64_t* seg_off, int32_t nseg, int32_t q,
                                                     int32_t is_biased, int64_t e0, int64_t e1, float* xhat_self,
                                                     float* memory, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed_list && norms_list && weights && memory, "null pointer argument");
  CHOCO_REQUIRE(nmsg >= 1 && nmsg <= kQMaxMsg, "nmsg must be in [1, %d]", kQMaxMsg);
  CHOCO_REQUIRE(self_slot >= -1 && self_slot < nmsg, "bad self_slot");
  CHOCO_REQUIRE(q >= 1 && q <= 16, "q must be in [1, 16]");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(memory) && (!xhat_self || aligned16(xhat_self)), "buffers must be 16-byte aligned");
  if (int rc = qsgd_range_ok(n, e0, e1)) return rc;
  const int cw = container_bits(q);
  QMsgs M{};
  for (int m = 0; m < nmsg; ++m) {
    CHOCO_REQUIRE(packed_list[m] && norms_list[m], "null message pointer");
    CHOCO_REQUIRE(aligned16(packed_list[m]), "packed messages must be 16-byte aligned");
    range_planes(packed_list[m], e0, e1 - e0, cw, &M.lvl[m], &M.sgn[m]);
    M.norms[m] = norms_list[m];
    M.w[m] = weights[m];
  }
  M.nmsg = nmsg;
  M.self_slot = self_slot;
  profile_begin("qsgd_accumulate", st);
  launch_decode_cw<1>(cw, M, n, seg_off, nseg, (1 << q) - 1, is_biased, xhat_self, memory, st, e0, e1);
  profile_end("qsgd_accumulate", st);
  CHOCO_LAUNCHED("qsgd_decode_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_qsgd_decode(const uint8_t* packed, const float* norms, int64_t n, const int64_t* seg_off,
                                int32_t nseg, int32_t q, int32_t is_biased, float* out, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed && norms && out, "null pointer argument");
  CHOCO_REQUIRE(q >= 1 && q <= 16, "q must be in [1, 16]");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(packed) && aligned16(out), "buffers must be 16-byte aligned");
  const int cw = container_bits(q);
  QMsgs M{};
  M.lvl[0] = packed;
  M.sgn[0] = packed + plane_bytes(n, cw);
  M.norms[0] = norms;
  M.w[0] = 1.0f;
  M.nmsg = 1;
  M.self_slot = -1;
  launch_decode_cw<0>(cw, M, n, seg_off, nseg, (1 << q) - 1, is_biased, out, nullptr, st);
  CHOCO_LAUNCHED("qsgd_decode_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_qsgd_decompress_accumulate(const uint8_t* const* packed_list, const float* const* norms_list,
                                               const float* weights, int32_t nmsg, int32_t self_slot, int64_t n,
                                               const int64_t* seg_off, int32_t nseg, int32_t q, int32_t is_biased,
                                               float* xhat_self, float* memory, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed_list && norms_list && weights && memory, "null pointer argument");
  CHOCO_REQUIRE(nmsg >= 1 && nmsg <= kQMaxMsg, "nmsg must be in [1, %d]", kQMaxMsg);
  CHOCO_REQUIRE(self_slot >= -1 && self_slot < nmsg, "bad self_slot");
  CHOCO_REQUIRE(q >= 1 && q <= 16, "q must be in [1, 16]");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(memory) && (!xhat_self || aligned16(xhat_self)), "buffers must be 16-byte aligned");
  const int cw = container_bits(q);
  QMsgs M{};
  for (int m = 0; m < nmsg; ++m) {
    CHOCO_REQUIRE(packed_list[m] && norms_list[m], "null message pointer");
    CHOCO_REQUIRE(aligned16(packed_list[m]), "packed messages must be 16-byte aligned");
    M.lvl[m] = packed_list[m];
    M.sgn[m] = packed_list[m] + plane_bytes(n, cw);
    M.norms[m] = norms_list[m];
    M.w[m] = weights[m];
  }
  M.nmsg = nmsg;
  M.self_slot = self_slot;
  profile_begin("qsgd_accumulate", st);
  launch_decode_cw<1>(cw, M, n, seg_off, nseg, (1 << q) - 1, is_biased, xhat_self, memory, st);
  profile_end("qsgd_accumulate", st);
  CHOCO_LAUNCHED("qsgd_decode_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_qsgd_recv_gossip_norms(const uint8_t* const* packed_list, const float* const* norms_list,
                                           const float* weights, int32_t nmsg, int32_t self_slot, float* x,
                                           float* memory, float* xhat, float gamma, int64_t n,
                                           const int64_t* seg_off, int32_t nseg, int32_t q, int32_t is_biased,
                                           float* norms_out, void* ws, size_t ws_bytes, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed_list && norms_list && weights && x && memory && xhat && norms_out, "null pointer argument");
  CHOCO_REQUIRE(nmsg >= 1 && nmsg <= kQMaxMsg, "nmsg must be in [1, %d]", kQMaxMsg);
  CHOCO_REQUIRE(self_slot >= -1 && self_slot < nmsg, "bad self_slot");
  CHOCO_REQUIRE(q >= 1 && q <= 16, "q must be in [1, 16]");
  if (int rc = qsgd_check(x, xhat, n, seg_off, nseg)) return rc;
  CHOCO_REQUIRE(aligned16(memory), "buffers must be 16-byte aligned");
  CHOCO_REQUIRE(ws && ws_bytes >= choco_qsgd_workspace_size(nseg), "qsgd workspace too small");
  const int cw = container_bits(q);
  QMsgs M{};
  for (int m = 0; m < nmsg; ++m) {
    CHOCO_REQUIRE(packed_list[m] && norms_list[m], "null message pointer");
    CHOCO_REQUIRE(aligned16(packed_list[m]), "packed messages must be 16-byte aligned");
    M.lvl[m] = packed_list[m];
    M.sgn[m] = packed_list[m] + plane_bytes(n, cw);
    M.norms[m] = norms_list[m];
    M.w[m] = weights[m];
  }
  M.nmsg = nmsg;
  M.self_slot = self_slot;
  const int s_levels = (1 << q) - 1;
  QsgdWs* w = static_cast<QsgdWs*>(ws);
  profile_begin("qsgd_recv_norm", st);
  switch (cw) {
    case 1: launch_recv_gossip<1>(M, n, seg_off, nseg, s_levels, is_biased, x, xhat, memory, gamma, w, norms_out, st); break;
    case 2: launch_recv_gossip<2>(M, n, seg_off, nseg, s_levels, is_biased, x, xhat, memory, gamma, w, norms_out, st); break;
    case 4: launch_recv_gossip<4>(M, n, seg_off, nseg, s_levels, is_biased, x, xhat, memory, gamma, w, norms_out, st); break;
    case 8: launch_recv_gossip<8>(M, n, seg_off, nseg, s_levels, is_biased, x, xhat, memory, gamma, w, norms_out, st); break;
    default: launch_recv_gossip<16>(M, n, seg_off, nseg, s_levels, is_biased, x, xhat, memory, gamma, w, norms_out, st); break;
  }
  profile_end("qsgd_recv_norm", st);
  CHOCO_LAUNCHED("qsgd_recv_gossip_norm_kernel");
  return CHOCO_OK;
}

CHOCO_API int choco_qsgd_decompress_extrapolate(const uint8_t* packed, const float* norms, int64_t n,
                                                const int64_t* seg_off, int32_t nseg, int32_t q, int32_t is_biased,
                                                float a, float b, float* target, void* stream) {
  hipStream_t st = as_stream(stream);
  CHOCO_REQUIRE(packed && norms && target, "null pointer argument");
  CHOCO_REQUIRE(q >= 1 && q <= 16, "q must be in [1, 16]");
  CHOCO_REQUIRE(n > 0 && n < (int64_t)INT32_MAX, "n out of range");
  CHOCO_REQUIRE(nseg >= 1 && (nseg == 1 || seg_off), "need seg_off for nseg > 1");
  CHOCO_REQUIRE(aligned16(packed) && aligned16(target), "buffers must be 16-byte aligned");
  const int cw = container_bits(q);
  QMsgs M{};
  M.lvl[0] = packed;
  M.sgn[0] = packed + plane_bytes(n, cw);
  M.norms[0] = norms;
  M.w[0] = b;
  M.nmsg = 1;
  M.self_slot = -1;
  M.extrap = 1;
  M.a = a;
  profile_begin("qsgd_accumulate", st);
  launch_decode_cw<1>(cw, M, n, seg_off, nseg, (1 << q) - 1, is_biased, nullptr, target, st);
  profile_end("qsgd_accumulate", st);
  CHOCO_LAUNCHED("qsgd_decode_kernel");
  return CHOCO_OK;
}
