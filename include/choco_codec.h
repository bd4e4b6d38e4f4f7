/*
 * choco_codec.h -- C ABI of the MI355X (gfx950) CHOCO compressor codec.
 *
 * This is the drop-in boundary for ChocoSGD's compressor operator path
 * (reference: epfml/ChocoSGD, dl_code/pcode).  Each entry point names the
 * reference interface it replaces (file:line relative to the reference's
 * dl_code/ directory).  All pointers are DEVICE pointers owned by the caller
 * unless documented as host arrays; all work is enqueued on `stream`
 * (a hipStream_t passed as void*), nothing allocates, nothing synchronises.
 *
 * Return value of every function: CHOCO_OK (0) or a negative CHOCO_ERR_*;
 * choco_last_error() returns the per-thread message of the last failure.
 *
 * Workspaces (`ws`, sized by the matching *_workspace_size): device memory the
 * caller zero-fills ONCE before first use; every call leaves it ready for the
 * next (self-resetting tickets and histograms).  A workspace carries state
 * between the kernels of one call, so calls that may run concurrently need
 * separate workspaces (one per stream).
 *
 * Element/index conventions:
 *   - n counts fp32 elements; every n must be < 2^31 (indices are int32 on the
 *     wire; the reference sends fp32 indices and is inexact above 2^24,
 *     pcode/utils/communication.py:69-72 + pcode/utils/sparsification.py:76).
 *   - "delta" inputs: if xhat != NULL the op works on d = x - xhat computed in
 *     fp32 (pcode/optim/parallel_choco_v.py:236,382,482), else on d = x.
 *   - segment tables `seg_off` are int64[nseg+1], seg_off[0] = 0,
 *     seg_off[nseg] = n (the per-tensor layout of create_optimizer.py:15-24).
 */
#ifndef CHOCO_CODEC_H_
#define CHOCO_CODEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CHOCO_OK 0
#define CHOCO_ERR_INVALID (-1)   /* bad argument / shape / alignment          */
#define CHOCO_ERR_HIP (-2)       /* HIP runtime error                          */
#define CHOCO_ERR_WORKSPACE (-3) /* workspace too small                        */

/* ---------------------------------------------------------------- library */
int choco_version(void);                          /* ABI version, currently 1 */
int choco_last_error(char* buf, size_t len);      /* copies message, returns its length */

/* k = max(1, int(n * (1 - ratio))) evaluated in IEEE double exactly as
 * SparsificationCompressor.get_top_k / get_random_k do
 * (pcode/utils/sparsification.py:22,45). */
int64_t choco_topk_k(int64_t n, double ratio);

/* --------------------------------------------------------------- top-k
 * Replaces SparsificationCompressor.get_top_k (pcode/utils/sparsification.py:18-31)
 * and the per-tensor loop of CHOCOSparsificationCompressor.compress
 * (pcode/optim/parallel_choco_v.py:229-260).
 * Output: exactly k (value, index) pairs of the largest |d|, SIGNED values,
 * in ascending index order.  Ties at the k-th magnitude are broken towards the
 * lowest index (the reference's k==1 path, torch.max, does the same; its
 * torch.topk order is implementation-defined). */
size_t choco_topk_workspace_size(int64_t n);
/* Warm start.  A top-k workspace keeps the previous call's exact threshold and
 * bucket counts, and the library keeps (host side, per workspace pointer) the
 * (n, k) and the call count of the last call made on it.  A call with the same
 * (n, k) as the previous call on the same workspace skips the sampling kernel
 * and selects inside a candidate window around the previous threshold (its
 * margin follows the drift observed between calls); a call whose window misses
 * takes the exact fallback, and leaves a fresh window for the next call.  The
 * output is identical on every path.  Calls on one workspace must be issued in
 * stream order (one stream per workspace, as above).
 * choco_topk_workspace_reset forgets every workspace inside [ws, ws + ws_bytes)
 * (call it whenever a top-k / random-k / segmented workspace is allocated or
 * zero-filled again: its next call is cold); choco_topk_set_warm_start(0) turns
 * the warm path off library-wide (every call samples). */
int choco_topk_workspace_reset(const void* ws, size_t ws_bytes);
int choco_topk_set_warm_start(int32_t enable);
/* Byte offset, in every top-k / random-k / segmented workspace, of a sticky uint32
 * status word.  Bit 0: a bounded wait inside the exact fallback gave up, so the
 * output of that call is invalid (never expected; the wait is bounded so that a
 * stuck producer cannot hang the GPU).  The device raises the same bits in a
 * pinned host mirror of the word with a system-scope store, so
 * choco_topk_host_status(ws, clear, stream) reads them with NO copy and NO
 * synchronisation: a call issued after the failing call has run on the GPU sees
 * them (the Python wrapper checks before every call and raises RuntimeError, the
 * exception the reference's pipelines catch, parallel_choco_v.py:226-227).  It
 * returns the bits (0: nothing raised); clear != 0 zeroes the mirror and queues a
 * zero of the device word on `stream`.  The mirror is released with the workspace
 * (choco_topk_workspace_reset). */
#define CHOCO_TOPK_STATUS_OFFSET 0
int choco_topk_host_status(const void* ws, int32_t clear, void* stream);
/* Byte offset of a uint32 counter of calls (flat: the exact fallback; segmented: segments
 * whose warm window missed) in the same workspaces: diagnostics, never reset by the codec. */
#define CHOCO_TOPK_FALLBACKS_OFFSET 4
/* Flat workspaces only, diagnostics: the uint32 cold-run length (calls left that take a
 * sampled window after a warm window missed) and a uint32 counter of calls whose stream
 * kernel took that sample itself (never with the fused consensus step, whose x changes
 * under the stream: the host then runs the separate sample kernel first). */
#define CHOCO_TOPK_COLD_LEFT_OFFSET 8
#define CHOCO_TOPK_K2_SAMPLES_OFFSET 16
#define CHOCO_TOPK_STATUS_POLL_TIMEOUT 1
int choco_topk_compress(const float* x, const float* xhat, int64_t n, int64_t k,
                        float* out_val, int32_t* out_idx,
                        void* ws, size_t ws_bytes, void* stream);

/* choco_topk_compress followed by the SELF message's part of
 * CHOCOSparsificationCompressor.uncompress (parallel_choco_v.py:307-310), folded into
 * the emission of the message (no second launch, no re-read of the message):
 *   if hat_self != NULL:  hat_self[idx] += val
 *   if memory   != NULL:  memory[idx]   += (float)weight * val
 * with the arithmetic of choco_sparse_accumulate (at least one target non-NULL).
 * hat_self may be xhat itself (the CHOCO case): it is written only after this call's
 * last read of it.  The reference applies the messages to memory in ascending rank
 * order (topology.py:161-162 get_neighborhood), so memory may be folded bit-identically
 * only when the self rank comes first among the neighbours (rank 0 of a ring, or a
 * single worker); pass memory = NULL otherwise and apply the self message to memory
 * with choco_sparse_accumulate in its turn. */
int choco_topk_compress_accumulate(const float* x, const float* xhat, int64_t n, int64_t k,
                                   float* out_val, int32_t* out_idx, float* hat_self, float* memory,
                                   float weight,
                                   void* ws, size_t ws_bytes, void* stream);

/* Per-segment top-k (one tensor per segment, as the reference loops over
 * parameter tensors): k_s = choco_topk_k(len_s, ratio), outputs concatenated in
 * segment order, indices GLOBAL (segment offset added in integer arithmetic --
 * the reference adds it in fp32, sparsification.py:76).  Every segment of up to
 * 16M elements is cut into 16K-element tiles and ALL of them are selected in the
 * same five launches (topk_seg.hip); longer segments run the flat pipeline.
 * choco_topk_segmented_plan fills a HOST int64 plan of
 * choco_topk_segmented_plan_len(seg_off, nseg) entries from the HOST table
 * seg_off[nseg+1]: nseg rows of 8 {off, len, k_s, out_off, first tile, tiles, ., .}
 * (row 0's last two = total tiles, batched segments), then the tile -> segment
 * map, then the batched segment ids, the random-k tile table (randk.hip) and the
 * collect launch's tile order (single-tile segments first).  It returns K = sum k_s (the reference's
 * selected_shapes are the k_s, parallel_choco_v.py:245); ratio must be in [0, 1).
 * The caller keeps a DEVICE copy of the whole plan (plan_dev) and passes both on
 * every call.  x / xhat need only 4-byte alignment.  The workspace
 * (choco_topk_segmented_workspace_size) is bound to ONE plan: its per-segment
 * histograms are left zeroed for the next call of that plan, so a workspace that
 * served another plan or call must be zero-filled again first. */
int64_t choco_topk_segmented_plan_len(const int64_t* seg_off_host, int32_t nseg);
int64_t choco_topk_segmented_plan(const int64_t* seg_off_host, int32_t nseg, double ratio,
                                  int64_t* plan_host);
size_t choco_topk_segmented_workspace_size(const int64_t* plan_host, int32_t nseg);
int choco_topk_compress_segmented(const float* x, const float* xhat, const int64_t* plan_dev,
                                  const int64_t* plan_host, int32_t nseg,
                                  float* out_val, int32_t* out_idx,
                                  void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------- random-k
 * Replaces SparsificationCompressor.get_random_k (sparsification.py:40-54).
 * The reference draws np.random.choice(n, k, replace=False) on the host (legacy
 * RandomState); here a uniform k-subset of [0, n) is drawn on the device, and
 * only the k selected elements are read (randk.hip):
 *   derive(K, i) = splitmix64_mix(K + (i + 1) * 0x9E3779B97F4A7C15);
 *   K = derive(key, 0), key = splitmix64_mix(seed + (offset + 1) * 0xD1B54A32D192ED03);
 *   pi_N(j; K): on B bits (2^B >= N, h = (B + 1) / 2), four rounds of
 *     x = (x + a_r) & mask; x = (x * m_r) & mask; x ^= x >> h,
 *     a_r = (u32)derive(K, 2r) & mask, m_r = ((u32)derive(K, 2r + 1) | 1) & mask,
 *     repeated while x >= N (cycle walking: a bijection of [0, N));
 *   tiles of 2^18 elements; tile t holds c_t = #{ j < k : pi_n(j; K) >> 18 == t }
 *     of the selected indices (one tile: c_0 = k; k >= n: every index);
 *   its positions are pi_{L_t}(j; derive(K, 8 + t)), j < c_t (L_t = the tile length).
 * Output in ascending index order.  `offset` selects an independent stream for the
 * same seed (e.g. the step number).  is_biased = 0 scales values by
 * (float)(n / k) like the reference's unbiased branch (sparsification.py:54).
 * Workspace: choco_randk_workspace_size(n) (zero-filled once; see the top-k
 * workspace rules; choco_topk_workspace_reset also resets it). */
size_t choco_randk_workspace_size(int64_t n);
int choco_randk_compress(const float* x, const float* xhat, int64_t n, int64_t k,
                         uint64_t seed, uint64_t offset, int32_t is_biased,
                         float* out_val, int32_t* out_idx,
                         void* ws, size_t ws_bytes, void* stream);

/* Gather at caller-given int64 indices (the reference's x_data[selected_indices],
 * sparsification.py:31,52); scale = 1 for the biased path, (float)(n/k) otherwise. */
int choco_gather(const float* x, const float* xhat, const int64_t* idx, int64_t k,
                 float scale, float* out_val, void* stream);

/* Per-segment random-k (CHOCOSparsificationCompressor.compress with
 * comm_op "random_k", parallel_choco_v.py:229-260 -> sparsification.py:40-54 per
 * tensor): the plan of choco_topk_segmented_plan (k_s = max(1, int(len_s*(1-ratio))),
 * which also carries the random-k tile table), segment s drawn as above with
 * K_s = derive(key, s), outputs concatenated in segment order with GLOBAL
 * indices.  Any 4-byte alignment; workspace: choco_topk_segmented_workspace_size. */
int choco_randk_compress_segmented(const float* x, const float* xhat, const int64_t* plan_dev,
                                   const int64_t* plan_host, int32_t nseg,
                                   uint64_t seed, uint64_t offset, int32_t is_biased,
                                   float* out_val, int32_t* out_idx,
                                   void* ws, size_t ws_bytes, void* stream);

/* Receiver side of CHOCOSparsificationCompressor.uncompress
 * (parallel_choco_v.py:307-310): for one message (val, idx) of k pairs,
 *   if xhat_self != NULL:  xhat_self[idx] += val
 *   memory[idx] += (float)weight * val        (two roundings, as torch does)
 * Indices within one message must be unique (true for top-k / random-k).
 * n = length of xhat_self / memory: an index outside [0, n) is skipped and
 * counted into *bad_count (device uint32, nullable) -- the reference's
 * index_put raises IndexError there. */
int choco_sparse_accumulate(const float* val, const int32_t* idx, int64_t k,
                            float* xhat_self, float* memory, int64_t n, float weight,
                            uint32_t* bad_count, void* stream);

/* Every neighbour's message of a receive step in ONE call: the per-neighbour loop of
 * CHOCOSparsificationCompressor.uncompress (parallel_choco_v.py:291-310) --
 *   for m in 0 .. nmsg-1 (neighbors_info order):
 *     if m == self_slot and xhat_self != NULL:  xhat_self[idx_m] += val_m
 *     memory[idx_m] += (float)weights[m] * val_m
 * bit-identical to nmsg choco_sparse_accumulate calls in that order (which is how it runs:
 * a merged sweep that applies all messages to each touched line of memory once measured
 * slower).  vals / idxs / ks / weights are HOST arrays of nmsg (1..8) entries
 * (device pointers inside).  Workspace: choco_sparse_accumulate_multi_workspace_size(n,
 * nmsg) bytes (0: none).  Out-of-range / non-ascending indices are counted into
 * *bad_count (nullable), as by choco_sparse_accumulate. */
size_t choco_sparse_accumulate_multi_workspace_size(int64_t n, int32_t nmsg);
int choco_sparse_accumulate_multi(const float* const* vals, const int32_t* const* idxs, const int64_t* ks,
                                  const float* weights, int32_t nmsg, int32_t self_slot, float* xhat_self,
                                  float* memory, int64_t n, void* ws, size_t ws_bytes, uint32_t* bad_count,
                                  void* stream);

/* ECDSparsificationCompressor.uncompress (ecd_psgd.py:287-303) for one message:
 * target[idx] = fmaf(b, val, target[idx] * a)   (hat[idx].mul(a).add(b, q_values),
 * a = 1 - 2/t, b = 2/t); out-of-range indices are skipped and counted as above. */
int choco_sparse_extrapolate(const float* val, const int32_t* idx, int64_t k, float* target,
                             int64_t n, float a, float b, uint32_t* bad_count, void* stream);

/* --------------------------------------------------------------- sign
 * Replaces SignCompressor.packing (sparsification.py:129-145, incl. the external
 * bit2byte.packing) and the per-tensor L1 norms of CHOCOSignCompressor.compress
 * (parallel_choco_v.py:476-499).  Layout = the reference's (32, N') view of the
 * zero-padded flat buffer, N' = ceil(n/32): word j holds elements j + r*N',
 * r = 0..31, element r at bit r (LSB first: this repo's documented convention,
 * the unvendored bit2byte's bit order is unpinned); bit set <=> d < 0
 * (sign(0), -0.0, NaN and padding encode as "+").
 * l1_norms (nullable) receives per-segment sum|d| accumulated in fp64 and
 * rounded once to fp32.  seg_off is a DEVICE int64[nseg+1] (may be NULL when
 * nseg == 1).  Workspace: choco_sign_workspace_size(nseg). */
int64_t choco_sign_words(int64_t n);
size_t choco_sign_workspace_size(int32_t nseg);
int choco_sign_compress(const float* x, const float* xhat, int64_t n,
                        const int64_t* seg_off, int32_t nseg,
                        int32_t* packed, float* l1_norms,
                        void* ws, size_t ws_bytes, void* stream);

/* Chunked sign pack (the exchange pipelined with compress, SURVEY.md §8(e);
 * parallel_choco.py exchange_chunks): choco_sign_compress over the words [w0, w1) of the
 * SAME layout (packed is the whole word array; w0 a multiple of 1024, w1 one too or N'),
 * so each range's words can be sent as soon as its launch is queued.  The per-segment L1
 * sums stay in the workspace's fp64 accumulators between calls; the call with finish = 1,
 * issued LAST on the same stream and workspace, writes l1_norms and clears them.  A
 * receiver needs the norms of every segment a range touches, and in the (32, N') layout
 * every range touches every row's segments, so the norms header is sent last and the
 * receiver decodes after the whole message (choco_sign_decompress_accumulate).
 * Words and norms equal the whole-buffer call's (the norms up to fp64 summation order). */
int choco_sign_compress_range(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                              int64_t w0, int64_t w1, int32_t finish, int32_t* packed, float* l1_norms,
                              void* ws, size_t ws_bytes, void* stream);

/* SignCompressor.unpacking (sparsification.py:147-163): +1.0 / -1.0 floats. */
int choco_sign_unpack(const int32_t* packed, int64_t n, float* out, void* stream);

/* Receiver side of CHOCOSignCompressor.uncompress (parallel_choco_v.py:524-558),
 * fused over all messages in the given order (the reference's neighbors_info
 * order).  For message m with per-segment norms norms[m][s] and packed signs:
 *   upd = (norms[m][s] / (float)numel_s) * sign
 *   if m == self_slot:  xhat_self += upd
 *   memory = fmaf((float)weights[m], upd, memory)     (torch add_(.., alpha=w))
 * packed_list/norms_list/weights are HOST arrays of length nmsg (<= 8) holding
 * device pointers / weights.  self_slot = -1 when no message is the local one. */
int choco_sign_decompress_accumulate(const int32_t* const* packed_list,
                                     const float* const* norms_list,
                                     const float* weights, int32_t nmsg, int32_t self_slot,
                                     int64_t n, const int64_t* seg_off, int32_t nseg,
                                     float* xhat_self, float* memory,
                                     void* ws, size_t ws_bytes, void* stream);

/* Receiver side of the other consumers of the sign codec: for each message m in
 * order, target += weights[m] * decode(m) per element, with the reference's
 * rounding: two_roundings = 0 -> fmaf(w, u, target) (torch add_(u, alpha=w):
 * DCDSignCompressor.uncompress, dcd_psgd.py:442-446, w = 1); 1 -> target + (w * u)
 * (torch add_(w * u): DeepSqueezeSignCompressor.uncompress, deep_squeeze.py:481-488,
 * w = consensus_stepsize * (w_r - [r == self])).  u = (norms[m][s] / numel_s) * sign. */
/* The deferred receive fused into the next step's pass (sign): the previous step's
 * messages applied exactly as choco_sign_decompress_accumulate (x_hat += u_self, memory =
 * fmaf(w, u, memory) in order; CHOCOSignCompressor.uncompress, parallel_choco_v.py:
 * 548-558), then this step's consensus step x += gamma (memory - x_hat) (optim/utils.py:
 * 67-72), then this step's message: packed signs of x - x_hat and l1_norms[s] -- ONE pass
 * over x, x_hat and memory, per-tensor layouts included (n >= 2^30 runs the receive and
 * choco_gossip_sign_compress as two kernels).  Bit-identical x, x_hat, memory and words
 * to that sequence.  packed must not alias a message's words (l1_norms may alias a
 * message's norms: every workgroup reads them before the last one writes).  nmsg 1..8;
 * ws of choco_sign_recv_workspace_size(n, nseg, nmsg) bytes (the pass runs over row runs of
 * the (32, N') view, the messages and the output words as bit planes). */
/* Workspace bytes of choco_sign_recv_gossip_compress for n elements in nseg segments and
 * nmsg messages (the per-segment accumulators plus bit planes of every message and of the
 * output; n >= 2^30: choco_sign_workspace_size(nseg)). */
size_t choco_sign_recv_workspace_size(int64_t n, int32_t nseg, int32_t nmsg);

int choco_sign_recv_gossip_compress(const int32_t* const* packed_list, const float* const* norms_list,
                                    const float* weights, int32_t nmsg, int32_t self_slot, float* x,
                                    float* memory, float* xhat, float gamma, int64_t n,
                                    const int64_t* seg_off, int32_t nseg, int32_t* packed,
                                    float* l1_norms, void* ws, size_t ws_bytes, void* stream);

int choco_sign_decompress_axpy(const int32_t* const* packed_list, const float* const* norms_list,
                               const float* weights, int32_t nmsg, int64_t n,
                               const int64_t* seg_off, int32_t nseg, int32_t two_roundings,
                               float* target, void* stream);

/* ECDSignCompressor.uncompress (ecd_psgd.py:448-454) for one message:
 * target_s = (target_s * a) + ((b * norm_s) / numel_s) * sign   (a = 1 - 2/t, b = 2/t). */
int choco_sign_decompress_extrapolate(const int32_t* packed, const float* norms, int64_t n,
                                      const int64_t* seg_off, int32_t nseg, float a, float b,
                                      float* target, void* stream);

/* DeepSqueezeSignCompressor.compress's local compressed copy (deep_squeeze.py:416-422):
 * out = (norms[s] * torch.sign(x)) / numel_s, sign(0) = 0, NaN stays NaN. */
int choco_sign_local_decode(const float* x, int64_t n, const int64_t* seg_off, int32_t nseg,
                            const float* norms, float* out, void* stream);

/* --------------------------------------------------------------- QSGD
 * Replaces QuantizationCompressor.get_qsgd/compress (sparsification.py:87-98,114-120)
 * applied per segment (parallel_choco_v.py:375-397).  s = 2^q - 1 levels.
 *   norm_s  = ||d_s||_2 (fp64 accumulation, rounded once)   or norm_in[s] if given
 *   lf      = ((float)s * |d|) / norm_s
 *   level   = floor(lf) + (u < lf - floor(lf)),  u = u_in[e] if given, else
 *             this codec's stream (the reference draws torch.rand_like,
 *             sparsification.py:91): key = splitmix64_mix(seed + (offset+1) *
 *             0xD1B54A32D192ED03); with g = (e & 8191) >> 11, element e
 *             belongs to stream sid = ((e >> 13) << 9) | ((g >> 1) << 8) |
 *             ((e & 8191) >> 3 & 255) at position p = (g & 1) * 8 + (e & 7)
 *             (16 uniforms per stream); stream sid is xoroshiro128+
 *             (a=24, b=16, c=37) started from (splitmix64_mix(z),
 *             splitmix64_mix(z + 0x9E3779B97F4A7C15)), z = key + (2 sid + 1) *
 *             0x9E3779B97F4A7C15; its output number p / 2, r = s0 + s1, gives
 *             u = (even p: r >> 40, odd p: (r >> 16) & 0xFFFFFF) * 2^-24
 *             (restated in oracle/choco_oracle.py qsgd_uniforms_at)
 * Wire format (packed, choco_qsgd_packed_bytes): level plane (container of
 * cw = 1,2,4,8,16 bits >= q, little-endian within 32-bit words) followed by a
 * sign plane (1 bit/element, bit set <=> d < 0), both padded to 16 bytes.
 * dense_out (nullable) receives the reference's decoded floats
 *   ((scale * sign(d)) * norm_s) * level / (float)s
 * bit-for-bit; norms_out (nullable) the per-segment fp32 norms. q in [1,16]. */
int64_t choco_qsgd_packed_bytes(int64_t n, int32_t q);
size_t choco_qsgd_workspace_size(int32_t nseg);
int choco_qsgd_compress(const float* x, const float* xhat, int64_t n,
                        const int64_t* seg_off, int32_t nseg,
                        int32_t q, int32_t is_biased,
                        const float* norm_in, const float* u_in,
                        uint64_t seed, uint64_t offset,
                        uint8_t* packed, float* norms_out, float* dense_out,
                        void* ws, size_t ws_bytes, void* stream);

/* Decode a packed message to the reference's dense floats (the value that
 * QuantizationCompressor.uncompress, sparsification.py:122-123, passes on). */
int choco_qsgd_decode(const uint8_t* packed, const float* norms, int64_t n,
                      const int64_t* seg_off, int32_t nseg, int32_t q, int32_t is_biased,
                      float* out, void* stream);

/* Receiver side of CHOCOQuantizationCompressor.uncompress (parallel_choco_v.py:415-433)
 * fused over messages:  v = decode(m);  if m == self_slot: xhat_self += v;
 * memory += (float)weights[m] * v   (two roundings). */
int choco_qsgd_decompress_accumulate(const uint8_t* const* packed_list,
                                     const float* const* norms_list,
                                     const float* weights, int32_t nmsg, int32_t self_slot,
                                     int64_t n, const int64_t* seg_off, int32_t nseg,
                                     int32_t q, int32_t is_biased,
                                     float* xhat_self, float* memory, void* stream);

/* The deferred receive fused into the next step's first pass (QSGD): the previous step's
 * messages applied exactly as choco_qsgd_decompress_accumulate (x_hat += q_self, memory +=
 * w * q in order; CHOCOQuantizationCompressor.uncompress, parallel_choco_v.py:430-433),
 * then this step's consensus step x += gamma (memory - x_hat) (optim/utils.py:67-72), then
 * norms_out[s] = ||x - x_hat||_2 per segment (fp64, rounded once) -- ONE pass over x,
 * x_hat and memory instead of the decode, gossip and norm passes; bit-identical x, x_hat
 * and memory.  Quantize this step's message afterwards with choco_qsgd_compress(...,
 * norm_in = norms_out, ...).  Valid wherever the receive of step t-1 and the consensus
 * step of step t are adjacent (ParallelCHOCO_V.step: apply_gradient, then the previous
 * gossip's join, then update_params_from_neighbor).  nmsg 1..8; ws as for
 * choco_qsgd_norms (choco_qsgd_workspace_size(nseg)).  norms_out MAY alias a message's
 * norms (e.g. the pending self message's header, reused as this step's): every workgroup
 * reads the message norms before it takes the last-workgroup ticket, and only the last
 * workgroup writes norms_out.  The level / sign planes must not overlap x, x_hat or memory. */
int choco_qsgd_recv_gossip_norms(const uint8_t* const* packed_list, const float* const* norms_list,
                                 const float* weights, int32_t nmsg, int32_t self_slot, float* x,
                                 float* memory, float* xhat, float gamma, int64_t n,
                                 const int64_t* seg_off, int32_t nseg, int32_t q, int32_t is_biased,
                                 float* norms_out, void* ws, size_t ws_bytes, void* stream);

/* ECDQuantizationCompressor.uncompress (ecd_psgd.py:415-423) for one message:
 * target = fmaf(b, decode(m), target * a)   (hat.mul_(a).add_(q, alpha=b)). */
int choco_qsgd_decompress_extrapolate(const uint8_t* packed, const float* norms, int64_t n,
                                      const int64_t* seg_off, int32_t nseg, int32_t q, int32_t is_biased,
                                      float a, float b, float* target, void* stream);

/* Chunked QSGD wire (the exchange pipelined with compress and decompress, SURVEY.md
 * §8(e); parallel_choco.py exchange_chunks): the norm pass alone, then the quantize
 * pass over element ranges [e0, e1), each range a self-contained message of
 * choco_qsgd_packed_bytes(e1 - e0, q) bytes ([level plane | sign plane] of its own
 * elements), and the receiver over the same ranges.  e0 must be a multiple of 8192
 * (the uniform-stream tile), e1 one too or n.  A range's levels, signs and uniforms
 * are exactly those of choco_qsgd_compress over the whole buffer (element e keeps its
 * stream position), so the decoded values, and memory / xhat_self after all ranges,
 * are bit-identical to the unchunked path; norms come from choco_qsgd_norms (or its
 * gossip form, which also applies the consensus step to x). */
int choco_qsgd_norms(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                     float* norms_out, void* ws, size_t ws_bytes, void* stream);
int choco_gossip_qsgd_norms(float* x, const float* memory, const float* xhat, float gamma, int64_t n,
                            const int64_t* seg_off, int32_t nseg, float* norms_out, void* ws, size_t ws_bytes,
                            void* stream);
int choco_qsgd_quantize_range(const float* x, const float* xhat, int64_t n, const int64_t* seg_off, int32_t nseg,
                              int32_t q, int32_t is_biased, const float* norms, uint64_t seed, uint64_t offset,
                              int64_t e0, int64_t e1, uint8_t* packed_range, void* stream);
int choco_qsgd_decompress_accumulate_range(const uint8_t* const* packed_list, const float* const* norms_list,
                                           const float* weights, int32_t nmsg, int32_t self_slot, int64_t n,
                                           const int64_t* seg_off, int32_t nseg, int32_t q, int32_t is_biased,
                                           int64_t e0, int64_t e1, float* xhat_self, float* memory,
                                           void* stream);

/* ------------------------------------------------------- gossip step
 * update_params_from_neighbor (pcode/optim/utils.py:67-72):
 *   x += (float)gamma * (memory - xhat)   (three roundings, as torch does). */
int choco_gossip_step(float* x, const float* memory, const float* xhat, float gamma,
                      int64_t n, void* stream);

/* ------------------------------------------- fused gossip step + compress
 * ParallelCHOCO_V.step's update_params_from_neighbor -> compress sequence
 * (pcode/optim/parallel_choco_v.py:116-142 -> :229-240, optim/utils.py:67-72) in
 * the codec's own passes: the FIRST full pass of the compressor reads x, memory
 * and xhat, writes x_new = x + (float)gamma * (memory - xhat) back into x (bit-
 * identical to choco_gossip_step) and compresses d = x_new - xhat, so the step
 * costs one pass of 12 B read + 4 B written per element less than
 * choco_gossip_step followed by the compressor.  Outputs, workspaces, plans and
 * alignment rules are those of the matching non-gossip entry point.  Paths with
 * no full first pass (random-k, which gathers k elements; pinned-norm QSGD; tiny
 * or k == n top-k) run choco_gossip_step first. */
int choco_gossip_topk_compress(float* x, const float* memory, const float* xhat, float gamma,
                               int64_t n, int64_t k, float* out_val, int32_t* out_idx,
                               void* ws, size_t ws_bytes, void* stream);
/* The fused step + top-k + self-message fold: xhat[idx] += val, and memory[idx] +=
 * (float)weight * val when fold_memory != 0 (the ordering rule of
 * choco_topk_compress_accumulate). */
int choco_gossip_topk_compress_accumulate(float* x, float* memory, float* xhat, float gamma,
                                          int64_t n, int64_t k, float* out_val, int32_t* out_idx,
                                          int32_t fold_memory, float weight,
                                          void* ws, size_t ws_bytes, void* stream);
int choco_gossip_topk_compress_segmented(float* x, const float* memory, const float* xhat, float gamma,
                                         const int64_t* plan_dev, const int64_t* plan_host, int32_t nseg,
                                         float* out_val, int32_t* out_idx,
                                         void* ws, size_t ws_bytes, void* stream);
int choco_gossip_randk_compress_segmented(float* x, const float* memory, const float* xhat, float gamma,
                                          const int64_t* plan_dev, const int64_t* plan_host, int32_t nseg,
                                          uint64_t seed, uint64_t offset, int32_t is_biased,
                                          float* out_val, int32_t* out_idx,
                                          void* ws, size_t ws_bytes, void* stream);
int choco_gossip_sign_compress(float* x, const float* memory, const float* xhat, float gamma,
                               int64_t n, const int64_t* seg_off, int32_t nseg,
                               int32_t* packed, float* l1_norms,
                               void* ws, size_t ws_bytes, void* stream);
int choco_gossip_sign_compress_range(float* x, const float* memory, const float* xhat, float gamma, int64_t n,
                                     const int64_t* seg_off, int32_t nseg, int64_t w0, int64_t w1, int32_t finish,
                                     int32_t* packed, float* l1_norms, void* ws, size_t ws_bytes, void* stream);
int choco_gossip_qsgd_compress(float* x, const float* memory, const float* xhat, float gamma,
                               int64_t n, const int64_t* seg_off, int32_t nseg,
                               int32_t q, int32_t is_biased, uint64_t seed, uint64_t offset,
                               uint8_t* packed, float* norms_out, float* dense_out,
                               void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------- profiling hooks
 * Optional: when enabled, the dominant kernel of each op is launched with a
 * pair of hipEvents attached to the dispatch itself (hipExtLaunchKernelGGL), so
 * the elapsed time is the kernel's own, not the queue ahead of it (the bench's
 * roofline source; agrees with rocprofv3 --kernel-trace). */
int choco_profile_enable(int32_t on);
/* Accumulated (sum of ms, count) of the named kernel since the last reset,
 * after synchronising its events.  Names: "topk_stream", "sign_pack",
 * "qsgd_quantize", "sparse_accumulate", ... */
/* Time only the launches whose name is in the comma-separated list `names`
 * (NULL or "" = all); events are reused. */
int choco_profile_filter(const char* names);
int choco_profile_read(const char* name, double* total_ms, int64_t* count);
int choco_profile_reset(void);
/* Launches of the named kernel since the library was loaded, counted whether or not
 * profiling is enabled (diagnostic: the bench's per-step warm-hit rates, e.g. how many
 * "topk_bounds" sample launches or "topk_seg_hist" cold passes a step took). */
int64_t choco_launch_count(const char* name);

#ifdef __cplusplus
}
#endif

#endif /* CHOCO_CODEC_H_ */
