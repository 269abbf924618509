// Persistent fused minibatch update for precision mode bf16:
// actor/critic forward, Normal log-prob, clipped surrogate + entropy / Huber loss heads, and the
// full backward of both networks (ppo.py:109-135) in ONE launch per minibatch.
//
// Scope: two hidden layers of equal width H (the MLP configs of BASELINE.json: 2x256; in_dim
// = W*O <= 32, A <= 8).  Other shapes and precision f32 use the layered GEMM path.
//
// Layout.  grid = (G, 2): blockIdx.y picks the net (0 actor, 1 critic), each workgroup (8 waves)
// owns one CU (LDS ~144 KB) and walks minibatch chunks of R = 64 rows, chunk = blockIdx.x + i*G.
// Per chunk everything stays on chip:
//   X   [64][32]  bf16 LDS image of the states (64-B rows)
//   A1  [64][H]   bf16 layer-0 output a1, later overwritten with its gradient d1
//   D2  [64][H]   bf16 gradient at layer 1's pre-activation (its first use: head partial sums)
//   A2F [64][H]   f32 layer-1 output a2 (the head runs in f32 on it, like the emulation oracle)
// Activations are written from the MFMA accumulators (column = batch row on the lane, rows =
// features in registers -> 8-B stores of 4 features) and read back either row-wise (16-B
// ds_read_b128: 8 consecutive features of one batch row, the operand of a product summing over
// features) or column-wise (ds_read_b64_tr_b16: 8 consecutive batch rows of one feature, the
// operand of a weight gradient summing over rows).  One XOR-swizzled image serves both reads
// conflict-free (cdna_hip_programming.md T10 "one image for row reads AND transposed reads").
// Weight gradients are summed over all chunks of the workgroup in registers (dW1: 8 32x32
// tiles per wave; dW0: one tile per wave), so HBM sees only the bf16 minibatch inputs, the
// L2-resident bf16 weights and, once per workgroup, one partial-gradient slab in the flat
// parameter layout.  reduce_slabs_kernel then folds the G slabs in a fixed order.
//
// Numerics = oracle.use_bf16_hidden_gemms: every hidden-layer product takes bf16(RNE) operands
// with f32 accumulation; the heads (forward, dH, head dW) and every bias gradient are f32 on the
// f32 values.  act'(a1) for tanh / ELU uses the f32 a1, recomputed in the dgrad epilogue (the
// image holds bf16(a1)); ReLU needs only its sign, which the bf16 image keeps.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "adam_elem.h"
#include "fused_common.h"
#include "gae_pipe.h"

namespace ppo {

using namespace fu;

__device__ __forceinline__ uint16_t bf16_bits(float x) { return static_cast<uint16_t>(pack2(x, 0.f) & 0xffffu); }

// ============================================================================================
// Prep: gather the minibatch rows once per minibatch into contiguous bf16 / f32 staging, and
// refresh the bf16 weight images (row-major and transposed W1) from the f32 masters.
// ============================================================================================
__global__ __launch_bounds__(256) void fused_prep_kernel(FusedArgs q, int row_blocks) {
  const int tid = threadIdx.x;
  if (static_cast<int>(blockIdx.x) < row_blocks && q.rec) {
    // staged records: 8 lanes copy one 128 B record (4 x 16 B state image, 4 x 16 B scalars)
    const int j = static_cast<int>((static_cast<int64_t>(blockIdx.x) * 256 + tid) >> 3);
    const int u = tid & 7;
    if (j >= q.b) return;
    const int count = q.rows_n ? *q.rows_n : q.b;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (j < count) {
      const int64_t sr = q.rows[j];
      if (sr >= 0 && sr < q.n_rec) v = q.rec[sr * (kRecordBytes / 16) + u];
    }
    if (u < 4) reinterpret_cast<uint4 *>(q.xb + static_cast<int64_t>(j) * kFusedKX)[u] = v;
    else reinterpret_cast<uint4 *>(q.srow + static_cast<int64_t>(j) * kFusedSP)[u - 4] = v;
    return;
  }
  if (static_cast<int>(blockIdx.x) < row_blocks) {
    const int j = blockIdx.x * 256 + tid;
    if (j >= q.b) return;
    const int count = q.rows_n ? *q.rows_n : q.b;
    const int A = q.act_dim;
    float x[kFusedKX];
    float s[kFusedSP];
#pragma unroll
    for (int k = 0; k < kFusedKX; ++k) x[k] = 0.f;
#pragma unroll
    for (int k = 0; k < kFusedSP; ++k) s[k] = 0.f;
    if (j < count) {
      const int64_t sr = q.rows[j];
      const float *src = q.states + sr * q.din;
#pragma unroll
      for (int k = 0; k < kFusedKX; ++k)
        if (k < q.din) x[k] = src[k];
      const float old_lp = q.old_logp[sr], adv = q.adv[sr], vt = q.vtarget[sr];
#pragma unroll
      for (int k = 0; k < kFusedSP; ++k)
        s[k] = k < A ? q.actions[sr * A + k]
                     : (k == A ? old_lp : (k == A + 1 ? adv : (k == A + 2 ? vt : 0.f)));
    }
    uint4 *xd = reinterpret_cast<uint4 *>(q.xb + static_cast<int64_t>(j) * kFusedKX);
#pragma unroll
    for (int u = 0; u < kFusedKX / 8; ++u)
      xd[u] = make_uint4(pack2(x[8 * u], x[8 * u + 1]), pack2(x[8 * u + 2], x[8 * u + 3]),
                         pack2(x[8 * u + 4], x[8 * u + 5]), pack2(x[8 * u + 6], x[8 * u + 7]));
    float4 *sd = reinterpret_cast<float4 *>(q.srow + static_cast<int64_t>(j) * kFusedSP);
#pragma unroll
    for (int u = 0; u < kFusedSP / 4; ++u)
      sd[u] = make_float4(s[4 * u], s[4 * u + 1], s[4 * u + 2], s[4 * u + 3]);
    return;
  }
  // weights: per net H*32 (W0 image) + H*H (W1 and its transpose) elements
  const int H = q.hidden;
  const int64_t per_net = static_cast<int64_t>(H) * kFusedKX + static_cast<int64_t>(H) * H;
  const int64_t e = static_cast<int64_t>(blockIdx.x - row_blocks) * 256 + tid;
  if (e >= 2 * per_net) return;
  const int z = e >= per_net;
  const FusedNet &N = z ? q.net[1] : q.net[0];
  const int64_t i = e - z * per_net;
  __bf16 *w0b = const_cast<__bf16 *>(N.w0b);
  __bf16 *w1b = const_cast<__bf16 *>(N.w1b);
  __bf16 *w1bt = const_cast<__bf16 *>(N.w1bt);
  if (i < static_cast<int64_t>(H) * kFusedKX) {
    const int f = static_cast<int>(i / kFusedKX), k = static_cast<int>(i % kFusedKX);
    const float v = k < q.din ? N.w0[static_cast<int64_t>(f) * q.din + k] : 0.f;
    w0b[i] = __builtin_bit_cast(__bf16, static_cast<uint16_t>(pack2(v, 0.f) & 0xffffu));
  } else {
    const int64_t t = i - static_cast<int64_t>(H) * kFusedKX;
    const int o = static_cast<int>(t / H), c = static_cast<int>(t % H);
    const __bf16 v = __builtin_bit_cast(__bf16, static_cast<uint16_t>(pack2(N.w1[t], 0.f) & 0xffffu));
    w1b[w_frag(o, c, H)] = v;   // fragment-major images (fused_common.h w_frag)
    w1bt[w_frag(c, o, H)] = v;
  }
}

// Records: thread = one stored row, written as 8 x 16 B (the prep row gather's exact values).
__global__ __launch_bounds__(256) void fused_records_kernel(uint4 *__restrict__ rec,
                                                            const float *__restrict__ states,
                                                            const float *__restrict__ actions,
                                                            const float *__restrict__ old_logp,
                                                            const float *__restrict__ adv,
                                                            const float *__restrict__ vtarget,
                                                            int64_t n_rows, int din, int A) {
  const int64_t sr = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (sr >= n_rows) return;
  float x[kFusedKX];
  float s[kFusedSP];
  const float *src = states + sr * din;
#pragma unroll
  for (int k = 0; k < kFusedKX; ++k) x[k] = k < din ? src[k] : 0.f;
  const float old_lp = old_logp[sr], ad = adv[sr], vt = vtarget[sr];
#pragma unroll
  for (int k = 0; k < kFusedSP; ++k)
    s[k] = k < A ? actions[sr * A + k]
                 : (k == A ? old_lp : (k == A + 1 ? ad : (k == A + 2 ? vt : 0.f)));
  uint4 *d = rec + sr * (kRecordBytes / 16);
#pragma unroll
  for (int u = 0; u < kFusedKX / 8; ++u)
    d[u] = make_uint4(pack2(x[8 * u], x[8 * u + 1]), pack2(x[8 * u + 2], x[8 * u + 3]),
                      pack2(x[8 * u + 4], x[8 * u + 5]), pack2(x[8 * u + 6], x[8 * u + 7]));
#pragma unroll
  for (int u = 0; u < kFusedSP / 4; ++u)
    d[kFusedKX / 8 + u] = make_uint4(__float_as_uint(s[4 * u]), __float_as_uint(s[4 * u + 1]),
                                     __float_as_uint(s[4 * u + 2]), __float_as_uint(s[4 * u + 3]));
}

// The staged-record pass fused into the GAE scan (gae_pipe.h): each row's record is written once
// its advantage / value target come out of the chain, with the row's state / action / old
// log-prob loads issued a chunk ahead (under the barrier and the chain).  Byte-identical to
// gae_pipe_kernel + fused_records_kernel; valid when nothing rewrites adv / vtarget in between
// (no advantage normalisation).
struct RecordEmit {
  const float *states, *actions, *old_logp;
  uint4 *rec;
  int din, A;
  float x[2][kFusedKX];
  float act[2][kFusedSP];
  float lp[2];
  __device__ __forceinline__ void load(int b, int64_t row, bool) {
    const float *src = states + row * din;
#pragma unroll
    for (int k = 0; k < kFusedKX; ++k) x[b][k] = k < din ? src[k] : 0.f;
#pragma unroll
    for (int k = 0; k < kFusedSP; ++k) act[b][k] = k < A ? actions[row * A + k] : 0.f;
    lp[b] = old_logp[row];
  }
  __device__ __forceinline__ void store(int b, int64_t row, float ad, float vt) {
    float s[kFusedSP];
#pragma unroll
    for (int k = 0; k < kFusedSP; ++k)
      s[k] = k < A ? act[b][k] : (k == A ? lp[b] : (k == A + 1 ? ad : (k == A + 2 ? vt : 0.f)));
    uint4 *d = rec + row * (kRecordBytes / 16);
#pragma unroll
    for (int u = 0; u < kFusedKX / 8; ++u)
      d[u] = make_uint4(pack2(x[b][8 * u], x[b][8 * u + 1]), pack2(x[b][8 * u + 2], x[b][8 * u + 3]),
                        pack2(x[b][8 * u + 4], x[b][8 * u + 5]), pack2(x[b][8 * u + 6], x[b][8 * u + 7]));
#pragma unroll
    for (int u = 0; u < kFusedSP / 4; ++u)
      d[kFusedKX / 8 + u] = make_uint4(__float_as_uint(s[4 * u]), __float_as_uint(s[4 * u + 1]),
                                       __float_as_uint(s[4 * u + 2]), __float_as_uint(s[4 * u + 3]));
  }
};

template <typename RT, int EB, int KMAX>
__global__ __launch_bounds__(EB * 16) void gae_records_kernel(GaeRecordArgs g) {
  RecordEmit em;
  em.states = g.states;
  em.actions = g.actions;
  em.old_logp = g.old_logp;
  em.rec = g.rec;
  em.din = g.din;
  em.A = g.act_dim;
  gae_pipe_body<RT, EB, KMAX>(g.value, g.next_value, static_cast<const RT *>(g.reward), g.done,
                              g.term, g.force_last, g.n, g.t_len, g.gamma_f, g.lg_f, g.adv,
                              g.vtarget, em);
}

// ============================================================================================
// Adam + weight images.  Blocks [0, gen_blocks): elementwise over the flat vector, skipping the
// two W1 blocks (W0 elements also land in the W0 image).  Blocks [gen_blocks, ...): one 32x32
// tile of one net's W1 each -- Adam on the tile, the row-major bf16 image written directly and
// the transposed image through an LDS transpose, so both image writes are coalesced.
// ============================================================================================
constexpr int kPackTile = 32;

__global__ __launch_bounds__(256) void adam_pack_kernel(AdamPackArgs a, int gen_blocks) {
  const float ns_a = a.sched ? a.sched[0] : a.neg_a;
  const float ns_c = a.sched ? a.sched[1] : a.neg_c;
  const float bc2 = a.sched ? a.sched[2] : a.bc2;
  const int tid = threadIdx.x;
  const int H = a.H;
  if (static_cast<int>(blockIdx.x) < gen_blocks) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + tid;
    if (i >= a.n) return;
#pragma unroll
    for (int z = 0; z < 2; ++z)
      if (i >= a.off_w1[z] && i < a.off_w1[z] + static_cast<int64_t>(H) * H) return;
    float m = a.m[i], v = a.v[i];
    const float p = adam_elem(a.p[i], a.g[i], m, v, i < a.n_actor ? ns_a : ns_c, a.w1, a.b2,
                              a.omb2, bc2, a.eps);
    a.p[i] = p;
    a.m[i] = m;
    a.v[i] = v;
#pragma unroll
    for (int z = 0; z < 2; ++z) {
      const int64_t e = i - a.off_w0[z];
      if (e >= 0 && e < static_cast<int64_t>(H) * a.din) {
        const int f = static_cast<int>(e / a.din), k = static_cast<int>(e % a.din);
        reinterpret_cast<uint16_t *>(a.w0b[z])[f * kFusedKX + k] = bf16_bits(p);
      }
    }
    return;
  }
  __shared__ uint16_t tile[kPackTile][kPackTile + 2];
  const int tiles = H / kPackTile;
  const int tb = static_cast<int>(blockIdx.x) - gen_blocks;
  const int z = tb / (tiles * tiles);
  const int to = (tb % (tiles * tiles)) / tiles, tc = tb % tiles;
  const int64_t base = a.off_w1[z];
  const float ns = base < a.n_actor ? ns_a : ns_c;
  uint16_t *w1b = reinterpret_cast<uint16_t *>(a.w1b[z]);
  uint16_t *w1bt = reinterpret_cast<uint16_t *>(a.w1bt[z]);
#pragma unroll 4
  for (int k = 0; k < kPackTile * kPackTile / 256; ++k) {
    const int idx = k * 256 + tid, lo = idx / kPackTile, lc = idx % kPackTile;
    const int64_t t = static_cast<int64_t>(to * kPackTile + lo) * H + tc * kPackTile + lc;
    const int64_t i = base + t;
    float m = a.m[i], v = a.v[i];
    const float p = adam_elem(a.p[i], a.g[i], m, v, ns, a.w1, a.b2, a.omb2, bc2, a.eps);
    a.p[i] = p;
    a.m[i] = m;
    a.v[i] = v;
    const uint16_t hb = bf16_bits(p);
    w1b[w_frag(to * kPackTile + lo, tc * kPackTile + lc, H)] = hb;
    tile[lo][lc] = hb;
  }
  __syncthreads();
#pragma unroll 4
  for (int k = 0; k < kPackTile * kPackTile / 256; ++k) {
    const int idx = k * 256 + tid, lc = idx / kPackTile, lo = idx % kPackTile;
    w1bt[w_frag(tc * kPackTile + lc, to * kPackTile + lo, H)] = tile[lo][lc];
  }
}

// ============================================================================================
// Optimizer-step tail: slab reduction + Adam + weight images, and the next rows' gather
// ============================================================================================
// thread index idx of the gather part: row idx / 8, 16-B unit idx % 8 of its record
__device__ __forceinline__ void tail_gather(const TailArgs &t, int64_t idx) {
  const int j = static_cast<int>(idx >> 3);
  const int u = static_cast<int>(idx & 7);
  if (j >= t.b) return;
  const int64_t sr = t.rows[j];
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (sr >= 0 && sr < t.n_rec) v = t.rec[sr * (kRecordBytes / 16) + u];
  if (u < 4) reinterpret_cast<uint4 *>(t.xb + static_cast<int64_t>(j) * kFusedKX)[u] = v;
  else reinterpret_cast<uint4 *>(t.srow + static_cast<int64_t>(j) * kFusedSP)[u - 4] = v;
}

// Adam on parameters i..i+3 (gradient g4, operands p4 / m4 / v4 already loaded) and their
// entries of the bf16 weight images.
__device__ __forceinline__ void adam_apply(const AdamPackArgs &a, int64_t i, float4 g4, float4 p4,
                                           float4 m4, float4 v4) {
  const float ns = i < a.n_actor ? (a.sched ? a.sched[0] : a.neg_a) : (a.sched ? a.sched[1] : a.neg_c);
  const float bc2 = a.sched ? a.sched[2] : a.bc2;
  p4.x = adam_elem(p4.x, g4.x, m4.x, v4.x, ns, a.w1, a.b2, a.omb2, bc2, a.eps);
  p4.y = adam_elem(p4.y, g4.y, m4.y, v4.y, ns, a.w1, a.b2, a.omb2, bc2, a.eps);
  p4.z = adam_elem(p4.z, g4.z, m4.z, v4.z, ns, a.w1, a.b2, a.omb2, bc2, a.eps);
  p4.w = adam_elem(p4.w, g4.w, m4.w, v4.w, ns, a.w1, a.b2, a.omb2, bc2, a.eps);
  *reinterpret_cast<float4 *>(a.p + i) = p4;
  *reinterpret_cast<float4 *>(a.m + i) = m4;
  *reinterpret_cast<float4 *>(a.v + i) = v4;
  const float pv[4] = {p4.x, p4.y, p4.z, p4.w};
  const int H = a.H;
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    const int64_t e1 = i - a.off_w1[z];
    if (e1 >= 0 && e1 < static_cast<int64_t>(H) * H) {  // 4 columns of one W1 row (H % 4 == 0)
      const int o = static_cast<int>(e1 / H), c = static_cast<int>(e1 % H);
      // 4 consecutive columns stay inside one 8-element fragment run (c % 4 == 0)
      *reinterpret_cast<uint2 *>(a.w1b[z] + w_frag(o, c, H)) = make_uint2(pack2(pv[0], pv[1]), pack2(pv[2], pv[3]));
      uint16_t *wt = reinterpret_cast<uint16_t *>(a.w1bt[z]);
#pragma unroll
      for (int e = 0; e < 4; ++e) wt[w_frag(c + e, o, H)] = bf16_bits(pv[e]);
    }
    const int64_t e0 = i - a.off_w0[z];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e0 + e >= 0 && e0 + e < static_cast<int64_t>(H) * a.din) {
        const int f = static_cast<int>((e0 + e) / a.din), k = static_cast<int>((e0 + e) % a.din);
        reinterpret_cast<uint16_t *>(a.w0b[z])[f * kFusedKX + k] = bf16_bits(pv[e]);
      }
    }
  }
}

// One parameter block of the tail: fold its slabs (reduce_slab_block_s, fixed order) or take
// the gradient already in a.g, then Adam + the bf16 weight images on the chunk-0 threads.
template <int G>
__device__ __forceinline__ void tail_block(const ReduceArgs &r, const TailArgs &t, int64_t blk,
                                           RedScratch sc) {
  const int tid = threadIdx.x;
  const AdamPackArgs &a = t.a;
  const int64_t i = blk * (4 * G) + 4 * (tid % G);
  const bool lead = tid < G;  // chunk 0: the threads that own the reduced sums
  float4 g4;
  if (t.reduce) {
    g4 = reduce_slab_block_s<G>(r, blk, sc);
    if (!lead || i >= r.total) return;
  } else {
    if (!lead || i >= a.n) return;
    g4 = *reinterpret_cast<const float4 *>(a.g + i);
  }
  adam_apply(a, i, g4, *reinterpret_cast<const float4 *>(a.p + i),
             *reinterpret_cast<const float4 *>(a.m + i), *reinterpret_cast<const float4 *>(a.v + i));
}

// Blocks of G float4 groups x kRedChunks chunks (the per-parameter order of every G is the
// same, reduce_slabs.h).  G = 32 (512 threads, 128 parameters a block) by default.  At 69 VGPRs a
// CU holds 3 such blocks, so the headline's 1,115 run in two rounds; smaller blocks that fit in
// one were measured slower all the same (PPO_TAIL_GROUPS, round 5: 1.32 ms per iteration at
// G = 32, 1.38 at 16, 1.67 at 8).
template <int G>
__global__ __launch_bounds__(G * kRedChunks) void step_tail_kernel(ReduceArgs r, TailArgs t, int red_blocks) {
  __shared__ __attribute__((aligned(16))) char scratch[red_scratch_bytes<G>()];
  constexpr int NT = G * kRedChunks;
  const int tid = threadIdx.x;
  if (static_cast<int>(blockIdx.x) >= red_blocks) {  // the next minibatch's record gather
    tail_gather(t, (static_cast<int64_t>(blockIdx.x) - red_blocks) * NT + tid);
    return;
  }
  tail_block<G>(r, t, blockIdx.x, red_scratch<G>(scratch));
}

// ============================================================================================
// The fused update kernel
// ============================================================================================
template <int H, bool F32A2>
struct Lds {
  static constexpr int PITCH = 2 * H;          // A1 / D2 / A2 / D1 bf16 row pitch (bytes), multiple of 256
  static constexpr int A2P = 4 * H + 16;       // A2F f32 row pitch (bytes): +16 B -> conflict-free b128 stores
  static constexpr int WHB = 0;                                 // bf16 head image [16][H + 8]
  static constexpr int BIAS = WHB + HeadImg<H>::BYTES;          // f32 b0[H], b1[H]
  static constexpr int X = BIAS + 2 * H * 4;                    // bf16 [64][32]
  static constexpr int A1 = X + R * 64;                         // bf16 [64][H]
  static constexpr int D2 = A1 + R * PITCH;                     // bf16 [64][H]
  // a2 after the layer-1 epilogue: the bf16 image (ReLU: act' needs only the sign it keeps) or
  // the f32 values (tanh / ELU: act'(a2) on the f32 a2, the head operands rounded on the fly);
  // the D1 image (bf16) takes the region over after phase 5
  static constexpr int A2 = D2 + R * PITCH;
  static constexpr int A2BYTES = F32A2 ? R * A2P : R * PITCH;
  static constexpr int DZ = A2 + A2BYTES;                       // bf16 dz [64][16]
  static constexpr int DZT = DZ + R * kDzRowBytes;              // bf16 dz^T [16][64 + 8]
  static constexpr int HS = DZT + 16 * kDzTPitch;               // f32 head bias, logstd, log std, 1/var, 1/(2 var) [16] each
  static constexpr int SROW = HS + 80 * 4;                      // f32 [64][16] the chunk's row scalars
  static constexpr int RED = SROW;                              // epilogue: f32 [8 waves][16 heads][4]
  // ReLU: the W0 image (H x 32 bf16, x_off-swizzled 64-B rows) LDS-resident for the whole kernel
  // (the tanh / ELU instantiations, with their f32 a2 region, read it from L2)
  static constexpr int W0 = SROW + R * kFusedSP * 4;
  // ReLU: W_h^T as a bf16 [H][16] image (32-B rows): the d2 product's A fragment is one 16-B read
  // (head_t_frag gathers it from the head image with 8 two-byte reads otherwise)
  static constexpr int WHT = W0 + (F32A2 ? 0 : H * 64);
  // ReLU, deferred dW0 (SCHED bit 0): the previous chunk's X image stays resident while the next
  // one is staged (the two buffers alternate chunk by chunk)
  static constexpr int X2 = WHT + (F32A2 ? 0 : H * 32);
  static constexpr int TOTAL = X2 + (F32A2 ? 0 : R * 64);
  static_assert(TOTAL <= 163840, "LDS budget");
  static_assert(R * PITCH <= A2BYTES, "D1 image must fit in the a2 region");
};


// 8 f32 (two float4) -> the bf16x8 MFMA operand (RNE), for the f32-a2 (tanh / ELU) instantiations
__device__ __forceinline__ bf16x8 pack8(float4 u, float4 v) {
  const uint4 p = make_uint4(pack2(u.x, u.y), pack2(u.z, u.w), pack2(v.x, v.y), pack2(v.z, v.w));
  return __builtin_bit_cast(bf16x8, p);
}

// VALU reads of a 16x16x32 result right after the (unrolled) MFMA chain: pinned wait states as
// mfma_drain does for the 32x32x16 accumulators
__device__ __forceinline__ void mfma16_drain(f32x4 &acc) { asm volatile("s_nop 15" : "+v"(acc)); }

// STAMP (diagnostic build, ppo_ctx_phase_stamps): wave 0 sums s_memtime deltas per phase segment
// over the chunks and writes them per workgroup; the product kernel has STAMP = false.

// One net's workgroup: 8 waves; wave w owns feature tile w (features 32w..32w+31) in every
// feature-tiled phase, dW1 tiles (o-tiles 2(w&3)+{0,1}) x (i-tiles 4(w>>2)+{0..3}), dW0 tile w and
// the head-dW tiles of its features.  NH = head width padded to 2/4/6/8 (actor) or 1 (critic),
// compile-time so the per-action loops are branch-free.  Every fc product -- the three hidden
// GEMMs and the head -- is a bf16-operand MFMA with f32 accumulation (oracle.use_bf16_gemms).
// Phase barriers are LDS-only (lds_sync): waves hand each other data through LDS only, so the
// record prefetch and the weight-ring primes stay in flight across them (__syncthreads drained
// them at every phase; measured 10.40-10.47 -> 10.29-10.33 ms per iteration, profiles/r04_lds_barrier/)
//
// SCHED (ReLU instantiations; tanh / ELU always run 0): wave-local work moved out of its own
// barrier-bounded phase into an MFMA pass of the same wave, where its LDS reads and MFMAs overlap
// the pass instead of serialising behind a barrier:
//   bit 0  dW0 += D1^T X of chunk c runs at the start of chunk c+1's L1 pass (phase 2): D1 sits in
//          the wave's OWN columns of the a2 region until the wave itself overwrites them in phase
//          3, and X(c) stays in the second X buffer; phase 7 and the chunk's closing barrier go
//          away (the last chunk's dW0 runs after the loop).  Same MFMA chain into gw0 in the same
//          order: bitwise the same gradient.
// Measured and dropped (round 6): the head dW inside phase 6a (a tie); the next
// chunk's layer 0 hoisted behind the dgrad pass with phases 0 and 1 removed (16 spilled VGPRs,
// 10-17 % slower); the deferred dW0 issued after the L1 pass (3 % slower) or without the
// first-chunk branch (a tie).
template <int H, int ACT, int NH, bool ACTOR, bool STAMP, int SCHED>
__device__ __forceinline__ void fused_body(const FusedArgs &q, const FusedNet &N, char *lds,
                                           uint64_t *stamps) {
  static_assert(H == 32 * NW, "wave w owns feature tile w");
  constexpr bool F32A2 = ACT != PPO_ACT_RELU;
  constexpr bool DEFER_DW0 = (SCHED & 1) && !F32A2;
  bool have_prev = false;  // DEFER_DW0: a previous chunk's dW0 is pending
  using L = Lds<H, F32A2>;
  constexpr int z = ACTOR ? 0 : 1;
  char *ximg = lds + L::X;        // this chunk's X image
  char *xprev = lds + L::X2;      // DEFER_DW0: the previous chunk's (its dW0 runs in phase 2)
  char *const a1img = lds + L::A1;
  char *const d2img = lds + L::D2;
  char *const a2img = lds + L::A2;
  char *const d1img = lds + L::A2;  // after phase 5
  char *const whb = lds + L::WHB;
  char *const dzimg = lds + L::DZ;
  char *const dztimg = lds + L::DZT;
  const float *const b0s = reinterpret_cast<const float *>(lds + L::BIAS);
  const float *const b1s = b0s + H;
  const float *const a2f = reinterpret_cast<const float *>(lds + L::A2);

  const int tid0 = threadIdx.x, w = tid0 >> 6;
  int tid = tid0, lane = tid & 63, r = lane & 31, h = lane >> 5;
  // Lane-derived LDS addresses are loop-invariant across chunks; re-deriving them from an
  // opaque copy of the lane ids in every phase keeps the compiler from hoisting (and spilling)
  // dozens of them out of the chunk loop.
#define OPAQUE_LANE()             \
  tid = tid0;                     \
  asm volatile("" : "+v"(tid));   \
  lane = tid & 63;                \
  r = lane & 31;                  \
  h = lane >> 5
  const int A = q.act_dim;        // real actor width (NH >= A; head rows A..15 are zero)
  const int G = q.G;
  const int nchunks = (q.b + R - 1) / R;
  const int count = q.rows_n ? *q.rows_n : q.b;

  // Row staging: thread -> 8-B unit tid & 7 of row slot tid >> 3 of a chunk, in the row's state
  // half (the X image: issued a chunk ahead, at phase 6a) or its scalar half (actions, old
  // log-prob, advantage, value target: issued at phase 0 for the head phase).  Direct mode reads
  // the row's 128-B record through rows[] -- the index loaded at the previous phase 0 -- otherwise
  // the gathered xb / srow copies.  Loads come from clamped addresses and are masked
  // where they are stored (slots >= b or >= count, out-of-range rows: zero, as the prep gather
  // writes them).  One uniform address form: base + row * pitch + 8 (tid & 7) + (scalars ? hi : 0).
  const char *const rbase = q.direct ? reinterpret_cast<const char *>(q.rec)
                                     : reinterpret_cast<const char *>(q.xb);
  const int rshift = q.direct ? 7 : 6;  // 128-B records, 64-B xb / srow rows
  const int64_t rhi = q.direct ? 64
                               : reinterpret_cast<const char *>(q.srow) - reinterpret_cast<const char *>(q.xb);
  const int rlast = static_cast<int>(min(q.n_rec, static_cast<int64_t>(INT32_MAX)) - 1);
  auto row_index = [&](int c) -> int {
    const int j = min(c * R + (tid0 >> 3), q.b - 1);
    return *gptr(q.rows + j);
  };
  auto row_ok = [&](int c, int sr, int t) -> bool {
    const int j = c * R + (t >> 3);
    return j < q.b && j < count && (!q.direct || (sr >= 0 && sr <= rlast));
  };
  auto load_half = [&](int c, int sr, int t, bool scalars) -> uint64_t {
    const int j = c * R + (t >> 3);
    const int row = q.direct ? min(max(sr, 0), rlast) : min(j, q.b - 1);
    const int64_t off = (static_cast<int64_t>(row) << rshift) + 8 * (t & 7) + (scalars ? rhi : 0);
    return *gptr(reinterpret_cast<const uint64_t *>(rbase + off));
  };
  const int i_first = row_index(blockIdx.x);

  uint64_t t_body0 = 0, t_real0 = 0;
  if constexpr (STAMP) {
    t_body0 = __builtin_amdgcn_s_memtime();
    t_real0 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  stage_head_image<H>(whb, N.wh, ACTOR ? A : 1, tid, NT);
  for (int i = tid; i < 2 * H; i += NT) {
    const float *b = i < H ? N.b0 : N.b1;
    (reinterpret_cast<float *>(lds + L::BIAS))[i] = b ? b[i % H] : 0.f;
  }
  if (tid < 32) {
    const int a = tid & 15;
    const bool ok = a < (ACTOR ? A : 1);
    (reinterpret_cast<float *>(lds + L::HS))[tid] =
        tid < 16 ? ((ok && N.bh) ? N.bh[a] : 0.f) : ((ACTOR && ok) ? q.logstd[a] : 0.f);
  }
  if (tid < 16) {  // per-head Normal constants: log(std), 1/var, 1/(2 var); std = exp(logstd)
    const bool ok = ACTOR && tid < A;
    const float sd = ok ? expf(q.logstd[tid]) : 1.f;
    const float var = sd * sd;
    (reinterpret_cast<float *>(lds + L::HS))[32 + tid] = ok ? logf(sd) : 0.f;
    (reinterpret_cast<float *>(lds + L::HS))[48 + tid] = 1.f / var;
    (reinterpret_cast<float *>(lds + L::HS))[64 + tid] = 1.f / (2.f * var);
  }
  if constexpr (!F32A2) {
    for (int i = tid; i < H * 4; i += NT) {  // 16-B chunk (row i / 4, chunk i % 4) of W0
      const uint4 v = reinterpret_cast<const uint4 *>(N.w0b)[i];
      *reinterpret_cast<uint4 *>(lds + L::W0 + x_off(i >> 2, i & 3)) = v;
    }
    const int nh_real = ACTOR ? A : 1;
    for (int i = tid; i < H * 16; i += NT) {  // W_h^T[f][a] = bf16(W_h[a][f]), heads >= A zero
      const int a = i / H, f = i % H;           // coalesced reads of W_h's rows
      const float v = a < nh_real ? N.wh[a * H + f] : 0.f;
      *reinterpret_cast<uint16_t *>(lds + L::WHT + 2 * (f * 16 + a)) = bf16_bits(v);
    }
  }
  const float *const hbias = reinterpret_cast<const float *>(lds + L::HS);
  uint64_t xpre = load_half(blockIdx.x, i_first, tid0, false);
  bool xok = row_ok(blockIdx.x, i_first, tid0);
  if constexpr (DEFER_DW0) {
    // a workgroup without chunks runs the after-loop dW0 on these: exact zeros (the D1 region
    // and L::X, its `ximg`), so it adds +0 instead of stale LDS contents
    for (int i = tid; i < R * (2 * H) / 16; i += NT)
      *reinterpret_cast<uint4 *>(lds + L::A2 + 16 * i) = make_uint4(0u, 0u, 0u, 0u);
    for (int i = tid; i < R * 64 / 16; i += NT)
      *reinterpret_cast<uint4 *>(lds + L::X + 16 * i) = make_uint4(0u, 0u, 0u, 0u);
  }
  lds_sync();

  // ---- persistent accumulators ----
  f32x16 gw1[2][4];   // dW1 tiles: o-tiles 2*(w&3)+{0,1}, i-tiles 4*(w>>2)+{0..3}
  f32x16 gw0;         // dW0 tile: features 32w.., input columns 0..31
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) gw1[a][b][e] = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) gw0[e] = 0.f;
  f32x4 ghw[2];       // head dW: heads 4*(lane>>4)+i, features 32w + 16u + (lane & 15)
#pragma unroll
  for (int u = 0; u < 2; ++u) ghw[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gb1 = 0.f, gb0 = 0.f;                 // rs16-scattered bias grads (feature rs16_feature)
  float g_bh = 0.f, g_ls = 0.f, g_loss = 0.f;  // head (lane & 15) partials

  int chunk = blockIdx.x;
  int icur = i_first;  // this chunk's row index (thread's slot)
  uint64_t t_prev = 0, t_acc[kStampSlots];
  if constexpr (STAMP) {
#pragma unroll
    for (int p = 0; p < kStampSlots; ++p) t_acc[p] = 0;
    t_prev = __builtin_amdgcn_s_memtime();
    t_acc[10] = t_prev - t_body0;
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
#define STAMP_AT(p)                                       \
  if constexpr (STAMP) {                                  \
    const uint64_t t_now = __builtin_amdgcn_s_memtime();  \
    t_acc[p] += t_now - t_prev;                           \
    t_prev = t_now;                                       \
  }

  bf16x8 ring[PD + 1];
  // the current chunk's row scalars / validity and the next chunk's row index (loop-carried)
  uint64_t srow_c = 0;
  bool sok_c = false;
  int inext = 0;
  for (; chunk < nchunks; chunk += G) {
    // ---- phase 0: the chunk's rows (loaded during the previous chunk) -> X image and the row
    //      scalars (actions, old log-prob, advantage, value target: 64 x 64 B); W0 fragments;
    //      the next chunk's row indices ----
    if constexpr (DEFER_DW0) {  // X(c) into the buffer X(c-2) used; X(c-1) stays for its dW0
      char *const t = ximg;
      ximg = xprev;
      xprev = t;
    }
    OPAQUE_LANE();
    *reinterpret_cast<uint64_t *>(ximg + x_off(tid >> 3, (tid & 7) >> 1) + 8 * (tid & 1)) = xok ? xpre : 0;
    sok_c = xok;
    srow_c = load_half(chunk, icur, tid, true);
    inext = row_index(chunk + G);  // lands by phase 6a
    bf16x8 w0f[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr (F32A2)
        w0f[s] = *reinterpret_cast<const bf16x8 *>(N.w0b + (32 * w + r) * kFusedKX + 16 * s + 8 * h);
      else
        w0f[s] = lds_b128(lds + L::W0 + x_off(32 * w + r, 2 * s + h));
    }
    lds_sync();
    STAMP_AT(0);

    // ---- phase 1: a1 = act(W0 x + b0) -> A1 image ----
    OPAQUE_LANE();
    wring_prime<H>(w_frag_base<H>(N.w1b, w, lane), ring);  // for phase 2
    {
      f32x16 acc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          acc[t] = mfma(w0f[s], lds_b128(ximg + x_off(32 * t + r, 2 * s + h)), acc[t]);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int f0 = 32 * w + 8 * g + 4 * h;
        const float4 bv = *reinterpret_cast<const float4 *>(b0s + f0);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const float y0 = act_forward(acc[t][4 * g] + bv.x, ACT);
          const float y1 = act_forward(acc[t][4 * g + 1] + bv.y, ACT);
          const float y2 = act_forward(acc[t][4 * g + 2] + bv.z, ACT);
          const float y3 = act_forward(acc[t][4 * g + 3] + bv.w, ACT);
          *reinterpret_cast<uint2 *>(a1img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h) =
              make_uint2(pack2(y0, y1), pack2(y2, y3));
        }
      }
    }
    lds_sync();
    STAMP_AT(1);

    // ---- phase 2: a2 = W1 a1 (f32 accumulators) ----
    OPAQUE_LANE();
    // the previous chunk's dW0 += D1^T X (phase 7 of the undeferred schedule): the wave's own D1
    // columns (untouched until its phase 3 below) and X(c-1); every transposed read first, then
    // the four chained MFMAs.
#define DEFERRED_DW0()                                                     \
  {                                                                        \
    bf16x8 fd[R / 16], fx[R / 16];                                         \
    _Pragma("unroll") for (int ks = 0; ks < R / 16; ++ks) {                \
      fd[ks] = tr_frag(d1img, L::PITCH, 16 * ks, 32 * w, lane);            \
      fx[ks] = tr_frag_x(xprev, 16 * ks, lane);                            \
    }                                                                      \
    _Pragma("unroll") for (int ks = 0; ks < R / 16; ++ks) gw0 = mfma(fd[ks], fx[ks], gw0); \
  }
    if constexpr (DEFER_DW0) {
      if (have_prev) DEFERRED_DW0()  // (a uniform branch: none before the first chunk)
      have_prev = true;
    }
    f32x16 a2[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) a2[t][e] = 0.f;
    mlp_pass<H>(w_frag_base<H>(N.w1b, w, lane), a1img, r, h, ring, a2);
    *reinterpret_cast<uint64_t *>(lds + L::SROW + tid0 * 8) = sok_c ? srow_c : 0;  // landed during phases 1-2
    STAMP_AT(2);

    // ---- phase 3: bias + act -> a2 region ----
    OPAQUE_LANE();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * w + 8 * g + 4 * h;
      const float4 bv = *reinterpret_cast<const float4 *>(b1s + f0);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float y0 = act_forward(a2[t][4 * g] + bv.x, ACT);
        const float y1 = act_forward(a2[t][4 * g + 1] + bv.y, ACT);
        const float y2 = act_forward(a2[t][4 * g + 2] + bv.z, ACT);
        const float y3 = act_forward(a2[t][4 * g + 3] + bv.w, ACT);
        if constexpr (F32A2)
          *reinterpret_cast<float4 *>(a2img + (32 * t + r) * L::A2P + 4 * f0) = make_float4(y0, y1, y2, y3);
        else
          *reinterpret_cast<uint2 *>(a2img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h) =
              make_uint2(pack2(y0, y1), pack2(y2, y3));
      }
    }
    lds_sync();
    STAMP_AT(3);

    // ---- phase 4: head z = a2 . W_h^T on the 16x16x32 MFMA, then the per-(row, action) loss
    //      head in registers -> dz images.  Waves w and w + 4 form the same 16-row z tile
    //      (8 MFMAs each) and split its rows: lane -> head n = lane & 15, rows
    //      16 (w & 3) + 4 (lane >> 4) + 2 (w >> 2) + {0, 1} ----
    OPAQUE_LANE();
    {
      const int n = lane & 15, qg = lane >> 4, tile = w & 3, half = w >> 2;
      const float *const srl = reinterpret_cast<const float *>(lds + L::SROW);
      const int lr0 = 16 * tile + 4 * qg + 2 * half;  // this lane's two rows: lr0, lr0 + 1
      // Every LDS operand of the loss is read here, unconditionally (in-range addresses; masked
      // where used), before the z products and the exchange barrier: behind per-lane branches
      // they were one LDS round trip each, after the barrier, row after row.  The two rows'
      // chains below are straight-line code (selects, not branches), so they interleave.
      float xs[2] = {0.f, 0.f}, olp[2] = {0.f, 0.f}, advs[2] = {0.f, 0.f}, vts[2] = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float *sp = srl + (lr0 + i) * kFusedSP;
        if constexpr (ACTOR) {
          xs[i] = sp[n];
          olp[i] = sp[A];
          advs[i] = sp[A + 1];
        } else {
          vts[i] = sp[A + 2];
        }
      }
      const float h_b = hbias[ACTOR ? n : 0];
      const float h_lsd = ACTOR ? hbias[32 + n] : 0.f, h_ivar = ACTOR ? hbias[48 + n] : 0.f;
      // K split between the wave pair: wave half 0 sums k-steps 0..H/64-1, half 1 the rest
      // (half the LDS reads and MFMAs per wave); each hands the partner the two rows it keeps
      // through the (still free) D2 region.  z = P_lo + P_hi on both sides (commutative), the
      // same order as the rollout's policy kernel.
      f32x4 zacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = half * (H / 64); s < (half + 1) * (H / 64); ++s) {
        bf16x8 av;
        if constexpr (F32A2) {
          const float *p = a2f + (16 * tile + n) * (L::A2P / 4) + 32 * s + 8 * qg;
          av = pack8(*reinterpret_cast<const float4 *>(p), *reinterpret_cast<const float4 *>(p + 4));
        } else {
          av = lds_b128(a2img + img_off(16 * tile + n, 4 * s + qg, L::PITCH));
        }
        zacc = mfma16(av, lds_b128(whb + n * HeadImg<H>::PITCH + 2 * (32 * s + 8 * qg)), zacc);
      }
      mfma16_drain(zacc);
      float *const xch = reinterpret_cast<float *>(lds + L::D2);  // [8 waves][64 lanes][2]
      *reinterpret_cast<float2 *>(xch + 2 * (w * 64 + lane)) =
          half ? make_float2(zacc[0], zacc[1]) : make_float2(zacc[2], zacc[3]);
      lds_sync();
      const float2 px = *reinterpret_cast<const float2 *>(xch + 2 * ((w ^ (NW / 2)) * 64 + lane));
      const float zr[2] = {(half ? zacc[2] : zacc[0]) + px.x, (half ? zacc[3] : zacc[1]) + px.y};
      bool valid[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) valid[i] = chunk * R + lr0 + i < count;
      float dz[2];
      if constexpr (ACTOR) {
        // row after row: the interleaved branch-free form of the critic raised this body's
        // register pressure past the cap (spills landing in the dW1 phase: measured slower)
        const bool act_lane = n < A;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          dz[i] = 0.f;
          float y = 0.f, d = 0.f, lp = 0.f;
          if (act_lane) {
            const float zz = N.bh ? zr[i] + h_b : zr[i];
            y = tanhf(zz);
            const float mu = q.omv * y;
            const float x = valid[i] ? xs[i] : mu;
            d = x - mu;
            lp = ((-(d * d)) * (0.5f * h_ivar) - h_lsd) - kLogSqrt2Pi;  // 0.5/var: exact scaling
          }
          // Normal.log_prob(...).sum(1): fixed xor tree over the 16 head lanes (pads are 0), the
          // same tree as the rollout's policy kernel
          const float logp = row16_sum(lp);
          const float old_lp = valid[i] ? olp[i] : logp;
          const float adv = valid[i] ? advs[i] : 0.f;
          const float ratio = expf(logp - old_lp);
          const float s1 = ratio * adv;
          const float cl = ratio < q.clip_lo ? q.clip_lo : (ratio > q.clip_hi ? q.clip_hi : ratio);
          const float s2 = cl * adv;
          const float mn = (s1 != s1 || s2 != s2) ? (s1 + s2) : (s2 < s1 ? s2 : s1);
          const float gg = -q.inv_b;
          const float g1 = (s1 < s2) ? gg : (s1 == s2 ? gg * 0.5f : 0.f);
          const float g2 = (s2 < s1) ? gg : (s1 == s2 ? gg * 0.5f : 0.f);
          const bool inside = (ratio >= q.clip_lo) && (ratio <= q.clip_hi);
          const float dratio = g1 * adv + (inside ? g2 * adv : 0.f);
          const float dlogp = valid[i] ? dratio * ratio : 0.f;
          if (act_lane) {
            const float dmu = dlogp * (d * h_ivar);
            dz[i] = (dmu * q.omv) * (1.f - y * y);
            if (valid[i]) {
              g_ls += dlogp * ((d * d) * h_ivar - 1.f) - q.ent_coef * q.inv_ba;
              g_bh += dz[i];
            }
          }
          if (valid[i] && n == 0) g_loss += mn;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const float v = N.bh ? zr[i] + h_b : zr[i];
          const float vt = valid[i] ? vts[i] : v;
          const float diff = v - vt;
          const float ad = fabsf(diff);
          const float hl = (ad < 1.f) ? 0.5f * ad * ad : (ad - 0.5f);
          g_loss = (valid[i] && n == 0) ? g_loss + hl : g_loss;
          dz[i] = n == 0 ? q.inv_b * (diff < -1.f ? -1.f : (diff > 1.f ? 1.f : diff)) : 0.f;
          g_bh = n == 0 ? g_bh + dz[i] : g_bh;
        }
      }
      // bf16 dz images (the head-backward operands; zero for padded heads and invalid rows)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        *reinterpret_cast<uint16_t *>(dzimg + (lr0 + i) * kDzRowBytes + 2 * n) = bf16_bits(dz[i]);
      *reinterpret_cast<uint32_t *>(dztimg + n * kDzTPitch + 2 * lr0) = pack2(dz[0], dz[1]);
    }
    lds_sync();
    STAMP_AT(4);

    // ---- phase 5: d2 = (dz . W_h) * act'(a2) on MFMA -> bias grad, D2 image; head dW ----
    OPAQUE_LANE();
    {
      // the A operand W_h^T of the wave's features, both row tiles' dz fragments and (ReLU) the
      // bf16 a2 values act' needs, all read up front: one LDS round trip for the phase's inputs
      bf16x8 wht;
      if constexpr (F32A2) wht = head_t_frag<H>(whb, w, lane);
      else wht = lds_b128(lds + L::WHT + (32 * w + r) * 32 + 16 * h);
      bf16x8 dzf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) dzf[t] = lds_b128(dzimg + (32 * t + r) * kDzRowBytes + 16 * h);
      uint2 yb[2][4];
      if constexpr (!F32A2) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            yb[t][g] = *reinterpret_cast<const uint2 *>(a2img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h);
      }
      float bsum[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) bsum[e] = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) {  // one row tile at a time (one live accumulator)
        f32x16 acc[1];
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[0][e] = 0.f;
        acc[0] = mfma(wht, dzf[t], acc[0]);
        mfma_drain(acc);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float ya, ybv, yc, yd;
          if constexpr (F32A2) {
            const float4 yv = *reinterpret_cast<const float4 *>(a2img + (32 * t + r) * L::A2P + 4 * (32 * w + 8 * g + 4 * h));
            ya = yv.x, ybv = yv.y, yc = yv.z, yd = yv.w;
          } else {
            const uint2 yv = yb[t][g];
            ya = bf_lo(yv.x), ybv = bf_hi(yv.x), yc = bf_lo(yv.y), yd = bf_hi(yv.y);
          }
          const float d0 = act_backward(acc[0][4 * g], ya, ACT);
          const float d1 = act_backward(acc[0][4 * g + 1], ybv, ACT);
          const float d2 = act_backward(acc[0][4 * g + 2], yc, ACT);
          const float d3 = act_backward(acc[0][4 * g + 3], yd, ACT);
          bsum[4 * g] += d0;
          bsum[4 * g + 1] += d1;
          bsum[4 * g + 2] += d2;
          bsum[4 * g + 3] += d3;
          *reinterpret_cast<uint2 *>(d2img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h) =
              make_uint2(pack2(d0, d1), pack2(d2, d3));
        }
      }
      gb1 += rs16(bsum, lane);
    }
    // head dW += dz^T a2 over the chunk's 64 rows: wave w's two 16-feature tiles
#define HEAD_DW()                                                                                 \
  _Pragma("unroll") for (int ks = 0; ks < R / 32; ++ks) {                                         \
    const bf16x8 af = lds_b128(dztimg + (lane & 15) * kDzTPitch + 2 * (32 * ks + 8 * (lane >> 4))); \
    _Pragma("unroll") for (int u = 0; u < 2; ++u) {                                               \
      bf16x8 bv;                                                                                  \
      if constexpr (F32A2) {                                                                      \
        float v[8];                                                                               \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) v[j] =                                      \
            a2f[(32 * ks + 8 * (lane >> 4) + j) * (L::A2P / 4) + 32 * w + 16 * u + (lane & 15)]; \
        bv = pack8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));     \
      } else {                                                                                    \
        bv = tr_frag16(a2img, L::PITCH, 32 * ks, 32 * w + 16 * u, lane);                          \
      }                                                                                           \
      ghw[u] = mfma16(af, bv, ghw[u]);                                                            \
    }                                                                                             \
  }
    HEAD_DW()
    lds_sync();
    STAMP_AT(5);

    // ---- phase 6a: dW1 += D2^T A1 (k = the chunk's 64 rows) ----
    // Rolled over the four 16-row k-steps (unrolled, the compiler hoists all 80 transposed
    // reads and spills).  The dgrad weight ring is primed first so its L2 latency hides behind
    // this LDS-only phase.
    OPAQUE_LANE();
    wring_prime<H>(w_frag_base<H>(N.w1bt, w, lane), ring);
    // the next chunk's states: in flight until the next phase 0
    xpre = load_half(chunk + G, inext, tid, false);
    xok = row_ok(chunk + G, inext, tid);
    icur = inext;
#pragma unroll 1
    for (int ks = 0; ks < R / 16; ++ks) {
      bf16x8 af[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = tr_frag(d2img, L::PITCH, 16 * ks, 32 * (2 * (w & 3) + a), lane);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const bf16x8 bv = tr_frag(a1img, L::PITCH, 16 * ks, 32 * (4 * (w >> 2) + b), lane);
#pragma unroll
        for (int a = 0; a < 2; ++a) gw1[a][b] = mfma(af[a], bv, gw1[a][b]);
      }
    }
    STAMP_AT(6);

    // ---- phase 6b: d1 = (W1^T d2) * act'(a1) -> D1 image (the a2 region is free) ----
    OPAQUE_LANE();
    {
      f32x16 acc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
      mlp_pass<H>(w_frag_base<H>(N.w1bt, w, lane), d2img, r, h, ring, acc);
      STAMP_AT(7);
      OPAQUE_LANE();
      // act'(a1): ReLU needs only the sign, which the bf16 image keeps exactly; tanh / ELU
      // recompute this wave's f32 a1 tile (the phase-1 product; X is still resident), one row
      // tile at a time
      float bsum[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) bsum[e] = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x16 y1;
        if constexpr (ACT != PPO_ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 16; ++e) y1[e] = 0.f;
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const bf16x8 wf = *reinterpret_cast<const bf16x8 *>(N.w0b + (32 * w + r) * kFusedKX + 16 * s + 8 * h);
            y1 = mfma(wf, lds_b128(ximg + x_off(32 * t + r, 2 * s + h)), y1);
          }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float ya, yb, yc, yd;
          if constexpr (ACT == PPO_ACT_RELU) {
            const uint2 yv = *reinterpret_cast<const uint2 *>(a1img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h);
            ya = bf_lo(yv.x), yb = bf_hi(yv.x), yc = bf_lo(yv.y), yd = bf_hi(yv.y);
          } else {
            const float4 bv = *reinterpret_cast<const float4 *>(b0s + 32 * w + 8 * g + 4 * h);
            ya = act_forward(y1[4 * g] + bv.x, ACT);
            yb = act_forward(y1[4 * g + 1] + bv.y, ACT);
            yc = act_forward(y1[4 * g + 2] + bv.z, ACT);
            yd = act_forward(y1[4 * g + 3] + bv.w, ACT);
          }
          const float d0 = act_backward(acc[t][4 * g], ya, ACT);
          const float d1 = act_backward(acc[t][4 * g + 1], yb, ACT);
          const float d2 = act_backward(acc[t][4 * g + 2], yc, ACT);
          const float d3 = act_backward(acc[t][4 * g + 3], yd, ACT);
          bsum[4 * g] += d0;
          bsum[4 * g + 1] += d1;
          bsum[4 * g + 2] += d2;
          bsum[4 * g + 3] += d3;
          *reinterpret_cast<uint2 *>(d1img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h) =
              make_uint2(pack2(d0, d1), pack2(d2, d3));
        }
      }
      gb0 += rs16(bsum, lane);
    }
    STAMP_AT(8);

    // ---- phase 7: dW0 += D1^T X (the wave's own D1 columns, written by this wave above: no
    //      barrier before it; the chunk's closing barrier follows).  DEFER_DW0: in the next
    //      chunk's phase 2 (or after the loop), and no closing barrier: the next chunk's X goes to
    //      the other buffer, and every other region it writes before its phase-0 barrier is
    //      read by no wave after this chunk's phase-5 barrier ----
    if constexpr (!DEFER_DW0) {
      OPAQUE_LANE();
      {
        // every transposed fragment read issued first (16 ds_read_b64_tr_b16, 32 registers: the
        // dgrad accumulators are dead here), then the four chained MFMAs -- one LDS round trip
        // for the phase instead of one per k-step
        bf16x8 fd[R / 16], fx[R / 16];
#pragma unroll
        for (int ks = 0; ks < R / 16; ++ks) {
          fd[ks] = tr_frag(d1img, L::PITCH, 16 * ks, 32 * w, lane);
          fx[ks] = tr_frag_x(ximg, 16 * ks, lane);
        }
#pragma unroll
        for (int ks = 0; ks < R / 16; ++ks) gw0 = mfma(fd[ks], fx[ks], gw0);
      }
      lds_sync();
    }
    STAMP_AT(9);
  }
  if constexpr (DEFER_DW0) {  // the last chunk's dW0 (wave-local: D1 own columns, its X image)
    {  // (a workgroup without chunks adds the prologue's zeros)
      OPAQUE_LANE();
      char *const xlast = ximg;
      bf16x8 fd[R / 16], fx[R / 16];
#pragma unroll
      for (int ks = 0; ks < R / 16; ++ks) {
        fd[ks] = tr_frag(d1img, L::PITCH, 16 * ks, 32 * w, lane);
        fx[ks] = tr_frag_x(xlast, 16 * ks, lane);
      }
#pragma unroll
      for (int ks = 0; ks < R / 16; ++ks) gw0 = mfma(fd[ks], fx[ks], gw0);
    }
  }
#undef STAMP_AT
#undef OPAQUE_LANE
#undef HEAD_DW
#undef DEFERRED_DW0

  // ================= epilogue: one partial-gradient slab per workgroup =================
  tid = tid0;
  lane = tid & 63;
  r = lane & 31;
  h = lane >> 5;
  if constexpr (STAMP) t_prev = __builtin_amdgcn_s_memtime();
  float *slab = q.slabs + static_cast<int64_t>(blockIdx.x) * q.slab_stride;
  // dW1 (o, i) row-major [H][H]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int o0 = 32 * (2 * (w & 3) + a), i0 = 32 * (4 * (w >> 2) + b);
#pragma unroll
      for (int e = 0; e < 16; ++e)
        slab[N.off_w1 + static_cast<int64_t>(o0 + reg_feature(e, h)) * H + i0 + r] = gw1[a][b][e];
    }
  // dW0 (f, k) row-major [H][din]
  if (r < q.din) {
#pragma unroll
    for (int e = 0; e < 16; ++e)
      slab[N.off_w0 + static_cast<int64_t>(32 * w + reg_feature(e, h)) * q.din + r] = gw0[e];
  }
  if ((lane & 1) == 0) {
    const int f = 32 * w + rs16_feature(lane);
    if (N.b1) slab[N.off_b1 + f] = gb1;
    if (N.b0) slab[N.off_b0 + f] = gb0;
  }
  // head dW (a, f) row-major [A_net][H]
  const int na = ACTOR ? A : 1;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int a = 4 * (lane >> 4) + i;
      if (a < na) slab[N.off_wh + static_cast<int64_t>(a) * H + 32 * w + 16 * u + (lane & 15)] = ghw[u][i];
    }
  // head bias / log-std / loss partials: per lane (head lane & 15) -> the 4 lane groups of a
  // wave in a fixed xor order -> waves 0..7 in order through LDS
  float *red = reinterpret_cast<float *>(lds + L::RED);  // [8][16][4]
  {
    g_bh += __shfl_xor(g_bh, 16, 64);
    g_bh += __shfl_xor(g_bh, 32, 64);
    g_ls += __shfl_xor(g_ls, 16, 64);
    g_ls += __shfl_xor(g_ls, 32, 64);
    g_loss += __shfl_xor(g_loss, 16, 64);
    g_loss += __shfl_xor(g_loss, 32, 64);
    if (lane < 16) {
      float *dst = red + (w * 16 + lane) * 4;
      dst[0] = g_bh;
      dst[1] = g_ls;
      dst[2] = g_loss;
    }
  }
  lds_sync();
  if (tid < na) {
    float sb = 0.f, sl = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      sb += red[(v * 16 + tid) * 4];
      sl += red[(v * 16 + tid) * 4 + 1];
    }
    if (N.bh) slab[N.off_bh + tid] = sb;
    if (ACTOR) slab[q.off_logstd + tid] = sl;
  }
  if (tid == 0) {
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) s += red[(v * 16) * 4 + 2];
    q.loss_part[2 * blockIdx.x + z] = s;
  }
  if constexpr (STAMP) {  // after every wave's slab stores have drained
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const uint64_t t_end = __builtin_amdgcn_s_memtime();
    const uint64_t r_end = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    t_acc[11] = t_end - t_prev;
    t_acc[12] = r_end - t_real0;
    if (tid0 == 0) {
      uint64_t *dst = stamps + (static_cast<int64_t>(z) * gridDim.x + blockIdx.x) * kStampSlots;
#pragma unroll
      for (int p = 0; p < kStampSlots; ++p) dst[p] = t_acc[p];
    }
  }
}

template <int H, int ACT, int NA, bool STAMP, int SCHED = 0>
__global__ __launch_bounds__(NT, 1) void fused_update_kernel(FusedArgs q, uint64_t *stamps) {
  __shared__ __attribute__((aligned(16))) char lds[Lds<H, ACT != PPO_ACT_RELU>::TOTAL];
  if (blockIdx.y == 0) fused_body<H, ACT, NA, true, STAMP, SCHED>(q, q.net[0], lds, stamps);
  else fused_body<H, ACT, 1, false, STAMP, SCHED>(q, q.net[1], lds, stamps);
}

bool fused_width_ok(int hidden) { return hidden == 256; }

int fused_prep_launch(const FusedArgs &q, const TimRec &rec, hipStream_t st) {
  const int row_blocks = q.rec ? static_cast<int>(ceil_div(static_cast<int64_t>(q.b) * 8, 256))
                               : ceil_div(q.b, 256);
  const int64_t per_net = static_cast<int64_t>(q.hidden) * (kFusedKX + q.hidden);
  const int w_blocks = q.pack_w ? static_cast<int>(ceil_div(2 * per_net, 256)) : 0;
  if (row_blocks + w_blocks == 0) return 0;
  launch_k(rec, fused_prep_kernel, dim3(row_blocks + w_blocks), dim3(256), 0, st, q, row_blocks);
  PPO_LAUNCHED();
  return 0;
}

int fused_records_launch(uint4 *rec, const float *states, const float *actions,
                         const float *old_logp, const float *adv, const float *vtarget,
                         int64_t n_rows, int din, int act_dim, const TimRec &trec, hipStream_t st) {
  PPO_REQUIRE(din >= 1 && din <= kFusedKX && act_dim >= 1 && act_dim + 3 <= kFusedSP,
              "fused records: din %d / act_dim %d out of range", din, act_dim);
  if (n_rows <= 0) return 0;
  launch_k(trec, fused_records_kernel, dim3(ceil_div(n_rows, 256)), dim3(256), 0, st, rec, states,
           actions, old_logp, adv, vtarget, n_rows, din, act_dim);
  PPO_LAUNCHED();
  return 0;
}

int gae_records_launch(const GaeRecordArgs &g, bool reward_f64, const TimRec &rec,
                       hipStream_t st) {
  PPO_REQUIRE(g.din >= 1 && g.din <= kFusedKX && g.act_dim >= 1 && g.act_dim + 3 <= kFusedSP &&
                  g.n > 0 && g.t_len > 0 && g.t_len <= 16 * 16,
              "gae_records: din %d / act_dim %d / n %d / t %d out of range", g.din, g.act_dim, g.n,
              g.t_len);
  auto go = [&](auto rt_tag, auto eb_tag, auto k_tag) {
    using RT = decltype(rt_tag);
    constexpr int EB = decltype(eb_tag)::value, KM = decltype(k_tag)::value;
    TimRec r = rec;
    if (tim_active())
      r.name = intern_name("gae_records_kernel<%s, %d, %d>", sizeof(RT) == 8 ? "double" : "float",
                           EB, KM);
    launch_k(r, gae_records_kernel<RT, EB, KM>, dim3(ceil_div(g.n, EB)), dim3(EB * 16), 0, st, g);
  };
  auto by_k = [&](auto rt_tag, auto eb_tag) {
    if (g.t_len <= 16 * 8) go(rt_tag, eb_tag, std::integral_constant<int, 8>{});
    else go(rt_tag, eb_tag, std::integral_constant<int, 16>{});
  };
  auto by_eb = [&](auto rt_tag) {  // gae_pipe_kernel's envs per block
    if (g.n >= 16384) by_k(rt_tag, std::integral_constant<int, 32>{});
    else by_k(rt_tag, std::integral_constant<int, 16>{});
  };
  if (reward_f64) by_eb(double{});
  else by_eb(float{});
  PPO_LAUNCHED();
  return 0;
}

int adam_pack_launch(const AdamPackArgs &a, const TimRec &rec, hipStream_t st) {
  PPO_REQUIRE(a.H % kPackTile == 0 && a.din >= 1 && a.din <= kFusedKX && a.n > 0,
              "adam_pack: H=%d din=%d", a.H, a.din);
  const int gen_blocks = static_cast<int>(ceil_div(a.n, 256));
  const int tiles = a.H / kPackTile;
  launch_k(rec, adam_pack_kernel, dim3(gen_blocks + 2 * tiles * tiles), dim3(256), 0, st, a,
           gen_blocks);
  PPO_LAUNCHED();
  return 0;
}

// PPO_TAIL_GROUPS=8|16|32: float4 groups per step-tail block (A/B knob; bitwise the same sums)
static const int g_tail_groups = [] {
  const char *v = getenv("PPO_TAIL_GROUPS");
  return v ? atoi(v) : 32;
}();

int step_tail_launch(const ReduceArgs &r, const TailArgs &t, const TimRec &rec, hipStream_t st) {
  PPO_REQUIRE(t.a.H % 4 == 0 && t.a.din >= 1 && t.a.din <= kFusedKX &&
                  (!t.reduce || r.total == t.a.n),
              "step tail: H=%d din=%d", t.a.H, t.a.din);
  auto go = [&](auto gc) {
    constexpr int G = decltype(gc)::value, NT = G * kRedChunks;
    const int red_blocks = static_cast<int>(ceil_div(t.a.n, 4 * G));
    const int gather_blocks = static_cast<int>(ceil_div(static_cast<int64_t>(t.b) * 8, NT));
    TimRec named = rec;  // the launched instantiation's name (rocprof's, for the agreement check)
    if (tim_active()) named.name = intern_name("step_tail_kernel<%d>", G);
    launch_k(named, step_tail_kernel<G>, dim3(red_blocks + gather_blocks), dim3(NT), 0, st, r, t,
             red_blocks);
  };
  if (g_tail_groups == 8) go(std::integral_constant<int, 8>{});
  else if (g_tail_groups == 16) go(std::integral_constant<int, 16>{});
  else go(std::integral_constant<int, 32>{});
  PPO_LAUNCHED();
  return 0;
}

// PPO_FUSED_SCHED=0|1: the ReLU kernel's phase schedule (fused_body SCHED; A/B knob, bitwise the
// same gradient for every value), read at every launch so one process can compare them
static int env_fused_sched() {
  const char *v = getenv("PPO_FUSED_SCHED");
  return v ? atoi(v) : 1;  // default: dW0 deferred (round 6: 1-4 % faster per launch, bitwise equal)
}

int fused_sched(int act) {
  const int s = env_fused_sched();
  return act == PPO_ACT_RELU && s == 1 ? 1 : 0;
}

template <int ACT, int NA, int SCHED>
static void launch_sched(const FusedArgs &q, const TimRec &rec, hipStream_t st) {
  uint64_t *nul = nullptr;
  if (ACT == PPO_ACT_RELU && q.stamps)
    launch_k(rec, fused_update_kernel<256, ACT, NA, true, SCHED>, dim3(q.G, 2), dim3(NT), 0, st, q, q.stamps);
  else
    launch_k(rec, fused_update_kernel<256, ACT, NA, false, SCHED>, dim3(q.G, 2), dim3(NT), 0, st, q, nul);
}

template <int ACT, int NA>
static void launch_na(const FusedArgs &q, const TimRec &rec, hipStream_t st) {
  if constexpr (ACT == PPO_ACT_RELU) {
    const int sched = fused_sched(ACT);
    if (sched == 1) return launch_sched<ACT, NA, 1>(q, rec, st);
  }
  launch_sched<ACT, NA, 0>(q, rec, st);
}

template <int ACT>
static void launch_act(const FusedArgs &q, const TimRec &rec, hipStream_t st) {
  if (q.act_dim <= 2) launch_na<ACT, 2>(q, rec, st);
  else if (q.act_dim <= 4) launch_na<ACT, 4>(q, rec, st);
  else if (q.act_dim <= 6) launch_na<ACT, 6>(q, rec, st);
  else launch_na<ACT, 8>(q, rec, st);
}

int fused_update_launch(const FusedArgs &q, const TimRec &rec, hipStream_t st) {
  PPO_REQUIRE(q.hidden == 256, "fused update: hidden width %d not compiled", q.hidden);
  PPO_REQUIRE(q.G >= 1 && q.G <= kFusedMaxWG, "fused update: bad workgroup count %d", q.G);
  PPO_REQUIRE(q.act_dim >= 1 && q.act_dim <= kFusedMaxAct, "fused update: act_dim %d", q.act_dim);
  PPO_REQUIRE(!q.stamps || q.act == PPO_ACT_RELU, "fused update: phase stamps only for ReLU");
  PPO_REQUIRE(q.rows && q.b > 0 && (!q.direct || (q.rec && q.n_rec > 0)),
              "fused update: rows / records missing (b=%d, direct=%d)", q.b, int(q.direct));
  if (q.act == PPO_ACT_RELU) launch_act<PPO_ACT_RELU>(q, rec, st);
  else if (q.act == PPO_ACT_TANH) launch_act<PPO_ACT_TANH>(q, rec, st);
  else launch_act<PPO_ACT_ELU>(q, rec, st);
  PPO_LAUNCHED();
  return 0;
}

}  // namespace ppo
