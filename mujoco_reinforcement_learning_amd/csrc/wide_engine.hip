// The wide layered path (wide_path.h): bf16-resident rollout forward and minibatch
// forward + loss + backward for ReLU actor-critics the fused kernels do not cover (Humanoid-v4:
// O=376, 3x512, A=17 -- BASELINE configs[3]).
//
// Per optimizer step (ppo.py:108-135 for one minibatch, both nets in every launch):
//   pack     bf16 weight images W [out][in] and W^T [in][out] from the f32 masters (zero padded)
//   gather   x[j] = bf16(states[rows[j]])                         (A5 row gather + operand rounding)
//   FWD      h_l = relu(h_{l-1} W_l^T + b_l)                       (wide_gemm.h NT, bf16 out)
//   F32      z = h_{L-1} W_L^T                                      (head pre-activations)
//   loss     tanh / Normal log-prob / clipped surrogate / Huber / entropy per row (A11-A13),
//            dz (bf16), per-block partials of the logstd and head-bias gradients and the losses
//   WGRAD    slab[s] = dz^T h_{L-1}, then per hidden layer dZ_l^T h_{l-1} (split-K over rows)
//   DGRAD    dZ_{l-1} = (dZ_l W_l) * relu'(h_{l-1}), written over h_{l-1}, + bias column sums
//   reduce   fixed-order sums of the slabs / partials into the flat gradient + loss scalars
// The same formulas as update_head_kernel / policy_head_kernel (mlp_engine.hip) on the bf16
// emulation's operands: every product's operands rounded to bf16, f32 accumulation, biases,
// losses and activation derivatives in f32 (the derivative of ReLU from the bf16 output: the
// sign of a value survives RNE rounding, so it is the f32 output's).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <new>

#include "common.h"
#include "fused_common.h"
#include "reduce_slabs.h"
#include "timing.h"
#include "wide_gemm.h"
#include "wide_ops.h"
#include "wide_path.h"

namespace ppo {

using wide::WideBatch;
using wide::WideProblem;

static inline int64_t rup(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
constexpr int kWideSplits = 16;      // WGRAD split-K slabs of the hidden layers (at most)
// Split-K slabs of the hidden-layer WGRAD: PPO_WIDE_SPLITS (1 .. 16, default 8).  Every slab is
// a full f32 copy of the layer's gradient written by WGRAD and read by wide_reduce_kernel, so at
// small minibatches (8,192 rows per rank) fewer, longer splits move fewer bytes; since the WGRAD
// shares its launch with the layer's DGRAD (wide_pair_kernel) its own block count matters less,
// and with 8-split slabs on the fold's fast path the Humanoid shard went 37.0 -> 36.1 ms.
static const int g_wide_splits = [] {
  const char *v = getenv("PPO_WIDE_SPLITS");
  const int n = v ? atoi(v) : kWideSplits / 2;
  return n < 1 ? 1 : (n > kWideSplits ? kWideSplits : n);
}();
constexpr int kWideHeadSplits = 64;  // ... of the heads (few output tiles)
static const int g_wide_enabled = [] {
  const char *v = getenv("PPO_WIDE");
  return v ? atoi(v) : 1;
}();
static bool wide_fused_rollout_enabled() {  // PPO_WIDE_FUSED_ROLLOUT=0 at context creation:
  const char *v = getenv("PPO_WIDE_FUSED_ROLLOUT");  // the layered rollout GEMMs (parity tests)
  return v ? atoi(v) != 0 : true;
}
constexpr int kFMaxW = 512;  // widest layer (and input row) of the fused rollout kernel

bool wide_shapes_ok(const ppo_ctx *ctx) {
  if (!g_wide_enabled || ctx->fused_ok) return false;
  if (ctx->cfg.activation != PPO_ACT_RELU || ctx->cfg.act_dim > 32) return false;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    for (int l = 0; l < nd.n_hidden; ++l)
      if (nd.layer[l].out % 8 != 0) return false;
  }
  return true;
}

bool wide_active(const ppo_ctx *ctx) {
  return ctx->wide != nullptr && ctx->prec == PPO_PREC_BF16 && wide_shapes_ok(ctx);
}

int wide_alloc(ppo_ctx *ctx) {
  if (ctx->wide || !wide_shapes_ok(ctx)) return 0;
  WideWork *w = new (std::nothrow) WideWork();
  PPO_REQUIRE(w != nullptr, "wide_alloc: out of host memory");
  const int64_t R = rup(ctx->cfg.max_rows, 256);
  w->rpad = static_cast<int>(R);
  const int din = ctx->cfg.obs_dim * ctx->cfg.window;
  w->ldx = static_cast<int>(rup(din, 128));  // whole 8-k-step groups for the fused rollout
  const int blocks = static_cast<int>(R / kWideLossRows);
  // carve-out in bytes; every buffer 256-B aligned, 1 KB of slack after each (tile reads past a
  // row end stay inside the allocation)
  int64_t bytes = 0;
  auto take = [&](int64_t b) {
    const int64_t o = bytes;
    bytes += rup(b, 256) + 1024;
    return o;
  };
  struct Off {
    int64_t h[PPO_MAX_LAYERS], dh[PPO_MAX_LAYERS], w[PPO_MAX_LAYERS + 1], wt[PPO_MAX_LAYERS + 1],
        cs[PPO_MAX_LAYERS];
    int64_t dz, z;
  } off[2];
  const int64_t ox = take(R * w->ldx * 2);
  int64_t img0 = -1, img_bytes = 0;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    WideNetWork &wn = w->net[z];
    for (int l = 0; l < nd.n_hidden; ++l) {
      wn.ldh[l] = static_cast<int>(rup(nd.layer[l].out, 64));
      off[z].h[l] = take(R * wn.ldh[l] * 2);
      off[z].dh[l] = take(R * wn.ldh[l] * 2);
      off[z].cs[l] = take((R / 64) * nd.layer[l].out * 4);
    }
    off[z].dz = take(R * 64 * 2);
    off[z].z = take(R * 32 * 4);
  }
  // weight images last and contiguous, so the pack kernel zero-fills them as one range
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    WideNetWork &wn = w->net[z];
    for (int l = 0; l <= nd.n_hidden; ++l) {
      const LayerDesc &L = nd.layer[l];
      wn.ldw[l] = static_cast<int>(rup(L.in, 64));
      wn.ldwt[l] = static_cast<int>(rup(L.out, 64));
      const int64_t a = rup(rup(L.out, 128) * wn.ldw[l] * 2, 256);
      const int64_t b = rup(rup(L.in, 128) * wn.ldwt[l] * 2, 256);
      off[z].w[l] = bytes;
      bytes += a;
      off[z].wt[l] = bytes;
      bytes += b;
      if (img0 < 0) img0 = off[z].w[l];
      img_bytes = bytes - img0;
    }
  }
  bytes += 1024;
  // fused rollout: every hidden width a multiple of 128 and at most kFMaxW, the input row too,
  // the actor head at most 32 wide
  bool fr = w->ldx <= kFMaxW && ctx->cfg.act_dim <= 32;
  for (int z = 0; z < 2; ++z)
    for (int l = 0; l < ctx->net[z].n_hidden; ++l)
      fr = fr && ctx->net[z].layer[l].out % 128 == 0 && ctx->net[z].layer[l].out <= kFMaxW;
  w->fused_rollout = fr && wide_fused_rollout_enabled();
  int64_t off_wf[2][PPO_MAX_LAYERS + 1] = {};
  if (w->fused_rollout)
    for (int z = 0; z < 2; ++z) {
      const NetDesc &nd = ctx->net[z];
      WideNetWork &wn = w->net[z];
      for (int l = 0; l <= nd.n_hidden; ++l) {
        const LayerDesc &L = nd.layer[l];
        wn.wf_tiles[l] = static_cast<int>(rup(L.out, 32) / 32);
        wn.wf_ks[l] = static_cast<int>(rup(L.in, 128) / 16);
        off_wf[z][l] = take(static_cast<int64_t>(wn.wf_tiles[l]) * wn.wf_ks[l] * 512 * 2);
      }
    }
  const int64_t opart = take(static_cast<int64_t>(blocks) * kWidePart * 4);
  const int64_t oloss = take(static_cast<int64_t>(blocks) * 2 * 4);
  void *arena = nullptr;
  hipError_t e = hipMalloc(&arena, bytes);
  if (e != hipSuccess) {
    delete w;
    set_error("wide_alloc: hipMalloc(%lld bytes) failed: %s", static_cast<long long>(bytes),
              hipGetErrorString(e));
    return PPO_EHIP;
  }
  e = hipMemset(arena, 0, bytes);  // pad rows / columns of every operand stay zero
  if (e != hipSuccess) {
    (void)hipFree(arena);
    delete w;
    set_error("wide_alloc: hipMemset failed: %s", hipGetErrorString(e));
    return PPO_EHIP;
  }
  char *base = static_cast<char *>(arena);
  w->arena = arena;
  w->x = reinterpret_cast<__bf16 *>(base + ox);
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    WideNetWork &wn = w->net[z];
    for (int l = 0; l < nd.n_hidden; ++l) {
      wn.h[l] = reinterpret_cast<__bf16 *>(base + off[z].h[l]);
      wn.dh[l] = reinterpret_cast<__bf16 *>(base + off[z].dh[l]);
      wn.colsum[l] = reinterpret_cast<float *>(base + off[z].cs[l]);
    }
    for (int l = 0; l <= nd.n_hidden; ++l) {
      wn.w[l] = reinterpret_cast<__bf16 *>(base + off[z].w[l]);
      wn.wt[l] = reinterpret_cast<__bf16 *>(base + off[z].wt[l]);
    }
    wn.dz = reinterpret_cast<__bf16 *>(base + off[z].dz);
    wn.z = reinterpret_cast<float *>(base + off[z].z);
    for (int l = 0; l <= nd.n_hidden; ++l)
      wn.wf[l] = w->fused_rollout ? reinterpret_cast<__bf16 *>(base + off_wf[z][l]) : nullptr;
  }
  w->part = reinterpret_cast<float *>(base + opart);
  w->loss_part = reinterpret_cast<float *>(base + oloss);
  w->img_elems = img_bytes / 2;
  ctx->wide = w;
  return 0;
}

void wide_free(ppo_ctx *ctx) {
  if (!ctx->wide) return;
  if (ctx->wide->arena) (void)hipFree(ctx->wide->arena);
  delete ctx->wide;
  ctx->wide = nullptr;
}

// ============================================================================================
// Row staging: x[j][0:ldx] = bf16(states[rows ? rows[j] : j][0:din]) for j < count, zero rows
// for count <= j < rows_pad (the padding contract of wide_gemm.h).
// ============================================================================================
struct GatherArgs {
  const float *states;
  const int32_t *rows, *rows_n;
  int n, rows_pad, din, ldx;
  __bf16 *x;
};

__device__ __forceinline__ void gather_block(const GatherArgs &g, int blk) {
  const float *__restrict__ states = g.states;
  const int32_t *__restrict__ rows = g.rows;
  const int din = g.din, ldx = g.ldx, rows_pad = g.rows_pad;
  __bf16 *__restrict__ x = g.x;
  const int count = g.rows_n ? *g.rows_n : g.n;
  const int per_row = ldx / 8;
  const int64_t i = static_cast<int64_t>(blk) * 256 + threadIdx.x;
  if (i >= static_cast<int64_t>(rows_pad) * per_row) return;
  const int j = static_cast<int>(i / per_row), c0 = static_cast<int>(i % per_row) * 8;
  const bool live = j < count;
  const int64_t sr = rows ? rows[live ? j : 0] : j;
  const float *src = states + (live ? sr : 0) * din;
  float v[8];
  if ((din & 3) == 0 && (reinterpret_cast<uintptr_t>(states) & 15) == 0) {
    // two 16-B loads from clamped addresses (din % 4 == 0: a 4-group is wholly in or out)
    const bool in0 = live && c0 < din, in1 = live && c0 + 4 < din;
    const float4 x0 = *reinterpret_cast<const float4 *>(src + (in0 ? c0 : 0));
    const float4 x1 = *reinterpret_cast<const float4 *>(src + (in1 ? c0 + 4 : 0));
    v[0] = in0 ? x0.x : 0.f, v[1] = in0 ? x0.y : 0.f, v[2] = in0 ? x0.z : 0.f, v[3] = in0 ? x0.w : 0.f;
    v[4] = in1 ? x1.x : 0.f, v[5] = in1 ? x1.y : 0.f, v[6] = in1 ? x1.z : 0.f, v[7] = in1 ? x1.w : 0.f;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool in = live && c0 + e < din;
      const float u = src[in ? c0 + e : 0];
      v[e] = in ? u : 0.f;
    }
  }
  *reinterpret_cast<uint4 *>(x + static_cast<int64_t>(j) * ldx + c0) =
      make_uint4(wide::pack2(v[0], v[1]), wide::pack2(v[2], v[3]), wide::pack2(v[4], v[5]),
                 wide::pack2(v[6], v[7]));
}

__global__ __launch_bounds__(256) void wide_gather_kernel(GatherArgs g) { gather_block(g, blockIdx.x); }

static GatherArgs gather_args(ppo_ctx *ctx, const float *states, const int32_t *rows,
                              const int32_t *count_d, int n, int rows_pad) {
  WideWork &W = *ctx->wide;
  GatherArgs g{};
  g.states = states;
  g.rows = rows;
  g.rows_n = count_d;
  g.n = n;
  g.rows_pad = rows_pad;
  g.din = ctx->cfg.obs_dim * ctx->cfg.window;
  g.ldx = W.ldx;
  g.x = W.x;
  return g;
}
static int gather_blocks(const GatherArgs &g) {
  return static_cast<int>(ceil_div(static_cast<int64_t>(g.rows_pad) * (g.ldx / 8), 256));
}
static double gather_bytes(const GatherArgs &g) {
  return static_cast<double>(g.n) * g.din * 4.0 + static_cast<double>(g.rows_pad) * g.ldx * 2.0;
}

static int stage_rows(ppo_ctx *ctx, const float *states, const int32_t *rows,
                      const int32_t *count_d, int n, int rows_pad, hipStream_t st) {
  const GatherArgs g = gather_args(ctx, states, rows, count_d, n, rows_pad);
  launch_k(TimRec{KC_GATHER, "wide_gather_kernel", 0.0, gather_bytes(g)}, wide_gather_kernel,
           dim3(gather_blocks(g)), dim3(256), 0, st, g);
  PPO_LAUNCHED();
  return 0;
}

// ============================================================================================
// Weight images: dst[r][c] = bf16(W[r][c]) (or W^T), zero outside the tensor.  One 64 x 64 tile
// of one image per block: the f32 master tile is read row-coalesced (64 consecutive `in` columns
// per wave row) into LDS, then every thread writes 8 consecutive image columns as one 16-B store,
// so the transposed images are written from the same coalesced reads as the plain ones.
// ============================================================================================
constexpr int kMaxImages = 2 * 2 * (PPO_MAX_LAYERS + 1);
constexpr int kPackT = 64;
struct ImageDesc {
  const float *w;   // [out][in] f32 master
  __bf16 *dst;
  int out, in;      // tensor shape
  int rows, cols;   // image shape (multiples of 64)
  int transposed;   // dst = W^T
  int blocks;       // first block of this image (prefix over images)
};
struct PackArgs {
  ImageDesc img[kMaxImages];
  int n;
};

__device__ __forceinline__ void pack_tile(const PackArgs &q, int blk) {
  __shared__ float tile[kPackT][kPackT + 1];
  int i = 0;
  while (i + 1 < q.n && q.img[i + 1].blocks <= blk) ++i;
  const ImageDesc d = q.img[i];
  const int t = blk - d.blocks;
  const int tiles_c = d.cols / kPackT;
  const int r0 = (t / tiles_c) * kPackT, c0 = (t % tiles_c) * kPackT;  // image tile origin
  // master tile: rows o0.. (out), columns i0.. (in); image (r, c) = master (r, c) or (c, r)
  const int o0 = d.transposed ? c0 : r0, i0 = d.transposed ? r0 : c0;
  const int tid = threadIdx.x;
  // 16 rows x 64 columns per pass, a float4 per thread (clamped address, masked values: no load
  // behind a branch); the masters' rows are 16-B aligned when d.in % 4 == 0
  const bool vec = d.in % 4 == 0 && reinterpret_cast<uintptr_t>(d.w) % 16 == 0;
  const int cg = 4 * (tid & 15);
#pragma unroll
  for (int k = 0; k < kPackT / 16; ++k) {
    const int lo = 16 * k + (tid >> 4);
    const int o = o0 + lo, in = i0 + cg;
    float v[4];
    if (vec) {
      const bool ok = o < d.out && in < d.in;  // d.in % 4 == 0: the whole float4 is in
      const float4 u = *reinterpret_cast<const float4 *>(d.w + static_cast<int64_t>(ok ? o : 0) * d.in + (ok ? in : 0));
      v[0] = ok ? u.x : 0.f, v[1] = ok ? u.y : 0.f, v[2] = ok ? u.z : 0.f, v[3] = ok ? u.w : 0.f;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = o < d.out && in + e < d.in;
        const float u = d.w[static_cast<int64_t>(ok ? o : 0) * d.in + (ok ? in + e : 0)];
        v[e] = ok ? u : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (d.transposed) tile[cg + e][lo] = v[e];  // tile[image row][image col]
      else tile[lo][cg + e] = v[e];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int item = k * 256 + tid, lr = item >> 3, cg = item & 7;
    const float *s = &tile[lr][8 * cg];
    *reinterpret_cast<uint4 *>(d.dst + static_cast<int64_t>(r0 + lr) * d.cols + c0 + 8 * cg) =
        make_uint4(wide::pack2(s[0], s[1]), wide::pack2(s[2], s[3]), wide::pack2(s[4], s[5]),
                   wide::pack2(s[6], s[7]));
  }
}

// Fragment-major image of one layer: element j of lane `lane` in the block of (k-step ks, tile ot)
// holds W[32 ot + (lane & 31)][16 ks + 8 (lane >> 5) + j] (zero outside the tensor); one thread
// writes one lane's 16-B fragment from 8 consecutive master elements.
struct FragDesc {
  const float *w;
  __bf16 *dst;
  int out, in, tiles, ks;
  int blocks;  // first block of this image
};
struct FragArgs {
  FragDesc img[2 * (PPO_MAX_LAYERS + 1)];
  int n;
};

__device__ __forceinline__ void pack_frag(const FragArgs &q, int b) {
  int i = 0;
  while (i + 1 < q.n && q.img[i + 1].blocks <= b) ++i;
  const FragDesc d = q.img[i];
  const int64_t f = static_cast<int64_t>(b - d.blocks) * 256 + threadIdx.x;  // fragment
  if (f >= static_cast<int64_t>(d.tiles) * d.ks * 64) return;
  const int lane = static_cast<int>(f & 63);
  const int blk = static_cast<int>(f >> 6), ks = blk / d.tiles, ot = blk - ks * d.tiles;
  const int o = 32 * ot + (lane & 31), i0 = 16 * ks + 8 * (lane >> 5);
  float v[8];
  if (d.in % 4 == 0 && reinterpret_cast<uintptr_t>(d.w) % 16 == 0) {
    // two float4 loads (d.in % 4 == 0: a 4-group is wholly inside or outside the row)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const bool ok = o < d.out && i0 + 4 * h2 < d.in;
      const float4 u = *reinterpret_cast<const float4 *>(d.w + (ok ? static_cast<int64_t>(o) * d.in + i0 + 4 * h2 : 0));
      v[4 * h2] = ok ? u.x : 0.f, v[4 * h2 + 1] = ok ? u.y : 0.f;
      v[4 * h2 + 2] = ok ? u.z : 0.f, v[4 * h2 + 3] = ok ? u.w : 0.f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = o < d.out && i0 + j < d.in;
      const float u = d.w[ok ? static_cast<int64_t>(o) * d.in + i0 + j : 0];
      v[j] = ok ? u : 0.f;
    }
  }
  reinterpret_cast<uint4 *>(d.dst)[f] =
      make_uint4(wide::pack2(v[0], v[1]), wide::pack2(v[2], v[3]), wide::pack2(v[4], v[5]),
                 wide::pack2(v[6], v[7]));
}

// One launch for every image an optimizer step refreshes: blocks [0, frag_blocks) the
// fragment-major images (fused forward / rollout), the rest the 64x64 tiles of the W^T (and, for
// the layered forward, W) images.
// A minibatch step's prep (wide_minibatch_grad) adds the row gather as the last blocks, so the
// weight refresh and the row staging -- independent work -- are one launch.
struct PrepGather {
  GatherArgs g;
  int first;  // first gather block (blocks before it pack), gridDim.x when there is none
};
__global__ __launch_bounds__(256) void wide_pack_kernel(PackArgs q, FragArgs fq, int frag_blocks,
                                                        PrepGather pg) {
  const int b = static_cast<int>(blockIdx.x);
  if (b >= pg.first) gather_block(pg.g, b - pg.first);
  else if (b < frag_blocks) pack_frag(fq, b);
  else pack_tile(q, b - frag_blocks);
}

// the fragment-major images' descriptors (blocks counted from 0)
static int frag_args(ppo_ctx *ctx, FragArgs &q, double &elems) {
  WideWork &W = *ctx->wide;
  int blocks = 0;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    const WideNetWork &wn = W.net[z];
    for (int l = 0; l <= nd.n_hidden; ++l) {
      FragDesc &d = q.img[q.n++];
      d.w = ctx->params + nd.layer[l].w_off;
      d.dst = wn.wf[l];
      d.out = nd.layer[l].out;
      d.in = nd.layer[l].in;
      d.tiles = wn.wf_tiles[l];
      d.ks = wn.wf_ks[l];
      d.blocks = blocks;
      blocks += static_cast<int>(ceil_div(static_cast<int64_t>(d.tiles) * d.ks * 64, 256));
      elems += static_cast<double>(d.out) * d.in;
    }
  }
  return blocks;
}

// gather (nullable): the minibatch rows to stage in the same launch
int wide_pack(ppo_ctx *ctx, hipStream_t st, bool frag, const GatherArgs *gather) {
  WideWork &W = *ctx->wide;
  FragArgs fq{};
  double elems = 0;
  const int frag_blocks = (frag && W.fused_rollout) ? frag_args(ctx, fq, elems) : 0;
  PackArgs q{};
  int blocks = 0;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    const WideNetWork &wn = W.net[z];
    for (int l = 0; l <= nd.n_hidden; ++l) {
      const LayerDesc &L = nd.layer[l];
      for (int t = 0; t < 2; ++t) {
        // only the images a minibatch step or rollout reads: W^T feeds DGRAD, which layer 0 has
        // none of; W feeds the layered forward, which the fused kernels (fragment-major images)
        // replace
        if ((t == 1 && l == 0) || (t == 0 && W.fused_rollout)) continue;
        ImageDesc &d = q.img[q.n++];
        d.w = ctx->params + L.w_off;
        d.out = L.out;
        d.in = L.in;
        d.transposed = t;
        d.dst = t ? wn.wt[l] : wn.w[l];
        d.rows = static_cast<int>(t ? rup(L.in, 128) : rup(L.out, 128));
        d.cols = t ? wn.ldwt[l] : wn.ldw[l];
        d.blocks = blocks;
        blocks += (d.rows / kPackT) * (d.cols / kPackT);
        elems += static_cast<double>(d.out) * d.in;
      }
    }
  }
  PrepGather pg{};
  pg.first = frag_blocks + blocks;
  int gblocks = 0;
  if (gather) {
    pg.g = *gather;
    gblocks = gather_blocks(*gather);
  }
  launch_k(TimRec{KC_GATHER, "wide_pack_kernel", 0.0,
                  elems * (4.0 + 2.0) + (gather ? gather_bytes(*gather) : 0.0)},
           wide_pack_kernel, dim3(frag_blocks + blocks + gblocks), dim3(256), 0, st, q, fq,
           frag_blocks, pg);
  PPO_LAUNCHED();
  return 0;
}


// ============================================================================================
// Forward through the hidden layers and the head pre-activations (both nets per launch)
// ============================================================================================
static int forward(ppo_ctx *ctx, const bool use[2], int rows_pad, const int32_t *count_d,
                   hipStream_t st) {
  WideWork &W = *ctx->wide;
  const int max_l = std::max(use[0] ? ctx->net[0].n_hidden : 0, use[1] ? ctx->net[1].n_hidden : 0);
  for (int l = 0; l < max_l; ++l) {
    WideBatch wb{};
    wb.rows_n = count_d;
    wb.act = ctx->cfg.activation;
    int np = 0, max_n = 0;
    for (int z = 0; z < 2; ++z) {
      const NetDesc &nd = ctx->net[z];
      if (!use[z] || l >= nd.n_hidden) continue;
      const LayerDesc &L = nd.layer[l];
      const WideNetWork &wn = W.net[z];
      WideProblem &P = wb.p[np++];
      P.a = l == 0 ? W.x : wn.h[l - 1];
      P.lda = l == 0 ? W.ldx : wn.ldh[l - 1];
      P.b = wn.w[l];
      P.ldb = wn.ldw[l];
      P.c = wn.h[l];
      P.ldc = wn.ldh[l];
      P.bias = L.b_off >= 0 ? ctx->params + L.b_off : nullptr;
      P.m = rows_pad;
      P.n = L.out;
      P.k = wn.ldw[l];
      max_n = std::max(max_n, L.out);
    }
    if (np)
      if (int rc = wide::run(wide::WK_FWD, wb, np, rows_pad, max_n, 0, st)) return rc;
  }
  WideBatch wb{};
  wb.rows_n = count_d;
  int np = 0;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    if (!use[z]) continue;
    const int L = nd.n_hidden;
    const WideNetWork &wn = W.net[z];
    WideProblem &P = wb.p[np++];
    P.a = wn.h[L - 1];
    P.lda = wn.ldh[L - 1];
    P.b = wn.w[L];
    P.ldb = wn.ldw[L];
    P.c = wn.z;
    P.ldc = 32;
    P.m = rows_pad;
    P.n = 32;
    P.k = wn.ldw[L];
  }
  return wide::run(wide::WK_F32, wb, np, rows_pad, 32, 0, st);
}

// ============================================================================================
// Rollout head: sampling + log-prob + value from the head pre-activations (policy_head_kernel's
// formulas, ppo_agent.py:27-43 and ppo.py:23-26): one thread per row, actions in order.
// ============================================================================================
struct WidePolicyArgs {
  const float *za, *zc;  // [rows][32] head pre-activations (nullable per net)
  int n, act_dim;
  const float *ba, *logstd, *bc;
  float omv;
  const float *eps;
  uint64_t seed, offset;
  const uint64_t *offset_base;
  float *action, *logp, *value, *mean;
};

// 32 lanes per row (A <= 32): lane a samples action a; the row's log-prob is summed in action
// order by the row's first lane (the sequential order of policy_head_kernel).
__global__ __launch_bounds__(256) void wide_policy_head_kernel(WidePolicyArgs q) {
  const int lane = threadIdx.x & 63, a = lane & 31;
  const int j = blockIdx.x * 8 + (threadIdx.x >> 5);
  const bool row_ok = j < q.n;  // uniform per 32-lane half; both halves take every shuffle
  if (q.za) {
    float lp = 0.f;
    if (row_ok && a < q.act_dim) {
      const float zr = q.za[static_cast<int64_t>(j) * 32 + a];
      const float z = q.ba ? zr + q.ba[a] : zr;
      const float mu = q.omv * tanhf(z);
      const float sd = expf(q.logstd[a]);
      const int64_t idx = static_cast<int64_t>(j) * q.act_dim + a;
      const uint64_t base = q.offset + (q.offset_base ? *q.offset_base : 0);
      const float e = q.eps ? q.eps[idx] : philox_normal_at(q.seed, base + idx);
      const float x = e * sd + mu;  // torch.normal: randn*std then + mean (two roundings)
      if (q.action) q.action[idx] = x;
      if (q.mean) q.mean[idx] = mu;
      const float d = x - mu;
      const float var = sd * sd;
      lp = ((-(d * d)) / (2.f * var) - logf(sd)) - kLogSqrt2Pi;
    }
    // the row's log-prob in action order (policy_head_kernel's sequential sum); a fixed trip
    // count so the 32 cross-lane reads issue back to back instead of one round trip per action
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const float v = __shfl(lp, (lane & 32) + k, 64);
      if (k < q.act_dim) s += v;
    }
    if (row_ok && a == 0 && q.logp) q.logp[j] = s;
  }
  if (row_ok && a == 0 && q.zc && q.value) {
    const float v = q.zc[static_cast<int64_t>(j) * 32];
    q.value[j] = q.bc ? v + q.bc[0] : v;
  }
}

// ============================================================================================
// Rollout observation step of the wide path, one launch (A1): the window push (helper.py:51-64,
// running_gym_sequential_vectorized.py:53-58), the per-(slot, slice) f64 standardisation
// (running_gym_sequential_vectorized.py:61-92) and the bf16 GEMM operand row x[env] -- three
// launches (ppo_obs_window_push, ppo_obs_normalize, the row staging) before.  One wave per env:
// every global load of the row (new observation, kept window slots) is issued up front from
// clamped addresses; the row is then standardised from an LDS copy in obs_normalize_wide_kernel's
// exact summation order (lane-strided partials over the slice, fixed xor tree), so the state is
// bitwise that kernel's.  Waves of rows in [n, rows_pad) write the zero operand rows of the
// padding contract (wide_gemm.h).
// ============================================================================================
constexpr int kObsMaxK = 8;       // W*O <= 64 * kObsMaxK elements per row
constexpr int kObsMaxSlices = 8;  // standardisation slices (Humanoid-v4: 6)
struct WideObserveArgs {
  double *window;        // (N, O, W) f64, updated in place when obs != null
  const double *obs;     // (N, O) f64 new observations, nullable (no push)
  const uint8_t *reset;  // nullable
  int all_reset;
  int n, rows_pad, o, w;
  PolicySlices tab;
  int normalize;
  float *state;          // (N, W*O) f32
  __bf16 *x;             // [rows_pad][ldx] bf16
  int ldx;
};

__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

__global__ __launch_bounds__(256) void wide_observe_kernel(WideObserveArgs q) {
  __shared__ double rowbuf[4][64 * kObsMaxK];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int env = blockIdx.x * 4 + wv;  // wave-uniform
  if (env >= q.rows_pad) return;
  const int o = q.o, w = q.w, ow = o * w;
  if (env >= q.n) {  // padding row: zero operand
    for (int c = 8 * lane; c < q.ldx; c += 512)
      *reinterpret_cast<uint4 *>(q.x + static_cast<int64_t>(env) * q.ldx + c) = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  double *win = rowbuf[wv];
  double *const grow = q.window + static_cast<int64_t>(env) * ow;
  // ---- every load of the row first: kept slots (element e + 1 of the old row) and the obs ----
  double old[kObsMaxK], ob[kObsMaxK];
  const bool push = q.obs != nullptr;
  const bool full = q.all_reset || (q.reset && q.reset[env]);
#pragma unroll
  for (int k = 0; k < kObsMaxK; ++k) {
    const int e = lane + 64 * k;            // element (f = e / w, slot = e % w)
    const int f = e / w, slot = e - f * w;
    const bool in = e < ow;
    const bool keep = in && !(push && (full || slot == w - 1));
    old[k] = grow[keep ? (push ? e + 1 : e) : 0];
    ob[k] = push ? q.obs[static_cast<int64_t>(env) * o + (in ? f : 0)] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < kObsMaxK; ++k) {
    const int e = lane + 64 * k;
    if (e < ow) {
      const int f = e / w, slot = e - f * w;
      const bool take_obs = push && (full || slot == w - 1);
      const double v = take_obs ? ob[k] : old[k];
      win[e] = v;
      if (push) grow[e] = v;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS row is complete
  __builtin_amdgcn_wave_barrier();
  float *const srow = q.state + static_cast<int64_t>(env) * ow;
  __bf16 *const xrow = q.x + static_cast<int64_t>(env) * q.ldx;
  // state (N, W, O): slot-major; x is the same row as bf16, zero past W*O
  for (int slot = 0; slot < w; ++slot) {
    const double *src = win + slot;  // feature f at f * w
    float *dst = srow + static_cast<int64_t>(slot) * o;
    __bf16 *xd = xrow + slot * o;
    if (!q.normalize) {
      for (int f = lane; f < o; f += 64) {
        const float v = static_cast<float>(src[f * w]);
        dst[f] = v;
        xd[f] = static_cast<__bf16>(v);
      }
      continue;
    }
    // the slices' statistics side by side: each pass's partials for every slice, then their
    // xor trees interleaved (independent shuffle chains) -- per slice the same operations in the
    // same order as obs_normalize_wide_kernel, so bitwise its state
    double mean[kObsMaxSlices], cmean[kObsMaxSlices], sd[kObsMaxSlices], acc[kObsMaxSlices];
#pragma unroll
    for (int sl = 0; sl < kObsMaxSlices; ++sl) {
      acc[sl] = 0.0;
      if (sl < q.tab.count)
        for (int f = q.tab.edge[sl] + lane; f < q.tab.edge[sl + 1]; f += 64) acc[sl] += src[f * w];
    }
#pragma unroll
    for (int sl = 0; sl < kObsMaxSlices; ++sl)
      mean[sl] = wave_sum64(acc[sl]) / (q.tab.edge[sl + 1] - q.tab.edge[sl]);
#pragma unroll
    for (int sl = 0; sl < kObsMaxSlices; ++sl) {
      acc[sl] = 0.0;
      if (sl < q.tab.count)
        for (int f = q.tab.edge[sl] + lane; f < q.tab.edge[sl + 1]; f += 64) acc[sl] += src[f * w] - mean[sl];
    }
#pragma unroll
    for (int sl = 0; sl < kObsMaxSlices; ++sl)
      cmean[sl] = wave_sum64(acc[sl]) / (q.tab.edge[sl + 1] - q.tab.edge[sl]);
#pragma unroll
    for (int sl = 0; sl < kObsMaxSlices; ++sl) {
      acc[sl] = 0.0;
      if (sl < q.tab.count)
        for (int f = q.tab.edge[sl] + lane; f < q.tab.edge[sl + 1]; f += 64) {
          const double d = (src[f * w] - mean[sl]) - cmean[sl];
          acc[sl] += d * d;
        }
    }
#pragma unroll
    for (int sl = 0; sl < kObsMaxSlices; ++sl) {
      // cnt == 1 -> NaN, as torch.std
      sd[sl] = sqrt(wave_sum64(acc[sl]) / (q.tab.edge[sl + 1] - q.tab.edge[sl] - 1));
      if (sd[sl] == 0.0) sd[sl] = 1.0;
    }
#pragma unroll
    for (int sl = 0; sl < kObsMaxSlices; ++sl) {
      if (sl >= q.tab.count) continue;
      for (int f = q.tab.edge[sl] + lane; f < q.tab.edge[sl + 1]; f += 64) {
        const float v = static_cast<float>((src[f * w] - mean[sl]) / sd[sl]);
        dst[f] = v;
        xd[f] = static_cast<__bf16>(v);
      }
    }
  }
  for (int c = ow + lane; c < q.ldx; c += 64) xrow[c] = static_cast<__bf16>(0.f);
}

int wide_observe(ppo_ctx *ctx, double *window_d, const double *obs_d, const uint8_t *reset_d,
                 int all_reset, const PolicySlices &tab, int normalize, float *state_d, int n,
                 hipStream_t st) {
  WideWork &W = *ctx->wide;
  const int o = ctx->cfg.obs_dim, w = ctx->cfg.window;
  PPO_REQUIRE(o * w <= 64 * kObsMaxK, "wide_observe: W*O = %d exceeds %d", o * w, 64 * kObsMaxK);
  PPO_REQUIRE(tab.count <= kObsMaxSlices, "wide_observe: %d slices (at most %d)", tab.count,
              kObsMaxSlices);
  WideObserveArgs q{};
  q.window = window_d;
  q.obs = obs_d;
  q.reset = reset_d;
  q.all_reset = all_reset;
  q.n = n;
  q.rows_pad = static_cast<int>(rup(n, 64));
  q.o = o;
  q.w = w;
  q.tab = tab;
  q.normalize = normalize;
  q.state = state_d;
  q.x = W.x;
  q.ldx = W.ldx;
  const double by = static_cast<double>(n) * o * w * (8.0 * (obs_d ? 2 : 1) + 4.0 + 2.0) +
                    (obs_d ? 8.0 * n * o : 0.0);
  launch_k(TimRec{KC_OBS, "wide_observe_kernel", 0.0, by}, wide_observe_kernel,
           dim3(ceil_div(q.rows_pad, 4)), dim3(256), 0, st, q);
  PPO_LAUNCHED();
  return 0;
}

bool wide_observe_ok(const ppo_ctx *ctx, int n_slices) {
  return ctx->cfg.obs_dim * ctx->cfg.window <= 64 * kObsMaxK && n_slices <= kObsMaxSlices;
}

// ============================================================================================
// Fused rollout policy step of the wide path (A2-A4 in one launch per step): both nets' hidden
// layers, heads, sampling and log-prob for 32 rollout rows per workgroup -- five launches of the
// layered rollout (three FWD GEMMs, the head GEMM, wide_policy_head_kernel) before.
//
// grid (rows_pad / 32, 2 nets), 8 waves.  The 32 rows' activations stay in LDS (two ping-pong
// [32][512] bf16 images, 16-B chunk c of row r at c ^ (r & 15): the B-operand row reads are
// conflict-free); each layer's weights stream from L2 as 32x32x16 A fragments of the
// fragment-major image (one 1 KB block per (k-step, 32-feature tile)), two 8-k-step groups in
// flight per wave.  Wave w owns the output features 64w..64w+63 (two tiles): C = W . act^T, so a
// lane holds one row's 4-feature runs and writes them as 8-B image stores.  Bias + ReLU in f32,
// the stored activation rounded to bf16 (the layered FWD epilogue).  The head (at most 32
// outputs) runs on wave 0 in the same k order as the head GEMM; then one thread per (row, action
// pair) applies wide_policy_head_kernel's formulas and the row's log-prob is summed in action order.
// ============================================================================================
constexpr int kFRows = 32;
constexpr int kFPitch = kFMaxW * 2;  // bytes per LDS image row
constexpr int kFGroup = 8;           // k-steps per fragment group

struct WideFusedNet {
  const __bf16 *wf[PPO_MAX_LAYERS + 1];
  const float *b[PPO_MAX_LAYERS + 1];
  int tiles[PPO_MAX_LAYERS + 1], ks[PPO_MAX_LAYERS + 1];
  int n_hidden;
};
struct WideFusedArgs {
  WideFusedNet net[2];
  int use[2];
  const __bf16 *x;
  int ldx, n;
  int act_dim;
  float omv;
  const float *logstd;
  const float *eps;
  uint64_t seed, offset;
  const uint64_t *offset_base;
  float *action, *logp, *value, *mean;
};

__device__ __forceinline__ int fimg_off(int row, int chunk) {
  return row * kFPitch + ((chunk ^ (row & 15)) << 4);
}

// one group of kFGroup k-steps of a wave's fragments (tiles ot0, ot0 + 1; NT of them valid)
template <int NT>
__device__ __forceinline__ void frag_load(const __bf16 *wf, int tiles, int ot0, int g, int lane,
                                          wide::bf16x8 (&f)[kFGroup][2]) {
#pragma unroll
  for (int s = 0; s < kFGroup; ++s)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int64_t blk = static_cast<int64_t>(g * kFGroup + s) * tiles + ot0 + t;
      f[s][t] = *reinterpret_cast<const wide::bf16x8 *>(wf + (blk * 64 + lane) * 8);
    }
}

// acc[t][u] += W[tile ot0 + t] . img[rows 32u..32u+31]^T over the layer's k-steps
template <int NT, int RT>
__device__ __forceinline__ void fused_layer(const __bf16 *wf, int tiles, int ks, int ot0,
                                            const char *img, int lane,
                                            wide::f32x16 (&acc)[2][RT]) {
  const int ng = ks / kFGroup;
  const int row = lane & 31, h = lane >> 5;
  wide::bf16x8 cur[kFGroup][2], nxt[kFGroup][2];
  frag_load<NT>(wf, tiles, ot0, 0, lane, cur);
  for (int g = 0; g < ng; ++g) {
    // unconditional (the last group re-reads itself): a load behind the g + 1 < ng test would
    // make the compiler wait for it at the branch merge, exposing the L2 latency every group
    frag_load<NT>(wf, tiles, ot0, g + 1 < ng ? g + 1 : g, lane, nxt);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this group's MFMAs
#pragma unroll
    for (int s = 0; s < kFGroup; ++s) {
      const int k16 = g * kFGroup + s;
#pragma unroll
      for (int u = 0; u < RT; ++u) {
        const wide::bf16x8 bv =
            *reinterpret_cast<const wide::bf16x8 *>(img + fimg_off(32 * u + row, 2 * k16 + h));
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[s][t], bv, acc[t][u], 0, 0, 0);
      }
    }
#pragma unroll
    for (int s = 0; s < kFGroup; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) cur[s][t] = nxt[s][t];
  }
}

// One hidden layer of a fused workgroup over RT row tiles: wave w's feature tiles 2w, 2w + 1,
// bias + ReLU, bf16 4-feature runs into the dst image.
template <int RT>
__device__ __forceinline__ void fused_hidden(const WideFusedNet &N, int l, const char *src,
                                             char *dst, int w, int lane) {
  const int tiles = N.tiles[l];
  const int ot0 = 2 * w;
  wide::f32x16 acc[2][RT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < RT; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;
  if (ot0 + 1 < tiles) fused_layer<2, RT>(N.wf[l], tiles, N.ks[l], ot0, src, lane, acc);
  else if (ot0 < tiles) fused_layer<1, RT>(N.wf[l], tiles, N.ks[l], ot0, src, lane, acc);
  const int row = lane & 31;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (ot0 + t >= tiles) continue;  // uniform per wave
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int o = 32 * (ot0 + t) + 8 * g + 4 * (lane >> 5);
      const float4 bv = N.b[l] ? *reinterpret_cast<const float4 *>(N.b[l] + o) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < RT; ++u) {
        const float y0 = act_forward(acc[t][u][4 * g] + bv.x, PPO_ACT_RELU);
        const float y1 = act_forward(acc[t][u][4 * g + 1] + bv.y, PPO_ACT_RELU);
        const float y2 = act_forward(acc[t][u][4 * g + 2] + bv.z, PPO_ACT_RELU);
        const float y3 = act_forward(acc[t][u][4 * g + 3] + bv.w, PPO_ACT_RELU);
        *reinterpret_cast<uint2 *>(dst + fimg_off(32 * u + row, o >> 3) + 2 * (o & 7)) =
            make_uint2(wide::pack2(y0, y1), wide::pack2(y2, y3));
      }
    }
  }
}

__global__ __launch_bounds__(512) void wide_policy_fused_kernel(WideFusedArgs q) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kFRows * kFPitch];
  __shared__ float zt[kFRows][33];   // head outputs [row][output]
  __shared__ float lpt[kFRows][33];  // per-(row, action) log-prob terms
  // (row block, net) from the linear block id: with a multiple of 4 row blocks per net, the actor
  // runs on XCDs 0-3 and the critic on XCDs 4-7 (blocks b, b + 8, ... share an XCD), so each
  // XCD's L2 holds one net's weight images instead of both
  const int nb = (q.n + kFRows - 1) / kFRows, b = static_cast<int>(blockIdx.x);
  int z, rb;
  if (nb % 4 == 0) {
    const int x = b % 8;
    z = x / 4;
    rb = (x % 4) + 4 * (b / 8);
  } else {
    z = b / nb;
    rb = b % nb;
  }
  if (!q.use[z]) return;  // uniform per block
  const WideFusedNet &N = q.net[z];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = rb * kFRows;
  // ---- the rows' bf16 states (x, zero-padded to ldx) -> image 0 ----
  const int cpr = q.ldx / 8;
  for (int e = tid; e < kFRows * cpr; e += 512) {
    const int row = e / cpr, c = e - row * cpr;
    const uint4 v = *reinterpret_cast<const uint4 *>(q.x + static_cast<int64_t>(r0 + row) * q.ldx + 8 * c);
    *reinterpret_cast<uint4 *>(lds + fimg_off(row, c)) = v;
  }
  lds_sync();
  int cur = 0;
  for (int l = 0; l < N.n_hidden; ++l) {
    fused_hidden<1>(N, l, lds + cur * kFRows * kFPitch, lds + (cur ^ 1) * kFRows * kFPitch, w, lane);
    lds_sync();
    cur ^= 1;
  }
  // ---- head pre-activations (<= 32 outputs) on wave 0 ----
  const int L = N.n_hidden;
  if (w == 0) {
    wide::f32x16 acc[2][1];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][0][r] = 0.f;
    fused_layer<1, 1>(N.wf[L], N.tiles[L], N.ks[L], 0, lds + cur * kFRows * kFPitch, lane, acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) zt[lane & 31][(r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)] = acc[0][0][r];
  }
  lds_sync();
  const int row = tid >> 4, j = r0 + row;
  const bool row_ok = j < q.n;
  if (z == 0) {
    const int A = q.act_dim;
    const uint64_t base = q.offset + (q.offset_base ? *q.offset_base : 0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int a = (tid & 15) + 16 * u;
      float lp = 0.f;
      if (row_ok && a < A) {
        const float zr = zt[row][a];
        const float zz = N.b[L] ? zr + N.b[L][a] : zr;
        const float mu = q.omv * tanhf(zz);
        const float sd = expf(q.logstd[a]);
        const int64_t idx = static_cast<int64_t>(j) * A + a;
        const float e = q.eps ? q.eps[idx] : philox_normal_at(q.seed, base + idx);
        const float x = e * sd + mu;  // torch.normal: randn*std then + mean (two roundings)
        if (q.action) q.action[idx] = x;
        if (q.mean) q.mean[idx] = mu;
        const float d = x - mu;
        const float var = sd * sd;
        lp = ((-(d * d)) / (2.f * var) - logf(sd)) - kLogSqrt2Pi;
      }
      lpt[row][a] = lp;
    }
    lds_sync();
    if ((tid & 15) == 0 && row_ok && q.logp) {
      float s = 0.f;
      for (int a = 0; a < A; ++a) s += lpt[row][a];  // action order (policy_head_kernel)
      q.logp[j] = s;
    }
  } else if ((tid & 15) == 0 && row_ok && q.value) {
    const float v = zt[row][0];
    q.value[j] = N.b[L] ? v + N.b[L][0] : v;
  }
}

// Minibatch forward of the wide path in one launch per optimizer step (ppo.py:109-115): both
// nets' hidden layers and head pre-activations for 64 minibatch rows per workgroup, the activations
// kept in LDS between layers (each layer's input is read from LDS, not HBM) and each hidden output
// copied out once, as the backward's operand -- the three FWD GEMM launches and the head GEMM of
// the layered forward, whose layer inputs made a round trip through HBM.  Same per-layer arithmetic
// as the rollout kernel above; rows at or past the device row count are written as zeros (the
// padding contract of wide_gemm.h).
constexpr int kFwdRows = 64;
struct WideFwdArgs {
  WideFusedNet net[2];
  const __bf16 *x;
  int ldx, rows_pad, b;
  const int32_t *rows_n;
  __bf16 *h[2][PPO_MAX_LAYERS];
  int ldh[2][PPO_MAX_LAYERS];
  float *z[2];  // [rows][32]
};

__global__ __launch_bounds__(512) void wide_forward_fused_kernel(WideFwdArgs q) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kFwdRows * kFPitch];
  const int nb = q.rows_pad / kFwdRows, b = static_cast<int>(blockIdx.x);
  int z, rb;
  if (nb % 4 == 0) {  // actor on XCDs 0-3, critic on 4-7 (one net's weights per L2)
    const int x = b % 8;
    z = x / 4;
    rb = (x % 4) + 4 * (b / 8);
  } else {
    z = b / nb;
    rb = b % nb;
  }
  const WideFusedNet &N = q.net[z];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = rb * kFwdRows;
  const int count = q.rows_n ? *q.rows_n : q.b;
  const int cpr = q.ldx / 8;
  for (int e = tid; e < kFwdRows * cpr; e += 512) {
    const int row = e / cpr, c = e - row * cpr;
    const uint4 v = *reinterpret_cast<const uint4 *>(q.x + static_cast<int64_t>(r0 + row) * q.ldx + 8 * c);
    *reinterpret_cast<uint4 *>(lds + fimg_off(row, c)) = v;
  }
  lds_sync();
  int cur = 0;
  for (int l = 0; l < N.n_hidden; ++l) {
    char *dst = lds + (cur ^ 1) * kFwdRows * kFPitch;
    fused_hidden<2>(N, l, lds + cur * kFwdRows * kFPitch, dst, w, lane);
    lds_sync();
    // the layer's output rows out (16-B coalesced), zero past the device count
    const int width = 32 * N.tiles[l], cw = width / 8, ld = q.ldh[z][l];
    __bf16 *hout = q.h[z][l];
    for (int e = tid; e < kFwdRows * cw; e += 512) {
      const int row = e / cw, c = e - row * cw;
      const uint4 v = *reinterpret_cast<const uint4 *>(dst + fimg_off(row, c));
      *reinterpret_cast<uint4 *>(hout + static_cast<int64_t>(r0 + row) * ld + 8 * c) =
          r0 + row < count ? v : make_uint4(0u, 0u, 0u, 0u);
    }
    cur ^= 1;  // the next layer reads dst and writes the other image (nobody reads it now)
  }
  // head pre-activations: waves 0 and 1, one 32-row tile each, in the head GEMM's k order
  const int L = N.n_hidden;
  if (w < 2) {
    wide::f32x16 acc[2][1];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][0][r] = 0.f;
    fused_layer<1, 1>(N.wf[L], N.tiles[L], N.ks[L], 0,
                      lds + cur * kFwdRows * kFPitch + 32 * w * kFPitch, lane, acc);
    const int row = r0 + 32 * w + (lane & 31);
    const bool live = row < count;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int o = 8 * g + 4 * (lane >> 5);
      *reinterpret_cast<float4 *>(q.z[z] + static_cast<int64_t>(row) * 32 + o) =
          live ? make_float4(acc[0][0][4 * g], acc[0][0][4 * g + 1], acc[0][0][4 * g + 2], acc[0][0][4 * g + 3])
               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

static int wide_forward_fused(ppo_ctx *ctx, int rows_pad, int b, const int32_t *count_d,
                              hipStream_t st) {
  WideWork &W = *ctx->wide;
  WideFwdArgs q{};
  double flops = 0;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    const WideNetWork &wn = W.net[z];
    WideFusedNet &f = q.net[z];
    f.n_hidden = nd.n_hidden;
    for (int l = 0; l <= nd.n_hidden; ++l) {
      const LayerDesc &L = nd.layer[l];
      f.wf[l] = wn.wf[l];
      f.b[l] = L.b_off >= 0 ? ctx->params + L.b_off : nullptr;
      f.tiles[l] = wn.wf_tiles[l];
      f.ks[l] = wn.wf_ks[l];
      flops += 2.0 * rows_pad * L.out * L.in;
      if (l < nd.n_hidden) {
        q.h[z][l] = wn.h[l];
        q.ldh[z][l] = wn.ldh[l];
      }
    }
    q.z[z] = wn.z;
  }
  q.x = W.x;
  q.ldx = W.ldx;
  q.rows_pad = rows_pad;
  q.b = b;
  q.rows_n = count_d;
  launch_k(TimRec{KC_GEMM_FWD, "wide_forward_fused_kernel", flops, 0.0}, wide_forward_fused_kernel,
           dim3(2 * (rows_pad / kFwdRows)), dim3(512), 0, st, q);
  PPO_LAUNCHED();
  return 0;
}

static int wide_policy_fused(ppo_ctx *ctx, const bool use[2], int n, const float *eps_d,
                             uint64_t seed, uint64_t offset, float *action_d, float *logp_d,
                             float *value_d, float *mean_d, hipStream_t st) {
  WideWork &W = *ctx->wide;
  WideFusedArgs q{};
  double flops = 0;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    const WideNetWork &wn = W.net[z];
    WideFusedNet &f = q.net[z];
    q.use[z] = use[z];
    f.n_hidden = nd.n_hidden;
    for (int l = 0; l <= nd.n_hidden; ++l) {
      const LayerDesc &L = nd.layer[l];
      f.wf[l] = wn.wf[l];
      f.b[l] = L.b_off >= 0 ? ctx->params + L.b_off : nullptr;
      f.tiles[l] = wn.wf_tiles[l];
      f.ks[l] = wn.wf_ks[l];
      if (use[z]) flops += 2.0 * n * L.out * L.in;
    }
  }
  q.x = W.x;
  q.ldx = W.ldx;
  q.n = n;
  q.act_dim = ctx->cfg.act_dim;
  q.omv = ctx->cfg.output_max_value;
  q.logstd = ctx->params + ctx->net[0].logstd_off;
  q.eps = eps_d;
  q.seed = seed;
  q.offset = offset;
  q.offset_base = ctx->rng_counter;
  q.action = action_d;
  q.logp = logp_d;
  q.value = value_d;
  q.mean = mean_d;
  launch_k(TimRec{KC_POLICY_HEAD, "wide_policy_fused_kernel", flops, 0.0},
           wide_policy_fused_kernel, dim3(2 * ceil_div(n, kFRows)), dim3(512), 0, st, q);
  PPO_LAUNCHED();
  return 0;
}

int wide_policy_step(ppo_ctx *ctx, const float *state_d, int n, const float *eps_d, uint64_t seed,
                     uint64_t offset, float *action_d, float *logp_d, float *value_d,
                     float *mean_d, bool pack, hipStream_t st, bool staged) {
  WideWork &W = *ctx->wide;
  const bool use[2] = {action_d || logp_d || mean_d, value_d != nullptr};
  if (!use[0] && !use[1]) return 0;
  const int rows_pad = static_cast<int>(rup(n, 64));
  if (pack)
    if (int rc = wide_pack(ctx, st)) return rc;
  if (!staged)  // (wide_observe wrote x already)
    if (int rc = stage_rows(ctx, state_d, nullptr, nullptr, n, rows_pad, st)) return rc;
  if (W.fused_rollout)  // the images are current (pack above, or ppo_pack_weights)
    return wide_policy_fused(ctx, use, n, eps_d, seed, offset, action_d, logp_d, value_d, mean_d,
                             st);
  if (int rc = forward(ctx, use, rows_pad, nullptr, st)) return rc;
  const NetDesc &A = ctx->net[0], &C = ctx->net[1];
  WidePolicyArgs q{};
  q.n = n;
  q.act_dim = ctx->cfg.act_dim;
  q.omv = ctx->cfg.output_max_value;
  if (use[0]) {
    const LayerDesc &hl = A.layer[A.n_hidden];
    q.za = W.net[0].z;
    q.ba = hl.b_off >= 0 ? ctx->params + hl.b_off : nullptr;
    q.logstd = ctx->params + A.logstd_off;
  }
  if (use[1]) {
    q.zc = W.net[1].z;
    q.bc = ctx->params + C.layer[C.n_hidden].b_off;
  }
  q.eps = eps_d;
  q.seed = seed;
  q.offset = offset;
  q.offset_base = ctx->rng_counter;
  q.action = action_d;
  q.logp = logp_d;
  q.value = value_d;
  q.mean = mean_d;
  const int na = q.act_dim;
  launch_k(TimRec{KC_POLICY_HEAD, "wide_policy_head_kernel", 0.0,
                  4.0 * n * (32.0 * (use[0] + use[1]) + (eps_d ? na : 0) + (action_d ? na : 0) +
                             (mean_d ? na : 0) + 2.0)},
           wide_policy_head_kernel, dim3(ceil_div(n, 8)), dim3(256), 0, st, q);
  PPO_LAUNCHED();
  return 0;
}

// ============================================================================================
// Minibatch loss heads (update_head_kernel's formulas, ppo.py:109-135): one thread per row.
// dz rows (bf16, 64 columns, zero past the head width and for rows >= count), and per block the
// fixed-order sums of d loss / d logstd, the head-bias gradients (the f32 dz before rounding) and
// the two loss terms.
// ============================================================================================
struct WideLossArgs {
  const float *za, *zc;
  __bf16 *dza, *dzc;
  int act_dim;
  const float *ba, *logstd, *bc;
  float omv;
  const int32_t *rows;
  const int32_t *rows_n;
  int b;
  const float *actions, *old_logp, *adv, *vtarget;
  float clip_lo, clip_hi, ent_coef, inv_b, inv_ba;
  float *part, *loss_part;
};

// One thread per (row, action): 32 lanes per row, kWideLossRows = 8 rows per 256-thread block, so
// an 8,192-row minibatch is 1,024 blocks (the first form ran one thread per row over the actions
// in a serial loop: 32 blocks, each lane a chain of 2 x 17 tanh / divide steps). The row's
// log-prob is the sum of its 32 lanes (DPP within 16-lane rows + v_permlane16_swap); the block
// partials per action (d loss / d logstd_a, dz_a), the critic bias gradient and the two loss terms
// are added over the block's 8 rows in row order.
__device__ __forceinline__ float half_sum32(float s) {  // sum over each 32-lane half, every lane
  s = fu::row16_sum(s);
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}

__global__ __launch_bounds__(256) void wide_loss_kernel(WideLossArgs q) {
  static_assert(kWideLossRows * 32 == 256, "32 lanes per row");
  __shared__ float rls[kWideLossRows][32], rdz[kWideLossRows][32], rrow[kWideLossRows][3];
  __shared__ float s_logsd[32], s_var[32], s_b[32];
  const int tid = threadIdx.x, a = tid & 31, r = tid >> 5;
  const int A = q.act_dim;
  if (tid < 32) {
    const float sd = tid < A ? expf(q.logstd[tid]) : 1.f;
    s_logsd[tid] = logf(sd);
    s_var[tid] = sd * sd;
    s_b[tid] = (q.ba && tid < A) ? q.ba[tid] : 0.f;
  }
  __syncthreads();
  const int count = q.rows_n ? *q.rows_n : q.b;
  const int j = blockIdx.x * kWideLossRows + r;
  const bool valid = j < count;
  const bool act = a < A;
  const int64_t sr = valid ? q.rows[j] : 0;
  const float var = s_var[a];
  const float z = q.za[static_cast<int64_t>(j) * 32 + a] + s_b[a];
  const float y = tanhf(z);
  const float mu = q.omv * y;
  const float x = (valid && act) ? q.actions[sr * A + a] : mu;
  const float d = x - mu;
  const float logp = half_sum32(act ? ((-(d * d)) / (2.f * var) - s_logsd[a]) - kLogSqrt2Pi : 0.f);
  const float old_lp = valid ? q.old_logp[sr] : logp;
  const float adv = valid ? q.adv[sr] : 0.f;
  const float ratio = expf(logp - old_lp);
  const float s1 = ratio * adv;
  const float cl = ratio < q.clip_lo ? q.clip_lo : (ratio > q.clip_hi ? q.clip_hi : ratio);
  const float s2 = cl * adv;
  const float mn = (s1 != s1 || s2 != s2) ? (s1 + s2) : (s2 < s1 ? s2 : s1);
  const float g = -q.inv_b;
  const float g1 = (s1 < s2) ? g : (s1 == s2 ? g * 0.5f : 0.f);
  const float g2 = (s2 < s1) ? g : (s1 == s2 ? g * 0.5f : 0.f);
  const bool inside = (ratio >= q.clip_lo) && (ratio <= q.clip_hi);
  const float dratio = g1 * adv + (inside ? g2 * adv : 0.f);
  const float dlogp = valid ? dratio * ratio : 0.f;
  const bool live = valid && act;
  const float dmu = dlogp * (d / var);
  const float dz = live ? (dmu * q.omv) * (1.f - y * y) : 0.f;
  const float ls = live ? dlogp * ((d * d) / var - 1.f) - q.ent_coef * q.inv_ba : 0.f;
  // dz row: column pairs (a, a + 1) packed by the even lane (columns >= A are zero)
  const float dz_next = fu::dpp_f<fu::kDppXor1>(dz);
  if ((a & 1) == 0)
    reinterpret_cast<uint32_t *>(q.dza + static_cast<int64_t>(j) * 64)[a >> 1] = wide::pack2(dz, dz_next);
  rls[r][a] = ls;
  rdz[r][a] = dz;
  if (a == 0) {  // critic and the row's loss terms
    const float zc0 = q.zc[static_cast<int64_t>(j) * 32];
    const float v = q.bc ? zc0 + q.bc[0] : zc0;
    const float vt = valid ? q.vtarget[sr] : v;
    const float diff = v - vt;
    const float ad = fabsf(diff);
    const float dv = valid ? q.inv_b * (diff < -1.f ? -1.f : (diff > 1.f ? 1.f : diff)) : 0.f;
    reinterpret_cast<uint32_t *>(q.dzc + static_cast<int64_t>(j) * 64)[0] = wide::pack2(dv, 0.f);
    rrow[r][0] = dv;
    rrow[r][1] = valid ? mn : 0.f;
    rrow[r][2] = valid ? ((ad < 1.f) ? 0.5f * ad * ad : (ad - 0.5f)) : 0.f;
  }
  __syncthreads();
  float *part = q.part + static_cast<int64_t>(blockIdx.x) * kWidePart;
  if (tid < 64) {  // logstd grads [0, 32), actor head bias [32, 64): rows in order
    const int col = tid & 31;
    if (col < A) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < kWideLossRows; ++k) s += tid < 32 ? rls[k][col] : rdz[k][col];
      part[tid] = s;
    }
  } else if (tid < 67) {  // critic bias [64], then the actor / critic loss partials
    const int c = tid - 64;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kWideLossRows; ++k) s += rrow[k][c];
    if (c == 0) part[64] = s;
    else q.loss_part[2 * blockIdx.x + c - 1] = s;
  }
}

// The wide path's slab fold in one launch of two block kinds (deterministic, fixed orders):
// - fast blocks, one thread per float4 group of the flat gradient: groups of segments with
//   kRedChunks splits (the hidden-layer WGRAD slabs, nearly all the bytes) issue all their slab
//   loads before the first add and sum them in split order (reduce_slab_block's order for these
//   segments: its chunks hold one split each); pure padding groups are written as zeros;
// - slow blocks over the groups of every other segment (heads: 64 splits, bias column sums, the
//   loss kernel's 1024 per-block partials, a tensor's partial last group, other split counts):
//   G groups x C chunks per block (C = 16, reduce_slab_block's layout and order, or C = 128 for
//   segments of more than 256 splits, so no thread reads more than a handful), then the C chunk
//   sums in chunk order.
// The 16-chunk reduce_slab_block kept one 16-B load in flight per thread on the 16-split slabs
// and 64 sequential loads per thread on the 1024-split partials.
constexpr int kHeavyChunks = 128;
struct WideRedPlan {
  int fast_blocks;
  int nslow;                      // slow runs: `groups` float4 groups from parameter `first`
  int seg[kMaxSegs];
  int chunks[kMaxSegs];           // kRedChunks or kHeavyChunks
  int64_t first[kMaxSegs];
  int64_t groups[kMaxSegs];
  int bprefix[kMaxSegs + 1];      // cumulative block counts of the runs
};

// fast segments: 16 or 8 splits (at most one split per reduce_slab_block chunk), aligned
__host__ __device__ __forceinline__ bool fast_seg(const ReduceSeg &g) {
  return (g.nsplit == kRedChunks || g.nsplit == kRedChunks / 2) && g.stride % 4 == 0 &&
         reinterpret_cast<uintptr_t>(g.src) % 16 == 0;
}

// The fast path's sum of S <= kRedChunks splits in reduce_slab_block's order: chunk c holds split
// S c / 16 when S (c + 1) / 16 exceeds it (one split, summed as (0 + v) + 0), else nothing (0);
// the chunks are added in order, every addition kept (adding +0 can change a -0).
template <int S>
__device__ __forceinline__ float4 fast_split_sum(const ReduceSeg &g, int64_t off) {
  float4 v[S];
#pragma unroll
  for (int k = 0; k < S; ++k) v[k] = *reinterpret_cast<const float4 *>(g.src + off + k * g.stride);
  auto chunk = [&](int c) {
    const int k0 = (S * c) / kRedChunks, k1 = (S * (c + 1)) / kRedChunks;
    if (k1 == k0) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 a = v[k0];
    return make_float4((0.f + a.x) + 0.f, (0.f + a.y) + 0.f, (0.f + a.z) + 0.f, (0.f + a.w) + 0.f);
  };
  float4 out = chunk(0);
#pragma unroll
  for (int c = 1; c < kRedChunks; ++c) {
    const float4 b = chunk(c);
    out = make_float4(out.x + b.x, out.y + b.y, out.z + b.z, out.w + b.w);
  }
  return out;
}

// splits [k0, k1) of parameters i..i+3 (i - g.dst = off >= 0): slab_item_sum's arithmetic (two
// interleaved float4 sums, or eight strided partial sums per element off the aligned path)
__device__ __forceinline__ float4 split_range_sum(const ReduceSeg &g, int64_t off, int k0, int k1) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (off + 3 < g.len && g.stride % 4 == 0 && reinterpret_cast<uintptr_t>(g.src) % 16 == 0) {
    const float *src = g.src + off;
    float4 acc1 = acc;
    int k = k0;
    for (; k + 1 < k1; k += 2) {
      const float4 v = *reinterpret_cast<const float4 *>(src + k * g.stride);
      const float4 u = *reinterpret_cast<const float4 *>(src + (k + 1) * g.stride);
      acc = make_float4(acc.x + v.x, acc.y + v.y, acc.z + v.z, acc.w + v.w);
      acc1 = make_float4(acc1.x + u.x, acc1.y + u.y, acc1.z + u.z, acc1.w + u.w);
    }
    if (k < k1) {
      const float4 v = *reinterpret_cast<const float4 *>(src + k * g.stride);
      acc = make_float4(acc.x + v.x, acc.y + v.y, acc.z + v.z, acc.w + v.w);
    }
    return make_float4(acc.x + acc1.x, acc.y + acc1.y, acc.z + acc1.z, acc.w + acc1.w);
  }
  float a4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (off + e >= g.len) continue;
    const float *src = g.src + off + e;
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int k = k0;
    for (; k + 7 < k1; k += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s8[j] += src[static_cast<int64_t>(k + j) * g.stride];
    }
    for (; k < k1; ++k) s8[0] += src[static_cast<int64_t>(k) * g.stride];
    a4[e] = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  }
  return make_float4(a4[0], a4[1], a4[2], a4[3]);
}

__global__ __launch_bounds__(kRedThreads) void wide_reduce_kernel(ReduceArgs q, WideRedPlan pl) {
  __shared__ __attribute__((aligned(16))) char scratch[kRedScratchBytes];
  const RedScratch sc = red_scratch(scratch);
  const int tid = threadIdx.x;
  if (tid < q.nseg) sc.sseg[tid] = q.seg[tid];
  __syncthreads();
  if (static_cast<int>(blockIdx.x) < pl.fast_blocks) {
    const int64_t i = (static_cast<int64_t>(blockIdx.x) * kRedThreads + tid) * 4;
    if (i < q.total) {
      const ReduceSeg &g = sc.sseg[seg_find(sc.sseg, q.nseg, i)];
      const int64_t off = i - g.dst;
      if (off < 0 || off >= g.len) {  // between tensors: padding
        *reinterpret_cast<float4 *>(q.grad + i) = make_float4(0.f, 0.f, 0.f, 0.f);
      } else if (fast_seg(g) && off + 3 < g.len) {
        const float4 out = g.nsplit == kRedChunks ? fast_split_sum<kRedChunks>(g, off)
                                                  : fast_split_sum<kRedChunks / 2>(g, off);
        *reinterpret_cast<float4 *>(q.grad + i) = out;
      }
    }
    if (blockIdx.x == 0 && q.loss_out) reduce_loss_block(q, sc.lred);
    return;
  }
  // slow block: G = kRedThreads / C groups of one run, C chunks each
  const int sb = static_cast<int>(blockIdx.x) - pl.fast_blocks;
  int run = 0;
  while (run + 1 < pl.nslow && pl.bprefix[run + 1] <= sb) ++run;
  const int C = pl.chunks[run], G = kRedThreads / C;
  const int grp = tid % G, chunk = tid / G;
  const int64_t gi = static_cast<int64_t>(sb - pl.bprefix[run]) * G + grp;
  const bool valid = gi < pl.groups[run];
  const ReduceSeg &g = sc.sseg[pl.seg[run]];
  const int64_t i = pl.first[run] + 4 * gi;
  float4 ps = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid) {
    const int k0 = (g.nsplit * chunk) / C, k1 = (g.nsplit * (chunk + 1)) / C;
    ps = split_range_sum(g, i - g.dst, k0, k1);
  }
  sc.part[chunk * G + grp] = ps;
  __syncthreads();
  if (chunk == 0 && valid) {
    float4 out = sc.part[grp];
    for (int c = 1; c < C; ++c) {
      const float4 b = sc.part[c * G + grp];
      out = make_float4(out.x + b.x, out.y + b.y, out.z + b.z, out.w + b.w);
    }
    *reinterpret_cast<float4 *>(q.grad + i) = out;
  }
}

int wide_minibatch_grad(ppo_ctx *ctx, const float *states_d, const float *actions_d,
                        const float *old_logp_d, const float *adv_d, const float *vtarget_d,
                        const int32_t *rows_d, int b, const int32_t *count_d, float clip_lo,
                        float clip_hi, float entropy_coef, float inv_b, float inv_ba,
                        float *grad_d, float *loss_d, hipStream_t st) {
  WideWork &W = *ctx->wide;
  const int rows_pad = static_cast<int>(rup(b, 64));
  const int64_t P = ctx->total_params;
  const int A = ctx->cfg.act_dim;
  NetDesc &NA = ctx->net[0], &NC = ctx->net[1];
  {  // weight images + the minibatch's rows, one launch
    const GatherArgs g = gather_args(ctx, states_d, rows_d, count_d, b, rows_pad);
    if (int rc = wide_pack(ctx, st, W.fused_rollout, &g)) return rc;
  }
  const bool both[2] = {true, true};
  if (W.fused_rollout) {  // one launch: hidden layers + heads, activations LDS-resident
    if (int rc = wide_forward_fused(ctx, rows_pad, b, count_d, st)) return rc;
  } else if (int rc = forward(ctx, both, rows_pad, count_d, st)) {
    return rc;
  }

  // ---- loss heads -----------------------------------------------------------------------------
  const int blocks = ceil_div(rows_pad, kWideLossRows);
  {
    WideLossArgs q{};
    q.za = W.net[0].z;
    q.zc = W.net[1].z;
    q.dza = W.net[0].dz;
    q.dzc = W.net[1].dz;
    q.act_dim = A;
    const LayerDesc &HA = NA.layer[NA.n_hidden], &HC = NC.layer[NC.n_hidden];
    q.ba = HA.b_off >= 0 ? ctx->params + HA.b_off : nullptr;
    q.logstd = ctx->params + NA.logstd_off;
    q.bc = ctx->params + HC.b_off;
    q.omv = ctx->cfg.output_max_value;
    q.rows = rows_d;
    q.rows_n = count_d;
    q.b = b;
    q.actions = actions_d;
    q.old_logp = old_logp_d;
    q.adv = adv_d;
    q.vtarget = vtarget_d;
    q.clip_lo = clip_lo;
    q.clip_hi = clip_hi;
    q.ent_coef = entropy_coef;
    q.inv_b = inv_b;
    q.inv_ba = inv_ba;
    q.part = W.part;
    q.loss_part = W.loss_part;
    launch_k(TimRec{KC_UPDATE_HEAD, "wide_loss_kernel", 0.0,
                    static_cast<double>(b) * (4.0 * 64 + 4.0 * A + 16.0 + 256.0)},
             wide_loss_kernel, dim3(blocks), dim3(256), 0, st, q);
    PPO_LAUNCHED();
  }

  // ---- backward, deepest layer first: layer l's WGRAD (dZ_l^T H_{l-1}) and DGRAD (dZ_{l-1} =
  // act'(H_{l-1}) * dZ_l W_l, into dh[l-1]) both read dZ_l and not each other's output, so
  // wide::run_pair issues them as one launch where the tiles allow (the hidden layers)
  int colsum_rows[2][PPO_MAX_LAYERS] = {};
  int splits_of[2][PPO_MAX_LAYERS + 1] = {};
  const int depth = std::max(NA.n_hidden, NC.n_hidden);
  for (int s = 0; s <= depth; ++s) {
    // weight gradient of layer l = n_hidden - s
    WideBatch wg{};
    wg.rows_n = count_d;
    int np = 0, max_m = 0, max_n = 0;
    for (int z = 0; z < 2; ++z) {
      const NetDesc &nd = ctx->net[z];
      const int l = nd.n_hidden - s;
      if (l < 0) continue;
      const LayerDesc &L = nd.layer[l];
      const WideNetWork &wn = W.net[z];
      WideProblem &Q = wg.p[np++];
      Q.a = l == nd.n_hidden ? wn.dz : wn.dh[l];
      Q.lda = l == nd.n_hidden ? 64 : wn.ldh[l];
      Q.b = l == 0 ? W.x : wn.h[l - 1];
      Q.ldb = l == 0 ? W.ldx : wn.ldh[l - 1];
      Q.c = ctx->slabs + L.w_off;
      Q.ldc = L.in;
      Q.m = L.out;
      Q.n = L.in;
      Q.k = rows_pad;
      Q.slab_stride = P;
      max_m = std::max(max_m, L.out);
      max_n = std::max(max_n, L.in);
    }
    const int np_w = np, max_m_w = max_m, max_n_w = max_n;
    if (np_w) {
      wg.splits = s == 0 ? kWideHeadSplits : g_wide_splits;
      for (int z = 0; z < 2; ++z)
        if (ctx->net[z].n_hidden - s >= 0) splits_of[z][ctx->net[z].n_hidden - s] = wg.splits;
    }
    // input gradient of layer l into dh[l-1] (l >= 1)
    WideBatch dg{};
    dg.rows_n = count_d;
    dg.act = ctx->cfg.activation;
    np = 0;
    max_n = 0;
    for (int z = 0; z < 2; ++z) {
      const NetDesc &nd = ctx->net[z];
      const int l = nd.n_hidden - s;
      if (l < 1) continue;
      const LayerDesc &L = nd.layer[l];
      const WideNetWork &wn = W.net[z];
      WideProblem &Q = dg.p[np++];
      Q.a = l == nd.n_hidden ? wn.dz : wn.dh[l];
      Q.lda = l == nd.n_hidden ? 64 : wn.ldh[l];
      Q.b = wn.wt[l];
      Q.ldb = wn.ldwt[l];
      Q.c = wn.dh[l - 1];
      Q.aux = wn.h[l - 1];
      Q.ldc = wn.ldh[l - 1];
      Q.colsum = nd.layer[l - 1].b_off >= 0 ? wn.colsum[l - 1] : nullptr;
      Q.n_colsum = L.in;
      Q.m = rows_pad;
      Q.n = L.in;
      Q.k = wn.ldwt[l];
      max_n = std::max(max_n, L.in);
    }
    if (np) {
      const int tile = wide::row_tile(wide::WK_DGRAD, rows_pad, max_n);
      for (int z = 0; z < 2; ++z) {
        const int l = ctx->net[z].n_hidden - s;
        if (l >= 1) colsum_rows[z][l - 1] = ceil_div(rows_pad, tile);
      }
      if (np_w) {
        if (int rc = wide::run_pair(wg, np_w, max_m_w, max_n_w, b, dg, np, rows_pad, max_n, st))
          return rc;
      } else if (int rc = wide::run(wide::WK_DGRAD, dg, np, rows_pad, max_n, 0, st)) {
        return rc;
      }
    } else if (np_w) {
      if (int rc = wide::run(wide::WK_WGRAD, wg, np_w, max_m_w, max_n_w, b, st)) return rc;
    }
  }

  // ---- fixed-order reduction into the flat gradient + loss scalars ----------------------------
  ReduceArgs r{};
  int ns = 0;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    if (z == 0) {
      ReduceSeg &g = r.seg[ns++];
      g.dst = nd.logstd_off;
      g.len = A;
      g.src = W.part;
      g.stride = kWidePart;
      g.nsplit = blocks;
    }
    for (int l = 0; l <= nd.n_hidden; ++l) {
      const LayerDesc &L = nd.layer[l];
      ReduceSeg &g = r.seg[ns++];
      g.dst = L.w_off;
      g.len = static_cast<int64_t>(L.out) * L.in;
      g.src = ctx->slabs + L.w_off;
      g.stride = P;
      g.nsplit = splits_of[z][l];
      if (L.b_off >= 0) {
        ReduceSeg &gb = r.seg[ns++];
        gb.dst = L.b_off;
        gb.len = L.out;
        if (l < nd.n_hidden) {
          gb.src = W.net[z].colsum[l];
          gb.stride = L.out;
          gb.nsplit = colsum_rows[z][l];
        } else {
          gb.src = W.part + (z == 0 ? 32 : 64);
          gb.stride = kWidePart;
          gb.nsplit = blocks;
        }
      }
    }
  }
  r.nseg = ns;
  r.total = P;
  r.grad = grad_d;
  r.loss_part = W.loss_part;
  r.loss_splits = blocks;
  r.inv_b = inv_b;
  r.logstd = ctx->params + NA.logstd_off;
  r.act_dim = A;
  r.ent_coef = entropy_coef * ctx->ent_log_share;
  r.loss_out = loss_d;
  double slab_floats = 0;
  for (int i = 0; i < ns; ++i) slab_floats += static_cast<double>(r.seg[i].nsplit) * r.seg[i].len;
  // the fold plan: fast groups (16-split aligned segments) by the fast blocks, the rest in runs
  WideRedPlan pl{};
  pl.fast_blocks = static_cast<int>(ceil_div(P, 4 * kRedThreads));
  auto add_run = [&](int seg, int64_t first, int64_t groups) {
    PPO_REQUIRE(pl.nslow < kMaxSegs, "wide reduce: more than %d slow runs", kMaxSegs);
    const int c = r.seg[seg].nsplit > 256 ? kHeavyChunks : kRedChunks;
    pl.seg[pl.nslow] = seg;
    pl.chunks[pl.nslow] = c;
    pl.first[pl.nslow] = first;
    pl.groups[pl.nslow] = groups;
    pl.bprefix[pl.nslow + 1] =
        pl.bprefix[pl.nslow] + static_cast<int>(ceil_div(groups, kRedThreads / c));
    ++pl.nslow;
    return 0;
  };
  for (int i = 0; i < ns; ++i) {
    const ReduceSeg &g = r.seg[i];
    const bool fast = fast_seg(g);
    if (!fast) {
      if (int rc = add_run(i, g.dst, ceil_div(g.len, 4))) return rc;
    } else if (g.len % 4) {  // the partial last group
      if (int rc = add_run(i, g.dst + 4 * (g.len / 4), 1)) return rc;
    }
  }
  const int slow_blocks = pl.bprefix[pl.nslow];
  launch_k(TimRec{KC_REDUCE, "wide_reduce_kernel", slab_floats, 4.0 * (slab_floats + P)},
           wide_reduce_kernel, dim3(pl.fast_blocks + slow_blocks), dim3(kRedThreads), 0, st, r, pl);
  PPO_LAUNCHED();
  return 0;
}

}  // namespace ppo
