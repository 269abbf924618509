// Deterministic split-K reduction of per-workgroup partial-gradient slabs into the flat
// gradient, plus the minibatch loss scalars (ppo.py:121,133 `loss.item()` values).  Shared by
// reduce_slabs_kernel (mlp_engine.hip) and step_tail_kernel (fused_update.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"

namespace ppo {

constexpr int kMaxSegs = 48;
struct ReduceSeg {
  int64_t dst, len;
  const float *src;
  int64_t stride;
  int nsplit;
};
struct ReduceArgs {
  ReduceSeg seg[kMaxSegs];
  int nseg;
  int64_t total;
  float *grad;
  const float *loss_part;
  int loss_splits;
  float inv_b;           // actor loss = -(sum min)*inv_b - ent_coef*H ; critic = sum*inv_b
  const float *logstd;   // H = mean_a(0.5 + 0.5 log 2pi + log(exp(logstd_a))) (Normal.entropy)
  int act_dim;
  float ent_coef;
  float *loss_out;
};

// Block = kRedGroups float4 groups x kRedChunks split-chunks (512 threads): each thread sums
// 1/kRedChunks of the splits for 4 consecutive parameters (tensors start 16-float aligned, so a
// group never straddles two tensors), then the chunks combine in a fixed order through LDS -- 16
// chunks of 8 slabs each keep 2x the loads in flight of a 4-chunk block, which is what the
// 128-slab fused reduction (step_tail_kernel) is bound by.  Block 0 also reduces the per-split
// loss partials with a fixed-shape tree.  Deterministic run to run; reduce_slabs_kernel and
// step_tail_kernel share this exact order, so their results are bitwise equal.
// Returns, on the chunk-0 threads (i < total), the final sums of parameters i..i+3 (also stored
// to q.grad); other threads get zeros.
// The group count G (float4 groups per block) sets only which parameters a block covers: the
// per-parameter order (kRedChunks chunks in order) and the loss tree (kLossSlots virtual slots)
// are the same for every G, so blocks of any G give bitwise the same sums.
constexpr int kRedGroups = 32;
constexpr int kRedChunks = 16;
constexpr int kRedThreads = kRedGroups * kRedChunks;
constexpr int kRedParams = 4 * kRedGroups;  // parameters per block
constexpr int kLossSlots = 512;             // the loss tree's fixed shape
// LDS scratch of one block reduction: part [kRedChunks][G], lred [2][kLossSlots], sseg
// [kMaxSegs] (the kernels declare it as one __shared__ array).
struct RedScratch {
  float4 *part;
  float *lred;
  ReduceSeg *sseg;
};
template <int G = kRedGroups>
constexpr int red_scratch_bytes() {
  return (kRedChunks * G) * 16 + 2 * kLossSlots * 4 + kMaxSegs * static_cast<int>(sizeof(ReduceSeg));
}
constexpr int kRedScratchBytes = red_scratch_bytes<kRedGroups>();
template <int G = kRedGroups>
__device__ __forceinline__ RedScratch red_scratch(char *lds) {
  return RedScratch{reinterpret_cast<float4 *>(lds),
                    reinterpret_cast<float *>(lds + kRedChunks * G * 16),
                    reinterpret_cast<ReduceSeg *>(lds + kRedChunks * G * 16 + 2 * kLossSlots * 4)};
}

// The segment holding parameter i: the last one with dst <= i (dst ascending).
__device__ __forceinline__ int seg_find(const ReduceSeg *sseg, int nseg, int64_t i) {
  int s = 0, hi = nseg - 1;
  while (s < hi) {
    const int mid = (s + hi + 1) >> 1;
    if (sseg[mid].dst <= i) s = mid;
    else hi = mid - 1;
  }
  return s;
}

// Chunk `chunk`'s share (splits [k0, k1)) of parameters i..i+3: the one summation order every
// slab reduction uses.  The aligned path keeps two interleaved partial sums (even / odd split)
// so 8 independent loads stay in flight per thread; the association is fixed, so the result is
// deterministic run to run.  The unaligned path (tail of a tensor, logstd partials, 1-wide
// biases) takes 8 strided partial sums per element; padding stays zero.
__device__ __forceinline__ float4 slab_item_sum(const ReduceArgs &q, const ReduceSeg *sseg,
                                                int64_t i, int chunk) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i >= q.total) return acc;
  const ReduceSeg &g = sseg[seg_find(sseg, q.nseg, i)];
  const int64_t off = i - g.dst;
  const int k0 = (g.nsplit * chunk) / kRedChunks, k1 = (g.nsplit * (chunk + 1)) / kRedChunks;
  if (off >= 0 && off + 3 < g.len && g.stride % 4 == 0 &&
      reinterpret_cast<uintptr_t>(g.src) % 16 == 0) {
    const float *src = g.src + off;
    float4 acc1 = make_float4(0.f, 0.f, 0.f, 0.f);
    int k = k0;
#pragma unroll 4
    for (; k + 1 < k1; k += 2) {
      const float4 v = *reinterpret_cast<const float4 *>(src + k * g.stride);
      const float4 u = *reinterpret_cast<const float4 *>(src + (k + 1) * g.stride);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
      acc1.x += u.x;
      acc1.y += u.y;
      acc1.z += u.z;
      acc1.w += u.w;
    }
    if (k < k1) {
      const float4 v = *reinterpret_cast<const float4 *>(src + k * g.stride);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    acc = make_float4(acc.x + acc1.x, acc.y + acc1.y, acc.z + acc1.z, acc.w + acc1.w);
  } else if (off >= 0) {
    float a4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (off + e >= g.len) continue;
      const float *src = g.src + off + e;
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int k = k0;
      for (; k + 7 < k1; k += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += src[static_cast<int64_t>(k + j) * g.stride];
      }
      for (; k < k1; ++k) s[0] += src[static_cast<int64_t>(k) * g.stride];
      a4[e] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    }
    acc = make_float4(a4[0], a4[1], a4[2], a4[3]);
  }
  return acc;
}

// The chunks of one float4 group combined in chunk order (part[c * stride + grp]).
__device__ __forceinline__ float4 chunk_combine(const float4 *part, int stride, int grp) {
  float4 out = part[grp];
#pragma unroll
  for (int c = 1; c < kRedChunks; ++c) {
    const float4 b = part[c * stride + grp];
    out = make_float4(out.x + b.x, out.y + b.y, out.z + b.z, out.w + b.w);
  }
  return out;
}

// The minibatch loss scalars from the per-split partials: slot v (of kLossSlots) sums partials
// v, v + kLossSlots, ... in order, then a fixed-shape tree over the slots -- the same order for
// any block size NT (every thread of the block must call it).
template <int NT = kRedThreads>
__device__ __forceinline__ void reduce_loss_block(const ReduceArgs &q, float *lred_flat) {
  static_assert(kLossSlots % NT == 0, "loss slots per thread");
  float (*lred)[kLossSlots] = reinterpret_cast<float (*)[kLossSlots]>(lred_flat);
  const int tid = threadIdx.x;
  for (int v = tid; v < kLossSlots; v += NT) {
    float la = 0.f, lc = 0.f;
    for (int k = v; k < q.loss_splits; k += kLossSlots) {
      la += q.loss_part[2 * k];
      lc += q.loss_part[2 * k + 1];
    }
    lred[0][v] = la;
    lred[1][v] = lc;
  }
  __syncthreads();
  for (int w = kLossSlots / 2; w > 0; w >>= 1) {
    for (int v = tid; v < w; v += NT) {
      lred[0][v] += lred[0][v + w];
      lred[1][v] += lred[1][v + w];
    }
    __syncthreads();
  }
  if (tid == 0) {
    float h = 0.f;
    if (q.logstd) {
      for (int a = 0; a < q.act_dim; ++a) h += kEntropyConst + logf(expf(q.logstd[a]));
      h = h / static_cast<float>(q.act_dim);
    }
    q.loss_out[0] = -(lred[0][0] * q.inv_b) - h * q.ent_coef;
    q.loss_out[1] = lred[1][0] * q.inv_b;
  }
}

template <int G = kRedGroups>
__device__ __forceinline__ float4 reduce_slab_block_s(const ReduceArgs &q, int64_t block,
                                                      RedScratch sc) {
  const int tid = threadIdx.x, grp = tid % G, chunk = tid / G;
  const int64_t i = block * (4 * G) + 4 * grp;
  // The segment table, staged once per block: a per-lane lookup straight from the kernel
  // arguments compiled to a chain of dependent loads (one round trip per probe and per field).
  if (tid < q.nseg) sc.sseg[tid] = q.seg[tid];
  __syncthreads();
  sc.part[chunk * G + grp] = slab_item_sum(q, sc.sseg, i, chunk);
  __syncthreads();
  float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
  if (chunk == 0 && i < q.total) {
    out = chunk_combine(sc.part, G, grp);
    *reinterpret_cast<float4 *>(q.grad + i) = out;
  }
  if (block == 0 && q.loss_out) reduce_loss_block<G * kRedChunks>(q, sc.lred);
  return out;
}

__device__ __forceinline__ float4 reduce_slab_block(const ReduceArgs &q, int64_t block) {
  __shared__ __attribute__((aligned(16))) char scratch[kRedScratchBytes];
  return reduce_slab_block_s(q, block, red_scratch(scratch));
}

}  // namespace ppo
