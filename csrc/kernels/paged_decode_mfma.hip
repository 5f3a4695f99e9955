// Paged GQA decode attention on MFMA for gfx950 (D = 128, 16-token KV pages).
//
// One query token per sequence against its paged KV cache; all G = H/KVH query
// heads of one KV head are processed together in ONE MFMA tile (the 16-wide
// column dimension holds the group's heads, zero-padded), so every K/V byte is
// read once per KV head:
//
//   S^T[tok][head] = K[tok][:] . Q[head][:]    v_mfma_f32_16x16x32_bf16, A = K page
//                                              rows straight from global memory
//                                              (lane = token, 16 B = 8 dims),
//                                              B = Q in registers (scores scaled after)
//   online softmax per head (exp2 domain), the 4 lane groups of a head
//   reduced with two xor-shuffles
//   O^T[dim][head] += V^T[dim][tok] . P^T[tok][head]
//                                              A = V^T from a per-wave LDS image
//                                              ([token][dim], 16-byte chunks XOR-
//                                              swizzled, read with the gfx950
//                                              transpose read ds_read_b64_tr_b16),
//                                              B = P straight from the S^T
//                                              accumulators (the image rows are
//                                              permuted so that lane group g's
//                                              k-slots are exactly the tokens whose
//                                              scores it already holds: no shuffle)
//
// A wave handles two 32-token chunks (two pages each): 2 x (8 x 16 B K + 8 x 16 B
// V) loads per lane in flight at once, then 8 + 8 MFMAs per chunk. A 256-thread
// block covers a partition of 256 tokens (4 waves x 2 chunks); the waves' (max, sum, O) are
// merged through LDS. Contexts longer than one partition write un-normalised
// partials that pdm_reduce merges ("flash-decoding"), so long contexts still
// spread over all 256 CUs.
#include "common.h"

namespace caamd {
namespace pdm {

typedef __attribute__((address_space(3))) char lds_char;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int D = 128, BS = 16, CH = 32, WAVES = 4, PART = WAVES * CH * 2;  // 256 tokens / block

__device__ __forceinline__ int mswz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

__device__ __forceinline__ void st_img(lds_char* img, int k, int m8, const bf16x8& v) {
  const int pos = (m8 >> 3) ^ mswz(k);
  *(__attribute__((address_space(3))) bf16x8*)(img + k * (D * 2) + pos * 16) = v;
}

// rows [rr, rr+16) (dims) x k [0, 32) (image rows): lane l gets row rr+(l&15), k = 8*(l>>4)+j
__device__ __forceinline__ bf16x8 frag_img(const lds_char* img, int rr, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int m = rr + 4 * p;
  const int chunk = m >> 3;
  const int within = (p & 1) * 8;
  s16x4 lo, hi;
  {
    const int k = 8 * g + q;
    lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (D * 2) + ((chunk ^ mswz(k)) * 16) + within));
  }
  {
    const int k = 8 * g + 4 + q;
    hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (D * 2) + ((chunk ^ mswz(k)) * 16) + within));
  }
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int G>
__global__ __launch_bounds__(256, 3) void paged_decode_mfma_kernel(
    const bf16* __restrict__ q, int q_stride, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ ctx_lens, bf16* __restrict__ out,
    float* __restrict__ part_acc, float* __restrict__ part_ml, int KVH, int max_parts, float scale_log2) {
  __shared__ __attribute__((aligned(16))) bf16 vimg[WAVES][CH * D];  // 8 KB per wave
  __shared__ float wm[WAVES][16], wl[WAVES][16];
  __shared__ float wo[WAVES][G][D];

  const int part = blockIdx.x, kvh = blockIdx.y, seq = blockIdx.z;
  const int ctx = ctx_lens[seq];
  const int t0 = part * PART;
  if (t0 >= ctx) return;  // uniform for the block (before any barrier)
  const int t1 = min(ctx, t0 + PART);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, g = lane >> 4, r16 = lane & 15;
  const int H = KVH * G;

  // Q (B operand of S^T): column = head r16 of the group, k-slots = dims 32s + 8g + j
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    // branch-free (a lane-divergent branch around each load serialises the four
    // loads behind their own waits) and unscaled (scaling here would wait for Q
    // before the K/V loads issue; the scores are scaled instead): padding columns
    // load head G-1, their scores land in output columns that are never stored
    qf[s] = *reinterpret_cast<const bf16x8*>(q + (size_t)seq * q_stride + (kvh * G + min(r16, G - 1)) * D +
                                             32 * s + 8 * g);
  }
  const int* bt = block_tables + (size_t)seq * max_blocks;
  lds_char* img = (lds_char*)vimg[wave];
  float m = -INFINITY, lsum = 0.f;
  f32x4 o[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A wave owns at most two 32-token chunks of the partition (PART = WAVES * CH * 2).
  // Both chunks' K and V loads are issued before either is consumed, so the wave
  // waits on one memory latency instead of a dependent chain of two (the kernel
  // moves ~10 MB per layer at batch 128: it is latency-bound, not bandwidth-bound).
  // A missing chunk re-loads a valid one (uniform, branch-free issue) and is masked.
  const int cA = t0 + wave * CH, cB = cA + WAVES * CH;
  const bool hasA = cA < t1, hasB = cB < t1;
  const int cAc = hasA ? cA : t0, cBc = hasB ? cB : cAc;
  const size_t page = (size_t)BS * D;
  // the four page ids, loaded together (second page of a chunk past the context
  // end -> the first page again; its scores are masked)
  int pb[4];
  pb[0] = bt[cAc / BS];
  pb[1] = bt[cAc / BS + (cAc + BS < t1 ? 1 : 0)];
  pb[2] = bt[cBc / BS];
  pb[3] = bt[cBc / BS + (cBc + BS < t1 ? 1 : 0)];
  bf16x8 kf[2][8], vv[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const bf16* K0 = kc + ((size_t)pb[2 * h] * KVH + kvh) * page;
    const bf16* K1 = kc + ((size_t)pb[2 * h + 1] * KVH + kvh) * page;
    const bf16* V0 = vc + ((size_t)pb[2 * h] * KVH + kvh) * page;
    const bf16* V1 = vc + ((size_t)pb[2 * h + 1] * KVH + kvh) * page;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[h][s] = *reinterpret_cast<const bf16x8*>(K0 + r16 * D + 32 * s + 8 * g);
      kf[h][4 + s] = *reinterpret_cast<const bf16x8*>(K1 + r16 * D + 32 * s + 8 * g);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int v = lane + 64 * u, t = v >> 4, cc = (v & 15) * 8;
      vv[h][u] = *reinterpret_cast<const bf16x8*>((t < 16 ? V0 : V1) + (t & 15) * D + cc);
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // straight-line for both chunks (a branch around chunk B would let the compiler
    // sink its loads into the branch, behind chunk A's compute): a missing chunk
    // starts at t1, so all of its scores are masked
    const int c0 = h == 0 ? (hasA ? cA : t1) : (hasB ? cB : t1);
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = mfma(kf[h][s], qf[s], s0);
      s1 = mfma(kf[h][4 + s], qf[s], s1);
    }
    // lane holds S^T[token 4g+i][head r16] of page 0 (s0) and page 1 (s1)
    float mt = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s0[i] = c0 + 4 * g + i >= t1 ? -INFINITY : s0[i] * scale_log2;
      s1[i] = c0 + 16 + 4 * g + i >= t1 ? -INFINITY : s1[i] * scale_log2;
      mt = fmaxf(mt, fmaxf(s0[i], s1[i]));
    }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float mref = mn == -INFINITY ? 0.f : mn;  // nothing valid yet: p = 0, alpha = 0 (o, lsum are 0)
    const float alpha = __builtin_amdgcn_exp2f(m - mref);
    m = mn;
    bf16x8 pf;
    float ps = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p0 = __builtin_amdgcn_exp2f(s0[i] - mref), p1 = __builtin_amdgcn_exp2f(s1[i] - mref);
      ps += p0 + p1;
      pf[i] = (bf16)p0;
      pf[4 + i] = (bf16)p1;
    }
    lsum = lsum * alpha + ps;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[c][i] *= alpha;
    }
    // V into the wave's image: token t -> image row so that lane group g's k-slots 8g..8g+7 are
    // page-0 tokens 4g..4g+3 then page-1 tokens 4g..4g+3 (the scores this group holds)
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int v = lane + 64 * u, t = v >> 4, cc = (v & 15) * 8;
      const int tt = t & 15;
      const int row = 8 * (tt >> 2) + (t >= 16 ? 4 : 0) + (tt & 3);
      st_img(img, row, cc, vv[h][u]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 8; ++c) o[c] = mfma(frag_img(img, 16 * c, lane), pf, o[c]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // image reads done before the next chunk's writes
    __builtin_amdgcn_wave_barrier();
  }
  float l = lsum + __shfl_xor(lsum, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (g == 0) {
    wm[wave][r16] = m;
    wl[wave][r16] = l;
  }
  if (r16 < G) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) wo[wave][r16][16 * c + 4 * g + i] = o[c][i];
  }
  __syncthreads();
  const int nparts = (ctx + PART - 1) / PART;
  for (int e = threadIdx.x; e < G * D; e += 256) {
    const int h = e / D, d = e % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) M = fmaxf(M, wm[w][h]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      const float f = (wm[w][h] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(wm[w][h] - M);
      num += f * wo[w][h][d];
      den += f * wl[w][h];
    }
    const int hh = kvh * G + h;
    if (nparts == 1) {
      out[((size_t)seq * H + hh) * D + d] = (bf16)(num / den);
    } else {
      part_acc[(((size_t)seq * H + hh) * max_parts + part) * D + d] = num;
      if (d == 0) {
        part_ml[(((size_t)seq * H + hh) * max_parts + part) * 2 + 0] = M;
        part_ml[(((size_t)seq * H + hh) * max_parts + part) * 2 + 1] = den;
      }
    }
  }
  // (partitions are merged by pdm_reduce_kernel; a last-arriver merge in this kernel
  // -- one agent-scope release per partition block -- measured 11.3 vs 6.65 ms TPOT
  // and was removed in round 4, profiles/llm_decode_ab_r3_paged_merge.txt)
}

// one block (D threads) per (seq, head): merge partitions (exp2 domain)
__global__ void pdm_reduce_kernel(const float* __restrict__ part_acc, const float* __restrict__ part_ml,
                                  const int* __restrict__ ctx_lens, bf16* __restrict__ out, int H, int max_parts) {
  const int seq = blockIdx.y, hh = blockIdx.x, d = threadIdx.x;
  const int nparts = (ctx_lens[seq] + PART - 1) / PART;
  if (nparts <= 1) return;
  const float* ml = part_ml + ((size_t)seq * H + hh) * max_parts * 2;
  float M = -INFINITY;
  for (int p = 0; p < nparts; ++p) M = fmaxf(M, ml[2 * p]);
  float num = 0.f, den = 0.f;
  const float* pa = part_acc + ((size_t)seq * H + hh) * max_parts * D;
  for (int p = 0; p < nparts; ++p) {
    const float w = __builtin_amdgcn_exp2f(ml[2 * p] - M);
    num += w * pa[(size_t)p * D + d];
    den += w * ml[2 * p + 1];
  }
  out[((size_t)seq * H + hh) * D + d] = (bf16)(num / den);
}

}  // namespace pdm

int paged_mfma_max_parts(int max_ctx) { return (max_ctx + pdm::PART - 1) / pdm::PART; }

bool paged_decode_mfma_launch(const bf16* q, int q_stride, const bf16* kc, const bf16* vc, const int* block_tables,
                              int max_blocks, const int* ctx_lens, bf16* out, float* part_acc, float* part_ml, int B,
                              int H, int KVH, int D, int BS, int max_ctx, float scale, hipStream_t st) {
  if (D != pdm::D || BS != pdm::BS) return false;
  const int G = H / KVH;
  const int mp = paged_mfma_max_parts(max_ctx);
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(mp, KVH, B), block(256);
#define PDM_CASE(GG)                                                                                          \
  if (G == GG) {                                                                                              \
    hipLaunchKernelGGL((pdm::paged_decode_mfma_kernel<GG>), grid, block, 0, st, q, q_stride, kc, vc,          \
                       block_tables, max_blocks, ctx_lens, out, part_acc, part_ml, KVH, mp, sl2);             \
    if (mp > 1)                                                                                               \
      hipLaunchKernelGGL(pdm::pdm_reduce_kernel, dim3(H, B), dim3(pdm::D), 0, st, part_acc, part_ml, ctx_lens, \
                         out, H, mp);                                                                         \
    return true;                                                                                              \
  }
  PDM_CASE(1) PDM_CASE(2) PDM_CASE(4) PDM_CASE(8) PDM_CASE(16)
#undef PDM_CASE
  return false;
}

}  // namespace caamd
