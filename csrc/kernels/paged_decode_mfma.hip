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
//                                              B = pre-scaled Q in registers
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
// A wave handles 32-token chunks (two pages): 8 x 16 B K loads and 8 x 16 B V
// loads per lane in flight, then 8 + 8 MFMAs. A 256-thread block covers a
// partition of 256 tokens (4 waves x 2 chunks); the waves' (max, sum, O) are
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
__global__ __launch_bounds__(256) void paged_decode_mfma_kernel(
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
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, r16 = lane & 15;
  const int H = KVH * G;

  // Q (B operand of S^T): column = head r16 of the group, k-slots = dims 32s + 8g + j
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf16x8 v = {};
    if (r16 < G) {
      const bf16x8 raw = *reinterpret_cast<const bf16x8*>(q + (size_t)seq * q_stride + (kvh * G + r16) * D +
                                                         32 * s + 8 * g);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)raw[j] * scale_log2);
    }
    qf[s] = v;
  }
  const int* bt = block_tables + (size_t)seq * max_blocks;
  lds_char* img = (lds_char*)vimg[wave];
  float m = -INFINITY, lsum = 0.f;
  f32x4 o[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = t0 + wave * CH; c0 < t1; c0 += WAVES * CH) {
    const int pg = c0 / BS;  // c0 is page aligned (multiple of 32)
    const bool has1 = c0 + BS < t1;
    const int b0 = bt[pg], b1 = has1 ? bt[pg + 1] : b0;
    const size_t page = (size_t)BS * D;
    const bf16* K0 = kc + ((size_t)b0 * KVH + kvh) * page;
    const bf16* K1 = kc + ((size_t)b1 * KVH + kvh) * page;
    const bf16* V0 = vc + ((size_t)b0 * KVH + kvh) * page;
    const bf16* V1 = vc + ((size_t)b1 * KVH + kvh) * page;
    bf16x8 k0f[4], k1f[4], vv[8];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      k0f[s] = *reinterpret_cast<const bf16x8*>(K0 + r16 * D + 32 * s + 8 * g);
      k1f[s] = *reinterpret_cast<const bf16x8*>(K1 + r16 * D + 32 * s + 8 * g);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int v = lane + 64 * u, t = v >> 4, cc = (v & 15) * 8;
      vv[u] = *reinterpret_cast<const bf16x8*>((t < 16 ? V0 : V1) + (t & 15) * D + cc);
    }
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = mfma(k0f[s], qf[s], s0);
      s1 = mfma(k1f[s], qf[s], s1);
    }
    // lane holds S^T[token 4g+i][head r16] of page 0 (s0) and page 1 (s1)
    float mt = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (c0 + 4 * g + i >= t1) s0[i] = -INFINITY;
      if (c0 + 16 + 4 * g + i >= t1) s1[i] = -INFINITY;
      mt = fmaxf(mt, fmaxf(s0[i], s1[i]));
    }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);  // finite: every chunk holds at least one valid token
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    bf16x8 pf;
    float ps = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p0 = __builtin_amdgcn_exp2f(s0[i] - mn), p1 = __builtin_amdgcn_exp2f(s1[i] - mn);
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
      st_img(img, row, cc, vv[u]);
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
