// LLM serving kernels for gfx950 (Llama-family decoder; Serve LLM path):
//   rmsnorm_fwd     : y = x * rsqrt(mean(x^2) + eps) * w, optional fused residual
//                     add (s = x + r written back), one wave per row, row in VGPRs.
//   silu_mul        : out = silu(gu[:, :F]) * gu[:, F:] (SwiGLU, 16-byte vectors).
//   rope_cache      : rotary embedding (rotate-half convention, fp32 cos/sin
//                     table) applied to q and k of the fused qkv projection
//                     IN PLACE, and k/v appended to the paged KV cache at
//                     `slot_mapping` (one thread per (token, head, rotary pair)).
//   paged_decode    : one query token per sequence against its paged KV cache,
//                     grouped-query attention. Grid (partition, kv_head, seq);
//                     a 256-thread block handles up to PART=512 cached tokens of
//                     one kv head for all G = H/KVH query heads sharing it:
//                       pass 1  16 lanes x 16 B per token row (a wave covers 4
//                               tokens per load), G dot products reduced over the
//                               16 lanes with xor-shuffles -> logits in LDS,
//                       pass 2  exact block max / exp / sum (no online rescaling),
//                       pass 3  P.V with the same 16-lane row mapping, per-group
//                               fp32 accumulators merged through LDS.
//                     Contexts longer than PART write un-normalised partials
//                     (acc, max, sum) and paged_reduce merges them (split-K /
//                     "flash-decoding"), so long contexts still fill 256 CUs.
// KV cache layout: [num_blocks, KVH, BS, D] so a page of one head is a single
// contiguous BS*D*2-byte run (BS=16, D=128: 4 KB).
#include "common.h"

namespace caamd {

// ---------------------------------------------------------------- RMSNorm
template <int NV, bool HAS_RES>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                      bf16* __restrict__ s_out, const bf16* __restrict__ w,
                                                      bf16* __restrict__ y, int rows, int D, float eps) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int nchunk = D >> 3;
  const size_t base = (size_t)row * D;
  float v[NV][8];
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = lane + c * 64;
    if (ch < nchunk) {
      load8(x + base + ch * 8, v[c]);
      if (HAS_RES) {
        float t[8];
        load8(r + base + ch * 8, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += t[j];
        store8(s_out + base + ch * 8, v[c]);
        // normalise the bf16-rounded sum (what the next residual add sees)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = (float)(bf16)v[c][j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sq += v[c][j] * v[c][j];
    }
  }
  const float rs = rsqrtf(wave_sum(sq) / (float)D + eps);
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = lane + c * 64;
    if (ch < nchunk) {
      float ww[8], o[8];
      load8(w + ch * 8, ww);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * rs * ww[j];
      store8(y + base + ch * 8, o);
    }
  }
}

// Few rows (decode: one row per sequence, 1..256 rows): the one-wave-per-row
// grid above would put only rows/4 blocks on 256 CUs, each wave walking a
// 4096-wide row serially. Here a 256-thread block owns a row (16 elements per
// thread at D = 4096), the weight load is issued before the reduction, and the
// four wave partial sums meet in LDS.
template <int NV, bool HAS_RES>
__global__ __launch_bounds__(256) void rmsnorm_row_kernel(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                          bf16* __restrict__ s_out, const bf16* __restrict__ w,
                                                          bf16* __restrict__ y, int D, float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x, t = threadIdx.x;
  const int nchunk = D >> 3;
  const size_t base = (size_t)row * D;
  float v[NV][8], ww[NV][8];
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = t + c * 256;
    if (ch < nchunk) {
      load8(x + base + ch * 8, v[c]);
      load8(w + ch * 8, ww[c]);
      if (HAS_RES) {
        float tr[8];
        load8(r + base + ch * 8, tr);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += tr[j];
        store8(s_out + base + ch * 8, v[c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = (float)(bf16)v[c][j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sq += v[c][j] * v[c][j];
    }
  }
  sq = wave_sum(sq);
  if ((t & 63) == 0) red[t >> 6] = sq;
  __syncthreads();
  const float rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)D + eps);
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = t + c * 256;
    if (ch < nchunk) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * rs * ww[c][j];
      store8(y + base + ch * 8, o);
    }
  }
}

void rmsnorm_launch(const bf16* x, const bf16* r, bf16* s_out, const bf16* w, bf16* y, int rows, int D,
                    float eps, hipStream_t st) {
  if (rows < 1024 && D <= 8 * 256 * 4) {
    const int nv = (D / 8 + 255) / 256;
#define RMS_ROW(N)                                                                                        \
  if (nv <= N) {                                                                                         \
    if (r) hipLaunchKernelGGL((rmsnorm_row_kernel<N, true>), dim3(rows), dim3(256), 0, st, x, r, s_out, w, y, D, eps); \
    else hipLaunchKernelGGL((rmsnorm_row_kernel<N, false>), dim3(rows), dim3(256), 0, st, x, r, s_out, w, y, D, eps); \
    return;                                                                                              \
  }
    RMS_ROW(1) RMS_ROW(2) RMS_ROW(4)
#undef RMS_ROW
  }
  dim3 grid((rows + 3) / 4), block(256);
  const int nv = (D / 8 + 63) / 64;
#define RMS_CASE(N)                                                                                       \
  if (nv <= N) {                                                                                         \
    if (r) hipLaunchKernelGGL((rmsnorm_kernel<N, true>), grid, block, 0, st, x, r, s_out, w, y, rows, D, eps); \
    else hipLaunchKernelGGL((rmsnorm_kernel<N, false>), grid, block, 0, st, x, r, s_out, w, y, rows, D, eps); \
    return;                                                                                              \
  }
  RMS_CASE(1) RMS_CASE(2) RMS_CASE(4) RMS_CASE(8) RMS_CASE(16)
#undef RMS_CASE
}

// ---------------------------------------------------------------- SwiGLU
__global__ __launch_bounds__(256) void silu_mul_kernel(const bf16* __restrict__ gu, bf16* __restrict__ out,
                                                       int rows, int F) {
  // grid (column-chunk blocks, rows): no 64-bit index division per element
  const int row = blockIdx.y;
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= F) return;
  const bf16* g_row = gu + (size_t)row * 2 * F;
  float g[8], u[8], o[8];
  load8(g_row + c, g);
  load8(g_row + F + c, u);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = __fdividef(g[j], 1.f + __expf(-g[j])) * u[j];
  store8(out + (size_t)row * F + c, o);
}

// ---------------------------------------------------------------- greedy argmax
// Row argmax of bf16 logits [M, V] (row stride ld) -> int64 [M]: one 1024-thread
// workgroup per row, 16-byte loads, ties to the lowest index (the first maximum).
// Replaces the fp32 copy + torch argmax of the greedy sampler (14 + 41 us per decode
// step at [128, 128256], profiles/llm_serving_prof_r4_final.md).
__device__ __forceinline__ void amax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

__global__ __launch_bounds__(1024) void argmax_rows_kernel(const bf16* __restrict__ x, int V, long long ld,
                                                           long long* __restrict__ out) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const bf16* row = x + (long long)blockIdx.x * ld;
  const int t = threadIdx.x;
  float best = -__builtin_inff();
  int bi = 0x7fffffff;
  const bool vec = ((reinterpret_cast<size_t>(row) & 15) == 0);
  const int nvec = vec ? V / 8 : 0;
  for (int c = t; c < nvec; c += 1024) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(row + 8 * c);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax_merge(best, bi, (float)v[j], 8 * c + j);
  }
  for (int c = 8 * nvec + t; c < V; c += 1024) amax_merge(best, bi, (float)row[c], c);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    amax_merge(best, bi, v2, i2);
  }
  if ((t & 63) == 0) {
    sv[t >> 6] = best;
    si[t >> 6] = bi;
  }
  __syncthreads();
  if (t == 0) {
    float b = sv[0];
    int i = si[0];
    for (int w = 1; w < 16; ++w) amax_merge(b, i, sv[w], si[w]);
    out[blockIdx.x] = i == 0x7fffffff ? 0 : i;
  }
}

void argmax_rows_launch(const bf16* x, int M, int V, long long ld, long long* out, hipStream_t st) {
  hipLaunchKernelGGL(argmax_rows_kernel, dim3(M), dim3(1024), 0, st, x, V, ld, out);
}

void silu_mul_launch(const bf16* gu, bf16* out, int rows, int F, hipStream_t st) {
  for (int r0 = 0; r0 < rows; r0 += 65535) {  // gridDim.y limit
    const int n = rows - r0 < 65535 ? rows - r0 : 65535;
    hipLaunchKernelGGL(silu_mul_kernel, dim3((F / 8 + 255) / 256, n), dim3(256), 0, st, gu + (size_t)r0 * 2 * F,
                       out + (size_t)r0 * F, n, F);
  }
}

// ---------------------------------------------------------------- RoPE + cache append
// qkv: [N, (H + 2*KVH) * D]; cos_sin: [max_pos, D/2, 2] fp32; positions/slots: [N]
// One thread per (token, head, 8 consecutive rotary pairs): 16-byte loads of both
// halves, 8 cos/sin pairs, 16-byte stores to qkv and to the paged cache page.
__global__ __launch_bounds__(256) void rope_cache_kernel(bf16* __restrict__ qkv, const float* __restrict__ cs,
                                                         const int* __restrict__ pos, const int* __restrict__ slot,
                                                         bf16* __restrict__ kc, bf16* __restrict__ vc, int N,
                                                         int H, int KVH, int D, int BS) {
  const int half = D / 2, ng = half / 8;
  const int heads = H + 2 * KVH;
  const int64_t total = (int64_t)N * heads * ng;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(i % ng) * 8;
    const int64_t th = i / ng;
    const int hd = (int)(th % heads);
    const int t = (int)(th / heads);
    bf16* row = qkv + (size_t)t * heads * D + (size_t)hd * D;
    float a[8], b[8];
    load8(row + p, a);
    load8(row + p + half, b);
    if (hd < H + KVH) {  // q or k: rotate
      const float4* c4 = reinterpret_cast<const float4*>(cs + ((size_t)pos[t] * half + p) * 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 c = c4[j];  // (cos, sin) of pairs p + 2j, p + 2j + 1
        const float a0 = a[2 * j], b0 = b[2 * j], a1 = a[2 * j + 1], b1 = b[2 * j + 1];
        a[2 * j] = a0 * c.x - b0 * c.y;
        b[2 * j] = b0 * c.x + a0 * c.y;
        a[2 * j + 1] = a1 * c.z - b1 * c.w;
        b[2 * j + 1] = b1 * c.z + a1 * c.w;
      }
      store8(row + p, a);
      store8(row + p + half, b);
    }
    if (hd >= H && kc != nullptr) {
      const int s = slot[t];
      if (s >= 0) {
        const int blk = s / BS, off = s % BS;
        const int kvh = hd < H + KVH ? hd - H : hd - H - KVH;
        bf16* dst = (hd < H + KVH ? kc : vc) + (((size_t)blk * KVH + kvh) * BS + off) * D;
        store8(dst + p, a);
        store8(dst + p + half, b);
      }
    }
  }
}

void rope_cache_launch(bf16* qkv, const float* cs, const int* pos, const int* slot, bf16* kc, bf16* vc, int N,
                       int H, int KVH, int D, int BS, hipStream_t st) {
  const int64_t total = (int64_t)N * (H + 2 * KVH) * (D / 16);
  hipLaunchKernelGGL(rope_cache_kernel, dim3(ew_grid(total, 256)), dim3(256), 0, st, qkv, cs, pos, slot, kc, vc,
                     N, H, KVH, D, BS);
}

// ---------------------------------------------------------------- paged decode attention
constexpr int kPart = 512;  // tokens per partition (one block)

template <int D, int G>
__global__ __launch_bounds__(256) void paged_decode_kernel(
    const bf16* __restrict__ q, int q_stride, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ ctx_lens,
    bf16* __restrict__ out, float* __restrict__ part_acc, float* __restrict__ part_ml, int KVH, int BS,
    int max_parts, float scale) {
  constexpr int LPT = D / 8;         // lanes per token row (16 for D=128)
  constexpr int TPW = 64 / LPT;      // tokens per wave per step (4)
  constexpr int GROUPS = 4 * TPW;    // token groups per block (16)
  __shared__ float logits[G][kPart];
  __shared__ float red[G][8];
  __shared__ float accs[4][G][D];  // per-wave partial P.V (16 KB for D=128, G=8)

  const int part = blockIdx.x, kvh = blockIdx.y, seq = blockIdx.z;
  const int ctx = ctx_lens[seq];
  const int t0 = part * kPart;
  if (t0 >= ctx) return;
  const int t1 = min(ctx, t0 + kPart);
  const int n = t1 - t0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sub = lane % LPT, grp = wave * TPW + lane / LPT;
  const int H = KVH * G;
  const int* bt = block_tables + (size_t)seq * max_blocks;

  // query fragments (fp32, pre-scaled): lane holds dims [8*sub, 8*sub+8) of each of the G heads
  float qf[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    load8(q + (size_t)seq * q_stride + (size_t)(kvh * G + g) * D + sub * 8, qf[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[g][j] *= scale;
  }

  // ---- pass 1: logits
  float mloc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) mloc[g] = -INFINITY;
  for (int base = 0; base < n; base += 4 * GROUPS) {
    float kv[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // issue 4 row loads before the math
      const int i = base + u * GROUPS + grp;
      if (i < n) {
        const int t = t0 + i;
        load8(kc + (((size_t)bt[t / BS] * KVH + kvh) * BS + (t % BS)) * D + sub * 8, kv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + u * GROUPS + grp;
      float s[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) a = __builtin_fmaf(qf[g][j], kv[u][j], a);
#pragma unroll
        for (int o = LPT / 2; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        s[g] = a;
        if (i < n) mloc[g] = fmaxf(mloc[g], a);
      }
      if (sub == 0 && i < n) {
#pragma unroll
        for (int g = 0; g < G; ++g) logits[g][i] = s[g];
      }
    }
  }
  // block max per head
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float m = wave_max(mloc[g]);
    if (lane == 0) red[g][wave] = m;
  }
  __syncthreads();
  float mx[G];
#pragma unroll
  for (int g = 0; g < G; ++g) mx[g] = fmaxf(fmaxf(red[g][0], red[g][1]), fmaxf(red[g][2], red[g][3]));
  __syncthreads();
  // ---- pass 2: p = exp(s - max), sums
  float lsum[G];
#pragma unroll
  for (int g = 0; g < G; ++g) lsum[g] = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float p = __expf(logits[g][i] - mx[g]);
      logits[g][i] = p;
      lsum[g] += p;
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float s = wave_sum(lsum[g]);
    if (lane == 0) red[g][4 + wave] = s;
  }
  __syncthreads();
  float l[G];
#pragma unroll
  for (int g = 0; g < G; ++g) l[g] = (red[g][4] + red[g][5]) + (red[g][6] + red[g][7]);

  // ---- pass 3: P.V
  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  for (int base = 0; base < n; base += 4 * GROUPS) {
    float vv[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + u * GROUPS + grp;
      if (i < n) {
        const int t = t0 + i;
        load8(vc + (((size_t)bt[t / BS] * KVH + kvh) * BS + (t % BS)) * D + sub * 8, vv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + u * GROUPS + grp;
      if (i < n) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float p = logits[g][i];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[g][j] = __builtin_fmaf(p, vv[u][j], acc[g][j]);
        }
      }
    }
  }
  // merge the wave's TPW token groups (lanes with equal `sub`) with xor-shuffles
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = acc[g][j];
#pragma unroll
      for (int o = LPT; o < 64; o <<= 1) a += __shfl_xor(a, o, 64);
      acc[g][j] = a;
    }
  if (lane < LPT) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) accs[wave][g][sub * 8 + j] = acc[g][j];
  }
  __syncthreads();
  const int nparts = (ctx + kPart - 1) / kPart;
  for (int e = threadIdx.x; e < G * D; e += 256) {
    const int g = e / D, d = e % D;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += accs[k][g][d];
    const int hh = kvh * G + g;
    if (nparts == 1) {
      out[((size_t)seq * H + hh) * D + d] = (bf16)(s / l[g]);
    } else {
      part_acc[(((size_t)seq * H + hh) * max_parts + part) * D + d] = s;
      if (d == 0) {
        part_ml[(((size_t)seq * H + hh) * max_parts + part) * 2 + 0] = mx[g];
        part_ml[(((size_t)seq * H + hh) * max_parts + part) * 2 + 1] = l[g];
      }
    }
  }
}

// one block (D threads) per (seq, head): merge the partitions' partial results
template <int D>
__global__ void paged_reduce_kernel(const float* __restrict__ part_acc, const float* __restrict__ part_ml,
                                    const int* __restrict__ ctx_lens, bf16* __restrict__ out, int H,
                                    int max_parts) {
  const int seq = blockIdx.y, hh = blockIdx.x, d = threadIdx.x;
  const int nparts = (ctx_lens[seq] + kPart - 1) / kPart;
  if (nparts <= 1) return;
  const float* ml = part_ml + ((size_t)seq * H + hh) * max_parts * 2;
  float M = -INFINITY;
  for (int p = 0; p < nparts; ++p) M = fmaxf(M, ml[2 * p]);
  float num = 0.f, den = 0.f;
  const float* pa = part_acc + ((size_t)seq * H + hh) * max_parts * D;
  for (int p = 0; p < nparts; ++p) {
    const float w = __expf(ml[2 * p] - M);
    num += w * pa[(size_t)p * D + d];
    den += w * ml[2 * p + 1];
  }
  out[((size_t)seq * H + hh) * D + d] = (bf16)(num / den);
}

int paged_max_parts(int max_ctx) { return (max_ctx + kPart - 1) / kPart; }

bool paged_decode_launch(const bf16* q, int q_stride, const bf16* kc, const bf16* vc, const int* block_tables,
                         int max_blocks, const int* ctx_lens, bf16* out, float* part_acc, float* part_ml,
                         int B, int H, int KVH, int D, int BS, int max_ctx, float scale, hipStream_t st) {
  const int G = H / KVH;
  const int mp = paged_max_parts(max_ctx);
  dim3 grid(mp, KVH, B), block(256);
#define PD_CASE(DD, GG)                                                                                    \
  if (D == DD && G == GG) {                                                                               \
    hipLaunchKernelGGL((paged_decode_kernel<DD, GG>), grid, block, 0, st, q, q_stride, kc, vc, block_tables, \
                       max_blocks, ctx_lens, out, part_acc, part_ml, KVH, BS, mp, scale);                  \
    if (mp > 1) hipLaunchKernelGGL((paged_reduce_kernel<DD>), dim3(H, B), dim3(DD), 0, st, part_acc, part_ml, \
                                   ctx_lens, out, H, mp);                                                  \
    return true;                                                                                          \
  }
  PD_CASE(128, 1) PD_CASE(128, 2) PD_CASE(128, 4) PD_CASE(128, 8)
  PD_CASE(64, 1) PD_CASE(64, 2) PD_CASE(64, 4) PD_CASE(64, 8)
#undef PD_CASE
  return false;
}

}  // namespace caamd
