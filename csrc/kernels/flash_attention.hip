// Causal flash attention for gfx950 on MFMA (v_mfma_f32_32x32x16_bf16), bf16 I/O,
// fp32 accumulate, head_dim D in {64, 128}. Operates IN PLACE on the packed
// projection layout: qkv [B, T, 3, H, D] (exactly x @ W_qkv^T), output
// o [B, T, H, D] (exactly what the output projection consumes), gradients into a
// packed dqkv [B, T, 3, H, D] — no permute / cat copies around the kernels.
//
// Orientation ("swapped" products, cdna_hip_programming.md §3): every score tile
// is computed with the QUERY (fwd, dQ) or the KEY (dK/dV) on the MFMA lane, so
//   * the online-softmax statistics of a query are lane-local (fwd, dQ),
//   * the fp32 accumulator of P / dS is directly the B operand of the next
//     product (registers 8s..8s+7 -> k-step s), no LDS round trip,
//   * the operand that must be read "across" keys/queries (V^T, K^T, Q^T, dO^T)
//     is staged transposed in LDS with a +4-element row pad (136-byte rows:
//     conflict-free ds_read_b64), row-major tiles use a +8-element pad
//     (144/272-byte rows: conflict-free ds_read_b128).
// Kernels:
//   fa_fwd   : per 256 query rows (4 waves x 2 x 32), loop over 64-key tiles.
//   fa_bwd_dq: per 256 query rows, recompute P^T and dP^T, dQ^T += K^T dS^T,
//              also produces Delta = rowsum(dO * O) for fa_bwd_dkdv.
//   fa_bwd_dkdv: per 128 keys (4 waves x 32), loop over 64-query tiles,
//              dV^T += dO^T P, dK^T += Q^T dS (no atomics anywhere).
// Blocks are remapped so the query/key blocks of one (batch, head) run on one
// XCD (shared K/V in that XCD's L2), heaviest causal blocks first.
#include "common.h"

#include <cstdlib>

namespace caamd {

// D = 64 second-generation kernels (flash_attn_d64.hip); CAAMD_FA_V1=1 selects
// the first-generation D = 64 kernels below (A/B timing).
void fa64_fwd_launch(const bf16*, const bf16*, const bf16*, int, int, int, bf16*, float*, int, int, int, int,
                     hipStream_t);
void fa128_fwd_launch(const bf16*, const bf16*, const bf16*, int, int, int, bf16*, float*, int, int, int, int,
                      hipStream_t);
void fa64_bwd_launch(const bf16*, const bf16*, const bf16*, const float*, float*, bf16*, int, int, int, int,
                     hipStream_t, float*);
static bool fa_v1() {
  static const bool v = [] {
    const char* e = std::getenv("CAAMD_FA_V1");
    return e && e[0] == '1';
  }();
  return v;
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// raw v_exp_f32 (no denormal range fix-up: softmax probabilities that small are 0 anyway)
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// C/D layout of 32x32: reg i of lane l -> row (i&3) + 8*(i>>2) + 4*(l>>5), col l&31.
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Accumulator registers 8s..8s+7 -> bf16 B-operand fragment for k-step s.
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (bf16)x[8 * s + j];
  return f;
}

// Fragment that pairs with acc_frag(.., s): element j <-> X row 16s + 8(j>>2) + 4h + (j&3).
// `t` is a transposed LDS image [rows r][cols] with row stride `ld` (elements).
__device__ __forceinline__ bf16x8 trans_frag(const bf16* t, int ld, int r, int col0, int s, int h) {
  const bf16* p = t + r * ld + col0 + 16 * s + 4 * h;
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(p);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(p + 8);
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// Row fragment: lane (r, h) holds M[r][16s + 8h .. +7] of a row-major LDS image.
__device__ __forceinline__ bf16x8 row_frag(const bf16* m, int ld, int r, int s, int h) {
  return *reinterpret_cast<const bf16x8*>(m + r * ld + 16 * s + 8 * h);
}

// A [64 x D] tile held in registers between its global load and its LDS write
// (software pipelining: tile k+1 is loaded while tile k is computed).
// 256 threads x (D/32) 16-byte chunks; chunk c -> row c/(D/8), col 8*(c%(D/8)).
template <int D>
struct TileRegs {
  static constexpr int N = D / 32;
  bf16x8 v[N];
};

template <int D>
__device__ __forceinline__ void tile_load(TileRegs<D>& t, const bf16* __restrict__ g,
                                          size_t gstride, int row0, int T) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::N; ++i) {
    const int c = threadIdx.x + i * 256;
    const int r = c / CPR, c8 = (c % CPR) * 8;
    if (row0 + r < T) t.v[i] = *reinterpret_cast<const bf16x8*>(g + (size_t)(row0 + r) * gstride + c8);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) t.v[i][j] = (bf16)0.f;
    }
  }
}

// row-major image, ld = D + 8
template <int D>
__device__ __forceinline__ void tile_store_rows(const TileRegs<D>& t, bf16* lds) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::N; ++i) {
    const int c = threadIdx.x + i * 256;
    *reinterpret_cast<bf16x8*>(lds + (c / CPR) * (D + 8) + (c % CPR) * 8) = t.v[i];
  }
}

// transposed image [D][64 + 4]
template <int D>
__device__ __forceinline__ void tile_store_trans(const TileRegs<D>& t, bf16* lds) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::N; ++i) {
    const int c = threadIdx.x + i * 256;
    const int r = c / CPR, c8 = (c % CPR) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[(c8 + j) * 68 + r] = t.v[i][j];
  }
}

template <int D>
constexpr int rows_img() { return 64 * (D + 8); }  // elements
template <int D>
constexpr int trans_img() { return D * 68; }       // elements

// Bijective XCD-grouping remap of a 1-D block id (guide §5 "XCD swizzle").
__device__ __forceinline__ int xcd_remap(int id, int n) {
  const int xcd = id & 7, q = n >> 3, r = n & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (id >> 3);
}

// ----------------------------------------------------------------------------
// forward: one wave owns QS=2 independent 32-query sub-blocks (64 queries), so
// every K / V^T LDS fragment feeds two MFMAs and four independent accumulator
// chains hide the MFMA latency; a block (4 waves) covers 256 queries.
// ----------------------------------------------------------------------------
// query sub-blocks per wave: 2 for D=64 (fits 256 VGPRs), 1 for D=128
template <int D>
constexpr int qs_for() { return D == 64 ? 2 : 1; }
template <int D>
constexpr int qblk_for() { return 4 * 32 * qs_for<D>(); }  // queries per block (fwd, dq)

template <int D>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(const bf16* __restrict__ qp,
                                                        const bf16* __restrict__ kp,
                                                        const bf16* __restrict__ vp, int q_rs,
                                                        int kv_rs, int group,
                                                        bf16* __restrict__ out,
                                                        float* __restrict__ lse, int T, int H,
                                                        int nqb, float scale_log2, int causal) {
  constexpr int NS = D / 16;  // k-steps over head dim
  constexpr int ND = D / 32;  // 32-wide head-dim blocks of O
  constexpr int kQS = qs_for<D>(), kQBlk = qblk_for<D>();
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  constexpr int BUF = rows_img<D>() + trans_img<D>();  // {K rows, V^T}, double-buffered
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = id / nqb;
  const int qb = nqb - 1 - (id % nqb);  // heavy (late) query blocks first
  const int b = bh / H, hh = bh % H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  // q rows of stride q_rs; k/v rows of stride kv_rs, kv head = hh / group (GQA)
  const size_t rs = (size_t)q_rs, krs = (size_t)kv_rs;
  const bf16* qbase = qp + (size_t)b * T * rs + (size_t)hh * D;
  const bf16* kbase = kp + (size_t)b * T * krs + (size_t)(hh / group) * D;
  const bf16* vbase = vp + (size_t)b * T * krs + (size_t)(hh / group) * D;
  const int q0w = qb * kQBlk + wave * 32 * kQS;

  bf16x8 qf[kQS][NS];
  f32x16 o[kQS][ND];
  float m[kQS], l[kQS];
#pragma unroll
  for (int qs = 0; qs < kQS; ++qs) {
    const int q = q0w + qs * 32 + r;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (q < T) qf[qs][s] = *reinterpret_cast<const bf16x8*>(qbase + (size_t)q * rs + 16 * s + 8 * h);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qs][s][j] = (bf16)0.f;
      }
    }
#pragma unroll
    for (int d = 0; d < ND; ++d) o[qs][d] = zero16();
    m[qs] = -INFINITY;
    l[qs] = 0.f;
  }

  const int qend = min(T, qb * kQBlk + kQBlk);
  const int nkt = causal ? (qend + 63) / 64 : (T + 63) / 64;
  TileRegs<D> kr, vr;
  tile_load<D>(kr, kbase, krs, 0, T);
  tile_load<D>(vr, vbase, krs, 0, T);
  tile_store_rows<D>(kr, smem);
  tile_store_trans<D>(vr, smem + rows_img<D>());
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const bf16* k_lds = smem + (kt & 1) * BUF;
    const bf16* vt_lds = k_lds + rows_img<D>();
    const bool more = kt + 1 < nkt;
    if (more) {
      tile_load<D>(kr, kbase, krs, k0 + 64, T);
      tile_load<D>(vr, vbase, krs, k0 + 64, T);
    }
    // wave-uniform: skip tiles entirely above this wave's causal diagonal
    const bool active = !(causal && k0 > q0w + 32 * kQS - 1) && q0w < T;
    if (active) {
      const bool need_mask = (causal && k0 + 63 > q0w) || (k0 + 64 > T);
      f32x16 sacc[kQS][2];
#pragma unroll
      for (int qs = 0; qs < kQS; ++qs)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) sacc[qs][kb] = zero16();
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const bf16x8 kf = row_frag(k_lds, D + 8, kb * 32 + r, s, h);
#pragma unroll
          for (int qs = 0; qs < kQS; ++qs) sacc[qs][kb] = mfma32(kf, qf[qs][s], sacc[qs][kb]);
        }
#pragma unroll
      for (int qs = 0; qs < kQS; ++qs) {
        const int q = q0w + qs * 32 + r;
        if (need_mask) {  // branch-free selects (v_cndmask), only on diagonal / tail tiles
          const int lim = causal ? min(q, T - 1) : T - 1;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              sacc[qs][kb][i] = (k0 + kb * 32 + crow(i, h) > lim) ? -INFINITY : sacc[qs][kb][i];
        }
        float mx4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) mx4[i & 3] = fmaxf(mx4[i & 3], sacc[qs][kb][i]);
        float mx = fmaxf(fmaxf(mx4[0], mx4[1]), fmaxf(mx4[2], mx4[3]));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * scale_log2;  // scale > 0 commutes with max
        const float mnew = fmaxf(m[qs], mx);
        const float muse = mnew == -INFINITY ? 0.f : mnew;
        const float alpha = fexp2(m[qs] - muse);
        float rs4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float p = fexp2(__builtin_fmaf(sacc[qs][kb][i], scale_log2, -muse));
            sacc[qs][kb][i] = p;
            rs4[i & 3] += p;
          }
        float rsum = (rs4[0] + rs4[1]) + (rs4[2] + rs4[3]);
        rsum += __shfl_xor(rsum, 32, 64);
        l[qs] = l[qs] * alpha + rsum;
        m[qs] = mnew;
#pragma unroll
        for (int d = 0; d < ND; ++d)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[qs][d][i] *= alpha;
      }
      // O^T += V^T P^T ; each V^T fragment feeds both query sub-blocks
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 pf[kQS];
#pragma unroll
          for (int qs = 0; qs < kQS; ++qs) pf[qs] = acc_frag(sacc[qs][kb], s);
#pragma unroll
          for (int d = 0; d < ND; ++d) {
            const bf16x8 vf = trans_frag(vt_lds, 68, d * 32 + r, kb * 32, s, h);
#pragma unroll
            for (int qs = 0; qs < kQS; ++qs) o[qs][d] = mfma32(vf, pf[qs], o[qs][d]);
          }
        }
    }
    if (more) {
      bf16* nb = smem + ((kt + 1) & 1) * BUF;
      tile_store_rows<D>(kr, nb);
      tile_store_trans<D>(vr, nb + rows_img<D>());
    }
    __syncthreads();
  }
#pragma unroll
  for (int qs = 0; qs < kQS; ++qs) {
    const int q = q0w + qs * 32 + r;
    if (q < T) {
      const float inv_l = l[qs] > 0.f ? 1.f / l[qs] : 0.f;
      bf16* orow = out + ((size_t)b * T + q) * H * D + (size_t)hh * D;
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[qs][d][4 * g + j] * inv_l);
          *reinterpret_cast<bf16x4*>(orow + d * 32 + 8 * g + 4 * h) = v;
        }
      if (h == 0) lse[(size_t)bh * T + q] = (m[qs] + __log2f(l[qs])) * 0.69314718056f;
    }
  }
}

// ----------------------------------------------------------------------------
// backward: dQ (+ Delta = rowsum(dO * O)), QS=2 query sub-blocks per wave
// ----------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256, D == 64 ? 2 : 1) void fa_bwd_dq_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv, int T,
    int H, int nqb, float scale_log2, float scale, int causal) {
  constexpr int NS = D / 16, ND = D / 32;
  constexpr int kQS = qs_for<D>(), kQBlk = qblk_for<D>();
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  constexpr int BUF = 2 * rows_img<D>() + trans_img<D>();  // {K rows, V rows, K^T}
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = id / nqb;
  const int qb = nqb - 1 - (id % nqb);
  const int b = bh / H, hh = bh % H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const size_t rs = (size_t)3 * H * D, ors = (size_t)H * D;
  const bf16* qbase = qkv + (size_t)b * T * rs + (size_t)hh * D;
  const bf16* kbase = qbase + (size_t)H * D;
  const bf16* vbase = kbase + (size_t)H * D;
  const int q0w = qb * kQBlk + wave * 32 * kQS;

  bf16x8 qf[kQS][NS], df[kQS][NS];
  float dlt[kQS], lse2[kQS];
  f32x16 dq[kQS][ND];
#pragma unroll
  for (int qs = 0; qs < kQS; ++qs) {
    const int q = q0w + qs * 32 + r;
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (q < T) {
        qf[qs][s] = *reinterpret_cast<const bf16x8*>(qbase + (size_t)q * rs + 16 * s + 8 * h);
        const size_t oo = ((size_t)b * T + q) * ors + (size_t)hh * D + 16 * s + 8 * h;
        df[qs][s] = *reinterpret_cast<const bf16x8*>(dout + oo);
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(o + oo);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += (float)df[qs][s][j] * (float)ov[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qs][s][j] = df[qs][s][j] = (bf16)0.f;
      }
    }
    dsum += __shfl_xor(dsum, 32, 64);
    dlt[qs] = dsum;
    lse2[qs] = q < T ? lse[(size_t)bh * T + q] * 1.44269504089f : 0.f;
    if (q < T && h == 0) delta[(size_t)bh * T + q] = dsum;
#pragma unroll
    for (int d = 0; d < ND; ++d) dq[qs][d] = zero16();
  }

  const int qend = min(T, qb * kQBlk + kQBlk);
  const int nkt = causal ? (qend + 63) / 64 : (T + 63) / 64;
  TileRegs<D> kr, vr;
  tile_load<D>(kr, kbase, rs, 0, T);
  tile_load<D>(vr, vbase, rs, 0, T);
  tile_store_rows<D>(kr, smem);
  tile_store_rows<D>(vr, smem + rows_img<D>());
  tile_store_trans<D>(kr, smem + 2 * rows_img<D>());
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const bf16* k_lds = smem + (kt & 1) * BUF;
    const bf16* v_lds = k_lds + rows_img<D>();
    const bf16* kt_lds = k_lds + 2 * rows_img<D>();
    const bool more = kt + 1 < nkt;
    if (more) {
      tile_load<D>(kr, kbase, rs, k0 + 64, T);
      tile_load<D>(vr, vbase, rs, k0 + 64, T);
    }
    const bool active = !(causal && k0 > q0w + 32 * kQS - 1) && q0w < T;
    if (active) {
      const bool need_mask = (causal && k0 + 63 > q0w) || (k0 + 64 > T);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        f32x16 sacc[kQS], dp[kQS];
#pragma unroll
        for (int qs = 0; qs < kQS; ++qs) sacc[qs] = dp[qs] = zero16();
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bf16x8 kf = row_frag(k_lds, D + 8, kb * 32 + r, s, h);
          const bf16x8 vf = row_frag(v_lds, D + 8, kb * 32 + r, s, h);
#pragma unroll
          for (int qs = 0; qs < kQS; ++qs) {
            sacc[qs] = mfma32(kf, qf[qs][s], sacc[qs]);
            dp[qs] = mfma32(vf, df[qs][s], dp[qs]);
          }
        }
#pragma unroll
        for (int qs = 0; qs < kQS; ++qs) {
          const int q = q0w + qs * 32 + r;
          const int lim = q >= T ? -1 : (causal ? min(q, T - 1) : T - 1);
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float p = fexp2(__builtin_fmaf(sacc[qs][i], scale_log2, -lse2[qs]));
            if (need_mask) p = (k0 + kb * 32 + crow(i, h) > lim) ? 0.f : p;
            sacc[qs][i] = p * (dp[qs][i] - dlt[qs]);  // dS^T
          }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 f[kQS];
#pragma unroll
          for (int qs = 0; qs < kQS; ++qs) f[qs] = acc_frag(sacc[qs], s);
#pragma unroll
          for (int d = 0; d < ND; ++d) {
            const bf16x8 a = trans_frag(kt_lds, 68, d * 32 + r, kb * 32, s, h);
#pragma unroll
            for (int qs = 0; qs < kQS; ++qs) dq[qs][d] = mfma32(a, f[qs], dq[qs][d]);
          }
        }
      }
    }
    if (more) {
      bf16* nb = smem + ((kt + 1) & 1) * BUF;
      tile_store_rows<D>(kr, nb);
      tile_store_rows<D>(vr, nb + rows_img<D>());
      tile_store_trans<D>(kr, nb + 2 * rows_img<D>());
    }
    __syncthreads();
  }
#pragma unroll
  for (int qs = 0; qs < kQS; ++qs) {
    const int q = q0w + qs * 32 + r;
    if (q < T) {
      bf16* row = dqkv + ((size_t)b * T + q) * rs + (size_t)hh * D;
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(dq[qs][d][4 * g + j] * scale);
          *reinterpret_cast<bf16x4*>(row + d * 32 + 8 * g + 4 * h) = v;
        }
    }
  }
}

// ----------------------------------------------------------------------------
// backward: dK, dV — key on the lane; per 64-query tile both 32-query halves'
// S and dP chains are issued together (4 independent accumulators).
// ----------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256, D == 64 ? 2 : 1) void fa_bwd_dkdv_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16* __restrict__ dqkv, int T, int H, int nkb,
    float scale_log2, float scale, int causal) {
  constexpr int NS = D / 16, ND = D / 32;
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  // {Q rows, Q^T, dO rows, dO^T, lse2[64] | delta[64]}, double-buffered
  constexpr int BUF = 2 * rows_img<D>() + 2 * trans_img<D>() + 2 * 64 * 2;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = id / nkb;
  const int kb0 = id % nkb;  // early key blocks are the heavy ones under the causal mask
  const int b = bh / H, hh = bh % H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const size_t rs = (size_t)3 * H * D, ors = (size_t)H * D;
  const bf16* qbase = qkv + (size_t)b * T * rs + (size_t)hh * D;
  const bf16* kbase = qbase + (size_t)H * D;
  const bf16* vbase = kbase + (size_t)H * D;
  const bf16* dobase = dout + (size_t)b * T * ors + (size_t)hh * D;
  const int key0w = kb0 * 128 + wave * 32;
  const int key = key0w + r;
  const bool kv = key < T;

  bf16x8 kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (kv) {
      kf[s] = *reinterpret_cast<const bf16x8*>(kbase + (size_t)key * rs + 16 * s + 8 * h);
      vf[s] = *reinterpret_cast<const bf16x8*>(vbase + (size_t)key * rs + 16 * s + 8 * h);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[s][j] = vf[s][j] = (bf16)0.f;
    }
  }
  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dk[d] = dv[d] = zero16();
  const int qt0 = causal ? (kb0 * 128) / 64 : 0;
  const int nqt = (T + 63) / 64;
  TileRegs<D> qr, dr;
  float st_reg = 0.f;  // threads < 128: lse2 (t < 64) or delta (64 <= t < 128) of one query
  auto load_stats = [&](int q0) {
    if (threadIdx.x < 128) {
      const int qq = q0 + (threadIdx.x & 63);
      if (qq < T)
        st_reg = threadIdx.x < 64 ? lse[(size_t)bh * T + qq] * 1.44269504089f
                                  : delta[(size_t)bh * T + qq];
      else
        st_reg = 0.f;
    }
  };
  auto store_all = [&](bf16* buf) {
    tile_store_rows<D>(qr, buf);
    tile_store_trans<D>(qr, buf + rows_img<D>());
    tile_store_rows<D>(dr, buf + rows_img<D>() + trans_img<D>());
    tile_store_trans<D>(dr, buf + 2 * rows_img<D>() + trans_img<D>());
    if (threadIdx.x < 128)
      reinterpret_cast<float*>(buf + 2 * rows_img<D>() + 2 * trans_img<D>())[threadIdx.x] = st_reg;
  };
  if (qt0 < nqt) {
    tile_load<D>(qr, qbase, rs, qt0 * 64, T);
    tile_load<D>(dr, dobase, ors, qt0 * 64, T);
    load_stats(qt0 * 64);
    store_all(smem);
  }
  __syncthreads();
  for (int qt = qt0; qt < nqt; ++qt) {
    const int q0 = qt * 64;
    const bf16* q_lds = smem + ((qt - qt0) & 1) * BUF;
    const bf16* qt_lds = q_lds + rows_img<D>();
    const bf16* do_lds = qt_lds + trans_img<D>();
    const bf16* dot_lds = do_lds + rows_img<D>();
    const float* st_lds = reinterpret_cast<const float*>(dot_lds + trans_img<D>());
    const bool more = qt + 1 < nqt;
    if (more) {
      tile_load<D>(qr, qbase, rs, q0 + 64, T);
      tile_load<D>(dr, dobase, ors, q0 + 64, T);
      load_stats(q0 + 64);
    }
    // wave-uniform: all 64 queries of this tile are before this wave's first key
    const bool active = !(causal && q0 + 63 < key0w) && key0w < T;
    if (active) {
      const bool need_mask = (causal && q0 < key0w + 31) || (q0 + 64 > T);
      f32x16 sacc[2], dp[2];
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) sacc[qh] = dp[qh] = zero16();
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          sacc[qh] = mfma32(row_frag(q_lds, D + 8, qh * 32 + r, s, h), kf[s], sacc[qh]);
          dp[qh] = mfma32(row_frag(do_lds, D + 8, qh * 32 + r, s, h), vf[s], dp[qh]);
        }
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int qi = qh * 32 + 8 * g + 4 * h;
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(st_lds + qi);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(st_lds + 64 + qi);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 4 * g + j;
            float p = fexp2(__builtin_fmaf(sacc[qh][i], scale_log2, -l4[j]));
            if (need_mask) {
              const int qq = q0 + qi + j;
              const bool bad = (qq >= T) | (!kv) | ((causal != 0) & (key > qq));
              p = bad ? 0.f : p;
            }
            sacc[qh][i] = p;
            dp[qh][i] = p * (dp[qh][i] - d4[j]);
          }
        }
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pf = acc_frag(sacc[qh], s), sf = acc_frag(dp[qh], s);
#pragma unroll
          for (int d = 0; d < ND; ++d) {
            dv[d] = mfma32(trans_frag(dot_lds, 68, d * 32 + r, qh * 32, s, h), pf, dv[d]);
            dk[d] = mfma32(trans_frag(qt_lds, 68, d * 32 + r, qh * 32, s, h), sf, dk[d]);
          }
        }
    }
    if (more) store_all(smem + ((qt + 1 - qt0) & 1) * BUF);
    __syncthreads();
  }
  if (kv) {
    bf16* krow = dqkv + ((size_t)b * T + key) * rs + (size_t)(H + hh) * D;
    bf16* vrow = krow + (size_t)H * D;
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 a, c;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = (bf16)(dk[d][4 * g + j] * scale);
          c[j] = (bf16)dv[d][4 * g + j];
        }
        *reinterpret_cast<bf16x4*>(krow + d * 32 + 8 * g + 4 * h) = a;
        *reinterpret_cast<bf16x4*>(vrow + d * 32 + 8 * g + 4 * h) = c;
      }
  }
}

// ----------------------------------------------------------------------------
template <int D>
static size_t fwd_lds() { return 2 * (size_t)(rows_img<D>() + trans_img<D>()) * sizeof(bf16); }
template <int D>
static size_t dq_lds() { return 2 * (size_t)(2 * rows_img<D>() + trans_img<D>()) * sizeof(bf16); }
template <int D>
static size_t dkdv_lds() {
  return 2 * (size_t)(2 * rows_img<D>() + 2 * trans_img<D>() + 256) * sizeof(bf16);
}

static bool g_fa_attr_done = false;
static void fa_set_attrs() {
  if (g_fa_attr_done) return;
  // allow > 64 KiB dynamic LDS (gfx950 has 160 KiB per CU)
  hipFuncSetAttribute((const void*)fa_bwd_dkdv_kernel<128>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)dkdv_lds<128>());
  hipFuncSetAttribute((const void*)fa_bwd_dq_kernel<128>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)dq_lds<128>());
  hipFuncSetAttribute((const void*)fa_fwd_kernel<128>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)fwd_lds<128>());
  hipFuncSetAttribute((const void*)fa_bwd_dkdv_kernel<64>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)dkdv_lds<64>());
  hipFuncSetAttribute((const void*)fa_bwd_dq_kernel<64>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)dq_lds<64>());
  hipFuncSetAttribute((const void*)fa_fwd_kernel<64>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)fwd_lds<64>());
  g_fa_attr_done = true;
}

void fa_fwd_gqa_launch(const bf16* q, const bf16* k, const bf16* v, int q_rs, int kv_rs, int group,
                       bf16* out, float* lse, int B, int T, int H, int D, int causal, hipStream_t st) {
  if (D == 64 && !fa_v1()) {
    fa64_fwd_launch(q, k, v, q_rs, kv_rs, group, out, lse, B, T, H, causal, st);
    return;
  }
  if (D == 128 && !fa_v1()) {
    fa128_fwd_launch(q, k, v, q_rs, kv_rs, group, out, lse, B, T, H, causal, st);
    return;
  }
  const int qblk = D == 64 ? qblk_for<64>() : qblk_for<128>();
  const int nqb = (T + qblk - 1) / qblk;
  const float scale_log2 = 1.44269504089f / sqrtf((float)D);
  fa_set_attrs();
  dim3 grid(B * H * nqb), block(256);
  if (D == 64)
    hipLaunchKernelGGL(fa_fwd_kernel<64>, grid, block, fwd_lds<64>(), st, q, k, v, q_rs, kv_rs, group,
                       out, lse, T, H, nqb, scale_log2, causal);
  else
    hipLaunchKernelGGL(fa_fwd_kernel<128>, grid, block, fwd_lds<128>(), st, q, k, v, q_rs, kv_rs, group,
                       out, lse, T, H, nqb, scale_log2, causal);
}

void fa_fwd_launch(const bf16* qkv, bf16* out, float* lse, int B, int T, int H, int D, int causal,
                   hipStream_t st) {
  // packed [B, T, 3, H, D]: q/k/v share the row stride 3*H*D, no grouping
  fa_fwd_gqa_launch(qkv, qkv + (size_t)H * D, qkv + (size_t)2 * H * D, 3 * H * D, 3 * H * D, 1, out, lse,
                    B, T, H, D, causal, st);
}

// dbias (optional, fp32 [3*H*D], accumulated): column sums of dqkv over the tokens,
// taken in the second-generation D = 64 kernels' epilogues; returns false when the
// path taken does not produce them (the caller sums dqkv itself).
bool fa_bwd_launch(const bf16* qkv, const bf16* out, const bf16* dout, const float* lse,
                   float* delta, bf16* dqkv, int B, int T, int H, int D, int causal,
                   hipStream_t st, float* dbias) {
  if (D == 64 && !fa_v1()) {  // delta: 2 * B * H * T floats
    fa64_bwd_launch(qkv, out, dout, lse, delta, dqkv, B, T, H, causal, st, dbias);
    return true;
  }
  const int qblk = D == 64 ? qblk_for<64>() : qblk_for<128>();
  const int nqb = (T + qblk - 1) / qblk;
  const int nkb = (T + 127) / 128;
  const float scale = 1.f / sqrtf((float)D);
  const float scale_log2 = 1.44269504089f * scale;
  fa_set_attrs();
  dim3 gq(B * H * nqb), gk(B * H * nkb), block(256);
  if (D == 64) {
    hipLaunchKernelGGL(fa_bwd_dq_kernel<64>, gq, block, dq_lds<64>(), st, qkv, out, dout, lse,
                       delta, dqkv, T, H, nqb, scale_log2, scale, causal);
    hipLaunchKernelGGL(fa_bwd_dkdv_kernel<64>, gk, block, dkdv_lds<64>(), st, qkv, dout, lse,
                       delta, dqkv, T, H, nkb, scale_log2, scale, causal);
  } else {
    hipLaunchKernelGGL(fa_bwd_dq_kernel<128>, gq, block, dq_lds<128>(), st, qkv, out, dout, lse,
                       delta, dqkv, T, H, nqb, scale_log2, scale, causal);
    hipLaunchKernelGGL(fa_bwd_dkdv_kernel<128>, gk, block, dkdv_lds<128>(), st, qkv, dout, lse,
                       delta, dqkv, T, H, nkb, scale_log2, scale, causal);
  }
  return dbias == nullptr;
}

}  // namespace caamd
