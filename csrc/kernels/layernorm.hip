// LayerNorm forward/backward for bf16 activations on gfx950, with optional
// fused residual add (s = x + r; y = LN(s)) — the GPT-2 pre-LN block pattern.
//
// Mapping: one 64-lane wave owns one row; each lane holds NV chunks of 8
// contiguous bf16 (16-byte loads), so a row of D <= 512*NV stays in VGPRs
// between the mean, variance and normalise passes (one HBM read, one write).
// Statistics in fp32. 4 waves (256 threads) per block.
//
// Backward: dx = rstd * (g*dy - mean(g*dy) - xhat*mean(g*dy*xhat)) [+ dres];
// dgamma/dbeta are accumulated per lane in registers over the rows a wave
// visits, merged across the block's 4 waves with LDS float atomics, written
// as one fp32 partial row per block, then summed by a column-reduce kernel.
#include "common.h"

namespace caamd {

// backward kernel selection (ln_bwd_config): 0 = one row per wave, 1 = prefetching,
// 2 = column-split, 4 rows per iteration; 3 = column-split, 2 rows (default where it
// applies: D <= 2048; 97.9 vs 142.5 us at 32k x 1600, tools/bench_ln_bwd.py)
static int g_ln_bwd_variant = 3;
static int g_ln_bwd_blocks = 0;  // 0 = default grid cap

template <int NV, bool HAS_RES>
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ r, bf16* __restrict__ s_out,
    const bf16* __restrict__ g, const bf16* __restrict__ b, bf16* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int rows, int D, float eps) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int nchunk = D >> 3;
  const size_t base = (size_t)row * D;
  float v[NV][8];
  float sum = 0.f;
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
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[c][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
  const float inv_d = 1.f / (float)D;
  const float mu = wave_sum(sum) * inv_d;
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = lane + c * 64;
    if (ch < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[c][j] - mu;
        sq += d * d;
      }
    }
  }
  const float rs = rsqrtf(wave_sum(sq) * inv_d + eps);
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = lane + c * 64;
    if (ch < nchunk) {
      float gg[8], bb[8], o[8];
      load8(g + ch * 8, gg);
      load8(b + ch * 8, bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mu) * rs * gg[j] + bb[j];
      store8(y + base + ch * 8, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rs;
  }
}

__device__ __forceinline__ void opt_barrier(bf16x8& a, bf16x8& b) {
  asm volatile("" : "+v"(a), "+v"(b));
}

// Backward in ONE HBM pass. A wave owns one row per iteration (x / dy chunks
// as packed bf16 in VGPRs between the statistics and the dx pass; dres loaded
// after pass 1, its latency overlapping the cross-lane reduction) and
// accumulates dgamma / dbeta of its columns in fp32 registers across all rows
// it visits; the 4 waves of a block merge them with LDS float atomics ONCE at
// the end (per-row LDS atomics from 4 waves on the same addresses serialize in
// the LDS and cost ~0.5 ms per call at 32k x 1600). One fp32 partial row per
// block, summed by colsum_bf16_kernel. ~170 VGPRs -> 2-3 waves per SIMD (the
// earlier two-rows-per-wave variant needed 314 = 1 wave per SIMD).
template <int NV, bool HAS_DRES>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const bf16* __restrict__ dy, const bf16* __restrict__ x, const bf16* __restrict__ g,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16* __restrict__ dres, bf16* __restrict__ dx, float* __restrict__ partial,
    int rows, int D) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2D] dgamma | dbeta
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nchunk = D >> 3;
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) red[i] = 0.f;
  float dg[NV][8], db[NV][8];
#pragma unroll
  for (int c = 0; c < NV; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[c][j] = db[c][j] = 0.f;
  const float inv_d = 1.f / (float)D;
  const int stride = gridDim.x * 4;
  for (int r = blockIdx.x * 4 + wave; r < rows; r += stride) {
    const size_t base = (size_t)r * D;
    bf16x8 xv[NV], dv[NV], rv[NV];
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        xv[c] = *reinterpret_cast<const bf16x8*>(x + base + ch * 8);
        dv[c] = *reinterpret_cast<const bf16x8*>(dy + base + ch * 8);
      }
    }
    const float mu = mean[r], rs = rstd[r];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + ch * 8);  // L1/L2-resident
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (float)dv[c][j], xh = ((float)xv[c][j] - mu) * rs;
          const float gd = d * (float)gv[j];
          s1 += gd;
          s2 += gd * xh;
        }
      }
    }
    if (HAS_DRES) {
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        const int ch = lane + c * 64;
        if (ch < nchunk) rv[c] = *reinterpret_cast<const bf16x8*>(dres + base + ch * 8);
      }
    }
    // Optimisation barrier: the fp32 unpacks of x / dy are recomputed in pass 2
    // instead of being CSE'd and held live across the reduction (dgamma / dbeta
    // accumulate in pass 2): 242 -> fewer VGPRs, more waves per SIMD.
#pragma unroll
    for (int c = 0; c < NV; ++c) opt_barrier(xv[c], dv[c]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    const float m1 = s1 * inv_d, m2 = s2 * inv_d;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + ch * 8);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = ((float)xv[c][j] - mu) * rs, d = (float)dv[c][j];
          dg[c][j] += d * xh;
          db[c][j] += d;
          float v = rs * (d * (float)gv[j] - m1 - xh * m2);
          if (HAS_DRES) v += (float)rv[c][j];
          o[j] = (bf16)v;
        }
        *reinterpret_cast<bf16x8*>(dx + base + ch * 8) = o;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = lane + c * 64;
    if (ch < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&red[ch * 8 + j], dg[c][j]);
        atomicAdd(&red[D + ch * 8 + j], db[c][j]);
      }
    }
  }
  __syncthreads();
  float* out = partial + (size_t)blockIdx.x * 2 * D;
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) out[i] = red[i];
}

// Software-pipelined variant: the next row's x / dy / dres loads are issued
// before the current row is reduced and written, so every wave keeps two rows
// of HBM traffic in flight (the one-row loop above exposes the full load
// latency once per row).
template <int NV, bool HAS_DRES>
__global__ __launch_bounds__(256) void ln_bwd_pf_kernel(
    const bf16* __restrict__ dy, const bf16* __restrict__ x, const bf16* __restrict__ g,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16* __restrict__ dres, bf16* __restrict__ dx, float* __restrict__ partial,
    int rows, int D) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2D] dgamma | dbeta
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nchunk = D >> 3;
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) red[i] = 0.f;
  float dg[NV][8], db[NV][8];
#pragma unroll
  for (int c = 0; c < NV; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[c][j] = db[c][j] = 0.f;
  const float inv_d = 1.f / (float)D;
  const int stride = gridDim.x * 4;
  bf16x8 xv[NV], dv[NV], rv[NV];
  float mu = 0.f, rs = 0.f;
  int r = blockIdx.x * 4 + wave;
  auto load_row = [&](int rr, bf16x8* X, bf16x8* Dv, bf16x8* R, float& m, float& s) {
    const size_t base = (size_t)rr * D;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        X[c] = *reinterpret_cast<const bf16x8*>(x + base + ch * 8);
        Dv[c] = *reinterpret_cast<const bf16x8*>(dy + base + ch * 8);
        if (HAS_DRES) R[c] = *reinterpret_cast<const bf16x8*>(dres + base + ch * 8);
      }
    }
    m = mean[rr];
    s = rstd[rr];
  };
  if (r < rows) load_row(r, xv, dv, rv, mu, rs);
  for (; r < rows; r += stride) {
    bf16x8 xn[NV], dn[NV], rn[NV];
    float mun = 0.f, rsn = 0.f;
    const int nxt = r + stride;
    if (nxt < rows) load_row(nxt, xn, dn, rn, mun, rsn);
    const size_t base = (size_t)r * D;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + ch * 8);  // L1/L2-resident
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (float)dv[c][j], xh = ((float)xv[c][j] - mu) * rs;
          const float gd = d * (float)gv[j];
          s1 += gd;
          s2 += gd * xh;
          dg[c][j] += d * xh;
          db[c][j] += d;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    const float m1 = s1 * inv_d, m2 = s2 * inv_d;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + ch * 8);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = ((float)xv[c][j] - mu) * rs;
          float v = rs * ((float)dv[c][j] * (float)gv[j] - m1 - xh * m2);
          if (HAS_DRES) v += (float)rv[c][j];
          o[j] = (bf16)v;
        }
        *reinterpret_cast<bf16x8*>(dx + base + ch * 8) = o;
      }
    }
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      xv[c] = xn[c];
      dv[c] = dn[c];
      if (HAS_DRES) rv[c] = rn[c];
    }
    mu = mun;
    rs = rsn;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = lane + c * 64;
    if (ch < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&red[ch * 8 + j], dg[c][j]);
        atomicAdd(&red[D + ch * 8 + j], db[c][j]);
      }
    }
  }
  __syncthreads();
  float* out = partial + (size_t)blockIdx.x * 2 * D;
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) out[i] = red[i];
}

// Column-split backward (variant 2, the default for D <= 2048): the 4 waves of a block
// share each row, wave w owning the column chunks [w*CPW, (w+1)*CPW) (CPW <= 64), so a
// lane holds ONE 16-byte chunk of x / dy / dres per row and 16 fp32 dgamma / dbeta
// accumulators (the one-row-per-wave kernels above hold 4 chunks and 64 accumulators:
// 168 VGPRs, 3 waves per SIMD, 2.9 TB/s). RB rows per iteration keep RB x 3 loads in
// flight per lane; the per-row sums of gd and gd*xhat are combined across the 4 waves
// through LDS (parity double-buffered: one barrier per RB rows). Waves own disjoint
// columns, so each block writes its dgamma / dbeta partial row without atomics.
// DXS: also the column sums of dx (the bias gradient of the layer whose output was
// the residual branch), as a third partial row section [2D, 3D).
template <int RB, bool HAS_DRES, bool DXS = false>
__global__ __launch_bounds__(256) void ln_bwd_cs_kernel(
    const bf16* __restrict__ dy, const bf16* __restrict__ x, const bf16* __restrict__ g,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16* __restrict__ dres, bf16* __restrict__ dx, float* __restrict__ partial,
    int rows, int D) {
  __shared__ float red[2][RB][4][2];  // [parity][row][wave][s1 | s2]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nchunk = D >> 3;
  const int cpw = (nchunk + 3) >> 2;
  const int ch = wave * cpw + lane;
  const bool act = lane < cpw && ch < nchunk;
  float gv[8], dg[8], db[8], dxs[8];
  {
    bf16x8 t = act ? *reinterpret_cast<const bf16x8*>(g + ch * 8) : bf16x8{};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      gv[j] = (float)t[j];
      dg[j] = db[j] = dxs[j] = 0.f;
    }
  }
  const float inv_d = 1.f / (float)D;
  const int ngroups = (rows + RB - 1) / RB;
  int parity = 0;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x, parity ^= 1) {
    const int r0 = grp * RB;
    bf16x8 xv[RB], dv[RB], rv[RB];
    float mu[RB], rs[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int r = r0 + i;
      const bool ok = act && r < rows;
      const size_t off = (size_t)r * D + ch * 8;
      xv[i] = ok ? *reinterpret_cast<const bf16x8*>(x + off) : bf16x8{};
      dv[i] = ok ? *reinterpret_cast<const bf16x8*>(dy + off) : bf16x8{};
      if (HAS_DRES) rv[i] = ok ? *reinterpret_cast<const bf16x8*>(dres + off) : bf16x8{};
      mu[i] = r < rows ? mean[r] : 0.f;
      rs[i] = r < rows ? rstd[r] : 0.f;
    }
    float s1[RB], s2[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (float)dv[i][j], xh = ((float)xv[i][j] - mu[i]) * rs[i];
        const float gd = d * gv[j];
        a += gd;
        b += gd * xh;
        dg[j] += d * xh;
        db[j] += d;
      }
      s1[i] = a;
      s2[i] = b;
    }
    // packed bf16 stays live across the reduction; the fp32 unpacks are redone in the
    // dx pass (keeps the wave near 100 VGPRs instead of holding 3 x RB x 8 floats)
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      opt_barrier(xv[i], dv[i]);
      if (HAS_DRES) asm volatile("" : "+v"(rv[i]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        s1[i] += __shfl_xor(s1[i], o, 64);
        s2[i] += __shfl_xor(s2[i], o, 64);
      }
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        red[parity][i][wave][0] = s1[i];
        red[parity][i][wave][1] = s2[i];
      }
    }
    __syncthreads();  // the other parity's slots are free again for the next group
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const float m1 = (red[parity][i][0][0] + red[parity][i][1][0] + red[parity][i][2][0] + red[parity][i][3][0]) * inv_d;
      const float m2 = (red[parity][i][0][1] + red[parity][i][1][1] + red[parity][i][2][1] + red[parity][i][3][1]) * inv_d;
      const int r = r0 + i;
      if (act && r < rows) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = ((float)xv[i][j] - mu[i]) * rs[i];
          float v = rs[i] * ((float)dv[i][j] * gv[j] - m1 - xh * m2);
          if (HAS_DRES) v += (float)rv[i][j];
          o[j] = (bf16)v;
          if (DXS) dxs[j] += (float)o[j];
        }
        *reinterpret_cast<bf16x8*>(dx + (size_t)r * D + ch * 8) = o;
      }
    }
  }
  if (act) {
    float* out = partial + (size_t)blockIdx.x * (DXS ? 3 : 2) * D + ch * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      out[j] = dg[j];
      out[D + j] = db[j];
      if (DXS) out[2 * D + j] = dxs[j];
    }
  }
}

// Column sum of an fp32 [nrow, ncol] slab -> bf16, split at column `split`
// (columns < split -> o0[c], the rest -> o1[c - split]). One block = 64 columns
// x 16 waves; wave w sums rows w, w+16, ... with 8 loads in flight; LDS merge.
__global__ __launch_bounds__(1024) void colsum_bf16_kernel(const float* __restrict__ partial,
                                                           int nrow, int ncol, int ld, int split,
                                                           bf16* __restrict__ o0,
                                                           bf16* __restrict__ o1, int accumulate) {
  __shared__ float red[16][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (c < ncol) {
    int r = wave;
    for (; r + 7 * 16 < nrow; r += 8 * 16) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = partial[(size_t)(r + u * 16) * ld + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += t[u];
    }
    for (; r < nrow; r += 16) acc += partial[(size_t)r * ld + c];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < ncol) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) s += red[w][lane];
    bf16* dst = c < split ? o0 + c : o1 + (c - split);
    if (accumulate) s += (float)*dst;  // accumulate into an existing (main) gradient
    *dst = (bf16)s;
  }
}

void colsum_bf16_launch_ld(const float* partial, int nrow, int ncol, int ld, int split, bf16* o0, bf16* o1,
                           hipStream_t st, int accumulate) {
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3((ncol + 63) / 64), dim3(1024), 0, st, partial, nrow,
                     ncol, ld, split, o0, o1, accumulate);
}

void colsum_bf16_launch(const float* partial, int nrow, int ncol, int split, bf16* o0, bf16* o1,
                        hipStream_t st, int accumulate) {
  colsum_bf16_launch_ld(partial, nrow, ncol, ncol, split, o0, o1, st, accumulate);
}

// The three column sums of the column-split LayerNorm backward in one launch:
// partial [nrow][3D] -> dg = cols [0, D), db = [D, 2D) (overwritten, or accumulated into
// the LayerNorm's own main-grads with acc_gb), dxsum = [2D, 3D) (accumulated into the
// residual producer's bias main-grad). Two launches before.
__global__ __launch_bounds__(1024) void colsum3_bf16_kernel(const float* __restrict__ partial, int nrow, int D,
                                                            bf16* __restrict__ dg, bf16* __restrict__ db,
                                                            bf16* __restrict__ dxsum, int acc_gb) {
  __shared__ float red[16][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ncol = 3 * D;
  const int c = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (c < ncol) {
    int r = wave;
    for (; r + 7 * 16 < nrow; r += 8 * 16) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = partial[(size_t)(r + u * 16) * ncol + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += t[u];
    }
    for (; r < nrow; r += 16) acc += partial[(size_t)r * ncol + c];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < ncol) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) s += red[w][lane];
    if (c < D) dg[c] = (bf16)(acc_gb ? s + (float)dg[c] : s);
    else if (c < 2 * D) db[c - D] = (bf16)(acc_gb ? s + (float)db[c - D] : s);
    else dxsum[c - 2 * D] = (bf16)(s + (float)dxsum[c - 2 * D]);
  }
}

template <int NV>
static void ln_fwd_dispatch(const bf16* x, const bf16* r, bf16* s, const bf16* g, const bf16* b,
                            bf16* y, float* mean, float* rstd, int rows, int D, float eps,
                            hipStream_t st) {
  dim3 grid((rows + 3) / 4), block(256);
  if (r)
    hipLaunchKernelGGL((ln_fwd_kernel<NV, true>), grid, block, 0, st, x, r, s, g, b, y, mean, rstd,
                       rows, D, eps);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<NV, false>), grid, block, 0, st, x, r, s, g, b, y, mean,
                       rstd, rows, D, eps);
}

template <int NV>
static void ln_bwd_dispatch(const bf16* dy, const bf16* x, const bf16* g, const float* mean,
                            const float* rstd, const bf16* dres, bf16* dx, float* partial,
                            int nblk, int rows, int D, hipStream_t st) {
  dim3 grid(nblk), block(256);
  size_t lds = (size_t)2 * D * sizeof(float);
  if (g_ln_bwd_variant == 1) {
    if (dres)
      hipLaunchKernelGGL((ln_bwd_pf_kernel<NV, true>), grid, block, lds, st, dy, x, g, mean, rstd,
                         dres, dx, partial, rows, D);
    else
      hipLaunchKernelGGL((ln_bwd_pf_kernel<NV, false>), grid, block, lds, st, dy, x, g, mean, rstd,
                         dres, dx, partial, rows, D);
    return;
  }
  if (dres)
    hipLaunchKernelGGL((ln_bwd_kernel<NV, true>), grid, block, lds, st, dy, x, g, mean, rstd, dres,
                       dx, partial, rows, D);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<NV, false>), grid, block, lds, st, dy, x, g, mean, rstd,
                       dres, dx, partial, rows, D);
}

int ln_nv_for(int D) {
  const int need = (D + 511) / 512;
  if (need <= 1) return 1;
  if (need <= 2) return 2;
  if (need <= 4) return 4;
  if (need <= 8) return 8;
  return -1;
}

int ln_bwd_num_blocks(int rows) {
  // 768 blocks = 3 per CU (the VGPR-limited residency), >= 8 rows per block
  const int cap = g_ln_bwd_blocks > 0 ? g_ln_bwd_blocks : 768;
  int nb = (rows + 7) / 8;
  return nb < cap ? nb : cap;
}

void ln_bwd_config(int variant, int max_blocks) {
  g_ln_bwd_variant = variant;
  g_ln_bwd_blocks = max_blocks;
}

void ln_fwd_launch(const bf16* x, const bf16* r, bf16* s, const bf16* g, const bf16* b, bf16* y,
                   float* mean, float* rstd, int rows, int D, float eps, hipStream_t st) {
  switch (ln_nv_for(D)) {
    case 1: ln_fwd_dispatch<1>(x, r, s, g, b, y, mean, rstd, rows, D, eps, st); break;
    case 2: ln_fwd_dispatch<2>(x, r, s, g, b, y, mean, rstd, rows, D, eps, st); break;
    case 4: ln_fwd_dispatch<4>(x, r, s, g, b, y, mean, rstd, rows, D, eps, st); break;
    case 8: ln_fwd_dispatch<8>(x, r, s, g, b, y, mean, rstd, rows, D, eps, st); break;
  }
}

constexpr int LN_CS_RB = 4;

int ln_bwd_cs_blocks(int rows) {
  // 1024: every block resident at once (4 per CU at ~100 VGPRs; 2048 blocks ran 1.6
  // rounds) and half the partial rows for colsum3: 96 vs 106-113 us standalone in the
  // step form, step 101.1k / 101.0k vs 100.9k / 100.5k (profiles/ln_bwd_dxsum_r6.jsonl,
  // profiles/step_ab_ln_bwd_cap_r6.txt)
  const int cap = g_ln_bwd_blocks > 0 ? g_ln_bwd_blocks : 1024;
  const int ng = (rows + LN_CS_RB - 1) / LN_CS_RB;
  return ng < cap ? ng : cap;
}

static bool ln_bwd_cs_ok(int D) { return (g_ln_bwd_variant == 2 || g_ln_bwd_variant == 3) && D <= 2048 && D % 8 == 0; }

// partial slab rows the backward writes (the caller sizes `partial` as [rows][2D])
int ln_bwd_partial_rows(int rows, int D) {
  return ln_bwd_cs_ok(D) ? ln_bwd_cs_blocks(rows) : ln_bwd_num_blocks(rows);
}

bool ln_bwd_dxsum_ok(int D) { return ln_bwd_cs_ok(D); }

// dxsum (optional, cs path only; partial sized [rows][3D] then): bf16 vector += the
// column sums of dx (accumulated into an existing main gradient). acc_gb: dg / db are
// the LayerNorm's main-grad views and take += (no separate accumulate launch per tensor).
void ln_bwd_launch(const bf16* dy, const bf16* x, const bf16* g, const float* mean,
                   const float* rstd, const bf16* dres, bf16* dx, float* partial, bf16* dg,
                   bf16* db, int rows, int D, hipStream_t st, bf16* dxsum, int acc_gb) {
  if (dxsum && ln_bwd_cs_ok(D)) {
    const int nb = ln_bwd_cs_blocks(rows);
    // variant 2: four rows per iteration (more loads in flight), variant 3 (default): two
    if (dres && g_ln_bwd_variant == 2)
      hipLaunchKernelGGL((ln_bwd_cs_kernel<LN_CS_RB, true, true>), dim3(nb), dim3(256), 0, st, dy, x, g, mean, rstd,
                         dres, dx, partial, rows, D);
    else if (dres)
      hipLaunchKernelGGL((ln_bwd_cs_kernel<2, true, true>), dim3(nb), dim3(256), 0, st, dy, x, g, mean, rstd, dres,
                         dx, partial, rows, D);
    else
      hipLaunchKernelGGL((ln_bwd_cs_kernel<2, false, true>), dim3(nb), dim3(256), 0, st, dy, x, g, mean, rstd,
                         dres, dx, partial, rows, D);
    hipLaunchKernelGGL(colsum3_bf16_kernel, dim3((3 * D + 63) / 64), dim3(1024), 0, st, partial, nb, D, dg, db,
                       dxsum, acc_gb);
    return;
  }
  if (ln_bwd_cs_ok(D)) {
    const int nb = ln_bwd_cs_blocks(rows);
    if (g_ln_bwd_variant == 3) {  // two rows per iteration (fewer VGPRs, more waves)
      if (dres)
        hipLaunchKernelGGL((ln_bwd_cs_kernel<2, true>), dim3(nb), dim3(256), 0, st, dy, x, g, mean, rstd, dres,
                           dx, partial, rows, D);
      else
        hipLaunchKernelGGL((ln_bwd_cs_kernel<2, false>), dim3(nb), dim3(256), 0, st, dy, x, g, mean, rstd, dres,
                           dx, partial, rows, D);
      colsum_bf16_launch(partial, nb, 2 * D, D, dg, db, st, acc_gb);
      return;
    }
    if (dres)
      hipLaunchKernelGGL((ln_bwd_cs_kernel<LN_CS_RB, true>), dim3(nb), dim3(256), 0, st, dy, x, g, mean, rstd,
                         dres, dx, partial, rows, D);
    else
      hipLaunchKernelGGL((ln_bwd_cs_kernel<LN_CS_RB, false>), dim3(nb), dim3(256), 0, st, dy, x, g, mean, rstd,
                         dres, dx, partial, rows, D);
    colsum_bf16_launch(partial, nb, 2 * D, D, dg, db, st, acc_gb);
    return;
  }
  const int nblk = ln_bwd_num_blocks(rows);
  switch (ln_nv_for(D)) {
    case 1: ln_bwd_dispatch<1>(dy, x, g, mean, rstd, dres, dx, partial, nblk, rows, D, st); break;
    case 2: ln_bwd_dispatch<2>(dy, x, g, mean, rstd, dres, dx, partial, nblk, rows, D, st); break;
    case 4: ln_bwd_dispatch<4>(dy, x, g, mean, rstd, dres, dx, partial, nblk, rows, D, st); break;
    case 8: ln_bwd_dispatch<8>(dy, x, g, mean, rstd, dres, dx, partial, nblk, rows, D, st); break;
  }
  colsum_bf16_launch(partial, nblk, 2 * D, D, dg, db, st, acc_gb);
}

}  // namespace caamd
