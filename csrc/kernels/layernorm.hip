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

// Backward in ONE HBM pass: a wave owns TWO rows at a time (two independent
// load -> cross-lane-reduction -> store chains hide each other's latency), keeps
// both rows' x and dy as packed bf16 in VGPRs between the statistics and the dx
// pass, and accumulates dgamma/dbeta of its columns in fp32 registers across
// the rows it visits (merged per block with LDS atomics at the end).
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
  bf16x8 gv[NV];
  float dg[NV][8], db[NV][8];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = lane + c * 64;
    if (ch < nchunk) gv[c] = *reinterpret_cast<const bf16x8*>(g + ch * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (ch >= nchunk) gv[c][j] = (bf16)0.f;
      dg[c][j] = db[c][j] = 0.f;
    }
  }
  const float inv_d = 1.f / (float)D;
  const int stride = gridDim.x * 4;
  for (int r0 = blockIdx.x * 4 + wave; r0 < rows; r0 += 2 * stride) {
    const int r1 = r0 + stride;
    const bool v1 = r1 < rows;
    const size_t b0 = (size_t)r0 * D, b1 = (size_t)(v1 ? r1 : r0) * D;
    bf16x8 xa[NV], da[NV], xb[NV], dbb[NV];
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        xa[c] = *reinterpret_cast<const bf16x8*>(x + b0 + ch * 8);
        da[c] = *reinterpret_cast<const bf16x8*>(dy + b0 + ch * 8);
        xb[c] = *reinterpret_cast<const bf16x8*>(x + b1 + ch * 8);
        dbb[c] = *reinterpret_cast<const bf16x8*>(dy + b1 + ch * 8);
      }
    }
    const float mua = mean[r0], rsa = rstd[r0];
    const float mub = mean[v1 ? r1 : r0], rsb = rstd[v1 ? r1 : r0];
    float s1a = 0.f, s2a = 0.f, s1b = 0.f, s2b = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gj = (float)gv[c][j];
          const float dva = (float)da[c][j], xha = ((float)xa[c][j] - mua) * rsa;
          const float dvb = v1 ? (float)dbb[c][j] : 0.f, xhb = ((float)xb[c][j] - mub) * rsb;
          s1a += dva * gj;
          s2a += dva * gj * xha;
          s1b += dvb * gj;
          s2b += dvb * gj * xhb;
          dg[c][j] += dva * xha + dvb * xhb;
          db[c][j] += dva + dvb;
        }
      }
    }
    s1a = wave_sum(s1a);
    s2a = wave_sum(s2a);
    s1b = wave_sum(s1b);
    s2b = wave_sum(s2b);
    const float m1a = s1a * inv_d, m2a = s2a * inv_d, m1b = s1b * inv_d, m2b = s2b * inv_d;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        float oa[8], ob[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gj = (float)gv[c][j];
          oa[j] = rsa * ((float)da[c][j] * gj - m1a - ((float)xa[c][j] - mua) * rsa * m2a);
          ob[j] = rsb * ((float)dbb[c][j] * gj - m1b - ((float)xb[c][j] - mub) * rsb * m2b);
        }
        if (HAS_DRES) {
          float ta[8], tb[8];
          load8(dres + b0 + ch * 8, ta);
          if (v1) load8(dres + b1 + ch * 8, tb);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            oa[j] += ta[j];
            if (v1) ob[j] += tb[j];
          }
        }
        store8(dx + b0 + ch * 8, oa);
        if (v1) store8(dx + b1 + ch * 8, ob);
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

// Column sum of an fp32 [nrow, ncol] slab -> bf16, split at column `split`
// (columns < split -> o0[c], the rest -> o1[c - split]). One block = 64 columns
// x 16 waves; wave w sums rows w, w+16, ... with 8 loads in flight; LDS merge.
__global__ __launch_bounds__(1024) void colsum_bf16_kernel(const float* __restrict__ partial,
                                                           int nrow, int ncol, int split,
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
    bf16* dst = c < split ? o0 + c : o1 + (c - split);
    if (accumulate) s += (float)*dst;  // accumulate into an existing (main) gradient
    *dst = (bf16)s;
  }
}

void colsum_bf16_launch(const float* partial, int nrow, int ncol, int split, bf16* o0, bf16* o1,
                        hipStream_t st, int accumulate) {
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3((ncol + 63) / 64), dim3(1024), 0, st, partial, nrow,
                     ncol, split, o0, o1, accumulate);
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
  int nb = (rows + 7) / 8;
  return nb < 512 ? nb : 512;
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

void ln_bwd_launch(const bf16* dy, const bf16* x, const bf16* g, const float* mean,
                   const float* rstd, const bf16* dres, bf16* dx, float* partial, bf16* dg,
                   bf16* db, int rows, int D, hipStream_t st) {
  const int nblk = ln_bwd_num_blocks(rows);
  switch (ln_nv_for(D)) {
    case 1: ln_bwd_dispatch<1>(dy, x, g, mean, rstd, dres, dx, partial, nblk, rows, D, st); break;
    case 2: ln_bwd_dispatch<2>(dy, x, g, mean, rstd, dres, dx, partial, nblk, rows, D, st); break;
    case 4: ln_bwd_dispatch<4>(dy, x, g, mean, rstd, dres, dx, partial, nblk, rows, D, st); break;
    case 8: ln_bwd_dispatch<8>(dy, x, g, mean, rstd, dres, dx, partial, nblk, rows, D, st); break;
  }
  colsum_bf16_launch(partial, nblk, 2 * D, D, dg, db, st, 0);
}

}  // namespace caamd
