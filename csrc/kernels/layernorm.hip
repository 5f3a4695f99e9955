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

template <int NV, bool HAS_DRES>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const bf16* __restrict__ dy, const bf16* __restrict__ x, const bf16* __restrict__ g,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16* __restrict__ dres, bf16* __restrict__ dx, float* __restrict__ partial,
    int rows, int D) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // 2*D floats
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nchunk = D >> 3;
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) red[i] = 0.f;
  float gg[NV][8], dg[NV][8], db[NV][8];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = lane + c * 64;
    if (ch < nchunk) load8(g + ch * 8, gg[c]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dg[c][j] = 0.f;
      db[c][j] = 0.f;
      if (ch >= nchunk) gg[c][j] = 0.f;
    }
  }
  const float inv_d = 1.f / (float)D;
  for (int row = blockIdx.x * 4 + wave; row < rows; row += gridDim.x * 4) {
    const size_t base = (size_t)row * D;
    const float mu = mean[row], rs = rstd[row];
    float xh[NV][8], gdy[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        float xv[8], dv[8];
        load8(x + base + ch * 8, xv);
        load8(dy + base + ch * 8, dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] = (xv[j] - mu) * rs;
          gdy[c][j] = dv[j] * gg[c][j];
          s1 += gdy[c][j];
          s2 += gdy[c][j] * xh[c][j];
          dg[c][j] += dv[j] * xh[c][j];
          db[c][j] += dv[j];
        }
      }
    }
    const float m1 = wave_sum(s1) * inv_d, m2 = wave_sum(s2) * inv_d;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int ch = lane + c * 64;
      if (ch < nchunk) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (gdy[c][j] - m1 - xh[c][j] * m2);
        if (HAS_DRES) {
          float t[8];
          load8(dres + base + ch * 8, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += t[j];
        }
        store8(dx + base + ch * 8, o);
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

// out[c] = sum_b partial[b][c] for c < ncol; written as bf16 split in two
// destination arrays (first D columns -> o0, next D -> o1).
__global__ __launch_bounds__(256) void colsum_to_bf16_kernel(
    const float* __restrict__ partial, int nblk, int D, bf16* __restrict__ o0,
    bf16* __restrict__ o1) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * D) return;
  float acc = 0.f;
  for (int b = 0; b < nblk; ++b) acc += partial[(size_t)b * 2 * D + c];
  if (c < D) o0[c] = (bf16)acc;
  else o1[c - D] = (bf16)acc;
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
  int nb = (rows + 3) / 4;
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
  hipLaunchKernelGGL(colsum_to_bf16_kernel, dim3((2 * D + 255) / 256), dim3(256), 0, st, partial,
                     nblk, D, dg, db);
}

}  // namespace caamd
