// Microbenchmark: the dK/dV inner pattern on the matrix pipe, without memory.
// MODE 0: 32 MFMA 32x32x16 per iteration, 8 independent chains (pure throughput)
// MODE 1: the dK/dV half pattern x2: S/dP (2 chains x 4) -> 16 cvt_pk -> dV/dK (4 chains x 2)
// MODE 2: MODE 1 with both halves' S/dP first (software-pipelined)
// Grid: blocks of 256 threads; occupancy set by launch bounds (2 waves/SIMD at 2 blocks/CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)x[8 * s + j];
  return f;
}

template <int MODE>
__global__ __launch_bounds__(256, 2) void k(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[s][j] = (__bf16)(0.001f * (lane + s + j));
      b[s][j] = (__bf16)(0.002f * (lane - s + j));
    }
  f32x16 dv[2], dk[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) dv[0][i] = dv[1][i] = dk[0][i] = dk[1][i] = 0.f;
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
      f32x16 c[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) c[q] = z;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q) c[q] = mfma(a[r], b[(r + q) & 3], c[q]);
#pragma unroll
      for (int q = 0; q < 8; ++q) dv[q & 1] += c[q];
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x16 s = mfma(a[0], b[0], z), p = mfma(a[1], b[1], z);
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          s = mfma(a[r], b[r], s);
          p = mfma(a[(r + 1) & 3], b[(r + 2) & 3], p);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bf16x8 pf = frag(s, u), sf = frag(p, u);
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            dv[d] = mfma(a[2 * u + d], pf, dv[d]);
            dk[d] = mfma(b[2 * u + d], sf, dk[d]);
          }
        }
      }
    } else {
      f32x16 s[2], p[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        s[h] = mfma(a[0], b[h], z);
        p[h] = mfma(a[1], b[h + 1], z);
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          s[h] = mfma(a[r], b[r], s[h]);
          p[h] = mfma(a[(r + 1) & 3], b[(r + 2) & 3], p[h]);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bf16x8 pf = frag(s[h], u), sf = frag(p[h], u);
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            dv[d] = mfma(a[2 * u + d], pf, dv[d]);
            dk[d] = mfma(b[2 * u + d], sf, dk[d]);
          }
        }
    }
  }
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) t += dv[0][i] + dv[1][i] + dk[0][i] + dk[1][i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int MODE>
void run(float* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = (double)blocks * 4 * iters * 32;  // per wave 32 MFMAs per iteration
  const double per_simd = mfmas / 1024.0;
  printf("{\"mode\": %d, \"blocks\": %d, \"iters\": %d, \"ms\": %.3f, \"ns_per_mfma_per_simd\": %.3f, \"tflops\": %.1f}\n",
         MODE, blocks, iters, ms, ms * 1e6 / per_simd, mfmas * 32768.0 / (ms * 1e-3) / 1e12);
}


// MODE 3: the dK/dV block structure: 6400 blocks x 4 waves, block id%8 -> 16-2*(id%8) tiles,
// K/V fragments loaded from HBM in the prologue, dK/dV stored at the end.
template <int LD, int ST, int PERSIST>
__global__ __launch_bounds__(256, 2) void kblk(const bf16x8* __restrict__ kvbuf, float* __restrict__ out, int scale_tiles) {
  const int lane = threadIdx.x & 63;
  for (int id = blockIdx.x; id < 6400; id += PERSIST ? gridDim.x : 6400) {
  const int ntiles = (16 - 2 * (id % 8)) * scale_tiles;
  const bf16x8* src = kvbuf + ((size_t)id * 256 + threadIdx.x) * 8;
  bf16x8 a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (LD) { a[s] = src[s]; b[s] = src[4 + s]; }
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[s][j] = (__bf16)(0.001f * (lane + s + j)); b[s][j] = (__bf16)(0.002f * (lane - s + j)); }
    }
  }
  f32x16 dv[2], dk[2], z;
#pragma unroll
  for (int i = 0; i < 16; ++i) dv[0][i] = dv[1][i] = dk[0][i] = dk[1][i] = z[i] = 0.f;
  for (int it = 0; it < ntiles; ++it) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x16 s = mfma(a[0], b[0], z), p = mfma(a[1], b[1], z);
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        s = mfma(a[r], b[r], s);
        p = mfma(a[(r + 1) & 3], b[(r + 2) & 3], p);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bf16x8 pf = frag(s, u), sf = frag(p, u);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = mfma(a[2 * u + d], pf, dv[d]);
          dk[d] = mfma(b[2 * u + d], sf, dk[d]);
        }
      }
    }
  }
  float* o = out + ((size_t)id * 256 + threadIdx.x) * 64;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (ST || dv[0][i] == 12345.f) { o[i] = dv[0][i]; o[16 + i] = dv[1][i]; o[32 + i] = dk[0][i]; o[48 + i] = dk[1][i]; }
  }
  }
}

int main() {
  float* out;
  hipMalloc(&out, (size_t)6400 * 256 * 64 * sizeof(float));
  for (int blocks : {256, 512, 1024}) {
    run<0>(out, blocks, 2000);
    run<1>(out, blocks, 2000);
    run<2>(out, blocks, 2000);
  }
  bf16x8* kvb;
  hipMalloc(&kvb, (size_t)6400 * 256 * 8 * sizeof(bf16x8));
  hipMemset(kvb, 0, (size_t)6400 * 256 * 8 * sizeof(bf16x8));
  auto timek = [&](auto kern, int grid, const char* name, int sc) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, kvb, out, sc);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, kvb, out, sc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double mfmas = 6400.0 * 4 * 9 * 32 * sc;
    printf("{\"mode\": \"%s\", \"tile_scale\": %d, \"us\": %.1f, \"ideal_us_at_13.7ns\": %.1f}\n", name, sc,
           ms * 1e3, mfmas / 1024 * 13.7e-3);
  };
  for (int sc : {1, 2}) {
    timek(kblk<1, 1, 0>, 6400, "ld+st", sc);
    timek(kblk<0, 0, 0>, 6400, "none", sc);
    timek(kblk<1, 0, 0>, 6400, "ld", sc);
    timek(kblk<0, 1, 0>, 6400, "st", sc);
    timek(kblk<1, 1, 1>, 512, "ld+st persistent512", sc);
    timek(kblk<0, 0, 1>, 512, "none persistent512", sc);
  }
  hipFree(kvb);
  hipFree(out);
  return 0;
}
