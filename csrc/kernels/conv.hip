// Implicit-GEMM NHWC convolution on MFMA (gfx950) with the epilogue fused, for the
// BN-folded ResNet inference path of the Data GPU map_batches benchmark
// (models/resnet.py; BASELINE.json config 3).
//
//   Y[m, n] = act( sum_k A(m, k) * Wt[n, k] + bias[n] (+ R[m, n]) )
//   m = (img, ho, wo) output pixel (row of the NHWC output), n = output channel,
//   k = (kh * KS + kw) * Cin + ci, the weight laid out [Cout][KS][KS][Cin] (K-major,
//   zero-padded to Kp = a multiple of 32).
//
// Design (MI355X-first, /opt/skills/guides/cdna_hip_programming.md):
//  * No im2col buffer: the A tile is GATHERED straight from the NHWC input by
//    LDS-DMA (`global_load_lds_dwordx4`, one 16-byte chunk = 8 channels of one tap
//    of one output pixel per lane). Every lane keeps the (image, hi0, wi0) origin of
//    its 4 tile rows in registers; per K-step it derives (kh, kw, ci) from k and
//    points padding taps (and rows past M, and the K padding) at a 16-byte zero
//    page, so the DMA itself writes the zeros — no predicated register path.
//    Cin must be a multiple of 8 (the stem's 3 channels are padded to 8 by the
//    normalisation kernel), a power of two (shift / mask decomposition).
//  * B (weights) by LDS-DMA as K-major rows. Both images use the XOR swizzle of
//    gemm.hip's 64-byte-row K-major tiles (chunk c of row r at c ^ ((r >> 3) & 1) * 2,
//    conflict-free for the 16-row ds_read_b128 fragment reads).
//  * 3-stage LDS ring, DMA two K-steps ahead, counted `s_waitcnt vmcnt` (never a
//    full drain in the steady state), one s_barrier per K-step.
//  * v_mfma_f32_16x16x32_bf16 with the operands swapped (D = B_frag * A_frag) so
//    each lane owns 4 consecutive output channels of one pixel.
//  * Epilogue staged through LDS: acc + bias rounded to bf16 into a padded
//    [BM][BN] image, then the workgroup streams whole 16-byte channel vectors out,
//    adding the residual (bottleneck join) and applying ReLU on the way — the conv
//    output is written once and never re-read by a separate bias / add / ReLU pass.
//  * XCD-aware tile order: each XCD owns a contiguous range of (m-tile, n-tile)
//    ids with n fastest, so the n-tiles of one gathered A panel share an L2.
#include "common.h"

#include <algorithm>

namespace caamd {
namespace conv {

typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) const bf16x8 lds_cbf16x8;
typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

struct Args {
  const bf16* X;     // [N, H, W, Cin]
  const bf16* Wt;    // [Cout, Kp]
  const bf16* bias;  // [Cout]
  const bf16* R;     // [M, Cout] residual or nullptr
  bf16* Y;           // [M, Cout]
  const bf16* zero;  // 16-byte zero page (16-byte aligned)
  int H, W, lcin, Ho, Wo, stride, pad, Cout, Kp, M, tiles_n;
  int stride_w, pad_w;  // horizontal stride / padding (stride, pad: vertical)
};

constexpr int NTHR = 256;
constexpr int BKB = 64;  // bytes of one K-step row (32 bf16)
constexpr int NST = 3;

__device__ __forceinline__ int kswz(int row) { return ((row >> 3) & 1) * 2; }

__device__ __forceinline__ bf16x8 frag(const lds_char* img, int rr, int lane) {
  const int row = rr + (lane & 15);
  const int pos = (lane >> 4) ^ kswz(row);
  return *(lds_cbf16x8*)(img + row * BKB + pos * 16);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN>
struct Cfg {
  static constexpr int A_ST = BM * BKB, B_ST = BN * BKB, ST = A_ST + B_ST;
  static constexpr int AP = BM * 4 / NTHR, BP = BN * 4 / NTHR;  // 16-B DMA pieces per lane per step
  static constexpr int ROWB = BN * 2 + 16;                        // padded epilogue image row
  static constexpr int LDS = (NST * ST > BM * ROWB) ? NST * ST : BM * ROWB;
  static_assert((BM * 4) % NTHR == 0 && (BN * 4) % NTHR == 0, "tile / DMA mismatch");
};

template <int BM, int BN, int WM, int WN, int KH, int KW, bool RES, bool RELU>
__global__ __launch_bounds__(NTHR, 2) void conv_kernel(Args p) {
  using C_ = Cfg<BM, BN>;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(WM * WN == NTHR / 64 && TM * WM * 16 == BM && TN * WN * 16 == BN, "wave grid");
  constexpr int AP = C_::AP, BP = C_::BP, CNT = AP + BP;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid - (wid / WN) * WN;

  int sid;
  {
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, loc = bid >> 3, q = nwg >> 3, r = nwg & 7;
    sid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int tm = sid / p.tiles_n, tn = sid - (sid / p.tiles_n) * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-lane gather state: rows j*64 + wid*16 + lane/4 of the A tile -------------
  // (kswz of those rows only depends on lane bit 5, so the chunk is fixed per lane)
  const int c = (lane & 3) ^ (((lane >> 5) & 1) * 2);
  const int HoWo = p.Ho * p.Wo;
  int a_base[AP], a_hi[AP], a_wi[AP];
#pragma unroll
  for (int j = 0; j < AP; ++j) {
    const int m = m0 + j * 64 + wid * 16 + (lane >> 2);
    if (m < p.M) {
      const int img = m / HoWo, rem = m - img * HoWo;
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      a_base[j] = img * p.H;
      a_hi[j] = ho * p.stride - p.pad;
      a_wi[j] = wo * p.stride_w - p.pad_w;
    } else {
      a_base[j] = 0;
      a_hi[j] = -(1 << 20);  // never in range
      a_wi[j] = 0;
    }
  }
  const int cmask = (1 << p.lcin) - 1;
  const bf16* wrow[BP];
#pragma unroll
  for (int j = 0; j < BP; ++j) wrow[j] = p.Wt + (size_t)(n0 + j * 64 + wid * 16 + (lane >> 2)) * p.Kp + c * 8;

  auto dma = [&](int t) {
    lds_char* base = smem + (t % NST) * C_::ST;
    const int k0 = t * 32;
    const int kc = k0 + c * 8;
    const int tap = kc >> p.lcin, ci = kc & cmask;
    const int kh = tap / KW, kw = tap - (tap / KW) * KW;
    const bool tap_ok = tap < KH * KW;
#pragma unroll
    for (int j = 0; j < AP; ++j) {
      const int hi = a_hi[j] + kh, wi = a_wi[j] + kw;
      const bool ok = tap_ok && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
      const bf16* src = ok ? p.X + ((size_t)((a_base[j] + hi) * p.W + wi) << p.lcin) + ci : p.zero;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (void __attribute__((address_space(3)))*)(base + (j * NTHR + wid * 64) * 16),
                                       16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BP; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(wrow[j] + k0),
                                       (void __attribute__((address_space(3)))*)(base + C_::A_ST +
                                                                                 (j * NTHR + wid * 64) * 16),
                                       16, 0, 0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.Kp / 32;
  dma(0);
  if (nk > 1) dma(1);
  for (int t = 0; t < nk; ++t) {
    // own pieces of step t landed (step t+1 may stay in flight), then the barrier
    // makes every wave's pieces visible and frees stage (t+2) % 3 = (t-1) % 3
    if (t + 1 < nk) wait_vm<CNT>(); else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < nk) dma(t + 2);
    const lds_char* As = smem + (t % NST) * C_::ST;
    const lds_char* Bs = As + C_::A_ST;
    bf16x8 bfr[TN], afr[TM];
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = frag(Bs, wc * (TN * 16) + j * 16, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i) afr[i] = frag(As, wr * (TM * 16) + i * 16, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], afr[i], acc[i][j], 0, 0, 0);
  }

  // ---- epilogue: acc + bias -> bf16 LDS image -> (+R) -> ReLU -> 16-byte stores ------
  // The residual rows this thread will add are loaded first (all of them, into the
  // registers the accumulators free up), so their latency overlaps the LDS staging.
  constexpr int CPR = BN / 8, RPP = NTHR / CPR, NIT = BM / RPP;
  const int cc = tid % CPR, rr0 = tid / CPR;
  bf16x8 rv[RES ? NIT : 1];
  if constexpr (RES) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int m = m0 + rr0 + it * RPP;
      if (m < p.M) rv[it] = *reinterpret_cast<const bf16x8*>(p.R + (size_t)m * p.Cout + n0 + cc * 8);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  constexpr int ROWB = C_::ROWB;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wc * (TN * 16) + j * 16 + 4 * (lane >> 4);
    const bf16x4 bb = *reinterpret_cast<const bf16x4*>(p.bias + n0 + col);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wr * (TM * 16) + i * 16 + (lane & 15);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[i][j][r] + (float)bb[r]);
      *(lds_bf16x4*)(smem + row * ROWB + col * 2) = o;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int row = rr0 + it * RPP;
    const int m = m0 + row;
    if (m < p.M) {
      bf16x8 v = *(lds_cbf16x8*)(smem + row * ROWB + cc * 16);
      if constexpr (RES || RELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float f = (float)v[e];
          if constexpr (RES) f += (float)rv[it][e];
          if constexpr (RELU) f = fmaxf(f, 0.f);
          v[e] = (bf16)f;
        }
      }
      *reinterpret_cast<bf16x8*>(p.Y + (size_t)m * p.Cout + n0 + cc * 8) = v;
    }
  }
}

// ---- stem input: uint8 NHWC (C = 3) -> bf16 NHWC padded to 8 channels -------------
// (x / 255 - mean) / std on the 3 real channels, zeros in 3..7, one 16-byte store
// per pixel: the layout the implicit-GEMM gather takes (16-byte chunk = one tap).
// A block takes 4,096 pixels: 12 KB of input in by 16-byte loads into LDS, then
// thread t converts pixels t, t + 256, ... so a wave's stores are 1 KB contiguous.
constexpr int NP_PIX = 4096;
__global__ __launch_bounds__(256) void normalize_pad8_kernel(const uint8_t* __restrict__ in, bf16* __restrict__ out,
                                                             int64_t npix, float s0, float s1, float s2, float b0,
                                                             float b1, float b2) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[NP_PIX * 3];
  const int t = threadIdx.x;
  for (int64_t p0 = (int64_t)blockIdx.x * NP_PIX; p0 < npix; p0 += (int64_t)gridDim.x * NP_PIX) {
    const int n = (int)min((int64_t)NP_PIX, npix - p0);
    const uint8_t* src = in + p0 * 3;
    if (n == NP_PIX) {
#pragma unroll
      for (int j = 0; j < 3; ++j)
        reinterpret_cast<uint4*>(buf)[j * 256 + t] = reinterpret_cast<const uint4*>(src)[j * 256 + t];
    } else {
      for (int i = t; i < n * 3; i += 256) buf[i] = src[i];
    }
    __syncthreads();
    for (int i = t; i < n; i += 256) {
      bf16x8 o;
      o[0] = (bf16)__builtin_fmaf((float)buf[3 * i], s0, b0);
      o[1] = (bf16)__builtin_fmaf((float)buf[3 * i + 1], s1, b1);
      o[2] = (bf16)__builtin_fmaf((float)buf[3 * i + 2], s2, b2);
#pragma unroll
      for (int e = 3; e < 8; ++e) o[e] = (bf16)0.f;
      reinterpret_cast<bf16x8*>(out)[p0 + i] = o;
    }
    __syncthreads();
  }
}

// ---- stem input, pixel-pair form: uint8 [N, H, W, 3] -> bf16 [N, H + 6, (W + 6) / 2, 8] ---
// The 7x7 / stride-2 / pad-3 stem convolution on 3 channels padded to 8 spends 5/8 of
// its MFMA work on zero channels. Here the image is zero-bordered by 3 pixels and
// stored with 4 channels (RGB + 0) per pixel, two horizontally adjacent pixels per
// 16-byte "virtual pixel": the stem becomes a 7 x 4-tap convolution, stride (2, 1),
// no padding, over 8 virtual channels (tap pair (2j, 2j+1) = virtual tap j; the 8th
// real tap's weights are zero), K = 7 * 4 * 8 = 224 instead of 7 * 7 * 8 = 392 (+32 pad).
// One thread per virtual pixel: two 3-byte reads, one 16-byte store.
__global__ __launch_bounds__(256) void normalize_pairs_kernel(const uint8_t* __restrict__ in, bf16* __restrict__ out,
                                                              int N, int H, int W, float s0, float s1, float s2,
                                                              float b0, float b1, float b2) {
  const int Hp = H + 6, Wv = (W + 6) / 2;
  const int64_t total = (int64_t)N * Hp * Wv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int xv = (int)(i % Wv);
    const int64_t r = i / Wv;
    const int yp = (int)(r % Hp), n = (int)(r / Hp);
    const int y = yp - 3;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int x = 2 * xv + q - 3;
      if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
        const uint8_t* px = in + (((int64_t)n * H + y) * W + x) * 3;
        o[4 * q + 0] = (bf16)__builtin_fmaf((float)px[0], s0, b0);
        o[4 * q + 1] = (bf16)__builtin_fmaf((float)px[1], s1, b1);
        o[4 * q + 2] = (bf16)__builtin_fmaf((float)px[2], s2, b2);
      }
    }
    reinterpret_cast<bf16x8*>(out)[i] = o;
  }
}

// ---- 3x3 / stride-2 / pad-1 max pool, NHWC, 8 channels per lane -------------------
__global__ __launch_bounds__(256) void maxpool3s2_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N,
                                                          int H, int W, int C, int Ho, int Wo) {
  const int c8 = C >> 3;
  const int64_t total = (int64_t)N * Ho * Wo * c8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(i % c8);
    const int64_t pix = i / c8;
    const int wo = (int)(pix % Wo), ho = (int)((pix / Wo) % Ho), n = (int)(pix / ((int64_t)Wo * Ho));
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {
      const int hi = ho * 2 - 1 + dh;
      if ((unsigned)hi >= (unsigned)H) continue;
#pragma unroll
      for (int dw = 0; dw < 3; ++dw) {
        const int wi = wo * 2 - 1 + dw;
        if ((unsigned)wi >= (unsigned)W) continue;
        const bf16x8 v = reinterpret_cast<const bf16x8*>(x)[(((int64_t)n * H + hi) * W + wi) * c8 + cv];
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)v[e]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)m[e];
    reinterpret_cast<bf16x8*>(y)[i] = o;
  }
}

}  // namespace conv

// ---- host launchers ----------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int KH, int KW, bool RES, bool RELU>
static hipError_t conv_go(const conv::Args& a, hipStream_t st) {
  using C_ = conv::Cfg<BM, BN>;
  auto k = conv::conv_kernel<BM, BN, WM, WN, KH, KW, RES, RELU>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C_::LDS);
    attr = true;
  }
  conv::Args b = a;
  b.tiles_n = a.Cout / BN;
  const int grid = ((a.M + BM - 1) / BM) * b.tiles_n;
  hipLaunchKernelGGL(k, dim3(grid), dim3(conv::NTHR), C_::LDS, st, b);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int KH, int KW>
static hipError_t conv_epi(const conv::Args& a, bool relu, hipStream_t st) {
  if (a.R)
    return relu ? conv_go<BM, BN, WM, WN, KH, KW, true, true>(a, st)
                : conv_go<BM, BN, WM, WN, KH, KW, true, false>(a, st);
  return relu ? conv_go<BM, BN, WM, WN, KH, KW, false, true>(a, st)
              : conv_go<BM, BN, WM, WN, KH, KW, false, false>(a, st);
}

template <int KH, int KW>
static hipError_t conv_tile(const conv::Args& a, int tile, bool relu, hipStream_t st) {
  switch (tile) {
    case 0: return conv_epi<256, 128, 2, 2, KH, KW>(a, relu, st);  // Cout % 128 == 0
    case 1: return conv_epi<256, 64, 4, 1, KH, KW>(a, relu, st);   // Cout == 64
    case 2: return conv_epi<128, 128, 2, 2, KH, KW>(a, relu, st);  // few pixels (late stages)
    default: return hipErrorInvalidValue;
  }
}

// tile: 0 = 256x128, 1 = 256x64, 2 = 128x128. Kernel KH x KW (1x1, 3x3, 7x7, or the
// pixel-pair stem's 7x4), stride / pad per direction.
hipError_t conv2d_launch(const bf16* X, const bf16* Wt, const bf16* bias, const bf16* R, bf16* Y, const bf16* zero,
                         int N, int H, int W, int lcin, int Ho, int Wo, int KH, int KW, int stride_h, int stride_w,
                         int pad_h, int pad_w, int Cout, int Kp, bool relu, int tile, hipStream_t st) {
  conv::Args a{X, Wt, bias, R, Y, zero, H, W, lcin, Ho, Wo, stride_h, pad_h, Cout, Kp, N * Ho * Wo, 0,
               stride_w, pad_w};
  if (KH == 1 && KW == 1) return conv_tile<1, 1>(a, tile, relu, st);
  if (KH == 3 && KW == 3) return conv_tile<3, 3>(a, tile, relu, st);
  if (KH == 7 && KW == 7) return conv_tile<7, 7>(a, tile, relu, st);
  if (KH == 7 && KW == 4) return conv_tile<7, 4>(a, tile, relu, st);
  return hipErrorInvalidValue;
}

void normalize_pairs_launch(const uint8_t* in, bf16* out, int N, int H, int W, const float* sc, const float* bi,
                            hipStream_t st) {
  const int64_t total = (int64_t)N * (H + 6) * ((W + 6) / 2);
  hipLaunchKernelGGL(conv::normalize_pairs_kernel, dim3(ew_grid(total, 256)), dim3(256), 0, st, in, out, N, H, W,
                     sc[0], sc[1], sc[2], bi[0], bi[1], bi[2]);
}

void normalize_pad8_launch(const uint8_t* in, bf16* out, int64_t npix, const float* sc, const float* bi,
                           hipStream_t st) {
  const int64_t blocks = (npix + conv::NP_PIX - 1) / conv::NP_PIX;
  hipLaunchKernelGGL(conv::normalize_pad8_kernel, dim3((unsigned)std::min<int64_t>(blocks, 2048)), dim3(256), 0, st, in,
                     out, npix, sc[0],
                     sc[1], sc[2], bi[0], bi[1], bi[2]);
}

void maxpool3s2_launch(const bf16* x, bf16* y, int N, int H, int W, int C, int Ho, int Wo, hipStream_t st) {
  const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(conv::maxpool3s2_kernel, dim3(ew_grid(total, 256)), dim3(256), 0, st, x, y, N, H, W, C, Ho,
                     Wo);
}

}  // namespace caamd
