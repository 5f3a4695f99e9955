// RLlib learner kernels for gfx950: the default PPO / IMPALA encoder (Nature-CNN
// convs + MLP layers) and the fused PPO loss, all on MFMA.
//
// Encoder convolutions are NHWC and "valid" (no padding), computed as GEMMs:
//   forward  y[m,n]   = act(sum_k col[m,k] W[n,k] + b[n])      m = (b,oh,ow), k = (kh,kw,ci)
//   wgrad    dW[n,k] += sum_m dz[m,n] col[m,k]                 (split over m, fp32 atomics)
//   dgrad    dcol[m,k] = sum_n dz[m,n] W[n,k]  -> col2im gather (+ activation mask)
// with `col` materialised by an im2col gather (for the first layer straight from the
// uint8 frames, scaled by 1/255 on the way). Every (kh) row of a window is one
// contiguous run of KW*C elements in NHWC, so im2col / col2im move 16-byte vectors.
//
// rl_gemm: one templated MFMA GEMM for all three layouts.
//   C(m,n) = sum_k A(m,k) B(k,n); A(m,k) = AK ? A[m*lda+k] : A[k*lda+m];
//                                 B(k,n) = BK ? B[n*ldb+k] : B[k*ldb+n]
//   * 256 threads = 4 waves (2 x 2) over a BM x BN tile, BK = 32 per K step;
//     v_mfma_f32_16x16x32_bf16 with swapped operands so each lane owns 4
//     consecutive output columns (8-byte bf16x4 / 16-byte f32x4 epilogue stores).
//   * global -> registers (16-byte vectors; the next K tile is loaded while the
//     current one is multiplied) -> LDS in a k-contiguous [row][BK+8] image (the
//     8-element pad makes the 16-byte fragment reads conflict free); M-major
//     operands are transposed on the LDS store.
//   * split-K over blockIdx.z (wgrad reduces over up to 2e5 rows).
//   * block order: tiles of one XCD are contiguous in M (blockIdx.x is XCD-strided
//     by the hardware dispatcher; the remap gives each XCD a contiguous M range,
//     so neighbouring tiles share their B panel in one L2).
//   * epilogues: bf16 (+bias)(+ReLU / tanh), bf16 * act'(aux) (fused activation
//     backward for the dgrad of the next layer), fp32 atomics (wgrad).
//
// ppo_loss_cat: one thread per sample computes log-softmax, the clipped surrogate,
// the clipped value loss, entropy and KL(old||new) and writes dlogits / dvalue
// directly (no autograd graph), plus block-reduced loss statistics.
#include "common.h"

namespace caamd {
namespace rl {

enum RlEpi : int {
  RE_BF16 = 0,       // C = acc (+ bias)
  RE_BIAS_RELU = 1,  // C = relu(acc + bias)
  RE_BIAS_TANH = 2,  // C = tanh(acc + bias)
  RE_F32_ATOMIC = 3, // Cf32 += acc
  RE_DRELU = 4,      // C = acc * (aux > 0)
  RE_DTANH = 5,      // C = acc * (1 - aux^2)
};

struct GemmP {
  const bf16* A;
  const bf16* B;
  void* C;
  const bf16* bias;
  const bf16* aux;
  int M, N, K, lda, ldb, ldc;
  int kper;  // reduction length per split (multiple of 32)
};

constexpr int kBK = 32;
constexpr int kLDK = kBK + 8;  // LDS row stride in elements (80 bytes)

typedef __attribute__((address_space(3))) char lds_char;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// M-major operand tiles (A^T / B^T layouts, R >= 64 rows of the output) are kept in
// LDS as a [k][R] image, 16-byte chunks XOR-swizzled per k so the gfx950 transpose
// read (ds_read_b64_tr_b16) that builds k-consecutive MFMA fragments from it is
// bank-conflict free (same image / swizzle as gemm.hip's MN-major path).
template <int R>
__device__ __forceinline__ int mswz(int k) {
  if constexpr ((R % 128) == 0) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}

template <int R>
__device__ __forceinline__ void st_mmaj(lds_char* img, int k, int m8, const bf16x8& v) {
  const int pos = (m8 >> 3) ^ mswz<R>(k);
  *(__attribute__((address_space(3))) bf16x8*)(img + k * (R * 2) + pos * 16) = v;
}

// rows [rr, rr+16) x k [0, 32): lane l gets row rr+(l&15), k = 8*(l>>4) + j
template <int R>
__device__ __forceinline__ bf16x8 frag_mmaj(const lds_char* img, int rr, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int m = rr + 4 * p;
  const int chunk = m >> 3;
  const int within = (p & 1) * 8;
  s16x4 lo, hi;
  {
    const int k = 8 * g + q;
    const int pos = chunk ^ mswz<R>(k);
    lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (R * 2) + pos * 16 + within));
  }
  {
    const int k = 8 * g + 4 + q;
    const int pos = chunk ^ mswz<R>(k);
    hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (R * 2) + pos * 16 + within));
  }
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int BM, int BN, bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(256) void rl_gemm_kernel(GemmP p) {
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 fragments per wave (2x2 waves)
  constexpr int VA = BM * kBK / 8, VB = BN * kBK / 8;  // 16-byte vectors per tile
  constexpr int RA = (VA + 255) / 256, RB = (VB + 255) / 256;
  // M-major operands with >= 64 rows use the swizzled [k][R] image + transpose reads
  constexpr bool TRA = !AK && BM >= 64, TRB = !BKM && BN >= 64;
  __shared__ __attribute__((aligned(16))) bf16 sA[BM * kLDK];
  __shared__ __attribute__((aligned(16))) bf16 sB[BN * kLDK];
  lds_char* lA = (lds_char*)sA;
  lds_char* lB = (lds_char*)sB;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  // XCD-aware tile order: consecutive hardware block ids go round-robin over the 8
  // XCDs; give each XCD a contiguous run of M tiles instead.
  const int gx = gridDim.x;
  int bx = blockIdx.x;
  if (gx >= 16 && (gx & 7) == 0) bx = (bx & 7) * (gx >> 3) + (bx >> 3);
  const int m0 = bx * BM, n0 = blockIdx.y * BN;
  const int kbeg = blockIdx.z * p.kper;
  const int kend = min(p.K, kbeg + p.kper);

  bf16x8 ra[RA], rb[RB];
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < RA; ++r) {
      const int v = tid + r * 256;
      bf16x8 x = {};
      if (v < VA) {
        if constexpr (AK) {
          const int row = v >> 2, kc = (v & 3) * 8;
          if (m0 + row < p.M && k0 + kc < kend)
            x = *reinterpret_cast<const bf16x8*>(p.A + (int64_t)(m0 + row) * p.lda + k0 + kc);
        } else {
          const int k = v / (BM / 8), mc = (v % (BM / 8)) * 8;
          if (k0 + k < kend && m0 + mc < p.M)
            x = *reinterpret_cast<const bf16x8*>(p.A + (int64_t)(k0 + k) * p.lda + m0 + mc);
        }
      }
      ra[r] = x;
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int v = tid + r * 256;
      bf16x8 x = {};
      if (v < VB) {
        if constexpr (BKM) {
          const int row = v >> 2, kc = (v & 3) * 8;
          if (n0 + row < p.N && k0 + kc < kend)
            x = *reinterpret_cast<const bf16x8*>(p.B + (int64_t)(n0 + row) * p.ldb + k0 + kc);
        } else {
          const int k = v / (BN / 8), nc = (v % (BN / 8)) * 8;
          if (k0 + k < kend && n0 + nc < p.N)
            x = *reinterpret_cast<const bf16x8*>(p.B + (int64_t)(k0 + k) * p.ldb + n0 + nc);
        }
      }
      rb[r] = x;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int r = 0; r < RA; ++r) {
      const int v = tid + r * 256;
      if (v >= VA) continue;
      if constexpr (AK) {
        *reinterpret_cast<bf16x8*>(&sA[(v >> 2) * kLDK + (v & 3) * 8]) = ra[r];
      } else if constexpr (TRA) {
        st_mmaj<BM>(lA, v / (BM / 8), (v % (BM / 8)) * 8, ra[r]);
      } else {
        const int k = v / (BM / 8), mc = (v % (BM / 8)) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) sA[(mc + j) * kLDK + k] = ra[r][j];
      }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int v = tid + r * 256;
      if (v >= VB) continue;
      if constexpr (BKM) {
        *reinterpret_cast<bf16x8*>(&sB[(v >> 2) * kLDK + (v & 3) * 8]) = rb[r];
      } else if constexpr (TRB) {
        st_mmaj<BN>(lB, v / (BN / 8), (v % (BN / 8)) * 8, rb[r]);
      } else {
        const int k = v / (BN / 8), nc = (v % (BN / 8)) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) sB[(nc + j) * kLDK + k] = rb[r][j];
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kbeg < kend) {
    load(kbeg);
    store();
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += kBK) {
      const bool more = k0 + kBK < kend;
      if (more) load(k0 + kBK);  // in flight during the MFMAs below
      const int kq = 8 * (lane >> 4);
      bf16x8 bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int rr = wc * (BN / 2) + j * 16;
        if constexpr (TRB) bfr[j] = frag_mmaj<BN>(lB, rr, lane);
        else bfr[j] = *reinterpret_cast<const bf16x8*>(&sB[(rr + (lane & 15)) * kLDK + kq]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rr = wr * (BM / 2) + i * 16;
        bf16x8 afr;
        if constexpr (TRA) afr = frag_mmaj<BM>(lA, rr, lane);
        else afr = *reinterpret_cast<const bf16x8*>(&sA[(rr + (lane & 15)) * kLDK + kq]);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], afr, acc[i][j], 0, 0, 0);
      }
      __syncthreads();
      if (more) {
        store();
        __syncthreads();
      }
    }
  }

  // epilogue: lane owns C[m][n..n+3]
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wr * (BM / 2) + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
      if (n >= p.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      const int64_t off = (int64_t)m * p.ldc + n;
      if constexpr (EPI == RE_F32_ATOMIC) {
        float* c = reinterpret_cast<float*>(p.C) + off;
#pragma unroll
        for (int q = 0; q < 4; ++q) atomicAdd(c + q, v[q]);
      } else {
        if constexpr (EPI == RE_BF16 || EPI == RE_BIAS_RELU || EPI == RE_BIAS_TANH) {
          if (p.bias) {
            const bf16x4 b = *reinterpret_cast<const bf16x4*>(p.bias + n);
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] += (float)b[q];
          }
        }
        if constexpr (EPI == RE_BIAS_RELU) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
        } else if constexpr (EPI == RE_BIAS_TANH) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = tanhf(v[q]);
        } else if constexpr (EPI == RE_DRELU || EPI == RE_DTANH) {
          const bf16x4 a = *reinterpret_cast<const bf16x4*>(p.aux + off);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float y = (float)a[q];
            v[q] *= (EPI == RE_DRELU) ? (y > 0.f ? 1.f : 0.f) : (1.f - y * y);
          }
        }
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)v[q];
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(p.C) + off) = o;
      }
    }
  }
}

template <int BM, int BN, bool AK, bool BKM>
static void launch_layout(const GemmP& p, int epi, int splits, hipStream_t st) {
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, splits);
  switch (epi) {
    case RE_BF16: rl_gemm_kernel<BM, BN, AK, BKM, RE_BF16><<<grid, 256, 0, st>>>(p); break;
    case RE_BIAS_RELU: rl_gemm_kernel<BM, BN, AK, BKM, RE_BIAS_RELU><<<grid, 256, 0, st>>>(p); break;
    case RE_BIAS_TANH: rl_gemm_kernel<BM, BN, AK, BKM, RE_BIAS_TANH><<<grid, 256, 0, st>>>(p); break;
    case RE_F32_ATOMIC: rl_gemm_kernel<BM, BN, AK, BKM, RE_F32_ATOMIC><<<grid, 256, 0, st>>>(p); break;
    case RE_DRELU: rl_gemm_kernel<BM, BN, AK, BKM, RE_DRELU><<<grid, 256, 0, st>>>(p); break;
    case RE_DTANH: rl_gemm_kernel<BM, BN, AK, BKM, RE_DTANH><<<grid, 256, 0, st>>>(p); break;
  }
}

// layout: 0 = NT (A[M,K], B[N,K]) forward; 1 = NN (A[M,K], B[K,N]) dgrad;
//         2 = TN (A[K,M], B[K,N]) wgrad.  Tile: 128 x 32 when N <= 32, else 64 x 64.
void rl_gemm_launch(int layout, const GemmP& p, int epi, int splits, hipStream_t st) {
  const bool narrow = p.N <= 32;
  if (layout == 0) {
    if (narrow) launch_layout<128, 32, true, true>(p, epi, splits, st);
    else launch_layout<64, 64, true, true>(p, epi, splits, st);
  } else if (layout == 1) {
    if (narrow) launch_layout<128, 32, true, false>(p, epi, splits, st);
    else launch_layout<64, 64, true, false>(p, epi, splits, st);
  } else {
    if (narrow) launch_layout<128, 32, false, false>(p, epi, splits, st);
    else launch_layout<64, 64, false, false>(p, epi, splits, st);
  }
}

// ---------------------------------------------------------------- im2col / col2im
template <typename T>
__global__ __launch_bounds__(256) void im2col_kernel(const T* __restrict__ x, bf16* __restrict__ col, int64_t nvec,
                                                     int H, int W, int C, int KW, int S, int OH, int OW, int K,
                                                     float scale) {
  const int kv = K / 8;
  for (int64_t v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int64_t m = v / kv;
    const int k = (int)(v - m * kv) * 8;
    const int run = KW * C;
    const int kh = k / run, rem = k - kh * run;
    const int ow = (int)(m % OW);
    const int64_t t = m / OW;
    const int oh = (int)(t % OH);
    const int64_t b = t / OH;
    const int64_t src = ((b * H + oh * S + kh) * W + (int64_t)ow * S) * C + rem;
    bf16x8 o;
    if constexpr (sizeof(T) == 1) {
      const uint2 raw = *reinterpret_cast<const uint2*>(x + src);
      const uint8_t* u = reinterpret_cast<const uint8_t*>(&raw);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)u[j] * scale);
    } else {
      o = *reinterpret_cast<const bf16x8*>(x + src);
    }
    *reinterpret_cast<bf16x8*>(col + m * K + k) = o;
  }
}

// dz[b,ih,iw,c..c+7] = act'(y[b,ih,iw,c..]) * sum over windows covering (ih,iw) of dcol
__global__ __launch_bounds__(256) void col2im_kernel(const bf16* __restrict__ dcol, const bf16* __restrict__ y,
                                                     bf16* __restrict__ dz, int64_t nvec, int H, int W, int C,
                                                     int KH, int KW, int S, int OH, int OW, int act) {
  const int K = KH * KW * C;
  const int cv = C / 8;
  for (int64_t v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int c = (int)(v % cv) * 8;
    int64_t t = v / cv;
    const int iw = (int)(t % W);
    t /= W;
    const int ih = (int)(t % H);
    const int64_t b = t / H;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kh = ih % S; kh < KH; kh += S) {
      const int oh = (ih - kh) / S;
      if (oh < 0 || oh >= OH) continue;
      for (int kw = iw % S; kw < KW; kw += S) {
        const int ow = (iw - kw) / S;
        if (ow < 0 || ow >= OW) continue;
        const bf16x8 g = *reinterpret_cast<const bf16x8*>(
            dcol + ((b * OH + oh) * OW + ow) * (int64_t)K + (kh * KW + kw) * C + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += (float)g[j];
      }
    }
    const int64_t off = ((b * H + ih) * W + iw) * (int64_t)C + c;
    if (act) {
      const bf16x8 yy = *reinterpret_cast<const bf16x8*>(y + off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = (float)yy[j];
        s[j] *= (act == 1) ? (a > 0.f ? 1.f : 0.f) : (1.f - a * a);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)s[j];
    *reinterpret_cast<bf16x8*>(dz + off) = o;
  }
}

// db[n] += sum_m x[m, n]  (bf16 [M, N] row-major, N % 8 == 0, N <= 2048; fp32 atomics).
// Each thread owns one 8-column group and strides over rows; partial sums of the
// threads sharing a column group are combined in LDS, then one atomic per column.
constexpr int kColsumRows = 1024;
__global__ __launch_bounds__(256) void colsum_kernel(const bf16* __restrict__ x, float* __restrict__ db, int M,
                                                     int N) {
  __shared__ float part[256][9];
  const int groups = N / 8;                   // 8-column groups per row
  const int tpr = groups < 256 ? groups : 256;  // threads per row-pass
  const int rows_per_pass = 256 / tpr;
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * kColsumRows, r1 = min(M, r0 + kColsumRows);
  for (int g0 = 0; g0 < groups; g0 += tpr) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int g = g0 + t % tpr;
    if (t < rows_per_pass * tpr && g < groups) {
      for (int r = r0 + t / tpr; r < r1; r += rows_per_pass) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (int64_t)r * N + g * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += (float)v[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[t][j] = s[j];
    __syncthreads();
    for (int idx = t; idx < tpr * 8; idx += 256) {
      const int gi = idx / 8, j = idx % 8;  // one (group, column-in-group) per iteration
      if (g0 + gi < groups) {
        float acc = 0.f;
        for (int rp = 0; rp < rows_per_pass; ++rp) acc += part[rp * tpr + gi][j];
        atomicAdd(db + (g0 + gi) * 8 + j, acc);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- fused PPO loss
// stats[0..3] += sum over samples of (surrogate, clipped vf loss, entropy, kl)
__global__ __launch_bounds__(256) void ppo_loss_cat_kernel(
    const float* __restrict__ logits, const float* __restrict__ vf, const int64_t* __restrict__ act,
    const float* __restrict__ old_logp, const float* __restrict__ adv, const float* __restrict__ vt,
    const float* __restrict__ old_logits, int B, int A, float clip, float vf_clip, float vf_coeff,
    float ent_coeff, float kl_coeff, const float* __restrict__ kl_dev, float* __restrict__ dlogits,
    float* __restrict__ dvf, float* __restrict__ stats) {
  __shared__ float red[4][4];
  if (kl_dev) kl_coeff = kl_dev[0];  // device-resident coefficient (HIP-graph replays)
  const int i = blockIdx.x * 256 + threadIdx.x;
  float s_surr = 0.f, s_vf = 0.f, s_ent = 0.f, s_kl = 0.f;
  if (i < B) {
    const float* z = logits + (int64_t)i * A;
    const float* zo = old_logits + (int64_t)i * A;
    float mx = -INFINITY, mxo = -INFINITY;
    for (int j = 0; j < A; ++j) {
      mx = fmaxf(mx, z[j]);
      mxo = fmaxf(mxo, zo[j]);
    }
    float se = 0.f, seo = 0.f;
    for (int j = 0; j < A; ++j) {
      se += __expf(z[j] - mx);
      seo += __expf(zo[j] - mxo);
    }
    const float lse = mx + __logf(se), lseo = mxo + __logf(seo);
    float ent = 0.f, kl = 0.f;
    for (int j = 0; j < A; ++j) {
      const float lp = z[j] - lse, lpo = zo[j] - lseo;
      const float pp = __expf(lp), po = __expf(lpo);
      ent -= pp * lp;
      kl += po * (lpo - lp);
    }
    int a = (int)act[i];
    a = a < 0 ? 0 : (a >= A ? A - 1 : a);  // never index outside the logits row
    const float logp = z[a] - lse;
    const float r = __expf(logp - old_logp[i]);
    const float ad = adv[i];
    const float rc = fminf(fmaxf(r, 1.f - clip), 1.f + clip);
    const float u = r * ad, c = rc * ad;
    const float surr = fminf(u, c);
    // d(-mean surr)/dlogp: through r*adv when it is the min (ties split with the clamp
    // branch, which passes the same gradient inside the clip range)
    const float g_logp = (u <= c) ? -ad * r / (float)B : 0.f;
    const float invB = 1.f / (float)B;
    for (int j = 0; j < A; ++j) {
      const float lp = z[j] - lse;
      const float pp = __expf(lp), po = __expf(zo[j] - lseo);
      float g = g_logp * ((j == a ? 1.f : 0.f) - pp);
      g += ent_coeff * invB * pp * (lp + ent);
      g += kl_coeff * invB * (pp - po);
      dlogits[(int64_t)i * A + j] = g;
    }
    const float d = vf[i] - vt[i];
    const float sq = d * d;
    dvf[i] = (sq <= vf_clip) ? vf_coeff * invB * 2.f * d : 0.f;
    s_surr = surr;
    s_vf = fminf(sq, vf_clip);
    s_ent = ent;
    s_kl = kl;
  }
  s_surr = wave_sum(s_surr);
  s_vf = wave_sum(s_vf);
  s_ent = wave_sum(s_ent);
  s_kl = wave_sum(s_kl);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) {
    red[w][0] = s_surr;
    red[w][1] = s_vf;
    red[w][2] = s_ent;
    red[w][3] = s_kl;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(stats + threadIdx.x, t);
  }
}

}  // namespace rl

void rl_gemm(int layout, const bf16* A, const bf16* B, void* C, const bf16* bias, const bf16* aux, int M, int N,
             int K, int lda, int ldb, int ldc, int epi, int splits, hipStream_t st) {
  rl::GemmP p{A, B, C, bias, aux, M, N, K, lda, ldb, ldc, 0};
  splits = splits < 1 ? 1 : splits;
  int kper = (K + splits - 1) / splits;
  kper = ((kper + rl::kBK - 1) / rl::kBK) * rl::kBK;
  p.kper = kper;
  splits = (K + kper - 1) / kper;
  rl::rl_gemm_launch(layout, p, epi, splits, st);
}

void rl_im2col(const void* x, bool u8, bf16* col, int B, int H, int W, int C, int KH, int KW, int S, float scale,
               hipStream_t st) {
  const int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1, K = KH * KW * C;
  const int64_t nvec = (int64_t)B * OH * OW * (K / 8);
  const int grid = ew_grid(nvec, 256);
  if (u8)
    rl::im2col_kernel<uint8_t><<<grid, 256, 0, st>>>((const uint8_t*)x, col, nvec, H, W, C, KW, S, OH, OW, K, scale);
  else
    rl::im2col_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)x, col, nvec, H, W, C, KW, S, OH, OW, K, scale);
}

void rl_col2im(const bf16* dcol, const bf16* y, bf16* dz, int B, int H, int W, int C, int KH, int KW, int S, int act,
               hipStream_t st) {
  const int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1;
  const int64_t nvec = (int64_t)B * H * W * (C / 8);
  rl::col2im_kernel<<<ew_grid(nvec, 256), 256, 0, st>>>(dcol, y, dz, nvec, H, W, C, KH, KW, S, OH, OW, act);
}

void rl_colsum(const bf16* x, float* db, int M, int N, hipStream_t st) {
  rl::colsum_kernel<<<(M + rl::kColsumRows - 1) / rl::kColsumRows, 256, 0, st>>>(x, db, M, N);
}

void ppo_loss_cat(const float* logits, const float* vf, const int64_t* act, const float* old_logp,
                  const float* adv, const float* vt, const float* old_logits, int B, int A, float clip,
                  float vf_clip, float vf_coeff, float ent_coeff, float kl_coeff, const float* kl_dev,
                  float* dlogits, float* dvf, float* stats, hipStream_t st) {
  rl::ppo_loss_cat_kernel<<<(B + 255) / 256, 256, 0, st>>>(logits, vf, act, old_logp, adv, vt, old_logits, B, A,
                                                           clip, vf_clip, vf_coeff, ent_coeff, kl_coeff, kl_dev,
                                                           dlogits, dvf, stats);
}

}  // namespace caamd
