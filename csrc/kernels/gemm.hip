// Hand-written CDNA4 (gfx950) bf16 GEMM on MFMA for the training hot path.
//
//   C[M,N] (+)= sum_k A(m,k) * B(k,n)   (fp32 accumulate, epilogue below)
//
// Operand layouts (template flags):
//   A_KMAJ: A(m,k) = A[m*lda + k]   (activations X, dY)      else A[k*lda + m] (dY for wgrad)
//   B_KMAJ: B(k,n) = B[n*ldb + k]   (nn.Linear weight W[N,K]) else B[k*ldb + n] (W in dgrad, X in wgrad)
// so  forward  y  = x W^T      -> <A_KMAJ, B_KMAJ>
//     dgrad    dx = dy W       -> <A_KMAJ, !B_KMAJ>
//     wgrad    dW = dy^T x     -> <!A_KMAJ, !B_KMAJ>
//
// Design (MI355X-first; see /opt/skills/guides/cdna_hip_programming.md §5):
//  * 512-thread workgroup = 8 waves (2 x 4 over the BM x BN tile), 2 waves per
//    SIMD, tile BM x BN x BK=64 with BM = 256 and BN = 256 or 320 (320 divides
//    GPT-2-XL's 1600 / 4800 / 6400 widths exactly; 256 does not).
//  * Global -> LDS by LDS-DMA (`global_load_lds_dwordx4`, 16 B per lane, no VGPR
//    staging), two LDS stages, the next K-tile's DMA issued before the current
//    tile's MFMAs.
//  * LDS images are XOR-swizzled on the DMA *source* address (the DMA writes
//    lane-linear), read with the same XOR: K-major tiles (128-B rows) are read
//    with ds_read_b128, MN-major tiles ([k][BM] rows) with the gfx950 hardware
//    transpose read ds_read_b64_tr_b16. Both swizzles are bank-conflict free
//    (checked by tools/gemm_swizzle_check.py).
//  * v_mfma_f32_16x16x32_bf16 with the operands swapped (D = B_frag * A_frag):
//    each lane then owns 4 consecutive output COLUMNS of one row, so the
//    epilogue stores 8-byte bf16x4 (or 16-byte f32x4) vectors.
//  * XCD-aware block order: the 8 XCDs each get a contiguous range of tiles in
//    GROUP_M-grouped order, so neighbouring tiles share A/B panels in one L2.
//  * Epilogues: bf16 store (+bias), bf16 read-add-store (gradient accumulation),
//    fp32 partial slabs for split-K, bias+GELU(tanh) (stores pre-activation and
//    activation), and dGELU (dz = acc * gelu'(z)) with fused bias-grad column sums.
#include "common.h"

#ifndef CAAMD_EPI_SYNC
#define CAAMD_EPI_SYNC 0  // 1: staging passes wait for the previous pass's stores (pre-round-5)
#endif

#include <mutex>
#include <unordered_set>

namespace caamd {
namespace gemm {

typedef __attribute__((address_space(3))) char lds_char;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int BKT = 64;  // K-tile depth
constexpr int NTHR = 512;

enum Epi : int {
  EPI_BF16 = 0,       // C = acc (+ bias[n])
  EPI_BF16_ACC = 1,   // C = C + acc (+ bias[n])
  EPI_F32 = 2,        // Cf32[slice] = acc          (split-K partial slab)
  EPI_BIAS_GELU = 3,  // Z = acc + bias ; C = gelu(Z)
  EPI_DGELU = 4,      // C = acc * gelu'(Z[m,n]) ; dbias[n] += colsum(C) (f32 atomics)
  EPI_SWIGLU = 5,     // B rows = [gate; up] in 64-row blocks: C[m, n/2] = silu(g) * u (ldc = N/2)
};

// gelu_tanh / gelu_tanh_grad: common.h (sigmoid form on v_exp_f32 + v_rcp_f32).

// K-major swizzle: 16-B chunk c of row r lives at chunk position c ^ ((r >> 1) & 7).
__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }
// MN-major swizzle for [k][R] images (R = 256: 32 chunks/row, R = 320: 40 chunks/row).
template <int R>
__device__ __forceinline__ int mswz(int k) {
  if constexpr ((R % 128) == 0) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}

template <int BM, int BN, bool AK, bool BK_>
struct Cfg {
  static constexpr int WM = 2, WN = 4;
  static constexpr int TM = BM / WM / 16;
  static constexpr int TN = BN / WN / 16;
  static constexpr int A_BYTES = BM * BKT * 2;
  static constexpr int B_BYTES = BN * BKT * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_DMA = A_BYTES / (NTHR * 16);
  static constexpr int B_DMA = B_BYTES / (NTHR * 16);
  static constexpr int LDS = 2 * STAGE;
  static_assert(A_BYTES % (NTHR * 16) == 0 && B_BYTES % (NTHR * 16) == 0, "tile/DMA mismatch");
  static_assert(TM * 16 * WM == BM && TN * 16 * WN == BN, "tile/wave mismatch");
};

// ---- global -> LDS (one operand, one K-tile) ------------------------------------
// K-major operand: rows [r0, r0+R) x k [k0, k0+64) of X[r*ld + k].
template <int R>
__device__ __forceinline__ void dma_kmaj(const bf16* __restrict__ X, int ld, int r0, int k0,
                                         lds_char* dst, int wid, int lane) {
  constexpr int N = R * BKT * 2 / (NTHR * 16);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int lin = j * NTHR + wid * 64 + lane;  // 16-B chunk index in LDS order
    const int row = lin >> 3, pos = lin & 7;
    const int c = pos ^ kswz(row);
    const bf16* src = X + (size_t)(r0 + row) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (void __attribute__((address_space(3)))*)(dst + (j * NTHR + wid * 64) * 16),
                                     16, 0, 0);
  }
}
// MN-major operand: k [k0, k0+64) x rows [r0, r0+R) of X[k*ld + r].
template <int R>
__device__ __forceinline__ void dma_mmaj(const bf16* __restrict__ X, int ld, int r0, int k0,
                                         lds_char* dst, int wid, int lane) {
  constexpr int N = R * BKT * 2 / (NTHR * 16);
  constexpr int CPR = R / 8;  // chunks per k-row
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int lin = j * NTHR + wid * 64 + lane;
    const int k = lin / CPR, pos = lin - k * CPR;
    const int c = pos ^ mswz<R>(k);
    const bf16* src = X + (size_t)(k0 + k) * ld + r0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (void __attribute__((address_space(3)))*)(dst + (j * NTHR + wid * 64) * 16),
                                     16, 0, 0);
  }
}

// ---- LDS -> MFMA fragments ------------------------------------------------------
// Fragment of 16 rows [rr, rr+16) x k-sub ks (32 deep): lane l gets row rr+(l&15),
// k = ks*32 + 8*(l>>4) + j, j = 0..7.
__device__ __forceinline__ bf16x8_t frag_kmaj(const lds_char* img, int rr, int ks, int lane) {
  const int row = rr + (lane & 15);
  const int c = ks * 4 + (lane >> 4);
  const int pos = c ^ kswz(row);
  typedef __attribute__((address_space(3))) const bf16x8_t lds_bf16x8;
  return *(lds_bf16x8*)(img + row * 128 + pos * 16);
}
template <int R>
__device__ __forceinline__ bf16x8_t frag_mmaj(const lds_char* img, int rr, int ks, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int m = rr + 4 * p;
  const int chunk = m >> 3;
  const int within = (p & 1) * 8;
  s16x4 lo, hi;
  {
    const int k = ks * 32 + 8 * g + q;
    const int pos = chunk ^ mswz<R>(k);
    lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (R * 2) + pos * 16 + within));
  }
  {
    const int k = ks * 32 + 8 * g + 4 + q;
    const int pos = chunk ^ mswz<R>(k);
    hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (R * 2) + pos * 16 + within));
  }
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// frag_mmaj by inline asm: hipcc treats the tr16 BUILTIN as possibly aliasing an
// in-flight LDS-DMA and emits s_waitcnt vmcnt(0) before it, which drains the DMA
// prefetch on every K-step (measured in the stream-K weight-gradient kernel's ISA;
// the D = 64 attention kernels hit the same). The asm reads are invisible to the
// compiler's counters: every batch ends in tr_wait(), an lgkmcnt(0) that names the
// destination registers, so nothing reads them before the data has landed.
template <int R>
__device__ __forceinline__ bf16x8_t frag_mmaj_asm(const lds_char* img, int rr, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int m = rr + 4 * p;
  const int chunk = m >> 3;
  const int within = (p & 1) * 8;
  const int k0 = 8 * g + q, k1 = 8 * g + 4 + q;
  const unsigned a0 = (unsigned)(size_t)(img + k0 * (R * 2) + (chunk ^ mswz<R>(k0)) * 16 + within);
  const unsigned a1 = (unsigned)(size_t)(img + k1 * (R * 2) + (chunk ^ mswz<R>(k1)) * 16 + within);
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a1) : "memory");
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

struct Args {
  const bf16* A;
  const bf16* B;
  void* C;
  const bf16* bias;   // [N] or null
  const bf16* Z;      // dGELU: pre-activation [M,N] (ldc); BIAS_GELU: out pre-activation
  bf16* Zout;
  float* dbias;       // dGELU: [N] fp32 accumulated
  int M, N, K;
  int lda, ldb, ldc;
  int splitk;         // K slices (EPI_F32 only)
  int tiles_m, tiles_n;
  long long slab;     // elements between split-K slabs
  int algo;           // 0: 2-stage BK=64 kernel, 1: ping-pong BK=32 4-stage kernel
  // split-K TAIL (pp kernel): tiles [tfull, T) -- the ones past the last full round
  // of CUs -- are each split over tS K-slices; slices publish fp32 slabs to tws and
  // the last arriver (ticket in tcnt, reset by it) combines and runs the epilogue.
  int tfull, tS;
  float* tws;
  int* tcnt;
  // algo 9 only: B is in the decode GEMM's packed order (ops/llm.py pack_decode_weight:
  // per 128-row slab and 64-deep K-tile one contiguous swizzled 16 KiB image), so the
  // serving prefill reads the same weight copy as decode
  int bpack;
  int group_m;  // algo 9: m-tiles per tile-order group (0: 8); a tuning knob (gemm_set_group_m)
  // algo 9 with a split tail: dispatch the split (tail) workgroups FIRST, so the CUs
  // that start on a half-length slice run half a tile out of phase with the rest for the
  // whole launch and the output-store bursts of the two groups no longer coincide
  int tail_first;
};

// Workgroup barrier for the LDS image only: waits for this wave's LDS reads / writes
// (lgkmcnt), NOT for its global stores -- __syncthreads() also waits vmcnt(0), so every
// staging pass waited for the previous pass's stores to reach memory and the tile's
// output write (up to 327 KB per tile) never overlapped anything. The memory clobbers
// keep the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Output tile staged through LDS: the MFMA fragments (each lane: 4 columns of one
// row) are rounded to bf16 and written into a padded [BM/2][BN] image, one m-half
// of every wave at a time, then the whole workgroup streams the image out row by
// row with 16-byte vectors (a 320-wide row = 40 lanes = 5 full 128-B lines),
// applying the elementwise epilogue on the way. Direct per-fragment stores touch
// 16 rows x 32 B per instruction and ran the store path at ~1.6 TB/s.
template <int BM, int BN, int TM, int TN, int EPI, int ABL>
__device__ __forceinline__ void epilogue_staged(const Args& p, f32x4 (&acc)[TM][TN], int m0, int n0,
                                                int wr, int wc, int lane, lds_char* smem, int tid) {
  constexpr int ROWB = BN * 2 + 16;       // padded image row (bytes)
  constexpr int HR = BM / 2;              // image rows per pass
  constexpr int CPR = BN / 8;             // 16-B chunks per row
  constexpr int TMH = TM / 2;
  constexpr int ITERS = (HR * CPR + NTHR - 1) / NTHR;
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
  typedef __attribute__((address_space(3))) const bf16x8_t lds_bf16x8;
  const int mrow = lane & 15, ncol = 4 * (lane >> 4);
  // row pass: thread t owns column chunk t % CPR and rows t / CPR + RG * it, so a
  // thread's bias-gradient partial sums stay in one column chunk for the whole tile
  constexpr int RG = NTHR / CPR;          // row groups per iteration
  constexpr int ACTIVE = RG * CPR;
  constexpr int RITERS = (HR + RG - 1) / RG;
  const int c = tid % CPR, rg = tid / CPR;
  const int n = n0 + c * 8;
  float dsum[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) dsum[r] = 0.f;
  float bv[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) bv[r] = 0.f;
  if constexpr (EPI == EPI_BF16 || EPI == EPI_BF16_ACC || EPI == EPI_BIAS_GELU) {
    if (p.bias && tid < ACTIVE) {
      bf16x8_t b8 = *reinterpret_cast<const bf16x8_t*>(p.bias + n);
#pragma unroll
      for (int r = 0; r < 8; ++r) bv[r] = (float)b8[r];
    }
  }
  // the epilogue's global reads (dGELU: Z; accumulate: the previous C) for this
  // half's rows, issued before the LDS staging so their latency overlaps it: loaded
  // inside the row loop they serialise behind that loop's stores (C may alias Z for
  // the compiler), one HBM round trip per row iteration
  // (dGELU only: for the accumulate epilogue the extra live registers pushed the
  // stream-K weight-gradient kernel's main loop into scratch spills -- 3x slower)
  constexpr bool PRE = EPI == EPI_DGELU;
  // dGELU: the second half's Z loads are issued right after the first half is staged
  // (its accumulators are dead by then), so their latency overlaps the first half's
  // row loop instead of sitting between the two halves: fc-shape dGELU 660-663 ->
  // 649-651 us, bitwise equal (profiles/gemm_epi_ab_r6.jsonl)
  constexpr bool PRE2 = PRE;
  bf16x8_t pre[PRE2 ? 2 : 1][PRE ? RITERS : 1];
  auto zload = [&](int hh, int slot) {
    if (tid < ACTIVE && !(ABL & 8)) {
      const bf16* src = p.Z;
#pragma unroll
      for (int it = 0; it < RITERS; ++it) {
        const int ir = it * RG + rg;
        const int wr_ = ir / (TMH * 16), rem = ir - wr_ * (TMH * 16);
        const int m = m0 + wr_ * (TM * 16) + hh * (TMH * 16) + rem;
        if (ir < HR && m < p.M) pre[slot][it] = *reinterpret_cast<const bf16x8_t*>(src + (size_t)m * p.ldc + n);
      }
    }
  };
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if constexpr (PRE) {
      if (!PRE2 || h == 0) zload(h, 0);
    }
#if CAAMD_EPI_SYNC
    __syncthreads();
#else
    lds_barrier();  // image free (the previous pass's stores stay in flight)
#endif
#pragma unroll
    for (int i = 0; i < TMH; ++i) {
      const int ir = wr * (TMH * 16) + i * 16 + mrow;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nc = wc * (TN * 16) + j * 16 + ncol;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)acc[h * TMH + i][j][r];
        *(lds_bf16x4*)(smem + ir * ROWB + nc * 2) = o;
      }
    }
#if CAAMD_EPI_SYNC
    __syncthreads();
#else
    lds_barrier();  // image written
#endif
    if constexpr (PRE2) {
      if (h == 0) zload(1, 1);
    }
    if constexpr (ABL & 8) continue;
    if (tid >= ACTIVE) continue;
    if constexpr (EPI == EPI_SWIGLU) {
      // chunk c of a gate block (c / 8 even) pairs with chunk c + 8 of the up block
      // that follows it; the up-chunk threads have nothing to store
      static_assert(BN % 128 == 0, "SwiGLU: whole 64-row gate/up block pairs per tile");
      if ((c >> 3) & 1) continue;
      const int on = (n0 >> 1) + (c >> 4) * 64 + (c & 7) * 8;
      for (int it = 0; it < RITERS; ++it) {
        const int ir = it * RG + rg;
        if (ir >= HR) break;
        const int wr_ = ir / (TMH * 16), rem = ir - wr_ * (TMH * 16);
        const int m = m0 + wr_ * (TM * 16) + h * (TMH * 16) + rem;
        if (m >= p.M) continue;
        const bf16x8_t g = *(lds_bf16x8*)(smem + ir * ROWB + c * 16);
        const bf16x8_t u = *(lds_bf16x8*)(smem + ir * ROWB + (c + 8) * 16);
        bf16x8_t o;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float gf = (float)g[r];
          o[r] = (bf16)(__fdividef(gf, 1.f + __expf(-gf)) * (float)u[r]);
        }
        *reinterpret_cast<bf16x8_t*>((bf16*)p.C + (size_t)m * p.ldc + on) = o;
      }
      continue;
    }
#pragma unroll
    for (int it = 0; it < RITERS; ++it) {  // unrolled: pre[] stays in registers
      const int ir = it * RG + rg;
      if (ir >= HR) break;
      const int wr_ = ir / (TMH * 16), rem = ir - wr_ * (TMH * 16);
      const int m = m0 + wr_ * (TM * 16) + h * (TMH * 16) + rem;
      if (m >= p.M) continue;  // ragged M (stream-K weight-gradient tiles)
      bf16x8_t v = *(lds_bf16x8*)(smem + ir * ROWB + c * 16);
      const size_t off = (size_t)m * p.ldc + n;
      float f[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) f[r] = (float)v[r] + bv[r];
      bf16x8_t o;
      if constexpr (EPI == EPI_BF16) {
#pragma unroll
        for (int r = 0; r < 8; ++r) o[r] = (bf16)f[r];
      } else if constexpr (EPI == EPI_BF16_ACC) {
        const bf16x8_t prev = *reinterpret_cast<const bf16x8_t*>((bf16*)p.C + off);
#pragma unroll
        for (int r = 0; r < 8; ++r) o[r] = (bf16)(f[r] + (float)prev[r]);
      } else if constexpr (EPI == EPI_BIAS_GELU) {
        bf16x8_t z;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          z[r] = (bf16)f[r];
          o[r] = (bf16)gelu_tanh((float)z[r]);
        }
        *reinterpret_cast<bf16x8_t*>(p.Zout + off) = z;
      } else if constexpr (EPI == EPI_DGELU) {
        const bf16x8_t z = pre[PRE2 ? h : 0][it];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          o[r] = (bf16)(f[r] * gelu_tanh_grad((float)z[r]));
          dsum[r] += (float)o[r];
        }
      }
      *reinterpret_cast<bf16x8_t*>((bf16*)p.C + off) = o;
    }
  }
  if constexpr (EPI == EPI_DGELU) {
    // reduce the RG row-group partials of each column chunk in LDS, then one fp32
    // atomic per output column per tile
    typedef __attribute__((address_space(3))) float lds_float;
    lds_float* red = (lds_float*)smem;
    lds_barrier();  // image reads done
    if (tid < ACTIVE) {
#pragma unroll
      for (int r = 0; r < 8; ++r) red[rg * (CPR * 8) + c * 8 + r] = dsum[r];
    }
    lds_barrier();
    for (int col = tid; col < CPR * 8; col += NTHR) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < RG; ++g) t += red[g * (CPR * 8) + col];
      atomicAdd(p.dbias + n0 + col, t);
    }
  }
}

template <int BM, int BN, int TM, int TN, int EPI>
__device__ __forceinline__ void epilogue(const Args& p, f32x4 (&acc)[TM][TN], int m0, int n0, int wr,
                                         int wc, int lane, int slice) {
  // lane owns C[m][n..n+3] for every (i, j)
  const int mrow = lane & 15;
  const int ncol = 4 * (lane >> 4);
  if constexpr (EPI == EPI_DGELU) {
    // column sums of the output tile for the bias gradient: reduce over this
    // lane's rows, then across the 16 lanes of the same column group.
    float csum[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) csum[j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * (TM * 16) + i * 16 + mrow;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wc * (TN * 16) + j * 16 + ncol;
        const size_t off = (size_t)m * p.ldc + n;
        bf16x4 z = *reinterpret_cast<const bf16x4*>(p.Z + off);
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] * gelu_tanh_grad((float)z[r]);
          o[r] = (bf16)v;
          csum[j][r] += (float)o[r];
        }
        *reinterpret_cast<bf16x4*>((bf16*)p.C + off) = o;
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = csum[j][r];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        csum[j][r] = v;
      }
    if (mrow == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wc * (TN * 16) + j * 16 + ncol;
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(p.dbias + n + r, csum[j][r]);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wc * (TN * 16) + j * 16 + ncol;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == EPI_BF16 || EPI == EPI_BF16_ACC || EPI == EPI_BIAS_GELU) {
        if (p.bias) {
          bf16x4 b4 = *reinterpret_cast<const bf16x4*>(p.bias + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) bv[r] = (float)b4[r];
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wr * (TM * 16) + i * 16 + mrow;
        const size_t off = (size_t)m * p.ldc + n;
        if constexpr (EPI == EPI_F32) {
          float* Cf = (float*)p.C + (size_t)slice * p.slab;
          *reinterpret_cast<f32x4*>(Cf + off) = acc[i][j];
        } else if constexpr (EPI == EPI_BF16) {
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[i][j][r] + bv[r]);
          *reinterpret_cast<bf16x4*>((bf16*)p.C + off) = o;
        } else if constexpr (EPI == EPI_BF16_ACC) {
          bf16x4 prev = *reinterpret_cast<const bf16x4*>((bf16*)p.C + off);
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[i][j][r] + bv[r] + (float)prev[r]);
          *reinterpret_cast<bf16x4*>((bf16*)p.C + off) = o;
        } else if constexpr (EPI == EPI_BIAS_GELU) {
          bf16x4 z, o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            z[r] = (bf16)(acc[i][j][r] + bv[r]);
            o[r] = (bf16)gelu_tanh((float)z[r]);
          }
          *reinterpret_cast<bf16x4*>(p.Zout + off) = z;
          *reinterpret_cast<bf16x4*>((bf16*)p.C + off) = o;
        }
      }
    }
  }
}

// ABL (development ablations, tools/gemm_dev.py --ablate): bit 0 = no DMA in the
// loop, bit 1 = no LDS fragment reads, bit 2 = no MFMA. Production uses ABL = 0.
template <int BM, int BN, bool AK, bool BK_, int EPI, int ABL = 0>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(Args p) {
  using C_ = Cfg<BM, BN, AK, BK_>;
  constexpr int TM = C_::TM, TN = C_::TN;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  // ---- XCD-aware tile order ----------------------------------------------------
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  int sid;
  {
    const int xcd = bid & 7, loc = bid >> 3;
    const int q = nwg >> 3, r = nwg & 7;
    sid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int slice = sid % p.splitk;
  const int tile = sid / p.splitk;
  constexpr int GROUP_M = 8;
  const int group_sz = GROUP_M * p.tiles_n;
  const int g = tile / group_sz;
  const int first_m = g * GROUP_M;
  const int gm = min(p.tiles_m - first_m, GROUP_M);
  const int tin = tile - g * group_sz;
  const int tm = first_m + tin % gm;
  const int tn = tin / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int nk_total = p.K / BKT;
  const int per = (nk_total + p.splitk - 1) / p.splitk;
  const int kt0 = slice * per;
  const int kt1 = min(nk_total, kt0 + per);
  const int nk = kt1 - kt0;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int s, int kt) {
    lds_char* base = smem + s * C_::STAGE;
    const int k0 = kt * BKT;
    if constexpr (AK) dma_kmaj<BM>(p.A, p.lda, m0, k0, base, wid, lane);
    else dma_mmaj<BM>(p.A, p.lda, m0, k0, base, wid, lane);
    if constexpr (BK_) dma_kmaj<BN>(p.B, p.ldb, n0, k0, base + C_::A_BYTES, wid, lane);
    else dma_mmaj<BN>(p.B, p.ldb, n0, k0, base + C_::A_BYTES, wid, lane);
  };

  if (nk > 0) {
    stage(0, kt0);
    __syncthreads();  // vmcnt(0) + barrier: tile kt0 landed
    for (int it = 0; it < nk; ++it) {
      const int cur = it & 1;
      if (!(ABL & 1) && it + 1 < nk) stage(cur ^ 1, kt0 + it + 1);
      const lds_char* As = smem + cur * C_::STAGE;
      const lds_char* Bs = As + C_::A_BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t bf[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int rr = wc * (TN * 16) + j * 16;
          if constexpr (ABL & 2) { bf[j] = bf16x8_t{}; asm volatile("" : "+v"(bf[j])); }
          else if constexpr (BK_) bf[j] = frag_kmaj(Bs, rr, ks, lane);
          else bf[j] = frag_mmaj<BN>(Bs, rr, ks, lane);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int rr = wr * (TM * 16) + i * 16;
          bf16x8_t af;
          if constexpr (ABL & 2) { af = bf16x8_t{}; asm volatile("" : "+v"(af)); }
          else if constexpr (AK) af = frag_kmaj(As, rr, ks, lane);
          else af = frag_mmaj<BM>(As, rr, ks, lane);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if constexpr (ABL & 4) asm volatile("" :: "v"(bf[j]), "v"(af));
            else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af, acc[i][j], 0, 0, 0);
        }
      }
      __syncthreads();  // next tile landed (vmcnt(0)); everyone done with `cur`
    }
  }

  if constexpr (EPI == EPI_F32) epilogue<BM, BN, TM, TN, EPI>(p, acc, m0, n0, wr, wc, lane, slice);
  else epilogue_staged<BM, BN, TM, TN, EPI, ABL>(p, acc, m0, n0, wr, wc, lane, smem, tid);
}

// ================================================================================
// Ping-pong kernel ("pp"): BK = 32 K-steps through a 4-deep LDS ring, LDS-DMA two
// steps ahead with COUNTED vmcnt waits (never vmcnt(0) in the steady state), and
// the two waves of every SIMD (wave w and w+4 = the two wave-rows) staggered by
// one barrier so that one of them is in its MFMA segment while the other issues
// its LDS reads and DMA. Per K-step a wave runs two phases (m-half 0/1):
//   R(mh): [DMA step t+2 (mh=0)] ds_read A frags (4 m-tiles) [+ B frags (mh=0)]
//   barrier | M(mh): (TM/2) x TN MFMAs | barrier
// Intervals between barriers alternate (g0 R / g1 M), (g0 M / g1 R): the MFMA
// pipe of each SIMD is always fed by one of its two waves.
// RAW: step t+1 is read first by g0 after barrier 4t+4; every wave retires its
// step-t+1 DMA with vmcnt(#DMA of step t+2) at the end of R(t,1), before it.
// WAR: step t+2 reuses the stage of step t-2, whose last reads (g1, R(t-2,1))
// were consumed 4 intervals before the DMA issue at R(t,0).
// ================================================================================
__device__ __forceinline__ int kswz64(int row) { return ((row >> 3) & 1) * 2; }

template <int R>
__device__ __forceinline__ void dma_kmaj32_one(const bf16* __restrict__ X, int ld, int r0, int k0,
                                               lds_char* dst, int j, int wid, int lane) {
  const int lin = j * NTHR + wid * 64 + lane;
  const int row = lin >> 2, pos = lin & 3;
  const int c = pos ^ kswz64(row);
  const bf16* src = X + (size_t)(r0 + row) * ld + k0 + c * 8;
  __builtin_amdgcn_global_load_lds((const void*)src,
                                   (void __attribute__((address_space(3)))*)(dst + (j * NTHR + wid * 64) * 16),
                                   16, 0, 0);
}
template <int R>
__device__ __forceinline__ void dma_mmaj32_one(const bf16* __restrict__ X, int ld, int r0, int k0,
                                               lds_char* dst, int j, int wid, int lane) {
  constexpr int CPR = R / 8;
  const int lin = j * NTHR + wid * 64 + lane;
  const int k = lin / CPR, pos = lin - k * CPR;
  const int c = pos ^ mswz<R>(k);
  const bf16* src = X + (size_t)(k0 + k) * ld + r0 + c * 8;
  __builtin_amdgcn_global_load_lds((const void*)src,
                                   (void __attribute__((address_space(3)))*)(dst + (j * NTHR + wid * 64) * 16),
                                   16, 0, 0);
}
// One K-step (32 deep) of an R-row operand: FULL whole 8-KiB rounds, then a
// partial round issued by the first REM/1KiB waves only (wave-uniform branch).
template <int R, bool KMAJ>
__device__ __forceinline__ void dma_step32(const bf16* __restrict__ X, int ld, int r0, int k0,
                                           lds_char* dst, int wid, int lane) {
  constexpr int BYTES = R * 32 * 2;
  constexpr int FULL = BYTES / (NTHR * 16);
  constexpr int REM = BYTES - FULL * NTHR * 16;
#pragma unroll
  for (int j = 0; j < FULL; ++j) {
    if constexpr (KMAJ) dma_kmaj32_one<R>(X, ld, r0, k0, dst, j, wid, lane);
    else dma_mmaj32_one<R>(X, ld, r0, k0, dst, j, wid, lane);
  }
  if constexpr (REM > 0) {
    if (wid * 1024 < REM) {
      if constexpr (KMAJ) dma_kmaj32_one<R>(X, ld, r0, k0, dst, FULL, wid, lane);
      else dma_mmaj32_one<R>(X, ld, r0, k0, dst, FULL, wid, lane);
    }
  }
}
// DMA instructions one wave issues per K-step for an R-row operand (wave-uniform).
template <int R>
__device__ __forceinline__ constexpr int dma_count32(int wid) {
  constexpr int BYTES = R * 32 * 2;
  constexpr int FULL = BYTES / (NTHR * 16);
  constexpr int REM = BYTES - FULL * NTHR * 16;  // multiple of 1 KiB
  return FULL + (wid * 1024 < REM ? 1 : 0);
}
__device__ __forceinline__ bf16x8_t frag_kmaj64(const lds_char* img, int rr, int lane) {
  const int row = rr + (lane & 15);
  const int c = lane >> 4;
  const int pos = c ^ kswz64(row);
  typedef __attribute__((address_space(3))) const bf16x8_t lds_bf16x8;
  return *(lds_bf16x8*)(img + row * 64 + pos * 16);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// (An algo-7 variant issued K-step t+3's DMA pieces between the MFMA groups of the M
// segment: 1 % slower in the step, removed in round 4.)
template <int BM, int BN, bool AK, bool BK_, int EPI, int ABL = 0, int PH = 2, int DIST = 2>
__global__ __launch_bounds__(NTHR, 2) void gemm_pp_kernel(Args p) {
  static_assert(DIST == 2 || (DIST == 3 && PH == 1), "prefetch distance 3 is WAR-safe only with one phase");
  constexpr int WM = 2, WN = 4;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int TMH = TM / PH;  // m-tiles per phase (PH phases per K-step)
  static_assert(TM % PH == 0, "pp kernel splits the wave's m-tiles evenly over the phases");
  constexpr int KS = 32, NST = 4;
  constexpr int A_ST = BM * KS * 2, B_ST = BN * KS * 2, ST = A_ST + B_ST;
  static_assert(A_ST % 1024 == 0 && B_ST % 1024 == 0, "stage must be whole KiB");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  int slice, tile, nsplit;
  bool tail = false;
  {
    const int xcd = bid & 7, loc = bid >> 3;
    if (p.tS > 1) {
      // whole tiles: 1/8 per XCD (contiguous); then 1/8 of the tail slices per XCD,
      // dispatched last on every XCD (the slices of one tile stay on one XCD)
      const int nfx = p.tfull >> 3, ntx = (nwg - p.tfull) >> 3;
      if (loc < nfx) {
        tile = xcd * nfx + loc;
        slice = 0;
        nsplit = 1;
      } else {
        const int s = xcd * ntx + (loc - nfx);
        tile = p.tfull + s / p.tS;
        slice = s - (s / p.tS) * p.tS;
        nsplit = p.tS;
        tail = true;
      }
    } else {
      const int q = nwg >> 3, r = nwg & 7;
      const int sid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
      slice = sid % p.splitk;
      tile = sid / p.splitk;
      nsplit = p.splitk;
    }
  }
  constexpr int GROUP_M = 8;
  const int group_sz = GROUP_M * p.tiles_n;
  const int g = tile / group_sz;
  const int first_m = g * GROUP_M;
  const int gm = min(p.tiles_m - first_m, GROUP_M);
  const int tin = tile - g * group_sz;
  const int tm = first_m + tin % gm;
  const int tn = tin / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int ns_total = p.K / KS;
  const int per = (ns_total + nsplit - 1) / nsplit;
  const int s0 = slice * per;
  const int nk = max(0, min(ns_total, s0 + per) - s0);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto dma = [&](int t) {
    lds_char* base = smem + (t & (NST - 1)) * ST;
    const int k0 = (ABL & 16) ? s0 * KS : (s0 + t) * KS;  // ABL 16: L2-hot re-reads (timing only)
    dma_step32<BM, AK>(p.A, p.lda, m0, k0, base, wid, lane);
    dma_step32<BN, BK_>(p.B, p.ldb, n0, k0, base + A_ST, wid, lane);
  };
  // per-step DMA count of this wave: the two wave rows differ when a stage is not a
  // whole number of 8 KiB rounds (BN = 320)
  const bool lo_grp = wr == 0;
  constexpr int CNT_LO = dma_count32<BM>(0) + dma_count32<BN>(0);
  constexpr int CNT_HI = dma_count32<BM>(4) + dma_count32<BN>(4);
  // (count of waves 0..3 equals count of wave 0, waves 4..7 that of wave 4)
  static_assert(dma_count32<BM>(3) == dma_count32<BM>(0) && dma_count32<BN>(3) == dma_count32<BN>(0),
                "DMA count must be uniform per wave row");
  static_assert(dma_count32<BM>(7) == dma_count32<BM>(4) && dma_count32<BN>(7) == dma_count32<BN>(4),
                "DMA count must be uniform per wave row");
  // retire step t+1's DMA: leave the DMAs of the (up to DIST-1) newer steps in flight
  auto wait_ahead = [&](int newer) {
    if (newer >= 2 && DIST >= 3) {
      if (lo_grp) wait_vm<2 * CNT_LO>(); else wait_vm<2 * CNT_HI>();
    } else if (newer >= 1) {
      if (lo_grp) wait_vm<CNT_LO>(); else wait_vm<CNT_HI>();
    } else {
      wait_vm<0>();
    }
  };

  if (nk > 0) {
#pragma unroll
    for (int d = 0; d < DIST; ++d)
      if (d < nk) dma(d);
    wait_ahead(min(nk, DIST) - 1);
    __builtin_amdgcn_s_barrier();
    if (!lo_grp) __builtin_amdgcn_s_barrier();  // stagger the second wave row by one barrier
    bf16x8_t bf[TN];
    bf16x8_t af[TMH];
    for (int t = 0; t < nk; ++t) {
      const lds_char* As = smem + (t & (NST - 1)) * ST;
      const lds_char* Bs = As + A_ST;
#pragma unroll
      for (int mh = 0; mh < PH; ++mh) {
        // ---- R segment
        if (mh == 0) {
          if (!(ABL & 1) && t + DIST < nk) dma(t + DIST);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int rr = wc * (TN * 16) + j * 16;
            if constexpr (ABL & 2) { bf[j] = bf16x8_t{}; asm volatile("" : "+v"(bf[j])); }
            else if constexpr (BK_) bf[j] = frag_kmaj64(Bs, rr, lane);
            else bf[j] = frag_mmaj<BN>(Bs, rr, 0, lane);
          }
        }
#pragma unroll
        for (int i = 0; i < TMH; ++i) {
          const int rr = wr * (TM * 16) + (mh * TMH + i) * 16;
          if constexpr (ABL & 2) { af[i] = bf16x8_t{}; asm volatile("" : "+v"(af[i])); }
          else if constexpr (AK) af[i] = frag_kmaj64(As, rr, lane);
          else af[i] = frag_mmaj<BM>(As, rr, 0, lane);
        }
        if (mh == PH - 1 && !(ABL & 32)) {
          wait_ahead(min(nk - 1, t + DIST) - (t + 1));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // ---- M segment
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TMH; ++i) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if constexpr (ABL & 4) asm volatile("" :: "v"(bf[j]), "v"(af[i]));
            else acc[mh * TMH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[mh * TMH + i][j], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (lo_grp) __builtin_amdgcn_s_barrier();  // equal barrier counts for both rows
  }
  if constexpr (EPI != EPI_F32) {
    if (tail) {
      // ---- split-K tail: publish this slice; the last arriver combines -----------
      // (release/acquire ticket: cdna_hip_programming.md §5 "Projection GEMM" item 2)
      const int tt = tile - p.tfull;
      constexpr int SLAB = BM * BN;
      float* mine = p.tws + ((size_t)tt * p.tS + slice) * SLAB;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          *reinterpret_cast<f32x4*>(mine + ((size_t)((wid * TM + i) * TN + j) * 64 + lane) * 4) = acc[i][j];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      typedef __attribute__((address_space(3))) int lds_int;
      lds_int* flag = (lds_int*)smem;
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(p.tcnt + tt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == p.tS - 1;
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          p.tcnt[tt] = 0;  // ready for the next launch
        }
        *flag = last;
      }
      __syncthreads();
      const int last = *flag;
      if (!last) return;
      // all slices (own included, re-read) in slice order: reproducible sums
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < p.tS; ++s) {
        const float* other = p.tws + ((size_t)tt * p.tS + s) * SLAB;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] += *reinterpret_cast<const f32x4*>(other + ((size_t)((wid * TM + i) * TN + j) * 64 + lane) * 4);
      }
    }
  }
  if constexpr (EPI == EPI_F32) epilogue<BM, BN, TM, TN, EPI>(p, acc, m0, n0, wr, wc, lane, slice);
  else epilogue_staged<BM, BN, TM, TN, EPI, ABL>(p, acc, m0, n0, wr, wc, lane, smem, tid);
}

// ================================================================================
// Persistent ping-pong kernel (algo 4): one workgroup per CU walks a fixed list of
// output tiles (each XCD owns a contiguous, GROUP_M-grouped range of tiles; its
// workgroups stride through it), and the LDS ring of K-steps runs continuously
// ACROSS tiles: the first two K-steps of tile i+1 are already in flight while the
// last steps of tile i compute and while tile i's epilogue stores directly from
// the accumulators (no LDS staging, no barrier). That hides the per-tile pipeline
// fill and spreads the output stores over the next tile's main loop instead of
// bunching every CU's stores into one chip-wide burst. Same R / M segments,
// counted vmcnt and wave-row stagger as gemm_pp_kernel (one phase per K-step).
// ================================================================================
template <int BM, int BN, bool AK, bool BK_, int EPI>
__global__ __launch_bounds__(NTHR, 2) void gemm_persist_kernel(Args p) {
  constexpr int WM = 2, WN = 4;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int KS = 32, NST = 4, DIST = 2;
  constexpr int A_ST = BM * KS * 2, B_ST = BN * KS * 2, ST = A_ST + B_ST;
  static_assert(A_ST % 1024 == 0 && B_ST % 1024 == 0, "stage must be whole KiB");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const bool lo_grp = wr == 0;

  const int T = p.tiles_m * p.tiles_n;
  const int bid = blockIdx.x, G = gridDim.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = T >> 3, r = T & 7;
  const int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int size = q + (xcd < r ? 1 : 0);
  const int nbx = (G >> 3) + (xcd < (G & 7) ? 1 : 0);
  const int my_tiles = loc < size ? (size - loc + nbx - 1) / nbx : 0;
  constexpr int GROUP_M = 8;
  auto tile_origin = [&](int i, int& m0, int& n0) {
    const int tile = start + loc + i * nbx;
    const int group_sz = GROUP_M * p.tiles_n;
    const int g = tile / group_sz;
    const int first_m = g * GROUP_M;
    const int gm = min(p.tiles_m - first_m, GROUP_M);
    const int tin = tile - g * group_sz;
    m0 = (first_m + tin % gm) * BM;
    n0 = (tin / gm) * BN;
  };
  const int nk = p.K / KS;
  const int total = my_tiles * nk;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto dma = [&](int gs) {
    const int ti = gs / nk, ks = gs - ti * nk;
    int m0, n0;
    tile_origin(ti, m0, n0);
    lds_char* base = smem + (gs & (NST - 1)) * ST;
    const int k0 = ks * KS;
    dma_step32<BM, AK>(p.A, p.lda, m0, k0, base, wid, lane);
    dma_step32<BN, BK_>(p.B, p.ldb, n0, k0, base + A_ST, wid, lane);
  };
  constexpr int CNT_LO = dma_count32<BM>(0) + dma_count32<BN>(0);
  constexpr int CNT_HI = dma_count32<BM>(4) + dma_count32<BN>(4);
  auto wait_ahead = [&](int newer) {
    if (newer >= 1) {
      if (lo_grp) wait_vm<CNT_LO>(); else wait_vm<CNT_HI>();
    } else {
      wait_vm<0>();
    }
  };

  if (total > 0) {
    dma(0);
    if (total > 1) dma(1);
    wait_ahead(min(total, DIST) - 1);
    __builtin_amdgcn_s_barrier();
    if (!lo_grp) __builtin_amdgcn_s_barrier();
    int m0c, n0c;
    tile_origin(0, m0c, n0c);
    int ti = 0, ks = 0;
    bf16x8_t bf[TN];
    bf16x8_t af[TM];
    for (int gs = 0; gs < total; ++gs) {
      const lds_char* As = smem + (gs & (NST - 1)) * ST;
      const lds_char* Bs = As + A_ST;
      if (gs + DIST < total) dma(gs + DIST);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int rr = wc * (TN * 16) + j * 16;
        if constexpr (BK_) bf[j] = frag_kmaj64(Bs, rr, lane);
        else bf[j] = frag_mmaj<BN>(Bs, rr, 0, lane);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rr = wr * (TM * 16) + i * 16;
        if constexpr (AK) af[i] = frag_kmaj64(As, rr, lane);
        else af[i] = frag_mmaj<BM>(As, rr, 0, lane);
      }
      wait_ahead(min(total - 1, gs + DIST) - (gs + 1));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (++ks == nk) {
        epilogue<BM, BN, TM, TN, EPI>(p, acc, m0c, n0c, wr, wc, lane, 0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        ks = 0;
        if (++ti < my_tiles) tile_origin(ti, m0c, n0c);
      }
    }
    if (lo_grp) __builtin_amdgcn_s_barrier();
  }
}


// (A persistent variant of the ping-pong kernel with an asynchronous staged epilogue,
// algo 8, measured level or slower on every step shape -- fc fwd 670 vs 652 us, step
// 86.6k vs 87.8k tok/s, profiles/gemm_pst_r3.jsonl -- and was removed in round 4.)

// ================================================================================
// Stream-K ping-pong kernel (weight gradients: K = tokens = 32768, only 95-280
// output tiles of 256 x 320 for 256 CUs). Grid = the CUs (one 147 KB workgroup
// each); the tiles x K-steps iteration space is cut into gridDim.x equal runs, so
// every CU streams the same number of K-steps. A run covers the end of one tile,
// possibly whole tiles, and the start of another; a tile computed by one run gets
// the normal epilogue, a tile shared by several runs is combined by its LAST
// arriving contributor (agent-scope release -> ticket -> acquire; the others only
// publish an fp32 slab and move on), so no workgroup ever waits for another and
// nothing depends on co-residency. Each run has at most two partial tiles (its
// first and its last): slab slot 2*g (first) / 2*g+1 (last).
// Ragged M (1600 / 4800 output rows): A columns past M are clamped on load and
// never stored. Same R / M segments, counted vmcnt and wave-row stagger as
// gemm_pp_kernel (one phase per 32-deep K-step, DMA two steps ahead).
// Lockstep mode (p.tfull = S > 0, G = tiles x S): run g is slice g / tiles of tile
// g % tiles, the slices cut the K-steps evenly (+-1 when S does not divide them).
// Runs are slice-major, so the ~32 consecutive runs an XCD holds are neighbouring
// tiles of ONE token window at the same time and share its dY / X rows in that
// XCD's L2 (the stream-K order gives an XCD consecutive windows of a few tiles:
// nothing shared, HBM-bound at 1600 x 1600).
// ================================================================================
template <int BM, int BN, bool AK, bool BK_, int EPI>
__global__ __launch_bounds__(NTHR, 2) void gemm_sk_kernel(Args p) {
  constexpr int WM = 2, WN = 4;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int KS = 32, NST = 4, DIST = 2;
  constexpr int A_ST = BM * KS * 2, B_ST = BN * KS * 2, ST = A_ST + B_ST;
  static_assert(A_ST % 1024 == 0 && B_ST % 1024 == 0, "stage must be whole KiB");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const bool lo_grp = wr == 0;

  const int G = gridDim.x;
  int g;  // consecutive runs on one XCD (bijective for any G)
  {
    const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q = G >> 3, r = G & 7;
    g = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int nk_tile = p.K / KS;
  const int T = p.tiles_m * p.tiles_n;
  const int LS = p.tfull;  // > 0: lockstep split-K over LS slices (G == T * LS)
  const long long W = (long long)T * nk_tile;
  long long r0 = (long long)g * W / G, r1 = (long long)(g + 1) * W / G;
  if (LS > 0) {
    const int sl = g / T, tl = g - sl * T;
    r0 = (long long)tl * nk_tile + (long long)sl * nk_tile / LS;
    r1 = (long long)tl * nk_tile + (long long)(sl + 1) * nk_tile / LS;
  }
  auto run_start = [&](int gg) { return (long long)gg * W / G; };
  // first run containing global step x: largest gg with run_start(gg) <= x
  auto run_of = [&](long long x) { return (int)(((x + 1) * G + W - 1) / W - 1); };

  constexpr int CNT_LO = dma_count32<BM>(0) + dma_count32<BN>(0);
  constexpr int CNT_HI = dma_count32<BM>(4) + dma_count32<BN>(4);
  static_assert(dma_count32<BM>(3) == dma_count32<BM>(0) && dma_count32<BN>(3) == dma_count32<BN>(0), "");
  static_assert(dma_count32<BM>(7) == dma_count32<BM>(4) && dma_count32<BN>(7) == dma_count32<BN>(4), "");
  auto wait_ahead = [&](int newer) {
    if (newer >= 1) {
      if (lo_grp) wait_vm<CNT_LO>(); else wait_vm<CNT_HI>();
    } else {
      wait_vm<0>();
    }
  };
  const int a_last = AK ? p.M - 1 : p.M - 8;
  typedef __attribute__((address_space(3))) int lds_int;

  long long x = r0;
  while (x < r1) {
    const int tile = (int)(x / nk_tile);
    const int s0 = (int)(x - (long long)tile * nk_tile);
    const long long tile_end = (long long)(tile + 1) * nk_tile;
    const int nk = (int)((r1 < tile_end ? r1 : tile_end) - x);
    x += nk;
    constexpr int GROUP_M = 8;
    const int group_sz = GROUP_M * p.tiles_n;
    const int gq = tile / group_sz;
    const int first_m = gq * GROUP_M;
    const int gm = min(p.tiles_m - first_m, GROUP_M);
    const int tin = tile - gq * group_sz;
    const int m0 = (first_m + tin % gm) * BM, n0 = (tin / gm) * BN;

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto dma = [&](int t) {
      lds_char* base = smem + (t & (NST - 1)) * ST;
      const int k0 = (s0 + t) * KS;
      // A: clamp rows (K-major) / 8-aligned columns (MN-major) past M
      {
        constexpr int BYTES = BM * 32 * 2, FULL = BYTES / (NTHR * 16);
        static_assert(BYTES % (NTHR * 16) == 0, "A stage must be whole rounds");
#pragma unroll
        for (int j = 0; j < FULL; ++j) {
          const int lin = j * NTHR + wid * 64 + lane;
          const bf16* src;
          if constexpr (AK) {
            const int row = lin >> 2, pos = lin & 3;
            const int c = pos ^ kswz64(row);
            src = p.A + (size_t)min(m0 + row, a_last) * p.lda + k0 + c * 8;
          } else {
            constexpr int CPR = BM / 8;
            const int k = lin / CPR, pos = lin - k * CPR;
            const int c = pos ^ mswz<BM>(k);
            src = p.A + (size_t)(k0 + k) * p.lda + min(m0 + c * 8, a_last);
          }
          __builtin_amdgcn_global_load_lds((const void*)src,
                                           (void __attribute__((address_space(3)))*)(base + (j * NTHR + wid * 64) * 16),
                                           16, 0, 0);
        }
      }
      dma_step32<BN, BK_>(p.B, p.ldb, n0, k0, base + A_ST, wid, lane);
    };

    __syncthreads();  // the previous segment's epilogue / slab reads are done with the LDS
    dma(0);
    if (nk > 1) dma(1);
    wait_ahead(min(nk, DIST) - 1);
    __builtin_amdgcn_s_barrier();
    if (!lo_grp) __builtin_amdgcn_s_barrier();
    // two phases per K-step (m-halves), as gemm_pp_kernel with PH = 2: half the A
    // fragments live at a time (the MN-major tr16 reads otherwise spill at 256 VGPRs)
    constexpr int PH = 2, TMH = TM / PH;
    bf16x8_t bf[TN];
    bf16x8_t af[TMH];
    for (int t = 0; t < nk; ++t) {
      const lds_char* As = smem + (t & (NST - 1)) * ST;
      const lds_char* Bs = As + A_ST;
#pragma unroll
      for (int mh = 0; mh < PH; ++mh) {
        if (mh == 0) {
          if (t + DIST < nk) dma(t + DIST);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int rr = wc * (TN * 16) + j * 16;
            if constexpr (BK_) bf[j] = frag_kmaj64(Bs, rr, lane);
            else bf[j] = frag_mmaj_asm<BN>(Bs, rr, lane);
          }
        }
#pragma unroll
        for (int i = 0; i < TMH; ++i) {
          const int rr = wr * (TM * 16) + (mh * TMH + i) * 16;
          if constexpr (AK) af[i] = frag_kmaj64(As, rr, lane);
          else af[i] = frag_mmaj_asm<BM>(As, rr, lane);
        }
        if (mh == PH - 1) wait_ahead(min(nk - 1, t + DIST) - (t + 1));
        static_assert(TN == 5 && TMH == 4, "tr_wait below names 5 B and 4 A fragments");
        if (mh == 0)
          asm volatile("s_waitcnt lgkmcnt(0)"
                       : "+v"(bf[0]), "+v"(bf[1]), "+v"(bf[2]), "+v"(bf[3]), "+v"(bf[4]), "+v"(af[0]), "+v"(af[1]),
                         "+v"(af[2]), "+v"(af[3])::"memory");
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3])::"memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TMH; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[mh * TMH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[mh * TMH + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (lo_grp) __builtin_amdgcn_s_barrier();

    if (nk < nk_tile) {
      // ---- shared tile: publish, and combine if this is the last contributor -----
      const long long t_first = (long long)tile * nk_tile;
      const int c0 = LS > 0 ? 0 : run_of(t_first), c1 = LS > 0 ? LS - 1 : run_of(tile_end - 1);
      constexpr int SLAB = BM * BN;
      auto slot_of = [&](int gg) {  // a run's first tile uses slot 2g, its last 2g+1
        return 2 * gg + ((run_start(gg) / nk_tile) == tile ? 0 : 1);
      };
      // contributor c0 + i of this tile -> its slab (lockstep: slice i's run)
      auto slab_of = [&](int c) { return LS > 0 ? c * T + tile : slot_of(c); };
      float* mine = p.tws + (size_t)(LS > 0 ? g : slot_of(g)) * SLAB;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          *reinterpret_cast<f32x4*>(mine + ((size_t)((wid * TM + i) * TN + j) * 64 + lane) * 4) = acc[i][j];
      // algo 15: slices only publish; sk_reduce_kernel combines every tile in its own
      // launch over all CUs (the last-arriver combine leaves one workgroup per tile
      // re-reading LS slabs at the end: ~120 us of fixed cost at 1600 x 1600)
      if (p.algo == 15) continue;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      lds_int* flag = (lds_int*)smem;
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(p.tcnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == c1 - c0;
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          p.tcnt[tile] = 0;  // ready for the next launch
        }
        *flag = last;
      }
      __syncthreads();
      const int last = *flag;
      if (!last) continue;
      // every contributor (own included, re-read) in run order: reproducible sums
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int gg = c0; gg <= c1; ++gg) {
        const float* other = p.tws + (size_t)slab_of(gg) * SLAB;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] += *reinterpret_cast<const f32x4*>(other + ((size_t)((wid * TM + i) * TN + j) * 64 + lane) * 4);
      }
    }
    epilogue_staged<BM, BN, TM, TN, EPI, 0>(p, acc, m0, n0, wr, wc, lane, smem, tid);
  }
}

// Combine of the lockstep weight-gradient slabs (algo 15): one thread per f32x4 of
// a tile, the LS slices summed in slice order (same bits as the in-kernel
// combine), rounded to bf16 as the staged epilogue does (+ the previous C for the
// accumulate epilogue). Ragged M rows are skipped.
template <int BM, int BN, bool ACC>
__global__ __launch_bounds__(256) void sk_reduce_kernel(Args p, int LS) {
  constexpr int WM = 2, WN = 4, TM = BM / WM / 16, TN = BN / WN / 16, SLAB = BM * BN;
  const int T = p.tiles_m * p.tiles_n;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)T * (SLAB / 4)) return;
  const int tile = (int)(idx / (SLAB / 4));
  const int e = (int)(idx - (long long)tile * (SLAB / 4));
  const int lane = e & 63;
  int q = e >> 6;
  const int j = q % TN;
  q /= TN;
  const int i = q % TM, wid = q / TM;
  const int wr = wid >> 2, wc = wid & 3;
  // tile -> (m0, n0) exactly as the producing kernel: gemm_sk_kernel (8; its launches
  // pass group_m 0) or gemm_tn64_kernel (p.group_m, gemm_set_tn_group_m)
  const int GROUP_M = p.group_m > 0 ? p.group_m : 8;
  const int group_sz = GROUP_M * p.tiles_n;
  const int gq = tile / group_sz;
  const int first_m = gq * GROUP_M;
  const int gm = min(p.tiles_m - first_m, GROUP_M);
  const int tin = tile - gq * group_sz;
  const int m0 = (first_m + tin % gm) * BM, n0 = (tin / gm) * BN;
  const int row = m0 + wr * (TM * 16) + i * 16 + (lane & 15);
  const int col = n0 + wc * (TN * 16) + j * 16 + 4 * (lane >> 4);
  if (row >= p.M) return;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < LS; ++k)
    s += *reinterpret_cast<const f32x4*>(p.tws + ((size_t)k * T + tile) * SLAB + (size_t)e * 4);
  bf16* out = (bf16*)p.C + (size_t)row * p.ldc + col;
  bf16x4 o;
  if constexpr (ACC) {
    const bf16x4 prev = *reinterpret_cast<const bf16x4*>(out);
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (bf16)((float)(bf16)s[r] + (float)prev[r]);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (bf16)s[r];
  }
  *reinterpret_cast<bf16x4*>(out) = o;
}

// ================================================================================
// Full-line kernel (algo 9, NT layout: A[M][K], B[N][K], both K-major).
//
// What limited the 32-deep ping-pong kernel (profiles/gemm_ablations_r3.jsonl:
// "DMA + barriers only" 452 of 622 us at 32768 x 6400 x 1600): a 32-deep K-major
// slot holds 64 B of each 128-B row, so every LDS-DMA wave-instruction touched 16
// half-used cache lines (16 rows x 64 B), twice the address / tag work per byte of
// full lines (cdna_hip_programming.md §5 "Projection GEMM": fragment-shaped loads,
// TA_BUSY 2x at equal traffic). Here a K-step is 64 deep: every DMA instruction
// moves 8 whole rows x 128 B.
//
//  * Two LDS buffers of one 64-deep K-tile each (A 256 x 128 B + B BN x 128 B:
//    144 KB at BN = 320), XOR-swizzled 16-B chunks (c ^ ((row >> 1) & 7)),
//    ds_read_b128 fragments (frag_kmaj).
//  * DMA by buffer_load ... lds: one 128-bit descriptor per operand and tile (SGPRs),
//    one 32-bit lane offset per DMA round, the K offset in soffset -- no 64-bit
//    address math in the loop.
//  * Four phases per K-tile, (k-sub, m-half) = (0,0) (0,1) (1,0) (1,1): each an R
//    segment (DMA rounds of K-tile t+1, 4 A fragments, + TN B fragments on m-half 0)
//    and an M segment (4 x TN MFMAs), the two wave rows staggered by one barrier so
//    that every SIMD pairs one wave's R with the other's M (as gemm_pp_kernel).
//  * K-tile t+1's DMA rounds (9 per wave at BN = 320) are spread over the R segments
//    of phases 0 .. DSPLIT-1 of K-tile t (DSPLIT 2: 5 + 4). Buffer (t+1)&1 last held
//    K-tile t-1, whose last reads (phase 3) every wave retired (lgkmcnt(0)) before the
//    barrier that opens phase 0 of t. RAW: the leading row reads t+1 after the barrier
//    that closes its M(t,3) and the lagging row's R(t,3); both rows wait vmcnt(0) just
//    before it (nothing newer than K-tile t+1 is ever in flight there).
// ================================================================================
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  // wave-uniform inputs made provably uniform (cdna_hip_programming.md T20)
  const size_t b = (size_t)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const void* pb = (const void*)(((size_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc((void*)pb, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}

// one 16-B-per-lane LDS-DMA round: dst = wave-uniform LDS base (+ lane * 16)
__device__ __forceinline__ void dma_lds16(__amdgpu_buffer_rsrc_t r, lds_char* dst, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (void __attribute__((address_space(3)))*)dst, 16, voff,
                                           __builtin_amdgcn_readfirstlane(soff), 0, 0);
}

// PH = 4: phases (k-sub, m-half), 4 x TN MFMAs each; PH = 2: phases = m-halves with
// both k-subs, 8 x TN MFMAs each (half the barriers, twice the fragment registers).
// ABL (timing ablations): 1 no in-loop DMA, 2 no LDS reads, 4 no MFMA, 8 no epilogue
// stores, 16 no vmcnt waits, 32 every K-tile re-reads the first (L2-hot).
// (An L2 prefetch of K-tile t+2 -- one plain buffer load per 128-B line, issued behind
// K-tile t+1's DMA -- measured 4-8 % slower on every shape and was removed;
// profiles/gemm_k64_r4.jsonl, algos 5009-7009.)
template <int BM, int BN, int EPI, int ABL = 0, int DSPLIT = 2, int PH = 4>
__global__ __launch_bounds__(NTHR, 2) void gemm_k64_kernel(Args p) {
  constexpr int WM = 2, WN = 4;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int TMH = TM / 2;
  static_assert(PH == 2 || PH == 4, "phases per K-tile");
  static_assert(PH == 4 || DSPLIT == 1, "two phases: all DMA rounds in phase 0");
  constexpr int A_ST = BM * 128, B_ST = BN * 128, ST = A_ST + B_ST;
  constexpr int NA = A_ST / (NTHR * 16), NB = B_ST / (NTHR * 16), NR = NA + NB;
  static_assert(A_ST % (NTHR * 16) == 0 && B_ST % (NTHR * 16) == 0, "whole DMA rounds");
  static_assert(DSPLIT >= 1 && DSPLIT <= PH - 1, "DMA rounds go into phases 0 .. DSPLIT-1");
  static_assert(TM % 2 == 0, "two m-halves");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const bool lo_grp = wr == 0;

  // ---- tile / slice (same XCD-aware order and split-K tail as gemm_pp_kernel) ------
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  int slice, tile, nsplit;
  bool tail = false;
  {
    const int xcd = bid & 7, loc = bid >> 3;
    if (p.tS > 1) {
      const int nfx = p.tfull >> 3, ntx = (nwg - p.tfull) >> 3;
      const int lf = p.tail_first ? loc - ntx : loc;  // full-tile index (tail_first: after the tail)
      const int lt = p.tail_first ? loc : loc - nfx;  // tail index
      if (p.tail_first ? loc >= ntx : loc < nfx) {
        tile = xcd * nfx + lf;
        slice = 0;
        nsplit = 1;
      } else {
        const int s = xcd * ntx + lt;
        tile = p.tfull + s / p.tS;
        slice = s - (s / p.tS) * p.tS;
        nsplit = p.tS;
        tail = true;
      }
    } else {
      const int q = nwg >> 3, r = nwg & 7;
      tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
      slice = 0;
      nsplit = 1;
    }
  }
  const int GROUP_M = p.group_m > 0 ? p.group_m : 8;
  const int group_sz = GROUP_M * p.tiles_n;
  const int g = tile / group_sz;
  const int first_m = g * GROUP_M;
  const int gm = min(p.tiles_m - first_m, GROUP_M);
  const int tin = tile - g * group_sz;
  const int m0 = (first_m + tin % gm) * BM, n0 = (tin / gm) * BN;

  const int nt_total = p.K / 64;
  const int per = (nt_total + nsplit - 1) / nsplit;
  const int t0 = slice * per;
  const int nk = max(0, min(nt_total, t0 + per) - t0);

  // ---- DMA: descriptors per tile, one lane offset per round ------------------------
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A + (size_t)m0 * p.lda, (unsigned)(BM * p.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B + (size_t)n0 * p.ldb, (unsigned)(BN * p.ldb * 2));
  // Round j covers rows 64 j + 8 wid + (lane >> 3); the swizzle (row >> 1) & 7 does not
  // depend on j, so a lane's offset is one VGPR per operand and the round's row offset
  // (64 j rows) goes with the K offset into soffset.
  const int lrow = wid * 8 + (lane >> 3);
  const int lchunk = (lane & 7) ^ kswz(lrow);
  const int voff_a = (lrow * p.lda + lchunk * 8) * 2;
  // packed B: logical chunk c of slab row r sits at position c ^ s(r), s(r) = x ^ ((x & 1) << 2),
  // x = (r >> 1) & 7 (decode_gemm.hip swz); rows r and r + 64 share s, so one lane offset
  // serves every round and the slab / half-slab / K-tile offsets go into soffset
  const int bx = (lrow >> 1) & 7;
  const bool bpk = p.bpack != 0;
  const int voff_b = bpk ? lrow * 128 + (lchunk ^ (bx ^ ((bx & 1) << 2))) * 16 : (lrow * p.ldb + lchunk * 8) * 2;
  const int slab_bytes = 128 * p.K * 2;
  // round j of K-tile t -> buffer t & 1
#define K64_DMA_ROUND(t_, j_)                                                                          \
  dma_lds16((j_) < NA ? ra : rb,                                                                      \
            smem + ((t_) & 1) * ST +                                                                  \
                ((j_) < NA ? ((j_) * NTHR + wid * 64) * 16 : A_ST + (((j_) - NA) * NTHR + wid * 64) * 16), \
            (j_) < NA ? voff_a : voff_b,                                                              \
            ((j_) >= NA && bpk)                                                                       \
                ? (((j_) - NA) >> 1) * slab_bytes + (t0 + (t_)) * 16384 + (((j_) - NA) & 1) * 8192     \
                : ((ABL & 32) ? t0 : t0 + (t_)) * 128 + ((j_) < NA ? (j_) * 64 * p.lda : ((j_) - NA) * 64 * p.ldb) * 2)
  // rounds of phase q: [lo, hi)
  auto rlo = [](int q) { return q >= DSPLIT ? NR : (NR * q) / DSPLIT; };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
#pragma unroll
    for (int j = 0; j < NR; ++j) K64_DMA_ROUND(0, j);
    if (nk > 1) {
#pragma unroll
      for (int j = 0; j < NR; ++j) K64_DMA_ROUND(1, j);
      if constexpr (!(ABL & 16)) wait_vm<NR>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (!lo_grp) __builtin_amdgcn_s_barrier();  // stagger the second wave row by one barrier
    constexpr int NKS = PH == 4 ? 1 : 2;  // k-subs per phase
    bf16x8_t bf[NKS][TN];
    bf16x8_t af[NKS][TMH];
    for (int t = 0; t < nk; ++t) {
      const lds_char* As = smem + (t & 1) * ST;
      const lds_char* Bs = As + A_ST;
      const bool pre = !(ABL & 1) && t >= 1 && t + 1 < nk;  // K-tile t+1 (t = 0: issued in the prologue)
#pragma unroll
      for (int q = 0; q < PH; ++q) {
        const int mh = PH == 4 ? (q & 1) : q;
        // ---- R segment
        if (pre) {
#pragma unroll
          for (int j = rlo(q); j < rlo(q + 1); ++j) K64_DMA_ROUND(t + 1, j);
        }
#pragma unroll
        for (int u = 0; u < NKS; ++u) {
          const int ks = PH == 4 ? (q >> 1) : u;
          if (mh == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              if constexpr (ABL & 2) { bf[u][j] = bf16x8_t{}; asm volatile("" : "+v"(bf[u][j])); }
              else bf[u][j] = frag_kmaj(Bs, wc * (TN * 16) + j * 16, ks, lane);
            }
          }
#pragma unroll
          for (int i = 0; i < TMH; ++i) {
            if constexpr (ABL & 2) { af[u][i] = bf16x8_t{}; asm volatile("" : "+v"(af[u][i])); }
            else af[u][i] = frag_kmaj(As, wr * (TM * 16) + (mh * TMH + i) * 16, ks, lane);
          }
        }
        if (!(ABL & 16) && q == PH - 1 && !lo_grp) wait_vm<0>();  // lagging row: K-tile t+1 landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // ---- M segment
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int u = 0; u < NKS; ++u)
#pragma unroll
          for (int i = 0; i < TMH; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              if constexpr (ABL & 4) asm volatile("" :: "v"(bf[u][j]), "v"(af[u][i]));
              else acc[mh * TMH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[u][j], af[u][i], acc[mh * TMH + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (!(ABL & 16) && q == PH - 1 && lo_grp) wait_vm<0>();  // leading row: K-tile t+1 landed
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (lo_grp) __builtin_amdgcn_s_barrier();  // equal barrier counts for both rows
  }
  if (tail) {
    // ---- split-K tail: publish this slice; the last arriver combines (as gemm_pp_kernel)
    const int tt = tile - p.tfull;
    constexpr int SLAB = BM * BN;
    float* mine = p.tws + ((size_t)tt * p.tS + slice) * SLAB;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4*>(mine + ((size_t)((wid * TM + i) * TN + j) * 64 + lane) * 4) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    typedef __attribute__((address_space(3))) int lds_int;
    lds_int* flag = (lds_int*)smem;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(p.tcnt + tt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == p.tS - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        p.tcnt[tt] = 0;  // ready for the next launch
      }
      *flag = last;
    }
    __syncthreads();
    const int last = *flag;
    if (!last) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < p.tS; ++s) {
      const float* other = p.tws + ((size_t)tt * p.tS + s) * SLAB;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] += *reinterpret_cast<const f32x4*>(other + ((size_t)((wid * TM + i) * TN + j) * 64 + lane) * 4);
    }
  }
  epilogue_staged<BM, BN, TM, TN, EPI, (ABL & 8)>(p, acc, m0, n0, wr, wc, lane, smem, tid);
}
#undef K64_DMA_ROUND

// Split-K combine: out(bf16) [+]= sum_s slab_s (+ bias); f32 partials [S][M][ldc].
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S,
                                                            long long slab, bf16* __restrict__ out,
                                                            int M, int N, int ldc, bool accumulate) {
  const long long total4 = (long long)M * (N / 4);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total4;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / (N / 4);
    const int n = (int)(i - m * (N / 4)) * 4;
    const size_t off = (size_t)m * ldc + n;
    f32x4 s = *reinterpret_cast<const f32x4*>(part + off);
    for (int k = 1; k < S; ++k) s += *reinterpret_cast<const f32x4*>(part + (size_t)k * slab + off);
    bf16x4 o;
    if (accumulate) {
      bf16x4 prev = *reinterpret_cast<const bf16x4*>(out + off);
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)(s[r] + (float)prev[r]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)s[r];
    }
    *reinterpret_cast<bf16x4*>(out + off) = o;
  }
}

template <int BM, int BN, bool AK, bool BK_, int EPI, int ABL>
static hipError_t launch_abl(const Args& a, hipStream_t st);

// Raise the dynamic-LDS limit once per kernel (above 64 KiB needs the attribute).
static void ensure_lds(const void* k, int bytes) {
  static std::mutex mu;
  static std::unordered_set<const void*> done;
  std::lock_guard<std::mutex> g(mu);
  if (done.insert(k).second)
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// algo 9 (full-line kernel): algo = 9 + 10 * ABL + 1000 * DSPLIT (0 -> 2). Development
// ablations only on 256 x 320 bf16 tiles at the default DMA split.
template <int BM, int BN, int EPI, int ABL, int DS, int PH = 4>
static hipError_t launch_k64_v(const Args& a, hipStream_t st) {
  auto k = gemm_k64_kernel<BM, BN, EPI, ABL, DS, PH>;
  constexpr int lds = 2 * (BM + BN) * 128;
  ensure_lds((const void*)k, lds);
  const int T = a.tiles_m * a.tiles_n;
  const int grid = a.tS > 1 ? a.tfull + (T - a.tfull) * a.tS : T;
  hipLaunchKernelGGL(k, dim3(grid), dim3(NTHR), lds, st, a);
  return hipGetLastError();
}

// variant v = algo / 1000: 0 / 2 -> 4 phases, DMA over phases 0-1; 1 -> phase 0; 3 ->
// phases 0-2; 4 -> 2 phases (DMA in phase 0). Ablations (abl = algo / 10 % 100) on
// 256 x 320 bf16 tiles for variants 2 and 4.
template <int BM, int BN, int EPI>
static hipError_t launch_k64(const Args& a, hipStream_t st) {
  const int abl = (a.algo / 10) % 100, v = a.algo / 1000;
  if (a.splitk != 1) return hipErrorInvalidValue;
  if (abl == 0) {
    switch (v) {
      case 1: return launch_k64_v<BM, BN, EPI, 0, 1>(a, st);
      case 0:
      case 2: return launch_k64_v<BM, BN, EPI, 0, 2>(a, st);
      case 3: return launch_k64_v<BM, BN, EPI, 0, 3>(a, st);
      case 4: return launch_k64_v<BM, BN, EPI, 0, 1, 2>(a, st);
      default: return hipErrorInvalidValue;
    }
  }
  if constexpr (BM == 256 && BN == 320 && EPI == EPI_BF16) {
#define K64_ABL(n)                                                                                     \
  case n:                                                                                              \
    return v == 4 ? launch_k64_v<BM, BN, EPI, n, 1, 2>(a, st) : launch_k64_v<BM, BN, EPI, n, 2>(a, st);
    switch (abl) {
      K64_ABL(1) K64_ABL(2) K64_ABL(3) K64_ABL(4) K64_ABL(6) K64_ABL(8) K64_ABL(22) K64_ABL(38) K64_ABL(54)
      default: break;
    }
#undef K64_ABL
  }
  if constexpr (BM == 256 && BN == 320 && (EPI == EPI_BIAS_GELU || EPI == EPI_DGELU)) {
    // epilogue ablation (full-line variant 4 only): 8 = no epilogue (tools/gemm_epi_ab.py)
    if (v == 4 && abl == 8) return launch_k64_v<BM, BN, EPI, 8, 1, 2>(a, st);
  }
  return hipErrorInvalidValue;
}

// (A four-wave 256 x 256 variant -- 128 x 128 per wave in AGPRs, one wave per SIMD,
// fragment reads and DMA software-pipelined under the MFMAs -- measured 12-18 % slower
// than the full-line kernel on the prefill shapes (qkv 688 vs 611 us, o 474 vs 402 us
// at 16384 tokens): with one wave per SIMD nothing covers the per-K-tile barrier.
// Removed in round 4.)

template <int BM, int BN, bool AK, bool BK_, int EPI>
static hipError_t launch_t(const Args& a, hipStream_t st) {
  if (a.bpack && a.algo % 10 != 9) return hipErrorInvalidValue;
  // SwiGLU: staged epilogue of the ping-pong (2) and full-line (9) kernels only
  if (EPI == EPI_SWIGLU && (a.splitk != 1 || !(a.algo % 10 == 9 || a.algo == 2))) return hipErrorInvalidValue;
  if (a.algo % 10 == 9) {
    if constexpr (AK && BK_ && EPI != EPI_F32 && BM == 256) return launch_k64<BM, BN, EPI>(a, st);
    return hipErrorInvalidValue;
  }
  if constexpr (BM == 256 && BN == 320 && AK && BK_ && EPI == 0) {
    if (a.algo >= 10) {
      switch (a.algo / 10) {
        case 1: return launch_abl<BM, BN, AK, BK_, EPI, 1>(a, st);
        case 2: return launch_abl<BM, BN, AK, BK_, EPI, 2>(a, st);
        case 3: return launch_abl<BM, BN, AK, BK_, EPI, 3>(a, st);
        case 4: return launch_abl<BM, BN, AK, BK_, EPI, 4>(a, st);
        case 5: return launch_abl<BM, BN, AK, BK_, EPI, 5>(a, st);
        case 6: return launch_abl<BM, BN, AK, BK_, EPI, 6>(a, st);
        case 7: return launch_abl<BM, BN, AK, BK_, EPI, 7>(a, st);
        case 8: return launch_abl<BM, BN, AK, BK_, EPI, 8>(a, st);
        case 15: return launch_abl<BM, BN, AK, BK_, EPI, 15>(a, st);
        case 16: return launch_abl<BM, BN, AK, BK_, EPI, 16>(a, st);
        case 32: return launch_abl<BM, BN, AK, BK_, EPI, 32>(a, st);
        case 48: return launch_abl<BM, BN, AK, BK_, EPI, 48>(a, st);
        case 24: return launch_abl<BM, BN, AK, BK_, EPI, 24>(a, st);
        default: return hipErrorInvalidValue;
      }
    }
  }
  return launch_abl<BM, BN, AK, BK_, EPI, 0>(a, st);
}

template <int BM, int BN, bool AK, bool BK_, int EPI, int ABL>
static hipError_t launch_abl(const Args& a, hipStream_t st) {
  using C_ = Cfg<BM, BN, AK, BK_>;
  const int T = a.tiles_m * a.tiles_n;
  const int grid = a.tS > 1 ? a.tfull + (T - a.tfull) * a.tS : T * a.splitk;
  if (a.tS > 1 && !(a.algo % 10 >= 1 && a.algo % 10 <= 3) && a.algo != 5 && a.algo != 15)
    return hipErrorInvalidValue;
  if (a.algo == 5 || a.algo == 15) {  // stream-K / lockstep: the weight-gradient layout (TN), 256 x 320 tiles
    if constexpr ((EPI == EPI_BF16 || EPI == EPI_BF16_ACC) && BM == 256 && BN == 320 && !AK && !BK_) {
      auto k = gemm_sk_kernel<BM, BN, AK, BK_, EPI>;
      constexpr int lds = 4 * (BM + BN) * 32 * 2;
      ensure_lds((const void*)k, lds);
      hipLaunchKernelGGL(k, dim3(a.tS), dim3(NTHR), lds, st, a);  // tS = number of runs
      if (a.algo == 15) {  // lockstep slabs combined by their own launch
        if (a.tfull <= 0) return hipErrorInvalidValue;
        const long long n4 = (long long)a.tiles_m * a.tiles_n * (BM * BN / 4);
        hipLaunchKernelGGL((sk_reduce_kernel<BM, BN, EPI == EPI_BF16_ACC>), dim3((unsigned)((n4 + 255) / 256)),
                           dim3(256), 0, st, a, a.tfull);
      }
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (a.algo % 10 == 4 && a.splitk == 1) {
    auto k = gemm_persist_kernel<BM, BN, AK, BK_, EPI>;
    constexpr int lds = 4 * (BM + BN) * 32 * 2;
    ensure_lds((const void*)k, lds);
    const int tiles = a.tiles_m * a.tiles_n;
    hipLaunchKernelGGL(k, dim3(tiles < 256 ? tiles : 256), dim3(NTHR), lds, st, a);
  } else if (a.algo % 10 >= 1 && a.algo % 10 <= 3) {
    auto k = (a.algo % 10 == 1) ? gemm_pp_kernel<BM, BN, AK, BK_, EPI, ABL, 2, 2>
             : (a.algo % 10 == 2) ? gemm_pp_kernel<BM, BN, AK, BK_, EPI, ABL, 1, 2>
                                  : gemm_pp_kernel<BM, BN, AK, BK_, EPI, ABL, 1, 3>;
    constexpr int lds = 4 * (BM + BN) * 32 * 2;
    ensure_lds((const void*)k, lds);
    hipLaunchKernelGGL(k, dim3(grid), dim3(NTHR), lds, st, a);
  } else {
    auto k = gemm_kernel<BM, BN, AK, BK_, EPI, ABL>;
    ensure_lds((const void*)k, C_::LDS);
    hipLaunchKernelGGL(k, dim3(grid), dim3(NTHR), C_::LDS, st, a);
  }
  return hipGetLastError();
}

template <int BM, int BN, int EPI>
static hipError_t launch_layout(int layout, const Args& a, hipStream_t st) {
  switch (layout) {
    case 0: return launch_t<BM, BN, true, true, EPI>(a, st);    // NT  (fwd)
    case 1: return launch_t<BM, BN, true, false, EPI>(a, st);   // NN  (dgrad)
    case 2: return launch_t<BM, BN, false, false, EPI>(a, st);  // TN  (wgrad)
    default: return hipErrorInvalidValue;
  }
}

template <int BM, int BN>
static hipError_t launch_epi(int layout, int epi, const Args& a, hipStream_t st) {
  switch (epi) {
    case EPI_BF16: return launch_layout<BM, BN, EPI_BF16>(layout, a, st);
    case EPI_BF16_ACC: return launch_layout<BM, BN, EPI_BF16_ACC>(layout, a, st);
    case EPI_F32: return launch_layout<BM, BN, EPI_F32>(layout, a, st);
    case EPI_BIAS_GELU: return launch_t<BM, BN, true, true, EPI_BIAS_GELU>(a, st);
    case EPI_DGELU: return launch_t<BM, BN, true, true, EPI_DGELU>(a, st);
    case EPI_SWIGLU:
      if constexpr (BN % 128 == 0) return launch_t<BM, BN, true, true, EPI_SWIGLU>(a, st);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}


// ---- bf16 transpose (W -> W^T for the dgrad GEMM's K-major B operand) ---------------
// 64 x 64 tiles through LDS: coalesced 16-byte loads of input rows, 16-byte stores of
// output rows. LDS in dwords (bf16 pairs): each thread writes its 8 input elements as
// 4 dwords and gathers, for one PAIR of input columns, 8 rows as 8 dwords (row stride 33
// dwords: the 64 lanes of a gather hit 64 distinct banks), then splits low / high
// halves into two output rows -- half the LDS instructions of a bf16-granular tile.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ in,
                                                             bf16* __restrict__ out, int R, int C) {
  __shared__ unsigned tile[64][33];
  const int tiles_c = C / 64;
  const int tr = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = h * 32 + (t >> 3), c = (t & 7) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(in + (size_t)(tr * 64 + r) * C + tc * 64 + c);
    tile[r][c / 2 + 0] = v.x;
    tile[r][c / 2 + 1] = v.y;
    tile[r][c / 2 + 2] = v.z;
    tile[r][c / 2 + 3] = v.w;
  }
  __syncthreads();
  const int cp = t >> 3;        // input column pair -> output rows 2 cp, 2 cp + 1
  const int orr = (t & 7) * 8;  // output column chunk = input rows orr .. orr + 7
  unsigned w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = tile[orr + j][cp];
  uint4 lo, hi;  // output row 2 cp: the low halves; row 2 cp + 1: the high halves
  lo.x = __builtin_amdgcn_perm(w[1], w[0], 0x05040100u);
  lo.y = __builtin_amdgcn_perm(w[3], w[2], 0x05040100u);
  lo.z = __builtin_amdgcn_perm(w[5], w[4], 0x05040100u);
  lo.w = __builtin_amdgcn_perm(w[7], w[6], 0x05040100u);
  hi.x = __builtin_amdgcn_perm(w[1], w[0], 0x07060302u);
  hi.y = __builtin_amdgcn_perm(w[3], w[2], 0x07060302u);
  hi.z = __builtin_amdgcn_perm(w[5], w[4], 0x07060302u);
  hi.w = __builtin_amdgcn_perm(w[7], w[6], 0x07060302u);
  *reinterpret_cast<uint4*>(out + (size_t)(tc * 64 + 2 * cp) * R + tr * 64 + orr) = lo;
  *reinterpret_cast<uint4*>(out + (size_t)(tc * 64 + 2 * cp + 1) * R + tr * 64 + orr) = hi;
}

// ================================================================================
// TN full-line weight-gradient kernel (algo 25): C[M][N] (+)= sum_k A[k][m] B[k][n]
// with BOTH operands MN-major (A = dY [tokens][N_out], B = X [tokens][K_in]).
//
// What held the stream-K kernel above at 0.45 MFMA utilisation against 0.58 for the
// NT full-line kernel on the same tile (PERF.md, round 4): its ISA spends, per 32-deep
// K-step and wave, 53 VALU + 40 SALU + 26 tr16 reads + 5 LDS-DMA pieces around 40
// MFMAs -- a v_add per tr16 read (the swizzled fragment address plus the stage base:
// inline asm cannot fold an immediate) and a 64-bit v_mad per DMA piece. The full-line
// NT kernel needs 7 VALU per 80 MFMAs. This kernel keeps the NT kernel's schedule and
// removes that overhead:
//  * 64-deep K-tiles in two LDS buffers, [A0][A1][B0][B1], images [k][BM] / [k][BN]
//    with the mswz XOR swizzle (the same conflict-free tr16 images as the stream-K
//    kernel; K-sub 1 and the hi half of a fragment move only k bits 5 / 2, which the
//    swizzle does not use).
//  * Every per-lane address is computed ONCE: one VGPR per fragment (the swizzle
//    folded in) and one per DMA round. The loop is unrolled over the two stages, so a
//    tr16 read is `ds_read_b64_tr_b16 v, vaddr offset:<stage + k-sub + half>` and a
//    DMA piece is `buffer_load_dword ... lds` with the K-tile's row offset in soffset:
//    no VALU in the main loop.
//  * Four phases per K-tile ((k-sub, m-half) as the NT kernel), the two wave rows
//    staggered by one barrier so each SIMD pairs one wave's reads with the other's
//    MFMAs; K-tile t+1's DMA rounds spread over phases 0-1 of K-tile t (same RAW / WAR
//    argument as gemm_k64_kernel: buffer (t+1)&1 last held K-tile t-1, retired before
//    the barrier that opens phase 0 of t).
//  * Lockstep split-K: grid = tiles x S, run g = slice g / tiles of tile g % tiles,
//    slice-major so the ~31 runs of one XCD stream the same token window at the same
//    time (their dY / X rows are fetched once into that XCD's L2). S > 1: each run
//    stores an fp32 slab, sk_reduce_kernel sums the slices in order (deterministic).
//  * Ragged M (1600 = 6.25 x 256): A columns past M are clamped on load (the lane's
//    round offsets are computed once), rows past M are never stored.
// BM = 192 serves the 4800-row qkv gradient: 25 x 5 tiles x 2 slices = 250 runs for
// 256 CUs (256-row tiles: 95 tiles, 190 runs).
// ================================================================================
//
// AKM (NN layout, "gemm_nn64"): A K-major (A[m][k], activations / dY) with B still
// MN-major (B[k][n] = a weight W[N_out][K_in] read as stored): the dgrad dx = dY W and
// the transposed-storage fc2 forward without a weight transpose pass. A K-tile of A is
// the k64 kernel's image (BM rows x 128 B, kswz-swizzled, ds_read_b128 fragments at two
// precomputed lane addresses per fragment -- the k-sub moves the swizzled chunk, not a
// constant offset); B, the phases and the epilogue are the TN kernel's. No split (LS 1).
// (A BKM variant -- B K-major too, i.e. the NT layout on this schedule -- measured level
// with the k64 kernel at K = 1600 and 4-10 % slower at K = 6400, and was removed:
// profiles/gemm_nt_sched_ab_r6.txt.)
template <int BM, int BN, int EPI, bool COMBINE = false, bool AKM = false>
__global__ __launch_bounds__(NTHR, 2) void gemm_tn64_kernel(Args p) {
  constexpr int WM = 2, WN = 4;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16, TMH = TM / 2;
  static_assert(TM % 2 == 0 && TN == 5, "two m-halves; 5 B fragments per wave");
  constexpr int A_ST = 64 * BM * 2, B_ST = 64 * BN * 2;
  constexpr int NA = A_ST / (NTHR * 16), NB = B_ST / (NTHR * 16), NR = NA + NB;
  static_assert(A_ST % (NTHR * 16) == 0 && B_ST % (NTHR * 16) == 0, "whole DMA rounds");
  constexpr int B_BASE = 2 * A_ST;
  // largest immediate: stage 1 + k-sub 1 + hi half
  static_assert(A_ST + 32 * BM * 2 + 4 * BM * 2 < 65536 && B_ST + 32 * BN * 2 + 4 * BN * 2 < 65536,
                "ds_read offsets must fit 16 bits");
  constexpr int DSPLIT = 2;  // DMA rounds of K-tile t+1 over phases 0 and 1 of t
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const bool lo_grp = wr == 0;

  // ---- run -> (slice, tile) ------------------------------------------------------------
  const int G = gridDim.x;
  int g;
  {
    const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q = G >> 3, r = G & 7;
    g = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int T = p.tiles_m * p.tiles_n;
  const int LS = p.tfull > 0 ? p.tfull : 1;
  const int sl = g / T, tile = g - sl * T;
  const int nkt = p.K / 64;
  const int t0 = (int)((long long)sl * nkt / LS);
  const int nk = (int)((long long)(sl + 1) * nkt / LS) - t0;
  const int GROUP_M = p.group_m > 0 ? p.group_m : 8;  // tile order as sk_reduce_kernel
  const int group_sz = GROUP_M * p.tiles_n;
  const int gq = tile / group_sz;
  const int first_m = gq * GROUP_M;
  const int gm = min(p.tiles_m - first_m, GROUP_M);
  const int tin = tile - gq * group_sz;
  const int m0 = (first_m + tin % gm) * BM, n0 = (tin / gm) * BN;

  // ---- DMA: one descriptor per operand, one lane offset per round ------------------------
  const __amdgpu_buffer_rsrc_t ra =
      AKM ? make_rsrc(p.A + (size_t)m0 * p.lda, (unsigned)(BM * p.lda * 2))
          : make_rsrc(p.A + m0, (unsigned)(((size_t)p.K * p.lda - m0) * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B + n0, (unsigned)(((size_t)p.K * p.ldb - n0) * 2));
  int voa[NA], vob[NB];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    if constexpr (AKM) {
      // round j: rows 64 j + 8 wid + (lane >> 3), 16-B chunk (lane & 7) ^ kswz(row) of the
      // K-tile's 128-B row segment; kswz does not see the 64 j part of the row, so every
      // round uses round 0's lane offset and its 64 j rows go into soffset (dma_round)
      const int row = wid * 8 + (lane >> 3);
      voa[j] = (row * p.lda + ((lane & 7) ^ kswz(row)) * 8) * 2;
    } else {
      constexpr int CPR = BM / 8;
      const int lin = j * NTHR + wid * 64 + lane;
      const int k = lin / CPR, pos = lin - k * CPR;
      const int col = min(m0 + (pos ^ mswz<BM>(k)) * 8, p.M - 8) - m0;  // ragged M: clamp
      voa[j] = (k * p.lda + col) * 2;
    }
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    constexpr int CPR = BN / 8;
    const int lin = j * NTHR + wid * 64 + lane;
    const int k = lin / CPR, pos = lin - k * CPR;
    vob[j] = (k * p.ldb + (pos ^ mswz<BN>(k)) * 8) * 2;
  }
  const int arow = AKM ? 128 : 64 * p.lda * 2, brow = 64 * p.ldb * 2;  // bytes per K-tile
  auto dma_round = [&](int t, int stage, int j) {
    if (j < NA)
      dma_lds16(ra, smem + stage * A_ST + (j * NTHR + wid * 64) * 16, AKM ? voa[0] : voa[j],
                (t0 + t) * arow + (AKM ? j * 64 * p.lda * 2 : 0));
    else
      dma_lds16(rb, smem + B_BASE + stage * B_ST + ((j - NA) * NTHR + wid * 64) * 16, vob[j - NA],
                (t0 + t) * brow);
  };

  // ---- fragment lane addresses (tr16 reads of k rows 8g+q and 8g+4+q) ----------------------
  unsigned fa[TM], fb[TN];
  // AKM: k-sub 0 row-read lane address per fragment; k-sub 1 reads chunk c ^ 4, i.e.
  // the address XOR 64 (the image base -- the start of the dynamic LDS -- and every row
  // are 128-B aligned)
  unsigned fk[AKM ? TM : 1];
  {
    const int g4 = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    const int kk = 8 * g4 + q;
    const int within = (pp & 1) * 8;
    const unsigned base = (unsigned)(size_t)smem;
#pragma unroll
    for (int f = 0; f < TM; ++f) {
      if constexpr (AKM) {
        const int row = wr * TM * 16 + f * 16 + i16;
        fk[f] = base + row * 128 + ((g4 ^ kswz(row)) << 4);
        fa[f] = 0;
      } else {
        const int chunk = (wr * TM * 16 + f * 16 + 4 * pp) >> 3;
        fa[f] = base + kk * (BM * 2) + (chunk ^ mswz<BM>(kk)) * 16 + within;
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int chunk = (wc * TN * 16 + j * 16 + 4 * pp) >> 3;
      fb[j] = base + B_BASE + kk * (BN * 2) + (chunk ^ mswz<BN>(kk)) * 16 + within;
    }
  }
#define TN64_TR(dst, addr, imm) asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(imm) : "memory")

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8_t bf[TN];
  bf16x8_t af[TMH];
  // one K-tile out of LDS stage S (compile-time: every read offset is an immediate)
  auto ktile = [&](auto S_, int t) {
    constexpr int S = decltype(S_)::value;
    const bool pre = t >= 1 && t + 1 < nk;  // K-tile t+1 (t = 0: issued in the prologue)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mh = q & 1, ks = q >> 1;
      // ---- R segment
      if (pre && q < DSPLIT) {
#pragma unroll
        for (int j = (NR * q) / DSPLIT; j < (NR * (q + 1)) / DSPLIT; ++j) dma_round(t + 1, S ^ 1, j);
      }
      if (mh == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          s16x4 lo, hi;
          if (ks == 0) {
            TN64_TR(lo, fb[j], S * B_ST);
            TN64_TR(hi, fb[j], S * B_ST + 4 * BN * 2);
          } else {
            TN64_TR(lo, fb[j], S * B_ST + 32 * BN * 2);
            TN64_TR(hi, fb[j], S * B_ST + 32 * BN * 2 + 4 * BN * 2);
          }
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bf[j] = __builtin_bit_cast(bf16x8_t, v);
        }
      }
#pragma unroll
      for (int i = 0; i < TMH; ++i) {
        if constexpr (AKM) {
          unsigned a = fk[mh * TMH + i];
          if (ks == 1) {
            asm volatile("" : "+v"(a));  // keeps the XOR here (hoisted, 8 more live VGPRs spilled)
            a ^= 64u;
          }
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(af[i]) : "v"(a), "i"(S * A_ST) : "memory");
        } else {
          s16x4 lo, hi;
          const unsigned a = fa[mh * TMH + i];
          if (ks == 0) {
            TN64_TR(lo, a, S * A_ST);
            TN64_TR(hi, a, S * A_ST + 4 * BM * 2);
          } else {
            TN64_TR(lo, a, S * A_ST + 32 * BM * 2);
            TN64_TR(hi, a, S * A_ST + 32 * BM * 2 + 4 * BM * 2);
          }
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8_t, v);
        }
      }
      if (q == 3 && !lo_grp) wait_vm<0>();  // lagging row: K-tile t+1 landed
      // the asm reads are invisible to the compiler's counters: wait here, naming the
      // fragment registers so no MFMA is scheduled above the wait
      if constexpr (TMH == 4) {
        if (mh == 0)
          asm volatile("s_waitcnt lgkmcnt(0)"
                       : "+v"(bf[0]), "+v"(bf[1]), "+v"(bf[2]), "+v"(bf[3]), "+v"(bf[4]), "+v"(af[0]), "+v"(af[1]),
                         "+v"(af[2]), "+v"(af[3])::"memory");
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3])::"memory");
      } else {
        static_assert(TMH == 3, "3 or 4 A fragments per phase");
        if (mh == 0)
          asm volatile("s_waitcnt lgkmcnt(0)"
                       : "+v"(bf[0]), "+v"(bf[1]), "+v"(bf[2]), "+v"(bf[3]), "+v"(bf[4]), "+v"(af[0]), "+v"(af[1]),
                         "+v"(af[2])::"memory");
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0]), "+v"(af[1]), "+v"(af[2])::"memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- M segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TMH; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[mh * TMH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[mh * TMH + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (q == 3 && lo_grp) wait_vm<0>();  // leading row: K-tile t+1 landed
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if (nk > 0) {
#pragma unroll
    for (int j = 0; j < NR; ++j) dma_round(0, 0, j);
    if (nk > 1) {
#pragma unroll
      for (int j = 0; j < NR; ++j) dma_round(1, 1, j);
      wait_vm<NR>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (!lo_grp) __builtin_amdgcn_s_barrier();  // stagger the second wave row by one barrier
    for (int t = 0; t < nk; t += 2) {
      ktile(std::integral_constant<int, 0>{}, t);
      if (t + 1 < nk) ktile(std::integral_constant<int, 1>{}, t + 1);
    }
    if (lo_grp) __builtin_amdgcn_s_barrier();  // equal barrier counts for both rows
  }
#undef TN64_TR
  if (LS > 1) {
    // slice partial: fp32 slab in fragment order (sk_reduce_kernel's layout)
    constexpr int SLAB = BM * BN;
    if constexpr (!COMBINE) {  // algo 25: a separate reduce launch combines the slabs
      float* mine = p.tws + ((size_t)sl * T + tile) * SLAB;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          *reinterpret_cast<f32x4*>(mine + ((size_t)((wid * TM + i) * TN + j) * 64 + lane) * 4) = acc[i][j];
      return;
    } else {
    // algo 26: the tile's LAST arriving slice combines (no reduce launch). Hand-off
    // with write-through slabs (cdna_hip_programming.md Guideline 16, R1): every slab
    // byte is stored `sc1` and drained by its wave before the workgroup barrier, one
    // lane then adds to the tile's ticket (relaxed, agent scope); the last arriver
    // reads the other slabs with `sc1` loads only (no release / acquire fences: the
    // L2 write-backs they cost were what made the stream-K kernel's combine slow).
    // Slices are summed in slice order: the same bits as sk_reduce_kernel.
    typedef int v4i __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rw =
        make_rsrc(p.tws, (unsigned)min((size_t)0xFFFFFFF0u, (size_t)LS * T * SLAB * 4));
    // lane part of every slab address in one VGPR, the rest wave-uniform (soffset):
    // 40 per-fragment VGPR offsets spilled the main loop
    const int vlane = lane * 16;
    auto frag_soff = [&](int s_, int i, int j) {
      return __builtin_amdgcn_readfirstlane(
          (int)((((size_t)s_ * T + tile) * SLAB + (size_t)((wid * TM + i) * TN + j) * 256) * 4));
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, acc[i][j]), rw, vlane, frag_soff(sl, i, j), 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains (Pitfall 14)
    __syncthreads();
    typedef __attribute__((address_space(3))) int lds_int;
    lds_int* flag = (lds_int*)smem;
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.tcnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == LS - 1;
      if (last) __hip_atomic_store(p.tcnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    // two slices (the host allows no other count here): the other slice's partial
    // added to this one's registers -- a0 + a1, the bits of sk_reduce_kernel's
    // (0 + a0) + a1. One m-row of fragments at a time: the sched barriers keep the
    // compiler from hoisting all 40 slab loads (160 more live VGPRs spilled the
    // main loop).
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      f32x4 o[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        o[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, vlane, frag_soff(sl ^ 1, i, j), 16));
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += o[j];
    }
    }
  }
  __syncthreads();  // the last phase's LDS reads are done before the staging overwrites
  epilogue_staged<BM, BN, TM, TN, EPI, 0>(p, acc, m0, n0, wr, wc, lane, smem, tid);
}

template <int BM, int EPI>
static hipError_t launch_tn64(const Args& a, hipStream_t st) {
  constexpr int BN = 320;
  auto k = a.algo == 26 ? gemm_tn64_kernel<BM, BN, EPI, true> : gemm_tn64_kernel<BM, BN, EPI, false>;
  constexpr int lds = 2 * 64 * (BM + BN) * 2;
  ensure_lds((const void*)k, lds);
  const int T = a.tiles_m * a.tiles_n;
  const int LS = a.tfull > 0 ? a.tfull : 1;
  hipLaunchKernelGGL(k, dim3(T * LS), dim3(NTHR), lds, st, a);
  if (LS > 1 && a.algo != 26) {
    const long long n4 = (long long)T * (BM * BN / 4);
    hipLaunchKernelGGL((sk_reduce_kernel<BM, BN, EPI == EPI_BF16_ACC>), dim3((unsigned)((n4 + 255) / 256)),
                       dim3(256), 0, st, a, LS);
  }
  return hipGetLastError();
}

template <int EPI>
static hipError_t launch_nn64(const Args& a, hipStream_t st) {
  constexpr int BM = 256, BN = 320;
  auto k = gemm_tn64_kernel<BM, BN, EPI, false, true>;
  constexpr int lds = 2 * 64 * (BM + BN) * 2;
  ensure_lds((const void*)k, lds);
  hipLaunchKernelGGL(k, dim3(a.tiles_m * a.tiles_n), dim3(NTHR), lds, st, a);
  return hipGetLastError();
}

}  // namespace gemm

// NN GEMM on the full-line TN schedule (algo 27): C[M][N] = A[M][K] B[K][N] (+ bias[N]),
// A K-major, B row-major (a weight read as stored: no transpose pass); M % 256 == 0,
// N % 320 == 0, K % 64 == 0 (validated by the binding).
hipError_t gemm_nn64_launch(const bf16* A, const bf16* B, bf16* C, const bf16* bias, int M, int N, int K, int lda,
                            int ldb, int ldc, hipStream_t st) {
  gemm::Args a{A, B, C, bias, nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, 1,
               M / 256, N / 320, 0, 27, 0, 0, nullptr, nullptr, 0, 0, 0};
  return gemm::launch_nn64<gemm::EPI_BF16>(a, st);
}

static int g_tn_group_m = 0;  // m-tiles per tile-order group of the TN kernel (0: 8)
void gemm_set_tn_group_m(int g) { g_tn_group_m = g; }

// TN weight-gradient GEMM on the full-line kernel (algo 25): c[M][N] (+)= a[K][M]^T b[K][N],
// lockstep split over `slices` (> 1: fp32 slabs in ws, combined by a reduce launch).
hipError_t gemm_tn64_launch(int bm, bool accumulate, const bf16* A, const bf16* B, bf16* C, int M, int N, int K,
                            int lda, int ldb, int ldc, int slices, float* ws, hipStream_t st, int* tickets) {
  // tickets != null: the last arriving slice of each tile combines (algo 26), else a reduce launch (25)
  gemm::Args a{A, B, C, nullptr, nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, 1,
               (M + bm - 1) / bm, N / 320, 0, tickets ? 26 : 25, slices, 0, ws, tickets, 0, g_tn_group_m, 0};
  if (bm == 256) return accumulate ? gemm::launch_tn64<256, gemm::EPI_BF16_ACC>(a, st)
                                   : gemm::launch_tn64<256, gemm::EPI_BF16>(a, st);
  if (bm == 192) return accumulate ? gemm::launch_tn64<192, gemm::EPI_BF16_ACC>(a, st)
                                   : gemm::launch_tn64<192, gemm::EPI_BF16>(a, st);
  return hipErrorInvalidValue;
}

// Host entry: shapes are validated by the caller (bindings.cpp).
// 0: the default tile-order group -- 4 m-tiles at M >= 16384 (the training step's 32768
// rows: 101.4-102.0k vs 101.1k tok/s at 8, 100.7-101.3k at 2, 100.0-100.3k at 16 on one
// box, profiles/step_ab_group_m_r6.txt), 8 below (the serving prefill chunks, as tuned)
static int g_group_m = 0;
void gemm_set_group_m(int g) { g_group_m = g; }
static int g_tail_first = 0;  // algo 9 split tails dispatched first (see Args::tail_first)
void gemm_set_tail_first(int v) { g_tail_first = v; }

hipError_t gemm_launch(int layout, int epi, int bm, int bn, const bf16* A, const bf16* B, void* C,
                       const bf16* bias, const bf16* Z, bf16* Zout, float* dbias, int M, int N,
                       int K, int lda, int ldb, int ldc, int splitk, int algo, hipStream_t st,
                       int tfull, int tS, float* tws, int* tcnt, int bpack) {
  gemm::Args a{A, B, C, bias, Z, Zout, dbias, M, N, K, lda, ldb, ldc, splitk,
               (algo == 5 || algo == 15) ? (M + bm - 1) / bm : M / bm, N / bn, (long long)M * ldc, algo, tfull, tS, tws, tcnt,
               bpack, algo % 10 != 9 ? 0 : (g_group_m > 0 ? g_group_m : (M >= 16384 ? 4 : 8)), g_tail_first};
  if (bm == 256 && bn == 256) return gemm::launch_epi<256, 256>(layout, epi, a, st);
  if (bm == 256 && bn == 320) return gemm::launch_epi<256, 320>(layout, epi, a, st);
  if (bm == 128 && bn == 320) return gemm::launch_epi<128, 320>(layout, epi, a, st);
  return hipErrorInvalidValue;
}

// Split-K tail plan for a grid of whole tiles over `slots` resident workgroups: the
// tiles past the last full round are split into S K-slices (S <= max_split, >= 8
// K-steps of `ks` per slice, tail workgroups divisible over the 8 XCDs).
void gemm_tail_plan(int tiles, int K, int ks, int slots, int max_split, int* full, int* S) {
  int f = tiles, s = 1;
  const int tail = tiles % slots;
  if (max_split > 1 && tail > 0 && tail * 2 <= slots) {
    int cand = slots / tail;
    if (cand > max_split) cand = max_split;
    while (cand > 1 && ((K / ks) / cand < 8 || (tail * cand) % 8 != 0)) --cand;
    if (cand > 1 && (tiles - tail) % 8 == 0) {
      f = tiles - tail;
      s = cand;
    }
  }
  *full = f;
  *S = s;
}

void transpose_bf16(const bf16* in, bf16* out, int R, int C, hipStream_t st) {
  hipLaunchKernelGGL(gemm::transpose_bf16_kernel, dim3((R / 64) * (C / 64)), dim3(256), 0, st, in, out, R, C);
}

void gemm_splitk_reduce(const float* part, int S, long long slab, bf16* out, int M, int N, int ldc,
                        bool accumulate, hipStream_t st) {
  const long long total4 = (long long)M * (N / 4);
  int grid = (int)std::min<long long>((total4 + 255) / 256, 2048);
  hipLaunchKernelGGL(gemm::splitk_reduce_kernel, dim3(grid), dim3(256), 0, st, part, S, slab, out, M,
                     N, ldc, accumulate);
}

}  // namespace caamd
