// Second-generation gfx950 bf16 GEMM for the GPT-2-XL training step: TWO
// workgroups per CU, so one workgroup's epilogue (output stores, GELU, the
// dGELU bias-gradient sums, the split-K combine) runs while the other keeps the
// matrix pipes busy, plus a split-K "tail" that removes the half-empty last
// round of output tiles.
//
//   C[M,N] (+)= sum_k A(m,k) * B(k,n), fp32 accumulate, fused epilogues (below).
//   layout 0 (NT): A(m,k) = A[m*lda + k], B(k,n) = B[n*ldb + k]   (y = x W^T, dx = dy (W^T)^T)
//   layout 2 (TN): A(m,k) = A[k*lda + m], B(k,n) = B[k*ldb + n]   (dW = dy^T x)
//
// Why this shape (measured on the first-generation kernel, gemm.hip, at
// 32768 x 6400 x 1600): one 147 KB workgroup per CU left the matrix pipes idle
// during every tile's epilogue -- removing the stores alone took 612 -> 482 us
// (profiles/gemm_ablation.jsonl), and the fused GELU / dGELU epilogues, which
// move twice the bytes, ran at 0.88-0.94 PF/s against 1.16 for the plain one.
// And the N = 1600 GEMMs (more than half of the step's fwd/dgrad FLOPs) have
// 640 tiles of 256 x 320 = 2.5 rounds over 256 CUs, so the last round ran half
// empty.
//
// Design:
//  * 256-thread workgroup = 4 waves (one per SIMD), 2 x 2 over a BM x BN =
//    256 x 160 tile, each wave 128 x 80 (8 x 5 fragments of 16 x 16, 160 fp32
//    accumulators per lane). __launch_bounds__(256, 2): <= 256 VGPRs so two
//    workgroups share every CU; each SIMD then holds one wave of each and its
//    matrix pipe is fed by whichever of the two is in its MFMA segment.
//  * K-step 32, a 3-stage LDS ring of (256 + 160) x 32 bf16 = 26 KiB per stage
//    (78 KiB per workgroup, 156 KiB for the pair), filled by LDS-DMA
//    (`global_load_lds_dwordx4`) two K-steps ahead; counted `vmcnt` waits and
//    raw `s_barrier` (never `__syncthreads()` in the loop, whose implied
//    vmcnt(0) would drain the prefetch); one barrier per K-step:
//       DMA(t+2) | ds_read frags(t) | vmcnt(retire t+1) | lgkmcnt(0) | barrier | MFMA(t)
//    RAW: step t+1 is read only after the barrier that follows every wave's
//    wait for its own DMA(t+1). WAR: DMA(t+2) overwrites stage (t-1)%3, whose
//    reads all completed (lgkmcnt(0)) before barrier t-1, which precedes it.
//  * LDS images XOR-swizzled on the DMA source address (the DMA writes
//    lane-linear), read with the same XOR (ds_read_b128 for K-major 64-byte rows,
//    ds_read_b64_tr_b16 for MN-major rows).
//  * v_mfma_f32_16x16x32_bf16 with the operands swapped (D = B_frag x A_frag):
//    a lane owns 4 consecutive output columns of one row.
//  * Work mapping: the 8 XCDs each own 1/8 of the whole tiles (contiguous,
//    GROUP_M-grouped, so neighbouring tiles share A/B panels in one L2) followed
//    by 1/8 of the tail work. Tail = the tiles past the last full round of
//    2 x CUs workgroups, each split over S K-slices so the tail fills a round.
//    Slices write fp32 partials (lane-linear, 1 KiB per wave store) to a slab;
//    the last arriver (agent-scope ticket, the release/acquire recipe of
//    cdna_hip_programming.md §5 "Projection GEMM" item 2) adds the other slabs
//    and runs the normal epilogue. The ticket is reset by the last arriver.
//  * Ragged M (weight-gradient outputs with 1600 / 4800 rows): A rows/columns
//    past M are clamped to row M-1 on load and never stored.
//  * Epilogue staged through the (now idle) LDS ring: bf16 image of half the
//    tile, then 16-byte row stores with bias / GELU / dGELU / accumulate applied
//    on the way (per-fragment stores touch 16 rows x 8 B per instruction).
#include "common.h"

#include <mutex>
#include <unordered_set>

namespace caamd {
namespace g2 {

typedef __attribute__((address_space(3))) char lds_char;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int NT = 256;   // threads per workgroup (4 waves)
constexpr int KS = 32;    // K-step
constexpr int NST = 3;    // LDS ring stages
constexpr int GROUP_M = 8;

enum Epi : int {
  EPI_BF16 = 0,       // C = acc (+ bias[n])
  EPI_BF16_ACC = 1,   // C = C + acc (+ bias[n])
  EPI_BIAS_GELU = 3,  // Zout = acc + bias ; C = gelu(Zout)
  EPI_DGELU = 4,      // C = acc * gelu'(Z) ; dbias[n] += colsum(C)
};

// gelu_tanh / gelu_tanh_grad: common.h

struct Args {
  const bf16* A;
  const bf16* B;
  bf16* C;
  const bf16* bias;  // [N] or null
  const bf16* Z;     // dGELU: pre-activation [M, ldc]
  bf16* Zout;        // bias+GELU: pre-activation out
  float* dbias;      // dGELU: [N] fp32, accumulated
  float* ws;         // tail slabs: [tail tiles][S][BM*BN] fp32
  int* cnt;          // tail tickets: [tail tiles], zero between launches
  int M, N, K, lda, ldb, ldc;
  int tiles_m, tiles_n;
  int full;          // whole tiles (multiple of 8 when S > 1)
  int S;             // K-slices per tail tile (1: no tail split)
};

// ---- LDS images ----------------------------------------------------------------------
// K-major operand, 32-deep K-step: R rows of 64 bytes; 16-B chunk c of row r is stored
// at chunk position c ^ kswz(r). Conflict-free ds_read_b128 of 16 rows x 16 B per group.
__device__ __forceinline__ int kswz(int row) { return ((row >> 3) & 1) * 2; }
// MN-major operand: 32 k-rows of R elements (R/8 chunks); chunk c of k-row k at c ^ mswz(k).
template <int R>
__device__ __forceinline__ int mswz(int k) {
  if constexpr ((R % 128) == 0) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else if constexpr ((R % 64) == 0) return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
  else return 2 * ((k >> 3) & 1);  // R = 160: 20 chunks per row, XOR stays inside groups of 4
                                   // (conflict-free tr16 reads: tools/gemm_swizzle_check.py)
}

// DMA instructions a wave issues for one K-step of an R-row operand.
template <int R>
__host__ __device__ constexpr int dma_full() { return (R * KS * 2) / (NT * 16); }
template <int R>
__host__ __device__ constexpr int dma_rem() { return (R * KS * 2) - dma_full<R>() * NT * 16; }

template <int R, bool KMAJ>
__device__ __forceinline__ void dma_one(const bf16* __restrict__ X, int ld, int r0, int rlast, int k0,
                                        lds_char* dst, int j, int wid, int lane) {
  const int lin = j * NT + wid * 64 + lane;  // 16-B chunk index in LDS order
  const bf16* src;
  if constexpr (KMAJ) {
    const int row = lin >> 2, pos = lin & 3;
    const int c = pos ^ kswz(row);
    const int gr = min(r0 + row, rlast);
    src = X + (size_t)gr * ld + k0 + c * 8;
  } else {
    constexpr int CPR = R / 8;
    const int k = lin / CPR, pos = lin - k * CPR;
    const int c = pos ^ mswz<R>(k);
    const int gc = min(r0 + c * 8, rlast);  // rlast: last valid 8-aligned column
    src = X + (size_t)(k0 + k) * ld + gc;
  }
  __builtin_amdgcn_global_load_lds((const void*)src,
                                   (void __attribute__((address_space(3)))*)(dst + (j * NT + wid * 64) * 16), 16, 0, 0);
}

template <int R, bool KMAJ>
__device__ __forceinline__ void dma_step(const bf16* __restrict__ X, int ld, int r0, int rlast, int k0,
                                         lds_char* dst, int wid, int lane) {
  constexpr int FULL = dma_full<R>(), REM = dma_rem<R>();
  static_assert(REM % 1024 == 0, "partial DMA round must be whole waves");
#pragma unroll
  for (int j = 0; j < FULL; ++j) dma_one<R, KMAJ>(X, ld, r0, rlast, k0, dst, j, wid, lane);
  if constexpr (REM > 0) {
    if (wid * 1024 < REM) dma_one<R, KMAJ>(X, ld, r0, rlast, k0, dst, FULL, wid, lane);
  }
}

__device__ __forceinline__ bf16x8_t frag_k(const lds_char* img, int rr, int lane) {
  const int row = rr + (lane & 15);
  const int pos = (lane >> 4) ^ kswz(row);
  typedef __attribute__((address_space(3))) const bf16x8_t lds_bf16x8;
  return *(lds_bf16x8*)(img + row * 64 + pos * 16);
}
template <int R>
__device__ __forceinline__ bf16x8_t frag_m(const lds_char* img, int rr, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int m = rr + 4 * p;
  const int chunk = m >> 3;
  const int within = (p & 1) * 8;
  s16x4 lo, hi;
  {
    const int k = 8 * g + q;
    lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (R * 2) + (chunk ^ mswz<R>(k)) * 16 + within));
  }
  {
    const int k = 8 * g + 4 + q;
    hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (R * 2) + (chunk ^ mswz<R>(k)) * 16 + within));
  }
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- epilogue ------------------------------------------------------------------------
template <int BM, int BN, int TM, int TN, int EPI>
__device__ __forceinline__ void epilogue(const Args& p, f32x4 (&acc)[TM][TN], int m0, int n0, int wr, int wc,
                                         int lane, lds_char* smem, int tid) {
  constexpr int ROWB = BN * 2 + 16;  // padded bf16 image row
  constexpr int TMH = TM / 2;
  constexpr int HR = BM / 2;         // image rows per pass
  constexpr int CPR = BN / 8;        // 16-B chunks per row
  constexpr int RG = NT / CPR;       // row groups
  constexpr int ACTIVE = RG * CPR;
  constexpr int RITERS = (HR + RG - 1) / RG;
  static_assert(HR * ROWB <= NST * (BM + BN) * KS * 2, "epilogue image must fit the ring");
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
  typedef __attribute__((address_space(3))) const bf16x8_t lds_bf16x8;
  const int mrow = lane & 15, ncol = 4 * (lane >> 4);
  const int c = tid % CPR, rg = tid / CPR;
  const int n = n0 + c * 8;
  float bv[8], dsum[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) bv[r] = dsum[r] = 0.f;
  if constexpr (EPI != EPI_DGELU) {
    if (p.bias && tid < ACTIVE) {
      bf16x8_t b8 = *reinterpret_cast<const bf16x8_t*>(p.bias + n);
#pragma unroll
      for (int r = 0; r < 8; ++r) bv[r] = (float)b8[r];
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();  // image free (previous pass / ring reads done)
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
    __syncthreads();
    if (tid < ACTIVE) {
      for (int it = 0; it < RITERS; ++it) {
        const int ir = it * RG + rg;
        if (ir >= HR) break;
        const int wr_ = ir / (TMH * 16), rem = ir - wr_ * (TMH * 16);
        const int m = m0 + wr_ * (TM * 16) + h * (TMH * 16) + rem;
        if (m >= p.M) continue;
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
          bf16x8_t prev = *reinterpret_cast<const bf16x8_t*>(p.C + off);
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
          bf16x8_t z = *reinterpret_cast<const bf16x8_t*>(p.Z + off);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            o[r] = (bf16)(f[r] * gelu_tanh_grad((float)z[r]));
            dsum[r] += (float)o[r];
          }
        }
        *reinterpret_cast<bf16x8_t*>(p.C + off) = o;
      }
    }
  }
  if constexpr (EPI == EPI_DGELU) {
    typedef __attribute__((address_space(3))) float lds_float;
    lds_float* red = (lds_float*)smem;
    __syncthreads();
    if (tid < ACTIVE) {
#pragma unroll
      for (int r = 0; r < 8; ++r) red[rg * (CPR * 8) + c * 8 + r] = dsum[r];
    }
    __syncthreads();
    for (int col = tid; col < CPR * 8; col += NT) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < RG; ++g) t += red[g * (CPR * 8) + col];
      atomicAdd(p.dbias + n0 + col, t);
    }
  }
}

// ---- kernel --------------------------------------------------------------------------
template <int BM, int BN, bool AK, bool BK_, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm2_kernel(Args p) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int A_ST = BM * KS * 2, B_ST = BN * KS * 2, ST = A_ST + B_ST;
  static_assert(dma_rem<BM>() == 0, "A stage must be whole DMA rounds");
  static_assert(A_ST % 1024 == 0 && B_ST % 1024 == 0, "stage must be whole KiB");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  // ---- work mapping (XCD-aware; whole tiles first, then the split tail) --------------
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, loc = bid >> 3;
  int tile, slice = 0;
  if (p.S == 1) {
    const int q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  } else {
    const int nfx = p.full >> 3;
    const int ntx = (nwg - p.full) >> 3;
    if (loc < nfx) {
      tile = xcd * nfx + loc;
    } else {
      const int s = xcd * ntx + (loc - nfx);
      tile = p.full + s / p.S;
      slice = s - (s / p.S) * p.S;
    }
  }
  const bool split = tile >= p.full && p.S > 1;
  const int group_sz = GROUP_M * p.tiles_n;
  const int g = tile / group_sz;
  const int first_m = g * GROUP_M;
  const int gm = min(p.tiles_m - first_m, GROUP_M);
  const int tin = tile - g * group_sz;
  const int m0 = (first_m + tin % gm) * BM, n0 = (tin / gm) * BN;

  const int ns_total = p.K / KS;
  int s0 = 0, nk = ns_total;
  if (split) {
    const int per = (ns_total + p.S - 1) / p.S;
    s0 = slice * per;
    nk = max(0, min(ns_total, s0 + per) - s0);
  }
  // last valid row (K-major A) or 8-aligned column (MN-major A) of this tile
  const int a_last = AK ? p.M - 1 : p.M - 8;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto dma = [&](int t, lds_char* base) {
    const int k0 = (s0 + t) * KS;
    dma_step<BM, AK>(p.A, p.lda, m0, a_last, k0, base, wid, lane);
    dma_step<BN, BK_>(p.B, p.ldb, n0, BK_ ? p.N - 1 : p.N - 8, k0, base + A_ST, wid, lane);
  };
  // DMAs this wave issues per step: the B stage may end in a partial round (BN = 160)
  const bool more = wid * 1024 < dma_rem<BN>();
  constexpr int CNT_LO = dma_full<BM>() + dma_full<BN>();
  constexpr int CNT_HI = CNT_LO + (dma_rem<BN>() > 0 ? 1 : 0);

  if (nk > 0) {
    lds_char* st0 = smem;
    lds_char* st1 = smem + ST;
    lds_char* st2 = smem + 2 * ST;
    dma(0, st0);
    if (nk > 1) {
      dma(1, st1);
      if (more) wait_vm<CNT_HI>(); else wait_vm<CNT_LO>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    for (int t = 0; t < nk; ++t) {
      // stage t in st0, t+1 in st1, t+2 goes to st2
      if (t + 2 < nk) dma(t + 2, st2);
      const lds_char* As = st0;
      const lds_char* Bs = st0 + A_ST;
      bf16x8_t bf[TN], af[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int rr = wc * (TN * 16) + j * 16;
        if constexpr (BK_) bf[j] = frag_k(Bs, rr, lane);
        else bf[j] = frag_m<BN>(Bs, rr, lane);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rr = wr * (TM * 16) + i * 16;
        if constexpr (AK) af[i] = frag_k(As, rr, lane);
        else af[i] = frag_m<BM>(As, rr, lane);
      }
      if (t + 2 < nk) {
        if (more) wait_vm<CNT_HI>(); else wait_vm<CNT_LO>();
      } else {
        wait_vm<0>();
      }
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
      lds_char* tmp = st0;
      st0 = st1;
      st1 = st2;
      st2 = tmp;
    }
  }

  if (split) {
    // ---- split-K tail: publish this slice, the last arriver combines ------------------
    const int tt = tile - p.full;
    constexpr int SLAB = BM * BN;  // floats per slice
    float* mine = p.ws + ((size_t)tt * p.S + slice) * SLAB;
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
      const int old = __hip_atomic_fetch_add(p.cnt + tt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == p.S - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        p.cnt[tt] = 0;  // ready for the next launch
      }
      *flag = last;
    }
    __syncthreads();
    const int last = *flag;
    if (!last) return;
    for (int s = 0; s < p.S; ++s) {
      if (s == slice) continue;
      const float* other = p.ws + ((size_t)tt * p.S + s) * SLAB;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] += *reinterpret_cast<const f32x4*>(other + ((size_t)((wid * TM + i) * TN + j) * 64 + lane) * 4);
    }
  }
  epilogue<BM, BN, TM, TN, EPI>(p, acc, m0, n0, wr, wc, lane, smem, tid);
}

static void ensure_lds(const void* k, int bytes) {
  static std::mutex mu;
  static std::unordered_set<const void*> done;
  std::lock_guard<std::mutex> g(mu);
  if (done.insert(k).second) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

template <int BM, int BN, bool AK, bool BK_, int EPI>
static hipError_t launch(const Args& a, int grid, hipStream_t st) {
  auto k = gemm2_kernel<BM, BN, AK, BK_, EPI>;
  constexpr int lds = NST * (BM + BN) * KS * 2;
  ensure_lds((const void*)k, lds);
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, st, a);
  return hipGetLastError();
}

template <int EPI>
static hipError_t launch_layout(int layout, const Args& a, int grid, hipStream_t st) {
  if (layout == 0) return launch<256, 160, true, true, EPI>(a, grid, st);
  if constexpr (EPI == EPI_BF16 || EPI == EPI_BF16_ACC) {
    if (layout == 2) return launch<256, 160, false, false, EPI>(a, grid, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace g2

// Plan of a launch: whole tiles, tail split and grid. `slots` = workgroups resident at
// once (2 per CU). Returns the workspace floats / tickets the tail needs.
void gemm2_plan(int M, int N, int K, int slots, int max_split, int* full, int* S, int* grid,
                long long* ws_floats, int* tickets) {
  const int tm = (M + 255) / 256, tn = N / 160;
  const int T = tm * tn;
  int f = T, s = 1;
  const int tail = T % slots;
  if (max_split > 1 && tail > 0 && tail * 2 <= slots) {
    int cand = slots / tail;
    if (cand > max_split) cand = max_split;
    // >= 8 K-steps per slice, and the tail's workgroups divisible over the 8 XCDs
    while (cand > 1 && ((K / 32) / cand < 8 || (tail * cand) % 8 != 0)) --cand;
    const int ff = T - tail;
    if (cand > 1 && ff % 8 == 0) {
      f = ff;
      s = cand;
    }
  }
  *full = f;
  *S = s;
  *grid = s > 1 ? f + (T - f) * s : T;
  *ws_floats = s > 1 ? (long long)(T - f) * s * 256 * 160 : 0;
  *tickets = s > 1 ? T - f : 0;
}

hipError_t gemm2_launch(int layout, int epi, const bf16* A, const bf16* B, bf16* C, const bf16* bias,
                        const bf16* Z, bf16* Zout, float* dbias, float* ws, int* cnt, int M, int N, int K,
                        int lda, int ldb, int ldc, int full, int S, int grid, hipStream_t st) {
  g2::Args a{A, B, C, bias, Z, Zout, dbias, ws, cnt, M, N, K, lda, ldb, ldc, (M + 255) / 256, N / 160,
             full, S};
  switch (epi) {
    case g2::EPI_BF16: return g2::launch_layout<g2::EPI_BF16>(layout, a, grid, st);
    case g2::EPI_BF16_ACC: return g2::launch_layout<g2::EPI_BF16_ACC>(layout, a, grid, st);
    case g2::EPI_BIAS_GELU: return layout == 0 ? g2::launch<256, 160, true, true, g2::EPI_BIAS_GELU>(a, grid, st)
                                               : hipErrorInvalidValue;
    case g2::EPI_DGELU: return layout == 0 ? g2::launch<256, 160, true, true, g2::EPI_DGELU>(a, grid, st)
                                           : hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

}  // namespace caamd
