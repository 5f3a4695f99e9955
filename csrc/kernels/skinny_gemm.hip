// Decode-time ("skinny") GEMM for LLM serving on gfx950:
//
//   Y[M, N] = X[M, K] . W[N, K]^T      M <= 128 (one row per running sequence)
//
// At decode batch sizes every weight element is used M times, so the GEMM is a
// stream over W (Llama-3-8B: 436 MB per layer) and its floor is W bytes / HBM
// bandwidth. hipBLASLt's selections for these shapes ran at 2.0-4.1 TB/s of weight
// traffic (profiles/llm_decode_prof_r2_smallk.md). Design:
//
//  * A workgroup (4 waves) owns a 64-column slab of Y and one K chunk (split-K
//    across workgroups so every shape launches enough workgroups); each wave owns
//    32 of the (padded) 128 output rows, so no cross-wave reduction is needed and
//    the four waves read the same W lines through the CU's L1.
//  * Per 64-k step the W tile (64 rows x 128 B) and the X tile (128 rows x 128 B)
//    arrive by LDS-DMA, one 128-byte line per row (8 lanes each), into a 3-stage
//    ring two steps ahead (48 KB in flight per workgroup); each W byte is fetched
//    once and shared by the four waves through LDS (a first version that loaded
//    operands straight into registers, one 32-byte run per lane and row, reached
//    only 0.4-0.8 TB/s).
//  * With split-K the workgroup writes an fp32 partial tile, and the last workgroup of a column
//    slab to arrive (agent-scope release/acquire counter) sums the partials and
//    writes bf16 Y, then re-arms the counter -- one launch, graph-replay safe.
#include "common.h"

namespace caamd {
namespace skinny {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 256;   // threads per workgroup
constexpr int BN = 64;    // output columns per workgroup
constexpr int KS = 64;    // k per step (4 MFMAs per accumulator)
constexpr int KI = KS / 16;

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) char lds_t;

// 16-B chunk c of image row `row` (128-B rows) sits at chunk c ^ swz(row): the
// ds_read_b128 operand reads (lane: row R0 + (l & 31), chunk 2i + (l >> 5)) hit 16
// distinct slots in each b128 lane group (the flash_attn_d64.hip swizzle).
__device__ __forceinline__ int swz(int row) {
  const int x = (row >> 1) & 7;
  return x ^ ((x & 1) << 2);
}
// rows [0, R) x k [k0, k0 + 64) of G (row stride ld; rows clamped to rmax) -> LDS
// image, NT threads, R * 8 / NT pieces of 16 B per thread (one 128-B line per row)
template <int R>
__device__ __forceinline__ void dma_rows(const bf16* __restrict__ G, size_t ld, int r0, int rmax, int k0,
                                         lds_t* dst, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < R * 8 / NT; ++j) {
    const int lin = j * NT + wave * 64 + lane;
    const int row = lin >> 3, pos = lin & 7;
    const int c = pos ^ swz(row);
    const bf16* src = G + (size_t)min(r0 + row, rmax) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (void __attribute__((address_space(3)))*)(dst + (j * NT + wave * 64) * 16),
                                     16, 0, 0);
  }
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Workgroup barrier that leaves younger DMA in flight: __syncthreads() compiles to
// `s_waitcnt vmcnt(0) lgkmcnt(0); s_barrier`, which would drain the prefetched
// steps at every iteration. The caller has already waited for the step it needs
// (counted vmcnt); LDS reads must be complete before a stage is overwritten.
__device__ __forceinline__ void barrier_keep_dma() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Per 64-k step the workgroup DMAs a 64-row W tile (8 KB, 2 pieces per wave) and
// the 128-row X tile (16 KB, 4 pieces per wave) into one of three LDS stages; the
// DMA runs two steps ahead. Wave w owns output rows [32w, 32w + 32) (rows >= M are
// clamped copies, never stored) for both 32-column blocks: 8 MFMAs per step.
constexpr int W_IMG = BN * 128, X_IMG = 128 * 128, STAGE = W_IMG + X_IMG, NSTAGE = 3;
constexpr int PIECES = (BN + 128) * 8 / NT;  // DMA instructions per wave per step

__global__ __launch_bounds__(NT, 2) void skinny_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                       bf16* __restrict__ Y, float* __restrict__ part,
                                                       unsigned* __restrict__ counters, int M, int N, int K,
                                                       int ldx, int kchunk, int splits) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_t* smem = (lds_t*)smem_raw;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int slab = blockIdx.x, split = blockIdx.y;
  const int n0 = slab * BN;
  const int kb0 = split * kchunk;
  const int nsteps = kchunk / KS;

  auto issue = [&](int t) {
    lds_t* st = smem + (t % NSTAGE) * STAGE;
    dma_rows<BN>(W, (size_t)K, n0, N - 1, kb0 + t * KS, st, wave, lane);
    dma_rows<128>(X, (size_t)ldx, 0, M - 1, kb0 + t * KS, st + W_IMG, wave, lane);
  };
  // lane-constant read offsets: chunk 2i + h of rows r (+32 cb / +32 wave)
  int off[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) off[i] = r * 128 + (((2 * i + h) ^ swz(r)) << 4);

  f32x16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;

  issue(0);
  if (nsteps > 1) issue(1);
  typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
  for (int t = 0; t < nsteps; ++t) {
    if (t + 1 < nsteps) wait_vm<PIECES>();  // step t landed, step t + 1 may still fly
    else wait_vm<0>();
    barrier_keep_dma();  // every wave's pieces of step t landed; stage (t + 2) % 3 is free
    if (t + 2 < nsteps) issue(t + 2);
    const lds_t* st = smem + (t % NSTAGE) * STAGE;
    bf16x8 a[KI], b0[KI], b1[KI];
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      b0[i] = *(lds_bf16x8*)(st + off[i]);
      b1[i] = *(lds_bf16x8*)(st + off[i] + 32 * 128);
      a[i] = *(lds_bf16x8*)(st + W_IMG + off[i] + wave * 32 * 128);
    }
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      acc0 = mfma32(a[i], b0[i], acc0);
      acc1 = mfma32(a[i], b1[i], acc1);
    }
  }

  // acc layout: reg i of lane (r, h) -> row 32 wave + (i & 3) + 8 (i >> 2) + 4 h, column 32 cb + r
  if (splits == 1) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = 32 * wave + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (m < M) {
        Y[(size_t)m * N + n0 + r] = (bf16)acc0[i];
        Y[(size_t)m * N + n0 + 32 + r] = (bf16)acc1[i];
      }
    }
    return;
  }
  // split-K: publish this split's fp32 partial tile [128 rows][64 cols], the last
  // split of the slab to arrive sums them
  float* mine = part + ((size_t)split * (N / BN) + slab) * (128 * BN);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = 32 * wave + (i & 3) + 8 * (i >> 2) + 4 * h;
    mine[m * BN + r] = acc0[i];
    mine[m * BN + 32 + r] = acc1[i];
  }
  __shared__ unsigned last;
  wait_vm<0>();  // this wave's partial stores done
  __syncthreads();
  if (tid == 0) {
    // release this workgroup's partial tile and count it (agent scope: other XCDs)
    const unsigned prev = __hip_atomic_fetch_add(counters + slab, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == (unsigned)(splits - 1);
  }
  __syncthreads();
  if (!last) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // see the other splits' partials
  const int rows = min(M, 128);
  for (int i = tid; i < rows * (BN / 4); i += NT) {
    const int m = i / (BN / 4), c = (i % (BN / 4)) * 4;
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < splits; ++sp)
      sum += __builtin_nontemporal_load(
          reinterpret_cast<const f32x4*>(part + ((size_t)sp * (N / BN) + slab) * (128 * BN) + m * BN + c));
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (bf16)sum[j];
    *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n0 + c) = o;
  }
  if (tid == 0) __hip_atomic_store(counters + slab, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
}

}  // namespace skinny

// Host entry. Shapes are validated by the binding: M <= 128, N % 64 == 0,
// K % (128 * splits) == 0. part: splits * N * 128 floats; counters: N / 64
// zero-initialised uints (every launch leaves them zeroed).
hipError_t skinny_gemm_launch(const bf16* X, const bf16* W, bf16* Y, float* part, unsigned* counters, int M,
                              int N, int K, int ldx, int splits, hipStream_t st) {
  if (M < 1 || M > 128 || N % skinny::BN || splits < 1 || K % (2 * skinny::KS * splits)) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)skinny::skinny_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              skinny::NSTAGE * skinny::STAGE);
    attr = true;
  }
  hipLaunchKernelGGL(skinny::skinny_kernel, dim3(N / skinny::BN, splits), dim3(skinny::NT),
                     skinny::NSTAGE * skinny::STAGE, st, X, W, Y, part, counters, M, N, K, ldx, K / splits, splits);
  return hipGetLastError();
}

}  // namespace caamd
