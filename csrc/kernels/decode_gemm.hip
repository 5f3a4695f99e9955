// Decode GEMM v3 for LLM serving on gfx950 (Llama decode, batch <= 128):
//
//   Y[M, N] = X[M, K] . W[N, K]^T            M <= 128, W streamed from HBM once
//   SwiGLU:  Y[M, N/2] = silu(G) * U with W's rows interleaved in 64-row blocks
//            (block b = gate rows [64b, 64b+64) then up rows [64b, 64b+64); the
//            model permutes w_gate_up once at load time, ops/llm.py)
//
// What the first decode kernel (skinny_gemm.hip) measured: 64-column tiles stage
// the 128-row X tile (16 KB per 64-k step) next to only 8 KB of W, so every CU's
// load path moved 3x the weight bytes, and its split-K was fixed per shape; it ran
// level with hipBLASLt (2.0-4.1 TB/s of weights, profiles/skinny_gemm_v2_experiment.md).
//
// Design (MI355X_MICROARCH.md "ldsdma-fill", "nt-weights", "ring-gemm"):
//  * one 256-thread workgroup (4 waves, one per SIMD) per CU owns a 128-column
//    slab of Y (all <= 128 rows) and a K range (split-K over workgroups so the
//    launch covers the CUs); W and X tiles are staged 1:1 (16 KB each per 64-k step);
//  * a 4-stage LDS ring (128 KiB) filled by LDS-DMA three steps ahead, counted
//    vmcnt + raw s_barrier (no vmcnt(0) in the loop); weights with the
//    non-temporal policy (read once), X with the default policy (L2-resident,
//    re-read by every workgroup);
//  * wave w owns columns [32w, 32w+32) of the slab and all 128 rows: per 16-k
//    substep one W fragment and four X fragments (ds_read_b128 on an XOR-swizzled
//    image), four v_mfma_f32_32x32x16_bf16;
//  * split-K: fp32 partial tiles in fragment order (1 KiB per wave store), an
//    agent-scope release -> ticket -> acquire, and the LAST arriving split sums the
//    partials in registers and runs the epilogue (no extra launch, nothing waits);
//    the ticket is re-armed by the last arriver (graph-replay safe);
//  * epilogues: bf16 store, residual add (Y = acc + R), or SwiGLU (waves 2,3 hand
//    their "up" columns to waves 0,1 through LDS).
#include "common.h"

#include <cstdlib>
#include <mutex>
#include <unordered_set>

namespace caamd {
namespace dg {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) char lds_t;

constexpr int NT = 256;          // consumer threads (4 waves); the workgroup adds 4 producer waves
constexpr int WG = 2 * NT;
constexpr int BN = 128;          // output columns per workgroup
constexpr int KS = 64;           // k per step
constexpr int IMG = 128 * 128;   // one step of 128 rows x 64 k (16 KiB), a W or an X image
constexpr int PPW = IMG / (128 * 16);  // DMA pieces per producer wave per image (two waves per image): 8

enum Epi : int { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2 };

__device__ __forceinline__ int swz(int row) {
  const int x = (row >> 1) & 7;
  return x ^ ((x & 1) << 2);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ds_read_b128 outside the compiler's waitcnt tracking: the waits below name the
// destination registers, so counted lgkmcnt waits replace the compiler's lgkmcnt(0)
__device__ __forceinline__ bf16x8 ldsr(const lds_t* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((unsigned)(size_t)p) : "memory");
  return v;
}

template <int N>
__device__ __forceinline__ void wait_frags(bf16x8& b, bf16x8 (&a)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%5)" : "+v"(b), "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]) : "n"(N)
               : "memory");
}

// leave `younger` later steps (PER pieces each) in flight
template <int PER>
__device__ __forceinline__ void wait_younger(int younger) {
  switch (younger) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<PER>(); break;
    case 2: wait_vm<2 * PER>(); break;
    case 3: wait_vm<3 * PER>(); break;
    case 4: wait_vm<4 * PER>(); break;
    case 5: wait_vm<5 * PER>(); break;
    default: wait_vm<6 * PER>(); break;
  }
}

// rows [r0, r0 + 128) x k [k0, k0 + 64) of G (row stride ld, rows clamped to rmax) by
// producer wave pw of 2: 128 rows x 8 chunks of 16 B = 8 pieces per lane; piece j of
// lane l is LDS chunk j*128 + pw*64 + l (lane-linear per wave), source chunk pos ^ swz(row).
template <int AUX>
__device__ __forceinline__ void dma_rows(const bf16* __restrict__ G, size_t ld, int r0, int rmax, int k0,
                                         lds_t* dst, int pw, int lane) {
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int lin = j * 128 + pw * 64 + lane;
    const int row = lin >> 3, pos = lin & 7;
    const int c = pos ^ swz(row);
    const bf16* src = G + (size_t)min(r0 + row, rmax) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (void __attribute__((address_space(3)))*)(dst + (j * 128 + pw * 64) * 16),
                                     16, 0, AUX);
  }
}

struct Args {
  const bf16* X;
  const bf16* W;
  bf16* Y;
  const bf16* R;     // residual (EPI_RESID), [M, ldy]
  float* part;       // split-K partials: [slabs][splits][BN*128] floats
  unsigned* tick;    // split-K tickets: [slabs], zero between launches
  int M, N, K, ldx, ldy, splits, kchunk;
  int ext;           // 1: split-K partials only, dg_reduce_kernel combines (own launch);
                     // 2: row-major partials, dg_reduce_norm_kernel combines
  float* ssp;        // RMSNorm folded in: per-row sums of squares of X, [slabs][splits][128]
                     // (nullptr: plain GEMM); the norm weight is folded into W's columns
  float eps;
};

// sum of squares of a lane's 8 X values (the RMSNorm statistic, accumulated while
// the X tiles stream through for the MFMAs)
__device__ __forceinline__ float sumsq8(const bf16x8& v, float acc) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bf16x2 p2 = {v[2 * e], v[2 * e + 1]};
    acc = __builtin_amdgcn_fdot2_f32_bf16(p2, p2, acc, false);  // v_dot2_f32_bf16
  }
  return acc;
}

// W prepacked (ops/llm.py pack_decode_weight): per 128-row slab and 64-k step the
// 16 KiB LDS image (swizzle included) is stored contiguously, so a stage is one
// linear 16 KiB read instead of 128 B from each of 128 rows 2K bytes apart.
__device__ __forceinline__ void dma_packed(const bf16* __restrict__ Wp, size_t img, lds_t* dst, int pw,
                                           int lane) {
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int lin = j * 128 + pw * 64 + lane;
    __builtin_amdgcn_global_load_lds((const void*)(Wp + img * (BN * 64) + lin * 8),
                                     (void __attribute__((address_space(3)))*)(dst + (j * 128 + pw * 64) * 16),
                                     16, 0, 2);
  }
}

// 8 waves with fixed roles. Waves 0-3 only read LDS and multiply; waves 4-5 stream W
// into a ring of NWS images (NWS-1 steps in flight: HBM latency x per-CU rate needs
// the depth), waves 6-7 stream X into a ring of NXS images (X is L2-resident: a short
// distance suffices). An LDS-DMA piece costs its wave 60-185 cycles of issue inside an
// MFMA phase (MI355X_MICROARCH.md "LDS-DMA piece issue cost"), so no DMA is issued by
// a computing wave; each producer's vmcnt tracks only its own stream, so the two
// rings run at different distances. All 8 waves share one barrier per step.
template <int EPI, bool PK, int NWS, int NXS>
__global__ __launch_bounds__(WG, 1) void decode_gemm_kernel(Args p) {
  constexpr int DW = NWS - 1, DX = NXS - 1;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_t* smem = (lds_t*)smem_raw;
  lds_t* wring = smem;
  lds_t* xring = smem + NWS * IMG;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool consumer = wave < 4, wprod = (wave >> 1) == 2, xprod = (wave >> 1) == 3;
  const int pw = wave & 1;
  const int slab = blockIdx.x, split = blockIdx.y;
  const int n0 = slab * BN;
  const int kb0 = split * p.kchunk;
  const int nsteps = min(p.kchunk, p.K - kb0) / KS;  // the last split may be shorter (ragged split-K)

  auto issue_w = [&](int t) {
    lds_t* st = wring + (t % NWS) * IMG;
    if constexpr (PK)
      dma_packed(p.W, (size_t)slab * (p.K / KS) + kb0 / KS + t, st, pw, lane);
    else
      dma_rows<2>(p.W, (size_t)p.K, n0, p.N - 1, kb0 + t * KS, st, pw, lane);  // nt: read once
  };
  auto issue_x = [&](int t) {
    dma_rows<0>(p.X, (size_t)p.ldx, 0, p.M - 1, kb0 + t * KS, xring + (t % NXS) * IMG, pw, lane);
  };

  const int r = lane & 31, h = lane >> 5;
  int off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) off[i] = r * 128 + (((2 * i + h) ^ swz(r)) << 4);

  f32x16 acc[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;
  float ssq = 0.f;  // producer wave pi = wave - 4, lane l: row 32 pi + (l & 31), half l >> 5
  const bool rn = p.ssp != nullptr;

  if (wprod)
    for (int t = 0; t < min(nsteps, DW); ++t) issue_w(t);
  if (xprod)
    for (int t = 0; t < min(nsteps, DX); ++t) issue_x(t);
  typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
  for (int t = 0; t < nsteps; ++t) {
    // step t landed; the younger steps of each stream stay in flight
    if (wprod) wait_younger<PPW>(min(nsteps - 1 - t, DW - 1));
    if (xprod) wait_younger<PPW>(min(nsteps - 1 - t, DX - 1));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // step t visible to all; slots (t-1) of both rings are free
    __builtin_amdgcn_sched_barrier(0);
    if (wprod && t + DW < nsteps) issue_w(t + DW);
    if (xprod && t + DX < nsteps) issue_x(t + DX);
    if (rn && !consumer) {
      // the RMSNorm statistic, off the MFMA waves and spread over the four producer
      // waves (one per SIMD): lane l of producer wave pi sums the squares of half
      // l >> 5 of row 32 pi + (l & 31) of step t's X image (4 of its 8 16-byte chunks;
      // the swizzle only permutes chunks within the row); slot t stays valid until
      // barrier t + 1
      const lds_t* xr = xring + (t % NXS) * IMG + (32 * (wave - 4) + (lane & 31)) * 128 + (lane >> 5) * 64;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bf16x8 v = *(const __attribute__((address_space(3))) bf16x8*)(xr + c * 16);
        ssq = sumsq8(v, ssq);
      }
    }
    if (consumer) {
      const lds_t* ws = wring + (t % NWS) * IMG;
      const lds_t* xs = xring + (t % NXS) * IMG;
      // fragment reads run two substeps ahead of the MFMAs (<= 10 in flight; lgkmcnt
      // counts to 15) with waits that name their registers: the LDS latency is exposed
      // once per step instead of once per substep
      bf16x8 b[4], a[4][4];
      auto rd = [&](int kk) {
        b[kk] = ldsr(ws + off[kk] + wave * 32 * 128);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) a[kk][mt] = ldsr(xs + off[kk] + mt * 32 * 128);
      };
      auto mm = [&](int kk) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kk][mt], b[kk], acc[mt], 0, 0, 0);
      };
      rd(0);
      rd(1);
      wait_frags<5>(b[0], a[0]);
      mm(0);
      rd(2);
      wait_frags<5>(b[1], a[1]);
      mm(1);
      rd(3);
      wait_frags<5>(b[2], a[2]);
      mm(2);
      wait_frags<0>(b[3], a[3]);
      mm(3);
    }
  }

  if (rn && !consumer) ssq += __shfl_xor(ssq, 32, 64);  // both halves: row 32 (wave - 4) + (lane & 31)
  const int srow = 32 * (wave - 4) + lane;               // valid for producer lanes < 32
  typedef __attribute__((address_space(3))) float lds_float;
  lds_float* rsl = (lds_float*)(smem + 32 * 1024);  // row scales [128], past the SwiGLU hand-off
  if (p.splits > 1) {
    // ---- split-K: publish this split; the last arriver combines (release / ticket /
    // acquire: cdna_hip_programming.md §5 "Projection GEMM" item 2)
    float* base = p.part + (size_t)slab * p.splits * (BN * 128);
    float* mine = base + (size_t)split * (BN * 128);
    if (rn && !consumer && lane < 32) p.ssp[((size_t)slab * p.splits + split) * 128 + srow] = ssq;
    if (consumer && p.ext == 2) {
      // row-major [splits][128][N] partials for dg_reduce_norm_kernel (a workgroup per
      // row): for each accumulator value the 32 lanes of a half write 128 contiguous
      // bytes of one row
      float* rowp = p.part + (size_t)split * 128 * p.N + n0 + 32 * wave + r;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = 32 * mt + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (m < p.M) rowp[(size_t)m * p.N] = acc[mt][i];
        }
    } else if (consumer) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f32x4 v = {acc[mt][4 * q], acc[mt][4 * q + 1], acc[mt][4 * q + 2], acc[mt][4 * q + 3]};
          *reinterpret_cast<f32x4*>(mine + ((size_t)((wave * 4 + mt) * 4 + q) * 64 + lane) * 4) = v;
        }
    }
    if (p.ext) return;  // combined by dg_reduce_kernel
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    typedef __attribute__((address_space(3))) int lds_int;
    lds_int* flag = (lds_int*)smem;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(p.tick + slab, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == (unsigned)(p.splits - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        p.tick[slab] = 0u;  // re-armed for the next launch
      }
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    // sum every split (own included, re-read from its slab) in split order, so the
    // result does not depend on which split arrived last (bitwise reproducible)
    if (consumer) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mt][e] = 0.f;
    }
    for (int s = 0; s < p.splits && consumer; ++s) {
      const float* other = base + (size_t)s * (BN * 128);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(other + ((size_t)((wave * 4 + mt) * 4 + q) * 64 + lane) * 4);
          acc[mt][4 * q] += v[0];
          acc[mt][4 * q + 1] += v[1];
          acc[mt][4 * q + 2] += v[2];
          acc[mt][4 * q + 3] += v[3];
        }
    }
    if (rn) {
      if (tid < 128) {
        float t = 0.f;
        for (int s2 = 0; s2 < p.splits; ++s2) t += p.ssp[((size_t)slab * p.splits + s2) * 128 + tid];
        rsl[tid] = __builtin_amdgcn_rsqf(t / (float)p.K + p.eps);
      }
      __syncthreads();
    }
  } else if (rn) {
    __syncthreads();  // every wave is past its last ring read
    if (!consumer && lane < 32) rsl[srow] = __builtin_amdgcn_rsqf(ssq / (float)p.K + p.eps);
    __syncthreads();
  }
  if (rn && consumer) {
    const int h = lane >> 5;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][i] *= rsl[32 * mt + (i & 3) + 8 * (i >> 2) + 4 * h];
  }

  // ---- epilogue: lane (r, h) of wave w holds column n0 + 32w + r, rows
  // 32 mt + (i & 3) + 8 (i >> 2) + 4 h
  if constexpr (EPI == EPI_SWIGLU) {
    // waves 0,1: gate columns [32w, 32w+32) of the block; waves 2,3: the matching up
    // columns. Up values go through LDS (the ring is idle now).
    lds_float* upv = (lds_float*)smem;  // [2 waves][4 mt][16 i][64 lanes]
    __syncthreads();
    if (consumer && wave >= 2) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) upv[(((wave - 2) * 4 + mt) * 16 + i) * 64 + lane] = acc[mt][i];
    }
    __syncthreads();
    if (wave < 2) {
      const int col = slab * (BN / 2) + 32 * wave + r;  // output column (N/2 wide)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = 32 * mt + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (m < p.M) {
            const float g = acc[mt][i];
            const float u = upv[((wave * 4 + mt) * 16 + i) * 64 + lane];
            const float s = g * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * g));
            p.Y[(size_t)m * p.ldy + col] = (bf16)(s * u);
          }
        }
    }
  } else if (consumer) {
    const int col = n0 + 32 * wave + r;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = 32 * mt + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < p.M) {
          float v = acc[mt][i];
          if constexpr (EPI == EPI_RESID) v += (float)p.R[(size_t)m * p.ldy + col];
          p.Y[(size_t)m * p.ldy + col] = (bf16)v;
        }
      }
  }
}

// Split-K combine as a launch of its own (decode_gemm_config(1), the default): the GEMM's splits
// only publish their partial tiles, so no workgroup serially re-reads every split's
// 64 KiB tile after the stream (the last-arriver combine costs the whole launch one
// CU's read of splits x 64 KiB; Llama-3-8B batch 128, cold weights: down 41.9 -> 33.9 us,
// o 22.1 -> 15.8, qkv 25.4 -> 20.3 incl. the reduce launch, profiles/decode_gemm_ext_reduce_r3.jsonl).
// Thread t of a slab owns one f32x4 of the
// fragment-ordered tile (4 consecutive rows of one column) and sums the splits in
// split order: the same bits as the in-kernel combine.
// RMSNorm row scale from the splits' partial sums of squares (decode_gemm_kernel ssp)
__device__ __forceinline__ float row_scale(const float* __restrict__ ssp, int slab, int splits, int m, int K,
                                           float eps) {
  float t = 0.f;
  for (int s = 0; s < splits; ++s) t += ssp[((size_t)slab * splits + s) * 128 + m];
  return __builtin_amdgcn_rsqf(t / (float)K + eps);
}

template <bool RES>
__global__ __launch_bounds__(256) void dg_reduce_kernel(const float* __restrict__ part, const bf16* __restrict__ R,
                                                        bf16* __restrict__ Y, int M, int ldy, int splits,
                                                        const float* __restrict__ ssp, int K, float eps) {
  const int slab = blockIdx.x;
  const int idx = blockIdx.y * 256 + threadIdx.x;  // [0, 4096)
  const float* base = part + (size_t)slab * splits * (BN * 128) + (size_t)idx * 4;
  __shared__ float rs[128];
  if (ssp && threadIdx.x < 128) rs[threadIdx.x] = row_scale(ssp, slab, splits, threadIdx.x, K, eps);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int k = 0; k < splits; ++k) s += *reinterpret_cast<const f32x4*>(base + (size_t)k * (BN * 128));
  if (ssp) __syncthreads();
  const int lane = idx & 63, t = idx >> 6;
  const int q = t & 3, mt = (t >> 2) & 3, wave = t >> 4;
  const int col = slab * BN + 32 * wave + (lane & 31);
  const int m0 = 32 * mt + 8 * q + 4 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + j;
    if (m < M) {
      float v = s[j];
      if (ssp) v *= rs[m];
      if constexpr (RES) v += (float)R[(size_t)m * ldy + col];
      Y[(size_t)m * ldy + col] = (bf16)v;
    }
  }
}

// Split-K combine + residual add + RMSNorm of the decode o / down projections (ext 2),
// one launch instead of dg_reduce_kernel + rmsnorm_row_kernel (2 x ~5 us per
// projection, profiles/llm_serving_prof_r4_final.md): one workgroup per row sums the
// row's splits x N fp32 partials in split order, rounds to bf16 (the value the unfused
// GEMM stored), adds the residual stream in place (res = bf16(x + res)) and writes
// h = rmsnorm(res) * w -- the numerics of the two launches it replaces.
template <int NV>
__global__ __launch_bounds__(256) void dg_reduce_norm_kernel(const float* __restrict__ part, int splits, int N,
                                                             bf16* __restrict__ res, const bf16* __restrict__ w,
                                                             bf16* __restrict__ hout, float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x, t = threadIdx.x;
  const int nchunk = N >> 3;
  const size_t rbase = (size_t)row * N;
  const size_t sstride = (size_t)128 * N;
  float v[NV][8];
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = t + c * 256;
    if (ch < nchunk) {
      const float* pp = part + rbase + ch * 8;
      f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int k = 0; k < splits; ++k) {
        a += *reinterpret_cast<const f32x4*>(pp + k * sstride);
        b += *reinterpret_cast<const f32x4*>(pp + k * sstride + 4);
      }
      const bf16x8 rr = *reinterpret_cast<const bf16x8*>(res + rbase + ch * 8);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = (float)(bf16)(j < 4 ? a[j] : b[j - 4]);
        o[j] = (bf16)(x + (float)rr[j]);
        v[c][j] = (float)o[j];
        sq += v[c][j] * v[c][j];
      }
      *reinterpret_cast<bf16x8*>(res + rbase + ch * 8) = o;
    }
  }
  sq = wave_sum(sq);
  if ((t & 63) == 0) red[t >> 6] = sq;
  __syncthreads();
  const float rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)N + eps);
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int ch = t + c * 256;
    if (ch < nchunk) {
      const bf16x8 ww = *reinterpret_cast<const bf16x8*>(w + ch * 8);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)(v[c][j] * rs * (float)ww[j]);
      *reinterpret_cast<bf16x8*>(hout + rbase + ch * 8) = o;
    }
  }
}

// The qkv projection's reduce launch with RoPE + paged-cache append fused
// (llm.hip rope_cache_kernel's math on the fp32 sums): head_dim 128 = one 128-column
// slab = one head, so rotary pair (d, d + 64) is f32x4 idx and idx + 2048 of the
// slab's fragment-ordered tile (waves w and w + 2). cs: [max_pos, 64, 2] fp32
// (cos, sin); pos / slot: [M]; cache pages [blocks, KVH, BS, 128].
__global__ __launch_bounds__(256) void dg_reduce_rope_kernel(const float* __restrict__ part, bf16* __restrict__ Y,
                                                             int M, int ldy, int splits, const float* __restrict__ cs,
                                                             const int* __restrict__ pos, const int* __restrict__ slot,
                                                             bf16* __restrict__ kc, bf16* __restrict__ vc, int H,
                                                             int KVH, int BS, const float* __restrict__ ssp, int K,
                                                             float eps) {
  const int head = blockIdx.x;
  const int idx = blockIdx.y * 256 + threadIdx.x;  // [0, 2048): waves 0, 1
  const float* base = part + (size_t)head * splits * (BN * 128) + (size_t)idx * 4;
  __shared__ float rs[128];
  if (ssp && threadIdx.x < 128) rs[threadIdx.x] = row_scale(ssp, head, splits, threadIdx.x, K, eps);
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k = 0; k < splits; ++k) {
    a += *reinterpret_cast<const f32x4*>(base + (size_t)k * (BN * 128));
    b += *reinterpret_cast<const f32x4*>(base + (size_t)k * (BN * 128) + 2048 * 4);
  }
  if (ssp) __syncthreads();
  const int lane = idx & 63, t = idx >> 6;
  const int q = t & 3, mt = (t >> 2) & 3, wave = t >> 4;
  const int d = 32 * wave + (lane & 31);  // rotary pair (d, d + 64)
  const int m0 = 32 * mt + 8 * q + 4 * (lane >> 5);
  const bool rot = head < H + KVH, cache = head >= H && kc != nullptr;
  const int kvh = head < H + KVH ? head - H : head - H - KVH;
  bf16* cbase = head < H + KVH ? kc : vc;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + j;
    if (m >= M) continue;
    float lo = a[j], hi = b[j];
    if (ssp) {
      lo *= rs[m];
      hi *= rs[m];
    }
    if (rot) {
      const float2 c = *reinterpret_cast<const float2*>(cs + ((size_t)pos[m] * 64 + d) * 2);
      const float l0 = lo;
      lo = l0 * c.x - hi * c.y;
      hi = hi * c.x + l0 * c.y;
    }
    const bf16 blo = (bf16)lo, bhi = (bf16)hi;
    bf16* row = Y + (size_t)m * ldy + head * BN;
    row[d] = blo;
    row[d + 64] = bhi;
    if (cache) {
      const int sl = slot[m];
      if (sl >= 0) {
        bf16* dst = cbase + (((size_t)(sl / BS) * KVH + kvh) * BS + sl % BS) * BN;
        dst[d] = blo;
        dst[d + 64] = bhi;
      }
    }
  }
}

static void ensure_lds(const void* k, int bytes) {
  static std::mutex mu;
  static std::unordered_set<const void*> done;
  std::lock_guard<std::mutex> g(mu);
  if (done.insert(k).second) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

}  // namespace dg

// Host entry (shapes validated by the binding): M <= 128, N % 128 == 0,
// K % 64 == 0 and every split non-empty (dg_kchunk); part >= (N/128) * splits * 128*128 floats when splits > 1;
// tick >= N/128 zeroed uints (left zeroed by every launch).
template <int EPI, bool PK, int NWS, int NXS>
static void launch_cfg(const dg::Args& a, dim3 grid, hipStream_t st) {
  const int lds = (NWS + NXS) * dg::IMG;
  dg::ensure_lds((const void*)dg::decode_gemm_kernel<EPI, PK, NWS, NXS>, lds);
  hipLaunchKernelGGL((dg::decode_gemm_kernel<EPI, PK, NWS, NXS>), grid, dim3(dg::WG), lds, st, a);
}

// ring depths (W images, X images): (4, 4) by default -- three K-steps of each stream
// in flight -- or CAAMD_DG_RING = 0 -> (6, 3), 1 -> (8, 2). Serving bench, alternating
// on two boxes: steady TPOT 6.28-6.32 vs 6.42-6.44 ms and 6.38-6.43 vs 6.41-6.43 ms for
// (4, 4) vs (6, 3); (5, 5) and (6, 4) 6.46-6.51, (4, 6) level (profiles/decode_ring_ab_r6.txt)
template <int EPI, bool PK>
static void launch_one(const dg::Args& a, dim3 grid, hipStream_t st) {
  static const int ring = [] {
    const char* e = getenv("CAAMD_DG_RING");
    return e ? atoi(e) : 2;
  }();
  if (ring == 1) launch_cfg<EPI, PK, 8, 2>(a, grid, st);
  else if (ring == 0) launch_cfg<EPI, PK, 6, 3>(a, grid, st);
  else launch_cfg<EPI, PK, 4, 4>(a, grid, st);
}

static int g_dg_ext = [] {
  const char* e = getenv("CAAMD_DG_EXT");
  return e ? atoi(e) : 1;
}();

// K range per split, in whole 64-k steps: ceil(steps / splits); the last split takes
// the rest, so any split count with (splits - 1) * chunk < K works (e.g. 5 splits of
// K = 4096 fill 240 of 256 CUs with the 48 qkv slabs, where 4 equal ones fill 192).
// Returns 0 when some split would be empty.
static int dg_kchunk(int K, int splits) {
  if (K % dg::KS || splits < 1) return 0;
  const int steps = K / dg::KS, per = (steps + splits - 1) / splits;
  return (splits - 1) * per < steps ? per * dg::KS : 0;
}

// 0: last-arriver combine inside the GEMM; 1: separate dg_reduce_kernel launch
void decode_gemm_config(int ext) { g_dg_ext = ext; }

hipError_t decode_gemm_launch(int epi, const bf16* X, const bf16* W, bf16* Y, const bf16* R, float* part,
                              unsigned* tick, int M, int N, int K, int ldx, int ldy, int splits, bool packed,
                              float* ssp, float eps, hipStream_t st) {
  const int kchunk = dg_kchunk(K, splits);
  if (M < 1 || M > 128 || N % dg::BN || !kchunk) return hipErrorInvalidValue;
  const int ext = (splits > 1 && epi != dg::EPI_SWIGLU && g_dg_ext) ? 1 : 0;
  dg::Args a{X, W, Y, R, part, tick, M, N, K, ldx, ldy, splits, kchunk, ext, ssp, eps};
  dim3 grid(N / dg::BN, splits);
  switch (epi * 2 + (packed ? 1 : 0)) {
    case 0: launch_one<dg::EPI_STORE, false>(a, grid, st); break;
    case 1: launch_one<dg::EPI_STORE, true>(a, grid, st); break;
    case 2: launch_one<dg::EPI_RESID, false>(a, grid, st); break;
    case 3: launch_one<dg::EPI_RESID, true>(a, grid, st); break;
    case 4: launch_one<dg::EPI_SWIGLU, false>(a, grid, st); break;
    case 5: launch_one<dg::EPI_SWIGLU, true>(a, grid, st); break;
    default: return hipErrorInvalidValue;
  }
  if (ext) {
    if (epi == dg::EPI_RESID)
      hipLaunchKernelGGL(dg::dg_reduce_kernel<true>, dim3(N / dg::BN, 16), dim3(256), 0, st, part, R, Y, M, ldy,
                         splits, (const float*)ssp, K, eps);
    else
      hipLaunchKernelGGL(dg::dg_reduce_kernel<false>, dim3(N / dg::BN, 16), dim3(256), 0, st, part, R, Y, M, ldy,
                         splits, (const float*)ssp, K, eps);
  }
  return hipGetLastError();
}

// qkv projection + RoPE + cache append (head_dim 128, splits > 1, W prepacked):
// the GEMM's splits publish partials, dg_reduce_rope_kernel combines and rotates.
hipError_t decode_gemm_qkv_rope_launch(const bf16* X, const bf16* W, bf16* Y, float* part, int M, int N, int K,
                                       int ldx, int ldy, int splits, const float* cs, const int* pos,
                                       const int* slot, bf16* kc, bf16* vc, int H, int KVH, int BS,
                                       float* ssp, float eps, hipStream_t st) {
  const int kchunk = dg_kchunk(K, splits);
  if (M < 1 || M > 128 || N % dg::BN || splits < 2 || !kchunk || N != (H + 2 * KVH) * dg::BN)
    return hipErrorInvalidValue;
  dg::Args a{X, W, Y, nullptr, part, nullptr, M, N, K, ldx, ldy, splits, kchunk, 1, ssp, eps};
  launch_one<dg::EPI_STORE, true>(a, dim3(N / dg::BN, splits), st);
  hipLaunchKernelGGL(dg::dg_reduce_rope_kernel, dim3(N / dg::BN, 8), dim3(256), 0, st, part, Y, M, ldy, splits, cs,
                     pos, slot, kc, vc, H, KVH, BS, (const float*)ssp, K, eps);
  return hipGetLastError();
}


// o / down projection + split-K combine + residual add + RMSNorm (w prepacked,
// splits > 1, N % 8 == 0, N <= 8192): res [M, N] updated in place, h = rmsnorm(res) * nw.
hipError_t decode_gemm_norm_launch(const bf16* X, const bf16* W, float* part, int M, int N, int K, int ldx,
                                   int splits, bf16* res, const bf16* nw, bf16* h, float eps, hipStream_t st) {
  const int kchunk = dg_kchunk(K, splits);
  if (M < 1 || M > 128 || N % dg::BN || N > 8192 || splits < 2 || !kchunk) return hipErrorInvalidValue;
  dg::Args a{X, W, nullptr, nullptr, part, nullptr, M, N, K, ldx, N, splits, kchunk, 2, nullptr, eps};
  launch_one<dg::EPI_STORE, true>(a, dim3(N / dg::BN, splits), st);
  const int nv = (N / 8 + 255) / 256;
  if (nv <= 1)
    hipLaunchKernelGGL(dg::dg_reduce_norm_kernel<1>, dim3(M), dim3(256), 0, st, part, splits, N, res, nw, h, eps);
  else if (nv <= 2)
    hipLaunchKernelGGL(dg::dg_reduce_norm_kernel<2>, dim3(M), dim3(256), 0, st, part, splits, N, res, nw, h, eps);
  else
    hipLaunchKernelGGL(dg::dg_reduce_norm_kernel<4>, dim3(M), dim3(256), 0, st, part, splits, N, res, nw, h, eps);
  return hipGetLastError();
}

}  // namespace caamd
