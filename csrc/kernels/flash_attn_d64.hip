// Causal flash attention for head_dim 64 on gfx950 (v_mfma_f32_32x32x16_bf16),
// second generation: the D = 64 path of GPT-2-XL training (25 heads x 64).
//
// Why a separate D = 64 design: at D = 64 every score costs only 4*D = 256 MFMA
// flops but ~5 VALU instructions (max, fma, exp, sum, cvt), so the kernels are
// VALU-issue-bound, not MFMA-bound. A rocprofv3 PMC pass of the first-generation
// kernels (flash_attention.hip) measured 13-15 VALU instructions per MFMA
// (profiles/attn_pmc_v1.md): operand tiles were staged through registers and
// the transposed operands (V^T, K^T, Q^T, dO^T) were written into LDS with
// 16-32 ds_write_b16 + v_perm per thread per tile, and the online softmax
// rescaled O on every tile. This generation removes that overhead:
//
//  * Every K/V/Q/dO tile (64 rows x 128 B) reaches LDS by LDS-DMA
//    (global_load_lds_dwordx4, 16 B per lane, no VGPR staging) into ONE
//    row-major image, XOR-swizzled on the DMA source address:
//       16-B chunk c of row r sits at chunk position c ^ f((r >> 1) & 7),
//       f(x) = x ^ ((x & 1) << 2)
//    f is a bijection of x, so the ds_read_b128 row reads of the 32x32x16
//    operand (lane: row R0 + (l & 31), chunk 2s + (l >> 5)) hit 16 distinct
//    16-B slots in each of the four b128 lane groups, and bit 2 of f flips
//    between rows 4k+{0,1} and 4k+{2,3}, so the ds_read_b64_tr_b16 transposed
//    reads (per 32-lane half: 4 rows x 64 B) cover all 64 banks exactly once.
//    The same image serves row reads AND transposed reads (dq: K; dkdv: Q, dO).
//  * Transposed operands come from ds_read_b64_tr_b16 (hardware transpose),
//    no transposed copies.
//  * Lazy softmax rescale (forward): the running max used for exp2 is only
//    raised when some query's max grew by more than 8 (log2 units), so O and l
//    are rescaled on a few early tiles instead of every tile; P <= 2^8 stays
//    exact to bf16 relative precision and l/O stay in fp32.
//  * Per-lane partial row sums (both lanes of a query keep their own half and
//    combine once at the end).
//  * The backward keeps two kernels (dQ and dK/dV). A fused single kernel
//    needs dQ summed across key blocks: at D = 64 that is one f32 atomic byte
//    per 640 flops, ~0.9 GB of atomics per GPT-2-XL layer at B=32, T=1024,
//    which at the ~1.3 TB/s chip-wide float-atomic rate costs more than the
//    whole two-kernel backward; recomputing S and dP in the dQ kernel is cheaper.
//
// Layout (same as flash_attention.hip): packed qkv [B, T, 3, H, D] in place,
// o [B, T, H, D], dqkv packed like qkv. GQA forward via q/kv row strides.
#include "common.h"

#include <cstdlib>
#include <type_traits>
#include <utility>

namespace caamd {
namespace fa64 {

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// compile-time unrolled loop: f(std::integral_constant<int, i>) for i = 0..N-1
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) char lds_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int D = 64;
constexpr int IMG = 64 * 128;  // one 64-row bf16 tile image (bytes)
constexpr float kThr = 8.f;    // lazy-rescale threshold (log2 units)

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// C/D layout of 32x32: reg i of lane l -> row (i&3) + 8*(i>>2) + 4*(l>>5), col l&31.
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// accumulator registers 8s..8s+7 -> bf16 operand fragment for k-step s
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (bf16)x[8 * s + j];
  return f;
}

__device__ __forceinline__ int swz(int row) {
  const int x = (row >> 1) & 7;
  return x ^ ((x & 1) << 2);
}

// 64-row tile rows [row0, row0 + 64) of g (row stride rs elements, 64 bf16 per
// row) -> swizzled LDS image; 256 threads, two 1-KiB DMA pieces per wave. Rows
// past T are clamped to T - 1 (finite data; masked by the caller).
template <int NT = 256>
__device__ __forceinline__ void dma_tile(const bf16* __restrict__ g, size_t rs, int row0, int T,
                                         lds_t* dst, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 512 / NT; ++j) {
    const int lin = j * NT + wave * 64 + lane;
    const int row = lin >> 3, pos = lin & 7;
    const int c = pos ^ swz(row);
    const int gr = min(row0 + row, T - 1);
    const bf16* src = g + (size_t)gr * rs + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (void __attribute__((address_space(3)))*)(dst + (j * NT + wave * 64) * 16),
                                     16, 0, 0);
  }
}
// 64 floats st[row0 .. row0 + 64) -> LDS (one wave, 4 B per lane)
__device__ __forceinline__ void dma_stats(const float* __restrict__ st, int row0, int T, lds_t* dst,
                                          int lane) {
  const int gr = min(row0 + lane, T - 1);
  __builtin_amdgcn_global_load_lds((const void*)(st + gr), (void __attribute__((address_space(3)))*)dst, 4, 0,
                                   0);
}

// Row fragment of the 32x32x16 operand: lane (r, h) gets X[row][16 s + 8 h .. +7].
__device__ __forceinline__ bf16x8 rd_row(const lds_t* img, int row, int s, int h) {
  const int c = 2 * s + h;
  typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
  return *(lds_bf16x8*)(img + row * 128 + ((c ^ swz(row)) << 4));
}

// Transposed fragment: lane (r, h) gets X[rb + 8 (j >> 2) + 4 h + (j & 3)][c0 + r],
// j = 0..7 -- the k order of acc_frag(., s) when rb = 32 kb + 16 s. Two
// ds_read_b64_tr_b16 (rows rb + 4h + q and rb + 8 + 4h + q of a 16-lane group).
//
// Issued by inline asm: hipcc treats the tr16 builtin as possibly aliasing the
// in-flight LDS-DMA of the NEXT tiles and puts an s_waitcnt vmcnt(0) before it,
// which would expose the whole prefetch latency on every tile. The asm reads are
// invisible to the compiler's counters, so every batch ends with tr_wait*, an
// lgkmcnt(0) that also names the destination registers (nothing reads them
// before it). LDS reads complete in order, so the compiler's own counted
// lgkmcnt waits stay correct with these extra reads in flight.
struct TrFrag {
  s16x4 lo, hi;
};
__device__ __forceinline__ void tr_issue(TrFrag& t, const lds_t* img, int rb, int c0, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = rb + 4 * (G >> 1) + q;
  const int col = c0 + 16 * (G & 1) + 4 * p;
  const int c = col >> 3, within = (col & 7) * 2;
  const int row2 = row + 8;
  const unsigned a0 = (unsigned)(size_t)(img + row * 128 + ((c ^ swz(row)) << 4) + within);
  const unsigned a1 = (unsigned)(size_t)(img + row2 * 128 + ((c ^ swz(row2)) << 4) + within);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(t.lo) : "v"(a0) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(t.hi) : "v"(a1) : "memory");
}
__device__ __forceinline__ void tr_wait2(TrFrag& a, TrFrag& b) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a.lo), "+v"(a.hi), "+v"(b.lo), "+v"(b.hi)::"memory");
}
__device__ __forceinline__ void tr_wait4(TrFrag& a, TrFrag& b, TrFrag& c, TrFrag& d) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a.lo), "+v"(a.hi), "+v"(b.lo), "+v"(b.hi), "+v"(c.lo), "+v"(c.hi), "+v"(d.lo), "+v"(d.hi)::"memory");
}
// Lane-constant parts of the transposed-read addresses. For a block starting
// at row rb (a multiple of 16) swz() is unchanged, and row + 8 flips bit 2 of
// swz(), which maps the d = 0 hi read onto the d = 1 lo pattern and vice versa:
// two lane offsets (A: d = 0 lo, B: d = 1 lo) serve every transposed read of an
// image, the rest is the instruction's immediate offset (rb * 128, + 1024).
struct TrBase {
  unsigned a, b;
};
__device__ __forceinline__ TrBase tr_base(int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = 4 * (G >> 1) + q;
  const int c = 2 * (G & 1) + (p >> 1), within = (p & 1) * 8;
  return {(unsigned)(row * 128 + ((c ^ swz(row)) << 4) + within),
          (unsigned)(row * 128 + (((c + 4) ^ swz(row)) << 4) + within)};
}
template <int OFF>
__device__ __forceinline__ s16x4 tr_at(unsigned addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
  return v;
}
// fragment rows [RB, RB + 16), head-dim block DD (columns 32 DD .. 32 DD + 31) of
// the image at LDS byte address `img` (lane bases from tr_base)
template <int RB, int DD>
__device__ __forceinline__ void tr_frag(TrFrag& t, unsigned img, const TrBase& tb) {
  if constexpr (DD == 0) {
    t.lo = tr_at<RB * 128>(img + tb.a);
    t.hi = tr_at<RB * 128 + 1024>(img + tb.b);
  } else {
    t.lo = tr_at<RB * 128>(img + tb.b);
    t.hi = tr_at<RB * 128 + 1024>(img + tb.a);
  }
}

__device__ __forceinline__ bf16x8 tr_join(const TrFrag& t) {
  const s16x8 v = {t.lo[0], t.lo[1], t.lo[2], t.lo[3], t.hi[0], t.hi[1], t.hi[2], t.hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// x (op) x[lane ^ 32] with v_permlane32_swap (VALU, no LDS bpermute)
__device__ __forceinline__ float max_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ void wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// Workgroup barrier that keeps younger LDS-DMA in flight: __syncthreads() compiles
// to `s_waitcnt vmcnt(0) lgkmcnt(0); s_barrier`, which would drain the tile
// prefetched two steps ahead at every step (the ring would be one deep). Callers
// wait for the tile they need with a counted vmcnt first; lgkmcnt(0) finishes this
// wave's LDS reads before another wave's DMA may overwrite the stage.
__device__ __forceinline__ void barrier_keep_dma() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// Three-stage ring, DMA two tiles ahead: at the end of step t, tile t + 1 must
// have landed while tile t + 2's N pieces (issued this step) stay in flight.
template <int N>
__device__ __forceinline__ void wait_next(bool t2_issued) {
  if (t2_issued) wait_vm<N>();
  else wait_dma();
}

__device__ __forceinline__ int xcd_remap(int id, int n) {
  const int xcd = id & 7, q = n >> 3, r = n & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (id >> 3);
}

// ----------------------------------------------------------------------------
// forward: 4 waves x 64 queries (two 32-query sub-blocks) per block, 64-key tiles
// double-buffered in LDS ({K image, V image} per stage, three stages, DMA two tiles ahead).
// ----------------------------------------------------------------------------
// ABL (timing ablations, tools/bench_attn.py with CAAMD_FA64_ABL; production 0):
// bit 0 no DMA inside the loop (stale tiles), bit 1 no per-tile wait + barrier,
// bit 2 no exp (p = s), bit 3 no tile compute at all.
// ----------------------------------------------------------------------------
// A wave's 32 x 64 fp32 MFMA output (acc[d][4g + j] at row lane & 31, column d*32 + 8g
// + 4h + j) written as bf16 rows through the wave's 4 KB of LDS (16-byte units XOR-
// swizzled by row): eight lanes store one whole 128-byte row, so a store instruction
// covers 8 full rows instead of 8 bytes in each of 32 rows (the direct per-lane stores
// cost the dK / dV kernel 50 us of the 694 us backward; tools/gpu/r5_dkdv_store.sh).
// `mul` scales the lane's row; rows >= nrows are not written; row i goes to base + i*rs.
// The caller makes sure no wave still reads the LDS it hands over.
__device__ __forceinline__ void store_rows_lds(const f32x16 (&acc)[2], float mul, lds_t* wb,
                                               bf16* __restrict__ base, size_t rs, int nrows) {
  typedef __attribute__((address_space(3))) bf16x4 lds_b4;
  typedef __attribute__((address_space(3))) const bf16x8 lds_b8;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = (bf16)(acc[d][4 * g + j] * mul);
      *(lds_b4*)(wb + r * 128 + (((4 * d + g) ^ (r & 7)) << 4) + 8 * h) = a;
    }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int c16 = lane & 7;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int row = 8 * it + (lane >> 3);
    const bf16x8 v = *(lds_b8*)(wb + row * 128 + ((c16 ^ (row & 7)) << 4));
    if (row < nrows) *reinterpret_cast<bf16x8*>(base + (size_t)row * rs + 8 * c16) = v;
  }
}

template <int QS, int ABL = 0, int NW = 4, int STG = 1, int PRE = 0>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 4 : (QS == 2 ? 2 : 3)) void fwd_kernel(const bf16* __restrict__ qp, const bf16* __restrict__ kp,
                                                     const bf16* __restrict__ vp, int q_rs, int kv_rs, int group,
                                                     bf16* __restrict__ out, float* __restrict__ lse, int T,
                                                     int H, int nqb, float scale_log2, int causal) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_t* smem = (lds_t*)smem_raw;
  constexpr int STAGE = 2 * IMG;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = id / nqb;
  const int qb = nqb - 1 - (id % nqb);  // heavy (late) query blocks first
  const int b = bh / H, hh = bh % H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const size_t rs = (size_t)q_rs, krs = (size_t)kv_rs;
  const bf16* qbase = qp + (size_t)b * T * rs + (size_t)hh * D;
  const bf16* kbase = kp + (size_t)b * T * krs + (size_t)(hh / group) * D;
  const bf16* vbase = vp + (size_t)b * T * krs + (size_t)(hh / group) * D;
  constexpr int NT = 64 * NW, QBLK = 32 * QS * NW;  // queries per block (NW waves x QS x 32)
  constexpr int DMA_N = 2 * (512 / NT);  // DMA pieces per wave per tile (K + V)
  const int q0w = qb * QBLK + wave * 32 * QS;

  const int qend = min(T, qb * QBLK + QBLK);
  const int nkt = causal ? (qend + 63) / 64 : (T + 63) / 64;
  dma_tile<NT>(kbase, krs, 0, T, smem, wave, lane);
  dma_tile<NT>(vbase, krs, 0, T, smem + IMG, wave, lane);
  if (nkt > 1) {
    dma_tile<NT>(kbase, krs, 64, T, smem + STAGE, wave, lane);
    dma_tile<NT>(vbase, krs, 64, T, smem + STAGE + IMG, wave, lane);
  }

  // lane-constant LDS offsets: K row reads (k-step s) and V transposed reads
  int koff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) koff[s] = r * 128 + (((2 * s + h) ^ swz(r)) << 4);
  const TrBase vtb = tr_base(lane);

  bf16x8 qf[QS][4];
  f32x16 o[QS][2];
  float m[QS], l[QS];
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
    const int q = q0w + qs * 32 + r;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (q < T) qf[qs][s] = *reinterpret_cast<const bf16x8*>(qbase + (size_t)q * rs + 16 * s + 8 * h);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qs][s][j] = (bf16)0.f;
      }
    }
    o[qs][0] = o[qs][1] = zero16();
    m[qs] = -INFINITY;
    l[qs] = 0.f;
  }
  // PRE: Q pre-scaled by log2(e)/sqrt(D) and the S accumulators started from
  // -(reference max) (minit, a splat kept in registers and rewritten only when the
  // lazy rescale raises the max): the MFMA chain leaves exp2's argument, p = exp2(S')
  // needs no FMA per score
  f32x16 minit[QS];
  if constexpr (PRE) {
#pragma unroll
    for (int qs = 0; qs < QS; ++qs) {
      minit[qs] = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qs][s][j] = (bf16)((float)qf[qs][s][j] * scale_log2);
    }
  }
  wait_dma();
  __syncthreads();

  // one 64-key tile; need_mask (wave-uniform): causal diagonal / sequence tail.
  // The mask compares kb*32 + crow(i, h) (an immediate + 4h) against one
  // per-lane limit, so the unmasked tiles carry no index arithmetic.
  auto tile = [&](auto need_mask_c, const lds_t* kimg, unsigned vimg, int k0) {
    // compile-time: the unmasked tiles (all but the diagonal / tail ones) carry no
    // compare / select code (as a runtime flag the compiler predicated it onto every tile)
    constexpr bool need_mask = decltype(need_mask_c)::value;
    typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
    f32x16 sacc[QS][2];
    // the four K fragments of each 32-key half in flight at once (one LDS latency)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      bf16x8 kf[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) kf[s] = *(lds_bf16x8*)(kimg + koff[s] + kb * 4096);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int qs = 0; qs < QS; ++qs) sacc[qs][kb] = mfma32(kf[0], qf[qs][0], PRE ? minit[qs] : zero16());
#pragma unroll
      for (int s = 1; s < 4; ++s)
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) sacc[qs][kb] = mfma32(kf[s], qf[qs][s], sacc[qs][kb]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // V^T fragments of the first key half requested now, consumed after the softmax
    TrFrag vt[2][2];
    static_for<2>([&](auto s_c) {
      constexpr int s = decltype(s_c)::value;
      tr_frag<s * 16, 0>(vt[s][0], vimg, vtb);
      tr_frag<s * 16, 1>(vt[s][1], vimg, vtb);
    });
#pragma unroll
    for (int qs = 0; qs < QS; ++qs) {
      if constexpr (need_mask) {
        const int q = q0w + qs * 32 + r;
        const int lim = (causal ? min(q, T - 1) : T - 1) - k0 - 4 * h;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            sacc[qs][kb][i] = (kb * 32 + crow(i, 0) > lim) ? -INFINITY : sacc[qs][kb][i];
      }
      float mxa = sacc[qs][0][0], mxb = sacc[qs][1][0];
#pragma unroll
      for (int i = 1; i < 16; ++i) {
        mxa = fmaxf(mxa, sacc[qs][0][i]);
        mxb = fmaxf(mxb, sacc[qs][1][i]);
      }
      float mx = fmaxf(mxa, mxb);
      float rs4[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (PRE) {
        // sacc = c S - muse (muse = the reference max, 0 before the first tile)
        mx = max_xor32(mx);
        if (__builtin_amdgcn_ballot_w64(mx > kThr || (m[qs] == -INFINITY && mx > -INFINITY)) != 0) {
          asm volatile("");  // a real (rarely taken) branch
          const float muse_old = m[qs] == -INFINITY ? 0.f : m[qs];
          const float mnew = fmaxf(m[qs], mx + muse_old);
          const float alpha = m[qs] == -INFINITY ? 0.f : fexp2(m[qs] - mnew);
          l[qs] *= alpha;
#pragma unroll
          for (int d = 0; d < 2; ++d)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[qs][d][i] *= alpha;
          m[qs] = mnew;
          const float shift = (mnew == -INFINITY ? 0.f : mnew) - muse_old;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) sacc[qs][kb][i] -= shift;
#pragma unroll
          for (int i = 0; i < 16; ++i) minit[qs][i] = mnew == -INFINITY ? 0.f : -mnew;
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float p = fexp2(sacc[qs][kb][i]);
            sacc[qs][kb][i] = p;
            rs4[i & 3] += p;
          }
      } else {
      mx = max_xor32(mx) * scale_log2;  // scale > 0 commutes with max
      // lazy rescale: raise the reference max only when it grew by > kThr somewhere
      if (__builtin_amdgcn_ballot_w64(mx > m[qs] + kThr) != 0) {
        asm volatile("");  // keep this a real (rarely taken) branch: no speculated rescale
        const float mnew = fmaxf(m[qs], mx);
        const float alpha = m[qs] == -INFINITY ? 0.f : fexp2(m[qs] - mnew);
        l[qs] *= alpha;
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[qs][d][i] *= alpha;
        m[qs] = mnew;
      }
      const float muse = m[qs] == -INFINITY ? 0.f : m[qs];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = (ABL & 4) ? __builtin_fmaf(sacc[qs][kb][i], scale_log2, -muse)
                                    : fexp2(__builtin_fmaf(sacc[qs][kb][i], scale_log2, -muse));
          sacc[qs][kb][i] = p;
          rs4[i & 3] += p;
        }
      }
      l[qs] += (rs4[0] + rs4[1]) + (rs4[2] + rs4[3]);  // this lane's key half only
    }
    // O^T += V^T P^T ; each V^T fragment feeds both query sub-blocks
    static_for<2>([&](auto kb_c) {
      constexpr int kb = decltype(kb_c)::value;
      tr_wait4(vt[0][0], vt[0][1], vt[1][0], vt[1][1]);
      TrFrag cur[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int d = 0; d < 2; ++d) cur[s][d] = vt[s][d];
      if constexpr (kb == 0) {  // second key half's V^T under this half's MFMAs
        static_for<2>([&](auto s_c) {
          constexpr int s = decltype(s_c)::value;
          tr_frag<32 + s * 16, 0>(vt[s][0], vimg, vtb);
          tr_frag<32 + s * 16, 1>(vt[s][1], vimg, vtb);
        });
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pf[QS];
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) pf[qs] = acc_frag(sacc[qs][kb], s);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const bf16x8 vf = tr_join(cur[s][d]);
#pragma unroll
          for (int qs = 0; qs < QS; ++qs) o[qs][d] = mfma32(vf, pf[qs], o[qs][d]);
        }
      }
    });
  };

  const unsigned smem_u = (unsigned)(size_t)smem;
  // key tiles [0, mfirst) are below every query of the block (no mask); the causal
  // diagonal and a partial last tile run the masked tile body in their own loop (a
  // runtime mask flag was predicated onto every tile)
  auto iter = [&](int kt, auto mask_c) {
    const int k0 = kt * 64;
    const int st = kt % 3;
    const lds_t* kimg = smem + st * STAGE;
    const unsigned vimg = smem_u + st * STAGE + IMG;
    const bool ahead = kt + 2 < nkt && !(ABL & 1);
    if (ahead) {
      lds_t* nb = smem + ((kt + 2) % 3) * STAGE;
      dma_tile<NT>(kbase, krs, k0 + 128, T, nb, wave, lane);
      dma_tile<NT>(vbase, krs, k0 + 128, T, nb + IMG, wave, lane);
    }
    const bool active = !(causal && k0 > q0w + 32 * QS - 1) && q0w < T && !(ABL & 8);  // wave-uniform
    if (active) tile(mask_c, kimg, vimg, k0);
    if constexpr (!(ABL & 2)) {
      wait_next<DMA_N>(ahead);
      barrier_keep_dma();
    }
  };
  {
    const int qblk0 = qb * QBLK;  // the block's first query
    // first tile with k0 + 63 > (first query of any wave of the block)
    const int mfirst = min(nkt, min(T / 64, causal ? (qblk0 >= 63 ? (qblk0 - 63) / 64 + 1 : 0) : nkt));
    int kt = 0;
    for (; kt < mfirst; ++kt) iter(kt, std::false_type{});
    for (; kt < nkt; ++kt) iter(kt, std::true_type{});
  }
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
    const int q = q0w + qs * 32 + r;
    const float lt = sum_xor32(l[qs]);
    const float inv_l = lt > 0.f ? 1.f / lt : 0.f;
    if constexpr (STG) {
      if (qs == 0) __syncthreads();  // every wave is past its last tile: the stage images are free
      store_rows_lds(o[qs], inv_l, smem + wave * 4096, out + ((size_t)b * T + q0w + qs * 32) * H * D + (size_t)hh * D,
                     (size_t)H * D, T - q0w - qs * 32);
    }
    if (q < T) {
      if constexpr (!STG) {
        bf16* orow = out + ((size_t)b * T + q) * H * D + (size_t)hh * D;
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            bf16x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[qs][d][4 * g + j] * inv_l);
            *reinterpret_cast<bf16x4*>(orow + d * 32 + 8 * g + 4 * h) = v;
          }
      }
      if (h == 0) lse[(size_t)bh * T + q] = (m[qs] + __log2f(lt)) * 0.69314718056f;
    }
  }
}

// ----------------------------------------------------------------------------
// forward, head_dim 128 (Llama prefill: GQA through the q / kv row strides):
// the D = 64 design with each 64-key K / V tile held as TWO swizzled 64-dim images
// (dims 0-63, 64-127; the same DMA, row reads and transposed reads as D = 64).
// 4 waves x 32 queries per block, two stages of {K0, K1, V0, V1} (64 KiB: two
// blocks per CU), the next tile's DMA issued under the current tile's MFMAs.
// Per tile and wave: 16 MFMAs for S (8 k-steps over the head dim) and 16 for
// O^T += V^T P^T (4 32-dim blocks), i.e. twice the MFMA work per softmax element of
// the D = 64 kernel. Replaces flash_attention.hip's first-generation
// fa_fwd_kernel<128> (131.9 us per Llama-3-8B prefill chunk, B16 T512 H32 KVH8).
// ----------------------------------------------------------------------------
template <int PRE = 1>
__global__ __launch_bounds__(256, 2) void fwd128_kernel(const bf16* __restrict__ qp, const bf16* __restrict__ kp,
                                                        const bf16* __restrict__ vp, int q_rs, int kv_rs, int group,
                                                        bf16* __restrict__ out, float* __restrict__ lse, int T, int H,
                                                        int nqb, float scale_log2, int causal) {
  constexpr int DH = 128;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_t* smem = (lds_t*)smem_raw;
  constexpr int STAGE = 4 * IMG;  // K0, K1, V0, V1
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = id / nqb;
  const int qb = nqb - 1 - (id % nqb);  // heavy (late) query blocks first
  const int b = bh / H, hh = bh % H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const size_t rs = (size_t)q_rs, krs = (size_t)kv_rs;
  const bf16* qbase = qp + (size_t)b * T * rs + (size_t)hh * DH;
  const bf16* kbase = kp + (size_t)b * T * krs + (size_t)(hh / group) * DH;
  const bf16* vbase = vp + (size_t)b * T * krs + (size_t)(hh / group) * DH;
  constexpr int QBLK = 128;
  const int q0w = qb * QBLK + wave * 32;
  const int qend = min(T, qb * QBLK + QBLK);
  const int nkt = causal ? (qend + 63) / 64 : (T + 63) / 64;
  auto issue = [&](int kt, lds_t* st) {
    dma_tile(kbase, krs, kt * 64, T, st, wave, lane);
    dma_tile(kbase + 64, krs, kt * 64, T, st + IMG, wave, lane);
    dma_tile(vbase, krs, kt * 64, T, st + 2 * IMG, wave, lane);
    dma_tile(vbase + 64, krs, kt * 64, T, st + 3 * IMG, wave, lane);
  };
  issue(0, smem);

  int koff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) koff[s] = r * 128 + (((2 * s + h) ^ swz(r)) << 4);
  const TrBase vtb = tr_base(lane);

  bf16x8 qf[8];
  f32x16 o[4];
  const int q = q0w + r;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    if (q < T) qf[s] = *reinterpret_cast<const bf16x8*>(qbase + (size_t)q * rs + 16 * s + 8 * h);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[s][j] = (bf16)0.f;
    }
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = zero16();
  float m = -INFINITY, l = 0.f;
  // PRE (as fwd_kernel): Q pre-scaled by log2(e)/sqrt(D), S accumulators start from
  // -(reference max), p = exp2(S') with no FMA per score
  f32x16 minit = zero16();
  if constexpr (PRE) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[s][j] = (bf16)((float)qf[s][j] * scale_log2);
  }
  wait_dma();
  __syncthreads();

  auto tile = [&](auto need_mask_c, const lds_t* kimg, unsigned vimg, int k0) {
    constexpr bool need_mask = decltype(need_mask_c)::value;
    typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
    f32x16 sacc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {  // head dims 64 * half .. + 63 (image `half`)
        bf16x8 kf[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) kf[s] = *(lds_bf16x8*)(kimg + half * IMG + koff[s] + kb * 4096);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
          sacc[kb] = mfma32(kf[s], qf[4 * half + s], (half == 0 && s == 0) ? (PRE ? minit : zero16()) : sacc[kb]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // V^T fragments of the first key half requested now, consumed after the softmax
    TrFrag vt[2][4];
    static_for<2>([&](auto s_c) {
      constexpr int s = decltype(s_c)::value;
      tr_frag<s * 16, 0>(vt[s][0], vimg, vtb);
      tr_frag<s * 16, 1>(vt[s][1], vimg, vtb);
      tr_frag<s * 16, 0>(vt[s][2], vimg + IMG, vtb);
      tr_frag<s * 16, 1>(vt[s][3], vimg + IMG, vtb);
    });
    if constexpr (need_mask) {
      const int lim = (causal ? min(q, T - 1) : T - 1) - k0 - 4 * h;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[kb][i] = (kb * 32 + crow(i, 0) > lim) ? -INFINITY : sacc[kb][i];
    }
    float mxa = sacc[0][0], mxb = sacc[1][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) {
      mxa = fmaxf(mxa, sacc[0][i]);
      mxb = fmaxf(mxb, sacc[1][i]);
    }
    float mx = fmaxf(mxa, mxb);
    float rs4[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (PRE) {
      mx = max_xor32(mx);  // relative to the current reference max (0 before the first)
      if (__builtin_amdgcn_ballot_w64(mx > kThr || (m == -INFINITY && mx > -INFINITY)) != 0) {
        asm volatile("");
        const float muse_old = m == -INFINITY ? 0.f : m;
        const float mnew = fmaxf(m, mx + muse_old);
        const float alpha = m == -INFINITY ? 0.f : fexp2(m - mnew);
        l *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[d][i] *= alpha;
        m = mnew;
        const float shift = (mnew == -INFINITY ? 0.f : mnew) - muse_old;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) sacc[kb][i] -= shift;
#pragma unroll
        for (int i = 0; i < 16; ++i) minit[i] = mnew == -INFINITY ? 0.f : -mnew;
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fexp2(sacc[kb][i]);
          sacc[kb][i] = p;
          rs4[i & 3] += p;
        }
    } else {
    mx = max_xor32(mx) * scale_log2;
    if (__builtin_amdgcn_ballot_w64(mx > m + kThr) != 0) {
      asm volatile("");
      const float mnew = fmaxf(m, mx);
      const float alpha = m == -INFINITY ? 0.f : fexp2(m - mnew);
      l *= alpha;
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[d][i] *= alpha;
      m = mnew;
    }
    const float muse = m == -INFINITY ? 0.f : m;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = fexp2(__builtin_fmaf(sacc[kb][i], scale_log2, -muse));
        sacc[kb][i] = p;
        rs4[i & 3] += p;
      }
    }
    l += (rs4[0] + rs4[1]) + (rs4[2] + rs4[3]);
    static_for<2>([&](auto kb_c) {
      constexpr int kb = decltype(kb_c)::value;
      tr_wait4(vt[0][0], vt[0][1], vt[0][2], vt[0][3]);
      tr_wait4(vt[1][0], vt[1][1], vt[1][2], vt[1][3]);
      TrFrag cur[2][4];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int d = 0; d < 4; ++d) cur[s][d] = vt[s][d];
      if constexpr (kb == 0) {  // second key half's V^T under this half's MFMAs
        static_for<2>([&](auto s_c) {
          constexpr int s = decltype(s_c)::value;
          tr_frag<32 + s * 16, 0>(vt[s][0], vimg, vtb);
          tr_frag<32 + s * 16, 1>(vt[s][1], vimg, vtb);
          tr_frag<32 + s * 16, 0>(vt[s][2], vimg + IMG, vtb);
          tr_frag<32 + s * 16, 1>(vt[s][3], vimg + IMG, vtb);
        });
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_frag(sacc[kb], s);
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = mfma32(tr_join(cur[s][d]), pf, o[d]);
      }
    });
  };

  const unsigned smem_u = (unsigned)(size_t)smem;
  auto iter = [&](int kt, auto mask_c) {
    const int k0 = kt * 64;
    const int st = kt & 1;
    if (kt + 1 < nkt) issue(kt + 1, smem + (st ^ 1) * STAGE);  // stage st^1 was released by the last barrier
    const bool active = !(causal && k0 > q0w + 31) && q0w < T;  // wave-uniform
    if (active) tile(mask_c, smem + st * STAGE, smem_u + st * STAGE + 2 * IMG, k0);
    wait_dma();
    barrier_keep_dma();
  };
  {
    const int qblk0 = qb * QBLK;
    const int mfirst = min(nkt, min(T / 64, causal ? (qblk0 >= 63 ? (qblk0 - 63) / 64 + 1 : 0) : nkt));
    int kt = 0;
    for (; kt < mfirst; ++kt) iter(kt, std::false_type{});
    for (; kt < nkt; ++kt) iter(kt, std::true_type{});
  }
  const float lt = sum_xor32(l);
  const float inv_l = lt > 0.f ? 1.f / lt : 0.f;
  // the last barrier: every wave is past its last tile, the stage images are free
  const f32x16 lo[2] = {o[0], o[1]}, hi[2] = {o[2], o[3]};
  bf16* ob = out + ((size_t)b * T + q0w) * H * DH + (size_t)hh * DH;
  store_rows_lds(lo, inv_l, smem + wave * 4096, ob, (size_t)H * DH, T - q0w);
  store_rows_lds(hi, inv_l, smem + wave * 4096, ob + 64, (size_t)H * DH, T - q0w);
  if (q < T && h == 0) lse[(size_t)bh * T + q] = (m + __log2f(lt)) * 0.69314718056f;
}

// ----------------------------------------------------------------------------
// Column sums of the block's 32-row output fragments (lane row = lane & 31, columns
// d*32 + 8g + 4h + j for value 4g + j of acc[d], h = lane >> 5), added to out[col]:
// the projection-bias gradient (colsum over tokens of dQ / dK / dV) taken from
// registers, so no separate pass re-reads the 3-wide dqkv tensor. Reduced across the
// 32 rows of a wave by shuffles, across the 4 waves in LDS, then ONE 64-lane atomic
// instruction per block (f32 atomics cost a memory op per wave instruction whatever
// the lane count: 64 one-lane atomics per wave made the backward 5 % slower).
// Every thread of the block must call it (barriers inside).
__device__ __forceinline__ void colsum_atomic(const f32x16 (&a)[2], float mul, float* __restrict__ out,
                                              float* __restrict__ red /* LDS [4][64] */) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float v = a[d][i];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
      if ((lane & 31) == 0) red[wave * 64 + d * 32 + 8 * (i >> 2) + 4 * h + (i & 3)] = v;
    }
  __syncthreads();
  if (wave == 0) atomicAdd(out + lane, mul * (red[lane] + red[64 + lane] + red[128 + lane] + red[192 + lane]));
  __syncthreads();
}

// backward dQ (+ Delta = rowsum(dO * O), lse2 = lse * log2 e for the dK/dV
// kernel): 4 waves x 64 queries per block, 64-key tiles {K image, V image}.
// ----------------------------------------------------------------------------
template <int QS, int STG = 1, int NEG = 0>
__global__ __launch_bounds__(256, QS == 2 ? 2 : 3) void bwd_dq_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ o,
                                                        const bf16* __restrict__ dout, const float* __restrict__ lse,
                                                        float* __restrict__ delta, float* __restrict__ lse2o,
                                                        bf16* __restrict__ dqkv, int T, int H, int nqb,
                                                        float scale_log2, float scale, int causal,
                                                        float* __restrict__ dbias) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_t* smem = (lds_t*)smem_raw;
  constexpr int STAGE = 2 * IMG;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = id / nqb;
  const int qb = nqb - 1 - (id % nqb);
  const int b = bh / H, hh = bh % H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const size_t rs = (size_t)3 * H * D, ors = (size_t)H * D;
  const bf16* qbase = qkv + (size_t)b * T * rs + (size_t)hh * D;
  const bf16* kbase = qbase + (size_t)H * D;
  const bf16* vbase = kbase + (size_t)H * D;
  constexpr int QBLK = 128 * QS;
  const int q0w = qb * QBLK + wave * 32 * QS;
  const int qend = min(T, qb * QBLK + QBLK);
  const int nkt = causal ? (qend + 63) / 64 : (T + 63) / 64;
  dma_tile(kbase, rs, 0, T, smem, wave, lane);
  dma_tile(vbase, rs, 0, T, smem + IMG, wave, lane);
  if (nkt > 1) {
    dma_tile(kbase, rs, 64, T, smem + STAGE, wave, lane);
    dma_tile(vbase, rs, 64, T, smem + STAGE + IMG, wave, lane);
  }

  bf16x8 qf[QS][4], df[QS][4];
  float dlt[QS], lse2[QS];
  f32x16 dq[QS][2];
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
    const int q = q0w + qs * 32 + r;
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (q < T) {
        qf[qs][s] = *reinterpret_cast<const bf16x8*>(qbase + (size_t)q * rs + 16 * s + 8 * h);
        const size_t oo = ((size_t)b * T + q) * ors + (size_t)hh * D + 16 * s + 8 * h;
        df[qs][s] = *reinterpret_cast<const bf16x8*>(dout + oo);
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(o + oo);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += (float)df[qs][s][j] * (float)ov[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qs][s][j] = df[qs][s][j] = (bf16)0.f;
      }
    }
    dsum += __shfl_xor(dsum, 32, 64);
    dlt[qs] = dsum;
    lse2[qs] = q < T ? lse[(size_t)bh * T + q] * 1.44269504089f : 0.f;
    if (q < T && h == 0) {
      // NEG: negated for the dK/dV kernel's accumulator initialisation (OPT & 32)
      delta[(size_t)bh * T + q] = NEG ? -dsum : dsum;
      lse2o[(size_t)bh * T + q] = NEG ? -lse2[qs] : lse2[qs];
    }
    dq[qs][0] = dq[qs][1] = zero16();
  }
  int koff[4];  // lane-constant row-read offsets (K and V images share the layout)
#pragma unroll
  for (int s = 0; s < 4; ++s) koff[s] = r * 128 + (((2 * s + h) ^ swz(r)) << 4);
  const TrBase ktb = tr_base(lane);
  wait_dma();
  __syncthreads();

  auto tile = [&](auto need_mask_c, const lds_t* kimg, unsigned kimg_u, int k0) {
    // compile-time: the unmasked tiles (all but the diagonal / tail ones) carry no
    // compare / select code (as a runtime flag the compiler predicated it onto every tile)
    constexpr bool need_mask = decltype(need_mask_c)::value;
    typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
    static_for<2>([&](auto kb_c) {
      constexpr int kb = decltype(kb_c)::value;
      f32x16 sacc[QS], dp[QS];
      // the 32-key half's eight row fragments in flight at once
      bf16x8 kr[4], vr[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        kr[s] = *(lds_bf16x8*)(kimg + koff[s] + kb * 4096);
        vr[s] = *(lds_bf16x8*)(kimg + IMG + koff[s] + kb * 4096);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int qs = 0; qs < QS; ++qs) {
        sacc[qs] = mfma32(kr[0], qf[qs][0], zero16());
        dp[qs] = mfma32(vr[0], df[qs][0], zero16());
      }
#pragma unroll
      for (int s = 1; s < 4; ++s)
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) {
          sacc[qs] = mfma32(kr[s], qf[qs][s], sacc[qs]);
          dp[qs] = mfma32(vr[s], df[qs][s], dp[qs]);
        }
      // K^T fragments for dQ requested now, consumed after the VALU pass
      __builtin_amdgcn_sched_barrier(0);
      TrFrag t[2][2];
      static_for<2>([&](auto s_c) {
        constexpr int s = decltype(s_c)::value;
        tr_frag<kb * 32 + s * 16, 0>(t[s][0], kimg_u, ktb);
        tr_frag<kb * 32 + s * 16, 1>(t[s][1], kimg_u, ktb);
      });
#pragma unroll
      for (int qs = 0; qs < QS; ++qs) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[qs][i] = fexp2(__builtin_fmaf(sacc[qs][i], scale_log2, -lse2[qs]));
        if constexpr (need_mask) {
          const int q = q0w + qs * 32 + r;
          const int lim = (q >= T ? -1 : (causal ? min(q, T - 1) : T - 1)) - k0 - 4 * h;
#pragma unroll
          for (int i = 0; i < 16; ++i) sacc[qs][i] = (kb * 32 + crow(i, 0) > lim) ? 0.f : sacc[qs][i];
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[qs][i] *= dp[qs][i] - dlt[qs];  // dS^T
      }
      // dQ^T += K^T dS^T
      tr_wait4(t[0][0], t[0][1], t[1][0], t[1][1]);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 f[QS];
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) f[qs] = acc_frag(sacc[qs], s);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const bf16x8 a = tr_join(t[s][d]);
#pragma unroll
          for (int qs = 0; qs < QS; ++qs) dq[qs][d] = mfma32(a, f[qs], dq[qs][d]);
        }
      }
    });
  };

  const unsigned smem_u = (unsigned)(size_t)smem;
  // unmasked key tiles first, then the causal diagonal / partial last tile with the
  // masked body (as in the forward)
  auto iter = [&](int kt, auto mask_c) {
    const int k0 = kt * 64;
    const int st = kt % 3;
    const bool ahead = kt + 2 < nkt;
    if (ahead) {
      lds_t* nb = smem + ((kt + 2) % 3) * STAGE;
      dma_tile(kbase, rs, k0 + 128, T, nb, wave, lane);
      dma_tile(vbase, rs, k0 + 128, T, nb + IMG, wave, lane);
    }
    if (!(causal && k0 > q0w + 32 * QS - 1) && q0w < T)  // wave-uniform
      tile(mask_c, smem + st * STAGE, smem_u + st * STAGE, k0);
    wait_next<4>(ahead);
    barrier_keep_dma();
  };
  {
    const int qblk0 = qb * QBLK;
    const int mfirst = min(nkt, min(T / 64, causal ? (qblk0 >= 63 ? (qblk0 - 63) / 64 + 1 : 0) : nkt));
    int kt = 0;
    for (; kt < mfirst; ++kt) iter(kt, std::false_type{});
    for (; kt < nkt; ++kt) iter(kt, std::true_type{});
  }
  if (dbias) {  // q-bias gradient: rows past T hold zeros (never-computed tiles)
    f32x16 sum[2];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      sum[d] = zero16();
#pragma unroll
      for (int qs = 0; qs < QS; ++qs)
        if (q0w + qs * 32 + r < T) sum[d] += dq[qs][d];
    }
    __shared__ float red[256];
    colsum_atomic(sum, scale, dbias + (size_t)hh * D, red);
  }
  if constexpr (STG) {
    __syncthreads();  // every wave is past its last tile: the stage images are free
#pragma unroll
    for (int qs = 0; qs < QS; ++qs)
      store_rows_lds(dq[qs], scale, smem + wave * 4096, dqkv + ((size_t)b * T + q0w + qs * 32) * rs + (size_t)hh * D,
                     rs, T - q0w - qs * 32);
    return;
  }
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
    const int q = q0w + qs * 32 + r;
    if (q < T) {
      bf16* row = dqkv + ((size_t)b * T + q) * rs + (size_t)hh * D;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(dq[qs][d][4 * g + j] * scale);
          *reinterpret_cast<bf16x4*>(row + d * 32 + 8 * g + 4 * h) = v;
        }
    }
  }
}

// ----------------------------------------------------------------------------
// backward dK, dV: key on the lane, 4 waves x 32 keys per block; 64-query tiles
// {Q image, dO image, lse2[64], delta[64]} double-buffered. Q and dO are read
// by rows (S^T, dP^T) and transposed (dK^T, dV^T) from the same image.
// ----------------------------------------------------------------------------
// ABL (timing ablations, tools/bench_attn.py with CAAMD_FA64_BWD_ABL; production 0):
// bit 0 no DMA inside the loop (stale tiles), bit 1 no per-tile wait + barrier,
// bit 2 no softmax / dS VALU (P = S, dS = dP), bit 3 no transposed reads, bit 4 no
// row-fragment reads, bit 5 no dK / dV stores.
// OPT (schedule variants, CAAMD_FA64_DKDV_OPT): bit 0 = the second half's Q / dO
// row fragments loaded during the first half's VALU pass (into the registers the
// first half's S / dP MFMAs just released); bit 1 = the transposed fragments of a
// half requested before its S / dP MFMAs instead of after them; bit 2 = the half's
// lse2 / delta rows read (and retired) before its S / dP MFMAs; bit 3 = dK / dV
// written through an LDS transpose as whole rows; bit 5 = K pre-scaled by
// log2(e)/sqrt(D) and the S / dP accumulators initialised with -lse2 / -delta (the dQ
// kernel stores them negated), so the softmax pass is exp2 + one multiply per score;
// bit 6 = the block's K rows by LDS-DMA through the third stage in the prologue.
template <int ABL = 0, int OPT = 0>
__global__ __launch_bounds__(256, 2) void bwd_dkdv_kernel(const bf16* __restrict__ qkv,
                                                          const bf16* __restrict__ dout,
                                                          const float* __restrict__ lse2g,
                                                          const float* __restrict__ delta,
                                                          bf16* __restrict__ dqkv, int T, int H, int nkb,
                                                          float scale_log2, float scale, int causal,
                                                          float* __restrict__ dbias) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_t* smem = (lds_t*)smem_raw;
  constexpr int STAGE = 2 * IMG + 512;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = id / nkb;
  const int kb0 = id % nkb;  // early key blocks are the heavy ones under the causal mask
  const int b = bh / H, hh = bh % H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const size_t rs = (size_t)3 * H * D, ors = (size_t)H * D;
  const bf16* qbase = qkv + (size_t)b * T * rs + (size_t)hh * D;
  const bf16* kbase = qbase + (size_t)H * D;
  const bf16* vbase = kbase + (size_t)H * D;
  const bf16* dobase = dout + (size_t)b * T * ors + (size_t)hh * D;
  const float* l2b = lse2g + (size_t)bh * T;
  const float* dlb = delta + (size_t)bh * T;
  const int key0w = kb0 * 128 + wave * 32;
  const int key = key0w + r;
  const bool kv = key < T;
  const int qt0 = causal ? (kb0 * 128) / 64 : 0;
  const int nqt = (T + 63) / 64;

  auto issue = [&](int qt, lds_t* buf) {
    dma_tile(qbase, rs, qt * 64, T, buf, wave, lane);
    dma_tile(dobase, ors, qt * 64, T, buf + IMG, wave, lane);
    if (wave == 0) dma_stats(l2b, qt * 64, T, buf + 2 * IMG, lane);
    else if (wave == 1) dma_stats(dlb, qt * 64, T, buf + 2 * IMG + 256, lane);
  };
  if (qt0 < nqt) issue(qt0, smem);
  if (qt0 + 1 < nqt) issue(qt0 + 1, smem + STAGE);

  bf16x8 kf[4], vf[4];
  if constexpr (OPT & 64) {
    // the block's 128 K rows by LDS-DMA into the third stage (whole 128-byte rows, 8
    // lanes a row) instead of per-lane 16-byte loads that touch 32 rows per instruction;
    // read back as row fragments before that stage's first tile is issued
    dma_tile(kbase, rs, kb0 * 128, T, smem + 2 * STAGE, wave, lane);
    dma_tile(kbase, rs, kb0 * 128 + 64, T, smem + 2 * STAGE + IMG, wave, lane);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (kv) {
      if constexpr (!(OPT & 64)) kf[s] = *reinterpret_cast<const bf16x8*>(kbase + (size_t)key * rs + 16 * s + 8 * h);
      vf[s] = *reinterpret_cast<const bf16x8*>(vbase + (size_t)key * rs + 16 * s + 8 * h);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[s][j] = vf[s][j] = (bf16)0.f;
    }
  }
  if constexpr (OPT & 64) {
    wait_dma();
    __syncthreads();
    typedef __attribute__((address_space(3))) const bf16x8 lds_kf;
    const lds_t* kimg = smem + 2 * STAGE + (wave >> 1) * IMG;
    const int row = (wave & 1) * 32 + r;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 v = *(lds_kf*)(kimg + row * 128 + (((2 * s + h) ^ swz(row)) << 4));
      if (kv) kf[s] = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every wave has its K fragments: the stage is free for tile qt0 + 2
  }
  if constexpr (OPT & 32) {
    // K pre-scaled by log2(e) / sqrt(D) once per block: S' = Q (c K)^T - lse2 comes out
    // of the MFMA chain (accumulator initialised with -lse2), so p = exp2(S') needs no
    // FMA per score
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[s][j] = (bf16)((float)kf[s][j] * scale_log2);
  }
  f32x16 dk[2], dv[2];
  dk[0] = dk[1] = dv[0] = dv[1] = zero16();
  int qoff[4];  // lane-constant row-read offsets (Q and dO images share the layout)
#pragma unroll
  for (int s = 0; s < 4; ++s) qoff[s] = r * 128 + (((2 * s + h) ^ swz(r)) << 4);
  const TrBase tb = tr_base(lane);
  wait_dma();
  __syncthreads();

  // mask: query q0 + 4h + c (c = qh*32 + 8g + j, an immediate) is dropped when
  // c < key - q0 - 4h (causal) or c > T - 1 - q0 - 4h (tail). Lanes with key >= T
  // compute on zero K/V and are never stored.
  auto tile = [&](auto need_mask_c, const lds_t* qimg, unsigned qimg_u, int q0) {
    // compile-time: the unmasked tiles (all but the diagonal / tail ones) carry no
    // compare / select code (as a runtime flag the compiler predicated it onto every tile)
    constexpr bool need_mask = decltype(need_mask_c)::value;
    typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
    const float* st = (const float*)(qimg + 2 * IMG);
    const int lo_lim = causal ? key - q0 - 4 * h : -0x7fffffff;
    const int hi_lim = T - 1 - q0 - 4 * h;
    // the half's eight row fragments in flight at once (one LDS latency)
    bf16x8 qr[4], dr[4];
    auto load_rows = [&](auto qh_c) {
      constexpr int qh = decltype(qh_c)::value;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if constexpr (ABL & 16) {  // ablation: no row-fragment reads (stale registers)
          bf16x8* q = qr;  // (a plain use, so the lambda captures the arrays)
          bf16x8* d = dr;
          asm volatile("" : "+v"(q[s]), "+v"(d[s]));
        } else {
          qr[s] = *(lds_bf16x8*)(qimg + qoff[s] + qh * 4096);
          dr[s] = *(lds_bf16x8*)(qimg + IMG + qoff[s] + qh * 4096);
        }
      }
    };
    load_rows(std::integral_constant<int, 0>{});
    // one 32-query half at a time (S^T, dP^T live for 16 MFMAs only)
    static_for<2>([&](auto qh_c) {
      constexpr int qh = decltype(qh_c)::value;
      if constexpr (qh == 1 && !(OPT & 1)) load_rows(std::integral_constant<int, 1>{});
      TrFrag tv[2][2], tk[2][2];
      auto issue_tr = [&]() {
        if constexpr (ABL & 8) {  // ablation: no transposed reads (stale registers)
          TrFrag(*v)[2] = tv;  // (a plain use, so the lambda captures the arrays)
          TrFrag(*k)[2] = tk;
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int d = 0; d < 2; ++d)
              asm volatile("" : "+v"(v[s][d].lo), "+v"(v[s][d].hi), "+v"(k[s][d].lo), "+v"(k[s][d].hi));
          return;
        }
        static_for<2>([&](auto s_c) {
          constexpr int s = decltype(s_c)::value;
          tr_frag<qh * 32 + s * 16, 0>(tv[s][0], qimg_u + IMG, tb);
          tr_frag<qh * 32 + s * 16, 1>(tv[s][1], qimg_u + IMG, tb);
          tr_frag<qh * 32 + s * 16, 0>(tk[s][0], qimg_u, tb);
          tr_frag<qh * 32 + s * 16, 1>(tk[s][1], qimg_u, tb);
        });
      };
      if constexpr (OPT & 2) issue_tr();
      // OPT & 4: the half's lse2 / delta rows read with the row fragments, before the
      // S / dP MFMAs; the asm wait (naming the registers) retires them there, so the
      // VALU pass does not wait on LDS (the compiler's own wait for them would land
      // behind the transposed reads and wait for those too)
      f32x4 l4s[4], d4s[4];
      if constexpr (OPT & (4 | 32)) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int qi = qh * 32 + 8 * g + 4 * h;
          l4s[g] = *reinterpret_cast<const f32x4*>(st + qi);
          d4s[g] = *reinterpret_cast<const f32x4*>(st + 64 + qi);
        }
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(l4s[0]), "+v"(l4s[1]), "+v"(l4s[2]), "+v"(l4s[3]), "+v"(d4s[0]), "+v"(d4s[1]),
                       "+v"(d4s[2]), "+v"(d4s[3])::"memory");
      }
      f32x16 sinit = zero16(), dinit = zero16();
      if constexpr (OPT & 32) {  // row constants as the initial accumulators: -lse2, -delta
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            sinit[4 * g + j] = l4s[g][j];
            dinit[4 * g + j] = d4s[g][j];
          }
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x16 sacc = mfma32(qr[0], kf[0], sinit);
      f32x16 dp = mfma32(dr[0], vf[0], dinit);
#pragma unroll
      for (int s = 1; s < 4; ++s) {
        sacc = mfma32(qr[s], kf[s], sacc);
        dp = mfma32(dr[s], vf[s], dp);
      }
      // transposed dO / Q fragments requested now, consumed after the VALU pass
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(OPT & 2)) issue_tr();
      if constexpr (qh == 0 && (OPT & 1)) load_rows(std::integral_constant<int, 1>{});
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int qi = qh * 32 + 8 * g + 4 * h;
        f32x4 l4, d4;
        if constexpr (OPT & (4 | 32)) {
          l4 = l4s[g];
          d4 = d4s[g];
        } else {
          l4 = *reinterpret_cast<const f32x4*>(st + qi);
          d4 = *reinterpret_cast<const f32x4*>(st + 64 + qi);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * g + j;
          if constexpr (ABL & 4) {
            continue;
          }
          float p = (OPT & 32) ? fexp2(sacc[i]) : fexp2(__builtin_fmaf(sacc[i], scale_log2, -l4[j]));
          if constexpr (need_mask) {
            const int c = qh * 32 + 8 * g + j;
            p = (c < lo_lim || c > hi_lim) ? 0.f : p;
          }
          sacc[i] = p;
          dp[i] = (OPT & 32) ? p * dp[i] : p * (dp[i] - d4[j]);
        }
      }
      tr_wait4(tv[0][0], tv[0][1], tk[0][0], tk[0][1]);
      tr_wait4(tv[1][0], tv[1][1], tk[1][0], tk[1][1]);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_frag(sacc, s), sf = acc_frag(dp, s);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = mfma32(tr_join(tv[s][d]), pf, dv[d]);
          dk[d] = mfma32(tr_join(tk[s][d]), sf, dk[d]);
        }
      }
    });
  };

  const unsigned smem_u = (unsigned)(size_t)smem;
  // One iteration per 64-query tile. Only the first two tiles of a key block (the
  // causal diagonal) and a partial last tile need the mask: they run in their own
  // loops with the masked tile body, the rest with the unmasked one (a runtime flag
  // was predicated onto every tile: 96 compares / selects per tile).
  auto iter = [&](int qt, auto mask_c) {
    const int q0 = qt * 64;
    const int stg = (qt - qt0) % 3;
    const bool ahead = (ABL & 1) ? false : qt + 2 < nqt;
    if (ahead) issue(qt + 2, smem + ((qt + 2 - qt0) % 3) * STAGE);
    if (!(causal && q0 + 63 < key0w) && key0w < T)  // wave-uniform
      tile(mask_c, smem + stg * STAGE, smem_u + stg * STAGE, q0);
    if constexpr (!(ABL & 2)) {
      if (wave < 2) wait_next<5>(ahead);  // waves 0 / 1 also DMA the lse2 / delta rows
      else wait_next<4>(ahead);
      barrier_keep_dma();
    }
  };
  const int nfull = T / 64;  // tiles entirely inside the sequence
  const int pro = min(nqt, qt0 + (causal ? 2 : 0));
  int qt = qt0;
  for (; qt < pro; ++qt) iter(qt, std::true_type{});
  for (; qt < nfull; ++qt) iter(qt, std::false_type{});
  for (; qt < nqt; ++qt) iter(qt, std::true_type{});
  if (dbias) {  // k / v bias gradients (block-uniform; keys past T contribute zeros)
    __shared__ float red[256];
    f32x16 k2[2], v2[2];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      k2[d] = kv ? dk[d] : zero16();
      v2[d] = kv ? dv[d] : zero16();
    }
    colsum_atomic(k2, scale, dbias + (size_t)(H + hh) * D, red);
    colsum_atomic(v2, 1.f, dbias + (size_t)(2 * H + hh) * D, red);
  }
  if constexpr (OPT & 8) {
    __syncthreads();  // every wave is past its last tile: the stage images are free
    bf16* kr = dqkv + ((size_t)b * T + key0w) * rs + (size_t)(H + hh) * D;
    store_rows_lds(dk, scale, smem + wave * 8192, kr, rs, T - key0w);
    store_rows_lds(dv, 1.f, smem + wave * 8192 + 4096, kr + (size_t)H * D, rs, T - key0w);
    return;
  }
  // ABL & 32: no dK / dV stores (kept behind a never-true test so the math stays live)
  if (kv && (!(ABL & 32) || dk[0][0] == 12345.f)) {
    bf16* krow = dqkv + ((size_t)b * T + key) * rs + (size_t)(H + hh) * D;
    bf16* vrow = krow + (size_t)H * D;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 a, c;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = (bf16)(dk[d][4 * g + j] * scale);
          c[j] = (bf16)dv[d][4 * g + j];
        }
        *reinterpret_cast<bf16x4*>(krow + d * 32 + 8 * g + 4 * h) = a;
        *reinterpret_cast<bf16x4*>(vrow + d * 32 + 8 * g + 4 * h) = c;
      }
  }
}

// ----------------------------------------------------------------------------
// dK, dV with PAIRED key blocks (fewer, longer blocks): one workgroup walks key block
// j and key block nkb - 1 - j of one (batch, head) as ONE continuous stream of
// 64-query tiles. Under the causal mask key block j needs nqt - 2j tiles, so every
// pair carries nqt + 2 tiles (uniform work, half the blocks of the one-item kernel);
// the LDS-DMA ring keeps prefetching across the seam between the two items, item B's
// K / V rows sit in registers from the prologue on, and item A's dK / dV leave
// through a 16 KB staging region of their own while item B's first tiles are
// already in flight. Per tile the body is bwd_dkdv_kernel's production schedule
// (OPT 104: K pre-scaled, S / dP accumulators started from -lse2 / -delta, K of the
// first item by LDS-DMA, dK / dV stored as whole rows through LDS).
// Measured lever: tools/lab/mfma_dep_bench.hip -- the dK/dV MFMA chain runs ~95 %
// busy inside one long block; the one-item kernel's 6,400 short blocks pay a
// prologue load and an epilogue store each (PERF.md round 5).
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void bwd_dkdv_pair_kernel(const bf16* __restrict__ qkv,
                                                               const bf16* __restrict__ dout,
                                                               const float* __restrict__ lse2g,
                                                               const float* __restrict__ delta,
                                                               bf16* __restrict__ dqkv, int T, int H, int nkb,
                                                               int npair, float scale_log2, float scale, int causal,
                                                               float* __restrict__ dbias) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_t* smem = (lds_t*)smem_raw;
  constexpr int STAGE = 2 * IMG + 512;
  lds_t* stg_out = smem + 3 * STAGE;  // 16 KB: 4 KB per wave, dK then dV of a finished item
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = id / npair;
  const int pj = id % npair;
  const int kbs[2] = {pj, nkb - 1 - pj};
  const int nitem = kbs[1] == kbs[0] ? 1 : 2;
  const int b = bh / H, hh = bh % H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const size_t rs = (size_t)3 * H * D, ors = (size_t)H * D;
  const bf16* qbase = qkv + (size_t)b * T * rs + (size_t)hh * D;
  const bf16* kbase = qbase + (size_t)H * D;
  const bf16* vbase = kbase + (size_t)H * D;
  const bf16* dobase = dout + (size_t)b * T * ors + (size_t)hh * D;
  const float* l2b = lse2g + (size_t)bh * T;
  const float* dlb = delta + (size_t)bh * T;
  const int nqt = (T + 63) / 64;
  const int nfull = T / 64;
  // tile stream: item 0's tiles [qt0(0), nqt), then item 1's [qt0(1), nqt)
  auto qt0_of = [&](int it) { return causal ? (kbs[it] * 128) / 64 : 0; };
  const int qt0A = qt0_of(0);
  const int cntA = max(0, nqt - qt0A);
  const int cnt = cntA + (nitem == 2 ? max(0, nqt - qt0_of(1)) : 0);
  auto qt_of = [&](int g) { return g < cntA ? qt0A + g : qt0_of(1) + (g - cntA); };

  auto issue = [&](int g, lds_t* buf) {
    const int qt = qt_of(g);
    dma_tile(qbase, rs, qt * 64, T, buf, wave, lane);
    dma_tile(dobase, ors, qt * 64, T, buf + IMG, wave, lane);
    if (wave == 0) dma_stats(l2b, qt * 64, T, buf + 2 * IMG, lane);
    else if (wave == 1) dma_stats(dlb, qt * 64, T, buf + 2 * IMG + 256, lane);
  };
  if (cnt > 0) issue(0, smem);
  if (cnt > 1) issue(1, smem + STAGE);

  // K / V rows: item 0's K by LDS-DMA through the third stage and its V by per-lane
  // 16-byte loads; item 1's K / V by per-lane loads issued at the seam (they land
  // while item 0's dK / dV are written out)
  bf16x8 kf[4], vf[4];
  int key0w = kbs[0] * 128 + wave * 32;
  int key = key0w + r;
  bool kv = key < T;
  dma_tile(kbase, rs, kbs[0] * 128, T, smem + 2 * STAGE, wave, lane);
  dma_tile(kbase, rs, kbs[0] * 128 + 64, T, smem + 2 * STAGE + IMG, wave, lane);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (kv) {
      vf[s] = *reinterpret_cast<const bf16x8*>(vbase + (size_t)key * rs + 16 * s + 8 * h);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[s][j] = vf[s][j] = (bf16)0.f;
    }
  }
  wait_dma();
  __syncthreads();
  {
    typedef __attribute__((address_space(3))) const bf16x8 lds_kf;
    const lds_t* kimg = smem + 2 * STAGE + (wave >> 1) * IMG;
    const int row = (wave & 1) * 32 + r;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 v = *(lds_kf*)(kimg + row * 128 + (((2 * s + h) ^ swz(row)) << 4));
      if (kv) kf[s] = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __syncthreads();  // every wave has its K fragments: the stage is free for tile 2
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) kf[s][j] = (bf16)((float)kf[s][j] * scale_log2);
  f32x16 dk[2], dv[2];
  dk[0] = dk[1] = dv[0] = dv[1] = zero16();
  int qoff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qoff[s] = r * 128 + (((2 * s + h) ^ swz(r)) << 4);
  const TrBase tb = tr_base(lane);

  auto tile = [&](auto need_mask_c, const lds_t* qimg, unsigned qimg_u, int q0) {
    constexpr bool need_mask = decltype(need_mask_c)::value;
    typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
    const float* st = (const float*)(qimg + 2 * IMG);
    const int lo_lim = causal ? key - q0 - 4 * h : -0x7fffffff;
    const int hi_lim = T - 1 - q0 - 4 * h;
    bf16x8 qr[4], dr[4];
    auto load_rows = [&](int qh) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        qr[s] = *(lds_bf16x8*)(qimg + qoff[s] + qh * 4096);
        dr[s] = *(lds_bf16x8*)(qimg + IMG + qoff[s] + qh * 4096);
      }
    };
    load_rows(0);
    static_for<2>([&](auto qh_c) {
      constexpr int qh = decltype(qh_c)::value;
      if constexpr (qh == 1) load_rows(1);
      TrFrag tv[2][2], tk[2][2];
      f32x4 l4s[4], d4s[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int qi = qh * 32 + 8 * g + 4 * h;
        l4s[g] = *reinterpret_cast<const f32x4*>(st + qi);
        d4s[g] = *reinterpret_cast<const f32x4*>(st + 64 + qi);
      }
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(l4s[0]), "+v"(l4s[1]), "+v"(l4s[2]), "+v"(l4s[3]), "+v"(d4s[0]), "+v"(d4s[1]),
                     "+v"(d4s[2]), "+v"(d4s[3])::"memory");
      f32x16 sinit, dinit;
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sinit[4 * g + j] = l4s[g][j];
          dinit[4 * g + j] = d4s[g][j];
        }
      __builtin_amdgcn_sched_barrier(0);
      f32x16 sacc = mfma32(qr[0], kf[0], sinit);
      f32x16 dp = mfma32(dr[0], vf[0], dinit);
#pragma unroll
      for (int s = 1; s < 4; ++s) {
        sacc = mfma32(qr[s], kf[s], sacc);
        dp = mfma32(dr[s], vf[s], dp);
      }
      __builtin_amdgcn_sched_barrier(0);
      static_for<2>([&](auto s_c) {
        constexpr int s = decltype(s_c)::value;
        tr_frag<qh * 32 + s * 16, 0>(tv[s][0], qimg_u + IMG, tb);
        tr_frag<qh * 32 + s * 16, 1>(tv[s][1], qimg_u + IMG, tb);
        tr_frag<qh * 32 + s * 16, 0>(tk[s][0], qimg_u, tb);
        tr_frag<qh * 32 + s * 16, 1>(tk[s][1], qimg_u, tb);
      });
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * g + j;
          float p = fexp2(sacc[i]);
          if constexpr (need_mask) {
            const int c = qh * 32 + 8 * g + j;
            p = (c < lo_lim || c > hi_lim) ? 0.f : p;
          }
          sacc[i] = p;
          dp[i] = p * dp[i];
        }
      }
      tr_wait4(tv[0][0], tv[0][1], tk[0][0], tk[0][1]);
      tr_wait4(tv[1][0], tv[1][1], tk[1][0], tk[1][1]);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_frag(sacc, s), sf = acc_frag(dp, s);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = mfma32(tr_join(tv[s][d]), pf, dv[d]);
          dk[d] = mfma32(tr_join(tk[s][d]), sf, dk[d]);
        }
      }
    });
  };

  // dK / dV of the finished item (keys key0w .. key0w + 31 of this wave): through the
  // wave's 4 KB of the staging region, dK then dV (the region is this wave's only)
  auto finish_item = [&]() {
    if (dbias) {
      __shared__ float red[256];
      f32x16 k2[2], v2[2];
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        k2[d] = kv ? dk[d] : zero16();
        v2[d] = kv ? dv[d] : zero16();
      }
      colsum_atomic(k2, scale, dbias + (size_t)(H + hh) * D, red);
      colsum_atomic(v2, 1.f, dbias + (size_t)(2 * H + hh) * D, red);
    }
    bf16* kr = dqkv + ((size_t)b * T + key0w) * rs + (size_t)(H + hh) * D;
    lds_t* wb = stg_out + wave * 4096;
    store_rows_lds(dk, scale, wb, kr, rs, T - key0w);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's row reads of dK done
    __builtin_amdgcn_wave_barrier();
    store_rows_lds(dv, 1.f, wb, kr + (size_t)H * D, rs, T - key0w);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  };

  const unsigned smem_u = (unsigned)(size_t)smem;
  // one tile of the stream: prefetch stream tile g + 2, compute tile g (= query tile qt)
  auto iter = [&](int g, int qt, auto mask_c) {
    const int q0 = qt * 64;
    const bool ahead = g + 2 < cnt;
    if (ahead) issue(g + 2, smem + ((g + 2) % 3) * STAGE);
    if (!(causal && q0 + 63 < key0w) && key0w < T)  // wave-uniform
      tile(mask_c, smem + (g % 3) * STAGE, smem_u + (g % 3) * STAGE, q0);
    if (wave < 2) wait_next<5>(ahead);
    else wait_next<4>(ahead);
    barrier_keep_dma();
  };
  int g = 0;
  for (int it = 0; it < nitem; ++it) {
    if (it == 1) {  // seam: item 0 done, item 1's first tiles are already in the ring
      const int keyB = kbs[1] * 128 + wave * 32 + r;
      const bool kvB = keyB < T;
      bf16x8 kn[4], vn[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (kvB) {
          kn[s] = *reinterpret_cast<const bf16x8*>(kbase + (size_t)keyB * rs + 16 * s + 8 * h);
          vn[s] = *reinterpret_cast<const bf16x8*>(vbase + (size_t)keyB * rs + 16 * s + 8 * h);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) kn[s][j] = vn[s][j] = (bf16)0.f;
        }
      }
      finish_item();
      key0w = kbs[1] * 128 + wave * 32;
      key = keyB;
      kv = kvB;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) kf[s][j] = (bf16)((float)kn[s][j] * scale_log2);
        vf[s] = vn[s];
      }
      dk[0] = dk[1] = dv[0] = dv[1] = zero16();
    }
    const int q0t = qt0_of(it);
    const int pro = min(nqt, q0t + 2);  // the causal diagonal tiles need the mask
    int qt = q0t;
    for (; qt < pro; ++qt, ++g) iter(g, qt, std::true_type{});
    for (; qt < nfull; ++qt, ++g) iter(g, qt, std::false_type{});
    for (; qt < nqt; ++qt, ++g) iter(g, qt, std::true_type{});
  }
  finish_item();
}

}  // namespace fa64

// Outputs written through the LDS row transpose (fa64::store_rows_lds); CAAMD_FA64_STG=0
// selects the direct per-lane stores (A/B)
static bool fa64_staged_stores() {
  static const bool on = [] {
    const char* e = std::getenv("CAAMD_FA64_STG");
    return !(e && e[0] == '0');
  }();
  return on;
}

// head_dim 128 forward (fwd128_kernel); GQA through the row strides and `group`
void fa128_fwd_launch(const bf16* q, const bf16* k, const bf16* v, int q_rs, int kv_rs, int group, bf16* out,
                      float* lse, int B, int T, int H, int causal, hipStream_t st) {
  const float scale_log2 = 1.44269504089f / sqrtf(128.f);
  const int nqb = (T + 127) / 128;
  static const bool pre = [] {  // CAAMD_FA64_FWD_PRE=0: FMA per score (A/B)
    const char* e = std::getenv("CAAMD_FA64_FWD_PRE");
    return !(e && e[0] == '0');
  }();
  auto kern = pre ? fa64::fwd128_kernel<1> : fa64::fwd128_kernel<0>;
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void*)fa64::fwd128_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              8 * fa64::IMG);
    (void)hipFuncSetAttribute((const void*)fa64::fwd128_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              8 * fa64::IMG);
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, dim3(B * H * nqb), dim3(256), 8 * fa64::IMG, st, q, k, v, q_rs, kv_rs,
                     group, out, lse, T, H, nqb, scale_log2, causal);
}

void fa64_fwd_launch(const bf16* q, const bf16* k, const bf16* v, int q_rs, int kv_rs, int group, bf16* out,
                     float* lse, int B, int T, int H, int causal, hipStream_t st) {
  // 128-query blocks of four waves, three waves per SIMD. (256-query blocks -- two
  // 32-query sub-blocks per wave, or eight waves per block -- measured slower,
  // 267 vs 243 us at B32 T1024 H25, and were removed in round 4.)
  const float scale_log2 = 1.44269504089f / 8.f;
  static const int abl = [] {  // development timing ablations (tools/gpu/attn_abl.sh)
    const char* e = std::getenv("CAAMD_FA64_ABL");
    return e ? std::atoi(e) : 0;
  }();
  const int nqb = (T + 127) / 128;
  static const bool pre = [] {  // CAAMD_FA64_FWD_PRE=0: the FMA-per-score forward (A/B)
    const char* e = std::getenv("CAAMD_FA64_FWD_PRE");
    return !(e && e[0] == '0');
  }();
  auto kern = fa64_staged_stores() ? (pre ? fa64::fwd_kernel<1, 0, 4, 1, 1> : fa64::fwd_kernel<1, 0>)
                                   : (pre ? fa64::fwd_kernel<1, 0, 4, 0, 1> : fa64::fwd_kernel<1, 0, 4, 0>);
  switch (abl) {
    case 1: kern = fa64::fwd_kernel<1, 1>; break;
    case 2: kern = fa64::fwd_kernel<1, 2>; break;
    case 3: kern = fa64::fwd_kernel<1, 3>; break;
    case 4: kern = fa64::fwd_kernel<1, 4>; break;
    case 7: kern = fa64::fwd_kernel<1, 7>; break;
    case 8: kern = fa64::fwd_kernel<1, 8>; break;
    default: break;
  }
  hipLaunchKernelGGL(kern, dim3(B * H * nqb), dim3(256), 6 * fa64::IMG, st, q, k, v, q_rs, kv_rs, group, out, lse, T,
                     H, nqb, scale_log2, causal);
}

static int g_fa64_pair = -1;  // -1: from CAAMD_FA64_PAIR (default on)
static bool fa64_pair_mode() {
  if (g_fa64_pair < 0) {
    const char* e = std::getenv("CAAMD_FA64_PAIR");
    g_fa64_pair = (e && e[0] == '0') ? 0 : 1;
  }
  return g_fa64_pair != 0;
}
void fa64_set_pair(int v) { g_fa64_pair = v ? 1 : 0; }

// ws: 2 * B * H * T floats (delta, then lse * log2 e)
void fa64_bwd_launch(const bf16* qkv, const bf16* out, const bf16* dout, const float* lse, float* ws, bf16* dqkv,
                     int B, int T, int H, int causal, hipStream_t st, float* dbias) {
  const int nkb = (T + 127) / 128;
  const float scale = 0.125f;
  const float scale_log2 = 1.44269504089f * scale;
  float* delta = ws;
  float* lse2 = ws + (size_t)B * H * T;
  const int nqb = (T + 127) / 128;  // (a 256-query dQ block variant spilled and was removed in round 4)
  static const int abl = [] {  // development timing ablations of dK/dV (tools/bench_attn.py)
    const char* e = std::getenv("CAAMD_FA64_BWD_ABL");
    return e ? std::atoi(e) : 0;
  }();
  static const int opt = [] {  // dK/dV schedule variants (see bwd_dkdv_kernel)
    const char* e = std::getenv("CAAMD_FA64_DKDV_OPT");
    return e ? std::atoi(e) : (fa64_staged_stores() ? 104 : 32);
  }();
  const bool neg = (opt & 32) && abl == 0;  // the dK/dV variant reads negated lse2 / delta
  auto dq_kern = fa64_staged_stores() ? (neg ? fa64::bwd_dq_kernel<1, 1, 1> : fa64::bwd_dq_kernel<1>)
                                      : (neg ? fa64::bwd_dq_kernel<1, 0, 1> : fa64::bwd_dq_kernel<1, 0>);
  hipLaunchKernelGGL(dq_kern, dim3(B * H * nqb), dim3(256), 6 * fa64::IMG, st, qkv, out, dout, lse,
                     delta, lse2, dqkv, T, H, nqb, scale_log2, scale, causal, dbias);
  auto kern = fa64::bwd_dkdv_kernel<0>;
  switch (opt) {
    case 1: kern = fa64::bwd_dkdv_kernel<0, 1>; break;
    case 2: kern = fa64::bwd_dkdv_kernel<0, 2>; break;
    case 3: kern = fa64::bwd_dkdv_kernel<0, 3>; break;
    case 4: kern = fa64::bwd_dkdv_kernel<0, 4>; break;
    case 5: kern = fa64::bwd_dkdv_kernel<0, 5>; break;
    case 6: kern = fa64::bwd_dkdv_kernel<0, 6>; break;
    case 8: kern = fa64::bwd_dkdv_kernel<0, 8>; break;
    case 12: kern = fa64::bwd_dkdv_kernel<0, 12>; break;
    case 32: kern = fa64::bwd_dkdv_kernel<0, 32>; break;
    case 40: kern = fa64::bwd_dkdv_kernel<0, 40>; break;
    case 44: kern = fa64::bwd_dkdv_kernel<0, 44>; break;
    case 104: kern = fa64::bwd_dkdv_kernel<0, 104>; break;
    default: break;
  }
  switch (abl) {
    case 1: kern = fa64::bwd_dkdv_kernel<1>; break;
    case 2: kern = fa64::bwd_dkdv_kernel<2>; break;
    case 3: kern = fa64::bwd_dkdv_kernel<3>; break;
    case 4: kern = fa64::bwd_dkdv_kernel<4>; break;
    case 7: kern = fa64::bwd_dkdv_kernel<7>; break;
    case 15: kern = fa64::bwd_dkdv_kernel<15>; break;
    case 23: kern = fa64::bwd_dkdv_kernel<23>; break;
    case 31: kern = fa64::bwd_dkdv_kernel<31>; break;
    case 32: kern = fa64::bwd_dkdv_kernel<32>; break;
    case 63: kern = fa64::bwd_dkdv_kernel<63>; break;
    case 95: kern = fa64::bwd_dkdv_kernel<31, 8>; break;  // stripped, staged stores
    default: break;
  }
  // paired key blocks (bwd_dkdv_pair_kernel): CAAMD_FA64_PAIR=0 (or fa64_set_pair(0))
  // -> one key block per workgroup
  if (fa64_pair_mode() && opt == 104 && abl == 0 && causal) {
    const int npair = (nkb + 1) / 2;
    static const bool attr = [] {
      (void)hipFuncSetAttribute((const void*)fa64::bwd_dkdv_pair_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 6 * fa64::IMG + 1536 + 16384);
      return true;
    }();
    (void)attr;
    hipLaunchKernelGGL(fa64::bwd_dkdv_pair_kernel, dim3(B * H * npair), dim3(256), 6 * fa64::IMG + 1536 + 16384, st,
                       qkv, dout, lse2, delta, dqkv, T, H, nkb, npair, scale_log2, scale, causal, dbias);
    return;
  }
  hipLaunchKernelGGL(kern, dim3(B * H * nkb), dim3(256), 6 * fa64::IMG + 1536, st, qkv, dout,
                     lse2, delta, dqkv, T, H, nkb, scale_log2, scale, causal, dbias);
}

}  // namespace caamd
