// Fused softmax cross-entropy over a large vocabulary (GPT-2: V = 50257,
// padded row stride), bf16 logits, fp32 math.
//   fwd: one 256-thread block per row; single streaming pass with an online
//        (max, sum-exp) pair per thread over 16-byte chunks, merged across the
//        block. Writes loss[row] = lse - logit[target] and lse[row].
//   bwd: dlogits[row, j] = dl[row] * (exp(logit - lse) - [j == target]),
//        written IN PLACE over the logits (no second V-wide buffer); padded
//        columns (j >= V) get 0. Rows with target < 0 (ignore_index) get 0.
#include "common.h"

#include <cstdlib>

namespace caamd {

constexpr int kXentThreads = 256;

__global__ __launch_bounds__(kXentThreads) void xent_fwd_kernel(
    const bf16* __restrict__ logits, const int64_t* __restrict__ target, float* __restrict__ loss,
    float* __restrict__ lse_out, int V, int stride) {
  __shared__ float sm[kXentThreads / 64], ss[kXentThreads / 64];
  const int row = blockIdx.x;
  const bf16* x = logits + (size_t)row * stride;
  float m = -INFINITY, s = 0.f;
  const int nfull = V >> 3;
  for (int c = threadIdx.x; c < nfull; c += kXentThreads) {
    float v[8];
    load8(x + c * 8, v);
    float cm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) cm = fmaxf(cm, v[j]);
    const float nm = fmaxf(m, cm);
    float acc = s * __expf(m - nm);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(v[j] - nm);
    m = nm;
    s = acc;
  }
  for (int j = nfull * 8 + threadIdx.x; j < V; j += kXentThreads) {
    const float v = (float)x[j];
    const float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
  }
  // wave merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < kXentThreads / 64; ++i) {
      const float nm = fmaxf(M, sm[i]);
      S = S * __expf(M - nm) + ss[i] * __expf(sm[i] - nm);
      M = nm;
    }
    const float lse = M + __logf(S);
    const int64_t t = target[row];
    lse_out[row] = lse;
    loss[row] = (t >= 0 && t < V) ? (lse - (float)x[t]) : 0.f;
  }
}

__global__ __launch_bounds__(kXentThreads) void xent_bwd_kernel(
    bf16* __restrict__ logits, const int64_t* __restrict__ target, const float* __restrict__ lse,
    const float* __restrict__ dl, int V, int stride) {
  const int row = blockIdx.x;
  bf16* x = logits + (size_t)row * stride;
  const int64_t t = target[row];
  const float g = (t >= 0) ? dl[row] : 0.f;
  const float L = lse[row];
  const int nvec = stride >> 3;  // stride is a multiple of 8
  for (int c = threadIdx.x; c < nvec; c += kXentThreads) {
    float v[8];
    load8(x + c * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c * 8 + j;
      float p = (col < V) ? __expf(v[j] - L) : 0.f;
      if (col == t) p -= 1.f;
      v[j] = g * p;
    }
    store8(x + c * 8, v);
  }
}

// ---- fused forward + backward (the chunked LM head, ops/loss.py) ---------------
// One 1024-thread block per row; the whole row is held in registers (NCH 16-byte
// chunks per lane: a 50,432-wide GPT-2 row is 6,304 chunks = 7 per lane), so the
// logits are read from HBM once and the gradient written once:
//   max -> sum exp -> lse -> loss[row], then dlogits = scale * (softmax - onehot)
// in place. `scale` is a device scalar (1 / #valid targets for a mean loss), so no
// host sync is needed to know the loss normaliser.
// TPB threads per block: 512 (the default) lets two blocks share a CU at the GPT-2 row
// width -- at 1024 threads and ~84 VGPRs only one 16-wave block fits, and its two
// block-wide reductions leave the CU idle (3.7 TB/s); CAAMD_XENT_TPB=1024 is the
// previous launch (A/B).
template <int NCH, int kXentFusedThreads>
__device__ __forceinline__ void xent_fused_body(
    bf16* __restrict__ logits, const int64_t* __restrict__ target, float* __restrict__ loss,
    float* __restrict__ lse_out, const float* __restrict__ scale, int V, int stride) {
  __shared__ float red[kXentFusedThreads / 64];
  __shared__ float bcast;
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  bf16* x = logits + (size_t)row * stride;
  const int nvec = stride >> 3;
  bf16x8 r[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = tid + j * kXentFusedThreads;
    if (c < nvec) r[j] = *reinterpret_cast<const bf16x8*>(x + c * 8);
  }
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = tid + j * kXentFusedThreads;
    if (c < nvec) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c * 8 + e < V) m = fmaxf(m, (float)r[j][e]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) red[w] = m;
  __syncthreads();
  if (tid < 64) {
    float v = tid < kXentFusedThreads / 64 ? red[tid] : -INFINITY;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    if (tid == 0) bcast = v;
  }
  __syncthreads();
  const float M = bcast;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = tid + j * kXentFusedThreads;
    if (c < nvec) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c * 8 + e < V) s += __expf((float)r[j][e] - M);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __syncthreads();  // everyone has read bcast / red before they are reused
  if (lane == 0) red[w] = s;
  __syncthreads();
  if (tid < 64) {
    float v = tid < kXentFusedThreads / 64 ? red[tid] : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (tid == 0) bcast = v;
  }
  __syncthreads();
  const float L = M + __logf(bcast);
  const int64_t t = target[row];
  const bool valid = t >= 0 && t < V;
  const float g = t >= 0 ? scale[0] : 0.f;
  if (tid == 0) {
    lse_out[row] = L;
    if (!valid) loss[row] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = tid + j * kXentFusedThreads;
    if (c < nvec) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = c * 8 + e;
        const float v = (float)r[j][e];
        float p = col < V ? __expf(v - L) : 0.f;
        if (col == t) {
          loss[row] = L - v;
          p -= 1.f;
        }
        o[e] = (bf16)(g * p);
      }
      *reinterpret_cast<bf16x8*>(x + c * 8) = o;
    }
  }
}

template <int NCH>
__global__ __launch_bounds__(1024) void xent_fused_kernel(bf16* __restrict__ logits, const int64_t* __restrict__ target,
                                                          float* __restrict__ loss, float* __restrict__ lse_out,
                                                          const float* __restrict__ scale, int V, int stride) {
  xent_fused_body<NCH, 1024>(logits, target, loss, lse_out, scale, V, stride);
}
// 512 threads, at most 128 VGPRs (4 waves per SIMD): two blocks per CU
template <int NCH>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void xent_fused512_kernel(
    bf16* __restrict__ logits, const int64_t* __restrict__ target, float* __restrict__ loss,
    float* __restrict__ lse_out, const float* __restrict__ scale, int V, int stride) {
  xent_fused_body<NCH, 512>(logits, target, loss, lse_out, scale, V, stride);
}

bool xent_fused_launch(bf16* logits, const int64_t* target, float* loss, float* lse, const float* scale,
                       int rows, int V, int stride, hipStream_t st) {
  const int nvec = stride >> 3;
  static const int tpb_env = [] {
    const char* e = std::getenv("CAAMD_XENT_TPB");
    return e ? std::atoi(e) : 512;
  }();
  if (tpb_env == 512 && nvec > 4 * 1024 && nvec <= 13 * 512) {  // wide rows: 512-thread blocks
    hipLaunchKernelGGL(xent_fused512_kernel<13>, dim3(rows), dim3(512), 0, st, logits, target, loss, lse, scale, V,
                       stride);
    return true;
  }
#define XENT_FUSED(N, T)                                                                                    \
  hipLaunchKernelGGL(xent_fused_kernel<N>, dim3(rows), dim3(T), 0, st, logits, target, loss, lse, scale, V, stride)
  const int nch = (nvec + 1023) / 1024;
  if (nch <= 1) XENT_FUSED(1, 1024);
  else if (nch <= 2) XENT_FUSED(2, 1024);
  else if (nch <= 4) XENT_FUSED(4, 1024);
  else if (nch <= 7) XENT_FUSED(7, 1024);
  else if (nch <= 8) XENT_FUSED(8, 1024);
  else if (nch <= 16) XENT_FUSED(16, 1024);
  else return false;
#undef XENT_FUSED
  return true;
}

void xent_fwd_launch(const bf16* logits, const int64_t* target, float* loss, float* lse, int rows,
                     int V, int stride, hipStream_t st) {
  hipLaunchKernelGGL(xent_fwd_kernel, dim3(rows), dim3(kXentThreads), 0, st, logits, target, loss,
                     lse, V, stride);
}

void xent_bwd_launch(bf16* logits, const int64_t* target, const float* lse, const float* dl,
                     int rows, int V, int stride, hipStream_t st) {
  hipLaunchKernelGGL(xent_bwd_kernel, dim3(rows), dim3(kXentThreads), 0, st, logits, target, lse,
                     dl, V, stride);
}

}  // namespace caamd
