// Fused softmax cross-entropy over a large vocabulary (GPT-2: V = 50257,
// padded row stride), bf16 logits, fp32 math.
//   fwd: one 256-thread block per row; single streaming pass with an online
//        (max, sum-exp) pair per thread over 16-byte chunks, merged across the
//        block. Writes loss[row] = lse - logit[target] and lse[row].
//   bwd: dlogits[row, j] = dl[row] * (exp(logit - lse) - [j == target]),
//        written IN PLACE over the logits (no second V-wide buffer); padded
//        columns (j >= V) get 0. Rows with target < 0 (ignore_index) get 0.
#include "common.h"

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
