// Fused bias + GELU(tanh) forward and backward (GPT-2 MLP), bf16 I/O.
//   fwd: y = gelu(h + b)                               (one read of h, one write)
//   bwd: dh = dy * gelu'(h + b);  db = sum_rows dh     (dbias fused: per-thread
//        column accumulators over a row slab -> fp32 partials -> column reduce)
// 16-byte (8 x bf16) vector accesses everywhere (CDNA guideline 13).
#include "common.h"

namespace caamd {

// gelu_tanh / gelu_tanh_grad: common.h

__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const bf16* __restrict__ h,
                                                            const bf16* __restrict__ b,
                                                            bf16* __restrict__ y, int64_t nvec,
                                                            int ncv) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(i % ncv);
    float hv[8], bv[8], o[8];
    load8(h + i * 8, hv);
    if (b) load8(b + cv * 8, bv);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = gelu_tanh(hv[j] + bv[j]);
    store8(y + i * 8, o);
  }
}

// grid: x = ceil(ncv / 256) column tiles, y = row slabs.
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(
    const bf16* __restrict__ dy, const bf16* __restrict__ h, const bf16* __restrict__ b,
    bf16* __restrict__ dh, float* __restrict__ partial, int rows, int ncv, int rows_per) {
  const int cv = blockIdx.x * blockDim.x + threadIdx.x;
  if (cv >= ncv) return;
  const int N = ncv * 8;
  float bv[8], acc[8];
  if (b) load8(b + cv * 8, bv);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    acc[j] = 0.f;
    if (!b) bv[j] = 0.f;
  }
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(rows, r0 + rows_per);
#pragma unroll 4
  for (int r = r0; r < r1; ++r) {
    const size_t off = (size_t)r * N + cv * 8;
    float hv[8], dv[8], o[8];
    load8(h + off, hv);
    load8(dy + off, dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = dv[j] * gelu_tanh_grad(hv[j] + bv[j]);
      acc[j] += o[j];
    }
    store8(dh + off, o);
  }
  if (partial) {
    float* p = partial + (size_t)blockIdx.y * N + cv * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = acc[j];
  }
}

void colsum_bf16_launch(const float* partial, int nrow, int ncol, int split, bf16* o0, bf16* o1,
                        hipStream_t st, int accumulate);

void bias_gelu_fwd_launch(const bf16* h, const bf16* b, bf16* y, int64_t rows, int N,
                          hipStream_t st) {
  const int64_t nvec = rows * (int64_t)N / 8;
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, dim3(ew_grid(nvec, 256)), dim3(256), 0, st, h, b, y,
                     nvec, N / 8);
}

int bias_gelu_bwd_slabs(int rows) {
  int s = (rows + 63) / 64;  // 64 rows per slab
  return s < 1 ? 1 : s;
}

void bias_gelu_bwd_launch(const bf16* dy, const bf16* h, const bf16* b, bf16* dh, float* partial,
                          bf16* db, int rows, int N, hipStream_t st) {
  const int ncv = N / 8;
  const int slabs = bias_gelu_bwd_slabs(rows);
  const int rows_per = (rows + slabs - 1) / slabs;
  hipLaunchKernelGGL(bias_gelu_bwd_kernel, dim3((ncv + 255) / 256, slabs), dim3(256), 0, st, dy, h,
                     b, dh, partial, rows, ncv, rows_per);
  if (db) colsum_bf16_launch(partial, slabs, N, N, db, db, st, 0);
}

// dbias = sum over rows of dy [rows, N] (bf16) -> fp32 slab partials -> bf16,
// optionally accumulated into an existing gradient (the flat main-grad buffer).
__global__ __launch_bounds__(256) void rowsum_partial_kernel(const bf16* __restrict__ dy,
                                                             float* __restrict__ partial, int rows,
                                                             int ncv, int rows_per) {
  const int cv = blockIdx.x * blockDim.x + threadIdx.x;
  if (cv >= ncv) return;
  const int N = ncv * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(rows, r0 + rows_per);
#pragma unroll 4
  for (int r = r0; r < r1; ++r) {
    float v[8];
    load8(dy + (size_t)r * N + cv * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  float* p = partial + (size_t)blockIdx.y * N + cv * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) p[j] = acc[j];
}

// dst (bf16 main gradient) += src (fp32 accumulator, e.g. the dGELU GEMM epilogue's
// atomic bias-gradient sums), then src = 0 for its next use: one launch in place of
// zero-fill + convert + add.
__global__ __launch_bounds__(256) void drain_f32_kernel(float* __restrict__ src, bf16* __restrict__ dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    dst[i] = (bf16)((float)dst[i] + src[i]);
    src[i] = 0.f;
  }
}

void drain_f32_launch(float* src, bf16* dst, int n, hipStream_t st) {
  hipLaunchKernelGGL(drain_f32_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, n);
}

void bias_grad_launch(const bf16* dy, float* partial, bf16* out, int rows, int N, int accumulate,
                      hipStream_t st) {
  const int ncv = N / 8;
  const int slabs = bias_gelu_bwd_slabs(rows);
  const int rows_per = (rows + slabs - 1) / slabs;
  hipLaunchKernelGGL(rowsum_partial_kernel, dim3((ncv + 255) / 256, slabs), dim3(256), 0, st, dy,
                     partial, rows, ncv, rows_per);
  colsum_bf16_launch(partial, slabs, N, N, out, out, st, accumulate);
}

}  // namespace caamd
