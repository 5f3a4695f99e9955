// Fused AdamW over FLAT buffers (one launch for the whole model):
//   fp32 master weights p, fp32 moments m/v, bf16 (or fp32) gradients g,
//   optional bf16 model-weight copy written in the same pass.
// Weight decay is applied per 8-element chunk where wd_mask[chunk] != 0 (params
// are 8-aligned in the flat buffer, so a chunk never straddles two params).
// Global-norm gradient clipping and the data-parallel 1/world factor are folded
// into a device-resident scale (no host sync): scale = inv_world *
// min(1, max_norm / (||g * inv_world|| + 1e-6)), computed from the sum of
// squares produced by grad_sumsq (one fp32 atomic per block).
// Memory-bound: 8 elements / thread / iteration, 16-byte bf16 and 2x16-byte
// fp32 accesses, grid capped at 2048 blocks with a grid-stride loop.
#include "common.h"

namespace caamd {

template <typename GT>
__device__ __forceinline__ void load_grad8(const GT* g, float (&f)[8]);
template <>
__device__ __forceinline__ void load_grad8<bf16>(const bf16* g, float (&f)[8]) {
  load8(g, f);
}
template <>
__device__ __forceinline__ void load_grad8<float>(const float* g, float (&f)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(g);
  const f32x4 b = *reinterpret_cast<const f32x4*>(g + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = a[j];
    f[4 + j] = b[j];
  }
}

template <typename GT>
__global__ __launch_bounds__(256) void sumsq_kernel(const GT* __restrict__ g, int64_t nvec,
                                                    float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    load_grad8<GT>(g + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j] * v[j];
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) atomicAdd(out, acc);
}

struct AdamHyper {
  float lr, beta1, beta2, eps, wd, bc1, bc2;  // bc = 1 - beta^t
  float inv_world, max_norm;                  // max_norm <= 0 disables clipping
};

template <typename GT, bool WRITE_BF16>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, float* __restrict__ m,
                                                    float* __restrict__ v,
                                                    const GT* __restrict__ g,
                                                    bf16* __restrict__ pbf, int64_t nvec,
                                                    AdamHyper h, const float* __restrict__ sumsq,
                                                    const uint8_t* __restrict__ wd_mask) {
  float scale = h.inv_world;
  if (h.max_norm > 0.f && sumsq) {
    const float norm = sqrtf(*sumsq) * h.inv_world;
    scale *= fminf(1.f, h.max_norm / (norm + 1e-6f));
  }
  const float step = h.lr / h.bc1;
  const float inv_bc2_sqrt = rsqrtf(h.bc2);
  const float decay_on = 1.f - h.lr * h.wd;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gv[8];
    load_grad8<GT>(g + i * 8, gv);
    const float decay = (wd_mask == nullptr || wd_mask[i]) ? decay_on : 1.f;
    f32x4* p4 = reinterpret_cast<f32x4*>(p + i * 8);
    f32x4* m4 = reinterpret_cast<f32x4*>(m + i * 8);
    f32x4* v4 = reinterpret_cast<f32x4*>(v + i * 8);
    f32x4 pa = p4[0], pb = p4[1], ma = m4[0], mb = m4[1], va = v4[0], vb = v4[1];
    float pp[8] = {pa[0], pa[1], pa[2], pa[3], pb[0], pb[1], pb[2], pb[3]};
    float mm[8] = {ma[0], ma[1], ma[2], ma[3], mb[0], mb[1], mb[2], mb[3]};
    float vv[8] = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gj = gv[j] * scale;
      mm[j] = h.beta1 * mm[j] + (1.f - h.beta1) * gj;
      vv[j] = h.beta2 * vv[j] + (1.f - h.beta2) * gj * gj;
      const float denom = sqrtf(vv[j]) * inv_bc2_sqrt + h.eps;
      pp[j] = pp[j] * decay - step * mm[j] / denom;
    }
    p4[0] = f32x4{pp[0], pp[1], pp[2], pp[3]};
    p4[1] = f32x4{pp[4], pp[5], pp[6], pp[7]};
    m4[0] = f32x4{mm[0], mm[1], mm[2], mm[3]};
    m4[1] = f32x4{mm[4], mm[5], mm[6], mm[7]};
    v4[0] = f32x4{vv[0], vv[1], vv[2], vv[3]};
    v4[1] = f32x4{vv[4], vv[5], vv[6], vv[7]};
    if (WRITE_BF16) store8(pbf + i * 8, pp);
  }
}

void grad_sumsq_launch(const void* g, bool g_bf16, int64_t n, float* out, hipStream_t st) {
  const int64_t nvec = n / 8;
  const int grid = ew_grid(nvec, 256);
  if (g_bf16)
    hipLaunchKernelGGL(sumsq_kernel<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)g, nvec, out);
  else
    hipLaunchKernelGGL(sumsq_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)g, nvec,
                       out);
}

void adamw_launch(float* p, float* m, float* v, const void* g, bool g_bf16, bf16* pbf, int64_t n,
                  float lr, float beta1, float beta2, float eps, float wd, float bc1, float bc2,
                  float inv_world, float max_norm, const float* sumsq, const uint8_t* wd_mask,
                  hipStream_t st) {
  AdamHyper h{lr, beta1, beta2, eps, wd, bc1, bc2, inv_world, max_norm};
  const int64_t nvec = n / 8;
  const int grid = ew_grid(nvec, 256);
#define CA_ADAM(GT, W)                                                                        \
  hipLaunchKernelGGL((adamw_kernel<GT, W>), dim3(grid), dim3(256), 0, st, p, m, v, (const GT*)g, \
                     pbf, nvec, h, sumsq, wd_mask)
  if (g_bf16) {
    if (pbf) CA_ADAM(bf16, true);
    else CA_ADAM(bf16, false);
  } else {
    if (pbf) CA_ADAM(float, true);
    else CA_ADAM(float, false);
  }
#undef CA_ADAM
}

}  // namespace caamd
