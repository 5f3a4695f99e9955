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

template <bool NT>
__device__ __forceinline__ f32x4 ld4(const f32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(f32x4* p, f32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// NT: non-temporal (streaming) loads / stores — every byte is touched once per
// step, so they need not displace the L2 / MALL. UNR: vectors per thread per
// iteration (all loads issued before any math, for more bytes in flight).
template <typename GT, bool WRITE_BF16, bool NT, int UNR>
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
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < nvec; i0 += stride * UNR) {
    float gv[UNR][8];
    f32x4 pa[UNR], pb[UNR], ma[UNR], mb[UNR], va[UNR], vb[UNR];
    float decay[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < nvec) {
        load_grad8<GT>(g + i * 8, gv[u]);
        decay[u] = (wd_mask == nullptr || wd_mask[i]) ? decay_on : 1.f;
        const f32x4* p4 = reinterpret_cast<const f32x4*>(p + i * 8);
        const f32x4* m4 = reinterpret_cast<const f32x4*>(m + i * 8);
        const f32x4* v4 = reinterpret_cast<const f32x4*>(v + i * 8);
        pa[u] = ld4<NT>(p4); pb[u] = ld4<NT>(p4 + 1);
        ma[u] = ld4<NT>(m4); mb[u] = ld4<NT>(m4 + 1);
        va[u] = ld4<NT>(v4); vb[u] = ld4<NT>(v4 + 1);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= nvec) break;
      float pp[8] = {pa[u][0], pa[u][1], pa[u][2], pa[u][3], pb[u][0], pb[u][1], pb[u][2], pb[u][3]};
      float mm[8] = {ma[u][0], ma[u][1], ma[u][2], ma[u][3], mb[u][0], mb[u][1], mb[u][2], mb[u][3]};
      float vv[8] = {va[u][0], va[u][1], va[u][2], va[u][3], vb[u][0], vb[u][1], vb[u][2], vb[u][3]};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gj = gv[u][j] * scale;
        mm[j] = h.beta1 * mm[j] + (1.f - h.beta1) * gj;
        vv[j] = h.beta2 * vv[j] + (1.f - h.beta2) * gj * gj;
        const float denom = sqrtf(vv[j]) * inv_bc2_sqrt + h.eps;
        pp[j] = pp[j] * decay[u] - step * mm[j] / denom;
      }
      f32x4* p4 = reinterpret_cast<f32x4*>(p + i * 8);
      f32x4* m4 = reinterpret_cast<f32x4*>(m + i * 8);
      f32x4* v4 = reinterpret_cast<f32x4*>(v + i * 8);
      st4<NT>(p4, f32x4{pp[0], pp[1], pp[2], pp[3]});
      st4<NT>(p4 + 1, f32x4{pp[4], pp[5], pp[6], pp[7]});
      st4<NT>(m4, f32x4{mm[0], mm[1], mm[2], mm[3]});
      st4<NT>(m4 + 1, f32x4{mm[4], mm[5], mm[6], mm[7]});
      st4<NT>(v4, f32x4{vv[0], vv[1], vv[2], vv[3]});
      st4<NT>(v4 + 1, f32x4{vv[4], vv[5], vv[6], vv[7]});
      if (WRITE_BF16) store8(pbf + i * 8, pp);
    }
  }
}

// bit 0: non-temporal (3.3 vs 4.8 TB/s: slower), bit 1: 2 vectors per thread per
// iteration (8.82-8.91 vs 9.08 ms over 1.56 B params: the default), bit 2: no
// grid-stride loop (grid covers the buffer once), bit 3: 4 vectors per thread;
// tools/bench_adamw.py
static int g_adam_variant = 4;
void adamw_config(int variant) { g_adam_variant = variant; }

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
  // bit 2: one pass, no grid-stride loop (a block per 256 x UNR vectors)
  const int unr = (g_adam_variant & 2) ? 2 : ((g_adam_variant & 8) ? 4 : 1);
  const int64_t full = (nvec + 256LL * unr - 1) / (256LL * unr);
  const int grid = (g_adam_variant & 4) ? (int)std::min<int64_t>(full, 1 << 30) : ew_grid(nvec, 256);
#define CA_ADAM2(GT, W, NT, U)                                                                   \
  hipLaunchKernelGGL((adamw_kernel<GT, W, NT, U>), dim3(grid), dim3(256), 0, st, p, m, v, (const GT*)g, \
                     pbf, nvec, h, sumsq, wd_mask)
#define CA_ADAM(GT, W)                                          \
  do {                                                          \
    if (g_adam_variant & 8) { CA_ADAM2(GT, W, false, 4); break; } \
    switch (g_adam_variant & 3) {                               \
      case 1: CA_ADAM2(GT, W, true, 1); break;                  \
      case 2: CA_ADAM2(GT, W, false, 2); break;                 \
      case 3: CA_ADAM2(GT, W, true, 2); break;                  \
      default: CA_ADAM2(GT, W, false, 1); break;                \
    }                                                           \
  } while (0)
  if (g_bf16) {
    if (pbf) CA_ADAM(bf16, true);
    else CA_ADAM(bf16, false);
  } else {
    if (pbf) CA_ADAM(float, true);
    else CA_ADAM(float, false);
  }
#undef CA_ADAM2
#undef CA_ADAM
}

}  // namespace caamd
