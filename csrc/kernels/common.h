// Shared device helpers for the gfx950 (CDNA4) kernels.
// Wave = 64 lanes. bf16 is the native __bf16 type so the compiler emits
// v_cvt_pk_bf16_f32 for float->bf16 (round-to-nearest-even).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

namespace caamd {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ void load8(const bf16* p, float (&f)[8]) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
}

__device__ __forceinline__ void store8(bf16* p, const float (&f)[8]) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)f[j];
  *reinterpret_cast<bf16x8*>(p) = v;
}

// Grid for a memory-bound elementwise launch: cap at 256 CUs x 8 blocks.
inline int ew_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// GELU(tanh) in sigmoid form: 0.5 (1 + tanh(u)) = sigmoid(2u), so
//   gelu(z)  = z * s,                    s = 1 / (1 + 2^(-2u log2 e)), u = k0 (z + k1 z^3)
//   gelu'(z) = s + z * s * (1 - s) * 2 k0 (1 + 3 k1 z^2)
// on one v_exp_f32 and one v_rcp_f32 (the fused epilogues run after the MFMA loop,
// so their VALU count is exposed; __fdividef compiled to the full IEEE division
// sequence, ~10 VALU per element). Saturates through exp overflow / underflow:
// rcp(inf) = 0 gives gelu = 0 and gelu' = 0 for very negative z.
constexpr float GELU_K0 = 0.7978845608028654f, GELU_K1 = 0.044715f;
constexpr float GELU_C0 = -2.f * GELU_K0 * 1.4426950408889634f;  // -2 k0 log2(e)
constexpr float GELU_C1 = GELU_C0 * GELU_K1;
__device__ __forceinline__ float gelu_sig(float z, float z2) {
  const float t = z * __builtin_fmaf(GELU_C1, z2, GELU_C0);  // -2u log2 e
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(t));
}
__device__ __forceinline__ float gelu_tanh(float z) {
  return z * gelu_sig(z, z * z);
}
__device__ __forceinline__ float gelu_tanh_grad(float z) {
  const float z2 = z * z;
  const float s = gelu_sig(z, z2);
  const float dv = __builtin_fmaf(6.f * GELU_K0 * GELU_K1, z2, 2.f * GELU_K0);  // d(2u)/dz
  return __builtin_fmaf(z * s * (1.f - s), dv, s);
}

}  // namespace caamd
