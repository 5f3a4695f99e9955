// Vision inference helpers for the Data GPU map_batches path (ResNet-50):
//   * image_normalize: uint8 NHWC (the object-store block layout of decoded
//     images) -> bf16 NHWC ("channels_last", what MIOpen's NHWC convolutions
//     consume) with per-channel (x/255 - mean) / std, in one HBM pass.
//   * add_relu_: y = max(y + r, 0) in place — the residual join of a
//     bottleneck block after the BN-folded conv (one pass instead of two).
// Both are HBM-bound elementwise kernels: 16-byte loads/stores per lane,
// grid capped to a few waves per SIMD with a grid-stride loop.
#include "common.h"

namespace caamd {

// Each lane converts 16 pixels = 48 input bytes (3 x 16-byte loads) to 48 bf16
// (6 x 16-byte stores); 48 is a multiple of C=3 so the channel of element j is
// j % 3 for every chunk.
__global__ __launch_bounds__(256) void image_normalize_kernel(const uint8_t* __restrict__ in,
                                                              bf16* __restrict__ out, int64_t nchunk,
                                                              float s0, float s1, float s2, float b0,
                                                              float b1, float b2) {
  const float sc[3] = {s0, s1, s2}, bi[3] = {b0, b1, b2};
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < nchunk;
       c += (int64_t)gridDim.x * blockDim.x) {
    const uint4* src = reinterpret_cast<const uint4*>(in + c * 48);
    uint4 raw[3] = {src[0], src[1], src[2]};
    const uint8_t* b = reinterpret_cast<const uint8_t*>(raw);
    bf16x8 o[6];
#pragma unroll
    for (int j = 0; j < 48; ++j) o[j >> 3][j & 7] = (bf16)__builtin_fmaf((float)b[j], sc[j % 3], bi[j % 3]);
    bf16x8* dst = reinterpret_cast<bf16x8*>(out + c * 48);
#pragma unroll
    for (int k = 0; k < 6; ++k) dst[k] = o[k];
  }
}

// tail (< 48 bytes) handled per element
__global__ void image_normalize_tail_kernel(const uint8_t* __restrict__ in, bf16* __restrict__ out,
                                            int64_t start, int64_t n, float s0, float s1, float s2,
                                            float b0, float b1, float b2) {
  const int64_t i = start + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int ch = (int)(i % 3);
  const float s = ch == 0 ? s0 : (ch == 1 ? s1 : s2), bb = ch == 0 ? b0 : (ch == 1 ? b1 : b2);
  out[i] = (bf16)__builtin_fmaf((float)in[i], s, bb);
}

void image_normalize_launch(const uint8_t* in, bf16* out, int64_t n, const float* scale,
                            const float* bias, hipStream_t st) {
  const int64_t nchunk = n / 48;
  if (nchunk > 0) {
    hipLaunchKernelGGL(image_normalize_kernel, dim3(ew_grid(nchunk, 256)), dim3(256), 0, st, in, out,
                       nchunk, scale[0], scale[1], scale[2], bias[0], bias[1], bias[2]);
  }
  const int64_t done = nchunk * 48;
  if (done < n) {
    hipLaunchKernelGGL(image_normalize_tail_kernel, dim3((unsigned)((n - done + 255) / 256)), dim3(256), 0,
                       st, in, out, done, n, scale[0], scale[1], scale[2], bias[0], bias[1], bias[2]);
  }
}

__global__ __launch_bounds__(256) void add_relu_kernel(bf16* __restrict__ y, const bf16* __restrict__ r,
                                                       int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    bf16x8 a = reinterpret_cast<const bf16x8*>(y)[i];
    const bf16x8 b = reinterpret_cast<const bf16x8*>(r)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (bf16)fmaxf((float)a[j] + (float)b[j], 0.f);
    reinterpret_cast<bf16x8*>(y)[i] = a;
  }
}

void add_relu_launch(bf16* y, const bf16* r, int64_t n, hipStream_t st) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(add_relu_kernel, dim3(ew_grid(n8, 256)), dim3(256), 0, st, y, r, n8);
}

// Epilogue of a bias-free MIOpen convolution in NHWC: y = act(y + b[c] (+ r)).
// Replaces MIOpen's separate bias kernel + torch's ReLU (+ the residual add):
// one read-modify-write pass instead of three. C % 8 == 0, so every 8-element
// chunk lies inside one pixel and its channels are c0 .. c0 + 7.
template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bias_act_kernel(bf16* __restrict__ y, const bf16* __restrict__ b,
                                                       const bf16* __restrict__ r, int64_t n8, int C) {
  const int c8 = C >> 3;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    bf16x8 a = reinterpret_cast<const bf16x8*>(y)[i];
    const bf16x8 bb = reinterpret_cast<const bf16x8*>(b)[i % c8];
    bf16x8 rr;
    if (RES) rr = reinterpret_cast<const bf16x8*>(r)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = (float)a[j] + (float)bb[j];
      if (RES) v += (float)rr[j];
      if (RELU) v = fmaxf(v, 0.f);
      a[j] = (bf16)v;
    }
    reinterpret_cast<bf16x8*>(y)[i] = a;
  }
}

void bias_act_launch(bf16* y, const bf16* b, const bf16* r, int64_t n, int C, bool relu, hipStream_t st) {
  const int64_t n8 = n / 8;
  dim3 g(ew_grid(n8, 256)), blk(256);
  if (r) {
    if (relu) hipLaunchKernelGGL((bias_act_kernel<true, true>), g, blk, 0, st, y, b, r, n8, C);
    else hipLaunchKernelGGL((bias_act_kernel<true, false>), g, blk, 0, st, y, b, r, n8, C);
  } else {
    if (relu) hipLaunchKernelGGL((bias_act_kernel<false, true>), g, blk, 0, st, y, b, r, n8, C);
    else hipLaunchKernelGGL((bias_act_kernel<false, false>), g, blk, 0, st, y, b, r, n8, C);
  }
}

}  // namespace caamd
