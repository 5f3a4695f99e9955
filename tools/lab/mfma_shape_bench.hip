// Microbenchmark: v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 as the GEMM
// main loop uses them -- every operand fragment re-read from LDS by ds_read_b128 each
// K-step, the same 128 x 64 output tile per wave (the k64 kernel's 256 x 256 tile over
// 2 x 4 waves), 2 waves per SIMD, random bf16 data (zero operands let the chip hold a
// higher clock and rank the shapes by cycles only: MI355X_MICROARCH.md "Clock" (7)).
//
// Per wave and per 32-deep K-step both shapes read the same 12 KB of fragments from LDS
// (A 128 rows x 32 k, B 64 cols x 32 k) and do the same 524,288 FLOPs:
//   SHAPE 16: 8 A x 4 B fragments (16 x 32 each), 32 MFMAs 16x16x32
//   SHAPE 32: per 16-deep half, 4 A x 2 B fragments (32 x 16 each), 8 MFMAs 32x32x16
// so LDS bytes per FLOP depend on the wave tile, not on the MFMA shape; what differs is
// the clock the chip holds and the issue pattern. The two shapes alternate, each
// launched back to back for >= 1.5 s before it is timed.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/lab/mfma_shape_bench tools/lab/mfma_shape_bench.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) const bf16x8 lds_v;
typedef __attribute__((address_space(3))) const char lds_c;

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

constexpr int IMG = 24 * 1024;  // per-wave-pair image: A 16 KB + B 8 KB (bf16, 128 + 64 rows x 64 B)

// lane-linear 16-byte reads: conflict-free for ds_read_b128
__device__ __forceinline__ bf16x8 rd(lds_c* base, int frag, int lane) {
  return *(lds_v*)(base + frag * 1024 + lane * 16);
}

template <int SHAPE>
__global__ __launch_bounds__(512, 1) void bench(const bf16x8* __restrict__ src, float* __restrict__ out, int iters) {
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // fill the LDS with random data from global (one image per pair of waves)
  for (int i = tid; i < 4 * IMG / 16; i += 512) *(bf16x8*)(smem + i * 16) = src[(blockIdx.x * 97 + i) % 65536];
  __syncthreads();
  lds_c* img = (lds_c*)(smem + (wave >> 1) * IMG);
  float sink = 0.f;
  if constexpr (SHAPE == 16) {
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
      bf16x8 a[8], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = rd(img + 16384, j + 4 * (it & 1), lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = rd(img, i + 8 * (it & 1), lane);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sink += acc[i][j][0] + acc[i][j][3];
  } else {
    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8 a[4], b[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = rd(img + 16384, j + 2 * h + 4 * (it & 1), lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = rd(img, i + 4 * h + 8 * (it & 1), lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) sink += acc[i][j][0] + acc[i][j][15];
  }
  out[blockIdx.x * 512 + tid] = sink;
}

template <int SHAPE>
static double run(const bf16x8* src, float* out, int grid, int iters, double warm_s) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < warm_s) {
    for (int r = 0; r < 4; ++r) hipLaunchKernelGGL(bench<SHAPE>, dim3(grid), dim3(512), 0, 0, src, out, iters);
    CHECK(hipDeviceSynchronize());
  }
  const int reps = 8;
  CHECK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(bench<SHAPE>, dim3(grid), dim3(512), 0, 0, src, out, iters);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  const double flops = (double)reps * grid * 8 /*waves*/ * iters * 524288.0;
  return flops / (ms * 1e-3) / 1e12;  // TFLOP/s
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
  const int grid = 256 * 2;  // one 8-wave workgroup per CU at a time (2 waves per SIMD), two rounds
  std::vector<unsigned short> h(65536 * 8);
  unsigned s = 12345u;
  for (auto& v : h) {
    s = s * 1664525u + 1013904223u;
    const float f = ((s >> 9) & 0xffff) / 65536.0f - 0.5f;  // random in [-0.5, 0.5)
    unsigned u;
    std::memcpy(&u, &f, 4);
    v = (unsigned short)(u >> 16);
  }
  bf16x8* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMalloc(&out, (size_t)grid * 512 * 4));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  for (int round = 0; round < 3; ++round) {
    const double t16 = run<16>(src, out, grid, iters, 1.5);
    const double t32 = run<32>(src, out, grid, iters, 1.5);
    std::printf("{\"round\": %d, \"tflops_16x16x32\": %.1f, \"tflops_32x32x16\": %.1f, \"ratio_16_over_32\": %.3f}\n",
                round, t16, t32, t16 / t32);
    std::fflush(stdout);
  }
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
