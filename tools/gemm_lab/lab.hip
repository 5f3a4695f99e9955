// Standalone GEMM lab: numerics (vs an fp32 GPU reference) and interleaved timing of
// the gemm.hip variants on the GPT-2-XL training shapes, without torch (a fresh GPU
// box runs it in seconds). Build: tools/gemm_lab/build.sh; run: ./gemm_lab [filter]
//
// Every variant of one shape is timed in the same process, rounds interleaved
// (cdna_hip_programming.md §5.4 rule 24), on uniform random [-1, 1) bf16 operands
// (rule 25). Output: one JSON line per (shape, variant).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../csrc/kernels/common.h"

namespace caamd {
hipError_t gemm_launch(int layout, int epi, int bm, int bn, const bf16* A, const bf16* B, void* C,
                       const bf16* bias, const bf16* Z, bf16* Zout, float* dbias, int M, int N, int K,
                       int lda, int ldb, int ldc, int splitk, int algo, hipStream_t st, int tfull, int tS,
                       float* tws, int* tcnt, int bpack);
void gemm_tail_plan(int tiles, int K, int ks, int slots, int max_split, int* full, int* S);
void gemm_set_group_m(int g);
}  // namespace caamd
using caamd::bf16;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

__global__ void fill_kernel(bf16* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    p[i] = (bf16)(scale * ((x >> 8) * (2.0f / 16777216.0f) - 1.0f));
  }
}

// fp32 reference of rows [r0, r0 + R) of C = A B^T (+ bias) (NT layout)
__global__ void ref_kernel(const bf16* A, const bf16* B, const bf16* bias, float* out, int r0, int R, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = blockIdx.y;
  if (n >= N || r >= R) return;
  const bf16* a = A + (size_t)(r0 + r) * K;
  const bf16* b = B + (size_t)n * K;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)a[k] * (float)b[k];
  if (bias) s += (float)bias[n];
  out[(size_t)r * N + n] = s;
}

static float bf2f(bf16 v) { return (float)v; }

struct Shape {
  const char* name;
  int M, N, K, epi;  // epi: 0 bf16 (+bias), 3 bias+gelu, 4 dgelu
};

static double gelu_ref(double z) { return 0.5 * z * (1.0 + tanh(0.7978845608028654 * (z + 0.044715 * z * z * z))); }
static double gelu_grad_ref(double z) {
  const double u = 0.7978845608028654 * (z + 0.044715 * z * z * z), t = tanh(u);
  return 0.5 * (1.0 + t) + 0.5 * z * (1.0 - t * t) * 0.7978845608028654 * (1.0 + 3 * 0.044715 * z * z);
}

int main(int argc, char** argv) {
  const char* filter = argc > 1 ? argv[1] : "";
  const int iters = argc > 2 ? atoi(argv[2]) : 10;
  const int rounds = argc > 3 ? atoi(argv[3]) : 5;
  std::vector<int> algos;
  if (argc > 4) {
    char buf[256];
    strncpy(buf, argv[4], 255);
    buf[255] = 0;
    for (char* t = strtok(buf, ","); t; t = strtok(nullptr, ",")) algos.push_back(atoi(t));
  } else {
    algos = {2, 9, 1009, 3009};
  }
  // argv[5] (optional): m-tiles per tile-order group of the full-line kernel
  if (argc > 5) caamd::gemm_set_group_m(atoi(argv[5]));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::vector<Shape> shapes = {
      {"qkv_fwd", 32768, 4800, 1600, 0},  {"proj_fwd", 32768, 1600, 1600, 0}, {"fc_fwd", 32768, 6400, 1600, 3},
      {"fc2_fwd", 32768, 1600, 6400, 0},  {"qkv_dgrad", 32768, 1600, 4800, 0}, {"fc2_dgrad", 32768, 6400, 1600, 4},
      {"fc_fwd_plain", 32768, 6400, 1600, 0},
      // Llama-3-8B prefill at 16384 tokens (256 x 256 tiles)
      {"pf_qkv", 16384, 6144, 4096, 0},   {"pf_o", 16384, 4096, 4096, 0},      {"pf_gate_up", 16384, 28672, 4096, 0},
      {"pf_down", 16384, 4096, 14336, 0},
  };
  const size_t maxA = (size_t)16384 * 14336, maxB = (size_t)28672 * 4096, maxC = (size_t)16384 * 28672;
  bf16 *A, *B, *C, *Z, *Zo, *bias;
  float *dbias, *ref, *tws;
  int* tcnt;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&B, maxB * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&Z, maxC * 2));
  CK(hipMalloc(&Zo, maxC * 2));
  // every per-column buffer sized for the widest shape (N = 28672: the prefill gate/up)
  constexpr int MAXN = 28672;
  for (const Shape& s : shapes)
    if (s.N > MAXN) { fprintf(stderr, "shape %s: N > MAXN\n", s.name); return 1; }
  CK(hipMalloc(&bias, MAXN * 2));
  CK(hipMalloc(&dbias, MAXN * 4));
  const int RR = 64;  // reference rows
  CK(hipMalloc(&ref, (size_t)RR * MAXN * 4));
  CK(hipMalloc(&tws, (size_t)256 * 4 * 256 * 320 * 4));
  CK(hipMalloc(&tcnt, 4096 * 4));
  CK(hipMemset(tcnt, 0, 4096 * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, A, maxA, 1u, 1.0f);
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, B, maxB, 2u, 1.0f);
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, Z, maxC, 3u, 2.0f);
  hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, 0, bias, (size_t)MAXN, 4u, 1.0f);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  for (const Shape& s : shapes) {
    if (*filter && !strstr(s.name, filter)) continue;
    const int bm = 256, bn0 = (s.N % 320 == 0) ? 320 : 256;
    auto launch = [&](int algo) {
      const int bn = bn0;
      const int tiles = (s.M / bm) * (s.N / bn);
      int tfull = tiles, tS = 1;
      if (s.K >= 4096) caamd::gemm_tail_plan(tiles, s.K, algo % 10 == 9 ? 64 : 32, cus, 4, &tfull, &tS);
      return caamd::gemm_launch(0, s.epi, bm, bn, A, B, C, s.epi == 4 ? nullptr : bias, s.epi == 4 ? Z : nullptr,
                                s.epi == 3 ? Zo : nullptr, s.epi == 4 ? dbias : nullptr, s.M, s.N, s.K, s.K, s.K,
                                s.N, 1, algo, 0, tfull, tS, tws, tcnt, 0);
    };
    // ---- numerics: first RR rows and a block of rows in the last tile row
    for (int algo : algos) {
      if ((algo / 10) % 100) continue;  // timing ablations compute garbage by design
      CK(hipMemset(dbias, 0, MAXN * 4));
      CK(hipMemset(C, 0, (size_t)s.M * s.N * 2));
      CK(launch(algo));
      CK(hipDeviceSynchronize());
      double max_err = 0, max_ref = 0;
      for (int blk = 0; blk < 2; ++blk) {
        const int r0 = blk == 0 ? 0 : s.M - 200;
        hipLaunchKernelGGL(ref_kernel, dim3((s.N + 255) / 256, RR), dim3(256), 0, 0, A, B,
                           s.epi == 4 ? nullptr : bias, ref, r0, RR, s.N, s.K);
        CK(hipDeviceSynchronize());
        std::vector<float> hr((size_t)RR * s.N);
        std::vector<bf16> hc((size_t)RR * s.N), hz((size_t)RR * s.N);
        CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hc.data(), C + (size_t)r0 * s.N, hc.size() * 2, hipMemcpyDeviceToHost));
        if (s.epi == 4) CK(hipMemcpy(hz.data(), Z + (size_t)r0 * s.N, hz.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < hr.size(); ++i) {
          double r = hr[i];
          if (s.epi == 3) r = gelu_ref(r);
          if (s.epi == 4) r = r * gelu_grad_ref(bf2f(hz[i]));
          max_ref = std::max(max_ref, fabs(r));
          max_err = std::max(max_err, fabs(r - bf2f(hc[i])));
        }
      }
      printf("{\"check\": \"%s\", \"algo\": %d, \"rel_err\": %.3e}\n", s.name, algo, max_err / max_ref);
      fflush(stdout);
      if (!(max_err / max_ref < 2e-2)) {
        printf("NUMERICS FAILED\n");
        return 2;
      }
    }
    // ---- timing: rounds x (every algo: iters launches), interleaved
    std::vector<int> run;
    for (int algo : algos) run.push_back(algo);
    std::vector<std::vector<float>> ts(run.size());
    for (int algo : run) CK(launch(algo));
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r) {
      for (size_t a = 0; a < run.size(); ++a) {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) CK(launch(run[a]));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts[a].push_back(ms * 1000.f / iters);
      }
    }
    const double fl = 2.0 * s.M * s.N * s.K;
    for (size_t a = 0; a < run.size(); ++a) {
      std::vector<float> v = ts[a];
      std::sort(v.begin(), v.end());
      const float med = v[v.size() / 2], mn = v[0];
      printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"epi\": %d, \"algo\": %d, \"us_med\": %.1f, "
             "\"us_min\": %.1f, \"pfs_med\": %.3f}\n",
             s.name, s.M, s.N, s.K, s.epi, run[a], med, mn, fl / med / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
