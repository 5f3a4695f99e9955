// RL return estimators on the GPU, time-major [T, B] layout so that the
// reverse-time scan is coalesced across the B trajectories (one lane each).
//   GAE (PPO):  delta_t = r_t + g * v_{t+1} * nt_t - v_t
//               A_t     = delta_t + g * lam * nt_t * A_{t+1};  target_t = A_t + v_t
//   V-trace (IMPALA/APPO), Espeholt et al. 2018:
//               rho_t = min(rho_bar, exp(log_rho_t)), c_t = min(1, exp(log_rho_t))
//               vs_t - v_t = rho_t*(r_t + d_t v_{t+1} - v_t) + d_t c_t (vs_{t+1} - v_{t+1})
//               pg_adv_t  = min(pg_rho_bar, exp(log_rho_t)) * (r_t + d_t vs_{t+1} - v_t)
// Reference semantics: rllib/evaluation/postprocessing.py:86 (compute_advantages),
// rllib/algorithms/impala/vtrace_torch.py:252 (from_importance_weights).
#include "common.h"

namespace caamd {

__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ r,
                                                  const float* __restrict__ v,  // [T+1, B]
                                                  const float* __restrict__ nonterm,
                                                  float* __restrict__ adv,
                                                  float* __restrict__ tgt, int T, int B,
                                                  float gamma, float lam) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float a = 0.f;
  float vnext = v[(size_t)T * B + b];
  for (int t = T - 1; t >= 0; --t) {
    const size_t i = (size_t)t * B + b;
    const float vt = v[i], nt = nonterm[i];
    const float delta = r[i] + gamma * vnext * nt - vt;
    a = delta + gamma * lam * nt * a;
    adv[i] = a;
    tgt[i] = a + vt;
    vnext = vt;
  }
}

__global__ __launch_bounds__(256) void vtrace_kernel(
    const float* __restrict__ log_rhos, const float* __restrict__ discounts,
    const float* __restrict__ rewards, const float* __restrict__ values,
    const float* __restrict__ bootstrap, float* __restrict__ vs, float* __restrict__ pg_adv, int T,
    int B, float clip_rho, float clip_pg_rho) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float acc = 0.f;                // vs_{t+1} - v_{t+1}
  float v_next = bootstrap[b];    // v_{t+1}
  float vs_next = bootstrap[b];   // vs_{t+1}
  for (int t = T - 1; t >= 0; --t) {
    const size_t i = (size_t)t * B + b;
    const float rho = __expf(log_rhos[i]);
    const float crho = clip_rho > 0.f ? fminf(clip_rho, rho) : rho;
    const float cs = fminf(1.f, rho);
    const float d = discounts[i], vt = values[i], rt = rewards[i];
    const float delta = crho * (rt + d * v_next - vt);
    acc = delta + d * cs * acc;
    const float vst = vt + acc;
    const float cpg = clip_pg_rho > 0.f ? fminf(clip_pg_rho, rho) : rho;
    pg_adv[i] = cpg * (rt + d * vs_next - vt);
    vs[i] = vst;
    v_next = vt;
    vs_next = vst;
  }
}

void gae_launch(const float* r, const float* v, const float* nt, float* adv, float* tgt, int T,
                int B, float gamma, float lam, hipStream_t st) {
  hipLaunchKernelGGL(gae_kernel, dim3((B + 255) / 256), dim3(256), 0, st, r, v, nt, adv, tgt, T, B,
                     gamma, lam);
}

void vtrace_launch(const float* lr, const float* d, const float* r, const float* v,
                   const float* boot, float* vs, float* pg, int T, int B, float clip_rho,
                   float clip_pg_rho, hipStream_t st) {
  hipLaunchKernelGGL(vtrace_kernel, dim3((B + 255) / 256), dim3(256), 0, st, lr, d, r, v, boot, vs,
                     pg, T, B, clip_rho, clip_pg_rho);
}

}  // namespace caamd
