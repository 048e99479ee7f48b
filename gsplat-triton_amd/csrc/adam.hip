// Multi-tensor Adam for the Gaussian parameter groups, one launch, gfx950.
//
// The reference trainer steps six torch.optim.Adam instances, one per
// parameter group (examples/simple_trainer.py:235-277).  This kernel applies
// the identical update (torch.optim.Adam, amsgrad=False, weight_decay=0,
// bias-corrected, exp_avg via lerp) to every group in one grid-stride launch.
// HBM-bound: 28 B per element (p, g, m, v read; p, m, v written), moved as
// 16-B vectors (4 elements per lane-iteration, scalar tail per group).
#include "common.h"
#include "../../include/gsplat_hip.h"

namespace gs {
namespace adam {

constexpr int kMaxGroups = 8;

struct Groups {
  float *param[kMaxGroups];
  const float *grad[kMaxGroups];
  float *m[kMaxGroups];
  float *v[kMaxGroups];
  int64_t numel[kMaxGroups];
  int64_t begin[kMaxGroups + 1];  // prefix offsets in 4-element slots
  float step_size[kMaxGroups];    // lr / (1 - beta1^t)
  float inv_bc2_sqrt[kMaxGroups]; // 1 / sqrt(1 - beta2^t)
  int n;
};

GS_INLINE void upd(float &p, float gr, float &m, float &v, float b1, float b2, float eps,
                   float ss, float ib) {
  m = m + (1.f - b1) * (gr - m);  // lerp(m, g, 1 - beta1)
  v = b2 * v + (1.f - b2) * gr * gr;
  p -= ss * m / (sqrtf(v) * ib + eps);
}

__global__ void __launch_bounds__(256)
step_kernel(Groups g, float beta1, float beta2, float eps) {
  const int64_t total = g.begin[g.n];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int grp = 0;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total; s += stride) {
    while (s >= g.begin[grp + 1]) ++grp;
    const int64_t k0 = 4 * (s - g.begin[grp]);
    const float ss = g.step_size[grp], ib = g.inv_bc2_sqrt[grp];
    float *P = g.param[grp];
    const float *G = g.grad[grp];
    float *M = g.m[grp], *V = g.v[grp];
    if (k0 + 4 <= g.numel[grp]) {
      float4 p = *reinterpret_cast<float4 *>(P + k0);
      const float4 gr = G ? *reinterpret_cast<const float4 *>(G + k0) : make_float4(0, 0, 0, 0);
      float4 m = *reinterpret_cast<float4 *>(M + k0);
      float4 v = *reinterpret_cast<float4 *>(V + k0);
      upd(p.x, gr.x, m.x, v.x, beta1, beta2, eps, ss, ib);
      upd(p.y, gr.y, m.y, v.y, beta1, beta2, eps, ss, ib);
      upd(p.z, gr.z, m.z, v.z, beta1, beta2, eps, ss, ib);
      upd(p.w, gr.w, m.w, v.w, beta1, beta2, eps, ss, ib);
      *reinterpret_cast<float4 *>(P + k0) = p;
      *reinterpret_cast<float4 *>(M + k0) = m;
      *reinterpret_cast<float4 *>(V + k0) = v;
    } else {
      for (int64_t k = k0; k < g.numel[grp]; ++k) {
        float p = P[k], m = M[k], v = V[k];
        upd(p, G ? G[k] : 0.f, m, v, beta1, beta2, eps, ss, ib);
        P[k] = p;
        M[k] = m;
        V[k] = v;
      }
    }
  }
}

}  // namespace adam
}  // namespace gs

using namespace gs;

// One Adam step over n_groups parameter groups.  Arrays are host arrays of
// length n_groups; grads[i] may be NULL (treated as zero).  Every pointer must
// be 16-B aligned.  `step` is the 1-based step count.
extern "C" int gsplat_hip_adam_step(int n_groups, float *const *params, const float *const *grads,
                                    float *const *exp_avgs, float *const *exp_avg_sqs,
                                    const int64_t *numels, const float *lrs, float beta1,
                                    float beta2, float eps, int step, void *stream) {
  GS_REQUIRE(n_groups > 0 && n_groups <= adam::kMaxGroups, "adam: 1..%d groups supported",
             adam::kMaxGroups);
  GS_REQUIRE(step >= 1, "adam: step must be >= 1");
  adam::Groups g{};
  g.n = n_groups;
  g.begin[0] = 0;
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  for (int i = 0; i < n_groups; ++i) {
    const uintptr_t al = (uintptr_t)params[i] | (uintptr_t)grads[i] | (uintptr_t)exp_avgs[i] |
                         (uintptr_t)exp_avg_sqs[i];
    GS_REQUIRE((al & 15) == 0, "adam: group %d pointers must be 16-B aligned", i);
    g.param[i] = params[i];
    g.grad[i] = grads[i];
    g.m[i] = exp_avgs[i];
    g.v[i] = exp_avg_sqs[i];
    g.numel[i] = numels[i];
    g.begin[i + 1] = g.begin[i] + (numels[i] + 3) / 4;
    g.step_size[i] = (float)(lrs[i] / bc1);
    g.inv_bc2_sqrt[i] = (float)(1.0 / sqrt(bc2));
  }
  for (int i = n_groups; i < adam::kMaxGroups; ++i) g.begin[i + 1] = g.begin[n_groups];
  const int64_t total = g.begin[n_groups];
  if (total == 0) return 0;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(adam::step_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, g, beta1,
                     beta2, eps);
  GS_CHECK_LAUNCH("adam_step");
  return 0;
}
