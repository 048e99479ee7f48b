// Multi-tensor Adam for the Gaussian parameter groups, one launch, gfx950.
//
// The reference trainer steps six torch.optim.Adam instances, one per
// parameter group (examples/simple_trainer.py:235-277).  This kernel applies
// the identical update (torch.optim.Adam, amsgrad=False, weight_decay=0,
// bias-corrected, exp_avg via lerp) to every group in one grid-stride launch:
// HBM-bound, 28 B per element (p, g, m, v read; p, m, v written).
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
  int64_t begin[kMaxGroups + 1];  // prefix offsets over the flattened groups
  float step_size[kMaxGroups];    // lr / (1 - beta1^t)
  float inv_bc2_sqrt[kMaxGroups]; // 1 / sqrt(1 - beta2^t)
  int n;
};

__global__ void __launch_bounds__(256)
step_kernel(Groups g, float beta1, float beta2, float eps) {
  const int64_t total = g.begin[g.n];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int grp = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    while (i >= g.begin[grp + 1]) ++grp;
    const int64_t k = i - g.begin[grp];
    const float gr = g.grad[grp] ? g.grad[grp][k] : 0.f;
    float m = g.m[grp][k], v = g.v[grp][k];
    m = m + (1.f - beta1) * (gr - m);  // lerp(m, g, 1 - beta1)
    v = beta2 * v + (1.f - beta2) * gr * gr;
    const float denom = sqrtf(v) * g.inv_bc2_sqrt[grp] + eps;
    g.param[grp][k] -= g.step_size[grp] * m / denom;
    g.m[grp][k] = m;
    g.v[grp][k] = v;
  }
}

}  // namespace adam
}  // namespace gs

using namespace gs;

// One Adam step over n_groups parameter groups.  Arrays are host arrays of
// length n_groups; grads[i] may be NULL (treated as zero, as for a parameter
// that received no gradient but is still stepped).  `step` is the 1-based step.
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
    g.param[i] = params[i];
    g.grad[i] = grads[i];
    g.m[i] = exp_avgs[i];
    g.v[i] = exp_avg_sqs[i];
    g.begin[i + 1] = g.begin[i] + numels[i];
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
