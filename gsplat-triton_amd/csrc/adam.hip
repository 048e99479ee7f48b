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

// Gradient transform per group (gsplat_hip_adam_step_ex): the update's
// gradient is formed in-register from what the backward left, replacing the
// separate VJP / accumulation launches.  Same arithmetic as those kernels.
enum GradMode : int {
  kGrad = 0,     // g
  kSum = 1,      // g + aux        (two gradient contributions, autograd's sum)
  kExpVjp = 2,   // g * aux        (exp: aux = exp(x), activate_bwd_kernel)
  kSigVjp = 3,   // g * (1 - aux) * aux   (sigmoid: aux = sigmoid(x))
};

struct Groups {
  float *param[kMaxGroups];
  const float *grad[kMaxGroups];
  const float *aux[kMaxGroups];  // second gradient or activation (modes 1-3)
  int mode[kMaxGroups];
  float *m[kMaxGroups];
  float *v[kMaxGroups];
  int64_t numel[kMaxGroups];
  int64_t begin[kMaxGroups + 1];  // prefix offsets in 4-element slots
  float step_size[kMaxGroups];    // lr / (1 - beta1^t)
  float inv_bc2_sqrt[kMaxGroups]; // 1 / sqrt(1 - beta2^t)
  // captured-step form (gsplat_hip_adam_step_dev): the two factors per group
  // read on the device ([2 i], [2 i + 1]), and a void step (*skip != 0)
  // updates nothing
  const float *hyper;
  const int32_t *skip;
  int n;
};

GS_INLINE void upd(float &p, float gr, float &m, float &v, float b1, float b2, float eps,
                   float ss, float ib) {
  adam_update(p, gr, m, v, b1, b2, eps, ss, ib);
}

GS_INLINE float xform(int mode, float g, float a) {
  if (mode == kSum) return g + a;
  if (mode == kExpVjp) return g * a;
  if (mode == kSigVjp) return g * (1.f - a) * a;
  return g;
}

typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
GS_INLINE float4 ld4(const float *p) {
  if (NT) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return *reinterpret_cast<const float4 *>(p);
}
template <bool NT>
GS_INLINE void st4(float *p, float4 v) {
  if (NT) __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v *>(p));
  else *reinterpret_cast<float4 *>(p) = v;
}

// U slots (4 elements each) per lane per iteration, loads of all U issued
// before any update; NT: non-temporal (streaming) loads and stores.
template <int U, bool NT>
__global__ void __launch_bounds__(256)
step_kernel(Groups g, float beta1, float beta2, float eps) {
  if (g.skip && *g.skip) return;
  const int64_t total = g.begin[g.n];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s0 < total;
       s0 += stride * U) {
    float4 p[U], gr[U], m[U], v[U], ax[U];
    int grp[U];
    int64_t k0[U];
    bool full[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t s = s0 + u * stride;
      int gi = 0;
      while (gi < g.n - 1 && s >= g.begin[gi + 1]) ++gi;
      grp[u] = gi;
      k0[u] = 4 * (s - g.begin[gi]);
      full[u] = s < total && k0[u] + 4 <= g.numel[gi];
      if (full[u]) {
        p[u] = ld4<NT>(g.param[gi] + k0[u]);
        gr[u] = g.grad[gi] ? ld4<NT>(g.grad[gi] + k0[u]) : make_float4(0, 0, 0, 0);
        ax[u] = g.aux[gi] ? ld4<NT>(g.aux[gi] + k0[u]) : make_float4(0, 0, 0, 0);
        m[u] = ld4<NT>(g.m[gi] + k0[u]);
        v[u] = ld4<NT>(g.v[gi] + k0[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int gi = grp[u];
      const float ss = g.hyper ? g.hyper[2 * gi] : g.step_size[gi];
      const float ib = g.hyper ? g.hyper[2 * gi + 1] : g.inv_bc2_sqrt[gi];
      if (full[u]) {
        const int md = g.mode[gi];
        upd(p[u].x, xform(md, gr[u].x, ax[u].x), m[u].x, v[u].x, beta1, beta2, eps, ss, ib);
        upd(p[u].y, xform(md, gr[u].y, ax[u].y), m[u].y, v[u].y, beta1, beta2, eps, ss, ib);
        upd(p[u].z, xform(md, gr[u].z, ax[u].z), m[u].z, v[u].z, beta1, beta2, eps, ss, ib);
        upd(p[u].w, xform(md, gr[u].w, ax[u].w), m[u].w, v[u].w, beta1, beta2, eps, ss, ib);
        st4<NT>(g.param[gi] + k0[u], p[u]);
        st4<NT>(g.m[gi] + k0[u], m[u]);
        st4<NT>(g.v[gi] + k0[u], v[u]);
      } else if (s0 + u * stride < total) {  // scalar tail of a group
        float *P = g.param[gi], *M = g.m[gi], *V = g.v[gi];
        const float *G = g.grad[gi], *A = g.aux[gi];
        const int md = g.mode[gi];
        for (int64_t k = k0[u]; k < g.numel[gi]; ++k) {
          float pp = P[k], mm = M[k], vv = V[k];
          upd(pp, xform(md, G ? G[k] : 0.f, A ? A[k] : 0.f), mm, vv, beta1, beta2, eps, ss, ib);
          P[k] = pp;
          M[k] = mm;
          V[k] = vv;
        }
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
static int adam_launch(int n_groups, float *const *params, const float *const *grads,
                       const float *const *aux, const int32_t *modes, float *const *exp_avgs,
                       float *const *exp_avg_sqs, const int64_t *numels, const float *lrs,
                       float beta1, float beta2, float eps, int step, void *stream, const float *hyper = nullptr,
                       const int32_t *skip = nullptr) {
  GS_REQUIRE(n_groups > 0 && n_groups <= adam::kMaxGroups, "adam: 1..%d groups supported",
             adam::kMaxGroups);
  GS_REQUIRE(hyper || step >= 1, "adam: step must be >= 1");
  adam::Groups g{};
  g.n = n_groups;
  g.hyper = hyper;
  g.skip = skip;
  g.begin[0] = 0;
  const int t = step >= 1 ? step : 1;
  const double bc1 = 1.0 - pow((double)beta1, t), bc2 = 1.0 - pow((double)beta2, t);
  for (int i = 0; i < n_groups; ++i) {
    const uintptr_t al = (uintptr_t)params[i] | (uintptr_t)grads[i] | (uintptr_t)exp_avgs[i] |
                         (uintptr_t)exp_avg_sqs[i];
    GS_REQUIRE((al & 15) == 0, "adam: group %d pointers must be 16-B aligned", i);
    g.param[i] = params[i];
    g.grad[i] = grads[i];
    g.aux[i] = aux ? aux[i] : nullptr;
    g.mode[i] = modes ? modes[i] : 0;
    GS_REQUIRE(g.mode[i] >= 0 && g.mode[i] <= 3, "adam: group %d mode %d not in [0, 3]", i,
               g.mode[i]);
    GS_REQUIRE(g.mode[i] == 0 || g.aux[i] != nullptr, "adam: group %d mode %d needs aux", i,
               g.mode[i]);
    GS_REQUIRE(((uintptr_t)g.aux[i] & 15) == 0, "adam: group %d aux must be 16-B aligned", i);
    g.m[i] = exp_avgs[i];
    g.v[i] = exp_avg_sqs[i];
    g.numel[i] = numels[i];
    g.begin[i + 1] = g.begin[i] + (numels[i] + 3) / 4;
    g.step_size[i] = hyper ? 0.f : (float)(lrs[i] / bc1);
    g.inv_bc2_sqrt[i] = hyper ? 0.f : (float)(1.0 / sqrt(bc2));
  }
  for (int i = n_groups; i < adam::kMaxGroups; ++i) g.begin[i + 1] = g.begin[n_groups];
  const int64_t total = g.begin[n_groups];
  if (total == 0) return 0;
  // one 16-B slot per lane per iteration; deeper unrolling and non-temporal
  // accesses measured no faster (tools/adam_bench.py: ~5.8 TB/s; inside the
  // M2 step non-temporal ran 776.4 / 785.0 / 804.3 against 803.8 x 3
  // images/s, profiles/r4_batch12/ -- unlike the SH Adam's rows)
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 64);
  hipLaunchKernelGGL((adam::step_kernel<1, false>), dim3(blocks), dim3(256), 0,
                     (hipStream_t)stream, g, beta1, beta2, eps);
  GS_CHECK_LAUNCH("adam_step");
  return 0;
}

extern "C" int gsplat_hip_adam_step(int n_groups, float *const *params, const float *const *grads,
                                    float *const *exp_avgs, float *const *exp_avg_sqs,
                                    const int64_t *numels, const float *lrs, float beta1,
                                    float beta2, float eps, int step, void *stream) {
  return adam_launch(n_groups, params, grads, nullptr, nullptr, exp_avgs, exp_avg_sqs, numels, lrs,
                     beta1, beta2, eps, step, stream);
}

extern "C" int gsplat_hip_adam_step_ex(int n_groups, float *const *params,
                                       const float *const *grads, const float *const *aux,
                                       const int32_t *modes, float *const *exp_avgs,
                                       float *const *exp_avg_sqs, const int64_t *numels,
                                       const float *lrs, float beta1, float beta2, float eps,
                                       int step, void *stream) {
  return adam_launch(n_groups, params, grads, aux, modes, exp_avgs, exp_avg_sqs, numels, lrs,
                     beta1, beta2, eps, step, stream);
}

// The gsplat_hip_adam_step_ex update with the step-dependent factors read on
// the device (ABI 20, a captured training step): hyper_device[2 i] =
// lr_i / (1 - beta1^t), hyper_device[2 i + 1] = 1 / sqrt(1 - beta2^t), which
// the host computes as gsplat_hip_adam_step does; skip_device (may be NULL)
// non-zero: nothing is updated (a void step).
extern "C" int gsplat_hip_adam_step_dev(int n_groups, float *const *params,
                                        const float *const *grads, const float *const *aux,
                                        const int32_t *modes, float *const *exp_avgs,
                                        float *const *exp_avg_sqs, const int64_t *numels,
                                        const float *hyper_device, float beta1, float beta2,
                                        float eps, const int32_t *skip_device, void *stream) {
  GS_REQUIRE(hyper_device != nullptr, "adam_step_dev: null hyper_device");
  return adam_launch(n_groups, params, grads, aux, modes, exp_avgs, exp_avg_sqs, numels, nullptr,
                     beta1, beta2, eps, 0, stream, hyper_device, skip_device);
}
