// The geometry groups' Adam step inside a projection backward: the 3DGS one
// (projection.hip, ABI 31) and the 2DGS one (surfel.hip, ABI 33).
#pragma once

#include "common.h"

namespace gs {

// The geometry groups' Adam step fused into the backward (ABI 31,
// gsplat_hip_projection_bwd_adam; C == 1, non-packed): instead of storing
// v_means / v_quats / v_scales, every lane applies torch.optim.Adam to its
// Gaussian's rows of the four geometry parameters in place, with the
// gradients the trainer's FusedAdam would have formed (adam_step_ex modes):
// means  g = v_means + v_dirs          (the SH backward's part; autograd's sum)
// quats  g = v_quats
// log-scales  g = v_scales * exp(log_scales)   (exp's VJP, the activated scale)
// logits      g = v_opac * (1 - o) * o         (sigmoid's VJP, o = sigmoid(logits))
// -- the same arithmetic as activate_bwd_kernel / adam::xform, the same
// element update (common.h adam_update), so the result is bit-identical to
// projection backward + activation backward + FusedAdam (the gradient
// algebra above is the unfused kernel's own code: the fusion is a runtime
// branch of the epilogue).  88 B per Gaussian of gradients never reach HBM.
struct GeomAdam {
  float *p[4];  // means [N,3], log-scales [N,3], quats [N,4], logits [N] (the trainer's order)
  float *m[4], *v[4];
  const float *v_dirs;  // [N,3] or null
  const float *v_opac;  // [N] dL/d sigmoid(logits), or null
  const float *opac;    // [N] sigmoid(logits) of the forward
  float ss[4], ib;      // lr_i / (1 - beta1^t), 1 / sqrt(1 - beta2^t)
  const float *hyper;   // device [8]: (ss_i, ib) per group (captured step), or null
  const int32_t *skip;  // device flag: non-zero = void step (nothing updated), or null
  float b1, b2, eps;
};

// A lane's rows of the four groups (parameters, both moments) and the other
// gradient inputs, loaded at the kernel's start so that their latency
// overlaps the gradient algebra (the 2DGS projection backward's epilogue;
// the 3DGS one keeps its own copy of this code).
struct GeomRows {
  static constexpr int kG = 11;  // means 3 | log-scales 3 | quats 4 | logits 1
  float p[kG], m[kG], v[kG], vd[3], vo, op, sc[3];
};

GS_INLINE void geom_rows_load(const GeomAdam &ga, size_t i, const float *scales, GeomRows &r) {
  constexpr int off[4] = {0, 3, 6, 10}, wid[4] = {3, 3, 4, 1};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < wid[q]; ++e) {
      r.p[off[q] + e] = ga.p[q][wid[q] * i + e];
      r.m[off[q] + e] = ga.m[q][wid[q] * i + e];
      r.v[off[q] + e] = ga.v[q][wid[q] * i + e];
    }
#pragma unroll
  for (int j = 0; j < 3; ++j) r.vd[j] = ga.v_dirs ? ga.v_dirs[3 * i + j] : 0.f;
  r.vo = ga.v_opac ? ga.v_opac[i] : 0.f;
  r.op = ga.v_opac ? ga.opac[i] : 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) r.sc[j] = scales[3 * i + j];
}

// torch.optim.Adam on the lane's rows from the projection backward's
// gradients vm / vs / vq (each an already-rounded value: the caller keeps
// them apart with an asm barrier), the trainer's FusedAdam gradient algebra
// (adam_step_ex modes 1-3), written back in place.
GS_INLINE void geom_rows_update(const GeomAdam &ga, size_t i, GeomRows &r, const float (&vm)[3],
                                const float (&vs)[3], const float (&vq)[4]) {
  constexpr int kG = GeomRows::kG;
  float ss[4], ib;
  if (ga.hyper) {
#pragma unroll
    for (int q = 0; q < 4; ++q) ss[q] = ga.hyper[2 * q];
    ib = ga.hyper[1];
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) ss[q] = ga.ss[q];
    ib = ga.ib;
  }
  float g[kG];
#pragma unroll
  for (int j = 0; j < 3; ++j) g[j] = ga.v_dirs ? vm[j] + r.vd[j] : vm[j];
#pragma unroll
  for (int j = 0; j < 3; ++j) g[3 + j] = vs[j] * r.sc[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) g[6 + j] = vq[j];
  g[10] = ga.v_opac ? r.vo * (1.f - r.op) * r.op : 0.f;
  // each gradient its own rounded value (no VJP product contracted into
  // adam_update's arithmetic, as adam::step_kernel's runtime select keeps them)
#pragma unroll
  for (int e = 0; e < kG; ++e) asm volatile("" : "+v"(g[e]));
  constexpr int grp[kG] = {0, 0, 0, 1, 1, 1, 2, 2, 2, 2, 3};
#pragma unroll
  for (int e = 0; e < kG; ++e)
    adam_update(r.p[e], g[e], r.m[e], r.v[e], ga.b1, ga.b2, ga.eps, ss[grp[e]], ib);
  constexpr int off[4] = {0, 3, 6, 10}, wid[4] = {3, 3, 4, 1};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < wid[q]; ++e) {
      ga.p[q][wid[q] * i + e] = r.p[off[q] + e];
      ga.m[q][wid[q] * i + e] = r.m[off[q] + e];
      ga.v[q][wid[q] * i + e] = r.v[off[q] + e];
    }
}

// The host side of both entries: group arrays and factors into a GeomAdam
// (gsplat_hip_adam_step's host arithmetic for the factors); 0 or an error.
inline int geom_adam_setup(GeomAdam &ga, float *const *params, float *const *exp_avgs,
                           float *const *exp_avg_sqs, const float *lrs, float beta1, float beta2,
                           float eps, int step, const float *hyper_device,
                           const int32_t *skip_device, const float *v_dirs, const float *v_opac,
                           const float *opac, const char *who) {
  GS_REQUIRE(params && exp_avgs && exp_avg_sqs, "%s: null group arrays", who);
  GS_REQUIRE(hyper_device || (lrs && step >= 1), "%s: lrs and step >= 1, or hyper", who);
  GS_REQUIRE(!v_opac || opac, "%s: v_opac needs opac", who);
  ga = GeomAdam{};
  for (int k = 0; k < 4; ++k) {
    GS_REQUIRE(params[k] && exp_avgs[k] && exp_avg_sqs[k],
               "%s: null parameter / moment of group %d", who, k);
    ga.p[k] = params[k];
    ga.m[k] = exp_avgs[k];
    ga.v[k] = exp_avg_sqs[k];
  }
  ga.v_dirs = v_dirs;
  ga.v_opac = v_opac;
  ga.opac = opac;
  ga.hyper = hyper_device;
  ga.skip = skip_device;
  ga.b1 = beta1;
  ga.b2 = beta2;
  ga.eps = eps;
  if (!hyper_device) {
    const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
    for (int k = 0; k < 4; ++k) ga.ss[k] = (float)(lrs[k] / bc1);
    ga.ib = (float)(1.0 / sqrt(bc2));
  }
  return 0;
}

}  // namespace gs
