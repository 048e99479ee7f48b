// Per-step trainer glue around the rasterizer, one launch each, gfx950:
//
//   update_state   DefaultStrategy._update_state for packed=False
//                  (gsplat/strategy/default.py:213-262): grad2d += |scaled
//                  means2d.grad| and count += 1 where radii > 0, summed over
//                  cameras in camera order -- without torch.where's host sync
//                  and the six elementwise launches of the torch version.
//   activate_fwd   scales = exp(log_scales), opacities = sigmoid(logits)
//   activate_bwd   their VJPs with torch's formulas (exp: g * out;
//                  sigmoid_backward: g * (1 - out) * out), as the trainer's
//                  torch.exp / torch.sigmoid (examples/simple_trainer.py:565-566).
// All HBM-bound streaming kernels, one lane per Gaussian.
#include "common.h"
#include "../../include/gsplat_hip.h"

namespace gs {
namespace strat {

__global__ void __launch_bounds__(256)
update_state_kernel(int C, int64_t N, const float *__restrict__ g2d,
                    const int32_t *__restrict__ radii, float sx, float sy,
                    float *__restrict__ grad2d, float *__restrict__ count) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= N) return;
  float acc = grad2d[g], cnt = count[g];
  bool any = false;
  for (int c = 0; c < C; ++c) {
    const int64_t i = (int64_t)c * N + g;
    if (radii[i] > 0) {
      const float2 v = *reinterpret_cast<const float2 *>(g2d + 2 * i);
      const float x = v.x * sx, y = v.y * sy;
      acc += sqrtf(x * x + y * y);  // .norm(dim=-1) of a 2-vector
      cnt += 1.f;
      any = true;
    }
  }
  if (any) {
    grad2d[g] = acc;
    count[g] = cnt;
  }
}

__global__ void __launch_bounds__(256)
activate_fwd_kernel(int64_t n_s, int64_t n_o, const float *__restrict__ log_scales,
                    const float *__restrict__ logits, float *__restrict__ scales,
                    float *__restrict__ opacities) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n_s) scales[i] = expf(log_scales[i]);
  if (i < n_o) opacities[i] = 1.f / (1.f + expf(-logits[i]));
}

__global__ void __launch_bounds__(256)
activate_bwd_kernel(int64_t n_s, int64_t n_o, const float *__restrict__ scales,
                    const float *__restrict__ opacities, const float *__restrict__ v_scales,
                    const float *__restrict__ v_opacities, float *__restrict__ v_log_scales,
                    float *__restrict__ v_logits) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n_s) v_log_scales[i] = v_scales[i] * scales[i];
  if (i < n_o) {
    const float o = opacities[i];
    v_logits[i] = v_opacities[i] * (1.f - o) * o;
  }
}

}  // namespace strat
}  // namespace gs

using namespace gs;

extern "C" int gsplat_hip_update_state(int C, int64_t N, const float *means2d_grad,
                                       const int32_t *radii, float scale_x, float scale_y,
                                       float *grad2d, float *count, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "update_state: bad sizes C=%d N=%lld", C, (long long)N);
  if (N == 0 || C == 0) return 0;
  hipLaunchKernelGGL(strat::update_state_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, C, N, means2d_grad, radii, scale_x, scale_y, grad2d,
                     count);
  GS_CHECK_LAUNCH("update_state");
  return 0;
}

extern "C" int gsplat_hip_activate_fwd(int64_t n_scales, int64_t n_opacities,
                                       const float *log_scales, const float *logits,
                                       float *scales, float *opacities, void *stream) {
  const int64_t n = n_scales > n_opacities ? n_scales : n_opacities;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(strat::activate_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n_scales, n_opacities, log_scales, logits, scales,
                     opacities);
  GS_CHECK_LAUNCH("activate_fwd");
  return 0;
}

extern "C" int gsplat_hip_activate_bwd(int64_t n_scales, int64_t n_opacities, const float *scales,
                                       const float *opacities, const float *v_scales,
                                       const float *v_opacities, float *v_log_scales,
                                       float *v_logits, void *stream) {
  const int64_t n = n_scales > n_opacities ? n_scales : n_opacities;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(strat::activate_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n_scales, n_opacities, scales, opacities, v_scales,
                     v_opacities, v_log_scales, v_logits);
  GS_CHECK_LAUNCH("activate_bwd");
  return 0;
}
