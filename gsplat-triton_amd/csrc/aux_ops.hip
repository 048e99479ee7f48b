// Auxiliary per-Gaussian kernels that the reference's strategies and
// optimizers reach through its CUDA extension even on the Triton backend
// (SURVEY L15, §8 f4), for gfx950:
//
//   quat_scale_to_covar_preci_{fwd,bwd}  gsplat/cuda/csrc/QuatScaleToCovarCUDA.cu
//       (+ quat_scale_to_covar_vjp / quat_scale_to_preci_vjp,
//        gsplat/cuda/include/Utils.cuh:224-303) -- MCMCStrategy's position noise
//        (gsplat/strategy/ops.py:352)
//   relocation                           gsplat/cuda/csrc/RelocationCUDA.cu:10-44
//       -- MCMCStrategy relocate / sample_add (gsplat/strategy/ops.py:272,314)
//   selective adam                       gsplat/cuda/csrc/AdamCUDA.cu:12-46
//       -- SelectiveAdam (gsplat/optimizers/selective_adam.py)
//
// One lane per Gaussian (per element for Adam); HBM-bound streaming kernels.
#include "common.h"
#include "../../include/gsplat_hip.h"

namespace gs {
namespace auxk {

// ---------------------------------------------------- covariance / precision
// Row-major R S^2 R^T (covar) and R S^-2 R^T (preci); triu = [xx, xy, xz, yy, yz, zz].
__global__ void __launch_bounds__(256)
covar_preci_fwd_kernel(int64_t N, const float *__restrict__ quats,
                       const float *__restrict__ scales, int triu, float *__restrict__ covars,
                       float *__restrict__ precis) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float4 q = *reinterpret_cast<const float4 *>(quats + 4 * n);
  const M3 R = quat_to_rotmat(q.x, q.y, q.z, q.w);
  const float s[3] = {scales[3 * n], scales[3 * n + 1], scales[3 * n + 2]};
  for (int which = 0; which < 2; ++which) {
    float *out = which ? precis : covars;
    if (!out) continue;
    float w[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) w[k] = which ? 1.f / (s[k] * s[k]) : s[k] * s[k];
    float c[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        c[i][j] = R.m[i][0] * w[0] * R.m[j][0] + R.m[i][1] * w[1] * R.m[j][1] +
                  R.m[i][2] * w[2] * R.m[j][2];
    if (triu) {
      float *o = out + 6 * n;
      o[0] = c[0][0]; o[1] = c[0][1]; o[2] = c[0][2];
      o[3] = c[1][1]; o[4] = c[1][2]; o[5] = c[2][2];
    } else {
      float *o = out + 9 * n;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) o[3 * i + j] = c[i][j];
    }
  }
}

// d/d(q, s) of C = (R S)(R S)^T with S = diag(s) (covar) or diag(1/s) (preci):
// v_M = (G + G^T) M, v_R = v_M S, v_s_k from v_M (Utils.cuh:224-303).
GS_INLINE void sym_vjp(const M3 &R, const float sk[3], bool inv, const float G[3][3], float4 q,
                       float vq[4], float vs[3]) {
  float S[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) S[k] = inv ? 1.f / sk[k] : sk[k];
  float vM[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) a += (G[i][k] + G[k][i]) * R.m[k][j] * S[j];
      vM[i][j] = a;
    }
  M3 vR;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) vR.m[i][j] = vM[i][j] * S[j];
  float dq[4];
  quat_to_rotmat_vjp(q.x, q.y, q.z, q.w, vR, dq);
#pragma unroll
  for (int k = 0; k < 4; ++k) vq[k] += dq[k];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float d = R.m[0][j] * vM[0][j] + R.m[1][j] * vM[1][j] + R.m[2][j] * vM[2][j];
    vs[j] += inv ? -S[j] * S[j] * d : d;
  }
}

__global__ void __launch_bounds__(256)
covar_preci_bwd_kernel(int64_t N, const float *__restrict__ quats,
                       const float *__restrict__ scales, int triu,
                       const float *__restrict__ v_covars, const float *__restrict__ v_precis,
                       float *__restrict__ v_quats, float *__restrict__ v_scales) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float4 q = *reinterpret_cast<const float4 *>(quats + 4 * n);
  const M3 R = quat_to_rotmat(q.x, q.y, q.z, q.w);
  const float s[3] = {scales[3 * n], scales[3 * n + 1], scales[3 * n + 2]};
  float vq[4] = {0.f, 0.f, 0.f, 0.f}, vs[3] = {0.f, 0.f, 0.f};
  for (int which = 0; which < 2; ++which) {
    const float *g = which ? v_precis : v_covars;
    if (!g) continue;
    float G[3][3];
    if (triu) {  // off-diagonal gradients split over the symmetric pair
      const float *t = g + 6 * n;
      G[0][0] = t[0]; G[1][1] = t[3]; G[2][2] = t[5];
      G[0][1] = G[1][0] = 0.5f * t[1];
      G[0][2] = G[2][0] = 0.5f * t[2];
      G[1][2] = G[2][1] = 0.5f * t[4];
    } else {
      const float *t = g + 9 * n;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) G[i][j] = t[3 * i + j];
    }
    sym_vjp(R, s, which == 1, G, q, vq, vs);
  }
  *reinterpret_cast<float4 *>(v_quats + 4 * n) = make_float4(vq[0], vq[1], vq[2], vq[3]);
  v_scales[3 * n] = vs[0];
  v_scales[3 * n + 1] = vs[1];
  v_scales[3 * n + 2] = vs[2];
}

// ------------------------------------------------------------- relocation
// MCMC relocation (RelocationCUDA.cu:10-44): o' = 1 - (1 - o)^(1/n),
// s' = s * o / sum_{i=1..n} sum_{k<i} C(i-1, k) (-1)^k o'^(k+1) / sqrt(k+1).
__global__ void __launch_bounds__(256)
relocation_kernel(int64_t N, const float *__restrict__ opacities, const float *__restrict__ scales,
                  const int32_t *__restrict__ ratios, const float *__restrict__ binoms, int n_max,
                  float *__restrict__ new_opacities, float *__restrict__ new_scales) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int r = ratios[n];
  const float o = opacities[n];
  const float no = 1.f - powf(1.f - o, 1.f / (float)r);
  float denom = 0.f;
  for (int i = 1; i <= r; ++i) {
    float pk = no;  // no^(k+1)
    for (int k = 0; k <= i - 1; ++k) {
      const float term = ((k & 1) ? -1.f : 1.f) / sqrtf((float)(k + 1)) * pk;
      denom += binoms[(i - 1) * n_max + k] * term;
      pk *= no;
    }
  }
  new_opacities[n] = no;
  const float coeff = o / denom;
#pragma unroll
  for (int k = 0; k < 3; ++k) new_scales[3 * n + k] = coeff * scales[3 * n + k];
}

// ------------------------------------------------------- MCMC position noise
// inject_noise_to_position (gsplat/strategy/ops.py:343-369) in one pass:
// the reference's covariance launch, its activation / op_sigmoid passes, the
// einsum and the add become 68 B per Gaussian (means read + written, quats,
// log-scales, logit and the normal draw read; 56 B with the draw made here).
// Sigma w = R (s^2 * (R^T w)).
//
// The draw: z[n] when given (torch's randn_like, the reference's), else three
// standard normals of Philox-4x32-10 keyed by the seed, counter (n, step):
// a pure function of (seed, step, n), so a replayed or re-run step draws the
// same numbers (the captured training step reads step and scaler from its
// input block, and skips a void step).
struct Philox {
  static GS_INLINE void round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
    const uint32_t m0 = 0xD2511F53u, m1 = 0xCD9E8D57u;
    const uint32_t h0 = __umulhi(m0, c[0]), l0 = m0 * c[0];
    const uint32_t h1 = __umulhi(m1, c[2]), l1 = m1 * c[2];
    const uint32_t r0 = h1 ^ c[1] ^ k0, r2 = h0 ^ c[3] ^ k1;
    c[0] = r0, c[1] = l1, c[2] = r2, c[3] = l0;
  }
  static GS_INLINE void draw(uint32_t (&c)[4], uint64_t key) {
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      round(c, k0, k1);
      k0 += 0x9E3779B9u, k1 += 0xBB67AE85u;
    }
  }
};

// uniform in (0, 1]: 24 random bits, never 0 (the Box-Muller log)
GS_INLINE float u01(uint32_t x) { return ((float)(x >> 8) + 1.f) * (1.f / 16777216.f); }

__global__ void __launch_bounds__(256)
mcmc_noise_kernel(int64_t N, float *__restrict__ means, const float *__restrict__ quats,
                  const float *__restrict__ log_scales, const float *__restrict__ logits,
                  const float *__restrict__ z, uint64_t seed, int64_t step,
                  const int64_t *__restrict__ step_dev, float scaler,
                  const float *__restrict__ scaler_dev, const int32_t *__restrict__ skip) {
  if (skip && *skip) return;  // a void step of the captured training step
  if (scaler_dev) scaler = *scaler_dev;
  if (scaler == 0.f) return;  // nothing moves (a refine step: noise after the refine)
  if (step_dev) step = *step_dev;
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float zn[3];
  if (z) {
#pragma unroll
    for (int k = 0; k < 3; ++k) zn[k] = z[3 * n + k];
  } else {
    uint32_t c[4] = {(uint32_t)n, (uint32_t)((uint64_t)n >> 32), (uint32_t)step,
                     (uint32_t)((uint64_t)step >> 32)};
    Philox::draw(c, seed);
    // Box-Muller: (c0, c1) -> two normals, (c2, c3) -> the third
    const float r0 = sqrtf(-2.f * logf(u01(c[0]))), t0 = 6.2831853071795864f * u01(c[1]);
    const float r1 = sqrtf(-2.f * logf(u01(c[2]))), t1 = 6.2831853071795864f * u01(c[3]);
    float sn, cs;
    sincosf(t0, &sn, &cs);
    zn[0] = r0 * cs;
    zn[1] = r0 * sn;
    zn[2] = r1 * cosf(t1);
  }
  const float4 q = *reinterpret_cast<const float4 *>(quats + 4 * n);
  const M3 R = quat_to_rotmat(q.x, q.y, q.z, q.w);
  const float o = 1.f / (1.f + expf(-logits[n]));
  // op_sigmoid(1 - o), k = 100, x0 = 0.995 (ops.py:360-361)
  const float f = scaler / (1.f + expf(-100.f * ((1.f - o) - 0.995f)));
  const float w[3] = {zn[0] * f, zn[1] * f, zn[2] * f};
  float u[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float s = expf(log_scales[3 * n + k]);
    u[k] = s * s * (R.m[0][k] * w[0] + R.m[1][k] * w[1] + R.m[2][k] * w[2]);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
    means[3 * n + i] += R.m[i][0] * u[0] + R.m[i][1] * u[1] + R.m[i][2] * u[2];
}

// -------------------------------------------------------- selective adam
// The reference's fused Adam (AdamCUDA.cu:12-46): no bias correction,
// m = b1 m + (1-b1) g, v = b2 v + (1-b2) g^2, p -= lr m / (sqrt(v) + eps);
// rows whose visibility is false are untouched.  A row is the `row`
// consecutive elements of one Gaussian.
__global__ void __launch_bounds__(256)
selective_adam_kernel(int64_t n_rows, int64_t row, float *__restrict__ param,
                      const float *__restrict__ grad, float *__restrict__ exp_avg,
                      float *__restrict__ exp_avg_sq, const uint8_t *__restrict__ visible,
                      float lr, float b1, float b2, float eps) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_rows * row) return;
  if (visible && !visible[e / row]) return;
  const float g = grad[e];
  const float m = b1 * exp_avg[e] + (1.f - b1) * g;
  const float v = b2 * exp_avg_sq[e] + (1.f - b2) * g * g;
  param[e] += -lr * m / (sqrtf(v) + eps);
  exp_avg[e] = m;
  exp_avg_sq[e] = v;
}


// Normals from depth maps by central differences (gsplat/utils.py:137-224,
// depth_to_normal): back-project the 4-neighbourhood of each pixel,
// n = normalize((p[y+1,x] - p[y-1,x]) x (p[y,x+1] - p[y,x-1])), zero on the
// one-pixel border.  One lane per pixel; the torch formula is a dozen
// full-image passes.
__device__ __forceinline__ void d2n_point(const float *dep, int64_t ps, const float *c2w,
                                          const float *K, int W, int x, int y, int z_depth,
                                          float p[3]) {
  const float dx = ((float)x - K[2] + 0.5f) / K[0], dy = ((float)y - K[5] + 0.5f) / K[4];
  float d[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) d[i] = c2w[4 * i] * dx + c2w[4 * i + 1] * dy + c2w[4 * i + 2];
  if (!z_depth) {
    const float n = fmaxf(sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]), 1e-12f);
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] /= n;
  }
  const float z = dep[((int64_t)y * W + x) * ps];
#pragma unroll
  for (int i = 0; i < 3; ++i) p[i] = c2w[4 * i + 3] + z * d[i];
}

__global__ void __launch_bounds__(256)
depth_to_normal_kernel(int C, int H, int W, const float *__restrict__ depths, int64_t ps,
                       const float *__restrict__ camtoworlds, const float *__restrict__ Ks,
                       int z_depth, float *__restrict__ normals) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t HW = (int64_t)H * W;
  if (i >= C * HW) return;
  const int c = (int)(i / HW);
  const int64_t r = i - c * HW;
  const int y = (int)(r / W), x = (int)(r - (int64_t)y * W);
  float *out = normals + 3 * i;
  if (x == 0 || y == 0 || x == W - 1 || y == H - 1) {
    out[0] = out[1] = out[2] = 0.f;
    return;
  }
  const float *dep = depths + c * HW * ps, *c2w = camtoworlds + 16 * c, *K = Ks + 9 * c;
  float pu[3], pd[3], pl[3], pr[3];
  d2n_point(dep, ps, c2w, K, W, x, y + 1, z_depth, pd);
  d2n_point(dep, ps, c2w, K, W, x, y - 1, z_depth, pu);
  d2n_point(dep, ps, c2w, K, W, x + 1, y, z_depth, pr);
  d2n_point(dep, ps, c2w, K, W, x - 1, y, z_depth, pl);
  const float a[3] = {pd[0] - pu[0], pd[1] - pu[1], pd[2] - pu[2]};
  const float b[3] = {pr[0] - pl[0], pr[1] - pl[1], pr[2] - pl[2]};
  const float n[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2],
                      a[0] * b[1] - a[1] * b[0]};
  const float l = fmaxf(sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]), 1e-12f);
  out[0] = n[0] / l;
  out[1] = n[1] / l;
  out[2] = n[2] / l;
}

// out[c, p, i] = sum_j c2w[c][i][j] v[c, p, j] (the rotation of the
// camera-to-world matrices), one lane per pixel.
__global__ void __launch_bounds__(256)
rotate3_kernel(int C, int64_t HW, const float *__restrict__ c2w, const float *__restrict__ v,
               float *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= C * HW) return;
  const float *R = c2w + 16 * (i / HW);
  const float x = v[3 * i], y = v[3 * i + 1], z = v[3 * i + 2];
#pragma unroll
  for (int r = 0; r < 3; ++r) out[3 * i + r] = R[4 * r] * x + R[4 * r + 1] * y + R[4 * r + 2] * z;
}

}  // namespace auxk
}  // namespace gs

using namespace gs;

extern "C" int gsplat_hip_quat_scale_to_covar_preci_fwd(int64_t N, const float *quats,
                                                        const float *scales, int triu,
                                                        float *covars, float *precis,
                                                        void *stream) {
  GS_REQUIRE(N >= 0, "quat_scale_to_covar_preci_fwd: negative N");
  if (N == 0) return 0;
  GS_REQUIRE(quats && scales && (covars || precis), "quat_scale_to_covar_preci_fwd: null pointer");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0,
             "quat_scale_to_covar_preci_fwd: quats must be 16-B aligned");
  hipLaunchKernelGGL(auxk::covar_preci_fwd_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, N, quats, scales, triu, covars, precis);
  GS_CHECK_LAUNCH("quat_scale_to_covar_preci_fwd");
  return 0;
}

extern "C" int gsplat_hip_quat_scale_to_covar_preci_bwd(int64_t N, const float *quats,
                                                        const float *scales, int triu,
                                                        const float *v_covars,
                                                        const float *v_precis, float *v_quats,
                                                        float *v_scales, void *stream) {
  GS_REQUIRE(N >= 0, "quat_scale_to_covar_preci_bwd: negative N");
  if (N == 0) return 0;
  GS_REQUIRE(quats && scales && v_quats && v_scales, "quat_scale_to_covar_preci_bwd: null pointer");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)v_quats & 15) == 0,
             "quat_scale_to_covar_preci_bwd: quats / v_quats must be 16-B aligned");
  hipLaunchKernelGGL(auxk::covar_preci_bwd_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, N, quats, scales, triu, v_covars, v_precis, v_quats,
                     v_scales);
  GS_CHECK_LAUNCH("quat_scale_to_covar_preci_bwd");
  return 0;
}

extern "C" int gsplat_hip_relocation(int64_t N, const float *opacities, const float *scales,
                                     const int32_t *ratios, const float *binoms, int n_max,
                                     float *new_opacities, float *new_scales, void *stream) {
  GS_REQUIRE(N >= 0 && n_max >= 1, "relocation: bad sizes");
  if (N == 0) return 0;
  GS_REQUIRE(opacities && scales && ratios && binoms && new_opacities && new_scales,
             "relocation: null pointer");
  hipLaunchKernelGGL(auxk::relocation_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, N, opacities, scales, ratios, binoms, n_max,
                     new_opacities, new_scales);
  GS_CHECK_LAUNCH("relocation");
  return 0;
}

extern "C" int gsplat_hip_mcmc_inject_noise(int64_t N, float *means, const float *quats,
                                            const float *log_scales, const float *logits,
                                            const float *z, uint64_t seed, int64_t step,
                                            const int64_t *step_device, float scaler,
                                            const float *scaler_device, const int32_t *skip_device,
                                            void *stream) {
  GS_REQUIRE(N >= 0, "mcmc_inject_noise: negative N");
  if (N == 0) return 0;
  GS_REQUIRE(means && quats && log_scales && logits, "mcmc_inject_noise: null pointer");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0, "mcmc_inject_noise: quats must be 16-B aligned");
  hipLaunchKernelGGL(auxk::mcmc_noise_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, N, means, quats, log_scales, logits, z, seed, step,
                     step_device, scaler, scaler_device, skip_device);
  GS_CHECK_LAUNCH("mcmc_inject_noise");
  return 0;
}

extern "C" int gsplat_hip_selective_adam(int64_t n_rows, int64_t row, float *param,
                                         const float *grad, float *exp_avg, float *exp_avg_sq,
                                         const uint8_t *visible, float lr, float beta1,
                                         float beta2, float eps, void *stream) {
  GS_REQUIRE(n_rows >= 0 && row >= 1, "selective_adam: bad sizes");
  const int64_t n = n_rows * row;
  if (n == 0) return 0;
  GS_REQUIRE(param && grad && exp_avg && exp_avg_sq, "selective_adam: null pointer");
  hipLaunchKernelGGL(auxk::selective_adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n_rows, row, param, grad, exp_avg, exp_avg_sq, visible,
                     lr, beta1, beta2, eps);
  GS_CHECK_LAUNCH("selective_adam");
  return 0;
}

extern "C" int gsplat_hip_depth_to_normal(int C, int H, int W, const float *depths,
                                          int64_t depth_stride, const float *camtoworlds,
                                          const float *Ks, int z_depth, float *normals,
                                          void *stream) {
  GS_REQUIRE(C >= 0 && H >= 0 && W >= 0, "depth_to_normal: negative sizes");
  const int64_t n = (int64_t)C * H * W;
  if (n == 0) return 0;
  GS_REQUIRE(depths && camtoworlds && Ks && normals, "depth_to_normal: null pointer");
  GS_REQUIRE(depth_stride >= 1, "depth_to_normal: depth_stride %lld < 1", (long long)depth_stride);
  hipLaunchKernelGGL(auxk::depth_to_normal_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256),
                     0, (hipStream_t)stream, C, H, W, depths, depth_stride, camtoworlds, Ks,
                     z_depth, normals);
  GS_CHECK_LAUNCH("depth_to_normal");
  return 0;
}

extern "C" int gsplat_hip_rotate3(int C, int64_t HW, const float *camtoworlds, const float *v,
                                  float *out, void *stream) {
  GS_REQUIRE(C >= 0 && HW >= 0, "rotate3: negative sizes");
  const int64_t n = (int64_t)C * HW;
  if (n == 0) return 0;
  GS_REQUIRE(camtoworlds && v && out, "rotate3: null pointer");
  hipLaunchKernelGGL(auxk::rotate3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, C, HW, camtoworlds, v, out);
  GS_CHECK_LAUNCH("rotate3");
  return 0;
}
