// Shared device helpers for the gsplat HIP backend (gfx950 / CDNA4).
//
// Everything here is written for wave64 CDNA4: reductions use the 64-lane
// wave, atomics are native no-return `global_atomic_add_f32`.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#define GS_INLINE __device__ __forceinline__

namespace gs {

constexpr int kWave = 64;

// Per-thread last-error slot used by the C-ABI (see abi.cpp).
void set_error(const char *fmt, ...);

#define GS_CHECK_LAUNCH(name)                                                  \
  do {                                                                         \
    hipError_t _e = hipGetLastError();                                         \
    if (_e != hipSuccess) {                                                    \
      gs::set_error("%s: launch failed: %s", name, hipGetErrorString(_e));     \
      return 2;                                                                \
    }                                                                          \
  } while (0)

#define GS_HIP(call)                                                           \
  do {                                                                         \
    hipError_t _e = (call);                                                    \
    if (_e != hipSuccess) {                                                    \
      gs::set_error("%s: %s", #call, hipGetErrorString(_e));                   \
      return 2;                                                                \
    }                                                                          \
  } while (0)

#define GS_REQUIRE(cond, ...)                                                  \
  do {                                                                         \
    if (!(cond)) {                                                             \
      gs::set_error(__VA_ARGS__);                                              \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// ------------------------------------------------------------- zero fill
// Zeroing as a kernel instead of hipMemsetAsync: a captured training step
// (gsplat_hip/graph_step.py) then holds kernel nodes only -- its replays
// faulted with the backward's memset nodes in the graph (the forward,
// without memsets, replayed cleanly).  16-B stores where the buffer allows.
template <int V>
__global__ void __launch_bounds__(256) zero_fill_kernel(void *p, int64_t n_vec, int64_t bytes) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (V == 16) {
    uint4 *q = reinterpret_cast<uint4 *>(p);
    for (int64_t k = i; k < n_vec; k += stride) q[k] = make_uint4(0u, 0u, 0u, 0u);
  } else {
    uint32_t *q = reinterpret_cast<uint32_t *>(p);
    for (int64_t k = i; k < n_vec; k += stride) q[k] = 0u;
  }
  // the bytes past the last whole vector
  const int64_t t = n_vec * V + i;
  if (t < bytes && i < V) reinterpret_cast<uint8_t *>(p)[t] = 0;
}

// Zero fill by kernel, never hipMemsetAsync: a captured memset node of the
// bundled HIP runtime replays with a wrong fill value, and the
// captured training step must hold kernel nodes only.
inline hipError_t zero_async(void *p, size_t bytes, hipStream_t st) {
  if (bytes == 0) return hipSuccess;
  const bool v16 = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  const int V = v16 ? 16 : 4;
  if (!v16 && (reinterpret_cast<uintptr_t>(p) & 3)) return hipErrorInvalidValue;
  const int64_t n_vec = (int64_t)(bytes / V);
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>((n_vec + 255) / 256, 1), 2048);
  if (v16)
    hipLaunchKernelGGL(zero_fill_kernel<16>, dim3((unsigned)blocks), dim3(256), 0, st, p, n_vec,
                       (int64_t)bytes);
  else
    hipLaunchKernelGGL(zero_fill_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, st, p, n_vec,
                       (int64_t)bytes);
  return hipGetLastError();
}

// ------------------------------------------------------------------- Adam
// torch.optim.Adam's element update (amsgrad=False, no weight decay):
// exp_avg via lerp, bias corrections folded into ss = lr / (1 - beta1^t) and
// ib = 1 / sqrt(1 - beta2^t).  Shared by adam.hip and the SH backward with
// the update fused in (sh.hip), so both round identically.
// Every operation is spelled out (explicit fma / rounded mul, add, div) so
// the compiler's contraction choices cannot differ between the two callers.
GS_INLINE void adam_update(float &p, float gr, float &m, float &v, float b1, float b2, float eps,
                           float ss, float ib) {
  m = __fmaf_rn(1.f - b1, __fsub_rn(gr, m), m);  // lerp(m, g, 1 - beta1)
  v = __fmaf_rn(b2, v, __fmul_rn(__fmul_rn(1.f - b2, gr), gr));
  const float den = __fmaf_rn(sqrtf(v), ib, eps);
  p = __fsub_rn(p, __fdiv_rn(__fmul_rn(ss, m), den));
}

// ------------------------------------------------------------- wave reduce
// Butterfly sum over the 64 lanes; every lane ends with the total.
GS_INLINE float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  return v;
}

GS_INLINE void atomic_add_f32(float *p, float v) {
  // gfx950 has native no-return fp32 global atomics; unsafeAtomicAdd lowers
  // to a single global_atomic_add_f32 (no CAS loop).
  unsafeAtomicAdd(p, v);
}

// ------------------------------------------------------------- 3x3 algebra
struct M3 {
  float m[3][3];
};

GS_INLINE M3 mul(const M3 &a, const M3 &b) {
  M3 c;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      c.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
  return c;
}

GS_INLINE M3 transpose(const M3 &a) {
  M3 c;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) c.m[i][j] = a.m[j][i];
  return c;
}

// Rotation from a (w,x,y,z) quaternion normalised with rsqrt
// (reference: quat_scale_to_covar.py:147-203).
GS_INLINE M3 quat_to_rotmat(float q0, float q1, float q2, float q3) {
  float inv = rsqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
  float w = q0 * inv, x = q1 * inv, y = q2 * inv, z = q3 * inv;
  float x2 = x * x, y2 = y * y, z2 = z * z;
  float xy = x * y, xz = x * z, yz = y * z;
  float xw = x * w, yw = y * w, zw = z * w;
  M3 R;
  R.m[0][0] = 1.f - 2.f * (y2 + z2);
  R.m[0][1] = 2.f * (xy - zw);
  R.m[0][2] = 2.f * (xz + yw);
  R.m[1][0] = 2.f * (xy + zw);
  R.m[1][1] = 1.f - 2.f * (x2 + z2);
  R.m[1][2] = 2.f * (yz - xw);
  R.m[2][0] = 2.f * (xz - yw);
  R.m[2][1] = 2.f * (yz + xw);
  R.m[2][2] = 1.f - 2.f * (x2 + y2);
  return R;
}

// VJP of quat_to_rotmat including the normalisation
// (reference: quat_scale_to_covar.py:206-271).
GS_INLINE void quat_to_rotmat_vjp(float q0, float q1, float q2, float q3, const M3 &dR,
                                  float dq[4]) {
  float inv = rsqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
  float w = q0 * inv, x = q1 * inv, y = q2 * inv, z = q3 * inv;
  float zy_m_yz = dR.m[2][1] - dR.m[1][2];
  float xz_m_zx = dR.m[0][2] - dR.m[2][0];
  float yx_m_xy = dR.m[1][0] - dR.m[0][1];
  float xy_p_yx = dR.m[0][1] + dR.m[1][0];
  float xz_p_zx = dR.m[0][2] + dR.m[2][0];
  float yz_p_zy = dR.m[1][2] + dR.m[2][1];
  float dw = 2.f * (x * zy_m_yz + y * xz_m_zx + z * yx_m_xy);
  float dx = 2.f * (-2.f * x * (dR.m[1][1] + dR.m[2][2]) + y * xy_p_yx + z * xz_p_zx + w * zy_m_yz);
  float dy = 2.f * (x * xy_p_yx - 2.f * y * (dR.m[0][0] + dR.m[2][2]) + z * yz_p_zy + w * xz_m_zx);
  float dz = 2.f * (x * xz_p_zx + y * yz_p_zy - 2.f * z * (dR.m[0][0] + dR.m[1][1]) + w * yx_m_xy);
  float dot = w * dw + x * dx + y * dy + z * dz;
  dq[0] = (dw - w * dot) * inv;
  dq[1] = (dx - x * dot) * inv;
  dq[2] = (dy - y * dot) * inv;
  dq[3] = (dz - z * dot) * inv;
}

}  // namespace gs
