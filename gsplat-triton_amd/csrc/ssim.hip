// Fused SSIM (+ L1) training loss, forward and backward, gfx950.
//
// The reference trainer's photometric loss is
//   0.8 * L1 + 0.2 * (1 - fused_ssim(render, gt, padding="valid"))
// (examples/simple_trainer.py:642-646), where fused_ssim is the CUDA
// extension rahul-goel/fused-ssim@1272e21a (examples/requirements.txt:22; not
// vendored in the reference).  This file restates its published algorithm:
// 11x11 Gaussian window (sigma 1.5), C1 = 0.01^2, C2 = 0.03^2, SSIM map on the
// "valid" region only, mean over that map; the backward propagates through
// mu, sigma^2 and sigma_12 exactly (no approximation).
//
// Layout: images [B, H, W, C] fp32 (the renderer's native layout, no permute
// copy).  Per 16x16 output tile a workgroup stages the 26x26 input window in
// LDS and runs the separable blur in two LDS passes.  The forward stores, per
// valid map pixel and channel, the three partials dSSIM/dmu1, dSSIM/dE[x^2]
// and dSSIM/dE[xy]; the backward blurs those back onto the image.
#include "common.h"
#include "../../include/gsplat_hip.h"

namespace gs {
namespace ssim {

constexpr int R = 5, K = 11, TS = 16, WIN = TS + 2 * R;  // 26
__constant__ float kG[K] = {1.028380084e-03f, 7.598758135e-03f, 3.600077213e-02f,
                            1.093606895e-01f, 2.130055377e-01f, 2.660117249e-01f,
                            2.130055377e-01f, 1.093606895e-01f, 3.600077213e-02f,
                            7.598758135e-03f, 1.028380084e-03f};
constexpr float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;

// maps: [B][C][3][Hm][Wm]
__global__ void __launch_bounds__(256)
fwd_kernel(int B, int H, int W, int C, const float *__restrict__ x, const float *__restrict__ y,
           float *__restrict__ maps, float *__restrict__ partials) {
  __shared__ float sx[WIN][WIN], sy[WIN][WIN];
  __shared__ float h[5][WIN][TS];
  __shared__ float red[2][4];
  const int Hm = H - 2 * R, Wm = W - 2 * R;
  const int b = blockIdx.z;
  const int mi0 = blockIdx.y * TS, mj0 = blockIdx.x * TS;  // map tile origin
  const int tid = threadIdx.x, ti = tid / TS, tj = tid % TS;
  const int mi = mi0 + ti, mj = mj0 + tj;
  const bool valid = mi < Hm && mj < Wm;
  float ssum = 0.f, lsum = 0.f;
  for (int c = 0; c < C; ++c) {
    // image window rows [mi0, mi0+26), cols [mj0, mj0+26)
    for (int e = tid; e < WIN * WIN; e += 256) {
      const int r = e / WIN, q = e % WIN;
      const int gi = mi0 + r, gj = mj0 + q;
      float vx = 0.f, vy = 0.f;
      if (gi < H && gj < W) {
        const int64_t o = (((int64_t)b * H + gi) * W + gj) * C + c;
        vx = x[o];
        vy = y[o];
      }
      sx[r][q] = vx;
      sy[r][q] = vy;
    }
    __syncthreads();
    for (int e = tid; e < WIN * TS; e += 256) {
      const int r = e / TS, q = e % TS;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float g = kG[k], vx = sx[r][q + k], vy = sy[r][q + k];
        a0 += g * vx;
        a1 += g * vy;
        a2 += g * vx * vx;
        a3 += g * vy * vy;
        a4 += g * vx * vy;
      }
      h[0][r][q] = a0; h[1][r][q] = a1; h[2][r][q] = a2; h[3][r][q] = a3; h[4][r][q] = a4;
    }
    __syncthreads();
    float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float g = kG[k];
      m1 += g * h[0][ti + k][tj];
      m2 += g * h[1][ti + k][tj];
      e11 += g * h[2][ti + k][tj];
      e22 += g * h[3][ti + k][tj];
      e12 += g * h[4][ti + k][tj];
    }
    if (valid) {
      const float s11 = e11 - m1 * m1, s22 = e22 - m2 * m2, s12 = e12 - m1 * m2;
      const float A1 = 2.f * m1 * m2 + C1, A2 = 2.f * s12 + C2;
      const float B1 = m1 * m1 + m2 * m2 + C1, B2 = s11 + s22 + C2;
      const float Dn = B1 * B2, inv = 1.f / Dn;
      const float s = A1 * A2 * inv;
      ssum += s;
      // partials w.r.t. mu1, E[x^2], E[xy] (E's independent of mu1)
      const float dN = 2.f * m2 * (A2 - A1), dD = 2.f * m1 * (B2 - B1);
      const float d_mu1 = (dN - s * dD) * inv;
      const float d_e11 = -s * B1 * inv;
      const float d_e12 = 2.f * A1 * inv;
      const int64_t plane = (int64_t)Hm * Wm;
      float *mp = maps + (((int64_t)b * C + c) * 3) * plane + (int64_t)mi * Wm + mj;
      mp[0] = d_mu1;
      mp[plane] = d_e11;
      mp[2 * plane] = d_e12;
    }
    __syncthreads();
  }
  // L1 over the whole image: each workgroup owns the image pixels of its map
  // tile (edge workgroups also cover the 2R-pixel border beyond the map)
  {
    const int ri0 = mi0, rj0 = mj0;
    const int ri1 = (mi0 + TS >= Hm) ? H : mi0 + TS;
    const int rj1 = (mj0 + TS >= Wm) ? W : mj0 + TS;
    for (int e = tid; e < (ri1 - ri0) * (rj1 - rj0); e += 256) {
      const int gi = ri0 + e / (rj1 - rj0), gj = rj0 + e % (rj1 - rj0);
      const int64_t o = (((int64_t)b * H + gi) * W + gj) * C;
      for (int c = 0; c < C; ++c) lsum += fabsf(x[o + c] - y[o + c]);
    }
  }
  ssum = wave_sum(ssum);
  lsum = wave_sum(lsum);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = ssum;
    red[1][tid >> 6] = lsum;
  }
  __syncthreads();
  if (tid == 0) {  // per-workgroup partials (no same-address atomics)
    const int blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    partials[2 * blk] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    partials[2 * blk + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// Deterministic sum of the per-workgroup partials -> sums[2].
__global__ void __launch_bounds__(1024) reduce_partials_kernel(int n, const float *partials,
                                                               float *sums) {
  __shared__ float red[2][16];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) {
    a += partials[2 * i];
    b += partials[2 * i + 1];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[threadIdx.x][w];
    sums[threadIdx.x] = t;
  }
}

__global__ void __launch_bounds__(256)
bwd_kernel(int B, int H, int W, int C, const float *__restrict__ x, const float *__restrict__ y,
           const float *__restrict__ maps, const float *__restrict__ dloss,
           float *__restrict__ grad) {
  __shared__ float sm[3][WIN][WIN];
  __shared__ float h[3][WIN][TS];
  const int Hm = H - 2 * R, Wm = W - 2 * R;
  const int b = blockIdx.z;
  const int qi0 = blockIdx.y * TS, qj0 = blockIdx.x * TS;  // image tile origin
  const int tid = threadIdx.x, ti = tid / TS, tj = tid % TS;
  const int qi = qi0 + ti, qj = qj0 + tj;
  const float n_map = (float)B * C * Hm * Wm, n_img = (float)B * C * H * W;
  const float g_ssim = dloss[0] / n_map, g_l1 = dloss[1] / n_img;
  const int64_t plane = (int64_t)Hm * Wm;
  for (int c = 0; c < C; ++c) {
    const float *mp = maps + (((int64_t)b * C + c) * 3) * plane;
    // map window rows [qi0-10, qi0+16), cols [qj0-10, qj0+16)
    for (int e = tid; e < WIN * WIN; e += 256) {
      const int r = e / WIN, q = e % WIN;
      const int pi = qi0 - 2 * R + r, pj = qj0 - 2 * R + q;
      const bool in = pi >= 0 && pi < Hm && pj >= 0 && pj < Wm;
      const int64_t o = (int64_t)pi * Wm + pj;
      sm[0][r][q] = in ? mp[o] : 0.f;
      sm[1][r][q] = in ? mp[plane + o] : 0.f;
      sm[2][r][q] = in ? mp[2 * plane + o] : 0.f;
    }
    __syncthreads();
    for (int e = tid; e < WIN * TS; e += 256) {
      const int r = e / TS, q = e % TS;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float g = kG[k];
        a0 += g * sm[0][r][q + k];
        a1 += g * sm[1][r][q + k];
        a2 += g * sm[2][r][q + k];
      }
      h[0][r][q] = a0; h[1][r][q] = a1; h[2][r][q] = a2;
    }
    __syncthreads();
    float A = 0.f, Bv = 0.f, Cv = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float g = kG[k];
      A += g * h[0][ti + k][tj];
      Bv += g * h[1][ti + k][tj];
      Cv += g * h[2][ti + k][tj];
    }
    if (qi < H && qj < W) {
      const int64_t o = (((int64_t)b * H + qi) * W + qj) * C + c;
      const float vx = x[o], vy = y[o];
      const float d = vx - vy;
      const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      grad[o] = g_ssim * (A + 2.f * vx * Bv + vy * Cv) + g_l1 * sgn;
    }
    __syncthreads();
  }
}

}  // namespace ssim
}  // namespace gs

using namespace gs;

static int64_t ssim_map_floats(int B, int H, int W, int C) {
  return (int64_t)B * C * 3 * (int64_t)(H - 10) * (W - 10);
}
static int64_t ssim_blocks(int B, int H, int W) {
  return (int64_t)((W - 10 + 15) / 16) * ((H - 10 + 15) / 16) * B;
}

extern "C" int64_t gsplat_hip_ssim_workspace_bytes(int B, int H, int W, int C) {
  if (H <= 10 || W <= 10) return 0;
  return (int64_t)sizeof(float) * (ssim_map_floats(B, H, W, C) + 2 * ssim_blocks(B, H, W));
}

extern "C" int gsplat_hip_ssim_l1_fwd(int B, int H, int W, int C, const float *img1,
                                      const float *img2, float *sums, void *workspace,
                                      void *stream) {
  GS_REQUIRE(B > 0 && C > 0 && H > 10 && W > 10,
             "ssim_l1_fwd: images must be larger than the 11x11 window (got %dx%d)", H, W);
  hipStream_t st = (hipStream_t)stream;
  float *maps = reinterpret_cast<float *>(workspace);
  float *partials = maps + ssim_map_floats(B, H, W, C);
  dim3 grid((W - 10 + 15) / 16, (H - 10 + 15) / 16, B);
  hipLaunchKernelGGL(ssim::fwd_kernel, grid, dim3(256), 0, st, B, H, W, C, img1, img2, maps,
                     partials);
  hipLaunchKernelGGL(ssim::reduce_partials_kernel, dim3(1), dim3(1024), 0, st,
                     (int)ssim_blocks(B, H, W), partials, sums);
  GS_CHECK_LAUNCH("ssim_l1_fwd");
  return 0;
}

extern "C" int gsplat_hip_ssim_l1_bwd(int B, int H, int W, int C, const float *img1,
                                      const float *img2, const void *workspace,
                                      const float *dloss, float *grad_img1, void *stream) {
  GS_REQUIRE(B > 0 && C > 0 && H > 10 && W > 10, "ssim_l1_bwd: bad image size %dx%d", H, W);
  dim3 grid((W + 15) / 16, (H + 15) / 16, B);
  hipLaunchKernelGGL(ssim::bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, B, H, W, C, img1,
                     img2, reinterpret_cast<const float *>(workspace), dloss, grad_img1);
  GS_CHECK_LAUNCH("ssim_l1_bwd");
  return 0;
}
