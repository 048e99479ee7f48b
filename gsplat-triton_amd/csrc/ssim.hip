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
// copy).  Per 32x32 output tile a workgroup stages the 42x42 input window in
// LDS and runs the separable blur in two LDS passes with packed fp32 (the
// (x, y) and (x^2, y^2) planes as float2, two sums per v_pk_fma_f32).  The forward stores, per
// valid map pixel and channel, the three partials dSSIM/dmu1, dSSIM/dE[x^2]
// and dSSIM/dE[xy]; the backward blurs those back onto the image.
#include "common.h"
#include "../../include/gsplat_hip.h"

namespace gs {
namespace ssim {

constexpr int R = 5, K = 11;
constexpr int TW = 32, WN = TW + 2 * R;  // 32x32 output tile, 42x42 input window
__constant__ float kG[K] = {1.028380084e-03f, 7.598758135e-03f, 3.600077213e-02f,
                            1.093606895e-01f, 2.130055377e-01f, 2.660117249e-01f,
                            2.130055377e-01f, 1.093606895e-01f, 3.600077213e-02f,
                            7.598758135e-03f, 1.028380084e-03f};
constexpr float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;

typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kRows = (WN + 3) / 4;  // window rows per wave in the staging loops

// 1-D grid over (tile, image-channel) so that the channels of one tile run
// back to back on the same XCD (workgroup i goes to XCD i % 8): the
// interleaved [H, W, C] image lines fetched by channel 0 are L2 hits for
// channels 1, 2.  Grid size roundup(n_tiles, 8) * n_bc.
GS_INLINE bool decode_block(int n_tiles, int n_bc, int &t, int &bc) {
  const int L = blockIdx.x, xcd = L & 7, q = L >> 3;
  bc = q % n_bc;
  t = (q / n_bc) * 8 + xcd;
  return t < n_tiles;
}
inline int grid_blocks(int n_tiles, int n_bc) { return ((n_tiles + 7) / 8) * 8 * n_bc; }

// Separable 11-tap blur of a 42x42 window to the 32x32 tile, three planes at
// once (two packed float2 planes + one float plane).  256 threads: column
// tq = tid & 31; the horizontal pass covers rows tr, tr+8, ...; the vertical
// pass gives rows 4 tr .. 4 tr + 3 of column tq with a sliding window.
struct Blur3 {
  f2v a[4], b[4];
  float c[4];
};

template <bool TWO>  // TWO: planes a, b (float2) and c; else a and c
GS_INLINE void blur3(const f2v (*sa)[WN], const f2v (*sb)[WN], const float (*sc)[WN],
                     f2v (*ha)[TW], f2v (*hb)[TW], float (*hc)[TW], int tid, Blur3 &o) {
  const int tq = tid & 31, tr = tid >> 5;
  for (int r = tr; r < WN; r += 8) {
    f2v a = {0.f, 0.f}, b = {0.f, 0.f};
    float c = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float g = kG[k];
      a = __builtin_elementwise_fma(f2v{g, g}, sa[r][tq + k], a);
      if (TWO) b = __builtin_elementwise_fma(f2v{g, g}, sb[r][tq + k], b);
      c = __builtin_fmaf(g, sc[r][tq + k], c);
    }
    ha[r][tq] = a;
    if (TWO) hb[r][tq] = b;
    hc[r][tq] = c;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o.a[j] = f2v{0.f, 0.f};
    o.b[j] = f2v{0.f, 0.f};
    o.c[j] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < K + 3; ++i) {
    const int r = 4 * tr + i;
    const f2v a = ha[r][tq], b = TWO ? hb[r][tq] : f2v{0.f, 0.f};
    const float c = hc[r][tq];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = i - j;
      if (k >= 0 && k < K) {
        const float g = kG[k];
        o.a[j] = __builtin_elementwise_fma(f2v{g, g}, a, o.a[j]);
        if (TWO) o.b[j] = __builtin_elementwise_fma(f2v{g, g}, b, o.b[j]);
        o.c[j] = __builtin_fmaf(g, c, o.c[j]);
      }
    }
  }
}

// Forward flavour: one staged plane (x, y); the horizontal pass forms
// (x^2, y^2) and x y on the fly (LDS 41 KB -> 3 workgroups per CU).
GS_INLINE void blur_xy(const f2v (*sa)[WN], f2v (*ha)[TW], f2v (*hb)[TW], float (*hc)[TW],
                       int tid, Blur3 &o) {
  const int tq = tid & 31, tr = tid >> 5;
  for (int r = tr; r < WN; r += 8) {
    f2v a = {0.f, 0.f}, b = {0.f, 0.f};
    float c = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float g = kG[k];
      const f2v v = sa[r][tq + k];
      const f2v gv = f2v{g, g} * v;
      a += gv;
      b = __builtin_elementwise_fma(gv, v, b);
      c = __builtin_fmaf(gv.x, v.y, c);
    }
    ha[r][tq] = a;
    hb[r][tq] = b;
    hc[r][tq] = c;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o.a[j] = f2v{0.f, 0.f};
    o.b[j] = f2v{0.f, 0.f};
    o.c[j] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < K + 3; ++i) {
    const int r = 4 * tr + i;
    const f2v a = ha[r][tq], b = hb[r][tq];
    const float c = hc[r][tq];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = i - j;
      if (k >= 0 && k < K) {
        const float g = kG[k];
        o.a[j] = __builtin_elementwise_fma(f2v{g, g}, a, o.a[j]);
        o.b[j] = __builtin_elementwise_fma(f2v{g, g}, b, o.b[j]);
        o.c[j] = __builtin_fmaf(g, c, o.c[j]);
      }
    }
  }
}

// maps: [B][C][3][Hm][Wm] -- dSSIM/dmu1, dSSIM/dE[x^2], dSSIM/dE[xy] per map pixel
__global__ void __launch_bounds__(256)
fwd_kernel(int B, int H, int W, int C, const float *__restrict__ x, const float *__restrict__ y,
           float *__restrict__ maps, float *__restrict__ partials) {
  __shared__ f2v s_xy[WN][WN];  // (x, y)
  __shared__ f2v h_xy[WN][TW], h_sq[WN][TW];
  __shared__ float h_p[WN][TW];
  __shared__ float red[2][4];
  const int Hm = H - 2 * R, Wm = W - 2 * R;
  const int tx = (Wm + TW - 1) / TW, ty = (Hm + TW - 1) / TW;
  int t, bc;
  if (!decode_block(tx * ty, B * C, t, bc)) return;
  const int b = bc / C, c = bc - b * C;  // one channel per workgroup
  const int mi0 = (t / tx) * TW, mj0 = (t % tx) * TW;  // map tile origin
  const int tid = threadIdx.x, tq = tid & 31, tr = tid >> 5;
  const int64_t plane = (int64_t)Hm * Wm;
  float ssum = 0.f, lsum = 0.f;
  {
    // window staging: lane = window column, wave w = rows w, w+4, ...; row
    // pointers are wave-uniform, so the loads are saddr + per-lane offset and
    // all of them are in flight before the first LDS store
    const int lane = tid & 63, w4 = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int gj = mj0 + lane;
    const bool col_ok = lane < WN && gj < W;
    const int64_t img0 = (int64_t)b * H * W * C + c;
    const uint32_t lo = (uint32_t)(min(gj, W - 1) * C);  // clamped: loads are unconditional
    float vx[kRows], vy[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = w4 + 4 * k, gi = min(mi0 + r, H - 1);
      const float *xr = x + img0 + (int64_t)gi * W * C;
      const float *yr = y + img0 + (int64_t)gi * W * C;
      vx[k] = xr[lo];
      vy[k] = yr[lo];
    }
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const bool ok = col_ok && mi0 + w4 + 4 * k < H;
      vx[k] = ok ? vx[k] : 0.f;
      vy[k] = ok ? vy[k] : 0.f;
    }
    // L1 over the whole image from the window: each workgroup owns the image
    // pixels of its map tile (edge workgroups also the 2R-pixel border)
    const int ri1 = (mi0 + TW >= Hm) ? H - mi0 : TW;
    const int rj1 = (mj0 + TW >= Wm) ? W - mj0 : TW;
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = w4 + 4 * k;
      if (r < WN && lane < WN) {
        s_xy[r][lane] = f2v{vx[k], vy[k]};
        if (r < ri1 && lane < rj1) lsum += fabsf(vx[k] - vy[k]);
      }
    }
    __syncthreads();
    Blur3 o;
    blur_xy(s_xy, h_xy, h_sq, h_p, tid, o);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int mi = mi0 + 4 * tr + j, mj = mj0 + tq;
      if (mi < Hm && mj < Wm) {
        const float m1 = o.a[j].x, m2 = o.a[j].y;
        const float s11 = o.b[j].x - m1 * m1, s22 = o.b[j].y - m2 * m2, s12 = o.c[j] - m1 * m2;
        const float A1 = 2.f * m1 * m2 + C1, A2 = 2.f * s12 + C2;
        const float B1 = m1 * m1 + m2 * m2 + C1, B2 = s11 + s22 + C2;
        const float inv = 1.f / (B1 * B2);
        const float sv = A1 * A2 * inv;
        ssum += sv;
        // partials w.r.t. mu1, E[x^2], E[xy] (the E's independent of mu1)
        const float dN = 2.f * m2 * (A2 - A1), dD = 2.f * m1 * (B2 - B1);
        float *mp = maps + (((int64_t)b * C + c) * 3) * plane + (int64_t)mi * Wm + mj;
        mp[0] = (dN - sv * dD) * inv;
        mp[plane] = -sv * B1 * inv;
        mp[2 * plane] = 2.f * A1 * inv;
      }
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
    const int blk = bc * tx * ty + t;
    partials[2 * blk] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    partials[2 * blk + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// Forward, all C channels of a 32x32 map tile in one workgroup: the 42-row
// window of both images is loaded as 42 contiguous runs of 42*C floats (the
// [H, W, C] rows: coalesced, every load of the three channels in flight at
// once), then each channel is staged to LDS from registers and blurred in
// turn.  One workgroup per (tile, image) instead of per (tile, image,
// channel): a third of the prologues and of the load-latency rounds.
// Partials: one (ssim, l1) pair per workgroup, channels summed.
template <int C>
__global__ void __launch_bounds__(256)
fwd_c_kernel(int B, int H, int W, const float *__restrict__ x, const float *__restrict__ y,
             float *__restrict__ maps, float *__restrict__ partials) {
  constexpr int SPAN = WN * C;             // floats per window row
  constexpr int PER_ROW = (SPAN + 63) / 64;  // loads per lane per row
  __shared__ f2v s_xy[WN][WN];
  __shared__ f2v h_xy[WN][TW], h_sq[WN][TW];
  __shared__ float h_p[WN][TW];
  __shared__ float red[2][4];
  const int Hm = H - 2 * R, Wm = W - 2 * R;
  const int tx = (Wm + TW - 1) / TW, ty = (Hm + TW - 1) / TW;
  const int t = blockIdx.x % (tx * ty), b = blockIdx.x / (tx * ty);
  if (b >= B) return;
  const int mi0 = (t / tx) * TW, mj0 = (t % tx) * TW;
  const int tid = threadIdx.x, tq = tid & 31, tr = tid >> 5;
  const int lane = tid & 63, w4 = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t plane = (int64_t)Hm * Wm;
  const int ri1 = (mi0 + TW >= Hm) ? H - mi0 : TW;  // image rows / cols this tile owns for L1
  const int rj1 = (mj0 + TW >= Wm) ? W - mj0 : TW;
  float vx[kRows][PER_ROW], vy[kRows][PER_ROW];
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    const int r = w4 + 4 * k, gi = min(mi0 + r, H - 1);
    const int64_t row0 = (((int64_t)b * H + gi) * W + mj0) * C;
#pragma unroll
    for (int q = 0; q < PER_ROW; ++q) {
      const int e = lane + 64 * q;
      const int gj = mj0 + e / C;
      const int64_t off = gj < W ? row0 + e : row0;  // clamped: loads are unconditional
      vx[k][q] = x[off];
      vy[k][q] = y[off];
    }
  }
  float lsum = 0.f, ssum = 0.f;
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    const int r = w4 + 4 * k;
#pragma unroll
    for (int q = 0; q < PER_ROW; ++q) {
      const int e = lane + 64 * q, col = e / C;
      const bool ok = r < WN && e < SPAN && mi0 + r < H && mj0 + col < W;
      vx[k][q] = ok ? vx[k][q] : 0.f;
      vy[k][q] = ok ? vy[k][q] : 0.f;
      if (ok && r < ri1 && col < rj1) lsum += fabsf(vx[k][q] - vy[k][q]);
    }
  }
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = w4 + 4 * k;
#pragma unroll
      for (int q = 0; q < PER_ROW; ++q) {
        const int e = lane + 64 * q;
        if (r < WN && e < SPAN && e % C == c) s_xy[r][e / C] = f2v{vx[k][q], vy[k][q]};
      }
    }
    __syncthreads();
    Blur3 o;
    blur_xy(s_xy, h_xy, h_sq, h_p, tid, o);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int mi = mi0 + 4 * tr + j, mj = mj0 + tq;
      if (mi < Hm && mj < Wm) {
        const float m1 = o.a[j].x, m2 = o.a[j].y;
        const float s11 = o.b[j].x - m1 * m1, s22 = o.b[j].y - m2 * m2, s12 = o.c[j] - m1 * m2;
        const float A1 = 2.f * m1 * m2 + C1, A2 = 2.f * s12 + C2;
        const float B1 = m1 * m1 + m2 * m2 + C1, B2 = s11 + s22 + C2;
        const float inv = 1.f / (B1 * B2);
        const float sv = A1 * A2 * inv;
        ssum += sv;
        const float dN = 2.f * m2 * (A2 - A1), dD = 2.f * m1 * (B2 - B1);
        float *mp = maps + (((int64_t)b * C + c) * 3) * plane + (int64_t)mi * Wm + mj;
        mp[0] = (dN - sv * dD) * inv;
        mp[plane] = -sv * B1 * inv;
        mp[2 * plane] = 2.f * A1 * inv;
      }
    }
    __syncthreads();  // s_xy / h_* are rewritten for the next channel
  }
  ssum = wave_sum(ssum);
  lsum = wave_sum(lsum);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = ssum;
    red[1][tid >> 6] = lsum;
  }
  __syncthreads();
  if (tid == 0) {
    partials[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    partials[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// Deterministic sum of the per-workgroup partials -> sums[2].
// With loss != nullptr also loss[0..2] = (w_l1 L1/n_img + lam (1 - S/n_map),
// S/n_map, L1/n_img).
__global__ void __launch_bounds__(1024) reduce_partials_kernel(int n, const float *partials,
                                                               float *sums, float *loss,
                                                               float lam, float n_map,
                                                               float n_img,
                                                               float *ring = nullptr,
                                                               int64_t ring_len = 0,
                                                               const int64_t *seq = nullptr) {
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
  if (threadIdx.x == 0) {
    float t[2] = {0.f, 0.f};
    for (int w = 0; w < 16; ++w) {
      t[0] += red[0][w];
      t[1] += red[1][w];
    }
    if (sums) {
      sums[0] = t[0];
      sums[1] = t[1];
    }
    if (loss) {
      const float s = t[0] / n_map, l1 = t[1] / n_img;
      loss[0] = l1 * (1.f - lam) + (1.f - s) * lam;
      loss[1] = s;
      loss[2] = l1;
      if (ring) {
        int64_t k = (seq[0] - 1) % ring_len;
        ring[k < 0 ? k + ring_len : k] = loss[0];
      }
    }
  }
}

__global__ void __launch_bounds__(256)
bwd_kernel(int B, int H, int W, int C, const float *__restrict__ x, const float *__restrict__ y,
           const float *__restrict__ maps, const float *__restrict__ dloss, float s_ssim,
           float s_l1, int l1_index, float *__restrict__ grad) {
  __shared__ f2v s_01[WN][WN];  // (dSSIM/dmu1, dSSIM/dE[x^2])
  __shared__ float s_2[WN][WN];  // dSSIM/dE[xy]
  __shared__ f2v h_01[WN][TW];
  __shared__ float h_2[WN][TW];
  const int Hm = H - 2 * R, Wm = W - 2 * R;
  const int tx = (W + TW - 1) / TW, ty = (H + TW - 1) / TW;
  int t, bc;
  if (!decode_block(tx * ty, B * C, t, bc)) return;
  const int b = bc / C, c = bc - b * C;  // one channel per workgroup
  const int qi0 = (t / tx) * TW, qj0 = (t % tx) * TW;  // image tile origin
  const int tid = threadIdx.x, tq = tid & 31, tr = tid >> 5;
  // dL/d(SSIM map sum) and dL/d(L1 sum)
  const float g_ssim = dloss[0] * s_ssim, g_l1 = dloss[l1_index] * s_l1;
  const int64_t plane = (int64_t)Hm * Wm;
  {
    const float *mp = maps + (((int64_t)b * C + c) * 3) * plane;
    // map window rows [qi0-10, qi0+32), cols [qj0-10, qj0+32), zero outside;
    // lane = window column, wave w = rows w, w+4, ... (see fwd_kernel)
    const int lane = tid & 63, w4 = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int pj = qj0 - 2 * R + lane;
    const bool col_ok = lane < WN && pj >= 0 && pj < Wm;
    const int pjc = min(max(pj, 0), Wm - 1);  // clamped: loads are unconditional
    float m0[kRows], m1[kRows], m2[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int pi = min(max(qi0 - 2 * R + w4 + 4 * k, 0), Hm - 1);
      const float *row = mp + (int64_t)pi * Wm;
      m0[k] = row[pjc];
      m1[k] = row[plane + pjc];
      m2[k] = row[2 * plane + pjc];
    }
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int pi = qi0 - 2 * R + w4 + 4 * k;
      const bool ok = col_ok && pi >= 0 && pi < Hm;
      m0[k] = ok ? m0[k] : 0.f;
      m1[k] = ok ? m1[k] : 0.f;
      m2[k] = ok ? m2[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = w4 + 4 * k;
      if (r < WN && lane < WN) {
        s_01[r][lane] = f2v{m0[k], m1[k]};
        s_2[r][lane] = m2[k];
      }
    }
    __syncthreads();
    // the adjoint of the valid correlation is the full correlation with the
    // flipped kernel, and the Gaussian window is symmetric
    Blur3 o;
    blur3<false>(s_01, nullptr, s_2, h_01, nullptr, h_2, tid, o);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qi = qi0 + 4 * tr + j, qj = qj0 + tq;
      if (qi < H && qj < W) {
        const int64_t off = (((int64_t)b * H + qi) * W + qj) * C + c;
        const float vx = x[off], vy = y[off];
        const float d = vx - vy;
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        grad[off] = g_ssim * (o.a[j].x + 2.f * vx * o.a[j].y + vy * o.c[j]) + g_l1 * sgn;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Loss and gradient in one pass (training forward).  Per 32x32 IMAGE tile a
// workgroup loads the 52x52 image window (both images, all channels, rows of
// 52*C contiguous floats), and per channel
//   A. blurs x, y, x^2, y^2, xy horizontally (52 rows -> 42 columns),
//   B. vertically -> the 42x42 SSIM map pixels whose windows touch the tile,
//      with their three partials dSSIM/dmu1, dSSIM/dE[x^2], dSSIM/dE[xy]
//      (zero outside the valid map), kept in LDS,
//   C. blurs those back horizontally (42 rows -> 32 columns) and vertically
//      onto the tile's pixels: dSSIMsum/dx, combined with the L1 sign term.
// The map pixels of the tile's own 32x32 range (every map pixel has exactly
// one) feed the loss sum.  Against fwd (maps to HBM) + bwd (maps back) it
// trades a 1.7x recompute of the map statistics for 150 MB less traffic at
// 1080p, one launch and the 75 MB map workspace less; the gradient is for
// dL/dloss = 1 and the backward only scales it (fused_scale_kernel).
// Measured at 1080p RGB (profiles/r2_s4_ssim): 117.6 us vs 55 + 62 us for
// the pair -- parity, not a win: the kernel is neither HBM- nor VALU-bound
// (VALU issue ~0.3, ~42 % of wave cycles waiting on the per-channel window
// loads and the four barriers per channel at 2 workgroups per CU).
constexpr int FT = 32, FM = FT + 2 * R, FI = FM + 2 * R;  // 32, 42, 52
constexpr int kFThreads = 512, kFRows = (FI + 7) / 8;     // window rows per wave
// LDS (rows padded by one element so that the column-blocked passes, whose
// lanes walk down consecutive rows, hit distinct banks):
//   s_xy f2v[FI][SX] | hA f2v[FI][SH] | hB f2v[FI][SH] | hC float[FI][SH].
// Once pass A has read the window (each thread keeps the (x, y) of its two
// output pixels in registers) the maps (f2v[FM][SH] + float[FM][SH]) reuse
// s_xy; the backward's horizontal pass (f2v[FM][SG] + float[FM][SG]) reuses
// hA.  Four barriers per channel.
constexpr int SX = FI + 1, SH = FM + 1, SG = FT + 1;
constexpr int kOffA = FI * SX * 8, kOffB = kOffA + FI * SH * 8, kOffC = kOffB + FI * SH * 8;
constexpr int kFusedLds = kOffC + FI * SH * 4;
static_assert(FM * SH * 12 <= FI * SX * 8, "maps fit in s_xy");
static_assert(FM * SG * 12 <= FI * SH * 8, "backward h-pass fits in hA");
constexpr int kHA = 6, kHC = 4;  // adjacent outputs per work item in passes A, C1

// BR: map rows per work item of pass B (sliding window of K + BR - 1 rows).
// Passes A and C1 are register-blocked: kHA / kHC adjacent outputs of one
// row from one run of K + kHA - 1 / K + kHC - 1 LDS values.
// CPW: channels per workgroup (C / CPW workgroups per tile, channel groups of
// a tile adjacent in the XCD-aware order so they share that XCD's L2).
// XS: floats per pixel of x and grad (a compile-time constant: a runtime
// stride cost the C = 3 kernel 114 -> 148 us at 1080p).
template <int C, int BR, int CPW = C, int XS = C>
__global__ void __launch_bounds__(kFThreads) __attribute__((amdgpu_waves_per_eu(4)))
fused_kernel(int B, int H, int W, const float *__restrict__ x,
             const float *__restrict__ y, const int64_t *__restrict__ y_index, float cs, float cl,
             float *__restrict__ grad, float *__restrict__ partials) {
  static_assert(C % CPW == 0, "channel groups");
  constexpr int CG = C / CPW;
  __shared__ __attribute__((aligned(16))) char lds[kFusedLds];
  __shared__ float red[2][kFThreads / 64];
  f2v(*s_xy)[SX] = reinterpret_cast<f2v(*)[SX]>(lds);
  f2v(*hA)[SH] = reinterpret_cast<f2v(*)[SH]>(lds + kOffA);
  f2v(*hB)[SH] = reinterpret_cast<f2v(*)[SH]>(lds + kOffB);
  float(*hC)[SH] = reinterpret_cast<float(*)[SH]>(lds + kOffC);
  f2v(*m01)[SH] = reinterpret_cast<f2v(*)[SH]>(lds);
  float(*m2)[SH] = reinterpret_cast<float(*)[SH]>(lds + FM * SH * 8);
  f2v(*g01)[SG] = reinterpret_cast<f2v(*)[SG]>(lds + kOffA);
  float(*g2)[SG] = reinterpret_cast<float(*)[SG]>(lds + kOffA + FM * SG * 8);

  const int Hm = H - 2 * R, Wm = W - 2 * R;
  const int tx = (W + FT - 1) / FT, ty = (H + FT - 1) / FT, nt = tx * ty, ntc = nt * CG;
  // XCD-aware: workgroup L runs on XCD L % 8; each XCD takes a contiguous
  // run of (tile, channel group)s so neighbouring windows' shared apron rows
  // (and a tile's other channel groups) hit its L2
  const int per = (ntc + 7) / 8, L = blockIdx.x;
  const int b = L / (8 * per), q = L - b * 8 * per;
  const int tc = (q & 7) * per + (q >> 3);
  if (b >= B || tc >= ntc) return;
  const int t = tc / CG, cg = tc - t * CG;
  if (y_index) y += y_index[0] * ((int64_t)B * H * W * C);  // image y_index of a stack
  const int qi0 = (t / tx) * FT, qj0 = (t % tx) * FT;  // image tile origin
  const int ri0 = qi0 - 2 * R, rj0 = qj0 - 2 * R;       // window origin (image coords)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w8 = __builtin_amdgcn_readfirstlane(tid >> 6);

  // window loads of one channel: lane = window column, wave w = rows w, w+8,
  // ...; clamped addresses (unconditional loads), zeroed outside the image
  // (row pointers are wave-uniform: saddr + one 32-bit lane offset per load)
  // x (the render, and its gradient) has XS >= C floats per pixel (an RGB+D
  // render read in place: XS = 4, C = 3); y has C
  const int colc = min(max(rj0 + lane, 0), W - 1);
  const uint32_t lox = (uint32_t)(colc * XS), loy = (uint32_t)(colc * C);
  const bool col_ok = lane < FI && rj0 + lane >= 0 && rj0 + lane < W;
  const float *xb = x + (int64_t)b * H * W * XS, *yb = y + (int64_t)b * H * W * C;
  float vx[kFRows], vy[kFRows];
  auto load = [&](int c) {
#pragma unroll
    for (int k = 0; k < kFRows; ++k) {
      const int64_t row = (int64_t)min(max(ri0 + w8 + 8 * k, 0), H - 1) * W;
      vx[k] = (xb + row * XS)[lox + c];
      vy[k] = (yb + row * C)[loy + c];
    }
  };
  float lsum = 0.f, ssum = 0.f;
  // backward vertical pass mapping: column gc, image rows 2 gr, 2 gr + 1
  const int gc = tid & 31, gr = tid >> 5;
  // the loaded window into s_xy (+ its L1 over the tile's own pixels, window
  // rows / cols 2R .. 2R+31)
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k < kFRows; ++k) {
      const int r = w8 + 8 * k, gi = ri0 + r;
      const bool ok = col_ok && r < FI && gi >= 0 && gi < H;
      const float a = ok ? vx[k] : 0.f, bb = ok ? vy[k] : 0.f;
      if (r < FI && lane < FI) s_xy[r][lane] = f2v{a, bb};
      if (r >= 2 * R && r < 2 * R + FT && lane >= 2 * R && lane < 2 * R + FT)
        lsum += fabsf(a - bb);
    }
  };
  // The next channel's window is loaded while pass C1 runs (its latency
  // hidden behind C1) and staged while C2 runs: s_xy's last readers of this
  // channel (pass C1, through m01 / m2) are behind C1's barrier, and this
  // channel's own pixels (px0 / px1) were read into registers before pass A.
  const int c_end = cg * CPW + CPW;
  load(cg * CPW);
  stage();
  __syncthreads();
#pragma nounroll
  for (int c = cg * CPW; c < c_end; ++c) {
    const f2v px0 = s_xy[2 * R + 2 * gr][2 * R + gc], px1 = s_xy[2 * R + 2 * gr + 1][2 * R + gc];
    // ---- A: horizontal blur of the statistics, FI rows x FM columns
    static_assert(FM % kHA == 0 && FT % kHC == 0, "pass A / C1 blocking");
    for (int idx = tid; idx < FI * (FM / kHA); idx += kFThreads) {
      const int jg = idx / FI, r = idx - jg * FI, j0 = jg * kHA;
      f2v v[K + kHA - 1], sq[K + kHA - 1];
      float xy[K + kHA - 1];
#pragma unroll
      for (int i = 0; i < K + kHA - 1; ++i) {
        v[i] = s_xy[r][j0 + i];
        sq[i] = v[i] * v[i];
        xy[i] = v[i].x * v[i].y;
      }
#pragma unroll
      for (int o = 0; o < kHA; ++o) {
        f2v a = {0.f, 0.f}, bb = {0.f, 0.f};
        float cc = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float g = kG[k];
          a = __builtin_elementwise_fma(f2v{g, g}, v[o + k], a);
          bb = __builtin_elementwise_fma(f2v{g, g}, sq[o + k], bb);
          cc = __builtin_fmaf(g, xy[o + k], cc);
        }
        hA[r][j0 + o] = a;
        hB[r][j0 + o] = bb;
        hC[r][j0 + o] = cc;
      }
    }
    __syncthreads();
    // ---- B: vertical blur -> the partials of map pixels (local rows / cols
    // 0..FM-1 = map coords ri0.., rj0..; zero outside the valid map), into s_xy
    constexpr int kItems = (FM + BR - 1) / BR * FM;
    for (int it = tid; it < kItems; it += kFThreads) {
      const int mg = it / FM, mc = it - mg * FM;
      f2v oa[BR], ob[BR];
      float oc[BR];
#pragma unroll
      for (int j = 0; j < BR; ++j) {
        oa[j] = f2v{0.f, 0.f};
        ob[j] = f2v{0.f, 0.f};
        oc[j] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < K + BR - 1; ++i) {
        const int r = min(BR * mg + i, FI - 1);  // rows past FI only feed discarded outputs
        const f2v a = hA[r][mc], bb = hB[r][mc];
        const float cc = hC[r][mc];
#pragma unroll
        for (int j = 0; j < BR; ++j) {
          const int k = i - j;
          if (k >= 0 && k < K) {
            const float g = kG[k];
            oa[j] = __builtin_elementwise_fma(f2v{g, g}, a, oa[j]);
            ob[j] = __builtin_elementwise_fma(f2v{g, g}, bb, ob[j]);
            oc[j] = __builtin_fmaf(g, cc, oc[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < BR; ++j) {
        const int mr = BR * mg + j, pi = ri0 + mr, pj = rj0 + mc;
        float p0 = 0.f, p1 = 0.f, p2 = 0.f;
        if (pi >= 0 && pi < Hm && pj >= 0 && pj < Wm) {
          const float u1 = oa[j].x, u2 = oa[j].y;
          const float s11 = ob[j].x - u1 * u1, s22 = ob[j].y - u2 * u2, s12 = oc[j] - u1 * u2;
          const float A1 = 2.f * u1 * u2 + C1, A2 = 2.f * s12 + C2;
          const float B1 = u1 * u1 + u2 * u2 + C1, B2 = s11 + s22 + C2;
          const float inv = 1.f / (B1 * B2);
          const float sv = A1 * A2 * inv;
          if (mr >= 2 * R && mr < FM && mc >= 2 * R) ssum += sv;  // the tile's own map pixels
          const float dN = 2.f * u2 * (A2 - A1), dD = 2.f * u1 * (B2 - B1);
          p0 = (dN - sv * dD) * inv;
          p1 = -sv * B1 * inv;
          p2 = 2.f * A1 * inv;
        }
        if (mr < FM) {
          m01[mr][mc] = f2v{p0, p1};
          m2[mr][mc] = p2;
        }
      }
    }
    __syncthreads();
    const bool more = c + 1 < c_end;
    if (more) load(c + 1);
    // ---- C1: horizontal blur of the partials, FM rows x FT columns (the
    // adjoint of the valid correlation: full correlation with the symmetric
    // kernel, see bwd_kernel), into hA
    for (int idx = tid; idx < FM * (FT / kHC); idx += kFThreads) {
      const int jg = idx / FM, r = idx - jg * FM, j0 = jg * kHC;
      f2v v[K + kHC - 1];
      float w[K + kHC - 1];
#pragma unroll
      for (int i = 0; i < K + kHC - 1; ++i) {
        v[i] = m01[r][j0 + i];
        w[i] = m2[r][j0 + i];
      }
#pragma unroll
      for (int o = 0; o < kHC; ++o) {
        f2v a = {0.f, 0.f};
        float cc = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float g = kG[k];
          a = __builtin_elementwise_fma(f2v{g, g}, v[o + k], a);
          cc = __builtin_fmaf(g, w[o + k], cc);
        }
        g01[r][j0 + o] = a;
        g2[r][j0 + o] = cc;
      }
    }
    __syncthreads();
    if (more) stage();  // the next channel's window (s_xy is free: see above)
    // ---- C2: vertical blur onto the tile pixels, gradient out.  (The next
    // channel's pass A rewrites hA, which C2 reads, only after the barrier
    // below.)
    {
      f2v oa[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
      float oc[2] = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < K + 1; ++i) {
        const int r = 2 * gr + i;
        const f2v a = g01[r][gc];
        const float cc = g2[r][gc];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int k = i - j;
          if (k >= 0 && k < K) {
            const float g = kG[k];
            oa[j] = __builtin_elementwise_fma(f2v{g, g}, a, oa[j]);
            oc[j] = __builtin_fmaf(g, cc, oc[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int qi = qi0 + 2 * gr + j, qj = qj0 + gc;
        const f2v v = j ? px1 : px0;
        const float d = v.x - v.y;
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        if (qi < H && qj < W)
          grad[(((int64_t)b * H + qi) * W + qj) * XS + c] =
              cs * (oa[j].x + 2.f * v.x * oa[j].y + v.y * oc[j]) + cl * sgn;
      }
    }
    if (more) __syncthreads();  // the staged window, and C2's reads of hA done
  }
  if (XS > C && cg == CG - 1) {  // the render's other channels: no loss term, zero gradient
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int qi = qi0 + 2 * gr + j, qj = qj0 + gc;
      if (qi < H && qj < W)
        for (int e = C; e < XS; ++e) grad[(((int64_t)b * H + qi) * W + qj) * XS + e] = 0.f;
    }
  }
  ssum = wave_sum(ssum);
  lsum = wave_sum(lsum);
  if (lane == 0) {
    red[0][tid >> 6] = ssum;
    red[1][tid >> 6] = lsum;
  }
  __syncthreads();
  if (tid == 0) {
    float s = 0.f, l = 0.f;
    for (int w = 0; w < kFThreads / 64; ++w) {
      s += red[0][w];
      l += red[1][w];
    }
    partials[2 * ((int64_t)b * ntc + tc)] = s;
    partials[2 * ((int64_t)b * ntc + tc) + 1] = l;
  }
}

// grad = g_loss[0] * unit (float4 where aligned)
__global__ void __launch_bounds__(256) fused_scale_kernel(int64_t n, const float *__restrict__ unit,
                                                         const float *__restrict__ g_loss,
                                                         float *__restrict__ grad) {
  const float g = g_loss[0];
  const int64_t n4 = n >> 2;
  const float4 *u4 = reinterpret_cast<const float4 *>(unit);
  float4 *o4 = reinterpret_cast<float4 *>(grad);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = u4[i];
    o4[i] = make_float4(g * v.x, g * v.y, g * v.z, g * v.w);
  }
  for (int64_t i = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    grad[i] = g * unit[i];
}

}  // namespace ssim
}  // namespace gs

using namespace gs;

static int64_t ssim_map_floats(int B, int H, int W, int C) {
  return (int64_t)B * C * 3 * (int64_t)(H - 10) * (W - 10);
}
static int64_t ssim_blocks(int B, int H, int W, int C) {
  return (int64_t)((W - 10 + 31) / 32) * ((H - 10 + 31) / 32) * B * C;
}
static dim3 ssim_grid(int B, int H, int W, int C, bool map_tiles) {
  const int pad = map_tiles ? 10 : 0;
  return dim3((unsigned)ssim::grid_blocks(((W - pad + 31) / 32) * ((H - pad + 31) / 32), B * C));
}

extern "C" int64_t gsplat_hip_ssim_workspace_bytes(int B, int H, int W, int C) {
  if (H <= 10 || W <= 10) return 0;
  return (int64_t)sizeof(float) * (ssim_map_floats(B, H, W, C) + 2 * ssim_blocks(B, H, W, C));
}

static float n_map(int B, int H, int W, int C) { return (float)B * C * (H - 10) * (W - 10); }
static float n_img(int B, int H, int W, int C) { return (float)B * C * H * W; }

// The forward with all channels of a tile in one workgroup (fwd_c_kernel,
// C = 3; 66 -> 56 us at 1080p against one channel per workgroup, fwd_kernel,
// which other channel counts use).  The same change in the backward (map
// windows of all channels in one round) measured slower, 81 vs 62 us: its
// 99 map values per lane in flight cost occupancy the blur needs.
static int ssim_fwd(int B, int H, int W, int C, const float *img1, const float *img2,
                    float *sums, float *loss, float lam, void *workspace, void *stream) {
  GS_REQUIRE(B > 0 && C > 0 && H > 10 && W > 10,
             "ssim_l1_fwd: images must be larger than the 11x11 window (got %dx%d)", H, W);
  hipStream_t st = (hipStream_t)stream;
  float *maps = reinterpret_cast<float *>(workspace);
  float *partials = maps + ssim_map_floats(B, H, W, C);
  const int n_tiles = ((W - 10 + 31) / 32) * ((H - 10 + 31) / 32);
  if (C == 3) {
    hipLaunchKernelGGL(ssim::fwd_c_kernel<3>, dim3((unsigned)(n_tiles * B)), dim3(256), 0, st, B,
                       H, W, img1, img2, maps, partials);
    hipLaunchKernelGGL(ssim::reduce_partials_kernel, dim3(1), dim3(1024), 0, st, n_tiles * B,
                       partials, sums, loss, lam, n_map(B, H, W, C), n_img(B, H, W, C));
  } else {
    hipLaunchKernelGGL(ssim::fwd_kernel, ssim_grid(B, H, W, C, true), dim3(256), 0, st, B, H, W,
                       C, img1, img2, maps, partials);
    hipLaunchKernelGGL(ssim::reduce_partials_kernel, dim3(1), dim3(1024), 0, st,
                       (int)ssim_blocks(B, H, W, C), partials, sums, loss, lam, n_map(B, H, W, C),
                       n_img(B, H, W, C));
  }
  GS_CHECK_LAUNCH("ssim_l1_fwd");
  return 0;
}

static int ssim_bwd(int B, int H, int W, int C, const float *img1, const float *img2,
                    const void *workspace, const float *dloss, float s_ssim, float s_l1,
                    int l1_index, float *grad_img1, void *stream) {
  GS_REQUIRE(B > 0 && C > 0 && H > 10 && W > 10, "ssim_l1_bwd: bad image size %dx%d", H, W);
  hipLaunchKernelGGL(ssim::bwd_kernel, ssim_grid(B, H, W, C, false), dim3(256), 0, (hipStream_t)stream, B, H, W, C, img1,
                     img2, reinterpret_cast<const float *>(workspace), dloss, s_ssim, s_l1, l1_index,
                     grad_img1);
  GS_CHECK_LAUNCH("ssim_l1_bwd");
  return 0;
}

extern "C" int gsplat_hip_ssim_l1_fwd(int B, int H, int W, int C, const float *img1,
                                      const float *img2, float *sums, void *workspace,
                                      void *stream) {
  return ssim_fwd(B, H, W, C, img1, img2, sums, nullptr, 0.f, workspace, stream);
}

extern "C" int gsplat_hip_ssim_l1_bwd(int B, int H, int W, int C, const float *img1,
                                      const float *img2, const void *workspace,
                                      const float *dloss, float *grad_img1, void *stream) {
  return ssim_bwd(B, H, W, C, img1, img2, workspace, dloss, 1.f / n_map(B, H, W, C),
                  1.f / n_img(B, H, W, C), 1, grad_img1, stream);
}

extern "C" int gsplat_hip_l1_ssim_loss_fwd(int B, int H, int W, int C, const float *img1,
                                           const float *img2, float lam, float *out,
                                           void *workspace, void *stream) {
  GS_REQUIRE(out != nullptr, "l1_ssim_loss_fwd: out is null");
  return ssim_fwd(B, H, W, C, img1, img2, nullptr, out, lam, workspace, stream);
}

extern "C" int gsplat_hip_l1_ssim_loss_bwd(int B, int H, int W, int C, const float *img1,
                                           const float *img2, const void *workspace, float lam,
                                           const float *g_loss, float *grad_img1, void *stream) {
  return ssim_bwd(B, H, W, C, img1, img2, workspace, g_loss, -lam / n_map(B, H, W, C),
                  (1.f - lam) / n_img(B, H, W, C), 0, grad_img1, stream);
}

// ---- loss + unit gradient in one pass (ssim::fused_kernel)
static int64_t fused_tiles(int H, int W) {
  return (int64_t)((W + ssim::FT - 1) / ssim::FT) * ((H + ssim::FT - 1) / ssim::FT);
}

extern "C" int64_t gsplat_hip_l1_ssim_loss_fused_workspace_bytes(int B, int H, int W, int C) {
  if (H <= 10 || W <= 10) return 0;
  return (int64_t)sizeof(float) * 2 * B * fused_tiles(H, W);
}

static int fused_fwd(int B, int H, int W, int C, int XS, const float *img1, const float *img2,
                     const int64_t *img2_index, float lam, float *out, float *grad_unit,
                     void *workspace, float *ring, int64_t ring_len, const int64_t *seq,
                     void *stream) {
  GS_REQUIRE(B > 0 && H > 10 && W > 10,
             "l1_ssim_loss_fused_fwd: images must be larger than the 11x11 window (got %dx%d)", H,
             W);
  GS_REQUIRE(C == 1 || C == 3, "l1_ssim_loss_fused_fwd: C must be 1 or 3 (got %d)", C);
  GS_REQUIRE(out != nullptr && grad_unit != nullptr, "l1_ssim_loss_fused_fwd: null output");
  GS_REQUIRE(XS >= C, "l1_ssim_loss_fused_fwd: pixel stride %d < C = %d", XS, C);
  hipStream_t st = (hipStream_t)stream;
  float *partials = reinterpret_cast<float *>(workspace);
  // one workgroup per tile, all its channels (one channel per workgroup --
  // three times the workgroups at a third of the LDS each -- measured 112-114
  // us either way, M2 805.2 / 809.7 against 813.3 / 811.4 images/s,
  // profiles/r5/b10; removed)
  const int64_t nt = fused_tiles(H, W), per = (nt + 7) / 8;
  const dim3 grid((unsigned)(B * 8 * per));
  const float cs = -lam / n_map(B, H, W, C), cl = (1.f - lam) / n_img(B, H, W, C);
#define GS_FUSED(CC, BR, CPW, XS_)                                                           \
  hipLaunchKernelGGL((ssim::fused_kernel<CC, BR, CPW, XS_>), grid, dim3(ssim::kFThreads), 0, st, \
                     B, H, W, img1, img2, img2_index, cs, cl, grad_unit, partials)
  GS_REQUIRE(XS == C || (C == 3 && XS == 4),
             "l1_ssim_loss_fused_fwd: pixel stride %d with C = %d (supported: C, or 4 with C = 3)",
             XS, C);
  // map rows per pass-B item: 4 for the contiguous RGB images; 2 for an
  // RGB+D render read in place (x stride 4: the 4-row form spilled 25 VGPRs
  // there, 171.5 against 125.3 us; the 2-row form for the contiguous loss
  // measured M2 814.0 / 817.2 against 817.6 / 817.8 images/s, profiles/r5/b22)
  if (C == 3 && XS == 4) {
    GS_FUSED(3, 2, 3, 4);
  } else if (C == 3) {
    GS_FUSED(3, 4, 3, 3);
  } else {
    GS_FUSED(1, 2, 1, 1);
  }
#undef GS_FUSED
  hipLaunchKernelGGL(ssim::reduce_partials_kernel, dim3(1), dim3(1024), 0, st, (int)(B * nt),
                     partials, nullptr, out, lam, n_map(B, H, W, C), n_img(B, H, W, C), ring,
                     ring_len, seq);
  GS_CHECK_LAUNCH("l1_ssim_loss_fused_fwd");
  return 0;
}

extern "C" int gsplat_hip_l1_ssim_loss_fused_fwd(int B, int H, int W, int C, int x_stride,
                                                 const float *img1, const float *img2,
                                                 const int64_t *img2_index, float lam, float *out,
                                                 float *grad_unit, void *workspace, void *stream) {
  return fused_fwd(B, H, W, C, x_stride, img1, img2, img2_index, lam, out, grad_unit, workspace,
                   nullptr, 0, nullptr, stream);
}

extern "C" int gsplat_hip_l1_ssim_loss_fused_fwd_ring(int B, int H, int W, int C, int x_stride,
                                                      const float *img1, const float *img2,
                                                      const int64_t *img2_index, float lam,
                                                      float *out, float *grad_unit,
                                                      void *workspace, float *loss_ring,
                                                      int64_t ring_len, const int64_t *seq_device,
                                                      void *stream) {
  GS_REQUIRE(loss_ring && seq_device && ring_len > 0,
             "l1_ssim_loss_fused_fwd_ring: null ring / step counter or empty ring");
  return fused_fwd(B, H, W, C, x_stride, img1, img2, img2_index, lam, out, grad_unit, workspace,
                   loss_ring, ring_len, seq_device, stream);
}

extern "C" int gsplat_hip_l1_ssim_loss_fused_bwd(int64_t n, const float *grad_unit,
                                                 const float *g_loss, float *grad_img1,
                                                 void *stream) {
  GS_REQUIRE(n >= 0, "l1_ssim_loss_fused_bwd: n < 0");
  if (n == 0) return 0;
  GS_REQUIRE(((uintptr_t)grad_unit & 15) == 0 && ((uintptr_t)grad_img1 & 15) == 0,
             "l1_ssim_loss_fused_bwd: buffers must be 16-byte aligned");
  const int64_t blocks = std::min<int64_t>((n / 4 + 255) / 256 + 1, 4096);
  hipLaunchKernelGGL(ssim::fused_scale_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, n, grad_unit, g_loss, grad_img1);
  GS_CHECK_LAUNCH("l1_ssim_loss_fused_bwd");
  return 0;
}
