// Fused EWA projection (pinhole), forward and backward, for gfx950.
//
// Replaces the reference Triton kernels
//   fused_projection_fwd_kernel  gsplat/triton_impl/fused_projection_fwd.py:16-228
//   fused_projection_bwd_kernel  gsplat/triton_impl/fused_projection_bwd.py:24-363
// and follows their algebra (cam_proj.py, transform.py, quat_scale_to_covar.py,
// util_kernels.py) so that gradients agree within fp32 rounding.
//
// Layout: one lane per (camera, Gaussian); the grid is (ceil(N/256), C) so the
// camera parameters are wave-uniform scalar loads.  Inputs stay AoS as the
// caller holds them ([N,3] means, [N,4] quats, [N,3] scales).
#include "common.h"
#include "geom_adam.h"
#include "../../include/gsplat_hip.h"

namespace gs {

struct Cam {
  M3 R;
  float t[3];
  float fx, fy, cx, cy;
};

GS_INLINE Cam load_cam(const float *__restrict__ viewmats, const float *__restrict__ Ks, int c) {
  Cam k;
  const float *V = viewmats + c * 16;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) k.R.m[i][j] = V[i * 4 + j];
    k.t[i] = V[i * 4 + 3];
  }
  const float *K = Ks + c * 9;
  k.fx = K[0];
  k.fy = K[4];
  k.cx = K[2];
  k.cy = K[5];
  return k;
}

// Covariance in world space: (R S)(R S)^T (quat_scale_to_covar.py:7-64).
GS_INLINE M3 covar_world(const M3 &Rq, float s0, float s1, float s2) {
  M3 RS;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    RS.m[i][0] = Rq.m[i][0] * s0;
    RS.m[i][1] = Rq.m[i][1] * s1;
    RS.m[i][2] = Rq.m[i][2] * s2;
  }
  return mul(RS, transpose(RS));
}

struct ProjOut {
  float mx, my;             // projected mean
  float cxx, cxy, cyy;      // 2D covariance (before blur)
  float Jxx, Jxz, Jyy, Jyz; // Jacobian (clamped screen coordinates)
  bool clamp_x, clamp_y;
};

// Pinhole projection with the 15% screen-margin clamp (cam_proj.py:5-81).
GS_INLINE ProjOut persp(float x, float y, float z, const M3 &Cc, const Cam &k, int W, int H) {
  ProjOut o;
  float iz = 1.f / z;
  float marx = 0.15f * (float)W / k.fx;
  float mary = 0.15f * (float)H / k.fy;
  float lox = -marx - k.cx / k.fx, hix = marx + ((float)W - k.cx) / k.fx;
  float loy = -mary - k.cy / k.fy, hiy = mary + ((float)H - k.cy) / k.fy;
  float sx = x * iz, sy = y * iz;
  o.clamp_x = (sx < lox) | (sx > hix);
  o.clamp_y = (sy < loy) | (sy > hiy);
  sx = fminf(fmaxf(sx, lox), hix);
  sy = fminf(fmaxf(sy, loy), hiy);
  o.Jxx = k.fx * iz;
  o.Jxz = -k.fx * sx * iz;
  o.Jyy = k.fy * iz;
  o.Jyz = -k.fy * sy * iz;
  const float(*c)[3] = Cc.m;
  o.cxx = o.Jxx * c[0][0] * o.Jxx + 2.f * o.Jxx * c[0][2] * o.Jxz + o.Jxz * c[2][2] * o.Jxz;
  o.cxy = o.Jxx * (c[0][1] * o.Jyy + c[0][2] * o.Jyz) + o.Jxz * (c[1][2] * o.Jyy + c[2][2] * o.Jyz);
  o.cyy = o.Jyy * c[1][1] * o.Jyy + 2.f * o.Jyy * c[1][2] * o.Jyz + o.Jyz * c[2][2] * o.Jyz;
  o.mx = k.fx * x * iz + k.cx;
  o.my = k.fy * y * iz + k.cy;
  return o;
}

struct ProjFwdArgs {
  int C, N, W, H;
  float eps2d, near_plane, far_plane, radius_clip;
  const float *means, *quats, *scales, *viewmats, *Ks;
  int32_t *radii;
  float *means2d, *depths, *conics, *comps;  // comps may be null
  // packed mode (projection_ewa_3dgs_packed_fwd): per-block counts of kept
  // (camera, Gaussian) pairs, then their exclusive prefix, in (c, n) order
  int64_t *block_cnt;
  const int64_t *block_off;
  int64_t *camera_ids, *gaussian_ids;
};

// MODE 0: dense [C, N] outputs.  MODE 1: count the kept pairs per block.
// MODE 2: write the kept pairs packed at block_off[block] + rank in block.
template <int MODE>
__global__ void __launch_bounds__(256) projection_fwd_kernel(ProjFwdArgs a) {
  const int c = blockIdx.y;
  const int n_raw = blockIdx.x * blockDim.x + threadIdx.x;
  const Cam k = load_cam(a.viewmats, a.Ks, c);
  if (MODE == 0 && n_raw >= a.N) return;
  const bool in = n_raw < a.N;
  const int n = in ? n_raw : a.N - 1;  // packed modes: every lane reaches the block scan
  const float4 q = *reinterpret_cast<const float4 *>(a.quats + 4 * (size_t)n);
  const float *sp = a.scales + 3 * (size_t)n;
  const float *mp = a.means + 3 * (size_t)n;
  const float s0 = sp[0], s1 = sp[1], s2 = sp[2];
  const float m0 = mp[0], m1 = mp[1], m2 = mp[2];

  const M3 C3 = covar_world(quat_to_rotmat(q.x, q.y, q.z, q.w), s0, s1, s2);
  float mc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    mc[i] = k.R.m[i][0] * m0 + k.R.m[i][1] * m1 + k.R.m[i][2] * m2 + k.t[i];
  const M3 Cc = mul(mul(k.R, C3), transpose(k.R));

  const size_t idx = (size_t)c * a.N + n;
  if (MODE == 0) a.depths[idx] = mc[2];
  bool keep = in & (mc[2] > a.near_plane) & (mc[2] < a.far_plane);

  ProjOut p = persp(mc[0], mc[1], mc[2], Cc, k, a.W, a.H);
  // add blur (util_kernels.py:64-94)
  const float det0 = p.cxx * p.cyy - p.cxy * p.cxy;
  const float bxx = p.cxx + a.eps2d, byy = p.cyy + a.eps2d;
  const float det = bxx * byy - p.cxy * p.cxy;
  keep &= det > 0.f;
  const float inv_det = 1.f / det;
  const float b = 0.5f * (bxx + byy);
  const float v1 = b + sqrtf(fmaxf(0.01f, b * b - det));
  const float r = ceilf(3.f * sqrtf(v1));
  keep &= (r > a.radius_clip) & (p.mx + r > 0.f) & (p.mx - r < (float)a.W) &
          (p.my + r > 0.f) & (p.my - r < (float)a.H);

  if (MODE == 0) {
    a.radii[idx] = keep ? (int32_t)r : 0;
    float2 m2d = keep ? make_float2(p.mx, p.my) : make_float2(0.f, 0.f);
    *reinterpret_cast<float2 *>(a.means2d + 2 * idx) = m2d;
    float *cn = a.conics + 3 * idx;
    cn[0] = keep ? inv_det * byy : 0.f;
    cn[1] = keep ? -inv_det * p.cxy : 0.f;
    cn[2] = keep ? inv_det * bxx : 0.f;
    if (a.comps) a.comps[idx] = keep ? sqrtf(fmaxf(det0 / det, 0.f)) : 0.f;
    return;
  }
  // packed: rank of this pair among the block's kept pairs (wave ballots)
  __shared__ int wave_cnt[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t m = __ballot(keep);
  if (lane == 0) wave_cnt[wid] = __popcll(m);
  __syncthreads();
  const int64_t blk = (int64_t)c * gridDim.x + blockIdx.x;
  if (MODE == 1) {
    if (threadIdx.x == 0) a.block_cnt[blk] = wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
    return;
  }
  if (!keep) return;
  int before = 0;
  for (int w = 0; w < wid; ++w) before += wave_cnt[w];
  const int64_t o = a.block_off[blk] + before +
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  a.camera_ids[o] = c;
  a.gaussian_ids[o] = n;
  a.radii[o] = (int32_t)r;
  *reinterpret_cast<float2 *>(a.means2d + 2 * o) = make_float2(p.mx, p.my);
  a.depths[o] = mc[2];
  float *cn = a.conics + 3 * o;
  cn[0] = inv_det * byy;
  cn[1] = -inv_det * p.cxy;
  cn[2] = inv_det * bxx;
  if (a.comps) a.comps[o] = sqrtf(fmaxf(det0 / det, 0.f));
}

// Exclusive scan of the packed per-block counts in place, total -> total[0]
// (one 1024-lane workgroup walking the C * blocks_per_row counts).
__global__ void __launch_bounds__(1024) packed_scan_kernel(int64_t nb, int64_t *cnt,
                                                           int64_t *total) {
  __shared__ int64_t wave_tot[16];
  __shared__ int64_t chunk_tot;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t carry = 0;
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < nb ? cnt[i] : 0;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wave_tot[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t run = 0;
      for (int w = 0; w < 16; ++w) {
        const int64_t t = wave_tot[w];
        wave_tot[w] = run;
        run += t;
      }
      chunk_tot = run;
    }
    __syncthreads();
    if (i < nb) cnt[i] = carry + wave_tot[wid] + x - v;
    carry += chunk_tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) total[0] = carry;
}

struct ProjBwdArgs {
  int C, N, W, H;
  float eps2d;
  const float *means, *quats, *scales, *viewmats, *Ks;
  const int32_t *radii;
  const float *conics, *comps;                                 // comps may be null
  const float *v_means2d, *v_depths, *v_conics, *v_comps;      // v_depths, v_comps may be null
  float *v_means, *v_quats, *v_scales, *v_viewmats;            // v_viewmats may be null
  int store_mode;  // 1: C == 1, every lane stores its own row (no atomics, no memset)
  // packed inputs (projection_ewa_3dgs_packed_bwd): entry e is the pair
  // (camera_ids[e], gaussian_ids[e]); sparse: per-entry gradient rows [nnz, .]
  const int64_t *camera_ids, *gaussian_ids;
  int64_t nnz;
  int sparse;
  GeomAdam ga;  // projection_bwd_kernel<true>: the geometry Adam instead of the stores
};

// FUSE: the geometry-Adam epilogue (struct GeomAdam; C == 1, store mode).
// Its lane's optimizer rows (33 floats) and gradient inputs are loaded at
// the start, so their latency overlaps the gradient algebra instead of
// following it group by group (the stores of one group could alias the next
// group's loads as far as the compiler knows): 93.6 us as an epilogue
// issuing them after the algebra at M2 (profiles/r5/).
template <bool FUSE = false>
__global__ void __launch_bounds__(256) projection_bwd_kernel(ProjBwdArgs a) {
  const bool packed = a.camera_ids != nullptr;
  int c, n;
  size_t idx;
  bool valid;
  if (packed) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    valid = e < a.nnz;
    c = valid ? (int)a.camera_ids[e] : 0;
    n = valid ? (int)a.gaussian_ids[e] : 0;
    idx = valid ? (size_t)e : 0;
  } else {
    c = blockIdx.y;
    n = blockIdx.x * blockDim.x + threadIdx.x;
    idx = (size_t)c * a.N + n;
    valid = (n < a.N) && (a.radii[idx] > 0);
  }
  const Cam k = load_cam(a.viewmats, a.Ks, c);

  // FUSE: the lane's rows of the four geometry groups -- parameters, both
  // moments -- and the other gradient terms, in flight from here
  constexpr int kG = 11;  // means 3 | log-scales 3 | quats 4 | logits 1
  float gp[kG], gm[kG], gv[kG], gvd[3] = {0.f, 0.f, 0.f}, gvo = 0.f, gop = 0.f, gsc[3];
  const bool fuse_on = FUSE && n < a.N && !(a.ga.skip && *a.ga.skip);
  if (FUSE && fuse_on) {
    const GeomAdam &ga = a.ga;
    const size_t i = (size_t)n;
    constexpr int off[4] = {0, 3, 6, 10}, wid[4] = {3, 3, 4, 1};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < wid[q]; ++e) {
        gp[off[q] + e] = ga.p[q][wid[q] * i + e];
        gm[off[q] + e] = ga.m[q][wid[q] * i + e];
        gv[off[q] + e] = ga.v[q][wid[q] * i + e];
      }
    if (ga.v_dirs) {
#pragma unroll
      for (int j = 0; j < 3; ++j) gvd[j] = ga.v_dirs[3 * i + j];
    }
    if (ga.v_opac) {
      gvo = ga.v_opac[i];
      gop = ga.opac[i];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) gsc[j] = a.scales[3 * i + j];
  }

  float vR[3][3] = {{0.f}}, vt[3] = {0.f, 0.f, 0.f};
  float vm[3] = {0.f, 0.f, 0.f}, vq[4] = {0.f, 0.f, 0.f, 0.f}, vs[3] = {0.f, 0.f, 0.f};

  if (valid) {
    // ---- conic inverse VJP (util_kernels.py:27-61); v_conic_xy halved
    const float *cn = a.conics + 3 * idx;
    const float ca = cn[0], cb = cn[1], cc = cn[2];
    const float *vc = a.v_conics + 3 * idx;
    const float va = vc[0], vb = 0.5f * vc[1], vcc = vc[2];
    float dxx = -(ca * va * ca + cb * vcc * cb + 2.f * cb * vb * ca);
    float dxy = -(ca * vb * cc + cb * vb * cb + cb * vcc * cc + ca * va * cb);
    float dyy = -(cb * va * cb + cc * vcc * cc + 2.f * cc * vb * cb);
    if (a.comps) {  // blur VJP (util_kernels.py:97-144)
      const float cp = a.comps[idx], vcp = a.v_comps[idx];
      const float det_i = ca * cc - cb * cb;
      const float Da = 0.5f * vcp / (cp + 1e-6f);
      const float oma = 1.f - cp * cp;
      dxx += Da * (oma * ca - a.eps2d * det_i);
      dxy += Da * (oma * cb);
      dyy += Da * (oma * cc - a.eps2d * det_i);
    }
    // ---- recompute the forward intermediates
    const float4 q = *reinterpret_cast<const float4 *>(a.quats + 4 * (size_t)n);
    const float *sp = a.scales + 3 * (size_t)n;
    const float *mp = a.means + 3 * (size_t)n;
    const float s0 = sp[0], s1 = sp[1], s2 = sp[2];
    const float m[3] = {mp[0], mp[1], mp[2]};
    const M3 Rq = quat_to_rotmat(q.x, q.y, q.z, q.w);
    const M3 C3 = covar_world(Rq, s0, s1, s2);
    float mc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      mc[i] = k.R.m[i][0] * m[0] + k.R.m[i][1] * m[1] + k.R.m[i][2] * m[2] + k.t[i];
    const M3 Cc = mul(mul(k.R, C3), transpose(k.R));
    const ProjOut p = persp(mc[0], mc[1], mc[2], Cc, k, a.W, a.H);
    const float iz = 1.f / mc[2];

    // ---- perspective VJP (cam_proj.py:84-242)
    M3 v3;
    v3.m[0][0] = p.Jxx * dxx * p.Jxx;
    v3.m[1][1] = p.Jyy * dyy * p.Jyy;
    v3.m[2][2] = p.Jxz * dxx * p.Jxz + p.Jyz * dyy * p.Jyz + 2.f * p.Jyz * dxy * p.Jxz;
    v3.m[0][1] = v3.m[1][0] = p.Jxx * dxy * p.Jyy;
    v3.m[0][2] = v3.m[2][0] = p.Jxx * dxx * p.Jxz + p.Jxx * dxy * p.Jyz;
    v3.m[1][2] = v3.m[2][1] = p.Jyy * dxy * p.Jxz + p.Jyy * dyy * p.Jyz;

    const float vm2x = a.v_means2d[2 * idx], vm2y = a.v_means2d[2 * idx + 1];
    float vmc[3];
    vmc[0] = p.Jxx * vm2x;
    vmc[1] = p.Jyy * vm2y;
    vmc[2] = p.Jxz * vm2x + p.Jyz * vm2y;
    const float(*cm)[3] = Cc.m;
    const float Jc_xx = p.Jxx * cm[0][0] + p.Jxz * cm[0][2];
    const float Jc_xy = p.Jxx * cm[0][1] + p.Jxz * cm[1][2];
    const float Jc_xz = p.Jxx * cm[0][2] + p.Jxz * cm[2][2];
    const float Jc_yx = p.Jyy * cm[0][1] + p.Jyz * cm[0][2];
    const float Jc_yy = p.Jyy * cm[1][1] + p.Jyz * cm[1][2];
    const float Jc_yz = p.Jyy * cm[1][2] + p.Jyz * cm[2][2];
    const float vJxx = 2.f * (dxx * Jc_xx + dxy * Jc_yx);
    const float vJxz = 2.f * (dxx * Jc_xz + dxy * Jc_yz);
    const float vJyy = 2.f * (dxy * Jc_xy + dyy * Jc_yy);
    const float vJyz = 2.f * (dxy * Jc_xz + dyy * Jc_yz);
    const float iz2 = iz * iz;
    vmc[0] += p.clamp_x ? 0.f : -vJxz * k.fx * iz2;
    vmc[1] += p.clamp_y ? 0.f : -vJyz * k.fy * iz2;
    float tmp = vJxx * p.Jxx + vJyy * p.Jyy + 2.f * (vJxz * p.Jxz + vJyz * p.Jyz);
    tmp -= p.clamp_x ? vJxz * p.Jxz : 0.f;
    tmp -= p.clamp_y ? vJyz * p.Jyz : 0.f;
    vmc[2] -= iz * tmp;
    if (a.v_depths) vmc[2] += a.v_depths[idx];  // null: depths unused downstream

    // ---- world->camera VJP (transform.py:38-119, 184-297)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      vm[j] = k.R.m[0][j] * vmc[0] + k.R.m[1][j] * vmc[1] + k.R.m[2][j] * vmc[2];
    const M3 vSR = mul(v3, k.R);
    const M3 vC3 = mul(transpose(k.R), vSR);
    if (a.v_viewmats) {
      const M3 vRc = mul(vSR, C3);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        vt[i] = vmc[i];
#pragma unroll
        for (int j = 0; j < 3; ++j) vR[i][j] = vmc[i] * m[j] + 2.f * vRc.m[i][j];
      }
    }
    // ---- covariance VJP (quat_scale_to_covar.py:67-144)
    M3 twoRS;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      twoRS.m[i][0] = 2.f * Rq.m[i][0] * s0;
      twoRS.m[i][1] = 2.f * Rq.m[i][1] * s1;
      twoRS.m[i][2] = 2.f * Rq.m[i][2] * s2;
    }
    const M3 dRS = mul(vC3, twoRS);
    M3 dR;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      dR.m[i][0] = dRS.m[i][0] * s0;
      dR.m[i][1] = dRS.m[i][1] * s1;
      dR.m[i][2] = dRS.m[i][2] * s2;
    }
    quat_to_rotmat_vjp(q.x, q.y, q.z, q.w, dR, vq);
#pragma unroll
    for (int j = 0; j < 3; ++j)
      vs[j] = Rq.m[0][j] * dRS.m[0][j] + Rq.m[1][j] * dRS.m[1][j] + Rq.m[2][j] * dRS.m[2][j];
  }
  // the gradients are formed once, here, for every epilogue below: without
  // this the compiler may duplicate their algebra into the branches and
  // contract the multiply-adds differently per branch (the geometry-Adam
  // epilogue then differs from the stored gradients in the last bit)
  asm volatile("" : "+v"(vm[0]), "+v"(vm[1]), "+v"(vm[2]), "+v"(vq[0]), "+v"(vq[1]),
               "+v"(vq[2]), "+v"(vq[3]), "+v"(vs[0]), "+v"(vs[1]), "+v"(vs[2]));

  if (a.sparse) {
    if (valid) {  // COO values, one row per packed entry
      float *o = a.v_means + 3 * idx;
      o[0] = vm[0]; o[1] = vm[1]; o[2] = vm[2];
      *reinterpret_cast<float4 *>(a.v_quats + 4 * idx) = make_float4(vq[0], vq[1], vq[2], vq[3]);
      o = a.v_scales + 3 * idx;
      o[0] = vs[0]; o[1] = vs[1]; o[2] = vs[2];
    }
  } else if (FUSE) {
    if (fuse_on) {
      const GeomAdam &ga = a.ga;
      const size_t i = (size_t)n;
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
      // means: v_means + v_dirs (autograd's sum); log-scales: exp's VJP with
      // the activated scale (the input `scales`); quats; logits: sigmoid's VJP
#pragma unroll
      for (int j = 0; j < 3; ++j) g[j] = ga.v_dirs ? vm[j] + gvd[j] : vm[j];
#pragma unroll
      for (int j = 0; j < 3; ++j) g[3 + j] = vs[j] * gsc[j];
#pragma unroll
      for (int j = 0; j < 4; ++j) g[6 + j] = vq[j];
      g[10] = ga.v_opac ? gvo * (1.f - gop) * gop : 0.f;
      // each gradient its own rounded value: no VJP multiply may be
      // contracted into adam_update's subtraction (adam::step_kernel forms
      // them through a runtime select, which keeps them apart there)
#pragma unroll
      for (int e = 0; e < kG; ++e) asm volatile("" : "+v"(g[e]));
      constexpr int grp[kG] = {0, 0, 0, 1, 1, 1, 2, 2, 2, 2, 3};
#pragma unroll
      for (int e = 0; e < kG; ++e)
        adam_update(gp[e], g[e], gm[e], gv[e], ga.b1, ga.b2, ga.eps, ss[grp[e]], ib);
      constexpr int off[4] = {0, 3, 6, 10}, wid[4] = {3, 3, 4, 1};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < wid[q]; ++e) {
          ga.p[q][wid[q] * i + e] = gp[off[q] + e];
          ga.m[q][wid[q] * i + e] = gm[off[q] + e];
          ga.v[q][wid[q] * i + e] = gv[off[q] + e];
        }
    }
  } else if (a.store_mode) {
    if (n < a.N) {
      float *o = a.v_means + 3 * (size_t)n;
      o[0] = vm[0]; o[1] = vm[1]; o[2] = vm[2];
      *reinterpret_cast<float4 *>(a.v_quats + 4 * (size_t)n) = make_float4(vq[0], vq[1], vq[2], vq[3]);
      o = a.v_scales + 3 * (size_t)n;
      o[0] = vs[0]; o[1] = vs[1]; o[2] = vs[2];
    }
  } else if (valid) {
#pragma unroll
    for (int j = 0; j < 3; ++j) atomic_add_f32(a.v_means + 3 * (size_t)n + j, vm[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) atomic_add_f32(a.v_quats + 4 * (size_t)n + j, vq[j]);
#pragma unroll
    for (int j = 0; j < 3; ++j) atomic_add_f32(a.v_scales + 3 * (size_t)n + j, vs[j]);
  }

  if (a.v_viewmats && packed) {
    // entries are camera-major: a wave spans one camera except at camera
    // boundaries, where its lanes add their partials one by one
    const int lane = threadIdx.x & 63;
    float v[12];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) v[i * 4 + j] = vR[i][j];
      v[i * 4 + 3] = vt[i];
    }
    const int c0 = __shfl(c, 0, 64);
    if (__ballot(valid && c != c0) == 0) {
#pragma unroll
      for (int e = 0; e < 12; ++e) v[e] = wave_sum(v[e]);
      if (lane == 0)
        for (int e = 0; e < 12; ++e)
          if (v[e] != 0.f) atomic_add_f32(a.v_viewmats + c0 * 16 + e, v[e]);
    } else if (valid) {
      for (int e = 0; e < 12; ++e)
        if (v[e] != 0.f) atomic_add_f32(a.v_viewmats + c * 16 + e, v[e]);
    }
  } else if (a.v_viewmats) {
    // block reduction of the 12 viewmat partials: wave butterfly, then LDS
    __shared__ float red[4][12];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float v[12];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) v[i * 4 + j] = vR[i][j];
      v[i * 4 + 3] = vt[i];
    }
#pragma unroll
    for (int e = 0; e < 12; ++e) v[e] = wave_sum(v[e]);
    if (lane == 0) {
#pragma unroll
      for (int e = 0; e < 12; ++e) red[wid][e] = v[e];
    }
    __syncthreads();
    if (threadIdx.x < 12) {
      float s = 0.f;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w][threadIdx.x];
      if (s != 0.f) atomic_add_f32(a.v_viewmats + c * 16 + threadIdx.x, s);
    }
  }
}

}  // namespace gs

using namespace gs;

extern "C" int gsplat_hip_projection_fwd(int C, int N, const float *means, const float *quats,
                                         const float *scales, const float *viewmats,
                                         const float *Ks, int width, int height, float eps2d,
                                         float near_plane, float far_plane, float radius_clip,
                                         int32_t *radii, float *means2d, float *depths,
                                         float *conics, float *compensations, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "projection_fwd: negative sizes C=%d N=%d", C, N);
  if (C == 0 || N == 0) return 0;
  GS_REQUIRE(means && quats && scales && viewmats && Ks && radii && means2d && depths && conics,
             "projection_fwd: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)means2d & 7) == 0,
             "projection_fwd: quats must be 16-B aligned, means2d 8-B aligned");
  ProjFwdArgs a{C, N, width, height, eps2d, near_plane, far_plane, radius_clip,
                means, quats, scales, viewmats, Ks, radii, means2d, depths, conics, compensations};
  dim3 grid((N + 255) / 256, C);
  hipLaunchKernelGGL(projection_fwd_kernel<0>, grid, dim3(256), 0, (hipStream_t)stream, a);
  GS_CHECK_LAUNCH("projection_fwd");
  return 0;
}

extern "C" int gsplat_hip_projection_bwd(
    int C, int N, const float *means, const float *quats, const float *scales,
    const float *viewmats, const float *Ks, int width, int height, float eps2d,
    const int32_t *radii, const float *conics, const float *compensations,
    const float *v_means2d, const float *v_depths, const float *v_conics,
    const float *v_compensations, float *v_means, float *v_quats, float *v_scales,
    float *v_viewmats, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "projection_bwd: negative sizes C=%d N=%d", C, N);
  hipStream_t st = (hipStream_t)stream;
  if (v_viewmats && C > 0) GS_HIP(gs::zero_async(v_viewmats, sizeof(float) * 16 * C, st));
  if (N == 0) return 0;
  if (C == 0) {
    GS_HIP(gs::zero_async(v_means, sizeof(float) * 3 * N, st));
    GS_HIP(gs::zero_async(v_quats, sizeof(float) * 4 * N, st));
    GS_HIP(gs::zero_async(v_scales, sizeof(float) * 3 * N, st));
    return 0;
  }
  GS_REQUIRE(!compensations == !v_compensations,
             "projection_bwd: compensations and v_compensations must both be given or both null");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)v_quats & 15) == 0,
             "projection_bwd: quats / v_quats must be 16-B aligned");
  const int store_mode = (C == 1);
  if (!store_mode) {
    GS_HIP(gs::zero_async(v_means, sizeof(float) * 3 * N, st));
    GS_HIP(gs::zero_async(v_quats, sizeof(float) * 4 * N, st));
    GS_HIP(gs::zero_async(v_scales, sizeof(float) * 3 * N, st));
  }
  ProjBwdArgs a{C, N, width, height, eps2d, means, quats, scales, viewmats, Ks, radii, conics,
                compensations, v_means2d, v_depths, v_conics, v_compensations, v_means, v_quats,
                v_scales, v_viewmats, store_mode};
  dim3 grid((N + 255) / 256, C);
  hipLaunchKernelGGL(projection_bwd_kernel<false>, grid, dim3(256), 0, st, a);
  GS_CHECK_LAUNCH("projection_bwd");
  return 0;
}

// gsplat_hip_projection_bwd with the geometry groups' Adam step fused in
// (ABI 31, see struct GeomAdam): C == 1; params / exp_avgs / exp_avg_sqs are
// [means, log_scales, quats, logits]; lrs[4] with the 1-based step, or
// hyper_device f32[8] = (lr_i / (1 - beta1^t), 1 / sqrt(1 - beta2^t)) per
// group in that order (then lrs / step are unused); skip_device may be NULL.
extern "C" int gsplat_hip_projection_bwd_adam(
    int N, const float *means, const float *quats, const float *scales, const float *viewmats,
    const float *Ks, int width, int height, float eps2d, const int32_t *radii,
    const float *conics, const float *v_means2d, const float *v_depths, const float *v_conics,
    const float *v_dirs, const float *v_opac, const float *opac, float *const *params,
    float *const *exp_avgs, float *const *exp_avg_sqs, const float *lrs, float beta1,
    float beta2, float eps, int step, const float *hyper_device, const int32_t *skip_device,
    void *stream) {
  GS_REQUIRE(N >= 0, "projection_bwd_adam: negative N=%d", N);
  if (N == 0) return 0;
  GS_REQUIRE(params && exp_avgs && exp_avg_sqs, "projection_bwd_adam: null group arrays");
  GS_REQUIRE(hyper_device || (lrs && step >= 1), "projection_bwd_adam: lrs and step >= 1, or hyper");
  GS_REQUIRE(!v_opac || opac, "projection_bwd_adam: v_opac needs opac");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0, "projection_bwd_adam: quats must be 16-B aligned");
  GeomAdam ga{};
  for (int k = 0; k < 4; ++k) {
    GS_REQUIRE(params[k] && exp_avgs[k] && exp_avg_sqs[k],
               "projection_bwd_adam: null parameter / moment of group %d", k);
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

  if (!hyper_device) {  // gsplat_hip_adam_step's host arithmetic
    const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
    for (int k = 0; k < 4; ++k) ga.ss[k] = (float)(lrs[k] / bc1);
    ga.ib = (float)(1.0 / sqrt(bc2));
  }
  ProjBwdArgs a{1, N, width, height, eps2d, means, quats, scales, viewmats, Ks, radii, conics,
                nullptr, v_means2d, v_depths, v_conics, nullptr, nullptr, nullptr, nullptr,
                nullptr, 1};
  a.ga = ga;
  hipLaunchKernelGGL(projection_bwd_kernel<true>, dim3((N + 255) / 256, 1), dim3(256), 0,
                     (hipStream_t)stream, a);
  GS_CHECK_LAUNCH("projection_bwd_adam");
  return 0;
}

namespace gs {
// the packed-count scan, shared with the 2DGS packed projection (surfel.hip)
void launch_packed_scan(int64_t nb, int64_t *cnt, int64_t *total, hipStream_t st) {
  hipLaunchKernelGGL(packed_scan_kernel, dim3(1), dim3(1024), 0, st, nb, cnt, total);
}
}  // namespace gs

// ------------------------------------------------------------------ packed --
// projection_ewa_3dgs_packed_fwd (gsplat/cuda/csrc/ProjectionEWA3DGSPacked.cu:17-244):
// a counting pass, a scan of the per-block counts, and a pass that recomputes
// and writes the kept (camera, Gaussian) pairs in (camera, Gaussian) order.
extern "C" int64_t gsplat_hip_projection_packed_workspace_bytes(int C, int N) {
  const int64_t nb = (int64_t)C * ((N + 255) / 256);
  return (nb + 1) * (int64_t)sizeof(int64_t);
}

extern "C" int gsplat_hip_projection_packed_count(int C, int N, const float *means,
                                                  const float *quats, const float *scales,
                                                  const float *viewmats, const float *Ks,
                                                  int width, int height, float eps2d,
                                                  float near_plane, float far_plane,
                                                  float radius_clip, void *workspace,
                                                  int64_t *nnz_device, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "projection_packed_count: negative sizes C=%d N=%d", C, N);
  hipStream_t st = (hipStream_t)stream;
  if (C == 0 || N == 0) {
    GS_HIP(gs::zero_async(nnz_device, sizeof(int64_t), st));
    return 0;
  }
  GS_REQUIRE(means && quats && scales && viewmats && Ks && workspace && nnz_device,
             "projection_packed_count: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0, "projection_packed_count: quats must be 16-B aligned");
  ProjFwdArgs a{C, N, width, height, eps2d, near_plane, far_plane, radius_clip,
                means, quats, scales, viewmats, Ks, nullptr, nullptr, nullptr, nullptr, nullptr};
  a.block_cnt = reinterpret_cast<int64_t *>(workspace);
  dim3 grid((N + 255) / 256, C);
  hipLaunchKernelGGL(projection_fwd_kernel<1>, grid, dim3(256), 0, st, a);
  hipLaunchKernelGGL(packed_scan_kernel, dim3(1), dim3(1024), 0, st,
                     (int64_t)grid.x * grid.y, a.block_cnt, nnz_device);
  GS_CHECK_LAUNCH("projection_packed_count");
  return 0;
}

extern "C" int gsplat_hip_projection_packed_fwd(
    int C, int N, const float *means, const float *quats, const float *scales,
    const float *viewmats, const float *Ks, int width, int height, float eps2d,
    float near_plane, float far_plane, float radius_clip, const void *workspace,
    int64_t *camera_ids, int64_t *gaussian_ids, int32_t *radii, float *means2d, float *depths,
    float *conics, float *compensations, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "projection_packed_fwd: negative sizes C=%d N=%d", C, N);
  if (C == 0 || N == 0) return 0;
  GS_REQUIRE(means && quats && scales && viewmats && Ks && workspace && camera_ids &&
                 gaussian_ids && radii && means2d && depths && conics,
             "projection_packed_fwd: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)means2d & 7) == 0,
             "projection_packed_fwd: quats must be 16-B aligned, means2d 8-B aligned");
  ProjFwdArgs a{C, N, width, height, eps2d, near_plane, far_plane, radius_clip,
                means, quats, scales, viewmats, Ks, radii, means2d, depths, conics, compensations};
  a.block_off = reinterpret_cast<const int64_t *>(workspace);
  a.camera_ids = camera_ids;
  a.gaussian_ids = gaussian_ids;
  dim3 grid((N + 255) / 256, C);
  hipLaunchKernelGGL(projection_fwd_kernel<2>, grid, dim3(256), 0, (hipStream_t)stream, a);
  GS_CHECK_LAUNCH("projection_packed_fwd");
  return 0;
}

// projection_ewa_3dgs_packed_bwd (ProjectionEWA3DGSPacked.cu:348-630): one lane
// per packed entry; dense [N, .] gradients by atomics, or (sparse_grad) one
// row per entry for the COO gradients of _wrapper.py:1127-1170.
extern "C" int gsplat_hip_projection_packed_bwd(
    int C, int N, int64_t nnz, const float *means, const float *quats, const float *scales,
    const float *viewmats, const float *Ks, int width, int height, float eps2d,
    const int64_t *camera_ids, const int64_t *gaussian_ids, const float *conics,
    const float *compensations, const float *v_means2d, const float *v_depths,
    const float *v_conics, const float *v_compensations, int sparse_grad, float *v_means,
    float *v_quats, float *v_scales, float *v_viewmats, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0 && nnz >= 0, "projection_packed_bwd: negative sizes");
  hipStream_t st = (hipStream_t)stream;
  if (v_viewmats && C > 0) GS_HIP(gs::zero_async(v_viewmats, sizeof(float) * 16 * C, st));
  if (!sparse_grad && N > 0) {
    GS_HIP(gs::zero_async(v_means, sizeof(float) * 3 * N, st));
    GS_HIP(gs::zero_async(v_quats, sizeof(float) * 4 * N, st));
    GS_HIP(gs::zero_async(v_scales, sizeof(float) * 3 * N, st));
  }
  if (nnz == 0) return 0;
  GS_REQUIRE(!compensations == !v_compensations,
             "projection_packed_bwd: compensations and v_compensations must both be given or "
             "both null");
  GS_REQUIRE(camera_ids && gaussian_ids && conics && v_means2d && v_conics && v_means && v_quats &&
                 v_scales,
             "projection_packed_bwd: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)v_quats & 15) == 0,
             "projection_packed_bwd: quats / v_quats must be 16-B aligned");
  ProjBwdArgs a{C, N, width, height, eps2d, means, quats, scales, viewmats, Ks, nullptr, conics,
                compensations, v_means2d, v_depths, v_conics, v_compensations, v_means, v_quats,
                v_scales, v_viewmats, 0};
  a.camera_ids = camera_ids;
  a.gaussian_ids = gaussian_ids;
  a.nnz = nnz;
  a.sparse = sparse_grad;
  hipLaunchKernelGGL(projection_bwd_kernel<false>, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, st,
                     a);
  GS_CHECK_LAUNCH("projection_packed_bwd");
  return 0;
}
