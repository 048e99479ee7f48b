// 2DGS (surfel) hot path for gfx950: ray-splat projection and the surfel
// rasterizer, forward and backward.
//
// Replaces the reference CUDA kernels (hieu1999210/gsplat-triton)
//   projection_2dgs_fused_fwd_kernel   gsplat/cuda/csrc/Projection2DGSFused.cu:17-238
//   projection_2dgs_fused_bwd_kernel   gsplat/cuda/csrc/Projection2DGSFused.cu:319-457
//     (+ compute_ray_transforms_aabb_vjp, gsplat/cuda/csrc/Projection2DGS.cuh:10-87)
//   rasterize_to_pixels_2dgs_fwd_kernel gsplat/cuda/csrc/RasterizeToPixels2DGSFwd.cu:18-452
//   rasterize_to_pixels_2dgs_bwd_kernel gsplat/cuda/csrc/RasterizeToPixels2DGSBwd.cu:16-700
// with the same per-pixel algebra, on a CDNA4 mapping:
//
//  * projection: one lane per (camera, surfel), grid (ceil(N/256), C) so the
//    camera is a wave-uniform scalar load; the backward stores its gradients
//    (atomics only when several cameras share a surfel).
//  * rasterizer: a workgroup per tile, each wave64 owns 64 consecutive pixels
//    of the tile (a 16x4 strip of a 16x16 tile) and walks the tile's isects on
//    its own: the lanes gather 64 records into a per-wave LDS queue, then every
//    lane composites its pixel against the queue with LDS broadcast reads.  No
//    workgroup barriers, and a wave stops as soon as its 64 pixels are
//    saturated.  The forward keeps the next batch's gather in flight while it
//    composites the current one.
//  * backward: per (record, wave) the D + 15 gradient fields are summed over
//    the 64 lanes with reduce_scatter (wave_ops.h) and 16 lanes add the totals
//    into the surfel's packed gradient row with one coalesced fp32 atomic;
//    unpack_kernel scatters the rows into the autograd tensors and forms the
//    densification gradient.
#include "common.h"
#include "geom_adam.h"
#include "wave_ops.h"
#include "surfel_cull.h"
#include "../../include/gsplat_hip.h"

namespace gs {
namespace surfel {

constexpr float kAlphaMax = 0.999f;
constexpr float kTMin = 1e-4f;
constexpr float kFilterInvSquare = 2.f;  // FILTER_INV_SQUARE_2DGS, Rasterization.h:11
constexpr float kLog2e = 1.4426950408889634f;

// ------------------------------------------------------------- projection
struct ProjFwdArgs {
  int C, N, W, H;
  float near_plane, far_plane, radius_clip;
  const float *means, *quats, *scales, *viewmats, *Ks;
  int32_t *radii;
  float *means2d, *depths, *ray_transforms, *normals;
  // packed mode (projection_2dgs_packed_fwd, Projection2DGSPacked.cu:17-205):
  // per-block counts of kept (camera, surfel) pairs, then their exclusive
  // prefix, in (c, n) order
  int64_t *block_cnt;
  const int64_t *block_off;
  int64_t *camera_ids, *gaussian_ids;
};

struct Cam {
  M3 R;
  float t[3], fx, fy, cx, cy;
};

GS_INLINE Cam load_cam(const float *__restrict__ viewmats, const float *__restrict__ Ks, int c) {
  Cam k;
  const float *V = viewmats + 16 * c;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) k.R.m[i][j] = V[4 * i + j];
    k.t[i] = V[4 * i + 3];
  }
  const float *K = Ks + 9 * c;  // the reference reads K[0], K[2], K[4], K[5] only
  k.fx = K[0];
  k.cx = K[2];
  k.fy = K[4];
  k.cy = K[5];
  return k;
}

// Camera-space surfel: mean, the two scaled tangent axes and the normal axis
// (columns of R_cw * R(q) * diag(s0, s1, 1), Projection2DGSFused.cu:164-167).
struct Frame {
  float mc[3], t0[3], t1[3], nz[3];
  M3 Rq;
};

GS_INLINE Frame surfel_frame(const Cam &k, const float *m, float4 q, float s0, float s1) {
  Frame f;
  f.Rq = quat_to_rotmat(q.x, q.y, q.z, q.w);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    f.mc[i] = k.R.m[i][0] * m[0] + k.R.m[i][1] * m[1] + k.R.m[i][2] * m[2] + k.t[i];
    float a = 0.f, b = 0.f, c = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      a += k.R.m[i][j] * f.Rq.m[j][0];
      b += k.R.m[i][j] * f.Rq.m[j][1];
      c += k.R.m[i][j] * f.Rq.m[j][2];
    }
    f.t0[i] = a * s0;
    f.t1[i] = b * s1;
    f.nz[i] = c;
  }
  return f;
}

// MODE 0: dense [C, N] outputs.  MODE 1: count the kept pairs per block.
// MODE 2: write the kept pairs packed at block_off[block] + rank in block.
template <int MODE>
__global__ void __launch_bounds__(256) proj_fwd_kernel(ProjFwdArgs a) {
  const int c = blockIdx.y;
  const int n_raw = blockIdx.x * blockDim.x + threadIdx.x;
  const Cam k = load_cam(a.viewmats, a.Ks, c);
  if (MODE == 0 && n_raw >= a.N) return;
  const bool in = n_raw < a.N;
  const int n = in ? n_raw : a.N - 1;  // packed modes: every lane reaches the block scan
  const size_t idx = (size_t)c * a.N + n;
  const float4 q = *reinterpret_cast<const float4 *>(a.quats + 4 * (size_t)n);
  const float *sp = a.scales + 3 * (size_t)n;
  const Frame f = surfel_frame(k, a.means + 3 * (size_t)n, q, sp[0], sp[1]);
  if (MODE == 0) a.depths[idx] = f.mc[2];

  // rows of K * [t0 | t1 | mc] (the ray transform, M0/M1/M2 of the reference)
  float M[9];
  M[0] = k.fx * f.t0[0] + k.cx * f.t0[2];
  M[1] = k.fx * f.t1[0] + k.cx * f.t1[2];
  M[2] = k.fx * f.mc[0] + k.cx * f.mc[2];
  M[3] = k.fy * f.t0[1] + k.cy * f.t0[2];
  M[4] = k.fy * f.t1[1] + k.cy * f.t1[2];
  M[5] = k.fy * f.mc[1] + k.cy * f.mc[2];
  M[6] = f.t0[2];
  M[7] = f.t1[2];
  M[8] = f.mc[2];

  bool keep = in && !(f.mc[2] < a.near_plane || f.mc[2] > a.far_plane);
  // AABB from the (1, 1, -1) corner (Projection2DGSFused.cu:200-219)
  const float dist = M[6] * M[6] + M[7] * M[7] - M[8] * M[8];
  keep &= dist != 0.f;
  const float fi = 1.f / dist;
  const float mx = (fi * M[0]) * M[6] + (fi * M[1]) * M[7] + (-fi * M[2]) * M[8];
  const float my = (fi * M[3]) * M[6] + (fi * M[4]) * M[7] + (-fi * M[5]) * M[8];
  const float ex = mx * mx - ((fi * M[0]) * M[0] + (fi * M[1]) * M[1] + (-fi * M[2]) * M[2]);
  const float ey = my * my - ((fi * M[3]) * M[3] + (fi * M[4]) * M[4] + (-fi * M[5]) * M[5]);
  const float radius = ceilf(3.f * sqrtf(fmaxf(1e-4f, fmaxf(ex, ey))));
  keep &= radius > a.radius_clip;
  keep &= !(mx + radius <= 0.f || mx - radius >= (float)a.W || my + radius <= 0.f ||
            my - radius >= (float)a.H);

  const float sgn = -(f.nz[0] * f.mc[0] + f.nz[1] * f.mc[1] + f.nz[2] * f.mc[2]) > 0.f ? 1.f : -1.f;
  if (MODE == 0) {
    a.radii[idx] = keep ? (int32_t)radius : 0;
    *reinterpret_cast<float2 *>(a.means2d + 2 * idx) = keep ? make_float2(mx, my) : make_float2(0.f, 0.f);
    float *rt = a.ray_transforms + 9 * idx;
#pragma unroll
    for (int i = 0; i < 9; ++i) rt[i] = keep ? M[i] : 0.f;
    float *nr = a.normals + 3 * idx;
#pragma unroll
    for (int i = 0; i < 3; ++i) nr[i] = keep ? sgn * f.nz[i] : 0.f;
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
  a.radii[o] = (int32_t)radius;
  *reinterpret_cast<float2 *>(a.means2d + 2 * o) = make_float2(mx, my);
  a.depths[o] = f.mc[2];
  float *rt = a.ray_transforms + 9 * o;
#pragma unroll
  for (int i = 0; i < 9; ++i) rt[i] = M[i];
  float *nr = a.normals + 3 * o;
#pragma unroll
  for (int i = 0; i < 3; ++i) nr[i] = sgn * f.nz[i];
}

struct ProjBwdArgs {
  int C, N;
  const float *means, *quats, *scales, *viewmats, *Ks;
  const int32_t *radii;
  const float *ray_transforms, *v_means2d, *v_depths, *v_normals, *v_ray_transforms;
  float *v_means, *v_quats, *v_scales;
  int store_mode;  // C == 1: plain stores of every row; else atomics of valid rows
  // packed inputs (projection_2dgs_packed_bwd, Projection2DGSPacked.cu:274-420):
  // entry e is the pair (camera_ids[e], gaussian_ids[e]); sparse: one
  // gradient row per entry [nnz, .]
  const int64_t *camera_ids, *gaussian_ids;
  int64_t nnz;
  int sparse;
  GeomAdam ga;  // proj_bwd_kernel: the geometry Adam instead of the stores
};

// a.ga.p[0] set (ABI 33, gsplat_hip_projection_2dgs_bwd_adam; C == 1,
// dense): the geometry groups' Adam step on the lane's rows instead of
// storing v_means / v_quats / v_scales (geom_adam.h).  A runtime branch of
// the one kernel, so that the fused update consumes exactly the gradient
// values the plain backward stores (two instantiations contracted the
// algebra differently: 1 ulp in the log-scales).
__global__ void __launch_bounds__(256) proj_bwd_kernel(ProjBwdArgs a) {
  int c, n;
  size_t idx;
  bool valid;
  const bool packed = a.camera_ids != nullptr;
  if (packed) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.nnz) return;
    c = (int)a.camera_ids[e];
    n = (int)a.gaussian_ids[e];
    idx = (size_t)e;
    valid = true;
  } else {
    c = blockIdx.y;
    n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= a.N) return;
    idx = (size_t)c * a.N + n;
    valid = a.radii[idx] > 0;
  }
  GeomRows gr;
  const bool fuse = a.ga.p[0] != nullptr;
  const bool fuse_on = fuse && !(a.ga.skip && *a.ga.skip);
  if (fuse_on) geom_rows_load(a.ga, (size_t)n, a.scales, gr);  // in flight from here
  const Cam k = load_cam(a.viewmats, a.Ks, c);
  float vm[3] = {0.f, 0.f, 0.f}, vq[4] = {0.f, 0.f, 0.f, 0.f}, vs[3] = {0.f, 0.f, 0.f};
  if (valid) {
    const float4 q = *reinterpret_cast<const float4 *>(a.quats + 4 * (size_t)n);
    const float *sp = a.scales + 3 * (size_t)n;
    const float s0 = sp[0], s1 = sp[1];
    const Frame f = surfel_frame(k, a.means + 3 * (size_t)n, q, s0, s1);
    const float *rt = a.ray_transforms + 9 * idx;
    float V[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) V[i] = a.v_ray_transforms[9 * idx + i];
    if (a.v_depths) V[8] += a.v_depths[idx];
    // means2d through the AABB formula, as the reference differentiates it
    // (Projection2DGS.cuh:25-65)
    const float gx = a.v_means2d[2 * idx], gy = a.v_means2d[2 * idx + 1];
    if (gx != 0.f || gy != 0.f) {
      float r[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) r[i] = rt[i];
      const float fi = 1.f / (r[6] * r[6] + r[7] * r[7] - r[8] * r[8]);
      const float f2 = 2.f * fi * fi;
      V[0] += gx * (fi * r[6]);
      V[1] += gx * (fi * r[7]);
      V[2] += gx * (-fi * r[8]);
      V[3] += gy * (fi * r[6]);
      V[4] += gy * (fi * r[7]);
      V[5] += gy * (-fi * r[8]);
      const float e6 = fi - f2 * r[6] * r[6], e7 = fi - f2 * r[7] * r[7], e8 = fi + f2 * r[8] * r[8];
      V[6] += gx * (r[0] * e6) + gy * (r[3] * e6);
      V[7] += gx * (r[1] * e7) + gy * (r[4] * e7);
      V[8] += gx * (-r[2] * e8) + gy * (-r[5] * e8);
    }
    // d/d[t0 | t1 | mc] = K^T V (camera space), then R^T to world
    float dW[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      dW[0][j] = k.fx * V[j];
      dW[1][j] = k.fy * V[3 + j];
      dW[2][j] = k.cx * V[j] + k.cy * V[3 + j] + V[6 + j];
    }
    float vRS[3][3];  // vRS[i][j]: world-space gradient of column j
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        vRS[i][j] = k.R.m[0][i] * dW[0][j] + k.R.m[1][i] * dW[1][j] + k.R.m[2][i] * dW[2][j];
    // v_normals may be null (ABI 33: a render whose normals carry no
    // gradient): zeros through the same arithmetic
    float gn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) gn[i] = a.v_normals ? a.v_normals[3 * idx + i] : 0.f;
    const float sgn =
        -(f.nz[0] * f.mc[0] + f.nz[1] * f.mc[1] + f.nz[2] * f.mc[2]) > 0.f ? 1.f : -1.f;
    float vtn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      vtn[i] = sgn * (k.R.m[0][i] * gn[0] + k.R.m[1][i] * gn[1] + k.R.m[2][i] * gn[2]);
    M3 dR;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      dR.m[i][0] = vRS[i][0] * s0;
      dR.m[i][1] = vRS[i][1] * s1;
      dR.m[i][2] = vtn[i];
    }
    quat_to_rotmat_vjp(q.x, q.y, q.z, q.w, dR, vq);
    vs[0] = vRS[0][0] * f.Rq.m[0][0] + vRS[1][0] * f.Rq.m[1][0] + vRS[2][0] * f.Rq.m[2][0];
    vs[1] = vRS[0][1] * f.Rq.m[0][1] + vRS[1][1] * f.Rq.m[1][1] + vRS[2][1] * f.Rq.m[2][1];
#pragma unroll
    for (int i = 0; i < 3; ++i) vm[i] = vRS[i][2];
  }
  // the gradients are formed once, here, for every epilogue below, each
  // rounded on its own: the fused Adam epilogue (FUSE) then consumes exactly
  // the values the plain kernel stores (without the barrier the compiler may
  // contract the algebra differently in the two instantiations)
  asm volatile("" : "+v"(vm[0]), "+v"(vm[1]), "+v"(vm[2]), "+v"(vq[0]), "+v"(vq[1]),
               "+v"(vq[2]), "+v"(vq[3]), "+v"(vs[0]), "+v"(vs[1]), "+v"(vs[2]));
  if (fuse) {
    if (fuse_on) geom_rows_update(a.ga, (size_t)n, gr, vm, vs, vq);
    return;
  }
  if (packed && a.sparse) {  // COO values, one row per packed entry
    float *o = a.v_means + 3 * idx;
    o[0] = vm[0]; o[1] = vm[1]; o[2] = vm[2];
    *reinterpret_cast<float4 *>(a.v_quats + 4 * idx) = make_float4(vq[0], vq[1], vq[2], vq[3]);
    o = a.v_scales + 3 * idx;
    o[0] = vs[0]; o[1] = vs[1]; o[2] = 0.f;
  } else if (a.store_mode) {
    float *o = a.v_means + 3 * (size_t)n;
    o[0] = vm[0]; o[1] = vm[1]; o[2] = vm[2];
    *reinterpret_cast<float4 *>(a.v_quats + 4 * (size_t)n) = make_float4(vq[0], vq[1], vq[2], vq[3]);
    o = a.v_scales + 3 * (size_t)n;
    o[0] = vs[0]; o[1] = vs[1]; o[2] = 0.f;
  } else if (valid) {
#pragma unroll
    for (int j = 0; j < 3; ++j) atomic_add_f32(a.v_means + 3 * (size_t)n + j, vm[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) atomic_add_f32(a.v_quats + 4 * (size_t)n + j, vq[j]);
    atomic_add_f32(a.v_scales + 3 * (size_t)n, vs[0]);
    atomic_add_f32(a.v_scales + 3 * (size_t)n + 1, vs[1]);
  }
}

// ------------------------------------------------------------- rasterizer
// Record of one isect in a wave's LDS queue (floats):
//   [0] x [1] y [2] opacity [3] isect index (int bits)
//   [4..13) ray transform rows u, v, w   [13] surfel id (int bits)
//   [14..17) normal   [17..17+D) colour (the last channel is the depth that
//   the distortion and median terms read, as in the reference)
template <int D>
struct Rec {
  static constexpr int X = 0, Y = 1, OP = 2, IDX = 3, M = 4, G = 13, NRM = 14, COL = 17;
  static constexpr int NF = ((COL + D + 3) / 4) * 4;
  static constexpr int N4 = NF / 4;
};

typedef float f2v __attribute__((ext_vector_type(2)));

struct RasterArgs {
  int C, W, H, ts, tw, th, n_tiles;
  int64_t n_isects;       // isect count, or with n_dev the capacity of flatten_ids
  const int64_t *n_dev;   // the isect count on the device (sync-free isect) or null
  const int32_t *order;   // dispatch order of the tiles (heaviest first) or null
  const float *means2d, *ray_transforms, *colors, *opacities, *normals, *backgrounds;
  // depths (ABI 33, or null): the last colour channel from this [G] array,
  // `colors` then holding D - 1 channels per row (no concatenated copy)
  const float *depths;
  const uint8_t *masks;
  const int32_t *offsets, *flatten_ids;
  // forward outputs / backward inputs
  float *render_colors, *render_alphas, *render_normals, *render_distort, *render_median;
  int32_t *last_ids, *median_ids;
  // backward
  const float *v_render_colors, *v_render_alphas, *v_render_normals, *v_render_distort,
      *v_render_median;
  float *packed;  // [G][S] gradient rows
  int S;
  int dbg;  // gsplat_hip_debug_set_flags: backward bits 0 / 2 / 3 as the 3DGS kernel's
  int xcd_runs;  // deal runs of 4 consecutive order entries to one XCD (order_tile)
};

// The tile of workgroup blockIdx.x, or -1 (a surplus workgroup of a grid
// rounded up to whole rounds).  With xcd_runs, runs of four consecutive
// entries of the heaviest-first order (same bucket, mostly neighbouring
// tiles, which share surfels) go to one XCD (workgroup b runs on XCD b % 8),
// dealt round-robin so the order is kept across the chip.
GS_INLINE int order_tile(const RasterArgs &a) {
  if (!a.order) return (int)blockIdx.x;
  int b = (int)blockIdx.x;
  if (a.xcd_runs) {
    const int x = b & 7, kk = b >> 3;
    b = ((kk >> 2) * 8 + x) * 4 + (kk & 3);
  }
  return b < a.n_tiles ? a.order[b] : -1;
}

// Pixel of lane `lane` in wave `w`: the 64w + lane-th pixel of the tile in
// row-major order (a 16x4 strip for 16x16 tiles).
struct Pix {
  int c, tile, px, py;
  bool inside;
  int64_t pid;  // flat pixel index in [C*H*W] (clamped)
  int64_t start, end;
  GS_INLINE Pix(const RasterArgs &a, int tile_, int w, int lane) {
    tile = tile_;
    const int ntile = a.tw * a.th;
    c = tile / ntile;
    const int rem = tile - c * ntile;
    const int ty = rem / a.tw, tx = rem - ty * a.tw;
    const int p = 64 * w + lane;
    const int ly = p / a.ts, lx = p - ly * a.ts;
    px = tx * a.ts + lx;
    py = ty * a.ts + ly;
    inside = (p < a.ts * a.ts) && px < a.W && py < a.H;
    const int64_t off = (int64_t)c * a.H * a.W;
    pid = off + (inside ? (int64_t)py * a.W + px : 0);
    start = a.offsets[tile];
    end = (tile == a.n_tiles - 1) ? (a.n_dev ? a.n_dev[0] : a.n_isects)
                                  : (int64_t)a.offsets[tile + 1];
    // pixel-centre rectangle of the wave's rows (whole tile width)
    const int r0 = (64 * w) / a.ts, r1 = min(a.ts - 1, (64 * w + 63) / a.ts);
    x0 = tx * a.ts + 0.5f;
    x1 = x0 + (a.ts - 1);
    y0 = ty * a.ts + r0 + 0.5f;
    y1 = ty * a.ts + r1 + 0.5f;
  }
  float x0, x1, y0, y1;
};

// Strip culling: surfel_keep (surfel_cull.h, shared with the isect's tile culling).

template <int D>
struct Gathered {
  int32_t g;
  float2 xy;
  float op;
  float m[9];
  float nrm[3];
  float col[D];
};

// The attributes of surfel g (NRM: its normal too).
template <int D, bool NRM = true>
GS_INLINE void gather_at(const RasterArgs &a, int32_t g, Gathered<D> &r) {
  r.g = g;
  r.xy = *reinterpret_cast<const float2 *>(a.means2d + 2 * (int64_t)g);
  r.op = a.opacities[g];
  const float *m = a.ray_transforms + 9 * (int64_t)g;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.m[i] = m[i];
  if (NRM) {
    const float *nr = a.normals + 3 * (int64_t)g;
#pragma unroll
    for (int i = 0; i < 3; ++i) r.nrm[i] = nr[i];
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) r.nrm[i] = 0.f;
  }
  if (a.depths) {
    const float *cl = a.colors + (D - 1) * (int64_t)g;
#pragma unroll
    for (int i = 0; i < D - 1; ++i) r.col[i] = cl[i];
    r.col[D - 1] = a.depths[g];
  } else {
    const float *cl = a.colors + D * (int64_t)g;
#pragma unroll
    for (int i = 0; i < D; ++i) r.col[i] = cl[i];
  }
}

template <int D>
GS_INLINE void gather(const RasterArgs &a, int64_t j, bool ok, Gathered<D> &r) {
  gather_at<D>(a, ok ? a.flatten_ids[j] : 0, r);
}

template <int D>
GS_INLINE void stage(float *slot, const Gathered<D> &r, int32_t idx) {
  using R = Rec<D>;
  float v[R::NF];
  v[R::X] = r.xy.x;
  v[R::Y] = r.xy.y;
  v[R::OP] = r.op;
  v[R::IDX] = __int_as_float(idx);
#pragma unroll
  for (int i = 0; i < 9; ++i) v[R::M + i] = r.m[i];
  v[R::G] = __int_as_float(r.g);
#pragma unroll
  for (int i = 0; i < 3; ++i) v[R::NRM + i] = r.nrm[i];
#pragma unroll
  for (int i = 0; i < D; ++i) v[R::COL + i] = r.col[i];
#pragma unroll
  for (int i = R::COL + D; i < R::NF; ++i) v[i] = 0.f;
  float4 *s4 = reinterpret_cast<float4 *>(slot);
#pragma unroll
  for (int q = 0; q < R::N4; ++q) s4[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// Forward record: the ray-splat cross product is linear in the pixel centre,
//   (px w - u) x (py w - v) = px (v x w) + py (w x u) + (u x v),
// so the staging lane precomputes A = v x w, B = w x u, Cc = u x v (x and y
// components pre-scaled by sqrt(log2(e) / 2), making |s|^2 come out as
// sigma * log2(e) directly) and smax = log2(255 opacity): a pixel hits iff
// min(g3, g2) * log2(e) / 2 <= smax and the exponential is a bare exp2.
template <int D>
struct FRec {
  static constexpr int X = 0, Y = 1, OP = 2, IDX = 3, A = 4, B = 7, CC = 10, SMAX = 13, NRM = 14,
                       COL = 17;
  static constexpr int NF = ((COL + D + 3) / 4) * 4;
  static constexpr int N4 = NF / 4;
};

constexpr float kSqrtHalfLog2e = 0.84932180028801907f;  // sqrt(log2(e) / 2)

template <int D>
GS_INLINE void stage_fwd(float *slot, const Gathered<D> &r, int32_t idx) {
  using R = FRec<D>;
  const float *u = r.m, *v = r.m + 3, *w = r.m + 6;
  float v_[R::NF];
  v_[R::X] = r.xy.x;
  v_[R::Y] = r.xy.y;
  v_[R::OP] = r.op;
  v_[R::IDX] = __int_as_float(idx);
  const float k = kSqrtHalfLog2e;
  v_[R::A + 0] = k * (v[1] * w[2] - v[2] * w[1]);
  v_[R::A + 1] = k * (v[2] * w[0] - v[0] * w[2]);
  v_[R::A + 2] = v[0] * w[1] - v[1] * w[0];
  v_[R::B + 0] = k * (w[1] * u[2] - w[2] * u[1]);
  v_[R::B + 1] = k * (w[2] * u[0] - w[0] * u[2]);
  v_[R::B + 2] = w[0] * u[1] - w[1] * u[0];
  v_[R::CC + 0] = k * (u[1] * v[2] - u[2] * v[1]);
  v_[R::CC + 1] = k * (u[2] * v[0] - u[0] * v[2]);
  v_[R::CC + 2] = u[0] * v[1] - u[1] * v[0];
  v_[R::SMAX] = __builtin_amdgcn_logf(255.f * r.op);  // log2
#pragma unroll
  for (int i = 0; i < 3; ++i) v_[R::NRM + i] = r.nrm[i];
#pragma unroll
  for (int i = 0; i < D; ++i) v_[R::COL + i] = r.col[i];
#pragma unroll
  for (int i = R::COL + D; i < R::NF; ++i) v_[i] = 0.f;
  float4 *s4 = reinterpret_cast<float4 *>(slot);
#pragma unroll
  for (int q = 0; q < R::N4; ++q)
    s4[q] = make_float4(v_[4 * q], v_[4 * q + 1], v_[4 * q + 2], v_[4 * q + 3]);
}

template <int NF>
GS_INLINE void read_f4(const float *slot, float (&v)[NF]) {
  const float4 *s4 = reinterpret_cast<const float4 *>(slot);
#pragma unroll
  for (int q = 0; q < NF / 4; ++q) {
    const float4 t = s4[q];
    v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
  }
}

template <int D>
GS_INLINE void read_rec(const float *slot, float (&v)[Rec<D>::NF]) {
  const float4 *s4 = reinterpret_cast<const float4 *>(slot);
#pragma unroll
  for (int q = 0; q < Rec<D>::N4; ++q) {
    const float4 t = s4[q];
    v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
  }
}

// Ray-splat evaluation of one record at pixel centre (px, py)
// (RasterizeToPixels2DGSFwd.cu:333-361).
struct Hit {
  float hu[3], hv[3], rc[3], s[2], g3, g2, vis, alpha;
  bool ok;
};

GS_INLINE Hit eval_hit(const float *m, float x, float y, float op, float px, float py) {
  Hit h;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    h.hu[i] = px * m[6 + i] - m[i];
    h.hv[i] = py * m[6 + i] - m[3 + i];
  }
  h.rc[0] = h.hu[1] * h.hv[2] - h.hu[2] * h.hv[1];
  h.rc[1] = h.hu[2] * h.hv[0] - h.hu[0] * h.hv[2];
  h.rc[2] = h.hu[0] * h.hv[1] - h.hu[1] * h.hv[0];
  const float iz = __builtin_amdgcn_rcpf(h.rc[2]);
  h.s[0] = h.rc[0] * iz;
  h.s[1] = h.rc[1] * iz;
  h.g3 = h.s[0] * h.s[0] + h.s[1] * h.s[1];
  const float dx = x - px, dy = y - py;
  h.g2 = kFilterInvSquare * (dx * dx + dy * dy);
  const float sigma = 0.5f * fminf(h.g3, h.g2);
  h.vis = __builtin_amdgcn_exp2f(-sigma * kLog2e);
  h.alpha = fminf(kAlphaMax, op * h.vis);
  h.ok = (h.rc[2] != 0.f) && !(sigma < 0.f) && !(h.alpha < kAlphaMin);
  return h;
}

// One workgroup per tile, ceil(ts^2 / 64) waves, a 64-record queue per wave.
template <int D>
__global__ void __launch_bounds__(1024) fwd_kernel(RasterArgs a) {
  using R = FRec<D>;
  extern __shared__ float4 lds4[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float *q = reinterpret_cast<float *>(lds4) + (size_t)w * 64 * R::NF;
  const int otile = order_tile(a);
  if (otile < 0) return;
  const Pix p(a, otile, w, lane);
  const float fx = (float)p.px + 0.5f, fy = (float)p.py + 0.5f;
  const float *bg = a.backgrounds ? a.backgrounds + (int64_t)p.c * D : nullptr;

  float T = 1.f, col[D], nrm[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int d = 0; d < D; ++d) col[d] = 0.f;
  float distort = 0.f, acc_vd = 0.f, median = 0.f;
  int32_t cur = 0, med = 0;
  bool done = !p.inside;
  const bool masked = a.masks && !a.masks[p.tile];
  if (masked) done = true;

  int64_t b = p.start;
  const bool run = !masked && b < p.end;
  Gathered<D> nxt;
  if (run) gather<D>(a, b + lane, b + lane < p.end, nxt);
  for (; run && b < p.end; b += 64) {
    if (__ballot(!done) == 0) break;
    const bool keep = (b + lane < p.end) &&
                      surfel_keep(nxt.m, nxt.xy.x, nxt.xy.y, nxt.op, p.x0, p.x1, p.y0, p.y1);
    const uint64_t km = __ballot(keep);
    const int n = __popcll(km);
    if (keep) stage_fwd<D>(q + ballot_slot(km) * R::NF, nxt, (int32_t)(b + lane));
    wave_sync_lds();
    if (b + 64 < p.end) gather<D>(a, b + 64 + lane, b + 64 + lane < p.end, nxt);
    for (int t = 0; t < n; ++t) {
      float r[R::NF];
      read_f4<R::NF>(q + t * R::NF, r);
      if (!done) {
        const float rx = fx * r[R::A] + fy * r[R::B] + r[R::CC];
        const float ry = fx * r[R::A + 1] + fy * r[R::B + 1] + r[R::CC + 1];
        const float rz = fx * r[R::A + 2] + fy * r[R::B + 2] + r[R::CC + 2];
        const float iz = __builtin_amdgcn_rcpf(rz);
        const float g3 = (rx * rx + ry * ry) * (iz * iz);
        const float dx = r[R::X] - fx, dy = r[R::Y] - fy;
        const float g2 = kLog2e * (dx * dx + dy * dy);
        const float m = fminf(g3, g2);  // sigma * log2(e)
        if (rz != 0.f && m <= r[R::SMAX]) {
          const float alpha = fminf(kAlphaMax, r[R::OP] * __builtin_amdgcn_exp2f(-m));
          const float nT = T * (1.f - alpha);
          if (nT <= kTMin) {
            done = true;
          } else {
            const float vis = alpha * T;
#pragma unroll
            for (int d = 0; d < D; ++d) col[d] += r[R::COL + d] * vis;
#pragma unroll
            for (int i = 0; i < 3; ++i) nrm[i] += r[R::NRM + i] * vis;
            const float depth = r[R::COL + D - 1];
            distort += 2.f * (vis * depth * (1.f - T) - vis * acc_vd);
            acc_vd += vis * depth;
            const int32_t idx = __float_as_int(r[R::IDX]);
            if (T > 0.5f) {
              median = depth;
              med = idx;
            }
            cur = idx;
            T = nT;
          }
        }
      }
      if ((t & 7) == 7 && __ballot(!done) == 0) break;
    }
    wave_sync_lds();
  }
  if (!p.inside) return;
  const int64_t pid = p.pid;
  if (masked) {  // reference writes the background only; the rest is defined here as empty
#pragma unroll
    for (int d = 0; d < D; ++d) a.render_colors[pid * D + d] = bg ? bg[d] : 0.f;
    a.render_alphas[pid] = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) a.render_normals[pid * 3 + i] = 0.f;
    a.render_distort[pid] = 0.f;
    a.render_median[pid] = 0.f;
    a.last_ids[pid] = 0;
    a.median_ids[pid] = 0;
    return;
  }
  a.render_alphas[pid] = 1.f - T;
#pragma unroll
  for (int d = 0; d < D; ++d) a.render_colors[pid * D + d] = bg ? col[d] + T * bg[d] : col[d];
#pragma unroll
  for (int i = 0; i < 3; ++i) a.render_normals[pid * 3 + i] = nrm[i];
  a.render_distort[pid] = distort;
  a.render_median[pid] = median;
  a.last_ids[pid] = cur;
  a.median_ids[pid] = med;
}

// Forward with two pixels per lane (tile_size 16): wave w of the 2 owns the
// 16x8 band of rows 8w..8w+7, lane l the pixels (l & 15, 8w + (l >> 4)) and
// 4 rows below.  Two independent transmittance chains per lane give the
// scheduler independent work between dependent steps, and the gather,
// culling test and LDS reads of a record are shared by both pixels.  Same
// per-pixel arithmetic as fwd_kernel.
template <int D, bool LEAN = false>  // LEAN: fwd2s_kernel's colours-only form (unused here)
__global__ void __launch_bounds__(128) fwd2_kernel(RasterArgs a) {
  using R = FRec<D>;
  extern __shared__ float4 lds4[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float *q = reinterpret_cast<float *>(lds4) + (size_t)w * 64 * R::NF;
  const int tile = order_tile(a);
  if (tile < 0) return;
  const int ntile = a.tw * a.th;
  const int c = tile / ntile;
  const int rem = tile - c * ntile;
  const int ty = rem / a.tw, tx = rem - ty * a.tw;
  const int64_t start = a.offsets[tile];
  const int64_t end = (tile == a.n_tiles - 1) ? (a.n_dev ? a.n_dev[0] : a.n_isects)
                                              : (int64_t)a.offsets[tile + 1];
  const float rx0 = tx * 16 + 0.5f, rx1 = rx0 + 15.f;
  const float ry0 = ty * 16 + 8 * w + 0.5f, ry1 = ry0 + 7.f;
  const float *bg = a.backgrounds ? a.backgrounds + (int64_t)c * D : nullptr;
  const bool masked = a.masks && !a.masks[tile];
  const float fx = (float)(tx * 16 + (lane & 15)) + 0.5f;
  float fy[2], T[2], col[2][D], nrm[2][3], distort[2], acc_vd[2], median[2];
  int32_t cur[2], med[2];
  bool done[2], inside[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int py = ty * 16 + 8 * w + 4 * k + (lane >> 4);
    fy[k] = (float)py + 0.5f;
    inside[k] = (tx * 16 + (lane & 15)) < a.W && py < a.H;
    T[k] = 1.f;
#pragma unroll
    for (int d = 0; d < D; ++d) col[k][d] = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) nrm[k][i] = 0.f;
    distort[k] = acc_vd[k] = median[k] = 0.f;
    cur[k] = med[k] = 0;
    done[k] = !inside[k] || masked;
  }

  int64_t b = start;
  const bool run = !masked && b < end;
  Gathered<D> nxt;
  if (run) gather<D>(a, b + lane, b + lane < end, nxt);
  for (; run && b < end; b += 64) {
    if (__ballot(!(done[0] & done[1])) == 0) break;
    const bool keep = (b + lane < end) &&
                      surfel_keep(nxt.m, nxt.xy.x, nxt.xy.y, nxt.op, rx0, rx1, ry0, ry1);
    const uint64_t km = __ballot(keep);
    const int n = __popcll(km);
    if (keep) stage_fwd<D>(q + ballot_slot(km) * R::NF, nxt, (int32_t)(b + lane));
    wave_sync_lds();
    if (b + 64 < end) gather<D>(a, b + 64 + lane, b + 64 + lane < end, nxt);
    for (int t = 0; t < n; ++t) {
      float r[R::NF];
      read_f4<R::NF>(q + t * R::NF, r);
      const float rxb = fx * r[R::A] + r[R::CC], ryb = fx * r[R::A + 1] + r[R::CC + 1],
                  rzb = fx * r[R::A + 2] + r[R::CC + 2];
      const float dx = r[R::X] - fx, dx2 = dx * dx;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (done[k]) continue;
        const float rx = fy[k] * r[R::B] + rxb;
        const float ry = fy[k] * r[R::B + 1] + ryb;
        const float rz = fy[k] * r[R::B + 2] + rzb;
        const float iz = __builtin_amdgcn_rcpf(rz);
        const float g3 = (rx * rx + ry * ry) * (iz * iz);
        const float dy = r[R::Y] - fy[k];
        const float g2 = kLog2e * (dx2 + dy * dy);
        const float m = fminf(g3, g2);  // sigma * log2(e)
        if (rz != 0.f && m <= r[R::SMAX]) {
          const float alpha = fminf(kAlphaMax, r[R::OP] * __builtin_amdgcn_exp2f(-m));
          const float nT = T[k] * (1.f - alpha);
          if (nT <= kTMin) {
            done[k] = true;
          } else {
            const float vis = alpha * T[k];
#pragma unroll
            for (int d = 0; d < D; ++d) col[k][d] += r[R::COL + d] * vis;
#pragma unroll
            for (int i = 0; i < 3; ++i) nrm[k][i] += r[R::NRM + i] * vis;
            const float depth = r[R::COL + D - 1];
            distort[k] += 2.f * (vis * depth * (1.f - T[k]) - vis * acc_vd[k]);
            acc_vd[k] += vis * depth;
            const int32_t idx = __float_as_int(r[R::IDX]);
            if (T[k] > 0.5f) {
              median[k] = depth;
              med[k] = idx;
            }
            cur[k] = idx;
            T[k] = nT;
          }
        }
      }
      if ((t & 7) == 7 && __ballot(!(done[0] & done[1])) == 0) break;
    }
    wave_sync_lds();
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (!inside[k]) continue;
    const int64_t pid = ((int64_t)c * a.H + (ty * 16 + 8 * w + 4 * k + (lane >> 4))) * a.W +
                        tx * 16 + (lane & 15);
    if (masked) {  // as fwd_kernel
#pragma unroll
      for (int d = 0; d < D; ++d) a.render_colors[pid * D + d] = bg ? bg[d] : 0.f;
      a.render_alphas[pid] = 0.f;
      a.last_ids[pid] = 0;
      if (!LEAN) {
#pragma unroll
        for (int i = 0; i < 3; ++i) a.render_normals[pid * 3 + i] = 0.f;
        a.render_distort[pid] = 0.f;
        a.render_median[pid] = 0.f;
        a.median_ids[pid] = 0;
      }
      continue;
    }
    a.render_alphas[pid] = 1.f - T[k];
#pragma unroll
    for (int d = 0; d < D; ++d)
      a.render_colors[pid * D + d] = bg ? col[k][d] + T[k] * bg[d] : col[k][d];
    a.last_ids[pid] = cur[k];
    if (!LEAN) {
#pragma unroll
      for (int i = 0; i < 3; ++i) a.render_normals[pid * 3 + i] = nrm[k][i];
      a.render_distort[pid] = distort[k];
      a.render_median[pid] = median[k];
      a.median_ids[pid] = med[k];
    }
  }
}

// ---- Scalar-operand records (GSPLAT_HIP_SURFEL_SREC=1; D <= 4, 16x16
// tiles).  fwd2_kernel spends, per (record, wave), six ds_read_b128 on the
// staged record (every lane reads the same 96 B: 48 of the CU's 128 B/clk LDS
// cycles) besides the staging writes.  Here pack_srec_kernel writes one 128-B
// record per surfel with everything the culling test and the compositing
// read, precomputed; the lanes cull their candidates from vector loads of the
// first 80 B, and the kept records are composited in ascending isect order
// from scalar loads (constant address space, wave-uniform address from
// v_readlane of the candidate's id): the fields reach the VALU as SGPR
// operands, with no LDS traffic at all.  Same per-pixel arithmetic and order
// as fwd2_kernel (bit-identical outputs).
// Dispatch order (GSPLAT_HIP_SURFEL_ORDER=1): the tiles bucketed by
// floor(log2(isects)), heaviest bucket first, so the longest tiles start in
// the first wave of workgroups instead of finishing last (order inside a
// bucket: arrival at an LDS counter).  One workgroup; any tile count: the
// tiles are taken in blocks of 16384 (16 per thread), and with more than one
// block each pass reloads its block's keys.
__global__ void __launch_bounds__(1024)
tile_order_kernel(int n_tiles, const int32_t *__restrict__ offsets, int64_t n_isects,
                  const int64_t *__restrict__ n_dev, int32_t *__restrict__ order) {
  constexpr int MAXR = 16;  // tiles per thread and block
  constexpr int BLK = 1024 * MAXR;
  __shared__ int hist[34];
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < 34) hist[tid] = 0;
  const int64_t total = n_dev ? n_dev[0] : n_isects;
  const int n_blk = (n_tiles + BLK - 1) / BLK;
  // a block's offsets loaded up front (one load latency, not one per round),
  // its keys kept in registers (for both passes when there is one block)
  int k[MAXR];
  auto load_keys = [&](int b0) {
#pragma unroll
    for (int rd = 0; rd < MAXR; ++rd) {
      const int t = b0 + tid + 1024 * rd;
      int64_t n = -1;
      if (t < n_tiles) n = (t == n_tiles - 1 ? total : (int64_t)offsets[t + 1]) - offsets[t];
      // 2^31.. -> 1, 1 -> 32, empty -> 33, no tile -> -1
      k[rd] = n < 0 ? -1 : (n > 0 ? 32 - (63 - __builtin_clzll((uint64_t)n)) : 33);
    }
  };
  __syncthreads();
  // per wave and distinct key one LDS atomic (a few keys per wave: M5's
  // tiles fall into 2-3 buckets, and 64 lanes on one counter serialised)
  for (int b = 0; b < n_blk; ++b) {
    load_keys(b * BLK);
#pragma unroll
    for (int rd = 0; rd < MAXR; ++rd) {
      uint64_t todo = __ballot(k[rd] >= 0);
      while (todo) {
        const int kk = __builtin_amdgcn_readlane(k[rd], __builtin_ctzll(todo));
        const uint64_t m = __ballot(k[rd] == kk) & todo;
        if (lane == __builtin_ctzll(m)) atomicAdd(&hist[kk], __popcll(m));
        todo &= ~m;
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int q = 0; q < 34; ++q) {
      const int h = hist[q];
      hist[q] = run;
      run += h;
    }
  }
  __syncthreads();
  for (int b = 0; b < n_blk; ++b) {
    if (n_blk > 1) load_keys(b * BLK);
#pragma unroll
    for (int rd = 0; rd < MAXR; ++rd) {
      const int t = b * BLK + tid + 1024 * rd;
      uint64_t todo = __ballot(k[rd] >= 0);
      while (todo) {
        const int kk = __builtin_amdgcn_readlane(k[rd], __builtin_ctzll(todo));
        const uint64_t m = __ballot(k[rd] == kk) & todo;
        const int leader = __builtin_ctzll(m);
        int base = 0;
        if (lane == leader) base = atomicAdd(&hist[kk], __popcll(m));
        base = __shfl(base, leader, 64);
        if (k[rd] == kk) order[base + __popcll(m & ((1ull << lane) - 1))] = t;
        todo &= ~m;
      }
    }
  }
}

constexpr int kSRecMaxD = 4;
namespace srec {
// floats of a record
constexpr int NF = 32;
constexpr int X = 0, Y = 1, OP = 2, SMAX = 3,   // chunk 0
    AZ = 4, BZ = 5, CZ = 6,                      // chunk 1 (z parts: unscaled)
    BOX = 8,                                     // chunk 2: xlo, xhi, ylo, yhi
    U0X = 12, U0Y = 13, U1X = 14, U1Y = 15,      // chunk 3: v x w, w x u (unscaled)
    U2X = 16, U2Y = 17, NRM0 = 18, NRM1 = 19,    // chunk 4: u x v
    AX = 20, AY = 21, BX = 22, BY = 23,          // chunk 5 (scaled)
    CX = 24, CY = 25, NRM2 = 26,                 // chunk 6
    COL = 28;                                    // chunk 7: colour[D <= 4]
}  // namespace srec

template <int D>
__global__ void __launch_bounds__(256)
pack_srec_kernel(int64_t G, const float *__restrict__ means2d, const float *__restrict__ rt,
                 const float *__restrict__ opac, const float *__restrict__ nrm,
                 const float *__restrict__ col, const float *__restrict__ depths,
                 const int32_t *__restrict__ visible, float *__restrict__ rec) {
  using namespace srec;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= G) return;
  if (visible && visible[g] <= 0) return;  // never gathered: no record
  float m[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) m[i] = rt[9 * g + i];
  const float *u = m, *v = m + 3, *w = m + 6;
  const float op = opac[g];
  float r[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) r[i] = 0.f;
  r[X] = means2d[2 * g];
  r[Y] = means2d[2 * g + 1];
  r[OP] = op;
  r[SMAX] = __builtin_amdgcn_logf(255.f * op);  // log2, as stage_fwd
  // surfel_keep's quantities, in its expressions
  const float lnv = 0.69314718f * r[SMAX] + 0.05f;
  const float r2 = 2.f * lnv;
  const float c22 = r2 * (m[6] * m[6] + m[7] * m[7]) - m[8] * m[8];
  float xlo = -INFINITY, xhi = INFINITY, ylo = -INFINITY, yhi = INFINITY;
  if (c22 < 0.f) {
    const float ic = 1.f / c22;
    const float c00 = r2 * (m[0] * m[0] + m[1] * m[1]) - m[2] * m[2];
    const float c11 = r2 * (m[3] * m[3] + m[4] * m[4]) - m[5] * m[5];
    const float c02 = r2 * (m[0] * m[6] + m[1] * m[7]) - m[2] * m[8];
    const float c12 = r2 * (m[3] * m[6] + m[4] * m[7]) - m[5] * m[8];
    const float cx = c02 * ic, cy = c12 * ic;
    const float hx = sqrtf(fmaxf(cx * cx - c00 * ic, 0.f)) + 1.f;
    const float hy = sqrtf(fmaxf(cy * cy - c11 * ic, 0.f)) + 1.f;
    xlo = cx - hx; xhi = cx + hx; ylo = cy - hy; yhi = cy + hy;
  }
  r[BOX] = xlo; r[BOX + 1] = xhi; r[BOX + 2] = ylo; r[BOX + 3] = yhi;
  r[U0X] = v[1] * w[2] - v[2] * w[1];
  r[U0Y] = v[2] * w[0] - v[0] * w[2];
  r[AZ] = v[0] * w[1] - v[1] * w[0];
  r[U1X] = w[1] * u[2] - w[2] * u[1];
  r[U1Y] = w[2] * u[0] - w[0] * u[2];
  r[BZ] = w[0] * u[1] - w[1] * u[0];
  r[U2X] = u[1] * v[2] - u[2] * v[1];
  r[U2Y] = u[2] * v[0] - u[0] * v[2];
  r[CZ] = u[0] * v[1] - u[1] * v[0];
  const float k = kSqrtHalfLog2e;  // stage_fwd's scaling
  r[AX] = k * (v[1] * w[2] - v[2] * w[1]);
  r[AY] = k * (v[2] * w[0] - v[0] * w[2]);
  r[BX] = k * (w[1] * u[2] - w[2] * u[1]);
  r[BY] = k * (w[2] * u[0] - w[0] * u[2]);
  r[CX] = k * (u[1] * v[2] - u[2] * v[1]);
  r[CY] = k * (u[2] * v[0] - u[0] * v[2]);
  r[NRM0] = nrm[3 * g];
  r[NRM1] = nrm[3 * g + 1];
  r[NRM2] = nrm[3 * g + 2];
  if (depths) {  // colors: D - 1 channels, the last one from depths (ABI 33)
#pragma unroll
    for (int d = 0; d < D - 1; ++d) r[COL + d] = col[(D - 1) * g + d];
    r[COL + D - 1] = depths[g];
  } else {
#pragma unroll
    for (int d = 0; d < D; ++d) r[COL + d] = col[D * g + d];
  }
  float4 *o = reinterpret_cast<float4 *>(rec + NF * g);
#pragma unroll
  for (int q = 0; q < NF / 4; ++q) o[q] = make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
}

// The culling fields of a candidate (the record's first five float4s).
struct SCull {
  float4 c[5];
};

GS_INLINE void srec_load_cull(const float *rec, int32_t g, SCull &k) {
  const float4 *p = reinterpret_cast<const float4 *>(rec + (int64_t)srec::NF * g);
#pragma unroll
  for (int q = 0; q < 5; ++q) k.c[q] = p[q];
}

// surfel_keep from the record's precomputed fields (same tests, same values).
GS_INLINE bool srec_keep(const SCull &k, float x0, float x1, float y0, float y1) {
  const float x = k.c[0].x, y = k.c[0].y, op = k.c[0].z, smax = k.c[0].w;
  if (!(op >= kAlphaMin)) return false;
  const float lnv = 0.69314718f * smax + 0.05f;
  const float ddx = fmaxf(fmaxf(x0 - x, x - x1), 0.f), ddy = fmaxf(fmaxf(y0 - y, y - y1), 0.f);
  if (ddx * ddx + ddy * ddy <= lnv) return true;
  const float r2 = 2.f * lnv;
  if (k.c[2].y < x0 || k.c[2].x > x1 || k.c[2].w < y0 || k.c[2].z > y1) return false;
  const float a0x = k.c[3].x, a0y = k.c[3].y, a0z = k.c[1].x;
  const float a1x = k.c[3].z, a1y = k.c[3].w, a1z = k.c[1].y;
  const float a2x = k.c[4].x, a2y = k.c[4].y, a2z = k.c[1].z;
  float sx[4], sy[4], zmin = 3.4e38f, zmax = -3.4e38f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float X = (i == 1 || i == 2) ? x1 : x0, Y = i >= 2 ? y1 : y0;
    const float zx = X * a0x + Y * a1x + a2x, zy = X * a0y + Y * a1y + a2y,
                zz = X * a0z + Y * a1z + a2z;
    zmin = fminf(zmin, zz);
    zmax = fmaxf(zmax, zz);
    const float iz = 1.f / zz;
    sx[i] = zx * iz;
    sy[i] = zy * iz;
  }
  if (!(zmin > 0.f || zmax < 0.f)) return true;
  float best = 3.4e38f;
  bool pos = true, neg = true;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = (i + 1) & 3;
    const float ex = sx[j] - sx[i], ey = sy[j] - sy[i];
    const float cr = ey * sx[i] - ex * sy[i];
    pos &= cr >= 0.f;
    neg &= cr <= 0.f;
    const float L = ex * ex + ey * ey;
    const float t = L > 0.f ? fminf(fmaxf(-(sx[i] * ex + sy[i] * ey) / L, 0.f), 1.f) : 0.f;
    const float dx = sx[i] + t * ex, dy = sy[i] + t * ey;
    best = fminf(best, dx * dx + dy * dy);
  }
  return pos || neg || best <= r2;
}

typedef __attribute__((address_space(4))) const float cfloat_t;

// The compositing fields of one kept record, read with scalar loads.
template <int D>
struct SBlend {
  float x, y, op, smax, az, bz, cz, ax, ay, bx, by, cx, cy, n0, n1, n2, col[D];
};

template <int D>
GS_INLINE void srec_load_blend(const float *rec, int32_t g, SBlend<D> &r) {
  cfloat_t *p = (cfloat_t *)(rec) + (int64_t)srec::NF * g;
  using namespace srec;
  r.x = p[X]; r.y = p[Y]; r.op = p[OP]; r.smax = p[SMAX];
  r.az = p[AZ]; r.bz = p[BZ]; r.cz = p[CZ];
  r.n0 = p[NRM0]; r.n1 = p[NRM1];
  r.ax = p[AX]; r.ay = p[AY]; r.bx = p[BX]; r.by = p[BY];
  r.cx = p[CX]; r.cy = p[CY]; r.n2 = p[NRM2];
#pragma unroll
  for (int d = 0; d < D; ++d) r.col[d] = p[COL + d];
}

// LEAN (a colours-only render: render_normals / distort / median and
// median_ids null): only the colours, alphas and last ids are formed.
template <int D, bool LEAN = false>
__global__ void __launch_bounds__(128) fwd2s_kernel(RasterArgs a, const float *__restrict__ rec) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tile = order_tile(a);
  if (tile < 0) return;
  const int ntile = a.tw * a.th;
  const int c = tile / ntile;
  const int rem = tile - c * ntile;
  const int ty = rem / a.tw, tx = rem - ty * a.tw;
  const int64_t start = a.offsets[tile];
  const int64_t end = (tile == a.n_tiles - 1) ? (a.n_dev ? a.n_dev[0] : a.n_isects)
                                              : (int64_t)a.offsets[tile + 1];
  const float rx0 = tx * 16 + 0.5f, rx1 = rx0 + 15.f;
  const float ry0 = ty * 16 + 8 * w + 0.5f, ry1 = ry0 + 7.f;
  const float *bg = a.backgrounds ? a.backgrounds + (int64_t)c * D : nullptr;
  const bool masked = a.masks && !a.masks[tile];
  const float fx = (float)(tx * 16 + (lane & 15)) + 0.5f;
  float fy[2], T[2], col[2][D], nrm[2][3], distort[2], acc_vd[2], median[2];
  int32_t cur[2], med[2];
  bool done[2], inside[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int py = ty * 16 + 8 * w + 4 * k + (lane >> 4);
    fy[k] = (float)py + 0.5f;
    inside[k] = (tx * 16 + (lane & 15)) < a.W && py < a.H;
    T[k] = 1.f;
#pragma unroll
    for (int d = 0; d < D; ++d) col[k][d] = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) nrm[k][i] = 0.f;
    distort[k] = acc_vd[k] = median[k] = 0.f;
    cur[k] = med[k] = 0;
    done[k] = !inside[k] || masked;
  }
  // one record into both pixels of the lane (fwd2_kernel's arithmetic)
  auto blend = [&](const SBlend<D> &r, int32_t idx) {
    const float rxb = fx * r.ax + r.cx, ryb = fx * r.ay + r.cy, rzb = fx * r.az + r.cz;
    const float dx = r.x - fx, dx2 = dx * dx;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (done[k]) continue;
      const float rx = fy[k] * r.bx + rxb;
      const float ry = fy[k] * r.by + ryb;
      const float rz = fy[k] * r.bz + rzb;
      const float iz = __builtin_amdgcn_rcpf(rz);
      const float g3 = (rx * rx + ry * ry) * (iz * iz);
      const float dy = r.y - fy[k];
      const float g2 = kLog2e * (dx2 + dy * dy);
      const float m = fminf(g3, g2);
      if (rz != 0.f && m <= r.smax) {
        const float alpha = fminf(kAlphaMax, r.op * __builtin_amdgcn_exp2f(-m));
        const float nT = T[k] * (1.f - alpha);
        if (nT <= kTMin) {
          done[k] = true;
        } else {
          const float vis = alpha * T[k];
#pragma unroll
          for (int d = 0; d < D; ++d) col[k][d] += r.col[d] * vis;
          if (!LEAN) {
            nrm[k][0] += r.n0 * vis;
            nrm[k][1] += r.n1 * vis;
            nrm[k][2] += r.n2 * vis;
            const float depth = r.col[D - 1];
            distort[k] += 2.f * (vis * depth * (1.f - T[k]) - vis * acc_vd[k]);
            acc_vd[k] += vis * depth;
            if (T[k] > 0.5f) {
              median[k] = depth;
              med[k] = idx;
            }
          }
          cur[k] = idx;
          T[k] = nT;
        }
      }
    }
  };

  int64_t b = start;
  const bool run = !masked && b < end;
  int32_t gn = 0;
  SCull kn;
  if (run) {
    gn = b + lane < end ? a.flatten_ids[b + lane] : 0;
    srec_load_cull(rec, gn, kn);
  }
  for (; run && b < end; b += 64) {
    if (__ballot(!(done[0] & done[1])) == 0) break;
    const bool keep = (b + lane < end) && srec_keep(kn, rx0, rx1, ry0, ry1);
    uint64_t km = __ballot(keep);
    const int32_t gc = gn;
    if (b + 64 < end) {  // the next batch's candidates, in flight while this one composites
      gn = b + 64 + lane < end ? a.flatten_ids[b + 64 + lane] : 0;
      srec_load_cull(rec, gn, kn);
    }
    // kept records in ascending isect order, two per round: both records'
    // scalar loads are issued before the first is blended (no record value
    // is carried across rounds, so the compiler keeps them in SGPRs)
    int n = 0;
    while (km) {
      const int t0 = __builtin_ctzll(km);
      km &= km - 1;
      const bool two = km != 0;
      const int t1 = two ? __builtin_ctzll(km) : t0;
      km &= km - 1;
      SBlend<D> r0, r1;
      srec_load_blend<D>(rec, __builtin_amdgcn_readlane(gc, t0), r0);
      srec_load_blend<D>(rec, __builtin_amdgcn_readlane(gc, t1), r1);
      blend(r0, (int32_t)(b + t0));
      if ((++n & 7) == 0 && __ballot(!(done[0] & done[1])) == 0) break;
      if (!two) break;
      blend(r1, (int32_t)(b + t1));
      if ((++n & 7) == 0 && __ballot(!(done[0] & done[1])) == 0) break;
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (!inside[k]) continue;
    const int64_t pid = ((int64_t)c * a.H + (ty * 16 + 8 * w + 4 * k + (lane >> 4))) * a.W +
                        tx * 16 + (lane & 15);
    if (masked) {  // as fwd_kernel
#pragma unroll
      for (int d = 0; d < D; ++d) a.render_colors[pid * D + d] = bg ? bg[d] : 0.f;
      a.render_alphas[pid] = 0.f;
      a.last_ids[pid] = 0;
      if (!LEAN) {
#pragma unroll
        for (int i = 0; i < 3; ++i) a.render_normals[pid * 3 + i] = 0.f;
        a.render_distort[pid] = 0.f;
        a.render_median[pid] = 0.f;
        a.median_ids[pid] = 0;
      }
      continue;
    }
    a.render_alphas[pid] = 1.f - T[k];
#pragma unroll
    for (int d = 0; d < D; ++d)
      a.render_colors[pid * D + d] = bg ? col[k][d] + T[k] * bg[d] : col[k][d];
    a.last_ids[pid] = cur[k];
    if (!LEAN) {
#pragma unroll
      for (int i = 0; i < 3; ++i) a.render_normals[pid * 3 + i] = nrm[k][i];
      a.render_distort[pid] = distort[k];
      a.render_median[pid] = median[k];
      a.median_ids[pid] = med[k];
    }
  }
}

// Gradient fields of a packed row: colour[D], normal[3], ray transform[9],
// means2d[2], opacity, |means2d|[2] (absgrad only).
// LEAN (the backward of a render whose normals, distortion and median carry
// no gradient -- the training step's RGB(+D) loss): no normal fields, so
// D + 12 fields (one reduce-scatter group for RGB+D instead of two).
template <int D, bool ABS, bool LEAN = false>
struct Fields {
  static constexpr int NN = LEAN ? 0 : 3;  // normal fields
  static constexpr int COL = 0, NRM = D, M = D + NN, XY = D + NN + 9, OP = D + NN + 11,
                       AB = D + NN + 12;
  static constexpr int NF = D + NN + 12 + (ABS ? 2 : 0);
  static constexpr int NV = (NF + 15) / 16;  // reduce_scatter groups
  static constexpr int S = 16 * NV;          // packed row stride (floats)
};

template <int D, bool ABS>
__global__ void __launch_bounds__(256) bwd_kernel(RasterArgs a) {
  using R = Rec<D>;
  using F = Fields<D, ABS>;
  extern __shared__ float4 lds4[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float *q = reinterpret_cast<float *>(lds4) + (size_t)w * 64 * R::NF;
  const int otile = order_tile(a);
  if (otile < 0) return;
  const Pix p(a, otile, w, lane);
  if (a.masks && !a.masks[p.tile]) return;
  const float fx = (float)p.px + 0.5f, fy = (float)p.py + 0.5f;
  const int64_t pid = p.pid;

  const float Tf = 1.f - a.render_alphas[pid];
  float T = Tf;
  const int32_t bin_final = p.inside ? a.last_ids[pid] : 0;
  const int32_t med_idx = p.inside ? a.median_ids[pid] : 0;
  float vc[D], buf[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    vc[d] = a.v_render_colors[pid * D + d];
    buf[d] = 0.f;
  }
  const float va = a.v_render_alphas ? a.v_render_alphas[pid] : 0.f;
  float vn[3], bufn[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 3; ++i) vn[i] = a.v_render_normals ? a.v_render_normals[pid * 3 + i] : 0.f;
  const float vdist = a.v_render_distort ? a.v_render_distort[pid] : 0.f;
  const float accum_d = a.render_colors[pid * D + D - 1], accum_w = 1.f - Tf;
  float accd_buf = accum_d, accw_buf = accum_w, dist_buf = 0.f;
  const float vmed = a.v_render_median ? a.v_render_median[pid] : 0.f;
  float bg_dot = 0.f;
  if (a.backgrounds) {
#pragma unroll
    for (int d = 0; d < D; ++d) bg_dot += a.backgrounds[(int64_t)p.c * D + d] * vc[d];
  }
  // records past every lane's last contributor are skipped (the reference's
  // warp_bin_final, RasterizeToPixels2DGSBwd.cu:336-337)
  int32_t wmax = bin_final;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) wmax = max(wmax, __shfl_xor(wmax, m, 64));
  const int64_t end = min(p.end, (int64_t)wmax + 1);
  const int lf = rs_field(lane);

  for (int64_t b1 = end; b1 > p.start; b1 -= 64) {
    const int64_t b0 = max(p.start, b1 - 64);
    int n;
    {
      Gathered<D> g;
      const int64_t j = b0 + lane;
      gather<D>(a, j, j < b1, g);
      const bool keep = (j < b1) && surfel_keep(g.m, g.xy.x, g.xy.y, g.op, p.x0, p.x1, p.y0, p.y1);
      const uint64_t km = __ballot(keep);
      n = __popcll(km);
      if (keep) stage<D>(q + ballot_slot(km) * R::NF, g, (int32_t)j);
    }
    wave_sync_lds();
    for (int t = n - 1; t >= 0; --t) {
      float r[R::NF];
      read_rec<D>(q + t * R::NF, r);
      const int32_t idx = __float_as_int(r[R::IDX]);
      const float *m = r + R::M;
      Hit h = eval_hit(m, r[R::X], r[R::Y], r[R::OP], fx, fy);
      const bool valid = p.inside && idx <= bin_final && h.ok;
      if (__ballot(valid) == 0) continue;
      float v[16 * F::NV];
#pragma unroll
      for (int k = 0; k < 16 * F::NV; ++k) v[k] = 0.f;
      if (valid) {
        if (idx == med_idx) v[F::COL + D - 1] += vmed;
        const float ra = __builtin_amdgcn_rcpf(1.f - h.alpha);
        T *= ra;
        const float fac = h.alpha * T;
        float v_alpha = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          v[F::COL + d] += fac * vc[d];
          v_alpha += (r[R::COL + d] * T - buf[d] * ra) * vc[d];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          v[F::NRM + i] = fac * vn[i];
          v_alpha += (r[R::NRM + i] * T - bufn[i] * ra) * vn[i];
        }
        v_alpha += Tf * ra * va;
        v_alpha += -Tf * ra * bg_dot;
        {  // distortion (RasterizeToPixels2DGSBwd.cu:483-503)
          const float depth = r[R::COL + D - 1];
          const float dl_dw =
              2.f * (2.f * (depth * accw_buf - accd_buf) + (accum_d - depth * accum_w));
          v_alpha += (dl_dw * T - dist_buf * ra) * vdist;
          accd_buf -= fac * depth;
          accw_buf -= fac;
          dist_buf += dl_dw * fac;
          v[F::COL + D - 1] += 2.f * fac * (2.f - 2.f * T - accum_w + fac) * vdist;
        }
        if (r[R::OP] * h.vis <= kAlphaMax) {
          const float vG = r[R::OP] * v_alpha;
          if (h.g3 <= h.g2) {
            const float vsx = vG * -h.vis * h.s[0], vsy = vG * -h.vis * h.s[1];
            const float iz = __builtin_amdgcn_rcpf(h.rc[2]);
            const float ax = vsx * iz, ay = vsy * iz;
            const float vrc[3] = {ax, ay, -(ax * h.s[0] + ay * h.s[1])};
            // v_h_u = h_v x v_rc, v_h_v = v_rc x h_u
            const float vhu[3] = {h.hv[1] * vrc[2] - h.hv[2] * vrc[1],
                                  h.hv[2] * vrc[0] - h.hv[0] * vrc[2],
                                  h.hv[0] * vrc[1] - h.hv[1] * vrc[0]};
            const float vhv[3] = {vrc[1] * h.hu[2] - vrc[2] * h.hu[1],
                                  vrc[2] * h.hu[0] - vrc[0] * h.hu[2],
                                  vrc[0] * h.hu[1] - vrc[1] * h.hu[0]};
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              v[F::M + i] = -vhu[i];
              v[F::M + 3 + i] = -vhv[i];
              v[F::M + 6 + i] = fx * vhu[i] + fy * vhv[i];
            }
          } else {
            const float dx = r[R::X] - fx, dy = r[R::Y] - fy;
            v[F::XY] = vG * (-h.vis * kFilterInvSquare * dx);
            v[F::XY + 1] = vG * (-h.vis * kFilterInvSquare * dy);
            if (ABS) {
              v[F::AB] = fabsf(v[F::XY]);
              v[F::AB + 1] = fabsf(v[F::XY + 1]);
            }
          }
          v[F::OP] = h.vis * v_alpha;
        }
#pragma unroll
        for (int d = 0; d < D; ++d) buf[d] += r[R::COL + d] * fac;
#pragma unroll
        for (int i = 0; i < 3; ++i) bufn[i] += r[R::NRM + i] * fac;
      }
      const int32_t g = __float_as_int(r[R::G]);
      float *row = a.packed + (int64_t)g * F::S;
#pragma unroll
      for (int k = 0; k < F::NV; ++k) {
        constexpr int NQ = F::NF - 16 * (F::NV - 1);
        const float tot = k < F::NV - 1 ? reduce_scatter<16>(v + 16 * k, lane)
                                        : reduce_scatter<NQ>(v + 16 * k, lane);
        if ((lane & 3) == 0 && lf < (k < F::NV - 1 ? 16 : NQ) && tot != 0.f)
          atomic_add_f32(row + 16 * k + lf, tot);
      }
    }
    wave_sync_lds();
  }
}

// Backward with two pixels per lane (tile_size 16): wave w of the 2 owns
// the 16x8 band of rows 8w..8w+7, lane l the pixels (l & 15, 8w + (l >> 4))
// and 4 rows below.  Both pixels' gradient terms of a record are summed
// in-lane before the one reduce-scatter of the D + 15 fields, halving the
// cross-lane work, LDS reads and atomics per pixel (as bwd2_kernel of
// rasterize16.hip).  Same per-pixel arithmetic as bwd_kernel.
template <int D>
struct PixState {
  float T, tfvb, vc[D], buf[D], vn[3], bufn[3], vdist, accum_d, accum_w, accd_buf, accw_buf,
      dist_buf, vmed, fx, fy;
  int32_t bin_final, med_idx;
  bool inside;
};

// LEAN: v_render_normals, v_render_distort and v_render_median are null (the
// terms they feed are exact zeros, skipped): 26 fewer VGPRs of per-pixel state
// and no normal fields in the reduce-scatter.
// DBG (LEAN only, launched when gsplat_hip_debug_set_flags bits 0 / 2 / 3 or
// 6 -- this instance with nothing skipped -- are set): the timing-attribution instance (its checks cost 19 VGPRs, so the
// production instance does not carry them; held to the production's 4 waves
// per SIMD)
template <int D, bool ABS, bool LEAN = false, bool DBG = false>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(DBG ? 4 : 1)))
bwd2_kernel(RasterArgs a) {
  using R = Rec<D>;
  using F = Fields<D, ABS, LEAN>;
  extern __shared__ float4 lds4[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float *q = reinterpret_cast<float *>(lds4) + (size_t)w * 64 * R::NF;
  const int tile = order_tile(a);
  if (tile < 0) return;
  if (a.masks && !a.masks[tile]) return;
  const int ntile = a.tw * a.th;
  const int c = tile / ntile;
  const int rem = tile - c * ntile;
  const int ty = rem / a.tw, tx = rem - ty * a.tw;
  const int64_t start = a.offsets[tile];
  const int64_t tend = (tile == a.n_tiles - 1) ? (a.n_dev ? a.n_dev[0] : a.n_isects)
                                               : (int64_t)a.offsets[tile + 1];
  const float rx0 = tx * 16 + 0.5f, rx1 = rx0 + 15.f;
  const float ry0 = ty * 16 + 8 * w + 0.5f, ry1 = ry0 + 7.f;
  PixState<D> ps[2];
  int32_t wmax = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    PixState<D> &s = ps[k];
    const int px = tx * 16 + (lane & 15), py = ty * 16 + 8 * w + 4 * k + (lane >> 4);
    s.inside = px < a.W && py < a.H;
    const int64_t pid = (int64_t)c * a.H * a.W + (s.inside ? (int64_t)py * a.W + px : 0);
    s.fx = (float)px + 0.5f;
    s.fy = (float)py + 0.5f;
    const float Tf = 1.f - a.render_alphas[pid];
    s.T = Tf;
    s.bin_final = s.inside ? a.last_ids[pid] : 0;
    s.med_idx = (!LEAN && s.inside) ? a.median_ids[pid] : 0;  // LEAN: may be null
    float bg_dot = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      s.vc[d] = a.v_render_colors[pid * D + d];
      s.buf[d] = 0.f;
      if (a.backgrounds) bg_dot += a.backgrounds[(int64_t)c * D + d] * s.vc[d];
    }
    s.tfvb = Tf * ((a.v_render_alphas ? a.v_render_alphas[pid] : 0.f) - bg_dot);
    if (!LEAN) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        s.vn[i] = a.v_render_normals ? a.v_render_normals[pid * 3 + i] : 0.f;
        s.bufn[i] = 0.f;
      }
      s.vdist = a.v_render_distort ? a.v_render_distort[pid] : 0.f;
      s.accum_d = a.render_colors[pid * D + D - 1];
      s.accum_w = 1.f - Tf;
      s.accd_buf = s.accum_d;
      s.accw_buf = s.accum_w;
      s.dist_buf = 0.f;
      s.vmed = a.v_render_median ? a.v_render_median[pid] : 0.f;
    }
    wmax = max(wmax, s.bin_final);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) wmax = max(wmax, __shfl_xor(wmax, m, 64));
  const int64_t end = min(tend, (int64_t)wmax + 1);
  const int lf = rs_field(lane);
  // LEAN: the two pixels' state as packed pairs (.x pixel 0, .y pixel 1)
  f2v T2 = f2v{ps[0].T, ps[1].T}, tfvb2 = f2v{ps[0].tfvb, ps[1].tfvb};
  f2v buf2[D], vc2[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    buf2[d] = f2v{0.f, 0.f};
    vc2[d] = f2v{ps[0].vc[d], ps[1].vc[d]};
  }

  // LEAN: the next batch's surfel ids loaded while this one composites (the
  // batch's gathers then wait one global load, not two), and no normals
  // gathered (their record fields are never read)
  int32_t gid_next = 0;
  if (LEAN && end > start) {
    const int64_t j = max(start, end - 64) + lane;
    gid_next = j < end ? a.flatten_ids[j] : 0;
  }
  for (int64_t b1 = end; b1 > start; b1 -= 64) {
    const int64_t b0 = max(start, b1 - 64);
    int n;
    {
      Gathered<D> g;
      const int64_t j = b0 + lane;
      if constexpr (LEAN) {
        gather_at<D, false>(a, gid_next, g);
        const int64_t b1n = b1 - 64;
        if (b1n > start) {
          const int64_t jn = max(start, b1n - 64) + lane;
          gid_next = jn < b1n ? a.flatten_ids[jn] : 0;
        }
      } else {
        gather<D>(a, j, j < b1, g);
      }
      const bool keep = (j < b1) && surfel_keep(g.m, g.xy.x, g.xy.y, g.op, rx0, rx1, ry0, ry1);
      const uint64_t km = __ballot(keep);
      n = __popcll(km);
      if (keep) stage<D>(q + ballot_slot(km) * R::NF, g, (int32_t)j);
    }
    wave_sync_lds();
    for (int t = n - 1; t >= 0; --t) {
      float r[R::NF];
      read_rec<D>(q + t * R::NF, r);
      const int32_t idx = __float_as_int(r[R::IDX]);
      const float *m = r + R::M;
      Hit h[2];
      bool valid[2];
      if constexpr (LEAN) {
        // both pixels as one packed pair: same column fx (h_u = fx w - u
        // shared), rows fy0 / fy1; the reference's cross product h_u x h_v
        const float fx = ps[0].fx;
        const f2v fy = f2v{ps[0].fy, ps[1].fy};
        float hu[3];
        f2v hv[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          hu[i] = fx * m[6 + i] - m[i];
          hv[i] = __builtin_elementwise_fma(fy, f2v{m[6 + i], m[6 + i]}, f2v{-m[3 + i], -m[3 + i]});
        }
        f2v rc[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
          rc[i] = f2v{hu[i1], hu[i1]} * hv[i2] - f2v{hu[i2], hu[i2]} * hv[i1];
        }
        const f2v iz = f2v{__builtin_amdgcn_rcpf(rc[2].x), __builtin_amdgcn_rcpf(rc[2].y)};
        const f2v sx = rc[0] * iz, sy = rc[1] * iz;
        const f2v g3 = __builtin_elementwise_fma(sx, sx, sy * sy);
        const float dx = r[R::X] - fx;
        const f2v dy = f2v{r[R::Y], r[R::Y]} - fy;
        const f2v g2 = kFilterInvSquare * __builtin_elementwise_fma(dy, dy, f2v{dx * dx, dx * dx});
        const f2v sigma = 0.5f * f2v{fminf(g3.x, g2.x), fminf(g3.y, g2.y)};
        const f2v ex = sigma * -kLog2e;
        const f2v vis = f2v{__builtin_amdgcn_exp2f(ex.x), __builtin_amdgcn_exp2f(ex.y)};
        const f2v al = r[R::OP] * vis;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          h[k].s[0] = sx[k];
          h[k].s[1] = sy[k];
          h[k].rc[2] = rc[2][k];
          h[k].g3 = g3[k];
          h[k].g2 = g2[k];
          h[k].vis = vis[k];
          h[k].alpha = fminf(kAlphaMax, al[k]);
          h[k].ok = (rc[2][k] != 0.f) && !(sigma[k] < 0.f) && !(h[k].alpha < kAlphaMin);
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            h[k].hu[i] = hu[i];
            h[k].hv[i] = hv[i][k];
          }
          valid[k] = ps[k].inside && idx <= ps[k].bin_final && h[k].ok;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          h[k] = eval_hit(m, r[R::X], r[R::Y], r[R::OP], ps[k].fx, ps[k].fy);
          valid[k] = ps[k].inside && idx <= ps[k].bin_final && h[k].ok;
        }
      }
      if (__ballot(valid[0] | valid[1]) == 0) continue;
      float v[16 * F::NV];
      if constexpr (LEAN && !DBG) {
        // both pixels' gradient terms as packed pairs, branch-free: an
        // invalid pixel enters with alpha 0 (ra = 1, fac = 0: its T and
        // colour sums unchanged) and weight 0; the inputs of the branch not
        // taken are zeroed, so no inf / NaN of an unused branch reaches a sum
        const f2v al = f2v{valid[0] ? h[0].alpha : 0.f, valid[1] ? h[1].alpha : 0.f};
        const f2v vis = f2v{h[0].vis, h[1].vis};
        const f2v ra = f2v{__builtin_amdgcn_rcpf(1.f - al.x), __builtin_amdgcn_rcpf(1.f - al.y)};
        T2 = T2 * ra;
        const f2v fac = al * T2;
        f2v va = f2v{0.f, 0.f};
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const f2v cT = __builtin_elementwise_fma(f2v{r[R::COL + d], r[R::COL + d]}, T2,
                                                   -(buf2[d] * ra));
          va = __builtin_elementwise_fma(cT, vc2[d], va);
        }
        va = __builtin_elementwise_fma(ra, tfvb2, va);
        // pixels past the clamp (op * vis > kAlphaMax) take no opacity /
        // geometry gradient
        const float op = r[R::OP];
        const f2v wt = f2v{(valid[0] && op * h[0].vis <= kAlphaMax) ? va.x : 0.f,
                           (valid[1] && op * h[1].vis <= kAlphaMax) ? va.y : 0.f};
        const f2v vG = op * wt;
        const bool s0 = h[0].g3 <= h[0].g2, s1 = h[1].g3 <= h[1].g2;
        // the ray-splat branch (g3 <= g2): vrc from the UV-plane gradient
        const bool b0 = s0 && valid[0], b1 = s1 && valid[1];
        const f2v ssx = f2v{b0 ? h[0].s[0] : 0.f, b1 ? h[1].s[0] : 0.f};
        const f2v ssy = f2v{b0 ? h[0].s[1] : 0.f, b1 ? h[1].s[1] : 0.f};
        const f2v izs = f2v{b0 ? __builtin_amdgcn_rcpf(h[0].rc[2]) : 0.f,
                            b1 ? __builtin_amdgcn_rcpf(h[1].rc[2]) : 0.f};
        const f2v nvG = vG * -vis;
        const f2v ax = nvG * ssx * izs, ay = nvG * ssy * izs;
        const f2v vrc[3] = {ax, ay, -__builtin_elementwise_fma(ax, ssx, ay * ssy)};
        const float fx = ps[0].fx;
        const f2v fy = f2v{ps[0].fy, ps[1].fy};
        f2v hv[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) hv[i] = f2v{h[0].hv[i], h[1].hv[i]};
        const float *hu = h[0].hu;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
          const f2v vhu = hv[i1] * vrc[i2] - hv[i2] * vrc[i1];
          const f2v vhv = vrc[i1] * hu[i2] - vrc[i2] * hu[i1];
          const f2v t6 = __builtin_elementwise_fma(fy, vhv, fx * vhu);
          v[F::M + i] = -vhu.x - vhu.y;
          v[F::M + 3 + i] = -vhv.x - vhv.y;
          v[F::M + 6 + i] = t6.x + t6.y;
        }
        // the screen-space branch (g3 > g2): means2d
        const f2v vG2 = f2v{s0 ? 0.f : vG.x, s1 ? 0.f : vG.y};
        const float dx = r[R::X] - fx;
        const f2v dy = f2v{r[R::Y], r[R::Y]} - fy;
        const f2v nk = -vis * kFilterInvSquare;
        const f2v gx = vG2 * (nk * dx), gy = vG2 * (nk * dy);
        v[F::XY] = gx.x + gx.y;
        v[F::XY + 1] = gy.x + gy.y;
        if constexpr (ABS) {
          v[F::AB] = fabsf(gx.x) + fabsf(gx.y);
          v[F::AB + 1] = fabsf(gy.x) + fabsf(gy.y);
        }
        const f2v vo = vis * wt;
        v[F::OP] = vo.x + vo.y;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const f2v vcol = fac * vc2[d];
          v[F::COL + d] = vcol.x + vcol.y;
          buf2[d] = __builtin_elementwise_fma(f2v{r[R::COL + d], r[R::COL + d]}, fac, buf2[d]);
        }
#pragma unroll
        for (int kk = F::NF; kk < 16 * F::NV; ++kk) v[kk] = 0.f;
      } else {
#pragma unroll
      for (int kk = 0; kk < 16 * F::NV; ++kk) v[kk] = 0.f;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        PixState<D> &s = ps[k];
        const Hit &hk = h[k];
        if (!valid[k]) continue;
        if (!LEAN && idx == s.med_idx) v[F::COL + D - 1] += s.vmed;
        const float ra = __builtin_amdgcn_rcpf(1.f - hk.alpha);
        s.T *= ra;
        const float T = s.T;
        const float fac = hk.alpha * T;
        if (DBG && (a.dbg & 8)) {  // timing attribution only: no gradient algebra
          v[0] += fac;
          continue;
        }
        float v_alpha = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          v[F::COL + d] += fac * s.vc[d];
          v_alpha += (r[R::COL + d] * T - s.buf[d] * ra) * s.vc[d];
        }
        if (!LEAN) {
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            v[F::NRM + i] += fac * s.vn[i];
            v_alpha += (r[R::NRM + i] * T - s.bufn[i] * ra) * s.vn[i];
          }
        }
        v_alpha += ra * s.tfvb;
        if (!LEAN) {  // distortion (RasterizeToPixels2DGSBwd.cu:483-503)
          const float depth = r[R::COL + D - 1];
          const float dl_dw =
              2.f * (2.f * (depth * s.accw_buf - s.accd_buf) + (s.accum_d - depth * s.accum_w));
          v_alpha += (dl_dw * T - s.dist_buf * ra) * s.vdist;
          s.accd_buf -= fac * depth;
          s.accw_buf -= fac;
          s.dist_buf += dl_dw * fac;
          v[F::COL + D - 1] += 2.f * fac * (2.f - 2.f * T - s.accum_w + fac) * s.vdist;
        }
        if (r[R::OP] * hk.vis <= kAlphaMax) {
          const float vG = r[R::OP] * v_alpha;
          if (hk.g3 <= hk.g2) {
            const float vsx = vG * -hk.vis * hk.s[0], vsy = vG * -hk.vis * hk.s[1];
            const float iz = __builtin_amdgcn_rcpf(hk.rc[2]);
            const float ax = vsx * iz, ay = vsy * iz;
            const float vrc[3] = {ax, ay, -(ax * hk.s[0] + ay * hk.s[1])};
            const float vhu[3] = {hk.hv[1] * vrc[2] - hk.hv[2] * vrc[1],
                                  hk.hv[2] * vrc[0] - hk.hv[0] * vrc[2],
                                  hk.hv[0] * vrc[1] - hk.hv[1] * vrc[0]};
            const float vhv[3] = {vrc[1] * hk.hu[2] - vrc[2] * hk.hu[1],
                                  vrc[2] * hk.hu[0] - vrc[0] * hk.hu[2],
                                  vrc[0] * hk.hu[1] - vrc[1] * hk.hu[0]};
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              v[F::M + i] -= vhu[i];
              v[F::M + 3 + i] -= vhv[i];
              v[F::M + 6 + i] += s.fx * vhu[i] + s.fy * vhv[i];
            }
          } else {
            const float dx = r[R::X] - s.fx, dy = r[R::Y] - s.fy;
            const float gx = vG * (-hk.vis * kFilterInvSquare * dx);
            const float gy = vG * (-hk.vis * kFilterInvSquare * dy);
            v[F::XY] += gx;
            v[F::XY + 1] += gy;
            if constexpr (ABS) {
              v[F::AB] += fabsf(gx);
              v[F::AB + 1] += fabsf(gy);
            }
          }
          v[F::OP] += hk.vis * v_alpha;
        }
#pragma unroll
        for (int d = 0; d < D; ++d) s.buf[d] += r[R::COL + d] * fac;
        if (!LEAN) {
#pragma unroll
          for (int i = 0; i < 3; ++i) s.bufn[i] += r[R::NRM + i] * fac;
        }
      }
      }
      const int32_t g = __float_as_int(r[R::G]);
      float *row = a.packed + (int64_t)g * F::S;
#pragma unroll
      for (int kq = 0; kq < F::NV; ++kq) {
        constexpr int NQ = F::NF - 16 * (F::NV - 1);
        float tot;
        if (DBG && (a.dbg & 4)) {  // timing attribution only: the lane's own partial
          tot = v[16 * kq];
#pragma unroll
          for (int i = 1; i < 16; ++i)
            if (lf == i) tot = v[16 * kq + i];
        } else {
          tot = kq < F::NV - 1 ? reduce_scatter<16>(v + 16 * kq, lane)
                               : reduce_scatter<NQ>(v + 16 * kq, lane);
        }
        if ((lane & 3) == 0 && lf < (kq < F::NV - 1 ? 16 : NQ) && tot != 0.f &&
            !(DBG && (a.dbg & 1)))
          atomic_add_f32(row + 16 * kq + lf, tot);
      }
    }
    wave_sync_lds();
  }
}

// Zero the packed gradient rows of the visible surfels (the rows the
// backward's atomics can reach); one lane per row, S / 4 16-B stores.
__global__ void __launch_bounds__(256)
zero_rows_kernel(int64_t G, int S, const int32_t *__restrict__ visible, float *__restrict__ packed) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= G || visible[g] <= 0) return;
  float4 *r = reinterpret_cast<float4 *>(packed + g * S);
  for (int q = 0; q < S / 4; ++q) r[q] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// packed [G][S] -> autograd tensors; densify = (v_M[0][2], v_M[1][2]) * depth
// with depth = M[2][2] (the reference writes this racily from partial sums,
// RasterizeToPixels2DGSBwd.cu:689-697; here it is formed from the final sums).
template <int D, bool ABS, bool LEAN = false>
__global__ void __launch_bounds__(256)
unpack_kernel(int64_t G, const int32_t *__restrict__ visible, const float *__restrict__ packed,
              const float *__restrict__ rt,
              float *__restrict__ v_means2d, float *__restrict__ v_rt, float *__restrict__ v_colors,
              float *__restrict__ v_depths, float *__restrict__ v_opacities,
              float *__restrict__ v_normals, float *__restrict__ v_densify,
              float *__restrict__ v_abs) {
  using F = Fields<D, ABS, LEAN>;
  // v_depths (ABI 33, or null): the last channel's gradient there, v_colors
  // then [G, D - 1]
  const int DC = v_depths ? D - 1 : D;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  if (visible && visible[g] <= 0) {  // no isect: every gradient is zero (row never zeroed)
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d < DC) v_colors[g * DC + d] = 0.f;
    if (v_depths) v_depths[g] = 0.f;
    if (v_normals) {
#pragma unroll
      for (int i = 0; i < 3; ++i) v_normals[g * 3 + i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) v_rt[g * 9 + i] = 0.f;
    *reinterpret_cast<float2 *>(v_means2d + 2 * g) = make_float2(0.f, 0.f);
    v_opacities[g] = 0.f;
    *reinterpret_cast<float2 *>(v_densify + 2 * g) = make_float2(0.f, 0.f);
    if (ABS) *reinterpret_cast<float2 *>(v_abs + 2 * g) = make_float2(0.f, 0.f);
    return;
  }
  const float *r = packed + g * F::S;
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < DC) v_colors[g * DC + d] = r[F::COL + d];
  if (v_depths) v_depths[g] = r[F::COL + D - 1];
  if (v_normals) {  // null: the render's normals had no gradient (all zero)
#pragma unroll
    for (int i = 0; i < 3; ++i) v_normals[g * 3 + i] = LEAN ? 0.f : r[F::NRM + i];
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) v_rt[g * 9 + i] = r[F::M + i];
  *reinterpret_cast<float2 *>(v_means2d + 2 * g) = make_float2(r[F::XY], r[F::XY + 1]);
  v_opacities[g] = r[F::OP];
  const float depth = rt[g * 9 + 8];
  *reinterpret_cast<float2 *>(v_densify + 2 * g) =
      make_float2(r[F::M + 2] * depth, r[F::M + 5] * depth);
  if (ABS) *reinterpret_cast<float2 *>(v_abs + 2 * g) = make_float2(r[F::AB], r[F::AB + 1]);
}

}  // namespace surfel
}  // namespace gs

namespace gs {
int dbg_flags();  // rasterize16.hip: GSPLAT_HIP_DBG / gsplat_hip_debug_set_flags
}
using namespace gs;
using namespace gs::surfel;

namespace {

// Colour channel counts with compiled kernels (the caller pads others).
#define GS_SURFEL_CHANNELS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(16) X(17) X(32) X(33)

bool channels_supported(int D) {
#define GS_CASE(n) if (D == n) return true;
  GS_SURFEL_CHANNELS(GS_CASE)
#undef GS_CASE
  return false;
}

// 16x16 tiles: two pixels per lane in the forward and the backward (fwd2 /
// bwd2 kernels; the one-pixel kernels, which measured 1.62 / 1.76 against
// 1.10 / 1.63 ms at M5, serve the other tile sizes)
bool fwd2_enabled() { return true; }
// the XCD runs of the tile order (RasterArgs::xcd_runs; GSPLAT_HIP_DBG bit 4:
// one tile after the other, as the 3DGS rasterizer's flag)
int xcd_runs() { return !(gs::dbg_flags() & 16); }
bool bwd2_enabled() { return true; }

int fields_stride(int D, int absgrad) {
  const int nf = D + 15 + (absgrad ? 2 : 0);
  return 16 * ((nf + 15) / 16);
}

int lean_stride(int D, int absgrad) {  // Fields<D, ABS, true>::S
  const int nf = D + 12 + (absgrad ? 2 : 0);
  return 16 * ((nf + 15) / 16);
}

int check_tiles(int C, int W, int H, int ts, int tw, int th) {
  GS_REQUIRE(C >= 0 && W >= 0 && H >= 0, "rasterize_2dgs: negative sizes");
  GS_REQUIRE(ts >= 1 && ts <= 32, "rasterize_2dgs: tile_size %d not in [1, 32]", ts);
  GS_REQUIRE((int64_t)tw * ts >= W && (int64_t)th * ts >= H,
             "rasterize_2dgs: %dx%d tiles of %d do not cover %dx%d", tw, th, ts, W, H);
  return 0;
}

}  // namespace

extern "C" int gsplat_hip_projection_2dgs_fwd(int C, int N, const float *means, const float *quats,
                                              const float *scales, const float *viewmats,
                                              const float *Ks, int width, int height,
                                              float near_plane, float far_plane,
                                              float radius_clip, int32_t *radii, float *means2d,
                                              float *depths, float *ray_transforms,
                                              float *normals, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "projection_2dgs_fwd: negative sizes C=%d N=%d", C, N);
  if (C == 0 || N == 0) return 0;
  GS_REQUIRE(means && quats && scales && viewmats && Ks && radii && means2d && depths &&
                 ray_transforms && normals,
             "projection_2dgs_fwd: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)means2d & 7) == 0,
             "projection_2dgs_fwd: quats must be 16-B aligned, means2d 8-B aligned");
  ProjFwdArgs a{C, N, width, height, near_plane, far_plane, radius_clip, means, quats, scales,
                viewmats, Ks, radii, means2d, depths, ray_transforms, normals};
  hipLaunchKernelGGL(proj_fwd_kernel<0>, dim3((N + 255) / 256, C), dim3(256), 0,
                     (hipStream_t)stream, a);
  GS_CHECK_LAUNCH("projection_2dgs_fwd");
  return 0;
}

extern "C" int gsplat_hip_projection_2dgs_bwd(
    int C, int N, const float *means, const float *quats, const float *scales,
    const float *viewmats, const float *Ks, int width, int height, const int32_t *radii,
    const float *ray_transforms, const float *v_means2d, const float *v_depths,
    const float *v_normals, const float *v_ray_transforms, float *v_means, float *v_quats,
    float *v_scales, float *v_viewmats, void *stream) {
  (void)width;
  (void)height;
  GS_REQUIRE(C >= 0 && N >= 0, "projection_2dgs_bwd: negative sizes C=%d N=%d", C, N);
  hipStream_t st = (hipStream_t)stream;
  // the reference allocates v_viewmats but its kernel never writes it
  // (Projection2DGSFused.cu:319-457): zeros
  if (v_viewmats && C > 0) GS_HIP(gs::zero_async(v_viewmats, sizeof(float) * 16 * C, st));
  if (N == 0) return 0;
  const int store_mode = (C == 1);
  if (!store_mode) {
    GS_HIP(gs::zero_async(v_means, sizeof(float) * 3 * N, st));
    GS_HIP(gs::zero_async(v_quats, sizeof(float) * 4 * N, st));
    GS_HIP(gs::zero_async(v_scales, sizeof(float) * 3 * N, st));
  }
  if (C == 0) return 0;
  GS_REQUIRE(means && quats && scales && viewmats && Ks && radii && ray_transforms &&
                 v_means2d && v_ray_transforms && v_means && v_quats && v_scales,
             "projection_2dgs_bwd: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)v_quats & 15) == 0,
             "projection_2dgs_bwd: quats / v_quats must be 16-B aligned");
  ProjBwdArgs a{C, N, means, quats, scales, viewmats, Ks, radii, ray_transforms, v_means2d,
                v_depths, v_normals, v_ray_transforms, v_means, v_quats, v_scales, store_mode};
  hipLaunchKernelGGL(proj_bwd_kernel, dim3((N + 255) / 256, C), dim3(256), 0, st, a);
  GS_CHECK_LAUNCH("projection_2dgs_bwd");
  return 0;
}

// gsplat_hip_projection_2dgs_bwd with the geometry groups' Adam step fused in
// (ABI 33; geom_adam.h, as gsplat_hip_projection_bwd_adam for 3DGS): one
// camera; params / exp_avgs / exp_avg_sqs are [means, log_scales, quats,
// logits]; lrs[4] with the 1-based step, or hyper_device f32[8]; skip_device
// may be NULL.  No gradient is stored.
extern "C" int gsplat_hip_projection_2dgs_bwd_adam(
    int N, const float *means, const float *quats, const float *scales, const float *viewmats,
    const float *Ks, const int32_t *radii, const float *ray_transforms, const float *v_means2d,
    const float *v_depths, const float *v_normals, const float *v_ray_transforms,
    const float *v_dirs, const float *v_opac, const float *opac, float *const *params,
    float *const *exp_avgs, float *const *exp_avg_sqs, const float *lrs, float beta1,
    float beta2, float eps, int step, const float *hyper_device, const int32_t *skip_device,
    void *stream) {
  GS_REQUIRE(N >= 0, "projection_2dgs_bwd_adam: negative N=%d", N);
  if (N == 0) return 0;
  GS_REQUIRE(means && quats && scales && viewmats && Ks && radii && ray_transforms &&
                 v_means2d && v_ray_transforms,
             "projection_2dgs_bwd_adam: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0, "projection_2dgs_bwd_adam: quats must be 16-B aligned");
  GeomAdam ga;
  if (int e = geom_adam_setup(ga, params, exp_avgs, exp_avg_sqs, lrs, beta1, beta2, eps, step,
                              hyper_device, skip_device, v_dirs, v_opac, opac,
                              "projection_2dgs_bwd_adam"))
    return e;
  ProjBwdArgs a{1, N, means, quats, scales, viewmats, Ks, radii, ray_transforms, v_means2d,
                v_depths, v_normals, v_ray_transforms, nullptr, nullptr, nullptr, 1};
  a.ga = ga;
  hipLaunchKernelGGL(proj_bwd_kernel, dim3((N + 255) / 256, 1), dim3(256), 0,
                     (hipStream_t)stream, a);
  GS_CHECK_LAUNCH("projection_2dgs_bwd_adam");
  return 0;
}

// ------------------------------------------------------------------ packed --
// projection_2dgs_packed_fwd (gsplat/cuda/csrc/Projection2DGSPacked.cu:17-270):
// a counting pass, a scan of the per-block counts and a pass that recomputes
// and writes the kept (camera, surfel) pairs in (camera, surfel) order.
namespace gs {
void launch_packed_scan(int64_t nb, int64_t *cnt, int64_t *total, hipStream_t st);
}

extern "C" int64_t gsplat_hip_projection_2dgs_packed_workspace_bytes(int C, int N) {
  const int64_t nb = (int64_t)C * ((N + 255) / 256);
  return (nb + 1) * (int64_t)sizeof(int64_t);
}

extern "C" int gsplat_hip_projection_2dgs_packed_count(
    int C, int N, const float *means, const float *quats, const float *scales,
    const float *viewmats, const float *Ks, int width, int height, float near_plane,
    float far_plane, float radius_clip, void *workspace, int64_t *nnz_device, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "projection_2dgs_packed_count: negative sizes C=%d N=%d", C, N);
  hipStream_t st = (hipStream_t)stream;
  if (C == 0 || N == 0) {
    GS_HIP(gs::zero_async(nnz_device, sizeof(int64_t), st));
    return 0;
  }
  GS_REQUIRE(means && quats && scales && viewmats && Ks && workspace && nnz_device,
             "projection_2dgs_packed_count: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0,
             "projection_2dgs_packed_count: quats must be 16-B aligned");
  ProjFwdArgs a{C, N, width, height, near_plane, far_plane, radius_clip, means, quats, scales,
                viewmats, Ks};
  a.block_cnt = reinterpret_cast<int64_t *>(workspace);
  const dim3 grid((N + 255) / 256, C);
  hipLaunchKernelGGL(proj_fwd_kernel<1>, grid, dim3(256), 0, st, a);
  gs::launch_packed_scan((int64_t)grid.x * grid.y, a.block_cnt, nnz_device, st);
  GS_CHECK_LAUNCH("projection_2dgs_packed_count");
  return 0;
}

extern "C" int gsplat_hip_projection_2dgs_packed_fwd(
    int C, int N, const float *means, const float *quats, const float *scales,
    const float *viewmats, const float *Ks, int width, int height, float near_plane,
    float far_plane, float radius_clip, const void *workspace, int64_t *camera_ids,
    int64_t *gaussian_ids, int32_t *radii, float *means2d, float *depths, float *ray_transforms,
    float *normals, void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "projection_2dgs_packed_fwd: negative sizes C=%d N=%d", C, N);
  if (C == 0 || N == 0) return 0;
  GS_REQUIRE(means && quats && scales && viewmats && Ks && workspace && camera_ids &&
                 gaussian_ids && radii && means2d && depths && ray_transforms && normals,
             "projection_2dgs_packed_fwd: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)means2d & 7) == 0,
             "projection_2dgs_packed_fwd: quats must be 16-B aligned, means2d 8-B aligned");
  ProjFwdArgs a{C, N, width, height, near_plane, far_plane, radius_clip, means, quats, scales,
                viewmats, Ks, radii, means2d, depths, ray_transforms, normals};
  a.block_off = reinterpret_cast<const int64_t *>(workspace);
  a.camera_ids = camera_ids;
  a.gaussian_ids = gaussian_ids;
  hipLaunchKernelGGL(proj_fwd_kernel<2>, dim3((N + 255) / 256, C), dim3(256), 0,
                     (hipStream_t)stream, a);
  GS_CHECK_LAUNCH("projection_2dgs_packed_fwd");
  return 0;
}

// projection_2dgs_packed_bwd (Projection2DGSPacked.cu:274-420): one lane per
// packed entry; dense [N, .] gradients by atomics, or (sparse_grad) one row
// per entry for the COO gradients of _wrapper.py:1529-1570.  v_viewmats, as
// in the reference, is not differentiated (zeros).
extern "C" int gsplat_hip_projection_2dgs_packed_bwd(
    int C, int N, int64_t nnz, const float *means, const float *quats, const float *scales,
    const float *viewmats, const float *Ks, int width, int height, const int64_t *camera_ids,
    const int64_t *gaussian_ids, const float *ray_transforms, const float *v_means2d,
    const float *v_depths, const float *v_normals, const float *v_ray_transforms,
    int sparse_grad, float *v_means, float *v_quats, float *v_scales, float *v_viewmats,
    void *stream) {
  (void)width;
  (void)height;
  GS_REQUIRE(C >= 0 && N >= 0 && nnz >= 0, "projection_2dgs_packed_bwd: negative sizes");
  hipStream_t st = (hipStream_t)stream;
  if (v_viewmats && C > 0) GS_HIP(gs::zero_async(v_viewmats, sizeof(float) * 16 * C, st));
  if (!sparse_grad && N > 0) {
    GS_HIP(gs::zero_async(v_means, sizeof(float) * 3 * N, st));
    GS_HIP(gs::zero_async(v_quats, sizeof(float) * 4 * N, st));
    GS_HIP(gs::zero_async(v_scales, sizeof(float) * 3 * N, st));
  }
  if (nnz == 0) return 0;
  GS_REQUIRE(means && quats && scales && viewmats && Ks && camera_ids && gaussian_ids &&
                 ray_transforms && v_means2d && v_normals && v_ray_transforms && v_means &&
                 v_quats && v_scales,
             "projection_2dgs_packed_bwd: null pointer argument");
  GS_REQUIRE(((uintptr_t)quats & 15) == 0 && ((uintptr_t)v_quats & 15) == 0,
             "projection_2dgs_packed_bwd: quats / v_quats must be 16-B aligned");
  ProjBwdArgs a{C, N, means, quats, scales, viewmats, Ks, nullptr, ray_transforms, v_means2d,
                v_depths, v_normals, v_ray_transforms, v_means, v_quats, v_scales, 0};
  a.camera_ids = camera_ids;
  a.gaussian_ids = gaussian_ids;
  a.nnz = nnz;
  a.sparse = sparse_grad;
  hipLaunchKernelGGL(proj_bwd_kernel, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, st, a);
  GS_CHECK_LAUNCH("projection_2dgs_packed_bwd");
  return 0;
}

extern "C" int gsplat_hip_rasterize_2dgs_supported_channels(int D) {
  return channels_supported(D) ? 1 : 0;
}

extern "C" int gsplat_hip_rasterize_2dgs_fwd(
    int C, int D, int width, int height, int tile_size, int tile_width, int tile_height,
    const float *means2d, const float *ray_transforms, const float *colors, const float *depths,
    const float *opacities, const float *normals, const float *backgrounds,
    const uint8_t *masks, const int32_t *isect_offsets, int64_t n_isects,
    const int64_t *n_isects_device, const int32_t *flatten_ids, const float *records,
    int32_t *tile_order, float *render_colors, float *render_alphas, float *render_normals,
    float *render_distort, float *render_median, int32_t *last_ids, int32_t *median_ids,
    void *stream) {
  if (int e = check_tiles(C, width, height, tile_size, tile_width, tile_height)) return e;
  GS_REQUIRE(channels_supported(D), "rasterize_2dgs_fwd: unsupported channel count %d", D);
  const int n_tiles = C * tile_width * tile_height;
  if (n_tiles == 0 || width == 0 || height == 0) return 0;
  // a colours-only render (ABI 33): render_normals, render_distort,
  // render_median and median_ids all null -- the record path forms the
  // colours, alphas and last ids alone (its backward then takes no gradient
  // of the other outputs)
  const bool lean = !render_normals && !render_distort && !render_median && !median_ids;
  GS_REQUIRE(isect_offsets && render_colors && render_alphas && last_ids &&
                 (lean || (render_normals && render_distort && render_median && median_ids)),
             "rasterize_2dgs_fwd: null pointer argument");
  GS_REQUIRE(!lean || (records && tile_size == 16 && fwd2_enabled()),
             "rasterize_2dgs_fwd: a colours-only render needs the record path (16x16 tiles, D <= %d)",
             kSRecMaxD);
  GS_REQUIRE(n_isects == 0 || (means2d && ray_transforms && colors && opacities && normals &&
                               flatten_ids),
             "rasterize_2dgs_fwd: null pointer argument");
  GS_REQUIRE(((uintptr_t)means2d & 7) == 0, "rasterize_2dgs_fwd: means2d must be 8-B aligned");
  RasterArgs a{};
  a.C = C; a.W = width; a.H = height; a.ts = tile_size; a.tw = tile_width; a.th = tile_height;
  a.n_tiles = n_tiles; a.n_isects = n_isects; a.n_dev = n_isects_device;
  a.means2d = means2d; a.ray_transforms = ray_transforms; a.colors = colors; a.depths = depths;
  a.opacities = opacities; a.normals = normals; a.backgrounds = backgrounds; a.masks = masks;
  a.offsets = isect_offsets; a.flatten_ids = flatten_ids;
  a.render_colors = render_colors; a.render_alphas = render_alphas;
  a.render_normals = render_normals; a.render_distort = render_distort;
  a.render_median = render_median; a.last_ids = last_ids; a.median_ids = median_ids;
  const int waves = (tile_size * tile_size + 63) / 64;
  hipStream_t st = (hipStream_t)stream;
  unsigned grid_t = (unsigned)n_tiles;
  if (tile_order && n_tiles > 0) {  // written here, read by this launch and the backward
    hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, st, n_tiles, isect_offsets,
                       n_isects, n_isects_device, tile_order);
    a.order = tile_order;
    a.xcd_runs = xcd_runs();
    if (a.xcd_runs) grid_t = (unsigned)((n_tiles + 31) / 32 * 32);
  }
  // 16x16 tiles: two pixels per lane (fwd2_kernel)
  const bool px2 = tile_size == 16 && fwd2_enabled();
  if (records) {  // scalar-operand records (gsplat_hip_rasterize_2dgs_pack_records)
    GS_REQUIRE(px2 && D <= kSRecMaxD, "rasterize_2dgs_fwd: records need 16x16 tiles, D <= %d",
               kSRecMaxD);
#define GS_CASE(n)                                                                            \
  if (D == n && lean)                                                                         \
    hipLaunchKernelGGL((fwd2s_kernel<n, true>), dim3(grid_t), dim3(128), 0, st, a, records); \
  else if (D == n)                                                                            \
    hipLaunchKernelGGL((fwd2s_kernel<n, false>), dim3(grid_t), dim3(128), 0, st, a, records);
    GS_CASE(1) GS_CASE(2) GS_CASE(3) GS_CASE(4)
#undef GS_CASE
    GS_CHECK_LAUNCH("rasterize_2dgs_fwd");
    return 0;
  }
#define GS_CASE(n)                                                                            \
  if (D == n) {                                                                               \
    const size_t lds = (size_t)waves * 64 * Rec<n>::NF * sizeof(float);                       \
    if (px2)                                                                                  \
      hipLaunchKernelGGL(fwd2_kernel<n>, dim3(grid_t), dim3(128), lds / 2, st, a);           \
    else                                                                                      \
      hipLaunchKernelGGL(fwd_kernel<n>, dim3(grid_t), dim3(64 * waves), lds, st, a);         \
  }
  GS_SURFEL_CHANNELS(GS_CASE)
#undef GS_CASE
  GS_CHECK_LAUNCH("rasterize_2dgs_fwd");
  return 0;
}

extern "C" int gsplat_hip_rasterize_2dgs_record_floats(int D, int tile_size) {
  return (tile_size == 16 && D >= 1 && D <= kSRecMaxD && fwd2_enabled()) ? srec::NF : 0;
}

extern "C" int gsplat_hip_rasterize_2dgs_pack_records(int64_t n_gaussians, int D,
                                                      const float *means2d,
                                                      const float *ray_transforms,
                                                      const float *opacities, const float *normals,
                                                      const float *colors, const float *depths,
                                                      const int32_t *visible, float *records,
                                                      void *stream) {
  GS_REQUIRE(D >= 1 && D <= kSRecMaxD, "rasterize_2dgs_pack_records: D %d not in [1, %d]", D,
             kSRecMaxD);
  GS_REQUIRE(n_gaussians >= 0, "rasterize_2dgs_pack_records: negative count");
  if (n_gaussians == 0) return 0;
  GS_REQUIRE(means2d && ray_transforms && opacities && normals && colors && records,
             "rasterize_2dgs_pack_records: null pointer argument");
  GS_REQUIRE(((uintptr_t)records & 15) == 0, "rasterize_2dgs_pack_records: records not 16-B aligned");
  const dim3 grid((unsigned)((n_gaussians + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
#define GS_CASE(n)                                                                            \
  if (D == n)                                                                                 \
    hipLaunchKernelGGL(pack_srec_kernel<n>, grid, dim3(256), 0, st, n_gaussians, means2d,     \
                       ray_transforms, opacities, normals, colors, depths, visible, records);
  GS_CASE(1) GS_CASE(2) GS_CASE(3) GS_CASE(4)
#undef GS_CASE
  GS_CHECK_LAUNCH("rasterize_2dgs_pack_records");
  return 0;
}

extern "C" int64_t gsplat_hip_rasterize_2dgs_bwd_workspace_bytes(int64_t n_gaussians, int D,
                                                                 int absgrad) {
  return n_gaussians * fields_stride(D, absgrad) * (int64_t)sizeof(float);
}

extern "C" int gsplat_hip_rasterize_2dgs_bwd(
    int C, int D, int width, int height, int tile_size, int tile_width, int tile_height,
    int64_t n_gaussians, const float *means2d, const float *ray_transforms, const float *colors,
    const float *depths, const float *opacities, const float *normals, const float *backgrounds,
    const uint8_t *masks, const int32_t *isect_offsets, int64_t n_isects,
    const int64_t *n_isects_device, const int32_t *flatten_ids, const int32_t *tile_order,
    const int32_t *visible, const float *render_colors, const float *render_alphas,
    const int32_t *last_ids,
    const int32_t *median_ids, const float *v_render_colors,
    const float *v_render_alphas, const float *v_render_normals, const float *v_render_distort,
    const float *v_render_median, float *v_means2d, float *v_ray_transforms, float *v_colors,
    float *v_depths, float *v_opacities, float *v_normals, float *v_densify,
    float *v_means2d_abs, void *workspace, int64_t workspace_bytes, void *stream) {
  if (int e = check_tiles(C, width, height, tile_size, tile_width, tile_height)) return e;
  GS_REQUIRE(!depths == !v_depths, "rasterize_2dgs_bwd: depths and v_depths: both or neither");
  GS_REQUIRE(channels_supported(D), "rasterize_2dgs_bwd: unsupported channel count %d", D);
  GS_REQUIRE(tile_size * tile_size <= 256, "rasterize_2dgs_bwd: tile_size %d > 16", tile_size);
  const int absgrad = v_means2d_abs != nullptr;
  // LEAN kernels (bwd2_kernel, 16x16 tiles, D <= 4) whenever no normal / distortion / median gradient is
  // asked for (a colours-only forward, which writes no median ids, has only
  // that backward)
  const bool px2 = tile_size == 16 && bwd2_enabled();
  const bool lean = px2 && D <= 4 && !v_render_normals && !v_render_distort && !v_render_median;
  const int S = lean ? lean_stride(D, absgrad) : fields_stride(D, absgrad);
  const int64_t G = n_gaussians;
  GS_REQUIRE(workspace_bytes >= G * S * (int64_t)sizeof(float),
             "rasterize_2dgs_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (G == 0) return 0;
  GS_REQUIRE(workspace && v_means2d && v_ray_transforms && v_colors && v_opacities &&
                 v_densify && ray_transforms,
             "rasterize_2dgs_bwd: null pointer argument");
  if (visible)
    hipLaunchKernelGGL(zero_rows_kernel, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, st, G, S,
                       visible, (float *)workspace);
  else
    GS_HIP(gs::zero_async(workspace, (size_t)G * S * sizeof(float), st));
  const int n_tiles = C * tile_width * tile_height;
  if (n_tiles > 0 && n_isects > 0 && width > 0 && height > 0) {
    GS_REQUIRE(isect_offsets && flatten_ids && render_colors && render_alphas && last_ids &&
                   (median_ids || lean) && v_render_colors,
               "rasterize_2dgs_bwd: null pointer argument (median_ids: null only for a "
               "colours-only render's backward)");
    RasterArgs a{};
    a.dbg = gs::dbg_flags();
    a.C = C; a.W = width; a.H = height; a.ts = tile_size; a.tw = tile_width;
    a.th = tile_height; a.n_tiles = n_tiles; a.n_isects = n_isects; a.n_dev = n_isects_device;
    a.order = tile_order;
    a.xcd_runs = tile_order ? xcd_runs() : 0;
    const unsigned grid_t =
        a.xcd_runs ? (unsigned)((n_tiles + 31) / 32 * 32) : (unsigned)n_tiles;
    a.means2d = means2d; a.ray_transforms = ray_transforms; a.colors = colors; a.depths = depths;
    a.opacities = opacities; a.normals = normals; a.backgrounds = backgrounds; a.masks = masks;
    a.offsets = isect_offsets; a.flatten_ids = flatten_ids;
    a.render_colors = const_cast<float *>(render_colors);
    a.render_alphas = const_cast<float *>(render_alphas);
    a.last_ids = const_cast<int32_t *>(last_ids);
    a.median_ids = const_cast<int32_t *>(median_ids);
    a.v_render_colors = v_render_colors; a.v_render_alphas = v_render_alphas;
    a.v_render_normals = v_render_normals; a.v_render_distort = v_render_distort;
    a.v_render_median = v_render_median;
    a.packed = (float *)workspace; a.S = S;
    const int waves = (tile_size * tile_size + 63) / 64;
    // 16x16 tiles: two pixels per lane (bwd2_kernel)
#define GS_CASE(n)                                                                            \
  if (D == n) {                                                                               \
    const size_t lds = (size_t)waves * 64 * Rec<n>::NF * sizeof(float);                       \
    if (lean && absgrad)                                                                      \
      hipLaunchKernelGGL((bwd2_kernel<n <= 4 ? n : 4, true, true>), dim3(grid_t), dim3(128), \
                         lds / 2, st, a);                                                     \
    else if (lean && (a.dbg & 77))                                                            \
      hipLaunchKernelGGL((bwd2_kernel<n <= 4 ? n : 4, false, true, true>), dim3(grid_t),     \
                         dim3(128), lds / 2, st, a);                                          \
    else if (lean)                                                                            \
      hipLaunchKernelGGL((bwd2_kernel<n <= 4 ? n : 4, false, true>), dim3(grid_t), dim3(128),\
                         lds / 2, st, a);                                                     \
    else if (px2 && absgrad)                                                                       \
      hipLaunchKernelGGL((bwd2_kernel<n, true>), dim3(grid_t), dim3(128), lds / 2, st, a);    \
    else if (px2)                                                                             \
      hipLaunchKernelGGL((bwd2_kernel<n, false>), dim3(grid_t), dim3(128), lds / 2, st, a);   \
    else if (absgrad)                                                                         \
      hipLaunchKernelGGL((bwd_kernel<n, true>), dim3(grid_t), dim3(64 * waves), lds, st, a);  \
    else                                                                                      \
      hipLaunchKernelGGL((bwd_kernel<n, false>), dim3(grid_t), dim3(64 * waves), lds, st, a); \
  }
    GS_SURFEL_CHANNELS(GS_CASE)
#undef GS_CASE
    GS_CHECK_LAUNCH("rasterize_2dgs_bwd");
  }
  const dim3 grid((unsigned)((G + 255) / 256));
#define GS_CASE(n)                                                                             \
  if (D == n && lean) {                                                                        \
    if (absgrad)                                                                               \
      hipLaunchKernelGGL((unpack_kernel<n <= 4 ? n : 4, true, true>), grid, dim3(256), 0, st, G, \
                         visible, (const float *)workspace, ray_transforms, v_means2d,         \
                         v_ray_transforms, v_colors, v_depths, v_opacities, v_normals, v_densify,\
                         v_means2d_abs);                                                       \
    else                                                                                       \
      hipLaunchKernelGGL((unpack_kernel<n <= 4 ? n : 4, false, true>), grid, dim3(256), 0, st, G,\
                         visible, (const float *)workspace, ray_transforms, v_means2d,         \
                         v_ray_transforms, v_colors, v_depths, v_opacities, v_normals, v_densify,\
                         v_means2d_abs);                                                       \
  } else if (D == n) {                                                                         \
    if (absgrad)                                                                               \
      hipLaunchKernelGGL((unpack_kernel<n, true>), grid, dim3(256), 0, st, G, visible, (const float *)workspace, \
                         ray_transforms, v_means2d, v_ray_transforms, v_colors, v_depths, v_opacities,\
                         v_normals, v_densify, v_means2d_abs);                                 \
    else                                                                                       \
      hipLaunchKernelGGL((unpack_kernel<n, false>), grid, dim3(256), 0, st, G, visible, (const float *)workspace, \
                         ray_transforms, v_means2d, v_ray_transforms, v_colors, v_depths, v_opacities,\
                         v_normals, v_densify, v_means2d_abs);                                 \
  }
  GS_SURFEL_CHANNELS(GS_CASE)
#undef GS_CASE
  GS_CHECK_LAUNCH("rasterize_2dgs_unpack");
  return 0;
}
