// Tile rasterizer: front-to-back alpha compositing (forward) and its reverse
// sweep (backward) for gfx950.
//
// Replaces the reference Triton kernels
//   rasterize_to_pixels_fwd_kernel  gsplat/triton_impl/rasterize_to_pixels_fwd.py:13-196
//   rasterize_to_pixels_bwd_kernel  gsplat/triton_impl/rasterize_to_pixels_bwd.py:13-337
//
// Mapping (CDNA4): one workgroup per image tile, one lane per pixel (16x16
// tile = 4 wave64s).  The tile's depth-sorted Gaussian list is streamed
// through LDS in batches of up to 256 records staged with one coalesced
// gather per lane (id -> xy, conic+opacity, D colours); every lane then reads
// each record with a broadcast ds_read.  The forward keeps transmittance
// multiplicatively (T *= 1 - alpha) with the reference's exclusive stop at
// T <= 1e-4; `last_ids` is the global isect index of the last contributor.
// The backward walks the same records back to front, rebuilding T from
// T_final, and reduces every per-Gaussian gradient across the wave with a
// butterfly before one fp32 atomic per wave and field.
#include "common.h"
#include "../../include/gsplat_hip.h"

namespace gs {

constexpr int kMaxBatch = 256;
constexpr float kAlphaMin = 1.f / 255.f;
constexpr float kAlphaMax = 0.999f;
constexpr float kTMin = 1e-4f;

struct RasterArgs {
  int C, W, H, ts, tw, th;
  int64_t n_isects;
  const float *means2d, *conics, *colors, *opacities, *backgrounds;  // backgrounds nullable
  const uint8_t *masks;                                              // nullable
  const int32_t *offsets, *flatten_ids;
  // forward outputs / backward inputs
  float *render_colors, *render_alphas;
  int32_t *last_ids;
  // backward
  const float *v_render_colors, *v_render_alphas;
  float *v_means2d, *v_conics, *v_colors, *v_opacities, *v_means2d_abs;  // abs nullable
};

struct TileCtx {
  int c, tile, px, py;
  bool inside;
  int64_t start, end;
};

GS_INLINE TileCtx tile_ctx(const RasterArgs &a) {
  TileCtx t;
  const int ntile = a.tw * a.th;
  t.tile = blockIdx.x;
  t.c = t.tile / ntile;
  const int rem = t.tile - t.c * ntile;
  const int ty = rem / a.tw, tx = rem - ty * a.tw;
  const int npx = a.ts * a.ts;
  const int lid = threadIdx.x;
  const int ly = lid / a.ts, lx = lid - ly * a.ts;
  t.px = tx * a.ts + lx;
  t.py = ty * a.ts + ly;
  t.inside = (lid < npx) && (t.px < a.W) && (t.py < a.H);
  t.start = a.offsets[t.tile];
  t.end = (t.tile == a.C * ntile - 1) ? a.n_isects : (int64_t)a.offsets[t.tile + 1];
  return t;
}

template <int D>
struct Stage {
  float2 xy[kMaxBatch];
  float4 con[kMaxBatch];  // conic a, b, c, opacity
  float col[kMaxBatch][D];
  int32_t gid[kMaxBatch];
};

template <int D>
GS_INLINE void stage_batch(const RasterArgs &a, Stage<D> &s, int64_t b0, int nb) {
  const int j = threadIdx.x;
  if (j < nb) {
    const int32_t g = a.flatten_ids[b0 + j];
    s.gid[j] = g;
    s.xy[j] = *reinterpret_cast<const float2 *>(a.means2d + 2 * (int64_t)g);
    const float *cn = a.conics + 3 * (int64_t)g;
    s.con[j] = make_float4(cn[0], cn[1], cn[2], a.opacities[g]);
    const float *cl = a.colors + (int64_t)g * D;
#pragma unroll
    for (int d = 0; d < D; ++d) s.col[j][d] = cl[d];
  }
}

template <int D>
__global__ void __launch_bounds__(256) rasterize_fwd_kernel(RasterArgs a) {
  __shared__ Stage<D> s;
  const TileCtx t = tile_ctx(a);
  const int batch = min((int)blockDim.x, kMaxBatch);
  const int64_t pix = ((int64_t)t.c * a.H + t.py) * a.W + t.px;

  float T = 1.f;
  float acc[D];
#pragma unroll
  for (int d = 0; d < D; ++d) acc[d] = 0.f;
  int32_t last = 0;

  // Tile masks follow the Triton backend: masks[tile] == true skips the tile
  // (rasterize_to_pixels_fwd.py:54-58); its pixels are written as background.
  const bool skip_tile = a.masks && a.masks[t.tile];
  bool done = !t.inside || skip_tile;
  const float fx = (float)t.px + 0.5f, fy = (float)t.py + 0.5f;

  if (!skip_tile) {
    for (int64_t b0 = t.start; b0 < t.end; b0 += batch) {
      // every pixel terminated -> the whole tile stops (also the LDS WAR fence)
      if (__syncthreads_count(!done) == 0) break;
      const int nb = (int)min((int64_t)batch, t.end - b0);
      stage_batch<D>(a, s, b0, nb);
      __syncthreads();
      if (!done) {
        for (int k = 0; k < nb; ++k) {
          const float2 xy = s.xy[k];
          const float4 cn = s.con[k];
          const float dx = xy.x - fx, dy = xy.y - fy;
          const float sigma = 0.5f * (cn.x * dx * dx + cn.z * dy * dy) + cn.y * dx * dy;
          const float alpha = fminf(kAlphaMax, cn.w * __expf(-sigma));
          if (sigma < 0.f || alpha < kAlphaMin) continue;
          const float next_T = T * (1.f - alpha);
          if (next_T <= kTMin) {
            done = true;
            break;
          }
          const float vis = alpha * T;
#pragma unroll
          for (int d = 0; d < D; ++d) acc[d] += vis * s.col[k][d];
          T = next_T;
          last = (int32_t)(b0 + k);
        }
      }
    }
  }

  if (t.inside) {
    float *oc = a.render_colors + pix * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float bg = a.backgrounds ? a.backgrounds[t.c * D + d] : 0.f;
      oc[d] = acc[d] + T * bg;
    }
    a.render_alphas[pix] = 1.f - T;
    a.last_ids[pix] = last;
  }
}

template <int D, bool ABS>
__global__ void __launch_bounds__(256) rasterize_bwd_kernel(RasterArgs a) {
  __shared__ Stage<D> s;
  __shared__ int32_t s_maxlast[4];
  const TileCtx t = tile_ctx(a);
  if (a.masks && a.masks[t.tile]) return;
  const int batch = min((int)blockDim.x, kMaxBatch);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t pix = ((int64_t)t.c * a.H + t.py) * a.W + t.px;

  float T_final = 1.f, Dra = 0.f, Drc[D];
  int32_t my_last = -1;
#pragma unroll
  for (int d = 0; d < D; ++d) Drc[d] = 0.f;
  if (t.inside) {
    T_final = 1.f - a.render_alphas[pix];
    Dra = a.v_render_alphas ? a.v_render_alphas[pix] : 0.f;  // null: alphas unused
    my_last = a.last_ids[pix];
#pragma unroll
    for (int d = 0; d < D; ++d) Drc[d] = a.v_render_colors[pix * D + d];
  }
  float bg_term = 0.f;
  if (a.backgrounds) {
#pragma unroll
    for (int d = 0; d < D; ++d) bg_term += a.backgrounds[t.c * D + d] * Drc[d];
    bg_term *= T_final;
  }

  // truncate the tile range at the last contributor of any pixel
  // (rasterize_to_pixels_bwd.py:95-101)
  int32_t wmax = my_last;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) wmax = max(wmax, __shfl_xor(wmax, m, 64));
  if (lane == 0) s_maxlast[wid] = wmax;
  __syncthreads();
  int32_t max_last = s_maxlast[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) max_last = max(max_last, s_maxlast[w]);
  const int64_t end = min(t.end, (int64_t)max_last + 1);

  float T = T_final;  // exclusive transmittance of the Gaussian being visited
  float rD = 0.f;     // sum over visited Gaussians of (colour . Drc) * T * alpha
  const float fx = (float)t.px + 0.5f, fy = (float)t.py + 0.5f;

  for (int64_t b1 = end; b1 > t.start; b1 -= batch) {
    const int64_t b0 = max(t.start, b1 - batch);
    const int nb = (int)(b1 - b0);
    __syncthreads();  // previous batch fully consumed
    stage_batch<D>(a, s, b0, nb);
    __syncthreads();
    for (int k = nb - 1; k >= 0; --k) {
      const int64_t idx = b0 + k;
      const float2 xy = s.xy[k];
      const float4 cn = s.con[k];
      const float dx = xy.x - fx, dy = xy.y - fy;
      const float sigma = 0.5f * cn.x * dx * dx + 0.5f * cn.z * dy * dy + cn.y * dx * dy;
      const float ex = __expf(-sigma);
      const float alpha_raw = cn.w * ex;
      const bool valid = t.inside && (idx <= my_last) && (sigma >= 0.f) && (alpha_raw >= kAlphaMin);
      if (__ballot(valid) == 0) continue;  // wave-uniform skip

      float g_col[D], g_op = 0.f, g_mx = 0.f, g_my = 0.f, g_ca = 0.f, g_cb = 0.f, g_cc = 0.f;
      float g_ax = 0.f, g_ay = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) g_col[d] = 0.f;
      if (valid) {
        const float alpha = fminf(kAlphaMax, alpha_raw);
        const float ra = 1.f / (1.f - alpha);
        T *= ra;
        const float w = alpha * T;
        float gD = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          g_col[d] = w * Drc[d];
          gD += s.col[k][d] * Drc[d];
        }
        rD += gD * w;
        float Dalpha = ra * (T_final * Dra + T * gD - rD - bg_term);
        if (alpha_raw > kAlphaMax) Dalpha = 0.f;  // clamped alpha has no gradient
        g_op = Dalpha * ex;
        const float aD = alpha * Dalpha;
        g_mx = -aD * (cn.x * dx + cn.y * dy);
        g_my = -aD * (cn.y * dx + cn.z * dy);
        g_ca = -0.5f * aD * dx * dx;
        g_cb = -aD * dx * dy;
        g_cc = -0.5f * aD * dy * dy;
        if (ABS) {
          g_ax = fabsf(g_mx);
          g_ay = fabsf(g_my);
        }
      }
#pragma unroll
      for (int d = 0; d < D; ++d) g_col[d] = wave_sum(g_col[d]);
      g_op = wave_sum(g_op);
      g_mx = wave_sum(g_mx);
      g_my = wave_sum(g_my);
      g_ca = wave_sum(g_ca);
      g_cb = wave_sum(g_cb);
      g_cc = wave_sum(g_cc);
      if (ABS) {
        g_ax = wave_sum(g_ax);
        g_ay = wave_sum(g_ay);
      }
      if (lane == 0) {
        const int64_t g = s.gid[k];
#pragma unroll
        for (int d = 0; d < D; ++d) atomic_add_f32(a.v_colors + g * D + d, g_col[d]);
        atomic_add_f32(a.v_opacities + g, g_op);
        atomic_add_f32(a.v_means2d + 2 * g, g_mx);
        atomic_add_f32(a.v_means2d + 2 * g + 1, g_my);
        atomic_add_f32(a.v_conics + 3 * g, g_ca);
        atomic_add_f32(a.v_conics + 3 * g + 1, g_cb);
        atomic_add_f32(a.v_conics + 3 * g + 2, g_cc);
        if (ABS) {
          atomic_add_f32(a.v_means2d_abs + 2 * g, g_ax);
          atomic_add_f32(a.v_means2d_abs + 2 * g + 1, g_ay);
        }
      }
    }
  }
}

template <int D>
int launch_fwd(const RasterArgs &a, int threads, hipStream_t st) {
  hipLaunchKernelGGL(rasterize_fwd_kernel<D>, dim3(a.C * a.tw * a.th), dim3(threads), 0, st, a);
  GS_CHECK_LAUNCH("rasterize_fwd");
  return 0;
}

template <int D>
int launch_bwd(const RasterArgs &a, int threads, hipStream_t st) {
  if (a.v_means2d_abs)
    hipLaunchKernelGGL((rasterize_bwd_kernel<D, true>), dim3(a.C * a.tw * a.th), dim3(threads), 0,
                       st, a);
  else
    hipLaunchKernelGGL((rasterize_bwd_kernel<D, false>), dim3(a.C * a.tw * a.th), dim3(threads),
                       0, st, a);
  GS_CHECK_LAUNCH("rasterize_bwd");
  return 0;
}

inline bool supported_channels(int D) {
  return D == 1 || D == 2 || D == 3 || D == 4 || D == 8 || D == 16 || D == 32;
}

}  // namespace gs

namespace gs {
int rasterize16_fwd(int C, int D, int W, int H, int tw, int th, const float *means2d,
                    const float *conics, const float *colors, const float *opacities,
                    const float *backgrounds, const uint8_t *masks, const int32_t *offsets,
                    int64_t n_isects, const int64_t *n_isects_dev, const int32_t *flatten_ids,
                    float *render_colors, float *render_alphas, int32_t *last_ids,
                    const float *records, void *state, int64_t state_bytes, hipStream_t st);
int rasterize16_record_floats(int D);
int rasterize16_pack_records(int64_t G, int D, const float *means2d, const float *conics,
                             const float *colors, const float *opacities, const int32_t *visible,
                             const int32_t *vis_rank, float *records, hipStream_t st);
int64_t rasterize16_fwd_state_bytes(int D, int n_tiles, int64_t n_isects);
int rasterize16_prepare(int D, int C, int tw, int th, const int32_t *offsets, int64_t n_isects,
                        const int64_t *n_isects_dev, void *state, int64_t state_bytes,
                        hipStream_t st);
int64_t rasterize16_bwd_workspace(int64_t G, int D, bool absgrad, int n_tiles, int64_t n_isects);
int rasterize16_bwd(int C, int64_t G, int D, int W, int H, int tw, int th,
                    const float *means2d, const float *conics, const float *colors,
                    const float *opacities, const float *backgrounds, const uint8_t *masks,
                    const int32_t *offsets, int64_t n_isects, const int64_t *n_isects_dev,
                    const int32_t *flatten_ids, const float *render_alphas,
                    const int32_t *last_ids, const float *v_render_colors,
                    const float *v_render_alphas, float *v_means2d, float *v_conics,
                    float *v_colors, float *v_opacities, float *v_abs, const float *render_colors,
                    const float *records, const void *state, int64_t state_bytes,
                    void *workspace, const int32_t *visible, const int32_t *vis_rank,
                    hipStream_t st);
}  // namespace gs

using namespace gs;

extern "C" int gsplat_hip_rasterize_supported_channels(int D) { return supported_channels(D); }

// 16x16 tiles (the gsplat default) run the wave-per-tile kernels of
// rasterize16.hip; other tile sizes run the workgroup-per-tile kernels here.
extern "C" int64_t gsplat_hip_rasterize_fwd_state_bytes(int C, int D, int tile_size,
                                                        int tile_width, int tile_height,
                                                        int64_t n_isects) {
  if (tile_size != 16 || !supported_channels(D)) return 0;
  return rasterize16_fwd_state_bytes(D, C * tile_width * tile_height, n_isects);
}

extern "C" int gsplat_hip_rasterize_prepare(int C, int D, int tile_size, int tile_width,
                                           int tile_height, const int32_t *isect_offsets,
                                           int64_t n_isects, const int64_t *n_isects_device,
                                           void *state, int64_t state_bytes, void *stream) {
  if (tile_size != 16 || !supported_channels(D)) return 0;
  return rasterize16_prepare(D, C, tile_width, tile_height, isect_offsets, n_isects,
                             n_isects_device, state, state_bytes, (hipStream_t)stream);
}

extern "C" int64_t gsplat_hip_rasterize_bwd_workspace_bytes(int64_t n_gaussians, int D,
                                                            int tile_size, int absgrad, int C,
                                                            int tile_width, int tile_height,
                                                            int64_t n_isects) {
  if (tile_size != 16 || !supported_channels(D)) return 0;
  return rasterize16_bwd_workspace(n_gaussians, D, absgrad != 0, C * tile_width * tile_height,
                                   n_isects);
}

extern "C" int gsplat_hip_rasterize_record_floats(int D, int tile_size) {
  return tile_size == 16 ? rasterize16_record_floats(D) : 0;
}

extern "C" int gsplat_hip_rasterize_pack_records(int64_t n_gaussians, int D, const float *means2d,
                                                 const float *conics, const float *colors,
                                                 const float *opacities, const int32_t *visible,
                                                 const int32_t *vis_rank, float *records,
                                                 void *stream) {
  GS_REQUIRE(!vis_rank || visible, "rasterize_pack_records: vis_rank needs visible");
  return rasterize16_pack_records(n_gaussians, D, means2d, conics, colors, opacities, visible,
                                  vis_rank, records, (hipStream_t)stream);
}

static int check_common(int C, int D, int W, int H, int ts, int tw, int th) {
  GS_REQUIRE(supported_channels(D), "rasterize: unsupported channel count %d", D);
  GS_REQUIRE(ts > 0 && ts * ts <= 256, "rasterize: tile_size %d not in [1, 16]", ts);
  GS_REQUIRE((int64_t)tw * ts >= W && (int64_t)th * ts >= H,
             "rasterize: tile grid %dx%d x %d does not cover %dx%d", tw, th, ts, W, H);
  GS_REQUIRE(C >= 0 && W >= 0 && H >= 0, "rasterize: negative sizes");
  return 0;
}

static int block_threads(int ts) { return ((ts * ts + 63) / 64) * 64; }

extern "C" int gsplat_hip_rasterize_fwd(int C, int D, int width, int height, int tile_size,
                                        int tile_width, int tile_height, const float *means2d,
                                        const float *conics, const float *colors,
                                        const float *opacities, const float *backgrounds,
                                        const uint8_t *masks, const int32_t *isect_offsets,
                                        int64_t n_isects, const int64_t *n_isects_device,
                                        const int32_t *flatten_ids, float *render_colors,
                                        float *render_alphas, int32_t *last_ids,
                                        const float *records, void *state, int64_t state_bytes,
                                        void *stream) {
  if (int e = check_common(C, D, width, height, tile_size, tile_width, tile_height)) return e;
  GS_REQUIRE(tile_size == 16 || !n_isects_device,
             "rasterize_fwd: a device isect count needs 16x16 tiles");
  if ((int64_t)C * tile_width * tile_height == 0) return 0;
  RasterArgs a{};
  a.C = C; a.W = width; a.H = height; a.ts = tile_size; a.tw = tile_width; a.th = tile_height;
  a.n_isects = n_isects;
  a.means2d = means2d; a.conics = conics; a.colors = colors; a.opacities = opacities;
  a.backgrounds = backgrounds; a.masks = masks; a.offsets = isect_offsets;
  a.flatten_ids = flatten_ids;
  a.render_colors = render_colors; a.render_alphas = render_alphas; a.last_ids = last_ids;
  hipStream_t st = (hipStream_t)stream;
  if (tile_size == 16)
    return rasterize16_fwd(C, D, width, height, tile_width, tile_height, means2d, conics, colors,
                           opacities, backgrounds, masks, isect_offsets, n_isects,
                           n_isects_device, flatten_ids, render_colors, render_alphas, last_ids,
                           records, state, state_bytes, st);
  const int thr = block_threads(tile_size);
  switch (D) {
    case 1: return launch_fwd<1>(a, thr, st);
    case 2: return launch_fwd<2>(a, thr, st);
    case 3: return launch_fwd<3>(a, thr, st);
    case 4: return launch_fwd<4>(a, thr, st);
    case 8: return launch_fwd<8>(a, thr, st);
    case 16: return launch_fwd<16>(a, thr, st);
    case 32: return launch_fwd<32>(a, thr, st);
  }
  return 1;
}

// Gradient buffers are zeroed here (on `stream`) before accumulation.
extern "C" int gsplat_hip_rasterize_bwd(
    int C, int64_t n_gaussians, int D, int width, int height, int tile_size, int tile_width,
    int tile_height, const float *means2d, const float *conics, const float *colors,
    const float *opacities, const float *backgrounds, const uint8_t *masks,
    const int32_t *isect_offsets, int64_t n_isects, const int64_t *n_isects_device,
    const int32_t *flatten_ids, const float *render_alphas, const int32_t *last_ids,
    const float *v_render_colors,
    const float *v_render_alphas, float *v_means2d, float *v_conics, float *v_colors,
    float *v_opacities, float *v_means2d_abs, const float *render_colors, const float *records,
    const void *state, int64_t state_bytes, void *workspace, int64_t workspace_bytes,
    const int32_t *visible, const int32_t *vis_rank, void *stream) {
  if (int e = check_common(C, D, width, height, tile_size, tile_width, tile_height)) return e;
  GS_REQUIRE(tile_size == 16 || !n_isects_device,
             "rasterize_bwd: a device isect count needs 16x16 tiles");
  hipStream_t st = (hipStream_t)stream;
  const size_t G = (size_t)n_gaussians;
  if (tile_size == 16) {
    const int64_t need = rasterize16_bwd_workspace(n_gaussians, D, v_means2d_abs != nullptr,
                                                   C * tile_width * tile_height, n_isects);
    GS_REQUIRE(workspace_bytes >= need && (need == 0 || workspace),
               "rasterize_bwd: workspace of %lld bytes needed, %lld given", (long long)need,
               (long long)workspace_bytes);
    return rasterize16_bwd(C, n_gaussians, D, width, height, tile_width, tile_height, means2d,
                           conics, colors, opacities, backgrounds, masks, isect_offsets,
                           n_isects, n_isects_device, flatten_ids, render_alphas, last_ids,
                           v_render_colors,
                           v_render_alphas, v_means2d, v_conics, v_colors, v_opacities,
                           v_means2d_abs, render_colors, records, state, state_bytes, workspace,
                           visible, vis_rank, st);
  }
  GS_HIP(gs::zero_async(v_means2d, sizeof(float) * 2 * G, st));
  GS_HIP(gs::zero_async(v_conics, sizeof(float) * 3 * G, st));
  GS_HIP(gs::zero_async(v_colors, sizeof(float) * D * G, st));
  GS_HIP(gs::zero_async(v_opacities, sizeof(float) * G, st));
  if (v_means2d_abs) GS_HIP(gs::zero_async(v_means2d_abs, sizeof(float) * 2 * G, st));
  if ((int64_t)C * tile_width * tile_height == 0 || n_isects == 0) return 0;
  RasterArgs a{};
  a.C = C; a.W = width; a.H = height; a.ts = tile_size; a.tw = tile_width; a.th = tile_height;
  a.n_isects = n_isects;
  a.means2d = means2d; a.conics = conics; a.colors = colors; a.opacities = opacities;
  a.backgrounds = backgrounds; a.masks = masks; a.offsets = isect_offsets;
  a.flatten_ids = flatten_ids;
  a.render_alphas = const_cast<float *>(render_alphas);
  a.last_ids = const_cast<int32_t *>(last_ids);
  a.v_render_colors = v_render_colors; a.v_render_alphas = v_render_alphas;
  a.v_means2d = v_means2d; a.v_conics = v_conics; a.v_colors = v_colors;
  a.v_opacities = v_opacities; a.v_means2d_abs = v_means2d_abs;
  const int thr = block_threads(tile_size);
  switch (D) {
    case 1: return launch_bwd<1>(a, thr, st);
    case 2: return launch_bwd<2>(a, thr, st);
    case 3: return launch_bwd<3>(a, thr, st);
    case 4: return launch_bwd<4>(a, thr, st);
    case 8: return launch_bwd<8>(a, thr, st);
    case 16: return launch_bwd<16>(a, thr, st);
    case 32: return launch_bwd<32>(a, thr, st);
  }
  return 1;
}
