// Per-pixel contributor lists: rasterize_to_indices_in_range for 3DGS
// (conics) and 2DGS (ray transforms).
//
// Replaces the reference CUDA kernels
//   rasterize_to_indices_3dgs_kernel  gsplat/cuda/csrc/RasterizeToIndices3DGS.cu:14-185
//   rasterize_to_indices_2dgs_kernel  gsplat/cuda/csrc/RasterizeToIndices2DGS.cu:14-200
// and the two-pass host driver of gsplat/cuda/csrc/Rasterization.cpp:224-296.
//
// The same front-to-back sweep runs twice: a COUNT pass writes the number of
// contributors of every pixel in batches [range_start, range_end) (batch =
// ts*ts records of the tile's depth-sorted list), the caller scans the counts
// (exclusive, pixel-major [C, H, W] order), and a WRITE pass stores
// (gaussian id = flatten id % N, pixel index = c*H*W + y*W + x) at that base,
// in record order.  The starting transmittance comes from the caller
// (`transmittances`, the product of earlier ranges).  A contributor is a
// record with sigma >= 0 and alpha >= 1/255 whose product keeps
// T * (1 - alpha) > 1e-4 (exclusive stop, as in rasterization).
//
// Mapping: one workgroup per tile, one lane per pixel; each batch of records
// is gathered by the workgroup with one lane per record into LDS (SoA) and
// read back as LDS broadcasts.  This is a debug / playground path (the
// reference's `_rasterize_to_pixels` + `accumulate`), so it favours a plain
// layout over the wave-per-strip machinery of the training rasterizers.
#include "common.h"
#include "../../include/gsplat_hip.h"

namespace idxk {

constexpr float kAlphaMin = 1.f / 255.f;
constexpr float kAlphaMax = 0.999f;
constexpr float kTMin = 1e-4f;
constexpr float kFilterInvSquare = 2.f;  // FILTER_INV_SQUARE_2DGS, Rasterization.h:11
constexpr int kMaxLanes = 1024;

struct IdxArgs {
  int C, N, W, H, ts, tw, th;
  int64_t n_isects;
  uint32_t range_start, range_end;
  const float *transmittances;  // [C, H, W]
  const float *means2d;         // [C, N, 2]
  const float *shape;           // conics [C, N, 3] (3DGS) or ray transforms [C, N, 9] (2DGS)
  const float *opacities;       // [C, N]
  const int32_t *offsets, *flatten_ids;
  int32_t *chunk_cnts;          // COUNT pass output [C, H, W]
  const int32_t *chunk_starts;  // WRITE pass input [C, H, W]
  int64_t *gaussian_ids, *pixel_ids;
};

// KIND 0: 3DGS (RasterizeToIndices3DGS.cu:142-150); KIND 1: 2DGS
// (RasterizeToIndices2DGS.cu:150-176).  Per record LDS holds x, y, opacity and
// 3 (conic) or 9 (ray transform) shape floats.
template <int KIND>
struct Rec {
  static constexpr int S = KIND == 0 ? 3 : 9;
};

template <int KIND>
GS_INLINE float record_sigma(const float *sh, float x, float y, float fx, float fy, bool &skip) {
  skip = false;
  if constexpr (KIND == 0) {
    const float dx = x - fx, dy = y - fy;
    return 0.5f * (sh[0] * dx * dx + sh[2] * dy * dy) + sh[1] * dx * dy;
  } else {
    // h_u = px * w_M - u_M, h_v = py * w_M - v_M; s = (h_u x h_v).xy / .z
    const float hu0 = fx * sh[6] - sh[0], hu1 = fx * sh[7] - sh[1], hu2 = fx * sh[8] - sh[2];
    const float hv0 = fy * sh[6] - sh[3], hv1 = fy * sh[7] - sh[4], hv2 = fy * sh[8] - sh[5];
    const float cx = hu1 * hv2 - hu2 * hv1;
    const float cy = hu2 * hv0 - hu0 * hv2;
    const float cz = hu0 * hv1 - hu1 * hv0;
    if (cz == 0.f) {
      skip = true;
      return 0.f;
    }
    const float sx = cx / cz, sy = cy / cz;
    const float g3 = sx * sx + sy * sy;
    const float dx = x - fx, dy = y - fy;
    const float g2 = kFilterInvSquare * (dx * dx + dy * dy);
    return 0.5f * fminf(g3, g2);
  }
}

template <int KIND, bool WRITE>
__global__ void __launch_bounds__(1024) indices_kernel(IdxArgs a) {
  constexpr int S = Rec<KIND>::S;
  __shared__ int32_t s_gid[kMaxLanes];
  __shared__ float s_xyo[3][kMaxLanes];
  __shared__ float s_sh[S][kMaxLanes];

  const int ntile = a.tw * a.th;
  const int tile = blockIdx.x;
  const int c = tile / ntile;
  const int rem = tile - c * ntile;
  const int ty = rem / a.tw, tx = rem - ty * a.tw;
  const int bs = a.ts * a.ts;
  const int lid = threadIdx.x;
  const int ly = lid / a.ts, lx = lid - ly * a.ts;
  const int px = tx * a.ts + lx, py = ty * a.ts + ly;
  const bool inside = px < a.W && py < a.H;
  const int64_t pix = ((int64_t)c * a.H + py) * a.W + px;  // also the output pixel index

  const int64_t start = a.offsets[tile];
  const int64_t end = (tile == a.C * ntile - 1) ? a.n_isects : (int64_t)a.offsets[tile + 1];
  const uint32_t num_batches = (uint32_t)((end - start + bs - 1) / bs);
  const uint32_t b_end = min(a.range_end, num_batches);

  float T = inside ? a.transmittances[pix] : 0.f;
  int64_t base = 0;
  if (WRITE && inside) base = a.chunk_starts[pix];
  bool done = !inside;
  int32_t cnt = 0;
  const float fx = (float)px + 0.5f, fy = (float)py + 0.5f;

  for (uint32_t b = a.range_start; b < b_end; ++b) {
    // all pixels done -> stop (also the LDS write-after-read fence)
    if (__syncthreads_count(!done) == 0) break;
    const int64_t b0 = start + (int64_t)bs * b;
    const int nb = (int)min((int64_t)bs, end - b0);
    if (lid < nb) {
      const int32_t g = a.flatten_ids[b0 + lid];
      s_gid[lid] = g;
      s_xyo[0][lid] = a.means2d[2 * (int64_t)g];
      s_xyo[1][lid] = a.means2d[2 * (int64_t)g + 1];
      s_xyo[2][lid] = a.opacities[g];
      const float *src = a.shape + (int64_t)S * g;
#pragma unroll
      for (int k = 0; k < S; ++k) s_sh[k][lid] = src[k];
    }
    __syncthreads();
    for (int t = 0; t < nb && !done; ++t) {
      float sh[S];
#pragma unroll
      for (int k = 0; k < S; ++k) sh[k] = s_sh[k][t];
      bool skip;
      const float sigma = record_sigma<KIND>(sh, s_xyo[0][t], s_xyo[1][t], fx, fy, skip);
      if (skip) continue;
      const float alpha = fminf(kAlphaMax, s_xyo[2][t] * expf(-sigma));
      if (sigma < 0.f || alpha < kAlphaMin) continue;
      const float nT = T * (1.f - alpha);
      if (nT <= kTMin) {
        done = true;
        break;
      }
      if (WRITE) {
        a.gaussian_ids[base + cnt] = (int64_t)(s_gid[t] % a.N);
        a.pixel_ids[base + cnt] = pix;
      }
      ++cnt;
      T = nT;
    }
  }
  if (!WRITE && inside) a.chunk_cnts[pix] = cnt;
}

template <int KIND>
int launch(IdxArgs &a, bool write, void *stream, const char *name) {
  GS_REQUIRE(a.C >= 1 && a.N >= 0 && a.W >= 1 && a.H >= 1 && a.ts >= 1,
             "%s: bad sizes", name);
  GS_REQUIRE(a.ts * a.ts <= kMaxLanes, "%s: tile_size %d too large (ts*ts <= %d)", name, a.ts,
             kMaxLanes);
  GS_REQUIRE(a.tw * a.ts >= a.W && a.th * a.ts >= a.H, "%s: tile grid does not cover the image",
             name);
  GS_REQUIRE(a.n_isects >= 0, "%s: negative n_isects", name);
  GS_REQUIRE(a.transmittances && a.offsets, "%s: null pointer", name);
  if (a.n_isects > 0)
    GS_REQUIRE(a.means2d && a.shape && a.opacities && a.flatten_ids, "%s: null pointer", name);
  if (write)
    GS_REQUIRE(a.chunk_starts && a.gaussian_ids && a.pixel_ids, "%s: null output", name);
  else
    GS_REQUIRE(a.chunk_cnts, "%s: null chunk_cnts", name);
  const dim3 grid((unsigned)(a.C * a.tw * a.th)), block((unsigned)(a.ts * a.ts));
  if (write)
    hipLaunchKernelGGL((indices_kernel<KIND, true>), grid, block, 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL((indices_kernel<KIND, false>), grid, block, 0, (hipStream_t)stream, a);
  GS_CHECK_LAUNCH(name);
  return 0;
}

}  // namespace idxk

namespace {

idxk::IdxArgs make_args(int C, int N, int W, int H, int ts, int tw, int th, int64_t n_isects,
                        int64_t range_start, int64_t range_end, const float *transmittances,
                        const float *means2d, const float *shape, const float *opacities,
                        const int32_t *offsets, const int32_t *flatten_ids) {
  idxk::IdxArgs a{};
  a.C = C, a.N = N, a.W = W, a.H = H, a.ts = ts, a.tw = tw, a.th = th;
  a.n_isects = n_isects;
  // ranges are in batches of ts*ts records; clamp to the 32-bit counters of
  // the reference kernel (range_end = 1e10 means "all")
  a.range_start = (uint32_t)std::min<int64_t>(std::max<int64_t>(range_start, 0), 0x7fffffff);
  a.range_end = (uint32_t)std::min<int64_t>(std::max<int64_t>(range_end, 0), 0x7fffffff);
  a.transmittances = transmittances, a.means2d = means2d, a.shape = shape;
  a.opacities = opacities, a.offsets = offsets, a.flatten_ids = flatten_ids;
  return a;
}

}  // namespace

extern "C" int gsplat_hip_rasterize_to_indices_count(
    int kind, int C, int N, int W, int H, int tile_size, int tile_width, int tile_height,
    int64_t n_isects, int64_t range_start, int64_t range_end, const float *transmittances,
    const float *means2d, const float *shape, const float *opacities, const int32_t *offsets,
    const int32_t *flatten_ids, int32_t *chunk_cnts, void *stream) {
  idxk::IdxArgs a = make_args(C, N, W, H, tile_size, tile_width, tile_height, n_isects,
                              range_start, range_end, transmittances, means2d, shape, opacities,
                              offsets, flatten_ids);
  a.chunk_cnts = chunk_cnts;
  GS_REQUIRE(kind == 0 || kind == 1, "rasterize_to_indices_count: kind must be 0 or 1");
  return kind == 0 ? idxk::launch<0>(a, false, stream, "rasterize_to_indices_count")
                   : idxk::launch<1>(a, false, stream, "rasterize_to_indices_count");
}

extern "C" int gsplat_hip_rasterize_to_indices_write(
    int kind, int C, int N, int W, int H, int tile_size, int tile_width, int tile_height,
    int64_t n_isects, int64_t range_start, int64_t range_end, const float *transmittances,
    const float *means2d, const float *shape, const float *opacities, const int32_t *offsets,
    const int32_t *flatten_ids, const int32_t *chunk_starts, int64_t *gaussian_ids,
    int64_t *pixel_ids, void *stream) {
  idxk::IdxArgs a = make_args(C, N, W, H, tile_size, tile_width, tile_height, n_isects,
                              range_start, range_end, transmittances, means2d, shape, opacities,
                              offsets, flatten_ids);
  a.chunk_starts = chunk_starts, a.gaussian_ids = gaussian_ids, a.pixel_ids = pixel_ids;
  GS_REQUIRE(kind == 0 || kind == 1, "rasterize_to_indices_write: kind must be 0 or 1");
  return kind == 0 ? idxk::launch<0>(a, true, stream, "rasterize_to_indices_write")
                   : idxk::launch<1>(a, true, stream, "rasterize_to_indices_write");
}
