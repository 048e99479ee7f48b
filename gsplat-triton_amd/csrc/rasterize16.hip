// Wave-per-tile rasterizer for 16x16 tiles (the gsplat default), gfx950.
//
// Same semantics as rasterize.hip (reference: rasterize_to_pixels_fwd.py:13-196,
// rasterize_to_pixels_bwd.py:13-337), different mapping, built for CDNA4:
//
//  * one wave64 owns one 16x16 tile, every lane owns a 2x2 pixel quad, so the
//    per-Gaussian LDS broadcast reads, culling and (backward) cross-lane
//    reductions are amortised over 4 pixels and no workgroup barrier is
//    needed (a workgroup is 4 independent waves = 4 tiles);
//  * each batch of 64 isects is gathered one record per lane, culled against
//    the tile with the exact rectangle minimum of the Gaussian's quadratic
//    form (a record that cannot reach alpha >= 1/255 on any pixel centre of
//    the tile is dropped -- the per-pixel test would skip it anyway), and
//    compacted into LDS with ballot/mbcnt;
//  * backward: the per-lane partial gradients (up to 16 fields) are combined
//    across the 64 lanes with a reduce-scatter (permlane32/16 swaps, then DPP
//    mirrors and quad permutes: 35 VALU ops for 16 sums instead of 16
//    butterflies), after which 16 lanes issue ONE coalesced 64-B fp32 atomic
//    into a packed [G][S] gradient row.  MI355X float atomics execute at the
//    memory side (MI355X_MICROARCH.md "Global float atomics"), so one 64-B
//    request per (Gaussian, tile) replaces 4 waves x 9 single-lane requests.
#include "common.h"
#include "../../include/gsplat_hip.h"

#include <stdlib.h>

namespace gs {
namespace r16 {

constexpr int kTS = 16;
constexpr float kAlphaMin = 1.f / 255.f;
constexpr float kAlphaMax = 0.999f;
constexpr float kTMin = 1e-4f;

template <int CTRL>
GS_INLINE float dpp(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

GS_INLINE float swap32_sum(float a, float b) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

GS_INLINE float swap16_sum(float a, float b) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Reduce-scatter of 16 per-lane values over the wave: returns, in every lane,
// the wave-wide total of value (lane >> 2).
GS_INLINE float reduce_scatter16(const float *v, int lane) {
  float w[8], x[4], y[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = swap32_sum(v[i], v[i + 8]);  // lane ^ 32
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = swap16_sum(w[i], w[i + 4]);  // lane ^ 16
  const bool b3 = lane & 8, b2 = lane & 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // row mirror pairs lanes across bit 3
    const float keep = b3 ? x[i + 2] : x[i];
    const float send = b3 ? x[i] : x[i + 2];
    y[i] = keep + dpp<0x140>(send);
  }
  const float keep = b2 ? y[1] : y[0];  // half-row mirror pairs across bit 2
  const float send = b2 ? y[0] : y[1];
  float z = keep + dpp<0x141>(send);
  z += dpp<0xB1>(z);  // quad lane ^ 1
  z += dpp<0x4E>(z);  // quad lane ^ 2
  return z;
}

struct Args {
  int C, W, H, tw, th, n_tiles;
  int64_t n_isects;
  const float *means2d, *conics, *colors, *opacities, *backgrounds;
  const uint8_t *masks;
  const int32_t *offsets, *flatten_ids;
  float *render_colors, *render_alphas;
  int32_t *last_ids;
  const float *v_render_colors, *v_render_alphas;
  float *packed;  // [G][S] gradient rows (backward)
  int S;
};

template <int D>
struct WaveStage {
  float2 xy[64];
  float4 con[64];
  float col[64][D];
  int32_t idx[64];  // global isect index
  int32_t gid[64];
};

// Minimum over the rectangle [x0,x1]x[y0,y1] of
//   q(dx,dy) = 0.5*(a dx^2 + c dy^2) + b dx dy,  (dx,dy) = (mx - x, my - y).
// Conservative: returns 0 for a non positive-definite conic.
GS_INLINE float rect_min_sigma(float mx, float my, float a, float b, float c, float x0, float x1,
                               float y0, float y1) {
  if (!(a > 0.f && c > 0.f && a * c - b * b > 0.f)) return 0.f;
  if (mx >= x0 && mx <= x1 && my >= y0 && my <= y1) return 0.f;
  const float dxl = mx - x1, dxh = mx - x0;  // dx range over the rect
  const float dyl = my - y1, dyh = my - y0;
  auto q = [&](float dx, float dy) { return 0.5f * (a * dx * dx + c * dy * dy) + b * dx * dy; };
  float m = 3.0e38f;
  // vertical edges: dx fixed, best dy = -b dx / c clamped
  for (int e = 0; e < 2; ++e) {
    const float dx = e ? dxh : dxl;
    const float dy = fminf(fmaxf(-b * dx / c, dyl), dyh);
    m = fminf(m, q(dx, dy));
  }
  for (int e = 0; e < 2; ++e) {
    const float dy = e ? dyh : dyl;
    const float dx = fminf(fmaxf(-b * dy / a, dxl), dxh);
    m = fminf(m, q(dx, dy));
  }
  return fmaxf(m, 0.f);
}

// Geometry of one wave: PPL pixels per lane, WPT = 4 / PPL waves share a
// tile, each owning a 16 x (4*PPL) strip; lane l owns column (l & 15) and
// rows strip_y0 + PPL*(l >> 4) + p, p < PPL.
template <int PPL>
struct WaveGeom {
  static constexpr int WPT = 4 / PPL;
  static constexpr int SH = 4 * PPL;
  int tile, c, tx, ty, strip;
  int px, py0;  // this lane's column and first row
  float x0, x1, y0, y1;  // strip rectangle of pixel centres

  GS_INLINE WaveGeom(const Args &a, int lane) {
    const int w = threadIdx.x >> 6;
    tile = blockIdx.x * PPL + w / WPT;
    strip = w % WPT;
    const int ntile = a.tw * a.th;
    c = tile / ntile;
    const int rem = tile - c * ntile;
    ty = rem / a.tw;
    tx = rem - ty * a.tw;
    px = tx * kTS + (lane & 15);
    py0 = ty * kTS + SH * strip + PPL * (lane >> 4);
    x0 = tx * kTS + 0.5f;
    x1 = x0 + (kTS - 1);
    y0 = ty * kTS + SH * strip + 0.5f;
    y1 = y0 + (SH - 1);
  }
};

template <int D>
GS_INLINE bool stage_record(const Args &a, int64_t j, float x0, float x1, float y0, float y1,
                            float2 &xy, float4 &con, float (&col)[D], int32_t &g) {
  g = a.flatten_ids[j];
  xy = *reinterpret_cast<const float2 *>(a.means2d + 2 * (int64_t)g);
  const float *cn = a.conics + 3 * (int64_t)g;
  con = make_float4(cn[0], cn[1], cn[2], a.opacities[g]);
  const float *cl = a.colors + (int64_t)g * D;
#pragma unroll
  for (int d = 0; d < D; ++d) col[d] = cl[d];
  if (!(con.w >= kAlphaMin)) return false;  // alpha <= opacity < 1/255 everywhere
  const float ms = rect_min_sigma(xy.x, xy.y, con.x, con.y, con.z, x0, x1, y0, y1);
  // keep iff some pixel can have opacity*exp(-sigma) >= 1/255 (margin 0.02
  // absorbs float rounding of the per-pixel sigma and __expf)
  return ms <= 0.69314718f * __builtin_amdgcn_logf(255.f * con.w) + 0.02f;
}

template <int D, int PPL>
__global__ void __launch_bounds__(256) fwd_kernel(Args a) {
  __shared__ WaveStage<D> stage_all[4];
  const int lane = threadIdx.x & 63;
  WaveStage<D> &st = stage_all[threadIdx.x >> 6];
  const WaveGeom<PPL> geo(a, lane);
  if (geo.tile >= a.n_tiles) return;
  const int tile = geo.tile, c = geo.c;
  const float x0 = geo.x0, x1 = geo.x1, y0 = geo.y0, y1 = geo.y1;
  float fx[PPL], fy[PPL];
  bool inside[PPL];
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    const int px = geo.px, py = geo.py0 + p;
    inside[p] = px < a.W && py < a.H;
    fx[p] = (float)px + 0.5f;
    fy[p] = (float)py + 0.5f;
  }
  const int64_t start = a.offsets[tile];
  const int64_t end = (tile == a.n_tiles - 1) ? a.n_isects : (int64_t)a.offsets[tile + 1];

  float T[PPL];
  float acc[PPL][D];
#pragma unroll
  for (int p = 0; p < PPL; ++p)
#pragma unroll
    for (int d = 0; d < D; ++d) acc[p][d] = 0.f;
  int32_t last[PPL];
  const bool skip_tile = a.masks && a.masks[tile];
  // A terminated (or outside) pixel is encoded by a negative T: |T| is its
  // final transmittance.  Keeps the per-pixel state in plain floats.
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    T[p] = (!inside[p] || skip_tile) ? -1.f : 1.f;
    last[p] = 0;
  }
  auto any_alive = [&]() {
    bool al = false;
#pragma unroll
    for (int p = 0; p < PPL; ++p) al |= T[p] > 0.f;
    return al;
  };

  for (int64_t b0 = start; b0 < end && !skip_tile; b0 += 64) {
    if (__ballot(any_alive()) == 0) break;
    const int64_t j = b0 + lane;
    float2 xy;
    float4 con;
    float col[D];
    int32_t g = 0;
    bool keep = false;
    if (j < end) keep = stage_record<D>(a, j, x0, x1, y0, y1, xy, con, col, g);
    const uint64_t m = __ballot(keep);
    const int slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    const int cnt = __popcll(m);
    if (keep) {
      st.xy[slot] = xy;
      st.con[slot] = con;
#pragma unroll
      for (int d = 0; d < D; ++d) st.col[slot][d] = col[d];
      st.idx[slot] = (int32_t)j;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int k = 0; k < cnt; ++k) {
      // wave-uniform record (broadcast LDS reads)
      const float2 gxy = st.xy[k];
      const float4 cn = st.con[k];
      const int32_t gidx = st.idx[k];
      float gc[D];
#pragma unroll
      for (int d = 0; d < D; ++d) gc[d] = st.col[k][d];
      // branch-free per pixel: every update is a select, so the four pixels
      // of a lane cost straight-line VALU with no exec-mask juggling
#pragma unroll
      for (int p = 0; p < PPL; ++p) {
        const float dx = gxy.x - fx[p], dy = gxy.y - fy[p];
        const float sigma = 0.5f * (cn.x * dx * dx + cn.z * dy * dy) + cn.y * dx * dy;
        const float alpha = fminf(kAlphaMax, cn.w * __expf(-sigma));
        const float Tp = T[p];
        const bool hit = (Tp > 0.f) & (sigma >= 0.f) & (alpha >= kAlphaMin);
        const float nT = Tp * (1.f - alpha);
        const bool term = hit & (nT <= kTMin);  // exclusive stop: not blended
        const bool ok = hit & (nT > kTMin);
        const float vis = ok ? alpha * Tp : 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) acc[p][d] += vis * gc[d];
        T[p] = ok ? nT : (term ? -Tp : Tp);
        last[p] = ok ? gidx : last[p];
      }
      if ((k & 15) == 15 && __ballot(any_alive()) == 0) break;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    if (!inside[p]) continue;
    const int64_t pix = ((int64_t)c * a.H + geo.py0 + p) * a.W + geo.px;
    float *oc = a.render_colors + pix * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float bg = a.backgrounds ? a.backgrounds[c * D + d] : 0.f;
      oc[d] = acc[p][d] + fabsf(T[p]) * bg;
    }
    a.render_alphas[pix] = 1.f - fabsf(T[p]);
    a.last_ids[pix] = last[p];
  }
}

template <int D, bool ABS, int PPL>
__global__ void __launch_bounds__(256) bwd_kernel(Args a) {
  constexpr int F = D + 6 + (ABS ? 2 : 0);
  constexpr int NV = (F + 15) / 16;
  __shared__ WaveStage<D> stage_all[4];
  const int lane = threadIdx.x & 63;
  WaveStage<D> &st = stage_all[threadIdx.x >> 6];
  const WaveGeom<PPL> geo(a, lane);
  if (geo.tile >= a.n_tiles) return;
  const int tile = geo.tile, c = geo.c;
  if (a.masks && a.masks[tile]) return;

  float fx[PPL], fy[PPL], T[PPL], Tf[PPL], Dra[PPL], rD[PPL], bgt[PPL], Drc[PPL][D];
  int32_t mylast[PPL];
  int32_t lmax = -1;
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    const int px = geo.px, py = geo.py0 + p;
    const bool in = px < a.W && py < a.H;
    fx[p] = (float)px + 0.5f;
    fy[p] = (float)py + 0.5f;
    Tf[p] = 1.f; Dra[p] = 0.f; mylast[p] = -1; rD[p] = 0.f; bgt[p] = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) Drc[p][d] = 0.f;
    if (in) {
      const int64_t pix = ((int64_t)c * a.H + py) * a.W + px;
      Tf[p] = 1.f - a.render_alphas[pix];
      Dra[p] = a.v_render_alphas[pix];
      mylast[p] = a.last_ids[pix];
#pragma unroll
      for (int d = 0; d < D; ++d) Drc[p][d] = a.v_render_colors[pix * D + d];
      if (a.backgrounds) {
        float s = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) s += a.backgrounds[c * D + d] * Drc[p][d];
        bgt[p] = s * Tf[p];
      }
    }
    T[p] = Tf[p];
    lmax = max(lmax, mylast[p]);
  }
#pragma unroll
  for (int msk = 32; msk >= 1; msk >>= 1) lmax = max(lmax, __shfl_xor(lmax, msk, 64));
  const float x0 = geo.x0, x1 = geo.x1, y0 = geo.y0, y1 = geo.y1;
  const int64_t start = a.offsets[tile];
  const int64_t tend = (tile == a.n_tiles - 1) ? a.n_isects : (int64_t)a.offsets[tile + 1];
  const int64_t end = min(tend, (int64_t)lmax + 1);

  for (int64_t b1 = end; b1 > start; b1 -= 64) {
    const int64_t b0 = max(start, b1 - 64);
    const int64_t j = b0 + lane;
    float2 xy;
    float4 con;
    float col[D];
    int32_t g = 0;
    bool keep = false;
    if (j < b1) keep = stage_record<D>(a, j, x0, x1, y0, y1, xy, con, col, g);
    const uint64_t m = __ballot(keep);
    const int slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    const int cnt = __popcll(m);
    if (keep) {
      st.xy[slot] = xy;
      st.con[slot] = con;
#pragma unroll
      for (int d = 0; d < D; ++d) st.col[slot][d] = col[d];
      st.idx[slot] = (int32_t)j;
      st.gid[slot] = g;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int k = cnt - 1; k >= 0; --k) {
      const float2 gxy = st.xy[k];
      const float4 cn = st.con[k];
      const int32_t idx = st.idx[k];
      float v[NV * 16];
#pragma unroll
      for (int f = 0; f < NV * 16; ++f) v[f] = 0.f;
      float gc[D];
#pragma unroll
      for (int d = 0; d < D; ++d) gc[d] = st.col[k][d];
      bool any = false;
      // branch-free per pixel (selects instead of divergent `continue`s)
#pragma unroll
      for (int p = 0; p < PPL; ++p) {
        const float dx = gxy.x - fx[p], dy = gxy.y - fy[p];
        const float sigma = 0.5f * cn.x * dx * dx + 0.5f * cn.z * dy * dy + cn.y * dx * dy;
        const float ex = __expf(-sigma);
        const float alpha_raw = cn.w * ex;
        const bool valid = (idx <= mylast[p]) & (sigma >= 0.f) & (alpha_raw >= kAlphaMin);
        any |= valid;
        const float alpha = fminf(kAlphaMax, alpha_raw);
        const float ra = __builtin_amdgcn_rcpf(1.f - alpha);
        T[p] = valid ? T[p] * ra : T[p];
        const float w = valid ? alpha * T[p] : 0.f;
        float gD = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          v[d] += w * Drc[p][d];
          gD += gc[d] * Drc[p][d];
        }
        rD[p] += gD * w;
        const float Da_raw = ra * (Tf[p] * Dra[p] + T[p] * gD - rD[p] - bgt[p]);
        // clamped alpha (> 0.999) has no gradient (rasterize_to_pixels_bwd.py:184-187)
        const float Da = (valid & (alpha_raw <= kAlphaMax)) ? Da_raw : 0.f;
        const float aD = alpha * Da;
        const float gmx = -aD * (cn.x * dx + cn.y * dy);
        const float gmy = -aD * (cn.y * dx + cn.z * dy);
        v[D] += valid ? Da * ex : 0.f;
        v[D + 1] += gmx;
        v[D + 2] += gmy;
        v[D + 3] += -0.5f * aD * dx * dx;
        v[D + 4] += -aD * dx * dy;
        v[D + 5] += -0.5f * aD * dy * dy;
        if (ABS) {
          v[D + 6] += fabsf(gmx);
          v[D + 7] += fabsf(gmy);
        }
      }
      if (__ballot(any) == 0) continue;
      float *row = a.packed + (int64_t)st.gid[k] * a.S;
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const float tot = reduce_scatter16(v + 16 * q, lane);
        const int field = 16 * q + (lane >> 2);
        if ((lane & 3) == 0 && field < F && tot != 0.f) atomic_add_f32(row + field, tot);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// packed [G][S] -> the autograd tensors
template <int D, bool ABS>
__global__ void __launch_bounds__(256)
unpack_kernel(int64_t G, int S, const float *__restrict__ packed, float *__restrict__ v_means2d,
              float *__restrict__ v_conics, float *__restrict__ v_colors,
              float *__restrict__ v_opacities, float *__restrict__ v_abs) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const float *r = packed + g * S;
#pragma unroll
  for (int d = 0; d < D; ++d) v_colors[g * D + d] = r[d];
  v_opacities[g] = r[D];
  *reinterpret_cast<float2 *>(v_means2d + 2 * g) = make_float2(r[D + 1], r[D + 2]);
  v_conics[3 * g] = r[D + 3];
  v_conics[3 * g + 1] = r[D + 4];
  v_conics[3 * g + 2] = r[D + 5];
  if (ABS) *reinterpret_cast<float2 *>(v_abs + 2 * g) = make_float2(r[D + 6], r[D + 7]);
}

}  // namespace r16

// pixels per lane (1: 4 waves per tile; 4: one wave per tile); GSPLAT_HIP_PPL
// overrides it for experiments.
static int ppl_choice(int dflt) {
  static int v = [] {
    const char *e = getenv("GSPLAT_HIP_PPL");
    return e ? atoi(e) : 0;
  }();
  return (v == 1 || v == 2 || v == 4) ? v : dflt;
}

template <int D>
int r16_fwd(const r16::Args &a, hipStream_t st) {
  const int ppl = ppl_choice(1);
  const int blocks = (a.n_tiles + ppl - 1) / ppl;
  if (ppl == 1) hipLaunchKernelGGL((r16::fwd_kernel<D, 1>), dim3(blocks), dim3(256), 0, st, a);
  else if (ppl == 2) hipLaunchKernelGGL((r16::fwd_kernel<D, 2>), dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((r16::fwd_kernel<D, 4>), dim3(blocks), dim3(256), 0, st, a);
  GS_CHECK_LAUNCH("rasterize_fwd16");
  return 0;
}

template <int D, bool ABS>
int r16_bwd(r16::Args a, int64_t G, float *v_means2d, float *v_conics, float *v_colors,
            float *v_opacities, float *v_abs, void *workspace, hipStream_t st) {
  constexpr int F = D + 6 + (ABS ? 2 : 0);
  a.S = ((F + 15) / 16) * 16;
  a.packed = reinterpret_cast<float *>(workspace);
  GS_HIP(hipMemsetAsync(a.packed, 0, sizeof(float) * (size_t)a.S * G, st));
  if (a.n_isects > 0) {
    const int ppl = ppl_choice(1);
    const int blocks = (a.n_tiles + ppl - 1) / ppl;
    if (ppl == 1)
      hipLaunchKernelGGL((r16::bwd_kernel<D, ABS, 1>), dim3(blocks), dim3(256), 0, st, a);
    else if (ppl == 2)
      hipLaunchKernelGGL((r16::bwd_kernel<D, ABS, 2>), dim3(blocks), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((r16::bwd_kernel<D, ABS, 4>), dim3(blocks), dim3(256), 0, st, a);
    GS_CHECK_LAUNCH("rasterize_bwd16");
  }
  if (G > 0) {
    hipLaunchKernelGGL((r16::unpack_kernel<D, ABS>), dim3((unsigned)((G + 255) / 256)), dim3(256),
                       0, st, G, a.S, a.packed, v_means2d, v_conics, v_colors, v_opacities, v_abs);
    GS_CHECK_LAUNCH("rasterize_bwd16_unpack");
  }
  return 0;
}

int rasterize16_fwd(int C, int D, int W, int H, int tw, int th, const float *means2d,
                    const float *conics, const float *colors, const float *opacities,
                    const float *backgrounds, const uint8_t *masks, const int32_t *offsets,
                    int64_t n_isects, const int32_t *flatten_ids, float *render_colors,
                    float *render_alphas, int32_t *last_ids, hipStream_t st) {
  r16::Args a{};
  a.C = C; a.W = W; a.H = H; a.tw = tw; a.th = th; a.n_tiles = C * tw * th;
  a.n_isects = n_isects;
  a.means2d = means2d; a.conics = conics; a.colors = colors; a.opacities = opacities;
  a.backgrounds = backgrounds; a.masks = masks; a.offsets = offsets; a.flatten_ids = flatten_ids;
  a.render_colors = render_colors; a.render_alphas = render_alphas; a.last_ids = last_ids;
  switch (D) {
    case 1: return r16_fwd<1>(a, st);
    case 2: return r16_fwd<2>(a, st);
    case 3: return r16_fwd<3>(a, st);
    case 4: return r16_fwd<4>(a, st);
    case 8: return r16_fwd<8>(a, st);
    case 16: return r16_fwd<16>(a, st);
    case 32: return r16_fwd<32>(a, st);
  }
  GS_REQUIRE(false, "rasterize16_fwd: unsupported channels %d", D);
}

int64_t rasterize16_bwd_workspace(int64_t G, int D, bool absgrad) {
  const int F = D + 6 + (absgrad ? 2 : 0);
  return (int64_t)sizeof(float) * ((F + 15) / 16) * 16 * G;
}

int rasterize16_bwd(int C, int64_t G, int D, int W, int H, int tw, int th,
                    const float *means2d, const float *conics, const float *colors,
                    const float *opacities, const float *backgrounds, const uint8_t *masks,
                    const int32_t *offsets, int64_t n_isects, const int32_t *flatten_ids,
                    const float *render_alphas, const int32_t *last_ids,
                    const float *v_render_colors, const float *v_render_alphas,
                    float *v_means2d, float *v_conics, float *v_colors, float *v_opacities,
                    float *v_abs, void *workspace, hipStream_t st) {
  r16::Args a{};
  a.C = C; a.W = W; a.H = H; a.tw = tw; a.th = th; a.n_tiles = C * tw * th;
  a.n_isects = n_isects;
  a.means2d = means2d; a.conics = conics; a.colors = colors; a.opacities = opacities;
  a.backgrounds = backgrounds; a.masks = masks; a.offsets = offsets; a.flatten_ids = flatten_ids;
  a.render_alphas = const_cast<float *>(render_alphas);
  a.last_ids = const_cast<int32_t *>(last_ids);
  a.v_render_colors = v_render_colors; a.v_render_alphas = v_render_alphas;
  const bool ab = v_abs != nullptr;
#define GS_R16B(DD)                                                                            \
  case DD:                                                                                     \
    return ab ? r16_bwd<DD, true>(a, G, v_means2d, v_conics, v_colors, v_opacities, v_abs,     \
                                  workspace, st)                                               \
              : r16_bwd<DD, false>(a, G, v_means2d, v_conics, v_colors, v_opacities, v_abs,    \
                                   workspace, st);
  switch (D) { GS_R16B(1) GS_R16B(2) GS_R16B(3) GS_R16B(4) GS_R16B(8) GS_R16B(16) GS_R16B(32) }
#undef GS_R16B
  GS_REQUIRE(false, "rasterize16_bwd: unsupported channels %d", D);
}

}  // namespace gs
