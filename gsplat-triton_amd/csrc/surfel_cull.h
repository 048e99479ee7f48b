// The 2DGS rasterizer's culling test, shared by the rasterizer (per strip of
// a tile, csrc/surfel.hip) and the supertile isect emission's tile culling of
// large surfels (csrc/isect_st.h, the captured 2DGS training step).
#pragma once
#include "common.h"

namespace gs {
namespace surfel {

constexpr float kAlphaMin = 1.f / 255.f;

// Strip culling: false only if no pixel centre of [x0,x1]x[y0,y1] can reach
// alpha >= 1/255, i.e. sigma = min(g3, g2) / 2 > ln(255 opacity) everywhere
// (0.05 of margin on sigma and 1 px on the ellipse box absorb fp32 rounding).
//  * g2 = 2 |mean2d - p|^2: the disk |d|^2 <= ln(255 op) against the rectangle;
//  * g3 = |s(p)|^2 <= r^2 with r^2 = 2 ln(255 op) is the image of the surfel's
//    UV disk of radius r, an ellipse whose exact bounding box follows from the
//    dual conic T diag(r^2, r^2, -1) T^T of the ray transform T (the AABB
//    formula of Projection2DGSFused.cu:200-209 with the axes scaled by r).
//    It is bounded (c22 < 0) only when the whole disk lies in front of the
//    camera.  Bounded or not (a surfel whose plane passes near the camera
//    centre projects to a huge or unbounded conic), the region itself is then
//    tested against the rectangle in the UV plane (below).
GS_INLINE bool surfel_keep(const float *m, float x, float y, float op, float x0, float x1,
                           float y0, float y1) {
  if (!(op >= kAlphaMin)) return false;  // alpha <= opacity < 1/255 everywhere
  const float lnv = 0.69314718f * __builtin_amdgcn_logf(255.f * op) + 0.05f;
  const float ddx = fmaxf(fmaxf(x0 - x, x - x1), 0.f), ddy = fmaxf(fmaxf(y0 - y, y - y1), 0.f);
  if (ddx * ddx + ddy * ddy <= lnv) return true;
  const float r2 = 2.f * lnv;
  const float c22 = r2 * (m[6] * m[6] + m[7] * m[7]) - m[8] * m[8];
  if (c22 < 0.f) {  // bounded ellipse: cheap reject by its box first
    const float ic = 1.f / c22;
    const float c00 = r2 * (m[0] * m[0] + m[1] * m[1]) - m[2] * m[2];
    const float c11 = r2 * (m[3] * m[3] + m[4] * m[4]) - m[5] * m[5];
    const float c02 = r2 * (m[0] * m[6] + m[1] * m[7]) - m[2] * m[8];
    const float c12 = r2 * (m[3] * m[6] + m[4] * m[7]) - m[5] * m[8];
    const float cx = c02 * ic, cy = c12 * ic;
    const float hx = sqrtf(fmaxf(cx * cx - c00 * ic, 0.f)) + 1.f;
    const float hy = sqrtf(fmaxf(cy * cy - c11 * ic, 0.f)) + 1.f;
    if (cx + hx < x0 || cx - hx > x1 || cy + hy < y0 || cy - hy > y1) return false;
  }
  // The box overlaps: test the ellipse itself, in the surfel's UV plane
  // where it is the disk |s| <= r.  The rectangle's corners map to
  // s = c_xy / c_z with c(p) = px (v x w) + py (w x u) + (u x v) (the ray
  // cross product of the rasterizer, linear in the pixel); when c_z has one
  // sign over the rectangle the projective map sends it to a convex
  // quadrilateral, which meets the disk iff it contains the origin or an edge
  // passes within r of it.  (An edge-on surfel is a thin ellipse across the
  // image: its box covers every strip, the ellipse crosses few.  Evaluated in
  // the UV plane the test is as well conditioned as the per-pixel g3.)
  const float *u = m, *v = m + 3, *w = m + 6;
  const float a0x = v[1] * w[2] - v[2] * w[1], a0y = v[2] * w[0] - v[0] * w[2],
              a0z = v[0] * w[1] - v[1] * w[0];
  const float a1x = w[1] * u[2] - w[2] * u[1], a1y = w[2] * u[0] - w[0] * u[2],
              a1z = w[0] * u[1] - w[1] * u[0];
  const float a2x = u[1] * v[2] - u[2] * v[1], a2y = u[2] * v[0] - u[0] * v[2],
              a2z = u[0] * v[1] - u[1] * v[0];
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
  if (!(zmin > 0.f || zmax < 0.f)) return true;  // c_z changes sign: keep
  float best = 3.4e38f;
  bool pos = true, neg = true;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = (i + 1) & 3;
    const float ex = sx[j] - sx[i], ey = sy[j] - sy[i];
    const float cr = ey * sx[i] - ex * sy[i];  // (s_j - s_i) x (0 - s_i)
    pos &= cr >= 0.f;
    neg &= cr <= 0.f;
    const float L = ex * ex + ey * ey;
    const float t = L > 0.f ? fminf(fmaxf(-(sx[i] * ex + sy[i] * ey) / L, 0.f), 1.f) : 0.f;
    const float dx = sx[i] + t * ex, dy = sy[i] + t * ey;
    best = fminf(best, dx * dx + dy * dy);
  }
  return pos || neg || best <= r2;
}

}  // namespace surfel
}  // namespace gs
