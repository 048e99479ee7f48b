// Real spherical harmonics (degree 0..4) -> RGB, forward and backward, gfx950.
//
// Replaces the reference Triton kernels
//   _sh_to_color_kernel      gsplat/triton_impl/sh_fwd.py:69-191
//   _sh_to_color_vjp_kernel  gsplat/triton_impl/sh_bwd.py:36-380
// plus the torch glue `colors[~masks] = 0` / `v_coeffs[~masks] = 0`
// (gsplat/triton_impl/_wrapper.py:567-568, 589-592), which is fused here:
// masked rows are written as zeros without reading their coefficients.
//
// Mapping: one lane per row (Gaussian x camera) computing all three channels,
// so v_dirs needs no atomics (the reference uses one lane per channel and
// relaxed atomics).  The basis uses the reference's constants and the same
// g/h recurrences; the VJP uses the analytic partials of each basis function.
#include "common.h"
#include "../../include/gsplat_hip.h"

namespace gs {

// Basis values B[k] and partials dB[k] = (dB/dx, dB/dy, dB/dz) w.r.t. the
// normalised direction (sh_fwd.py:43-66 constants).
template <int DEG, bool GRAD>
GS_INLINE void sh_basis(float x, float y, float z, float *B, float (*dB)[3]) {
  B[0] = 0.28209479177387814f;
  if (GRAD) dB[0][0] = dB[0][1] = dB[0][2] = 0.f;
  if (DEG < 1) return;
  const float C1 = 0.4886025119029199f;
  B[1] = -C1 * y;
  B[2] = C1 * z;
  B[3] = -C1 * x;
  if (GRAD) {
    dB[1][0] = 0.f; dB[1][1] = -C1; dB[1][2] = 0.f;
    dB[2][0] = 0.f; dB[2][1] = 0.f; dB[2][2] = C1;
    dB[3][0] = -C1; dB[3][1] = 0.f; dB[3][2] = 0.f;
  }
  if (DEG < 2) return;
  const float zz = z * z;
  const float g2 = 2.f * x * y, h2 = x * x - y * y;
  const float C22 = 0.5462742152960396f;
  const float c21 = -1.0925484305920792f * z;
  B[4] = C22 * g2;
  B[5] = c21 * y;
  B[6] = 0.9461746957575601f * zz - 0.3153915652525201f;
  B[7] = c21 * x;
  B[8] = C22 * h2;
  if (GRAD) {
    dB[4][0] = 2.f * C22 * y; dB[4][1] = 2.f * C22 * x; dB[4][2] = 0.f;
    dB[5][0] = 0.f; dB[5][1] = c21; dB[5][2] = -1.0925484305920792f * y;
    dB[6][0] = 0.f; dB[6][1] = 0.f; dB[6][2] = 1.8923493915151202f * z;
    dB[7][0] = c21; dB[7][1] = 0.f; dB[7][2] = -1.0925484305920792f * x;
    dB[8][0] = 2.f * C22 * x; dB[8][1] = -2.f * C22 * y; dB[8][2] = 0.f;
  }
  if (DEG < 3) return;
  const float g3 = x * g2 + y * h2, h3 = x * h2 - y * g2;
  const float C33 = -0.5900435899266435f, C32 = 1.445305721320277f;
  const float c31 = -2.285228997322329f * zz + 0.4570457994644658f;
  B[9] = C33 * g3;
  B[10] = C32 * g2 * z;
  B[11] = c31 * y;
  B[12] = z * (1.865881662950577f * zz - 1.119528997770346f);
  B[13] = c31 * x;
  B[14] = C32 * h2 * z;
  B[15] = C33 * h3;
  if (GRAD) {
    const float dc31 = -4.570457994644658f * z;
    dB[9][0] = 3.f * C33 * g2; dB[9][1] = 3.f * C33 * h2; dB[9][2] = 0.f;
    dB[10][0] = 2.f * C32 * y * z; dB[10][1] = 2.f * C32 * x * z; dB[10][2] = C32 * g2;
    dB[11][0] = 0.f; dB[11][1] = c31; dB[11][2] = dc31 * y;
    dB[12][0] = 0.f; dB[12][1] = 0.f; dB[12][2] = 5.597644988851731f * zz - 1.119528997770346f;
    dB[13][0] = c31; dB[13][1] = 0.f; dB[13][2] = dc31 * x;
    dB[14][0] = 2.f * C32 * x * z; dB[14][1] = -2.f * C32 * y * z; dB[14][2] = C32 * h2;
    dB[15][0] = 3.f * C33 * h2; dB[15][1] = -3.f * C33 * g2; dB[15][2] = 0.f;
  }
  if (DEG < 4) return;
  const float g4 = x * g3 + y * h3, h4 = x * h3 - y * g3;
  const float C44 = 0.6258357354491761f, C43 = -1.7701307697799304f;
  const float c41 = z * (-4.683325804901024f * zz + 2.0071396306718676f);
  const float c42 = 3.31161143515146f * zz - 0.47308734787878f;
  B[16] = C44 * g4;
  B[17] = C43 * g3 * z;
  B[18] = c42 * g2;
  B[19] = c41 * y;
  B[20] = zz * (3.7024941420321507f * zz - 3.1735664074561294f) + 0.31735664074561293f;
  B[21] = c41 * x;
  B[22] = c42 * h2;
  B[23] = C43 * h3 * z;
  B[24] = C44 * h4;
  if (GRAD) {
    const float dc41 = -14.049977414703072f * zz + 2.0071396306718676f;
    const float dc42 = 6.62322287030292f * z;
    dB[16][0] = 4.f * C44 * g3; dB[16][1] = 4.f * C44 * h3; dB[16][2] = 0.f;
    dB[17][0] = 3.f * C43 * g2 * z; dB[17][1] = 3.f * C43 * h2 * z; dB[17][2] = C43 * g3;
    dB[18][0] = 2.f * c42 * y; dB[18][1] = 2.f * c42 * x; dB[18][2] = dc42 * g2;
    dB[19][0] = 0.f; dB[19][1] = c41; dB[19][2] = dc41 * y;
    dB[20][0] = 0.f; dB[20][1] = 0.f; dB[20][2] = z * (14.809976568128603f * zz - 6.347132814912259f);
    dB[21][0] = c41; dB[21][1] = 0.f; dB[21][2] = dc41 * x;
    dB[22][0] = 2.f * c42 * x; dB[22][1] = -2.f * c42 * y; dB[22][2] = dc42 * h2;
    dB[23][0] = 3.f * C43 * h2 * z; dB[23][1] = -3.f * C43 * g2 * z; dB[23][2] = C43 * h3;
    dB[24][0] = 4.f * C44 * h3; dB[24][1] = -4.f * C44 * g3; dB[24][2] = 0.f;
  }
}

// Coefficient addressing: basis 0 (the DC term) lives at c0 + row*s0, bases
// k >= 1 at cr + row*sr + 3*(k-1).  One [rows,K,3] tensor is c0 = coeffs,
// cr = coeffs + 3, s0 = sr = 3K; the trainer's separate sh0 [N,1,3] / shN
// [N,K-1,3] parameters are read in place (no torch.cat copy per step).
struct Coeffs {
  const float *c0, *cr;
  int64_t s0, sr;
};
struct VCoeffs {
  float *c0, *cr;
  int64_t s0, sr;
};

// The rasterization() colour path fused in (gsplat/rendering.py:396-406):
// dirs = means - camera centre (the centre from the world-to-camera matrix,
// -R^T t, instead of torch.inverse), masks = radii > 0, and the output
// transform clamp_min(sh + 0.5, 0) with its backward mask (input >= 0, as
// torch.clamp_min).  Masked rows give 0.5, as `colors[~masks] = 0` then + 0.5.
struct Fused {
  const float *means;     // [N, 3]
  const float *viewmats;  // [C, 4, 4]
  const int32_t *radii;   // [C, N]
  int64_t N;
};

GS_INLINE void fused_dir_cg(const Fused &fz, int64_t c, int64_t g, float &x, float &y, float &z) {
  const float *vm = fz.viewmats + 16 * c;
  const float t0 = vm[3], t1 = vm[7], t2 = vm[11];
  const float px = -(vm[0] * t0 + vm[4] * t1 + vm[8] * t2);
  const float py = -(vm[1] * t0 + vm[5] * t1 + vm[9] * t2);
  const float pz = -(vm[2] * t0 + vm[6] * t1 + vm[10] * t2);
  const float *m = fz.means + 3 * g;
  x = m[0] - px;
  y = m[1] - py;
  z = m[2] - pz;
}

// row i of [C, N]; one camera (n == N, the training step): no 64-bit
// division per lane
GS_INLINE void fused_dir(const Fused &fz, int64_t i, float &x, float &y, float &z, bool one_cam) {
  const int64_t c = one_cam ? 0 : i / fz.N;
  fused_dir_cg(fz, c, i - c * fz.N, x, y, z);
}

template <int DEG, bool FUSED>
__global__ void __launch_bounds__(256)
sh_fwd_kernel(int64_t n, int64_t n_coeff_rows, Coeffs cf, const float *__restrict__ dirs,
              const uint8_t *__restrict__ masks, float *__restrict__ colors, Fused fz) {
  constexpr int NB = (DEG + 1) * (DEG + 1);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float *o = colors + 3 * i;
  const bool on = FUSED ? fz.radii[i] > 0 : (!masks || masks[i]);
  if (!on) {
    const float v = FUSED ? 0.5f : 0.f;
    o[0] = v; o[1] = v; o[2] = v;
    return;
  }
  float x = 0.f, y = 0.f, z = 0.f;
  if (DEG > 0) {
    if (FUSED) {
      fused_dir(fz, i, x, y, z, n == fz.N);
    } else {
      const float *d = dirs + 3 * i;
      x = d[0]; y = d[1]; z = d[2];
    }
    const float inorm = rsqrtf(x * x + y * y + z * z);
    x *= inorm; y *= inorm; z *= inorm;
  }
  float B[NB];
  sh_basis<DEG, false>(x, y, z, B, nullptr);
  const int64_t row = n_coeff_rows == n ? i : i % n_coeff_rows;
  const float *p0 = cf.c0 + row * cf.s0;
  const float *pr = cf.cr + row * cf.sr;
  float r = B[0] * p0[0], g = B[0] * p0[1], b = B[0] * p0[2];
#pragma unroll
  for (int k = 1; k < NB; ++k) {
    r += B[k] * pr[3 * (k - 1)];
    g += B[k] * pr[3 * (k - 1) + 1];
    b += B[k] * pr[3 * (k - 1) + 2];
  }
  if (FUSED) {
    r = fmaxf(r + 0.5f, 0.f);
    g = fmaxf(g + 0.5f, 0.f);
    b = fmaxf(b + 0.5f, 0.f);
  }
  o[0] = r; o[1] = g; o[2] = b;
}

template <int DEG, bool FUSED>
__global__ void __launch_bounds__(256)
sh_bwd_kernel(int64_t n, int K, int64_t n_coeff_rows, Coeffs cf, const float *__restrict__ dirs,
              const uint8_t *__restrict__ masks, const float *__restrict__ v_colors, VCoeffs vc,
              float *__restrict__ v_dirs, Fused fz) {
  constexpr int NB = (DEG + 1) * (DEG + 1);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float *v0 = vc.c0 + i * vc.s0;
  float *vr_ = vc.cr + i * vc.sr;
  const bool on = FUSED ? fz.radii[i] > 0 : (!masks || masks[i]);
  if (!on) {
    v0[0] = 0.f; v0[1] = 0.f; v0[2] = 0.f;
    for (int k = 0; k < 3 * (K - 1); ++k) vr_[k] = 0.f;
    if (v_dirs) { v_dirs[3 * i] = 0.f; v_dirs[3 * i + 1] = 0.f; v_dirs[3 * i + 2] = 0.f; }
    return;
  }
  float vr = v_colors[3 * i], vg = v_colors[3 * i + 1], vb = v_colors[3 * i + 2];
  float x = 0.f, y = 0.f, z = 0.f, inorm = 0.f;
  if (DEG > 0) {
    if (FUSED) {
      fused_dir(fz, i, x, y, z, n == fz.N);
    } else {
      const float *d = dirs + 3 * i;
      x = d[0]; y = d[1]; z = d[2];
    }
    inorm = rsqrtf(x * x + y * y + z * z);
    x *= inorm; y *= inorm; z *= inorm;
  }
  float B[NB];
  float dB[NB][3];
  const bool want_dirs = (v_dirs != nullptr) && DEG > 0;
  if (want_dirs) sh_basis<DEG, true>(x, y, z, B, dB);
  else sh_basis<DEG, false>(x, y, z, B, nullptr);
  if (FUSED) {  // clamp_min(sh + 0.5, 0) passes the gradient where sh + 0.5 >= 0
    const int64_t row = i % n_coeff_rows;
    const float *p0 = cf.c0 + row * cf.s0;
    const float *pr = cf.cr + row * cf.sr;
    float r = B[0] * p0[0], g = B[0] * p0[1], b = B[0] * p0[2];
#pragma unroll
    for (int k = 1; k < NB; ++k) {
      r += B[k] * pr[3 * (k - 1)];
      g += B[k] * pr[3 * (k - 1) + 1];
      b += B[k] * pr[3 * (k - 1) + 2];
    }
    vr = (r + 0.5f >= 0.f) ? vr : 0.f;
    vg = (g + 0.5f >= 0.f) ? vg : 0.f;
    vb = (b + 0.5f >= 0.f) ? vb : 0.f;
  }
  v0[0] = B[0] * vr; v0[1] = B[0] * vg; v0[2] = B[0] * vb;
#pragma unroll
  for (int k = 1; k < NB; ++k) {
    vr_[3 * (k - 1)] = B[k] * vr;
    vr_[3 * (k - 1) + 1] = B[k] * vg;
    vr_[3 * (k - 1) + 2] = B[k] * vb;
  }
  for (int k = 3 * (NB - 1); k < 3 * (K - 1); ++k) vr_[k] = 0.f;
  if (v_dirs) {
    if (DEG == 0) {
      v_dirs[3 * i] = 0.f; v_dirs[3 * i + 1] = 0.f; v_dirs[3 * i + 2] = 0.f;
      return;
    }
    const float *pr = cf.cr + (i % n_coeff_rows) * cf.sr;
    float vx = 0.f, vy = 0.f, vz = 0.f;
#pragma unroll
    for (int k = 1; k < NB; ++k) {
      const float w = pr[3 * (k - 1)] * vr + pr[3 * (k - 1) + 1] * vg + pr[3 * (k - 1) + 2] * vb;
      vx += dB[k][0] * w;
      vy += dB[k][1] * w;
      vz += dB[k][2] * w;
    }
    // VJP of the normalisation (sh_bwd.py:367-380)
    const float dot = x * vx + y * vy + z * vz;
    v_dirs[3 * i] = (vx - dot * x) * inorm;
    v_dirs[3 * i + 1] = (vy - dot * y) * inorm;
    v_dirs[3 * i + 2] = (vz - dot * z) * inorm;
  }
}

// Walks the elements e = lane, lane + 64, ... of a block of rows of WID
// floats, tracking (row, column) without divisions.
template <int WID>
struct RowWalk {
  int rr, c;
  GS_INLINE explicit RowWalk(int lane) : rr(lane / WID), c(lane % WID) {}
  GS_INLINE void next() {
    rr += 64 / WID;
    c += 64 % WID;
    if (c >= WID) {
      c -= WID;
      rr += 1;
    }
  }
};

// Backward with the gradient rows staged through LDS (K == (DEG+1)^2 and one
// coefficient row per lane row, i.e. C == 1).  A visible lane loads its row's
// coefficients straight into registers (all loads in flight at once) and
// writes its gradient row to LDS; the wave then stores its 64 rows (zeros
// for masked rows) lane-contiguously, instead of 3K stores per lane that each
// touch 64 cache lines.  LDS rows have an odd stride (bank-conflict free).
//
// ADAM: instead of storing the gradient rows, apply torch.optim.Adam to the
// coefficient rows in place (the optimizer step fused into its producer:
// the gradient never goes through HBM).  KR = rest coefficients per row
// (the parameter's K - 1; those above the active degree get zero gradient
// and still their Adam update).


struct AdamSH {
  float *m0, *v0, *mr, *vr;  // moments of coeffs / coeffs_rest, same layout
  float ss0, ssr, ib, b1, b2, eps;
  // captured-step form (gsplat_hip_sh_colors_bwd_adam_dev): {ss0, ssr, ib}
  // read on the device, and a void step (*skip != 0) leaves the state alone
  const float *hyper;
  const int32_t *skip;
  int nt;  // non-temporal row loads / stores (always on)
};

// The rows are touched once per step: non-temporal loads / stores stream
// them past the caches (M2 804.8 / 805.4 against 795.3 / 797.2 images/s
// with plain accesses, alternating in one call, profiles/r4_batch10/).
static int sh_adam_nt() { return 1; }
typedef float f4v __attribute__((ext_vector_type(4)));
GS_INLINE float4 ld4(const float4 *p, bool nt) {
  if (nt) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return *p;
}
GS_INLINE void st4(float4 *p, const float4 &v, bool nt) {
  if (nt)
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v *>(p));
  else
    *p = v;
}

// Adam over `rows` consecutive rows of WID floats (16-B aligned start): the
// gradient of element (r, c) is g[r * GS + c] (LDS); 4 elements per lane and
// iteration as float4, a scalar tail.  kU float4 slots per lane and
// iteration, all their loads issued before any update (the stores may alias
// the next slot's loads as far as the compiler knows): at the 3 workgroups
// per CU the LDS staging allows, one slot left 3 x 16 B per lane in flight
// (M2 776.2 / 774.1 vs 773.8 / 765.5 images/s, profiles/r4_batch/).
constexpr int kU = 4;
template <int WID, int GS>
GS_INLINE void adam_rows(float *P, float *M, float *V, const float *g, int rows, int lane,
                         float ss, const AdamSH &ad) {
  const int count = rows * WID, n4 = count >> 2;
  float4 *P4 = reinterpret_cast<float4 *>(P);
  float4 *M4 = reinterpret_cast<float4 *>(M);
  float4 *V4 = reinterpret_cast<float4 *>(V);
  auto gr = [&](int e) {
    const int r = e / WID;
    return g[r * GS + (e - r * WID)];
  };
  for (int q0 = lane; q0 < n4; q0 += 64 * kU) {
    float4 p[kU], m[kU], v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int q = q0 + 64 * u;
      if (q < n4) {
        p[u] = ld4(P4 + q, ad.nt);
        m[u] = ld4(M4 + q, ad.nt);
        v[u] = ld4(V4 + q, ad.nt);
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int q = q0 + 64 * u;
      if (q < n4) {
        const int e = 4 * q;
        adam_update(p[u].x, gr(e), m[u].x, v[u].x, ad.b1, ad.b2, ad.eps, ss, ad.ib);
        adam_update(p[u].y, gr(e + 1), m[u].y, v[u].y, ad.b1, ad.b2, ad.eps, ss, ad.ib);
        adam_update(p[u].z, gr(e + 2), m[u].z, v[u].z, ad.b1, ad.b2, ad.eps, ss, ad.ib);
        adam_update(p[u].w, gr(e + 3), m[u].w, v[u].w, ad.b1, ad.b2, ad.eps, ss, ad.ib);
        st4(P4 + q, p[u], ad.nt);
        st4(M4 + q, m[u], ad.nt);
        st4(V4 + q, v[u], ad.nt);
      }
    }
  }
  for (int e = 4 * n4 + lane; e < count; e += 64) {
    float pp = P[e], mm = M[e], vv = V[e];
    adam_update(pp, gr(e), mm, vv, ad.b1, ad.b2, ad.eps, ss, ad.ib);
    P[e] = pp;
    M[e] = mm;
    V[e] = vv;
  }
}

// CAMS (FUSED): the row of lane i is Gaussian i seen from all C cameras of
// fz (C = fz's camera count, rows c * N + i of radii / v_colors): the
// coefficients are read once, the gradient rows and the means gradient
// (v_dirs [N, 3]) are summed over the cameras in registers -- the shared
// coefficients of a Gaussian-sharded render's N-camera colours, whose sum
// is also what the fused Adam needs.  C == 1 is the one-camera kernel.
template <int DEG, bool FUSED, int KR = (DEG + 1) * (DEG + 1) - 1, bool ADAM = false,
          bool CAMS = false>
__global__ void __launch_bounds__(256)
sh_bwd_staged_kernel(int64_t n, Coeffs cf, const float *__restrict__ dirs,
                     const uint8_t *__restrict__ masks, const float *__restrict__ v_colors,
                     VCoeffs vc, float *__restrict__ v_dirs, Fused fz, AdamSH ad = AdamSH{},
                     int C = 1) {
  static_assert(!CAMS || FUSED, "the camera loop is the fused colour path's");
  if (!CAMS) C = 1;
  constexpr int NB = (DEG + 1) * (DEG + 1), WR = 3 * KR, RSR = WR | 1;
  static_assert(KR >= NB - 1, "KR covers the active coefficients");
  __shared__ float l_dc[4][64 * 3];               // row stride 3 (odd)
  __shared__ float l_rest[4][64 * (RSR > 1 ? RSR : 1)];  // odd row stride
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t i0 = (int64_t)blockIdx.x * 256 + wid * 64;
  if (i0 >= n) return;
  const int rows = (int)min<int64_t>(64, n - i0);
  const int64_t i = i0 + lane;
  float *sd = l_dc[wid], *sr = l_rest[wid];
  bool seen = false;
  if (FUSED && lane < rows)
    for (int c = 0; c < (CAMS ? C : 1); ++c) seen |= fz.radii[(int64_t)c * fz.N + i] > 0;
  const bool on = lane < rows && (FUSED ? seen : (!masks || masks[i]));
  float *rd = sd + lane * 3, *rw = sr + lane * RSR;
  // this lane's gradient row in LDS (coefficient k, channel ch)
  auto grow = [&](int k, int ch) -> float & { return k == 0 ? rd[ch] : rw[3 * (k - 1) + ch]; };
  if (on) {
    // the row's coefficients straight into registers: all loads in flight at
    // once (strided per lane, but every fetched line is used)
    float cr[NB][3];
    {
      const float *p0 = cf.c0 + i * cf.s0, *pr = cf.cr + i * cf.sr;
#pragma unroll
      for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) cr[k][ch] = k == 0 ? p0[ch] : pr[3 * (k - 1) + ch];
    }
    auto coef = [&](int k, int ch) { return cr[k][ch]; };
    const bool want_dirs = (v_dirs != nullptr) && DEG > 0;
    float ga[NB][3];
#pragma unroll
    for (int k = 0; k < NB; ++k) ga[k][0] = ga[k][1] = ga[k][2] = 0.f;
    float sx = 0.f, sy = 0.f, sz = 0.f;  // the means gradient, summed over cameras
    for (int c = 0; c < (CAMS ? C : 1); ++c) {
      const int64_t ri = CAMS ? (int64_t)c * fz.N + i : i;
      if (CAMS && !(fz.radii[ri] > 0)) continue;
      float vr = v_colors[3 * ri], vg = v_colors[3 * ri + 1], vb = v_colors[3 * ri + 2];
      float x = 0.f, y = 0.f, z = 0.f, inorm = 0.f;
      if (DEG > 0) {
        if (FUSED) {
          // CAMS: ri = c N + i.  Otherwise row i of [C, N] (per-camera
          // coefficients [C, N, K, 3]): camera and Gaussian from i, with no
          // division when there is one camera (n == N)
          if (CAMS) fused_dir_cg(fz, c, i, x, y, z);
          else fused_dir(fz, i, x, y, z, n == fz.N);
        } else {
          x = dirs[3 * i]; y = dirs[3 * i + 1]; z = dirs[3 * i + 2];
        }
        inorm = rsqrtf(x * x + y * y + z * z);
        x *= inorm; y *= inorm; z *= inorm;
      }
      float B[NB];
      float dB[NB][3];
      if (want_dirs) sh_basis<DEG, true>(x, y, z, B, dB);
      else sh_basis<DEG, false>(x, y, z, B, nullptr);
      if (FUSED) {  // clamp_min(sh + 0.5, 0) passes the gradient where sh + 0.5 >= 0
        float r = 0.f, g = 0.f, b = 0.f;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          r += B[k] * coef(k, 0);
          g += B[k] * coef(k, 1);
          b += B[k] * coef(k, 2);
        }
        vr = (r + 0.5f >= 0.f) ? vr : 0.f;
        vg = (g + 0.5f >= 0.f) ? vg : 0.f;
        vb = (b + 0.5f >= 0.f) ? vb : 0.f;
      }
      if (want_dirs) {
        float vx = 0.f, vy = 0.f, vz = 0.f;
#pragma unroll
        for (int k = 1; k < NB; ++k) {
          const float w = coef(k, 0) * vr + coef(k, 1) * vg + coef(k, 2) * vb;
          vx += dB[k][0] * w;
          vy += dB[k][1] * w;
          vz += dB[k][2] * w;
        }
        // VJP of the normalisation (sh_bwd.py:367-380)
        const float dot = x * vx + y * vy + z * vz;
        sx += (vx - dot * x) * inorm;
        sy += (vy - dot * y) * inorm;
        sz += (vz - dot * z) * inorm;
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        ga[k][0] += B[k] * vr;
        ga[k][1] += B[k] * vg;
        ga[k][2] += B[k] * vb;
      }
    }
    if (v_dirs) {
      v_dirs[3 * i] = sx; v_dirs[3 * i + 1] = sy; v_dirs[3 * i + 2] = sz;
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      grow(k, 0) = ga[k][0];
      grow(k, 1) = ga[k][1];
      grow(k, 2) = ga[k][2];
    }
#pragma unroll
    for (int k = NB; k <= KR; ++k) grow(k, 0) = grow(k, 1) = grow(k, 2) = 0.f;
  } else if (lane < rows) {
#pragma unroll
    for (int k = 0; k <= KR; ++k) grow(k, 0) = grow(k, 1) = grow(k, 2) = 0.f;
    if (v_dirs) { v_dirs[3 * i] = 0.f; v_dirs[3 * i + 1] = 0.f; v_dirs[3 * i + 2] = 0.f; }
  }
  __builtin_amdgcn_wave_barrier();
  if (ADAM) {  // Adam on the wave's 64 coefficient rows: 16-B vectors, lane-contiguous
    if (ad.skip && *ad.skip) return;
    AdamSH a = ad;
    if (ad.hyper) {
      a.ss0 = ad.hyper[0];
      a.ssr = ad.hyper[1];
      a.ib = ad.hyper[2];
    }
    adam_rows<3, 3>(const_cast<float *>(cf.c0) + i0 * 3, a.m0 + i0 * 3, a.v0 + i0 * 3, sd,
                    rows, lane, a.ss0, a);
    if (WR > 0)
      adam_rows<(WR > 0 ? WR : 1), RSR>(const_cast<float *>(cf.cr) + i0 * WR, a.mr + i0 * WR,
                                         a.vr + i0 * WR, sr, rows, lane, a.ssr, a);
    return;
  }
  {  // gradient rows out, lane-contiguous
    float *g0 = vc.c0 + i0 * vc.s0;
    RowWalk<3> w0(lane);
    for (int e = lane; e < rows * 3; e += 64, w0.next())
      g0[(int64_t)w0.rr * vc.s0 + w0.c] = sd[w0.rr * 3 + w0.c];
    if (WR > 0) {
      float *gr = vc.cr + i0 * vc.sr;
      RowWalk<(WR > 0 ? WR : 1)> wr(lane);
      for (int e = lane; e < rows * WR; e += 64, wr.next())
        gr[(int64_t)wr.rr * vc.sr + wr.c] = sr[wr.rr * RSR + wr.c];
    }
  }
}

}  // namespace gs

using namespace gs;

static int sh_check(int degree, int64_t n, int64_t n_coeff_rows, int K, const char *who) {
  GS_REQUIRE(degree >= 0 && degree <= 4, "%s: degree %d not in [0, 4]", who, degree);
  GS_REQUIRE(K >= (degree + 1) * (degree + 1) && K <= 25, "%s: K=%d too small for degree %d",
             who, K, degree);
  GS_REQUIRE(n_coeff_rows > 0 && n % n_coeff_rows == 0,
             "%s: n=%lld not a multiple of n_coeff_rows=%lld", who, (long long)n,
             (long long)n_coeff_rows);
  return 0;
}

extern "C" int gsplat_hip_sh_fwd(int degree, int64_t n, int64_t n_coeff_rows, int K,
                                 const float *dirs, const float *coeffs,
                                 const float *coeffs_rest, const uint8_t *masks, float *colors,
                                 void *stream) {
  if (n <= 0) return 0;
  if (int e = sh_check(degree, n, n_coeff_rows, K, "sh_fwd")) return e;
  Coeffs cf = coeffs_rest ? Coeffs{coeffs, coeffs_rest, 3, 3 * (int64_t)(K - 1)}
                          : Coeffs{coeffs, coeffs + 3, 3 * (int64_t)K, 3 * (int64_t)K};
  dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
#define GS_SH_FWD(D)                                                                   \
  case D:                                                                              \
    hipLaunchKernelGGL((sh_fwd_kernel<D, false>), grid, dim3(256), 0, st, n, n_coeff_rows, \
                       cf, dirs, masks, colors, Fused{});                                \
    break;
  switch (degree) { GS_SH_FWD(0) GS_SH_FWD(1) GS_SH_FWD(2) GS_SH_FWD(3) GS_SH_FWD(4) }
#undef GS_SH_FWD
  GS_CHECK_LAUNCH("sh_fwd");
  return 0;
}

extern "C" int gsplat_hip_sh_bwd(int degree, int64_t n, int64_t n_coeff_rows, int K,
                                 const float *dirs, const float *coeffs,
                                 const float *coeffs_rest, const uint8_t *masks,
                                 const float *v_colors, float *v_coeffs, float *v_coeffs_rest,
                                 float *v_dirs, void *stream) {
  if (n <= 0) return 0;
  if (int e = sh_check(degree, n, n_coeff_rows, K, "sh_bwd")) return e;
  GS_REQUIRE(!coeffs_rest == !v_coeffs_rest,
             "sh_bwd: coeffs_rest and v_coeffs_rest must both be given or both null");
  Coeffs cf = coeffs_rest ? Coeffs{coeffs, coeffs_rest, 3, 3 * (int64_t)(K - 1)}
                          : Coeffs{coeffs, coeffs + 3, 3 * (int64_t)K, 3 * (int64_t)K};
  VCoeffs vc = v_coeffs_rest ? VCoeffs{v_coeffs, v_coeffs_rest, 3, 3 * (int64_t)(K - 1)}
                             : VCoeffs{v_coeffs, v_coeffs + 3, 3 * (int64_t)K, 3 * (int64_t)K};
  dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  const bool staged = n_coeff_rows == n && K == (degree + 1) * (degree + 1);
#define GS_SH_BWD(D)                                                                       \
  case D:                                                                                  \
    if (staged)                                                                            \
      hipLaunchKernelGGL((sh_bwd_staged_kernel<D, false>), grid, dim3(256), 0, st, n, cf,  \
                         dirs, masks, v_colors, vc, v_dirs, Fused{});                      \
    else                                                                                   \
      hipLaunchKernelGGL((sh_bwd_kernel<D, false>), grid, dim3(256), 0, st, n, K,          \
                         n_coeff_rows, cf, dirs, masks, v_colors, vc, v_dirs, Fused{});    \
    break;
  switch (degree) { GS_SH_BWD(0) GS_SH_BWD(1) GS_SH_BWD(2) GS_SH_BWD(3) GS_SH_BWD(4) }
#undef GS_SH_BWD
  GS_CHECK_LAUNCH("sh_bwd");
  return 0;
}

// rasterization()'s colour path in one kernel each way (see struct Fused):
// colors[C,N,3] = clamp_min(SH(means - campos(viewmats)) + 0.5, 0), radii
// masking.  Backward: v_coeffs (and v_coeffs_rest) per row, v_dirs[C,N,3]
// (= the gradient of means per camera; NULL to skip).
extern "C" int gsplat_hip_sh_colors_fwd(int degree, int C, int64_t N, int64_t n_coeff_rows, int K,
                                        const float *means, const float *viewmats,
                                        const float *coeffs, const float *coeffs_rest,
                                        const int32_t *radii, float *colors, void *stream) {
  const int64_t n = (int64_t)C * N;
  if (n <= 0) return 0;
  if (int e = sh_check(degree, n, n_coeff_rows, K, "sh_colors_fwd")) return e;
  Coeffs cf = coeffs_rest ? Coeffs{coeffs, coeffs_rest, 3, 3 * (int64_t)(K - 1)}
                          : Coeffs{coeffs, coeffs + 3, 3 * (int64_t)K, 3 * (int64_t)K};
  const Fused fz{means, viewmats, radii, N};
  dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
#define GS_SH_FWD(D)                                                                        \
  case D:                                                                                   \
    hipLaunchKernelGGL((sh_fwd_kernel<D, true>), grid, dim3(256), 0, st, n, n_coeff_rows, cf, \
                       nullptr, nullptr, colors, fz);                                       \
    break;
  switch (degree) { GS_SH_FWD(0) GS_SH_FWD(1) GS_SH_FWD(2) GS_SH_FWD(3) GS_SH_FWD(4) }
#undef GS_SH_FWD
  GS_CHECK_LAUNCH("sh_colors_fwd");
  return 0;
}

extern "C" int gsplat_hip_sh_colors_bwd(int degree, int C, int64_t N, int64_t n_coeff_rows, int K,
                                        const float *means, const float *viewmats,
                                        const float *coeffs, const float *coeffs_rest,
                                        const int32_t *radii, const float *v_colors,
                                        float *v_coeffs, float *v_coeffs_rest, float *v_dirs,
                                        void *stream) {
  const int64_t n = (int64_t)C * N;
  if (n <= 0) return 0;
  if (int e = sh_check(degree, n, n_coeff_rows, K, "sh_colors_bwd")) return e;
  GS_REQUIRE(!coeffs_rest == !v_coeffs_rest,
             "sh_colors_bwd: coeffs_rest and v_coeffs_rest must both be given or both null");
  Coeffs cf = coeffs_rest ? Coeffs{coeffs, coeffs_rest, 3, 3 * (int64_t)(K - 1)}
                          : Coeffs{coeffs, coeffs + 3, 3 * (int64_t)K, 3 * (int64_t)K};
  VCoeffs vc = v_coeffs_rest ? VCoeffs{v_coeffs, v_coeffs_rest, 3, 3 * (int64_t)(K - 1)}
                             : VCoeffs{v_coeffs, v_coeffs + 3, 3 * (int64_t)K, 3 * (int64_t)K};
  const Fused fz{means, viewmats, radii, N};
  dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  const bool staged = n_coeff_rows == n && K == (degree + 1) * (degree + 1);
#define GS_SH_BWD(D)                                                                       \
  case D:                                                                                  \
    if (staged)                                                                            \
      hipLaunchKernelGGL((sh_bwd_staged_kernel<D, true>), grid, dim3(256), 0, st, n, cf,   \
                         nullptr, nullptr, v_colors, vc, v_dirs, fz);                      \
    else                                                                                   \
      hipLaunchKernelGGL((sh_bwd_kernel<D, true>), grid, dim3(256), 0, st, n, K,           \
                         n_coeff_rows, cf, nullptr, nullptr, v_colors, vc, v_dirs, fz);    \
    break;
  switch (degree) { GS_SH_BWD(0) GS_SH_BWD(1) GS_SH_BWD(2) GS_SH_BWD(3) GS_SH_BWD(4) }
#undef GS_SH_BWD
  GS_CHECK_LAUNCH("sh_colors_bwd");
  return 0;
}

// gsplat_hip_sh_colors_bwd with the coefficients' Adam step fused in (C == 1,
// one coefficient row per Gaussian, K == 16 with coeffs_rest): coeffs and
// coeffs_rest are updated in place with torch.optim.Adam (lr0 / lr_rest,
// shared betas / eps, 1-based step) from the gradient this backward computes,
// which is never stored; v_dirs as in gsplat_hip_sh_colors_bwd.
static int sh_colors_bwd_adam_launch(int degree, int C, int64_t N, const float *means,
                                     const float *viewmats, float *coeffs, float *coeffs_rest,
                                     const int32_t *radii, const float *v_colors, float *v_dirs,
                                     const AdamSH &ad, hipStream_t st);

extern "C" int gsplat_hip_sh_colors_bwd_adam(int degree, int C, int64_t N, const float *means,
                                             const float *viewmats, float *coeffs,
                                             float *coeffs_rest, const int32_t *radii,
                                             const float *v_colors, float *v_dirs, float *m0,
                                             float *v0, float *m_rest, float *v_rest, float lr0,
                                             float lr_rest, float beta1, float beta2, float eps,
                                             int step, void *stream) {
  if (N <= 0) return 0;
  GS_REQUIRE(degree >= 0 && degree <= 3, "sh_colors_bwd_adam: degree %d not in [0, 3]", degree);
  GS_REQUIRE(coeffs && coeffs_rest && m0 && v0 && m_rest && v_rest,
             "sh_colors_bwd_adam: null coefficient or moment buffer");
  GS_REQUIRE(step >= 1, "sh_colors_bwd_adam: step must be >= 1");
  GS_REQUIRE((((uintptr_t)coeffs | (uintptr_t)coeffs_rest | (uintptr_t)m0 | (uintptr_t)v0 |
               (uintptr_t)m_rest | (uintptr_t)v_rest) & 15) == 0,
             "sh_colors_bwd_adam: coefficient and moment buffers must be 16-B aligned");
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  AdamSH ad{m0, v0, m_rest, v_rest, (float)(lr0 / bc1), (float)(lr_rest / bc1),
            (float)(1.0 / sqrt(bc2)), beta1, beta2, eps, nullptr, nullptr, sh_adam_nt()};
  return sh_colors_bwd_adam_launch(degree, C, N, means, viewmats, coeffs, coeffs_rest, radii,
                                   v_colors, v_dirs, ad, (hipStream_t)stream);
}

// The same with the step-dependent factors read on the device (ABI 20, a
// captured training step): hyper_device = {lr0 / (1 - beta1^t),
// lr_rest / (1 - beta1^t), 1 / sqrt(1 - beta2^t)}; skip_device (may be NULL)
// non-zero: the coefficients and moments are left alone (v_dirs is written).
extern "C" int gsplat_hip_sh_colors_bwd_adam_dev(int degree, int C, int64_t N,
                                                 const float *means,
                                                 const float *viewmats, float *coeffs,
                                                 float *coeffs_rest, const int32_t *radii,
                                                 const float *v_colors, float *v_dirs, float *m0,
                                                 float *v0, float *m_rest, float *v_rest,
                                                 const float *hyper_device, float beta1,
                                                 float beta2, float eps,
                                                 const int32_t *skip_device, void *stream) {
  if (N <= 0) return 0;
  GS_REQUIRE(degree >= 0 && degree <= 3, "sh_colors_bwd_adam: degree %d not in [0, 3]", degree);
  GS_REQUIRE(coeffs && coeffs_rest && m0 && v0 && m_rest && v_rest && hyper_device,
             "sh_colors_bwd_adam: null coefficient, moment or hyper buffer");
  GS_REQUIRE((((uintptr_t)coeffs | (uintptr_t)coeffs_rest | (uintptr_t)m0 | (uintptr_t)v0 |
               (uintptr_t)m_rest | (uintptr_t)v_rest) & 15) == 0,
             "sh_colors_bwd_adam: coefficient and moment buffers must be 16-B aligned");
  AdamSH ad{m0, v0, m_rest, v_rest, 0.f, 0.f, 0.f, beta1, beta2, eps, hyper_device, skip_device,
            sh_adam_nt()};
  return sh_colors_bwd_adam_launch(degree, C, N, means, viewmats, coeffs, coeffs_rest, radii,
                                   v_colors, v_dirs, ad, (hipStream_t)stream);
}

static int sh_colors_bwd_adam_launch(int degree, int C, int64_t N, const float *means,
                                     const float *viewmats, float *coeffs, float *coeffs_rest,
                                     const int32_t *radii, const float *v_colors, float *v_dirs,
                                     const AdamSH &ad, hipStream_t st) {
  GS_REQUIRE(C >= 1, "sh_colors_bwd_adam: C=%d cameras", C);
  Coeffs cf{coeffs, coeffs_rest, 3, 45};
  VCoeffs vc{nullptr, nullptr, 3, 45};
  const Fused fz{means, viewmats, radii, N};
  dim3 grid((unsigned)((N + 255) / 256));
#define GS_SH_BWD_ADAM(D)                                                                        \
  case D:                                                                                        \
    if (C == 1)                                                                                  \
      hipLaunchKernelGGL((sh_bwd_staged_kernel<D, true, 15, true>), grid, dim3(256), 0, st, N,   \
                         cf, nullptr, nullptr, v_colors, vc, v_dirs, fz, ad, 1);                 \
    else                                                                                         \
      hipLaunchKernelGGL((sh_bwd_staged_kernel<D, true, 15, true, true>), grid, dim3(256), 0, st, \
                         N, cf, nullptr, nullptr, v_colors, vc, v_dirs, fz, ad, C);              \
    break;
  switch (degree) { GS_SH_BWD_ADAM(0) GS_SH_BWD_ADAM(1) GS_SH_BWD_ADAM(2) GS_SH_BWD_ADAM(3) }
#undef GS_SH_BWD_ADAM
  GS_CHECK_LAUNCH("sh_colors_bwd_adam");
  return 0;
}

// rasterization()'s colour backward for C cameras sharing the coefficient
// rows (one [N] row set, the trainer's sh0 [N,1,3] + shN [N,15,3]): v_coeffs
// / v_coeffs_rest [N] and v_dirs [N, 3] are the sums over the cameras, formed
// in registers (gsplat_hip_sh_colors_bwd writes per-camera rows that torch
// then sums).  The Gaussian-sharded render's colours (C = world cameras).
extern "C" int gsplat_hip_sh_colors_bwd_sum(int degree, int C, int64_t N, const float *means,
                                            const float *viewmats, const float *coeffs,
                                            const float *coeffs_rest, const int32_t *radii,
                                            const float *v_colors, float *v_coeffs,
                                            float *v_coeffs_rest, float *v_dirs, void *stream) {
  if (N <= 0) return 0;
  GS_REQUIRE(degree >= 0 && degree <= 3, "sh_colors_bwd_sum: degree %d not in [0, 3]", degree);
  GS_REQUIRE(C >= 1, "sh_colors_bwd_sum: C=%d cameras", C);
  GS_REQUIRE(coeffs && coeffs_rest && v_coeffs && v_coeffs_rest,
             "sh_colors_bwd_sum: coefficients as (sh0 [N,1,3], shN [N,15,3]) and both gradients");
  Coeffs cf{coeffs, coeffs_rest, 3, 45};
  VCoeffs vc{v_coeffs, v_coeffs_rest, 3, 45};
  const Fused fz{means, viewmats, radii, N};
  dim3 grid((unsigned)((N + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
#define GS_SH_BWD_SUM(D)                                                                        \
  case D:                                                                                       \
    hipLaunchKernelGGL((sh_bwd_staged_kernel<D, true, 15, false, true>), grid, dim3(256), 0, st, \
                       N, cf, nullptr, nullptr, v_colors, vc, v_dirs, fz, AdamSH{}, C);         \
    break;
  switch (degree) { GS_SH_BWD_SUM(0) GS_SH_BWD_SUM(1) GS_SH_BWD_SUM(2) GS_SH_BWD_SUM(3) }
#undef GS_SH_BWD_SUM
  GS_CHECK_LAUNCH("sh_colors_bwd_sum");
  return 0;
}
