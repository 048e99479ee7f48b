// Rasterizer for 16x16 tiles (the gsplat default), gfx950.
//
// Same semantics as rasterize.hip (reference: rasterize_to_pixels_fwd.py:13-196,
// rasterize_to_pixels_bwd.py:13-337), different mapping, built for CDNA4:
//
//  * forward: a 256-thread workgroup per tile, each wave64 owns a 16x4 strip
//    (one pixel per lane) and walks the tile's isects alone -- no workgroup
//    barriers; heavy tiles may be split into chunks rendered by several
//    workgroups of the same launch ("Split heavy tiles");
//  * each batch of 64 isects is gathered one 64-B render record per lane,
//    culled against the strip with the exact rectangle minimum of the
//    Gaussian's quadratic form (a record that cannot reach alpha >= 1/255 on
//    any pixel centre of the strip is dropped -- the per-pixel test would skip
//    it anyway), and compacted into a per-wave LDS queue with ballot/mbcnt;
//  * backward: work items of at most L isects of one tile (chunked at the
//    forward's saved state), two waves of 16x8 pixels (two per lane); the
//    per-lane partial gradients are combined across the 64 lanes with a
//    reduce-scatter (permlane32/16 swaps, then DPP mirrors and quad permutes),
//    the item's rows summed in LDS, and one float atomic per non-zero field of
//    a (Gaussian, item) row goes into a packed [G][S] gradient row.
#include "common.h"
#include "wave_ops.h"
#include "../../include/gsplat_hip.h"

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

namespace gs {
static uint64_t *g_timeline = nullptr;
static int64_t g_timeline_waves = 0;

namespace r16 {

constexpr int kTS = 16;
constexpr float kAlphaMin = 1.f / 255.f;
constexpr float kAlphaMax = 0.999f;
constexpr float kTMin = 1e-4f;

typedef float f2v __attribute__((ext_vector_type(2)));

// keep + (give permuted by DPP), for both components of a pair, as two
// v_add_f32_dpp.  (The compiler packs such adds into v_pk_add_f32, which
// takes no DPP operand, and then needs a v_mov_b32_dpp plus a zeroed old
// value per component.)  s_nop 1: the VALU-write -> DPP-read hazard of gfx9
// needs two wait states, which the compiler does not insert for inline asm;
// one nop covers both adds.
#define GS_ADD_DPP2(NAME, MOD)                                                             \
  GS_INLINE f2v NAME(f2v keep, f2v give) {                                                \
    float rx, ry;                                                                          \
    asm("s_nop 1\n\t"                                                                      \
        "v_add_f32_dpp %0, %2, %3 " MOD " row_mask:0xf bank_mask:0xf\n\t"                  \
        "v_add_f32_dpp %1, %4, %5 " MOD " row_mask:0xf bank_mask:0xf"                       \
        : "=&v"(rx), "=v"(ry)                                                              \
        : "v"(give.x), "v"(keep.x), "v"(give.y), "v"(keep.y));                             \
    return f2v{rx, ry};                                                                    \
  }
GS_ADD_DPP2(add_quad_10322, "quad_perm:[1,0,3,2]")
GS_ADD_DPP2(add_quad_23012, "quad_perm:[2,3,0,1]")
#undef GS_ADD_DPP2

GS_INLINE f2v swap32_sum2(f2v a, f2v b) {
  return f2v{swap32_sum(a.x, b.x), swap32_sum(a.y, b.y)};
}
GS_INLINE f2v swap16_sum2(f2v a, f2v b) {
  return f2v{swap16_sum(a.x, b.x), swap16_sum(a.y, b.y)};
}
template <int CTRL>
GS_INLINE f2v dpp2(f2v v) {
  return f2v{dpp<CTRL>(v.x), dpp<CTRL>(v.y)};
}
template <int M>
GS_INLINE f2v pick2(const f2v (&a)[M], int i) {
  return i < M ? a[i < M ? i : 0] : f2v{0.f, 0.f};
}

// reduce_scatter for N float2 fields (two records at once, .x / .y); the
// adds run as packed fp32, the lane exchanges per component.
template <int N>
GS_INLINE f2v reduce_scatter2(const f2v *v, int lane) {
  static_assert(N >= 1 && N <= 16, "reduce_scatter2: 1..16 fields");
  constexpr int N1 = (N + 1) / 2, N2 = (N1 + 1) / 2, N3 = (N2 + 1) / 2;
  f2v w[N1], x[N2], y[N3];
#pragma unroll
  for (int i = 0; i < N1; ++i)
    w[i] = swap32_sum2(v[2 * i], 2 * i + 1 < N ? v[2 * i + 1] : f2v{0.f, 0.f});
#pragma unroll
  for (int i = 0; i < N2; ++i) x[i] = swap16_sum2(w[2 * i], pick2(w, 2 * i + 1));
  (void)lane;
  // lane bits 3 and 2: bank-masked DPP adds per component (wave_ops.h add_b3
  // / add_b2), no per-lane selects
#pragma unroll
  for (int i = 0; i < N3; ++i) {
    const f2v lo = x[2 * i], hi = pick2(x, 2 * i + 1);
    y[i] = f2v{add_b3(lo.x, hi.x), add_b3(lo.y, hi.y)};
  }
  const f2v lo = y[0], hi = pick2(y, 1);
  f2v z = f2v{add_b2(lo.x, hi.x), add_b2(lo.y, hi.y)};
  z = add_quad_10322(z, z);
  z = add_quad_23012(z, z);
  return z;
}

// Render records: one 64-B row per Gaussian, [x, y, a, b, c, opacity,
// colour[D], pad] (D <= kRecMaxD), so the per-isect gather of a batch touches
// one 64-B sector per lane instead of four lines of four arrays
// (rasterize_to_pixels_fwd.py:93-145 loads the four arrays separately).
constexpr int kItemRun = 4;  // backward work items per XCD run (bwd2_kernel)
constexpr int kRecFloats = 16;
constexpr int kRecMaxD = kRecFloats - 6;

struct Args {
  int C, W, H, tw, th, n_tiles;
  int64_t n_isects;  // isect count, or with n_dev the capacity of the isect arrays
  const int64_t *n_dev;  // the isect count on the device (capacity mode) or null
  const float *means2d, *conics, *colors, *opacities, *backgrounds;
  const float *records;  // [G][kRecFloats] render records, or null (gather the arrays)
  uint32_t rec_bytes;    // bytes of the record table (< 2^31: buffer-load offsets)
  const uint8_t *masks;
  const int32_t *offsets, *flatten_ids;
  float *render_colors, *render_alphas;
  int32_t *last_ids;
  const float *v_render_colors, *v_render_alphas;
  float *packed;  // [G][S] gradient rows (backward)
  int S;
  // Chunk states (see "Chunked backward"): slot s = boundary isect index / L
  // holds T[256] then acc[D][256] of the tile's pixels before that isect.
  float *state;
  int L;  // chunk length in isects (multiple of 64); 0 = no chunking
  // backward work items (tile, chunk): n_items[0] full-length chunks at
  // items[0..), n_items[1] tails at items_tail[0..)
  const int2 *items, *items_tail;
  const int32_t *n_items;
  const int32_t *order;  // forward: tile of workgroup b (heaviest tiles first) or null
  const int32_t *n_whole;  // forward: the number of tiles in `order` (device), or null: all
  // forward, split heavy tiles (fwd_plan_kernel, "Split heavy tiles"):
  // fitems[b] = (tile, k), chunk k of a split tile, n_chunks of them (device).
  // prod: per boundary slot (b / L) the product of (1 - alpha) over the chunk
  // ending at b, pflag[4 * slot + wave] its ready flags; cout: per chunk (its
  // index in fitems), the chunk's end T, last id and colour sum [2 + D][256];
  // ctr[index of chunk 0] the tile's finished chunks (chunk START slots are
  // not unique: a tile's first chunk can share b / L with the previous
  // tile's last one).
  const int2 *fitems;
  const int32_t *n_chunks;
  float *prod, *cout;
  int32_t *pflag, *ctr;
  int SL;  // split tiles: isects per chunk (a multiple of L)
  const float *render_colors_in;  // backward: forward colours (for suffix sums)
  int dbg;  // debug flags (gsplat_hip_debug_set_flags): bit 0 = backward skips its
            // atomics, bit 1 = split chunks never wait for a published product
  uint64_t *timeline;  // debug: per-wave (start, end) s_memrealtime stamps or null
};

// Isect count and the end of tile t's isect range.  Capacity mode (n_dev
// non-null, the sync-free isect of a captured training step): the arrays
// hold n_isects slots, the count is read on the device.
GS_INLINE int64_t isect_count(const int64_t *n_dev, int64_t n) { return n_dev ? *n_dev : n; }
GS_INLINE int64_t tile_end(const int32_t *offsets, int t, int n_tiles, const int64_t *n_dev,
                           int64_t n) {
  return t == n_tiles - 1 ? isect_count(n_dev, n) : (int64_t)offsets[t + 1];
}
GS_INLINE int64_t tile_end(const Args &a, int t) {
  return tile_end(a.offsets, t, a.n_tiles, a.n_dev, a.n_isects);
}

// Debug timeline (gsplat_hip_debug_set_timeline): lane 0 of every wave stores
// its start/end stamps of the 100 MHz constant clock into its own slots.
GS_INLINE uint64_t tl_now(const Args &a) {
  return a.timeline ? __builtin_amdgcn_s_memrealtime() : 0;
}
GS_INLINE void tl_store(const Args &a, uint64_t t0, int lane) {
  if (a.timeline && lane == 0) {
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    a.timeline[2 * w] = t0;
    a.timeline[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

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
  // approximate reciprocals: an argmin off by an ulp moves q only to second
  // order, far inside the caller's margin
  const float rc = __builtin_amdgcn_rcpf(c), ra = __builtin_amdgcn_rcpf(a);
  // vertical edges: dx fixed, best dy = -b dx / c clamped
  for (int e = 0; e < 2; ++e) {
    const float dx = e ? dxh : dxl;
    const float dy = fminf(fmaxf(-b * dx * rc, dyl), dyh);
    m = fminf(m, q(dx, dy));
  }
  for (int e = 0; e < 2; ++e) {
    const float dy = e ? dyh : dyl;
    const float dx = fminf(fmaxf(-b * dy * ra, dxl), dxh);
    m = fminf(m, q(dx, dy));
  }
  return fmaxf(m, 0.f);
}

// Gaussian record as staged in LDS, one per kept isect, read back as float4s
// with one wave-uniform address:
//   [0] x  [1] y  [2..4] conic terms  [5] opacity  [6] isect index
//   forward:  [7 .. 7+D) colour              (D = 3: 40 B = b128 + b128 + b64)
//   backward: [7] Gaussian id, [8 .. 8+D) colour
// The forward stores the conic pre-scaled for exp2: (0.5 a, b, 0.5 c) * log2(e),
// so sigma * log2(e) is three FMAs and the exponential is a bare v_exp_f32.
template <int D, bool FWD>
struct Rec {
  static constexpr int C0 = FWD ? 7 : 8;  // first colour slot
  static constexpr int NF = ((C0 + D + 3) / 4) * 4;  // floats per record
  static constexpr int N4 = NF / 4;
};

constexpr float kLog2e = 1.4426950408889634f;

// Attributes of one gathered record (registers of one lane).
template <int D>
struct Attr {
  int32_t g;
  float2 xy;
  float3 con;
  float op;
  float col[D];
};

// Unconditional (the caller clamps the isect index into the tile's range and
// masks the lanes past it), so the loads stay in flight across the batch.
// The record is read with buffer_load_dwordx4 (a raw buffer over the table,
// a.rec_bytes long): as plain global loads the compiler merged them with the
// four-array path's loads into one set of instructions with selected
// addresses -- a dwordx2 and seven dword gathers per lane, each touching 64
// lines (TCP_TOTAL_CACHE_ACCESSES 89 M per forward launch at M2).  Three
// 16-B loads per lane do the same in a third of the L1 tag lookups.
template <int D, class A>
GS_INLINE void load_attr(const A &a, int32_t g, Attr<D> &at) {
  at.g = g;
  if constexpr (D <= kRecMaxD) {
    if (a.records) {  // wave-uniform
      constexpr int N4 = (6 + D + 3) / 4;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float *>(a.records), (short)0, (int)a.rec_bytes, 0x00020000);
      const uint32_t base = (uint32_t)g * (uint32_t)(kRecFloats * 4);
      float v[4 * N4];
#pragma unroll
      for (int q = 0; q < N4; ++q) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16u * q, 0, 0);
        v[4 * q] = __uint_as_float(x[0]); v[4 * q + 1] = __uint_as_float(x[1]);
        v[4 * q + 2] = __uint_as_float(x[2]); v[4 * q + 3] = __uint_as_float(x[3]);
      }
      at.xy = make_float2(v[0], v[1]);
      at.con = make_float3(v[2], v[3], v[4]);
      at.op = v[5];
#pragma unroll
      for (int d = 0; d < D; ++d) at.col[d] = v[6 + d];
      return;
    }
  }
  at.xy = *reinterpret_cast<const float2 *>(a.means2d + 2 * (int64_t)g);
  const float *cn = a.conics + 3 * (int64_t)g;
  at.con = make_float3(cn[0], cn[1], cn[2]);
  at.op = a.opacities[g];
  const float *cl = a.colors + (int64_t)g * D;
#pragma unroll
  for (int d = 0; d < D; ++d) at.col[d] = cl[d];
}

// Strip culling: keep iff some pixel centre of [x0,x1]x[y0,y1] can reach
// opacity * exp(-sigma) >= 1/255 (margin 0.02 absorbs float rounding of the
// per-pixel sigma and the exponential).
template <int D>
GS_INLINE bool keep_attr(const Attr<D> &at, float x0, float x1, float y0, float y1) {
  if (!(at.op >= kAlphaMin)) return false;  // alpha <= opacity < 1/255 everywhere
  const float ms = rect_min_sigma(at.xy.x, at.xy.y, at.con.x, at.con.y, at.con.z, x0, x1, y0, y1);
  return ms <= 0.69314718f * __builtin_amdgcn_logf(255.f * at.op) + 0.02f;
}

template <int D, bool FWD>
GS_INLINE void stage_attr(float4 *slot, const Attr<D> &at, int32_t idx) {
  using R = Rec<D, FWD>;
  const int32_t g = at.g;
  float r[R::NF];
  r[0] = at.xy.x;
  r[1] = at.xy.y;
  if (FWD) {
    r[2] = 0.5f * kLog2e * at.con.x;
    r[3] = kLog2e * at.con.y;
    r[4] = 0.5f * kLog2e * at.con.z;
  } else {
    r[2] = at.con.x;
    r[3] = at.con.y;
    r[4] = at.con.z;
  }
  r[5] = at.op;
  r[6] = __int_as_float(idx);
  if (!FWD) r[7] = __int_as_float(g);
#pragma unroll
  for (int d = 0; d < D; ++d) r[R::C0 + d] = at.col[d];
#pragma unroll
  for (int d = R::C0 + D; d < R::NF; ++d) r[d] = 0.f;
#pragma unroll
  for (int q = 0; q < R::N4; ++q) slot[q] = make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
}

// WIDE: whole float4s -- the empty asm keeps every component live so the
// compiler cannot narrow a read to ds_read_b96 (8 LDS cycles per wave against
// 4 for ds_read_b128, MI355X_MICROARCH.md "LDS").
template <int D, bool FWD, bool WIDE>
GS_INLINE void read_rec(const float4 *slot, float (&r)[Rec<D, FWD>::NF]) {
  constexpr int N4 = Rec<D, FWD>::N4;
  float4 v[N4];
#pragma unroll
  for (int q = 0; q < N4; ++q) v[q] = slot[q];
#pragma unroll
  for (int q = 0; q < N4; ++q) {
    if (WIDE) asm volatile("" ::"v"(v[q].x), "v"(v[q].y), "v"(v[q].z), "v"(v[q].w));
    r[4 * q] = v[q].x; r[4 * q + 1] = v[q].y; r[4 * q + 2] = v[q].z; r[4 * q + 3] = v[q].w;
  }
}


// Geometry of one wave: 4 waves share a 16x16 tile, each owning a 16x4
// strip; lane l owns pixel column (l & 15), row strip_y0 + (l >> 4).
struct WaveGeom {
  int tile, c, px, py;
  float x0, x1, y0, y1;  // strip rectangle of pixel centres

  GS_INLINE WaveGeom(const Args &a, int lane, int tile_) {
    const int w = threadIdx.x >> 6;
    tile = tile_;
    const int ntile = a.tw * a.th;
    c = tile / ntile;
    const int rem = tile - c * ntile;
    const int ty = rem / a.tw, tx = rem - ty * a.tw;
    px = tx * kTS + (lane & 15);
    py = ty * kTS + 4 * w + (lane >> 4);
    x0 = tx * kTS + 0.5f;
    x1 = x0 + (kTS - 1);
    y0 = ty * kTS + 4 * w + 0.5f;
    y1 = y0 + 3.f;
  }
};

// Forward.  The gather of batch b+1 (its attributes) and the flatten ids of
// batch b+2 are in flight while batch b is composited, so a long tile pays
// the two dependent global-load latencies once, not once per 64 isects.
// Forward records are staged in PAIRS, field-interleaved: the pair holding
// kept records 2p and 2p+1 stores every field f as the float2 (f_2p, f_2p+1),
// so one ds_read_b128 yields two fields of both records in register pairs and
// the per-record algebra runs as packed fp32 (v_pk_fma/mul/add_f32: two lanes'
// worth per instruction; a wave64 v_fma_f32 costs 4 cycles per SIMD on
// MI355X, a v_pk_fma_f32 about 4.7 for twice the work -- tools/valu_bench.hip).
// Fields: x, y, (a, b, c) pre-scaled for exp2, opacity, smax = log2(255 op)
// (hit iff 0 <= s2 <= smax, one unsigned compare), isect index, colour[D].
template <int D>
struct FwdPair {
  static constexpr int NFP = 8 + D;                  // fields per record
  static constexpr int N4 = (2 * NFP + 3) / 4;       // float4s per pair
};

template <int D>
GS_INLINE void stage_fwd_pair(float4 *st, int slot, const Attr<D> &at, int32_t idx) {
  float *w = reinterpret_cast<float *>(st + (slot >> 1) * FwdPair<D>::N4) + (slot & 1);
  w[0] = at.xy.x;
  w[2] = at.xy.y;
  w[4] = 0.5f * kLog2e * at.con.x;
  w[6] = kLog2e * at.con.y;
  w[8] = 0.5f * kLog2e * at.con.z;
  w[10] = at.op;
  w[12] = __builtin_amdgcn_logf(255.f * at.op);  // log2
  w[14] = __int_as_float(idx);
#pragma unroll
  for (int d = 0; d < D; ++d) w[16 + 2 * d] = at.col[d];
}

// A pad slot (the odd slot of a final half-filled pair, or a whole padding
// pair): x = NaN never hits, and opacity = colour = 0 add nothing.
template <int D>
GS_INLINE void stage_fwd_pad(float4 *st, int slot) {
  float *w = reinterpret_cast<float *>(st + (slot >> 1) * FwdPair<D>::N4) + (slot & 1);
  w[0] = __int_as_float(0x7fc00000);
#pragma unroll
  for (int f = 1; f < FwdPair<D>::NFP; ++f) w[2 * f] = 0.f;
}

// Backward records, staged in pairs like the forward's.  Fields: x, y,
// (a, b, c) * log2(e) / 2 (so that s2 = dx gx + dy gy with gx = A dx + B dy,
// gy = B dx + C dy, and d s2 / d(dx, dy) = 2 (gx, gy)), opacity, smax, isect
// index, Gaussian id, colour[D].
template <int D>
struct BwdPair {
  static constexpr int NFP = 9 + D;
  static constexpr int N4 = (2 * NFP + 3) / 4;
};

template <int D>
GS_INLINE void stage_bwd_pair(float4 *st, int slot, const Attr<D> &at, int32_t idx) {
  float *w = reinterpret_cast<float *>(st + (slot >> 1) * BwdPair<D>::N4) + (slot & 1);
  w[0] = at.xy.x;
  w[2] = at.xy.y;
  w[4] = 0.5f * kLog2e * at.con.x;
  w[6] = 0.5f * kLog2e * at.con.y;
  w[8] = 0.5f * kLog2e * at.con.z;
  w[10] = at.op;
  w[12] = __builtin_amdgcn_logf(255.f * at.op);
  w[14] = __int_as_float(idx);
  w[16] = __int_as_float(at.g);
#pragma unroll
  for (int d = 0; d < D; ++d) w[18 + 2 * d] = at.col[d];
}

template <int D>
GS_INLINE void stage_bwd_pad(float4 *st, int slot) {
  float *w = reinterpret_cast<float *>(st + (slot >> 1) * BwdPair<D>::N4) + (slot & 1);
  w[0] = __int_as_float(0x7fc00000);  // NaN: never valid
  w[12] = 0.f;
  w[16] = __int_as_float(-1);  // no gradient row
#pragma unroll
  for (int f = 1; f < BwdPair<D>::NFP; ++f)
    if (f != 6 && f != 8) w[2 * f] = 0.f;
}

// One pair per iteration of the composite loop (80 VGPRs, 5-6 waves per
// SIMD).  Unrolling 2 or 4 pairs (their LDS reads together, the next pair's
// alpha math under this pair's blend chain) measured 0.193 / 0.23 ms against
// 0.184 at M2: the extra VGPRs cost more waves than the overlap gained.
// Gather depth one batch: the attributes of batch b+1 are gathered while
// batch b composites (two register buffers).  Depth 0 (only the flatten ids
// ahead, two more waves) measured 0.198 / 0.686 ms at M2 / M3 against 0.184 /
// 0.590, depth 2 (three buffers) no better than 1.
// ---- Split heavy tiles.  A tile with more isects than the threshold is
// rendered as chunks of SL isects by separate workgroups of the SAME forward
// launch (fwd_kernel<SPLIT>): the chunks are workgroups 0 .. n_chunks - 1,
// dispatched before the whole tiles that follow them, a tile's chunks at
// increasing block indices.  Chunk k needs the transmittance entering it, the
// product of the earlier chunks' (1 - alpha) products: every chunk but the
// last first computes its own product (chunk_product) and publishes it per
// wave, then takes the earlier chunks' products, composites from their product
// and publishes its end T, last id and colour; the tile's last chunk to finish
// combines them into the pixels.  Hand-offs (cdna_hip_programming.md
// Guideline 16, form R1): every published word is stored write-through (sc1,
// a relaxed agent-scope atomic store) and drained (s_waitcnt vmcnt(0)) by the
// storing wave before its relaxed agent-scope flag store or counter add, so
// no release fence -- an agent release is a buffer_wbl2, a write-back of the
// XCD's whole L2, and the forward keeps much of its output dirty there (one
// per published product and per chunk cost M3's forward 0.494 -> 0.615 ms);
// the consumer polls relaxed, runs ONE agent-scope acquire (this CU's L1)
// after ALL its polls have matched (or after the counter add that made it
// last), and reads the words with sc1 loads.  A chunk waits only for chunks
// at lower block indices, dispatched before it; the wait is bounded anyway --
// on timeout the chunk computes the missing products itself (same code, same
// value), so no schedule can hang it.
GS_INLINE void store_sc1(float *p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
GS_INLINE float load_sc1(const float *p) {
  return __hip_atomic_load(const_cast<float *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
GS_INLINE void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// producer side, after the published (sc1) stores, before the flag / counter
GS_INLINE void release_published() { drain_stores(); }
// consumer side, after the poll matched / the counter add returned
GS_INLINE void acquire_published() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  drain_stores();
}
// 2048 polls of s_sleep 8 (~0.2 us each) plus the load round trips: about
// 0.4-1 ms of waiting before the fallback computes the product itself
constexpr int kSpinPolls = 2048;
// the poll only; the caller runs ONE acquire after all its polls matched
GS_INLINE bool wait_flag(const int32_t *f) {
  for (int i = 0; i < kSpinPolls; ++i) {
    if (__hip_atomic_load(const_cast<int32_t *>(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return true;
    __builtin_amdgcn_s_sleep(8);
  }
  return false;
}

// The product over the records of [start, end) of (1 - alpha) where a record
// hits the lane's pixel, from 1 and without the termination rule (a product
// at or below 1e-4 is kept as 0: the pixel is finished).  Same culling, alpha
// and fma as the compositing.  The wave's strip; uses its LDS stage buffer.
template <int D>
GS_INLINE float chunk_product(const Args &a, const WaveGeom &geo, int64_t start, int64_t end,
                              float4 *st, int lane, float fx, float fy) {
  constexpr int N4 = FwdPair<D>::N4;
  float Pp = 1.f;
  auto id_at = [&](int64_t b0) -> int32_t { return a.flatten_ids[min(b0 + lane, end - 1)]; };
  int32_t g_n = id_at(start);
  for (int64_t b0 = start; b0 < end; b0 += 64) {
    if (__ballot(Pp > 0.f) == 0) break;
    Attr<D> A;
    load_attr<D>(a, g_n, A);
    g_n = id_at(b0 + 64);
    const bool keep = (b0 + lane < end) && keep_attr<D>(A, geo.x0, geo.x1, geo.y0, geo.y1);
    const uint64_t m = __ballot(keep);
    const int cnt = __popcll(m);
    if (keep) stage_fwd_pair<D>(st, ballot_slot(m), A, (int32_t)(b0 + lane));
    if ((cnt & 1) && lane == 0) stage_fwd_pad<D>(st, cnt);
    wave_sync_lds();
    for (int p = 0; p < (cnt + 1) >> 1; ++p) {
      f2v f[2 * N4];
      float4 v[N4];
#pragma unroll
      for (int i = 0; i < N4; ++i) v[i] = st[p * N4 + i];
#pragma unroll
      for (int i = 0; i < N4; ++i) {
        asm volatile("" ::"v"(v[i].x), "v"(v[i].y), "v"(v[i].z), "v"(v[i].w));
        f[2 * i] = f2v{v[i].x, v[i].y};
        f[2 * i + 1] = f2v{v[i].z, v[i].w};
      }
      const f2v dx = f[0] - fx, dy = f[1] - fy;
      const f2v s2 = dx * (f[2] * dx + f[3] * dy) + f[4] * dy * dy;
      f2v al = f[5] * f2v{__builtin_amdgcn_exp2f(-s2.x), __builtin_amdgcn_exp2f(-s2.y)};
      al.x = fminf(al.x, kAlphaMax);
      al.y = fminf(al.y, kAlphaMax);
      const bool h0 = __float_as_uint(s2.x) <= __float_as_uint(f[6].x);
      const bool h1 = __float_as_uint(s2.y) <= __float_as_uint(f[6].y);
      float n0 = h0 ? __builtin_fmaf(-Pp, al.x, Pp) : Pp;
      n0 = n0 > kTMin ? n0 : 0.f;
      float n1 = h1 ? __builtin_fmaf(-n0, al.y, n0) : n0;
      Pp = n1 > kTMin ? n1 : 0.f;
    }
    wave_sync_lds();
  }
  return Pp;
}

// One work item of the forward: SPLIT = chunk `item` of the split tiles'
// list, else the whole tile `item` of the dispatch order (past the plan's
// count of whole tiles: nothing).
template <int D, bool SPLIT>
GS_INLINE void fwd_item(const Args &a, float4 *st, int item) {
  using P = FwdPair<D>;
  constexpr int N4 = P::N4;
  const int lane = threadIdx.x & 63;
  const uint64_t t_start = SPLIT ? 0 : tl_now(a);
  int tile_, kc = -1;  // kc >= 0: chunk kc of a split tile
  if constexpr (SPLIT) {
    const int2 it = a.fitems[item];
    tile_ = it.x;
    kc = it.y;
  } else {
    if (a.n_whole && item >= a.n_whole[0]) return;  // the split tiles' slots
    tile_ = a.order ? a.order[item] : item;
    if (tile_ < 0) return;  // an empty slot of the XCD-grouped order
  }
  const WaveGeom geo(a, lane, tile_);
  const int tile = geo.tile, c = geo.c;
  const bool inside = geo.px < a.W && geo.py < a.H;
  const float fx = (float)geo.px + 0.5f, fy = (float)geo.py + 0.5f;
  // isect indices fit 32 bits (the offsets are int32); wave-uniform, kept
  // in SGPRs
  const int tstart = __builtin_amdgcn_readfirstlane(a.offsets[tile]);
  const int tend = __builtin_amdgcn_readfirstlane((int)tile_end(a, tile));
  const int start = kc >= 0 ? tstart + kc * a.SL : tstart;
  const int end = kc >= 0 ? min(tend, start + a.SL) : tend;
  const bool skip_tile = a.masks && a.masks[tile];

  // colour accumulated from even (.x) and odd (.y) records of each pair in the
  // current chunk; tot: the chunks before it (see "chunk state" below)
  f2v acc[D];
  float tot[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    acc[d] = f2v{0.f, 0.f};
    tot[d] = 0.f;
  }
  int32_t last = 0;
  // A terminated (or outside) pixel is encoded by a negative T: |T| is its
  // final transmittance.
  float T = (!inside || skip_tile) ? -1.f : 1.f;
  const int pix_in_tile = (threadIdx.x >> 6) * 64 + lane;  // row-major
  const int wv = threadIdx.x >> 6;
  // split tiles (see "Split heavy tiles"): product passes (this
  // chunk's own, then any earlier one not published in time), then the
  // transmittance entering the chunk
  const int nch = SPLIT ? (int)((tend - tstart + a.SL - 1) / a.SL) : 0;
  if (SPLIT && nch > 1 && !skip_tile) {
    float Tin = 1.f;
    if (kc < nch - 1) {  // this chunk's own product, published first
      const float Pp = chunk_product<D>(a, geo, start, end, st, lane, fx, fy);
      const int64_t sl = end / a.L;
      store_sc1(a.prod + sl * (kTS * kTS) + pix_in_tile, Pp);
      release_published();
      if (lane == 0)
        __hip_atomic_store(a.pflag + 4 * sl + wv, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the earlier chunks' products: poll their flags in order, ONE acquire for
    // the run that matched, their products; the rest (timed out) computed here
    int jm = 0;
    if (!(a.dbg & 2))
      for (; jm < kc; ++jm)
        if (!wait_flag(a.pflag + 4 * ((tstart + (jm + 1) * a.SL) / a.L) + wv)) break;
    if (jm > 0) {
      acquire_published();
      for (int j = 0; j < jm; ++j)
        Tin *= load_sc1(a.prod + ((tstart + (j + 1) * a.SL) / a.L) * (kTS * kTS) + pix_in_tile);
    }
    for (int j = jm; j < kc; ++j) {
      const int ps = tstart + j * a.SL;
      Tin *= chunk_product<D>(a, geo, ps, ps + a.SL, st, lane, fx, fy);
    }
    // at or below 1e-4 the pixel terminated in an earlier chunk (every
    // blended factor kept it above): -Tin marks it finished with about that
    // transmittance
    if (kc > 0 && inside) T = Tin > kTMin ? Tin : -fmaxf(Tin, 1e-30f);
  }
  const int rs = start, re = end;

  if (!skip_tile && rs < re) {
    // flatten id of lane `lane` of the batch at b0, clamped into the range
    auto id_at = [&](int b0) -> int32_t {
      return a.flatten_ids[min(b0 + lane, re - 1)];
    };
    bool done = false;
    // one record of a pair: sequential in T
    auto blend = [&](float s2, float smax, float al, float idx) -> float {
      const bool hit = __float_as_uint(s2) <= __float_as_uint(smax);  // 0 <= s2 <= smax
      const float nT = __builtin_fmaf(-T, al, T);  // T (1 - alpha)
      const bool gt = nT > kTMin;
      const bool ok = hit & gt;
      // plain selects (no control flow): blended -> nT; hit but T would drop
      // to <= 1e-4 -> exclusive stop, -|T| marks the pixel (and keeps dead
      // pixels dead); otherwise unchanged
      const float Tsel = ok ? nT : T;
      const float vis = T - Tsel;  // alpha * T when blended, else 0
      T = (hit & !gt) ? -fabsf(T) : Tsel;
      last = ok ? __float_as_int(idx) : last;
      return vis;
    };
    // composite one staged batch pair by pair, checking every 8 pairs
    // whether the strip is alive
    auto composite = [&](int cnt) {
      const int np = (cnt + 1) >> 1;
      for (int pb = 0; pb < np; pb += 8) {
        const int pe = min(np, pb + 8);
        for (int p = pb; p < pe; ++p) {
          f2v f[2 * N4];
          float4 v[N4];
#pragma unroll
          for (int i = 0; i < N4; ++i) v[i] = st[p * N4 + i];
#pragma unroll
          for (int i = 0; i < N4; ++i) {
            // keep every field live: no load may sink into a select's branch
            asm volatile("" ::"v"(v[i].x), "v"(v[i].y), "v"(v[i].z), "v"(v[i].w));
            f[2 * i] = f2v{v[i].x, v[i].y};
            f[2 * i + 1] = f2v{v[i].z, v[i].w};
          }
          const f2v dx = f[0] - fx, dy = f[1] - fy;
          const f2v s2 = dx * (f[2] * dx + f[3] * dy) + f[4] * dy * dy;  // sigma * log2(e)
          f2v al = f[5] * f2v{__builtin_amdgcn_exp2f(-s2.x), __builtin_amdgcn_exp2f(-s2.y)};
          al.x = fminf(al.x, kAlphaMax);
          al.y = fminf(al.y, kAlphaMax);
          const float v0 = blend(s2.x, f[6].x, al.x, f[7].x);
          const float v1 = blend(s2.y, f[6].y, al.y, f[7].y);
          const f2v vis = f2v{v0, v1};
#pragma unroll
          for (int d = 0; d < D; ++d) acc[d] = __builtin_elementwise_fma(vis, f[8 + d], acc[d]);
        }
        if (__ballot(T > 0.f) == 0) {
          done = true;
          return;
        }
      }
    };
    auto stage = [&](const Attr<D> &at, int b0) -> int {
      const bool keep = (b0 + lane < re) && keep_attr<D>(at, geo.x0, geo.x1, geo.y0, geo.y1);
      const uint64_t m = __ballot(keep);
      const int cnt = __popcll(m);
      if (keep) stage_fwd_pair<D>(st, ballot_slot(m), at, (int32_t)(b0 + lane));
      // the odd slot of a final half-filled pair
      if ((cnt & 1) && lane == 0) stage_fwd_pad<D>(st, cnt);
      wave_sync_lds();
      return cnt;
    };
    // Chunk state for the chunked backward, one slot per chunk boundary
    // b = start + m*L (m >= 1), slot b / L: T[256] = the pixel's transmittance
    // before isect b, S[D][256] = the colour the chunk starting at b adds.
    // Chunk-local sums keep the backward's suffix sums (sum of S over the
    // later chunks) as accurate as its own back-to-front accumulation; a
    // difference of running totals would cancel catastrophically.  A pixel's
    // slot b is written only while it is alive at b: the backward reads slot
    // b of a pixel only when b <= its last id (bwd2_kernel), and a pixel that
    // blends record last_id was alive at every boundary up to it.  Boundaries
    // past the strip's end (all pixels finished) are not written at all.
    const int L = a.L;
    auto slot = [&](int bidx) { return a.state + (int64_t)(bidx / L) * (kTS * kTS * (1 + D)); };
    int cur_b = start;  // start of the chunk being accumulated
    bool live_b = T > 0.f;  // the pixel was alive at cur_b
    auto close_chunk = [&]() {  // fold acc into tot; store S of the chunk at cur_b
      float *sl = slot(cur_b);
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const float cs = acc[d].x + acc[d].y;
        if (cur_b > tstart && live_b && !(a.dbg & 32)) sl[(1 + d) * kTS * kTS + pix_in_tile] = cs;
        tot[d] += cs;
        acc[d] = f2v{0.f, 0.f};
      }
    };
    auto save_state = [&](int bidx) {  // reached boundary bidx
      close_chunk();
      cur_b = bidx;
      live_b = T > 0.f;
      if (live_b && !(a.dbg & 32)) slot(bidx)[pix_in_tile] = T;
    };
    // a chunk of a split tile writes the state of the boundaries inside it
    // and the colour it adds at its own start boundary
    const bool chunked = a.state && L > 0 && (end - start > L || kc > 0);
    int b0 = rs;
    // two attribute buffers in alternation: while batch b is composited from
    // one, the other receives batch b+1, and the ids of batch b+2 load
    Attr<D> A, B;
    load_attr<D>(a, id_at(rs), A);
    int32_t g_n = id_at(rs + 64);
    while (b0 < re) {
      if (__ballot(T > 0.f) == 0) break;
      if (chunked && b0 > start && (b0 - start) % L == 0) save_state(b0);
      load_attr<D>(a, g_n, B);
      g_n = id_at(b0 + 128);
      composite(stage(A, b0));
      wave_sync_lds();
      b0 += 64;
      if (done || b0 >= re) break;
      if (chunked && (b0 - start) % L == 0) save_state(b0);
      load_attr<D>(a, g_n, A);
      g_n = id_at(b0 + 128);
      composite(stage(B, b0));
      wave_sync_lds();
      b0 += 64;
      if (done) break;
    }
    if (chunked) close_chunk();
  }

#pragma unroll
  for (int d = 0; d < D; ++d) tot[d] += acc[d].x + acc[d].y;

  if constexpr (SPLIT) {
    // chunk of a split tile: its end T, last id and colour for the combine;
    // and its end T at the next boundary of the backward's chunk state (the
    // running T the unsplit forward stores there; the loop above wrote the
    // boundaries inside the chunk and the colours)
    const int64_t sz = kTS * kTS;
    const int cid = item;
    float *co = a.cout + (int64_t)cid * sz * (2 + D);
    store_sc1(co + pix_in_tile, T);
    store_sc1(co + sz + pix_in_tile, __int_as_float(last));
#pragma unroll
    for (int d = 0; d < D; ++d) store_sc1(co + (2 + d) * sz + pix_in_tile, tot[d]);
    if (end < tend && a.state) a.state[(end / a.L) * sz * (1 + D) + pix_in_tile] = T;
    drain_stores();
    __syncthreads();
    __shared__ int s_last;
    if (threadIdx.x == 0) {
      s_last = __hip_atomic_fetch_add(a.ctr + (cid - kc), 1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) == nch - 1;
      if (s_last) acquire_published();
    }
    __syncthreads();
    if (s_last && inside) {
      // the tile's last chunk to finish: per pixel the sum of the chunks'
      // colours, the final T (the end T of the chunk where the pixel
      // terminated -- the first negative -- else of the last chunk) and the
      // largest last id
      float col[D];
#pragma unroll
      for (int d = 0; d < D; ++d) col[d] = 0.f;
      int32_t lst = 0;
      float Tf = 1.f;
      bool fin = false;
      for (int k = 0; k < nch; ++k) {
        const float *ck = a.cout + (int64_t)(cid - kc + k) * sz * (2 + D);
        const float Te = load_sc1(ck + pix_in_tile);
        lst = max(lst, __float_as_int(load_sc1(ck + sz + pix_in_tile)));
#pragma unroll
        for (int d = 0; d < D; ++d) col[d] += load_sc1(ck + (2 + d) * sz + pix_in_tile);
        if (!fin) {
          Tf = fabsf(Te);
          fin = Te < 0.f;
        }
      }
      const int64_t pix = ((int64_t)c * a.H + geo.py) * a.W + geo.px;
      float *oc = a.render_colors + pix * D;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const float bg = a.backgrounds ? a.backgrounds[c * D + d] : 0.f;
        oc[d] = col[d] + Tf * bg;
      }
      a.render_alphas[pix] = 1.f - Tf;
      a.last_ids[pix] = lst;
    }
  } else if (inside) {
    const int64_t pix = ((int64_t)c * a.H + geo.py) * a.W + geo.px;
    float *oc = a.render_colors + pix * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float bg = a.backgrounds ? a.backgrounds[c * D + d] : 0.f;
      oc[d] = tot[d] + fabsf(T) * bg;
    }
    a.render_alphas[pix] = 1.f - fabsf(T);
    a.last_ids[pix] = last;
  }
  if (!SPLIT) tl_store(a, t_start, lane);
}

// SPLIT: the split tiles' chunks (workgroups 0 .. n_chunks - 1, dispatched
// first: they are the longest work) and the other tiles in one launch, so the
// chunks overlap the whole tiles; else the whole tiles only (the split path's
// code costs registers: 80 -> 95 VGPRs, 6 -> 5 waves per SIMD at D = 3).
template <int D, bool SPLIT = false>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(!SPLIT && D <= 3 ? 6 : 5))) fwd_kernel(Args a) {
  __shared__ float4 stage_all[4][32 * FwdPair<D>::N4];
  float4 *st = stage_all[threadIdx.x >> 6];
  if constexpr (SPLIT) {
    const int nc = a.n_chunks[0];
    if ((int)blockIdx.x < nc) {
      fwd_item<D, true>(a, st, (int)blockIdx.x);
    } else {
      // the whole tiles: runs of kItemRun consecutive order entries (same
      // bucket, mostly neighbouring tiles) on one XCD, dealt round-robin
      // (workgroup b runs on XCD b % 8; the runs keep their XCD whatever nc)
      int j = (int)blockIdx.x - nc;
      if (!(a.dbg & 16)) {
        const int x = j & 7, kk = j >> 3;
        j = ((kk / kItemRun) * 8 + x) * kItemRun + kk % kItemRun;
      }
      fwd_item<D, false>(a, st, j);
    }
  } else {
    fwd_item<D, false>(a, st, (int)blockIdx.x);
  }
}

// Backward, PX pixels per lane (the default PX = 2): a wave owns a 16 x 4PX band
// of the tile, lane l the pixels (l & 15, 4PX w + 4q + (l >> 4)), q < PX, and
// the 4/PX waves of a workgroup cover the tile.  Each record's gradient
// terms of the PX pixels are summed in-lane before the one reduce-scatter and
// the atomics, which divides the cross-lane work and the LDS reads per pixel
// by PX; the price is coarser culling (16 x 4PX rectangles instead of 16x4)
// and fewer waves per SIMD.  Same arithmetic per pixel as bwd_kernel.
template <int PX>
struct BwdOcc {  // waves per SIMD that fit the VGPRs without spills
  static constexpr int W = PX == 2 ? 4 : 3;
};

// PFB: gather the next batch's records while compositing this one (one
// batch of latency hidden per wave; costs the record's registers).
template <int D, bool ABS, int PX, bool PFB = false>
__global__ void __launch_bounds__(256 / PX)
__attribute__((amdgpu_waves_per_eu(BwdOcc<PX>::W))) bwd2_kernel(Args a) {
  using P = BwdPair<D>;
  constexpr int N4 = P::N4;
  constexpr int F = D + 6 + (ABS ? 2 : 0);
  constexpr int NV = (F + 15) / 16;
  __shared__ float4 stage_all[4 / PX][32 * N4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float4 *st = stage_all[w];
  const uint64_t t_start = tl_now(a);
  int tile = blockIdx.x, k = 0;
  if (a.items) {
    const int nf = a.n_items[0];
    int b = blockIdx.x;
    if (!(a.dbg & 16)) {
      // XCD-aware: runs of kItemRun consecutive items (a tile's chunks, or
      // neighbouring tiles of a row, which share Gaussians) on one XCD
      // (workgroup b runs on XCD b % 8), the runs dealt round-robin so the
      // list order -- full chunks first -- is kept across the chip
      const int x = b & 7, kk = b >> 3;
      b = ((kk / kItemRun) * 8 + x) * kItemRun + kk % kItemRun;
    }
    if (b >= nf && b - nf >= a.n_items[1]) return;
    const int2 it = b < nf ? a.items[b] : a.items_tail[b - nf];
    tile = it.x;
    k = it.y;
  }
  const int ntile = a.tw * a.th;
  const int c = tile / ntile;
  const int rem = tile - c * ntile;
  const int ty = rem / a.tw, tx = rem - ty * a.tw;
  const int px = tx * kTS + (lane & 15);
  const int py0 = ty * kTS + 4 * PX * w + (lane >> 4);
  const float rx0 = tx * kTS + 0.5f, rx1 = rx0 + (kTS - 1);
  const float ry0 = ty * kTS + 4 * PX * w + 0.5f, ry1 = ry0 + (4 * PX - 1);
  if (a.masks && a.masks[tile]) return;
  // isect indices fit 32 bits (the offsets are int32); wave-uniform
  const int tstart = __builtin_amdgcn_readfirstlane(a.offsets[tile]);
  const int tend = __builtin_amdgcn_readfirstlane((int)tile_end(a, tile));
  const int start = a.items ? tstart + k * a.L : tstart;
  const int cend = a.items ? min(tend, start + a.L) : tend;

  const float fx = (float)px + 0.5f;
  float fy[PX], T[PX], rD[PX], bgt[PX], TfDra[PX], Drc[PX][D];
  int32_t mylast[PX];
#pragma unroll
  for (int q = 0; q < PX; ++q) {
    const int py = py0 + 4 * q;
    fy[q] = (float)py + 0.5f;
    T[q] = 1.f, rD[q] = 0.f, bgt[q] = 0.f, TfDra[q] = 0.f, mylast[q] = -1;
#pragma unroll
    for (int d = 0; d < D; ++d) Drc[q][d] = 0.f;
    if (px < a.W && py < a.H) {
      const int64_t pix = ((int64_t)c * a.H + py) * a.W + px;
      const float Tf = 1.f - a.render_alphas[pix];
      const float Dra = a.v_render_alphas ? a.v_render_alphas[pix] : 0.f;
      mylast[q] = a.last_ids[pix];
#pragma unroll
      for (int d = 0; d < D; ++d) Drc[q][d] = a.v_render_colors[pix * D + d];
      if (a.backgrounds) {
        float bgv = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) bgv += a.backgrounds[c * D + d] * Drc[q][d];
        bgt[q] = bgv * Tf;
      }
      TfDra[q] = Tf * Dra;
      T[q] = Tf;
      if (cend < tend && mylast[q] >= cend) {
        // chunk followed by others in which the pixel still blends: the
        // forward's state at the boundary cend, suffix sums up to its last id
        // (as in bwd_kernel)
        const int p = 64 * PX * w + 64 * q + lane;  // row-major pixel of the tile
        const int64_t per = (int64_t)(kTS * kTS * (1 + D));
        T[q] = fabsf(a.state[(cend / a.L) * per + p]);
        // the later chunks' colours, four boundaries' loads in flight at a
        // time (one round trip per four chunks of a long tile, not per
        // chunk); summed in the same order as one at a time
        float s = 0.f;
        for (int b0 = cend; b0 <= mylast[q]; b0 += 4 * a.L) {
          float v[4][D];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int bi = b0 + u * a.L;
            const float *sl = a.state + (min(bi, mylast[q]) / a.L) * per;
#pragma unroll
            for (int d = 0; d < D; ++d) v[u][d] = sl[(1 + d) * kTS * kTS + p];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (b0 + u * a.L > mylast[q]) break;
#pragma unroll
            for (int d = 0; d < D; ++d) s += v[u][d] * Drc[q][d];
          }
        }
        rD[q] = s;
      }
    }
  }
  int32_t lmax = mylast[0];
#pragma unroll
  for (int q = 1; q < PX; ++q) lmax = max(lmax, mylast[q]);
#pragma unroll
  for (int msk = 32; msk >= 1; msk >>= 1) lmax = max(lmax, __shfl_xor(lmax, msk, 64));
  const int end = min(cend, lmax + 1);

  if (start < end) {
    auto id_at = [&](int b1) -> int32_t {
      return a.flatten_ids[max(b1 - 64 + lane, start)];
    };
    auto stage = [&](const Attr<D> &at, int b1) -> int {
      const int j = b1 - 64 + lane;
      const bool keep = (j >= start) && keep_attr<D>(at, rx0, rx1, ry0, ry1);
      const uint64_t m = __ballot(keep);
      const int cnt = __popcll(m);
      if (keep) stage_bwd_pair<D>(st, ballot_slot(m), at, (int32_t)j);
      if ((cnt & 1) && lane == 0) stage_bwd_pad<D>(st, cnt);
      wave_sync_lds();
      return cnt;
    };
    const int lf = rs_field(lane);
    auto field_scale = [&](int f) -> float {
      constexpr float m2 = -2.f / kLog2e;
      if (f < D + 1) return 1.f;
      if (f < D + 3) return m2;
      if (f == D + 3 || f == D + 5) return -0.5f;
      if (f == D + 4) return -1.f;
      return -m2;
    };
    auto grad_seq = [&](int q, bool valid, bool unclamped, float al, float ra, float gD, float &wt,
                        float &Da) {
      T[q] = valid ? T[q] * ra : T[q];
      wt = valid ? al * T[q] : 0.f;
      rD[q] += gD * wt;
      const float Da_raw = ra * (TfDra[q] + T[q] * gD - rD[q] - bgt[q]);
      Da = (valid & unclamped) ? Da_raw : 0.f;
    };
    auto composite = [&](int cnt) {
      for (int p = (cnt - 1) >> 1; p >= 0; --p) {
        const float4 *qp = st + p * N4;
        float4 vv[N4];
#pragma unroll
        for (int i = 0; i < N4; ++i) vv[i] = qp[i];
        f2v f[2 * N4];
#pragma unroll
        for (int i = 0; i < N4; ++i) {
          asm volatile("" ::"v"(vv[i].x), "v"(vv[i].y), "v"(vv[i].z), "v"(vv[i].w));
          f[2 * i] = f2v{vv[i].x, vv[i].y};
          f[2 * i + 1] = f2v{vv[i].z, vv[i].w};
        }
        const f2v dx = f[0] - fx;
        f2v dy[PX], gx[PX], gy[PX], s2[PX], ex[PX], ar[PX];
        bool v0[PX], v1[PX];
        bool any = false;
#pragma unroll
        for (int q = 0; q < PX; ++q) {
          dy[q] = f[1] - fy[q];
          gx[q] = f[2] * dx + f[3] * dy[q];
          gy[q] = f[3] * dx + f[4] * dy[q];
          s2[q] = dx * gx[q] + dy[q] * gy[q];
          v0[q] = (__float_as_uint(s2[q].x) <= __float_as_uint(f[6].x)) &&
                  (__float_as_int(f[7].x) <= mylast[q]);
          v1[q] = (__float_as_uint(s2[q].y) <= __float_as_uint(f[6].y)) &&
                  (__float_as_int(f[7].y) <= mylast[q]);
          any |= v0[q] | v1[q];
        }
        if (__ballot(any) == 0) continue;
        f2v v[NV * 16];
#pragma unroll
        for (int kk = 0; kk < NV * 16; ++kk) v[kk] = f2v{0.f, 0.f};
#pragma unroll
        for (int q = 0; q < PX; ++q) {
          // this pair misses the wave's q-th 16x4 strip entirely (small
          // Gaussians touch one strip of the band): nothing to add, T unchanged
          if (PX > 1 && __ballot(v0[q] | v1[q]) == 0) continue;
          ex[q] = f2v{__builtin_amdgcn_exp2f(-s2[q].x), __builtin_amdgcn_exp2f(-s2[q].y)};
          ar[q] = f[5] * ex[q];
          const f2v al = f2v{fminf(ar[q].x, kAlphaMax), fminf(ar[q].y, kAlphaMax)};
          const f2v om = 1.f - al;
          const f2v ra = f2v{__builtin_amdgcn_rcpf(om.x), __builtin_amdgcn_rcpf(om.y)};
          f2v gD = f[9] * Drc[q][0];
#pragma unroll
          for (int d = 1; d < D; ++d)
            gD = __builtin_elementwise_fma(f[9 + d], f2v{Drc[q][d], Drc[q][d]}, gD);
          float w1, Da1, w0, Da0;
          grad_seq(q, v1[q], ar[q].y <= kAlphaMax, al.y, ra.y, gD.y, w1, Da1);
          grad_seq(q, v0[q], ar[q].x <= kAlphaMax, al.x, ra.x, gD.x, w0, Da0);
          const f2v wt = f2v{w0, w1}, Da = f2v{Da0, Da1};
          if (a.dbg & 8) {  // timing attribution only: no gradient algebra
            v[0] += wt + Da;
            continue;
          }
          const f2v aD = al * Da;
#pragma unroll
          for (int d = 0; d < D; ++d)
            v[d] = __builtin_elementwise_fma(wt, f2v{Drc[q][d], Drc[q][d]}, v[d]);
          v[D] = __builtin_elementwise_fma(Da, ex[q], v[D]);
          const f2v tgx = aD * gx[q], tgy = aD * gy[q];
          v[D + 1] += tgx;
          v[D + 2] += tgy;
          const f2v P_ = aD * dx, Q_ = aD * dy[q];
          v[D + 3] = __builtin_elementwise_fma(P_, dx, v[D + 3]);
          v[D + 4] = __builtin_elementwise_fma(P_, dy[q], v[D + 4]);
          v[D + 5] = __builtin_elementwise_fma(Q_, dy[q], v[D + 5]);
          if (ABS) {
            v[D + 6] += f2v{fabsf(tgx.x), fabsf(tgx.y)};
            v[D + 7] += f2v{fabsf(tgy.x), fabsf(tgy.y)};
          }
        }
        const int g0 = __float_as_int(f[8].x), g1 = __float_as_int(f[8].y);
#pragma unroll
        for (int qq = 0; qq < NV; ++qq) {
          constexpr int NQ = F - 16 * (NV - 1);
          // (GSPLAT_HIP_DBG bit 2, timing attribution only: no cross-lane
          // reduction, each lane's own partial of its field)
          f2v tot;
          if (a.dbg & 4) {
            tot = v[16 * qq];
#pragma unroll
            for (int i = 1; i < 16; ++i)
              if (16 * qq + i < NV * 16 && lf == i) tot = v[16 * qq + i];
          } else {
            tot = qq < NV - 1 ? reduce_scatter2<16>(v + 16 * qq, lane)
                              : reduce_scatter2<NQ>(v + 16 * qq, lane);
          }
          const int field = 16 * qq + lf;
          if ((lane & 3) == 0 && lf < (qq < NV - 1 ? 16 : NQ) && !(a.dbg & 1)) {
            const float sc = field_scale(field);
            if (tot.x != 0.f) atomic_add_f32(a.packed + (int64_t)g0 * a.S + field, sc * tot.x);
            if (g1 >= 0 && tot.y != 0.f)
              atomic_add_f32(a.packed + (int64_t)g1 * a.S + field, sc * tot.y);
          }
        }
      }
    };
    int32_t g_n = id_at(end);
    if (PFB) {
      Attr<D> A;
      load_attr<D>(a, g_n, A);
      g_n = id_at(end - 64);
      for (int b1 = end; b1 > start; b1 -= 64) {
        Attr<D> An;
        load_attr<D>(a, g_n, An);  // clamped ids: valid past the last batch too
        g_n = id_at(b1 - 128);
        composite(stage(A, b1));
        wave_sync_lds();
        A = An;
      }
    } else {
      for (int b1 = end; b1 > start; b1 -= 64) {
        Attr<D> A;
        load_attr<D>(a, g_n, A);
        g_n = id_at(b1 - 64);
        composite(stage(A, b1));
        wave_sync_lds();
      }
    }
  }
  tl_store(a, t_start, lane);
}

// packed [G][S] -> the autograd tensors.  visible (or null: every row):
// rows of Gaussians without an isect received no atomic and were not zeroed
// (zero_rows_kernel): their gradients are written as zeros, nothing read.
template <int D, bool ABS>
__global__ void __launch_bounds__(256)
unpack_kernel(int64_t G, int S, const float *__restrict__ packed, float *__restrict__ v_means2d,
              float *__restrict__ v_conics, float *__restrict__ v_colors,
              float *__restrict__ v_opacities, float *__restrict__ v_abs,
              const int32_t *__restrict__ visible, const int32_t *__restrict__ vis_rank) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  // both loads issued together (the rank does not wait for the visibility)
  const int32_t vg = visible ? visible[g] : 1;
  const int32_t rk = vis_rank ? vis_rank[g] : 0;
  if (vg <= 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) v_colors[g * D + d] = 0.f;
    v_opacities[g] = 0.f;
    *reinterpret_cast<float2 *>(v_means2d + 2 * g) = make_float2(0.f, 0.f);
    v_conics[3 * g] = 0.f;
    v_conics[3 * g + 1] = 0.f;
    v_conics[3 * g + 2] = 0.f;
    if (ABS) *reinterpret_cast<float2 *>(v_abs + 2 * g) = make_float2(0.f, 0.f);
    return;
  }
  const float *r = packed + (vis_rank ? min<int64_t>((uint32_t)rk, G - 1) : g) * S;
#pragma unroll
  for (int d = 0; d < D; ++d) v_colors[g * D + d] = r[d];
  v_opacities[g] = r[D];
  *reinterpret_cast<float2 *>(v_means2d + 2 * g) = make_float2(r[D + 1], r[D + 2]);
  v_conics[3 * g] = r[D + 3];
  v_conics[3 * g + 1] = r[D + 4];
  v_conics[3 * g + 2] = r[D + 5];
  if (ABS) *reinterpret_cast<float2 *>(v_abs + 2 * g) = make_float2(r[D + 6], r[D + 7]);
}

// The largest tile's isect count -> *out (lane 0 of the block; out may be
// null): read back by the host on a LATER render to decide whether to launch
// the split-capable forward (use_split_now), never for correctness.  Uses
// one barrier.
GS_INLINE void block_max_out(int64_t v, int32_t *out) {
  __shared__ int smax;
  if (threadIdx.x == 0) smax = 0;
  __syncthreads();
  int x = (int)min(v, (int64_t)INT32_MAX);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(&smax, x);
  __syncthreads();
  if (threadIdx.x == 0 && out) *out = smax;
}

// Forward dispatch order: tiles bucketed by isect count (>= 2048, >= 1024,
// >= 512, the rest), heaviest bucket first, so the longest tiles start in the
// first wave of workgroups instead of finishing last.  Inside a bucket: lane
// order (lane l holds tiles l, l + 1024, ...).  One 1024-lane workgroup; the
// four bucket counts of a lane are packed into one u64 (16 bits each) for a
// single block scan.
__global__ void __launch_bounds__(1024)
tile_order_kernel(int n_tiles, const int32_t *__restrict__ offsets, int64_t n_isects,
                  const int64_t *__restrict__ n_dev, int32_t *__restrict__ order,
                  int32_t *__restrict__ max_out) {
  constexpr int MAXPER = 16;  // tiles per thread (n_tiles <= 16384)
  __shared__ uint64_t wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int bucket[MAXPER];
  uint64_t mine = 0;
  int64_t nmax = 0;
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) {
    const int t = tid + 1024 * i;
    bucket[i] = -1;
    if (t < n_tiles) {
      const int64_t e = tile_end(offsets, t, n_tiles, n_dev, n_isects);
      const int64_t n = e - offsets[t];
      nmax = max(nmax, n);
      bucket[i] = n >= 2048 ? 0 : n >= 1024 ? 1 : n >= 512 ? 2 : 3;
      mine += (uint64_t)1 << (16 * bucket[i]);
    }
  }
  block_max_out(nmax, max_out);
  uint64_t x = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint64_t before = 0, total = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    before += i < w ? wsum[i] : 0;
    total += wsum[i];
  }
  before += x - mine;  // this thread's exclusive prefix, per bucket
  int pos[4], base = 0;
#pragma unroll
  for (int bk = 0; bk < 4; ++bk) {
    pos[bk] = base + (int)((before >> (16 * bk)) & 0xffff);
    base += (int)((total >> (16 * bk)) & 0xffff);
  }
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) {
    const int bk = bucket[i];
    if (bk >= 0) {
      int p = pos[0];
      p = bk == 1 ? pos[1] : p;
      p = bk == 2 ? pos[2] : p;
      p = bk == 3 ? pos[3] : p;
      order[p] = tid + 1024 * i;
      pos[0] += bk == 0;
      pos[1] += bk == 1;
      pos[2] += bk == 2;
      pos[3] += bk == 3;
    }
  }
}

// XCD-grouped dispatch order: the same heaviest-first buckets, per 2x2 group
// of neighbouring tiles instead of per tile (a group's bucket is its heaviest
// tile's), and the four tiles of group q (q-th in that order) in slots
// 32 (q / 8) + q % 8 + 8 k, k < 4.  Workgroup b runs on XCD b % 8, so a
// group's tiles run on ONE XCD, dispatched together: the Gaussians they share
// (at M3 a visible Gaussian covers ~5.5 tiles) are fetched into one L2 instead
// of up to four.  Slots of missing tiles (image edges) hold -1 (the workgroup
// exits); the grid covers order_slots() = 32 ceil(groups / 8) slots.  One
// 1024-lane workgroup, up to 8 groups per lane (8192 groups).
constexpr int kGS = 2;  // group side, tiles
__host__ __device__ inline int order_groups(int C, int tw, int th) {
  return C * ((tw + kGS - 1) / kGS) * ((th + kGS - 1) / kGS);
}
__global__ void __launch_bounds__(1024)
tile_order_grouped_kernel(int C, int tw, int th, const int32_t *__restrict__ offsets,
                          int64_t n_isects, const int64_t *__restrict__ n_dev,
                          int32_t *__restrict__ order, int32_t *__restrict__ max_out) {
  constexpr int MAXPER = 8;
  __shared__ uint64_t wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int gw = (tw + kGS - 1) / kGS, gh = (th + kGS - 1) / kGS, ng = C * gw * gh;
  const int n_tiles = C * tw * th;
  // the tiles of group g (-1: outside the grid)
  auto tiles_of = [&](int g, int (&t)[kGS * kGS]) {
    const int c = g / (gw * gh), r = g - c * (gw * gh);
    const int gy = r / gw, gx = r - gy * gw;
#pragma unroll
    for (int k = 0; k < kGS * kGS; ++k) {
      const int ty = gy * kGS + k / kGS, tx = gx * kGS + k % kGS;
      t[k] = (tx < tw && ty < th) ? (c * th + ty) * tw + tx : -1;
    }
  };
  int bucket[MAXPER];
  uint64_t mine = 0;
  int64_t nmax = 0;
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) {
    const int g = tid + 1024 * i;
    bucket[i] = -1;
    if (g < ng) {
      int t[kGS * kGS];
      tiles_of(g, t);
      int64_t gm = 0;
#pragma unroll
      for (int k = 0; k < kGS * kGS; ++k)
        if (t[k] >= 0)
          gm = max(gm, tile_end(offsets, t[k], n_tiles, n_dev, n_isects) - offsets[t[k]]);
      nmax = max(nmax, gm);
      bucket[i] = gm >= 2048 ? 0 : gm >= 1024 ? 1 : gm >= 512 ? 2 : 3;
      mine += (uint64_t)1 << (16 * bucket[i]);
    }
  }
  block_max_out(nmax, max_out);
  uint64_t x = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint64_t before = 0, total = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    before += i < w ? wsum[i] : 0;
    total += wsum[i];
  }
  before += x - mine;
  int pos[4], base = 0;
#pragma unroll
  for (int bk = 0; bk < 4; ++bk) {
    pos[bk] = base + (int)((before >> (16 * bk)) & 0xffff);
    base += (int)((total >> (16 * bk)) & 0xffff);
  }
  auto slot = [](int q, int k) { return 32 * (q >> 3) + (q & 7) + 8 * k; };
#pragma unroll
  for (int i = 0; i < MAXPER; ++i) {
    const int bk = bucket[i];
    if (bk >= 0) {
      int q = pos[0];
      q = bk == 1 ? pos[1] : q;
      q = bk == 2 ? pos[2] : q;
      q = bk == 3 ? pos[3] : q;
      int t[kGS * kGS];
      tiles_of(tid + 1024 * i, t);
#pragma unroll
      for (int k = 0; k < kGS * kGS; ++k) order[slot(q, k)] = t[k];
      pos[0] += bk == 0;
      pos[1] += bk == 1;
      pos[2] += bk == 2;
      pos[3] += bk == 3;
    }
  }
  // the slots of the group positions past the last group (up to a multiple of 8)
  const int q_end = (ng + 7) & ~7;
  for (int q = ng + tid; q < q_end; q += 1024)
#pragma unroll
    for (int k = 0; k < kGS * kGS; ++k) order[slot(q, k)] = -1;
}

// Forward plan with split heavy tiles, decided on this render's tiles.  A
// tile with more than `split` isects is rendered as ceil(n / SL) chunks that
// run in parallel in a launch of their own (see "Split heavy tiles"), so the
// longest tiles no longer serialise the end of the forward.  Outputs: `order` = the other tiles in tile_order_kernel's
// dispatch order (buckets of >= 2048, >= 1024, >= 512 isects, the rest; lane
// order inside a bucket), hdr[0] their number; `chunks` = (tile, k) of the
// split tiles, a tile's chunks consecutive in k, hdr[1] their number; the
// split tiles' hand-off flags and chunk counters cleared.  One 1024-lane
// workgroup, 16 tiles per lane (n_tiles <= 16384).
__global__ void __launch_bounds__(1024)
fwd_plan_kernel(int n_tiles, const int32_t *__restrict__ offsets, int64_t n_isects,
                const int64_t *__restrict__ n_dev, const uint8_t *__restrict__ masks, int SL,
                int L, int split, int32_t *__restrict__ hdr, int32_t *__restrict__ order,
                int2 *__restrict__ chunks, int32_t *__restrict__ pflag,
                int32_t *__restrict__ ctr, int32_t *__restrict__ max_out) {
  // quantities: [0..3] whole tiles per bucket, [4] chunks
  constexpr int PER = 16, NQ = 5;
  __shared__ int wsum[16][NQ];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // bucket (or -1: split) and chunk count of tile t (recomputed in the write
  // pass: keeps the 16 tiles' state out of registers)
  auto classify = [&](int t, int &nch) -> int {
    const int64_t n = tile_end(offsets, t, n_tiles, n_dev, n_isects) - offsets[t];
    nch = 0;
    if (n > split && !(masks && masks[t])) {
      nch = (int)((n + SL - 1) / SL);
      return -1;
    }
    return n >= 2048 ? 0 : n >= 1024 ? 1 : n >= 512 ? 2 : 3;
  };
  int mine[NQ] = {0, 0, 0, 0, 0};
  int64_t nmax = 0;
  for (int i = 0; i < PER; ++i) {
    const int t = tid + 1024 * i;
    if (t >= n_tiles) break;
    int nch;
    const int kd = classify(t, nch);
#pragma unroll
    for (int q = 0; q < 4; ++q) mine[q] += q == kd;
    mine[4] += nch;
    nmax = max(nmax, tile_end(offsets, t, n_tiles, n_dev, n_isects) - offsets[t]);
  }
  block_max_out(nmax, max_out);
  int x[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    x[q] = mine[q];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x[q], o, 64);
      if (lane >= o) x[q] += y;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) wsum[w][q] = x[q];
  }
  __syncthreads();
  int pos[NQ], total[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    pos[q] = x[q] - mine[q];
    total[q] = 0;
    for (int ww = 0; ww < 16; ++ww) {
      pos[q] += ww < w ? wsum[ww][q] : 0;
      total[q] += wsum[ww][q];
    }
  }
  // bucket q's whole tiles start after the heavier buckets
  int base = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    pos[q] += base;
    base += total[q];
  }
  for (int i = 0; i < PER; ++i) {
    const int t = tid + 1024 * i;
    if (t >= n_tiles) break;
    int nch;
    const int kd = classify(t, nch);
    if (kd < 0) {
      ctr[pos[4]] = 0;  // index of chunk 0
      for (int k = 0; k < nch; ++k) {
        chunks[pos[4]++] = make_int2(t, k);
        if (k < nch - 1) {
          const int64_t sl = ((int64_t)offsets[t] + (int64_t)(k + 1) * SL) / L;
          reinterpret_cast<int4 *>(pflag)[sl] = make_int4(0, 0, 0, 0);
        }
      }
    } else {
      int p = pos[0];
      p = kd == 1 ? pos[1] : p;
      p = kd == 2 ? pos[2] : p;
      p = kd == 3 ? pos[3] : p;
      order[p] = t;
      pos[0] += kd == 0;
      pos[1] += kd == 1;
      pos[2] += kd == 2;
      pos[3] += kd == 3;
    }
  }
  if (tid == 0) {
    hdr[0] = base;
    hdr[1] = total[4];
  }
}

// Backward work items.  A tile with n isects becomes ceil(n / L) items
// (tile, k): the full-length chunks go to `full`, the shorter tails to `tail`
// (the backward runs all full chunks first, so the longest items start
// first).  One lane per tile; one atomic per wave and list on the counters
// n_items[0..1], which the packed-gradient memset has zeroed.
__global__ void __launch_bounds__(256)
chunk_items_kernel(int n_tiles, const int32_t *__restrict__ offsets, int64_t n_isects,
                   const int64_t *__restrict__ n_dev, int L,
                   int2 *__restrict__ full, int2 *__restrict__ tail,
                   int32_t *__restrict__ n_items) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int nf = 0, nt = 0;
  if (t < n_tiles) {
    const int64_t e = tile_end(offsets, t, n_tiles, n_dev, n_isects);
    const int64_t n = e - offsets[t];
    nf = (int)(n / L);
    nt = (n % L) != 0;
  }
  int xf = nf, xt = nt;  // inclusive wave scans
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int yf = __shfl_up(xf, o, 64), yt = __shfl_up(xt, o, 64);
    if (lane >= o) {
      xf += yf;
      xt += yt;
    }
  }
  int bf = 0, bt = 0;
  if (lane == 63) {
    bf = xf ? atomicAdd(&n_items[0], xf) : 0;
    bt = xt ? atomicAdd(&n_items[1], xt) : 0;
  }
  bf = __shfl(bf, 63, 64) + xf - nf;
  bt = __shfl(bt, 63, 64) + xt - nt;
  for (int k = 0; k < nf; ++k) full[bf + k] = make_int2(t, k);
  if (nt) tail[bt] = make_int2(t, nf);
}

// Render records (see kRecFloats): one thread per Gaussian; rows whose
// `visible` count is 0 are never gathered and are skipped.
template <int D>
__global__ void __launch_bounds__(256)
pack_records_kernel(int64_t G, const float *__restrict__ means2d, const float *__restrict__ conics,
                    const float *__restrict__ colors, const float *__restrict__ opacities,
                    const int32_t *__restrict__ visible, const int32_t *__restrict__ vis_rank,
                    float *__restrict__ records) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  // both loads issued together (the rank does not wait for the visibility)
  const int32_t vg = visible ? visible[g] : 1;
  const int32_t rk = vis_rank ? vis_rank[g] : 0;
  if (vg <= 0) return;
  // rank-indexed table: row = the Gaussian's depth rank among the visible
  const int64_t row = vis_rank ? min<int64_t>((uint32_t)rk, G - 1) : g;
  constexpr int N4 = (6 + D + 3) / 4;
  float r[4 * N4];
  const float2 xy = *reinterpret_cast<const float2 *>(means2d + 2 * g);
  r[0] = xy.x;
  r[1] = xy.y;
  r[2] = conics[3 * g];
  r[3] = conics[3 * g + 1];
  r[4] = conics[3 * g + 2];
  r[5] = opacities[g];
#pragma unroll
  for (int d = 0; d < D; ++d) r[6 + d] = colors[g * D + d];
#pragma unroll
  for (int d = 6 + D; d < 4 * N4; ++d) r[d] = 0.f;
  float4 *o = reinterpret_cast<float4 *>(records + row * kRecFloats);
#pragma unroll
  for (int q = 0; q < N4; ++q) o[q] = make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
}

}  // namespace r16

int rasterize16_record_floats(int D) {
  return (D >= 1 && D <= r16::kRecMaxD) ? r16::kRecFloats : 0;
}

int rasterize16_pack_records(int64_t G, int D, const float *means2d, const float *conics,
                             const float *colors, const float *opacities, const int32_t *visible,
                             const int32_t *vis_rank, float *records, hipStream_t st) {
  GS_REQUIRE(rasterize16_record_floats(D) > 0, "rasterize_pack_records: %d channels > %d", D,
             r16::kRecMaxD);
  GS_REQUIRE(G < ((int64_t)1 << 31) / (r16::kRecFloats * 4),
             "rasterize_pack_records: %lld rows exceed the 2 GiB buffer-load range", (long long)G);
  if (G <= 0) return 0;
  const dim3 grid((unsigned)((G + 255) / 256));
  switch (D) {
#define GS_PACK(DD)                                                                              \
  case DD:                                                                                       \
    hipLaunchKernelGGL(r16::pack_records_kernel<DD>, grid, dim3(256), 0, st, G, means2d, conics, \
                       colors, opacities, visible, vis_rank, records);                          \
    break;
    GS_PACK(1) GS_PACK(2) GS_PACK(3) GS_PACK(4) GS_PACK(5) GS_PACK(6) GS_PACK(7) GS_PACK(8)
    GS_PACK(9) GS_PACK(10)
#undef GS_PACK
  }
  GS_CHECK_LAUNCH("rasterize_pack_records");
  return 0;
}

// Chunk length in isects for the chunked backward (multiple of 64; 0 turns
// chunking off).  GSPLAT_HIP_CHUNK overrides it for experiments.  256: at M2
// the two-pixel backward took 0.47 ms against 0.51 (512) and 0.61 (1024) on
// one box, for +6 us of chunk-state stores in the forward (tools/ab_chunk.sh).
static int g_chunk = -1;  // -1: not yet read from the environment

static int chunk_len() {
  if (g_chunk < 0) {
    const char *e = getenv("GSPLAT_HIP_CHUNK");
    const int x = e ? atoi(e) : 256;
    g_chunk = x <= 0 ? 0 : ((x + 63) / 64) * 64;
  }
  return g_chunk;
}

static int64_t state_floats_per_slot(int D) { return (int64_t)r16::kTS * r16::kTS * (1 + D); }

// [chunk slots (L > 0)][tile order: n_tiles i32 (n_tiles <= 16384)]
static int64_t chunk_slot_bytes(int D, int64_t n_isects) {
  const int L = chunk_len();
  if (L == 0 || n_isects <= 0) return 0;
  return (n_isects / L + 1) * state_floats_per_slot(D) * (int64_t)sizeof(float);
}

static bool use_order(int n_tiles, int64_t n_isects) {
  return n_isects > 0 && n_tiles > 0 && n_tiles <= 16384;
}

// Split heavy tiles in the forward (fwd_plan_kernel, "Split heavy tiles"):
// a tile with more isects than the threshold is rendered as parallel chunks
// of split_chunk() isects, concurrently with the other tiles, so that it no
// longer runs alone for the end of the launch.  Mode
// (GSPLAT_HIP_FWD_SPLIT / gsplat_hip_debug_set_fwd_split): unset or < 0 =
// adaptive, threshold max(2048, n_isects / GSPLAT_HIP_FWD_SPLIT_DIV) -- a
// tile longer than that fraction of all isects outlasts the rest of the
// launch (at M3 the heaviest, 21 k-isect tile ran 415 us against 250 us for
// 99 % of the waves) -- decided per tile on the device, so a render without
// such a tile runs the plain forward; > 0 = that fixed threshold; 0 = off.
static int g_fwd_split = INT32_MIN;  // not yet read from the environment

static int fwd_split_mode() {
  if (g_fwd_split == INT32_MIN) {
    const char *e = getenv("GSPLAT_HIP_FWD_SPLIT");
    g_fwd_split = (e && *e) ? atoi(e) : -1;  // (set but empty: the default)
    if (g_fwd_split < 0) g_fwd_split = -1;
  }
  return g_fwd_split;
}

static int split_div_default() {
  static const int div = [] {
    const char *e = getenv("GSPLAT_HIP_FWD_SPLIT_DIV");
    const int x = e ? atoi(e) : 550;
    return x > 0 ? x : 550;
  }();
  return div;
}
static int g_split_div = 0;  // gsplat_hip_set_fwd_split_div; 0: the default
static int split_div() { return g_split_div > 0 ? g_split_div : split_div_default(); }

static int64_t split_threshold(int64_t n_isects) {
  const int m = fwd_split_mode();
  if (m > 0) return m;
  return std::max<int64_t>(2048, n_isects / split_div());
}

static int chunk_len();
// Isects per chunk of a split tile (GSPLAT_HIP_FWD_SPLIT_CHUNK, default
// 1024), a multiple of the backward's chunk length.
static int split_chunk() {
  static const int x = [] {
    const char *e = getenv("GSPLAT_HIP_FWD_SPLIT_CHUNK");
    return e ? atoi(e) : 1024;
  }();
  const int L = chunk_len();
  return L > 0 ? std::max(L, (x + L - 1) / L * L) : 0;
}

// After the chunk slots and the tile order, the split area:
// [hdr 64 B][chunks int2 x (n_tiles + n_isects/SL + 1)][prod f32 x
// (n_isects/L + 1) x 256, by boundary slot][pflag i32 x (n_isects/L + 1) x 4]
// [ctr i32 x (n_tiles + n_isects/SL + 1)][cout f32 x (n_tiles + n_isects/SL
// + 1) x 256 x (2 + D)], each part 256-B aligned (chunks: sum over split
// tiles of ceil(n / SL) <= n_tiles + n_isects / SL).
struct SplitLayout {
  int64_t hdr, fitems, prod, pflag, ctr, cout, bytes;
};

static int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

// The state has room for the split forward whenever it can run; which tiles
// split is decided per render on the device (fwd_plan_kernel).
static bool split_capable(int n_tiles, int64_t n_isects) {
  return fwd_split_mode() != 0 && chunk_len() > 0 && use_order(n_tiles, n_isects);
}

// Largest tile of the most recent dispatch-order kernel, written by the
// kernel into mapped pinned host memory (no copy, no sync).
static int32_t *g_stat_host = nullptr, *g_stat_dev = nullptr;

static int32_t *stat_dev() {
  if (!g_stat_host) {
    if (hipHostMalloc((void **)&g_stat_host, 64, hipHostMallocMapped) != hipSuccess) {
      g_stat_host = nullptr;
      return nullptr;
    }
    g_stat_host[0] = 0;
    if (hipHostGetDevicePointer((void **)&g_stat_dev, g_stat_host, 0) != hipSuccess)
      g_stat_dev = nullptr;
  }
  return g_stat_dev;
}

// Launch the split-capable forward?  Fixed threshold: always; adaptive: when
// an earlier render's largest tile exceeded this render's threshold (tiles
// are similar from one training step to the next).  Which tiles split is
// then decided on the device from this render's tiles (fwd_plan_kernel); a
// wrong guess costs speed only: an unsplit heavy tile, or the split-capable
// kernel's lower occupancy with nothing to split.  A captured step keeps the
// choice of its capture.
// The trainer takes the decision out of this heuristic: from its first
// render it sets a fixed threshold (always the split-capable forward) or 0
// (never) with gsplat_hip_set_fwd_split_threshold (Trainer._tune_split), so
// every render of a run -- eager or captured -- takes the same variant with
// the same threshold.
static bool use_split_now(int n_tiles, int64_t n_isects) {
  if (!split_capable(n_tiles, n_isects)) return false;
  if (fwd_split_mode() > 0) return true;
  stat_dev();
  const int32_t prev = g_stat_host ? *(volatile int32_t *)g_stat_host : 0;
  return prev > split_threshold(n_isects);
}

static SplitLayout split_layout(int D, int n_tiles, int64_t n_isects) {
  SplitLayout l{};
  if (!split_capable(n_tiles, n_isects)) return l;
  const int64_t nc = n_isects / chunk_len() + 1, ns = n_isects / split_chunk() + 1;
  const int64_t px = r16::kTS * r16::kTS;
  l.hdr = 0;
  l.fitems = 256;
  l.prod = l.fitems + align256(8 * ((int64_t)n_tiles + ns));
  l.pflag = l.prod + align256(4 * nc * px);
  l.ctr = l.pflag + align256(16 * nc);
  l.cout = l.ctr + align256(4 * ((int64_t)n_tiles + ns));
  l.bytes = l.cout + align256(4 * ((int64_t)n_tiles + ns) * px * (2 + D));
  return l;
}

// XCD-grouped forward order (tile_order_grouped_kernel), the default for the
// unsplit forward; GSPLAT_HIP_DBG bit 4 restores the per-tile order.
// Measured (profiles/r6/xcd/, alternating bench runs, rocprofv3 counters of
// the forward): M2 forward 0.1622 / 0.1622 against 0.1655 / 0.1649 ms, L2 hit
// rate 0.618 -> 0.713, fetched bytes -27 %; M3 with the split off 0.605 /
// 0.603 against 0.608 / 0.608 ms, hit 0.451 -> 0.522, fetched -15 %.
int dbg_flags();
static int order_slots(int C, int tw, int th) {
  return 32 * ((r16::order_groups(C, tw, th) + 7) / 8);
}
static bool grouped_order(int C, int tw, int th) {
  const int64_t n_tiles = (int64_t)C * tw * th;
  return !(dbg_flags() & 16) && r16::order_groups(C, tw, th) <= 8192 &&
         order_slots(C, tw, th) <= 2 * n_tiles + 64;
}

static int64_t order_bytes(int n_tiles, int64_t n_isects) {
  // room for the grouped order's slots too (32 ceil(groups / 8) <= 2 n_tiles
  // + 64 for any grid)
  return use_order(n_tiles, n_isects) ? align256(4 * (2 * (int64_t)n_tiles + 64)) : 0;
}

static int64_t n_items_bound(int n_tiles, int64_t n_isects) {
  const int L = chunk_len();
  const int64_t n = L ? (int64_t)n_tiles + n_isects / L + 1 : (int64_t)n_tiles;
  const int64_t q = 8 * r16::kItemRun;  // whole rounds of the XCD-aware item order
  return (n + q - 1) / q * q;
}

int64_t rasterize16_fwd_state_bytes(int D, int n_tiles, int64_t n_isects) {
  return chunk_slot_bytes(D, n_isects) + order_bytes(n_tiles, n_isects) +
         split_layout(D, n_tiles, n_isects).bytes;
}

// The backward: two pixels per lane (bwd2_kernel<PX = 2>, a 16x8 band per
// wave) with the next batch's records gathered while the current one
// composites (PFB).  Measured against the alternatives, which were removed:
// one pixel per lane (16x4, 7 waves per SIMD) and four (16x16, 3 waves per
// SIMD) ran 0.47 / 0.465-0.473 ms against 0.427-0.430 ms at M2
// (profiles/r2_s4_bwdpf); without the prefetch 0.430 ms.
// One pixel per lane in the forward (16x4 per wave).  A two-pixel kernel
// (16x8 per wave, two transmittance chains per lane) measured 0.29 ms against
// 0.216 at M2 (158 VGPRs, 3 waves per SIMD, and the heaviest tiles' serial
// work per wave doubles) -- unlike the 2DGS forward, where two pixels per
// lane won 32 % -- and was removed.

static int g_dbg = INT32_MIN;  // not yet read from the environment
int dbg_flags() {  // also the 2DGS backward's (surfel.hip)
  if (g_dbg == INT32_MIN) {
    const char *e = getenv("GSPLAT_HIP_DBG");
    g_dbg = e ? atoi(e) : 0;
  }
  return g_dbg;
}
// State whose tile order gsplat_hip_rasterize_prepare already queued (so the
// forward call does not launch the order kernel again); cleared by the
// forward that consumes it.  Same host thread, same stream.
static thread_local const void *g_prepared_state = nullptr;
static thread_local bool g_prepared_split = false;  // the split decision of that preparation

static void launch_order(int C, int tw, int th, const int32_t *offsets, int64_t n_isects,
                         const int64_t *n_dev, int32_t *order, hipStream_t st,
                         char *split_base, int D) {
  const int n_tiles = C * tw * th;
  if (split_base) {
    const SplitLayout l = split_layout(D, n_tiles, n_isects);
    hipLaunchKernelGGL(r16::fwd_plan_kernel, dim3(1), dim3(1024), 0, st, n_tiles, offsets,
                       n_isects, n_dev, (const uint8_t *)nullptr, split_chunk(), chunk_len(),
                       (int)std::min<int64_t>(split_threshold(n_isects), INT32_MAX),
                       reinterpret_cast<int32_t *>(split_base + l.hdr), order,
                       reinterpret_cast<int2 *>(split_base + l.fitems),
                       reinterpret_cast<int32_t *>(split_base + l.pflag),
                       reinterpret_cast<int32_t *>(split_base + l.ctr), stat_dev());
  } else if (grouped_order(C, tw, th)) {
    hipLaunchKernelGGL(r16::tile_order_grouped_kernel, dim3(1), dim3(1024), 0, st, C, tw, th,
                       offsets, n_isects, n_dev, order,
                       split_capable(n_tiles, n_isects) ? stat_dev() : nullptr);
  } else {
    hipLaunchKernelGGL(r16::tile_order_kernel, dim3(1), dim3(1024), 0, st, n_tiles, offsets,
                       n_isects, n_dev, order,
                       split_capable(n_tiles, n_isects) ? stat_dev() : nullptr);
  }
}

template <int D>
int r16_fwd(r16::Args a, const void *state, char *split_base, hipStream_t st) {
  if (a.order && state != g_prepared_state)
    launch_order(a.C, a.tw, a.th, a.offsets, a.n_isects, a.n_dev, const_cast<int32_t *>(a.order),
                 st, split_base, D);
  g_prepared_state = nullptr;
  if (split_base) {
    // the split tiles' chunks and the other tiles in one launch; the grid is
    // an upper bound (the plan's counts are on the device; surplus
    // workgroups exit)
    const int64_t nc = std::min<int64_t>(
        (int64_t)a.n_tiles + a.n_isects / a.SL + 1,
        a.n_isects / a.SL + a.n_isects / std::max<int64_t>(1, split_threshold(a.n_isects)) + 1);
    const int64_t nw = ((int64_t)a.n_tiles + 8 * r16::kItemRun - 1) / (8 * r16::kItemRun) *
                       (8 * r16::kItemRun);  // whole rounds of the XCD runs
    hipLaunchKernelGGL((r16::fwd_kernel<D, true>), dim3((unsigned)(nw + nc)), dim3(256), 0, st,
                       a);
    GS_CHECK_LAUNCH("rasterize_fwd16_split");
    return 0;
  }
  const int grid = (a.order && grouped_order(a.C, a.tw, a.th)) ? order_slots(a.C, a.tw, a.th)
                                                                 : a.n_tiles;
  hipLaunchKernelGGL((r16::fwd_kernel<D>), dim3(grid), dim3(256), 0, st, a);
  GS_CHECK_LAUNCH("rasterize_fwd16");
  return 0;
}

static size_t packed_bytes(int D, bool absgrad, int64_t G) {
  const int F = D + 6 + (absgrad ? 2 : 0);
  return (((size_t)sizeof(float) * ((F + 15) / 16) * 16 * G + 255) / 256) * 256;
}

// Zero the gradient rows of the visible Gaussians only (visible[g] > 0: the
// rows the backward's atomics can reach) -- a quarter of the [G][S] table at
// M2 -- and the 256 bytes of item counters after the table.  One lane per
// row: one visibility load, S / 4 16-B stores.
__global__ void __launch_bounds__(256)
zero_rows_kernel(int64_t G, int S, const int32_t *__restrict__ visible,
                 const int32_t *__restrict__ vis_rank, float *__restrict__ packed,
                 int64_t tail_floats) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g < G && visible[g] > 0) {
    const int64_t row = vis_rank ? min<int64_t>((uint32_t)vis_rank[g], G - 1) : g;
    float4 *r = reinterpret_cast<float4 *>(packed + row * S);
    for (int q = 0; q < S / 4; ++q) r[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (blockIdx.x == 0 && threadIdx.x < tail_floats) packed[G * S + threadIdx.x] = 0.f;
}

// Rank-indexed rows with the visible count on the device (the sync-free
// isect's counts, {written, n_visible, ...}): the live rows are exactly rows
// 0 .. n_visible - 1, zeroed as one contiguous range -- consecutive lanes,
// consecutive rows, no per-Gaussian reads (zero_rows_kernel's scattered
// rows cost 9.5 us at M2).
__global__ void __launch_bounds__(256)
zero_ranked_rows_kernel(int64_t G, int S, const int64_t *__restrict__ counts,
                        float *__restrict__ packed, int64_t tail_floats) {
  const int64_t nv = min(G, counts[1]);
  // grid-stride over the live float4 slots (the grid is sized for the
  // expected live rows, not for all G: no workgroups that only exit)
  const int64_t n4 = nv * (S / 4);
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n4; q += (int64_t)gridDim.x * 256)
    reinterpret_cast<float4 *>(packed)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (blockIdx.x == 0 && threadIdx.x < tail_floats) packed[G * S + threadIdx.x] = 0.f;
}

template <int D, bool ABS>
int r16_bwd(r16::Args a, int64_t G, float *v_means2d, float *v_conics, float *v_colors,
            float *v_opacities, float *v_abs, void *workspace, const int32_t *visible,
            const int32_t *vis_rank, hipStream_t st) {
  constexpr int F = D + 6 + (ABS ? 2 : 0);
  a.S = ((F + 15) / 16) * 16;
  a.packed = reinterpret_cast<float *>(workspace);
  const bool chunked = a.n_isects > 0 && a.state && a.L > 0 && a.render_colors_in;
  // the gradient rows and, right after them, the item counters
  const size_t pb = packed_bytes(D, ABS, G);
  if (visible && G > 0) {
    // the counters start at byte pb (the table padded to 256 B): zero from
    // the table's end through them
    const int64_t tail = (int64_t)(pb / 4) - G * a.S + (chunked ? 64 : 0);
    if (vis_rank && a.n_dev)  // the counts of the sync-free isect: rows 0 .. n_visible - 1
      hipLaunchKernelGGL(zero_ranked_rows_kernel,
                         dim3((unsigned)std::min<int64_t>((G * (a.S / 4) + 255) / 256, 2048)),
                         dim3(256), 0, st, G, a.S, a.n_dev, a.packed, tail);
    else
      hipLaunchKernelGGL(zero_rows_kernel, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, st,
                         G, a.S, visible, vis_rank, a.packed, tail);
  } else {
    GS_HIP(gs::zero_async(a.packed, pb + (chunked ? 256 : 0), st));
  }
  if (a.n_isects > 0) {
    int64_t grid = a.n_tiles;
    if (chunked) {
      char *w = reinterpret_cast<char *>(workspace) + packed_bytes(D, ABS, G);
      a.n_items = reinterpret_cast<int32_t *>(w);
      a.items = reinterpret_cast<int2 *>(w + 256);
      a.items_tail = a.items + (a.n_isects / a.L + 1);
      hipLaunchKernelGGL(r16::chunk_items_kernel, dim3((unsigned)((a.n_tiles + 255) / 256)),
                         dim3(256), 0, st, a.n_tiles, a.offsets, a.n_isects, a.n_dev, a.L,
                         const_cast<int2 *>(a.items), const_cast<int2 *>(a.items_tail),
                         const_cast<int32_t *>(a.n_items));
      grid = n_items_bound(a.n_tiles, a.n_isects);
    } else {
      a.state = nullptr;
      a.items = nullptr;
      a.n_items = nullptr;
    }
    hipLaunchKernelGGL((r16::bwd2_kernel<D, ABS, 2, true>), dim3((unsigned)grid), dim3(128), 0,
                       st, a);
    GS_CHECK_LAUNCH("rasterize_bwd16");
  }
  if (G > 0) {
    hipLaunchKernelGGL((r16::unpack_kernel<D, ABS>), dim3((unsigned)((G + 255) / 256)), dim3(256),
                       0, st, G, a.S, a.packed, v_means2d, v_conics, v_colors, v_opacities, v_abs,
                       visible, vis_rank);
    GS_CHECK_LAUNCH("rasterize_bwd16_unpack");
  }
  return 0;
}

int rasterize16_fwd(int C, int D, int W, int H, int tw, int th, const float *means2d,
                    const float *conics, const float *colors, const float *opacities,
                    const float *backgrounds, const uint8_t *masks, const int32_t *offsets,
                    int64_t n_isects, const int64_t *n_isects_dev, const int32_t *flatten_ids,
                    float *render_colors, float *render_alphas, int32_t *last_ids,
                    const float *records, void *state, int64_t state_bytes, hipStream_t st) {
  r16::Args a{};
  a.n_dev = n_isects_dev;
  a.records = rasterize16_record_floats(D) ? records : nullptr;
  a.rec_bytes = 0x7fffffffu;  // rows < 2^31 / 64 (rasterize16_pack_records)
  a.C = C; a.W = W; a.H = H; a.tw = tw; a.th = th; a.n_tiles = C * tw * th;
  a.n_isects = n_isects;
  a.timeline = (g_timeline && g_timeline_waves >= 4 * (int64_t)a.n_tiles) ? g_timeline : nullptr;
  a.means2d = means2d; a.conics = conics; a.colors = colors; a.opacities = opacities;
  a.backgrounds = backgrounds; a.masks = masks; a.offsets = offsets; a.flatten_ids = flatten_ids;
  a.render_colors = render_colors; a.render_alphas = render_alphas; a.last_ids = last_ids;
  const int64_t need = rasterize16_fwd_state_bytes(D, a.n_tiles, n_isects);
  GS_REQUIRE(state_bytes == 0 || state_bytes >= need,
             "rasterize_fwd: state of %lld bytes needed, %lld given", (long long)need,
             (long long)state_bytes);
  a.L = chunk_len();
  a.dbg = dbg_flags();
  const int64_t slots = chunk_slot_bytes(D, n_isects);
  a.state = (state && slots > 0) ? reinterpret_cast<float *>(state) : nullptr;
  a.order = (state && use_order(a.n_tiles, n_isects))
                ? reinterpret_cast<int32_t *>(reinterpret_cast<char *>(state) + slots) : nullptr;
  char *split_base = nullptr;
  const bool split = state == g_prepared_state ? g_prepared_split
                                               : use_split_now(a.n_tiles, n_isects);
  if (a.order && a.state && split) {
    split_base = reinterpret_cast<char *>(state) + slots + order_bytes(a.n_tiles, n_isects);
    const SplitLayout l = split_layout(D, a.n_tiles, n_isects);
    a.n_whole = reinterpret_cast<const int32_t *>(split_base + l.hdr);
    a.n_chunks = a.n_whole + 1;
    a.fitems = reinterpret_cast<const int2 *>(split_base + l.fitems);
    a.prod = reinterpret_cast<float *>(split_base + l.prod);
    a.pflag = reinterpret_cast<int32_t *>(split_base + l.pflag);
    a.ctr = reinterpret_cast<int32_t *>(split_base + l.ctr);
    a.cout = reinterpret_cast<float *>(split_base + l.cout);
    a.SL = split_chunk();
    a.timeline = nullptr;  // per-wave stamps index blocks of the unsplit grid
  }
  switch (D) {
    case 1: return r16_fwd<1>(a, state, split_base, st);
    case 2: return r16_fwd<2>(a, state, split_base, st);
    case 3: return r16_fwd<3>(a, state, split_base, st);
    case 4: return r16_fwd<4>(a, state, split_base, st);
    case 8: return r16_fwd<8>(a, state, split_base, st);
    case 16: return r16_fwd<16>(a, state, split_base, st);
    case 32: return r16_fwd<32>(a, state, split_base, st);
  }
  GS_REQUIRE(false, "rasterize16_fwd: unsupported channels %d", D);
}

int rasterize16_prepare(int D, int C, int tw, int th, const int32_t *offsets, int64_t n_isects,
                        const int64_t *n_isects_dev, void *state, int64_t state_bytes,
                        hipStream_t st) {
  const int n_tiles = C * tw * th;
  g_prepared_state = nullptr;
  if (!state || !use_order(n_tiles, n_isects)) return 0;
  GS_REQUIRE(state_bytes >= rasterize16_fwd_state_bytes(D, n_tiles, n_isects),
             "rasterize_prepare: state too small");
  char *base = reinterpret_cast<char *>(state) + chunk_slot_bytes(D, n_isects);
  int32_t *order = reinterpret_cast<int32_t *>(base);
  const bool split = chunk_slot_bytes(D, n_isects) > 0 && use_split_now(n_tiles, n_isects);
  launch_order(C, tw, th, offsets, n_isects, n_isects_dev, order, st,
               split ? base + order_bytes(n_tiles, n_isects) : nullptr, D);
  GS_CHECK_LAUNCH("rasterize_prepare");
  g_prepared_state = state;
  g_prepared_split = split;
  return 0;
}

int64_t rasterize16_bwd_workspace(int64_t G, int D, bool absgrad, int n_tiles, int64_t n_isects) {
  int64_t b = (int64_t)packed_bytes(D, absgrad, G);
  if (chunk_len()) b += 256 + (int64_t)sizeof(int2) * n_items_bound(n_tiles, n_isects);
  return b;
}

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
                    hipStream_t st) {
  GS_REQUIRE(!vis_rank || visible, "rasterize_bwd: vis_rank needs visible");
  r16::Args a{};
  a.n_dev = n_isects_dev;
  a.records = rasterize16_record_floats(D) ? records : nullptr;
  a.rec_bytes = 0x7fffffffu;  // rows < 2^31 / 64 (rasterize16_pack_records)
  a.C = C; a.W = W; a.H = H; a.tw = tw; a.th = th; a.n_tiles = C * tw * th;
  a.n_isects = n_isects;
  a.timeline = (g_timeline && g_timeline_waves >= 4 * n_items_bound(a.n_tiles, n_isects))
                   ? g_timeline : nullptr;
  a.means2d = means2d; a.conics = conics; a.colors = colors; a.opacities = opacities;
  a.backgrounds = backgrounds; a.masks = masks; a.offsets = offsets; a.flatten_ids = flatten_ids;
  a.render_alphas = const_cast<float *>(render_alphas);
  a.last_ids = const_cast<int32_t *>(last_ids);
  a.v_render_colors = v_render_colors; a.v_render_alphas = v_render_alphas;
  // the backward reads the chunk slots only (the head of the state): the
  // tile-order and split areas after them depend on the forward's split
  // settings (a caller's gsplat_hip_set_fwd_split_threshold around the
  // forward alone, Trainer._tune_split), which must not turn the chunked
  // backward off
  const int64_t need = chunk_slot_bytes(D, n_isects);
  a.L = chunk_len();
  a.state = (state && need > 0 && state_bytes >= need)
                ? const_cast<float *>(reinterpret_cast<const float *>(state)) : nullptr;
  a.render_colors_in = render_colors;
  a.dbg = dbg_flags();
  const bool ab = v_abs != nullptr;
#define GS_R16B(DD)                                                                            \
  case DD:                                                                                     \
    return ab ? r16_bwd<DD, true>(a, G, v_means2d, v_conics, v_colors, v_opacities, v_abs,     \
                                  workspace, visible, vis_rank, st)                            \
              : r16_bwd<DD, false>(a, G, v_means2d, v_conics, v_colors, v_opacities, v_abs,    \
                                   workspace, visible, vis_rank, st);
  switch (D) { GS_R16B(1) GS_R16B(2) GS_R16B(3) GS_R16B(4) GS_R16B(8) GS_R16B(16) GS_R16B(32) }
#undef GS_R16B
  GS_REQUIRE(false, "rasterize16_bwd: unsupported channels %d", D);
}

}  // namespace gs

extern "C" int gsplat_hip_set_fwd_split_div(int div) {
  const int old = gs::split_div();
  gs::g_split_div = div > 0 ? div : 0;
  return old;
}

extern "C" int gsplat_hip_set_fwd_split_threshold(int isects) {
  const int old = gs::fwd_split_mode();
  gs::g_fwd_split = isects < 0 ? -1 : isects;
  return old;
}

extern "C" int64_t gsplat_hip_fwd_split_threshold(int64_t n_isects) {
  return gs::fwd_split_mode() == 0 ? -1 : gs::split_threshold(n_isects);
}

extern "C" int gsplat_hip_debug_set_fwd_split(int isects) {
  const int old = gs::fwd_split_mode();
  gs::g_fwd_split = isects < 0 ? -1 : isects;
  return old;
}

extern "C" int gsplat_hip_debug_set_flags(int flags) {
  const int old = gs::dbg_flags();
  gs::g_dbg = flags;
  return old;
}

extern "C" int gsplat_hip_debug_set_chunk(int isects) {
  gs::g_chunk = isects <= 0 ? 0 : ((isects + 63) / 64) * 64;
  return gs::g_chunk;
}

extern "C" int gsplat_hip_debug_set_timeline(uint64_t *device_buffer, int64_t capacity_waves) {
  gs::g_timeline = device_buffer;
  gs::g_timeline_waves = device_buffer ? capacity_waves : 0;
  return 0;
}
