// Supertile expansion: the sorted isects and the tile offsets from the
// depth-sorted visible Gaussians without sorting the isects themselves.
//
// The depth-first emission (isect.hip) writes every isect as a (camera | tile)
// key in depth order and sorts them stably by that key -- two 8-bit LSD
// passes over all isects (4 M at M2: emission 32 MB, two passes of 32 MB read
// + 32 MB written, the final 48 MB), then an offsets pass.  Here the isects
// are written once, at their final positions:
//   (1) rect_kernel   per visible Gaussian (depth order s): its tile rectangle
//                     (8 B) and the number of 4x4-tile supertiles it touches;
//   (2) emit_kernel   one (supertile key, s) pair per touched supertile, in
//                     depth order (0.78 M pairs at M2 against 4.04 M isects);
//   (3) one stable LSD pass over the pairs with a digit as wide as the key
//       (RX = 256 .. 2048 supertiles): every supertile's list in depth order;
//   (4) plan_kernel   supertile starts, the lists cut into segments of at
//                     most kSeg pairs (the work items of (5) and (7));
//   (5) seg_count     per segment and per tile of its supertile: the isects
//                     it holds (16 wave ballots per 64 pairs);
//       (and the tile totals, one atomic per (segment, tile));
//   (6) tile_scan     the exclusive scan of the tile totals in (camera, row,
//                     column) order = the isect offsets;
//   (7) seg_write     each segment's pairs in depth order: a lane's isect in
//                     tile t goes to base[t] + the lanes below it with a bit
//                     for t (ballot + mbcnt), so every tile's run is in depth
//                     order -- the reference's stable (camera | tile | depth)
//                     order, isect_ids / flatten_ids bit for bit.
// Negative depths (near_plane <= 0) form one virtual supertile after every
// real one: its Gaussians' isects (each repeated once per tile, all with the
// sign-extended id) go past the last real tile in depth-key order, exactly
// where the reference's masked 64-bit sort puts them.
// Capacity mode (the captured step): every count is read on the device; on an
// overflow nothing is written and every offset is 0.
// Tile culling of large surfels (the captured 2DGS training step,
// SurfelCull): a (supertile, surfel) pair of a surfel with more than
// kLanePairs pairs carries in its key's upper half the tiles of the supertile
// that its UV-plane image can reach (surfel_keep, the rasterizer's own strip
// test, on the whole tile); the other tiles of its rectangle get no isect.
// Near-degenerate surfels (the reference AABB's 1e-4 floor) cover every tile
// with their rectangle and light a few: at M5 ~1,000 of them held 41 % of
// the isects.  The rasterizer culls exactly these pairs per strip anyway
// (a strip is inside its tile), so images and gradients are unchanged; only
// the isect list -- an internal of the captured step -- is shorter.  The
// offsets and the isect count on the device (tile_scan) follow it.
#pragma once
#include "common.h"
#include "lsd_sort.h"
#include "surfel_cull.h"

namespace gs {
namespace st {

constexpr int S = 4;            // tiles per supertile side
constexpr int kSeg = 1024;      // pairs per segment (a 256-lane workgroup)
constexpr int kMaxKeys = 2048;  // supertiles (+ the virtual one) of the LSD pass
constexpr int kMaxTiles = kMaxKeys * S * S;

struct SurfelCull {  // all null: no tile culling
  const float *means2d;  // [G][2]
  const float *T;        // [G][3][3] ray transforms
  const float *opac;     // [G]
  int ts;                // tile size (pixels)
};
constexpr uint32_t kTightFlag = 1u << 15;  // key bits 16..31 hold the kept tiles

struct Geo {
  int C, N, tw, th, tile_bits;
  int stw, nst1;  // supertile columns, supertiles per camera
  int nst;        // C * nst1 + 1: the last key holds the negative-depth Gaussians
  int n_tiles;    // tiles per camera
};

inline Geo make_geo(int C, int N, int tw, int th, int tile_bits) {
  Geo g{};
  g.C = C; g.N = N; g.tw = tw; g.th = th; g.tile_bits = tile_bits;
  g.stw = (tw + S - 1) / S;
  g.nst1 = g.stw * ((th + S - 1) / S);
  g.nst = C * g.nst1 + 1;
  g.n_tiles = tw * th;
  return g;
}

GS_INLINE int cam_of(const int32_t *camera_ids, int N, int32_t g) {
  return camera_ids ? camera_ids[g] : g / N;
}

// tiles of the supertile d covered by rect r: bit 4*iy + ix
GS_INLINE uint32_t st_mask(const ushort4 r, int tx0, int ty0) {
  const int ix0 = max((int)r.x, tx0) - tx0, ix1 = min((int)r.y, tx0 + S) - tx0;
  const int iy0 = max((int)r.z, ty0) - ty0, iy1 = min((int)r.w, ty0 + S) - ty0;
  if (ix0 >= ix1 || iy0 >= iy1) return 0u;
  const uint32_t row = ((1u << ix1) - 1u) & ~((1u << ix0) - 1u);
  uint32_t m = 0u;
#pragma unroll
  for (int iy = 0; iy < S; ++iy)
    if (iy >= iy0 && iy < iy1) m |= row << (S * iy);
  return m;
}

template <typename T>
GS_INLINE T block_excl_scan256(T v, T *lds /* [5] */, T *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  T before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    before += w < wid ? lds[w] : (T)0;
    all += lds[w];
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

// capacity state of the sync-free isect (isect.hip cap_check): {n written or
// 0, n_visible, overflow, n}; null in the synchronous path
GS_INLINE bool void_call(const int64_t *cap) { return cap && cap[2]; }

// (1) rectangle and supertile count of every visible Gaussian, per-block sums
__global__ void __launch_bounds__(256)
rect_kernel(int64_t nV, const int64_t *__restrict__ cap, const int32_t *__restrict__ Vs,
            const uint32_t *__restrict__ dkeys, const float *__restrict__ means2d,
            const int32_t *__restrict__ radii, int ts, Geo geo, ushort4 *__restrict__ rect,
            int64_t *__restrict__ blk, int32_t *__restrict__ vis_rank,
            int32_t *__restrict__ n_huge) {
  __shared__ int64_t lds[5];
  // the ranks are written even when the call is void (an overflow): the
  // rasterizer's record packing and gradient rows read them for every
  // Gaussian with a tile
  if (cap) nV = min(nV, cap[1]);
  const bool vd = void_call(cap);
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n_huge && s == 0) *n_huge = 0;  // the huge list of emit_kernel (this launch precedes it)
  int np = 0;
  if (s < nV && vis_rank) vis_rank[Vs[s]] = (int32_t)s;
  if (s < nV && !vd) {
    const int32_t g = Vs[s];
    const float2 p = *reinterpret_cast<const float2 *>(means2d + 2 * (int64_t)g);
    const float r = (float)radii[g], t = (float)ts;
    const int x0 = min(max((int)floorf(__fdiv_rn(p.x - r, t)), 0), geo.tw);
    const int x1 = min(max((int)ceilf(__fdiv_rn(p.x + r, t)), 0), geo.tw);
    const int y0 = min(max((int)floorf(__fdiv_rn(p.y - r, t)), 0), geo.th);
    const int y1 = min(max((int)ceilf(__fdiv_rn(p.y + r, t)), 0), geo.th);
    rect[s] = make_ushort4((unsigned short)x0, (unsigned short)x1, (unsigned short)y0,
                           (unsigned short)y1);
    if ((int32_t)dkeys[s] < 0) np = 1;
    else np = ((x1 - 1) / S - x0 / S + 1) * ((y1 - 1) / S - y0 / S + 1);
  }
  int64_t tot;
  block_excl_scan256<int64_t>((int64_t)np, lds, &tot);
  if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}

// (2) (supertile key, s) pairs in depth order
constexpr int kLanePairs = 16;
// Huge (n_huge non-null: the captured 2DGS step, whose near-degenerate
// surfels span the whole image -- ~2,000 with ~510 pairs each at M5, all
// adjacent in depth order, so a few dozen waves each looped over 64 of them
// in turn while the rest of the grid idled): more than kHugePairs pairs go
// to a list that huge_emit_kernel spreads over the grid.
constexpr int kHugePairs = 128;
struct HugeEmit {
  int64_t cur;  // first output slot
  int32_t s, n, x0, y0, w;
  uint32_t kb;
};

__global__ void __launch_bounds__(256)
emit_kernel(int64_t nV, const int64_t *__restrict__ cap, const int32_t *__restrict__ Vs,
            const uint32_t *__restrict__ dkeys, const ushort4 *__restrict__ rect,
            const int32_t *__restrict__ camera_ids, Geo geo, const int64_t *__restrict__ blk_prefix,
            uint32_t *__restrict__ pkey, int32_t *__restrict__ pval,
            HugeEmit *__restrict__ huge_list, int32_t *__restrict__ n_huge) {
  __shared__ int64_t lds[5];
  if (cap) nV = void_call(cap) ? 0 : min(nV, cap[1]);
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int np = 0, sx0 = 0, sy0 = 0, w = 1;
  uint32_t kbase = 0;
  bool neg = false;
  if (s < nV) {
    const ushort4 r = rect[s];
    neg = (int32_t)dkeys[s] < 0;
    sx0 = r.x / S;
    sy0 = r.z / S;
    w = (r.y - 1) / S - sx0 + 1;
    np = neg ? 1 : w * ((r.w - 1) / S - sy0 + 1);
    kbase = neg ? (uint32_t)(geo.nst - 1)
                : (uint32_t)(cam_of(camera_ids, geo.N, Vs[s]) * geo.nst1);
  }
  int64_t tot;
  const int64_t cur0 = blk_prefix[blockIdx.x] + block_excl_scan256<int64_t>((int64_t)np, lds, &tot);
  if (np > 0 && np <= kLanePairs) {
    for (int k = 0; k < np; ++k) {
      const int yy = k / w, xx = k - yy * w;
      pkey[cur0 + k] = neg ? kbase : kbase + (uint32_t)((sy0 + yy) * geo.stw + sx0 + xx);
      pval[cur0 + k] = (int32_t)s;
    }
  }
  // huge (the list given): one slot per lane in the list, one atomic per wave
  const int huge_at = n_huge ? kHugePairs : 0x7fffffff;
  const uint64_t huge = __ballot(np > huge_at);
  if (huge) {
    int base = 0;
    if (lane == 0) base = atomicAdd(n_huge, __popcll(huge));
    base = __shfl(base, 0, 64);
    if (np > huge_at)
      huge_list[base + __popcll(huge & ((1ull << lane) - 1ull))] =
          HugeEmit{cur0, (int32_t)s, np, sx0, sy0, w, kbase};
  }
  // large Gaussians: the whole wave writes each one's pairs (coalesced)
  uint64_t big = __ballot(np > kLanePairs && np <= huge_at);
  while (big) {
    const int src = __builtin_ctzll(big);
    big &= big - 1;
    const int64_t c0 = __shfl(cur0, src, 64);
    const int n = __shfl(np, src, 64), bw = __shfl(w, src, 64);
    const int bx = __shfl(sx0, src, 64), by = __shfl(sy0, src, 64);
    const uint32_t kb = __shfl(kbase, src, 64);
    const int32_t bs = __shfl((int32_t)s, src, 64);
    for (int k = lane; k < n; k += 64) {
      const int yy = k / bw, xx = k - yy * bw;
      pkey[c0 + k] = kb + (uint32_t)((by + yy) * geo.stw + bx + xx);
      pval[c0 + k] = bs;
    }
  }
}

// (2a) the huge list: kHugeParts workgroups per entry, each writing a
// contiguous part of its pairs (coalesced); a grid-stride over the entries
constexpr int kHugeParts = 4;
constexpr int kHugeBlocks = 1024;

__global__ void __launch_bounds__(256)
huge_emit_kernel(const HugeEmit *__restrict__ huge_list, const int32_t *__restrict__ n_huge,
                 Geo geo, uint32_t *__restrict__ pkey, int32_t *__restrict__ pval) {
  const int nh = *n_huge;
  const int part = blockIdx.x % kHugeParts;
  for (int e = blockIdx.x / kHugeParts; e < nh; e += kHugeBlocks / kHugeParts) {
    const HugeEmit g = huge_list[e];
    const int k0 = (int)(((int64_t)g.n * part) / kHugeParts);
    const int k1 = (int)(((int64_t)g.n * (part + 1)) / kHugeParts);
    for (int k = k0 + (int)threadIdx.x; k < k1; k += 256) {
      const int yy = k / g.w, xx = k - yy * g.w;
      pkey[g.cur + k] = g.kb + (uint32_t)((g.y0 + yy) * geo.stw + g.x0 + xx);
      pval[g.cur + k] = g.s;
    }
  }
}

// (2b) tile culling of large surfels (SurfelCull), before the supertile pass:
// a pair of a surfel with more than kLanePairs pairs gets kTightFlag and, in
// key bits 16..31, the tiles of its supertile that the surfel's image can
// reach (surfel_keep on the tiles' pixel centres).  The emission writes a
// surfel's pairs consecutively, so a wave mostly holds one surfel's pairs,
// most of whose supertiles a thin surfel does not cross.  Two phases per wave:
// every lane tests its whole supertile (one test); then the surviving pairs'
// tiles are dealt out 16 lanes to a pair, 4 pairs per round (the pair's
// surfel from its lane by bpermute, the kept tiles back by one ballot), so a
// wave runs ceil(survivors / 4) tile tests instead of 16.  (Per-lane tile
// loops made it 88 us per M5 step: every wave paid for its busiest lane.)
GS_INLINE bool reach_tiles(const float *m9, float mx, float my, float op, int ts, int x0, int x1,
                           int y0, int y1) {  // tiles [x0, x1) x [y0, y1)
  return surfel::surfel_keep(m9, mx, my, op, (float)(x0 * ts) + 0.5f, (float)(x1 * ts) - 0.5f,
                             (float)(y0 * ts) + 0.5f, (float)(y1 * ts) - 0.5f);
}

__global__ void __launch_bounds__(256)
tight_kernel(int64_t cap_pairs, const int64_t *__restrict__ n_pairs, Geo geo,
             const int32_t *__restrict__ Vs, const ushort4 *__restrict__ rect,
             const int64_t *__restrict__ cap, uint32_t *__restrict__ pkey,
             const int32_t *__restrict__ pval, SurfelCull sc) {
  if (void_call(cap)) return;
  const int64_t n = min(cap_pairs, n_pairs[0]);
  const int lane = threadIdx.x & 63;
  // grid-stride over wave-sized chunks (the ballots need whole waves)
  for (int64_t base = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); base < n;
       base += (int64_t)gridDim.x * 256) {
    const int64_t p = base + lane;
    uint32_t key = 0u;
    bool big = false;
    ushort4 r = {0, 0, 0, 0};
    int32_t g = 0;
    if (p < n) {
      key = pkey[p];
      if ((int)key < geo.nst - 1) {  // not the negative-depth key: no tiles to cull
        const int32_t s = pval[p];
        r = rect[s];
        const int sx0 = r.x / S, sy0 = r.z / S;
        big = ((r.y - 1) / S - sx0 + 1) * ((r.w - 1) / S - sy0 + 1) > kLanePairs;
        if (big) g = Vs[s];
      }
    }
    if (__ballot(big) == 0ull) continue;
    float m9[9], mx = 0.f, my = 0.f, op = 0.f;
#pragma unroll
    for (int i = 0; i < 9; ++i) m9[i] = big ? sc.T[9 * (int64_t)g + i] : 0.f;
    if (big) {
      mx = sc.means2d[2 * (int64_t)g];
      my = sc.means2d[2 * (int64_t)g + 1];
      op = sc.opac[g];
    }
    const int rr = (int)key % geo.nst1;  // supertile within its camera
    const int sy = rr / geo.stw;
    const int tx0 = (rr - sy * geo.stw) * S, ty0 = sy * S;
    const int ix0 = max((int)r.x, tx0), ix1 = min((int)r.y, tx0 + S);
    const int iy0 = max((int)r.z, ty0), iy1 = min((int)r.w, ty0 + S);
    // phase 1: the pair's covered part of its supertile
    const bool live = big && ix0 < ix1 && iy0 < iy1 &&
                      reach_tiles(m9, mx, my, op, sc.ts, ix0, ix1, iy0, iy1);
    uint32_t keep = 0u;
    // phase 2: 4 surviving pairs per round, one tile per lane
    uint64_t rem = __ballot(live);
    const int q = lane >> 4, t = lane & 15;
    while (rem) {
      int own[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        own[j] = rem ? __builtin_ctzll(rem) : 64;
        rem &= rem - 1ull;
      }
      const int o = q == 0 ? own[0] : q == 1 ? own[1] : q == 2 ? own[2] : own[3];
      const int src = o & 63;
      float n9[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) n9[i] = __shfl(m9[i], src, 64);
      const float nx = __shfl(mx, src, 64), ny = __shfl(my, src, 64), nop = __shfl(op, src, 64);
      const int a0 = __shfl(ix0, src, 64), a1 = __shfl(ix1, src, 64);
      const int b0 = __shfl(iy0, src, 64), b1 = __shfl(iy1, src, 64);
      const int x = __shfl(tx0, src, 64) + (t & (S - 1)), y = __shfl(ty0, src, 64) + t / S;
      const bool hit = o < 64 && x >= a0 && x < a1 && y >= b0 && y < b1 &&
                       reach_tiles(n9, nx, ny, nop, sc.ts, x, x + 1, y, y + 1);
      const uint64_t hb = __ballot(hit);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (lane == own[j]) keep = (uint32_t)(hb >> (16 * j)) & 0xffffu;
    }
    if (big) pkey[p] = key | kTightFlag | (keep << 16);
  }
}

// (4) one workgroup: supertile starts, segments (kSeg pairs) and their keys
__global__ void __launch_bounds__(1024)
plan_kernel(int nst, const uint32_t *__restrict__ totals, int32_t *__restrict__ st_start,
            int32_t *__restrict__ seg_start, int32_t *__restrict__ seg_st, int n_tile_tot,
            int32_t *__restrict__ tile_tot) {
  __shared__ int32_t wa[16], wb[16];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  for (int i = t; i < n_tile_tot; i += 1024) tile_tot[i] = 0;  // seg_count adds into them
  // digits 2t, 2t + 1
  int c[2], sg[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int d = 2 * t + j;
    c[j] = d < nst ? (int)totals[d] : 0;
    sg[j] = (c[j] + kSeg - 1) / kSeg;
  }
  int a = c[0] + c[1], b = sg[0] + sg[1];
  int xa = a, xb = b;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int ya = __shfl_up(xa, o, 64), yb = __shfl_up(xb, o, 64);
    if (lane >= o) {
      xa += ya;
      xb += yb;
    }
  }
  if (lane == 63) {
    wa[wid] = xa;
    wb[wid] = xb;
  }
  __syncthreads();
  int pa = 0, pb = 0, ta = 0, tb = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    pa += w < wid ? wa[w] : 0;
    pb += w < wid ? wb[w] : 0;
    ta += wa[w];
    tb += wb[w];
  }
  int ra = pa + xa - a, rb = pb + xb - b;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int d = 2 * t + j;
    if (d < nst) {
      st_start[d] = ra;
      seg_start[d] = rb;
      for (int k = 0; k < sg[j]; ++k) seg_st[rb + k] = d;
    }
    ra += c[j];
    rb += sg[j];
  }
  if (t == 0) {
    st_start[nst] = ta;
    seg_start[nst] = tb;
  }
}

struct Seg {
  int d, p0, p1;
  bool virt;
  int tx0, ty0, cam;
};

GS_INLINE bool seg_of(int b, const Geo &geo, const int32_t *seg_start, const int32_t *seg_st,
                      const int32_t *st_start, Seg &sg) {
  if (b >= seg_start[geo.nst]) return false;
  const int d = seg_st[b];
  const int k = b - seg_start[d];
  sg.d = d;
  sg.p0 = st_start[d] + k * kSeg;
  sg.p1 = min(st_start[d + 1], sg.p0 + kSeg);
  sg.virt = d == geo.nst - 1;
  sg.cam = sg.virt ? 0 : d / geo.nst1;
  const int rr = d - sg.cam * geo.nst1;
  const int sy = rr / geo.stw, sx = rr - sy * geo.stw;
  sg.tx0 = sx * S;
  sg.ty0 = sy * S;
  return true;
}

// The wave's 4 x 64 pairs of the segment ([w*256, w*256+256)): every load
// issued before any is used (one round trip instead of four), then per pair
// the tile mask within the supertile -- or, in the virtual (negative-depth)
// segment, the Gaussian's tile count in m.
struct WavePairs {
  int32_t s[4];
  uint32_t m[4];
};

GS_INLINE void load_pairs(const Seg &sg, const int32_t *pval, const ushort4 *rect,
                          const int32_t *Vs, const int32_t *tpg, WavePairs &wp,
                          const uint32_t *pkey) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t kk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int p = sg.p0 + w * 256 + e * 64 + lane;
    wp.s[e] = p < sg.p1 ? pval[p] : -1;
    if (pkey && p < sg.p1) kk[e] = pkey[p];  // tile-culled pairs: their kept tiles
  }
  if (!sg.virt) {
    ushort4 r[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = rect[max(wp.s[e], 0)];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      wp.m[e] = wp.s[e] < 0 ? 0u
                : (kk[e] & kTightFlag) ? (kk[e] >> 16) : st_mask(r[e], sg.tx0, sg.ty0);
  } else {
    int32_t g[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) g[e] = Vs[max(wp.s[e], 0)];
#pragma unroll
    for (int e = 0; e < 4; ++e) wp.m[e] = wp.s[e] >= 0 ? (uint32_t)tpg[g[e]] : 0u;
  }
}

// per-wave isect counts per tile of the supertile -> wc[w][16] (virtual
// segment: wc[w][0] = the wave's isects)
GS_INLINE void wave_counts(const Seg &sg, const WavePairs &wp, int32_t (*wc)[S * S]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int cnt[S * S];
#pragma unroll
  for (int t = 0; t < S * S; ++t) cnt[t] = 0;
  if (!sg.virt) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int t = 0; t < S * S; ++t) cnt[t] += __popcll(__ballot((wp.m[e] >> t) & 1u));
  } else {
    int c = (int)(wp.m[0] + wp.m[1] + wp.m[2] + wp.m[3]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
    cnt[0] = c;
  }
  if (lane == 0) {
#pragma unroll
    for (int t = 0; t < S * S; ++t) wc[w][t] = cnt[t];
  }
}

// global tile index (camera, row, column) of bit t of the segment's
// supertile; the virtual segment's tile is T (past every real tile)
GS_INLINE int tile_index(const Geo &geo, const Seg &sg, int t) {
  if (sg.virt) return geo.C * geo.n_tiles;
  return sg.cam * geo.n_tiles + (sg.ty0 + t / S) * geo.tw + sg.tx0 + t % S;
}

// (5) per segment and tile: the isects it holds -> segcnt[b][16], and the
// tile totals (tile_tot zeroed by plan_kernel)
__global__ void __launch_bounds__(256)
seg_count_kernel(Geo geo, const int32_t *__restrict__ st_start, const int32_t *__restrict__ seg_start,
                 const int32_t *__restrict__ seg_st, const int32_t *__restrict__ pval,
                 const ushort4 *__restrict__ rect, const int32_t *__restrict__ Vs,
                 const int32_t *__restrict__ tpg, int32_t *__restrict__ segcnt,
                 int32_t *__restrict__ tile_tot, const uint32_t *__restrict__ pkey) {
  __shared__ int32_t wc[4][S * S];
  Seg sg;
  if (!seg_of(blockIdx.x, geo, seg_start, seg_st, st_start, sg)) return;
  WavePairs wp;
  load_pairs(sg, pval, rect, Vs, tpg, wp, pkey);
  wave_counts(sg, wp, wc);
  __syncthreads();
  if (threadIdx.x < S * S) {
    const int t = threadIdx.x;
    const int c = wc[0][t] + wc[1][t] + wc[2][t] + wc[3][t];
    segcnt[(int64_t)blockIdx.x * (S * S) + t] = c;
    if (c) atomicAdd(tile_tot + tile_index(geo, sg, t), c);
  }
}

// (6) one workgroup: exclusive scan of the tile totals [0, T] in place (tile
// T the virtual one); offsets[t] = tile_tot[t] for t < T (0 on a void call).
// Rounds of 8192 tiles staged through LDS: coalesced loads and stores, then
// 8 contiguous tiles per thread.
__global__ void __launch_bounds__(1024)
tile_scan_kernel(Geo geo, const int64_t *__restrict__ cap, int32_t *__restrict__ tile_tot,
                 int32_t *__restrict__ offsets, int64_t *__restrict__ n_out) {
  constexpr int R = 8192, PT = R / 1024;
  __shared__ int32_t buf[R];
  __shared__ int32_t wsum[16];
  const int T = geo.C * geo.n_tiles;
  const int nt = T + 1;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const bool vd = void_call(cap);
  int carry = 0;
  for (int base = 0; base < nt; base += R) {
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const int i = base + k * 1024 + t;
      buf[k * 1024 + t] = i < nt ? tile_tot[i] : 0;
    }
    __syncthreads();
    int v[PT], sum = 0;
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      v[k] = buf[t * PT + k];
      sum += v[k];
    }
    int x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int run = carry + x - sum, all = carry;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      run += w < wid ? wsum[w] : 0;
      all += wsum[w];
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      buf[t * PT + k] = run;
      run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const int i = base + k * 1024 + t;
      if (i < nt) {
        const int o = buf[k * 1024 + t];
        tile_tot[i] = o;
        if (i < T) offsets[i] = vd ? 0 : o;
      }
    }
    carry = all;
    __syncthreads();
  }
  // tile culling (SurfelCull): the isects written -- fewer than the count of
  // the tile rectangles -- are the count the rasterizer reads on the device
  if (n_out && t == 0 && !vd) n_out[0] = carry;
}

// (7) every segment's isects at their final slots: per tile, the tile's
// offset + the earlier segments of the supertile + the earlier waves
__global__ void __launch_bounds__(256)
seg_write_kernel(Geo geo, const int64_t *__restrict__ cap, const int32_t *__restrict__ st_start,
                 const int32_t *__restrict__ seg_start, const int32_t *__restrict__ seg_st,
                 const int32_t *__restrict__ pval, const ushort4 *__restrict__ rect,
                 const int32_t *__restrict__ Vs, const uint32_t *__restrict__ dkeys,
                 const int32_t *__restrict__ tpg, const int32_t *__restrict__ segcnt,
                 const int32_t *__restrict__ tile_off, int64_t *__restrict__ isect_ids,
                 int32_t *__restrict__ flatten_ids, int32_t *__restrict__ rank_ids,
                 const uint32_t *__restrict__ pkey) {
  __shared__ int32_t wc[4][S * S];
  __shared__ int32_t sbase[S * S];
  if (void_call(cap)) return;
  Seg sg;
  if (!seg_of(blockIdx.x, geo, seg_start, seg_st, st_start, sg)) return;
  WavePairs wp;
  load_pairs(sg, pval, rect, Vs, tpg, wp, pkey);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t g[4] = {0, 0, 0, 0};
  uint32_t db[4] = {0u, 0u, 0u, 0u};
  // isect_ids null: rank ids only, or flatten ids only (a rasterizer that
  // gathers by Gaussian id and reads the offsets, not the 64-bit keys)
  const bool ids = isect_ids != nullptr, fl = flatten_ids != nullptr;
  if (fl) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int s = max(wp.s[e], 0);
      g[e] = Vs[s];
      if (ids || sg.virt) db[e] = dkeys[s];
    }
  }
  if (threadIdx.x < S * S) {  // the earlier segments of this supertile
    const int t = threadIdx.x;
    // (a supertile bit past the grid's last row / column holds no isect)
    const bool in = sg.virt || (sg.tx0 + t % S < geo.tw && sg.ty0 + t / S < geo.th);
    int c = in ? tile_off[tile_index(geo, sg, t)] : 0;
    for (int b = seg_start[sg.d]; b < (int)blockIdx.x; ++b) c += segcnt[(int64_t)b * (S * S) + t];
    sbase[t] = c;
  }
  wave_counts(sg, wp, wc);
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  int cur[S * S];  // this wave's next slot per tile (wave-uniform)
#pragma unroll
  for (int t = 0; t < S * S; ++t) {
    int c = sbase[t];
    for (int v = 0; v < w; ++v) c += wc[v][t];
    cur[t] = c;
  }
  if (sg.virt) {
    // every isect of a negative-depth Gaussian carries its sign-extended id
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = (int)wp.m[e];
      int x = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      const int pos = cur[0] + x - c;
      const int64_t id = (int64_t)(int32_t)db[e];
      for (int k = 0; k < c; ++k) {
        if (ids) isect_ids[pos + k] = id;
        if (fl) flatten_ids[pos + k] = g[e];
        if (rank_ids) rank_ids[pos + k] = wp.s[e];
      }
      cur[0] += __shfl(x, 63, 64);
    }
    return;
  }
  const int64_t tkey0 = (int64_t)sg.cam << geo.tile_bits;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
#pragma unroll
    for (int t = 0; t < S * S; ++t) {
      const uint32_t bit = (wp.m[e] >> t) & 1u;
      const uint64_t bal = __ballot(bit);
      if (bal == 0) continue;
      if (bit) {
        const int pos = cur[t] + __popcll(bal & lt);
        if (ids) {
          const int tile = (sg.ty0 + t / S) * geo.tw + sg.tx0 + t % S;
          isect_ids[pos] = ((tkey0 | (int64_t)tile) << 32) | (int64_t)db[e];
        }
        if (fl) flatten_ids[pos] = g[e];
        if (rank_ids) rank_ids[pos] = wp.s[e];
      }
      cur[t] += __popcll(bal);
    }
  }
}

}  // namespace st
}  // namespace gs
