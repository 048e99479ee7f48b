// Tile intersection: per-Gaussian tile counts, prefix offsets, (isect_id,
// flatten_id) emission, radix sort and per-tile range offsets -- gfx950.
//
// Replaces the reference
//   get_tile_per_gauss_kernel / get_isect_ids_kernel  gsplat/triton_impl/isect_tiles.py:134-252
//   get_isec_tile                                    gsplat/triton_impl/isect_tiles.py:255-282
//   torch.cumsum + .item()                           gsplat/triton_impl/isect_tiles.py:101-102
//   radix_sort (CUB SortPairs, default stream)       gsplat/triton_impl/radix_sort/radix_sort.cu:9-62
//   get_isect_offsets_kernel                         gsplat/triton_impl/isect_offset.py:39-63
//
// Bit-exactness: tile rectangles use the Triton float formulas (L2), ids use
// the Triton tile-bit width (n_tiles-1).bit_length() (L1), depth bits are the
// int32 bitcast sign-extended to int64 exactly as the reference, emission
// order is Gaussian-major / tile-row-major, and the sort is a stable LSD
// radix sort over the low 32+tile_bits+cam_bits bits (rocPRIM), so
// isect_ids / flatten_ids equal the reference's element for element.
//
// Offsets: instead of materialising the int64 inclusive cumsum of
// tiles_per_gauss (8 B x C*N written and re-read), the count kernel writes
// one partial sum per 256-Gaussian block, a single-workgroup kernel scans
// those, and the write kernel redoes the block-local scan in LDS.
#include "common.h"
#include "../../include/gsplat_hip.h"

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include "isect_st.h"
#include "lsd_sort.h"
#include "wave_ops.h"

namespace gs {

constexpr int kIsectBlock = 256;

struct Rect {
  int x0, x1, y0, y1;
};

// isect_tiles.py:255-282 -- float32 (p -/+ r) / ts with floor/ceil, clamped.
GS_INLINE Rect tile_rect(float px, float py, int radius, int ts, int tw, int th) {
  const float r = (float)radius, t = (float)ts;
  Rect o;
  o.x0 = min(max((int)floorf(__fdiv_rn(px - r, t)), 0), tw);
  o.x1 = min(max((int)ceilf(__fdiv_rn(px + r, t)), 0), tw);
  o.y0 = min(max((int)floorf(__fdiv_rn(py - r, t)), 0), th);
  o.y1 = min(max((int)ceilf(__fdiv_rn(py + r, t)), 0), th);
  return o;
}

GS_INLINE int tiles_of(const float *means2d, const int32_t *radii, int64_t i, int ts, int tw,
                       int th, Rect *rect) {
  const int r = radii[i];
  if (r <= 0) return 0;
  const float2 p = *reinterpret_cast<const float2 *>(means2d + 2 * i);
  *rect = tile_rect(p.x, p.y, r, ts, tw, th);
  return (rect->x1 - rect->x0) * (rect->y1 - rect->y0);
}

template <typename T>
GS_INLINE T block_exclusive_scan(T v, T *lds /* [kIsectBlock/64 + 1] */, T *total) {
  // wave-level inclusive scan with shuffles, then across the 4 waves via LDS
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
    for (int w = 0; w < kIsectBlock / 64; ++w) {
      T s = lds[w];
      lds[w] = run;
      run += s;
    }
    lds[kIsectBlock / 64] = run;
  }
  __syncthreads();
  *total = lds[kIsectBlock / 64];
  return lds[wid] + x - v;
}

// Per-Gaussian tile counts; per-block sums of the counts (block_sums[b]) and
// of the number of Gaussians with at least one tile (vis_sums[b]).
__global__ void __launch_bounds__(kIsectBlock)
isect_count_kernel(int64_t G, const float *__restrict__ means2d, const int32_t *__restrict__ radii,
                   int ts, int tw, int th, int32_t *__restrict__ tiles_per_gauss,
                   int64_t *__restrict__ block_sums, int64_t *__restrict__ vis_sums) {
  __shared__ int64_t lds[kIsectBlock / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * kIsectBlock + threadIdx.x;
  Rect rc;
  int cnt = (i < G) ? tiles_of(means2d, radii, i, ts, tw, th, &rc) : 0;
  if (i < G) tiles_per_gauss[i] = cnt;
  int64_t tot, vtot;
  block_exclusive_scan<int64_t>((int64_t)cnt, lds, &tot);
  __syncthreads();
  block_exclusive_scan<int64_t>((int64_t)(cnt > 0), lds, &vtot);
  if (threadIdx.x == 0) {
    block_sums[blockIdx.x] = tot;
    vis_sums[blockIdx.x] = vtot;
  }
}

// Exclusive scan of the per-block sums in place; total -> block_sums[nb] (and
// -> totals[blockIdx.x] when totals is non-null).  One 1024-lane workgroup per
// array walks its (at most a few thousand) block sums: workgroup 0 scans
// `first`, workgroup 1 (if launched) `second`.  Each lane takes kScanK
// consecutive sums per round with all its loads in flight (a round of 8192
// covers M2's 3930 blocks: one load latency instead of one per 1024).
constexpr int kScanK = 8;
__global__ void __launch_bounds__(1024) isect_scan_blocks_kernel(int64_t nb, int64_t *first,
                                                                 int64_t *second,
                                                                 int64_t *totals) {
  int64_t *block_sums = blockIdx.x == 0 ? first : second;
  __shared__ int64_t wave_tot[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t carry = 0;  // identical in every lane
  for (int64_t base = 0; base < nb; base += 1024 * kScanK) {
    const int64_t i0 = base + (int64_t)threadIdx.x * kScanK;
    int64_t v[kScanK], s = 0;
#pragma unroll
    for (int k = 0; k < kScanK; ++k) v[k] = (i0 + k < nb) ? block_sums[i0 + k] : 0;
#pragma unroll
    for (int k = 0; k < kScanK; ++k) s += v[k];
    int64_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wave_tot[wid] = x;
    __syncthreads();
    int64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      before += w < wid ? wave_tot[w] : 0;
      all += wave_tot[w];
    }
    int64_t run = carry + before + x - s;
#pragma unroll
    for (int k = 0; k < kScanK; ++k) {
      if (i0 + k < nb) block_sums[i0 + k] = run;
      run += v[k];
    }
    carry += all;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    block_sums[nb] = carry;
    if (totals) totals[blockIdx.x] = carry;
  }
}

__global__ void __launch_bounds__(kIsectBlock)
isect_write_kernel(int64_t G, int N, const float *__restrict__ means2d,
                   const int32_t *__restrict__ radii, const float *__restrict__ depths,
                   const int32_t *__restrict__ camera_ids, int ts, int tw, int th, int tile_bits,
                   const int64_t *__restrict__ block_prefix, int64_t *__restrict__ isect_ids,
                   int32_t *__restrict__ flatten_ids) {
  __shared__ int64_t lds[kIsectBlock / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * kIsectBlock + threadIdx.x;
  Rect rc{0, 0, 0, 0};
  const int cnt = (i < G) ? tiles_of(means2d, radii, i, ts, tw, th, &rc) : 0;
  int64_t tot;
  const int64_t local = block_exclusive_scan<int64_t>((int64_t)cnt, lds, &tot);
  if (cnt == 0) return;
  int64_t cur = block_prefix[blockIdx.x] + local;
  const int64_t cam = camera_ids ? (int64_t)camera_ids[i] : (i / N);
  const int64_t hi = cam << (32 + tile_bits);
  // sign-extended bitcast of the depth, as the reference (isect_tiles.py:223)
  const int64_t dbits = (int64_t)__float_as_int(depths[i]);
  const int32_t fid = (int32_t)i;
  for (int y = rc.y0; y < rc.y1; ++y) {
    for (int x = rc.x0; x < rc.x1; ++x) {
      const int64_t tile = (int64_t)(y * tw + x);
      isect_ids[cur] = hi | (tile << 32) | dbits;
      flatten_ids[cur] = fid;
      ++cur;
    }
  }
}

// One lane per sorted isect: fill offsets for the (cam, tile) keys between
// the previous key and this one (CUDA-style fill; Triton tile-bit layout).
__global__ void __launch_bounds__(256)
isect_offsets_kernel(int64_t n, const int64_t *__restrict__ n_dev,
                     const int64_t *__restrict__ isect_ids, int n_tiles_total, int n_tiles,
                     int tile_bits, int32_t *__restrict__ offsets) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n_dev) {  // capacity mode: the grid covers max(capacity, tiles)
    n = min(n, *n_dev);
    if (n == 0) {
      if (i < n_tiles_total) offsets[i] = 0;
      return;
    }
  }
  if (i >= n) return;
  const int64_t tmask = (tile_bits >= 63) ? -1 : ((int64_t)1 << tile_bits) - 1;
  auto key_of = [&](int64_t id) -> int64_t {
    // ids of negative-depth isects are sign-extended (all upper bits set, as
    // the reference, isect_tiles.py:223); they sort past every real tile
    if (id < 0) return n_tiles_total;
    const int64_t k = id >> 32;
    const int64_t key = (k >> tile_bits) * n_tiles + (k & tmask);
    return key < n_tiles_total ? key : n_tiles_total;
  };
  const int64_t cur = key_of(isect_ids[i]);
  if (i == 0) {
    for (int64_t t = 0; t <= cur && t < n_tiles_total; ++t) offsets[t] = 0;
  } else {
    const int64_t prev = key_of(isect_ids[i - 1]);
    if (prev != cur)
      for (int64_t t = prev + 1; t <= cur && t < n_tiles_total; ++t) offsets[t] = (int32_t)i;
  }
  if (i == n - 1)
    for (int64_t t = cur + 1; t < n_tiles_total; ++t) offsets[t] = (int32_t)n;
}


// ---------------------------------------------------------------------------
// Depth-first sorted emission (sort=True).  The reference's stable sort of
// (cam | tile | depth) keys, restricted to one (cam, tile), orders isects by
// depth bits and then by Gaussian index.  The same order results from
//   (1) a stable sort of the visible Gaussians by depth bits (|V| ~ 0.3 N),
//   (2) emitting every Gaussian's tiles in that order, and
//   (3) a stable sort of the emitted isects by the (cam, tile) bits only
//       (tile_bits + cam_bits, e.g. 13 bits at 1080p instead of 45).
// Negative depths (near_plane <= 0) follow the reference's sign extension:
// their (cam, tile) field becomes all ones.

// Capacity check of the sync-free isect (see isect_capacity_kernel).
struct CapCheck {
  const int64_t *totals;  // (n_isects, n_visible) of gsplat_hip_isect_count
  int64_t capacity;
  int64_t *cap_state;     // [4], the caller's counts buffer
  int32_t *status;        // sticky overflow flag or null
  // the same four counts also into row *slot of a host-mapped ring (the
  // captured step's overflow check reads them there, no copy); or null
  int64_t *host_ring;
  const int64_t *slot;
};

GS_INLINE void cap_check(const CapCheck &cc) {
  const int64_t n = cc.totals[0];
  const bool over = n > cc.capacity;
  cc.cap_state[0] = over ? 0 : n;
  cc.cap_state[1] = cc.totals[1];
  cc.cap_state[2] = over ? 1 : 0;
  cc.cap_state[3] = n;
  if (over && cc.status) cc.status[0] |= 1;
  if (cc.host_ring) {
    int64_t *h = cc.host_ring + 4 * (*cc.slot);
    h[0] = over ? 0 : n;
    h[1] = cc.totals[1];
    h[2] = over ? 1 : 0;
    h[3] = n;
  }
}

// (1a) compact the Gaussians with tiles, in index order, with their depth bits.
// Capacity mode: workgroup 0 also writes the capacity state (one launch less;
// every reader of it runs after this kernel).
__global__ void __launch_bounds__(kIsectBlock)
isect_compact_kernel(int64_t G, const int32_t *__restrict__ tiles_per_gauss,
                     const float *__restrict__ depths, const int64_t *__restrict__ vis_prefix,
                     int32_t *__restrict__ V, uint32_t *__restrict__ dkey, CapCheck cc) {
  __shared__ int64_t lds[kIsectBlock / 64 + 1];
  if (cc.cap_state && blockIdx.x == 0 && threadIdx.x == 0) cap_check(cc);
  const int64_t i = (int64_t)blockIdx.x * kIsectBlock + threadIdx.x;
  const int on = (i < G) && tiles_per_gauss[i] > 0;
  int64_t tot;
  const int64_t local = block_exclusive_scan<int64_t>((int64_t)on, lds, &tot);
  if (!on) return;
  const int64_t s = vis_prefix[blockIdx.x] + local;
  V[s] = (int32_t)i;
  dkey[s] = __float_as_uint(depths[i]);
}

// (2a) per-block sums of the tile counts in depth order
__global__ void __launch_bounds__(kIsectBlock)
isect_sorted_count_kernel(int64_t nV, const int64_t *__restrict__ nV_dev,
                          const int32_t *__restrict__ Vs,
                          const int32_t *__restrict__ tiles_per_gauss,
                          int64_t *__restrict__ block_sums, int32_t *__restrict__ n_big) {
  __shared__ int64_t lds[kIsectBlock / 64 + 1];
  if (nV_dev) nV = min(nV, *nV_dev);
  if (blockIdx.x == 0 && threadIdx.x == 0) *n_big = 0;  // big list of the emit kernel
  const int64_t s = (int64_t)blockIdx.x * kIsectBlock + threadIdx.x;
  const int cnt = (s < nV) ? tiles_per_gauss[Vs[s]] : 0;
  int64_t tot;
  block_exclusive_scan<int64_t>((int64_t)cnt, lds, &tot);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

// (2b) emit (cam|tile key, Gaussian index) in depth order.  A Gaussian with
// at most kLaneTiles tiles is written by its own lane; a larger one by its
// whole wave (lanes stride over its tiles, coalesced stores); one with more
// than kGridTiles (near-camera or near-degenerate 2DGS surfels cover the
// whole image) goes to a list that isect_big_emit_kernel spreads over the
// whole grid -- adjacent in depth order, such Gaussians would otherwise
// serialise a few waves for hundreds of thousands of stores.
constexpr int kLaneTiles = 32;
constexpr int kGridTiles = 1024;

struct BigEmit {
  int64_t cur;  // first output slot
  int32_t i, n, x0, y0, w;
  uint32_t hi;
};

__global__ void __launch_bounds__(kIsectBlock)
isect_sorted_emit_kernel(int64_t nV, int N, const int32_t *__restrict__ Vs,
                         const float *__restrict__ means2d, const int32_t *__restrict__ radii,
                         const float *__restrict__ depths, const int32_t *__restrict__ camera_ids,
                         int ts, int tw, int th, int tile_bits, uint32_t key_all_ones,
                         const int64_t *__restrict__ block_prefix, uint32_t *__restrict__ tkey,
                         int32_t *__restrict__ val, BigEmit *__restrict__ big_list,
                         int32_t *__restrict__ n_big, const int64_t *__restrict__ cap_state) {
  __shared__ int64_t lds[kIsectBlock / 64 + 1];
  // capacity mode: cap_state = {n_isects if it fits else 0, n_visible,
  // overflow of this call}; nothing is written past the arrays on overflow
  if (cap_state) {
    if (cap_state[2]) return;
    nV = min(nV, cap_state[1]);
  }
  const int64_t s = (int64_t)blockIdx.x * kIsectBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  Rect rc{0, 0, 0, 0};
  int32_t i = 0;
  int cnt = 0;
  if (s < nV) {
    i = Vs[s];
    cnt = tiles_of(means2d, radii, i, ts, tw, th, &rc);
  }
  int64_t tot;
  const int64_t local = block_exclusive_scan<int64_t>((int64_t)cnt, lds, &tot);
  const int64_t cur0 = block_prefix[blockIdx.x] + local;
  uint32_t hi = key_all_ones;  // all ones: negative depth (every tile gets the all-ones key)
  if (cnt > 0 && __float_as_int(depths[i]) >= 0)
    hi = (camera_ids ? (uint32_t)camera_ids[i] : (uint32_t)(i / N)) << tile_bits;
  if (cnt > 0 && cnt <= kLaneTiles) {
    int64_t cur = cur0;
    for (int y = rc.y0; y < rc.y1; ++y)
      for (int x = rc.x0; x < rc.x1; ++x) {
        tkey[cur] = hi == key_all_ones ? key_all_ones : (hi | (uint32_t)(y * tw + x));
        val[cur] = i;
        ++cur;
      }
  }
  // (a wave-cooperative expansion of these runs -- coalesced stores -- measured
  // no faster: 35.1 vs 34-38 us at M2)
  // huge: one slot per lane in the big list (one atomic per wave)
  const uint64_t huge = __ballot(cnt > kGridTiles);
  if (huge) {
    int base = 0;
    if (lane == 0) base = atomicAdd(n_big, __popcll(huge));
    base = __shfl(base, 0, 64);
    if (cnt > kGridTiles) {
      BigEmit e;
      e.cur = cur0;
      e.i = i;
      e.n = cnt;
      e.x0 = rc.x0;
      e.y0 = rc.y0;
      e.w = rc.x1 - rc.x0;
      e.hi = hi;
      big_list[base + ballot_slot(huge)] = e;
    }
  }
  uint64_t big = __ballot(cnt > kLaneTiles && cnt <= kGridTiles);
  while (big) {
    const int src = __builtin_ctzll(big);
    big &= big - 1;
    const int64_t c0 = __shfl(cur0, src, 64);
    const int n = __shfl(cnt, src, 64);
    const int gx0 = __shfl(rc.x0, src, 64), gy0 = __shfl(rc.y0, src, 64);
    const uint32_t w = (uint32_t)(__shfl(rc.x1, src, 64) - gx0);
    const uint32_t ghi = __shfl(hi, src, 64);
    const int32_t gi = __shfl(i, src, 64);
    for (int k = lane; k < n; k += 64) {
      const uint32_t yy = (uint32_t)k / w, xx = (uint32_t)k - yy * w;
      const uint32_t tile = (uint32_t)((gy0 + (int)yy) * tw + gx0 + (int)xx);
      tkey[c0 + k] = ghi == key_all_ones ? key_all_ones : (ghi | tile);
      val[c0 + k] = gi;
    }
  }
}

// (2c) the huge Gaussians of the list: kBigParts workgroups per Gaussian,
// each writing a contiguous 1/kBigParts of its tiles (coalesced).
constexpr int kBigParts = 16;
constexpr int kBigBlocks = 4096;

__global__ void __launch_bounds__(256)
isect_big_emit_kernel(const BigEmit *__restrict__ big_list, const int32_t *__restrict__ n_big,
                      int tw, uint32_t key_all_ones, uint32_t *__restrict__ tkey,
                      int32_t *__restrict__ val) {
  const int nb = *n_big;
  const int part = blockIdx.x % kBigParts;
  for (int e = blockIdx.x / kBigParts; e < nb; e += kBigBlocks / kBigParts) {
    const BigEmit g = big_list[e];
    const int k0 = (int)(((int64_t)g.n * part) / kBigParts);
    const int k1 = (int)(((int64_t)g.n * (part + 1)) / kBigParts);
    const uint32_t w = (uint32_t)g.w;
    for (int k = k0 + threadIdx.x; k < k1; k += 256) {
      const uint32_t yy = (uint32_t)k / w, xx = (uint32_t)k - yy * w;
      const uint32_t tile = (uint32_t)((g.y0 + (int)yy) * tw + g.x0 + (int)xx);
      tkey[g.cur + k] = g.hi == key_all_ones ? key_all_ones : (g.hi | tile);
      val[g.cur + k] = g.i;
    }
  }
}

// (3b) assemble the reference's 64-bit ids from the sorted (key, Gaussian)
__global__ void __launch_bounds__(256)
isect_sorted_finalize_kernel(int64_t n, const int64_t *__restrict__ n_dev,
                             const uint32_t *__restrict__ tkey,
                             const int32_t *__restrict__ val, const float *__restrict__ depths,
                             int64_t *__restrict__ isect_ids, int32_t *__restrict__ flatten_ids) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n_dev) n = min(n, *n_dev);
  if (p >= n) return;
  const int32_t i = val[p];
  const int32_t db = __float_as_int(depths[i]);
  isect_ids[p] = db < 0 ? (int64_t)db : (((int64_t)tkey[p] << 32) | (int64_t)(uint32_t)db);
  flatten_ids[p] = i;
}

// Capacity check of the sync-free isect: cap_state = {n_isects if it fits
// in `capacity` else 0, n_visible, 1 if it did not fit, n_isects}; status[0] |= 1 on
// overflow (sticky: the training step's state updates read it and become
// no-ops until the host has grown the arrays and cleared it).
__global__ void isect_capacity_kernel(CapCheck cc) {
  if (threadIdx.x == 0) cap_check(cc);
}

}  // namespace gs

using namespace gs;

// count workspace: [0, nb] scanned isect block sums (+ total), [nb+1, 2nb+1]
// scanned visible-Gaussian block sums (+ total).
extern "C" int64_t gsplat_hip_isect_workspace_bytes(int64_t n_gaussians) {
  const int64_t nb = (n_gaussians + kIsectBlock - 1) / kIsectBlock;
  return (2 * nb + 2) * (int64_t)sizeof(int64_t);
}

extern "C" int gsplat_hip_isect_count(int64_t n_gaussians, const float *means2d,
                                      const int32_t *radii, int tile_size, int tile_width,
                                      int tile_height, int32_t *tiles_per_gauss,
                                      void *workspace, int64_t *totals_device, void *stream) {
  GS_REQUIRE(n_gaussians >= 0 && tile_size > 0, "isect_count: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  int64_t *ws = reinterpret_cast<int64_t *>(workspace);
  const int64_t nb = (n_gaussians + kIsectBlock - 1) / kIsectBlock;
  if (nb == 0) {
    GS_HIP(gs::zero_async(totals_device, 2 * sizeof(int64_t), st));
    return 0;
  }
  int64_t *vis = ws + nb + 1;
  hipLaunchKernelGGL(isect_count_kernel, dim3((unsigned)nb), dim3(kIsectBlock), 0, st,
                     n_gaussians, means2d, radii, tile_size, tile_width, tile_height,
                     tiles_per_gauss, ws, vis);
  // both scans in one launch; their totals are (n_isects, n_visible)
  hipLaunchKernelGGL(isect_scan_blocks_kernel, dim3(2), dim3(1024), 0, st, nb, ws, vis,
                     totals_device);
  GS_CHECK_LAUNCH("isect_count");
  return 0;
}

extern "C" int gsplat_hip_isect_write(int64_t n_gaussians, int N, const float *means2d,
                                      const int32_t *radii, const float *depths,
                                      const int32_t *camera_ids, int tile_size, int tile_width,
                                      int tile_height, int tile_bits, const void *workspace,
                                      int64_t *isect_ids, int32_t *flatten_ids, void *stream) {
  GS_REQUIRE(n_gaussians >= 0 && (camera_ids || N > 0 || n_gaussians == 0),
             "isect_write: N must be > 0 when camera_ids is null");
  const int64_t nb = (n_gaussians + kIsectBlock - 1) / kIsectBlock;
  if (nb == 0) return 0;
  hipLaunchKernelGGL(isect_write_kernel, dim3((unsigned)nb), dim3(kIsectBlock), 0,
                     (hipStream_t)stream, n_gaussians, N, means2d, radii, depths, camera_ids,
                     tile_size, tile_width, tile_height, tile_bits,
                     reinterpret_cast<const int64_t *>(workspace), isect_ids, flatten_ids);
  GS_CHECK_LAUNCH("isect_write");
  return 0;
}

extern "C" int64_t gsplat_hip_sort_workspace_bytes(int64_t n) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                            (const int32_t *)nullptr, (int32_t *)nullptr, (size_t)n, 0u, 64u,
                            (hipStream_t)0);
  return (int64_t)bytes;
}

// Stable LSD radix sort of (isect_id, flatten_id) on bits [0, n_bits).
extern "C" int gsplat_hip_radix_sort(int64_t n, int n_bits, const int64_t *keys_in,
                                     const int32_t *vals_in, int64_t *keys_out,
                                     int32_t *vals_out, void *workspace,
                                     int64_t workspace_bytes, void *stream) {
  GS_REQUIRE(n_bits > 0 && n_bits <= 64, "radix_sort: n_bits=%d out of range", n_bits);
  if (n <= 0) return 0;
  size_t bytes = (size_t)workspace_bytes;
  hipError_t e = rocprim::radix_sort_pairs(
      workspace, bytes, reinterpret_cast<const uint64_t *>(keys_in),
      reinterpret_cast<uint64_t *>(keys_out), vals_in, vals_out, (size_t)n, 0u,
      (unsigned)n_bits, (hipStream_t)stream);
  GS_REQUIRE(e == hipSuccess, "radix_sort: %s", hipGetErrorString(e));
  return 0;
}

extern "C" int gsplat_hip_isect_offsets(int64_t n_isects, const int64_t *n_isects_device,
                                        const int64_t *isect_ids, int C, int tile_width,
                                        int tile_height, int32_t *offsets, void *stream) {
  const int n_tiles = tile_width * tile_height;
  hipStream_t st = (hipStream_t)stream;
  if ((int64_t)C * n_tiles == 0) return 0;
  if (n_isects_device) {  // capacity mode: n_isects is the arrays' capacity
    int tile_bits = 0;
    while ((1 << tile_bits) < n_tiles) ++tile_bits;
    const int64_t span = std::max<int64_t>(n_isects, (int64_t)C * n_tiles);
    hipLaunchKernelGGL(isect_offsets_kernel, dim3((unsigned)((span + 255) / 256)), dim3(256), 0,
                       st, n_isects, n_isects_device, isect_ids, C * n_tiles, n_tiles, tile_bits,
                       offsets);
    GS_CHECK_LAUNCH("isect_offsets");
    return 0;
  }
  if (n_isects <= 0) {
    GS_HIP(gs::zero_async(offsets, sizeof(int32_t) * (size_t)C * n_tiles, st));
    return 0;
  }
  int tile_bits = 0;
  while ((1 << tile_bits) < n_tiles) ++tile_bits;  // == (n_tiles - 1).bit_length()
  hipLaunchKernelGGL(isect_offsets_kernel, dim3((unsigned)((n_isects + 255) / 256)), dim3(256), 0,
                     st, n_isects, (const int64_t *)nullptr, isect_ids, C * n_tiles, n_tiles,
                     tile_bits, offsets);
  GS_CHECK_LAUNCH("isect_offsets");
  return 0;
}

// ------------------------------------------------------- depth-first path --
namespace {
struct SortedLayout {
  size_t V, dkey, Vs, dkeys, blk, big, nbig, tkey, val, tkeys, vals, tmp, total;
  size_t tmp_bytes;
  // supertile expansion (isect_st.h)
  size_t rect, st_start, seg_start, seg_st, segcnt, tile_tot, offs;
  int64_t segcap;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

SortedLayout sorted_layout(int64_t nV, int64_t n, int key_bits) {
  (void)key_bits;
  const size_t t1 = lsd_sort_scratch_bytes(nV), t2 = lsd_sort_scratch_bytes(n);
  SortedLayout L{};
  size_t o = 0;
  L.V = o; o = align256(o + 4 * (size_t)nV);
  L.dkey = o; o = align256(o + 4 * (size_t)nV);
  L.Vs = o; o = align256(o + 4 * (size_t)nV);
  L.dkeys = o; o = align256(o + 4 * (size_t)nV);
  L.blk = o; o = align256(o + 8 * (size_t)((nV + kIsectBlock - 1) / kIsectBlock + 2));
  L.big = o; o = align256(o + sizeof(BigEmit) * (size_t)nV);
  L.nbig = o; o = align256(o + 4);
  L.tkey = o; o = align256(o + 4 * (size_t)n);
  L.val = o; o = align256(o + 4 * (size_t)n);
  L.tkeys = o; o = align256(o + 4 * (size_t)n);
  L.vals = o; o = align256(o + 4 * (size_t)n);
  L.tmp = o;
  L.tmp_bytes = t1 > t2 ? t1 : t2;
  o = align256(o + L.tmp_bytes + 1);
  L.segcap = n / st::kSeg + st::kMaxKeys + 1;
  L.rect = o; o = align256(o + 8 * (size_t)nV);
  L.st_start = o; o = align256(o + 4 * (size_t)(st::kMaxKeys + 1));
  L.seg_start = o; o = align256(o + 4 * (size_t)(st::kMaxKeys + 1));
  L.seg_st = o; o = align256(o + 4 * (size_t)L.segcap);
  L.segcnt = o; o = align256(o + 4 * st::S * st::S * (size_t)L.segcap);
  L.tile_tot = o; o = align256(o + 4 * (size_t)(st::kMaxTiles + 1));
  L.offs = o; o = align256(o + 4 * (size_t)st::kMaxTiles);
  L.total = o;
  return L;
}

// The supertile expansion runs for at most kMaxKeys supertiles (with the
// negative-depth one); GSPLAT_HIP_ISECT_ST=0 keeps the emission + tile sort.
bool st_enabled(const st::Geo &g) {
  static const bool on = [] {
    const char *e = getenv("GSPLAT_HIP_ISECT_ST");
    return !(e && atoi(e) == 0);
  }();
  return on && g.nst <= st::kMaxKeys;
}
}  // namespace

extern "C" int64_t gsplat_hip_isect_sorted_workspace_bytes(int64_t n_visible, int64_t n_isects,
                                                           int key_bits) {
  return (int64_t)sorted_layout(n_visible, n_isects, key_bits).total;
}

extern "C" int gsplat_hip_isect_ranked(int n_cameras, int tile_width, int tile_height);

// Sorted isects without sorting 64-bit keys: see "Depth-first sorted emission".
// count_workspace is the gsplat_hip_isect_count workspace (scanned block sums).
// cnt_dev (capacity mode): the {n_isects, n_visible, overflow} state on the
// device; n_visible / n_isects are then the capacities the grids are sized for.
// offsets (may be null): the tile offsets too (gsplat_hip_isect_offsets'
// output, C * tile_width * tile_height int32).
static int isect_write_sorted_impl(
    int64_t n_gaussians, int N, const float *means2d, const int32_t *radii, const float *depths,
    const int32_t *camera_ids, const int32_t *tiles_per_gauss, int tile_size, int tile_width,
    int tile_height, int tile_bits, int cam_bits, const void *count_workspace, int64_t n_visible,
    int64_t n_isects, const int64_t *cnt_dev, void *workspace, int64_t workspace_bytes,
    int64_t *isect_ids, int32_t *flatten_ids, int32_t *offsets, int n_cameras, hipStream_t st,
    CapCheck cc = CapCheck{}, int32_t *rank_ids = nullptr, int32_t *vis_rank = nullptr,
    const st::SurfelCull *sc = nullptr) {
  GS_REQUIRE(n_gaussians >= 0 && (camera_ids || N > 0 || n_gaussians == 0),
             "isect_write_sorted: N must be > 0 when camera_ids is null");
  GS_REQUIRE(tile_bits + cam_bits <= 32, "isect_write_sorted: tile_bits + cam_bits > 32");
  GS_REQUIRE(n_isects < ((int64_t)1 << 30), "isect_write_sorted: more than 2^30 isects");
  GS_REQUIRE(!offsets || n_cameras > 0, "isect_write_sorted: offsets need n_cameras");
  GS_REQUIRE(!rank_ids == !vis_rank, "isect_write_sorted: rank_ids and vis_rank go together");
  GS_REQUIRE(!sc || (cnt_dev && gsplat_hip_isect_ranked(n_cameras, tile_width, tile_height)),
             "isect_write_sorted: tile culling needs the capacity mode and the supertiles");
  GS_REQUIRE(!rank_ids || gsplat_hip_isect_ranked(n_cameras, tile_width, tile_height),
             "isect_write_sorted: rank ids need the supertile expansion");
  // isect_ids / flatten_ids may both be null when rank_ids and offsets are
  // written (a caller that walks the ranks and never reads the ids: the
  // training step) -- 12 of the 16 bytes per isect not written; isect_ids
  // alone may be null when flatten_ids and offsets are (ABI 33: the 2DGS
  // training step, whose rasterizer gathers by Gaussian id) -- 8 of 12.
  // Both forms need the supertile expansion.
  GS_REQUIRE(n_isects <= 0 || (isect_ids && flatten_ids) ||
                 (!isect_ids && !flatten_ids && rank_ids && offsets) ||
                 (!isect_ids && flatten_ids && offsets &&
                  gsplat_hip_isect_ranked(n_cameras, tile_width, tile_height)),
             "isect_write_sorted: null isect_ids need rank_ids or flatten_ids, and offsets");
  auto plain_offsets = [&]() -> int {  // offsets from the written ids (or all zero)
    if (!offsets) return 0;
    if (!isect_ids)  // nothing written (no isect or no visible Gaussian): all zero
      return gs::zero_async(offsets, sizeof(int32_t) * (size_t)n_cameras * tile_width *
                                         tile_height, st) == hipSuccess ? 0 : 2;
    return gsplat_hip_isect_offsets(cnt_dev ? n_isects : (n_visible > 0 ? n_isects : 0), cnt_dev,
                                    isect_ids, n_cameras, tile_width, tile_height, offsets, st);
  };
  if (n_isects <= 0 || n_visible <= 0) return plain_offsets();
  const int key_bits = tile_bits + cam_bits;
  const SortedLayout L = sorted_layout(n_visible, n_isects, key_bits);
  GS_REQUIRE(workspace_bytes >= (int64_t)L.total, "isect_write_sorted: workspace %lld < %lld",
             (long long)workspace_bytes, (long long)L.total);
  char *ws = reinterpret_cast<char *>(workspace);
  int32_t *V = reinterpret_cast<int32_t *>(ws + L.V), *Vs = reinterpret_cast<int32_t *>(ws + L.Vs);
  uint32_t *dkey = reinterpret_cast<uint32_t *>(ws + L.dkey);
  uint32_t *dkeys = reinterpret_cast<uint32_t *>(ws + L.dkeys);
  int64_t *blk = reinterpret_cast<int64_t *>(ws + L.blk);
  uint32_t *tkey = reinterpret_cast<uint32_t *>(ws + L.tkey);
  uint32_t *tkeys = reinterpret_cast<uint32_t *>(ws + L.tkeys);
  int32_t *val = reinterpret_cast<int32_t *>(ws + L.val), *vals = reinterpret_cast<int32_t *>(ws + L.vals);
  void *tmp = ws + L.tmp;

  const int64_t nbG = (n_gaussians + kIsectBlock - 1) / kIsectBlock;
  const int64_t *vis_prefix = reinterpret_cast<const int64_t *>(count_workspace) + nbG + 1;
  hipLaunchKernelGGL(isect_compact_kernel, dim3((unsigned)nbG), dim3(kIsectBlock), 0, st,
                     n_gaussians, tiles_per_gauss, depths, vis_prefix, V, dkey, cc);
  // stable depth sort of the visible Gaussians (32 key bits)
  const uint32_t *dks = dkeys;
  if (lsd_sort_pairs(dkey, V, dkeys, Vs, n_visible, 0, 32, tmp, st, nullptr,
                     cnt_dev ? cnt_dev + 1 : nullptr) == 0) {
    Vs = V;
    dks = dkey;
  }
  const int64_t nbV = (n_visible + kIsectBlock - 1) / kIsectBlock;
  const st::Geo geo = st::make_geo(n_cameras > 0 ? n_cameras : 1, N, tile_width, tile_height,
                                   tile_bits);
  if (gsplat_hip_isect_ranked(n_cameras, tile_width, tile_height)) {
    // supertile expansion (isect_st.h): isects written once, offsets included
    ushort4 *rect = reinterpret_cast<ushort4 *>(ws + L.rect);
    int32_t *st_start = reinterpret_cast<int32_t *>(ws + L.st_start);
    int32_t *seg_start = reinterpret_cast<int32_t *>(ws + L.seg_start);
    int32_t *seg_st = reinterpret_cast<int32_t *>(ws + L.seg_st);
    int32_t *segcnt = reinterpret_cast<int32_t *>(ws + L.segcnt);
    int32_t *tile_tot = reinterpret_cast<int32_t *>(ws + L.tile_tot);
    int32_t *offs = offsets ? offsets : reinterpret_cast<int32_t *>(ws + L.offs);
    // the captured 2DGS step (sc): huge surfels' pairs spread over the grid
    static_assert(sizeof(st::HugeEmit) <= sizeof(BigEmit), "the huge list fits L.big");
    st::HugeEmit *huge_list = sc ? reinterpret_cast<st::HugeEmit *>(ws + L.big) : nullptr;
    int32_t *n_huge = sc ? reinterpret_cast<int32_t *>(ws + L.nbig) : nullptr;
    hipLaunchKernelGGL(st::rect_kernel, dim3((unsigned)nbV), dim3(256), 0, st, n_visible, cnt_dev,
                       Vs, dks, means2d, radii, tile_size, geo, rect, blk, vis_rank, n_huge);
    hipLaunchKernelGGL(isect_scan_blocks_kernel, dim3(1), dim3(1024), 0, st, nbV, blk, nullptr,
                       nullptr);
    hipLaunchKernelGGL(st::emit_kernel, dim3((unsigned)nbV), dim3(256), 0, st, n_visible, cnt_dev,
                       Vs, dks, rect, camera_ids, geo, blk, tkey, val, huge_list, n_huge);
    if (sc)
      hipLaunchKernelGGL(st::huge_emit_kernel, dim3(st::kHugeBlocks), dim3(256), 0, st, huge_list,
                         n_huge, geo, tkey, val);
    if (sc)  // large surfels' pairs: the tiles of the supertile they can reach
      hipLaunchKernelGGL(st::tight_kernel,
                         dim3((unsigned)std::min<int64_t>((n_isects + 255) / 256, 2048)),
                         dim3(256), 0, st, n_isects, blk + nbV, geo, Vs, rect, cnt_dev, tkey, val,
                         *sc);
    int kb = 0;
    while ((1 << kb) < geo.nst) ++kb;
    // the pair count (<= n_isects) is the scan's total, blk[nbV]
    const uint32_t *totals = lsd_one_pass(tkey, val, tkeys, vals, n_isects, kb < 1 ? 1 : kb, tmp,
                                          st, blk + nbV);
    const int n_tt = geo.C * geo.n_tiles + 1;
    hipLaunchKernelGGL(st::plan_kernel, dim3(1), dim3(1024), 0, st, geo.nst, totals, st_start,
                       seg_start, seg_st, n_tt, tile_tot);
    const unsigned nseg = (unsigned)(n_isects / st::kSeg + geo.nst + 1);
    const uint32_t *pk = sc ? tkeys : nullptr;  // the culled pairs' kept tiles
    hipLaunchKernelGGL(st::seg_count_kernel, dim3(nseg), dim3(256), 0, st, geo, st_start,
                       seg_start, seg_st, vals, rect, Vs, tiles_per_gauss, segcnt, tile_tot, pk);
    hipLaunchKernelGGL(st::tile_scan_kernel, dim3(1), dim3(1024), 0, st, geo, cnt_dev, tile_tot,
                       offs, sc ? const_cast<int64_t *>(cnt_dev) : nullptr);
    hipLaunchKernelGGL(st::seg_write_kernel, dim3(nseg), dim3(256), 0, st, geo, cnt_dev, st_start,
                       seg_start, seg_st, vals, rect, Vs, dks, tiles_per_gauss, segcnt, tile_tot,
                       isect_ids, flatten_ids, rank_ids, pk);
    GS_CHECK_LAUNCH("isect_write_sorted (supertiles)");
    return 0;
  }
  BigEmit *big_list = reinterpret_cast<BigEmit *>(ws + L.big);
  int32_t *n_big = reinterpret_cast<int32_t *>(ws + L.nbig);
  hipLaunchKernelGGL(isect_sorted_count_kernel, dim3((unsigned)nbV), dim3(kIsectBlock), 0, st,
                     n_visible, cnt_dev ? cnt_dev + 1 : nullptr, Vs, tiles_per_gauss, blk, n_big);
  hipLaunchKernelGGL(isect_scan_blocks_kernel, dim3(1), dim3(1024), 0, st, nbV, blk, nullptr,
                     nullptr);
  const uint32_t all_ones = key_bits >= 32 ? 0xffffffffu : ((1u << key_bits) - 1u);
  hipLaunchKernelGGL(isect_sorted_emit_kernel, dim3((unsigned)nbV), dim3(kIsectBlock), 0, st,
                     n_visible, N, Vs, means2d, radii, depths, camera_ids, tile_size, tile_width,
                     tile_height, tile_bits, all_ones, blk, tkey, val, big_list, n_big, cnt_dev);
  hipLaunchKernelGGL(isect_big_emit_kernel, dim3(kBigBlocks), dim3(256), 0, st, big_list, n_big,
                     tile_width, all_ones, tkey, val);
  // stable (camera, tile) sort keeps the depth order inside every tile; its
  // last pass writes isect_ids / flatten_ids directly
  if (key_bits > 0) {
    const lsd::FinalOut fo{depths, isect_ids, flatten_ids};
    lsd_sort_pairs(tkey, val, tkeys, vals, n_isects, 0, key_bits, tmp, st, &fo, cnt_dev);
  } else {
    hipLaunchKernelGGL(isect_sorted_finalize_kernel, dim3((unsigned)((n_isects + 255) / 256)),
                       dim3(256), 0, st, n_isects, cnt_dev, tkey, val, depths, isect_ids,
                       flatten_ids);
  }
  GS_CHECK_LAUNCH("isect_write_sorted");
  return plain_offsets();
}

extern "C" int gsplat_hip_isect_write_sorted(
    int64_t n_gaussians, int N, const float *means2d, const int32_t *radii, const float *depths,
    const int32_t *camera_ids, const int32_t *tiles_per_gauss, int tile_size, int tile_width,
    int tile_height, int tile_bits, int cam_bits, const void *count_workspace, int64_t n_visible,
    int64_t n_isects, void *workspace, int64_t workspace_bytes, int64_t *isect_ids,
    int32_t *flatten_ids, int n_cameras, int32_t *offsets, int32_t *rank_ids, int32_t *vis_rank,
    void *stream) {
  return isect_write_sorted_impl(n_gaussians, N, means2d, radii, depths, camera_ids,
                                 tiles_per_gauss, tile_size, tile_width, tile_height, tile_bits,
                                 cam_bits, count_workspace, n_visible, n_isects, nullptr,
                                 workspace, workspace_bytes, isect_ids, flatten_ids, offsets,
                                 n_cameras, (hipStream_t)stream, CapCheck{}, rank_ids, vis_rank);
}

// Whether gsplat_hip_isect_write_sorted(_capped) with these dimensions (and
// offsets) runs the supertile expansion -- the path that can write rank ids.
extern "C" int gsplat_hip_isect_ranked(int n_cameras, int tile_width, int tile_height) {
  if (n_cameras <= 0 || tile_width <= 0 || tile_height <= 0) return 0;
  const st::Geo geo = st::make_geo(n_cameras, 1, tile_width, tile_height, 0);
  return ((int64_t)n_cameras * tile_width * tile_height <= st::kMaxTiles && st_enabled(geo)) ? 1
                                                                                              : 0;
}

extern "C" int64_t gsplat_hip_isect_sorted_capped_workspace_bytes(int64_t n_gaussians,
                                                                  int64_t capacity, int key_bits) {
  // the visible Gaussians are at most n_gaussians; + the capacity state
  return (int64_t)sorted_layout(n_gaussians, capacity, key_bits).total + 256;
}

// The sorted emission without a host sync: the counts stay on the device
// (totals_device from gsplat_hip_isect_count), isect_ids / flatten_ids have
// `capacity` slots and every grid is sized for it.  counts_device[0] receives
// the number of isects written (0 when they did not fit: status_device[0]
// gets bit 0 set, sticky), counts_device[1] the visible Gaussians; pass
// counts_device to offsets / rasterize as their n_isects_device.
static int isect_write_sorted_capped_impl(
    int64_t n_gaussians, int N, const float *means2d, const int32_t *radii, const float *depths,
    const int32_t *camera_ids, const int32_t *tiles_per_gauss, int tile_size, int tile_width,
    int tile_height, int tile_bits, int cam_bits, const void *count_workspace,
    const int64_t *totals_device, int64_t capacity, int64_t *counts_device,
    int32_t *status_device, int64_t *counts_host_ring, const int64_t *slot_device,
    void *workspace, int64_t workspace_bytes, int64_t *isect_ids, int32_t *flatten_ids,
    int n_cameras, int32_t *offsets, int32_t *rank_ids, int32_t *vis_rank, void *stream,
    const st::SurfelCull *sc) {
  GS_REQUIRE(capacity >= 0 && capacity < ((int64_t)1 << 30),
             "isect_write_sorted_capped: capacity %lld out of range", (long long)capacity);
  GS_REQUIRE(counts_device && totals_device, "isect_write_sorted_capped: null count buffers");
  GS_REQUIRE(!counts_host_ring == !slot_device,
             "isect_write_sorted_capped: counts_host_ring and slot_device go together");
  const int64_t need = gsplat_hip_isect_sorted_capped_workspace_bytes(n_gaussians, capacity,
                                                                      tile_bits + cam_bits);
  GS_REQUIRE(workspace_bytes >= need, "isect_write_sorted_capped: workspace %lld < %lld",
             (long long)workspace_bytes, (long long)need);
  hipStream_t st = (hipStream_t)stream;
  // cap_state [4] lives in the caller's counts buffer; the compact kernel
  // writes it, or this one when the emission launches nothing
  const CapCheck cc{totals_device, capacity, counts_device, status_device, counts_host_ring,
                    slot_device};
  if (capacity <= 0 || n_gaussians <= 0) {
    hipLaunchKernelGGL(isect_capacity_kernel, dim3(1), dim3(64), 0, st, cc);
    GS_CHECK_LAUNCH("isect_write_sorted_capped");
  }
  return isect_write_sorted_impl(n_gaussians, N, means2d, radii, depths, camera_ids,
                                 tiles_per_gauss, tile_size, tile_width, tile_height, tile_bits,
                                 cam_bits, count_workspace, n_gaussians, capacity, counts_device,
                                 workspace, workspace_bytes - 256, isect_ids, flatten_ids, offsets,
                                 n_cameras, st, cc, rank_ids, vis_rank, sc);
}

extern "C" int gsplat_hip_isect_write_sorted_capped(
    int64_t n_gaussians, int N, const float *means2d, const int32_t *radii, const float *depths,
    const int32_t *camera_ids, const int32_t *tiles_per_gauss, int tile_size, int tile_width,
    int tile_height, int tile_bits, int cam_bits, const void *count_workspace,
    const int64_t *totals_device, int64_t capacity, int64_t *counts_device,
    int32_t *status_device, int64_t *counts_host_ring, const int64_t *slot_device,
    void *workspace, int64_t workspace_bytes, int64_t *isect_ids, int32_t *flatten_ids,
    int n_cameras, int32_t *offsets, int32_t *rank_ids, int32_t *vis_rank, void *stream) {
  return isect_write_sorted_capped_impl(
      n_gaussians, N, means2d, radii, depths, camera_ids, tiles_per_gauss, tile_size, tile_width,
      tile_height, tile_bits, cam_bits, count_workspace, totals_device, capacity, counts_device,
      status_device, counts_host_ring, slot_device, workspace, workspace_bytes, isect_ids,
      flatten_ids, n_cameras, offsets, rank_ids, vis_rank, stream, nullptr);
}

extern "C" int gsplat_hip_isect_write_sorted_capped_surfel(
    int64_t n_gaussians, int N, const float *means2d, const int32_t *radii, const float *depths,
    const int32_t *camera_ids, const int32_t *tiles_per_gauss, int tile_size, int tile_width,
    int tile_height, int tile_bits, int cam_bits, const void *count_workspace,
    const int64_t *totals_device, int64_t capacity, int64_t *counts_device,
    int32_t *status_device, int64_t *counts_host_ring, const int64_t *slot_device,
    void *workspace, int64_t workspace_bytes, int32_t *flatten_ids, int n_cameras,
    int32_t *offsets, const float *ray_transforms, const float *opacities, void *stream) {
  GS_REQUIRE(means2d && ray_transforms && opacities && flatten_ids && offsets && !camera_ids,
             "isect_write_sorted_capped_surfel: null argument (or packed camera ids)");
  const st::SurfelCull sc{means2d, ray_transforms, opacities, tile_size};
  return isect_write_sorted_capped_impl(
      n_gaussians, N, means2d, radii, depths, camera_ids, tiles_per_gauss, tile_size, tile_width,
      tile_height, tile_bits, cam_bits, count_workspace, totals_device, capacity, counts_device,
      status_device, counts_host_ring, slot_device, workspace, workspace_bytes, nullptr,
      flatten_ids, n_cameras, offsets, nullptr, nullptr, stream, &sc);
}

// -------------------------------------------------------- tile-first path --
// Sorted isects with two 32-bit sorts and no depth sort of the Gaussians:
// (1) emission in Gaussian-major order with 32-bit (camera, tile) keys,
// (2) a stable radix sort by those keys (tile_bits + cam_bits bits), which
//     keeps Gaussian-index order inside every (camera, tile),
// (3) a segmented radix sort of each (camera, tile) run by the depth bits
//     (stable: equal depths stay in Gaussian-index order).
// The result is the reference's stable sort of (cam | tile | depth) keys
// element for element.  Negative depths: all-ones (camera, tile) key, and
// unsigned depth order inside that run, exactly as the reference's masked
// 64-bit keys.
namespace gs {

__global__ void __launch_bounds__(kIsectBlock)
isect_write_tiles_kernel(int64_t G, int N, const float *__restrict__ means2d,
                         const int32_t *__restrict__ radii, const float *__restrict__ depths,
                         const int32_t *__restrict__ camera_ids, int ts, int tw, int th,
                         int tile_bits, uint32_t key_all_ones,
                         const int64_t *__restrict__ block_prefix, uint32_t *__restrict__ tkey,
                         int32_t *__restrict__ val) {
  __shared__ int64_t lds[kIsectBlock / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * kIsectBlock + threadIdx.x;
  Rect rc{0, 0, 0, 0};
  const int cnt = (i < G) ? tiles_of(means2d, radii, i, ts, tw, th, &rc) : 0;
  int64_t tot;
  const int64_t local = block_exclusive_scan<int64_t>((int64_t)cnt, lds, &tot);
  if (cnt == 0) return;
  int64_t cur = block_prefix[blockIdx.x] + local;
  const uint32_t cam = camera_ids ? (uint32_t)camera_ids[i] : (uint32_t)(i / N);
  const bool neg = __float_as_int(depths[i]) < 0;
  for (int y = rc.y0; y < rc.y1; ++y) {
    for (int x = rc.x0; x < rc.x1; ++x) {
      tkey[cur] = neg ? key_all_ones : ((cam << tile_bits) | (uint32_t)(y * tw + x));
      val[cur] = (int32_t)i;
      ++cur;
    }
  }
}

// starts[t] = first sorted isect with (camera, tile) key index >= t, for
// t in [0, n_total]; starts[n_total + 1] = n.  Keys outside the grid (the
// all-ones key when it is not a real tile) form the last run.
__global__ void __launch_bounds__(256)
isect_key_starts_kernel(int64_t n, const uint32_t *__restrict__ tkey, int n_total, int n_tiles,
                        int tile_bits, int32_t *__restrict__ starts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t tmask = (1u << tile_bits) - 1u;
  auto idx_of = [&](uint32_t k) -> int64_t {
    const int64_t t = (int64_t)(k >> tile_bits) * n_tiles + (k & tmask);
    return t < n_total ? t : n_total;
  };
  const int64_t cur = idx_of(tkey[i]);
  if (i == 0) {
    for (int64_t t = 0; t <= cur; ++t) starts[t] = 0;
  } else {
    const int64_t prev = idx_of(tkey[i - 1]);
    for (int64_t t = prev + 1; t <= cur; ++t) starts[t] = (int32_t)i;
  }
  if (i == n - 1) {
    for (int64_t t = cur + 1; t <= n_total; ++t) starts[t] = (int32_t)n;
    starts[n_total + 1] = (int32_t)n;
  }
}

// Depth order inside every (camera, tile) run, and the final 64-bit ids.
// A run (Gaussian-index order after the stable key sort) is sorted stably by
// depth bits and written out as isect_ids / flatten_ids.
//   isect_tile_sort_small_kernel: one 256-lane workgroup per run, rocPRIM
//     block radix sort in LDS for runs up to kSmallCap; longer runs are
//     appended to a list;
//   isect_tile_sort_large_kernel: one 1024-lane workgroup per listed run,
//     block radix sort up to kLargeCap, beyond that a bitonic sort of unique
//     (depth bits, position) keys in a private global scratch region
//     (pathological scenes).
constexpr int kSmallCap = 4096;
constexpr int kLargeCap = 16384;

template <int NT>
__device__ __forceinline__ void bitonic_sort(uint64_t *k, int P) {
  for (int kk = 2; kk <= P; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t a = k[i], b = k[ixj];
          if ((a > b) == ((i & kk) == 0)) {
            k[i] = b;
            k[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

// One run of m <= NT * IPT isects with rocPRIM's block radix sort (LSD,
// stable): keys = depth bits, values = positions in the run (Gaussian-index
// order), blocked arrangement -- so equal depths keep Gaussian order.
template <int NT, int IPT, class Storage>
__device__ __forceinline__ void run_radix_sort(Storage &storage, int64_t b, int m, uint32_t key32,
                                               const int32_t *__restrict__ val,
                                               const float *__restrict__ depths,
                                               int64_t *__restrict__ isect_ids,
                                               int32_t *__restrict__ flatten_ids) {
  using BRS = rocprim::block_radix_sort<uint32_t, NT, IPT, int32_t, 1, 1, 8>;  // 8-bit passes
  uint32_t key[IPT];
  int32_t pos[IPT], g[IPT];
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int i = threadIdx.x * IPT + e;
    g[e] = i < m ? val[b + i] : 0;
  }
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int i = threadIdx.x * IPT + e;
    key[e] = i < m ? __float_as_uint(depths[g[e]]) : 0xffffffffu;
    pos[e] = i;
  }
  BRS().sort(key, pos, reinterpret_cast<typename BRS::storage_type &>(storage));
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int i = threadIdx.x * IPT + e;
    if (i < m) {
      const int32_t db = (int32_t)key[e];
      isect_ids[b + i] = db < 0 ? (int64_t)db : (((int64_t)key32 << 32) | (int64_t)(uint32_t)db);
      flatten_ids[b + i] = val[b + pos[e]];
    }
  }
}

union SmallSortStorage {
  rocprim::block_radix_sort<uint32_t, 256, 1, int32_t, 1, 1, 8>::storage_type s1;
  rocprim::block_radix_sort<uint32_t, 256, 2, int32_t, 1, 1, 8>::storage_type s2;
  rocprim::block_radix_sort<uint32_t, 256, 4, int32_t, 1, 1, 8>::storage_type s4;
  rocprim::block_radix_sort<uint32_t, 256, 8, int32_t, 1, 1, 8>::storage_type s8;
  rocprim::block_radix_sort<uint32_t, 256, 16, int32_t, 1, 1, 8>::storage_type s16;
};

__global__ void __launch_bounds__(256)
isect_tile_sort_small_kernel(const int32_t *__restrict__ starts, const uint32_t *__restrict__ tkey,
                             const int32_t *__restrict__ val, const float *__restrict__ depths,
                             int32_t *__restrict__ large_list, int32_t *__restrict__ n_large,
                             int64_t *__restrict__ isect_ids, int32_t *__restrict__ flatten_ids) {
  __shared__ SmallSortStorage storage;
  const int64_t b = starts[blockIdx.x], e = starts[blockIdx.x + 1];
  const int m = (int)(e - b);
  if (m <= 0) return;
  if (m > kSmallCap) {
    if (threadIdx.x == 0) large_list[atomicAdd(n_large, 1)] = blockIdx.x;
    return;
  }
  const uint32_t k32 = tkey[b];
  if (m <= 256) run_radix_sort<256, 1>(storage, b, m, k32, val, depths, isect_ids, flatten_ids);
  else if (m <= 512) run_radix_sort<256, 2>(storage, b, m, k32, val, depths, isect_ids, flatten_ids);
  else if (m <= 1024) run_radix_sort<256, 4>(storage, b, m, k32, val, depths, isect_ids, flatten_ids);
  else if (m <= 2048) run_radix_sort<256, 8>(storage, b, m, k32, val, depths, isect_ids, flatten_ids);
  else run_radix_sort<256, 16>(storage, b, m, k32, val, depths, isect_ids, flatten_ids);
}

// Runs longer than kLargeCap sort in global scratch, in slices of kLargeCap
// gathered per pass (the EPT registers cover kLargeCap elements).
template <int NT>
__device__ __forceinline__ void tile_run_sort_global(uint64_t *k, int64_t b, int m,
                                                     uint32_t key32,
                                                     const int32_t *__restrict__ val,
                                                     const float *__restrict__ depths,
                                                     int64_t *__restrict__ isect_ids,
                                                     int32_t *__restrict__ flatten_ids) {
  int P = 1;
  while (P < m) P <<= 1;
  for (int i = threadIdx.x; i < P; i += NT)
    k[i] = i < m ? (((uint64_t)__float_as_uint(depths[val[b + i]]) << 32) | (uint32_t)i)
                 : ~(uint64_t)0;
  __syncthreads();
  bitonic_sort<NT>(k, P);
  for (int i = threadIdx.x; i < m; i += NT) {
    const uint64_t kv = k[i];
    const int32_t db = (int32_t)(kv >> 32);
    isect_ids[b + i] = db < 0 ? (int64_t)db : (((int64_t)key32 << 32) | (int64_t)(uint32_t)db);
    flatten_ids[b + i] = val[b + (int64_t)(uint32_t)kv];
  }
}

union LargeSortStorage {
  rocprim::block_radix_sort<uint32_t, 1024, 8, int32_t, 1, 1, 8>::storage_type s8;
  rocprim::block_radix_sort<uint32_t, 1024, 16, int32_t, 1, 1, 8>::storage_type s16;
};

__global__ void __launch_bounds__(1024)
isect_tile_sort_large_kernel(const int32_t *__restrict__ starts, const uint32_t *__restrict__ tkey,
                             const int32_t *__restrict__ val, const float *__restrict__ depths,
                             const int32_t *__restrict__ large_list,
                             const int32_t *__restrict__ n_large, uint64_t *__restrict__ scratch,
                             int64_t *__restrict__ isect_ids, int32_t *__restrict__ flatten_ids) {
  __shared__ LargeSortStorage storage;
  if ((int)blockIdx.x >= *n_large) return;
  const int run = large_list[blockIdx.x];
  const int64_t b = starts[run], e = starts[run + 1];
  const int m = (int)(e - b);
  const uint32_t k32 = tkey[b];
  if (m <= 8192)
    run_radix_sort<1024, 8>(storage, b, m, k32, val, depths, isect_ids, flatten_ids);
  else if (m <= kLargeCap)
    run_radix_sort<1024, 16>(storage, b, m, k32, val, depths, isect_ids, flatten_ids);
  else  // runs are disjoint [b, b+m) and P < 2m: [2b, 2b+P) of scratch is private
    tile_run_sort_global<1024>(scratch + 2 * b, b, m, k32, val, depths, isect_ids, flatten_ids);
}

namespace {
// [tkeys 4n][vals 4n][starts][scratch 16n][rocPRIM temp]; the unsorted keys
// and values (sort input, dead after the sort) live at the head of scratch.
struct TileFirstLayout {
  size_t tkeys, vals, starts, scratch, tmp, total, tmp_bytes;
};

TileFirstLayout tilefirst_layout(int64_t n, int n_total, int key_bits) {
  (void)key_bits;
  const size_t t1 = lsd_sort_scratch_bytes(n);
  TileFirstLayout L{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align256(o + bytes);
    return at;
  };
  L.tkeys = take(4 * (size_t)n);
  L.vals = take(4 * (size_t)n);
  L.starts = take(4 * (size_t)(n_total + 2) + 4 * (size_t)(n_total + 2));  // + large-run list
  L.scratch = take(16 * (size_t)n);
  L.tmp_bytes = t1;
  L.tmp = take(L.tmp_bytes + 1);
  L.total = o;
  return L;
}
}  // namespace
}  // namespace gs

extern "C" int64_t gsplat_hip_isect_tilefirst_workspace_bytes(int64_t n_isects, int n_tiles_total,
                                                              int key_bits) {
  return (int64_t)tilefirst_layout(n_isects, n_tiles_total, key_bits).total;
}

extern "C" int gsplat_hip_isect_write_tilefirst(
    int64_t n_gaussians, int N, const float *means2d, const int32_t *radii, const float *depths,
    const int32_t *camera_ids, int tile_size, int tile_width, int tile_height, int n_cameras,
    int tile_bits, int cam_bits, const void *count_workspace, int64_t n_isects, void *workspace,
    int64_t workspace_bytes, int64_t *isect_ids, int32_t *flatten_ids, void *stream) {
  GS_REQUIRE(n_gaussians >= 0 && (camera_ids || N > 0 || n_gaussians == 0),
             "isect_write_tilefirst: N must be > 0 when camera_ids is null");
  GS_REQUIRE(tile_bits + cam_bits <= 32, "isect_write_tilefirst: tile_bits + cam_bits > 32");
  GS_REQUIRE(n_isects < (int64_t)1 << 30, "isect_write_tilefirst: more than 2^30 isects");
  if (n_isects <= 0) return 0;
  const int key_bits = tile_bits + cam_bits;
  const int n_tiles = tile_width * tile_height;
  const int n_total = n_cameras * n_tiles;
  const TileFirstLayout L = tilefirst_layout(n_isects, n_total, key_bits);
  GS_REQUIRE(workspace_bytes >= (int64_t)L.total, "isect_write_tilefirst: workspace %lld < %lld",
             (long long)workspace_bytes, (long long)L.total);
  hipStream_t st = (hipStream_t)stream;
  char *ws = reinterpret_cast<char *>(workspace);
  uint32_t *tkeys = reinterpret_cast<uint32_t *>(ws + L.tkeys);
  int32_t *vals = reinterpret_cast<int32_t *>(ws + L.vals);
  int32_t *starts = reinterpret_cast<int32_t *>(ws + L.starts);
  uint64_t *scratch = reinterpret_cast<uint64_t *>(ws + L.scratch);
  // The LSD sort ping-pongs between the emission buffers and (tkeys, vals):
  // emit where an even/odd number of passes ends in (tkeys, vals), so the
  // global-scratch run sort below never overwrites live keys.
  const bool emit_alt = ((key_bits + 7) / 8) % 2 == 1;
  uint32_t *tkey = emit_alt ? reinterpret_cast<uint32_t *>(ws + L.scratch) : tkeys;
  int32_t *val = emit_alt ? reinterpret_cast<int32_t *>(ws + L.scratch + 4 * (size_t)n_isects) : vals;
  uint32_t *akey = emit_alt ? tkeys : reinterpret_cast<uint32_t *>(ws + L.scratch);
  int32_t *aval = emit_alt ? vals : reinterpret_cast<int32_t *>(ws + L.scratch + 4 * (size_t)n_isects);
  void *tmp = ws + L.tmp;

  const int64_t nbG = (n_gaussians + kIsectBlock - 1) / kIsectBlock;
  const uint32_t all_ones = key_bits >= 32 ? 0xffffffffu : ((1u << key_bits) - 1u);
  hipLaunchKernelGGL(isect_write_tiles_kernel, dim3((unsigned)nbG), dim3(kIsectBlock), 0, st,
                     n_gaussians, N, means2d, radii, depths, camera_ids, tile_size, tile_width,
                     tile_height, tile_bits, all_ones,
                     reinterpret_cast<const int64_t *>(count_workspace), tkey, val);
  lsd_sort_pairs(tkey, val, akey, aval, n_isects, 0, key_bits, tmp, st);
  const uint32_t *sk = tkeys;  // see emit_alt (key_bits == 0: no pass, emitted there)
  const int32_t *sv = vals;
  const unsigned nb = (unsigned)((n_isects + 255) / 256);
  hipLaunchKernelGGL(isect_key_starts_kernel, dim3(nb), dim3(256), 0, st, n_isects, sk, n_total,
                     n_tiles, tile_bits, starts);
  int32_t *large_list = starts + (n_total + 2);
  int32_t *n_large = reinterpret_cast<int32_t *>(ws + L.tmp);  // rocPRIM temp is free again
  GS_HIP(gs::zero_async(n_large, sizeof(int32_t), st));
  hipLaunchKernelGGL(isect_tile_sort_small_kernel, dim3((unsigned)(n_total + 1)), dim3(256), 0,
                     st, starts, sk, sv, depths, large_list, n_large, isect_ids, flatten_ids);
  hipLaunchKernelGGL(isect_tile_sort_large_kernel,
                     dim3((unsigned)(n_isects / (kSmallCap + 1) + 1)), dim3(1024), 0, st, starts,
                     sk, sv, depths, large_list, n_large, scratch, isect_ids, flatten_ids);
  GS_CHECK_LAUNCH("isect_write_tilefirst");
  return 0;
}
