// Stable LSD radix sort of (uint32 key, int32 value) pairs for gfx950, used by
// the isect paths in place of rocPRIM's device sort (whose per-pass fixed cost,
// ~25 us for a 0.3 M-item onesweep pass, dominated the depth sort).
//
// One pass = 8 key bits (lsd_sort_pairs; lsd_one_pass: one digit as wide as
// its key, up to 11 bits), three launches:
//   lsd_hist     per tile of NT*IPT items: LDS digit histogram -> hist[d][tile]
//   lsd_scan     one workgroup per digit: exclusive scan of its row in place,
//                row total -> totals[d]
//   lsd_scatter  per tile: digit bases (scan of totals + hist[d][tile]),
//                stable in-tile ranks by wave ballots, reorder through LDS,
//                digit-contiguous (coalesced) stores
// The last pass can write the caller's final isect output directly (FinalOut).
// (A single-launch onesweep pass with decoupled look-back was tried: with all
// ~1000 tiles of a 4 M-item pass co-resident, the look-back chains cost more
// than the two small launches it saves.)
// The in-tile sort is stable and the tiles are laid out in input order, so the
// pass is stable and the whole sort equals a stable sort on bits
// [begin_bit, end_bit).  Traffic per pass: 4 B/item (hist) + 16 B/item
// (scatter read + write).
// Device count (n_dev non-null, the sync-free isect of a captured step): the
// grids are sized for the capacity n and every kernel reads the item count
// min(*n_dev, n) itself; the tiles past it exit at once and the scans stop
// at the last tile holding items.
#pragma once
#include <stdlib.h>

#include "common.h"

namespace gs {
namespace lsd {

constexpr int NT = 256;
constexpr int RADIX = 256;          // 8-bit digits
constexpr int RADIX_WIDE = 2048;    // 11-bit digits

inline int64_t n_tiles(int64_t n, int ipt) { return (n + (int64_t)NT * ipt - 1) / ((int64_t)NT * ipt); }

// Few items: small tiles so the grid still covers the chip.
inline int pick_ipt(int64_t n) { return n <= ((int64_t)1 << 20) ? 4 : 16; }

// Last-pass output of the isect sorts: instead of (key, value) write
// isect_ids[dst] = key << 32 | depth bits of depths[value] (the reference's
// sign-extended int64 id when the depth bits are negative) and
// flatten_ids[dst] = value.
struct FinalOut {
  const float *depths;
  int64_t *isect_ids;
  int32_t *flatten_ids;
};

template <int IPT, int RX>
__global__ void __launch_bounds__(NT)
hist_kernel(const uint32_t *__restrict__ keys, int64_t n, const int64_t *__restrict__ n_dev,
            int shift, uint32_t mask, uint32_t *__restrict__ hist, int64_t nt) {
  __shared__ uint32_t h[RX];
  if (n_dev) n = min(n, *n_dev);
  const int64_t base = (int64_t)blockIdx.x * NT * IPT;
  if (n_dev && base >= n) return;  // past the items: the scan does not read this tile
#pragma unroll
  for (int d = threadIdx.x; d < RX; d += NT) h[d] = 0;
  __syncthreads();
  if (mask < 64u) {
    // few digits (the short last pass of the tile sort): runs of equal
    // digits would serialise on one LDS address, so the lanes of a wave
    // holding the same digit are matched by ballots and one adds their count
    const int lane = threadIdx.x & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int e = 0; e < IPT; ++e) {
      const int64_t i = base + e * NT + threadIdx.x;
      const bool ok = i < n;
      const uint32_t dg = ok ? (keys[i] >> shift) & mask : 0u;
      uint64_t peers = __ballot(ok);
      for (uint32_t b = 1; b <= mask; b <<= 1) {
        const bool bit = (dg & b) != 0u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
      }
      if (ok && (peers & lt) == 0) atomicAdd(&h[dg], (uint32_t)__popcll(peers));
    }
  } else {
#pragma unroll
    for (int e = 0; e < IPT; ++e) {
      const int64_t i = base + e * NT + threadIdx.x;
      if (i < n) atomicAdd(&h[(keys[i] >> shift) & mask], 1u);
    }
  }
  __syncthreads();
#pragma unroll
  for (int d = threadIdx.x; d < RX; d += NT) hist[(int64_t)d * nt + blockIdx.x] = h[d];
}

// Exclusive scan of row d (nt entries) in place; the row sum -> totals[d].
// Device count: only the tiles holding items (tile = tile_items items).
__global__ void __launch_bounds__(NT)
scan_kernel(uint32_t *__restrict__ hist, int64_t nt, uint32_t *__restrict__ totals,
            const int64_t *__restrict__ n_dev, int64_t n, int64_t tile_items) {
  __shared__ uint32_t wsum[NT / 64];
  uint32_t *row = hist + (int64_t)blockIdx.x * nt;
  if (n_dev) nt = min(nt, (min(n, *n_dev) + tile_items - 1) / tile_items);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (int64_t b0 = 0; b0 < nt; b0 += NT) {
    const int64_t i = b0 + threadIdx.x;
    const uint32_t v = i < nt ? row[i] : 0u;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t before = carry, all = carry;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      before += w < wid ? wsum[w] : 0u;
      all += wsum[w];
    }
    if (i < nt) row[i] = before + x - v;
    carry = all;
    __syncthreads();
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// Stable in-tile ranking without sorting the tile: wave w owns the items
// [w*64*IPT, (w+1)*64*IPT) of the tile, visited e-major (coalesced loads).
// For every item the lanes holding the same digit are found with nbits
// ballots; the rank is the wave's running count for that digit plus the
// number of such lanes below.  Cross-wave offsets and the tile's digit starts
// come from the 4 x 256 wave counts; items are then reordered through LDS so
// the global stores are digit-contiguous.
template <int IPT, bool FINAL, int RX>
__global__ void __launch_bounds__(NT)
scatter_kernel(const uint32_t *__restrict__ kin, const int32_t *__restrict__ vin,
               uint32_t *__restrict__ kout, int32_t *__restrict__ vout, int64_t n,
               const int64_t *__restrict__ n_dev, int shift, int nbits,
               const uint32_t *__restrict__ hist, const uint32_t *__restrict__ totals, int64_t nt,
               FinalOut fo) {
  constexpr int NW = NT / 64, TILE = NT * IPT, DPT = RX / NT;  // digits per thread
  __shared__ uint32_t cnt[NW][RX];
  __shared__ uint32_t gbase[RX];  // global position of tile slot 0 of digit d's range
  __shared__ uint32_t wsum[NW];
  __shared__ uint32_t kbuf[TILE];
  __shared__ int32_t vbuf[TILE];
  const uint32_t mask = (1u << nbits) - 1u;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
#pragma unroll
  for (int w = 0; w < NW; ++w)
#pragma unroll
    for (int j = 0; j < DPT; ++j) cnt[w][t * DPT + j] = 0;
  const int64_t base = (int64_t)blockIdx.x * TILE;
  if (n_dev) n = min(n, *n_dev);
  const int nvalid = (int)max<int64_t>(0, min<int64_t>((int64_t)TILE, n - base));
  if (n_dev && nvalid == 0) return;  // past the items
  uint32_t key[IPT];
  int32_t val[IPT];
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int j = wid * 64 * IPT + e * 64 + lane;
    key[e] = j < nvalid ? kin[base + j] : 0u;
    val[e] = j < nvalid ? vin[base + j] : 0;
  }
  __syncthreads();
  uint32_t rank[IPT];
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int j = wid * 64 * IPT + e * 64 + lane;
    const bool ok = j < nvalid;
    const uint32_t dg = (key[e] >> shift) & mask;
    uint64_t peers = __ballot(ok);
    for (int b = 0; b < nbits; ++b) {
      const bool bit = (dg >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      peers &= bit ? bal : ~bal;
    }
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    const uint32_t old = ok ? cnt[wid][dg] : 0u;
    // LDS ops of one wave complete in order: every peer read `old` above.
    if (ok && below == 0) cnt[wid][dg] = old + (uint32_t)__popcll(peers);
    rank[e] = old + below;
  }
  __syncthreads();
  // digits t*DPT .. t*DPT+DPT-1: offsets of the waves, tile totals, and the
  // exclusive scans (tile-local and global) across all digits
  uint32_t woff[DPT][NW], tot[DPT], tsum = 0, gv[DPT], gsum = 0;
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const int d = t * DPT + j;
    tot[j] = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      woff[j][w] = tot[j];
      tot[j] += cnt[w][d];
    }
    tsum += tot[j];
    gv[j] = totals[d];
    gsum += gv[j];
  }
  uint32_t x = tsum, g = gsum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64), z = __shfl_up(g, o, 64);
    if (lane >= o) {
      x += y;
      g += z;
    }
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t lbefore = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) lbefore += w < wid ? wsum[w] : 0u;
  uint32_t lrun = lbefore + x - tsum;  // tile slot of digit t*DPT's first item
  __syncthreads();
  if (lane == 63) wsum[wid] = g;
  __syncthreads();
  uint32_t gbefore = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) gbefore += w < wid ? wsum[w] : 0u;
  uint32_t grun = gbefore + g - gsum;  // global start of digit t*DPT
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const int d = t * DPT + j;
    gbase[d] = grun + hist[(int64_t)d * nt + blockIdx.x] - lrun;
#pragma unroll
    for (int w = 0; w < NW; ++w) cnt[w][d] = lrun + woff[j][w];  // tile slot of wave w's first
    lrun += tot[j];
    grun += gv[j];
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int j = wid * 64 * IPT + e * 64 + lane;
    if (j < nvalid) {
      const uint32_t slot = cnt[wid][(key[e] >> shift) & mask] + rank[e];
      kbuf[slot] = key[e];
      vbuf[slot] = val[e];
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int s = e * NT + t;
    if (s < nvalid) {
      const uint32_t k = kbuf[s];
      const int32_t v = vbuf[s];
      const uint32_t dst = gbase[(k >> shift) & mask] + (uint32_t)s;
      if (FINAL) {
        const int32_t db = __float_as_int(fo.depths[v]);
        fo.isect_ids[dst] = db < 0 ? (int64_t)db : (((int64_t)k << 32) | (int64_t)(uint32_t)db);
        fo.flatten_ids[dst] = v;
      } else {
        kout[dst] = k;
        vout[dst] = v;
      }
    }
  }
}

}  // namespace lsd

// Scratch for lsd_sort_pairs: hist rows + totals (sized for 11-bit digits).
inline size_t lsd_sort_scratch_bytes(int64_t n) {
  const int64_t nt = lsd::n_tiles(n, lsd::pick_ipt(n));
  return 4 * (size_t)(lsd::RADIX_WIDE * nt + lsd::RADIX_WIDE);
}

// Stable sort of n pairs by key bits [begin_bit, end_bit), ping-ponging
// between (k0, v0) and (k1, v1).  Returns 0 if the result is in (k0, v0),
// 1 if in (k1, v1).  With `fo` non-null the last pass writes the final isect
// output instead (see FinalOut; the return value is then meaningless).
// n < 2^32.
inline int lsd_sort_pairs(uint32_t *k0, int32_t *v0, uint32_t *k1, int32_t *v1, int64_t n,
                          int begin_bit, int end_bit, void *scratch, hipStream_t st,
                          const lsd::FinalOut *fo = nullptr, const int64_t *n_dev = nullptr) {
  if (n <= 0 || end_bit <= begin_bit) return 0;
  const int ipt = lsd::pick_ipt(n);
  const int64_t nt = lsd::n_tiles(n, ipt);
  // 8-bit digits throughout: 11-bit digits for the 32-bit depth sort (3
  // passes) measured slower at M2, 78 us against 68 us for 4 passes (the
  // 2048-bin histograms and scans cost more than the pass they save); removed
  constexpr int dbits = 8, radix = lsd::RADIX;
  uint32_t *hist = reinterpret_cast<uint32_t *>(scratch);
  uint32_t *totals = hist + (int64_t)radix * nt;
  int cur = 0;
  for (int shift = begin_bit; shift < end_bit; shift += dbits) {
    const int nbits = end_bit - shift < dbits ? end_bit - shift : dbits;
    const uint32_t mask = (1u << nbits) - 1u;
    uint32_t *ki = cur ? k1 : k0, *ko = cur ? k0 : k1;
    int32_t *vi = cur ? v1 : v0, *vo = cur ? v0 : v1;
    if (ipt == 4)
      hipLaunchKernelGGL((lsd::hist_kernel<4, lsd::RADIX>), dim3((unsigned)nt), dim3(lsd::NT), 0,
                         st, ki, n, n_dev, shift, mask, hist, nt);
    else
      hipLaunchKernelGGL((lsd::hist_kernel<16, lsd::RADIX>), dim3((unsigned)nt), dim3(lsd::NT), 0,
                         st, ki, n, n_dev, shift, mask, hist, nt);
    hipLaunchKernelGGL(lsd::scan_kernel, dim3((unsigned)radix), dim3(lsd::NT), 0, st, hist, nt,
                       totals, n_dev, n, (int64_t)lsd::NT * ipt);
    const bool fin = fo && shift + dbits >= end_bit;
    const lsd::FinalOut f = fin ? *fo : lsd::FinalOut{nullptr, nullptr, nullptr};
#define GS_LSD_SCATTER(I, F, RX)                                                              \
  hipLaunchKernelGGL((lsd::scatter_kernel<I, F, RX>), dim3((unsigned)nt), dim3(lsd::NT), 0, st, \
                     ki, vi, ko, vo, n, n_dev, shift, nbits, hist, totals, nt, f)
    if (ipt == 4) {
      if (fin) GS_LSD_SCATTER(4, true, lsd::RADIX); else GS_LSD_SCATTER(4, false, lsd::RADIX);
    } else {
      if (fin) GS_LSD_SCATTER(16, true, lsd::RADIX); else GS_LSD_SCATTER(16, false, lsd::RADIX);
    }
#undef GS_LSD_SCATTER
    cur ^= 1;
  }
  return cur;
}

// One stable pass over keys < 2^nbits (nbits <= 11) with a digit as wide as
// the key (RX = 256 .. 2048 bins), (k0, v0) -> (k1, v1).  Returns the digit
// totals (the scan's row sums, inside `scratch`).  Device count as above.
inline const uint32_t *lsd_one_pass(const uint32_t *k0, const int32_t *v0, uint32_t *k1,
                                    int32_t *v1, int64_t n, int nbits, void *scratch,
                                    hipStream_t st, const int64_t *n_dev) {
  const int ipt = lsd::pick_ipt(n);
  const int64_t nt = lsd::n_tiles(n, ipt);
  const int rx = nbits <= 8 ? 256 : nbits <= 9 ? 512 : nbits <= 10 ? 1024 : 2048;
  uint32_t *hist = reinterpret_cast<uint32_t *>(scratch);
  uint32_t *totals = hist + (int64_t)rx * nt;
  if (n <= 0) return totals;
  const uint32_t mask = (1u << nbits) - 1u;
  const lsd::FinalOut none{nullptr, nullptr, nullptr};
#define GS_LSD1(I, RX)                                                                            \
  do {                                                                                            \
    hipLaunchKernelGGL((lsd::hist_kernel<I, RX>), dim3((unsigned)nt), dim3(lsd::NT), 0, st, k0,   \
                       n, n_dev, 0, mask, hist, nt);                                              \
    hipLaunchKernelGGL(lsd::scan_kernel, dim3((unsigned)RX), dim3(lsd::NT), 0, st, hist, nt,      \
                       totals, n_dev, n, (int64_t)lsd::NT * I);                                   \
    hipLaunchKernelGGL((lsd::scatter_kernel<I, false, RX>), dim3((unsigned)nt), dim3(lsd::NT), 0, \
                       st, k0, v0, k1, v1, n, n_dev, 0, nbits, hist, totals, nt, none);           \
  } while (0)
#define GS_LSD1_RX(RX) \
  do {                 \
    if (ipt == 4)      \
      GS_LSD1(4, RX);  \
    else               \
      GS_LSD1(16, RX); \
  } while (0)
  if (rx == 256) GS_LSD1_RX(256);
  else if (rx == 512) GS_LSD1_RX(512);
  else if (rx == 1024) GS_LSD1_RX(1024);
  else GS_LSD1_RX(2048);
#undef GS_LSD1_RX
#undef GS_LSD1
  return totals;
}

}  // namespace gs
