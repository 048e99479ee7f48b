// Stable LSD radix sort of (uint32 key, int32 value) pairs for gfx950, used by
// the isect paths in place of rocPRIM's device sort (whose per-pass fixed cost,
// ~25 us for a 0.3 M-item onesweep pass, dominated the depth sort).
//
// One pass = 8 key bits, three launches:
//   lsd_hist     per tile of NT*IPT items: LDS digit histogram -> hist[d][tile]
//   lsd_scan     one workgroup per digit: exclusive scan of its row in place,
//                row total -> totals[d]
//   lsd_scatter  per tile: digit bases (scan of totals + hist[d][tile]),
//                stable in-tile sort by the digit (rocPRIM block radix sort,
//                one 8-bit internal pass), striped output -> coalesced stores
// The in-tile sort is stable and the tiles are laid out in input order, so the
// pass is stable and the whole sort equals a stable sort on bits
// [begin_bit, end_bit).  Traffic per pass: 4 B/item (hist) + 16 B/item
// (scatter read + write).
#pragma once
#include "common.h"

#include <rocprim/block/block_radix_sort.hpp>

namespace gs {
namespace lsd {

constexpr int NT = 256;
constexpr int RADIX = 256;

inline int64_t n_tiles(int64_t n, int ipt) { return (n + (int64_t)NT * ipt - 1) / ((int64_t)NT * ipt); }

// Few items: small tiles so the grid still covers the chip.
inline int pick_ipt(int64_t n) { return n <= ((int64_t)1 << 20) ? 4 : 16; }

template <int IPT>
__global__ void __launch_bounds__(NT)
hist_kernel(const uint32_t *__restrict__ keys, int64_t n, int shift, uint32_t mask,
            uint32_t *__restrict__ hist, int64_t nt) {
  __shared__ uint32_t h[RADIX];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * NT * IPT;
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int64_t i = base + e * NT + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & mask], 1u);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * nt + blockIdx.x] = h[threadIdx.x];
}

// Exclusive scan of row d (nt entries) in place; the row sum -> totals[d].
__global__ void __launch_bounds__(NT)
scan_kernel(uint32_t *__restrict__ hist, int64_t nt, uint32_t *__restrict__ totals) {
  __shared__ uint32_t wsum[NT / 64];
  uint32_t *row = hist + (int64_t)blockIdx.x * nt;
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

template <int IPT>
__global__ void __launch_bounds__(NT)
scatter_kernel(const uint32_t *__restrict__ kin, const int32_t *__restrict__ vin,
               uint32_t *__restrict__ kout, int32_t *__restrict__ vout, int64_t n, int shift,
               int nbits, const uint32_t *__restrict__ hist, const uint32_t *__restrict__ totals,
               int64_t nt) {
  using BRS = rocprim::block_radix_sort<uint32_t, NT, IPT, int32_t, 1, 1, 8>;
  __shared__ typename BRS::storage_type storage;
  __shared__ uint32_t gbase[RADIX];  // global destination of the tile's first item of digit d
  __shared__ uint32_t lcnt[RADIX];
  __shared__ uint32_t wsum[NT / 64];
  const uint32_t mask = (1u << nbits) - 1u;
  const int d = threadIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  lcnt[d] = 0;
  // exclusive scan of the digit totals (one digit per lane)
  const uint32_t tv = totals[d];
  uint32_t x = tv;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) before += w < wid ? wsum[w] : 0u;
  const uint32_t dbase = before + x - tv + hist[(int64_t)d * nt + blockIdx.x];

  const int64_t base = (int64_t)blockIdx.x * NT * IPT;
  const int nvalid = (int)min<int64_t>((int64_t)NT * IPT, n - base);
  uint32_t key[IPT];
  int32_t val[IPT];
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int j = threadIdx.x * IPT + e;  // blocked: input order = (thread, item)
    key[e] = j < nvalid ? kin[base + j] : 0xffffffffu;
    val[e] = j < nvalid ? vin[base + j] : 0;
    if (j < nvalid) atomicAdd(&lcnt[(key[e] >> shift) & mask], 1u);
  }
  __syncthreads();
  // exclusive scan of the in-tile digit counts -> gbase[d] = dbase - lstart[d]
  const uint32_t c = lcnt[d];
  x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __syncthreads();  // wsum reuse
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  before = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) before += w < wid ? wsum[w] : 0u;
  gbase[d] = dbase - (before + x - c);
  BRS().sort_to_striped(key, val, storage, (unsigned)shift, (unsigned)(shift + nbits));
  // sort_to_striped ends with a barrier-free exchange; gbase was written
  // before its internal barriers.
#pragma unroll
  for (int e = 0; e < IPT; ++e) {
    const int s = e * NT + threadIdx.x;  // striped: sorted position in the tile
    if (s < nvalid) {
      const uint32_t dst = gbase[(key[e] >> shift) & mask] + (uint32_t)s;
      kout[dst] = key[e];
      vout[dst] = val[e];
    }
  }
}

}  // namespace lsd

// Scratch for lsd_sort_pairs: hist rows + totals.
inline size_t lsd_sort_scratch_bytes(int64_t n) {
  const int64_t nt = lsd::n_tiles(n, lsd::pick_ipt(n));
  return 4 * (size_t)(lsd::RADIX * nt + lsd::RADIX);
}

// Stable sort of n pairs by key bits [begin_bit, end_bit), ping-ponging
// between (k0, v0) and (k1, v1).  Returns 0 if the result is in (k0, v0),
// 1 if in (k1, v1).  n < 2^32.
inline int lsd_sort_pairs(uint32_t *k0, int32_t *v0, uint32_t *k1, int32_t *v1, int64_t n,
                          int begin_bit, int end_bit, void *scratch, hipStream_t st) {
  if (n <= 0 || end_bit <= begin_bit) return 0;
  const int ipt = lsd::pick_ipt(n);
  const int64_t nt = lsd::n_tiles(n, ipt);
  uint32_t *hist = reinterpret_cast<uint32_t *>(scratch);
  uint32_t *totals = hist + (int64_t)lsd::RADIX * nt;
  int cur = 0;
  for (int shift = begin_bit; shift < end_bit; shift += 8) {
    const int nbits = end_bit - shift < 8 ? end_bit - shift : 8;
    const uint32_t mask = (1u << nbits) - 1u;
    uint32_t *ki = cur ? k1 : k0, *ko = cur ? k0 : k1;
    int32_t *vi = cur ? v1 : v0, *vo = cur ? v0 : v1;
    if (ipt == 4)
      hipLaunchKernelGGL(lsd::hist_kernel<4>, dim3((unsigned)nt), dim3(lsd::NT), 0, st, ki, n,
                         shift, mask, hist, nt);
    else
      hipLaunchKernelGGL(lsd::hist_kernel<16>, dim3((unsigned)nt), dim3(lsd::NT), 0, st, ki, n,
                         shift, mask, hist, nt);
    hipLaunchKernelGGL(lsd::scan_kernel, dim3(lsd::RADIX), dim3(lsd::NT), 0, st, hist, nt, totals);
    if (ipt == 4)
      hipLaunchKernelGGL(lsd::scatter_kernel<4>, dim3((unsigned)nt), dim3(lsd::NT), 0, st, ki, vi,
                         ko, vo, n, shift, nbits, hist, totals, nt);
    else
      hipLaunchKernelGGL(lsd::scatter_kernel<16>, dim3((unsigned)nt), dim3(lsd::NT), 0, st, ki, vi,
                         ko, vo, n, shift, nbits, hist, totals, nt);
    cur ^= 1;
  }
  return cur;
}

}  // namespace gs
