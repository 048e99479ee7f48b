// One-launch stable LSD sort of the visible Gaussians' 32-bit depth keys
// (with their Gaussian ids), gfx950.  Replaces lsd_sort_pairs' 4 passes x
// (hist, scan, scatter) = 12 launches for the depth sort of the isect
// (isect.hip "Depth-first sorted emission" step (i)) when the item count fits
// one resident grid.
//
// kWG workgroups of kNT threads stay resident for the whole sort; each owns a
// contiguous chunk of at most kTile items (the chunk is one tile of
// lsd::scatter_kernel: the same ballot ranking, the same LDS reorder and
// digit-contiguous stores, hence the same stable order).  Per 8-bit pass:
//   1. load the chunk, rank it per digit (wave ballots), store the chunk's
//      256-bin histogram to H[wg];
//   2. grid barrier;
//   3. every workgroup reads all of H: its digit bases are the digit's start
//      (exclusive scan of the totals) plus the counts of the workgroups before
//      it (what lsd::scan_kernel's rows hold);
//   4. reorder through LDS, store the digit runs;
//   5. grid barrier (the next pass reads other workgroups' stores).
// Seven barriers instead of eleven kernel boundaries.  A barrier is the
// kernel boundary's cache work done in place: every wave drains its stores,
// one thread per workgroup writes the XCD's L2 back (agent-scope release),
// adds to the barrier's counter (device-scope atomic) and polls it, then
// invalidates (agent-scope acquire).  Co-residency: kWG = 128 workgroups of
// ~73 KB LDS on 256 CUs (2 fit per CU) -- the sort runs between other
// kernels of one stream.  The polls are bounded: on
// timeout a sticky error word is set and the sort runs on (no hang; the
// caller's tests see the error word).
//
// Traffic per pass: 8 B/item read + 8 B/item written (as one lsd pass's
// scatter), plus the 128 KB histogram table read by every workgroup (16-B
// loads, 16 per thread; L2 hits after the first workgroup of an XCD).
#pragma once
#include "common.h"

namespace gs {
namespace dsort {

constexpr int kNT = 512;                 // threads per workgroup (8 waves)
constexpr int kIPT = 16;                 // items per thread
constexpr int kTile = kNT * kIPT;        // 8192 items per workgroup at most
constexpr int kWG = 128;                 // resident workgroups (2 fit per CU)
constexpr int64_t kMaxItems = (int64_t)kTile * kWG;  // 1 M items
constexpr int kRX = 256;                 // 8-bit digits
constexpr int kBars = 8;                 // barrier counters (7 used) + error word

GS_INLINE void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// All kWG workgroups past this point see each other's earlier global stores.
GS_INLINE void grid_sync(unsigned *ctr, unsigned *err) {
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_stores();
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int it = 0;
         __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)kWG;
         ++it) {
      if (it > (1 << 16)) {  // not co-resident: give up waiting (results invalid)
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    drain_stores();
  }
  __syncthreads();
}

// (k0, v0) -> 4 passes -> (k0, v0), ping-ponging through (k1, v1).  n items
// (min(n, *n_dev) with a device count).  H: kWG x 256 u32 scratch.  bar:
// kBars u32, zeroed before the launch (isect_compact_kernel does it).
__global__ void __launch_bounds__(kNT)
sort_kernel(uint32_t *__restrict__ k0, int32_t *__restrict__ v0, uint32_t *__restrict__ k1,
            int32_t *__restrict__ v1, int64_t n, const int64_t *__restrict__ n_dev,
            uint32_t *__restrict__ H, unsigned *__restrict__ bar) {
  constexpr int NW = kNT / 64;
  __shared__ uint32_t cnt[NW][kRX];
  __shared__ uint32_t gbase[kRX];
  __shared__ uint32_t dsum[kRX / 64];
  __shared__ __attribute__((aligned(16))) uint32_t kbuf[kTile];
  __shared__ int32_t vbuf[kTile];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wg = blockIdx.x;
  if (n_dev) n = min(n, *n_dev);
  // contiguous chunks of equal size (the last ones may be short or empty)
  const int64_t chunk = (n + kWG - 1) / kWG;
  const int64_t base = min<int64_t>((int64_t)wg * chunk, n);
  const int nvalid = (int)(min<int64_t>(base + chunk, n) - base);
  const uint64_t lt = (1ull << lane) - 1ull;
  unsigned *err = bar + kBars - 1;
#pragma unroll 1
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    const uint32_t *ki = (pass & 1) ? k1 : k0;
    const int32_t *vi = (pass & 1) ? v1 : v0;
    uint32_t *ko = (pass & 1) ? k0 : k1;
    int32_t *vo = (pass & 1) ? v0 : v1;
    // ---- 1. load + stable in-chunk ranking (lsd::scatter_kernel's order:
    // wave w owns items [w*64*IPT, (w+1)*64*IPT), visited e-major)
    for (int d = t; d < NW * kRX; d += kNT) (&cnt[0][0])[d] = 0;
    uint32_t key[kIPT];
    int32_t val[kIPT];
#pragma unroll
    for (int e = 0; e < kIPT; ++e) {
      const int j = wid * 64 * kIPT + e * 64 + lane;
      key[e] = j < nvalid ? ki[base + j] : 0u;
      val[e] = j < nvalid ? vi[base + j] : 0;
    }
    __syncthreads();
    uint32_t rank[kIPT];
#pragma unroll
    for (int e = 0; e < kIPT; ++e) {
      const int j = wid * 64 * kIPT + e * 64 + lane;
      const bool ok = j < nvalid;
      const uint32_t dg = (key[e] >> shift) & 255u;
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const bool bit = (dg >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
      }
      const uint32_t below = (uint32_t)__popcll(peers & lt);
      const uint32_t old = ok ? cnt[wid][dg] : 0u;
      // LDS ops of one wave complete in order: every peer read `old` above
      if (ok && below == 0) cnt[wid][dg] = old + (uint32_t)__popcll(peers);
      rank[e] = old + below;
    }
    __syncthreads();
    // chunk histogram (thread d < 256: digit d) and the waves' offsets
    uint32_t tot = 0, woff[NW];
    if (t < kRX) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        woff[w] = tot;
        tot += cnt[w][t];
      }
      H[(int64_t)wg * kRX + t] = tot;
    }
    // ---- 2.
    grid_sync(bar + 2 * pass, err);
    // ---- 3. digit d: start = sum of the totals of digits < d, plus the
    // counts of digit d in the chunks before this one.  Thread t sums digits
    // 4 (t & 63) .. +3 over the chunks w = t >> 6 (mod 8) (16-B loads), the
    // eight partial sums meet in LDS (kbuf, free until step 4)
    {
      const int dq = t & 63, ws = t >> 6;
      uint4 p4 = make_uint4(0, 0, 0, 0), a4 = make_uint4(0, 0, 0, 0);
      const uint4 *H4 = reinterpret_cast<const uint4 *>(H);
#pragma unroll
      for (int w = ws; w < kWG; w += NW) {
        const uint4 h = H4[w * (kRX / 4) + dq];
        a4.x += h.x; a4.y += h.y; a4.z += h.z; a4.w += h.w;
        if (w < wg) {
          p4.x += h.x; p4.y += h.y; p4.z += h.z; p4.w += h.w;
        }
      }
      uint4 *red = reinterpret_cast<uint4 *>(kbuf);  // [2][NW][64] uint4
      red[ws * 64 + dq] = p4;
      red[(NW + ws) * 64 + dq] = a4;
    }
    __syncthreads();
    uint32_t pre = 0, all = 0;
    if (t < kRX) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        pre += kbuf[w * kRX + t];
        all += kbuf[(NW + w) * kRX + t];
      }
    }
    // exclusive scans over the 256 digits: of the totals (global start) and
    // of this chunk's counts (slot of the digit's first item in the chunk)
    uint32_t g = all, l = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(g, o, 64), z = __shfl_up(l, o, 64);
      if (lane >= o) {
        g += y;
        l += z;
      }
    }
    __shared__ uint32_t lsum[kRX / 64];
    if (t < kRX && lane == 63) {
      dsum[wid] = g;
      lsum[wid] = l;
    }
    __syncthreads();
    if (t < kRX) {
      uint32_t gb = 0, lb = 0;
#pragma unroll
      for (int w = 0; w < kRX / 64; ++w) {
        gb += w < wid ? dsum[w] : 0u;
        lb += w < wid ? lsum[w] : 0u;
      }
      const uint32_t gstart = gb + g - all, lstart = lb + l - tot;
      gbase[t] = gstart + pre - lstart;  // + chunk slot = destination
#pragma unroll
      for (int w = 0; w < NW; ++w) cnt[w][t] = lstart + woff[w];  // slot of wave w's first
    }
    __syncthreads();
    // ---- 4. reorder through LDS, digit-contiguous stores
#pragma unroll
    for (int e = 0; e < kIPT; ++e) {
      const int j = wid * 64 * kIPT + e * 64 + lane;
      if (j < nvalid) {
        const uint32_t s = cnt[wid][(key[e] >> shift) & 255u] + rank[e];
        kbuf[s] = key[e];
        vbuf[s] = val[e];
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kIPT; ++e) {
      const int s = e * kNT + t;
      if (s < nvalid) {
        const uint32_t k = kbuf[s];
        const uint32_t dst = gbase[(k >> shift) & 255u] + (uint32_t)s;
        if (dst < (uint32_t)n) {  // always, unless a barrier timed out
          ko[dst] = k;
          vo[dst] = vbuf[s];
        }
      }
    }
    // ---- 5.
    if (pass < 3) grid_sync(bar + 2 * pass + 1, err);
  }
}

}  // namespace dsort
}  // namespace gs
