// Wave64 lane-exchange helpers shared by the rasterizers (gfx950).
//
// reduce_scatter<N>: the per-lane partial gradients of N <= 16 fields are
// summed over the 64 lanes with permlane32/16 swaps, DPP row mirrors and quad
// permutes; afterwards lane l holds the wave total of field rs_field(l) (the
// four lanes of a quad hold the same total), so 16 lanes can issue one
// coalesced atomic into a packed gradient row.
#pragma once

#include "common.h"

namespace gs {

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

// Pair exchange of lane bit 3 / bit 2 with the reduction, selected by DPP
// bank masks instead of per-lane selects (a bank is 4 lanes of a 16-lane
// row).  add_b3(lo, hi): lanes with bit 3 clear (banks 0, 1) get
// lo + lo[lane ^ 8], lanes with it set (banks 2, 3) hi + hi[lane ^ 8]
// (row_ror:8 pairs exactly lane ^ 8).  add_b2: the same for bit 2 (banks 0,
// 2 read lane + 4 = row_ror:12, banks 1, 3 lane - 4 = row_ror:4).  Two
// v_add_f32_dpp per value; the select-based form took 2 v_cndmask_b32 more.
// s_nop 1: the VALU-write -> DPP-read hazard needs two wait states, which the
// compiler does not insert for inline asm.
GS_INLINE float add_b3(float lo, float hi) {
  float r;
  asm("s_nop 1\n\t"
      "v_add_f32_dpp %0, %1, %1 row_ror:8 row_mask:0xf bank_mask:0x3\n\t"
      "v_add_f32_dpp %0, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xc"
      : "=&v"(r)
      : "v"(lo), "v"(hi));
  return r;
}
GS_INLINE float add_b2(float lo, float hi) {
  float r;
  asm("s_nop 1\n\t"
      "v_add_f32_dpp %0, %1, %1 row_ror:12 row_mask:0xf bank_mask:0x5\n\t"
      "v_add_f32_dpp %0, %2, %2 row_ror:4 row_mask:0xf bank_mask:0xa"
      : "=&v"(r)
      : "v"(lo), "v"(hi));
  return r;
}

// Reduce-scatter of N <= 16 per-lane values over the wave: every lane ends
// with the wave-wide total of field rs_field(lane).  Fields are paired
// adjacently at each halving (lane bits 5, 4, 3, 2 choose the half), so an
// odd count costs no padded swaps: 9 fields take 5 + 3 + 2 + 1 combining
// steps plus two quad adds.
// a[i] for i < M, else 0 (index clamped so that no access is out of range)
template <int M>
GS_INLINE float pick(const float (&a)[M], int i) {
  return i < M ? a[i < M ? i : 0] : 0.f;
}

template <int N>
GS_INLINE float reduce_scatter(const float *v, int lane) {
  static_assert(N >= 1 && N <= 16, "reduce_scatter: 1..16 fields");
  constexpr int N1 = (N + 1) / 2, N2 = (N1 + 1) / 2, N3 = (N2 + 1) / 2;
  float w[N1], x[N2], y[N3];
#pragma unroll
  for (int i = 0; i < N1; ++i) w[i] = swap32_sum(v[2 * i], 2 * i + 1 < N ? v[2 * i + 1] : 0.f);
#pragma unroll
  for (int i = 0; i < N2; ++i) x[i] = swap16_sum(w[2 * i], pick(w, 2 * i + 1));
  (void)lane;
#pragma unroll
  for (int i = 0; i < N3; ++i) y[i] = add_b3(x[2 * i], pick(x, 2 * i + 1));  // bit 3
  float z = add_b2(y[0], pick(y, 1));  // bit 2
  z += dpp<0xB1>(z);  // quad lane ^ 1
  z += dpp<0x4E>(z);  // quad lane ^ 2
  return z;
}

// The field whose total lane `lane` holds after reduce_scatter.
GS_INLINE int rs_field(int lane) {
  return ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2) |
         (((lane >> 2) & 1) << 3);
}

GS_INLINE void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

GS_INLINE int ballot_slot(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

}  // namespace gs
