// Micro-benchmark: wave64 VALU issue rate of the instruction classes the
// rasterizer uses (profiling aid; not part of the library).
//   hipcc -O3 --offload-arch=gfx950 tools/valu_bench.hip -o /tmp/valu_bench
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 4096;

#define KERNEL(NAME, INIT, BODY)                                                   \
  __global__ void __launch_bounds__(256) NAME(float *out, float s) {            \
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;       \
    float a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                   \
    INIT;                                                                        \
    for (int i = 0; i < ITERS; ++i) { BODY; }                                    \
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
  }

// 8 independent chains, one instruction each per iteration
KERNEL(k_fma, , a0 = fmaf(a0, s, 1.f); a1 = fmaf(a1, s, 1.f); a2 = fmaf(a2, s, 1.f);
       a3 = fmaf(a3, s, 1.f); a4 = fmaf(a4, s, 1.f); a5 = fmaf(a5, s, 1.f);
       a6 = fmaf(a6, s, 1.f); a7 = fmaf(a7, s, 1.f))
KERNEL(k_mul, , a0 *= s; a1 *= s; a2 *= s; a3 *= s; a4 *= s; a5 *= s; a6 *= s; a7 *= s)
KERNEL(k_exp, , a0 = __builtin_amdgcn_exp2f(a0); a1 = __builtin_amdgcn_exp2f(a1);
       a2 = __builtin_amdgcn_exp2f(a2); a3 = __builtin_amdgcn_exp2f(a3);
       a4 = __builtin_amdgcn_exp2f(a4); a5 = __builtin_amdgcn_exp2f(a5);
       a6 = __builtin_amdgcn_exp2f(a6); a7 = __builtin_amdgcn_exp2f(a7))
KERNEL(k_sel, bool c = threadIdx.x & 1, a0 = c ? a1 : a0; a1 = c ? a2 : a1; a2 = c ? a3 : a2;
       a3 = c ? a4 : a3; a4 = c ? a5 : a4; a5 = c ? a6 : a5; a6 = c ? a7 : a6;
       a7 = c ? a0 : a7)
KERNEL(k_cmpsel, , a0 = a0 > s ? a1 : a0; a1 = a1 > s ? a2 : a1; a2 = a2 > s ? a3 : a2;
       a3 = a3 > s ? a4 : a3; a4 = a4 > s ? a5 : a4; a5 = a5 > s ? a6 : a5;
       a6 = a6 > s ? a7 : a6; a7 = a7 > s ? a0 : a7)
KERNEL(k_dpp, ,
       a0 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a0), 0x140, 0xf, 0xf, false));
       a1 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a1), 0x140, 0xf, 0xf, false));
       a2 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a2), 0x140, 0xf, 0xf, false));
       a3 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a3), 0x140, 0xf, 0xf, false));
       a4 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a4), 0x140, 0xf, 0xf, false));
       a5 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a5), 0x140, 0xf, 0xf, false));
       a6 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a6), 0x140, 0xf, 0xf, false));
       a7 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a7), 0x140, 0xf, 0xf, false)))
KERNEL(k_perm32, , {
  auto r0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a1), false, false);
  auto r1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a2), __float_as_uint(a3), false, false);
  auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a4), __float_as_uint(a5), false, false);
  auto r3 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a6), __float_as_uint(a7), false, false);
  a0 = __uint_as_float(r0[0]) + s; a1 = __uint_as_float(r0[1]); a2 = __uint_as_float(r1[0]) + s;
  a3 = __uint_as_float(r1[1]); a4 = __uint_as_float(r2[0]) + s; a5 = __uint_as_float(r2[1]);
  a6 = __uint_as_float(r3[0]) + s; a7 = __uint_as_float(r3[1]); })

template <typename K>
void run(const char *name, K k, float *out, int blocks, int instr_per_iter) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.999f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double waves = blocks * 4.0;
  const double winstr = waves * ITERS * instr_per_iter;  // wave-instructions
  const double per_simd = winstr / 1024.0;
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const double cycles = ms * 1e-3 * clk_khz * 1e3;
  printf("%-10s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (clock %d MHz)\n", name, ms,
         cycles / per_simd, clk_khz / 1000);
}

int main() {
  float *out;
  const int blocks = 256 * 8 * 4;  // 8 waves per SIMD x 4 rounds
  hipMalloc(&out, sizeof(float) * blocks * 256);
  run("fma", k_fma, out, blocks, 8);
  run("mul", k_mul, out, blocks, 8);
  run("exp2", k_exp, out, blocks, 8);
  run("select", k_sel, out, blocks, 8);
  run("cmp+sel", k_cmpsel, out, blocks, 16);
  run("dpp+add", k_dpp, out, blocks, 8);
  run("perm32", k_perm32, out, blocks, 8);
  hipFree(out);
  return 0;
}
