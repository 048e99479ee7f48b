// Probe: which XCC id do blocks see (vs blockIdx % 8), and what does a
// per-block dequeue (one returning atomicAdd by thread 0 + barrier) cost.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void who(int *xcc) {
  if (threadIdx.x == 0) xcc[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
}

// spin ~`work` iterations so the blocks overlap like rasterizer tiles
__global__ void __launch_bounds__(256) deq(int *heads, int stride, int mode, int work, float *sink) {
  __shared__ int s;
  if (threadIdx.x == 0) {
    int v = 0;
    if (mode == 1) v = atomicAdd(&heads[0], 1);
    if (mode == 2) {
      const int x = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7;
      v = atomicAdd(&heads[x * stride], 1);
    }
    s = v;
  }
  __syncthreads();
  float acc = (float)s;
  for (int i = 0; i < work; ++i) acc = acc * 0.999f + 1.0f;
  if (acc == 12345.f) sink[threadIdx.x] = acc;
}

int main() {
  const int nb = 8160;
  int *d;
  hipMalloc(&d, nb * 4);
  hipLaunchKernelGGL(who, dim3(nb), dim3(64), 0, 0, d);
  std::vector<int> h(nb);
  hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost);
  int hist[16][8] = {};
  for (int b = 0; b < nb; ++b) hist[h[b] & 15][b % 8]++;
  printf("xcc_id x (blockIdx %% 8) counts:\n");
  for (int x = 0; x < 16; ++x) {
    int tot = 0;
    for (int r = 0; r < 8; ++r) tot += hist[x][r];
    if (!tot) continue;
    printf("  xcc %2d:", x);
    for (int r = 0; r < 8; ++r) printf(" %5d", hist[x][r]);
    printf("\n");
  }
  int *heads;
  float *sink;
  hipMalloc(&heads, 4096 * 4);
  hipMalloc(&sink, 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int work : {0, 2000}) {
    for (int mode = 0; mode < 3; ++mode) {
      for (int stride : {1, 32}) {
        if (mode != 2 && stride != 1) continue;
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
          hipMemset(heads, 0, 4096 * 4);
          hipEventRecord(e0);
          hipLaunchKernelGGL(deq, dim3(nb), dim3(256), 0, 0, heads, stride, mode, work, sink);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms;
          hipEventElapsedTime(&ms, e0, e1);
          best = ms < best ? ms : best;
        }
        printf("work %4d mode %d (0 none, 1 one head, 2 per-XCC head) stride %2d: %.1f us\n", work,
               mode, stride, best * 1e3);
      }
    }
  }
  return 0;
}
