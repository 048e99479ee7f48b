// Per-step trainer glue around the rasterizer, one launch each, gfx950:
//
//   update_state   DefaultStrategy._update_state for packed=False
//                  (gsplat/strategy/default.py:213-262): grad2d += |scaled
//                  means2d.grad| and count += 1 where radii > 0, summed over
//                  cameras in camera order -- without torch.where's host sync
//                  and the six elementwise launches of the torch version.
//   activate_fwd   scales = exp(log_scales), opacities = sigmoid(logits)
//   activate_bwd   their VJPs with torch's formulas (exp: g * out;
//                  sigmoid_backward: g * (1 - out) * out), as the trainer's
//                  torch.exp / torch.sigmoid (examples/simple_trainer.py:565-566).
//   densify_*      DefaultStrategy's refine step (gsplat/strategy/default.py:
//                  264-340 _grow_gs / _prune_gs over ops.py:86-211 duplicate /
//                  split / remove) as ONE compaction: the reference rebuilds
//                  every parameter and both Adam moments three times (torch.cat
//                  for the duplicates, again for the split, index for the
//                  prune); here a plan pass classifies each Gaussian, a scan
//                  places the survivors, and one apply pass writes the final
//                  layout of all arrays once.
// All HBM-bound streaming kernels, one lane per Gaussian.
#include <string.h>

#include "common.h"
#include "../../include/gsplat_hip.h"

namespace gs {
namespace strat {

__global__ void __launch_bounds__(256)
update_state_kernel(int C, int64_t N, const float *__restrict__ g2d,
                    const int32_t *__restrict__ radii, float sx, float sy,
                    float *__restrict__ grad2d, float *__restrict__ count,
                    const int32_t *__restrict__ skip) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= N || (skip && *skip)) return;
  float acc = grad2d[g], cnt = count[g];
  bool any = false;
  for (int c = 0; c < C; ++c) {
    const int64_t i = (int64_t)c * N + g;
    if (radii[i] > 0) {
      const float2 v = *reinterpret_cast<const float2 *>(g2d + 2 * i);
      const float x = v.x * sx, y = v.y * sy;
      acc += sqrtf(x * x + y * y);  // .norm(dim=-1) of a 2-vector
      cnt += 1.f;
      any = true;
    }
  }
  if (any) {
    grad2d[g] = acc;
    count[g] = cnt;
  }
}

// The captured training step's input block (gsplat_hip_step_fetch): slot
// seq % ring of a host-mapped ring into the device block, its slot index
// into the block's last 8 bytes, seq += 1 -- by one wave.
struct StepFetch {
  const uint32_t *ring;  // null: nothing to fetch
  int64_t slot_words;
  int n_ring;
  int64_t *seq;
  uint32_t *blk;
};

GS_INLINE void step_fetch_wave(const StepFetch &f, int lane) {
  const int64_t q = *f.seq;
  const int64_t slot = q % f.n_ring;
  const uint32_t *src = f.ring + slot * f.slot_words;
  // the slot crosses PCIe: every load of a round is issued before any store
  // (a load / store loop pays one host round trip per 64 words -- the
  // compiler cannot move a load above a store that may alias it)
  constexpr int kU = 8;
  const int64_t nw = f.slot_words - 2;
  for (int64_t w0 = 0; w0 < nw; w0 += 64 * kU) {
    uint32_t v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t w = w0 + lane + 64 * u;
      v[u] = w < nw ? src[w] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t w = w0 + lane + 64 * u;
      if (w < nw) f.blk[w] = v[u];
    }
  }
  if (lane == 0) {
    reinterpret_cast<int64_t *>(f.blk)[f.slot_words / 2 - 1] = slot;
    *f.seq = q + 1;
  }
}

// fetch (the first kernel of a captured step): its first wave also fetches
// the step's input block
template <bool VEC>
__global__ void __launch_bounds__(256)
activate_fwd_kernel(int64_t n_s, int64_t n_o, const float *__restrict__ log_scales,
                    const float *__restrict__ logits, float *__restrict__ scales,
                    float *__restrict__ opacities, StepFetch fetch) {
  if (fetch.ring && blockIdx.x == 0 && threadIdx.x < 64) step_fetch_wave(fetch, threadIdx.x);
  // four elements per lane (16-B loads and stores where the arrays are
  // 16-B aligned; the same expf per element)
  const int64_t i4 = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (i4 + 4 <= n_s && VEC) {
    const float4 v = *reinterpret_cast<const float4 *>(log_scales + i4);
    *reinterpret_cast<float4 *>(scales + i4) = make_float4(expf(v.x), expf(v.y), expf(v.z), expf(v.w));
  } else {
    for (int64_t i = i4; i < min(i4 + 4, n_s); ++i) scales[i] = expf(log_scales[i]);
  }
  if (i4 + 4 <= n_o && VEC) {
    const float4 v = *reinterpret_cast<const float4 *>(logits + i4);
    *reinterpret_cast<float4 *>(opacities + i4) =
        make_float4(1.f / (1.f + expf(-v.x)), 1.f / (1.f + expf(-v.y)), 1.f / (1.f + expf(-v.z)),
                    1.f / (1.f + expf(-v.w)));
  } else {
    for (int64_t i = i4; i < min(i4 + 4, n_o); ++i) opacities[i] = 1.f / (1.f + expf(-logits[i]));
  }
}

inline bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }
inline unsigned activate_blocks(int64_t n) { return (unsigned)std::max<int64_t>((n + 1023) / 1024, 1); }

__global__ void __launch_bounds__(256)
activate_bwd_kernel(int64_t n_s, int64_t n_o, const float *__restrict__ scales,
                    const float *__restrict__ opacities, const float *__restrict__ v_scales,
                    const float *__restrict__ v_opacities, float *__restrict__ v_log_scales,
                    float *__restrict__ v_logits) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n_s) v_log_scales[i] = v_scales[i] * scales[i];
  if (i < n_o) {
    const float o = opacities[i];
    v_logits[i] = v_opacities[i] * (1.f - o) * o;
  }
}


// ------------------------------------------------------------ densification
// Final layout of the reference's duplicate -> split -> remove sequence:
//   [originals neither split nor pruned] ++ [duplicates not pruned]
//   ++ [first split child of each split Gaussian not pruned]
//   ++ [second split children, same order]
// (duplicate appends p[sel]; split keeps p[rest] -- the duplicates included,
// they are never split -- and appends the children sampled as [2, n, 3];
// remove is a stable filter).  A duplicate has its parent's parameters and
// so its prune decision; both children of a split share theirs (same scales
// and opacity).
enum : uint8_t { kKeep = 1, kDup = 2, kChild = 4, kSplit = 8, kDupAny = 16 };
constexpr int kRows = 5;  // block-count rows: one per flag bit
constexpr int kDB = 256;  // Gaussians per block

struct DensifyCfg {
  float grow_grad2d, grow_scale3d, prune_opa, prune_scale3d;
  float grow_scale2d, prune_scale2d;  // used only with radii2d (scale2d refine)
  int prune_big, revised_opacity;
};

GS_INLINE float sigmoid_t(float x) { return 1.f / (1.f + expf(-x)); }
// the split children's opacity logit and log-scale, as the reference's torch
// expressions (ops.py:152-167): log(exp(s) / 1.6) (a CUDA/HIP division by a
// CPU scalar is a multiplication by its float reciprocal), and
// logit(1 - sqrt(1 - sigmoid(o))) when revised
GS_INLINE float child_log_scale(float s) { return logf(expf(s) * (1.f / 1.6f)); }
GS_INLINE float child_logit(float o, bool revised) {
  if (!revised) return o;
  const float p = 1.f - sqrtf(1.f - sigmoid_t(o));
  return logf(p / (1.f - p));
}

__global__ void __launch_bounds__(kDB)
densify_plan_kernel(int64_t N, const float *__restrict__ grad2d, const float *__restrict__ count,
                    const float *__restrict__ log_scales, const float *__restrict__ logits,
                    const float *__restrict__ radii2d, DensifyCfg cfg, uint8_t *__restrict__ flags,
                    int64_t *__restrict__ block_counts /* [kRows][nb] */, int64_t nb) {
  __shared__ int wcnt[kRows][kDB / 64];
  const int64_t i = (int64_t)blockIdx.x * kDB + threadIdx.x;
  uint8_t f = 0;
  if (i < N) {
    const float g = grad2d[i] / fmaxf(count[i], 1.f);  // grad2d / count.clamp_min(1)
    const bool high = g > cfg.grow_grad2d;
    const float s0 = log_scales[3 * i], s1 = log_scales[3 * i + 1], s2 = log_scales[3 * i + 2];
    const float smax = fmaxf(fmaxf(expf(s0), expf(s1)), expf(s2));
    const bool small = smax <= cfg.grow_scale3d;
    const bool dup = high && small;
    bool split = high && !small;
    const float o = logits[i];
    bool prune = sigmoid_t(o) < cfg.prune_opa || (cfg.prune_big && smax > cfg.prune_scale3d);
    if (radii2d) {  // refine_scale2d_stop_iter > 0 (default.py:283-284, 325-326)
      split = split || radii2d[i] > cfg.grow_scale2d;
      prune = prune || (cfg.prune_big && radii2d[i] > cfg.prune_scale2d);
    }
    if (!split && !prune) f |= kKeep;
    if (dup && !prune) f |= kDup;
    if (dup) f |= kDupAny;
    if (split) {
      f |= kSplit;
      const float co = child_logit(o, cfg.revised_opacity);
      const float cmax = fmaxf(fmaxf(expf(child_log_scale(s0)), expf(child_log_scale(s1))),
                               expf(child_log_scale(s2)));
      bool cprune = sigmoid_t(co) < cfg.prune_opa || (cfg.prune_big && cmax > cfg.prune_scale3d);
      // the children inherit the running state, radii included (ops.py:172-176)
      if (radii2d) cprune = cprune || (cfg.prune_big && radii2d[i] > cfg.prune_scale2d);
      if (!cprune) f |= kChild;
    }
    flags[i] = f;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    const uint64_t m = __ballot((f >> k) & 1);
    if (lane == 0) wcnt[k][w] = __popcll(m);
  }
  __syncthreads();
  if (threadIdx.x < kRows) {
    int64_t t = 0;
    for (int q = 0; q < kDB / 64; ++q) t += wcnt[threadIdx.x][q];
    block_counts[threadIdx.x * nb + blockIdx.x] = t;
  }
}

// Exclusive scan of each of the kRows block-count rows (workgroup k scans row k);
// its total goes to totals[k].
__global__ void __launch_bounds__(1024)
densify_scan_kernel(int64_t nb, int64_t *__restrict__ block_counts, int64_t *__restrict__ totals) {
  int64_t *row = block_counts + blockIdx.x * nb;
  __shared__ int64_t wave_tot[16];
  __shared__ int64_t chunk_tot;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t carry = 0;
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = (i < nb) ? row[i] : 0;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wave_tot[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t run = 0;
      for (int q = 0; q < 16; ++q) {
        const int64_t t = wave_tot[q];
        wave_tot[q] = run;
        run += t;
      }
      chunk_tot = run;
    }
    __syncthreads();
    if (i < nb) row[i] = carry + wave_tot[wid] + x - v;
    carry += chunk_tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

constexpr int kMaxArrays = 24;
struct DensifyArrays {
  const float *src[kMaxArrays];
  float *dst[kMaxArrays];
  int row[kMaxArrays];   // floats per Gaussian
  int kind[kMaxArrays];  // GSPLAT_HIP_DENSIFY_* (include/gsplat_hip.h)
  int n;
  const float *means, *quats, *log_scales, *logits;  // the sources the children derive from
};

__global__ void __launch_bounds__(kDB)
densify_apply_kernel(int64_t N, const uint8_t *__restrict__ flags,
                     const int64_t *__restrict__ block_offsets /* [4][nb] scanned */, int64_t nb,
                     const int64_t *__restrict__ totals, const float *__restrict__ randn,
                     int revised_opacity, DensifyArrays arr) {
  __shared__ int wpre[4][kDB / 64];
  const int64_t i = (int64_t)blockIdx.x * kDB + threadIdx.x;
  const uint8_t f = i < N ? flags[i] : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int rank[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t m = __ballot((f >> k) & 1);
    rank[k] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (lane == 0) wpre[k][w] = __popcll(m);
  }
  __syncthreads();
  if (i >= N || f == 0) return;
  int64_t pos[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int64_t p = block_offsets[k * nb + blockIdx.x] + rank[k];
    for (int q = 0; q < w; ++q) p += wpre[k][q];
    pos[k] = p;
  }
  const int64_t nA = totals[0], nB = totals[1], nC = totals[2], nS = totals[3];
  const int64_t dA = pos[0], dB = nA + pos[1], dC0 = nA + nB + pos[2],
                dC1 = nA + nB + nC + pos[2];
  const bool isA = f & kKeep, isB = f & kDup, isC = f & kChild;
  // split children: mean + R(normalize(q)) diag(exp(s)) z_b  (ops.py:143-152),
  // z = randn[2, n_split, 3] indexed by this Gaussian's rank among ALL split
  // Gaussians (pruned children included)
  float c_mean[2][3], c_ls[3], c_logit = 0.f;
  if (isC) {
    const float *q = arr.quats + 4 * i;
    const float qn = fmaxf(sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]), 1e-12f);
    const float qw = q[0] / qn, qx = q[1] / qn, qy = q[2] / qn, qz = q[3] / qn;
    const float R[3][3] = {
        {1.f - 2.f * (qy * qy + qz * qz), 2.f * (qx * qy - qw * qz), 2.f * (qx * qz + qw * qy)},
        {2.f * (qx * qy + qw * qz), 1.f - 2.f * (qx * qx + qz * qz), 2.f * (qy * qz - qw * qx)},
        {2.f * (qx * qz - qw * qy), 2.f * (qy * qz + qw * qx), 1.f - 2.f * (qx * qx + qy * qy)}};
    float sc[3];
    for (int k = 0; k < 3; ++k) {
      sc[k] = expf(arr.log_scales[3 * i + k]);
      c_ls[k] = child_log_scale(arr.log_scales[3 * i + k]);
    }
    const int64_t j = pos[3];
    for (int b = 0; b < 2; ++b) {
      const float *z = randn + ((int64_t)b * nS + j) * 3;
      for (int r = 0; r < 3; ++r)
        c_mean[b][r] = arr.means[3 * i + r] +
                       (R[r][0] * sc[0] * z[0] + R[r][1] * sc[1] * z[1] + R[r][2] * sc[2] * z[2]);
    }
    c_logit = child_logit(arr.logits[i], revised_opacity);
  }
  for (int a = 0; a < arr.n; ++a) {
    const int row = arr.row[a], kind = arr.kind[a];
    const float *src = arr.src[a] + (int64_t)row * i;
    float *dst = arr.dst[a];
    const bool moment = kind == GSPLAT_HIP_DENSIFY_MOMENT;
    for (int e = 0; e < row; ++e) {
      const float v = src[e];
      if (isA) dst[dA * row + e] = v;
      if (isB) dst[dB * row + e] = moment ? 0.f : v;
      if (isC) {
        float v0 = v, v1 = v;
        if (moment) {
          v0 = v1 = 0.f;
        } else if (kind == GSPLAT_HIP_DENSIFY_MEANS) {
          v0 = c_mean[0][e];
          v1 = c_mean[1][e];
        } else if (kind == GSPLAT_HIP_DENSIFY_SCALES) {
          v0 = v1 = c_ls[e];
        } else if (kind == GSPLAT_HIP_DENSIFY_OPACITIES) {
          v0 = v1 = c_logit;
        }
        dst[dC0 * row + e] = v0;
        dst[dC1 * row + e] = v1;
      }
    }
  }
}

// gsplat_hip_step_fetch on its own: one wave; every later kernel of the
// step reads the block after this one (stream order).
__global__ void __launch_bounds__(64) step_fetch_kernel(StepFetch f) {
  step_fetch_wave(f, threadIdx.x);
}

// The ranks' agreed overflow flag into the overflow field of the step's row
// of the host-mapped count ring (gsplat_hip_status_to_ring).
__global__ void __launch_bounds__(64) status_to_ring_kernel(const int32_t *status,
                                                            int64_t *ring, const int64_t *slot) {
  if (threadIdx.x == 0 && status[0] != 0) ring[4 * slot[0] + 2] = 1;
}

}  // namespace strat
}  // namespace gs

using namespace gs;

// Host-mapped, coherent memory (fine-grained: GPU reads see the host's
// latest stores at kernel start, GPU stores are visible to the host once the
// kernel is complete), zeroed.  For the captured step's input and count rings.
extern "C" int gsplat_hip_host_mapped_alloc(int64_t bytes, void **host_ptr, void **device_ptr) {
  GS_REQUIRE(bytes > 0 && host_ptr && device_ptr, "host_mapped_alloc: bad arguments");
  void *h = nullptr;
  GS_HIP(hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent));
  memset(h, 0, (size_t)bytes);
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    GS_REQUIRE(false, "host_mapped_alloc: no device pointer");
  }
  *host_ptr = h;
  *device_ptr = d;
  return 0;
}

extern "C" int gsplat_hip_host_mapped_free(void *host_ptr) {
  if (host_ptr) GS_HIP(hipHostFree(host_ptr));
  return 0;
}

extern "C" int gsplat_hip_step_fetch(const void *ring_device, int64_t slot_bytes, int n_ring,
                                     int64_t *seq_device, void *block_device, void *stream) {
  GS_REQUIRE(ring_device && seq_device && block_device && n_ring > 0,
             "step_fetch: null buffer or empty ring");
  GS_REQUIRE(slot_bytes >= 16 && slot_bytes % 8 == 0 && slot_bytes <= 65536,
             "step_fetch: slot_bytes %lld not a multiple of 8 in [16, 65536]",
             (long long)slot_bytes);
  const strat::StepFetch f{reinterpret_cast<const uint32_t *>(ring_device), slot_bytes / 4, n_ring,
                           seq_device, reinterpret_cast<uint32_t *>(block_device)};
  hipLaunchKernelGGL(strat::step_fetch_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, f);
  GS_CHECK_LAUNCH("step_fetch");
  return 0;
}

extern "C" int gsplat_hip_status_to_ring(const int32_t *status_device, void *ring_device,
                                         const int64_t *slot_device, void *stream) {
  GS_REQUIRE(status_device && ring_device && slot_device, "status_to_ring: null buffer");
  hipLaunchKernelGGL(strat::status_to_ring_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     status_device, reinterpret_cast<int64_t *>(ring_device), slot_device);
  GS_CHECK_LAUNCH("status_to_ring");
  return 0;
}

extern "C" int gsplat_hip_update_state(int C, int64_t N, const float *means2d_grad,
                                       const int32_t *radii, float scale_x, float scale_y,
                                       float *grad2d, float *count, const int32_t *skip_device,
                                       void *stream) {
  GS_REQUIRE(C >= 0 && N >= 0, "update_state: bad sizes C=%d N=%lld", C, (long long)N);
  if (N == 0 || C == 0) return 0;
  hipLaunchKernelGGL(strat::update_state_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, C, N, means2d_grad, radii, scale_x, scale_y, grad2d,
                     count, skip_device);
  GS_CHECK_LAUNCH("update_state");
  return 0;
}

extern "C" int gsplat_hip_activate_fwd(int64_t n_scales, int64_t n_opacities,
                                       const float *log_scales, const float *logits,
                                       float *scales, float *opacities, void *stream) {
  const int64_t n = n_scales > n_opacities ? n_scales : n_opacities;
  if (n <= 0) return 0;
  const bool vec = strat::aligned16(log_scales) && strat::aligned16(logits) &&
                   strat::aligned16(scales) && strat::aligned16(opacities);
  if (vec)
    hipLaunchKernelGGL(strat::activate_fwd_kernel<true>, dim3(strat::activate_blocks(n)), dim3(256),
                       0, (hipStream_t)stream, n_scales, n_opacities, log_scales, logits, scales,
                       opacities, strat::StepFetch{});
  else
    hipLaunchKernelGGL(strat::activate_fwd_kernel<false>, dim3(strat::activate_blocks(n)), dim3(256),
                       0, (hipStream_t)stream, n_scales, n_opacities, log_scales, logits, scales,
                       opacities, strat::StepFetch{});
  GS_CHECK_LAUNCH("activate_fwd");
  return 0;
}

extern "C" int gsplat_hip_activate_fwd_fetch(int64_t n_scales, int64_t n_opacities,
                                             const float *log_scales, const float *logits,
                                             float *scales, float *opacities,
                                             const void *ring_device, int64_t slot_bytes,
                                             int n_ring, int64_t *seq_device,
                                             void *block_device, void *stream) {
  GS_REQUIRE(ring_device && seq_device && block_device && n_ring > 0,
             "activate_fwd_fetch: null buffer or empty ring");
  GS_REQUIRE(slot_bytes >= 16 && slot_bytes % 8 == 0 && slot_bytes <= 65536,
             "activate_fwd_fetch: slot_bytes %lld not a multiple of 8 in [16, 65536]",
             (long long)slot_bytes);
  const strat::StepFetch f{reinterpret_cast<const uint32_t *>(ring_device), slot_bytes / 4, n_ring,
                           seq_device, reinterpret_cast<uint32_t *>(block_device)};
  const int64_t n = n_scales > n_opacities ? n_scales : n_opacities;
  const bool vec = strat::aligned16(log_scales) && strat::aligned16(logits) &&
                   strat::aligned16(scales) && strat::aligned16(opacities);
  if (vec)
    hipLaunchKernelGGL(strat::activate_fwd_kernel<true>, dim3(strat::activate_blocks(n)), dim3(256),
                       0, (hipStream_t)stream, n_scales, n_opacities, log_scales, logits, scales,
                       opacities, f);
  else
    hipLaunchKernelGGL(strat::activate_fwd_kernel<false>, dim3(strat::activate_blocks(n)), dim3(256),
                       0, (hipStream_t)stream, n_scales, n_opacities, log_scales, logits, scales,
                       opacities, f);
  GS_CHECK_LAUNCH("activate_fwd_fetch");
  return 0;
}

extern "C" int gsplat_hip_activate_bwd(int64_t n_scales, int64_t n_opacities, const float *scales,
                                       const float *opacities, const float *v_scales,
                                       const float *v_opacities, float *v_log_scales,
                                       float *v_logits, void *stream) {
  const int64_t n = n_scales > n_opacities ? n_scales : n_opacities;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(strat::activate_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n_scales, n_opacities, scales, opacities, v_scales,
                     v_opacities, v_log_scales, v_logits);
  GS_CHECK_LAUNCH("activate_bwd");
  return 0;
}

extern "C" int64_t gsplat_hip_densify_workspace_bytes(int64_t N) {
  const int64_t nb = (N + strat::kDB - 1) / strat::kDB;
  return strat::kRows * nb * (int64_t)sizeof(int64_t) + ((N + 15) / 16) * 16;
}

extern "C" int gsplat_hip_densify_plan(int64_t N, const float *grad2d, const float *count,
                                       const float *log_scales, const float *logits,
                                       const float *radii2d, float grow_grad2d,
                                       float grow_scale3d, float prune_opa, int prune_big,
                                       float prune_scale3d, float grow_scale2d,
                                       float prune_scale2d, int revised_opacity, void *workspace,
                                       int64_t *totals, void *stream) {
  GS_REQUIRE(N >= 0, "densify_plan: bad N=%lld", (long long)N);
  const int64_t nb = (N + strat::kDB - 1) / strat::kDB;
  int64_t *bc = (int64_t *)workspace;
  uint8_t *flags = (uint8_t *)(bc + strat::kRows * nb);
  hipStream_t st = (hipStream_t)stream;
  if (N == 0) {
    GS_HIP(gs::zero_async(totals, strat::kRows * sizeof(int64_t), st));
    return 0;
  }
  strat::DensifyCfg cfg{grow_grad2d, grow_scale3d, prune_opa, prune_scale3d,
                        grow_scale2d, prune_scale2d, prune_big, revised_opacity};
  hipLaunchKernelGGL(strat::densify_plan_kernel, dim3((unsigned)nb), dim3(strat::kDB), 0, st, N,
                     grad2d, count, log_scales, logits, radii2d, cfg, flags, bc, nb);
  GS_CHECK_LAUNCH("densify_plan");
  hipLaunchKernelGGL(strat::densify_scan_kernel, dim3(strat::kRows), dim3(1024), 0, st, nb, bc,
                     totals);
  GS_CHECK_LAUNCH("densify_scan");
  return 0;
}

extern "C" int gsplat_hip_densify_apply(int64_t N, const void *workspace, const int64_t *totals,
                                        const float *randn, int revised_opacity, int n_arrays,
                                        const float *const *src, float *const *dst,
                                        const int32_t *row_floats, const int32_t *kinds,
                                        const float *means, const float *quats,
                                        const float *log_scales, const float *logits,
                                        void *stream) {
  GS_REQUIRE(N >= 0 && n_arrays >= 0 && n_arrays <= strat::kMaxArrays,
             "densify_apply: bad sizes N=%lld n_arrays=%d (max %d)", (long long)N, n_arrays,
             strat::kMaxArrays);
  if (N == 0) return 0;
  const int64_t nb = (N + strat::kDB - 1) / strat::kDB;
  strat::DensifyArrays a{};
  a.n = n_arrays;
  for (int k = 0; k < n_arrays; ++k) {
    GS_REQUIRE(kinds[k] >= GSPLAT_HIP_DENSIFY_COPY && kinds[k] <= GSPLAT_HIP_DENSIFY_MOMENT,
               "densify_apply: array %d has unknown kind %d", k, kinds[k]);
    GS_REQUIRE(row_floats[k] > 0 && (kinds[k] != GSPLAT_HIP_DENSIFY_MEANS || row_floats[k] == 3) &&
                   (kinds[k] != GSPLAT_HIP_DENSIFY_SCALES || row_floats[k] == 3) &&
                   (kinds[k] != GSPLAT_HIP_DENSIFY_OPACITIES || row_floats[k] == 1),
               "densify_apply: array %d: %d floats per Gaussian for kind %d", k, row_floats[k],
               kinds[k]);
    a.src[k] = src[k];
    a.dst[k] = dst[k];
    a.row[k] = row_floats[k];
    a.kind[k] = kinds[k];
  }
  a.means = means;
  a.quats = quats;
  a.log_scales = log_scales;
  a.logits = logits;
  const int64_t *bc = (const int64_t *)workspace;
  const uint8_t *flags = (const uint8_t *)(bc + strat::kRows * nb);
  hipLaunchKernelGGL(strat::densify_apply_kernel, dim3((unsigned)nb), dim3(strat::kDB), 0,
                     (hipStream_t)stream, N, flags, bc, nb, totals, randn, revised_opacity, a);
  GS_CHECK_LAUNCH("densify_apply");
  return 0;
}
