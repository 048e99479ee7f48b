/*
 * gsplat_hip.h -- C ABI of libgsplat_hip.so, the MI355X (gfx950) backend for
 * the gsplat rasterization hot path.
 *
 * Conventions
 *   - Plain device pointers (HIP/torch allocations on the current device),
 *     element counts and a `stream` (hipStream_t passed as void*).  Every
 *     kernel is enqueued on `stream`; nothing touches the default stream,
 *     nothing allocates, nothing synchronises.
 *   - All float tensors are contiguous fp32, row-major, shapes as documented.
 *   - Return value: 0 = ok, 1 = argument error, 2 = HIP error; the message is
 *     available from gsplat_hip_last_error() (thread-local).
 *   - Optional inputs/outputs are NULL when absent.
 *   - Gradient outputs are fully written by the call (zeroed on `stream`
 *     where accumulation is needed); callers may pass uninitialised memory.
 *
 * Each entry point names the reference interface it replaces
 * (hieu1999210/gsplat-triton, paths relative to the repository root).
 */
#ifndef GSPLAT_HIP_H
#define GSPLAT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char *gsplat_hip_last_error(void);
/* 29: the lazy SH-Adam entries of 28 (gsplat_hip_sh_colors_fwd_lazy,
 * gsplat_hip_sh_lazy_flush and the lazy arguments of the fused SH backward)
 * removed -- measured slower.
 * 30: gsplat_hip_l1_ssim_loss_fused_fwd_ring (the loss also into a device
 * ring slot chosen by a device step counter), gsplat_hip_set_fwd_split_div.
 * 31: gsplat_hip_projection_bwd_adam, gsplat_hip_graph_memcpy_census.
 * 32: gsplat_hip_status_to_ring; n_isects_device of the 2DGS rasterizer.
 * 33: colours-only 2DGS renders (render_normals / distort / median and
 *     median_ids NULL in gsplat_hip_rasterize_2dgs_fwd and _bwd); the 2DGS
 *     rasterizer's last colour channel from a separate depths array
 *     (depths / v_depths of _pack_records, _fwd, _bwd);
 *     gsplat_hip_projection_2dgs_bwd_adam; v_normals may be NULL in the
 *     2DGS rasterizer's backward (output) and projection backward (input);
 *     isect_ids alone may be NULL in the sorted emission (flatten_ids and
 *     offsets written: a rasterizer that gathers by id).
 * 34: gsplat_hip_isect_write_sorted_capped_surfel (tile culling of large
 *     surfels in the captured 2DGS step); gsplat_hip_set_fwd_split_threshold,
 *     gsplat_hip_fwd_split_threshold
 *     (the split-forward variant chosen once by the caller: deterministic
 *     renders); gsplat_hip_watchdog_arm / _beat / _disarm (bounded waits of
 *     a multi-GPU job); gsplat_hip_debug_set_lane_histogram, the
 *     deferred-SH gsplat_hip_adam_step_bounded and the compiled-in variants
 *     measured slower removed. */
int gsplat_hip_abi_version(void);

/* ---------------------------------------------------------------------------
 * Fused EWA projection (pinhole).
 * Replaces fused_projection_fwd() / fused_projection_fwd_kernel
 *   gsplat/triton_impl/fused_projection_fwd.py:16-307, called from
 *   _FullyFusedProjection.forward (gsplat/triton_impl/_wrapper.py:304-353).
 * means[N,3] quats[N,4] (16-B aligned) scales[N,3] viewmats[C,4,4] Ks[C,3,3]
 * -> radii i32[C,N], means2d[C,N,2], depths[C,N], conics[C,N,3],
 *    compensations[C,N] (NULL unless calc_compensations).
 * Entries with radii == 0 have means2d/conics/compensations written as 0.
 */
int gsplat_hip_projection_fwd(int C, int N, const float *means, const float *quats,
                              const float *scales, const float *viewmats, const float *Ks,
                              int width, int height, float eps2d, float near_plane,
                              float far_plane, float radius_clip, int32_t *radii,
                              float *means2d, float *depths, float *conics,
                              float *compensations, void *stream);

/* Replaces fused_projection_bwd() / fused_projection_bwd_kernel
 *   gsplat/triton_impl/fused_projection_bwd.py:24-465, called from
 *   _FullyFusedProjection.backward (gsplat/triton_impl/_wrapper.py:355-426).
 * Only (c, n) with radii > 0 contribute.  v_viewmats[C,4,4] may be NULL
 * (viewmats does not require grad, _wrapper.py:394); v_depths may be NULL
 * (depths without a gradient, read as zeros -- no zero-filled buffer). */
int gsplat_hip_projection_bwd(int C, int N, const float *means, const float *quats,
                              const float *scales, const float *viewmats, const float *Ks,
                              int width, int height, float eps2d, const int32_t *radii,
                              const float *conics, const float *compensations,
                              const float *v_means2d, const float *v_depths,
                              const float *v_conics, const float *v_compensations,
                              float *v_means, float *v_quats, float *v_scales,
                              float *v_viewmats, void *stream);

/* gsplat_hip_projection_bwd (C == 1) with the trainer's geometry Adam step
 * fused in (ABI 31): no gradient is stored; params / exp_avgs / exp_avg_sqs
 * [4] = means [N,3], log-scales [N,3], quats [N,4], logits [N] (the trainer's
 * parameters, in its order; `scales` is exp(log-scales)) are updated in place with
 * torch.optim.Adam from g_means = v_means + v_dirs, g_quats = v_quats,
 * g_logscales = v_scales * scales, g_logits = v_opac * (1 - opac) * opac
 * (v_dirs / v_opac may be NULL: zero).  lrs[4] and the 1-based step, or
 * hyper_device f32[8] (lr_i / (1 - beta1^t), 1 / sqrt(1 - beta2^t) per group;
 * a captured step); skip_device (may be NULL) non-zero updates nothing.
 * Bit-identical to projection_bwd + activate_bwd + adam_step. */
int gsplat_hip_projection_bwd_adam(
    int N, const float *means, const float *quats, const float *scales, const float *viewmats,
    const float *Ks, int width, int height, float eps2d, const int32_t *radii,
    const float *conics, const float *v_means2d, const float *v_depths, const float *v_conics,
    const float *v_dirs, const float *v_opac, const float *opac, float *const *params,
    float *const *exp_avgs, float *const *exp_avg_sqs, const float *lrs, float beta1,
    float beta2, float eps, int step, const float *hyper_device, const int32_t *skip_device,
    void *stream);

/* ---------------------------------------------------------------------------
 * Spherical harmonics, degree 0..4, RGB.
 * Replaces sh_to_color_fwd() (gsplat/triton_impl/sh_fwd.py:194-233) and the
 * mask zeroing of _SphericalHarmonics.forward (_wrapper.py:555-572).
 * dirs[n,3], coeffs[n_coeff_rows,K,3] (row i uses coeff row i % n_coeff_rows,
 * so [N,K,3] coefficients broadcast over C cameras need no copy),
 * masks u8[n] or NULL -> colors[n,3] (0 where masks[i] == 0).
 * If coeffs_rest is non-NULL the coefficients are split as the trainer holds
 * them: coeffs = DC term [rows,1,3], coeffs_rest = bases 1..K-1 [rows,K-1,3]
 * (replaces the per-step torch.cat of sh0/shN, examples/simple_trainer.py:469). */
int gsplat_hip_sh_fwd(int degree, int64_t n, int64_t n_coeff_rows, int K, const float *dirs,
                      const float *coeffs, const float *coeffs_rest, const uint8_t *masks,
                      float *colors, void *stream);

/* Replaces sh_to_color_bwd() (gsplat/triton_impl/sh_bwd.py:383-436) and
 * _SphericalHarmonics.backward (_wrapper.py:574-593).
 * -> v_coeffs[n,K,3] (bases >= (degree+1)^2 and masked rows are 0),
 *    v_dirs[n,3] or NULL.  Split form: v_coeffs [n,1,3] + v_coeffs_rest [n,K-1,3]. */
int gsplat_hip_sh_bwd(int degree, int64_t n, int64_t n_coeff_rows, int K, const float *dirs,
                      const float *coeffs, const float *coeffs_rest, const uint8_t *masks,
                      const float *v_colors, float *v_coeffs, float *v_coeffs_rest,
                      float *v_dirs, void *stream);

/* rasterization()'s colour path fused (gsplat/rendering.py:396-406 with the
 * SH of _wrapper.py:596-620): colors[C,N,3] = clamp_min(SH(degree, means -
 * campos) + 0.5, 0) with campos = -R^T t from viewmats[C,4,4] (instead of
 * torch.inverse), rows with radii[C,N] <= 0 -> 0.5 (the reference zeroes
 * masked SH colours, then adds 0.5).  Coefficient layout as gsplat_hip_sh_fwd.
 * Backward: v_coeffs(/v_coeffs_rest) per row with the clamp_min mask
 * (sh + 0.5 >= 0), v_dirs[C,N,3] = d loss / d means per camera (NULL: skip). */
int gsplat_hip_sh_colors_fwd(int degree, int C, int64_t N, int64_t n_coeff_rows, int K,
                             const float *means, const float *viewmats, const float *coeffs,
                             const float *coeffs_rest, const int32_t *radii, float *colors,
                             void *stream);
int gsplat_hip_sh_colors_bwd(int degree, int C, int64_t N, int64_t n_coeff_rows, int K,
                             const float *means, const float *viewmats, const float *coeffs,
                             const float *coeffs_rest, const int32_t *radii,
                             const float *v_colors, float *v_coeffs, float *v_coeffs_rest,
                             float *v_dirs, void *stream);

/* ---------------------------------------------------------------------------
 * Tile intersection.  Replaces isect_tiles() (gsplat/triton_impl/isect_tiles.py:13-131)
 * as three calls so that the caller can size the outputs after ONE device->host
 * read of n_isects (the reference's cumsum(...)[-1].item(), isect_tiles.py:101-102):
 *   1. gsplat_hip_isect_count: tiles_per_gauss i32[G] + per-block prefixes in
 *      `workspace` (gsplat_hip_isect_workspace_bytes(G) bytes) + totals_device[2]
 *      (int64 on device): {n_isects, n_visible = #Gaussians with >= 1 tile}.
 *   2. gsplat_hip_isect_write: isect_ids i64[n_isects], flatten_ids i32[n_isects]
 *      (unsorted; Gaussian-major, tile-row-major order).  tile_bits =
 *      (tile_width*tile_height - 1).bit_length() (Triton convention, isect_tiles.py:105).
 *      camera_ids i32[G] for packed inputs, else NULL and cam = i / N.
 *   3. gsplat_hip_radix_sort: stable sort on bits [0, 32+tile_bits+cam_bits)
 *      (replaces radix_sort, gsplat/triton_impl/radix_sort/radix_sort.cu:9-62).
 * G = C*N Gaussians (non-packed) or nnz (packed). */
int64_t gsplat_hip_isect_workspace_bytes(int64_t n_gaussians);
int gsplat_hip_isect_count(int64_t n_gaussians, const float *means2d, const int32_t *radii,
                           int tile_size, int tile_width, int tile_height,
                           int32_t *tiles_per_gauss, void *workspace,
                           int64_t *totals_device, void *stream);
int gsplat_hip_isect_write(int64_t n_gaussians, int N, const float *means2d,
                           const int32_t *radii, const float *depths, const int32_t *camera_ids,
                           int tile_size, int tile_width, int tile_height, int tile_bits,
                           const void *workspace, int64_t *isect_ids, int32_t *flatten_ids,
                           void *stream);
/* Sorted emission in one call (the sort=True path of isect_tiles): writes the
 * SAME isect_ids / flatten_ids as write + radix_sort, but sorts only 32-bit
 * keys: a stable depth sort of the n_visible Gaussians, emission in that
 * order, then a stable sort by the tile_bits+cam_bits (camera, tile) bits.
 * count_workspace is step 1's workspace; key_bits = tile_bits + cam_bits <= 32. */
int64_t gsplat_hip_isect_sorted_workspace_bytes(int64_t n_visible, int64_t n_isects,
                                                int key_bits);
int gsplat_hip_isect_write_sorted(int64_t n_gaussians, int N, const float *means2d,
                                  const int32_t *radii, const float *depths,
                                  const int32_t *camera_ids, const int32_t *tiles_per_gauss,
                                  int tile_size, int tile_width, int tile_height, int tile_bits,
                                  int cam_bits, const void *count_workspace, int64_t n_visible,
                                  int64_t n_isects, void *workspace, int64_t workspace_bytes,
                                  int64_t *isect_ids, int32_t *flatten_ids, int n_cameras,
                                  int32_t *offsets, int32_t *rank_ids, int32_t *vis_rank,
                                  void *stream);
/* n_cameras / offsets (ABI 27): offsets (may be NULL) receives the tile
 * offsets i32[n_cameras, tile_height, tile_width] as gsplat_hip_isect_offsets
 * computes them from the written ids (isect_offset.py:8-33).  With them the
 * isects are produced by the supertile expansion (csrc/isect_st.h: pairs of
 * (4x4-tile supertile, Gaussian) in depth order, one stable pass over those,
 * then every isect written once at its final slot; up to 2047 supertiles,
 * GSPLAT_HIP_ISECT_ST=0 for the emission + tile sort) -- the same ids. */
/* The same sorted emission with NO host sync (ABI 20; the reference reads
 * n_isects with .item(), isect_tiles.py:101-102): the totals stay on the
 * device (step 1's totals_device), isect_ids / flatten_ids have `capacity`
 * slots and every launch is sized for it.  counts_device i64[4] receives
 * {isects written -- 0 when they do not fit --, n_visible, 1 if they did not
 * fit, n_isects}; status_device[0] (may be NULL) gets bit 0 set on overflow and keeps it
 * (sticky, cleared by the caller).  Pass counts_device as the n_isects_device
 * of gsplat_hip_isect_offsets / gsplat_hip_rasterize_*, with n_isects =
 * capacity.  The written isects equal gsplat_hip_isect_write_sorted's.
 * counts_host_ring / slot_device (ABI 22, both NULL or both set): the four
 * counts also go to row slot_device[0] of an i64[ring][4] host-mapped
 * buffer (gsplat_hip_host_mapped_alloc) -- a captured step's overflow check
 * reads them there without a device->host copy. */
int64_t gsplat_hip_isect_sorted_capped_workspace_bytes(int64_t n_gaussians, int64_t capacity,
                                                       int key_bits);
int gsplat_hip_isect_write_sorted_capped(
    int64_t n_gaussians, int N, const float *means2d, const int32_t *radii, const float *depths,
    const int32_t *camera_ids, const int32_t *tiles_per_gauss, int tile_size, int tile_width,
    int tile_height, int tile_bits, int cam_bits, const void *count_workspace,
    const int64_t *totals_device, int64_t capacity, int64_t *counts_device,
    int32_t *status_device, int64_t *counts_host_ring, const int64_t *slot_device,
    void *workspace, int64_t workspace_bytes, int64_t *isect_ids, int32_t *flatten_ids,
    int n_cameras, int32_t *offsets, int32_t *rank_ids, int32_t *vis_rank, void *stream);
/* rank_ids / vis_rank (ABI 27, both NULL or both set; only when
 * gsplat_hip_isect_ranked says the supertile expansion runs): rank_ids
 * i32[n_isects] = the depth rank of each isect's Gaussian among the visible
 * Gaussians (flatten_ids[i] is the Gaussian itself), vis_rank i32[G] = that
 * rank for every Gaussian with tiles_per_gauss > 0 (other entries untouched):
 * the render records and gradient rows can then be indexed by rank.
 * When the supertile expansion runs, isect_ids and flatten_ids may both be
 * NULL (rank_ids and offsets set: a rasterizer that walks ranks), or
 * isect_ids alone (ABI 33; flatten_ids and offsets set: one that gathers by
 * Gaussian id and reads the offsets, not the 64-bit keys). */
int gsplat_hip_isect_ranked(int n_cameras, int tile_width, int tile_height);
/* The capped emission for the 2DGS rasterizer with tile culling of large
 * surfels (ABI 34; the captured 2DGS training step): a surfel whose tile
 * rectangle spans more than 16 supertiles gets isects only in the tiles its
 * UV-plane image can reach (the rasterizer's own strip test,
 * csrc/surfel_cull.h, on the whole tile); near-degenerate surfels (the
 * reference AABB's 1e-4 floor) otherwise cover every tile (41 % of the isects
 * at M5).  The rasterizer would cull exactly those isects on every strip, so
 * renders and gradients are unchanged; the isect list, an internal of the
 * training step, is not the reference's.  flatten_ids and offsets written
 * (no isect ids, no ranks); counts_device[0] receives the number written
 * (fewer than counts_device[3], the tile-rectangle count, which the capacity
 * check uses).  means2d [G][2], ray_transforms [G][3][3], opacities [G] of
 * the (camera, surfel) rows; non-packed (camera_ids NULL).  No reference
 * counterpart (the reference's isect is bit-exact; this path is not). */
int gsplat_hip_isect_write_sorted_capped_surfel(
    int64_t n_gaussians, int N, const float *means2d, const int32_t *radii, const float *depths,
    const int32_t *camera_ids, const int32_t *tiles_per_gauss, int tile_size, int tile_width,
    int tile_height, int tile_bits, int cam_bits, const void *count_workspace,
    const int64_t *totals_device, int64_t capacity, int64_t *counts_device,
    int32_t *status_device, int64_t *counts_host_ring, const int64_t *slot_device,
    void *workspace, int64_t workspace_bytes, int32_t *flatten_ids, int n_cameras,
    int32_t *offsets, const float *ray_transforms, const float *opacities, void *stream);
/* Sorted emission, tile-first (the default of isect_tiles(sort=True)): the
 * SAME isect_ids / flatten_ids again, from Gaussian-major emission with
 * 32-bit (camera, tile) keys, a stable sort by those keys, and a segmented
 * sort of each (camera, tile) run by depth bits.  No depth sort of the
 * Gaussians; n_isects < 2^31. */
int64_t gsplat_hip_isect_tilefirst_workspace_bytes(int64_t n_isects, int n_tiles_total,
                                                   int key_bits);
int gsplat_hip_isect_write_tilefirst(int64_t n_gaussians, int N, const float *means2d,
                                     const int32_t *radii, const float *depths,
                                     const int32_t *camera_ids, int tile_size, int tile_width,
                                     int tile_height, int n_cameras, int tile_bits, int cam_bits,
                                     const void *count_workspace, int64_t n_isects,
                                     void *workspace, int64_t workspace_bytes,
                                     int64_t *isect_ids, int32_t *flatten_ids, void *stream);
int64_t gsplat_hip_sort_workspace_bytes(int64_t n);
int gsplat_hip_radix_sort(int64_t n, int n_bits, const int64_t *keys_in, const int32_t *vals_in,
                          int64_t *keys_out, int32_t *vals_out, void *workspace,
                          int64_t workspace_bytes, void *stream);

/* Replaces get_isect_offsets() (gsplat/triton_impl/isect_offset.py:8-63).
 * offsets i32[C,tile_height,tile_width]: index of the first sorted isect of
 * each tile (= number of isects with a smaller (camera, tile) key).
 * n_isects_device (ABI 20, may be NULL): the count on the device, n_isects
 * then being the capacity of isect_ids (gsplat_hip_isect_write_sorted_capped). */
int gsplat_hip_isect_offsets(int64_t n_isects, const int64_t *n_isects_device,
                             const int64_t *isect_ids, int C, int tile_width, int tile_height,
                             int32_t *offsets, void *stream);

/* ---------------------------------------------------------------------------
 * Rasterization.  D in {1,2,3,4,8,16,32} (gsplat_hip_rasterize_supported_channels);
 * tile_size <= 16.
 * Replaces rasterize_to_pixels_fwd() (gsplat/triton_impl/rasterize_to_pixels_fwd.py:199-285)
 * called from _RasterizeToPixels.forward (_wrapper.py:46-102).
 * means2d[G,2] conics[G,3] colors[G,D] opacities[G] (G = C*N or nnz),
 * backgrounds[C,D] or NULL, masks u8[C,th,tw] or NULL (true = skip tile),
 * isect_offsets i32[C,th,tw], flatten_ids i32[n_isects]
 * -> render_colors[C,H,W,D], render_alphas[C,H,W], last_ids i32[C,H,W],
 *    and, when `state` is non-NULL, the per-pixel compositing state at every
 *    chunk boundary of a long tile (gsplat_hip_rasterize_fwd_state_bytes bytes;
 *    0 bytes = no state) that lets the backward split long tiles into chunks
 *    that run in parallel, plus the forward's heaviest-tiles-first dispatch
 *    order.  Keep it for the matching gsplat_hip_rasterize_bwd. */
int gsplat_hip_rasterize_supported_channels(int D);
/* Optional: queue the forward's per-launch preparation (its dispatch order,
 * kept in `state`) ahead of gsplat_hip_rasterize_fwd on the same stream and
 * host thread, so the forward call launches the rasterizer kernel alone
 * (lets a caller time that kernel by itself).  Without it the forward does
 * the preparation itself. */
/* n_isects_device (here, in _fwd and in _bwd; ABI 20; 16x16 tiles, else
 * NULL): the isect count on the device, n_isects being the capacity of
 * flatten_ids (the sync-free isect, gsplat_hip_isect_write_sorted_capped). */
int gsplat_hip_rasterize_prepare(int C, int D, int tile_size, int tile_width, int tile_height,
                                 const int32_t *isect_offsets, int64_t n_isects,
                                 const int64_t *n_isects_device, void *state,
                                 int64_t state_bytes, void *stream);
int64_t gsplat_hip_rasterize_fwd_state_bytes(int C, int D, int tile_size, int tile_width,
                                             int tile_height, int64_t n_isects);
/* Optional render records (16x16 tiles, D <= 10): one 64-B row per Gaussian
 * [x, y, conic(3), opacity, colour(D), pad] packed from the four attribute
 * arrays, so that the rasterizer's per-isect gather (the four separate loads
 * of rasterize_to_pixels_fwd.py:93-145 / rasterize_to_pixels_bwd.py:110-125)
 * reads one 64-B sector.  record_floats: floats per row (16), 0 when the
 * configuration has no record path.  pack_records writes records f32[G][16];
 * rows with visible[g] <= 0 (e.g. tiles_per_gauss; NULL = all rows) are never
 * gathered and are left unwritten.  Pass the same records (or NULL for the
 * plain gathers) to gsplat_hip_rasterize_fwd and _bwd. */
int gsplat_hip_rasterize_record_floats(int D, int tile_size);
int gsplat_hip_rasterize_pack_records(int64_t n_gaussians, int D, const float *means2d,
                                      const float *conics, const float *colors,
                                      const float *opacities, const int32_t *visible,
                                      const int32_t *vis_rank, float *records, void *stream);
/* vis_rank (ABI 27, may be NULL; needs visible): rank-indexed records -- the
 * row of Gaussian g is vis_rank[g] (its depth rank among the visible ones,
 * gsplat_hip_isect_write_sorted's vis_rank), so the live rows are the first
 * n_visible, in depth order.  The rasterizer then takes the isects' ranks
 * (rank_ids) in place of flatten_ids, and the backward (same vis_rank) sums
 * its gradient rows by rank and unpacks them to the Gaussians. */
int gsplat_hip_rasterize_fwd(int C, int D, int width, int height, int tile_size, int tile_width,
                             int tile_height, const float *means2d, const float *conics,
                             const float *colors, const float *opacities,
                             const float *backgrounds, const uint8_t *masks,
                             const int32_t *isect_offsets, int64_t n_isects,
                             const int64_t *n_isects_device, const int32_t *flatten_ids,
                             float *render_colors, float *render_alphas, int32_t *last_ids,
                             const float *records, void *state, int64_t state_bytes,
                             void *stream);

/* Replaces rasterize_to_pixels_bwd() (gsplat/triton_impl/rasterize_to_pixels_bwd.py:340-457)
 * called from _RasterizeToPixels.backward (_wrapper.py:104-182).
 * -> v_means2d[G,2], v_conics[G,3], v_colors[G,D], v_opacities[G],
 *    v_means2d_abs[G,2] or NULL (absgrad).
 * `workspace` must hold gsplat_hip_rasterize_bwd_workspace_bytes(...) bytes
 * (packed per-Gaussian gradient rows and the chunk work list of the 16x16
 * kernels; 0 bytes for other tile sizes).  render_colors / state: the forward's
 * outputs; with state == NULL every tile runs as one work item. */
int64_t gsplat_hip_rasterize_bwd_workspace_bytes(int64_t n_gaussians, int D, int tile_size,
                                                 int absgrad, int C, int tile_width,
                                                 int tile_height, int64_t n_isects);
/* v_render_alphas may be NULL (alphas without a gradient: read as zeros). */
int gsplat_hip_rasterize_bwd(int C, int64_t n_gaussians, int D, int width, int height,
                             int tile_size, int tile_width, int tile_height,
                             const float *means2d, const float *conics, const float *colors,
                             const float *opacities, const float *backgrounds,
                             const uint8_t *masks, const int32_t *isect_offsets,
                             int64_t n_isects, const int64_t *n_isects_device,
                             const int32_t *flatten_ids,
                             const float *render_alphas, const int32_t *last_ids,
                             const float *v_render_colors, const float *v_render_alphas,
                             float *v_means2d, float *v_conics, float *v_colors,
                             float *v_opacities, float *v_means2d_abs,
                             const float *render_colors, const float *records,
                             const void *state, int64_t state_bytes, void *workspace,
                             int64_t workspace_bytes, const int32_t *visible,
                             const int32_t *vis_rank, void *stream);
/* visible (ABI 27, may be NULL): i32[G] with visible[g] > 0 for every
 * Gaussian that has an isect (tiles_per_gauss); the 16x16 path then zeroes
 * and reads back only those Gaussians' gradient rows (the others' gradients
 * are written as zeros without reading anything).  With vis_rank and
 * n_isects_device both set, n_isects_device is the counts_device of
 * gsplat_hip_isect_write_sorted_capped and its n_visible (element 1) bounds
 * the rank-indexed rows, zeroed as one range. */

/* Debug/profiling: when device_buffer (u64[2*capacity_waves]) is non-NULL, the
 * 16x16 rasterizer kernels store each wave's (start, end) s_memrealtime stamps
 * (100 MHz) at [2w, 2w+1], w = global wave index (4 waves per tile).  Not part
 * of the reference surface; NULL disables (the default). */
int gsplat_hip_debug_set_timeline(uint64_t *device_buffer, int64_t capacity_waves);
/* Chunk length (isects, rounded up to a multiple of 64; <= 0 disables) of the
 * chunked 16x16 backward; returns the value in effect.  Default 1024, or the
 * GSPLAT_HIP_CHUNK environment variable.  Forward and backward of one
 * rasterization must run with the same setting. */
int gsplat_hip_debug_set_chunk(int isects);
/* Split mode of the 16x16 forward: tiles with more isects than the
 * threshold are rendered as parallel chunks (ABI 25: workgroups of the same
 * forward launch, dispatched before the whole tiles; the chunks hand their
 * transmittance products to later chunks; which tiles split is decided per
 * render on the device).
 * isects > 0: that threshold; 0: off; < 0: adaptive, max(2048, n_isects /
 * GSPLAT_HIP_FWD_SPLIT_DIV) (the default, or GSPLAT_HIP_FWD_SPLIT).  Returns
 * the previous mode.  Results do not depend on it beyond the float rounding
 * of the chunks' transmittance products. */
int gsplat_hip_debug_set_fwd_split(int isects);
/* The adaptive threshold's divisor (ABI 30): div > 0 sets it, div <= 0
 * restores the default (GSPLAT_HIP_FWD_SPLIT_DIV, else 550).  Returns the
 * divisor in effect before the call.  The trainer picks 1100 for scenes
 * whose pixels rarely terminate early (train_step.Trainer._tune_split). */
int gsplat_hip_set_fwd_split_div(int div);
/* The split forward's threshold (ABI 34): > 0 = always the split-capable
 * forward, tiles above that many isects split (which ones is decided per
 * render on the device); 0 = never split; -1 = the library default
 * (GSPLAT_HIP_FWD_SPLIT, else adaptive: max(2048, n_isects / divisor), the
 * split-capable variant launched when an earlier render's largest tile
 * exceeded it -- a heuristic read of host-mapped memory, speed only; the two
 * variants' renders differ by the chunk products' rounding).  The trainer
 * sets it once from its first render, so every later render -- eager or
 * captured -- runs the same variant with the same threshold.  Returns the
 * previous value (-1 for the adaptive default). */
int gsplat_hip_set_fwd_split_threshold(int isects);
/* The split threshold (isects per tile) for a render of n_isects with the
 * divisor in effect; -1 when splitting is off (ABI 34). */
int64_t gsplat_hip_fwd_split_threshold(int64_t n_isects);
/* Debug flags of the 16x16 rasterizer (ABI 25; default 0, or GSPLAT_HIP_DBG):
 * bit 0 = the backward skips its gradient atomics (timing experiments);
 * bit 2 = the backward skips its cross-lane reduction, bit 3 its gradient
 * algebra, bit 5 = the forward stores no chunk state (timing / traffic
 * attribution only: wrong gradients); bit 4 = the per-tile dispatch order
 * of the unsplit forward and the list order of the split forward's whole
 * tiles and of the backward's work items, and the 2DGS rasterizer's tile
 * order taken one tile after the other, instead of the XCD-grouped ones
 * (same results);
 * bit 1 = a chunk of a split tile never waits for an earlier chunk's
 * published product and computes it itself (the timeout path; results are
 * identical).  Bits 0, 2 and 3 also apply to the 2DGS colours-only (LEAN)
 * backward, which then runs its attribution instance; bit 6 runs that
 * instance with nothing skipped (its baseline).  Returns the previous flags. */
int gsplat_hip_debug_set_flags(int flags);

/* ---------------------------------------------------------------------------
 * Trainer-side kernels of the training step (not part of the 5-function
 * backend surface; used by gsplat_hip.train_step).
 *
 * Photometric loss terms of examples/simple_trainer.py:642-646:
 * fused_ssim(render, gt, padding="valid") (rahul-goel/fused-ssim@1272e21a,
 * examples/requirements.txt:22) and the L1 term.  Images [B,H,W,C] fp32.
 * fwd: sums[0] = sum of the SSIM map over the valid region, sums[1] = sum |img1-img2|
 *      (device floats, zeroed by the call); workspace = per-pixel partials.
 * bwd: grad_img1 = dloss[0]/n_map * dSSIMsum + dloss[1]/n_img * sign(img1-img2)
 *      where dloss (device, [2]) = dL/d(mean SSIM), dL/d(mean L1). */
int64_t gsplat_hip_ssim_workspace_bytes(int B, int H, int W, int C);
int gsplat_hip_ssim_l1_fwd(int B, int H, int W, int C, const float *img1, const float *img2,
                           float *sums, void *workspace, void *stream);
int gsplat_hip_ssim_l1_bwd(int B, int H, int W, int C, const float *img1, const float *img2,
                           const void *workspace, const float *dloss, float *grad_img1,
                           void *stream);
/* The trainer's whole loss in the same two launches (no scalar torch glue):
 * fwd: out[0] = (1-lam)*mean L1 + lam*(1 - mean SSIM), out[1] = mean SSIM,
 *      out[2] = mean L1 (device floats).
 * bwd: grad_img1 = dL/dimg1 for dL = g_loss[0] (device scalar). */
int gsplat_hip_l1_ssim_loss_fwd(int B, int H, int W, int C, const float *img1,
                                const float *img2, float lam, float *out, void *workspace,
                                void *stream);
int gsplat_hip_l1_ssim_loss_bwd(int B, int H, int W, int C, const float *img1,
                                const float *img2, const void *workspace, float lam,
                                const float *g_loss, float *grad_img1, void *stream);
/* The same loss with its gradient computed in the forward pass (ABI 16), the
 * training path: one kernel per 32x32 image tile recomputes the SSIM map
 * partials of the map pixels its pixels depend on and blurs them back, so no
 * per-pixel partials reach HBM.  C is 1 or 3.
 * fused_fwd: out[0..2] as l1_ssim_loss_fwd; grad_unit [B,H,W,C] = dout[0]/dimg1;
 *            workspace = gsplat_hip_l1_ssim_loss_fused_workspace_bytes.
 *            img2_index (ABI 21, may be NULL): device int64; img2 is then a
 *            stack of [B,H,W,C] images and image img2_index[0] is the target
 *            (a captured training step picks its camera's target on the device).
 *            x_stride (ABI 32, >= C): floats per pixel of img1 and grad_unit
 *            (img2 has C): an RGB+D render's colour channels read in place
 *            (x_stride 4, C 3); grad_unit's channels C .. x_stride-1 are
 *            written as zeros (the loss does not read them).
 * fused_bwd: grad_img1[i] = g_loss[0] * grad_unit[i] (16-B aligned buffers). */
int64_t gsplat_hip_l1_ssim_loss_fused_workspace_bytes(int B, int H, int W, int C);
int gsplat_hip_l1_ssim_loss_fused_fwd(int B, int H, int W, int C, int x_stride,
                                      const float *img1, const float *img2,
                                      const int64_t *img2_index, float lam, float *out,
                                      float *grad_unit, void *workspace, void *stream);
int gsplat_hip_l1_ssim_loss_fused_bwd(int64_t n, const float *grad_unit, const float *g_loss,
                                      float *grad_img1, void *stream);
/* fused_fwd_ring (ABI 30): fused_fwd, and the loss out[0] also written to
 * loss_ring[(seq_device[0] - 1) % ring_len] by the same reduction launch --
 * a captured training step returns that slot instead of copying its static
 * output after every replay (seq_device: the step counter the step's fetch
 * launch has already incremented; gsplat_hip/graph_step.py). */
int gsplat_hip_l1_ssim_loss_fused_fwd_ring(int B, int H, int W, int C, int x_stride,
                                           const float *img1, const float *img2,
                                           const int64_t *img2_index,
                                           float lam, float *out, float *grad_unit,
                                           void *workspace, float *loss_ring, int64_t ring_len,
                                           const int64_t *seq_device, void *stream);

/* The captured training step's per-step input without copy engines (ABI 22;
 * gsplat_hip/graph_step.py, not a reference function):
 * host_mapped_alloc: `bytes` of zeroed host memory, mapped and coherent
 *   (fine-grained), *host_ptr for the host, *device_ptr for kernels; free
 *   with host_mapped_free.
 * step_fetch: one-wave launch: slot = seq_device[0] % n_ring; copies the
 *   first slot_bytes - 8 bytes of ring slot `slot` (ring_device, n_ring
 *   slots of slot_bytes, a multiple of 8) into block_device, writes `slot`
 *   (i64) into its last 8 bytes and increments seq_device[0].  The host
 *   fills slot k % n_ring before the k-th launch and reuses it only after
 *   that launch's step has run. */
int gsplat_hip_host_mapped_alloc(int64_t bytes, void **host_ptr, void **device_ptr);
int gsplat_hip_host_mapped_free(void *host_ptr);
int gsplat_hip_step_fetch(const void *ring_device, int64_t slot_bytes, int n_ring,
                          int64_t *seq_device, void *block_device, void *stream);
/* gsplat_hip_activate_fwd whose launch also performs gsplat_hip_step_fetch
 * (its first wave; ABI 24): the first kernel of a captured step, one launch
 * instead of two. */
int gsplat_hip_activate_fwd_fetch(int64_t n_scales, int64_t n_opacities,
                                  const float *log_scales, const float *logits, float *scales,
                                  float *opacities, const void *ring_device, int64_t slot_bytes,
                                  int n_ring, int64_t *seq_device, void *block_device,
                                  void *stream);
/* Node census of a captured graph (ABI 26; host-side check of
 * gsplat_hip/graph_step.py, not a reference function): `graph` is a
 * hipGraph_t; counts[t] += the number of nodes of hipGraphNodeType t (t < 16,
 * larger types in counts[15]); for the first max_memsets memset nodes,
 * memsets[4k .. 4k+3] = (destination, bytes per row, rows, element size). */
int gsplat_hip_graph_node_census(void *graph, int64_t *counts, int64_t *memsets,
                                 int max_memsets);

/* The memcpy nodes of a captured graph (ABI 31): for the first max_nodes,
 * out[4k .. 4k+3] = (destination, source, bytes, hipMemcpyKind), -1 where
 * unreadable; *n_out = the number of memcpy nodes.  (RCCL's one-rank
 * all_to_all inside a captured Gaussian-sharded step copies the rank's own
 * block with such nodes.) */
int gsplat_hip_graph_memcpy_census(void *graph, int64_t *out, int max_nodes, int *n_out);

/* The ranks' agreed overflow flag of a captured multi-rank step (ABI 32;
 * gsplat_hip/graph_step.py, not a reference function): one-wave launch; when
 * status_device[0] != 0, sets the overflow field (index 2) of row
 * slot_device[0] of the host-mapped count ring ring_device (i64[4] rows, as
 * gsplat_hip_isect_write_sorted_capped's counts_host_ring). */
int gsplat_hip_status_to_ring(const int32_t *status_device, void *ring_device,
                              const int64_t *slot_device, void *stream);

/* DefaultStrategy._update_state for packed=False (gsplat/strategy/default.py:
 * 213-262): for every (c, g) with radii[c,g] > 0, in camera order,
 * grad2d[g] += |(means2d_grad[c,g,0]*scale_x, means2d_grad[c,g,1]*scale_y)|
 * and count[g] += 1.  scale_x = width/2 * C, scale_y = height/2 * C. */
/* skip_device (ABI 20, may be NULL): when *skip_device != 0 nothing is
 * accumulated (a void step of a captured training step). */
int gsplat_hip_update_state(int C, int64_t N, const float *means2d_grad, const int32_t *radii,
                            float scale_x, float scale_y, float *grad2d, float *count,
                            const int32_t *skip_device, void *stream);

/* The trainer's parameter activations (examples/simple_trainer.py:565-566)
 * in one launch each way: scales = exp(log_scales), opacities =
 * sigmoid(logits); backward with torch's formulas (g * exp, g * (1-o) * o). */
int gsplat_hip_activate_fwd(int64_t n_scales, int64_t n_opacities, const float *log_scales,
                            const float *logits, float *scales, float *opacities, void *stream);
int gsplat_hip_activate_bwd(int64_t n_scales, int64_t n_opacities, const float *scales,
                            const float *opacities, const float *v_scales,
                            const float *v_opacities, float *v_log_scales, float *v_logits,
                            void *stream);

/* DefaultStrategy's refine step -- _grow_gs + _prune_gs of
 * gsplat/strategy/default.py:264-340 over duplicate / split / remove of
 * gsplat/strategy/ops.py:86-211 -- as one compaction around one host sync.
 *
 * gsplat_hip_densify_plan classifies every Gaussian (grad2d / max(count, 1)
 * against grow_grad2d, max exp(log_scales) against grow_scale3d [absolute:
 * the caller multiplies by scene_scale], sigmoid(logits) against prune_opa,
 * and with prune_big also max exp(log_scales) against prune_scale3d; radii2d
 * (nullable) adds the refine_scale2d rules with grow_scale2d / prune_scale2d)
 * and writes totals[5] (device int64) = (originals kept, duplicates kept,
 * split Gaussians whose children are kept, split Gaussians, duplicated
 * Gaussians).  The caller reads them (the sync), allocates n_out = t0 + t1 +
 * 2 t2 rows per array and draws randn[2, t3, 3] (ops.py:147-152 draws
 * torch.randn(2, n_split, 3)); the reference's pruned count is
 * N + t4 + t3 - n_out.
 *
 * gsplat_hip_densify_apply writes the final layout
 *   [kept originals] ++ [kept duplicates] ++ [first children] ++ [second children]
 * of every array: kind COPY copies the row to every output, MEANS / SCALES /
 * OPACITIES give the children mean + R(q) diag(exp(s)) z_b, log(exp(s) / 1.6)
 * and (revised_opacity) logit(1 - sqrt(1 - sigmoid(o))), MOMENT copies the
 * row of a kept original and zero-fills the new rows (the optimizer state of
 * ops.py:104-105,169-170).  means/quats/log_scales/logits are the sources the
 * children derive from.  At most 24 arrays. */
#define GSPLAT_HIP_DENSIFY_COPY 0
#define GSPLAT_HIP_DENSIFY_MEANS 1
#define GSPLAT_HIP_DENSIFY_SCALES 2
#define GSPLAT_HIP_DENSIFY_OPACITIES 3
#define GSPLAT_HIP_DENSIFY_MOMENT 4
int64_t gsplat_hip_densify_workspace_bytes(int64_t N);
int gsplat_hip_densify_plan(int64_t N, const float *grad2d, const float *count,
                            const float *log_scales, const float *logits, const float *radii2d,
                            float grow_grad2d, float grow_scale3d, float prune_opa, int prune_big,
                            float prune_scale3d, float grow_scale2d, float prune_scale2d,
                            int revised_opacity, void *workspace, int64_t *totals, void *stream);
int gsplat_hip_densify_apply(int64_t N, const void *workspace, const int64_t *totals,
                             const float *randn, int revised_opacity, int n_arrays,
                             const float *const *src, float *const *dst, const int32_t *row_floats,
                             const int32_t *kinds, const float *means, const float *quats,
                             const float *log_scales, const float *logits, void *stream);

/* gsplat_hip_sh_colors_bwd with the coefficients' Adam step fused in (ABI 18;
 * C cameras sharing the coefficient rows since ABI 23: the gradient is the
 * sum over the C rows c*N + g of radii / v_colors, formed in registers
 * first): coeffs [N,1,3] and coeffs_rest [N,15,3] are updated in place
 * by torch.optim.Adam (lr0 / lr_rest, shared betas and eps, 1-based step,
 * moments m0/v0 and m_rest/v_rest in the coefficients' layout) from the
 * gradient this backward computes, which is never written; v_dirs [N,3] =
 * the means gradient summed over the cameras.  degree 0..3 (zero gradient
 * above it).  The trainer's optimizer-in-backward for the SH groups (81 % of
 * Adam's bytes). */
int gsplat_hip_sh_colors_bwd_adam(int degree, int C, int64_t N, const float *means,
                                  const float *viewmats, float *coeffs, float *coeffs_rest,
                                  const int32_t *radii, const float *v_colors, float *v_dirs,
                                  float *m0, float *v0, float *m_rest, float *v_rest, float lr0,
                                  float lr_rest, float beta1, float beta2, float eps, int step,
                                  void *stream);
/* The same with the step's factors on the device (ABI 20; a captured
 * training step replays with a new step count): hyper_device = {lr0 /
 * (1 - beta1^t), lr_rest / (1 - beta1^t), 1 / sqrt(1 - beta2^t)}, computed
 * on the host as above; skip_device (may be NULL) != 0 leaves the
 * coefficients and moments unchanged (v_dirs is still written). */
int gsplat_hip_sh_colors_bwd_adam_dev(int degree, int C, int64_t N, const float *means,
                                      const float *viewmats, float *coeffs, float *coeffs_rest,
                                      const int32_t *radii, const float *v_colors, float *v_dirs,
                                      float *m0, float *v0, float *m_rest, float *v_rest,
                                      const float *hyper_device, float beta1, float beta2,
                                      float eps, const int32_t *skip_device, void *stream);
/* gsplat_hip_sh_colors_bwd for C cameras sharing one set of coefficient rows
 * in the trainer's layout (coeffs [N,1,3], coeffs_rest [N,15,3], degree
 * 0..3; ABI 23): v_coeffs [N,1,3], v_coeffs_rest [N,15,3] and v_dirs [N,3]
 * are the sums over the cameras (gsplat_hip_sh_colors_bwd writes C rows per
 * Gaussian for the caller to sum).  The colours of a Gaussian-sharded
 * render (gsplat/rendering.py:298-310: every rank's cameras). */
int gsplat_hip_sh_colors_bwd_sum(int degree, int C, int64_t N, const float *means,
                                 const float *viewmats, const float *coeffs,
                                 const float *coeffs_rest, const int32_t *radii,
                                 const float *v_colors, float *v_coeffs, float *v_coeffs_rest,
                                 float *v_dirs, void *stream);

/* One torch.optim.Adam step (amsgrad=False, no weight decay) over up to 8
 * parameter groups in a single launch (replaces the per-group optimizers of
 * examples/simple_trainer.py:265-276).  Host arrays of length n_groups. */
int gsplat_hip_adam_step(int n_groups, float *const *params, const float *const *grads,
                         float *const *exp_avgs, float *const *exp_avg_sqs,
                         const int64_t *numels, const float *lrs, float beta1, float beta2,
                         float eps, int step, void *stream);
/* The same update with the gradient formed in-register per group (ABI 19):
 * modes[i] 0: grads[i]; 1: grads[i] + aux[i] (two gradient contributions);
 * 2: grads[i] * aux[i] (VJP of exp, aux = exp(x)); 3: grads[i] * (1 - aux[i])
 * * aux[i] (VJP of sigmoid, aux = sigmoid(x)) -- the trainer's activation
 * VJPs and means-gradient sum folded into the geometry groups' update.
 * aux / modes may be NULL (all mode 0); aux pointers 16-B aligned. */
int gsplat_hip_adam_step_ex(int n_groups, float *const *params, const float *const *grads,
                            const float *const *aux, const int32_t *modes,
                            float *const *exp_avgs, float *const *exp_avg_sqs,
                            const int64_t *numels, const float *lrs, float beta1, float beta2,
                            float eps, int step, void *stream);
/* gsplat_hip_adam_step_ex with the step's factors on the device (ABI 20):
 * hyper_device[2 i] = lr_i / (1 - beta1^t), hyper_device[2 i + 1] =
 * 1 / sqrt(1 - beta2^t) (the host's double-precision values rounded to
 * float, as gsplat_hip_adam_step computes them); skip_device (may be NULL)
 * != 0 updates nothing. */
int gsplat_hip_adam_step_dev(int n_groups, float *const *params, const float *const *grads,
                             const float *const *aux, const int32_t *modes,
                             float *const *exp_avgs, float *const *exp_avg_sqs,
                             const int64_t *numels, const float *hyper_device, float beta1,
                             float beta2, float eps, const int32_t *skip_device, void *stream);

/* ---------------------------------------------------------------------------
 * 2DGS (surfels).  Replaces the CUDA kernels that gsplat.rendering.rasterization_2dgs
 * (gsplat/rendering.py:1018-1339) reaches through gsplat/cuda/_wrapper.py.
 *
 * Projection: replaces projection_2dgs_fused_fwd (gsplat/cuda/csrc/Projection2DGSFused.cu:17-238,
 * host gsplat/cuda/csrc/Projection.cpp:517-567, bound by _FullyFusedProjection2DGS.forward,
 * gsplat/cuda/_wrapper.py:1333-1389).
 * means[N,3] quats[N,4] (16-B aligned) scales[N,3] viewmats[C,4,4] Ks[C,3,3]
 * -> radii i32[C,N], means2d[C,N,2], depths[C,N], ray_transforms[C,N,3,3]
 *    (rows of K [t_u | t_v | mean_c]), normals[C,N,3].
 * Culled entries (near/far, degenerate AABB, radius <= radius_clip, off-screen)
 * have radii 0 and zero means2d / ray_transforms / normals (the reference
 * leaves them uninitialised). */
int gsplat_hip_projection_2dgs_fwd(int C, int N, const float *means, const float *quats,
                                   const float *scales, const float *viewmats, const float *Ks,
                                   int width, int height, float near_plane, float far_plane,
                                   float radius_clip, int32_t *radii, float *means2d,
                                   float *depths, float *ray_transforms, float *normals,
                                   void *stream);

/* Replaces projection_2dgs_fused_bwd (Projection2DGSFused.cu:319-457 with
 * compute_ray_transforms_aabb_vjp, Projection2DGS.cuh:10-87; host
 * Projection.cpp:569-633; _FullyFusedProjection2DGS.backward, _wrapper.py:1391-1437).
 * -> v_means[N,3], v_quats[N,4], v_scales[N,3] (v_scales[:,2] = 0).
 * v_viewmats[C,4,4] (or NULL) is written as zeros, as the reference's kernel
 * never writes it.  v_depths may be NULL; v_normals too (ABI 33; zeros). */
int gsplat_hip_projection_2dgs_bwd(int C, int N, const float *means, const float *quats,
                                   const float *scales, const float *viewmats, const float *Ks,
                                   int width, int height, const int32_t *radii,
                                   const float *ray_transforms, const float *v_means2d,
                                   const float *v_depths, const float *v_normals,
                                   const float *v_ray_transforms, float *v_means,
                                   float *v_quats, float *v_scales, float *v_viewmats,
                                   void *stream);
/* The same backward for one camera with the geometry groups' Adam step fused
 * in (ABI 33; as gsplat_hip_projection_bwd_adam for 3DGS): no gradient is
 * stored; params / exp_avgs / exp_avg_sqs are [means, log_scales, quats,
 * logits]; v_dirs [N,3] (the SH backward's means gradient) and v_opac [N]
 * (dL/d sigmoid(logits), with opac = sigmoid(logits)) may be NULL; lrs[4]
 * with the 1-based step, or hyper_device f32[8]; skip_device may be NULL. */
int gsplat_hip_projection_2dgs_bwd_adam(
    int N, const float *means, const float *quats, const float *scales, const float *viewmats,
    const float *Ks, const int32_t *radii, const float *ray_transforms, const float *v_means2d,
    const float *v_depths, const float *v_normals, const float *v_ray_transforms,
    const float *v_dirs, const float *v_opac, const float *opac, float *const *params,
    float *const *exp_avgs, float *const *exp_avg_sqs, const float *lrs, float beta1,
    float beta2, float eps, int step, const float *hyper_device, const int32_t *skip_device,
    void *stream);
/* Packed 2DGS projection.  Replaces projection_2dgs_packed_fwd / _bwd
 * (gsplat/cuda/csrc/Projection2DGSPacked.cu:17-270, 274-420) behind
 * _FullyFusedProjectionPacked2DGS (gsplat/cuda/_wrapper.py:1440-1592).
 * count: per-block counts of the kept (camera, surfel) pairs into `workspace`
 * (gsplat_hip_projection_2dgs_packed_workspace_bytes), scanned in place,
 * nnz -> nnz_device[0].  fwd (same inputs and workspace): the nnz kept pairs
 * in (camera, surfel) order -> camera_ids i64[nnz], gaussian_ids i64[nnz],
 * radii i32[nnz], means2d[nnz,2], depths[nnz], ray_transforms[nnz,3,3],
 * normals[nnz,3].  bwd: dense v_means[N,3] v_quats[N,4] v_scales[N,3]
 * (zeroed here, atomics), or with sparse_grad one row per entry [nnz, .];
 * v_viewmats[C,4,4] or NULL is zeroed (the reference does not differentiate
 * it). */
int64_t gsplat_hip_projection_2dgs_packed_workspace_bytes(int C, int N);
int gsplat_hip_projection_2dgs_packed_count(int C, int N, const float *means, const float *quats,
                                            const float *scales, const float *viewmats,
                                            const float *Ks, int width, int height,
                                            float near_plane, float far_plane, float radius_clip,
                                            void *workspace, int64_t *nnz_device, void *stream);
int gsplat_hip_projection_2dgs_packed_fwd(int C, int N, const float *means, const float *quats,
                                          const float *scales, const float *viewmats,
                                          const float *Ks, int width, int height,
                                          float near_plane, float far_plane, float radius_clip,
                                          const void *workspace, int64_t *camera_ids,
                                          int64_t *gaussian_ids, int32_t *radii, float *means2d,
                                          float *depths, float *ray_transforms, float *normals,
                                          void *stream);
int gsplat_hip_projection_2dgs_packed_bwd(int C, int N, int64_t nnz, const float *means,
                                          const float *quats, const float *scales,
                                          const float *viewmats, const float *Ks, int width,
                                          int height, const int64_t *camera_ids,
                                          const int64_t *gaussian_ids,
                                          const float *ray_transforms, const float *v_means2d,
                                          const float *v_depths, const float *v_normals,
                                          const float *v_ray_transforms, int sparse_grad,
                                          float *v_means, float *v_quats, float *v_scales,
                                          float *v_viewmats, void *stream);

/* Surfel rasterizer.  D in {1..9, 16, 17, 32, 33}
 * (gsplat_hip_rasterize_2dgs_supported_channels); the caller pads other
 * channel counts keeping the depth channel last, as
 * rasterize_to_pixels_2dgs does (gsplat/cuda/_wrapper.py:1657-1683).
 * tile_size <= 32 forward, <= 16 backward.
 * Forward replaces rasterize_to_pixels_2dgs_fwd
 * (gsplat/cuda/csrc/RasterizeToPixels2DGSFwd.cu:18-452, host
 * gsplat/cuda/csrc/Rasterization.cpp:322-410): means2d[G,2],
 * ray_transforms[G,3,3], colors[G,D], opacities[G], normals[G,3],
 * backgrounds[C,D] or NULL, masks u8[C,th,tw] or NULL ->
 * render_colors[C,H,W,D], render_alphas[C,H,W,1], render_normals[C,H,W,3],
 * render_distort[C,H,W,1], render_median[C,H,W,1], last_ids i32[C,H,W],
 * median_ids i32[C,H,W].
 * n_isects_device (ABI 32, here and in _bwd, may be NULL): the isect count on
 * the device, n_isects then being the capacity of flatten_ids (the sync-free
 * isect, gsplat_hip_isect_write_sorted_capped: a captured 2DGS step).
 * records (ABI 32, may be NULL): the surfels' compositing records
 * (gsplat_hip_rasterize_2dgs_pack_records): the forward then culls from them
 * and composites with scalar loads instead of its LDS queue; same outputs.
 * record_floats: floats per record (32), 0 when the configuration (D,
 * tile_size) has no record path; pack_records writes records f32[G][32]
 * from the rasterizer's inputs (G rows of means2d ...); rows with
 * visible[g] <= 0 (e.g. tiles_per_gauss; NULL = all) are never gathered and
 * are left unwritten.
 * tile_order (ABI 32, may be NULL; i32[C*th*tw]): the forward writes the
 * tiles' dispatch order there (heaviest first, by floor(log2(isects))) and
 * runs in it; pass it to the backward, which then runs in it too.
 * A colours-only render (ABI 33; the record path only): render_normals,
 * render_distort, render_median and median_ids all NULL -- only
 * render_colors, render_alphas and last_ids are formed; its backward gets
 * median_ids = NULL and no gradient of those outputs.
 * depths (ABI 33, may be NULL; f32[G]): the last of the D colour channels is
 * read from depths[g], `colors` then holding D - 1 channels per row (the
 * RGB+D render without a concatenated colour copy); the backward then takes
 * the same depths and writes that channel's gradient to v_depths[G]
 * (v_colors [G, D - 1]). */
int gsplat_hip_rasterize_2dgs_record_floats(int D, int tile_size);
int gsplat_hip_rasterize_2dgs_pack_records(int64_t n_gaussians, int D, const float *means2d,
                                           const float *ray_transforms, const float *opacities,
                                           const float *normals, const float *colors,
                                           const float *depths, const int32_t *visible,
                                           float *records, void *stream);
int gsplat_hip_rasterize_2dgs_supported_channels(int D);
int gsplat_hip_rasterize_2dgs_fwd(int C, int D, int width, int height, int tile_size,
                                  int tile_width, int tile_height, const float *means2d,
                                  const float *ray_transforms, const float *colors,
                                  const float *depths, const float *opacities,
                                  const float *normals,
                                  const float *backgrounds, const uint8_t *masks,
                                  const int32_t *isect_offsets, int64_t n_isects,
                                  const int64_t *n_isects_device, const int32_t *flatten_ids,
                                  const float *records, int32_t *tile_order, float *render_colors,
                                  float *render_alphas, float *render_normals,
                                  float *render_distort, float *render_median,
                                  int32_t *last_ids, int32_t *median_ids, void *stream);

/* Backward replaces rasterize_to_pixels_2dgs_bwd
 * (gsplat/cuda/csrc/RasterizeToPixels2DGSBwd.cu:16-700, host Rasterization.cpp:441-560;
 * _RasterizeToPixels2DGS.backward, gsplat/cuda/_wrapper.py:1893-1971).
 * workspace: gsplat_hip_rasterize_2dgs_bwd_workspace_bytes(G, D, absgrad) bytes.
 * -> v_means2d[G,2], v_ray_transforms[G,3,3], v_colors[G,D], v_opacities[G],
 *    v_normals[G,3], v_densify[G,2] = (v_rt[0][2], v_rt[1][2]) * rt[2][2]
 *    (formed from the final sums; the reference writes it racily from partial
 *    sums), v_means2d_abs[G,2] or NULL (absgrad off).
 * v_render_alphas / v_render_normals (ABI 32) / v_render_distort /
 * v_render_median may be NULL (no gradient).  depths / v_depths (ABI 33, both
 * NULL or both set): the forward's separate last channel and its gradient.
 * v_normals (ABI 33) may be NULL when v_render_normals is: that gradient is
 * then exactly zero and not written.  visible (ABI 32, may be NULL;
 * i32[G], e.g. tiles_per_gauss): only the rows with visible[g] > 0 can
 * receive gradient -- the others are written as zeros without a read. */
int64_t gsplat_hip_rasterize_2dgs_bwd_workspace_bytes(int64_t n_gaussians, int D, int absgrad);
int gsplat_hip_rasterize_2dgs_bwd(
    int C, int D, int width, int height, int tile_size, int tile_width, int tile_height,
    int64_t n_gaussians, const float *means2d, const float *ray_transforms, const float *colors,
    const float *depths, const float *opacities, const float *normals, const float *backgrounds,
    const uint8_t *masks, const int32_t *isect_offsets, int64_t n_isects,
    const int64_t *n_isects_device, const int32_t *flatten_ids, const int32_t *tile_order,
    const int32_t *visible, const float *render_colors, const float *render_alphas,
    const int32_t *last_ids, const int32_t *median_ids, const float *v_render_colors,
    const float *v_render_alphas, const float *v_render_normals, const float *v_render_distort,
    const float *v_render_median, float *v_means2d, float *v_ray_transforms, float *v_colors,
    float *v_depths, float *v_opacities, float *v_normals, float *v_densify,
    float *v_means2d_abs, void *workspace, int64_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Auxiliary kernels reached by the reference's strategies / optimizers through
 * its CUDA extension on every backend.
 *
 * Replaces quat_scale_to_covar_preci_fwd/bwd (gsplat/cuda/csrc/QuatScaleToCovarCUDA.cu,
 * gsplat/cuda/_wrapper.py:111-142,651-689; used by MCMCStrategy,
 * gsplat/strategy/ops.py:352).  quats[N,4] (16-B aligned), scales[N,3] ->
 * covars / precis [N,3,3] or, with triu, [N,6] (xx, xy, xz, yy, yz, zz);
 * either output may be NULL.  Backward: v_quats[N,4], v_scales[N,3]. */
int gsplat_hip_quat_scale_to_covar_preci_fwd(int64_t N, const float *quats, const float *scales,
                                             int triu, float *covars, float *precis,
                                             void *stream);
int gsplat_hip_quat_scale_to_covar_preci_bwd(int64_t N, const float *quats, const float *scales,
                                             int triu, const float *v_covars,
                                             const float *v_precis, float *v_quats,
                                             float *v_scales, void *stream);

/* Replaces relocation (gsplat/cuda/csrc/RelocationCUDA.cu:10-44, gsplat/relocation.py:10-51;
 * MCMC relocate / sample_add, gsplat/strategy/ops.py:272,314).
 * opacities[N], scales[N,3], ratios i32[N] (clamped to [1, n_max] by the
 * caller), binoms[n_max,n_max] -> new_opacities[N], new_scales[N,3]. */
int gsplat_hip_relocation(int64_t N, const float *opacities, const float *scales,
                          const int32_t *ratios, const float *binoms, int n_max,
                          float *new_opacities, float *new_scales, void *stream);

/* Replaces inject_noise_to_position (ABI 35; gsplat/strategy/ops.py:343-369: its
 * quat_scale_to_covar_preci launch, the sigmoid / exp / op_sigmoid torch
 * passes, the einsum and the add) with one launch, in place:
 * means[n] += Sigma_n (z[n] * op_sigmoid(1 - sigmoid(logits[n])) * scaler),
 * Sigma_n = R(quats[n]) diag(exp(log_scales[n]))^2 R^T, op_sigmoid(x) =
 * 1 / (1 + exp(-100 (x - 0.995))).  means/log_scales [N,3], quats [N,4]
 * (16-B aligned), logits [N].
 * z [N,3]: the caller's standard normal draw (the reference's
 * randn_like(means)); NULL: three normals per Gaussian from Philox-4x32-10
 * keyed by `seed` with counter (n, step) (Box-Muller), a pure function of
 * (seed, step, n).  step_device / scaler_device (may be NULL): read step /
 * scaler from device memory instead (a captured step's input block); a zero
 * scaler moves nothing.  skip_device (may be NULL): non-zero = void step,
 * nothing written. */
int gsplat_hip_mcmc_inject_noise(int64_t N, float *means, const float *quats,
                                 const float *log_scales, const float *logits, const float *z,
                                 uint64_t seed, int64_t step, const int64_t *step_device,
                                 float scaler, const float *scaler_device,
                                 const int32_t *skip_device, void *stream);

/* Replaces adam (gsplat/cuda/csrc/AdamCUDA.cu:12-46, used by SelectiveAdam,
 * gsplat/optimizers/selective_adam.py): the reference's update without bias
 * correction on the rows (`row` consecutive elements each) whose visible[] is
 * non-zero; visible may be NULL (every row). */
int gsplat_hip_selective_adam(int64_t n_rows, int64_t row, float *param, const float *grad,
                              float *exp_avg, float *exp_avg_sq, const uint8_t *visible,
                              float lr, float beta1, float beta2, float eps, void *stream);

/* ---------------------------------------------------------------------------
 * Packed projection (§8 f3).  Replaces projection_ewa_3dgs_packed_fwd/bwd
 * (gsplat/cuda/csrc/ProjectionEWA3DGSPacked.cu:17-244,348-630, bound by
 * _FullyFusedProjectionPacked, gsplat/cuda/_wrapper.py:998-1190; the Triton
 * backend cannot run packed mode).  Same algebra as
 * gsplat_hip_projection_fwd; the kept (camera, Gaussian) pairs are written in
 * (camera, Gaussian) order, so the packed outputs equal the dense ones
 * compacted.  Three calls around the one host read of nnz:
 *   1. gsplat_hip_projection_packed_count: per-block counts and their scan in
 *      `workspace` (gsplat_hip_projection_packed_workspace_bytes(C, N) bytes),
 *      nnz -> nnz_device[0];
 *   2. gsplat_hip_projection_packed_fwd: camera_ids i64[nnz], gaussian_ids
 *      i64[nnz], radii i32[nnz], means2d[nnz,2], depths[nnz], conics[nnz,3],
 *      compensations[nnz] or NULL;
 *   3. gsplat_hip_projection_packed_bwd: v_means[N,3], v_quats[N,4],
 *      v_scales[N,3] (zeroed, then summed over entries), or with sparse_grad
 *      one row per entry ([nnz,3], [nnz,4], [nnz,3]: the COO values);
 *      v_viewmats[C,4,4] or NULL; v_depths may be NULL. */
int64_t gsplat_hip_projection_packed_workspace_bytes(int C, int N);
int gsplat_hip_projection_packed_count(int C, int N, const float *means, const float *quats,
                                       const float *scales, const float *viewmats,
                                       const float *Ks, int width, int height, float eps2d,
                                       float near_plane, float far_plane, float radius_clip,
                                       void *workspace, int64_t *nnz_device, void *stream);
int gsplat_hip_projection_packed_fwd(int C, int N, const float *means, const float *quats,
                                     const float *scales, const float *viewmats, const float *Ks,
                                     int width, int height, float eps2d, float near_plane,
                                     float far_plane, float radius_clip, const void *workspace,
                                     int64_t *camera_ids, int64_t *gaussian_ids, int32_t *radii,
                                     float *means2d, float *depths, float *conics,
                                     float *compensations, void *stream);
int gsplat_hip_projection_packed_bwd(int C, int N, int64_t nnz, const float *means,
                                     const float *quats, const float *scales,
                                     const float *viewmats, const float *Ks, int width, int height,
                                     float eps2d, const int64_t *camera_ids,
                                     const int64_t *gaussian_ids, const float *conics,
                                     const float *compensations, const float *v_means2d,
                                     const float *v_depths, const float *v_conics,
                                     const float *v_compensations, int sparse_grad,
                                     float *v_means, float *v_quats, float *v_scales,
                                     float *v_viewmats, void *stream);

/* ---------------------------------------------------------------------------
 * Per-pixel contributor lists (§8 f4).  Replace rasterize_to_indices_3dgs /
 * _2dgs (gsplat/cuda/csrc/RasterizeToIndices3DGS.cu:14-185,
 * RasterizeToIndices2DGS.cu:14-200) and their two-pass host driver
 * (gsplat/cuda/csrc/Rasterization.cpp:224-296, 586-660), bound by
 * rasterize_to_indices_in_range{,_2dgs} (gsplat/cuda/_wrapper.py:577-650,
 * 1729-1800).
 *   kind 0 = 3DGS, shape = conics[C,N,3]; kind 1 = 2DGS, shape =
 *   ray_transforms[C,N,3,3].  Ranges are in batches of tile_size^2 records of
 *   each tile's list, [range_start, range_end); transmittances[C,H,W] is the
 *   starting T per pixel.
 *   count: chunk_cnts[C,H,W] (every pixel written) = contributors per pixel.
 *   The caller forms chunk_starts = exclusive scan of chunk_cnts (pixel-major)
 *   and M = its total, allocates gaussian_ids/pixel_ids int64[M], then
 *   write: gaussian_ids = flatten_id % N, pixel_ids = c*H*W + y*W + x, in
 *   pixel-major, front-to-back order (the reference's output order). */
int gsplat_hip_rasterize_to_indices_count(int kind, int C, int N, int W, int H, int tile_size,
                                          int tile_width, int tile_height, int64_t n_isects,
                                          int64_t range_start, int64_t range_end,
                                          const float *transmittances, const float *means2d,
                                          const float *shape, const float *opacities,
                                          const int32_t *offsets, const int32_t *flatten_ids,
                                          int32_t *chunk_cnts, void *stream);
int gsplat_hip_rasterize_to_indices_write(int kind, int C, int N, int W, int H, int tile_size,
                                          int tile_width, int tile_height, int64_t n_isects,
                                          int64_t range_start, int64_t range_end,
                                          const float *transmittances, const float *means2d,
                                          const float *shape, const float *opacities,
                                          const int32_t *offsets, const int32_t *flatten_ids,
                                          const int32_t *chunk_starts, int64_t *gaussian_ids,
                                          int64_t *pixel_ids, void *stream);

/* Normals from depth maps (gsplat/utils.py:201-224, depth_to_normal, called by
 * rasterization_2dgs for render_normals_from_depth): depths[C,H,W] (the [..,1]
 * channel; depth_stride (ABI 32): floats from one pixel's depth to the next,
 * e.g. 4 for the last channel of an RGB+D render read in place),
 * camtoworlds[C,4,4], Ks[C,3,3] -> normals[C,H,W,3], zero border.
 * Forward only; the Python binding differentiates the torch formula. */
int gsplat_hip_depth_to_normal(int C, int H, int W, const float *depths, int64_t depth_stride,
                               const float *camtoworlds, const float *Ks, int z_depth,
                               float *normals, void *stream);
/* rasterization_2dgs's rotation of the rendered normals into world space
 * (gsplat/rendering.py, the einsum of camtoworlds[..., :3, :3] with
 * render_normals; ABI 32): out[c,p,i] = sum_j camtoworlds[c][i][j] v[c,p,j]
 * for v, out f32[C,HW,3]; one launch.  Forward only. */
int gsplat_hip_rotate3(int C, int64_t HW, const float *camtoworlds, const float *v, float *out,
                       void *stream);

/* ---------------------------------------------------------------------------
 * Progress watchdog (ABI 34; csrc/watchdog.cpp).  A native thread that ends
 * the process when no progress is reported within a timeout: a collective one
 * rank never joins -- also one replayed inside a HIP graph, which RCCL's own
 * watchdog does not track -- must end a multi-GPU job with a diagnosis and a
 * non-zero status, not hang it.  No interpreter lock is needed, so a host
 * thread blocked in a HIP wait is no obstacle.  All return 0 (arm: 1 for a
 * non-positive timeout).
 *   _arm:           (re)start with `timeout_s`; `tag` names the process
 *                   ("rank 3"); `exit_code` (non-zero) is the status on expiry.
 *   _beat:          progress; `state` (one line) is printed on expiry.
 *   _set_fallback:  on expiry also write `text` to `fd` and end with
 *                   `exit_code` (fd < 0 clears it): a later phase's hang still
 *                   delivers the result of a phase that completed.
 *   _disarm:        stop watching (the thread stays, idle).
 * No reference counterpart: gsplat/distributed.py relies on NCCL's timeout,
 * which sees eager collectives only. */
int gsplat_hip_watchdog_arm(double timeout_s, const char *tag, int exit_code);
int gsplat_hip_watchdog_beat(const char *state);
int gsplat_hip_watchdog_set_fallback(int fd, const char *text, int exit_code);
int gsplat_hip_watchdog_disarm(void);

#ifdef __cplusplus
}
#endif

#endif /* GSPLAT_HIP_H */
