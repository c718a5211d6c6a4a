/*
 * dfhip.h — C-ABI of the MI355X (gfx950) NeRF hot-path kernels.
 *
 * This is the drop-in boundary that replaces the four pybind11 extension
 * modules of the reference (torch-ngp style): `_raymarching`, `_gridencoder`,
 * `_freqencoder`, `_shencoder`.  Every entry point below names the reference
 * binding it replaces (file:line, relative to the reference repo root).
 *
 * Conventions (all entry points):
 *   - plain device pointers + sizes; no torch / HIP types in signatures.
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).
 *     The reference launches on the legacy default stream
 *     (raymarching/src/raymarching.cu:154); our Python shims pass torch's
 *     current stream.
 *   - all buffers contiguous, row-major, AoS exactly as the reference.
 *   - the caller owns and allocates every buffer (reference ownership rule,
 *     raymarching/raymarching.py:205-218).  Entry points marked [scratch]
 *     take an explicit caller-provided scratch buffer; the reference-signature
 *     form allocates stream-ordered scratch itself (hipMallocAsync).
 *   - return 0 on success, a DFHIP_E* code otherwise; dfhip_last_error()
 *     returns a thread-local message for the last failing call on that thread.
 *     (Reference: TORCH_CHECK / std::runtime_error -> Python RuntimeError,
 *     gridencoder/src/gridencoder.cu:354,372,425-441.)
 *   - `dtype` selects the floating storage type of the `void*` float buffers
 *     (reference: AT_DISPATCH_FLOATING_TYPES_AND_HALF).  Arithmetic inside the
 *     kernels is f32 as in the reference (f64 for the f64 storage variant of
 *     the compositing accumulators).
 */
#ifndef DFHIP_H
#define DFHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *dfhip_stream_t; /* hipStream_t */

/* DFHIP_BF16: bfloat16 storage (the C5 bf16 option; no reference counterpart,
 * the reference dispatches f32 / f16 / f64 only). */
enum dfhip_dtype { DFHIP_F32 = 0, DFHIP_F16 = 1, DFHIP_F64 = 2, DFHIP_BF16 = 3 };
/* Shadings of the non-albedo train steps (nerf/network_grid.py:124-144). */
enum dfhip_shading { DFHIP_SHADING_TEXTURELESS = 1, DFHIP_SHADING_LAMBERTIAN = 2 };

enum dfhip_status {
    DFHIP_OK = 0,
    DFHIP_EINVAL = 1,     /* bad size / null pointer / unsupported D,C */
    DFHIP_EDTYPE = 2,     /* unsupported dtype */
    DFHIP_ELAUNCH = 3,    /* HIP launch / runtime error */
    DFHIP_ENOMEM = 4      /* stream-ordered scratch allocation failed */
};

/* ABI version: a hash of this header's text taken at build time
 * (dfhip_build.py passes it as DFHIP_ABI_HASH).  The Python binding hashes
 * the header it was written against the same way and refuses a library whose
 * value differs, so a stale library fails to load instead of being called
 * with another signature. */
int dfhip_abi_version(void);
const char *dfhip_last_error(void);

/* ---------------------------------------------------------------- raymarching
 * Reference: raymarching/src/raymarching.h:7-18, bindings.cpp:5-18. */

/* raymarching.cu:148 near_far_from_aabb(rays_o, rays_d, aabb, N, min_near, nears, fars) */
int dfhip_near_far_from_aabb(int dtype, const void *rays_o, const void *rays_d,
                             const void *aabb, uint32_t N, float min_near,
                             void *nears, void *fars, dfhip_stream_t stream);

/* nerf/utils.py:42-106 get_rays(poses, intrinsics, H, W, N=-1) for one pose,
 * as one launch (the reference runs ~10 torch ops per train step).  `pose` is a
 * HOST pointer to the 3x4 cam2world matrix (row-major, 12 floats: rotation
 * rows with the centre as 4th column); it is passed to the kernel by value.
 * Writes rays_o, rays_d [H*W, 3] f32 for pixel centres (w + 0.5, h + 0.5),
 * pixel n = h*W + w. */
int dfhip_get_rays(const float *pose, float fx, float fy, float cx, float cy,
                   uint32_t H, uint32_t W, float *rays_o, float *rays_d,
                   dfhip_stream_t stream);

/* nerf/renderer.py:562-615 update_extra_state, sync-free form (native).
 * dfhip_density_grid_ema: for each queried point p, cell c = indices[p]
 *   (int32, cascade offset included, c < cells): if grid[c] >= 0 then
 *   grid[c] = max(grid[c] * decay, sigma[p]) (torch.maximum, NaN-propagating),
 *   and that new value is added to acc[0], 1 to acc[1] (f64, device; the caller
 *   zeroes acc before the first cascade).  Every cell must be queried once.
 * dfhip_packbits_mean: thresh = min(acc[0] / acc[1], density_thresh) on the
 *   device; bit i of byte n = grid[8n + i] > thresh (grid 16-B aligned f32);
 *   mean_out[0] (optional) = acc[0] / acc[1] as f32. */
int dfhip_density_grid_ema(const float *sigma, const int32_t *indices, uint32_t n,
                           uint32_t cells, float decay, float *grid, double *acc,
                           dfhip_stream_t stream);
int dfhip_packbits_mean(const float *grid, uint32_t N, const double *acc,
                        float density_thresh, uint8_t *bitfield, float *mean_out,
                        dfhip_stream_t stream);
/* renderer.py:611-613 mean_count = int(step_counter[:total_step, 0].sum() /
 * total_step) on the device (step_counter int32 [>= total_step, 2] contiguous,
 * 1 <= total_step <= 64; mean_count one int64). total_step 0 is a no-op. */
int dfhip_mean_count(const int32_t *step_counter, uint32_t total_step,
                     int64_t *mean_count, dfhip_stream_t stream);

/* raymarching.cu:201 sph_from_ray(rays_o, rays_d, radius, N, coords) */
int dfhip_sph_from_ray(int dtype, const void *rays_o, const void *rays_d,
                       float radius, uint32_t N, void *coords,
                       dfhip_stream_t stream);

/* raymarching.cu:229 morton3D(coords, N, indices) */
int dfhip_morton3D(const int32_t *coords, uint32_t N, int32_t *indices,
                   dfhip_stream_t stream);

/* raymarching.cu:257 morton3D_invert(indices, N, coords) */
int dfhip_morton3D_invert(const int32_t *indices, uint32_t N, int32_t *coords,
                          dfhip_stream_t stream);

/* raymarching.cu:292 packbits(grid, N, density_thresh, bitfield) */
int dfhip_packbits(int dtype, const void *grid, uint32_t N, float density_thresh,
                   uint8_t *bitfield, dfhip_stream_t stream);

/* raymarching.cu:482 march_rays_train(rays_o, rays_d, grid, bound, dt_gamma,
 *   max_steps, N, C, H, M, nears, fars, xyzs, dirs, deltas, rays, counter, noises)
 * Reference-signature form.  Deterministic: rays[i] = (i, offset_i, count_i)
 * with offsets the exclusive prefix sum of counts in ray order (the reference
 * assigns offsets by atomicAdd arrival order, raymarching.cu:405-406; per-ray
 * contents are identical).  counter[0] += total points, counter[1] += N. */
int dfhip_march_rays_train(int dtype, const void *rays_o, const void *rays_d,
                           const uint8_t *grid, float bound, float dt_gamma,
                           uint32_t max_steps, uint32_t N, uint32_t C, uint32_t H,
                           uint32_t M, const void *nears, const void *fars,
                           void *xyzs, void *dirs, void *deltas, int32_t *rays,
                           int32_t *counter, const void *noises,
                           dfhip_stream_t stream);

/* [scratch] Split form used by the native Python path.
 * Pass 1 (count): rays[i] = (i, -, count_i); block_sums[ceil(N/64)];
 *   counter[0] += total, counter[1] += N.
 * Pass 2 (emit): offsets from block_sums + in-block scan; writes samples.
 *   Let W = end of the rows actually written (total, or the offset of the first
 *   ray that does not fit in M).  zero_tail < 0: rows [W, M) are zeroed;
 *   zero_tail = a > 0: rows [W, min(align_up(total), M)) are zeroed, with the
 *   reference's align rule align_up(m) = m + a - m % a (raymarching.py:225-226);
 *   zero_tail = 0: nothing is zeroed.  Either way the caller can allocate the
 *   outputs uninitialised (no N*max_steps memset). */
uint32_t dfhip_march_rays_train_scratch_ints(uint32_t N);
int dfhip_march_rays_train_count(int dtype, const void *rays_o, const void *rays_d,
                                 const uint8_t *grid, float bound, float dt_gamma,
                                 uint32_t max_steps, uint32_t N, uint32_t C,
                                 uint32_t H, const void *nears, const void *fars,
                                 int32_t *rays, int32_t *counter,
                                 const void *noises, int32_t *block_sums,
                                 dfhip_stream_t stream);
int dfhip_march_rays_train_emit(int dtype, const void *rays_o, const void *rays_d,
                                const uint8_t *grid, float bound, float dt_gamma,
                                uint32_t max_steps, uint32_t N, uint32_t C,
                                uint32_t H, uint32_t M, const void *nears,
                                const void *fars, void *xyzs, void *dirs,
                                void *deltas, int32_t *rays, const void *noises,
                                const int32_t *block_sums, int zero_tail,
                                dfhip_stream_t stream);

/* [scratch] Staged split form (native train step): the count pass also keeps
 * every sample as f32 (x, y, z, dt, dl) at row i*max_steps + j of `stage`
 * (dfhip_march_rays_train_stage_floats(N, max_steps) floats), and the emit
 * pass copies those rows to the ray-ordered outputs (same conversions to
 * `dtype`, dirs = rays_d) instead of marching each ray a second time.  Same
 * outputs, zero_tail and block_sums contract as the pair above; dirs may be
 * NULL (not written: a caller that reads rays_d per ray). */
uint64_t dfhip_march_rays_train_stage_floats(uint32_t N, uint32_t max_steps);
int dfhip_march_rays_train_count_staged(int dtype, const void *rays_o, const void *rays_d,
                                        const uint8_t *grid, float bound, float dt_gamma,
                                        uint32_t max_steps, uint32_t N, uint32_t C, uint32_t H,
                                        const void *nears, const void *fars, int32_t *rays,
                                        int32_t *counter, const void *noises,
                                        int32_t *block_sums, float *stage,
                                        dfhip_stream_t stream);
int dfhip_march_rays_train_emit_staged(int dtype, const void *rays_d, uint32_t max_steps,
                                       uint32_t N, uint32_t M, void *xyzs, void *dirs,
                                       void *deltas, int32_t *rays, const int32_t *block_sums,
                                       int zero_tail, const float *stage,
                                       dfhip_stream_t stream);

/* raymarching.cu:580 composite_rays_train_forward(sigmas, rgbs, deltas, rays,
 *   M, N, T_thresh, weights_sum, depth, image) */
int dfhip_composite_rays_train_forward(int dtype, const void *sigmas,
                                       const void *rgbs, const void *deltas,
                                       const int32_t *rays, uint32_t M, uint32_t N,
                                       float T_thresh, void *weights_sum,
                                       void *depth, void *image,
                                       dfhip_stream_t stream);

/* raymarching.cu:685 composite_rays_train_backward(grad_weights_sum, grad_image,
 *   sigmas, rgbs, deltas, rays, weights_sum, image, M, N, T_thresh,
 *   grad_sigmas, grad_rgbs).  Rows past a ray's early break are left untouched
 *   (the caller zero-fills, raymarching.py:283-284). */
int dfhip_composite_rays_train_backward(int dtype, const void *grad_weights_sum,
                                        const void *grad_image, const void *sigmas,
                                        const void *rgbs, const void *deltas,
                                        const int32_t *rays, const void *weights_sum,
                                        const void *image, uint32_t M, uint32_t N,
                                        float T_thresh, void *grad_sigmas,
                                        void *grad_rgbs, dfhip_stream_t stream);

/* Native variant: also writes zeros into rows that the reference leaves
 * untouched (past the early break, empty / overflowing rays), so grad_sigmas /
 * grad_rgbs may be allocated uninitialised.  Requires ray-ordered, contiguous
 * rays (as produced by dfhip_march_rays_train*): row ranges of consecutive
 * rays tile [0, total).  Rows in [total, M) are zeroed by the last block. */
int dfhip_composite_rays_train_backward_dense(int dtype, const void *grad_weights_sum,
                                              const void *grad_image,
                                              const void *sigmas, const void *rgbs,
                                              const void *deltas, const int32_t *rays,
                                              const void *weights_sum,
                                              const void *image, uint32_t M,
                                              uint32_t N, float T_thresh,
                                              void *grad_sigmas, void *grad_rgbs,
                                              dfhip_stream_t stream);

/* Native mixed-precision form of the two calls above for the fp16 train step:
 * sigmas, deltas, weights_sum, depth, image and their gradients are f32, the
 * colours `rgbs` and `grad_rgbs` are `rgb_dtype` (DFHIP_F32, DFHIP_F16 or DFHIP_BF16).
 * Same arithmetic as the reference, whose custom_fwd casts f16 colours to f32
 * (exact) and whose autograd casts the f32 colour gradient back to f16 once.
 * The backward is the dense form (needs ray-ordered contiguous rays);
 * zero_tail = 0 leaves rows [total, M) untouched, for capacity-sized buffers
 * whose consumers stop at the live sample count. */
int dfhip_composite_rays_train_forward_mixed(int rgb_dtype, const float *sigmas,
                                             const void *rgbs, const float *deltas,
                                             const int32_t *rays, uint32_t M, uint32_t N,
                                             float T_thresh, float *weights_sum,
                                             float *depth, float *image,
                                             dfhip_stream_t stream);
int dfhip_composite_rays_train_backward_mixed(int rgb_dtype, const float *grad_weights_sum,
                                              const float *grad_image, const float *sigmas,
                                              const void *rgbs, const float *deltas,
                                              const int32_t *rays, const float *weights_sum,
                                              const float *image, uint32_t M, uint32_t N,
                                              float T_thresh, float *grad_sigmas,
                                              void *grad_rgbs, int zero_tail,
                                              dfhip_stream_t stream);

/* raymarching.cu:808 march_rays(n_alive, n_step, rays_alive, rays_t, rays_o,
 *   rays_d, bound, dt_gamma, max_steps, C, H, grid, near, far, xyzs, dirs,
 *   deltas, noises).  Every one of a ray's n_step slots is written (zeros past
 *   the last occupied step), so the caller only needs to zero its align tail. */
int dfhip_march_rays(int dtype, uint32_t n_alive, uint32_t n_step,
                     const int32_t *rays_alive, const void *rays_t,
                     const void *rays_o, const void *rays_d, float bound,
                     float dt_gamma, uint32_t max_steps, uint32_t C, uint32_t H,
                     const uint8_t *grid, const void *nears, const void *fars,
                     void *xyzs, void *dirs, void *deltas, const void *noises,
                     dfhip_stream_t stream);

/* raymarching.cu:908 composite_rays(n_alive, n_step, T_thresh, rays_alive,
 *   rays_t, sigmas, rgbs, deltas, weights, depth, image) — in place. */
int dfhip_composite_rays(int dtype, uint32_t n_alive, uint32_t n_step,
                         float T_thresh, int32_t *rays_alive, void *rays_t,
                         const void *sigmas, const void *rgbs, const void *deltas,
                         void *weights_sum, void *depth, void *image,
                         dfhip_stream_t stream);

/* ---------------------------------------------------------------- gridencoder
 * Reference: gridencoder/src/gridencoder.h:12-13, bindings.cpp.
 * `dtype` is the embeddings / outputs / grad dtype (F32, F16, F64); `inputs`
 * are always f32 (gridencoder.cu:445).  gridtype: 0 = hash, 1 = tiled. */

/* gridencoder.cu:424 grid_encode_forward(inputs, embeddings, offsets, outputs,
 *   B, D, C, L, S, H, dy_dx?, gridtype, align_corners); outputs [L, B, C],
 *   dy_dx (nullable) [B, L*D*C]. */
int dfhip_grid_encode_forward(int dtype, const float *inputs, const void *embeddings,
                              const int32_t *offsets, void *outputs, uint32_t B,
                              uint32_t D, uint32_t C, uint32_t L, float S,
                              uint32_t H, void *dy_dx, uint32_t gridtype,
                              int align_corners, dfhip_stream_t stream);

/* gridencoder.cu:449 grid_encode_backward(grad [L,B,C], inputs, embeddings,
 *   offsets, grad_embeddings, B, D, C, L, S, H, dy_dx?, grad_inputs?, gridtype,
 *   align_corners).  grad_embeddings is accumulated into (caller zero-fills). */
int dfhip_grid_encode_backward(int dtype, const void *grad, const float *inputs,
                               const void *embeddings, const int32_t *offsets,
                               void *grad_embeddings, uint32_t B, uint32_t D,
                               uint32_t C, uint32_t L, float S, uint32_t H,
                               const void *dy_dx, void *grad_inputs,
                               uint32_t gridtype, int align_corners,
                               dfhip_stream_t stream);

/* Native layout variants: outputs / grad in [B, L*C] (the layout the caller
 * wants after the reference's permute, grid.py:42,70), which removes the two
 * permute copies per call.  Same numerics as the [L,B,C] forms. */
int dfhip_grid_encode_forward_blc(int dtype, const float *inputs,
                                  const void *embeddings, const int32_t *offsets,
                                  void *outputs, uint32_t B, uint32_t D, uint32_t C,
                                  uint32_t L, float S, uint32_t H, void *dy_dx,
                                  uint32_t gridtype, int align_corners,
                                  dfhip_stream_t stream);
/* dfhip_grid_encode_forward_blc over a capacity-sized batch (GridEncoder.forward
 * on the capacity-sized samples of the device-count march, grid.py:138-154):
 * rows [0, *m_dev) are encoded (all B rows when m_dev is NULL), rows
 * [*m_dev, B) are written as zeros (and their dy_dx rows); with bound > 0
 * `inputs` are raw positions in [-bound, bound], mapped to [0, 1] as
 * grid.py:142 does ((x + bound) / (2 bound), bit-identical to that torch op). */
int dfhip_grid_encode_forward_dyn(int dtype, const float *inputs, float bound,
                                  const void *embeddings, const int32_t *offsets,
                                  void *outputs, uint32_t B, const int32_t *m_dev, uint32_t D,
                                  uint32_t C, uint32_t L, float S, uint32_t H, void *dy_dx,
                                  uint32_t gridtype, int align_corners, dfhip_stream_t stream);
/* grad_dtype: dtype of `grad` ([B, L*C]); acc_dtype: dtype of grad_embeddings
 * (F32 accumulation is allowed with F16 grads: more accurate than the
 * reference's half2 atomics, same request count). */
/* dy_dx ([B, L*D*C], grad_dtype) and grad_inputs ([B, D], grad_dtype) are
 * nullable: when both are given, grad_inputs = sum_l,c grad * dy_dx
 * (gridencoder.cu:316-342). */
int dfhip_grid_encode_backward_blc(int grad_dtype, int acc_dtype, const void *grad,
                                   const float *inputs, const int32_t *offsets,
                                   void *grad_embeddings, uint32_t B, uint32_t D,
                                   uint32_t C, uint32_t L, float S, uint32_t H,
                                   const void *dy_dx, void *grad_inputs,
                                   uint32_t gridtype, int align_corners,
                                   dfhip_stream_t stream);

/* As dfhip_grid_encode_backward_sliced, for capacity-sized buffers: grad is
 * [L, B, C] with B the capacity (plane stride), only samples [0, *m_dev) are
 * walked when m_dev is given, and with bound > 0 `inputs` are raw positions in
 * [-bound, bound] mapped to [0, 1] as grid.py:142 (bound == 0: already [0,1]). */
int dfhip_grid_encode_backward_sliced_dyn(int grad_dtype, int out_dtype, const void *grad,
                                          const float *inputs, float bound,
                                          const int32_t *offsets, void *grad_embeddings,
                                          uint32_t total_rows, uint32_t B, const int32_t *m_dev,
                                          uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                                          uint32_t gridtype, int align_corners, float *partial,
                                          uint32_t parts, int accumulate, dfhip_stream_t stream);

/* Sliced embedding backward (native, no global atomics): the table's rows are
 * cut into LDS-sized slices; workgroup (slice, part) accumulates the corner
 * contributions of its part of the samples that land in its slice with LDS
 * atomics, writes the slice to partial[part], and a second pass sums the
 * parts in a fixed order.  grad: [L, B, C] (the reference's backward layout,
 * gridencoder.cu:404) of grad_dtype (F32/F16).  grad_embeddings
 * [total_rows, C] of out_dtype (F32/F16) is overwritten (accumulate == 0) or
 * added into.  partial: dfhip_grid_backward_partial_floats(total_rows, C,
 * parts) floats of caller scratch; parts >= 1 (default_parts() fills the CUs).
 * Replaces gridencoder.cu:226-313 on the native path. */
/* [B, L*C] -> [L, B, C] copy of the native encoder gradient into the layout
 * the sliced backward walks (the reference forms the same layout with a torch
 * permute, grid.py:70).  dtype F16/BF16/F32/F64; C * sizeof(dtype) in {2,4,8,16}. */
int dfhip_grid_grad_blc_to_lbc(int dtype, const void *src, void *dst, uint32_t B, uint32_t L,
                               uint32_t C, dfhip_stream_t stream);
uint32_t dfhip_grid_backward_default_parts(uint32_t total_rows, uint32_t C);
uint64_t dfhip_grid_backward_partial_floats(uint32_t total_rows, uint32_t C, uint32_t parts);
int dfhip_grid_encode_backward_sliced(int grad_dtype, int out_dtype, const void *grad,
                                      const float *inputs, const int32_t *offsets,
                                      void *grad_embeddings, uint32_t total_rows, uint32_t B,
                                      uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                                      uint32_t gridtype, int align_corners, float *partial,
                                      uint32_t parts, int accumulate, dfhip_stream_t stream);

/* ---------------------------------------------------------------- freqencoder
 * Reference: freqencoder/src/freqencoder.h:6-9 (f32 only, freqencoder.cu:109). */
int dfhip_freq_encode_forward(const float *inputs, uint32_t B, uint32_t D,
                              uint32_t deg, uint32_t C, float *outputs,
                              dfhip_stream_t stream);
int dfhip_freq_encode_backward(const float *grad, const float *outputs, uint32_t B,
                               uint32_t D, uint32_t deg, uint32_t C,
                               float *grad_inputs, dfhip_stream_t stream);

/* ---------------------------------------------------------------- shencoder
 * Reference: shencoder/src/shencoder.h:8-9.  C = degree (1..8), D = 3. */
int dfhip_sh_encode_forward(int dtype, const void *inputs, void *outputs,
                            uint32_t B, uint32_t D, uint32_t C, void *dy_dx,
                            dfhip_stream_t stream);
/* grad_inputs is accumulated into (caller zero-fills, sphere_harmonics.py). */
int dfhip_sh_encode_backward(int dtype, const void *grad, const void *inputs,
                             uint32_t B, uint32_t D, uint32_t C, const void *dy_dx,
                             void *grad_inputs, dfhip_stream_t stream);

/* ---------------------------------------------------------------- fused field head
 * Replaces the torch ops of nerf/network_grid.py:13-32 (MLP: 3 nn.Linear +
 * ReLU under fp16 autocast) and :76-87 (common_forward: sigma =
 * trunc_exp(h0 + 5 exp(-|x|^2/0.08)), activation.py:5-18; albedo =
 * sigmoid(h[1:4])).  Fixed shape: 32 -> 64 -> 64 -> 4 (the reference's
 * sigma_net).  Parameters are the f32 nn.Linear tensors (w1 [64,32], b1 [64],
 * w2 [64,64], b2 [64], w3 [4,64], b3 [4]), rounded to f16 inside as autocast
 * does.  enc: [M, 32] f16 encoder features; xyz: [M, 3] f32 positions in
 * [-bound, bound] (for the Gaussian blob). */
uint32_t dfhip_field_mlp_params(void); /* 6532 */
int dfhip_field_mlp_forward(const void *enc, const float *xyz, const float *w1, const float *b1,
                            const float *w2, const float *b2, const float *w3, const float *b3,
                            float *sigma, void *rgb, int rgb_dtype, uint32_t M,
                            dfhip_stream_t stream);
/* Backward from grad_sigma [M] f32 and grad_rgb [M, 3] (grad_rgb_dtype F16/F32):
 * d_enc_lbc [16, M, 2] f16 receives the feature gradient in the level-major
 * layout dfhip_grid_encode_backward_sliced consumes; gw1..gb3 (f32, shaped as
 * the parameters) are overwritten (accumulate == 0) or added into.  partial:
 * parts * dfhip_field_mlp_params() floats of scratch with
 * parts = dfhip_field_mlp_backward_parts(M).  Deterministic. */
uint32_t dfhip_field_mlp_backward_parts(uint32_t M);
int dfhip_field_mlp_backward(const void *enc, const float *xyz, const float *w1, const float *b1,
                             const float *w2, const float *b2, const float *w3, const float *b3,
                             const float *grad_sigma, const void *grad_rgb, int grad_rgb_dtype,
                             uint32_t M, void *d_enc_lbc, float *partial, uint32_t parts,
                             float *gw1, float *gb1, float *gw2, float *gb2, float *gw3,
                             float *gb3, int accumulate, dfhip_stream_t stream);

/* The MLP module alone (nerf/network_grid.py:13-32, the reference's sigma_net
 * = 3 nn.Linear + ReLU under autocast; the reference runs 3 hipBLASLt GEMMs +
 * ~20 elementwise / reduction kernels forward and backward): elem DFHIP_F16
 * (fp16 autocast) or DFHIP_BF16; x [cap, 32] and h [cap, 4] in elem, f16 /
 * bf16 GEMM operands with f32 accumulation, elem activations (autocast's
 * numerics), parameters as in dfhip_field_mlp_forward.  With m_dev (device
 * int32 live-row count, e.g. the march's counter[0]) rows [0, *m_dev) are
 * computed and rows [*m_dev, cap) of h (backward: of dx) written as zeros.
 * Backward: dh [cap, 4] elem -> dx [cap, 32] elem (natural layout) and the
 * f32 weight gradients (overwritten, or added into with accumulate);
 * partial: parts * dfhip_field_mlp_params() floats of scratch with parts =
 * dfhip_field_mlp_backward_parts(cap).  Deterministic. */
int dfhip_mlp_forward(int elem, const void *x, const float *w1, const float *b1, const float *w2,
                      const float *b2, const float *w3, const float *b3, void *h, uint32_t cap,
                      const int32_t *m_dev, dfhip_stream_t stream);
int dfhip_mlp_backward(int elem, const void *x, const float *w1, const float *b1,
                       const float *w2, const float *b2, const float *w3, const float *b3,
                       const void *dh, uint32_t cap, const int32_t *m_dev, void *dx,
                       float *partial, uint32_t parts, float *gw1, float *gb1, float *gw2,
                       float *gb2, float *gw3, float *gb3, int accumulate,
                       dfhip_stream_t stream);

/* Fused grid field (native path of nerf/field.py): tiled-grid encoding
 * (gridencoder.cu:75-178 arithmetic, f16 table) + the MLP/heads above in ONE
 * kernel.  xyz: [cap, 3] f32 in [-bound, bound] (mapped to [0,1] as
 * grid.py:142); table: [rows, 2] f16; L must be 16 (C = 2, D = 3).  Only
 * samples [0, *m_dev) are processed when m_dev (device int32, e.g. the
 * march's counter[0]) is given, else [0, cap): no host round trip is needed
 * to size the batch.  enc (nullable): [cap, 32] f16 features in the kernel's
 * permuted order, saved for dfhip_grid_field_backward. */
int dfhip_grid_field_forward(const float *xyz, float bound, const void *table,
                             const int32_t *offsets, uint32_t L, float S, uint32_t H,
                             uint32_t gridtype, int align_corners, const float *w1,
                             const float *b1, const float *w2, const float *b2, const float *w3,
                             const float *b3, void *enc, float *sigma, void *rgb, int rgb_dtype,
                             uint32_t cap, const int32_t *m_dev, dfhip_stream_t stream);
/* bf16 form (BASELINE configs[4], bf16 autocast; new capability — the
 * reference's kernels have no bf16): table [rows, 2] bf16, enc [cap, 32] bf16,
 * hidden activations bf16, v_mfma_f32_16x16x32_bf16 with f32 accumulation,
 * rgb f32 or DFHIP_BF16.  Grid features accumulate in f32 (fmaf per corner,
 * corner order) and are rounded to bf16 once. */
int dfhip_grid_field_forward_bf16(const float *xyz, float bound, const void *table,
                                  const int32_t *offsets, uint32_t L, float S, uint32_t H,
                                  uint32_t gridtype, int align_corners, const float *w1,
                                  const float *b1, const float *w2, const float *b2,
                                  const float *w3, const float *b3, void *enc, float *sigma,
                                  void *rgb, int rgb_dtype, uint32_t cap, const int32_t *m_dev,
                                  dfhip_stream_t stream);
/* The autocast table of the f32 embeddings [rows, 2] (grid.py:38-39's cast to
 * elem = DFHIP_F16 or DFHIP_BF16, written to table [rows, 2]) and its corner
 * quads [rows] x 16 B (16-byte aligned): entry r of a tiled / dense level holds
 * the rows r, r + 1, r + m1, r + m1 + 1 (m1 the level's y stride, wrapped as
 * the corners are), so the quad forward loads a cell's corners 0-3 and 4-7
 * with two 16-byte gathers.  Replaces the per-step cast of the table. */
int dfhip_grid_quads(int elem, const float *embeddings, const int32_t *offsets, uint32_t L,
                     float S, uint32_t H, uint32_t gridtype, int align_corners, uint32_t rows,
                     void *table, void *quads, dfhip_stream_t stream);
/* dfhip_grid_field_forward (elem DFHIP_F16) / _bf16 (DFHIP_BF16) reading the
 * corner quads of dfhip_grid_quads for tiled / dense levels (the table for
 * the others): identical results, 25 instead of 50 gathers per sample. */
int dfhip_grid_field_forward_quads(int elem, const float *xyz, float bound, const void *table,
                                   const void *quads, const int32_t *offsets, uint32_t L,
                                   float S, uint32_t H, uint32_t gridtype, int align_corners,
                                   const float *w1, const float *b1, const float *w2,
                                   const float *b2, const float *w3, const float *b3, void *enc,
                                   float *sigma, void *rgb, int rgb_dtype, uint32_t cap,
                                   const int32_t *m_dev, dfhip_stream_t stream);
/* Backward of dfhip_grid_field_forward: MLP backward (d_enc_lbc [16, cap, 2] f16
 * scratch, mlp_partial: dfhip_field_mlp_backward_parts(cap) * params floats),
 * f32 weight gradients (overwritten), then the sliced embedding backward into
 * grad_embeddings [total_rows, 2] f32 (overwritten; nullable to skip) with
 * grid_partial: dfhip_grid_backward_partial_floats(total_rows, 2, grid_parts). */
int dfhip_grid_field_backward(const void *enc, const float *xyz, float bound, const float *w1,
                              const float *b1, const float *w2, const float *b2,
                              const float *w3, const float *b3, const float *grad_sigma,
                              const void *grad_rgb, int grad_rgb_dtype, uint32_t cap,
                              const int32_t *m_dev, void *d_enc_lbc, float *mlp_partial,
                              uint32_t mlp_parts, float *gw1, float *gb1, float *gw2, float *gb2,
                              float *gw3, float *gb3, const int32_t *offsets,
                              uint32_t total_rows, uint32_t L, float S, uint32_t H,
                              uint32_t gridtype, int align_corners, float *grad_embeddings,
                              float *grid_partial, uint32_t grid_parts, dfhip_stream_t stream);
/* Same, but the weight gradients (and grad_embeddings when given) are ADDED
 * into (dst + new, f32): the second backward of the reference's two-pass step
 * (SDS latents.backward, sd.py:115, then scaler.scale(loss).backward(),
 * utils.py:708), where autograd accumulates each parameter's .grad. */
int dfhip_grid_field_backward_accumulate(
    const void *enc, const float *xyz, float bound, const float *w1, const float *b1,
    const float *w2, const float *b2, const float *w3, const float *b3, const float *grad_sigma,
    const void *grad_rgb, int grad_rgb_dtype, uint32_t cap, const int32_t *m_dev,
    void *d_enc_lbc, float *mlp_partial, uint32_t mlp_parts, float *gw1, float *gb1, float *gw2,
    float *gb2, float *gw3, float *gb3, const int32_t *offsets, uint32_t total_rows, uint32_t L,
    float S, uint32_t H, uint32_t gridtype, int align_corners, float *grad_embeddings,
    float *grid_partial, uint32_t grid_parts, dfhip_stream_t stream);

/* bf16 backward of dfhip_grid_field_forward_bf16: enc and d_enc_lbc
 * [16, cap, 2] are bf16, grad_rgb f32 or DFHIP_BF16; weight gradients f32,
 * overwritten (accumulate == 0) or added into.  The embedding gradient is
 * dfhip_grid_encode_backward_binned with grad_dtype DFHIP_BF16. */
int dfhip_grid_field_backward_bf16(const void *enc, const float *xyz, float bound,
                                   const float *w1, const float *b1, const float *w2,
                                   const float *b2, const float *w3, const float *b3,
                                   const float *grad_sigma, const void *grad_rgb,
                                   int grad_rgb_dtype, uint32_t cap, const int32_t *m_dev,
                                   void *d_enc_lbc, float *mlp_partial, uint32_t mlp_parts,
                                   float *gw1, float *gb1, float *gw2, float *gb2, float *gw3,
                                   float *gb3, int accumulate, dfhip_stream_t stream);

/* Binned owner-computes form of grid_encode_backward (gridencoder.cu:226-313,
 * csrc/gridbin.hip) for D = 3, C in {1, 2, 4}: (sample, level) pairs are binned
 * by the 8192-row LDS slices their corners touch, each slice walks only its
 * bin, partials are summed in a fixed order.  grad_lbc [L, B, C] (f16/f32, B =
 * capacity; rows [0, *m_dev) walked when m_dev != NULL), inputs [B, 3] raw
 * positions mapped (x + bound) / (2 bound) when bound > 0, else already in
 * [0, 1].  offsets_host is a HOST copy of the L + 1 offsets (slice layout);
 * offsets the device copy.  grad_embeddings [rows, C] f32 is overwritten, or
 * added into when accumulate != 0.  [scratch] entries (u16 tile-relative ids,
 * sized in u32 words) / counts (u32) and
 * partial (f32) sized by dfhip_grid_backward_binned_scratch for capacity B. */
int dfhip_grid_backward_binned_scratch(uint32_t cap, const int32_t *offsets_host, uint32_t L,
                                       uint32_t C, uint64_t *entries_u32, uint64_t *counts_u32,
                                       uint64_t *partial_f32);
int dfhip_grid_encode_backward_binned(int grad_dtype, const void *grad_lbc, const float *inputs,
                                      float bound, const int32_t *offsets,
                                      const int32_t *offsets_host, float *grad_embeddings,
                                      uint32_t B, const int32_t *m_dev, uint32_t D, uint32_t C,
                                      uint32_t L, float S, uint32_t H, uint32_t gridtype,
                                      int align_corners, uint32_t *entries, uint32_t *counts,
                                      float *partial, int accumulate, dfhip_stream_t stream);
/* The same in two phases, so the binning (which reads positions only) can run
 * on a second stream beside the forward / MLP backward: phase 1 = bin the
 * samples (entries / counts), 2 = walk + sum (needs phase 1's entries / counts
 * for the same positions and count), 3 = both (dfhip_grid_encode_backward_binned). */
int dfhip_grid_encode_backward_binned_phase(int phase, int grad_dtype, const void *grad_lbc,
                                            const float *inputs, float bound,
                                            const int32_t *offsets, const int32_t *offsets_host,
                                            float *grad_embeddings, uint32_t B,
                                            const int32_t *m_dev, uint32_t D, uint32_t C,
                                            uint32_t L, float S, uint32_t H, uint32_t gridtype,
                                            int align_corners, uint32_t *entries,
                                            uint32_t *counts, float *partial, int accumulate,
                                            dfhip_stream_t stream);
/* The same over finite-difference stencil groups (the textureless /
 * lambertian train step, network_grid.py:90-114): with group = 7, field row
 * 7 g + a of grad_lbc [L, 7 B, C] belongs to point a of sample g (inputs [B,
 * 3] the samples' raw positions): a = 0 the sample, a = 1 + s the point
 * clamp(x + (s odd ? -eps : eps) e_(s >> 1), -bound, bound) — the rows
 * dfhip_shading_stencil lays out.  Binned and walked per group (one entry per
 * (group, slice)), rows [0, *m_dev) of groups; the result equals the row-wise
 * call on the 7 B rows up to the f64 summation order.  Needs C = 2, f16 / bf16
 * gradients, bound > 0 and a mask-form level layout (the reference's grid);
 * group = 1 is dfhip_grid_encode_backward_binned_phase.  Scratch as
 * dfhip_grid_backward_binned_scratch for capacity B (groups). */
int dfhip_grid_encode_backward_binned_stencil(int phase, int grad_dtype, const void *grad_lbc,
                                              const float *inputs, float bound,
                                              const int32_t *offsets, const int32_t *offsets_host,
                                              float *grad_embeddings, uint32_t B,
                                              const int32_t *m_dev, uint32_t D, uint32_t C,
                                              uint32_t L, float S, uint32_t H, uint32_t gridtype,
                                              int align_corners, uint32_t group, float eps,
                                              uint32_t *entries, uint32_t *counts,
                                              float *partial, int accumulate,
                                              dfhip_stream_t stream);
/* Per-call options of the binned backward: A/B and test switches of one call,
 * nothing kept between calls (the library holds no mode state).  A field < 0
 * (or 0 where noted) keeps the default; NULL options = all defaults. */
typedef struct dfhip_binned_opts {
    int32_t walk_mode;          /* -1 default: per-segment walk for single samples, flat walk
                                   for stencil groups; 0 per-segment, 1 flat (mask-form
                                   layouts) */
    int32_t fast_bin;           /* -1 / 1: mask-form fast binning where it applies; 0 the
                                   generic binning kernel */
    int32_t walk_groups_per_cu; /* 0 default (3); 1..16 walk workgroups per CU (changes the
                                   partial scratch size: pass the same opts to the scratch call) */
    int32_t lane_perm;          /* -1 default (1): per-segment walk lanes take runs in
                                   bit-reversed order (1) or in lane order (0) */
    int32_t kept_clean;         /* <= 0 default: the call clears the counts scratch's totals /
                                   plan words with a fill launch; 1: no fill launch — the
                                   counts scratch is freshly zeroed or was last used by a
                                   completed binned call with the same B and group (every
                                   call leaves its totals zero and the walk rewrites every
                                   bin's plan; the totals' place depends on B) */
    uint64_t *trace;            /* debug: per-workgroup walk timeline, 8 u64 per walk
                                   workgroup {bin, XCC id << 32 | HW_ID, parts, entries,
                                   t0 (start), t1 (plan done), part, t2 (end)} (every walk
                                   form, wall clock at 100 MHz); NULL = off */
} dfhip_binned_opts;
/* dfhip_grid_backward_binned_scratch / dfhip_grid_encode_backward_binned_stencil
 * with per-call options (group 1 = single samples, eps ignored; group 7 =
 * stencil groups; any other group is DFHIP_EINVAL).  The partial scratch
 * depends on the options (walk_groups_per_cu): size it with the opts the
 * launches will use.  Host only (no device work, no device pointers). */
int dfhip_grid_backward_binned_scratch_opts(uint32_t cap, const int32_t *offsets_host,
                                            uint32_t L, uint32_t C, uint32_t group,
                                            const dfhip_binned_opts *opts, uint64_t *entries_u32,
                                            uint64_t *counts_u32, uint64_t *partial_f32);
/* Samples per binning tile (the id slots of one (tile, slice) segment of the
 * entries scratch) of a call with this group and these options; 0 on bad
 * options. */
uint32_t dfhip_grid_backward_binned_tile(uint32_t group, const dfhip_binned_opts *opts);
int dfhip_grid_encode_backward_binned_opts(int phase, int grad_dtype, const void *grad_lbc,
                                           const float *inputs, float bound,
                                           const int32_t *offsets, const int32_t *offsets_host,
                                           float *grad_embeddings, uint32_t B,
                                           const int32_t *m_dev, uint32_t D, uint32_t C,
                                           uint32_t L, float S, uint32_t H, uint32_t gridtype,
                                           int align_corners, uint32_t group, float eps,
                                           uint32_t *entries, uint32_t *counts, float *partial,
                                           int accumulate, const dfhip_binned_opts *opts,
                                           dfhip_stream_t stream);

/* nerf/utils.py:708-713 scaler.step(optimizer); scaler.update() for
 * torch.optim.Adam (csrc/optim.hip): non-finite check of every grad, then (if
 * all finite) torch's fused Adam update with grad / *scale, then step += 1 per
 * tensor and torch._amp_update_scale_ on (*scale, *growth_tracker);
 * *found_inf (f32, zero on entry) is reset to 0 on exit.  Per tensor k (at
 * most 24): f32 param / grad / exp_avg / exp_avg_sq [numel[k]], the device f32
 * step counter, and the group's lr, betas, eps, weight_decay.  Pointer and
 * hyper-parameter arrays are HOST arrays. */
int dfhip_adam_amp_step(int count, float *const *params, const float *const *grads,
                        float *const *exp_avg, float *const *exp_avg_sq, float *const *steps,
                        const uint64_t *numel, const float *lr, const float *beta1,
                        const float *beta2, const float *eps, const float *weight_decay,
                        float *scale, int32_t *growth_tracker, float *found_inf,
                        float growth_factor, float backoff_factor, int growth_interval,
                        dfhip_stream_t stream);
/* The same update with the learning rates read on the device at run time:
 * tensor k uses lr_dev[lr_slot[k]] (lr_slot: HOST int array, values 0..255;
 * lr_dev: DEVICE f32 array), so the launches can be captured once in a HIP
 * graph and replayed while LambdaLR changes the rates (main.py:131; the native
 * train step writes lr_dev from its prologue, dfhip_train_step_prologue_lr). */
int dfhip_adam_amp_step_lr_dev(int count, float *const *params, const float *const *grads,
                               float *const *exp_avg, float *const *exp_avg_sq,
                               float *const *steps, const uint64_t *numel,
                               const int32_t *lr_slot, const float *lr_dev, const float *beta1,
                               const float *beta2, const float *eps, const float *weight_decay,
                               float *scale, int32_t *growth_tracker, float *found_inf,
                               float growth_factor, float backoff_factor, int growth_interval,
                               dfhip_stream_t stream);
/* Per-ray tail of run_cuda (nerf/renderer.py:536-551, csrc/head.hip).
 * Forward: bg = sigmoid(W2 relu(W1 freq6(rays_d) + b1) + b2) with the
 * reference's fp16 autocast rounding (w1 != NULL: W1 [64, 39], b1 [64], W2
 * [3, 64], b2 [3] f32), else bg = bg_color [N, 3] (or 1 when NULL);
 * out_image [3, N] (channel-major) = image + (1 - ws) * bg;
 * out_depth = max(depth - near, 0) / (far - near); mask = near < far (0/1
 * bytes).  Backward: grad_image [N, 3] = g_image^T, grad_ws = -sum_c g_c bg_c,
 * grad_bg = g * (1 - ws) (bg_color mode, optional) or the MLP weight grads
 * gw1..gb2 (f32, overwritten) via `partial` sized by
 * dfhip_ray_head_partial_floats(N). */
uint32_t dfhip_ray_head_partial_floats(uint32_t N);
int dfhip_ray_head_forward(uint32_t N, const float *ws, const float *depth, const float *image,
                           const float *rays_d, const float *nears, const float *fars,
                           const float *w1, const float *b1, const float *w2, const float *b2,
                           const float *bg_color, float *out_image, float *out_depth,
                           uint8_t *mask, dfhip_stream_t stream);
int dfhip_ray_head_backward(uint32_t N, const float *g_image, const float *ws,
                            const float *rays_d, const float *w1, const float *b1,
                            const float *w2, const float *b2, const float *bg_color,
                            float *grad_image, float *grad_ws, float *grad_bg, float *partial,
                            float *gw1, float *gb1, float *gw2, float *gb2,
                            dfhip_stream_t stream);
/* The same with the entropy regulariser's backward fused (utils.py:386-391):
 * grad_ws = -(sum_c g_c bg_c) + grad_loss[0] * lambda / N * log2((1 - a) / a)
 * (zero where the clamp to [1e-5, 1 - 1e-5] is active), i.e. what
 * dfhip_ray_head_backward followed by dfhip_entropy_backward_accumulate write,
 * bit for bit, in one pass (native train step). */
int dfhip_ray_head_backward_entropy(uint32_t N, const float *g_image, const float *ws,
                                    const float *rays_d, const float *w1, const float *b1,
                                    const float *w2, const float *b2, const float *bg_color,
                                    float *grad_image, float *grad_ws, float *grad_bg,
                                    float *partial, float *gw1, float *gb1, float *gw2,
                                    float *gb2, const float *grad_loss, float lambda,
                                    dfhip_stream_t stream);
/* dfhip_ray_head_backward_entropy that also writes the entropy loss
 * lambda * mean(entropy(clamp(ws))) (dfhip_entropy_forward's value, same
 * reduction) to loss[0], computed inside the weight-gradient sum launch. */
int dfhip_ray_head_backward_entropy_loss(uint32_t N, const float *g_image, const float *ws,
                                         const float *rays_d, const float *w1, const float *b1,
                                         const float *w2, const float *b2,
                                         const float *bg_color, float *grad_image,
                                         float *grad_ws, float *grad_bg, float *partial,
                                         float *gw1, float *gb1, float *gw2, float *gb2,
                                         const float *grad_loss, float lambda, float *loss,
                                         dfhip_stream_t stream);
/* dfhip_ray_head_forward followed by dfhip_ray_head_backward_entropy_loss, in
 * two launches instead of three (the backward's recomputed background is the
 * forward's: outputs bit-identical), for an upstream g_image that does not
 * depend on out_image (the native step's injected SDS gradient).  Background
 * network only (w1 != NULL); no bg_color / grad_bg. */
int dfhip_ray_head_forward_backward_entropy_loss(
    uint32_t N, const float *ws, const float *depth, const float *image, const float *rays_d,
    const float *nears, const float *fars, const float *w1, const float *b1, const float *w2,
    const float *b2, float *out_image, float *out_depth, uint8_t *mask, const float *g_image,
    float *grad_image, float *grad_ws, float *partial, float *gw1, float *gb1, float *gw2,
    float *gb2, const float *grad_loss, float lambda, float *loss, dfhip_stream_t stream);

/* nerf/utils.py:386-391 entropy regulariser: loss[0] = lambda * mean(-a log2 a
 * - (1 - a) log2(1 - a)), a = clamp(ws, 1e-5, 1 - 1e-5) (f64 sum); backward
 * grad_ws = grad_loss[0] * lambda / N * log2((1 - a) / a) where the clamp
 * passes, 0 elsewhere. */
int dfhip_entropy_forward(uint32_t N, const float *ws, float lambda, float *loss,
                          dfhip_stream_t stream);
int dfhip_entropy_backward(uint32_t N, const float *ws, const float *grad_loss, float lambda,
                           float *grad_ws, dfhip_stream_t stream);
/* The same gradient added into grad_ws (grad_ws += ...): the autograd sum of
 * the entropy term and the ray head's gradient of the weights sum, one
 * launch (the native train step, nerf/native_step.py). */
int dfhip_entropy_backward_accumulate(uint32_t N, const float *ws, const float *grad_loss,
                                      float lambda, float *grad_ws, dfhip_stream_t stream);

/* Prologue of the native albedo train step (nerf/native_step.py), one launch:
 * camera rays of an H x W pinhole image from a host 3x4 cam2world `pose`
 * (as dfhip_get_rays; nerf/utils.py:42-106), their box intersection with
 * aabb[6] and min_near (as dfhip_near_far_from_aabb; raymarching.py:19-49),
 * the march noise (raymarching.py:200, 0 unless perturb), the background
 * colour draw bg_color [N,3] (utils.py:349; NULL to skip), the synthetic SDS
 * gradient g_image [3,N] = (1 - alphas[t]) * eps, t ~ U{min_step..max_step},
 * eps ~ N(0,1) (nerf/sd.py InjectedSDS; NULL to skip) and counter[0..1] = 0
 * (renderer.py:470; NULL to skip).  Random numbers: Philox4x32-10 keyed by
 * `seed`, counter (ray, step, stream) — fresh per step index, independent of
 * the launch shape. */
int dfhip_train_step_prologue(const float *pose, float fx, float fy, float cx, float cy,
                              uint32_t H, uint32_t W, const float *aabb, float min_near,
                              uint64_t seed, uint64_t step, int perturb, const float *alphas,
                              uint32_t min_step, uint32_t max_step, float *rays_o,
                              float *rays_d, float *nears, float *fars, float *noises,
                              float *bg_color, float *g_image, int32_t *counter,
                              dfhip_stream_t stream);
/* The same launch also writing this step's learning rates lr_dev[0..n_lr) =
 * lr_host[0..n_lr) (n_lr <= 8; lr_host a HOST array copied into the launch's
 * arguments, lr_dev DEVICE memory), read later in the step by
 * dfhip_adam_amp_step_lr_dev inside the replayed graph. */
int dfhip_train_step_prologue_lr(const float *pose, float fx, float fy, float cx, float cy,
                                 uint32_t H, uint32_t W, const float *aabb, float min_near,
                                 uint64_t seed, uint64_t step, int perturb, const float *alphas,
                                 uint32_t min_step, uint32_t max_step, float *rays_o,
                                 float *rays_d, float *nears, float *fars, float *noises,
                                 float *bg_color, float *g_image, int32_t *counter,
                                 const float *lr_host, uint32_t n_lr, float *lr_dev,
                                 dfhip_stream_t stream);

/* nerf/renderer.py:496-532 — the inference branch of run_cuda (the host loop
 * of march_rays raymarching.cu:700-804 -> network_grid.common_forward
 * network_grid.py:76-87 under fp16 autocast -> composite_rays
 * raymarching.cu:818-905 -> rays_alive compaction), fused into ONE persistent
 * launch for the albedo shading of the reference's grid field (16 levels x 2
 * channels, sigma MLP 32 -> 64 -> 64 -> 4).
 * In:  rays_o, rays_d [N,3] f32; nears, fars [N] f32 (near_far_from_aabb);
 *      noises [N] f32 or NULL (perturbation of the first march step);
 *      bound, dt_gamma, max_steps, C (cascade), H (density grid size), grid =
 *      density bitfield [C*H^3/8] u8; T_thresh; table [rows,2] f16 (the
 *      autocast copy of the embeddings), offsets [L+1] i32, L, S = log2
 *      per-level scale, base_res, gridtype, align_corners (as
 *      dfhip_grid_encode_forward); w1..b3 the f32 nn.Linear parameters.
 * Out: weights_sum [N], depth [N] (sum of w * t with t measured from the
 *      near plane's rays_t, as composite_rays leaves it), image [N,3] f32 —
 *      every ray written once (no zero-fill needed).
 * work: [4] u32 caller scratch, zeroed here; after the launch work[1] +
 *      2^32 work[2] = number of samples evaluated.
 * quads: the table's corner quads [rows, 4] u32 (dfhip_grid_quads of the
 *      same table) or NULL: with them the field gathers each level's corners
 *      0-3 / 4-7 as two 16-byte loads (bit-identical features). */
int dfhip_render_rays_infer(uint32_t N, const float *rays_o, const float *rays_d,
                            const float *nears, const float *fars, const float *noises,
                            float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
                            uint32_t H, const uint8_t *grid, float T_thresh, const void *table,
                            const int32_t *offsets, uint32_t L, float S, uint32_t base_res,
                            uint32_t gridtype, int align_corners, const float *w1,
                            const float *b1, const float *w2, const float *b2, const float *w3,
                            const float *b3, float *weights_sum, float *depth, float *image,
                            uint32_t *work, const void *quads, dfhip_stream_t stream);
/* The same with a debug profile of this call: prof (DEVICE u64 [16 + 16 W];
 * caller sets [6] and [7] to UINT64_MAX, [10] to W >= 0 and the others to 0)
 * receives the per-wave
 * phase cycles of the persistent kernel summed {refill, march, field,
 * composite, rounds, field tiles}, then wall-clock ticks (100 MHz): [6] the
 * first wave's start, [7] the first time a wave found the ray queue empty,
 * [8] the last wave's end, [9] the waves' lifetimes summed (the drain after
 * the queue ran dry and the mean resident waves), and for the first W waves
 * of the grid a record at [16 + 16 w]: {start, the time it first found the
 * queue empty (0: never), end, rounds << 32 | rounds then << 8 | rays held
 * then, the most samples one of its rays marched, its samples composited,
 * the most one of its rays composited, its rays retired, its phase cycles
 * [0..5] as above, 0, 0}.  NULL = the call above.
 * Used by tools/infer_case.py. */
int dfhip_render_rays_infer_prof(uint32_t N, const float *rays_o, const float *rays_d,
                                 const float *nears, const float *fars, const float *noises,
                                 float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
                                 uint32_t H, const uint8_t *grid, float T_thresh,
                                 const void *table, const int32_t *offsets, uint32_t L, float S,
                                 uint32_t base_res, uint32_t gridtype, int align_corners,
                                 const float *w1, const float *b1, const float *w2,
                                 const float *b2, const float *w3, const float *b3,
                                 float *weights_sum, float *depth, float *image, uint32_t *work,
                                 const void *quads, uint64_t *prof, dfhip_stream_t stream);
/* dfhip_render_rays_infer[_prof] taking rays from the queue chunk by chunk:
 * order[0 .. ceil(N / 2^chunk_log2)) (DEVICE int32, a permutation of the
 * chunk indices; NULL = pixel order) names the chunks of 2^chunk_log2
 * consecutive rays in queue order (tile_w > 0: chunk c is the 8 x 8 pixel
 * tile c of a row-major image tile_w pixels wide, tiles row-major; needs
 * chunk_log2 6 and N a multiple of 8 tile_w).  The persistent kernel's tail
 * is the rays still marching after the queue ran dry, so a caller puts the
 * costly chunks first (dfhip_render_ray_order); whole chunks keep a wave's
 * refills on neighbouring pixels.  The queue takes the order in blocks of G
 * positions (G = the launch's resident waves, so every wave's first grab is
 * in the first block): grab g of a block takes the first half of chunk g and
 * the second half of chunk G-1-g, so no wave starts on two halves of the
 * costliest chunks (chunk_log2 >= 1).  Outputs are per ray: any order gives
 * the same results; ids >= N (the partial last chunk) and order entries that
 * are not chunk indices are skipped. */
int dfhip_render_rays_infer_ordered(uint32_t N, const float *rays_o, const float *rays_d,
                                    const float *nears, const float *fars, const float *noises,
                                    float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
                                    uint32_t H, const uint8_t *grid, float T_thresh,
                                    const void *table, const int32_t *offsets, uint32_t L,
                                    float S, uint32_t base_res, uint32_t gridtype,
                                    int align_corners, const float *w1, const float *b1,
                                    const float *w2, const float *b2, const float *w3,
                                    const float *b3, float *weights_sum, float *depth,
                                    float *image, uint32_t *work, const void *quads,
                                    const int32_t *order, uint32_t chunk_log2, uint32_t tile_w,
                                    uint64_t *prof, dfhip_stream_t stream);
/* The queue order for dfhip_render_rays_infer_ordered: the chunks of
 * 2^chunk_log2 consecutive rays (rays_o / rays_d [N, 3] f32) by ascending
 * summed squared distance of their rays' lines from the scene centre (the
 * bound box's centre, the origin), i.e. the rays crossing the most of the
 * scene first — the cost quantised to 64 levels between its min and max,
 * ties in chunk order (a stable counting sort).  cost: [nchunks] f32
 * scratch (the per-chunk cost, a partial last chunk scaled to a whole one);
 * order: [nchunks] int32 out; nchunks = ceil(N / 2^chunk_log2) <= 16384;
 * tile_w: the chunks are 8 x 8 pixel tiles as in
 * dfhip_render_rays_infer_ordered (0: consecutive rays).  Two launches,
 * deterministic. */
int dfhip_render_ray_order(const float *rays_o, const float *rays_d, uint32_t N,
                           uint32_t chunk_log2, uint32_t tile_w, float *cost, int32_t *order,
                           dfhip_stream_t stream);
/* The same order from the occupancy grid (grid: the march's bitfield, C
 * cascades of H^3; nears / fars [N] f32): a chunk's cost is minus the occupied
 * cells met at 16 evenly spaced points of each ray's [near, far), so the
 * rays crossing the most occupied space come first. */
int dfhip_render_ray_order_occ(const float *rays_o, const float *rays_d, const float *nears,
                               const float *fars, const uint8_t *grid, float bound, uint32_t C,
                               uint32_t H, uint32_t max_steps, uint32_t N, uint32_t chunk_log2,
                               uint32_t tile_w, float *cost, int32_t *order,
                               dfhip_stream_t stream);

/* ---- non-albedo shading of the train step (csrc/shade.hip) ------------------
 * Replaces, for the `textureless` / `lambertian` steps, network_grid.py:90-144
 * (finite_difference_normal: six common_forward calls at the clamped stencil
 * points, safe_normalize, NaN -> 0, lambertian = ratio + (1 - ratio) *
 * clamp(normal @ l, min=0), colour) and renderer.py:485-489 (orientation
 * loss).  The stencil evaluations are extra rows of one field launch over a
 * [7 cap, 3] position buffer: row 7 i = sample i (of the M = *m_dev march
 * samples), rows 7 i + 1 + a = its stencil point a (+x, -x, +y, -y, +z, -z).
 *
 * dfhip_shading_stencil: xyz [cap, 3] (march samples) -> xyz7 [7 cap, 3] rows
 *   7 i + k (clamp(x_i + eps e, -bound, bound)) and *m7_dev = 7 M. */
int dfhip_shading_stencil(const float *xyz, const int32_t *m_dev, uint32_t cap, float eps,
                          float bound, float *xyz7, int32_t *m7_dev, dfhip_stream_t stream);
/* Scratch doubles for dfhip_shading_forward's orientation partial sums. */
uint32_t dfhip_shading_partial_doubles(uint32_t cap);
/* sigma7 [7 cap] f32 / albedo7 [7 cap, 3] f16 = the field on the 7 M rows,
 * dirs [cap, 3], light [3] f32 (device) -> sigma [cap] f32 and color [cap, 3]
 * f16 of the samples (compositing inputs), normal [cap, 3] f32, the
 * orientation mean over the march's padded row count M'
 * (raymarching.py:224-227) into *orient (nullable), and
 * *loss += lambda_orient * orient (nullable). */
int dfhip_shading_forward(const float *sigma7, const void *albedo7, const float *dirs,
                          const float *light, float ratio, float eps, int shading,
                          const int32_t *m_dev, uint32_t cap, float *sigma, void *color,
                          float *normal, double *partial, float lambda_orient, float *orient,
                          float *loss, dfhip_stream_t stream);
/* grad_sigma [cap] f32 / grad_color [cap, 3] f16 (compositing backward) and the
 * loss scale grad_loss[0] (upstream of lambda_orient * orient) -> the field-row
 * gradients grad_sigma7 [7 cap] f32 and grad_albedo7 [7 cap, 3] f16 of all 7 M
 * rows. */
int dfhip_shading_backward(const float *sigma7, const void *albedo7, const float *dirs,
                           const float *light, float ratio, float eps, int shading,
                           const int32_t *m_dev, uint32_t cap, const float *grad_sigma,
                           const void *grad_color, const float *grad_loss, float lambda_orient,
                           float *grad_sigma7, void *grad_albedo7, dfhip_stream_t stream);
/* bf16 forms (bf16 autocast, the C5 option): albedo7 / color / grad_color /
 * grad_albedo7 are bf16 and the autocast rounding points round to bf16. */
int dfhip_shading_forward_bf16(const float *sigma7, const void *albedo7, const float *dirs,
                               const float *light, float ratio, float eps, int shading,
                               const int32_t *m_dev, uint32_t cap, float *sigma, void *color,
                               float *normal, double *partial, float lambda_orient,
                               float *orient, float *loss, dfhip_stream_t stream);
int dfhip_shading_backward_bf16(const float *sigma7, const void *albedo7, const float *dirs,
                                const float *light, float ratio, float eps, int shading,
                                const int32_t *m_dev, uint32_t cap, const float *grad_sigma,
                                const void *grad_color, const float *grad_loss,
                                float lambda_orient, float *grad_sigma7, void *grad_albedo7,
                                dfhip_stream_t stream);
/* The step's light direction safe_normalize(rays_o[0] + randn(3))
 * (renderer.py:462-464), drawn from Philox keyed by (seed, step). */
int dfhip_shading_light(const float *rays_o, uint64_t seed, uint64_t step, float *light,
                        dfhip_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* DFHIP_H */
