// Multi-resolution tiled / hashed grid encoding for gfx950 (MI355X).
//
// Behavioural spec: reference gridencoder/src/gridencoder.cu (cited per kernel)
// and gridencoder/grid.py.  Numerics: explicit fmaf() where nvcc contracts
// (gridencoder.cu:134,165), half accumulators rounded per corner exactly as
// c10::Half arithmetic does (gridencoder.cu:142,165: the product w*g is rounded
// to half, then added in half), compiled with -ffp-contract=off.
//
// MI355X design:
//  * One thread per sample loops over all levels: at every gather instruction
//    the 64 lanes of a wave sit on the SAME level (level-major gathers, good L2
//    line reuse at the coarse levels) while the thread keeps 16 independent
//    level chains in flight (ILP for the ~500-cycle L2/MALL latency).
//  * Per-level constants (scale, resolution) are computed once on the host and
//    passed as kernel arguments, with a correctly rounded exp2 (exact at the
//    integer exponents of levels 0 and L-1).
//  * Levels whose tiled index drops a trailing dimension (stride overflow,
//    gridtype.cu:60) gather each shared corner once and reuse it; the backward
//    merges those corners' weights into one atomic per shared table row.
//  * The native [B, L*C] output / grad layout removes the reference's two
//    permute copies (grid.py:42,70).
#include "common.h"

#include "grid_common.h"

namespace dfhip {
namespace ge {

// ------------------------------------------------------------ forward

// gridencoder.cu:75-223.  BLC: outputs [B, L*C] (native) else [L, B, C].
// dyn (grid_common.h SliceDyn): with a device count, rows [*m_dev, B) of a
// capacity-sized batch are written as zeros (their features stay finite for
// whatever reads the whole batch) and no table row is gathered for them; with
// bound > 0 the inputs are raw positions mapped as grid.py:142 does.
template <typename scalar_t, uint32_t D, uint32_t C, bool BLC>
__global__ __launch_bounds__(256) void k_grid_fwd(const float *__restrict__ inputs,
                                                  const scalar_t *__restrict__ grid,
                                                  const int32_t *__restrict__ offsets,
                                                  scalar_t *__restrict__ outputs, uint32_t B,
                                                  uint32_t L, Levels lv,
                                                  scalar_t *__restrict__ dy_dx,
                                                  uint32_t gridtype, int align_corners,
                                                  SliceDyn dyn) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const bool align = align_corners != 0;

    float x[D];
    // a row past the live count reads no input and comes out as zeros, like
    // an out-of-bounds sample
    bool oob = b >= dyn_count(dyn, B);
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        x[d] = oob ? 0.0f : dyn_map(dyn, inputs[(size_t)b * D + d]);
        if (x[d] < 0.0f || x[d] > 1.0f) oob = true;
    }

    for (uint32_t l = 0; l < L; ++l) {
        scalar_t *out = BLC ? outputs + (size_t)b * L * C + (size_t)l * C
                            : outputs + (size_t)l * B * C + (size_t)b * C;
        if (oob) {
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) out[ch] = (scalar_t)0.0f;
            if (dy_dx) {
                scalar_t *g = dy_dx + (size_t)b * D * L * C + (size_t)l * D * C;
                for (uint32_t i = 0; i < D * C; ++i) g[i] = (scalar_t)0.0f;
            }
            continue;
        }
        const LevelCtx c = level_ctx<D>(offsets, lv, l, gridtype, align);
        const scalar_t *tab = grid + (size_t)c.base * C;

        float frac[D];
        uint32_t cell[D];
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) {
            const float p = fmaf(x[d], c.scale, align ? 0.0f : 0.5f);
            cell[d] = (uint32_t)floorf(p);
            frac[d] = p - (float)cell[d];
        }

        scalar_t acc[C];
#pragma unroll
        for (uint32_t ch = 0; ch < C; ++ch) acc[ch] = (scalar_t)0.0f;

        // Tiled levels whose index ignores the trailing dims: every corner with
        // the same leading-dim bits reads the same row; gather it once.
        const uint32_t lead = (!c.hashed) ? c.used : D;
        const uint32_t lead_mask = (1u << lead) - 1u;
        scalar_t cached[1u << D][C];
#pragma unroll
        for (uint32_t k = 0; k < (1u << D); ++k) {
            float w = 1.0f;
            uint32_t p[D];
#pragma unroll
            for (uint32_t d = 0; d < D; ++d) {
                if (k & (1u << d)) { w *= frac[d]; p[d] = cell[d] + 1u; }
                else { w *= 1.0f - frac[d]; p[d] = cell[d]; }
            }
            if ((k & ~lead_mask) == 0 || dy_dx) {
                const uint32_t row = row_index<D>(c, p);
#pragma unroll
                for (uint32_t ch = 0; ch < C; ++ch) cached[k][ch] = tab[(size_t)row * C + ch];
            } else {
#pragma unroll
                for (uint32_t ch = 0; ch < C; ++ch) cached[k][ch] = cached[k & lead_mask][ch];
            }
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) acc_corner(acc[ch], w, cached[k][ch]);
        }
#pragma unroll
        for (uint32_t ch = 0; ch < C; ++ch) out[ch] = acc[ch];

        if (dy_dx) {
            // gridencoder.cu:179-222: d(out)/d(x_gd) = scale * sum over the
            // other dims' corners of w * (right - left).
            scalar_t *g = dy_dx + (size_t)b * D * L * C + (size_t)l * D * C;
#pragma unroll
            for (uint32_t gd = 0; gd < D; ++gd) {
                scalar_t rg[C];
#pragma unroll
                for (uint32_t ch = 0; ch < C; ++ch) rg[ch] = (scalar_t)0.0f;
#pragma unroll
                for (uint32_t k = 0; k < (1u << (D - 1)); ++k) {
                    float w = c.scale;
                    uint32_t kl = 0;
#pragma unroll
                    for (uint32_t nd = 0; nd < D - 1; ++nd) {
                        const uint32_t d = (nd >= gd) ? nd + 1 : nd;
                        if (k & (1u << nd)) { w *= frac[d]; kl |= 1u << d; }
                        else { w *= 1.0f - frac[d]; }
                    }
                    const uint32_t kr = kl | (1u << gd);
#pragma unroll
                    for (uint32_t ch = 0; ch < C; ++ch) {
                        // scalar_t subtraction (c10::Half - Half -> Half)
                        const scalar_t diff = (scalar_t)(cached[kr][ch] - cached[kl][ch]);
                        acc_corner(rg[ch], w, diff);
                    }
                }
#pragma unroll
                for (uint32_t ch = 0; ch < C; ++ch) g[gd * C + ch] = rg[ch];
            }
        }
    }
}

// ------------------------------------------------------------ backward

// No-return atomic adds of one table row's C channels.
template <uint32_t C>
__device__ __forceinline__ void row_atomic_add(float *dst, const float v[C]) {
#pragma unroll
    for (uint32_t ch = 0; ch < C; ++ch) unsafeAtomicAdd(dst + ch, v[ch]);
}
template <uint32_t C>
__device__ __forceinline__ void row_atomic_add(double *dst, const float v[C]) {
#pragma unroll
    for (uint32_t ch = 0; ch < C; ++ch) unsafeAtomicAdd(dst + ch, (double)v[ch]);
}
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
template <uint32_t C>
__device__ __forceinline__ void row_atomic_add(half_t *dst, const float v[C]) {
    // gridencoder.cu:298-304: each product rounded to half, packed pairs added
    // with one global_atomic_pk_add_f16.
#pragma unroll
    for (uint32_t ch = 0; ch < C; ch += 2) {
        half2_t p;
        p.x = (half_t)f32_rounded(v[ch]);
        p.y = (half_t)f32_rounded(v[ch + 1]);
        typedef __attribute__((address_space(1))) half2_t global_half2_t;
        __builtin_amdgcn_global_atomic_fadd_v2f16((global_half2_t *)(dst + ch), p);
    }
}

// gridencoder.cu:226-313.  Grad layout: BLC [B, L*C] (native) or [L, B, C].
// Corners that share a row (tiled levels with dropped trailing dims) are merged
// into one atomic with the summed weight.
template <typename grad_t, typename acc_t, uint32_t D, uint32_t C, bool BLC>
__global__ __launch_bounds__(256) void k_grid_bwd(const grad_t *__restrict__ grad,
                                                  const float *__restrict__ inputs,
                                                  const int32_t *__restrict__ offsets,
                                                  acc_t *__restrict__ grad_grid, uint32_t B,
                                                  uint32_t L, Levels lv, uint32_t gridtype,
                                                  int align_corners) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const bool align = align_corners != 0;
    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        x[d] = inputs[(size_t)b * D + d];
        if (x[d] < 0.0f || x[d] > 1.0f) return;  // grads stay zero
    }
    for (uint32_t l = 0; l < L; ++l) {
        const grad_t *gp = BLC ? grad + (size_t)b * L * C + (size_t)l * C
                               : grad + (size_t)l * B * C + (size_t)b * C;
        float g[C];
#pragma unroll
        for (uint32_t ch = 0; ch < C; ++ch) g[ch] = (float)gp[ch];

        const LevelCtx c = level_ctx<D>(offsets, lv, l, gridtype, align);
        acc_t *tab = grad_grid + (size_t)c.base * C;
        float frac[D];
        uint32_t cell[D];
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) {
            const float p = fmaf(x[d], c.scale, align ? 0.0f : 0.5f);
            cell[d] = (uint32_t)floorf(p);
            frac[d] = p - (float)cell[d];
        }
        const uint32_t lead = (!c.hashed) ? c.used : D;
        // Leading-dim corners, each carrying the summed weight of the trailing
        // corners that map to the same row.
        float tw = 1.0f;  // sum over trailing-dim corners = prod(1 - f + f)
#pragma unroll
        for (uint32_t d = 0; d < D; ++d)
            if (d >= lead) tw *= (1.0f - frac[d]) + frac[d];
#pragma unroll
        for (uint32_t k = 0; k < (1u << D); ++k) {
            if (k >> lead) continue;  // uniform per level
            float w = tw;
            uint32_t p[D];
#pragma unroll
            for (uint32_t d = 0; d < D; ++d) {
                if (d < lead) {
                    if (k & (1u << d)) { w *= frac[d]; p[d] = cell[d] + 1u; }
                    else { w *= 1.0f - frac[d]; p[d] = cell[d]; }
                } else {
                    p[d] = cell[d];
                }
            }
            const uint32_t row = row_index<D>(c, p);
            float v[C];
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) v[ch] = w * g[ch];
            row_atomic_add<C>(tab + (size_t)row * C, v);
        }
    }
}

// ------------------------------------------------------------ backward, sliced
//
// gridencoder.cu:226-313 restructured for gfx950.  The reference scatters
// 2^D * L * C / 2 half2 atomics per sample straight to HBM: at the coarse
// levels dozens of lanes of one wave hit the same row (serialised at the
// memory-side atomic unit) and at the fine levels every lane hits its own
// 64-B line, so the kernel runs at ~1 % of the chip's atomic rate.
//
// Owner-computes instead: the table's rows are cut into slices that fit in
// one CU's 160 KiB LDS.  Workgroup (slice s, part p) walks the samples of
// part p for every level overlapping slice s, and accumulates the corner
// contributions that land in s with LDS atomics.  The accumulators are f64:
// on gfx950 ds_add_f64 sustains ~2.5 lane-ops/CU/cycle against ~0.33 for
// ds_add_f32 / ds_pk_add_f16 (tools/micro/lds_atomic.hip), so doubles halve
// the rows per slice but make the accumulation ~8x faster (and the sums
// exact to f32 output precision).  The slice is then written out as f32 with
// plain coalesced stores into partial[p]; a second pass sums the P partials
// per row (fixed order) into the gradient.
// No global atomics, HBM traffic = inputs + grads read once per slice of
// their level + 2 * P * table bytes.
// Flush the accumulated corner contributions of one cell into the LDS slice.
template <uint32_t D, uint32_t C>
__device__ __forceinline__ void flush_cell(double *acc, uint32_t r0, uint32_t r1,
                                           const LevelCtx &c, uint32_t lead,
                                           const uint32_t cell[D], const float (&cw)[1u << D][C]) {
#pragma unroll
    for (uint32_t k = 0; k < (1u << D); ++k) {
        if (k >> lead) continue;
        uint32_t p[D];
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) p[d] = cell[d] + ((d < lead && (k & (1u << d))) ? 1u : 0u);
        const uint32_t row = c.base + row_index<D>(c, p);
        if (row >= r0 && row < r1) {
            double *dst = acc + (row - r0) * C;
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) atomicAdd(dst + ch, (double)cw[k][ch]);
        }
    }
}

constexpr uint32_t kRunLen = 8;  // samples walked sequentially per thread and level

// Load n <= K consecutive items of W 32-bit words each into registers, as
// 16-byte vectors when the run is full and aligned.
template <uint32_t K, uint32_t W>
__device__ __forceinline__ void load_run(const uint32_t *__restrict__ src, uint32_t n, bool vec,
                                         uint32_t (&dst)[K * W]) {
    if (vec && n == K) {
        static_assert((K * W) % 4 == 0, "run must be a whole number of 16-B vectors");
        const uint4 *v = reinterpret_cast<const uint4 *>(src);
#pragma unroll
        for (uint32_t i = 0; i < K * W / 4; ++i) {
            const uint4 q = v[i];
            dst[4 * i] = q.x; dst[4 * i + 1] = q.y; dst[4 * i + 2] = q.z; dst[4 * i + 3] = q.w;
        }
    } else {
#pragma unroll
        for (uint32_t i = 0; i < K * W; ++i) dst[i] = (i < n * W) ? src[i] : 0u;
    }
}

// Generic shapes: one sample per lane, no run merging (lanes of a wave read
// consecutive samples, coalesced).
template <typename grad_t, uint32_t D, uint32_t C>
__global__ __launch_bounds__(1024) void k_grid_bwd_sliced_simple(
    const grad_t *__restrict__ grad, const float *__restrict__ inputs,
    const int32_t *__restrict__ offsets, float *__restrict__ partial, uint32_t B, uint32_t L,
    Levels lv, uint32_t gridtype, int align_corners, uint32_t rows_per_slice,
    uint32_t total_rows, int vec_ok, SliceDyn dyn) {
    (void)vec_ok;
    extern __shared__ double acc[];
    const uint32_t r0 = blockIdx.x * rows_per_slice;
    const uint32_t r1 = min(r0 + rows_per_slice, total_rows);
    const uint32_t n = (r1 - r0) * C;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) acc[i] = 0.0;
    __syncthreads();
    const bool align = align_corners != 0;
    const uint32_t M = dyn_count(dyn, B);
    const uint32_t chunk = ceil_div(M, gridDim.y);
    const uint32_t b0 = blockIdx.y * chunk;
    const uint32_t b1 = min(M, b0 + chunk);
    for (uint32_t l = 0; l < L; ++l) {
        const LevelCtx c = level_ctx<D>(offsets, lv, l, gridtype, align);
        if (c.base >= r1 || c.base + c.hsize <= r0) continue;
        const grad_t *gl = grad + (size_t)l * B * C;
        const uint32_t lead = (!c.hashed) ? c.used : D;
        for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
            float x[D];
            bool oob = false;
#pragma unroll
            for (uint32_t d = 0; d < D; ++d) {
                x[d] = dyn_map(dyn, inputs[(size_t)b * D + d]);
                oob |= (x[d] < 0.0f) || (x[d] > 1.0f);
            }
            if (oob) continue;
            float frac[D], cw[1u << D][C], g[C];
            uint32_t cell[D];
#pragma unroll
            for (uint32_t d = 0; d < D; ++d) {
                const float p = fmaf(x[d], c.scale, align ? 0.0f : 0.5f);
                cell[d] = (uint32_t)floorf(p);
                frac[d] = p - (float)cell[d];
            }
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) g[ch] = (float)gl[(size_t)b * C + ch];
            float tw = 1.0f;
#pragma unroll
            for (uint32_t d = 0; d < D; ++d)
                if (d >= lead) tw *= (1.0f - frac[d]) + frac[d];
#pragma unroll
            for (uint32_t k = 0; k < (1u << D); ++k) {
                float w = tw;
#pragma unroll
                for (uint32_t d = 0; d < D; ++d)
                    if (d < lead) w *= (k & (1u << d)) ? frac[d] : 1.0f - frac[d];
#pragma unroll
                for (uint32_t ch = 0; ch < C; ++ch) cw[k][ch] = w * g[ch];
            }
            flush_cell<D, C>(acc, r0, r1, c, lead, cell, cw);
        }
    }
    __syncthreads();
    float *out = partial + ((size_t)blockIdx.y * total_rows + r0) * C;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) out[i] = (float)acc[i];
}

// Runs of K consecutive samples per lane (the march emits each ray's samples
// contiguously): a run is loaded with 16-B vector loads into registers and
// walked in order; contributions to the same cell are summed in registers
// and flushed to LDS once per cell change.
template <typename grad_t, uint32_t D, uint32_t C, uint32_t K>
__global__ __launch_bounds__(1024) void k_grid_bwd_sliced(
    const grad_t *__restrict__ grad,  // [L, B, C] (reference layout)
    const float *__restrict__ inputs, const int32_t *__restrict__ offsets,
    float *__restrict__ partial,      // [P, total_rows, C]
    uint32_t B, uint32_t L, Levels lv, uint32_t gridtype, int align_corners,
    uint32_t rows_per_slice, uint32_t total_rows, int vec_ok, SliceDyn dyn) {
    constexpr uint32_t GW = (C * sizeof(grad_t) + 3) / 4;  // 32-bit words of one sample's grad
    constexpr bool GPACK = (C * sizeof(grad_t)) % 4 == 0;  // grads tile 32-bit words
    extern __shared__ double acc[];
    const uint32_t r0 = blockIdx.x * rows_per_slice;
    const uint32_t r1 = min(r0 + rows_per_slice, total_rows);
    const uint32_t n = (r1 - r0) * C;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) acc[i] = 0.0;
    __syncthreads();
    const bool align = align_corners != 0;
    // parts split the samples in whole runs, so every run starts 16-B aligned
    const uint32_t M = dyn_count(dyn, B);
    const uint32_t chunk = ceil_div(ceil_div(M, gridDim.y), K) * K;
    const uint32_t b0 = blockIdx.y * chunk;
    const uint32_t b1 = min(M, b0 + chunk);
    const uint32_t runs = b1 > b0 ? ceil_div(b1 - b0, K) : 0u;
    // Interleave runs over lanes: neighbouring lanes walk runs blockDim/64
    // apart, so one LDS atomic instruction rarely has two lanes on one row.
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t waves = blockDim.x >> 6;
    const uint32_t my_run0 = lane * waves + wave;
    for (uint32_t l = 0; l < L; ++l) {
        const LevelCtx c = level_ctx<D>(offsets, lv, l, gridtype, align);
        if (c.base >= r1 || c.base + c.hsize <= r0) continue;  // level not in this slice
        const grad_t *gl = grad + (size_t)l * B * C;
        const uint32_t lead = (!c.hashed) ? c.used : D;
        for (uint32_t run = my_run0; run < runs; run += blockDim.x) {
            const uint32_t s0 = b0 + run * K;
            const uint32_t cnt = min(b1 - s0, K);
            // the whole run's inputs and grads in registers, vector loads
            uint32_t xw[K * D];
            load_run<K, D>(reinterpret_cast<const uint32_t *>(inputs + (size_t)s0 * D), cnt,
                           vec_ok != 0, xw);
            grad_t gv[K * C];
            if constexpr (GPACK) {
                uint32_t gw[K * GW];
                load_run<K, GW>(reinterpret_cast<const uint32_t *>(gl + (size_t)s0 * C), cnt,
                                vec_ok != 0, gw);
                __builtin_memcpy(gv, gw, sizeof(gv));
            } else {
#pragma unroll
                for (uint32_t i = 0; i < K * C; ++i)
                    gv[i] = (i < cnt * C) ? gl[(size_t)s0 * C + i] : (grad_t)0.0f;
            }
            float cw[1u << D][C];
            uint32_t cur[D];
            bool have = false;
#pragma unroll
            for (uint32_t i = 0; i < K; ++i) {
                // guard, not break: a break keeps the loop rolled and forces
                // the run's register arrays into scratch
                if (i < cnt) {
                float x[D];
                bool oob = false;
#pragma unroll
                for (uint32_t d = 0; d < D; ++d) {
                    x[d] = dyn_map(dyn, __uint_as_float(xw[i * D + d]));
                    oob |= (x[d] < 0.0f) || (x[d] > 1.0f);
                }
                if (!oob) {  // else grads stay zero (gridencoder.cu:253-258)
                float frac[D];
                uint32_t cell[D];
#pragma unroll
                for (uint32_t d = 0; d < D; ++d) {
                    const float p = fmaf(x[d], c.scale, align ? 0.0f : 0.5f);
                    cell[d] = (uint32_t)floorf(p);
                    frac[d] = p - (float)cell[d];
                }
                // same rows as the run so far? (only the dims the index uses)
                bool same = have;
#pragma unroll
                for (uint32_t d = 0; d < D; ++d)
                    if (d < lead) same = same && (cell[d] == cur[d]);
                if (!same) {
                    if (have) flush_cell<D, C>(acc, r0, r1, c, lead, cur, cw);
#pragma unroll
                    for (uint32_t k = 0; k < (1u << D); ++k)
#pragma unroll
                        for (uint32_t ch = 0; ch < C; ++ch) cw[k][ch] = 0.0f;
#pragma unroll
                    for (uint32_t d = 0; d < D; ++d) cur[d] = cell[d];
                    have = true;
                }
                float g[C];
#pragma unroll
                for (uint32_t ch = 0; ch < C; ++ch) g[ch] = (float)gv[i * C + ch];
                float tw = 1.0f;
#pragma unroll
                for (uint32_t d = 0; d < D; ++d)
                    if (d >= lead) tw *= (1.0f - frac[d]) + frac[d];
#pragma unroll
                for (uint32_t k = 0; k < (1u << D); ++k) {
                    if (k >> lead) continue;
                    float w = tw;
#pragma unroll
                    for (uint32_t d = 0; d < D; ++d)
                        if (d < lead) w *= (k & (1u << d)) ? frac[d] : 1.0f - frac[d];
#pragma unroll
                    for (uint32_t ch = 0; ch < C; ++ch) cw[k][ch] = fmaf(w, g[ch], cw[k][ch]);
                }
                }  // !oob
                }  // i < cnt
            }
            if (have) flush_cell<D, C>(acc, r0, r1, c, lead, cur, cw);
        }
    }
    __syncthreads();
    float *out = partial + ((size_t)blockIdx.y * total_rows + r0) * C;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) out[i] = (float)acc[i];
}

// Sum the P partial tables (fixed order) into the gradient: overwrite, or add
// into an existing buffer (accumulate != 0, the reference's zero-filled +=).
template <typename out_t>
__global__ __launch_bounds__(256) void k_sum_partials(const float *__restrict__ partial,
                                                      uint32_t P, uint64_t n,
                                                      out_t *__restrict__ out, int accumulate) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        float s = accumulate ? (float)out[i] : 0.0f;
        for (uint32_t p = 0; p < P; ++p) s += partial[(uint64_t)p * n + i];
        out[i] = (out_t)s;
    }
}

constexpr uint32_t kSliceLdsBytes = 160 * 1024;

static uint32_t slice_rows_cap(uint32_t C) {
    // rows of C f64 accumulators that fit the CU's LDS, multiple of 256
    return (kSliceLdsBytes / (8u * C)) & ~255u;
}

// Rows per slice for P parts: the smallest slices that still give one
// workgroup per CU (slices * P <= CUs), capped by the LDS.  Larger slices
// mean fewer redundant walks over the samples; more slices fill the chip.
static uint32_t slice_rows(uint32_t total_rows, uint32_t C, uint32_t parts, uint32_t cus) {
    const uint32_t cap = slice_rows_cap(C);
    const uint32_t want_slices = cus / (parts ? parts : 1u);
    if (want_slices == 0) return cap;
    const uint32_t r = (ceil_div(total_rows, want_slices) + 255u) & ~255u;
    return r < cap ? r : cap;
}

// gridencoder.cu:316-342.  BLC: grad in [B, L*C] (native) else [L, B, C].
template <typename scalar_t, uint32_t D, uint32_t C, bool BLC>
__global__ __launch_bounds__(256) void k_grid_input_bwd(const scalar_t *__restrict__ grad,
                                                        const scalar_t *__restrict__ dy_dx,
                                                        scalar_t *__restrict__ grad_inputs,
                                                        uint32_t B, uint32_t L) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * D) return;
    const uint32_t b = t / D, d = t - b * D;
    const scalar_t *j = dy_dx + (size_t)b * L * D * C;
    scalar_t r = (scalar_t)0.0f;
    for (uint32_t l = 0; l < L; ++l) {
#pragma unroll
        for (uint32_t ch = 0; ch < C; ++ch) {
            const scalar_t a = BLC ? grad[(size_t)b * L * C + (size_t)l * C + ch]
                                   : grad[(size_t)l * B * C + (size_t)b * C + ch];
            const scalar_t m = j[l * D * C + d * C + ch];
            if constexpr (sizeof(scalar_t) == 2) {
                const half_t p = (half_t)f32_rounded((float)a * (float)m);
                r = (half_t)((float)r + (float)p);
            } else {
                r = fma(a, m, r);
            }
        }
    }
    grad_inputs[t] = r;
}

// [B, L] -> [L, B] transposition of one (sample, level) cell of W bytes (the
// native [B, L*C] encoder gradient into the [L, B, C] layout the sliced
// backward walks): a tile of 256 samples is read contiguously into LDS and
// written out level by level, both sides coalesced.
template <typename word_t>
__global__ __launch_bounds__(256) void k_blc_to_lbc(const word_t *__restrict__ src,
                                                   word_t *__restrict__ dst, uint32_t B,
                                                   uint32_t L) {
    extern __shared__ unsigned char tile_raw[];
    word_t *tile = reinterpret_cast<word_t *>(tile_raw);  // [blockDim][L + 1]
    const uint32_t tb = blockDim.x;
    const uint32_t b0 = blockIdx.x * tb;
    const uint32_t nb = min(tb, B - b0);
    const word_t *s = src + (size_t)b0 * L;
    for (uint32_t i = threadIdx.x; i < nb * L; i += tb) {
        const uint32_t b = i / L, l = i - b * L;
        tile[b * (L + 1) + l] = s[i];
    }
    __syncthreads();
    if (threadIdx.x < nb)
        for (uint32_t l = 0; l < L; ++l)
            dst[(size_t)l * B + b0 + threadIdx.x] = tile[threadIdx.x * (L + 1) + l];
}

// ------------------------------------------------------------ dispatch

template <typename scalar_t, uint32_t D, bool BLC>
static void launch_fwd_c(uint32_t C, dim3 g, dim3 blk, hipStream_t s, const float *in,
                         const scalar_t *emb, const int32_t *off, scalar_t *out, uint32_t B,
                         uint32_t L, const Levels &lv, scalar_t *dy, uint32_t gt, int ac,
                         SliceDyn dn) {
    switch (C) {
    case 1: k_grid_fwd<scalar_t, D, 1, BLC><<<g, blk, 0, s>>>(in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    case 2: k_grid_fwd<scalar_t, D, 2, BLC><<<g, blk, 0, s>>>(in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    case 4: k_grid_fwd<scalar_t, D, 4, BLC><<<g, blk, 0, s>>>(in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    case 8: k_grid_fwd<scalar_t, D, 8, BLC><<<g, blk, 0, s>>>(in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    }
}

template <typename scalar_t, bool BLC>
static void launch_fwd(uint32_t D, uint32_t C, dim3 g, dim3 blk, hipStream_t s, const float *in,
                       const scalar_t *emb, const int32_t *off, scalar_t *out, uint32_t B,
                       uint32_t L, const Levels &lv, scalar_t *dy, uint32_t gt, int ac,
                       SliceDyn dn) {
    switch (D) {
    case 1: launch_fwd_c<scalar_t, 1, BLC>(C, g, blk, s, in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    case 2: launch_fwd_c<scalar_t, 2, BLC>(C, g, blk, s, in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    case 3: launch_fwd_c<scalar_t, 3, BLC>(C, g, blk, s, in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    case 4: launch_fwd_c<scalar_t, 4, BLC>(C, g, blk, s, in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    case 5: launch_fwd_c<scalar_t, 5, BLC>(C, g, blk, s, in, emb, off, out, B, L, lv, dy, gt, ac, dn); break;
    }
}

template <typename grad_t, typename acc_t, uint32_t D, bool BLC>
static void launch_bwd_c(uint32_t C, dim3 g, dim3 blk, hipStream_t s, const grad_t *grad,
                         const float *in, const int32_t *off, acc_t *gg, uint32_t B, uint32_t L,
                         const Levels &lv, uint32_t gt, int ac) {
    switch (C) {
    case 1:
        if constexpr (sizeof(acc_t) != 2)
            k_grid_bwd<grad_t, acc_t, D, 1, BLC><<<g, blk, 0, s>>>(grad, in, off, gg, B, L, lv, gt, ac);
        break;
    case 2: k_grid_bwd<grad_t, acc_t, D, 2, BLC><<<g, blk, 0, s>>>(grad, in, off, gg, B, L, lv, gt, ac); break;
    case 4: k_grid_bwd<grad_t, acc_t, D, 4, BLC><<<g, blk, 0, s>>>(grad, in, off, gg, B, L, lv, gt, ac); break;
    case 8: k_grid_bwd<grad_t, acc_t, D, 8, BLC><<<g, blk, 0, s>>>(grad, in, off, gg, B, L, lv, gt, ac); break;
    }
}

template <typename grad_t, typename acc_t, bool BLC>
static void launch_bwd(uint32_t D, uint32_t C, dim3 g, dim3 blk, hipStream_t s, const grad_t *grad,
                       const float *in, const int32_t *off, acc_t *gg, uint32_t B, uint32_t L,
                       const Levels &lv, uint32_t gt, int ac) {
    switch (D) {
    case 1: launch_bwd_c<grad_t, acc_t, 1, BLC>(C, g, blk, s, grad, in, off, gg, B, L, lv, gt, ac); break;
    case 2: launch_bwd_c<grad_t, acc_t, 2, BLC>(C, g, blk, s, grad, in, off, gg, B, L, lv, gt, ac); break;
    case 3: launch_bwd_c<grad_t, acc_t, 3, BLC>(C, g, blk, s, grad, in, off, gg, B, L, lv, gt, ac); break;
    case 4: launch_bwd_c<grad_t, acc_t, 4, BLC>(C, g, blk, s, grad, in, off, gg, B, L, lv, gt, ac); break;
    case 5: launch_bwd_c<grad_t, acc_t, 5, BLC>(C, g, blk, s, grad, in, off, gg, B, L, lv, gt, ac); break;
    }
}

template <typename scalar_t, bool BLC>
static void launch_input_bwd(uint32_t D, uint32_t C, hipStream_t s, const scalar_t *grad,
                             const scalar_t *dy, scalar_t *gi, uint32_t B, uint32_t L) {
    const dim3 g(ceil_div(B * D, 256u)), blk(256);
#define DFHIP_IB(DD)                                                                           \
    switch (C) {                                                                               \
    case 1: k_grid_input_bwd<scalar_t, DD, 1, BLC><<<g, blk, 0, s>>>(grad, dy, gi, B, L); break; \
    case 2: k_grid_input_bwd<scalar_t, DD, 2, BLC><<<g, blk, 0, s>>>(grad, dy, gi, B, L); break; \
    case 4: k_grid_input_bwd<scalar_t, DD, 4, BLC><<<g, blk, 0, s>>>(grad, dy, gi, B, L); break; \
    case 8: k_grid_input_bwd<scalar_t, DD, 8, BLC><<<g, blk, 0, s>>>(grad, dy, gi, B, L); break; \
    }
    switch (D) {
    case 1: DFHIP_IB(1) break;
    case 2: DFHIP_IB(2) break;
    case 3: DFHIP_IB(3) break;
    case 4: DFHIP_IB(4) break;
    case 5: DFHIP_IB(5) break;
    }
#undef DFHIP_IB
}

template <typename grad_t, uint32_t D, uint32_t C>
static void launch_sliced_dc(hipStream_t s, dim3 g, size_t lds, const grad_t *grad,
                             const float *in, const int32_t *off, float *partial, uint32_t B,
                             uint32_t L, const Levels &lv, uint32_t gt, int ac, uint32_t rows,
                             uint32_t total_rows, SliceDyn dyn) {
    // the run-merging kernel for the NeRF grid shape (D=3, C=2), the simple
    // one otherwise
    void (*kern)(const grad_t *, const float *, const int32_t *, float *, uint32_t, uint32_t,
                 Levels, uint32_t, int, uint32_t, uint32_t, int, SliceDyn);
    if constexpr (D == 3 && C == 2)
        kern = k_grid_bwd_sliced<grad_t, D, C, kRunLen>;
    else
        kern = k_grid_bwd_sliced_simple<grad_t, D, C>;
    ensure_dynamic_lds((const void *)kern, (int)kSliceLdsBytes);
    // 16-B vector loads of whole runs: bases aligned and every level's grad
    // plane a multiple of 16 B
    const int vec_ok = (((uintptr_t)grad | (uintptr_t)in) & 15) == 0 &&
                       ((uint64_t)B * C * sizeof(grad_t)) % 16 == 0;
    kern<<<g, 1024, lds, s>>>(grad, in, off, partial, B, L, lv, gt, ac, rows, total_rows, vec_ok,
                              dyn);
}

template <typename grad_t>
static void launch_sliced(uint32_t D, uint32_t C, hipStream_t s, dim3 g, size_t lds,
                          const grad_t *grad, const float *in, const int32_t *off,
                          float *partial, uint32_t B, uint32_t L, const Levels &lv, uint32_t gt,
                          int ac, uint32_t rows, uint32_t total_rows, SliceDyn dyn) {
#define DFHIP_SL(DD, CC)                                                                    \
    launch_sliced_dc<grad_t, DD, CC>(s, g, lds, grad, in, off, partial, B, L, lv, gt, ac, rows, \
                                     total_rows, dyn)
#define DFHIP_SL_C(DD)                       \
    switch (C) {                             \
    case 1: DFHIP_SL(DD, 1); break;          \
    case 2: DFHIP_SL(DD, 2); break;          \
    case 4: DFHIP_SL(DD, 4); break;          \
    case 8: DFHIP_SL(DD, 8); break;          \
    }
    switch (D) {
    case 1: DFHIP_SL_C(1) break;
    case 2: DFHIP_SL_C(2) break;
    case 3: DFHIP_SL_C(3) break;
    case 4: DFHIP_SL_C(4) break;
    case 5: DFHIP_SL_C(5) break;
    }
#undef DFHIP_SL_C
#undef DFHIP_SL
}

static bool check_dc(const char *what, uint32_t D, uint32_t C, uint32_t L) {
    if (D < 1 || D > 5) {  // gridencoder.cu:372
        set_error("%s: GridEncoding: D must be 1, 2, 3, 4, or 5.", what);
        return false;
    }
    if (C != 1 && C != 2 && C != 4 && C != 8) {  // gridencoder.cu:354
        set_error("%s: GridEncoding: C must be 1, 2, 4, or 8.", what);
        return false;
    }
    if (L > kMaxLevels) {
        set_error("%s: at most %u levels supported (got %u)", what, kMaxLevels, L);
        return false;
    }
    return true;
}

}  // namespace ge
}  // namespace dfhip

using namespace dfhip;
using namespace dfhip::ge;

template <bool BLC>
static int grid_fwd_impl(const char *name, int dtype, const float *inputs,
                         const void *embeddings, const int32_t *offsets, void *outputs,
                         uint32_t B, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                         void *dy_dx, uint32_t gridtype, int align_corners,
                         dfhip_stream_t stream, SliceDyn dyn = SliceDyn{nullptr, 0.0f}) {
    if (!check_dc(name, D, C, L)) return DFHIP_EINVAL;
    if (B == 0 || L == 0) return DFHIP_OK;
    // the reference grid's shape under autocast: the tile gather (same bits)
    if (BLC && dtype == DFHIP_F16 && D == 3 && C == 2 && dy_dx == nullptr &&
        grid_forward_tiles_f16(inputs, dyn.bound, embeddings, offsets, L, S, H, gridtype,
                               align_corners, outputs, B, dyn.m_dev, as_stream(stream)))
        return check_launch(name);
    const Levels lv = make_levels(L, S, H);
    const dim3 g(ceil_div(B, 256u)), blk(256);
    DFHIP_DISPATCH(dtype, name,
        launch_fwd<scalar_t, BLC>(D, C, g, blk, as_stream(stream), inputs,
                                  (const scalar_t *)embeddings, offsets, (scalar_t *)outputs, B,
                                  L, lv, (scalar_t *)dy_dx, gridtype, align_corners, dyn));
    return check_launch(name);
}

extern "C" int dfhip_grid_encode_forward(int dtype, const float *inputs, const void *embeddings,
                                         const int32_t *offsets, void *outputs, uint32_t B,
                                         uint32_t D, uint32_t C, uint32_t L, float S,
                                         uint32_t H, void *dy_dx, uint32_t gridtype,
                                         int align_corners, dfhip_stream_t stream) {
    return grid_fwd_impl<false>("grid_encode_forward", dtype, inputs, embeddings, offsets,
                                outputs, B, D, C, L, S, H, dy_dx, gridtype, align_corners,
                                stream);
}

extern "C" int dfhip_grid_encode_forward_blc(int dtype, const float *inputs,
                                             const void *embeddings, const int32_t *offsets,
                                             void *outputs, uint32_t B, uint32_t D, uint32_t C,
                                             uint32_t L, float S, uint32_t H, void *dy_dx,
                                             uint32_t gridtype, int align_corners,
                                             dfhip_stream_t stream) {
    return grid_fwd_impl<true>("grid_encode_forward_blc", dtype, inputs, embeddings, offsets,
                               outputs, B, D, C, L, S, H, dy_dx, gridtype, align_corners,
                               stream);
}

extern "C" int dfhip_grid_encode_forward_dyn(int dtype, const float *inputs, float bound,
                                             const void *embeddings, const int32_t *offsets,
                                             void *outputs, uint32_t B, const int32_t *m_dev,
                                             uint32_t D, uint32_t C, uint32_t L, float S,
                                             uint32_t H, void *dy_dx, uint32_t gridtype,
                                             int align_corners, dfhip_stream_t stream) {
    if (!(bound >= 0.0f)) {
        set_error("grid_encode_forward_dyn: bound must be >= 0");
        return DFHIP_EINVAL;
    }
    return grid_fwd_impl<true>("grid_encode_forward_dyn", dtype, inputs, embeddings, offsets,
                               outputs, B, D, C, L, S, H, dy_dx, gridtype, align_corners, stream,
                               SliceDyn{m_dev, bound});
}

template <bool BLC>
static int grid_bwd_impl(const char *name, int grad_dtype, int acc_dtype, const void *grad,
                         const float *inputs, const int32_t *offsets, void *grad_embeddings,
                         uint32_t B, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                         uint32_t gridtype, int align_corners, dfhip_stream_t stream) {
    if (!check_dc(name, D, C, L)) return DFHIP_EINVAL;
    if (acc_dtype == DFHIP_F16 && (C % 2) != 0) {
        // The reference's half atomicAdd for odd C is an empty stub
        // (gridencoder.cu:22-26); refuse instead of silently dropping grads.
        set_error("%s: f16 accumulation needs an even C (got C=%u)", name, C);
        return DFHIP_EDTYPE;
    }
    if (B == 0 || L == 0) return DFHIP_OK;
    const Levels lv = make_levels(L, S, H);
    const dim3 g(ceil_div(B, 256u)), blk(256);
    hipStream_t s = as_stream(stream);
#define DFHIP_BWD_ACC(GT)                                                                    \
    switch (acc_dtype) {                                                                     \
    case DFHIP_F32: launch_bwd<GT, float, BLC>(D, C, g, blk, s, (const GT *)grad, inputs,     \
                                               offsets, (float *)grad_embeddings, B, L, lv,   \
                                               gridtype, align_corners); break;               \
    case DFHIP_F16: launch_bwd<GT, half_t, BLC>(D, C, g, blk, s, (const GT *)grad, inputs,    \
                                                offsets, (half_t *)grad_embeddings, B, L, lv, \
                                                gridtype, align_corners); break;              \
    case DFHIP_F64: launch_bwd<GT, double, BLC>(D, C, g, blk, s, (const GT *)grad, inputs,    \
                                                offsets, (double *)grad_embeddings, B, L, lv, \
                                                gridtype, align_corners); break;              \
    default: set_error("%s: unsupported accumulation dtype %d", name, acc_dtype);            \
             return DFHIP_EDTYPE;                                                            \
    }
    switch (grad_dtype) {
    case DFHIP_F32: DFHIP_BWD_ACC(float) break;
    case DFHIP_F16: DFHIP_BWD_ACC(half_t) break;
    case DFHIP_F64: DFHIP_BWD_ACC(double) break;
    default: set_error("%s: unsupported grad dtype %d", name, grad_dtype); return DFHIP_EDTYPE;
    }
#undef DFHIP_BWD_ACC
    return check_launch(name);
}

extern "C" int dfhip_grid_encode_backward(int dtype, const void *grad, const float *inputs,
                                          const void *embeddings, const int32_t *offsets,
                                          void *grad_embeddings, uint32_t B, uint32_t D,
                                          uint32_t C, uint32_t L, float S, uint32_t H,
                                          const void *dy_dx, void *grad_inputs,
                                          uint32_t gridtype, int align_corners,
                                          dfhip_stream_t stream) {
    (void)embeddings;  // only its dtype matters (gridencoder.cu:475)
    int rc = grid_bwd_impl<false>("grid_encode_backward", dtype, dtype, grad, inputs, offsets,
                                  grad_embeddings, B, D, C, L, S, H, gridtype, align_corners,
                                  stream);
    if (rc != DFHIP_OK || dy_dx == nullptr || grad_inputs == nullptr || B == 0) return rc;
    DFHIP_DISPATCH(dtype, "grid_encode_backward",
        (launch_input_bwd<scalar_t, false>)(D, C, as_stream(stream), (const scalar_t *)grad,
                                   (const scalar_t *)dy_dx, (scalar_t *)grad_inputs, B, L));
    return check_launch("grid_encode_backward(inputs)");
}

extern "C" int dfhip_grid_encode_backward_blc(int grad_dtype, int acc_dtype, const void *grad,
                                              const float *inputs, const int32_t *offsets,
                                              void *grad_embeddings, uint32_t B, uint32_t D,
                                              uint32_t C, uint32_t L, float S, uint32_t H,
                                              const void *dy_dx, void *grad_inputs,
                                              uint32_t gridtype, int align_corners,
                                              dfhip_stream_t stream) {
    int rc = grid_bwd_impl<true>("grid_encode_backward_blc", grad_dtype, acc_dtype, grad, inputs,
                                 offsets, grad_embeddings, B, D, C, L, S, H, gridtype,
                                 align_corners, stream);
    if (rc != DFHIP_OK || dy_dx == nullptr || grad_inputs == nullptr || B == 0) return rc;
    DFHIP_DISPATCH(grad_dtype, "grid_encode_backward_blc",
        (launch_input_bwd<scalar_t, true>)(D, C, as_stream(stream), (const scalar_t *)grad,
                                           (const scalar_t *)dy_dx, (scalar_t *)grad_inputs, B, L));
    return check_launch("grid_encode_backward_blc(inputs)");
}

extern "C" uint32_t dfhip_grid_backward_default_parts(uint32_t total_rows, uint32_t C) {
    if (C == 0 || total_rows == 0) return 1;
    // several workgroups per CU: one WG per CU (160 KiB LDS) cannot hide the
    // walk's latency, so more, shorter parts win until the partial traffic
    // (2 * parts * table bytes) shows (tools/bench_kernels.py: 1.1 M samples,
    // 2 parts 2.6 ms, 8 parts 1.3 ms, 16 parts 1.16 ms, 24 parts 1.12 ms)
    const uint32_t slices = ceil_div(total_rows, slice_rows_cap(C));
    const uint32_t p = ceil_div(6u * device_cus(), slices);
    return p < 1 ? 1 : (p > 16 ? 16 : p);
}

extern "C" uint64_t dfhip_grid_backward_partial_floats(uint32_t total_rows, uint32_t C,
                                                       uint32_t parts) {
    return (uint64_t)total_rows * C * (parts ? parts : 1);
}

namespace dfhip {
namespace ge {
int grid_backward_sliced(const char *name, int grad_dtype, int out_dtype, const void *grad,
                         const float *inputs, const int32_t *offsets, void *grad_embeddings,
                         uint32_t total_rows, uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                         float S, uint32_t H, uint32_t gridtype, int align_corners,
                         float *partial, uint32_t parts, int accumulate, SliceDyn dyn,
                         hipStream_t s) {
    if (!check_dc(name, D, C, L)) return DFHIP_EINVAL;
    if (parts == 0 || partial == nullptr) {
        set_error("%s: needs parts >= 1 and a partial buffer", name);
        return DFHIP_EINVAL;
    }
    if (out_dtype != DFHIP_F32 && out_dtype != DFHIP_F16) {
        set_error("%s: output dtype must be f32 or f16", name);
        return DFHIP_EDTYPE;
    }
    if (total_rows == 0) return DFHIP_OK;
    const uint64_t n = (uint64_t)total_rows * C;
    if (B > 0 && L > 0) {
        const Levels lv = make_levels(L, S, H);
        const uint32_t rows = slice_rows(total_rows, C, parts, device_cus());
        const dim3 g(ceil_div(total_rows, rows), parts);
        const size_t lds = (size_t)rows * C * sizeof(double);
        switch (grad_dtype) {
        case DFHIP_F32: launch_sliced<float>(D, C, s, g, lds, (const float *)grad, inputs, offsets,
                                             partial, B, L, lv, gridtype, align_corners, rows,
                                             total_rows, dyn); break;
        case DFHIP_F16: launch_sliced<half_t>(D, C, s, g, lds, (const half_t *)grad, inputs,
                                              offsets, partial, B, L, lv, gridtype, align_corners,
                                              rows, total_rows, dyn); break;
        default: set_error("%s: unsupported grad dtype %d", name, grad_dtype); return DFHIP_EDTYPE;
        }
    } else {
        (void)hipMemsetAsync(partial, 0, n * parts * sizeof(float), s);
    }
    const uint64_t want_blocks = ceil_div<uint64_t>(n, 256);
    const uint32_t blocks = (uint32_t)(want_blocks < 4096 ? want_blocks : 4096);
    if (out_dtype == DFHIP_F32)
        k_sum_partials<float><<<blocks, 256, 0, s>>>(partial, parts, n, (float *)grad_embeddings,
                                                     accumulate);
    else
        k_sum_partials<half_t><<<blocks, 256, 0, s>>>(partial, parts, n, (half_t *)grad_embeddings,
                                                      accumulate);
    return check_launch(name);
}
}  // namespace ge
}  // namespace dfhip

extern "C" int dfhip_grid_encode_backward_sliced(int grad_dtype, int out_dtype, const void *grad,
                                                 const float *inputs, const int32_t *offsets,
                                                 void *grad_embeddings, uint32_t total_rows,
                                                 uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                                                 float S, uint32_t H, uint32_t gridtype,
                                                 int align_corners, float *partial,
                                                 uint32_t parts, int accumulate,
                                                 dfhip_stream_t stream) {
    return ge::grid_backward_sliced("grid_encode_backward_sliced", grad_dtype, out_dtype, grad,
                                    inputs, offsets, grad_embeddings, total_rows, B, D, C, L, S,
                                    H, gridtype, align_corners, partial, parts, accumulate,
                                    ge::SliceDyn{nullptr, 0.0f}, as_stream(stream));
}

extern "C" int dfhip_grid_grad_blc_to_lbc(int dtype, const void *src, void *dst, uint32_t B,
                                          uint32_t L, uint32_t C, dfhip_stream_t stream) {
    const char *name = "grid_grad_blc_to_lbc";
    size_t esz = (dtype == DFHIP_F16 || dtype == DFHIP_BF16) ? 2
                 : dtype == DFHIP_F32 ? 4 : dtype == DFHIP_F64 ? 8 : 0;
    if (esz == 0) {
        set_error("%s: unsupported dtype %d", name, dtype);
        return DFHIP_EDTYPE;
    }
    if (L == 0 || L > kMaxLevels || C == 0) {
        set_error("%s: bad L=%u C=%u", name, L, C);
        return DFHIP_EINVAL;
    }
    if (B == 0) return DFHIP_OK;
    const size_t w = esz * C;  // bytes of one (sample, level) cell
    hipStream_t s = as_stream(stream);
    // tile of tb samples x (L + 1) cells in LDS, within 64 KiB
    uint32_t tb = 256;
    while (tb > 64 && (size_t)tb * (L + 1) * w > 64 * 1024) tb /= 2;
    const size_t lds = (size_t)tb * (L + 1) * w;
    if (lds > 64 * 1024) {
        set_error("%s: cell of %zu bytes x %u levels too large", name, w, L);
        return DFHIP_EINVAL;
    }
    const uint32_t blocks = ceil_div(B, tb);
    switch (w) {
    case 2: k_blc_to_lbc<uint16_t><<<blocks, tb, lds, s>>>((const uint16_t *)src, (uint16_t *)dst, B, L); break;
    case 4: k_blc_to_lbc<uint32_t><<<blocks, tb, lds, s>>>((const uint32_t *)src, (uint32_t *)dst, B, L); break;
    case 8: k_blc_to_lbc<uint2><<<blocks, tb, lds, s>>>((const uint2 *)src, (uint2 *)dst, B, L); break;
    case 16: k_blc_to_lbc<uint4><<<blocks, tb, lds, s>>>((const uint4 *)src, (uint4 *)dst, B, L); break;
    default:
        set_error("%s: cell of %zu bytes unsupported (C * dtype size must be 2, 4, 8 or 16)", name, w);
        return DFHIP_EINVAL;
    }
    return check_launch(name);
}

extern "C" int dfhip_grid_encode_backward_sliced_dyn(
    int grad_dtype, int out_dtype, const void *grad, const float *inputs, float bound,
    const int32_t *offsets, void *grad_embeddings, uint32_t total_rows, uint32_t B,
    const int32_t *m_dev, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
    uint32_t gridtype, int align_corners, float *partial, uint32_t parts, int accumulate,
    dfhip_stream_t stream) {
    if (bound < 0.0f) {
        set_error("grid_encode_backward_sliced_dyn: bound must be >= 0");
        return DFHIP_EINVAL;
    }
    return ge::grid_backward_sliced("grid_encode_backward_sliced_dyn", grad_dtype, out_dtype, grad,
                                    inputs, offsets, grad_embeddings, total_rows, B, D, C, L, S,
                                    H, gridtype, align_corners, partial, parts, accumulate,
                                    ge::SliceDyn{m_dev, bound}, as_stream(stream));
}
