// Grid-encoder level geometry and corner arithmetic shared by the grid
// kernels (gridencoder.hip) and the fused field kernels (fieldmlp.hip).
// Behavioural spec: reference gridencoder/src/gridencoder.cu:35-72,125-165.
#pragma once

#include <math.h>

#include <cmath>

#include "common.h"

namespace dfhip {
namespace ge {

constexpr uint32_t kMaxLevels = 64;

struct Levels {
    float scale[kMaxLevels];
    uint32_t res[kMaxLevels];
};

// gridencoder.cu:125-126, evaluated on the host.
static Levels make_levels(uint32_t L, float S, uint32_t H) {
    Levels lv;
    for (uint32_t l = 0; l < L; ++l) {
        const float ls = (float)l * S;
        const float e = (float)exp2((double)ls);
        const float scale = fmaf(e, (float)H, -1.0f);
        lv.scale[l] = scale;
        lv.res[l] = (uint32_t)ceilf(scale) + 1u;
    }
    return lv;
}

// gridencoder.cu:35-51 — instant-ngp spatial hash.
template <uint32_t D>
__device__ __forceinline__ uint32_t spatial_hash(const uint32_t p[D]) {
    constexpr uint32_t kPrimes[7] = {1u, 2654435761u, 805459861u, 3674653429u,
                                     2097192037u, 1434869437u, 2165219737u};
    uint32_t h = 0;
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) h ^= p[d] * kPrimes[d];
    return h;
}

// Wave-uniform per-level context.
struct LevelCtx {
    uint32_t base;     // first table row of the level (offsets[l])
    uint32_t hsize;    // rows in the level
    uint32_t smul;     // stride multiplier: res (align_corners) or res + 1
    uint32_t used;     // dims consumed by the tiled index before stride > hsize
    bool hashed;       // gridtype == hash and stride overflowed -> spatial_hash
    bool pow2;         // hsize is a power of two -> modulo is a mask
    float scale;
};

template <uint32_t D>
__device__ __forceinline__ LevelCtx level_ctx(const int32_t *__restrict__ offsets,
                                              const Levels &lv, uint32_t l,
                                              uint32_t gridtype, bool align) {
    LevelCtx c;
    c.base = (uint32_t)offsets[l];
    c.hsize = (uint32_t)offsets[l + 1] - c.base;
    c.scale = lv.scale[l];
    c.smul = align ? lv.res[l] : lv.res[l] + 1u;
    // gridencoder.cu:56-63: for (d < D && stride <= hashmap_size)
    uint32_t stride = 1, used = 0;
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        if (stride <= c.hsize) { stride *= c.smul; ++used; }
    }
    c.used = used;
    c.hashed = (gridtype == 0) && (stride > c.hsize);
    c.pow2 = (c.hsize & (c.hsize - 1)) == 0;
    return c;
}

// gridencoder.cu:54-72 (row index; the caller multiplies by C).
template <uint32_t D>
__device__ __forceinline__ uint32_t row_index(const LevelCtx &c, const uint32_t p[D]) {
    uint32_t idx;
    if (c.hashed) {
        idx = spatial_hash<D>(p);
    } else {
        idx = 0;
        uint32_t stride = 1;
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) {
            if (d < c.used) { idx += p[d] * stride; stride *= c.smul; }
        }
    }
    return c.pow2 ? (idx & (c.hsize - 1)) : (idx % c.hsize);
}

// Corner rows of one level without the generic per-corner index loop and
// modulo (same u32 arithmetic as row_index): the tiled index of cell + corner
// offset o_k is i0 + o_k with i0 = c0 + c1 m1 + c2 m2 (m1 / m2 zero for the
// dimensions the tiled index stops before), wrapped by a mask when the level
// is a power of two or the index can never reach hsize, else by % hsize; the
// hashed form keeps the spatial hash.  Per-level constants are uniform.
struct LevelRows {
    uint32_t hsize, wmask, m1, m2, lead;
    bool hashed, modulo;
};

template <uint32_t D>
__device__ __forceinline__ LevelRows level_rows(const LevelCtx &c) {
    LevelRows r;
    r.hsize = c.hsize;
    r.hashed = c.hashed;
    r.lead = c.hashed ? D : c.used;
    r.m1 = (D > 1 && r.lead > 1) ? c.smul : 0u;
    r.m2 = (D > 2 && r.lead > 2) ? c.smul * c.smul : 0u;
    uint64_t span = 1;  // largest tiled index + 1
    for (uint32_t d = 0; d < c.used; ++d) span *= c.smul;
    r.modulo = !c.pow2 && (c.hashed || span > (uint64_t)c.hsize);
    r.wmask = c.pow2 ? c.hsize - 1u : 0xFFFFFFFFu;
    return r;
}

// Row (relative to the level base) of corner k (bit d = +1 along d < lead).
// MODE fixes the wrap at compile time (0: mask, 1: % hsize, 2: hash, then
// mask or % by r.modulo); callers branch once per level on row_mode(r), a
// uniform value, instead of evaluating every form per corner and selecting.
template <uint32_t D, int MODE>
__device__ __forceinline__ uint32_t corner_row_m(const LevelRows &r, const uint32_t cell[D],
                                                 uint32_t k) {
    uint32_t idx;
    if (MODE == 2) {
        uint32_t p[D];
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) p[d] = cell[d] + ((k >> d) & 1u);
        idx = spatial_hash<D>(p);
        return r.modulo ? idx % r.hsize : (idx & r.wmask);
    }
    idx = cell[0] + (k & 1u);
    if (D > 1) idx += (cell[1] + ((k >> 1) & 1u)) * r.m1;
    if (D > 2) idx += (cell[D > 2 ? 2 : 0] + ((k >> 2) & 1u)) * r.m2;
    return MODE == 1 ? idx % r.hsize : (idx & r.wmask);
}

__device__ __forceinline__ int row_mode(const LevelRows &r) {
    return r.hashed ? 2 : (r.modulo ? 1 : 0);
}

template <uint32_t D>
__device__ __forceinline__ uint32_t corner_row(const LevelRows &r, const uint32_t cell[D],
                                               uint32_t k) {
    uint32_t idx;
    if (r.hashed) {
        uint32_t p[D];
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) p[d] = cell[d] + ((k >> d) & 1u);
        idx = spatial_hash<D>(p);
    } else {
        idx = cell[0] + (k & 1u);
        if (D > 1) idx += (cell[1] + ((k >> 1) & 1u)) * r.m1;
        if (D > 2) idx += (cell[D > 2 ? 2 : 0] + ((k >> 2) & 1u)) * r.m2;
    }
    return r.modulo ? idx % r.hsize : (idx & r.wmask);
}

// ------------------------------------------------------------ storage helpers
// Accumulate one corner contribution into a per-channel register, following
// the reference's scalar_t arithmetic exactly (gridencoder.cu:142,165).
__device__ __forceinline__ void acc_corner(float &r, float w, float g) { r = fmaf(w, g, r); }
__device__ __forceinline__ void acc_corner(double &r, float w, double g) {
    r = fma((double)w, g, r);
}
__device__ __forceinline__ void acc_corner(half_t &r, float w, half_t g) {
    // c10::Half: Half += float  ==>  Half(float(r) + float(Half(w * float(g))))
    const half_t p = (half_t)f32_rounded(w * (float)g);
    r = (half_t)((float)r + (float)p);
}

// Dynamic sample count / coordinate mapping of the sliced embedding backward
// (see gridencoder.hip k_grid_bwd_sliced).
struct SliceDyn {
    const int32_t *m_dev;
    float bound;
};

// Dynamic sample count / coordinate mapping of the fused field path: when
// m_dev is set, only samples [0, *m_dev) of the B-row planes are walked (B is
// then the plane stride, the capacity); when bound > 0 the inputs are raw
// positions in [-bound, bound], mapped to [0, 1] as grid.py:142 does.
__device__ __forceinline__ uint32_t dyn_count(const SliceDyn &dyn, uint32_t B) {
    if (!dyn.m_dev) return B;
    const int32_t m = *dyn.m_dev;
    return m < 0 ? 0u : ((uint32_t)m < B ? (uint32_t)m : B);
}

__device__ __forceinline__ float dyn_map(const SliceDyn &dyn, float x) {
    return dyn.bound > 0.0f ? (x + dyn.bound) / (2.0f * dyn.bound) : x;
}

// dyn_map for a kernel instantiated knowing that 2 * bound is a power of two
// (bound 1, the reference default): the quotient is the product with the
// exact reciprocal `inv`, bit for bit, without the correctly-rounded division.
inline bool dyn_pow2(float bound) {
    if (!(bound > 0.0f)) return false;
    const float d = 2.0f * bound;
    int e = 0;
    return std::frexp(d, &e) == 0.5f && d > 1.0e-30f && d < 1.0e30f;
}
template <bool POW2>
__device__ __forceinline__ float dyn_map_t(const SliceDyn &dyn, float inv, float x) {
    if constexpr (POW2) return (x + dyn.bound) * inv;
    return dyn_map(dyn, x);
}

// Host side of dfhip_grid_encode_backward_sliced, shared with the fused
// field backward (fieldmlp.hip).
int grid_backward_sliced(const char *name, int grad_dtype, int out_dtype, const void *grad,
                         const float *inputs, const int32_t *offsets, void *grad_embeddings,
                         uint32_t total_rows, uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                         float S, uint32_t H, uint32_t gridtype, int align_corners,
                         float *partial, uint32_t parts, int accumulate, SliceDyn dyn,
                         hipStream_t s);

}  // namespace ge
}  // namespace dfhip
