// Binned owner-computes embedding backward of the tiled / hashed grid encoder
// (reference gridencoder/src/gridencoder.cu:226-313 kernel_grid_backward,
// restructured for gfx950).
//
// The LDS-sliced backward (gridencoder.hip k_grid_bwd_sliced) lets every
// slice walk every sample of its level: a 2^16-row level cut into 7-8 slices
// re-reads and re-derives each sample's corners 7-8 times, although a sample's
// corners touch only 1-3 of them.  Here the (sample, level) pairs are first
// binned by the slices their corners touch, so every walk is useful:
//
//   1. k_bin: per tile of kTile consecutive samples (one workgroup), every
//      in-bounds sample derives, level by level, the slices of its 2^D corner
//      rows and appends its tile-relative id (u16) to the (tile, slice)
//      segment (LDS counters give the slot; segments hold kTile ids, so no
//      scan is needed).
//   2. k_walk: workgroup (slice, part) zeroes the slice's f64 accumulators in
//      LDS, walks the segments of its part's tiles (one wave per segment,
//      gathering the sample's position and feature gradient), adds the
//      contributions of the corners inside the slice with ds_add_f64, and
//      writes the slice to its partial buffer (f32, plain coalesced stores).
//   3. k_sum: every table row sums its slice's partials in a fixed order.
//
// Slices are 2^shift rows of one level (8192 rows x 2 channels x f64 =
// 128 KiB of LDS).  The walk is XCD-aware: the tiles are cut into 8
// contiguous ranges, one per XCD, and every slice gets workgroups on every
// XCD, so a sample's position and gradient are only ever read through one
// XCD's L2.  Levels with fewer slices get more workgroups per slice, so every
// level gets about the same number of workgroups.
// Products w * g are formed in f64 (exact) and summed in f64; the result is
// the f64 sum rounded to f32 once.  Deterministic up to the f64 summation
// order of the LDS atomics.
#include "grid_common.h"

#include <type_traits>

namespace dfhip {
namespace gb {

using ge::Levels;
using ge::LevelCtx;
using ge::SliceDyn;

constexpr uint32_t kTile = 1024;     // samples per binning tile (ids per segment)
constexpr uint32_t kMaxBins = 1024;
constexpr uint32_t kLdsBytes = 160 * 1024;

constexpr uint32_t kXcds = 8;  // MI355X: 8 XCDs, workgroup i dispatched to XCD i % 8

struct BinInfo {
    uint32_t L, nbins, shift, nslots;
    uint32_t bin0[ge::kMaxLevels + 1];   // first bin of level l (bin0[L] = nbins)
    uint32_t parts[ge::kMaxLevels];      // walk workgroups per slice of level l (kXcds * q)
    uint32_t q[ge::kMaxLevels];          // ... of which on one XCD
    uint32_t slot0[ge::kMaxLevels + 1];  // first per-XCD work slot of level l
    uint32_t base[ge::kMaxLevels];       // first row of level l
    uint32_t rows[ge::kMaxLevels];       // rows of level l
    uint64_t pbase[ge::kMaxLevels];      // first partial float of level l
};

static uint32_t slice_shift(uint32_t C) {
    uint32_t shift = 0;
    while ((2ull << shift) * 8ull * C <= kLdsBytes) ++shift;
    return shift;  // largest 2^shift rows with 2^shift * C doubles <= LDS
}

// Host: bins / parts / partial layout from the HOST copy of the offsets.
static bool make_bins(const int32_t *offsets_host, uint32_t L, uint32_t C, uint32_t cus,
                      BinInfo &bi) {
    if (L == 0 || L > ge::kMaxLevels) return false;
    bi.L = L;
    bi.shift = slice_shift(C);
    uint32_t nb = 0, maxslices = 1;
    for (uint32_t l = 0; l < L; ++l) {
        const uint32_t rows = (uint32_t)(offsets_host[l + 1] - offsets_host[l]);
        const uint32_t ns = rows ? ((rows - 1) >> bi.shift) + 1 : 0;
        if (ns > 64) return false;  // slice masks are 64-bit
        bi.bin0[l] = nb;
        bi.base[l] = (uint32_t)offsets_host[l];
        bi.rows[l] = rows;
        nb += ns;
        if (ns > maxslices) maxslices = ns;
    }
    bi.bin0[L] = nb;
    bi.nbins = nb;
    if (nb == 0 || nb > kMaxBins) return false;
    // XCD-aware walk: XCD x owns the x-th contiguous eighth of the tiles, so
    // each sample's position / gradient is read by the workgroups of one XCD
    // only (its L2).  Per XCD, each slice of level l gets q_l workgroups, q_l
    // chosen so that every level gets about 4 * CUs / L workgroups in total
    // (2 * CUs / L left the coarse levels' long walks as the tail: +4 %).
    const uint32_t per_level = (4u * cus + L - 1) / L;
    (void)maxslices;
    uint64_t pf = 0;
    uint32_t slots = 0;
    for (uint32_t l = 0; l < L; ++l) {
        const uint32_t ns = bi.bin0[l + 1] - bi.bin0[l];
        uint32_t q = ns ? per_level / (kXcds * ns) : 1;
        if (q < 1) q = 1;
        if (q > 16) q = 16;
        bi.q[l] = q;
        bi.parts[l] = kXcds * q;
        bi.slot0[l] = slots;
        slots += ns * q;
        bi.pbase[l] = pf;
        pf += (uint64_t)ns * bi.parts[l] * (1ull << bi.shift) * C;
    }
    bi.slot0[L] = slots;
    bi.nslots = slots;
    return true;
}

static uint64_t partial_floats(const BinInfo &bi, uint32_t C) {
    const uint32_t l = bi.L - 1;
    return bi.pbase[l] + (uint64_t)(bi.bin0[l + 1] - bi.bin0[l]) * bi.parts[l] *
                             (1ull << bi.shift) * C;
}

// Cell and fractional position of x at level c (gridencoder.cu:146-154).
template <uint32_t D>
__device__ __forceinline__ void locate(const LevelCtx &c, bool align, const float x[D],
                                       uint32_t cell[D], float frac[D]) {
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        const float p = fmaf(x[d], c.scale, align ? 0.0f : 0.5f);
        cell[d] = (uint32_t)floorf(p);
        frac[d] = p - (float)cell[d];
    }
}

template <uint32_t D, bool POW2>
__device__ __forceinline__ bool load_pos(const float *__restrict__ inputs, const SliceDyn &dyn,
                                         float inv, uint32_t s, float x[D]) {
    bool oob = false;
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        x[d] = ge::dyn_map_t<POW2>(dyn, inv, inputs[(size_t)s * D + d]);
        oob |= (x[d] < 0.0f) || (x[d] > 1.0f);
    }
    return !oob;  // out-of-bounds samples contribute nothing (gridencoder.cu:253-258)
}

// Slices (bits) touched by the corners of a cell at one level.
template <uint32_t D, int MODE>
__device__ __forceinline__ uint64_t slice_mask(const ge::LevelRows &lr, const uint32_t cell[D],
                                               uint32_t shift) {
    uint64_t mask = 0;
#pragma unroll
    for (uint32_t k = 0; k < (1u << D); ++k) {
        if (k >> lr.lead) continue;
        mask |= 1ull << (ge::corner_row_m<D, MODE>(lr, cell, k) >> shift);
    }
    return mask;
}

// ---------------------------------------------------------------- 1. binning
template <uint32_t D, bool POW2>
__global__ __launch_bounds__(1024) void k_bin(const float *__restrict__ inputs,
                                             const int32_t *__restrict__ offsets, Levels lv,
                                             BinInfo bi, uint32_t gridtype, int align_corners,
                                             SliceDyn dyn, float inv, uint32_t B,
                                             uint32_t *__restrict__ counts,
                                             uint16_t *__restrict__ entries) {
    __shared__ uint32_t cnt[kMaxBins];
    const bool align = align_corners != 0;
    const uint32_t M = ge::dyn_count(dyn, B);
    const uint32_t ntiles = ceil_div(M, kTile);
    const uint32_t nb = bi.nbins;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) cnt[b] = 0;
        __syncthreads();
        uint16_t *seg = entries + (size_t)tile * nb * kTile;
        const uint32_t s_end = min(M, (tile + 1) * kTile);
        for (uint32_t s = tile * kTile + threadIdx.x; s < s_end; s += blockDim.x) {
            float x[D];
            if (!load_pos<D, POW2>(inputs, dyn, inv, s, x)) continue;
            for (uint32_t l = 0; l < bi.L; ++l) {
                const LevelCtx c = ge::level_ctx<D>(offsets, lv, l, gridtype, align);
                const ge::LevelRows lr = ge::level_rows<D>(c);
                uint32_t cell[D];
                float frac[D];
                locate<D>(c, align, x, cell, frac);
                uint64_t mask = 0;
                const int mode = ge::row_mode(lr);
                if (mode == 0) mask = slice_mask<D, 0>(lr, cell, bi.shift);
                else if (mode == 1) mask = slice_mask<D, 1>(lr, cell, bi.shift);
                else mask = slice_mask<D, 2>(lr, cell, bi.shift);
                const uint32_t b0 = bi.bin0[l];
                while (mask) {
                    const uint32_t k = (uint32_t)__builtin_ctzll(mask);
                    mask &= mask - 1;
                    const uint32_t b = b0 + k;
                    const uint32_t slot = atomicAdd(&cnt[b], 1u);
                    seg[(size_t)b * kTile + slot] = (uint16_t)(s - tile * kTile);
                }
            }
        }
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) counts[(size_t)tile * nb + b] = cnt[b];
        __syncthreads();
    }
}

// ---------------------------------------------------------------- 2. walk
// Flush one cell's merged corner contributions into the LDS slice [r0, r1).
template <uint32_t D, uint32_t C, int MODE>
__device__ __forceinline__ void flush_m(double *acc, uint32_t r0, uint32_t r1, const LevelCtx &c,
                                        const ge::LevelRows &lr, const uint32_t cell[D],
                                        const double (&cw)[1u << D][C]);

template <uint32_t D, uint32_t C>
__device__ __forceinline__ void flush(double *acc, uint32_t r0, uint32_t r1, const LevelCtx &c,
                                      const ge::LevelRows &lr, const uint32_t cell[D],
                                      const double (&cw)[1u << D][C]) {
    const int mode = ge::row_mode(lr);  // uniform: one scalar branch per flush
    if (mode == 0) flush_m<D, C, 0>(acc, r0, r1, c, lr, cell, cw);
    else if (mode == 1) flush_m<D, C, 1>(acc, r0, r1, c, lr, cell, cw);
    else flush_m<D, C, 2>(acc, r0, r1, c, lr, cell, cw);
}

template <uint32_t D, uint32_t C, int MODE>
__device__ __forceinline__ void flush_m(double *acc, uint32_t r0, uint32_t r1, const LevelCtx &c,
                                        const ge::LevelRows &lr, const uint32_t cell[D],
                                        const double (&cw)[1u << D][C]) {
#pragma unroll
    for (uint32_t k = 0; k < (1u << D); ++k) {
        if (k >> lr.lead) continue;
        const uint32_t row = c.base + ge::corner_row_m<D, MODE>(lr, cell, k);
        if (row >= r0 && row < r1) {
            double *dst = acc + (size_t)(row - r0) * C;
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) atomicAdd(dst + ch, cw[k][ch]);
        }
    }
}

constexpr uint32_t kRun = 8;  // entries gathered per lane before they are walked

// One sample's position as one 12-byte load (global_load_dwordx3) for D = 3:
// one L1 line lookup per lane instead of three.
typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
template <uint32_t D>
__device__ __forceinline__ void load_pos3(const float *__restrict__ inputs, uint32_t s,
                                          float (&x)[D]) {
    if constexpr (D == 3) {
        const f3u v = *reinterpret_cast<const f3u *>(inputs + (size_t)s * 3);
        x[0] = v.x;
        x[1] = v.y;
        x[2] = v.z;
    } else {
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) x[d] = inputs[(size_t)s * D + d];
    }
}

// One sample's C gradient channels as one load where the row is 4 or 8 bytes.
template <typename grad_t, uint32_t C>
__device__ __forceinline__ void load_grad(const grad_t *__restrict__ p, float (&g)[C]) {
    if constexpr (sizeof(grad_t) * C == 4 && sizeof(grad_t) == 2) {
        typedef grad_t v2 __attribute__((ext_vector_type(2)));
        const v2 v = *reinterpret_cast<const v2 *>(p);
        g[0] = (float)v.x;
        g[C - 1] = (float)v.y;
    } else if constexpr (sizeof(grad_t) * C == 8 && sizeof(grad_t) == 4) {
        const float2 v = *reinterpret_cast<const float2 *>(p);
        g[0] = v.x;
        g[C - 1] = v.y;
    } else {
#pragma unroll
        for (uint32_t ch = 0; ch < C; ++ch) g[ch] = (float)p[ch];
    }
}

// A segment's entries are (in chunks) in sample order, i.e. consecutive
// samples of one ray.  Lane i walks the contiguous run [i*Q, (i+1)*Q) of the
// segment (Q = ceil(cnt / 64)): neighbouring lanes sit Q samples apart, so one
// LDS atomic instruction rarely has two lanes on a row, and along its run a
// lane merges consecutive contributions to the same cell in registers (at the
// coarse levels a cell spans tens of samples of a ray).
template <typename grad_t, uint32_t D, uint32_t C, bool POW2>
__global__ __launch_bounds__(1024) void k_walk(const grad_t *__restrict__ grad,  // [L, B, C]
                                               const float *__restrict__ inputs,
                                               const int32_t *__restrict__ offsets, Levels lv,
                                               BinInfo bi, uint32_t gridtype, int align_corners,
                                               SliceDyn dyn, float inv, uint32_t B,
                                               const uint32_t *__restrict__ counts,
                                               const uint16_t *__restrict__ entries,
                                               float *__restrict__ partial) {
    extern __shared__ double acc[];
    // workgroup -> (XCD x, slot) -> (level, slice k, sub-part q)
    const uint32_t x = blockIdx.x % kXcds, slot = blockIdx.x / kXcds;
    uint32_t l = 0;
    while (l + 1 < bi.L && bi.slot0[l + 1] <= slot) ++l;
    const uint32_t Q = bi.q[l];
    const uint32_t k = (slot - bi.slot0[l]) / Q, q = (slot - bi.slot0[l]) - k * Q;
    const uint32_t b = bi.bin0[l] + k;
    const uint32_t P = bi.parts[l];
    const uint32_t part = x * Q + q;
    const uint32_t srows = 1u << bi.shift;
    const uint32_t r0 = bi.base[l] + (k << bi.shift);
    const uint32_t r1 = min(r0 + srows, bi.base[l] + bi.rows[l]);
    const uint32_t n = (r1 - r0) * C;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) acc[i] = 0.0;
    __syncthreads();
    const bool align = align_corners != 0;
    const LevelCtx c = ge::level_ctx<D>(offsets, lv, l, gridtype, align);
    const ge::LevelRows lr = ge::level_rows<D>(c);
    const uint32_t lead = lr.lead;
    const uint32_t M = ge::dyn_count(dyn, B);
    const uint32_t ntiles = ceil_div(M, kTile);
    const uint32_t nb = bi.nbins;
    const grad_t *gl = grad + (size_t)l * B * C;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
    // XCD x: tiles [t0, t1); sub-part q: t0 + q, t0 + q + Q, ...; wave w takes
    // every waves-th of those
    const uint32_t t0 = (uint32_t)(((uint64_t)ntiles * x) / kXcds);
    const uint32_t t1 = (uint32_t)(((uint64_t)ntiles * (x + 1)) / kXcds);
    for (uint32_t t = t0 + q + Q * wave; t < t1; t += Q * waves) {
        const uint32_t cnt = counts[(size_t)t * nb + b];
        const uint16_t *seg = entries + ((size_t)t * nb + b) * kTile;
        const uint32_t tbase = t * kTile;
        const uint32_t Q = (cnt + 63) >> 6;
        const uint32_t e0 = min(lane * Q, cnt), e1 = min(e0 + Q, cnt);
        double cw[1u << D][C];
        uint32_t cur[D];
        bool have = false;
        // a lane walks a run of Q entries in batches of RUN loads; segments
        // with Q == 1 (the fine levels) take single-entry batches instead of
        // eight clamped duplicate loads per entry
        auto walk = [&](auto run_c) {
            constexpr uint32_t RUN = decltype(run_c)::value;
            for (uint32_t e = e0; e < e1; e += RUN) {
                const uint32_t m = min(e1 - e, RUN);
                // every load of the batch is issued before the first use: clamped
                // indices instead of guarded loads (a guarded load is a branch
                // with its own wait)
                uint32_t sid[RUN];
                float xs[RUN][D];
                float gs[RUN][C];
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) sid[i] = tbase + seg[min(e + i, e1 - 1)];
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) {
                    load_pos3<D>(inputs, sid[i], xs[i]);
                    load_grad<grad_t, C>(gl + (size_t)sid[i] * C, gs[i]);
                }
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) {
                    if (i < m) {  // guard, not break: keeps the run in registers
                        float x[D];
#pragma unroll
                        for (uint32_t d = 0; d < D; ++d) x[d] = ge::dyn_map_t<POW2>(dyn, inv, xs[i][d]);
                        uint32_t cell[D];
                        float frac[D];
                        locate<D>(c, align, x, cell, frac);
                        bool same = have;
#pragma unroll
                        for (uint32_t d = 0; d < D; ++d)
                            if (d < lead) same = same && (cell[d] == cur[d]);
                        if (!same) {
                            if (have) flush<D, C>(acc, r0, r1, c, lr, cur, cw);
#pragma unroll
                            for (uint32_t kc = 0; kc < (1u << D); ++kc)
#pragma unroll
                                for (uint32_t ch = 0; ch < C; ++ch) cw[kc][ch] = 0.0;
#pragma unroll
                            for (uint32_t d = 0; d < D; ++d) cur[d] = cell[d];
                            have = true;
                        }
                        float tw = 1.0f;  // trailing dims dropped from the index: corners coincide
#pragma unroll
                        for (uint32_t d = 0; d < D; ++d)
                            if (d >= lead) tw *= (1.0f - frac[d]) + frac[d];
#pragma unroll
                        for (uint32_t kc = 0; kc < (1u << D); ++kc) {
                            if (kc >> lead) continue;
                            float w = tw;
#pragma unroll
                            for (uint32_t d = 0; d < D; ++d)
                                if (d < lead) w *= (kc & (1u << d)) ? frac[d] : 1.0f - frac[d];
#pragma unroll
                            for (uint32_t ch = 0; ch < C; ++ch)
                                cw[kc][ch] = fma((double)w, (double)gs[i][ch], cw[kc][ch]);
                        }
                    }
                }
            }
        };
        if (Q <= 1)
            walk(std::integral_constant<uint32_t, 1>{});
        else
            walk(std::integral_constant<uint32_t, kRun>{});
        if (have) flush<D, C>(acc, r0, r1, c, lr, cur, cw);
    }
    __syncthreads();
    float *out = partial + bi.pbase[l] + ((size_t)k * P + part) * ((size_t)srows * C);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) out[i] = (float)acc[i];
}

// ---------------------------------------------------------------- 3. sum
template <typename out_t>
__global__ __launch_bounds__(256) void k_sum(const float *__restrict__ partial, BinInfo bi,
                                             uint32_t C, uint32_t total_rows,
                                             out_t *__restrict__ out, int accumulate) {
    const uint64_t n = (uint64_t)total_rows * C;
    const uint32_t srows = 1u << bi.shift;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t row = (uint32_t)(i / C), ch = (uint32_t)(i - (uint64_t)row * C);
        uint32_t l = 0;
        while (l + 1 < bi.L && bi.base[l + 1] <= row) ++l;
        const uint32_t rel = row - bi.base[l];
        const uint32_t k = rel >> bi.shift, off = rel & (srows - 1);
        const uint32_t P = bi.parts[l];
        const float *src = partial + bi.pbase[l] + (size_t)k * P * srows * C + (size_t)off * C + ch;
        float s = accumulate ? (float)out[i] : 0.0f;
        double t = 0.0;
        uint32_t p = 0;
        for (; p + 4 <= P; p += 4) {  // parts added in order, four loads in flight
            float x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = src[(size_t)(p + u) * srows * C];
#pragma unroll
            for (int u = 0; u < 4; ++u) t += (double)x[u];
        }
        for (; p < P; ++p) t += (double)src[(size_t)p * srows * C];
        out[i] = (out_t)(s + (float)t);
    }
}

static uint32_t device_cus() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            v > 0)
            cus = v;
        else
            cus = 256;
    }
    return (uint32_t)cus;
}

template <typename grad_t, uint32_t C>
static void launch_walk(hipStream_t s, dim3 g, size_t lds, const grad_t *grad,
                        const float *inputs, const int32_t *offsets, const Levels &lv,
                        const BinInfo &bi, uint32_t gridtype, int align, SliceDyn dyn,
                        uint32_t B, const uint32_t *counts, const uint16_t *entries,
                        float *partial) {
    const bool pow2 = ge::dyn_pow2(dyn.bound);
    const float inv = pow2 ? 1.0f / (2.0f * dyn.bound) : 0.0f;
    auto kern = pow2 ? k_walk<grad_t, 3, C, true> : k_walk<grad_t, 3, C, false>;
    static bool attr[2] = {false, false};
    if (!attr[pow2]) {
        (void)hipFuncSetAttribute((const void *)kern,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
        attr[pow2] = true;
    }
    kern<<<g, 1024, lds, s>>>(grad, inputs, offsets, lv, bi, gridtype, align, dyn, inv, B,
                              counts, entries, partial);
}

}  // namespace gb
}  // namespace dfhip

using namespace dfhip;

extern "C" int dfhip_grid_backward_binned_scratch(uint32_t cap, const int32_t *offsets_host,
                                                  uint32_t L, uint32_t C, uint64_t *entries_u32,
                                                  uint64_t *counts_u32, uint64_t *partial_f32) {
    gb::BinInfo bi;
    if (!offsets_host || !gb::make_bins(offsets_host, L, C, gb::device_cus(), bi)) {
        set_error("grid_backward_binned_scratch: unsupported level layout");
        return DFHIP_EINVAL;
    }
    const uint64_t tiles = ceil_div<uint64_t>(cap ? cap : 1, gb::kTile);
    // tile-relative sample ids, u16 (kTile <= 65536), counted in u32 words
    if (entries_u32) *entries_u32 = (tiles * bi.nbins * gb::kTile + 1) / 2;
    if (counts_u32) *counts_u32 = tiles * bi.nbins;
    if (partial_f32) *partial_f32 = gb::partial_floats(bi, C);
    return DFHIP_OK;
}

extern "C" int dfhip_grid_encode_backward_binned_phase(
    int phase, int grad_dtype, const void *grad_lbc, const float *inputs, float bound,
    const int32_t *offsets, const int32_t *offsets_host, float *grad_embeddings, uint32_t B,
    const int32_t *m_dev, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
    uint32_t gridtype, int align_corners, uint32_t *entries, uint32_t *counts, float *partial,
    int accumulate, dfhip_stream_t stream) {
    const char *name = "grid_encode_backward_binned";
    if (phase < 1 || phase > 3) {
        set_error("%s: phase must be 1 (bin), 2 (walk + sum) or 3 (both), got %d", name, phase);
        return DFHIP_EINVAL;
    }
    if (D != 3 || (C != 1 && C != 2 && C != 4)) {
        set_error("%s: supports D=3 with C in {1,2,4} (got D=%u C=%u)", name, D, C);
        return DFHIP_EINVAL;
    }
    gb::BinInfo bi;
    if (!offsets_host || !gb::make_bins(offsets_host, L, C, gb::device_cus(), bi)) {
        set_error("%s: unsupported level layout", name);
        return DFHIP_EINVAL;
    }
    if (!offsets || !grad_embeddings || !entries || !counts || !partial) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (grad_dtype != DFHIP_F16 && grad_dtype != DFHIP_F32) {
        set_error("%s: grad dtype must be f16 or f32", name);
        return DFHIP_EDTYPE;
    }
    hipStream_t s = as_stream(stream);
    const uint32_t total_rows = (uint32_t)offsets_host[L];
    const ge::Levels lv = ge::make_levels(L, S, H);
    const ge::SliceDyn dyn{m_dev, bound};
    if (B > 0) {
        if (!grad_lbc || !inputs) {
            set_error("%s: null pointer", name);
            return DFHIP_EINVAL;
        }
        const uint32_t tiles = ceil_div(B, gb::kTile);
        const uint32_t gbin = tiles < 4096u ? tiles : 4096u;
        if (phase & 1) {
            const bool pow2 = ge::dyn_pow2(dyn.bound);
            const float inv = pow2 ? 1.0f / (2.0f * dyn.bound) : 0.0f;
            if (pow2)
                gb::k_bin<3, true><<<gbin, 1024, 0, s>>>(inputs, offsets, lv, bi, gridtype,
                                                         align_corners, dyn, inv, B, counts,
                                                         (uint16_t *)entries);
            else
                gb::k_bin<3, false><<<gbin, 1024, 0, s>>>(inputs, offsets, lv, bi, gridtype,
                                                          align_corners, dyn, inv, B, counts,
                                                          (uint16_t *)entries);
        }
        if (!(phase & 2)) return check_launch(name);
        const dim3 g(gb::kXcds * bi.nslots);
        const size_t lds = ((size_t)1 << bi.shift) * C * sizeof(double);
#define DFHIP_WALK(GT, CC)                                                                      \
    gb::launch_walk<GT, CC>(s, g, lds, (const GT *)grad_lbc, inputs, offsets, lv, bi, gridtype, \
                            align_corners, dyn, B, counts, (const uint16_t *)entries, partial)
        if (grad_dtype == DFHIP_F16) {
            if (C == 1) DFHIP_WALK(half_t, 1); else if (C == 2) DFHIP_WALK(half_t, 2); else DFHIP_WALK(half_t, 4);
        } else {
            if (C == 1) DFHIP_WALK(float, 1); else if (C == 2) DFHIP_WALK(float, 2); else DFHIP_WALK(float, 4);
        }
#undef DFHIP_WALK
    } else {
        if (!(phase & 2)) return DFHIP_OK;
        (void)hipMemsetAsync(partial, 0, gb::partial_floats(bi, C) * sizeof(float), s);
    }
    const uint64_t want = ceil_div<uint64_t>((uint64_t)total_rows * C, 256);
    gb::k_sum<float><<<(uint32_t)(want < 4096 ? want : 4096), 256, 0, s>>>(
        partial, bi, C, total_rows, grad_embeddings, accumulate);
    return check_launch(name);
}

extern "C" int dfhip_grid_encode_backward_binned(
    int grad_dtype, const void *grad_lbc, const float *inputs, float bound,
    const int32_t *offsets, const int32_t *offsets_host, float *grad_embeddings, uint32_t B,
    const int32_t *m_dev, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
    uint32_t gridtype, int align_corners, uint32_t *entries, uint32_t *counts, float *partial,
    int accumulate, dfhip_stream_t stream) {
    return dfhip_grid_encode_backward_binned_phase(
        3, grad_dtype, grad_lbc, inputs, bound, offsets, offsets_host, grad_embeddings, B, m_dev,
        D, C, L, S, H, gridtype, align_corners, entries, counts, partial, accumulate, stream);
}
