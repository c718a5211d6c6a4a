// Binned owner-computes embedding backward of the tiled / hashed grid encoder
// (reference gridencoder/src/gridencoder.cu:226-313 kernel_grid_backward,
// restructured for gfx950).
//
// The reference issues one half2 global atomic per (sample, level, corner).
// Here every table row is owned by one LDS slice image at a time:
//
//   1. k_bin: per tile of kTile consecutive samples (one workgroup), every
//      in-bounds sample derives, level by level, the slices of its corner
//      rows and appends its tile-relative id (u16) to the (tile, slice)
//      segment (LDS counters give the slot; segments hold kTile ids, so no
//      scan is needed).  Per-(bin, tile) counts are stored bin-major, and
//      each bin's total is accumulated.
//   2. k_walk: G walk workgroups are dealt out to the bins in proportion to
//      their entries (every non-empty bin gets at least one: P_b = 1 +
//      E_b (G - nonempty) / T), so every workgroup walks about T / G entries
//      however the occupancy loads individual slices.  Part j of bin b's P_b
//      walks tiles j, j + P_b, j + 2 P_b, ...: it zeroes the slice's f64
//      accumulators in LDS, walks the segments (one wave per segment,
//      gathering the sample's position and feature gradient), adds the
//      contributions of the corners inside the slice with ds_add_f64, and
//      writes the slice to its f32 image (one per workgroup).
//   3. k_sum: every table row sums its bin's P_b images in a fixed order.
//
// Slices are 2^shift rows of one level (8192 rows x 2 channels x f64 =
// 128 KiB of LDS, one walk workgroup per CU at a time; G = 3 per CU).
// Measured on gfx950 (tools/walk_trace.py): the walk is bound by per-entry
// issue and gather latency, not by the LDS atomics (removing all of them
// gained 6 %); an XCD-local tile split bought nothing (the same per-entry
// rate without it) while piling a hot slice's entries onto few workgroups;
// and lanes must stay on nearby samples (one wave per tile segment, short
// runs per lane): equal long runs per thread cost 1.8x per entry.
// Products w * g are formed in f64 (exact) and summed in f64; each image is
// rounded to f32 once and the images are added in a fixed order (the
// reference: f16 / f32 global atomics in arbitrary order).
#include "grid_common.h"

#include <algorithm>

#include <type_traits>

namespace dfhip {
namespace gb {

using ge::Levels;
using ge::LevelCtx;
using ge::SliceDyn;
typedef unsigned long long u64;

constexpr uint32_t kTile = 1024;              // samples per binning tile (ids per segment)
constexpr uint32_t kMaxBins = 4096;
constexpr uint32_t kMaxSlices = 128;          // slices per level (k_bin's 128-bit masks)
constexpr uint32_t kSliceBytes = 128 * 1024;  // f64 accumulators of one walk workgroup
constexpr uint32_t kTotSplit = 16;            // bin totals as 16 partial sums (tile % 16)
// Segment entries are u16: the tile-relative id in bits 0..9; for stencil
// groups a satellite entry (below) carries its moved-point mask in bits 10..15.
constexpr uint32_t kIdBits = 10;
constexpr uint32_t kIdMask = (1u << kIdBits) - 1u;
static_assert(kTile == (1u << kIdBits), "ids fill the low kIdBits bits of an entry");
constexpr uint32_t kCentreCost = 4;  // walk cost of a centre entry in satellite entries
// Walk cost of a non-empty (tile, slice) segment, in entries, added to the
// bin totals that deal out the walk parts (P_b ~ cost): a segment pays a
// dependent count -> ids -> data round trip whatever its size, so a slice
// whose samples are few per tile but spread over every tile (the scene's
// edge slices) is slow per entry.  Entries alone (r05 walk timeline, 1.1 M
// samples): such single-part bins walked 67-180 entries/us against ~300 for
// the others, and the slowest of them (173 us) set the 260 us kernel span
// beside a 75 us mean workgroup.
#ifndef DFHIP_SEG_COST
#define DFHIP_SEG_COST 48
#endif
#ifndef DFHIP_SEG_COST7  // the same for stencil groups, in satellite entries
#define DFHIP_SEG_COST7 48
#endif

struct BinInfo {
    uint32_t L, nbins, shift, tcap;      // tcap: tiles of the capacity (counts row stride)
    uint32_t tile;                       // samples per tile = id slots per segment
    uint32_t G;                          // walk workgroups
    uint32_t lane_perm;                  // walk: bit-reversed lane -> run map (1) or identity
    uint32_t o_totals, o_plan;           // word offsets into `counts` (layout below)
    uint32_t clear_totals;               // k_sum zeroes the totals after use (kept-clean scratch)
    uint32_t bin0[ge::kMaxLevels + 1];   // first bin of level l (bin0[L] = nbins)
    uint32_t base[ge::kMaxLevels];       // first row of level l
    uint32_t rows[ge::kMaxLevels];       // rows of level l
    uint64_t *trace;                     // debug: per-workgroup walk timeline (null: off)
};

// Debug walk timeline: where a workgroup ran — XCC id in the high word, the
// HW_ID register (CU / SH / SE ids) in the low word.
__device__ __forceinline__ uint64_t trace_hw_id() {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    return ((uint64_t)xcc << 32) | hw;
}

// Walk workgroups per CU (default 3: walk + sum 216.5 -> 208.4 us per C2
// step against 4; 2 and 5-6 slower).  A/B: dfhip_binned_opts.walk_groups_per_cu.
#ifndef DFHIP_WALK_G_DEFAULT
#define DFHIP_WALK_G_DEFAULT 3
#endif
// Walk form of a NULL / -1 walk_mode (-1: per group, see flat_walk_mode);
// variant libraries (tools/variant_lib.sh) set it for A/B of the replayed step.
#ifndef DFHIP_WALK_MODE_DEFAULT
#define DFHIP_WALK_MODE_DEFAULT -1
#endif

// The per-call options (dfhip_binned_opts, NULL = defaults) resolved once per
// call; the library keeps no mode state between calls.
struct Opts {
    int walk_mode;        // -1: per group (per-segment for single samples, flat for groups)
    bool fast_bin;        // mask-form fast binning where it applies
    uint32_t walk_g;      // walk workgroups per CU
    uint32_t lane_perm;   // per-segment walk: bit-reversed lane -> run map
    bool clean;           // the counts scratch's totals / plan words are zero on entry
    uint64_t *trace;      // debug walk timeline or null
};

static bool resolve_opts(const dfhip_binned_opts *o, Opts &r) {
    r.walk_mode = DFHIP_WALK_MODE_DEFAULT;
    r.fast_bin = true;
    r.walk_g = DFHIP_WALK_G_DEFAULT;
    r.lane_perm = 1;
    r.clean = false;
    r.trace = nullptr;
    if (!o) return true;
    if (o->walk_mode < -1 || o->walk_mode > 1) {
        set_error("binned backward: walk_mode must be -1, 0 or 1 (got %d)",
                  (int)o->walk_mode);
        return false;
    }
    if (o->walk_groups_per_cu < 0 || o->walk_groups_per_cu > 16) {
        set_error("binned backward: walk_groups_per_cu must be 0..16 (got %d)",
                  (int)o->walk_groups_per_cu);
        return false;
    }
    if (o->walk_mode >= 0) r.walk_mode = o->walk_mode;
    r.fast_bin = o->fast_bin != 0;
    if (o->walk_groups_per_cu > 0) r.walk_g = (uint32_t)o->walk_groups_per_cu;
    if (o->lane_perm >= 0) r.lane_perm = o->lane_perm != 0;
    r.clean = o->kept_clean > 0;
    r.trace = o->trace;
    return true;
}

static uint32_t slice_shift(uint32_t C) {
    uint32_t shift = 0;
    while ((2ull << shift) * 8ull * C <= kSliceBytes) ++shift;
    return shift;  // largest 2^shift rows with 2^shift * C doubles <= kSliceBytes
}

// scratch layout (u32 words of `counts`):
//   [tcap][nbins]  per-(tile, bin) counts          (k_bin)
//   [nbins][16]    totals, as 16 partial sums      (k_bin; zeroed before it)
//   [nbins][2]     first image slot, parts         (k_walk; zeroed before k_bin)
// Host: bins and layout from the HOST copy of the offsets.
static int flat_walk_mode(uint32_t group, const Opts &op);
static bool make_bins(const int32_t *offsets_host, uint32_t L, uint32_t C, uint32_t cap,
                      uint32_t group, const Opts &op, BinInfo &bi) {
    if (L == 0 || L > ge::kMaxLevels || C == 0) return false;
    bi.L = L;
    bi.trace = op.trace;
    bi.clear_totals = 0;
    bi.shift = slice_shift(C);
    bi.tile = kTile;
    bi.tcap = ceil_div<uint32_t>(cap ? cap : 1u, bi.tile);
    bi.G = op.walk_g * device_cus();
    bi.lane_perm = op.lane_perm;
    uint32_t nb = 0;
    for (uint32_t l = 0; l < L; ++l) {
        const uint32_t rows = (uint32_t)(offsets_host[l + 1] - offsets_host[l]);
        const uint32_t ns = rows ? ((rows - 1) >> bi.shift) + 1 : 0;
        if (ns > kMaxSlices) return false;
        bi.bin0[l] = nb;
        bi.base[l] = (uint32_t)offsets_host[l];
        bi.rows[l] = rows;
        nb += ns;
    }
    bi.bin0[L] = nb;
    bi.nbins = nb;
    if (nb == 0 || nb > kMaxBins) return false;
    if (bi.G < nb) bi.G = nb;  // every bin can get a workgroup
    // totals + plan start on a 16-byte boundary and span whole 16-byte words,
    // so the per-call clear is ONE aligned fill (an unaligned one took two
    // fill launches)
    const uint64_t tot = ((uint64_t)nb * bi.tcap + 3ull) & ~3ull;
    if (tot + (kTotSplit + 2ull) * nb + 4ull >= (1ull << 32)) return false;
    bi.o_totals = (uint32_t)tot;
    bi.o_plan = bi.o_totals + nb * kTotSplit;
    return true;
}
static uint64_t counts_words(const BinInfo &bi) {
    return ((uint64_t)bi.o_plan + 2ull * bi.nbins + 3ull) & ~3ull;
}

__device__ __forceinline__ uint32_t bin_total(const uint32_t *__restrict__ totals, uint32_t b) {
    const uint4 *p = reinterpret_cast<const uint4 *>(totals + (size_t)b * kTotSplit);
    uint32_t t = 0;
#pragma unroll
    for (uint32_t i = 0; i < kTotSplit / 4; ++i) {
        const uint4 v = p[i];
        t += v.x + v.y + v.z + v.w;
    }
    return t;
}
static uint64_t partial_floats(const BinInfo &bi, uint32_t C) {
    return (uint64_t)bi.G * ((uint64_t)1 << bi.shift) * C;
}

// Exclusive prefix over a wave (64 lanes) and the wave total.
__device__ __forceinline__ u64 wave_excl_scan(u64 v, uint32_t lane, u64 *total) {
    u64 inc = v;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const u64 u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
    }
    *total = __shfl(inc, 63, 64);
    return inc - v;
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

// Slices touched by the corners of a cell at one level, as a bit mask of
// W words (W = 1 for levels of at most 64 slices, else 2).
template <uint32_t D, int MODE, uint32_t W>
__device__ __forceinline__ void slice_mask(const ge::LevelRows &lr, const uint32_t cell[D],
                                           uint32_t shift, uint64_t (&mask)[W]) {
#pragma unroll
    for (uint32_t h = 0; h < W; ++h) mask[h] = 0;
    if constexpr (MODE == 0 && D == 3) {
        // mask form (as the walk's flush): the cell's tiled index once, the
        // corner offsets {0, 1, m1, m1 + 1, m2, ...} uniform
        const uint32_t i0 = cell[0] + cell[1] * lr.m1 + cell[2] * lr.m2;
#pragma unroll
        for (uint32_t k = 0; k < 8u; ++k) {
            if (k >> lr.lead) continue;
            const uint32_t o = (k & 1u) + ((k & 2u) ? lr.m1 : 0u) + ((k & 4u) ? lr.m2 : 0u);
            const uint32_t v = ((i0 + o) & lr.wmask) >> shift;
            if constexpr (W == 1) {
                mask[0] |= 1ull << v;
            } else {
                if (v < 64) mask[0] |= 1ull << v;
                else mask[1] |= 1ull << (v - 64);
            }
        }
        return;
    }
#pragma unroll
    for (uint32_t k = 0; k < (1u << D); ++k) {
        if (k >> lr.lead) continue;
        const uint32_t v = ge::corner_row_m<D, MODE>(lr, cell, k) >> shift;
        if constexpr (W == 1) {
            mask[0] |= 1ull << v;
        } else {
            if (v < 64) mask[0] |= 1ull << v;
            else mask[1] |= 1ull << (v - 64);
        }
    }
}

// Append sample s (tile-relative id) to the segments of the slices in mask.
template <uint32_t W>
__device__ __forceinline__ void append(const uint64_t (&mask)[W], uint32_t b0, uint32_t *cnt,
                                       uint16_t *seg, uint16_t id, uint32_t tile) {
#pragma unroll
    for (uint32_t h = 0; h < W; ++h) {
        uint64_t mk = mask[h];
        while (mk) {
            const uint32_t b = b0 + (uint32_t)__builtin_ctzll(mk) + 64u * h;
            mk &= mk - 1;
            const uint32_t slot = atomicAdd(&cnt[b], 1u);
            seg[(size_t)b * tile + slot] = id;
        }
    }
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
    const uint32_t T = bi.tile;
    const uint32_t ntiles = ceil_div(M, T);
    const uint32_t nb = bi.nbins;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) cnt[b] = 0;
        __syncthreads();
        uint16_t *seg = entries + (size_t)tile * nb * T;
        const uint32_t s_end = min(M, (tile + 1) * T);
        for (uint32_t s = tile * T + threadIdx.x; s < s_end; s += blockDim.x) {
            float x[D];
            if (!load_pos<D, POW2>(inputs, dyn, inv, s, x)) continue;
            for (uint32_t l = 0; l < bi.L; ++l) {
                const LevelCtx c = ge::level_ctx<D>(offsets, lv, l, gridtype, align);
                const ge::LevelRows lr = ge::level_rows<D>(c);
                uint32_t cell[D];
                float frac[D];
                locate<D>(c, align, x, cell, frac);
                const int mode = ge::row_mode(lr);
                const uint32_t b0 = bi.bin0[l];
                const uint16_t id = (uint16_t)(s - tile * T);
                if (bi.bin0[l + 1] - b0 <= 64) {  // uniform: one mask word
                    uint64_t mask[1];
                    if (mode == 0) slice_mask<D, 0, 1>(lr, cell, bi.shift, mask);
                    else if (mode == 1) slice_mask<D, 1, 1>(lr, cell, bi.shift, mask);
                    else slice_mask<D, 2, 1>(lr, cell, bi.shift, mask);
                    append<1>(mask, b0, cnt, seg, id, T);
                } else {
                    uint64_t mask[2];
                    if (mode == 0) slice_mask<D, 0, 2>(lr, cell, bi.shift, mask);
                    else if (mode == 1) slice_mask<D, 1, 2>(lr, cell, bi.shift, mask);
                    else slice_mask<D, 2, 2>(lr, cell, bi.shift, mask);
                    append<2>(mask, b0, cnt, seg, id, T);
                }
            }
        }
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
            const uint32_t v = cnt[b];
            counts[(size_t)tile * nb + b] = v;
            if (v)
                atomicAdd(&counts[bi.o_totals + b * kTotSplit + tile % kTotSplit],
                          v + (uint32_t)DFHIP_SEG_COST);
        }
        __syncthreads();
    }
}

// Binning, mask-form fast path: every level wraps rows by a mask (or never
// wraps), has at most 64 slices and L <= kFastLevels (the reference's grid:
// three dense levels + thirteen 2^16-row tiled levels).  The per-level
// constants are host-evaluated kernel arguments (scalar loads) instead of
// level_ctx / level_rows per sample and level, and the slices of the 2^lead
// corners come from the 2^(lead-1) x-neighbour pairs: corner rows r and
// r + 1 share a slice unless r is the slice's last row (then r + 1 wraps by
// the mask or starts the next slice).  Same entries as k_bin.
constexpr uint32_t kFastLevels = 16;

struct FastLevels {
    float scale[kFastLevels];
    uint32_t m1[kFastLevels], m2[kFastLevels], wmask[kFastLevels];
    uint32_t lead[kFastLevels], bin0[kFastLevels];
};

// Finite-difference stencil groups (the shaded train step, csrc/shade.hip):
// field row GROUP g + a (GROUP = 7) is point a of sample g, a = 0 the sample
// itself, a = 1 + s the clamped x + (s odd ? -eps : eps) e_(s >> 1)
// (k_stencil's arithmetic, network_grid.py:90-104).  Binned per group, one
// entry per (group, slice) instead of one per (row, slice), of two kinds:
//   * centre entries (front of the segment): the slices the sample's own
//     corners touch; the walk derives all seven points from the sample's
//     position and reads the group's seven gradient rows (adjacent in the
//     [L, 7 M, C] planes);
//   * satellite entries (back of the segment, counted in the high 16 bits of
//     the segment count): slices that only moved points touch (at the mid and
//     fine levels a +-eps move along y or z is one or more slices away), with
//     the mask of those points in the entry's bits 10..15; the walk takes
//     only them (usually one) instead of all seven.
// On the reference grid this cuts the walked points per group from ~243 to
// ~165 (34.7 entries per group: 21.6 centre, 13.2 satellite).
struct Stencil {
    float eps, bound;
};

template <uint32_t GROUP>
__device__ __forceinline__ void group_point(const float (&xr)[3], uint32_t a, const Stencil &st,
                                            float (&p)[3]) {
    if (GROUP == 1 || a == 0) {
#pragma unroll
        for (uint32_t d = 0; d < 3; ++d) p[d] = xr[d];
        return;
    }
    const uint32_t s = a - 1u, axis = s >> 1;
    const float off = (s & 1u) ? -st.eps : st.eps;
#pragma unroll
    for (uint32_t d = 0; d < 3; ++d) {
        const float v = xr[d] + (d == axis ? off : 0.0f);
        p[d] = fminf(fmaxf(v, -st.bound), st.bound);
    }
}

// Wave-aggregated appends of one level, called by all 64 lanes of a wave:
// centre entries (slice mask mc, front of the segment, +1 on the packed
// count) and, for stencil groups, satellite entries (mask ms, back of the
// segment, +2^16) carrying their moved-point masks (from mo).  Per slice k of
// the level a ballot per kind gives each lane its rank; lane k adds the wave's
// counts of slice k to that slice's counter, i.e. the level's ns counters in
// ONE LDS atomic instruction on distinct addresses, instead of one atomic per
// entry (a one-slice coarse level put all 64 lanes of an instruction on the
// same counter: r04 PMC, conflict cycles 8.7x the LDS-active ones).
// Levels of at most this many slices append wave-aggregated (wave_append);
// the others one LDS atomic per entry (lane_append).  All levels wave-
// aggregated (every slice of every level a ballot, twice) removed the bank
// conflicts but cost more VALU than they saved: k_bin_fast 64 -> 102 us
// (1.1 M samples), <7> 173 -> 269 us per textureless step.
#ifndef DFHIP_BIN_BALLOT_NS
#define DFHIP_BIN_BALLOT_NS 0
#endif

// One lane's appends (an LDS atomic per entry: slot = the counter's old value).
template <bool SAT>
__device__ __forceinline__ void lane_append(uint32_t *cnt, uint16_t *seg, uint32_t b0,
                                            uint64_t mc, uint64_t ms, const uint64_t (&mo)[6],
                                            uint16_t id, uint32_t tile) {
    while (mc) {
        const uint32_t b = b0 + (uint32_t)__builtin_ctzll(mc);
        mc &= mc - 1;
        const uint32_t slot = atomicAdd(&cnt[b], 1u) & 0xFFFFu;
        seg[(size_t)b * tile + slot] = id;
    }
    if constexpr (SAT) {
        while (ms) {
            const uint32_t sl = (uint32_t)__builtin_ctzll(ms);
            ms &= ms - 1;
            uint32_t m6 = 0;
#pragma unroll
            for (uint32_t a = 0; a < 6; ++a) m6 |= (uint32_t)((mo[a] >> sl) & 1ull) << a;
            const uint32_t b = b0 + sl;
            const uint32_t slot = tile - 1u - (atomicAdd(&cnt[b], 1u << 16) >> 16);
            seg[(size_t)b * tile + slot] = (uint16_t)(id | (m6 << kIdBits));
        }
    }
}

template <bool SAT>
__device__ __forceinline__ void wave_append(uint32_t *cnt, uint16_t *seg, uint32_t b0, uint32_t ns,
                                            uint64_t mc, uint64_t ms, const uint64_t (&mo)[6],
                                            uint16_t id, uint32_t lane, uint32_t tile) {
    uint32_t myc = 0;
    for (uint32_t k = 0; k < ns; ++k) {  // uniform
        uint32_t v = (uint32_t)__popcll(__ballot((mc >> k) & 1ull));
        if constexpr (SAT) v |= (uint32_t)__popcll(__ballot((ms >> k) & 1ull)) << 16;
        if (lane == k) myc = v;
    }
    uint32_t base = 0;
    if (lane < ns && myc) base = atomicAdd(&cnt[b0 + lane], myc);
    for (uint32_t k = 0; k < ns; ++k) {  // uniform
        const u64 bc = __ballot((mc >> k) & 1ull);
        const u64 bs = SAT ? __ballot((ms >> k) & 1ull) : 0ull;
        if (!(bc | bs)) continue;  // uniform
        const uint32_t bk = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)k);
        uint16_t *sg = seg + (size_t)(b0 + k) * tile;
        if ((mc >> k) & 1ull)
            sg[(bk & 0xFFFFu) + __builtin_amdgcn_mbcnt_hi((uint32_t)(bc >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bc, 0u))] = id;
        if constexpr (SAT) {
            if ((ms >> k) & 1ull) {
                uint32_t m6 = 0;
#pragma unroll
                for (uint32_t a = 0; a < 6; ++a) m6 |= (uint32_t)((mo[a] >> k) & 1ull) << a;
                const uint32_t r = (bk >> 16) + __builtin_amdgcn_mbcnt_hi(
                                                    (uint32_t)(bs >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)bs, 0u));
                sg[tile - 1u - r] = (uint16_t)(id | (m6 << kIdBits));
            }
        }
    }
}

template <bool POW2, uint32_t GROUP = 1>
__global__ __launch_bounds__(1024) void k_bin_fast(const float *__restrict__ inputs,
                                                  FastLevels fl, BinInfo bi, int align_corners,
                                                  SliceDyn dyn, float inv, uint32_t B,
                                                  uint32_t *__restrict__ counts,
                                                  uint16_t *__restrict__ entries,
                                                  Stencil st = Stencil{0.0f, 0.0f}) {
    __shared__ uint32_t cnt[kMaxBins];
    const float half = align_corners ? 0.0f : 0.5f;
    const uint32_t M = ge::dyn_count(dyn, B);
    const uint32_t T = GROUP == 1 ? bi.tile : kTile;
    const uint32_t ntiles = ceil_div(M, T);
    const uint32_t nb = bi.nbins, shift = bi.shift, smask = (1u << bi.shift) - 1u;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) cnt[b] = 0;
        __syncthreads();
        uint16_t *seg = entries + (size_t)tile * nb * T;
        const uint32_t s_end = min(M, (tile + 1) * T);
        // a uniform trip count: every lane of a wave reaches the per-level
        // appends, which may be wave-wide
        for (uint32_t s0 = tile * T; s0 < s_end; s0 += blockDim.x) {
            const uint32_t s = s0 + threadIdx.x;
            // the group's points, mapped to [0, 1]; out-of-range points skip
            float xg[GROUP][3];
            uint32_t in = 0;
#pragma unroll
            for (uint32_t a = 0; a < GROUP; ++a) xg[a][0] = xg[a][1] = xg[a][2] = 0.0f;
            if constexpr (GROUP == 1) {
                if (s < s_end && load_pos<3, POW2>(inputs, dyn, inv, s, xg[0])) in = 1;
            } else if (s < s_end) {
                float xr[3];
#pragma unroll
                for (uint32_t d = 0; d < 3; ++d) xr[d] = inputs[(size_t)s * 3 + d];
#pragma unroll
                for (uint32_t a = 0; a < GROUP; ++a) {
                    float p[3];
                    group_point<GROUP>(xr, a, st, p);
                    bool ok = true;
#pragma unroll
                    for (uint32_t d = 0; d < 3; ++d) {
                        xg[a][d] = ge::dyn_map_t<POW2>(dyn, inv, p[d]);
                        ok = ok && !(xg[a][d] < 0.0f) && !(xg[a][d] > 1.0f);
                    }
                    in |= (ok ? 1u : 0u) << a;
                }
            }
            const uint16_t id = (uint16_t)(s - tile * T);
            const uint32_t lane = threadIdx.x & 63u;
            // stencil groups: point 1 + 2 axis + k moves only along `axis`, so
            // when its other two mapped coordinates equal the sample's (the
            // sample inside the bound: the clamp is the identity) its cell
            // differs from the sample's along that axis only, and its tiled
            // index is the sample's plus (c' - c) times the axis stride (one
            // floor per point instead of three; a z move is invisible at the
            // z-dropped levels)
            bool incr = false;
            if constexpr (GROUP == 7) {
                incr = in == 0x7Fu;
#pragma unroll
                for (uint32_t a = 1; a < 7; ++a) {
                    const uint32_t ax = (a - 1u) >> 1;
#pragma unroll
                    for (uint32_t d = 0; d < 3; ++d)
                        if (d != ax) incr = incr && xg[a][d] == xg[0][d];
                }
            }
            for (uint32_t l = 0; l < bi.L; ++l) {
                const float sc = fl.scale[l];
                const uint32_t m1 = fl.m1[l], m2 = fl.m2[l], wm = fl.wmask[l], lead = fl.lead[l];
                // slices of the corners of the cell with tiled index i0 into mk
                auto pairs = [&](uint32_t i0, uint64_t &mk) {
#pragma unroll
                    for (uint32_t p = 0; p < 4; ++p) {  // x-neighbour pairs {0,1} + {0, m1, m2, m1+m2}
                        if (p >= (1u << (lead - 1u))) break;  // uniform
                        const uint32_t o = ((p & 1u) ? m1 : 0u) + ((p & 2u) ? m2 : 0u);
                        const uint32_t r = (i0 + o) & wm;
                        mk |= 1ull << (r >> shift);
                        if ((r & smask) == smask) mk |= 1ull << (((r + 1u) & wm) >> shift);
                    }
                };
                const uint32_t b0 = fl.bin0[l], ns = bi.bin0[l + 1] - b0;
                if constexpr (GROUP == 1) {
                    uint64_t mask = 0;
                    if (in) {
                        const uint32_t c0 = (uint32_t)floorf(fmaf(xg[0][0], sc, half));
                        const uint32_t c1 = (uint32_t)floorf(fmaf(xg[0][1], sc, half));
                        const uint32_t c2 = (uint32_t)floorf(fmaf(xg[0][2], sc, half));
                        pairs(c0 + c1 * m1 + c2 * m2, mask);
                    }
                    const uint64_t none[6] = {0, 0, 0, 0, 0, 0};
                    if (ns <= DFHIP_BIN_BALLOT_NS)  // uniform
                        wave_append<false>(cnt, seg, b0, ns, mask, 0, none, id, lane, T);
                    else
                        lane_append<false>(cnt, seg, b0, mask, 0, none, id, T);
                } else {
                    // mc: slices of the sample's own corners; mo[a - 1]: those of
                    // moved point a (0 when its cell is the sample's)
                    uint64_t mc = 0, mo[6] = {0, 0, 0, 0, 0, 0};
                    if (incr) {
                        uint32_t c[3];
#pragma unroll
                        for (uint32_t d = 0; d < 3; ++d) c[d] = (uint32_t)floorf(fmaf(xg[0][d], sc, half));
                        const uint32_t i0 = c[0] + c[1] * m1 + c[2] * m2;
                        pairs(i0, mc);
#pragma unroll
                        for (uint32_t a = 1; a < 7; ++a) {
                            const uint32_t ax = (a - 1u) >> 1;
                            const uint32_t stride = ax == 0 ? 1u : (ax == 1 ? m1 : m2);
                            if (stride == 0) continue;  // uniform: a dim the index drops
                            const uint32_t ca = (uint32_t)floorf(fmaf(xg[a][ax], sc, half));
                            if (ca != c[ax]) pairs(i0 + (ca - c[ax]) * stride, mo[a - 1]);
                        }
                    } else if (in) {
#pragma unroll
                        for (uint32_t a = 0; a < 7; ++a) {
                            if (!((in >> a) & 1u)) continue;
                            const uint32_t c0 = (uint32_t)floorf(fmaf(xg[a][0], sc, half));
                            const uint32_t c1 = (uint32_t)floorf(fmaf(xg[a][1], sc, half));
                            const uint32_t c2 = (uint32_t)floorf(fmaf(xg[a][2], sc, half));
                            if (a == 0) pairs(c0 + c1 * m1 + c2 * m2, mc);
                            else pairs(c0 + c1 * m1 + c2 * m2, mo[a - 1]);
                        }
                    }
                    // centre entries (front of the segment): every slice the
                    // sample's corners touch; the walk takes all seven points
                    // there.  Satellite entries (back of the segment): slices
                    // only moved points touch, with the mask of those points in
                    // bits 10..15.  (A mask of the moved points touching a centre
                    // entry's slice, to skip the others there, cost more in the
                    // binning than it saved in the walk: bin 173 -> 192 us, walk
                    // 972 -> 964 us.)
                    const uint64_t ms = (mo[0] | mo[1] | mo[2] | mo[3] | mo[4] | mo[5]) & ~mc;
                    if (ns <= DFHIP_BIN_BALLOT_NS)  // uniform
                        wave_append<true>(cnt, seg, b0, ns, mc, ms, mo, id, lane, T);
                    else
                        lane_append<true>(cnt, seg, b0, mc, ms, mo, id, T);
                }
            }
        }
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
            const uint32_t v = cnt[b];
            counts[(size_t)tile * nb + b] = v;
            // bin totals weigh a centre entry (seven points) as kCentreCost
            // satellite entries (one point) for the walk's part plan
            const uint32_t w = (v & 0xFFFFu) * (GROUP > 1 ? kCentreCost : 1u) + (v >> 16);
            if (w)
                atomicAdd(&counts[bi.o_totals + b * kTotSplit + tile % kTotSplit],
                          w + (uint32_t)(GROUP > 1 ? DFHIP_SEG_COST7 : DFHIP_SEG_COST));
        }
        __syncthreads();
    }
}

// Host: the FastLevels of a layout, or false when the fast path does not
// apply (the host restatement of ge::level_ctx / level_rows, D = 3).
static bool make_fast_levels(const int32_t *offsets_host, const Levels &lv, const BinInfo &bi,
                             uint32_t gridtype, bool align, FastLevels &fl) {
    if (bi.L > kFastLevels) return false;
    for (uint32_t l = 0; l < bi.L; ++l) {
        // u32 stride as the device (and gridencoder.cu:56-63) evaluate it
        const uint32_t hsize = (uint32_t)(offsets_host[l + 1] - offsets_host[l]);
        const uint32_t smul = align ? lv.res[l] : lv.res[l] + 1u;
        uint32_t stride = 1, used = 0;
        uint64_t span = 1;
        for (uint32_t d = 0; d < 3; ++d)
            if (stride <= hsize) {
                stride *= smul;
                ++used;
            }
        for (uint32_t d = 0; d < used; ++d) span *= smul;
        const bool hashed = gridtype == 0 && stride > hsize;
        const bool pow2 = (hsize & (hsize - 1)) == 0;
        if (hashed || (!pow2 && span > hsize)) return false;  // not the mask form
        if (bi.bin0[l + 1] - bi.bin0[l] > 64 || used == 0) return false;
        fl.scale[l] = lv.scale[l];
        fl.lead[l] = used;
        fl.m1[l] = used > 1 ? smul : 0u;
        fl.m2[l] = used > 2 ? smul * smul : 0u;
        fl.wmask[l] = pow2 ? hsize - 1u : 0xFFFFFFFFu;
        fl.bin0[l] = bi.bin0[l];
    }
    return true;
}

// ---------------------------------------------------------------- 2. walk
__device__ __forceinline__ void lds_add(double *acc, uint32_t idx, double v, uint32_t k) {
    (void)k;
    atomicAdd(acc + idx, v);
}

// Flush one cell's merged corner contributions into the LDS slice [r0, r1).
template <uint32_t D, uint32_t C, int MODE, uint32_t LEAD>
__device__ __forceinline__ void flush_m(double *acc, uint32_t cs, uint32_t r0, uint32_t r1,
                                        const LevelCtx &c, const ge::LevelRows &lr,
                                        const uint32_t cell[D], const double (&cw)[1u << D][C]);

constexpr int kModeAny = 3;  // MODE: the corner-row wrap fixed at compile time, or any

// LEAD: the level's corner count exponent (lr.lead) fixed at compile time
// (the walk dispatches on it once per workgroup), or 0 to read lr.lead
template <uint32_t D, uint32_t C, int MODE, uint32_t LEAD = 0>
__device__ __forceinline__ void flush(double *acc, uint32_t cs, uint32_t r0, uint32_t r1,
                                      const LevelCtx &c, const ge::LevelRows &lr,
                                      const uint32_t cell[D], const double (&cw)[1u << D][C]) {
    if constexpr (MODE != kModeAny) {
        flush_m<D, C, MODE, LEAD>(acc, cs, r0, r1, c, lr, cell, cw);
    } else {
        const int mode = ge::row_mode(lr);  // uniform: one scalar branch per flush
        if (mode == 0) flush_m<D, C, 0, LEAD>(acc, cs, r0, r1, c, lr, cell, cw);
        else if (mode == 1) flush_m<D, C, 1, LEAD>(acc, cs, r0, r1, c, lr, cell, cw);
        else flush_m<D, C, 2, LEAD>(acc, cs, r0, r1, c, lr, cell, cw);
    }
}

template <uint32_t D, uint32_t C, int MODE, uint32_t LEAD>
__device__ __forceinline__ void flush_m(double *acc, uint32_t cs, uint32_t r0, uint32_t r1,
                                        const LevelCtx &c, const ge::LevelRows &lr,
                                        const uint32_t cell[D], const double (&cw)[1u << D][C]) {
    const uint32_t lead = LEAD ? LEAD : lr.lead;
    if constexpr (MODE == 0 && D == 3) {
        // mask form: corner k's row is base + ((i0 + o_k) & wmask) with the
        // cell's tiled index i0 (two multiplies per flush, not per corner) and
        // the uniform corner offsets o_k = {0, 1, m1, m1 + 1, m2, ...}; one
        // unsigned compare against the slice's relative range
        const uint32_t i0 = cell[0] + cell[1] * lr.m1 + cell[2] * lr.m2;
        const uint32_t lo = r0 - c.base, n = r1 - r0;
#pragma unroll
        for (uint32_t k = 0; k < 8u; ++k) {
            if (k >> lead) continue;
            const uint32_t o = (k & 1u) + ((k & 2u) ? lr.m1 : 0u) + ((k & 4u) ? lr.m2 : 0u);
            const uint32_t rel = ((i0 + o) & lr.wmask) - lo;
            if (rel < n) {
#pragma unroll
                for (uint32_t ch = 0; ch < C; ++ch) lds_add(acc, rel + ch * cs, cw[k][ch], k);
            }
        }
        return;
    }
#pragma unroll
    for (uint32_t k = 0; k < (1u << D); ++k) {
        if (k >> lead) continue;
        const uint32_t row = c.base + ge::corner_row_m<D, MODE>(lr, cell, k);
        if (row >= r0 && row < r1) {
            double *dst = acc + (row - r0);
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) atomicAdd(dst + ch * cs, cw[k][ch]);
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
//
// GROUP > 1 (stencil groups, see Stencil): an entry is a group; the lane
// takes the group's points one after another through the same cell merge
// (at the coarse levels a sample and its stencil points share a cell).
// Walk plan of every walk workgroup: this workgroup's bin b and part j of
// P_b (P_b = 1 + E_b (G - nz) / T, parts laid out in bin order); part 0
// records the bin's image slots for k_sum.  Every thread stages the bin
// totals in LDS (tot_s, kMaxBins words: one round of independent loads), then
// wave 0 scans them (twice reading the totals from global memory was 2 nb / 64
// dependent load rounds on one wave, ~4.7 us of every workgroup's start).
// All threads call it; returns in sh_b / sh_j / sh_p (sh_p = 0: an idle
// workgroup) after a barrier.
__device__ __forceinline__ void walk_plan(const BinInfo &bi, uint32_t *counts, uint32_t *tot_s,
                                          uint32_t &sh_b, uint32_t &sh_j, uint32_t &sh_p) {
    const uint32_t nb = bi.nbins, G = bi.G, slot = blockIdx.x;
    const uint32_t *totals = counts + bi.o_totals;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) tot_s[b] = bin_total(totals, b);
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t ln = threadIdx.x;
        u64 T = 0, nz = 0;
        for (uint32_t b0 = 0; b0 < nb; b0 += 64) {
            const uint32_t e = b0 + ln < nb ? tot_s[b0 + ln] : 0u;
            u64 t, z;
            (void)wave_excl_scan(e, ln, &t);
            (void)wave_excl_scan(e ? 1u : 0u, ln, &z);
            T += t;
            nz += z;
        }
        const u64 extra = G > nz ? G - nz : 0;
        uint32_t carry = 0;
        if (ln == 0) sh_p = 0;
        for (uint32_t b0 = 0; b0 < nb; b0 += 64) {
            const uint32_t b = b0 + ln;
            const uint32_t e = b < nb ? tot_s[b] : 0u;
            const uint32_t p = e ? 1u + (uint32_t)((u64)e * extra / (T ? T : 1)) : 0u;
            u64 tot;
            const uint32_t s = carry + (uint32_t)wave_excl_scan(p, ln, &tot);
            if (b < nb && p && slot >= s && slot < s + p) {
                sh_b = b;
                sh_j = slot - s;
                sh_p = p;
            }
            if (b < nb && p && slot == s) {
                counts[bi.o_plan + 2 * b] = s;
                counts[bi.o_plan + 2 * b + 1] = p;
            } else if (b < nb && !p && slot == 0) {
                // an empty bin's plan is written too, so the plan needs no
                // clearing launch (kept-clean scratch)
                counts[bi.o_plan + 2 * b] = 0;
                counts[bi.o_plan + 2 * b + 1] = 0;
            }
            carry += (uint32_t)tot;
        }
    }
    __syncthreads();
}

template <typename grad_t, uint32_t D, uint32_t C, bool POW2, int MODE, uint32_t GROUP = 1>
__global__ __launch_bounds__(1024) void k_walk(const grad_t *__restrict__ grad,  // [L, GROUP B, C]
                                               const float *__restrict__ inputs,
                                               const int32_t *__restrict__ offsets, Levels lv,
                                               BinInfo bi, uint32_t gridtype, int align_corners,
                                               SliceDyn dyn, float inv, uint32_t B,
                                               uint32_t *counts,
                                               const uint16_t *__restrict__ entries,
                                               float *__restrict__ partial,
                                               Stencil st = Stencil{0.0f, 0.0f}) {
    extern __shared__ double acc[];
    __shared__ uint32_t sh_b, sh_j, sh_p;
    __shared__ uint32_t n_seen;
    __shared__ uint32_t tot_s[kMaxBins];
    uint64_t tr0 = 0;
    if (bi.trace) tr0 = wall_clock64();
    const uint32_t nb = bi.nbins, slot = blockIdx.x;
    const uint32_t srows = 1u << bi.shift;
    // channel-major slice image (acc[ch * srows + row]): a wave's f64 adds to
    // random rows then spread over 32 bank pairs instead of 16 row groups;
    // zeroed before the plan (its barriers cover it)
    for (uint32_t i = threadIdx.x; i < srows * C; i += blockDim.x) acc[i] = 0.0;
    if (threadIdx.x == 0) n_seen = 0;
    walk_plan(bi, counts, tot_s, sh_b, sh_j, sh_p);
    const uint32_t P = sh_p;
    if (P == 0) return;  // uniform: more workgroups than parts
    const uint32_t b = sh_b, part = sh_j;
    uint32_t l = 0;
    while (l + 1 < bi.L && bi.bin0[l + 1] <= b) ++l;
    const uint32_t k = b - bi.bin0[l];
    const uint32_t r0 = bi.base[l] + (k << bi.shift);
    const uint32_t r1 = min(r0 + srows, bi.base[l] + bi.rows[l]);
    const uint32_t n = (r1 - r0) * C;
    const bool align = align_corners != 0;
    const LevelCtx c = ge::level_ctx<D>(offsets, lv, l, gridtype, align);
    const ge::LevelRows lr = ge::level_rows<D>(c);
    const uint32_t M = ge::dyn_count(dyn, B);
    const uint32_t T = GROUP == 1 ? bi.tile : kTile;
    const uint32_t ntiles = ceil_div(M, T);
    const grad_t *gl = grad + (size_t)l * GROUP * B * C;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
    // the level's lead (corners 2^lead) is uniform over the workgroup: the
    // walk is instantiated per lead, so the corner loops and the trailing-dim
    // weights are resolved at compile time (as selects on a runtime lead they
    // cost two v_cndmask per f64 accumulator per entry)
    auto tiles = [&](auto lead_c) {
    constexpr uint32_t lead = decltype(lead_c)::value;
    // part j of P: tiles j, j + P, ...; wave w takes every waves-th of those
    for (uint32_t t = part + P * wave; t < ntiles; t += P * waves) {
        const uint32_t raw = counts[(size_t)t * nb + b];
        const uint32_t cnt = raw & 0xFFFFu, nsat = raw >> 16;  // centre / satellite entries
        if (bi.trace && lane == 0) atomicAdd(&n_seen, cnt + nsat);
        const uint16_t *seg = entries + ((size_t)t * nb + b) * T;
        const uint32_t tbase = t * T;
        const uint32_t Q = (cnt + 63) >> 6;
        // lane -> run: bit-reversed lane index (lanes next to each other in a
        // wave instruction take runs far apart in the segment, i.e. different
        // rays: their flushes then rarely hit the same LDS rows at the coarse
        // levels, where a cell holds many consecutive samples)
        const uint32_t rl = bi.lane_perm ? (__builtin_bitreverse32(lane) >> 26) : lane;
        const uint32_t e0 = min(rl * Q, cnt), e1 = min(e0 + Q, cnt);
        double cw[1u << D][C];
        uint32_t cur[D];
        bool have = false;
        // one contribution: the point x (in [0, 1]) with gradient g, merged
        // into the lane's current cell or flushing it
        auto take = [&](const float (&x)[D], const float (&g)[C]) {
            uint32_t cell[D];
            float frac[D];
            locate<D>(c, align, x, cell, frac);
            bool same = have;
#pragma unroll
            for (uint32_t d = 0; d < D; ++d)
                if (d < lead) same = same && (cell[d] == cur[d]);
            if (!same) {
                if (have) flush<D, C, MODE, lead>(acc, srows, r0, r1, c, lr, cur, cw);
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
                    cw[kc][ch] = fma((double)w, (double)g[ch], cw[kc][ch]);
            }
        };
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
                float gs[RUN][GROUP][C];
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) sid[i] = tbase + seg[min(e + i, e1 - 1)];
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) {
                    load_pos3<D>(inputs, sid[i], xs[i]);
#pragma unroll
                    for (uint32_t a = 0; a < GROUP; ++a)
                        load_grad<grad_t, C>(gl + ((size_t)sid[i] * GROUP + a) * C, gs[i][a]);
                }
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) {
                    if (i < m) {  // guard, not break: keeps the run in registers
                        if constexpr (GROUP == 1) {
                            float x[D];
#pragma unroll
                            for (uint32_t d = 0; d < D; ++d)
                                x[d] = ge::dyn_map_t<POW2>(dyn, inv, xs[i][d]);
                            take(x, gs[i][0]);
                        } else {
#pragma unroll
                            for (uint32_t a = 0; a < GROUP; ++a) {
                                float p[3], x[D];
                                group_point<GROUP>(xs[i], a, st, p);
                                bool ok = true;
#pragma unroll
                                for (uint32_t d = 0; d < D; ++d) {
                                    x[d] = ge::dyn_map_t<POW2>(dyn, inv, p[d]);
                                    ok = ok && !(x[d] < 0.0f) && !(x[d] > 1.0f);
                                }
                                if (ok) take(x, gs[i][a]);
                            }
                        }
                    }
                }
            }
        };
        if (GROUP > 1 || Q <= 1)
            walk(std::integral_constant<uint32_t, 1>{});
        else if (Q <= 4)  // most mid / fine-level segments: no 8-slot batch of duplicates
            walk(std::integral_constant<uint32_t, 4>{});
        else
            walk(std::integral_constant<uint32_t, kRun>{});
        if constexpr (GROUP > 1) {
            // satellite entries (back of the segment): only the moved points
            // of the entry's mask touch this slice
            const uint16_t *sseg = seg + (T - nsat);
            const uint32_t Q2 = (nsat + 63) >> 6;
            const uint32_t f0 = min(rl * Q2, nsat), f1 = min(f0 + Q2, nsat);
            for (uint32_t e = f0; e < f1; ++e) {
                const uint32_t v = sseg[e];
                const uint32_t sid = tbase + (v & kIdMask);
                float xr[3];
                load_pos3<3>(inputs, sid, xr);
                uint32_t m6 = v >> kIdBits;
                while (m6) {
                    const uint32_t a = 1u + (uint32_t)__builtin_ctz(m6);
                    m6 &= m6 - 1u;
                    float g[C];
                    load_grad<grad_t, C>(gl + ((size_t)sid * GROUP + a) * C, g);
                    float p[3], x[D];
                    group_point<GROUP>(xr, a, st, p);
                    bool ok = true;
#pragma unroll
                    for (uint32_t d = 0; d < D; ++d) {
                        x[d] = ge::dyn_map_t<POW2>(dyn, inv, p[d]);
                        ok = ok && !(x[d] < 0.0f) && !(x[d] > 1.0f);
                    }
                    if (ok) take(x, g);
                }
            }
        }
        if (have) flush<D, C, MODE, lead>(acc, srows, r0, r1, c, lr, cur, cw);
    }
    };
    if (lr.lead >= 3 && D >= 3) tiles(std::integral_constant<uint32_t, (D >= 3 ? 3u : D)>{});
    else if (lr.lead == 2 && D >= 2) tiles(std::integral_constant<uint32_t, (D >= 2 ? 2u : D)>{});
    else tiles(std::integral_constant<uint32_t, 1u>{});
    __syncthreads();
    float *out = partial + (size_t)slot * ((size_t)srows * C);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
        out[i] = (float)acc[(i % C) * srows + i / C];
    if (bi.trace) {
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t *r = bi.trace + (size_t)blockIdx.x * 8;
            r[0] = b;
            r[1] = trace_hw_id();
            r[2] = P;
            r[3] = n_seen;
            r[4] = tr0;
            r[5] = tr0;
            r[6] = part;
            r[7] = wall_clock64();
        }
    }
}

// ---------------------------------------------------------------- 2b. flat walk
// k_walk_flat: the same slice ownership, plan and arithmetic as k_walk for the
// mask-form layouts (FastLevels), with the work of a part laid out as ONE
// sequence instead of one wave per tile segment:
//
//   * the part's tiles (part, part + P, ...) are taken in chunks of up to 1024;
//     each thread loads one tile's count and a workgroup scan lays the chunk's
//     segments end to end (E entries);
//   * the E entries are cut into 1024 equal runs, one per thread: wave w
//     takes the w-th sixteenth (its lanes stay on neighbouring samples, which
//     hit in L1: equal runs spread over the whole part cost 1.7x per entry),
//     lanes take its runs bit-reversed (one LDS instruction's lanes flush
//     different rays); a run may cross tile segments (the cursor moves to the
//     next non-empty segment in LDS, no global round trip);
//   * a lane's next batch of ids is loaded before the current batch's
//     positions / gradients are used.
//
// k_walk gave each wave whole segments: a part of ~30 tiles left half its
// 16 waves one segment behind the others, each segment paid a dependent
// count -> ids -> data round trip, and short segments left lanes idle.
// Cells are compared by their tiled index (one compare), a new cell's
// accumulators start at the products (f64, exact) instead of zero + fma, and
// the level's corner count is a template parameter.
constexpr uint32_t kChunkTiles = 1024;
#ifndef DFHIP_WALK_RUN
#define DFHIP_WALK_RUN 6
#endif
#ifndef DFHIP_WALK_RUN7  // the same for stencil groups (textureless walk: 2 -> 1 costs 20 %)
#define DFHIP_WALK_RUN7 2
#endif
#ifndef DFHIP_WALK_RUN_SAT  // the same for stencil satellite entries (one point each)
#define DFHIP_WALK_RUN_SAT 4
#endif

template <uint32_t C>
struct FlatCell {
    double cw[8][C];
    uint32_t i0;
    bool have;
};

// Cell and fractional position of a point's coordinate (gridencoder.cu:146-154).
__device__ __forceinline__ void flat_locate1(float x, float sc, float half, float &fr,
                                             uint32_t &ci) {
    const float p = fmaf(x, sc, half);
    const float fl = floorf(p);
    fr = p - fl;
    ci = (uint32_t)fl;
}

template <uint32_t C, uint32_t LEAD>
__device__ __forceinline__ void flat_take_at(FlatCell<C> &st, double *acc, uint32_t srows,
                                             uint32_t lo, uint32_t n, uint32_t m1, uint32_t m2,
                                             uint32_t wm, const float (&fr)[3],
                                             const uint32_t (&ci)[3], const float (&g)[C]);

// One point (x in [0, 1]^3) with gradient g into the lane's current cell.
template <uint32_t C, uint32_t LEAD>
__device__ __forceinline__ void flat_take(FlatCell<C> &st, double *acc, uint32_t srows,
                                          uint32_t lo, uint32_t n, float sc, float half,
                                          uint32_t m1, uint32_t m2, uint32_t wm,
                                          const float (&x)[3], const float (&g)[C]) {
    float fr[3];
    uint32_t ci[3];
#pragma unroll
    for (uint32_t d = 0; d < 3; ++d) flat_locate1(x[d], sc, half, fr[d], ci[d]);
    flat_take_at<C, LEAD>(st, acc, srows, lo, n, m1, m2, wm, fr, ci, g);
}

// The point located at (fr, ci) with gradient g into the lane's current cell.
template <uint32_t C, uint32_t LEAD>
__device__ __forceinline__ void flat_take_at(FlatCell<C> &st, double *acc, uint32_t srows,
                                             uint32_t lo, uint32_t n, uint32_t m1, uint32_t m2,
                                             uint32_t wm, const float (&fr)[3],
                                             const uint32_t (&ci)[3], const float (&g)[C]) {
    uint32_t i0 = ci[0];
    if (LEAD > 1) i0 += ci[1] * m1;
    if (LEAD > 2) i0 += ci[2] * m2;
    float tw = 1.0f;  // trailing dims dropped from the index: their corners coincide
#pragma unroll
    for (uint32_t d = LEAD; d < 3; ++d) tw *= (1.0f - fr[d]) + fr[d];
    double gd[C];
#pragma unroll
    for (uint32_t ch = 0; ch < C; ++ch) gd[ch] = (double)g[ch];
    const bool same = st.have && i0 == st.i0;
    if (!same) {
        if (st.have) {
#pragma unroll
            for (uint32_t k = 0; k < (1u << LEAD); ++k) {
                const uint32_t o = (k & 1u) + ((k & 2u) ? m1 : 0u) + ((k & 4u) ? m2 : 0u);
                const uint32_t rel = ((st.i0 + o) & wm) - lo;
                if (rel < n) {
#pragma unroll
                    for (uint32_t ch = 0; ch < C; ++ch)
                        lds_add(acc, ch * srows + rel, st.cw[k][ch], k);
                }
            }
        }
        st.i0 = i0;
        st.have = true;
        // zeroed on the (divergent) new-cell path, then one fma per value for
        // every lane (a select between fma and mul costs two more per value)
#pragma unroll
        for (uint32_t k = 0; k < (1u << LEAD); ++k)
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) st.cw[k][ch] = 0.0;
    }
#pragma unroll
    for (uint32_t k = 0; k < (1u << LEAD); ++k) {
        float w = tw;
#pragma unroll
        for (uint32_t d = 0; d < LEAD; ++d) w *= (k & (1u << d)) ? fr[d] : 1.0f - fr[d];
        const double wd = (double)w;
#pragma unroll
        for (uint32_t ch = 0; ch < C; ++ch) st.cw[k][ch] = fma(wd, gd[ch], st.cw[k][ch]);
    }
}

template <uint32_t C, uint32_t LEAD>
__device__ __forceinline__ void flat_flush(FlatCell<C> &st, double *acc, uint32_t srows,
                                           uint32_t lo, uint32_t n, uint32_t m1, uint32_t m2,
                                           uint32_t wm) {
    if (!st.have) return;
#pragma unroll
    for (uint32_t k = 0; k < (1u << LEAD); ++k) {
        const uint32_t o = (k & 1u) + ((k & 2u) ? m1 : 0u) + ((k & 4u) ? m2 : 0u);
        const uint32_t rel = ((st.i0 + o) & wm) - lo;
        if (rel < n) {
#pragma unroll
            for (uint32_t ch = 0; ch < C; ++ch) lds_add(acc, ch * srows + rel, st.cw[k][ch], k);
        }
    }
    st.have = false;
}

// A sample's GROUP gradient rows (adjacent in the [L, GROUP B, C] planes) as
// wide loads where the rows are dwords (C = 2 of f16 / bf16): 7 rows = one
// 16-byte + one 12-byte load instead of seven.
typedef uint32_t u4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u3a __attribute__((ext_vector_type(3), aligned(4)));
template <typename grad_t, uint32_t C, uint32_t GROUP>
__device__ __forceinline__ void load_group_grads(const grad_t *__restrict__ p,
                                                 float (&g)[GROUP][C]) {
    if constexpr (sizeof(grad_t) == 2 && C == 2 && GROUP == 7) {
        const u4a a = *reinterpret_cast<const u4a *>(p);
        const u3a b = *reinterpret_cast<const u3a *>(p + 8);
        const uint32_t w[7] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z};
#pragma unroll
        for (uint32_t i = 0; i < 7; ++i) {
            grad_t lo, hi;
            const uint16_t l16 = (uint16_t)(w[i] & 0xFFFFu), h16 = (uint16_t)(w[i] >> 16);
            __builtin_memcpy(&lo, &l16, 2);
            __builtin_memcpy(&hi, &h16, 2);
            g[i][0] = (float)lo;
            g[i][1] = (float)hi;
        }
    } else {
#pragma unroll
        for (uint32_t a = 0; a < GROUP; ++a) load_grad<grad_t, C>(p + a * C, g[a]);
    }
}

// One entry: sample position xr (raw) and its GROUP gradient rows g, taken
// into the lane's cell state (GROUP 7: the finite-difference stencil).
template <typename grad_t, uint32_t C, bool POW2, uint32_t GROUP, uint32_t LEAD>
__device__ __forceinline__ void flat_entry(FlatCell<C> &cell, double *acc, uint32_t srows,
                                           uint32_t lo, uint32_t n, float sc, float half,
                                           uint32_t m1, uint32_t m2, uint32_t wm,
                                           const SliceDyn &dyn, float inv, const Stencil &st,
                                           const float (&xr)[3], const float (&g)[GROUP][C]) {
    if constexpr (GROUP == 1) {
        float x[3];
#pragma unroll
        for (uint32_t d = 0; d < 3; ++d)
            x[d] = ge::dyn_map_t<POW2>(dyn, inv, xr[d]);
        flat_take<C, LEAD>(cell, acc, srows, lo, n, sc, half, m1, m2, wm, x,
                           g[0]);
    } else {
        // the sample inside the bound (the clamp of the
        // unmoved coordinates is the identity): point
        // 1 + 2 ax + k differs from the sample along ax
        // only, so only that coordinate is located again
        bool inb = true;
#pragma unroll
        for (uint32_t d = 0; d < 3; ++d)
            inb = inb && xr[d] >= -st.bound && xr[d] <= st.bound;
        float x0[3];
#pragma unroll
        for (uint32_t d = 0; d < 3; ++d) {
            x0[d] = ge::dyn_map_t<POW2>(dyn, inv, xr[d]);
            inb = inb && !(x0[d] < 0.0f) && !(x0[d] > 1.0f);
        }
        if (inb) {
            float fr0[3];
            uint32_t ci0[3];
#pragma unroll
            for (uint32_t d = 0; d < 3; ++d)
                flat_locate1(x0[d], sc, half, fr0[d], ci0[d]);
            flat_take_at<C, LEAD>(cell, acc, srows, lo, n, m1, m2, wm, fr0,
                                  ci0, g[0]);
#pragma unroll
            for (uint32_t a2 = 1; a2 < GROUP; ++a2) {
                const uint32_t ax = (a2 - 1u) >> 1;
                const float off = ((a2 - 1u) & 1u) ? -st.eps : st.eps;
                const float v = fminf(fmaxf(xr[ax] + off, -st.bound),
                                      st.bound);
                float fr[3] = {fr0[0], fr0[1], fr0[2]};
                uint32_t ci[3] = {ci0[0], ci0[1], ci0[2]};
                flat_locate1(ge::dyn_map_t<POW2>(dyn, inv, v), sc, half,
                             fr[ax], ci[ax]);
                flat_take_at<C, LEAD>(cell, acc, srows, lo, n, m1, m2, wm, fr, ci, g[a2]);
            }
        } else {  // rare (a sample on the bound): the general form
#pragma unroll
            for (uint32_t a2 = 0; a2 < GROUP; ++a2) {
                float p[3], x[3];
                group_point<GROUP>(xr, a2, st, p);
                bool ok = true;
#pragma unroll
                for (uint32_t d = 0; d < 3; ++d) {
                    x[d] = ge::dyn_map_t<POW2>(dyn, inv, p[d]);
                    ok = ok && !(x[d] < 0.0f) && !(x[d] > 1.0f);
                }
                if (ok)
                    flat_take<C, LEAD>(cell, acc, srows, lo, n, sc, half, m1,
                                       m2, wm, x, g[a2]);
            }
        }
    }
}

// A satellite entry of a stencil group (see k_bin_fast): only the moved
// points in m6 (bit a - 1: point a) touch the slice; they are taken one after
// another (usually one).  g0: the gradient of the first of them, loaded with
// the position; grow: the group's gradient rows.
template <typename grad_t, uint32_t C, bool POW2, uint32_t LEAD>
__device__ __forceinline__ void sat_entry(FlatCell<C> &cell, double *acc, uint32_t srows,
                                          uint32_t lo, uint32_t n, float sc, float half,
                                          uint32_t m1, uint32_t m2, uint32_t wm,
                                          const SliceDyn &dyn, float inv, const Stencil &st,
                                          const float (&xr)[3], uint32_t m6,
                                          const float (&g0)[C],
                                          const grad_t *__restrict__ grow) {
    float g[C];
#pragma unroll
    for (uint32_t ch = 0; ch < C; ++ch) g[ch] = g0[ch];
    bool first = true;
    while (m6) {
        const uint32_t a = 1u + (uint32_t)__builtin_ctz(m6);
        m6 &= m6 - 1u;
        if (!first) load_grad<grad_t, C>(grow + a * C, g);
        first = false;
        float p[3], x[3];
        group_point<7>(xr, a, st, p);
        bool ok = true;
#pragma unroll
        for (uint32_t d = 0; d < 3; ++d) {
            x[d] = ge::dyn_map_t<POW2>(dyn, inv, p[d]);
            ok = ok && !(x[d] < 0.0f) && !(x[d] > 1.0f);
        }
        if (ok) flat_take<C, LEAD>(cell, acc, srows, lo, n, sc, half, m1, m2, wm, x, g);
    }
}

// The loads of one entry (position; the gradient rows of a centre entry, or
// the first moved point's row of a satellite entry) and its walk.
template <typename grad_t, uint32_t C, uint32_t GROUP, bool SAT>
struct EntryIn {
    float xs[3];
    float gs[SAT ? 1 : GROUP][C];
    uint32_t m6;
};

template <typename grad_t, uint32_t C, uint32_t GROUP, bool SAT>
__device__ __forceinline__ void load_entry(EntryIn<grad_t, C, GROUP, SAT> &in,
                                           const grad_t *__restrict__ gl,
                                           const float *__restrict__ inputs, uint32_t tbase,
                                           uint32_t v) {
    // satellite entries carry their point mask above the id; other entries
    // are the plain tile-relative id (up to 16 bits for single samples)
    const uint32_t s = tbase + (SAT ? (v & kIdMask) : v);
    load_pos3<3>(inputs, s, in.xs);
    if constexpr (SAT) {
        in.m6 = v >> kIdBits;
        const uint32_t a = 1u + (uint32_t)__builtin_ctz(in.m6 | 0x40u);  // 7: none (not read)
        load_grad<grad_t, C>(gl + ((size_t)s * GROUP + (a < GROUP ? a : 0u)) * C, in.gs[0]);
    } else {
        in.m6 = 0;
        load_group_grads<grad_t, C, GROUP>(gl + (size_t)s * GROUP * C, in.gs);
    }
}

template <typename grad_t, uint32_t C, bool POW2, uint32_t GROUP, uint32_t LEAD, bool SAT>
__device__ __forceinline__ void walk_entry(FlatCell<C> &cell, const EntryIn<grad_t, C, GROUP, SAT> &in,
                                           const grad_t *__restrict__ gl, uint32_t tbase,
                                           uint32_t v, double *acc, uint32_t srows, uint32_t lo,
                                           uint32_t n, float sc, float half, uint32_t m1,
                                           uint32_t m2, uint32_t wm, const SliceDyn &dyn,
                                           float inv, const Stencil &st) {
    if constexpr (SAT) {
        sat_entry<grad_t, C, POW2, LEAD>(cell, acc, srows, lo, n, sc, half, m1, m2, wm, dyn, inv,
                                         st, in.xs, in.m6, in.gs[0],
                                         gl + (size_t)(tbase + (v & kIdMask)) * GROUP * C);
    } else {
        flat_entry<grad_t, C, POW2, GROUP, LEAD>(cell, acc, srows, lo, n, sc, half, m1, m2, wm,
                                                 dyn, inv, st, in.xs, in.gs);
    }
}

// One phase of a part's walk over a chunk of nc tiles (part + (cb + i) P):
// the centre entries (front of each segment; every entry for GROUP 1) or the
// satellite entries (back of each segment, stencil groups only).
template <typename grad_t, uint32_t C, bool POW2, uint32_t GROUP, uint32_t LEAD, uint32_t RUN,
          bool SAT>
__device__ __forceinline__ void flat_walk_chunk(
    FlatCell<C> &cell, const grad_t *__restrict__ gl, const float *__restrict__ inputs,
    const uint32_t *counts, const uint16_t *__restrict__ entries, double *acc, uint32_t *pre,
    uint32_t *wsum, uint32_t nb, uint32_t b, uint32_t part, uint32_t P, uint32_t cb,
    uint32_t nc, uint32_t srows, uint32_t lo, uint32_t n, float sc, float half, uint32_t m1,
    uint32_t m2, uint32_t wm, const SliceDyn &dyn, float inv, const Stencil &st,
    uint32_t *entries_seen) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t waves = blockDim.x >> 6, nthr = blockDim.x;
    // the chunk's segments end to end: exclusive scan of the counts
    const uint32_t raw = tid < nc ? counts[(size_t)(part + (cb + tid) * P) * nb + b] : 0u;
    const uint32_t v = SAT ? (raw >> 16) : (raw & 0xFFFFu);
    uint32_t inc = v;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t wofs = 0;
    for (uint32_t w = 0; w < wave; ++w) wofs += wsum[w];
    if (tid < nc) pre[tid] = wofs + inc - v;
    if (tid == 0) {
        uint32_t tot = 0;
        for (uint32_t w = 0; w < waves; ++w) tot += wsum[w];
        pre[nc] = tot;
    }
    __syncthreads();
    const uint32_t E = pre[nc];
    if (tid == 0) *entries_seen += E;  // the debug trace's entry count
    // entries of chunk tile ti: front slots [0, cnt) or back slots [kTile - cnt, kTile)
    constexpr uint32_t T = kTile;
    auto seg_of = [&](uint32_t ti) {
        const uint32_t t = part + (cb + ti) * P;
        const uint16_t *sg = entries + ((size_t)t * nb + b) * T;
        return SAT ? sg + (T - (pre[ti + 1] - pre[ti])) : sg;
    };
    {
        const uint32_t Q = ceil_div(E, nthr);
        // wave w takes the w-th 1/waves of the chunk, so its lanes stay on
        // neighbouring samples (one or two tile segments: positions and
        // gradients hit in L1); inside it lane -> run is bit-reversed, so the
        // lanes of one LDS instruction flush different rays
        const uint32_t r = wave * 64u + (__builtin_bitreverse32(lane) >> 26);
        uint32_t e = min(r * Q, E);
        const uint32_t e1 = min(e + Q, E);
        if (e < e1) {
            // segment of entry e: the last ti with pre[ti] <= e
            uint32_t a = 0, z = nc;  // pre[a] <= e < pre[z]
            while (z - a > 1) {
                const uint32_t mid = (a + z) >> 1;
                if (pre[mid] <= e) a = mid;
                else z = mid;
            }
            uint32_t ti = a, tend = pre[ti + 1], slot = e - pre[ti];
            uint32_t t = part + (cb + ti) * P;
            // batch descriptor: (segment, first slot, size, tile base)
            auto batch_size = [&](uint32_t ee, uint32_t te) { return min(RUN, min(e1, te) - ee); };
            uint32_t m = batch_size(e, tend);
            const uint16_t *seg = seg_of(ti);
            uint32_t ids[RUN];
#pragma unroll
            for (uint32_t i = 0; i < RUN; ++i) ids[i] = seg[slot + min(i, m - 1)];
            while (true) {
                const uint32_t tbase = t * T;
                // next batch: cursor and its entries, loaded ahead of this batch's data
                uint32_t ne = e + m, nslot = slot + m, nti = ti, ntend = tend, nt2 = t;
                const uint16_t *nseg = seg;
                if (ne == ntend && ne < e1) {
                    // the next non-empty segment (ne < e1 <= E: one exists); an
                    // empty one would make a batch of zero entries whose clamped
                    // loads read slots never written
                    do {
                        ++nti;
                        ntend = pre[nti + 1];
                    } while (ntend == ne);
                    nslot = 0;
                    nt2 = part + (cb + nti) * P;
                    nseg = seg_of(nti);
                }
                const bool more = ne < e1;
                const uint32_t nm = more ? batch_size(ne, ntend) : 1u;
                uint32_t nids[RUN];
                if (more) {
#pragma unroll
                    for (uint32_t i = 0; i < RUN; ++i) nids[i] = nseg[nslot + min(i, nm - 1)];
                }
                EntryIn<grad_t, C, GROUP, SAT> in[RUN];
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) load_entry(in[i], gl, inputs, tbase, ids[i]);
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) {
                    if (i < m)
                        walk_entry<grad_t, C, POW2, GROUP, LEAD, SAT>(
                            cell, in[i], gl, tbase, ids[i], acc, srows, lo, n, sc, half, m1, m2,
                            wm, dyn, inv, st);
                }
                if (!more) break;
                e = ne;
                slot = nslot;
                ti = nti;
                tend = ntend;
                t = nt2;
                seg = nseg;
                m = nm;
#pragma unroll
                for (uint32_t i = 0; i < RUN; ++i) ids[i] = nids[i];
            }
        }
    }
    __syncthreads();  // pre / wsum are rewritten by the next phase / chunk
}

template <typename grad_t, uint32_t C, bool POW2, uint32_t GROUP, uint32_t LEAD, uint32_t RUN,
          uint32_t RUN_SAT>
__device__ __forceinline__ void flat_walk_level(
    const grad_t *__restrict__ gl, const float *__restrict__ inputs, const uint32_t *counts,
    const uint16_t *__restrict__ entries, double *acc, uint32_t *pre, uint32_t *wsum,
    uint32_t nb, uint32_t b, uint32_t part, uint32_t P, uint32_t ntiles, uint32_t srows,
    uint32_t lo, uint32_t n, float sc, float half, uint32_t m1, uint32_t m2, uint32_t wm,
    const SliceDyn &dyn, float inv, const Stencil &st, uint32_t *entries_seen) {
    const uint32_t nt = ntiles > part ? ceil_div(ntiles - part, P) : 0u;
    FlatCell<C> cell;
    cell.have = false;
    cell.i0 = 0;
    for (uint32_t cb = 0; cb < nt; cb += kChunkTiles) {
        const uint32_t nc = min(nt - cb, kChunkTiles);
        flat_walk_chunk<grad_t, C, POW2, GROUP, LEAD, RUN, false>(
            cell, gl, inputs, counts, entries, acc, pre, wsum, nb, b, part, P, cb, nc, srows, lo,
            n, sc, half, m1, m2, wm, dyn, inv, st, entries_seen);
        if constexpr (GROUP > 1)
            flat_walk_chunk<grad_t, C, POW2, GROUP, LEAD, RUN_SAT, true>(
                cell, gl, inputs, counts, entries, acc, pre, wsum, nb, b, part, P, cb, nc, srows,
                lo, n, sc, half, m1, m2, wm, dyn, inv, st, entries_seen);
    }
    flat_flush<C, LEAD>(cell, acc, srows, lo, n, m1, m2, wm);
}

template <typename grad_t, uint32_t C, bool POW2, uint32_t GROUP>
__global__ __launch_bounds__(1024) void k_walk_flat(const grad_t *__restrict__ grad,  // [L, GROUP B, C]
                                                    const float *__restrict__ inputs,
                                                    FastLevels fl, BinInfo bi, int align_corners,
                                                    SliceDyn dyn, float inv, uint32_t B,
                                                    uint32_t *counts,
                                                    const uint16_t *__restrict__ entries,
                                                    float *__restrict__ partial, Stencil st) {
    extern __shared__ double acc[];
    __shared__ uint32_t pre[kChunkTiles + 1];
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t sh_b, sh_j, sh_p, sh_entries;
    __shared__ uint32_t tot_s[kMaxBins];
    const uint64_t tr0 = bi.trace ? wall_clock64() : 0;
    const uint32_t nb = bi.nbins, slot = blockIdx.x;
    const uint32_t srows = 1u << bi.shift;
    for (uint32_t i = threadIdx.x; i < srows * C; i += blockDim.x) acc[i] = 0.0;
    if (threadIdx.x == 0) sh_entries = 0;
    walk_plan(bi, counts, tot_s, sh_b, sh_j, sh_p);  // (its barriers cover the zeroing)
    const uint32_t P = sh_p;
    if (P == 0) return;  // uniform
    const uint32_t b = sh_b, part = sh_j;
    uint32_t l = 0;
    while (l + 1 < bi.L && bi.bin0[l + 1] <= b) ++l;
    const uint32_t lo = (b - bi.bin0[l]) << bi.shift;  // slice start, relative to the level
    const uint32_t n = min(srows, bi.rows[l] - lo);
    const uint64_t tr1 = bi.trace ? wall_clock64() : 0;
    const uint32_t M = ge::dyn_count(dyn, B);
    const uint32_t ntiles = ceil_div(M, kTile);
    const grad_t *gl = grad + (size_t)l * GROUP * B * C;
    const float sc = fl.scale[l], half = align_corners ? 0.0f : 0.5f;
    const uint32_t m1 = fl.m1[l], m2 = fl.m2[l], wm = fl.wmask[l], lead = fl.lead[l];
    // entries whose loads are in flight together per lane (and the next
    // batch's ids): 6 keeps the f16 walk within 128 VGPRs (8 spilled)
    constexpr uint32_t RUN = GROUP > 1 ? (uint32_t)DFHIP_WALK_RUN7 : (uint32_t)DFHIP_WALK_RUN;
    constexpr uint32_t RUN_SAT = DFHIP_WALK_RUN_SAT;
#define DFHIP_FLAT(LD)                                                                         \
    flat_walk_level<grad_t, C, POW2, GROUP, LD, RUN, RUN_SAT>(gl, inputs, counts, entries, acc,  \
                                                            pre, wsum, nb, b, part, P, ntiles,   \
                                                            srows, lo, n, sc, half, m1, m2, wm,  \
                                                            dyn, inv, st, &sh_entries)
    if (lead >= 3) DFHIP_FLAT(3);
    else if (lead == 2) DFHIP_FLAT(2);
    else DFHIP_FLAT(1);
#undef DFHIP_FLAT
    __syncthreads();
    float *out = partial + (size_t)slot * ((size_t)srows * C);
    for (uint32_t i = threadIdx.x; i < n * C; i += blockDim.x)
        out[i] = (float)acc[(i % C) * srows + i / C];
    if (bi.trace && threadIdx.x == 0) {  // debug timeline (dfhip_binned_opts.trace)
        uint64_t *r = bi.trace + (size_t)blockIdx.x * 8;
        r[0] = b;
        r[1] = trace_hw_id();
        r[2] = P;
        r[3] = sh_entries;
        r[4] = tr0;
        r[5] = tr1;
        r[6] = part;
        r[7] = wall_clock64();
    }
}

// ---------------------------------------------------------------- 3. sum
// Every call leaves its counts scratch clean: the bin totals, read last by
// the walk plan, are zeroed here (k_sum reads only the plan, which the walk
// rewrites for every bin), so a call with dfhip_binned_opts.kept_clean needs
// no clearing launch before its binning.
__device__ __forceinline__ void clear_totals(const BinInfo &bi, uint32_t *counts) {
    if (!bi.clear_totals) return;
    const uint32_t n = bi.nbins * kTotSplit;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        counts[bi.o_totals + i] = 0u;
}

// Every (row, channel) of the table sums its bin's P_b images (slots
// S_b .. S_b + P_b - 1, recorded by k_walk) in order.
template <typename out_t>
__global__ __launch_bounds__(256) void k_sum(const float *__restrict__ partial, BinInfo bi,
                                             uint32_t C, uint32_t total_rows,
                                             uint32_t *__restrict__ counts,
                                             out_t *__restrict__ out, int accumulate) {
    clear_totals(bi, counts);
    const uint32_t srows = 1u << bi.shift;
    const size_t img = (size_t)srows * C;
    const uint64_t n = (uint64_t)total_rows * C;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t row = (uint32_t)(i / C), ch = (uint32_t)(i - (uint64_t)row * C);
        uint32_t l = 0;
        while (l + 1 < bi.L && bi.base[l + 1] <= row) ++l;
        const uint32_t rel = row - bi.base[l];
        const uint32_t b = bi.bin0[l] + (rel >> bi.shift);
        const uint32_t S = counts[bi.o_plan + 2 * b], P = counts[bi.o_plan + 2 * b + 1];
        const float *src = partial + (size_t)S * img + (size_t)(rel & (srows - 1)) * C + ch;
        double t = 0.0;
        uint32_t p = 0;
        for (; p + 4 <= P; p += 4) {  // parts added in order, four loads in flight
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = src[(size_t)(p + u) * img];
#pragma unroll
            for (int u = 0; u < 4; ++u) t += (double)v[u];
        }
        for (; p < P; ++p) t += (double)src[(size_t)p * img];
        const float s = accumulate ? (float)out[i] : 0.0f;
        out[i] = (out_t)(s + (float)t);
    }
}

// C = 2: one thread per row, both channels as one 8-byte load per image and
// eight images in flight (the same fixed order and f64 sums as k_sum).
template <typename out_t>
__global__ __launch_bounds__(256) void k_sum2(const float *__restrict__ partial, BinInfo bi,
                                              uint32_t total_rows,
                                              uint32_t *__restrict__ counts,
                                              out_t *__restrict__ out, int accumulate) {
    clear_totals(bi, counts);
    const uint32_t srows = 1u << bi.shift;
    const size_t img = (size_t)srows * 2;
    for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < total_rows;
         row += gridDim.x * blockDim.x) {
        uint32_t l = 0;  // the row's level: binary search over the level bases
        static_assert(ge::kMaxLevels <= 64, "the search below reaches level 63 at most");
#pragma unroll
        for (uint32_t step = 32; step > 0; step >>= 1)
            if (l + step < bi.L && bi.base[l + step] <= row) l += step;
        const uint32_t rel = row - bi.base[l];
        const uint32_t b = bi.bin0[l] + (rel >> bi.shift);
        const uint32_t S = counts[bi.o_plan + 2 * b], P = counts[bi.o_plan + 2 * b + 1];
        const float2 *src = reinterpret_cast<const float2 *>(partial + (size_t)S * img +
                                                             (size_t)(rel & (srows - 1)) * 2);
        const size_t step2 = img / 2;
        double t0 = 0.0, t1 = 0.0;
        uint32_t p = 0;
        for (; p + 8 <= P; p += 8) {
            float2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(p + u) * step2];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                t0 += (double)v[u].x;
                t1 += (double)v[u].y;
            }
        }
        for (; p < P; ++p) {
            const float2 v = src[(size_t)p * step2];
            t0 += (double)v.x;
            t1 += (double)v.y;
        }
        const float s0 = accumulate ? (float)out[2 * (size_t)row] : 0.0f;
        const float s1 = accumulate ? (float)out[2 * (size_t)row + 1] : 0.0f;
        out[2 * (size_t)row] = (out_t)(s0 + (float)t0);
        out[2 * (size_t)row + 1] = (out_t)(s1 + (float)t1);
    }
}

// Corner-row wrap mode shared by every level (0 mask, 1 modulo, 2 hash; the
// host restatement of ge::level_ctx / level_rows / row_mode), or kModeAny.
static int uniform_mode(const int32_t *offsets_host, const Levels &lv, uint32_t L, uint32_t D,
                        uint32_t gridtype, bool align) {
    int mode = -1;
    for (uint32_t l = 0; l < L; ++l) {
        const uint64_t hsize = (uint64_t)(offsets_host[l + 1] - offsets_host[l]);
        const uint64_t smul = align ? lv.res[l] : lv.res[l] + 1u;
        uint64_t stride = 1, span = 1;
        for (uint32_t d = 0; d < D; ++d) {
            if (stride <= hsize) {
                stride *= smul;
                span *= smul;
            }
        }
        const bool hashed = gridtype == 0 && stride > hsize;
        const bool pow2 = (hsize & (hsize - 1)) == 0;
        const bool modulo = !pow2 && (hashed || span > hsize);
        const int m = hashed ? 2 : (modulo ? 1 : 0);
        if (mode < 0) mode = m;
        else if (mode != m) return kModeAny;
    }
    return mode == 0 ? 0 : kModeAny;  // only the mask form is specialised
}

// Walk form for mask-form layouts (dfhip_binned_opts.walk_mode: 0 the
// per-segment k_walk, 1 the flat k_walk_flat; A/B runs, tests).  Default:
// flat for stencil groups (textureless step, rocprof: walk 1307 -> 1051 us),
// per-segment for single samples (albedo step: 189 us against 269 flat — one
// entry's work is too short to pay for lanes spread over a part's tiles).
static int flat_walk_mode(uint32_t group, const Opts &op) {
    if (op.walk_mode >= 0) return op.walk_mode;
    return group > 1 ? 1 : 0;
}

template <typename grad_t, uint32_t C, uint32_t GROUP = 1>
static void launch_walk(hipStream_t s, size_t lds, const grad_t *grad, const float *inputs,
                        const int32_t *offsets, const int32_t *offsets_host, const Levels &lv,
                        const BinInfo &bi, uint32_t gridtype, int align, SliceDyn dyn,
                        uint32_t B, uint32_t *counts, const uint16_t *entries, float *partial,
                        const FastLevels *fl, const Opts &op,
                        Stencil st = Stencil{0.0f, 0.0f}) {
    const bool pow2 = ge::dyn_pow2(dyn.bound);
    const float inv = pow2 ? 1.0f / (2.0f * dyn.bound) : 0.0f;
    if constexpr (C == 2) if (fl && flat_walk_mode(GROUP, op)) {
        typedef void (*flat_fn)(const grad_t *, const float *, FastLevels, BinInfo, int,
                                SliceDyn, float, uint32_t, uint32_t *, const uint16_t *,
                                float *, Stencil);
        const flat_fn kf = pow2 ? k_walk_flat<grad_t, C, true, GROUP>
                                : k_walk_flat<grad_t, C, false, GROUP>;
        ensure_dynamic_lds((const void *)kf, (int)kSliceBytes);
        kf<<<bi.G, 1024, lds, s>>>(grad, inputs, *fl, bi, align, dyn, inv, B, counts, entries,
                                   partial, st);
        return;
    }
    // stencil groups are binned by the mask-form fast path only
    const bool m0 = GROUP > 1 || uniform_mode(offsets_host, lv, bi.L, 3, gridtype, align != 0) == 0;
    typedef void (*walk_fn)(const grad_t *, const float *, const int32_t *, Levels, BinInfo,
                            uint32_t, int, SliceDyn, float, uint32_t, uint32_t *,
                            const uint16_t *, float *, Stencil);
    walk_fn kern;
    if constexpr (GROUP > 1) {
        kern = pow2 ? k_walk<grad_t, 3, C, true, 0, GROUP> : k_walk<grad_t, 3, C, false, 0, GROUP>;
    } else {
        if (pow2)
            kern = m0 ? k_walk<grad_t, 3, C, true, 0> : k_walk<grad_t, 3, C, true, kModeAny>;
        else
            kern = m0 ? k_walk<grad_t, 3, C, false, 0> : k_walk<grad_t, 3, C, false, kModeAny>;
    }
    ensure_dynamic_lds((const void *)kern, (int)kSliceBytes);
    kern<<<bi.G, 1024, lds, s>>>(grad, inputs, offsets, lv, bi, gridtype, align, dyn, inv, B,
                                 counts, entries, partial, st);
}

}  // namespace gb
}  // namespace dfhip

using namespace dfhip;

extern "C" int dfhip_grid_backward_binned_scratch_opts(
    uint32_t cap, const int32_t *offsets_host, uint32_t L, uint32_t C, uint32_t group,
    const dfhip_binned_opts *opts, uint64_t *entries_u32, uint64_t *counts_u32,
    uint64_t *partial_f32) {
    gb::Opts op;
    if (!gb::resolve_opts(opts, op)) return DFHIP_EINVAL;
    if (group != 1 && group != 7) {
        set_error("grid_backward_binned_scratch: group must be 1 or 7 (got %u)", group);
        return DFHIP_EINVAL;
    }
    gb::BinInfo bi;
    if (!offsets_host || !gb::make_bins(offsets_host, L, C, cap, group, op, bi)) {
        set_error("grid_backward_binned_scratch: unsupported level layout");
        return DFHIP_EINVAL;
    }
    // single samples and stencil groups tile alike (kTile ids per segment),
    // so one scratch serves both; tile-relative sample ids are u16, counted
    // in u32 words
    if (entries_u32) *entries_u32 = ((uint64_t)bi.tcap * bi.nbins * bi.tile + 1) / 2;
    if (counts_u32) *counts_u32 = gb::counts_words(bi);
    if (partial_f32) *partial_f32 = gb::partial_floats(bi, C);
    return DFHIP_OK;
}

// Samples per binning tile (= id slots per (tile, slice) segment) of a call
// with this group and these options (tests read segments with it).
extern "C" uint32_t dfhip_grid_backward_binned_tile(uint32_t group, const dfhip_binned_opts *opts) {
    gb::Opts op;
    if ((group != 1 && group != 7) || !gb::resolve_opts(opts, op)) return 0;
    return gb::kTile;
}

extern "C" int dfhip_grid_backward_binned_scratch(uint32_t cap, const int32_t *offsets_host,
                                                  uint32_t L, uint32_t C, uint64_t *entries_u32,
                                                  uint64_t *counts_u32, uint64_t *partial_f32) {
    return dfhip_grid_backward_binned_scratch_opts(cap, offsets_host, L, C, 1, nullptr,
                                                   entries_u32, counts_u32, partial_f32);
}

static int binned_backward(const char *name, int phase, int grad_dtype, const void *grad_lbc,
                           const float *inputs, float bound, const int32_t *offsets,
                           const int32_t *offsets_host, float *grad_embeddings, uint32_t B,
                           const int32_t *m_dev, uint32_t D, uint32_t C, uint32_t L, float S,
                           uint32_t H, uint32_t gridtype, int align_corners, uint32_t group,
                           float eps, uint32_t *entries, uint32_t *counts, float *partial,
                           int accumulate, const dfhip_binned_opts *opts, hipStream_t s) {
    gb::Opts op;
    if (!gb::resolve_opts(opts, op)) return DFHIP_EINVAL;
    if (phase < 1 || phase > 3) {
        set_error("%s: phase must be 1 (bin), 2 (walk + sum) or 3 (both), got %d", name, phase);
        return DFHIP_EINVAL;
    }
    if (D != 3 || (C != 1 && C != 2 && C != 4)) {
        set_error("%s: supports D=3 with C in {1,2,4} (got D=%u C=%u)", name, D, C);
        return DFHIP_EINVAL;
    }
    gb::BinInfo bi;
    if (!offsets_host || !gb::make_bins(offsets_host, L, C, B, group, op, bi)) {
        set_error("%s: unsupported level layout", name);
        return DFHIP_EINVAL;
    }
    if (!offsets || !grad_embeddings || !entries || !counts || !partial) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (grad_dtype != DFHIP_F16 && grad_dtype != DFHIP_F32 && grad_dtype != DFHIP_BF16) {
        set_error("%s: grad dtype must be f16, bf16 or f32", name);
        return DFHIP_EDTYPE;
    }
    if (B > 0 && (!grad_lbc || !inputs)) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    const ge::Levels lv = ge::make_levels(L, S, H);
    const ge::SliceDyn dyn{m_dev, bound};
    gb::FastLevels fl;
    const bool fast = gb::make_fast_levels(offsets_host, lv, bi, gridtype, align_corners != 0, fl);
    if (group != 1) {
        if (group != 7 || C != 2 || grad_dtype == DFHIP_F32 || !fast || !(bound > 0.0f) ||
            !(eps >= 0.0f)) {
            set_error("%s: stencil groups need group 7, C = 2, f16 / bf16 gradients, bound > 0, "
                      "eps >= 0 and a mask-form level layout", name);
            return DFHIP_EINVAL;
        }
    }
    const gb::Stencil st{eps, bound};
    bi.clear_totals = 1u;  // every call leaves the totals zero (see clear_totals)
    if (phase & 1) {
        // totals (k_bin adds) and the plan (k_walk sets): cleared here, or
        // kept clean by the previous call's k_sum (the walk writes every
        // bin's plan; with B = 0 no walk runs, so clear anyway)
        if (!op.clean || B == 0)
            (void)hipMemsetAsync(counts + bi.o_totals, 0,
                                 (size_t)(gb::counts_words(bi) - bi.o_totals) * sizeof(uint32_t),
                                 s);
        if (B > 0) {
            const uint32_t gbin = bi.tcap < 4096u ? bi.tcap : 4096u;
            const bool pow2 = ge::dyn_pow2(dyn.bound);
            const float inv = pow2 ? 1.0f / (2.0f * dyn.bound) : 0.0f;
            if (group == 7) {
                if (pow2)
                    gb::k_bin_fast<true, 7><<<gbin, 1024, 0, s>>>(inputs, fl, bi, align_corners,
                                                                   dyn, inv, B, counts,
                                                                   (uint16_t *)entries, st);
                else
                    gb::k_bin_fast<false, 7><<<gbin, 1024, 0, s>>>(inputs, fl, bi, align_corners,
                                                                    dyn, inv, B, counts,
                                                                    (uint16_t *)entries, st);
            } else if (op.fast_bin && fast) {
                if (pow2)
                    gb::k_bin_fast<true><<<gbin, 1024, 0, s>>>(inputs, fl, bi, align_corners,
                                                                dyn, inv, B, counts,
                                                                (uint16_t *)entries);
                else
                    gb::k_bin_fast<false><<<gbin, 1024, 0, s>>>(inputs, fl, bi, align_corners,
                                                                 dyn, inv, B, counts,
                                                                 (uint16_t *)entries);
            } else if (pow2) {
                gb::k_bin<3, true><<<gbin, 1024, 0, s>>>(inputs, offsets, lv, bi, gridtype,
                                                         align_corners, dyn, inv, B, counts,
                                                         (uint16_t *)entries);
            } else {
                gb::k_bin<3, false><<<gbin, 1024, 0, s>>>(inputs, offsets, lv, bi, gridtype,
                                                          align_corners, dyn, inv, B, counts,
                                                          (uint16_t *)entries);
            }
        }
    }
    if (!(phase & 2)) return check_launch(name);
    if (B > 0) {
        const size_t lds = ((size_t)1 << bi.shift) * C * sizeof(double);
        const gb::FastLevels *flp = fast ? &fl : nullptr;
#define DFHIP_WALK(GT, CC)                                                                    \
    gb::launch_walk<GT, CC>(s, lds, (const GT *)grad_lbc, inputs, offsets, offsets_host, lv, \
                            bi, gridtype, align_corners, dyn, B, counts,                     \
                            (const uint16_t *)entries, partial, flp, op)
#define DFHIP_WALK7(GT)                                                                       \
    gb::launch_walk<GT, 2, 7>(s, lds, (const GT *)grad_lbc, inputs, offsets, offsets_host, lv, \
                              bi, gridtype, align_corners, dyn, B, counts,                   \
                              (const uint16_t *)entries, partial, flp, op, st)
        if (group == 7) {
            if (grad_dtype == DFHIP_F16) DFHIP_WALK7(half_t);
            else DFHIP_WALK7(bf16_t);
        } else if (grad_dtype == DFHIP_F16) {
            if (C == 1) DFHIP_WALK(half_t, 1); else if (C == 2) DFHIP_WALK(half_t, 2); else DFHIP_WALK(half_t, 4);
        } else if (grad_dtype == DFHIP_BF16) {
            if (C == 2) DFHIP_WALK(bf16_t, 2);
            else {
                set_error("%s: bf16 gradients are supported for C = 2", name);
                return DFHIP_EINVAL;
            }
        } else {
            if (C == 1) DFHIP_WALK(float, 1); else if (C == 2) DFHIP_WALK(float, 2); else DFHIP_WALK(float, 4);
        }
#undef DFHIP_WALK
#undef DFHIP_WALK7
    }
    // every row is written: rows of bins no walk touched get zero (or keep
    // their value when accumulating)
    const uint32_t total_rows = (uint32_t)offsets_host[L];
    if (C == 2) {
        const uint64_t want = ceil_div<uint64_t>((uint64_t)total_rows, 256);
        gb::k_sum2<float><<<(uint32_t)(want < 8192 ? want : 8192), 256, 0, s>>>(
            partial, bi, total_rows, counts, grad_embeddings, accumulate);
    } else {
        const uint64_t want = ceil_div<uint64_t>((uint64_t)total_rows * C, 256);
        gb::k_sum<float><<<(uint32_t)(want < 4096 ? want : 4096), 256, 0, s>>>(
            partial, bi, C, total_rows, counts, grad_embeddings, accumulate);
    }
    return check_launch(name);
}

extern "C" int dfhip_grid_encode_backward_binned_phase(
    int phase, int grad_dtype, const void *grad_lbc, const float *inputs, float bound,
    const int32_t *offsets, const int32_t *offsets_host, float *grad_embeddings, uint32_t B,
    const int32_t *m_dev, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
    uint32_t gridtype, int align_corners, uint32_t *entries, uint32_t *counts, float *partial,
    int accumulate, dfhip_stream_t stream) {
    return binned_backward("grid_encode_backward_binned", phase, grad_dtype, grad_lbc, inputs,
                           bound, offsets, offsets_host, grad_embeddings, B, m_dev, D, C, L, S,
                           H, gridtype, align_corners, 1, 0.0f, entries, counts, partial,
                           accumulate, nullptr, as_stream(stream));
}

extern "C" int dfhip_grid_encode_backward_binned_stencil(
    int phase, int grad_dtype, const void *grad_lbc, const float *inputs, float bound,
    const int32_t *offsets, const int32_t *offsets_host, float *grad_embeddings, uint32_t B,
    const int32_t *m_dev, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
    uint32_t gridtype, int align_corners, uint32_t group, float eps, uint32_t *entries,
    uint32_t *counts, float *partial, int accumulate, dfhip_stream_t stream) {
    return binned_backward("grid_encode_backward_binned_stencil", phase, grad_dtype, grad_lbc,
                           inputs, bound, offsets, offsets_host, grad_embeddings, B, m_dev, D, C,
                           L, S, H, gridtype, align_corners, group, eps, entries, counts,
                           partial, accumulate, nullptr, as_stream(stream));
}

extern "C" int dfhip_grid_encode_backward_binned_opts(
    int phase, int grad_dtype, const void *grad_lbc, const float *inputs, float bound,
    const int32_t *offsets, const int32_t *offsets_host, float *grad_embeddings, uint32_t B,
    const int32_t *m_dev, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
    uint32_t gridtype, int align_corners, uint32_t group, float eps, uint32_t *entries,
    uint32_t *counts, float *partial, int accumulate, const dfhip_binned_opts *opts,
    dfhip_stream_t stream) {
    return binned_backward("grid_encode_backward_binned", phase, grad_dtype, grad_lbc, inputs,
                           bound, offsets, offsets_host, grad_embeddings, B, m_dev, D, C, L, S,
                           H, gridtype, align_corners, group, eps, entries, counts, partial,
                           accumulate, opts, as_stream(stream));
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
