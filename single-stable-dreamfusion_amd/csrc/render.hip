// Fused persistent inference renderer for gfx950: occupancy-grid march +
// tiled-grid gather + sigma MLP (MFMA) + front-to-back compositing of the
// albedo field in ONE launch with a device work queue of rays.
//
// Behavioural spec: the reference's inference branch of run_cuda
// (nerf/renderer.py:496-532): a host loop of
//   march_rays (raymarching.cu:700-804) -> network_grid.common_forward
//   (network_grid.py:76-87, under fp16 autocast) -> composite_rays
//   (raymarching.cu:818-905) -> rays_alive compaction (one host sync)
// for up to max_steps / n_step iterations.  The per-ray arithmetic is the
// same sequence of operations, instruction for instruction:
//   * the march is rm::march_next, the reference loop in register form;
//   * the field is fm::grid_features + fm::forward_tile, the kernels the
//     train path and the eval loop run (f16 per-corner accumulation, f16
//     activations, f32 MFMA accumulators, expf density, f16 albedo);
//   * compositing is k_composite_infer's: T = 1 - sum(w), alpha =
//     1 - __expf(-sigma dt), t (relative to the near plane's rays_t) summed
//     from deltas[1], the T < T_thresh break.
// The loop restarts each ray's march from the composited t (rays_t = near +
// the f32 sum of deltas[1]) at iteration boundaries, and the boundaries come
// from a global schedule (n_step = clamp(N / n_alive, 1, 8)).  This kernel
// restarts after every sample, i.e. it is the loop with n_step = 1, which is
// the reference's own schedule while more than half the rays are alive, and
// is bit-identical to it (same samples, same compositing, and the loop's
// max_steps iterations become at most max_steps samples per ray).  Under a
// larger n_step the loop continues from the march's own t inside an
// iteration; the two agree except where near + sum(t_i - last_t) != t in
// f32 (a rounding of the difference after an empty-space jump), a 1-ulp
// shift of the following samples (tests: bit-exact vs n_step = 1, 1e-4 vs
// the default schedule).
//
// MI355X design:
//  * one lane owns one ray; a wave runs 64 rays.  The march runs AHEAD of the
//    field: every iteration each lane takes one march step (up to kAhead
//    grid cells, their occupancy bytes loaded together,
//    rm::march_step_ahead) and stages the sample it finds in a per-wave LDS batch
//    (slot = ballot / mbcnt, no atomics), up to kK (8) pending samples per
//    ray, until the batch holds kBatch (64) samples or no lane may march
//    (kK 4 -> 8: 2.86 -> 2.73 ms per frame; batches of 48-128 the same).  Lanes
//    do not wait for the wave's slowest ray between samples (the previous
//    form marched up to 4 samples per lane per round, so every round lasted
//    as long as the lane with the longest empty-space run: the march was
//    0.62 of the wave cycles; now 0.41, 4.07 -> 3.0 ms per 800x800 frame).
//  * the batch is then evaluated as 16-sample MFMA tiles, two tiles per pass
//    (lane group h gathers levels h, h+4, h+8, h+12 of a tile's sample; both
//    tiles' gathers are issued before either MLP), and each lane composites
//    its pending samples in order.  A ray retires on T < T_thresh,
//    max_samples or far; samples it marched past its termination are dropped
//    (~1 % extra field work), so the outputs are the loop's.
//  * persistent waves + one global atomic per refill: a lane whose ray
//    terminated takes the next ray id (ballot / mbcnt), so there is no host
//    loop, no compaction, no per-iteration sync, and the xyzs / dirs /
//    deltas / sigma / rgb intermediates never touch HBM.  Every ray id
//    taken is finished before its wave exits, so each output is written
//    exactly once (no zero-fill).
#include "march_common.h"
#include <type_traits>
#include "field_common.h"

namespace dfhip {
namespace rd {

constexpr int kWaves = 4;
#ifndef DFHIP_RENDER_K
#define DFHIP_RENDER_K 8
#endif
#ifndef DFHIP_RENDER_BATCH
#define DFHIP_RENDER_BATCH 64
#endif
constexpr int kK = DFHIP_RENDER_K;          // samples a ray may have pending per batch
constexpr int kBatch = DFHIP_RENDER_BATCH;  // a batch closes at >= kBatch staged samples
#ifndef DFHIP_RENDER_TPP
#define DFHIP_RENDER_TPP 2
#endif
constexpr int kTPP = DFHIP_RENDER_TPP;  // field tiles per pass
// empty cells a lane checks per march iteration (rm::march_step_ahead): their
// occupancy bytes load together.  K = 2: 1.830 -> 1.776 ms per frame (R0),
// 2.005 -> 1.963 (R1); K = 3 / 4 lose to the discarded candidates' work in
// occupied space (profiles/r06/c4_march_ahead_ab.txt)
#ifndef DFHIP_RENDER_AHEAD
#define DFHIP_RENDER_AHEAD 2
#endif
constexpr int kAhead = DFHIP_RENDER_AHEAD;
// pending slots, 8 bits each: one u64 holds 8, a second one up to 16
static_assert(kK >= 1 && kK <= 16, "kK: 1..16 pending samples");
struct PendSlots {
    uint64_t lo = 0, hi = 0;
    __device__ __forceinline__ void put(uint32_t i, uint32_t slot) {
        if (kK <= 8 || i < 8) lo |= (uint64_t)slot << (8 * (i & 7));
        else hi |= (uint64_t)slot << (8 * (i & 7));
    }
    __device__ __forceinline__ uint32_t get(uint32_t i) const {
        const uint64_t w = (kK <= 8 || i < 8) ? lo : hi;
        return (uint32_t)(w >> (8 * (i & 7))) & 0xFFu;
    }
};
constexpr int kSlots = kBatch + 64; // per-wave staged samples (< 64 added after the last check)
static_assert(kSlots <= 256, "PendSlots keeps LDS slot numbers in 8 bits: DFHIP_RENDER_BATCH <= 192");

// Per-wave LDS staging of one batch of samples, in the order the lanes found
// them.  pos holds the sample position until the field has read it, then
// (sigma, rgb as f16).
struct Stage {
    float pos[kSlots * 3];
    float dt[kSlots];
    float tc[kSlots];  // rays_t after the sample (the depth weight's t)
};

// Ray j of queue chunk ch: 2^cl consecutive ray ids, or with tile_w (the
// width of a row-major image; cl = 6) pixel (j / 8, j % 8) of the image's
// 8 x 8 tile ch (tiles row-major).  A tile's rays stay closer in 3-D than a
// 64-pixel row strip's, so a wave's field gathers share more cache lines.
__device__ __forceinline__ uint32_t chunk_ray(uint32_t ch, uint32_t j, uint32_t cl,
                                              uint32_t tile_w) {
    if (!tile_w) return (ch << cl) + j;
    const uint32_t tw = tile_w >> 3, ty = ch / tw, tx = ch - ty * tw;
    return ((ty << 3) + (j >> 3)) * tile_w + (tx << 3) + (j & 7u);
}

__device__ __forceinline__ uint32_t pack_h2(half_t a, half_t b) {
    uint16_t ua, ub;
    __builtin_memcpy(&ua, &a, 2);
    __builtin_memcpy(&ub, &b, 2);
    return (uint32_t)ua | ((uint32_t)ub << 16);
}
__device__ __forceinline__ float lo_h(uint32_t v) {
    const uint16_t u = (uint16_t)(v & 0xFFFFu);
    half_t h;
    __builtin_memcpy(&h, &u, 2);
    return (float)h;
}
__device__ __forceinline__ float hi_h(uint32_t v) {
    const uint16_t u = (uint16_t)(v >> 16);
    half_t h;
    __builtin_memcpy(&h, &u, 2);
    return (float)h;
}

// 3 waves per SIMD (<= 170 VGPRs): the register count sits at that
// boundary, and one more wave per SIMD is worth ~6 % of the frame
__global__ __launch_bounds__(256, 3) void k_render_infer(
    uint32_t N, const float *__restrict__ rays_o, const float *__restrict__ rays_d,
    const float *__restrict__ nears, const float *__restrict__ fars,
    const float *__restrict__ noises, rm::MarchConsts k, const uint8_t *__restrict__ grid,
    uint32_t max_samples, float T_thresh, const half_t *__restrict__ table,
    const int32_t *__restrict__ offsets, ge::Levels lv, uint32_t gridtype, int align_corners,
    const float *w1, const float *b1, const float *w2, const float *b2, const float *w3,
    const float *b3, float *__restrict__ weights_sum, float *__restrict__ depth,
    float *__restrict__ image, uint32_t *__restrict__ work,
    const fm::u32x4 *__restrict__ quads, uint64_t *prof, const int32_t *__restrict__ order,
    uint32_t chunk_log2, uint32_t tile_w) {
    __shared__ fm::Weights W;
    __shared__ fm::LevelK LK[fm::kLevels];
    __shared__ Stage stages[kWaves];
    const bool align = align_corners != 0;
    fm::load_weights<true>(W, nullptr, w1, b1, w2, b2, w3, b3);
    fm::stage_levels(LK, offsets, lv, gridtype, align);
    __syncthreads();
    Stage &S = stages[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63, c = lane & 15, h = lane >> 4;
    const float inv_extent = 1.0f / (2.0f * k.bound);
    // queue positions: N, or whole chunks of the order
    const uint32_t nchunks = ceil_div(N, 1u << chunk_log2);
    const uint32_t Nq = order ? nchunks << chunk_log2 : N;
    // mirrored halves: in blocks of G chunk positions (G = the grid's waves,
    // so that the first grab of every wave falls in the first block), grab g
    // takes the first half of chunk g and the second half of chunk G-1-g
    // (none for single-ray chunks)
    const uint32_t G = order && chunk_log2 ? gridDim.x * kWaves : 0u;

    int ray = -1;
    bool exhausted = false;
    rm::Ray r{};
    // march state: t, last_t (the march loop's), tc (rays_t: near + the f32
    // sum of deltas[1], where the loop restarts after every sample), whether
    // the march reached far, and the samples marched for this ray
    float t = 0.0f, far = 0.0f, last_t = 0.0f, tc = 0.0f;
    bool at_far = false;
    uint32_t marched = 0;
    // compositing state
    float ws = 0.0f, dp = 0.0f, cr = 0.0f, cg = 0.0f, cb = 0.0f;
    uint32_t taken = 0;
    bool finished = false;  // T < T_thresh or max_samples: later samples are dropped
    uint32_t samples = 0;   // per-lane count of evaluated samples (stats)
    // debug phase profile (dfhip_render_rays_infer_prof): cycles of refill,
    // march, field and compositing, rounds and field tiles, per wave
    uint64_t pc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t c0 = prof ? clock64() : 0;
    const uint64_t w0 = prof ? wall_clock64() : 0;
    bool dry = false;  // this wave has seen the queue empty (prof)
    uint64_t wdry = 0;     // ... since (wall clock), holding held_dry rays
    uint32_t held_dry = 0;
    uint32_t max_marched = 0, max_taken = 0, retired = 0;  // prof records

    while (true) {
        // ---- refill lanes without a ray from the global queue
        const bool need = ray < 0 && !exhausted;
        const uint64_t needm = __ballot(need);
        if (needm) {
            const int leader = __ffsll((unsigned long long)needm) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(&work[0], (uint32_t)__popcll(needm));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
                const uint32_t q = base + rank;
                // the queue's q-th ray: ray q, or ray r of chunk order[q >> cl]
                // (chunks of 2^cl consecutive rays, the costly ones first, so
                // that they do not finish alone after the queue ran dry); an id
                // >= N (the partial last chunk, or an order entry that is not a
                // chunk index: checked before the shift, which could wrap it
                // onto a valid chunk) is skipped, never read or written
                uint32_t id = N;
                if (q < Nq) {
                    if (order) {
                        const uint32_t j = q & ((1u << chunk_log2) - 1u);
                        uint32_t pos = q >> chunk_log2;
                        if (G && (j >> (chunk_log2 - 1))) {
                            const uint32_t base = pos / G * G;
                            pos = base + min(G, nchunks - base) - 1u - (pos - base);
                        }
                        const uint32_t ch = (uint32_t)order[pos];
                        if (ch < nchunks) id = chunk_ray(ch, j, chunk_log2, tile_w);
                    } else {
                        id = q;
                    }
                }
                if (q >= Nq) {
                    exhausted = true;
                } else if (id < N) {
                    ray = (int)id;
                    r = rm::load_ray(rays_o + 3 * (size_t)id, rays_d + 3 * (size_t)id);
                    // rays_t starts at the near plane (renderer.py:509); the
                    // perturbation applies to the first march only (:522)
                    tc = nears[id];
                    far = fars[id];
                    t = tc;
                    if (noises)
                        t = fmaf(rm::clampf(t * k.dt_gamma, k.dt_min, k.dt_max), noises[id], t);
                    last_t = t;
                    at_far = false;
                    marched = 0;
                    ws = dp = cr = cg = cb = 0.0f;
                    taken = 0;
                    finished = false;
                }
            }
            if (prof && !dry && __ballot(exhausted)) {  // uniform
                dry = true;
                wdry = wall_clock64();
                held_dry = (uint32_t)__popcll(__ballot(ray >= 0)) | (uint32_t)(pc[4] << 8);
                if (lane == 0) atomicMin((unsigned long long *)&prof[7], (unsigned long long)wdry);
            }
        }
        // done when no lane holds a ray and the queue is dry for all (a lane
        // whose queue entry was skipped refills next round)
        if (__ballot(ray >= 0 || !exhausted) == 0) break;
        if (prof) {
            const uint64_t c1 = clock64();
            pc[0] += c1 - c0;
            c0 = c1;
            pc[4] += 1;
        }

        // ---- march ahead: every lane takes one march step (one cell) per
        // iteration and stages each sample it finds, until the wave has a
        // batch of kBatch samples or no lane may march (at far, kK samples
        // pending, or max_samples marched).  Lanes do not wait for the
        // slowest ray of the wave between samples; the staged samples are the
        // loop's (after each sample the march restarts from rays_t, as
        // raymarching.cu:739-748 at n_step = 1), so marching past a ray's
        // termination only adds samples that the compositing drops.
        uint32_t count = 0, npend = 0;
        PendSlots pslots;  // slots of the pending samples
        while (true) {
            const bool can = ray >= 0 && !at_far && !finished && npend < (uint32_t)kK &&
                             marched < max_samples;
            if (__ballot(can) == 0) break;
            bool emit = false;
            float px[3], pdt = 0.0f, dl = 0.0f;
            if (can) {
                const int st =
                    rm::march_step_ahead<kAhead>(k, r, grid, t, last_t, far, px, pdt, dl);
                if (st == 2) {
                    at_far = true;
                } else if (st == 1) {
                    emit = true;
                    tc += dl;
                    t = tc;
                    last_t = tc;
                    ++marched;
                }
            }
            const uint64_t em = __ballot(emit);
            if (emit) {
                const uint32_t slot =
                    count + __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
                S.pos[3 * slot] = px[0];
                S.pos[3 * slot + 1] = px[1];
                S.pos[3 * slot + 2] = px[2];
                S.dt[slot] = pdt;
                S.tc[slot] = tc;
                pslots.put(npend, slot);
                ++npend;
            }
            count += (uint32_t)__popcll(em);
            if (count >= (uint32_t)kBatch) break;
        }
        fm::wave_lds_sync();
        if (prof) {
            const uint64_t c1 = clock64();
            pc[1] += c1 - c0;
            c0 = c1;
        }

        // ---- field over the staged samples, 16 per MFMA tile
        const uint32_t total = count;
        const uint32_t tiles = ceil_div(total, 16u);
        if (prof) pc[5] += tiles;
        // kTPP tiles per pass: their table gathers are issued before any MLP
        // waits on them (more loads in flight per lane)
        for (uint32_t tile = 0; tile < tiles; tile += kTPP) {
            float x[kTPP][3], x01[kTPP][3];
            bool valid[kTPP];
            fm::half8 xb[kTPP];
#pragma unroll
            for (int u = 0; u < kTPP; ++u) {
                const uint32_t s = (tile + u) * 16 + c;
                valid[u] = s < total;
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    x[u][d] = valid[u] ? S.pos[3 * s + d] : 0.0f;
                    x01[u][d] = valid[u] ? (x[u][d] + k.bound) * inv_extent : -1.0f;
                }
            }
#pragma unroll
            for (int u = 0; u < kTPP; ++u)
                xb[u] = quads ? fm::grid_features<half_t, true>(table, LK, align, x01[u], h, quads)
                              : fm::grid_features(table, LK, align, x01[u], h);
#pragma unroll
            for (int u = 0; u < kTPP; ++u) {
                if (u > 0 && tile + u >= tiles) break;  // uniform
                const uint32_t s = (tile + u) * 16 + c;
                fm::Fwd F;
                fm::forward_tile(W, xb[u], c, h, F);
                if (valid[u]) {
                    // k_field_fwd_fused's heads (f16-rounded outputs, f32 density),
                    // lane group h on output h: the density into word 3 s, albedo
                    // channel q = h - 1 into half q of words 3 s + 1, 3 s + 2
                    if (h == 0) {
                        S.pos[3 * s] = expf((float)(half_t)F.o[0] + fm::gaussian(x[u]));
                    } else {
                        const float v = (float)(half_t)F.o[0];
                        const half_t a = (half_t)(1.0f / (1.0f + expf(-v)));
                        if (h == 3)
                            S.pos[3 * s + 2] = __uint_as_float(pack_h2(a, (half_t)0.0f));
                        else
                            reinterpret_cast<half_t *>(S.pos + 3 * s + 1)[h - 1] = a;
                    }
                }
            }
        }
        fm::wave_lds_sync();
        if (prof) {
            const uint64_t c1 = clock64();
            pc[2] += c1 - c0;
            c0 = c1;
        }

        // ---- composite each ray's staged samples in order (k_composite_infer,
        // raymarching.cu:848-873); a ray retires on T < T_thresh or
        // max_samples, or when its march reached far with nothing pending
        if (ray >= 0) {
            for (uint32_t q = 0; q < npend && !finished; ++q) {
                const uint32_t slot = pslots.get(q);
                const float sigma = S.pos[3 * slot];
                const uint32_t rg = __float_as_uint(S.pos[3 * slot + 1]);
                const uint32_t bz = __float_as_uint(S.pos[3 * slot + 2]);
                const float alpha = 1.0f - __expf(-sigma * S.dt[slot]);
                const float T = 1.0f - ws;
                const float w = alpha * T;
                ws += w;
                dp = fmaf(w, S.tc[slot], dp);
                cr = fmaf(w, lo_h(rg), cr);
                cg = fmaf(w, hi_h(rg), cg);
                cb = fmaf(w, lo_h(bz), cb);
                ++taken;
                ++samples;
                if (T < T_thresh || taken >= max_samples) finished = true;
            }
            if (finished || at_far || marched >= max_samples) {
                weights_sum[ray] = ws;
                depth[ray] = dp;
                image[3 * (size_t)ray] = cr;
                image[3 * (size_t)ray + 1] = cg;
                image[3 * (size_t)ray + 2] = cb;
                ray = -1;
                if (prof) {
                    max_marched = max(max_marched, marched);
                    max_taken = max(max_taken, taken);
                    ++retired;
                }
            }
        }
        fm::wave_lds_sync();
        if (prof) {
            const uint64_t c1 = clock64();
            pc[3] += c1 - c0;
            c0 = c1;
        }
    }
    uint32_t tot = samples;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off);
    if (prof) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            max_marched = max(max_marched, (uint32_t)__shfl_xor(max_marched, off));
            max_taken = max(max_taken, (uint32_t)__shfl_xor(max_taken, off));
            retired += __shfl_xor(retired, off);
        }
    }
    if (prof && lane == 0) {
#pragma unroll
        for (int i = 0; i < 6; ++i) atomicAdd((unsigned long long *)&prof[i], pc[i]);
        const uint64_t w1 = wall_clock64();
        atomicMin((unsigned long long *)&prof[6], (unsigned long long)w0);
        atomicMax((unsigned long long *)&prof[8], (unsigned long long)w1);
        atomicAdd((unsigned long long *)&prof[9], (unsigned long long)(w1 - w0));
        // the per-wave record (prof[10] = records wanted)
        const uint64_t gw = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
        if (gw < prof[10]) {
            uint64_t *rec = prof + 16 + 16 * gw;
            rec[0] = w0;
            rec[1] = wdry;
            rec[2] = w1;
            rec[3] = (pc[4] << 32) | held_dry;
            rec[4] = max_marched;
            rec[5] = tot;
            rec[6] = max_taken;
            rec[7] = retired;
            for (int i = 0; i < 6; ++i) rec[8 + i] = pc[i];
        }
    }
    // stats: composited samples (64-bit, low / high words)
    if (lane == 0 && tot) {
        const uint32_t old = atomicAdd(&work[1], tot);
        if (old + tot < old) atomicAdd(&work[2], 1u);
    }
}

}  // namespace rd
}  // namespace dfhip

using namespace dfhip;

static int render_infer(
    uint32_t N, const float *rays_o, const float *rays_d, const float *nears, const float *fars,
    const float *noises, float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
    uint32_t H, const uint8_t *grid, float T_thresh, const void *table, const int32_t *offsets,
    uint32_t L, float S, uint32_t base_res, uint32_t gridtype, int align_corners,
    const float *w1, const float *b1, const float *w2, const float *b2, const float *w3,
    const float *b3, float *weights_sum, float *depth, float *image, uint32_t *work,
    const void *quads, uint64_t *prof, const int32_t *order, uint32_t chunk_log2,
    uint32_t tile_w, dfhip_stream_t stream) {
    const char *name = "render_rays_infer";
    if (order && tile_w && (chunk_log2 != 6 || tile_w % 8 || N % (8 * tile_w))) {
        set_error("%s: tile chunks need chunk_log2 6, tile_w a multiple of 8 and N of 8 tile_w "
                  "(got chunk_log2 %u, tile_w %u, N %u)", name, chunk_log2, tile_w, N);
        return DFHIP_EINVAL;
    }
    if (order && (chunk_log2 > 16 || N > 0xFFFFFFFFu - (1u << chunk_log2))) {
        set_error("%s: chunk_log2 must be <= 16 and N + 2^chunk_log2 < 2^32 (got %u, N=%u)",
                  name, chunk_log2, N);
        return DFHIP_EINVAL;
    }
    if (L != 16) {
        set_error("%s: the fused renderer supports the reference's 16-level x 2-channel 3-D "
                  "grid (got L=%u)", name, L);
        return DFHIP_EINVAL;
    }
    if (C < 1 || C > 16 || H < 2 || H > 1024 || max_steps == 0 || !(bound > 0.0f)) {
        set_error("%s: invalid C=%u H=%u max_steps=%u bound=%g", name, C, H, max_steps,
                  (double)bound);
        return DFHIP_EINVAL;
    }
    if (!rays_o || !rays_d || !nears || !fars || !grid || !table || !offsets || !w1 || !b1 ||
        !w2 || !b2 || !w3 || !b3 || !weights_sum || !depth || !image || !work) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(work, 0, 4 * sizeof(uint32_t), s) != hipSuccess) return check_launch(name);
    if (N == 0) return DFHIP_OK;
    const rm::MarchConsts k = rm::make_consts(bound, dt_gamma, max_steps, C, H);
    const ge::Levels lv = ge::make_levels(L, S, base_res);
    // persistent waves: as many workgroups as are co-resident on the chip
    // (occupancy query, cached per device); the queue balances the rays
    const uint32_t resident =
        resident_blocks((const void *)rd::k_render_infer, 64 * rd::kWaves, 2);
    const uint32_t want = ceil_div(N, 64u * rd::kWaves);
    const uint32_t blocks = want < resident ? want : resident;
    rd::k_render_infer<<<blocks, 64 * rd::kWaves, 0, s>>>(
        N, rays_o, rays_d, nears, fars, noises, k, grid, max_steps, T_thresh,
        (const half_t *)table, offsets, lv, gridtype, align_corners, w1, b1, w2, b2, w3, b3,
        weights_sum, depth, image, work, (const fm::u32x4 *)quads, prof, order, chunk_log2,
        tile_w);
    return check_launch(name);
}

extern "C" int dfhip_render_rays_infer(
    uint32_t N, const float *rays_o, const float *rays_d, const float *nears, const float *fars,
    const float *noises, float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
    uint32_t H, const uint8_t *grid, float T_thresh, const void *table, const int32_t *offsets,
    uint32_t L, float S, uint32_t base_res, uint32_t gridtype, int align_corners,
    const float *w1, const float *b1, const float *w2, const float *b2, const float *w3,
    const float *b3, float *weights_sum, float *depth, float *image, uint32_t *work,
    const void *quads, dfhip_stream_t stream) {
    return render_infer(N, rays_o, rays_d, nears, fars, noises, bound, dt_gamma, max_steps, C, H,
                        grid, T_thresh, table, offsets, L, S, base_res, gridtype, align_corners,
                        w1, b1, w2, b2, w3, b3, weights_sum, depth, image, work, quads, nullptr,
                        nullptr, 0, 0, stream);
}

extern "C" int dfhip_render_rays_infer_prof(
    uint32_t N, const float *rays_o, const float *rays_d, const float *nears, const float *fars,
    const float *noises, float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
    uint32_t H, const uint8_t *grid, float T_thresh, const void *table, const int32_t *offsets,
    uint32_t L, float S, uint32_t base_res, uint32_t gridtype, int align_corners,
    const float *w1, const float *b1, const float *w2, const float *b2, const float *w3,
    const float *b3, float *weights_sum, float *depth, float *image, uint32_t *work,
    const void *quads, uint64_t *prof, dfhip_stream_t stream) {
    return render_infer(N, rays_o, rays_d, nears, fars, noises, bound, dt_gamma, max_steps, C, H,
                        grid, T_thresh, table, offsets, L, S, base_res, gridtype, align_corners,
                        w1, b1, w2, b2, w3, b3, weights_sum, depth, image, work, quads, prof,
                        nullptr, 0, 0, stream);
}

extern "C" int dfhip_render_rays_infer_ordered(
    uint32_t N, const float *rays_o, const float *rays_d, const float *nears, const float *fars,
    const float *noises, float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
    uint32_t H, const uint8_t *grid, float T_thresh, const void *table, const int32_t *offsets,
    uint32_t L, float S, uint32_t base_res, uint32_t gridtype, int align_corners,
    const float *w1, const float *b1, const float *w2, const float *b2, const float *w3,
    const float *b3, float *weights_sum, float *depth, float *image, uint32_t *work,
    const void *quads, const int32_t *order, uint32_t chunk_log2, uint32_t tile_w,
    uint64_t *prof, dfhip_stream_t stream) {
    return render_infer(N, rays_o, rays_d, nears, fars, noises, bound, dt_gamma, max_steps, C, H,
                        grid, T_thresh, table, offsets, L, S, base_res, gridtype, align_corners,
                        w1, b1, w2, b2, w3, b3, weights_sum, depth, image, work, quads, prof,
                        order, chunk_log2, tile_w, stream);
}

// ---------------------------------------------------------------- queue order
namespace dfhip {
namespace rd {

constexpr uint32_t kMaxOrderChunks = 16384;  // one workgroup's counting sort (256 blocks of 64)

// Cost of each chunk of 2^cl consecutive rays: the summed squared distance
// of the rays' lines from the scene centre (the origin of the reference's
// bound box).  One wave per chunk.
__global__ __launch_bounds__(256) void k_chunk_cost(const float *__restrict__ rays_o,
                                                    const float *__restrict__ rays_d, uint32_t N,
                                                    uint32_t cl, uint32_t nchunks,
                                                    float *__restrict__ cost, uint32_t tile_w) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ch = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (ch >= nchunks) return;  // uniform per wave
    const uint32_t r0 = ch << cl, r1 = min(N, (ch + 1) << cl);
    float acc = 0.0f;
    for (uint32_t j = lane; j < r1 - r0; j += 64) {
        const uint32_t r = chunk_ray(ch, j, cl, tile_w);
        const float ox = rays_o[3 * (size_t)r], oy = rays_o[3 * (size_t)r + 1],
                    oz = rays_o[3 * (size_t)r + 2];
        const float dx = rays_d[3 * (size_t)r], dy = rays_d[3 * (size_t)r + 1],
                    dz = rays_d[3 * (size_t)r + 2];
        const float dd = fmaxf(dx * dx + dy * dy + dz * dz, 1e-20f);
        const float t = -(ox * dx + oy * dy + oz * dz) / dd;
        const float px = fmaf(t, dx, ox), py = fmaf(t, dy, oy), pz = fmaf(t, dz, oz);
        acc += px * px + py * py + pz * pz;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    // a partial last chunk: the mean over its rays, scaled to a whole chunk
    if (lane == 0) cost[ch] = acc * (float)(1u << cl) / (float)(r1 - r0);
}

// The same chunks' cost from the occupancy grid: minus the occupied cells
// found at kOccProbes evenly spaced points of each ray's [near, far) (the
// bitfield the march reads, level of each point as the march takes it at
// dt_min), so that the rays crossing the most occupied space come first.
constexpr uint32_t kOccProbes = 16;
__global__ __launch_bounds__(256) void k_chunk_cost_occ(
    const float *__restrict__ rays_o, const float *__restrict__ rays_d,
    const float *__restrict__ nears, const float *__restrict__ fars,
    const uint8_t *__restrict__ grid, rm::MarchConsts k, uint32_t N, uint32_t cl,
    uint32_t nchunks, float *__restrict__ cost, uint32_t tile_w) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ch = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (ch >= nchunks) return;  // uniform per wave
    const uint32_t r0 = ch << cl, r1 = min(N, (ch + 1) << cl);
    uint32_t occ = 0;
    for (uint32_t j = lane; j < r1 - r0; j += 64) {
        const uint32_t r = chunk_ray(ch, j, cl, tile_w);
        const float n0 = nears[r], f0 = fars[r];
        if (!(f0 > n0)) continue;  // a ray missing the box
        const float ox = rays_o[3 * (size_t)r], oy = rays_o[3 * (size_t)r + 1],
                    oz = rays_o[3 * (size_t)r + 2];
        const float dx = rays_d[3 * (size_t)r], dy = rays_d[3 * (size_t)r + 1],
                    dz = rays_d[3 * (size_t)r + 2];
        const float step = (f0 - n0) / (float)kOccProbes;
#pragma unroll 4
        for (uint32_t i = 0; i < kOccProbes; ++i) {
            const float t = fmaf((float)i + 0.5f, step, n0);
            const float x = rm::clampf(fmaf(t, dx, ox), -k.bound, k.bound);
            const float y = rm::clampf(fmaf(t, dy, oy), -k.bound, k.bound);
            const float z = rm::clampf(fmaf(t, dz, oz), -k.bound, k.bound);
            const rm::Mip m = rm::mip_of(k, x, y, z, k.dt_min);
            const uint32_t idx = rm::grid_index(k, m.level, rm::cell_of(k, x, m.rbound),
                                                rm::cell_of(k, y, m.rbound),
                                                rm::cell_of(k, z, m.rbound));
            occ += (grid[idx >> 3] >> (idx & 7)) & 1u;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) occ += __shfl_xor(occ, off);
    if (lane == 0) cost[ch] = -(float)occ * (float)(1u << cl) / (float)(r1 - r0);
}

// The chunks by ascending cost, quantised to kOrderBuckets levels between the
// costs' min and max (NaN last), ties by chunk index: a stable counting sort
// in one workgroup of 16 waves.  The chunks are taken in blocks of 64, one per
// lane: six ballots over the bucket's bits give every lane the lanes of its
// block with the same bucket, hence its rank among them and the block's count
// per bucket (no LDS atomics, no serial per-thread ranges); the counts are
// scanned over blocks by 16 parts of 64 threads (one per bucket), the bucket
// totals over buckets by one wave, and each lane writes its chunk at bucket
// base + block offset + rank.  (The previous form: 256 threads with a serial
// 256-step scan per bucket, 25 us per frame; a full bitonic sort of 16 k keys
// in one workgroup took 229 us; a queue order needs only the coarse rank.)
constexpr uint32_t kOrderBuckets = 64;
constexpr uint32_t kOrderThreads = 1024;
constexpr uint32_t kOrderWaves = kOrderThreads / 64;
constexpr uint32_t kOrderBlocks = kMaxOrderChunks / 64;  // 64-chunk blocks
static_assert(kOrderBuckets == 64, "the ballot rank takes six bucket bits");
__global__ __launch_bounds__(kOrderThreads) void k_chunk_order(const float *__restrict__ cost,
                                                               uint32_t nchunks,
                                                               int32_t *__restrict__ order) {
    __shared__ uint8_t bk[kMaxOrderChunks];                     // each chunk's bucket
    __shared__ uint16_t cnt[kOrderBlocks * kOrderBuckets];      // [block][bucket]: count, then offset
    __shared__ uint32_t part[kOrderWaves * kOrderBuckets];      // [part][bucket] sums, then offsets
    __shared__ uint32_t base[kOrderBuckets];
    __shared__ float rmin[kOrderWaves], rmax[kOrderWaves];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t nblk = ceil_div(nchunks, 64u);
    // the costs once, coalesced: range, then every chunk's bucket into LDS
    float lo = INFINITY, hi = -INFINITY;
    for (uint32_t c = t; c < nchunks; c += kOrderThreads) {
        const float v = cost[c];
        if (v == v) {
            lo = fminf(lo, v);
            hi = fmaxf(hi, v);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, o));
        hi = fmaxf(hi, __shfl_xor(hi, o));
    }
    if (lane == 0) {
        rmin[wave] = lo;
        rmax[wave] = hi;
    }
    __syncthreads();
    lo = rmin[0];
    hi = rmax[0];
    for (uint32_t w = 1; w < kOrderWaves; ++w) {
        lo = fminf(lo, rmin[w]);
        hi = fmaxf(hi, rmax[w]);
    }
    const float cmin = lo, span = hi - lo;
    const float scale = span > 0.0f ? (float)kOrderBuckets / span : 0.0f;
    for (uint32_t c = t; c < nchunks; c += kOrderThreads) {
        const float v = cost[c];
        uint32_t b = kOrderBuckets - 1;  // NaN last
        if (v == v) {
            const float q = (v - cmin) * scale;
            b = q >= (float)(kOrderBuckets - 1) ? kOrderBuckets - 1 : (uint32_t)fmaxf(q, 0.0f);
        }
        bk[c] = (uint8_t)b;
    }
    __syncthreads();
    // per 64-chunk block: each lane's rank among the block's chunks of its
    // bucket (lanes below it with the same six bits) and the block's counts
    auto same_bucket = [&](uint32_t b, bool valid) {
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const uint64_t bal = __ballot(valid && ((b >> i) & 1u));
            m &= ((b >> i) & 1u) ? bal : ~bal;
        }
        return m;
    };
    for (uint32_t k = wave; k < nblk; k += kOrderWaves) {
        cnt[k * kOrderBuckets + lane] = 0;
        __builtin_amdgcn_wave_barrier();
        const uint32_t c = k * 64 + lane;
        const bool valid = c < nchunks;
        const uint32_t b = valid ? bk[c] : 0u;
        const uint64_t m = same_bucket(b, valid);
        if (valid && (m & ((1ull << lane) - 1ull)) == 0)  // the bucket's first lane
            cnt[k * kOrderBuckets + b] = (uint16_t)__popcll(m);
    }
    __syncthreads();
    // exclusive scan over blocks per bucket: part w (one wave) sums its blocks
    // [w per, (w + 1) per) for bucket = lane, then the parts are scanned
    const uint32_t per = ceil_div(nblk, kOrderWaves);
    const uint32_t k0 = min(nblk, wave * per), k1 = min(nblk, k0 + per);
    uint32_t sum = 0;
    for (uint32_t k = k0; k < k1; ++k) sum += cnt[k * kOrderBuckets + lane];
    part[wave * kOrderBuckets + lane] = sum;
    __syncthreads();
    if (wave == 0) {
        uint32_t acc = 0;
        for (uint32_t w = 0; w < kOrderWaves; ++w) {
            const uint32_t v = part[w * kOrderBuckets + lane];
            part[w * kOrderBuckets + lane] = acc;
            acc += v;
        }
        // the bucket totals (lane = bucket), exclusive over buckets
        uint32_t x = acc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        base[lane] = x - acc;
    }
    __syncthreads();
    uint32_t off = part[wave * kOrderBuckets + lane];
    for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t v = cnt[k * kOrderBuckets + lane];
        cnt[k * kOrderBuckets + lane] = (uint16_t)off;
        off += v;
    }
    __syncthreads();
    for (uint32_t k = wave; k < nblk; k += kOrderWaves) {
        const uint32_t c = k * 64 + lane;
        const bool valid = c < nchunks;
        const uint32_t b = valid ? bk[c] : 0u;
        const uint64_t m = same_bucket(b, valid);
        if (valid) {
            const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            order[base[b] + cnt[k * kOrderBuckets + b] + rank] = (int32_t)c;
        }
    }
}

}  // namespace rd
}  // namespace dfhip

extern "C" int dfhip_render_ray_order_occ(const float *rays_o, const float *rays_d,
                                          const float *nears, const float *fars,
                                          const uint8_t *grid, float bound, uint32_t C,
                                          uint32_t H, uint32_t max_steps, uint32_t N,
                                          uint32_t chunk_log2, uint32_t tile_w, float *cost,
                                          int32_t *order, dfhip_stream_t stream) {
    const char *name = "render_ray_order_occ";
    if (tile_w && (chunk_log2 != 6 || tile_w % 8 || N % (8 * tile_w))) {
        set_error("%s: tile chunks need chunk_log2 6, tile_w a multiple of 8 and N of 8 tile_w "
                  "(got chunk_log2 %u, tile_w %u, N %u)", name, chunk_log2, tile_w, N);
        return DFHIP_EINVAL;
    }
    if (chunk_log2 > 16 || C < 1 || C > 16 || H < 2 || H > 1024 || max_steps == 0 ||
        !(bound > 0.0f)) {
        set_error("%s: invalid chunk_log2=%u C=%u H=%u max_steps=%u bound=%g", name,
                  chunk_log2, C, H, max_steps, (double)bound);
        return DFHIP_EINVAL;
    }
    if (N == 0) return DFHIP_OK;
    const uint32_t nchunks = ceil_div(N, 1u << chunk_log2);
    if (nchunks > rd::kMaxOrderChunks) {
        set_error("%s: %u chunks of 2^%u rays exceed %u (use larger chunks)", name, nchunks,
                  chunk_log2, rd::kMaxOrderChunks);
        return DFHIP_EINVAL;
    }
    if (!rays_o || !rays_d || !nears || !fars || !grid || !cost || !order) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const rm::MarchConsts k = rm::make_consts(bound, 0.0f, max_steps, C, H);
    rd::k_chunk_cost_occ<<<ceil_div(nchunks, 4u), 256, 0, s>>>(rays_o, rays_d, nears, fars, grid,
                                                               k, N, chunk_log2, nchunks, cost,
                                                               tile_w);
    rd::k_chunk_order<<<1, rd::kOrderThreads, 0, s>>>(cost, nchunks, order);
    return check_launch(name);
}

extern "C" int dfhip_render_ray_order(const float *rays_o, const float *rays_d, uint32_t N,
                                      uint32_t chunk_log2, uint32_t tile_w, float *cost,
                                      int32_t *order, dfhip_stream_t stream) {
    const char *name = "render_ray_order";
    if (tile_w && (chunk_log2 != 6 || tile_w % 8 || N % (8 * tile_w))) {
        set_error("%s: tile chunks need chunk_log2 6, tile_w a multiple of 8 and N of 8 tile_w "
                  "(got chunk_log2 %u, tile_w %u, N %u)", name, chunk_log2, tile_w, N);
        return DFHIP_EINVAL;
    }
    if (chunk_log2 > 16) {
        set_error("%s: chunk_log2 must be <= 16 (got %u)", name, chunk_log2);
        return DFHIP_EINVAL;
    }
    if (N == 0) return DFHIP_OK;
    const uint32_t nchunks = ceil_div(N, 1u << chunk_log2);
    if (nchunks > rd::kMaxOrderChunks) {
        set_error("%s: %u chunks of 2^%u rays exceed %u (use larger chunks)", name, nchunks,
                  chunk_log2, rd::kMaxOrderChunks);
        return DFHIP_EINVAL;
    }
    if (!rays_o || !rays_d || !cost || !order) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    rd::k_chunk_cost<<<ceil_div(nchunks, 4u), 256, 0, s>>>(rays_o, rays_d, N, chunk_log2,
                                                           nchunks, cost, tile_w);
    rd::k_chunk_order<<<1, rd::kOrderThreads, 0, s>>>(cost, nchunks, order);
    return check_launch(name);
}
