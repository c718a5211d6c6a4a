// Occupancy-grid ray marching + volume compositing for gfx950 (MI355X).
//
// Behavioural spec: reference raymarching/src/raymarching.cu (cited per kernel).
// Numerics follow the reference's nvcc build: every multiply-add that nvcc
// contracts by default (-fmad=true) is an explicit fmaf() here, and the file is
// compiled with -ffp-contract=off so nothing else is contracted.  The CPU oracle
// (oracle/oracle.c) makes the same choices, which makes per-ray sample counts and
// sample contents bit-exact between the two.
//
// MI355X design notes:
//  * march_rays_train marches one ray per wave64: 64 consecutive candidate
//    steps are tested at once and the reference's visit order is replayed on
//    the wave's ballots (march_wave, march_common.h), so a ray costs a few
//    bitfield round trips instead of one per step.  It is deterministic: a
//    count pass (block totals, integer atomics only for the API counter), then
//    an emit pass that derives each ray's offset from the block totals.
//    Samples land in ray order, contiguous per ray, so compositing and the
//    encoders read each ray's samples as one run.
//  * No N*max_steps zero-fill: the emit pass zeroes only the align tail.
//  * One wave per workgroup for the per-ray compositing kernels: 16k rays =
//    256 workgroups = one per CU, instead of 64 CUs with 256-thread blocks.
#include "march_common.h"

#include <type_traits>

namespace dfhip {
namespace rm {

// ------------------------------------------------------------------ utils

// numeric_limits<scalar_t>::max() of the reference's miss value (raymarching.cu:122)
template <typename T> __device__ __forceinline__ T max_value();
template <> __device__ __forceinline__ float max_value<float>() { return FLT_MAX; }
template <> __device__ __forceinline__ double max_value<double>() { return DBL_MAX; }
template <> __device__ __forceinline__ half_t max_value<half_t>() { return (half_t)65504.0f; }

// raymarching.cu:91-145
template <typename scalar_t>
__global__ __launch_bounds__(256) void k_near_far(const scalar_t *__restrict__ rays_o,
                                                  const scalar_t *__restrict__ rays_d,
                                                  const scalar_t *__restrict__ aabb,
                                                  uint32_t N, float min_near,
                                                  scalar_t *nears, scalar_t *fars) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const Ray r = load_ray(rays_o + 3 * n, rays_d + 3 * n);
    float b[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) b[i] = to_f(aabb[i]);
    float lo, hi;
    if (!ray_aabb(r, b, min_near, lo, hi)) {
        nears[n] = fars[n] = max_value<scalar_t>();
        return;
    }
    nears[n] = from_f<scalar_t>(lo);
    fars[n] = from_f<scalar_t>(hi);
}

// raymarching.cu:162-198
template <typename scalar_t>
__global__ __launch_bounds__(256) void k_sph_from_ray(const scalar_t *__restrict__ rays_o,
                                                      const scalar_t *__restrict__ rays_d,
                                                      float radius, uint32_t N,
                                                      scalar_t *coords) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const Ray r = load_ray(rays_o + 3 * n, rays_d + 3 * n);
    // Contraction model (LLVM DAG combine, as nvcc): a*b + c*d -> fma(a, b, c*d).
    const float A = fmaf(r.dz, r.dz, fmaf(r.dx, r.dx, r.dy * r.dy));
    const float Bh = fmaf(r.oz, r.dz, fmaf(r.ox, r.dx, r.oy * r.dy));
    const float Cc = fmaf(-radius, radius, fmaf(r.oz, r.oz, fmaf(r.ox, r.ox, r.oy * r.oy)));
    const float t = (-Bh + sqrtf(fmaf(Bh, Bh, -(A * Cc)))) / A;
    const float x = fmaf(t, r.dx, r.ox), y = fmaf(t, r.dy, r.oy), z = fmaf(t, r.dz, r.oz);
    const float theta = atan2f(sqrtf(fmaf(x, x, z * z)), y);
    const float phi = atan2f(z, x);
    coords[2 * n + 0] = from_f<scalar_t>(fmaf(2.0f * theta, kInvPi, -1.0f));
    coords[2 * n + 1] = from_f<scalar_t>(phi * kInvPi);
}

// raymarching.cu:214-226
__global__ __launch_bounds__(256) void k_morton3D(const int32_t *__restrict__ coords,
                                                  uint32_t N, int32_t *indices) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const int32_t *c = coords + 3 * n;
    indices[n] = (int32_t)morton3((uint32_t)c[0], (uint32_t)c[1], (uint32_t)c[2]);
}

// raymarching.cu:237-254
__global__ __launch_bounds__(256) void k_morton3D_invert(const int32_t *__restrict__ indices,
                                                         uint32_t N, int32_t *coords) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const uint32_t v = (uint32_t)indices[n];
    coords[3 * n + 0] = (int32_t)compact3(v);
    coords[3 * n + 1] = (int32_t)compact3(v >> 1);
    coords[3 * n + 2] = (int32_t)compact3(v >> 2);
}

// raymarching.cu:267-289 — one thread per output byte; the 8 grid values of a
// byte are read as two 16-B vectors when the storage is f32.
template <typename scalar_t>
__global__ __launch_bounds__(256) void k_packbits(const scalar_t *__restrict__ grid,
                                                  uint32_t N, float thresh,
                                                  uint8_t *bitfield) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const scalar_t *g = grid + 8 * (size_t)n;
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) bits |= (to_f(g[i]) > thresh ? 1u : 0u) << i;
    bitfield[n] = (uint8_t)bits;
}

// 16-B aligned f32 storage: the 8 values of a byte as two float4 loads.
__global__ __launch_bounds__(256) void k_packbits_f32v(const float *__restrict__ grid,
                                                         uint32_t N, float thresh,
                                                         uint8_t *bitfield) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const float4 *g = reinterpret_cast<const float4 *>(grid) + 2 * (size_t)n;
    const float4 a = g[0], b = g[1];
    const uint32_t bits = (a.x > thresh) | ((a.y > thresh) << 1) | ((a.z > thresh) << 2) |
                          ((a.w > thresh) << 3) | ((b.x > thresh) << 4) |
                          ((b.y > thresh) << 5) | ((b.z > thresh) << 6) | ((b.w > thresh) << 7);
    bitfield[n] = (uint8_t)bits;
}

// ------------------------------------------------------------------ training march

// Rays per workgroup of the train marcher: one wave per ray, 16 waves (8:
// count 61.7 -> 57.0 us per C2 step, emit 14.2 -> 14.8; tools/ab_march.sh).  The
// count pass leaves one total per workgroup in block_sums; the emit pass
// derives a ray's offset from the preceding totals plus the block's counts.
#ifndef DFHIP_MARCH_RPB
#define DFHIP_MARCH_RPB 16
#endif
constexpr uint32_t kMarchRaysPerBlock = DFHIP_MARCH_RPB;
// march_wave's s_vis[1024] holds one 64-byte flag row per wave, and a
// workgroup is at most 1024 threads
static_assert(kMarchRaysPerBlock >= 1 && kMarchRaysPerBlock <= 16,
              "DFHIP_MARCH_RPB: 1..16 rays per workgroup");
constexpr uint32_t kStageFloats = 5;  // x, y, z, dt, dl of a staged sample

// Pass 1 (raymarching.cu:341-400): count occupied samples per ray.
// STAGE: also keep each sample (x, y, z, dt, dl as f32) at row n * max_steps + i
// of `stage`, so the emit pass copies instead of marching again.
template <typename scalar_t, bool STAGE = false>
__global__ __launch_bounds__(64 * kMarchRaysPerBlock) void k_march_train_count(
    const scalar_t *__restrict__ rays_o, const scalar_t *__restrict__ rays_d,
    const uint8_t *__restrict__ grid, MarchConsts k, uint32_t max_steps, uint32_t N,
    const scalar_t *__restrict__ nears, const scalar_t *__restrict__ fars,
    int32_t *rays, int32_t *counter, const scalar_t *__restrict__ noises,
    int32_t *block_sums, float *__restrict__ stage = nullptr) {
    __shared__ int s_cnt[kMarchRaysPerBlock];
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t n = blockIdx.x * kMarchRaysPerBlock + w;
    int cnt = 0;
    if (n < N) {
        const Ray r = load_ray(rays_o + 3 * n, rays_d + 3 * n);
        const float near = to_f(nears[n]), far = to_f(fars[n]);
        const float t0 = fmaf(clampf(near * k.dt_gamma, k.dt_min, k.dt_max),
                              to_f(noises[n]), near);
        if constexpr (STAGE) {
            float *st = stage + (size_t)n * max_steps * kStageFloats;
            cnt = (int)march_wave(k, r, grid, t0, far, max_steps,
                                  [&](uint32_t i, float x, float y, float z, float dt, float dl) {
                                      float *row = st + (size_t)i * kStageFloats;
                                      row[0] = x; row[1] = y; row[2] = z;
                                      row[3] = dt; row[4] = dl;
                                  });
        } else {
            cnt = (int)march_wave(k, r, grid, t0, far, max_steps,
                                  [](uint32_t, float, float, float, float, float) {});
        }
        if ((threadIdx.x & 63) == 0) {
            rays[3 * n + 0] = (int32_t)n;
            rays[3 * n + 2] = cnt;
        }
    }
    if ((threadIdx.x & 63) == 0) s_cnt[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
#pragma unroll
        for (uint32_t i = 0; i < kMarchRaysPerBlock; ++i) tot += s_cnt[i];
        block_sums[blockIdx.x] = tot;
        atomicAdd(counter, tot);
        atomicAdd(counter + 1, (int)min(kMarchRaysPerBlock, N - blockIdx.x * kMarchRaysPerBlock));
    }
}

template <typename scalar_t>
__device__ __forceinline__ void zero_rows(scalar_t *xyzs, scalar_t *dirs, scalar_t *deltas,
                                          uint64_t begin, uint64_t end, uint32_t first,
                                          uint32_t stride) {
    const scalar_t zero = from_f<scalar_t>(0.0f);
    for (uint64_t row = begin + first; row < end; row += stride) {
        xyzs[3 * row] = zero; xyzs[3 * row + 1] = zero; xyzs[3 * row + 2] = zero;
        if (dirs) {
            dirs[3 * row] = zero; dirs[3 * row + 1] = zero; dirs[3 * row + 2] = zero;
        }
        deltas[2 * row] = zero; deltas[2 * row + 1] = zero;
    }
}

// Pass 2 (raymarching.cu:405-479): offset = preceding block totals + the
// counts of the block's earlier rays; then the wave re-marches its ray and
// each lane writes the samples it holds (consecutive rows across the wave).
// Rays whose range would cross M are not written (raymarching.cu:416).
// STAGED: the samples come from the count pass's stage rows (a copy with
// the same f32 -> scalar_t conversions) instead of a second march.
template <typename scalar_t, bool STAGED = false>
__global__ __launch_bounds__(64 * kMarchRaysPerBlock) void k_march_train_emit(
    const scalar_t *__restrict__ rays_o, const scalar_t *__restrict__ rays_d,
    const uint8_t *__restrict__ grid, MarchConsts k, uint32_t N, uint32_t M,
    const scalar_t *__restrict__ nears, const scalar_t *__restrict__ fars,
    scalar_t *xyzs, scalar_t *dirs, scalar_t *deltas, int32_t *rays,
    const scalar_t *__restrict__ noises, const int32_t *__restrict__ block_sums,
    int zero_tail, const float *__restrict__ stage = nullptr, uint32_t max_steps = 0) {
    __shared__ int s_part[kMarchRaysPerBlock];
    __shared__ int s_cnt[kMarchRaysPerBlock];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t n = blockIdx.x * kMarchRaysPerBlock + w;
    int part = 0;
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += blockDim.x) part += block_sums[i];
    part = wave_reduce_add(part);
    const int cnt = (n < N) ? rays[3 * n + 2] : 0;
    if (lane == 0) {
        s_part[w] = part;
        s_cnt[w] = cnt;
    }
    __syncthreads();
    int prefix = 0, before = 0, block_tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < kMarchRaysPerBlock; ++i) {
        prefix += s_part[i];
        before += i < w ? s_cnt[i] : 0;
        block_tot += s_cnt[i];
    }
    const uint32_t off = (uint32_t)(prefix + before);
    if (n < N) {
        if (lane == 0) rays[3 * n + 1] = (int32_t)off;
        if (STAGED && cnt > 0 && off + (uint32_t)cnt <= M) {
            const scalar_t d0 = rays_d[3 * n], d1 = rays_d[3 * n + 1], d2 = rays_d[3 * n + 2];
            const float *st = stage + (size_t)n * max_steps * kStageFloats;
            for (uint32_t i = lane; i < (uint32_t)cnt; i += 64) {
                const float *row = st + (size_t)i * kStageFloats;
                const size_t o = (size_t)off + i;
                xyzs[3 * o + 0] = from_f<scalar_t>(row[0]);
                xyzs[3 * o + 1] = from_f<scalar_t>(row[1]);
                xyzs[3 * o + 2] = from_f<scalar_t>(row[2]);
                if (dirs) {  // uniform: NULL when the caller reads rays_d per ray instead
                    dirs[3 * o + 0] = d0;
                    dirs[3 * o + 1] = d1;
                    dirs[3 * o + 2] = d2;
                }
                deltas[2 * o + 0] = from_f<scalar_t>(row[3]);
                deltas[2 * o + 1] = from_f<scalar_t>(row[4]);
            }
        } else if (cnt > 0 && off + (uint32_t)cnt <= M) {
            const Ray r = load_ray(rays_o + 3 * n, rays_d + 3 * n);
            const float near = to_f(nears[n]), far = to_f(fars[n]);
            const float t0 = fmaf(clampf(near * k.dt_gamma, k.dt_min, k.dt_max),
                                  to_f(noises[n]), near);
            scalar_t *px = xyzs + 3 * (size_t)off;
            scalar_t *pd = dirs + 3 * (size_t)off;
            scalar_t *pl = deltas + 2 * (size_t)off;
            march_wave(k, r, grid, t0, far, (uint32_t)cnt,
                       [&](uint32_t i, float x, float y, float z, float dt, float dl) {
                           px[3 * i + 0] = from_f<scalar_t>(x);
                           px[3 * i + 1] = from_f<scalar_t>(y);
                           px[3 * i + 2] = from_f<scalar_t>(z);
                           pd[3 * i + 0] = from_f<scalar_t>(r.dx);
                           pd[3 * i + 1] = from_f<scalar_t>(r.dy);
                           pd[3 * i + 2] = from_f<scalar_t>(r.dz);
                           pl[2 * i + 0] = from_f<scalar_t>(dt);
                           pl[2 * i + 1] = from_f<scalar_t>(dl);
                       });
        } else if (zero_tail != 0 && cnt > 0 && off < M) {
            // first ray that does not fit: rows [off, M) stay unwritten -> zero
            // (end clipped by the align limit, like the tail below)
            uint64_t end = M;
            if (zero_tail > 0) {
                uint64_t total = (uint64_t)prefix;  // global total, rare path
                for (uint32_t i = blockIdx.x; i < gridDim.x; ++i) total += (uint32_t)block_sums[i];
                end = min(end, total + (uint64_t)zero_tail - total % (uint64_t)zero_tail);
            }
            zero_rows(xyzs, dirs, deltas, off, end, lane, 64);
        }
    }
    if (zero_tail != 0 && blockIdx.x == gridDim.x - 1) {
        const uint64_t total = (uint64_t)prefix + (uint32_t)block_tot;
        uint64_t end = M;
        if (zero_tail > 0) end = min(end, total + (uint64_t)zero_tail - total % (uint64_t)zero_tail);
        zero_rows(xyzs, dirs, deltas, total, end, threadIdx.x, blockDim.x);
    }
}

// ------------------------------------------------------------------ compositing

template <typename scalar_t> struct Acc { typedef float type; };
template <> struct Acc<double> { typedef double type; };

// raymarching.cu:500-577
template <typename scalar_t, typename rgb_t = scalar_t>
__global__ __launch_bounds__(64) void k_composite_train_fwd(
    const scalar_t *__restrict__ sigmas, const rgb_t *__restrict__ rgbs,
    const scalar_t *__restrict__ deltas, const int32_t *__restrict__ rays, uint32_t M,
    uint32_t N, float T_thresh, scalar_t *weights_sum, scalar_t *depth, scalar_t *image) {
    typedef typename Acc<scalar_t>::type acc_t;
    const uint32_t n = blockIdx.x * 64 + threadIdx.x;
    if (n >= N) return;
    const uint32_t index = (uint32_t)rays[3 * n];
    const uint32_t offset = (uint32_t)rays[3 * n + 1];
    const uint32_t num = (uint32_t)rays[3 * n + 2];
    acc_t T = 1, r = 0, g = 0, b = 0, ws = 0, t = 0, d = 0;
    if (num != 0 && offset + num <= M) {
        const scalar_t *s = sigmas + offset;
        const rgb_t *c = rgbs + 3 * (size_t)offset;
        const scalar_t *dl = deltas + 2 * (size_t)offset;
        for (uint32_t i = 0; i < num; ++i) {
            const acc_t alpha = (acc_t)1.0f - (acc_t)__expf(-to_f(s[i]) * to_f(dl[2 * i]));
            const acc_t w = alpha * T;
            r = fma(w, (acc_t)to_f(c[3 * i + 0]), r);
            g = fma(w, (acc_t)to_f(c[3 * i + 1]), g);
            b = fma(w, (acc_t)to_f(c[3 * i + 2]), b);
            t += (acc_t)to_f(dl[2 * i + 1]);
            d = fma(w, t, d);
            ws += w;
            T *= (acc_t)1.0f - alpha;
            if (T < (acc_t)T_thresh) break;
        }
    }
    weights_sum[index] = (scalar_t)ws;
    depth[index] = (scalar_t)d;
    image[3 * index + 0] = (scalar_t)r;
    image[3 * index + 1] = (scalar_t)g;
    image[3 * index + 2] = (scalar_t)b;
}

// Colour-gradient store.  f32 compositing of f16 colours: the f32 product is
// rounded to f16 once, as the reference's autograd cast of its f32 gradient
// does.  f32_rounded keeps the backend from fusing product and conversion into
// one v_fma_mix, which rounds the exact product once and can differ in the
// last f16 bit.
template <typename scalar_t, typename rgb_t, typename acc_t>
__device__ __forceinline__ rgb_t grad_cast(acc_t v) { return (rgb_t)v; }
template <>
__device__ __forceinline__ half_t grad_cast<float, half_t, float>(float v) {
    return (half_t)f32_rounded(v);
}
template <>
__device__ __forceinline__ bf16_t grad_cast<float, bf16_t, float>(float v) {
    return (bf16_t)f32_rounded(v);
}

// raymarching.cu:601-682.  DENSE: also zero rows the reference leaves untouched
// (past each ray's break; with `tail`, also rows [total, M) after the last ray).
// rgb_t = f16 reads the field's f16 colours and writes their f16 gradient
// directly: the reference casts them to f32 on entry (custom_fwd) and its
// autograd casts the f32 gradient back to f16 once, which is this rounding.
template <typename scalar_t, bool DENSE, typename rgb_t = scalar_t>
__global__ __launch_bounds__(64) void k_composite_train_bwd(
    const scalar_t *__restrict__ grad_ws, const scalar_t *__restrict__ grad_image,
    const scalar_t *__restrict__ sigmas, const rgb_t *__restrict__ rgbs,
    const scalar_t *__restrict__ deltas, const int32_t *__restrict__ rays,
    const scalar_t *__restrict__ weights_sum, const scalar_t *__restrict__ image,
    uint32_t M, uint32_t N, float T_thresh, scalar_t *grad_sigmas, rgb_t *grad_rgbs,
    int tail = 1) {
    typedef typename Acc<scalar_t>::type acc_t;
    const uint32_t n = blockIdx.x * 64 + threadIdx.x;
    if (n >= N) return;
    const uint32_t index = (uint32_t)rays[3 * n];
    const uint32_t offset = (uint32_t)rays[3 * n + 1];
    const uint32_t num = (uint32_t)rays[3 * n + 2];
    const scalar_t zero = (scalar_t)0.0f;
    const rgb_t czero = (rgb_t)0.0f;
    uint32_t i = 0;
    if (num != 0 && offset + num <= M) {
        const scalar_t *s = sigmas + offset;
        const rgb_t *c = rgbs + 3 * (size_t)offset;
        const scalar_t *dl = deltas + 2 * (size_t)offset;
        scalar_t *gs = grad_sigmas + offset;
        rgb_t *gc = grad_rgbs + 3 * (size_t)offset;
        const acc_t gr = to_f(grad_image[3 * index + 0]);
        const acc_t gg = to_f(grad_image[3 * index + 1]);
        const acc_t gb = to_f(grad_image[3 * index + 2]);
        const acc_t gw = to_f(grad_ws[index]);
        const acc_t rf = to_f(image[3 * index + 0]);
        const acc_t gf = to_f(image[3 * index + 1]);
        const acc_t bf = to_f(image[3 * index + 2]);
        const acc_t wsf = to_f(weights_sum[index]);
        acc_t T = 1, r = 0, g = 0, b = 0, ws = 0;
        for (; i < num; ++i) {
            const acc_t sg = to_f(s[i]), dt = to_f(dl[2 * i]);
            const acc_t cr = to_f(c[3 * i]), cg = to_f(c[3 * i + 1]), cb = to_f(c[3 * i + 2]);
            const acc_t alpha = (acc_t)1.0f - (acc_t)__expf(-(float)sg * (float)dt);
            const acc_t w = alpha * T;
            r = fma(w, cr, r);
            g = fma(w, cg, g);
            b = fma(w, cb, b);
            ws += w;
            T *= (acc_t)1.0f - alpha;
            gc[3 * i + 0] = grad_cast<scalar_t, rgb_t>(gr * w);
            gc[3 * i + 1] = grad_cast<scalar_t, rgb_t>(gg * w);
            gc[3 * i + 2] = grad_cast<scalar_t, rgb_t>(gb * w);
            // ((gr*A + gg*B) + gb*C) + gw*D, nvcc contraction: fuse the left product.
            acc_t acc = fma(gr, fma(T, cr, -(rf - r)), gg * fma(T, cg, -(gf - g)));
            acc = fma(gb, fma(T, cb, -(bf - b)), acc);
            acc = fma(gw, (acc_t)1 - wsf, acc);
            gs[i] = (scalar_t)(dt * acc);
            if (T < (acc_t)T_thresh) { ++i; break; }
        }
    }
    if (DENSE) {
        // Zero rows [offset + i, offset + num) of this ray, clipped to M.
        const uint64_t end = min((uint64_t)offset + num, (uint64_t)M);
        for (uint64_t row = (uint64_t)offset + i; row < end; ++row) {
            grad_sigmas[row] = zero;
            grad_rgbs[3 * row] = czero; grad_rgbs[3 * row + 1] = czero; grad_rgbs[3 * row + 2] = czero;
        }
        if (tail && n == N - 1) {
            for (uint64_t row = (uint64_t)offset + num; row < M; ++row) {
                grad_sigmas[row] = zero;
                grad_rgbs[3 * row] = czero; grad_rgbs[3 * row + 1] = czero; grad_rgbs[3 * row + 2] = czero;
            }
        }
    }
}

// ------------------------------------------------------------------ compositing, row per ray
// The same arithmetic as k_composite_train_fwd / _bwd in the same order, with
// one ray per 16-lane row of a wave (4 rays per wave): each lane loads one
// sample of the ray's 16-sample window (coalesced), computes its alpha, and
// the row then runs the reference's serial chain (T, the colour / weight /
// depth sums) over the window, each step reading sample j's values with a DPP
// row broadcast (row_newbcast:j) that the compiler folds into the consuming
// VALU instruction.  One VALU instruction thus advances four rays, where a
// whole-wave chain (readlane per value) spends it on one.  Bit-identical to
// the one-thread-per-ray loop (same f32 operations, same order, same break).
//
// The chain is branch-free inside a window: the reference's
// `if (T < T_thresh) break` becomes a row-uniform `alive` flag that zeroes the
// weight of every later sample (fmaf(0, c, x) == x and x + 0 == x, so the sums
// are unchanged), and lanes past the window's count hold alpha 0, 1 - alpha 1,
// zero colour and delta (no-ops).  Only the window loop branches (per row).
constexpr uint32_t kCompRaysPerBlock = 16;   // 4 waves x 4 rows

template <int J>
__device__ __forceinline__ float row_bcast(float v) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + J, 0xF, 0xF, false));
}

template <typename rgb_t>
__device__ __forceinline__ void load_rgb3(const rgb_t *c, float &r, float &g, float &b) {
    r = to_f(c[0]);
    g = to_f(c[1]);
    b = to_f(c[2]);
}

struct FwdChain {
    float T = 1.0f, r = 0.0f, g = 0.0f, b = 0.0f, ws = 0.0f, t = 0.0f, d = 0.0f;
    bool alive = true;
    template <int J>
    __device__ __forceinline__ void step(float a, float om, float cr, float cg, float cb,
                                         float dl, float T_thresh) {
        const float w = alive ? row_bcast<J>(a) * T : 0.0f;
        r = fmaf(w, row_bcast<J>(cr), r);
        g = fmaf(w, row_bcast<J>(cg), g);
        b = fmaf(w, row_bcast<J>(cb), b);
        t += row_bcast<J>(dl);
        d = fmaf(w, t, d);
        ws += w;
        T *= row_bcast<J>(om);
        alive = alive && !(T < T_thresh);
    }
};

// raymarching.cu:500-577
template <typename scalar_t, typename rgb_t>
__global__ __launch_bounds__(256) void k_composite_train_fwd_w(
    const scalar_t *__restrict__ sigmas, const rgb_t *__restrict__ rgbs,
    const scalar_t *__restrict__ deltas, const int32_t *__restrict__ rays, uint32_t M,
    uint32_t N, float T_thresh, scalar_t *weights_sum, scalar_t *depth, scalar_t *image) {
    const uint32_t n = blockIdx.x * kCompRaysPerBlock + (threadIdx.x >> 4);
    const int lane = (int)(threadIdx.x & 15);
    uint32_t index = 0, offset = 0, num = 0;
    if (n < N) {
        index = (uint32_t)rays[3 * n];
        offset = (uint32_t)rays[3 * n + 1];
        num = (uint32_t)rays[3 * n + 2];
        if (offset + num > M) num = 0;
    }
    FwdChain c;
    for (uint32_t base = 0; base < num && c.alive; base += 16) {
        const uint32_t cnt = min(16u, num - base);
        float a = 0.0f, om = 1.0f, cr = 0.0f, cg = 0.0f, cb = 0.0f, dl = 0.0f;
        if ((uint32_t)lane < cnt) {
            const size_t i = (size_t)offset + base + lane;
            a = 1.0f - __expf(-to_f(sigmas[i]) * to_f(deltas[2 * i]));
            om = 1.0f - a;
            dl = to_f(deltas[2 * i + 1]);
            load_rgb3(rgbs + 3 * i, cr, cg, cb);
        }
#define DFHIP_FSTEP(J) c.step<J>(a, om, cr, cg, cb, dl, T_thresh);
        DFHIP_FSTEP(0) DFHIP_FSTEP(1) DFHIP_FSTEP(2) DFHIP_FSTEP(3)
        DFHIP_FSTEP(4) DFHIP_FSTEP(5) DFHIP_FSTEP(6) DFHIP_FSTEP(7)
        DFHIP_FSTEP(8) DFHIP_FSTEP(9) DFHIP_FSTEP(10) DFHIP_FSTEP(11)
        DFHIP_FSTEP(12) DFHIP_FSTEP(13) DFHIP_FSTEP(14) DFHIP_FSTEP(15)
#undef DFHIP_FSTEP
    }
    if (lane == 0 && n < N) {
        weights_sum[index] = (scalar_t)c.ws;
        depth[index] = (scalar_t)c.d;
        image[3 * index + 0] = (scalar_t)c.r;
        image[3 * index + 1] = (scalar_t)c.g;
        image[3 * index + 2] = (scalar_t)c.b;
    }
}

// Backward chain: lane l of the row captures the state after sample l of the
// window (weight, T, colour sums) and whether the reference loop reached it.
struct BwdChain {
    float T = 1.0f, r = 0.0f, g = 0.0f, b = 0.0f;
    bool alive = true;
    float wl, Tl, rl, gl, bl;
    bool taken;
    template <int J>
    __device__ __forceinline__ void step(int lane, float a, float om, float cr, float cg,
                                         float cb, float T_thresh) {
        const float w = row_bcast<J>(a) * T;
        r = fmaf(w, row_bcast<J>(cr), r);
        g = fmaf(w, row_bcast<J>(cg), g);
        b = fmaf(w, row_bcast<J>(cb), b);
        T *= row_bcast<J>(om);
        const bool mine = lane == J;
        wl = mine ? w : wl;
        Tl = mine ? T : Tl;
        rl = mine ? r : rl;
        gl = mine ? g : gl;
        bl = mine ? b : bl;
        taken = mine ? alive : taken;
        alive = alive && !(T < T_thresh);
    }
};

// raymarching.cu:601-682, DENSE as k_composite_train_bwd.
template <typename scalar_t, bool DENSE, typename rgb_t>
__global__ __launch_bounds__(256) void k_composite_train_bwd_w(
    const scalar_t *__restrict__ grad_ws, const scalar_t *__restrict__ grad_image,
    const scalar_t *__restrict__ sigmas, const rgb_t *__restrict__ rgbs,
    const scalar_t *__restrict__ deltas, const int32_t *__restrict__ rays,
    const scalar_t *__restrict__ weights_sum, const scalar_t *__restrict__ image,
    uint32_t M, uint32_t N, float T_thresh, scalar_t *grad_sigmas, rgb_t *grad_rgbs,
    int tail) {
    const uint32_t n = blockIdx.x * kCompRaysPerBlock + (threadIdx.x >> 4);
    const int lane = (int)(threadIdx.x & 15);
    const int row_shift = (int)(threadIdx.x & 48);   // this row's bits in a wave ballot
    const scalar_t zero = (scalar_t)0.0f;
    const rgb_t czero = (rgb_t)0.0f;
    uint32_t index = 0, offset = 0, num = 0, num_all = 0;
    if (n < N) {
        index = (uint32_t)rays[3 * n];
        offset = (uint32_t)rays[3 * n + 1];
        num_all = (uint32_t)rays[3 * n + 2];
        num = (offset + num_all <= M) ? num_all : 0u;
    }
    uint32_t done = 0;   // samples taken (the reference loop's final i)
    if (num != 0) {
        const float gr = to_f(grad_image[3 * index + 0]);
        const float gg = to_f(grad_image[3 * index + 1]);
        const float gb = to_f(grad_image[3 * index + 2]);
        const float gw = to_f(grad_ws[index]);
        const float rf = to_f(image[3 * index + 0]);
        const float gf = to_f(image[3 * index + 1]);
        const float bf = to_f(image[3 * index + 2]);
        const float wsf = to_f(weights_sum[index]);
        BwdChain c;
        for (uint32_t base = 0; base < num && c.alive; base += 16) {
            const uint32_t cnt = min(16u, num - base);
            const size_t i = (size_t)offset + base + lane;
            float a = 0.0f, om = 1.0f, dt = 0.0f, cr = 0.0f, cg = 0.0f, cb = 0.0f;
            if ((uint32_t)lane < cnt) {
                dt = to_f(deltas[2 * i]);
                a = 1.0f - __expf(-to_f(sigmas[i]) * dt);
                om = 1.0f - a;
                load_rgb3(rgbs + 3 * i, cr, cg, cb);
            }
            c.wl = c.Tl = c.rl = c.gl = c.bl = 0.0f;
            c.taken = false;
#define DFHIP_BSTEP(J) c.step<J>(lane, a, om, cr, cg, cb, T_thresh);
            DFHIP_BSTEP(0) DFHIP_BSTEP(1) DFHIP_BSTEP(2) DFHIP_BSTEP(3)
            DFHIP_BSTEP(4) DFHIP_BSTEP(5) DFHIP_BSTEP(6) DFHIP_BSTEP(7)
            DFHIP_BSTEP(8) DFHIP_BSTEP(9) DFHIP_BSTEP(10) DFHIP_BSTEP(11)
            DFHIP_BSTEP(12) DFHIP_BSTEP(13) DFHIP_BSTEP(14) DFHIP_BSTEP(15)
#undef DFHIP_BSTEP
            const bool taken = c.taken && (uint32_t)lane < cnt;
            if (taken) {
                grad_rgbs[3 * i + 0] = grad_cast<scalar_t, rgb_t>(gr * c.wl);
                grad_rgbs[3 * i + 1] = grad_cast<scalar_t, rgb_t>(gg * c.wl);
                grad_rgbs[3 * i + 2] = grad_cast<scalar_t, rgb_t>(gb * c.wl);
                float acc = fmaf(gr, fmaf(c.Tl, cr, -(rf - c.rl)), gg * fmaf(c.Tl, cg, -(gf - c.gl)));
                acc = fmaf(gb, fmaf(c.Tl, cb, -(bf - c.bl)), acc);
                acc = fmaf(gw, 1.0f - wsf, acc);
                grad_sigmas[i] = (scalar_t)(dt * acc);
            }
            done = base + (uint32_t)__popcll((__ballot(taken) >> row_shift) & 0xFFFFull);
        }
    }
    if (DENSE && n < N) {
        // rows [offset + done, offset + num) of this ray, clipped to M
        const uint64_t end = min((uint64_t)offset + num_all, (uint64_t)M);
        for (uint64_t row = (uint64_t)offset + done + lane; row < end; row += 16) {
            grad_sigmas[row] = zero;
            grad_rgbs[3 * row] = czero; grad_rgbs[3 * row + 1] = czero; grad_rgbs[3 * row + 2] = czero;
        }
        if (tail && n == N - 1) {
            for (uint64_t row = (uint64_t)offset + num_all + lane; row < M; row += 16) {
                grad_sigmas[row] = zero;
                grad_rgbs[3 * row] = czero; grad_rgbs[3 * row + 1] = czero; grad_rgbs[3 * row + 2] = czero;
            }
        }
    }
}

template <typename scalar_t, typename rgb_t>
static void launch_comp_fwd(hipStream_t s, const scalar_t *sig, const rgb_t *rgb,
                            const scalar_t *dl, const int32_t *rays, uint32_t M, uint32_t N,
                            float T_thresh, scalar_t *ws, scalar_t *depth, scalar_t *image) {
    if constexpr (std::is_same<scalar_t, double>::value)
        k_composite_train_fwd<scalar_t, rgb_t><<<ceil_div(N, 64u), 64, 0, s>>>(
            sig, rgb, dl, rays, M, N, T_thresh, ws, depth, image);
    else
        k_composite_train_fwd_w<scalar_t, rgb_t>
            <<<ceil_div(N, kCompRaysPerBlock), 256, 0, s>>>(
                sig, rgb, dl, rays, M, N, T_thresh, ws, depth, image);
}

template <typename scalar_t, bool DENSE, typename rgb_t>
static void launch_comp_bwd(hipStream_t s, const scalar_t *gws, const scalar_t *gimg,
                            const scalar_t *sig, const rgb_t *rgb, const scalar_t *dl,
                            const int32_t *rays, const scalar_t *ws, const scalar_t *img,
                            uint32_t M, uint32_t N, float T_thresh, scalar_t *gsig,
                            rgb_t *grgb, int tail) {
    if constexpr (std::is_same<scalar_t, double>::value)
        k_composite_train_bwd<scalar_t, DENSE, rgb_t><<<ceil_div(N, 64u), 64, 0, s>>>(
            gws, gimg, sig, rgb, dl, rays, ws, img, M, N, T_thresh, gsig, grgb, tail);
    else
        k_composite_train_bwd_w<scalar_t, DENSE, rgb_t>
            <<<ceil_div(N, kCompRaysPerBlock), 256, 0, s>>>(
                gws, gimg, sig, rgb, dl, rays, ws, img, M, N, T_thresh, gsig, grgb, tail);
}

// ------------------------------------------------------------------ inference

// raymarching.cu:700-804; also writes zeros into the slots it does not fill.
template <typename scalar_t>
__global__ __launch_bounds__(64) void k_march_infer(
    uint32_t n_alive, uint32_t n_step, const int32_t *__restrict__ rays_alive,
    const scalar_t *__restrict__ rays_t, const scalar_t *__restrict__ rays_o,
    const scalar_t *__restrict__ rays_d, MarchConsts k, const uint8_t *__restrict__ grid,
    const scalar_t *__restrict__ fars, scalar_t *xyzs, scalar_t *dirs, scalar_t *deltas,
    const scalar_t *__restrict__ noises) {
    const uint32_t n = blockIdx.x * 64 + threadIdx.x;
    if (n >= n_alive) return;
    const int index = rays_alive[n];
    const Ray r = load_ray(rays_o + 3 * (size_t)index, rays_d + 3 * (size_t)index);
    float t = to_f(rays_t[index]);
    const float far = to_f(fars[index]);
    t = fmaf(clampf(t * k.dt_gamma, k.dt_min, k.dt_max), to_f(noises[n]), t);
    scalar_t *px = xyzs + 3 * (size_t)n * n_step;
    scalar_t *pd = dirs + 3 * (size_t)n * n_step;
    scalar_t *pl = deltas + 2 * (size_t)n * n_step;
    const uint32_t got = march<true, scalar_t>(k, r, grid, t, far, n_step, px, pd, pl, nullptr);
    const scalar_t zero = from_f<scalar_t>(0.0f);
    for (uint32_t s = got; s < n_step; ++s) {
        px[3 * s] = zero; px[3 * s + 1] = zero; px[3 * s + 2] = zero;
        pd[3 * s] = zero; pd[3 * s + 1] = zero; pd[3 * s + 2] = zero;
        pl[2 * s] = zero; pl[2 * s + 1] = zero;
    }
}

// raymarching.cu:818-905
template <typename scalar_t>
__global__ __launch_bounds__(64) void k_composite_infer(
    uint32_t n_alive, uint32_t n_step, float T_thresh, int32_t *rays_alive,
    scalar_t *rays_t, const scalar_t *__restrict__ sigmas,
    const scalar_t *__restrict__ rgbs, const scalar_t *__restrict__ deltas,
    scalar_t *weights_sum, scalar_t *depth, scalar_t *image) {
    typedef typename Acc<scalar_t>::type acc_t;
    const uint32_t n = blockIdx.x * 64 + threadIdx.x;
    if (n >= n_alive) return;
    const int index = rays_alive[n];
    const scalar_t *s = sigmas + (size_t)n * n_step;
    const scalar_t *c = rgbs + 3 * (size_t)n * n_step;
    const scalar_t *dl = deltas + 2 * (size_t)n * n_step;
    acc_t t = to_f(rays_t[index]);
    acc_t wsum = to_f(weights_sum[index]);
    acc_t d = to_f(depth[index]);
    acc_t r = to_f(image[3 * index]), g = to_f(image[3 * index + 1]), b = to_f(image[3 * index + 2]);
    uint32_t step = 0;
    while (step < n_step) {
        const acc_t dt = to_f(dl[2 * step]);
        if (dt == (acc_t)0) break;
        const acc_t alpha = (acc_t)1.0f - (acc_t)__expf(-to_f(s[step]) * (float)dt);
        const acc_t T = (acc_t)1 - wsum;
        const acc_t w = alpha * T;
        wsum += w;
        t += (acc_t)to_f(dl[2 * step + 1]);
        d = fma(w, t, d);
        r = fma(w, (acc_t)to_f(c[3 * step]), r);
        g = fma(w, (acc_t)to_f(c[3 * step + 1]), g);
        b = fma(w, (acc_t)to_f(c[3 * step + 2]), b);
        if (T < (acc_t)T_thresh) break;
        ++step;
    }
    if (step < n_step) rays_alive[n] = -1;
    else rays_t[index] = (scalar_t)t;
    weights_sum[index] = (scalar_t)wsum;
    depth[index] = (scalar_t)d;
    image[3 * index] = (scalar_t)r;
    image[3 * index + 1] = (scalar_t)g;
    image[3 * index + 2] = (scalar_t)b;
}

static bool march_args_ok(const char *what, uint32_t C, uint32_t H, uint32_t max_steps) {
    if (C < 1 || C > 16 || H < 2 || H > 1024 || max_steps == 0) {
        set_error("%s: invalid C=%u H=%u max_steps=%u", what, C, H, max_steps);
        return false;
    }
    return true;
}

}  // namespace rm
}  // namespace dfhip

using namespace dfhip;
using namespace dfhip::rm;

// ====================================================================== C ABI

extern "C" int dfhip_near_far_from_aabb(int dtype, const void *rays_o, const void *rays_d,
                                        const void *aabb, uint32_t N, float min_near,
                                        void *nears, void *fars, dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    DFHIP_DISPATCH(dtype, "near_far_from_aabb",
        k_near_far<scalar_t><<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(
            (const scalar_t *)rays_o, (const scalar_t *)rays_d, (const scalar_t *)aabb, N,
            min_near, (scalar_t *)nears, (scalar_t *)fars));
    return check_launch("near_far_from_aabb");
}

extern "C" int dfhip_sph_from_ray(int dtype, const void *rays_o, const void *rays_d,
                                  float radius, uint32_t N, void *coords,
                                  dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    DFHIP_DISPATCH(dtype, "sph_from_ray",
        k_sph_from_ray<scalar_t><<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(
            (const scalar_t *)rays_o, (const scalar_t *)rays_d, radius, N,
            (scalar_t *)coords));
    return check_launch("sph_from_ray");
}

extern "C" int dfhip_morton3D(const int32_t *coords, uint32_t N, int32_t *indices,
                              dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    k_morton3D<<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(coords, N, indices);
    return check_launch("morton3D");
}

extern "C" int dfhip_morton3D_invert(const int32_t *indices, uint32_t N, int32_t *coords,
                                     dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    k_morton3D_invert<<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(indices, N, coords);
    return check_launch("morton3D_invert");
}

extern "C" int dfhip_packbits(int dtype, const void *grid, uint32_t N, float density_thresh,
                              uint8_t *bitfield, dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    if (dtype == DFHIP_F32 && ((uintptr_t)grid & 15) == 0) {
        k_packbits_f32v<<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(
            (const float *)grid, N, density_thresh, bitfield);
        return check_launch("packbits");
    }
    DFHIP_DISPATCH(dtype, "packbits",
        k_packbits<scalar_t><<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(
            (const scalar_t *)grid, N, density_thresh, bitfield));
    return check_launch("packbits");
}

extern "C" uint32_t dfhip_march_rays_train_scratch_ints(uint32_t N) {
    return ceil_div(N, kMarchRaysPerBlock) > 0 ? ceil_div(N, kMarchRaysPerBlock) : 1u;
}

extern "C" int dfhip_march_rays_train_count(int dtype, const void *rays_o, const void *rays_d,
                                            const uint8_t *grid, float bound, float dt_gamma,
                                            uint32_t max_steps, uint32_t N, uint32_t C,
                                            uint32_t H, const void *nears, const void *fars,
                                            int32_t *rays, int32_t *counter,
                                            const void *noises, int32_t *block_sums,
                                            dfhip_stream_t stream) {
    if (!march_args_ok("march_rays_train_count", C, H, max_steps)) return DFHIP_EINVAL;
    if (N == 0) return DFHIP_OK;
    const MarchConsts k = make_consts(bound, dt_gamma, max_steps, C, H);
    DFHIP_DISPATCH(dtype, "march_rays_train_count",
        k_march_train_count<scalar_t><<<ceil_div(N, kMarchRaysPerBlock), 64 * kMarchRaysPerBlock,
                                        0, as_stream(stream)>>>(
            (const scalar_t *)rays_o, (const scalar_t *)rays_d, grid, k, max_steps, N,
            (const scalar_t *)nears, (const scalar_t *)fars, rays, counter,
            (const scalar_t *)noises, block_sums));
    return check_launch("march_rays_train_count");
}

extern "C" int dfhip_march_rays_train_emit(int dtype, const void *rays_o, const void *rays_d,
                                           const uint8_t *grid, float bound, float dt_gamma,
                                           uint32_t max_steps, uint32_t N, uint32_t C,
                                           uint32_t H, uint32_t M, const void *nears,
                                           const void *fars, void *xyzs, void *dirs,
                                           void *deltas, int32_t *rays, const void *noises,
                                           const int32_t *block_sums, int zero_tail,
                                           dfhip_stream_t stream) {
    if (!march_args_ok("march_rays_train_emit", C, H, max_steps)) return DFHIP_EINVAL;
    if (N == 0) return DFHIP_OK;
    const MarchConsts k = make_consts(bound, dt_gamma, max_steps, C, H);
    DFHIP_DISPATCH(dtype, "march_rays_train_emit",
        k_march_train_emit<scalar_t><<<ceil_div(N, kMarchRaysPerBlock), 64 * kMarchRaysPerBlock,
                                       0, as_stream(stream)>>>(
            (const scalar_t *)rays_o, (const scalar_t *)rays_d, grid, k, N, M,
            (const scalar_t *)nears, (const scalar_t *)fars, (scalar_t *)xyzs,
            (scalar_t *)dirs, (scalar_t *)deltas, rays, (const scalar_t *)noises,
            block_sums, zero_tail));
    return check_launch("march_rays_train_emit");
}

extern "C" uint64_t dfhip_march_rays_train_stage_floats(uint32_t N, uint32_t max_steps) {
    return (uint64_t)N * max_steps * kStageFloats;
}

extern "C" int dfhip_march_rays_train_count_staged(
    int dtype, const void *rays_o, const void *rays_d, const uint8_t *grid, float bound,
    float dt_gamma, uint32_t max_steps, uint32_t N, uint32_t C, uint32_t H, const void *nears,
    const void *fars, int32_t *rays, int32_t *counter, const void *noises, int32_t *block_sums,
    float *stage, dfhip_stream_t stream) {
    if (!march_args_ok("march_rays_train_count_staged", C, H, max_steps)) return DFHIP_EINVAL;
    if (N == 0) return DFHIP_OK;
    if (!stage) {
        set_error("march_rays_train_count_staged: null stage");
        return DFHIP_EINVAL;
    }
    const MarchConsts k = make_consts(bound, dt_gamma, max_steps, C, H);
    DFHIP_DISPATCH(dtype, "march_rays_train_count_staged",
        (k_march_train_count<scalar_t, true><<<ceil_div(N, kMarchRaysPerBlock),
                                               64 * kMarchRaysPerBlock, 0, as_stream(stream)>>>(
            (const scalar_t *)rays_o, (const scalar_t *)rays_d, grid, k, max_steps, N,
            (const scalar_t *)nears, (const scalar_t *)fars, rays, counter,
            (const scalar_t *)noises, block_sums, stage)));
    return check_launch("march_rays_train_count_staged");
}

extern "C" int dfhip_march_rays_train_emit_staged(
    int dtype, const void *rays_d, uint32_t max_steps, uint32_t N, uint32_t M, void *xyzs,
    void *dirs, void *deltas, int32_t *rays, const int32_t *block_sums, int zero_tail,
    const float *stage, dfhip_stream_t stream) {
    if (max_steps == 0) {
        set_error("march_rays_train_emit_staged: max_steps must be > 0");
        return DFHIP_EINVAL;
    }
    if (N == 0) return DFHIP_OK;
    if (!stage || !rays_d || !rays || !block_sums || !xyzs || !deltas) {
        set_error("march_rays_train_emit_staged: null pointer");
        return DFHIP_EINVAL;
    }
    const MarchConsts k{};
    DFHIP_DISPATCH(dtype, "march_rays_train_emit_staged",
        (k_march_train_emit<scalar_t, true><<<ceil_div(N, kMarchRaysPerBlock),
                                              64 * kMarchRaysPerBlock, 0, as_stream(stream)>>>(
            nullptr, (const scalar_t *)rays_d, nullptr, k, N, M, nullptr, nullptr,
            (scalar_t *)xyzs, (scalar_t *)dirs, (scalar_t *)deltas, rays, nullptr, block_sums,
            zero_tail, stage, max_steps)));
    return check_launch("march_rays_train_emit_staged");
}

extern "C" int dfhip_march_rays_train(int dtype, const void *rays_o, const void *rays_d,
                                      const uint8_t *grid, float bound, float dt_gamma,
                                      uint32_t max_steps, uint32_t N, uint32_t C, uint32_t H,
                                      uint32_t M, const void *nears, const void *fars,
                                      void *xyzs, void *dirs, void *deltas, int32_t *rays,
                                      int32_t *counter, const void *noises,
                                      dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    int32_t *scratch = nullptr;
    const size_t bytes = sizeof(int32_t) * dfhip_march_rays_train_scratch_ints(N);
    if (hipMallocAsync((void **)&scratch, bytes, as_stream(stream)) != hipSuccess) {
        (void)hipGetLastError();
        set_error("march_rays_train: scratch allocation of %zu bytes failed", bytes);
        return DFHIP_ENOMEM;
    }
    int rc = dfhip_march_rays_train_count(dtype, rays_o, rays_d, grid, bound, dt_gamma,
                                          max_steps, N, C, H, nears, fars, rays, counter,
                                          noises, scratch, stream);
    if (rc == DFHIP_OK)
        rc = dfhip_march_rays_train_emit(dtype, rays_o, rays_d, grid, bound, dt_gamma,
                                         max_steps, N, C, H, M, nears, fars, xyzs, dirs,
                                         deltas, rays, noises, scratch, 0, stream);
    (void)hipFreeAsync(scratch, as_stream(stream));
    return rc;
}

extern "C" int dfhip_composite_rays_train_forward(int dtype, const void *sigmas,
                                                  const void *rgbs, const void *deltas,
                                                  const int32_t *rays, uint32_t M, uint32_t N,
                                                  float T_thresh, void *weights_sum,
                                                  void *depth, void *image,
                                                  dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    DFHIP_DISPATCH(dtype, "composite_rays_train_forward",
        (launch_comp_fwd<scalar_t, scalar_t>(as_stream(stream),
            (const scalar_t *)sigmas, (const scalar_t *)rgbs, (const scalar_t *)deltas, rays,
            M, N, T_thresh, (scalar_t *)weights_sum, (scalar_t *)depth, (scalar_t *)image)));
    return check_launch("composite_rays_train_forward");
}

template <bool DENSE>
static int composite_bwd_impl(const char *name, int dtype, const void *grad_weights_sum,
                              const void *grad_image, const void *sigmas, const void *rgbs,
                              const void *deltas, const int32_t *rays,
                              const void *weights_sum, const void *image, uint32_t M,
                              uint32_t N, float T_thresh, void *grad_sigmas,
                              void *grad_rgbs, dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    DFHIP_DISPATCH(dtype, name,
        (launch_comp_bwd<scalar_t, DENSE, scalar_t>(as_stream(stream),
            (const scalar_t *)grad_weights_sum, (const scalar_t *)grad_image,
            (const scalar_t *)sigmas, (const scalar_t *)rgbs, (const scalar_t *)deltas, rays,
            (const scalar_t *)weights_sum, (const scalar_t *)image, M, N, T_thresh,
            (scalar_t *)grad_sigmas, (scalar_t *)grad_rgbs, 1)));
    return check_launch(name);
}

extern "C" int dfhip_composite_rays_train_backward(
    int dtype, const void *grad_weights_sum, const void *grad_image, const void *sigmas,
    const void *rgbs, const void *deltas, const int32_t *rays, const void *weights_sum,
    const void *image, uint32_t M, uint32_t N, float T_thresh, void *grad_sigmas,
    void *grad_rgbs, dfhip_stream_t stream) {
    return composite_bwd_impl<false>("composite_rays_train_backward", dtype, grad_weights_sum,
                                     grad_image, sigmas, rgbs, deltas, rays, weights_sum, image,
                                     M, N, T_thresh, grad_sigmas, grad_rgbs, stream);
}

extern "C" int dfhip_composite_rays_train_backward_dense(
    int dtype, const void *grad_weights_sum, const void *grad_image, const void *sigmas,
    const void *rgbs, const void *deltas, const int32_t *rays, const void *weights_sum,
    const void *image, uint32_t M, uint32_t N, float T_thresh, void *grad_sigmas,
    void *grad_rgbs, dfhip_stream_t stream) {
    return composite_bwd_impl<true>("composite_rays_train_backward_dense", dtype,
                                    grad_weights_sum, grad_image, sigmas, rgbs, deltas, rays,
                                    weights_sum, image, M, N, T_thresh, grad_sigmas, grad_rgbs,
                                    stream);
}

// Mixed-precision train compositing (native): sigmas / deltas / outputs f32,
// colours (and their gradient) in `rgb_dtype` (f32 or f16).  The backward is
// the dense form; `zero_tail` = 0 leaves rows past the last ray untouched (the
// capacity-sized buffers of the device-count march, whose consumers stop at
// the live count).
extern "C" int dfhip_composite_rays_train_forward_mixed(
    int rgb_dtype, const float *sigmas, const void *rgbs, const float *deltas,
    const int32_t *rays, uint32_t M, uint32_t N, float T_thresh, float *weights_sum,
    float *depth, float *image, dfhip_stream_t stream) {
    const char *name = "composite_rays_train_forward_mixed";
    if (N == 0) return DFHIP_OK;
    hipStream_t s = as_stream(stream);
    if (rgb_dtype == DFHIP_F32)
        launch_comp_fwd<float, float>(s, sigmas, (const float *)rgbs, deltas, rays, M, N,
                                      T_thresh, weights_sum, depth, image);
    else if (rgb_dtype == DFHIP_F16)
        launch_comp_fwd<float, half_t>(s, sigmas, (const half_t *)rgbs, deltas, rays, M, N,
                                       T_thresh, weights_sum, depth, image);
    else if (rgb_dtype == DFHIP_BF16)
        launch_comp_fwd<float, bf16_t>(s, sigmas, (const bf16_t *)rgbs, deltas, rays, M, N,
                                       T_thresh, weights_sum, depth, image);
    else {
        set_error("%s: rgb dtype must be f32, f16 or bf16 (got %d)", name, rgb_dtype);
        return DFHIP_EDTYPE;
    }
    return check_launch(name);
}

extern "C" int dfhip_composite_rays_train_backward_mixed(
    int rgb_dtype, const float *grad_weights_sum, const float *grad_image, const float *sigmas,
    const void *rgbs, const float *deltas, const int32_t *rays, const float *weights_sum,
    const float *image, uint32_t M, uint32_t N, float T_thresh, float *grad_sigmas,
    void *grad_rgbs, int zero_tail, dfhip_stream_t stream) {
    const char *name = "composite_rays_train_backward_mixed";
    if (N == 0) return DFHIP_OK;
    hipStream_t s = as_stream(stream);
    if (rgb_dtype == DFHIP_F32)
        launch_comp_bwd<float, true, float>(s, grad_weights_sum, grad_image, sigmas,
                                            (const float *)rgbs, deltas, rays, weights_sum,
                                            image, M, N, T_thresh, grad_sigmas,
                                            (float *)grad_rgbs, zero_tail);
    else if (rgb_dtype == DFHIP_F16)
        launch_comp_bwd<float, true, half_t>(s, grad_weights_sum, grad_image, sigmas,
                                             (const half_t *)rgbs, deltas, rays, weights_sum,
                                             image, M, N, T_thresh, grad_sigmas,
                                             (half_t *)grad_rgbs, zero_tail);
    else if (rgb_dtype == DFHIP_BF16)
        launch_comp_bwd<float, true, bf16_t>(s, grad_weights_sum, grad_image, sigmas,
                                             (const bf16_t *)rgbs, deltas, rays, weights_sum,
                                             image, M, N, T_thresh, grad_sigmas,
                                             (bf16_t *)grad_rgbs, zero_tail);
    else {
        set_error("%s: rgb dtype must be f32, f16 or bf16 (got %d)", name, rgb_dtype);
        return DFHIP_EDTYPE;
    }
    return check_launch(name);
}

extern "C" int dfhip_march_rays(int dtype, uint32_t n_alive, uint32_t n_step,
                                const int32_t *rays_alive, const void *rays_t,
                                const void *rays_o, const void *rays_d, float bound,
                                float dt_gamma, uint32_t max_steps, uint32_t C, uint32_t H,
                                const uint8_t *grid, const void *nears, const void *fars,
                                void *xyzs, void *dirs, void *deltas, const void *noises,
                                dfhip_stream_t stream) {
    (void)nears;  // read but unused by the reference kernel (raymarching.cu:737)
    if (!march_args_ok("march_rays", C, H, max_steps)) return DFHIP_EINVAL;
    if (n_alive == 0 || n_step == 0) return DFHIP_OK;
    const MarchConsts k = make_consts(bound, dt_gamma, max_steps, C, H);
    DFHIP_DISPATCH(dtype, "march_rays",
        k_march_infer<scalar_t><<<ceil_div(n_alive, 64u), 64, 0, as_stream(stream)>>>(
            n_alive, n_step, rays_alive, (const scalar_t *)rays_t, (const scalar_t *)rays_o,
            (const scalar_t *)rays_d, k, grid, (const scalar_t *)fars, (scalar_t *)xyzs,
            (scalar_t *)dirs, (scalar_t *)deltas, (const scalar_t *)noises));
    return check_launch("march_rays");
}

extern "C" int dfhip_composite_rays(int dtype, uint32_t n_alive, uint32_t n_step,
                                    float T_thresh, int32_t *rays_alive, void *rays_t,
                                    const void *sigmas, const void *rgbs, const void *deltas,
                                    void *weights_sum, void *depth, void *image,
                                    dfhip_stream_t stream) {
    if (n_alive == 0 || n_step == 0) return DFHIP_OK;
    DFHIP_DISPATCH(dtype, "composite_rays",
        k_composite_infer<scalar_t><<<ceil_div(n_alive, 64u), 64, 0, as_stream(stream)>>>(
            n_alive, n_step, T_thresh, rays_alive, (scalar_t *)rays_t,
            (const scalar_t *)sigmas, (const scalar_t *)rgbs, (const scalar_t *)deltas,
            (scalar_t *)weights_sum, (scalar_t *)depth, (scalar_t *)image));
    return check_launch("composite_rays");
}
