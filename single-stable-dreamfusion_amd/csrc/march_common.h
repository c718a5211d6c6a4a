// Occupancy-grid marcher shared by the train / inference marchers
// (raymarching.hip) and the fused inference renderer (render.hip).
// Behavioural spec: reference raymarching/src/raymarching.cu:19-81, 337-400.
// Every multiply-add nvcc contracts is an explicit fmaf(); compile with
// -ffp-contract=off (see raymarching.hip).
#pragma once

#include "common.h"

#include <float.h>
#include <math.h>

namespace dfhip {
namespace rm {

constexpr float kSqrt3 = 1.7320508075688772f;
constexpr float kInvPi = 0.3183098861837907f;

__device__ __forceinline__ float clampf(float x, float lo, float hi) {
    return fminf(hi, fmaxf(lo, x));
}

// raymarching.cu:56-71 (expand_bits / morton3D) — same integer semantics for
// every uint32 input (the multiplies are written as shift-adds).
__host__ __device__ __forceinline__ uint32_t spread3(uint32_t v) {
    v = (v + (v << 16)) & 0xFF0000FFu;
    v = (v + (v << 8)) & 0x0F00F00Fu;
    v = (v + (v << 4)) & 0xC30C30C3u;
    v = (v + (v << 2)) & 0x49249249u;
    return v;
}
__host__ __device__ __forceinline__ uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    return spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
}
// raymarching.cu:73-81
__host__ __device__ __forceinline__ uint32_t compact3(uint32_t v) {
    v &= 0x49249249u;
    v = (v | (v >> 2)) & 0xC30C30C3u;
    v = (v | (v >> 4)) & 0x0F00F00Fu;
    v = (v | (v >> 8)) & 0xFF0000FFu;
    v = (v | (v >> 16)) & 0x0000FFFFu;
    return v;
}

// Per-launch constants of the marcher (raymarching.cu:337-346).
struct MarchConsts {
    float bound, dt_gamma, dt_min, dt_max, rH, H3, Hf, Cf, Hm1;
    uint32_t H;
};

inline MarchConsts make_consts(float bound, float dt_gamma, uint32_t max_steps,
                               uint32_t C, uint32_t H) {
    MarchConsts k;
    k.bound = bound;
    k.dt_gamma = dt_gamma;
    k.dt_min = (2.0f * kSqrt3) / (float)max_steps;
    k.dt_max = (2.0f * kSqrt3 * (float)(1u << (C - 1))) / (float)H;
    k.rH = 1.0f / (float)H;
    k.H3 = (float)(H * H * H);
    k.Hf = (float)H;
    k.Cf = (float)C;
    k.Hm1 = (float)(H - 1);
    k.H = H;
    return k;
}

// Cascade level of a point (raymarching.cu:42-54, max over position and dt).
__device__ __forceinline__ int mip_level(const MarchConsts &k, float x, float y, float z,
                                         float dt) {
    int ep, ed;
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    frexpf(mx, &ep);
    const float lp = fminf(k.Cf - 1.0f, fmaxf(0.0f, (float)ep));
    const float md = (float)((double)(dt * k.Hf) * 0.5);
    frexpf(md, &ed);
    const float ld = fminf(k.Cf - 1.0f, fmaxf(0.0f, (float)ed));
    return max((int)lp, (int)ld);
}

// Grid cell of a clamped coordinate (raymarching.cu:374-376: the product is
// formed in double, then narrowed to float by the float clamp()).
__device__ __forceinline__ int cell_of(const MarchConsts &k, float c, float rbound) {
    const float u = fmaf(c, rbound, 1.0f);
    const float v = (float)(0.5 * (double)u * (double)k.H);
    return (int)clampf(v, 0.0f, k.Hm1);
}

// Distance (in t) to the far face of the current cell along one axis
// (raymarching.cu:390-392, nvcc contraction model).
__device__ __forceinline__ float face_dist(const MarchConsts &k, int n, float d, float rd,
                                           float c, float mip_bound) {
    const float a = fmaf(0.5f, copysignf(1.0f, d), (float)n + 0.5f);
    const float b = fmaf(a * k.rH, 2.0f, -1.0f);
    return fmaf(b, mip_bound, -c) * rd;
}

struct Ray {
    float ox, oy, oz, dx, dy, dz, rdx, rdy, rdz;
};

template <typename scalar_t>
__device__ __forceinline__ Ray load_ray(const scalar_t *o, const scalar_t *d) {
    Ray r;
    r.ox = to_f(o[0]); r.oy = to_f(o[1]); r.oz = to_f(o[2]);
    r.dx = to_f(d[0]); r.dy = to_f(d[1]); r.dz = to_f(d[2]);
    r.rdx = 1.0f / r.dx; r.rdy = 1.0f / r.dy; r.rdz = 1.0f / r.dz;
    return r;
}

// The march loop shared by the count pass, the emit pass and the inference
// marcher (raymarching.cu:359-400, 427-479, 750-804).  Visits the same
// t-sequence in every mode.  WRITE: store each occupied sample at out[step].
// Returns the number of occupied samples taken (<= limit).
template <bool WRITE, typename scalar_t>
__device__ __forceinline__ uint32_t march(const MarchConsts &k, const Ray &r,
                                          const uint8_t *__restrict__ grid, float t,
                                          float far, uint32_t limit, scalar_t *xyzs,
                                          scalar_t *dirs, scalar_t *deltas,
                                          float *t_out) {
    uint32_t step = 0;
    float last_t = t;
    while (t < far && step < limit) {
        const float x = clampf(fmaf(t, r.dx, r.ox), -k.bound, k.bound);
        const float y = clampf(fmaf(t, r.dy, r.oy), -k.bound, k.bound);
        const float z = clampf(fmaf(t, r.dz, r.oz), -k.bound, k.bound);
        const float dt = clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
        const int level = mip_level(k, x, y, z, dt);
        const float mip_bound = fminf(scalbnf(1.0f, level), k.bound);
        const float rbound = 1.0f / mip_bound;
        const int nx = cell_of(k, x, rbound);
        const int ny = cell_of(k, y, rbound);
        const int nz = cell_of(k, z, rbound);
        const uint32_t idx =
            (uint32_t)fmaf((float)level, k.H3, (float)morton3(nx, ny, nz));
        const bool occ = (grid[idx >> 3] >> (idx & 7)) & 1;
        if (occ) {
            if (WRITE) {
                scalar_t *px = xyzs + 3 * step;
                scalar_t *pd = dirs + 3 * step;
                scalar_t *pl = deltas + 2 * step;
                px[0] = from_f<scalar_t>(x);
                px[1] = from_f<scalar_t>(y);
                px[2] = from_f<scalar_t>(z);
                pd[0] = from_f<scalar_t>(r.dx);
                pd[1] = from_f<scalar_t>(r.dy);
                pd[2] = from_f<scalar_t>(r.dz);
                t += dt;
                pl[0] = from_f<scalar_t>(dt);
                pl[1] = from_f<scalar_t>(t - last_t);
                last_t = t;
            } else {
                t += dt;
            }
            ++step;
        } else {
            const float tx = face_dist(k, nx, r.dx, r.rdx, x, mip_bound);
            const float ty = face_dist(k, ny, r.dy, r.rdy, y, mip_bound);
            const float tz = face_dist(k, nz, r.dz, r.rdz, z, mip_bound);
            const float tt = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
            do {
                t += clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
            } while (t < tt);
        }
    }
    if (t_out) *t_out = t;
    return step;
}

// One step of the same march in register form (the fused inference renderer,
// render.hip): advance from t to the next occupied sample before `far`.
// On success returns true with the sample position, dt and t - last_t
// (deltas[0], deltas[1] of raymarching.cu:778-779) and t, last_t advanced as
// the reference's loop leaves them; else t >= far.
__device__ __forceinline__ bool march_next(const MarchConsts &k, const Ray &r,
                                           const uint8_t *__restrict__ grid, float &t,
                                           float &last_t, float far, float (&xyz)[3],
                                           float &dt_out, float &dl_out) {
    while (t < far) {
        const float x = clampf(fmaf(t, r.dx, r.ox), -k.bound, k.bound);
        const float y = clampf(fmaf(t, r.dy, r.oy), -k.bound, k.bound);
        const float z = clampf(fmaf(t, r.dz, r.oz), -k.bound, k.bound);
        const float dt = clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
        const int level = mip_level(k, x, y, z, dt);
        const float mip_bound = fminf(scalbnf(1.0f, level), k.bound);
        const float rbound = 1.0f / mip_bound;
        const int nx = cell_of(k, x, rbound);
        const int ny = cell_of(k, y, rbound);
        const int nz = cell_of(k, z, rbound);
        const uint32_t idx =
            (uint32_t)fmaf((float)level, k.H3, (float)morton3(nx, ny, nz));
        if ((grid[idx >> 3] >> (idx & 7)) & 1) {
            xyz[0] = x;
            xyz[1] = y;
            xyz[2] = z;
            t += dt;
            dt_out = dt;
            dl_out = t - last_t;
            last_t = t;
            return true;
        }
        const float tx = face_dist(k, nx, r.dx, r.rdx, x, mip_bound);
        const float ty = face_dist(k, ny, r.dy, r.rdy, y, mip_bound);
        const float tz = face_dist(k, nz, r.dz, r.rdz, z, mip_bound);
        const float tt = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
        do {
            t += clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
        } while (t < tt);
    }
    return false;
}

}  // namespace rm
}  // namespace dfhip
