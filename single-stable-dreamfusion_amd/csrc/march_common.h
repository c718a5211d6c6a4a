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
// The same for coordinates < 256 (the marchers' cells, clamped to H - 1 with
// H <= 256): the first spread step is the identity there.  The barriers keep
// the compiler from folding "(v + (v << 2)) << 1" into a quarter-rate
// v_mul_lo_u32 by 10 / 20.
__device__ __forceinline__ uint32_t spread3_8(uint32_t v) {
    v = (v + (v << 8)) & 0x0F00F00Fu;
    v = (v + (v << 4)) & 0xC30C30C3u;
    v = (v + (v << 2)) & 0x49249249u;
    return v;
}
__device__ __forceinline__ uint32_t morton3_8(uint32_t x, uint32_t y, uint32_t z) {
    uint32_t sy = spread3_8(y), sz = spread3_8(z);
    asm("" : "+v"(sy), "+v"(sz));
    return spread3_8(x) | (sy << 1) | (sz << 2);
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
    float half_H;   // 0.5f * H (exact product when H is a power of two)
    uint32_t H;
    uint32_t H_pow2;
    float mip_bound0, rbound0;  // level-0 mip bound min(1, bound) and its reciprocal
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
    k.half_H = 0.5f * (float)H;
    k.H = H;
    k.H_pow2 = (H >= 2 && (H & (H - 1)) == 0) ? 1u : 0u;
    k.mip_bound0 = fminf(1.0f, bound);   // scalbnf(1, 0) clamped as the kernels do
    k.rbound0 = 1.0f / k.mip_bound0;     // IEEE f32 division, as on the device
    return k;
}

// Cascade level of a point (raymarching.cu:42-54, max over position and dt).
__device__ __forceinline__ int mip_level(const MarchConsts &k, float x, float y, float z,
                                         float dt) {
    if (k.Cf == 1.0f) return 0;   // one cascade (bound <= 1): both terms clamp to 0
    int ep, ed;
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    frexpf(mx, &ep);
    const float lp = fminf(k.Cf - 1.0f, fmaxf(0.0f, (float)ep));
    const float md = (float)((double)(dt * k.Hf) * 0.5);
    frexpf(md, &ed);
    const float ld = fminf(k.Cf - 1.0f, fmaxf(0.0f, (float)ed));
    return max((int)lp, (int)ld);
}

// Mip level, its bound and the bound's reciprocal for a point.  With one
// cascade (the train default, bound <= 1) the level is 0 for every point and
// the bound and reciprocal are the host-evaluated constants: a uniform branch
// instead of a per-lane correctly-rounded division.
struct Mip {
    int level;
    float bound, rbound;
};
__device__ __forceinline__ Mip mip_of(const MarchConsts &k, float x, float y, float z, float dt) {
    Mip m;
    if (k.Cf == 1.0f) {
        m.level = 0;
        m.bound = k.mip_bound0;
        m.rbound = k.rbound0;
    } else {
        m.level = mip_level(k, x, y, z, dt);
        m.bound = fminf(scalbnf(1.0f, m.level), k.bound);
        m.rbound = 1.0f / m.bound;
    }
    return m;
}

// Grid cell of a clamped coordinate (raymarching.cu:374-376: the product is
// formed in double, then narrowed to float by the float clamp()).
// For a power-of-two H the double product is u scaled by a power of two, so the
// f32 product u * (H/2) has the same bits (no overflow at |u| <= 2).
__device__ __forceinline__ int cell_of(const MarchConsts &k, float c, float rbound) {
    const float u = fmaf(c, rbound, 1.0f);
    const float v = k.H_pow2 ? u * k.half_H : (float)(0.5 * (double)u * (double)k.H);
    return (int)clampf(v, 0.0f, k.Hm1);
}

// Bitfield index of a cell (raymarching.cu:377-378: the f32 fma of the level
// offset and the Morton code).  With one cascade the level is 0 and, for
// H <= 256, the code is < 2^24, so the fma returns the code itself; both
// branches are uniform.
__device__ __forceinline__ uint32_t grid_index(const MarchConsts &k, int level, int nx, int ny,
                                               int nz) {
    if (k.H <= 256u) {
        const uint32_t m = morton3_8((uint32_t)nx, (uint32_t)ny, (uint32_t)nz);
        if (k.Cf == 1.0f) return m;
        return (uint32_t)fmaf((float)level, k.H3, (float)m);
    }
    return (uint32_t)fmaf((float)level, k.H3, (float)morton3(nx, ny, nz));
}

// floor(n / d) for a quotient below ~2^16 (n < 2^30, 1 <= d < 2^24): the f32
// estimate with an approximate reciprocal rd ~ 1/d is within one of the
// quotient, and one 24-bit multiply fixes it (no quarter-rate integer
// division sequence).
__device__ __forceinline__ uint32_t small_udiv(uint32_t n, uint32_t d, float rd) {
    uint32_t q = (uint32_t)((float)n * rd);
    const uint32_t p = __umul24(q, d);
    if (p > n) q -= 1u;
    else if (n - p >= d) q += 1u;
    return q;
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

// Slab intersection of a ray with the box b = (x0, y0, z0, x1, y1, z1)
// (raymarching.cu:104-145): false on a miss, else the entry / exit t with the
// entry raised to min_near.
__device__ __forceinline__ bool ray_aabb(const Ray &r, const float b[6], float min_near,
                                         float &near, float &far) {
    float lo = (b[0] - r.ox) * r.rdx, hi = (b[3] - r.ox) * r.rdx;
    if (lo > hi) { float s = lo; lo = hi; hi = s; }
    float lo_y = (b[1] - r.oy) * r.rdy, hi_y = (b[4] - r.oy) * r.rdy;
    if (lo_y > hi_y) { float s = lo_y; lo_y = hi_y; hi_y = s; }
    if (lo > hi_y || lo_y > hi) return false;
    if (lo_y > lo) lo = lo_y;
    if (hi_y < hi) hi = hi_y;
    float lo_z = (b[2] - r.oz) * r.rdz, hi_z = (b[5] - r.oz) * r.rdz;
    if (lo_z > hi_z) { float s = lo_z; lo_z = hi_z; hi_z = s; }
    if (lo > hi_z || lo_z > hi) return false;
    if (lo_z > lo) lo = lo_z;
    if (hi_z < hi) hi = hi_z;
    if (lo < min_near) lo = min_near;
    near = lo;
    far = hi;
    return true;
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
        const Mip mp = mip_of(k, x, y, z, dt);
        const int level = mp.level;
        const float mip_bound = mp.bound;
        const float rbound = mp.rbound;
        const int nx = cell_of(k, x, rbound);
        const int ny = cell_of(k, y, rbound);
        const int nz = cell_of(k, z, rbound);
        const uint32_t idx = grid_index(k, level, nx, ny, nz);
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
// One iteration of that loop: returns 2 if t >= far (nothing done), 1 with
// the sample (position, dt, t - last_t; t and last_t advanced) when the cell
// at t is occupied, else 0 after the skip to the cell's far face.
template <typename Occ>
__device__ __forceinline__ int march_step(const MarchConsts &k, const Ray &r, Occ occupied,
                                          float &t, float &last_t, float far, float (&xyz)[3],
                                          float &dt_out, float &dl_out) {
    if (!(t < far)) return 2;
    const float x = clampf(fmaf(t, r.dx, r.ox), -k.bound, k.bound);
    const float y = clampf(fmaf(t, r.dy, r.oy), -k.bound, k.bound);
    const float z = clampf(fmaf(t, r.dz, r.oz), -k.bound, k.bound);
    const float dt = clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
    const Mip mp = mip_of(k, x, y, z, dt);
    const int level = mp.level;
    const float mip_bound = mp.bound;
    const float rbound = mp.rbound;
    const int nx = cell_of(k, x, rbound);
    const int ny = cell_of(k, y, rbound);
    const int nz = cell_of(k, z, rbound);
    const uint32_t idx = grid_index(k, level, nx, ny, nz);
    if (occupied(idx)) {
        xyz[0] = x;
        xyz[1] = y;
        xyz[2] = z;
        t += dt;
        dt_out = dt;
        dl_out = t - last_t;
        last_t = t;
        return 1;
    }
    const float tx = face_dist(k, nx, r.dx, r.rdx, x, mip_bound);
    const float ty = face_dist(k, ny, r.dy, r.rdy, y, mip_bound);
    const float tz = face_dist(k, nz, r.dz, r.rdz, z, mip_bound);
    const float tt = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    do {
        t += clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
    } while (t < tt);
    return 0;
}

// Up to K iterations of march_step in one call, for empty space: the skip
// target of a cell does not depend on its occupancy bit, so the K candidate
// points the loop would visit if every cell were empty (each the first t of
// the dt sequence at or past the previous cell's far face) are computed
// first and their K bitfield bytes loaded together; the first occupied
// candidate is then taken as march_step takes it, and the candidates after it
// are dropped.  Returns 1 with the sample, 0 after K empty cells (t at the
// last one's skip target), 2 when t reached far before an occupied cell (t
// at that skip target).  The same t sequence, samples and deltas as K calls
// of march_step; one load latency per K cells instead of K.
template <int K>
__device__ __forceinline__ int march_step_ahead(const MarchConsts &k, const Ray &r,
                                                const uint8_t *__restrict__ grid, float &t,
                                                float &last_t, float far, float (&xyz)[3],
                                                float &dt_out, float &dl_out) {
    if (!(t < far)) return 2;
    float tc[K];
    uint32_t idx[K];
    int n = 0;
    float tn = t;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        if (i > 0 && !(tn < far)) break;
        tc[i] = tn;
        const float x = clampf(fmaf(tn, r.dx, r.ox), -k.bound, k.bound);
        const float y = clampf(fmaf(tn, r.dy, r.oy), -k.bound, k.bound);
        const float z = clampf(fmaf(tn, r.dz, r.oz), -k.bound, k.bound);
        const float dt = clampf(tn * k.dt_gamma, k.dt_min, k.dt_max);
        const Mip mp = mip_of(k, x, y, z, dt);
        const int nx = cell_of(k, x, mp.rbound);
        const int ny = cell_of(k, y, mp.rbound);
        const int nz = cell_of(k, z, mp.rbound);
        idx[i] = grid_index(k, mp.level, nx, ny, nz);
        n = i + 1;
        const float tx = face_dist(k, nx, r.dx, r.rdx, x, mp.bound);
        const float ty = face_dist(k, ny, r.dy, r.rdy, y, mp.bound);
        const float tz = face_dist(k, nz, r.dz, r.rdz, z, mp.bound);
        const float tt = tn + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
        do {
            tn += clampf(tn * k.dt_gamma, k.dt_min, k.dt_max);
        } while (tn < tt);
    }
    uint32_t bits[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        bits[i] = i < n ? ((uint32_t)grid[idx[i] >> 3] >> (idx[i] & 7u)) & 1u : 0u;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        if (bits[i]) {
            const float ts = tc[i];
            xyz[0] = clampf(fmaf(ts, r.dx, r.ox), -k.bound, k.bound);
            xyz[1] = clampf(fmaf(ts, r.dy, r.oy), -k.bound, k.bound);
            xyz[2] = clampf(fmaf(ts, r.dz, r.oz), -k.bound, k.bound);
            const float dt = clampf(ts * k.dt_gamma, k.dt_min, k.dt_max);
            t = ts + dt;
            dt_out = dt;
            dl_out = t - last_t;
            last_t = t;
            return 1;
        }
    }
    t = tn;
    return n < K ? 2 : 0;
}

template <typename Occ>
__device__ __forceinline__ bool march_next_f(const MarchConsts &k, const Ray &r, Occ occupied,
                                             float &t, float &last_t, float far,
                                             float (&xyz)[3], float &dt_out, float &dl_out) {
    for (;;) {
        const int st = march_step(k, r, occupied, t, last_t, far, xyz, dt_out, dl_out);
        if (st != 0) return st == 1;
    }
}

__device__ __forceinline__ bool march_next(const MarchConsts &k, const Ray &r,
                                           const uint8_t *__restrict__ grid, float &t,
                                           float &last_t, float far, float (&xyz)[3],
                                           float &dt_out, float &dl_out) {
    return march_next_f(
        k, r, [&](uint32_t idx) { return ((grid[idx >> 3] >> (idx & 7)) & 1) != 0; }, t, last_t,
        far, xyz, dt_out, dl_out);
}

// ---------------------------------------------------------------- wave march
// One ray per wave64 (the train marcher, raymarching.hip).  Both branches of
// the reference loop advance t by dt(t) = clamp(t*dt_gamma, dt_min, dt_max)
// per step (raymarching.cu:380-398), so the t values a ray can visit form a
// fixed sequence t_{j+1} = fl(t_j + dt(t_j)).  A window of 64 consecutive
// candidates is evaluated at once, one per lane (position, cell, occupancy
// bit, far-face distance), and the reference's visit order is then replayed
// on the wave's ballots: a run of occupied candidates is taken as a block and
// each skip jumps to the first candidate with t >= tt.  Visited samples,
// counts and deltas are the serial loop's, bit for bit.

// Lane j's candidate t_j, j steps after t_base; returns the window length L
// (lanes >= L hold no candidate) and, when the window is arithmetic, the
// bit pattern step `inc` (else 0).  dt_gamma == 0 (the train default) inside
// one binade: t_base + j*dt rounds to t_base + j*inc ulps exactly, with
// inc = rint(dt/ulp) unless dt/ulp is a tie; the window stops before the
// binade ends.  Otherwise lane j repeats the reference's f32 additions.
__device__ __forceinline__ int wave_window_t(const MarchConsts &k, float t_base, int lane,
                                             float &tj, uint32_t &inc, float &rinc) {
    if (k.dt_gamma == 0.0f) {
        const uint32_t b0 = __float_as_uint(t_base);
        const uint32_t ex = b0 >> 23;
        if (b0 >= 0x00800000u && b0 < 0x7F800000u) {   // positive, normal, finite
            const float dt = clampf(0.0f, k.dt_min, k.dt_max);
            const float D = ldexpf(dt, 150 - (int)ex);   // dt in ulps of t_base
            const float Dr = rintf(D);
            if (D >= 0.5f && D < 8388608.0f && fabsf(D - Dr) != 0.5f) {
                inc = (uint32_t)Dr;
                rinc = __builtin_amdgcn_rcpf(Dr);
                // room = rem / inc + 1 candidates before the binade ends
                const uint32_t rem = 0x7FFFFFu - (b0 & 0x7FFFFFu);
                tj = __uint_as_float(b0 + (uint32_t)lane * inc);
                if (rem >= 63u * inc) return 64;
                return (int)small_udiv(rem, inc, rinc) + 1;
            }
        }
    }
    inc = 0;
    rinc = 0.0f;
    float t = t_base;
    for (int i = 0; i < lane; ++i) t += clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
    tj = t;
    return 64;
}

__device__ __forceinline__ float lane_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ uint64_t lanes_below(int j) {
    return j >= 64 ? ~0ull : ((1ull << j) - 1ull);
}
__device__ __forceinline__ int top_lane(uint64_t m) { return 63 - __clzll((long long)m); }

// March one ray with the whole wave (every lane passes the same ray; call from
// wave-uniform control flow).  Calls emit(i, x, y, z, dt, dl) on each lane
// holding the ray's i-th occupied sample (i < limit) and returns the sample
// count: the serial march()'s samples and return value, bit for bit.
//
// Per window each lane j gets its successor in the reference's visit order:
// j+1 if occupied, else the first lane with t >= tt_j (64: beyond the
// window).  The lanes actually visited are the successor chain from the start
// lane, found with binary lifting (lane m computes the m-th chain node in six
// shuffle rounds) instead of a serial walk over the skips.
template <typename Emit>
__device__ __forceinline__ uint32_t march_wave(const MarchConsts &k, const Ray &r,
                                               const uint8_t *__restrict__ grid, float t0,
                                               float far, uint32_t limit, Emit emit) {
    __shared__ uint8_t s_vis[1024];   // one 64-lane flag row per wave (<= 16 waves)
    const int lane = (int)(threadIdx.x & 63);
    uint8_t *vis = s_vis + (threadIdx.x & ~63u);
    uint32_t count = 0;
    float last_t = t0;          // t after the previous sample (deltas[1])
    float t_base = t0;          // candidate 0 of the window
    float pend = -INFINITY;     // a skip in flight: resume at the first t >= pend
    if (limit == 0 || !(t0 < far)) return 0;
    for (;;) {
        float tj, rinc;
        uint32_t inc;
        const int L = wave_window_t(k, t_base, lane, tj, inc, rinc);
        const bool valid = lane < L && tj < far;
        const uint64_t vmask = __ballot(valid);
        const int Lf = __popcll(vmask);   // t is increasing: a lane prefix

        const float dt = clampf(tj * k.dt_gamma, k.dt_min, k.dt_max);
        const float x = clampf(fmaf(tj, r.dx, r.ox), -k.bound, k.bound);
        const float y = clampf(fmaf(tj, r.dy, r.oy), -k.bound, k.bound);
        const float z = clampf(fmaf(tj, r.dz, r.oz), -k.bound, k.bound);
        const Mip mp = mip_of(k, x, y, z, dt);
        const int level = mp.level;
        const float mip_bound = mp.bound;
        const float rbound = mp.rbound;
        const int nx = cell_of(k, x, rbound);
        const int ny = cell_of(k, y, rbound);
        const int nz = cell_of(k, z, rbound);
        bool occ = false;
        if (valid) {
            const uint32_t idx = grid_index(k, level, nx, ny, nz);
            occ = (grid[idx >> 3] >> (idx & 7)) & 1;
        }
        const uint64_t omask = __ballot(occ);
        const float tx = face_dist(k, nx, r.dx, r.rdx, x, mip_bound);
        const float ty = face_dist(k, ny, r.dy, r.rdy, y, mip_bound);
        const float tz = face_dist(k, nz, r.dz, r.rdz, z, mip_bound);
        const float tt = tj + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));

        // successor of each lane (64 = beyond the valid lanes)
        int nxt;
        if (occ) {
            nxt = lane + 1;
        } else if (inc != 0) {
            // t_i >= tt  <=>  bits(t_i) >= bits(tt) for positive floats
            // need = ceil((bt - b0) / inc), only below 65 matters
            const uint32_t b0 = __float_as_uint(t_base), bt = __float_as_uint(tt);
            const uint32_t n = bt > b0 ? bt - b0 : 0u;
            const uint32_t need = n > 64u * inc ? 65u : small_udiv(n + inc - 1u, inc, rinc);
            nxt = (int)min(max(need, (uint32_t)lane + 1u), 64u);
        } else {
            int lo = lane + 1, hi = 64;   // first lane in [lo, hi) with t >= tt
#pragma unroll
            for (int it = 0; it < 7; ++it) {
                const int mid = (lo + hi) >> 1;
                const float tm = __shfl(tj, mid & 63, 64);
                const bool ge = tm >= tt;
                if (lo < hi) {
                    if (ge) hi = mid;
                    else lo = mid + 1;
                }
            }
            nxt = lo;
        }
        if (nxt >= Lf) nxt = 64;

        // start lane of the chain
        int s0;
        if (pend == -INFINITY) {
            s0 = Lf > 0 ? 0 : 64;
        } else {
            const uint64_t m = __ballot(valid && tj >= pend);
            s0 = m ? __ffsll((long long)m) - 1 : 64;
        }

        uint64_t V = 0;   // visited lanes
        if (s0 < 64) {
            // P[b] = successor^(2^b); lane m follows the chain m steps from s0
            // (raw ds_bpermute on byte addresses measured 2 % slower)
            int P[6];
            P[0] = nxt;
#pragma unroll
            for (int b = 1; b < 6; ++b) {
                const int q = __shfl(P[b - 1], P[b - 1] & 63, 64);
                P[b] = P[b - 1] >= 64 ? 64 : q;
            }
            int node = s0;
#pragma unroll
            for (int b = 0; b < 6; ++b) {
                const int q = __shfl(P[b], node & 63, 64);
                if ((lane >> b) & 1) node = node >= 64 ? 64 : q;
            }
            vis[lane] = 0;
            __builtin_amdgcn_wave_barrier();
            if (node < 64) vis[node] = 1;
            __builtin_amdgcn_wave_barrier();
            V = __ballot(vis[lane] != 0);
        }

        bool done;
        if (V) {
            const int u = top_lane(V);
            const float tt_u = lane_f(tt, u);
            done = Lf < L;
            if (!done) pend = ((omask >> u) & 1ull) ? -INFINITY : tt_u;
        } else {
            done = Lf < L;   // pend (if any) carries to the next window
        }

        uint64_t E = V & omask;   // emitted, in visit (= lane) order
        const uint32_t room = limit - count;
        if ((uint32_t)__popcll(E) >= room) {
            for (uint32_t i = (uint32_t)__popcll(E); i > room; --i) E &= ~(1ull << top_lane(E));
            done = true;
        }
        if (E) {
            const float tn = tj + dt;   // t after taking this sample
            const uint64_t below = E & lanes_below(lane);
            const int prev = below ? top_lane(below) : lane;
            const float tprev = __shfl(tn, prev, 64);
            if ((E >> lane) & 1ull) {
                emit(count + (uint32_t)__popcll(below), x, y, z, dt,
                     tn - (below ? tprev : last_t));
            }
            last_t = lane_f(tn, top_lane(E));
            count += (uint32_t)__popcll(E);
        }
        if (done) break;
        // candidate L = candidate L-1 plus one reference step
        const float tl = lane_f(tj, L - 1);
        t_base = tl + clampf(tl * k.dt_gamma, k.dt_min, k.dt_max);
    }
    return count;
}
}  // namespace rm
}  // namespace dfhip
