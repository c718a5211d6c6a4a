/*
 * oracle.c — CPU restatement of the reference's NeRF hot-path kernels.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this; the product path never does.
 *
 * Restates (scalar C, one ray / sample at a time):
 *   raymarching/src/raymarching.cu:42-914   (near/far, sph, morton, packbits,
 *                                            march train/infer, composite)
 *   gridencoder/src/gridencoder.cu:35-342   (grid fwd incl. dy_dx, bwd)
 *   freqencoder/src/freqencoder.cu:28-94
 *
 * Parity status: UNPINNED against the reference itself.  The reference ships
 * no tests, fixtures or golden vectors, and building or
 * importing its CUDA extensions was refused by the environment (SURVEY.md
 * §8c), so this restatement is checked against analytic known-answer tests
 * (tests/test_oracle_kat.py) and line-by-line review of the .cu text only.
 *
 * Numerics: compiled with -ffp-contract=off; every multiply-add that nvcc
 * contracts by default (-fmad=true, LLVM DAG-combine order: in a*b + c*d the
 * left product is fused) is an explicit fmaf().  __expf is modelled as the
 * gfx950/CUDA hardware form exp2(x * log2e) with the product rounded to f32.
 * c10::Half arithmetic (gridencoder.cu:142,165) is emulated bit-exactly with
 * explicit round-to-nearest-even float <-> binary16 conversions.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ helpers */

static float clampf_(float x, float lo, float hi) { return fminf(hi, fmaxf(lo, x)); }

/* raymarching.cu:56-71 */
static uint32_t expand_bits_(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
static uint32_t morton_(uint32_t x, uint32_t y, uint32_t z) {
    return expand_bits_(x) | (expand_bits_(y) << 1) | (expand_bits_(z) << 2);
}
/* raymarching.cu:73-81 */
static uint32_t morton_inv_(uint32_t x) {
    x &= 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

/* __expf as the hardware evaluates it: v_exp_f32(x * 0x1.715476p+0) */
static float fast_expf_(float x) {
    const float y = x * 0x1.715476p+0f;
    return (float)exp2((double)y);
}

/* IEEE binary16 <-> float, round to nearest even (torch.half semantics) */
static uint16_t f2h_(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t e = (x >> 23) & 0xff;
    uint32_t m = x & 0x7fffffu;
    if (e == 0xff) return (uint16_t)(sign | 0x7c00u | (m ? 0x200u : 0));
    int32_t exp = (int32_t)e - 127 + 15;
    if (exp >= 0x1f) return (uint16_t)(sign | 0x7c00u);
    if (exp <= 0) {
        if (exp < -10) return (uint16_t)sign;
        m |= 0x800000u;
        const uint32_t shift = (uint32_t)(14 - exp);
        uint32_t hm = m >> shift;
        const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (hm & 1))) hm++;
        return (uint16_t)(sign | hm);
    }
    uint32_t hm = m >> 13;
    const uint32_t rem = m & 0x1fffu;
    uint32_t h = sign | ((uint32_t)exp << 10) | hm;
    if (rem > 0x1000u || (rem == 0x1000u && (hm & 1))) h++;
    return (uint16_t)h;
}
static float h2f_(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ffu, x;
    if (e == 0) {
        if (m == 0) {
            x = sign;
        } else {
            int k = -1;
            do { k++; m <<= 1; } while (!(m & 0x400u));
            x = sign | ((uint32_t)(127 - 15 - k) << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 0x1f) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((e + 127 - 15) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}
float orc_round_half(float f) { return h2f_(f2h_(f)); }

/* bfloat16 <-> float, round to nearest even (torch.bfloat16 / v_cvt_pk_bf16_f32) */
static uint16_t f2bf_(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    if ((x & 0x7f800000u) == 0x7f800000u && (x & 0x7fffffu))
        return (uint16_t)((x >> 16) | 0x40u); /* quiet NaN */
    x += 0x7fffu + ((x >> 16) & 1u);
    return (uint16_t)(x >> 16);
}
static float bf2f_(uint16_t h) {
    const uint32_t x = (uint32_t)h << 16;
    float f;
    memcpy(&f, &x, 4);
    return f;
}
float orc_round_bf16(float f) { return bf2f_(f2bf_(f)); }
void orc_f32_to_f16(const float *src, uint16_t *dst, int64_t n) {
    for (int64_t i = 0; i < n; ++i) dst[i] = f2h_(src[i]);
}
void orc_f16_to_f32(const uint16_t *src, float *dst, int64_t n) {
    for (int64_t i = 0; i < n; ++i) dst[i] = h2f_(src[i]);
}

/* ------------------------------------------------------------- utilities */

/* raymarching.cu:91-145 */
void orc_near_far_from_aabb(const float *rays_o, const float *rays_d, const float *aabb,
                            uint32_t N, float min_near, float *nears, float *fars) {
    for (uint32_t n = 0; n < N; ++n) {
        const float *o = rays_o + 3 * (size_t)n, *d = rays_d + 3 * (size_t)n;
        const float rdx = 1 / d[0], rdy = 1 / d[1], rdz = 1 / d[2];
        float near = (aabb[0] - o[0]) * rdx, far = (aabb[3] - o[0]) * rdx, s;
        if (near > far) { s = near; near = far; far = s; }
        float ny = (aabb[1] - o[1]) * rdy, fy = (aabb[4] - o[1]) * rdy;
        if (ny > fy) { s = ny; ny = fy; fy = s; }
        if (near > fy || ny > far) { nears[n] = fars[n] = FLT_MAX; continue; }
        if (ny > near) near = ny;
        if (fy < far) far = fy;
        float nz = (aabb[2] - o[2]) * rdz, fz = (aabb[5] - o[2]) * rdz;
        if (nz > fz) { s = nz; nz = fz; fz = s; }
        if (near > fz || nz > far) { nears[n] = fars[n] = FLT_MAX; continue; }
        if (nz > near) near = nz;
        if (fz < far) far = fz;
        if (near < min_near) near = min_near;
        nears[n] = near;
        fars[n] = far;
    }
}

/* raymarching.cu:162-198 */
void orc_sph_from_ray(const float *rays_o, const float *rays_d, float radius, uint32_t N,
                      float *coords) {
    const float rpi = 0.3183098861837907f;
    for (uint32_t n = 0; n < N; ++n) {
        const float ox = rays_o[3 * n], oy = rays_o[3 * n + 1], oz = rays_o[3 * n + 2];
        const float dx = rays_d[3 * n], dy = rays_d[3 * n + 1], dz = rays_d[3 * n + 2];
        const float A = fmaf(dz, dz, fmaf(dx, dx, dy * dy));
        const float B = fmaf(oz, dz, fmaf(ox, dx, oy * dy));
        const float C = fmaf(-radius, radius, fmaf(oz, oz, fmaf(ox, ox, oy * oy)));
        const float t = (-B + sqrtf(fmaf(B, B, -(A * C)))) / A;
        const float x = fmaf(t, dx, ox), y = fmaf(t, dy, oy), z = fmaf(t, dz, oz);
        const float theta = atan2f(sqrtf(fmaf(x, x, z * z)), y);
        const float phi = atan2f(z, x);
        coords[2 * n] = fmaf(2 * theta, rpi, -1.0f);
        coords[2 * n + 1] = phi * rpi;
    }
}

void orc_morton3D(const int32_t *coords, uint32_t N, int32_t *indices) {
    for (uint32_t n = 0; n < N; ++n)
        indices[n] = (int32_t)morton_((uint32_t)coords[3 * n], (uint32_t)coords[3 * n + 1],
                                      (uint32_t)coords[3 * n + 2]);
}

void orc_morton3D_invert(const int32_t *indices, uint32_t N, int32_t *coords) {
    for (uint32_t n = 0; n < N; ++n) {
        const uint32_t v = (uint32_t)indices[n];
        coords[3 * n] = (int32_t)morton_inv_(v);
        coords[3 * n + 1] = (int32_t)morton_inv_(v >> 1);
        coords[3 * n + 2] = (int32_t)morton_inv_(v >> 2);
    }
}

/* raymarching.cu:267-289 */
void orc_packbits(const float *grid, uint32_t N, float thresh, uint8_t *bitfield) {
    for (uint32_t n = 0; n < N; ++n) {
        uint8_t bits = 0;
        for (int i = 0; i < 8; ++i)
            if (grid[8 * (size_t)n + i] > thresh) bits |= (uint8_t)(1u << i);
        bitfield[n] = bits;
    }
}

/* ------------------------------------------------------------- marching */

typedef struct {
    float bound, dt_gamma, dt_min, dt_max, rH, H3, Hf, Cf;
    uint32_t H;
} consts_t;

static consts_t consts_(float bound, float dt_gamma, uint32_t max_steps, uint32_t C, uint32_t H) {
    consts_t k;
    const float sqrt3 = 1.7320508075688772f;
    k.bound = bound;
    k.dt_gamma = dt_gamma;
    k.dt_min = 2 * sqrt3 / (float)max_steps;                         /* :345 */
    k.dt_max = 2 * sqrt3 * (float)(1u << (C - 1)) / (float)H;        /* :346 */
    k.rH = 1 / (float)H;
    k.H3 = (float)(H * H * H);
    k.Hf = (float)H;
    k.Cf = (float)C;
    k.H = H;
    return k;
}

/* raymarching.cu:42-54 */
static int mip_from_pos_(float x, float y, float z, float max_cascade) {
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    int e;
    frexpf(mx, &e);
    return (int)fminf(max_cascade - 1, fmaxf(0, (float)e));
}
static int mip_from_dt_(float dt, float H, float max_cascade) {
    const float mx = (float)((double)(dt * H) * 0.5);
    int e;
    frexpf(mx, &e);
    return (int)fminf(max_cascade - 1, fmaxf(0, (float)e));
}

/* One ray of raymarching.cu:341-479 (and :736-804 for inference): march from
 * t, visiting the same t-sequence in every mode.  Writes up to `limit`
 * samples into (xyzs, dirs, deltas) if they are non-NULL.  Returns the number
 * of occupied samples; *t_end receives the final t. */
static uint32_t march_one_(const consts_t *k, const float *o, const float *d,
                           const uint8_t *grid, float t, float far, uint32_t limit,
                           float *xyzs, float *dirs, float *deltas, float *t_end) {
    const float ox = o[0], oy = o[1], oz = o[2], dx = d[0], dy = d[1], dz = d[2];
    const float rdx = 1 / dx, rdy = 1 / dy, rdz = 1 / dz;
    uint32_t step = 0;
    float last_t = t;
    while (t < far && step < limit) {
        const float x = clampf_(fmaf(t, dx, ox), -k->bound, k->bound);
        const float y = clampf_(fmaf(t, dy, oy), -k->bound, k->bound);
        const float z = clampf_(fmaf(t, dz, oz), -k->bound, k->bound);
        const float dt = clampf_(t * k->dt_gamma, k->dt_min, k->dt_max);
        const int lp = mip_from_pos_(x, y, z, k->Cf), ld = mip_from_dt_(dt, k->Hf, k->Cf);
        const int level = lp > ld ? lp : ld;
        const float mip_bound = fminf(scalbnf(1.0f, level), k->bound);
        const float mip_rbound = 1 / mip_bound;
        /* 0.5 * (x * rbound + 1) * H evaluated in double, narrowed by clamp(float) */
        const int nx = (int)clampf_((float)(0.5 * (double)fmaf(x, mip_rbound, 1.0f) * (double)k->H),
                                    0.0f, (float)(k->H - 1));
        const int ny = (int)clampf_((float)(0.5 * (double)fmaf(y, mip_rbound, 1.0f) * (double)k->H),
                                    0.0f, (float)(k->H - 1));
        const int nz = (int)clampf_((float)(0.5 * (double)fmaf(z, mip_rbound, 1.0f) * (double)k->H),
                                    0.0f, (float)(k->H - 1));
        const uint32_t index = (uint32_t)fmaf((float)level, k->H3,
                                              (float)morton_((uint32_t)nx, (uint32_t)ny, (uint32_t)nz));
        const int occ = (grid[index / 8] & (1u << (index % 8))) != 0;
        if (occ) {
            if (xyzs) {
                xyzs[3 * step] = x; xyzs[3 * step + 1] = y; xyzs[3 * step + 2] = z;
                dirs[3 * step] = dx; dirs[3 * step + 1] = dy; dirs[3 * step + 2] = dz;
            }
            t += dt;
            if (xyzs) {
                deltas[2 * step] = dt;
                deltas[2 * step + 1] = t - last_t;
            }
            last_t = t;
            step++;
        } else {
            const float sx = copysignf(1.0f, dx), sy = copysignf(1.0f, dy), sz = copysignf(1.0f, dz);
            const float tx = fmaf(fmaf(fmaf(0.5f, sx, (float)nx + 0.5f) * k->rH, 2.0f, -1.0f),
                                  mip_bound, -x) * rdx;
            const float ty = fmaf(fmaf(fmaf(0.5f, sy, (float)ny + 0.5f) * k->rH, 2.0f, -1.0f),
                                  mip_bound, -y) * rdy;
            const float tz = fmaf(fmaf(fmaf(0.5f, sz, (float)nz + 0.5f) * k->rH, 2.0f, -1.0f),
                                  mip_bound, -z) * rdz;
            const float tt = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
            do {
                t += clampf_(t * k->dt_gamma, k->dt_min, k->dt_max);
            } while (t < tt);
        }
    }
    if (t_end) *t_end = t;
    return step;
}

/* raymarching.cu:311-479 in ray order.  counts[N] always written.  If xyzs
 * is non-NULL, the samples of ray n are written at rows offsets[n] .. where
 * offsets is the exclusive prefix sum of counts (the caller sizes the
 * buffers with the total returned by a first counts-only call). */
uint64_t orc_march_rays_train(const float *rays_o, const float *rays_d, const uint8_t *grid,
                              float bound, float dt_gamma, uint32_t max_steps, uint32_t N,
                              uint32_t C, uint32_t H, const float *nears, const float *fars,
                              const float *noises, int32_t *counts, float *xyzs, float *dirs,
                              float *deltas) {
    const consts_t k = consts_(bound, dt_gamma, max_steps, C, H);
    uint64_t off = 0;
    for (uint32_t n = 0; n < N; ++n) {
        const float near = nears[n], far = fars[n];
        const float t0 = fmaf(clampf_(near * k.dt_gamma, k.dt_min, k.dt_max), noises[n], near);
        const uint32_t c = march_one_(&k, rays_o + 3 * (size_t)n, rays_d + 3 * (size_t)n, grid, t0,
                                      far, max_steps, NULL, NULL, NULL, NULL);
        counts[n] = (int32_t)c;
        if (xyzs && c) {
            march_one_(&k, rays_o + 3 * (size_t)n, rays_d + 3 * (size_t)n, grid, t0, far, c,
                       xyzs + 3 * off, dirs + 3 * off, deltas + 2 * off, NULL);
        }
        off += c;
    }
    return off;
}

/* raymarching.cu:700-804 (inference).  Every slot of an alive ray is written;
 * unused slots are zero (the kernel's caller zero-fills them). */
void orc_march_rays(uint32_t n_alive, uint32_t n_step, const int32_t *rays_alive,
                    const float *rays_t, const float *rays_o, const float *rays_d, float bound,
                    float dt_gamma, uint32_t max_steps, uint32_t C, uint32_t H,
                    const uint8_t *grid, const float *fars, float *xyzs, float *dirs,
                    float *deltas, const float *noises) {
    const consts_t k = consts_(bound, dt_gamma, max_steps, C, H);
    memset(xyzs, 0, sizeof(float) * 3 * (size_t)n_alive * n_step);
    memset(dirs, 0, sizeof(float) * 3 * (size_t)n_alive * n_step);
    memset(deltas, 0, sizeof(float) * 2 * (size_t)n_alive * n_step);
    for (uint32_t n = 0; n < n_alive; ++n) {
        const int32_t id = rays_alive[n];
        float t = rays_t[id];
        t = fmaf(clampf_(t * k.dt_gamma, k.dt_min, k.dt_max), noises[n], t);
        march_one_(&k, rays_o + 3 * (size_t)id, rays_d + 3 * (size_t)id, grid, t, fars[id], n_step,
                   xyzs + 3 * (size_t)n * n_step, dirs + 3 * (size_t)n * n_step,
                   deltas + 2 * (size_t)n * n_step, NULL);
    }
}

/* ---------------------------------------------------------- compositing */

/* raymarching.cu:500-577 */
void orc_composite_rays_train_forward(const float *sigmas, const float *rgbs, const float *deltas,
                                      const int32_t *rays, uint32_t M, uint32_t N, float T_thresh,
                                      float *weights_sum, float *depth, float *image) {
    for (uint32_t n = 0; n < N; ++n) {
        const uint32_t idx = (uint32_t)rays[3 * n], off = (uint32_t)rays[3 * n + 1],
                       num = (uint32_t)rays[3 * n + 2];
        float T = 1, r = 0, g = 0, b = 0, ws = 0, t = 0, d = 0;
        if (num != 0 && off + num <= M) {
            for (uint32_t i = 0; i < num; ++i) {
                const uint32_t s = off + i;
                const float alpha = 1.0f - fast_expf_(-sigmas[s] * deltas[2 * s]);
                const float w = alpha * T;
                r = fmaf(w, rgbs[3 * s], r);
                g = fmaf(w, rgbs[3 * s + 1], g);
                b = fmaf(w, rgbs[3 * s + 2], b);
                t += deltas[2 * s + 1];
                d = fmaf(w, t, d);
                ws += w;
                T *= 1.0f - alpha;
                if (T < T_thresh) break;
            }
        }
        weights_sum[idx] = ws;
        depth[idx] = d;
        image[3 * idx] = r; image[3 * idx + 1] = g; image[3 * idx + 2] = b;
    }
}

/* raymarching.cu:601-682 (rows past the break stay as the caller left them) */
void orc_composite_rays_train_backward(const float *grad_ws, const float *grad_image,
                                       const float *sigmas, const float *rgbs,
                                       const float *deltas, const int32_t *rays,
                                       const float *weights_sum, const float *image, uint32_t M,
                                       uint32_t N, float T_thresh, float *grad_sigmas,
                                       float *grad_rgbs) {
    for (uint32_t n = 0; n < N; ++n) {
        const uint32_t idx = (uint32_t)rays[3 * n], off = (uint32_t)rays[3 * n + 1],
                       num = (uint32_t)rays[3 * n + 2];
        if (num == 0 || off + num > M) continue;
        const float gr = grad_image[3 * idx], gg = grad_image[3 * idx + 1],
                    gb = grad_image[3 * idx + 2], gw = grad_ws[idx];
        const float rf = image[3 * idx], gf = image[3 * idx + 1], bf = image[3 * idx + 2];
        const float wsf = weights_sum[idx];
        float T = 1, r = 0, g = 0, b = 0, ws = 0;
        for (uint32_t i = 0; i < num; ++i) {
            const uint32_t s = off + i;
            const float alpha = 1.0f - fast_expf_(-sigmas[s] * deltas[2 * s]);
            const float w = alpha * T;
            r = fmaf(w, rgbs[3 * s], r);
            g = fmaf(w, rgbs[3 * s + 1], g);
            b = fmaf(w, rgbs[3 * s + 2], b);
            ws += w;
            T *= 1.0f - alpha;
            grad_rgbs[3 * s] = gr * w;
            grad_rgbs[3 * s + 1] = gg * w;
            grad_rgbs[3 * s + 2] = gb * w;
            float acc = fmaf(gr, fmaf(T, rgbs[3 * s], -(rf - r)),
                             gg * fmaf(T, rgbs[3 * s + 1], -(gf - g)));
            acc = fmaf(gb, fmaf(T, rgbs[3 * s + 2], -(bf - b)), acc);
            acc = fmaf(gw, 1 - wsf, acc);
            grad_sigmas[s] = deltas[2 * s] * acc;
            if (T < T_thresh) break;
        }
        (void)ws;
    }
}

/* raymarching.cu:818-905 (in place) */
void orc_composite_rays(uint32_t n_alive, uint32_t n_step, float T_thresh, int32_t *rays_alive,
                        float *rays_t, const float *sigmas, const float *rgbs, const float *deltas,
                        float *weights_sum, float *depth, float *image) {
    for (uint32_t n = 0; n < n_alive; ++n) {
        const int32_t id = rays_alive[n];
        const float *s = sigmas + (size_t)n * n_step;
        const float *c = rgbs + 3 * (size_t)n * n_step;
        const float *dl = deltas + 2 * (size_t)n * n_step;
        float t = rays_t[id], wsum = weights_sum[id], d = depth[id];
        float r = image[3 * id], g = image[3 * id + 1], b = image[3 * id + 2];
        uint32_t step = 0;
        while (step < n_step) {
            if (dl[2 * step] == 0) break;
            const float alpha = 1.0f - fast_expf_(-s[step] * dl[2 * step]);
            const float T = 1 - wsum;
            const float w = alpha * T;
            wsum += w;
            t += dl[2 * step + 1];
            d = fmaf(w, t, d);
            r = fmaf(w, c[3 * step], r);
            g = fmaf(w, c[3 * step + 1], g);
            b = fmaf(w, c[3 * step + 2], b);
            if (T < T_thresh) break;
            step++;
        }
        if (step < n_step) rays_alive[n] = -1;
        else rays_t[id] = t;
        weights_sum[id] = wsum;
        depth[id] = d;
        image[3 * id] = r; image[3 * id + 1] = g; image[3 * id + 2] = b;
    }
}

/* ------------------------------------------------------------ grid encoder */

static const uint32_t kPrimes_[7] = {1u, 2654435761u, 805459861u, 3674653429u,
                                     2097192037u, 1434869437u, 2165219737u};

/* gridencoder.cu:54-72 */
static uint32_t grid_index_(uint32_t gridtype, int align, uint32_t hsize, uint32_t res,
                            const uint32_t *p, uint32_t D) {
    uint32_t stride = 1, index = 0;
    for (uint32_t d = 0; d < D && stride <= hsize; d++) {
        index += p[d] * stride;
        stride *= align ? res : (res + 1);
    }
    if (gridtype == 0 && stride > hsize) {
        index = 0;
        for (uint32_t d = 0; d < D; ++d) index ^= p[d] * kPrimes_[d];
    }
    return index % hsize;
}

/* gridencoder.cu:125-126: scale = exp2f(l * S) * H - 1 (contracted to an fma),
 * exp2 correctly rounded */
static float level_scale_(uint32_t l, float S, uint32_t H) {
    const float e = (float)exp2((double)((float)l * S));
    return fmaf(e, (float)H, -1.0f);
}

/* storage: 0 = f32, 1 = f16 (uint16 bits), 2 = f64 */
/* storage types: 0 f32, 1 f16, 2 f64, 3 bf16 (the C5 option; no reference
 * counterpart: accumulated in f32 like st 0, rounded to bf16 once on store) */
static double load_(const void *p, int st, size_t i) {
    if (st == 0) return ((const float *)p)[i];
    if (st == 1) return h2f_(((const uint16_t *)p)[i]);
    if (st == 3) return bf2f_(((const uint16_t *)p)[i]);
    return ((const double *)p)[i];
}
static void store_(void *p, int st, size_t i, double v) {
    if (st == 0) ((float *)p)[i] = (float)v;
    else if (st == 1) ((uint16_t *)p)[i] = f2h_((float)v);
    else if (st == 3) ((uint16_t *)p)[i] = f2bf_((float)v);
    else ((double *)p)[i] = v;
}
/* one corner contribution in the storage type's arithmetic (gridencoder.cu:165) */
static double acc_(int st, double r, float w, double g) {
    if (st == 0 || st == 3) return fmaf(w, (float)g, (float)r);
    if (st == 1) {
        const float p = h2f_(f2h_(w * (float)g));   /* Half(w * float(g)) */
        return h2f_(f2h_((float)r + p));             /* Half(float(r) + float(p)) */
    }
    return fma((double)w, g, r);
}

/* gridencoder.cu:75-223.  outputs [B, L*C] (blc != 0) or [L, B, C].
 * dy_dx [B, L*D*C] or NULL. */
void orc_grid_encode_forward(const float *inputs, const void *emb, int st, const int32_t *offsets,
                             void *outputs, uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                             float S, uint32_t H, void *dy_dx, uint32_t gridtype, int align,
                             int blc) {
    uint32_t p[8], q[8];
    float pos[8];
    for (uint32_t b = 0; b < B; ++b) {
        const float *x = inputs + (size_t)b * D;
        int oob = 0;
        for (uint32_t d = 0; d < D; ++d)
            if (x[d] < 0 || x[d] > 1) oob = 1;
        for (uint32_t l = 0; l < L; ++l) {
            const size_t obase = blc ? (size_t)b * L * C + (size_t)l * C : (size_t)l * B * C + (size_t)b * C;
            const size_t jbase = (size_t)b * D * L * C + (size_t)l * D * C;
            if (oob) {
                for (uint32_t ch = 0; ch < C; ++ch) store_(outputs, st, obase + ch, 0);
                if (dy_dx)
                    for (uint32_t i = 0; i < D * C; ++i) store_(dy_dx, st, jbase + i, 0);
                continue;
            }
            const uint32_t base = (uint32_t)offsets[l];
            const uint32_t hsize = (uint32_t)offsets[l + 1] - base;
            const float scale = level_scale_(l, S, H);
            const uint32_t res = (uint32_t)ceilf(scale) + 1;
            for (uint32_t d = 0; d < D; ++d) {
                const float v = fmaf(x[d], scale, align ? 0.0f : 0.5f);
                p[d] = (uint32_t)floorf(v);
                pos[d] = v - (float)p[d];
            }
            double res_c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (uint32_t k = 0; k < (1u << D); ++k) {
                float w = 1;
                for (uint32_t d = 0; d < D; ++d) {
                    if (k & (1u << d)) { w *= pos[d]; q[d] = p[d] + 1; }
                    else { w *= 1 - pos[d]; q[d] = p[d]; }
                }
                const uint32_t row = grid_index_(gridtype, align, hsize, res, q, D);
                for (uint32_t ch = 0; ch < C; ++ch)
                    res_c[ch] = acc_(st, res_c[ch], w, load_(emb, st, (size_t)(base + row) * C + ch));
            }
            for (uint32_t ch = 0; ch < C; ++ch) store_(outputs, st, obase + ch, res_c[ch]);
            if (!dy_dx) continue;
            for (uint32_t gd = 0; gd < D; ++gd) {
                double rg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                for (uint32_t k = 0; k < (1u << (D - 1)); ++k) {
                    float w = scale;
                    for (uint32_t nd = 0; nd < D - 1; ++nd) {
                        const uint32_t d = nd >= gd ? nd + 1 : nd;
                        if (k & (1u << nd)) { w *= pos[d]; q[d] = p[d] + 1; }
                        else { w *= 1 - pos[d]; q[d] = p[d]; }
                    }
                    q[gd] = p[gd];
                    const uint32_t left = grid_index_(gridtype, align, hsize, res, q, D);
                    q[gd] = p[gd] + 1;
                    const uint32_t right = grid_index_(gridtype, align, hsize, res, q, D);
                    for (uint32_t ch = 0; ch < C; ++ch) {
                        double diff = load_(emb, st, (size_t)(base + right) * C + ch) -
                                      load_(emb, st, (size_t)(base + left) * C + ch);
                        if (st == 0) diff = (float)diff;
                        if (st == 1) diff = h2f_(f2h_((float)diff));  /* Half - Half -> Half */
                        rg[ch] = acc_(st, rg[ch], w, diff);
                    }
                }
                for (uint32_t ch = 0; ch < C; ++ch) store_(dy_dx, st, jbase + gd * C + ch, rg[ch]);
            }
        }
    }
}

/* gridencoder.cu:226-313 with exact (double) accumulation in a fixed order:
 * grad_grid[row*C + ch] += w * grad, summed over every sample, level and
 * corner.  grad is read from storage type st in [B, L*C] (blc) or [L, B, C].
 * This is the value the atomics approximate; tests compare with a tolerance. */
void orc_grid_encode_backward(const void *grad, int st, const float *inputs, const int32_t *offsets,
                              double *grad_grid, uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                              float S, uint32_t H, uint32_t gridtype, int align, int blc) {
    uint32_t p[8], q[8];
    float pos[8];
    for (uint32_t b = 0; b < B; ++b) {
        const float *x = inputs + (size_t)b * D;
        int oob = 0;
        for (uint32_t d = 0; d < D; ++d)
            if (x[d] < 0 || x[d] > 1) oob = 1;
        if (oob) continue;
        for (uint32_t l = 0; l < L; ++l) {
            const uint32_t base = (uint32_t)offsets[l];
            const uint32_t hsize = (uint32_t)offsets[l + 1] - base;
            const float scale = level_scale_(l, S, H);
            const uint32_t res = (uint32_t)ceilf(scale) + 1;
            for (uint32_t d = 0; d < D; ++d) {
                const float v = fmaf(x[d], scale, align ? 0.0f : 0.5f);
                p[d] = (uint32_t)floorf(v);
                pos[d] = v - (float)p[d];
            }
            for (uint32_t k = 0; k < (1u << D); ++k) {
                float w = 1;
                for (uint32_t d = 0; d < D; ++d) {
                    if (k & (1u << d)) { w *= pos[d]; q[d] = p[d] + 1; }
                    else { w *= 1 - pos[d]; q[d] = p[d]; }
                }
                const uint32_t row = grid_index_(gridtype, align, hsize, res, q, D);
                for (uint32_t ch = 0; ch < C; ++ch) {
                    const size_t gi = blc ? (size_t)b * L * C + (size_t)l * C + ch
                                          : (size_t)l * B * C + (size_t)b * C + ch;
                    grad_grid[(size_t)(base + row) * C + ch] += (double)w * load_(grad, st, gi);
                }
            }
        }
    }
}

/* gridencoder.cu:316-342 (f32 only): grad_inputs[b, d] = sum grad * dy_dx */
void orc_grid_input_backward(const float *grad, const float *dy_dx, float *grad_inputs, uint32_t B,
                             uint32_t D, uint32_t C, uint32_t L, int blc) {
    for (uint32_t b = 0; b < B; ++b)
        for (uint32_t d = 0; d < D; ++d) {
            float r = 0;
            for (uint32_t l = 0; l < L; ++l)
                for (uint32_t ch = 0; ch < C; ++ch) {
                    const float g = blc ? grad[(size_t)b * L * C + (size_t)l * C + ch]
                                        : grad[(size_t)l * B * C + (size_t)b * C + ch];
                    r = fmaf(g, dy_dx[(size_t)b * L * D * C + (size_t)l * D * C + d * C + ch], r);
                }
            grad_inputs[(size_t)b * D + d] = r;
        }
}

/* ------------------------------------------------------------ freq encoder */

/* freqencoder.cu:30-58 with the accurate sin (the GPU build also uses it) */
void orc_freq_encode_forward(const float *inputs, uint32_t B, uint32_t D, uint32_t deg, uint32_t C,
                             float *outputs) {
    const float half_pi = 3.141592653589793f / 2;
    for (uint32_t b = 0; b < B; ++b)
        for (uint32_t c = 0; c < C; ++c) {
            const float *x = inputs + (size_t)b * D;
            float v;
            if (c < D) {
                v = x[c];
            } else {
                const uint32_t col = c / D - 1, d = c % D;
                v = (float)sin((double)(scalbnf(x[d], (int)(col / 2)) + (float)(col % 2) * half_pi));
            }
            outputs[(size_t)b * C + c] = v;
        }
}

/* freqencoder.cu:63-94 */
void orc_freq_encode_backward(const float *grad, const float *outputs, uint32_t B, uint32_t D,
                              uint32_t deg, uint32_t C, float *grad_inputs) {
    for (uint32_t b = 0; b < B; ++b)
        for (uint32_t d = 0; d < D; ++d) {
            const float *g = grad + (size_t)b * C, *o = outputs + (size_t)b * C;
            float r = g[d];
            for (uint32_t f = 0; f < deg; ++f) {
                const uint32_t s = D + 2 * f * D + d;
                r = fmaf(scalbnf(1.0f, (int)f), fmaf(g[s], o[s + D], -(g[s + D] * o[s])), r);
            }
            grad_inputs[(size_t)b * D + d] = r;
        }
}
