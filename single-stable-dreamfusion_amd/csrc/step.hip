// Prologue of the native albedo train step: everything the step draws or
// derives per ray before the march, as ONE launch (nerf/native_step.py).
//
// Replaces, per 128x128 step, the reference's camera rays (nerf/utils.py:42-106
// get_rays), the ray/box intersection (raymarching.py:19-49 near_far_from_aabb,
// min_near 0.2 as renderer.py:458 leaves it), the march noise
// (raymarching.py:200 torch.rand), the background colour draw
// (utils.py:349 torch.rand, only when no background net), the zeroing of the
// step counter (renderer.py:470) and the synthetic SDS gradient w(t) * eps
// injected at pred_rgb (nerf/sd.py InjectedSDS: t ~ U{min_step..max_step},
// w = 1 - alphas_cumprod[t], eps ~ N(0, 1)) — eleven launches in the autograd
// step.  The camera ray and the box intersection are the same device code as
// dfhip_get_rays / dfhip_near_far_from_aabb (camera_common.h, march_common.h),
// so rays, nears and fars are bit-identical to theirs.
//
// Random numbers: Philox4x32-10 keyed by the run seed, counter (ray, step,
// stream): stateless, so a replayed step draws fresh numbers from its step
// index, the draws do not depend on the launch shape, and every rank of a
// data-parallel run draws its own stream from its own seed.
#include "camera_common.h"
#include "march_common.h"

namespace dfhip {
namespace st {

struct U4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11), the generator family of torch's CUDA RNG.
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t lo0 = c.x * 0xD2511F53u, hi0 = __umulhi(c.x, 0xD2511F53u);
        const uint32_t lo1 = c.z * 0xCD9E8D57u, hi1 = __umulhi(c.z, 0xCD9E8D57u);
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// [0, 1) and (0, 1] from the top 24 bits
__device__ __forceinline__ float unit(uint32_t v) { return (float)(v >> 8) * 0x1p-24f; }
__device__ __forceinline__ float unit_open0(uint32_t v) {
    return (float)((v >> 8) + 1u) * 0x1p-24f;
}

// Box-Muller pair
__device__ __forceinline__ void normal2(uint32_t a, uint32_t b, float &z0, float &z1) {
    const float r = sqrtf(-2.0f * logf(unit_open0(a)));
    float s, c;
    sincosf(6.283185307179586f * unit(b), &s, &c);
    z0 = r * c;
    z1 = r * s;
}

constexpr uint32_t kMaxLr = 8;

struct Args {
    cam::Pose pose;
    float fx, fy, cx, cy;
    uint32_t H, W;
    float aabb[6];
    float min_near;
    uint32_t seed_lo, seed_hi, step_lo, step_hi;
    int perturb;
    const float *alphas;  // alphas_cumprod [T]
    uint32_t min_step, max_step;
    // per-step scalars for later launches of a replayed graph (the optimizer's
    // learning rates): lr_dev[0..n_lr) = lr[0..n_lr)
    float lr[kMaxLr];
    uint32_t n_lr;
    float *lr_dev;
};

__global__ __launch_bounds__(256) void k_step_prologue(Args a, float *__restrict__ rays_o,
                                                       float *__restrict__ rays_d,
                                                       float *__restrict__ nears,
                                                       float *__restrict__ fars,
                                                       float *__restrict__ noises,
                                                       float *__restrict__ bg_color,
                                                       float *__restrict__ g_image,
                                                       int32_t *__restrict__ counter) {
    const uint32_t N = a.H * a.W;
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n == 0 && counter) {
        counter[0] = 0;
        counter[1] = 0;
    }
    if (n < a.n_lr) a.lr_dev[n] = a.lr[n];
    if (n >= N) return;
    float o[3], d[3];
    cam::pixel_ray(a.pose, a.fx, a.fy, a.cx, a.cy, a.W, n, o, d);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        rays_o[3 * (size_t)n + k] = o[k];
        rays_d[3 * (size_t)n + k] = d[k];
    }
    rm::Ray r;
    r.ox = o[0]; r.oy = o[1]; r.oz = o[2];
    r.dx = d[0]; r.dy = d[1]; r.dz = d[2];
    r.rdx = 1.0f / r.dx; r.rdy = 1.0f / r.dy; r.rdz = 1.0f / r.dz;
    float lo, hi;
    if (!rm::ray_aabb(r, a.aabb, a.min_near, lo, hi)) lo = hi = FLT_MAX;
    nears[n] = lo;
    fars[n] = hi;

    const U4 r0 = philox(U4{n, a.step_lo, a.step_hi, 0u}, a.seed_lo, a.seed_hi);
    const U4 r1 = philox(U4{n, a.step_lo, a.step_hi, 1u}, a.seed_lo, a.seed_hi);
    if (noises) noises[n] = a.perturb ? unit(r0.x) : 0.0f;
    if (bg_color) {
        bg_color[3 * (size_t)n + 0] = unit(r0.w);
        bg_color[3 * (size_t)n + 1] = unit(r1.z);
        bg_color[3 * (size_t)n + 2] = unit(r1.w);
    }
    if (g_image) {
        // one timestep per step: every thread draws the same (ray-independent counter)
        const U4 rt = philox(U4{0xFFFFFFFFu, a.step_lo, a.step_hi, 2u}, a.seed_lo, a.seed_hi);
        const uint32_t span = a.max_step - a.min_step + 1u;
        const uint32_t t = a.min_step + rt.x % span;
        const float w = 1.0f - a.alphas[t];
        float z0, z1, z2, z3;
        normal2(r0.y, r0.z, z0, z1);
        normal2(r1.x, r1.y, z2, z3);
        (void)z3;
        g_image[n] = w * z0;  // channel-major [3, N], as pred_rgb
        g_image[(size_t)N + n] = w * z1;
        g_image[2 * (size_t)N + n] = w * z2;
    }
}

}  // namespace st
}  // namespace dfhip

using namespace dfhip;

extern "C" int dfhip_train_step_prologue_lr(
    const float *pose, float fx, float fy, float cx, float cy, uint32_t H, uint32_t W,
    const float *aabb, float min_near, uint64_t seed, uint64_t step, int perturb,
    const float *alphas, uint32_t min_step, uint32_t max_step, float *rays_o, float *rays_d,
    float *nears, float *fars, float *noises, float *bg_color, float *g_image, int32_t *counter,
    const float *lr_host, uint32_t n_lr, float *lr_dev, dfhip_stream_t stream) {
    const char *name = "train_step_prologue";
    if (!pose || !aabb || !rays_o || !rays_d || !nears || !fars) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (!(fx != 0.0f) || !(fy != 0.0f)) {
        set_error("%s: focal lengths must be non-zero", name);
        return DFHIP_EINVAL;
    }
    if (g_image && (!alphas || max_step < min_step)) {
        set_error("%s: the SDS draw needs alphas and min_step <= max_step", name);
        return DFHIP_EINVAL;
    }
    if (n_lr > st::kMaxLr || (n_lr && (!lr_host || !lr_dev))) {
        set_error("%s: at most %u learning rates, with host and device arrays", name,
                  st::kMaxLr);
        return DFHIP_EINVAL;
    }
    const uint64_t n = (uint64_t)H * W;
    if (n > 0xFFFFFFFFull) {
        set_error("%s: H*W too large", name);
        return DFHIP_EINVAL;
    }
    st::Args a;
    a.pose = cam::pose_from_3x4(pose);
    a.fx = fx; a.fy = fy; a.cx = cx; a.cy = cy;
    a.H = H; a.W = W;
    for (int i = 0; i < 6; ++i) a.aabb[i] = aabb[i];
    a.min_near = min_near;
    a.seed_lo = (uint32_t)seed; a.seed_hi = (uint32_t)(seed >> 32);
    a.step_lo = (uint32_t)step; a.step_hi = (uint32_t)(step >> 32);
    a.perturb = perturb;
    a.alphas = alphas;
    a.min_step = min_step;
    a.max_step = max_step;
    a.n_lr = n_lr;
    a.lr_dev = lr_dev;
    for (uint32_t i = 0; i < st::kMaxLr; ++i) a.lr[i] = i < n_lr ? lr_host[i] : 0.0f;
    // at least one block: the counter reset and the lr pack run with no rays
    const uint32_t blocks = n ? ceil_div((uint32_t)n, 256u) : 1u;
    st::k_step_prologue<<<blocks, 256, 0, as_stream(stream)>>>(a, rays_o, rays_d, nears, fars,
                                                                noises, bg_color, g_image,
                                                                counter);
    return check_launch(name);
}

extern "C" int dfhip_train_step_prologue(const float *pose, float fx, float fy, float cx,
                                         float cy, uint32_t H, uint32_t W, const float *aabb,
                                         float min_near, uint64_t seed, uint64_t step,
                                         int perturb, const float *alphas, uint32_t min_step,
                                         uint32_t max_step, float *rays_o, float *rays_d,
                                         float *nears, float *fars, float *noises,
                                         float *bg_color, float *g_image, int32_t *counter,
                                         dfhip_stream_t stream) {
    return dfhip_train_step_prologue_lr(pose, fx, fy, cx, cy, H, W, aabb, min_near, seed, step,
                                        perturb, alphas, min_step, max_step, rays_o, rays_d,
                                        nears, fars, noises, bg_color, g_image, counter,
                                        nullptr, 0, nullptr, stream);
}
