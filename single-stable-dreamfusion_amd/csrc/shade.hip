// Non-albedo shading of the grid NeRF train step on the device (the
// `textureless` and `lambertian` steps, 80 % of the reference's steps after
// albedo_iters: nerf/utils.py:346-359):
//
//   normal  = safe_normalize(-(sigma(x + eps e_a) - sigma(x - eps e_a)) * 0.5 / eps)
//             (network_grid.py:90-121: six extra common_forward calls at the
//              clamped stencil points, NaN -> 0)
//   lam     = ratio + (1 - ratio) * clamp(normal @ l, min=0)       (:135, f16 under autocast)
//   color   = lam.repeat(3) (textureless) | albedo * lam (lambertian)   (:137-142)
//   orient  = mean(w.detach() * clamp(normal . d, min=0)^2), w = 1 - exp(-sigma)
//             (renderer.py:485-489, mean over the march's M' rows)
//
// The six stencil evaluations are extra rows of ONE fused field launch: the
// stencil kernel lays out the M live samples with their stencil points
// interleaved (row 7 i = sample i, rows 7 i + 1 + a, a = 0..5: +x, -x, +y,
// -y, +z, -z) and writes the live row count 7 M, so the field forward, the
// field backward and the embedding backward each run once over 7 M rows.  The
// interleaving keeps a sample's seven points adjacent: at the coarse grid
// levels (cells wider than the 2 eps stencil) they fall in one cell, and the
// binned embedding backward merges their contributions in registers before
// its LDS atomics; their table gathers hit the same lines.
//
// The shading kernels keep the reference's dtypes and rounding points: the normal and the orientation loss in f32, the
// light product, lambertian and colour as f16 values (autocast casts normal @ l
// to f16), the gradients of the f16 tensors rounded to f16 where autograd
// would hold them in f16.  Loss-scale handling follows autograd: the
// orientation term's gradient carries the GradScaler scale, as the entropy
// term's does.  Under bf16 autocast (the C5 option) the same rounding points
// round to bf16 (the kernels are instantiated on the element type E).
#include "common.h"

#include <type_traits>

#include <math.h>

namespace dfhip {
namespace shd {

constexpr int kStencil = 6;
constexpr uint32_t kThreads = 256;

// round to the autocast element type E (f16 or bf16), through an f32 value
template <typename E>
__device__ __forceinline__ float rnd(float x) { return (float)(E)f32_rounded(x); }

__device__ __forceinline__ uint32_t live(const int32_t *m_dev, uint32_t cap) {
    const int32_t m = *m_dev;
    return m < 0 ? 0u : ((uint32_t)m < cap ? (uint32_t)m : cap);
}

// March rows M' of the reference (raymarching.py:224-227: m += align - m % align)
__device__ __forceinline__ float padded_rows(uint32_t m) {
    return (float)(m + 128u - m % 128u);
}

// Samples and their stencil points, interleaved, + the live count 7 M.
__global__ __launch_bounds__(kThreads) void k_stencil(const float *__restrict__ xyz,
                                                      const int32_t *__restrict__ m_dev,
                                                      uint32_t cap, float eps, float bound,
                                                      float *__restrict__ xyz7,
                                                      int32_t *__restrict__ m7_dev) {
    // a block's kThreads samples are staged in LDS, then its 21 x kThreads output
    // floats are written by consecutive threads (contiguous stores; a thread
    // per sample wrote 21 floats at an 84-byte lane stride)
    constexpr uint32_t kOut = 3u * (1u + kStencil);  // floats per sample (7 rows)
    __shared__ float sx[3 * kThreads];
    const uint32_t M = live(m_dev, cap);
    if (blockIdx.x == 0 && threadIdx.x == 0) *m7_dev = (int32_t)(7u * M);
    for (uint32_t base = blockIdx.x * kThreads; base < M; base += gridDim.x * kThreads) {
        const uint32_t n = min((uint32_t)kThreads, M - base);
        for (uint32_t j = threadIdx.x; j < 3 * n; j += kThreads) sx[j] = xyz[3 * (size_t)base + j];
        __syncthreads();
        float *dst = xyz7 + kOut * (size_t)base;
        for (uint32_t j = threadIdx.x; j < kOut * n; j += kThreads) {
            const uint32_t i = j / kOut, k = j - kOut * i, r = k / 3u, d = k - 3u * r;
            const float x = sx[3 * i + d];
            float v = x;
            if (r > 0) {
                // x + tensor([[eps, 0, 0]]) then clamp(-bound, bound)
                const uint32_t s1 = r - 1u, a = s1 >> 1;
                const float off = (s1 & 1u) ? -eps : eps;
                v = fminf(fmaxf(x + (d == a ? off : 0.0f), -bound), bound);
            }
            dst[j] = v;
        }
        __syncthreads();  // sx is rewritten next
    }
}

struct Normal {
    float v[3], n[3], r, ss;
    bool nan[3];
};

// network_grid.py:90-121 (f32): v = -(0.5 * (s+ - s-) / eps), n = v / sqrt(clamp(|v|^2, 1e-20))
__device__ __forceinline__ Normal fd_normal(const float *__restrict__ sigma7, uint32_t i,
                                            float eps) {
    Normal o;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float sp = sigma7[7 * (size_t)i + 1 + 2 * a];
        const float sn = sigma7[7 * (size_t)i + 2 + 2 * a];
        o.v[a] = -((0.5f * (sp - sn)) / eps);
    }
    o.ss = (o.v[0] * o.v[0] + o.v[1] * o.v[1]) + o.v[2] * o.v[2];
    o.r = sqrtf(fmaxf(o.ss, 1e-20f));
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float q = o.v[a] / o.r;
        o.nan[a] = q != q;
        o.n[a] = o.nan[a] ? 0.0f : q;
    }
    return o;
}

// (normal @ l) under autocast: E operands, f32 accumulation, E result
template <typename E>
__device__ __forceinline__ float dot16(const float n[3], const float l16[3]) {
    const float p0 = rnd<E>(n[0]) * l16[0], p1 = rnd<E>(n[1]) * l16[1],
                p2 = rnd<E>(n[2]) * l16[2];
    return rnd<E>((p0 + p1) + p2);
}

struct Shade {
    float d16, lam16;
};

template <typename E>
__device__ __forceinline__ Shade lambert(const float n[3], const float l16[3], float ratio,
                                         float omr) {
    Shade s;
    s.d16 = dot16<E>(n, l16);
    const float c16 = s.d16 > 0.0f ? s.d16 : 0.0f;     // clamp(min=0)
    s.lam16 = rnd<E>(ratio + rnd<E>(c16 * omr));       // ratio + (1 - ratio) * c
    return s;
}

// Forward: the samples' density (f32) and colour (f16) for the compositing,
// the normal (f32, kept for the backward) and per-block partial sums of the
// orientation term (f64).  sigma7 / albedo7: the field on the 7 M rows.
template <typename E>
__global__ __launch_bounds__(kThreads) void k_shade_fwd(
    const float *__restrict__ sigma7, const E *__restrict__ albedo7,
    const float *__restrict__ dirs, const float *__restrict__ light, float ratio, float omr,
    float eps, int lambertian, const int32_t *__restrict__ m_dev, uint32_t cap,
    float *__restrict__ sigma, E *__restrict__ color, float *__restrict__ normal,
    double *__restrict__ part) {
    __shared__ double red[kThreads / 64];
    const uint32_t M = live(m_dev, cap);
    float l16[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) l16[d] = rnd<E>(light[d]);
    double acc = 0.0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x) {
        const Normal nm = fd_normal(sigma7, i, eps);
        const Shade sh = lambert<E>(nm.n, l16, ratio, omr);
        const float sg = sigma7[7 * (size_t)i];
        sigma[i] = sg;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            normal[3 * (size_t)i + d] = nm.n[d];
            const float c = lambertian ? rnd<E>((float)albedo7[21 * (size_t)i + d] * sh.lam16)
                                       : sh.lam16;
            color[3 * (size_t)i + d] = (E)c;
        }
        // orientation term: (1 - exp(-sigma)) * clamp(n . d, min=0)^2
        const float w = 1.0f - expf(-sg);
        const float nd = (nm.n[0] * dirs[3 * (size_t)i] + nm.n[1] * dirs[3 * (size_t)i + 1]) +
                         nm.n[2] * dirs[3 * (size_t)i + 2];
        const float c = nd > 0.0f ? nd : 0.0f;
        acc += (double)(w * (c * c));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < (int)(kThreads / 64); ++w) s += red[w];
        part[blockIdx.x] = s;
    }
}

// loss += lambda * sum / M' (fixed-order sum of the block partials)
__global__ __launch_bounds__(64) void k_orient_finish(const double *__restrict__ part,
                                                      uint32_t parts, const int32_t *m_dev,
                                                      uint32_t cap, float lambda,
                                                      float *__restrict__ orient,
                                                      float *__restrict__ loss) {
    double s = 0.0;
    for (uint32_t p = threadIdx.x; p < parts; p += 64) s += part[p];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (threadIdx.x == 0) {
        const float mean = (float)s / padded_rows(live(m_dev, cap));
        if (orient) *orient = mean;
        if (loss) *loss = *loss + lambda * mean;
    }
}

// Backward.  grad_sigma [cap] f32 / grad_color [cap, 3] f16: d loss / d
// (density, colour) from the compositing backward.  Writes the field-row
// gradients grad_sigma7 [7 M] (sample rows: the compositing's, stencil rows:
// through the normal) and grad_albedo7 [7 M, 3] (sample rows: the lambertian
// product's albedo gradient, else 0; stencil rows 0).
template <typename E>
__global__ __launch_bounds__(kThreads) void k_shade_bwd(
    const float *__restrict__ sigma7, const E *__restrict__ albedo7,
    const float *__restrict__ dirs, const float *__restrict__ light, float ratio, float omr,
    float eps, int lambertian, const int32_t *__restrict__ m_dev, uint32_t cap,
    const float *__restrict__ grad_sigma, const E *__restrict__ grad_color,
    const float *__restrict__ grad_loss, float lambda, float *__restrict__ grad_sigma7,
    E *__restrict__ grad_albedo7) {
    const uint32_t M = live(m_dev, cap);
    float l16[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) l16[d] = rnd<E>(light[d]);
    // d loss / d orient_i: (scale * lambda) / M' (MulBackward, MeanBackward)
    const float go = (grad_loss[0] * lambda) / padded_rows(M);
    // a block's samples are computed one per thread into LDS images of their
    // 21 albedo-gradient and 7 density-gradient values, which consecutive
    // threads then copy out (contiguous stores)
    __shared__ E s_ga[21 * kThreads];
    __shared__ float s_gs[7 * kThreads];
    for (uint32_t base = blockIdx.x * kThreads; base < M; base += gridDim.x * kThreads) {
      const uint32_t nblk = min((uint32_t)kThreads, M - base);
      const uint32_t i = base + threadIdx.x;
      if (i < M) {
        const Normal nm = fd_normal(sigma7, i, eps);
        const Shade sh = lambert<E>(nm.n, l16, ratio, omr);
        E *ga = s_ga + 21 * threadIdx.x;
        float g[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) g[d] = (float)grad_color[3 * (size_t)i + d];
        float glam;
        if (lambertian) {
            float gl[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const float a = (float)albedo7[21 * (size_t)i + d];
                ga[d] = (E)rnd<E>(g[d] * sh.lam16);
                gl[d] = rnd<E>(g[d] * a);
            }
            glam = rnd<E>((gl[0] + gl[1]) + gl[2]);  // sum over the broadcast dim
        } else {
#pragma unroll
            for (int d = 0; d < 3; ++d) ga[d] = (E)0.0f;
            glam = rnd<E>((g[0] + g[1]) + g[2]);  // RepeatBackward
        }
        const float gc = rnd<E>(glam * omr);              // (1 - ratio) * c
        const float gd = sh.d16 >= 0.0f ? gc : 0.0f;      // clamp(min=0)
        float gn[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) gn[d] = rnd<E>(gd * l16[d]);  // mv backward (E), cast back
        // orientation term: d/dn of go * w * clamp(n . d, 0)^2
        const float w = 1.0f - expf(-sigma7[7 * (size_t)i]);
        const float dx = dirs[3 * (size_t)i], dy = dirs[3 * (size_t)i + 1],
                    dz = dirs[3 * (size_t)i + 2];
        const float nd = (nm.n[0] * dx + nm.n[1] * dy) + nm.n[2] * dz;
        const float c = nd > 0.0f ? nd : 0.0f;
        const float g2 = nd >= 0.0f ? (go * w) * (2.0f * c) : 0.0f;
        gn[0] = gn[0] + g2 * dx;
        gn[1] = gn[1] + g2 * dy;
        gn[2] = gn[2] + g2 * dz;
#pragma unroll
        for (int d = 0; d < 3; ++d)
            if (nm.nan[d]) gn[d] = 0.0f;  // normal[isnan] = 0
        // n = v / r, r = sqrt(clamp(ss, 1e-20)), ss = sum v^2
        const float r2 = nm.r * nm.r;
        const float gr = ((-gn[0] * nm.v[0]) / r2 + (-gn[1] * nm.v[1]) / r2) +
                         (-gn[2] * nm.v[2]) / r2;
        const float gs = nm.ss >= 1e-20f ? gr / (2.0f * nm.r) : 0.0f;
        float *gs7 = s_gs + 7 * threadIdx.x;
        gs7[0] = grad_sigma[i];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float gv = gn[a] / nm.r + (gs * nm.v[a] + gs * nm.v[a]);
            // v = -((0.5 * (s+ - s-)) / eps)
            const float gdiff = 0.5f * (-gv / eps);
            gs7[1 + 2 * a] = gdiff;
            gs7[2 + 2 * a] = -gdiff;
        }
        // the stencil rows carry no albedo gradient
#pragma unroll
        for (int k = 3; k < 21; ++k) ga[k] = (E)0.0f;
      }
      __syncthreads();
      for (uint32_t j = threadIdx.x; j < 21 * nblk; j += kThreads)
          grad_albedo7[21 * (size_t)base + j] = s_ga[j];
      for (uint32_t j = threadIdx.x; j < 7 * nblk; j += kThreads)
          grad_sigma7[7 * (size_t)base + j] = s_gs[j];
      __syncthreads();  // the images are rewritten next
    }
}

// Light direction of the step (renderer.py:462-464): safe_normalize(rays_o[0]
// + randn(3)), the normal draws from Philox keyed like the step prologue.
struct U4 {
    uint32_t x, y, z, w;
};
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

__global__ void k_light(const float *__restrict__ rays_o, uint32_t seed_lo, uint32_t seed_hi,
                        uint32_t step_lo, uint32_t step_hi, float *__restrict__ light) {
    if (threadIdx.x != 0) return;
    const U4 r = philox(U4{0xFFFFFFFEu, step_lo, step_hi, 3u}, seed_lo, seed_hi);
    auto u = [](uint32_t v) { return (float)(v >> 8) * 0x1p-24f; };
    const float ra = sqrtf(-2.0f * logf((float)((r.x >> 8) + 1u) * 0x1p-24f));
    const float rb = sqrtf(-2.0f * logf((float)((r.z >> 8) + 1u) * 0x1p-24f));
    float s0, c0, s1, c1;
    sincosf(6.283185307179586f * u(r.y), &s0, &c0);
    sincosf(6.283185307179586f * u(r.w), &s1, &c1);
    const float z[3] = {ra * c0, ra * s0, rb * c1};
    float v[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) v[d] = rays_o[d] + z[d];
    const float ss = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
    const float rr = sqrtf(fmaxf(ss, 1e-20f));
#pragma unroll
    for (int d = 0; d < 3; ++d) light[d] = v[d] / rr;
}

}  // namespace shd
}  // namespace dfhip

using namespace dfhip;

static uint32_t shade_blocks(uint32_t cap) {
    // grid-stride: enough workgroups for 4 per CU, never more than the rows need
    uint32_t b = ceil_div(cap, shd::kThreads);
    return b < 1024u ? (b ? b : 1u) : 1024u;
}

extern "C" uint32_t dfhip_shading_partial_doubles(uint32_t cap) { return shade_blocks(cap); }

extern "C" int dfhip_shading_stencil(const float *xyz, const int32_t *m_dev, uint32_t cap,
                                     float eps, float bound, float *xyz7, int32_t *m7_dev,
                                     dfhip_stream_t stream) {
    if (!xyz || !m_dev || !xyz7 || !m7_dev) {
        set_error("shading_stencil: null pointer");
        return DFHIP_EINVAL;
    }
    if (!(bound > 0.0f)) {
        set_error("shading_stencil: bound must be > 0");
        return DFHIP_EINVAL;
    }
    shd::k_stencil<<<shade_blocks(cap), shd::kThreads, 0, as_stream(stream)>>>(
        xyz, m_dev, cap, eps, bound, xyz7, m7_dev);
    return check_launch("shading_stencil");
}

static bool shading_mode(const char *name, int shading, int &lambertian) {
    if (shading == DFHIP_SHADING_TEXTURELESS) lambertian = 0;
    else if (shading == DFHIP_SHADING_LAMBERTIAN) lambertian = 1;
    else {
        set_error("%s: shading must be DFHIP_SHADING_TEXTURELESS or _LAMBERTIAN", name);
        return false;
    }
    return true;
}

// elem: DFHIP_F16 (fp16 autocast) or DFHIP_BF16 (bf16 autocast) for the
// albedo / colour tensors and the rounding points
static int shading_forward(const char *name, int elem, const float *sigma7, const void *albedo7,
                           const float *dirs, const float *light, float ratio, float eps,
                           int shading, const int32_t *m_dev, uint32_t cap, float *sigma,
                           void *color, float *normal, double *partial, float lambda_orient,
                           float *orient, float *loss, dfhip_stream_t stream) {
    int lam = 0;
    if (!shading_mode(name, shading, lam)) return DFHIP_EINVAL;
    if (!sigma7 || !albedo7 || !dirs || !light || !m_dev || !sigma || !color || !normal ||
        !partial) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const uint32_t blocks = shade_blocks(cap);
    const float omr = (float)(1.0 - (double)ratio);
    if (elem == DFHIP_BF16)
        shd::k_shade_fwd<bf16_t><<<blocks, shd::kThreads, 0, s>>>(
            sigma7, (const bf16_t *)albedo7, dirs, light, ratio, omr, eps, lam, m_dev, cap, sigma,
            (bf16_t *)color, normal, partial);
    else
        shd::k_shade_fwd<half_t><<<blocks, shd::kThreads, 0, s>>>(
            sigma7, (const half_t *)albedo7, dirs, light, ratio, omr, eps, lam, m_dev, cap, sigma,
            (half_t *)color, normal, partial);
    shd::k_orient_finish<<<1, 64, 0, s>>>(partial, blocks, m_dev, cap, lambda_orient, orient,
                                          loss);
    return check_launch(name);
}

static int shading_backward(const char *name, int elem, const float *sigma7,
                            const void *albedo7, const float *dirs, const float *light,
                            float ratio, float eps, int shading, const int32_t *m_dev,
                            uint32_t cap, const float *grad_sigma, const void *grad_color,
                            const float *grad_loss, float lambda_orient, float *grad_sigma7,
                            void *grad_albedo7, dfhip_stream_t stream) {
    int lam = 0;
    if (!shading_mode(name, shading, lam)) return DFHIP_EINVAL;
    if (!sigma7 || !albedo7 || !dirs || !light || !m_dev || !grad_sigma || !grad_color ||
        !grad_loss || !grad_sigma7 || !grad_albedo7) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    const float omr = (float)(1.0 - (double)ratio);
    hipStream_t s = as_stream(stream);
    if (elem == DFHIP_BF16)
        shd::k_shade_bwd<bf16_t><<<shade_blocks(cap), shd::kThreads, 0, s>>>(
            sigma7, (const bf16_t *)albedo7, dirs, light, ratio, omr, eps, lam, m_dev, cap,
            grad_sigma, (const bf16_t *)grad_color, grad_loss, lambda_orient, grad_sigma7,
            (bf16_t *)grad_albedo7);
    else
        shd::k_shade_bwd<half_t><<<shade_blocks(cap), shd::kThreads, 0, s>>>(
            sigma7, (const half_t *)albedo7, dirs, light, ratio, omr, eps, lam, m_dev, cap,
            grad_sigma, (const half_t *)grad_color, grad_loss, lambda_orient, grad_sigma7,
            (half_t *)grad_albedo7);
    return check_launch(name);
}

extern "C" int dfhip_shading_forward(const float *sigma7, const void *albedo7, const float *dirs,
                                     const float *light, float ratio, float eps, int shading,
                                     const int32_t *m_dev, uint32_t cap, float *sigma,
                                     void *color, float *normal, double *partial,
                                     float lambda_orient, float *orient, float *loss,
                                     dfhip_stream_t stream) {
    return shading_forward("shading_forward", DFHIP_F16, sigma7, albedo7, dirs, light, ratio,
                           eps, shading, m_dev, cap, sigma, color, normal, partial,
                           lambda_orient, orient, loss, stream);
}

extern "C" int dfhip_shading_forward_bf16(const float *sigma7, const void *albedo7,
                                          const float *dirs, const float *light, float ratio,
                                          float eps, int shading, const int32_t *m_dev,
                                          uint32_t cap, float *sigma, void *color,
                                          float *normal, double *partial, float lambda_orient,
                                          float *orient, float *loss, dfhip_stream_t stream) {
    return shading_forward("shading_forward_bf16", DFHIP_BF16, sigma7, albedo7, dirs, light,
                           ratio, eps, shading, m_dev, cap, sigma, color, normal, partial,
                           lambda_orient, orient, loss, stream);
}

extern "C" int dfhip_shading_backward(const float *sigma7, const void *albedo7,
                                      const float *dirs, const float *light, float ratio,
                                      float eps, int shading, const int32_t *m_dev, uint32_t cap,
                                      const float *grad_sigma, const void *grad_color,
                                      const float *grad_loss, float lambda_orient,
                                      float *grad_sigma7, void *grad_albedo7,
                                      dfhip_stream_t stream) {
    return shading_backward("shading_backward", DFHIP_F16, sigma7, albedo7, dirs, light, ratio,
                            eps, shading, m_dev, cap, grad_sigma, grad_color, grad_loss,
                            lambda_orient, grad_sigma7, grad_albedo7, stream);
}

extern "C" int dfhip_shading_backward_bf16(const float *sigma7, const void *albedo7,
                                           const float *dirs, const float *light, float ratio,
                                           float eps, int shading, const int32_t *m_dev,
                                           uint32_t cap, const float *grad_sigma,
                                           const void *grad_color, const float *grad_loss,
                                           float lambda_orient, float *grad_sigma7,
                                           void *grad_albedo7, dfhip_stream_t stream) {
    return shading_backward("shading_backward_bf16", DFHIP_BF16, sigma7, albedo7, dirs, light,
                            ratio, eps, shading, m_dev, cap, grad_sigma, grad_color, grad_loss,
                            lambda_orient, grad_sigma7, grad_albedo7, stream);
}

extern "C" int dfhip_shading_light(const float *rays_o, uint64_t seed, uint64_t step,
                                   float *light, dfhip_stream_t stream) {
    if (!rays_o || !light) {
        set_error("shading_light: null pointer");
        return DFHIP_EINVAL;
    }
    shd::k_light<<<1, 64, 0, as_stream(stream)>>>(rays_o, (uint32_t)seed, (uint32_t)(seed >> 32),
                                                  (uint32_t)step, (uint32_t)(step >> 32), light);
    return check_launch("shading_light");
}
