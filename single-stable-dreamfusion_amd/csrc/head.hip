// Per-ray tail of the render and its regulariser, fused (reference
// nerf/renderer.py:536-551 and nerf/utils.py:386-391):
//
//   bg    = sigmoid(W2 relu(W1 freq(d) + b1) + b2)         (network_grid.py:158-167,
//                                                           fp16 Linear layers under autocast)
//   image = image + (1 - ws) * bg                          -> written channel-major [3, N]
//   depth = clamp(depth - near, min=0) / (far - near);  mask = near < far
//   loss  = lambda * mean(-a log2 a - (1 - a) log2 (1 - a)),  a = clamp(ws, 1e-5, 1 - 1e-5)
//
// The reference runs these as ~45 small torch launches forward and backward
// (frequency encoding, casts, two GEMMs, activations, the mix, the depth
// normalisation, the permute of pred_rgb, the entropy terms).  Here: one
// forward kernel, a backward kernel that also forms per-block partials of the
// background MLP's weight gradients, one partial-sum kernel; one kernel each
// way for the entropy term.  Rounding follows the reference's autocast
// dtypes: the MLP's inputs, weights, hidden and output activations are f16
// values (f32 accumulation), the colour mix is f32.  The writes of pred_rgb
// channel-major make the reference's reshape/permute/contiguous a no-op.
#include "common.h"

#include <math.h>

namespace dfhip {
namespace hd {

constexpr int kDeg = 6;
constexpr int kIn = 3 + 3 * 2 * kDeg;  // 39
constexpr int kHid = 64;
constexpr int kOut = 3;
constexpr int kW1 = kHid * kIn, kB1 = kHid, kW2 = kOut * kHid, kB2 = kOut;
constexpr int kParams = kW1 + kB1 + kW2 + kB2;  // 2755
constexpr float kHalfPi = 3.141592653589793f / 2.0f;

__device__ __forceinline__ float r16(float x) { return (float)(half_t)f32_rounded(x); }

// w1 transposed ([kIn][kHid]: sub-lane q's four hidden units of input i are
// one 16-byte LDS read; 39 instead of 156 reads per lane), w2 as in the
// reference ([kOut][kHid]: q's four units of output k are contiguous too)
struct alignas(16) W {
    float w1t[kW1], b1[kB1], w2[kW2], b2[kB2];
};

__device__ __forceinline__ void load_w(W &w, const float *w1, const float *b1, const float *w2,
                                       const float *b2) {
    for (int i = threadIdx.x; i < kW1; i += blockDim.x) {
        const int j = i / kIn, c = i - j * kIn;  // w1 [kHid, kIn] row-major
        w.w1t[c * kHid + j] = r16(w1[i]);
    }
    for (int i = threadIdx.x; i < kB1; i += blockDim.x) w.b1[i] = r16(b1[i]);
    for (int i = threadIdx.x; i < kW2; i += blockDim.x) w.w2[i] = r16(w2[i]);
    for (int i = threadIdx.x; i < kB2; i += blockDim.x) w.b2[i] = r16(b2[i]);
}  // (callers __syncthreads before reading)

// The network kernels give each ray kSub = 16 lanes (consecutive threads):
// sub-lane q makes frequency column q (q < 12) and hidden units
// [kPer q, kPer q + kPer), the output layer's partial sums are combined with
// four xor-shuffles (the same order in all sixteen lanes).  A block is 16
// rays; 16k rays are 4096 waves (4 per SIMD; four lanes per ray left one wave
// per SIMD to hide every LDS and global latency).
// Workgroups of 64 rays (1,024 threads): every workgroup stages the f16
// weights once and the backward writes one weight-gradient partial per
// workgroup, so 64 rays per workgroup instead of 16 load the weights and write
// (and k_head_wsum reads) a quarter of the partials.
#ifndef DFHIP_HEAD_THREADS
#define DFHIP_HEAD_THREADS 1024
#endif
constexpr int kSub = 16;
constexpr int kPer = kHid / kSub;  // hidden units per lane
constexpr int kThreads = DFHIP_HEAD_THREADS;
constexpr int kRays = kThreads / kSub;  // rays per workgroup
static_assert(kThreads % 64 == 0 && kThreads <= 1024, "DFHIP_HEAD_THREADS: waves, <= 1024");

// freqencoder.cu:30-58 for D = 3, degree 6 (same expression as k_freq_fwd),
// then the autocast cast to f16; this sub-lane's share into sx[ray][*].
__device__ __forceinline__ void features_part(const float *d, int q, float *sx) {
    if (q == 0)
#pragma unroll
        for (int c = 0; c < 3; ++c) sx[c] = r16(d[c]);
#pragma unroll
    for (int i = 0; i < (12 + kSub - 1) / kSub; ++i) {
        const int col = q + kSub * i;  // 0..11: frequency col >> 1, sin / cos col & 1
        if (col >= 12) break;
        const float phase = (float)(col & 1) * kHalfPi;
#pragma unroll
        for (int c = 0; c < 3; ++c) sx[3 + 3 * col + c] = r16(sinf(scalbnf(d[c], col >> 1) + phase));
    }
}

// This sub-lane's 16 hidden units (f16 values) and the full f16 output
// pre-activation (partials combined across the ray's four lanes).
__device__ __forceinline__ void mlp_part(const W &w, const float *x, int q, float h[kPer],
                                        float o[kOut]) {
    static_assert(kPer == 4, "one float4 of hidden units per sub-lane");
    // the four units' sums side by side, each in input order (the same fmaf
    // chain per unit as one unit at a time)
    float a[kPer] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < kIn; ++i) {
        const float4 wv = *reinterpret_cast<const float4 *>(&w.w1t[i * kHid + kPer * q]);
        a[0] = fmaf(x[i], wv.x, a[0]);
        a[1] = fmaf(x[i], wv.y, a[1]);
        a[2] = fmaf(x[i], wv.z, a[2]);
        a[3] = fmaf(x[i], wv.w, a[3]);
    }
#pragma unroll
    for (int jj = 0; jj < kPer; ++jj) {
        const float v = a[jj] + w.b1[kPer * q + jj];
        h[jj] = r16(v > 0.0f ? v : 0.0f);
    }
#pragma unroll
    for (int k = 0; k < kOut; ++k) {
        float a = 0.0f;
        const float4 wv = *reinterpret_cast<const float4 *>(&w.w2[k * kHid + kPer * q]);
        const float w2q[kPer] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
        for (int jj = 0; jj < kPer; ++jj) a = fmaf(h[jj], w2q[jj], a);
#pragma unroll
        for (int o2 = 1; o2 < kSub; o2 <<= 1) a = a + __shfl_xor(a, o2, 64);
        o[k] = r16(a + w.b2[k]);
    }
}

// A ray's staged features (16-byte aligned row of kIn + 1 floats) into x:
// nine 16-byte reads and three words instead of 39 reads
__device__ __forceinline__ void load_x(const float *row, bool live, float (&x)[kIn]) {
#pragma unroll
    for (int i = 0; i < kIn / 4; ++i) {
        const float4 v = *reinterpret_cast<const float4 *>(row + 4 * i);
        x[4 * i] = live ? v.x : 0.0f;
        x[4 * i + 1] = live ? v.y : 0.0f;
        x[4 * i + 2] = live ? v.z : 0.0f;
        x[4 * i + 3] = live ? v.w : 0.0f;
    }
#pragma unroll
    for (int i = kIn / 4 * 4; i < kIn; ++i) x[i] = live ? row[i] : 0.0f;
}

__device__ __forceinline__ float sigmoid16(float o) { return r16(1.0f / (1.0f + expf(-o))); }

__device__ __forceinline__ void write_outputs(uint32_t N, uint32_t n, const float bg[3],
                                             const float *ws, const float *depth,
                                             const float *image, const float *nears,
                                             const float *fars, float *out_image,
                                             float *out_depth, uint8_t *mask) {
    const float t = 1.0f - ws[n];
#pragma unroll
    for (int k = 0; k < 3; ++k) out_image[(size_t)k * N + n] = image[3 * (size_t)n + k] + t * bg[k];
    const float nr = nears[n], fr = fars[n];
    const float dd = depth[n] - nr;
    out_depth[n] = (dd < 0.0f ? 0.0f : dd) / (fr - nr);
    mask[n] = nr < fr ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_head_fwd_plain(
    uint32_t N, const float *__restrict__ ws, const float *__restrict__ depth,
    const float *__restrict__ image, const float *__restrict__ nears,
    const float *__restrict__ fars, const float *__restrict__ bg_color,
    float *__restrict__ out_image, float *__restrict__ out_depth, uint8_t *__restrict__ mask) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    float bg[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) bg[k] = bg_color ? bg_color[3 * (size_t)n + k] : 1.0f;
    write_outputs(N, n, bg, ws, depth, image, nears, fars, out_image, out_depth, mask);
}

__global__ __launch_bounds__(kThreads) void k_head_fwd_net(
    uint32_t N, const float *__restrict__ ws, const float *__restrict__ depth,
    const float *__restrict__ image, const float *__restrict__ rays_d,
    const float *__restrict__ nears, const float *__restrict__ fars, const float *w1,
    const float *b1, const float *w2, const float *b2, float *__restrict__ out_image,
    float *__restrict__ out_depth, uint8_t *__restrict__ mask) {
    __shared__ W w;
    __shared__ alignas(16) float s_x[kRays][kIn + 1];
    const int q = threadIdx.x & (kSub - 1), r = threadIdx.x / kSub;
    const uint32_t n = blockIdx.x * kRays + r;
    const bool live = n < N;
    // the ray's direction and (sub-lane 0) the mix / depth operands are
    // loaded ahead of the weight staging, so their latency overlaps it
    float d[3] = {0.0f, 0.0f, 0.0f}, tl[7] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (live) {
#pragma unroll
        for (int c = 0; c < 3; ++c) d[c] = rays_d[3 * (size_t)n + c];
        if (q == 0) {
            tl[0] = ws[n];
            tl[1] = depth[n];
#pragma unroll
            for (int k = 0; k < 3; ++k) tl[2 + k] = image[3 * (size_t)n + k];
            tl[5] = nears[n];
            tl[6] = fars[n];
        }
    }
    load_w(w, w1, b1, w2, b2);
    if (live) features_part(d, q, s_x[r]);
    __syncthreads();
    float x[kIn], h[kPer], o[kOut];
    load_x(s_x[r], live, x);
    mlp_part(w, x, q, h, o);
    if (!live || q != 0) return;
    // write_outputs' arithmetic on the preloaded operands
    const float t = 1.0f - tl[0];
#pragma unroll
    for (int k = 0; k < 3; ++k) out_image[(size_t)k * N + n] = tl[2 + k] + t * sigmoid16(o[k]);
    const float dd = tl[1] - tl[5];
    out_depth[n] = (dd < 0.0f ? 0.0f : dd) / (tl[6] - tl[5]);
    mask[n] = tl[5] < tl[6] ? 1 : 0;
}

// Backward.  grad_image [N, 3] = g; grad_ws = -sum_c g_c bg_c; grad_bg =
// g (1 - ws) when bg_color needs it.
__global__ __launch_bounds__(256) void k_head_bwd_plain(
    uint32_t N, const float *__restrict__ g_image /* [3, N] */, const float *__restrict__ ws,
    const float *__restrict__ bg_color, float *__restrict__ grad_image,
    float *__restrict__ grad_ws, float *__restrict__ grad_bg) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    float g[3], sw = 0.0f;
    const float t = 1.0f - ws[n];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        g[k] = g_image[(size_t)k * N + n];
        grad_image[3 * (size_t)n + k] = g[k];
        const float bg = bg_color ? bg_color[3 * (size_t)n + k] : 1.0f;
        sw = sw + g[k] * bg;
        if (grad_bg) grad_bg[3 * (size_t)n + k] = g[k] * t;
    }
    grad_ws[n] = -sw;
}

constexpr float kLo = 1e-5f, kHi = 1.0f - 1e-5f;

// d loss / d ws of lambda * mean(entropy(clamp(ws))) for upstream gradient g:
// g * lambda / N * log2((1 - a) / a), zero where the clamp is active.
__device__ __forceinline__ float entropy_grad(uint32_t N, float a, const float *g, float lambda) {
    const float scale = g[0] * lambda / (float)N;
    return (a >= kLo && a <= kHi) ? scale * (log2f(1.0f - a) - log2f(a)) : 0.0f;
}

// The forward's operands and outputs for the combined launch (FWD).
struct FwdIO {
    const float *depth, *image, *nears, *fars;
    float *out_image, *out_depth;
    uint8_t *mask;
};

// Network backward: the forward is recomputed (four lanes per ray), then the
// sigmoid and the two f16 Linear layers are run backward and this block's
// weight-gradient partials (f32 sums over its 64 rays of f16 products) formed
// from LDS images of the activations.  FWD: the recomputed forward is also the
// forward's output (k_head_fwd_net's values bit for bit: the same mlp_part,
// sigmoid and mix), so a step whose upstream gradient does not depend on
// pred_rgb (the native step's injected SDS gradient) runs the head as ONE
// launch instead of two.
template <bool FWD>
__global__ __launch_bounds__(kThreads) void k_head_bwd_net(
    uint32_t N, const float *__restrict__ g_image /* [3, N] */, const float *__restrict__ ws,
    const float *__restrict__ rays_d, const float *w1, const float *b1, const float *w2,
    const float *b2, float *__restrict__ grad_image, float *__restrict__ grad_ws,
    float *__restrict__ partial, const float *__restrict__ ent_grad_loss, float ent_lambda,
    FwdIO io) {
    __shared__ W w;
    __shared__ alignas(16) float s_x[kRays][kIn + 1];
    __shared__ half_t s_dh[kRays][kHid];  // relu-masked hidden grads (f16 values)
    __shared__ half_t s_h[kRays][kHid];   // hidden activations
    __shared__ float s_do[kRays][4];      // output pre-activation grads (f16 values)
    load_w(w, w1, b1, w2, b2);
    const int q = threadIdx.x & (kSub - 1), r = threadIdx.x / kSub;
    const uint32_t n = blockIdx.x * kRays + r;
    const bool live = n < N;
    if (live) features_part(rays_d + 3 * (size_t)n, q, s_x[r]);
    else if (q == 0)
        for (int i = 0; i < kIn; ++i) s_x[r][i] = 0.0f;
    __syncthreads();
    float x[kIn], h[kPer], o[kOut];
    load_x(s_x[r], true, x);
    mlp_part(w, x, q, h, o);
    float g[3] = {0.0f, 0.0f, 0.0f}, bg[3];
    if (live)
#pragma unroll
        for (int k = 0; k < 3; ++k) g[k] = g_image[(size_t)k * N + n];
#pragma unroll
    for (int k = 0; k < 3; ++k) bg[k] = sigmoid16(o[k]);
    if (FWD && live && q == 0) {  // write_outputs on the recomputed background
        const float t = 1.0f - ws[n];
#pragma unroll
        for (int k = 0; k < 3; ++k)
            io.out_image[(size_t)k * N + n] = io.image[3 * (size_t)n + k] + t * bg[k];
        const float nr = io.nears[n], fr = io.fars[n];
        const float dd = io.depth[n] - nr;
        io.out_depth[n] = (dd < 0.0f ? 0.0f : dd) / (fr - nr);
        io.mask[n] = nr < fr ? 1 : 0;
    }
    if (live && q == 0) {
        // ((1 - ws) * bg) backward: d ws = -(sum_c g_c * bg_c)
        float sw = 0.0f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            grad_image[3 * (size_t)n + k] = g[k];
            sw = sw + g[k] * bg[k];
        }
        // the entropy regulariser's gradient added as autograd sums the two
        // uses of ws (k_entropy_bwd's value, same f32 arithmetic)
        grad_ws[n] = ent_grad_loss ? -sw + entropy_grad(N, ws[n], ent_grad_loss, ent_lambda)
                                   : -sw;
    }
    const float t = live ? 1.0f - ws[n] : 0.0f;
    float dout[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float dbg = r16(g[k] * t);             // grad of the f16 bg
        dout[k] = r16(dbg * (1.0f - bg[k]) * bg[k]);  // sigmoid_backward, f16
    }
#pragma unroll
    for (int jj = 0; jj < kPer; ++jj) {
        const int j = kPer * q + jj;
        float a = 0.0f;
#pragma unroll
        for (int k = 0; k < kOut; ++k) a = fmaf(dout[k], w.w2[k * kHid + j], a);
        s_dh[r][j] = (half_t)(h[jj] > 0.0f ? r16(a) : 0.0f);
        s_h[r][j] = (half_t)h[jj];
    }
    if (q == 0)
#pragma unroll
        for (int k = 0; k < kOut; ++k) s_do[r][k] = dout[k];
    __syncthreads();
    float *out = partial + (size_t)blockIdx.x * kParams;
    for (int p = threadIdx.x; p < kParams; p += blockDim.x) {
        float s = 0.0f;
        if (p < kW1) {
            const int j = p / kIn, i = p - j * kIn;
            for (int y = 0; y < kRays; ++y) s = fmaf((float)s_dh[y][j], s_x[y][i], s);
        } else if (p < kW1 + kB1) {
            const int j = p - kW1;
            for (int y = 0; y < kRays; ++y) s += (float)s_dh[y][j];
        } else if (p < kW1 + kB1 + kW2) {
            const int k = (p - kW1 - kB1) / kHid, j = (p - kW1 - kB1) - k * kHid;
            for (int y = 0; y < kRays; ++y) s = fmaf(s_do[y][k], (float)s_h[y][j], s);
        } else {
            const int k = p - kW1 - kB1 - kW2;
            for (int y = 0; y < kRays; ++y) s += s_do[y][k];
        }
        out[p] = s;
    }
}

// Fixed-order sum of the per-block partials: block = 64 outputs, its 16
// waves take every 16th partial, then a fixed-order sum of the 16.
// (declared ahead of k_head_wsum, which may run it as its last block)
__device__ __forceinline__ void entropy_loss_block(uint32_t N, const float *__restrict__ ws,
                                                   float lambda, float *__restrict__ loss);

// With `loss`, one extra (last) block computes the entropy loss of ws — the
// forward value k_entropy_fwd would give, by the same code — so the native
// step needs no launch of its own for it.
__global__ __launch_bounds__(1024) void k_head_wsum(const float *__restrict__ partial,
                                                    uint32_t blocks, float *gw1, float *gb1,
                                                    float *gw2, float *gb2,
                                                    const float *__restrict__ ent_ws = nullptr,
                                                    uint32_t ent_n = 0, float ent_lambda = 0.0f,
                                                    float *__restrict__ loss = nullptr) {
    if (loss && blockIdx.x == gridDim.x - 1) {
        entropy_loss_block(ent_n, ent_ws, ent_lambda, loss);
        return;
    }
    __shared__ float red[16][64];
    const int o = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int p = blockIdx.x * 64 + o;
    float s = 0.0f;
    if (p < kParams) {
        // rows grp, grp + 16, ... added in that order; eight loads in flight
        uint32_t b = grp;
        for (; b + 7 * 16 < blocks; b += 8 * 16) {
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = partial[(size_t)(b + 16 * u) * kParams + p];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += x[u];
        }
        for (; b < blocks; b += 16) s += partial[(size_t)b * kParams + p];
    }
    red[grp][o] = s;
    __syncthreads();
    if (grp != 0 || p >= kParams) return;
    s = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i][o];
    if (p < kW1) gw1[p] = s;
    else if (p < kW1 + kB1) gb1[p - kW1] = s;
    else if (p < kW1 + kB1 + kW2) gw2[p - kW1 - kB1] = s;
    else gb2[p - kW1 - kB1 - kW2] = s;
}

// ---------------------------------------------------------------- entropy
// lambda * mean(entropy(clamp(ws))) by one 1024-thread block (fixed order).
__device__ __forceinline__ void entropy_loss_block(uint32_t N, const float *__restrict__ ws,
                                                   float lambda, float *__restrict__ loss) {
    __shared__ double part[16];
    double s = 0.0;
    // elements n, n + blockDim, ... added in that order; eight loads in flight
    // (one dependent load per element left this single block latency-bound)
    auto term = [](float a) {
        a = a < kLo ? kLo : (a > kHi ? kHi : a);
        return -a * log2f(a) - (1.0f - a) * log2f(1.0f - a);
    };
    uint32_t n = threadIdx.x;
    for (; n + 7 * blockDim.x < N; n += 8 * blockDim.x) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ws[n + u * blockDim.x];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += (double)term(v[u]);
    }
    for (; n < N; n += blockDim.x) s += (double)term(ws[n]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += part[i];
        loss[0] = lambda * (float)(t / (double)N);
    }
}

__global__ __launch_bounds__(1024) void k_entropy_fwd(uint32_t N, const float *__restrict__ ws,
                                                      float lambda, float *__restrict__ loss) {
    entropy_loss_block(N, ws, lambda, loss);
}

// d loss / d ws = g * lambda / N * log2((1 - a) / a), zero where the clamp is
// active (torch.clamp's backward passes the gradient for lo <= ws <= hi).
template <bool ACC>
__global__ __launch_bounds__(256) void k_entropy_bwd(uint32_t N, const float *__restrict__ ws,
                                                     const float *__restrict__ g, float lambda,
                                                     float *__restrict__ grad_ws) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const float v = entropy_grad(N, ws[n], g, lambda);
    grad_ws[n] = ACC ? grad_ws[n] + v : v;
}

}  // namespace hd
}  // namespace dfhip

using namespace dfhip;

extern "C" uint32_t dfhip_ray_head_partial_floats(uint32_t N) {
    return ceil_div(N, (uint32_t)hd::kRays) * (uint32_t)hd::kParams;
}

extern "C" int dfhip_ray_head_forward(uint32_t N, const float *ws, const float *depth,
                                      const float *image, const float *rays_d, const float *nears,
                                      const float *fars, const float *w1, const float *b1,
                                      const float *w2, const float *b2, const float *bg_color,
                                      float *out_image, float *out_depth, uint8_t *mask,
                                      dfhip_stream_t stream) {
    const char *name = "ray_head_forward";
    if (N == 0) return DFHIP_OK;
    if (!ws || !depth || !image || !nears || !fars || !out_image || !out_depth || !mask) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    const bool net = w1 != nullptr;
    if (net && (!b1 || !w2 || !b2 || !rays_d)) {
        set_error("%s: the background network needs w1, b1, w2, b2 and rays_d", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (net)
        hd::k_head_fwd_net<<<ceil_div(N, (uint32_t)hd::kRays), hd::kThreads, 0, s>>>(
            N, ws, depth, image, rays_d, nears, fars, w1, b1, w2, b2, out_image, out_depth, mask);
    else
        hd::k_head_fwd_plain<<<ceil_div(N, 256u), 256, 0, s>>>(N, ws, depth, image, nears, fars,
                                                               bg_color, out_image, out_depth,
                                                               mask);
    return check_launch(name);
}

static int ray_head_backward(uint32_t N, const float *g_image, const float *ws,
                             const float *rays_d, const float *w1, const float *b1,
                             const float *w2, const float *b2, const float *bg_color,
                             float *grad_image, float *grad_ws, float *grad_bg, float *partial,
                             float *gw1, float *gb1, float *gw2, float *gb2,
                             const float *ent_grad_loss, float ent_lambda,
                             dfhip_stream_t stream, float *ent_loss = nullptr,
                             const hd::FwdIO *fwd = nullptr) {
    const char *name = "ray_head_backward";
    if (N == 0) return DFHIP_OK;
    if (!g_image || !ws || !grad_image || !grad_ws) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    const bool net = w1 != nullptr;
    if (net && (!b1 || !w2 || !b2 || !rays_d || !partial || !gw1 || !gb1 || !gw2 || !gb2)) {
        set_error("%s: the background network needs its weights, rays_d, partial and grads",
                  name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (net) {
        const uint32_t blocks = ceil_div(N, (uint32_t)hd::kRays);
        if (fwd)
            hd::k_head_bwd_net<true><<<blocks, hd::kThreads, 0, s>>>(
                N, g_image, ws, rays_d, w1, b1, w2, b2, grad_image, grad_ws, partial,
                ent_grad_loss, ent_lambda, *fwd);
        else
            hd::k_head_bwd_net<false><<<blocks, hd::kThreads, 0, s>>>(
                N, g_image, ws, rays_d, w1, b1, w2, b2, grad_image, grad_ws, partial,
                ent_grad_loss, ent_lambda, hd::FwdIO{});
        hd::k_head_wsum<<<ceil_div((uint32_t)hd::kParams, 64u) + (ent_loss ? 1u : 0u), 1024, 0,
                          s>>>(partial, blocks, gw1, gb1, gw2, gb2, ws, N, ent_lambda,
                               ent_loss);
    } else {
        hd::k_head_bwd_plain<<<ceil_div(N, 256u), 256, 0, s>>>(N, g_image, ws, bg_color,
                                                               grad_image, grad_ws, grad_bg);
        if (ent_grad_loss)
            hd::k_entropy_bwd<true><<<ceil_div(N, 256u), 256, 0, s>>>(N, ws, ent_grad_loss,
                                                                     ent_lambda, grad_ws);
        if (ent_loss) hd::k_entropy_fwd<<<1, 1024, 0, s>>>(N, ws, ent_lambda, ent_loss);
    }
    return check_launch(name);
}

extern "C" int dfhip_ray_head_backward(uint32_t N, const float *g_image, const float *ws,
                                       const float *rays_d, const float *w1, const float *b1,
                                       const float *w2, const float *b2, const float *bg_color,
                                       float *grad_image, float *grad_ws, float *grad_bg,
                                       float *partial, float *gw1, float *gb1, float *gw2,
                                       float *gb2, dfhip_stream_t stream) {
    return ray_head_backward(N, g_image, ws, rays_d, w1, b1, w2, b2, bg_color, grad_image,
                             grad_ws, grad_bg, partial, gw1, gb1, gw2, gb2, nullptr, 0.0f,
                             stream);
}

extern "C" int dfhip_ray_head_backward_entropy(
    uint32_t N, const float *g_image, const float *ws, const float *rays_d, const float *w1,
    const float *b1, const float *w2, const float *b2, const float *bg_color, float *grad_image,
    float *grad_ws, float *grad_bg, float *partial, float *gw1, float *gb1, float *gw2,
    float *gb2, const float *grad_loss, float lambda, dfhip_stream_t stream) {
    if (N > 0 && !grad_loss) {
        set_error("ray_head_backward_entropy: null grad_loss");
        return DFHIP_EINVAL;
    }
    return ray_head_backward(N, g_image, ws, rays_d, w1, b1, w2, b2, bg_color, grad_image,
                             grad_ws, grad_bg, partial, gw1, gb1, gw2, gb2, grad_loss, lambda,
                             stream);
}

// dfhip_ray_head_backward_entropy that also writes the entropy loss
// (dfhip_entropy_forward's value) to `loss`, inside the weight-sum launch.
extern "C" int dfhip_ray_head_backward_entropy_loss(
    uint32_t N, const float *g_image, const float *ws, const float *rays_d, const float *w1,
    const float *b1, const float *w2, const float *b2, const float *bg_color, float *grad_image,
    float *grad_ws, float *grad_bg, float *partial, float *gw1, float *gb1, float *gw2,
    float *gb2, const float *grad_loss, float lambda, float *loss, dfhip_stream_t stream) {
    if (!loss) {
        set_error("ray_head_backward_entropy_loss: null loss");
        return DFHIP_EINVAL;
    }
    if (N == 0) return dfhip_entropy_forward(N, ws, lambda, loss, stream);
    if (!grad_loss) {
        set_error("ray_head_backward_entropy_loss: null grad_loss");
        return DFHIP_EINVAL;
    }
    return ray_head_backward(N, g_image, ws, rays_d, w1, b1, w2, b2, bg_color, grad_image,
                             grad_ws, grad_bg, partial, gw1, gb1, gw2, gb2, grad_loss, lambda,
                             stream, loss);
}

// dfhip_ray_head_forward + dfhip_ray_head_backward_entropy_loss in two
// launches instead of three, for an upstream gradient that does not depend on
// the forward's outputs (background network only).
extern "C" int dfhip_ray_head_forward_backward_entropy_loss(
    uint32_t N, const float *ws, const float *depth, const float *image, const float *rays_d,
    const float *nears, const float *fars, const float *w1, const float *b1, const float *w2,
    const float *b2, float *out_image, float *out_depth, uint8_t *mask, const float *g_image,
    float *grad_image, float *grad_ws, float *partial, float *gw1, float *gb1, float *gw2,
    float *gb2, const float *grad_loss, float lambda, float *loss, dfhip_stream_t stream) {
    const char *name = "ray_head_forward_backward_entropy_loss";
    if (!loss) {
        set_error("%s: null loss", name);
        return DFHIP_EINVAL;
    }
    if (N == 0) return dfhip_entropy_forward(N, ws, lambda, loss, stream);
    if (!w1 || !depth || !image || !nears || !fars || !out_image || !out_depth || !mask ||
        !grad_loss) {
        set_error("%s: null pointer (the combined launch needs the background network)", name);
        return DFHIP_EINVAL;
    }
    const hd::FwdIO io{depth, image, nears, fars, out_image, out_depth, mask};
    return ray_head_backward(N, g_image, ws, rays_d, w1, b1, w2, b2, nullptr, grad_image,
                             grad_ws, nullptr, partial, gw1, gb1, gw2, gb2, grad_loss, lambda,
                             stream, loss, &io);
}

extern "C" int dfhip_entropy_forward(uint32_t N, const float *ws, float lambda, float *loss,
                                     dfhip_stream_t stream) {
    if (!ws || !loss) {
        set_error("entropy_forward: null pointer");
        return DFHIP_EINVAL;
    }
    hd::k_entropy_fwd<<<1, 1024, 0, as_stream(stream)>>>(N, ws, lambda, loss);
    return check_launch("entropy_forward");
}

extern "C" int dfhip_entropy_backward(uint32_t N, const float *ws, const float *grad_loss,
                                      float lambda, float *grad_ws, dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    if (!ws || !grad_loss || !grad_ws) {
        set_error("entropy_backward: null pointer");
        return DFHIP_EINVAL;
    }
    hd::k_entropy_bwd<false><<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(
        N, ws, grad_loss, lambda, grad_ws);
    return check_launch("entropy_backward");
}

extern "C" int dfhip_entropy_backward_accumulate(uint32_t N, const float *ws,
                                                 const float *grad_loss, float lambda,
                                                 float *grad_ws, dfhip_stream_t stream) {
    if (N == 0) return DFHIP_OK;
    if (!ws || !grad_loss || !grad_ws) {
        set_error("entropy_backward_accumulate: null pointer");
        return DFHIP_EINVAL;
    }
    hd::k_entropy_bwd<true><<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(
        N, ws, grad_loss, lambda, grad_ws);
    return check_launch("entropy_backward_accumulate");
}
