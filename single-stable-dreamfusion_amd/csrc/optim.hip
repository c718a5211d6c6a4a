// GradScaler + Adam step of the SDS train loop as three launches (reference
// nerf/utils.py:708-713: scaler.scale(loss).backward(); scaler.step(optimizer);
// scaler.update(), with torch.optim.Adam(betas=(0.9, 0.99), eps=1e-15),
// main.py).  torch's path for a fused Adam is ~15 launches and ~0.4 ms of host
// Python per step (non-finite check with a dummy scale, foreach step += 1,
// the fused kernel, foreach step -= found_inf, the scale update); here:
//
//   1. k_nonfinite: found_inf = any(!isfinite(grad)) over every tensor
//      (torch._amp_foreach_non_finite_check_and_unscale_ with inv_scale 1,
//      as GradScaler._check_inf_per_device does for a fused optimizer);
//   2. k_adam: if !found_inf, per element exactly torch's fused Adam
//      (the bias corrections, per-tensor constants, are evaluated once per
//      block with the same f32 expressions; blocks map to tensors through a
//      block table and stream float4s)
//      (ATen FusedAdamKernel / fused_adam_utils.cuh, ADAM mode, no amsgrad):
//        g = grad / scale;  g += wd * p
//        m = b1 * m + (1 - b1) * g;  v = b2 * v + (1 - b2) * g * g
//        step_size = lr / (1 - b1^t);  denom = sqrt(v) / sqrt(1 - b2^t) + eps
//        p -= step_size * m / denom                     (t = step + 1)
//   3. k_finalize: step += 1 per tensor unless found_inf, then
//      torch._amp_update_scale_ (backoff 0.5 on inf, x2 after 2000 clean
//      steps).
// The per-tensor descriptors (pointers, sizes, group hyper-parameters) travel
// by value; the scale, growth tracker, found_inf and step counters are the
// torch GradScaler / Adam state tensors themselves, so checkpoints keep the
// reference's layout.
#include "common.h"

#include <math.h>

namespace dfhip {
namespace opt {

constexpr int kMaxTensors = 24;
constexpr uint32_t kThreads = 256;
constexpr uint32_t kPerBlock = kThreads * 4 * 2;  // two float4 per thread

struct Tensor {
    float *p;
    const float *g;
    float *m;
    float *v;
    float *step;
    uint64_t n;
    uint32_t block0;  // first block of this tensor (blocks of kPerBlock elements)
    float lr, b1, b2, eps, wd;
};

struct Batch {
    Tensor t[kMaxTensors];
    int count;
    uint32_t blocks;
    // device learning rates (graph-replayed step): tensor k's lr is
    // lr_dev[lr_slot[k]] read at run time; null: the by-value t.lr
    const float *lr_dev;
    uint8_t lr_slot[kMaxTensors];
};

// The tensor of (wave-uniform) chunk blk: a scalar scan of the block table.
__device__ __forceinline__ int chunk_tensor(const Batch &B, uint32_t blk) {
    int k = 0;
    while (k + 1 < B.count && B.t[k + 1].block0 <= blk) ++k;
    return k;
}
__device__ __forceinline__ int block_tensor(const Batch &B) { return chunk_tensor(B, blockIdx.x); }

// Elements [e0, e0 + kPerBlock) of tensor t: vectorised when the tensor's
// base is 16-byte aligned and the chunk is whole, else element by element.
template <typename F4, typename F1>
__device__ __forceinline__ void for_chunk(const Tensor &t, uint64_t e0, F4 f4, F1 f1) {
    const bool vec = ((reinterpret_cast<uintptr_t>(t.p) | reinterpret_cast<uintptr_t>(t.g) |
                       reinterpret_cast<uintptr_t>(t.m) | reinterpret_cast<uintptr_t>(t.v)) &
                      15u) == 0 && e0 + kPerBlock <= t.n;
    if (vec) {
#pragma unroll
        for (uint32_t u = 0; u < kPerBlock / (4 * kThreads); ++u) f4(e0 / 4 + u * kThreads + threadIdx.x);
    } else {
        for (uint64_t j = e0 + threadIdx.x; j < t.n && j < e0 + kPerBlock; j += kThreads) f1(j);
    }
}

__global__ __launch_bounds__(kThreads) void k_nonfinite(Batch B, float *found_inf) {
    const Tensor &t = B.t[block_tensor(B)];
    const uint64_t e0 = (uint64_t)(blockIdx.x - t.block0) * kPerBlock;
    bool bad = false;
    for_chunk(
        t, e0,
        [&](uint64_t q) {
            const float4 g = reinterpret_cast<const float4 *>(t.g)[q];
            bad |= !(isfinite(g.x) && isfinite(g.y) && isfinite(g.z) && isfinite(g.w));
        },
        [&](uint64_t j) { bad |= !isfinite(t.g[j]); });
    if (__syncthreads_or(bad) && threadIdx.x == 0) *found_inf = 1.0f;
}

struct AdamK {
    float s, step_size, bc2s;
};

__device__ __forceinline__ float adam1(const Tensor &t, const AdamK &k, float g, float &p,
                                       float &m, float &v) {
    g = g / k.s;
    if (t.wd != 0.0f) g += t.wd * p;
    m = t.b1 * m + (1.0f - t.b1) * g;
    v = t.b2 * v + (1.0f - t.b2) * g * g;
    const float denom = (sqrtf(v) / k.bc2s) + t.eps;
    p -= k.step_size * m / denom;
    return p;
}

// The Adam update of chunk blk (kPerBlock elements of one tensor).
__device__ __forceinline__ void adam_chunk(const Batch &B, uint32_t blk, float scale) {
    const int ti = chunk_tensor(B, blk);
    const Tensor &t = B.t[ti];
    const uint64_t e0 = (uint64_t)(blk - t.block0) * kPerBlock;
    // per-tensor constants (the same f32 expressions torch evaluates per element)
    const float step = *t.step + 1.0f;
    AdamK k;
    k.s = scale;
    const float lr = B.lr_dev ? B.lr_dev[B.lr_slot[ti]] : t.lr;
    k.step_size = lr / (1.0f - powf(t.b1, step));
    k.bc2s = sqrtf(1.0f - powf(t.b2, step));
    for_chunk(
        t, e0,
        [&](uint64_t q) {
            float4 p = reinterpret_cast<float4 *>(t.p)[q];
            float4 m = reinterpret_cast<float4 *>(t.m)[q];
            float4 v = reinterpret_cast<float4 *>(t.v)[q];
            const float4 g = reinterpret_cast<const float4 *>(t.g)[q];
            adam1(t, k, g.x, p.x, m.x, v.x);
            adam1(t, k, g.y, p.y, m.y, v.y);
            adam1(t, k, g.z, p.z, m.z, v.z);
            adam1(t, k, g.w, p.w, m.w, v.w);
            reinterpret_cast<float4 *>(t.p)[q] = p;
            reinterpret_cast<float4 *>(t.m)[q] = m;
            reinterpret_cast<float4 *>(t.v)[q] = v;
        },
        [&](uint64_t j) {
            float p = t.p[j], m = t.m[j], v = t.v[j];
            adam1(t, k, t.g[j], p, m, v);
            t.p[j] = p;
            t.m[j] = m;
            t.v[j] = v;
        });
}

__global__ __launch_bounds__(kThreads) void k_adam(Batch B, const float *scale,
                                                   const float *found_inf) {
    if (*found_inf != 0.0f) return;
    adam_chunk(B, blockIdx.x, *scale);
}

// One wave: lane k bumps tensor k's step (independent RMWs in parallel, not
// one thread's serial chain of dependent global round trips), lane 0 updates
// the scale.
__device__ __forceinline__ void finalize_wave(const Batch &B, bool inf, float *scale,
                                              int32_t *growth_tracker, float *found_inf,
                                              float growth_factor, float backoff_factor,
                                              int growth_interval) {
    const int k = (int)(threadIdx.x & 63);
    if (!inf && k < B.count) *B.t[k].step += 1.0f;
    if (k != 0) return;
    // ATen amp_update_scale_cuda_kernel
    if (inf) {
        *scale = (*scale) * backoff_factor;
        *growth_tracker = 0;
    } else {
        const int successful = *growth_tracker + 1;
        if (successful == growth_interval) {
            const float grown = (*scale) * growth_factor;
            if (isfinite(grown)) *scale = grown;
            *growth_tracker = 0;
        } else {
            *growth_tracker = successful;
        }
    }
    *found_inf = 0.0f;  // every lane read it above; the wave runs in lock step
}

__global__ __launch_bounds__(64) void k_finalize(Batch B, float *scale, int32_t *growth_tracker,
                                                 float *found_inf, float growth_factor,
                                                 float backoff_factor, int growth_interval) {
    if (blockIdx.x != 0) return;
    finalize_wave(B, *found_inf != 0.0f, scale, growth_tracker, found_inf, growth_factor,
                  backoff_factor, growth_interval);
}

}  // namespace opt
}  // namespace dfhip

using namespace dfhip;

namespace dfhip {
namespace opt {

static int adam_amp_step(int count, float *const *params, const float *const *grads,
                         float *const *exp_avg, float *const *exp_avg_sq, float *const *steps,
                         const uint64_t *numel, const float *lr, const int32_t *lr_slot,
                         const float *lr_dev, const float *beta1, const float *beta2,
                         const float *eps, const float *weight_decay, float *scale,
                         int32_t *growth_tracker, float *found_inf, float growth_factor,
                         float backoff_factor, int growth_interval, hipStream_t s) {
    const char *name = "adam_amp_step";
    if (count <= 0) return DFHIP_OK;
    if (count > kMaxTensors) {
        set_error("%s: at most %d tensors (got %d)", name, kMaxTensors, count);
        return DFHIP_EINVAL;
    }
    if (!scale || !growth_tracker || !found_inf) {
        set_error("%s: null scaler state", name);
        return DFHIP_EINVAL;
    }
    Batch B;
    B.count = count;
    B.lr_dev = lr_dev;
    uint32_t blocks = 0;
    for (int k = 0; k < count; ++k) {
        if (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k] || !steps[k]) {
            set_error("%s: null pointer in tensor %d", name, k);
            return DFHIP_EINVAL;
        }
        Tensor &t = B.t[k];
        t.p = params[k];
        t.g = grads[k];
        t.m = exp_avg[k];
        t.v = exp_avg_sq[k];
        t.step = steps[k];
        t.n = numel[k];
        t.block0 = blocks;
        t.lr = lr ? lr[k] : 0.0f;
        if (lr_dev) {
            if (lr_slot[k] < 0 || lr_slot[k] > 255) {
                set_error("%s: lr slot of tensor %d out of range", name, k);
                return DFHIP_EINVAL;
            }
            B.lr_slot[k] = (uint8_t)lr_slot[k];
        }
        t.b1 = beta1[k];
        t.b2 = beta2[k];
        t.eps = eps[k];
        t.wd = weight_decay[k];
        const uint64_t nb = ceil_div<uint64_t>(numel[k], kPerBlock);
        if (nb > 0x7FFFFFFFull - blocks) {
            set_error("%s: tensor %d has an unsupported size", name, k);
            return DFHIP_EINVAL;
        }
        blocks += (uint32_t)nb;
    }
    B.blocks = blocks;
    if (blocks == 0) blocks = 1;  // all tensors empty: one block that finds no work
    k_nonfinite<<<blocks, kThreads, 0, s>>>(B, found_inf);
    k_adam<<<blocks, kThreads, 0, s>>>(B, scale, found_inf);
    k_finalize<<<1, 64, 0, s>>>(B, scale, growth_tracker, found_inf, growth_factor,
                                backoff_factor, growth_interval);
    return check_launch(name);
}

}  // namespace opt
}  // namespace dfhip

extern "C" int dfhip_adam_amp_step(int count, float *const *params, const float *const *grads,
                                   float *const *exp_avg, float *const *exp_avg_sq,
                                   float *const *steps, const uint64_t *numel, const float *lr,
                                   const float *beta1, const float *beta2, const float *eps,
                                   const float *weight_decay, float *scale,
                                   int32_t *growth_tracker, float *found_inf,
                                   float growth_factor, float backoff_factor,
                                   int growth_interval, dfhip_stream_t stream) {
    if (count > 0 && !lr) {
        set_error("adam_amp_step: null lr array");
        return DFHIP_EINVAL;
    }
    return opt::adam_amp_step(count, params, grads, exp_avg, exp_avg_sq, steps, numel, lr,
                              nullptr, nullptr, beta1, beta2, eps, weight_decay, scale,
                              growth_tracker, found_inf, growth_factor, backoff_factor,
                              growth_interval, as_stream(stream));
}

extern "C" int dfhip_adam_amp_step_lr_dev(int count, float *const *params,
                                          const float *const *grads, float *const *exp_avg,
                                          float *const *exp_avg_sq, float *const *steps,
                                          const uint64_t *numel, const int32_t *lr_slot,
                                          const float *lr_dev, const float *beta1,
                                          const float *beta2, const float *eps,
                                          const float *weight_decay, float *scale,
                                          int32_t *growth_tracker, float *found_inf,
                                          float growth_factor, float backoff_factor,
                                          int growth_interval, dfhip_stream_t stream) {
    if (count > 0 && (!lr_slot || !lr_dev)) {
        set_error("adam_amp_step_lr_dev: null lr slot array or device lr");
        return DFHIP_EINVAL;
    }
    return opt::adam_amp_step(count, params, grads, exp_avg, exp_avg_sq, steps, numel, nullptr,
                              lr_slot, lr_dev, beta1, beta2, eps, weight_decay, scale,
                              growth_tracker, found_inf, growth_factor, backoff_factor,
                              growth_interval, as_stream(stream));
}
