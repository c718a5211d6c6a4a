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

struct Tensor {
    float *p;
    const float *g;
    float *m;
    float *v;
    float *step;
    uint64_t n;
    uint64_t start;  // first element in the concatenated index space
    float lr, b1, b2, eps, wd;
};

struct Batch {
    Tensor t[kMaxTensors];
    int count;
    uint64_t total;
};

__device__ __forceinline__ int find_tensor(const Batch &B, uint64_t i) {
    int k = 0;
    while (k + 1 < B.count && B.t[k + 1].start <= i) ++k;
    return k;
}

__global__ __launch_bounds__(256) void k_nonfinite(Batch B, float *found_inf) {
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const Tensor &t = B.t[find_tensor(B, i)];
        bad |= !isfinite(t.g[i - t.start]);
    }
    if (__syncthreads_or(bad) && threadIdx.x == 0) *found_inf = 1.0f;
}

__global__ __launch_bounds__(256) void k_adam(Batch B, const float *scale, const float *found_inf) {
    if (*found_inf != 0.0f) return;
    const float s = *scale;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const Tensor &t = B.t[find_tensor(B, i)];
        const uint64_t j = i - t.start;
        const float step = *t.step + 1.0f;
        float g = t.g[j] / s;
        float p = t.p[j];
        if (t.wd != 0.0f) g += t.wd * p;
        float m = t.m[j], v = t.v[j];
        m = t.b1 * m + (1.0f - t.b1) * g;
        v = t.b2 * v + (1.0f - t.b2) * g * g;
        const float bc1 = 1.0f - powf(t.b1, step);
        const float step_size = t.lr / bc1;
        const float bc2 = 1.0f - powf(t.b2, step);
        const float denom = (sqrtf(v) / sqrtf(bc2)) + t.eps;
        p -= step_size * m / denom;
        t.p[j] = p;
        t.m[j] = m;
        t.v[j] = v;
    }
}

__global__ void k_finalize(Batch B, float *scale, int32_t *growth_tracker, float *found_inf,
                           float growth_factor, float backoff_factor, int growth_interval) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const bool inf = *found_inf != 0.0f;
    if (!inf)
        for (int k = 0; k < B.count; ++k) *B.t[k].step += 1.0f;
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
    *found_inf = 0.0f;
}

}  // namespace opt
}  // namespace dfhip

using namespace dfhip;

extern "C" int dfhip_adam_amp_step(int count, float *const *params, const float *const *grads,
                                   float *const *exp_avg, float *const *exp_avg_sq,
                                   float *const *steps, const uint64_t *numel, const float *lr,
                                   const float *beta1, const float *beta2, const float *eps,
                                   const float *weight_decay, float *scale,
                                   int32_t *growth_tracker, float *found_inf,
                                   float growth_factor, float backoff_factor,
                                   int growth_interval, dfhip_stream_t stream) {
    const char *name = "adam_amp_step";
    if (count <= 0) return DFHIP_OK;
    if (count > opt::kMaxTensors) {
        set_error("%s: at most %d tensors (got %d)", name, opt::kMaxTensors, count);
        return DFHIP_EINVAL;
    }
    if (!scale || !growth_tracker || !found_inf) {
        set_error("%s: null scaler state", name);
        return DFHIP_EINVAL;
    }
    opt::Batch B;
    B.count = count;
    uint64_t total = 0;
    for (int k = 0; k < count; ++k) {
        if (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k] || !steps[k]) {
            set_error("%s: null pointer in tensor %d", name, k);
            return DFHIP_EINVAL;
        }
        opt::Tensor &t = B.t[k];
        t.p = params[k];
        t.g = grads[k];
        t.m = exp_avg[k];
        t.v = exp_avg_sq[k];
        t.step = steps[k];
        t.n = numel[k];
        t.start = total;
        t.lr = lr[k];
        t.b1 = beta1[k];
        t.b2 = beta2[k];
        t.eps = eps[k];
        t.wd = weight_decay[k];
        total += numel[k];
    }
    B.total = total;
    hipStream_t s = as_stream(stream);
    const uint64_t want = ceil_div<uint64_t>(total, 256);
    const uint32_t blocks = (uint32_t)(want < 2048 ? (want ? want : 1) : 2048);
    opt::k_nonfinite<<<blocks, 256, 0, s>>>(B, found_inf);
    opt::k_adam<<<blocks, 256, 0, s>>>(B, scale, found_inf);
    opt::k_finalize<<<1, 64, 0, s>>>(B, scale, growth_tracker, found_inf, growth_factor,
                                     backoff_factor, growth_interval);
    return check_launch(name);
}
