// Occupancy-grid refresh without host synchronisation (reference
// nerf/renderer.py:562-615 NeRFRenderer.update_extra_state, run every
// `update_extra_interval` = 16 train steps).
//
// The reference scatters the jittered density queries into a temporary grid,
// applies the EMA-max with boolean-mask indexing, reads the mean density to the
// host (`.item()`), and packs the bitfield with that host threshold: two host
// round trips that drain the GPU queue every 16 steps.  Here:
//   1. dfhip_density_grid_ema: per queried cell, new = max(old * decay, sigma)
//      where old >= 0 (the reference's `valid` mask, taken before the update),
//      and the valid cells' new values summed in f64 into acc[0], their count
//      into acc[1] (per-workgroup partials, then a fixed-order sum);
//   2. dfhip_packbits_mean: thresh = min(acc[0] / acc[1], density_thresh)
//      evaluated on the device, the bitfield packed with it (strict >, as
//      raymarching.cu:263-290), and the mean written for the host to read
//      lazily.
// The f64 sum makes the mean exact to f32 rounding; the reference's f32 tree
// reduction (torch.mean) is order-dependent in the last bits.
#include "common.h"

#include <math.h>

namespace dfhip {
namespace occ {

__device__ __forceinline__ float torch_maximum(float a, float b) {
    return (isnan(a) || isnan(b)) ? NAN : fmaxf(a, b);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One point per thread, point p -> cell indices[p] (cascade offset included).
// The caller queries every cell exactly once per refresh (the reference's
// loops cover the whole grid), so the sum over the touched valid cells is the
// sum over all valid cells.
__global__ __launch_bounds__(256) void k_grid_ema(const float *__restrict__ sigma,
                                                  const int32_t *__restrict__ indices,
                                                  uint32_t n, uint32_t cells, float decay,
                                                  float *__restrict__ grid,
                                                  double *__restrict__ partial) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    double s = 0.0, c = 0.0;
    if (p < n) {
        const int32_t cell = indices[p];
        if (cell >= 0 && (uint32_t)cell < cells) {
            const float old = grid[cell];
            if (old >= 0.0f) {  // valid (the mask is taken before the update)
                const float v = torch_maximum(old * decay, sigma[p]);
                grid[cell] = v;
                s = (double)v;
                c = 1.0;
            }
        }
    }
    __shared__ double ws[2][4];
    s = wave_sum(s);
    c = wave_sum(c);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        ws[0][wave] = s;
        ws[1][wave] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ts = 0.0, tc = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            ts += ws[0][w];
            tc += ws[1][w];
        }
        // per-block partials (one f64 atomic pair per block on two addresses
        // serialised at the memory-side atomic unit: ~0.2 ms for 8k blocks)
        partial[2 * blockIdx.x] = ts;
        partial[2 * blockIdx.x + 1] = tc;
    }
}

// acc[0..1] += the fixed-order sum of the per-block partials (one workgroup).
__global__ __launch_bounds__(1024) void k_grid_ema_sum(const double *__restrict__ partial,
                                                       uint32_t blocks, double *acc) {
    __shared__ double red[2][16];
    double s = 0.0, c = 0.0;
    for (uint32_t b = threadIdx.x; b < blocks; b += blockDim.x) {
        s += partial[2 * b];
        c += partial[2 * b + 1];
    }
    s = wave_sum(s);
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = s;
        red[1][threadIdx.x >> 6] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ts = 0.0, tc = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            ts += red[0][w];
            tc += red[1][w];
        }
        acc[0] += ts;
        acc[1] += tc;
    }
}

__device__ __forceinline__ float mean_thresh(const double *acc, float density_thresh,
                                             float *mean) {
    const double cnt = acc[1];
    const float m = cnt > 0.0 ? (float)(acc[0] / cnt) : NAN;
    if (mean) *mean = m;
    // Python min(mean, thresh): thresh if mean is NaN (comparison false)
    return (m < density_thresh) ? m : density_thresh;
}

__global__ __launch_bounds__(256) void k_packbits_mean(const float *__restrict__ grid,
                                                       uint32_t N, const double *__restrict__ acc,
                                                       float density_thresh,
                                                       uint8_t *__restrict__ bitfield,
                                                       float *__restrict__ mean_out) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    float mean;
    const float thresh = mean_thresh(acc, density_thresh, &mean);
    if (n == 0 && mean_out) mean_out[0] = mean;
    if (n >= N) return;
    const float4 *g = reinterpret_cast<const float4 *>(grid) + 2 * (size_t)n;
    const float4 a = g[0], b = g[1];
    const uint32_t bits = (a.x > thresh) | ((a.y > thresh) << 1) | ((a.z > thresh) << 2) |
                          ((a.w > thresh) << 3) | ((b.x > thresh) << 4) |
                          ((b.y > thresh) << 5) | ((b.z > thresh) << 6) | ((b.w > thresh) << 7);
    bitfield[n] = (uint8_t)bits;
}

// mean_count = int(step_counter[:total_step, 0].sum() / total_step)
// (renderer.py:611-613; the sum is exact in int64, the quotient truncated
// toward zero as Python's int() of the float quotient does for a sum < 2^53).
__global__ __launch_bounds__(64) void k_mean_count(const int32_t *__restrict__ step_counter,
                                                   uint32_t total_step,
                                                   int64_t *__restrict__ mean_count) {
    const uint32_t lane = threadIdx.x;
    int64_t s = lane < total_step ? (int64_t)step_counter[2 * lane] : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) mean_count[0] = (int64_t)((double)s / (double)total_step);
}

}  // namespace occ
}  // namespace dfhip

using namespace dfhip;

extern "C" int dfhip_density_grid_ema(const float *sigma, const int32_t *indices, uint32_t n,
                                      uint32_t cells, float decay, float *grid, double *acc,
                                      dfhip_stream_t stream) {
    const char *name = "density_grid_ema";
    if (n == 0) return DFHIP_OK;
    if (!sigma || !indices || !grid || !acc) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    // per-block partials in stream-ordered scratch, then a fixed-order sum
    const uint32_t blocks = ceil_div(n, 256u);
    hipStream_t s = as_stream(stream);
    double *partial = nullptr;
    if (hipMallocAsync((void **)&partial, sizeof(double) * 2 * blocks, s) != hipSuccess) {
        set_error("%s: scratch allocation failed", name);
        return DFHIP_EINVAL;
    }
    occ::k_grid_ema<<<blocks, 256, 0, s>>>(sigma, indices, n, cells, decay, grid, partial);
    occ::k_grid_ema_sum<<<1, 1024, 0, s>>>(partial, blocks, acc);
    (void)hipFreeAsync(partial, s);
    return check_launch(name);
}

extern "C" int dfhip_packbits_mean(const float *grid, uint32_t N, const double *acc,
                                   float density_thresh, uint8_t *bitfield, float *mean_out,
                                   dfhip_stream_t stream) {
    const char *name = "packbits_mean";
    if (N == 0) return DFHIP_OK;
    if (!grid || !acc || !bitfield) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (reinterpret_cast<uintptr_t>(grid) % 16 != 0) {
        set_error("%s: grid must be 16-byte aligned", name);
        return DFHIP_EINVAL;
    }
    occ::k_packbits_mean<<<ceil_div(N, 256u), 256, 0, as_stream(stream)>>>(
        grid, N, acc, density_thresh, bitfield, mean_out);
    return check_launch(name);
}

extern "C" int dfhip_mean_count(const int32_t *step_counter, uint32_t total_step,
                                int64_t *mean_count, dfhip_stream_t stream) {
    const char *name = "mean_count";
    if (total_step == 0) return DFHIP_OK;
    if (!step_counter || !mean_count) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (total_step > 64) {
        set_error("%s: total_step must be <= 64 (got %u)", name, total_step);
        return DFHIP_EINVAL;
    }
    occ::k_mean_count<<<1, 64, 0, as_stream(stream)>>>(step_counter, total_step, mean_count);
    return check_launch(name);
}
