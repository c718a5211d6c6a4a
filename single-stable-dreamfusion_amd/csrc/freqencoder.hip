// NeRF positional (frequency) encoding for gfx950.
// Behavioural spec: reference freqencoder/src/freqencoder.cu:28-94.
//   out[b] = [x (D), then for k = 0..deg-1: sin(2^k x) (D), cos(2^k x) (D)]
// with cos written as sin(. + pi/2).  The reference compiles with
// -use_fast_math (__sinf); here the full-precision sinf is used (the outputs
// differ from the reference only by __sinf's own approximation error).
#include "common.h"

#include <math.h>

namespace dfhip {
namespace fe {

constexpr float kHalfPi = 3.141592653589793f / 2.0f;

// One thread per output element (freqencoder.cu:30-58): stores coalesced.
__global__ __launch_bounds__(256) void k_freq_fwd(const float *__restrict__ inputs, uint32_t B,
                                                  uint32_t D, uint32_t deg, uint32_t C,
                                                  float *__restrict__ outputs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * C) return;
    const uint32_t b = t / C;
    const uint32_t c = t - b * C;
    const float *x = inputs + (size_t)b * D;
    if (c < D) {
        outputs[t] = x[c];
        return;
    }
    const uint32_t col = c / D - 1;
    const uint32_t d = c % D;
    const float phase = (float)(col & 1u) * kHalfPi;
    outputs[t] = sinf(scalbnf(x[d], (int)(col >> 1)) + phase);
}

// freqencoder.cu:63-94: chain rule from the saved outputs (sin <-> cos).
__global__ __launch_bounds__(256) void k_freq_bwd(const float *__restrict__ grad,
                                                  const float *__restrict__ outputs, uint32_t B,
                                                  uint32_t D, uint32_t deg, uint32_t C,
                                                  float *__restrict__ grad_inputs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * D) return;
    const uint32_t b = t / D;
    const uint32_t d = t - b * D;
    const float *g = grad + (size_t)b * C;
    const float *o = outputs + (size_t)b * C;
    float r = g[d];
    for (uint32_t f = 0; f < deg; ++f) {
        const uint32_t s = D + 2 * f * D + d;  // sin column; cos column is s + D
        // nvcc contraction: a*b - c*d -> fma(a, b, -(c*d)); r += k*x -> fma(k, x, r)
        const float inner = fmaf(g[s], o[s + D], -(g[s + D] * o[s]));
        r = fmaf(scalbnf(1.0f, (int)f), inner, r);
    }
    grad_inputs[t] = r;
}

}  // namespace fe
}  // namespace dfhip

using namespace dfhip;
using namespace dfhip::fe;

extern "C" int dfhip_freq_encode_forward(const float *inputs, uint32_t B, uint32_t D,
                                         uint32_t deg, uint32_t C, float *outputs,
                                         dfhip_stream_t stream) {
    if (D == 0 || C != D + 2 * D * deg) {
        set_error("freq_encode_forward: C (%u) must equal D + 2*D*deg (D=%u deg=%u)", C, D, deg);
        return DFHIP_EINVAL;
    }
    if (B == 0) return DFHIP_OK;
    k_freq_fwd<<<ceil_div(B * C, 256u), 256, 0, as_stream(stream)>>>(inputs, B, D, deg, C, outputs);
    return check_launch("freq_encode_forward");
}

extern "C" int dfhip_freq_encode_backward(const float *grad, const float *outputs, uint32_t B,
                                          uint32_t D, uint32_t deg, uint32_t C,
                                          float *grad_inputs, dfhip_stream_t stream) {
    if (D == 0 || C != D + 2 * D * deg) {
        set_error("freq_encode_backward: C (%u) must equal D + 2*D*deg (D=%u deg=%u)", C, D, deg);
        return DFHIP_EINVAL;
    }
    if (B == 0) return DFHIP_OK;
    k_freq_bwd<<<ceil_div(B * D, 256u), 256, 0, as_stream(stream)>>>(grad, outputs, B, D, deg, C,
                                                                    grad_inputs);
    return check_launch("freq_encode_backward");
}
