// Real spherical-harmonics encoding (degree 1..8) for gfx950.
//
// Behavioural spec: reference shencoder/src/shencoder.cu:27-382 (same output
// polynomials, same [B, D, C^2] dy_dx layout, same accumulate-into backward).
// Instead of 64 unrolled sympy expressions, each band is evaluated in factored
// form  Y_l^m = A_m(x, y) * q_l^|m|(z)  with A_m = Re / Im of (x + i y)^|m| and
// q a Horner polynomial from the generated table sh_table.h
// (tools/gen_sh_table.py).  Results agree with the reference's expressions to
// float rounding (different evaluation order).
#include "common.h"
#include "sh_table.h"

namespace dfhip {
namespace sh {

template <typename scalar_t> struct MathT { typedef float type; };
template <> struct MathT<double> { typedef double type; };

template <typename T>
__device__ __forceinline__ void q_eval(int row, int deg, T z, T &q, T &dq) {
    // Horner for q and q' simultaneously
    q = (T)kShQ[row][deg];
    dq = (T)0;
    for (int k = deg - 1; k >= 0; --k) {
        dq = dq * z + q;
        q = q * z + (T)kShQ[row][k];
    }
}

template <typename scalar_t>
__global__ __launch_bounds__(256) void k_sh_fwd(const scalar_t *__restrict__ inputs,
                                                scalar_t *__restrict__ outputs, uint32_t B,
                                                uint32_t D, uint32_t C,
                                                scalar_t *__restrict__ dy_dx) {
    typedef typename MathT<scalar_t>::type T;
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint32_t C2 = C * C;
    const T x = (T)inputs[(size_t)b * D], y = (T)inputs[(size_t)b * D + 1],
            z = (T)inputs[(size_t)b * D + 2];
    // powers of (x + i y)
    T cr[DFHIP_SH_LMAX], ci[DFHIP_SH_LMAX];
    cr[0] = (T)1; ci[0] = (T)0;
#pragma unroll
    for (int m = 1; m < DFHIP_SH_LMAX; ++m) {
        cr[m] = cr[m - 1] * x - ci[m - 1] * y;
        ci[m] = cr[m - 1] * y + ci[m - 1] * x;
    }
    scalar_t *out = outputs + (size_t)b * C2;
    scalar_t *jx = dy_dx ? dy_dx + (size_t)b * D * C2 : nullptr;
    scalar_t *jy = jx ? jx + C2 : nullptr;
    scalar_t *jz = jy ? jy + C2 : nullptr;
    for (int l = 0; l < (int)C; ++l) {
        const int center = l * l + l;
        for (int m = 0; m <= l; ++m) {
            T q, dq;
            q_eval<T>(l * (l + 1) / 2 + m, l - m, z, q, dq);
            if (m == 0) {
                out[center] = (scalar_t)q;
                if (jx) {
                    jx[center] = (scalar_t)0;
                    jy[center] = (scalar_t)0;
                    jz[center] = (scalar_t)dq;
                }
                continue;
            }
            out[center + m] = (scalar_t)(cr[m] * q);
            out[center - m] = (scalar_t)(ci[m] * q);
            if (jx) {
                const T mm = (T)m;
                jx[center + m] = (scalar_t)(mm * cr[m - 1] * q);
                jy[center + m] = (scalar_t)(-mm * ci[m - 1] * q);
                jz[center + m] = (scalar_t)(cr[m] * dq);
                jx[center - m] = (scalar_t)(mm * ci[m - 1] * q);
                jy[center - m] = (scalar_t)(mm * cr[m - 1] * q);
                jz[center - m] = (scalar_t)(ci[m] * dq);
            }
        }
    }
}

// shencoder.cu:358-382: grad_inputs[b, d] += sum_k grad[b, k] * dy_dx[b, d, k]
template <typename scalar_t>
__global__ __launch_bounds__(256) void k_sh_bwd(const scalar_t *__restrict__ grad,
                                                uint32_t B, uint32_t D, uint32_t C,
                                                const scalar_t *__restrict__ dy_dx,
                                                scalar_t *__restrict__ grad_inputs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = t / D;
    if (b >= B) return;
    const uint32_t d = t - b * D;
    const uint32_t C2 = C * C;
    const scalar_t *g = grad + (size_t)b * C2;
    const scalar_t *j = dy_dx + (size_t)b * D * C2 + (size_t)d * C2;
    scalar_t r = grad_inputs[t];
    for (uint32_t k = 0; k < C2; ++k) {
        if constexpr (sizeof(scalar_t) == 2) {
            const half_t p = (half_t)f32_rounded((float)g[k] * (float)j[k]);
            r = (half_t)((float)r + (float)p);
        } else {
            r = fma(g[k], j[k], r);
        }
    }
    grad_inputs[t] = r;
}

static bool check_sh(const char *what, uint32_t D, uint32_t C) {
    if (D != 3) {
        set_error("%s: SH encoder only supports input dim == 3 (got %u)", what, D);
        return false;
    }
    if (C < 1 || C > 8) {
        set_error("%s: SH encoder only supports degree in [1, 8] (got %u)", what, C);
        return false;
    }
    return true;
}

}  // namespace sh
}  // namespace dfhip

using namespace dfhip;
using namespace dfhip::sh;

extern "C" int dfhip_sh_encode_forward(int dtype, const void *inputs, void *outputs, uint32_t B,
                                       uint32_t D, uint32_t C, void *dy_dx,
                                       dfhip_stream_t stream) {
    if (!check_sh("sh_encode_forward", D, C)) return DFHIP_EINVAL;
    if (B == 0) return DFHIP_OK;
    DFHIP_DISPATCH(dtype, "sh_encode_forward",
        k_sh_fwd<scalar_t><<<ceil_div(B, 256u), 256, 0, as_stream(stream)>>>(
            (const scalar_t *)inputs, (scalar_t *)outputs, B, D, C, (scalar_t *)dy_dx));
    return check_launch("sh_encode_forward");
}

extern "C" int dfhip_sh_encode_backward(int dtype, const void *grad, const void *inputs,
                                        uint32_t B, uint32_t D, uint32_t C, const void *dy_dx,
                                        void *grad_inputs, dfhip_stream_t stream) {
    (void)inputs;
    if (!check_sh("sh_encode_backward", D, C)) return DFHIP_EINVAL;
    if (B == 0) return DFHIP_OK;
    DFHIP_DISPATCH(dtype, "sh_encode_backward",
        k_sh_bwd<scalar_t><<<ceil_div(B * D, 256u), 256, 0, as_stream(stream)>>>(
            (const scalar_t *)grad, B, D, C, (const scalar_t *)dy_dx, (scalar_t *)grad_inputs));
    return check_launch("sh_encode_backward");
}
