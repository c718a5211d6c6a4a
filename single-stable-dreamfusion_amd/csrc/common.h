// Shared device/host helpers for the gfx950 NeRF hot-path kernels.
// Written for CDNA4 directly: wave64, no CUDA shims, no dual-platform ifdefs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#include "../../include/dfhip.h"

namespace dfhip {

// ---------------------------------------------------------------- errors
// Thread-local message of the last failing call (see dfhip_last_error()).
void set_error(const char *fmt, ...);

// Report the launch status of the kernels issued by one entry point.
inline int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return DFHIP_ELAUNCH;
    }
    return DFHIP_OK;
}

// ---------------------------------------------------------------- launch setup
// The current device and its CU count (queried per call).
int current_device();
uint32_t device_cus();
// hipFuncSetAttribute(MaxDynamicSharedMemorySize, bytes) once per (kernel,
// device), thread-safe.
void ensure_dynamic_lds(const void *kernel, int bytes);
// Workgroups of `threads` threads of `kernel` co-resident on the current
// device (occupancy query once per (kernel, device, threads); fallback_per_cu
// per CU if the query fails).
uint32_t resident_blocks(const void *kernel, int threads, int fallback_per_cu);

inline hipStream_t as_stream(dfhip_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// GridEncoder forward on the fused field's tile gather (csrc/fieldmlp.hip) for
// D = 3, C = 2, L = 16 with an f16 table and no dy_dx ([B, 32] output, rows
// [*m_dev, B) zero, raw positions when bound > 0); false when L does not fit.
bool grid_forward_tiles_f16(const float *inputs, float bound, const void *table,
                            const int32_t *offsets, uint32_t L, float S, uint32_t H,
                            uint32_t gridtype, int align_corners, void *outputs, uint32_t B,
                            const int32_t *m_dev, hipStream_t s);

template <typename T>
__host__ __device__ inline T ceil_div(T a, T b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- storage types
// f16 storage uses the compiler's native _Float16 (IEEE binary16, RNE casts),
// bit-identical to torch.half.
typedef _Float16 half_t;
typedef __bf16 bf16_t;  // the C5 bf16 option (DFHIP_BF16)

template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v) { return (T)v; }

// Value barrier: stops the backend from fusing an f32 product with the f16
// conversion that follows it (fptrunc(fmul) -> v_fma_mixlo_f16 rounds ONCE,
// the reference's c10::Half arithmetic rounds twice: to f32, then to f16).
__device__ __forceinline__ float f32_rounded(float x) {
    asm("" : "+v"(x));
    return x;
}

// Dispatch a templated launcher over the storage dtype (the reference's
// AT_DISPATCH_FLOATING_TYPES_AND_HALF).
#define DFHIP_DISPATCH(dtype, NAME, ...)                                        \
    switch (dtype) {                                                            \
    case DFHIP_F32: { typedef float scalar_t; __VA_ARGS__; break; }             \
    case DFHIP_F16: { typedef dfhip::half_t scalar_t; __VA_ARGS__; break; }     \
    case DFHIP_F64: { typedef double scalar_t; __VA_ARGS__; break; }            \
    default: dfhip::set_error("%s: unsupported dtype %d", NAME, (int)(dtype));  \
             return DFHIP_EDTYPE;                                               \
    }

// ---------------------------------------------------------------- wave64 helpers
__device__ __forceinline__ int wave_reduce_add(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Inclusive scan across the 64 lanes of a wave.
__device__ __forceinline__ int wave_inclusive_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

}  // namespace dfhip
