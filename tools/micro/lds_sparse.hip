// Microbenchmark: cost of an LDS f64 atomic wave instruction against the
// number of active lanes (does a sparse exec mask make ds_add_f64 cheaper?),
// and of conflict-free versus random rows.  Prints CU cycles per wave
// instruction and lane-ops per CU-cycle.  Used to choose the walk's flush
// structure (csrc/gridbin.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(1024) void k(float *out, int iters, int active, uint32_t seed) {
    extern __shared__ double lds[];
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = 0.0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t h = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
    const double v = 1.0 + threadIdx.x * 1e-3;
    const bool on = (int)lane < active;
    for (int it = 0; it < iters; ++it) {
        h = h * 1664525u + 1013904223u;
        uint32_t a = (h >> 8) & 16383u;
        if (MODE == 1) a = ((h >> 8) & (16383u & ~63u)) | lane;  // distinct banks pattern
        if (on) atomicAdd(&lds[a], v);
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (float)lds[blockIdx.x & 1023];
}

// f32 LDS add with the same patterns (ds_add_f32), for comparison
template <int MODE>
__global__ __launch_bounds__(1024) void kf(float *out, int iters, int active, uint32_t seed) {
    extern __shared__ float ldsf[];
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) ldsf[i] = 0.f;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t h = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
    const float v = 1.0f + threadIdx.x * 1e-3f;
    const bool on = (int)lane < active;
    for (int it = 0; it < iters; ++it) {
        h = h * 1664525u + 1013904223u;
        uint32_t a = (h >> 8) & 32767u;
        if (MODE == 1) a = ((h >> 8) & (32767u & ~63u)) | lane;
        if (on) atomicAdd(&ldsf[a], v);
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = ldsf[blockIdx.x & 1023];
}

typedef void (*kfn)(float *, int, int, uint32_t);

static void run(const char *name, kfn f, int active, int cus, int clk, float *out) {
    const int iters = 4096;
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(f, dim3(cus), dim3(1024), 131072, 0, out, iters, active, 7u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    const double cycles = ms * 1e-3 * clk * 1e3;
    const double winstr = 16.0 * iters;  // wave instructions per CU
    printf("%-26s active %2d  %8.3f ms  %6.2f CU-cycles/wave-instr  %6.2f lane-ops/CU/cycle\n",
           name, active, ms, cycles / winstr, winstr * active / cycles);
}

int main() {
    float *out;
    hipMalloc(&out, 4096 * 4);
    int dev = 0, cus = 0, clk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    hipFuncSetAttribute((const void *)k<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    hipFuncSetAttribute((const void *)k<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    hipFuncSetAttribute((const void *)kf<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    hipFuncSetAttribute((const void *)kf<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    const int act[] = {64, 32, 16, 8, 4, 2, 1};
    for (int a : act) run("ds_add_f64 random", k<0>, a, cus, clk, out);
    for (int a : act) run("ds_add_f64 bank-distinct", k<1>, a, cus, clk, out);
    for (int a : act) run("ds_add_f32 random", kf<0>, a, cus, clk, out);
    for (int a : act) run("ds_add_f32 bank-distinct", kf<1>, a, cus, clk, out);
    return 0;
}
