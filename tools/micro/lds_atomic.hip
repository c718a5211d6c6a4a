// Microbenchmark: LDS float atomic throughput on gfx950 (random rows, same row,
// versus int atomics and plain read+write).  Prints lane-ops per CU-cycle.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE>
__global__ __launch_bounds__(1024) void k(float *out, int iters, uint32_t mask, uint32_t seed) {
    extern __shared__ float lds[];
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = 0.f;
    __syncthreads();
    uint32_t h = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
    float v = 1.0f + threadIdx.x * 1e-3f;
    for (int it = 0; it < iters; ++it) {
        h = h * 1664525u + 1013904223u;
        uint32_t a = (h >> 8) & mask;
        if (MODE == 0) atomicAdd(&lds[a], v);                        // ds_add_f32
        if (MODE == 1) atomicAdd((uint32_t *)&lds[a], 1u);            // ds_add_u32
        if (MODE == 2) { lds[a] += v; }                               // racy RMW
        if (MODE == 3) atomicAdd(&lds[(threadIdx.x >> 6) & 7], v);    // 64 lanes same row
        if (MODE == 4) atomicAdd(&lds[a & ~63u | (threadIdx.x & 63)], v); // distinct rows, conflict-free
        if (MODE == 5) atomicAdd((unsigned long long *)&lds[(a & ~1u)], 1ull);   // ds_add_u64
        if (MODE == 6) atomicAdd((double *)&lds[(a & ~1u)], (double)v);        // ds_add_f64
        if (MODE == 7) {                                                        // ds_pk_add_f16
            typedef _Float16 h2 __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(3))) h2 lh2;
            h2 p; p.x = (_Float16)v; p.y = (_Float16)v;
            __builtin_amdgcn_ds_atomic_fadd_v2f16((lh2 *)((__attribute__((address_space(3))) char *)lds + 4 * a), p);
        }
        if (MODE == 8) atomicMax((int *)&lds[a], (int)h);                       // ds_max_i32
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = lds[blockIdx.x & 1023];
}

int main() {
    float *out;
    hipMalloc(&out, 4096 * 4);
    int dev = 0, cus = 0, clk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    const int iters = 4096;
    const char *names[] = {"ds_add_f32 random", "ds_add_u32 random", "racy ld+st random",
                           "ds_add_f32 same row/wave", "ds_add_f32 lane-distinct", "ds_add_u64 random",
                           "ds_add_f64 random", "ds_pk_add_f16 random", "ds_max_i32 random"};
    for (int mode = 0; mode < 9; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            dim3 g(cus), b(1024);
            switch (mode) {
            case 0: k<0><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            case 1: k<1><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            case 2: k<2><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            case 3: k<3><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            case 4: k<4><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            case 5: k<5><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            case 6: k<6><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            case 7: k<7><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            case 8: k<8><<<g, b, 65536>>>(out, iters, 16383, 7); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 1) {
                double lane_ops = (double)cus * 1024 * iters;
                double cycles = ms * 1e-3 * clk * 1e3;  // clk in kHz
                printf("%-28s %8.3f ms  %6.2f lane-ops/CU/cycle (clk %d MHz)\n", names[mode], ms,
                       lane_ops / cus / cycles, clk / 1000);
            }
        }
    }
    return 0;
}
