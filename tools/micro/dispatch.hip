// Workgroup dispatch rate on gfx950: near-empty kernels of G workgroups of T
// threads (each wave spins S clocks), timed with HIP events.  Tells whether a
// short-lived-wave kernel (the train march count: 2,048 x 512, ~6 us per
// wave) is bound by how fast workgroups are launched.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_spin(int *out, long long spin) {
    const long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
    if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFF) out[0] = 1;
}

int main() {
    int *d;
    hipMalloc(&d, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int cfg[][2] = {{2048, 512}, {4096, 256}, {16384, 64}, {1024, 1024}, {256, 1024}};
    const long long spins[] = {0, 2000, 13000};
    for (long long sp : spins) {
        for (auto &c : cfg) {
            k_spin<<<c[0], c[1]>>>(d, sp);
            hipDeviceSynchronize();
            hipEventRecord(a);
            for (int r = 0; r < 20; ++r) k_spin<<<c[0], c[1]>>>(d, sp);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            printf("spin %6lld clk  grid %6d x %4d threads: %8.2f us per launch\n", sp, c[0], c[1],
                   ms * 1e3 / 20);
        }
    }
    hipFree(d);
    return 0;
}
