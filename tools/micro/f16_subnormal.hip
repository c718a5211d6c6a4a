// Micro-probe: f32 -> f16 conversion of values in the f16 subnormal range,
// and v_mfma_f32_16x16x32_f16 with f16-subnormal B operands, against exact
// host arithmetic.  Prints mismatch counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <cstring>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_cvt(const float *in, _Float16 *out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (_Float16)in[i];
}

// one 16x16x32 product: A [16][32] row-major, B [32][16] (k-major), D [16][16]
__global__ void k_mfma(const _Float16 *A, const _Float16 *B, float *D) {
    int l = threadIdx.x, c = l & 15, h = l >> 4;
    half8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = A[c * 32 + 8 * h + j];
        b[j] = B[(8 * h + j) * 16 + c];
    }
    f4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, f4{0, 0, 0, 0}, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[(4 * h + r) * 16 + c] = d[r];
}

static float h2f(_Float16 v) { return (float)v; }

int main() {
    // conversions: values k * 2^-26 for k = 0 .. 2^16 (covers subnormal f16 range and ties)
    const int n = 1 << 17;
    std::vector<float> in(n);
    for (int i = 0; i < n; ++i) in[i] = (float)i * ldexpf(1.0f, -27) * ((i & 1) ? -1.0f : 1.0f);
    float *din; _Float16 *dout;
    hipMalloc(&din, n * 4); hipMalloc(&dout, n * 2);
    hipMemcpy(din, in.data(), n * 4, hipMemcpyHostToDevice);
    k_cvt<<<n / 256, 256>>>(din, dout, n);
    std::vector<_Float16> out(n);
    hipMemcpy(out.data(), dout, n * 2, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        _Float16 want = (_Float16)in[i];  // host conversion (RNE)
        uint16_t a, b; memcpy(&a, &out[i], 2); memcpy(&b, &want, 2);
        if (a != b && bad++ < 8) printf("cvt %.9g: gpu %.9g host %.9g\n", in[i], h2f(out[i]), h2f(want));
    }
    printf("cvt mismatches: %d of %d\n", bad, n);

    // MFMA with subnormal B operands, many random trials
    srand(1);
    _Float16 *dA, *dB; float *dD;
    hipMalloc(&dA, 16 * 32 * 2); hipMalloc(&dB, 32 * 16 * 2); hipMalloc(&dD, 256 * 4);
    long total[2] = {0, 0}, mism[2] = {0, 0}; double worst[2] = {0, 0};
    for (int trial = 0; trial < 2000; ++trial) {
        std::vector<_Float16> A(512), B(512);
        for (int i = 0; i < 512; ++i) A[i] = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.2f);
        for (int i = 0; i < 512; ++i) {
            int k = rand() % 2048 - 1024;  // subnormal: k * 2^-24
            B[i] = (trial & 1) ? (_Float16)ldexpf((float)k, -24) : (_Float16)ldexpf((float)k, -14);
        }
        hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
        k_mfma<<<1, 64>>>(dA, dB, dD);
        std::vector<float> D(256);
        hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                double e = 0, s = 0;
                for (int k = 0; k < 32; ++k) {
                    double t = (double)h2f(A[i * 32 + k]) * (double)h2f(B[k * 16 + j]);
                    e += t; s += fabs(t);
                }
                float ef = (float)e;
                const int kind = trial & 1;
                ++total[kind];
                if (ef != D[i * 16 + j]) {
                    ++mism[kind];
                    double rel = fabs(D[i * 16 + j] - e) / (s > 0 ? s : 1);
                    if (rel > worst[kind]) worst[kind] = rel;
                }
            }
    }
    for (int kind = 0; kind < 2; ++kind)
        printf("%s B: mfma != round(exact) %ld of %ld, worst |err|/sum|t| %.3e (= %.1f u)\n",
               kind ? "subnormal" : "normal", mism[kind], total[kind], worst[kind],
               worst[kind] / ldexp(1.0, -24));
    // split by kind
    return 0;
}
