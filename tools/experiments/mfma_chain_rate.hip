// What MFMA rate does conv_psa_kernel's inner structure allow with no memory at
// all?  Per "K step" each wave runs TM x TN tiles, each a chain of 6 dependent
// v_mfma_f32_32x32x16_bf16 (C = the previous result, first from zero) followed by
// the f32 add of the chunk into the accumulator (conv_split.hip mfma_split0 +
// acc += tmp), 256-thread workgroups, 2 per CU (the kernel's occupancy).
//   mode 0: one temporary, tiles in sequence (what hipcc emits for conv_psa)
//   mode 1: two tiles' chains interleaved (two temporaries)
//   mode 2: no chunking — 6 MFMAs straight into the accumulator (upper bound)
// Prints achieved bf16 TFLOP/s vs the 2.5 PF dense peak.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_chain_rate mfma_chain_rate.hip && ./mfma_chain_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define MF(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0)

template <int MODE>
__global__ void __launch_bounds__(256, 2) chain_kernel(float* out, int steps) {
    constexpr int TM = 2, TN = 4;
    floatx16 acc[TM][TN];
    for (int i = 0; i < TM; ++i)
        for (int j = 0; j < TN; ++j)
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    bf16x8 a[TM][3], b[TN][3];
    const float s = (float)(threadIdx.x + 1) * 1e-3f;
    for (int i = 0; i < TM; ++i)
        for (int p = 0; p < 3; ++p)
            for (int e = 0; e < 8; ++e) a[i][p][e] = (__bf16)(s * (e + p + i));
    for (int j = 0; j < TN; ++j)
        for (int p = 0; p < 3; ++p)
            for (int e = 0; e < 8; ++e) b[j][p][e] = (__bf16)(s * (e - p + j));
    const floatx16 zero = {};
    for (int t = 0; t < steps; ++t) {
        if constexpr (MODE == 0) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    floatx16 c = MF(a[i][2], b[j][0], zero);
                    c = MF(a[i][1], b[j][1], c);
                    c = MF(a[i][0], b[j][2], c);
                    c = MF(a[i][1], b[j][0], c);
                    c = MF(a[i][0], b[j][1], c);
                    c = MF(a[i][0], b[j][0], c);
                    acc[i][j] += c;
                }
        } else if constexpr (MODE == 1) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; j += 2) {
                    floatx16 c = MF(a[i][2], b[j][0], zero);
                    floatx16 d = MF(a[i][2], b[j + 1][0], zero);
                    c = MF(a[i][1], b[j][1], c);
                    d = MF(a[i][1], b[j + 1][1], d);
                    c = MF(a[i][0], b[j][2], c);
                    d = MF(a[i][0], b[j + 1][2], d);
                    c = MF(a[i][1], b[j][0], c);
                    d = MF(a[i][1], b[j + 1][0], d);
                    c = MF(a[i][0], b[j][1], c);
                    d = MF(a[i][0], b[j + 1][1], d);
                    c = MF(a[i][0], b[j][0], c);
                    d = MF(a[i][0], b[j + 1][0], d);
                    acc[i][j] += c;
                    acc[i][j + 1] += d;
                }
        } else {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = MF(a[i][2], b[j][0], acc[i][j]);
                    acc[i][j] = MF(a[i][1], b[j][1], acc[i][j]);
                    acc[i][j] = MF(a[i][0], b[j][2], acc[i][j]);
                    acc[i][j] = MF(a[i][1], b[j][0], acc[i][j]);
                    acc[i][j] = MF(a[i][0], b[j][1], acc[i][j]);
                    acc[i][j] = MF(a[i][0], b[j][0], acc[i][j]);
                }
        }
        // keep the operands live and varying (the compiler must not hoist the chains)
        a[0][0][0] = (__bf16)((float)a[0][0][0] + 1e-3f);
    }
    float sum = 0.f;
    for (int i = 0; i < TM; ++i)
        for (int j = 0; j < TN; ++j)
            for (int r = 0; r < 16; ++r) sum += acc[i][j][r];
    out[blockIdx.x * 256 + threadIdx.x] = sum;
}

template <int MODE>
void run(const char* name, float* d, int grid, int steps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(chain_kernel<MODE>, dim3(grid), dim3(256), 0, 0, d, steps);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(chain_kernel<MODE>, dim3(grid), dim3(256), 0, 0, d, steps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 5.0 * grid * 4 /*waves*/ * (double)steps * 48 * 32768;
    printf("%-28s %8.3f ms  %7.1f TF/s bf16  (%.3f of 2.5 PF)\n", name, ms / 5, flops / (ms * 1e-3) / 1e12,
           flops / (ms * 1e-3) / 2.5e15);
}

int main() {
    float* d;
    const int grid = 512, steps = 4000;
    hipMalloc(&d, grid * 256 * sizeof(float));
    run<0>("one temp, tiles in sequence", d, grid, steps);
    run<1>("two chains interleaved", d, grid, steps);
    run<2>("no chunking (direct acc)", d, grid, steps);
    hipFree(d);
    return 0;
}
