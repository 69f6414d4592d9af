// Shared helpers for the UBPL hot-path kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define UBPL_API extern "C" __attribute__((visibility("default")))

#define UBPL_LAUNCH_CHECK()                         \
    do {                                            \
        hipError_t e__ = hipGetLastError();         \
        if (e__ != hipSuccess) return (int)e__;     \
    } while (0)

namespace ubpl {

constexpr int WAVE = 64;

// Linear block id L of G -> logical tile id such that consecutive logical ids
// run on the same XCD (blocks are dispatched round-robin over the 8 XCDs, each
// with its own L2).  Affinity only: correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int L, int G) {
    constexpr int X = 8;
    const int q = G / X, r = G % X, x = L % X, s = L / X;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + s;
}

// Channel group of the conv weight K order: k = (ci/G)*G*T + tap*G + ci%G
// (G = 16 when it divides the input channels, else all of them).
__host__ __device__ __forceinline__ int conv_kgroup(int cin) { return (cin % 16 == 0) ? 16 : cin; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024); result valid in all threads.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* smem /* >= 16 */) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) smem[wid] = v;
    __syncthreads();
    T r = 0;
    for (int i = 0; i < nw; ++i) r += smem[i];
    return r;
}

__device__ __forceinline__ float block_max(float v, float* smem) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) smem[wid] = v;
    __syncthreads();
    float r = smem[0];
    for (int i = 1; i < nw; ++i) r = fmaxf(r, smem[i]);
    return r;
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace ubpl
