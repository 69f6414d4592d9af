// Shared helpers for the UBPL hot-path kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ubpl_hip.h"

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

// MFMA accumulators (32x32 C/D map: lane l holds pixel l&31 of rows (r&3) +
// 8(r>>2) + 4(l>>5)) seeded with bias (+ residual) before the K loop, so the
// epilogue only stores; an element is read and written by the same lane, so
// res may alias the output.  The cases are wave-uniform branches; inside one,
// loads are unconditional (clamped rows): a load under a per-lane condition
// becomes a branch + vmcnt(0) per element.  No residual: nothing is read.
// GROUPED: a scheduling barrier after each fragment's 16 loads (their
// addresses die once issued) — keeps the widest tiles (conv_psa 128 x 256)
// within 256 VGPRs without scratch.
// sc: the scale of the accumulators (a power of two: the 2xfp16 path's operand
// scales, see split2; 1 elsewhere) — the seed is (bias + res) * sc, exactly.
template <int TM, int TN, bool GROUPED = false, typename ACC>
__device__ __forceinline__ void seed_acc(ACC (&acc)[TM][TN], const float* bias, const float* res,
                                         const int64_t (&obase)[TN], int mrow0, int M, int P, float sc = 1.f) {
    const int h = (threadIdx.x & 63) >> 5;
    if (res != nullptr) {
        const bool hb = bias != nullptr;
        const float* bp = hb ? bias : res;
        // 32-bit offsets from one base per fragment column: with a 64-bit
        // address per element live at once the wide kernels spilled to scratch
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float* rj = res + obase[j];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = min(mrow0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h, M - 1);
                    const float bv = bp[m];
                    acc[i][j][r] = ((hb ? bv : 0.f) + rj[m * P]) * sc;
                }
                if (GROUPED) __builtin_amdgcn_sched_barrier(0);
            }
    } else if (bias != nullptr) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float bv = bias[min(mrow0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h, M - 1)] * sc;
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j][r] = bv;
            }
    } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }
}

// Two floats -> NP packed 16-bit pairs (piece p of a in the low half).
// NP = 3 (6xbf16) and 1 (bf16): the split-bf16 representation v = v0 + v1 (+ v2),
// v_p = bf16(v - v_0 - ... - v_{p-1}) — three bf16 pieces carry an f32 exactly.
// NP = 2 (2xfp16): two IEEE fp16 pieces, v = f16(v) + f16(v - f16(v)) to <= 2^-22
// relative (two 11-bit significands), the piece products hi.hi + hi.lo + lo.hi exact
// in f32: operands within a few f32 ulps with 3 MFMA products instead of 6.  fp16's exponent range is narrow
// (normal from 2^-14, max 65504), so the callers pass values pre-scaled by a power
// of two that puts them there (conv_split.hip: FP16_ACT_SCALE, fp16_wscale) and
// undo the scale exactly on the accumulators.
constexpr float FP16_ACT_SCALE = 32.f;   // activations: |v| up to 2047 without overflow, full
                                         // precision from |v| >= 2^-7 (below: absolute error <= 2^-30)
// weights of a GEMM with contraction length K (Cin * taps): 2^(9 + ceil(log2 sqrt K)), so
// the default init's bound 1/sqrt(K) lands at 2^9 .. 2^10 (64x headroom to the fp16 max)
__host__ __device__ __forceinline__ float fp16_wscale(int K) {
    int e = 0;
    while ((1 << (2 * e)) < K) ++e;            // 2^e >= sqrt(K)
    return (float)(1 << (9 + e));
}
template <int NP>
__device__ __forceinline__ void split2(float a, float b, uint32_t (&o)[NP]) {
    if constexpr (NP == 2) {
        typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
        const _Float16 ha = (_Float16)a, hb = (_Float16)b;
        const f16x2_t v0 = {ha, hb};
        const f16x2_t v1 = {(_Float16)(a - (float)ha), (_Float16)(b - (float)hb)};
        o[0] = __builtin_bit_cast(uint32_t, v0);
        o[1] = __builtin_bit_cast(uint32_t, v1);
        return;
    }
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const __bf16 ha = (__bf16)a, hb = (__bf16)b;
        const bf16x2_t v = {ha, hb};
        o[p] = __builtin_bit_cast(uint32_t, v);
        if (p + 1 < NP) {
            a -= (float)ha;
            b -= (float)hb;
        }
    }
}

// 16 channel values of one pixel -> the NP bf16 planes of a PSA image row
// (conv_split.hip split_act_kernel layout): 32 contiguous bytes per plane.
template <int NP>
__device__ __forceinline__ void store_psa_row(const float (&v)[16], uint16_t* d, int64_t plane, float sc = 1.f) {
    uint32_t pk[NP][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t o[NP];
        split2<NP>(v[2 * i] * sc, v[2 * i + 1] * sc, o);
#pragma unroll
        for (int p = 0; p < NP; ++p) pk[p][i] = o[p];
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        *reinterpret_cast<uint4*>(d + p * plane) = make_uint4(pk[p][0], pk[p][1], pk[p][2], pk[p][3]);
        *reinterpret_cast<uint4*>(d + p * plane + 8) = make_uint4(pk[p][4], pk[p][5], pk[p][6], pk[p][7]);
    }
}

// Sum over the 32 lanes of each wave half by DPP row shifts (Hillis-Steele
// within a 16-lane row, then row_bcast:15 into rows 1 and 3): the total of
// lanes 0-31 lands in lane 31, of lanes 32-63 in lane 63.
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF,
                                                                     true));
}
// Sum over each 16-lane row (lane 15 of the row holds it).
__device__ __forceinline__ float row_sum16(float v) {
    v = dpp_add<0x111>(v);   // row_shr:1
    v = dpp_add<0x112>(v);   // row_shr:2
    v = dpp_add<0x114>(v);   // row_shr:4
    return dpp_add<0x118>(v);   // row_shr:8
}
__device__ __forceinline__ float half_sum_dpp(float v) {
    v = dpp_add<0x111>(v);   // row_shr:1
    v = dpp_add<0x112>(v);   // row_shr:2
    v = dpp_add<0x114>(v);   // row_shr:4
    v = dpp_add<0x118>(v);   // row_shr:8
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF,
                                                                     false));   // row_bcast:15
}

// BatchNorm partial statistics of a conv output tile, straight from the MFMA
// accumulators (C/D map: lane l holds pixel n0 + l&31 of rows (r&3) + 8(r>>2) +
// 4(l>>5)): per channel m and per 64-pixel slice q = n/64 of the flat (b, p)
// range, part[(m*np + q)*2 + {0,1}] = (S, M2): S = sum y, M2 = sum (y - S/n)^2
// over the slice's n valid pixels (Chan's parallel form: no E[y^2] - E[y]^2
// cancellation; the finalize combines slices in f64).  A wave covers TN/2
// slices (2 fragments of 32 pixels each).
template <int TM, int TN, typename ACC>
__device__ __forceinline__ void tile_bn_partials(const ACC (&acc)[TM][TN], const bool (&nok)[TN], int mrow0, int M,
                                                 int64_t nwave0, int64_t N, float* part) {
    static_assert(TN % 2 == 0, "a wave covers whole 64-pixel slices (2 fragments of 32 each)");
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int64_t np = (N + 63) / 64;
#pragma unroll
    for (int sp = 0; sp < TN / 2; ++sp) {
        const int64_t ns0 = nwave0 + 64 * sp;
        if (ns0 >= N) break;
        const int64_t q = ns0 / 64;
        const float inv_n = 1.f / (float)(N - ns0 < 64 ? N - ns0 : 64);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mrow0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float y0 = nok[2 * sp] ? acc[i][2 * sp][r] : 0.f;
                const float y1 = nok[2 * sp + 1] ? acc[i][2 * sp + 1][r] : 0.f;
                const float s = half_sum_dpp(y0 + y1);
                const float s_lo =
                    __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s), 31));
                const float s_hi =
                    __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s), 63));
                const float mu = (h ? s_hi : s_lo) * inv_n;
                const float d0 = nok[2 * sp] ? y0 - mu : 0.f;
                const float d1 = nok[2 * sp + 1] ? y1 - mu : 0.f;
                const float m2 = half_sum_dpp(fmaf(d0, d0, d1 * d1));
                if ((lane & 31) == 31 && m < M) {
                    part[(m * np + q) * 2] = s;
                    part[(m * np + q) * 2 + 1] = m2;
                }
            }
    }
}

// BatchNorm BACKWARD partials of a data-gradient tile (the conv output is dz
// of the BN whose input is x): per channel m and 64-pixel slice q,
// (S1, S2) = (sum g, sum g*(x - mean)), g = dz under the recomputed ReLU mask
// — bn.hip bn_bwd_partials_kernel's layout and formula, from the accumulators
// (no dz re-read; x is read at the tile's own addresses).
struct BnBwdEpi {
    const float* x;      // BN input [B][M][P] (nullptr: off)
    const float* coef;   // scale | shift | mean, M floats each
    int relu;
    float* part;         // [M][ceil(N/64)][2]
};

template <int TM, int TN, typename ACC>
__device__ __forceinline__ void tile_bn_bwd_partials(const ACC (&acc)[TM][TN], const bool (&nok)[TN],
                                                     const int64_t (&obase)[TN], int mrow0, int M, int P,
                                                     int64_t nwave0, int64_t N, const BnBwdEpi& e) {
    static_assert(TN % 2 == 0, "a wave covers whole 64-pixel slices (2 fragments of 32 each)");
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int64_t np = (N + 63) / 64;
#pragma unroll
    for (int sp = 0; sp < TN / 2; ++sp) {
        const int64_t ns0 = nwave0 + 64 * sp;
        if (ns0 >= N) break;
        const int64_t q = ns0 / 64;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mrow0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int mc = m < M ? m : M - 1;
                const float sc = e.coef[mc], sh = e.coef[M + mc], mu = e.coef[2 * M + mc];
                const float x0 = e.x[obase[2 * sp] + (int64_t)mc * P];
                const float x1 = e.x[obase[2 * sp + 1] + (int64_t)mc * P];
                float g0 = nok[2 * sp] ? acc[i][2 * sp][r] : 0.f;
                float g1 = nok[2 * sp + 1] ? acc[i][2 * sp + 1][r] : 0.f;
                if (e.relu && !(fmaf(x0, sc, sh) > 0.f)) g0 = 0.f;
                if (e.relu && !(fmaf(x1, sc, sh) > 0.f)) g1 = 0.f;
                const float s1 = half_sum_dpp(g0 + g1);
                const float s2 = half_sum_dpp(fmaf(g0, x0 - mu, g1 * (x1 - mu)));
                if ((lane & 31) == 31 && m < M) {
                    e.part[((int64_t)m * np + q) * 2] = s1;
                    e.part[((int64_t)m * np + q) * 2 + 1] = s2;
                }
            }
    }
}

}  // namespace ubpl
