// D1-D4 — argmax decoder, affine back-transform and PCK.
//
// Replaces get_preds / final_preds / transform_preds (utils/udaap/evaluation.py:13-30,215-238;
// utils/udaap/transforms.py:119-168) and EvaluationUtils.acc_pck (utils/evaluation.py:91-139),
// which the reference runs on the host after a D2H copy of every heatmap, with
// per-point Python loops.
//
// decode: one wave per (sample, keypoint) map.  Each lane scans a strided
// slice keeping the FIRST maximal index (strict >), then a wave reduction
// keeps the larger value and, on ties, the smaller index — torch.max's
// documented first-index rule.  NaN ranks above every number, as in torch.
// The 1-based (col, row) is zeroed where the max is not > 0, then mapped
// through the host-computed float64 inverse transform (same entries as the
// reference: float32 arithmetic for h = 200*scale, np.linalg.inv in f64) with
// un-fused f64 multiply/add in np.dot's order, truncated toward zero, + 1.
#include "common.h"

namespace {

__device__ __forceinline__ bool beats(float v, int i, float bv, int bi) {
    const bool vn = isnan(v), bn = isnan(bv);
    if (vn != bn) return vn;
    if (vn && bn) return i < bi;
    return v > bv || (v == bv && i < bi);
}

__global__ void __launch_bounds__(256) argmax_kernel(const float* __restrict__ hm, int maps, int H, int W,
                                                    const double* __restrict__ tinv, int K,
                                                    float* __restrict__ raw, float* __restrict__ preds,
                                                    float* __restrict__ scores) {
    const int lane = threadIdx.x & 63;
    const int map = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (map >= maps) return;
    const int HW = H * W;
    const float* m = hm + (int64_t)map * HW;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = lane; i < HW; i += 64) {
        const float v = m[i];
        if (beats(v, i, bv, bi)) {
            bv = v;
            bi = i;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (beats(ov, oi, bv, bi)) {
            bv = ov;
            bi = oi;
        }
    }
    if (lane != 0) return;
    const float on = bv > 0.f ? 1.f : 0.f;
    const float px = (float)(bi % W + 1) * on;   // utils/udaap/evaluation.py:25,28-29
    const float py = (float)(bi / W + 1) * on;   // :26
    if (raw) {
        raw[map * 2 + 0] = px;
        raw[map * 2 + 1] = py;
    }
    if (scores) scores[map] = bv;
    if (preds) {
        const double* t = tinv + (int64_t)(map / K) * 6;
        const double vx = (double)px - 1.0, vy = (double)py - 1.0;  // transforms.py:156
        const double rx = __dadd_rn(__dadd_rn(__dmul_rn(t[0], vx), __dmul_rn(t[1], vy)), t[2]);
        const double ry = __dadd_rn(__dadd_rn(__dmul_rn(t[3], vx), __dmul_rn(t[4], vy)), t[5]);
        preds[map * 2 + 0] = (float)((long long)rx + 1);  // astype(int) + 1 (:158)
        preds[map * 2 + 1] = (float)((long long)ry + 1);
    }
}

// PCK (utils/evaluation.py:91-139).  One workgroup; thread per keypoint.
__global__ void __launch_bounds__(256) pck_kernel(const float* __restrict__ preds, const float* __restrict__ gts,
                                                 int N, int K, int ref0, int ref1, float thr,
                                                 float* __restrict__ errs, float* __restrict__ accs,
                                                 int* __restrict__ hits, int* __restrict__ valid) {
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        float esum = 0.f;
        int nh = 0, nv = 0;
        for (int b = 0; b < N; ++b) {
            const float* g = gts + ((int64_t)b * K) * 3;
            const float nx = g[ref0 * 3] - g[ref1 * 3], ny = g[ref0 * 3 + 1] - g[ref1 * 3 + 1];
            const float norm = sqrtf(nx * nx + ny * ny);          // torch.dist (:121)
            const float gx = g[k * 3], gy = g[k * 3 + 1];
            float d = -1.f;
            if (gx > 1.f && gy > 1.f) {                          // :123
                const float dx = preds[((int64_t)b * K + k) * 2] - gx;
                const float dy = preds[((int64_t)b * K + k) * 2 + 1] - gy;
                d = sqrtf(dx * dx + dy * dy);
                const float dr = d / norm;
                nv += 1;
                nh += dr < thr;                                   // _acc_counting (:134-139)
            }
            esum += d;                                           // -1 sentinels included (:99-101)
        }
        errs[k] = esum / (float)N;
        accs[k] = nv > 0 ? (float)((double)nh / (double)nv) : -1.f;
        if (hits) hits[k] = nh;
        if (valid) valid[k] = nv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float es = 0.f, as = 0.f;
        int an = 0;
        for (int k = 0; k < K; ++k) es += errs[k];
        errs[K] = es / (float)K;                                 // :102-104
        for (int k = 0; k < K; ++k)
            if (accs[k] >= 0.f) {
                as += accs[k];
                an += 1;
            }
        accs[K] = an != 0 ? as / (float)an : 0.f;                // :110-114
    }
}

}  // namespace

// hm [N,K,H,W]; tinv [N,6] f64 (rows 0-1 of the inverse of get_transform) or
// null; raw/preds [N,K,2] f32 (nullable), scores [N,K] (nullable).
UBPL_API int ubpl_decode_heatmaps(const float* hm, int N, int K, int H, int W, const double* tinv, float* raw,
                                  float* preds, float* scores, void* stream) {
    const int maps = N * K;
    if (maps == 0) return 0;
    hipLaunchKernelGGL(argmax_kernel, dim3(ubpl::cdiv(maps, 4)), dim3(256), 0, (hipStream_t)stream, hm, maps, H, W,
                       tinv, K, raw, preds, scores);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// preds [N,K,2], gts [N,K,3]; errs/accs [K+1]; hits/valid [K] int32 (nullable).
UBPL_API int ubpl_pck(const float* preds, const float* gts, int N, int K, int ref0, int ref1, float thr, float* errs,
                      float* accs, int* hits, int* valid, void* stream) {
    hipLaunchKernelGGL(pck_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, preds, gts, N, K, ref0, ref1, thr,
                       errs, accs, hits, valid);
    UBPL_LAUNCH_CHECK();
    return 0;
}
