// E1 — Mean-Teacher EMA update, plus the fused AdamW step, over FLAT buffers.
//
// The reference walks 454 parameter tensors per model with two in-place ops
// each (utils/parameters.py:4-8) — 908 tiny launches per model per step — and
// torch.optim.AdamW over the same 454 tensors.  Here every model keeps its
// parameters in one contiguous f32 buffer (grad-carrying ones first, the
// never-trained skip_layer parameters last), so each update is ONE streaming
// kernel, 16 B per lane, HBM-bound:
//   EMA   ema = ema*alpha (rounded), then += (1-alpha)*p  — the two in-place
//         ops of the reference, second one fused multiply-add as torch does;
//   AdamW torch.optim.AdamW (decoupled weight decay, bias-corrected moments,
//         amsgrad off) on the live prefix only.
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) ema_kernel(float* __restrict__ ema, const float* __restrict__ p, int64_t n,
                                                 int64_t n4, float alpha, float oma) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float4* e4 = reinterpret_cast<float4*>(ema);
    const float4* p4 = reinterpret_cast<const float4*>(p);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 e = e4[i];
        const float4 q = p4[i];
        e.x = fmaf(q.x, oma, e.x * alpha);
        e.y = fmaf(q.y, oma, e.y * alpha);
        e.z = fmaf(q.z, oma, e.z * alpha);
        e.w = fmaf(q.w, oma, e.w * alpha);
        e4[i] = e;
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        ema[i] = fmaf(p[i], oma, ema[i] * alpha);
}

// AdamW, torch.optim.adamw single-tensor math:
//   p *= 1 - lr*wd; m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g;
//   denom = sqrt(v)/sqrt(bc2) + eps; p += -step_size * m / denom.
__device__ __forceinline__ void adamw_one(float& p, float g, float& m, float& v, float decay, float omb1, float b2,
                                          float omb2, float bc2_sqrt, float eps, float neg_step) {
    p = p * decay;
    m = m + omb1 * (g - m);  // lerp with weight < 0.5
    v = fmaf(omb2 * g, g, v * b2);
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = fmaf(neg_step, m / denom, p);
}

__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   float decay, float omb1, float b2, float omb2,
                                                   float bc2_sqrt, float eps, float neg_step, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 pp = p4[i], mm = m4[i], vv = v4[i];
        const float4 gg = g4[i];
        adamw_one(pp.x, gg.x, mm.x, vv.x, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
        adamw_one(pp.y, gg.y, mm.y, vv.y, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
        adamw_one(pp.z, gg.z, mm.z, vv.z, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
        adamw_one(pp.w, gg.w, mm.w, vv.w, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
        p4[i] = pp;
        m4[i] = mm;
        v4[i] = vv;
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        adamw_one(p[i], g[i], m[i], v[i], decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
}

// Graph-replayable AdamW: the step count lives on the device.  adamw_prep
// increments it and derives (decay, sqrt(bc2), -lr/bc1) exactly as the host
// path does (f64, then f32); adamw_dev_kernel reads them from memory.
__global__ void adamw_prep_kernel(int64_t* __restrict__ step, double lr, double beta1, double beta2,
                                  double weight_decay, float* __restrict__ coef) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int64_t s = ++(*step);
    const double bc1 = 1.0 - pow(beta1, (double)s);
    const double bc2 = 1.0 - pow(beta2, (double)s);
    coef[0] = (float)(1.0 - lr * weight_decay);
    coef[1] = (float)sqrt(bc2);
    coef[2] = (float)(-(lr / bc1));
}

__global__ void __launch_bounds__(256) adamw_dev_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                       const float* __restrict__ coef, float omb1, float b2,
                                                       float omb2, float eps, int64_t n4) {
    const float decay = coef[0], bc2_sqrt = coef[1], neg_step = coef[2];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 pp = p4[i], mm = m4[i], vv = v4[i];
        const float4 gg = g4[i];
        adamw_one(pp.x, gg.x, mm.x, vv.x, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
        adamw_one(pp.y, gg.y, mm.y, vv.y, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
        adamw_one(pp.z, gg.z, mm.z, vv.z, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
        adamw_one(pp.w, gg.w, mm.w, vv.w, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
        p4[i] = pp;
        m4[i] = mm;
        v4[i] = vv;
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        adamw_one(p[i], g[i], m[i], v[i], decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
}

// AdamW on the student's live prefix and the Mean-Teacher EMA of the whole
// buffer in one pass: element i < nlive takes the AdamW step
// and the teacher reads the updated value from registers; nlive <= i < n (the
// never-trained parameters) only the EMA.  Same per-element arithmetic as
// adamw_dev_kernel followed by ema_kernel, so results are bit-identical to the
// two launches, with one read of p (and one launch) fewer.
__global__ void __launch_bounds__(256) adamw_ema_dev_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                           float* __restrict__ m, float* __restrict__ v,
                                                           int64_t nlive4, const float* __restrict__ coef,
                                                           float omb1, float b2, float omb2, float eps,
                                                           float* __restrict__ ema, int64_t n4, float alpha,
                                                           float oma) {
    const float decay = coef[0], bc2_sqrt = coef[1], neg_step = coef[2];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    float4* e4 = reinterpret_cast<float4*>(ema);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 pp = p4[i];
        float4 e = e4[i];
        if (i < nlive4) {
            float4 mm = m4[i], vv = v4[i];
            const float4 gg = g4[i];
            adamw_one(pp.x, gg.x, mm.x, vv.x, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
            adamw_one(pp.y, gg.y, mm.y, vv.y, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
            adamw_one(pp.z, gg.z, mm.z, vv.z, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
            adamw_one(pp.w, gg.w, mm.w, vv.w, decay, omb1, b2, omb2, bc2_sqrt, eps, neg_step);
            p4[i] = pp;
            m4[i] = mm;
            v4[i] = vv;
        }
        e.x = fmaf(pp.x, oma, e.x * alpha);
        e.y = fmaf(pp.y, oma, e.y * alpha);
        e.z = fmaf(pp.z, oma, e.z * alpha);
        e.w = fmaf(pp.w, oma, e.w * alpha);
        e4[i] = e;
    }
}

__global__ void __launch_bounds__(256) scale_kernel(float* __restrict__ x, int64_t n, float s) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= s;
}

// float4 path only when every pointer is 16-B aligned (flat buffers are).
int64_t vec4_count(int64_t n, const void* a, const void* b, const void* c = nullptr, const void* d = nullptr) {
    const uintptr_t m = (uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)d;
    return (m & 15) ? 0 : (n >> 2);
}

int grid_for(int64_t n) {
    int64_t g = (n / 4 + 255) / 256;
    if (g > 2048) g = 2048;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

// ema, p: flat f32 [n] (16-B aligned).  alpha = min(1 - 1/(epo+1), ema_decay).
UBPL_API int ubpl_ema_update(float* ema, const float* p, int64_t n, double alpha, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(ema_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, ema, p, n,
                       vec4_count(n, ema, p), (float)alpha,
                       (float)(1.0 - alpha));
    UBPL_LAUNCH_CHECK();
    return 0;
}

// One AdamW step (step = 1-based count after increment) on flat buffers.
UBPL_API int ubpl_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1,
                             double beta2, double eps, double weight_decay, int64_t step, void* stream) {
    if (n <= 0) return 0;
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    const double step_size = lr / bc1;
    const double bc2s = sqrt(bc2);
    hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                       (float)(1.0 - lr * weight_decay), (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                       (float)bc2s, (float)eps, (float)(-step_size), vec4_count(n, p, g, m, v));
    UBPL_LAUNCH_CHECK();
    return 0;
}

// Same step with the 1-based count on the device (incremented here) so a
// captured HIP graph replays correctly; coef: scratch of 4 floats.
UBPL_API int ubpl_adamw_step_dev(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1,
                                 double beta2, double eps, double weight_decay, int64_t* step, float* coef,
                                 void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(adamw_prep_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step, lr, beta1, beta2,
                       weight_decay, coef);
    UBPL_LAUNCH_CHECK();
    hipLaunchKernelGGL(adamw_dev_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, coef,
                       (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                       vec4_count(n, p, g, m, v));
    UBPL_LAUNCH_CHECK();
    return 0;
}

// ubpl_adamw_step_dev on p[0, nlive) fused with ubpl_ema_update(ema, p, n):
// flat buffers, 16-B aligned, nlive and n multiples of 4 (the flat layouts pad
// every segment to 4 floats).  alpha = min(1 - 1/(epo+1), ema_decay)
// (utils/parameters.py:4-8).
UBPL_API int ubpl_adamw_ema_step_dev(float* p, const float* g, float* m, float* v, int64_t nlive, double lr,
                                     double beta1, double beta2, double eps, double weight_decay, int64_t* step,
                                     float* coef, float* ema, int64_t n, double alpha, void* stream) {
    if (n <= 0 || nlive < 0 || nlive > n || (nlive & 3) || (n & 3)) return (int)hipErrorInvalidValue;
    if (vec4_count(n, p, ema) == 0 || (nlive > 0 && vec4_count(nlive, p, g, m, v) == 0))
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(adamw_prep_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step, lr, beta1, beta2,
                       weight_decay, coef);
    UBPL_LAUNCH_CHECK();
    hipLaunchKernelGGL(adamw_ema_dev_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v,
                       nlive >> 2, coef, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps, ema,
                       n >> 2, (float)alpha, (float)(1.0 - alpha));
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_scale_(float* x, int64_t n, float s, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n * 4)), dim3(256), 0, (hipStream_t)stream, x, n, s);
    UBPL_LAUNCH_CHECK();
    return 0;
}
