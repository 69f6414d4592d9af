// Hourglass resampling: MaxPool2d(2,2) (models/base/layers.py:93, hourglass.py:24),
// nearest Upsample(x2) + skip add (layers.py:102,110-111), and the feature
// projection AvgPool2d(2,2) (models/pose/hourglass.py:92-99).  All HBM-bound;
// one thread per output pair (float2 along W), backward recomputes the
// max-pool argmax from the saved input (first maximum in row-major window
// order, as PyTorch's CPU kernel) instead of storing indices.
#include "common.h"

namespace {

int grid_ew(int64_t n) {
    int64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    return (int)g;
}

// BatchNorm partials of an output written in NCHW order by one element per
// lane, Ho*Wo % 64 == 0: the 64 outputs of a wave are one 64-pixel slice of
// one channel (the conv epilogue's layout, common.h tile_bn_partials): S and
// M2 about the slice mean.  i0 = the wave's first flat index.
__device__ __forceinline__ void wave_bn_partial(float v, int64_t i0, int C, int P, int64_t np, float* part) {
    const float s = ubpl::wave_sum(v);
    const float d = v - s * (1.f / 64.f);
    const float m2 = ubpl::wave_sum(d * d);
    if ((threadIdx.x & 63) == 0) {
        const int64_t bc = i0 / P;
        const int c = (int)(bc % C);
        const int64_t q = ((bc / C) * P + (i0 - bc * P)) >> 6;
        part[((int64_t)c * np + q) * 2] = s;
        part[((int64_t)c * np + q) * 2 + 1] = m2;
    }
}

// planes = B*C; output Ho x Wo with Ho = H/2, Wo = W/2 (floor).
template <bool STATS>
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const float* __restrict__ x, int64_t planes, int H, int W,
                                                         float* __restrict__ y, int C, float* __restrict__ part) {
    const int Ho = H >> 1, Wo = W >> 1;
    const int64_t total = planes * Ho * Wo;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int ow = (int)(i % Wo);
        const int64_t t = i / Wo;
        const int oh = (int)(t % Ho);
        const int64_t pl = t / Ho;
        const float* p = x + (pl * H + 2 * oh) * W + 2 * ow;
        float m = p[0];
        float v = p[1];
        if (v > m || isnan(v)) m = v;
        v = p[W];
        if (v > m || isnan(v)) m = v;
        v = p[W + 1];
        if (v > m || isnan(v)) m = v;
        y[i] = m;
        if (STATS) wave_bn_partial(m, i - (threadIdx.x & 63), C, Ho * Wo, planes / C * Ho * Wo / 64, part);
    }
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                         int64_t planes, int H, int W, float* __restrict__ dx,
                                                         int accumulate) {
    const int Ho = H >> 1, Wo = W >> 1;
    const int64_t total = planes * Ho * Wo;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int ow = (int)(i % Wo);
        const int64_t t = i / Wo;
        const int oh = (int)(t % Ho);
        const int64_t pl = t / Ho;
        const int64_t base = (pl * H + 2 * oh) * W + 2 * ow;
        const float* p = x + base;
        int am = 0;
        float m = p[0];
        const int offs[4] = {0, 1, W, W + 1};
#pragma unroll
        for (int q = 1; q < 4; ++q) {
            const float v = p[offs[q]];
            if (v > m || isnan(v)) {
                m = v;
                am = q;
            }
        }
        const float g = dy[i];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float v = (q == am) ? g : 0.f;
            float* d = dx + base + offs[q];
            *d = accumulate ? *d + v : v;
        }
    }
}

// y = (sum of the 2x2 window) / 4, summed row-major like avg_pool2d's CPU loop.
__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const float* __restrict__ x, int64_t planes, int H, int W,
                                                         float* __restrict__ y) {
    const int Ho = H >> 1, Wo = W >> 1;
    const int64_t total = planes * Ho * Wo;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int ow = (int)(i % Wo);
        const int64_t t = i / Wo;
        const int oh = (int)(t % Ho);
        const int64_t pl = t / Ho;
        const float* p = x + (pl * H + 2 * oh) * W + 2 * ow;
        y[i] = (((p[0] + p[1]) + p[W]) + p[W + 1]) / 4.f;
    }
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const float* __restrict__ dy, int64_t planes, int H, int W,
                                                         float* __restrict__ dx, int accumulate) {
    const int Ho = H >> 1, Wo = W >> 1;
    const int64_t total = planes * Ho * Wo;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int ow = (int)(i % Wo);
        const int64_t t = i / Wo;
        const int oh = (int)(t % Ho);
        const int64_t pl = t / Ho;
        const int64_t base = (pl * H + 2 * oh) * W + 2 * ow;
        const float g = dy[i] / 4.f;
        const int64_t offs[4] = {0, 1, W, W + 1};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float* d = dx + base + offs[q];
            *d = accumulate ? *d + g : g;
        }
    }
}

// UBPL_UPADD_FENCE (diagnostic): every upsample-add workgroup starts with an
// agent-scope acquire fence (its XCD's L2 invalidated before it reads up / low)
#ifndef UBPL_UPADD_FENCE
#define UBPL_UPADD_FENCE 0
#endif

// The same, W % 4 == 0 and 16-B aligned: 4 outputs (one float4 of up / out, one
// float2 of low) per thread.  total4 = planes*H*W/4.
__global__ void __launch_bounds__(256) upadd_fwd_vec_kernel(const float* up, const float* __restrict__ low,
                                                           int H, int W, int64_t total4, float* out) {
    if (UBPL_UPADD_FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int W4 = W >> 2, Wl = W >> 1;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += stride) {
        const int w4 = (int)(i % W4);
        const int64_t t = i / W4;
        const int h = (int)(t % H);
        const int64_t pl = t / H;
        const float4 u = reinterpret_cast<const float4*>(up)[i];
        const float2 l = *reinterpret_cast<const float2*>(low + (pl * (H >> 1) + (h >> 1)) * Wl + 2 * w4);
        reinterpret_cast<float4*>(out)[i] = make_float4(u.x + l.x, u.y + l.x, u.z + l.y, u.w + l.y);
    }
}

// out[b,c,h,w] = up[b,c,h,w] + low[b,c,h/2,w/2]   (out may alias up)
template <bool STATS>
__global__ void __launch_bounds__(256) upadd_fwd_kernel(const float* up, const float* __restrict__ low,
                                                       int64_t planes, int H, int W, float* out, int C,
                                                       float* __restrict__ part) {
    if (UBPL_UPADD_FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int Hl = H >> 1, Wl = W >> 1;
    const int64_t total = planes * H * W;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int w = (int)(i % W);
        const int64_t t = i / W;
        const int h = (int)(t % H);
        const int64_t pl = t / H;
        const float v = up[i] + low[(pl * Hl + (h >> 1)) * Wl + (w >> 1)];
        out[i] = v;
        if (STATS) wave_bn_partial(v, i - (threadIdx.x & 63), C, H * W, planes / C * H * W / 64, part);
    }
}

// dlow[b,c,i,j] (+)= sum of the 2x2 block of dout (upsample_nearest2d backward)
__global__ void __launch_bounds__(256) upadd_bwd_kernel(const float* __restrict__ dout, int64_t planes, int H, int W,
                                                       float* __restrict__ dlow, int accumulate) {
    const int Hl = H >> 1, Wl = W >> 1;
    const int64_t total = planes * Hl * Wl;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int j = (int)(i % Wl);
        const int64_t t = i / Wl;
        const int r = (int)(t % Hl);
        const int64_t pl = t / Hl;
        const float* p = dout + (pl * H + 2 * r) * W + 2 * j;
        const float s = ((p[0] + p[1]) + p[W]) + p[W + 1];
        dlow[i] = accumulate ? dlow[i] + s : s;
    }
}

__global__ void __launch_bounds__(256) add_kernel(const float* a, const float* b, int64_t n, float* out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = a[i] + b[i];
}

}  // namespace

UBPL_API int ubpl_maxpool2x2_forward(const float* x, int64_t planes, int H, int W, float* y, void* stream) {
    const int64_t n = planes * (H / 2) * (W / 2);
    if (n == 0) return 0;
    hipLaunchKernelGGL(maxpool_fwd_kernel<false>, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, x, planes, H,
                       W, y, 1, nullptr);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// + BatchNorm partials of y for the BN that consumes it (ubpl_bn_partials
// layout; N = B*(H/2)*(W/2)).  Needs (H/2)*(W/2) % 64 == 0.
UBPL_API int ubpl_maxpool2x2_forward_stats(const float* x, int B, int C, int H, int W, float* y, float* part,
                                           void* stream) {
    const int64_t planes = (int64_t)B * C;
    if (((H / 2) * (W / 2)) % 64 != 0 || part == nullptr) return (int)hipErrorInvalidValue;
    const int64_t n = planes * (H / 2) * (W / 2);
    if (n == 0) return 0;
    hipLaunchKernelGGL(maxpool_fwd_kernel<true>, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, x, planes, H,
                       W, y, C, part);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_maxpool2x2_backward(const float* x, const float* dy, int64_t planes, int H, int W, float* dx,
                                      int accumulate, void* stream) {
    const int64_t n = planes * (H / 2) * (W / 2);
    if (n == 0) return 0;
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, x, dy, planes, H, W,
                       dx, accumulate);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_avgpool2x2_forward(const float* x, int64_t planes, int H, int W, float* y, void* stream) {
    const int64_t n = planes * (H / 2) * (W / 2);
    if (n == 0) return 0;
    hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, x, planes, H, W, y);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_avgpool2x2_backward(const float* dy, int64_t planes, int H, int W, float* dx, int accumulate,
                                      void* stream) {
    const int64_t n = planes * (H / 2) * (W / 2);
    if (n == 0) return 0;
    hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, dy, planes, H, W, dx,
                       accumulate);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_upsample2x_add_forward(const float* up, const float* low, int64_t planes, int H, int W, float* out,
                                         void* stream) {
    const int64_t n = planes * H * W;
    if (n == 0) return 0;
    if ((W % 4) == 0 && ((((uintptr_t)up) | ((uintptr_t)out)) & 15) == 0 && (((uintptr_t)low) & 7) == 0) {
        hipLaunchKernelGGL(upadd_fwd_vec_kernel, dim3(grid_ew(n / 4)), dim3(256), 0, (hipStream_t)stream, up, low, H,
                           W, n / 4, out);
        UBPL_LAUNCH_CHECK();
        return 0;
    }
    hipLaunchKernelGGL(upadd_fwd_kernel<false>, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, up, low, planes,
                       H, W, out, 1, nullptr);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// + BatchNorm partials of out (ubpl_bn_partials layout; N = B*H*W).  H*W % 64 == 0.
UBPL_API int ubpl_upsample2x_add_forward_stats(const float* up, const float* low, int B, int C, int H, int W,
                                               float* out, float* part, void* stream) {
    const int64_t planes = (int64_t)B * C;
    if ((H * W) % 64 != 0 || part == nullptr) return (int)hipErrorInvalidValue;
    const int64_t n = planes * H * W;
    if (n == 0) return 0;
    hipLaunchKernelGGL(upadd_fwd_kernel<true>, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, up, low, planes,
                       H, W, out, C, part);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_upsample2x_add_backward(const float* dout, int64_t planes, int H, int W, float* dlow,
                                          int accumulate, void* stream) {
    const int64_t n = planes * (H / 2) * (W / 2);
    if (n == 0) return 0;
    hipLaunchKernelGGL(upadd_bwd_kernel, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, dout, planes, H, W, dlow,
                       accumulate);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_add(const float* a, const float* b, int64_t n, float* out, void* stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(add_kernel, dim3(grid_ew(n)), dim3(256), 0, (hipStream_t)stream, a, b, n, out);
    UBPL_LAUNCH_CHECK();
    return 0;
}
